// microbench.hip - design-time measurements on MI355X for the word-count hot path:
// global integer atomics (scattered), CAS, random 16B probes, LDS atomics, HBM streaming.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench tools/microbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x;
}

template <int SCOPE>
__global__ void k_atomic_u64(unsigned long long* t, uint64_t mask, int iters) {
    uint64_t id = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (int i = 0; i < iters; i++) {
        uint64_t s = mix(id * 1315423911ull + i) & mask;
        if (SCOPE == 0) __hip_atomic_fetch_add(&t[s], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else __hip_atomic_fetch_add(&t[s], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}
__global__ void k_atomic_u32(unsigned* t, uint64_t mask, int iters) {
    uint64_t id = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (int i = 0; i < iters; i++) {
        uint64_t s = mix(id * 1315423911ull + i) & mask;
        __hip_atomic_fetch_add(&t[s], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// zipf-like hot set: 90% of ops into the first 8K slots
__global__ void k_atomic_hot(unsigned long long* t, uint64_t mask, int iters) {
    uint64_t id = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (int i = 0; i < iters; i++) {
        uint64_t h = mix(id * 1315423911ull + i);
        uint64_t s = (h >> 60) < 14 ? (h & 8191) : (h & mask);
        __hip_atomic_fetch_add(&t[s], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
__global__ void k_cas_u64(unsigned long long* t, uint64_t mask, int iters) {
    uint64_t id = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (int i = 0; i < iters; i++) {
        uint64_t s = mix(id * 1315423911ull + i) & mask;
        unsigned long long exp = 0;
        __hip_atomic_compare_exchange_strong(&t[s], &exp, id + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
__global__ void k_probe16(const uint4* t, uint64_t mask, int iters, unsigned* out) {
    uint64_t id = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    unsigned acc = 0;
    for (int i = 0; i < iters; i++) {
        uint64_t s = mix(id * 1315423911ull + i + acc) & mask;
        uint4 v = t[s];
        acc += v.x ^ v.w;
    }
    if (acc == 0x12345678) out[0] = acc;
}
__global__ void k_probe16_atomic(uint64_t* t, uint64_t mask, int iters, unsigned* out) {
    uint64_t id = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    unsigned acc = 0;
    for (int i = 0; i < iters; i++) {
        uint64_t s = mix(id * 1315423911ull + i + acc) & mask;
        uint64_t a = __hip_atomic_load(&t[2 * s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint64_t b = __hip_atomic_load(&t[2 * s + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        acc += (unsigned)(a ^ b);
    }
    if (acc == 0x12345678) out[0] = acc;
}
template <int SLOTS>
__global__ void k_lds_atomic(int iters, unsigned* out) {
    __shared__ unsigned tab[SLOTS];
    for (int i = threadIdx.x; i < SLOTS; i += blockDim.x) tab[i] = 0;
    __syncthreads();
    uint64_t id = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (int i = 0; i < iters; i++) {
        uint32_t s = (uint32_t)mix(id * 1315423911ull + i) % SLOTS;
        atomicAdd(&tab[s], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0 && tab[0] == 0x7fffffff) out[0] = 1;
}
__global__ void k_stream_read(const uint4* in, uint64_t n16, unsigned* out) {
    uint64_t id = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, st = (uint64_t)gridDim.x * blockDim.x;
    unsigned acc = 0;
    for (uint64_t i = id; i < n16; i += st) { uint4 v = in[i]; acc ^= v.x + v.y + v.z + v.w; }
    if (acc == 0x12345678) out[0] = acc;
}
__global__ void k_stream_write(uint4* o, uint64_t n16) {
    uint64_t id = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, st = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = id; i < n16; i += st) o[i] = make_uint4((unsigned)i, 1, 2, 3);
}

template <typename F>
float timeit(F f, int reps = 5) {
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; i++) f();
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    const int B = 256, G = 256 * 8;
    const double nthreads = (double)B * G;
    unsigned* out; CK(hipMalloc(&out, 64));
    size_t big = 1ull << 30;
    void* buf; CK(hipMalloc(&buf, big)); CK(hipMemset(buf, 0, big));
    int iters = 64;
    double ops = nthreads * iters;
    for (uint64_t bytes : {1ull << 20, 4ull << 20, 64ull << 20, 1ull << 30}) {
        uint64_t mask = bytes / 8 - 1;
        float ms = timeit([&] { k_atomic_u64<0><<<G, B>>>((unsigned long long*)buf, mask, iters); });
        printf("atomic_add_u64 agent  table %6llu KiB: %8.3f ms  %.3e op/s\n", (unsigned long long)(bytes >> 10), ms, ops / ms * 1e3);
        ms = timeit([&] { k_atomic_u64<1><<<G, B>>>((unsigned long long*)buf, mask, iters); });
        printf("atomic_add_u64 wgscope table %6llu KiB: %8.3f ms  %.3e op/s\n", (unsigned long long)(bytes >> 10), ms, ops / ms * 1e3);
        ms = timeit([&] { k_atomic_u32<<<G, B>>>((unsigned*)buf, bytes / 4 - 1, iters); });
        printf("atomic_add_u32 agent  table %6llu KiB: %8.3f ms  %.3e op/s\n", (unsigned long long)(bytes >> 10), ms, ops / ms * 1e3);
        ms = timeit([&] { k_atomic_hot<<<G, B>>>((unsigned long long*)buf, mask, iters); });
        printf("atomic_add_u64 hot90%% table %6llu KiB: %8.3f ms  %.3e op/s\n", (unsigned long long)(bytes >> 10), ms, ops / ms * 1e3);
        CK(hipMemset(buf, 0, bytes));
        ms = timeit([&] { k_cas_u64<<<G, B>>>((unsigned long long*)buf, mask, iters); }, 1);
        printf("cas_u64 agent         table %6llu KiB: %8.3f ms  %.3e op/s\n", (unsigned long long)(bytes >> 10), ms, ops / ms * 1e3);
        ms = timeit([&] { k_probe16<<<G, B>>>((const uint4*)buf, bytes / 16 - 1, iters, out); });
        printf("probe16 plain         table %6llu KiB: %8.3f ms  %.3e op/s\n", (unsigned long long)(bytes >> 10), ms, ops / ms * 1e3);
        ms = timeit([&] { k_probe16_atomic<<<G, B>>>((uint64_t*)buf, bytes / 16 - 1, iters, out); });
        printf("probe16 atomic-load   table %6llu KiB: %8.3f ms  %.3e op/s\n", (unsigned long long)(bytes >> 10), ms, ops / ms * 1e3);
    }
    {
        float ms = timeit([&] { k_lds_atomic<32768><<<G, B>>>(iters * 4, out); });
        printf("lds atomic u32 32K slots: %.3f ms %.3e op/s\n", ms, ops * 4 / ms * 1e3);
        ms = timeit([&] { k_lds_atomic<32768><<<512, 1024>>>(iters * 4, out); });
        printf("lds atomic u32 32K slots (1024thr): %.3f ms %.3e op/s\n", ms, 512.0 * 1024 * iters * 4 / ms * 1e3);
    }
    for (int g : {1024, 2048, 4096, 8192}) {
        float ms = timeit([&] { k_stream_read<<<g, 256>>>((const uint4*)buf, big / 16, out); });
        printf("stream read 1GiB grid %d: %.3f ms %.1f GB/s\n", g, ms, big / ms / 1e6);
    }
    float ms = timeit([&] { k_stream_write<<<4096, 256>>>((uint4*)buf, big / 16); });
    printf("stream write 1GiB: %.3f ms %.1f GB/s\n", ms, big / ms / 1e6);
    CK(hipFree(buf)); CK(hipFree(out));
    return 0;
}
