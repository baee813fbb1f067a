// Streaming-read probe (measurement only): how fast can 16 waves/CU stream 1 GiB with the
// k_map access pattern?  Variants isolate the descriptor-per-step buffer loads, the extra
// (prefix/look-ahead) load, the LDS footprint and the in-flight depth.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/stream_probe tools/stream_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4i rsrc(const void* base, uint32_t n) {
    uint64_t p = (uint64_t)base; v4i r;
    r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)p);
    r.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(p >> 32) & 0xFFFFu));
    r.z = __builtin_amdgcn_readfirstlane((int)n); r.w = 0x00020000; return r;
}
#define LD(TAG) __device__ __forceinline__ v4u ld_##TAG(v4i r, uint32_t o) { v4u v; \
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=&v"(v) : "v"(o), "s"(r) : "memory"); return v; }
LD(a) LD(b) LD(c) LD(d) LD(e) LD(f) LD(g) LD(h)
#define W(N, x, y) asm volatile("s_waitcnt vmcnt(" #N ")" : "+v"(x), "+v"(y) :: "memory")

// plain grid-stride loads, compiler-managed (the microbench reference)
__global__ __launch_bounds__(1024) void k_plain(const uint4* in, uint64_t n16, unsigned* out) {
    uint64_t id = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, st = (uint64_t)gridDim.x * blockDim.x;
    unsigned acc = 0;
#pragma unroll 4
    for (uint64_t i = id; i < n16; i += st) { uint4 v = in[i]; acc ^= v.x + v.y + v.z + v.w; }
    if (acc == 0x12345678) out[0] = acc;
}

// k_map pattern: wave steps of 1 KiB dealt chip-wide, descriptor per step, 4 sets in flight
template <int XLOAD, int LDSKB>
__global__ __launch_bounds__(1024) void k_sets(const uint8_t* in, uint64_t n, unsigned* out) {
    __shared__ uint32_t pad[LDSKB * 256 + 1024];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (LDSKB) pad[threadIdx.x] = 0;
    const uint64_t nsteps = n / 1024, stride = (uint64_t)gridDim.x * 16;
    uint64_t s = (uint64_t)blockIdx.x * 16 + wave;
    const int xc = lane == 0 ? 0 : (lane == 63 ? 65 : (lane == 1 ? 66 : -1));
    auto addr = [&](uint64_t step, v4i& r, uint32_t& om, uint32_t& ox) {
        bool live = step < nsteps;
        uint64_t org = (step == 0 || !live) ? 0 : step * 1024 - 16;
        uint64_t span = live ? n - org : 0;
        r = rsrc(in + org, span > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)span);
        uint32_t rel = (uint32_t)(step * 1024 - org);
        om = live ? rel + 16 * lane : 0xFFFFFFF0u;
        ox = (live && xc >= 0 && XLOAD) ? rel - 16 + 16 * xc : 0xFFFFFFF0u;
    };
    v4u ma, xa, mb, xb, mc, xc_, md, xd;
    unsigned acc = 0;
    { v4i r; uint32_t om, ox;
      addr(s, r, om, ox); ma = ld_a(r, om); xa = ld_b(r, ox);
      addr(s + stride, r, om, ox); mb = ld_c(r, om); xb = ld_d(r, ox);
      addr(s + 2 * stride, r, om, ox); mc = ld_e(r, om); xc_ = ld_f(r, ox);
      addr(s + 3 * stride, r, om, ox); md = ld_g(r, om); xd = ld_h(r, ox); }
    while (true) {
        v4i r; uint32_t om, ox;
        if (s >= nsteps) break;
        addr(s + 4 * stride, r, om, ox); W(6, ma, xa); acc ^= ma.x + xa.y; ma = ld_a(r, om); xa = ld_b(r, ox); s += stride;
        if (s >= nsteps) break;
        addr(s + 4 * stride, r, om, ox); W(6, mb, xb); acc ^= mb.x + xb.y; mb = ld_c(r, om); xb = ld_d(r, ox); s += stride;
        if (s >= nsteps) break;
        addr(s + 4 * stride, r, om, ox); W(6, mc, xc_); acc ^= mc.x + xc_.y; mc = ld_e(r, om); xc_ = ld_f(r, ox); s += stride;
        if (s >= nsteps) break;
        addr(s + 4 * stride, r, om, ox); W(6, md, xd); acc ^= md.x + xd.y; md = ld_g(r, om); xd = ld_h(r, ox); s += stride;
    }
    W(0, ma, xa); W(0, mb, xb); W(0, mc, xc_); W(0, md, xd);
    if (LDSKB) acc ^= pad[(threadIdx.x * 7) & 1023];
    if (acc == 0x12345678) out[0] = acc;
}

template <typename F>
float timeit(F f, int reps = 10) {
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; i++) f();
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    const size_t n = 1ull << 30;
    uint8_t* buf; CK(hipMalloc(&buf, n + 4096)); CK(hipMemset(buf, 1, n + 4096));
    unsigned* out; CK(hipMalloc(&out, 64));
    auto rep = [&](const char* name, float ms) { printf("%-44s %.4f ms  %7.1f GB/s\n", name, ms, n / (ms * 1e-3) / 1e9); };
    rep("plain grid-stride, 256 x 1024 thr", timeit([&] { k_plain<<<256, 1024>>>((const uint4*)buf, n / 16, out); }));
    rep("plain grid-stride, 512 x 1024 thr", timeit([&] { k_plain<<<512, 1024>>>((const uint4*)buf, n / 16, out); }));
    rep("sets4 +xload, no LDS", timeit([&] { k_sets<1, 0><<<256, 1024>>>(buf, n, out); }));
    rep("sets4 no xload, no LDS", timeit([&] { k_sets<0, 0><<<256, 1024>>>(buf, n, out); }));
    rep("sets4 +xload, 156 KiB LDS", timeit([&] { k_sets<1, 156><<<256, 1024>>>(buf, n, out); }));
    rep("sets4 no xload, 156 KiB LDS", timeit([&] { k_sets<0, 156><<<256, 1024>>>(buf, n, out); }));
    return 0;
}
