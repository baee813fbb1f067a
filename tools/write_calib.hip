// WRITE_SIZE calibration for 32-byte records (measurement tool, not product code; VERDICT r03
// asked to calibrate before reading k_ss_scatter's WRITE_SIZE as amplification): N records of
// 32 bytes written (a) in order, (b) each to a pseudo-random slot of a permutation (the scatter's
// pattern), (c) in random pairs of neighbours (64 contiguous bytes).  Run under
// rocprofv3 --pmc WRITE_SIZE (and --kernel-trace for times).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/write_calib tools/write_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

struct __align__(32) R { uint64_t a, b, c, d; };

// a bijection of [0, n) for n a power of two: odd multiplier then xor-shift, masked
__device__ __forceinline__ uint64_t perm(uint64_t i, uint64_t mask) {
    uint64_t x = (i * 0x9E3779B97F4A7C15ull) & mask;
    x ^= x >> 7;
    return (x * 0xD6E8FEB86659FD93ull) & mask;  // odd multiplier mod 2^k: still a bijection
}
__global__ void k_seq32(R* o, uint64_t n) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n) o[i] = R{i, i + 1, i + 2, i + 3};
}
__global__ void k_rand32(R* o, uint64_t n) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n) o[perm(i, n - 1)] = R{i, i + 1, i + 2, i + 3};
}
__global__ void k_rand64(R* o, uint64_t n) {   // thread i writes records 2j, 2j+1 of pair j
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n / 2) {
        const uint64_t j = perm(i, n / 2 - 1);
        o[2 * j] = R{i, 0, 0, 0};
        o[2 * j + 1] = R{i, 1, 0, 0};
    }
}

int main() {
    const uint64_t n = 1ull << 25;               // 32 Mi records = 1 GiB
    R* o = nullptr;
    if (hipMalloc(&o, n * sizeof(R)) != hipSuccess) { printf("hipMalloc failed\n"); return 1; }
    hipMemset(o, 0, n * sizeof(R));
    const unsigned nt = 256;
    for (int rep = 0; rep < 3; rep++) {
        k_seq32<<<(unsigned)((n + nt - 1) / nt), nt>>>(o, n);
        k_rand32<<<(unsigned)((n + nt - 1) / nt), nt>>>(o, n);
        k_rand64<<<(unsigned)((n / 2 + nt - 1) / nt), nt>>>(o, n);
    }
    hipDeviceSynchronize();
    printf("records %llu x 32 B = %.3f GB written by each kernel per launch\n", (unsigned long long)n, n * 32.0 / 1e9);
    hipFree(o);
    return 0;
}
