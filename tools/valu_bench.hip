// VALU issue-cost microbenchmark (measurement tool, not product code): one 1024-thread
// workgroup per CU (4 waves per SIMD, k_map's geometry), each wave runs R rounds of 32
// independent instructions of one kind over 8 register chains; prints instructions per cycle
// per SIMD (clock from s_memtime deltas inside the kernel).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_bench tools/valu_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define R 4096

#define OPS8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define OPS32(I) OPS8(I) OPS8(I) OPS8(I) OPS8(I)

template <int K>
__global__ __launch_bounds__(1024) void k_valu(unsigned* out, unsigned long long* cyc, unsigned seed) {
    unsigned v0 = threadIdx.x ^ seed, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 * 11, v5 = v0 * 13, v6 = v0 * 17,
             v7 = v0 * 19;
    unsigned long long w0 = v0, w1 = v1, w2 = v2, w3 = v3, w4 = v4, w5 = v5, w6 = v6, w7 = v7;
    unsigned m = seed | 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; r++) {
#define A32(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v##i) : "v"(m));
#define M32(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v##i) : "v"(m));
#define M24(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(v##i) : "v"(m));
#define SH64(i) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(w##i));
#define AB(i) asm volatile("v_alignbyte_b32 %0, %0, %1, %1" : "+v"(v##i) : "v"(m));
#define DPP(i) asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(v##i));
#define CMP64(i) asm volatile("v_cmp_eq_u64 vcc, %1, %2\n\tv_cndmask_b32 %0, %0, %3, vcc" : "+v"(v##i) : "v"(w##i), "v"(w0), "v"(m) : "vcc");
#define CMP32(i) asm volatile("v_cmp_eq_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(v##i) : "v"(m) : "vcc");
#define BFE(i) asm volatile("v_bfe_u32 %0, %0, 3, 7" : "+v"(v##i));
#define ADD64(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(w##i) : "v"(w1));
        if (K == 0) { OPS32(A32) }
        if (K == 1) { OPS32(M32) }
        if (K == 2) { OPS32(M24) }
        if (K == 3) { OPS32(SH64) }
        if (K == 4) { OPS32(AB) }
        if (K == 5) { OPS32(DPP) }
        if (K == 6) { OPS32(CMP64) }
        if (K == 7) { OPS32(CMP32) }
        if (K == 8) { OPS32(BFE) }
        if (K == 9) { OPS32(ADD64) }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 1024 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7 ^ (unsigned)(w0 ^ w1 ^ w2 ^ w3 ^ w4 ^ w5 ^ w6 ^ w7);
}

template <int K>
void run(const char* name, int per_round, unsigned* out, unsigned long long* cyc, int ncu) {
    hipLaunchKernelGGL(k_valu<K>, dim3(ncu), dim3(1024), 0, 0, out, cyc, 7u);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_valu<K>, dim3(ncu), dim3(1024), 0, 0, out, cyc, 9u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    unsigned long long h[1024];
    hipMemcpy(h, cyc, ncu * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < ncu; i++) avg += h[i];
    avg /= ncu;
    // per SIMD: 4 waves x R rounds x 32 x per_round instructions
    const double inst = 4.0 * R * 32 * per_round;
    printf("%-10s %8.3f ms  %.3f inst/cycle/SIMD (s_memtime)  %.3f inst/cycle/SIMD at 2.4 GHz wall\n", name, ms,
           inst / avg, inst / (ms * 1e-3 * 2.4e9));
}

int main() {
    int ncu = 256;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) == hipSuccess) ncu = p.multiProcessorCount;
    unsigned* out;
    unsigned long long* cyc;
    hipMalloc(&out, ncu * 1024 * sizeof(unsigned));
    hipMalloc(&cyc, ncu * sizeof(unsigned long long));
    run<0>("add32", 1, out, cyc, ncu);
    run<1>("mul_lo32", 1, out, cyc, ncu);
    run<2>("mul24", 1, out, cyc, ncu);
    run<3>("lshl_b64", 1, out, cyc, ncu);
    run<4>("alignbyte", 1, out, cyc, ncu);
    run<5>("mov_dpp", 1, out, cyc, ncu);
    run<6>("cmp64+cnd", 2, out, cyc, ncu);
    run<7>("cmp32+cnd", 2, out, cyc, ncu);
    run<8>("bfe", 1, out, cyc, ncu);
    run<9>("add64", 1, out, cyc, ncu);
    return 0;
}
