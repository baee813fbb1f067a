// wcg_agg.h - second aggregation stage: the miss log of k_map, one hash bucket at a time.
//
// k_map leaves, per (workgroup w, bucket p), a region of miss-log units (wcg_lds_table.h): keys that missed
// w's LDS table plus w's flushed LDS slots (with counts).  Every key of bucket p lands only in
// bucket-p regions, so a workgroup that aggregates bucket p over a slice of source regions
// needs LDS for (distinct keys of p) / 1 - about 1/P of the vocabulary - and flushes each
// distinct key once: the per-token global atomics of a naive design become per-(slice, key)
// atomics.  Overflow of the LDS table still falls back to the global table (exact, slower).
#pragma once
#include "wcg_common.h"
#include "wcg_lds_table.h"

namespace wcg {

constexpr int AGG_NT = 1024;
constexpr int AGG_ILP = 4;
constexpr int AGG_NB = 1696;           // 1696 x 4 slots x 24 B (u64 counts) = 162816 B

struct AggArgs {
    const u64* pool;
    const u32* region_len;
    u64 region_cap;
    u32 P;                 // miss buckets
    u32 nsrc;              // source workgroups of k_map
    u32 slices;            // workgroups per bucket
    GEntry* gtab;
    u64 gmask;
    DevState* st;
};

__global__ __launch_bounds__(AGG_NT) void k_agg(AggArgs a) {
    __shared__ __align__(16) u64 tk0[AGG_NB][4];
    __shared__ __align__(16) u64 tk1[AGG_NB][4];
    __shared__ u64 tcnt[AGG_NB][4];
    const int tid = threadIdx.x;
    LdsTable<AGG_NB, u64> tab{tk0, tk1, tcnt};
    tab.init(tid, AGG_NT);
    __syncthreads();

    const u32 p = blockIdx.x % a.P, s = blockIdx.x / a.P;
    const u32 w0 = (u32)(((u64)a.nsrc * s) / a.slices), w1 = (u32)(((u64)a.nsrc * (s + 1)) / a.slices);
    u64 my_global = 0;
    // units are read AGG_ILP at a time per thread (independent loads in flight), decoded, and
    // looked up two at a time (both probes' bucket reads issued before either is matched)
    auto decode = [&](const u64* base, u32 i, u64 u, u64& k0, u64& k1, u64& c) -> bool {
        const u32 T = (u32)(u >> 56);
        if (T == 0) return false;                            // count / filler
        bool has;
        u32 j;
        k1 = 0;
        if (T < 0x41) {
            if ((T & 0x1F) >= 8) return false;               // medium-key tail
            k0 = u & ~U_CNT;
            has = (u & U_CNT) != 0;
            j = i + 1;
        } else {
            k0 = u;
            k1 = base[i + 1];
            has = (k1 & U_CNT) != 0;
            k1 &= ~U_CNT;
            j = i + 2;
        }
        c = has ? base[j] : 1;
        return true;
    };
    auto spill = [&](u64 k0, u64 k1, u64 c) {
        my_global++;
        ginsert(a.gtab, a.gmask, k0, k1, gslot(key_hash(k0, k1)), c, a.st);
    };
    for (u32 w = w0; w < w1; w++) {
        const u64 reg = (u64)w * a.P + p;
        const u32 len = a.region_len[reg];
        const u64* base = a.pool + reg * a.region_cap;
        for (u32 i0 = tid; i0 < len; i0 += AGG_NT * AGG_ILP) {
            u64 u[AGG_ILP];
#pragma unroll
            for (int k = 0; k < AGG_ILP; k++) {
                const u32 i = i0 + k * AGG_NT;
                u[k] = i < len ? base[i] : 0;
            }
#pragma unroll
            for (int k = 0; k < AGG_ILP; k += 2) {
                u64 a0, a1, ac, b0, b1, bc;
                const bool va = decode(base, i0 + k * AGG_NT, u[k], a0, a1, ac);
                const bool vb = decode(base, i0 + (k + 1) * AGG_NT, u[k + 1], b0, b1, bc);
                typename decltype(tab)::Probe pa, pb;
                if (va) tab.start(lds_hash(a0, a1), pa);
                if (vb) tab.start(lds_hash(b0, b1), pb);
                if (va && !tab.finish(a0, a1, pa, ac)) spill(a0, a1, ac);
                if (vb && !tab.finish(b0, b1, pb, bc)) spill(b0, b1, bc);
            }
        }
    }
    __syncthreads();
    for (int i = tid; i < AGG_NB * 4; i += AGG_NT) {
        const u64 c = (&tcnt[0][0])[i];
        if (!c) continue;
        const u64 k0 = (&tk0[0][0])[i], k1 = (&tk1[0][0])[i];
        my_global++;
        ginsert(a.gtab, a.gmask, k0, k1, gslot(key_hash(k0, k1)), c, a.st);
    }
    for (int d = 32; d >= 1; d >>= 1) my_global += __shfl_xor(my_global, d, 64);
    if ((tid & 63) == 0) atomicAdd(&a.st->global_ops, my_global);
}

}  // namespace wcg
