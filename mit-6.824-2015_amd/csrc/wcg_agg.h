// wcg_agg.h - second aggregation stage: the miss log of k_map, one hash bucket at a time.
//
// k_map leaves, per (workgroup w, bucket p), a region of 16-byte entries: keys that missed
// w's LDS table plus w's flushed LDS slots (with counts).  Every key of bucket p lands only in
// bucket-p regions, so a workgroup that aggregates bucket p over a slice of source regions
// needs LDS for (distinct keys of p) / 1 - about 1/P of the vocabulary - and flushes each
// distinct key once: the per-token global atomics of a naive design become per-(slice, key)
// atomics.  Overflow of the LDS table still falls back to the global table (exact, slower).
#pragma once
#include "wcg_common.h"
#include "wcg_lds_table.h"

namespace wcg {

constexpr int AGG_NT = 512;
constexpr int AGG_NB = 1664;           // 1664 x 4 slots x 24 B (u64 counts) = 159744 B

struct AggArgs {
    const uint4* pool;
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
    for (u32 w = w0; w < w1; w++) {
        const u64 reg = (u64)w * a.P + p;
        const u32 len = a.region_len[reg];
        const uint4* base = a.pool + reg * a.region_cap;
        for (u32 i = tid; i < len; i += AGG_NT) {
            const uint4 e = base[i];
            const u64 k0 = (u64)e.y << 32 | e.x;
            u64 k1 = (u64)e.w << 32 | e.z;
            if (k0 == 0) continue;                       // count carrier / filler
            u64 c = 1;
            if (k1 & CNT_FLAG) {
                const uint4 f = base[i + 1];
                c = (u64)f.w << 32 | f.z;
                k1 &= ~CNT_FLAG;
            }
            if (!tab.add(k0, k1, lds_hash(k0, k1), c)) {
                my_global++;
                ginsert(a.gtab, a.gmask, k0, k1, gslot(key_hash(k0, k1)), c, a.st);
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
