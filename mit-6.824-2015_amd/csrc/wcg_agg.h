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
constexpr u32 AGG_BATCH = AGG_NT * 4;     // units per batch (4 per thread)
constexpr int AGG_W = 2;               // ways per bucket (16-byte k0 rows: wcg_lds_table.h)
constexpr int AGG_NB = 3380;           // 3380 x 2 slots x 24 B (u64 counts) = 162240 B (+ 1.5 KiB)
constexpr u32 AGG_SLACK_UNITS = AGG_BATCH + 8;   // pool tail slack for k_agg's unmasked loads
constexpr u32 AGG_MAX_SRC = 256;       // source regions per workgroup (+1 KiB LDS = 160 KiB)

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
    const u64* map_stats;  // k_map's per-workgroup stats [nsrc][4], summed by workgroup 0
};

__global__ __launch_bounds__(AGG_NT) void k_agg(AggArgs a) {
    __shared__ __align__(16) u64 tk0[AGG_NB][AGG_W];
    __shared__ __align__(16) u64 tk1[AGG_NB][AGG_W];
    __shared__ u64 tcnt[AGG_NB][AGG_W];
    __shared__ u32 rlen_s[AGG_MAX_SRC];
    const int tid = threadIdx.x;
    LdsTable<AGG_NB, u64, AGG_W> tab{tk0, tk1, tcnt};
    tab.init(tid, AGG_NT);
    const u32 p = blockIdx.x % a.P, s = blockIdx.x / a.P;
    const u32 w0 = (u32)(((u64)a.nsrc * s) / a.slices), w1 = (u32)(((u64)a.nsrc * (s + 1)) / a.slices);
    // region lengths of this slice, staged once: a global load in the batch walk would be a
    // vmcnt wait that drains the prefetch
    for (u32 w = w0 + tid; w < w1; w += AGG_NT) rlen_s[w - w0] = a.region_len[(u64)w * a.P + p];
    __syncthreads();
    u64 my_global = 0;
    // Every wave walks its own regions (w0 + wave, + 16, ...) in wave batches of 256 units:
    // lane l takes units [4l, 4l + 4) and also loads the two after them, so a medium-key head or
    // a count flag finds its neighbours in registers (units past the region's length are masked
    // to 0 = filler).  The next wave batch is loaded into the other register set while this one
    // is aggregated, and no barrier ties the waves together, so 16 waves x 2 batches are in
    // flight per CU: a workgroup-wide batch walk kept only 2, and k_agg ran at the HBM latency
    // of one batch per region even for nearly empty regions.
    const int wave = tid >> 6, lane = tid & 63;
    constexpr u32 WB = 256;                          // units per wave batch
    constexpr u32 WSTRIDE = AGG_NT / 64;             // regions between a wave's regions
    auto rlen = [&](u32 w) -> u32 { return rlen_s[w - w0]; };
    auto next_batch = [&](u32& w, u32& b) {          // wave-uniform walk over non-empty batches
        b++;
        while (w < w1 && (u64)b * WB >= rlen(w)) { w += WSTRIDE; b = 0; }
    };
    auto load = [&](u32 w, u32 b, v4u& x0, v4u& x1, v4u& x2) {
        const bool live = w < w1;
        const u32 i = b * WB + 4 * lane, lim = live ? rlen(w) : 0;
        const v4u* q = reinterpret_cast<const v4u*>(a.pool + ((u64)(live ? w : w0) * a.P + p) * a.region_cap + i);
        (void)lim;                    // units past the region's length are masked in process()
        x0 = q[0];                    // unconditional (the pool has AGG_SLACK_UNITS of slack),
        x1 = q[1];                    // so no branch splits the loads from the waits that let
        x2 = q[2];                    // the next batch stay in flight
    };
    auto unit = [](const v4u& x, int h) -> u64 { return h ? ((u64)x.w << 32 | x.z) : ((u64)x.y << 32 | x.x); };
    auto process = [&](u32 w, u32 b, const v4u& x0, const v4u& x1, const v4u& x2) {
        u64 u[6] = {unit(x0, 0), unit(x0, 1), unit(x1, 0), unit(x1, 1), unit(x2, 0), unit(x2, 1)};
        const u32 i0 = b * WB + 4 * lane, len = rlen(w);
#pragma unroll
        for (int k = 0; k < 6; k++) u[k] = i0 + k < len ? u[k] : 0;
        u64 k0[4], k1[4], c[4];
        bool v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const u32 T = (u32)(u[k] >> 56);
            const bool head = T >= 0x41;
            v[k] = T != 0 && (head || (T & 0x1F) < 8);   // skip counts, fillers, medium tails
            const u64 last = head ? u[k + 1] : u[k];     // unit carrying the count flag
            k0[k] = head ? u[k] : (u[k] & ~U_CNT);
            k1[k] = head ? (u[k + 1] & ~U_CNT) : 0;
            c[k] = (last & U_CNT) ? (head ? u[k + 2] : u[k + 1]) : 1;
        }
#pragma unroll
        for (int k = 0; k < 4; k += 2) {
            typename decltype(tab)::Probe pa, pb;
            if (v[k]) tab.start(lds_hash(k0[k], k1[k]), pa);
            if (v[k + 1]) tab.start(lds_hash(k0[k + 1], k1[k + 1]), pb);
            if (v[k] && !tab.finish(k0[k], k1[k], pa, c[k])) {
                my_global++;
                ginsert(a.gtab, a.gmask, k0[k], k1[k], gslot(key_hash(k0[k], k1[k])), c[k], a.st);
            }
            if (v[k + 1] && !tab.finish(k0[k + 1], k1[k + 1], pb, c[k + 1])) {
                my_global++;
                ginsert(a.gtab, a.gmask, k0[k + 1], k1[k + 1], gslot(key_hash(k0[k + 1], k1[k + 1])), c[k + 1], a.st);
            }
        }
    };
    u32 wa = w0 + wave, ba = (u32)-1;
    next_batch(wa, ba);
    u32 wb = wa, bb = ba;
    next_batch(wb, bb);
    v4u a0, a1, a2, b0, b1, b2;
    load(wa, ba, a0, a1, a2);
    load(wb, bb, b0, b1, b2);
    while (wa < w1) {
        process(wa, ba, a0, a1, a2);
        u32 wn = wb, bn = bb;
        next_batch(wn, bn);
        wa = wn; ba = bn;
        load(wa, ba, a0, a1, a2);
        if (wb >= w1) break;
        process(wb, bb, b0, b1, b2);
        wn = wa; bn = ba;
        next_batch(wn, bn);
        wb = wn; bb = bn;
        load(wb, bb, b0, b1, b2);
    }
    __syncthreads();
    for (int i = tid; i < AGG_NB * AGG_W; i += AGG_NT) {
        const u64 c = (&tcnt[0][0])[i];
        if (!c) continue;
        const u64 k0 = (&tk0[0][0])[i], k1 = (&tk1[0][0])[i];
        my_global++;
        ginsert(a.gtab, a.gmask, k0, k1, gslot(key_hash(k0, k1)), c, a.st);
    }
    // one atomic per workgroup (a per-wave atomic on one DevState line serialises)
    __shared__ u64 wsum[AGG_NT / 64][4];
    for (int d = 32; d >= 1; d >>= 1) my_global += __shfl_xor(my_global, d, 64);
    u64 ms = 0;
    if (blockIdx.x == 0)                       // k_map's stats: tokens, lds hits, global ops, long
        for (u32 w = tid >> 2; w < a.nsrc; w += AGG_NT / 4) ms += a.map_stats[(u64)w * 4 + (tid & 3)];
    for (int d = 32; d >= 4; d >>= 1) ms += __shfl_xor(ms, d, 64);
    if ((tid & 63) < 4) wsum[tid >> 6][tid & 3] = ms + ((tid & 63) == 2 ? my_global : 0);
    __syncthreads();
    if (tid < 4) {
        u64 t = 0;
        for (int w = 0; w < AGG_NT / 64; w++) t += wsum[w][tid];
        u64* dst[4] = {&a.st->tokens, &a.st->lds_hits, &a.st->global_ops, &a.st->long_tokens};
        if (t) atomicAdd(dst[tid], t);
    }
}

}  // namespace wcg
