// wcg_sort.h - the key sort of DoReduce + Merge on gfx950 (sort.Strings, mapreduce.go:268,309).
//
// Records (wcg_common.h Rec) are ordered by their 128-bit big-endian key prefix, which is Go's
// bytewise string order for keys <= 15 bytes (fact F4).  Keys of 16+ bytes that share a prefix
// are ordered by their full bytes afterwards (tie groups).
//
//   sample sort   k_ss_sample -> (k_tile_sort + k_merge over the sample) -> k_ss_hist ->
//                 scan -> k_ss_scatter -> k_ss_bucket: the sample's order statistics split the
//                 records into B buckets of ~SS_TARGET records (sampling keeps buckets even
//                 whatever the key distribution: UTF-8 words share their first bytes, which is
//                 what makes an MSD radix sort's buckets collapse); every bucket is then sorted
//                 in one workgroup's LDS.  The order is (prefix, record index), a total order, so
//                 splitters are unique and equal prefixes cannot pile into one bucket.  Two
//                 passes over the records instead of log2(n / 2048) merge passes.
//   tie groups    k_tie_mark + k_tie_sort: runs of long keys with one 16-byte prefix, sorted
//                 in parallel per group by the next 16 bytes (cached), then by the rest.
//   merge runs    k_merge_runs: pairwise merge passes over k sorted runs (the cross-GPU Merge).
#pragma once
#include "wcg_common.h"

namespace wcg {

__device__ __forceinline__ bool pre_lt(u64 ah, u64 al, u64 bh, u64 bl) { return ah < bh || (ah == bh && al < bl); }
__device__ __forceinline__ bool key3_lt(u64 ah, u64 al, u32 ai, u64 bh, u64 bl, u32 bi) {
    return ah < bh || (ah == bh && (al < bl || (al == bl && ai < bi)));
}

// ---------------------------------------------------------------- LDS bitonic network
// Sorts P (a power of two) entries (hi, lo, pos) in LDS by that triple, NT threads.  Thread t
// takes compare-exchange pairs t, t + NT, ...; a block of 64 consecutive pairs belongs to one wave
// and, for compare distances j <= 64, touches only its own 128 entries - so those stages (most of
// the network: 49 of 55 for P = 1024) are ordered by a wave barrier, and only stages with
// j >= 128 pay a workgroup barrier.  The caller's __syncthreads precedes and follows the call.
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int NT>
__device__ __forceinline__ void lds_bitonic(u64* kh, u64* kl, uint16_t* kp, u32 P) {
    const u32 tid = threadIdx.x;
    for (u32 k = 2; k <= P; k <<= 1)
        for (u32 j = k >> 1; j > 0; j >>= 1) {
            const bool wide = j >= 128;
            if (wide) __syncthreads();
            for (u32 t = tid; t < P / 2; t += NT) {
                const u32 i = 2 * t - (t & (j - 1)), p = i + j;
                const u64 ah = kh[i], al = kl[i], bh = kh[p], bl = kl[p];
                const uint16_t ai = kp[i], bi = kp[p];
                if (key3_lt(bh, bl, bi, ah, al, ai) == ((i & k) == 0)) {
                    kh[i] = bh; kl[i] = bl; kp[i] = bi;
                    kh[p] = ah; kl[p] = al; kp[p] = ai;
                }
            }
            if (wide) __syncthreads();
            else wave_sync_lds();
        }
}

// ---- bitonic network in registers: thread t of NT holds entries i = t * E + e (e < E) of
//      P = NT * E.  Stages with compare distance j < E are register compare-exchanges, j < 64 E
//      lane exchanges within the wave (__shfl_xor by j / E), and only j >= 64 E (3 of 55 stages
//      for P = 1024) go through LDS with a workgroup barrier.  (An LDS network reads and writes
//      both entries of every pair at every stage: 18 LDS operations per thread and stage.)
__device__ __forceinline__ u64 shfl_xor64(u64 v, int d) {
    const u32 lo = (u32)__shfl_xor((int)(u32)v, d, 64), hi = (u32)__shfl_xor((int)(u32)(v >> 32), d, 64);
    return (u64)hi << 32 | lo;
}
template <int E, int J>
__device__ __forceinline__ void rb_local(u64 (&h)[E], u64 (&l)[E], u32 (&q)[E], u32 k) {   // j = J < E
    const u32 t = threadIdx.x;
#pragma unroll
    for (int e = 0; e < E; e++) {
        if (e & J) continue;
        const int f = e | J;
        const bool asc = (((u32)(t * E + e)) & k) == 0;
        if (key3_lt(h[f], l[f], q[f], h[e], l[e], q[e]) == asc) {
            const u64 th = h[e], tl = l[e]; const u32 tq = q[e];
            h[e] = h[f]; l[e] = l[f]; q[e] = q[f];
            h[f] = th; l[f] = tl; q[f] = tq;
        }
    }
}
#ifndef WCG_SORT_NET
#define WCG_SORT_NET 1
#endif
#ifndef WCG_SORT_NET_BIG
#define WCG_SORT_NET_BIG 0     // 1: the 8-entry networks (buckets of 1025-2048 records) unrolled too (177 VGPRs: measured no faster)
#endif
#ifndef WCG_SORT_NET_FENCE
#define WCG_SORT_NET_FENCE 1
#endif
// ---- the same network with every stage unrolled (r03): the compare distance is a constant, so
//      the lane exchanges are single cross-lane moves (DPP quad_perm for 1 and 2, DPP row_ror:8
//      for 8, ds_swizzle for 4 and 16, v_permlane32_swap for 32) instead of ds_bpermute with an
//      address, and the compare-exchanges are selects instead of branches.  The position q is a
//      payload only: equal prefixes may end in any order (the tie sort orders long keys; repeated
//      inline keys are merged), so a pair compares (hi, lo) alone.  (The loop form ran ~48 VALU
//      per entry and stage: C4's bucket sorts were 1.5 ms.)
template <int D>
__device__ __forceinline__ u32 lane_xor(u32 v) {
    if constexpr (D == 1) return (u32)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
    else if constexpr (D == 2) return (u32)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad_perm 2,3,0,1
    else if constexpr (D == 4) return (u32)__builtin_amdgcn_ds_swizzle((int)v, (4 << 10) | 0x1F);
    else if constexpr (D == 8) return (u32)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    else if constexpr (D == 16) return (u32)__builtin_amdgcn_ds_swizzle((int)v, (16 << 10) | 0x1F);
    else {
        static_assert(D == 32, "lane_xor: distance 1..32");
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);   // r[0]: lanes 32-63 hold
        return (threadIdx.x & 32) ? r[0] : r[1];                               // lanes 0-31 of v, r[1] vice versa
    }
}
template <int D>
__device__ __forceinline__ u64 lane_xor64(u64 v) {
    return (u64)lane_xor<D>((u32)(v >> 32)) << 32 | lane_xor<D>((u32)v);
}
__device__ __forceinline__ bool hl_lt(u64 ah, u64 al, u64 bh, u64 bl) { return ah < bh || (ah == bh && al < bl); }
// keep (p) if the pair's order asks for it: keep_min takes p when p < mine, the other side when
// mine < p (both sides evaluate the same comparison, so a pair always swaps consistently)
// (x < y when dir, y < x otherwise, as lane-mask logic: a select between two comparisons was
// materialised through VGPRs)
__device__ __forceinline__ bool hl_dir_lt(bool dir, u64 xh, u64 xl, u64 yh, u64 yl) {
    const bool heq = xh == yh, lt = (xh < yh) | (heq & (xl < yl)), eq = heq & (xl == yl);
    return (dir & lt) | (!dir & !lt & !eq);
}
__device__ __forceinline__ void net_take(bool keep_min, u64& h, u64& l, u32& q, u64 ph, u64 pl, u32 pq) {
    const bool take = hl_dir_lt(keep_min, ph, pl, h, l);
    h = take ? ph : h; l = take ? pl : l; q = take ? pq : q;
}
template <int NT, int E, u32 K, u32 J>
__device__ __forceinline__ void net_stage(u64 (&h)[E], u64 (&l)[E], u32 (&q)[E], u64* kh, u64* kl, uint16_t* kp) {
    const u32 t = threadIdx.x;
    if constexpr (J < (u32)E) {                   // both entries in this thread
#pragma unroll
        for (int e = 0; e < E; e++) {
            if (e & J) continue;
            const int f = e | (int)J;
            const bool asc = (((u32)(t * E + e)) & K) == 0;
            const bool sw = hl_dir_lt(asc, h[f], l[f], h[e], l[e]);
            const u64 eh = h[e], el = l[e]; const u32 eq = q[e];
            h[e] = sw ? h[f] : eh; l[e] = sw ? l[f] : el; q[e] = sw ? q[f] : eq;
            h[f] = sw ? eh : h[f]; l[f] = sw ? el : l[f]; q[f] = sw ? eq : q[f];
        }
    } else {
        // J >= E: the pair's direction depends on the thread only
        const u32 i0 = t * E;
        const bool keep_min = ((i0 & J) == 0) == ((i0 & K) == 0);
        if constexpr (J < 64u * E) {
            constexpr int D = (int)(J / E);
#pragma unroll
            for (int e = 0; e < E; e++) {
                const u64 ph = lane_xor64<D>(h[e]), pl = lane_xor64<D>(l[e]);
                const u32 pq = lane_xor<D>(q[e]);
                net_take(keep_min, h[e], l[e], q[e], ph, pl, pq);
            }
        } else {
            __syncthreads();                      // the previous LDS stage's readers are done
#pragma unroll
            for (int e = 0; e < E; e++) { const u32 i = t * E + e; kh[i] = h[e]; kl[i] = l[e]; kp[i] = (uint16_t)q[e]; }
            __syncthreads();
#pragma unroll
            for (int e = 0; e < E; e++) {
                const u32 i = (t * E + e) ^ J;
                net_take(keep_min, h[e], l[e], q[e], kh[i], kl[i], kp[i]);
            }
        }
    }
}
template <int NT, int E, u32 K, u32 J>
__device__ __forceinline__ void net_stages_j(u64 (&h)[E], u64 (&l)[E], u32 (&q)[E], u64* kh, u64* kl, uint16_t* kp) {
    net_stage<NT, E, K, J>(h, l, q, kh, kl, kp);
#if WCG_SORT_NET_FENCE
    __builtin_amdgcn_sched_barrier(0);            // stages stay apart (register pressure)
#endif
    if constexpr (J > 1) net_stages_j<NT, E, K, J / 2>(h, l, q, kh, kl, kp);
}
template <int NT, int E, u32 K>
__device__ __forceinline__ void net_stages_k(u64 (&h)[E], u64 (&l)[E], u32 (&q)[E], u64* kh, u64* kl, uint16_t* kp) {
    net_stages_j<NT, E, K, K / 2>(h, l, q, kh, kl, kp);
    if constexpr (K < (u32)NT * E) net_stages_k<NT, E, K * 2>(h, l, q, kh, kl, kp);
}

template <int NT, int E>
__device__ __forceinline__ void reg_bitonic_unrolled(u64 (&h)[E], u64 (&l)[E], u32 (&q)[E], u64* kh, u64* kl, uint16_t* kp) {
    const u32 t = threadIdx.x;
    net_stages_k<NT, E, 2>(h, l, q, kh, kl, kp);
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; e++) { const u32 i = t * E + e; kh[i] = h[e]; kl[i] = l[e]; kp[i] = (uint16_t)q[e]; }
    __syncthreads();
}

// ---- r04: the same unrolled network on ONE 64-bit word per record and the position.  The word
//      is the record's (hi, lo) order compressed to the bucket: hi - min hi over the bucket, which
//      needs 64 - s bits (s = leading zeros of the bucket's hi range), followed by the top s bits
//      of lo.  The compressed order agrees with (hi, lo) except inside runs of equal words, which
//      the thread holding each run's first entry then insertion-sorts by the full (hi, lo) (an
//      all-hi-equal bucket - C4's Greek and Cyrillic words share their first 8 bytes - compares lo
//      alone).  A pair moves 3 dwords across lanes instead of 5 and compares 64 bits instead of
//      128.  Records' words are clamped below all ones, the padding's word.  A bucket with a run
//      longer than SB_RUN_MAX (records sharing a 16-byte prefix: long-key tie groups) is sorted
//      again by the (hi, lo) network.
#ifndef WCG_SORT_HIONLY
#define WCG_SORT_HIONLY 1
#endif
#ifndef WCG_SORT_HIONLY_BIG
#define WCG_SORT_HIONLY_BIG 1          // the 8-entry networks (buckets of 1025-2048) too
#endif
__device__ __forceinline__ bool h_dir_lt(bool dir, u64 x, u64 y) {
    const bool lt = x < y, eq = x == y;
    return (dir & lt) | (!dir & !lt & !eq);
}
template <int NT, int E, u32 K, u32 J>
__device__ __forceinline__ void net_stage_hi(u64 (&h)[E], u32 (&q)[E], u64* kh, uint16_t* kp) {
    const u32 t = threadIdx.x;
    if constexpr (J < (u32)E) {
#pragma unroll
        for (int e = 0; e < E; e++) {
            if (e & J) continue;
            const int f = e | (int)J;
            const bool asc = (((u32)(t * E + e)) & K) == 0;
            const bool sw = h_dir_lt(asc, h[f], h[e]);
            const u64 eh = h[e]; const u32 eq = q[e];
            h[e] = sw ? h[f] : eh; q[e] = sw ? q[f] : eq;
            h[f] = sw ? eh : h[f]; q[f] = sw ? eq : q[f];
        }
    } else {
        const u32 i0 = t * E;
        const bool keep_min = ((i0 & J) == 0) == ((i0 & K) == 0);
        if constexpr (J < 64u * E) {
            constexpr int D = (int)(J / E);
#pragma unroll
            for (int e = 0; e < E; e++) {
                const u64 ph = lane_xor64<D>(h[e]);
                const u32 pq = lane_xor<D>(q[e]);
                const bool take = h_dir_lt(keep_min, ph, h[e]);
                h[e] = take ? ph : h[e]; q[e] = take ? pq : q[e];
            }
        } else {
            __syncthreads();
#pragma unroll
            for (int e = 0; e < E; e++) { const u32 i = t * E + e; kh[i] = h[e]; kp[i] = (uint16_t)q[e]; }
            __syncthreads();
#pragma unroll
            for (int e = 0; e < E; e++) {
                const u32 i = (t * E + e) ^ J;
                const u64 ph = kh[i]; const u32 pq = kp[i];
                const bool take = h_dir_lt(keep_min, ph, h[e]);
                h[e] = take ? ph : h[e]; q[e] = take ? pq : q[e];
            }
        }
    }
}
template <int NT, int E, u32 K, u32 J>
__device__ __forceinline__ void net_stages_j_hi(u64 (&h)[E], u32 (&q)[E], u64* kh, uint16_t* kp) {
    net_stage_hi<NT, E, K, J>(h, q, kh, kp);
#if WCG_SORT_NET_FENCE
    __builtin_amdgcn_sched_barrier(0);
#endif
    if constexpr (J > 1) net_stages_j_hi<NT, E, K, J / 2>(h, q, kh, kp);
}
template <int NT, int E, u32 K>
__device__ __forceinline__ void net_stages_k_hi(u64 (&h)[E], u32 (&q)[E], u64* kh, uint16_t* kp) {
    net_stages_j_hi<NT, E, K, K / 2>(h, q, kh, kp);
    if constexpr (K < (u32)NT * E) net_stages_k_hi<NT, E, K * 2>(h, q, kh, kp);
}
#ifndef SB_RUN_MAX
#define SB_RUN_MAX 32
#endif
// w, q sorted by the compressed word: leaves (hi, lo, position) in kh/kl/kp sorted by (hi, lo)
// over [0, m) and returns true, or false (a run longer than SB_RUN_MAX; kh/kl/kp undefined)
template <int NT, int E>
__device__ __forceinline__ bool reg_bitonic_unrolled_hi(u64 (&w)[E], u32 (&q)[E], const Rec* X, u32 m, u64* kh,
                                                        u64* kl, uint16_t* kp) {
    const u32 t = threadIdx.x;
    net_stages_k_hi<NT, E, 2>(w, q, kh, kp);
    __syncthreads();   // the network's last LDS stage has read kh/kp
#pragma unroll
    for (int e = 0; e < E; e++) { const u32 i = t * E + e; kh[i] = w[e]; kp[i] = (uint16_t)q[e]; }
    __syncthreads();
    // runs of equal words: the thread with a run's first entry will sort it
    bool too_long = false;
    u64 runs = 0;                     // byte e: the length of the run starting at entry e (0: none)
#pragma unroll
    for (int e = 0; e < E; e++) {
        const u32 i = t * E + e;
        if (i + 1 >= m || kh[i + 1] != kh[i] || (i > 0 && kh[i - 1] == kh[i])) continue;
        u32 r = i + 2;
        while (r < m && r - i <= SB_RUN_MAX && kh[r] == kh[i]) r++;
        too_long |= r - i > SB_RUN_MAX;
        runs |= (u64)(r - i) << (8 * e);
    }
    // the records' (hi, lo) by sorted position (the bucket's region is L2-resident)
    u64 ch[E], cl[E];
#pragma unroll
    for (int e = 0; e < E; e++) {
        const bool r = q[e] < m;
        const Rec& x = X[r ? q[e] : 0];
        ch[e] = r ? x.hi : ~0ull; cl[e] = r ? x.lo : ~0ull;
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; e++) { const u32 i = t * E + e; kh[i] = ch[e]; kl[i] = cl[e]; }
    if (__syncthreads_or(too_long)) return false;
    for (; runs; runs &= runs - 1) {   // insertion sorts, one run at a time (registers: occupancy)
        const u32 e = (u32)__builtin_ctzll(runs) >> 3;
        const u32 i = t * E + e, r = i + (u32)(runs >> (8 * e) & 0xFF);
        runs &= ~(0xFFull << (8 * e));
        runs |= 1ull << (8 * e);          // the loop's own step clears this bit
        for (u32 x = i + 1; x < r; x++) {
            const u64 vh = kh[x], vl = kl[x];
            const uint16_t pv = kp[x];
            u32 y = x;
            while (y > i && (kh[y - 1] > vh || (kh[y - 1] == vh && kl[y - 1] > vl))) {
                kh[y] = kh[y - 1]; kl[y] = kl[y - 1]; kp[y] = kp[y - 1]; y--;
            }
            kh[y] = vh; kl[y] = vl; kp[y] = pv;
        }
    }
    __syncthreads();
    return true;
}

// the loop form: (hi, lo, position) order
template <int NT, int E>
__device__ __forceinline__ void reg_bitonic(u64 (&h)[E], u64 (&l)[E], u32 (&q)[E], u64* kh, u64* kl, uint16_t* kp) {
    constexpr u32 P = NT * E;
    const u32 t = threadIdx.x;
    for (u32 k = 2; k <= P; k <<= 1)
        for (u32 j = k >> 1; j > 0; j >>= 1) {
            if (j < (u32)E) {
                if (j == 1) rb_local<E, 1>(h, l, q, k);
                else if (E > 2 && j == 2) rb_local<E, (E > 2 ? 2 : 1)>(h, l, q, k);
                else if (E > 4 && j == 4) rb_local<E, (E > 4 ? 4 : 1)>(h, l, q, k);
                continue;
            }
            u64 bh[E], bl[E];
            u32 bq[E];
            if (j < 64u * E) {
                const int d = (int)(j / E);
#pragma unroll
                for (int e = 0; e < E; e++) {
                    bh[e] = shfl_xor64(h[e], d); bl[e] = shfl_xor64(l[e], d);
                    bq[e] = (u32)__shfl_xor((int)q[e], d, 64);
                }
            } else {
                __syncthreads();                      // the previous stage's readers are done
#pragma unroll
                for (int e = 0; e < E; e++) { const u32 i = t * E + e; kh[i] = h[e]; kl[i] = l[e]; kp[i] = (uint16_t)q[e]; }
                __syncthreads();
#pragma unroll
                for (int e = 0; e < E; e++) { const u32 i = (t * E + e) ^ j; bh[e] = kh[i]; bl[e] = kl[i]; bq[e] = kp[i]; }
            }
#pragma unroll
            for (int e = 0; e < E; e++) {
                const u32 i = t * E + e;
                const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
                if (key3_lt(bh[e], bl[e], bq[e], h[e], l[e], q[e]) == keep_min) { h[e] = bh[e]; l[e] = bl[e]; q[e] = bq[e]; }
            }
        }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; e++) { const u32 i = t * E + e; kh[i] = h[e]; kl[i] = l[e]; kp[i] = (uint16_t)q[e]; }
    __syncthreads();
}
// ---------------------------------------------------------------- merge sort (the sample, runs)
// k_tile_sort orders each 2048-record tile by an LDS bitonic network, stable (ties by position),
// then k_merge passes double the run length (A first on equal prefixes: stable).  A stable sort
// on (hi, lo) of records stored in index order IS the (hi, lo, index) order the sample sort
// needs for its splitters.
constexpr int TS_NT = 1024, TS_TILE = 2048;
constexpr int MG_NT = 256, MG_CHUNK = 1024;

__global__ __launch_bounds__(TS_NT) void k_tile_sort(const Rec* in, Rec* out, u64 n) {
    __shared__ u64 sh[TS_TILE], sl[TS_TILE];
    __shared__ uint16_t si[TS_TILE];
    const u64 base = (u64)blockIdx.x * TS_TILE;
    const int tid = threadIdx.x;
    for (int k = 0; k < TS_TILE / TS_NT; k++) {
        const int i = k * TS_NT + tid;
        const u64 g = base + i;
        if (g < n) {
            const Rec r = in[g];
            sh[i] = r.hi; sl[i] = r.lo;
        } else {                                  // padding: no key has an all-0xFF prefix
            sh[i] = ~0ull; sl[i] = ~0ull;
        }
        si[i] = (uint16_t)i;
    }
    __syncthreads();
    lds_bitonic<TS_NT>(sh, sl, si, TS_TILE);
    __syncthreads();
    for (int k = 0; k < TS_TILE / TS_NT; k++) {
        const int i = k * TS_NT + tid;
        if (base + i < n) out[base + i] = in[base + si[i]];
    }
}

// merge path: number of A records among the first d outputs of merge(A, B) (A first on equal
// prefixes).  One wave, 64-way search: each round samples 64 split candidates.
__device__ __forceinline__ u64 merge_split(const Rec* A, u64 la, const Rec* B, u64 lb, u64 d, int lane) {
    u64 lo = d > lb ? d - lb : 0, hi = d < la ? d : la;
    while (hi > lo) {
        const u64 s = hi - lo;
        const u64 p = s <= 64 ? lo + lane : lo + (u64)lane * s / 64;
        bool t = false;
        if (p < hi) {
            const Rec& x = A[p];
            const Rec& y = B[d - 1 - p];
            t = !pre_lt(y.hi, y.lo, x.hi, x.lo);
        }
        const int c = __popcll(__ballot(t));
        if (s <= 64) return lo + c;
        const u64 nlo = c > 0 ? __shfl(p, c - 1) + 1 : lo;
        const u64 nhi = c < 64 ? __shfl(p, c) : hi;
        lo = nlo; hi = nhi;
    }
    return lo;
}

// merge A = in[a0, a0 + la) and B = in[a0 + la, a0 + la + lb) for the outputs [d0, d1) of that
// pair, d1 - d0 <= 1024 (workgroup-cooperative)
__device__ __forceinline__ void merge_block(const Rec* in, Rec* out, u64 a0, u64 la, u64 lb, u64 d0, u64 d1) {
    __shared__ u64 sh[MG_CHUNK], sl[MG_CHUNK];
    __shared__ u64 split[2];
    const Rec* A = in + a0;
    const Rec* B = A + la;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (wv < 2) {
        const u64 sp = merge_split(A, la, B, lb, wv ? d1 : d0, lane);
        if (lane == 0) split[wv] = sp;
    }
    __syncthreads();
    const u64 i0 = split[0], i1 = split[1];
    const u64 j0 = d0 - i0;
    const int na = (int)(i1 - i0), m = (int)(d1 - d0);
    Rec r[MG_CHUNK / MG_NT];
#pragma unroll
    for (int k = 0; k < MG_CHUNK / MG_NT; k++) {
        const int e = k * MG_NT + tid;
        if (e < m) {
            r[k] = e < na ? A[i0 + e] : B[j0 + (e - na)];
            sh[e] = r[k].hi; sl[e] = r[k].lo;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < MG_CHUNK / MG_NT; k++) {
        const int e = k * MG_NT + tid;
        if (e >= m) continue;
        const u64 xh = r[k].hi, xl = r[k].lo;
        int lo, hi, pos;
        if (e < na) {                              // B window records strictly below x
            lo = na; hi = m;
            while (lo < hi) { const int mid = (lo + hi) >> 1; if (pre_lt(sh[mid], sl[mid], xh, xl)) lo = mid + 1; else hi = mid; }
            pos = e + (lo - na);
        } else {                                   // A window records at or below x
            lo = 0; hi = na;
            while (lo < hi) { const int mid = (lo + hi) >> 1; if (!pre_lt(xh, xl, sh[mid], sl[mid])) lo = mid + 1; else hi = mid; }
            pos = (e - na) + lo;
        }
        out[a0 + d0 + pos] = r[k];
    }
    __syncthreads();                               // LDS reused by the caller's next pair
}

// one merge pass: runs of length w -> 2w; workgroup b writes outputs [b * 1024, +1024)
__global__ __launch_bounds__(MG_NT) void k_merge(const Rec* in, Rec* out, u64 n, u64 w) {
    const u64 c0 = (u64)blockIdx.x * MG_CHUNK;
    const u64 a0 = c0 / (2 * w) * (2 * w);
    const u64 la = n - a0 < w ? n - a0 : w;
    const u64 rest = n - a0 - la;
    const u64 lb = rest < w ? rest : w;
    const u64 d0 = c0 - a0;                        // runs of 2w >= 4096 records: the chunk is
    merge_block(in, out, a0, la, lb, d0, d0 + MG_CHUNK < la + lb ? d0 + MG_CHUNK : la + lb);   // in one pair
}

// one merge pass over runs of any length: b0[0] = 0 <= b0[1] <= ... <= b0[nr] = n are the
// boundaries of the nr original runs; after passes of width s (1, 2, 4, ...) runs [2js, 2js + s)
// and [2js + s, 2js + 2s) are merged.  Workgroup blk writes outputs [blk * 1024, +1024), which
// may cover the ends of several pairs (runs of any length): it merges its part of each.
__global__ __launch_bounds__(MG_NT) void k_merge_runs(const Rec* in, Rec* out, const u64* b0, u32 nr, u32 s) {
    const u64 c0 = (u64)blockIdx.x * MG_CHUNK, n = b0[nr];
    const u64 c1 = c0 + MG_CHUNK < n ? c0 + MG_CHUNK : n;
    auto B = [&](u64 r) -> u64 { return b0[r < nr ? r : nr]; };
    const u32 npairs = (nr + 2 * s - 1) / (2 * s);
    u32 lo = 0, hi = npairs;                       // the last pair starting at or before c0
    while (hi - lo > 1) {
        const u32 mid = (lo + hi) / 2;
        if (B((u64)2 * mid * s) <= c0) lo = mid; else hi = mid;
    }
    for (u32 j = lo; j < npairs; j++) {            // workgroup-uniform
        const u64 a0 = B((u64)2 * j * s), am = B((u64)2 * j * s + s), ae = B((u64)2 * j * s + 2 * s);
        if (a0 >= c1) break;
        if (ae <= c0 || ae == a0) continue;
        const u64 d0 = (c0 > a0 ? c0 : a0) - a0, d1 = (c1 < ae ? c1 : ae) - a0;
        merge_block(in, out, a0, am - a0, ae - am, d0, d1);
    }
}

// ---------------------------------------------------------------- scans
// exclusive scan of u64 (in place) by one workgroup of 1024 threads; total in *total
__global__ __launch_bounds__(1024) void k_scan_u64(u64* v, u64 n, u64* total) {
    __shared__ u64 ws[16];
    __shared__ u64 carry_s;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) carry_s = 0;
    __syncthreads();
    for (u64 base = 0; base < n; base += 1024 * 4) {
        u64 x[4], s = 0;
        for (int k = 0; k < 4; k++) {
            u64 i = base + (u64)tid * 4 + k;
            x[k] = i < n ? v[i] : 0;
            s += x[k];
        }
        u64 incl = s;
        for (int d = 1; d < 64; d <<= 1) { u64 y = __shfl_up(incl, d, 64); if (lane >= d) incl += y; }
        if (lane == 63) ws[w] = incl;
        __syncthreads();
        u64 wpre = 0, all = 0;
        for (int k = 0; k < 16; k++) { if (k < w) wpre += ws[k]; all += ws[k]; }
        u64 run = carry_s + wpre + incl - s;
        for (int k = 0; k < 4; k++) {
            u64 i = base + (u64)tid * 4 + k;
            if (i < n) v[i] = run;
            run += x[k];
        }
        __syncthreads();
        if (tid == 0) carry_s += all;
        __syncthreads();
    }
    if (tid == 0 && total) *total = carry_s;
}

// multi-block exclusive scan of u32 (in place): k_scan_part sums SC_SEG-element segments into
// part[], k_scan_u64 scans part[], k_scan_apply scans each segment from its base
constexpr int SC_NT = 1024, SC_IPT = 8, SC_SEG = SC_NT * SC_IPT;

__device__ __forceinline__ u64 block_sum_u64(u64 s, u64* ws) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
    if (lane == 0) ws[w] = s;
    __syncthreads();
    u64 all = 0;
    for (int k = 0; k < (int)(blockDim.x / 64); k++) all += ws[k];
    __syncthreads();
    return all;
}

__global__ __launch_bounds__(SC_NT) void k_scan_part(const u32* v, u64 n, u64* part) {
    __shared__ u64 ws[SC_NT / 64];
    const u64 base = (u64)blockIdx.x * SC_SEG;
    u64 s = 0;
#pragma unroll
    for (int k = 0; k < SC_IPT; k++) {
        const u64 i = base + (u64)k * SC_NT + threadIdx.x;
        s += i < n ? v[i] : 0u;
    }
    const u64 all = block_sum_u64(s, ws);
    if (threadIdx.x == 0) part[blockIdx.x] = all;
}

__global__ __launch_bounds__(SC_NT) void k_scan_apply(u32* v, u64 n, const u64* part) {
    __shared__ u64 ws[SC_NT / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u64 base = (u64)blockIdx.x * SC_SEG + (u64)tid * SC_IPT;   // consecutive per thread
    u32 x[SC_IPT];
    u64 s = 0;
#pragma unroll
    for (int k = 0; k < SC_IPT; k++) { x[k] = base + k < n ? v[base + k] : 0u; s += x[k]; }
    u64 incl = s;
    for (int d = 1; d < 64; d <<= 1) { const u64 y = __shfl_up(incl, d, 64); if (lane >= d) incl += y; }
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    u64 pre = 0;
    for (int k = 0; k < w; k++) pre += ws[k];
    u64 run = part[blockIdx.x] + pre + incl - s;
#pragma unroll
    for (int k = 0; k < SC_IPT; k++) {
        if (base + k < n) v[base + k] = (u32)run;
        run += x[k];
    }
}

// one segment (m <= SC_ONE_MAX): one workgroup (walking several segments in order with a running
// carry took 49 us on C2's 50K-entry histogram, against 18 us for the three-kernel scan: each
// segment waits for its loads in turn)
constexpr u64 SC_ONE_MAX = SC_SEG;
__global__ __launch_bounds__(SC_NT) void k_scan_apply1(u32* v, u64 m) {
    __shared__ u64 ws[SC_NT / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    u64 carry = 0;
    for (u64 seg = 0; seg < m; seg += SC_SEG) {
        const u64 base = seg + (u64)tid * SC_IPT;
        u32 x[SC_IPT];
        u64 s = 0;
#pragma unroll
        for (int k = 0; k < SC_IPT; k++) { x[k] = base + k < m ? v[base + k] : 0u; s += x[k]; }
        u64 incl = s;
        for (int d = 1; d < 64; d <<= 1) { const u64 y = __shfl_up(incl, d, 64); if (lane >= d) incl += y; }
        if (lane == 63) ws[w] = incl;
        __syncthreads();
        u64 pre = 0, all = 0;
        for (int k = 0; k < SC_NT / 64; k++) { if (k < w) pre += ws[k]; all += ws[k]; }
        u64 run = carry + pre + incl - s;
#pragma unroll
        for (int k = 0; k < SC_IPT; k++) {
            if (base + k < m) v[base + k] = (u32)run;
            run += x[k];
        }
        carry += all;
        __syncthreads();                  // ws is rewritten by the next segment
    }
}

// ---------------------------------------------------------------- sample sort
#ifndef WCG_SS_TARGET
#define WCG_SS_TARGET 512
#endif
#ifndef WCG_SS_OVS
#define WCG_SS_OVS 8
#endif
constexpr u32 SS_TARGET = WCG_SS_TARGET;  // expected records per bucket (small buckets: many
                                          // workgroups sort at once, each bitonic network short)
constexpr u32 SS_OVS = WCG_SS_OVS;     // samples per bucket
constexpr u32 SS_MAXB = 32768;         // buckets (k_ss_hist / k_ss_scatter LDS: 4 B each)
constexpr int SS_NT = 256;             // hist / scatter workgroups, up to SS_LDSB buckets
constexpr int SSL_NT = 1024;           // hist / scatter workgroups above SS_LDSB buckets
constexpr u32 SS_TOP = 1024;           // top-level splitters staged in LDS above SS_LDSB buckets
constexpr u32 SB_CAP = 2048;           // bucket records sorted in LDS (18 B each: 36 KiB)
constexpr int SB_NT = 256;             // bucket sort workgroups
#ifndef WCG_SS_U
#define WCG_SS_U 2
#endif
#ifndef WCG_SS_TR
#define WCG_SS_TR 1                    // large B: workgroup-major histogram + k_ss_colscan
#endif
#ifndef WCG_SS_UX
#define WCG_SS_UX 2                    // the scatter's records per thread in flight (C4: 2 1.05 ms, 4 1.06, 8 1.09)
#endif
constexpr int SS_UX = WCG_SS_UX;
constexpr int SS_U = WCG_SS_U;         // records per thread in flight (hist / scatter; r03: 2 - 4 and 1
                                       // measured 40-70 us slower on C4's 2.4e7-record sort)
#ifndef WCG_SS_ABL
#define WCG_SS_ABL 0                   // diagnostics: 1 = k_ss_hist skips its global search levels (wrong order)
#endif

struct SortArgs {
    const Rec* rec;          // compacted records (index = position)
    u64 n;                   // records, or (nd set) the buffers' capacity
    const u64* nd;           // device-sized sorts: the record count in device memory (<= n), so
                             // that the host plans the launches without reading it back
    const Rec* smp;          // sorted sample: hi, lo, cnt = record index
    u64 S;                   // samples
    u32 B;                   // buckets
    u32 G;                   // hist/scatter workgroups
    u32* bid;                // bucket of every record
    u32* hist;               // [B][G] counts -> exclusive offsets (bucket-major)
    Rec* irec;               // records by bucket (n) ...
    Rec* irec2;              // ... and the scratch of the oversized-bucket path (n)
    Rec* out;                // sorted records
    u32 dedupe;              // merge repeated inline keys (record log jobs) while writing out
    u64* nkeys;              // distinct keys (dedupe)
    u64* sph; u64* spl; u32* spi;   // splitters 0..B-2 as arrays (hi, lo, record index): the
                                    // searches' global reads stay within 20 B per splitter (L2)
    u32* bstart;             // large B (SS_TR): hist is workgroup-major [G][B] and bstart[b] the
                             // start of bucket b (k_ss_colscan); null: hist is [B][G]
    u64* groups; u64* ngroups;   // r04: tie-group starts marked by the bucket sort (null: k_tie_mark)
    u64* tie_zero;           // r04: the tie sort's big-group counter, zeroed by k_tie_edge
    u32 cls2;                // r04: buckets of SB_CAP..SB_CAP2 records take k_ss_bucket<2> (else the
                             // global path: plans whose buckets average <= 1024 records)
};

// the records to sort: a.n, or the count the device holds (a plan made for another count only
// changes the buckets' sizes: samples repeat when S > n, and buckets may be empty or oversized)
__device__ __forceinline__ u64 ss_count(const SortArgs& a) { return a.nd ? (*a.nd < a.n ? *a.nd : a.n) : a.n; }

// sample j = record floor(j * n / S): stored in index order, so a stable sort gives the
// (hi, lo, index) order
__global__ void k_ss_sample(SortArgs a, Rec* smp) {
    const u64 j = blockIdx.x * (u64)blockDim.x + threadIdx.x;
    if (j >= a.S) return;
    const u64 i = j * ss_count(a) / a.S;
    const Rec r = a.rec[i];
    Rec s;
    s.hi = r.hi; s.lo = r.lo; s.cnt = i; s.ref = 0;
    smp[j] = s;
}

// splitter b (0 <= b < B - 1) = sample (b + 1) * S / B; bucket(x) = number of splitters <= x in
// the (hi, lo, record index) order - a total order, so equal prefixes spread over buckets
__device__ __forceinline__ const Rec& ss_splitter(const SortArgs& a, u32 b) { return a.smp[(u64)(b + 1) * a.S / a.B]; }

// the splitters as arrays (large B): 32768 splitters are 640 KiB, L2-resident, where the
// sample records they come from span 8 MiB (one 128-byte line per splitter)
__global__ void k_ss_split(SortArgs a) {
    const u32 b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b + 1 >= a.B) return;
    const Rec& s = ss_splitter(a, b);
    a.sph[b] = s.hi; a.spl[b] = s.lo; a.spi[b] = (u32)s.cnt;
}

// The logical workgroup of a hist / scatter block (its record range and histogram column).
// Within a bucket the scatter writes workgroup 0's records, then workgroup 1's, ...: a bucket's
// 128-byte lines are shared by neighbouring workgroups, and blocks are dispatched to the 8 XCDs
// round-robin, so with the identity mapping every shared line was written from up to four XCDs'
// L2s (partial-line write-backs).  Consecutive logical workgroups run on one XCD instead.
#ifndef WCG_SS_XCD
#define WCG_SS_XCD 1
#endif
__device__ __forceinline__ u32 ss_wg(const SortArgs& a) {
    const u32 b = blockIdx.x;
    if (!WCG_SS_XCD || (a.G & 7u)) return b;
    return (b & 7u) * (a.G >> 3) + (b >> 3);
}

__device__ __forceinline__ void ss_range(const SortArgs& a, u64& i0, u64& i1) {
    const u64 n = ss_count(a);
    const u32 g = ss_wg(a);
    i0 = n * g / a.G;
    i1 = n * (g + 1) / a.G;
}

// Up to SS_LDSB buckets every splitter is staged in LDS (a binary search of LDS reads), and the
// histogram is small: several workgroups fit a CU.
constexpr u32 SS_LDSB = 2048;

// Above SS_LDSB buckets (large key counts, C4): SS_TOP evenly spaced splitters in LDS narrow the
// search to ~B / SS_TOP splitters, and a few dependent (L2-resident) global reads finish it;
// 1024-thread workgroups keep 16 waves of searches in flight beside the 128 KiB histogram.
__device__ __forceinline__ u32 ss_top_index(const SortArgs& a, u32 t) { return (u32)((u64)(t + 1) * (a.B - 1) / (SS_TOP + 1)); }

template <bool SMALL>
__device__ __forceinline__ u32 ss_find(const SortArgs& a, u64 hi, u64 lo, u32 idx, const u64* sp_hi, const u64* sp_lo,
                                       const u32* sp_i) {
    u32 l = 0, h;
    if (SMALL) {
        h = a.B - 1;
        while (l < h) {
            const u32 mid = (l + h) >> 1;
            if (!key3_lt(hi, lo, idx, sp_hi[mid], sp_lo[mid], sp_i[mid])) l = mid + 1; else h = mid;
        }
        return l;
    }
    u32 tl = 0, th = SS_TOP;                      // top splitters <= x
    while (tl < th) {
        const u32 mid = (tl + th) >> 1;
        if (!key3_lt(hi, lo, idx, sp_hi[mid], sp_lo[mid], sp_i[mid])) tl = mid + 1; else th = mid;
    }
    l = tl > 0 ? ss_top_index(a, tl - 1) + 1 : 0;
    h = tl < SS_TOP ? ss_top_index(a, tl) : a.B - 1;
    while (l < h) {
        const u32 mid = (l + h) >> 1;
        const u64 sh = a.sph[mid];
        const bool lt = hi != sh ? hi < sh : key3_lt(hi, lo, idx, sh, a.spl[mid], a.spi[mid]);
        if (!lt) l = mid + 1; else h = mid;
    }
    return l;
}

template <bool SMALL>
__global__ __launch_bounds__(SMALL ? SS_NT : SSL_NT) void k_ss_hist(SortArgs a) {
    constexpr int NT = SMALL ? SS_NT : SSL_NT;
    constexpr u32 NSP = SMALL ? SS_LDSB : SS_TOP;
    __shared__ u32 h[SMALL ? SS_LDSB : SS_MAXB];
    __shared__ u64 sp_hi[NSP], sp_lo[NSP];
    __shared__ u32 sp_i[NSP];
    for (u32 b = threadIdx.x; b < a.B; b += NT) h[b] = 0;
    for (u32 t = threadIdx.x; t < NSP; t += NT) {
        const bool live = SMALL ? t + 1 < a.B : true;
        if (live) {
            if (SMALL) {
                const Rec& s = ss_splitter(a, t);
                sp_hi[t] = s.hi; sp_lo[t] = s.lo; sp_i[t] = (u32)s.cnt;
            } else {
                const u32 k = ss_top_index(a, t);
                sp_hi[t] = a.sph[k]; sp_lo[t] = a.spl[k]; sp_i[t] = a.spi[k];
            }
        }
    }
    __syncthreads();
    u64 i0, i1;
    ss_range(a, i0, i1);
    // an inline key searches as (key, 0): every copy of a repeated key (record log jobs) lands in
    // one bucket, so the bucket sort can merge them; long keys keep their index so equal 16-byte
    // prefixes still spread over buckets
    if (!SMALL) {
        // SS_U records per thread at a time: their global search steps issue together (each
        // search is a chain of dependent L2 reads)
        for (u64 i = i0 + threadIdx.x; i < i1; i += (u64)NT * SS_U) {
            u64 hi[SS_U], lo[SS_U];
            u32 si[SS_U], l[SS_U], m[SS_U];
#pragma unroll
            for (int k = 0; k < SS_U; k++) {
                const u64 j = i + (u64)k * NT;
                const Rec r = j < i1 ? a.rec[j] : Rec{~0ull, ~0ull, 0, 0};
                hi[k] = r.hi; lo[k] = r.lo;
                si[k] = (r.ref & LONG_FLAG) ? (u32)j : 0u;
            }
#pragma unroll
            for (int k = 0; k < SS_U; k++) {
                u32 tl = 0, th = SS_TOP;              // top splitters <= x (LDS)
                while (tl < th) {
                    const u32 mid = (tl + th) >> 1;
                    if (!key3_lt(hi[k], lo[k], si[k], sp_hi[mid], sp_lo[mid], sp_i[mid])) tl = mid + 1; else th = mid;
                }
                l[k] = tl > 0 ? ss_top_index(a, tl - 1) + 1 : 0;
                m[k] = (tl < SS_TOP ? ss_top_index(a, tl) : a.B - 1) - l[k];
            }
            while (!WCG_SS_ABL) {                     // lower bounds in [l, l + m), interleaved
                bool any = false;
                u64 sh[SS_U];
#pragma unroll
                for (int k = 0; k < SS_U; k++) {
                    sh[k] = m[k] ? a.sph[l[k] + m[k] / 2] : 0;
                    any |= m[k] != 0;
                }
                if (!any) break;
#pragma unroll
                for (int k = 0; k < SS_U; k++) {
                    if (!m[k]) continue;
                    const u32 half = m[k] / 2, mid = l[k] + half;
                    const bool lt = hi[k] != sh[k] ? hi[k] < sh[k]
                                                   : key3_lt(hi[k], lo[k], si[k], sh[k], a.spl[mid], a.spi[mid]);
                    if (!lt) { l[k] = mid + 1; m[k] -= half + 1; } else m[k] = half;
                }
            }
#pragma unroll
            for (int k = 0; k < SS_U; k++) {
                const u64 j = i + (u64)k * NT;
                if (j < i1) { a.bid[j] = l[k]; atomicAdd(&h[l[k]], 1u); }
            }
        }
        __syncthreads();
        if (a.bstart) {                          // one contiguous row per workgroup
            u32* row = a.hist + (u64)ss_wg(a) * a.B;
            for (u32 b = threadIdx.x; b < a.B; b += NT) row[b] = h[b];
        } else {
            for (u32 b = threadIdx.x; b < a.B; b += NT) a.hist[(u64)b * a.G + ss_wg(a)] = h[b];
        }
        return;
    }
    for (u64 i = i0 + threadIdx.x; i < i1; i += NT) {
        const Rec r = a.rec[i];
        const u32 si = (r.ref & LONG_FLAG) ? (u32)i : 0u;
        const u32 b = ss_find<SMALL>(a, r.hi, r.lo, si, sp_hi, sp_lo, sp_i);
        a.bid[i] = b;
        atomicAdd(&h[b], 1u);
    }
    __syncthreads();
    for (u32 b = threadIdx.x; b < a.B; b += NT) a.hist[(u64)b * a.G + ss_wg(a)] = h[b];
}

// Large B, r04: the search and the histogram as two kernels.  k_ss_hist<false> ran at one
// 1024-thread workgroup per CU (its 128 KiB histogram beside 1024 top splitters) with 75% of its
// wave cycles waiting on the ~5 dependent L2 reads each search made below the LDS levels.
// k_ss_find keeps SS_TOP2 top splitters' hi words in LDS (64 KiB: two workgroups per CU, twice the
// waves) so that only ~2 levels are left for L2; an equal hi word at an LDS level decides by the
// splitter's (lo, index) from the global arrays (exact, rare).  k_ss_count then histograms the
// bucket ids (4 bytes per record) with the 128 KiB LDS histogram.
#ifndef WCG_SS_SPLIT
#define WCG_SS_SPLIT 1
#endif
// r05: the top splitters sit in LDS in Eytzinger (breadth-first) order: node k of
// a perfect tree of SS_TOP_D levels at top_e[k], k = 1 .. 2^D - 1.  A sorted array searched by
// bisection sends every lane of a wave to the same few midpoints in its first levels, and those
// midpoints (multiples of large powers of two) all fall in one LDS bank: 92% of the search's LDS
// cycles were bank conflicts (r04_pmc_c4_1gib_final.txt).  Breadth-first, the nodes of the first
// levels are neighbours (different banks), and the descent k -> 2k + (x >= node) ends at leaf
// 2^D + (the number of top splitters <= x): the same count as the bisection.
constexpr u32 SS_TOP_D = 13;
constexpr u32 SS_TOP2 = (1u << SS_TOP_D) - 1;  // top splitters: 8191
constexpr int SSF_NT = 1024;
__device__ __forceinline__ u32 ss_ntop2(const SortArgs& a) { return a.B - 1 < SS_TOP2 ? a.B - 1 : SS_TOP2; }
__device__ __forceinline__ u32 ss_top2_index(const SortArgs& a, u32 t, u32 ntop) {
    return (t + 1) * (a.B - 1) / (ntop + 1);     // < 8192 * 32767 < 2^32: a 32-bit division
}
// the sorted position of breadth-first node k
__device__ __forceinline__ u32 ss_top_inorder(u32 k) {
    const u32 d = 31u - (u32)__builtin_clz(k), h = SS_TOP_D - 1 - d;
    return ((((k - (1u << d)) << 1) + 1) << h) - 1;
}
__global__ __launch_bounds__(SSF_NT) void k_ss_find(SortArgs a) {
    __shared__ u64 top_e[SS_TOP2 + 1];
    const u32 ntop = ss_ntop2(a);
    for (u32 k = threadIdx.x + 1; k <= SS_TOP2; k += SSF_NT) {
        const u32 t = ss_top_inorder(k);
        top_e[k] = t < ntop ? a.sph[ss_top2_index(a, t, ntop)] : ~0ull;   // past ntop: above every key
    }
    __syncthreads();
    const u64 n = ss_count(a);
    const u64 stride = (u64)gridDim.x * SSF_NT;
    for (u64 i = blockIdx.x * (u64)SSF_NT + threadIdx.x; i < n; i += stride * SS_U) {
        u64 hi[SS_U], lo[SS_U];
        u32 si[SS_U], l[SS_U], m[SS_U];
#pragma unroll
        for (int k = 0; k < SS_U; k++) {
            const u64 j = i + (u64)k * stride;
            const Rec r = j < n ? a.rec[j] : Rec{~0ull, ~0ull, 0, 0};
            hi[k] = r.hi; lo[k] = r.lo;
            // an inline key searches as (key, 0) (see k_ss_hist); long keys keep their index
            si[k] = (r.ref & LONG_FLAG) ? (u32)j : 0u;
        }
#pragma unroll
        for (int k = 0; k < SS_U; k++) {
            u32 e = 1;                                // top splitters <= x (LDS, hi words)
            for (u32 lev = 0; lev < SS_TOP_D; lev++) {
                const u64 sh = top_e[e];
                bool lt;
                if (hi[k] != sh) lt = hi[k] < sh;
                else {
                    const u32 t = ss_top_inorder(e);
                    if (t >= ntop) lt = true;         // padding (an all-ones prefix meets it)
                    else {
                        const u32 g = ss_top2_index(a, t, ntop);
                        lt = key3_lt(hi[k], lo[k], si[k], sh, a.spl[g], a.spi[g]);
                    }
                }
                e = 2 * e + (lt ? 0u : 1u);
            }
            const u32 tl = e - (1u << SS_TOP_D);
            l[k] = tl > 0 ? ss_top2_index(a, tl - 1, ntop) + 1 : 0;
            m[k] = (tl < ntop ? ss_top2_index(a, tl, ntop) : a.B - 1) - l[k];
        }
        while (true) {                                // lower bounds in [l, l + m), interleaved
            bool any = false;
            u64 sh[SS_U];
#pragma unroll
            for (int k = 0; k < SS_U; k++) {
                sh[k] = m[k] ? a.sph[l[k] + m[k] / 2] : 0;
                any |= m[k] != 0;
            }
            if (!any) break;
#pragma unroll
            for (int k = 0; k < SS_U; k++) {
                if (!m[k]) continue;
                const u32 half = m[k] / 2, mid = l[k] + half;
                const bool lt = hi[k] != sh[k] ? hi[k] < sh[k]
                                               : key3_lt(hi[k], lo[k], si[k], sh[k], a.spl[mid], a.spi[mid]);
                if (!lt) { l[k] = mid + 1; m[k] -= half + 1; } else m[k] = half;
            }
        }
#pragma unroll
        for (int k = 0; k < SS_U; k++) {
            const u64 j = i + (u64)k * stride;
            if (j < n) a.bid[j] = l[k];
        }
    }
}

// per logical workgroup (the scatter's record ranges): bucket counts of its records, one
// contiguous row per workgroup (k_ss_colscan turns the rows into offsets)
__global__ __launch_bounds__(SSL_NT) void k_ss_count(SortArgs a) {
    __shared__ u32 h[SS_MAXB];
    for (u32 b = threadIdx.x; b < a.B; b += SSL_NT) h[b] = 0;
    __syncthreads();
    u64 i0, i1;
    ss_range(a, i0, i1);
    constexpr int CU4 = 4;                            // bucket ids per thread in flight
    for (u64 i = i0 + threadIdx.x; i < i1; i += (u64)SSL_NT * CU4) {
        u32 b[CU4];
#pragma unroll
        for (int k = 0; k < CU4; k++) {
            const u64 j = i + (u64)k * SSL_NT;
            b[k] = j < i1 ? a.bid[j] : ~0u;
        }
#pragma unroll
        for (int k = 0; k < CU4; k++)
            if (b[k] != ~0u) atomicAdd(&h[b[k]], 1u);
    }
    __syncthreads();
    u32* row = a.hist + (u64)ss_wg(a) * a.B;
    for (u32 b = threadIdx.x; b < a.B; b += SSL_NT) row[b] = h[b];
}

// the sample of a small sort (S <= TS_TILE) by ranks: rank = the samples below it in the
// (hi, lo, sample index) order, a permutation.  One wave per sample: its 64 lanes compare the
// sample with S / 64 entries each of the sample staged in LDS, and the counts are summed across
// the wave.  (A one-workgroup network over 2048 entries took 37 us - 66 stages of lane exchanges
// on one CU; fewer lanes per sample left one long compare loop per wave, 49-195 us.)
constexpr int RK_NT = 256, RK_SPB = RK_NT / 64;   // samples per block: one per wave
__global__ __launch_bounds__(RK_NT) void k_ss_rank_sort(SortArgs a, Rec* smp) {
    __shared__ u64 sh[TS_TILE], sl[TS_TILE];
    const u32 S = (u32)a.S;
    const u64 n = ss_count(a);
    for (u32 j = threadIdx.x; j < S; j += RK_NT) {
        const Rec& r = a.rec[j * n / S];
        sh[j] = r.hi; sl[j] = r.lo;
    }
    __syncthreads();
    const u32 j = blockIdx.x * RK_SPB + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (j >= S) return;                      // wave-uniform
    const u64 h = sh[j], l = sl[j];
    u32 rank = 0;
    for (u32 k = lane; k < S; k += 64) rank += key3_lt(sh[k], sl[k], k, h, l, j) ? 1u : 0u;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) rank += __shfl_xor((int)rank, d, 64);
    if (lane != 0) return;
    Rec o;
    o.hi = h; o.lo = l; o.cnt = (u64)j * n / S; o.ref = 0;
    smp[rank] = o;
}

// records of workgroup g go to [hist[b][g], ...) of their bucket, whole (the bucket sort then
// reads its records from one small region instead of gathering them from the whole array); the
// order inside a bucket does not matter
template <bool SMALL>
__global__ __launch_bounds__(SMALL ? SS_NT : SSL_NT) void k_ss_scatter(SortArgs a) {
    constexpr int NT = SMALL ? SS_NT : SSL_NT;
    __shared__ u32 cur[SMALL ? SS_LDSB : SS_MAXB];
    if (!SMALL && a.bstart) {
        const u32* row = a.hist + (u64)ss_wg(a) * a.B;
        for (u32 b = threadIdx.x; b < a.B; b += NT) cur[b] = a.bstart[b] + row[b];
    } else {
        for (u32 b = threadIdx.x; b < a.B; b += NT) cur[b] = a.hist[(u64)b * a.G + ss_wg(a)];
    }
    __syncthreads();
    u64 i0, i1;
    ss_range(a, i0, i1);
    // SS_UX records per thread at a time: their loads, cursor atomics and stores issue together
    for (u64 i = i0 + threadIdx.x; i < i1; i += (u64)NT * SS_UX) {
        u32 b[SS_UX], d[SS_UX];
        Rec r[SS_UX];
#pragma unroll
        for (int k = 0; k < SS_UX; k++) {
            const u64 j = i + (u64)k * NT;
            if (j < i1) { b[k] = a.bid[j]; r[k] = a.rec[j]; }
        }
#pragma unroll
        for (int k = 0; k < SS_UX; k++)
            if (i + (u64)k * NT < i1) d[k] = atomicAdd(&cur[b[k]], 1u);
#pragma unroll
        for (int k = 0; k < SS_UX; k++)
            if (i + (u64)k * NT < i1) a.irec[d[k]] = r[k];
    }
}

// r05: the large-B scatter in two passes.  One pass (k_ss_scatter) put every
// record straight into its bucket among up to 32768: runs of ~3 records per (workgroup, bucket),
// so nearly every write was a lone 32-byte piece of a line.  Here pass 1 moves each record into
// its coarse bucket (bucket >> sh: at most 256, each the final range of 2^sh consecutive
// buckets) and pass 2, within that range, into its bucket.  A pass takes a tile of SX_T records:
// their keys ranked in LDS, one global cursor reservation per key present in the tile, then the
// tile written in key order (runs of SX_T / keys records: 16 in pass 1 at 256 coarse buckets,
// 32 in pass 2 at 128 buckets per range), every store coalesced with its neighbours.  Pass 2's
// tiles span one or two coarse ranges; a tile whose buckets span more than SX_NK (tiny ranges)
// reserves per record, as the one-pass scatter does.  Twice the record traffic of one pass, in
// whole lines.
#ifndef WCG_SS_SX
#define WCG_SS_SX 1
#endif
#ifndef WCG_SX_NT
#define WCG_SX_NT 1024
#endif
#ifndef WCG_SX_T
#define WCG_SX_T 4096
#endif
constexpr int SX_NT = WCG_SX_NT;
constexpr u32 SX_T = WCG_SX_T;             // records per tile (u16 positions in LDS)
constexpr int SX_R = SX_T / SX_NT;
constexpr u32 SX_NK = 1024;                // keys ranked in LDS
constexpr u32 SX_CS = 1024;                // coarse cursors 4 KiB apart: every workgroup of pass 1
                                           // reserves on all of them (one line each, not eight)
struct SxArgs {
    const Rec* in; const u32* bin;         // records and their buckets
    Rec* out; u32* bout;                   // pass 1 also moves the buckets (bout)
    u32* cur;                              // pass 1: coarse cursors (SX_CS apart); pass 2: bucket cursors
    u32 sh;                                // coarse bucket = bucket >> sh
};

// cursors at the bucket starts: fcur[b] = bstart[b], ccur[c] = bstart[c << sh]
__global__ void k_ss_sxinit(SortArgs a, u32* ccur, u32* fcur, u32 sh) {
    const u32 b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= a.B) return;
    const u32 s = a.bstart[b];
    fcur[b] = s;
    if ((b & ((1u << sh) - 1u)) == 0u) ccur[(b >> sh) * SX_CS] = s;
}

template <int PASS>
__global__ __launch_bounds__(SX_NT) void k_ss_sx(SortArgs a, SxArgs x) {
    __shared__ u32 hcnt[SX_NK];            // key counts -> the keys' first positions in the tile
    __shared__ u32 gb[SX_NK];              // the keys' reserved global positions
    __shared__ uint16_t perm[SX_T];        // tile record at position p (key order)
    __shared__ u32 pbk[SX_T];              // its bucket
    __shared__ u32 wred[2][SX_NT / 64];
    const u64 n = ss_count(a);
    const u64 t0 = (u64)blockIdx.x * SX_T;
    if (t0 >= n) return;                   // workgroup-uniform (device-sized sorts)
    const u32 m = (u32)(n - t0 < SX_T ? n - t0 : SX_T);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    u32 b[SX_R];
#pragma unroll
    for (int k = 0; k < SX_R; k++) {
        const u32 i = tid + k * SX_NT;
        b[k] = i < m ? x.bin[t0 + i] : ~0u;
    }
    u32 kmin = 0, nk;
    if (PASS == 1) {
        nk = ((a.B - 1u) >> x.sh) + 1u;
    } else {
        u32 lo = ~0u, hi = 0;
#pragma unroll
        for (int k = 0; k < SX_R; k++)
            if (b[k] != ~0u) { lo = min(lo, b[k]); hi = max(hi, b[k]); }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            lo = min(lo, (u32)__shfl_xor((int)lo, d, 64));
            hi = max(hi, (u32)__shfl_xor((int)hi, d, 64));
        }
        if (lane == 0) { wred[0][w] = lo; wred[1][w] = hi; }
        __syncthreads();
        lo = ~0u; hi = 0;
        for (int k = 0; k < SX_NT / 64; k++) { lo = min(lo, wred[0][k]); hi = max(hi, wred[1][k]); }
        kmin = lo;
        nk = hi - lo + 1u;                 // m >= 1: lo <= hi
        if (nk > SX_NK) {                  // workgroup-uniform: one reservation per record
#pragma unroll
            for (int k = 0; k < SX_R; k++) {
                const u32 i = tid + k * SX_NT;
                if (i < m) x.out[atomicAdd(&x.cur[b[k]], 1u)] = x.in[t0 + i];
            }
            return;
        }
    }
    for (u32 j = tid; j < nk; j += SX_NT) hcnt[j] = 0;
    __syncthreads();
    u32 r[SX_R];
#pragma unroll
    for (int k = 0; k < SX_R; k++) {
        const u32 key = PASS == 1 ? b[k] >> x.sh : b[k] - kmin;
        r[k] = b[k] != ~0u ? atomicAdd(&hcnt[key], 1u) : 0u;
    }
    __syncthreads();
    // exclusive scan of the counts (consecutive keys per thread) and one global reservation per
    // key present in the tile
    constexpr int KP = (SX_NK + SX_NT - 1) / SX_NT;
    u32 cnt[KP], tot = 0;
#pragma unroll
    for (int q = 0; q < KP; q++) {
        const u32 j = tid * KP + q;
        cnt[q] = j < nk ? hcnt[j] : 0u;
        tot += cnt[q];
    }
    u32 incl = tot;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const u32 y = (u32)__shfl_up((int)incl, d, 64);
        if (lane >= d) incl += y;
    }
    if (lane == 63) wred[0][w] = incl;
    __syncthreads();                       // also: every count read before it is overwritten
    u32 run = incl - tot;
    for (int k = 0; k < w; k++) run += wred[0][k];
#pragma unroll
    for (int q = 0; q < KP; q++) {
        const u32 j = tid * KP + q;
        if (j < nk) {
            hcnt[j] = run;
            if (cnt[q]) gb[j] = atomicAdd(&x.cur[PASS == 1 ? j * SX_CS : kmin + j], cnt[q]);
            run += cnt[q];
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SX_R; k++) {
        if (b[k] == ~0u) continue;
        const u32 key = PASS == 1 ? b[k] >> x.sh : b[k] - kmin;
        const u32 p = hcnt[key] + r[k];
        perm[p] = (uint16_t)(tid + k * SX_NT);
        pbk[p] = b[k];
    }
    __syncthreads();
    // the tile in key order, a record per lane pair (16 bytes each): the stores are whole runs,
    // each load one 32-byte record
    for (u32 h = tid; h < 2 * m; h += SX_NT) {
        const u32 p = h >> 1, half = h & 1u;
        const u32 i = perm[p], bk = pbk[p], kk = PASS == 1 ? bk >> x.sh : bk - kmin;
        const u32 d = gb[kk] + (p - hcnt[kk]);
        reinterpret_cast<uint4*>(x.out + d)[half] = reinterpret_cast<const uint4*>(x.in + t0 + i)[half];
        if (PASS == 1 && half == 0u) x.bout[d] = bk;
    }
}

// Workgroup-major histogram (large B): per bucket b, the exclusive prefix over workgroups in place
// and the bucket's total in bstart[b] (then scanned into the starts).  Threads take consecutive
// buckets, so every read and write is coalesced.  ([B][G] written by the histogram kernel was a
// column per workgroup: 32768 scattered 4-byte writes per workgroup, and as many scattered reads
// in the scatter.)
__global__ void k_ss_colscan(u32* hist, u32 B, u32 G, u32* bstart) {
    const u32 b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    u32 run = 0;
    constexpr u32 CS_U = 32;                  // loads in flight per thread (G <= ncu: a few rounds)
    for (u32 g0 = 0; g0 < G; g0 += CS_U) {
        u32 v[CS_U];
#pragma unroll
        for (u32 k = 0; k < CS_U; k++) v[k] = g0 + k < G ? hist[(u64)(g0 + k) * B + b] : 0u;
#pragma unroll
        for (u32 k = 0; k < CS_U; k++) {
            if (g0 + k < G) hist[(u64)(g0 + k) * B + b] = run;
            run += v[k];
        }
    }
    bstart[b] = run;
}

// Repeated inline keys (the record log of k_agg's pass 2 and the compacted tables may hold one
// key more than once: the global table, other map calls, pass 2's overflow) are merged while a
// bucket is written out: the first record of a run takes the run's total and the others count 0,
// which formats to no line (wcg_reduce.h: line_len).  An inline key's 16-byte prefix is the whole
// key (byte 15 is 0; a long key's is a letter byte), so dd_same never merges long keys.  Long keys
// CAN repeat: k_long_agg emits a partition's keys into the record log once per map call, and a key
// may also be counted through the long-key table (fallbacks, imports).  Those repeats share their
// 16-byte prefix, so they land in one tie group, and the tie kernels (k_tie_tiny / k_tie_sort)
// merge equal full keys - which only happens because sort_records runs the tie pass whenever
// nlong + lemit >= 2 (wcg_api.hip): a change to that gate must keep repeated long keys merged.
__device__ __forceinline__ bool dd_same(u64 ah, u64 al, u64 bh, u64 bl) {
    return ah == bh && al == bl && (al & 0xFFu) == 0;
}
// distinct keys: one atomic per workgroup
template <int NT = SB_NT>
__device__ __forceinline__ void dd_count(const SortArgs& a, u32 heads) {
    if (!a.dedupe) return;
    __shared__ u32 wh[NT / 64];
    for (int d = 32; d >= 1; d >>= 1) heads += __shfl_xor(heads, d, 64);
    if ((threadIdx.x & 63) == 0) wh[threadIdx.x >> 6] = heads;
    __syncthreads();
    if (threadIdx.x == 0) {
        u32 t = 0;
        for (int w = 0; w < NT / 64; w++) t += wh[w];
        if (t) atomicAdd((unsigned long long*)a.nkeys, (unsigned long long)t);
    }
}

// load records X[0:cm) as (hi, lo, position) into LDS, padded to P entries
__device__ __forceinline__ void sb_load(const Rec* X, u32 cm, u32 P, u64* kh, u64* kl, uint16_t* kp) {
    for (u32 j = threadIdx.x; j < P; j += SB_NT) {
        if (j < cm) { const Rec r = X[j]; kh[j] = r.hi; kl[j] = r.lo; }
        else { kh[j] = ~0ull; kl[j] = ~0ull; }
        kp[j] = (uint16_t)j;
    }
}

// Oversized bucket (more than SB_CAP2 records: rare with SS_OVS samples per bucket, or forced by
// WCG_SORT_TARGET in the tests): LDS-sorted chunks of SB_CAP, then pairwise merge passes between
// irec and irec2 (thread t writes outputs [t * L / SB_NT, (t + 1) * L / SB_NT) of each pair,
// split by merge path; A first on equal prefixes).  Equal prefixes (long keys) end up in any
// order: the tie sort orders them afterwards.
__device__ void ss_global_sort(const SortArgs& a, u64 s, u64 m, u64* kh, u64* kl, uint16_t* kp) {
    const int tid = threadIdx.x;
    Rec* X = a.irec + s;
    Rec* Y = a.irec2 + s;
    for (u64 c0 = 0; c0 < m; c0 += SB_CAP) {
        const u32 cm = (u32)(m - c0 < SB_CAP ? m - c0 : SB_CAP);
        sb_load(X + c0, cm, SB_CAP, kh, kl, kp);
        __syncthreads();
        lds_bitonic<SB_NT>(kh, kl, kp, SB_CAP);
        __syncthreads();
        for (u32 e = tid; e < cm; e += SB_NT) Y[c0 + e] = X[c0 + kp[e]];
        __syncthreads();
    }
    const Rec* src = Y;
    Rec* dst = X;
    for (u64 w = SB_CAP; w < m; w *= 2) {
        for (u64 p0 = 0; p0 < m; p0 += 2 * w) {
            const u64 la = m - p0 < w ? m - p0 : w;
            const u64 lb = m - p0 - la < w ? m - p0 - la : w;
            const u64 L = la + lb;
            const Rec* A = src + p0;
            const Rec* Bq = A + la;
            const u64 d0 = L * tid / SB_NT, d1 = L * (tid + 1) / SB_NT;
            u64 lo = d0 > lb ? d0 - lb : 0, hi = d0 < la ? d0 : la;   // #A among the first d0
            while (lo < hi) {
                const u64 mid = (lo + hi) >> 1;
                const Rec& x = Bq[d0 - 1 - mid];
                const Rec& y = A[mid];
                if (pre_lt(x.hi, x.lo, y.hi, y.lo)) hi = mid; else lo = mid + 1;
            }
            u64 ia = lo, ib = d0 - lo;
            for (u64 d = d0; d < d1; d++) {
                bool takeA;
                if (ia >= la) takeA = false;
                else if (ib >= lb) takeA = true;
                else takeA = !pre_lt(Bq[ib].hi, Bq[ib].lo, A[ia].hi, A[ia].lo);
                dst[p0 + d] = takeA ? A[ia++] : Bq[ib++];
            }
        }
        __syncthreads();
        const Rec* t = src; src = dst; dst = const_cast<Rec*>(t);
    }
    u32 heads = 0;
    for (u64 j = tid; j < m; j += SB_NT) {
        Rec r = src[j];
        if (a.dedupe) {
            if (j > 0 && dd_same(src[j - 1].hi, src[j - 1].lo, r.hi, r.lo)) r.cnt = 0;
            else {
                heads++;
                for (u64 q = j + 1; q < m && dd_same(r.hi, r.lo, src[q].hi, src[q].lo); q++) r.cnt += src[q].cnt;
            }
        }
        a.out[s + j] = r;
    }
    dd_count(a, heads);
}

// load records X[0:m) as (hi, lo, position), padded to SB_NT * E entries, sort them, leave the
// sorted entries in LDS
template <int NT, int E>
__device__ __forceinline__ void sb_sort_regs(const Rec* X, u32 m, u64* kh, u64* kl, uint16_t* kp, bool cmp) {
    u64 h[E], l[E];
    u32 q[E];
    bool maxkey = false;
#pragma unroll
    for (int e = 0; e < E; e++) {
        const u32 i = threadIdx.x * E + e;
        if (i < m) { h[e] = X[i].hi; l[e] = X[i].lo; } else { h[e] = ~0ull; l[e] = ~0ull; }
        q[e] = i;
        maxkey |= i < m && (h[e] & l[e]) == ~0ull;
    }
    if (WCG_SORT_HIONLY && cmp) {
        // the bucket's hi range: wave reductions, then one LDS word pair per wave
        u64 mn = ~0ull, mx = 0;
#pragma unroll
        for (int e = 0; e < E; e++)
            if (threadIdx.x * E + e < m) { mn = h[e] < mn ? h[e] : mn; mx = h[e] > mx ? h[e] : mx; }
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const u64 a = __shfl_xor(mn, d), b = __shfl_xor(mx, d);
            mn = a < mn ? a : mn; mx = b > mx ? b : mx;
        }
        __shared__ u64 rng[2][NT / 64];
        if ((threadIdx.x & 63) == 0) { rng[0][threadIdx.x >> 6] = mn; rng[1][threadIdx.x >> 6] = mx; }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < NT / 64; k++) {
            mn = rng[0][k] < mn ? rng[0][k] : mn; mx = rng[1][k] > mx ? rng[1][k] : mx;
        }
        const u64 range = mx - mn;
        const u32 sh = range ? (u32)__clzll((long long)range) : 64u;   // lo bits that fit
        u64 w[E];
#pragma unroll
        for (int e = 0; e < E; e++) {
            const u64 d = h[e] - mn;
            u64 k = sh == 64 ? l[e] : (sh == 0 ? d : (d << sh) | (l[e] >> (64 - sh)));
            k = k == ~0ull ? ~0ull - 1 : k;
            w[e] = threadIdx.x * E + e < m ? k : ~0ull;
        }
        if (reg_bitonic_unrolled_hi<NT, E>(w, q, X, m, kh, kl, kp)) return;
        // a long run: the (hi, lo) network below, from the records as they lie in LDS now (a
        // reload from X would be merged with the first loads, keeping them live throughout)
#pragma unroll
        for (int e = 0; e < E; e++) {
            const u32 i = threadIdx.x * E + e;
            h[e] = kh[i]; l[e] = kl[i]; q[e] = kp[i];
        }
        __syncthreads();
    }
    // The unrolled network orders (hi, lo) only, so the padding (all ones) must compare above
    // every record: a record whose prefix is all ones (no key the map produces: byte 15 is 0 or a
    // letter byte - only a crafted import or run) takes the (hi, lo, position) network.
    if (WCG_SORT_NET && (E < 8 || WCG_SORT_NET_BIG) && !__syncthreads_or(maxkey))
        reg_bitonic_unrolled<NT, E>(h, l, q, kh, kl, kp);
    else reg_bitonic<NT, E>(h, l, q, kh, kl, kp);
}

// one workgroup per bucket: bitonic sort of (hi, lo, position) in registers (LDS for the widest
// stages), then the records are permuted from the bucket's region (L2-resident) into place.
// Size classes (their register networks need different registers and LDS, and one kernel would
// give every bucket the largest one's occupancy): CLS 0 buckets of <= 4 * SB_NT records; CLS 1
// up to SB_CAP (8-entry networks) and the oversized ones (> SB_CAP2: the global path); CLS 2
// (r04) up to SB_CAP2 with 512 threads (8-entry networks: C4 at 64 GiB sorts 5e7 records in
// 32768 buckets of ~1500, ~9% of them past SB_CAP, which the global path took)
constexpr u32 SB_CAP2 = 4096;
constexpr int SB_NT2 = 512;
template <int CLS>
__global__ __launch_bounds__(CLS == 2 ? SB_NT2 : SB_NT) void k_ss_bucket(SortArgs a) {
    constexpr int NT = CLS == 2 ? SB_NT2 : SB_NT;
    constexpr u32 CAP = CLS == 2 ? SB_CAP2 : CLS == 1 ? SB_CAP : 4 * SB_NT;   // 18 KiB for CLS 0: 6
    __shared__ u64 kh[CAP], kl[CAP];               // workgroups per CU (the register limit)
    __shared__ uint16_t kp[CAP];
    const u32 b = blockIdx.x;
    const u64 s = a.bstart ? a.bstart[b] : a.hist[(u64)b * a.G];
    const u64 e = b + 1 < a.B ? (a.bstart ? a.bstart[b + 1] : a.hist[(u64)(b + 1) * a.G]) : ss_count(a);
    const u64 m = e - s;
    const u64 over = a.cls2 ? SB_CAP2 : SB_CAP;     // past this: the global path (CLS 1)
    const int cls = m <= 4 * SB_NT ? 0 : (m <= SB_CAP || m > over) ? 1 : 2;
    if (m == 0 || cls != CLS) return;
    if (CLS == 1 && m > over) { ss_global_sort(a, s, m, kh, kl, kp); return; }
    const Rec* X = a.irec + s;
    static_assert(SB_CAP == 8 * SB_NT && SB_CAP2 == 8 * SB_NT2, "k_ss_bucket's register networks cover the caps");
    if (CLS == 2) sb_sort_regs<NT, 8>(X, (u32)m, kh, kl, kp, WCG_SORT_HIONLY_BIG);
    else if (CLS == 1) sb_sort_regs<NT, 8>(X, (u32)m, kh, kl, kp, WCG_SORT_HIONLY_BIG);
    else if (m <= SB_NT) sb_sort_regs<NT, 1>(X, (u32)m, kh, kl, kp, true);
    else if (m <= 2 * SB_NT) sb_sort_regs<NT, 2>(X, (u32)m, kh, kl, kp, true);
    else sb_sort_regs<NT, 4>(X, (u32)m, kh, kl, kp, true);
    u32 heads = 0;
    for (u32 j = threadIdx.x; j < m; j += NT) {
        Rec r = X[kp[j]];
        if (a.dedupe) {                               // sorted keys in LDS; counts from X (rare)
            if (j > 0 && dd_same(kh[j - 1], kl[j - 1], kh[j], kl[j])) r.cnt = 0;
            else {
                heads++;
                for (u32 q = j + 1; q < m && dd_same(kh[j], kl[j], kh[q], kl[q]); q++) r.cnt += X[kp[q]].cnt;
            }
        }
        // r04: tie-group starts with both neighbours in this bucket (the first and last records:
        // k_tie_edge); equal prefixes are both long keys or both inline (byte 15: a letter byte
        // or 0), so the neighbours' prefixes in LDS decide
        if (a.groups && j > 0 && j + 1 < m && (r.ref & LONG_FLAG) && kh[j + 1] == kh[j] && kl[j + 1] == kl[j] &&
            !(kh[j - 1] == kh[j] && kl[j - 1] == kl[j]))
            a.groups[atomicAdd((unsigned long long*)a.ngroups, 1ull)] = s + j;
        a.out[s + j] = r;
    }
    dd_count<NT>(a, heads);
}

// group start test at sorted position i (k_tie_mark's predicate)
__device__ __forceinline__ bool tie_start(const Rec* r, u64 n, u64 i);
// r04: the tie-group starts k_ss_bucket leaves out: every bucket's first and last records, and
// all records of buckets past SB_CAP2 (sorted by the global path).  One thread per bucket; an
// oversized bucket is scanned by the whole workgroup afterwards.
constexpr int TE_NT = 256;
__global__ __launch_bounds__(TE_NT) void k_tie_edge(SortArgs a) {
    __shared__ u32 big[TE_NT];
    __shared__ u32 nbig;
    if (threadIdx.x == 0) nbig = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0 && a.tie_zero) *a.tie_zero = 0;   // (a memset: 2 dispatches)
    __syncthreads();
    const u64 n = ss_count(a);
    const u64 over = a.cls2 ? SB_CAP2 : SB_CAP;
    const u32 b = blockIdx.x * TE_NT + threadIdx.x;
    if (b < a.B) {
        const u64 s = a.bstart ? a.bstart[b] : a.hist[(u64)b * a.G];
        const u64 e = b + 1 < a.B ? (a.bstart ? a.bstart[b + 1] : a.hist[(u64)(b + 1) * a.G]) : n;
        if (e > s) {
            if (e - s > over) big[atomicAdd(&nbig, 1u)] = b;
            else {
                if (tie_start(a.out, n, s)) a.groups[atomicAdd((unsigned long long*)a.ngroups, 1ull)] = s;
                if (e - s > 1 && tie_start(a.out, n, e - 1))
                    a.groups[atomicAdd((unsigned long long*)a.ngroups, 1ull)] = e - 1;
            }
        }
    }
    __syncthreads();
    for (u32 k = 0; k < nbig; k++) {
        const u32 bb = big[k];
        const u64 s = a.bstart ? a.bstart[bb] : a.hist[(u64)bb * a.G];
        const u64 e = bb + 1 < a.B ? (a.bstart ? a.bstart[bb + 1] : a.hist[(u64)(bb + 1) * a.G]) : n;
        for (u64 i = s + threadIdx.x; i < e; i += TE_NT)
            if (tie_start(a.out, n, i)) a.groups[atomicAdd((unsigned long long*)a.ngroups, 1ull)] = i;
    }
}

// ---------------------------------------------------------------- tie groups
__device__ __forceinline__ u64 ik_hi(uint4 k) { return (u64)k.w << 32 | k.z; }
__device__ __forceinline__ u64 ik_lo(uint4 k) { return (u64)k.y << 32 | k.x; }

// A record's key bytes: inline keys are their prefix; a long key (ref & LONG_FLAG) lives at
// base + (ref & LONG_OFF_MASK), (ref >> 40) & LONG_LEN_MAX bytes - base is the long-key arena
// (zero-padded 16-byte cells) or, for merged runs, the formatted text (any alignment).
__device__ __forceinline__ bool rec_long(const Rec& r) { return (r.ref & LONG_FLAG) != 0; }
__device__ __forceinline__ u64 key_bytes_len(const Rec& r) { return (r.ref >> 40) & LONG_LEN_MAX; }

// big-endian 8 bytes of key x from byte k on (zeros past its end)
__device__ __forceinline__ u64 key_word_be(const uint8_t* base, const Rec& r, u64 k) {
    const u64 len = key_bytes_len(r);
    const uint8_t* p = base + (r.ref & LONG_OFF_MASK);
    u64 v = 0;
    for (int q = 0; q < 8; q++) v = (v << 8) | (k + q < len ? p[k + q] : 0u);
    return v;
}

// full bytewise order of two long keys with equal first 32 bytes (the slow path of the tie sort)
// (r04: 16 bytes at a time when both keys sit in 16-byte aligned, zero-padded arena cells - a
// repeated long key compares equal to its end, byte loads one dependent HBM read each)
__device__ int key_cmp_from(const uint8_t* base, const Rec& x, const Rec& y, u64 from) {
    const u64 lx = key_bytes_len(x), ly = key_bytes_len(y);
    const uint8_t* px = base + (x.ref & LONG_OFF_MASK);
    const uint8_t* py = base + (y.ref & LONG_OFF_MASK);
    const u64 m = lx < ly ? lx : ly;
    u64 i = from;
    if ((((uintptr_t)px | (uintptr_t)py | from) & 15) == 0) {
        for (; i + 16 <= m; i += 16) {
            const uint4 a = *reinterpret_cast<const uint4*>(px + i), b = *reinterpret_cast<const uint4*>(py + i);
            const u64 a0 = bswap64((u64)a.y << 32 | a.x), b0 = bswap64((u64)b.y << 32 | b.x);
            if (a0 != b0) return a0 < b0 ? -1 : 1;
            const u64 a1 = bswap64((u64)a.w << 32 | a.z), b1 = bswap64((u64)b.w << 32 | b.z);
            if (a1 != b1) return a1 < b1 ? -1 : 1;
        }
    }
    for (; i < m; i++)
        if (px[i] != py[i]) return px[i] < py[i] ? -1 : 1;
    return lx < ly ? -1 : (lx > ly ? 1 : 0);
}

__device__ __forceinline__ bool same_prefix(const Rec& x, const Rec& y) { return x.hi == y.hi && x.lo == y.lo; }

// group starts: long keys whose successor shares their 16-byte prefix and whose predecessor
// does not
__device__ __forceinline__ bool tie_start(const Rec* r, u64 n, u64 i) {
    if (i + 1 >= n) return false;
    const Rec x = r[i], y = r[i + 1];
    if (!rec_long(x) || !rec_long(y) || !same_prefix(x, y)) return false;
    if (i > 0) {
        const Rec w = r[i - 1];
        if (rec_long(w) && same_prefix(w, x)) return false;
    }
    return true;
}
__global__ void k_tie_mark(const Rec* r, u64 n, const u64* nd, u64* groups, u64* ngroups) {
    if (nd && *nd < n) n = *nd;                  // device-sized: the sorted records only
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i + 1 < n; i += (u64)gridDim.x * blockDim.x)
        if (tie_start(r, n, i)) groups[atomicAdd(ngroups, 1ull)] = i;
}

// One workgroup per group (grid-stride over the group list): the group's extent, then a
// bitonic sort by (bytes 16-31, then the full key from byte 32, slow path), in LDS up to
// TG_CAP records, through scratch (2 * start, padded to a power of two) beyond that; the
// records are permuted through `tmp` (the compacted array, free by then).
constexpr int TG_NT = 1024;
constexpr u32 TG_CAP = 2048;

struct TieArgs {
    Rec* r;                // sorted records
    u64 n;                 // records, or (nd set) the capacity
    const u64* nd;         // device-sized: the record count in device memory
    const uint8_t* base;   // key bytes of long records
    const u64* groups;
    const u64* ngroups;
    Rec* tmp;              // >= n records
    uint4* sc_key;         // >= 2n scratch items (bytes 16-31 big-endian) ...
    u32* sc_pos;           // ... and the record position
    u64* nkeys;            // record-log jobs (the sort's distinct-key count): a long key may appear
                           // more than once (other map calls, the table as well as the log); the
                           // copies are merged into the first and the count lowered
};
__device__ __forceinline__ bool long_same(const uint8_t* base, const Rec& x, const Rec& y) {
    return ((x.ref >> 40) & LONG_LEN_MAX) == ((y.ref >> 40) & LONG_LEN_MAX) && key_cmp_from(base, x, y, 16) == 0;
}

__device__ __forceinline__ bool tie_lt(const TieArgs& a, u64 xh, u64 xl, u32 xp, u64 yh, u64 yl, u32 yp) {
    if (xh != yh) return xh < yh;
    if (xl != yl) return xl < yl;
    if (xp == yp) return false;
    if (xp == ~0u || yp == ~0u) return yp == ~0u;     // padding sorts last
    return key_cmp_from(a.base, a.r[xp], a.r[yp], 32) < 0;
}

// r04: small tie groups without workgroup barriers.  A multi-call job holds long keys that
// several map calls emitted (the record log, then the table once the log is full): every
// repeated key is a tie group of 2-8 copies, and a 1024-thread workgroup per group (k_tie_sort:
// extent, network and merge separated by barriers and dependent global reads) took 120 ms on C4
// at 64 GiB.  Groups of <= TT_MAX records take one thread each, <= 64 one wave each
// (tie_wave_group, in the same kernel); larger ones are listed for k_tie_sort (big / nbig).
__device__ __forceinline__ u64 wave_shfl_up_u64(u64 v, int d) {
    const u32 lo = (u32)__shfl_up((int)(u32)v, d, 64), hi = (u32)__shfl_up((int)(u32)(v >> 32), d, 64);
    return (u64)hi << 32 | lo;
}
// tie_lt on plain values (the argument block by reference puts it in scratch)
__device__ __forceinline__ bool tie_lt_v(const uint8_t* base, const Rec* r, u64 xh, u64 xl, u32 xp, u64 yh, u64 yl,
                                         u32 yp) {
    if (xh != yh) return xh < yh;
    if (xl != yl) return xl < yl;
    if (xp == yp) return false;
    if (xp == ~0u || yp == ~0u) return yp == ~0u;     // padding sorts last
    return key_cmp_from(base, r[xp], r[yp], 32) < 0;
}
// bytes 16-31 of a long key, big-endian (zeros past its end): one 16-byte load from an aligned,
// zero-padded arena cell, else byte by byte (merged runs: keys inside the formatted text)
__device__ __forceinline__ void key_words_16(const uint8_t* base, const Rec& r, u64& h, u64& l) {
    const uint8_t* p = base + (r.ref & LONG_OFF_MASK);
    if (((uintptr_t)p & 15) == 0) {
        const uint4 v = *reinterpret_cast<const uint4*>(p + 16);
        h = bswap64((u64)v.y << 32 | v.x);
        l = bswap64((u64)v.w << 32 | v.z);
        return;
    }
    h = key_word_be(base, r, 16);
    l = key_word_be(base, r, 24);
}
// r04: tie groups of <= TT_MAX records, one thread each (a repeated long key of a multi-call job
// is a group of 2-3, one per repeated key - each a chain of dependent reads, so many must be in
// flight at once).  A 4-entry sorting network on (bytes 16-31, position); padding sorts last.
constexpr u32 TT_MAX = 4;
__device__ __forceinline__ void tt_cx(const uint8_t* base, const Rec* R, u64& ah, u64& al, u32& ap, u64& bh, u64& bl,
                                      u32& bp) {
    if (tie_lt_v(base, R, bh, bl, bp, ah, al, ap)) {
        u64 t = ah; ah = bh; bh = t;
        t = al; al = bl; bl = t;
        const u32 q = ap; ap = bp; bp = q;
    }
}
__device__ __forceinline__ void tie_wave_group(const uint8_t* base, Rec* R, u64 n, u64* nkeys, u64 s, u64* big,
                                               u64* nbig, u32 lane);
// One lane per group; groups of TT_MAX+1..64 records are then taken by the whole wave at once
// (tie_wave_group: one kernel instead of two), larger ones listed for k_tie_sort (big / nbig).
// The loop is wave-uniform so that every lane joins the wave's group sorts.
__global__ __launch_bounds__(256) void k_tie_tiny(TieArgs a, u64* big, u64* nbig) {
    const uint8_t* const base = a.base;
    Rec* const R = a.r;
    const u32 lane = threadIdx.x & 63;
    u64 n = a.n;
    if (a.nd && *a.nd < n) n = *a.nd;
    const u64 ng = *a.ngroups;
    u64 merged = 0;
    const u64 wstride = (u64)gridDim.x * (256 / 64) * 64;
    for (u64 g0 = ((u64)blockIdx.x * (256 / 64) + (threadIdx.x >> 6)) * 64; g0 < ng; g0 += wstride) {
        const u64 g = g0 + lane;
        const bool live = g < ng;
        const u64 s = live ? a.groups[g] : 0;
        bool is_mid = false;
        if (live) {
            const Rec x0 = R[s];
            // extent, up to TT_MAX + 1 records (the reads issue together)
            bool in[TT_MAX];
#pragma unroll
            for (u32 k = 1; k <= TT_MAX; k++) {
                bool v = s + k < n;
                if (v) { const Rec y = R[s + k]; v = rec_long(y) && same_prefix(x0, y); }
                in[k - 1] = v;
            }
            u32 m = 1;
#pragma unroll
            for (u32 k = 0; k < TT_MAX; k++) m += (in[k] && m == k + 1) ? 1u : 0u;
            is_mid = m > TT_MAX;
            if (!is_mid) {
                u64 h0, l0, h1 = ~0ull, l1 = ~0ull, h2 = ~0ull, l2 = ~0ull, h3 = ~0ull, l3 = ~0ull;
                u32 p0 = (u32)s, p1 = ~0u, p2 = ~0u, p3 = ~0u;
                key_words_16(base, x0, h0, l0);
                if (m > 1) { p1 = (u32)(s + 1); key_words_16(base, R[s + 1], h1, l1); }
                if (m > 2) { p2 = (u32)(s + 2); key_words_16(base, R[s + 2], h2, l2); }
                if (m > 3) { p3 = (u32)(s + 3); key_words_16(base, R[s + 3], h3, l3); }
                tt_cx(base, R, h0, l0, p0, h1, l1, p1);
                tt_cx(base, R, h2, l2, p2, h3, l3, p3);
                tt_cx(base, R, h0, l0, p0, h2, l2, p2);
                tt_cx(base, R, h1, l1, p1, h3, l3, p3);
                tt_cx(base, R, h1, l1, p1, h2, l2, p2);
                // the sorted records (read before any write), repeated keys merged into the first
                Rec y0 = R[p0], y1 = m > 1 ? R[p1] : x0, y2 = m > 2 ? R[p2] : x0, y3 = m > 3 ? R[p3] : x0;
                if (a.nkeys) {
                    if (m > 3 && long_same(base, y2, y3)) { y2.cnt += y3.cnt; y3.cnt = 0; merged++; }
                    if (m > 2 && long_same(base, y1, y2)) { y1.cnt += y2.cnt; y2.cnt = 0; merged++; }
                    if (m > 1 && long_same(base, y0, y1)) { y0.cnt += y1.cnt; y1.cnt = 0; merged++; }
                }
                R[s] = y0;
                if (m > 1) R[s + 1] = y1;
                if (m > 2) R[s + 2] = y2;
                if (m > 3) R[s + 3] = y3;
            }
        }
        for (u64 mm = __ballot(is_mid); mm; mm &= mm - 1) {   // the larger groups, the whole wave each
            const int src = (int)__builtin_ctzll(mm);
            const u64 sm = (u64)(u32)__shfl((int)(u32)s, src, 64) | (u64)(u32)__shfl((int)(u32)(s >> 32), src, 64) << 32;
            tie_wave_group(base, R, n, a.nkeys, sm, big, nbig, lane);
        }
    }
    for (int d = 32; d >= 1; d >>= 1) merged += __shfl_xor(merged, d, 64);
    if ((threadIdx.x & 63) == 0 && merged) atomicAdd((unsigned long long*)a.nkeys, (unsigned long long)(0ull - merged));
}

// one tie group of <= 64 records starting at s, by the whole wave (all 64 lanes active); a larger
// group is listed for k_tie_sort
__device__ __forceinline__ void tie_wave_group(const uint8_t* base, Rec* R, u64 n, u64* nkeys, u64 s, u64* big,
                                               u64* nbig, u32 lane) {
    const Rec x0 = R[s];
    // extent: the first of the next 64 records that is short or has another prefix
    const u64 i = s + 1 + lane;
    bool stop = i >= n;
    if (!stop) { const Rec y = R[i]; stop = !rec_long(y) || !same_prefix(x0, y); }
    const u64 bal = __ballot(stop);
    if (bal == 0) {                              // > 64 records: the workgroup path
        if (lane == 0) big[atomicAdd((unsigned long long*)nbig, 1ull)] = s;
        return;
    }
    const u32 m = 1 + (u32)__builtin_ctzll(bal);
    const bool v = lane < m;
    u64 th = ~0ull, tl = ~0ull;
    u32 tp = ~0u;
    if (v) {
        const Rec y = R[s + lane];
        th = key_word_be(base, y, 16); tl = key_word_be(base, y, 24); tp = (u32)(s + lane);
    }
    // bitonic over the first P >= m lanes (padding ~0 sorts last; lanes past P hold padding)
    u32 P = 2;
    while (P < m) P <<= 1;
    for (u32 k = 2; k <= P; k <<= 1)
        for (u32 j = k >> 1; j > 0; j >>= 1) {
            const u64 oh = shfl_xor64(th, (int)j), ol = shfl_xor64(tl, (int)j);
            const u32 op = (u32)__shfl_xor((int)tp, (int)j, 64);
            const bool keep_min = ((lane & j) == 0) == ((lane & k) == 0);
            const bool take = keep_min ? tie_lt_v(base, R, oh, ol, op, th, tl, tp) : tie_lt_v(base, R, th, tl, tp, oh, ol, op);
            if (take) { th = oh; tl = ol; tp = op; }
        }
    Rec x = v ? R[tp] : x0;
    if (nkeys) {                               // equal keys are adjacent: the first takes the sum
        const u32 pp = (u32)__shfl_up((int)tp, 1, 64);
        bool head = lane == 0 || !v;
        if (v && lane > 0) head = !long_same(base, R[pp], x);
        const u64 H = __ballot(head) | (~0ull << m);   // run heads (lanes past m close runs)
        u64 c = v ? x.cnt : 0;                         // inclusive prefix sum of the counts
        for (int d = 1; d < 64; d <<= 1) { const u64 y = wave_shfl_up_u64(c, d); if ((int)lane >= d) c += y; }
        const u64 hi_mask = lane == 63 ? 0ull : (H >> (lane + 1));
        const u32 end = hi_mask ? lane + 1 + (u32)__builtin_ctzll(hi_mask) : 64u;   // next head
        const u64 last = __shfl(c, (int)(end - 1), 64);
        const u64 before = wave_shfl_up_u64(c, 1);
        const u64 run = last - (lane > 0 ? before : 0ull);
        if (v) x.cnt = head ? run : 0;
        const u32 merged = (u32)__popcll(__ballot(v && !head));
        if (lane == 0 && merged) atomicAdd((unsigned long long*)nkeys, (unsigned long long)(0ull - merged));
    }
    if (v) R[s + lane] = x;
}
__global__ __launch_bounds__(TG_NT) void k_tie_sort(TieArgs a) {
    __shared__ u64 th[TG_CAP], tl[TG_CAP];
    __shared__ u32 tp[TG_CAP];
    __shared__ u64 end_s;
    const int tid = threadIdx.x;
    const u64 ng = *a.ngroups;
    if (a.nd && *a.nd < a.n) a.n = *a.nd;
    for (u64 g = blockIdx.x; g < ng; g += gridDim.x) {
        const u64 s = a.groups[g];
        const Rec x0 = a.r[s];
        // extent: the first record past s that is short or has another prefix, 1024 at a time
        if (tid == 0) end_s = a.n;
        __syncthreads();
        for (u64 base = s + 1; base < a.n; base += TG_NT) {
            const u64 i = base + tid;
            bool stop = false;
            if (i < a.n) { const Rec y = a.r[i]; stop = !rec_long(y) || !same_prefix(x0, y); }
            if (stop) atomicMin((unsigned long long*)&end_s, (unsigned long long)i);
            __syncthreads();
            const u64 e = end_s;
            __syncthreads();
            if (e < a.n) break;
        }
        const u64 m = end_s - s;
        if (m <= TG_CAP) {
            u32 P = 2;
            while (P < m) P <<= 1;
            for (u32 j = tid; j < P; j += TG_NT) {
                if (j < m) {
                    const Rec y = a.r[s + j];
                    th[j] = key_word_be(a.base, y, 16); tl[j] = key_word_be(a.base, y, 24); tp[j] = (u32)(s + j);
                } else { th[j] = ~0ull; tl[j] = ~0ull; tp[j] = ~0u; }
            }
            __syncthreads();
            for (u32 k = 2; k <= P; k <<= 1)
                for (u32 j = k >> 1; j > 0; j >>= 1) {
                    for (u32 t = tid; t < P / 2; t += TG_NT) {
                        const u32 i = 2 * t - (t & (j - 1)), p = i + j;
                        if (tie_lt(a, th[p], tl[p], tp[p], th[i], tl[i], tp[i]) == ((i & k) == 0)) {
                            u64 v = th[i]; th[i] = th[p]; th[p] = v;
                            v = tl[i]; tl[i] = tl[p]; tl[p] = v;
                            const u32 q = tp[i]; tp[i] = tp[p]; tp[p] = q;
                        }
                    }
                    __syncthreads();
                }
            for (u32 j = tid; j < m; j += TG_NT) a.tmp[s + j] = a.r[tp[j]];
        } else {
            u64 P = 2;
            while (P < m) P <<= 1;
            uint4* K = a.sc_key + 2 * s;
            u32* Q = a.sc_pos + 2 * s;
            for (u64 j = tid; j < P; j += TG_NT) {
                if (j < m) {
                    const Rec y = a.r[s + j];
                    const u64 h = key_word_be(a.base, y, 16), l = key_word_be(a.base, y, 24);
                    K[j] = make_uint4((u32)l, (u32)(l >> 32), (u32)h, (u32)(h >> 32));
                    Q[j] = (u32)(s + j);
                } else { K[j] = make_uint4(~0u, ~0u, ~0u, ~0u); Q[j] = ~0u; }
            }
            __syncthreads();
            for (u64 k = 2; k <= P; k <<= 1)
                for (u64 j = k >> 1; j > 0; j >>= 1) {
                    for (u64 t = tid; t < P / 2; t += TG_NT) {
                        const u64 i = 2 * t - (t & (j - 1)), p = i + j;
                        const uint4 ki = K[i], kp = K[p];
                        const u32 qi = Q[i], qp = Q[p];
                        if (tie_lt(a, ik_hi(kp), ik_lo(kp), qp, ik_hi(ki), ik_lo(ki), qi) == ((i & k) == 0)) {
                            K[i] = kp; K[p] = ki; Q[i] = qp; Q[p] = qi;
                        }
                    }
                    __syncthreads();
                }
            for (u64 j = tid; j < m; j += TG_NT) a.tmp[s + j] = a.r[Q[j]];
        }
        __syncthreads();
        u32 merged = 0;
        for (u64 j = tid; j < m; j += TG_NT) {
            Rec x = a.tmp[s + j];
            if (a.nkeys) {                    // equal keys are adjacent now: the first takes the sum
                if (j > 0 && long_same(a.base, a.tmp[s + j - 1], x)) { x.cnt = 0; merged++; }
                else for (u64 q = j + 1; q < m && long_same(a.base, x, a.tmp[s + q]); q++) x.cnt += a.tmp[s + q].cnt;
            }
            a.r[s + j] = x;
        }
        if (merged) atomicAdd((unsigned long long*)a.nkeys, (unsigned long long)(0ull - merged));
        __syncthreads();
    }
}

}  // namespace wcg
