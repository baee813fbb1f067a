// wcg_fused.h - DoReduce + Merge of a small job in ONE launch (r05): compaction, sample sort,
// tie order and "key: count\n" formatting (mapreduce.go:239-321: DoReduce's sort.Strings and
// Reduce, Merge's sort.Strings and Fprintf) for one-pass jobs of up to FR_NMAX keys.
//
// The general reduce (wcg_reduce.h + wcg_sort.h) is ~20 launches: on the metric's config (C2:
// 1e5 keys) they were 4-18 us each, ~175 us of a 1.3 ms step for a few MB of records
// (profiles/r04_kernel_summary_c2_final.txt).  Here the same work is four phases of one
// persistent launch:
//   P0 compaction    the tables' slots in blocks of 2048 (compact_block) -> records
//   P1 sample runs   S = 4 samples per bucket, sorted in runs of 512 (one register network each)
//   P2 scatter       every item ranks the runs' samples against each other (merge ranks: the
//                    splitters are the samples of rank (k + 1) S / B), finds each record's bucket by
//                    binary search over the splitters in LDS and appends it to its bucket's region
//                    (one global atomic per item and bucket); a full region spills to a list
//   P3 buckets       one item per bucket, in bucket order: register network on (hi, lo) (the
//                    unrolled networks of wcg_sort.h), long keys sharing a 16-byte prefix ordered
//                    by their full bytes, lines sized and scanned, the bucket's byte offset from
//                    the byte counts every earlier bucket publishes (look-back), the lines staged
//                    in LDS and written with 16-byte stores
// Work is handed out by per-phase ticket counters, and a workgroup waits for a phase only once
// every item of the phase before it has been taken (by running workgroups), so the launch cannot
// deadlock whatever the residency: a workgroup that starts late finds no tickets and leaves.  The
// workgroup that completes a phase's last item publishes the next phase's parameters (release
// fence, then the phase's ready word = the launch's epoch); the others poll that word and acquire
// (MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup visibility": producer waves drain
// their stores, a barrier, one lane's agent release; consumer: one poll, one agent acquire, a
// barrier, plain loads).  The last workgroup to leave zeroes the counters for the next launch.
//
// Rare cases stay exact, only slower: a bucket past its region (FR_RCAP records: the sample put
// too few splitters there, p ~ 1e-6 per bucket) is gathered from the spill list and merge-sorted
// by the workgroup in global memory with the full-key order; a long-key tie run of any length is
// ordered by counting ranks under the full-key order.
#pragma once
#include "wcg_common.h"
#include "wcg_sort.h"
#include "wcg_reduce.h"

namespace wcg {

constexpr int FR_NT = 256;
constexpr u32 FR_CAP = 2048;            // bucket records sorted in LDS (8 per thread)
constexpr u32 FR_RCAP = FR_CAP;         // records per bucket region
constexpr u32 FR_BMAX = 512;            // buckets
constexpr u32 FR_OVS = 4;               // samples per bucket
constexpr u32 FR_RUN = 512;             // sample run: one 2-entry register network
constexpr u32 FR_SMAX = FR_BMAX * FR_OVS;
constexpr u32 FR_CHUNK = 4 * FR_NT;     // records per scatter item
constexpr u32 FR_TARGET = 384;          // mean records per bucket (the region holds 5.3x that)
constexpr u32 FR_STAGE = 16384;         // a bucket's lines staged in LDS (more: written directly)
constexpr u64 FR_NMAX = 1ull << 17;     // the host takes this path for jobs up to this many keys
constexpr int FR_NPH = 4;
constexpr u32 FR_SPIN_LIMIT = 1u << 24;  // polls (s_sleep 2 each, ~1 s): then spin_fail
static_assert(FR_SMAX <= FR_CAP, "the sample runs are staged in the bucket sort's LDS arrays");
static_assert(FR_RUN == 2 * FR_NT, "a sample run is one 2-entry register network");

// counters and parameters, one 128-byte line each (the counters take every workgroup's atomics)
struct FrCtl {
    u32 ticket[FR_NPH][32];
    u32 done[FR_NPH][32];
    u32 ready[FR_NPH][32];               // = the launch's epoch once the phase's parameters are out
    u32 exits[32];
    u32 nspill[32];
    u64 n, B, S, nrun, nchunk, pad[3];  // parameters (plain stores before a ready word)
};

struct FrArgs {
    const GEntry* gtab; u64 gslots;
    const GEntry* ltab; u64 lslots;
    const uint8_t* arena;
    DevState* st;
    u64* total_out;          // formatted bytes (the scalar the host reads back)
    Rec* rec; u64 rec_cap;   // compaction output; scratch of the oversized-bucket path after P2
    Rec* out_rec;            // sorted records (wcg_partition_all and the exports read them)
    uint8_t* out;            // formatted text
    Rec* reg;                // FR_BMAX x FR_RCAP bucket regions
    Rec* spill; u32* spill_bid; u64 spill_cap;
    u64* smp;                // sample runs: hi words [FR_SMAX], then lo words [FR_SMAX]
    u32* bcnt;               // [FR_BMAX] records per bucket
    u64* bstart;             // [FR_BMAX + 1] bucket starts in the sorted order
    u64* bflag;              // [FR_BMAX] epoch << 40 | the bucket's formatted bytes
    FrCtl* ctl;
    u32 epoch;               // 1 .. 2^24 - 1, a new one per launch
    u32 target;              // mean records per bucket
    u32 nitems0;             // compaction blocks
};

__device__ __forceinline__ u32 fr_poll(const u32* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ u64 fr_poll64(const u64* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// producer side of a hand-off, by the whole workgroup: every wave's stores drained, a barrier,
// one lane's agent-scope release (the L2 write-back), drained again before any signal
__device__ __forceinline__ void fr_release_wg() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}
// consumer side, after thread 0's poll matched: one agent acquire (this CU's L1), then a barrier
__device__ __forceinline__ void fr_acquire_wg() {
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
}

// Go's bytewise order of two records of distinct keys: the 16-byte prefix, then (long keys
// sharing it) the bytes from 16 on in the arena
__device__ __forceinline__ bool fr_less(const Rec& x, const Rec& y, const uint8_t* arena) {
    if (x.hi != y.hi) return x.hi < y.hi;
    if (x.lo != y.lo) return x.lo < y.lo;
    const bool lx = (x.ref & LONG_FLAG) != 0, ly = (y.ref & LONG_FLAG) != 0;
    if (!lx || !ly) return !lx && ly;           // (equal prefixes are both long in one-pass jobs)
    return key_cmp_from(arena, x, y, 16) < 0;
}

// workgroup exclusive scan of one u64 per thread (FR_NT threads); *all = the sum
__device__ __forceinline__ u64 fr_scan(u64 s, u64* ws, u64* all) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    u64 incl = s;
    for (int d = 1; d < 64; d <<= 1) { const u64 y = __shfl_up(incl, d, 64); if (lane >= d) incl += y; }
    __syncthreads();                              // ws of an earlier scan has been read
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    u64 pre = 0, t = 0;
    for (int k = 0; k < FR_NT / 64; k++) { if (k < w) pre += ws[k]; t += ws[k]; }
    *all = t;
    return pre + incl - s;
}

// Long keys sharing their 16-byte prefix sit next to each other after the (hi, lo) network, in any
// order: each such run of kp[0, m) is reordered by counting, for each member, the members below
// it in the full-key order (keys are distinct, so the counts are a permutation).  X[kp[j]] is the
// record at sorted position j.
__device__ __attribute__((noinline)) void fr_fix_runs(const Rec* X, u32 m, const u64* kh, const u64* kl, uint16_t* kp, uint16_t* kq,
                            const uint8_t* arena, uint16_t* runs, u32* nruns, u32* rend) {
    const u32 tid = threadIdx.x;
    if (tid == 0) *nruns = 0;
    __syncthreads();
    for (u32 j = tid; j + 1 < m; j += FR_NT)
        if (kh[j + 1] == kh[j] && kl[j + 1] == kl[j] && (j == 0 || kh[j - 1] != kh[j] || kl[j - 1] != kl[j]))
            runs[atomicAdd(nruns, 1u)] = (uint16_t)j;
    __syncthreads();
    const u32 nr = *nruns;
    for (u32 r = 0; r < nr; r++) {
        const u32 s = runs[r];
        if (tid == 0) {
            u32 e = s + 1;
            while (e < m && kh[e] == kh[s] && kl[e] == kl[s]) e++;
            *rend = e;
        }
        __syncthreads();
        const u32 k = *rend - s;
        for (u32 u = tid; u < k; u += FR_NT) {
            const uint16_t me = kp[s + u];
            const Rec x = X[me];
            u32 rank = 0;
            for (u32 v = 0; v < k; v++)
                if (v != u && fr_less(X[kp[s + v]], x, arena)) rank++;
            kq[s + rank] = me;
        }
        __syncthreads();
        for (u32 u = tid; u < k; u += FR_NT) kp[s + u] = kq[s + u];
        __syncthreads();
    }
}

// a bucket past its region: its records (the region, then its entries of the spill list) are
// gathered into A = rec + start, sorted in LDS chunks of FR_CAP, merged in passes between A and
// D = out_rec + start by merge path under the full-key order; the result ends in D
__device__ __attribute__((noinline)) void fr_sort_global(const FrArgs& a, u32 b, u64 s0, u64 m, u64* kh, u64* kl, uint16_t* kp, uint16_t* kq,
                               uint16_t* runs, u32* nruns, u32* rend, u32* cnt) {
    const u32 tid = threadIdx.x;
    Rec* const A = a.rec + s0;
    Rec* const D = a.out_rec + s0;
    for (u32 i = tid; i < FR_RCAP; i += FR_NT) A[i] = a.reg[(u64)b * FR_RCAP + i];
    if (tid == 0) *cnt = 0;
    __syncthreads();
    const u64 ns = (u64)atomicAdd(&a.ctl->nspill[0], 0u);
    const u64 nsl = ns < a.spill_cap ? ns : a.spill_cap;
    for (u64 o = tid; o < nsl; o += FR_NT)
        if (a.spill_bid[o] == b) A[FR_RCAP + atomicAdd(cnt, 1u)] = a.spill[o];
    fr_release_wg();                              // (the same workgroup reads A below)
    fr_acquire_wg();
    if (FR_RCAP + *cnt != m && tid == 0) atomicAdd(&a.st->spin_fail, 1u);   // never expected
    for (u64 c0 = 0; c0 < m; c0 += FR_CAP) {
        const u32 cm = (u32)(m - c0 < FR_CAP ? m - c0 : FR_CAP);
        for (u32 j = tid; j < FR_CAP; j += FR_NT) {
            if (j < cm) { const Rec r = A[c0 + j]; kh[j] = r.hi; kl[j] = r.lo; }
            else { kh[j] = ~0ull; kl[j] = ~0ull; }
            kp[j] = (uint16_t)j;
        }
        __syncthreads();
        lds_bitonic<FR_NT>(kh, kl, kp, FR_CAP);
        __syncthreads();
        fr_fix_runs(A + c0, cm, kh, kl, kp, kq, a.arena, runs, nruns, rend);
        for (u32 j = tid; j < cm; j += FR_NT) D[c0 + j] = A[c0 + kp[j]];
        __syncthreads();
    }
    const Rec* src = D;
    Rec* dst = A;
    for (u64 w = FR_CAP; w < m; w *= 2) {
        for (u64 p0 = 0; p0 < m; p0 += 2 * w) {
            const u64 la = m - p0 < w ? m - p0 : w;
            const u64 lb = m - p0 - la < w ? m - p0 - la : w;
            const u64 L = la + lb;
            const Rec* X = src + p0;
            const Rec* Y = X + la;
            const u64 d0 = L * tid / FR_NT, d1 = L * (tid + 1) / FR_NT;
            u64 lo = d0 > lb ? d0 - lb : 0, hi = d0 < la ? d0 : la;      // records of X among the first d0
            while (lo < hi) {
                const u64 mid = (lo + hi) >> 1;
                if (fr_less(Y[d0 - 1 - mid], X[mid], a.arena)) hi = mid; else lo = mid + 1;
            }
            u64 ia = lo, ib = d0 - lo;
            for (u64 d = d0; d < d1; d++) {
                const bool takeX = ia < la && (ib >= lb || !fr_less(Y[ib], X[ia], a.arena));
                dst[p0 + d] = takeX ? X[ia++] : Y[ib++];
            }
        }
        __syncthreads();
        const Rec* t = src; src = dst; dst = const_cast<Rec*>(t);
    }
    if (src != D) {
        for (u64 j = tid; j < m; j += FR_NT) D[j] = src[j];
        __syncthreads();
    }
}

// one "key: count\n" line of record x at o (Merge's format, mapreduce.go:316-318; the record is
// passed whole: fmt_lines indexes its record array with a loop variable, which put it in scratch)
template <typename P>
__device__ __forceinline__ void fr_line(const Rec& x, const uint8_t* arena, P o) {
    const u64 len = rec_len(x);
    if (x.ref & LONG_FLAG) {
        const uint8_t* src = arena + (x.ref & LONG_OFF_MASK);
        for (u64 k = 0; k < len; k++) *o++ = src[k];
    } else {
        for (u64 k = 0; k < len; k++) *o++ = (uint8_t)(k < 8 ? x.hi >> (56 - 8 * k) : x.lo >> (56 - 8 * (k - 8)));
    }
    *o++ = ':';
    *o++ = ' ';
    const u32 nd = ndigits(x.cnt);
    put_digits(o, x.cnt, nd);
    o[nd] = '\n';
}
static_assert(2 * FM_IPT == 8, "a bucket window is formatted as two halves of FM_IPT records per thread");

// the bucket's register network by size class (a call each: the 8-entry class alone needs more
// registers than the rest of the kernel, and inlined it spilled everything around it)
template <int E>
__device__ __attribute__((noinline)) void fr_bucket_sort(const Rec* X, u32 m, u64* kh, u64* kl, uint16_t* kp) {
    sb_sort_regs<FR_NT, E>(X, m, kh, kl, kp, E < 8 ? true : (bool)WCG_SORT_HIONLY_BIG);
}

__global__ __launch_bounds__(FR_NT, 2) void k_fused_reduce(FrArgs a) {
    __shared__ u64 kh[FR_CAP], kl[FR_CAP];
    __shared__ uint16_t kp[FR_CAP], kq[FR_CAP];
    __shared__ uint16_t runs[FR_CAP / 2];
    __shared__ u64 sp_hi[FR_BMAX], sp_lo[FR_BMAX];
    __shared__ u32 hcnt[FR_BMAX], gbase[FR_BMAX];
    __shared__ __align__(16) uint8_t stage[FR_STAGE];
    __shared__ u64 ws[FR_NT / 64];
    __shared__ u64 s_base;
    __shared__ u32 s_item, s_last, s_fail, s_nruns, s_rend, s_cnt;
    const u32 tid = threadIdx.x;
    FrCtl* const C = a.ctl;
    const u32 ep = a.epoch;
    u64 n = 0, B = 0, S = 0;

    // the parameters of phase q, published by the workgroup that completed phase q - 1 (a
    // phase without items publishes the next one at once)
    auto publish = [&](int q) {
        for (; q <= FR_NPH; q++) {
            u64 items = 0;
            if (q == 1) {                             // after compaction: n, buckets, samples
                if (tid == 0) {
                    const u64 nn = atomicAdd((unsigned long long*)&a.st->nrec, 0ull);
                    const u64 n1 = nn < a.rec_cap ? nn : a.rec_cap;
                    u64 bb = n1 ? (n1 + a.target - 1) / a.target : 0;
                    bb = bb > FR_BMAX ? FR_BMAX : bb;
                    const u64 ss = bb > 1 ? bb * FR_OVS : 0;
                    C->n = n1; C->B = bb; C->S = ss; C->nrun = (ss + FR_RUN - 1) / FR_RUN;
                    s_base = bb;
                }
                __syncthreads();
                for (u64 b = tid; b < s_base; b += FR_NT) a.bcnt[b] = 0;
                items = (s_base > 1) ? (s_base * FR_OVS + FR_RUN - 1) / FR_RUN : 0;
            } else if (q == 2) {                      // after the sample runs: scatter chunks
                if (tid == 0) { C->nchunk = (C->n + FR_CHUNK - 1) / FR_CHUNK; s_base = C->nchunk; }
                __syncthreads();
                items = s_base;
            } else if (q == 3) {                      // after the scatter: bucket starts
                const u64 bb = C->B;
                u64 c[2];
                for (int k = 0; k < 2; k++) {
                    const u64 b = 2 * tid + k;
                    c[k] = b < bb ? (u64)atomicAdd(&a.bcnt[b], 0u) : 0;
                }
                u64 all;
                const u64 pre = fr_scan(c[0] + c[1], ws, &all);
                if (2 * tid < bb) a.bstart[2 * tid] = pre;
                if (2 * tid + 1 < bb) a.bstart[2 * tid + 1] = pre + c[0];
                if (tid == 0) a.bstart[bb] = all;
                if (tid == 0 && all != C->n) atomicAdd(&a.st->spin_fail, 1u);   // never expected
                items = bb;
                if (bb == 0 && tid == 0) *a.total_out = 0;
            } else {
                break;                                 // q == FR_NPH: nothing after the buckets
            }
            fr_release_wg();
            if (tid == 0) __hip_atomic_store(&C->ready[q][0], ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
            if (items) break;
        }
    };

    bool failed = false, have_sp = false;
    for (int p = 0; p < FR_NPH && !failed; p++) {
        if (p > 0) {
            if (tid == 0) {
                u32 spins = 0, f = 0;
                while (fr_poll(&C->ready[p][0]) != ep) {
                    __builtin_amdgcn_s_sleep(2);
                    if (++spins > FR_SPIN_LIMIT) { f = 1; atomicAdd(&a.st->spin_fail, 1u); break; }
                }
                s_fail = f;
            }
            fr_acquire_wg();
            if (s_fail) { failed = true; break; }
            n = C->n; B = C->B; S = C->S;
        }
        const u64 nitems = p == 0 ? a.nitems0 : p == 1 ? C->nrun : p == 2 ? C->nchunk : B;
        while (true) {
            if (tid == 0) s_item = atomicAdd(&C->ticket[p][0], 1u);
            __syncthreads();
            const u64 item = s_item;
            __syncthreads();
            if (item >= nitems) break;
            if (p == 0) {
                compact_block(a.gtab, a.gslots, a.ltab, a.lslots, a.arena, a.rec, a.rec_cap, a.st, nullptr, nullptr,
                              item);
            } else if (p == 1) {
                // ---- sample run `item`: samples j = item * FR_RUN + i, record j * n / S
                u64 h[2], l[2];
                u32 q[2];
#pragma unroll
                for (int e = 0; e < 2; e++) {
                    const u32 i = tid * 2 + e;
                    const u64 j = item * FR_RUN + i;
                    q[e] = i;
                    if (j < S) { const Rec& r = a.rec[j * n / S]; h[e] = r.hi; l[e] = r.lo; }
                    else { h[e] = ~0ull; l[e] = ~0ull; }
                }
                reg_bitonic_unrolled<FR_NT, 2>(h, l, q, kh, kl, kp);
                const u64 r0 = item * FR_RUN;
                for (u32 i = tid; i < FR_RUN && r0 + i < S; i += FR_NT) {
                    a.smp[r0 + i] = kh[i]; a.smp[FR_SMAX + r0 + i] = kl[i];
                }
            } else if (p == 2) {
                if (!have_sp && B > 1) {
                    // ---- the splitters, from the sample runs (each scatter workgroup, once)
                    for (u32 j = tid; j < S; j += FR_NT) { kh[j] = a.smp[j]; kl[j] = a.smp[FR_SMAX + j]; }
                    __syncthreads();
                    const u32 nrun = (u32)((S + FR_RUN - 1) / FR_RUN);
                    for (u32 j = tid; j < S; j += FR_NT) {
                        const u32 rs = j / FR_RUN;
                        const u64 xh = kh[j], xl = kl[j];
                        u64 rank = j - rs * FR_RUN;
                        for (u32 r = 0; r < nrun; r++) {
                            if (r == rs) continue;
                            const u32 r0 = r * FR_RUN, rl = (u32)(S - r0 < FR_RUN ? S - r0 : FR_RUN);
                            u32 lo = 0, hi = rl;                // runs before: entries <= x; after: entries < x
                            while (lo < hi) {
                                const u32 mid = (lo + hi) >> 1;
                                const u64 yh = kh[r0 + mid], yl = kl[r0 + mid];
                                const bool below = r < rs ? !(xh < yh || (xh == yh && xl < yl)) : (yh < xh || (yh == xh && yl < xl));
                                if (below) lo = mid + 1; else hi = mid;
                            }
                            rank += lo;
                        }
                        const u64 m1 = (rank * B + S - 1) / S;  // splitter m1 - 1 = the sample of rank floor(m1 S / B)
                        if (m1 >= 1 && m1 <= B - 1 && (m1 * S) / B == rank) { sp_hi[m1 - 1] = xh; sp_lo[m1 - 1] = xl; }
                    }
                    __syncthreads();
                    have_sp = true;
                }
                // ---- scatter chunk `item` into the bucket regions
                for (u32 b = tid; b < B; b += FR_NT) hcnt[b] = 0;
                __syncthreads();
                Rec r[4];
                u32 bk[4], loc[4];
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const u64 i = item * FR_CHUNK + e * FR_NT + tid;
                    bk[e] = ~0u;
                    if (i < n) {
                        r[e] = a.rec[i];
                        u32 lo = 0, hi = (u32)B - 1;   // splitters <= the record
                        while (lo < hi) {
                            const u32 mid = (lo + hi) >> 1;
                            const bool le = sp_hi[mid] < r[e].hi || (sp_hi[mid] == r[e].hi && sp_lo[mid] <= r[e].lo);
                            if (le) lo = mid + 1; else hi = mid;
                        }
                        bk[e] = lo;
                        loc[e] = atomicAdd(&hcnt[lo], 1u);
                    }
                }
                __syncthreads();
                for (u32 b = tid; b < B; b += FR_NT) gbase[b] = hcnt[b] ? atomicAdd(&a.bcnt[b], hcnt[b]) : 0u;
                __syncthreads();
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    if (bk[e] == ~0u) continue;
                    const u32 pos = gbase[bk[e]] + loc[e];
                    if (pos < FR_RCAP) a.reg[(u64)bk[e] * FR_RCAP + pos] = r[e];
                    else {
                        const u32 o = atomicAdd(&C->nspill[0], 1u);
                        if (o < a.spill_cap) { a.spill[o] = r[e]; a.spill_bid[o] = bk[e]; }
                        else atomicAdd(&a.st->overflow, 1u);   // (the list holds every record)
                    }
                }
            } else {
                // ---- bucket `item`: sort, tie runs, lines, look-back, write
                const u32 b = (u32)item;
                const u64 s0 = a.bstart[b], m = a.bstart[b + 1] - s0;
                const bool inl = m <= FR_RCAP;
                const Rec* X = a.reg + (u64)b * FR_RCAP;
                if (m > 0 && inl) {
                    if (m <= FR_NT) fr_bucket_sort<1>(X, (u32)m, kh, kl, kp);
                    else if (m <= 2 * FR_NT) fr_bucket_sort<2>(X, (u32)m, kh, kl, kp);
                    else if (m <= 4 * FR_NT) fr_bucket_sort<4>(X, (u32)m, kh, kl, kp);
                    else fr_bucket_sort<8>(X, (u32)m, kh, kl, kp);
                    fr_fix_runs(X, (u32)m, kh, kl, kp, kq, a.arena, runs, &s_nruns, &s_rend);
                } else if (m > 0) {
                    fr_sort_global(a, b, s0, m, kh, kl, kp, kq, runs, &s_nruns, &s_rend, &s_cnt);
                }
                const Rec* const D = a.out_rec + s0;
                // the sorted record at position j
                auto rec_at = [&](u64 j) -> Rec { return inl ? X[kp[j]] : D[j]; };
                // the lines' lengths of window w0 (thread t: positions w0 + 8 t + e); the records
                // are read again when their lines are written (holding 8 records would cost 64 VGPRs)
                u32 L[8];
                auto lengths = [&](u64 w0, bool copy) -> u64 {
                    u64 s = 0;
#pragma unroll
                    for (int e = 0; e < 8; e++) {
                        const u64 j = w0 + tid * 8 + e;
                        L[e] = 0;
                        if (j < m) {
                            const Rec x = rec_at(j);
                            L[e] = (u32)line_len(x, FMT_MERGED, 1, 0, a.arena);
                            if (copy) a.out_rec[s0 + j] = x;
                        }
                        s += L[e];
                    }
                    return s;
                };
                // the bucket's bytes (a bucket of more than one window is summed first)
                u64 T = 0;
                for (u64 w0 = 0; w0 < m; w0 += FR_CAP) T += block_sum_u64(lengths(w0, inl), ws);
                if (tid == 0) {
                    __hip_atomic_store(&a.bflag[b], (u64)ep << 40 | T, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                // look-back: the bytes of every earlier bucket (wave 0 polls 64 flags at a time)
                if (m > 0 || b + 1 == B) {
                    if (tid < 64) {
                        u64 sum = 0;
                        u32 f = 0;
                        for (u32 b0 = 0; b0 < b; b0 += 64) {
                            const u32 bb = b0 + tid;
                            if (bb < b) {
                                u64 v;
                                u32 spins = 0;
                                while (((v = fr_poll64(&a.bflag[bb])) >> 40) != ep) {
                                    __builtin_amdgcn_s_sleep(2);
                                    if (++spins > FR_SPIN_LIMIT) { f = 1; break; }
                                }
                                sum += v & ((1ull << 40) - 1);
                            }
                        }
                        for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, 64);
                        f = __any(f) ? 1u : 0u;
                        if (tid == 0) {
                            s_base = sum;
                            s_fail = f;
                            if (f) atomicAdd(&a.st->spin_fail, 1u);
                        }
                    }
                    __syncthreads();
                    const u64 base = s_base;
                    if (b + 1 == B && tid == 0) *a.total_out = base + T;
                    u64 woff = 0;                         // bytes of the earlier windows
                    for (u64 w0 = 0; w0 < m && !s_fail; w0 += FR_CAP) {
                        const u64 s = m > FR_CAP ? lengths(w0, false) : (u64)L[0] + L[1] + L[2] + L[3] + L[4] + L[5] + L[6] + L[7];
                        u64 W;
                        const u64 lo = fr_scan(s, ws, &W);
                        uint8_t* const dst = a.out + base + woff;
                        const u32 pad = (u32)((uintptr_t)dst & 15);
                        const bool staged = pad + W <= FR_STAGE;
                        u64 o = lo;
#pragma unroll
                        for (int h = 0; h < 2; h++) {
                            Rec y[FM_IPT];
                            u64 LL[FM_IPT];
#pragma unroll
                            for (int e = 0; e < FM_IPT; e++) {
                                const u64 j = w0 + tid * 8 + h * FM_IPT + e;
                                LL[e] = L[h * FM_IPT + e];
                                if (LL[e]) y[e] = rec_at(j);
                            }
#pragma unroll
                            for (int e = 0; e < FM_IPT; e++) {
                                if (!LL[e]) continue;
                                if (staged) fr_line(y[e], a.arena, stage + pad + o);
                                else fr_line(y[e], a.arena, dst + o);
                                o += LL[e];
                            }
                        }
                        if (staged) {
                            __syncthreads();
                            uint8_t* const base16 = dst - pad;
                            const u32 tot = pad + (u32)W;
                            for (u32 c = tid; 16 * c < tot; c += FR_NT) {
                                const u32 b0 = 16 * c, b1 = b0 + 16 < tot ? b0 + 16 : tot;
                                if (b0 >= pad && b1 == b0 + 16)
                                    *reinterpret_cast<uint4*>(base16 + b0) = *reinterpret_cast<const uint4*>(stage + b0);
                                else
                                    for (u32 q = b0 > pad ? b0 : pad; q < b1; q++) base16[q] = stage[q];
                            }
                        }
                        __syncthreads();                  // the stage is rewritten by the next window
                        woff += W;
                    }
                }
            }
            // ---- the item is done: publish its stores, count it; the last one opens the next phase
            fr_release_wg();
            if (tid == 0) s_last = atomicAdd(&C->done[p][0], 1u) == (u32)nitems - 1 ? 1u : 0u;
            __syncthreads();
            if (s_last) {
                fr_acquire_wg();                      // the phase's data, for the parameters
                publish(p + 1);
            }
        }
    }
    // leave; the last workgroup out zeroes the counters for the next launch
    __syncthreads();
    if (tid == 0 && atomicAdd(&C->exits[0], 1u) == gridDim.x - 1) {
        for (int p = 0; p < FR_NPH; p++) { C->ticket[p][0] = 0; C->done[p][0] = 0; }
        C->nspill[0] = 0;
        C->exits[0] = 0;
    }
}

}  // namespace wcg
