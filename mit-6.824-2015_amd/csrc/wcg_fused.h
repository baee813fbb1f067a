// wcg_fused.h - DoReduce + Merge of a small job in ONE launch (r05): compaction, sample sort,
// tie order and "key: count\n" formatting (mapreduce.go:239-321: DoReduce's sort.Strings and
// Reduce, Merge's sort.Strings and Fprintf) for one-pass jobs of up to FR_NMAX keys.
//
// The general reduce (wcg_reduce.h + wcg_sort.h) is ~20 launches: on the metric's config (C2:
// 1e5 keys) they were 4-18 us each, ~175 us of a 1.3 ms step for a few MB of records
// (profiles/r04_kernel_summary_c2_final.txt).  Here the same work is four phases of one
// persistent launch:
//   P0 sample        S = 2048 keys straight from the hash tables (slot j T / S, then the first
//                    key in the next 64 slots; one wave, one read each), and the occupied slots
//                    those windows saw: the key-count estimate that sets the bucket count B
//   P1 splitters     the sample ranked by whole waves against the sample in LDS; the samples of
//                    rank (k + 1) S / B are the splitters
//   P2 scatter       compaction itself: one item per block of 2048 table slots builds each key's
//                    record, finds its bucket by binary search over the splitters in LDS and
//                    appends it to the bucket's region (one global atomic per item and bucket), and
//                    adds its line's bytes to the bucket's byte count; a full region spills to a list
//   P3 buckets       one item per bucket: register network on (hi, lo) (the unrolled networks of
//                    wcg_sort.h), long keys sharing a 16-byte prefix ordered by their full bytes,
//                    the lines staged in LDS and written with 16-byte stores at the bucket's place
//                    (the exclusive prefix of the byte counts: no bucket waits for another)
// Work is handed out by per-phase ticket counters (64 shards per phase: shard s hands out items s,
// s + 64, ...; a workgroup draws from shard blockIdx % 64 and, once that is empty, from any other
// that its wave's lanes see open), and a workgroup waits for a phase only once
// every item of the phase before it has been taken (by running workgroups), so the launch cannot
// deadlock whatever the residency: a workgroup that starts late finds no tickets and leaves.  The
// workgroup that completes a phase's last item publishes the next phase's parameters (release
// fence, then the phase's ready words = the launch's epoch | B << 32); the others poll a copy.
// Visibility across the 8 XCDs (whose L2s are not coherent with each other):
//   - items write what a later phase reads with write-through stores (fr_st: sc1) and drain them
//     (vmcnt(0)) before they are counted; the publisher's own stores go out with its release;
//   - consumers read with plain loads after the poll and take NO acquire.  An agent acquire is an
//     L2 invalidate of the XCD (buffer_inv sc1): 64 workgroups per XCD invalidating in turn spread
//     each phase's wake-up over ~4.5 us (r05 clock: entry q10-max 9.0-12.2 us with it, 7.8-8.2
//     without).  No stale copy can be hit instead: the dispatch invalidates the caches at the
//     launch's start, and no line a phase hands over (samples, splitters, bucket regions, spill
//     list, bucket starts) is read by anyone in the launch before it is handed over.
// The last workgroup to leave zeroes the counters for the next launch.
//
// Rare cases stay exact, only slower: a bucket past its region (FR_RCAP records: the sample put
// too few splitters there, or the estimate of the key count was far off) is gathered from the spill
// list and merge-sorted
// by the workgroup in global memory with the full-key order; a long-key tie run of any length is
// ordered by counting ranks under the full-key order.
#pragma once
#include <cstddef>

#include "wcg_common.h"
#include "wcg_sort.h"
#include "wcg_reduce.h"

namespace wcg {

constexpr int FR_NT = 256;
constexpr u32 FR_CAP = 2048;            // bucket records sorted in LDS (8 per thread)
constexpr u32 FR_RCAP = FR_CAP;         // records per bucket region
constexpr u32 FR_BMAX = 512;            // buckets
constexpr u32 FR_SMAX = 2048;           // samples (always; >= 4 per bucket)
constexpr u32 FR_WIN = 64;              // table slots a sample wave reads (its first key is the sample)
constexpr u32 FR_TARGET = 256;          // mean records per bucket (the region holds 8x that)
constexpr u32 FR_STAGE = 16384;         // a bucket's lines staged in LDS (more: written directly)
constexpr u64 FR_NMAX = 1ull << 17;     // the host takes this path for jobs up to this many keys
constexpr int FR_NPH = 4;
constexpr u32 FR_SPIN_LIMIT = 1u << 24;  // polls (s_sleep 1 each, ~1 s): then spin_fail
static_assert(FR_SMAX <= FR_CAP, "the sample is staged in the bucket sort's LDS arrays");

// counters and parameters, one 128-byte line each (the counters take every workgroup's atomics)
constexpr u32 FR_SHARDS = 8;             // done counters per phase (workgroup % 8: one per XCD under
                                         // round-robin dispatch), then one top counter per phase
// Words that many workgroups hit at once are spread over FR_SPREAD-byte strides (device-scope
// atomics and polls are served one at a time per address at the memory side: 512 workgroups polling
// one ready word woke over ~4.5 us, the last ones ~10 ns x 512 after the first).
#ifndef FR_ENTRY_ACQUIRE
#define FR_ENTRY_ACQUIRE 0      // 1: an agent acquire at every phase entry (measurement only)
#endif
constexpr u32 FR_SPREAD = 4096 / sizeof(u32);
constexpr u32 FR_TSHARDS = 64;           // ticket shards per phase (one lane each in the draw)
constexpr u32 FR_RCOPIES = 16;           // copies of each ready word; workgroup w polls w % 16
struct FrCtl {
    u32 done[FR_NPH][32];                // top: shards completed
    u32 exits[32];
    u32 nspill[32];
    u64 B, pad[15];                      // parameters (plain stores before a ready word), a line alone
    u32 dshard[FR_NPH][FR_SHARDS][FR_SPREAD];    // items completed per shard
    u32 tk[FR_NPH][FR_TSHARDS][FR_SPREAD];       // tickets drawn per shard (may pass its item count)
    u64 ready[FR_NPH][FR_RCOPIES][FR_SPREAD / 2];   // epoch | B << 32 once the phase's parameters are out
};

// ---- the hand-over invariant of the header, executable.  Consumers read
// handed-over data with plain loads and no acquire, which is only exact while no 128-byte line a
// phase hands over shares a cache line with anything read (or written) before the hand-over.  So:
// every field of FrCtl that one party writes and another reads starts a line of its own, and every
// array of the fused reduce's allocation (fr_layout below: bucket regions, spill records, spill
// buckets, samples and splitters, sample occupancy, counts, bytes, starts, offsets, the control
// block) starts on a line boundary and ends on one.
constexpr u64 FR_LINE = 128;
static_assert(offsetof(FrCtl, done) % FR_LINE == 0 && sizeof(FrCtl::done[0]) == FR_LINE, "done: a line per phase");
static_assert(offsetof(FrCtl, exits) % FR_LINE == 0 && sizeof(FrCtl::exits) == FR_LINE, "exits: one line");
static_assert(offsetof(FrCtl, nspill) % FR_LINE == 0 && sizeof(FrCtl::nspill) == FR_LINE, "nspill: one line");
static_assert(offsetof(FrCtl, B) % FR_LINE == 0 && offsetof(FrCtl, dshard) - offsetof(FrCtl, B) == FR_LINE,
              "B: a line of its own (it shared one with dshard until r06)");
static_assert(offsetof(FrCtl, dshard) % FR_LINE == 0 && (FR_SPREAD * sizeof(u32)) % FR_LINE == 0, "dshard: line strides");
static_assert(offsetof(FrCtl, tk) % FR_LINE == 0, "tk: line strides");
static_assert(offsetof(FrCtl, ready) % FR_LINE == 0 && (FR_SPREAD / 2 * sizeof(u64)) % FR_LINE == 0, "ready: line strides");
static_assert(sizeof(FrCtl) % FR_LINE == 0, "the control block ends on a line");

// the allocation's arrays, in order (host: reduce_fused); T = table slots (gtab + ltab)
struct FrLayout { u64 reg, spill, spill_bid, smp, socc, bcnt, bbytes, bstart, boff, ctl, all; };
__host__ __device__ constexpr u64 fr_round(u64 x) { return (x + 255) & ~255ull; }
__host__ __device__ constexpr FrLayout fr_layout(u64 T) {
    FrLayout L{};
    u64 q = 0;
    L.reg = q;       q += fr_round((u64)FR_BMAX * FR_RCAP * sizeof(Rec));
    L.spill = q;     q += fr_round(T * sizeof(Rec));
    L.spill_bid = q; q += fr_round(T * sizeof(u32));
    L.smp = q;       q += fr_round(4ull * FR_SMAX * sizeof(u64));
    L.socc = q;      q += fr_round(FR_SMAX * sizeof(u32));
    L.bcnt = q;      q += fr_round(FR_BMAX * sizeof(u32));
    L.bbytes = q;    q += fr_round(FR_BMAX * sizeof(u64));
    L.bstart = q;    q += fr_round((FR_BMAX + 1) * sizeof(u64));
    L.boff = q;      q += fr_round((FR_BMAX + 1) * sizeof(u64));
    L.ctl = q;       q += fr_round(sizeof(FrCtl));
    L.all = q;
    return L;
}
__host__ __device__ constexpr bool fr_layout_lines(u64 T) {
    const FrLayout L = fr_layout(T);
    const u64 o[] = {L.reg, L.spill, L.spill_bid, L.smp, L.socc, L.bcnt, L.bbytes, L.bstart, L.boff, L.ctl, L.all};
    for (u64 x : o)
        if (x % FR_LINE) return false;
    return true;
}
static_assert(fr_layout_lines(1) && fr_layout_lines(3) && fr_layout_lines(1ull << 17) && fr_layout_lines((1ull << 17) + 7) &&
              fr_layout_lines(12345679), "every fused-reduce array starts and ends on a 128-byte line");

struct FrArgs {
    const GEntry* gtab; u64 gslots;
    const GEntry* ltab; u64 lslots;
    const uint8_t* arena;
    DevState* st;
    u64* total_out;          // formatted bytes (the scalar the host reads back)
    Rec* rec; u64 rec_cap;   // scratch of the oversized-bucket path
    Rec* out_rec;            // sorted records (wcg_partition_all and the exports read them)
    uint8_t* out;            // formatted text
    Rec* reg;                // FR_BMAX x FR_RCAP bucket regions
    Rec* spill; u32* spill_bid; u64 spill_cap;
    u64* smp;                // [4][FR_SMAX]: the sample's hi and lo words, then the splitters' hi and lo
    u32* socc;               // [FR_SMAX / 4] occupied slots seen by each sample item (the key-count estimate)
    u32* bcnt;               // [FR_BMAX] records per bucket
    u64* bbytes;             // [FR_BMAX] formatted bytes per bucket
    u64* bstart;             // [FR_BMAX + 1] bucket starts in the sorted order
    u64* boff;               // [FR_BMAX + 1] bucket starts in the formatted text
    FrCtl* ctl;
    u32 epoch;               // 1 .. 2^24 - 1, a new one per launch
    u32 target;              // mean records per bucket
    u32 nitems0;             // table blocks (CP_NT * CP_IPT slots each)
    u64* clk;                // diagnostics (WCG_FUSED_CLOCK): per workgroup [FR_CLK] wall clocks, or null
    u64* host_st;            // the pinned host copy of DevState + scalars (device pointer): written by
                             // the last workgroup out, in place of a read-back copy after the launch
};
// clk[w * FR_CLK + ...]: 0 start; 1 + 3p phase p entered (ready seen), 2 + 3p its first item taken,
// 3 + 3p phase p left (no more tickets); FR_CLK - 1: items done by this workgroup
constexpr int FR_CLK = 16;
constexpr u32 FR_CLK_ITEMS = 4096;     // + per item of each phase: [FR_NPH][FR_CLK_ITEMS][8] after the
                                       // workgroup rows: taken, 4 sub-steps, work done, released, counted


// ---- device view of the arguments: the same pointers typed global (address space 1) and held in
// LDS.  Every phase is a call of its own (inlined into one body, the phases' live ranges merged into
// 256 VGPRs and ~150 scratch spills, and every item ran several times slower than the same code as a
// kernel); a call's generic pointers are flat pointers, whose loads also count in lgkmcnt, so every
// LDS wait of the networks and the formatting drained them.  Pointers read from this block keep the
// global address space through the calls and through the inlined helpers they are cast back for.
#if defined(__HIP_DEVICE_COMPILE__)
#define FR_G __attribute__((address_space(1)))
#else
#define FR_G                                              // (the host pass only parses the device code)
#endif
struct FrG {
    const FR_G GEntry* gtab; const FR_G GEntry* ltab; const FR_G uint8_t* arena;
    FR_G DevState* st; FR_G u64* total_out;
    FR_G Rec* rec; FR_G Rec* out_rec; FR_G uint8_t* out; FR_G Rec* reg;
    FR_G Rec* spill; FR_G u32* spill_bid; FR_G u64* smp; FR_G u32* socc; FR_G u32* bcnt; FR_G u64* bbytes;
    FR_G u64* bstart; FR_G u64* boff;
    FR_G FrCtl* ctl; FR_G u64* clk;
    u64* host_st;
    u64 gslots, lslots, rec_cap, spill_cap;
    u32 epoch, target, nitems0;
};

// the launch's LDS (namespace scope: the calls below name it directly, so it stays LDS)
__shared__ FrG fr_g;
__shared__ u64 fr_kh[FR_CAP], fr_kl[FR_CAP];
__shared__ uint16_t fr_kp[FR_CAP], fr_kq[FR_CAP];
__shared__ uint16_t fr_runs[FR_CAP / 2];
__shared__ u64 fr_sph[FR_BMAX], fr_spl[FR_BMAX];
__shared__ u32 fr_hcnt[FR_BMAX], fr_gbase[FR_BMAX];
__shared__ u64 fr_hbytes[FR_BMAX];
__shared__ __align__(16) uint8_t fr_stage[FR_STAGE];
__shared__ u64 fr_ws[FR_NT / 64];
__shared__ u64 fr_sb, fr_sn, fr_ss;
__shared__ u32 fr_s_item, fr_s_last, fr_s_fail, fr_s_nruns, fr_s_rend, fr_s_cnt;

#define FR_NOINLINE __device__ __attribute__((noinline))

__device__ __forceinline__ u32 fr_poll(const FR_G u32* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ u64 fr_poll64(const FR_G u64* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ u32 fr_add(FR_G u32* p, u32 v) { return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ u64 fr_add64(FR_G u64* p, u64 v) { return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// write-through (sc1) stores for what a later phase reads on other CUs: with every storing wave's
// stores drained before the item is counted, no per-item release fence (an L2 write-back, 2-11 us
// per item under load) is needed; the consumers acquire at the phase entry (MI355X_MICROARCH.md,
// valid forms: sc1 payload + drained counter + consumer acquire)
__device__ __forceinline__ void fr_st(FR_G u64* p, u64 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void fr_st(FR_G u32* p, u32 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
#ifndef FR_REC_STORE
#define FR_REC_STORE 1          // 0: four 8-byte write-through stores, 1: two 16-byte ones, 2: plain
#endif                          //    stores (the item then ends with an L2 write-back)
__device__ __forceinline__ void fr_st(FR_G Rec* p, const Rec& r) {
#if FR_REC_STORE == 0
    FR_G u64* q = reinterpret_cast<FR_G u64*>(p);
    fr_st(q, r.hi); fr_st(q + 1, r.lo); fr_st(q + 2, r.cnt); fr_st(q + 3, r.ref);
#elif FR_REC_STORE == 1
    typedef u32 v4u __attribute__((ext_vector_type(4)));
    const v4u a = {(u32)r.hi, (u32)(r.hi >> 32), (u32)r.lo, (u32)(r.lo >> 32)};
    const v4u b = {(u32)r.cnt, (u32)(r.cnt >> 32), (u32)r.ref, (u32)(r.ref >> 32)};
    FR_G v4u* q = reinterpret_cast<FR_G v4u*>(p);
    asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(q), "v"(a) : "memory");
    asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(q + 1), "v"(b) : "memory");
#else
    *p = r;
#endif
}

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
__device__ __forceinline__ u64 fr_scan(u64 s, u64* all) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    u64 incl = s;
    for (int d = 1; d < 64; d <<= 1) { const u64 y = __shfl_up(incl, d, 64); if (lane >= d) incl += y; }
    __syncthreads();                              // fr_ws of an earlier scan has been read
    if (lane == 63) fr_ws[w] = incl;
    __syncthreads();
    u64 pre = 0, t = 0;
    for (int k = 0; k < FR_NT / 64; k++) { if (k < w) pre += fr_ws[k]; t += fr_ws[k]; }
    *all = t;
    return pre + incl - s;
}

// Long keys sharing their 16-byte prefix sit next to each other after the (hi, lo) network, in any
// order: each such run of fr_kp[0, m) is reordered by counting, for each member, the members below
// it in the full-key order (keys are distinct, so the counts are a permutation).  X[fr_kp[j]] is
// the record at sorted position j.
__device__ __forceinline__ void fr_fix_runs(const Rec* X, u32 m, const uint8_t* arena) {
    const u32 tid = threadIdx.x;
    if (tid == 0) fr_s_nruns = 0;
    __syncthreads();
    for (u32 j = tid; j + 1 < m; j += FR_NT)
        if (fr_kh[j + 1] == fr_kh[j] && fr_kl[j + 1] == fr_kl[j] &&
            (j == 0 || fr_kh[j - 1] != fr_kh[j] || fr_kl[j - 1] != fr_kl[j]))
            fr_runs[atomicAdd(&fr_s_nruns, 1u)] = (uint16_t)j;
    __syncthreads();
    const u32 nr = fr_s_nruns;
    for (u32 r = 0; r < nr; r++) {
        const u32 s = fr_runs[r];
        if (tid == 0) {
            u32 e = s + 1;
            while (e < m && fr_kh[e] == fr_kh[s] && fr_kl[e] == fr_kl[s]) e++;
            fr_s_rend = e;
        }
        __syncthreads();
        const u32 k = fr_s_rend - s;
        for (u32 u = tid; u < k; u += FR_NT) {
            const uint16_t me = fr_kp[s + u];
            const Rec x = X[me];
            u32 rank = 0;
            for (u32 v = 0; v < k; v++)
                if (v != u && fr_less(X[fr_kp[s + v]], x, arena)) rank++;
            fr_kq[s + rank] = me;
        }
        __syncthreads();
        for (u32 u = tid; u < k; u += FR_NT) fr_kp[s + u] = fr_kq[s + u];
        __syncthreads();
    }
}

// a bucket past its region: its records (the region, then its entries of the spill list) are
// gathered into A = rec + start, sorted in LDS chunks of FR_CAP, merged in passes between A and
// D = out_rec + start by merge path under the full-key order; the result ends in D
FR_NOINLINE void fr_sort_global(u32 b, u64 s0, u64 m) {
    const FrG& g = fr_g;
    const u32 tid = threadIdx.x;
    const uint8_t* const arena = (const uint8_t*)g.arena;
    Rec* const A = (Rec*)(g.rec + s0);
    Rec* const D = (Rec*)(g.out_rec + s0);
    for (u32 i = tid; i < FR_RCAP; i += FR_NT) A[i] = g.reg[(u64)b * FR_RCAP + i];
    if (tid == 0) fr_s_cnt = 0;
    __syncthreads();
    const u64 ns = (u64)fr_add(&g.ctl->nspill[0], 0u);
    const u64 nsl = ns < g.spill_cap ? ns : g.spill_cap;
    for (u64 o = tid; o < nsl; o += FR_NT)
        if (g.spill_bid[o] == b) A[FR_RCAP + atomicAdd(&fr_s_cnt, 1u)] = g.spill[o];
    fr_release_wg();                              // (the same workgroup reads A below)
    fr_acquire_wg();
    if (FR_RCAP + fr_s_cnt != m && tid == 0) atomicAdd((u32*)&g.st->spin_fail, 1u);   // never expected
    for (u64 c0 = 0; c0 < m; c0 += FR_CAP) {
        const u32 cm = (u32)(m - c0 < FR_CAP ? m - c0 : FR_CAP);
        for (u32 j = tid; j < FR_CAP; j += FR_NT) {
            if (j < cm) { const Rec r = A[c0 + j]; fr_kh[j] = r.hi; fr_kl[j] = r.lo; }
            else { fr_kh[j] = ~0ull; fr_kl[j] = ~0ull; }
            fr_kp[j] = (uint16_t)j;
        }
        __syncthreads();
        lds_bitonic<FR_NT>(fr_kh, fr_kl, fr_kp, FR_CAP);
        __syncthreads();
        fr_fix_runs(A + c0, cm, arena);
        for (u32 j = tid; j < cm; j += FR_NT) D[c0 + j] = A[c0 + fr_kp[j]];
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
                if (fr_less(Y[d0 - 1 - mid], X[mid], arena)) hi = mid; else lo = mid + 1;
            }
            u64 ia = lo, ib = d0 - lo;
            for (u64 d = d0; d < d1; d++) {
                const bool takeX = ia < la && (ib >= lb || !fr_less(Y[ib], X[ia], arena));
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

// the record of table slot i (of the concatenated gtab ++ ltab) with entry e; q = the arena's 16
// bytes at a long key's home (read by the caller only for ltab slots)
__device__ __forceinline__ Rec fr_slot_rec(const GEntry& e, u64 i, u64 gslots, uint4 q) {
    if (i < gslots) return inline_rec(e.k0, e.k1, e.cnt);
    Rec r;
    r.hi = bswap64((u64)q.y << 32 | q.x);
    r.lo = bswap64((u64)q.w << 32 | q.z);
    r.cnt = e.cnt;
    r.ref = LONG_FLAG | (e.aux << 40) | (e.k1 - 1);
    return r;
}

// P0: the sample, straight from the tables (a hash table's slots are in no key order): sample j is
// the first key in the FR_WIN slots from j T / S (T = all slots), read by one wave in one pass (a
// ballot finds the first occupied slot); an empty window gives the all-ones sample (ranks last).
// Each item also counts the occupied slots its windows saw: the key-count estimate that sizes the
// buckets, with no compaction pass before the sort.
constexpr u32 FR_SPI = FR_NT / 64;                        // samples per item: one per wave
FR_NOINLINE void fr_sample_item(u64 item) {
    const FrG& g = fr_g;
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u64 T = g.gslots + g.lslots;
    const u64 j = item * FR_SPI + w;
    const u64 i = (j * T / FR_SMAX + lane) % T;
    const GEntry e = i < g.gslots ? g.gtab[i] : g.ltab[i - g.gslots];
    const u64 occ = __ballot(e.k0 != 0);
    const bool first = occ && lane == (u32)__builtin_ctzll(occ);
    u64 h = ~0ull, l = ~0ull;
    if (first) {
        uint4 q = make_uint4(0, 0, 0, 0);
        if (i >= g.gslots) { const uint4 v = *reinterpret_cast<const FR_G uint4*>(g.arena + (e.k1 - 1)); q = v; }
        const Rec r = fr_slot_rec(e, i, g.gslots, q);
        h = r.hi; l = r.lo;
    }
    if (first || (!occ && lane == 0)) { fr_st(&g.smp[j], h); fr_st(&g.smp[FR_SMAX + j], l); }
    if (lane == 0) fr_hcnt[w] = (u32)__popcll(occ);
    __syncthreads();
    if (tid == 0) {
        u32 t = 0;
        for (u32 k = 0; k < FR_SPI; k++) t += fr_hcnt[k];
        fr_st(&g.socc[item], t);
    }
}

// P1: the sample ranked in the (hi, lo, j) order - a permutation - one wave per sample: its 64
// lanes compare the sample with S / 64 entries each of the whole sample in LDS; a sample of rank
// floor((k + 1) S / B) is splitter k (smp[2 FR_SMAX + k], smp[3 FR_SMAX + k]).  (Sorting the sample
// in runs of 512 by register networks and ranking the runs against each other in every scatter
// workgroup took 11 + 27 us on the metric's config.)
FR_NOINLINE void fr_rank_item(u64 item, u64 B) {
    const FrG& g = fr_g;
    constexpr u64 S = FR_SMAX;
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (u32 j = tid; j < S; j += FR_NT) { fr_kh[j] = g.smp[j]; fr_kl[j] = g.smp[FR_SMAX + j]; }
    __syncthreads();
    const u32 j = (u32)item * FR_SPI + w;
    const u64 h = fr_kh[j], l = fr_kl[j];
    u32 r0 = 0, r1 = 0, r2 = 0, r3 = 0;                   // four independent compare chains
#pragma unroll 2
    for (u32 k = lane; k < S; k += 256) {
        r0 += key3_lt(fr_kh[k], fr_kl[k], k, h, l, j) ? 1u : 0u;
        r1 += key3_lt(fr_kh[k + 64], fr_kl[k + 64], k + 64, h, l, j) ? 1u : 0u;
        r2 += key3_lt(fr_kh[k + 128], fr_kl[k + 128], k + 128, h, l, j) ? 1u : 0u;
        r3 += key3_lt(fr_kh[k + 192], fr_kl[k + 192], k + 192, h, l, j) ? 1u : 0u;
    }
    u32 rank = r0 + r1 + r2 + r3;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) rank += __shfl_xor((int)rank, d, 64);
    if (lane == 0) {
        const u64 m1 = ((u64)rank * B + S - 1) / S;       // splitter m1 - 1 has rank floor(m1 S / B)
        if (m1 >= 1 && m1 <= B - 1 && (m1 * S) / B == rank) {
            fr_st(&g.smp[2 * FR_SMAX + m1 - 1], h);
            fr_st(&g.smp[3 * FR_SMAX + m1 - 1], l);
        }
    }
}
static_assert(FR_SMAX % 256 == 0, "fr_rank_item compares four 64-entry strides per round");

// P2: table block `item` (CP_NT * CP_IPT slots) compacted straight into the bucket regions: the
// block's keys become records, packed into LDS in rounds of FR_SROUND (a block is ~15% full: a
// search per slot ran 8 lockstep searches per thread for ~1.2 live ones), each record's bucket by
// binary search over the splitters in LDS (splitters <= the record by (hi, lo): equal prefixes -
// long-key ties - share a bucket), counted per bucket in LDS with its line's bytes, then one global
// atomic per bucket for the records and one for the bytes (so the bucket phase knows where every
// bucket's text goes), and the records written through to their regions.  A failed job (a full
// table, a malformed import) compacts nothing.
constexpr u32 FR_SROUND = FR_STAGE / sizeof(Rec);
FR_NOINLINE void fr_scatter_item(u64 item, u64 B, bool load_sp, FR_G u64* ick) {
    const FrG& g = fr_g;
    const u32 tid = threadIdx.x;
    if (load_sp) {                                        // the splitters (once per workgroup)
        for (u32 k = tid; k + 1 < B; k += FR_NT) { fr_sph[k] = g.smp[2 * FR_SMAX + k]; fr_spl[k] = g.smp[3 * FR_SMAX + k]; }
    }
    for (u32 b = tid; b < B; b += FR_NT) { fr_hcnt[b] = 0; fr_hbytes[b] = 0; }
    if (g.st->overflow | g.st->spin_fail | g.st->bad_input) return;    // (workgroup-uniform)
    const u64 T = g.gslots + g.lslots;
    const u64 b0 = item * (CP_NT * CP_IPT);
    GEntry e[CP_IPT];
#pragma unroll
    for (int k = 0; k < CP_IPT; k++) {                    // every slot first (one round trip)
        const u64 i = b0 + (u64)k * CP_NT + tid;
        const u64 li = i < T ? i - g.gslots : 0;
        e[k] = i < g.gslots ? g.gtab[i] : g.ltab[i < T ? li : 0];
        if (i >= T) e[k].k0 = 0;
    }
    uint4 q[CP_IPT];
    const bool has_long = b0 + (u64)CP_NT * CP_IPT > g.gslots;        // (workgroup-uniform)
#pragma unroll
    for (int k = 0; k < CP_IPT; k++) {
        const u64 i = b0 + (u64)k * CP_NT + tid;
        const bool lng = has_long && i >= g.gslots && e[k].k0 != 0;
        q[k] = make_uint4(0, 0, 0, 0);
        if (has_long) {
            const uint4 v = *reinterpret_cast<const FR_G uint4*>(g.arena + (lng ? e[k].k1 - 1 : 0));
            q[k] = v;
        }
    }
    u32 mine = 0, nlong = 0;
#pragma unroll
    for (int k = 0; k < CP_IPT; k++) {
        const u64 i = b0 + (u64)k * CP_NT + tid;
        mine += e[k].k0 != 0 ? 1u : 0u;
        nlong += e[k].k0 != 0 && i >= g.gslots ? 1u : 0u;
    }
    for (int d = 32; d >= 1; d >>= 1) nlong += __shfl_xor(nlong, d, 64);
    if ((tid & 63) == 0 && nlong) atomicAdd((unsigned long long*)&g.st->nlong, (unsigned long long)nlong);
    u64 all;
    const u32 first = (u32)fr_scan(mine, &all);           // this thread's records' positions in the block
    if (ick) ick[2] = wall_clock64();
    Rec* const stg = reinterpret_cast<Rec*>(fr_stage);
    for (u32 base = 0; base < all; base += FR_SROUND) {   // (one round unless the block is dense)
        u32 p = first;
#pragma unroll
        for (int k = 0; k < CP_IPT; k++) {
            if (e[k].k0 == 0) continue;
            if (p >= base && p < base + FR_SROUND) stg[p - base] = fr_slot_rec(e[k], b0 + (u64)k * CP_NT + tid, g.gslots, q[k]);
            p++;
        }
        __syncthreads();
        const u32 cnt = (u32)(all - base < FR_SROUND ? all - base : FR_SROUND);
        constexpr int RPT = FR_SROUND / FR_NT;            // records per thread in a round
        Rec r[RPT];
        u32 bk[RPT], loc[RPT], lo[RPT], len[RPT];
#pragma unroll
        for (int k = 0; k < RPT; k++) {
            const u32 j = tid + k * FR_NT;
            r[k] = stg[j < cnt ? j : 0];
            lo[k] = 0;
            len[k] = j < cnt ? (u32)B - 1 : 0;
        }
        for (u32 step = (u32)B; step; step >>= 1) {
#pragma unroll
            for (int k = 0; k < RPT; k++) {
                const u32 half = len[k] >> 1, mid = lo[k] + half;
                const u64 sh = fr_sph[mid];
                const bool le = sh < r[k].hi || (sh == r[k].hi && fr_spl[mid] <= r[k].lo);
                const bool live = len[k] != 0;
                lo[k] = live && le ? mid + 1 : lo[k];
                len[k] = !live ? 0u : le ? len[k] - half - 1 : half;
            }
        }
#pragma unroll
        for (int k = 0; k < RPT; k++) {
            bk[k] = tid + k * FR_NT < cnt ? lo[k] : ~0u;
            if (bk[k] == ~0u) continue;
            loc[k] = atomicAdd(&fr_hcnt[bk[k]], 1u);
            atomicAdd((unsigned long long*)&fr_hbytes[bk[k]], (unsigned long long)line_len(r[k], FMT_MERGED, 1, 0, nullptr));
        }
        __syncthreads();
        if (ick) ick[3] = wall_clock64();
        for (u32 b = tid; b < B; b += FR_NT) {
            fr_gbase[b] = fr_hcnt[b] ? fr_add(&g.bcnt[b], fr_hcnt[b]) : 0u;
            if (fr_hbytes[b]) fr_add64(&g.bbytes[b], fr_hbytes[b]);
        }
        __syncthreads();
        if (ick) ick[4] = wall_clock64();
#pragma unroll
        for (int k = 0; k < RPT; k++) {
            if (bk[k] == ~0u) continue;
            const u32 pos = fr_gbase[bk[k]] + loc[k];
            if (pos < FR_RCAP) fr_st(&g.reg[(u64)bk[k] * FR_RCAP + pos], r[k]);
            else {
                const u32 o = fr_add(&g.ctl->nspill[0], 1u);
                if (o < g.spill_cap) { fr_st(&g.spill[o], r[k]); fr_st(&g.spill_bid[o], bk[k]); }
                else atomicAdd((u32*)&g.st->overflow, 1u);   // (the list holds every record)
            }
        }
        __syncthreads();                                  // the stage and the counters are reused
        for (u32 b = tid; b < B; b += FR_NT) { fr_hcnt[b] = 0; fr_hbytes[b] = 0; }
    }
}

// the bucket's register network by size class (a call each: the 8-entry class alone needs more
// registers than the rest)
#ifndef FR_SORT_CMP
#define FR_SORT_CMP 1           // 0: the (hi, lo) network only (no compressed-word pass)
#endif
#ifndef FR_ABL_SORT
#define FR_ABL_SORT 0           // diagnostics (wrong order): 1 = the bucket's loads only, no network
#endif
template <int E>
FR_NOINLINE void fr_bucket_sort(const FR_G Rec* X, u32 m) {
    if (FR_ABL_SORT) {
        for (u32 i = threadIdx.x; i < m; i += FR_NT) {
            const uint4 v = *reinterpret_cast<const FR_G uint4*>(X + i);
            fr_kh[i] = (u64)v.y << 32 | v.x;
            fr_kl[i] = (u64)v.w << 32 | v.z;
            fr_kp[i] = (uint16_t)i;
        }
        __syncthreads();
        return;
    }
    sb_sort_regs<FR_NT, E>((const Rec*)X, m, fr_kh, fr_kl, fr_kp, FR_SORT_CMP && (E < 8 ? true : (bool)WCG_SORT_HIONLY_BIG));
}

// the lines of x[0, 8) with lengths L (0: none) at dst + lo: staged in LDS and written out in
// aligned 16-byte stores when the window's W bytes fit the stage, else byte by byte in place
__device__ __forceinline__ void fr_write_lines(const Rec (&x)[8], const u32 (&L)[8], const uint8_t* arena,
                                               FR_G uint8_t* dst, u64 lo, u64 W) {
    const u32 tid = threadIdx.x;
    const u32 pad = (u32)((uintptr_t)dst & 15);
    const bool staged = pad + W <= FR_STAGE;
    u64 o = lo;
#pragma unroll
    for (int e = 0; e < 8; e++) {
        if (!L[e]) continue;
        if (staged) fr_line(x[e], arena, fr_stage + pad + o);
        else fr_line(x[e], arena, dst + o);
        o += L[e];
    }
    if (!staged) return;                                  // (workgroup-uniform)
    __syncthreads();
    FR_G uint8_t* const base16 = dst - pad;
    const u32 tot = pad + (u32)W;
    for (u32 c = tid; 16 * c < tot; c += FR_NT) {
        const u32 b0 = 16 * c, b1 = b0 + 16 < tot ? b0 + 16 : tot;
        if (b0 >= pad && b1 == b0 + 16)
            *reinterpret_cast<FR_G uint4*>(base16 + b0) = *reinterpret_cast<const uint4*>(fr_stage + b0);
        else
            for (u32 q = b0 > pad ? b0 : pad; q < b1; q++) base16[q] = fr_stage[q];
    }
    __syncthreads();                                      // the stage is reused
}

// P3, a bucket of at most FR_CAP records sorted in LDS (fr_kp: sorted position -> region index):
// its sorted records, and its lines at the bucket's place in the text (known from the scatter's
// byte counts: no bucket waits for another)
FR_NOINLINE void fr_format_small(u32 b, u64 s0, u64 m) {
    const FrG& g = fr_g;
    const u32 tid = threadIdx.x;
    const uint8_t* const arena = (const uint8_t*)g.arena;
    const FR_G Rec* const X = g.reg + (u64)b * FR_RCAP;
    // this thread's ept = ceil(m / FR_NT) consecutive sorted positions (8 per thread left all but
    // m / 8 threads idle: a ~400-record bucket formatted on 48 lanes), read together
    const u32 ept = (u32)((m + FR_NT - 1) / FR_NT);
    const u64 j0 = (u64)tid * ept;
    Rec x[8];
    u32 L[8];
    u64 s = 0;
#pragma unroll
    for (int e = 0; e < 8; e++) {
        const u64 j = j0 + e;
        x[e] = X[(u32)e < ept && j < m ? fr_kp[j] : 0];
    }
#pragma unroll
    for (int e = 0; e < 8; e++) {
        const u64 j = j0 + e;
        const bool v = (u32)e < ept && j < m;
        L[e] = v ? (u32)line_len(x[e], FMT_MERGED, 1, 0, arena) : 0u;
        s += L[e];
        if (v) g.out_rec[s0 + j] = x[e];
    }
    u64 T;
    const u64 lo = fr_scan(s, &T);
    fr_write_lines(x, L, arena, g.out + g.boff[b], lo, T);
}

// P3, a bucket past its region, sorted by fr_sort_global into out_rec: windows of FR_CAP records
FR_NOINLINE void fr_format_big(u32 b, u64 s0, u64 m) {
    const FrG& g = fr_g;
    const u32 tid = threadIdx.x;
    const uint8_t* const arena = (const uint8_t*)g.arena;
    const FR_G Rec* const D = g.out_rec + s0;
    Rec x[8];
    u32 L[8];
    u64 woff = g.boff[b];
    for (u64 w0 = 0; w0 < m; w0 += FR_CAP) {
        u64 s = 0;
#pragma unroll
        for (int e = 0; e < 8; e++) {
            const u64 j = w0 + tid * 8 + e;
            x[e] = D[j < m ? j : 0];
            L[e] = j < m ? (u32)line_len(x[e], FMT_MERGED, 1, 0, arena) : 0u;
            s += L[e];
        }
        u64 W;
        const u64 lo = fr_scan(s, &W);
        fr_write_lines(x, L, arena, g.out + woff, lo, W);
        woff += W;
    }
}

// P3: bucket b - sort, tie runs, then the lines
FR_NOINLINE void fr_bucket_item(u32 b, FR_G u64* ick) {
    const FrG& g = fr_g;
    const u64 s0 = g.bstart[b], m = g.bstart[b + 1] - s0;
    if (m > FR_RCAP) {
        fr_sort_global(b, s0, m);
        fr_format_big(b, s0, m);
        return;
    }
    if (m == 0) return;                                   // (workgroup-uniform)
    const FR_G Rec* const X = g.reg + (u64)b * FR_RCAP;
    if (ick) ick[3] = m | 1ull << 62;                     // (the clock report's bucket size)
    if (m <= FR_NT) fr_bucket_sort<1>(X, (u32)m);   // (a rank sort - every record against all
                                                      // in LDS - measured 2x slower at 256: r05)
    else if (m <= 2 * FR_NT) fr_bucket_sort<2>(X, (u32)m);
    else if (m <= 4 * FR_NT) fr_bucket_sort<4>(X, (u32)m);
    else fr_bucket_sort<8>(X, (u32)m);
    if (ick) ick[1] = wall_clock64();
    fr_fix_runs((const Rec*)X, (u32)m, (const uint8_t*)g.arena);
    if (ick) ick[2] = wall_clock64();
    fr_format_small(b, s0, m);
}

// the parameters of phase q, by the workgroup that completed phase q - 1's last item (a phase
// without items publishes the next one at once)
FR_NOINLINE void fr_publish(int q) {
    const FrG& g = fr_g;
    const u32 tid = threadIdx.x;
    FR_G FrCtl* const C = g.ctl;
    for (bool chained = false; q < FR_NPH; q++, chained = true) {
        FR_G u64* const pk = g.clk && tid == 0 ? g.clk + (u64)gridDim.x * FR_CLK + 8ull * FR_NPH * FR_CLK_ITEMS + 8 * q : nullptr;
        if (pk) pk[0] = wall_clock64();
        // a chained phase reads what this workgroup's thread 0 published for the one before: past
        // the release above, an acquire (this CU's L1 may hold those lines from before)
        if (chained) fr_acquire_wg();
        if (pk) pk[1] = wall_clock64();
        u64 items = 0;
        if (q == 1) {                                     // after the sample: the key-count estimate, buckets
            u64 c[2];
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const u32 i = 2 * tid + k;
                c[k] = i < FR_SMAX / FR_SPI ? g.socc[i] : 0;
            }
            u64 occ;
            (void)fr_scan(c[0] + c[1], &occ);
            if (tid == 0) {
                const u64 T = g.gslots + g.lslots;
                const u64 n_est = occ * T / ((u64)FR_SMAX * FR_WIN);
                u64 bb = (n_est + g.target - 1) / g.target;
                bb = bb < 1 ? 1 : bb > FR_BMAX ? FR_BMAX : bb;
                C->B = bb;
                fr_sb = bb;
            }
            __syncthreads();
            const u64 bb = fr_sb;
            for (u64 b = tid; b < bb; b += FR_NT) { g.bcnt[b] = 0; g.bbytes[b] = 0; }
            items = bb > 1 ? FR_SMAX / FR_SPI : 0;
        } else if (q == 2) {                              // after the ranks: the table blocks
            items = g.nitems0;
        } else {                                          // q == 3, after the scatter: bucket starts
            const u64 bb = C->B;
            u64 c[2], y[2];
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const u64 b = 2 * tid + k;
                c[k] = b < bb ? (u64)fr_add(&g.bcnt[b], 0u) : 0;
                y[k] = b < bb ? fr_add64(&g.bbytes[b], 0ull) : 0;
            }
            u64 all, ally;
            const u64 pre = fr_scan(c[0] + c[1], &all);
            const u64 prey = fr_scan(y[0] + y[1], &ally);
            if (2 * tid < bb) { g.bstart[2 * tid] = pre; g.boff[2 * tid] = prey; }
            if (2 * tid + 1 < bb) { g.bstart[2 * tid + 1] = pre + c[0]; g.boff[2 * tid + 1] = prey + y[0]; }
            if (tid == 0) {
                g.bstart[bb] = all; g.boff[bb] = ally;
                g.st->nrec = all;                         // the record count the host reads back
                *g.total_out = ally;                      // and the text's size
            }
            items = bb;
        }
        if (pk) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); pk[2] = wall_clock64(); }
        fr_release_wg();
        if (pk) pk[3] = wall_clock64();
        if (tid < FR_RCOPIES)               // (fr_sb = B in every publisher: set by the poll, or above)
            __hip_atomic_store(&C->ready[q][tid][0], (u64)g.epoch | fr_sb << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (items) break;
    }
}

static_assert(FR_BMAX <= 2 * FR_NT, "fr_publish scans two bucket counts per thread");

__global__ __launch_bounds__(FR_NT, 2) void k_fused_reduce(FrArgs a) {
    const u32 tid = threadIdx.x;
    if (tid == 0) {
        FrG& g = fr_g;
        g.gtab = (const FR_G GEntry*)a.gtab; g.ltab = (const FR_G GEntry*)a.ltab;
        g.arena = (const FR_G uint8_t*)a.arena; g.st = (FR_G DevState*)a.st; g.total_out = (FR_G u64*)a.total_out;
        g.rec = (FR_G Rec*)a.rec; g.out_rec = (FR_G Rec*)a.out_rec; g.out = (FR_G uint8_t*)a.out;
        g.reg = (FR_G Rec*)a.reg; g.spill = (FR_G Rec*)a.spill; g.spill_bid = (FR_G u32*)a.spill_bid;
        g.smp = (FR_G u64*)a.smp; g.bcnt = (FR_G u32*)a.bcnt; g.bstart = (FR_G u64*)a.bstart;
        g.socc = (FR_G u32*)a.socc; g.bbytes = (FR_G u64*)a.bbytes; g.boff = (FR_G u64*)a.boff;
        g.ctl = (FR_G FrCtl*)a.ctl; g.clk = (FR_G u64*)a.clk; g.host_st = a.host_st;
        g.gslots = a.gslots; g.lslots = a.lslots; g.rec_cap = a.rec_cap; g.spill_cap = a.spill_cap;
        g.epoch = a.epoch; g.target = a.target; g.nitems0 = a.nitems0;
    }
    __syncthreads();
    const FrG& g = fr_g;
    FR_G FrCtl* const C = g.ctl;
    u64 B = 0;
    FR_G u64* const clk = g.clk && tid == 0 ? g.clk + (u64)blockIdx.x * FR_CLK : nullptr;
    u64 nitems_done = 0;
    if (clk) { clk[0] = wall_clock64(); for (int k = 1; k < FR_CLK; k++) clk[k] = 0; }
    bool failed = false, have_sp = false;
    for (int p = 0; p < FR_NPH && !failed; p++) {
        u32 pre_t = ~0u;                          // (thread 0) the phase's first ticket, drawn early
        if (p > 0) {
            if (tid == 0) {
                // the first ticket of the phase is drawn before its ready word is seen (a ticket
                // is only a number until the phase's item count is known): its round trip overlaps
                // the wait.  Still no residency assumption: it is drawn by a running workgroup.
                pre_t = fr_add(&C->tk[p][blockIdx.x % FR_TSHARDS][0], 1u);
                u32 spins = 0, f = 0;
                u64 rw;
                while ((u32)(rw = fr_poll64(&C->ready[p][blockIdx.x % FR_RCOPIES][0])) != g.epoch) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > FR_SPIN_LIMIT) { f = 1; atomicAdd((u32*)&g.st->spin_fail, 1u); break; }
                }
                fr_s_fail = f;
                fr_sb = rw >> 32;
            }
#if FR_ENTRY_ACQUIRE
            fr_acquire_wg();
#else
            __syncthreads();
#endif
            if (fr_s_fail) { failed = true; break; }
            B = fr_sb;
        }
        if (clk) clk[1 + 3 * p] = wall_clock64();
        bool first_item = true;
        const u64 nitems = p == 0 ? FR_SMAX / FR_SPI : p == 1 ? (B > 1 ? FR_SMAX / FR_SPI : 0) : p == 2 ? g.nitems0 : B;
        for (bool first = true;; first = false) {
            // A ticket from this workgroup's shard (8 workgroups per word: 512 on one word queued
            // 3-6 us, 64 on one ~1 us), else from any other shard still open: wave 0's 64 lanes
            // read the 64 shard counters at once and the first open one is drawn from.  A workgroup leaves the phase
            // only once it has SEEN every shard empty, so every item has been drawn by a running
            // workgroup before anyone waits for the next phase: no residency assumption (a fixed
            // first item per workgroup deadlocked when another process's kernel held half the CUs
            // and the item's workgroup could not start).
            if (tid < 64) {
                const u32 lane = tid, sh = (blockIdx.x + lane) % FR_TSHARDS;
                const u32 lim = nitems > sh ? (u32)((nitems - sh + FR_TSHARDS - 1) / FR_TSHARDS) : 0u;
                u32 item = ~0u;
                if (first) {                      // the phase's first draw: straight at the own shard
                    u32 got = ~0u;
                    if (lane == 0) {
                        const u32 t = p > 0 ? pre_t : fr_add(&C->tk[p][sh][0], 1u);
                        if (t < lim) got = sh + FR_TSHARDS * t;
                    }
                    item = (u32)__shfl((int)got, 0, 64);
                }
                while (item == ~0u) {
                    const u32 v = lim ? fr_poll(&C->tk[p][sh][0]) : 0u;
                    const u64 open = __ballot(v < lim);
                    if (!open) break;                                  // every shard drawn out
                    const u32 pick = (u32)__builtin_ctzll(open);       // own shard first
                    u32 got = ~0u;
                    if (lane == pick) {
                        const u32 t = fr_add(&C->tk[p][sh][0], 1u);
                        if (t < lim) got = sh + FR_TSHARDS * t;
                    }
                    got = (u32)__shfl((int)got, (int)pick, 64);
                    if (got != ~0u) { item = got; break; }
                }
                if (lane == 0) fr_s_item = item;
            }
            __syncthreads();
            const u64 item = fr_s_item == ~0u ? ~0ull : (u64)fr_s_item;
            __syncthreads();
            if (item >= nitems) break;
            if (clk && first_item) clk[2 + 3 * p] = wall_clock64();
            first_item = false;
            nitems_done++;
            FR_G u64* const ick = clk && item < FR_CLK_ITEMS
                                      ? g.clk + (u64)gridDim.x * FR_CLK + ((u64)p * FR_CLK_ITEMS + item) * 8 : nullptr;
            if (ick) ick[0] = wall_clock64();
            if (p == 0) fr_sample_item(item);
            else if (p == 1) fr_rank_item(item, B);
            else if (p == 2) {
                fr_scatter_item(item, B, !have_sp, ick);
                have_sp = true;
            } else fr_bucket_item((u32)item, ick);
            // ---- the item is done: its stores (write-through) drained, it is counted in the
            // workgroup's shard; the last item of a shard counts the shard, and the workgroup that
            // completes the last shard opens the next phase
            if (ick) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); ick[5] = wall_clock64(); }
#if FR_REC_STORE == 2
            if (p == 2) fr_release_wg();
#endif
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (ick) ick[6] = wall_clock64();
            if (tid == 0) {
                // item i counts in shard i % FR_SHARDS (neighbouring items hit different words)
                const u32 ish = (u32)(item % FR_SHARDS);
                const u64 per = nitems / FR_SHARDS + ((u64)ish < nitems % FR_SHARDS ? 1 : 0);
                u32 last = 0;
                if (fr_add(&C->dshard[p][ish][0], 1u) == (u32)per - 1)
                    last = fr_add(&C->done[p][0], 1u) == (u32)(nitems < FR_SHARDS ? nitems : FR_SHARDS) - 1;
                fr_s_last = last;
            }
            if (ick) ick[7] = wall_clock64();
            __syncthreads();
            if (fr_s_last) {
                fr_acquire_wg();                          // the phase's data, for the parameters
                fr_publish(p + 1);
            }
        }
        if (clk) clk[3 + 3 * p] = wall_clock64();
    }
    if (clk) clk[FR_CLK - 1] = nitems_done;
    // leave; the last workgroup out zeroes the counters for the next launch
    __syncthreads();
    if (tid == 0 && fr_add(&C->exits[0], 1u) == gridDim.x - 1) {
        for (int p = 0; p < FR_NPH; p++) {
            C->done[p][0] = 0;
            for (u32 k = 0; k < FR_SHARDS; k++) C->dshard[p][k][0] = 0;
            for (u32 k = 0; k < FR_TSHARDS; k++) C->tk[p][k][0] = 0;
        }
        C->nspill[0] = 0;
        C->exits[0] = 0;
        if (g.host_st) {
            // the job's counters, error flags and sizes straight to the host's pinned copy (the
            // read-back copy after the launch was a ~4 us blit dispatch of its own); every other
            // workgroup has left, and their stores were released before they counted their items
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            const volatile FR_G u64* src = (const volatile FR_G u64*)g.st;
            for (u32 k = 0; k < (ST_SCALAR_OFF + 9 * sizeof(u64)) / sizeof(u64); k++) g.host_st[k] = src[k];
        }
    }
}

}  // namespace wcg
