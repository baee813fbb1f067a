// wcg_agg.h - aggregation of k_map's miss log, one hash bucket at a time, in two passes.
//
// k_map leaves, per (workgroup w, bucket p), a region of miss-log units (wcg_lds_table.h): keys that missed
// w's LDS table plus w's flushed LDS slots (with counts).  Every key of bucket p lands only in
// bucket-p regions, so a workgroup that aggregates bucket p over a slice of source regions
// needs LDS for (distinct keys of p) / 1 - about 1/P of the vocabulary - and flushes each
// distinct key once: the per-token global atomics of a naive design become per-(slice, key)
// atomics.
//
// Pass 1 (k_agg, mode AGG_SPILL): workgroup (p, s) aggregates bucket p over slice s; its LDS table
// is flushed to the global table.  An entry the full table cannot take is appended, whole, to
// the workgroup's spill region (an LDS cursor: no global atomic).  Low-cardinality text (C2) never
// spills.  High-cardinality text (C4: 22M distinct inline keys per GiB, 347K per bucket against
// 6,760 LDS slots) spills nearly everything, and per-occurrence global inserts of the spilled
// entries were 5.8 of a 19 ms step.
// k_rp: each pass-1 workgroup's spill is split by 7 bits of another hash into AGG_Q sub-buckets (LDS
// staging, whole entries), so a sub-bucket holds ~1/8192 of the keys.
// Pass 2 (k_agg, mode AGG_EMIT): one workgroup per (p, q) sub-bucket aggregates it in LDS and emits
// each distinct key as a record straight into the record log (no global-table insert); the
// sub-buckets are disjoint, and keys also counted in the global table (pass-1 flushes) or emitted
// by another map call are merged by the bucket sort (wcg_sort.h: dd_same).  An entry a full LDS
// table cannot take is logged as a partial-count record (merged the same way); only a full record
// log falls back to global-table inserts (exact either way).
#pragma once
#include "wcg_common.h"
#include "wcg_lds_table.h"
#include "wcg_map.h"

namespace wcg {

constexpr int AGG_NT = 1024;
constexpr u32 AGG_BATCH = AGG_NT * 4;     // units per batch (4 per thread)
constexpr int AGG_W = 2;               // ways per bucket (16-byte k0 rows: wcg_lds_table.h)
constexpr int AGG_NB = 3350;           // 3350 x 2 slots x 24 B (u64 counts) = 160800 B (+ 2.5 KiB)
constexpr u32 AGG_SLACK_UNITS = AGG_BATCH + 8;   // pool tail slack for k_agg's unmasked loads
constexpr u32 AGG_MAX_SRC = 256;       // source regions per workgroup (+1 KiB LDS = 160 KiB)
constexpr u32 AGG_Q = 128;             // pass-2 sub-buckets per bucket
constexpr u32 AGG_OVF_CAP = 4096;      // pass 2: overflow records staged per workgroup (128 KiB)
constexpr int AGG_SPILL = 0, AGG_EMIT = 1;
#ifndef WCG_AGG_PROBES
#define WCG_AGG_PROBES 2       // lookups per lane whose LDS reads are in flight together (2; 4 measured no faster: r03_kagg_experiments)
#endif
constexpr int AGG_PROBES = WCG_AGG_PROBES;
#ifndef WCG_AGG_SPEC_K1
#define WCG_AGG_SPEC_K1 0      // 1: medium keys read their k1 rows with the k0 rows (measured slower on C2 and C4)
#endif
constexpr bool AGG_SPEC_K1 = WCG_AGG_SPEC_K1;
#ifndef WCG_AGG_SPEC_MED
#define WCG_AGG_SPEC_MED 1     // medium-only buckets (r06): k1 rows read with the k0 rows
#endif
#ifndef WCG_AGG_KINDS
#define WCG_AGG_KINDS 1        // 0: split buckets aggregated by the any-key code (measurement)
#endif
#ifndef WCG_AGG_ABLATE
#define WCG_AGG_ABLATE 0       // diagnostics: 1 = loads only, 2 = + decode and hash, 3 = no flush, 4 = short keys only (wrong counts)
#endif

struct AggArgs {
    // sources: bucket b's regions are pool + ((wbase + k * wstep) * rstride + b % rmod) * region_cap
    // for k in [k0, k1) (pass 1: every map workgroup in a slice; pass 2: the pass-1 workgroups of
    // the sub-bucket's bucket), region_len indexed like the regions
    const u64* pool;
    const u32* region_len;
    u64 region_cap;
    u32 P;                 // pass 1: miss buckets; pass 2: buckets x AGG_Q sub-buckets
    u32 nsrc;              // pass 1: source workgroups of k_map; pass 2: pass-1 slices
    u32 slices;            // workgroups per bucket (pass 2: 1)
    u32 pm;                // pass 1 (r06): buckets [pm, P) hold medium keys only and take slices_m
    u32 slices_m;          //   workgroups each (pm = P: no such buckets)
    u32 nbi;               // (bucket, slice) items: pm * slices + (P - pm) * slices_m
    u32 ls_nreg;           // pass 1 (r06): workgroup nbi (the grid's last) runs long_small over
                           //   ls_nreg map regions (wcg_map.h; 0: no such workgroup)
    u32 rstride, rmod;     // region index = w * rstride + b % rmod
    u32 P1;                // pass 2: pass-1 buckets (source w of sub-bucket b: b / AGG_Q + P1 * s)
    int mode;              // AGG_SPILL (pass 1) or AGG_EMIT (pass 2)
    GEntry* gtab;
    u64 gmask;
    DevState* st;
    const u64* map_stats;  // k_map's per-workgroup stats [nsrc][4], summed by workgroup 0 (pass 1)
    u64* spill;            // pass 1: spill region of workgroup b = spill + b * spill_cap
    u64 spill_cap;
    u32* spill_len;
    Rec* emit;             // pass 2: record log (emit_cap records; st->nemit used)
    u64 emit_cap;
    Rec* ovf;              // pass 2: per-workgroup staging of the entries a full LDS table
    u32 ovf_cap;           //   cannot take (ovf_cap records per workgroup)
    u64* clk;              // diagnostics (WCG_AGG_CLOCK): per workgroup start / end wall clock, or null
    uint16_t* flist;       // one-pass flush (r05): the occupied slots of workgroup bi's table at
                           // flist + bi * AGG_NB * AGG_W (null: the slot-by-slot flush)
};

// bucket choices of pass 2's tables: the high half of the 64-bit key hash (a sub-bucket's keys
// share 13 bits of the 32-bit LDS hash, which pass 1 uses: it is cheaper and its keys vary in all
// bits)
#ifndef WCG_AGG2_LDSHASH
#define WCG_AGG2_LDSHASH 0
#endif
__device__ __forceinline__ u32 agg_hash(u64 k0, u64 k1) {
    if (WCG_AGG2_LDSHASH) return lds_hash(k0, k1) * 0x9E3779B1u;   // measurement variant (cheaper)
    return (u32)(key_hash(k0, k1) >> 32);
}

// decode the entries headed by 4 of a lane's units (u[0..6): its 4 units and the 2 after them;
// units past the region are 0 = filler)
__device__ __forceinline__ void agg_decode(const u64 (&u)[6], u64 (&k0)[4], u64 (&k1)[4], u64 (&c)[4], bool (&v)[4],
                                           u32 (&nu)[4]) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const u32 T = (u32)(u[k] >> 56);
        const bool head = T >= 0x41;
        v[k] = T != 0 && (head || (T & 0x1F) < 8);   // skip counts, fillers, medium tails
        const u64 last = head ? u[k + 1] : u[k];     // unit carrying the count flag
        k0[k] = head ? u[k] : (u[k] & ~U_CNT);
        k1[k] = head ? (u[k + 1] & ~U_CNT) : 0;
        const bool hc = (last & U_CNT) != 0;
        c[k] = hc ? (head ? u[k + 2] : u[k + 1]) : 1;
        nu[k] = (head ? 2u : 1u) + (hc ? 1u : 0u);
    }
}

// the same for buckets of one kind (r06, one-pass jobs: k_map logs short and medium keys to
// separate buckets).  Short buckets hold short keys (T = length 1..7, U_CNT perhaps set) and count
// units (T = 0); medium buckets hold heads (T >= 0x41), tails and count units (both skipped).
__device__ __forceinline__ void agg_decode_short(const u64 (&u)[6], u64 (&k0)[4], u64 (&k1)[4], u64 (&c)[4], bool (&v)[4],
                                                 u32 (&nu)[4]) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
        v[k] = (u[k] >> 56) != 0;
        const bool hc = (u[k] & U_CNT) != 0;
        k0[k] = u[k] & ~U_CNT;
        k1[k] = 0;
        c[k] = hc ? u[k + 1] : 1;
        nu[k] = hc ? 2u : 1u;
    }
}
__device__ __forceinline__ void agg_decode_medium(const u64 (&u)[6], u64 (&k0)[4], u64 (&k1)[4], u64 (&c)[4], bool (&v)[4],
                                                  u32 (&nu)[4]) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
        v[k] = (u32)(u[k] >> 56) >= 0x41;
        const bool hc = (u[k + 1] & U_CNT) != 0;
        k0[k] = u[k];
        k1[k] = u[k + 1] & ~U_CNT;
        c[k] = hc ? u[k + 2] : 1;
        nu[k] = hc ? 3u : 2u;
    }
}

// k_agg's prefetch register sets: three tagged 16-byte loads per set and a wait naming the set's
// registers (tools/check_inflight.py; the k_map sets use the same tags with one load each)
#define WCG_AGG_SET_OPS(S)                                                                      \
    __device__ __forceinline__ void agg_load_##S(const v4u* q, v4u& x0, v4u& x1, v4u& x2) {     \
        asm volatile("global_load_dwordx4 %0, %3, off ; wcg-load " #S "0\n\t"                   \
                     "global_load_dwordx4 %1, %3, off offset:16 ; wcg-load " #S "1\n\t"         \
                     "global_load_dwordx4 %2, %3, off offset:32 ; wcg-load " #S "2"              \
                     : "=&v"(x0), "=&v"(x1), "=&v"(x2) : "v"(q) : "memory");                    \
    }                                                                                           \
    template <int N>                                                                            \
    __device__ __forceinline__ void agg_wait_##S(v4u& x0, v4u& x1, v4u& x2) {                   \
        asm volatile("s_waitcnt vmcnt(%3) ; wcg-wait " #S " %0 %1 %2"                            \
                     : "+v"(x0), "+v"(x1), "+v"(x2) : "n"(N) : "memory");                       \
    }
WCG_AGG_SET_OPS(A)
WCG_AGG_SET_OPS(B)
WCG_AGG_SET_OPS(C)
#undef WCG_AGG_SET_OPS
// register sets (batches in flight per wave).  r04 measured a third (C2's pass 1 spends 54% of
// its wave cycles waiting with two): pass 1 0.284-0.292 ms with three against 0.288-0.293 with
// two, pass 2 1.29-1.33 ms either way (profiles/r04_kagg_three_sets.txt): two kept
#ifndef WCG_AGG_SETS1
#define WCG_AGG_SETS1 2
#endif
#ifndef WCG_AGG_SETS2
#define WCG_AGG_SETS2 2
#endif

// One (bucket, slice) of k_agg: index bi = p + P * s.  Returns the global-table inserts made.
// MODE is a template parameter: one kernel for both passes held the union of their registers
// (128 VGPRs with a spill)
// KIND (r06): 0 = any keys; 1 / 2 = a short / medium bucket of a split one-pass log
template <int MODE, int KIND>
__device__ __forceinline__ u64 agg_one(const AggArgs& a, u32 bi, u64 (*tk0)[AGG_W], u64 (*tk1)[AGG_W], u64 (*tcnt)[AGG_W], u32* rlen_s,
                       u32* bstart, u32& spos, u64 (*wsum)[4]) {
    const int tid = threadIdx.x;
    // (a first-fit variant that reads b2's row only when b1 is full - half the LDS bytes - measured
    // slower on C2, 0.333 vs 0.310 ms: a wave waits for the second round trip whenever any of its
    // lanes needs it)
    LdsTable<AGG_NB, u64, AGG_W> tab{tk0, tk1, tcnt};
    constexpr bool emit = MODE == AGG_EMIT;
    // item bi -> (bucket p, slice s of sl): the short-key buckets [0, pm) first, slices major,
    // then the medium-key buckets [pm, P)
    u32 p, s, sl;
    if (bi < a.pm * a.slices) { p = bi % a.pm; s = bi / a.pm; sl = a.slices; }
    else { const u32 b2 = bi - a.pm * a.slices, nm = a.P - a.pm; p = a.pm + b2 % nm; s = b2 / nm; sl = a.slices_m; }
#ifdef WCG_AGG_MREV
    if (p >= a.pm && a.pm < a.P) p = a.P - 1 - (p - a.pm);    // measurement: medium buckets reversed
#endif
    u32 k0_, k1_, wbase, wstep;
    if (!emit) {
        k0_ = (u32)(((u64)a.nsrc * s) / sl); k1_ = (u32)(((u64)a.nsrc * (s + 1)) / sl);
        wbase = 0; wstep = 1;
    } else {
        k0_ = 0; k1_ = a.nsrc;
        wbase = p / AGG_Q; wstep = a.P1;
    }
    const u32 nk = k1_ - k0_;
    auto region = [&](u32 k) -> u64 { return (u64)(wbase + k * wstep) * a.rstride + p % a.rmod; };
    constexpr u32 WB = 256;                          // units per wave batch
    // region lengths and the running count of batches before each region, staged once: a global
    // load in the batch walk would be a vmcnt wait that drains the prefetch
    for (u32 k = tid; k < nk; k += AGG_NT) rlen_s[k] = a.region_len[region(k0_ + k)];
    __syncthreads();
    if (tid == 0) {
        u32 t = 0;
        for (u32 k = 0; k < nk; k++) { bstart[k] = t; t += (rlen_s[k] + WB - 1) / WB; }
        bstart[nk] = t;
        spos = 0;
    }
    __syncthreads();
    const u32 nbat = bstart[nk];
    if (nbat == 0) {                                  // nothing to read (pass 2 on low-cardinality
        if (!emit && tid == 0 && a.spill_len) a.spill_len[bi] = 0;   // text: every sub-bucket empty): done before
        return 0;                                     // the table's 162 KiB are initialised
    }
    tab.init(tid, AGG_NT);
    __syncthreads();
    u64 my_global = 0;
    u64* const sp = emit ? nullptr : a.spill + (u64)bi * a.spill_cap;
    // count c of (k0, k1) the table could not take: pass 1 spills the entry; pass 2 stages it as a
    // partial-count record (appended to the record log with the table's records, the duplicates
    // merged after the sort as for keys emitted by several map calls), so that the global table
    // stays empty and compaction skips its scan; a full spill region or staging area inserts it
    // into the global table
    auto overflow = [&](u64 k0, u64 k1, u64 c, u32 nu) {
        if (emit) {
            const u32 pos = atomicAdd(&spos, 1u);
            if (pos < a.ovf_cap) { a.ovf[(u64)blockIdx.x * a.ovf_cap + pos] = inline_rec(k0, k1, c); return; }
        } else {
            const u32 pos = atomicAdd(&spos, nu);
            if (pos + nu <= a.spill_cap) {
                u64 e[3];
                const u64 f = c > 1 ? U_CNT : 0;
                if (key_short(k0)) { e[0] = k0 | f; e[1] = c; }
                else { e[0] = k0; e[1] = k1 | f; e[2] = c; }
                for (u32 j = 0; j < nu; j++) sp[pos + j] = e[j];
                return;
            }
            for (u64 j = pos; j < a.spill_cap; j++) sp[j] = 0;   // reserved, inside: fillers
        }
        my_global++;
        ginsert(a.gtab, a.gmask, k0, k1, gslot(key_hash(k0, k1)), c, a.st);
    };
    // The workgroup's wave batches (256 units) are dealt round-robin over its 16 waves: lane l
    // takes units [4l, 4l + 4) and also loads the two after them, so a medium-key head or a count
    // flag finds its neighbours in registers (units past the region's length are masked to 0 =
    // filler).  The next batch is loaded into the other register set while this one is
    // aggregated, and no barrier ties the waves together, so 16 waves x 2 batches are in flight
    // per CU (a workgroup-wide batch walk kept only 2, and ran at the HBM latency of one batch
    // per region even for nearly empty regions; a region per wave left most waves idle when a
    // workgroup has few regions, as in pass 2).
    // the wave index as a scalar: the batch walk below is then uniform control flow (a per-lane
    // `wave` made the compiler run it as a divergent loop, with its region state spilled)
    const u32 wave = (u32)__builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    constexpr u32 WSTRIDE = AGG_NT / 64;
    // (region k, batch b) of a wave's batch g, advanced incrementally: g grows by WSTRIDE per
    // step, which crosses at most a few region ends
    // Pass 1 (64 regions per workgroup) walks a region per wave instead (k, k + 16, ...): measured
    // 10% faster there than the round-robin deal, which pass 2 (4 regions) needs.
    const bool per_wave = !emit;
    auto advance = [&](u32& k, u32& b, u32 step) {
        if (per_wave) {
            b += step / WSTRIDE;                      // one batch of the wave's own region
            while (k < nk && b >= bstart[k + 1] - bstart[k]) { k += WSTRIDE; b = 0; }
            return;
        }
        b += step;
        while (k < nk) {
            const u32 nbk = bstart[k + 1] - bstart[k];
            if (b < nbk) break;
            b -= nbk;
            k++;
        }
    };
    // a batch's units: lane l reads [4l, 4l + 6) of the batch (a dead batch, k >= nk, reads the
    // first batch of the first region: the loads are unconditional, see below)
    auto batch_ptr = [&](u32 k, u32 b) -> const v4u* {
        const bool live = k < nk;
        const u64 i = (live ? (u64)b * WB : 0) + 4 * lane;
        return reinterpret_cast<const v4u*>(a.pool + region(k0_ + (live ? k : 0)) * a.region_cap + i);
    };
    auto unit = [](const v4u& x, int h) -> u64 { return h ? ((u64)x.w << 32 | x.z) : ((u64)x.y << 32 | x.x); };
    auto process = [&](u32 k, u32 b, const v4u& x0, const v4u& x1, const v4u& x2) {
        u64 u[6] = {unit(x0, 0), unit(x0, 1), unit(x1, 0), unit(x1, 1), unit(x2, 0), unit(x2, 1)};
        const u32 i0 = b * WB + 4 * lane, len = rlen_s[k];
#pragma unroll
        for (int j = 0; j < 6; j++) u[j] = i0 + j < len ? u[j] : 0;
        if (WCG_AGG_ABLATE == 1) { asm volatile("" ::"v"(u[0] ^ u[1] ^ u[2] ^ u[3] ^ u[4] ^ u[5])); return; }
        u64 k0[4], k1[4], c[4];
        bool v[4];
        u32 nu[4];
        if (KIND == 1) agg_decode_short(u, k0, k1, c, v, nu);
        else if (KIND == 2) agg_decode_medium(u, k0, k1, c, v, nu);
        else agg_decode(u, k0, k1, c, v, nu);
        if (WCG_AGG_ABLATE == 4) {            // diagnostics: short keys only (medium entries dropped)
#pragma unroll
            for (int j = 0; j < 4; j++) v[j] = v[j] && key_short(k0[j]);
        }
        if (WCG_AGG_ABLATE == 2) {
            u32 x = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) x ^= v[j] ? lds_hash(k0[j], k1[j]) + (u32)c[j] : 0u;
            asm volatile("" ::"v"(x));
            return;
        }
        // the AGG_PROBES lookups' row reads issue together (one LDS round trip for them; a
        // lookup that inserts a key another of the lane's lookups also inserts may leave the key
        // in two slots: harmless, as between lanes)
        static_assert(4 % AGG_PROBES == 0, "probe groups split a lane's 4 units");
        // a medium bucket reads its k1 rows with the k0 rows (every key needs them: no dependent
        // read); mixed buckets do not (measured slower there: short keys paid the extra reads)
        constexpr bool SPEC = KIND == 2 ? WCG_AGG_SPEC_MED : AGG_SPEC_K1;
#pragma unroll
        for (int j = 0; j < 4; j += AGG_PROBES) {
            typename decltype(tab)::Probe pr[AGG_PROBES];
#pragma unroll
            for (int q = 0; q < AGG_PROBES; q++) {
                const u32 h = emit ? agg_hash(k0[j + q], k1[j + q]) : lds_hash(k0[j + q], k1[j + q]);
                if (!v[j + q]) continue;
                if (SPEC) tab.start_k1(h, KIND == 2 || !key_short(k0[j + q]), pr[q]);
                else tab.start(h, pr[q]);
            }
#pragma unroll
            for (int q = 0; q < AGG_PROBES; q++) {
                if (!v[j + q]) continue;
                const bool ok = SPEC ? tab.template finish_k1<KIND>(k0[j + q], k1[j + q], pr[q], c[j + q])
                                     : tab.template finish<KIND>(k0[j + q], k1[j + q], pr[q], c[j + q]);
                if (!ok) overflow(k0[j + q], k1[j + q], c[j + q], nu[j + q]);
            }
        }
    };
    // Two batches in flight per wave, in register sets A and B that hold the wave's batches g and
    // g + 1: the loads are tagged asm and each set's wait counts only the other set's three loads
    // issued after it (tools/check_inflight.py checks that no copy of an in-flight register sits
    // between a load and its wait).  The compiler's own wait placement drained both sets at the
    // top of every batch (s_waitcnt vmcnt(0)), exposing one HBM latency per batch.  Loads are
    // unconditional (a dead batch reads the first region's first batch), so the count never
    // depends on which batches are live.  An overflow insert waits for all loads itself (harmless).
    constexpr int NSETS = emit ? WCG_AGG_SETS2 : WCG_AGG_SETS1;
    static_assert(NSETS == 2 || NSETS == 3, "k_agg's batch walk names two or three register sets");
    u32 kA = 0, bA = 0, kB, bB, kC = 0, bC = 0;
    if (per_wave) { kA = wave; bA = (u32)-1; advance(kA, bA, WSTRIDE); }
    else advance(kA, bA, wave);
    kB = kA; bB = bA;
    advance(kB, bB, WSTRIDE);
    v4u a0, a1, a2, b0, b1, b2, c0, c1, c2;
    agg_load_A(batch_ptr(kA, bA), a0, a1, a2);
    agg_load_B(batch_ptr(kB, bB), b0, b1, b2);
    if (NSETS == 3) {
        // batch g in A, g + 1 in B, g + 2 in C; each wait leaves the other two sets' six loads in flight
        kC = kB; bC = bB;
        advance(kC, bC, WSTRIDE);
        agg_load_C(batch_ptr(kC, bC), c0, c1, c2);
        while (kA < nk) {
            agg_wait_A<6>(a0, a1, a2);
            process(kA, bA, a0, a1, a2);
            kA = kC; bA = bC;
            advance(kA, bA, WSTRIDE);
            agg_load_A(batch_ptr(kA, bA), a0, a1, a2);
            if (kB >= nk) break;
            agg_wait_B<6>(b0, b1, b2);
            process(kB, bB, b0, b1, b2);
            kB = kA; bB = bA;
            advance(kB, bB, WSTRIDE);
            agg_load_B(batch_ptr(kB, bB), b0, b1, b2);
            if (kC >= nk) break;
            agg_wait_C<6>(c0, c1, c2);
            process(kC, bC, c0, c1, c2);
            kC = kB; bC = bB;
            advance(kC, bC, WSTRIDE);
            agg_load_C(batch_ptr(kC, bC), c0, c1, c2);
        }
        agg_wait_C<0>(c0, c1, c2);                    // nothing may land in a dead register
    } else {
        while (kA < nk) {
            agg_wait_A<3>(a0, a1, a2);
            process(kA, bA, a0, a1, a2);
            kA = kB; bA = bB;
            advance(kA, bA, WSTRIDE);
            agg_load_A(batch_ptr(kA, bA), a0, a1, a2);
            if (kB >= nk) break;
            agg_wait_B<3>(b0, b1, b2);
            process(kB, bB, b0, b1, b2);
            kB = kA; bB = bA;
            advance(kB, bB, WSTRIDE);
            agg_load_B(batch_ptr(kB, bB), b0, b1, b2);
        }
    }
    agg_wait_A<0>(a0, a1, a2);                        // nothing may land in a dead register
    agg_wait_B<0>(b0, b1, b2);
    __syncthreads();
    if (!emit && a.flist && !a.spill_cap && WCG_AGG_ABLATE != 3) {
        // ---- one-pass flush (r05): the occupied slots listed first, then the inserts dealt
        // evenly.  The slot-by-slot loop ran 6.5 iterations per thread, and in nearly every wave
        // some lane of each iteration held a key (23% of the slots), so a workgroup paid 6.5
        // dependent insert chains (~38 us of its ~244: WCG_AGG_ABLATE=3); listed, ~1.5 keys per
        // thread are 2 chains.  (The list goes through global memory: the LDS is the table.)
        constexpr u32 NE = AGG_NB * AGG_W;
        uint16_t* const L = a.flist + (u64)bi * NE;
        u32 mine = 0;
        for (int i = tid; i < (int)NE; i += AGG_NT) mine += (&tcnt[0][0])[i] ? 1u : 0u;
        u32 incl = mine;
        for (int d = 1; d < 64; d <<= 1) { const u32 y = __shfl_up(incl, d, 64); if (lane >= (u32)d) incl += y; }
        if (lane == 63) wsum[wave][0] = incl;
        __syncthreads();
        u32 pos = 0, all = 0;
        for (u32 w = 0; w < AGG_NT / 64; w++) { if (w < wave) pos += (u32)wsum[w][0]; all += (u32)wsum[w][0]; }
        pos += incl - mine;
        for (int i = tid; i < (int)NE; i += AGG_NT)
            if ((&tcnt[0][0])[i]) L[pos++] = (uint16_t)i;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (u32 j = tid; j < all; j += AGG_NT) {
            // (an L1-bypassing read: other waves of this workgroup wrote the list)
            const u32 i = __hip_atomic_load(&L[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const u64 c = (&tcnt[0][0])[i], k0 = (&tk0[0][0])[i], k1 = (&tk1[0][0])[i];
            my_global++;
            ginsert(a.gtab, a.gmask, k0, k1, gslot(key_hash(k0, k1)), c, a.st);
        }
        __syncthreads();
    } else if (!emit) {
        // one-pass mode: the table goes to the global table (one insert per slice and key);
        // two-pass mode: it is spilled too, so every inline key of the bucket reaches exactly one
        // pass-2 sub-bucket and is emitted once per map call (no duplicate with the global table)
        for (int i = tid; i < AGG_NB * AGG_W; i += AGG_NT) {
            const u64 c = (&tcnt[0][0])[i];
            if (!c || WCG_AGG_ABLATE == 3) continue;     // 3: no flush (diagnostics: wrong counts)
            const u64 k0 = (&tk0[0][0])[i], k1 = (&tk1[0][0])[i];
            if (a.spill_cap) { overflow(k0, k1, c, (u32)entry_units(k0, (u32)(c > 1 ? 2 : 1))); continue; }
            my_global++;
            ginsert(a.gtab, a.gmask, k0, k1, gslot(key_hash(k0, k1)), c, a.st);
        }
        __syncthreads();
        if (tid == 0 && a.spill_len) a.spill_len[bi] = spos < a.spill_cap ? spos : (u32)a.spill_cap;
    } else {
        // pass 2: this sub-bucket's keys, one record each, placed by one atomic per workgroup;
        // positions past the log's end go to the global table instead (the log stays dense:
        // k_copy_emit takes min(nemit, cap) records)
        u32 mine = 0;
        for (int i = tid; i < AGG_NB * AGG_W; i += AGG_NT) mine += (&tcnt[0][0])[i] ? 1u : 0u;
        u32 incl = mine;
        for (int d = 1; d < 64; d <<= 1) { const u32 y = __shfl_up(incl, d, 64); if (lane >= d) incl += y; }
        if (lane == 63) wsum[wave][0] = incl;
        __syncthreads();
        u32 pre = 0, all = 0;
        for (int w = 0; w < AGG_NT / 64; w++) { if (w < wave) pre += (u32)wsum[w][0]; all += (u32)wsum[w][0]; }
        const u32 nov = spos < a.ovf_cap ? spos : a.ovf_cap;       // staged overflow records
        if (tid == 0)
            wsum[0][1] = all + nov ? atomicAdd((unsigned long long*)&a.st->nemit, (unsigned long long)(all + nov)) : 0;
        __syncthreads();
        const u64 base = wsum[0][1];
        for (u32 i = tid; i < nov; i += AGG_NT) {                    // after the table's records
            const Rec r = a.ovf[(u64)blockIdx.x * a.ovf_cap + i];
            if (base + all + i < a.emit_cap) a.emit[base + all + i] = r;
            else {
                my_global++;
                u64 k0, k1;
                rec_inline_key(r, k0, k1);
                ginsert(a.gtab, a.gmask, k0, k1, gslot(key_hash(k0, k1)), r.cnt, a.st);
            }
        }
        u64 pos = base + pre + incl - mine;
        for (int i = tid; i < AGG_NB * AGG_W; i += AGG_NT) {
            const u64 c = (&tcnt[0][0])[i];
            if (!c) continue;
            const u64 k0 = (&tk0[0][0])[i], k1 = (&tk1[0][0])[i];
            if (pos < a.emit_cap) a.emit[pos] = inline_rec(k0, k1, c);
            else { my_global++; ginsert(a.gtab, a.gmask, k0, k1, gslot(key_hash(k0, k1)), c, a.st); }
            pos++;
        }
    }
    __syncthreads();                                  // the LDS is reused by the next bucket
    return my_global;
}

// pass 1: one workgroup per (bucket, slice); pass 2: a persistent grid over the sub-buckets (most
// are empty on low-cardinality text, and an empty one costs a few LDS reads instead of a launch
// of a 160 KiB workgroup)
struct AggTabs {
    u64 tk0[AGG_NB][AGG_W];
    u64 tk1[AGG_NB][AGG_W];
    u64 tcnt[AGG_NB][AGG_W];
};
union AggLds {
    AggTabs t;
    LsLds ls;
};
static_assert(LS_NT == AGG_NT, "long_small runs as a k_agg workgroup");
template <int MODE>
__global__ __launch_bounds__(AGG_NT) void k_agg(AggArgs a, MapArgs ma) {
    __shared__ __align__(16) AggLds lds;
    u64 (*const tk0)[AGG_W] = lds.t.tk0;
    u64 (*const tk1)[AGG_W] = lds.t.tk1;
    u64 (*const tcnt)[AGG_W] = lds.t.tcnt;
    __shared__ u32 rlen_s[AGG_MAX_SRC];
    __shared__ u32 bstart[AGG_MAX_SRC + 1];
    __shared__ u32 spos;                       // pass 1: spill cursor
    __shared__ u64 wsum[AGG_NT / 64][4];       // per-wave sums (the record log's counts, stats)
    const int tid = threadIdx.x;
    const u32 nb = a.nbi;
    if (MODE == AGG_SPILL && a.ls_nreg && blockIdx.x == nb) {
        long_small(ma, a.ls_nreg, lds.ls);
        return;
    }
    const u64 t0 = a.clk ? wall_clock64() : 0;
    // one-pass map calls: compaction's counters start at zero (its memset dispatch cost ~4 us)
    if (MODE == AGG_SPILL && blockIdx.x == 0 && tid == 0) { a.st->nrec = 0; a.st->nlong = 0; }
    u64 my_global = 0;
    for (u32 bi = blockIdx.x; bi < nb; bi += gridDim.x)
        if (MODE == AGG_SPILL && WCG_AGG_KINDS && a.pm < a.P)    // split buckets: one kind each
            my_global += bi < a.pm * a.slices ? agg_one<MODE, 1>(a, bi, tk0, tk1, tcnt, rlen_s, bstart, spos, wsum)
                                              : agg_one<MODE, 2>(a, bi, tk0, tk1, tcnt, rlen_s, bstart, spos, wsum);
        else
            my_global += agg_one<MODE, 0>(a, bi, tk0, tk1, tcnt, rlen_s, bstart, spos, wsum);
    // one atomic per workgroup (a per-wave atomic on one DevState line serialises)
    for (int d = 32; d >= 1; d >>= 1) my_global += __shfl_xor(my_global, d, 64);
    u64 ms = 0;
    if (blockIdx.x == 0 && MODE != AGG_EMIT)    // k_map's stats: tokens, lds hits, global ops, long
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
    if (a.clk && tid == 0) { a.clk[2 * blockIdx.x] = t0; a.clk[2 * blockIdx.x + 1] = wall_clock64(); }
}

// k_rp (two-pass jobs): workgroup b = (bucket p, slice s) reads the miss-log regions of bucket p
// written by the map workgroups of slice s and splits their entries into its AGG_Q sub-bucket
// regions (b, q) of pool2, q = 7 bits of the key's 64-bit hash (the 32-bit LDS hash's low bits,
// a single multiply away from the key bytes, left C4's UTF-8 keys unevenly spread: sub-buckets
// overflowed their LDS tables).  (Until r02 a pass-1 k_agg aggregated each bucket slice in LDS
// first and k_rp split its spill: on C4 that pass cut 126M units to 90M for 1.5 ms, more than
// the 0.6 ms the smaller input saved k_rp and pass 2.)
// Rounds of AGG_BATCH units: every lane appends its entries, whole, to its sub-bucket's LDS buffer
// (or, when that buffer is full, straight to the region); then the buffers are written out
// together.  The regions belong to this workgroup alone, so their cursors live in LDS too.  A full
// region falls back to global-table inserts (exact).  Workgroup 0 also adds k_map's per-workgroup
// stats to DevState (pass 1 does that in one-pass jobs).
#ifndef WCG_RP_QB
#define WCG_RP_QB 48
#endif
#ifndef WCG_RP_PREFETCH
#define WCG_RP_PREFETCH 0
#endif
constexpr u32 RP_QB = WCG_RP_QB;       // LDS units per sub-bucket buffer (48 KiB in all: two k_rp
                                       // workgroups per CU; 96 measured 6% slower on C4)
struct RpArgs {
    const u64* pool; const u32* region_len; u64 region_cap;   // the miss log (k_map)
    u32 P, nsrc, slices;                                       // buckets, map workgroups, slices
    const u64* map_stats;
    u64* pool2; u64 cap2; u32* region_len2;                    // sub-bucket regions (pass 2's input)
    GEntry* gtab; u64 gmask; DevState* st;
};
#ifndef WCG_RP_MINB
#define WCG_RP_MINB 1
#endif
__global__ __launch_bounds__(AGG_NT, WCG_RP_MINB) void k_rp(RpArgs a) {
    __shared__ u64 sbuf[AGG_Q][RP_QB];
    __shared__ u32 scnt[AGG_Q], sfill[AGG_Q], gpos[AGG_Q], gbase[AGG_Q];
    __shared__ u32 sdirect[AGG_Q];            // 1: this round's buffer goes out entry by entry
    __shared__ u64 wsum[AGG_NT / 64][4];
    const u32 b = blockIdx.x, tid = threadIdx.x;
    const u32 p = b % a.P, sl = b / a.P;
    const u32 k0_ = (u32)(((u64)a.nsrc * sl) / a.slices), k1_ = (u32)(((u64)a.nsrc * (sl + 1)) / a.slices);
    u64* const pool2 = a.pool2;
    const u64 cap2 = a.cap2;
    GEntry* const gtab = a.gtab;
    const u64 gmask = a.gmask;
    DevState* const st = a.st;
    if (b == 0) {                              // k_map's stats: tokens, lds hits, global ops, long
        u64 ms = 0;
        for (u32 w = tid >> 2; w < a.nsrc; w += AGG_NT / 4) ms += a.map_stats[(u64)w * 4 + (tid & 3)];
        for (int d = 32; d >= 4; d >>= 1) ms += __shfl_xor(ms, d, 64);
        if ((tid & 63) < 4) wsum[tid >> 6][tid & 3] = ms;
        __syncthreads();
        if (tid < 4) {
            u64 t = 0;
            for (int w = 0; w < AGG_NT / 64; w++) t += wsum[w][tid];
            u64* dst4[4] = {&st->tokens, &st->lds_hits, &st->global_ops, &st->long_tokens};
            if (t) atomicAdd(dst4[tid], t);
        }
    }
    for (u32 q = tid; q < AGG_Q; q += AGG_NT) { scnt[q] = 0; sfill[q] = 0; gpos[q] = 0; }
    __syncthreads();
    u64* const dst = pool2 + (u64)b * AGG_Q * cap2;
    u64 my_global = 0;
    auto encode = [](u64 k0, u64 k1, u64 c, u64 (&e)[3]) {
        const u64 f = c > 1 ? U_CNT : 0;
        if (key_short(k0)) { e[0] = k0 | f; e[1] = c; }
        else { e[0] = k0; e[1] = k1 | f; e[2] = c; }
    };
    // one whole entry into region q at a reserved place, or (past the region's end) into the
    // global table, zero-filling the reserved units that lie inside the region (fillers)
    auto to_region = [&](u32 q, u64 pos, const u64 (&e)[3], u32 nu, u64 k0, u64 k1, u64 c) {
        u64* r = dst + (u64)q * cap2;
        if (pos + nu <= cap2) { for (u32 t = 0; t < nu; t++) r[pos + t] = e[t]; return; }
        for (u64 t = pos; t < cap2; t++) r[t] = 0;
        my_global++;
        ginsert(gtab, gmask, k0, k1, gslot(key_hash(k0, k1)), c, st);
    };
#if WCG_RP_PREFETCH
    // batches in (region, offset) order; the next batch's units are loaded before this one is
    // split, so their latency overlaps the LDS work, the barriers and the stores
    u32 k = k0_, base = 0, n = k < k1_ ? a.region_len[(u64)k * a.P + p] : 0u;
    while (k < k1_ && n == 0) { k++; n = k < k1_ ? a.region_len[(u64)k * a.P + p] : 0u; }
    u64 nu[6];
    auto load6 = [&](u32 kk, u32 bb, u32 nn, u64 (&x)[6]) {
        const u64* s = a.pool + ((u64)kk * a.P + p) * a.region_cap;
        const u32 i = bb + 4 * tid;
#pragma unroll
        for (int j = 0; j < 6; j++) x[j] = kk < k1_ && i + j < nn ? s[i + j] : 0;
    };
    load6(k, 0, n, nu);
    while (k < k1_) {
        u64 u[6];
#pragma unroll
        for (int j = 0; j < 6; j++) u[j] = nu[j];
        u32 kn = k, bn = base + AGG_BATCH, nn = n;
        if (bn >= n) {
            bn = 0;
            do { kn++; nn = kn < k1_ ? a.region_len[(u64)kn * a.P + p] : 0u; } while (kn < k1_ && nn == 0);
        }
        load6(kn, bn, nn, nu);
        {
#else
    for (u32 k = k0_; k < k1_; k++) {
    const u64 reg = (u64)k * a.P + p;
    const u32 n = a.region_len[reg];
    const u64* src = a.pool + reg * a.region_cap;
    for (u32 base = 0; base < n; base += AGG_BATCH) {
        const u32 i0 = base + 4 * tid;
        u64 u[6];
#pragma unroll
        for (int j = 0; j < 6; j++) u[j] = i0 + j < n ? src[i0 + j] : 0;
#endif
        u64 k0[4], k1[4], c[4];
        bool v[4];
        u32 nu[4];
        agg_decode(u, k0, k1, c, v, nu);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (!v[j]) continue;
            const u32 q = (u32)(key_hash(k0[j], k1[j]) >> 40) & (AGG_Q - 1);
            u64 e[3];
            encode(k0[j], k1[j], c[j], e);
            const u32 pos = atomicAdd(&scnt[q], nu[j]);
            if (pos + nu[j] <= RP_QB) {        // the entries that fit are a prefix of the buffer
                for (u32 t = 0; t < nu[j]; t++) sbuf[q][pos + t] = e[t];
                atomicMax(&sfill[q], pos + nu[j]);
            } else {
                to_region(q, atomicAdd(&gpos[q], nu[j]), e, nu[j], k0[j], k1[j], c[j]);
            }
        }
        __syncthreads();
        for (u32 q = tid; q < AGG_Q; q += AGG_NT) {         // reserve each buffer's place
            gbase[q] = gpos[q];
            gpos[q] += sfill[q];
            sdirect[q] = (u64)gbase[q] + sfill[q] > cap2;
        }
        __syncthreads();
        for (u32 t = tid; t < AGG_Q * RP_QB; t += AGG_NT) {  // write the buffers out
            const u32 q = t / RP_QB, j = t % RP_QB;
            if (j < sfill[q] && !sdirect[q]) dst[(u64)q * cap2 + gbase[q] + j] = sbuf[q][j];
        }
        for (u32 q = tid; q < AGG_Q; q += AGG_NT) {         // a buffer running past its region
            if (!sdirect[q]) continue;                        // (rare): entry by entry
            u64 pos = gbase[q];
            for (u32 j = 0; j < sfill[q];) {
                u64 y[6] = {sbuf[q][j], j + 1 < sfill[q] ? sbuf[q][j + 1] : 0, j + 2 < sfill[q] ? sbuf[q][j + 2] : 0, 0, 0, 0};
                u64 kk0[4], kk1[4], cc[4];
                bool vv[4];
                u32 nn[4];
                agg_decode(y, kk0, kk1, cc, vv, nn);
                u64 e[3];
                encode(kk0[0], kk1[0], cc[0], e);
                to_region(q, pos, e, nn[0], kk0[0], kk1[0], cc[0]);
                pos += nn[0];
                j += nn[0];
            }
        }
        __syncthreads();
        for (u32 q = tid; q < AGG_Q; q += AGG_NT) { scnt[q] = 0; sfill[q] = 0; }
        __syncthreads();
    }
#if WCG_RP_PREFETCH
        k = kn; base = bn; n = nn;
#endif
    }
    for (u32 q = tid; q < AGG_Q; q += AGG_NT) a.region_len2[(u64)b * AGG_Q + q] = gpos[q] < cap2 ? gpos[q] : (u32)cap2;
    for (int d = 32; d >= 1; d >>= 1) my_global += __shfl_xor(my_global, d, 64);
    if ((tid & 63) == 0 && my_global) atomicAdd(&st->global_ops, my_global);
}

}  // namespace wcg
