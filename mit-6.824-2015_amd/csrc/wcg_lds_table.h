// wcg_lds_table.h - exact-key hash tables in LDS (one per workgroup).
//
// LdsTable (k_agg): 2-choice x W-way buckets.  Keys are the fixed-width identities of fact F4
// (k0 = bytes 0-7 [| len << 56 for len <= 7], k1 = bytes 8-14 | len << 56 or 0).  A key may
// live in 2W slots: W in bucket b1 and W in bucket b2.  A probe reads both buckets' k0 rows
// (independent ds_read_b128s), so a lookup costs ONE LDS round trip; the measured alternatives
// (tag bytes first, or bucket b1 before b2) add a dependent round trip and were slower.  Rows
// are W x 8 bytes: random 16-byte rows (W = 2) start on 16 distinct bank quads, 32-byte rows on
// only 8, and a 16-lane ds_read_b128 group of random rows conflicts less the more quads it can
// spread over (k_agg measured 74% of its LDS cycles in bank conflicts with W = 4).  The probe is
// split into start() (issue the reads) and finish() (match / insert) so a lane can keep two
// lookups in flight.  Insertion claims an empty slot with a 64-bit LDS CAS on k0 and then
// publishes k1.  Two lanes inserting the same new key at the same moment can end up in two
// different slots: that duplicate is harmless (both counts are flushed and summed downstream),
// so no lane ever waits for another lane's publish.
#pragma once
#include "wcg_common.h"
#ifndef WCG_DIAG_SLOTS
#define WCG_DIAG_SLOTS 0
#endif
#ifndef WCG_MAP_ROW2
#define WCG_MAP_ROW2 0                       // k_map short keys: one 2-slot row instead of two choices
#endif
#ifndef WCG_DIAG_NOCOUNT
#define WCG_DIAG_NOCOUNT 0                   // diagnostics: 1 = k_map's short-key hits not counted
#endif

namespace wcg {

template <int NB, typename CNT, int W>
struct LdsTable {
    static_assert(W == 2 || W == 4, "rows of one or two 16-byte reads");
    u64 (*k0)[W];      // [NB][W]  (W x 8-byte rows)
    u64 (*k1)[W];      // [NB][W]
    CNT (*cnt)[W];     // [NB][W]

    struct Probe {
        u32 b1, b2;
        u64 v[W], w[W];
        u64 v1[W], w1[W];     // start_k1: the k1 rows too (medium keys)
    };

    __device__ __forceinline__ void init(int tid, int nt) {
        for (int i = tid; i < NB * W; i += nt) {
            (&k0[0][0])[i] = 0;
            (&k1[0][0])[i] = 0;
            (&cnt[0][0])[i] = 0;
        }
    }

    // b1 from the high bits of h; b2 from all of h, mixed: the low bits select the miss bucket
    // (pass 1) and the sub-bucket (pass 2), so they are constant within a workgroup's keys
    __device__ __forceinline__ static void buckets(u32 h, u32& b1, u32& b2) {
        b1 = __umulhi(h, (u32)NB);
        u32 m = h * 0x85EBCA6Bu;
        m ^= m >> 15;
        b2 = __umulhi(m * 0xC2B2AE35u, (u32)NB);
        if (b2 == b1) b2 = (b1 + 1 == (u32)NB) ? 0 : b1 + 1;
    }

    __device__ __forceinline__ void readrow(u32 b, u64 (&v)[W]) const {
        const uint4* p = reinterpret_cast<const uint4*>(&k0[b][0]);
#pragma unroll
        for (int q = 0; q < W / 2; q++) {
            const uint4 x = p[q];
            v[2 * q] = (u64)x.y << 32 | x.x;
            v[2 * q + 1] = (u64)x.w << 32 | x.z;
        }
    }

    __device__ __forceinline__ void start(u32 h, Probe& p) const {
        buckets(h, p.b1, p.b2);
        readrow(p.b1, p.v);
        readrow(p.b2, p.w);
    }

    // the same, with both buckets' k1 rows read in the same round trip when the key has 8+ bytes
    // (finish_k1 then confirms a k0 match without a dependent read)
    __device__ __forceinline__ void start_k1(u32 h, bool med, Probe& p) const {
        buckets(h, p.b1, p.b2);
        readrow(p.b1, p.v);
        readrow(p.b2, p.w);
        if (med) {
            const uint4* q1 = reinterpret_cast<const uint4*>(&k1[p.b1][0]);
            const uint4* q2 = reinterpret_cast<const uint4*>(&k1[p.b2][0]);
#pragma unroll
            for (int q = 0; q < W / 2; q++) {
                const uint4 x = q1[q], y = q2[q];
                p.v1[2 * q] = (u64)x.y << 32 | x.x; p.v1[2 * q + 1] = (u64)x.w << 32 | x.z;
                p.w1[2 * q] = (u64)y.y << 32 | y.x; p.w1[2 * q + 1] = (u64)y.w << 32 | y.z;
            }
        } else {
#pragma unroll
            for (int j = 0; j < W; j++) { p.v1[j] = 0; p.w1[j] = 0; }
        }
    }

    __device__ __forceinline__ void add_cnt(u32 b, int j, CNT c) { atomicAdd(&cnt[b][j], c); }

    // finish() after start_k1: a match is decided from the rows already read (short keys have
    // k1 == 0 and compare with the zeros start_k1 put there); the insert path is finish()'s
    template <int KIND = 0>
    __device__ __forceinline__ bool finish_k1(u64 a0, u64 a1, const Probe& p, CNT c) {
        u32 m = 0;
#pragma unroll
        for (int j = 0; j < W; j++) {
            m |= (u32)(p.v[j] == a0 && p.v1[j] == a1) << j;
            m |= (u32)(p.w[j] == a0 && p.w1[j] == a1) << (W + j);
        }
        if (m) {
            const int s = __ffs(m) - 1;
            add_cnt(s < W ? p.b1 : p.b2, s % W, c);
            return true;
        }
        return finish<KIND>(a0, a1, p, c);
    }

    // match (slot s: bucket b1 for s < W, else b2; way s % W) or insert; false when both
    // buckets are full of other keys.  Straight-line common path: bit masks and one atomic at a
    // computed address.  KIND: 0 = any key, 1 = short keys only, 2 = medium keys only (k_agg's
    // split buckets, r06: the key-length tests fold away)
    template <int KIND = 0>
    __device__ __forceinline__ bool finish(u64 a0, u64 a1, const Probe& p, CNT c) {
        const bool shrt = KIND == 1 ? true : KIND == 2 ? false : key_short(a0);
        u32 m = 0, e = 0;
#pragma unroll
        for (int j = 0; j < W; j++) {
            m |= (u32)(p.v[j] == a0) << j;
            m |= (u32)(p.w[j] == a0) << (W + j);
            e |= (u32)(p.v[j] == 0) << j;
            e |= (u32)(p.w[j] == 0) << (W + j);
        }
        if (!shrt && m) {                       // keys of 8+ bytes: confirm k1 (usually 1 candidate)
            u32 mm = m;
            m = 0;
            while (mm) {
                const int s = __ffs(mm) - 1;
                mm &= mm - 1;
                if (k1[s < W ? p.b1 : p.b2][s % W] == a1) { m = 1u << s; break; }
            }
        }
        if (m) {
            const int s = __ffs(m) - 1;
            add_cnt(s < W ? p.b1 : p.b2, s % W, c);
            return true;
        }
        // insert into the emptier of the two buckets first (two choices by load keep the buckets
        // even; first-fit into b1 left enough full pairs at 40% load that 1.5% of pass-2 keys
        // found both of their buckets full)
        const u32 e1 = e & ((1u << W) - 1), e2 = e >> W;
        const bool second = __popc(e2) > __popc(e1);
        auto try_bucket = [&](u32 b, u32 m) -> bool {
            while (m) {
                const int j = __ffs(m) - 1;
                m &= m - 1;
                const u64 old = atomicCAS(&k0[b][j], 0ull, a0);
                if (old == 0) {
                    if (!shrt) k1[b][j] = a1;
                    add_cnt(b, j, c);
                    return true;
                }
                if (old == a0 && (shrt || k1[b][j] == a1)) { add_cnt(b, j, c); return true; }
            }
            return false;
        };
        if (second) return try_bucket(p.b2, e2) || try_bucket(p.b1, e1);
        return try_bucket(p.b1, e1) || try_bucket(p.b2, e2);
    }

    __device__ __forceinline__ bool add(u64 a0, u64 a1, u32 h, CNT c) {
        Probe p;
        start(h, p);
        return finish(a0, a1, p, c);
    }
};

// k_map's tables: short keys (<= 7 bytes: the k0 word is the whole key, 12 bytes per slot) and
// medium keys (8-15 bytes: k0 + k1, 20 bytes per slot), each 2 choices x 1 slot.  Measured on
// the C2 corpus (and a simulation of the same stream): associativity hardly moves the hit rate
// (2-choice x 1-way 0.678 vs 2-choice x 4-way 0.693 at equal slots) but capacity does, and
// short keys need 40% less room without a k1 word.  A probe is 2 slots x (k0, k1) loads and
// compares, the same instructions for both kinds (the table bases are selected per lane; the
// short keys' k1 is a shared zero word), so a wave never runs two probe paths.
template <int NS, int NM>
struct MapTable {
    u64* sk0;      // [NS]
    u32* scnt;     // [NS]
    u64* mk0;      // [NM]
    u64* mk1;      // [NM]
    u32* mcnt;     // [NM]
    u64* zero;     // one word, always 0
    u32* seen;     // admission filter (WCG_ADMIT2): ADMIT_BITS bits, or null

    __device__ __forceinline__ void init(int tid, int nt) {
        for (int i = tid; i < NS; i += nt) { sk0[i] = 0; scnt[i] = 0; }
        for (int i = tid; i < NM; i += nt) { mk0[i] = 0; mk1[i] = 0; mcnt[i] = 0; }
        if (seen) for (int i = tid; i < (int)(ADMIT_BITS / 32); i += nt) seen[i] = 0;
        if (tid == 0) *zero = 0;
    }
    // Admission on second sight: a key takes a free slot only if its filter bit was already set
    // (it missed once before); its first occurrence goes to the miss log like any miss.  The
    // table then fills with keys that recur, close to the most frequent ones, instead of with the
    // first distinct keys a workgroup meets (a rare key that shows up early holds its slot for
    // the whole launch).  Only the insert path, which runs while the table has free slots, pays.
    static constexpr u32 ADMIT_BITS = 16384;
    __device__ __forceinline__ bool admit(u32 h) {
        if (!seen) return true;
        const u32 b = (h * 0x9E3779B1u) >> 18;
        const u32 bit = 1u << (b & 31);
        return (atomicOr(&seen[b >> 5], bit) & bit) != 0;
    }
    // slot choices from 24-bit fields of h by the high half of full-rate 24-bit multiplies
    // (v_mul_hi_u32_u24: bits 8-31 and 0-23, each choice ruled by its field's top bits; bits 0-5
    // are the miss bucket, so a bucket's keys still spread over both choices).  r06: one
    // instruction per choice (two: the shift) against three (multiply, shift, field extract)
    __device__ __forceinline__ static void slots(u32 h, u32 n, u32& s1, u32& s2) {
#if WCG_DIAG_SLOTS                           // diagnostics only: conflict-free probes, wrong counts
        s1 = __lane_id(); s2 = __lane_id() + 64; (void)h; (void)n;
#else
        s1 = (u32)(((u64)(h >> 8) * (u64)(n << 8)) >> 32);
        s2 = (u32)(((u64)(h & 0xFFFFFFu) * (u64)(n << 8)) >> 32);
#endif
    }
    // A probe split in two so that k_map can issue its reads together with the next token's:
    // probe() computes the candidate slots and reads them, finish() counts one occurrence of
    // key (a0, a1) (a1 == 0 for short keys) when `valid` and returns true on a hit or insert,
    // false = both candidate slots hold other keys.  One divergent branch on the hit path (the
    // count add); the insert path (a probe saw an empty slot) is rare once the table has filled.
    struct Probe { u32 s1, s2; u64 x1, x2, y1, y2; };
    __device__ __forceinline__ Probe probe(bool med, u32 h) const {
        static_assert(NS < 65536 && NM < 65536, "n << 8 fits the 24-bit multiply");
        Probe p;
        slots(h, med ? (u32)NM : (u32)NS, p.s1, p.s2);
        const u64* K0 = med ? mk0 : sk0;
        p.x1 = K0[p.s1]; p.x2 = K0[p.s2];
        // a short key's k1 "slot" is a shared zero word (a broadcast read): no branch (the
        // exec-masked form, reads for medium lanes only, measured no faster)
        const u64* K1a = med ? mk1 + p.s1 : zero;
        const u64* K1b = med ? mk1 + p.s2 : zero;
        p.y1 = *K1a; p.y2 = *K1b;
        return p;
    }
    // short keys only (k_map's short-entry iterations: every lane holds a valid short key)
    struct ProbeS { u32 s1, s2; u64 x1, x2; };
    __device__ __forceinline__ ProbeS probe_short(u32 h) const {
        ProbeS p;
#if WCG_MAP_ROW2
        // one choice of a 16-byte row of two slots: one ds_read_b128, one slot multiply
        static_assert(NS % 2 == 0, "rows of two short slots");
        p.s1 = 2 * (u32)(((u64)(h >> 8) * (u64)((NS / 2) << 8)) >> 32);
        p.s2 = p.s1 + 1;
        const uint4 r = *reinterpret_cast<const uint4*>(sk0 + p.s1);
        p.x1 = (u64)r.y << 32 | r.x; p.x2 = (u64)r.w << 32 | r.z;
#else
        slots(h, (u32)NS, p.s1, p.s2);
        p.x1 = sk0[p.s1]; p.x2 = sk0[p.s2];
#endif
        return p;
    }
    __device__ __forceinline__ bool finish_short(u64 a0, u32 h, const ProbeS& p) {
        const bool h1 = p.x1 == a0, hit = h1 || p.x2 == a0;
        if (!WCG_DIAG_NOCOUNT) atomicAdd(&scnt[h1 ? p.s1 : p.s2], hit ? 1u : 0u);
        if (hit || (p.x1 != 0 && p.x2 != 0) || !admit(h)) return hit;
        if (p.x1 == 0) {
            const u64 old = atomicCAS(&sk0[p.s1], 0ull, a0);
            if (old == 0 || old == a0) { atomicAdd(&scnt[p.s1], 1u); return true; }
        }
        if (p.x2 == 0) {
            const u64 old = atomicCAS(&sk0[p.s2], 0ull, a0);
            if (old == 0 || old == a0) { atomicAdd(&scnt[p.s2], 1u); return true; }
        }
        return false;
    }

    // the same for a lane that may hold no token (valid false: no count, no insert)
    __device__ __forceinline__ bool finish_short_v(bool valid, u64 a0, u32 h, const ProbeS& p) {
        const bool h1 = p.x1 == a0, hit = valid && (h1 || p.x2 == a0);
        atomicAdd(&scnt[h1 ? p.s1 : p.s2], hit ? 1u : 0u);
        if (!valid || hit || (p.x1 != 0 && p.x2 != 0) || !admit(h)) return hit;
        if (p.x1 == 0) {
            const u64 old = atomicCAS(&sk0[p.s1], 0ull, a0);
            if (old == 0 || old == a0) { atomicAdd(&scnt[p.s1], 1u); return true; }
        }
        if (p.x2 == 0) {
            const u64 old = atomicCAS(&sk0[p.s2], 0ull, a0);
            if (old == 0 || old == a0) { atomicAdd(&scnt[p.s2], 1u); return true; }
        }
        return false;
    }

    __device__ __forceinline__ bool finish(bool valid, bool med, u64 a0, u64 a1, u32 h, const Probe& p) {
        u64* K0 = med ? mk0 : sk0;
        u32* C = med ? mcnt : scnt;
        const bool h1 = p.x1 == a0 && p.y1 == a1, h2 = p.x2 == a0 && p.y2 == a1;
        const bool hit = valid && (h1 || h2);
        atomicAdd(&C[h1 ? p.s1 : p.s2], hit ? 1u : 0u);     // every lane (0 = no hit): no branch
        if (!valid || hit || (p.x1 != 0 && p.x2 != 0) || !admit(h)) return hit;
        // insert: claim an empty slot's k0, then publish k1 (a reader that sees k0 before k1
        // treats the slot as another key and may insert a duplicate: harmless, both counts are
        // flushed and summed downstream)
        if (p.x1 == 0) {
            const u64 old = atomicCAS(&K0[p.s1], 0ull, a0);
            if (old == 0) {
                if (med) mk1[p.s1] = a1;
                atomicAdd(&C[p.s1], 1u);
                return true;
            }
            if (old == a0 && !med) { atomicAdd(&C[p.s1], 1u); return true; }
        }
        if (p.x2 == 0) {
            const u64 old = atomicCAS(&K0[p.s2], 0ull, a0);
            if (old == 0) {
                if (med) mk1[p.s2] = a1;
                atomicAdd(&C[p.s2], 1u);
                return true;
            }
            if (old == a0 && !med) { atomicAdd(&C[p.s2], 1u); return true; }
        }
        return false;
    }
};

// Hash-derived indices shared by every kernel that touches a key (they must agree):
//   LDS slots / buckets: lds_hash (MapTable::add, LdsTable::buckets, from its high bits)
//   miss-log bucket: the low bits of lds_hash (k_map has it already; LDS slot choice uses
//   the high bits, so a miss bucket's keys still spread over k_agg's whole table)
//   global-table slot: key_hash, an independent 64-bit function, bits 16+
__device__ __forceinline__ u32 miss_bucket(u32 h, u32 pmask) { return h & pmask; }
__device__ __forceinline__ u64 gslot(u64 h2) { return h2 >> 16; }

// Miss-log units are 8 bytes; an entry is 1-3 units:
//   short key (<= 7 bytes):   k0          (top byte = len, 1..7)
//   medium key (8-15 bytes):  k0, k1      (k0 top byte = key byte 7, a letter byte >= 0x41;
//                                          k1 top byte = len, 8..15)
//   a count c > 1 sets U_CNT in the entry's last key unit and appends the unit c (top byte 0).
// So every unit says what it is from its top byte T alone, and k_agg reads units in parallel:
//   T == 0: count or filler (skip)     (T & 0x1F) < 8: short key      (T & 0x1F) >= 8, T < 0x41:
//   medium-key tail (skip: owned by the head's reader)                 T >= 0x41: medium-key head
constexpr u64 U_CNT = 1ull << 61;

__device__ __forceinline__ int entry_units(u64 k0, u32 c) { return (key_short(k0) ? 1 : 2) + (c > 1 ? 1 : 0); }

// write entry {k0, k1} x c at u[0..entry_units)
__device__ __forceinline__ void put_entry(u64* u, u64 k0, u64 k1, u32 c) {
    const u64 f = c > 1 ? U_CNT : 0;
    if (key_short(k0)) {
        u[0] = k0 | f;
        if (c > 1) u[1] = c;
    } else {
        u[0] = k0;
        u[1] = k1 | f;
        if (c > 1) u[2] = c;
    }
}

}  // namespace wcg
