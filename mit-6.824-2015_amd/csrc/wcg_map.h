// wcg_map.h - the map kernel: DoMap + Map (mapreduce.go:193-231, wc.go:17-30) on gfx950.
//
// One workgroup (16 waves) per CU.  Wave w of workgroup g processes the steps
// g*16 + w + k*(G*16), k = 0, 1, ... on its own (no workgroup barrier in the main loop).  A step
// is 62 chunks of 16 bytes (992 input bytes); the wave loads the 1 KiB window that starts one
// chunk before it, so lane 0 holds the prefix chunk, lanes 1-62 the step's own chunks and lane
// 63 the look-ahead chunk - one coalesced 1 KiB buffer load per wave, no extra loads:
//   1. MAP_SETS windows are in flight per wave (register sets A-D, waits counted exactly: see
//      "prefetch accounting" below);
//   2. the window is staged in the wave's LDS slice (key bytes and UTF-8 context only: every
//      lane computes its chunk's letter mask from registers - SWAR on all-ASCII chunks (fact
//      F2), Go UTF-8 decode + Unicode-13 letter bitmap otherwise (fact F1));
//   3. token starts = letter & ~prev_letter (fact F3) with the neighbour chunks' masks taken by
//      DPP lane shifts; each start's run length is read off the 32-bit mask window (own | next);
//      the wave compacts {offset, length} entries into two LDS lists, short keys (<= 7 bytes)
//      and the others (one DPP prefix sum gives every lane both list offsets);
//   4. tokens, 64 per uniform iteration, the short list then the other: key identity (<= 15
//      bytes, fact F4) from aligned dword LDS reads -> the workgroup's LDS tables (exact keys,
//      u32 counts: MapTable); a miss is appended to this workgroup's region of the miss log for
//      k_agg; a token > 15 bytes is logged for k_long_hash / long_small.  A list's partial last
//      iteration is carried in registers into the next step's first iteration (r06);
//   5. after its last step the wave runs its carried tokens, and the workgroup flushes its LDS
//      table into the miss log too.
// Token ownership: a token belongs to the 16-byte chunk holding its first byte (exactly once);
// only lanes 1-62 own chunks.
//
// Prefetch accounting.  `s_waitcnt vmcnt(N)` waits until all but this wave's N youngest vector
// memory operations are done (loads and stores retire in issue order).  A step's processing
// issues exactly 1 miss-log store per short-key iteration and 2 per medium-key iteration, plus 2
// after its last medium iteration (inline-asm buffer stores executed by the whole wave,
// out-of-range offsets for lanes without a miss), so when set s is due the number of operations
// issued after its loads is known: the other sets' MAP_SETS - 1 loads + the stores of each of the MAP_SETS - 1
// steps processed since.  The
// wait uses the largest quantised N not above that count; any operation the count does not know about (rare paths: long tokens, a full miss-log
// region, UTF-8 table loads) can only make the wait stronger.
#pragma once
#include <type_traits>

#include "wcg_common.h"
#include "wcg_lds_table.h"

namespace wcg {

#ifndef WCG_MAP_NT
#define WCG_MAP_NT 1024
#endif
#ifndef WCG_MAP_WGS
#define WCG_MAP_WGS 1                        // workgroups per CU (LDS and registers split between them)
#endif
constexpr int MAP_NT = WCG_MAP_NT;           // threads per workgroup
constexpr int MAP_WGS = WCG_MAP_WGS;
constexpr int MAP_WAVES = MAP_NT / 64;       // 16 independent waves
constexpr int MAP_OWN = 62;                  // chunks owned per step (lanes 1-62)
constexpr int MAP_STEP = 16 * MAP_OWN;       // 992 input bytes per wave step
constexpr int MAP_WIN = 1024;                // bytes loaded per step: [step base - 16, + 1024)
constexpr int MAP_WREG = MAP_WIN + 8;        // staging (+8: keyread's third word at the end)
constexpr int MAP_SST = 512;                 // max token starts per step (992 / 2 = 496)
#ifndef WCG_DIRECT
#define WCG_DIRECT 0                         // 1: no start list (measured slower: r03_kmap_experiments)
#endif
#ifndef WCG_ADMIT2
#define WCG_ADMIT2 1                         // k_map LDS tables admit keys on their second miss
#endif
// LDS short-key slots (12 B each; the 2 KiB admission filter takes 192 of them, the LDS letter
// table 4.3 KiB); without the start list the window staging (16 x 1032 B) and the lists
// (16 x 1 KiB) are free for 2736 more
#ifndef WCG_MAP_NS
#define WCG_MAP_NS ((WCG_ADMIT2 ? 8410 : 8602) + (WCG_DIRECT ? 2736 : 0))   // (r06: 22 fewer for 64 more cursors)
#endif
#ifndef WCG_MAP_NM
#define WCG_MAP_NM 1024
#endif
constexpr int MAP_NS = WCG_MAP_NS;
constexpr int MAP_NM = WCG_MAP_NM;           // LDS medium-key slots (20 B each)
#ifndef WCG_MAP_SETS
#define WCG_MAP_SETS 4
#endif
constexpr int MAP_SETS = WCG_MAP_SETS;       // steps in flight per wave (2 or 4)
#ifndef WCG_WAIT0
#define WCG_WAIT0 0                          // diagnostics: 1 = wait for every older memory op
#endif
#ifndef WCG_NOWAIT
#define WCG_NOWAIT 0                         // diagnostics: 1 = never wait for the window loads
#endif
#ifndef WCG_STAMPS
#define WCG_STAMPS 0                         // diagnostics: s_memtime cycles per k_map phase
#endif
constexpr int MAP_NSTAMP = 7;                // {loop, window wait, staging+mask, start list, short loop,
                                             //  general loop, steps}
constexpr int MAX_MISS_BUCKETS = 128;        // miss buckets P (the host uses 64 + 32, or 64)
// A key's miss bucket (k_map<ABL, SPLIT>, r06): one-pass jobs (SPLIT) log short keys (<= 7 bytes)
// to buckets 0-63 and medium keys to 64-95, so that every k_agg workgroup aggregates one kind (a
// wave that mixed them paid the medium keys' dependent k1 reads on nearly every probe); 32 medium
// buckets, not 64: a medium region then fills at half a short one's rate (64 left partial lines
// for the L2 to write back, +9% WRITE_SIZE).  Two-pass jobs keep 64 buckets of both kinds.  The
// bucket maps are compile-time constants: as kernel arguments they cost k_map SGPR spills (+2.5%).
constexpr u32 MISS_SHORT_BUCKETS = 64;
template <bool SPLIT> __device__ __forceinline__ u32 short_bucket(u32 h) { return h & (MISS_SHORT_BUCKETS - 1); }
template <bool SPLIT> __device__ __forceinline__ u32 medium_bucket(u32 h) {
    return SPLIT ? (h & (MISS_SHORT_BUCKETS / 2 - 1)) + MISS_SHORT_BUCKETS : (h & (MISS_SHORT_BUCKETS - 1));
}
constexpr u32 SST_LEN_SHIFT = 10;            // start entry = window offset | min(run, 16) << 10

struct MapArgs {
    const uint8_t* in;
    u64 n;
    u64 ntiles;
    u64 tiles_per_wg;
    GEntry* gtab;  u64 gmask;      // inline-key table
    GEntry* ltab;  u64 lmask;      // long-key table
    uint8_t* arena; u64 arena_cap;
    u64 lheap_cap;                 // two-pass contexts: the log heap after the table's heap (bytes)
    DevState* st;
    u64* pool;     u64 region_cap;  // miss log: region (wg, p) = pool[(wg * P + p) * region_cap ...]
    u32* region_len;               // units written per region
    u32 pmask;                     // P - 1 (P = number of miss buckets, power of two)
    u64* wg_stats;                 // [grid][4] per-workgroup {tokens, lds hits, global ops, long}
    u64* llog;     u32 llog_cap;    // long-token log: region wg = llog[wg * llog_cap ...]
    u32* llog_len;                 // records written per region
    Rec* emit;     u64 emit_cap;    // two-pass jobs: the record log (k_long_hash's inline runs)
    u64* stamps;                    // WCG_STAMPS builds: MAP_NSTAMP sums over all waves
};
constexpr u64 LLOG_OFF_MASK = (1ull << 40) - 1;   // record = input offset | len << 40 (len 0: walk)
constexpr u32 LLOG_PER_STEP = 64;                 // long-token log records per step: a bound (a
                                                  // step's 992 bytes start at most 59 tokens of
                                                  // 16+ bytes), so a region never fills

// append one miss-log entry (wcg_lds_table.h) for this workgroup; false when the region is
// full (the units of a region's last, cut-off entry are zeroed so k_agg skips them)
__device__ __forceinline__ bool log_push(const MapArgs& a, u32* cursor, u32 p, u64 k0, u64 k1, u32 c) {
    const u32 nu = (u32)entry_units(k0, c);
    const u32 pos = atomicAdd(&cursor[p], nu);
    u64* r = a.pool + ((u64)blockIdx.x * (a.pmask + 1) + p) * a.region_cap + pos;
    if (pos + nu <= a.region_cap) {
        put_entry(r, k0, k1, c);
        return true;
    }
    for (u32 k = pos; k < a.region_cap; k++) r[k - pos] = 0;
    return false;
}

__device__ __forceinline__ uint4 load_chunk(const uint8_t* in, u64 n, long pos) {
    if (pos >= 0 && (u64)pos + 16 <= n) return *reinterpret_cast<const uint4*>(in + pos);
    uint8_t b[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
        long q = pos + i;
        b[i] = (q >= 0 && (u64)q < n) ? in[q] : 0;
    }
    uint4 v;
    v.x = b[0] | (b[1] << 8) | (b[2] << 16) | ((u32)b[3] << 24);
    v.y = b[4] | (b[5] << 8) | (b[6] << 16) | ((u32)b[7] << 24);
    v.z = b[8] | (b[9] << 8) | (b[10] << 16) | ((u32)b[11] << 24);
    v.w = b[12] | (b[13] << 8) | (b[14] << 16) | ((u32)b[15] << 24);
    return v;
}

__device__ __forceinline__ u64 long_tag(u64 h, u64 len) { return mix64(h ^ len) | 1ull; }

// count c occurrences of one long key (> 15 bytes; tag = long_tag(FNV-1a 64 of its bytes, len))
// in the long-key table; w(j) returns key word j (little-endian bytes 4j..4j+3, zeros past len).
// Key bytes are written and compared 16 bytes at a time against the zero-padded arena cells
// (wcg_common.h): a byte loop over global memory is a chain of dependent loads per byte.
// Publication: `fenced` (any key, any workgroup, concurrently): the arena bytes are released
// before k1 publishes them and acquired before they are compared.  Unfenced (k_long_agg's flush):
// within one launch a key reaches the table from ONE workgroup only (its partition's), so the
// only writer a reader can race is its own workgroup - same CU, same L2 - and the bytes are
// compared with L1-bypassing loads; an agent-scope fence per key wrote back the whole XCD L2
// (~2-6 us) and made the old per-occurrence k_long take 8.8 ms on 1 GiB of C4.
// Returns the slot that counted the key + 1 (0 when nothing was counted).
template <typename W>
__device__ __forceinline__ u64 ltab_add(const MapArgs& a, u64 len, u64 tag, W w, u64 c, bool fenced) {
    if (len > LONG_LEN_MAX) { atomicAdd(&a.st->overflow, 1u); return 0; }
    u64 s = tag & a.lmask, probes = 0;
    int spins = 0;
    while (true) {
        GEntry* e = &a.ltab[s];
        // the entry's three words in one round trip (independent loads); aux (the length) is
        // written once, before k1 is published: a 0 read here is re-read after k1, any other
        // value is final
        u64 c0 = ld_agent(&e->k0);
        u64 r = ld_agent(&e->k1);
        u64 elen = ld_agent(&e->aux);
        if (c0 == 0) {
            u64 exp;
            if (ltab_claim(a.st, e, s, tag, &exp)) {
                const u64 off = long_home(s, len, a.lmask + 1, a.arena_cap, &a.st->arena_top);
                if (off == ~0ull) { atomicAdd(&a.st->overflow, 1u); return 0; }
                const u64 cells = long_cells(len);
                for (u64 j = 0; j < cells; j += 16)
                    *reinterpret_cast<uint4*>(a.arena + off + j) =
                        make_uint4(w(j / 4), w(j / 4 + 1), w(j / 4 + 2), w(j / 4 + 3));
                st_agent(&e->aux, len);
                if (fenced) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(&e->k1, off + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                add_agent(&e->cnt, c);
                return s + 1;
            }
            c0 = exp;
            r = ld_agent(&e->k1);
        }
        if (c0 == tag) {
            if (r == 0) {
                if (++spins > SPIN_LIMIT) { atomicAdd(&a.st->spin_fail, 1u); return 0; }
                continue;
            }
            if (fenced) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            if (elen == 0) elen = ld_agent(&e->aux);
            bool same = elen == len;
            if (same) {                 // 16-byte cells, zero-padded on both sides
                u32 diff = 0;
                for (u64 j = 0; j < len; j += 16) {
                    const u64* q = reinterpret_cast<const u64*>(a.arena + r - 1 + j);
                    const u64 v0 = fenced ? q[0] : ld_agent(q), v1 = fenced ? q[1] : ld_agent(q + 1);
                    diff |= ((u32)v0 ^ w(j / 4)) | ((u32)(v0 >> 32) ^ w(j / 4 + 1)) | ((u32)v1 ^ w(j / 4 + 2)) |
                            ((u32)(v1 >> 32) ^ w(j / 4 + 3));
                }
                same = diff == 0;
            }
            if (same) {
                add_agent(&e->cnt, c);
                return s + 1;
            }
        }
        s = (s + 1) & a.lmask;
        if (++probes > a.lmask) { atomicAdd(&a.st->overflow, 1u); return 0; }
    }
}

// aligned input dword at byte offset off (a multiple of 4); bytes past the input read as 0
__device__ __forceinline__ u32 input_dword(const MapArgs& a, u64 off) {
    if (off + 4 <= a.n) return *reinterpret_cast<const u32*>(a.in + off);
    u32 v = 0;
    for (u32 b = 0; b < 4; b++) if (off + b < a.n) v |= (u32)a.in[off + b] << (8 * b);
    return v;
}

// length of the letter run at absolute offset p (a run that reached the map window's look-ahead
// chunk).  16-byte chunks are loaded whole (one round trip each): an all-ASCII chunk is classified
// by the SWAR mask, any other one rune by rune from its registers (r04: the byte-at-a-time walk
// waited on a global load per byte - C4's walked runs cost k_long_hash most of its 0.9-1.3 ms)
__device__ u64 long_walk(const MapArgs& a, u64 p) {
    const u64 n = a.n;
    u64 q = p;
    while (q < n) {
        const u64 base = q & ~15ull;
        const uint4 c = load_chunk(a.in, n, (long)base);
        const u32 off = (u32)(q - base);
        if (all_ascii(c)) {
            const u32 m = ascii_mask16(c) >> off;
            const u32 run = (u32)__builtin_ctz(~m);          // letters from q within the chunk
            q += run;
            if (run < 16 - off) return q - p;
            continue;
        }
        const u32 d4 = input_dword(a, base + 16);           // runes may end up to 3 bytes past
        const u32 d[5] = {c.x, c.y, c.z, c.w, d4};
        auto at = [&](long i) -> u32 {                       // chunk byte i (0..19); 0 past the input
            if ((u64)(base + i) >= n) return 0u;
            u32 w = 0;                                       // masks, not selects (no indexed array)
#pragma unroll
            for (int k = 0; k < 5; k++) w |= d[k] & (0u - (u32)((i >> 2) == k));
            return (w >> (8 * (i & 3))) & 0xFFu;
        };
        u32 j = off;
        while (j < 16) {
            u32 cp;
            const int w = go_decode(at, (long)j, &cp);
            if (w == 0 || !lt_is_letter(cp)) return base + j - p;
            j += (u32)w;
        }
        q = base + j;
    }
    return n - p;
}

// a run that turned out to be an inline key (<= 15 bytes: measured only after a rune walk); called
// by the lanes of a wave that found one
__device__ __forceinline__ void count_inline_run(const MapArgs& a, u64 p, u64 len) {
    u64 b0 = 0, b1 = 0;
    for (u64 i = 0; i < len; i++) {
        if (i < 8) b0 |= (u64)a.in[p + i] << (8 * i);
        else b1 |= (u64)a.in[p + i] << (8 * (i - 8));
    }
    u64 k0, k1;
    make_key(b0, b1, (int)len, k0, k1);
    if (a.emit) {                     // two-pass job: one record in the record log (merged after
        const u64 act = __ballot(1);  // the sort), one atomic per wave: the global table stays empty
        const u32 rank = __builtin_amdgcn_mbcnt_hi((u32)(act >> 32), __builtin_amdgcn_mbcnt_lo((u32)act, 0u));
        u64 base = 0;
        if (rank == 0) base = atomicAdd((unsigned long long*)&a.st->nemit, (unsigned long long)__popcll(act));
        base = (u64)__builtin_amdgcn_readfirstlane((u32)(base >> 32)) << 32 | __builtin_amdgcn_readfirstlane((u32)base);
        if (base + rank < a.emit_cap) { a.emit[base + rank] = inline_rec(k0, k1, 1); return; }
    }
    ginsert(a.gtab, a.gmask, k0, k1, gslot(key_hash(k0, k1)), 1, a.st);
    atomicAdd(&a.st->global_ops, 1ull);
}

// key word j (little-endian bytes 4j..4j+3 of the key at input offset p, zeros past len) from
// the resident input: two aligned loads + alignbyte
__device__ __forceinline__ u32 input_word(const MapArgs& a, u64 p, u32 len, u64 j) {
    if (4 * (u32)j >= len) return 0u;
    const u64 base = p + 4 * j, q = base & ~3ull;
    const u32 rem = len - 4 * (u32)j;
    u32 v;
    if (q + 8 <= a.n) {
        const u32* wq = reinterpret_cast<const u32*>(a.in + q);
        v = __builtin_amdgcn_alignbyte(wq[1], wq[0], (u32)(base & 3));
    } else {
        v = 0;
        for (u32 b = 0; b < 4 && b < rem; b++) v |= (u32)a.in[base + b] << (8 * b);
    }
    return rem >= 4 ? v : v & ((1u << (8 * rem)) - 1);
}


// key words j0 .. j0+7 of the key at input offset p (len bytes; zeros past len), from 9 aligned
// dword loads issued together: a word-at-a-time loop waits for each load in turn, and these
// loads go to HBM (long tokens are scattered over the input)
__device__ __forceinline__ void input_words8(const MapArgs& a, u64 p, u32 len, u32 j0, u32* v) {
    const u64 base = p + 4 * (u64)j0, q = base & ~3ull;
    const u32 sh = (u32)(base & 3);
    u32 d[9];
#pragma unroll
    for (int k = 0; k < 9; k++) d[k] = 4 * (j0 + k) < len + 4 ? input_dword(a, q + 4 * k) : 0u;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const u32 at = 4 * (j0 + k);
        const u32 w = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
        v[k] = at >= len ? 0u : (len - at >= 4 ? w : w & ((1u << (8 * (len - at))) - 1));
    }
}

// the long-key hash (lhash_step) of the key at input offset p (len bytes), and its first 8 words
// (key bytes 0-31, zeros past len) in w8
__device__ __forceinline__ u64 input_lhash(const MapArgs& a, u64 p, u32 len, u32 (&w8)[8]) {
    u64 h = LHASH_INIT;
    for (u32 j0 = 0; 4 * j0 < len; j0 += 8) {
        u32 v[8];
        input_words8(a, p, len, j0, v);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (j0 == 0) w8[k] = v[k];
            if (4 * (j0 + k) < len) h = lhash_step(h, v[k]);
        }
    }
    return h;
}

// do the long keys at input offsets p and q (both len bytes) have the same bytes?  (32 bytes of
// both per round trip)
__device__ __forceinline__ bool input_same(const MapArgs& a, u64 p, u64 q, u32 len) {
    if (p == q) return true;
    u32 diff = 0;
    for (u32 j0 = 0; 4 * j0 < len && diff == 0; j0 += 8) {
        u32 x[8], y[8];
        input_words8(a, p, len, j0, x);
        input_words8(a, q, len, j0, y);
#pragma unroll
        for (int k = 0; k < 8; k++) diff |= x[k] ^ y[k];
    }
    return diff == 0;
}

// long token (> 15 bytes) starting at window offset rp (absolute offset p): its length from the
// wave's chunk letter masks (LDS), then one record in the workgroup's long-token log; k_long
// counts it.  A run that reaches the look-ahead chunk may continue past the window: its record
// has length 0 and k_long walks its runes.  The global-table work stays out of k_map's token
// loop: a dependent global load there waits for every older load of the wave, which drains the
// window prefetch (measured: 40 ms of 47 per GiB of C4 text with the insert done here).
template <int ABL = 0>
__device__ __forceinline__ void long_token_log(const MapArgs& a, u64 p, u32 rp, const uint16_t* wm, u32* lcur) {
    u32 c = rp >> 4, b = rp & 15, len = 0;
    while (true) {
        if (c >= 63) { len = 0; break; }
        const u32 mm = (u32)wm[c] >> b;             // the chunk's bits from b on (zeros above)
        const u32 t = __builtin_ctz(~mm);
        if (t < 16 - b) { len += t; break; }
        len += 16 - b;
        c++;
        b = 0;
    }
    if (ABL == 7) { asm volatile("" ::"v"(len)); return; }
    const u32 pos = atomicAdd(lcur, 1u);
    if (pos < a.llog_cap) a.llog[(u64)blockIdx.x * a.llog_cap + pos] = p | (u64)len << 40;
    else atomicAdd(&a.st->overflow, 1u);   // cannot happen (LLOG_PER_STEP); fails loudly if it does
}

// ---- long keys: k_long_hash -> k_long_agg.  Every occurrence of a long key is routed, by its
//      tag, to one of LQ partitions, so ONE workgroup aggregates all of a key's occurrences in
//      LDS (exact: bytes compared against a representative occurrence in the resident input) and
//      adds the key to the long-key table once, unfenced.  The per-occurrence table inserts of a
//      flat design serialise on hot keys and on the fences that publish arena bytes across CUs.
constexpr u32 LQ = 2048;                      // partitions
// an entry: lhash, input offset | len << 40, occurrences, and the key's bytes 0-31 (zeros past
// len), so that k_long_agg compares keys of up to 32 bytes (C4: nearly all long keys) in LDS
// instead of re-reading two occurrences from the input (r04)
struct LEnt { u64 h; u64 rec; u64 cnt; u64 pad; uint4 w0, w1; };
static_assert(sizeof(LEnt) == 64, "four 16-byte stores per entry");
struct LongPart { LEnt* ent; u32* cur; u32 cap; };
__device__ __forceinline__ u32 long_part(u64 tag) { return (u32)(tag >> 40) & (LQ - 1); }
__device__ __forceinline__ bool w8_same(const u32 (&x)[8], const uint4& y0, const uint4& y1) {
    return ((x[0] ^ y0.x) | (x[1] ^ y0.y) | (x[2] ^ y0.z) | (x[3] ^ y0.w) | (x[4] ^ y1.x) | (x[5] ^ y1.y) |
            (x[6] ^ y1.z) | (x[7] ^ y1.w)) == 0;
}
// the words of a long key for ltab_add: words 0-7 (bytes 0-31, zeros past len) held here, the rest
// read from the input at offset p.  A plain struct (no reference to the kernel's arguments and no
// array indexed at run time: either put the whole argument block or the array in scratch)
struct LongKeyWords {
    const uint8_t* in; u64 n; u64 p; u32 len; u32 w[8];
    __device__ __forceinline__ u32 operator()(u64 j) const {
        if (j >= 8) {
            if (4 * (u32)j >= len) return 0u;
            u32 v = 0;
            for (u32 b = 0; b < 4 && 4 * (u32)j + b < len; b++) v |= (u32)in[p + 4 * j + b] << (8 * b);
            return v;
        }
        u32 r = 0;                    // masks, not selects (selects fold back into an indexed load)
#pragma unroll
        for (int k = 0; k < 8; k++) r |= w[k] & (0u - (u32)(j == (u64)k));
        return r;
    }
};
__device__ __forceinline__ LongKeyWords long_words(const MapArgs& a, u64 p, u64 len, const u32 (&w)[8]) {
    LongKeyWords k;
    k.in = a.in; k.n = a.n; k.p = p; k.len = (u32)len;
#pragma unroll
    for (int i = 0; i < 8; i++) k.w[i] = w[i];
    return k;
}
// the same long key (len bytes each) at input offsets p and q, whose bytes 0-31 are known equal
__device__ __forceinline__ bool long_rest_same(const MapArgs& a, u64 p, u64 q, u32 len) {
    return len <= 32 || input_same(a, p + 32, q + 32, len - 32);
}

// k_long_hash: workgroup b reads map region b % nreg (its LONG_PARTS workgroups stride over the
// region's records in rounds of LONG_NT), hashes each logged token from the resident input
// (walking runes for records of length 0) and emits {h, rec, count, bytes 0-31} to the token's
// partition.  Repeats are pre-aggregated in an LDS cache keyed by tag (hot keys: C4's top long key
// occurs 1.2e5 times per GiB), compared byte-exactly against the cached representative's bytes
// (LDS; bytes past 32 from the input) - no other CU's writes are read, so no fence is needed.  A
// lane never waits on another's LDS write: a cache entry claimed in the same round may still have
// no representative (rec 0), and such a lane simply emits its own entry.  A full partition falls
// back to a fenced table insert.
#ifndef WCG_LH_ABL
#define WCG_LH_ABL 0      // diagnostics (wrong counts): 1 = no partition atomics, 2 = no input reads, 4 = no LDS cache
#endif
constexpr int LONG_NT = 256;
constexpr int LONG_PARTS = 8;
#ifndef WCG_LCACHE
#define WCG_LCACHE 512
#endif
constexpr int LCACHE = WCG_LCACHE;            // LDS cache entries (60 B each: 512 -> 5 workgroups per CU)
#ifndef WCG_LH_U
#define WCG_LH_U 2
#endif
constexpr int LH_U = WCG_LH_U;
__global__ __launch_bounds__(LONG_NT) void k_long_hash(MapArgs a, LongPart lp, u32 nreg) {
    __shared__ u64 ctag[LCACHE];
    __shared__ u64 crec[LCACHE];              // representative occurrence (0 = not yet set)
    __shared__ u64 chash[LCACHE];
    __shared__ u32 ccnt[LCACHE];
    __shared__ uint4 cw[LCACHE][2];           // representative's bytes 0-31
    // a persistent grid over the (region, part) items: on low-cardinality text nearly every item
    // is empty (C2: ~200 long tokens per GiB) and costs one read of its region's length, not a
    // workgroup launch
    for (u32 item = blockIdx.x; item < nreg * LONG_PARTS; item += gridDim.x) {
    const u32 reg = item % nreg, part = item / nreg;
    const u32 nrec = a.llog_len[reg];
    const u64* recs = a.llog + (u64)reg * a.llog_cap;
    const u32 stride = LONG_PARTS * LONG_NT, first = part * LONG_NT;
    const u32 rounds = nrec > first ? (nrec - first + stride - 1) / stride : 0;   // workgroup-uniform
    if (rounds == 0) continue;
    for (int e = threadIdx.x; e < LCACHE; e += LONG_NT) { ctag[e] = 0; crec[e] = 0; ccnt[e] = 0; }
    __syncthreads();
    // an entry into its partition at a reserved position (pos >= cap: partition full, counted here
    // instead: fenced, exact)
    auto put = [&](u32 q, u32 pos, u64 h, u64 rec, u64 c, const u32 (&w)[8]) {
        if (pos < lp.cap) {
            uint4* d = reinterpret_cast<uint4*>(lp.ent + (u64)q * lp.cap + pos);
            d[0] = make_uint4((u32)h, (u32)(h >> 32), (u32)rec, (u32)(rec >> 32));
            d[1] = make_uint4((u32)c, (u32)(c >> 32), 0u, 0u);
            d[2] = make_uint4(w[0], w[1], w[2], w[3]);
            d[3] = make_uint4(w[4], w[5], w[6], w[7]);
        } else {
            const u64 len = rec >> 40, p = rec & LLOG_OFF_MASK;
            atomicAdd(&a.st->long_fb, 1u);
            ltab_add(a, len, long_tag(h, len), long_words(a, p, len, w), c, true);
        }
    };
    auto emit = [&](u64 h, u64 rec, u64 c, const u32 (&w)[8]) {
        const u32 q = long_part(long_tag(h, rec >> 40));
        put(q, (WCG_LH_ABL & 1) ? (u32)(h & 63) : atomicAdd(&lp.cur[q], 1u), h, rec, c, w);
    };
    // one occurrence into the LDS cache: true when it was counted there
    auto cache_add = [&](u64 h, u64 p, u64 len, const u32 (&w)[8]) -> bool {
        const u64 tag = long_tag(h, len), rec = p | len << 40;
        const u32 c0 = (u32)(tag >> 24) & (LCACHE - 1);
        for (u32 q = 0; q < 4; q++) {
            const u32 cs = (c0 + q) & (LCACHE - 1);
            u64 t = ctag[cs];
            if (t == 0) {
                t = atomicCAS((unsigned long long*)&ctag[cs], 0ull, (unsigned long long)tag);
                if (t == 0) {
                    cw[cs][0] = make_uint4(w[0], w[1], w[2], w[3]);
                    cw[cs][1] = make_uint4(w[4], w[5], w[6], w[7]);
                    chash[cs] = h;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __hip_atomic_store(&crec[cs], rec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    atomicAdd(&ccnt[cs], 1u);
                    return true;
                }
            }
            if (t != tag) continue;
            const u64 rr = __hip_atomic_load(&crec[cs], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (rr != 0 && (rr >> 40) == len) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                if (w8_same(w, cw[cs][0], cw[cs][1]) && long_rest_same(a, p, rr & LLOG_OFF_MASK, (u32)len)) {
                    atomicAdd(&ccnt[cs], 1u);
                    return true;
                }
            }
            return false;             // same tag, other key or not yet set: emit
        }
        return false;
    };
    // LH_U records per thread and round: their input reads, and then their partition atomics,
    // are in flight together (the round was one dependent chain: record, input words, cache,
    // partition atomic, stores)
    for (u32 k = 0; k < rounds; k += LH_U) {
        u64 hh[LH_U], pp[LH_U], ll[LH_U];
        u32 ww[LH_U][8];
#pragma unroll
        for (int u = 0; u < LH_U; u++) {
            const u32 i = first + (k + u) * stride + threadIdx.x;
            const bool live = k + u < rounds && i < nrec;
            const u64 r = live ? recs[i] : 0;
            pp[u] = r & LLOG_OFF_MASK;
            ll[u] = r >> 40;
            hh[u] = 0;
#pragma unroll
            for (int j = 0; j < 8; j++) ww[u][j] = 0;
            if (live && ll[u] == 0) {             // a run to measure (length 0 in the log)
                u64 len = long_walk(a, pp[u]);
                if (len <= 15) { count_inline_run(a, pp[u], len); len = 0; }
                else if (len > LONG_LEN_MAX) { atomicAdd(&a.st->overflow, 1u); len = 0; }
                ll[u] = len;
            }
        }
#pragma unroll
        for (int u = 0; u < LH_U; u++) {
            if (ll[u] == 0) continue;
            if (WCG_LH_ABL & 2) { ww[u][0] = (u32)pp[u]; hh[u] = pp[u] * 0x9E3779B97F4A7C15ull; }   // diagnostics
            else hh[u] = input_lhash(a, pp[u], (u32)ll[u], ww[u]);
        }
        bool em[LH_U];
#pragma unroll
        for (int u = 0; u < LH_U; u++) {
            em[u] = ll[u] != 0;
            if (em[u] && !(WCG_LH_ABL & 4)) em[u] = !cache_add(hh[u], pp[u], ll[u], ww[u]);
            if (LH_U > 1 && u + 1 < LH_U) __syncthreads();   // representatives of u visible to u + 1
        }
        u32 qq[LH_U], pos[LH_U];
#pragma unroll
        for (int u = 0; u < LH_U; u++) {
            qq[u] = long_part(long_tag(hh[u], ll[u]));
            pos[u] = 0;
            if (em[u]) pos[u] = (WCG_LH_ABL & 1) ? (u32)(hh[u] & 63) : atomicAdd(&lp.cur[qq[u]], 1u);
        }
#pragma unroll
        for (int u = 0; u < LH_U; u++)
            if (em[u]) put(qq[u], pos[u], hh[u], pp[u] | ll[u] << 40, 1, ww[u]);
        __syncthreads();              // this round's representatives are visible to the next
    }
    for (int e = threadIdx.x; e < LCACHE; e += LONG_NT) {
        const u64 rr = crec[e];
        if (rr == 0 || ccnt[e] == 0) continue;
        const uint4 x = cw[e][0], y = cw[e][1];
        const u32 w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
        emit(chash[e], rr, ccnt[e], w);
    }
    __syncthreads();                  // the cache is reused by the next item
    }
}

// k_long_agg: one workgroup per partition.  Rounds of LA_NT entries: (1) each entry claims or
// finds its tag's LDS slot (linear probing) and the claimer stores its key bytes 0-31 and
// occurrence as the slot's representative; barrier; (2) each entry compares its bytes with the
// representative's (LDS; bytes past 32 from the input) and adds its count.  A tag collision
// between different keys, or a full table, falls back to a fenced table insert of that entry
// (exact).  Finally every slot is added to the long-key table once, from its LDS bytes.
#ifndef WCG_LA_ABL
#define WCG_LA_ABL 0                          // diagnostics (wrong counts): 1 = no table inserts, 2 = no fallbacks
#endif
constexpr u32 LA_SLOTS = 2048;
constexpr u32 LA_PROBES = 32;
constexpr int LA_NT = 512;                    // one 112 KiB workgroup per CU: 8 waves
constexpr u32 LA_MAXQ = 64;                   // partitions per workgroup (grid >= LQ / LA_MAXQ)
// A persistent grid over the LQ partitions (one 112 KiB workgroup per CU; on low-cardinality
// text nearly every partition is empty and costs one read of its cursor, not a launch slot)
__global__ __launch_bounds__(LA_NT) void k_long_agg(MapArgs a, LongPart lp) {
    __shared__ u64 stag[LA_SLOTS], srec[LA_SLOTS], scnt[LA_SLOTS];
    __shared__ uint4 sw[LA_SLOTS][2];
    __shared__ u32 qn[LA_MAXQ];               // this workgroup's partitions' entry counts
    __shared__ u32 la_wk[LA_NT / 64], la_wb[LA_NT / 64];   // per-wave key / heap byte sums
    __shared__ u64 la_base[2];                // the partition's record-log and heap reservations
    // every cursor of the workgroup's partitions read at once (one round trip, not one per
    // partition), then reset for the next map call
    for (u32 t = threadIdx.x, q = blockIdx.x + t * gridDim.x; t < LA_MAXQ; t += LA_NT, q += LA_NT * gridDim.x) {
        const u32 cq = q < LQ ? lp.cur[q] : 0u;
        qn[t] = cq;
        if (cq) lp.cur[q] = 0;
    }
    __syncthreads();
    for (u32 t = 0, q = blockIdx.x; q < LQ; t++, q += gridDim.x) {
    const u32 nq = qn[t] < lp.cap ? qn[t] : lp.cap;
    if (nq == 0) continue;
    for (u32 s = threadIdx.x; s < LA_SLOTS; s += LA_NT) { stag[s] = 0; srec[s] = 0; scnt[s] = 0; }
    __syncthreads();
    const LEnt* E = lp.ent + (u64)q * lp.cap;
    for (u32 base = 0; base < nq; base += LA_NT) {
        const u32 e = base + threadIdx.x;
        const bool valid = e < nq;
        uint4 d0 = make_uint4(0, 0, 0, 0), d1 = d0, d2 = d0, d3 = d0;
        if (valid) {
            const uint4* src = reinterpret_cast<const uint4*>(E + e);
            d0 = src[0]; d1 = src[1]; d2 = src[2]; d3 = src[3];
        }
        const u64 h = (u64)d0.y << 32 | d0.x, rec = (u64)d0.w << 32 | d0.z, cnt = (u64)d1.y << 32 | d1.x;
        const u32 w[8] = {d2.x, d2.y, d2.z, d2.w, d3.x, d3.y, d3.z, d3.w};
        const u64 len = rec >> 40, p = rec & LLOG_OFF_MASK;
        const u64 tag = long_tag(h, len);
        int slot = -1;
        if (valid) {
            const u32 s0 = (u32)(tag >> 8) & (LA_SLOTS - 1);
            for (u32 j = 0; j < LA_PROBES; j++) {
                const u32 s = (s0 + j) & (LA_SLOTS - 1);
                u64 t = stag[s];
                if (t == 0) {
                    t = atomicCAS((unsigned long long*)&stag[s], 0ull, (unsigned long long)tag);
                    if (t == 0) { srec[s] = rec; sw[s][0] = d2; sw[s][1] = d3; slot = (int)s; break; }
                }
                if (t == tag) { slot = (int)s; break; }
            }
        }
        __syncthreads();
        bool fallback = valid && slot < 0;
        if (valid && slot >= 0) {
            const u64 rr = srec[slot];
            if ((rr >> 40) == len && w8_same(w, sw[slot][0], sw[slot][1]) &&
                long_rest_same(a, p, rr & LLOG_OFF_MASK, (u32)len))
                atomicAdd((unsigned long long*)&scnt[slot], (unsigned long long)cnt);
            else fallback = true;
        }
        if (fallback && !(WCG_LA_ABL & 2)) {
            atomicAdd(&a.st->long_fb, 1u);
            ltab_add(a, len, tag, long_words(a, p, len, w), cnt, true);
        }
        __syncthreads();              // slots claimed in the next round cannot be confused with ...
    }                                 // ... representatives read in this one
    // Two-pass jobs (a record log): the partition's keys become records of the log directly, their
    // bytes copied to the arena heap - one reservation of log records and one of heap bytes per
    // partition.  (r04: adding them to the long-key table took 1.4 of the kernel's 1.6 ms on C4:
    // 1.6M dependent probe / claim / publish chains over a 512 MiB table.)  A key repeated by
    // another map call, or also counted through the table (fallbacks, imports), is merged after
    // the sort (k_tie_sort).  Otherwise, or when the log or the heap is full: the table, once.
    bool to_log = a.emit != nullptr && a.lheap_cap != 0 && !(WCG_LA_ABL & 1);
    u32 rk[LA_SLOTS / LA_NT];                 // this thread's slots: rank among filled ones, heap bytes
    u32 hb[LA_SLOTS / LA_NT];
    if (to_log) {
        // slots t * LA_NT + tid: per-thread counts, then a block prefix sum (waves in order)
        u32 nk = 0, nb = 0;
#pragma unroll
        for (u32 k = 0; k < LA_SLOTS / LA_NT; k++) {
            const u32 sl = k * LA_NT + threadIdx.x;
            const bool f = scnt[sl] != 0;
            rk[k] = nk; hb[k] = nb;
            nk += f ? 1u : 0u;
            nb += f ? (u32)long_cells(srec[sl] >> 40) : 0u;
        }
        const u32 lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        u32 ik = nk, ib = nb;
        for (int d = 1; d < 64; d <<= 1) {
            const u32 yk = __shfl_up(ik, d, 64), yb = __shfl_up(ib, d, 64);
            if (lane >= (u32)d) { ik += yk; ib += yb; }
        }
        if (lane == 63) { la_wk[wv] = ik; la_wb[wv] = ib; }
        __syncthreads();
        u32 pk = 0, pb = 0, tk = 0, tb = 0;
        for (u32 v = 0; v < LA_NT / 64; v++) {
            if (v < wv) { pk += la_wk[v]; pb += la_wb[v]; }
            tk += la_wk[v]; tb += la_wb[v];
        }
        if (threadIdx.x == 0) {
            // log-heap bytes first (a heap of their own: a reservation past its cap leaves the
            // table's heap untouched; r04: a CAS loop on the shared top serialised the 256
            // workgroups, ~1.5 ms), then the log records; nothing once the log is full
            u64 h0 = ~0ull, r0 = ~0ull;
            if (tk && ld_agent(&a.st->nemit) < a.emit_cap) {
                const u64 h = atomicAdd((unsigned long long*)&a.st->lheap_top, (unsigned long long)tb);
                if (h + tb <= a.lheap_cap) {
                    h0 = h;
                    r0 = atomicAdd((unsigned long long*)&a.st->nemit, (unsigned long long)tk);
                }
            }
            la_base[0] = r0;
            la_base[1] = h0;
            // keys past the log's cap go to the table (their heap bytes stay unused)
            const u64 fit = r0 == ~0ull || r0 >= a.emit_cap ? 0 : (a.emit_cap - r0 < tk ? a.emit_cap - r0 : tk);
            if (fit) atomicAdd((unsigned long long*)&a.st->lemit, (unsigned long long)fit);
        }
        __syncthreads();
        to_log = la_base[0] != ~0ull;
#pragma unroll
        for (u32 k = 0; k < LA_SLOTS / LA_NT; k++) { rk[k] += pk + ik - nk; hb[k] += pb + ib - nb; }
    }
#pragma unroll
    for (u32 k = 0; k < LA_SLOTS / LA_NT; k++) {
        const u32 s = k * LA_NT + threadIdx.x;
        const u64 c = scnt[s];
        if (c == 0) continue;
        const u64 rr = srec[s], len = rr >> 40, p = rr & LLOG_OFF_MASK;
        const uint4 x = sw[s][0], y = sw[s][1];
        const u32 w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
        if (to_log && la_base[0] + rk[k] < a.emit_cap) {
            const u64 off = (a.lmask + 1) * LONG_CELL + a.arena_cap + la_base[1] + hb[k];
            const LongKeyWords kw = long_words(a, p, len, w);
            const u64 cells = long_cells(len);
            for (u64 j = 0; j < cells; j += 16)
                *reinterpret_cast<uint4*>(a.arena + off + j) =
                    make_uint4(kw(j / 4), kw(j / 4 + 1), kw(j / 4 + 2), kw(j / 4 + 3));
            Rec r;
            r.hi = bswap64((u64)x.y << 32 | x.x);
            r.lo = bswap64((u64)x.w << 32 | x.z);
            r.cnt = c;
            r.ref = LONG_FLAG | (len << 40) | off;
            a.emit[la_base[0] + rk[k]] = r;
        } else if (!(WCG_LA_ABL & 1)) {
            ltab_add(a, len, stag[s], long_words(a, p, len, w), c, false);
        }
    }
    __syncthreads();                          // the LDS is reused by the next partition
    }
}

// long_small: the long-key work of a one-pass map call with few long tokens, in ONE workgroup
// (C2 logs ~200 long tokens per GiB; k_long_hash + k_long_agg, a 1024-workgroup and a
// 256-workgroup launch that nearly all find nothing to do, took 17.5 us per step: r05 trace).
// Rounds of LS_NT logged tokens over every region (a region found by binary search over the
// regions' prefix in LDS): each token is walked if its length was left open, hashed from the
// input, and claims or finds its tag's LDS slot (the claimer's occurrence is the slot's
// representative); after a barrier it is compared with the representative (bytes 0-31 in LDS, the
// rest from the input) and counted there.  Then every slot is added to the long-key table once,
// unfenced: this workgroup is the table's only writer in the launch (as a partition's workgroup is
// in k_long_agg).  Exact for any number of tokens: a tag collision or a full LDS table falls back to
// a fenced insert of that occurrence; more tokens only take more rounds.
constexpr int LS_NT = 1024;
constexpr u32 LS_SLOTS = 2048;
constexpr u32 LS_MAXREG = LS_NT;              // map regions (one length per thread)
struct LsLds {
    u64 stag[LS_SLOTS], srec[LS_SLOTS], scnt[LS_SLOTS];
    u32 sw[LS_SLOTS][8];
    u32 rpre[LS_MAXREG + 1];
    u32 ws[LS_NT / 64];
};
// r06: run by the last workgroup of k_agg's one-pass launch (lds: k_agg's table memory), which
// starts on the first CU a k_agg workgroup leaves: the separate one-workgroup launch and its
// dependency cost ~15 us of every C2 step
__device__ __forceinline__ void long_small(const MapArgs& a, u32 nreg, LsLds& L) {
    u64* const stag = L.stag;
    u64* const srec = L.srec;
    u64* const scnt = L.scnt;
    u32* const rpre = L.rpre;
    u32* const ls_ws = L.ws;
    const u32 tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (u32 s = tid; s < LS_SLOTS; s += LS_NT) { stag[s] = 0; srec[s] = 0; scnt[s] = 0; }
    // the regions' record counts (clamped to the log: a fuller region was flagged by k_map) and
    // their exclusive prefix
    u32 cnt = tid < nreg ? a.llog_len[tid] : 0u;
    cnt = cnt < a.llog_cap ? cnt : a.llog_cap;
    u32 incl = cnt;
    for (int d = 1; d < 64; d <<= 1) { const u32 y = __shfl_up(incl, d, 64); if (lane >= (u32)d) incl += y; }
    if (lane == 63) ls_ws[wv] = incl;
    __syncthreads();
    u32 pre = 0, total = 0;
    for (u32 v = 0; v < LS_NT / 64; v++) { if (v < wv) pre += ls_ws[v]; total += ls_ws[v]; }
    if (tid <= nreg) rpre[tid] = tid < nreg ? pre + incl - cnt : total;
    __syncthreads();
    for (u32 base = 0; base < total; base += LS_NT) {
        const u32 i = base + tid;
        u64 p = 0, len = 0, h = 0;
        u32 w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (i < total) {
            u32 lo = 0, hi = nreg;                    // the region: the last r with rpre[r] <= i
            while (hi - lo > 1) {
                const u32 mid = (lo + hi) >> 1;
                if (rpre[mid] <= i) lo = mid; else hi = mid;
            }
            const u64 r = a.llog[(u64)lo * a.llog_cap + (i - rpre[lo])];
            p = r & LLOG_OFF_MASK;
            len = r >> 40;
            if (len == 0) {                           // a run to measure (length 0 in the log)
                u64 L = long_walk(a, p);
                if (L <= 15) { count_inline_run(a, p, L); L = 0; }
                else if (L > LONG_LEN_MAX) { atomicAdd(&a.st->overflow, 1u); L = 0; }
                len = L;
            }
            if (len) h = input_lhash(a, p, (u32)len, w);
        }
        const bool valid = len != 0;
        const u64 tag = valid ? long_tag(h, len) : 0;
        int slot = -1;
        if (valid) {
            const u32 s0 = (u32)(tag >> 8) & (LS_SLOTS - 1);
            for (u32 j = 0; j < LA_PROBES; j++) {
                const u32 s = (s0 + j) & (LS_SLOTS - 1);
                u64 t = stag[s];
                if (t == 0) {
                    t = atomicCAS((unsigned long long*)&stag[s], 0ull, (unsigned long long)tag);
                    if (t == 0) {
                        srec[s] = p | len << 40;
                        *reinterpret_cast<uint4*>(&L.sw[s][0]) = make_uint4(w[0], w[1], w[2], w[3]);
                        *reinterpret_cast<uint4*>(&L.sw[s][4]) = make_uint4(w[4], w[5], w[6], w[7]);
                        slot = (int)s;
                        break;
                    }
                }
                if (t == tag) { slot = (int)s; break; }
            }
        }
        __syncthreads();                              // representatives written
        bool fallback = valid && slot < 0;
        if (valid && slot >= 0) {
            const u64 rr = srec[slot];
            if ((rr >> 40) == len && w8_same(w, *reinterpret_cast<const uint4*>(&L.sw[slot][0]),
                                             *reinterpret_cast<const uint4*>(&L.sw[slot][4])) &&
                long_rest_same(a, p, rr & LLOG_OFF_MASK, (u32)len))
                atomicAdd((unsigned long long*)&scnt[slot], 1ull);
            else fallback = true;
        }
        if (fallback) {
            atomicAdd(&a.st->long_fb, 1u);
            ltab_add(a, len, tag, long_words(a, p, len, w), 1, true);
        }
        __syncthreads();                              // (as in k_long_agg: no slot of the next round
    }                                                 // is confused with this round's representatives)
    for (u32 s = tid; s < LS_SLOTS; s += LS_NT) {
        const u64 c = scnt[s];
        if (c == 0) continue;
        const u64 rr = srec[s], len = rr >> 40, p = rr & LLOG_OFF_MASK;
        const uint4 x = *reinterpret_cast<const uint4*>(&L.sw[s][0]), y = *reinterpret_cast<const uint4*>(&L.sw[s][4]);
        const u32 w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
        ltab_add(a, len, stag[s], long_words(a, p, len, w), c, false);
    }
}

// wave-local ordering of LDS accesses between lanes (the LDS executes one wave's
// instructions in order; this keeps the compiler from moving accesses across)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- prefetch registers: tagged asm loads per set (tools/check_inflight.py) and waits with a
//      quantised count (largest listed value <= n; n counts operations younger than the set)
// the quantised wait as ONE asm statement (a chain of scalar compares and branches around
// s_waitcnt): one asm keeps the set's registers in place (a chain of C++ branches, each with
// its own asm, makes the compiler merge their outputs through register copies)
#define WCG_W1(N, L) "s_cmp_ge_u32 %1, " #N "\n\ts_cbranch_scc0 " #L "f\n\ts_waitcnt vmcnt(" #N ")\n\ts_branch 99f\n" #L ":\n\t"
#ifndef WCG_WAIT_FIRST
#define WCG_WAIT_FIRST 1                     // try vmcnt(14) first (steady state: one compare); 0: the full chain
#endif
#if WCG_WAIT_FIRST
// steady state: n >= 14 (3 loads + >= 2 stores per step), so the first compare decides; vmcnt(14)
// leaves the last two steps' windows in flight (2 vs 4 sets in flight measured equal in r02)
#define WCG_WAIT_CHAIN(TAG)                                                                     \
    WCG_W1(14, 86) WCG_W1(12, 87) WCG_W1(10, 88) WCG_W1(8, 89) WCG_W1(6, 90) WCG_W1(4, 91)      \
    WCG_W1(2, 92) "s_waitcnt vmcnt(0)\n99: ; " TAG
#else
#define WCG_WAIT_CHAIN(TAG)                                                                     \
    WCG_W1(48, 81) WCG_W1(36, 82) WCG_W1(28, 83) WCG_W1(22, 84) WCG_W1(18, 85) WCG_W1(14, 86)   \
    WCG_W1(12, 87) WCG_W1(10, 88) WCG_W1(8, 89) WCG_W1(6, 90) WCG_W1(4, 91) WCG_W1(2, 92)        \
    "s_waitcnt vmcnt(0)\n99: ; " TAG
#endif
#define WCG_SET_OPS(S)                                                                          \
    __device__ __forceinline__ void set_load_##S(v4i rsrc, u32 om, v4u& m) {                    \
        /* s_nop 4: the descriptor SGPRs may have just been written by a VALU readfirstlane */    \
        asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, 0 offen ; wcg-load " #S "0"    \
                     : "=&v"(m) : "v"(om), "s"(rsrc) : "memory");                               \
    }                                                                                           \
    template <int N>                                                                            \
    __device__ __forceinline__ void set_wait_n_##S(v4u& m) {                                    \
        asm volatile("s_waitcnt vmcnt(%1) ; wcg-wait " #S " %0" : "+v"(m) : "n"(N) : "memory"); \
    }                                                                                           \
    __device__ __forceinline__ void set_wait_##S(u32 n, v4u& m) {                               \
        asm volatile(WCG_WAIT_CHAIN("wcg-wait " #S " %0") : "+v"(m) : "s"(n) : "memory", "scc"); \
    }

WCG_SET_OPS(A)
WCG_SET_OPS(B)
WCG_SET_OPS(C)
WCG_SET_OPS(D)
#undef WCG_SET_OPS
static_assert(MAP_SETS == 2 || MAP_SETS == 4, "k_map's main loop names two or four register sets");

// one miss-log unit store issued by the whole wave (lanes without a unit pass an out-of-range
// offset: the buffer range check drops the write); counted by the prefetch accounting
#ifndef WCG_DIAG_NOSTORE
#define WCG_DIAG_NOSTORE 0                   // diagnostics: 1 = no miss-log stores (wrong counts)
#endif
__device__ __forceinline__ void unit_store(v4i rsrc, u32 off, u64 v) {
    if (WCG_DIAG_NOSTORE) { asm volatile("; wcg-nostore" :: "v"(v), "v"(off), "s"(rsrc) : "memory"); return; }
    asm volatile("buffer_store_dwordx2 %0, %1, %2, 0 offen ; wcg-store" :: "v"(v), "v"(off), "s"(rsrc) : "memory");
}
constexpr u32 OOB = 0xFFFFFFF0u;

// inclusive prefix sum over the 64 lanes by DPP: within rows (row_shr 1-3 of the input, then
// row_shr 4 / 8 on banks 1-3 / 2-3), then across rows (row_bcast 15 / 31)
__device__ __forceinline__ u32 wave_incl_scan(u32 x) {
    u32 s = x + (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true)
              + (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true)
              + (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x113, 0xF, 0xF, true);
    s += (u32)__builtin_amdgcn_update_dpp(0, (int)s, 0x114, 0xF, 0xE, true);
    s += (u32)__builtin_amdgcn_update_dpp(0, (int)s, 0x118, 0xF, 0xC, true);
    s += (u32)__builtin_amdgcn_update_dpp(0, (int)s, 0x142, 0xA, 0xF, false);
    s += (u32)__builtin_amdgcn_update_dpp(0, (int)s, 0x143, 0xC, 0xF, false);
    return s;
}

// ABL (measurement builds only, selected by WCG_MAP_ABLATE; results are wrong when ABL != 0):
//   5 = input loads only, 4 = + LDS staging and letter masks, 1 = + token starts and compaction,
//   2 = + the per-step decode of both lists' first tokens, 3 = + the short-key iterations' probes
//   and decodes (no table update, no miss; medium iterations in full); 6 = full but long
//   tokens only counted, 7 = full but long tokens only measured and hashed
// ---- r04: the letter mask of a wave's window with non-ASCII bytes, by a wave-wide list of the
//      UTF-8 leads.  The lead-compacted form (utf8_mask_lds) decodes eight lead slots per lane,
//      so a wave pays max-over-lanes (8 on C4: ~615 VALU per step, half of k_map's time there);
//      here every lane lists its leads (window offsets, in the start list's LDS, which is built
//      later), then the wave decodes the list 64 leads per iteration (C4: ~250 leads per step)
//      from the staged window bytes, and each letter's span is OR-ed into its owner's mask word
//      in LDS (bits past the chunk into the next lane's word: the carry the DPP step makes).
//      The same decode as utf8_mask_lds (Go's utf8.DecodeRune: continuation bytes, overlongs,
//      surrogates, > U+10FFFF), continuation bytes tested in the decoded word itself.
#ifndef WCG_UTF8_LIST
#define WCG_UTF8_LIST 1
#endif
#ifndef WCG_UL_K
#define WCG_UL_K 1
#endif
#ifndef WCG_UL_MASKED
#define WCG_UL_MASKED 0                      // pipelined rounds: exec-masked block-id / bits reads
#endif
#ifndef WCG_UL_PIPE
#define WCG_UL_PIPE 1                        // r06: pipelined rounds (UL_K = 1 only)
#endif
static_assert(!WCG_UL_PIPE || WCG_UL_K == 1, "the pipelined decode rounds take one lead per lane");
constexpr int UL_K = WCG_UL_K;                // leads per lane per decode round (C4 k_map: 1 2.01-2.03 ms,
                                              // 2 2.11, 4 2.29-2.31: the rounds past the list's end
                                              // decode nothing at full VALU cost; 8 slots 2.04-2.06)
__device__ __forceinline__ u32 utf8_mask_list(uint4 c, u32 nx, LdsLetters lt, const uint8_t* bytes, uint16_t* list,
                                              uint16_t* wm, u32 lane) {
    u32 m = (ascii_mask4(c.x & 0x7F7F7F7Fu) & ~high_mask4(c.x)) |
            ((ascii_mask4(c.y & 0x7F7F7F7Fu) & ~high_mask4(c.y)) << 4) |
            ((ascii_mask4(c.z & 0x7F7F7F7Fu) & ~high_mask4(c.z)) << 8) |
            ((ascii_mask4(c.w & 0x7F7F7F7Fu) & ~high_mask4(c.w)) << 12);
    const u32 cont = cont_mask4(c.x) | (cont_mask4(c.y) << 4) | (cont_mask4(c.z) << 8) |
                     (cont_mask4(c.w) << 12) | (cont_mask4(nx) << 16);   // bit j: byte j
    u32 L = (lead_mask4(c.x) | (lead_mask4(c.y) << 4) | (lead_mask4(c.z) << 8) | (lead_mask4(c.w) << 12)) &
            (cont >> 1);                      // <= 8 per chunk (a lead's next byte is no lead)
#ifdef WCG_UL_ABL
    if (WCG_UL_ABL >= 2) L = 0;               // diagnostics (wrong masks): no lead list
#endif
    const u32 nl = (u32)__popc(L);
    const u32 incl = wave_incl_scan(nl);
    const u32 tot = (u32)__builtin_amdgcn_readlane((int)incl, 63);
    u32 o = incl - nl;
    wm[lane] = (uint16_t)m;
    while (L) {
        list[o++] = (uint16_t)(16 * lane + (u32)__builtin_ctz(L));
        L &= L - 1;
    }
    wave_lds_sync();
    u32* const wm32 = reinterpret_cast<u32*>(wm);
#ifdef WCG_UL_ABL
    if (WCG_UL_ABL >= 1) return wm[lane] | (tot & 0x10000u);   // diagnostics (wrong masks): no decode
#endif
#if WCG_UL_PIPE
    // r06: the rounds software-pipelined (one lead per lane per round): round r + 1's list entry
    // and bytes are read while round r is decoded and looked up, so a round's dependent chain is
    // two LDS round trips (block id, letter bits) instead of four (+ the list entry and the
    // bytes).  C4: the rounds were 0.70 ms of k_map's 1.94 (r06_experiments, WCG_UL_ABL)
    if (tot) {
        auto entry = [&](u32 base) -> u32 { return list[(base + lane) & (MAP_SST - 1)]; };
        auto pos = [&](u32 base, u32 e) -> u32 { return base + lane < tot ? e & (MAP_WIN - 1) : 0u; };
        auto word = [&](u32 q0) -> u32 {
            const u32* q = reinterpret_cast<const u32*>(bytes + (q0 & ~3u));
            return __builtin_amdgcn_alignbyte(q[1], q[0], q0 & 3u);
        };
        u32 p = pos(0, entry(0));
        u32 wd = word(p);
        for (u32 base = 0; base < tot; base += 64) {
            const u32 en = entry(base + 64);              // the next round's entry (unused past tot)
            __builtin_amdgcn_sched_barrier(0);
            const bool act = base + lane < tot;
            const u32 room = (u32)MAP_WIN - p;            // bytes past the window read as 0
            const u32 x0 = wd & (room >= 4 ? 0xFFFFFFFFu : (1u << (8 * room)) - 1u);
            const u32 b0 = x0 & 0xFFu;                    // C2-F4 (a listed lead)
            const u32 w = __builtin_clz(~(x0 << 24));     // 2-4
            const u32 need = (0xFFFFFFFFu >> ((32 - 8 * w) & 31)) & 0xFFFFFF00u;   // bytes 1..w-1
            const bool conts = (((x0 & 0xC0C0C0C0u) ^ 0x80808080u) & need) == 0u;
            const u32 x = ((b0 & (0x7Fu >> (w & 31))) << 18) | ((x0 << 4) & 0x3F000u) | ((x0 >> 10) & 0xFC0u) |
                          ((x0 >> 24) & 0x3Fu);
            const u32 v = x >> ((24 - 6 * w) & 31);
            const bool ok = act & conts & ((v >> ((5 * w - 4) & 31)) != 0u) & (v - 0xD800u >= 0x800u) &
                            (v <= 0x10FFFFu);
            const u32 cp = ok ? v : 0u;
            const u32 b = cp >> 8;
#if WCG_UL_MASKED
            // only the lanes that need them read the block id (3- and 4-byte runes) and the bits
            // (a letter candidate): fewer lanes in the random-address LDS reads
            u32 t = 0;
            if (b >= 8) t = lt.idx[b < LT_LDS_BLOCKS ? b : LT_LDS_BLOCKS];
#else
            const u32 t = lt.idx[b < LT_LDS_BLOCKS ? b : LT_LDS_BLOCKS];
#endif
            __builtin_amdgcn_sched_barrier(0);
            const u32 pn = pos(base + 64, en);             // the next round's bytes, read behind the
            const u32 wdn = word(pn);                      // block id
            __builtin_amdgcn_sched_barrier(0);
#if WCG_UL_MASKED
            u32 bits = 0;
            if (cp) bits = lt.bits[(b < 8 ? b : t) * 8 + ((cp >> 5) & 7)];
#else
            const u32 bits = lt.bits[(b < 8 ? b : t) * 8 + ((cp >> 5) & 7)];
#endif
            __builtin_amdgcn_sched_barrier(0);
            if ((bits >> (cp & 31)) & 1u) {
                const u32 own = p >> 4;
                const u32 span = __builtin_amdgcn_ubfe(0xFFFFFFFFu, 0, w & 31) << (p & 15u);
                atomicOr(&wm32[own >> 1], (span & 0xFFFFu) << (16 * (own & 1)));
                if ((span >> 16) && own < 63)                  // into the next chunk's word
                    atomicOr(&wm32[(own + 1) >> 1], (span >> 16) << (16 * ((own + 1) & 1)));
            }
            p = pn;
            wd = wdn;
        }
    }
#else
    // UL_K leads per lane per round, each stage's LDS reads issued together (one round trip per
    // stage, not per lead: the list entry, the bytes, the block id, the letter bits)
    for (u32 base = 0; base < tot; base += 64 * UL_K) {
        u32 p[UL_K], wd[UL_K], cp[UL_K], w[UL_K], t[UL_K], bits[UL_K];
#pragma unroll
        for (int k = 0; k < UL_K; k++) {           // past the list: position 0 (decodes as no letter)
            const u32 e = list[(base + 64 * k + lane) & (MAP_SST - 1)];
            p[k] = base + 64 * k + lane < tot ? e & (MAP_WIN - 1) : 0u;
        }
#pragma unroll
        for (int k = 0; k < UL_K; k++) {
            const u32* q = reinterpret_cast<const u32*>(bytes + (p[k] & ~3u));
            wd[k] = __builtin_amdgcn_alignbyte(q[1], q[0], p[k] & 3u);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < UL_K; k++) {
            const bool act = base + 64 * k + lane < tot;
            const u32 room = (u32)MAP_WIN - p[k];              // bytes past the window read as 0
            const u32 x0 = wd[k] & (room >= 4 ? 0xFFFFFFFFu : (1u << (8 * room)) - 1u);
            const u32 b0 = x0 & 0xFFu;                         // C2-F4 (a listed lead)
            w[k] = __builtin_clz(~(x0 << 24));                 // 2-4
            const u32 need = (0xFFFFFFFFu >> ((32 - 8 * w[k]) & 31)) & 0xFFFFFF00u;   // bytes 1..w-1
            const bool conts = (((x0 & 0xC0C0C0C0u) ^ 0x80808080u) & need) == 0u;
            const u32 x = ((b0 & (0x7Fu >> (w[k] & 31))) << 18) | ((x0 << 4) & 0x3F000u) | ((x0 >> 10) & 0xFC0u) |
                          ((x0 >> 24) & 0x3Fu);
            const u32 v = x >> ((24 - 6 * w[k]) & 31);
            const bool ok = act & conts & ((v >> ((5 * w[k] - 4) & 31)) != 0u) & (v - 0xD800u >= 0x800u) &
                            (v <= 0x10FFFFu);
            cp[k] = ok ? v : 0u;
        }
#pragma unroll
        for (int k = 0; k < UL_K; k++) {
            const u32 b = cp[k] >> 8;
            t[k] = lt.idx[b < LT_LDS_BLOCKS ? b : LT_LDS_BLOCKS];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < UL_K; k++) {
            const u32 b = cp[k] >> 8;
            bits[k] = lt.bits[(b < 8 ? b : t[k]) * 8 + ((cp[k] >> 5) & 7)];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < UL_K; k++) {
            if (!((bits[k] >> (cp[k] & 31)) & 1u)) continue;
            const u32 own = p[k] >> 4;
            const u32 span = __builtin_amdgcn_ubfe(0xFFFFFFFFu, 0, w[k] & 31) << (p[k] & 15u);
            atomicOr(&wm32[own >> 1], (span & 0xFFFFu) << (16 * (own & 1)));
            if ((span >> 16) && own < 63)                      // into the next chunk's word
                atomicOr(&wm32[(own + 1) >> 1], (span >> 16) << (16 * ((own + 1) & 1)));
        }
    }
#endif
    wave_lds_sync();
    return wm[lane];
}

template <int ABL, bool SPLIT>
#if WCG_MAP_WGS > 1
// occupancy experiments (r06): 8 waves per SIMD also needs <= 80 SGPRs
#define WCG_MAP_ATTR __attribute__((amdgpu_waves_per_eu(4 * WCG_MAP_WGS * WCG_MAP_NT / 1024, 4 * WCG_MAP_WGS * WCG_MAP_NT / 1024)))
#else
#define WCG_MAP_ATTR
#endif
__global__ __launch_bounds__(MAP_NT, MAP_WGS * MAP_NT / 256) WCG_MAP_ATTR void k_map(MapArgs a) {
#if !WCG_DIRECT
    __shared__ __align__(16) uint8_t wbytes[MAP_WAVES][MAP_WREG];
    __shared__ __align__(16) uint16_t wstart[MAP_WAVES][MAP_SST];
#endif
    __shared__ __align__(4) uint16_t wmask[MAP_WAVES][64];   // chunk letter masks of the wave's window
    __shared__ __align__(16) u64 sk0[MAP_NS];
    __shared__ __align__(16) u64 mk0[MAP_NM];
    __shared__ __align__(16) u64 mk1[MAP_NM];
    __shared__ u64 zero_w;
    __shared__ u32 seen_w[WCG_ADMIT2 ? MapTable<MAP_NS, MAP_NM>::ADMIT_BITS / 32 : 1];
    __shared__ u32 scnt[MAP_NS];
    __shared__ u32 mcnt[MAP_NM];
    __shared__ u32 cursor[MAX_MISS_BUCKETS];
    __shared__ u32 lcur;                        // long-token log cursor
    __shared__ uint8_t lt_idx[LT_LDS_BLOCKS + 4];   // letter table (UTF-8 chunks)
    __shared__ u32 lt_bits[WCG_LT_NBLOCKS * 8];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);     // wave-uniform (scalar)
    MapTable<MAP_NS, MAP_NM> tab{sk0, scnt, mk0, mk1, mcnt, &zero_w, WCG_ADMIT2 ? seen_w : nullptr};
    tab.init(tid, MAP_NT);
    for (int i = tid; i < MAX_MISS_BUCKETS; i += MAP_NT) cursor[i] = 0;
    if (tid == 0) lcur = 0;
    lds_letters_init(lt_idx, lt_bits, tid, MAP_NT);
    __syncthreads();
    const LdsLetters lt{lt_idx, lt_bits};

#if !WCG_DIRECT
    uint8_t* const bytes = wbytes[wave];
    uint16_t* const sst = wstart[wave];
#endif
    u64 stp[MAP_NSTAMP] = {};                     // WCG_STAMPS: cycles per phase (wave-uniform)
    u64 t_last = WCG_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
    auto stamp = [&](int i) {
        if (WCG_STAMPS) { const u64 t = __builtin_amdgcn_s_memtime(); stp[i] += t - t_last; t_last = t; }
    };
    // Steps are dealt chip-wide: wave w of workgroup g takes steps (g * 16 + w) + k * G * 16, so
    // the chip sweeps the input front to back (HBM-friendly) while every workgroup still sees
    // a uniform sample of it for its LDS table.
    const u64 nsteps = a.ntiles;
    const u64 stride = (u64)gridDim.x * MAP_WAVES;
    // window chunk c <-> input bytes [step base - 16 + 16c, +16); lane c holds chunk c
    u64 my_tokens = 0;                           // wave-uniform (WCG_DIRECT: per lane)
    // token starts are owned by lanes 1-62 only (lane 0: the prefix chunk, 63: the look-ahead)
    const u32 own16 = (u32)(lane - 1) < (u32)MAP_OWN ? 0xFFFFu : 0u;
    u32 my_hits = 0, my_global = 0, my_long = 0;
    u64 hits_w = 0;                              // wave-uniform: hits counted from the hit masks (SALU)

    // miss-log stores of this workgroup: one buffer resource over its regions
    const u32 P = a.pmask + 1;
    u64* const wpool = a.pool + (u64)blockIdx.x * P * a.region_cap;
    const v4i prsrc = make_rsrc(wpool, (u32)(P * a.region_cap * 8));

    // Input loads: raw buffer loads through a per-step descriptor based at the window start
    // (at the input start for step 0, whose prefix chunk is out of range and reads zeros).
    // Every prefetch is unconditional: steps past the end load offset 0xFFFFFFF0, which reads
    // zeros without touching memory.
    auto addr = [&](u64 step, v4i& rsrc, u32& om) {
        const bool live = step < nsteps;
        const u64 org = (step == 0 || !live) ? 0 : step * MAP_STEP - 16;
        const u64 span = live ? a.n - org : 0;
        const u32 nrec = span > 0xFFFFFFFFull ? 0xFFFFFFFFu : (u32)span;
        rsrc = make_rsrc(a.in + org, nrec);
        const u32 rel = step == 0 ? 0u : 16u;
        om = live ? 16 * lane + rel - 16 : OOB;                  // step 0, lane 0: wraps to OOB
    };

#if !WCG_DIRECT
    // ---- token decoding.  An entry of the start list -> the key's bytes from aligned dword LDS
    //      reads (r03: dwords from rp & ~3, ds_read2_b32 pairs, so the word at rp is one alignbyte
    //      away; unaligned 8-byte LDS reads cost ~20x the LDS cycles), then the key identity of
    //      fact F4 with byte masks, and its LDS hash
    struct TokS { u64 k; u32 h; };                   // short key (<= 7 bytes): k0 alone
    struct TokM { u64 k0, k1; u32 h; bool valid; };  // medium key (8-15 bytes); long tokens: !valid
    // short key: its bytes lie in [rp & ~3, +12)
    auto keyread_s = [&](u32 e) -> uint3 {
        const u32* q = reinterpret_cast<const u32*>(bytes + ((e & ((1u << SST_LEN_SHIFT) - 1)) & ~3u));
        return make_uint3(q[0], q[1], q[2]);
    };
    auto decode_s = [&](u32 e, const uint3& kw) -> TokS {
        const u32 rp = e & ((1u << SST_LEN_SHIFT) - 1), len = e >> SST_LEN_SHIFT;
        const u32 bsh = rp & 3u;
        const u64 w = (u64)__builtin_amdgcn_alignbyte(kw.z, kw.y, bsh) << 32 | __builtin_amdgcn_alignbyte(kw.y, kw.x, bsh);
        TokS t;
        t.k = (w & ((1ull << (8 * len)) - 1)) | (u64)len << 56;
        t.h = lds_hash32((u32)t.k, (u32)(t.k >> 32), 0u, 0u);
        return t;
    };
    // medium key (or a long token's first 16 bytes): [rp & ~3, +20)
    struct KeyWords { u32 d0, d1, d2, d3, d4; };
    auto keyread = [&](u32 e) -> KeyWords {
        const u32* q = reinterpret_cast<const u32*>(bytes + ((e & ((1u << SST_LEN_SHIFT) - 1)) & ~3u));
        return KeyWords{q[0], q[1], q[2], q[3], q[4]};
    };
    // act: the entry is one of this step's tokens.  A long token (> 15 bytes) is measured and
    // logged here, while its step's window masks are in LDS (its TokM may be carried to the next
    // step), and takes no part in the table
    auto decode_m = [&](u32 e, bool act, const KeyWords& kw, long wbase) -> TokM {
        const u32 rp = e & ((1u << SST_LEN_SHIFT) - 1), len = e >> SST_LEN_SHIFT;
        const u32 bsh = rp & 3u;
        const u32 w0 = __builtin_amdgcn_alignbyte(kw.d1, kw.d0, bsh), w1 = __builtin_amdgcn_alignbyte(kw.d2, kw.d1, bsh);
        const u32 w2 = __builtin_amdgcn_alignbyte(kw.d3, kw.d2, bsh), w3 = __builtin_amdgcn_alignbyte(kw.d4, kw.d3, bsh);
        const u32 nb = len - 8;                            // bytes in k1: 0..7
        const u32 ml = nb >= 4 ? 0xFFFFFFFFu : (1u << (8 * nb)) - 1;
        const u32 mh = nb >= 4 ? (1u << ((8 * nb - 32) & 31)) - 1 : 0u;
        TokM t;
        const u32 k1l = w2 & ml, k1h = (w3 & mh) | (len << 24);
        t.k0 = (u64)w1 << 32 | w0;
        t.k1 = (u64)k1h << 32 | k1l;
        t.h = lds_hash32(w0, w1, k1l, k1h);
        t.valid = act && len < 16;
        if (act && len >= 16) {
            my_long++;
            if (ABL != 6) long_token_log<ABL>(a, (u64)(wbase + rp), rp, wmask[wave], &lcur);
        }
        return t;
    };

    // ---- carried tokens (r06).  A list's last, partial iteration is not run in its step: its
    //      tokens, already decoded, stay in registers (lanes [0, n)) and fill the first lanes of
    //      the next step's first iteration, whose list reads are shifted by n (entry i of a step's
    //      list goes to lane (n + i) % 64).  So every iteration but the wave's last two (the drain
    //      after the main loop) runs 64 tokens, and short keys never take the medium-key body (C2:
    //      2 short + 1 mixed iteration per step before, ~2.3 short + ~0.3 medium now)
    TokS cs{0, 0};
    TokM cm{0, 0, 0, false};
    u32 ncs = 0, ncm = 0;                 // carried short / medium tokens (wave-uniform)
    // A miss reserves its units with an LDS atomic whose result is read one iteration later (after
    // that iteration's probe reads have returned, so the reservation adds no round trip of its
    // own), and the wave stores them then: 1 unit store per short iteration, 2 per medium
    // iteration, 2 after a step's last medium iteration (prefetch accounting); a short miss may
    // stay pending across steps
    bool missp = false;                   // the pending miss: bucket, units, reservation and key
    u32 pp = 0, nup = 0, posp = 0;
    u64 k0p = 0, k1p = 0;
    const u32 rcap = (u32)a.region_cap;   // < 2^22 (host), so offsets fit 24-bit multiplies
    auto store_pending = [&](bool two) {
        const bool fits = missp && posp + nup <= rcap;
        const u32 o0 = fits ? (__umul24(pp, rcap) + posp) * 8u : OOB;
        unit_store(prsrc, o0, k0p);
        if (two) unit_store(prsrc, fits && nup == 2 ? o0 + 8u : OOB, k1p);
        if (missp && !fits) {             // region full: zero its tail, global table
            u64* r = wpool + (u64)pp * a.region_cap;
            for (u32 k = posp; k < rcap; k++) r[k] = 0;
            my_global++;
            ginsert(a.gtab, a.gmask, k0p, k1p, gslot(key_hash(k0p, k1p)), 1, a.st);
        }
    };
    auto miss_short = [&](bool miss, const TokS& t) {
        missp = miss;
        pp = short_bucket<SPLIT>(t.h);
        nup = 1u;
        posp = atomicAdd(&cursor[pp], miss ? 1u : 0u);   // every lane (0 = no miss)
        k0p = t.k; k1p = 0;
    };
    auto miss_medium = [&](bool miss, const TokM& t) {
        missp = miss;
        pp = medium_bucket<SPLIT>(t.h);
        nup = 2u;
        posp = atomicAdd(&cursor[pp], miss ? 2u : 0u);
        k0p = t.k0; k1p = t.k1;
    };

    // one step: returns the number of unit stores it issued (prefetch accounting)
    auto process = [&](u64 step, const uint4 mine) -> u32 {
        const long wbase = (long)(step * MAP_STEP) - 16;        // input offset of window byte 0
        if (ABL == 5) { asm volatile("" ::"v"(mine.x)); return 0; }
        reinterpret_cast<uint4*>(bytes)[lane] = mine;
        // ---- letter mask of the lane's chunk (lane 0: only bit 15 is used - the predecessor of
        //      the step's first byte; lane 63: only as the successor of chunk 62, and on the
        //      UTF-8 path its last 3 bits, whose runes may end past the window, are forced to
        //      letters, so a run reaching them is measured exactly by the long-token path)
        // the next chunk's first dword by DPP (all lanes active; lane 63 gets zeros)
        const u32 nx = (u32)__builtin_amdgcn_update_dpp(0, (int)mine.x, 0x130, 0xF, 0xF, false);   // wave_shl:1
        u32 m;
#if WCG_UTF8_LIST
        if (__ballot(!all_ascii(mine)) == 0) {
            m = ascii_mask16(mine);
        } else {
            m = utf8_mask_list(mine, nx, lt, bytes, sst, wmask[wave], lane);   // carries included
            if (lane == 63 && !all_ascii(mine)) m |= 0xE000u;
        }
#else
        if (all_ascii(mine)) {
            m = ascii_mask16(mine);
        } else {
            m = utf8_mask_lds(mine, nx, lt);
            if (lane == 63) m |= 0xE000u;
        }
#endif
        // bytes of this chunk covered by a letter rune that started in the previous chunk
        m = (m | ((u32)__builtin_amdgcn_update_dpp(0, (int)(m >> 16), 0x138, 0xF, 0xF, false) & 7u)) & 0xFFFFu;
        if (ABL == 4) { asm volatile("" ::"v"(m)); return 0; }
        wmask[wave][lane] = (uint16_t)m;
        stamp(2);
        // neighbours' masks by DPP lane shifts
        const u32 prevm = (u32)__builtin_amdgcn_update_dpp(0, (int)m, 0x138, 0xF, 0xF, false);   // wave_shr:1
        const u32 nextm = (u32)__builtin_amdgcn_update_dpp(0, (int)m, 0x130, 0xF, 0xF, false);   // wave_shl:1
        u32 starts = m & ~((m << 1) | (prevm >> 15)) & own16;
        const u32 w32 = m | (nextm << 16);
        // Start list, short keys (<= 7 bytes: 89% of C2 tokens) first, then the others: a start
        // whose letter run reaches 8 bytes has bits b..b+7 of w32 set.  Iterations over short
        // entries only run a short-key body (one key word, one table, no k1 reads).
        u32 r8 = w32 & (w32 >> 1);
        r8 &= r8 >> 2;
        r8 &= r8 >> 4;
        // both counts in one word (each <= 16 per lane, <= 496 per wave) and ONE wave-wide DPP
        // prefix sum for the lanes' list offsets (4 bit-plane ballots + mbcnt per count were ~4x
        // the VALU)
        const u32 packed = (u32)__popc(starts & ~r8) | (u32)__popc(starts & r8) << 16;
        const u32 incl = wave_incl_scan(packed);
        const u32 tot = (u32)__builtin_amdgcn_readlane((int)incl, 63);
        const u32 tot_s = tot & 0xFFFFu;
        const u32 total = tot_s + (tot >> 16);
        const u32 excl = incl - packed;
        const u32 o_s = excl & 0xFFFFu, o_o = (excl >> 16) + tot_s;
        // r06: the short starts and the others in two loops of straight-line slots (the k-th
        // start of a lane goes to its list offset + k, an immediate store offset), each ending
        // when no lane has a start left.  One loop over all starts picked the list and bumped
        // two offsets per start: 15 VALU per iteration against 9 here, for max(all) = 4.2
        // iterations per step against max(short) + max(other) = 4.2 + 1.6 (C2)
        const u32 lbase = 16 * lane;
        auto list = [&](uint16_t* w, u32 msk, bool shrt) {
#pragma unroll
            for (int k = 0; k < 8; k++) {                   // <= 8 starts per 16-byte chunk
                if (__ballot(msk != 0) == 0) break;
                if (msk) {
                    const u32 b = __builtin_ctz(msk);
                    msk &= msk - 1;
                    const u32 run = __builtin_ctz(~(w32 >> b));   // >= 1; 32 - b when the window is all letters
                    const u32 len = shrt ? run : (run < 16 ? run : 16u);   // 16 = long token (> 15 bytes)
                    w[k] = (uint16_t)((lbase + b) | (len << SST_LEN_SHIFT));
                }
            }
        };
        list(sst + o_s, starts & ~r8, true);
        list(sst + o_o, starts & r8, false);
        wave_lds_sync();
        stamp(3);
        my_tokens += total;
        if (ABL == 1) return 0;

        // ---- tokens: uniform iterations of 64 tokens, the short list first, then the medium/long
        //      one, each software-pipelined so that one LDS round trip per iteration carries this
        //      token's table probe, the next token's key bytes and the entry after that; decodes
        //      past a list's end are unconditional (entries read other LDS words, key reads stay
        //      inside the wave's staging bytes) and only the carried lanes' ones are used
        const u32 ts = tot_s, tm = tot >> 16;
        const u32 ns = ncs + ts, nfs = ns >> 6;          // short tokens; full iterations
        const u32 nm = ncm + tm, nfm = nm >> 6;          // medium/long tokens; full iterations
        const u32 ls = (u32)lane - ncs;                  // iteration 0's short entry (wraps for carried lanes)
        const u32 lm = (u32)lane - ncm;
        // entry i of an iteration's lane: ps[64 * i] / pm[64 * i] (the carried lanes of iteration
        // 0 and the lanes past a list's end read other LDS words of the workgroup: unused)
        const uint16_t* const ps = sst + (int)ls;
        const uint16_t* const pm = sst + (int)(ts + lm);
        // both lists' first entries and key bytes in one round trip each
        const u32 es0 = ps[0], em0 = pm[0];
        u32 e_nxt = ps[64], f_nxt = pm[64];
        {
            const uint3 kws = keyread_s(es0);
            const KeyWords kwm = keyread(em0);
            const TokS t = decode_s(es0, kws);
            const TokM u = decode_m(em0, lm < tm, kwm, wbase);
            if ((u32)lane >= ncs) cs = t;
            if ((u32)lane >= ncm) cm = u;
        }
        stamp(4);
        if (ABL == 2) { asm volatile("" ::"v"(cs.h), "v"(cm.h), "v"(e_nxt), "v"(f_nxt)); ncs = ns & 63; ncm = nm & 63; return 0; }
        for (u32 it = 0; it < nfs; it++) {
            const auto pr = tab.probe_short(cs.h);
            const uint3 nks = keyread_s(e_nxt);
            const u32 e_nn = ps[64 * (it + 2)];
            __builtin_amdgcn_sched_barrier(0);  // all three reads issue before the probe's wait
            if (ABL == 3) {                   // probe reads and decodes, no table update or miss
                asm volatile("" ::"v"(pr.x1), "v"(pr.x2));
                cs = decode_s(e_nxt, nks);
                e_nxt = e_nn;
                continue;
            }
            const bool hit = tab.finish_short(cs.k, cs.h, pr);
            hits_w += (u64)__popcll(__ballot(hit));
            store_pending(false);             // short keys: one unit
            miss_short(!hit, cs);
            cs = decode_s(e_nxt, nks);
            e_nxt = e_nn;
        }
        ncs = ns & 63;
        for (u32 it = 0; it < nfm; it++) {
            const auto pr = tab.probe(true, cm.h);
            const KeyWords nkw = keyread(f_nxt);
            const u32 f_nn = pm[64 * (it + 2)];
            __builtin_amdgcn_sched_barrier(0);
            const bool hit = tab.finish(cm.valid, true, cm.k0, cm.k1, cm.h, pr);
            hits_w += (u64)__popcll(__ballot(hit));
            store_pending(true);              // the previous iteration's miss units
            miss_medium(cm.valid && !hit, cm);
            cm = decode_m(f_nxt, lm + 64 * (it + 1) < tm, nkw, wbase);
            f_nxt = f_nn;
        }
        ncm = nm & 63;
        u32 nst = nfs + 2 * nfm;
        if (nfm) {                            // a medium miss does not stay pending (a short
            store_pending(true);              // iteration stores one unit)
            missp = false;
            nst += 2;
        }
        wave_lds_sync();
        stamp(5);
        if (WCG_STAMPS) stp[6]++;
        return nst;
    };

#else
    // ---- one step without a start list.  Every owner lane counts the tokens that start in its
    //      own 16-byte chunk, one token per lane per iteration: the short keys (<= 7 bytes, the
    //      k0 word alone) in a first pass, the others in a second.  A token of <= 15 bytes lies in
    //      the lane's chunk and the next one, so its key bytes come from registers (the next
    //      chunk's four dwords by DPP): no staging of the window in LDS, no compacted start list
    //      and no key reads from LDS - a step's only LDS traffic is the table.  Within a pass the
    //      next token's key is extracted and its probe issued before this token's probe is
    //      finished, so two probes are in flight per lane.  A pass runs as many iterations as
    //      the lane with the most such starts has (C2: 4.2 per step for all starts).
    struct TokS { u64 k; u32 h; };
    struct TokG { u64 k0, k1; u32 h; bool lng; };
    auto process = [&](u64 step, const uint4 mine) -> u32 {
        const long wbase = (long)(step * MAP_STEP) - 16;        // input offset of window byte 0
        // the next chunk's dwords by DPP wave_shl:1 (all lanes active; lane 63 gets zeros)
        const u32 D0 = mine.x, D1 = mine.y, D2 = mine.z, D3 = mine.w;
        const u32 D4 = (u32)__builtin_amdgcn_update_dpp(0, (int)mine.x, 0x130, 0xF, 0xF, false);
        const u32 D5 = (u32)__builtin_amdgcn_update_dpp(0, (int)mine.y, 0x130, 0xF, 0xF, false);
        const u32 D6 = (u32)__builtin_amdgcn_update_dpp(0, (int)mine.z, 0x130, 0xF, 0xF, false);
        const u32 D7 = (u32)__builtin_amdgcn_update_dpp(0, (int)mine.w, 0x130, 0xF, 0xF, false);
        // ---- letter mask of the lane's chunk (as the list path: SWAR on ASCII, Go UTF-8 decode
        //      + letter table otherwise; lane 63's last 3 bits forced to letters on that path)
        u32 m;
        if (all_ascii(mine)) {
            m = ascii_mask16(mine);
        } else {
            m = utf8_mask_lds(mine, D4, lt);
            if (lane == 63) m |= 0xE000u;
        }
        m = (m | ((u32)__builtin_amdgcn_update_dpp(0, (int)(m >> 16), 0x138, 0xF, 0xF, false) & 7u)) & 0xFFFFu;
        wmask[wave][lane] = (uint16_t)m;                      // read by long tokens only
        const u32 prevm = (u32)__builtin_amdgcn_update_dpp(0, (int)m, 0x138, 0xF, 0xF, false);   // wave_shr:1
        const u32 nextm = (u32)__builtin_amdgcn_update_dpp(0, (int)m, 0x130, 0xF, 0xF, false);   // wave_shl:1
        const bool owner = lane >= 1 && lane <= MAP_OWN;
        const u32 starts = owner ? (m & ~((m << 1) | (prevm >> 15)) & 0xFFFFu) : 0u;
        const u32 w32 = m | (nextm << 16);
        u32 r8 = w32 & (w32 >> 1);                            // bit b: bytes b..b+7 all letters
        r8 &= r8 >> 2;
        r8 &= r8 >> 4;
        u32 ss = starts & ~r8, so = starts & r8;
        my_tokens += (u32)__popc(starts);
        wave_lds_sync();                                      // wmask before the long tokens' reads
        // the first set start of msk (false: none left), removed from msk
        auto next_start = [](u32& msk, u32& b) -> bool {
            const bool v = msk != 0;
            b = v ? (u32)__builtin_ctz(msk) : 0u;
            msk &= msk - 1;
            return v;
        };
        // window dwords e_k = D[d + k], d = b >> 2 (two levels of selects)
        auto sel = [&](u32 b, u32 (&e)[5], int n) {
            const bool s0 = (b & 4u) != 0, s1 = (b & 8u) != 0;
            const u32 P0 = s0 ? D1 : D0, P1 = s0 ? D2 : D1, P2 = s0 ? D3 : D2, P3 = s0 ? D4 : D3;
            const u32 P4 = s0 ? D5 : D4;
            e[0] = s1 ? P2 : P0; e[1] = s1 ? P3 : P1; e[2] = s1 ? P4 : P2;
            if (n > 3) {
                const u32 P5 = s0 ? D6 : D5, P6 = s0 ? D7 : D6;
                e[3] = s1 ? P5 : P3; e[4] = s1 ? P6 : P4;
            }
        };
        auto short_at = [&](u32 b) -> TokS {
            const u32 len = (u32)__builtin_ctz(~(w32 >> b));   // 1..7 for a short start
            u32 e[5];
            sel(b, e, 3);
            const u32 bs = b & 3u;
            const u64 w = (u64)__builtin_amdgcn_alignbyte(e[2], e[1], bs) << 32 | __builtin_amdgcn_alignbyte(e[1], e[0], bs);
            TokS t;
            t.k = (w & ((1ull << (8 * len)) - 1)) | (u64)len << 56;
            t.h = lds_hash32((u32)t.k, (u32)(t.k >> 32), 0u, 0u);
            return t;
        };
        auto gen_at = [&](u32 b) -> TokG {
            const u32 run = (u32)__builtin_ctz(~(w32 >> b));   // >= 8; 32 - b if all letters
            const u32 len = run < 16 ? run : 16u;              // 16 = long token (> 15 bytes)
            u32 e[5];
            sel(b, e, 5);
            const u32 bs = b & 3u;
            const u32 w0 = __builtin_amdgcn_alignbyte(e[1], e[0], bs), w1 = __builtin_amdgcn_alignbyte(e[2], e[1], bs);
            const u32 w2 = __builtin_amdgcn_alignbyte(e[3], e[2], bs), w3 = __builtin_amdgcn_alignbyte(e[4], e[3], bs);
            const u32 nb = len - 8;                            // bytes in k1: 0..7 (8 for a long token)
            const u32 ml = nb >= 4 ? 0xFFFFFFFFu : (1u << (8 * nb)) - 1;
            const u32 mh = nb >= 8 ? 0xFFFFFFFFu : (nb >= 4 ? (1u << (8 * nb - 32)) - 1 : 0u);
            TokG t;
            t.k0 = (u64)w1 << 32 | w0;
            t.k1 = (u64)((w3 & mh) | (len << 24)) << 32 | (w2 & ml);
            t.lng = len >= 16;
            t.h = lds_hash32(w0, w1, (u32)t.k1, (u32)(t.k1 >> 32));
            return t;
        };

        // miss-log units: a miss reserves its units with an LDS atomic whose result is read one
        // iteration later, and the wave stores them then (1 store per short iteration, 2 per
        // other iteration, 2 at the end: the prefetch accounting)
        bool missp = false;
        u32 pp = 0, nup = 0, posp = 0;
        u64 k0p = 0, k1p = 0;
        const u32 rcap = (u32)a.region_cap;   // < 2^22 (host), so offsets fit 24-bit multiplies
        auto store_pending = [&](bool two) {
            const bool fits = missp && posp + nup <= rcap;
            const u32 o0 = fits ? (__umul24(pp, rcap) + posp) * 8u : OOB;
            unit_store(prsrc, o0, k0p);
            if (two) unit_store(prsrc, fits && nup == 2 ? o0 + 8u : OOB, k1p);
            if (missp && !fits) {             // region full: zero its tail, global table
                u64* r = wpool + (u64)pp * a.region_cap;
                for (u32 k = posp; k < rcap; k++) r[k] = 0;
                my_global++;
                ginsert(a.gtab, a.gmask, k0p, k1p, gslot(key_hash(k0p, k1p)), 1, a.st);
            }
        };
        u32 n_s = 0, n_o = 0;
        // Each pass is unrolled by two with fixed roles (token A, token B): a loop-carried copy of
        // a probe's result registers would wait for its reads (lgkmcnt) before the next probe
        // is issued, which is exactly the overlap the pipeline is for.
        // ---- short keys
        {
            auto finish_s = [&](bool v, const TokS& t, const typename decltype(tab)::ProbeS& pr) {
                const bool hit = tab.finish_short_v(v, t.k, t.h, pr);
                my_hits += (u32)hit;
                store_pending(false);
                missp = v && !hit;
                pp = short_bucket<SPLIT>(t.h);
                nup = 1u;
                posp = atomicAdd(&cursor[pp], missp ? 1u : 0u);
                k0p = t.k; k1p = 0;
                n_s++;
            };
            u32 bA, bB;
            bool vA = next_start(ss, bA), vB;
            TokS A = short_at(bA), B;
            auto prA = tab.probe_short(A.h);
            decltype(prA) prB;
            while (__ballot(vA)) {
                vB = next_start(ss, bB);
                B = short_at(bB);
                prB = tab.probe_short(B.h);
                __builtin_amdgcn_sched_barrier(0);            // B's probe reads issue before A's wait
                finish_s(vA, A, prA);
                if (!__ballot(vB)) break;
                vA = next_start(ss, bA);
                A = short_at(bA);
                prA = tab.probe_short(A.h);
                __builtin_amdgcn_sched_barrier(0);
                finish_s(vB, B, prB);
            }
        }
        // ---- medium (8-15 bytes) and long keys
        {
            auto finish_g = [&](bool v, u32 b, const TokG& t, const typename decltype(tab)::Probe& pr) {
                if (v && t.lng) {
                    my_long++;
                    const u32 rp = 16 * lane + b;
                    long_token_log<ABL>(a, (u64)(wbase + rp), rp, wmask[wave], &lcur);
                }
                const bool val = v && !t.lng;
                const bool hit = tab.finish(val, true, t.k0, t.k1, t.h, pr);
                my_hits += (u32)hit;
                store_pending(true);
                missp = val && !hit;
                pp = medium_bucket<SPLIT>(t.h);
                nup = 2u;
                posp = atomicAdd(&cursor[pp], missp ? 2u : 0u);
                k0p = t.k0; k1p = t.k1;
                n_o++;
            };
            u32 bA, bB;
            bool vA = next_start(so, bA), vB;
            TokG A = gen_at(bA), B;
            auto prA = tab.probe(true, A.h);
            decltype(prA) prB;
            while (__ballot(vA)) {
                vB = next_start(so, bB);
                B = gen_at(bB);
                prB = tab.probe(true, B.h);
                __builtin_amdgcn_sched_barrier(0);
                finish_g(vA, bA, A, prA);
                if (!__ballot(vB)) break;
                vA = next_start(so, bA);
                A = gen_at(bA);
                prA = tab.probe(true, A.h);
                __builtin_amdgcn_sched_barrier(0);
                finish_g(vB, bB, B, prB);
            }
        }
        store_pending(true);
        wave_lds_sync();
        if (WCG_STAMPS) stp[6]++;
        return n_s + 2 * n_o + 2;
    };
#endif

    // ---- main loop, unrolled over the register sets so that each set's load and waits name
    //      fixed registers (tools/check_inflight.py); a set's load was issued MAP_SETS steps
    //      earlier; h1..h3 = unit stores of the last three steps (the wait count)
    auto is_tail = [&](u64 step) { return step * MAP_STEP - 16 + MAP_WIN > a.n; };
    auto u4 = [](v4u v) { return make_uint4(v.x, v.y, v.z, v.w); };
    v4u mA, mB, mC, mD;
    u64 st = (u64)blockIdx.x * MAP_WAVES + wave;
    {
        v4i r; u32 om;
        addr(st, r, om);              set_load_A(r, om, mA);
        addr(st + stride, r, om);     set_load_B(r, om, mB);
        if (MAP_SETS == 4) {
            addr(st + 2 * stride, r, om); set_load_C(r, om, mC);
            addr(st + 3 * stride, r, om); set_load_D(r, om, mD);
        }
    }
    u32 h1 = 0, h2 = 0, h3 = 0;
#define WCG_MAP_STEP(S)                                                                         \
    {                                                                                           \
        if (st >= nsteps || is_tail(st)) break;                                                 \
        v4i r; u32 om;                                                                          \
        addr(st + MAP_SETS * stride, r, om);                                                    \
        stamp(0);                                                                               \
        if (WCG_NOWAIT) set_wait_##S(63, m##S); /* diagnostics only: results are wrong */       \
        else if (WCG_WAIT0) set_wait_##S(0, m##S);                                              \
        else set_wait_##S((MAP_SETS - 1) + h1 + (MAP_SETS == 4 ? h2 + h3 : 0), m##S);           \
        stamp(1);                                                                               \
        const u32 it_ = process(st, u4(m##S));                                                  \
        set_load_##S(r, om, m##S);                                                              \
        h3 = h2; h2 = h1; h1 = it_;                                                             \
        st += stride;                                                                           \
    }
    while (true) {
        WCG_MAP_STEP(A)
        WCG_MAP_STEP(B)
#if WCG_MAP_SETS == 4
        WCG_MAP_STEP(C)
        WCG_MAP_STEP(D)
#endif
    }
#undef WCG_MAP_STEP
    set_wait_n_A<0>(mA);                  // nothing may land in a dead register
    set_wait_n_B<0>(mB);
    if (MAP_SETS == 4) {
        set_wait_n_C<0>(mC);
        set_wait_n_D<0>(mD);
    }
    for (; st < nsteps; st += stride)     // tail steps: byte-exact reloads
        process(st, load_chunk(a.in, a.n, (long)(st * MAP_STEP) - 16 + 16 * lane));
#if !WCG_DIRECT
    if (ABL == 0 || ABL >= 6) {           // the carried partial iterations
        const auto pr = tab.probe_short(cs.h);
        const auto pm = tab.probe(true, cm.h);
        const bool vs = (u32)lane < ncs;
        const bool hs = tab.finish_short_v(vs, cs.k, cs.h, pr);
        const bool hm = tab.finish(cm.valid, true, cm.k0, cm.k1, cm.h, pm);
        my_hits += (u32)hs + (u32)hm;
        store_pending(false);             // pending: a short miss or none
        miss_short(vs && !hs, cs);
        store_pending(false);
        miss_medium(cm.valid && !hm, cm);
        store_pending(true);
    }
#endif

    if (WCG_STAMPS && lane == 0)
        for (int i = 0; i < MAP_NSTAMP; i++) atomicAdd((unsigned long long*)&a.stamps[i], (unsigned long long)stp[i]);
    // ---- flush the LDS table into this workgroup's miss-log regions (entries with counts);
    //      a full region -> global table
    __syncthreads();
    auto flush = [&](u64 k0, u64 k1, u32 c) {
        if (!c) return;
        const u32 h = lds_hash(k0, k1);
        if (!log_push(a, cursor, key_short(k0) ? short_bucket<SPLIT>(h) : medium_bucket<SPLIT>(h), k0, k1, c)) {
            my_global++;
            ginsert(a.gtab, a.gmask, k0, k1, gslot(key_hash(k0, k1)), c, a.st);
        }
    };
    for (int i = tid; i < MAP_NS; i += MAP_NT) flush(sk0[i], 0, scnt[i]);
    for (int i = tid; i < MAP_NM; i += MAP_NT) flush(mk0[i], mk1[i], mcnt[i]);
    __syncthreads();
    if (tid == 0) a.llog_len[blockIdx.x] = lcur < a.llog_cap ? lcur : a.llog_cap;
    for (u32 p = tid; p <= a.pmask; p += MAP_NT) {
        const u32 c = cursor[p];
        a.region_len[(u64)blockIdx.x * (a.pmask + 1) + p] = c < a.region_cap ? c : (u32)a.region_cap;
    }
    // stats: per-workgroup partial sums with plain stores (k_agg's first workgroup adds them
    // to DevState).  Per-wave atomics on DevState cost ~12 ns each serialised on one line:
    // 16K of them added 0.2 ms to every launch.
    __shared__ u64 wsum[MAP_WAVES][4];
    u64 v0 = (WCG_DIRECT || lane == 0) ? my_tokens : 0, v1 = my_hits + (lane == 0 ? hits_w : 0), v2 = my_global, v3 = my_long;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        v0 += __shfl_xor(v0, d, 64); v1 += __shfl_xor(v1, d, 64);
        v2 += __shfl_xor(v2, d, 64); v3 += __shfl_xor(v3, d, 64);
    }
    if (lane == 0) { wsum[wave][0] = v0; wsum[wave][1] = v1; wsum[wave][2] = v2; wsum[wave][3] = v3; }
    __syncthreads();
    if (tid < 4) {
        u64 t = 0;
        for (int w = 0; w < MAP_WAVES; w++) t += wsum[w][tid];
        a.wg_stats[(u64)blockIdx.x * 4 + tid] = t;
    }
}

}  // namespace wcg
