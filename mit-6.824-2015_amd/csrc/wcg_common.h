// wcg_common.h - device-side building blocks of the MI355X word-count engine (gfx950).
//
// Semantics restated (reference paths relative to /root/reference):
//   token   = maximal run of runes with unicode.IsLetter (src/main/wc.go:18-21,
//             strings.FieldsFunc); runes decoded with Go's utf8 rules, an invalid byte is
//             U+FFFD of width 1 (a separator).
//   ihash   = FNV-1a 32 (src/mapreduce/mapreduce.go:185-189).
//
// Byte-level facts the kernels rely on (proved in DESIGN.md section 3):
//   F1  every byte that is not a UTF-8 continuation byte (80..BF) starts a rune in Go's
//       decoding, so a byte's letter-ness depends only on bytes [p-3, p+3];
//   F2  a 16-byte chunk whose bytes are all < 0x80 is ASCII regardless of its neighbours;
//   F3  tokens are the maximal runs of "letter bytes"; a token start is a letter byte whose
//       predecessor is not a letter byte, and it is always a rune start;
//   F4  letters never contain the byte 0x00, so a key of <= 15 bytes zero-padded to 16 bytes
//       (+ its length in byte 15) is an exact, fixed-width identity, and big-endian
//       comparison of the zero-padded bytes is Go's bytewise string order (sort.Strings).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define WCG_LT_QUAL __constant__
#include "letter_table.h"

namespace wcg {

typedef unsigned long long u64;
typedef unsigned int u32;

// ---- key identity (fact F4), shared by the LDS tables, the miss log and the global table:
//   len <= 7 : k0 = key bytes 0..len-1 (little-endian, zero padded) | len << 56, k1 = 0
//   len 8-15 : k0 = key bytes 0-7, k1 = key bytes 8..len-1 (zero padded) | len << 56
// Byte 7 of a key of 8+ bytes is a letter byte (>= 0x41), so k0 >> 56 < 8 identifies short
// keys and one 64-bit compare decides equality for them (89% of tokens of the C2 corpus).
// k0 is never 0 and k1 is never 0 for keys of 8+ bytes.
__device__ __forceinline__ bool key_short(u64 k0) { return (k0 >> 56) < 8; }
__device__ __forceinline__ int key_len(u64 k0, u64 k1) {
    u32 t = (u32)(k0 >> 56);
    return t < 8 ? (int)t : (int)(k1 >> 56);
}
// raw little-endian key bytes -> identity (b0/b1 already hold only the key's bytes)
__device__ __forceinline__ void make_key(u64 b0, u64 b1, int len, u64& k0, u64& k1) {
    if (len <= 7) { k0 = b0 | (u64)len << 56; k1 = 0; }
    else { k0 = b0; k1 = b1 | (u64)len << 56; }
}

// ---- global aggregation table entry (HBM): inline keys {k0, k1, cnt}; the long-key table
// uses k0 = 64-bit hash tag (|1), k1 = arena offset + 1 (publish word), aux = key length.
struct __align__(32) GEntry { u64 k0, k1, cnt, aux; };

// ---- sorted record (after compaction): the 128-bit big-endian prefix is the sort key.
// inline: ref = len (1..15); long: ref = LONG_FLAG | len << 40 | arena offset.
struct __align__(32) Rec { u64 hi, lo, cnt, ref; };
constexpr u64 LONG_FLAG = 1ull << 63;
constexpr u64 LONG_OFF_MASK = (1ull << 40) - 1;
constexpr u64 LONG_LEN_MAX = (1ull << 23) - 1;

// ---- long-key arena: [lslots x LONG_CELL-byte cells | heap].  A long key of <= LONG_CELL bytes
// lives in the cell of the ltab slot that claimed it (no allocation, so no contended atomic on
// one counter); a longer key gets a 16-byte aligned heap reservation (DevState::arena_top counts
// heap bytes only).  Every key's bytes are zero-padded to its 16-byte cells, so readers compare
// with 16-byte loads.
constexpr u64 LONG_CELL = 32;
__device__ __forceinline__ u64 long_cells(u64 len) { return len <= LONG_CELL ? LONG_CELL : (len + 15) & ~15ull; }
// arena offset for a key claimed in slot s, or ~0 when the heap is full
__device__ __forceinline__ u64 long_home(u64 s, u64 len, u64 lslots, u64 heap_cap, u64* arena_top) {
    if (len <= LONG_CELL) return s * LONG_CELL;
    const u64 r = long_cells(len);
    const u64 ho = atomicAdd(arena_top, r);
    return ho + r > heap_cap ? ~0ull : lslots * LONG_CELL + ho;
}

// ---- device-side counters/status (one per context)
constexpr u64 ST_SCALAR_OFF = 128;   // the scalars follow DevState in one allocation (wcg_api.hip)
constexpr u64 ST_TIE_GROUPS = 16;    // scalar slot of the tie-group count (the scans use 0, the sort 8)
constexpr u64 ST_TIE_BIG = 17;       // scalar slot: tie groups of more than 64 records (k_tie_tiny -> k_tie_sort)
constexpr u64 ST_GLIST = 24;         // scalar slot: two-pass contexts' global-table claim list, or 0
constexpr u64 GLIST_CAP = 1ull << 20;   // claims listed (more: compaction and reset scan it all)
constexpr u64 ST_LLIST = 25;         // scalar slot: large contexts' long-key-table claim list, or 0
constexpr u64 LLIST_CAP = 1ull << 22;   // (C4 1 GiB: 1.6M long keys in a 16M-slot, 512 MiB table)
struct DevState {
    u64 tokens;          // tokens seen by map kernels
    u64 lds_hits;        // tokens aggregated in LDS
    u64 global_ops;      // global-table insertions (misses + flushes)
    u64 long_tokens;     // tokens longer than 15 bytes
    u64 arena_top;       // bytes used in the long-key arena heap (keys > 32 B; shorter keys use slot cells)
    u64 nrec;            // records produced by compaction
    u64 nlong;           // ... of which long keys (> 15 bytes)
    u64 nemit;           // records emitted by k_agg's pass 2 (the record log, across map calls)
    u64 gnew;            // global-table slots claimed since wcg_reset (two-pass contexts list them)
    u64 lnew;            // long-key-table slots claimed since wcg_reset (large contexts list them)
    u64 lemit;           // long-key records k_long_agg put in the record log (two-pass jobs)
    u64 lheap_top;       // bytes of those records' keys in the log heap (after the table's heap)
    u32 overflow;        // table / arena full -> WCG_EFULL
    u32 spin_fail;       // bounded spin gave up -> WCG_EFULL (never expected)
    u32 bad_input;       // malformed record units (wcg_import) or lines (wcg_merge_runs) -> WCG_EINVAL
    u32 long_fb;         // diagnostics: long-key entries counted by a fenced table insert (fallbacks)
};

// ------------------------------------------------------------------ letters
__device__ __forceinline__ bool lt_is_letter(u32 cp) {
    if (cp < 0x80) return ((cp | 0x20) - 'a') < 26u;
    if (cp >= 0x110000) return false;
    u32 blk = WCG_LT_STAGE1[cp >> 8];
    return (WCG_LT_STAGE2[blk][(cp >> 5) & 7] >> (cp & 31)) & 1u;
}

// Go utf8.DecodeRune at p of a byte source `at(i)` returning 0 beyond the end.
// Returns width (0 = invalid -> treat as RuneError width 1) and the code point.
template <typename At>
__device__ __forceinline__ int go_decode(At at, long p, u32* cp_out) {
    u32 b0 = at(p);
    if (b0 < 0x80) { *cp_out = b0; return 1; }
    int w; u32 lo = 0x80, hi = 0xBF;
    if (b0 >= 0xC2 && b0 <= 0xDF) w = 2;
    else if (b0 >= 0xE0 && b0 <= 0xEF) { w = 3; if (b0 == 0xE0) lo = 0xA0; else if (b0 == 0xED) hi = 0x9F; }
    else if (b0 >= 0xF0 && b0 <= 0xF4) { w = 4; if (b0 == 0xF0) lo = 0x90; else if (b0 == 0xF4) hi = 0x8F; }
    else return 0;
    u32 b1 = at(p + 1);
    if (b1 < lo || b1 > hi) return 0;
    if (w == 2) { *cp_out = ((b0 & 0x1F) << 6) | (b1 & 0x3F); return 2; }
    u32 b2 = at(p + 2);
    if ((b2 & 0xC0) != 0x80) return 0;
    if (w == 3) { *cp_out = ((b0 & 0x0F) << 12) | ((b1 & 0x3F) << 6) | (b2 & 0x3F); return 3; }
    u32 b3 = at(p + 3);
    if ((b3 & 0xC0) != 0x80) return 0;
    *cp_out = ((b0 & 0x07) << 18) | ((b1 & 0x3F) << 12) | ((b2 & 0x3F) << 6) | (b3 & 0x3F);
    return 4;
}

// Is byte p part of a letter rune?  (fact F1: look back at most 3 bytes for the lead)
template <typename At>
__device__ __forceinline__ bool letter_byte(At at, long p) {
    u32 b = at(p);
    if (b < 0x80) return ((b | 0x20) - 'a') < 26u;
    u32 cp;
    if ((b & 0xC0) == 0x80) {
        for (int k = 1; k <= 3; k++) {
            u32 q = at(p - k);
            if ((q & 0xC0) == 0x80) continue;          // another continuation byte
            int w = go_decode(at, p - k, &cp);
            return w > k && lt_is_letter(cp);         // covered by a valid rune starting at p-k
        }
        return false;                                 // 4+ continuation bytes: invalid
    }
    int w = go_decode(at, p, &cp);
    return w > 0 && lt_is_letter(cp);
}

// 16 ASCII bytes (4 little-endian dwords) -> 16-bit letter mask (SWAR, bytes < 0x80 only)
__device__ __forceinline__ u32 ascii_mask4(u32 x) {
    u32 t = x | 0x20202020u;
    u32 a = t + 0x1F1F1F1Fu;            // >= 'a'  (no carries: t <= 0x7F per byte)
    u32 b = t + 0x05050505u;            // >= '{'
    u32 hi = a & ~b & 0x80808080u;
    return (((hi >> 7) * 0x00204081u) >> 21) & 0xFu;
}
// 16 ASCII bytes -> letter mask.  The letter flags sit in bit 7 of each byte; one multiply by
// 2^0 + 2^7 + 2^14 + 2^21 gathers the four flags of a dword into bits 28-31 (the partial
// products land on distinct bits: no carries), and each nibble is shifted straight to its place
__device__ __forceinline__ u32 ascii_hi4(u32 x) {
    const u32 t = x | 0x20202020u;
    return (t + 0x1F1F1F1Fu) & ~(t + 0x05050505u) & 0x80808080u;   // >= 'a' and < '{'
}
__device__ __forceinline__ u32 ascii_mask16(uint4 v) {
    constexpr u32 G = 0x00204081u;
    return ((ascii_hi4(v.x) * G) >> 28) | (((ascii_hi4(v.y) * G) >> 24) & 0xF0u) |
           (((ascii_hi4(v.z) * G) >> 20) & 0xF00u) | (((ascii_hi4(v.w) * G) >> 16) & 0xF000u);
}
__device__ __forceinline__ bool all_ascii(uint4 v) { return ((v.x | v.y | v.z | v.w) & 0x80808080u) == 0; }

// 4 bytes -> 4-bit mask of the bytes with the high bit set
__device__ __forceinline__ u32 high_mask4(u32 x) {
    return ((((x & 0x80808080u) >> 7) * 0x00204081u) >> 21) & 0xFu;
}

// k_map's copy of the letter table in LDS.  A load from the global table would be followed by
// s_waitcnt vmcnt(0), which also waits for every window prefetch in flight (vmcnt counts all
// older loads): on mixed UTF-8 text that drained k_map's prefetch pipeline almost every step.
// Blocks 0-7 (U+0000-07FF) are table blocks 0-7, so 2-byte runes need no index read.
constexpr u32 LT_LDS_BLOCKS = 0x314;          // 256-code-point blocks up to the last letter (U+3134A)
struct LdsLetters {
    const uint8_t* idx;                       // [LT_LDS_BLOCKS + 1]: block ids; the last is empty
    const u32* bits;                          // [WCG_LT_NBLOCKS * 8]
};
// fill the LDS copy (all threads of the workgroup; a barrier must follow)
__device__ __forceinline__ void lds_letters_init(uint8_t* idx, u32* bits, int tid, int nt) {
    for (int i = tid; i <= (int)LT_LDS_BLOCKS; i += nt)
        idx[i] = WCG_LT_STAGE1[i < (int)LT_LDS_BLOCKS ? i : 0x10FF];
    for (int i = tid; i < WCG_LT_NBLOCKS * 8; i += nt) bits[i] = WCG_LT_STAGE2[i >> 3][i & 7];
}

// 4 bytes -> 4-bit mask of the continuation bytes (80-BF)
__device__ __forceinline__ u32 cont_mask4(u32 x) {
    const u32 t = (x & 0xC0C0C0C0u) ^ 0x80808080u;          // zero bytes = continuation bytes
    const u32 c = ~(t | (t << 1)) & 0x80808080u;
    return (((c >> 7) * 0x00204081u) >> 21) & 0xFu;
}

// 19-bit letter mask of a chunk containing non-ASCII bytes (fact F1).  Bits 0-15: the chunk's
// ASCII letters and the bytes of the letter runes that START in the chunk; bits 16-18: bytes of
// the next chunk covered by such a rune.  The caller ORs the predecessor chunk's bits 16-18 into
// bits 0-2 (one DPP lane shift), which replaces decoding three look-back positions per chunk.
// `nx` = the first 4 bytes after the chunk (zeros outside the input or the window).
// Branch-free over the 16 positions: every non-ASCII lead decodes (Go's utf8.DecodeRune: the
// continuation bytes, then the code point's range, which rules out exactly what the E0/ED/F0/F4
// second-byte rules reject - overlong forms, surrogates and > U+10FFFF); a position that is not
// a valid lead gets cp 0.  The LDS table reads of a group of positions issue back to back and
// complete under one wait.  (A branch per position ran the whole decode for every position any
// lane needed, with two dependent LDS round trips each: 2.5 ms per GiB of C4 text.)
#ifndef WCG_UTF8_GROUP
#define WCG_UTF8_GROUP 8
#endif
#ifndef WCG_UTF8_COMPACT
#define WCG_UTF8_COMPACT 1
#endif
// 4 bytes -> 4-bit mask of the possible lead bytes C2-F4 (SWAR: bit 7 set and low 7 bits in
// 42-74; the additions cannot carry out of a byte)
__device__ __forceinline__ u32 lead_mask4(u32 x) {
    const u32 t = x & 0x7F7F7F7Fu;
    const u32 c = (t + 0x3E3E3E3Eu) & ~(t + 0x0B0B0B0Bu) & x & 0x80808080u;
    return (((c >> 7) * 0x00204081u) >> 21) & 0xFu;
}
__device__ __forceinline__ u32 utf8_mask_lds_all(uint4 c, u32 nx, LdsLetters lt);
// Lead-compacted form (r03): only positions holding a lead byte (C2-F4) followed by a
// continuation byte can start a multi-byte letter, and no two such positions are adjacent (the
// byte after one is a continuation byte), so a chunk has at most 8 of them.  Eight slots decode
// the chunk's such positions in turn (the lowest first; an empty slot decodes cp 0, not a letter)
// instead of all 16 positions: C4 text averages 4.5 per non-ASCII chunk, and the decode's VALU is
// what bounds k_map there.
__device__ __forceinline__ u32 utf8_mask_lds(uint4 c, u32 nx, LdsLetters lt) {
#if !WCG_UTF8_COMPACT
    return utf8_mask_lds_all(c, nx, lt);
#else
    const u32 d0 = c.x, d1 = c.y, d2 = c.z, d3 = c.w, d4 = nx;
    u32 m = (ascii_mask4(c.x & 0x7F7F7F7Fu) & ~high_mask4(c.x)) |
            ((ascii_mask4(c.y & 0x7F7F7F7Fu) & ~high_mask4(c.y)) << 4) |
            ((ascii_mask4(c.z & 0x7F7F7F7Fu) & ~high_mask4(c.z)) << 8) |
            ((ascii_mask4(c.w & 0x7F7F7F7Fu) & ~high_mask4(c.w)) << 12);
    const u32 cont = cont_mask4(c.x) | (cont_mask4(c.y) << 4) | (cont_mask4(c.z) << 8) |
                     (cont_mask4(c.w) << 12) | (cont_mask4(nx) << 16);   // bit j: byte j
    u32 L = (lead_mask4(c.x) | (lead_mask4(c.y) << 4) | (lead_mask4(c.z) << 8) | (lead_mask4(c.w) << 12)) &
            (cont >> 1);
    constexpr int NS = 8;
    u32 cp[NS], span[NS];
#pragma unroll
    for (int g = 0; g < NS; g++) {
        const bool has = L != 0u;
        const u32 i = (u32)__builtin_ctz(L | 0x10000u) & 15u;
        L &= L - 1u;
        // dwords i >> 2 and (i >> 2) + 1 of the chunk (two levels of selects)
        const bool s0 = (i & 4u) != 0, s1 = (i & 8u) != 0;
        const u32 p0 = s0 ? d1 : d0, p1 = s0 ? d2 : d1, p2 = s0 ? d3 : d2, p3 = s0 ? d4 : d3;
        const u32 wd = __builtin_amdgcn_alignbyte(s1 ? p3 : p1, s1 ? p2 : p0, i & 3u);
        // as utf8_mask_lds_all, minus the lead test (b0 is C2-F4 in a filled slot)
        const u32 b0 = wd & 0xFFu;
        const u32 w = __builtin_clz(~(wd << 24));          // leading ones of b0: 2-4
        const u32 need = (1u << ((w - 1) & 31)) - 1u;
        const bool conts = ((cont >> (i + 1)) & need) == need;
        const u32 x = ((b0 & (0x7Fu >> (w & 31))) << 18) | ((wd << 4) & 0x3F000u) | ((wd >> 10) & 0xFC0u) |
                      ((wd >> 24) & 0x3Fu);
        const u32 v = x >> ((24 - 6 * w) & 31);
        const bool ok = has & conts & ((v >> ((5 * w - 4) & 31)) != 0u) & (v - 0xD800u >= 0x800u) &
                        (v <= 0x10FFFFu);
        cp[g] = ok ? v : 0u;
        span[g] = __builtin_amdgcn_ubfe(0xFFFFFFFFu, 0, w & 31) << i;
    }
    u32 t[NS], bits[NS];
#pragma unroll
    for (int g = 0; g < NS; g++) {
        const u32 b = cp[g] >> 8;
        t[g] = lt.idx[b < LT_LDS_BLOCKS ? b : LT_LDS_BLOCKS];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int g = 0; g < NS; g++) {
        const u32 b = cp[g] >> 8;
        bits[g] = lt.bits[(b < 8 ? b : t[g]) * 8 + ((cp[g] >> 5) & 7)];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int g = 0; g < NS; g++) m |= ((bits[g] >> (cp[g] & 31)) & 1u) ? span[g] : 0u;
    return m;
#endif
}
// every position decoded (the form before r03's lead compaction; WCG_UTF8_COMPACT=0)
__device__ __forceinline__ u32 utf8_mask_lds_all(uint4 c, u32 nx, LdsLetters lt) {
    const u32 d[5] = {c.x, c.y, c.z, c.w, nx};
    u32 m = (ascii_mask4(c.x & 0x7F7F7F7Fu) & ~high_mask4(c.x)) |
            ((ascii_mask4(c.y & 0x7F7F7F7Fu) & ~high_mask4(c.y)) << 4) |
            ((ascii_mask4(c.z & 0x7F7F7F7Fu) & ~high_mask4(c.z)) << 8) |
            ((ascii_mask4(c.w & 0x7F7F7F7Fu) & ~high_mask4(c.w)) << 12);
    const u32 cont = cont_mask4(c.x) | (cont_mask4(c.y) << 4) | (cont_mask4(c.z) << 8) |
                     (cont_mask4(c.w) << 12) | (cont_mask4(nx) << 16);   // bit j: byte j
    constexpr int G = WCG_UTF8_GROUP;
#pragma unroll
    for (int k0 = 0; k0 < 16; k0 += G) {
        u32 cp[G], span[G], blk[G];
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int i = k0 + g;
            const u32 wd = (i & 3) ? __builtin_amdgcn_alignbyte(d[(i >> 2) + 1], d[i >> 2], i & 3) : d[i >> 2];
            // arithmetic forms only (no selects between literals: each literal a select needs
            // would be held in a VGPR across k_map's token loops)
            const u32 b0 = wd & 0xFFu;
            const bool lead = b0 - 0xC2u <= 0xF4u - 0xC2u;
            const u32 w = __builtin_clz(~(wd << 24));          // leading ones of b0: 2-4 for a lead
            const u32 need = (1u << ((w - 1) & 31)) - 1u;      // continuation bytes 1..w-1
            const bool conts = ((cont >> (i + 1)) & need) == need;
            const u32 x = ((b0 & (0x7Fu >> (w & 31))) << 18) | ((wd << 4) & 0x3F000u) | ((wd >> 10) & 0xFC0u) |
                          ((wd >> 24) & 0x3Fu);
            const u32 v = x >> ((24 - 6 * w) & 31);
            // overlong (3 bytes: < U+0800, 4 bytes: < U+10000; 2 bytes: C2-DF never are),
            // surrogates, > U+10FFFF
            const bool ok = lead & conts & ((v >> ((5 * w - 4) & 31)) != 0u) & (v - 0xD800u >= 0x800u) &
                            (v <= 0x10FFFFu);
            cp[g] = ok ? v : 0u;                               // cp 0: not a letter
            span[g] = __builtin_amdgcn_ubfe(0xFFFFFFFFu, 0, w & 31) << i;   // w bytes from i
        }
        // the reads of a group issue before any of their uses (the scheduler otherwise waited
        // for each read in turn)
        u32 t[G], bits[G];
#pragma unroll
        for (int g = 0; g < G; g++) {
            const u32 b = cp[g] >> 8;
            t[g] = lt.idx[b < LT_LDS_BLOCKS ? b : LT_LDS_BLOCKS];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < G; g++) {
            const u32 b = cp[g] >> 8;
            blk[g] = b < 8 ? b : t[g];
            bits[g] = lt.bits[blk[g] * 8 + ((cp[g] >> 5) & 7)];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < G; g++) m |= ((bits[g] >> (cp[g] & 31)) & 1u) ? span[g] : 0u;
        __builtin_amdgcn_sched_barrier(0);           // groups stay apart (register pressure)
    }
    return m;
}

// ------------------------------------------------------------------ hashing
__device__ __host__ __forceinline__ u64 mix64(u64 x) {
    x ^= x >> 32; x *= 0xD6E8FEB86659FD93ull; x ^= x >> 32; x *= 0xD6E8FEB86659FD93ull; x ^= x >> 32;
    return x;
}

// Long keys (> 15 bytes) are tagged by a hash of their bytes taken a little-endian 32-bit word at a
// time (zeros past the key's end), finished by mix64 with the length: every kernel that tags a
// long key (k_long_hash / k_long_agg / k_import) must use these.  Internal only - the partition
// hash of the reference (ihash, FNV-1a 32) is computed separately.  (r04: it was FNV-1a 64 byte by
// byte, ~5 VALU per byte on the hashing lane.)
__device__ __forceinline__ u64 lhash_step(u64 h, u32 w) { return (h ^ w) * 0x100000001B3ull; }
constexpr u64 LHASH_INIT = 0xCBF29CE484222325ull;
// 64-bit key hash: miss-log bucket and global-table slot (computed off the hit path)
__device__ __forceinline__ u64 key_hash(u64 k0, u64 k1) {
    return mix64(k0 * 0x9E3779B97F4A7C15ull + (k1 ^ (k1 >> 29)) * 0xC2B2AE3D27D4EB4Full);
}
// 32-bit key hash for the LDS tables and the miss-log bucket: the four key words folded with
// rotations, then one multiply between two xor-shifts (one quarter-rate multiply on k_map's hot
// path; the multiply mixes low bits up, the final shift brings high bits down to the bucket bits)
__device__ __forceinline__ u32 lds_hash32(u32 a, u32 b, u32 c, u32 d) {
    u32 x = a ^ __builtin_rotateleft32(b, 9) ^ __builtin_rotateleft32(c, 17) ^ __builtin_rotateleft32(d, 25);
    x ^= x >> 15;
    x *= 0x2C1B3C6Du;
    x ^= x >> 12;
    return x;
}
__device__ __forceinline__ u32 lds_hash(u64 k0, u64 k1) {
    return lds_hash32((u32)k0, (u32)(k0 >> 32), (u32)k1, (u32)(k1 >> 32));
}
__device__ __forceinline__ u32 fnv1a_step(u32 h, u32 byte) { return (h ^ byte) * 0x01000193u; }

__device__ __forceinline__ u64 bswap64(u64 x) { return __builtin_bswap64(x); }

// the record of an inline key (k0, k1) of fact F4 (the same conversion as k_compact's)
__device__ __forceinline__ Rec inline_rec(u64 k0, u64 k1, u64 cnt) {
    Rec r;
    if (key_short(k0)) {
        r.hi = bswap64(k0 & 0x00FFFFFFFFFFFFFFull);
        r.lo = 0;
        r.ref = k0 >> 56;
    } else {
        r.hi = bswap64(k0);
        r.lo = bswap64(k1 & 0x00FFFFFFFFFFFFFFull);
        r.ref = k1 >> 56;
    }
    r.cnt = cnt;
    return r;
}
// ... and back (ref = the key's length, < 16)
__device__ __forceinline__ void rec_inline_key(const Rec& r, u64& k0, u64& k1) {
    if (r.ref < 8) { k0 = bswap64(r.hi) | r.ref << 56; k1 = 0; }
    else { k0 = bswap64(r.hi); k1 = bswap64(r.lo) | r.ref << 56; }
}

// mask keeping the low `nbytes` bytes (0..8)
__device__ __forceinline__ u64 low_bytes_mask(int nbytes) {
    return nbytes >= 8 ? ~0ull : ((1ull << (8 * nbytes)) - 1);
}

// ------------------------------------------------------------------ atomics helpers
__device__ __forceinline__ u64 ld_agent(const u64* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(u64* p, u64 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool cas_agent(u64* p, u64* expected, u64 desired) {
    return __hip_atomic_compare_exchange_strong(p, expected, desired, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void add_agent(u64* p, u64 v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int SPIN_LIMIT = 1 << 20;

// a table slot just claimed by this thread, appended to the context's claim list when it keeps one
// (scalar slot `which` of DevState's block): compaction and wcg_reset then visit the listed slots
// instead of the whole table; past `cap` claims they scan it all
__device__ __forceinline__ void list_claim(DevState* st, u64 which, u64* counter, u64 cap, u64 s) {
    u64* const l = *reinterpret_cast<u64* const*>(reinterpret_cast<const uint8_t*>(st) + ST_SCALAR_OFF +
                                                  which * sizeof(u64));
    if (l) {
        const u64 i = atomicAdd((unsigned long long*)counter, 1ull);
        if (i < cap) l[i] = s;
    }
}

// THE claim of an empty table slot (CAS k0: 0 -> key) and, when it succeeds, its entry in the
// table's claim list (large contexts clear and compact only the listed slots: a claim that skipped
// the list would survive wcg_reset and drop out of compaction).  Every insert path claims through
// these two: ginsert, ltab_add (k_long_*, fallbacks), k_import.  On failure *seen
// holds the slot's current k0.
__device__ __forceinline__ bool gtab_claim(DevState* st, GEntry* e, u64 s, u64 key, u64* seen) {
    *seen = 0;
    if (!cas_agent(&e->k0, seen, key)) return false;
    list_claim(st, ST_GLIST, &st->gnew, GLIST_CAP, s);
    return true;
}
__device__ __forceinline__ bool ltab_claim(DevState* st, GEntry* e, u64 s, u64 tag, u64* seen) {
    *seen = 0;
    if (!cas_agent(&e->k0, seen, tag)) return false;
    list_claim(st, ST_LLIST, &st->lnew, LLIST_CAP, s);
    return true;
}

// Insert/accumulate an inline key into the global table (open addressing, linear probing from
// slot_hash).  Claim protocol: CAS k0 0 -> key; a key of 8+ bytes then publishes k1 (never 0).
// A reader that sees k0 == key but k1 == 0 re-reads in a later iteration (the claimer publishes
// in the same iteration of its own loop, so no lane waits on a lane parked behind it).
__device__ __forceinline__ void ginsert(GEntry* tab, u64 mask, u64 k0, u64 k1, u64 slot_hash, u64 cnt, DevState* st) {
    u64 s = slot_hash & mask;
    u64 probes = 0;
    int spins = 0;
    const bool shrt = key_short(k0);
    while (true) {
        GEntry* e = &tab[s];
        u64 c0 = ld_agent(&e->k0);
        if (c0 == 0) {
            u64 exp;
            // (two-pass contexts keep the global table nearly empty - a few fallback inserts per
            // GiB - and list its claimed slots, so that compaction and wcg_reset visit those slots
            // instead of the whole GB-sized table)
            if (gtab_claim(st, e, s, k0, &exp)) {
                if (!shrt) st_agent(&e->k1, k1);
                add_agent(&e->cnt, cnt);
                return;
            }
            c0 = exp;
        }
        if (c0 == k0) {
            if (shrt) { add_agent(&e->cnt, cnt); return; }
            u64 c1 = ld_agent(&e->k1);
            if (c1 == k1) { add_agent(&e->cnt, cnt); return; }
            if (c1 == 0) {                                   // claimed, not yet published
                if (++spins > SPIN_LIMIT) { atomicAdd(&st->spin_fail, 1u); return; }
                continue;
            }
        }
        s = (s + 1) & mask;
        if (++probes > mask) { atomicAdd(&st->overflow, 1u); return; }
    }
}

// ---------------------------------------------------------------- streaming buffer loads
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));

// k_map's input stream uses inline-asm buffer loads with hand-counted waits: the compiler's
// waitcnt pass drains every load (vmcnt(0)) at the top of that loop, which serialises the
// prefetch.  Rules kept here: each wait names its registers as "+v"
// so no use moves above it, every asm-loaded register is waited for before it can die or be
// copied, and N counts only this wave's own younger asm loads (compiler-issued memory ops in
// between can only make a wait stronger).
//
// Each load and wait carries a tag in an assembly comment ("wcg-load A0", "wcg-wait A v[..]")
// naming its register set (the set ops are in wcg_map.h).  tools/check_inflight.py requires
// every tagged load and wait of a set to use the same physical registers: a register copy
// between an asm load and its wait (which would read data that has not landed) cannot pass that
// check (tests/test_isa.py).
__device__ __forceinline__ v4i make_rsrc(const void* base, u32 nbytes) {
    const u64 p = (u64)base;
    v4i r;
    r.x = __builtin_amdgcn_readfirstlane((int)(u32)p);
    r.y = __builtin_amdgcn_readfirstlane((int)((u32)(p >> 32) & 0xFFFFu));
    r.z = __builtin_amdgcn_readfirstlane((int)nbytes);
    r.w = 0x00020000;
    return r;
}

}  // namespace wcg
