// wcg_map.h - the map kernel: DoMap + Map (mapreduce.go:193-231, wc.go:17-30) on gfx950.
//
// One workgroup (16 waves) per CU walks a contiguous range of tiles (TILE = NT * 16 bytes):
//   1. every thread loads one 16-byte chunk (coalesced dwordx4; the next tile is prefetched
//      into registers while the current one is processed), plus a 16-byte prefix and a
//      64-byte look-ahead so tokens that cross the tile end can be read whole;
//   2. per chunk: 16-bit letter-byte mask - SWAR on all-ASCII chunks, Go UTF-8 decode +
//      Unicode-13 letter bitmap otherwise;
//   3. token starts = letter & ~prev_letter; each wave compacts its starts (ballot/mbcnt
//      prefix sum, no LDS shuffles) into an LDS list and processes them 64 at a time;
//   4. per token: length from the LDS mask, key identity (<= 15 bytes, fact F4) -> LDS hash
//      table (exact keys, 2-choice x 4-way buckets, u32 counts); an LDS miss is appended to
//      this workgroup's region of the miss log (plain stores, no atomics) for k_agg; tokens
//      > 15 bytes go to the long-key table with an arena copy of their bytes;
//   5. at the end of its range the workgroup flushes its LDS table into the miss log too.
// Token ownership: a token belongs to the tile holding its first byte (counted exactly once).
#pragma once
#include "wcg_common.h"
#include "wcg_lds_table.h"

namespace wcg {

constexpr int MAP_NT = 1024;                 // threads per workgroup (16 waves)
constexpr int MAP_TILE = MAP_NT * 16;        // bytes per tile
constexpr int MAP_PRE = 16;                  // prefix bytes (need 4)
constexpr int MAP_LOOK = 64;                 // look-ahead bytes (tokens <= 15 need 15)
constexpr int MAP_REG = MAP_PRE + MAP_TILE + MAP_LOOK;
constexpr int MAP_NCH = MAP_REG / 16;        // chunks in the LDS region
constexpr int MAP_WAVES = MAP_NT / 64;
constexpr int MAP_NB = 1584;                 // LDS table buckets (x4 slots, 20 B per slot)
constexpr int MAX_MISS_BUCKETS = 256;

struct MapArgs {
    const uint8_t* in;
    u64 n;
    u64 ntiles;
    u64 tiles_per_wg;
    GEntry* gtab;  u64 gmask;      // inline-key table
    GEntry* ltab;  u64 lmask;      // long-key table
    uint8_t* arena; u64 arena_cap;
    DevState* st;
    uint4* pool;   u64 region_cap;  // miss log: region (wg, p) = pool[(wg * P + p) * region_cap ...]
    u32* region_len;               // entries written per region
    u32 pmask;                     // P - 1 (P = number of miss buckets, power of two)
};

// append one miss-log entry for this workgroup; returns false when the region is full
__device__ __forceinline__ bool log_push(const MapArgs& a, u32* cursor, u32 p, uint4 e) {
    u32 pos = atomicAdd(&cursor[p], 1u);
    if (pos >= a.region_cap) return false;
    a.pool[((u64)blockIdx.x * (a.pmask + 1) + p) * a.region_cap + pos] = e;
    return true;
}
__device__ __forceinline__ uint4 entry(u64 x, u64 y) {
    return make_uint4((u32)x, (u32)(x >> 32), (u32)y, (u32)(y >> 32));
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

// long token (> 15 bytes) starting at absolute offset p: walk runes in global memory
__device__ void long_token(const MapArgs& a, u64 p) {
    const uint8_t* in = a.in;
    u64 n = a.n;
    auto at = [&](long i) -> u32 { return (i >= 0 && (u64)i < n) ? in[i] : 0u; };
    u64 q = p;
    u64 h = 0xCBF29CE484222325ull;
    while (q < n) {
        u32 cp;
        int w = go_decode(at, (long)q, &cp);
        if (w == 0 || !lt_is_letter(cp)) break;
        for (int k = 0; k < w; k++) { h ^= in[q + k]; h *= 0x100000001B3ull; }
        q += w;
    }
    u64 len = q - p;
    if (len > LONG_LEN_MAX) { atomicAdd(&a.st->overflow, 1u); return; }
    u64 tag = mix64(h ^ len) | 1ull;
    u64 s = tag & a.lmask, probes = 0;
    int spins = 0;
    while (true) {
        GEntry* e = &a.ltab[s];
        u64 c0 = ld_agent(&e->k0);
        if (c0 == 0) {
            u64 exp = 0;
            if (cas_agent(&e->k0, &exp, tag)) {
                u64 off = atomicAdd(&a.st->arena_top, len);
                if (off + len > a.arena_cap) { atomicAdd(&a.st->overflow, 1u); return; }
                for (u64 i = 0; i < len; i++) a.arena[off + i] = in[p + i];
                st_agent(&e->aux, len);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                __hip_atomic_store(&e->k1, off + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                add_agent(&e->cnt, 1);
                return;
            }
            c0 = exp;
        }
        if (c0 == tag) {
            u64 r = ld_agent(&e->k1);
            if (r == 0) {
                if (++spins > SPIN_LIMIT) { atomicAdd(&a.st->spin_fail, 1u); return; }
                continue;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            u64 elen = ld_agent(&e->aux);
            bool same = (elen == len);
            for (u64 i = 0; same && i < len; i++) same = (a.arena[r - 1 + i] == in[p + i]);
            if (same) { add_agent(&e->cnt, 1); return; }
        }
        s = (s + 1) & a.lmask;
        if (++probes > a.lmask) { atomicAdd(&a.st->overflow, 1u); return; }
    }
}

// ABL (measurement builds only, selected by WCG_MAP_ABLATE; results are wrong when ABL != 0):
//   1 = tokenize + compact only, 2 = + key extraction and hash, 3 = + LDS lookup, misses dropped
template <int ABL>
__global__ __launch_bounds__(MAP_NT) void k_map(MapArgs a) {
    __shared__ __align__(16) uint8_t sbytes[MAP_REG];
    __shared__ __align__(16) uint16_t smask[MAP_NCH + 8];
    __shared__ uint16_t sstart[MAP_WAVES][512];
    __shared__ __align__(16) u64 tk0[MAP_NB][4];
    __shared__ __align__(16) u64 tk1[MAP_NB][4];
    __shared__ u32 tcnt[MAP_NB][4];
    __shared__ u32 cursor[MAX_MISS_BUCKETS];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    LdsTable<MAP_NB, u32> tab{tk0, tk1, tcnt};
    tab.init(tid, MAP_NT);
    for (int i = tid; i < MAX_MISS_BUCKETS; i += MAP_NT) cursor[i] = 0;
    if (tid < 8) smask[MAP_NCH + tid] = 0;

    const u64 t0 = (u64)blockIdx.x * a.tiles_per_wg;
    u64 t1 = t0 + a.tiles_per_wg;
    if (t1 > a.ntiles) t1 = a.ntiles;

    // chunk c of the region <-> input bytes [base - PRE + 16c, +16)
    // thread tid owns chunk tid+1; threads 0..4 also own chunk 0 and chunks NT+1..NT+4
    const int xc = (tid == 0) ? 0 : (tid <= 4 ? MAP_NT + tid : -1);
    uint4 cur = make_uint4(0, 0, 0, 0), curx = cur;
    if (t0 < t1) {
        long base = (long)(t0 * MAP_TILE);
        cur = load_chunk(a.in, a.n, base - MAP_PRE + 16 * (tid + 1));
        if (xc >= 0) curx = load_chunk(a.in, a.n, base - MAP_PRE + 16 * xc);
    }
    u64 my_tokens = 0, my_hits = 0, my_global = 0, my_long = 0;
    __syncthreads();

    for (u64 t = t0; t < t1; t++) {
        const long base = (long)(t * MAP_TILE);
        // ---- stage the tile in LDS, prefetch the next one into registers
        reinterpret_cast<uint4*>(sbytes)[tid + 1] = cur;
        if (xc >= 0) reinterpret_cast<uint4*>(sbytes)[xc] = curx;
        const uint4 mine = cur;
        if (t + 1 < t1) {
            long nb = base + MAP_TILE;
            cur = load_chunk(a.in, a.n, nb - MAP_PRE + 16 * (tid + 1));
            if (xc >= 0) curx = load_chunk(a.in, a.n, nb - MAP_PRE + 16 * xc);
        }
        __syncthreads();

        // ---- letter masks (fact F2: an all-ASCII chunk needs no context)
        auto at = [&](long i) -> u32 { return (i >= 0 && i < MAP_REG) ? (u32)sbytes[i] : 0u; };
        {
            const int ch = tid + 1;
            u32 m;
            if (all_ascii(mine)) {
                m = ascii_mask16(mine);
            } else {
                m = 0;
                for (int i = 0; i < 16; i++)
                    if (letter_byte(at, (long)(16 * ch + i))) m |= 1u << i;
            }
            smask[ch] = (uint16_t)m;
            if (xc >= 0) {
                uint4 v = reinterpret_cast<const uint4*>(sbytes)[xc];
                if (all_ascii(v)) {
                    m = ascii_mask16(v);
                } else {
                    m = 0;
                    for (int i = (xc == 0 ? 4 : 0); i < 16; i++)      // prefix chunk: only its tail matters
                        if (letter_byte(at, (long)(16 * xc + i))) m |= 1u << i;
                }
                smask[xc] = (uint16_t)m;
            }
        }
        __syncthreads();

        // ---- token starts in my chunk; wave prefix sum of the counts (<= 8) from 4 ballots
        {
            const int ch = tid + 1;
            const u32 m = smask[ch];
            const u32 prev = smask[ch - 1] >> 15;
            u32 starts = m & ~((m << 1) | prev) & 0xFFFFu;
            const u32 cnt = __popc(starts);
            u32 o = 0, total = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const u64 bal = __ballot((cnt >> b) & 1);
                o += __builtin_amdgcn_mbcnt_hi((u32)(bal >> 32), __builtin_amdgcn_mbcnt_lo((u32)bal, 0u)) << b;
                total += (u32)__popcll(bal) << b;
            }
            while (starts) {
                const int b = __ffs(starts) - 1;
                starts &= starts - 1;
                sstart[wave][o++] = (uint16_t)(16 * (ch - 1) + b);   // tile-relative offset
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            my_tokens += (lane == 0) ? (u64)total : 0;

            u32 sink = 0;
            for (u32 i = lane; i < total; i += 64) {
                if (ABL == 1) { sink += sstart[wave][i]; continue; }
                const int off = sstart[wave][i];
                const int rp = MAP_PRE + off;                       // region position
                const int wi = rp >> 4, bi = rp & 15;
                const u32 w32 = (u32)smask[wi] | ((u32)smask[wi + 1] << 16);
                const u32 v = ~(w32 >> bi);                         // >= 17 valid bits
                const int len = v ? __ffs(v) - 1 : 32;              // v == 0: run covers the window
                if (len >= 16) {
                    my_long++;
                    long_token(a, (u64)(base + off));
                    continue;
                }
                // key bytes [rp, rp+16) from LDS via 5 aligned dwords
                const int al = rp & ~3, sh = rp & 3;
                const u32* d = reinterpret_cast<const u32*>(sbytes + al);
                const u32 d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3], d4 = d[4];
                const u32 o0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
                const u32 o1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
                const u32 o2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
                const u32 o3 = __builtin_amdgcn_alignbyte(d4, d3, sh);
                const u64 b0 = ((u64)o1 << 32 | o0) & low_bytes_mask(len);
                const u64 b1 = len > 8 ? (((u64)o3 << 32 | o2) & low_bytes_mask(len - 8)) : 0ull;
                u64 k0, k1;
                make_key(b0, b1, len, k0, k1);
                if (ABL == 2) { sink += lds_hash(k0, k1); continue; }
                if (ABL == 3) { sink += tab.add(k0, k1, lds_hash(k0, k1), 1u); continue; }
                if (tab.add(k0, k1, lds_hash(k0, k1), 1u)) {
                    my_hits++;
                } else {
                    const u64 h2 = key_hash(k0, k1);
                    if (!log_push(a, cursor, miss_bucket(h2, a.pmask), entry(k0, k1))) {
                        my_global++;
                        ginsert(a.gtab, a.gmask, k0, k1, gslot(h2), 1, a.st);
                    }
                }
            }
            if (ABL) asm volatile("" ::"v"(sink));
        }
        __syncthreads();
    }

    // ---- flush the LDS table into this workgroup's miss-log regions (count 1: one entry,
    //      count c > 1: {k0, k1|CNT_FLAG} + carrier {0, c}); a full region -> global table
    __syncthreads();
    for (int i = tid; i < MAP_NB * 4; i += MAP_NT) {
        const u32 c = (&tcnt[0][0])[i];
        if (!c) continue;
        const u64 k0 = (&tk0[0][0])[i], k1 = (&tk1[0][0])[i];
        const u64 h2 = key_hash(k0, k1);
        const u32 p = miss_bucket(h2, a.pmask);
        bool ok;
        if (c == 1) {
            ok = log_push(a, cursor, p, entry(k0, k1));
        } else {
            const u32 pos = atomicAdd(&cursor[p], 2u);
            uint4* r = a.pool + ((u64)blockIdx.x * (a.pmask + 1) + p) * a.region_cap + pos;
            ok = pos + 1 < a.region_cap;
            if (ok) {
                r[0] = entry(k0, k1 | CNT_FLAG);
                r[1] = entry(0, (u64)c);
            } else if (pos < a.region_cap) {
                r[0] = entry(0, 0);                 // last slot of the region: a filler k_agg skips
            }
        }
        if (!ok) { my_global++; ginsert(a.gtab, a.gmask, k0, k1, gslot(h2), c, a.st); }
    }
    __syncthreads();
    for (u32 p = tid; p <= a.pmask; p += MAP_NT) {
        const u32 c = cursor[p];
        a.region_len[(u64)blockIdx.x * (a.pmask + 1) + p] = c < a.region_cap ? c : (u32)a.region_cap;
    }
    // stats: one atomic per wave
    u64 v0 = my_tokens, v1 = my_hits, v2 = my_global, v3 = my_long;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        v0 += __shfl_xor(v0, d, 64); v1 += __shfl_xor(v1, d, 64);
        v2 += __shfl_xor(v2, d, 64); v3 += __shfl_xor(v3, d, 64);
    }
    if (lane == 0) {
        atomicAdd(&a.st->tokens, v0); atomicAdd(&a.st->lds_hits, v1);
        atomicAdd(&a.st->global_ops, v2); atomicAdd(&a.st->long_tokens, v3);
    }
}

}  // namespace wcg
