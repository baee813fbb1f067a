// wcg_map.h - the map kernel: DoMap + Map (mapreduce.go:193-231, wc.go:17-30) on gfx950.
//
// One workgroup per CU walks a contiguous range of tiles (TILE = NT * 16 bytes):
//   1. every thread loads one 16-byte chunk (coalesced dwordx4; the next tile is prefetched
//      into registers while the current one is processed), plus a 16-byte prefix and a
//      64-byte look-ahead so tokens that cross the tile end can be read whole;
//   2. per chunk: 16-bit letter-byte mask - SWAR on all-ASCII chunks, Go UTF-8 decode +
//      Unicode-13 letter bitmap otherwise;
//   3. token starts = letter & ~prev_letter; each wave compacts its starts (wave prefix sum)
//      into an LDS list and processes them 64 at a time;
//   4. per token: length from the LDS mask, key = zero-padded bytes (<= 15) -> LDS hash table
//      (exact keys, CAS claim, u32 counts); table miss -> global HBM table; tokens > 15 bytes
//      -> long-key table with an arena copy of the bytes;
//   5. at the end of its range the workgroup flushes its LDS table into the global table.
// Token ownership: a token belongs to the tile holding its first byte (counted exactly once).
#pragma once
#include "wcg_common.h"

namespace wcg {

constexpr int MAP_NT = 512;                  // threads per workgroup (8 waves)
constexpr int MAP_TILE = MAP_NT * 16;        // bytes per tile
constexpr int MAP_PRE = 16;                  // prefix bytes (need 4)
constexpr int MAP_LOOK = 64;                 // look-ahead bytes (tokens <= 15 need 15)
constexpr int MAP_REG = MAP_PRE + MAP_TILE + MAP_LOOK;
constexpr int MAP_NCH = MAP_REG / 16;        // chunks in the LDS region
constexpr int MAP_WAVES = MAP_NT / 64;
constexpr int LDS_SLOTS = 6912;              // LDS hash table slots (20 B each)
constexpr int LDS_MAXPROBE = 24;

struct MapArgs {
    const uint8_t* in;
    u64 n;
    u64 ntiles;
    u64 tiles_per_wg;
    GEntry* gtab;  u64 gmask;      // inline-key table
    GEntry* ltab;  u64 lmask;      // long-key table
    uint8_t* arena; u64 arena_cap;
    DevState* st;
};

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

__global__ __launch_bounds__(MAP_NT) void k_map(MapArgs a) {
    __shared__ __align__(16) uint8_t sbytes[MAP_REG];
    __shared__ __align__(16) uint16_t smask[MAP_NCH + 8];
    __shared__ uint16_t sstart[MAP_WAVES][512];
    __shared__ __align__(16) u64 skey[LDS_SLOTS][2];
    __shared__ u32 scnt[LDS_SLOTS];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < LDS_SLOTS; i += MAP_NT) { skey[i][0] = 0; skey[i][1] = 0; scnt[i] = 0; }
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
        if (t + 1 < t1) {
            long nb = base + MAP_TILE;
            cur = load_chunk(a.in, a.n, nb - MAP_PRE + 16 * (tid + 1));
            if (xc >= 0) curx = load_chunk(a.in, a.n, nb - MAP_PRE + 16 * xc);
        }
        __syncthreads();

        // ---- letter masks
        auto at = [&](long i) -> u32 { return (i >= 0 && i < MAP_REG) ? (u32)sbytes[i] : 0u; };
        for (int c = (xc >= 0 ? 0 : 1); c < 2; c++) {
            int ch = (c == 0) ? xc : tid + 1;
            uint4 v = reinterpret_cast<const uint4*>(sbytes)[ch];
            u32 m;
            if (all_ascii(v)) {
                m = ascii_mask16(v);
            } else {
                m = 0;
                int lo = (ch == 0) ? 4 : 0;   // prefix chunk: only its tail matters
                for (int i = lo; i < 16; i++)
                    if (letter_byte(at, (long)(16 * ch + i))) m |= 1u << i;
            }
            smask[ch] = (uint16_t)m;
        }
        __syncthreads();

        // ---- token starts in my chunk, wave-level compaction
        {
            const int ch = tid + 1;
            u32 m = smask[ch];
            u32 prev = smask[ch - 1] >> 15;
            u32 starts = m & ~((m << 1) | prev) & 0xFFFFu;
            int cnt = __popc(starts);
            int incl = cnt;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                int y = __shfl_up(incl, d, 64);
                if (lane >= d) incl += y;
            }
            int total = __shfl(incl, 63, 64);
            int o = incl - cnt;
            while (starts) {
                int b = __ffs(starts) - 1;
                starts &= starts - 1;
                sstart[wave][o++] = (uint16_t)(16 * (ch - 1) + b);   // tile-relative offset
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            my_tokens += (lane == 0) ? (u64)total : 0;

            for (int i = lane; i < total; i += 64) {
                const int off = sstart[wave][i];
                const int rp = MAP_PRE + off;                       // region position
                const int wi = rp >> 4, bi = rp & 15;
                u64 w64 = (u64)smask[wi] | ((u64)smask[wi + 1] << 16) | ((u64)smask[wi + 2] << 32) |
                          ((u64)smask[wi + 3] << 48);
                u64 v = ~(w64 >> bi);
                int len = v ? __ffsll((long long)v) - 1 : 64;
                if (len >= 16) {
                    my_long++;
                    long_token(a, (u64)(base + off));
                    continue;
                }
                // key bytes [rp, rp+16) from LDS via 5 aligned dwords
                const int al = rp & ~3, sh = rp & 3;
                const u32* d = reinterpret_cast<const u32*>(sbytes + al);
                u32 d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3], d4 = d[4];
                u32 o0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
                u32 o1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
                u32 o2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
                u32 o3 = __builtin_amdgcn_alignbyte(d4, d3, sh);
                u64 k0 = ((u64)o1 << 32 | o0) & low_bytes_mask(len);
                u64 k1 = len > 8 ? (((u64)o3 << 32 | o2) & low_bytes_mask(len - 8)) : 0ull;
                k1 |= (u64)len << 56;
                const u64 h = key_hash(k0, k1);
                // ---- LDS table
                u32 s = __umulhi((u32)(h >> 32), (u32)LDS_SLOTS);
                bool done = false;
                for (int p = 0; p < LDS_MAXPROBE && !done; p++) {
                    u64 c0 = skey[s][0];
                    bool adv = true;
                    if (c0 == 0) {
                        u64 old = atomicCAS(&skey[s][0], 0ull, k0);
                        if (old == 0) {
                            skey[s][1] = k1;
                            atomicAdd(&scnt[s], 1u);
                            done = true;
                        } else if (old == k0) {
                            adv = false;                     // same first 8 bytes: re-read k1
                        }
                    } else if (c0 == k0) {
                        u64 c1 = skey[s][1];
                        if (c1 == k1) { atomicAdd(&scnt[s], 1u); done = true; }
                        else if (c1 == 0) adv = false;        // being published
                    }
                    if (!done && adv) { s++; if (s == (u32)LDS_SLOTS) s = 0; }
                }
                if (done) { my_hits++; }
                else { my_global++; ginsert(a.gtab, a.gmask, k0, k1, h, 1, a.st); }
            }
        }
        __syncthreads();
    }

    // ---- flush the LDS table into the global table
    for (int i = tid; i < LDS_SLOTS; i += MAP_NT) {
        u32 c = scnt[i];
        if (c) {
            u64 k0 = skey[i][0], k1 = skey[i][1];
            ginsert(a.gtab, a.gmask, k0, k1, key_hash(k0, k1), c, a.st);
            my_global++;
        }
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
