// wcg_map.h - the map kernel: DoMap + Map (mapreduce.go:193-231, wc.go:17-30) on gfx950.
//
// One workgroup (16 waves) per CU owns a contiguous range of 1 KiB steps; wave w of the
// workgroup processes steps w, w+16, w+32, ... of that range on its own - its own LDS slice,
// no workgroup barrier in the main loop, so the 16 waves overlap each other's latencies:
//   1. every lane loads one 16-byte chunk of the step (one coalesced 1 KiB dwordx4 load per
//      wave), lanes 0-4 also the 16-byte prefix and the 64-byte look-ahead that lets tokens
//      crossing the step end be read whole; the loads run 2 steps ahead in registers;
//   2. per chunk: 16-bit letter-byte mask - SWAR on all-ASCII chunks (fact F2), Go UTF-8
//      decode + Unicode-13 letter bitmap otherwise (fact F1);
//   3. token starts = letter & ~prev_letter (fact F3); the wave compacts them (prefix sum from
//      4 ballots + mbcnt) into its LDS list and processes them 64 at a time;
//   4. per token: length from the mask, key identity (<= 15 bytes, fact F4) -> the
//      workgroup's LDS tables (exact keys; short and medium keys in separate 2-choice x 1-slot
//      tables, u32 counts: MapTable); an LDS miss is appended to this workgroup's region of the
//      miss log (plain stores) for k_agg; tokens > 15 bytes go to the long-key table with an
//      arena copy of their bytes;
//   5. at the end the workgroup flushes its LDS table into the miss log too.
// Token ownership: a token belongs to the 16-byte chunk holding its first byte (exactly once).
#pragma once
#include <type_traits>

#include "wcg_common.h"
#include "wcg_lds_table.h"

namespace wcg {

constexpr int MAP_NT = 1024;                 // threads per workgroup
constexpr int MAP_WAVES = MAP_NT / 64;       // 16 independent waves
constexpr int MAP_STEP = 1024;               // bytes per wave step (64 lanes x 16 B)
constexpr int MAP_PRE = 16;                  // prefix bytes (need 4)
constexpr int MAP_LOOK = 64;                 // look-ahead bytes (tokens <= 15 need 15)
constexpr int MAP_WREG = MAP_PRE + MAP_STEP + MAP_LOOK;   // 1104 = 69 chunks
constexpr int MAP_WNCH = MAP_WREG / 16;
constexpr int MAP_WMASK = 72;                // mask slots per wave (69 + padding)
constexpr int MAP_NS = 8800;                 // LDS short-key slots (12 B each)
constexpr int MAP_NM = 1024;                 // LDS medium-key slots (20 B each)
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
    u64* pool;     u64 region_cap;  // miss log: region (wg, p) = pool[(wg * P + p) * region_cap ...]
    u32* region_len;               // units written per region
    u32 pmask;                     // P - 1 (P = number of miss buckets, power of two)
};

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
//   5 = input loads only, 4 = + LDS staging and letter masks, 1 = + token starts and compaction,
//   2 = + key extraction and hash, 3 = + LDS lookup with misses dropped
template <int ABL>
__global__ __launch_bounds__(MAP_NT) void k_map(MapArgs a) {
    __shared__ __align__(16) uint8_t wbytes[MAP_WAVES][MAP_WREG];
    __shared__ __align__(16) uint16_t wmask[MAP_WAVES][MAP_WMASK];
    __shared__ uint16_t wstart[MAP_WAVES][512];
    __shared__ __align__(16) u64 sk0[MAP_NS];
    __shared__ __align__(16) u64 mk0[MAP_NM];
    __shared__ __align__(16) u64 mk1[MAP_NM];
    __shared__ u64 zero_w;
    __shared__ u32 scnt[MAP_NS];
    __shared__ u32 mcnt[MAP_NM];
    __shared__ u32 cursor[MAX_MISS_BUCKETS];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);     // wave-uniform (scalar)
    MapTable<MAP_NS, MAP_NM> tab{sk0, scnt, mk0, mk1, mcnt, &zero_w};
    tab.init(tid, MAP_NT);
    for (int i = tid; i < MAX_MISS_BUCKETS; i += MAP_NT) cursor[i] = 0;
    if (lane < MAP_WMASK - MAP_WNCH) wmask[wave][MAP_WNCH + lane] = 0;
    __syncthreads();

    uint8_t* const bytes = wbytes[wave];
    uint16_t* const msk = wmask[wave];
    uint16_t* const sst = wstart[wave];
    // Steps are dealt chip-wide: wave w of workgroup g takes steps (g * 16 + w) + k * G * 16, so
    // the chip sweeps the input front to back (HBM-friendly) while every workgroup still sees
    // a uniform sample of it for its LDS table.
    const u64 nsteps = a.ntiles;
    const u64 stride = (u64)gridDim.x * MAP_WAVES;
    // region chunk c <-> input bytes [step_base - PRE + 16c, +16): lane owns chunk lane+1;
    // lane 0 also chunk 0 (prefix), lane 63 chunk 65 (first look-ahead chunk, its DPP "next"),
    // lanes 1-3 chunks 66-68 (rest of the 64-byte look-ahead used by the UTF-8 path)
    const int xc = (lane == 0) ? 0 : (lane == 63 ? 65 : (lane <= 3 ? 65 + lane : -1));
    u64 my_tokens = 0;                           // wave-uniform
    u32 my_hits = 0, my_global = 0, my_long = 0;

    // Input loads: raw buffer loads through a per-step descriptor based at the step's prefix
    // (at the input start for step 0); the hardware range check returns zeros for the prefix
    // of step 0 and past the end.  Every prefetch is unconditional (the waitcnt pass can only
    // count younger loads that are certainly issued): lanes without an extra chunk and steps
    // past the end load offset 0xFFFFFFF0, which reads zeros without touching memory.
    auto load = [&](auto set, u64 step, v4u& m, v4u& x) {      // set: 0 = A registers, 1 = B
        const bool live = step < nsteps;
        const u64 org = (step == 0 || !live) ? 0 : step * MAP_STEP - MAP_PRE;
        const u64 span = live ? a.n - org : 0;
        const u32 nrec = span > 0xFFFFFFFFull ? 0xFFFFFFFFu : (u32)span;
        const v4i rsrc = make_rsrc(a.in + org, nrec);
        const u32 rel = (u32)(step * MAP_STEP - org);            // 0 for step 0, else 16
        const u32 om = live ? rel + 16 * lane : 0xFFFFFFF0u;
        const u32 ox = (live && xc >= 0) ? rel - MAP_PRE + 16 * xc : 0xFFFFFFF0u;
        if constexpr (decltype(set)::value == 0) {
            m = buf_load16_A0(rsrc, om);
            x = buf_load16_A1(rsrc, ox);
        } else {
            m = buf_load16_B0(rsrc, om);
            x = buf_load16_B1(rsrc, ox);
        }
    };

    // miss handling shared by both paths
    auto miss = [&](u64 k0, u64 k1, u32 h) {
        if (!log_push(a, cursor, miss_bucket(h, a.pmask), k0, k1, 1u)) {
            my_global++;
            ginsert(a.gtab, a.gmask, k0, k1, gslot(key_hash(k0, k1)), 1, a.st);
        }
    };

    auto process = [&](u64 step, const uint4 mine, const uint4 extra) {
        const long base = (long)(step * MAP_STEP);
        if (ABL == 5) { asm volatile("" ::"v"(mine.x ^ extra.y)); return; }
        reinterpret_cast<uint4*>(bytes)[lane + 1] = mine;
        if (xc >= 0) reinterpret_cast<uint4*>(bytes)[xc] = extra;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // ---- letter masks
        auto at = [&](long i) -> u32 { return (i >= 0 && i < MAP_WREG) ? (u32)bytes[i] : 0u; };
        {
            u32 m;
            if (all_ascii(mine)) {
                m = ascii_mask16(mine);
            } else {
                m = 0;
                for (int i = 0; i < 16; i++)
                    if (letter_byte(at, (long)(16 * (lane + 1) + i))) m |= 1u << i;
            }
            msk[lane + 1] = (uint16_t)m;
            if (xc >= 0) {
                if (all_ascii(extra)) {
                    m = ascii_mask16(extra);
                } else {
                    m = 0;
                    for (int i = (xc == 0 ? 4 : 0); i < 16; i++)   // prefix chunk: only its tail matters
                        if (letter_byte(at, (long)(16 * xc + i))) m |= 1u << i;
                }
                msk[xc] = (uint16_t)m;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (ABL == 4) { asm volatile("" ::"v"((u32)msk[lane + 1])); return; }
        // ---- token starts in my chunk; wave prefix sum of the counts (<= 8) from 4 ballots
        const u32 m = msk[lane + 1];
        const u32 prev = msk[lane] >> 15;
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
            sst[o++] = (uint16_t)(16 * lane + b);               // step-relative offset
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        my_tokens += total;

        // ---- tokens, one per lane per iteration (two per lane with both probes in flight was
        //      measured slower: ~177 tokens per step fill 3 x 64 slots but 2 x 128)
        u32 sink = 0;
        auto token_key = [&](int off, int& len, u64& k0, u64& k1) {
            const int rp = MAP_PRE + off;                       // region position
            const int wi = rp >> 4, bi = rp & 15;
            const u32 w32 = (u32)msk[wi] | ((u32)msk[wi + 1] << 16);
            const u32 v = ~(w32 >> bi);                         // >= 17 valid bits
            len = v ? __ffs(v) - 1 : 32;                        // v == 0: run covers the window
            // key bytes [rp, rp+16) from LDS via 5 aligned dwords
            const int al = rp & ~3, sh = rp & 3;
            const u32* d = reinterpret_cast<const u32*>(bytes + al);
            const u32 d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3], d4 = d[4];
            const u32 o0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
            const u32 o1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
            const u32 o2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
            const u32 o3 = __builtin_amdgcn_alignbyte(d4, d3, sh);
            const int kl = len < 16 ? len : 15;
            const u64 b0 = ((u64)o1 << 32 | o0) & low_bytes_mask(kl);
            const u64 b1 = kl > 8 ? (((u64)o3 << 32 | o2) & low_bytes_mask(kl - 8)) : 0ull;
            make_key(b0, b1, kl, k0, k1);
        };
        for (u32 i = lane; i < total; i += 64) {
            if (ABL == 1) { sink += sst[i]; continue; }
            const int off = sst[i];
            int len;
            u64 k0, k1;
            token_key(off, len, k0, k1);
            if (len >= 16) { my_long++; long_token(a, (u64)(base + off)); continue; }
            const u32 h = lds_hash(k0, k1);
            if (ABL == 2) { sink += h; continue; }
            const bool hit = tab.add(k0, k1, h);
            if (ABL == 3) { sink += hit; continue; }
            my_hits += (u32)hit;
            if (!hit) miss(k0, k1, h);
        }
        if (ABL) asm volatile("" ::"v"(sink));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };

    // two steps in flight per wave (A/B register sets, no copies between them).  A wave's
    // steps increase, so once one reaches past the input end (a "tail" step) all later ones do:
    // the main loop stops there and the tail steps are reloaded byte-exactly after it (keeping
    // the cold reload path's registers out of the loop)
    auto is_tail = [&](u64 step) { return step * MAP_STEP + MAP_STEP + MAP_LOOK > a.n; };
    auto u4 = [](v4u v) { return make_uint4(v.x, v.y, v.z, v.w); };
    v4u ma, xa, mb, xb;
    u64 st = (u64)blockIdx.x * MAP_WAVES + wave;
    const std::integral_constant<int, 0> SA;
    const std::integral_constant<int, 1> SB;
    load(SA, st, ma, xa);
    load(SB, st + stride, mb, xb);
    while (st < nsteps && !is_tail(st)) {
        buf_wait_A<2>(ma, xa);                   // younger: B's two loads
        process(st, u4(ma), u4(xa));
        load(SA, st + 2 * stride, ma, xa);
        st += stride;
        if (st >= nsteps || is_tail(st)) break;
        buf_wait_B<2>(mb, xb);                   // younger: A's two loads
        process(st, u4(mb), u4(xb));
        load(SB, st + 2 * stride, mb, xb);
        st += stride;
    }
    buf_wait_A<0>(ma, xa);                       // nothing may land in a dead register
    buf_wait_B<0>(mb, xb);
    for (; st < nsteps; st += stride) {
        const long org = (long)(st * MAP_STEP) - MAP_PRE;
        const uint4 mine = load_chunk(a.in, a.n, org + 16 * (lane + 1));
        const uint4 extra = xc >= 0 ? load_chunk(a.in, a.n, org + 16 * xc) : make_uint4(0, 0, 0, 0);
        process(st, mine, extra);
    }

    // ---- flush the LDS table into this workgroup's miss-log regions (entries with counts);
    //      a full region -> global table
    __syncthreads();
    auto flush = [&](u64 k0, u64 k1, u32 c) {
        if (!c) return;
        if (!log_push(a, cursor, miss_bucket(lds_hash(k0, k1), a.pmask), k0, k1, c)) {
            my_global++;
            ginsert(a.gtab, a.gmask, k0, k1, gslot(key_hash(k0, k1)), c, a.st);
        }
    };
    for (int i = tid; i < MAP_NS; i += MAP_NT) flush(sk0[i], 0, scnt[i]);
    for (int i = tid; i < MAP_NM; i += MAP_NT) flush(mk0[i], mk1[i], mcnt[i]);
    __syncthreads();
    for (u32 p = tid; p <= a.pmask; p += MAP_NT) {
        const u32 c = cursor[p];
        a.region_len[(u64)blockIdx.x * (a.pmask + 1) + p] = c < a.region_cap ? c : (u32)a.region_cap;
    }
    // stats: one atomic per wave
    u64 v0 = lane == 0 ? my_tokens : 0, v1 = my_hits, v2 = my_global, v3 = my_long;
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
