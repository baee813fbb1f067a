// wcg_reduce.h - DoReduce + Merge on gfx950 (mapreduce.go:239-321, wc.go:35-38).
//
//   k_compact   global tables -> dense records {128-bit big-endian prefix, count, ref}
//   k_hist16    one pass over the records: global histogram of all 16 prefix bytes, so the
//               host can skip sort passes whose digit is constant (fact F4 makes the
//               zero-padded prefix Go's sort.Strings order for keys <= 15 bytes)
//   k_digit_hist / k_scan / k_scatter   one stable LSD radix pass over an 8-bit digit
//   k_ties      long keys (> 15 bytes) that share a 16-byte prefix: ordered by full bytes
//   k_linelen / k_scan / k_write        "key: count\n" (Merge, mapreduce.go:316-318) or
//               {"Key":"k","Value":"count"}\n for ihash(k)%R == r (DoReduce, :274-278)
#pragma once
#include "wcg_common.h"
#include "wcg_lds_table.h"

namespace wcg {

constexpr int RS_NT = 256;            // threads per sort block
constexpr int RS_IPT = 8;             // records per thread
constexpr int RS_TILE = RS_NT * RS_IPT;

// ---------------------------------------------------------------- compaction
__global__ void k_compact(const GEntry* gtab, u64 gslots, const GEntry* ltab, u64 lslots, const uint8_t* arena,
                          Rec* out, DevState* st) {
    const u64 total = gslots + lslots;
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i - threadIdx.x < total; i += (u64)gridDim.x * blockDim.x) {
        Rec r;
        bool have = false;
        if (i < gslots) {
            GEntry e = gtab[i];
            if (e.k0 != 0) {
                have = true;
                if (key_short(e.k0)) {
                    r.hi = bswap64(e.k0 & 0x00FFFFFFFFFFFFFFull);
                    r.lo = 0;
                    r.ref = e.k0 >> 56;
                } else {
                    r.hi = bswap64(e.k0);
                    r.lo = bswap64(e.k1 & 0x00FFFFFFFFFFFFFFull);
                    r.ref = e.k1 >> 56;
                }
                r.cnt = e.cnt;
            }
        } else if (i < total) {
            GEntry e = ltab[i - gslots];
            if (e.k0 != 0) {
                have = true;
                u64 off = e.k1 - 1, len = e.aux;
                u64 hi = 0, lo = 0;
                for (int k = 0; k < 8; k++) hi = (hi << 8) | arena[off + k];
                for (int k = 8; k < 16; k++) lo = (lo << 8) | arena[off + k];
                r.hi = hi; r.lo = lo; r.cnt = e.cnt;
                r.ref = LONG_FLAG | (len << 40) | off;
            }
        }
        u64 bal = __ballot(have);
        if (bal == 0) continue;
        const int lane = threadIdx.x & 63;
        u64 base = 0;
        int leader = __ffsll((long long)bal) - 1;
        if (lane == leader) base = atomicAdd(&st->nrec, (u64)__popcll(bal));
        base = __shfl(base, leader, 64);
        if (have) out[base + __popcll(bal & ((1ull << lane) - 1))] = r;
    }
}

__device__ __forceinline__ u32 rec_digit(const Rec& r, int d) {
    return d < 8 ? (u32)(r.lo >> (8 * d)) & 0xFF : (u32)(r.hi >> (8 * (d - 8))) & 0xFF;
}

__global__ void k_hist16(const Rec* recs, u64 n, DevState* st) {
    __shared__ u32 h[16][256];
    for (int i = threadIdx.x; i < 16 * 256; i += blockDim.x) (&h[0][0])[i] = 0;
    __syncthreads();
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        Rec r = recs[i];
#pragma unroll
        for (int d = 0; d < 16; d++) atomicAdd(&h[d][rec_digit(r, d)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 16 * 256; i += blockDim.x) {
        u32 v = (&h[0][0])[i];
        if (v) atomicAdd(&(&st->hist[0][0])[i], (u64)v);
    }
}

// per-block digit histogram, digit-major: bh[d * nblocks + b]
__global__ __launch_bounds__(RS_NT) void k_digit_hist(const Rec* recs, u64 n, int d, u32* bh, u32 nblocks) {
    __shared__ u32 h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const u64 b0 = (u64)blockIdx.x * RS_TILE;
    for (int j = 0; j < RS_IPT; j++) {
        u64 i = b0 + (u64)j * RS_NT + threadIdx.x;
        if (i < n) atomicAdd(&h[rec_digit(recs[i], d)], 1u);
    }
    __syncthreads();
    bh[(u64)threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

// exclusive scan of u32 (in place) by one workgroup of 1024 threads; returns total in *total
__global__ __launch_bounds__(1024) void k_scan_u32(u32* v, u64 n, u64* total) {
    __shared__ u32 ws[16];
    __shared__ u32 carry_s;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) carry_s = 0;
    __syncthreads();
    for (u64 base = 0; base < n; base += 1024 * 4) {
        u32 x[4], s = 0;
        for (int k = 0; k < 4; k++) {
            u64 i = base + (u64)tid * 4 + k;
            x[k] = i < n ? v[i] : 0;
            s += x[k];
        }
        u32 incl = s;
        for (int d = 1; d < 64; d <<= 1) { u32 y = __shfl_up(incl, d, 64); if (lane >= d) incl += y; }
        if (lane == 63) ws[w] = incl;
        __syncthreads();
        u32 wpre = 0, all = 0;
        for (int k = 0; k < 16; k++) { if (k < w) wpre += ws[k]; all += ws[k]; }
        u32 run = carry_s + wpre + incl - s;
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

// stable scatter for digit d; records of a block are ranked in index order
__global__ __launch_bounds__(RS_NT) void k_scatter(const Rec* in, Rec* out, u64 n, int d, const u32* boff, u32 nblocks) {
    __shared__ u32 run[256];          // block-local count of each digit so far
    __shared__ u32 wh[RS_NT / 64][256];
    __shared__ u32 goff[256];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    run[tid] = 0;
    goff[tid] = boff[(u64)tid * nblocks + blockIdx.x];
    const u64 b0 = (u64)blockIdx.x * RS_TILE;
    for (int j = 0; j < RS_IPT; j++) {
        for (int k = 0; k < RS_NT / 64; k++) wh[k][tid] = 0;
        __syncthreads();
        u64 i = b0 + (u64)j * RS_NT + tid;
        bool valid = i < n;
        Rec r;
        u32 dg = 0;
        if (valid) { r = in[i]; dg = rec_digit(r, d); }
        // lanes of this wave holding the same digit
        u64 peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            u64 bb = __ballot((dg >> b) & 1);
            peers &= ((dg >> b) & 1) ? bb : ~bb;
        }
        u32 rank_in_wave = (u32)__popcll(peers & ((1ull << lane) - 1));
        if (valid && rank_in_wave == 0) wh[w][dg] = (u32)__popcll(peers);
        __syncthreads();
        // digit tid: offsets of each wave = run + counts of earlier waves
        u32 acc = run[tid];
        for (int k = 0; k < RS_NT / 64; k++) { u32 c = wh[k][tid]; wh[k][tid] = acc; acc += c; }
        run[tid] = acc;
        __syncthreads();
        if (valid) out[goff[dg] + wh[w][dg] + rank_in_wave] = r;
        __syncthreads();
    }
}

// ---------------------------------------------------------------- long-key ties
__device__ int cmp_full(const Rec& a, const Rec& b, const uint8_t* arena) {
    // both long: compare full bytes
    u64 la = (a.ref >> 40) & LONG_LEN_MAX, lb = (b.ref >> 40) & LONG_LEN_MAX;
    const uint8_t* pa = arena + (a.ref & LONG_OFF_MASK);
    const uint8_t* pb = arena + (b.ref & LONG_OFF_MASK);
    u64 m = la < lb ? la : lb;
    for (u64 i = 0; i < m; i++) if (pa[i] != pb[i]) return pa[i] < pb[i] ? -1 : 1;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

__global__ void k_tie_detect(const Rec* r, u64 n, DevState* st) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i + 1 < n; i += (u64)gridDim.x * blockDim.x)
        if (r[i].hi == r[i + 1].hi && r[i].lo == r[i + 1].lo) atomicOr(&st->tie_flag, 1u);
}

// one thread per run of equal prefixes: insertion sort by full key bytes
__global__ void k_tie_fix(Rec* r, u64 n, const uint8_t* arena) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i + 1 < n; i += (u64)gridDim.x * blockDim.x) {
        bool start = (r[i].hi == r[i + 1].hi && r[i].lo == r[i + 1].lo) &&
                     (i == 0 || r[i - 1].hi != r[i].hi || r[i - 1].lo != r[i].lo);
        if (!start) continue;
        u64 e = i + 1;
        while (e + 1 < n && r[e + 1].hi == r[i].hi && r[e + 1].lo == r[i].lo) e++;
        for (u64 a = i + 1; a <= e; a++) {
            Rec x = r[a];
            u64 b = a;
            while (b > i && cmp_full(r[b - 1], x, arena) > 0) { r[b] = r[b - 1]; b--; }
            r[b] = x;
        }
    }
}

// ---------------------------------------------------------------- formatting
__device__ __forceinline__ u32 ndigits(u64 v) {
    u32 d = 1;
    while (v >= 10) { v /= 10; d++; }
    return d;
}
__device__ __forceinline__ u64 rec_len(const Rec& r) { return (r.ref & LONG_FLAG) ? ((r.ref >> 40) & LONG_LEN_MAX) : r.ref; }
__device__ __forceinline__ u32 rec_byte(const Rec& r, u64 k, const uint8_t* arena) {
    if (r.ref & LONG_FLAG) return arena[(r.ref & LONG_OFF_MASK) + k];
    return k < 8 ? (u32)(r.hi >> (56 - 8 * k)) & 0xFF : (u32)(r.lo >> (56 - 8 * (k - 8))) & 0xFF;
}
__device__ u32 rec_ihash(const Rec& r, const uint8_t* arena) {
    u32 h = 0x811C9DC5u;
    u64 len = rec_len(r);
    for (u64 k = 0; k < len; k++) h = fnv1a_step(h, rec_byte(r, k, arena));
    return h;
}

constexpr int FMT_MERGED = 0, FMT_JSON = 1;
constexpr u64 JSON_FIXED = 8 + 11 + 3;   // {"Key":" + ","Value":" + "}\n

__global__ void k_linelen(const Rec* r, u64 n, int fmt, u32 nreduce, u32 part, const uint8_t* arena, u64* len) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        Rec x = r[i];
        u64 L;
        if (fmt == FMT_MERGED) L = rec_len(x) + 3 + ndigits(x.cnt);
        else L = (rec_ihash(x, arena) % nreduce == part) ? rec_len(x) + JSON_FIXED + ndigits(x.cnt) : 0;
        len[i] = L;
    }
}

__global__ void k_write(const Rec* r, u64 n, int fmt, u32 nreduce, u32 part, const uint8_t* arena, const u64* off,
                        uint8_t* out) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        Rec x = r[i];
        if (fmt == FMT_JSON && rec_ihash(x, arena) % nreduce != part) continue;
        uint8_t* o = out + off[i];
        u64 len = rec_len(x);
        if (fmt == FMT_JSON) {
            const char* pre = "{\"Key\":\"";
            for (int k = 0; k < 8; k++) *o++ = pre[k];
        }
        for (u64 k = 0; k < len; k++) *o++ = (uint8_t)rec_byte(x, k, arena);
        if (fmt == FMT_JSON) {
            const char* mid = "\",\"Value\":\"";
            for (int k = 0; k < 11; k++) *o++ = mid[k];
        } else {
            *o++ = ':'; *o++ = ' ';
        }
        u32 nd = ndigits(x.cnt);
        u64 c = x.cnt;
        for (int k = (int)nd - 1; k >= 0; k--) { o[k] = (uint8_t)('0' + c % 10); c /= 10; }
        o += nd;
        if (fmt == FMT_JSON) { *o++ = '"'; *o++ = '}'; }
        *o = '\n';
    }
}

// ---------------------------------------------------------------- multi-GPU shuffle
// Exchange unit = 32 bytes.  An inline key is one unit (a Rec).  A long key is a header unit
// {hi, lo, cnt, LONG_FLAG | len << 40} followed by ceil(len / 24) continuation units, each
// carrying 24 key bytes in {hi, lo, cnt} and CONT_MARK in ref - so every unit says what it is
// and import runs fully in parallel.  owner = (ihash(key) % nreduce) % nranks.
constexpr u64 CONT_MARK = 1ull << 62;
constexpr int CONT_BYTES = 24;

__device__ __forceinline__ u64 rec_units(const Rec& r) {
    return (r.ref & LONG_FLAG) ? 1 + ((rec_len(r) + CONT_BYTES - 1) / CONT_BYTES) : 1;
}

__global__ void k_export_count(const Rec* r, u64 n, u32 nreduce, u32 nranks, const uint8_t* arena, u32* owner,
                               u64* per_rank) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        Rec x = r[i];
        u32 o = (rec_ihash(x, arena) % nreduce) % nranks;
        owner[i] = o;
        atomicAdd(&per_rank[o], rec_units(x));
    }
}

// cursor[o] starts at the exclusive prefix of per_rank; order inside a destination is
// irrelevant (the receiver re-aggregates and re-sorts).
__global__ void k_export_write(const Rec* r, u64 n, const u32* owner, u64* cursor, const uint8_t* arena, Rec* out) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        Rec x = r[i];
        u64 u = rec_units(x);
        u64 pos = atomicAdd(&cursor[owner[i]], u);
        if (!(x.ref & LONG_FLAG)) { out[pos] = x; continue; }
        u64 len = rec_len(x);
        Rec h = x;
        h.ref = LONG_FLAG | (len << 40);
        out[pos] = h;
        const uint8_t* src = arena + (x.ref & LONG_OFF_MASK);
        for (u64 c = 1; c < u; c++) {
            u64 w[3] = {0, 0, 0};
            for (int k = 0; k < CONT_BYTES; k++) {
                u64 q = (c - 1) * CONT_BYTES + k;
                u64 b = q < len ? src[q] : 0;
                w[k >> 3] |= b << (8 * (k & 7));
            }
            Rec cr;
            cr.hi = w[0]; cr.lo = w[1]; cr.cnt = w[2]; cr.ref = CONT_MARK;
            out[pos + c] = cr;
        }
    }
}

__device__ __forceinline__ uint8_t cont_byte(const Rec* units, u64 k) {
    const Rec& c = units[k / CONT_BYTES];
    int q = (int)(k % CONT_BYTES);
    u64 w = q < 8 ? c.hi : (q < 16 ? c.lo : c.cnt);
    return (uint8_t)(w >> (8 * (q & 7)));
}

__global__ void k_import(const Rec* in, u64 n, GEntry* gtab, u64 gmask, GEntry* ltab, u64 lmask, uint8_t* arena,
                         u64 arena_cap, DevState* st) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        Rec x = in[i];
        if (x.ref == CONT_MARK) continue;
        if (!(x.ref & LONG_FLAG)) {
            u64 k0, k1;
            make_key(bswap64(x.hi), bswap64(x.lo), (int)x.ref, k0, k1);
            ginsert(gtab, gmask, k0, k1, gslot(key_hash(k0, k1)), x.cnt, st);
            continue;
        }
        u64 len = (x.ref >> 40) & LONG_LEN_MAX;
        const Rec* src = in + i + 1;
        if (i + 1 + (len + CONT_BYTES - 1) / CONT_BYTES > n) { atomicAdd(&st->overflow, 1u); continue; }
        u64 h = 0xCBF29CE484222325ull;
        for (u64 k = 0; k < len; k++) { h ^= cont_byte(src, k); h *= 0x100000001B3ull; }
        u64 tag = mix64(h ^ len) | 1ull;
        u64 s = tag & lmask, probes = 0;
        int spins = 0;
        while (true) {
            GEntry* e = &ltab[s];
            u64 c0 = ld_agent(&e->k0);
            if (c0 == 0) {
                u64 exp = 0;
                if (cas_agent(&e->k0, &exp, tag)) {
                    u64 off = atomicAdd(&st->arena_top, len);
                    if (off + len > arena_cap) { atomicAdd(&st->overflow, 1u); break; }
                    for (u64 k = 0; k < len; k++) arena[off + k] = cont_byte(src, k);
                    st_agent(&e->aux, len);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    st_agent(&e->k1, off + 1);
                    add_agent(&e->cnt, x.cnt);
                    break;
                }
                c0 = exp;
            }
            if (c0 == tag) {
                u64 rr = ld_agent(&e->k1);
                if (rr == 0) {
                    if (++spins > SPIN_LIMIT) { atomicAdd(&st->spin_fail, 1u); break; }
                    continue;
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                bool same = ld_agent(&e->aux) == len;
                for (u64 k = 0; same && k < len; k++) same = arena[rr - 1 + k] == cont_byte(src, k);
                if (same) { add_agent(&e->cnt, x.cnt); break; }
            }
            s = (s + 1) & lmask;
            if (++probes > lmask) { atomicAdd(&st->overflow, 1u); break; }
        }
    }
}

}  // namespace wcg
