// wcg_reduce.h - DoReduce + Merge on gfx950 (mapreduce.go:239-321, wc.go:35-38).
//
//   k_compact   global tables -> dense records {128-bit big-endian prefix, count, ref}
//   k_tile_sort / k_merge   merge sort by the 128-bit big-endian prefix (fact F4 makes the
//               zero-padded prefix Go's sort.Strings order for keys <= 15 bytes)
//   k_tie_fix   long keys (> 15 bytes) that share a 16-byte prefix: ordered by full bytes
//   k_fmt_sum / k_scan_u64 / k_fmt_write  "key: count\n" (Merge, mapreduce.go:316-318) or
//               {"Key":"k","Value":"count"}\n for ihash(k)%R == r (DoReduce, :274-278)
#pragma once
#include "wcg_common.h"
#include "wcg_lds_table.h"

namespace wcg {

// ---------------------------------------------------------------- compaction
constexpr int CP_NT = 256, CP_IPT = 8;          // 2048 table slots per block, one atomic each

__device__ __forceinline__ bool slot_to_rec(const GEntry* gtab, u64 gslots, const GEntry* ltab, u64 total, u64 i,
                                            const uint8_t* arena, Rec& r) {
    if (i < gslots) {
        const GEntry e = gtab[i];
        if (e.k0 == 0) return false;
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
        return true;
    }
    if (i >= total) return false;
    const GEntry e = ltab[i - gslots];
    if (e.k0 == 0) return false;
    const u64 off = e.k1 - 1, len = e.aux;
    u64 hi = 0, lo = 0;
    for (int k = 0; k < 8; k++) hi = (hi << 8) | arena[off + k];
    for (int k = 8; k < 16; k++) lo = (lo << 8) | arena[off + k];
    r.hi = hi; r.lo = lo; r.cnt = e.cnt;
    r.ref = LONG_FLAG | (len << 40) | off;
    return true;
}

__global__ __launch_bounds__(CP_NT) void k_compact(const GEntry* gtab, u64 gslots, const GEntry* ltab, u64 lslots,
                                                  const uint8_t* arena, Rec* out, DevState* st) {
    __shared__ u32 wsum[CP_NT / 64];
    __shared__ u64 base_s;
    const u64 total = gslots + lslots;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u64 b0 = (u64)blockIdx.x * CP_NT * CP_IPT;
    Rec r[CP_IPT];
    u32 have = 0, nlong = 0;
#pragma unroll
    for (int j = 0; j < CP_IPT; j++)
        if (slot_to_rec(gtab, gslots, ltab, total, b0 + (u64)j * CP_NT + tid, arena, r[j])) {
            have |= 1u << j;
            nlong += (r[j].ref & LONG_FLAG) ? 1 : 0;
        }
    if (nlong) atomicAdd(&st->nlong, (u64)nlong);
    const u32 cnt = __popc(have);
    // block exclusive prefix of cnt (<= 8 per thread): 4 ballots per wave, then waves in order
    u32 o = 0, wt = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
        const u64 bal = __ballot((cnt >> b) & 1);
        o += __builtin_amdgcn_mbcnt_hi((u32)(bal >> 32), __builtin_amdgcn_mbcnt_lo((u32)bal, 0u)) << b;
        wt += (u32)__popcll(bal) << b;
    }
    if (lane == 0) wsum[w] = wt;
    __syncthreads();
    if (tid == 0) {
        u32 all = 0;
        for (int k = 0; k < CP_NT / 64; k++) { const u32 v = wsum[k]; wsum[k] = all; all += v; }
        base_s = all ? atomicAdd(&st->nrec, (u64)all) : 0;
    }
    __syncthreads();
    u64 pos = base_s + wsum[w] + o;
#pragma unroll
    for (int j = 0; j < CP_IPT; j++)
        if (have & (1u << j)) out[pos++] = r[j];
}

// ---------------------------------------------------------------- sort
// Merge sort on the 128-bit big-endian prefix: k_tile_sort orders each 2048-record tile with an
// LDS bitonic network, then log2(n / 2048) k_merge passes double the sorted run length.  Cost
// does not depend on the key distribution (a radix sort's MSD buckets collapse on UTF-8 text,
// where every word of a script shares its first byte or two) and no pass needs the host.
constexpr int TS_NT = 1024, TS_TILE = 2048;
constexpr int MG_NT = 256, MG_CHUNK = 1024;

__device__ __forceinline__ bool pre_lt(u64 ah, u64 al, u64 bh, u64 bl) { return ah < bh || (ah == bh && al < bl); }

__global__ __launch_bounds__(TS_NT) void k_tile_sort(const Rec* in, Rec* out, u64 n) {
    __shared__ u64 sh[TS_TILE], sl[TS_TILE];
    __shared__ uint16_t si[TS_TILE];
    const u64 base = (u64)blockIdx.x * TS_TILE;
    const int tid = threadIdx.x;
    for (int k = 0; k < TS_TILE / TS_NT; k++) {
        const int i = k * TS_NT + tid;
        const u64 g = base + i;
        if (g < n) {
            const Rec r = in[g];
            sh[i] = r.hi; sl[i] = r.lo;
        } else {                                  // padding: no key has an all-0xFF prefix
            sh[i] = ~0ull; sl[i] = ~0ull;
        }
        si[i] = (uint16_t)i;
    }
    __syncthreads();
    for (int k = 2; k <= TS_TILE; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
            for (int q = 0; q < TS_TILE / 2 / TS_NT; q++) {
                const int t = q * TS_NT + tid;               // compare-exchange pair t
                const int i = 2 * t - (t & (j - 1)), p = i + j;
                const u64 ah = sh[i], al = sl[i], bh = sh[p], bl = sl[p];
                if (pre_lt(bh, bl, ah, al) == ((i & k) == 0)) {
                    sh[i] = bh; sl[i] = bl; sh[p] = ah; sl[p] = al;
                    const uint16_t x = si[i]; si[i] = si[p]; si[p] = x;
                }
            }
            __syncthreads();
        }
    }
    for (int k = 0; k < TS_TILE / TS_NT; k++) {
        const int i = k * TS_NT + tid;
        if (base + i < n) out[base + i] = in[base + si[i]];
    }
}

// merge path: number of A records among the first d outputs of merge(A, B) (A first on equal
// prefixes).  One wave, 64-way search: each round samples 64 split candidates, so a run of a
// million records is settled in four rounds of two loads each.
__device__ __forceinline__ u64 merge_split(const Rec* A, u64 la, const Rec* B, u64 lb, u64 d, int lane) {
    u64 lo = d > lb ? d - lb : 0, hi = d < la ? d : la;
    while (hi > lo) {
        const u64 s = hi - lo;
        const u64 p = s <= 64 ? lo + lane : lo + (u64)lane * s / 64;
        bool t = false;
        if (p < hi) {
            const Rec& x = A[p];
            const Rec& y = B[d - 1 - p];
            t = !pre_lt(y.hi, y.lo, x.hi, x.lo);
        }
        const int c = __popcll(__ballot(t));
        if (s <= 64) return lo + c;
        const u64 nlo = c > 0 ? __shfl(p, c - 1) + 1 : lo;
        const u64 nhi = c < 64 ? __shfl(p, c) : hi;
        lo = nlo; hi = nhi;
    }
    return lo;
}

// one merge pass: runs of length w -> 2w; workgroup b writes outputs [b * 1024, +1024)
__global__ __launch_bounds__(MG_NT) void k_merge(const Rec* in, Rec* out, u64 n, u64 w) {
    __shared__ u64 sh[MG_CHUNK], sl[MG_CHUNK];
    __shared__ u64 split[2];
    const u64 c0 = (u64)blockIdx.x * MG_CHUNK;
    const u64 a0 = c0 / (2 * w) * (2 * w);
    const u64 la = n - a0 < w ? n - a0 : w;
    const u64 rest = n - a0 - la;
    const u64 lb = rest < w ? rest : w;
    const Rec* A = in + a0;
    const Rec* B = A + la;
    const u64 d0 = c0 - a0, d1 = (d0 + MG_CHUNK < la + lb) ? d0 + MG_CHUNK : la + lb;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (wv < 2) {
        const u64 sp = merge_split(A, la, B, lb, wv ? d1 : d0, lane);
        if (lane == 0) split[wv] = sp;
    }
    __syncthreads();
    const u64 i0 = split[0], i1 = split[1];
    const u64 j0 = d0 - i0;
    const int na = (int)(i1 - i0), m = (int)(d1 - d0);
    Rec r[MG_CHUNK / MG_NT];
#pragma unroll
    for (int k = 0; k < MG_CHUNK / MG_NT; k++) {
        const int e = k * MG_NT + tid;
        if (e < m) {
            r[k] = e < na ? A[i0 + e] : B[j0 + (e - na)];
            sh[e] = r[k].hi; sl[e] = r[k].lo;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < MG_CHUNK / MG_NT; k++) {
        const int e = k * MG_NT + tid;
        if (e >= m) continue;
        const u64 xh = r[k].hi, xl = r[k].lo;
        int lo, hi, pos;
        if (e < na) {                              // B window records strictly below x
            lo = na; hi = m;
            while (lo < hi) { const int mid = (lo + hi) >> 1; if (pre_lt(sh[mid], sl[mid], xh, xl)) lo = mid + 1; else hi = mid; }
            pos = e + (lo - na);
        } else {                                   // A window records at or below x
            lo = 0; hi = na;
            while (lo < hi) { const int mid = (lo + hi) >> 1; if (!pre_lt(xh, xl, sh[mid], sl[mid])) lo = mid + 1; else hi = mid; }
            pos = (e - na) + lo;
        }
        out[a0 + d0 + pos] = r[k];
    }
}

// exclusive scan of u64 (in place) by one workgroup of 1024 threads; total in *total
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

__device__ __forceinline__ u64 line_len(const Rec& x, int fmt, u32 nreduce, u32 part, const uint8_t* arena) {
    if (fmt == FMT_MERGED) return rec_len(x) + 3 + ndigits(x.cnt);
    return (rec_ihash(x, arena) % nreduce == part) ? rec_len(x) + JSON_FIXED + ndigits(x.cnt) : 0;
}

// Formatting runs in tiles of 1024 lines (4 consecutive lines per thread): k_fmt_sum writes each
// tile's byte count, k_scan_u64 turns those into tile offsets, k_fmt_write recomputes its lines'
// lengths, scans them inside the tile and writes the bytes.
constexpr int FM_NT = 256, FM_IPT = 4, FM_TILE = FM_NT * FM_IPT;

__device__ __forceinline__ u64 block_excl_scan(u64 s, u64* ws, u64& all) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    u64 incl = s;
    for (int d = 1; d < 64; d <<= 1) { const u64 y = __shfl_up(incl, d, 64); if (lane >= d) incl += y; }
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    u64 pre = 0;
    all = 0;
    for (int k = 0; k < FM_NT / 64; k++) { if (k < w) pre += ws[k]; all += ws[k]; }
    return pre + incl - s;
}

__global__ __launch_bounds__(FM_NT) void k_fmt_sum(const Rec* r, u64 n, int fmt, u32 nreduce, u32 part,
                                                  const uint8_t* arena, u64* tsum) {
    __shared__ u64 ws[FM_NT / 64];
    const u64 i0 = (u64)blockIdx.x * FM_TILE + (u64)threadIdx.x * FM_IPT;
    u64 s = 0;
    for (int k = 0; k < FM_IPT; k++)
        if (i0 + k < n) s += line_len(r[i0 + k], fmt, nreduce, part, arena);
    u64 all;
    (void)block_excl_scan(s, ws, all);
    if (threadIdx.x == 0) tsum[blockIdx.x] = all;
}

__global__ __launch_bounds__(FM_NT) void k_fmt_write(const Rec* r, u64 n, int fmt, u32 nreduce, u32 part,
                                                    const uint8_t* arena, const u64* toff, uint8_t* out) {
    __shared__ u64 ws[FM_NT / 64];
    const u64 i0 = (u64)blockIdx.x * FM_TILE + (u64)threadIdx.x * FM_IPT;
    u64 L[FM_IPT], s = 0;
    for (int k = 0; k < FM_IPT; k++) {
        L[k] = i0 + k < n ? line_len(r[i0 + k], fmt, nreduce, part, arena) : 0;
        s += L[k];
    }
    u64 all;
    uint8_t* o = out + toff[blockIdx.x] + block_excl_scan(s, ws, all);
    for (int q = 0; q < FM_IPT; q++) {
        if (L[q] == 0) continue;
        const Rec x = r[i0 + q];
        const u64 len = rec_len(x);
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
        const u32 nd = ndigits(x.cnt);
        u64 c = x.cnt;
        for (int k = (int)nd - 1; k >= 0; k--) { o[k] = (uint8_t)('0' + c % 10); c /= 10; }
        o += nd;
        if (fmt == FMT_JSON) { *o++ = '"'; *o++ = '}'; }
        *o++ = '\n';
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

// Both export kernels take EX_TILE records per workgroup and count units per owner in LDS, so
// global atomics are one per (workgroup, owner): with one atomic per record, all records of an
// owner serialise on one address (~12 ns each: 1.2 ms for 1e5 records to one owner).
constexpr int EX_NT = 256, EX_IPT = 8, EX_TILE = EX_NT * EX_IPT;
constexpr u32 EX_MAX_RANKS = 1024;

__global__ __launch_bounds__(EX_NT) void k_export_count(const Rec* r, u64 n, u32 nreduce, u32 nranks,
                                                        const uint8_t* arena, u32* owner, u64* per_rank) {
    __shared__ u32 units[EX_MAX_RANKS];
    for (u32 o = threadIdx.x; o < nranks; o += EX_NT) units[o] = 0;
    __syncthreads();
    const u64 base = (u64)blockIdx.x * EX_TILE;
#pragma unroll
    for (int k = 0; k < EX_IPT; k++) {
        const u64 i = base + k * EX_NT + threadIdx.x;
        if (i < n) {
            const Rec x = r[i];
            const u32 o = (rec_ihash(x, arena) % nreduce) % nranks;
            owner[i] = o;
            atomicAdd(&units[o], (u32)rec_units(x));
        }
    }
    __syncthreads();
    for (u32 o = threadIdx.x; o < nranks; o += EX_NT)
        if (units[o]) atomicAdd(&per_rank[o], (u64)units[o]);
}

// cursor[o] starts at the exclusive prefix of per_rank; a workgroup reserves one range per owner
// and places its records inside it by LDS atomics.  Order inside a destination is irrelevant
// (the receiver re-aggregates and re-sorts).
__global__ __launch_bounds__(EX_NT) void k_export_write(const Rec* r, u64 n, u32 nranks, const u32* owner,
                                                        u64* cursor, const uint8_t* arena, Rec* out) {
    __shared__ u32 units[EX_MAX_RANKS];
    __shared__ u64 first[EX_MAX_RANKS];
    for (u32 o = threadIdx.x; o < nranks; o += EX_NT) units[o] = 0;
    __syncthreads();
    const u64 base = (u64)blockIdx.x * EX_TILE;
    u32 local[EX_IPT];
#pragma unroll
    for (int k = 0; k < EX_IPT; k++) {
        const u64 i = base + k * EX_NT + threadIdx.x;
        local[k] = i < n ? atomicAdd(&units[owner[i]], (u32)rec_units(r[i])) : 0u;
    }
    __syncthreads();
    for (u32 o = threadIdx.x; o < nranks; o += EX_NT)
        first[o] = units[o] ? atomicAdd(&cursor[o], (u64)units[o]) : 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < EX_IPT; k++) {
        const u64 i = base + k * EX_NT + threadIdx.x;
        if (i >= n) continue;
        const Rec x = r[i];
        const u64 u = rec_units(x);
        const u64 pos = first[owner[i]] + local[k];
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
                    const u64 off = long_home(s, len, lmask + 1, arena_cap, &st->arena_top);
                    if (off == ~0ull) { atomicAdd(&st->overflow, 1u); break; }
                    const u64 cells = long_cells(len);
                    for (u64 k = 0; k < cells; k++) arena[off + k] = k < len ? cont_byte(src, k) : 0;
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
