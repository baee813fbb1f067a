// wcg_reduce.h - DoReduce + Merge on gfx950 (mapreduce.go:239-321, wc.go:35-38).
//
//   k_compact   global tables -> dense records {128-bit big-endian prefix, count, ref}
//   (the sort: wcg_sort.h)
//   k_fmt_sum / k_scan_u64 / k_fmt_write  "key: count\n" (Merge, mapreduce.go:316-318),
//               {"Key":"k","Value":"count"}\n lines (DoReduce, :274-278), or line copies (the
//               merge of formatted runs)
//   k_part_hist / k_part_scatter  records grouped by ihash(key) % R, each group in key order:
//               every -res-<r> file in one formatting pass
//   k_json_count / k_json_write  DoMap's per-occurrence JSON lines (mapreduce.go:214-230)
//   k_nl_*      line index of formatted runs (the cross-GPU Merge input)
//   k_export_* / k_import  the ihash % nReduce shuffle between GPUs
#pragma once
#include "wcg_common.h"
#include "wcg_lds_table.h"
#include "wcg_sort.h"

namespace wcg {

// ---------------------------------------------------------------- compaction
constexpr int CP_NT = 256, CP_IPT = 8;          // 2048 table slots per block, one atomic each

// Each thread takes CP_IPT slots: every slot entry is loaded first, unconditionally (a load in a
// per-slot branch made a serial chain of memory latencies), then long keys' 16-byte prefixes.
// glist (two-pass jobs): the gtab part is the gslots listed slots gtab[glist[i]], not gtab[0, gslots);
// llist (large contexts): the ltab part is the lslots listed slots ltab[llist[i]]
// block `blk` of CP_NT * CP_IPT slots (a CP_NT-thread workgroup; k_compact and the fused reduce's
// compaction phase, wcg_fused.h).  Workgroup-uniform early return only.  blk_count (the fused
// reduce): the block's records go to out[blk * CP_NT * CP_IPT, ...) and their number to
// blk_count[blk] (no shared counter: 320 returning atomics on DevState::nrec serialised)
__device__ __forceinline__ void compact_block(const GEntry* gtab, u64 gslots, const GEntry* ltab, u64 lslots,
                                              const uint8_t* arena, Rec* out, u64 cap, DevState* st,
                                              const u64* glist, const u64* llist, u64 blk, u32* blk_count = nullptr) {
    __shared__ u32 wsum[CP_NT / 64], wlong[CP_NT / 64];
    __shared__ u64 base_s;
    // a failed job (full table or arena, malformed import) compacts nothing: its slots may hold
    // half-published long keys (no arena offset), and the reduce's sort and formatting may run
    // before the host reads the error (device-sized jobs)
    if (st->overflow | st->spin_fail | st->bad_input) {
        if (blk_count && threadIdx.x == 0) blk_count[blk] = 0;
        return;
    }
    const u64 total = gslots + lslots;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u64 b0 = blk * CP_NT * CP_IPT;
    GEntry e[CP_IPT];
#pragma unroll
    for (int j = 0; j < CP_IPT; j++) {
        const u64 i = b0 + (u64)j * CP_NT + tid;
        // (past the end: slot 0 of ltab, a valid address whose entry is then ignored)
        const u64 li = i < total ? i - gslots : 0;
        const GEntry* src = i < gslots ? gtab + (glist ? glist[i] : i) : ltab + (llist && i < total ? llist[li] : li);
        e[j] = *src;
        if (i >= total) e[j].k0 = 0;
    }
    uint4 q[CP_IPT];
    if (b0 + (u64)CP_NT * CP_IPT > gslots) {          // (workgroup-uniform: a block of the global table
#pragma unroll                                        // has no long key and skips this round trip)
        for (int j = 0; j < CP_IPT; j++) {
            const bool lng = b0 + (u64)j * CP_NT + tid >= gslots && e[j].k0 != 0;
            q[j] = *reinterpret_cast<const uint4*>(arena + (lng ? e[j].k1 - 1 : 0));   // arena cells: 16-byte aligned
        }
    } else {
#pragma unroll
        for (int j = 0; j < CP_IPT; j++) q[j] = make_uint4(0, 0, 0, 0);
    }
    Rec r[CP_IPT];
    u32 have = 0, nlong = 0;
#pragma unroll
    for (int j = 0; j < CP_IPT; j++) {
        const GEntry& x = e[j];
        if (x.k0 == 0) continue;
        have |= 1u << j;
        if (b0 + (u64)j * CP_NT + tid < gslots) {
            r[j] = inline_rec(x.k0, x.k1, x.cnt);
        } else {                                    // long key: {tag, arena offset + 1, cnt, len}
            r[j].hi = bswap64((u64)q[j].y << 32 | q[j].x);
            r[j].lo = bswap64((u64)q[j].w << 32 | q[j].z);
            r[j].cnt = x.cnt;
            r[j].ref = LONG_FLAG | (x.aux << 40) | (x.k1 - 1);
            nlong++;
        }
    }
    const u32 cnt = __popc(have);
    // block exclusive prefix of cnt (<= 8 per thread): 4 ballots per wave, then waves in order;
    // the long keys are summed the same way (one atomic per block: a per-thread atomic on one
    // DevState word serialised ~1M times on C4, most of the kernel's 0.5 ms)
    u32 o = 0, wt = 0, wl = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
        const u64 bal = __ballot((cnt >> b) & 1);
        o += __builtin_amdgcn_mbcnt_hi((u32)(bal >> 32), __builtin_amdgcn_mbcnt_lo((u32)bal, 0u)) << b;
        wt += (u32)__popcll(bal) << b;
        wl += (u32)__popcll(__ballot((nlong >> b) & 1)) << b;
    }
    if (lane == 0) { wsum[w] = wt; wlong[w] = wl; }
    __syncthreads();
    if (tid == 0) {
        u32 all = 0, al = 0;
        for (int k = 0; k < CP_NT / 64; k++) { const u32 v = wsum[k]; wsum[k] = all; all += v; al += wlong[k]; }
        if (blk_count) { base_s = b0; blk_count[blk] = all; }
        else base_s = all ? atomicAdd(&st->nrec, (u64)all) : 0;
        if (al) atomicAdd(&st->nlong, (u64)al);
    }
    __syncthreads();
    u64 pos = base_s + wsum[w] + o;
#pragma unroll
    for (int j = 0; j < CP_IPT; j++)
        if (have & (1u << j)) { if (pos < cap) out[pos] = r[j]; pos++; }   // more: host grows, reruns
}

__global__ __launch_bounds__(CP_NT) void k_compact(const GEntry* gtab, u64 gslots, const GEntry* ltab, u64 lslots,
                                                  const uint8_t* arena, Rec* out, u64 cap, DevState* st, u64* zero,
                                                  const u64* glist, const u64* llist = nullptr) {
    if (zero && blockIdx.x == 0 && threadIdx.x == 0) *zero = 0;   // a later kernel's counter
    compact_block(gtab, gslots, ltab, lslots, arena, out, cap, st, glist, llist, blockIdx.x);
}

// wcg_reset: zero n1 + n2 16-byte words of two tables and the DevState counters, one dispatch;
// with list1 the first table's part is the n1 / 2 listed 32-byte entries t1[2 list1[i] + {0, 1}]
// (list2: the same for the second table)
__global__ void k_clear(uint4* t1, u64 n1, uint4* t2, u64 n2, DevState* st, const u64* list1, const u64* list2) {
    const uint4 z = make_uint4(0, 0, 0, 0);
    const u64 stride = (u64)gridDim.x * blockDim.x;
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n1 + n2; i += stride) {
        const u64 j = i - n1;
        if (i < n1) t1[list1 ? 2 * list1[i >> 1] + (i & 1) : i] = z;
        else t2[list2 ? 2 * list2[j >> 1] + (j & 1) : j] = z;
    }
    if (blockIdx.x == 0) {
        u32* w = reinterpret_cast<u32*>(st);
        for (u32 k = threadIdx.x; k < sizeof(DevState) / 4; k += blockDim.x) w[k] = 0;
    }
}

// two-pass jobs compact into the record log itself: the tables' records follow its
// min(nemit, cap) records
__global__ void k_log_len(u64 cap, DevState* st) {
    const u64 n = st->nemit;
    st->nrec = n < cap ? n : cap;
}

// the record log of k_agg's pass 2 -> the front of the compaction output (nrec = its length;
// k_agg sent records past the log's capacity to the global table)
__global__ void k_copy_emit(const Rec* src, Rec* dst, u64 cap, DevState* st) {
    const u64 n = st->nemit, m = n < cap ? n : cap;
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < m; i += (u64)gridDim.x * blockDim.x) dst[i] = src[i];
    if (blockIdx.x == 0 && threadIdx.x == 0) st->nrec = m;
}

// ---------------------------------------------------------------- formatting
// decimal digits of a count: compares against powers of ten (a u64 division is a long software
// routine on the GPU)
__device__ __forceinline__ u32 ndigits(u64 v) {
    u32 d = 1;
    u64 p = 10;
#pragma unroll
    for (int k = 1; k < 20; k++) { d += v >= p ? 1u : 0u; p *= 10; }
    return d;
}
// the nd decimal digits of v at o[0..nd) (32-bit divisions by 10 are multiplies)
template <typename P>
__device__ __forceinline__ void put_digits(P o, u64 v, u32 nd) {
    if (v < (1ull << 32)) {
        u32 c = (u32)v;
        for (int k = (int)nd - 1; k >= 0; k--) { o[k] = (uint8_t)('0' + c % 10u); c /= 10u; }
    } else {
        for (int k = (int)nd - 1; k >= 0; k--) { o[k] = (uint8_t)('0' + v % 10); v /= 10; }
    }
}
__device__ __forceinline__ u64 rec_len(const Rec& r) { return (r.ref & LONG_FLAG) ? ((r.ref >> 40) & LONG_LEN_MAX) : r.ref; }
__device__ __forceinline__ u32 rec_byte(const Rec& r, u64 k, const uint8_t* arena) {
    if (r.ref & LONG_FLAG) return arena[(r.ref & LONG_OFF_MASK) + k];
    return k < 8 ? (u32)(r.hi >> (56 - 8 * k)) & 0xFF : (u32)(r.lo >> (56 - 8 * (k - 8))) & 0xFF;
}
__device__ u32 rec_ihash(const Rec& r, const uint8_t* arena) {
    u32 h = 0x811C9DC5u;
    const u64 len = rec_len(r);
    if (!(r.ref & LONG_FLAG)) {            // inline key: its bytes are the prefix words
        for (u64 k = 0; k < len; k++) h = fnv1a_step(h, k < 8 ? (u32)(r.hi >> (56 - 8 * k)) & 0xFF
                                                              : (u32)(r.lo >> (120 - 8 * k)) & 0xFF);
        return h;
    }
    const uint8_t* p = arena + (r.ref & LONG_OFF_MASK);
    for (u64 k = 0; k < len; k++) h = fnv1a_step(h, p[k]);
    return h;
}

// FMT_MERGED "key: count\n"; FMT_JSON {"Key":"k","Value":"count"}\n for ihash(k) % nreduce ==
// part; FMT_JSON_ALL the same for every record (records pre-grouped by partition); FMT_COPY
// copies line records of formatted text (cnt = line bytes, ref & LONG_OFF_MASK = offset in `arena`)
constexpr int FMT_MERGED = 0, FMT_JSON = 1, FMT_JSON_ALL = 2, FMT_COPY = 3;
constexpr u64 JSON_FIXED = 8 + 11 + 3;   // {"Key":" + ","Value":" + "}\n

// a record with count 0 is a merged duplicate (k_ss_bucket, wcg_sort.h: dd_same): no line
__device__ __forceinline__ u64 line_len(const Rec& x, int fmt, u32 nreduce, u32 part, const uint8_t* arena) {
    if (x.cnt == 0 && fmt != FMT_COPY) return 0;
    if (fmt == FMT_MERGED) return rec_len(x) + 3 + ndigits(x.cnt);
    if (fmt == FMT_COPY) return x.cnt;
    if (fmt == FMT_JSON_ALL) return rec_len(x) + JSON_FIXED + ndigits(x.cnt);
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

// a thread's FM_IPT records, loaded unconditionally (a load inside a per-record branch was a
// serial chain of memory latencies); records past n are not used
__device__ __forceinline__ void fmt_load(const Rec* r, u64 n, u64 i0, Rec* x) {
#pragma unroll
    for (int k = 0; k < FM_IPT; k++) x[k] = r[i0 + k < n ? i0 + k : (n ? n - 1 : 0)];
}
// device-sized formatting: n is the capacity the tiles were launched for, *nd the records
__device__ __forceinline__ u64 fmt_count(u64 n, const u64* nd) { return nd && *nd < n ? *nd : n; }

template <int FMT>
__global__ __launch_bounds__(FM_NT) void k_fmt_sum(const Rec* r, u64 n, const u64* nd, u32 nreduce, u32 part,
                                                  const uint8_t* arena, u64* tsum) {
    __shared__ u64 ws[FM_NT / 64];
    n = fmt_count(n, nd);
    const u64 i0 = (u64)blockIdx.x * FM_TILE + (u64)threadIdx.x * FM_IPT;
    Rec x[FM_IPT];
    fmt_load(r, n, i0, x);
    u64 s = 0;
#pragma unroll
    for (int k = 0; k < FM_IPT; k++) s += i0 + k < n ? line_len(x[k], FMT, nreduce, part, arena) : 0;
    u64 all;
    (void)block_excl_scan(s, ws, all);
    if (threadIdx.x == 0) tsum[blockIdx.x] = all;
}

// the lines of records x[0, FM_IPT) with lengths L[] at o (global memory or LDS)
template <int FMT, typename P>
__device__ __forceinline__ void fmt_lines(const Rec* x, const u64* L, const uint8_t* arena, P o) {
    for (int q = 0; q < FM_IPT; q++) {
        if (L[q] == 0) continue;
        if (FMT == FMT_COPY) {
            const uint8_t* src = arena + (x[q].ref & LONG_OFF_MASK);
            for (u64 k = 0; k < L[q]; k++) o[k] = src[k];
            o += L[q];
            continue;
        }
        const bool json = FMT != FMT_MERGED;
        const u64 len = rec_len(x[q]);
        if (json) {
            const char* pre = "{\"Key\":\"";
            for (int k = 0; k < 8; k++) *o++ = pre[k];
        }
        if (x[q].ref & LONG_FLAG) {
            const uint8_t* src = arena + (x[q].ref & LONG_OFF_MASK);
            for (u64 k = 0; k < len; k++) *o++ = src[k];
        } else {
            for (u64 k = 0; k < len; k++)
                *o++ = (uint8_t)(k < 8 ? x[q].hi >> (56 - 8 * k) : x[q].lo >> (56 - 8 * (k - 8)));
        }
        if (json) {
            const char* mid = "\",\"Value\":\"";
            for (int k = 0; k < 11; k++) *o++ = mid[k];
        } else {
            *o++ = ':'; *o++ = ' ';
        }
        const u32 nd = ndigits(x[q].cnt);
        put_digits(o, x[q].cnt, nd);
        o += nd;
        if (json) { *o++ = '"'; *o++ = '}'; }
        *o++ = '\n';
    }
}

// A tile's lines are formatted into LDS (byte stores there are cheap) and leave in aligned
// 16-byte stores; the destination's alignment is kept by offsetting the LDS image by
// (dst & 15).  A tile larger than the stage (long keys) writes its bytes directly.
constexpr u32 FM_STAGE = 32768;
template <int FMT>
__global__ __launch_bounds__(FM_NT) void k_fmt_write(const Rec* r, u64 n, const u64* nd, u32 nreduce, u32 part,
                                                    const uint8_t* arena, const u64* toff, uint8_t* out) {
    __shared__ u64 ws[FM_NT / 64];
    __shared__ __align__(16) uint8_t sb[FM_STAGE];
    n = fmt_count(n, nd);
    const u64 i0 = (u64)blockIdx.x * FM_TILE + (u64)threadIdx.x * FM_IPT;
    Rec x[FM_IPT];
    fmt_load(r, n, i0, x);
    u64 L[FM_IPT], s = 0;
#pragma unroll
    for (int k = 0; k < FM_IPT; k++) {
        L[k] = i0 + k < n ? line_len(x[k], FMT, nreduce, part, arena) : 0;
        s += L[k];
    }
    u64 all;
    const u64 lo = block_excl_scan(s, ws, all);
    uint8_t* const dst = out + toff[blockIdx.x];
    const u32 pad = (u32)((uintptr_t)dst & 15);
    if (pad + all > FM_STAGE) {                     // workgroup-uniform
        fmt_lines<FMT>(x, L, arena, dst + lo);
        return;
    }
    fmt_lines<FMT>(x, L, arena, sb + pad + lo);
    __syncthreads();
    uint8_t* const base = dst - pad;                // 16-byte aligned; sb[b] is base[b]
    const u32 total = pad + (u32)all;
    for (u32 c = threadIdx.x; 16 * c < total; c += FM_NT) {
        const u32 b0 = 16 * c, b1 = b0 + 16 < total ? b0 + 16 : total;
        if (b0 >= pad && b1 == b0 + 16) *reinterpret_cast<uint4*>(base + b0) = *reinterpret_cast<const uint4*>(sb + b0);
        else for (u32 b = b0 > pad ? b0 : pad; b < b1; b++) base[b] = sb[b];
    }
}

// ---------------------------------------------------------------- every -res-<r> at once
// The sorted records are regrouped by partition p = ihash(key) % R, stably (each group keeps
// key order), so one formatting pass writes all R DoReduce files back to back.  Tiles of
// PT_TILE records: k_part_hist counts records (and JSON bytes) per (p, tile); after a scan,
// k_part_scatter places each record at its group offset + its rank among the tile's earlier
// records of the same partition (wave ballots on the partition bits give the rank in order).
constexpr int PT_NT = 256, PT_TILE = 1024;
constexpr u32 PT_MAXR = 1024;

__global__ __launch_bounds__(PT_NT) void k_part_hist(const Rec* r, u64 n, u32 R, const uint8_t* arena, u32* pid,
                                                     u32* hist, u64* part_bytes) {
    __shared__ u32 c[PT_MAXR];
    __shared__ u64 bsum[PT_MAXR];
    for (u32 p = threadIdx.x; p < R; p += PT_NT) { c[p] = 0; bsum[p] = 0; }
    __syncthreads();
    const u64 T = (n + PT_TILE - 1) / PT_TILE;
    for (int k = 0; k < PT_TILE / PT_NT; k++) {
        const u64 i = (u64)blockIdx.x * PT_TILE + k * PT_NT + threadIdx.x;
        if (i >= n) continue;
        const Rec x = r[i];
        const u32 p = rec_ihash(x, arena) % R;
        pid[i] = p;
        atomicAdd(&c[p], 1u);
        if (x.cnt) atomicAdd((unsigned long long*)&bsum[p], (unsigned long long)(rec_len(x) + JSON_FIXED + ndigits(x.cnt)));
    }
    __syncthreads();
    for (u32 p = threadIdx.x; p < R; p += PT_NT) {
        hist[(u64)p * T + blockIdx.x] = c[p];
        if (bsum[p]) atomicAdd((unsigned long long*)&part_bytes[p], (unsigned long long)bsum[p]);
    }
}

__global__ __launch_bounds__(PT_NT) void k_part_scatter(const Rec* r, u64 n, u32 R, const u32* pid, const u32* off,
                                                        Rec* out) {
    __shared__ u32 base[PT_MAXR];
    __shared__ u32 wc[PT_NT / 64][PT_MAXR];
    const u64 T = (n + PT_TILE - 1) / PT_TILE;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (u32 p = tid; p < R; p += PT_NT) base[p] = off[(u64)p * T + blockIdx.x];
    for (u32 q = tid; q < (PT_NT / 64) * R; q += PT_NT) wc[q / R][q % R] = 0;
    u32 bits = 0;
    while ((1u << bits) < R) bits++;
    for (int k = 0; k < PT_TILE / PT_NT; k++) {
        const u64 i = (u64)blockIdx.x * PT_TILE + k * PT_NT + tid;
        const bool valid = i < n;
        const u32 p = valid ? pid[i] : 0u;
        u64 m = __ballot(valid);
        for (u32 b = 0; b < bits; b++) {
            const u64 bal = __ballot((p >> b) & 1);
            m &= ((p >> b) & 1) ? bal : ~bal;
        }
        const u64 below = lane ? (~0ull >> (64 - lane)) : 0ull;
        const u32 rank = (u32)__popcll(m & below);
        __syncthreads();                                     // base[] / wc[] of the last round used
        if (valid && rank == 0) wc[w][p] = (u32)__popcll(m);  // the lowest lane of each partition
        __syncthreads();
        if (valid) {
            u32 d = base[p] + rank;
            for (int v = 0; v < w; v++) d += wc[v][p];        // earlier waves of this round
            out[d] = r[i];
        }
        __syncthreads();
        // advance the bases past this round's records; clear the wave counts this round set
        if (valid && rank == 0) atomicAdd(&base[p], wc[w][p]);
        __syncthreads();
        if (valid && rank == 0) wc[w][p] = 0;
    }
}

// ---------------------------------------------------------------- DoMap's JSON (-m-r) lines
// Reference-exact map output (mapreduce.go:214-230): for every token, in input order, the line
// {"Key":"tok","Value":"1"}\n in file ihash(tok) % R.  Each thread walks its JS_SUB input bytes
// (tokens owned by their first byte, fact F3) with the byte-exact letter test; partitions are
// processed JS_PG at a time.  k_json_count sums line bytes per (partition, workgroup);
// k_json_write re-walks, turns per-thread sums into in-order offsets and writes the lines.
constexpr int JS_NT = 128;
constexpr u64 JS_SUB = 2048;
constexpr u32 JS_PG = 128;
constexpr u64 JS_LINE = 23;              // {"Key":" + ","Value":"1"}\n

template <typename F>
__device__ __forceinline__ void for_tokens(const uint8_t* in, u64 n, u64 c0, u64 c1, F f) {
    auto at = [&](long i) -> u32 { return (i >= 0 && (u64)i < n) ? in[i] : 0u; };
    u64 p = c0;
    if (p > 0 && p < n && letter_byte(at, (long)p - 1) && letter_byte(at, (long)p))
        while (p < n && letter_byte(at, (long)p)) p++;              // the previous owner's token
    while (p < c1 && p < n) {
        if (!letter_byte(at, (long)p)) { p++; continue; }
        u64 q = p + 1;
        while (q < n && letter_byte(at, (long)q)) q++;
        f(p, q - p);
        p = q;
    }
}

__device__ __forceinline__ u32 fnv32_bytes(const uint8_t* p, u64 len) {
    u32 h = 0x811C9DC5u;
    for (u64 k = 0; k < len; k++) h = fnv1a_step(h, p[k]);
    return h;
}

__global__ __launch_bounds__(JS_NT) void k_json_count(const uint8_t* in, u64 n, u32 R, u64* hist) {
    __shared__ unsigned long long s[JS_PG];
    const u64 W = gridDim.x;
    const u64 c0 = ((u64)blockIdx.x * JS_NT + threadIdx.x) * JS_SUB;
    for (u32 pg = 0; pg < R; pg += JS_PG) {
        for (u32 p = threadIdx.x; p < JS_PG; p += JS_NT) s[p] = 0;
        __syncthreads();
        for_tokens(in, n, c0, c0 + JS_SUB, [&](u64 p, u64 len) {
            const u32 r = fnv32_bytes(in + p, len) % R;
            if (r >= pg && r < pg + JS_PG) atomicAdd(&s[r - pg], (unsigned long long)(JS_LINE + len));
        });
        __syncthreads();
        for (u32 p = threadIdx.x; p < JS_PG && pg + p < R; p += JS_NT) hist[(u64)(pg + p) * W + blockIdx.x] = s[p];
        __syncthreads();
    }
}

__global__ __launch_bounds__(JS_NT) void k_json_write(const uint8_t* in, u64 n, u32 R, const u64* off, uint8_t* out) {
    __shared__ u32 t[JS_PG][JS_NT + 1];            // per-thread line bytes per partition -> offsets
    const u64 W = gridDim.x;
    const int tid = threadIdx.x;
    const u64 c0 = ((u64)blockIdx.x * JS_NT + tid) * JS_SUB;
    for (u32 pg = 0; pg < R; pg += JS_PG) {
        for (u32 p = 0; p < JS_PG; p++) t[p][tid] = 0;
        for_tokens(in, n, c0, c0 + JS_SUB, [&](u64 p, u64 len) {
            const u32 r = fnv32_bytes(in + p, len) % R;
            if (r >= pg && r < pg + JS_PG) t[r - pg][tid] += (u32)(JS_LINE + len);
        });
        __syncthreads();
        for (u32 p = tid; p < JS_PG; p += JS_NT) {   // exclusive scan over the threads, in order
            u32 run = 0;
            for (int q = 0; q < JS_NT; q++) { const u32 v = t[p][q]; t[p][q] = run; run += v; }
        }
        __syncthreads();
        for_tokens(in, n, c0, c0 + JS_SUB, [&](u64 p, u64 len) {
            const u32 r = fnv32_bytes(in + p, len) % R;
            if (r < pg || r >= pg + JS_PG) return;
            uint8_t* o = out + off[(u64)r * W + blockIdx.x] + t[r - pg][tid];
            t[r - pg][tid] += (u32)(JS_LINE + len);
            const char* pre = "{\"Key\":\"";
            for (int k = 0; k < 8; k++) *o++ = pre[k];
            for (u64 k = 0; k < len; k++) *o++ = in[p + k];
            const char* suf = "\",\"Value\":\"1\"}\n";
            for (int k = 0; k < 15; k++) *o++ = suf[k];
        });
        __syncthreads();
    }
}

// ---------------------------------------------------------------- line index (merge of runs)
// Formatted runs "key: count\n" -> one record per line: {hi, lo} = the key's first 16 bytes
// (big-endian, zero-padded: the sort prefix), cnt = line bytes, ref = line offset | key length
// << 40 (| LONG_FLAG for keys of 16+ bytes: the tie groups).  k_nl_count counts '\n' per 64 KiB
// block, k_scan_u64 makes offsets, k_nl_recs emits the records in order.
constexpr int NL_NT = 256;
constexpr u64 NL_BLK = 65536;

__global__ __launch_bounds__(NL_NT) void k_nl_count(const uint8_t* t, u64 n, u64* cnt) {
    __shared__ u64 ws[NL_NT / 64];
    const u64 b0 = (u64)blockIdx.x * NL_BLK;
    u64 c = 0;
    for (u64 i = b0 + threadIdx.x; i < b0 + NL_BLK && i < n; i += NL_NT) c += t[i] == '\n';
    const u64 all = block_sum_u64(c, ws);
    if (threadIdx.x == 0) cnt[blockIdx.x] = all;
}

__global__ __launch_bounds__(NL_NT) void k_nl_recs(const uint8_t* t, u64 n, const u64* off, u64* nlpos) {
    // positions of the '\n' bytes, in order (one pass per block, ordered by a wave scan)
    __shared__ u64 ws[NL_NT / 64];
    const u64 b0 = (u64)blockIdx.x * NL_BLK;
    u64 base = off[blockIdx.x];
    for (u64 i0 = b0; i0 < b0 + NL_BLK && i0 < n; i0 += NL_NT) {
        const u64 i = i0 + threadIdx.x;
        const u64 f = (i < n && i < b0 + NL_BLK && t[i] == '\n') ? 1 : 0;
        u64 all;
        const u64 pre = block_excl_scan(f, ws, all);
        if (f) nlpos[base + pre] = i;
        base += all;
        __syncthreads();
    }
}

__global__ void k_line_recs(const uint8_t* t, const u64* nlpos, u64 nl, Rec* out, DevState* st) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < nl; i += (u64)gridDim.x * blockDim.x) {
        const u64 s = i ? nlpos[i - 1] + 1 : 0, e = nlpos[i] + 1;
        u64 k = s;
        u64 hi = 0, lo = 0;
        while (k < e && t[k] != ':') {                   // keys are letters: the first ':' ends it
            const u64 j = k - s;
            if (j < 8) hi |= (u64)t[k] << (56 - 8 * j);
            else if (j < 16) lo |= (u64)t[k] << (120 - 8 * j);
            k++;
        }
        const u64 klen = k - s;
        if (k == e || klen == 0 || klen > LONG_LEN_MAX) atomicAdd(&st->bad_input, 1u);   // not "key: count"
        Rec r;
        r.hi = hi; r.lo = lo; r.cnt = e - s;
        r.ref = (klen >= 16 ? LONG_FLAG : 0ull) | ((klen < LONG_LEN_MAX ? klen : LONG_LEN_MAX) << 40) | s;
        out[i] = r;
    }
}

// run r of the concatenated text starts at byte rb[r]: its first line record is the number of
// '\n' before that byte
__global__ void k_run_bounds(const u64* nlpos, u64 nl, const u64* rb, u32 nruns, u64* b) {
    const u32 r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r > nruns) return;
    const u64 x = rb[r];
    u64 lo = 0, hi = nl;
    while (lo < hi) { const u64 mid = (lo + hi) >> 1; if (nlpos[mid] < x) lo = mid + 1; else hi = mid; }
    b[r] = lo;
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
        if (!(x.ref & LONG_FLAG) ? (x.ref == 0 || x.ref > 15) : (((x.ref >> 40) & LONG_LEN_MAX) < 16)) {
            atomicAdd(&st->bad_input, 1u);                // not a unit k_export_write produces
            continue;
        }
        if (!(x.ref & LONG_FLAG)) {
            u64 k0, k1;
            make_key(bswap64(x.hi), bswap64(x.lo), (int)x.ref, k0, k1);
            ginsert(gtab, gmask, k0, k1, gslot(key_hash(k0, k1)), x.cnt, st);
            continue;
        }
        u64 len = (x.ref >> 40) & LONG_LEN_MAX;
        const Rec* src = in + i + 1;
        if (i + 1 + (len + CONT_BYTES - 1) / CONT_BYTES > n) { atomicAdd(&st->overflow, 1u); continue; }
        u64 h = LHASH_INIT;
        for (u64 k = 0; k < len; k += 4) {
            u32 w = 0;
            for (u64 b = 0; b < 4 && k + b < len; b++) w |= (u32)cont_byte(src, k + b) << (8 * b);
            h = lhash_step(h, w);
        }
        u64 tag = mix64(h ^ len) | 1ull;
        u64 s = tag & lmask, probes = 0;
        int spins = 0;
        while (true) {
            GEntry* e = &ltab[s];
            u64 c0 = ld_agent(&e->k0);
            if (c0 == 0) {
                u64 exp;
                if (ltab_claim(st, e, s, tag, &exp)) {
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
