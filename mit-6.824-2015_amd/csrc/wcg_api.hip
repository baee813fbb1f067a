// wcg_api.hip - C ABI of libwcg.so (declared in include/wcg.h).
//
// One context = one GPU's share of a word-count job.  Device memory is allocated once at
// wcg_open and sized for 288 GB HBM parts: the aggregation tables, the record buffers for
// the sort and the formatted output all stay resident, so a job is a fixed sequence of
// launches on one stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/wcg.h"
#include "wcg_common.h"
#include "wcg_map.h"
#include "wcg_agg.h"
#include "wcg_reduce.h"

using namespace wcg;

struct wcg_ctx {
    int device = 0;
    int ncu = 256;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    u64 max_input = 0, max_keys = 0;
    uint8_t* d_in = nullptr;
    GEntry* gtab = nullptr; u64 gslots = 0;
    GEntry* ltab = nullptr; u64 lslots = 0;
    uint8_t* arena = nullptr; u64 arena_cap = 0;
    DevState* st = nullptr;
    DevState* h_st = nullptr;                 // pinned mirror
    Rec* recA = nullptr; Rec* recB = nullptr; u64 rec_cap = 0;
    Rec* sorted = nullptr;
    u64* lens = nullptr;
    u64* d_scalar = nullptr;                  // scan totals
    u64* h_scalar = nullptr;                  // pinned mirror of d_scalar[0]
    uint8_t* d_out = nullptr; u64 out_cap = 0; u64 out_len = 0;
    uint8_t* d_part = nullptr; u64 part_cap = 0;
    u64 nrec = 0;
    bool compacted = false, reduced = false;
    // export
    u32* owner = nullptr;
    u64* d_per_rank = nullptr;                // [2 * 1024]: counts, cursors
    Rec* exp_buf = nullptr; u64 exp_cap = 0;
    // miss log (k_map -> k_agg)
    u64* pool = nullptr; u64 pool_bytes = 0;
    u32* region_len = nullptr; u64 region_len_cap = 0;
    u64* wg_stats = nullptr; u64 wg_stats_cap = 0;   // k_map per-workgroup stats [grid][4]
    // long-token log (k_map -> k_long): one region of {offset | len << 40} records per workgroup
    u64* llog = nullptr; u64 llog_cap = 0;
    u32* llog_len = nullptr; u64 llog_len_cap = 0;
    u32 nbuckets = 64;
    // timing
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> map_ev, agg_ev;
    hipEvent_t phase_ev[6] = {};
    bool phase_rec = false;
    u64 map_launches = 0;
    std::string err;
};

namespace {

#define HIPCHK(ctx, call)                                                                   \
    do {                                                                                    \
        hipError_t e_ = (call);                                                             \
        if (e_ != hipSuccess) {                                                             \
            (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);                 \
            return WCG_EHIP;                                                                \
        }                                                                                   \
    } while (0)

u64 next_pow2(u64 x) {
    u64 p = 1;
    while (p < x) p <<= 1;
    return p;
}

int set_dev(wcg_ctx* c) {
    hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) { c->err = std::string("hipSetDevice: ") + hipGetErrorString(e); return WCG_EHIP; }
    return WCG_OK;
}

int grid_for(u64 n, int nt, int cap) {
    u64 g = (n + nt - 1) / nt;
    if (g < 1) g = 1;
    if (g > (u64)cap) g = cap;
    return (int)g;
}

hipEvent_t take_event(wcg_ctx* c) {
    if (c->ev_used == c->ev_pool.size()) {
        hipEvent_t e;
        (void)hipEventCreate(&e);
        c->ev_pool.push_back(e);
    }
    return c->ev_pool[c->ev_used++];
}

int check_status(wcg_ctx* c) {
    HIPCHK(c, hipMemcpyAsync(c->h_st, c->st, sizeof(DevState), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->h_st->overflow || c->h_st->spin_fail) {
        char buf[256];
        snprintf(buf, sizeof buf,
                 "aggregation table full (overflow=%u spin=%u): raise max_keys (%llu) / arena (%llu bytes)",
                 c->h_st->overflow, c->h_st->spin_fail, (unsigned long long)c->max_keys,
                 (unsigned long long)c->arena_cap);
        c->err = buf;
        return WCG_EFULL;
    }
    return WCG_OK;
}

int ensure(wcg_ctx* c, uint8_t** p, u64* cap, u64 need) {
    if (need <= *cap) return WCG_OK;
    u64 nc = std::max<u64>(need + need / 4, 1 << 20);
    if (*p) HIPCHK(c, hipFree(*p));
    *p = nullptr;
    *cap = 0;
    HIPCHK(c, hipMalloc(p, nc));
    *cap = nc;
    return WCG_OK;
}

int compact(wcg_ctx* c) {
    if (c->compacted) return WCG_OK;
    HIPCHK(c, hipMemsetAsync(&c->st->nrec, 0, 2 * sizeof(u64), c->stream));   // nrec, nlong
    if (c->timing) { c->phase_ev[0] = take_event(c); HIPCHK(c, hipEventRecord(c->phase_ev[0], c->stream)); }
    u64 total = c->gslots + c->lslots;
    k_compact<<<(unsigned)((total + CP_NT * CP_IPT - 1) / (CP_NT * CP_IPT)), CP_NT, 0, c->stream>>>(
        c->gtab, c->gslots, c->ltab, c->lslots, c->arena, c->recA, c->st);
    HIPCHK(c, hipGetLastError());
    if (c->timing) { c->phase_ev[1] = take_event(c); HIPCHK(c, hipEventRecord(c->phase_ev[1], c->stream)); }
    int rc = check_status(c);
    if (rc) return rc;
    c->nrec = c->h_st->nrec;
    c->compacted = true;
    return WCG_OK;
}

// merge sort of recA[0:nrec) by the 128-bit prefix (no host round trip); result in c->sorted
int sort_records(wcg_ctx* c) {
    const u64 n = c->nrec;
    c->sorted = c->recA;
    if (n <= 1) return WCG_OK;
    Rec* src = c->recA;
    Rec* dst = c->recB;
    k_tile_sort<<<(unsigned)((n + TS_TILE - 1) / TS_TILE), TS_NT, 0, c->stream>>>(src, dst, n);
    HIPCHK(c, hipGetLastError());
    std::swap(src, dst);
    for (u64 w = TS_TILE; w < n; w *= 2) {
        k_merge<<<(unsigned)((n + MG_CHUNK - 1) / MG_CHUNK), MG_NT, 0, c->stream>>>(src, dst, n, w);
        HIPCHK(c, hipGetLastError());
        std::swap(src, dst);
    }
    c->sorted = src;
    // long keys sharing a 16-byte prefix (needs two long keys at least)
    if (c->h_st->nlong >= 2)
        k_tie_fix<<<grid_for(n, 256, c->ncu * 4), 256, 0, c->stream>>>(c->sorted, n, c->arena);
    HIPCHK(c, hipGetLastError());
    return WCG_OK;
}

// format sorted records into a device buffer sized by an upper bound (so nothing waits for
// the host before the write); one synchronisation at the end returns the exact size
int format(wcg_ctx* c, int fmt, u32 nreduce, u32 part, uint8_t** dbuf, u64* cap, u64* nbytes) {
    const u64 n = c->nrec;
    if (n == 0) { *nbytes = 0; return WCG_OK; }
    const u64 bound = n * (LONG_CELL + JSON_FIXED + 20) + c->h_st->arena_top + 64;   // keys <= 32 B + heap keys
    int rc = ensure(c, dbuf, cap, bound);
    if (rc) return rc;
    const unsigned nt = (unsigned)((n + FM_TILE - 1) / FM_TILE);
    k_fmt_sum<<<nt, FM_NT, 0, c->stream>>>(c->sorted, n, fmt, nreduce, part, c->arena, c->lens);
    k_scan_u64<<<1, 1024, 0, c->stream>>>(c->lens, nt, c->d_scalar);
    k_fmt_write<<<nt, FM_NT, 0, c->stream>>>(c->sorted, n, fmt, nreduce, part, c->arena, c->lens, *dbuf);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(c->h_scalar, c->d_scalar, sizeof(u64), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *nbytes = *c->h_scalar;
    return WCG_OK;
}

}  // namespace

extern "C" {

const char* wcg_version(void) { return "wcg 0.1 gfx950 (unicode " WCG_UNICODE_VERSION ")"; }

const char* wcg_last_error(const wcg_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

uint32_t wcg_ihash(const uint8_t* key, uint64_t len) {
    uint32_t h = 0x811C9DC5u;
    for (uint64_t i = 0; i < len; i++) { h ^= key[i]; h *= 0x01000193u; }
    return h;
}

int wcg_open(int device, uint64_t max_input_bytes, uint64_t max_keys, wcg_ctx** out) {
    if (!out) return WCG_EINVAL;
    *out = nullptr;
    wcg_ctx* c = new wcg_ctx();
    c->device = device;
    c->max_input = max_input_bytes;
    c->max_keys = std::max<u64>(max_keys, 1024);
    int rc = set_dev(c);
    if (rc) { *out = c; return rc; }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        c->ncu = prop.multiProcessorCount;
    *out = c;
    HIPCHK(c, hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
    c->stream = c->own_stream;
    c->gslots = next_pow2(2 * c->max_keys);
    c->lslots = std::max<u64>(next_pow2(c->gslots / 4), 4096);
    c->arena_cap = std::max<u64>(64ull << 20, c->lslots * 32);   // heap part (after the slot cells)
    c->rec_cap = c->gslots / 2 + c->lslots / 2 + 16;
    if (c->max_input) HIPCHK(c, hipMalloc(&c->d_in, c->max_input + 64));
    HIPCHK(c, hipMalloc(&c->gtab, c->gslots * sizeof(GEntry)));
    HIPCHK(c, hipMalloc(&c->ltab, c->lslots * sizeof(GEntry)));
    HIPCHK(c, hipMalloc(&c->arena, c->lslots * LONG_CELL + c->arena_cap + 64));
    HIPCHK(c, hipMalloc(&c->st, sizeof(DevState)));
    HIPCHK(c, hipHostMalloc(&c->h_st, sizeof(DevState), hipHostMallocDefault));
    // records: compaction output is bounded by the number of occupied slots
    u64 recs = c->gslots + c->lslots;
    c->rec_cap = recs;
    HIPCHK(c, hipMalloc(&c->recA, recs * sizeof(Rec)));
    HIPCHK(c, hipMalloc(&c->recB, recs * sizeof(Rec)));
    HIPCHK(c, hipMalloc(&c->lens, recs * sizeof(u64)));
    HIPCHK(c, hipMalloc(&c->d_scalar, 64));
    HIPCHK(c, hipHostMalloc(&c->h_scalar, 64, hipHostMallocDefault));
    HIPCHK(c, hipMalloc(&c->owner, recs * sizeof(u32)));
    HIPCHK(c, hipMalloc(&c->d_per_rank, 2 * 1024 * sizeof(u64)));
    return wcg_reset(c);
}

int wcg_close(wcg_ctx* c) {
    if (!c) return WCG_EINVAL;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    void* bufs[] = {c->d_in, c->gtab, c->ltab, c->arena, c->st, c->recA, c->recB, c->lens,
                    c->d_scalar, c->d_out, c->d_part, c->owner, c->d_per_rank, c->exp_buf,
                    c->pool, c->region_len, c->wg_stats, c->llog, c->llog_len};
    for (void* b : bufs) if (b) (void)hipFree(b);
    if (c->h_st) (void)hipHostFree(c->h_st);
    if (c->h_scalar) (void)hipHostFree(c->h_scalar);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
    return WCG_OK;
}

int wcg_set_stream(wcg_ctx* c, void* stream) {
    if (!c) return WCG_EINVAL;
    c->stream = stream ? (hipStream_t)stream : c->own_stream;
    return WCG_OK;
}

int wcg_enable_timing(wcg_ctx* c, int on) {
    if (!c) return WCG_EINVAL;
    c->timing = on != 0;
    return WCG_OK;
}

int wcg_reset(wcg_ctx* c) {
    if (!c) return WCG_EINVAL;
    int rc = set_dev(c);
    if (rc) return rc;
    HIPCHK(c, hipMemsetAsync(c->gtab, 0, c->gslots * sizeof(GEntry), c->stream));
    HIPCHK(c, hipMemsetAsync(c->ltab, 0, c->lslots * sizeof(GEntry), c->stream));
    HIPCHK(c, hipMemsetAsync(c->st, 0, sizeof(DevState), c->stream));
    c->compacted = c->reduced = false;
    c->nrec = 0;
    c->out_len = 0;
    c->map_ev.clear();
    c->agg_ev.clear();
    c->ev_used = 0;
    c->phase_rec = false;
    c->map_launches = 0;
    return WCG_OK;
}

int wcg_map_device(wcg_ctx* c, const void* dev_bytes, uint64_t n) {
    if (!c) return WCG_EINVAL;
    if (n == 0) return WCG_OK;
    if (!dev_bytes || ((uintptr_t)dev_bytes & 15)) { c->err = "wcg_map_device: input must be 16-byte aligned"; return WCG_EINVAL; }
    int rc = set_dev(c);
    if (rc) return rc;
    MapArgs a;
    a.in = (const uint8_t*)dev_bytes;
    a.n = n;
    a.ntiles = (n + MAP_STEP - 1) / MAP_STEP;      // 992-byte wave steps (1 KiB windows)
    // one workgroup per CU (LDS-bound); steps are dealt chip-wide inside the kernel
    u64 grid = std::min<u64>((u64)c->ncu, (a.ntiles + MAP_WAVES - 1) / MAP_WAVES);
    a.tiles_per_wg = (a.ntiles + grid - 1) / grid;          // steps per workgroup (sizing only)
    a.gtab = c->gtab; a.gmask = c->gslots - 1;
    a.ltab = c->ltab; a.lmask = c->lslots - 1;
    a.arena = c->arena; a.arena_cap = c->arena_cap;
    a.st = c->st;
    // miss log: one region per (workgroup, bucket) of 8-byte units; the whole pool is ~2n
    // bytes: a unit for every 4 input bytes covers every token missing the LDS table even on
    // high-cardinality UTF-8 text (C4: 0.1 tokens per byte, 79% misses, 2-unit keys), where a
    // 1-per-8 pool overflowed into per-token global-table inserts; only written units cost time
    const u32 P = c->nbuckets;
    u64 per_wg_bytes = (u64)a.tiles_per_wg * MAP_STEP;
    // even (16-byte aligned regions); a workgroup's regions stay under 2 GiB so k_map's unit
    // offsets fit 32 bits and its 24-bit multiplies (P * region_cap * 8 <= 2^31)
    a.region_cap = std::min<u64>(std::max<u64>(2048, per_wg_bytes / (4ull * P)), (1ull << 31) / (8ull * P)) & ~1ull;
    a.pmask = P - 1;
    u64 need = (grid * P * a.region_cap + AGG_SLACK_UNITS) * sizeof(u64);
    if (need > c->pool_bytes) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->pool) HIPCHK(c, hipFree(c->pool));
        c->pool = nullptr; c->pool_bytes = 0;
        HIPCHK(c, hipMalloc(&c->pool, need));
        c->pool_bytes = need;
    }
    if (grid * P > c->region_len_cap) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->region_len) HIPCHK(c, hipFree(c->region_len));
        c->region_len = nullptr; c->region_len_cap = 0;
        HIPCHK(c, hipMalloc(&c->region_len, grid * P * sizeof(u32)));
        c->region_len_cap = grid * P;
    }
    if (grid > c->wg_stats_cap) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->wg_stats) HIPCHK(c, hipFree(c->wg_stats));
        c->wg_stats = nullptr; c->wg_stats_cap = 0;
        HIPCHK(c, hipMalloc(&c->wg_stats, grid * 4 * sizeof(u64)));
        c->wg_stats_cap = grid;
    }
    // long-token log: a token > 15 bytes takes >= 17 input bytes, so a 992-byte step logs at
    // most 59 of them; 60 records per step bound a workgroup's region
    a.llog_cap = (u32)std::min<u64>((u64)a.tiles_per_wg * 60 + 64, 0xFFFFFFFFull);
    const u64 lneed = grid * (u64)a.llog_cap * sizeof(u64);
    if (lneed > c->llog_cap) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->llog) HIPCHK(c, hipFree(c->llog));
        c->llog = nullptr; c->llog_cap = 0;
        HIPCHK(c, hipMalloc(&c->llog, lneed));
        c->llog_cap = lneed;
    }
    if (grid > c->llog_len_cap) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->llog_len) HIPCHK(c, hipFree(c->llog_len));
        c->llog_len = nullptr; c->llog_len_cap = 0;
        HIPCHK(c, hipMalloc(&c->llog_len, grid * sizeof(u32)));
        c->llog_len_cap = grid;
    }
    a.llog = c->llog;
    a.llog_len = c->llog_len;
    a.pool = c->pool;
    a.region_len = c->region_len;
    a.wg_stats = c->wg_stats;
    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
    if (c->timing) { e0 = take_event(c); HIPCHK(c, hipEventRecord(e0, c->stream)); }
    static const int ablate = getenv("WCG_MAP_ABLATE") ? atoi(getenv("WCG_MAP_ABLATE")) : 0;
    switch (ablate) {
        case 1: k_map<1><<<(unsigned)grid, MAP_NT, 0, c->stream>>>(a); break;
        case 2: k_map<2><<<(unsigned)grid, MAP_NT, 0, c->stream>>>(a); break;
        case 3: k_map<3><<<(unsigned)grid, MAP_NT, 0, c->stream>>>(a); break;
        case 4: k_map<4><<<(unsigned)grid, MAP_NT, 0, c->stream>>>(a); break;
        case 5: k_map<5><<<(unsigned)grid, MAP_NT, 0, c->stream>>>(a); break;
        case 6: k_map<6><<<(unsigned)grid, MAP_NT, 0, c->stream>>>(a); break;
        case 7: k_map<7><<<(unsigned)grid, MAP_NT, 0, c->stream>>>(a); break;
        default: k_map<0><<<(unsigned)grid, MAP_NT, 0, c->stream>>>(a); break;
    }
    HIPCHK(c, hipGetLastError());
    if (c->timing) { e1 = take_event(c); HIPCHK(c, hipEventRecord(e1, c->stream)); }
    // the logged long tokens: LONG_PARTS workgroups per map workgroup's region
    if (ablate == 0 || ablate >= 6) {
        static const int lab = getenv("WCG_LONG_ABLATE") ? atoi(getenv("WCG_LONG_ABLATE")) : 0;
        k_long<<<(unsigned)(grid * LONG_PARTS), LONG_NT, 0, c->stream>>>(a, (u32)grid, lab);
        HIPCHK(c, hipGetLastError());
    }
    AggArgs g;
    g.pool = c->pool; g.region_len = c->region_len; g.region_cap = a.region_cap;
    g.P = P; g.nsrc = (u32)grid;
    g.slices = std::max<u32>(1, std::min<u32>((u32)grid, (u32)(c->ncu + P - 1) / P));
    g.slices = std::max<u32>(g.slices, (u32)((grid + AGG_MAX_SRC - 1) / AGG_MAX_SRC));
    g.gtab = c->gtab; g.gmask = c->gslots - 1; g.st = c->st;
    g.map_stats = c->wg_stats;
    k_agg<<<P * g.slices, AGG_NT, 0, c->stream>>>(g);
    HIPCHK(c, hipGetLastError());
    if (c->timing) {
        e2 = take_event(c);
        HIPCHK(c, hipEventRecord(e2, c->stream));
        c->map_ev.push_back({e0, e1});
        c->agg_ev.push_back({e1, e2});
    }
    c->map_launches++;
    c->compacted = c->reduced = false;
    return WCG_OK;
}

int wcg_map(wcg_ctx* c, const uint8_t* host_bytes, uint64_t n) {
    if (!c) return WCG_EINVAL;
    if (n == 0) return WCG_OK;
    if (!c->d_in || n > c->max_input) { c->err = "wcg_map: split larger than max_input_bytes"; return WCG_EINVAL; }
    int rc = set_dev(c);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(c->d_in, host_bytes, n, hipMemcpyHostToDevice, c->stream));
    rc = wcg_map_device(c, c->d_in, n);
    if (rc) return rc;
    // the staging buffer is reused by the next call: finish this one first
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return WCG_OK;
}

int wcg_reduce(wcg_ctx* c, uint64_t* nkeys, uint64_t* nbytes) {
    if (!c) return WCG_EINVAL;
    int rc = set_dev(c);
    if (rc) return rc;
    if ((rc = compact(c))) return rc;
    if (c->timing) { c->phase_ev[2] = take_event(c); HIPCHK(c, hipEventRecord(c->phase_ev[2], c->stream)); }
    if ((rc = sort_records(c))) return rc;
    if (c->timing) { c->phase_ev[3] = take_event(c); HIPCHK(c, hipEventRecord(c->phase_ev[3], c->stream)); }
    if ((rc = format(c, FMT_MERGED, 1, 0, &c->d_out, &c->out_cap, &c->out_len))) return rc;
    if (c->timing) {
        c->phase_ev[4] = take_event(c);
        HIPCHK(c, hipEventRecord(c->phase_ev[4], c->stream));
        c->phase_rec = true;
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->reduced = true;
    if (nkeys) *nkeys = c->nrec;
    if (nbytes) *nbytes = c->out_len;
    return WCG_OK;
}

int wcg_result_device(wcg_ctx* c, const void** dev_ptr, uint64_t* nbytes) {
    if (!c) return WCG_EINVAL;
    if (!c->reduced) { c->err = "wcg_result_device before wcg_reduce"; return WCG_ESTATE; }
    if (dev_ptr) *dev_ptr = c->d_out;
    if (nbytes) *nbytes = c->out_len;
    return WCG_OK;
}

int wcg_result_copy(wcg_ctx* c, uint8_t* host_out, uint64_t cap) {
    if (!c) return WCG_EINVAL;
    if (!c->reduced) { c->err = "wcg_result_copy before wcg_reduce"; return WCG_ESTATE; }
    if (cap < c->out_len) { c->err = "wcg_result_copy: buffer too small"; return WCG_EINVAL; }
    int rc = set_dev(c);
    if (rc) return rc;
    if (c->out_len) {
        HIPCHK(c, hipMemcpyAsync(host_out, c->d_out, c->out_len, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return WCG_OK;
}

int wcg_partition(wcg_ctx* c, uint32_t nreduce, uint32_t r, uint8_t* host_out, uint64_t cap, uint64_t* nbytes) {
    if (!c) return WCG_EINVAL;
    if (!c->reduced) { c->err = "wcg_partition before wcg_reduce"; return WCG_ESTATE; }
    if (nreduce == 0 || r >= nreduce) { c->err = "wcg_partition: bad partition"; return WCG_EINVAL; }
    int rc = set_dev(c);
    if (rc) return rc;
    u64 len = 0;
    if ((rc = format(c, FMT_JSON, nreduce, r, &c->d_part, &c->part_cap, &len))) return rc;
    if (nbytes) *nbytes = len;
    if (host_out) {
        if (cap < len) { c->err = "wcg_partition: buffer too small"; return WCG_EINVAL; }
        if (len) HIPCHK(c, hipMemcpyAsync(host_out, c->d_part, len, hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return WCG_OK;
}

int wcg_export(wcg_ctx* c, uint32_t nreduce, uint32_t nranks, const void** dev_records, uint64_t* counts) {
    if (!c || !counts || nreduce == 0 || nranks == 0 || nranks > EX_MAX_RANKS) return WCG_EINVAL;
    int rc = set_dev(c);
    if (rc) return rc;
    if ((rc = compact(c))) return rc;
    u64 n = c->nrec;
    HIPCHK(c, hipMemsetAsync(c->d_per_rank, 0, 2 * 1024 * sizeof(u64), c->stream));
    if (n) {
        k_export_count<<<(unsigned)((n + EX_TILE - 1) / EX_TILE), EX_NT, 0, c->stream>>>(c->recA, n, nreduce, nranks,
                                                                                        c->arena, c->owner, c->d_per_rank);
        HIPCHK(c, hipGetLastError());
    }
    std::vector<u64> per(nranks), cur(nranks);
    HIPCHK(c, hipMemcpyAsync(per.data(), c->d_per_rank, nranks * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    u64 tot = 0;
    for (u32 i = 0; i < nranks; i++) { cur[i] = tot; tot += per[i]; counts[i] = per[i]; }
    rc = ensure(c, reinterpret_cast<uint8_t**>(&c->exp_buf), &c->exp_cap, (tot + 1) * sizeof(Rec));
    if (rc) return rc;
    if (n) {
        HIPCHK(c, hipMemcpyAsync(c->d_per_rank + 1024, cur.data(), nranks * sizeof(u64), hipMemcpyHostToDevice, c->stream));
        k_export_write<<<(unsigned)((n + EX_TILE - 1) / EX_TILE), EX_NT, 0, c->stream>>>(
            c->recA, n, nranks, c->owner, c->d_per_rank + 1024, c->arena, c->exp_buf);
        HIPCHK(c, hipGetLastError());
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (dev_records) *dev_records = c->exp_buf;
    return WCG_OK;
}

int wcg_import(wcg_ctx* c, const void* dev_records, uint64_t nrecords) {
    if (!c) return WCG_EINVAL;
    if (nrecords == 0) return WCG_OK;
    if (!dev_records) return WCG_EINVAL;
    int rc = set_dev(c);
    if (rc) return rc;
    k_import<<<grid_for(nrecords, 256, c->ncu * 8), 256, 0, c->stream>>>((const Rec*)dev_records, nrecords, c->gtab,
                                                                          c->gslots - 1, c->ltab, c->lslots - 1,
                                                                          c->arena, c->arena_cap, c->st);
    HIPCHK(c, hipGetLastError());
    c->compacted = c->reduced = false;
    return check_status(c);
}

int wcg_timings(wcg_ctx* c, double* ms, int n, uint64_t* map_launches) {
    if (!c || !ms || n < 0) return WCG_EINVAL;
    int rc = set_dev(c);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    double v[5] = {0, 0, 0, 0, 0};
    float f = 0;
    for (auto& p : c->map_ev) { HIPCHK(c, hipEventElapsedTime(&f, p.first, p.second)); v[0] += f; }
    for (auto& p : c->agg_ev) { HIPCHK(c, hipEventElapsedTime(&f, p.first, p.second)); v[1] += f; }
    if (c->phase_rec) {
        HIPCHK(c, hipEventElapsedTime(&f, c->phase_ev[0], c->phase_ev[1])); v[2] = f;
        HIPCHK(c, hipEventElapsedTime(&f, c->phase_ev[2], c->phase_ev[3])); v[3] = f;
        HIPCHK(c, hipEventElapsedTime(&f, c->phase_ev[3], c->phase_ev[4])); v[4] = f;
    }
    for (int i = 0; i < n && i < 5; i++) ms[i] = v[i];
    if (map_launches) *map_launches = c->map_launches;
    return WCG_OK;
}

int wcg_stats(wcg_ctx* c, uint64_t* s8) {
    if (!c || !s8) return WCG_EINVAL;
    int rc = set_dev(c);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(c->h_st, c->st, sizeof(DevState), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    s8[0] = c->h_st->tokens; s8[1] = c->nrec; s8[2] = c->h_st->lds_hits; s8[3] = c->h_st->global_ops;
    s8[4] = c->h_st->long_tokens; s8[5] = c->h_st->arena_top; s8[6] = c->h_st->overflow; s8[7] = c->h_st->spin_fail;
    return WCG_OK;
}

}  // extern "C"
