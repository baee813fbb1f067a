// wcg_api.hip - C ABI of libwcg.so (declared in include/wcg.h).
//
// One context = one GPU's share of a word-count job.  Device memory is allocated at wcg_open
// (tables, records) or on first need (sort items, staging), sized for 288 GB HBM parts: the
// aggregation tables, the record buffers for the sort and the formatted output all stay
// resident, so a job is a fixed sequence of launches on one stream.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/wcg.h"
#include "wcg_common.h"
#include "wcg_map.h"
#include "wcg_agg.h"
#include "wcg_reduce.h"
#include "wcg_fused.h"
#include "wcg_ingest.h"

using namespace wcg;

struct wcg_ctx {
    int device = 0;
    int ncu = 256;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    hipStream_t long_stream = nullptr;                // k_long_* beside k_agg (independent work)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    u64 max_input = 0, max_keys = 0;
    GEntry* gtab = nullptr; u64 gslots = 0;
    GEntry* ltab = nullptr; u64 lslots = 0;
    uint8_t* arena = nullptr; u64 arena_cap = 0;
    u64 lheap_cap = 0;                        // two-pass contexts: the log heap after arena_cap
    DevState* st = nullptr;
    DevState* h_st = nullptr;                 // pinned mirror
    Rec* recA = nullptr; Rec* recB = nullptr; u64 rec_cap = 0;
    Rec* crec = nullptr;                      // the compacted records: recA, or the record log
    Rec* sorted = nullptr;                    // recB, or a merge pass's last output
    u64* lens = nullptr; u64 lens_cap = 0;    // per-tile sums of the formatter
    u64* d_scalar = nullptr;                  // scan totals (in st's block, ST_SCALAR_OFF on)
    u64* h_scalar = nullptr;                  // pinned scratch (64 u64, in h_st's block)
    uint8_t* d_out = nullptr; u64 out_cap = 0; u64 out_len = 0;
    u64 nrec = 0;
    u64 nkeys = 0;                            // distinct keys among the nrec sorted records
    bool compacted = false, reduced = false;
    // sort (wcg_sort.h)
    Rec* smp = nullptr; u64 smp_cap = 0;      // 2 x sample records (merge ping-pong)
    u32* bid = nullptr; u64 bid_cap = 0;
    u64* spx = nullptr; u64 spx_cap = 0;    // sort splitters as arrays (large B)
    bool nkeys_on_device = false;            // the sort's distinct-key count is still in d_scalar[8]
    // Device-sized reduce (one-pass jobs after the first): compaction, sort and formatting run on
    // the record count in device memory; c->nrec is the buffers' capacity until wcg_reduce's one
    // read-back, and the sort is planned for the previous job's count (nrec_hint)
    bool dev_sized = false;
    u64 nrec_hint = 0;
    u64 long_hint = ~0ull;                    // long tokens of the previous job (unknown: ~0)
    // DevState's nrec / nlong are zero on the device: wcg_reset cleared them, or a one-pass
    // k_agg did, and no compaction has counted into them since (a second wcg_reduce
    // without a map in between would otherwise append to the first one's count)
    bool counts_clean = false;
    Rec* irec = nullptr; u64 irec_cap = 0;
    LEnt* lent = nullptr; u64 lent_cap = 0;   // long-key partitions: LQ x lpart_cap entries
    u64* spill = nullptr; u64 spill_cap = 0;  // k_agg pass-1 spill regions
    u32* spill_len = nullptr; u64 spill_len_cap = 0;
    u64* pool2 = nullptr; u64 pool2_cap = 0;  // k_rp sub-bucket regions
    u32* rlen2 = nullptr; u64 rlen2_cap = 0;
    Rec* remit = nullptr; u64 remit_cap = 0;  // record log of k_agg's pass 2
    Rec* ovf = nullptr; u64 ovf_cap = 0;      // pass 2's per-workgroup overflow staging
    bool two_pass_used = false;               // a map call since wcg_reset ran the two passes
    bool gtab_zero = false;                   // the global table was cleared by the last wcg_reset
    u64* glist = nullptr;                     // two-pass contexts: claimed global-table slots
    u64* llist = nullptr;                     // large contexts: claimed long-key-table slots
    bool ltab_zero = false;                   // the long-key table was cleared and nothing claimed since
    bool imported = false;                    // wcg_import since wcg_reset
    u32* lpcur = nullptr; u64 lpcur_cap = 0;    // 2n records: by bucket, and the oversized-bucket scratch
    u32* hist = nullptr; u64 hist_cap = 0;    // [B][G] bucket counts / partition counts
    u64* spart = nullptr; u64 spart_cap = 0;  // multi-block scan partials
    uint4* ikey = nullptr; u32* iidx = nullptr; u64 item_cap = 0;   // 2n items
    u64* groups = nullptr; u64 groups_cap = 0;
    // every -res-<r> (wcg_partition_all): valid for part_R while reduced
    u32 part_R = 0;
    std::vector<u64> part_bytes;
    u32* pid = nullptr; u64 pid_cap = 0;
    u64* d_partb = nullptr; u64 partb_cap = 0;
    uint8_t* d_part = nullptr; u64 part_cap = 0;
    // export
    u32* owner = nullptr; u64 owner_cap = 0;
    u64* d_per_rank = nullptr;                // [2 * 1024]: counts, cursors
    u64* h_cur = nullptr;                     // pinned cursors (1024)
    bool exp_ready = false; u32 exp_nranks = 0; u64 exp_total = 0;
    Rec* exp_buf = nullptr; u64 exp_cap = 0;
    // merge of formatted runs
    u64* nlpos = nullptr; u64 nlpos_cap = 0;
    u64* d_rb = nullptr; u64 rb_cap = 0;
    u64* d_b0 = nullptr; u64 b0_cap = 0;
    bool merged = false;                      // the result is a merge of runs (wcg_merge_runs): the
                                              // sorted records are line records, not keys
    // RCCL shuffle (wcg_comm_init / wcg_exchange / wcg_gather_merge)
    ncclComm_t comm = nullptr;
    int comm_rank = 0, comm_world = 0;
    u32 x_world = 0;                          // the exchange buffers are sized for this world
    u64* d_xrow = nullptr;                    // this rank's row, the status word, the gathered matrix
    u64* h_x = nullptr;                       // pinned: row header, status, send offsets, matrix
    Rec* xrecv = nullptr; u64 xrecv_cap = 0;  // received units
    uint8_t* grecv = nullptr; u64 grecv_cap = 0;   // root: the gathered runs
    u64* h_rb = nullptr; u64 h_rb_cap = 0;    // pinned run bounds
    // per-occurrence JSON map output (wcg_map_json)
    uint8_t* d_jin = nullptr; u64 jin_cap = 0;
    uint8_t* d_jout = nullptr; u64 jout_cap = 0;
    u64* jhist = nullptr; u64 jhist_cap = 0;
    std::vector<u64> jparts;
    // miss log (k_map -> k_agg)
    u64* pool = nullptr; u64 pool_bytes = 0;
    u32* region_len = nullptr; u64 region_len_cap = 0;
    u64* wg_stats = nullptr; u64 wg_stats_cap = 0;   // k_map per-workgroup stats [grid][4]
    // long-token log (k_map -> k_long): one region of {offset | len << 40} records per workgroup
    u64* llog = nullptr; u64 llog_cap = 0;
    u32* llog_len = nullptr; u64 llog_len_cap = 0;
    // ingest (wcg_ingest.h): two pinned staging buffers, two device buffers, a reader pool
    u64 chunk = 64ull << 20;
    uint8_t* hb[INGEST_SLOTS] = {};
    uint8_t* db[INGEST_SLOTS] = {};
    uint8_t* dbig = nullptr; u64 dbig_cap = 0;
    hipEvent_t ev_copied[INGEST_SLOTS] = {}, ev_mapped[INGEST_SLOTS] = {};
    // the last ingest's own breakdown (wcg_ingest_stats): timing events around each chunk's copy
    // (copy stream) and map kernels (work stream), four per chunk, kept for the context's life
    std::vector<hipEvent_t> ing_ev;
    double ing[3] = {};                       // host: issue wall, reading, waiting for a slot (ms)
    u64 ing_chunks = 0;
    hipStream_t copy_stream = nullptr;
    std::unique_ptr<TaskPool> readers;
    u64 ingest_bytes = 0;                     // bytes mapped by the last wcg_map / wcg_map_file
    // timing
    bool timing = false;
    bool timing_all = false;                 // every phase (modes 1, 2); mode 3: the map kernel only
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> map_ev, agg_ev;
    hipEvent_t phase_ev[6] = {};
    u64 map_launches_since_reset = 0;
    int timing_mode = 0;                     // 1: the last job; 2: every job since enable (no reads in between)
    std::vector<std::array<hipEvent_t, 5>> phase_jobs;   // mode 2: each job's phase events
    bool phase_rec = false;
    // shuffle phases (wcg_timings ms[5..9]): {phase, start, end}
    std::vector<std::tuple<int, hipEvent_t, hipEvent_t>> xev;
    double acc[10] = {};                      // mode 2: phases folded in from recycled events
    u64 map_launches = 0;
    // r05: the one-launch reduce of small one-pass jobs (wcg_fused.h): bucket regions, the spill
    // list, sample runs, bucket counts / starts / byte flags and the control block, one allocation
    uint8_t* fr_buf = nullptr;
    FrArgs fr{};                              // the buffers' pointers (set once)
    u32 fr_epoch = 0;
    bool fused_last = false;                  // the last wcg_reduce took that path (diagnostics)
    bool pending = false;                     // wcg_reduce_async queued a job not yet read back
    uint16_t* flist = nullptr; u64 flist_cap = 0;   // r05: k_agg's one-pass flush lists
    u64* h_st_dev = nullptr;                  // h_st's device address (the fused launch writes it)
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

#define RC(call)                                                                            \
    do {                                                                                    \
        int rc_ = (call);                                                                   \
        if (rc_) return rc_;                                                                \
    } while (0)

u64 next_pow2(u64 x) {
    u64 p = 1;
    while (p < x) p <<= 1;
    return p;
}

u64 cdiv(u64 a, u64 b) { return (a + b - 1) / b; }

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
    if (c->h_st->bad_input) {
        c->err = "malformed record units were imported (wcg_import of a buffer wcg_export did not write)";
        return WCG_EINVAL;
    }
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

// device buffer of at least `need` elements of T (contents are not kept); waits for the stream
// before freeing a buffer that in-flight work may still use
template <typename T>
int ensure(wcg_ctx* c, T** p, u64* cap, u64 need) {
    if (need <= *cap && *p) return WCG_OK;
    u64 nc = std::max<u64>(need + need / 4, (1u << 20) / sizeof(T));
    if (*p) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipFree(*p));
    }
    *p = nullptr;
    *cap = 0;
    HIPCHK(c, hipMalloc((void**)p, nc * sizeof(T)));
    *cap = nc;
    return WCG_OK;
}

// record buffers (compaction output, sort / merge ping-pong) for n records; the contents of
// recA are kept (records may already be in it)
int ensure_recs(wcg_ctx* c, u64 n) {
    if (n <= c->rec_cap) return WCG_OK;
    const u64 nc = n + n / 4;
    Rec *a = nullptr, *b = nullptr;
    HIPCHK(c, hipMalloc(&a, nc * sizeof(Rec)));
    HIPCHK(c, hipMalloc(&b, nc * sizeof(Rec)));
    HIPCHK(c, hipMemcpyAsync(a, c->recA, c->rec_cap * sizeof(Rec), hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipFree(c->recA));
    HIPCHK(c, hipFree(c->recB));
    c->recA = a; c->recB = b; c->rec_cap = nc;
    return WCG_OK;
}

// tables -> compacted records (c->crec).  Two-pass jobs append the tables' records to the
// record log itself (no copy of the log); otherwise, or when the log's buffer cannot hold them,
// the log is copied to the front of recA and the tables follow.  The record buffers start at
// max_keys records and grow (then the compaction runs again) when the tables hold more keys.
int compact(wcg_ctx* c, bool defer = false) {
    if (c->compacted) return WCG_OK;
    c->dev_sized = false;
    // wcg_reduce of a one-pass job: no read-back of the count here (a host round trip between
    // compaction and the sort); the records are bounded by the tables' slots, and the buffers are
    // sized for that
    static const bool exact_env = getenv("WCG_EXACT_REDUCE") != nullptr || getenv("WCG_SORT_TARGET") != nullptr;
    if (defer && !c->two_pass_used && !c->imported && c->nrec_hint >= 2 && !exact_env) {
        const u64 total = c->gslots + c->lslots;
        RC(ensure_recs(c, total));
        // nrec and nlong are zero after wcg_reset and after every one-pass map call's k_agg (a tiny
        // memset dispatch costs ~4 us); otherwise (a reduce again with no map in between) clear them
        if (!c->counts_clean) HIPCHK(c, hipMemsetAsync(&c->st->nrec, 0, 2 * sizeof(u64), c->stream));
        c->counts_clean = false;
        if (c->timing_all) { c->phase_ev[0] = take_event(c); HIPCHK(c, hipEventRecord(c->phase_ev[0], c->stream)); }
        k_compact<<<(unsigned)cdiv(total, CP_NT * CP_IPT), CP_NT, 0, c->stream>>>(
            c->gtab, c->gslots, c->ltab, c->lslots, c->arena, c->recA, c->rec_cap, c->st,
            c->d_scalar + ST_TIE_GROUPS, nullptr);
        HIPCHK(c, hipGetLastError());
        if (c->timing_all) { c->phase_ev[1] = take_event(c); HIPCHK(c, hipEventRecord(c->phase_ev[1], c->stream)); }
        c->nrec = total;                           // a capacity until wcg_reduce reads the count
        c->crec = c->recA;
        c->compacted = true;
        c->dev_sized = true;
        return WCG_OK;
    }
    // Two-pass jobs emit their inline keys as records; when nothing else reached the global
    // table (no fallback insert, no import), its slots are all empty and the scan is skipped.
    bool scan_gtab = true;
    const u64* glist = nullptr;                    // the listed claims instead of the whole table
    u64 gs = c->gslots;
    const u64* llist = nullptr;
    u64 ls = c->lslots;
    if ((c->two_pass_used && !c->imported) || c->llist) {
        HIPCHK(c, hipMemcpyAsync(c->h_st, c->st, sizeof(DevState), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->two_pass_used && !c->imported) {
            scan_gtab = c->h_st->global_ops != 0;
            if (scan_gtab && c->glist && c->h_st->gnew <= GLIST_CAP) { glist = c->glist; gs = c->h_st->gnew; }
        }
        // listed long-key claims (the table was cleared by a listed or full clear since: every
        // claim since is listed while lnew <= LLIST_CAP)
        if (c->llist && c->ltab_zero && c->h_st->lnew <= LLIST_CAP) { llist = c->llist; ls = c->h_st->lnew; }
    }
    if (!scan_gtab) gs = 0;
    c->counts_clean = false;
    const u64 total = gs + ls;
    const u64 emit_cap = c->max_keys + 65536;     // the log's length: min(nemit, emit_cap)
    if (c->two_pass_used && c->remit) {
        HIPCHK(c, hipMemsetAsync(&c->st->nlong, 0, sizeof(u64), c->stream));
        if (c->timing_all) { c->phase_ev[0] = take_event(c); HIPCHK(c, hipEventRecord(c->phase_ev[0], c->stream)); }
        k_log_len<<<1, 1, 0, c->stream>>>(emit_cap, c->st);
        k_compact<<<(unsigned)cdiv(std::max<u64>(total, 1), CP_NT * CP_IPT), CP_NT, 0, c->stream>>>(
            c->gtab, gs, c->ltab, ls, c->arena, c->remit, c->remit_cap, c->st, nullptr, glist, llist);
        HIPCHK(c, hipGetLastError());
        if (c->timing_all) { c->phase_ev[1] = take_event(c); HIPCHK(c, hipEventRecord(c->phase_ev[1], c->stream)); }
        RC(check_status(c));
        c->nrec = c->h_st->nrec;
        if (c->nrec <= c->remit_cap) {
            RC(ensure_recs(c, c->nrec));           // the sort's output
            c->crec = c->remit;
            c->compacted = true;
            return WCG_OK;
        }
    }
    for (int pass = 0; pass < 2; pass++) {
        HIPCHK(c, hipMemsetAsync(&c->st->nrec, 0, 2 * sizeof(u64), c->stream));   // nrec, nlong
        if (c->timing_all) { c->phase_ev[0] = take_event(c); HIPCHK(c, hipEventRecord(c->phase_ev[0], c->stream)); }
        if (c->remit && c->two_pass_used)   // the record log of pass 2 first (nrec = nemit; only
                                            // two-pass map calls write it)
            k_copy_emit<<<(unsigned)(c->ncu * 4), 256, 0, c->stream>>>(
                c->remit, c->recA, std::min<u64>(c->rec_cap, emit_cap), c->st);
        k_compact<<<(unsigned)cdiv(std::max<u64>(total, 1), CP_NT * CP_IPT), CP_NT, 0, c->stream>>>(
            c->gtab, gs, c->ltab, ls, c->arena, c->recA, c->rec_cap, c->st, nullptr, glist, llist);
        HIPCHK(c, hipGetLastError());
        if (c->timing_all) { c->phase_ev[1] = take_event(c); HIPCHK(c, hipEventRecord(c->phase_ev[1], c->stream)); }
        RC(check_status(c));
        c->nrec = c->h_st->nrec;
        if (c->nrec <= c->rec_cap) break;
        RC(ensure_recs(c, c->nrec));
    }
    c->crec = c->recA;
    c->compacted = true;
    return WCG_OK;
}

// One-launch reduce (wcg_fused.h) of a one-pass job: when the previous job of the context had at
// most FR_NMAX keys (the plan of the device-sized path, which this replaces for small jobs) and no
// record log is involved.  Imported keys (the owners' reduce after wcg_exchange) are table entries
// like any others (k_import inserts them exactly; a malformed unit sets bad_input, which the
// launch reports).  WCG_FUSED=0 keeps the multi-launch path (A/B, tests).
u64 merged_bound(wcg_ctx* c, u64 n, bool json);

bool fused_eligible(wcg_ctx* c) {
    static const char* env = getenv("WCG_FUSED");
    static const bool exact_env = getenv("WCG_EXACT_REDUCE") != nullptr || getenv("WCG_SORT_TARGET") != nullptr;
    if (env && atoi(env) == 0) return false;
    return !c->compacted && !c->two_pass_used && !exact_env && c->nrec_hint >= 2 &&
           c->nrec_hint <= FR_NMAX;
}

int reduce_fused(wcg_ctx* c) {
    const u64 total = c->gslots + c->lslots;
    RC(ensure_recs(c, total));
    c->dev_sized = true;                          // merged_bound: the whole long-key heap
    RC(ensure(c, &c->d_out, &c->out_cap, merged_bound(c, total, false) + 64));
    if (!c->fr_buf) {
        // one allocation: regions | spill records | spill buckets | samples and splitters | sample
        // occupancy | counts | bytes | starts | offsets | control block (zeroed once; each launch's
        // last workgroup re-zeroes its counters); every array on 128-byte lines of its own
        // (fr_layout, checked at compile time in wcg_fused.h)
        const FrLayout L = fr_layout(total);
        HIPCHK(c, hipMalloc(&c->fr_buf, L.all));
        HIPCHK(c, hipMemsetAsync(c->fr_buf, 0, L.all, c->stream));
        uint8_t* q = c->fr_buf;
        c->fr.reg = reinterpret_cast<Rec*>(q + L.reg);
        c->fr.spill = reinterpret_cast<Rec*>(q + L.spill);
        c->fr.spill_bid = reinterpret_cast<u32*>(q + L.spill_bid);
        c->fr.smp = reinterpret_cast<u64*>(q + L.smp);
        c->fr.socc = reinterpret_cast<u32*>(q + L.socc);
        c->fr.bcnt = reinterpret_cast<u32*>(q + L.bcnt);
        c->fr.bbytes = reinterpret_cast<u64*>(q + L.bbytes);
        c->fr.bstart = reinterpret_cast<u64*>(q + L.bstart);
        c->fr.boff = reinterpret_cast<u64*>(q + L.boff);
        c->fr.ctl = reinterpret_cast<FrCtl*>(q + L.ctl);
        c->fr.spill_cap = total;
    }
    // compaction counts into nrec / nlong: zero after wcg_reset and after a one-pass k_agg
    if (!c->counts_clean) HIPCHK(c, hipMemsetAsync(&c->st->nrec, 0, 2 * sizeof(u64), c->stream));
    c->counts_clean = false;
    FrArgs a = c->fr;
    a.gtab = c->gtab; a.gslots = c->gslots; a.ltab = c->ltab; a.lslots = c->lslots;
    a.arena = c->arena; a.st = c->st; a.total_out = c->d_scalar;
    a.rec = c->recA; a.rec_cap = c->rec_cap; a.out_rec = c->recB; a.out = c->d_out;
    c->fr_epoch = (c->fr_epoch + 1) & 0xFFFFFF;
    if (c->fr_epoch == 0) c->fr_epoch = 1;
    a.epoch = c->fr_epoch;
    const char* tenv = getenv("WCG_FUSED_TARGET");             // tests: records per bucket
    a.target = tenv ? (u32)std::max(1, atoi(tenv)) : FR_TARGET;
    a.nitems0 = (u32)cdiv(total, (u64)CP_NT * CP_IPT);
    if (c->timing_all) { c->phase_ev[2] = take_event(c); HIPCHK(c, hipEventRecord(c->phase_ev[2], c->stream)); }
    static const bool fclock = getenv("WCG_FUSED_CLOCK") != nullptr;   // diagnostics: phase clocks
    static u64* d_fclk = nullptr;
    const unsigned fgrid = (unsigned)(2 * c->ncu);
    a.clk = nullptr;
    if (fclock) {
        if (!d_fclk) HIPCHK(c, hipMalloc(&d_fclk, ((u64)fgrid * FR_CLK + 8ull * FR_NPH * FR_CLK_ITEMS + 8ull * FR_NPH) * sizeof(u64)));
        HIPCHK(c, hipMemsetAsync(d_fclk, 0, ((u64)fgrid * FR_CLK + 8ull * FR_NPH * FR_CLK_ITEMS + 8ull * FR_NPH) * sizeof(u64), c->stream));
        a.clk = d_fclk;
    }
    if (!c->h_st_dev) HIPCHK(c, hipHostGetDevicePointer((void**)&c->h_st_dev, c->h_st, 0));
    a.host_st = c->h_st_dev;
    k_fused_reduce<<<fgrid, FR_NT, 0, c->stream>>>(a);
    HIPCHK(c, hipGetLastError());
    if (fclock) {
        std::vector<u64> h((u64)fgrid * FR_CLK + 8ull * FR_NPH * FR_CLK_ITEMS + 8ull * FR_NPH);
        HIPCHK(c, hipMemcpyAsync(h.data(), d_fclk, h.size() * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        u64 t0 = ~0ull, tend = 0;
        for (unsigned w = 0; w < fgrid; w++) { t0 = std::min(t0, h[w * FR_CLK]); }
        fprintf(stderr, "wcg fused clock (us from the first workgroup's start):");
        for (int p = 0; p < FR_NPH; p++) {
            u64 ent = ~0ull, first = ~0ull, lastfirst = 0, left = 0;
            unsigned nw = 0;
            for (unsigned w = 0; w < fgrid; w++) {
                const u64* r = &h[w * FR_CLK];
                if (r[1 + 3 * p]) ent = std::min(ent, r[1 + 3 * p]);
                if (r[2 + 3 * p]) { first = std::min(first, r[2 + 3 * p]); lastfirst = std::max(lastfirst, r[2 + 3 * p]); nw++; }
                left = std::max(left, r[3 + 3 * p]);
            }
            tend = std::max(tend, left);
            fprintf(stderr, " | P%d entered %.1f first item %.1f last first item %.1f (%u wgs) all left %.1f", p,
                    ent == ~0ull ? -1.0 : (ent - t0) / 100.0, first == ~0ull ? -1.0 : (first - t0) / 100.0,
                    lastfirst ? (lastfirst - t0) / 100.0 : -1.0, nw, (left - t0) / 100.0);
        }
        u64 smax = 0;
        for (unsigned w = 0; w < fgrid; w++) smax = std::max(smax, h[w * FR_CLK]);
        fprintf(stderr, " | last wg start %.1f, end %.1f\n", (smax - t0) / 100.0, (tend - t0) / 100.0);
        for (int p = 1; p < FR_NPH; p++) {      // per workgroup: entry spread and what preceded the latest
            std::vector<double> ent, fi;
            double worst = -1, wprev = 0, went = 0;
            for (unsigned w = 0; w < fgrid; w++) {
                const u64* r = &h[w * FR_CLK];
                if (r[1 + 3 * p]) ent.push_back((r[1 + 3 * p] - t0) / 100.0);
                if (r[2 + 3 * p]) {
                    const double f = (r[2 + 3 * p] - t0) / 100.0;
                    fi.push_back(f);
                    if (f > worst) { worst = f; wprev = (r[3 * p] - t0) / 100.0; went = (r[1 + 3 * p] - t0) / 100.0; }
                }
            }
            if (ent.empty() || fi.empty()) continue;
            std::sort(ent.begin(), ent.end());
            std::sort(fi.begin(), fi.end());
            auto qt = [](const std::vector<double>& v, double f) { return v[(size_t)(f * (v.size() - 1))]; };
            fprintf(stderr, "  P%d entered q10/50/90/max %.1f %.1f %.1f %.1f; first item %.1f %.1f %.1f %.1f; latest: left P%d %.1f entered %.1f\n",
                    p, qt(ent, .1), qt(ent, .5), qt(ent, .9), ent.back(), qt(fi, .1), qt(fi, .5), qt(fi, .9), fi.back(), p - 1, wprev, went);
        }
        fprintf(stderr, "  publish (at / acquire, parameters, release us):");
        for (int q = 1; q < FR_NPH; q++) {
            const u64* k = &h[(u64)fgrid * FR_CLK + 8ull * FR_NPH * FR_CLK_ITEMS + 8 * q];
            if (k[0] && k[3]) fprintf(stderr, " | P%d %.1f / %.1f %.1f %.1f", q, (k[0] - t0) / 100.0, (k[1] - k[0]) / 100.0,
                                      (k[2] - k[1]) / 100.0, (k[3] - k[2]) / 100.0);
        }
        fprintf(stderr, "\n");
        for (int p = 0; p < FR_NPH; p++) {      // per item: sub-steps, work, release, count (median / max, us)
            std::vector<std::vector<double>> d(7);
            std::vector<std::pair<double, u64>> slow;      // P3: (item time, bucket size)
            for (u32 i = 0; i < FR_CLK_ITEMS; i++) {
                u64 q[8];
                std::copy(&h[(u64)fgrid * FR_CLK + ((u64)p * FR_CLK_ITEMS + i) * 8],
                          &h[(u64)fgrid * FR_CLK + ((u64)p * FR_CLK_ITEMS + i) * 8] + 8, q);
                if (!q[0] || !q[7]) continue;
                if (q[3] >> 62 == 1) {
                    slow.push_back({(q[7] - q[0]) / 100.0, q[3] & ~(1ull << 62)});
                    q[3] = 0;
                }
                u64 prev = q[0];
                for (int k = 1; k < 8; k++) {
                    if (!q[k]) { d[k - 1].push_back(0); continue; }
                    d[k - 1].push_back((q[k] - prev) / 100.0);
                    prev = q[k];
                }
            }
            if (d[0].empty()) continue;
            fprintf(stderr, "  P%d %zu items (med/p90/max us): ", p, d[0].size());
            const char* nm[7] = {"s1", "s2", "s3", "s4", "work", "release", "count"};
            for (int k = 0; k < 7; k++) {
                std::vector<double> v = d[k];
                std::sort(v.begin(), v.end());
                fprintf(stderr, "%s %.1f/%.1f/%.1f  ", nm[k], v[v.size() / 2], v[v.size() * 9 / 10], v.back());
            }
            fprintf(stderr, "\n");
            if (!slow.empty()) {
                std::sort(slow.begin(), slow.end());
                fprintf(stderr, "  P%d slowest items (us, records):", p);
                for (size_t k = slow.size() > 6 ? slow.size() - 6 : 0; k < slow.size(); k++)
                    fprintf(stderr, " %.1f/%llu", slow[k].first, (unsigned long long)slow[k].second);
                fprintf(stderr, "; median item %.1f/%llu\n", slow[slow.size() / 2].first, (unsigned long long)slow[slow.size() / 2].second);
            }
        }
    }
    if (c->timing_all) { c->phase_ev[3] = take_event(c); HIPCHK(c, hipEventRecord(c->phase_ev[3], c->stream)); }
    // the job's one host round trip: counters, errors and the formatted size, written into the
    // pinned host block by the launch's last workgroup (waited for by reduce_fused_finish: at once
    // in wcg_reduce, later after wcg_reduce_async)
    c->dev_sized = false;
    c->compacted = false;                         // recA is the fused launch's scratch
    c->fused_last = true;
    return WCG_OK;
}

// the job's results on the host: waits for the read-back of reduce_fused
int reduce_fused_finish(wcg_ctx* c) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->sorted = c->recB;
    c->crec = c->recA;
    c->nrec = c->nkeys = c->h_st->nrec;
    c->out_len = *c->h_scalar;
    if (c->h_st->bad_input || c->h_st->overflow || c->h_st->spin_fail) {
        c->nrec = 0; c->out_len = 0; c->reduced = false;
        RC(check_status(c));                      // the error message (nothing was compacted)
    }
    c->nrec_hint = c->nrec;
    c->long_hint = c->h_st->long_tokens;
    return WCG_OK;
}

// a wcg_reduce_async job's results, before anything that reads them
int resolve(wcg_ctx* c) {
    if (!c->pending) return WCG_OK;
    c->pending = false;
    return reduce_fused_finish(c);
}

// WCG_DEBUG=1: synchronise and report after each stage of the rarely used paths (diagnostics)
int dbg(wcg_ctx* c, const char* what) {
    static const bool on = getenv("WCG_DEBUG") != nullptr;
    if (!on) return WCG_OK;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    fprintf(stderr, "wcg: %s done\n", what);
    return WCG_OK;
}

// exclusive scan of m u32 in place (multi-block)
int scan_u32(wcg_ctx* c, u32* v, u64 m) {
    const u64 nb = cdiv(m, SC_SEG);
    if (m <= SC_ONE_MAX) {                         // one workgroup, one launch
        k_scan_apply1<<<1, SC_NT, 0, c->stream>>>(v, m);
        HIPCHK(c, hipGetLastError());
        return WCG_OK;
    }
    RC(ensure(c, &c->spart, &c->spart_cap, nb + 1));
    k_scan_part<<<(unsigned)nb, SC_NT, 0, c->stream>>>(v, m, c->spart);
    k_scan_u64<<<1, 1024, 0, c->stream>>>(c->spart, nb, nullptr);
    k_scan_apply<<<(unsigned)nb, SC_NT, 0, c->stream>>>(v, m, c->spart);
    HIPCHK(c, hipGetLastError());
    return WCG_OK;
}

// stable merge sort of n records (tile sort + passes); returns the buffer holding the result
int merge_sort(wcg_ctx* c, Rec* a, Rec* b, u64 n, Rec** result) {
    k_tile_sort<<<(unsigned)cdiv(n, TS_TILE), TS_NT, 0, c->stream>>>(a, b, n);
    HIPCHK(c, hipGetLastError());
    Rec *src = b, *dst = a;
    for (u64 w = TS_TILE; w < n; w *= 2) {
        k_merge<<<(unsigned)cdiv(n, MG_CHUNK), MG_NT, 0, c->stream>>>(src, dst, n, w);
        HIPCHK(c, hipGetLastError());
        std::swap(src, dst);
    }
    *result = src;
    return WCG_OK;
}

// items (2n): ikey and iidx are allocated together
int ensure_items(wcg_ctx* c, u64 n2) {
    if (n2 <= c->item_cap && c->ikey && c->iidx) return WCG_OK;
    if (c->ikey || c->iidx) HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->ikey) HIPCHK(c, hipFree(c->ikey));
    if (c->iidx) HIPCHK(c, hipFree(c->iidx));
    c->ikey = nullptr; c->iidx = nullptr; c->item_cap = 0;
    const u64 nc = std::max<u64>(n2 + n2 / 4, 1 << 16);
    HIPCHK(c, hipMalloc(&c->ikey, nc * sizeof(uint4)));
    HIPCHK(c, hipMalloc(&c->iidx, nc * sizeof(u32)));
    c->item_cap = nc;
    return WCG_OK;
}

// long keys sharing a 16-byte prefix in r[0:n): ordered by their full bytes (key bytes at
// `base`); `tmp` is a free record buffer of n records
// tie-group lists: starts (<= n / 2), then groups past 64 records (<= n / 64)
static u64 tie_list_cap(u64 n) { return (n / 2 + 2) + (n / 64 + 2); }

// marked = true: the group starts are already listed (the sample sort's bucket kernels and
// k_tie_edge, sort_records)
int fix_ties(wcg_ctx* c, Rec* r, u64 n, const uint8_t* base, Rec* tmp, const u64* nd = nullptr, u64* nkeys = nullptr,
             bool marked = false) {
    if (n < 2) return WCG_OK;
    RC(ensure(c, &c->groups, &c->groups_cap, tie_list_cap(n)));   // starts, mid and big groups
    RC(ensure_items(c, 2 * n));
    u64* const ng = c->d_scalar + ST_TIE_GROUPS;   // device-sized jobs: k_compact zeroed it
    if (!marked) {
        if (!nd) HIPCHK(c, hipMemsetAsync(ng, 0, sizeof(u64), c->stream));
        k_tie_mark<<<grid_for(n, 256, c->ncu * 4), 256, 0, c->stream>>>(r, n, nd, c->groups, ng);
    }
    TieArgs t;
    t.r = r; t.n = n; t.nd = nd; t.base = base; t.groups = c->groups; t.ngroups = ng;
    t.tmp = tmp; t.sc_key = c->ikey; t.sc_pos = c->iidx; t.nkeys = nkeys;
    // groups of <= TT_MAX records one thread each, <= 64 one wave each (one kernel), the larger
    // ones by workgroups (listed after the starts)
    u64* const big = c->groups + (n / 2 + 2);
    u64* const nbig = c->d_scalar + ST_TIE_BIG;
    if (!marked) HIPCHK(c, hipMemsetAsync(nbig, 0, sizeof(u64), c->stream));   // else k_tie_edge zeroed it
    k_tie_tiny<<<(unsigned)c->ncu * 8, 256, 0, c->stream>>>(t, big, nbig);
    t.groups = big; t.ngroups = nbig;
    k_tie_sort<<<(unsigned)c->ncu, TG_NT, 0, c->stream>>>(t);
    HIPCHK(c, hipGetLastError());
    return WCG_OK;
}

#ifndef WCG_TIE_FUSED
#define WCG_TIE_FUSED 1
#endif
// sample sort of recA[0:nrec) into recB (wcg_sort.h), then the tie groups
int sort_records(wcg_ctx* c) {
    // device-sized: n is the capacity (buffers), np the count the launches are planned for
    const bool dev = c->dev_sized;
    // (the plan: the previous job's count, but no fewer than 1/16 of the slots, so that a tiny
    // job followed by a large one does not put the large one into a few oversized buckets)
    const u64 n = c->nrec, np = dev ? std::min<u64>(std::max<u64>(c->nrec_hint, n / 16), n) : n;
    c->nkeys = n;
    c->sorted = c->recB;
    if (n == 0) return WCG_OK;
    if (n == 1 && !dev) {
        HIPCHK(c, hipMemcpyAsync(c->recB, c->crec, sizeof(Rec), hipMemcpyDeviceToDevice, c->stream));
        return WCG_OK;
    }
    if (n >= (1ull << 32)) { c->err = "sort: more than 2^32 distinct keys"; return WCG_EINVAL; }
    // WCG_SORT_TARGET (tests only): records per bucket; above SB_CAP it forces the global path
    const char* tenv = getenv("WCG_SORT_TARGET");
    const u64 target_env = tenv ? strtoull(tenv, nullptr, 10) : 0;
    u64 target = target_env ? target_env : SS_TARGET;
    // small sorts: buckets small enough for two workgroups per CU (C2: 1e5 keys -> 512 buckets
    // of ~200, one-entry networks) rather than fewer buckets than CUs
    if (!target_env) target = std::min<u64>(target, std::max<u64>(128, cdiv(np, 2ull * c->ncu)));
    target = std::max<u64>(target, cdiv(np, SS_MAXB));
    SortArgs a;
    a.rec = c->crec; a.n = n; a.out = c->recB;
    a.nd = dev ? &c->st->nrec : nullptr;
    // the record log: a key may repeat (the global table, other map calls, pass 2's overflow):
    // the bucket sort merges the copies and counts the distinct keys (device-sized jobs are
    // one-pass: no record log)
    a.dedupe = !dev && c->h_st->nemit != 0;
    a.nkeys = c->d_scalar + 8;                     // its own slot (the scans use d_scalar[0])
    if (a.dedupe) HIPCHK(c, hipMemsetAsync(a.nkeys, 0, sizeof(u64), c->stream));
    a.B = (u32)std::max<u64>(1, std::min<u64>(cdiv(np, target), SS_MAXB));
    a.cls2 = np / a.B > 4 * SB_NT;                 // a 512-thread class is worth a launch
    // large sorts sample twice as densely: bucket sizes vary as 1/sqrt(samples per bucket), and a
    // bucket past 4 * SB_NT records takes the 8-entry register network (twice the work per record)
    // bucket past 4 * SB_NT records takes the 8-entry register network (twice the work per record);
    // small sorts keep the sample within one workgroup's sort (TS_TILE) when 4+ per bucket allow
#ifndef WCG_SS_OVS_L
#define WCG_SS_OVS_L 2
#endif
    u64 ovs = a.B > SS_LDSB ? WCG_SS_OVS_L * SS_OVS : SS_OVS;
    if (a.B <= SS_LDSB && a.B * ovs > TS_TILE && a.B * 4 <= TS_TILE) ovs = TS_TILE / a.B;
    a.S = a.B > 1 ? std::min<u64>(np, (u64)a.B * ovs) : 0;
    a.smp = nullptr;
    if (a.B > 1) {
        RC(ensure(c, &c->smp, &c->smp_cap, 2 * a.S));
        if (a.S <= TS_TILE) {                      // ranked in S / 64 workgroups
            k_ss_rank_sort<<<(unsigned)cdiv(a.S, RK_SPB), RK_NT, 0, c->stream>>>(a, c->smp);
            a.smp = c->smp;
        } else {
            k_ss_sample<<<(unsigned)cdiv(a.S, 256), 256, 0, c->stream>>>(a, c->smp);
            Rec* s = nullptr;
            RC(merge_sort(c, c->smp, c->smp + a.S, a.S, &s));
            a.smp = s;
        }
        HIPCHK(c, hipGetLastError());
    }
    const bool small = a.B <= SS_LDSB;
    // enough workgroups that each thread takes a few records (the bucket search is a chain of
    // dependent reads); the large-B kernels keep one 128 KiB histogram per CU
    a.G = (u32)std::max<u64>(1, std::min<u64>(cdiv(np, small ? 1024 : 4096), (u64)c->ncu * (small ? 4 : 1)));
    // large B: a workgroup-major histogram and the bucket starts after it (B + 1 entries)
    const bool tr = !small && WCG_SS_TR;
    // the two-pass scatter: the records' buckets after pass 1 (n) and the cursors (B, and 256
    // coarse ones SX_CS apart)
    static const bool sx_off = getenv("WCG_SS_SX_OFF") != nullptr;   // A/B: the one-pass scatter
    const bool sx = tr && WCG_SS_SX && !sx_off;
    RC(ensure(c, &c->bid, &c->bid_cap, sx ? 2 * n + a.B + 256 * SX_CS : n));
    RC(ensure(c, &c->hist, &c->hist_cap, (u64)a.B * a.G + (tr ? a.B + 1 : 0)));
    RC(ensure(c, &c->irec, &c->irec_cap, 2 * n));
    a.bid = c->bid; a.hist = c->hist;
    a.bstart = tr ? c->hist + (u64)a.B * a.G : nullptr;
    a.irec = c->irec; a.irec2 = c->irec + n;
    a.sph = a.spl = nullptr; a.spi = nullptr;
    // long records: from the table (nlong) and, in two-pass jobs, from the record log (lemit);
    // their tie groups are listed by the bucket kernels and k_tie_edge (r04: k_tie_mark re-read
    // every sorted record, 0.14 ms on C4)
    const bool ties = n >= 2 && (dev || c->h_st->nlong + c->h_st->lemit >= 2);
    a.groups = nullptr; a.ngroups = nullptr; a.tie_zero = nullptr;
    if (ties && WCG_TIE_FUSED) {
        RC(ensure(c, &c->groups, &c->groups_cap, tie_list_cap(n)));
        a.groups = c->groups;
        a.ngroups = c->d_scalar + ST_TIE_GROUPS;   // device-sized jobs: k_compact zeroed it
        a.tie_zero = c->d_scalar + ST_TIE_BIG;      // the big-group counter (fix_ties)
        if (!dev) HIPCHK(c, hipMemsetAsync(a.ngroups, 0, sizeof(u64), c->stream));
    }
    if (!small) {                                  // the splitters as arrays (hi, lo, index)
        RC(ensure(c, &c->spx, &c->spx_cap, (u64)3 * a.B));
        a.sph = c->spx; a.spl = c->spx + a.B; a.spi = reinterpret_cast<u32*>(c->spx + 2 * a.B);
        k_ss_split<<<cdiv(a.B, 256), 256, 0, c->stream>>>(a);
    }
    if (small) k_ss_hist<true><<<a.G, SS_NT, 0, c->stream>>>(a);
    else if (WCG_SS_SPLIT && tr) {                 // r04: the search, then the histogram (wcg_sort.h)
        k_ss_find<<<(unsigned)std::max<u64>(1, std::min<u64>(cdiv(np, SSF_NT * SS_U), (u64)c->ncu * 2)), SSF_NT, 0,
                    c->stream>>>(a);
        k_ss_count<<<a.G, SSL_NT, 0, c->stream>>>(a);
    } else k_ss_hist<false><<<a.G, SSL_NT, 0, c->stream>>>(a);
    HIPCHK(c, hipGetLastError());
    if (tr) {
        k_ss_colscan<<<cdiv(a.B, 256), 256, 0, c->stream>>>(a.hist, a.B, a.G, a.bstart);
        RC(scan_u32(c, a.bstart, a.B));
    } else {
        RC(scan_u32(c, c->hist, (u64)a.B * a.G));
    }
    if (small) {
        k_ss_scatter<true><<<a.G, SS_NT, 0, c->stream>>>(a);
    } else if (sx) {                               // coarse buckets, then buckets (wcg_sort.h)
        const u32 lb = a.B > 1 ? 32u - (u32)__builtin_clz(a.B - 1u) : 0u;   // bits of B - 1
        const u32 sh = lb > 8 ? lb - 8 : 0;        // <= 256 coarse buckets
        u32* bid2 = c->bid + n;
        u32* fcur = bid2 + n;
        u32* ccur = fcur + a.B;
        k_ss_sxinit<<<cdiv(a.B, 256), 256, 0, c->stream>>>(a, ccur, fcur, sh);
        const unsigned tiles = (unsigned)std::max<u64>(1, cdiv(n, SX_T));
        k_ss_sx<1><<<tiles, SX_NT, 0, c->stream>>>(a, SxArgs{a.rec, a.bid, a.irec2, bid2, ccur, sh});
        k_ss_sx<2><<<tiles, SX_NT, 0, c->stream>>>(a, SxArgs{a.irec2, bid2, a.irec, nullptr, fcur, sh});
    } else {
        k_ss_scatter<false><<<a.G, SSL_NT, 0, c->stream>>>(a);
    }
    k_ss_bucket<0><<<a.B, SB_NT, 0, c->stream>>>(a);
    k_ss_bucket<1><<<a.B, SB_NT, 0, c->stream>>>(a);
    if (a.cls2) k_ss_bucket<2><<<a.B, SB_NT2, 0, c->stream>>>(a);
    if (a.groups) k_tie_edge<<<cdiv(a.B, TE_NT), TE_NT, 0, c->stream>>>(a);
    HIPCHK(c, hipGetLastError());
    if (ties) RC(fix_ties(c, c->recB, n, c->arena, c->recA, a.nd, a.dedupe ? a.nkeys : nullptr, a.groups != nullptr));
    if (c->crec == c->recA) c->compacted = false;    // recA was scratch for the ties
    if (getenv("WCG_DEBUG"))
        fprintf(stderr, "wcg: nemit %llu global_ops %llu long fallbacks %u long claims %llu\n",
                (unsigned long long)c->h_st->nemit, (unsigned long long)c->h_st->global_ops, c->h_st->long_fb,
                (unsigned long long)c->h_st->lnew);
    c->nkeys = n;
    // record-log jobs count their distinct keys on the device (d_scalar[8]); the count is read
    // with the formatted size at the end of wcg_reduce (one host round trip fewer)
    c->nkeys_on_device = a.dedupe;
    return WCG_OK;
}

// format records r[0:n) (key bytes of long records at `base`) into *dbuf, `bound` bytes at most;
// one synchronisation at the end returns the exact size
int format(wcg_ctx* c, const Rec* r, u64 n, const uint8_t* base, int fmt, u32 nreduce, u32 part, u64 bound,
           uint8_t** dbuf, u64* cap, u64* nbytes, const u64* nd = nullptr) {
    if (n == 0) { *nbytes = 0; return WCG_OK; }
    RC(ensure(c, dbuf, cap, bound + 64));
    const u64 nt = cdiv(n, FM_TILE);
    RC(ensure(c, &c->lens, &c->lens_cap, nt + 1));
    switch (fmt) {
#define WCG_FMT_SUM(F) case F: k_fmt_sum<F><<<(unsigned)nt, FM_NT, 0, c->stream>>>(r, n, nd, nreduce, part, base, c->lens); break;
        WCG_FMT_SUM(FMT_MERGED) WCG_FMT_SUM(FMT_JSON) WCG_FMT_SUM(FMT_JSON_ALL) WCG_FMT_SUM(FMT_COPY)
#undef WCG_FMT_SUM
        default: c->err = "format: unknown format"; return WCG_EINVAL;
    }
    k_scan_u64<<<1, 1024, 0, c->stream>>>(c->lens, nt, c->d_scalar);
    switch (fmt) {
#define WCG_FMT_WRITE(F) case F: k_fmt_write<F><<<(unsigned)nt, FM_NT, 0, c->stream>>>(r, n, nd, nreduce, part, base, c->lens, *dbuf); break;
        WCG_FMT_WRITE(FMT_MERGED) WCG_FMT_WRITE(FMT_JSON) WCG_FMT_WRITE(FMT_JSON_ALL) WCG_FMT_WRITE(FMT_COPY)
#undef WCG_FMT_WRITE
    }
    HIPCHK(c, hipGetLastError());
    // the size, and the sort's distinct-key count (d_scalar[8]) in the same copy; device-sized
    // jobs read the counters (the record count, errors) with them: the job's one round trip
    if (nd) HIPCHK(c, hipMemcpyAsync(c->h_st, c->st, ST_SCALAR_OFF + 9 * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
    else HIPCHK(c, hipMemcpyAsync(c->h_scalar, c->d_scalar, 9 * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *nbytes = *c->h_scalar;
    return WCG_OK;
}

u64 merged_bound(wcg_ctx* c, u64 n, bool json) {
    // inline keys <= 15 bytes; long keys <= 32 bytes in their cell, longer ones on the heap (its
    // used part is not known on the host in a device-sized job: the whole heap)
    return n * (LONG_CELL + (json ? JSON_FIXED : 3) + 20) +
           (c->dev_sized ? c->arena_cap : c->h_st->arena_top + c->h_st->lheap_top) + 64;
}

// every -res-<r> for nreduce R, back to back in c->d_part (cached until the next job)
int partition_all(wcg_ctx* c, u32 R) {
    if (c->part_R == R) return WCG_OK;
    const u64 n = c->nrec;
    c->part_bytes.assign(R, 0);
    if (n == 0) { c->part_R = R; return WCG_OK; }
    if (R > PT_MAXR) { c->err = "wcg_partition: nreduce above 1024"; return WCG_EINVAL; }
    const u64 T = cdiv(n, PT_TILE);
    RC(ensure(c, &c->pid, &c->pid_cap, n));
    RC(ensure(c, &c->hist, &c->hist_cap, (u64)R * T));
    RC(ensure(c, &c->d_partb, &c->partb_cap, R));
    HIPCHK(c, hipMemsetAsync(c->d_partb, 0, R * sizeof(u64), c->stream));
    k_part_hist<<<(unsigned)T, PT_NT, 0, c->stream>>>(c->sorted, n, R, c->arena, c->pid, c->hist, c->d_partb);
    HIPCHK(c, hipGetLastError());
    RC(scan_u32(c, c->hist, (u64)R * T));
    Rec* grouped = c->sorted == c->recA ? c->recB : c->recA;
    k_part_scatter<<<(unsigned)T, PT_NT, 0, c->stream>>>(c->sorted, n, R, c->pid, c->hist, grouped);
    HIPCHK(c, hipGetLastError());
    c->compacted = false;
    HIPCHK(c, hipMemcpyAsync(c->part_bytes.data(), c->d_partb, R * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    u64 total = 0;
    for (u32 r = 0; r < R; r++) total += c->part_bytes[r];
    u64 got = 0;
    RC(format(c, grouped, n, c->arena, FMT_JSON_ALL, 1, 0, total, &c->d_part, &c->part_cap, &got));
    if (got != total) { c->err = "wcg_partition: formatted size mismatch"; return WCG_EHIP; }
    c->part_R = R;
    return WCG_OK;
}

// ---------------------------------------------------------------- ingest
// the ingest's timing events for chunk k: [4k] copy start, [4k + 1] copy end, [4k + 2] map start,
// [4k + 3] map end
int ingest_events(wcg_ctx* c, u64 k) {
    while (c->ing_ev.size() < 4 * (k + 1)) {
        hipEvent_t e;
        HIPCHK(c, hipEventCreate(&e));
        c->ing_ev.push_back(e);
    }
    return WCG_OK;
}

int ingest_init(wcg_ctx* c) {
    if (c->hb[0]) return WCG_OK;
    // measurement knobs: chunk bytes (default 64 MiB) and reader threads (default min(16, cores))
    if (const char* e = getenv("WCG_INGEST_CHUNK_MIB")) c->chunk = std::max<u64>(1, strtoull(e, nullptr, 10)) << 20;
    for (int i = 0; i < INGEST_SLOTS; i++) {
        HIPCHK(c, hipHostMalloc(&c->hb[i], c->chunk + SCAN_MAX_LINE + 64, hipHostMallocDefault));
        HIPCHK(c, hipMalloc(&c->db[i], c->chunk + SCAN_MAX_LINE + 64));
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_copied[i], hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_mapped[i], hipEventDisableTiming));
    }
    HIPCHK(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    unsigned hw = std::thread::hardware_concurrency();
    unsigned nr = std::max(1u, std::min(16u, hw ? hw : 1u));
    if (const char* e = getenv("WCG_INGEST_READERS")) nr = std::max(1u, std::min(64u, (unsigned)atoi(e)));
    c->readers.reset(new TaskPool((int)nr));
    return WCG_OK;
}

// long tokens of the previous job up to which a one-pass map call runs long_small (k_agg)
constexpr u64 LONG_SMALL_MAX = 4096;

// a byte after which no rune and no token continues: an ASCII byte that is not a letter
inline bool safe_cut_byte(uint8_t b) { return b < 0x80 && ((b | 0x20) - 'a') >= 26u; }

// Stream `size` bytes from `read(dst, off, len)` through the staging buffers into the map
// kernels.  split_mode: Split's semantics (cut after '\n', a line of 64 KiB or more ends the
// input: quirk P1); otherwise DoMap's (every byte is mapped; chunks are cut after any ASCII
// non-letter, so no token or rune straddles a cut).  *mapped = bytes mapped.
int ingest(wcg_ctx* c, u64 size, const std::function<void(uint8_t*, u64, u64)>& read, bool split_mode, u64* mapped) {
    *mapped = 0;
    if (size == 0) return WCG_OK;
    RC(ingest_init(c));
    TaskPool& pool = *c->readers;
    u64 fo = 0, carry = 0, cut_prev = 0;
    int slot = 0;
    std::vector<SliceLines> sl(pool.size());
    // the copies and map launches, in chunk order, from a thread of their own (Issuer): this
    // thread goes on reading the next chunk meanwhile.  The context belongs to the issuer while
    // chunks are queued; this thread touches it again only after drain().
    std::string ierr;
    using clk = std::chrono::steady_clock;
    const auto t_start = clk::now();
    double read_ms = 0, wait_ms = 0;
    u64 nchunk = 0;                                   // chunks issued (the issuer's count)
    Issuer issuer([&](int s, u64 cut) -> int {
        if (hipSetDevice(c->device) != hipSuccess) { ierr = "hipSetDevice (ingest issuer)"; return WCG_EHIP; }
        if (ingest_events(c, nchunk)) { ierr = c->err; return WCG_EHIP; }
        hipEvent_t* ev = &c->ing_ev[4 * nchunk];
        nchunk++;
        hipError_t e = hipStreamWaitEvent(c->copy_stream, c->ev_mapped[s], 0);   // device slot free
        if (e == hipSuccess) e = hipEventRecord(ev[0], c->copy_stream);
        if (e == hipSuccess) e = hipMemcpyAsync(c->db[s], c->hb[s], cut, hipMemcpyHostToDevice, c->copy_stream);
        if (e == hipSuccess) e = hipEventRecord(ev[1], c->copy_stream);
        if (e == hipSuccess) e = hipEventRecord(c->ev_copied[s], c->copy_stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, c->ev_copied[s], 0);
        if (e == hipSuccess) e = hipEventRecord(ev[2], c->stream);
        if (e != hipSuccess) { ierr = std::string("ingest copy: ") + hipGetErrorString(e); return WCG_EHIP; }
        const int rc = wcg_map_device(c, c->db[s], cut);
        if (rc) return rc;
        e = hipEventRecord(ev[3], c->stream);
        if (e == hipSuccess) e = hipEventRecord(c->ev_mapped[s], c->stream);
        if (e == hipSuccess) e = hipEventSynchronize(c->ev_copied[s]);       // the staging buffer is free
        if (e != hipSuccess) { ierr = std::string("ingest copy: ") + hipGetErrorString(e); return WCG_EHIP; }
        return WCG_OK;
    });
    // the host side of the breakdown, once every chunk is issued (the device side is read from
    // the chunks' events by wcg_ingest_stats, so the ingest itself never waits for them)
    auto breakdown = [&]() {
        c->ing[0] = std::chrono::duration<double, std::milli>(clk::now() - t_start).count();
        c->ing[1] = read_ms;
        c->ing[2] = wait_ms;
        c->ing_chunks = nchunk;
    };
    auto drain = [&]() -> int {
        const int rc = issuer.drain();
        if (rc && !ierr.empty()) c->err = ierr;
        if (!rc) breakdown();
        return rc;
    };
    while (true) {
        {
            const auto tw = clk::now();
            const int rc = issuer.wait_slot(slot);                    // staging slot free
            wait_ms += std::chrono::duration<double, std::milli>(clk::now() - tw).count();
            if (rc) { (void)drain(); if (!ierr.empty()) c->err = ierr; return rc; }
        }
        const auto tr = clk::now();
        uint8_t* h = c->hb[slot];
        if (carry) memmove(h, c->hb[(slot + INGEST_SLOTS - 1) % INGEST_SLOTS] + cut_prev, carry);
        // the staging buffers hold chunk + SCAN_MAX_LINE bytes (a split-mode carry is < 64 KiB; a
        // DoMap-mode carry can be larger, then less is read)
        const u64 want = std::min<u64>(c->chunk + SCAN_MAX_LINE - carry, size - fo);
        const int T = want >= (4ull << 20) ? pool.size() : 1;
        if (T == 1) {
            read(h + carry, fo, want);
            if (split_mode) sl[0] = scan_slice(h, (int64_t)carry, (int64_t)(carry + want));
        } else {
            pool.run(T, [&](int t) {
                const u64 a = carry + want * t / T, b = carry + want * (t + 1) / T;
                read(h + a, fo + (a - carry), b - a);
                if (split_mode) sl[t] = scan_slice(h, (int64_t)a, (int64_t)b);
            });
        }
        read_ms += std::chrono::duration<double, std::milli>(clk::now() - tr).count();
        const u64 len = carry + want;
        fo += want;
        const bool eof = fo == size;
        bool stop = eof;
        u64 cut;
        if (split_mode) {
            // the carry is one partial line (no '\n'); lines start at 0 and after every '\n'
            int64_t prev = -1, bad = -1;
            for (int t = 0; t < T && bad < 0; t++) {
                if (sl[t].first < 0) continue;
                if (sl[t].first - (prev + 1) >= (int64_t)SCAN_MAX_LINE) { bad = prev + 1; break; }
                if (sl[t].bad >= 0) { bad = sl[t].bad; break; }
                prev = sl[t].last;
            }
            if (bad < 0 && (int64_t)len - (prev + 1) >= (int64_t)SCAN_MAX_LINE) bad = prev + 1;
            if (bad >= 0) { cut = (u64)bad; stop = true; }
            else cut = eof ? len : (u64)(prev + 1);
        } else if (eof) {
            cut = len;
        } else {
            cut = 0;
            for (u64 i = len; i > 0; i--)
                if (safe_cut_byte(h[i - 1])) { cut = i; break; }
            if (cut == 0) {
                // a token or rune run longer than the chunk: map the whole rest in one call from
                // a device buffer of its size (pathological input, e.g. 64 MiB of letters)
                const u64 rest = len + (size - fo);
                RC(drain());
                RC(ensure(c, &c->dbig, &c->dbig_cap, rest + 64));
                HIPCHK(c, hipStreamSynchronize(c->stream));
                HIPCHK(c, hipMemcpy(c->dbig, h, len, hipMemcpyHostToDevice));
                u64 done = len;
                while (fo < size) {
                    const u64 w = std::min<u64>(c->chunk, size - fo);
                    read(h, fo, w);
                    HIPCHK(c, hipMemcpy(c->dbig + done, h, w, hipMemcpyHostToDevice));
                    fo += w;
                    done += w;
                }
                RC(wcg_map_device(c, c->dbig, done));
                *mapped += done;
                return WCG_OK;
            }
        }
        if (cut > 0) {
            issuer.push(slot, cut);       // copy (after the device slot's previous map), then map
            *mapped += cut;
            static const bool sync_env = getenv("WCG_INGEST_SYNC") != nullptr;   // A/B: r03's order
            if (sync_env) { const int rc = issuer.wait_slot(slot); if (rc) { (void)drain(); return rc; } }
        }
        if (stop) break;
        carry = len - cut;
        cut_prev = cut;
        slot = (slot + 1) % INGEST_SLOTS;
    }
    return drain();
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
    HIPCHK(c, hipStreamCreateWithFlags(&c->long_stream, hipStreamNonBlocking));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
    c->gslots = next_pow2(2 * c->max_keys);
    c->lslots = std::max<u64>(next_pow2(c->gslots / 4), 4096);
    c->arena_cap = std::max<u64>(64ull << 20, c->lslots * 32);   // heap part (after the slot cells)
    // two-pass (high-cardinality) contexts: k_long_agg puts long keys straight into the record log,
    // their bytes on a heap of their own (at least one 32-byte cell each): room for a full log
    if (c->max_keys > (4ull << 20)) c->lheap_cap = 32 * (c->max_keys + 65536);
    HIPCHK(c, hipMalloc(&c->gtab, c->gslots * sizeof(GEntry)));
    HIPCHK(c, hipMalloc(&c->ltab, c->lslots * sizeof(GEntry)));
    HIPCHK(c, hipMalloc(&c->arena, c->lslots * LONG_CELL + c->arena_cap + c->lheap_cap + 64));
    // DevState and the scalars (scan totals, the tie-group count) in one block, so that one copy
    // reads a device-sized job's counters and sizes back
    static_assert(sizeof(DevState) <= ST_SCALAR_OFF, "DevState fits before the scalars");
    {
        uint8_t *d = nullptr, *h = nullptr;
        HIPCHK(c, hipMalloc(&d, ST_SCALAR_OFF + 64 * sizeof(u64)));
        HIPCHK(c, hipHostMalloc(&h, ST_SCALAR_OFF + 64 * sizeof(u64), hipHostMallocDefault));
        c->st = reinterpret_cast<DevState*>(d);
        c->h_st = reinterpret_cast<DevState*>(h);
        c->d_scalar = reinterpret_cast<u64*>(d + ST_SCALAR_OFF);
        c->h_scalar = reinterpret_cast<u64*>(h + ST_SCALAR_OFF);
        HIPCHK(c, hipMemset(d, 0, ST_SCALAR_OFF + 64 * sizeof(u64)));
    }
    // high-cardinality (two-pass) contexts list their few global-table claims (ginsert)
    if (c->max_keys > (4ull << 20)) {
        HIPCHK(c, hipMalloc(&c->glist, GLIST_CAP * sizeof(u64)));
        HIPCHK(c, hipMemcpy(c->d_scalar + ST_GLIST, &c->glist, sizeof(u64*), hipMemcpyHostToDevice));
        // ... and their long-key table's claims (C4: 1.6M of 16M slots per GiB; clearing and
        // compacting the whole 512 MiB table took 0.13 + ~0.15 ms of a 9.6 ms job)
        HIPCHK(c, hipMalloc(&c->llist, LLIST_CAP * sizeof(u64)));
        HIPCHK(c, hipMemcpy(c->d_scalar + ST_LLIST, &c->llist, sizeof(u64*), hipMemcpyHostToDevice));
    }
    // records: compaction output is bounded by the number of occupied slots
    c->rec_cap = c->max_keys + 65536;
    HIPCHK(c, hipMalloc(&c->recA, c->rec_cap * sizeof(Rec)));
    HIPCHK(c, hipMalloc(&c->recB, c->rec_cap * sizeof(Rec)));
    HIPCHK(c, hipHostMalloc(&c->h_cur, EX_MAX_RANKS * sizeof(u64), hipHostMallocDefault));
    HIPCHK(c, hipMalloc(&c->d_per_rank, 2 * EX_MAX_RANKS * sizeof(u64)));
    return wcg_reset(c);
}

int wcg_close(wcg_ctx* c) {
    if (!c) return WCG_EINVAL;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
    if (c->long_stream) (void)hipStreamSynchronize(c->long_stream);
    c->readers.reset();
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    for (int i = 0; i < INGEST_SLOTS; i++) {
        if (c->ev_copied[i]) (void)hipEventDestroy(c->ev_copied[i]);
    for (auto e : c->ing_ev) (void)hipEventDestroy(e);
        if (c->ev_mapped[i]) (void)hipEventDestroy(c->ev_mapped[i]);
        if (c->hb[i]) (void)hipHostFree(c->hb[i]);
        if (c->db[i]) (void)hipFree(c->db[i]);
    }
    void* bufs[] = {c->gtab, c->ltab, c->arena, c->st, c->recA, c->recB, c->lens, c->d_out,
                    c->d_part, c->owner, c->d_per_rank, c->exp_buf, c->pool, c->region_len, c->wg_stats,
                    c->llog, c->llog_len, c->smp, c->bid, c->spx, c->irec, c->lent, c->lpcur, c->spill, c->spill_len, c->pool2, c->rlen2, c->remit, c->ovf, c->hist, c->spart, c->ikey, c->iidx, c->groups,
                    c->pid, c->d_partb, c->nlpos, c->d_rb, c->d_b0, c->d_jin, c->d_jout, c->jhist, c->dbig,
                    c->d_xrow, c->xrecv, c->grecv, c->glist, c->llist, c->fr_buf, c->flist};
    if (c->comm) (void)ncclCommDestroy(c->comm);
    for (void* b : bufs) if (b) (void)hipFree(b);
    if (c->h_x) (void)hipHostFree(c->h_x);
    if (c->h_st) (void)hipHostFree(c->h_st);
    if (c->h_cur) (void)hipHostFree(c->h_cur);
    if (c->h_rb) (void)hipHostFree(c->h_rb);
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    if (c->long_stream) (void)hipStreamDestroy(c->long_stream);
    delete c;
    return WCG_OK;
}

int wcg_set_stream(wcg_ctx* c, void* stream) {
    if (!c) return WCG_EINVAL;
    hipStream_t next = stream ? (hipStream_t)stream : c->own_stream;
    if (next != c->stream) {
        // work already queued on the old stream (wcg_open's table clear, a reset that the next
        // reset will assume done) is ordered before anything queued on the new one
        int rc = set_dev(c);
        if (rc) return rc;
        hipEvent_t e;
        HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        hipError_t r1 = hipEventRecord(e, c->stream);
        hipError_t r2 = r1 == hipSuccess ? hipStreamWaitEvent(next, e, 0) : r1;
        (void)hipEventDestroy(e);
        HIPCHK(c, r2);
        c->stream = next;
    }
    return WCG_OK;
}

int wcg_enable_timing(wcg_ctx* c, int on) {
    if (!c) return WCG_EINVAL;
    c->timing = on != 0;
    c->timing_all = on == 1 || on == 2;
    c->timing_mode = on >= 2 && on <= 3 ? on : (on ? 1 : 0);
    if (c->timing_mode >= 2) {           // a new accumulation epoch
        c->map_ev.clear(); c->agg_ev.clear(); c->phase_jobs.clear(); c->xev.clear();
        c->ev_used = 0; c->map_launches = 0; c->phase_rec = false;
        for (double& v : c->acc) v = 0;
    }
    return WCG_OK;
}

}  // extern "C"

namespace {

// timing mode 2 keeps every job's events until wcg_timings; past this many events the pending
// pairs are folded into c->acc (one host wait every few hundred jobs) and the events reused
constexpr size_t EV_FOLD = 4096;

double ev_ms(hipEvent_t a, hipEvent_t b) {
    float f = 0;
    if (!a || !b || hipEventElapsedTime(&f, a, b) != hipSuccess) return 0.0;
    return f;
}

// every recorded phase pair added to acc[] (the caller has synchronised the stream)
void sum_events(const wcg_ctx* c, double* acc) {
    for (auto& p : c->map_ev) acc[0] += ev_ms(p.first, p.second);
    for (auto& p : c->agg_ev) acc[1] += ev_ms(p.first, p.second);
    for (auto& j : c->phase_jobs) {
        acc[2] += ev_ms(j[0], j[1]);
        acc[3] += ev_ms(j[2], j[3]);
        acc[4] += ev_ms(j[3], j[4]);
    }
    for (auto& x : c->xev) acc[std::get<0>(x)] += ev_ms(std::get<1>(x), std::get<2>(x));
}

void record_x(wcg_ctx* c, int phase, hipEvent_t a, hipEvent_t b) {
    if (c->timing_all && a && b) c->xev.emplace_back(phase, a, b);
}

hipEvent_t mark(wcg_ctx* c) {
    if (!c->timing_all) return nullptr;
    hipEvent_t e = take_event(c);
    return hipEventRecord(e, c->stream) == hipSuccess ? e : nullptr;
}

// a new job's tables: clear what may have been written since the last clear, reset the job state
// (wcg_reset; wcg_exchange before it imports the partitions this rank owns - the job's timing
// events are kept there)
int reset_tables(wcg_ctx* c) {
    // The global table (up to GBs) is cleared only if something may have written it since it was
    // last cleared: every kernel that inserts into it counts global_ops, and wcg_import sets
    // `imported`; two-pass jobs normally leave it empty.
    // One-pass map calls flush their tables into it, so only after two-pass calls is it worth a
    // host round trip to ask; with no map call since the last clear it is still clear.
    bool clear_g = true;
    const u64* glist = nullptr;                    // clear only the listed claims
    u64 g16 = c->gslots * sizeof(GEntry) / 16;
    bool have_st = false;
    auto read_st = [&]() -> int {
        if (have_st) return WCG_OK;
        HIPCHK(c, hipMemcpyAsync(c->h_st, c->st, sizeof(DevState), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        have_st = true;
        return WCG_OK;
    };
    const bool touched = c->map_launches_since_reset != 0 || c->imported;
    if (c->gtab_zero && !c->imported) {
        if (c->map_launches_since_reset == 0) clear_g = false;
        else if (c->two_pass_used) {
            RC(read_st());
            clear_g = c->h_st->global_ops != 0;
            if (clear_g && c->glist && c->h_st->gnew <= GLIST_CAP) { glist = c->glist; g16 = 2 * c->h_st->gnew; }
        }
    }
    // the long-key table: untouched since its last clear, or (large contexts) its listed claims
    const u64* llist = nullptr;
    u64 l16 = c->lslots * sizeof(GEntry) / 16;
    if (c->llist && c->ltab_zero) {
        if (!touched) l16 = 0;
        else {
            RC(read_st());
            if (c->h_st->lnew <= LLIST_CAP) { llist = c->llist; l16 = 2 * c->h_st->lnew; }
        }
    }
    c->map_launches_since_reset = 0;
    // one launch clears the tables and the counters (three memsets were three dispatches)
    if (!clear_g) g16 = 0;
    static_assert(sizeof(GEntry) == 32, "k_clear's listed entries are two 16-byte words");
    static const char* cg_env = getenv("WCG_CLEAR_GRID");       // measurement: workgroups of k_clear
    const u64 cgrid = cg_env ? std::max<u64>(1, (u64)atoi(cg_env)) : grid_for(g16 + l16, 256, c->ncu * 4);
    k_clear<<<(unsigned)cgrid, 256, 0, c->stream>>>(
        reinterpret_cast<uint4*>(c->gtab), g16, reinterpret_cast<uint4*>(c->ltab), l16, c->st, glist, llist);
    HIPCHK(c, hipGetLastError());
    c->gtab_zero = true;
    c->ltab_zero = true;
    c->counts_clean = true;
    c->compacted = c->reduced = c->merged = false;
    c->exp_ready = false;
    c->part_R = 0;
    c->nrec = 0;
    c->out_len = 0;
    c->two_pass_used = false;
    c->imported = false;
    return WCG_OK;
}

// WCG_AGG_CLOCK diagnostics: k_agg's per-workgroup durations against the miss-log units of
// its (bucket, slice), printed to stderr
int agg_clock_report(wcg_ctx* c, const AggArgs& g, u32 nb1, u64 grid) {
    std::vector<u64> clk(2 * nb1);
    std::vector<u32> rl(grid * g.P);
    HIPCHK(c, hipMemcpyAsync(clk.data(), g.clk, clk.size() * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(rl.data(), g.region_len, rl.size() * sizeof(u32), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    u64 t0 = ~0ull, t1 = 0;
    for (u32 b = 0; b < nb1; b++) { t0 = std::min(t0, clk[2 * b]); t1 = std::max(t1, clk[2 * b + 1]); }
    double sd = 0, su = 0, md = 0, mu = 0;
    double kd[2] = {0, 0}, km[2] = {0, 0}, ku[2] = {0, 0};   // short / medium buckets (split jobs)
    u32 kn[2] = {0, 0};
    u32 bmax = 0;
    std::vector<u64> units(nb1, 0);
    for (u32 bi = 0; bi < nb1; bi++) {
        u32 p, s, sl;                     // as agg_one
        if (bi < g.pm * g.slices) { p = bi % g.pm; s = bi / g.pm; sl = g.slices; }
        else { const u32 b2 = bi - g.pm * g.slices, nm = g.P - g.pm; p = g.pm + b2 % nm; s = b2 / nm; sl = g.slices_m; }
        const u32 k0 = (u32)((grid * s) / sl), k1 = (u32)((grid * (s + 1)) / sl);
        for (u32 k = k0; k < k1; k++) units[bi] += rl[(u64)k * g.P + p];
        const double d = (double)(clk[2 * bi + 1] - clk[2 * bi]);
        sd += d; su += (double)units[bi];
        if (d > md) { md = d; bmax = bi; }
        mu = std::max(mu, (double)units[bi]);
        const int kind = bi >= g.pm * g.slices;
        kd[kind] += d; km[kind] = std::max(km[kind], d); ku[kind] += (double)units[bi]; kn[kind]++;
    }
    static const char* dump = getenv("WCG_AGG_CLOCK_DUMP");   // path: every workgroup's line
    if (dump) {
        if (FILE* f = fopen(dump, "a")) {
            for (u32 bi = 0; bi < nb1; bi++)
                fprintf(f, "%u %u %llu %.2f %.2f\n", bi, (u32)(bi >= g.pm * g.slices), (unsigned long long)units[bi],
                        (clk[2 * bi] - t0) / 100.0, (clk[2 * bi + 1] - clk[2 * bi]) / 100.0);
            fprintf(f, "--\n");
            fclose(f);
        }
    }
    {   // the five slowest workgroups
        std::vector<u32> ord(nb1);
        for (u32 i = 0; i < nb1; i++) ord[i] = i;
        std::sort(ord.begin(), ord.end(), [&](u32 x, u32 y) { return clk[2 * x + 1] - clk[2 * x] > clk[2 * y + 1] - clk[2 * y]; });
        for (u32 r = 0; r < std::min<u32>(5, nb1); r++) {
            const u32 bi = ord[r];
            fprintf(stderr, "wcg k_agg clock: slow #%u bi %u (%s) dur %.1f us units %llu\n", r, bi,
                    bi >= g.pm * g.slices ? "medium" : "short", (clk[2 * bi + 1] - clk[2 * bi]) / 100.0,
                    (unsigned long long)units[bi]);
        }
    }
    for (int kind = 0; kind < 2; kind++)
        if (kn[kind])
            fprintf(stderr, "wcg k_agg clock: %s workgroups %u, dur mean %.1f max %.1f us, units mean %.0f\n",
                    kind ? "medium" : "short", kn[kind], kd[kind] / kn[kind] / 100.0, km[kind] / 100.0, ku[kind] / kn[kind]);
    fprintf(stderr, "wcg k_agg clock: span %.1f us, wg dur mean %.1f max %.1f us (bi %u: %llu units, start +%.1f us), "
            "units mean %.0f max %.0f\n", (t1 - t0) / 100.0, sd / nb1 / 100.0, md / 100.0, bmax,
            (unsigned long long)units[bmax], (clk[2 * bmax] - t0) / 100.0, su / nb1, mu);
    return WCG_OK;
}

}  // namespace

extern "C" {

int wcg_reset(wcg_ctx* c) {
    if (!c) return WCG_EINVAL;
    c->pending = false;                 // a wcg_reduce_async job not waited for is dropped
    int rc = set_dev(c);
    if (rc) return rc;
    if (c->timing_mode >= 2 && c->ev_used >= EV_FOLD) {   // recycle the events of earlier jobs
        HIPCHK(c, hipStreamSynchronize(c->stream));
        sum_events(c, c->acc);
        c->map_ev.clear(); c->agg_ev.clear(); c->phase_jobs.clear(); c->xev.clear();
        c->ev_used = 0;
    }
    RC(reset_tables(c));
    if (c->timing_mode < 2) {           // modes 2, 3 keep every job's events until wcg_timings
        c->map_ev.clear();
        c->agg_ev.clear();
        c->xev.clear();
        c->ev_used = 0;
        c->phase_rec = false;
        c->map_launches = 0;
    }
    return WCG_OK;
}

int wcg_map_device(wcg_ctx* c, const void* dev_bytes, uint64_t n) {
    if (!c) return WCG_EINVAL;
    c->pending = false;
    if (n == 0) return WCG_OK;
    if (!dev_bytes || ((uintptr_t)dev_bytes & 15)) { c->err = "wcg_map_device: input must be 16-byte aligned"; return WCG_EINVAL; }
    int rc = set_dev(c);
    if (rc) return rc;
    MapArgs a;
    a.in = (const uint8_t*)dev_bytes;
    a.n = n;
    a.ntiles = (n + MAP_STEP - 1) / MAP_STEP;      // 992-byte wave steps (1 KiB windows)
    // one workgroup per CU (LDS-bound); steps are dealt chip-wide inside the kernel
    u64 grid = std::min<u64>((u64)c->ncu * MAP_WGS, (a.ntiles + MAP_WAVES - 1) / MAP_WAVES);
    // steps per workgroup (sizing only): wave w of workgroup g takes steps g*16 + w + k*G*16, so
    // a workgroup runs at most MAP_WAVES * ceil(ntiles / (G * MAP_WAVES)) of them
    a.tiles_per_wg = MAP_WAVES * ((a.ntiles + grid * MAP_WAVES - 1) / (grid * MAP_WAVES));
    a.gtab = c->gtab; a.gmask = c->gslots - 1;
    a.ltab = c->ltab; a.lmask = c->lslots - 1;
    a.arena = c->arena; a.arena_cap = c->arena_cap; a.lheap_cap = c->lheap_cap;
    a.st = c->st;
    // miss log: one region per (workgroup, bucket) of 8-byte units; the whole pool is ~2n
    // bytes: a unit for every 4 input bytes covers every token missing the LDS table even on
    // high-cardinality UTF-8 text (C4: 0.1 tokens per byte, 79% misses, 2-unit keys), where a
    // 1-per-8 pool overflowed into per-token global-table inserts; only written units cost time
    // miss buckets: one-pass jobs (r06) log short keys (<= 7 bytes) and medium keys to disjoint
    // halves, so that every k_agg workgroup aggregates one kind only (a wave that mixed them paid the
    // medium keys' dependent k1 reads on nearly every probe: C2 k_agg with medium entries dropped ran
    // 0.197 ms against 0.270, profiles/r06_experiments); two-pass jobs keep one set of buckets
    static const char* tp_env0 = getenv("WCG_AGG_TWO_PASS");
    const bool two_pass0 = tp_env0 ? atoi(tp_env0) != 0 : c->max_keys > (4ull << 20);
    static const char* sp_env = getenv("WCG_AGG_SPLIT");       // measurement: 0 = one set of buckets
    const bool split = !two_pass0 && !(sp_env && atoi(sp_env) == 0);
    const u32 P = split ? MISS_SHORT_BUCKETS + MISS_SHORT_BUCKETS / 2 : MISS_SHORT_BUCKETS;   // short, then medium
    static_assert(MISS_SHORT_BUCKETS + MISS_SHORT_BUCKETS / 2 <= MAX_MISS_BUCKETS, "k_map's LDS cursors cover P");
    u64 per_wg_bytes = (u64)a.tiles_per_wg * MAP_STEP;
    // even (16-byte aligned regions); a workgroup's regions stay under 2 GiB so k_map's unit
    // offsets fit 32 bits and its 24-bit multiplies (P * region_cap * 8 <= 2^31)
    // (split buckets: every region sized like an unsplit bucket's)
    a.region_cap = std::min<u64>(std::max<u64>(2048, per_wg_bytes / (4ull * MISS_SHORT_BUCKETS)), (1ull << 31) / (8ull * P)) & ~1ull;
    static const char* rpad_env = getenv("WCG_REGION_PAD");   // measurement: units added to a region
    if (rpad_env && a.region_cap + (u64)(atoi(rpad_env) & ~1) <= (1ull << 31) / (8ull * P))
        a.region_cap += (u64)(atoi(rpad_env) & ~1);
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
    // long-token log: LLOG_PER_STEP records per step, the most a step can start (C4 text logs
    // ~5.3 per step), so no region fills and k_map needs no inline fallback (an inlined insert
    // path pushed k_map past its register budget into spills of its prefetch registers)
    a.llog_cap = (u32)std::min<u64>((u64)a.tiles_per_wg * LLOG_PER_STEP + 64, 0xFFFFFFFFull);
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
    // Two passes only for high-cardinality jobs (the table is sized for more than 4M keys, or
    // WCG_AGG_TWO_PASS=1): on low-cardinality text nothing spills, and the extra launches and the
    // record-log merge would only cost time.  One pass sends an entry its LDS table cannot take
    // to the global table.  Two-pass jobs keep the global table empty: pass 2's records, its
    // overflow and k_long_hash's inline runs all go to the record log.
    const bool two_pass = two_pass0;
    const u64 rec_cap_emit = c->max_keys + 65536;
    RC(ensure(c, &c->remit, &c->remit_cap, rec_cap_emit));
    a.emit = two_pass ? c->remit : nullptr;
    a.emit_cap = rec_cap_emit;
    a.pool = c->pool;
    a.region_len = c->region_len;
    a.wg_stats = c->wg_stats;
    a.stamps = nullptr;
#if WCG_STAMPS
    static u64* d_stamps = nullptr;
    if (!d_stamps) HIPCHK(c, hipMalloc(&d_stamps, MAP_NSTAMP * sizeof(u64)));
    HIPCHK(c, hipMemsetAsync(d_stamps, 0, MAP_NSTAMP * sizeof(u64), c->stream));
    a.stamps = d_stamps;
#endif
    // timing: the kernel's own start / end timestamps through hipExtLaunchKernel (events recorded
    // as separate stream markers cost a ~5 us bubble each between the kernels around them)
    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
    if (c->timing) { e0 = take_event(c); e1 = take_event(c); }
    static const int ablate = getenv("WCG_MAP_ABLATE") ? atoi(getenv("WCG_MAP_ABLATE")) : 0;
    auto launch = [&](auto kern) {
        if (e0) hipExtLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(MAP_NT), 0, c->stream, e0, e1, 0u, a);
        else kern<<<(unsigned)grid, MAP_NT, 0, c->stream>>>(a);
    };
    switch (ablate) {
        case 1: split ? launch(k_map<1, true>) : launch(k_map<1, false>); break;
        case 2: split ? launch(k_map<2, true>) : launch(k_map<2, false>); break;
        case 3: split ? launch(k_map<3, true>) : launch(k_map<3, false>); break;
        case 4: split ? launch(k_map<4, true>) : launch(k_map<4, false>); break;
        case 5: split ? launch(k_map<5, true>) : launch(k_map<5, false>); break;
        case 6: split ? launch(k_map<6, true>) : launch(k_map<6, false>); break;
        case 7: split ? launch(k_map<7, true>) : launch(k_map<7, false>); break;
        default: split ? launch(k_map<0, true>) : launch(k_map<0, false>); break;
    }
    HIPCHK(c, hipGetLastError());
#if WCG_STAMPS
    {   // diagnostics: cycles per step and phase, averaged over every wave's steps
        u64 h[MAP_NSTAMP];
        HIPCHK(c, hipMemcpyAsync(h, d_stamps, sizeof h, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        const double ns = h[6] ? (double)h[6] : 1.0;
        fprintf(stderr, "wcg stamps (s_memtime ticks per wave step, %llu steps): loop %.0f wait %.0f mask %.0f "
                "list %.0f short %.0f general %.0f\n", (unsigned long long)h[6], h[0] / ns, h[1] / ns, h[2] / ns,
                h[3] / ns, h[4] / ns, h[5] / ns);
    }
#endif
    // the logged long tokens: hashed into LQ partitions (LONG_PARTS workgroups per map
    // workgroup's region), then one workgroup per partition.  Partition capacity: the log's
    // capacity spread evenly, with slack (the LDS cache folds hot keys before they are emitted;
    // a full partition falls back to exact per-entry inserts)
    // They run on long_stream, forked after k_map and joined before this call returns: they and
    // k_agg read k_map's outputs only and share nothing but atomic counters (the record log's
    // cursor, the global table's claim protocol), and both are latency-bound (C4 1 GiB: 1.7 ms of
    // long-key work beside 3.2 ms of aggregation)
    // Only two-pass (high-cardinality) jobs fork: on low-cardinality text the long-key kernels
    // take ~25 us and could not run beside k_agg anyway (its workgroups fill every CU's LDS),
    // while the fork and join cost ~25 us of dependency latency.
    const bool long_path = ablate == 0 || ablate >= 6;
    static const char* fork_env = getenv("WCG_LONG_FORK");     // diagnostics: 0 = in line (alone)
    const bool fork = long_path && two_pass && !(fork_env && atoi(fork_env) == 0);
    hipStream_t ls = fork ? c->long_stream : c->stream;
    if (fork) {
        HIPCHK(c, hipEventRecord(c->ev_fork, c->stream));
        HIPCHK(c, hipStreamWaitEvent(c->long_stream, c->ev_fork, 0));
    }
    // one-pass calls after a job with few long tokens: one workgroup (k_agg's last) does it all
    static const char* ls_env = getenv("WCG_LONG_SMALL");        // measurement: 0 = never, 1 = always
    const bool small = long_path && !two_pass && grid <= LS_MAXREG &&
                       (ls_env ? atoi(ls_env) != 0 : c->long_hint <= LONG_SMALL_MAX);
    if (small) {
        // (run by k_agg's last workgroup, below)
    } else if (long_path) {
        LongPart lp;
        const u64 expect = grid * (u64)a.tiles_per_wg * 16;     // 16 per step: 3x C4's rate
        lp.cap = (u32)std::min<u64>(std::max<u64>(1024, (expect * 5 / 4 + LQ - 1) / LQ), 0x7FFFFFFFull);
        RC(ensure(c, &c->lent, &c->lent_cap, (u64)LQ * lp.cap));
        u32* const old_cur = c->lpcur;
        RC(ensure(c, &c->lpcur, &c->lpcur_cap, (u64)LQ));
        // k_long_agg leaves every partition cursor at zero for the next map call
        if (c->lpcur != old_cur) HIPCHK(c, hipMemsetAsync(c->lpcur, 0, LQ * sizeof(u32), ls));
        lp.ent = c->lent; lp.cur = c->lpcur;
        k_long_hash<<<(unsigned)std::min<u64>(grid * LONG_PARTS, (u64)c->ncu * 4), LONG_NT, 0, ls>>>(a, lp, (u32)grid);
#ifndef WCG_LA_PERSIST
#define WCG_LA_PERSIST 1
#endif
        static_assert(LQ / LA_MAXQ <= 256, "k_long_agg's grid covers every partition");
        k_long_agg<<<(unsigned)(WCG_LA_PERSIST ? std::max<u64>(std::min<u64>(LQ, c->ncu), LQ / LA_MAXQ) : LQ), LA_NT,
                     0, ls>>>(a, lp);
        HIPCHK(c, hipGetLastError());
        if (fork) HIPCHK(c, hipEventRecord(c->ev_join, c->long_stream));
    }
    // k_agg pass 1 (spills what its LDS tables cannot hold) -> k_rp -> pass 2 (wcg_agg.h)
    AggArgs g;
    g.pool = c->pool; g.region_len = c->region_len; g.region_cap = a.region_cap;
    g.P = P; g.nsrc = (u32)grid;
    const u32 min_sl = (u32)((grid + AGG_MAX_SRC - 1) / AGG_MAX_SRC);   // <= AGG_MAX_SRC regions per item
    if (split) {
        // the medium buckets (~11% of C2's tokens, ~1/4 of the units) a quarter of the CUs, the
        // short buckets the rest: ~one workgroup per CU of ~equal time
        g.pm = MISS_SHORT_BUCKETS;
        const u32 nm = P - g.pm;
        static const char* ms_env = getenv("WCG_AGG_MSLICES");   // measurement: medium slices
        g.slices_m = std::max<u32>(min_sl, std::max<u32>(1, std::min<u32>((u32)grid,
                                   ms_env ? (u32)atoi(ms_env) : (u32)c->ncu / 4 / nm)));
        g.slices = std::max<u32>(min_sl, std::max<u32>(1, std::min<u32>((u32)grid,
                                 (u32)(c->ncu > g.slices_m * nm ? (c->ncu - g.slices_m * nm) / g.pm : 1))));
    } else {
        g.pm = P;
        g.slices_m = 1;
        g.slices = std::max<u32>(1, std::min<u32>((u32)grid, (u32)(c->ncu + P - 1) / P));
        g.slices = std::max<u32>(g.slices, min_sl);
    }
    g.nbi = g.pm * g.slices + (P - g.pm) * g.slices_m;
    g.ls_nreg = small ? (u32)grid : 0u;
    g.rstride = P; g.rmod = P; g.P1 = P; g.mode = AGG_SPILL;
    g.gtab = c->gtab; g.gmask = c->gslots - 1; g.st = c->st;
    g.map_stats = c->wg_stats;
    const u32 nb1 = g.nbi;
    g.spill_cap = 0;                      // one pass: a full LDS table inserts into the global table
    g.spill = nullptr; g.spill_len = nullptr;
    g.emit = c->remit; g.emit_cap = rec_cap_emit;
    g.ovf = nullptr; g.ovf_cap = 0;
    g.clk = nullptr;
    // one-pass flush through a list of the occupied slots (WCG_AGG_FLIST = 0: slot by slot)
    g.flist = nullptr;
    static const char* fl_env = getenv("WCG_AGG_FLIST");
    if (!two_pass && !(fl_env && atoi(fl_env) == 0)) {
        RC(ensure(c, &c->flist, &c->flist_cap, (u64)nb1 * AGG_NB * AGG_W));
        g.flist = c->flist;
    }
    static const bool agg_clock = getenv("WCG_AGG_CLOCK") != nullptr;
    static u64* d_clk = nullptr;
    if (agg_clock && !two_pass) {          // diagnostics: per-workgroup time against its units
        if (!d_clk) HIPCHK(c, hipMalloc(&d_clk, 2 * 65536 * sizeof(u64)));
        g.clk = nb1 <= 65536 ? d_clk : nullptr;
    }
    if (!two_pass) {
        k_agg<AGG_SPILL><<<nb1 + (small ? 1 : 0), AGG_NT, 0, c->stream>>>(g, a);
        HIPCHK(c, hipGetLastError());
        c->counts_clean = true;                // its block 0 zeroed nrec / nlong
        if (g.clk) RC(agg_clock_report(c, g, nb1, grid));
    } else {
    c->two_pass_used = true;
    // k_rp splits each (bucket, slice) of the miss log into AGG_Q sub-buckets; a sub-bucket region
    // holds 1.5x an even share of what its slice's regions can hold, a full one falls back to
    // exact global inserts
    // k_rp's slices of map workgroups: twice pass 1's, so that k_rp's 52 KiB workgroups run two
    // per CU (C4 1 GiB: aggregation 3.71 -> 3.49 ms against one 100 KiB workgroup per CU,
    // profiles/r03_kagg_experiments/rp_slices.txt; WCG_RP_SLICES: measurement override)
    static const char* rps_env = getenv("WCG_RP_SLICES");
    const u32 sl = std::max<u32>(1, std::min<u32>((u32)grid, rps_env ? (u32)atoi(rps_env) : 2 * g.slices));
    const u32 nrp = P * sl;
    const u64 slice_cap = (u64)cdiv(grid, sl) * a.region_cap;
    const u64 cap2 = ((slice_cap * 3 / 2) / AGG_Q + 1024) & ~1ull;
    RC(ensure(c, &c->pool2, &c->pool2_cap, (u64)nrp * AGG_Q * cap2 + AGG_SLACK_UNITS));
    RC(ensure(c, &c->rlen2, &c->rlen2_cap, (u64)nrp * AGG_Q));
    RpArgs rp;
    rp.pool = c->pool; rp.region_len = c->region_len; rp.region_cap = a.region_cap;
    rp.P = P; rp.nsrc = (u32)grid; rp.slices = sl; rp.map_stats = c->wg_stats;
    rp.pool2 = c->pool2; rp.cap2 = cap2; rp.region_len2 = c->rlen2;
    rp.gtab = c->gtab; rp.gmask = c->gslots - 1; rp.st = c->st;
    k_rp<<<nrp, AGG_NT, 0, c->stream>>>(rp);
    AggArgs g2 = g;
    g2.pool = c->pool2; g2.region_len = c->rlen2; g2.region_cap = cap2;
    g2.P = P * AGG_Q; g2.nsrc = sl; g2.slices = 1;
    g2.pm = g2.P; g2.slices_m = 1; g2.nbi = g2.P;
    g2.rstride = AGG_Q; g2.rmod = AGG_Q; g2.P1 = P; g2.mode = AGG_EMIT;
    const u32 grid2 = std::min<u32>(P * AGG_Q, (u32)c->ncu * 2);
    g2.ovf_cap = AGG_OVF_CAP;
    RC(ensure(c, &c->ovf, &c->ovf_cap, (u64)grid2 * AGG_OVF_CAP));
    g2.ovf = c->ovf;
    g2.ls_nreg = 0;
    k_agg<AGG_EMIT><<<grid2, AGG_NT, 0, c->stream>>>(g2, a);
    HIPCHK(c, hipGetLastError());
    }
    if (fork) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));
    if (c->timing) {
        c->map_ev.push_back({e0, e1});
        if (c->timing_all) {             // mode 3 times the map kernel only (an event is a ~5 us bubble)
            e2 = take_event(c);
            HIPCHK(c, hipEventRecord(e2, c->stream));
            c->agg_ev.push_back({e1, e2});
        }
    }
    c->map_launches++;
    c->map_launches_since_reset++;
    c->compacted = c->reduced = c->merged = false;
    c->exp_ready = false;
    c->part_R = 0;
    return WCG_OK;
}

int wcg_map(wcg_ctx* c, const uint8_t* host_bytes, uint64_t n) {
    if (!c) return WCG_EINVAL;
    c->pending = false;
    if (n == 0) return WCG_OK;
    if (!host_bytes) return WCG_EINVAL;
    int rc = set_dev(c);
    if (rc) return rc;
    return ingest(c, n, [&](uint8_t* dst, u64 off, u64 len) { memcpy(dst, host_bytes + off, len); }, false,
                  &c->ingest_bytes);
}

int wcg_map_file(wcg_ctx* c, const char* path, uint64_t* mapped_bytes, uint64_t* file_bytes) {
    if (!c || !path) return WCG_EINVAL;
    c->pending = false;
    int rc = set_dev(c);
    if (rc) return rc;
    const int fd = open(path, O_RDONLY);
    if (fd < 0) { c->err = std::string("wcg_map_file: open ") + path + ": " + strerror(errno); return WCG_EINVAL; }
    struct stat sb;
    if (fstat(fd, &sb) != 0) { close(fd); c->err = "wcg_map_file: stat failed"; return WCG_EINVAL; }
    const u64 size = (u64)sb.st_size;
    bool ioerr = false;
    rc = ingest(c, size, [&](uint8_t* dst, u64 off, u64 len) {
        while (len) {
            const ssize_t r = pread(fd, dst, len, (off_t)off);
            if (r <= 0) { ioerr = true; memset(dst, '\n', len); return; }
            dst += r; off += (u64)r; len -= (u64)r;
        }
    }, true, &c->ingest_bytes);
    close(fd);
    if (rc) return rc;
    if (ioerr) { c->err = "wcg_map_file: read error"; return WCG_EHIP; }
    if (mapped_bytes) *mapped_bytes = c->ingest_bytes;
    if (file_bytes) *file_bytes = size;
    return WCG_OK;
}

int wcg_ingest_stats(wcg_ctx* c, double* out, int n) {
    if (!c || !out || n < 0) return WCG_EINVAL;
    int rc = set_dev(c);
    if (rc) return rc;
    RC(resolve(c));
    double copy = 0, map = 0, span = 0, dev = 0;
    const u64 nk = c->ing_chunks;
    if (nk) {
        HIPCHK(c, hipStreamSynchronize(c->copy_stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        const hipEvent_t* ev = c->ing_ev.data();
        for (u64 k = 0; k < nk; k++) {
            float a = 0, b = 0;
            HIPCHK(c, hipEventElapsedTime(&a, ev[4 * k], ev[4 * k + 1]));
            HIPCHK(c, hipEventElapsedTime(&b, ev[4 * k + 2], ev[4 * k + 3]));
            copy += a;
            map += b;
        }
        float sp = 0, dv = 0;
        HIPCHK(c, hipEventElapsedTime(&sp, ev[0], ev[4 * (nk - 1) + 1]));
        HIPCHK(c, hipEventElapsedTime(&dv, ev[0], ev[4 * (nk - 1) + 3]));
        span = sp;
        dev = dv;
    }
    const double st[9] = {c->ing[0], c->ing[1], c->ing[2], copy, span, span > 0 ? std::max(0.0, 1.0 - copy / span) : 0.0,
                          map, dev, (double)nk};
    for (int i = 0; i < n && i < 9; i++) out[i] = st[i];
    return WCG_OK;
}

int wcg_reduce(wcg_ctx* c, uint64_t* nkeys, uint64_t* nbytes) {
    if (!c) return WCG_EINVAL;
    int rc = set_dev(c);
    if (rc) return rc;
    c->phase_ev[0] = c->phase_ev[1] = nullptr;     // set by compact() only when it runs now
    RC(resolve(c));
    c->fused_last = false;
    if (fused_eligible(c)) {
        rc = reduce_fused(c);
        if (!rc) rc = reduce_fused_finish(c);
        if (rc) return rc;
        if (c->timing_all) {                       // the fused launch counts as the sort phase
            c->phase_ev[4] = c->phase_ev[3];
            c->phase_rec = true;
            if (c->timing_mode == 2)
                c->phase_jobs.push_back({c->phase_ev[0], c->phase_ev[1], c->phase_ev[2], c->phase_ev[3], c->phase_ev[4]});
        }
        c->reduced = true;
        c->merged = false;
        c->part_R = 0;
        if (nkeys) *nkeys = c->nkeys;
        if (nbytes) *nbytes = c->out_len;
        return WCG_OK;
    }
    RC(compact(c, true));
    c->merged = false;
    // sort + format; a device-sized job that fails in them leaves no capacity-sized record count
    // behind for a later export or reduce to trust
    rc = [&]() -> int {
        if (c->timing_all) { c->phase_ev[2] = take_event(c); HIPCHK(c, hipEventRecord(c->phase_ev[2], c->stream)); }
        RC(sort_records(c));
        if (c->timing_all) { c->phase_ev[3] = take_event(c); HIPCHK(c, hipEventRecord(c->phase_ev[3], c->stream)); }
        RC(format(c, c->sorted, c->nrec, c->arena, FMT_MERGED, 1, 0, merged_bound(c, c->nrec, false), &c->d_out,
                  &c->out_cap, &c->out_len, c->dev_sized ? &c->st->nrec : nullptr));
        return WCG_OK;
    }();
    if (rc) {
        if (c->dev_sized) { c->dev_sized = false; c->compacted = false; c->nrec = 0; c->out_len = 0; }
        return rc;
    }
    if (c->dev_sized) {                            // the counters came back with the size
        c->dev_sized = false;
        c->nrec = c->nkeys = c->h_st->nrec;
        if (c->h_st->bad_input || c->h_st->overflow || c->h_st->spin_fail) {
            c->compacted = false;
            RC(check_status(c));                   // the error message (k_compact wrote nothing)
        }
    }
    c->nrec_hint = c->nrec;
    if (c->h_st) c->long_hint = c->h_st->long_tokens;     // (a hint: read back with the sizes)
    if (c->timing_all) {
        c->phase_ev[4] = take_event(c);
        HIPCHK(c, hipEventRecord(c->phase_ev[4], c->stream));
        c->phase_rec = true;
        if (c->timing_mode == 2)
            c->phase_jobs.push_back({c->phase_ev[0], c->phase_ev[1], c->phase_ev[2], c->phase_ev[3], c->phase_ev[4]});
    }
    if (c->nkeys_on_device) {
        if (c->nrec == 0) c->nkeys = 0;               // format returned early: nothing sorted
        else c->nkeys = c->h_scalar[8];
        c->nkeys_on_device = false;
    }
    c->reduced = true;
    c->part_R = 0;
    if (nkeys) *nkeys = c->nkeys;
    if (nbytes) *nbytes = c->out_len;
    return WCG_OK;
}

int wcg_reduce_async(wcg_ctx* c) {
    if (!c) return WCG_EINVAL;
    int rc = set_dev(c);
    if (rc) return rc;
    RC(resolve(c));
    if (!fused_eligible(c)) return wcg_reduce(c, nullptr, nullptr);   // the other paths read back at once
    c->phase_ev[0] = c->phase_ev[1] = nullptr;
    c->fused_last = false;
    RC(reduce_fused(c));
    if (c->timing_all) {
        c->phase_ev[4] = c->phase_ev[3];
        c->phase_rec = true;
        if (c->timing_mode == 2)
            c->phase_jobs.push_back({c->phase_ev[0], c->phase_ev[1], c->phase_ev[2], c->phase_ev[3], c->phase_ev[4]});
    }
    c->pending = true;
    c->reduced = true;
    c->merged = false;
    c->part_R = 0;
    return WCG_OK;
}

int wcg_reduce_wait(wcg_ctx* c, uint64_t* nkeys, uint64_t* nbytes) {
    if (!c) return WCG_EINVAL;
    if (!c->reduced) { c->err = "wcg_reduce_wait without a wcg_reduce_async job"; return WCG_ESTATE; }
    int rc = set_dev(c);
    if (rc) return rc;
    RC(resolve(c));
    if (nkeys) *nkeys = c->nkeys;
    if (nbytes) *nbytes = c->out_len;
    return WCG_OK;
}

int wcg_result_device(wcg_ctx* c, const void** dev_ptr, uint64_t* nbytes) {
    if (!c) return WCG_EINVAL;
    RC(resolve(c));
    if (!c->reduced) { c->err = "wcg_result_device before wcg_reduce"; return WCG_ESTATE; }
    if (dev_ptr) *dev_ptr = c->d_out;
    if (nbytes) *nbytes = c->out_len;
    return WCG_OK;
}

int wcg_free(wcg_ctx* c, const void* dev_ptr) {
    if (!c) return WCG_EINVAL;
    if (!dev_ptr) return WCG_OK;
    int rc = set_dev(c);
    if (rc) return rc;
    if (dev_ptr == c->d_out) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipFree(c->d_out));
        c->d_out = nullptr; c->out_cap = 0; c->out_len = 0;
        c->reduced = false;
        return WCG_OK;
    }
    if (dev_ptr == c->exp_buf) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipFree(c->exp_buf));
        c->exp_buf = nullptr; c->exp_cap = 0;
        return WCG_OK;
    }
    c->err = "wcg_free: not a buffer this context handed out";
    return WCG_EINVAL;
}

int wcg_result_copy(wcg_ctx* c, uint8_t* host_out, uint64_t cap) {
    if (!c) return WCG_EINVAL;
    RC(resolve(c));
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

int wcg_result_copy_device(wcg_ctx* c, void* dev_dst) {
    if (!c) return WCG_EINVAL;
    RC(resolve(c));
    if (!c->reduced) { c->err = "wcg_result_copy_device before wcg_reduce"; return WCG_ESTATE; }
    int rc = set_dev(c);
    if (rc) return rc;
    if (c->out_len) HIPCHK(c, hipMemcpyAsync(dev_dst, c->d_out, c->out_len, hipMemcpyDeviceToDevice, c->stream));
    return WCG_OK;
}

int wcg_sync(wcg_ctx* c) {
    if (!c) return WCG_EINVAL;
    RC(resolve(c));
    int rc = set_dev(c);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return WCG_OK;
}

int wcg_partition_all(wcg_ctx* c, uint32_t nreduce, uint8_t* host_out, uint64_t cap, uint64_t* part_bytes) {
    if (!c) return WCG_EINVAL;
    RC(resolve(c));
    if (!c->reduced) { c->err = "wcg_partition_all before wcg_reduce"; return WCG_ESTATE; }
    if (c->merged) { c->err = "wcg_partition_all after wcg_merge_runs (a merged file has no partitions)"; return WCG_ESTATE; }
    if (nreduce == 0) { c->err = "wcg_partition_all: nreduce 0"; return WCG_EINVAL; }
    int rc = set_dev(c);
    if (rc) return rc;
    RC(partition_all(c, nreduce));
    u64 total = 0;
    for (u32 r = 0; r < nreduce; r++) {
        if (part_bytes) part_bytes[r] = c->part_bytes[r];
        total += c->part_bytes[r];
    }
    if (host_out) {
        if (cap < total) { c->err = "wcg_partition_all: buffer too small"; return WCG_EINVAL; }
        if (total) {
            HIPCHK(c, hipMemcpyAsync(host_out, c->d_part, total, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
        }
    }
    return WCG_OK;
}

int wcg_partition(wcg_ctx* c, uint32_t nreduce, uint32_t r, uint8_t* host_out, uint64_t cap, uint64_t* nbytes) {
    if (!c) return WCG_EINVAL;
    RC(resolve(c));
    if (!c->reduced) { c->err = "wcg_partition before wcg_reduce"; return WCG_ESTATE; }
    if (c->merged) { c->err = "wcg_partition after wcg_merge_runs (a merged file has no partitions)"; return WCG_ESTATE; }
    if (nreduce == 0 || r >= nreduce) { c->err = "wcg_partition: bad partition"; return WCG_EINVAL; }
    int rc = set_dev(c);
    if (rc) return rc;
    RC(partition_all(c, nreduce));
    u64 off = 0;
    for (u32 q = 0; q < r; q++) off += c->part_bytes[q];
    const u64 len = c->part_bytes[r];
    if (nbytes) *nbytes = len;
    if (host_out) {
        if (cap < len) { c->err = "wcg_partition: buffer too small"; return WCG_EINVAL; }
        if (len) {
            HIPCHK(c, hipMemcpyAsync(host_out, c->d_part + off, len, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
        }
    }
    return WCG_OK;
}

int wcg_export_count(wcg_ctx* c, uint32_t nreduce, uint32_t nranks, uint64_t* counts) {
    if (!c || !counts || nreduce == 0 || nranks == 0 || nranks > EX_MAX_RANKS) return WCG_EINVAL;
    RC(resolve(c));
    if (c->merged) { c->err = "wcg_export after wcg_merge_runs"; return WCG_ESTATE; }
    int rc = set_dev(c);
    if (rc) return rc;
    RC(compact(c));
    const u64 n = c->nrec;
    RC(ensure(c, &c->owner, &c->owner_cap, n + 1));
    HIPCHK(c, hipMemsetAsync(c->d_per_rank, 0, EX_MAX_RANKS * sizeof(u64), c->stream));
    if (n) {
        k_export_count<<<(unsigned)cdiv(n, EX_TILE), EX_NT, 0, c->stream>>>(c->crec, n, nreduce, nranks, c->arena,
                                                                            c->owner, c->d_per_rank);
        HIPCHK(c, hipGetLastError());
    }
    HIPCHK(c, hipMemcpyAsync(counts, c->d_per_rank, nranks * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    u64 tot = 0;
    for (u32 i = 0; i < nranks; i++) { c->h_cur[i] = tot; tot += counts[i]; }
    c->exp_total = tot;
    c->exp_nranks = nranks;
    c->exp_ready = true;
    return WCG_OK;
}

int wcg_export_write(wcg_ctx* c, void* dev_dst) {
    if (!c) return WCG_EINVAL;
    if (!c->exp_ready || !c->compacted) { c->err = "wcg_export_write without wcg_export_count"; return WCG_ESTATE; }
    int rc = set_dev(c);
    if (rc) return rc;
    const u64 n = c->nrec;
    if (n && !dev_dst) return WCG_EINVAL;
    if (n) {
        HIPCHK(c, hipMemcpyAsync(c->d_per_rank + EX_MAX_RANKS, c->h_cur, c->exp_nranks * sizeof(u64),
                                 hipMemcpyHostToDevice, c->stream));
        k_export_write<<<(unsigned)cdiv(n, EX_TILE), EX_NT, 0, c->stream>>>(
            c->crec, n, c->exp_nranks, c->owner, c->d_per_rank + EX_MAX_RANKS, c->arena, (Rec*)dev_dst);
        HIPCHK(c, hipGetLastError());
    }
    c->exp_ready = false;          // the cursors were consumed (the pinned copy is in flight)
    return WCG_OK;
}

int wcg_export(wcg_ctx* c, uint32_t nreduce, uint32_t nranks, const void** dev_records, uint64_t* counts) {
    if (!c || !counts) return WCG_EINVAL;
    RC(wcg_export_count(c, nreduce, nranks, counts));
    RC(ensure(c, &c->exp_buf, &c->exp_cap, c->exp_total + 1));
    RC(wcg_export_write(c, c->exp_buf));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (dev_records) *dev_records = c->exp_buf;
    return WCG_OK;
}

int wcg_import(wcg_ctx* c, const void* dev_records, uint64_t nrecords) {
    if (!c) return WCG_EINVAL;
    c->pending = false;
    if (nrecords == 0) return WCG_OK;
    if (!dev_records) return WCG_EINVAL;
    int rc = set_dev(c);
    if (rc) return rc;
    k_import<<<grid_for(nrecords, 256, c->ncu * 8), 256, 0, c->stream>>>((const Rec*)dev_records, nrecords, c->gtab,
                                                                          c->gslots - 1, c->ltab, c->lslots - 1,
                                                                          c->arena, c->arena_cap, c->st);
    HIPCHK(c, hipGetLastError());
    c->imported = true;
    c->compacted = c->reduced = c->merged = false;
    c->exp_ready = false;
    c->part_R = 0;
    return WCG_OK;          // a full table is reported by the next wcg_reduce / wcg_export_count
}

int wcg_merge_runs(wcg_ctx* c, const void* dev_text, const uint64_t* run_bytes, uint32_t nruns, uint64_t* nkeys,
                   uint64_t* nbytes) {
    if (!c || (nruns && !run_bytes)) return WCG_EINVAL;
    c->pending = false;
    int rc = set_dev(c);
    if (rc) return rc;
    u64 total = 0;
    for (u32 r = 0; r < nruns; r++) total += run_bytes[r];
    c->compacted = false;
    c->exp_ready = false;
    c->part_R = 0;
    c->reduced = false;
    if (total == 0) {
        c->nrec = 0; c->nkeys = 0; c->out_len = 0; c->reduced = true; c->merged = true;
        if (nkeys) *nkeys = 0;
        if (nbytes) *nbytes = 0;
        return WCG_OK;
    }
    if (!dev_text) return WCG_EINVAL;
    const uint8_t* text = (const uint8_t*)dev_text;
    const u64 nb = cdiv(total, NL_BLK);
    RC(ensure(c, &c->lens, &c->lens_cap, nb + 1));
    HIPCHK(c, hipMemsetAsync(&c->st->bad_input, 0, sizeof(u32), c->stream));
    k_nl_count<<<(unsigned)nb, NL_NT, 0, c->stream>>>(text, total, c->lens);
    k_scan_u64<<<1, 1024, 0, c->stream>>>(c->lens, nb, c->d_scalar);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(c->h_scalar, c->d_scalar, sizeof(u64), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const u64 L = *c->h_scalar;
    if (L == 0) { c->err = "wcg_merge_runs: no complete line"; return WCG_EINVAL; }
    RC(dbg(c, "merge_runs: line count"));
    RC(ensure(c, &c->nlpos, &c->nlpos_cap, L));
    RC(ensure_recs(c, L));
    k_nl_recs<<<(unsigned)nb, NL_NT, 0, c->stream>>>(text, total, c->lens, c->nlpos);
    k_line_recs<<<grid_for(L, 256, c->ncu * 8), 256, 0, c->stream>>>(text, c->nlpos, L, c->recA, c->st);
    RC(dbg(c, "merge_runs: line records"));
    // run boundaries in line records
    if (c->h_rb_cap < nruns + 1) {
        if (c->h_rb) HIPCHK(c, hipHostFree(c->h_rb));
        HIPCHK(c, hipHostMalloc(&c->h_rb, (nruns + 1) * sizeof(u64), hipHostMallocDefault));
        c->h_rb_cap = nruns + 1;
    }
    RC(ensure(c, &c->d_rb, &c->rb_cap, nruns + 1));
    RC(ensure(c, &c->d_b0, &c->b0_cap, nruns + 1));
    u64 acc = 0;
    for (u32 r = 0; r <= nruns; r++) { c->h_rb[r] = acc; if (r < nruns) acc += run_bytes[r]; }
    HIPCHK(c, hipMemcpyAsync(c->d_rb, c->h_rb, (nruns + 1) * sizeof(u64), hipMemcpyHostToDevice, c->stream));
    k_run_bounds<<<(unsigned)cdiv(nruns + 1, 256), 256, 0, c->stream>>>(c->nlpos, L, c->d_rb, nruns, c->d_b0);
    HIPCHK(c, hipGetLastError());
    RC(dbg(c, "merge_runs: run bounds"));
    Rec *src = c->recA, *dst = c->recB;
    for (u32 s = 1; s < nruns; s *= 2) {
        k_merge_runs<<<(unsigned)cdiv(L, MG_CHUNK), MG_NT, 0, c->stream>>>(src, dst, c->d_b0, nruns, s);
        HIPCHK(c, hipGetLastError());
        std::swap(src, dst);
        RC(dbg(c, "merge_runs: merge pass"));
    }
    c->sorted = src;
    c->nrec = L;
    c->nkeys = L;
    RC(fix_ties(c, src, L, text, dst));
    RC(dbg(c, "merge_runs: ties"));
    RC(format(c, src, L, text, FMT_COPY, 1, 0, total, &c->d_out, &c->out_cap, &c->out_len));
    HIPCHK(c, hipMemcpyAsync(c->h_st, c->st, sizeof(DevState), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->h_st->bad_input) { c->err = "wcg_merge_runs: a line is not \"key: count\""; return WCG_EINVAL; }
    c->reduced = true;
    c->merged = true;
    if (nkeys) *nkeys = L;
    if (nbytes) *nbytes = c->out_len;
    return WCG_OK;
}

int wcg_map_json(wcg_ctx* c, const uint8_t* host_bytes, uint64_t n, uint32_t nreduce, uint8_t* host_out, uint64_t cap,
                 uint64_t* part_bytes) {
    if (!c || nreduce == 0 || (n && !host_bytes)) return WCG_EINVAL;
    int rc = set_dev(c);
    if (rc) return rc;
    c->jparts.assign(nreduce, 0);
    if (n) {
        RC(ensure(c, &c->d_jin, &c->jin_cap, n + 64));
        HIPCHK(c, hipMemcpyAsync(c->d_jin, host_bytes, n, hipMemcpyHostToDevice, c->stream));
        const u64 W = cdiv(n, (u64)JS_NT * JS_SUB);
        const u64 m = (u64)nreduce * W;
        RC(ensure(c, &c->jhist, &c->jhist_cap, m + 1));
        k_json_count<<<(unsigned)W, JS_NT, 0, c->stream>>>(c->d_jin, n, nreduce, c->jhist);
        k_scan_u64<<<1, 1024, 0, c->stream>>>(c->jhist, m, c->jhist + m);
        HIPCHK(c, hipGetLastError());
        std::vector<u64> off(m + 1);
        HIPCHK(c, hipMemcpyAsync(off.data(), c->jhist, (m + 1) * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        for (u32 r = 0; r < nreduce; r++) c->jparts[r] = off[(u64)(r + 1) * W] - off[(u64)r * W];
        const u64 total = off[m];
        if (total) {
            RC(ensure(c, &c->d_jout, &c->jout_cap, total + 64));
            k_json_write<<<(unsigned)W, JS_NT, 0, c->stream>>>(c->d_jin, n, nreduce, c->jhist, c->d_jout);
            HIPCHK(c, hipGetLastError());
        }
        if (host_out) {
            if (cap < total) { c->err = "wcg_map_json: buffer too small"; return WCG_EINVAL; }
            if (total) HIPCHK(c, hipMemcpyAsync(host_out, c->d_jout, total, hipMemcpyDeviceToHost, c->stream));
        }
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    if (part_bytes) for (u32 r = 0; r < nreduce; r++) part_bytes[r] = c->jparts[r];
    return WCG_OK;
}

// ---------------------------------------------------------------- RCCL shuffle and Merge
#define NCCLCHK(ctx, call)                                                                  \
    do {                                                                                    \
        ncclResult_t r_ = (call);                                                           \
        if (r_ != ncclSuccess) {                                                            \
            (ctx)->err = std::string(#call) + ": " + ncclGetErrorString(r_);                \
            return WCG_EHIP;                                                                \
        }                                                                                   \
    } while (0)

}  // extern "C"

namespace {

// The plan of one rank's part of the shuffle, from the count matrix every rank holds after the
// count all-gather: m[s * stride + d] = units rank s sends to rank d.  Send side: this rank's
// units for d sit at soff[d] of its send buffer (k_export_write's cursors start there); receive
// side: the units from s land at roff[s], in source-rank order.  Pure host arithmetic, shared by
// wcg_exchange, wcg_exchange_local and wcg_exchange_plan (the CPU tests).
template <typename T>
void plan_exchange(const T* m, u64 stride, u32 W, u32 me, T* soff, T* scnt, T* roff, T* rcnt, T* ts, T* tr) {
    u64 a = 0, b = 0;
    for (u32 d = 0; d < W; d++) {
        const u64 s = m[(u64)me * stride + d];
        if (soff) soff[d] = a;
        if (scnt) scnt[d] = s;
        a += s;
    }
    for (u32 s = 0; s < W; s++) {
        const u64 r = m[(u64)s * stride + me];
        if (roff) roff[s] = b;
        if (rcnt) rcnt[s] = r;
        b += r;
    }
    if (ts) *ts = a;
    if (tr) *tr = b;
}

// Merge's gather: rank p's run lands at off[p] of root's receive buffer (root's own run too: it
// is copied there, so the runs are back to back in rank order for wcg_merge_runs).
template <typename T>
void plan_gather(const T* sizes, u64 stride, u32 W, T* off, T* total) {
    u64 a = 0;
    for (u32 p = 0; p < W; p++) {
        if (off) off[p] = a;
        a += sizes[(u64)p * stride];
    }
    if (total) *total = a;
}

// Host and device buffers of the exchange for a world of W: a row per rank ([status, caps...,
// units per owner]), the gathered matrix, the pinned copies and the export cursors.
constexpr u64 X_HDR = 3;                  // row header: status, then two capacities
int x_buffers(wcg_ctx* c, u32 W) {
    if (c->x_world >= W && c->d_xrow) return WCG_OK;
    if (c->d_xrow) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipFree(c->d_xrow));
        HIPCHK(c, hipHostFree(c->h_x));
        c->d_xrow = nullptr; c->h_x = nullptr; c->x_world = 0;
    }
    const u64 S = W + X_HDR;
    // device: row (S), status word (1), matrix (W x S); pinned: row header + status (4), send
    // offsets (W), matrix (W x S)
    HIPCHK(c, hipMalloc(&c->d_xrow, (S + 1 + (u64)W * S) * sizeof(u64)));
    HIPCHK(c, hipHostMalloc(&c->h_x, (4 + W + (u64)W * S) * sizeof(u64), hipHostMallocDefault));
    c->x_world = W;
    return WCG_OK;
}
u64* x_dstat(wcg_ctx* c) { return c->d_xrow + c->x_world + X_HDR; }
u64* x_dmat(wcg_ctx* c) { return c->d_xrow + c->x_world + X_HDR + 1; }
u64* x_hsoff(wcg_ctx* c) { return c->h_x + 4; }
u64* x_hmat(wcg_ctx* c) { return c->h_x + 4 + c->x_world; }

// Shuffle, local part before any collective: compaction and this rank's units per owner rank
// into per_rank[0..W) on the device (the caller cleared it)
int x_count(wcg_ctx* c, u32 nreduce, u32 W, u64* per_rank) {
    RC(compact(c));
    const u64 n = c->nrec;
    RC(ensure(c, &c->owner, &c->owner_cap, n + 1));
    if (n) {
        k_export_count<<<(unsigned)cdiv(n, EX_TILE), EX_NT, 0, c->stream>>>(c->crec, n, nreduce, W, c->arena,
                                                                            c->owner, per_rank);
        HIPCHK(c, hipGetLastError());
    }
    return WCG_OK;
}

// the send buffer (ts units) and the receive buffer (tr units)
int x_alloc(wcg_ctx* c, u64 ts, u64 tr) {
    RC(ensure(c, &c->exp_buf, &c->exp_cap, ts + 1));
    RC(ensure(c, &c->xrecv, &c->xrecv_cap, tr + 1));
    return WCG_OK;
}

// the units into the send buffer, owner d's at soff[d] (soff: pinned, c->h_x)
int x_write(wcg_ctx* c, u32 W, const u64* soff) {
    if (!c->nrec) return WCG_OK;
    HIPCHK(c, hipMemcpyAsync(c->d_per_rank + EX_MAX_RANKS, soff, W * sizeof(u64), hipMemcpyHostToDevice, c->stream));
    k_export_write<<<(unsigned)cdiv(c->nrec, EX_TILE), EX_NT, 0, c->stream>>>(
        c->crec, c->nrec, W, c->owner, c->d_per_rank + EX_MAX_RANKS, c->arena, c->exp_buf);
    HIPCHK(c, hipGetLastError());
    return WCG_OK;
}

// this rank now keeps exactly its own partitions: tables cleared, the tr received units imported
int x_import(wcg_ctx* c, u64 tr) {
    RC(reset_tables(c));
    if (tr) {
        k_import<<<grid_for(tr, 256, c->ncu * 8), 256, 0, c->stream>>>(c->xrecv, tr, c->gtab, c->gslots - 1, c->ltab,
                                                                      c->lslots - 1, c->arena, c->arena_cap, c->st);
        HIPCHK(c, hipGetLastError());
        c->imported = true;
    }
    return WCG_OK;
}

// Every rank's status went around with its row (column 0 of the gathered matrix): a rank that
// failed locally has joined the collective anyway, so all ranks see the failure and return it
// instead of waiting in a send or receive that will not come.
int x_statuses(wcg_ctx* c, const u64* m, u64 stride, u32 W, int mine, const char* what) {
    if (mine) return mine;                    // c->err already says why
    for (u32 p = 0; p < W; p++) {
        const u64 s = m[(u64)p * stride];
        if (s) {
            char buf[160];
            snprintf(buf, sizeof buf, "%s: rank %u failed (status %llu); no data was exchanged", what, p,
                     (unsigned long long)s);
            c->err = buf;
            return (int)s;
        }
    }
    return WCG_OK;
}

// After buffers were grown on some ranks (every rank knows whether any did: the capacities came
// with the rows): one all-reduce(max) of the allocation status before any data moves.
int x_agree(wcg_ctx* c, int mine, const char* what) {
    c->h_x[3] = (u64)mine;
    HIPCHK(c, hipMemcpyAsync(x_dstat(c), c->h_x + 3, sizeof(u64), hipMemcpyHostToDevice, c->stream));
    NCCLCHK(c, ncclAllReduce(x_dstat(c), x_dstat(c), 1, ncclUint64, ncclMax, c->comm, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->h_x + 3, x_dstat(c), sizeof(u64), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (mine) return mine;
    if (c->h_x[3]) {
        c->err = std::string(what) + ": a peer rank could not allocate its buffers; no data was exchanged";
        return (int)c->h_x[3];
    }
    return WCG_OK;
}

}  // namespace

extern "C" {

int wcg_exchange_plan(const uint64_t* counts, uint32_t world, uint32_t rank, uint64_t* send_off, uint64_t* send_cnt,
                      uint64_t* recv_off, uint64_t* recv_cnt, uint64_t* totals) {
    if (!counts || world == 0 || world > EX_MAX_RANKS || rank >= world) return WCG_EINVAL;
    uint64_t ts = 0, tr = 0;
    plan_exchange(counts, world, world, rank, send_off, send_cnt, recv_off, recv_cnt, &ts, &tr);
    if (totals) { totals[0] = ts; totals[1] = tr; }
    return WCG_OK;
}

int wcg_gather_plan(const uint64_t* sizes, uint32_t world, uint32_t root, uint64_t* run_off, uint64_t* total) {
    if (!sizes || world == 0 || world > EX_MAX_RANKS || root >= world) return WCG_EINVAL;
    plan_gather(sizes, 1, world, run_off, total);
    return WCG_OK;
}

int wcg_comm_id(uint8_t* id_out) {
    if (!id_out) return WCG_EINVAL;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return WCG_EHIP;
    static_assert(sizeof(u.internal) == WCG_COMM_ID_BYTES, "ncclUniqueId size");
    memcpy(id_out, u.internal, WCG_COMM_ID_BYTES);
    return WCG_OK;
}

int wcg_comm_init(wcg_ctx* c, const uint8_t* id, int rank, int world) {
    if (!c) return WCG_EINVAL;
    if (!id || world < 1 || (u32)world > EX_MAX_RANKS || rank < 0 || rank >= world) {
        c->err = "wcg_comm_init: bad rank / world";
        return WCG_EINVAL;
    }
    int rc = set_dev(c);
    if (rc) return rc;
    if (c->comm) { (void)ncclCommDestroy(c->comm); c->comm = nullptr; }
    RC(x_buffers(c, (u32)world));
    ncclUniqueId u;
    memcpy(u.internal, id, WCG_COMM_ID_BYTES);
    NCCLCHK(c, ncclCommInitRank(&c->comm, world, u, rank));
    c->comm_rank = rank;
    c->comm_world = world;
    return WCG_OK;
}

// The shuffle of mapreduce.go:214-230 / 242-263 between the GPUs of one job: every rank's
// aggregate leaves as 32-byte units bucketed by owner rank and the owner imports what it
// receives.  Stream order: compaction -> k_export_count (into this rank's row) ->
// ncclAllGather(rows: status, buffer capacities, units per owner) -> [the one host read: the
// W x W count matrix] -> plan (plan_exchange) -> k_export_write into the send buffer -> grouped
// ncclSend/ncclRecv -> table clear -> k_import.  A rank that fails before the all-gather (a full
// table, a bad argument) joins it with its status, and every rank returns that error.
int wcg_exchange(wcg_ctx* c, uint32_t nreduce, uint64_t* sent, uint64_t* received) {
    if (!c) return WCG_EINVAL;
    if (!c->comm) { c->err = "wcg_exchange before wcg_comm_init"; return WCG_ESTATE; }
    int rc = set_dev(c);
    if (rc) return rc;
    const u32 W = (u32)c->comm_world, me = (u32)c->comm_rank;
    const u64 S = W + X_HDR;
    hipEvent_t e0 = mark(c);
    int mine = resolve(c);              // (a failed wcg_reduce_async job still joins the collectives)
    if (mine) {}
    else if (nreduce == 0) { c->err = "wcg_exchange: nreduce 0"; mine = WCG_EINVAL; }
    else if (c->merged) { c->err = "wcg_exchange after wcg_merge_runs"; mine = WCG_ESTATE; }
    HIPCHK(c, hipMemsetAsync(c->d_xrow + X_HDR, 0, W * sizeof(u64), c->stream));
    if (!mine) mine = x_count(c, nreduce, W, c->d_xrow + X_HDR);
    u64* hdr = c->h_x;
    hdr[0] = (u64)mine; hdr[1] = c->exp_buf ? c->exp_cap : 0; hdr[2] = c->xrecv ? c->xrecv_cap : 0;
    HIPCHK(c, hipMemcpyAsync(c->d_xrow, hdr, X_HDR * sizeof(u64), hipMemcpyHostToDevice, c->stream));
    NCCLCHK(c, ncclAllGather(c->d_xrow, x_dmat(c), S, ncclUint64, c->comm, c->stream));
    u64* m = x_hmat(c);
    HIPCHK(c, hipMemcpyAsync(m, x_dmat(c), (u64)W * S * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));     // the one host read of the exchange
    RC(x_statuses(c, m, S, W, mine, "wcg_exchange"));
    std::vector<u64> scnt(W), roff(W), rcnt(W);
    u64* soff = x_hsoff(c);
    u64 ts = 0, tr = 0;
    plan_exchange<u64>(m + X_HDR, S, W, me, soff, scnt.data(), roff.data(), rcnt.data(), &ts, &tr);
    // does any rank grow a buffer?  (all ranks decide alike: the capacities came with the rows)
    bool grow = false;
    for (u32 p = 0; p < W && !grow; p++) {
        u64 tsp = 0, trp = 0;
        plan_exchange<u64>(m + X_HDR, S, W, p, nullptr, nullptr, nullptr, nullptr, &tsp, &trp);
        grow = tsp + 1 > m[(u64)p * S + 1] || trp + 1 > m[(u64)p * S + 2];
    }
    const int arc = x_alloc(c, ts, tr);
    if (grow) RC(x_agree(c, arc, "wcg_exchange"));
    else RC(arc);
    RC(x_write(c, W, soff));
    hipEvent_t e1 = mark(c);
    NCCLCHK(c, ncclGroupStart());
    for (u32 p = 0; p < W; p++) {
        if (scnt[p])
            NCCLCHK(c, ncclSend(c->exp_buf + soff[p], scnt[p] * sizeof(Rec), ncclUint8, (int)p, c->comm, c->stream));
        if (rcnt[p])
            NCCLCHK(c, ncclRecv(c->xrecv + roff[p], rcnt[p] * sizeof(Rec), ncclUint8, (int)p, c->comm, c->stream));
    }
    NCCLCHK(c, ncclGroupEnd());
    hipEvent_t e2 = mark(c);
    RC(x_import(c, tr));
    hipEvent_t e3 = mark(c);
    record_x(c, 5, e0, e1);
    record_x(c, 6, e1, e2);
    record_x(c, 7, e2, e3);
    if (sent) *sent = ts;
    if (received) *received = tr;
    return WCG_OK;
}

// Merge (mapreduce.go:284-321) across the ranks: the owners' sorted runs (disjoint key sets)
// travel to root, which merges them without a re-sort (wcg_merge_runs).  Rows of the all-gather:
// {status, run bytes, root's receive capacity}.
int wcg_gather_merge(wcg_ctx* c, int root, uint64_t* nkeys, uint64_t* nbytes) {
    if (!c) return WCG_EINVAL;
    if (!c->comm) { c->err = "wcg_gather_merge before wcg_comm_init"; return WCG_ESTATE; }
    if (root < 0 || root >= c->comm_world) { c->err = "wcg_gather_merge: bad root"; return WCG_EINVAL; }
    int rc = set_dev(c);
    if (rc) return rc;
    const u32 W = (u32)c->comm_world;
    const bool am_root = c->comm_rank == root;
    const u64 S = 3;
    hipEvent_t e0 = mark(c);
    int mine = resolve(c);
    if (!mine && (!c->reduced || c->merged)) { c->err = "wcg_gather_merge needs a wcg_reduce result"; mine = WCG_ESTATE; }
    u64* hdr = c->h_x;
    hdr[0] = (u64)mine; hdr[1] = mine ? 0 : c->out_len; hdr[2] = c->grecv ? c->grecv_cap : 0;
    HIPCHK(c, hipMemcpyAsync(c->d_xrow, hdr, S * sizeof(u64), hipMemcpyHostToDevice, c->stream));
    NCCLCHK(c, ncclAllGather(c->d_xrow, x_dmat(c), S, ncclUint64, c->comm, c->stream));
    u64* m = x_hmat(c);
    HIPCHK(c, hipMemcpyAsync(m, x_dmat(c), (u64)W * S * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));     // the run sizes (one host read)
    RC(x_statuses(c, m, S, W, mine, "wcg_gather_merge"));
    std::vector<uint64_t> sizes(W);
    std::vector<u64> off(W);
    for (u32 p = 0; p < W; p++) sizes[p] = m[(u64)p * S + 1];
    u64 total = 0;
    plan_gather<u64>(m + 1, S, W, off.data(), &total);
    const bool grow = total + 64 > m[(u64)root * S + 2];
    const int arc = am_root ? ensure(c, &c->grecv, &c->grecv_cap, total + 64) : WCG_OK;
    if (grow) RC(x_agree(c, arc, "wcg_gather_merge"));
    else RC(arc);
    if (!am_root) {
        if (c->out_len)
            NCCLCHK(c, ncclSend(c->d_out, c->out_len, ncclUint8, root, c->comm, c->stream));
        hipEvent_t e1 = mark(c);
        record_x(c, 8, e0, e1);
        if (nkeys) *nkeys = 0;
        if (nbytes) *nbytes = 0;
        return WCG_OK;
    }
    NCCLCHK(c, ncclGroupStart());
    for (u32 p = 0; p < W; p++)
        if (sizes[p] && (int)p != root)
            NCCLCHK(c, ncclRecv(c->grecv + off[p], sizes[p], ncclUint8, (int)p, c->comm, c->stream));
    NCCLCHK(c, ncclGroupEnd());
    if (sizes[root])
        HIPCHK(c, hipMemcpyAsync(c->grecv + off[root], c->d_out, sizes[root], hipMemcpyDeviceToDevice, c->stream));
    hipEvent_t e1 = mark(c);
    RC(wcg_merge_runs(c, c->grecv, sizes.data(), W, nkeys, nbytes));
    hipEvent_t e2 = mark(c);
    record_x(c, 8, e0, e1);
    record_x(c, 9, e1, e2);
    return WCG_OK;
}

// ---- the same shuffle and Merge across the contexts of one process (a test transport): every
// step but the transport is the code above - the count matrix, plan_exchange / plan_gather, the
// export, import and merge kernels; device copies stand in for ncclSend / ncclRecv.
int wcg_exchange_local(wcg_ctx** cs, uint32_t W, uint32_t nreduce, uint64_t* sent, uint64_t* received) {
    if (!cs || W == 0 || W > EX_MAX_RANKS || nreduce == 0) return WCG_EINVAL;
    for (u32 p = 0; p < W; p++) {
        if (!cs[p]) return WCG_EINVAL;
        for (u32 q = 0; q < p; q++) if (cs[q] == cs[p]) return WCG_EINVAL;
    }
    // every context's status and counts first, as wcg_exchange's all-gather carries them: a
    // context that fails locally (a full table, a failed wcg_reduce_async job, a call out of order)
    // fails the exchange on every context, with no data moved and every table untouched
    std::vector<u64> m((u64)W * W);
    std::vector<u64> status(W, 0);
    for (u32 p = 0; p < W; p++) {
        wcg_ctx* c = cs[p];
        status[p] = (u64)[&]() -> int {
            RC(resolve(c));
            if (c->merged) { c->err = "wcg_exchange_local after wcg_merge_runs"; return WCG_ESTATE; }
            RC(set_dev(c));
            RC(x_buffers(c, W));
            HIPCHK(c, hipMemsetAsync(c->d_xrow + X_HDR, 0, W * sizeof(u64), c->stream));
            RC(x_count(c, nreduce, W, c->d_xrow + X_HDR));
            HIPCHK(c, hipMemcpyAsync(x_hmat(c), c->d_xrow + X_HDR, W * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            std::copy(x_hmat(c), x_hmat(c) + W, m.begin() + (u64)p * W);
            return WCG_OK;
        }();
    }
    for (u32 p = 0; p < W; p++) {
        if (!status[p]) continue;
        for (u32 q = 0; q < W; q++)
            if (!status[q]) (void)x_statuses(cs[q], status.data(), 1, W, WCG_OK, "wcg_exchange_local");
        return (int)status[p];
    }
    std::vector<u64> roff((u64)W * W), ts(W), tr(W);
    for (u32 p = 0; p < W; p++) {
        wcg_ctx* c = cs[p];
        RC(set_dev(c));
        plan_exchange<u64>(m.data(), W, W, p, x_hsoff(c), nullptr, roff.data() + (u64)p * W, nullptr, &ts[p], &tr[p]);
        RC(x_alloc(c, ts[p], tr[p]));
        RC(x_write(c, W, x_hsoff(c)));
    }
    for (u32 p = 0; p < W; p++) { RC(set_dev(cs[p])); HIPCHK(cs[p], hipStreamSynchronize(cs[p]->stream)); }
    for (u32 d = 0; d < W; d++) {
        wcg_ctx* c = cs[d];
        RC(set_dev(c));
        for (u32 s = 0; s < W; s++) {
            const u64 n = m[(u64)s * W + d];
            if (n)
                HIPCHK(c, hipMemcpyAsync(c->xrecv + roff[(u64)d * W + s], cs[s]->exp_buf + x_hsoff(cs[s])[d],
                                         n * sizeof(Rec), hipMemcpyDeviceToDevice, c->stream));
        }
        RC(x_import(c, tr[d]));
    }
    for (u32 p = 0; p < W; p++) {
        RC(set_dev(cs[p]));
        HIPCHK(cs[p], hipStreamSynchronize(cs[p]->stream));   // the send buffers are free again
        if (sent) sent[p] = ts[p];
        if (received) received[p] = tr[p];
    }
    return WCG_OK;
}

int wcg_gather_merge_local(wcg_ctx** cs, uint32_t W, uint32_t root, uint64_t* nkeys, uint64_t* nbytes) {
    if (!cs || W == 0 || W > EX_MAX_RANKS || root >= W) return WCG_EINVAL;
    std::vector<uint64_t> sizes(W), off(W);
    for (u32 p = 0; p < W; p++) {
        if (!cs[p]) return WCG_EINVAL;
        RC(resolve(cs[p]));
        if (!cs[p]->reduced || cs[p]->merged) { cs[p]->err = "wcg_gather_merge_local needs a wcg_reduce result"; return WCG_ESTATE; }
        sizes[p] = cs[p]->out_len;
    }
    uint64_t total = 0;
    plan_gather(sizes.data(), 1, W, off.data(), &total);
    wcg_ctx* r = cs[root];
    RC(set_dev(r));
    RC(ensure(r, &r->grecv, &r->grecv_cap, total + 64));
    for (u32 p = 0; p < W; p++) {
        RC(set_dev(cs[p]));
        HIPCHK(cs[p], hipStreamSynchronize(cs[p]->stream));
    }
    RC(set_dev(r));
    for (u32 p = 0; p < W; p++)
        if (sizes[p])
            HIPCHK(r, hipMemcpyAsync(r->grecv + off[p], cs[p]->d_out, sizes[p], hipMemcpyDeviceToDevice, r->stream));
    return wcg_merge_runs(r, r->grecv, sizes.data(), W, nkeys, nbytes);
}

int wcg_timings(wcg_ctx* c, double* ms, int n, uint64_t* map_launches) {
    if (!c || !ms || n < 0) return WCG_EINVAL;
    RC(resolve(c));
    int rc = set_dev(c);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    double v[10] = {};
    if (c->timing_mode >= 2) {          // summed over every job of the epoch (folded ones too)
        for (int i = 0; i < 10; i++) v[i] = c->acc[i];
        sum_events(c, v);
    } else {
        for (auto& p : c->map_ev) v[0] += ev_ms(p.first, p.second);
        for (auto& p : c->agg_ev) v[1] += ev_ms(p.first, p.second);
        if (c->phase_rec) {
            v[2] = ev_ms(c->phase_ev[0], c->phase_ev[1]);
            v[3] = ev_ms(c->phase_ev[2], c->phase_ev[3]);
            v[4] = ev_ms(c->phase_ev[3], c->phase_ev[4]);
        }
        for (auto& x : c->xev) v[std::get<0>(x)] += ev_ms(std::get<1>(x), std::get<2>(x));
    }
    for (int i = 0; i < n && i < 10; i++) ms[i] = v[i];
    if (map_launches) *map_launches = c->map_launches;
    return WCG_OK;
}

int wcg_reduce_path(const wcg_ctx* c, int* path) {
    if (!c || !path) return WCG_EINVAL;
    *path = c->fused_last ? 1 : 0;
    return WCG_OK;
}

int wcg_stats(wcg_ctx* c, uint64_t* s8) {   // 9 values (include/wcg.h)
    if (!c || !s8) return WCG_EINVAL;
    RC(resolve(c));
    int rc = set_dev(c);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(c->h_st, c->st, sizeof(DevState), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    s8[0] = c->h_st->tokens; s8[1] = c->reduced ? c->nkeys : c->nrec; s8[2] = c->h_st->lds_hits; s8[3] = c->h_st->global_ops;
    s8[4] = c->h_st->long_tokens; s8[5] = c->h_st->arena_top; s8[6] = c->h_st->overflow; s8[7] = c->h_st->spin_fail;
    s8[8] = c->h_st->nemit;
    return WCG_OK;
}

}  // extern "C"
