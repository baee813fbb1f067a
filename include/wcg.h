/*
 * wcg.h - C ABI of the MI355X word-count engine (libwcg.so).
 *
 * This is the drop-in boundary for the Lab 1 MapReduce word-count hot path of
 * wushan270/mit-6.824-2015.  The reference's "plugin API" is a pair of Go function values,
 *   Map    func(string) *list.List              (/root/reference/src/main/wc.go:17)
 *   Reduce func(string, *list.List) string      (/root/reference/src/main/wc.go:35)
 * run by the data plane of package mapreduce
 *   RunSingle  mapreduce.go:344-356   Split 141-179   DoMap 193-231   ihash 185-189
 *   DoReduce   mapreduce.go:239-280   Merge 284-321   MapName/ReduceName/MergeName 136,181,233
 * and by the worker RPC handler Worker.DoJob (worker.go:22-34).
 *
 * A GPU backend must implement Map AND Reduce together (the device pre-aggregates
 * (key, count) pairs, which the per-occurrence CPU Reduce = len(list) could not consume),
 * so the ABI is phase-shaped - one C call per phase, never one per token:
 *
 *   wcg_open     ~ InitMapReduce for a wc job on one GPU            (mapreduce.go:68-82)
 *   wcg_map*     ~ DoMap(job) + Map over one split's bytes           (mapreduce.go:193-231)
 *   wcg_reduce   ~ all DoReduce jobs + Merge: sorted "key: count\n"  (mapreduce.go:239-321)
 *   wcg_partition~ DoReduce(job=r) output bytes mrtmp.<f>-res-<r>    (mapreduce.go:264-279)
 *   wcg_export / wcg_import ~ the ihash%nReduce shuffle (mapreduce.go:214-230 + 242-263),
 *                  done as an all-to-all-v of pre-aggregated records between GPUs.
 *   wcg_map_file ~ Split + DoMap x nMap from the input file (mapreduce.go:141-179, 193-231)
 *   wcg_merge_runs ~ Merge of the owners' sorted DoReduce outputs  (mapreduce.go:284-321)
 *   wcg_map_json ~ DoMap's per-occurrence JSON intermediates       (mapreduce.go:214-230)
 *
 * Conventions:
 *   - Every entry point returns int status (WCG_OK = 0); the host turns non-zero into a fatal
 *     error exactly where the reference calls log.Fatal.  wcg_last_error() explains it.
 *   - Output buffers are library-owned (valid until the next call on the same context).
 *   - The library never retains caller pointers past a call.
 *   - Every entry point makes the context's device current (the HIP current device is
 *     per host thread; Go goroutines migrate between threads).
 *   - A context is not thread-safe.
 */
#ifndef WCG_H
#define WCG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef WCG_API
#define WCG_API __attribute__((visibility("default")))
#endif

typedef struct wcg_ctx wcg_ctx;

enum {
    WCG_OK = 0,
    WCG_EINVAL = 1,   /* bad argument                                                */
    WCG_ENOMEM = 2,   /* device allocation failed                                    */
    WCG_EHIP = 3,     /* HIP runtime error                                           */
    WCG_EFULL = 4,    /* aggregation table overflowed (max_keys too small)           */
    WCG_ESTATE = 5    /* call out of order (e.g. wcg_partition before wcg_reduce)    */
};

enum {
    WCG_FMT_MERGED = 0,    /* "key: count\n", all keys, bytewise order  (Merge output)   */
    WCG_FMT_RES_JSON = 1   /* {"Key":"k","Value":"count"}\n for ihash(k)%R == r          */
};

/* Open a context on HIP device `device`.
 *   max_input_bytes: a hint (kept for ABI compatibility): wcg_map streams splits of any size
 *                    through fixed pinned staging buffers; 0 is fine
 *   max_keys:        capacity in distinct keys of the device aggregation table */
WCG_API int wcg_open(int device, uint64_t max_input_bytes, uint64_t max_keys, wcg_ctx **out);
WCG_API int wcg_close(wcg_ctx *ctx);
WCG_API const char *wcg_last_error(const wcg_ctx *ctx);

/* Run all device work of this context on `stream` (a hipStream_t; NULL = the context's own
 * stream).  Lets a host framework time the phases with its own events. */
WCG_API int wcg_set_stream(wcg_ctx *ctx, void *stream);

/* Forget all aggregated keys (start a new job). */
WCG_API int wcg_reset(wcg_ctx *ctx);

/* DoMap + Map (mapreduce.go:193-231, wc.go:17-30) over one split held in host memory:
 * copy to HBM, tokenize into maximal unicode.IsLetter runs, aggregate (key, count).
 * Splits must be cut where a token cannot straddle (Split cuts at '\n').  Large splits are
 * streamed in chunks (cut after an ASCII non-letter) through pinned double buffers, so the
 * copy of one chunk overlaps the map of the previous one.  Returns once host_bytes has been
 * consumed (the caller may free it); the device work is asynchronous. */
WCG_API int wcg_map(wcg_ctx *ctx, const uint8_t *host_bytes, uint64_t n);

/* Same, input already resident in device memory (n bytes at dev_bytes). Asynchronous. */
WCG_API int wcg_map_device(wcg_ctx *ctx, const void *dev_bytes, uint64_t n);

/* Split (mapreduce.go:141-179) + DoMap x nMap over a whole input file, on the GPU: the file is
 * read by a pool of host threads into two pinned staging buffers and copied to HBM in
 * line-aligned chunks, each copy overlapping the map kernels of the previous chunk.  Split's
 * quirk P1 is kept: the first line that does not fit bufio.Scanner's 64 KiB buffer together with
 * its '\n' ends the input (the reference's scan stops there silently).  *mapped_bytes = bytes
 * counted (the whole file unless P1 cut it), *file_bytes = file size.  Asynchronous. */
WCG_API int wcg_map_file(wcg_ctx *ctx, const char *path, uint64_t *mapped_bytes, uint64_t *file_bytes);

/* DoReduce x nReduce + Merge (mapreduce.go:239-321): sort all keys bytewise on the device and
 * format the merged file "key: count\n".  Synchronous; returns key count and byte size. */
WCG_API int wcg_reduce(wcg_ctx *ctx, uint64_t *nkeys, uint64_t *nbytes);

/* The same job without the host wait: the reduce is queued on the context's stream (with the
 * read-back of its sizes and error flags) and the call returns at once, so a host can queue the
 * next job's wcg_reset / wcg_map* behind it (back-to-back jobs then run without host gaps).
 * wcg_reduce_wait returns what wcg_reduce would have (sizes, or the job's error); every call that
 * reads the job's results (wcg_result_*, wcg_partition*, wcg_export*, wcg_stats, wcg_timings,
 * wcg_sync, the collectives) waits for it first.  A job not waited for before the next wcg_reset
 * / wcg_map* / wcg_import is dropped, its results and its error status with it.  Jobs that take
 * the multi-launch reduce (the first job of a context, large or two-pass jobs) are reduced
 * synchronously here as by wcg_reduce. */
WCG_API int wcg_reduce_async(wcg_ctx *ctx);
WCG_API int wcg_reduce_wait(wcg_ctx *ctx, uint64_t *nkeys, uint64_t *nbytes);

/* Device pointer to / host copy of the formatted output of the last wcg_reduce(). */
WCG_API int wcg_result_device(wcg_ctx *ctx, const void **dev_ptr, uint64_t *nbytes);
WCG_API int wcg_result_copy(wcg_ctx *ctx, uint8_t *host_out, uint64_t cap);
/* Device-to-device copy of that output (nbytes of wcg_reduce) into dev_dst, asynchronous on the
 * context's stream (e.g. into a collective's send buffer). */
WCG_API int wcg_result_copy_device(wcg_ctx *ctx, void *dev_dst);

/* Wait for all device work queued on the context's stream. */
WCG_API int wcg_sync(wcg_ctx *ctx);

/* Release a library-owned device buffer before the context is closed: the formatted output of
 * wcg_result_device() or the records of wcg_export() (output buffers are
 * library-owned until wcg_free).  Waits for the context's stream first.  Afterwards the result
 * calls report WCG_ESTATE until the next wcg_reduce(); a later call that needs the buffer
 * allocates it again.  Any other pointer: WCG_EINVAL. */
WCG_API int wcg_free(wcg_ctx *ctx, const void *dev_ptr);

/* Bytes of mrtmp.<f>-res-<r> (DoReduce output, mapreduce.go:264-279) for partition r of
 * nreduce, in sorted key order, copied to host_out (cap bytes).  *nbytes gets the size;
 * host_out == NULL queries the size only.  Requires a prior wcg_reduce(). */
WCG_API int wcg_partition(wcg_ctx *ctx, uint32_t nreduce, uint32_t r, uint8_t *host_out, uint64_t cap,
                  uint64_t *nbytes);

/* Every DoReduce output file at once: the nreduce -res-<r> files back to back in partition order
 * (one formatting pass for all of them; nreduce <= 1024).  part_bytes[nreduce] gets each file's
 * size; host_out == NULL queries the sizes only (the files stay cached on the device until the
 * next job, so wcg_partition of any r is then a copy). */
WCG_API int wcg_partition_all(wcg_ctx *ctx, uint32_t nreduce, uint8_t *host_out, uint64_t cap,
                              uint64_t *part_bytes);

/* DoMap's reference-exact intermediate files (mapreduce.go:214-230) for one split: for every
 * token, in input order, the line {"Key":"tok","Value":"1"}\n in file ihash(tok) % nreduce - the
 * bytes the reference's json.Encoder writes to mrtmp.<f>-<m>-<r>, so an unmodified CPU DoReduce
 * can consume GPU map output.  Files back to back in partition order; part_bytes[nreduce] gets
 * each size; host_out == NULL queries the sizes only.  Independent of the aggregation tables. */
WCG_API int wcg_map_json(wcg_ctx *ctx, const uint8_t *host_bytes, uint64_t n, uint32_t nreduce,
                         uint8_t *host_out, uint64_t cap, uint64_t *part_bytes);

/* ---- multi-GPU shuffle (one process per GPU; the host moves the buffers with RCCL) ----
 * wcg_export: bucket the local aggregate by owner = (ihash(key) % nreduce) % nranks into a
 * device buffer of fixed 32-byte records (long keys > 15 bytes are carried in following
 * 32-byte continuation records).  counts[nranks] receives records per destination, in order.
 * wcg_import: aggregate records received from peers into this context's table (call after
 * wcg_reset() on the receiving side, or onto a live table). */
#define WCG_RECORD_BYTES 32
WCG_API int wcg_export(wcg_ctx *ctx, uint32_t nreduce, uint32_t nranks, const void **dev_records,
               uint64_t *counts);
WCG_API int wcg_import(wcg_ctx *ctx, const void *dev_records, uint64_t nrecords);

/* The same export in two steps, writing straight into a caller's device buffer (e.g. the send
 * buffer of an RCCL all-to-all-v): wcg_export_count returns the units per destination rank
 * (one host synchronisation); wcg_export_write then fills dev_dst (sum(counts) units, rank
 * order) asynchronously on the context's stream.  wcg_import is asynchronous too: a table that
 * filled is reported by the next wcg_reduce / wcg_export_count. */
WCG_API int wcg_export_count(wcg_ctx *ctx, uint32_t nreduce, uint32_t nranks, uint64_t *counts);
WCG_API int wcg_export_write(wcg_ctx *ctx, void *dev_dst);

/* ---- the shuffle and the final Merge inside the library, over RCCL (one process per GPU) ----
 * The reference moves partitions between its phases as files: DoMap writes mrtmp.<f>-<m>-<r>
 * for r = ihash(key) % nReduce (mapreduce.go:214-230), DoReduce r reads partition r of every
 * map job (mapreduce.go:242-263), Merge reads every -res-<r> (mapreduce.go:284-321).  On one
 * node of GPUs these hand-offs are RCCL collectives over xGMI on the context's stream:
 *   wcg_comm_id      ncclGetUniqueId: made on rank 0, handed to every rank by the host (the
 *                    config-5 master RPC, torch.distributed, a file - 128 opaque bytes)
 *   wcg_comm_init    ncclCommInitRank for this context (world may be 1)
 *   wcg_exchange     export the local aggregate by owner = (ihash % nreduce) % world into a send
 *                    buffer, ncclAllGather every rank's row {status, buffer capacities, units per
 *                    owner}, ONE host read of that world x world matrix, the plan of
 *                    wcg_exchange_plan, grouped ncclSend/ncclRecv of the 32-byte units, then this
 *                    context keeps exactly the keys of the partitions it owns (tables cleared,
 *                    received units imported).  All device work is ordered on the context's
 *                    stream; *sent / *received = units (may be NULL).  Follow with wcg_reduce
 *                    (DoReduce of the owned partitions: sorted "key: count" run of this rank).
 *   wcg_gather_merge after wcg_reduce on every rank: every rank's sorted run goes to `root`
 *                    (ncclAllGather of {status, run size, capacity}, one host read,
 *                    ncclSend/ncclRecv, placement of wcg_gather_plan), which merges the runs on
 *                    its GPU (as wcg_merge_runs) into its result.  On root *nkeys / *nbytes
 *                    describe the merged file; elsewhere they are 0.
 * Collective calls: every rank of the communicator makes them in the same order.  A rank that
 * fails before data moves (a full table: WCG_EFULL; a call out of order; an allocation) still
 * joins the collectives with its status, and then EVERY rank returns an error (no rank is left
 * waiting in a send or receive); no units have moved and the tables are as they were.  A device
 * fault (a sticky HIP error: the context's stream can run nothing more, collectives included) is
 * outside this contract: that rank cannot join, its peers wait in the collective until the job is
 * stopped (bench.py's launcher stops every rank after --launch-timeout).  wcg_exchange_local
 * applies the same agreement across its contexts (tests/test_gpu_exchange_local.py forces a full
 * table on one of them). */
#define WCG_COMM_ID_BYTES 128
WCG_API int wcg_comm_id(uint8_t *id_out /* WCG_COMM_ID_BYTES */);
WCG_API int wcg_comm_init(wcg_ctx *ctx, const uint8_t *id /* WCG_COMM_ID_BYTES */, int rank, int world);
WCG_API int wcg_exchange(wcg_ctx *ctx, uint32_t nreduce, uint64_t *sent, uint64_t *received);
WCG_API int wcg_gather_merge(wcg_ctx *ctx, int root, uint64_t *nkeys, uint64_t *nbytes);

/* The host-side plan of the shuffle and of Merge's gather (pure arithmetic, no device; what
 * wcg_exchange / wcg_gather_merge compute from the gathered counts).
 *   wcg_exchange_plan: counts[s * world + d] = units rank s sends to rank d.  For `rank`:
 *     send_off[d] / send_cnt[d] = where its units for d start in its send buffer and how many;
 *     recv_off[s] / recv_cnt[s] = where the units from s land in its receive buffer (source-rank
 *     order); totals[2] = {units sent, units received}.  Output arrays may be NULL.
 *   wcg_gather_plan: sizes[p] = bytes of rank p's sorted run; run_off[p] = where it lands in
 *     root's receive buffer (root's own run is copied to run_off[root]); *total = all bytes. */
WCG_API int wcg_exchange_plan(const uint64_t *counts, uint32_t world, uint32_t rank, uint64_t *send_off,
                              uint64_t *send_cnt, uint64_t *recv_off, uint64_t *recv_cnt, uint64_t *totals);
WCG_API int wcg_gather_plan(const uint64_t *sizes, uint32_t world, uint32_t root, uint64_t *run_off,
                            uint64_t *total);

/* The same shuffle and Merge across `world` contexts of ONE process (e.g. several contexts on one
 * GPU standing in for the ranks of a node): the count matrix, the plans above, the export, import
 * and merge kernels are wcg_exchange's and wcg_gather_merge's; device-to-device copies stand in
 * for the RCCL sends and receives.  sent[world] / received[world] get each context's units. A
 * test transport for world > 1 where one GPU cannot host several RCCL ranks. Synchronous. */
WCG_API int wcg_exchange_local(wcg_ctx **ctxs, uint32_t world, uint32_t nreduce, uint64_t *sent,
                               uint64_t *received);
WCG_API int wcg_gather_merge_local(wcg_ctx **ctxs, uint32_t world, uint32_t root, uint64_t *nkeys,
                                   uint64_t *nbytes);

/* Merge (mapreduce.go:284-321) of sorted runs: dev_text holds nruns formatted outputs back to
 * back (each a sorted "key: count\n" file, e.g. the wcg_reduce output of every owner rank, with
 * disjoint keys), run r being run_bytes[r] bytes.  The runs are merged pairwise on the device
 * (ceil(log2 nruns) merge passes, long-key ties by full bytes) into this context's result
 * (wcg_result_device / wcg_result_copy).  Synchronous. */
WCG_API int wcg_merge_runs(wcg_ctx *ctx, const void *dev_text, const uint64_t *run_bytes, uint32_t nruns,
                           uint64_t *nkeys, uint64_t *nbytes);

/* Per-phase device time of the last pipeline run, in milliseconds, measured with HIP events
 * on the context's stream: ms[0] map kernel (tokenize + LDS aggregation, summed over the
 * wcg_map* calls since wcg_reset), ms[1] long-token counting + miss-log aggregation kernels
 * (k_long_hash, k_long_agg, k_agg pass 1, k_rp, k_agg pass 2), ms[2] compaction,
 * ms[3] sort, ms[4] format; the shuffle of wcg_exchange: ms[5] export (counts + unit writes),
 * ms[6] RCCL exchange (counts all-to-all, its host read, grouped send/recv), ms[7] import;
 * wcg_gather_merge: ms[8] RCCL gather of the runs to root, ms[9] merge of the runs.
 * n = number of doubles the caller provides (<= 10). */
WCG_API int wcg_timings(wcg_ctx *ctx, double *ms, int n, uint64_t *map_launches);
/* Enable/disable the event timing above (off by default: it adds event records, each a ~5 us
 * bubble between the kernels it separates).  on = 1: the phases of the last job; on = 2: every job
 * from this call on, summed (wcg_reset keeps the events, so a timed loop needs no wcg_timings
 * call, and no host round trip, between its jobs); on = 3: as 2, the map kernel (ms[0]) only. */
WCG_API int wcg_enable_timing(wcg_ctx *ctx, int on);

/* Diagnostics, stats9 = {tokens, distinct keys, tokens counted in LDS, global-table operations,
 * tokens > 15 bytes, long-key heap bytes (keys > 32 bytes; shorter long keys live in their
 * table slot's cell), overflow, spin_fail, records emitted by the second aggregation pass}. */
WCG_API int wcg_stats(wcg_ctx *ctx, uint64_t *stats9);

/* Diagnostics: the last wcg_map_file / wcg_map ingest, from its own timers and events (ms unless
 * noted): out[0] host wall time until every chunk was issued, out[1] reading (pread + line scan)
 * on the calling thread and its reader pool, out[2] waiting for a free staging slot, out[3] the
 * chunks' H2D copies (sum of copy durations), out[4] the copy engine's span (first copy start to
 * last copy end), out[5] its idle fraction 1 - out[3] / out[4], out[6] the chunks' map kernels
 * (sum), out[7] device span from the first copy to the last chunk's map end, out[8] chunks.
 * Waits for the context's streams.  n = number of doubles the caller provides (<= 9). */
WCG_API int wcg_ingest_stats(wcg_ctx *ctx, double *out, int n);

/* Diagnostics: which reduce the last wcg_reduce ran: *path = 1 for the one-launch reduce of small
 * one-pass jobs (compaction, sort and formatting in one persistent kernel: jobs after the first of
 * a context whose previous job had at most 2^17 keys), 0 for the multi-launch path. */
WCG_API int wcg_reduce_path(const wcg_ctx *ctx, int *path);

/* FNV-1a 32 (= ihash, mapreduce.go:185-189), host side, for partition arithmetic. */
WCG_API uint32_t wcg_ihash(const uint8_t *key, uint64_t len);

WCG_API const char *wcg_version(void);

#ifdef __cplusplus
}
#endif
#endif /* WCG_H */
