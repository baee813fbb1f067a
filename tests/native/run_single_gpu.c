/*
 * run_single_gpu.c - a C caller of the drop-in boundary (include/wcg.h), replaying call for call
 * the cgo stub of INTEGRATION.md section 2 (runSingleGPU = RunSingle, mapreduce.go:344-356, with
 * the wc UDFs of src/main/wc.go:17-38) and the world-1 form of section 4 (wcg_comm_id /
 * wcg_comm_init / wcg_exchange / wcg_reduce / wcg_gather_merge).  Test infrastructure: built by
 * __graft_entry__.build() with gcc against libwcg.so, run by tests/test_gpu_native.py, which diffs
 * every file it writes against the oracle.
 *
 *   run_single_gpu <dir> <file> <nMap> <nReduce>
 *
 * In <dir> (the reference runs in its working directory):
 *   Split      mrtmp.<file>-<m>, as mapreduce.go:141-179 writes them (bufio.Scanner lines: a
 *              trailing '\r' dropped, a line of 65536+ bytes ends the scan - quirk P1; a new split
 *              when the bytes written exceed nchunk * m)
 *   DoMap      readSplit: ONE read of at most 1 GiB per split (quirk P2), then wcg_map
 *   DoReduce   wcg_reduce, then per r the size query wcg_partition(.., NULL, 0, &n) and the copy;
 *              mrtmp.<file>-res-<r>
 *   Merge      wcg_result_copy -> mrtmp.<file>; wcg_result_device + wcg_free (library-owned)
 *   async      the same job through wcg_reduce_async / wcg_reduce_wait -> mrtmp.<file>.async
 *   world 1    wcg_comm_id, wcg_comm_init(rank 0, world 1), wcg_reset, wcg_map of every split,
 *              wcg_exchange, wcg_reduce, wcg_gather_merge(root 0), wcg_result_copy ->
 *              mrtmp.<file>.comm
 * Any non-zero status ends the program with wcg_last_error (the reference's log.Fatal).
 */
#define _POSIX_C_SOURCE 200809L
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include "wcg.h"

static wcg_ctx *g_ctx;

static void wcg_check(int rc, const char *where) {
    if (rc != WCG_OK) {
        fprintf(stderr, "%s: status %d: %s\n", where, rc, wcg_last_error(g_ctx));
        exit(2);
    }
}

static void fatal(const char *where) {
    fprintf(stderr, "%s: %s\n", where, strerror(errno));
    exit(2);
}

static uint8_t *read_all(const char *path, uint64_t *n) {
    FILE *f = fopen(path, "rb");
    if (!f) fatal(path);
    struct stat sb;
    if (fstat(fileno(f), &sb) != 0) fatal(path);
    uint8_t *b = malloc(sb.st_size + 1);
    if (!b) fatal("malloc");
    *n = fread(b, 1, sb.st_size, f);
    fclose(f);
    return b;
}

static void write_all(const char *path, const uint8_t *b, uint64_t n) {
    FILE *f = fopen(path, "wb");
    if (!f) fatal(path);
    if (n && fwrite(b, 1, n, f) != n) fatal(path);
    if (fclose(f) != 0) fatal(path);
}

static void map_name(char *out, size_t cap, const char *file, int m) { snprintf(out, cap, "mrtmp.%s-%d", file, m); }

/* Split (mapreduce.go:141-179); returns the number of split files written */
static int split(const char *file, int nmap) {
    printf("Split %s\n", file);
    uint64_t size;
    uint8_t *data = read_all(file, &size);
    const int64_t nchunk = (int64_t)size / nmap + 1;
    char name[4096];
    int m = 1, files = 1;
    int64_t i = 0;
    map_name(name, sizeof name, file, 0);
    FILE *out = fopen(name, "wb");
    if (!out) fatal(name);
    uint64_t p = 0;
    while (p < size) {
        const uint8_t *nl = memchr(data + p, '\n', size - p);
        uint64_t len = nl ? (uint64_t)(nl - (data + p)) : size - p;
        if (len >= 65536) break;                    /* bufio.ErrTooLong ends the scan (P1) */
        if (i > nchunk * m) {
            if (fclose(out) != 0) fatal(name);
            map_name(name, sizeof name, file, m);
            out = fopen(name, "wb");
            if (!out) fatal(name);
            m++;
            files++;
        }
        uint64_t keep = len;
        if (keep && data[p + keep - 1] == '\r') keep--;   /* ScanLines drops one trailing CR */
        if (keep && fwrite(data + p, 1, keep, out) != keep) fatal(name);
        fputc('\n', out);
        i += (int64_t)keep + 1;
        p += len + (nl ? 1 : 0);
    }
    if (fclose(out) != 0) fatal(name);
    free(data);
    return files;
}

/* readSplit of the cgo stub: one read of at most 1 GiB (Go's os.File.Read cap, quirk P2) */
static uint8_t *read_split(const char *name, uint64_t *n) {
    int fd = open(name, O_RDONLY);
    if (fd < 0) fatal(name);          /* DoMap: log.Fatal on a missing split (quirk P3) */
    struct stat sb;
    if (fstat(fd, &sb) != 0) fatal(name);
    uint64_t want = (uint64_t)sb.st_size;
    uint8_t *b = malloc(want + 1);
    if (!b) fatal("malloc");
    uint64_t cap = want < (1ull << 30) ? want : (1ull << 30);
    ssize_t got = cap ? read(fd, b, cap) : 0;
    if (got < 0) fatal(name);
    close(fd);
    *n = (uint64_t)got;
    return b;
}

static void map_splits(const char *file, int nmap, int print) {
    char name[4096];
    for (int m = 0; m < nmap; m++) {
        map_name(name, sizeof name, file, m);
        uint64_t n;
        uint8_t *b = read_split(name, &n);
        if (print) printf("DoMap: read split %s %llu\n", name, (unsigned long long)n);
        if (n) wcg_check(wcg_map(g_ctx, b, n), "DoMap");
        free(b);
    }
}

static void write_result(const char *path, uint64_t nbytes) {
    uint8_t *out = malloc(nbytes + 1);
    if (!out) fatal("malloc");
    wcg_check(wcg_result_copy(g_ctx, out, nbytes + 1), "Merge");
    write_all(path, out, nbytes);
    free(out);
}

int main(int argc, char **argv) {
    if (argc != 5) {
        fprintf(stderr, "usage: %s <dir> <file> <nMap> <nReduce>\n", argv[0]);
        return 1;
    }
    if (chdir(argv[1]) != 0) fatal(argv[1]);
    const char *file = argv[2];
    const int nmap = atoi(argv[3]), nreduce = atoi(argv[4]);
    char name[4096];

    /* ---- runSingleGPU */
    int nsplit = split(file, nmap);
    printf("split files %d\n", nsplit);
    if (wcg_open(0, 1ull << 30, 1ull << 22, &g_ctx) != WCG_OK) {
        fprintf(stderr, "wcg_open: %s\n", g_ctx ? wcg_last_error(g_ctx) : "failed");
        return 2;
    }
    wcg_check(wcg_reset(g_ctx), "DoMap");
    map_splits(file, nmap, 1);
    uint64_t nkeys = 0, nbytes = 0;
    wcg_check(wcg_reduce(g_ctx, &nkeys, &nbytes), "DoReduce");
    for (int r = 0; r < nreduce; r++) {
        uint64_t n = 0;
        wcg_check(wcg_partition(g_ctx, (uint32_t)nreduce, (uint32_t)r, NULL, 0, &n), "DoReduce");
        uint8_t *buf = malloc(n + 1);
        if (!buf) fatal("malloc");
        wcg_check(wcg_partition(g_ctx, (uint32_t)nreduce, (uint32_t)r, buf, n + 1, &n), "DoReduce");
        snprintf(name, sizeof name, "mrtmp.%s-res-%d", file, r);
        write_all(name, buf, n);
        free(buf);
    }
    snprintf(name, sizeof name, "mrtmp.%s", file);
    write_result(name, nbytes);
    const void *dev = NULL;
    wcg_check(wcg_result_device(g_ctx, &dev, NULL), "Merge");
    wcg_check(wcg_free(g_ctx, dev), "Merge");
    printf("keys %llu bytes %llu\n", (unsigned long long)nkeys, (unsigned long long)nbytes);

    /* ---- the same job again, without the host wait (wcg_reduce_async / wcg_reduce_wait) */
    wcg_check(wcg_reset(g_ctx), "DoMap");
    map_splits(file, nmap, 0);
    wcg_check(wcg_reduce_async(g_ctx), "DoReduce");
    uint64_t ak = 0, ab = 0;
    wcg_check(wcg_reduce_wait(g_ctx, &ak, &ab), "DoReduce");
    int path = -1;
    wcg_check(wcg_reduce_path(g_ctx, &path), "DoReduce");
    snprintf(name, sizeof name, "mrtmp.%s.async", file);
    write_result(name, ab);
    printf("async keys %llu bytes %llu path %d\n", (unsigned long long)ak, (unsigned long long)ab, path);

    /* ---- world 1 over RCCL */
    uint8_t id[WCG_COMM_ID_BYTES];
    wcg_check(wcg_comm_id(id), "comm");
    wcg_check(wcg_comm_init(g_ctx, id, 0, 1), "comm");
    wcg_check(wcg_reset(g_ctx), "DoMap");
    map_splits(file, nmap, 0);
    uint64_t sent = 0, received = 0;
    wcg_check(wcg_exchange(g_ctx, (uint32_t)nreduce, &sent, &received), "shuffle");
    wcg_check(wcg_reduce(g_ctx, &nkeys, &nbytes), "DoReduce");
    wcg_check(wcg_gather_merge(g_ctx, 0, &nkeys, &nbytes), "Merge");
    snprintf(name, sizeof name, "mrtmp.%s.comm", file);
    write_result(name, nbytes);
    printf("comm sent %llu received %llu keys %llu bytes %llu\n", (unsigned long long)sent,
           (unsigned long long)received, (unsigned long long)nkeys, (unsigned long long)nbytes);
    wcg_check(wcg_close(g_ctx), "close");
    return 0;
}
