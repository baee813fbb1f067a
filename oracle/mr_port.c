/*
 * mr_port.c - file-based C port of the reference's sequential MapReduce driver with the wc UDFs.
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY (bench.py cpu_baseline leg, tests).  Never part of the
 * product.  It restates RunSingle (/root/reference/src/mapreduce/mapreduce.go:344-356) step by
 * step, keeping the reference's on-disk formats AND its I/O pattern, because that pattern is
 * what the reference's CPU time is made of:
 *
 *   Split    mapreduce.go:141-179  bufio.Scanner lines (64 KiB limit), bufio writer, files
 *                                  mrtmp.<f>-<m>, new file when written bytes i > nchunk*m
 *   DoMap    mapreduce.go:193-231  whole split read; Map = FieldsFunc(!IsLetter) (wc.go:17-30);
 *                                  for each r: create mrtmp.<f>-<m>-<r>, re-walk ALL tokens,
 *                                  ihash each, json.Encoder.Encode -> ONE write(2) per record
 *                                  (unbuffered *os.File, mapreduce.go:219,223)
 *   DoReduce mapreduce.go:239-280  decode every mrtmp.<f>-<m>-<r>, group, sort.Strings,
 *                                  Reduce = strconv.Itoa(len) (wc.go:35-38), one write(2)/key
 *   Merge    mapreduce.go:284-321  decode res files, sort.Strings, bufio "%s: %s\n"
 *
 * Differences from Go that are cost-only: no GC / reflection (so this port is FASTER than the
 * reference, i.e. the baseline it gives is generous to the CPU side).
 */
#include <fcntl.h>
#include <stdint.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#define WCO_API __attribute__((visibility("default")))

uint64_t wco_tokens(const uint8_t *s, uint64_t n, uint64_t *starts, uint32_t *lens, uint64_t cap);
uint32_t wco_ihash(const uint8_t *k, uint64_t len);

static void die(const char *what, const char *name) { fprintf(stderr, "mr_port: %s %s\n", what, name); exit(1); }

static uint8_t *read_all(const char *path, uint64_t *n) {
    FILE *f = fopen(path, "rb");
    if (!f) die("open", path);
    fseek(f, 0, SEEK_END); long sz = ftell(f); fseek(f, 0, SEEK_SET);
    uint8_t *b = (uint8_t *)malloc((size_t)sz + 1);
    if (sz && fread(b, 1, (size_t)sz, f) != (size_t)sz) die("read", path);
    fclose(f); *n = (uint64_t)sz; return b;
}

static void map_name(char *o, size_t cap, const char *dir, const char *f, int m) { snprintf(o, cap, "%s/mrtmp.%s-%d", dir, f, m); }
static void reduce_name(char *o, size_t cap, const char *dir, const char *f, int m, int r) { snprintf(o, cap, "%s/mrtmp.%s-%d-%d", dir, f, m, r); }
static void merge_name(char *o, size_t cap, const char *dir, const char *f, int r) { snprintf(o, cap, "%s/mrtmp.%s-res-%d", dir, f, r); }

/* Split: mapreduce.go:141-179. Returns the number of split files created. */
static int split(const char *dir, const char *file, int nmap) {
    char path[4096]; snprintf(path, sizeof path, "%s/%s", dir, file);
    uint64_t size; uint8_t *b = read_all(path, &size);
    int64_t nchunk = (int64_t)size / nmap + 1;
    char name[4096]; map_name(name, sizeof name, dir, file, 0);
    FILE *out = fopen(name, "wb"); if (!out) die("create", name);
    setvbuf(out, NULL, _IOFBF, 4096);           /* bufio.NewWriter default size */
    int m = 1; int64_t i = 0; uint64_t pos = 0;
    while (pos < size) {
        uint8_t *nl = (uint8_t *)memchr(b + pos, '\n', size - pos);
        uint64_t len = nl ? (uint64_t)(nl - (b + pos)) : size - pos;
        uint64_t adv = nl ? len + 1 : len;
        if (adv > 65536 || (!nl && len >= 65536)) break;      /* quirk P1 */
        if (len && b[pos + len - 1] == '\r') len--;
        if (i > nchunk * m) {
            fclose(out); map_name(name, sizeof name, dir, file, m);
            out = fopen(name, "wb"); if (!out) die("create", name);
            setvbuf(out, NULL, _IOFBF, 4096); m++;
        }
        fwrite(b + pos, 1, len, out); fputc('\n', out);
        i += (int64_t)len + 1; pos += adv;
    }
    fclose(out); free(b);
    return m;
}

static void write_json(int fd, const uint8_t *k, uint32_t len, const char *v) {
    char buf[65536 + 64]; size_t o = 0;
    memcpy(buf, "{\"Key\":\"", 8); o = 8;
    memcpy(buf + o, k, len); o += len;
    memcpy(buf + o, "\",\"Value\":\"", 11); o += 11;
    size_t vl = strlen(v); memcpy(buf + o, v, vl); o += vl;
    memcpy(buf + o, "\"}\n", 3); o += 3;
    if (write(fd, buf, o) != (ssize_t)o) die("write", "json");
}

/* DoMap: mapreduce.go:193-231 */
static void do_map(const char *dir, const char *file, int job, int nreduce) {
    char name[4096]; map_name(name, sizeof name, dir, file, job);
    uint64_t n; uint8_t *b = read_all(name, &n);
    uint64_t cap = n / 2 + 1;
    uint64_t *st = (uint64_t *)malloc(cap * sizeof(uint64_t)); uint32_t *ln = (uint32_t *)malloc(cap * sizeof(uint32_t));
    uint64_t nt = wco_tokens(b, n, st, ln, cap);
    for (int r = 0; r < nreduce; r++) {
        reduce_name(name, sizeof name, dir, file, job, r);
        int fd = open(name, O_WRONLY | O_CREAT | O_TRUNC, 0644); if (fd < 0) die("create", name);
        for (uint64_t t = 0; t < nt; t++)
            if (wco_ihash(b + st[t], ln[t]) % (uint32_t)nreduce == (uint32_t)r) write_json(fd, b + st[t], ln[t], "1");
        close(fd);
    }
    free(st); free(ln); free(b);
}

/* minimal decoder for the lines this package writes: {"Key":"<k>","Value":"<v>"} */
typedef struct { uint8_t *k; uint32_t klen; uint8_t *v; uint32_t vlen; } kv_t;
static uint64_t parse_lines(uint8_t *b, uint64_t n, kv_t **out) {
    uint64_t cap = 1024, cnt = 0; kv_t *v = (kv_t *)malloc(cap * sizeof(kv_t));
    uint64_t p = 0;
    while (p < n) {
        uint8_t *e = (uint8_t *)memchr(b + p, '\n', n - p); uint64_t end = e ? (uint64_t)(e - b) : n;
        uint8_t *ks = b + p + 8; uint8_t *ke = (uint8_t *)memchr(ks, '"', end - (p + 8));
        if (!ke) break;                                            /* decode error ends the file */
        uint8_t *vs = ke + 11; uint8_t *ve = (uint8_t *)memchr(vs, '"', (size_t)(b + end - vs));
        if (!ve) break;
        if (cnt == cap) { cap *= 2; v = (kv_t *)realloc(v, cap * sizeof(kv_t)); }
        v[cnt].k = ks; v[cnt].klen = (uint32_t)(ke - ks); v[cnt].v = vs; v[cnt].vlen = (uint32_t)(ve - vs); cnt++;
        p = end + 1;
    }
    *out = v; return cnt;
}

typedef struct { uint8_t *k; uint32_t len; uint64_t cnt; uint8_t *v; uint32_t vlen; uint32_t used; } slot_t;
static uint64_t fnv64(const uint8_t *k, uint32_t l) { uint64_t h = 1469598103934665603ull; for (uint32_t i = 0; i < l; i++) { h ^= k[i]; h *= 1099511628211ull; } return h; }
static int cmp_slot(const void *a, const void *b) {
    const slot_t *x = (const slot_t *)a, *y = (const slot_t *)b;
    uint32_t m = x->len < y->len ? x->len : y->len; int c = memcmp(x->k, y->k, m);
    return c ? c : (x->len > y->len) - (x->len < y->len);
}
typedef struct { slot_t *s; uint64_t cap, n; } map_t;
static slot_t *map_get(map_t *m, uint8_t *k, uint32_t len) {
    if ((m->n + 1) * 2 > m->cap) {
        map_t nm = { (slot_t *)calloc(m->cap * 2, sizeof(slot_t)), m->cap * 2, 0 };
        for (uint64_t i = 0; i < m->cap; i++) if (m->s[i].used) { slot_t *d = map_get(&nm, m->s[i].k, m->s[i].len); *d = m->s[i]; }
        free(m->s); *m = nm;
    }
    uint64_t i = fnv64(k, len) & (m->cap - 1);
    for (;;) {
        slot_t *s = &m->s[i];
        if (!s->used) { s->used = 1; s->k = k; s->len = len; s->cnt = 0; m->n++; return s; }
        if (s->len == len && memcmp(s->k, k, len) == 0) return s;
        i = (i + 1) & (m->cap - 1);
    }
}

/* DoReduce: mapreduce.go:239-280 */
static void do_reduce(const char *dir, const char *file, int job, int nmap) {
    map_t m = { (slot_t *)calloc(1024, sizeof(slot_t)), 1024, 0 };
    uint8_t **bufs = (uint8_t **)calloc((size_t)nmap, sizeof(void *));
    char name[4096];
    for (int i = 0; i < nmap; i++) {
        reduce_name(name, sizeof name, dir, file, i, job);
        uint64_t n; bufs[i] = read_all(name, &n);
        kv_t *kv; uint64_t c = parse_lines(bufs[i], n, &kv);
        for (uint64_t j = 0; j < c; j++) map_get(&m, kv[j].k, kv[j].klen)->cnt++;
        free(kv);
    }
    slot_t *v = (slot_t *)malloc((m.n ? m.n : 1) * sizeof(slot_t)); uint64_t k = 0;
    for (uint64_t i = 0; i < m.cap; i++) if (m.s[i].used) v[k++] = m.s[i];
    qsort(v, k, sizeof(slot_t), cmp_slot);
    merge_name(name, sizeof name, dir, file, job);
    int fd = open(name, O_WRONLY | O_CREAT | O_TRUNC, 0644); if (fd < 0) die("create", name);
    char num[24];
    for (uint64_t i = 0; i < k; i++) { snprintf(num, sizeof num, "%llu", (unsigned long long)v[i].cnt); write_json(fd, v[i].k, v[i].len, num); }
    close(fd);
    for (int i = 0; i < nmap; i++) free(bufs[i]);
    free(bufs); free(v); free(m.s);
}

/* Merge: mapreduce.go:284-321 */
static void merge(const char *dir, const char *file, int nreduce) {
    map_t m = { (slot_t *)calloc(1024, sizeof(slot_t)), 1024, 0 };
    uint8_t **bufs = (uint8_t **)calloc((size_t)nreduce, sizeof(void *));
    char name[4096];
    for (int r = 0; r < nreduce; r++) {
        merge_name(name, sizeof name, dir, file, r);
        uint64_t n; bufs[r] = read_all(name, &n);
        kv_t *kv; uint64_t c = parse_lines(bufs[r], n, &kv);
        for (uint64_t j = 0; j < c; j++) { slot_t *s = map_get(&m, kv[j].k, kv[j].klen); s->v = kv[j].v; s->vlen = kv[j].vlen; }
        free(kv);
    }
    slot_t *v = (slot_t *)malloc((m.n ? m.n : 1) * sizeof(slot_t)); uint64_t k = 0;
    for (uint64_t i = 0; i < m.cap; i++) if (m.s[i].used) v[k++] = m.s[i];
    qsort(v, k, sizeof(slot_t), cmp_slot);
    snprintf(name, sizeof name, "%s/mrtmp.%s", dir, file);
    FILE *out = fopen(name, "wb"); if (!out) die("create", name);
    setvbuf(out, NULL, _IOFBF, 4096);
    for (uint64_t i = 0; i < k; i++) { fwrite(v[i].k, 1, v[i].len, out); fputs(": ", out); fwrite(v[i].v, 1, v[i].vlen, out); fputc('\n', out); }
    fclose(out);
    for (int r = 0; r < nreduce; r++) free(bufs[r]);
    free(bufs); free(v); free(m.s);
}

/* RunSingle(nMap, nReduce, file, Map, Reduce): mapreduce.go:344-356.  Files live in dir.
 * Returns 0, or -1 when Split created fewer than nMap files (reference: DoMap log.Fatal, P3). */
WCO_API int mrp_run_single(const char *dir, const char *file, int nmap, int nreduce) {
    int made = split(dir, file, nmap);
    if (made != nmap) return -1;
    for (int i = 0; i < nmap; i++) do_map(dir, file, i, nreduce);
    for (int r = 0; r < nreduce; r++) do_reduce(dir, file, r, nmap);
    merge(dir, file, nreduce);
    return 0;
}

/* DoReduce(job) alone (mapreduce.go:239-280): reads mrtmp.<file>-<m>-<job> for m < nmap in dir,
 * which any DoMap wrote (tests: the GPU's JSON intermediates, wcg_map_json). */
WCO_API void mrp_do_reduce(const char *dir, const char *file, int job, int nmap) { do_reduce(dir, file, job, nmap); }

/* The distributed master/worker path's work on one host (master.go:29-88, worker.go:22-34):
 * Split, then nworkers worker threads take map jobs from the master's queue until the map phase
 * is done (the barrier of master.go:73), then reduce jobs, then Merge.  Same files and formats
 * as RunSingle; the RPC transport is not modelled (it carries no bytes of the data path). */
typedef struct {
    const char *dir, *file;
    int nmap, nreduce, next_job, phase;
    pthread_mutex_t mu;
    pthread_barrier_t bar;
} par_t;

static void *par_worker(void *arg) {
    par_t *p = (par_t *)arg;
    for (int phase = 0; phase < 2; phase++) {
        while (1) {
            pthread_mutex_lock(&p->mu);
            const int j = p->next_job++;
            pthread_mutex_unlock(&p->mu);
            if (phase == 0 ? j >= p->nmap : j >= p->nreduce) break;
            if (phase == 0) do_map(p->dir, p->file, j, p->nreduce);
            else do_reduce(p->dir, p->file, j, p->nmap);
        }
        if (pthread_barrier_wait(&p->bar) == PTHREAD_BARRIER_SERIAL_THREAD) p->next_job = 0;
        pthread_barrier_wait(&p->bar);
    }
    return NULL;
}

WCO_API int mrp_run_parallel(const char *dir, const char *file, int nmap, int nreduce, int nworkers) {
    int made = split(dir, file, nmap);
    if (made != nmap) return -1;
    par_t p;
    p.dir = dir; p.file = file; p.nmap = nmap; p.nreduce = nreduce; p.next_job = 0; p.phase = 0;
    pthread_mutex_init(&p.mu, NULL);
    pthread_barrier_init(&p.bar, NULL, (unsigned)nworkers);
    pthread_t *th = (pthread_t *)calloc((size_t)nworkers, sizeof(pthread_t));
    for (int i = 0; i < nworkers; i++) pthread_create(&th[i], NULL, par_worker, &p);
    for (int i = 0; i < nworkers; i++) pthread_join(th[i], NULL);
    pthread_barrier_destroy(&p.bar);
    pthread_mutex_destroy(&p.mu);
    free(th);
    merge(dir, file, nreduce);
    return 0;
}
