/*
 * wc_oracle.c - plain-C CPU restatement of the reference word-count path.
 *
 * TEST INFRASTRUCTURE ONLY.  Built into oracle/liboracle.so; only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg load it, and only as the checker.  The product
 * (mit-6.824-2015_amd/) never links or calls it.
 *
 * Restates (paths relative to /root/reference):
 *   Map      src/main/wc.go:17-30        strings.FieldsFunc(value, !unicode.IsLetter)
 *            - rune iteration: Go unicode/utf8 DecodeRune accept ranges, invalid -> U+FFFD w=1
 *            - unicode.IsLetter: Unicode 13.0.0 category L (oracle/letter_ranges.h)
 *   Reduce   src/main/wc.go:35-38        strconv.Itoa(values.Len())
 *   ihash    src/mapreduce/mapreduce.go:185-189   FNV-1a 32
 *   DoReduce src/mapreduce/mapreduce.go:239-280   JSON line {"Key":k,"Value":v} per key, sorted
 *   Merge    src/mapreduce/mapreduce.go:284-321   sort.Strings (bytewise) + "%s: %s\n"
 *
 * Under the parity domain of SURVEY.md 8(a) (P1-P4) the merged file depends only on the input
 * bytes: sorted_bytewise({(tok, count)}) rendered "tok: count\n".  This file computes exactly
 * that (multi-threaded: chunks are cut after an ASCII non-letter byte, where neither a rune nor
 * a token can straddle the cut).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "letter_ranges.h"

#define WCO_API __attribute__((visibility("default")))

/* ---------------- letters + UTF-8 (wc.go:18-21 via Go unicode / unicode/utf8) ---------- */

static int is_letter_cp(uint32_t cp) {
    if (cp < 0x80) return ((cp | 0x20) - 'a') < 26u;
    int lo = 0, hi = WCO_NLETTER_RANGES - 1;
    while (lo <= hi) {
        int mid = (lo + hi) >> 1;
        if (cp < WCO_LETTER_RANGES[mid][0]) hi = mid - 1;
        else if (cp > WCO_LETTER_RANGES[mid][1]) lo = mid + 1;
        else return 1;
    }
    return 0;
}

/* Go utf8.DecodeRune: returns width; *cp = code point or 0xFFFFFFFF for RuneError. */
static inline int decode_rune(const uint8_t *s, size_t n, size_t i, uint32_t *cp) {
    uint8_t b0 = s[i];
    if (b0 < 0x80) { *cp = b0; return 1; }
    int w; uint8_t lo = 0x80, hi = 0xBF;
    if (b0 >= 0xC2 && b0 <= 0xDF) w = 2;
    else if (b0 >= 0xE0 && b0 <= 0xEF) { w = 3; if (b0 == 0xE0) lo = 0xA0; else if (b0 == 0xED) hi = 0x9F; }
    else if (b0 >= 0xF0 && b0 <= 0xF4) { w = 4; if (b0 == 0xF0) lo = 0x90; else if (b0 == 0xF4) hi = 0x8F; }
    else { *cp = 0xFFFFFFFFu; return 1; }
    if (i + 1 >= n || s[i + 1] < lo || s[i + 1] > hi) { *cp = 0xFFFFFFFFu; return 1; }
    for (int k = 2; k < w; k++)
        if (i + k >= n || (s[i + k] & 0xC0) != 0x80) { *cp = 0xFFFFFFFFu; return 1; }
    uint32_t c;
    if (w == 2) c = ((uint32_t)(b0 & 0x1F) << 6) | (s[i + 1] & 0x3F);
    else if (w == 3) c = ((uint32_t)(b0 & 0x0F) << 12) | ((uint32_t)(s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
    else c = ((uint32_t)(b0 & 0x07) << 18) | ((uint32_t)(s[i + 1] & 0x3F) << 12) |
             ((uint32_t)(s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
    *cp = c;
    return w;
}

static inline int letter_rune(uint32_t cp) { return cp != 0xFFFFFFFFu && is_letter_cp(cp); }

WCO_API int wco_is_letter(uint32_t cp) { return is_letter_cp(cp); }
WCO_API const char *wco_unicode_version(void) { return WCO_UNICODE_VERSION; }

/* FieldsFunc token stream: writes up to cap (start,len) pairs, returns the token count. */
WCO_API uint64_t wco_tokens(const uint8_t *s, uint64_t n, uint64_t *starts, uint32_t *lens, uint64_t cap) {
    uint64_t nt = 0; int64_t start = -1; size_t i = 0;
    while (i < n) {
        uint32_t cp; int w = decode_rune(s, n, i, &cp);
        if (letter_rune(cp)) { if (start < 0) start = (int64_t)i; }
        else if (start >= 0) {
            if (nt < cap) { starts[nt] = (uint64_t)start; lens[nt] = (uint32_t)(i - start); }
            nt++; start = -1;
        }
        i += w;
    }
    if (start >= 0) { if (nt < cap) { starts[nt] = (uint64_t)start; lens[nt] = (uint32_t)(n - start); } nt++; }
    return nt;
}

/* ---------------- ihash (mapreduce.go:185-189) ---------------- */
WCO_API uint32_t wco_ihash(const uint8_t *k, uint64_t len) {
    uint32_t h = 0x811C9DC5u;
    for (uint64_t i = 0; i < len; i++) { h ^= k[i]; h *= 0x01000193u; }
    return h;
}

/* ---------------- counting table ---------------- */
typedef struct { const uint8_t *key; uint32_t len; uint32_t hash; uint64_t count; } entry_t;
typedef struct { entry_t *e; uint64_t cap, n; } table_t;

static uint32_t khash(const uint8_t *k, uint32_t len) {
    uint64_t h = 1469598103934665603ull;
    for (uint32_t i = 0; i < len; i++) { h ^= k[i]; h *= 1099511628211ull; }
    return (uint32_t)(h ^ (h >> 32)) | 1u;
}

static void table_init(table_t *t, uint64_t cap) {
    uint64_t c = 1024; while (c < cap) c <<= 1;
    t->cap = c; t->n = 0; t->e = (entry_t *)calloc(c, sizeof(entry_t));
}

static void table_add(table_t *t, const uint8_t *k, uint32_t len, uint32_t h, uint64_t cnt);

static void table_grow(table_t *t) {
    table_t nt; table_init(&nt, t->cap * 2);
    for (uint64_t i = 0; i < t->cap; i++)
        if (t->e[i].hash) table_add(&nt, t->e[i].key, t->e[i].len, t->e[i].hash, t->e[i].count);
    free(t->e); *t = nt;
}

static void table_add(table_t *t, const uint8_t *k, uint32_t len, uint32_t h, uint64_t cnt) {
    if ((t->n + 1) * 2 > t->cap) table_grow(t);
    uint64_t m = t->cap - 1, i = h & m;
    for (;;) {
        entry_t *e = &t->e[i];
        if (!e->hash) { e->key = k; e->len = len; e->hash = h; e->count = cnt; t->n++; return; }
        if (e->hash == h && e->len == len && memcmp(e->key, k, len) == 0) { e->count += cnt; return; }
        i = (i + 1) & m;
    }
}

typedef struct { const uint8_t *s; uint64_t n; table_t t; } job_t;

static void *count_job(void *arg) {
    job_t *j = (job_t *)arg;
    table_init(&j->t, 1 << 16);
    const uint8_t *s = j->s; uint64_t n = j->n; int64_t start = -1; uint64_t i = 0;
    while (i < n) {
        uint8_t b = s[i];
        int w = 1, let;
        if (b < 0x80) let = ((uint32_t)(b | 0x20) - 'a') < 26u;
        else { uint32_t cp; w = decode_rune(s, n, i, &cp); let = letter_rune(cp); }
        if (let) { if (start < 0) start = (int64_t)i; }
        else if (start >= 0) {
            uint32_t len = (uint32_t)(i - start);
            table_add(&j->t, s + start, len, khash(s + start, len), 1);
            start = -1;
        }
        i += w;
    }
    if (start >= 0) { uint32_t len = (uint32_t)(n - start); table_add(&j->t, s + start, len, khash(s + start, len), 1); }
    return NULL;
}

typedef struct wco_result {
    uint64_t nkeys;
    const uint8_t **keys; uint32_t *lens; uint64_t *counts;   /* sorted bytewise */
    uint64_t ntokens;
} wco_result;

static int cmp_entry(const void *a, const void *b) {
    const entry_t *x = (const entry_t *)a, *y = (const entry_t *)b;
    uint32_t m = x->len < y->len ? x->len : y->len;
    int c = memcmp(x->key, y->key, m);
    if (c) return c;
    return (x->len > y->len) - (x->len < y->len);
}

/* Word count of s[0:n) (Map + Reduce + Merge's sort), nthreads >= 1.  Keys alias s. */
WCO_API wco_result *wco_count(const uint8_t *s, uint64_t n, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (n < (1u << 20)) nthreads = 1;
    job_t *jobs = (job_t *)calloc((size_t)nthreads, sizeof(job_t));
    uint64_t pos = 0;
    for (int t = 0; t < nthreads; t++) {
        uint64_t end = (t == nthreads - 1) ? n : (n / nthreads) * (uint64_t)(t + 1);
        if (end < pos) end = pos;
        /* cut right after an ASCII non-letter byte: no rune or token straddles it */
        while (end < n && end > pos) {
            uint8_t b = s[end - 1];
            if (b < 0x80 && !(((uint32_t)(b | 0x20) - 'a') < 26u)) break;
            end++;
        }
        jobs[t].s = s + pos; jobs[t].n = end - pos; pos = end;
    }
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, count_job, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    table_t all = jobs[0].t;
    for (int t = 1; t < nthreads; t++) {
        for (uint64_t i = 0; i < jobs[t].t.cap; i++) {
            entry_t *e = &jobs[t].t.e[i];
            if (e->hash) table_add(&all, e->key, e->len, e->hash, e->count);
        }
        free(jobs[t].t.e);
    }
    entry_t *v = (entry_t *)malloc((all.n ? all.n : 1) * sizeof(entry_t));
    uint64_t k = 0, ntok = 0;
    for (uint64_t i = 0; i < all.cap; i++) if (all.e[i].hash) { v[k++] = all.e[i]; ntok += all.e[i].count; }
    free(all.e); free(jobs); free(th);
    qsort(v, k, sizeof(entry_t), cmp_entry);
    wco_result *r = (wco_result *)calloc(1, sizeof(wco_result));
    r->nkeys = k; r->ntokens = ntok;
    r->keys = (const uint8_t **)malloc((k ? k : 1) * sizeof(void *));
    r->lens = (uint32_t *)malloc((k ? k : 1) * sizeof(uint32_t));
    r->counts = (uint64_t *)malloc((k ? k : 1) * sizeof(uint64_t));
    for (uint64_t i = 0; i < k; i++) { r->keys[i] = v[i].key; r->lens[i] = v[i].len; r->counts[i] = v[i].count; }
    free(v);
    return r;
}

WCO_API uint64_t wco_nkeys(const wco_result *r) { return r->nkeys; }
WCO_API uint64_t wco_ntokens(const wco_result *r) { return r->ntokens; }
WCO_API void wco_key(const wco_result *r, uint64_t i, const uint8_t **key, uint32_t *len, uint64_t *count) {
    *key = r->keys[i]; *len = r->lens[i]; *count = r->counts[i];
}

static int fmt_u64(uint64_t v, char *buf) { return sprintf(buf, "%llu", (unsigned long long)v); }

/* Merge (mapreduce.go:311-319): "%s: %s\n" in sorted order.  out==NULL -> size only. */
WCO_API uint64_t wco_merged(const wco_result *r, uint8_t *out) {
    uint64_t o = 0; char num[24];
    for (uint64_t i = 0; i < r->nkeys; i++) {
        int d = fmt_u64(r->counts[i], num);
        if (out) { memcpy(out + o, r->keys[i], r->lens[i]); out[o + r->lens[i]] = ':'; out[o + r->lens[i] + 1] = ' ';
                   memcpy(out + o + r->lens[i] + 2, num, (size_t)d); out[o + r->lens[i] + 2 + d] = '\n'; }
        o += r->lens[i] + 3 + (uint64_t)d;
    }
    return o;
}

/* DoReduce output mrtmp.<f>-res-<r> (mapreduce.go:264-279) for wc. out==NULL -> size only. */
WCO_API uint64_t wco_res(const wco_result *r, uint32_t nreduce, uint32_t part, uint8_t *out) {
    static const char pre[] = "{\"Key\":\"", mid[] = "\",\"Value\":\"", post[] = "\"}\n";
    uint64_t o = 0; char num[24];
    for (uint64_t i = 0; i < r->nkeys; i++) {
        if (wco_ihash(r->keys[i], r->lens[i]) % nreduce != part) continue;
        int d = fmt_u64(r->counts[i], num);
        uint64_t len = (sizeof pre - 1) + r->lens[i] + (sizeof mid - 1) + (uint64_t)d + (sizeof post - 1);
        if (out) {
            uint8_t *p = out + o;
            memcpy(p, pre, sizeof pre - 1); p += sizeof pre - 1;
            memcpy(p, r->keys[i], r->lens[i]); p += r->lens[i];
            memcpy(p, mid, sizeof mid - 1); p += sizeof mid - 1;
            memcpy(p, num, (size_t)d); p += d;
            memcpy(p, post, sizeof post - 1);
        }
        o += len;
    }
    return o;
}

WCO_API void wco_free(wco_result *r) {
    if (!r) return;
    free(r->keys); free(r->lens); free(r->counts); free(r);
}

/* ---------------- exact check of a merged file against the input, for inputs too large for
 * wco_count (its per-thread tables, their merge and the final qsort take ~75 s per GiB of C4
 * text).  The merged file is parsed into a table of its lines (format "key: count\n" with a
 * decimal count > 0 and no leading zero, keys strictly ascending bytewise: Merge's sort.Strings
 * + "%s: %s\n", mapreduce.go:284-321), then the input is tokenized exactly as wco_count does
 * (FieldsFunc + IsLetter, wc.go:17-30) and every token decrements its line's count.  The file is
 * right iff every token finds its line and every count ends at 0: the same multiset of
 * (key, count) as the reference's, in the reference's order.  Returns 0, or an error code with
 * a message in msg. */
typedef struct { const uint8_t *key; uint32_t len; uint32_t hash; int64_t cnt; } vent_t;
typedef struct {
    const uint8_t *s; uint64_t n;
    vent_t *t; uint64_t mask;
    uint64_t tokens, missing, first_missing;
} vjob_t;

static vent_t *vfind(vent_t *t, uint64_t mask, const uint8_t *k, uint32_t len, uint32_t h) {
    for (uint64_t i = h & mask;; i = (i + 1) & mask) {
        vent_t *e = &t[i];
        if (!e->hash) return NULL;
        if (e->hash == h && e->len == len && memcmp(e->key, k, len) == 0) return e;
    }
}

static void vtoken(vjob_t *j, uint64_t start, uint32_t len) {
    const uint8_t *k = j->s + start;
    vent_t *e = vfind(j->t, j->mask, k, len, khash(k, len));
    j->tokens++;
    if (e) __atomic_fetch_sub(&e->cnt, 1, __ATOMIC_RELAXED);
    else if (j->missing++ == 0) j->first_missing = start;
}

static void *verify_job(void *arg) {
    vjob_t *j = (vjob_t *)arg;
    const uint8_t *s = j->s; uint64_t n = j->n, i = 0; int64_t start = -1;
    while (i < n) {
        uint8_t b = s[i];
        int w = 1, let;
        if (b < 0x80) let = ((uint32_t)(b | 0x20) - 'a') < 26u;
        else { uint32_t cp; w = decode_rune(s, n, i, &cp); let = letter_rune(cp); }
        if (let) { if (start < 0) start = (int64_t)i; }
        else if (start >= 0) { vtoken(j, (uint64_t)start, (uint32_t)(i - start)); start = -1; }
        i += w;
    }
    if (start >= 0) vtoken(j, (uint64_t)start, (uint32_t)(n - start));
    return NULL;
}

WCO_API int wco_verify_merged(const uint8_t *s, uint64_t n, const uint8_t *m, uint64_t mlen, int nthreads,
                              uint64_t *ntokens, uint64_t *nkeys, char *msg, uint64_t msgcap) {
    uint64_t lines = 0;
    for (uint64_t i = 0; i < mlen; i++) lines += m[i] == '\n';
    if (mlen && m[mlen - 1] != '\n') { snprintf(msg, msgcap, "merged file does not end in a newline"); return 1; }
    uint64_t cap = 1024; while (cap < 2 * lines + 2) cap <<= 1;
    vent_t *t = (vent_t *)calloc(cap, sizeof(vent_t));
    if (!t) { snprintf(msg, msgcap, "out of memory"); return 9; }
    const uint8_t *pk = NULL; uint32_t pl = 0;
    int rc = 0;
    for (uint64_t p = 0, ln = 0; p < mlen; ln++) {
        const uint8_t *nl = (const uint8_t *)memchr(m + p, '\n', mlen - p);
        const uint8_t *line = m + p; uint64_t L = (uint64_t)(nl - line);
        const uint8_t *colon = (const uint8_t *)memchr(line, ':', L);
        if (!colon || colon == line || (uint64_t)(colon - line) + 2 >= L || colon[1] != ' ') {
            snprintf(msg, msgcap, "line %llu: not \"key: count\"", (unsigned long long)ln); rc = 2; break;
        }
        uint32_t klen = (uint32_t)(colon - line);
        const uint8_t *d = colon + 2; uint64_t nd = L - klen - 2; int64_t c = 0;
        if (nd == 0 || nd > 19 || d[0] == '0') { snprintf(msg, msgcap, "line %llu: bad count", (unsigned long long)ln); rc = 2; break; }
        for (uint64_t q = 0; q < nd; q++) {
            if (d[q] < '0' || d[q] > '9') { rc = 2; break; }
            c = c * 10 + (d[q] - '0');
        }
        if (rc) { snprintf(msg, msgcap, "line %llu: bad count", (unsigned long long)ln); break; }
        if (pk) {
            uint32_t mm = pl < klen ? pl : klen;
            int cmp = memcmp(pk, line, mm);
            if (cmp > 0 || (cmp == 0 && pl >= klen)) {
                snprintf(msg, msgcap, "line %llu: keys not strictly ascending", (unsigned long long)ln); rc = 3; break;
            }
        }
        pk = line; pl = klen;
        uint32_t h = khash(line, klen);
        for (uint64_t i = h & (cap - 1);; i = (i + 1) & (cap - 1))
            if (!t[i].hash) { t[i].key = line; t[i].len = klen; t[i].hash = h; t[i].cnt = c; break; }
        p = (uint64_t)(nl - m) + 1;
    }
    if (!rc) {
        if (nthreads < 1) nthreads = 1;
        if (n < (1u << 20)) nthreads = 1;
        vjob_t *jobs = (vjob_t *)calloc((size_t)nthreads, sizeof(vjob_t));
        pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
        uint64_t pos = 0;
        for (int k = 0; k < nthreads; k++) {           /* cuts as in wco_count */
            uint64_t end = (k == nthreads - 1) ? n : (n / nthreads) * (uint64_t)(k + 1);
            if (end < pos) end = pos;
            while (end < n && end > pos) {
                uint8_t b = s[end - 1];
                if (b < 0x80 && !(((uint32_t)(b | 0x20) - 'a') < 26u)) break;
                end++;
            }
            jobs[k].s = s + pos; jobs[k].n = end - pos; jobs[k].t = t; jobs[k].mask = cap - 1;
            pos = end;
        }
        for (int k = 0; k < nthreads; k++) pthread_create(&th[k], NULL, verify_job, &jobs[k]);
        for (int k = 0; k < nthreads; k++) pthread_join(th[k], NULL);
        uint64_t tok = 0;
        for (int k = 0; k < nthreads; k++) {
            tok += jobs[k].tokens;
            if (jobs[k].missing && !rc) {
                snprintf(msg, msgcap, "%llu input tokens have no line (first at byte %llu)",
                         (unsigned long long)jobs[k].missing,
                         (unsigned long long)(jobs[k].first_missing + (uint64_t)(jobs[k].s - s)));
                rc = 4;
            }
        }
        if (ntokens) *ntokens = tok;
        if (nkeys) *nkeys = lines;
        for (uint64_t i = 0; !rc && i < cap; i++)
            if (t[i].hash && t[i].cnt != 0) {
                snprintf(msg, msgcap, "key %.*s: count off by %lld", (int)(t[i].len < 64 ? t[i].len : 64), t[i].key,
                         (long long)t[i].cnt);
                rc = 5;
            }
        free(jobs); free(th);
    }
    free(t);
    return rc;
}
