/*
 * gencorpus.c - deterministic synthetic corpora for the word-count configs of SURVEY.md 8(d).
 *
 * The reference's Part I corpus (kjv12.txt) is absent, so every benchmark input is synthetic:
 *   ascii (C2/C3): vocabulary of V distinct words over [a-z], 10% capitalised (distinct keys),
 *                  length 1+Poisson(4) clipped to [1,20]; Zipf(s) over rank; separators
 *                  ' ' 85%, one of ", " ". " "; " "'" "-" 12%, a digit run 3%; '\n' once the
 *                  line reaches 72+U(0,16) bytes.
 *   utf8  (C4):    words drawn from ASCII, Latin-1, Greek, Cyrillic, CJK (3-byte), Hangul and
 *                  CJK Ext-B (4-byte) letters - all category L in Unicode 13.0 (and later);
 *                  separators add combining marks, emoji, U+FFFD and ~0.1% invalid UTF-8.
 *
 * The output is cut into 1 MiB blocks, each generated from its own RNG stream
 * (seed, block index) and ending in '\n', so any byte range that starts on a block boundary
 * can be generated independently (one rank = one range) and by many threads.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define API __attribute__((visibility("default")))
#define BLOCK (1u << 20)

typedef struct { uint64_t s[4]; } rng_t;              /* xoshiro256** */
static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static inline uint64_t rnext(rng_t *r) {
    uint64_t *s = r->s, res = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return res;
}
static uint64_t splitmix(uint64_t *x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static void rseed(rng_t *r, uint64_t a, uint64_t b) {
    uint64_t x = a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull);
    for (int i = 0; i < 4; i++) r->s[i] = splitmix(&x);
}
static inline double runif(rng_t *r) { return (rnext(r) >> 11) * (1.0 / 9007199254740992.0); }
static inline uint32_t rbelow(rng_t *r, uint32_t n) { return (uint32_t)(((rnext(r) >> 32) * (uint64_t)n) >> 32); }

static int poisson(rng_t *r, double lam) {
    double L = exp(-lam), p = 1.0; int k = 0;
    do { k++; p *= runif(r); } while (p > L);
    return k - 1;
}

static int put_utf8(uint8_t *o, uint32_t cp) {
    if (cp < 0x80) { o[0] = (uint8_t)cp; return 1; }
    if (cp < 0x800) { o[0] = 0xC0 | (cp >> 6); o[1] = 0x80 | (cp & 0x3F); return 2; }
    if (cp < 0x10000) { o[0] = 0xE0 | (cp >> 12); o[1] = 0x80 | ((cp >> 6) & 0x3F); o[2] = 0x80 | (cp & 0x3F); return 3; }
    o[0] = 0xF0 | (cp >> 18); o[1] = 0x80 | ((cp >> 12) & 0x3F); o[2] = 0x80 | ((cp >> 6) & 0x3F); o[3] = 0x80 | (cp & 0x3F);
    return 4;
}

/* letter code point from one script; all ranges are category L in Unicode 13.0 */
static uint32_t script_letter(rng_t *r, int script, int first) {
    switch (script) {
    case 0: return (first && rbelow(r, 10) == 0 ? 'A' : 'a') + rbelow(r, 26);   /* unused: ascii words built separately */
    case 1: { uint32_t v = rbelow(r, 23 + 31 + 8); return v < 23 ? 0xC0 + v : (v < 54 ? 0xD8 + (v - 23) : 0xF8 + (v - 54)); }
    case 2: return first && rbelow(r, 4) == 0 ? 0x391 + (rbelow(r, 24) + 0) + 0 : 0x3B1 + rbelow(r, 25); /* 0x391..0x3A8 (skip 3A2 below) */
    case 3: return 0x410 + rbelow(r, 64);                                        /* U+0410..U+044F */
    case 4: return 0x4E00 + rbelow(r, 0x9FFC - 0x4E00 + 1);                       /* CJK unified (13.0 range) */
    case 5: return 0xAC00 + rbelow(r, 0xD7A3 - 0xAC00 + 1);                       /* Hangul syllables */
    default: return 0x20000 + rbelow(r, 0x2A6DD - 0x20000 + 1);                  /* CJK Ext B */
    }
}

typedef struct {
    int mode;
    uint64_t vocab;
    double zipf_s;
    uint64_t seed;
    /* built */
    uint8_t *words; uint64_t *off; uint32_t *len;
    double *prob; uint32_t *alias;
} gen_t;

static uint64_t h64(const uint8_t *p, uint32_t n) { uint64_t h = 1469598103934665603ull; for (uint32_t i = 0; i < n; i++) { h ^= p[i]; h *= 1099511628211ull; } return h; }

API void *wcgen_create(int mode, uint64_t vocab, double zipf_s, uint64_t seed) {
    gen_t *g = (gen_t *)calloc(1, sizeof(gen_t));
    g->mode = mode; g->vocab = vocab; g->zipf_s = zipf_s; g->seed = seed;
    uint64_t cap = vocab * (mode ? 40 : 21) + 64;
    g->words = (uint8_t *)malloc(cap); g->off = (uint64_t *)malloc(vocab * 8); g->len = (uint32_t *)malloc(vocab * 4);
    uint64_t tcap = 1; while (tcap < vocab * 2) tcap <<= 1;
    uint64_t *tab = (uint64_t *)calloc(tcap, 8);                  /* index+1 of stored word */
    rng_t r; rseed(&r, seed, 0xC0FFEEull);
    uint64_t pos = 0;
    /* Candidates come from one RNG stream whatever is accepted (a duplicate just draws the next
     * candidate), so they are generated PF ahead of the dedupe and their table slots prefetched:
     * the 1 GB table's random probes otherwise dominate (C4: 7.4e7 candidates). */
    enum { PF = 64 };
    struct cand { uint8_t buf[96]; uint32_t n; uint64_t h; } *ring = (struct cand *)malloc(PF * sizeof(struct cand));
    #define GEN_CAND(C) do {                                                                         \
        struct cand *c_ = (C); uint32_t n = 0; uint8_t *buf = c_->buf;                               \
        if (mode == 0) {                                                                             \
            int L = 1 + poisson(&r, 4.0); if (L > 20) L = 20;                                        \
            int cap1 = rbelow(&r, 10) == 0;                                                          \
            for (int k = 0; k < L; k++) buf[n++] = (uint8_t)((k == 0 && cap1 ? 'A' : 'a') + rbelow(&r, 26)); \
        } else {                                                                                     \
            uint32_t pick = rbelow(&r, 100);                                                         \
            int script = pick < 40 ? 0 : pick < 50 ? 1 : pick < 60 ? 2 : pick < 70 ? 3 : pick < 85 ? 4 : pick < 95 ? 5 : 6; \
            int L = 1 + poisson(&r, script >= 4 ? 1.5 : 4.0); if (L > 12) L = 12;                    \
            int cap1 = rbelow(&r, 10) == 0;                                                          \
            for (int k = 0; k < L; k++) {                                                            \
                if (script == 0) buf[n++] = (uint8_t)((k == 0 && cap1 ? 'A' : 'a') + rbelow(&r, 26)); \
                else {                                                                               \
                    uint32_t cp = script_letter(&r, script, k == 0);                                 \
                    if (cp == 0x3A2) cp = 0x3A3;                        /* U+03A2 is unassigned */   \
                    n += (uint32_t)put_utf8(buf + n, cp);                                            \
                }                                                                                    \
            }                                                                                        \
        }                                                                                            \
        c_->n = n; c_->h = h64(buf, n);                                                              \
        __builtin_prefetch(&tab[c_->h & (tcap - 1)], 1);                                             \
    } while (0)
    for (int k = 0; k < PF; k++) GEN_CAND(&ring[k]);
    for (uint64_t i = 0, head = 0; i < vocab; head = (head + 1) % PF) {
        struct cand *c = &ring[head];
        uint64_t s = c->h & (tcap - 1);
        int dup = 0;
        while (tab[s]) {
            uint64_t j = tab[s] - 1;
            if (g->len[j] == c->n && memcmp(g->words + g->off[j], c->buf, c->n) == 0) { dup = 1; break; }
            s = (s + 1) & (tcap - 1);
        }
        if (!dup) {
            tab[s] = i + 1;
            memcpy(g->words + pos, c->buf, c->n); g->off[i] = pos; g->len[i] = c->n; pos += c->n; i++;
        }
        GEN_CAND(c);                     /* the candidate PF places later in the stream */
    }
    #undef GEN_CAND
    free(ring);
    free(tab);
    /* Vose alias table for Zipf(s) over rank 1..V */
    double *p = (double *)malloc(vocab * sizeof(double)), sum = 0;
    for (uint64_t i = 0; i < vocab; i++) { p[i] = pow((double)(i + 1), -zipf_s); sum += p[i]; }
    g->prob = (double *)malloc(vocab * sizeof(double)); g->alias = (uint32_t *)malloc(vocab * 4);
    uint32_t *small = (uint32_t *)malloc(vocab * 4), *large = (uint32_t *)malloc(vocab * 4);
    uint64_t ns = 0, nl = 0;
    for (uint64_t i = 0; i < vocab; i++) { p[i] = p[i] * (double)vocab / sum; if (p[i] < 1.0) small[ns++] = (uint32_t)i; else large[nl++] = (uint32_t)i; }
    while (ns && nl) {
        uint32_t s = small[--ns], l = large[--nl];
        g->prob[s] = p[s]; g->alias[s] = l;
        p[l] = (p[l] + p[s]) - 1.0;
        if (p[l] < 1.0) small[ns++] = l; else large[nl++] = l;
    }
    while (nl) { uint32_t l = large[--nl]; g->prob[l] = 1.0; g->alias[l] = l; }
    while (ns) { uint32_t s = small[--ns]; g->prob[s] = 1.0; g->alias[s] = s; }
    free(p); free(small); free(large);
    return g;
}

API void wcgen_destroy(void *vg) {
    gen_t *g = (gen_t *)vg; if (!g) return;
    free(g->words); free(g->off); free(g->len); free(g->prob); free(g->alias); free(g);
}

API uint64_t wcgen_word(void *vg, uint64_t i, uint8_t *out) {
    gen_t *g = (gen_t *)vg; memcpy(out, g->words + g->off[i], g->len[i]); return g->len[i];
}

static inline uint32_t sample(gen_t *g, rng_t *r) {
    uint32_t i = rbelow(r, (uint32_t)g->vocab);
    return runif(r) < g->prob[i] ? i : g->alias[i];
}

/* separator after a word; returns bytes written (<= 16) */
static int put_sep(gen_t *g, rng_t *r, uint8_t *o, int newline) {
    if (newline) { o[0] = '\n'; return 1; }
    uint32_t u = rbelow(r, 1000);
    if (g->mode == 1 && u < 120) {
        uint32_t v = rbelow(r, 120);
        if (v < 30) { int n = put_utf8(o, 0x300 + rbelow(r, 0x70)); o[n] = ' '; return n + 1; }   /* combining mark (Mn) */
        if (v < 60) { int n = put_utf8(o, 0x1F600 + rbelow(r, 0x50)); o[n] = ' '; return n + 1; } /* emoji (So) */
        if (v < 80) { o[0] = ' '; int n = put_utf8(o + 1, 0xFFFD); return n + 1; }
        if (v < 100) { o[0] = 0xE3; o[1] = 0x80; o[2] = 0x80; return 3; }                          /* U+3000 ideographic space */
        if (v < 119) { o[0] = ','; o[1] = ' '; return 2; }
        /* ~0.1%: invalid UTF-8 */
        switch (rbelow(r, 6)) {
        case 0: o[0] = 0x80; return 1;
        case 1: o[0] = 0xFF; return 1;
        case 2: o[0] = 0xC0; o[1] = 0xAF; return 2;
        case 3: o[0] = 0xED; o[1] = 0xA0; o[2] = 0x80; return 3;
        case 4: o[0] = 0xE4; o[1] = 0xB8; o[2] = ' '; return 3;                                   /* truncated 3-byte */
        default: o[0] = 0xF0; o[1] = 0x9F; o[2] = 0x98; o[3] = '.'; return 4;                    /* truncated 4-byte */
        }
    }
    if (u < 850) { o[0] = ' '; return 1; }
    if (u < 970) {
        switch (rbelow(r, 5)) {
        case 0: o[0] = ','; o[1] = ' '; return 2;
        case 1: o[0] = '.'; o[1] = ' '; return 2;
        case 2: o[0] = ';'; o[1] = ' '; return 2;
        case 3: o[0] = '\''; return 1;
        default: o[0] = '-'; return 1;
        }
    }
    int nd = 1 + (int)rbelow(r, 4); o[0] = ' ';
    for (int k = 0; k < nd; k++) o[1 + k] = (uint8_t)('0' + rbelow(r, 10));
    o[1 + nd] = ' ';
    return nd + 2;
}

static void gen_block(gen_t *g, uint8_t *o, uint64_t n, uint64_t block_index) {
    rng_t r; rseed(&r, g->seed, block_index + 1);
    uint64_t p = 0; uint32_t linelen = 0, target = 72 + rbelow(&r, 17);
    if (n == 0) return;
    while (1) {
        uint32_t w = sample(g, &r);
        uint32_t L = g->len[w];
        uint8_t sep[24]; int nl = (linelen + L >= target);
        int sl = put_sep(g, &r, sep, nl);
        if (p + L + (uint64_t)sl + 1 > n) break;                 /* keep room for the final '\n' */
        memcpy(o + p, g->words + g->off[w], L); p += L;
        memcpy(o + p, sep, (size_t)sl); p += (uint64_t)sl;
        linelen += L + (uint32_t)sl;
        if (nl) { linelen = 0; target = 72 + rbelow(&r, 17); }
    }
    while (p < n - 1) o[p++] = ' ';
    o[n - 1] = '\n';
}

typedef struct { gen_t *g; uint8_t *out; uint64_t n, first_block; int tid, nthreads; } gjob_t;
static void *gen_worker(void *a) {
    gjob_t *j = (gjob_t *)a;
    uint64_t nb = (j->n + BLOCK - 1) / BLOCK;
    for (uint64_t b = (uint64_t)j->tid; b < nb; b += (uint64_t)j->nthreads) {
        uint64_t len = (b + 1) * BLOCK <= j->n ? BLOCK : j->n - b * BLOCK;
        gen_block(j->g, j->out + b * BLOCK, len, j->first_block + b);
    }
    return NULL;
}

/* Fill out[0:n) with blocks first_block, first_block+1, ... (1 MiB each; a short last block). */
API int wcgen_fill(void *vg, uint8_t *out, uint64_t n, uint64_t first_block, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    pthread_t th[256]; gjob_t jobs[256];
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (gjob_t){ (gen_t *)vg, out, n, first_block, t, nthreads };
        pthread_create(&th[t], NULL, gen_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    return 0;
}

API uint64_t wcgen_block_bytes(void) { return BLOCK; }
