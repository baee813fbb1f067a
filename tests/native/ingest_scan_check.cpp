// CPU check of wcg_scan.h (tests/test_ingest_scan.py): the windowed scan_slice against the
// per-line scan_slice_lines, through the caller's cut rule (wcg_api.hip wcg_map_file), on random
// chunks whose lines are short, near 64 KiB or far past it, split into 1-16 reader slices.
#include <cstdio>
#include <random>
#include <vector>

#include "wcg_scan.h"

using namespace wcg;

template <class F>
static void cut_of(const uint8_t* h, uint64_t carry, uint64_t want, int T, bool eof, F scan, uint64_t& cut,
                   bool& stop) {
    std::vector<SliceLines> sl(T);
    for (int t = 0; t < T; t++) {
        const uint64_t a = carry + want * t / T, b = carry + want * (t + 1) / T;
        sl[t] = scan(h, (int64_t)a, (int64_t)b);
    }
    const uint64_t len = carry + want;
    stop = eof;
    int64_t prev = -1, bad = -1;
    for (int t = 0; t < T && bad < 0; t++) {
        if (sl[t].first < 0) continue;
        if (sl[t].first - (prev + 1) >= (int64_t)SCAN_MAX_LINE) { bad = prev + 1; break; }
        if (sl[t].bad >= 0) { bad = sl[t].bad; break; }
        prev = sl[t].last;
    }
    if (bad < 0 && (int64_t)len - (prev + 1) >= (int64_t)SCAN_MAX_LINE) bad = prev + 1;
    if (bad >= 0) { cut = (uint64_t)bad; stop = true; }
    else cut = eof ? len : (uint64_t)(prev + 1);
}

int main() {
    std::mt19937_64 rng(7);
    std::vector<uint8_t> buf(3 << 20);
    long fails = 0, tests = 0;
    for (int it = 0; it < 1500; it++) {
        size_t n = 0;
        const int mode = it % 5;
        while (n < buf.size()) {
            size_t L;
            const uint64_t r = rng() % 1000;
            if (mode == 0) L = rng() % 200;
            else if (r < 3) L = 65534 + rng() % 4;
            else if (r < 5) L = 65536 + rng() % 200000;
            else L = rng() % (mode == 3 ? 40000 : mode == 4 ? 65535 : 300);
            for (size_t k = 0; k < L && n < buf.size(); k++) buf[n++] = (uint8_t)('a' + k % 26);
            if (n < buf.size()) buf[n++] = '\n';
        }
        for (int q = 0; q < 5; q++) {
            const uint64_t carry = rng() % 70000, want = rng() % (buf.size() - carry);
            const int T = 1 + (int)(rng() % 16);
            const bool eof = rng() & 1;
            uint64_t c1, c2;
            bool s1, s2;
            cut_of(buf.data(), carry, want, T, eof, scan_slice, c1, s1);
            cut_of(buf.data(), carry, want, T, eof, scan_slice_lines, c2, s2);
            tests++;
            if (c1 != c2 || s1 != s2) {
                if (fails < 5) printf("mismatch carry=%llu want=%llu T=%d: %llu/%d vs %llu/%d\n", (unsigned long long)carry,
                                      (unsigned long long)want, T, (unsigned long long)c1, s1, (unsigned long long)c2, s2);
                fails++;
            }
        }
    }
    printf("tests %ld mismatches %ld\n", tests, fails);
    return fails != 0;
}
