// wcg_scan.h - Split's line structure of one reader slice (host code, no HIP: the CPU suite
// compiles it directly, tests/test_ingest_scan.py).  mapreduce.go:141-179 splits with a
// bufio.Scanner: a line whose bytes plus '\n' exceed bufio.MaxScanTokenSize ends the input (P1).
#pragma once
#ifndef _GNU_SOURCE
#define _GNU_SOURCE 1                 // memrchr
#endif
#include <algorithm>
#include <cstdint>
#include <cstring>

namespace wcg {

constexpr uint64_t SCAN_MAX_LINE = 65536;   // bufio.MaxScanTokenSize: a line + '\n' must fit

// '\n' structure of one reader slice [a, b) of a chunk
struct SliceLines {
    int64_t first = -1, last = -1;   // first / last '\n' in the slice (-1: none)
    int64_t bad = -1;                // start of the first over-long line wholly inside the slice
};

// r04: from line start L, the last '\n' of the window [L, L + SCAN_MAX_LINE) is the next line
// start to test (memrchr over 64 KiB, every byte looked at about once); a window without one is an
// over-long line.  The first form called memchr once per line (~1e6 calls per 64 MiB chunk: the
// scan, not the read, set the ingest's pace: profiles/r04_ingest_*).
inline SliceLines scan_slice(const uint8_t* p, int64_t a, int64_t b) {
    SliceLines s;
    if (a >= b) return s;
    const void* q = memchr(p + a, '\n', (size_t)(b - a));
    if (!q) return s;
    s.first = (const uint8_t*)q - p;
    int64_t last = s.first, L = s.first + 1;
    while (L < b) {
        const int64_t w = std::min<int64_t>(L + (int64_t)SCAN_MAX_LINE, b);
        const void* r = memrchr(p + L, '\n', (size_t)(w - L));
        if (!r) {
            if (L + (int64_t)SCAN_MAX_LINE <= b) s.bad = L;   // SCAN_MAX_LINE bytes, no '\n'
            break;
        }
        last = (const uint8_t*)r - p;
        L = last + 1;
    }
    s.last = last;
    return s;
}

// the r03 form (per-line memchr), kept as the reference of tests/test_ingest_scan.py
inline SliceLines scan_slice_lines(const uint8_t* p, int64_t a, int64_t b) {
    SliceLines s;
    int64_t prev = -1;
    for (int64_t i = a; i < b;) {
        const void* q = memchr(p + i, '\n', (size_t)(b - i));
        if (!q) break;
        const int64_t nl = (const uint8_t*)q - p;
        if (s.first < 0) s.first = nl;
        else if (s.bad < 0 && nl - (prev + 1) >= (int64_t)SCAN_MAX_LINE) s.bad = prev + 1;
        prev = nl;
        i = nl + 1;
    }
    s.last = prev;
    return s;
}

}  // namespace wcg
