"""Pure-Python restatement of the reference word-count path.  TEST INFRASTRUCTURE ONLY.

This module is the small-input oracle: only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may import it, and only as a checker.  The product path
(`mit-6.824-2015_amd/`) never imports anything under `oracle/`.

Every function cites the reference line it restates (paths relative to /root/reference):

* tokenizer      - `Map`  src/main/wc.go:17-30  (strings.FieldsFunc(value, !unicode.IsLetter))
* UTF-8 decoding - Go `for _, r := range s` rune iteration used by FieldsFunc: invalid byte ->
                   U+FFFD width 1 (Go spec, "For statements with range clause"); accept ranges
                   of Go's unicode/utf8 (first byte class + second-byte accept range).
* letter test    - unicode.IsLetter = general category L, pinned to Unicode 13.0.0 via
                   `str.isalpha()` (== category L* for every code point, checked in
                   tools/gen_letter_table.py).
* ihash          - src/mapreduce/mapreduce.go:185-189 (hash/fnv New32a)
* Split          - src/mapreduce/mapreduce.go:141-179 (bufio.Scanner, 64 KiB token limit)
* DoMap          - src/mapreduce/mapreduce.go:193-231 (JSON line per token, partition ihash%R)
* DoReduce       - src/mapreduce/mapreduce.go:239-280 (decode, sort.Strings, Reduce, JSON)
* Reduce         - src/main/wc.go:35-38 (strconv.Itoa(values.Len()))
* Merge          - src/mapreduce/mapreduce.go:284-321 ("%s: %s\\n" in sort.Strings order)

Parity status: FNV-1a is pinned by the standard FNV-1a 32-bit test vectors; the merged-file
format and bytewise sort order are pinned by the reference's own `check()`
(src/mapreduce/test_test.go:45-83, restated in tests/test_oracle.py); the word-count top-10
golden (src/main/mr-testout.txt) pins ASCII tokenization + case sensitivity but its corpus
kjv12.txt is absent, so it only runs when that file is supplied.  Letter classification
beyond ASCII is restated from the Unicode 13.0.0 tables ("parity unpinned" by the reference's
own tests).
"""
from __future__ import annotations

import json
from typing import Dict, Iterable, List, Optional, Tuple

FNV32_OFFSET = 0x811C9DC5
FNV32_PRIME = 0x01000193
SCANNER_MAX_TOKEN = 64 * 1024  # bufio.MaxScanTokenSize, used by Split (mapreduce.go:164)


def _is_cont(b: int) -> bool:
    return 0x80 <= b <= 0xBF


def decode_rune(buf: bytes, i: int) -> Tuple[Optional[int], int]:
    """Go utf8.DecodeRune semantics at offset i: (code point or None for RuneError, width).

    Accept table of Go's unicode/utf8: C2-DF +1; E0 A0-BF +1; E1-EC,EE-EF 80-BF +1;
    ED 80-9F +1; F0 90-BF +2; F1-F3 80-BF +2; F4 80-8F +2; 00-7F ASCII; everything else
    (80-C1, F5-FF, truncated/invalid continuation) is RuneError of width 1.
    """
    n = len(buf)
    b0 = buf[i]
    if b0 < 0x80:
        return b0, 1
    if 0xC2 <= b0 <= 0xDF:
        w, lo, hi = 2, 0x80, 0xBF
    elif 0xE0 <= b0 <= 0xEF:
        w = 3
        lo, hi = (0xA0, 0xBF) if b0 == 0xE0 else ((0x80, 0x9F) if b0 == 0xED else (0x80, 0xBF))
    elif 0xF0 <= b0 <= 0xF4:
        w = 4
        lo, hi = (0x90, 0xBF) if b0 == 0xF0 else ((0x80, 0x8F) if b0 == 0xF4 else (0x80, 0xBF))
    else:
        return None, 1
    if i + 1 >= n or not (lo <= buf[i + 1] <= hi):
        return None, 1
    for k in range(2, w):
        if i + k >= n or not _is_cont(buf[i + k]):
            return None, 1
    if w == 2:
        cp = ((b0 & 0x1F) << 6) | (buf[i + 1] & 0x3F)
    elif w == 3:
        cp = ((b0 & 0x0F) << 12) | ((buf[i + 1] & 0x3F) << 6) | (buf[i + 2] & 0x3F)
    else:
        cp = ((b0 & 0x07) << 18) | ((buf[i + 1] & 0x3F) << 12) | ((buf[i + 2] & 0x3F) << 6) \
            | (buf[i + 3] & 0x3F)
    return cp, w


def is_letter(cp: Optional[int]) -> bool:
    """unicode.IsLetter (wc.go:19), Unicode 13.0.0. RuneError (None) is U+FFFD: not a letter."""
    if cp is None:
        return False
    if cp < 0x80:
        return (0x41 <= cp <= 0x5A) or (0x61 <= cp <= 0x7A)
    return chr(cp).isalpha()


def tokens(buf: bytes) -> List[bytes]:
    """strings.FieldsFunc(value, func(c) !unicode.IsLetter(c)) - wc.go:18-21.

    Maximal runs of letter runes, returned as byte slices of the input (tokens are always
    valid UTF-8 because every rune inside them decoded validly)."""
    out = []
    i = 0
    n = len(buf)
    start = -1
    while i < n:
        cp, w = decode_rune(buf, i)
        if is_letter(cp):
            if start < 0:
                start = i
        elif start >= 0:
            out.append(bytes(buf[start:i]))
            start = -1
        i += w
    if start >= 0:
        out.append(bytes(buf[start:n]))
    return out


def tokens_via_python_codec(buf: bytes) -> List[bytes]:
    """Independent second restatement (Python's strict UTF-8 codec with 'replace').

    Replacement characters are separators either way, so the token stream must equal
    `tokens()`; the tests cross-check the two."""
    s = buf.decode("utf-8", "replace")
    out, cur = [], []
    for ch in s:
        if ch != "�" and ch.isalpha():
            cur.append(ch)
        elif cur:
            out.append("".join(cur).encode("utf-8"))
            cur = []
    if cur:
        out.append("".join(cur).encode("utf-8"))
    return out


def ihash(key: bytes) -> int:
    """FNV-1a 32-bit, mapreduce.go:185-189."""
    h = FNV32_OFFSET
    for b in key:
        h ^= b
        h = (h * FNV32_PRIME) & 0xFFFFFFFF
    return h


def word_count(buf: bytes) -> Dict[bytes, int]:
    """Map (wc.go:17-30) + Reduce (wc.go:35-38) collapsed: key -> number of occurrences."""
    counts: Dict[bytes, int] = {}
    for t in tokens(buf):
        counts[t] = counts.get(t, 0) + 1
    return counts


def merged_output(counts: Dict[bytes, int]) -> bytes:
    """Merge's output file bytes: sort.Strings order (bytewise) + "%s: %s\\n"
    (mapreduce.go:305-319)."""
    return b"".join(k + b": " + str(counts[k]).encode() + b"\n" for k in sorted(counts))


def _json_line(key: bytes, value: str) -> bytes:
    # encoding/json of KeyValue{Key, Value}: {"Key":"...","Value":"..."}\n.  Letter-only keys
    # never need escaping (no quote, backslash, control, <>&, U+2028/2029).
    return b'{"Key":"' + key + b'","Value":"' + value.encode() + b'"}\n'


def res_file(counts: Dict[bytes, int], nreduce: int, r: int) -> bytes:
    """Bytes of mrtmp.<f>-res-<r> written by DoReduce (mapreduce.go:264-279) for wc."""
    keys = sorted(k for k in counts if ihash(k) % nreduce == r)
    return b"".join(_json_line(k, str(counts[k])) for k in keys)


def split(buf: bytes, nmap: int) -> List[bytes]:
    """Split (mapreduce.go:141-179): line scanner, new file when bytes written i > nchunk*m.

    bufio.ScanLines drops a trailing '\\r' before '\\n' and Split appends '\\n' to every line;
    a line longer than the scanner's 64 KiB buffer silently stops the scan (quirk P1)."""
    size = len(buf)
    nchunk = size // nmap + 1
    files = [bytearray()]
    m = 1
    i = 0
    pos = 0
    while pos < size:
        nl = buf.find(b"\n", pos)
        if nl < 0:
            line = buf[pos:]
            adv = size - pos
        else:
            line = buf[pos:nl]
            adv = nl - pos + 1
        # Scanner's buffer must hold the whole line including its '\n' (P1).
        if adv > SCANNER_MAX_TOKEN or (nl < 0 and len(line) >= SCANNER_MAX_TOKEN):
            break
        if line.endswith(b"\r"):
            line = line[:-1]
        if i > nchunk * m:
            files.append(bytearray())
            m += 1
        files[-1] += line + b"\n"
        i += len(line) + 1
        pos += adv
    return [bytes(f) for f in files]


# DoMap reads its split with ONE file.Read(b) of the split's size (mapreduce.go:205-207).  Go's
# os.File.Read on Linux passes at most 1 GiB to read(2) per call (internal/poll/fd_unix.go maxRW,
# Go 1.16-1.20 - the versions whose unicode tables restate Unicode 13, like this oracle's), and the
# error of the short read is nil, so a split larger than 1 GiB is mapped as its first 1 GiB
# followed by zero bytes; NUL is a separator, so that is exactly the token stream of the first
# 1 GiB alone (quirk P2).  `read_cap` is a parameter so tests can exercise the rule at small sizes.
DOMAP_READ_CAP = 1 << 30


def domap_read(split_bytes: bytes, read_cap: int = DOMAP_READ_CAP) -> bytes:
    """The bytes DoMap's single Read returns (P2): the first read_cap bytes of the split."""
    return split_bytes[:read_cap]


def map_files(split_bytes: bytes, nreduce: int) -> List[bytes]:
    """DoMap output files mrtmp.<f>-<m>-<r> (mapreduce.go:212-230): one JSON line per token."""
    outs = [bytearray() for _ in range(nreduce)]
    for t in tokens(split_bytes):
        outs[ihash(t) % nreduce] += _json_line(t, "1")
    return [bytes(o) for o in outs]


def run_single(buf: bytes, nmap: int, nreduce: int, read_cap: int = DOMAP_READ_CAP) -> Dict[str, object]:
    """RunSingle (mapreduce.go:344-356) restated in memory. Returns every artefact."""
    splits = split(buf, nmap)
    if len(splits) != nmap:
        raise RuntimeError("P3: Split created %d files for nMap=%d (DoMap would log.Fatal)"
                           % (len(splits), nmap))
    counts: Dict[bytes, int] = {}
    maps = []
    for s in splits:
        s = domap_read(s, read_cap)             # P2
        maps.append(map_files(s, nreduce))
        for t in tokens(s):
            counts[t] = counts.get(t, 0) + 1
    res = [res_file(counts, nreduce, r) for r in range(nreduce)]
    return {"splits": splits, "maps": maps, "res": res, "merged": merged_output(counts),
            "counts": counts}


def merge_res_files(res_files: Iterable[bytes]) -> bytes:
    """Merge (mapreduce.go:284-321) reading JSON lines back from res files."""
    kvs: Dict[bytes, bytes] = {}
    for data in res_files:
        for line in data.splitlines():
            if not line:
                continue
            obj = json.loads(line.decode("utf-8"))
            kvs[obj["Key"].encode("utf-8")] = obj["Value"].encode("utf-8")
    return b"".join(k + b": " + kvs[k] + b"\n" for k in sorted(kvs))


# ---------------------------------------------------------------------------------------------
# Generic MapReduce (arbitrary Map/Reduce), as exercised by src/mapreduce/test_test.go.  Used to
# pin Split / JSON intermediates / Merge formatting and sort order with the reference's own
# known-answer test `check()` (test_test.go:45-83).

def fields(value: bytes) -> List[bytes]:
    """strings.Fields: split on Unicode white space (ASCII subset suffices for test inputs)."""
    return value.split()


def run_single_generic(buf: bytes, nmap: int, nreduce: int, map_fn, reduce_fn) -> bytes:
    """RunSingle (mapreduce.go:344-356) with user Map/Reduce; returns the merged file bytes.

    map_fn(value: bytes) -> list of (key: bytes, value: str); reduce_fn(key, values) -> str."""
    splits = split(buf, nmap)
    if len(splits) != nmap:
        raise RuntimeError("P3: too few splits")
    # DoMap: per split, per reduce partition, JSON lines in list order (mapreduce.go:214-230)
    inter = [[[] for _ in range(nreduce)] for _ in range(nmap)]
    for m, s in enumerate(splits):
        for k, v in map_fn(s):
            inter[m][ihash(k) % nreduce].append((k, v))
    res_files = []
    for r in range(nreduce):                         # DoReduce (mapreduce.go:239-280)
        kvs: Dict[bytes, List[str]] = {}
        for m in range(nmap):
            for k, v in inter[m][r]:
                kvs.setdefault(k, []).append(v)
        res_files.append(b"".join(_json_line(k, reduce_fn(k, kvs[k])) for k in sorted(kvs)))
    return merge_res_files(res_files)                # Merge (mapreduce.go:284-321)


def reference_check(input_bytes: bytes, merged: bytes, n_number: int) -> None:
    """check() of test_test.go:45-83: sort the input lines with sort.Strings, output line i must
    parse (%d) to the same integer, and there must be exactly n_number output lines."""
    lines = sorted(input_bytes.split(b"\n")[:-1] if input_bytes.endswith(b"\n") else input_bytes.split(b"\n"))
    out = merged.split(b"\n")
    if out and out[-1] == b"":
        out = out[:-1]
    for i, text in enumerate(out):
        v1 = int(lines[i].split()[0])
        v2 = int(text.split(b":")[0])
        if v1 != v2:
            raise AssertionError(f"line {i}: {v1} != {v2}")
    if len(out) != n_number:
        raise AssertionError(f"Expected {n_number} lines in output")
