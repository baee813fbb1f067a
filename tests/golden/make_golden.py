#!/usr/bin/env python3
"""Regenerate tests/golden/ from the pure-Python restatement (oracle/wc_ref.py).

Each case = <name>.in (input bytes) + <name>.json (expected merged file, the -res-<r> files
for a few nReduce, token count, FNV of keys).  The reference itself cannot run here (Go is
absent); the restatement is pinned by the FNV-1a KATs, the reference's own
check() of test_test.go (tests/test_oracle.py) and mr-testout.txt when kjv12.txt is supplied.
Usage: python3 tests/golden/make_golden.py
"""
import base64
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import wc_ref  # noqa: E402


def case_inputs():
    c = {}
    c["empty"] = b""
    c["no_letters"] = b"0123 456, 789.\n\n  --- ;;; \r\n\t\x00\x01"
    c["one_word"] = b"hello"
    c["basic"] = b"the quick brown fox jumps over the lazy dog\nThe dog, the fox; the END.\n"
    c["case_pairs"] = b"And and AND aNd and And\n" * 7
    c["crlf"] = b"alpha beta\r\ngamma\r\r\ndelta\r\n\r\nalpha\r"
    c["punct_digits"] = b"it's co-op x1y2z3 a_b a.b.c 42nd 3rd-rate don't\n"
    c["nul_bytes"] = b"ab\x00cd\x00\x00ab\x00\n\x00ef"
    c["latin1"] = "café naïve Ærø ªº µ ÿ façade ×÷ Œuvre\n".encode()
    c["cjk_mixed"] = "中文字 和 한국어 日本語テキスト abcДЖ ΑΒΓαβγ\n".encode()
    c["smp_letters"] = "𠀀𠀁 𪛝x 𝒜𝒞 𐐀𐐨 🙂smile🙂 \n".encode()
    c["combining"] = "école résumé ño äb\n".encode()
    c["invalid_utf8"] = (b"ab\x80cd \xff ef\xc0\xafgh \xed\xa0\x80ij \xe4\xb8 kl \xf0\x9f\x98 mn "
                         b"\xc3 \xc3\xa9t\xc3\xa9 \xe0\x80\x80x \xf4\x90\x80\x80y \xf5z\n")
    c["surrogate_overlong"] = b"\xed\xbf\xbfA \xc1\xbfB \xe0\x9f\xbfC \xf0\x8f\xbf\xbfD\n"
    c["long_tokens"] = (b"a" * 15 + b" " + b"b" * 16 + b" " + b"c" * 17 + b" " + b"d" * 64 + b" " +
                        b"e" * 300 + b"\n" + b"x" * 15 + b"y" + b" " + b"x" * 15 + b"z" + b" " + b"x" * 15 + b"y\n")
    c["long_tie_prefix"] = b" ".join(b"abcdefghijklmnop" + s for s in
                                     [b"", b"q", b"a", b"qq", b"zz", b"", b"\xc3\xa9", b"a"]) + b"\n"
    c["unicode_long"] = ("ǅǈǋ" * 9 + " " + "キャラクター" * 4 + "\n").encode()
    c["no_trailing_newline"] = b"last word"
    c["only_newlines"] = b"\n" * 40
    c["tab_sep"] = b"a\tb\tc\ta\x0bb\x0cc\n"
    return c


def main():
    cases = case_inputs()
    for name, data in cases.items():
        counts = wc_ref.word_count(data)
        assert wc_ref.tokens(data) == wc_ref.tokens_via_python_codec(data), name
        exp = {
            "name": name,
            "input_b64": base64.b64encode(data).decode(),
            "ntokens": sum(counts.values()),
            "nkeys": len(counts),
            "merged_b64": base64.b64encode(wc_ref.merged_output(counts)).decode(),
            "res": {str(R): [base64.b64encode(wc_ref.res_file(counts, R, r)).decode() for r in range(R)]
                    for R in (1, 3, 7)},
        }
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(exp, f, indent=1, sort_keys=True)
            f.write("\n")
    # FNV-1a 32 known answers (standard test vectors + SURVEY.md 8(a) row 7)
    kat = {k: wc_ref.ihash(k.encode()) for k in ["", "a", "foobar", "the", "and", "And", "of", "über"]}
    with open(os.path.join(HERE, "fnv1a32_kat.json"), "w") as f:
        json.dump(kat, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"wrote {len(cases)} cases")


if __name__ == "__main__":
    main()
