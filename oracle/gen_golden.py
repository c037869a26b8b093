"""Generate the golden fixtures under tests/golden/ by RUNNING THE REFERENCE.

Test infrastructure, build container only (needs /root/reference).  Re-run with
``python oracle/gen_golden.py`` — outputs are deterministic.

Writes
  tests/golden/kat.json    — SURVEY.md Appendix B known-answer probes
  tests/golden/fuzz.json   — randomized small SAMs hitting every CIGAR op, the
                             maxdel rule, insertions, fill/min-depth, wrapping,
                             thresholds and the reference's error classes
  tests/golden/amb.json    — the reference's IUPAC dict (sam2consensus.py:317-329),
                             extracted from its source as DATA via ast.literal_eval
Each case = {"name", "sam", "args", "status", "files"}; status is "ok" or the
exception class the reference raised (then no files are written).
"""
from __future__ import annotations

import ast
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness  # noqa: E402

GOLD = os.path.join(os.path.dirname(HERE), "tests", "golden")


def rec(rname, pos, cigar, seq, qname="r"):
    return "%s\t0\t%s\t%s\t60\t%s\t*\t0\t0\t%s\t*\n" % (qname, rname, pos, cigar, seq)


def sam(refs, reads, hd=True):
    s = "@HD\tVN:1.0\tSO:unsorted\n" if hd else ""
    for n, L in refs:
        s += "@SQ\tSN:%s\tLN:%d\n" % (n, L)
    for r in reads:
        s += rec(*r)
    return s


def kat_cases():
    C = []

    def add(name, text, args):
        C.append({"name": name, "sam": text, "args": args})

    add("tiny", sam([("g1", 10)], [("g1", 1, "3M2I3M", "AAACCGGG"), ("g1", 2, "4M", "AATG")]), ["-p", "t"])
    md = sam([("g", 7)], [("g", 1, "2M3D2M", "AAAA"), ("g", 1, "7M", "CCCCCCC")])
    add("maxdel_default", md, [])
    add("maxdel_d2", md, ["-d", "2"])
    add("maxdel_d0", md, ["-d", "0"])
    big = sam([("g", 160)], [("g", 1, "2M152D2M", "AAAA"), ("g", 1, "156M", "C" * 156)])
    add("maxdel_big_default", big, [])
    add("maxdel_big_d150", big, ["-d", "150"])
    add("round_tie", sam([("g", 8)], [("g", 1, "8M", "A" * 8), ("g", 1, "1M", "A")]), [])
    add("negdash", sam([("g", 6)], [("g", 1, "3M2I", "AAACC"), ("g", 1, "3M2I", "AAACC"),
                                    ("g", 1, "3M2I", "AAAGG"), ("g", 4, "1M", "T")]), [])
    add("ins_multi", sam([("g", 8)], [("g", 1, "4M3I4M", "AAAACGTCCCC"), ("g", 1, "4M1I4M", "AAAACCCCC"),
                                      ("g", 1, "4M1I4M", "AAAAGCCCC"), ("g", 1, "8M", "AAAACCCC")]),
        ["-c", ".25,.5,.75"])
    add("ins_mindepth", sam([("g", 8)], [("g", 1, "4M2I", "AAAATT"), ("g", 4, "5M", "CCCCC")]), ["-m", "2"])
    add("dash_thr", sam([("g", 3)], [("g", 1, "1M1D1M", "AA")] * 3 + [("g", 1, "3M", "ACA")]), ["-c", ".25,.9"])
    add("np_ops", sam([("g", 10)], [("g", 1, "2M2N2M1P2M", "AACCGG"), ("g", 1, "9M", "T" * 9)]), [])
    add("sclip", sam([("g", 6)], [("g", 2, "2S2I3M", "TTGGAAA"), ("g", 1, "6M", "CAAACC")]), [])
    add("cig_garbage", sam([("g", 6)], [("g", 1, "003M?2M", "ACGTA")]), [])
    add("seqshort", sam([("g", 9)], [("g", 1, "5M3D2M", "ACGT"), ("g", 1, "9M", "T" * 9)]), ["-c", ".9"])
    add("pos0", sam([("g", 4)], [("g", 0, "2M", "AC")]), [])
    add("mindepth", sam([("g", 4)], [("g", 1, "4M", "AAAA"), ("g", 1, "2M", "AA")]), ["-m", "2", "-f", "N"])
    wr = sam([("g", 7)], [("g", 1, "7M", "ACGTACG")])
    add("wrap", wr, ["-n", "3", "-c", ".25,.5"])
    add("wrapneg", wr, ["-n", "-3"])
    add("t029", wr, ["-c", "0.29,0.57,1.0,0.25,0.25"])
    add("onlydel2", sam([("g", 3), ("h", 3)], [("g", 1, "1S1D", "AA"), ("h", 1, "3M", "ACG")]), [])
    add("err_acgnt", sam([("g", 1)], [("g", 1, "1M", b) for b in "ACGNT"]), ["-c", ".5"])
    add("err_t0", wr, ["-c", "0"])
    add("err_past_end", sam([("g", 4)], [("g", 3, "3M", "ACG")]), [])
    add("err_ins_at_end", sam([("g", 4)], [("g", 2, "3M2I", "ACGTT")]), [])
    add("err_lowercase", sam([("g", 4)], [("g", 1, "3M", "AcG")]), [])
    add("multifill", sam([("g", 6)], [("g", 2, "2M", "AC"), ("g", 5, "1M", "T")]), ["-f", "XY"])
    add("emptyfill_zero_len", sam([("g", 3)], [("g", 1, "1M", "A")]), ["-f", "", "-m", "5"])
    add("unknown_ref", sam([("g", 4)], [("q", 1, "2M", "AC")]), [])
    add("unmapped_star", sam([("g", 4)], [("g", 1, "*", "AC"), ("g", 2, "2M", "GT")]), [])
    add("two_refs_one_empty", sam([("a", 5), ("b", 5)], [("b", 1, "5M", "ACGTN")]), ["-c", "0.5,0.75"])
    add("gz_prefix", sam([("g", 5)], [("g", 1, "5M", "ACGTA")]), ["-p", "sample.x"])
    return C


# ----------------------------------------------------------------- fuzz cases
OPS = "MMMMMMIDNSHPX="


def rand_cigar(rng, L):
    ops = []
    for _ in range(rng.randint(1, 4)):
        ops.append((rng.choice(OPS), rng.randint(1, 4)))
    s = "".join("%d%s" % (n, o) for o, n in ops)
    if rng.random() < 0.03:
        s = s[:1] + "?" + s[1:]
    if rng.random() < 0.02:
        s = "0" + s
    return s, ops


def rand_seq(rng, ops):
    q = sum(n for o, n in ops if o in "MIS=X")
    r = rng.random()
    if r < 0.06:
        q = max(0, q - rng.randint(1, 4))
    elif r < 0.09:
        q += rng.randint(1, 3)
    alpha = "ACGT" * 6 + "N"
    s = [rng.choice(alpha) for _ in range(q)]
    for i in range(len(s)):
        x = rng.random()
        if x < 0.004:
            s[i] = "-"
        elif x < 0.006:
            s[i] = "a"
    return "".join(s)


def fuzz_case(rng, k):
    nref = rng.randint(1, 3)
    refs = [("g%d" % i, rng.randint(1, 30) if rng.random() < 0.15 else rng.randint(10, 30)) for i in range(nref)]
    reads = []
    depth_bias = rng.random() < 0.5
    for _ in range(rng.randint(0, 14 if depth_bias else 7)):
        rn, L = rng.choice(refs)
        if rng.random() < 0.015:
            rn = "zz"
        cig, ops = rand_cigar(rng, L)
        span = sum(n for o, n in ops if o in "MDNP=X")
        hi = max(1, L - span + 1)
        pos = rng.randint(1, hi)
        if rng.random() < 0.03:
            pos = 0
        if rng.random() < 0.02:
            pos = L + 1
        if rng.random() < 0.01:
            cig = "*"
        if ops[-1][0] == "I" and rng.random() < 0.7:
            cig, ops = cig + "1M", ops + [("M", 1)]
        reads.append((rn, pos, cig, rand_seq(rng, ops)))
    args = []
    th = rng.choice([None, "0.25", "0.5", "0.75", "0.25,0.5,0.75", "0.1,0.9", "1.0", "0.33,0.66",
                     "0.29", "0.6,0.25", "1.5"])
    if th:
        args += ["-c", th]
    if rng.random() < 0.25:
        args += ["-m", str(rng.choice([0, 2, 3]))]
    if rng.random() < 0.2:
        args += ["-f", rng.choice(["N", "-", "XY", "?"])]
    if rng.random() < 0.25:
        args += ["-d", rng.choice(["150", "2", "0"])]
    if rng.random() < 0.15:
        args += ["-n", str(rng.choice([3, 5, -2]))]
    text = sam(refs, reads, hd=rng.random() < 0.7)
    if rng.random() < 0.03:
        text += "\n"                     # trailing blank line → IndexError at :195
    return {"name": "fuzz%04d" % k, "sam": text, "args": args}


def extract_amb():
    import re
    src = open(ref_harness.REF_PATH, encoding="utf-8").read()
    m = re.search(r"amb = (\{.*?\})\n", src, re.S)
    return ast.literal_eval(m.group(1))


def build(cases):
    out = []
    for c in cases:
        r = ref_harness.run_case(c["sam"], c["args"])
        c = dict(c)
        c["status"] = r["status"]
        c["files"] = r["files"]
        out.append(c)
    return out


def main():
    os.makedirs(GOLD, exist_ok=True)
    kat = build(kat_cases())
    with open(os.path.join(GOLD, "kat.json"), "w") as fh:
        json.dump(kat, fh, indent=1, sort_keys=True)
    rng = random.Random(20260115)
    fz = build([fuzz_case(rng, k) for k in range(1500)])
    with open(os.path.join(GOLD, "fuzz.json"), "w") as fh:
        json.dump(fz, fh, indent=0, sort_keys=True)
    with open(os.path.join(GOLD, "amb.json"), "w") as fh:
        json.dump(extract_amb(), fh, indent=1, sort_keys=True)
    st = {}
    for c in fz:
        st[c["status"]] = st.get(c["status"], 0) + 1
    print("kat:", {c["name"]: c["status"] for c in kat})
    print("fuzz statuses:", st)


if __name__ == "__main__":
    main()
