"""Generate tests/golden/limits.json by RUNNING THE REFERENCE (test infrastructure, build
container only: needs /root/reference).

    python oracle/gen_golden_limits.py

Legal inputs at this build's former limits: a -c list of 300 thresholds (the reference takes
any number, sam2consensus.py:117-118; round 3 refused more than 256), on a SAM with a shallow
reference (dense tiles), one with insertion columns (k_tile) and one deep enough for
k_consensus.  Stored: the SAM text, args, status and the sha256 and length of every output.
"""
from __future__ import annotations

import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness  # noqa: E402

GOLD = os.path.join(os.path.dirname(HERE), "tests", "golden")


def case_sam(seed=300):
    rng = random.Random(seed)
    refs = [("g1", 160), ("g2", 160), ("g3", 96)]
    out = ["@HD\tVN:1.0\n"] + ["@SQ\tSN:%s\tLN:%d\n" % r for r in refs]
    genome = {n: "".join(rng.choice("ACGT") for _ in range(L)) for n, L in refs}

    def read(name, pos, n, cig_ins=False):
        s = list(genome[name][pos:pos + n])
        for i in range(len(s)):
            u = rng.random()
            if u < 0.12:
                s[i] = rng.choice("ACGT")   # mismatches: ambiguity codes at every threshold (no N: {A,C,G,N,T} has no amb key)
        seq = "".join(s)
        if cig_ins and n > 20:
            k = rng.randrange(5, n - 10)
            ins = "".join(rng.choice("ACGT") for _ in range(rng.randrange(1, 4)))
            return "%dM%dI%dM" % (k, len(ins), n - k), seq[:k] + ins + seq[k:]
        return "%dM" % n, seq

    k = 0
    for name, L in refs:
        depth = {"g1": 12, "g2": 10, "g3": 400}[name]
        rl = 40
        for _ in range(depth * L // rl):
            pos = rng.randrange(0, L - rl)
            cig, seq = read(name, pos, rl, cig_ins=(name == "g2"))
            out.append("r%d\t0\t%s\t%d\t60\t%s\t*\t0\t0\t%s\t*\n" % (k, name, pos + 1, cig, seq))
            k += 1
    return "".join(out)


def thresholds():
    return ",".join("%g" % (i / 300.0) for i in range(1, 301))


def main():
    sam = case_sam()
    cases = []
    for args in (["-c", thresholds()], ["-c", thresholds(), "-m", "3", "-f", "N", "-n", "60"]):
        r = ref_harness.run_case(sam, args)
        files = {k: {"sha256": hashlib.sha256(v.encode("latin-1")).hexdigest(), "bytes": len(v)}
                 for k, v in r["files"].items()}
        cases.append({"sam": sam, "args": args, "status": r["status"], "files": files})
        print(args[:1], r["status"], {k: v["bytes"] for k, v in files.items()})
    with open(os.path.join(GOLD, "limits.json"), "w") as fh:
        json.dump(cases, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
