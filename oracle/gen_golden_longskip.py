"""Generate tests/golden/longskip.json by RUNNING THE REFERENCE (test infrastructure, build
container only: needs /root/reference).

    python oracle/gen_golden_longskip.py

Reads whose seqout spans 2^24 positions or more — a CIGAR N skip of 16.7 Mb, legal SAM
(sam2consensus.py:70-72 writes one '-' per skipped position) — with -d given (its '-' are
counted, :210) and without (maxdel drops them).  Stored: the SAM text, args, status and the
sha256 and length of every output file (the files themselves are 16.7 MB).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness  # noqa: E402

GOLD = os.path.join(os.path.dirname(HERE), "tests", "golden")


def case_sam():
    L = (1 << 24) + 64
    skip = (1 << 24) + 2
    return ("@SQ\tSN:g\tLN:%d\n" % L +
            "r1\t0\tg\t1\t60\t5M%dN5M\t*\t0\t0\tACGTAACGTA\t*\n" % skip +
            "r2\t0\tg\t3\t60\t4M\t*\t0\t0\tGGGG\t*\n" +
            "r3\t0\tg\t%d\t60\t3M2I3M\t*\t0\t0\tTTTCCTTT\t*\n" % (skip + 1))


def main():
    sam = case_sam()
    cases = []
    for args in (["-d", "200"], []):
        r = ref_harness.run_case(sam, args)
        files = {k: {"sha256": hashlib.sha256(v.encode("latin-1")).hexdigest(), "bytes": len(v)}
                 for k, v in r["files"].items()}
        cases.append({"sam": sam, "args": args, "status": r["status"], "files": files})
        print(args, r["status"], files)
    with open(os.path.join(GOLD, "longskip.json"), "w") as fh:
        json.dump(cases, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
