"""Generate tests/golden/stdout.json: the reference's own stdout, captured by RUNNING THE
REFERENCE (test infrastructure, build container only: needs /root/reference).

    python oracle/gen_golden_stdout.py

Each case runs in a scratch directory as ``sam2consensus.py -i in.sam -o out <args>`` (the
same relative paths the test uses), so the printed paths are comparable.  Cases: a few KAT
probes (one and several thresholds, several references, an error class) and a generated
file of 1,200,003 lines whose reading crosses the progress counter's 500,000-line marks
(sam2consensus.py:143, :182, :194, :224-225, :420-426).  Stored per case: the KAT name (its
SAM text and args are in kat.json) or the generator parameters, the status and the stdout.
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness  # noqa: E402

GOLD = os.path.join(os.path.dirname(HERE), "tests", "golden")
KAT_NAMES = ["tiny", "maxdel_default", "round_tie", "negdash", "dash_thr", "multifill", "two_refs_one_empty",
             "err_acgnt", "unknown_ref", "err_past_end"]


def progress_sam(n_lines):
    """n_lines body lines: one mapped read per 1000 lines, the rest unmapped ('*' CIGAR)."""
    head = "@HD\tVN:1.0\tSO:unsorted\n@SQ\tSN:g\tLN:200\n"
    mapped = "r\t0\tg\t11\t60\t20M\t*\t0\t0\t" + "ACGT" * 5 + "\t*\n"
    unmapped = "u\t4\t*\t0\t0\t*\t*\t0\t0\tACGT\t*\n"
    return head + "".join(mapped if k % 1000 == 0 else unmapped for k in range(n_lines))


def capture(sam_text, args):
    with tempfile.TemporaryDirectory() as td:
        with open(os.path.join(td, "in.sam"), "wb") as fh:
            fh.write(sam_text.encode("latin-1"))
        status, out = ref_harness.run_reference(["-i", "in.sam", "-o", "out"] + list(args), cwd=td)
    return status, out


def main():
    with open(os.path.join(GOLD, "kat.json")) as fh:
        kat = {c["name"]: c for c in json.load(fh)}
    cases = []
    for name in KAT_NAMES:
        if name not in kat:
            continue
        status, out = capture(kat[name]["sam"], kat[name]["args"])
        cases.append({"kat": name, "args": kat[name]["args"], "status": status, "stdout": out})
    n = 1_200_001
    status, out = capture(progress_sam(n), [])
    cases.append({"progress_lines": n, "args": [], "status": status, "stdout": out})
    with open(os.path.join(GOLD, "stdout.json"), "w") as fh:
        json.dump(cases, fh, indent=1, sort_keys=True)
    print("wrote %d cases" % len(cases))


if __name__ == "__main__":
    main()
