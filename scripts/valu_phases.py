"""VALU instructions per phase of k_tile_dense, from one rocprofv3 --pmc run of
scripts/prof_dense.py over a list of ablation bits (prof build: each bit switches one phase
off, timing only — results wrong by design):

    rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d OUT -o run -- \
        python3 scripts/prof_dense.py c5 0,4,2,8,16,32,64
    python scripts/valu_phases.py OUT 0,4,2,8,16,32,64

prof_dense.py launches the dense kernel 1 + 5 times per ablation value, in order; the
dispatches are grouped that way and each group's mean SQ_INSTS_VALU per wave is compared
with ablation 0's.  Prints VALU per wave and the share each phase holds."""
import csv
import glob
import os
import sys
from collections import defaultdict

NAMES = {1: "events", 2: "count", 4: "walk (fast + queue)", 8: "vote + store", 16: "queued walk", 32: "N / '-' events",
         64: "slow votes"}


def main():
    base, bits = sys.argv[1], [int(b) for b in sys.argv[2].split(",")]
    rows = defaultdict(dict)
    for f in glob.glob(os.path.join(base, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "k_tile_dense" not in r["Kernel_Name"]:
                    continue
                rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(rows)
    per = 6   # (prof_dense.py: one warm-up launch + 5 timed per ablation value)
    if len(ids) < per * len(bits):
        sys.exit("expected %d dense dispatches, found %d" % (per * len(bits), len(ids)))
    ids = ids[-per * len(bits):]
    res = {}
    for k, b in enumerate(bits):
        grp = [rows[i] for i in ids[per * k:per * (k + 1)]]
        v = sum(g["SQ_INSTS_VALU"] for g in grp) / len(grp)
        w = sum(g["SQ_WAVES"] for g in grp) / len(grp)
        res[b] = (v, w)
    v0, w0 = res[bits[0]]
    print("ablation 0: %.1f M VALU per launch, %.0f waves, %.1f VALU per wave" % (v0 / 1e6, w0, v0 / w0))
    for b in bits[1:]:
        v, w = res[b]
        d = (v0 - v) / w0
        print("  off %-3d %-22s VALU/wave %7.1f  phase %6.1f (%4.1f %%)" % (b, NAMES.get(b, "?"), v / w, d, 100 * d / (v0 / w0)))


if __name__ == "__main__":
    main()
