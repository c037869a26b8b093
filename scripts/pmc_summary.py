"""Per-kernel averages (per dispatch) of every counter of the PMC passes in a directory.

    python scripts/pmc_summary.py gpurun_out/pmc_c3 [kernel-substring]
Prints one line per (kernel, counter); SQ_INSTS_* are per dispatch (all waves), and the
derived VALU cycles assume one wave64 VALU instruction per SIMD quad-cycle (4 clocks) on
1024 SIMDs at 2.4 GHz (MI355X_MICROARCH.md)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    base = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    acc = defaultdict(list)
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(base, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
                if sub not in name:
                    continue
                acc[(name, row["Counter_Name"])].append(float(row["Counter_Value"]))
                dur[name].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
    for (k, c), v in sorted(acc.items()):
        m = sum(v) / len(v)
        extra = ""
        if c == "SQ_INSTS_VALU":
            extra = "  (VALU floor %.3f ms)" % (m * 4 / 1024 / 2.4e9 * 1e3)
        print("%-40s %-24s %16.1f  (n=%d)%s" % (k[:40], c, m, len(v), extra))
    for k, v in sorted(dur.items()):
        print("%-40s duration under counters %.3f ms" % (k[:40], sum(v) / len(v)))


if __name__ == "__main__":
    main()
