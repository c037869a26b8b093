"""Kernel statistics (calls, average / min / max / total ns, share) from a rocprofv3 database
(`--kernel-trace` without `--output-format csv` writes out_results.db), written as the csv
rocprofv3 --stats produces, so the bench's kernel times can be checked against the trace.

    python scripts/kstats_db.py gpurun_out/prof_x/out_results.db [out.csv]"""
import csv
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sqlite3.connect(sys.argv[1])
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else "kernel_name"
    rows = db.execute("select %s, start, end from kernels" % name_col).fetchall()
    acc = defaultdict(list)
    for n, s, e in rows:
        acc[n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]].append(e - s)
    tot = sum(sum(v) for v in acc.values()) or 1
    out = [{"Name": k, "Calls": len(v), "TotalDurationNs": sum(v), "AverageNs": sum(v) / len(v), "MinNs": min(v),
            "MaxNs": max(v), "Percentage": 100.0 * sum(v) / tot} for k, v in acc.items()]
    out.sort(key=lambda r: -r["TotalDurationNs"])
    f = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
    w.writeheader()
    w.writerows(out)


if __name__ == "__main__":
    main()
