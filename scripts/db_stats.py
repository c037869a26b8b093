"""rocprofv3 results database (out_results.db) → the kernel-stats CSV of `--stats`
(Name,Calls,TotalDurationUs,AverageUs,Percentage), for profiles/.

    python scripts/db_stats.py gpurun_out/prof_v9_c5/out_results.db > profiles/r03/v9_c5_kernel_stats.csv
"""
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, count(*), sum(end - start) from kernels group by name"))
    tot = sum(r[2] for r in rows) or 1
    print("Name,Calls,TotalDurationUs,AverageUs,Percentage")
    for name, n, ns in sorted(rows, key=lambda r: -r[2]):
        print('"%s",%d,%.3f,%.3f,%s' % (name.replace('"', "'"), n, ns / 1e3, ns / 1e3 / n, 100.0 * ns / tot))


if __name__ == "__main__":
    main(sys.argv[1])
