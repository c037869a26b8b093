"""CPU-baseline calibration (test infrastructure, build container only: needs /root/reference).

    python oracle/calibrate_cpu.py [out.json]

SURVEY §8(d) asks for bench.py's cpu_baseline — oracle/s2c_oracle.py, the pure-Python
restatement of sam2consensus.py, timed on a bounded sample on the GPU box — to be calibrated
against the reference itself.  This runs the reference's own main() (oracle/ref_harness.py)
and the restatement on the same C1 / C2-sample SAM files, one thread each, in this
container, and records both rates (aligned bases / s) and their ratio; bench.py's
cpu_baseline sample cites it (profiles/cpu_calibration.json).
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [HERE, ROOT]
import ref_harness  # noqa: E402
import s2c_oracle  # noqa: E402

from sam2consensus_amd import configs  # noqa: E402


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "cpu_calibration.json")
    rows = []
    for wl, scale in (("c1", 1.0), ("c2", 0.05), ("c5", 0.016)):
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, wl + ".sam")
            configs.synth_write(wl, p, scale=scale)
            hb = configs.synth_batch(wl, scale=scale)
            bases = hb.aligned_bases
            hb.free()
            args = configs.cli_args(wl)
            t0 = time.perf_counter()
            ref_harness.run_file(p, args, os.path.join(td, "ref"))
            t_ref = time.perf_counter() - t0
            t0 = time.perf_counter()
            s2c_oracle.run_path(p, args)
            t_or = time.perf_counter() - t0
        rows.append({"workload": wl, "scale": scale, "aligned_bases": bases,
                     "reference_s": t_ref, "oracle_s": t_or,
                     "reference_bases_per_s": bases / t_ref, "oracle_bases_per_s": bases / t_or,
                     "oracle_over_reference": t_ref / t_or})
        print(rows[-1], flush=True)
    res = {"what": "sam2consensus.py's main() under oracle/ref_harness.py vs oracle/s2c_oracle.py, same SAM file, "
                   "1 thread each, this build container (Python %s)" % sys.version.split()[0],
           "rows": rows}
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
