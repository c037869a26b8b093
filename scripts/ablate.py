"""Timing ablations of the device stages (diagnostic; results are wrong by design).

    python scripts/ablate.py [workload] [reps]
Prints the median kernel time of k_pileup for each ablation mask, interleaved in one
process (cdna_hip_programming.md §5.4 rule 24)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sam2consensus_amd import configs  # noqa: E402
from sam2consensus_amd.engine import DeviceBatch, Workspace  # noqa: E402

MODES = {0: "full", 1: "skip counting loop", 2: "loads only (no counting)",
         4: "store counts, no vote", 5: "1|4 (zero+store only)", 6: "2|4", 12: "4|8 (no flush, no vote)",
         0x800: "empty kernel (launch)"}


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    hb = configs.synth_batch(wl)
    ws = Workspace(DeviceBatch(hb, dense_layers=True), [0.25, 0.5, 0.75], keep_counts=True)   # mode 4 stores all counts
    times = {m: [] for m in MODES}
    for _ in range(reps):
        for m in MODES:
            ws.dev.ablate = m
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ws.pileup()
            e1.record()
            ws.consensus()   # untimed
            torch.cuda.synchronize()
            times[m].append(e0.elapsed_time(e1))
    ws.dev.ablate = 0
    for m, name in MODES.items():
        t = sorted(times[m])
        print("ablate=%d %-36s median %.3f ms  min %.3f ms" % (m, name, t[len(t) // 2], t[0]))


if __name__ == "__main__":
    main()
