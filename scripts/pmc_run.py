"""A few k_pileup runs of a workload with a diagnostic ablate mask — the target program of
the PMC passes in scripts/pmc_ablate.sh (counters per variant, e.g. 0x200 = no insertions).

    python scripts/pmc_run.py [workload] [ablate_mask]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sam2consensus_amd import configs  # noqa: E402
from sam2consensus_amd.engine import DeviceBatch, Workspace  # noqa: E402


def configs_thresholds(wl):
    a = configs.cli_args(wl)
    return [float(x) for x in a[a.index("-c") + 1].split(",")] if "-c" in a else [0.25]


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
    mask = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0
    hb = configs.synth_batch(wl)
    ws = Workspace(DeviceBatch(hb, dense_layers=True), configs_thresholds(wl), keep_counts=True)
    ws.dev.ablate = mask
    for _ in range(3):
        ws.pileup()
    torch.cuda.synchronize()
    print("done", wl, hex(mask))


if __name__ == "__main__":
    main()
