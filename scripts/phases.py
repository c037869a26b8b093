"""Phase timeline of k_pileup (diagnostic): per work item, s_memrealtime stamps (100 MHz)
at 0 start, 1 prologue done (after the histogram-zeroing barrier), 2 counting + flush done,
3 insertion columns counted, 4 insertion vote done, 5 position vote done, 6 tile totals
stored, 7 end; 8-10 inside the column-parallel insertion vote.  Prints, per phase, the distribution over work items of the time since
the earliest start (µs) and of the phase's own duration.

    python scripts/phases.py [workload] [extra_ablate_bits]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sam2consensus_amd import configs  # noqa: E402
from sam2consensus_amd.engine import DeviceBatch, Workspace  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
    extra = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0
    hb = configs.synth_batch(wl)
    ws = Workspace(DeviceBatch(hb), [0.25, 0.5, 0.75], keep_counts=True)
    ni = hb.info.n_items
    for _ in range(3):
        ws.run()
    ws.counts.zero_()
    ws.dev.ablate = 0x100 | extra
    torch.cuda.synchronize()
    ws.pileup()
    ws.consensus()
    torch.cuda.synchronize()
    ws.dev.ablate = 0
    ws.dev.ablate = 0
    ts = ws.counts[: ni * 128].view(torch.int64).cpu().numpy().reshape(ni, 16).astype(np.float64) / 100.0  # µs
    t0 = ts[:, 0].min()
    rel = ts - t0
    names = ["start", "prologue", "count+flush", "ins count", "ins vote", "pos vote", "totals", "end"]
    print("items %d; kernel span %.2f us (earliest start -> latest end)" % (ni, rel[:, 7].max()))
    for k, nm in enumerate(names):
        col = rel[:, k]
        dur = rel[:, k] - rel[:, k - 1] if k else col
        print("%-12s at  med %6.2f p90 %6.2f max %6.2f | dur med %6.2f p90 %6.2f max %6.2f" % (
            nm, np.median(col), np.percentile(col, 90), col.max(), np.median(dur), np.percentile(dur, 90), dur.max()))
    extra_names = {8: "col pass start", 9: "col votes (thread 0)", 10: "col votes synced"}
    for k, nm in extra_names.items():
        col = rel[:, k]
        ok = ts[:, k] > 0
        if ok.any():
            print("%-20s at med %6.2f (items %d)" % (nm, np.median(col[ok]), ok.sum()))


if __name__ == "__main__":
    main()
