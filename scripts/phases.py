"""Phase timeline of k_pileup (diagnostic): per work item, s_memrealtime stamps (100 MHz)
at 0 start, 1 prologue done (after the histogram-zeroing barrier), 2 counting + flush done,
then in the fast epilogue (last chunk / pass): 3 phase A (votes) done, 4 after its barrier,
5 phase B (lengths, scans, statistics) done, 8 after its barrier, 9 phase C (body bytes)
done, 6 tile statistics stored, 7 end.  Prints, per phase, the distribution over work items of the time since
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
    ws = Workspace(DeviceBatch(hb, dense_layers=True), [0.25, 0.5, 0.75], keep_counts=True)
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
    ts = ws.counts[: ni * 128].view(torch.int64).cpu().numpy().reshape(ni, 16).astype(np.float64) / 100.0  # µs
    t0 = ts[:, 0].min()
    rel = ts - t0
    # stamp order of the fast epilogue (k_pileup's common case)
    order = [(0, "start"), (10, "ranges known"), (11, "records issued"), (1, "prologue"), (2, "count+flush"), (3, "A votes"), (4, "A barrier"),
             (5, "B lengths+scan"), (8, "B barrier"), (9, "C bytes"), (6, "stats"), (7, "end")]
    print("items %d; kernel span %.2f us (earliest start -> latest end)" % (ni, rel[:, 7].max()))
    prev = None
    for k, nm in order:
        col = rel[:, k]
        dur = col - rel[:, prev] if prev is not None else col
        print("%-16s at  med %6.2f p90 %6.2f max %6.2f | dur med %6.2f p90 %6.2f max %6.2f" % (
            nm, np.median(col), np.percentile(col, 90), col.max(), np.median(dur), np.percentile(dur, 90), dur.max()))
        prev = k
    # what the slow items have in common: records streamed, XCD (blockIdx mod 8), start time
    items = hb.items[:, :4].astype(np.int64)
    wrec = hb.wrec.astype(np.int64)
    recs = np.array([wrec[(b + 31) >> 5] - wrec[a >> 5] for a, b, _, _ in items])
    cnt = rel[:, 2] - rel[:, 1]
    print("count+flush vs records: corr %.2f; records med %d max %d" % (
        np.corrcoef(recs, cnt)[0, 1], np.median(recs), recs.max()))
    xcd = np.arange(ni) % 8
    print("per XCD: median count+flush " + " ".join("%.2f" % np.median(cnt[xcd == x]) for x in range(8)))
    print("per XCD: max end            " + " ".join("%.2f" % rel[xcd == x, 7].max() for x in range(8)))
    slow = np.argsort(-rel[:, 7])[:8]
    for i in slow:
        print("  item %4d xcd %d recs %6d start %.2f prologue-end %.2f count %.2f end %.2f" % (
            i, i % 8, recs[i], rel[i, 0], rel[i, 1], cnt[i], rel[i, 7]))


if __name__ == "__main__":
    main()
