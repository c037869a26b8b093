"""Lane utilisation of k_tile_dense's count loop on a workload, from the packed batch alone (no
GPU): per wave (16 words of a 32-word tile, G = 4 lanes per word) the loop runs to the
largest lane's record count, rounded to the 8-record groups / 4-record tail the kernel uses;
prints the fraction of those slots that hold one of the lane's candidate records.

    python scripts/lane_util.py [workload] [sampled tiles]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sam2consensus_amd import configs  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c5"
    nsample = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    t = time.time()
    hb = configs.synth_batch(wl, seed=configs.SEED)
    print("synth %.1f s" % (time.time() - t), flush=True)
    i = hb.info
    K = int(i.kwin)
    rs = np.asarray(hb.rs).astype(np.int64)
    dw = np.asarray(hb.dwin).reshape(-1, 16).astype(np.int64)
    print("kwin", K, "dense items", dw.shape[0], "tile_max", i.tile_max)
    G, NWPW = 4, 16
    tot_rec = tot_slots = 0
    hist = {}
    rng = np.random.default_rng(0)
    for it in rng.choice(dw.shape[0], min(nsample, dw.shape[0]), replace=False):
        a, b = dw[it, 1], dw[it, 2]
        W0, nw = a >> 5, (b - a + 31) // 32
        for wv in range(2):
            W = W0 + np.arange(wv * NWPW, min(wv * NWPW + NWPW, nw))
            cnt = rs[W + 1] - rs[np.maximum(W - K, 0)]
            nrec = np.concatenate([np.maximum((cnt - g + G - 1) // G, 0) for g in range(G)])
            nmx = int(nrec.max()) if len(nrec) else 0
            slots = 8 * (nmx // 8 + (1 if nmx % 8 > 4 else 0)) + (4 if 0 < nmx % 8 <= 4 else 0)
            tot_rec += int(nrec.sum())
            tot_slots += 64 * slots
            hist[slots] = hist.get(slots, 0) + 1
    print("lane utilisation of the count: %.3f" % (tot_rec / max(tot_slots, 1)))
    print("records per lane (mean): %.2f" % (tot_rec / (sum(hist.values()) * 64)))
    print("waves by record slots per lane:", sorted(hist.items()))
    hb.free()


if __name__ == "__main__":
    main()
