"""Per-step launch overhead of the bench step (diagnostic): K back-to-back steps as graph
replays vs direct launches, for the real kernel and for an empty one (ablate 0x800).

    python scripts/launch_overhead.py [workload] [K]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sam2consensus_amd import configs  # noqa: E402
from sam2consensus_amd.engine import DeviceBatch, Workspace  # noqa: E402


def timed(fn, K):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e6


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    hb = configs.synth_batch(wl)
    ws = Workspace(DeviceBatch(hb), [0.25, 0.5, 0.75])
    for mask, name in ((0, "full kernel"), (0x800, "empty kernel")):
        ws.dev.ablate = mask
        direct = timed(ws.run, K)
        ws.capture()
        graph = timed(ws.replay, K)
        print("%-13s direct launches %.2f us/step   graph replays %.2f us/step" % (name, direct, graph))
    ws.dev.ablate = 0


if __name__ == "__main__":
    main()
