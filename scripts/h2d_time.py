"""Where the C5 CLI's "h2d" phase goes (GPU box): HostBatch.ensure_layers, DeviceBatch's
upload through the pinned ring (engine.Uploader.timing: slot waits, pinned allocations,
packing, copy issue), the copy completion, Workspace allocation — three repetitions (the
first pays the pinned ring's and the caching allocator's first allocations).

    python scripts/h2d_time.py [workload]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from sam2consensus_amd import configs
    from sam2consensus_amd.engine import DeviceBatch, Workspace, default_uploader
    wl = sys.argv[1] if len(sys.argv) > 1 else "c5"
    hb = configs.synth_batch(wl)
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    torch.cuda.synchronize(dev)
    up = default_uploader(dev)
    for rep in range(3):
        for k in up.timing:
            up.timing[k] = 0.0
        t0 = time.perf_counter()
        hb.ensure_layers()
        t1 = time.perf_counter()
        db = DeviceBatch(hb, dev)
        t2 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        ws = Workspace(db, [0.25], 1, b"-")
        torch.cuda.synchronize(dev)
        t4 = time.perf_counter()
        out = {"rep": rep, "bytes": db.nbytes(), "layers_s": t1 - t0, "upload_host_s": t2 - t1, "copy_drain_s": t3 - t2,
               "workspace_s": t4 - t3, "total_s": t4 - t0, "uploader": dict(up.timing)}
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)
        del ws, db


if __name__ == "__main__":
    main()
