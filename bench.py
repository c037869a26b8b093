#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: aligned bases/s into consensus on MI355X.

A step = one pass of the device hot path (pileup + fused insertion columns, vote and FASTA
body bytes → flagged tiles) over one synthetic batch resident in HBM:
one `s2c_run` (direct kernel launches, queued back to back — a HIP graph replay costs
≈5 µs more GPU time per step on this ROCm, scripts/launch_overhead.py; `--graph` times
replays instead).  Host SAM parse and H2D are excluded; parse time is reported separately.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2]

N>1 is launched by torch.distributed.run, one process per GPU.  The path shards by
reference position with no exchange: each rank runs its own batch of the workload
(its own 353 loci for c2; seed = SEED + rank), so per-GPU work is fixed — weak scaling.
Timing: barrier + synchronize on both sides of exactly K steps, MAX over ranks.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (/opt/skills/guides/MI355X_MICROARCH.md)

WORKLOADS = {
    "c2": "c2: Hyb-seq 353 loci x 1 kb, 500x, 150 bp, 5% 1-4 bp I / 5% 1-5 bp D, -c 0.25,0.50,0.75",
    "c1": "c1: 10 genes x 1 kb, 100x, 150 bp, -c 0.25",
    "c3": "c3: bacterial 5 Mb, 1000x, 150 bp, shuffled, -m 10",
    "c4": "c4: chrM 16,569 bp, 100,000x, 166 amplicon starts",
    "c5": "c5: chr20 64,444,167 bp, 30x, 150 bp, 1% D reads, -d 150",
}


def b_alg(info, T):
    """Algorithmic bytes of one step, and of the fused k_pileup launch.

    step   = 0.5·Q + 16·N + 4·K + (48+T)·L + Σ_ins(8 + 0.5·len)   (SURVEY's formula, which
             prices the count tensor as written once + read once)
    k_pileup = step − 48·L: the same inputs (packed bases, read records, op words, insertion
             events) and the per-threshold consensus codes out, but the fused kernel keeps
             the counts in registers/LDS, so no count bytes are charged to it (deep tiles,
             none in c2, would add 24·L)."""
    Q, N, K, L = info.query_bases, info.reads_mapped, info.n_ops, info.total_len
    ins = 8 * info.n_ins + 0.5 * info.n_ins_bases
    step = 0.5 * Q + 16 * N + 4 * K + (48 + T) * L + ins
    return step, step - 48 * L


def cpu_baseline(workload, scale):
    """Time the oracle (pure-Python port of the reference, 1 core) on a bounded sample."""
    import tempfile

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import s2c_oracle
    from sam2consensus_amd import configs

    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "sample.sam")
        configs.synth_write(workload, p, scale=scale)
        hb = configs.synth_batch(workload, scale=scale)
        a = hb.aligned_bases
        hb.free()
        t0 = time.perf_counter()
        s2c_oracle.run_path(p, configs.cli_args(workload))
        dt = time.perf_counter() - t0
    sp = configs.spec(workload, scale=scale)
    return {"value": a / dt, "unit": "aligned bases/s", "cores": 1, "kind": "port",
            "sample": "%s with %d refs x %d bp (%d aligned bases, %.1f s): oracle/s2c_oracle.py, the "
                      "pure-Python restatement of sam2consensus.py, parse+pileup+vote+format, 1 thread"
                      % (workload, sp.n_refs, sp.ref_len, a, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-scale", type=float, default=0.4)
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--graph", action="store_true", help="time HIP graph replays of the step")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    from sam2consensus_amd import configs
    from sam2consensus_amd.engine import DeviceBatch, Workspace

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    wl = args.workload
    opt_args = configs.cli_args(wl)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    thresholds = [0.25]
    min_depth = 1
    if "-c" in opt_args:
        thresholds = [float(x) for x in opt_args[opt_args.index("-c") + 1].split(",")]
    if "-m" in opt_args:
        min_depth = int(opt_args[opt_args.index("-m") + 1])

    t0 = time.perf_counter()
    hb = configs.synth_batch(wl, seed=configs.SEED + rank)
    t_host = time.perf_counter() - t0
    info = hb.info
    T = len(thresholds)
    db = DeviceBatch(hb, dev)
    ws = Workspace(db, thresholds, min_depth, b"-")
    K = args.steps
    # k_pileup's own duration (roofline): one pair of HIP events on the launch stream around
    # K back-to-back pileup launches (per-launch event pairs would add their own packets to
    # every measured kernel); also the warm-up.
    for _ in range(args.warmup):
        ws.run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(K):
        ws.pileup()
    e1.record()
    torch.cuda.synchronize(dev)
    pileup_ms = e0.elapsed_time(e1) / K
    # the step: one s2c_run (or one replay of its captured HIP graph)
    if args.graph:
        ws.capture()
        step = ws.replay
    else:
        step = ws.run
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(K):
        step()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0

    stats = torch.tensor([elapsed, float(info.aligned_bases)], dtype=torch.float64, device=dev)
    if world > 1:
        mx = stats[:1].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = stats[1:].clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed, total_bases = float(mx.item()), float(sm.item())
    else:
        total_bases = float(info.aligned_bases)

    parity = None
    if rank == 0 and not args.no_parity:
        parity = check_parity(wl, hb, ws, thresholds)

    if rank == 0:
        step_bytes, pileup_bytes = b_alg(info, T)
        ms = elapsed / K * 1e3
        achieved = pileup_bytes / (pileup_ms * 1e-3) / 1e9
        line = {
            "metric": "aligned bases/sec into consensus (1/2/4/8 GPU); HBM GB/s; vs CPU script",
            "value": total_bases * K / elapsed,
            "unit": "aligned bases/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": WORKLOADS[wl], "aligned_bases_per_gpu": info.aligned_bases,
                       "reads_per_gpu": info.reads_mapped, "positions_per_gpu": info.total_len,
                       "thresholds": thresholds,
                       "parallelism": "one batch per GPU, sharded by reference (no collective on the data path)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic_from_profile(wl),
                         "kernel": "k_pileup (counting + fused insertion-column and vote epilogue)", "kernel_ms": pileup_ms,
                         "alg_bytes_per_launch": pileup_bytes},
            "step_alg_bytes": step_bytes,
            "step_achieved_gbps": step_bytes / (ms * 1e-3) / 1e9,
            "host_parse_s_per_gpu": t_host,
            "parity": parity,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(wl, args.cpu_sample_scale)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def traffic_from_profile(wl):
    """Per-launch HBM bytes of k_pileup from the committed PMC pass (profiles/), or None."""
    p = os.path.join(ROOT, "profiles", "traffic_%s.json" % wl)
    if os.path.exists(p):
        with open(p) as fh:
            return json.load(fh).get("k_pileup_hbm_bytes_per_launch")
    return None


def check_parity(wl, hb, ws, thresholds):
    """Rank 0 runs the default seed: compare the step's FASTA files with the reference's."""
    import hashlib

    gpath = os.path.join(ROOT, "tests", "golden", "configs.json")
    if not os.path.exists(gpath):
        return None
    g = json.load(open(gpath)).get(wl)
    if not g:
        return None
    from sam2consensus_amd import configs
    from sam2consensus_amd.records import build_records, render

    stats, offs, out = ws.fetch()
    a = configs.cli_args(wl)
    prefix = g["sam_file"].split(".")[0]
    recs = build_records(hb, thresholds, prefix, stats, offs, out)
    n = int(a[a.index("-n") + 1]) if "-n" in a else 0
    got = {name + "__" + prefix + ".fasta": hashlib.sha256(render(r, n)).hexdigest() for name, r in recs.items()}
    want = {k: v["sha256"] for k, v in g["files"].items()}
    return "byte-identical to reference (%d files)" % len(want) if got == want else "MISMATCH"


if __name__ == "__main__":
    main()
