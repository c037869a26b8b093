#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: aligned bases/s into consensus on MI355X.

A step = one pass of the device hot path over one synthetic batch resident in HBM: one
`s2c_run` = k_reads (parsecigar + maxdel per piece → run records, insertion events →
per-tile hash tables) → k_tile / k_tile_dense (pileup, insertion columns, vote, FASTA body
bytes) → k_consensus (deep / general tiles), launched back to back on one stream.  Host SAM
parse and H2D are excluded; parse time is reported separately (host_parse_s).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c5] [--shard]

Default workload: C5 (chr20 64.4 Mb × 30x, the largest single-GPU config of BASELINE.json;
its ~0.7 GB batch does not fit the 256 MiB Infinity Cache).  Per-kernel times come from
HIP events recorded on the launch stream between the stages of every timed step, so each
kernel's time is a sub-interval of the step it belongs to.

N>1 (torch.distributed.run, one process per GPU):
  default        weak scaling (the path partitions by position: per-GPU work fixed as N
                 grows): each rank runs its own batch of the workload (seed + rank), as the
                 position shards of an N-times larger genome would; no collective on the
                 data path;
  --shard        strong scaling, the north_star position split of ONE workload: contiguous
                 tile ranges (sam2consensus_amd.shard.split_tiles), each rank runs its shard;
                 the shards' FASTA bodies and statistics are gathered to rank 0 (RCCL) after
                 the timed steps and checked against the reference's golden.
Timing: barrier + synchronize on both sides of exactly K steps, MAX over ranks; value =
aligned bases of all ranks / that time.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (/opt/skills/guides/MI355X_MICROARCH.md)

WORKLOADS = {
    "c1": "c1: 10 genes x 1 kb, 100x, 150 bp, -c 0.25",
    "c2": "c2: Hyb-seq 353 loci x 1 kb, 500x, 150 bp, 5% 1-4 bp I / 5% 1-5 bp D, -c 0.25,0.50,0.75",
    "c3": "c3: bacterial 5 Mb, 1000x, 150 bp, shuffled, -m 10",
    "c4": "c4: chrM 16,569 bp, 100,000x, 166 amplicon starts",
    "c5": "c5: chr20 64,444,167 bp, 30x, 150 bp, 1% D reads, -d 150",
    "c5nd": "c5nd: chr20 64,444,167 bp, 30x, 150 bp, 1% D reads, maxdel 150 active (no -d)",
}


def b_alg(info, T):
    """Algorithmic bytes of one step and of its stages.

    step    = 0.5·Q + 16·N + 4·K + (48+T)·L + Σ_ins(8 + 0.5·len)  (SURVEY's formula: 4-bit
              query bases, 16 B per read, 4 B per CIGAR op, the count tensor written + read
              once, T vote bytes per position, the insertion events)
    pileup  = step − 48·L: the tile kernels keep the counts in registers / LDS (never the
              count tensor), and both k_tile_dense and k_tile walk their own window's piece
              records and CIGAR ops (16·N + 4·K are theirs; C3 / C4 / C5 launch no k_reads)
    reads   = Σ_ins(8 + 0.5·len): k_reads walks only the pieces emitting insertion events
              (C2) and the long pieces of k_tile's tiles, re-reading records the pileup's
              figure already holds; priced by the events it hashes, never added to a total"""
    Q, N, K, L = info.query_bases, info.reads_mapped, info.n_tokens, info.total_len
    ins = 8 * info.n_ins + 0.5 * info.n_ins_bases
    step = 0.5 * Q + 16 * N + 4 * K + (48 + T) * L + ins
    return step, ins, step - 48 * L

def cpu_baseline(workload, scale):
    """Time the oracle (pure-Python restatement of the reference, 1 core) on a bounded sample."""
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
    line = {"value": a / dt, "unit": "aligned bases/s", "cores": 1, "kind": "port",
            "sample": "%s at scale %g: %d refs x %d bp (%d aligned bases, %.1f s): oracle/s2c_oracle.py, the "
                      "pure-Python restatement of sam2consensus.py, parse+pileup+vote+format, 1 thread; %s"
                      % (workload, scale, sp.n_refs, sp.ref_len, a, dt, cpu_model())}
    # calibration against the reference itself: oracle/calibrate_cpu.py ran the
    # reference's main() and the restatement on the same files in the build container
    cal = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    if os.path.exists(cal):
        rows = {r["workload"]: r for r in json.load(open(cal))["rows"]}
        r = rows.get(workload)
        if r:
            line["calibration"] = {"oracle_over_reference": r["oracle_over_reference"], "sample": "%s at scale %g"
                                   % (workload, r["scale"]), "source": "profiles/cpu_calibration.json"}
            line["reference_equivalent_value"] = line["value"] / r["oracle_over_reference"]
            line["sample"] += ("; the reference's own main() runs the same %s sample %.2fx slower than this "
                               "restatement (calibration, build container)" % (workload, r["oracle_over_reference"]))
    return line


def cpu_threads():
    """Host threads this process may use (the GPU box's CPU share: OMP_NUM_THREADS)."""
    n = os.environ.get("OMP_NUM_THREADS")
    if n and n.isdigit() and int(n) > 0:
        return int(n)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline_mc(workload, scale):
    """Time oracle/s2c_oracle_mc — the C restatement of sam2consensus.py, parse + pileup +
    vote + FASTA on every host thread of this process — on the workload itself (scale 1)
    or a bounded sample of it; its FASTA is checked against the golden sha256 at scale 1."""
    import hashlib
    import subprocess
    import tempfile

    from sam2consensus_amd import configs

    binary = os.path.join(ROOT, "oracle", "build", "s2c_oracle_mc")
    if not os.path.exists(binary):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    T = cpu_threads()
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, workload + ".sam")
        configs.synth_write(workload, p, scale=scale)
        hb = configs.synth_batch(workload, scale=scale)
        a = hb.aligned_bases
        hb.free()
        out = os.path.join(td, "out")
        t0 = time.perf_counter()
        r = subprocess.run([binary, str(T), "-i", p, "-o", out] + configs.cli_args(workload),
                           capture_output=True, text=True)
        dt = time.perf_counter() - t0
        ok = r.returncode == 0 and "status: ok" in r.stdout
        check = None
        if ok and scale == 1.0:
            g = golden_for(workload)
            if g and g.get("files"):
                got = {f: hashlib.sha256(open(os.path.join(out, f), "rb").read()).hexdigest() for f in os.listdir(out)}
                check = got == {f: v["sha256"] for f, v in g["files"].items()}
    sp = configs.spec(workload, scale=scale)
    return {"value": a / dt if ok else None, "unit": "aligned bases/s", "cores": T, "kind": "port",
            "sample": "%s at scale %g: %d refs x %d bp (%d aligned bases, %.2f s incl. file read): "
                      "oracle/s2c_oracle_mc.c, the C restatement of sam2consensus.py, parse+pileup+vote+format "
                      "on %d threads; %s" % (workload, scale, sp.n_refs, sp.ref_len, a, dt, T, cpu_model()),
            "output_matches_golden": check}


def golden_for(workload):
    p = os.path.join(ROOT, "tests", "golden", "configs.json")
    try:
        with open(p) as fh:
            return json.load(fh).get(workload)
    except OSError:
        return None


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return "%s, %d CPUs visible" % (ln.split(":", 1)[1].strip(), os.cpu_count() or 0)
    except OSError:
        pass
    return platform.processor()


def rank_command(n, argv, port):
    """The torch.distributed.run command line that runs this script as n ranks on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def spawn_ranks(n, argv):
    """``--gpus N > 1`` with no WORLD_SIZE in the environment: start torch.distributed.run as a
    CHILD process (nothing here has touched the GPU: no torch.cuda call, no exec), one rank
    per GPU; forward every line the ranks print to stderr except rank 0's JSON line, which is
    printed last as this process's one line; return torchrun's exit status (non-zero when
    any rank failed)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    p = subprocess.Popen(rank_command(n, argv, port), stdout=subprocess.PIPE, text=True, env=dict(os.environ))
    line = None
    for ln in p.stdout:
        if ln.startswith("{") and '"metric"' in ln:
            line = ln.strip()
        else:
            sys.stderr.write(ln)
    rc = p.wait()
    if line is not None:
        print(line, flush=True)
    elif rc == 0:
        sys.stderr.write("bench.py: no rank printed a result line\n")
        rc = 1
    return rc


def timed_steps(ws, K, W, world, dev, graph=False, stage_events=False):
    """W untimed warmup steps, then EXACTLY K steps bracketed by a barrier + synchronize on
    both sides; returns (this rank's seconds, the max over ranks, per-stage GPU ms).

    An event is a timestamp packet with a cache release on this GPU (~5-9 us each), so by
    default the timed loop carries only two, on the launch stream around all K steps: their
    interval / K is the GPU time of a whole step (every stage; C5 launches only the pileup
    kernel), which the roofline prices the pileup's bytes against.  The per-stage split comes
    from a few more steps with events between the stages (--stage-events: events between
    all stages of every timed step instead)."""
    import torch
    import torch.distributed as dist
    stream = torch.cuda.current_stream(dev)
    for _ in range(W):
        ws.run()
    torch.cuda.synchronize(dev)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(K if stage_events else 0)]
    span = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    if graph:
        ws.capture()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    span[0].record(stream)
    for k in range(K):
        if graph:
            ws.replay()
            continue
        if stage_events:
            e = ev[k]
            e[0].record(stream)
            ws.reads()
            e[1].record(stream)
            ws.pileup()
            e[2].record(stream)
            ws.consensus()
            e[3].record(stream)
        else:
            ws.run()
    span[1].record(stream)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    kern = {"step_gpu": span[0].elapsed_time(span[1]) / K}   # ms, the timed steps
    if not graph:
        if not stage_events:   # the stages from a few more steps with all four events
            ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(5)]
            for e in ev:
                e[0].record(stream)
                ws.reads()
                e[1].record(stream)
                ws.pileup()
                e[2].record(stream)
                ws.consensus()
                e[3].record(stream)
            torch.cuda.synchronize(dev)
            kern["breakdown_steps"] = len(ev)
        for name, i0, i1 in (("k_reads", 0, 1), ("k_tile", 1, 2), ("k_consensus", 2, 3), ("step_events", 0, 3)):
            kern[name] = sum(e[i0].elapsed_time(e[i1]) for e in ev) / len(ev)   # ms
    mx = elapsed
    if world > 1:
        v = torch.tensor([elapsed], dtype=torch.float64, device=_coll_device(dev))
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        mx = float(v.item())
    return elapsed, mx, kern


def _coll_device(dev):
    import torch
    import torch.distributed as dist
    return dev if dist.get_backend() == "nccl" else torch.device("cpu")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c5", choices=sorted(WORKLOADS))
    ap.add_argument("--scaling", choices=("both", "strong", "weak"), default="both",
                    help="N>1: strong = one workload split by position across the ranks (the line's value), "
                         "weak = every rank the whole workload on its own GPU (no collective); both (default): "
                         "value = strong, the weak run in the line's 'weak' record")
    ap.add_argument("--shard", action="store_true", help="= --scaling strong")
    ap.add_argument("--independent", action="store_true", help="= --scaling weak")
    ap.add_argument("--no-file-parse", action="store_true", help="skip the timed SAM-file parse (host_parse_s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-scale", type=float, default=0.016)
    ap.add_argument("--no-cpu-mc", action="store_true", help="skip the multi-threaded C baseline")
    ap.add_argument("--cpu-mc-scale", type=float, default=1.0)
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--graph", action="store_true", help="time HIP graph replays of the step")
    ap.add_argument("--stage-events", action="store_true", help="HIP events between all stages in the timed steps")
    ap.add_argument("--rehearse-shards", type=int, default=0, metavar="N",
                    help="N=1 only: also run each of the N position shards of the workload alone on this GPU "
                         "(K steps each) and report their step times (projected N-GPU strong-scaling step)")
    args = ap.parse_args()
    if args.shard:
        args.scaling = "strong"
    elif args.independent:
        args.scaling = "weak"

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))   # (before anything touches the GPU)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.stderr.write("bench.py: --gpus %d but WORLD_SIZE %d\n" % (args.gpus, world))
        sys.exit(2)
    import torch
    import torch.distributed as dist

    from sam2consensus_amd import configs, shard
    from sam2consensus_amd.engine import DeviceBatch, Workspace

    backend = os.environ.get("S2C_DIST_BACKEND", "nccl")
    ndev = max(torch.cuda.device_count(), 1)
    if local >= ndev:
        if backend != "gloo":   # RCCL needs one device per rank
            raise SystemExit("LOCAL_RANK %d but only %d GPUs visible (S2C_DIST_BACKEND=gloo shares devices)" % (local, ndev))
        local %= ndev   # (ranks sharing a device: rehearsals on one GPU, gloo)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from sam2consensus_amd import _lib
    _lib.plan_for_device(dev)   # (the batch plan's grid shaping for this device's CUs)
    if world > 1:
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)
        if dist.get_world_size() != args.gpus:
            sys.stderr.write("bench.py: --gpus %d but the process group has %d ranks\n" % (args.gpus, dist.get_world_size()))
            sys.exit(2)

    wl = args.workload
    opt_args = configs.cli_args(wl)
    thresholds = [0.25]
    min_depth = 1
    if "-c" in opt_args:
        thresholds = [float(x) for x in opt_args[opt_args.index("-c") + 1].split(",")]
    if "-m" in opt_args:
        min_depth = int(opt_args[opt_args.index("-m") + 1])
    T = len(thresholds)
    K = args.steps

    t0 = time.perf_counter()
    full = configs.synth_batch(wl)   # (every rank the same workload: the seed of the goldens)
    full.workload = wl
    t_synth = time.perf_counter() - t0
    file_parse = None
    if world == 1 and not args.no_file_parse:
        file_parse = time_file_parse(wl, full)
    strong = world == 1 or args.scaling in ("strong", "both")
    weak = world > 1 and args.scaling in ("weak", "both")

    line = None
    if strong:
        # N = 1: the whole workload; N > 1: this rank's contiguous tile range of it
        hb = shard.sub_batch(full, rank, world) if world > 1 else full
        ws = Workspace(DeviceBatch(hb, dev), thresholds, min_depth, b"-")
        _, elapsed, kern = timed_steps(ws, K, args.warmup, world, dev, args.graph, args.stage_events)
        parity, exchange = None, None
        if world > 1:
            exchange, res = shard_exchange(ws, hb, full, rank, world, T, dev)
            if not args.no_parity and rank == 0:
                parity = check_parity_result(wl, full, res, thresholds, world)
        elif not args.no_parity:
            parity = check_parity(wl, hb, ws, thresholds)
        if rank == 0:
            line = result_line(wl, full, hb, thresholds, K, args, world, backend, elapsed, kern,
                               "weak" if args.scaling == "weak" else "strong", full.info.aligned_bases)
            line["parity"] = parity
            line["host_parse_s"] = file_parse["parse_s"] if file_parse else None
            line["host_parse"] = file_parse
            line["host_synth_feed_s"] = t_synth
            if exchange is not None:
                exchange["value_with_exchange"] = line["value"] * elapsed / (elapsed + K * exchange["exchange_ms"] * 1e-3)
                exchange["value_with_exchange_what"] = "aligned bases/s if every step's output were gathered: K steps + K exchanges"
                line["exchange"] = exchange
        del ws
        if hb is not full:
            hb.free()
    if weak:
        # every rank the whole workload on its own GPU: per-GPU work fixed as N grows, no
        # collective on the data path (the position shards of an N-times larger genome)
        ws = Workspace(DeviceBatch(full, dev), thresholds, min_depth, b"-")
        _, elapsed, kern = timed_steps(ws, K, args.warmup, world, dev, args.graph, args.stage_events)
        parity = check_parity(wl, full, ws, thresholds) if not args.no_parity and rank == 0 else None
        if rank == 0:
            wline = result_line(wl, full, full, thresholds, K, args, world, backend, elapsed, kern, "weak",
                                world * full.info.aligned_bases)
            wline["parity"] = parity
            if line is None:
                line = wline
                line["host_synth_feed_s"] = t_synth
            else:
                line["weak"] = {k: wline[k] for k in ("value", "ms_per_step", "scaling", "roofline", "kernels_ms",
                                                      "parity", "config")}
                line["weak"]["what"] = ("the same job with every rank running the whole workload on its own GPU "
                                        "(max over ranks of K steps): value = N x its aligned bases / that time")
        del ws

    if rank == 0:
        if world == 1 and args.rehearse_shards > 1:
            line["shard_rehearsal"] = rehearse_shards(full, args.rehearse_shards, thresholds, min_depth, dev,
                                                      args.steps, args.warmup, full.info.aligned_bases)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(wl, args.cpu_sample_scale)
            if not args.no_cpu_mc:
                line["cpu_baseline_mc"] = cpu_baseline_mc(wl, args.cpu_mc_scale)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def shard_exchange(ws, hb, full, rank, world, T, dev):
    """The strong split's exchange after the timed steps, once, on the record: this rank's
    bodies compacted on its GPU and the stats / sizes / bodies gathered to rank 0 straight
    from device memory (shard.gather_device: RCCL reduce / all_gather / gather), merged on
    rank 0's device and copied to the host once; every rank's step times synchronised, the
    max over ranks reported; and the read duplication the position split costs."""
    import torch
    import torch.distributed as dist

    from sam2consensus_amd import shard
    dist.barrier()
    t0 = time.perf_counter()
    tim = {}
    res = shard.gather_device(ws, hb, rank, world, T, timing=tim)
    dist.barrier()
    tim["exchange_s"] = time.perf_counter() - t0
    keys = ["fetch_s", "stats_reduce_s", "meta_s", "body_gather_s", "merge_s", "exchange_s"]
    cd = _coll_device(dev)
    v = torch.tensor([tim.get(k, 0.0) for k in keys], dtype=torch.float64, device=cd)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    dv = torch.tensor([float(hb.info.n_pieces), float(shard.batch_bytes(hb)), float(tim.get("body_gather_bytes", 0))],
                      dtype=torch.float64, device=cd)
    dist.all_reduce(dv, op=dist.ReduceOp.SUM)
    ex = {k.replace("_s", "_ms"): float(x) * 1e3 for k, x in zip(keys, v.tolist())}
    ex.update({"pieces_over_ranks": int(dv[0].item()), "pieces_total": int(full.info.n_pieces),
               "dup_frac": float(dv[0].item()) / max(int(full.info.n_pieces), 1),
               "batch_bytes_over_ranks": int(dv[1].item()), "batch_bytes_total": shard.batch_bytes(full),
               "body_gather_bytes": int(dv[2].item()),
               "what": "after the K steps, once: shard.gather_device (bodies compacted on each GPU, RCCL reduce / "
                       "all_gather / gather from device memory, merged on rank 0's GPU, one pinned D2H), max over "
                       "ranks; dup_frac = pieces summed over the ranks' shards / the workload's"})
    return ex, res


def result_line(wl, full, hb, thresholds, K, args, world, backend, elapsed, kern, scaling, bases):
    """Rank 0's JSON line for one timed run: value = ``bases`` (every rank's units) / the max
    over ranks of the K steps' time."""
    T = len(thresholds)
    sharded = hb is not full
    info = hb.info
    ms = elapsed / K * 1e3
    step_bytes, reads_bytes, tile_bytes = b_alg(full.info, T)
    per_rank = 1.0 / world if sharded else 1.0
    line = {
        "metric": "aligned bases/sec into consensus (1/2/4/8 GPU); HBM GB/s; vs CPU script",
        "value": bases * K / elapsed,
        "unit": "aligned bases/s",
        "n_gpus": world,
        "world_size": world,
        "backend": backend if world > 1 else None,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {"workload": WORKLOADS[wl], "aligned_bases_total": full.info.aligned_bases,
                   "aligned_bases_per_gpu": info.aligned_bases if sharded else full.info.aligned_bases,
                   "reads_per_gpu": info.reads_mapped, "positions_per_gpu": info.total_len,
                   "thresholds": thresholds,
                   "parallelism": ("one workload split into %d contiguous tile ranges, one per GPU; shard bodies and "
                                   "stats gathered to rank 0 after the timed steps" % world if sharded else
                                   "every GPU the whole workload, independently (no collective on the data path)"
                                   if world > 1 else "one GPU, the whole workload")},
    }
    if world > 1:
        line["value_what"] = ("strong scaling: the workload's aligned bases (counted once) / the slowest rank's K "
                              "steps over its shard" if sharded else
                              "weak scaling: N x the workload's aligned bases / the slowest rank's K steps")
    # the roofline's time: the whole step's GPU time in the timed loop (all stages, so an upper
    # bound on the pileup's own; --stage-events: the pileup's own events); rank 0's
    tile_ms = kern["k_tile"] if args.stage_events else kern["step_gpu"]
    achieved = tile_bytes * per_rank / (tile_ms * 1e-3) / 1e9
    traffic = traffic_from_profile(wl)
    bound = bound_from_profile(wl)
    line["roofline"] = {
        "bound": bound.get("bound", "unmeasured"), "bound_evidence": bound.get("evidence"), "achieved": achieved,
        "peak": HBM_PEAK_GBPS, "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic.get("bytes") if traffic else None,
        "traffic_range": traffic.get("range") if traffic else None,
        "traffic_frac": (traffic["bytes"] / (tile_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS) if traffic and not sharded else None,
        "kernel": "s2c_pileup = k_tile_dense + k_tile (CIGAR walk of dense tiles, pileup, insertion "
                  "columns, vote, FASTA bytes); time: HIP events on the launch stream around the K timed steps "
                  "(the whole step's GPU time, every stage: an upper bound on the pileup's)" +
                  ("; rank 0's shard, priced at 1/N of the workload's bytes" if sharded else ""),
        "kernel_ms": tile_ms, "alg_bytes_per_launch": tile_bytes * per_rank,
        "traffic_source": traffic.get("source") if traffic else None}
    line["kernels_ms"] = kern
    if "k_reads" in kern:
        line["kernels_alg_gbps"] = {"k_reads": reads_bytes * per_rank / (kern["k_reads"] * 1e-3) / 1e9,
                                    "k_tile": achieved}
    # SURVEY §8(d)'s formula counts a count tensor written and read (48 B per position) that
    # the fused tile kernels never materialise: reported as bytes only, not as a rate
    line["unfused_step_alg_bytes"] = step_bytes * per_rank
    line["host"] = cpu_model()
    return line


def rehearse_shards(full, n, thresholds, min_depth, dev, K, W, bases):
    """One GPU: each of the n position shards (shard.sub_batch, the N>1 strong split) run
    alone, W warmup + K timed steps each; the projected n-GPU step is the slowest shard's
    (every rank runs its shard concurrently on its own GPU; the gather after the timed loop
    is not part of a step).  The gather is rehearsed as shard.gather_device runs it: each
    shard's bodies compacted on the device (fetch_ms), then rank 0's merge — the shards'
    device bodies ordered on the device and copied to the host once (merge_ms)."""
    import torch

    from sam2consensus_amd import shard
    from sam2consensus_amd.engine import DeviceBatch, Workspace, to_host
    ms, fetch_ms, parts, bodies, subs_info, stats = [], [], [], [], [], None
    for r in range(n):
        sub = shard.sub_batch(full, r, n)
        ws = Workspace(DeviceBatch(sub, dev), thresholds, min_depth, b"-")
        for _ in range(W):
            ws.run()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(K):
            ws.run()
        torch.cuda.synchronize(dev)
        ms.append((time.perf_counter() - t0) / K * 1e3)
        t0 = time.perf_counter()
        st, offs, body = ws.fetch_device()   # (a rank's exchange starts here: compaction on its GPU)
        torch.cuda.synchronize(dev)
        fetch_ms.append((time.perf_counter() - t0) * 1e3)
        stats = st if stats is None else stats + st
        parts.append((sub.t0, sub.t1, offs))
        bodies.append(body)
        subs_info.append(sub)
        del ws
    vol = shard.exchange_volumes(full, subs_info)
    for sub in subs_info:
        sub.free()

    def merge():   # rank 0's merge of the gathered bodies: ordered on the device, one pinned D2H
        full_offs, segs = shard.merge_plan(parts, len(thresholds))
        pieces = [bodies[k][a:b] for k, a, b in segs if b > a]
        return full_offs, (to_host(torch.cat(pieces)) if pieces else b"")
    merge_first_ms = []
    for _ in range(2):   # (a process's first merge pays its one-time costs: the concatenation kernel's
        torch.cuda.synchronize(dev)   # load, the pinned block's allocation; reported apart)
        t0 = time.perf_counter()
        full_offs, merged = merge()
        merge_first_ms.append((time.perf_counter() - t0) * 1e3)
        if len(merge_first_ms) == 1:
            del merged
    merge_ms = merge_first_ms[-1]
    body = sum(int(b.numel()) + 8 * len(p[2]) for b, p in zip(bodies, parts))
    # rank 0 receives every other rank's bodies over its own xGMI link (≈153 GB/s per link,
    # 7 per GPU: priced at half of that, one direction): the largest rank's share over one link
    link_ms = max(int(b.numel()) + 8 * len(p[2]) for b, p in zip(bodies, parts)) / 76.5e9 * 1e3
    gather_ms = max(fetch_ms) + link_ms + merge_ms
    worst = max(ms)
    check = None
    g = _golden(full_wl(full))
    if g and g.get("files"):
        got = _files(full, thresholds, g["sam_file"].split(".")[0], stats, full_offs, merged, 0)
        check = got == {k: v["sha256"] for k, v in g["files"].items()}
    return {"shards": n, "ms_per_step": ms, "projected_ms_per_step": worst,
            "projected_value": bases / (worst * 1e-3),
            "fetch_ms": fetch_ms, "merge_ms": merge_ms, "merge_first_ms": merge_first_ms[0], "body_bytes": body,
            "gather_link_ms_est": link_ms,
            "gather_ms": gather_ms, "dup_frac": vol["dup_frac"], "exchange_volumes": vol,
            "merged_matches_golden": check,
            "projected_value_with_gather": bases / ((worst + gather_ms) * 1e-3),
            "what": "each shard of the %d-way position split run alone on one GPU; projected step = the slowest "
                    "shard's (wall clock over K steps, launches included); gather_ms = the slowest shard's fetch "
                    "(its bodies compacted on the device, stats and lengths to the host) + its bodies over one xGMI "
                    "link at 76.5 GB/s (estimated) + rank 0's merge (the shards' bodies ordered on the device, one "
                    "pinned D2H; measured warm — merge_first_ms: the process's first, with the one-time costs), once "
                    "per job: projected_value_with_gather charges it to every step" % n}


def full_wl(full):
    return getattr(full, "workload", None)


def bound_from_profile(wl):
    """What bounds the dominant kernel, from the committed PMC summary (scripts/bound.py):
    "valu" when its VALU instructions alone take most of its time, else "hbm"; with no
    committed summary for the workload the line says "unmeasured" (no claim without evidence)."""
    p = os.path.join(ROOT, "profiles", "bound_%s.json" % wl)
    if os.path.exists(p):
        with open(p) as fh:
            return json.load(fh)
    return {}


def time_file_parse(wl, ref_hb):
    """North_star's separately reported host SAM parse: the workload's SAM text written to a
    file (not timed), then parsed from it by the product parser (libs2c.so, threaded) into the
    packed batch; its counters must equal the batch the bench runs."""
    import tempfile

    from sam2consensus_amd import configs
    from sam2consensus_amd.batch import parse_file
    td = tempfile.mkdtemp(prefix="s2c_parse_")
    path = os.path.join(td, wl + ".sam")
    try:
        t0 = time.perf_counter()
        configs.synth_write(wl, path)
        tw = time.perf_counter() - t0
        size = os.path.getsize(path)
        runs, same = [], True
        for _ in range(2):   # (the first right after the write, while its pages are flushed)
            t0 = time.perf_counter()
            hb = parse_file(path, configs.maxdel_active(configs.cli_args(wl)), 150)
            runs.append(time.perf_counter() - t0)
            same = same and (hb.info.reads_mapped == ref_hb.info.reads_mapped and hb.info.aligned_bases == ref_hb.info.aligned_bases
                             and hb.info.n_tiles == ref_hb.info.n_tiles)
            hb.free()
        tp = min(runs)
    finally:
        try:
            os.remove(path)
            os.rmdir(td)
        except OSError:
            pass
    return {"parse_s": tp, "runs_s": runs, "file_bytes": size, "file_mb_per_s": size / tp / 1e6, "threads": cpu_threads(),
            "write_s": tw, "same_batch": same,
            "what": "libs2c.so s2c_parser_feed_file of the workload's .sam (read, parse, pack, plan) on %d threads, "
                    "best of %d runs (runs_s)" % (cpu_threads(), len(runs))}


def traffic_from_profile(wl):
    """Per-launch HBM bytes of the dominant tile kernel from the committed PMC pass, or None."""
    p = os.path.join(ROOT, "profiles", "traffic_%s.json" % wl)
    if os.path.exists(p):
        with open(p) as fh:
            t = json.load(fh)
        b = t.get("tile_hbm_bytes_per_launch")
        if b:
            return {"bytes": b, "range": t.get("tile_hbm_bytes_range"),
                    "source": "profiles/traffic_%s.json (%s)" % (wl, t.get("round", ""))}
    return None


def _files(hb, thresholds, prefix, stats, offs, out, n):
    import hashlib

    from sam2consensus_amd.records import build_records, render
    recs = build_records(hb, thresholds, prefix, stats, offs, out)
    return {name + "__" + prefix + ".fasta": hashlib.sha256(render(r, n)).hexdigest() for name, r in recs.items()}


def _golden(wl):
    gpath = os.path.join(ROOT, "tests", "golden", "configs.json")
    if not os.path.exists(gpath):
        return None
    return json.load(open(gpath)).get(wl)


def check_parity(wl, hb, ws, thresholds):
    """Rank 0 runs the default seed: compare the step's FASTA files with the reference's."""
    from sam2consensus_amd import configs
    g = _golden(wl)
    if not g:
        return None
    a = configs.cli_args(wl)
    n = int(a[a.index("-n") + 1]) if "-n" in a else 0
    got = _files(hb, thresholds, g["sam_file"].split(".")[0], *ws.fetch(), n)
    want = {k: v["sha256"] for k, v in g["files"].items()}
    return "byte-identical to reference (%d files)" % len(want) if got == want else "MISMATCH"


def check_parity_result(wl, full, res, thresholds, world):
    """Rank 0: the shards' results gathered (RCCL) and merged, compared with the golden."""
    g = _golden(wl)
    if not g:
        return None
    got = _files(full, thresholds, g["sam_file"].split(".")[0], *res, 0)
    want = {k: v["sha256"] for k, v in g["files"].items()}
    return "byte-identical to reference (%d files, %d shards)" % (len(want), world) if got == want else "MISMATCH"


if __name__ == "__main__":
    main()
