"""Position-range sharding of a packed batch across GPUs (one process per GPU).

North_star partitioning: the global coordinate (references concatenated in header order)
is cut into contiguous tile ranges of roughly equal work; each rank gets the sub-batch of
its tiles (``s2c_batch_shard``: the pieces whose runs can cover them — short pieces
starting up to kwin + 1 words before, the long pieces listed for them — and the pieces
whose insertion events are keyed inside them).  A position's counts depend only on the
runs covering it, so every rank computes the unsharded counts of its tiles: no count
exchange.  The exchange steps are real and small, over the process group (RCCL on GPUs):
an all-reduce of the per-(reference, threshold) record statistics (:352-397) of references
cut by a boundary, and an all-gather of the FASTA body bytes (length-prefixed tensors), from
which rank 0 writes the files.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .batch import HostBatch


def tile_weights(hb):
    """Work estimate per tile: its words' candidate run slots plus a vote term per 32 positions."""
    i = hb.info
    if not i.n_tiles:
        return np.zeros(0, np.float64)
    rs = hb.rs.astype(np.float64)
    a = hb.tiles[:, 0].astype(np.int64)
    b = hb.tiles[:, 1].astype(np.int64)
    K = int(i.kwin)
    w0, w1 = a >> 5, (b + 31) >> 5
    return (K + 1) * (rs[w1] - rs[np.maximum(w0 - K, 0)]) + (b - a) / 32.0


def split_tiles(hb, world):
    """Contiguous tile ranges [(t0, t1)] with ≈ equal weight (a rank may get none)."""
    nt = hb.info.n_tiles
    if world <= 1 or nt == 0:
        return [(0, nt)] + [(nt, nt)] * max(0, world - 1)
    c = np.cumsum(tile_weights(hb))
    tot = c[-1]
    cuts = [0]
    for k in range(1, world):
        cuts.append(int(np.searchsorted(c, tot * k / world)))
    cuts.append(nt)
    cuts = [min(max(x, 0), nt) for x in cuts]
    for k in range(1, len(cuts)):
        cuts[k] = max(cuts[k], cuts[k - 1])
    return [(cuts[k], cuts[k + 1]) for k in range(world)]


def sub_batch(hb, rank, world):
    """This rank's sub-batch (a HostBatch of its tile range); .t0/.t1 give the range."""
    t0, t1 = split_tiles(hb, world)[rank]
    h = C.c_void_p()
    L.check(L.lib.s2c_batch_shard(hb._b, t0, t1, C.byref(h)))
    sub = HostBatch(h)
    sub.t0, sub.t1 = t0, t1
    sub.parent_tiles = hb.info.n_tiles
    sub.maxdel_active, sub.maxdel = getattr(hb, "maxdel_active", True), getattr(hb, "maxdel", 150)
    return sub


def merge_plan(parts, T):
    """Rank results [(t0, t1, offs)] → (offs of the whole batch, segments): the merged body
    is, in [t][tile] order, the concatenation of part k's bytes [a, b) over the segments
    (k, a, b) — k indexes ``parts`` as given."""
    order = sorted(range(len(parts)), key=lambda k: parts[k][0])
    nb = max(p[1] for p in parts) if parts else 0
    lens = np.zeros(T * nb, np.int64)
    segs = []
    for t in range(T):
        for k in order:
            t0, t1, offs = parts[k][:3]
            nbr = t1 - t0
            a, b = int(offs[t * nbr]), int(offs[t * nbr + nbr])
            segs.append((k, a, b))
            lens[t * nb + t0:t * nb + t1] = np.diff(np.asarray(offs[t * nbr:t * nbr + nbr + 1]).astype(np.int64))
    full = np.zeros(T * nb + 1, np.uint64)
    full[1:] = np.cumsum(lens)
    return full, segs


def merge_outputs(parts, T):
    """Rank outputs [(t0, t1, offs, out)] → (offs, out) of the whole batch, [t][tile] order."""
    full, segs = merge_plan(parts, T)
    return full, b"".join(parts[k][3][a:b] for k, a, b in segs)


def force_collectives():
    """S2C_FORCE_COLLECTIVES=1: run the exchange collectives even at world size 1 (they are
    skipped there otherwise) — how a one-GPU box executes the RCCL path once
    (tests/test_gpu.py::test_rccl_exchange_at_world_one)."""
    import os
    return os.environ.get("S2C_FORCE_COLLECTIVES", "0") not in ("", "0")


def _tensor_device(group):
    import torch
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def gather_results(fetched, sub, rank, world, T, group=None, timing=None):
    """Merge every rank's (stats, offs, out) on rank 0 with tensor collectives: a reduce of
    the stats, an all-gather of (tile range, sizes) (four numbers per rank), then a gather of
    the padded offsets and body bytes to rank 0 only (no other rank holds every body).
    Returns the whole batch's (stats, offs, out) on rank 0, None elsewhere.  ``timing``: a dict
    that gets this rank's seconds per exchange step (stats_reduce, meta, body_gather, merge;
    device work synchronised) and the bytes each step moved from this rank."""
    import time

    import torch
    import torch.distributed as dist

    stats, offs, out = fetched
    dev = _tensor_device(group)

    def mark(name, t0, nbytes=None):
        if timing is None:
            return time.perf_counter()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        timing[name + "_s"] = timing.get(name + "_s", 0.0) + (t1 - t0)
        if nbytes is not None:
            timing[name + "_bytes"] = int(nbytes)
        return t1

    t0 = mark("start", time.perf_counter())
    st = torch.from_numpy(np.ascontiguousarray(stats).view(np.int64).copy()).to(dev)
    coll = world > 1 or force_collectives()
    if coll:
        dist.reduce(st, dst=0, op=dist.ReduceOp.SUM, group=group)   # record stats of cut references
    t0 = mark("stats_reduce", t0, st.numel() * 8)
    offs = np.asarray(offs, dtype=np.uint64)
    meta = torch.tensor([sub.t0, sub.t1, len(offs), len(out)], dtype=torch.int64, device=dev)
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group) if coll else metas.__setitem__(0, meta)
    metas = [m.cpu().tolist() for m in metas]
    t0 = mark("meta", t0, 32)
    mo = max(m[2] for m in metas)
    mb = max(max(m[3] for m in metas), 1)
    o_t = torch.zeros(mo, dtype=torch.int64, device=dev)
    o_t[: len(offs)] = torch.from_numpy(offs.view(np.int64).copy()).to(dev)
    b_t = torch.zeros(mb, dtype=torch.uint8, device=dev)
    if len(out):
        b_t[: len(out)] = torch.from_numpy(np.frombuffer(out, dtype=np.uint8).copy()).to(dev)
    if coll:
        os_ = [torch.empty_like(o_t) for _ in range(world)] if rank == 0 else None
        bs_ = [torch.empty_like(b_t) for _ in range(world)] if rank == 0 else None
        dist.gather(o_t, os_, dst=0, group=group)
        dist.gather(b_t, bs_, dst=0, group=group)
    else:
        os_, bs_ = [o_t], [b_t]
    t0 = mark("body_gather", t0, o_t.numel() * 8 + b_t.numel())
    if rank != 0:
        return None
    parts = []
    for m, o, b in zip(metas, os_, bs_):
        parts.append((m[0], m[1], o[: m[2]].cpu().numpy().view(np.uint64), b[: m[3]].cpu().numpy().tobytes()))
    full_offs, full_out = merge_outputs(parts, T)
    res = st.cpu().numpy().view(np.uint64).reshape(stats.shape), full_offs, full_out
    mark("merge", t0)
    return res


def gather_device(ws, sub, rank, world, T, group=None, timing=None):
    """``gather_results`` for a rank whose results are still on its GPU (``Workspace``): the
    bodies are compacted on the device (``Workspace.fetch_device``, s2c_gather_bodies_dev) and
    gathered to rank 0 straight from device memory — only the statistics and the body
    lengths cross to the host before the collectives.  Rank 0 orders the shards' bodies on its
    device and copies the merged bodies to the host once (pinned).  Collectives: a reduce of
    the stats, an all-gather of (tile range, sizes), a gather of the padded offsets and of the
    padded body bytes.  Returns (stats, offs, out) of the whole batch on rank 0, None
    elsewhere.  ``timing``: this rank's seconds per step (fetch, stats_reduce, meta,
    body_gather, merge; device work synchronised) and the bytes each step moved."""
    import time

    import torch
    import torch.distributed as dist

    from .engine import to_host

    t0 = time.perf_counter()
    stats, offs, body = ws.fetch_device()
    dev = _tensor_device(group)

    def mark(name, t0, nbytes=None):
        if timing is None:
            return time.perf_counter()
        torch.cuda.synchronize(body.device)
        if dev.type == "cuda" and dev != body.device:
            torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        timing[name + "_s"] = timing.get(name + "_s", 0.0) + (t1 - t0)
        if nbytes is not None:
            timing[name + "_bytes"] = int(nbytes)
        return t1

    t0 = mark("fetch", t0, body.numel())
    st = torch.from_numpy(np.ascontiguousarray(stats).view(np.int64).copy()).to(dev)
    coll = world > 1 or force_collectives()
    if coll:
        dist.reduce(st, dst=0, op=dist.ReduceOp.SUM, group=group)   # record stats of cut references
    t0 = mark("stats_reduce", t0, st.numel() * 8)
    offs = np.asarray(offs, dtype=np.uint64)
    meta = torch.tensor([sub.t0, sub.t1, len(offs), int(body.numel())], dtype=torch.int64, device=dev)
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group) if coll else metas.__setitem__(0, meta)
    metas = [m.cpu().tolist() for m in metas]
    t0 = mark("meta", t0, 32)
    mo = max(m[2] for m in metas)
    mb = max(max(m[3] for m in metas), 16)
    o_t = torch.zeros(mo, dtype=torch.int64, device=dev)
    o_t[: len(offs)] = torch.from_numpy(offs.view(np.int64).copy()).to(dev)
    src = body if dev == body.device else body.to(dev)
    if src.numel() == mb:
        b_t = src
    else:   # (the gather moves equal sizes: padded on the device)
        b_t = torch.empty(mb, dtype=torch.uint8, device=dev)
        b_t[: src.numel()] = src
    if coll:
        os_ = [torch.empty_like(o_t) for _ in range(world)] if rank == 0 else None
        bs_ = [torch.empty_like(b_t) for _ in range(world)] if rank == 0 else None
        dist.gather(o_t, os_, dst=0, group=group)
        dist.gather(b_t, bs_, dst=0, group=group)
    else:
        os_, bs_ = [o_t], [b_t]
    t0 = mark("body_gather", t0, o_t.numel() * 8 + b_t.numel())
    if rank != 0:
        return None
    parts = [(m[0], m[1], o[: m[2]].cpu().numpy().view(np.uint64)) for m, o in zip(metas, os_)]
    full_offs, segs = merge_plan(parts, T)
    pieces = [bs_[k][a:b] for k, a, b in segs if b > a]
    merged = torch.cat(pieces) if pieces else torch.empty(0, dtype=torch.uint8, device=dev)
    full_out = to_host(merged)
    res = st.cpu().numpy().view(np.uint64).reshape(stats.shape), full_offs, full_out
    mark("merge", t0, len(full_out))
    return res


def batch_bytes(hb):
    """Bytes of a packed batch's device arrays (what its rank uploads to HBM; the per-word
    arrays over its word span only)."""
    return int(sum(np.asarray(hb.device_view(n)).nbytes for n in
                   ("pc", "ops", "bq", "bx", "rs", "tiles", "items", "dense", "deep", "lp", "wtile", "rlist", "ps", "px",
                    "dwin")))


def exchange_volumes(full, subs):
    """What the position split costs in data, from the shards themselves:
    duplicated pieces / bytes (a read whose runs reach across a cut is in both shards' batches)
    against what north_star's count-tensor merge would move instead — a reduce-scatter of the
    u32 counts [6] of the positions that straddling reads cover past each cut (kwin + 1 words
    on either side: 24 B per position)."""
    np_full = int(full.info.n_pieces)
    np_sum = sum(int(s.info.n_pieces) for s in subs)
    b_full = batch_bytes(full)
    b_sum = sum(batch_bytes(s) for s in subs)
    cuts = sum(1 for s in subs[:-1] if s.t1 < full.info.n_tiles)
    seam_pos = 2 * (int(full.info.kwin) + 1) * 32
    return {"pieces_total": np_full, "pieces_over_shards": np_sum,
            "dup_frac": (np_sum / np_full) if np_full else 1.0,
            "batch_bytes_total": b_full, "batch_bytes_over_shards": b_sum,
            "dup_bytes": b_sum - b_full,
            "cuts": cuts, "count_merge_bytes": cuts * seam_pos * 24}
