"""Position-range sharding of a packed batch across GPUs (one process per GPU).

North_star partitioning: the global coordinate (references concatenated in header
order) is cut into contiguous tile ranges of roughly equal aligned bases; each rank gets
its tiles, the reads that overlap them (a contiguous range of the position-sorted reads
plus any long reads they list), and the insertion events keyed inside them.  Tiles pull
every read that covers them, so straddling reads are simply read by both neighbours —
no count exchange is needed.  The one real exchange step is the per-(reference,
threshold) record statistics (:352-397) of references cut by a shard boundary: an
all-reduce of a [R, T, 4] u64 tensor.  FASTA body bytes are gathered to rank 0, which
formats and writes the files.

Positions keep their global coordinates on every rank (position-indexed buffers are
sized to the whole batch; read/op/base/insertion arrays are sliced and re-indexed).
"""
from __future__ import annotations

import numpy as np

from . import _lib as L


class SubBatch:
    """Duck-types HostBatch for DeviceBatch/Workspace and the record builder."""

    def __init__(self, hb, t0, t1):
        i = hb.info
        self.parent = hb
        self.t0, self.t1 = t0, t1
        info = L.BatchInfo()
        for name, _ in L.BatchInfo._fields_:
            setattr(info, name, getattr(i, name))
        items = hb.items
        sel = (items[:, 7] >= t0) & (items[:, 7] < t1)
        it = items[sel].copy()
        n_short = int(i.n_reads - i.n_long)
        if len(it):
            r_lo = int(it[:, 2].min())
            r_hi = int(it[:, 3].max())
        else:
            r_lo = r_hi = 0
        r_hi = max(r_hi, r_lo)
        # long reads referenced by these items' extras
        xs = []
        for row in it:
            xs.extend(int(x) for x in hb.extras[int(row[4]):int(row[5])])
        longs = sorted(set(xs))
        reads = np.concatenate([np.arange(r_lo, r_hi, dtype=np.int64), np.asarray(longs, dtype=np.int64)])
        remap = {r: k for k, r in enumerate(longs, start=r_hi - r_lo)}
        # reads: positions global; ops / bases sliced
        self.rd_pos = hb.rd_pos[reads].copy() if len(reads) else np.zeros(0, np.uint32)
        self.rd_span = hb.rd_span[reads].copy() if len(reads) else np.zeros(0, np.uint32)
        op_lo = hb.rd_op[reads].astype(np.int64)
        op_hi = hb.rd_op[reads + 1].astype(np.int64)
        b_lo = hb.rd_base[reads].astype(np.int64)
        b_hi = hb.rd_base[reads + 1].astype(np.int64)
        op_len, b_len = op_hi - op_lo, b_hi - b_lo
        self.rd_op = np.zeros(len(reads) + 1, np.uint32)
        self.rd_op[1:] = np.cumsum(op_len)
        self.rd_base = np.zeros(len(reads) + 1, np.uint32)
        self.rd_base[1:] = np.cumsum(b_len)
        self.ops = np.concatenate([hb.ops[a:b] for a, b in zip(op_lo, op_hi)]) if len(reads) else np.zeros(0, np.uint32)
        self.bases = (np.concatenate([hb.bases[a:b] for a, b in zip(b_lo, b_hi)]) if len(reads)
                      else np.zeros(0, np.uint32))
        # kernel read records {start, span|flags, base word, op offset} + sentinel
        self.rd_meta = np.zeros((len(reads) + 1, 4), np.uint32)
        self.rd_meta[:-1, 0] = self.rd_pos
        self.rd_meta[:-1, 1] = self.rd_span
        self.rd_meta[:, 2] = self.rd_base
        self.rd_meta[:, 3] = self.rd_op
        # per-word short-read ranges, re-indexed to this shard's read window
        n_sub = r_hi - r_lo
        self.word_lo = np.clip(hb.word_lo.astype(np.int64) - r_lo, 0, n_sub).astype(np.uint32)
        self.word_hi = np.maximum(np.clip(hb.word_hi.astype(np.int64) - r_lo, 0, n_sub),
                                  self.word_lo).astype(np.uint32)
        # items / extras re-indexed
        extras = []
        for row in it:
            xl = len(extras)
            extras.extend(remap[int(x)] for x in hb.extras[int(row[4]):int(row[5])])
            row[4], row[5] = xl, len(extras)
            row[2] -= r_lo
            row[3] -= r_lo
            row[7] -= t0
        self.items = it.astype(np.uint32)
        self.extras = np.asarray(extras, dtype=np.uint32)
        self.blocks = hb.blocks[t0:t1].copy()
        self.deep = (hb.deep[(hb.deep >= t0) & (hb.deep < t1)] - t0).astype(np.uint32)
        # insertion events keyed inside [A, B)
        A = int(self.blocks[0, 0]) if len(self.blocks) else 0
        B = int(self.blocks[-1, 1]) if len(self.blocks) else 0
        keep = np.nonzero((hb.ins_key >= A) & (hb.ins_key < B))[0]
        self.ins_key = hb.ins_key[keep].copy()
        lens = (hb.ins_off[keep + 1].astype(np.int64) - hb.ins_off[keep].astype(np.int64))
        self.ins_off = np.zeros(len(keep) + 1, np.uint32)
        self.ins_off[1:] = np.cumsum(lens)
        nib_all = _unpack_nibbles(hb.ins_bases, int(hb.ins_off[-1]) if len(hb.ins_off) else 0)
        nibs = (np.concatenate([nib_all[int(hb.ins_off[e]):int(hb.ins_off[e + 1])] for e in keep])
                if len(keep) else np.zeros(0, np.uint8))
        self.ins_bases = _pack_nibbles(nibs)
        # info
        info.n_reads = len(reads)
        info.n_long = len(longs)
        info.n_ops = len(self.ops)
        info.n_base_words = len(self.bases)
        info.n_items = len(self.items)
        info.n_extras = len(self.extras)
        info.n_blocks = len(self.blocks)
        info.n_deep = len(self.deep)
        info.n_ins = len(keep)
        info.n_ins_bases = int(self.ins_off[-1])
        info.n_ins_words = len(self.ins_bases)
        info.tile_max = int((self.blocks[:, 1] - self.blocks[:, 0]).max()) if len(self.blocks) else 64
        # aligned bases counted by this shard (the metric's units): seqout chars in its tiles
        self.info = info
        self.names = hb.names
        self.ref_len, self.ref_off = hb.ref_len, hb.ref_off
        self.ref_reads = hb.ref_reads

    @property
    def aligned_bases(self):
        return int(self.info.aligned_bases)


def _unpack_nibbles(words, n):
    w = np.asarray(words, dtype=np.uint32)
    if n == 0:
        return np.zeros(0, np.uint8)
    sh = (np.arange(8, dtype=np.uint32) * 4)
    return ((w[:, None] >> sh[None, :]) & 15).astype(np.uint8).reshape(-1)[:n]


def _pack_nibbles(nibs):
    n = len(nibs)
    if n == 0:
        return np.zeros(0, np.uint32)
    pad = np.zeros((n + 7) // 8 * 8, np.uint32)
    pad[:n] = nibs
    sh = (np.arange(8, dtype=np.uint32) * 4)
    return (pad.reshape(-1, 8) << sh[None, :]).sum(axis=1, dtype=np.uint64).astype(np.uint32)


def tile_weights(hb):
    """Aligned-base estimate per tile: Σ over its items of reads × mean span."""
    nt = hb.info.n_blocks
    w = np.zeros(nt, np.float64)
    if hb.info.n_items:
        span = np.maximum(1, (hb.rd_span & 0x3FFFFFFF).mean() if hb.info.n_reads else 1)
        np.add.at(w, hb.items[:, 7].astype(np.int64),
                  (hb.items[:, 3].astype(np.float64) - hb.items[:, 2]) * float(span))
    w += (hb.blocks[:, 1].astype(np.float64) - hb.blocks[:, 0]) * 1.0   # vote cost per position
    return w


def split_tiles(hb, world):
    """Contiguous tile ranges [(t0, t1)] with ≈ equal weight (a rank may get none)."""
    nt = hb.info.n_blocks
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


def merge_outputs(parts, T):
    """Rank outputs [(t0, t1, offs, out)] → (offs, out) of the whole batch, [t][block] order."""
    parts = sorted(parts, key=lambda p: p[0])
    nb = max(p[1] for p in parts) if parts else 0
    lens = np.zeros(T * nb, np.int64)
    chunks = [[b""] * len(parts) for _ in range(T)]
    for k, (t0, t1, offs, out) in enumerate(parts):
        nbr = t1 - t0
        for t in range(T):
            a, b = int(offs[t * nbr]), int(offs[t * nbr + nbr])
            chunks[t][k] = out[a:b]
            lens[t * nb + t0:t * nb + t1] = np.diff(offs[t * nbr:t * nbr + nbr + 1].astype(np.int64))
    full = np.zeros(T * nb + 1, np.uint64)
    full[1:] = np.cumsum(lens)
    return full, b"".join(b"".join(chunks[t]) for t in range(T))


def run_sharded(hb, rank, world, thresholds, runner, group=None):
    """Run this rank's shard with ``runner(sub) -> (stats, offs, out)``; all-reduce stats,
    gather outputs to rank 0.  Returns (stats, offs, out) of the whole batch on rank 0,
    None elsewhere."""
    import torch
    import torch.distributed as dist

    t0, t1 = split_tiles(hb, world)[rank]
    sub = SubBatch(hb, t0, t1)
    stats, offs, out = runner(sub)
    st = torch.from_numpy(np.ascontiguousarray(stats).view(np.int64).copy())
    if world > 1:
        dev = st
        backend = dist.get_backend(group)
        if backend == "nccl":
            dev = st.cuda()
        dist.all_reduce(dev, op=dist.ReduceOp.SUM, group=group)   # record stats of cut references
        st = dev.cpu()
        gathered = [None] * world if rank == 0 else None
        dist.gather_object((t0, t1, np.asarray(offs), out), gathered, dst=0, group=group)
    else:
        gathered = [(t0, t1, np.asarray(offs), out)]
    if rank != 0:
        return None
    full_offs, full_out = merge_outputs(gathered, len(thresholds))
    return st.numpy().view(np.uint64).reshape(stats.shape), full_offs, full_out
