"""Position-range sharding of a packed batch across GPUs (one process per GPU).

North_star partitioning: the global coordinate (references concatenated in header
order) is cut into contiguous tile ranges of roughly equal work; each rank gets its
tiles, the word-major seqout records of their words (one contiguous slice: a read that
straddles a shard boundary already has one record per word, so each side holds its own
part — no count exchange is needed), and the insertion events keyed inside them.  The one real exchange step is the per-(reference,
threshold) record statistics (:352-397) of references cut by a shard boundary: an
all-reduce of a [R, T, 4] u64 tensor.  FASTA body bytes are gathered to rank 0, which
formats and writes the files.

Positions keep their global coordinates on every rank (position-indexed buffers are
sized to the whole batch; record and insertion arrays are sliced and re-indexed).
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
        self.blocks = hb.blocks[t0:t1].copy()
        sel = np.nonzero((hb.items[:, 3] >= t0) & (hb.items[:, 3] < t1))[0]
        it = hb.items[sel].astype(np.int64)
        # the items' placeholder words and '-'/'N' entries are contiguous ranges: slice, rebase
        i0, i1 = (int(sel[0]), int(sel[-1]) + 1) if len(sel) else (0, 0)
        nfix_all = np.append(hb.items[:, 4].astype(np.int64), hb.info.n_fix)
        f0, f1 = int(nfix_all[i0]), int(nfix_all[i1])
        x0 = int(hb.items[i0, 5]) if len(sel) else 0
        x1 = int(hb.items[i1 - 1, 6]) if len(sel) else 0
        self.fix = hb.fix[f0:f1].copy()
        self.exc = hb.exc[x0:x1].copy()
        it[:, 3] -= t0
        it[:, 4] -= f0
        it[:, 5:7] -= x0
        self._items64 = it   # the copied block words 8-13 and rbase are re-based below
        nwp = hb.info.n_iwr // max(hb.info.n_items, 1) // 2
        iw = hb.iwr.reshape(-1, nwp, 2)[sel].astype(np.int64)
        self.deep = (hb.deep[(hb.deep >= t0) & (hb.deep < t1)] - t0).astype(np.uint32)
        A = int(self.blocks[0, 0]) if len(self.blocks) else 0
        B = int(self.blocks[-1, 1]) if len(self.blocks) else 0
        # the records of the shard's words are contiguous: slice them, rebase the CSR
        # (positions stay global; words outside the shard get empty ranges)
        wrec = hb.wrec.astype(np.int64)
        r0, r1 = int(wrec[A >> 5]), int(wrec[(B + 31) >> 5])
        self.recs = hb.recs[r0:r1].copy()
        self.wrec = np.clip(wrec - r0, 0, r1 - r0).astype(np.uint32)
        live = iw[:, :, 1] > iw[:, :, 0]   # words past a tile keep {0, 0}
        iw = np.where(live[:, :, None], iw - r0, 0)
        self.iwr = iw.astype(np.uint32).reshape(-1)
        self._items64[:, 14] -= r0
        # the read-piece table stays with the parent (host-side only)
        self.rd_pos = self.rd_span = np.zeros(0, np.uint32)
        self.rd_op = np.zeros(1, np.uint32)
        self.ops = np.zeros(0, np.uint32)
        # insertion keys inside [A, B): a contiguous key range (keys ascending), hence
        # contiguous events and columns; re-based, the bitmap cleared outside the shard
        k0, k1 = (int(x) for x in np.searchsorted(hb.ins_key, [A, B]))
        koff, kcol = hb.ins_koff.astype(np.int64), hb.ins_kcol.astype(np.int64)
        e0, e1 = int(koff[k0]), int(koff[k1])
        self.ins_key = hb.ins_key[k0:k1].copy()
        self.ins_koff = (koff[k0:k1 + 1] - e0).astype(np.uint32)
        self.ins_kcol = (kcol[k0:k1 + 1] - kcol[k0]).astype(np.uint32)
        off = hb.ins_off.astype(np.int64)
        self.ins_off = (off[e0:e1 + 1] - off[e0]).astype(np.uint32)
        nib_all = _unpack_nibbles(hb.ins_bases, int(off[-1]))
        self.ins_bases = _pack_nibbles(nib_all[int(off[e0]):int(off[e1])])
        self.ins_ekey = (hb.ins_ekey[e0:e1].astype(np.int64) - k0).astype(np.uint32)
        # device records: event column offsets are tile-relative (unchanged), nibble offsets
        # and key columns rebase; the tiles' key/event/column ranges (block words 4-9) too
        ev = hb.ins_ev[e0:e1].astype(np.int64)
        ev[:, 2] -= int(off[e0])
        self.ins_ev = ev.astype(np.uint32).reshape(-1, 4)
        ki = hb.ins_kinfo[k0:k1].astype(np.int64)
        ki[:, 1] -= int(kcol[k0])
        self.ins_kinfo = ki.astype(np.uint32).reshape(-1, 4)
        bl = self.blocks.astype(np.int64)
        bl[:, 4:6] -= k0
        bl[:, 6:8] -= e0
        bl[:, 8:10] -= int(kcol[k0])
        self.blocks = bl.astype(np.uint32)
        it = self._items64
        it[:, 7:14] = bl[it[:, 3], 3:10]   # the items' copies of their tiles' block words
        self.items = it.astype(np.uint32)
        del self._items64
        bits = np.zeros_like(hb.ins_bits)
        wa, wb = A >> 5, (B + 31) >> 5
        bits[wa:wb] = hb.ins_bits[wa:wb]
        self.ins_bits = bits
        self.ins_rank = np.clip(hb.ins_rank.astype(np.int64) - k0, 0, k1 - k0).astype(np.uint32)
        info.n_reads = 0
        info.n_ops = 0
        info.n_recs = len(self.recs)
        info.n_items = len(self.items)
        info.n_blocks = len(self.blocks)
        info.n_deep = len(self.deep)
        info.n_exc = len(self.exc)
        info.n_fix = len(self.fix)
        info.n_iwr = len(self.iwr)
        info.n_ins = e1 - e0
        info.n_ins_bases = int(self.ins_off[-1])
        info.n_ins_words = len(self.ins_bases)
        info.n_keys = k1 - k0
        info.n_cols = int(self.ins_kcol[-1])
        # tile_max and chunk_recs stay the parent's: the items' chunk indices and the per-item
        # word ranges (iwr) are laid out for the parent's words per tile
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
    """Work estimate per tile: the seqout records of its words (one 12-B load + one
    count each) plus a vote term per 32 positions."""
    if not hb.info.n_blocks:
        return np.zeros(0, np.float64)
    wrec = hb.wrec.astype(np.float64)
    a = hb.blocks[:, 0].astype(np.int64)
    b = hb.blocks[:, 1].astype(np.int64)
    return wrec[(b + 31) >> 5] - wrec[a >> 5] + (b - a) / 32.0


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
