"""Device side: packed batch → HBM, workspace, the HIP stages, results → host.

PyTorch is used only as the device allocator / stream provider; all compute is
libs2c.so's hand-written HIP kernels (csrc/s2c_*.hip).  There is no CPU
fallback: without a visible GPU ``DeviceBatch`` raises.
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np
import torch

from . import _lib as L
from ._lib import lib
from .devargs import ARRAYS, fill_dev


def _dev(device):
    if device is None:
        device = "cuda:%d" % int(os.environ.get("LOCAL_RANK", "0"))
    d = torch.device(device)
    if d.type != "cuda" or not torch.cuda.is_available():
        raise RuntimeError("sam2consensus_amd needs a ROCm GPU (torch.cuda unavailable); no CPU fallback")
    return d


def _up(arr, device):
    """numpy u32/i64 array → device tensor (bit-preserving, ≥1 element)."""
    a = np.ascontiguousarray(arr)
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    elif a.dtype == np.uint64:
        a = a.view(np.int64)
    if a.size == 0:
        a = np.zeros(4, dtype=a.dtype if a.dtype != np.uint8 else np.uint8)
    return torch.from_numpy(a).to(device, non_blocking=False)


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p()


class Uploader:
    """H2D of packed batches through pinned host staging: a ring of ``nbuf`` pinned buffers of
    ``chunk`` bytes and a copy stream.  ``upload(arrays)`` lays the arrays out in ONE device
    allocation and streams them through the ring: each chunk is packed into the next pinned
    buffer (after that buffer's previous copy has completed) and copied on the copy stream, so
    packing chunk k + 1 overlaps the DMA of chunk k; the compute stream waits on the last
    copy's event, and the host goes on (parsing the next batch) while the copies and the
    kernels run.  Pageable H2D of a GB-sized batch runs at ~2 GB/s on the box; this at the
    memcpy rate."""

    ALIGN = 256

    def __init__(self, device=None, nbuf=4, chunk=32 << 20):
        self.device = _dev(device)
        self.copy_stream = torch.cuda.Stream(self.device)
        self.chunk = int(chunk)
        self.slots = [None] * nbuf      # pinned uint8 tensors of `chunk` bytes
        self.events = [None] * nbuf     # the copy out of each slot
        self.k = 0
        self.timing = {"alloc": 0.0, "wait": 0.0, "pack": 0.0, "issue": 0.0}   # host seconds, cumulative

    def _layout(self, arrays):
        offs, total = [], 0
        for a in arrays:
            offs.append(total)
            total += (max(a.nbytes, 16) + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        return offs, max(total, self.ALIGN)

    def _slot(self):
        i = self.k % len(self.slots)
        self.k += 1
        t0 = time.perf_counter()
        if self.events[i] is not None:
            self.events[i].synchronize()          # this slot's previous copy has left it
        t1 = time.perf_counter()
        if self.slots[i] is None:
            self.slots[i] = torch.empty(self.chunk, dtype=torch.uint8, pin_memory=True)
        self.timing["wait"] += t1 - t0
        self.timing["alloc"] += time.perf_counter() - t1
        return i

    def prime(self):
        """Allocate the whole pinned ring now (the CLI does it on its warm-up thread while the
        host parses: 4 × 32 MB of page-locked memory is milliseconds of host time each)."""
        for i, s in enumerate(self.slots):
            if s is None:
                self.slots[i] = torch.empty(self.chunk, dtype=torch.uint8, pin_memory=True)
        return self

    def upload(self, arrays):
        """numpy arrays → device uint8 views (each 256-byte aligned, ≥ 16 bytes, zero-padded
        to its 16-byte end), in HBM once the compute stream reaches this point."""
        arrays = [np.ascontiguousarray(a).reshape(-1).view(np.uint8) for a in arrays]
        offs, total = self._layout(arrays)
        compute = torch.cuda.current_stream(self.device)
        t0 = time.perf_counter()
        # the allocation on the copy stream (free there in its order: no wait for the compute
        # stream's queued kernels); the compute stream's use is recorded below
        with torch.cuda.stream(self.copy_stream):
            dev = torch.empty(total, dtype=torch.uint8, device=self.device)
        self.timing["alloc"] += time.perf_counter() - t0
        ends = [o + (max(a.nbytes, 16) + 15) // 16 * 16 for a, o in zip(arrays, offs)]   # (zero pad to 16 bytes)
        ai = 0
        ev = None
        for w0 in range(0, max(ends) if ends else 0, self.chunk):
            w1 = min(w0 + self.chunk, total)
            i = self._slot()
            host = self.slots[i].numpy()
            t0 = time.perf_counter()
            while ai < len(arrays) and ends[ai] <= w0:
                ai += 1
            j = ai
            while j < len(arrays) and offs[j] < w1:   # the arrays (and their pads) in [w0, w1)
                a, o = arrays[j], offs[j]
                lo, hi = max(o, w0), min(ends[j], w1)
                n_data = max(0, min(o + a.nbytes, hi) - lo)
                if n_data >= (1 << 20):   # (large pieces on the host threads)
                    L.check(lib.s2c_copy_bytes(host.ctypes.data + (lo - w0), a.ctypes.data + (lo - o), n_data))
                elif n_data:
                    host[lo - w0:lo - w0 + n_data] = a[lo - o:lo - o + n_data]
                if lo + n_data < hi:
                    host[lo - w0 + n_data:hi - w0] = 0
                j += 1
            t1 = time.perf_counter()
            with torch.cuda.stream(self.copy_stream):
                dev[w0:w1].copy_(self.slots[i][:w1 - w0], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.copy_stream)
            self.events[i] = ev
            self.timing["pack"] += t1 - t0
            self.timing["issue"] += time.perf_counter() - t1
        dev.record_stream(compute)   # (the kernels read it: not reused before they are done)
        if ev is not None:
            compute.wait_event(ev)
        return [dev[o:o + max(a.nbytes, 16)] for a, o in zip(arrays, offs)], dev


_UPLOADERS = {}
_SIDE = {}


def to_host(t):
    """A device uint8 tensor → the host, as a read-only memoryview of a pinned buffer (one DMA
    at the link's rate; no further copy: a 65 MB bytes object built from it would cost more
    than the transfer, its fresh pages faulted in by one thread).  The buffer comes from
    torch's caching host allocator and lives as long as the view; bytes-like everywhere
    (slicing, ``bytes +``, ``b"".join``, ``==``)."""
    n = int(t.numel())
    if n == 0:
        return memoryview(b"")
    if t.device.type != "cuda":
        return memoryview(t.contiguous().numpy()).toreadonly()
    buf = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    buf.copy_(t, non_blocking=True)
    torch.cuda.current_stream(t.device).synchronize()
    return memoryview(buf.numpy()).toreadonly()


def _side_stream(device):
    """A stream for result copies beside the compute stream (one per device)."""
    if device not in _SIDE:
        _SIDE[device] = torch.cuda.Stream(device)
    return _SIDE[device]


def default_uploader(device=None):
    """The process's Uploader for a device (its pinned ring allocated once)."""
    d = _dev(device)
    if d not in _UPLOADERS:
        _UPLOADERS[d] = Uploader(d)
    return _UPLOADERS[d]


def needs_dense_layers(fill=b"-", counts=False):
    """Whether a Workspace runs the dense tiles through k_tile (so its DeviceBatch needs
    ``dense_layers=True``): the counts-only modes, and a fill of length != 1 (k_tile_dense
    emits one char per position)."""
    return bool(counts) or len(fill.encode("latin-1") if isinstance(fill, str) else bytes(fill)) != 1


class DeviceBatch:
    """The packed batch resident in HBM (inputs of every launch).  With an ``Uploader`` (by
    default for batches of 64 MB or more) the arrays go through its pinned staging ring and
    copy stream (asynchronous); otherwise each array is copied synchronously."""

    ARRAYS = ARRAYS   # (devargs: s2c_dev's pointer fields, in upload order)

    def __init__(self, hb, device=None, uploader=None, dense_layers=False):
        self.device = _dev(device) if uploader is None else uploader.device
        # dense_layers: the dense tiles' layered windows too (Workspace's counts-only modes run
        # them through k_tile); the pileup reads them in place, so by default they are not built
        self.hb = hb.ensure_layers(dense_layers)
        self.info = type(hb.info).from_buffer_copy(hb.info)   # (the arrays as uploaded)
        # (the per-word arrays over the batch's word span only: HostBatch.device_view)
        arrays = [np.asarray(hb.device_view(n)).reshape(-1) for n in self.ARRAYS]
        if uploader is None and sum(a.nbytes for a in arrays) >= (64 << 20):
            uploader = default_uploader(self.device)   # (large batches: pinned chunks, not pageable copies)
        if uploader is not None:
            views, self._storage = uploader.upload(arrays)
            for name, v in zip(self.ARRAYS, views):
                setattr(self, name, v)
            return
        for name, a in zip(self.ARRAYS, arrays):
            setattr(self, name, _up(a, self.device))

    def nbytes(self):
        return sum(getattr(self, n).numel() * getattr(self, n).element_size() for n in self.ARRAYS)


class Workspace:
    """All scratch + output buffers for one (batch, thresholds, fill, maxdel) configuration."""

    def __init__(self, db: DeviceBatch, thresholds, min_depth=1, fill=b"-", keep_counts=False,
                 maxdel_active=None, maxdel=None, counts=None, tile_range=None):
        dev = db.device
        i = db.info
        self.db = db
        # tile_range (t0, t1): launch only those tiles (their work items, dense and deep lists
        # filtered) and fetch only their results — a streamed batch's final tiles without
        # cutting a sub-batch
        self.tile_range = tile_range
        if needs_dense_layers(fill, keep_counts or counts is not None) and i.n_dense > 0 and not i.layers_dense:
            raise ValueError("counts-only modes and a fill of length != 1 run the dense tiles through k_tile: "
                             "DeviceBatch(..., dense_layers=True)")
        self.T = len(thresholds)
        sz = L.WsSizes()
        L.check(lib.s2c_workspace_sizes(C.byref(i), self.T, C.byref(sz)))
        self.sizes = sz
        u8 = lambda n: torch.empty(max(int(n), 16), dtype=torch.uint8, device=dev)  # noqa: E731
        z8 = lambda n: torch.zeros(max(int(n), 16), dtype=torch.uint8, device=dev)  # noqa: E731
        self.thr = torch.tensor([float(t) for t in thresholds], dtype=torch.float64, device=dev)
        fill = bytes(fill)
        self.fill_bytes = fill
        self.fill = torch.tensor(list(fill) or [0], dtype=torch.uint8, device=dev)
        self.runs = u8(sz.runs)
        # insertion hash tables: zero before the first run; every run leaves them zero
        self.ibkt, self.ilong, self.ilong_n = z8(sz.ibkt), u8(sz.ilong), z8(sz.ilong_n)
        # counts live in HBM only for deep / general tiles (unless a test asks for all of them)
        self.keep_counts = keep_counts
        if counts is not None:   # running totals shared by streamed batches (u8 view, 6·L u32)
            if counts.numel() * counts.element_size() < 6 * i.padded_len * 4:
                raise ValueError("counts buffer smaller than 6 x padded_len u32")
            self.counts = counts
        else:   # (zero before the first run; s2c_consensus leaves it zero: s2c_dev.counts)
            self.counts = z8(6 * i.padded_len * 4 if keep_counts else sz.counts)
        self._counts_filled = False   # s2c_pileup_counts leaves counts filled: zeroed before a run
        self.ins_cols = u8(sz.ins_cols)
        self.ins_chr = u8(sz.ins_chr)
        self.blk_len = u8(sz.blk_len)
        self.tile_stats = u8(sz.tile_stats)
        # body slots: per threshold max(1, len(fill)) bytes per padded position + the columns
        self.fill_w = max(1, len(fill))
        self.out_stride = self.fill_w * i.padded_len + i.n_cols
        cap = int(sz.out_per_fill) * self.fill_w + int(sz.out_fixed)
        self.out = u8(cap)
        # the maxdel rule (:210) runs on the device: the parser's setting unless overridden
        if maxdel_active is None:
            maxdel_active = getattr(db.hb, "maxdel_active", True)
        if maxdel is None:
            maxdel = getattr(db.hb, "maxdel", 150)
        bufs = {n: getattr(self, n).data_ptr() for n in ("runs", "ibkt", "ilong", "ilong_n", "counts", "ins_cols",
                                                           "ins_chr", "tile_stats", "blk_len", "out")}
        bufs.update(thresholds=self.thr.data_ptr(), fill=self.fill.data_ptr())
        d = fill_dev(i, {name: getattr(db, name).data_ptr() for name in DeviceBatch.ARRAYS}, bufs, self.T, min_depth,
                     fill, maxdel_active, maxdel, cap)
        if tile_range is not None:
            t0, t1 = tile_range
            hb = db.hb
            keep = lambda a, col: a[(a[:, col] >= t0) & (a[:, col] < t1)] if len(a) else a  # noqa: E731
            self._sel = {"items": keep(hb.items, 0), "dense": keep(hb.dense, 0), "dwin": keep(hb.dwin, 0),
                         "deep": hb.deep[(hb.deep >= t0) & (hb.deep < t1)]}
            for name, a in self._sel.items():
                t = _up(np.ascontiguousarray(a).reshape(-1), dev)
                self._sel[name] = t
                setattr(d, name, _ptr(t))
            d.n_items = int(len(keep(hb.items, 0)))
            d.n_dense = int(len(keep(hb.dense, 0)))
            d.n_deep = int(((hb.deep >= t0) & (hb.deep < t1)).sum())
        self.dev = d

    def stream_handle(self):
        return C.c_void_p(torch.cuda.current_stream(self.db.device).cuda_stream)

    # ---- the stages in run order (each one C-ABI call; asynchronous on the current stream)
    def reads(self):
        """parsecigar + maxdel per piece → run records; insertion events → hash tables."""
        L.check(lib.s2c_reads(C.byref(self.dev), self.stream_handle()))

    def _counts_ready(self):
        if self._counts_filled:   # (after the counts-only diagnostic)
            self.counts.zero_()
            self._counts_filled = False

    def pileup(self):
        self._counts_ready()
        L.check(lib.s2c_pileup(C.byref(self.dev), self.stream_handle()))

    def consensus(self):
        L.check(lib.s2c_consensus(C.byref(self.dev), self.stream_handle()))

    def run(self):
        """reads → pileup (+ insertion columns, vote, FASTA bodies) → deep tiles (no host sync)."""
        self._counts_ready()
        L.check(lib.s2c_run(C.byref(self.dev), self.stream_handle()))

    def record_done(self):
        """An event after this workspace's launches so far on the compute stream: ``fetch(done)``
        then waits for these kernels only, not for later batches queued behind them."""
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.db.device))
        return ev

    # ---- HIP graph of one run (the stage launches replayed without host launch overhead)
    def capture(self):
        """Capture one ``run()`` into a HIP graph (torch.cuda.CUDAGraph is hipGraph on ROCm);
        the kernel arguments (this workspace's buffers) are baked in."""
        dev = self.db.device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            self.run()                      # warm-up launch outside the capture
        torch.cuda.current_stream(dev).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.run()
        self.graph = g
        return g

    def replay(self):
        self.graph.replay()

    # ---- results
    def accumulate(self, keep_tables=False):
        """Streamed batch of unsorted input: this batch's counts added to ``counts``."""
        L.check(lib.s2c_accumulate(C.byref(self.dev), 1 if keep_tables else 0, self.stream_handle()))

    def vote_all(self):
        """Last streamed batch of unsorted input: k_consensus votes every tile from ``counts``
        (after ``accumulate(keep_tables=True)``)."""
        nt = int(self.db.info.n_tiles)
        if nt == 0:
            return
        self._all_tiles = torch.arange(nt, dtype=torch.int32, device=self.db.device)
        d = L.Dev.from_buffer_copy(self.dev)
        d.deep, d.n_deep = _ptr(self._all_tiles), nt
        L.check(lib.s2c_consensus(C.byref(d), self.stream_handle()))

    def pileup_counts(self):
        """Diagnostic: k_reads, then every tile's counts stored to `counts` (no vote); needs
        keep_counts=True; returns counts[6][padded_len] as numpy u32."""
        if not self.keep_counts:
            raise ValueError("pileup_counts needs Workspace(keep_counts=True)")
        L.check(lib.s2c_pileup_counts(C.byref(self.dev), self.stream_handle()))
        self._counts_filled = True
        return self.counts_host()

    def counts_host(self):
        """counts[6][padded_len] as numpy u32 (for parity tests)."""
        Lp = self.db.info.padded_len
        return self.counts[: 6 * Lp * 4].view(torch.int32).cpu().numpy().view(np.uint32).reshape(6, Lp)

    def fetch(self, done=None):
        """Synchronise and copy results: (stats[R,T,4] u64, offs[T*nb+1] u64, out bytes).
        ``done`` (record_done): wait for that event only and copy on a side stream, so later
        batches' kernels on the compute stream neither delay nor are delayed by the copies.

        stats[r, t] = Σ over reference r's tiles of the device's per-tile statistics
        (tiles never straddle a reference; :352-397 sums)."""
        if done is None:
            torch.cuda.current_stream(self.db.device).synchronize()
            return self._fetch()
        side = _side_stream(self.db.device)
        side.wait_event(done)
        with torch.cuda.stream(side):
            return self._fetch()

    def _fetch(self):
        stats, offs, body = self.fetch_device()
        return stats, offs, to_host(body)

    def _body_starts(self):
        """Device int64 [T·tiles]: each fetched (threshold, tile) body's slot in ``out``,
        t·(F·padded_len + n_cols) + F·a + cb0 (s2c.h s2c_dev.out), in [t][tile] order."""
        if getattr(self, "_starts", None) is None:
            nb = self.db.info.n_tiles
            t0, t1 = self.tile_range if self.tile_range is not None else (0, nb)
            blocks = self.db.hb.tiles[t0:t1].astype(np.int64)
            slot = self.fill_w * blocks[:, 0] + blocks[:, 8]                     # F·a + cb0
            starts = (np.arange(self.T, dtype=np.int64)[:, None] * self.out_stride + slot[None, :]).reshape(-1)
            self._starts = _up(starts, self.db.device)
        return self._starts

    def fetch_device(self):
        """Results with the FASTA bodies left on the device: (stats[R,T,4] u64, offs[T*nb+1]
        u64, body) — ``body`` a device uint8 tensor of exactly offs[-1] bytes, the fetched
        tiles' bodies compacted in [t][tile] order by ``s2c_gather_bodies_dev`` (only the
        statistics and the body lengths cross to the host here).  The current stream must
        have the kernels' results (``fetch`` arranges that).

        stats[r, t] = Σ over reference r's tiles of the device's per-tile statistics
        (tiles never straddle a reference; :352-397 sums)."""
        i = self.db.info
        dev = self.db.device
        R, T, nb = i.n_refs, self.T, i.n_tiles
        t0, t1 = self.tile_range if self.tile_range is not None else (0, nb)
        stats = np.zeros((R, T, 4), dtype=np.uint64)
        if t1 > t0:
            ts = self.tile_stats[: T * nb * 32].view(torch.int64).cpu().numpy().view(np.uint64).reshape(T, nb, 4)
            ref = self.db.hb.tiles[t0:t1, 2].astype(np.int64)
            for t in range(T):
                np.add.at(stats[:, t, :], ref, ts[t, t0:t1])
        nr = t1 - t0
        if T * nr == 0:
            return stats, np.zeros(1, dtype=np.uint64), torch.empty(0, dtype=torch.uint8, device=dev)
        # each tile wrote its body into its slot; a reference's body is its tiles' pieces in
        # order: the slots compacted into [t][tile] order on the device
        lens = self.blk_len[: T * nb * 8].view(torch.int64).view(T, nb)[:, t0:t1].reshape(-1)
        offs_d = torch.zeros(T * nr + 1, dtype=torch.int64, device=dev)
        torch.cumsum(lens, 0, out=offs_d[1:])
        offs = offs_d.cpu().numpy()
        total = int(offs[-1])
        body = torch.empty(max(total, 16), dtype=torch.uint8, device=dev)
        L.check(lib.s2c_gather_bodies_dev(_ptr(self.out), self.out.numel(), _ptr(self._body_starts()), _ptr(offs_d),
                                          T * nr, _ptr(body), C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
        return stats, offs.astype(np.uint64), body[:total]
