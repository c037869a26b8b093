"""The whole-file CLI's device side without PyTorch: the HIP runtime through ctypes (the
copy libs2c.so is bound to, _lib._hip_runtime), for a process that runs one batch and exits.

`import torch` alone takes 1.8-1.9 s on the GPU box — twice the whole C5 pipeline (parse,
upload, kernels, records: 0.75-0.95 s) and more than the parse it overlapped on the CLI's
warm-up thread — so the one-process CLI (cli.consensus_files) allocates, uploads, launches
and fetches here: one device buffer for the packed batch and one for the workspace
(hipMalloc, reserved on the warm-up thread while the host parses), one pinned staging
buffer (hipHostMalloc) that the batch is packed into on the host threads and copied from in
one DMA, the run on the null stream, and the results back through the same staging buffer.
The kernels, their arguments (devargs.fill_dev) and the result layout are engine.Workspace's;
the library paths that need streams, graphs or collectives (streamed batches, shards, the
bench) keep engine.py.  No CPU fallback: without a GPU the runtime calls fail loudly.
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np

from . import _lib as L
from ._lib import lib
from .devargs import ARRAYS, BUFFERS, fill_dev

ALIGN = 256
_H2D, _D2H = 1, 2                       # hipMemcpyHostToDevice, hipMemcpyDeviceToHost
_ATTR_CUS = 63                          # hipDeviceAttributeMultiprocessorCount (ROCm 7 hip_runtime_api.h)


class Hip:
    """The few HIP runtime entry points the one-batch path needs (hipError_t = int)."""

    def __init__(self):
        # the runtime libs2c.so is bound to (its handle resolves the hip* symbols through its
        # dependencies: _lib._hip_runtime's copy, the one torch would use too)
        h = lib
        self.h = h
        vp, sz = C.c_void_p, C.c_size_t
        sig = {"hipSetDevice": [C.c_int], "hipGetDeviceCount": [C.POINTER(C.c_int)],
               "hipDeviceGetAttribute": [C.POINTER(C.c_int), C.c_int, C.c_int],
               "hipMalloc": [C.POINTER(vp), sz], "hipFree": [vp],
               "hipHostMalloc": [C.POINTER(vp), sz, C.c_uint], "hipHostFree": [vp],
               "hipMemcpy": [vp, vp, sz, C.c_int], "hipMemset": [vp, C.c_int, sz],
               "hipDeviceSynchronize": [], "hipGetErrorString": [C.c_int]}
        for n, args in sig.items():
            f = getattr(h, n)
            f.argtypes = args
            f.restype = C.c_char_p if n == "hipGetErrorString" else C.c_int
        # (after a failed HIP call the runtime's own message names it)

    def check(self, rc, what):
        if rc != 0:
            raise RuntimeError("%s failed: %s (hipError %d)" % (what, self.h.hipGetErrorString(rc).decode(), rc))

    def set_device(self, dev):
        n = C.c_int(0)
        rc = self.h.hipGetDeviceCount(C.byref(n))
        if rc != 0 or n.value <= dev:
            why = self.h.hipGetErrorString(rc).decode() if rc else "device %d of %d visible" % (dev, n.value)
            raise RuntimeError("sam2consensus_amd needs a ROCm GPU (%s); no CPU fallback" % why)
        self.check(self.h.hipSetDevice(dev), "hipSetDevice")

    def cus(self, dev):
        v = C.c_int(0)
        self.check(self.h.hipDeviceGetAttribute(C.byref(v), _ATTR_CUS, dev), "hipDeviceGetAttribute")
        return v.value

    def malloc(self, n):
        p = C.c_void_p()
        self.check(self.h.hipMalloc(C.byref(p), max(int(n), ALIGN)), "hipMalloc(%d)" % n)
        return p.value

    def host_malloc(self, n):
        p = C.c_void_p()
        self.check(self.h.hipHostMalloc(C.byref(p), max(int(n), ALIGN), 0), "hipHostMalloc(%d)" % n)
        return p.value

    def memcpy(self, dst, src, n, kind):
        if n:
            self.check(self.h.hipMemcpy(C.c_void_p(dst), C.c_void_p(src), int(n), kind), "hipMemcpy")

    def memset(self, p, n):
        if n:
            self.check(self.h.hipMemset(C.c_void_p(p), 0, int(n)), "hipMemset")

    def sync(self):
        self.check(self.h.hipDeviceSynchronize(), "hipDeviceSynchronize")

    def free(self, p):
        if p:
            self.h.hipFree(C.c_void_p(p))

    def host_free(self, p):
        if p:
            self.h.hipHostFree(C.c_void_p(p))


def _layout(sizes):
    offs, total = [], 0
    for n in sizes:
        offs.append(total)
        total += (max(int(n), 16) + ALIGN - 1) // ALIGN * ALIGN
    return offs, max(total, ALIGN)


class Session:
    """One device and its buffers for a one-batch run: `reserve` (the warm-up thread, while
    the host parses) makes the runtime, the plan's CU count and buffers of an estimated size
    ready; `run` grows them if the batch needs more."""

    def __init__(self, device=0):
        self.device = int(device)
        self.hip = None
        self.dbuf = self.dcap = 0      # the packed batch (device)
        self.hbuf = self.hcap = 0      # pinned staging: the batch out, the results back
        self.timing = {}

    def reserve(self, nbytes=0):
        t0 = time.perf_counter()
        self.hip = Hip()
        self.hip.set_device(self.device)
        L.check(lib.s2c_plan_set_cus(self.hip.cus(self.device)))   # (the plan's grid shaping)
        t1 = time.perf_counter()
        self.timing["warm_context"] = t1 - t0
        if nbytes > 0:
            self._grow(int(nbytes))
            # the device buffer's pages and the copy path brought up here, off the main thread
            # (a first 1 GB hipMemcpy after the parse took 0.11 s against 0.019 s warm)
            self.hip.memset(self.dbuf, self.dcap)
            self.hip.memcpy(self.dbuf, self.hbuf, 1 << 20, _H2D)
            self.hip.sync()
            self.timing["warm_reserve"] = time.perf_counter() - t1
        return self

    def _grow(self, n):
        if n > self.dcap:
            self.hip.free(self.dbuf)
            self.dbuf, self.dcap = self.hip.malloc(n), n
        if n > self.hcap:
            self.hip.host_free(self.hbuf)
            self.hbuf, self.hcap = self.hip.host_malloc(n), n

    def close(self):
        if self.hip is not None:
            self.hip.free(self.dbuf)
            self.hip.host_free(self.hbuf)
            self.dbuf = self.dcap = self.hbuf = self.hcap = 0

    def _staging(self, n):
        return np.ctypeslib.as_array((C.c_uint8 * max(int(n), 1)).from_address(self.hbuf))

    def run(self, hb, thresholds, min_depth=1, fill=b"-", timings=None):
        """The batch's one run (s2c_run) → (stats[R,T,4] u64, offs[T·tiles+1] u64, bodies) as
        engine.Workspace.fetch returns them; ``bodies`` a read-only view valid until close()."""
        t = timings if timings is not None else {}
        hip = self.hip
        fill = bytes(fill)
        t0 = time.perf_counter()
        hb.ensure_layers(len(fill) != 1)   # (engine.needs_dense_layers: a fill of length != 1)
        i = type(hb.info).from_buffer_copy(hb.info)
        arrays = [np.ascontiguousarray(np.asarray(hb.device_view(n)).reshape(-1)).view(np.uint8) for n in ARRAYS]
        offs, total = _layout([a.nbytes for a in arrays])
        self._grow(total)
        host = self._staging(total)
        for a, o in zip(arrays, offs):   # packed on the host threads (s2c_copy_bytes), 16-byte zero pads
            n = a.nbytes
            if n:
                L.check(lib.s2c_copy_bytes(self.hbuf + o, a.ctypes.data, n))
            end = o + (max(n, 16) + 15) // 16 * 16
            host[o + n:end] = 0
        t1 = time.perf_counter()
        hip.memcpy(self.dbuf, self.hbuf, total, _H2D)
        t2 = time.perf_counter()
        # the workspace in one allocation (its zeroed buffers: the insertion tables and counts)
        T = len(thresholds)
        sz = L.WsSizes()
        L.check(lib.s2c_workspace_sizes(C.byref(i), T, C.byref(sz)))
        fill_w = max(1, len(fill))
        cap = int(sz.out_per_fill) * fill_w + int(sz.out_fixed)
        wsz = {n: int(getattr(sz, n)) for n in BUFFERS if n != "out"}
        wsz["out"] = cap
        wsz["thresholds"], wsz["fill"] = 8 * T, max(len(fill), 1)
        names = list(wsz)
        woffs, wtotal = _layout([wsz[n] for n in names])
        wbuf = hip.malloc(wtotal)
        try:
            bufs = {n: wbuf + o for n, o in zip(names, woffs)}
            for n in ("ibkt", "ilong_n", "counts"):   # zero before the first run (s2c_dev)
                hip.memset(bufs[n], max(wsz[n], 16))
            thr = np.array([float(x) for x in thresholds], dtype=np.float64)
            fb = np.frombuffer(fill or b"\0", dtype=np.uint8)
            hip.memcpy(bufs["thresholds"], thr.ctypes.data, thr.nbytes, _H2D)
            hip.memcpy(bufs["fill"], fb.ctypes.data, fb.nbytes, _H2D)
            d = fill_dev(i, {n: self.dbuf + o for n, o in zip(ARRAYS, offs)}, bufs, T, min_depth, fill,
                         getattr(hb, "maxdel_active", True), getattr(hb, "maxdel", 150), cap)
            t3 = time.perf_counter()
            L.check(lib.s2c_run(C.byref(d), C.c_void_p()))
            hip.sync()
            t4 = time.perf_counter()
            res = self._fetch(hb, i, T, fill_w, cap, bufs)
        finally:
            hip.free(wbuf)
        t.update(h2d_pack=t1 - t0, h2d_copy=t2 - t1, workspace=t3 - t2, device_run=t4 - t3,
                 fetch=time.perf_counter() - t4)
        return res

    def _fetch(self, hb, i, T, fill_w, cap, bufs):
        """engine.Workspace.fetch_device + to_host: statistics and body lengths to the host, the
        bodies compacted on the device (s2c_gather_bodies_dev) and copied out once."""
        hip = self.hip
        R, nb = i.n_refs, i.n_tiles
        stats = np.zeros((R, T, 4), dtype=np.uint64)
        if T * nb == 0:
            return stats, np.zeros(1, dtype=np.uint64), b""
        ts = np.empty(T * nb * 4, dtype=np.uint64)
        hip.memcpy(ts.ctypes.data, bufs["tile_stats"], ts.nbytes, _D2H)
        ts = ts.reshape(T, nb, 4)
        ref = hb.tiles[:, 2].astype(np.int64)
        for t in range(T):
            np.add.at(stats[:, t, :], ref, ts[t])
        lens = np.empty(T * nb, dtype=np.int64)
        hip.memcpy(lens.ctypes.data, bufs["blk_len"], lens.nbytes, _D2H)
        offs = np.zeros(T * nb + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        total = int(offs[-1])
        blocks = hb.tiles.astype(np.int64)
        out_stride = fill_w * i.padded_len + i.n_cols
        starts = (np.arange(T, dtype=np.int64)[:, None] * out_stride
                  + (fill_w * blocks[:, 0] + blocks[:, 8])[None, :]).reshape(-1)
        # (the slots, their offsets and the compacted bodies in one more device allocation)
        aoffs, atotal = _layout([starts.nbytes, offs.nbytes, total])
        abuf = hip.malloc(atotal)
        try:
            hip.memcpy(abuf + aoffs[0], starts.ctypes.data, starts.nbytes, _H2D)
            hip.memcpy(abuf + aoffs[1], offs.ctypes.data, offs.nbytes, _H2D)
            L.check(lib.s2c_gather_bodies_dev(C.c_void_p(bufs["out"]), cap, C.c_void_p(abuf + aoffs[0]),
                                              C.c_void_p(abuf + aoffs[1]), T * nb, C.c_void_p(abuf + aoffs[2]),
                                              C.c_void_p()))
            self._grow(total)
            hip.memcpy(self.hbuf, abuf + aoffs[2], total, _D2H)   # (synchronous: the null stream's work is done)
        finally:
            hip.free(abuf)
        # a read-only view of the pinned staging buffer (valid until close(); no bytes copy of
        # the bodies: one thread faulting in 65 MB of fresh pages costs more than the DMA)
        body = memoryview(self._staging(total)[:total]).toreadonly() if total else memoryview(b"")
        return stats, offs.astype(np.uint64), body


def device_index(device=None):
    """The CLI's device: ``cuda:N`` / N / LOCAL_RANK (as engine._dev), as an index."""
    if device is None:
        return int(os.environ.get("LOCAL_RANK", "0"))
    if isinstance(device, int):
        return device
    s = str(device)
    if s.startswith("cuda"):
        return int(s.split(":")[1]) if ":" in s else 0
    raise RuntimeError("sam2consensus_amd needs a ROCm GPU device, not %r; no CPU fallback" % (device,))
