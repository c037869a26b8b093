"""Host side of the packed read batch (north_star subsystem 1).

``parse_file`` / ``parse_text`` / ``synth_batch`` drive libs2c.so's parser
(s2c_host.cpp), which reproduces the reference's read pass
(sam2consensus.py:147-228) and reformat-phase checks (:284-294), and returns a
``HostBatch`` whose arrays are zero-copy numpy views of the C++ buffers.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _lib as L
from ._lib import lib


class Parser:
    """Streaming SAM parser (``s2c_parser_*``).  ``maxdel_active=False`` is the
    reference's behaviour when ``-d`` is given at all (:102, :210)."""

    def __init__(self, maxdel_active=True, maxdel=150):
        self.maxdel_active, self.maxdel = bool(maxdel_active), int(maxdel)
        self._p = C.c_void_p()
        L.check(lib.s2c_parser_new(1 if maxdel_active else 0, int(maxdel), C.byref(self._p)))

    def feed(self, data):
        """bytes, or a writable buffer (bytearray / its memoryview: read in place)."""
        if isinstance(data, (bytearray, memoryview)):
            mv = memoryview(data).cast("B")
            if mv.nbytes == 0:
                return
            L.check(lib.s2c_parser_feed(self._p, (C.c_char * mv.nbytes).from_buffer(mv), mv.nbytes))
            return
        L.check(lib.s2c_parser_feed(self._p, data, len(data)))

    def feed_file(self, path: str):
        L.check(lib.s2c_parser_feed_file(self._p, os.fsencode(path)))

    def finish(self) -> "HostBatch":
        b = C.c_void_p()
        L.check(lib.s2c_parser_finish(self._p, C.byref(b)))
        hb = HostBatch(b)
        hb.maxdel_active, hb.maxdel = self.maxdel_active, self.maxdel   # the device applies :210
        return hb

    def progress(self):
        """(header ended, references, header lines, lines read, read-pass error code): where
        the read pass stands, also after it raised (s2c_parser_progress)."""
        c = (C.c_int64 * 5)()
        L.check(lib.s2c_parser_progress(self._p, c))
        return tuple(int(x) for x in c)

    def counters(self):
        """(header lines, lines, mapped reads, aligned bases) of a clean read pass."""
        c = (C.c_int64 * 4)()
        L.check(lib.s2c_parser_counters(self._p, c))
        return tuple(int(x) for x in c)

    def close(self):
        if self._p:
            lib.s2c_parser_free(self._p)
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def _view(ptr, n, dtype):
    if n <= 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    ct = C.c_int64 if dtype == np.int64 else C.c_uint32
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), shape=(int(n),)).view(dtype)


class HostBatch:
    """Packed batch owned by libs2c.so; arrays are numpy views valid until ``free()``."""

    def __init__(self, handle):
        self._b = handle
        self.info = L.BatchInfo()
        L.check(lib.s2c_batch_info_get(self._b, C.byref(self.info)))
        a = L.BatchArrays()
        L.check(lib.s2c_batch_arrays_get(self._b, C.byref(a)))
        i = self.info
        self.ref_len = _view(a.ref_len, i.n_refs, np.int64)
        self.ref_off = _view(a.ref_off, i.n_refs, np.int64)
        self.ref_reads = _view(a.ref_cov_reads, i.n_refs, np.int64)
        # pieces bucketed by start word (+ sentinel), their op words, the query base planes
        self.pc = _view(a.pc, 4 * (i.n_pieces + 1), np.uint32).reshape(-1, 4)
        self.ops = _view(a.ops, i.n_ops, np.uint32)
        self.bq = _view(a.bq, 2 * i.n_qwords, np.uint32).reshape(-1, 2)
        self.bx = _view(a.bx, i.n_qwords, np.uint32)
        self.rs = _view(a.rs, i.n_words + 1, np.uint32)
        self.ps = _view(a.ps, i.n_words + 1, np.uint32)
        self._layers = False
        # tile plan
        self.tiles = _view(a.tiles, i.n_tiles * L.S2C_TILE_WORDS, np.uint32).reshape(-1, L.S2C_TILE_WORDS)
        self.items = _view(a.items, i.n_items * L.S2C_ITEM_WORDS, np.uint32).reshape(-1, L.S2C_ITEM_WORDS)
        self.dense = _view(a.dense, i.n_dense * L.S2C_ITEM_WORDS, np.uint32).reshape(-1, L.S2C_ITEM_WORDS)
        self.deep = _view(a.deep, i.n_deep, np.uint32)
        self.rlist = _view(a.rlist, i.n_rlist, np.uint32)
        self.px = _view(a.px, i.n_pieces, np.uint32)   # non-ACGT SEQ offsets of S2C_PF_XFEW pieces
        self.dwin = _view(a.dwin, i.n_dense * L.S2C_DWIN_WORDS, np.uint32).reshape(-1, L.S2C_DWIN_WORDS)
        self.dpc = _view(a.dpc, i.n_dpc * L.S2C_DPC_WORDS, np.uint32).reshape(-1, L.S2C_DPC_WORDS)
        self.lp = _view(a.lp, i.n_long, np.uint32)
        self.wtile = _view(a.wtile, i.n_words, np.uint32)
        self.names = [lib.s2c_batch_ref_name(self._b, k).decode("latin-1") for k in range(i.n_refs)]
        # per-ref tile ranges (tiles are emitted ref by ref, in header order)
        nb = np.bincount(self.tiles[:, 2].astype(np.int64), minlength=i.n_refs) if i.n_tiles else \
            np.zeros(i.n_refs, dtype=np.int64)
        self.ref_nblocks = nb.astype(np.int64)
        self.ref_first_block = (np.cumsum(nb) - nb).astype(np.int64)

    def ensure_layers(self, dense=False):
        """Build the layered windows of the tiles k_tile does not read in place
        (s2c_batch_layers_mode; before the arrays go to the device) and view them.  The dense
        tiles' are built only with ``dense`` (the counts-only modes run them through k_tile;
        the pileup reads their windows in place); a later ``dense=True`` rebuilds them all."""
        if self._layers and (self.info.layers_dense or not dense):
            return self
        L.check(lib.s2c_batch_layers_mode(self._b, 1 if dense else 0))
        L.check(lib.s2c_batch_info_get(self._b, C.byref(self.info)))
        a = L.BatchArrays()
        L.check(lib.s2c_batch_arrays_get(self._b, C.byref(a)))
        i = self.info
        self.lly = _view(a.lly, 4 * (i.n_layers + 1), np.uint32).reshape(-1, 4)
        self.lpc = _view(a.lpc, 4 * (i.n_lpieces + 1), np.uint32).reshape(-1, 4)
        self.lops = _view(a.lops, max(i.n_lops, 4), np.uint32)
        self.lbq = _view(a.lbq, 2 * i.n_lqwords, np.uint32).reshape(-1, 2)
        self.lbx = _view(a.lbx, i.n_lqwords, np.uint32)
        self.lpx = _view(a.lpx, max(i.n_lpieces, 1), np.uint32)   # px of the layered pieces
        self._layers = True
        return self

    def device_view(self, name):
        """The part of array ``name`` that goes to the device: the per-word arrays only over
        the words a launch reads (info.word_lo / word_hi, ABI 13 — a shard's own words), the
        others whole."""
        a = getattr(self, name)
        lo, hi = int(self.info.word_lo), int(self.info.word_hi)
        if name in ("rs", "ps"):
            return a[lo:hi + 1]
        if name == "wtile":
            return a[lo:hi]
        return a

    @property
    def blocks(self):
        return self.tiles

    @property
    def aligned_bases(self):
        return int(self.info.aligned_bases)

    def free(self):
        if self._b:
            lib.s2c_batch_free(self._b)
            self._b = None

    def free_async(self):
        """Release the host arrays on a side thread (GBs of mappings for a large input: tens
        of ms of munmap, overlapped with what the caller does next); returns the thread (None
        when nothing was held).  The handle is detached first, so no second free can race it;
        this batch's array views must not be read afterwards (as after free())."""
        b, self._b = self._b, None
        if not b:
            return None
        import threading
        th = threading.Thread(target=lib.s2c_batch_free, args=(b,), daemon=True)
        th.start()
        return th

    def __del__(self):
        try:
            self.free()
        except Exception:  # noqa: BLE001
            pass


def parse_file(path, maxdel_active=True, maxdel=150) -> HostBatch:
    p = Parser(maxdel_active, maxdel)
    try:
        p.feed_file(path)
        return p.finish()
    finally:
        p.close()


def parse_text(text, maxdel_active=True, maxdel=150) -> HostBatch:
    data = text.encode("latin-1") if isinstance(text, str) else bytes(text)
    p = Parser(maxdel_active, maxdel)
    try:
        p.feed(data)
        return p.finish()
    finally:
        p.close()


def parsecigar(cigarstring, seq, pos_ref):
    """API mirror of the reference's ``parsecigar(cigarstring, seq, pos_ref)``
    (sam2consensus.py:46-82), computed by libs2c.so: returns
    ``(seqout, [(ref_pos, inserted_seq), ...])``."""
    cb = cigarstring.encode("latin-1")
    sb = seq.encode("latin-1")
    tok_len = sum(int(n) for n in __import__("re").findall(r"([0-9]+)[MDNPX=]", cigarstring))
    cap = max(len(sb), tok_len) + 2
    out = C.create_string_buffer(cap)
    n_out = C.c_size_t()
    max_ins = max(1, cigarstring.count("I"))
    ins = (C.c_int64 * (3 * max_ins))()
    n_ins = C.c_size_t()
    L.check(lib.s2c_parsecigar(cb, len(cb), sb, len(sb), int(pos_ref), out, cap, C.byref(n_out),
                               ins, max_ins, C.byref(n_ins)))
    seqout = out.raw[:n_out.value].decode("latin-1")
    inserts = [(ins[3 * k], seq[ins[3 * k + 1]:ins[3 * k + 1] + ins[3 * k + 2]]) for k in range(n_ins.value)]
    return seqout, inserts
