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
        self._p = C.c_void_p()
        L.check(lib.s2c_parser_new(1 if maxdel_active else 0, int(maxdel), C.byref(self._p)))

    def feed(self, data: bytes):
        L.check(lib.s2c_parser_feed(self._p, data, len(data)))

    def feed_file(self, path: str):
        L.check(lib.s2c_parser_feed_file(self._p, os.fsencode(path)))

    def finish(self) -> "HostBatch":
        b = C.c_void_p()
        L.check(lib.s2c_parser_finish(self._p, C.byref(b)))
        return HostBatch(b)

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
        # host-side read-piece table (file order)
        self.rd_pos = _view(a.rd_pos, i.n_reads, np.uint32)
        self.rd_op = _view(a.rd_op, i.n_reads + 1, np.uint32)
        self.rd_span = _view(a.rd_span, i.n_reads, np.uint32)
        self.ops = _view(a.ops, i.n_ops, np.uint32)
        # word-major seqout records (what the pileup kernel reads)
        self.wrec = _view(a.wrec, i.padded_len // 32 + 1, np.uint32)
        self.recs = _view(a.recs, 2 * i.n_recs, np.uint32).reshape(-1, 2)
        # per work item: A-placeholder counts (16 u32 u16-pairs per tile word) and the
        # seqout '-'/'N' entries
        self.fix = _view(a.fix, i.n_fix, np.uint32)
        self.exc = _view(a.exc, i.n_exc, np.uint32)
        self.iwr = _view(a.iwr, i.n_iwr, np.uint32)
        # insertion events grouped by key (keys ascending)
        nw = i.padded_len // 32
        self.ins_key = _view(a.ins_key, i.n_keys, np.uint32)
        self.ins_koff = _view(a.ins_koff, i.n_keys + 1, np.uint32)
        self.ins_kcol = _view(a.ins_kcol, i.n_keys + 1, np.uint32)
        self.ins_off = _view(a.ins_off, i.n_ins + 1, np.uint32)
        self.ins_bases = _view(a.ins_bases, i.n_ins_words, np.uint32)
        self.ins_ekey = _view(a.ins_ekey, i.n_ins, np.uint32)
        self.ins_ev = _view(a.ins_ev, 4 * i.n_ins, np.uint32).reshape(-1, 4)
        self.ins_kinfo = _view(a.ins_kinfo, 4 * i.n_keys, np.uint32).reshape(-1, 4)
        self.ins_bits = _view(a.ins_bits, nw, np.uint32)
        self.ins_rank = _view(a.ins_rank, nw + 1, np.uint32)
        self.items = _view(a.items, i.n_items * L.S2C_ITEM_WORDS, np.uint32).reshape(-1, L.S2C_ITEM_WORDS)
        self.blocks = _view(a.blocks, i.n_blocks * L.S2C_BLOCK_WORDS, np.uint32).reshape(-1, L.S2C_BLOCK_WORDS)
        self.deep = _view(a.deep, i.n_deep, np.uint32)
        self.names = [lib.s2c_batch_ref_name(self._b, k).decode("latin-1") for k in range(i.n_refs)]
        # per-ref block ranges (blocks are emitted ref by ref, in header order)
        nb = np.bincount(self.blocks[:, 2].astype(np.int64), minlength=i.n_refs) if i.n_blocks else \
            np.zeros(i.n_refs, dtype=np.int64)
        self.ref_nblocks = nb.astype(np.int64)
        self.ref_first_block = (np.cumsum(nb) - nb).astype(np.int64)

    @property
    def aligned_bases(self):
        return int(self.info.aligned_bases)

    def free(self):
        if self._b:
            lib.s2c_batch_free(self._b)
            self._b = None

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
