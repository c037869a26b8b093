"""ctypes binding of libs2c.so (include/s2c.h).

The shared library is built in-tree (``make`` / ``__graft_entry__.build()``) and
loaded from this package directory.  There is no fallback: if the library is
missing the import fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libs2c.so")

S2C_OK = 0
S2C_ERR_KEY = -1
S2C_ERR_INDEX = -2
S2C_ERR_VALUE = -3
S2C_ERR_ZERODIV = -4
S2C_ERR_OVERFLOW = -5
S2C_ERR_IO = -10
S2C_ERR_HIP = -11
S2C_ERR_ARG = -12
S2C_ERR_LIMIT = -13

S2C_NSYM = 6
S2C_POS_ALIGN = 64
S2C_ITEM_WORDS = 16
S2C_BLOCK_WORDS = 12
S2C_CODE_FILL = 0

# reference exception classes (SURVEY.md §5 "Failure detection")
_EXC = {S2C_ERR_KEY: KeyError, S2C_ERR_INDEX: IndexError, S2C_ERR_VALUE: ValueError,
        S2C_ERR_ZERODIV: ZeroDivisionError, S2C_ERR_OVERFLOW: OverflowError, S2C_ERR_IO: IOError}


class S2CError(RuntimeError):
    """Engine failure that is not one of the reference's exception classes."""

    def __init__(self, code, msg):
        super().__init__("s2c error %d: %s" % (code, msg))
        self.code = code


class BatchInfo(C.Structure):
    _fields_ = [(n, C.c_int64) for n in (
        "n_refs", "total_len", "padded_len", "header_lines", "lines_total", "reads_mapped",
        "aligned_bases", "query_bases", "n_reads", "n_ops", "n_recs", "chunk_recs", "n_ins",
        "n_ins_bases", "n_ins_words", "n_keys", "n_cols", "n_items", "n_blocks", "tile_max",
        "n_deep", "n_exc", "n_fix", "n_iwr")]


_P64 = C.POINTER(C.c_int64)
_P32 = C.POINTER(C.c_uint32)


class BatchArrays(C.Structure):
    _fields_ = [("ref_len", _P64), ("ref_off", _P64), ("ref_cov_reads", _P64),
                ("rd_pos", _P32), ("rd_op", _P32), ("rd_span", _P32), ("ops", _P32),
                ("wrec", _P32), ("recs", _P32), ("fix", _P32), ("exc", _P32),
                ("ins_key", _P32), ("ins_koff", _P32), ("ins_kcol", _P32), ("ins_off", _P32),
                ("ins_bases", _P32), ("ins_ekey", _P32), ("ins_ev", _P32), ("ins_kinfo", _P32),
                ("ins_bits", _P32), ("ins_rank", _P32),
                ("items", _P32), ("iwr", _P32), ("blocks", _P32), ("deep", _P32)]


class SynthSpec(C.Structure):
    _fields_ = [("n_refs", C.c_int32), ("ref_len", C.c_int64), ("depth", C.c_double),
                ("read_len", C.c_int32), ("ins_frac", C.c_double), ("ins_max", C.c_int32),
                ("del_frac", C.c_double), ("del_max", C.c_int32), ("long_del_frac", C.c_double),
                ("sub_rate", C.c_double), ("n_rate", C.c_double), ("amplicons", C.c_int32),
                ("shuffle", C.c_int32), ("seed", C.c_uint64), ("ref_prefix", C.c_char_p)]


_VP = C.c_void_p


class Dev(C.Structure):
    """Mirror of ``s2c_dev`` (include/s2c.h)."""
    _fields_ = [
        ("wrec", _VP), ("recs", _VP), ("fix", _VP), ("exc", _VP), ("iwr", _VP),
        ("items", _VP), ("blocks", _VP), ("deep", _VP),
        ("ins_ev", _VP), ("ins_kinfo", _VP), ("ins_bases", _VP), ("ins_bits", _VP),
        ("n_recs", C.c_int64), ("chunk_recs", C.c_int64),
        ("n_items", C.c_int64), ("n_blocks", C.c_int64), ("n_deep", C.c_int64),
        ("n_keys", C.c_int64), ("n_cols", C.c_int64), ("padded_len", C.c_int64), ("n_exc", C.c_int64),
        ("tile_max", C.c_int32), ("n_refs", C.c_int32),
        ("thresholds", _VP), ("n_thr", C.c_int32), ("min_depth", C.c_int32),
        ("fill_len", C.c_int32), ("fill_nondash", C.c_int32), ("fill", _VP),
        ("counts", _VP), ("ins_cols", _VP), ("ins_cnt", _VP), ("ins_chr", _VP),
        ("tile_stats", _VP), ("blk_len", _VP), ("out", _VP), ("out_cap", C.c_int64),
        ("ablate", C.c_int32), ("reserved", C.c_int32)]


class WsSizes(C.Structure):
    _fields_ = [(n, C.c_int64) for n in (
        "counts", "ins_cols", "ins_cnt", "ins_chr", "blk_len", "tile_stats", "out_per_fill", "out_fixed")]


# every symbol include/s2c.h declares (tests/test_lib.py checks the export table)
EXPORTS = [
    "s2c_last_error", "s2c_abi_version", "s2c_layout",
    "s2c_parser_new", "s2c_parser_feed", "s2c_parser_feed_file", "s2c_parser_finish", "s2c_parser_free",
    "s2c_batch_info_get", "s2c_batch_arrays_get", "s2c_batch_ref_name", "s2c_batch_free",
    "s2c_parsecigar", "s2c_synth_feed", "s2c_synth_write",
    "s2c_workspace_sizes", "s2c_pileup", "s2c_consensus", "s2c_run",
]


def _load():
    # One HIP runtime per process: torch (the device allocator) brings its own
    # libamdhip64.so.7; loading it first makes libs2c.so's DT_NEEDED libamdhip64.so.7 bind
    # to that same copy instead of mapping /opt/rocm's as a second runtime (which then
    # reports hipErrorNoDevice for our launches).
    import torch  # noqa: F401
    if not os.path.exists(LIB_PATH):
        raise ImportError("libs2c.so not built (%s): run `make` or __graft_entry__.build()" % LIB_PATH)
    lib = C.CDLL(LIB_PATH)
    pp = C.POINTER(C.c_void_p)
    sig = {
        "s2c_last_error": (C.c_char_p, []),
        "s2c_abi_version": (C.c_int, []),
        "s2c_layout": (C.c_int, [C.POINTER(C.c_int64), C.c_int]),
        "s2c_parser_new": (C.c_int, [C.c_int, C.c_int64, pp]),
        "s2c_parser_feed": (C.c_int, [_VP, C.c_char_p, C.c_size_t]),
        "s2c_parser_feed_file": (C.c_int, [_VP, C.c_char_p]),
        "s2c_parser_finish": (C.c_int, [_VP, pp]),
        "s2c_parser_free": (None, [_VP]),
        "s2c_batch_info_get": (C.c_int, [_VP, C.POINTER(BatchInfo)]),
        "s2c_batch_arrays_get": (C.c_int, [_VP, C.POINTER(BatchArrays)]),
        "s2c_batch_ref_name": (C.c_char_p, [_VP, C.c_int64]),
        "s2c_batch_free": (None, [_VP]),
        "s2c_parsecigar": (C.c_int, [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_int64,
                                     C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t),
                                     C.POINTER(C.c_int64), C.c_size_t, C.POINTER(C.c_size_t)]),
        "s2c_synth_feed": (C.c_int, [C.POINTER(SynthSpec), _VP, C.POINTER(C.c_int64)]),
        "s2c_synth_write": (C.c_int, [C.POINTER(SynthSpec), C.c_char_p, C.POINTER(C.c_int64)]),
        "s2c_workspace_sizes": (C.c_int, [C.POINTER(BatchInfo), C.c_int32, C.POINTER(WsSizes)]),
        "s2c_pileup": (C.c_int, [C.POINTER(Dev), _VP]),
        "s2c_consensus": (C.c_int, [C.POINTER(Dev), _VP]),
        "s2c_run": (C.c_int, [C.POINTER(Dev), _VP]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()


def _layout_check():
    """Compare the ctypes mirrors with the C structs (sizeof / offsetof)."""
    buf = (C.c_int64 * 16)()
    n = lib.s2c_layout(buf, 16)
    want = [C.sizeof(Dev), Dev.tile_max.offset, Dev.thresholds.offset, Dev.fill.offset,
            Dev.counts.offset, Dev.ins_chr.offset, Dev.tile_stats.offset, Dev.out_cap.offset,
            C.sizeof(SynthSpec), SynthSpec.seed.offset, C.sizeof(BatchInfo), C.sizeof(BatchArrays),
            C.sizeof(WsSizes)]
    got = list(buf[:n])
    if got != want:
        raise ImportError("libs2c.so ABI mismatch: C %r vs ctypes %r" % (got, want))


_layout_check()


def last_error():
    m = lib.s2c_last_error()
    return m.decode("latin-1") if m else ""


def check(rc):
    """Raise the reference's exception class (or S2CError) for a non-zero status."""
    if rc == S2C_OK:
        return
    msg = last_error()
    exc = _EXC.get(rc)
    if exc is not None:
        raise exc(msg)
    raise S2CError(rc, msg)
