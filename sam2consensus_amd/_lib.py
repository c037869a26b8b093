"""ctypes binding of libs2c.so (include/s2c.h).

The shared library is built in-tree (``make`` / ``__graft_entry__.build()``) and
loaded from this package directory.  There is no fallback: if the library is
missing the import fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, os.environ.get("S2C_LIB", "libs2c.so"))

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
ABI_VERSION = 14      # include/s2c.h S2C_ABI_VERSION: the structs below mirror this version
S2C_TILE_WORDS = 24
S2C_LY_MAIN = 0xFFFFFFFF
S2C_ITEM_WORDS = 4
S2C_DWIN_WORDS = 16
S2C_DPC_WORDS = 3     # compact piece records of the dense windows (ABI 12)
S2C_CODE_FILL = 0
S2C_SHORT_MOTIF = 16
S2C_TILE_DEEP, S2C_TILE_GENERAL, S2C_TILE_DENSE = 1, 2, 4
S2C_PF_X, S2C_PF_RANGE, S2C_PF_INS, S2C_PF_LONG, S2C_PF_RUNS, S2C_PF_DASH = 1, 2, 4, 8, 16, 32
S2C_PF_SIMPLE, S2C_PF_XFEW = 64, 128
S2C_RUN_EMPTY, S2C_RUN_BASES, S2C_RUN_DASH = 0, 1, 2
S2C_RUN_XBIT, S2C_RUN_DROP, S2C_RUN_LONG = 4, 8, 16
OPS = "MIDNSHP=X"   # opcode order of the token words (len << 4 | opcode)

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
        "aligned_bases", "query_bases", "n_pieces", "n_ops", "n_tokens", "n_qwords", "n_words",
        "n_tiles", "n_items", "n_dense", "n_deep", "n_long", "n_rlist", "kwin", "tile_max", "chunk",
        "n_ins", "n_ins_bases", "n_bkt", "n_lng", "n_cols", "runs_max", "dense_lds", "n_layers", "n_lpieces", "n_lops",
        "n_lqwords", "layers_dense", "layers_built", "n_dpc", "word_lo", "word_hi", "n_walked", "walk_queue", "tile_events", "n_rlist_run", "plan_t0", "plan_t1")]


_P64 = C.POINTER(C.c_int64)
_P32 = C.POINTER(C.c_uint32)


class BatchArrays(C.Structure):
    _fields_ = [("ref_len", _P64), ("ref_off", _P64), ("ref_cov_reads", _P64)] + \
        [(n, _P32) for n in ("pc", "ops", "bq", "bx", "rs", "tiles", "items", "dense", "deep", "rlist", "lp", "wtile",
                             "ps", "lly", "lpc", "lops", "lbq", "lbx", "px", "dwin", "lpx", "dpc")]


class SynthSpec(C.Structure):
    _fields_ = [("n_refs", C.c_int32), ("ref_len", C.c_int64), ("depth", C.c_double),
                ("read_len", C.c_int32), ("ins_frac", C.c_double), ("ins_max", C.c_int32),
                ("del_frac", C.c_double), ("del_max", C.c_int32), ("long_del_frac", C.c_double),
                ("sub_rate", C.c_double), ("n_rate", C.c_double), ("amplicons", C.c_int32),
                ("shuffle", C.c_int32), ("seed", C.c_uint64), ("ref_prefix", C.c_char_p)]


_VP = C.c_void_p


class Dev(C.Structure):
    """Mirror of ``s2c_dev`` (include/s2c.h)."""
    _fields_ = [(n, _VP) for n in ("pc", "ops", "bq", "bx", "rs", "tiles", "items", "dense", "deep", "lp", "wtile",
                                   "rlist", "ps", "lly", "lpc", "lops", "lbq", "lbx")] + \
        [(n, C.c_int64) for n in ("n_pieces", "n_ops", "n_qwords", "n_tiles", "n_items", "n_dense", "n_deep",
                                  "padded_len", "chunk", "n_rlist", "dense_lds", "n_layers", "n_lpieces", "n_lops",
                                  "n_lqwords")] + [
        ("kwin", C.c_int32), ("tile_max", C.c_int32),
        ("maxdel_active", C.c_int32), ("maxdel", C.c_int32),
        ("thresholds", _VP), ("n_thr", C.c_int32), ("min_depth", C.c_int32),
        ("fill_len", C.c_int32), ("fill_nondash", C.c_int32), ("fill", _VP),
        ("runs", _VP), ("ibkt", _VP), ("ilong", _VP), ("ilong_n", _VP), ("counts", _VP),
        ("ins_cols", _VP), ("ins_chr", _VP), ("n_cols", C.c_int64),
        ("tile_stats", _VP), ("blk_len", _VP), ("out", _VP), ("out_cap", C.c_int64), ("layers_dense", C.c_int64),
        ("px", _VP), ("layers_built", C.c_int64), ("dwin", _VP), ("lpx", _VP), ("dpc", _VP), ("walk_queue", C.c_int64), ("tile_events", C.c_int64), ("n_rlist_run", C.c_int64), ("word_lo", C.c_int64),
        ("word_hi", C.c_int64)]


class WsSizes(C.Structure):
    _fields_ = [(n, C.c_int64) for n in (
        "runs", "ibkt", "ilong", "ilong_n", "counts", "ins_cols", "ins_chr", "blk_len", "tile_stats",
        "out_per_fill", "out_fixed")]


# every symbol include/s2c.h declares (tests/test_lib.py checks the export table)
EXPORTS = [
    "s2c_last_error", "s2c_abi_version", "s2c_layout",
    "s2c_parser_new", "s2c_parser_feed", "s2c_parser_end_header", "s2c_parser_feed_file", "s2c_parser_finish", "s2c_parser_free",
    "s2c_reader_open", "s2c_reader_read", "s2c_reader_free",
    "s2c_parser_set_tile_width", "s2c_parser_snapshot", "s2c_parser_snapshot_from", "s2c_parser_retain", "s2c_parser_stream_state",
    "s2c_parser_retain_events", "s2c_parser_detach", "s2c_parser_attach", "s2c_accumulate",
    "s2c_parser_pos_weights", "s2c_parser_checks", "s2c_parser_counters", "s2c_parser_progress", "s2c_gather_bodies", "s2c_copy_bytes", "s2c_parser_pack",
    "s2c_parser_blob_copy", "s2c_parser_unpack",
    "s2c_batch_layers", "s2c_batch_layers_mode", "s2c_batch_info_get", "s2c_batch_arrays_get", "s2c_batch_ref_name", "s2c_batch_free", "s2c_batch_shard",
    "s2c_parsecigar", "s2c_synth_feed", "s2c_synth_write",
    "s2c_workspace_sizes", "s2c_reads", "s2c_pileup", "s2c_consensus", "s2c_run", "s2c_pileup_counts",
    "s2c_gather_bodies_dev", "s2c_plan_set_cus",
]


def _hip_runtime():
    """One HIP runtime per process: torch (the library paths' device allocator) brings its own
    libamdhip64.so.7; mapping that file first (by path, RTLD_GLOBAL — without importing torch,
    1.8 s on the box) makes libs2c.so's DT_NEEDED libamdhip64.so.7 bind to that same copy, and
    a later `import torch` reuses it, instead of /opt/rocm's being mapped as a second runtime
    (which then reports hipErrorNoDevice for our launches).  Without torch: the system's."""
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is not None and spec.origin:
        path = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
        if os.path.exists(path):
            C.CDLL(path, mode=C.RTLD_GLOBAL)


def _load():
    _hip_runtime()
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
        "s2c_parser_end_header": (C.c_int, [_VP]),
        "s2c_parser_feed_file": (C.c_int, [_VP, C.c_char_p]),
        "s2c_parser_finish": (C.c_int, [_VP, pp]),
        "s2c_parser_free": (None, [_VP]),
        "s2c_reader_open": (C.c_int, [C.c_char_p, pp]),
        "s2c_reader_read": (C.c_int, [_VP, _VP, C.c_size_t, C.POINTER(C.c_size_t)]),
        "s2c_reader_free": (None, [_VP]),
        "s2c_parser_set_tile_width": (C.c_int, [_VP, C.c_int64]),
        "s2c_parser_snapshot": (C.c_int, [_VP, pp]),
        "s2c_parser_snapshot_from": (C.c_int, [_VP, C.c_int64, pp]),
        "s2c_parser_retain": (C.c_int, [_VP, C.c_int64]),
        "s2c_parser_stream_state": (C.c_int, [_VP, C.POINTER(C.c_int64)]),
        "s2c_parser_retain_events": (C.c_int, [_VP]),
        "s2c_parser_detach": (C.c_int, [_VP, pp]),
        "s2c_parser_attach": (C.c_int, [_VP, _VP]),
        "s2c_accumulate": (C.c_int, [C.POINTER(Dev), C.c_int, _VP]),
        "s2c_parser_pos_weights": (C.c_int, [_VP, C.c_int64, C.POINTER(C.c_int64), C.c_int64]),
        "s2c_parser_checks": (C.c_int, [_VP, C.POINTER(C.c_uint8), C.c_int64]),
        "s2c_parser_counters": (C.c_int, [_VP, C.POINTER(C.c_int64)]),
        "s2c_parser_progress": (C.c_int, [_VP, C.POINTER(C.c_int64)]),
        "s2c_gather_bodies": (C.c_int, [_VP, C.c_int64, _VP, _VP, C.c_int64, _VP]),
        "s2c_copy_bytes": (C.c_int, [_VP, _VP, C.c_int64]),
        "s2c_parser_pack": (C.c_int, [_VP, C.c_int64, C.c_int64, C.POINTER(C.c_size_t)]),
        "s2c_parser_blob_copy": (C.c_int, [_VP, _VP, C.c_size_t]),
        "s2c_parser_unpack": (C.c_int, [_VP, _VP, C.c_size_t]),
        "s2c_batch_layers": (C.c_int, [_VP]),
        "s2c_batch_layers_mode": (C.c_int, [_VP, C.c_int]),
        "s2c_batch_info_get": (C.c_int, [_VP, C.POINTER(BatchInfo)]),
        "s2c_batch_arrays_get": (C.c_int, [_VP, C.POINTER(BatchArrays)]),
        "s2c_batch_ref_name": (C.c_char_p, [_VP, C.c_int64]),
        "s2c_batch_free": (None, [_VP]),
        "s2c_batch_shard": (C.c_int, [_VP, C.c_int64, C.c_int64, pp]),
        "s2c_parsecigar": (C.c_int, [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_int64,
                                     C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t),
                                     C.POINTER(C.c_int64), C.c_size_t, C.POINTER(C.c_size_t)]),
        "s2c_synth_feed": (C.c_int, [C.POINTER(SynthSpec), _VP, C.POINTER(C.c_int64)]),
        "s2c_synth_write": (C.c_int, [C.POINTER(SynthSpec), C.c_char_p, C.POINTER(C.c_int64)]),
        "s2c_workspace_sizes": (C.c_int, [C.POINTER(BatchInfo), C.c_int32, C.POINTER(WsSizes)]),
        "s2c_reads": (C.c_int, [C.POINTER(Dev), _VP]),
        "s2c_pileup": (C.c_int, [C.POINTER(Dev), _VP]),
        "s2c_pileup_counts": (C.c_int, [C.POINTER(Dev), _VP]),
        "s2c_consensus": (C.c_int, [C.POINTER(Dev), _VP]),
        "s2c_run": (C.c_int, [C.POINTER(Dev), _VP]),
        "s2c_gather_bodies_dev": (C.c_int, [_VP, C.c_int64, _VP, _VP, C.c_int64, _VP, _VP]),
        "s2c_plan_set_cus": (C.c_int, [C.c_int64]),
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
    want = [C.sizeof(Dev), Dev.kwin.offset, Dev.thresholds.offset, Dev.fill.offset,
            Dev.runs.offset, Dev.n_cols.offset, Dev.tile_stats.offset, Dev.out_cap.offset,
            C.sizeof(SynthSpec), SynthSpec.seed.offset, C.sizeof(BatchInfo), C.sizeof(BatchArrays),
            C.sizeof(WsSizes)]
    got = list(buf[:n])
    if got != want:
        raise ImportError("libs2c.so ABI mismatch: C %r vs ctypes %r" % (got, want))


if lib.s2c_abi_version() != ABI_VERSION:
    raise ImportError("libs2c.so ABI %d, these bindings ABI %d (rebuild: make)" % (lib.s2c_abi_version(), ABI_VERSION))
_layout_check()


def plan_for_device(device):
    """Plan batches for ``device``'s compute units (s2c_plan_set_cus: the deep tiles' grid
    shaping) — the product paths call it once they hold their GPU."""
    import torch
    check(lib.s2c_plan_set_cus(int(torch.cuda.get_device_properties(device).multi_processor_count)))


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
