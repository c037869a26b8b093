"""The ``s2c_dev`` argument block of one run (include/s2c.h) from a batch's info and the
device addresses of its arrays and workspace buffers — shared by the torch-backed engine
(engine.Workspace) and the torch-free whole-file CLI path (hiprun.py).  No torch here."""
from __future__ import annotations

from . import _lib as L

# the packed batch's device arrays, in upload order (s2c_dev's pointer fields)
ARRAYS = ("pc", "ops", "bq", "bx", "rs", "tiles", "items", "dense", "deep", "lp", "wtile", "rlist", "ps",
          "lly", "lpc", "lops", "lbq", "lbx", "px", "dwin", "lpx", "dpc")
# the workspace buffers a run writes (s2c_workspace_sizes), plus the thresholds and fill
BUFFERS = ("runs", "ibkt", "ilong", "ilong_n", "counts", "ins_cols", "ins_chr", "tile_stats", "blk_len", "out")


def fill_dev(info, arrays, bufs, n_thr, min_depth, fill, maxdel_active, maxdel, out_cap):
    """``arrays``: name → device address of each of ARRAYS; ``bufs``: name → device address of
    each of BUFFERS and of ``thresholds`` (n_thr f64) and ``fill`` (its bytes)."""
    i = info
    d = L.Dev()
    for name in ARRAYS:
        setattr(d, name, arrays[name])
    d.n_pieces, d.n_ops, d.n_qwords, d.n_tiles = i.n_pieces, i.n_ops, i.n_qwords, i.n_tiles
    d.n_items, d.n_dense, d.n_deep = i.n_items, i.n_dense, i.n_deep
    d.padded_len, d.chunk, d.kwin, d.tile_max = i.padded_len, i.chunk, i.kwin, i.tile_max
    d.dense_lds = i.dense_lds
    d.n_rlist = i.n_rlist
    d.n_layers, d.n_lpieces, d.n_lops, d.n_lqwords = i.n_layers, i.n_lpieces, i.n_lops, i.n_lqwords
    d.layers_dense, d.layers_built = i.layers_dense, i.layers_built
    d.word_lo, d.word_hi = i.word_lo, i.word_hi
    d.walk_queue, d.tile_events, d.n_rlist_run = i.walk_queue, i.tile_events, i.n_rlist_run
    d.maxdel_active, d.maxdel = 1 if maxdel_active else 0, int(maxdel)
    d.thresholds, d.n_thr = bufs["thresholds"], int(n_thr)
    d.min_depth = int(max(min(min_depth, 2**31 - 1), -2**31))
    fill = bytes(fill)
    d.fill_len, d.fill_nondash = len(fill), sum(1 for c in fill if c != ord("-"))
    d.fill = bufs["fill"]
    for name in BUFFERS:
        setattr(d, name, bufs[name])
    d.n_cols = i.n_cols
    d.out_cap = int(out_cap)
    return d
