"""BASELINE.json's five workloads as deterministic synthetic specs.

| id | workload                                                        | CLI flags            |
|----|-----------------------------------------------------------------|----------------------|
| c1 | 10 genes × 1 kb, 100x, 150 bp                                   | -c 0.25              |
| c2 | Hyb-seq 353 loci × 1 kb, 500x, 5 % 1-4 bp I, 5 % 1-5 bp D       | -c 0.25,0.50,0.75    |
| c3 | bacterial 5 Mb, 1000x, shuffled records (SAM.gz)                 | -m 10                |
| c4 | chrM 16,569 bp, 100,000x, 166 tiled amplicon starts              | (defaults)           |
| c5 | chr20 64,444,167 bp, 30x, 1 % D reads (0.1 % of them > 150 bp)   | -d 150               |
"""
from __future__ import annotations

import ctypes as C

from . import _lib as L
from .batch import HostBatch, Parser

CONFIGS = {
    "c1": dict(n_refs=10, ref_len=1000, depth=100.0, args=["-c", "0.25"], prefix="gene"),
    "c2": dict(n_refs=353, ref_len=1000, depth=500.0, ins_frac=0.05, ins_max=4, del_frac=0.05, del_max=5,
               args=["-c", "0.25,0.50,0.75"], prefix="locus"),
    "c3": dict(n_refs=1, ref_len=5_000_000, depth=1000.0, shuffle=1, args=["-m", "10"], prefix="chr"),
    "c4": dict(n_refs=1, ref_len=16569, depth=100000.0, amplicons=166, args=[], prefix="chrM"),
    "c4u": dict(n_refs=1, ref_len=16569, depth=100000.0, args=[], prefix="chrM"),
    "c5": dict(n_refs=1, ref_len=64_444_167, depth=30.0, del_frac=0.01, del_max=5, long_del_frac=0.001,
               args=["-d", "150"], prefix="chr20_"),
    # C5 without -d: the maxdel filter (:210) is active, the long-deletion reads' '-' are dropped
    "c5nd": dict(n_refs=1, ref_len=64_444_167, depth=30.0, del_frac=0.01, del_max=5, long_del_frac=0.001,
                 args=[], prefix="chr20_"),
}
SEED = 20260115


def spec(name, seed=SEED, scale=1.0, **over):
    """SynthSpec for config ``name``; ``scale`` shrinks the number of refs (or length)."""
    c = dict(CONFIGS[name])
    c.update(over)  # e.g. ref_len / depth / n_refs overrides for reduced-size tests
    n_refs, ref_len = c["n_refs"], c["ref_len"]
    if scale != 1.0:
        if n_refs > 1:
            n_refs = max(1, int(round(n_refs * scale)))
        else:
            ref_len = max(400, int(ref_len * scale))
    s = L.SynthSpec()
    s.n_refs = n_refs
    s.ref_len = ref_len
    s.depth = c["depth"]
    s.read_len = c.get("read_len", 150)
    s.ins_frac = c.get("ins_frac", 0.0)
    s.ins_max = c.get("ins_max", 1)
    s.del_frac = c.get("del_frac", 0.0)
    s.del_max = c.get("del_max", 1)
    s.long_del_frac = c.get("long_del_frac", 0.0)
    s.sub_rate = c.get("sub_rate", 0.01)
    s.n_rate = c.get("n_rate", 0.001)
    s.amplicons = c.get("amplicons", 0)
    s.shuffle = c.get("shuffle", 0)
    s.seed = seed
    s._prefix = c["prefix"].encode()  # keep alive
    s.ref_prefix = s._prefix
    return s


def cli_args(name):
    return list(CONFIGS[name]["args"])


def maxdel_active(args):
    return "-d" not in args and "--maxdel" not in args


def synth_batch(name, seed=SEED, scale=1.0, **over) -> HostBatch:
    """Generate config ``name`` and stream its SAM text through the parser (no file)."""
    sp = spec(name, seed, scale, **over)
    p = Parser(maxdel_active(cli_args(name)), 150)
    try:
        n = C.c_int64()
        L.check(L.lib.s2c_synth_feed(C.byref(sp), p._p, C.byref(n)))
        return p.finish()
    finally:
        p.close()


def synth_write(name, path, seed=SEED, scale=1.0, **over):
    sp = spec(name, seed, scale, **over)
    n = C.c_int64()
    L.check(L.lib.s2c_synth_write(C.byref(sp), path.encode(), C.byref(n)))
    return n.value
