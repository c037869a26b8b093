"""FASTA records from device results — header formatting with the reference's
Python-2 number semantics and the file layout of sam2consensus.py:394-418."""
from __future__ import annotations

import decimal
import math


def py2_round(x, n=2):
    """CPython 2.7 ``round(x, n)`` (sam2consensus.py:395): correctly rounded, with exact
    binary ties (odd multiples of 2^-(n+1)) rounded away from zero — Python 3 would
    round those half-to-even (9/8 → 1.13 here, 1.12 under Python 3)."""
    x = float(x)
    if x == 0.0 or math.isnan(x) or math.isinf(x):
        return x
    q = decimal.Decimal(1).scaleb(-n)
    return float(decimal.Decimal(x).quantize(q, context=decimal.Context(prec=400, rounding=decimal.ROUND_HALF_UP)))


def py2_str(x):
    """CPython 2.7 ``str(float)``: ``'%.12g'``, plus ``'.0'`` when the result reads as an integer."""
    s = "%.12g" % x
    if s.lstrip("-").isdigit():
        s += ".0"
    return s


def build_records(hb, thresholds, prefix, stats, offs, out):
    """{refname: [(header_bytes, body_bytes), ...]} exactly as :344-406 keeps them.

    Raises the reference's exception class for the first failing (ref, threshold):
    KeyError (vote hit a missing amb key, :367/:381), ValueError / OverflowError
    (int(t*100) of nan / inf, :394), ZeroDivisionError (empty record, :395)."""
    i = hb.info
    T, nb = len(thresholds), i.n_tiles
    fastas = {}
    pre = prefix.encode("latin-1") if isinstance(prefix, str) else prefix
    for r in range(i.n_refs):
        if hb.ref_reads[r] == 0:           # Σcoverage == 0 → erased (:334-341)
            continue
        name = hb.names[r]
        f0, n = int(hb.ref_first_block[r]), int(hb.ref_nblocks[r])
        for ti, t in enumerate(thresholds):
            sumcov, length, nondash, nerr = (int(v) for v in stats[r, ti])
            if nerr:
                raise KeyError("consensus vote selected a symbol set absent from amb (:367)")
            tag = str(int(t * 100))                                          # :394
            cov = py2_str(py2_round(float(sumcov) / float(length), 2))       # :395
            a, b = int(offs[ti * nb + f0]), int(offs[ti * nb + f0 + n])
            body = out[a:b]
            if nondash > 0:                                                  # :400
                hdr = (b">" + pre + b"|c" + tag.encode() + b" reference:" + name.encode("latin-1") +
                       b" coverage:" + cov.encode() + b" length:" + str(nondash).encode() +
                       b" consensus_threshold:" + tag.encode() + b"%")
                fastas.setdefault(name, []).append((hdr, body))
    return fastas


def render(recs, nchar):
    """File content of one reference (:414-417)."""
    if nchar == 0:
        return b"\n".join(h + b"\n" + s for h, s in recs) + b"\n"
    return b"\n".join(h + b"\n" + b"\n".join(s[k:k + nchar] for k in range(0, len(s), nchar))
                      for h, s in recs) + b"\n"
