"""CPU model of the four HIP stages, reading the PACKED BATCH exactly as the kernels do
(test infrastructure only).

It lets the CPU suite check the host side of the product — parser, packing, wrap
splitting, tile plan, block plan, insertion events, record formatting — against the
reference's golden outputs without a GPU, and gives the GPU tests a second,
kernel-shaped expectation (e.g. counts[6][L]) to diff against.
"""
from __future__ import annotations

import numpy as np

NSYM = 6
AMB = None


def _amb():
    global AMB
    if AMB is None:
        import os
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
        import s2c_oracle
        AMB = [None if c is None else ord(c) for c in s2c_oracle.AMB_TABLE]
    return AMB


def read_codes(hb, r):
    """Read piece r: (start, drop, effective ops [(cls, len)], seqout codes).  The packed
    planes hold the piece's seqout — M bases and '-' (code 0) for D/N/P — checked here
    against the effective ops."""
    o0 = int(hb.rd_op[r])
    o1 = int(hb.rd_op[r + 1])
    drop = bool(int(hb.rd_span[r]) >> 31)
    span = int(hb.rd_span[r]) & 0x3FFFFFFF
    assert sum(int(w) >> 1 for w in hb.ops[o0:o1]) == span
    assert bool(int(hb.rd_span[r]) >> 30 & 1) == (not drop and o1 - o0 == 1 and (int(hb.ops[o0]) & 1) == 0)
    ops = [(int(w) & 1, int(w) >> 1) for w in hb.ops[o0:o1]]
    w0 = int(hb.rd_base[r])
    assert int(hb.rd_base[r + 1]) - w0 == 3 * ((span + 31) // 32 + 1)
    assert not hb.bases[w0 + 3 * ((span + 31) // 32):w0 + 3 * ((span + 31) // 32 + 1)].any()
    words = hb.bases[w0:w0 + 3 * ((span + 31) // 32)].astype(np.int64).reshape(-1, 3)
    q = np.arange(span)
    bits = (words[q >> 5] >> (q & 31)[:, None]) & 1
    codes = (bits * np.array([1, 2, 4])).sum(axis=1)
    k = 0
    for cls, ln in ops:
        if cls == 1:
            assert not codes[k:k + ln].any()
        k += ln
    return int(hb.rd_pos[r]), drop, ops, codes


def read_arrays(hb, r):
    """Read r as (positions, symbol codes) of the entries the pileup counts: every seqout
    position, except '-' when the read is maxdel-dropped (:214-218)."""
    s, drop, ops, codes = read_codes(hb, r)
    pos = np.arange(s, s + len(codes), dtype=np.int64)
    c = np.asarray(codes, dtype=np.int64)
    if drop:
        keep = c != 0
        pos, c = pos[keep], c[keep]
    return pos, c


def model_counts(hb):
    """counts[6][padded_len] following k_pileup's item/tile/extras walk."""
    Lp = hb.info.padded_len
    counts = np.zeros((NSYM, Lp), dtype=np.int64)
    cache = {}
    for it in hb.items:
        a, b, lo, hi, xlo, xhi = (int(v) for v in it[:6])
        reads = list(range(lo, hi)) + [int(x) for x in hb.extras[xlo:xhi]]
        for r in reads:
            if r not in cache:
                cache[r] = read_arrays(hb, r)
            p, c = cache[r]
            m = (p >= a) & (p < b)
            np.add.at(counts, (c[m], p[m]), 1)
    return counts


def check_plan(hb):
    """Every real position is owned by exactly one tile; chunks of one tile share [a,b)."""
    Lp = hb.info.padded_len
    own = np.zeros(Lp, dtype=np.int64)
    seen = set()
    for it in hb.items:
        a, b, flags = int(it[0]), int(it[1]), int(it[6])
        if (a, b) in seen:
            assert flags & 1, "multi-item tile must be atomic"
            continue
        seen.add((a, b))
        own[a:b] += 1
    for r in range(hb.info.n_refs):
        o, L = int(hb.ref_off[r]), int(hb.ref_len[r])
        assert (own[o:o + L] == 1).all(), "ref %d positions not tiled exactly once" % r


def _vote(c, cov, t):
    amb = _amb()
    m = 0
    for i in range(NSYM):
        if c[i] != 0 and float(sum(x for x in c if x > c[i])) < t * float(cov):
            m |= 1 << i
    ch = amb[m]
    return 0xFF if ch is None else ch


def model_pipeline(hb, thresholds, min_depth=1, fill=b"-"):
    """(stats[R,T,4], offs[T*nb+1], out bytes) as the device produces them."""
    counts = model_counts(hb)
    Lp = hb.info.padded_len
    T = len(thresholds)
    cov = counts.sum(axis=0)
    # insertion columns per key (:264-294)
    cols = {}
    for e in range(hb.info.n_ins):
        key = int(hb.ins_key[e])
        o0, o1 = int(hb.ins_off[e]), int(hb.ins_off[e + 1])
        cl = cols.setdefault(key, [])
        for c in range(o1 - o0):
            q = o0 + c
            code = (int(hb.ins_bases[q >> 3]) >> (4 * (q & 7))) & 15
            while len(cl) <= c:
                cl.append([0] * NSYM)
            cl[c][code] += 1
    nb = hb.info.n_blocks
    R = hb.info.n_refs
    stats = np.zeros((R, T, 4), dtype=np.uint64)
    blk_len = np.zeros(T * nb + 1, dtype=np.int64)
    pieces = [[None] * nb for _ in range(T)]
    fl = len(fill)
    fnd = sum(1 for ch in fill if ch != ord("-"))
    for bi, (g0, g1, ref, _) in enumerate(hb.blocks):
        g0, g1, ref = int(g0), int(g1), int(ref)
        for ti, t in enumerate(thresholds):
            buf = bytearray()
            sumcov = length = nondash = nerr = 0
            for p in range(g0, g1):
                cv = int(cov[p])
                called = cv > 0 and cv >= min_depth
                if not called:
                    buf += fill
                    length += fl
                    nondash += fnd
                    sumcov += cv
                    continue
                ch = _vote([int(x) for x in counts[:, p]], cv, t)
                nerr += ch == 0xFF
                buf.append(ch if ch != 0xFF else 63)
                emitted = 0
                for col in cols.get(p, []):
                    v = list(col)
                    v[0] = cv - sum(col)
                    c2 = _vote(v, cv, t)
                    if c2 == 0xFF:
                        nerr += 1
                        continue
                    if c2 != ord("-"):
                        buf.append(c2)
                        emitted += 1
                length += 1 + emitted
                nondash += (ch != ord("-")) + emitted
                sumcov += cv * (1 + emitted)
            stats[ref, ti] += np.array([sumcov, length, nondash, nerr], dtype=np.uint64)
            blk_len[ti * nb + bi] = length
            pieces[ti][bi] = bytes(buf)
    offs = np.zeros(T * nb + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(blk_len[:-1])
    out = b"".join(pieces[ti][bi] for ti in range(T) for bi in range(nb))
    return stats, offs, out
