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


SYM_OF_BASE = np.array([1, 2, 3, 5], dtype=np.int64)   # 2-bit base (A C G T) → symbol index of "-ACGNT"


def record_bases(recs):
    """Records [n][2] bit-planes → 2-bit bases [n][32] (b1·2+b0: A C G T)."""
    q = np.arange(32, dtype=np.int64)
    r = np.asarray(recs, dtype=np.int64)
    return ((r[:, 0, None] >> q) & 1) + 2 * ((r[:, 1, None] >> q) & 1)


def model_counts(hb, block=1 << 18):
    """counts[6][padded_len] from the packed batch, as k_pileup forms them: every record
    position counted as its 2-bit base (placeholders as A), minus the A placeholders (fix),
    plus the '-'/'N' entries (exc), both per work item."""
    Lp = hb.info.padded_len
    wrec = hb.wrec.astype(np.int64)
    assert wrec[0] == 0 and wrec[-1] == hb.info.n_recs and (np.diff(wrec) >= 0).all()
    word_of = np.repeat(np.arange(Lp // 32, dtype=np.int64), np.diff(wrec))
    flat = np.zeros(NSYM * Lp, dtype=np.int64)
    for k in range(0, len(word_of), block):
        sym = SYM_OF_BASE[record_bases(hb.recs[k:k + block])]
        pos = word_of[k:k + block, None] * 32 + np.arange(32)
        flat += np.bincount((sym * Lp + pos).reshape(-1), minlength=NSYM * Lp)
    counts = flat.reshape(NSYM, Lp)
    fix = hb.fix.astype(np.int64)
    for a, b, _, _, fo, x0, x1 in hb.items[:, :7].astype(np.int64):   # per work item
        nw = (b + 31) // 32 - a // 32
        f = fix[fo:fo + 16 * nw].reshape(nw, 16)
        ph = np.concatenate([f & 0xFFFF, f >> 16], axis=1).reshape(-1)   # tile positions a..a+32·nw
        counts[1, a:a + 32 * nw] -= ph
        e = hb.exc[x0:x1].astype(np.int64)
        pos = a + (e >> 1)
        assert (pos < b).all()
        np.add.at(counts, (np.where(e & 1, 4, 0), pos), 1)
    for a, b in hb.blocks[:, :2].astype(np.int64):
        w1 = (b + 31) // 32 * 32
        assert (counts[1, a:w1] >= 0).all(), "A placeholders exceed the A-counted record positions"
    return counts


def check_plan(hb):
    """Every real position is owned by exactly one tile; a tile's items are chunks
    0..nch-1 whose record ranges cover every word of the tile; deep (flag bit 0) = nch > 1."""
    Lp = hb.info.padded_len
    own = np.zeros(Lp, dtype=np.int64)
    wrec = hb.wrec.astype(np.int64)
    ch = int(hb.info.chunk_recs)
    assert ch > 0
    chunks = {}
    for a, b, c, t in hb.items[:, :4].astype(np.int64):
        chunks.setdefault(int(t), []).append(int(c))
        assert (int(hb.blocks[t, 0]), int(hb.blocks[t, 1])) == (a, b)
    for t, (a, b, ref, deep) in enumerate(hb.blocks[:, :4].astype(np.int64)):
        cs = sorted(chunks[t])
        assert cs == list(range(len(cs))), "tile %d chunks %r" % (t, cs)
        assert bool(deep & 1) == (len(cs) > 1)
        assert a % 32 == 0
        words = np.arange(a // 32, (b + 31) // 32)
        assert (wrec[words + 1] - wrec[words]).max(initial=0) <= len(cs) * ch
        own[a:b] += 1
    for r in range(hb.info.n_refs):
        o, L = int(hb.ref_off[r]), int(hb.ref_len[r])
        assert (own[o:o + L] == 1).all(), "ref %d positions not tiled exactly once" % r
    check_item_descriptors(hb)
    check_ins_layout(hb)


def check_item_descriptors(hb):
    """Item words 7-13 copy their tile's block words 3-9, word 14 is the item's first record,
    and iwr holds each word's record range of the item's chunk."""
    it = hb.items.astype(np.int64)
    bl = hb.blocks.astype(np.int64)
    wrec = hb.wrec.astype(np.int64)
    ch = int(hb.info.chunk_recs)
    assert (it[:, 7:14] == bl[it[:, 3], 3:10]).all()
    assert (it[:, 14] == wrec[it[:, 0] >> 5]).all()
    nwp = hb.info.n_iwr // max(hb.info.n_items, 1) // 2
    iw = hb.iwr.astype(np.int64).reshape(-1, nwp, 2)
    for k, (a, b, c) in enumerate(it[:, :3]):
        for w in range(nwp):
            if 32 * w < b - a:
                W = (a >> 5) + w
                r0 = min(wrec[W + 1], wrec[W] + c * ch)
                assert (iw[k, w] == (r0, min(wrec[W + 1], r0 + ch))).all()
            else:
                assert (iw[k, w] == 0).all()


def check_ins_layout(hb):
    """Keys ascending and unique; bitmap/rank give each key's index; count units cover
    every event of their key exactly once, ≤ S2C_INS_UNIT events each."""
    nk = hb.info.n_keys
    key = hb.ins_key.astype(np.int64)
    assert (np.diff(key) > 0).all()
    bits = hb.ins_bits.astype(np.int64)
    pos = np.nonzero(((bits[:, None] >> np.arange(32)) & 1).reshape(-1))[0]
    assert (pos == key).all()
    rank = hb.ins_rank.astype(np.int64)
    assert rank[-1] == nk and (rank[key >> 5] + [int(bin(int(bits[k >> 5]) & ((1 << (k & 31)) - 1)).count("1"))
                                                 for k in key] == np.arange(nk)).all()
    koff = hb.ins_koff.astype(np.int64)
    assert koff[0] == 0 and koff[-1] == hb.info.n_ins and (np.diff(koff) > 0).all()
    ekey = hb.ins_ekey.astype(np.int64)
    assert (ekey == np.repeat(np.arange(nk), np.diff(koff))).all()
    check_device_records(hb)


def check_device_records(hb):
    """The device's 16-B event/key records and the tiles' insertion ranges (block words
    4-9) restate the grouped arrays exactly."""
    koff, kcol = hb.ins_koff.astype(np.int64), hb.ins_kcol.astype(np.int64)
    off = hb.ins_off.astype(np.int64)
    ki = hb.ins_kinfo.astype(np.int64)
    assert (ki[:, 0] == hb.ins_key).all() and (ki[:, 1] == kcol[:-1]).all() and (ki[:, 2] == np.diff(kcol)).all()
    ev = hb.ins_ev.astype(np.int64)
    rank = hb.ins_rank.astype(np.int64)
    seen = np.zeros(len(ev), np.int64)
    for a, b, _, _, klo, khi, e0, e1, cb0, cb1 in hb.blocks[:, :10].astype(np.int64):
        assert (klo, khi) == (rank[a >> 5], rank[(b + 31) >> 5])
        assert (e0, e1, cb0, cb1) == (koff[klo], koff[khi], kcol[klo], kcol[khi])
        for k in range(klo, khi):
            for e in range(koff[k], koff[k + 1]):
                seen[e] += 1
                n = off[e + 1] - off[e]
                assert (ev[e, 0], ev[e, 1], ev[e, 2]) == (kcol[k] - cb0, n, off[e])
                w0 = 0
                for c in range(min(n, 8)):
                    q = off[e] + c
                    w0 |= ((int(hb.ins_bases[q >> 3]) >> (4 * (q & 7))) & 15) << (4 * c)
                assert ev[e, 3] == w0
    assert (seen == 1).all()


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
    for k in range(hb.info.n_keys):
        key = int(hb.ins_key[k])
        cl = cols.setdefault(key, [])
        for e in range(int(hb.ins_koff[k]), int(hb.ins_koff[k + 1])):
            o0, o1 = int(hb.ins_off[e]), int(hb.ins_off[e + 1])
            for c in range(o1 - o0):
                q = o0 + c
                code = (int(hb.ins_bases[q >> 3]) >> (4 * (q & 7))) & 15
                while len(cl) <= c:
                    cl.append([0] * NSYM)
                cl[c][code] += 1
        assert len(cl) == int(hb.ins_kcol[k + 1]) - int(hb.ins_kcol[k])
    nb = hb.info.n_blocks
    R = hb.info.n_refs
    stats = np.zeros((R, T, 4), dtype=np.uint64)
    blk_len = np.zeros(T * nb + 1, dtype=np.int64)
    pieces = [[None] * nb for _ in range(T)]
    fl = len(fill)
    fnd = sum(1 for ch in fill if ch != ord("-"))
    for bi, (g0, g1, ref, _) in enumerate(hb.blocks[:, :4]):
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
                buf.append(ch)   # 0xFF at a vote error (the run raises KeyError; bytes unused)
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
