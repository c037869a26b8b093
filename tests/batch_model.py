"""CPU model of the HIP stages, reading the PACKED BATCH exactly as the kernels do
(test infrastructure only).

It restates k_reads (the token walk of parsecigar :46-82 and the maxdel rule :210 per
piece → run records; insertion events with their global keys), the counting of the runs
(:210-218), the insertion columns (:262-294), the vote and the FASTA body layout, so the
CPU suite checks the host side of the product — parser, packing, bucketing, tile plan —
against the reference's golden outputs without a GPU, and the GPU tests get a
kernel-shaped expectation (run records, counts[6][L], per-tile stats and bodies).
"""
from __future__ import annotations

import numpy as np

S2C_DENSE_LDS = 32768   # include/s2c.h

NSYM = 6
AMB = None
OP_BASES = (0, 7, 8)        # M = X
OP_DASH = (2, 3, 6)         # D N P
OP_I, OP_S = 1, 4
PF_X, PF_RANGE, PF_INS, PF_LONG, PF_SIMPLE = 1, 2, 4, 8, 64
RUN_BASES, RUN_DASH, RUN_XBIT, RUN_DROP, RUN_LONG = 1, 2, 4, 8, 16
RUN_KSHIFT = 27   # include/s2c.h S2C_RUN_KSHIFT


def _amb():
    global AMB
    if AMB is None:
        import os
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
        import s2c_oracle
        AMB = [None if c is None else ord(c) for c in s2c_oracle.AMB_TABLE]
    return AMB


def plane_codes(hb, q, n):
    """3-bit plane codes x·4 + p1·2 + p0 of query bases [q, q + n) (A 0 C 1 G 2 T 3 N 4 '-' 5)."""
    idx = np.arange(q, q + n, dtype=np.int64)
    w, sh = idx >> 5, (idx & 31).astype(np.uint32)
    bq = hb.bq
    p0 = (bq[w, 0] >> sh) & 1
    p1 = (bq[w, 1] >> sh) & 1
    x = (hb.bx[w] >> sh) & 1
    return (x << 2 | p1 << 1 | p0).astype(np.int64)


CODE_SYM = np.array([1, 2, 3, 5, 4, 0, -1, -1], dtype=np.int64)   # plane code → "-ACGNT" index


def model_reads(hb, maxdel_active=None, maxdel=None, with_piece=False):
    """k_reads: (runs [n_ops][4] u32, events [(gkey, (sym, ...))]) from the packed batch
    (with_piece: events [(gkey, (sym, ...), piece)])."""
    if maxdel_active is None:
        maxdel_active = getattr(hb, "maxdel_active", True)
    if maxdel is None:
        maxdel = getattr(hb, "maxdel", 150)
    pc, ops = hb.pc.astype(np.int64), hb.ops.astype(np.int64)
    runs = np.zeros((max(hb.info.n_ops, 1), 4), dtype=np.uint32)
    events = []
    for i in range(hb.info.n_pieces):
        gpos, qh, o, w3 = (int(v) for v in pc[i])
        oend = int(pc[i + 1, 2])
        slen, fl = w3 & 0xFFFFFF, w3 >> 24
        ka, kb = 0, 1 << 62
        if fl & PF_RANGE:
            ka, kb = int(ops[o]), int(ops[o + 1])
            o += 2
        key0 = roff = 0
        if fl & PF_INS:
            key0 = int(ops[o]) | (int(ops[o + 1]) << 32)
            key0 = key0 - (1 << 64) if key0 >= 1 << 63 else key0
            roff = int(ops[o + 2])
            o += 3
        q0 = 16 * qh
        toks = [(int(w) & 15, int(w) >> 4) for w in ops[o:oend]]
        drop = False
        if maxdel_active:   # :210 — '-' of seqout: D/N/P lengths + '-' chars of the bases taken
            dashes, start = 0, 0
            for op, ln in toks:
                if op in OP_BASES:
                    take = max(0, min(ln, slen - start))
                    if take and fl & PF_X:   # '-' chars of SEQ: only reads with non-ACGT chars
                        dashes += int((plane_codes(hb, q0 + start, take) == 5).sum())
                    start += ln
                elif op in OP_DASH:
                    dashes += ln
                elif op in (OP_I, OP_S):
                    start += ln
            drop = dashes > maxdel
        lng = RUN_LONG if fl & PF_LONG else 0
        bkind = RUN_BASES | (RUN_XBIT if fl & PF_X else 0) | (RUN_DROP if drop else 0) | lng
        k = start = 0
        for j, (op, ln) in enumerate(toks):
            if op in OP_BASES or op in OP_DASH:
                bases = op in OP_BASES
                take = max(0, min(ln, slen - start)) if bases else ln
                s, e = max(k, ka), min(k + take, kb)
                if e > s and (bases or not drop):
                    g = gpos + (s - ka)
                    if bases:
                        q = q0 + start + (s - k)
                        runs[o + j] = (g, (e - s) | (bkind << RUN_KSHIFT), q & 0xFFFFFFFF, q >> 32)
                    else:
                        runs[o + j] = (g, (e - s) | ((RUN_DASH | lng) << RUN_KSHIFT), 0, 0)
                k += take
                if bases:
                    start += ln
            elif op == OP_I:
                take = max(0, min(ln, slen - start))
                if fl & PF_INS and take and key0 + k >= roff:
                    syms = tuple(int(CODE_SYM[c]) for c in plane_codes(hb, q0 + start, take))
                    events.append((key0 + k, syms, i) if with_piece else (key0 + k, syms))
                start += ln
            elif op == OP_S:
                start += ln
    return runs, events


def model_counts(hb, runs=None):
    """counts[6][padded_len] of the run records, as the tile kernels form them."""
    if runs is None:
        runs, _ = model_reads(hb)
    Lp = hb.info.padded_len
    counts = np.zeros((NSYM, Lp), dtype=np.int64)
    r = runs.astype(np.int64)
    kind = r[:, 1] >> RUN_KSHIFT
    ln = r[:, 1] & ((1 << RUN_KSHIFT) - 1)
    for sel, is_bases in (((kind & 3) == RUN_BASES, True), ((kind & 3) == RUN_DASH, False)):
        g, n = r[sel, 0], ln[sel]
        if not len(g):
            continue
        off = np.arange(int(n.sum()), dtype=np.int64) - np.repeat(np.cumsum(n) - n, n)
        pos = np.repeat(g, n) + off
        if not is_bases:
            counts[0] += np.bincount(pos, minlength=Lp)
            continue
        q = np.repeat(r[sel, 2] | (r[sel, 3] << 32), n) + off
        w, sh = q >> 5, (q & 31).astype(np.uint32)
        code = ((hb.bx[w] >> sh) & 1).astype(np.int64) << 2 | ((hb.bq[w, 1] >> sh) & 1) << 1 | ((hb.bq[w, 0] >> sh) & 1)
        sym = CODE_SYM[code]
        assert (sym >= 0).all(), "a counted base outside -ACGNT"
        keep = ~((sym == 0) & np.repeat((kind[sel] & RUN_DROP) != 0, n))   # '-' of SEQ dropped (:216)
        np.add.at(counts, (sym[keep], pos[keep]), 1)
    return counts


def check_plan(hb):
    """Pieces bucketed by start word with a matching run-slot CSR; every real position in
    exactly one tile; short pieces within the window, long ones listed for every tile they
    overlap; items / dense lists cover every tile once with its chunk count."""
    i = hb.info
    pc = hb.pc.astype(np.int64)
    NP, K = i.n_pieces, i.kwin
    sw = pc[:NP, 0] >> 5
    assert (np.diff(sw) >= 0).all(), "pieces not bucketed by start word"
    rs = hb.rs.astype(np.int64)
    assert rs[0] == 0 and rs[-1] == i.n_ops and (np.diff(rs) >= 0).all()
    assert (np.diff(pc[:, 2]) >= 0).all() and pc[NP, 2] == i.n_ops
    if NP:
        first = np.searchsorted(sw, np.arange(i.n_words + 1))
        assert (rs == pc[first, 2]).all()
    own = np.zeros(i.padded_len, dtype=np.int64)
    T = hb.tiles.astype(np.int64)
    for t, row in enumerate(T):
        a, b = row[0], row[1]
        assert a % 64 == 0 and 0 < b - a <= 2048
        own[a:b] += 1
        assert (hb.wtile[a >> 5:(b + 31) >> 5] == t).all()
    for r in range(i.n_refs):
        o, L = int(hb.ref_off[r]), int(hb.ref_len[r])
        assert (own[o:o + L] == 1).all(), "ref %d positions not tiled exactly once" % r
    items = {}
    for t, c, l0, l1 in hb.items.astype(np.int64):
        items.setdefault(int(t), []).append((int(c), int(l0), int(l1)))
    for t, c, l0, l1 in hb.dense.astype(np.int64):
        assert int(t) not in items and c == 0 and l0 == 0 and l1 == T[t, 19]
        items[int(t)] = [(0, 0, int(l1))]
        assert T[t, 3] == 4
    # (a ranged snapshot, s2c_parser_snapshot_from, plans tiles [plan_t0, plan_t1) only)
    P0, P1 = int(i.plan_t0), int(i.plan_t1)
    assert 0 <= P0 <= P1 <= i.n_tiles
    assert sorted(items) == list(range(P0, P1))
    for t, cs in items.items():
        cs = sorted(cs)
        assert [c for c, _, _ in cs] == list(range(len(cs)))
        assert cs[0][1] == 0 and cs[-1][2] == T[t, 19] and all(cs[k][2] == cs[k + 1][1] for k in range(len(cs) - 1))
        assert bool(T[t, 3] & 1) == (len(cs) > 1)
    # piece CSR by start word; the sentinel's qh ends the planes
    if NP:
        assert (hb.ps.astype(np.int64) == np.searchsorted(sw, np.arange(i.n_words + 1))).all()
        assert pc[NP, 1] == pc[NP - 1, 1] + (((pc[NP - 1, 3] & 0xFFFFFF) + 15) // 16)
    check_layers(hb)
    lp = hb.lp.astype(np.int64)
    for k in range(NP):
        g, fl = pc[k, 0], pc[k, 3] >> 24
        span = _span(hb, k)
        if span == 0:
            continue
        w0, w1 = g >> 5, (g + span - 1) >> 5
        if fl & PF_LONG:
            for t in range(int(hb.wtile[w0]), int(hb.wtile[w1]) + 1):
                sl = set(lp[T[t, 10]:T[t, 11]].tolist())
                if T[t, 3] & 4:   # a dense tile lists its long pieces (k_tile_dense walks them)
                    assert k in sl
                else:             # the others their run slots (k_reads' records)
                    assert set(range(pc[k, 2], pc[k + 1, 2])) <= sl
        else:
            assert w1 - w0 <= K, "short piece beyond the window"
    assert sorted(hb.deep.tolist()) == [t for t in range(i.n_tiles) if T[t, 3] & 3]
    # window fields: pieces [pf0, pf1) start in words [a/32 - kwin, ceil(b/32)); slots, planes
    for t, row in enumerate(T):
        if not P0 <= t < P1:
            assert row[3] == 0 and row[19] == 0 and (row[13:19] == 0).all()
            continue
        w0, w1 = max((row[0] >> 5) - K, 0), (row[1] + 31) >> 5
        pf0, pf1 = np.searchsorted(sw, [w0, w1])
        assert (row[13], row[14]) == (pf0, pf1) and (row[15], row[16]) == (pc[pf0, 2], pc[pf1, 2])
        if pf1 > pf0:
            assert row[17] == (16 * pc[pf0, 1]) >> 5 and row[18] >= (16 * pc[pf1 - 1, 1] + (pc[pf1 - 1, 3] & 0xFFFFFF) + 31) // 32
        if row[3] == 4:
            ns, nq = row[16] - row[15], row[18] - row[17]
            assert 4 * ((ns + 65) & ~1) + 8 * (nq + 32) + 4 * ((nq + 65) & ~1) + 8 * ns <= S2C_DENSE_LDS and nq <= 4096
    # k_reads' list: the long pieces listed by non-dense tiles (their runs feed those tiles' long
    # lists) and the insertion emitters
    fl = pc[:NP, 3] >> 24
    assert (((fl & 16) != 0) <= ((fl & PF_LONG) != 0)).all()
    by_slot = set()
    for t in range(i.n_tiles):
        if not T[t, 3] & 4:
            for e in range(T[t, 10], T[t, 11]):
                by_slot.add(int(np.searchsorted(pc[:NP, 2], lp[e], side="right")) - 1)
    assert set(np.nonzero((fl & 16) != 0)[0].tolist()) == by_slot
    assert set(hb.rlist.tolist()) == set(np.nonzero(((fl & 16) != 0) | ((fl & PF_INS) != 0))[0].tolist())
    # (ABI 13) rlist's run prefix: what s2c_reads walks when k_tile's walk-queue variant records
    # its finish tiles' short-motif events itself (s2c_host.cpp mark_runs)
    assert bool(i.walk_queue) == (i.n_walked > 0 and 32 * i.n_walked >= i.n_pieces and i.tile_max <= 1024)
    wq = bool(i.tile_events)
    assert wq <= bool(i.walk_queue)
    assert i.n_walked == int((((fl & (PF_SIMPLE | PF_LONG)) == 0)).sum())
    nrr = int(i.n_rlist_run)
    rl = hb.rlist[: i.n_rlist].astype(np.int64)
    ins = set(np.nonzero((fl & PF_INS) != 0)[0].tolist())
    ev_keys = {}
    for g, syms, k in model_reads(hb, with_piece=True)[1]:
        ev_keys.setdefault(k, []).append((g, len(syms)))

    def tile_takes(k):
        if not wq or fl[k] & PF_LONG or k not in ev_keys or max(n for _, n in ev_keys[k]) > 16:
            return False
        g0, g1 = min(g for g, _ in ev_keys[k]), max(g for g, _ in ev_keys[k])
        t0, t1 = int(hb.wtile[g0 >> 5]), int(hb.wtile[g1 >> 5])
        ws = int(pc[k, 0]) >> 5
        for t in range(t0, t1 + 1):
            w0, w1 = int(T[t, 0]) >> 5, (int(T[t, 1]) + 31) >> 5
            if T[t, 3] & 7 or ws < max(w0 - K, 0) or ws >= w1:
                return False
        return True
    want = {k for k in range(NP) if fl[k] & 16} | {k for k in ins if not tile_takes(k)}
    assert set(rl[:nrr].tolist()) == want and set(rl[nrr:].tolist()) == ins - want
    assert len(set(rl.tolist())) == len(rl)


CHUNK_PIECES, CHUNK_QBYTES, CHUNK_OBYTES, CHUNK_RECS = 128, 4096, 1024, 192   # include/s2c.h (per wave)


def chunk_qbytes(nwp, wq):
    """include/s2c.h S2C_CHUNK_QBYTES_OF: a layer's plane bytes in k_tile<nwp, wq> (the
    non-ACGT words: half of it)."""
    return 4352 if nwp <= 16 else CHUNK_QBYTES
LY_MAIN = 0xFFFFFFFF
CHUNK_LANE_RECS, ITEM_RECS = 248, 60000


def layer_ranges(hb, t, nl=None):
    """k_tile's segments of tile t and, per layer l, [lo, hi) of each (s2c_tile.hip table)."""
    i = hb.info
    row = hb.tiles[t].astype(np.int64)
    W0, W1 = row[0] >> 5, (row[1] + 31) >> 5
    S0 = max(W0 - i.kwin, 0)
    ps = hb.ps.astype(np.int64)
    p0 = ps[S0:W1]
    cnt = ps[S0 + 1:W1 + 1] - p0
    nl = int(row[19]) if nl is None else nl
    rot = (np.arange(S0, W1, dtype=np.uint64) * np.uint64(2654435761)) % np.uint64(nl)   # s2c_host.cpp layer_rot
    rot = rot.astype(np.int64)
    return S0, W0, W1, [(p0 + (cnt * l + rot) // nl, p0 + (cnt * (l + 1) + rot) // nl) for l in range(nl)]


def _region(nbytes, phase):
    """LDS bytes of a 16-byte LDS-DMA copy of nbytes starting at source phase `phase`."""
    return (phase + nbytes + 15) & ~15


def check_layers(hb):
    """k_tile's layers: a tile read in place has one layer whose window fits the chunk at its
    arrays' own 16-byte phases; every other tile's layers are exact copies, in start-word
    order, of the short pieces of its proportional per-start-word slices (records, op words,
    the planes of SEQ[0:len]), 16-byte aligned, within the chunk's caps; records per word
    and counting lane; every item's records per word fit its u16 histogram."""
    hb.ensure_layers(dense=True)
    i = hb.info
    pc = hb.pc.astype(np.int64)
    nwp = 8
    while nwp * 32 < i.tile_max:
        nwp *= 2
    G = 64 // nwp   # counting lanes per word of one wave
    qb = chunk_qbytes(nwp, i.walk_queue)   # (the instantiation that runs the layers)
    K = i.kwin
    lly, lpc = hb.lly.astype(np.int64), hb.lpc.astype(np.int64)
    T = hb.tiles.astype(np.int64)
    for t in range(int(i.plan_t0), int(i.plan_t1)):
        row = T[t]
        S0, W0, W1, lays = layer_ranges(hb, t)
        assert W1 - S0 <= 128
        if row[20] == LY_MAIN:
            assert row[19] == 1
            np_, no, nq = row[14] - row[13], row[16] - row[15], row[18] - row[17]
            assert np_ <= CHUNK_PIECES and no <= CHUNK_RECS and _region(4 * no, 4 * (row[15] & 3)) <= CHUNK_OBYTES
            assert _region(8 * nq, 8 * (row[17] & 1)) <= qb and _region(4 * nq, 4 * (row[17] & 3)) <= qb // 2
            rs = hb.rs.astype(np.int64)
            for W in range(W0, W1):
                assert rs[W + 1] - rs[max(W - K, 0)] <= CHUNK_LANE_RECS * G
        else:
            for l, (lo, hi) in enumerate(lays):
                L = row[20] + l
                want = [k for s_lo, s_hi in zip(lo, hi) for k in range(s_lo, s_hi) if not (pc[k, 3] >> 24) & PF_LONG]
                p0, p1 = lly[L, 0], lly[L + 1, 0]
                o0, o1, h0, h1 = lly[L, 1], lly[L + 1, 1], lly[L, 2], lly[L + 1, 2]
                assert p1 - p0 == len(want)
                for j, k in enumerate(want):
                    c = lpc[p0 + j]
                    assert c[0] == pc[k, 0] and c[3] == pc[k, 3]
                    ne = (lpc[p0 + j + 1, 2] if j + 1 < len(want) else o1) - c[2]
                    assert ne == pc[k + 1, 2] - pc[k, 2]
                    assert (hb.lops[c[2]:c[2] + ne] == hb.ops[pc[k, 2]:pc[k + 1, 2]]).all()
                    ln = int(c[3] & 0xFFFFFF)
                    if ln:
                        a = _codes(hb.bq, hb.bx, 16 * int(pc[k, 1]), ln)
                        b = _codes(hb.lbq, hb.lbx, 16 * int(c[1]), ln)
                        assert (a == b).all()
                recs = np.zeros(len(lo), dtype=np.int64)
                for s_i, (s_lo, s_hi) in enumerate(zip(lo, hi)):
                    recs[s_i] = sum(pc[k + 1, 2] - pc[k, 2] for k in range(s_lo, s_hi) if not (pc[k, 3] >> 24) & PF_LONG)
                qa, nq = h0 >> 1, ((h1 + 1) >> 1) + 1 - (h0 >> 1)
                assert p1 - p0 <= CHUNK_PIECES and o1 - o0 == recs.sum() <= CHUNK_RECS
                assert _region(4 * (o1 - o0), 4 * (o0 & 3)) <= CHUNK_OBYTES
                assert _region(8 * nq, 8 * (qa & 1)) <= qb and _region(4 * nq, 4 * (qa & 3)) <= qb // 2
                for W in range(W0, W1):
                    a = max(W - K, S0) - S0
                    assert recs[a:W - S0 + 1].sum() <= CHUNK_LANE_RECS * G
        items = [it for it in hb.items.astype(np.int64) if it[0] == t]
        for _, _, l0, l1 in items:
            lo0, _ = lays[l0]
            _, hi1 = lays[l1 - 1]
            rec = pc[hi1, 2] - pc[lo0, 2]
            for W in range(W0, W1):
                a = max(W - K, S0) - S0
                assert rec[a:W - S0 + 1].sum() <= ITEM_RECS


def _codes(bq, bx, q, n):
    idx = np.arange(q, q + n, dtype=np.int64)
    w, sh = idx >> 5, (idx & 31).astype(np.uint32)
    return ((bx[w] >> sh) & 1) << 2 | ((bq[w, 1] >> sh) & 1) << 1 | ((bq[w, 0] >> sh) & 1)


def check_plan_shard(sub):
    """A shard's sub-batch: pieces bucketed, run-slot CSR consistent, its tiles mapped."""
    i = sub.info
    pc = sub.pc.astype(np.int64)
    sw = pc[:i.n_pieces, 0] >> 5
    assert (np.diff(sw) >= 0).all()
    rs = sub.rs.astype(np.int64)
    assert rs[0] == 0 and rs[-1] == i.n_ops
    T = sub.tiles.astype(np.int64)
    for t, row in enumerate(T):
        assert (sub.wtile[row[0] >> 5:(row[1] + 31) >> 5] == t).all()
    n = len(hb_items(sub))
    assert n == i.n_tiles + int(sum(max(0, c) for c in []))
    check_layers(sub)


def hb_items(hb):
    return sorted(set(hb.items[:, 0].tolist()) | set(hb.dense[:, 0].tolist()))


def _span(hb, k):
    """Seqout span of piece k (from its RANGE prefix or its tokens)."""
    pc, ops = hb.pc, hb.ops
    o, oend, w3 = int(pc[k, 2]), int(pc[k + 1, 2]), int(pc[k, 3])
    fl, slen = w3 >> 24, w3 & 0xFFFFFF
    if fl & PF_RANGE:
        return int(ops[o + 1]) - int(ops[o])
    o += 3 if fl & PF_INS else 0
    n = start = 0
    for w in ops[o:oend]:
        op, ln = int(w) & 15, int(w) >> 4
        if op in OP_BASES:
            n += max(0, min(ln, slen - start))
            start += ln
        elif op in OP_DASH:
            n += ln
        elif op in (OP_I, OP_S):
            start += ln
    return n


def _vote(c, cov, t):
    amb = _amb()
    m = 0
    for i in range(NSYM):
        if c[i] != 0 and float(sum(x for x in c if x > c[i])) < t * float(cov):
            m |= 1 << i
    ch = amb[m]
    return 0xFF if ch is None else ch


def model_columns(events):
    """{gkey: [6-count column, ...]} (:262-287), motifs aggregated per (key, motif)."""
    motifs = {}
    for key, syms in events:
        d = motifs.setdefault(key, {})
        d[syms] = d.get(syms, 0) + 1
    cols = {}
    for key, d in motifs.items():
        cl = [[0] * NSYM for _ in range(max(len(m) for m in d))]
        for m, mult in d.items():
            for c, s in enumerate(m):
                cl[c][s] += mult
        cols[key] = cl
    return cols


def model_pipeline(hb, thresholds, min_depth=1, fill=b"-", maxdel_active=None, counts_add=None):
    """(stats[R,T,4], offs[T*nb+1], out bytes) as the device produces them; ``counts_add``:
    running totals of earlier streamed batches added to this batch's counts."""
    runs, events = model_reads(hb, maxdel_active)
    counts = model_counts(hb, runs)
    if counts_add is not None:
        counts = counts + counts_add
    cols = model_columns(events)
    T = len(thresholds)
    cov = counts.sum(axis=0)
    nb = hb.info.n_tiles
    R = hb.info.n_refs
    stats = np.zeros((R, T, 4), dtype=np.uint64)
    blk_len = np.zeros(T * nb + 1, dtype=np.int64)
    pieces = [[None] * nb for _ in range(T)]
    fl = len(fill)
    fnd = sum(1 for ch in fill if ch != ord("-"))
    for bi, (g0, g1, ref) in enumerate(hb.tiles[:, :3]):
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
