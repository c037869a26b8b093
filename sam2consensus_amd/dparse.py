"""Parse once across ranks: the multi-GPU CLI's distributed read pass (SURVEY.md §8 e).

The reference reads the whole SAM on one core (sam2consensus.py:147-228).  With one
process per GPU, every rank parsing the whole file would make the parse N times the work
and leave the host side unscaled.  Here the file is cut into blocks of whole lines
(``BLOCK`` bytes; block k is parsed by rank k mod N, each with its own parser fed the
header first), and

1. every rank parses its blocks (``s2c_parser_feed``: large blocks parse on all threads)
   and reports per block its line counters, its first read-pass error, a histogram of read
   starts over 256-position bins and the per-reference insertion-check flags (:284-294);
2. one all-reduce combines them: the first failing block in file order gives the
   reference's first error (a block's parser stops at its first failing line, as the
   reference does); the insertion checks then raise in reference order, as
   ``s2c_parser_finish`` does for one batch; otherwise the histogram cuts the fixed-width
   tile list (``s2c_parser_set_tile_width``: the same tiles on every rank, from the header
   alone) into N contiguous ranges of about equal work;
3. each rank packs, per destination, the reads of its blocks that can change a position in
   that rank's range (``s2c_parser_pack``: the streamed retain's extent test — counted
   range, POS <= 0 wrap, emitted insertion keys) and one ``all_to_all`` moves them;
4. each rank unpacks what it received in block order (file order) into one parser, plans
   the batch (``s2c_parser_finish``) and cuts its tile range (``s2c_batch_shard``).

A position's counts depend only on the reads that can change it, and every such read
reaches the rank owning the position, so each rank's tiles are the whole-file tiles —
the streamed path's argument.  Every line is parsed once, by one rank.  The exchange is a
real data-path step (reads near range ends go to two ranks); on GPUs it runs over RCCL.
"""
from __future__ import annotations

import ctypes as C
import gzip

import numpy as np

from . import _lib as L
from .batch import HostBatch, Parser

BLOCK = 64 << 20          # bytes of SAM text per block
NO_BLOCK = 1 << 56        # "no failing block" (block keys: below 2^48)
BIN_SHIFT = 8             # read-start histogram bins of 256 positions
DENSE_DEPTH = 48.0        # at or below this mean depth: 1024-position dense tiles
E_TARGET = 262144.0       # aligned bases per deep tile (the planner's, s2c_host.cpp)


class BlockParser(Parser):
    """``Parser`` with the distributed-parse entry points (include/s2c.h)."""

    def pos_weights(self, n):
        w = np.zeros(max(n, 1), np.int64)
        L.check(L.lib.s2c_parser_pos_weights(self._p, BIN_SHIFT, w.ctypes.data_as(C.POINTER(C.c_int64)), n))
        return w[:n]

    def checks(self, n_refs):
        b = np.zeros(max(2 * n_refs, 1), np.uint8)
        L.check(L.lib.s2c_parser_checks(self._p, b.ctypes.data_as(C.POINTER(C.c_uint8)), n_refs))
        return b[:2 * n_refs]

    def counters(self):
        c = (C.c_int64 * 4)()
        L.check(L.lib.s2c_parser_counters(self._p, c))
        return list(c)

    def pack(self, g0, g1):
        n = C.c_size_t()
        L.check(L.lib.s2c_parser_pack(self._p, int(g0), int(g1), C.byref(n)))
        out = np.empty(n.value, np.uint8)
        L.check(L.lib.s2c_parser_blob_copy(self._p, out.ctypes.data_as(C.c_void_p), n.value))
        return out

    def unpack(self, blob):
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        L.check(L.lib.s2c_parser_unpack(self._p, blob.ctypes.data_as(C.c_void_p), blob.size))

    def set_tile_width(self, w):
        L.check(L.lib.s2c_parser_set_tile_width(self._p, int(w)))

    def feed_header(self, header):
        """The file's header lines, then the end of the header: a block from the middle of the
        file may start with an '@' line, which the read pass skips (:195) as a body line."""
        self.feed(header)
        L.check(L.lib.s2c_parser_end_header(self._p))


def split_header(head: bytes):
    """(header bytes, offset of the first record line) of a file's leading bytes; the header
    is every line up to the first one not starting with '@' (:149-158).  None if ``head``
    ends inside the header."""
    pos = 0
    while pos < len(head):
        if head[pos:pos + 1] != b"@":
            return head[:pos], pos
        nl = head.find(b"\n", pos)
        if nl < 0:
            return None
        pos = nl + 1
    return None


def _read_header(fh):
    head = b""
    while True:
        more = fh.read(1 << 20)
        head += more
        r = split_header(head)
        if r is not None:
            return r
        if not more:
            return head, len(head)


def plain_blocks(filename, rank, world, block=BLOCK):
    """(header, [(k, bytes)]) for the blocks k ≡ rank (mod world) of an uncompressed file:
    block k starts at the first line start at or after H + k·block."""
    import os
    size = os.path.getsize(filename)
    with open(filename, "rb") as fh:
        header, H = _read_header(fh)
        nb = -(-(size - H) // block) if size > H else 0

        def start(k):
            if k <= 0:
                return H
            nom = H + k * block
            if nom >= size:
                return size
            fh.seek(nom - 1)
            s = nom - 1
            while True:
                buf = fh.read(1 << 16)
                if not buf:
                    return size
                i = buf.find(b"\n")
                if i >= 0:
                    return s + i + 1
                s += len(buf)

        out = []
        for k in range(rank, nb, world):
            a, b = start(k), start(k + 1)
            fh.seek(a)
            out.append((k, fh.read(b - a)))
    return header, out


def gz_blocks(filename, rank, world, block=BLOCK):
    """The same for a gzip file (:111-114): every rank inflates the stream (gzip has no
    random access) and keeps its blocks, cut at line ends."""
    out = []
    with gzip.open(filename, "rb") as fh:
        header, H = _read_header(fh)
        fh.seek(H)
        k, carry = 0, b""
        while True:
            buf = fh.read(block)
            data = carry + buf
            if not buf:
                if data:
                    if k % world == rank:
                        out.append((k, data))
                break
            cut = data.rfind(b"\n") + 1
            if cut == 0:
                carry = data
                continue
            if k % world == rank:
                out.append((k, data[:cut]))
            carry = data[cut:]
            k += 1
    return header, out


def text_blocks(rest, block=BLOCK):
    """In-memory SAM text (after the header) cut into blocks of whole lines."""
    out, s = [], 0
    while s < len(rest):
        e = min(len(rest), s + block)
        if e < len(rest):
            nl = rest.find(b"\n", e - 1)
            e = len(rest) if nl < 0 else nl + 1
        out.append(rest[s:e])
        s = e
    return out


def bgzf_index(mm):
    """[(offset, size)] of the BGZF blocks (members with the 'BC' size field) of a mapped
    .gz file, or None if any member is not one."""
    idx, off, n = [], 0, len(mm)
    while off < n:
        if n - off < 18 or mm[off:off + 4] != b"\x1f\x8b\x08\x04":
            return None
        xlen = mm[off + 10] | (mm[off + 11] << 8)
        k, size = off + 12, 0
        while k + 4 <= off + 12 + xlen:
            sl = mm[k + 2] | (mm[k + 3] << 8)
            if mm[k:k + 2] == b"BC" and sl == 2:
                size = (mm[k + 4] | (mm[k + 5] << 8)) + 1
            k += 4 + sl
        if size < 12 + xlen + 8 or off + size > n:
            return None
        idx.append((off, size))
        off += size
    return idx


def _inflate(mm, blocks):
    """The blocks' text; each checked against its CRC32 and ISIZE trailer as gzip does
    (the reference reads with gzip.open, :111).  A mismatch raises IOError."""
    import struct
    import zlib
    out = []
    for off, size in blocks:
        xlen = mm[off + 10] | (mm[off + 11] << 8)
        data = zlib.decompress(mm[off + 12 + xlen:off + size - 8], -15)
        crc, isize = struct.unpack("<II", mm[off + size - 8:off + size])
        if zlib.crc32(data) != crc or len(data) & 0xFFFFFFFF != isize:
            raise IOError("CRC check failed in BGZF block at byte %d" % off)
        out.append(data)
    return b"".join(out)


def bgzf_text(filename, rank, world, group=None):
    """A BGZF .sam.gz cut over the ranks by compressed bytes: rank r inflates only its blocks
    (the header from the file's first blocks), and the lines cut by a range end are
    completed with the next ranks' leading bytes (an all-gather of the small head pieces).
    Returns (header, this rank's whole lines after the header), or None when the file is
    not BGZF or a line would span a rank's whole range (then every rank inflates the stream)."""
    import mmap

    import torch.distributed as dist
    with open(filename, "rb") as fh:
        mm = mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ)
        try:
            idx = bgzf_index(mm)
            ok = idx is not None and len(idx) > 0
            flags = [None] * world
            dist.all_gather_object(flags, ok, group=group)
            if not all(flags):
                return None
            C = idx[-1][0] + idx[-1][1]
            mine = [b for b in idx if rank * C // world <= b[0] < (rank + 1) * C // world]
            bad = ""
            try:
                text = _inflate(mm, mine)
                head = b""
                for k in range(0, len(idx), 64):   # the header: the file's first blocks until a record line
                    head += _inflate(mm, idx[k:k + 64])
                    if split_header(head) is not None:
                        break
            except (IOError, OSError, __import__("zlib").error) as e:
                bad = str(e) or "corrupt BGZF block"
            errs = [None] * world   # a corrupt block fails every rank alike (no rank left waiting)
            dist.all_gather_object(errs, bad, group=group)
            if any(errs):
                raise IOError(next(e for e in errs if e))
        finally:
            mm.close()
    header, H = split_header(head) or (head, len(head))
    # my range's bytes of the file's text: [text_start, text_start + len(text)); the records
    # start at H.  Head piece: my bytes up to and including my first '\n' (all of them if none).
    lens = [None] * world
    dist.all_gather_object(lens, len(text), group=group)
    start = sum(lens[:rank])
    lo = max(0, H - start)                      # header bytes in my range
    nl = text.find(b"\n", lo)
    headpiece = text[lo:nl + 1] if nl >= 0 else text[lo:]
    pieces = [None] * world
    dist.all_gather_object(pieces, (headpiece, nl >= 0, start + len(text) <= H), group=group)
    # a rank without a newline past the header would leave a line spanning its range
    if any(not p[1] and not p[2] and lens[r] > 0 for r, p in enumerate(pieces)):
        return None
    body = text[lo:]
    ends_nl = [None] * world
    mine_end = body.endswith(b"\n") or not body
    dist.all_gather_object(ends_nl, mine_end, group=group)
    # my leading piece belongs to the previous rank holding bytes unless that one ended a line
    prev = [r for r in range(rank) if lens[r] > 0 and not pieces[r][2]]
    if prev and not ends_nl[prev[-1]]:
        body = body[len(headpiece):]
    if not mine_end:   # complete my last line from the next ranks' head pieces
        for r in range(rank + 1, world):
            if lens[r] == 0 or pieces[r][2]:
                continue
            body += pieces[r][0]
            if pieces[r][1]:
                break
    return header, body


def file_blocks(filename, rank, world, block=BLOCK, group=None):
    if filename.endswith(".gz"):
        r = bgzf_text(filename, rank, world, group)
        if r is not None:   # block keys: rank << 32 | block of this rank's range (file order)
            header, body = r
            return header, [((rank << 32) | k, b) for k, b in enumerate(text_blocks(body, block))]
        return gz_blocks(filename, rank, world, block)
    return plain_blocks(filename, rank, world, block)


def tile_width_for(depth):
    """Fixed tile width from the mean depth, as the planner chooses (s2c_host.cpp tiles)."""
    if depth <= DENSE_DEPTH:
        return 1024
    w = int(np.ceil(E_TARGET / depth))
    w = (w + 63) // 64 * 64
    return int(min(max(w, 256), 2048))


def split_ranges(tiles, weights, world):
    """Contiguous tile ranges [(t0, t1)] of about equal work: a tile's weight is the read
    starts in its bins plus a vote term per 32 positions (shard.tile_weights' shape)."""
    nt = len(tiles)
    if world <= 1 or nt == 0:
        return [(0, nt)] + [(nt, nt)] * max(0, world - 1)
    a = tiles[:, 0].astype(np.int64)
    b = tiles[:, 1].astype(np.int64)
    c = np.concatenate([[0], np.cumsum(weights)])
    bins = len(weights)
    wa = c[np.minimum(a >> BIN_SHIFT, bins)]
    wb = c[np.minimum(b >> BIN_SHIFT, bins)]
    tw = (wb - wa).astype(np.float64) + (b - a) / 32.0
    cw = np.cumsum(tw)
    cuts = [0] + [int(np.searchsorted(cw, cw[-1] * k / world)) for k in range(1, world)] + [nt]
    for k in range(1, len(cuts)):
        cuts[k] = min(max(cuts[k], cuts[k - 1]), nt)
    return [(cuts[k], cuts[k + 1]) for k in range(world)]


class Parsed:
    """What a rank holds after the distributed parse."""

    def __init__(self, hb, sub, counters, ref_flags, ranges):
        self.hb = hb                  # this rank's whole-tile-list batch (its range populated)
        self.sub = sub                # its sub-batch of tiles [t0, t1) (.t0, .t1)
        self.header_lines, self.lines_total, self.reads_mapped, self.aligned_bases = counters
        self.ref_flags = ref_flags    # Σcoverage > 0 per reference over all ranks (:334-341)
        self.ranges = ranges          # every rank's tile range


def _allreduce(x, op, dev, dist, group):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    dist.all_reduce(t, op=op, group=group)
    return t.cpu().numpy()


def parse_distributed(filename, rank, world, maxdel_active=True, group=None, block=BLOCK, text=None):
    """The distributed read pass (module docstring) → ``Parsed``.  Raises the reference's
    exception class on every rank for a failing input.  ``text`` parses in-memory SAM
    bytes instead of a file (tests)."""
    import torch
    import torch.distributed as dist

    from .shard import _tensor_device
    dev = _tensor_device(group)
    if text is not None:
        header, H = split_header(text) or (text, len(text))
        blocks = [(k, b) for k, b in enumerate(text_blocks(text[H:], block)) if k % world == rank]
    else:
        header, blocks = file_blocks(filename, rank, world, block, group)

    # the reference table and the fixed-width tile list come from the header alone
    hp = BlockParser(maxdel_active, 150)
    hp.feed(header)
    hb0 = hp.finish()
    R, padded = int(hb0.info.n_refs), int(hb0.info.padded_len)
    total_len = int(hb0.info.total_len)
    hdr_lines = int(hb0.info.header_lines)
    hb0.free()
    hp.close()
    nbins = (padded >> BIN_SHIFT) + 1

    # 1. parse my blocks
    parsers, first_err, err_code = [], NO_BLOCK, 0
    weights = np.zeros(nbins, np.int64)
    bad = np.zeros(max(2 * R, 1), np.uint8)
    cnt = np.zeros(3, np.int64)   # body lines, mapped reads, aligned bases
    for k, data in blocks:
        p = BlockParser(maxdel_active, 150)
        try:
            p.feed_header(header)
            p.feed(data)
            c = p.counters()
        except Exception as e:  # noqa: BLE001 - re-raised on every rank below
            p.close()
            if k < first_err:
                first_err, err_code = k, _code(e)
            continue
        cnt += np.array([c[1] - c[0], c[2], c[3]], np.int64)
        weights += p.pos_weights(nbins)
        bad[:2 * R] |= p.checks(R)
        parsers.append((k, p))

    # 2. combine: errors, counters, work histogram, insertion checks
    err = _allreduce(np.array([first_err * 8 + err_code], np.int64), dist.ReduceOp.MIN, dev, dist, group)[0]
    if err < NO_BLOCK * 8:
        for _, p in parsers:
            p.close()
        raise _exc(int(err % 8))("read-pass error in block %d (first in file order)" % (err // 8))
    cnt = _allreduce(cnt, dist.ReduceOp.SUM, dev, dist, group)
    weights = _allreduce(weights, dist.ReduceOp.SUM, dev, dist, group)
    bad = _allreduce(bad.astype(np.int32), dist.ReduceOp.MAX, dev, dist, group)
    for r in range(R):   # s2c_parser_finish's order: motif symbols, then keys, per reference
        if bad[2 * r] or bad[2 * r + 1]:
            for _, p in parsers:
                p.close()
            if bad[2 * r]:
                raise KeyError("insertion base not in -ACGNT (:287)")
            raise IndexError("insertion key out of range (:294)")
    depth = float(cnt[2]) / float(total_len) if total_len else 0.0
    W = tile_width_for(depth)
    tp = BlockParser(maxdel_active, 150)
    tp.set_tile_width(W)
    tp.feed(header)
    hbt = tp.finish()
    tiles = hbt.tiles[:, :2].astype(np.int64).copy()
    hbt.free()
    tp.close()
    ranges = split_ranges(tiles, weights, world)

    def grange(t0, t1):
        return (int(tiles[t0, 0]), int(tiles[t1 - 1, 1])) if t1 > t0 else (0, 0)

    # 3. route: per destination, a directory {block, size} and the blobs of my blocks
    send = []
    for d in range(world):
        g0, g1 = grange(*ranges[d])
        parts = [(k, p.pack(g0, g1)) for k, p in parsers] if g1 > g0 else []
        dirn = np.array([len(parts)] + [v for k, b in parts for v in (k, b.size)], np.int64)
        send.append(np.concatenate([dirn.view(np.uint8)] + [b for _, b in parts]))
    for _, p in parsers:
        p.close()
    out_sizes = _alltoall_sizes([s.size for s in send], dev, dist, group, world)
    recv = _alltoall_bytes(send, out_sizes, dev, dist, group)

    # 4. my reads, in block order, into one parser; plan; cut my tile range
    got = []
    for buf in recv:
        n = int(buf[:8].view(np.int64)[0])
        meta = buf[8:8 + 16 * n].view(np.int64).reshape(-1, 2)
        o = 8 + 16 * n
        for k, sz in meta:
            got.append((int(k), buf[o:o + int(sz)]))
            o += int(sz)
    got.sort(key=lambda x: x[0])
    mp = BlockParser(maxdel_active, 150)
    mp.set_tile_width(W)
    mp.feed(header)
    for _, b in got:
        mp.unpack(b)
    hb = mp.finish()
    mp.close()
    hb.maxdel_active, hb.maxdel = bool(maxdel_active), 150
    t0, t1 = ranges[rank]
    h = C.c_void_p()
    L.check(L.lib.s2c_batch_shard(hb._b, t0, t1, C.byref(h)))
    sub = HostBatch(h)
    sub.t0, sub.t1 = t0, t1
    sub.parent_tiles = hb.info.n_tiles
    sub.maxdel_active, sub.maxdel = hb.maxdel_active, hb.maxdel
    flags = _allreduce((hb.ref_reads > 0).astype(np.int32), dist.ReduceOp.MAX, dev, dist, group)
    counters = (hdr_lines, hdr_lines + int(cnt[0]), int(cnt[1]), int(cnt[2]))
    return Parsed(hb, sub, counters, flags.astype(np.int64), ranges)


_CODES = {KeyError: 1, IndexError: 2, ValueError: 3, ZeroDivisionError: 4, OverflowError: 5}


def _code(e):
    for cls, c in _CODES.items():
        if isinstance(e, cls):
            return c
    return 7   # an engine error (S2CError: limits, I/O)


def _exc(c):
    return {v: k for k, v in _CODES.items()}.get(c, RuntimeError)


def _alltoall_sizes(sizes, dev, dist, group, world):
    import torch

    from .shard import force_collectives
    if world == 1 and not force_collectives():
        return list(sizes)
    s = torch.tensor(sizes, dtype=torch.int64, device=dev)
    o = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(o, s, group=group)
    return o.cpu().tolist()


def _alltoall_bytes(send, out_sizes, dev, dist, group):
    import torch
    from .shard import force_collectives
    world = len(send)
    if world == 1 and not force_collectives():
        return [send[0]]
    src = torch.from_numpy(np.concatenate(send)).to(dev)
    dst = torch.empty(int(sum(out_sizes)), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(dst, src, out_sizes, [int(s.size) for s in send], group=group)
    d = dst.cpu().numpy()
    offs = np.concatenate([[0], np.cumsum(out_sizes)])
    return [d[offs[i]:offs[i + 1]] for i in range(world)]
