"""Streamed batches: coordinate-sorted SAM input in bounded host memory.

The reference reads the whole file into per-reference lists before any consensus work
(sam2consensus.py:185-228); the whole-batch path here does the same with a packed batch.
For a coordinate-sorted file (SO:coordinate — what aligners emit after ``samtools sort``)
the positions a later read can change all lie at or after the last read's POS, so the
tiles that end before it are final.  The driver

1. feeds the file in blocks (``s2c_parser_feed``; large blocks parse in parallel pieces),
2. every ``batch_bytes`` of input takes a snapshot batch of the reads held
   (``s2c_parser_snapshot``, tile width fixed so every snapshot has the same tiles),
3. runs the tiles [t_done, t1) that end at or before the last read's position — the same
   ``s2c_batch_shard`` sub-batch the multi-GPU path runs (sam2consensus_amd/shard.py) —
4. keeps only the reads that reach tile t1 or later (``s2c_parser_retain``),

and at end of input runs the remaining tiles, merges the tile ranges' bodies and stats
(``shard.merge_outputs``) and formats the records as the whole-batch path does.  The
bytes are the reference's: a position's counts, insertion columns and vote depend only on
the reads that reach it, and each tile runs once with all of them.

Errors keep the reference's precedence: a read-pass error (:195-218) raises when its block
is fed; an insertion-check error (:284-294) seen in a snapshot stops the streaming and is
raised by the final ``s2c_parser_finish`` (which sees every read of the failing reference
and every later one, and no read pass error can follow it unseen); vote errors raise from
``build_records`` over the merged stats.

Input that is not coordinate-sorted is detected (a read parsed after a retain reaching
below it) and ``stream_batches`` raises ``NotSorted``; ``consensus_files_streamed`` then
re-reads the file with ``stream_unsorted``: each batch's counts are added into running
totals counts[6][padded_len] in HBM (``s2c_accumulate``) and its reads dropped except their
insertion events, which the last batch holds all of and votes every tile over the totals.
Host memory is then bounded by one batch plus the reads with insertions, as the
reference's is by its count tables (:206-221).
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np

from . import _lib as L
from .batch import HostBatch, Parser

DEFAULT_TILE = 1024               # positions per tile (C5's planner choice at 30x)
DEFAULT_BATCH = 256 << 20         # input bytes per streamed batch
BLOCK = 64 << 20                  # bytes per feed call (a 64 MB block parses on 16 host threads, ≥ 4 MB each)


def _env_bytes(name, default):
    """<bytes>[K|M|G] from the environment variable ``name`` (unset or empty: ``default``)."""
    v = os.environ.get(name, "").strip().upper()
    if not v:
        return default
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}.get(v[-1], 1)
    return int(float(v.rstrip("KMG")) * mult)


BLOCK = _env_bytes("S2C_STREAM_BLOCK", BLOCK)   # (measurement knob: the feed call's size)


class NotSorted(Exception):
    """A read changes positions already emitted: the input is not coordinate-sorted."""


class StreamParser(Parser):
    """``Parser`` with the streamed-batch entry points (include/s2c.h)."""

    def __init__(self, maxdel_active=True, maxdel=150, tile_width=DEFAULT_TILE):
        super().__init__(maxdel_active, maxdel)
        L.check(L.lib.s2c_parser_set_tile_width(self._p, int(tile_width)))

    def _wrap(self, h):
        hb = HostBatch(h)
        hb.maxdel_active, hb.maxdel = self.maxdel_active, self.maxdel
        return hb

    def snapshot(self, t_from=None) -> HostBatch:
        """The batch of the reads held; with ``t_from`` only tiles t_from .. the tile of the
        reads' last position are planned (``s2c_parser_snapshot_from``: info.plan_t0 / plan_t1)."""
        h = C.c_void_p()
        if t_from is None:
            L.check(L.lib.s2c_parser_snapshot(self._p, C.byref(h)))
        else:
            L.check(L.lib.s2c_parser_snapshot_from(self._p, int(t_from), C.byref(h)))
        return self._wrap(h)

    def retain(self, gmin):
        L.check(L.lib.s2c_parser_retain(self._p, int(gmin)))

    def retain_events(self):
        L.check(L.lib.s2c_parser_retain_events(self._p))

    def state(self):
        """(late, last reference index, last POS-1, reads held)."""
        s = (C.c_int64 * 4)()
        L.check(L.lib.s2c_parser_stream_state(self._p, s))
        return bool(s[0]), int(s[1]), int(s[2]), int(s[3])

    def detach(self) -> "StreamParser":
        """The reads held move to a new parser (s2c_parser_detach): it can be snapshot and
        retained on another thread while this one goes on feeding; ``attach`` it back."""
        d = StreamParser.__new__(StreamParser)
        d.maxdel_active, d.maxdel = self.maxdel_active, self.maxdel
        d._p = C.c_void_p()
        L.check(L.lib.s2c_parser_detach(self._p, C.byref(d._p)))
        return d

    def attach(self, d: "StreamParser"):
        """Put ``d``'s reads back in front of the ones fed since (``d`` is consumed)."""
        h, d._p = d._p, C.c_void_p()
        L.check(L.lib.s2c_parser_attach(self._p, h))


def _sub(hb, t0, t1):
    h = C.c_void_p()
    L.check(L.lib.s2c_batch_shard(hb._b, t0, t1, C.byref(h)))
    sub = HostBatch(h)
    sub.t0, sub.t1 = t0, t1
    sub.parent_tiles = hb.info.n_tiles
    sub.maxdel_active, sub.maxdel = hb.maxdel_active, hb.maxdel
    return sub


class StreamResult:
    """What ``stream_batches`` hands back: the final batch (tile plan, names, per-reference
    coverage flags over all batches), the merged (stats, offs, out) and the line counters."""

    def __init__(self, hb, stats, offs, out, header_lines, lines_total, reads_mapped, batches, held_max):
        self.hb, self.stats, self.offs, self.out = hb, stats, offs, out
        self.header_lines, self.lines_total, self.reads_mapped = header_lines, lines_total, reads_mapped
        self.n_refs = hb.info.n_refs
        self.batches = batches        # tile ranges run
        self.held_max = held_max      # most reads the parser held at a snapshot


_END = object()


class _Producer:
    """The parser side of a streamed run on its own host thread: it feeds the blocks, takes
    the snapshots, cuts the sub-batches and retains, handing each item to the consumer (the
    device side, on the calling thread) through a bounded queue — so parsing batch k + 1
    overlaps batch k's upload, kernels and fetch.  libs2c.so's calls release the GIL (ctypes).
    An exception ends the thread and is re-raised by the consumer in order."""

    def __init__(self, gen, depth=2):
        import queue
        import threading
        self.q = queue.Queue(maxsize=depth)
        self.stop = threading.Event()
        self.t = threading.Thread(target=self._run, args=(gen,), daemon=True)
        self.t.start()

    def _put(self, item):
        import queue
        while not self.stop.is_set():
            try:
                self.q.put(item, timeout=0.1)
                return True
            except queue.Full:
                continue
        return False

    def _run(self, gen):
        try:
            for item in gen:
                if not self._put(("item", item)):
                    gen.close()
                    return
            self._put(("end", None))
        except BaseException as e:  # noqa: BLE001 - re-raised on the consumer thread
            self._put(("error", e))

    def __iter__(self):
        try:
            while True:
                kind, v = self.q.get()
                if kind == "end":
                    return
                if kind == "error":
                    raise v
                yield v
        finally:
            self.stop.set()
            self.t.join()


def _sorted_items(blocks, maxdel_active, tile_width, batch_bytes, stats_hook, state, ranged=False):
    """Generator (producer thread) of the streamed run of sorted input: ("run", sub, t0, t1)
    for every final tile range — a cut sub-batch, or with ``ranged`` the snapshot itself
    (the device side runs its tiles [t0, t1)) — then ("last", hb) with the final batch.

    Pipelined (the default; S2C_STREAM_PIPE=0 turns it off): at each batch the reads held
    are detached into a parser of their own, whose snapshot, cut and retain run on a helper
    thread while this one goes on reading and feeding the next blocks; the retained reads
    are attached back in front of the new ones before the next batch is detached.  So the
    producer's time per batch is max(read + feed, snapshot + cut + retain), not their sum."""
    p = StreamParser(maxdel_active, 150, tile_width)
    t_done, pending, broken = 0, 0, False
    tm = state.setdefault("t", {})
    clk = time.perf_counter
    pipe = os.environ.get("S2C_STREAM_PIPE", "1").strip() != "0"

    def add(k, t0):
        tm[k] = tm.get(k, 0.0) + clk() - t0

    def stage(q, t_lo):
        """Snapshot / cut / retain of the reads ``q`` holds: ("broken",), ("skip", held) or
        ("run", sub, t_lo, t1, NT, held)."""
        try:
            t0 = clk()
            hb = q.snapshot(t_lo)    # (planned from t_lo: tiles before it ran with an earlier batch)
            add("snapshot", t0)
        except (KeyError, IndexError):
            return ("broken",)       # s2c_parser_finish raises it once the input is read
        try:
            late, ref, pos0, held = q.state()
            if late:
                raise NotSorted("a read reaches positions already emitted")
            if ref < 0:
                return ("skip", held)
            # every later read changes positions >= this bound only: POS clamped to the
            # reference's last position as the host plan clamps it (a read with no aligned
            # span may carry a POS past LN, and counts nothing there)
            bound = int(hb.ref_off[ref]) + min(max(pos0, 0), max(int(hb.ref_len[ref]) - 1, 0))
            NT = int(hb.info.n_tiles)
            t1 = int(np.searchsorted(hb.tiles[:, 1].astype(np.int64), bound, side="right"))
            if t1 > int(hb.info.plan_t1) and t1 > t_lo:   # (never with the clamp; a tile without a plan
                raise NotSorted("the batch's bound lies past its snapshot's plan")   # must not run: accumulate)
            if t1 <= t_lo:
                return ("skip", held)
            gmin = int(hb.tiles[t1, 0]) if t1 < NT else int(hb.info.padded_len)
            t0 = clk()
            state["absorb"](hb)
            add("absorb", t0)
            t0 = clk()
            if ranged:                # the device runs the snapshot's tiles [t_lo, t1) itself
                sub, hb = hb, None
                sub.t0_range = t_lo
            else:
                sub = _sub(hb, t_lo, t1)
            add("cut", t0)
            t0 = clk()
            q.retain(gmin)
            add("retain", t0)
            return ("run", sub, t_lo, t1, NT, held)
        finally:
            if hb is not None:
                hb.free()

    ex = None
    if pipe:
        from concurrent.futures import ThreadPoolExecutor
        ex = ThreadPoolExecutor(max_workers=1, thread_name_prefix="s2c-stage")
    run = None                       # (future, detached parser) of the stage in flight

    def join():
        """Wait for the stage in flight and attach its parser back; its outcome."""
        nonlocal run
        f, d = run
        run = None
        t0 = clk()
        try:
            return f.result()
        finally:
            p.attach(d)
            add("join", t0)

    def outcome(o):
        """The item to yield for a stage's outcome (None: nothing to run)."""
        nonlocal broken, t_done
        if o[0] == "broken":
            broken = True
            return None
        state["held_max"] = max(state["held_max"], o[-1])
        if o[0] == "skip":
            return None
        _, sub, t_lo, t1, NT, held = o
        t_done = t1
        if stats_hook:
            stats_hook(t_done, NT, held)
        return ("run", sub, t_lo, t1)

    try:
        it = iter(blocks)
        while True:
            t0 = clk()
            blk = next(it, None)   # (the input's next block: file read / inflate)
            add("read", t0)
            if blk is None:
                break
            t0 = clk()
            p.feed(blk)
            add("feed", t0)
            pending += len(blk)
            if run is not None and (run[0].done() or (not broken and pending >= batch_bytes)):
                item = outcome(join())
                if item is not None:
                    yield item
            if broken or pending < batch_bytes:
                continue
            pending = 0
            if ex is None:
                item = outcome(stage(p, t_done))
                if item is not None:
                    yield item
                continue
            d = p.detach()
            run = (ex.submit(stage, d, t_done), d)
        if run is not None:
            item = outcome(join())
            if item is not None:
                yield item
        t0 = clk()
        hb = p.finish()
        add("finish", t0)
        late, _, _, held = p.state()
        state["held_max"] = max(state["held_max"], held)
        if late:
            hb.free()
            raise NotSorted("a read reaches positions already emitted")
        NT = int(hb.info.n_tiles)
        state["absorb"](hb)
        if t_done < NT:
            yield ("run", _sub(hb, t_done, NT), t_done, NT)
        yield ("last", hb)
    finally:
        if run is not None:          # (closed or raised with a stage in flight)
            f, d = run
            try:
                o = f.result()
                if o[0] == "run":
                    o[1].free()
            except BaseException:  # noqa: BLE001 - the first error is the one raised
                pass
            d.close()
        if ex is not None:
            ex.shutdown(wait=True)
        p.close()


def stream_batches(blocks, thresholds, runner, maxdel_active=True, tile_width=DEFAULT_TILE,
                   batch_bytes=DEFAULT_BATCH, stats_hook=None):
    """Run ``runner`` over the streamed tile ranges of the SAM text in ``blocks`` (an
    iterable of bytes): ``runner(sub) -> (stats, offs, out)``, or, if it has a ``launch``
    method, ``runner.launch(sub) -> handle`` with ``handle.result() -> (stats, offs, out)``
    collected one batch later (batch k's results are fetched after batch k + 1 is launched).
    The parse runs on a producer thread (``_Producer``).  Raises NotSorted for unsorted input."""
    T = len(thresholds)
    parts = []
    stats = None
    state = {"held_max": 0, "cov": None, "lines": 0, "mapped": 0}

    def absorb(hb):
        flag = (hb.ref_reads > 0)
        state["cov"] = flag.copy() if state["cov"] is None else (state["cov"] | flag)
        state["lines"] += int(hb.info.lines_total)
        state["mapped"] += int(hb.info.reads_mapped)
    state["absorb"] = absorb

    launch = getattr(runner, "launch", None)
    pend = []            # (t0, t1, handle) launched, not yet collected

    def collect(entry):
        nonlocal stats
        t0, t1, h, sub = entry
        try:
            st, offs, out = h.result() if launch else h
        finally:
            sub.free()             # (the fetch reads the sub-batch's tile table)
        stats = st.copy() if stats is None else stats + st
        parts.append((t0, t1, np.asarray(offs, dtype=np.uint64), out))

    hb = None
    ct = {"launch": 0.0, "collect": 0.0, "wait": 0.0}
    clk = time.perf_counter
    tw = clk()
    ranged = getattr(runner, "launch_range", None)
    try:
        for item in _Producer(_sorted_items(blocks, maxdel_active, tile_width, batch_bytes, stats_hook, state,
                                            ranged is not None)):
            ct["wait"] += clk() - tw
            if item[0] == "last":
                hb = item[1]
                break
            _, sub, t0, t1 = item
            tl = clk()
            try:
                if ranged is not None and getattr(sub, "t0_range", None) is not None:
                    h = ranged(sub, t0, t1)
                else:
                    sub.t0, sub.t1 = t0, t1
                    h = launch(sub) if launch else runner(sub)
            except BaseException:
                sub.free()
                raise
            ct["launch"] += clk() - tl
            pend.append((t0, t1, h, sub))
            tl = clk()
            while len(pend) > 1:
                collect(pend.pop(0))
            ct["collect"] += clk() - tl
            tw = clk()
    except BaseException:
        # (NotSorted, or a reference error: the launched-but-uncollected batches' device
        # buffers and host snapshots go now, not with the traceback that holds this frame)
        for _, _, _, sub in pend:
            sub.free()
        pend.clear()
        raise
    tl = clk()
    while pend:
        collect(pend.pop(0))
    ct["collect"] += clk() - tl
    hb.ref_reads = state["cov"].astype(np.int64)          # Σcoverage > 0 in any batch (:334-341)
    offs, out = _merge(parts, T)
    if stats is None:
        stats = np.zeros((hb.info.n_refs, T, 4), np.uint64)
    res = StreamResult(hb, stats, offs, out, int(hb.info.header_lines), state["lines"], state["mapped"],
                       [(a, b) for a, b, _, _ in parts], state["held_max"])
    res.timings = {"producer_" + k: v for k, v in state.get("t", {}).items()}
    res.timings.update({"consumer_" + k: v for k, v in ct.items()})
    return res


class DeviceAccumulator:
    """Running totals counts[6][padded_len] u32 in HBM for unsorted input: ``add`` enqueues a
    batch's pileup into them (s2c_accumulate; the batch goes through the pinned staging ring
    and copy stream, nothing waits), ``finish`` adds the last batch and votes every tile from
    them (s2c_consensus over all tiles)."""

    def __init__(self, thresholds, min_depth=1, fill=b"-", device=None):
        self.thresholds, self.min_depth, self.fill, self.device = thresholds, min_depth, fill, device
        self.counts = None
        self.up = None

    def _ws(self, hb):
        import torch

        from .engine import DeviceBatch, Uploader, Workspace
        if self.up is None:
            self.up = Uploader(self.device)
        db = DeviceBatch(hb, uploader=self.up, dense_layers=True)   # (s2c_accumulate: k_tile takes the dense tiles)
        if self.counts is None:
            self.counts = torch.zeros(max(6 * int(hb.info.padded_len) * 4, 16), dtype=torch.uint8, device=db.device)
        return Workspace(db, self.thresholds, self.min_depth, self.fill, counts=self.counts)

    def add(self, hb):
        # (the batch's device buffers are released in stream order after its kernels; the
        # host arrays were copied into pinned staging by the upload)
        self._ws(hb).accumulate(keep_tables=False)

    def finish(self, hb):
        ws = self._ws(hb)
        ws.accumulate(keep_tables=True)
        ws.vote_all()
        return ws.fetch()


def _unsorted_items(blocks, maxdel_active, batch_bytes, state):
    """Generator (producer thread) of the unsorted streamed run: ("add", hb) per batch, then
    ("last", hb)."""
    p = StreamParser(maxdel_active, 150, 0)
    pending, broken = 0, False
    try:
        for blk in blocks:
            p.feed(blk)
            pending += len(blk)
            if broken or pending < batch_bytes:
                continue
            pending = 0
            _, ref, _, held = p.state()
            if ref < 0:
                continue
            state["held_max"] = max(state["held_max"], held)
            try:
                hb = p.snapshot()
            except (KeyError, IndexError):
                broken = True          # raised by s2c_parser_finish once the input is read
                continue
            state["absorb"](hb)
            p.retain_events()
            state["nb"] += 1
            yield ("add", hb)
        hb = p.finish()
        state["held_max"] = max(state["held_max"], p.state()[3])
        yield ("last", hb)
    finally:
        p.close()


def stream_unsorted(blocks, thresholds, acc, maxdel_active=True, batch_bytes=DEFAULT_BATCH):
    """Unsorted input in bounded host memory: every ``batch_bytes`` the reads held are
    counted into the accumulator's running totals and dropped, except their insertion
    events (``s2c_parser_retain_events``); the last batch holds every event of the file and
    is voted over the totals.  Same bytes and error precedence as one batch: the read-pass
    checks run as blocks are fed, and the last ``s2c_parser_finish`` sees every insertion
    event for the checks of :284-294.  The parse runs on a producer thread (``_Producer``)."""
    state = {"held_max": 0, "cov": None, "lines": 0, "mapped": 0, "nb": 0}

    def absorb(hb):
        flag = (hb.ref_reads > 0)
        state["cov"] = flag.copy() if state["cov"] is None else (state["cov"] | flag)
        state["lines"] += int(hb.info.lines_total)
        state["mapped"] += int(hb.info.reads_mapped)
    state["absorb"] = absorb

    hb = None
    for kind, b in _Producer(_unsorted_items(blocks, maxdel_active, batch_bytes, state)):
        if kind == "last":
            hb = b
            break
        try:
            acc.add(b)
        finally:
            b.free()
    stats, offs, out = acc.finish(hb)
    absorb(hb)
    hb.ref_reads = state["cov"].astype(np.int64)
    return StreamResult(hb, stats, offs, out, int(hb.info.header_lines), state["lines"], state["mapped"],
                        [(0, int(hb.info.n_tiles))] * (state["nb"] + 1), state["held_max"])


def _merge(parts, T):
    from .shard import merge_outputs
    return merge_outputs(parts, T)


def file_blocks(filename, block=BLOCK):
    """The file's bytes in blocks, read ahead on a thread into reused buffers (each block is a
    view, valid until the next is taken: the parser copies what it keeps).  A plain file by
    reads; a ".gz" (:111-114) through libs2c.so's reader — the one s2c_parser_feed_file uses:
    BGZF (bgzip / samtools) inflated block-parallel on the host threads, other gzip
    sequentially."""
    if filename.endswith(".gz"):
        yield from _read_ahead(filename, block, _native_source)
        return
    yield from _read_ahead(filename, block)


class _native_source:
    """libs2c.so's byte source (s2c_reader_*) with a file's readinto interface."""

    def __init__(self, filename):
        self._r = C.c_void_p()
        L.check(L.lib.s2c_reader_open(os.fsencode(filename), C.byref(self._r)))

    def readinto(self, b):
        n = C.c_size_t()
        mv = memoryview(b).cast("B")
        L.check(L.lib.s2c_reader_read(self._r, (C.c_char * mv.nbytes).from_buffer(mv), mv.nbytes, C.byref(n)))
        return n.value

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        if self._r:
            L.lib.s2c_reader_free(self._r)
            self._r = C.c_void_p()


def _plain_source(filename):
    return open(filename, "rb", buffering=0)


def _read_ahead(filename, block, source=_plain_source, nbuf=3):
    """A file's blocks read ahead on a thread (reads and inflates release the GIL) into a ring of
    ``nbuf`` reused buffers: block k + 1 is read while the caller parses block k.  With a
    hand-off queue of depth 1 the reader fills at most two buffers ahead, so the buffer it
    refills is one the caller has moved past (a block is valid until the next one is taken)."""
    import queue
    import threading
    bufs = [bytearray(block) for _ in range(nbuf)]
    q = queue.Queue(maxsize=1)
    stop = threading.Event()

    def reader():
        try:
            with source(filename) as fh:
                k = 0
                while not stop.is_set():
                    b = bufs[k % nbuf]
                    n = fh.readinto(b)
                    item = ("blk", memoryview(b)[:n]) if n else ("end", None)
                    while not stop.is_set():
                        try:
                            q.put(item, timeout=0.1)
                            break
                        except queue.Full:
                            continue
                    if not n:
                        return
                    k += 1
        except BaseException as e:  # noqa: BLE001 - re-raised by the caller
            q.put(("err", e))

    t = threading.Thread(target=reader, daemon=True)
    t.start()
    try:
        while True:
            kind, v = q.get()
            if kind == "end":
                return
            if kind == "err":
                raise v
            yield v
    finally:
        stop.set()
        while t.is_alive():   # (unblock a reader waiting to hand over a block)
            try:
                q.get_nowait()
            except queue.Empty:
                pass
            t.join(timeout=0.05)


class DeviceRunner:
    """The streamed batches' device side (sam2consensus_amd/engine.py): ``launch(sub)`` uploads
    the sub-batch through the pinned staging ring and copy stream (``Uploader``) and enqueues
    s2c_run on the compute stream without waiting; the handle's ``result()`` synchronises and
    fetches.  ``runner(sub)`` does both at once."""

    def __init__(self, thresholds, min_depth, fill, device=None):
        from .engine import Uploader
        self.thresholds, self.min_depth, self.fill = thresholds, min_depth, fill
        self.up = Uploader(device)

    def launch(self, sub):
        from .engine import DeviceBatch, Workspace, needs_dense_layers
        ws = Workspace(DeviceBatch(sub, uploader=self.up, dense_layers=needs_dense_layers(self.fill)), self.thresholds,
                       self.min_depth, self.fill)
        ws.run()
        return _Launched(ws, ws.record_done())

    def launch_range(self, hb, t0, t1):
        """The tiles [t0, t1) of a snapshot, without cutting a sub-batch (Workspace tile_range)."""
        from .engine import DeviceBatch, Workspace, needs_dense_layers
        ws = Workspace(DeviceBatch(hb, uploader=self.up, dense_layers=needs_dense_layers(self.fill)), self.thresholds,
                       self.min_depth, self.fill,
                       tile_range=(t0, t1))
        ws.run()
        return _Launched(ws, ws.record_done())

    def __call__(self, sub):
        return self.launch(sub).result()


class _Launched:
    """A launched batch: ``result()`` waits for its own kernels (the event recorded after
    them) and copies its results on a side stream while later batches run."""

    def __init__(self, ws, done=None):
        self.ws, self.done = ws, done

    def result(self):
        r = self.ws.fetch(self.done)
        self.ws = self.done = None
        return r


def device_runner(thresholds, min_depth, fill, device=None):
    """The streamed runner on the GPU (``DeviceRunner``)."""
    return DeviceRunner(thresholds, min_depth, fill, device)


def header_sort_order(filename):
    """The SO tag of the file's @HD line (plain or gzip, as the reference opens it, :111-114),
    or None without one."""
    import gzip
    opener = gzip.open if filename.endswith(".gz") else open
    try:
        with opener(filename, "rb") as fh:
            line = fh.readline(1 << 16)
    except (OSError, EOFError):
        return None
    if not line.startswith(b"@HD"):
        return None
    for tag in line.rstrip(b"\r\n").split(b"\t")[1:]:
        if tag.startswith(b"SO:"):
            return tag[3:].decode("latin-1")
    return None


def consensus_files_streamed(filename, thresholds, prefix, min_depth=1, fill=b"-", nchar=0, maxdel_active=True,
                             device=None, log=None, batch_bytes=DEFAULT_BATCH, tile_width=DEFAULT_TILE):
    """``cli.consensus_files`` in streamed batches (unsorted input: counts accumulated)."""
    from .cli import RunResult, _log_summary
    from .records import build_records, render

    t = {}
    t0 = time.perf_counter()
    res = None
    # a header that declares the records unsorted goes straight to accumulation (the sorted
    # pass would stop at its second snapshot and start over); any other runs the sorted pass,
    # which falls back when a read reaches below an emitted tile
    if header_sort_order(filename) not in ("unsorted", "queryname"):
        try:
            res = stream_batches(file_blocks(filename), thresholds, device_runner(thresholds, min_depth, fill, device),
                                 maxdel_active, tile_width, batch_bytes)
        except NotSorted:
            res = None   # (the second pass runs after the except block: no live traceback of the first)
    if res is None:   # counts added batch by batch into running totals in HBM
        res = stream_unsorted(file_blocks(filename), thresholds,
                              DeviceAccumulator(thresholds, min_depth, fill, device), maxdel_active, batch_bytes)
    t["stream"] = time.perf_counter() - t0
    t.update(getattr(res, "timings", {}))
    if log:
        _log_summary(log, res)
    t0 = time.perf_counter()
    fastas = build_records(res.hb, thresholds, prefix, res.stats, res.offs, res.out)
    pre = prefix.encode("latin-1") if isinstance(prefix, str) else prefix
    files = {n.encode("latin-1") + b"__" + pre + b".fasta": render(r, nchar) for n, r in fastas.items()}
    t["format"] = time.perf_counter() - t0
    r = RunResult(files, t, res.hb.info)
    r.batches = res.batches
    r.held_max = res.held_max
    return r


def stream_bytes_from_env():
    """S2C_STREAM=<bytes>[K|M|G] turns on streamed batches in the CLI (0 / unset: one batch)."""
    return _env_bytes("S2C_STREAM", 0)
