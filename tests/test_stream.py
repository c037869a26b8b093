"""Streamed batches (sam2consensus_amd/stream.py) on CPU: coordinate-sorted input fed in
blocks, cut into tile ranges by snapshot / shard / retain, must give the reference's bytes
and the whole-batch path's errors; unsorted input must be detected.  The per-range runner
is the kernel-shaped CPU model (tests/batch_model.py); tests/test_gpu.py runs the same
driver through libs2c.so's kernels."""
import os

import numpy as np
import pytest

import batch_model as bm
import golden_io
import s2c_oracle as o
from sam2consensus_amd import batch, configs, records, stream


def _blocks(data, n):
    for k in range(0, len(data), n):
        yield data[k:k + n]


def _runner(opt):
    return lambda sub: bm.model_pipeline(sub, opt.thresholds, opt.min_depth, opt.fill.encode("latin-1"))


def _files(res, opt):
    fastas = records.build_records(res.hb, opt.thresholds, opt.prefix, res.stats, res.offs, res.out)
    return {n + "__" + opt.prefix + ".fasta": records.render(r, opt.n).decode("latin-1") for n, r in fastas.items()}


def _stream(sam, args, block=97, batch_bytes=300, tile=64):
    opt = o.parse_argv(["-i", "in.sam"] + list(args))
    data = sam.encode("latin-1") if isinstance(sam, str) else sam
    res = stream.stream_batches(_blocks(data, block), opt.thresholds, _runner(opt), opt.maxdel_active,
                                tile, batch_bytes)
    return res, _files(res, opt)


def _sorted_case():
    """Several refs (header order = file order) with insertions, deletions, N runs, a POS=0
    wrap with an insertion and events with nothing counted."""
    sam = "@HD\tVN:1.6\tSO:coordinate\n@SQ\tSN:a\tLN:900\n@SQ\tSN:b\tLN:3000\n@SQ\tSN:c\tLN:40\n" \
          "@SQ\tSN:d\tLN:500\n"
    rows = []
    for s in range(1, 760, 3):
        rows.append(("a", s, "60M2I50M", "ACGT" * 28))
    rows.append(("b", 0, "1M2I3M", "AGGCCC"))                 # POS=0 wrap: changes b's end
    for s in range(1, 2800, 5):
        rows.append(("b", s, "40M3D60M", "TTGCA" * 20))
        if s == 10:
            rows.append(("b", 10, "10M2000N10M", "G" * 20))  # spans most of b
        if s == 1496:
            rows.append(("b", 1500, "5M2I", "GGGGGTT"))       # insertion after the last base
        if s == 1996:
            rows.append(("b", 2000, "3S4I", "AAACCCC"))       # events, nothing counted
    rows.append(("c", 0, "5M", "CCCCC"))
    rows.append(("c", 3, "4M", "NNAC"))
    for r in rows:
        sam += "r\t0\t%s\t%d\t60\t%s\t*\t0\t0\t%s\t*\n" % r
    sam += "u\t4\t*\t0\t0\t*\t*\t0\t0\tACGT\t*\n"             # unmapped tail
    return sam


@pytest.mark.parametrize("args", [[], ["-c", "0.25,0.75"], ["-d", "9"], ["-m", "3", "-f", "N"], ["-n", "50"]])
def test_sorted_stream_matches_reference(args):
    sam = _sorted_case()
    res, files = _stream(sam, args)
    assert len(res.batches) > 3, res.batches          # really cut into tile ranges
    assert files == o.run_case(sam, args)["files"]
    # line counters of the CLI summary (:224-228) over all batches
    hb = batch.parse_text(sam)
    assert (res.header_lines, res.lines_total, res.reads_mapped) == \
        (hb.info.header_lines, hb.info.lines_total, hb.info.reads_mapped)


@pytest.mark.parametrize("block,batch_bytes,tile", [(1, 1, 64), (4096, 2048, 128), (10 ** 6, 10 ** 6, 1024)])
def test_block_and_batch_sizes(block, batch_bytes, tile):
    sam = _sorted_case()
    _, files = _stream(sam, ["-c", "0.5"], block, batch_bytes, tile)
    assert files == o.run_case(sam, ["-c", "0.5"])["files"]


@pytest.mark.parametrize("pipe", ["0", "1"])
def test_pipelined_and_serial_snapshots_agree(monkeypatch, pipe):
    """S2C_STREAM_PIPE=1 (default): each batch's reads are detached and snapshot / retained
    on a helper thread while the feed goes on, then attached back (s2c_parser_detach /
    _attach); =0 does it in line.  Same bytes, counters and retained-read bound."""
    monkeypatch.setenv("S2C_STREAM_PIPE", pipe)
    sam = _sorted_case()
    for block, batch_bytes in ((97, 300), (1, 50), (4096, 2048)):
        res, files = _stream(sam, ["-c", "0.25,0.75"], block, batch_bytes)
        assert files == o.run_case(sam, ["-c", "0.25,0.75"])["files"]
        hb = batch.parse_text(sam)
        assert (res.header_lines, res.lines_total, res.reads_mapped) == \
            (hb.info.header_lines, hb.info.lines_total, hb.info.reads_mapped)
        assert len(res.batches) > 1 or batch_bytes > len(sam)
        assert [b[1] for b in res.batches] == sorted(b[1] for b in res.batches)


def test_detach_attach_round_trip():
    """Detached reads come back in front of the reads fed since; the batch equals one parse."""
    sam = _sorted_case().encode("latin-1")
    p = stream.StreamParser(True, 150, 64)
    cut = len(sam) // 2
    p.feed(sam[:cut])
    d = p.detach()
    with pytest.raises(Exception, match="detached parser takes no input"):
        d.feed(sam[cut:])
    p.feed(sam[cut:])
    p.attach(d)
    assert not d._p
    hb = p.finish()
    ref = batch.parse_text(sam.decode("latin-1"))
    assert (hb.info.lines_total, hb.info.reads_mapped) == (ref.info.lines_total, ref.info.reads_mapped)
    assert np.array_equal(np.asarray(hb.ref_reads), np.asarray(ref.ref_reads))
    hb.free()
    p.close()


def test_golden_cases_stream_or_detect_unsorted():
    """Every KAT case: byte-identical when streamed, or NotSorted (then the CLI runs one batch)."""
    n_streamed = 0
    for case in golden_io.load("kat"):
        try:
            _, files = _stream(case["sam"], case["args"], block=13, batch_bytes=40, tile=64)
        except stream.NotSorted:
            continue
        except (KeyError, IndexError, ValueError, ZeroDivisionError, OverflowError) as e:
            assert type(e).__name__ == case["status"], case["name"]
            n_streamed += 1
            continue
        assert case["status"] == "ok" and files == case["files"], case["name"]
        n_streamed += 1
    assert n_streamed >= 10


def test_unsorted_input_is_detected(tmp_path):
    sam = _sorted_case()
    head = [ln for ln in sam.splitlines(True) if ln.startswith("@")]
    body = [ln for ln in sam.splitlines(True) if not ln.startswith("@")]
    body = body[len(body) // 2:] + body[: len(body) // 2]
    with pytest.raises(stream.NotSorted):
        _stream("".join(head + body), [])
    # a synthetic shuffled config (C3's record order)
    path = str(tmp_path / "c3.sam")
    configs.synth_write("c3", path, scale=0.002)
    opt = o.parse_argv(["-i", path, "-m", "10"])
    with pytest.raises(stream.NotSorted):
        stream.stream_batches(stream.file_blocks(path, 1 << 16), opt.thresholds, _runner(opt), True, 256, 1 << 17)


def test_reformat_error_then_read_pass_error_keeps_precedence():
    """An insertion-key error (:294) in an early batch, a bad POS (:201) later: the read
    pass error wins, as in the reference; without the later line the IndexError is raised."""
    sam = "@SQ\tSN:a\tLN:10\n@SQ\tSN:b\tLN:2000\n"
    sam += "r\t0\ta\t9\t60\t2M3I\t*\t0\t0\tACGGG\t*\n"     # key 10 == LN → IndexError (:294)
    for s in range(1, 1800, 7):
        sam += "r\t0\tb\t%d\t60\t20M\t*\t0\t0\t%s\t*\n" % (s, "ACGTA" * 4)
    good = o.run_case(sam, [])
    assert good["status"] == "IndexError"
    with pytest.raises(IndexError):
        _stream(sam, [], block=50, batch_bytes=100)
    bad = sam + "r\t0\tb\tx\t60\t20M\t*\t0\t0\tACGT\t*\n"
    assert o.run_case(bad, [])["status"] == "ValueError"
    with pytest.raises(ValueError):
        _stream(bad, [], block=50, batch_bytes=100)


def test_retain_bounds_the_reads_held(tmp_path):
    """A sorted synthetic config (C2's shape, 30 loci): byte-identical to the whole batch,
    and the parser never holds more than a few batches' reads."""
    path = str(tmp_path / "c2.sam")
    configs.synth_write("c2", path, n_refs=30, depth=60.0)
    args = configs.cli_args("c2")
    opt = o.parse_argv(["-i", path] + args)
    size = os.path.getsize(path)
    res = stream.stream_batches(stream.file_blocks(path, 1 << 14), opt.thresholds, _runner(opt),
                                opt.maxdel_active, 512, size // 8)
    assert len(res.batches) >= 6
    hb = batch.parse_file(path, opt.maxdel_active)
    st, offs, out = bm.model_pipeline(hb, opt.thresholds, opt.min_depth, opt.fill.encode("latin-1"))
    whole = {n + "__" + opt.prefix + ".fasta": records.render(r, opt.n).decode("latin-1")
             for n, r in records.build_records(hb, opt.thresholds, opt.prefix, st, offs, out).items()}
    assert _files(res, opt) == whole
    assert res.held_max < 0.4 * hb.info.reads_mapped
    assert np.array_equal(res.stats.sum(axis=0), st.sum(axis=0))


class ModelAccumulator:
    """stream.DeviceAccumulator on the CPU model: running totals of the batches' counts."""

    def __init__(self, opt):
        self.opt, self.counts = opt, None

    def add(self, hb):
        c = bm.model_counts(hb)
        self.counts = c if self.counts is None else self.counts + c

    def finish(self, hb):
        o_ = self.opt
        return bm.model_pipeline(hb, o_.thresholds, o_.min_depth, o_.fill.encode("latin-1"), counts_add=self.counts)


def _stream_unsorted(sam, args, block=97, batch_bytes=300):
    opt = o.parse_argv(["-i", "in.sam"] + list(args))
    data = sam.encode("latin-1") if isinstance(sam, str) else sam
    res = stream.stream_unsorted(_blocks(data, block), opt.thresholds, ModelAccumulator(opt), opt.maxdel_active,
                                 batch_bytes)
    return res, _files(res, opt)


def _shuffled_case(seed=5):
    sam = _sorted_case()
    head = [ln for ln in sam.splitlines(True) if ln.startswith("@")]
    body = [ln for ln in sam.splitlines(True) if not ln.startswith("@")]
    np.random.default_rng(seed).shuffle(body)
    return "".join(head + body)


@pytest.mark.parametrize("args", [[], ["-c", "0.25,0.75"], ["-d", "9"], ["-m", "3", "-f", "N"]])
def test_unsorted_accumulation_matches_reference(args):
    sam = _shuffled_case()
    res, files = _stream_unsorted(sam, args)
    assert len(res.batches) > 5
    assert files == o.run_case(sam, args)["files"]
    hb = batch.parse_text(sam)
    assert (res.lines_total, res.reads_mapped) == (hb.info.lines_total, hb.info.reads_mapped)
    # only reads with insertion events are carried to the last batch
    assert res.held_max < hb.info.reads_mapped / 2


def test_unsorted_accumulation_on_every_kat_case():
    """Every KAT case through the accumulation driver: the reference's files or exception."""
    for case in golden_io.load("kat"):
        try:
            _, files = _stream_unsorted(case["sam"], case["args"], block=11, batch_bytes=30)
        except (KeyError, IndexError, ValueError, ZeroDivisionError, OverflowError) as e:
            assert type(e).__name__ == case["status"], case["name"]
            continue
        assert case["status"] == "ok" and files == case["files"], case["name"]


def test_unsorted_accumulation_shuffled_config(tmp_path):
    """C3's shuffled record order (reduced) in 6+ batches == the whole batch."""
    path = str(tmp_path / "c3.sam.gz")
    configs.synth_write("c3", path, scale=0.001)
    opt = o.parse_argv(["-i", path, "-m", "10"])
    with pytest.raises(stream.NotSorted):
        stream.stream_batches(stream.file_blocks(path, 1 << 16), opt.thresholds, _runner(opt), True, 256, 1 << 17)
    size = sum(len(b) for b in stream.file_blocks(path))
    res = stream.stream_unsorted(stream.file_blocks(path, 1 << 15), opt.thresholds, ModelAccumulator(opt), True,
                                 size // 6)
    assert len(res.batches) >= 6
    want, _ = o.run_path(path, ["-m", "10"])
    assert _files(res, opt) == want


def test_file_blocks_read_ahead(tmp_path):
    """stream.file_blocks on a plain file: the blocks (views of a reader thread's reused
    buffers, each consumed before the next is taken) concatenate to the file; an empty file
    gives none; closing the generator early stops the reader."""
    data = bytes(np.random.default_rng(5).integers(0, 256, size=300_001, dtype=np.uint8))
    path = str(tmp_path / "x.sam")
    with open(path, "wb") as fh:
        fh.write(data)
    for block in (7, 4096, 65536, 1 << 20):
        got = b"".join(bytes(b) for b in stream.file_blocks(path, block))
        assert got == data
    empty = str(tmp_path / "e.sam")
    open(empty, "wb").close()
    assert list(stream.file_blocks(empty, 4096)) == []
    g = stream.file_blocks(path, 1024)
    assert bytes(next(g)) == data[:1024]
    g.close()


def test_header_sort_order(tmp_path):
    """The streamed CLI reads the @HD SO tag (plain or gzip) to skip the sorted pass of input
    declared unsorted; no @HD line, or one without SO: None (the sorted pass runs)."""
    import gzip
    cases = {"a.sam": (b"@HD\tVN:1.6\tSO:coordinate\n@SQ\tSN:g\tLN:9\n", "coordinate"),
             "b.sam.gz": (b"@HD\tVN:1.6\tSO:unsorted\n", "unsorted"),
             "c.sam": (b"@SQ\tSN:g\tLN:9\n@HD\tSO:unsorted\n", None),
             "d.sam": (b"@HD\tVN:1.6\r\n", None),
             "e.sam": (b"", None)}
    for name, (data, want) in cases.items():
        p = tmp_path / name
        p.write_bytes(gzip.compress(data) if name.endswith(".gz") else data)
        assert stream.header_sort_order(str(p)) == want, name
    assert stream.header_sort_order(str(tmp_path / "missing.sam")) is None



def _slow_stages(monkeypatch, log, delay=0.1):
    """Make the pipelined stage (a detached parser's snapshot on the s2c-stage helper thread)
    slow and record, for the feeding parser, how many bytes were fed and whether a stage was
    in flight when the byte at ``log['mark']`` went in."""
    import threading
    import time
    snap, feed = stream.StreamParser.snapshot, stream.StreamParser.feed

    def slow_snapshot(self, *a):
        if threading.current_thread().name.startswith("s2c-stage"):
            log["in_stage"] += 1
            try:
                time.sleep(delay)
                return snap(self, *a)
            finally:
                log["in_stage"] -= 1
        return snap(self, *a)

    def logged_feed(self, data):
        n0 = log["fed"]
        log["fed"] += len(data)
        if n0 <= log["mark"] < log["fed"]:
            log["mark_in_stage"] = log["in_stage"] > 0
        return feed(self, data)

    monkeypatch.setattr(stream.StreamParser, "snapshot", slow_snapshot)
    monkeypatch.setattr(stream.StreamParser, "feed", logged_feed)


def _cli_like(sam, args, block, batch_bytes):
    """The CLI's streamed driver on the CPU model: sorted batches, or on NotSorted the
    accumulation pass over the whole input; (status, files)."""
    try:
        try:
            return "ok", _stream(sam, args, block, batch_bytes)[1]
        except stream.NotSorted:
            return "ok", _stream_unsorted(sam, args, block, batch_bytes)[1]
    except (KeyError, IndexError, ValueError, ZeroDivisionError, OverflowError) as e:
        return type(e).__name__, {}


def _with_line(sam, frac, line):
    head = [ln for ln in sam.splitlines(True) if ln.startswith("@")]
    body = [ln for ln in sam.splitlines(True) if not ln.startswith("@")]
    k = int(len(body) * frac)
    out = "".join(head + body[:k] + [line] + body[k:])
    return out, len("".join(head + body[:k]).encode("latin-1"))


def test_late_read_fed_while_a_stage_runs(monkeypatch):
    """Pipelined snapshots (advisor, round 4): a read that reaches already-emitted positions,
    fed while the previous batch's snapshot / retain runs on the helper thread, is caught
    (NotSorted) — and the CLI's fallback gives the reference's bytes, as the serial order does."""
    sam, at = _with_line(_sorted_case(), 0.6, "late\t0\ta\t1\t60\t30M\t*\t0\t0\t%s\t*\n" % ("C" * 30))
    size = len(sam.encode("latin-1"))
    log = {"fed": 0, "in_stage": 0, "mark": at, "mark_in_stage": None}
    _slow_stages(monkeypatch, log)
    monkeypatch.setenv("S2C_STREAM_PIPE", "1")
    with pytest.raises(stream.NotSorted):
        _stream(sam, [], block=97, batch_bytes=size // 3)
    assert log["mark_in_stage"] is True   # (the late read really went in during a stage)
    want = o.run_case(sam, [])
    assert want["status"] == "ok"
    for pipe in ("1", "0"):
        monkeypatch.setenv("S2C_STREAM_PIPE", pipe)
        assert _cli_like(sam, [], 97, size // 3) == ("ok", want["files"]), pipe


@pytest.mark.parametrize("late_frac", [None, 0.2, 0.5])
def test_feed_error_while_a_stage_runs(monkeypatch, late_frac):
    """A read-pass error (bad POS, :201) fed while a stage is in flight — alone, after a late
    read held by the in-flight stage (0.2), or after one fed during it (0.5): the pipelined and
    the serial driver end with the reference's exception class."""
    sam, at = _with_line(_sorted_case(), 0.6, "bad\t0\tb\tx\t60\t20M\t*\t0\t0\t%s\t*\n" % ("A" * 20))
    if late_frac is not None:
        sam, _ = _with_line(sam, late_frac, "late\t0\ta\t1\t60\t30M\t*\t0\t0\t%s\t*\n" % ("C" * 30))
        at += len("late\t0\ta\t1\t60\t30M\t*\t0\t0\t\t*\n") + 30
    size = len(sam.encode("latin-1"))
    want = o.run_case(sam, [])
    assert want["status"] == "ValueError"
    log = {"fed": 0, "in_stage": 0, "mark": at, "mark_in_stage": None}
    _slow_stages(monkeypatch, log)
    got = {}
    for pipe in ("1", "0"):
        monkeypatch.setenv("S2C_STREAM_PIPE", pipe)
        log.update(fed=0, mark_in_stage=None)
        got[pipe] = _cli_like(sam, [], 97, size // 3)
        if pipe == "1":
            assert log["mark_in_stage"] is True
    assert got["1"] == got["0"] == ("ValueError", {})


def test_ranged_snapshot_plans_only_the_tiles_a_batch_can_run():
    """s2c_parser_snapshot_from (ABI 13, the streamed driver's snapshots): tiles before t_from
    and after the tile of the held reads' last position get no window, layers or items; the
    tiles in between are planned exactly as a whole snapshot plans them."""
    sam = _sorted_case().encode("latin-1")
    p = stream.StreamParser(True, 150, 64)
    p.feed(sam[: len(sam) * 2 // 3])
    full = p.snapshot()
    nt = int(full.info.n_tiles)
    assert (full.info.plan_t0, full.info.plan_t1) == (0, nt)
    for t_from in (0, 5, nt // 3):
        part = p.snapshot(t_from)
        try:
            P0, P1 = int(part.info.plan_t0), int(part.info.plan_t1)
            assert P0 == t_from and t_from < P1 < nt
            bm.check_plan(part)
            _, ref, pos0, _ = p.state()
            bound = int(part.ref_off[ref]) + max(pos0, 0)
            t1 = int(np.searchsorted(part.tiles[:, 1].astype(np.int64), bound, side="right"))
            assert t1 <= P1                                      # every tile the batch can run is planned
            # planned tiles: the same records (windows, capacities, layers) and items
            assert np.array_equal(part.tiles[P0:P1, :20], full.tiles[P0:P1, :20])
            keep = lambda a: a[(a[:, 0] >= P0) & (a[:, 0] < P1)]  # noqa: E731
            assert np.array_equal(keep(part.items), keep(full.items)) and np.array_equal(keep(part.dense), keep(full.dense))
            assert (part.tiles[:P0, 3] == 0).all() and (part.tiles[P1:, 19] == 0).all()
            assert len(part.items) + len(part.dense) < len(full.items) + len(full.dense)
        finally:
            part.free()
    full.free()
    p.close()


@pytest.mark.parametrize("pos", [900, 1000, 5000])
def test_zero_span_read_past_the_reference_end(pos):
    """A kept read with no aligned span (a CIGAR of S only) whose POS is past LN (and past
    the 64-position padding) on a reference that is not the last: the reference counts
    nothing for it (:206-218) and goes on.  A streamed snapshot taken right after it bounds
    its final tiles like the host plan does (POS clamped to the reference's last position),
    never into the next reference's tiles."""
    sam = "@HD\tVN:1.6\tSO:coordinate\n@SQ\tSN:a\tLN:900\n@SQ\tSN:b\tLN:300\n"
    rows = [("a", s, "30M", "ACGTA" * 6) for s in range(1, 860, 7)]
    rows.append(("a", pos, "5S", "ACGTA"))
    rows += [("b", s, "20M", "TTGCA" * 4) for s in range(1, 280, 9)]
    for r in rows:
        sam += "r\t0\t%s\t%d\t60\t%s\t*\t0\t0\t%s\t*\n" % r
    want = o.run_case(sam, [])
    assert want["status"] == "ok"
    for block, batch_bytes in ((1, 1), (37, 64), (97, 300)):
        res, files = _stream(sam, [], block, batch_bytes)
        assert files == want["files"], (block, batch_bytes)
