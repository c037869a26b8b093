"""CPU tier: libs2c.so loads and exports the C-ABI; the host parser + packed batch + work
plan, run through a kernel-shaped CPU model (tests/batch_model.py), reproduce the
reference's golden outputs; parsecigar mirror; generator determinism."""
import hashlib
import os
import random
import subprocess
import tempfile

import numpy as np
import pytest

import batch_model as bm
import golden_io
import s2c_oracle as o
from sam2consensus_amd import _lib, batch, configs, records

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = golden_io.cases()


def test_library_exports_every_declared_symbol():
    header = open(os.path.join(ROOT, "include", "s2c.h")).read()
    import re
    declared = set(re.findall(r"\b(s2c_[a-z_0-9]+)\s*\(", header))
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert declared <= exported, declared - exported
    assert declared == set(_lib.EXPORTS)
    hv = int(re.search(r"#define S2C_ABI_VERSION (\d+)", header).group(1))
    assert _lib.lib.s2c_abi_version() == _lib.ABI_VERSION == hv == 14


def _model_case(sam, args):
    opt = o.parse_argv(["-i", "in.sam"] + list(args))
    try:
        hb = batch.parse_text(sam, opt.maxdel_active, 150)
        bm.check_plan(hb)
        stats, offs, out = bm.model_pipeline(hb, opt.thresholds, opt.min_depth, opt.fill.encode("latin-1"))
        fastas = records.build_records(hb, opt.thresholds, opt.prefix, stats, offs, out)
        return "ok", {n + "__" + opt.prefix + ".fasta": records.render(r, opt.n).decode("latin-1")
                      for n, r in fastas.items()}
    except (KeyError, IndexError, ValueError, ZeroDivisionError, OverflowError) as e:
        return type(e).__name__, {}


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_packed_batch_model_matches_reference(case):
    status, files = _model_case(case["sam"], case["args"])
    assert status == case["status"]
    assert files == case["files"]


def test_parsecigar_mirror_matches_oracle():
    rng = random.Random(3)
    for _ in range(3000):
        cig = "".join("%d%s" % (rng.randint(0, 7), rng.choice("MIDNSHPX=?")) for _ in range(rng.randint(0, 5)))
        seq = "".join(rng.choice("ACGTN-") for _ in range(rng.randint(0, 20)))
        pos = rng.randint(-3, 30)
        assert batch.parsecigar(cig, seq, pos) == o.parsecigar(cig, seq, pos), (cig, seq, pos)


def test_plan_covers_every_position_c2_scaled():
    hb = configs.synth_batch("c2", scale=0.05)
    bm.check_plan(hb)
    assert hb.info.n_ins > 0
    # the device's run records (k_reads restated) reproduce the oracle's counts exactly
    counts = bm.model_counts(hb)
    sp = configs.spec("c2", scale=0.05)
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "c2s.sam")
        import ctypes as C
        n = C.c_int64()
        _lib.check(_lib.lib.s2c_synth_write(C.byref(sp), p.encode(), C.byref(n)))
        text = open(p, "rb").read().decode("latin-1")
    lines = o._lines(text)
    refs = o.read_header(lines)
    ocounts, _ = o.pileup(lines, refs, o.parse_argv(["-i", "x"] + configs.cli_args("c2")))
    for r, name in enumerate(hb.names):
        off, L = int(hb.ref_off[r]), int(hb.ref_len[r])
        want = np.array(ocounts[name], dtype=np.int64).T
        assert (counts[:, off:off + L] == want).all()
    assert int(counts.sum()) == hb.info.aligned_bases  # no maxdel drops in c2


def test_long_reads_and_wrap_pieces():
    # a 3020-position read is a long piece (tile long lists); POS=0 wraps (:212) into two
    # pieces at the reference's end and start
    sam = "@SQ\tSN:g\tLN:5000\n"
    sam += "r\t0\tg\t1\t60\t10M3000N10M\t*\t0\t0\t%s\t*\n" % ("A" * 20)
    sam += "r\t0\tg\t0\t60\t5M\t*\t0\t0\tCCCCC\t*\n"
    for s in range(1, 4900, 7):
        sam += "r\t0\tg\t%d\t60\t100M\t*\t0\t0\t%s\t*\n" % (s, "G" * 100)
    hb = batch.parse_text(sam, True, 150)
    assert hb.info.n_pieces == 1 + 2 + len(range(1, 4900, 7))
    assert ((hb.pc[:-1, 3] >> 24) & 8).sum() == 8   # the long piece
    bm.check_plan(hb)
    counts = bm.model_counts(hb)
    assert counts[1, 0:10].tolist() == [1] * 10 and counts[1, 3010:3020].tolist() == [1] * 10
    assert counts[0, 10:3010].max() == 0               # 3000 '-' > maxdel 150: not counted (:214-218)
    assert counts[2, 4999] == 1 and counts[2, 0:4].tolist() == [1] * 4   # wrap: C at 4999, 0-3
    opt = o.parse_argv(["-i", "in.sam", "-d", "1"])
    hb2 = batch.parse_text(sam, False, 150)
    assert (bm.model_counts(hb2)[0, 10:3010] == 1).all()   # -d given: the filter is never applied
    stats, offs, out = bm.model_pipeline(hb2, opt.thresholds, 1, b"-")
    fastas = records.build_records(hb2, opt.thresholds, "in", stats, offs, out)
    got = {n + "__in.fasta": records.render(r, 0).decode() for n, r in fastas.items()}
    assert got == o.run_case(sam, ["-d", "1"])["files"]


ARRAYS = ("pc", "ops", "bq", "bx", "rs", "tiles", "items", "dense", "deep", "lp", "wtile")


def _same(a, b):
    for n in ARRAYS:
        assert (np.asarray(getattr(a, n)) == np.asarray(getattr(b, n))).all(), n


def test_text_and_file_and_gzip_parse_agree():
    sam = golden_io.load("kat")[0]["sam"]
    with tempfile.TemporaryDirectory() as td:
        import gzip
        p1, p2 = os.path.join(td, "a.sam"), os.path.join(td, "a.sam.gz")
        open(p1, "w").write(sam)
        with gzip.open(p2, "wt") as fh:
            fh.write(sam)
        hbs = [batch.parse_text(sam), batch.parse_file(p1), batch.parse_file(p2)]
    for h in hbs[1:]:
        _same(h, hbs[0])


def test_retain_after_unpack_keeps_reads(tmp_path):
    """Chunks made by s2c_parser_unpack carry no extent bound; a retain after an unpack must
    test their reads instead of dropping the chunk (advisor, round 4): retain(0) keeps every
    read, so the batch equals the one parsed from the text."""
    from sam2consensus_amd.dparse import BlockParser
    p = str(tmp_path / "c.sam")
    configs.synth_write("c2", p, scale=0.02)
    text = open(p, "rb").read()
    hdr = b"".join(line + b"\n" for line in text.split(b"\n") if line.startswith(b"@"))
    src = BlockParser(False, 150)
    src.feed(text)
    blob = src.pack(0, 1 << 40)
    src.close()
    dst = BlockParser(False, 150)
    dst.feed(hdr)
    dst.unpack(blob)
    _lib.check(_lib.lib.s2c_parser_retain(dst._p, 0))
    got = dst.finish()
    dst.close()
    want = batch.parse_text(text.decode("latin-1"), maxdel_active=False)
    assert len(np.asarray(want.pc)) > 1000
    _same(got, want)


def test_bgzf_block_parallel_inflate(tmp_path):
    """synth_write's .sam.gz is BGZF (the blocked gzip of bgzip / samtools): it reads back as
    the same text through Python's gzip, and the parser's block-parallel inflate gives the
    plain file's batch; a BGZF stream followed by an ordinary gzip member (sequential inflate
    from there), and a truncated file (IOError), too."""
    import gzip
    p, pz = str(tmp_path / "c.sam"), str(tmp_path / "c.sam.gz")
    configs.synth_write("c2", p, scale=0.02)
    configs.synth_write("c2", pz, scale=0.02)
    raw = open(p, "rb").read()
    zb = open(pz, "rb").read()
    assert zb[:4] == b"\x1f\x8b\x08\x04" and zb[12:14] == b"BC" and len(raw) > 200000
    assert gzip.decompress(zb) == raw
    a, b = batch.parse_file(p), batch.parse_file(pz)
    _same(a, b)
    assert a.info.lines_total == b.info.lines_total and a.info.reads_mapped == b.info.reads_mapped
    # BGZF blocks (without the EOF marker) + one ordinary gzip member of the rest
    cut = raw.rfind(b"\n", 0, len(raw) // 2) + 1
    pm = str(tmp_path / "m.sam.gz")
    import zlib
    blocks = []
    for i in range(0, cut, 60000):
        piece = raw[i:min(i + 60000, cut)]
        co = zlib.compressobj(1, zlib.DEFLATED, -15)
        d = co.compress(piece) + co.flush()
        total = 18 + len(d) + 8
        hdr = bytes([0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 66, 67, 2, 0, (total - 1) & 0xff, (total - 1) >> 8])
        blocks.append(hdr + d + zlib.crc32(piece).to_bytes(4, "little") + len(piece).to_bytes(4, "little"))
    open(pm, "wb").write(b"".join(blocks) + gzip.compress(raw[cut:]))
    c = batch.parse_file(pm)
    _same(a, c)
    pt = str(tmp_path / "t.sam.gz")
    open(pt, "wb").write(zb[: len(zb) // 2])
    with pytest.raises(IOError):
        batch.parse_file(pt)


def test_piece_flags_mark_non_acgt_and_dash_seq():
    """S2C_PF_X for a SEQ with any non-ACGT char, S2C_PF_DASH only when one is '-' (the maxdel
    rule, :210, scans the planes of those reads alone)."""
    sam = ("@SQ\tSN:g\tLN:100\n"
           "r1\t0\tg\t1\t60\t8M\t*\t0\t0\tACGTACGT\t*\n"
           "r2\t0\tg\t1\t60\t8M\t*\t0\t0\tACGNACGT\t*\n"
           "r3\t0\tg\t1\t60\t8M\t*\t0\t0\tAC-TACGT\t*\n"
           "r4\t0\tg\t1\t60\t8M\t*\t0\t0\tNC-TACGN\t*\n")
    hb = batch.parse_text(sam, True, 150)
    from sam2consensus_amd import _lib as L
    fl = sorted(int(f) for f in (hb.pc[:-1, 3] >> 24) & (L.S2C_PF_X | L.S2C_PF_DASH))
    assert fl == [0, L.S2C_PF_X, L.S2C_PF_X | L.S2C_PF_DASH, L.S2C_PF_X | L.S2C_PF_DASH]


def test_streaming_chunks_equal_whole():
    sam = "".join(c["sam"] for c in golden_io.load("kat")[:1])
    p = batch.Parser()
    for i in range(0, len(sam), 7):
        p.feed(sam[i:i + 7].encode())
    a = p.finish()
    b = batch.parse_text(sam)
    _same(a, b)


def test_generator_c2_is_pinned():
    g = golden_io.load("configs")["c2"]
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "c2.sam")
        n = configs.synth_write("c2", p)
        h = hashlib.sha256()
        with open(p, "rb") as fh:
            for chunk in iter(lambda: fh.read(1 << 22), b""):
                h.update(chunk)
    assert n == g["n_reads"] == 1176549
    assert h.hexdigest() == g["sam_sha256"]


def test_c2_batch_stats():
    hb = configs.synth_batch("c2")
    i = hb.info
    assert i.reads_mapped == 1176549 and i.n_refs == 353
    assert 176_000_000 < i.aligned_bases < 177_000_000
    assert i.n_items + i.n_dense >= 512 and i.tile_max <= 2048   # enough work items to fill 256 CUs
    bm.check_plan(hb)


def _batch_digest(path, maxdel_active):
    import hashlib
    try:
        hb = batch.parse_file(path, maxdel_active, 150)
    except (KeyError, IndexError, ValueError, ZeroDivisionError, OverflowError) as e:
        return type(e).__name__
    h = hashlib.sha256()
    for n in ARRAYS:
        h.update(np.ascontiguousarray(getattr(hb, n)).tobytes())
    i = hb.info
    h.update(repr((i.lines_total, i.reads_mapped, i.aligned_bases, i.query_bases, i.header_lines)).encode())
    return h.hexdigest()


def _text_digest(text, maxdel_active):
    try:
        hb = batch.parse_text(text, maxdel_active, 150)   # (< 4 MB: line by line, split_fields)
    except (KeyError, IndexError, ValueError, ZeroDivisionError, OverflowError) as e:
        return type(e).__name__
    h = hashlib.sha256()
    for n in ARRAYS:
        h.update(np.ascontiguousarray(getattr(hb, n)).tobytes())
    i = hb.info
    h.update(repr((i.lines_total, i.reads_mapped, i.aligned_bases, i.query_bases, i.header_lines)).encode())
    return h.hexdigest()


def _scan_cases():
    """Lines whose tabs and newlines fall on and around the file scanner's 32-byte steps."""
    head = "@SQ\tSN:g\tLN:400\n@SQ\tSN:h\tLN:90\n"
    out = []
    for pad in range(0, 40):
        name = "r" * (1 + pad)
        rows = [
            "%s\t0\tg\t%d\t60\t%dM\t*\t0\t0\t%s\t*\n" % (name, 1 + pad, 12 + pad, ("ACGT" * 20)[:12 + pad]),
            "%s\t0\th\t3\t60\t4M2I3M\t*\t0\t0\tACGTTTACG\tIIIIIIIII\textra\tfields\n" % name,
            "%s\t4\t*\t0\t0\t*\t*\t0\t0\tACGT\n" % name,                   # unmapped, 10 fields
            "@CO\tinside the records\n",
            "%s\t0\tg\t%d\t60\t%dM\t*\t0\t0\t%s" % (name, 5, 7, "NACGT-A"),   # last line, no '\n'
        ]
        out.append(head + "".join(rows))
        out.append(head + rows[0] + "%s\t0\tg\t1\t60\t3M\n" % name + rows[2])   # < 10 fields: IndexError
    return out


def test_file_scanner_splits_like_the_line_parser(tmp_path):
    """The file parse splits each line in one 32-byte-step pass (scan_line); the sequential
    feed splits it field by field (split_fields): same batch, same error, on every fuzz / KAT
    case and on lines whose tabs and newlines sit at every offset of the 32-byte steps."""
    p = tmp_path / "in.sam"
    for case in CASES[:200]:
        opt = o.parse_argv(["-i", "in.sam"] + list(case["args"]))
        p.write_bytes(case["sam"].encode("latin-1"))
        assert _batch_digest(str(p), opt.maxdel_active) == _text_digest(case["sam"], opt.maxdel_active), case["name"]
    for text in _scan_cases():
        p.write_bytes(text.encode("latin-1"))
        assert _batch_digest(str(p), True) == _text_digest(text, True), text[:80]


def test_parallel_file_parse_equals_sequential(tmp_path, monkeypatch):
    """The threaded file parse (record lines cut into chunks, merged in file order) builds
    the same batch as one thread, and raises the first error in file order."""
    p = tmp_path / "in.sam"
    for case in CASES[:400]:
        opt = o.parse_argv(["-i", "in.sam"] + list(case["args"]))
        p.write_bytes(case["sam"].encode("latin-1"))
        got = {}
        for t in ("1", "3", "7"):
            monkeypatch.setenv("S2C_PARSE_THREADS", t)
            got[t] = _batch_digest(str(p), opt.maxdel_active)
        assert got["1"] == got["3"] == got["7"], case["name"]   # (the error class, if any)
    # a larger input, chunks of many lines each
    sp = configs.spec("c2", scale=0.02)
    import ctypes as C
    n = C.c_int64()
    _lib.check(_lib.lib.s2c_synth_write(C.byref(sp), str(p).encode(), C.byref(n)))
    got = {}
    for t in ("1", "5"):
        monkeypatch.setenv("S2C_PARSE_THREADS", t)
        got[t] = _batch_digest(str(p), True)
    assert got["1"] == got["5"]


def test_worker_pools_concurrent_and_forked(tmp_path, monkeypatch):
    """The host's persistent worker pools (s2c_host.cpp WorkerPool): parses and plans run from
    several Python threads at once (a busy pool hands the second caller threads of its own)
    and from a forked child after the parent used the pools — each one the same batch as a
    serial parse."""
    import ctypes as C
    import multiprocessing as mp
    import threading
    p = tmp_path / "in.sam"
    sp = configs.spec("c2", scale=0.05)
    n = C.c_int64()
    _lib.check(_lib.lib.s2c_synth_write(C.byref(sp), str(p).encode(), C.byref(n)))
    monkeypatch.setenv("S2C_PARSE_THREADS", "4")
    want = _batch_digest(str(p), True)
    got, errs = [None] * 4, []

    def run(k):
        try:
            got[k] = _batch_digest(str(p), True)
        except BaseException as e:  # noqa: BLE001 - reported below
            errs.append(e)
    th = [threading.Thread(target=run, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs and got == [want] * 4
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    ch = ctx.Process(target=lambda: q.put(_batch_digest(str(p), True)))
    ch.start()
    try:
        assert q.get(timeout=120) == want
    finally:
        ch.join(timeout=30)
    assert ch.exitcode == 0


def test_batch_does_not_read_unwritten_memory(tmp_path):
    """The packed batch's arrays come from an allocator that leaves them uninitialised
    (uninit_alloc; fresh mappings happen to be zero pages).  With S2C_MAP_POISON=1 every such
    array starts as 0xA5 bytes: the batch (every array, the plan and the layered windows) must
    not change, i.e. no field is left unwritten and read as zero."""
    import ctypes as C
    import sys
    p = tmp_path / "in.sam"
    sp = configs.spec("c2", scale=0.05)
    n = C.c_int64()
    _lib.check(_lib.lib.s2c_synth_write(C.byref(sp), str(p).encode(), C.byref(n)))
    code = ("import sys, hashlib, numpy as np; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
            "from sam2consensus_amd import batch\n"
            "hb = batch.parse_file(%r, True, 150).ensure_layers(dense=True)\n"
            "h = hashlib.sha256()\n"
            "for k in sorted(vars(hb)):\n"
            "    v = getattr(hb, k)\n"
            "    if isinstance(v, np.ndarray): h.update(k.encode()); h.update(np.ascontiguousarray(v).tobytes())\n"
            "print(h.hexdigest())\n") % (ROOT, os.path.join(ROOT, "tests"), str(p))
    out = {}
    for poison in ("0", "1"):
        env = dict(os.environ)
        env.pop("S2C_MAP_POISON", None)
        if poison == "1":
            env["S2C_MAP_POISON"] = "1"
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        out[poison] = r.stdout.strip().splitlines()[-1]
    assert out["0"] == out["1"]


# ---------------------------------------------------------------- CLI progress lines
def _ref_progress(header_lines, lines_total):
    """:182, :194, :224-225 restated line by line (the counter starts at -header_length)."""
    out, t = [], -header_lines
    for _ in range(lines_total):
        t += 1
        if t % 500000 == 0:
            out.append(str(t) + " reads processed.")
    return out


@pytest.mark.parametrize("h,n", [(0, 0), (0, 10), (3, 3), (3, 10), (0, 500000), (2, 500002), (2, 500001),
                                 (5, 1500005), (600000, 600001), (600000, 1200000)])
def test_progress_lines_match_reference_counter(h, n):
    from sam2consensus_amd.cli import progress_lines
    assert progress_lines(h, n) == _ref_progress(h, n)


# ---------------------------------------------------------------- stdout vs the reference's own
def _stdout_case(c):
    """(SAM text, args) of a tests/golden/stdout.json case (oracle/gen_golden_stdout.py)."""
    if "kat" in c:
        kat = {k["name"]: k for k in golden_io.load("kat")}
        return kat[c["kat"]]["sam"], c["args"]
    n = c["progress_lines"]
    head = "@HD\tVN:1.0\tSO:unsorted\n@SQ\tSN:g\tLN:200\n"
    mapped = "r\t0\tg\t11\t60\t20M\t*\t0\t0\t" + "ACGT" * 5 + "\t*\n"
    unmapped = "u\t4\t*\t0\t0\t*\t*\t0\t0\tACGT\t*\n"
    return head + "".join(mapped if k % 1000 == 0 else unmapped for k in range(n)), c["args"]


def test_read_pass_stdout_matches_reference_capture():
    """The lines the CLI prints from the read pass (header count, progress counter, totals:
    :143, :182, :194, :224-227) equal the reference's captured stdout (tests/golden/stdout.json,
    the reference run by oracle/gen_golden_stdout.py), failing read passes included (the
    reference's lines up to the raise); the device part of the run is covered by
    test_gpu.py::test_cli_stdout_matches_reference."""
    from sam2consensus_amd.batch import Parser
    from sam2consensus_amd.cli import REF_ERRORS, _log_failed_parse, _log_summary
    for c in golden_io.load("stdout"):
        sam, args = _stdout_case(c)
        out = []
        log = lambda s: out.append(s + "\n")  # noqa: E731 - print()
        p = Parser("-d" not in args, 150)
        failed = False
        try:
            p.feed(sam.encode("latin-1"))
            hb = p.finish()
            _log_summary(log, hb.info)
            hb.free()
        except REF_ERRORS:
            _log_failed_parse(log, p)
            failed = True
        finally:
            p.close()
        want = c["stdout"][len("\nProcessing file in.sam:\n\n"):]
        if failed:
            assert "".join(out) == want, (c.get("kat"), "".join(out), want)
        else:
            assert want.startswith("".join(out)), (c.get("kat"), "".join(out), want)


# ---------------------------------------------------------------- seqout of 2^24+ positions
def test_long_skip_parses_into_long_pieces():
    """A 16.7 Mb CIGAR N skip (seqout ≥ 2^24 positions, legal SAM) parses (the limit is 2^27,
    include/s2c.h S2C_RUN_KSHIFT) into a long piece listed by every tile it spans; its device
    run is checked against the reference's files by test_gpu.py::test_long_skip_on_device_*
    (the numpy model takes ~40 s on it)."""
    c = golden_io.load("longskip")[0]
    hb = batch.parse_text(c["sam"], False, 150)
    try:
        bm.check_plan(hb)
        assert hb.info.n_long > 0 and len(hb.lp) >= (1 << 24) // 2048
        assert hb.info.total_len == (1 << 24) + 64
    finally:
        hb.free()


def test_gather_bodies_concatenates_blocks():
    """s2c_gather_bodies (FASTA body assembly, engine.Workspace.fetch): blocks of a raw
    buffer concatenated in order, any lengths, large outputs on the host threads."""
    import ctypes as C
    rng = np.random.default_rng(7)
    raw = rng.integers(0, 256, size=1 << 22, dtype=np.uint8)
    for n in (0, 1, 7, 5000):
        lens = rng.integers(0, 2000, size=n).astype(np.int64)
        starts = np.array([rng.integers(0, raw.size - L) for L in lens], dtype=np.int64).reshape(-1)
        want = b"".join(raw[s:s + L].tobytes() for s, L in zip(starts, lens))
        out = bytearray(max(len(want), 1))
        buf = (C.c_char * len(out)).from_buffer(out)
        _lib.check(_lib.lib.s2c_gather_bodies(raw.ctypes.data, raw.nbytes, starts.ctypes.data, lens.ctypes.data, n,
                                              C.addressof(buf)))
        assert bytes(out[:len(want)]) == want
    zl = np.zeros(3, dtype=np.int64)   # every block empty (e.g. all of a reference's tiles filtered): no output
    _lib.check(_lib.lib.s2c_gather_bodies(None, 0, zl.ctypes.data, zl.ctypes.data, 3, None))
    bad = np.array([-1], dtype=np.int64)
    with pytest.raises(_lib.S2CError):
        _lib.check(_lib.lib.s2c_gather_bodies(raw.ctypes.data, raw.nbytes, bad.ctypes.data, bad.ctypes.data, 1,
                                              raw.ctypes.data))
    # a block past the end of the device output (a length from a faulty kernel): refused
    st, ln = np.array([raw.size - 10], dtype=np.int64), np.array([11], dtype=np.int64)
    dst = np.zeros(16, dtype=np.uint8)
    with pytest.raises(_lib.S2CError):
        _lib.check(_lib.lib.s2c_gather_bodies(raw.ctypes.data, raw.nbytes, st.ctypes.data, ln.ctypes.data, 1,
                                              dst.ctypes.data))


def test_copy_bytes_matches_memcpy():
    """s2c_copy_bytes (engine.Uploader's staging copy into its pinned ring): any length, any
    alignment, split over the host threads, byte-identical to a plain copy."""
    rng = np.random.default_rng(11)
    src = rng.integers(0, 256, size=(1 << 23) + 77, dtype=np.uint8)
    for n, a, b in ((0, 0, 0), (1, 3, 5), (4097, 1, 0), ((1 << 21) + 13, 7, 3), (src.size - 9, 9, 0)):
        dst = np.zeros(n + 16, dtype=np.uint8)
        _lib.check(_lib.lib.s2c_copy_bytes(dst.ctypes.data + b, src.ctypes.data + a, n))
        assert np.array_equal(dst[b:b + n], src[a:a + n])
        assert not dst[:b].any() and not dst[b + n:].any()
    with pytest.raises(_lib.S2CError):
        _lib.check(_lib.lib.s2c_copy_bytes(None, src.ctypes.data, 5))


def test_layers_without_dense_tiles():
    """s2c_batch_layers_mode(b, 0) (DeviceBatch's default: the pileup reads dense windows in
    place): dense tiles get S2C_LY_NONE and no layered copies, every other tile the layers of
    the full build; mode 1 afterwards rebuilds them all (batch_model.check_layers)."""
    import batch_model
    from sam2consensus_amd import configs
    LY_NONE = 0xFFFFFFFE
    full = configs.synth_batch("c5", ref_len=200_000, ins_frac=0.01)
    full.ensure_layers(dense=True)
    hb = configs.synth_batch("c5", ref_len=200_000, ins_frac=0.01)
    hb.ensure_layers()
    i = hb.info
    dense = (hb.tiles[:, 3] & 4) != 0
    assert 0 < dense.sum() < i.n_tiles and i.layers_dense == 0
    assert (hb.tiles[dense, 20] == LY_NONE).all() and not (hb.tiles[~dense, 20] == LY_NONE).any()
    assert i.n_lpieces < full.info.n_lpieces
    for t in np.nonzero(~dense)[0]:   # the same layers, renumbered past the dense tiles'
        r, f = hb.tiles[t], full.tiles[t]
        if f[20] == 0xFFFFFFFF:
            assert r[20] == f[20]
            continue
        for l in range(int(f[19])):
            a, b = hb.lly[r[20] + l:r[20] + l + 2, 0], full.lly[f[20] + l:f[20] + l + 2, 0]
            assert a[1] - a[0] == b[1] - b[0]
            assert (hb.lpc[a[0]:a[1], [0, 3]] == full.lpc[b[0]:b[1], [0, 3]]).all()
    hb.ensure_layers(dense=True)
    assert hb.info.layers_dense == 1 and hb.info.n_lpieces == full.info.n_lpieces
    assert (hb.tiles[:, 20] == full.tiles[:, 20]).all()
    batch_model.check_layers(hb)


def test_xfew_lists_the_n_offsets():
    """S2C_PF_XFEW + px (ABI 10; the layered copies carry it too, ABI 11): a read whose SEQ holds one or two 'N' (and no '-') lists their
    SEQ offsets, so the dense kernel adds its 'N' counts through the runs without scanning the
    non-ACGT plane; three non-ACGT chars, or any '-', leave the flag off (the plane scan)."""
    from sam2consensus_amd import _lib as L
    seqs = ["ACGTACGTAC", "ACGNACGTAC", "NCGTACGTAN", "NCGNACGTAN", "AC-TACGTAC", "NC-TACGTAC"]
    long_n = "A" * 70 + "N" + "C" * 59   # an 'N' past the first 64 bases
    sam = "@SQ\tSN:g\tLN:400\n" + "".join(
        "r%d\t0\tg\t%d\t60\t%dM\t*\t0\t0\t%s\t*\n" % (i, 1 + i, len(s), s) for i, s in enumerate(seqs + [long_n]))
    hb = batch.parse_text(sam, True, 150)
    try:
        fl = (hb.pc[:-1, 3] >> 24).astype(np.int64)
        order = np.argsort(hb.pc[:-1, 0], kind="stable")   # pieces by start position = read order here
        want = {0: None, 1: (3,), 2: (0, 9), 3: None, 4: None, 5: None, 6: (70,)}
        for r, k in enumerate(order):
            if want[r] is None:
                assert not fl[k] & L.S2C_PF_XFEW, (r, fl[k])
                continue
            assert fl[k] & L.S2C_PF_XFEW and fl[k] & L.S2C_PF_X
            px = int(hb.px[k])
            offs = tuple(o for o in (px & 0xFFFF, px >> 16) if o != 0xFFFF)
            assert offs == want[r], (r, hex(px))
    finally:
        hb.free()


def test_layered_pieces_carry_their_px():
    """s2c_batch_arrays.lpx (ABI 11): every layered copy of a piece carries the piece's px, so
    k_tile adds the 'N' of S2C_PF_XFEW pieces from the listed offsets (no plane scan): a copy's
    (gpos, flags | len, px) is one of the originals', and px is 0xFFFFFFFF exactly when the copy
    is not flagged."""
    from sam2consensus_amd import _lib as L
    hb = configs.synth_batch("c2", scale=0.05)
    try:
        hb.ensure_layers(False)
        assert hb.info.n_lpieces > 0
        n = int(hb.info.n_lpieces)
        lp = hb.lpc[:n]
        lpx = hb.lpx[:n]
        flagged = ((lp[:, 3] >> 24) & L.S2C_PF_XFEW) != 0
        assert flagged.any() and (~flagged).any()
        assert (lpx[~flagged] == 0xFFFFFFFF).all() and (lpx[flagged] != 0xFFFFFFFF).all()
        orig = set(zip(hb.pc[:-1, 0].tolist(), hb.pc[:-1, 3].tolist(), hb.px[: int(hb.info.n_pieces)].tolist()))
        assert set(zip(lp[:, 0].tolist(), lp[:, 3].tolist(), lpx.tolist())) <= orig
    finally:
        hb.free()


def _host_dev(hb, fill=b"-", counts=False):
    """An s2c_dev over host pointers (never dereferenced: the calls below must return before
    any launch) with the batch's shapes, as a caller of the C-ABI would fill it."""
    import ctypes as C
    L = _lib
    i = hb.info
    scratch = (C.c_uint8 * 4096)()
    p = C.addressof(scratch)
    d = L.Dev()
    for name in ("pc", "ops", "bq", "bx", "rs", "tiles", "items", "dense", "deep", "lp", "wtile", "rlist", "ps", "px",
                 "dwin", "lly", "lpc", "lops", "lbq", "lbx", "lpx", "dpc"):
        setattr(d, name, p)
    d.n_pieces, d.n_ops, d.n_qwords, d.n_tiles = i.n_pieces, i.n_ops, i.n_qwords, i.n_tiles
    d.n_items, d.n_dense, d.n_deep = i.n_items, i.n_dense, i.n_deep
    d.padded_len, d.chunk, d.kwin, d.tile_max = i.padded_len, i.chunk, i.kwin, i.tile_max
    d.dense_lds, d.n_rlist = i.dense_lds, i.n_rlist
    d.layers_dense, d.layers_built = i.layers_dense, i.layers_built
    d.word_lo, d.word_hi = i.word_lo, i.word_hi
    d.walk_queue, d.tile_events, d.n_rlist_run = i.walk_queue, i.tile_events, i.n_rlist_run
    d.maxdel_active, d.maxdel = 1, 150
    d.thresholds, d.n_thr, d.min_depth = p, 1, 1
    d.fill_len, d.fill_nondash, d.fill = len(fill), sum(c != ord("-") for c in fill), p
    for name in ("runs", "ibkt", "ilong", "ilong_n", "ins_cols", "ins_chr", "tile_stats", "blk_len", "out"):
        setattr(d, name, p)
    d.counts = p if counts else None
    d.n_cols = i.n_cols
    d.out_cap = 1 << 40
    return d, scratch


def test_device_stages_refuse_unbuilt_layers_before_launch():
    """The guards added after round 3's GPU fault: s2c_pileup with a fill of length != 1, and
    the counts-only stages (s2c_pileup_counts, s2c_accumulate), refuse a batch whose dense
    tiles' layered windows are not built (S2C_ERR_ARG, before anything is launched — this runs
    without a GPU); so does any stage with work items on a batch whose layers were never built
    (a fresh shard: tile word 20 reset to S2C_LY_NONE, not the parent's layer numbers)."""
    import ctypes as C
    L = _lib
    sam = ("@SQ\tSN:g1\tLN:300\n@SQ\tSN:g2\tLN:300\n"
           + "".join("a%d\t0\tg1\t%d\t60\t50M\t*\t0\t0\t%s\t*\n" % (k, 1 + 5 * k, "ACGTA" * 10) for k in range(40))
           + "".join("b%d\t0\tg2\t%d\t60\t20M2I20M\t*\t0\t0\t%s\t*\n" % (k, 1 + 5 * k, "ACGTG" * 8 + "AC")
                     for k in range(40)))
    hb = batch.parse_text(sam, True, 150)
    try:
        hb.ensure_layers()   # DeviceBatch's default: no dense layers
        i = hb.info
        assert i.n_dense > 0 and i.n_items > 0 and i.layers_built == 1 and i.layers_dense == 0
        d, keep = _host_dev(hb, fill=b"NN")
        assert L.lib.s2c_pileup(C.byref(d), None) == L.S2C_ERR_ARG
        assert "layered" in L.last_error()
        d, keep = _host_dev(hb, counts=True)
        assert L.lib.s2c_pileup_counts(C.byref(d), None) == L.S2C_ERR_ARG
        assert L.lib.s2c_accumulate(C.byref(d), 0, None) == L.S2C_ERR_ARG
        d, keep = _host_dev(hb)
        d.layers_built = 0
        for f in (L.lib.s2c_pileup, L.lib.s2c_run):
            assert f(C.byref(d), None) == L.S2C_ERR_ARG
            assert "not built" in L.last_error()
        sh = C.c_void_p()
        L.check(L.lib.s2c_batch_shard(hb._b, 0, i.n_tiles, C.byref(sh)))
        sb = batch.HostBatch(sh)
        try:
            assert sb.info.layers_built == 0 and sb.info.layers_dense == 0
            assert (sb.tiles[:, 20] == 0xFFFFFFFE).all()
            d, keep = _host_dev(sb)
            assert L.lib.s2c_run(C.byref(d), None) == L.S2C_ERR_ARG
            sb.ensure_layers()
            assert sb.info.layers_built == 1
        finally:
            sb.free()
    finally:
        hb.free()


def test_dense_windows_mirror_tile_records():
    """s2c_batch_arrays.dwin (ABI 10): each dense item's window words are its tile record's
    (k_tile_dense's one scalar load per tile), in a batch and in its shards."""
    from sam2consensus_amd import shard
    hb = configs.synth_batch("c5", ref_len=200_000, ins_frac=0.01)
    try:
        for b in [hb] + [shard.sub_batch(hb, r, 3) for r in range(3)]:
            i = b.info
            assert b.dwin.shape == (i.n_dense, 16) and i.n_dense > 0
            t = b.dense[:, 0].astype(np.int64)
            assert (b.dwin[:, 0] == t).all()
            assert (b.dwin[:, 1:12] == b.tiles[t][:, [0, 1, 8, 10, 11, 13, 14, 15, 16, 17, 18]]).all()
            # word 12: the first compact record of the window (ABI 12), records in window order
            npw = (b.dwin[:, 7] - b.dwin[:, 6]).astype(np.int64)
            assert (b.dwin[:, 12].astype(np.int64) == np.concatenate([[0], np.cumsum(npw)[:-1]])).all()
            assert i.n_dpc == npw.sum() and b.dpc.shape == (i.n_dpc, 3)
            assert not b.dwin[:, 13:].any()
            _check_dpc(b)
            if b is not hb:
                b.free()
    finally:
        hb.free()


def _check_dpc(b):
    """Every compact piece record (s2c.h S2C_DPC_WORDS) decodes to its piece's record, px and
    op slot count, relative to its window."""
    pc = b.pc.astype(np.int64)
    for w in b.dwin.astype(np.int64):
        k = np.arange(w[6], w[7])
        r = b.dpc[w[12]:w[12] + len(k)].astype(np.int64)
        T0 = 32 * (w[1] >> 5)
        assert ((r[:, 0] & 0xFFF) == pc[k, 0] - T0 + 2048).all()
        assert (((r[:, 0] >> 12) & 0x1FFF) == pc[k, 1] - 2 * w[10]).all()
        assert ((r[:, 0] >> 25) == pc[k + 1, 2] - pc[k, 2]).all()
        assert ((r[:, 1] & 0x1FFF) == pc[k, 2] - w[8]).all()
        assert (((r[:, 1] >> 13) & 0x7FF) == (pc[k, 3] & 0xFFFFFF)).all()
        assert ((r[:, 1] >> 24) == pc[k, 3] >> 24).all()
        assert (r[:, 2] == b.px[k]).all()


def test_dense_needs_compact_records():
    """A window holding a piece the compact record cannot hold (len(SEQ) > 2047) is not dense;
    the other tiles of the batch still are."""
    sam = "@SQ\tSN:g\tLN:20000\n"
    for s in range(1, 19000, 5):
        sam += "r\t0\tg\t%d\t60\t100M\t*\t0\t0\t%s\t*\n" % (s, "ACGTA" * 20)
    sam += "x\t0\tg\t15000\t60\t3S60M\t*\t0\t0\t%s\t*\n" % ("C" * 2100)   # len(SEQ) 2100 (not one token)
    hb = batch.parse_text(sam, False, 150)
    try:
        t = hb.tiles
        dense = (t[:, 3] & 4) != 0
        assert dense.any() and not dense.all()
        a, e = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
        bad = (a <= 15000 + 32 * int(hb.info.kwin) + 32) & (e > 14999 - 32)
        assert not (dense & bad).any()
        _check_dpc(hb)
    finally:
        hb.free()


def test_host_code_under_sanitizers(tmp_path):
    """The host library's parse / plan / streaming paths (s2c_host.cpp) built with AddressSanitizer
    and UndefinedBehaviorSanitizer (host code only: no GPU code is sanitized) and driven by
    tests/native/*_drive.cpp over plain and BGZF inputs, 1 and 4 parse threads: clean."""
    import shutil
    if not shutil.which("g++"):
        pytest.skip("g++ not found")
    src = os.path.join(ROOT, "sam2consensus_amd", "csrc", "s2c_host.cpp")
    san = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"]
    obj = str(tmp_path / "host.o")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-I" + os.path.join(ROOT, "include")] + san + ["-c", src, "-o", obj],
                   check=True, timeout=600)
    exe = {}
    for name in ("parse_drive", "stream_drive"):
        exe[name] = str(tmp_path / name)
        subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-I" + os.path.join(ROOT, "include")] + san +
                       [os.path.join(ROOT, "tests", "native", name + ".cpp"), obj, "-o", exe[name], "-lz", "-lpthread"],
                       check=True, timeout=300)
    inputs = {"c2": str(tmp_path / "c2.sam"), "c3": str(tmp_path / "c3.sam.gz"), "c5": str(tmp_path / "c5.sam")}
    configs.synth_write("c2", inputs["c2"], scale=0.05)
    configs.synth_write("c3", inputs["c3"], scale=0.005)
    configs.synth_write("c5", inputs["c5"], scale=0.01)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    runs = [("parse_drive", inputs[w], t) for w in inputs for t in ("1", "4")] + [("stream_drive", inputs["c5"], "4")]
    for name, path, threads in runs:
        r = subprocess.run([exe[name], path], capture_output=True, text=True, timeout=600,
                           env=dict(env, S2C_PARSE_THREADS=threads))
        out = r.stdout + r.stderr
        assert r.returncode == 0 and "rc 0" in r.stdout, (name, path, threads, out[-3000:])
        assert "runtime error" not in out and "AddressSanitizer" not in out, out[-3000:]


def test_graft_build_entry():
    """__graft_entry__.build() (the driver's build check): make in-tree, import, ABI check."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("graft_entry", os.path.join(ROOT, "__graft_entry__.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    m.build()


def test_cli_path_imports_no_torch_and_one_hip_runtime():
    """The one-process CLI's modules import no PyTorch (`import torch` is 1.8 s on the box);
    libs2c.so is bound to the HIP runtime torch bundles, so a process that imports torch after
    it still maps one libamdhip64 (two runtimes fail our launches with hipErrorNoDevice)."""
    import subprocess
    import sys
    code = ("import sys\nimport sam2consensus_amd.cli, sam2consensus_amd.hiprun, sam2consensus_amd.records\n"
            "print('torch' in sys.modules)\nimport torch\n"
            "print(len(set(l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l)))\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT, timeout=300)
    assert r.returncode == 0, r.stderr[-1000:]
    assert r.stdout.split() == ["False", "1"], r.stdout


def test_cli_without_a_gpu_fails_loudly(tmp_path):
    """No CPU fallback: on a host without a GPU (this tier) the CLI raises from the HIP runtime
    and writes no FASTA file."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from sam2consensus_amd.cli import main
    p = tmp_path / "a.sam"
    p.write_text("@SQ\tSN:r\tLN:40\nq\t0\tr\t1\t60\t10M\t*\t0\t0\tACGTACGTAC\t*\n")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        main(["-i", str(p), "-o", str(tmp_path / "out")])
    assert not any(f.endswith(".fasta") for f in os.listdir(tmp_path / "out"))


def test_cli_upload_reservation_estimate(tmp_path):
    """The whole-file CLI's warm-up reservation (cli.upload_estimate): nothing below 64 MB of
    input or for a missing file (the parser raises the reference's error), 0.6 × a plain file,
    2.4 × a gzip one — above the packed batch of each (C5: 0.42 × its .sam)."""
    from sam2consensus_amd import cli
    assert cli.upload_estimate(str(tmp_path / "missing.sam")) == 0
    small = tmp_path / "s.sam"
    small.write_bytes(b"@HD\tVN:1.0\n")
    assert cli.upload_estimate(str(small)) == 0
    for name, f in (("big.sam", 0.6), ("big.sam.gz", 2.4)):
        p = tmp_path / name
        with open(p, "wb") as fh:
            fh.truncate(100 << 20)   # (sparse: no 100 MB written)
        assert cli.upload_estimate(str(p)) == int((100 << 20) * f)


def test_host_batch_release_on_a_side_thread():
    """HostBatch.free_async detaches the handle before its thread frees it: free() and the
    destructor after it are no-ops (no double free), and a second call returns None."""
    from sam2consensus_amd.batch import parse_text
    sam = "@SQ\tSN:r\tLN:40\nq\t0\tr\t1\t60\t10M\t*\t0\t0\tACGTACGTAC\t*\n"
    hb = parse_text(sam, True, 150)
    th = hb.free_async()
    assert th is not None
    th.join()
    assert hb.free_async() is None
    hb.free()
    del hb


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_bench_launches_ranks_as_child(monkeypatch, capsys):
    """bench.py --gpus N without WORLD_SIZE (how the driver runs it): torch.distributed.run is
    started as a child process (N ranks on 127.0.0.1), every line the ranks print goes to
    stderr except rank 0's JSON line, which is the parent's one stdout line; the parent exits
    with the child's status."""
    import sys
    m = _bench_module()
    cmd = m.rank_command(8, ["--gpus", "8", "--steps", "3"], 29555)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8" and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5].endswith("bench.py")
    script = ("import sys\nprint('rank noise')\nprint('{\"metric\": \"m\", \"value\": 1}')\n"
              "print('more', file=sys.stderr)\nsys.exit(%d)\n")
    for rc in (0, 3):
        monkeypatch.setattr(m, "rank_command", lambda n, argv, port, rc=rc: [sys.executable, "-c", script % rc])
        assert m.spawn_ranks(2, []) == rc
        out = capsys.readouterr()
        assert out.out == '{"metric": "m", "value": 1}\n'
        assert "rank noise" in out.err
    monkeypatch.setattr(m, "rank_command", lambda n, argv, port: [sys.executable, "-c", "print('no line')"])
    assert m.spawn_ranks(2, []) == 1   # (no result line: a failure even when every rank exits 0)


def test_bench_refuses_world_size_mismatch():
    """--gpus N must equal the launched world size (a mismatched torchrun would otherwise
    report the wrong n_gpus): exit 2 before anything imports torch."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True, text=True,
                       env=dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), timeout=60)
    assert r.returncode == 2 and "--gpus 2 but WORLD_SIZE 1" in r.stderr
