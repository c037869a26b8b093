"""GPU tier: the HIP path (libs2c.so kernels on an MI355X) vs the reference's golden
outputs and the oracle.  Run in ONE process: `pytest tests -m gpu`.

Parity bar: byte-identical FASTA files (integer counting end to end) and identical
exception class on failing inputs."""
import hashlib
import os
import tempfile

import numpy as np
import pytest

import batch_model as bm
import golden_io
import s2c_oracle as o

pytestmark = pytest.mark.gpu

CASES = golden_io.cases()
CONFIGS = golden_io.load("configs")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    assert torch.cuda.is_available(), "gpu tier needs a ROCm GPU (no CPU fallback exists)"
    yield


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_hip_path_matches_reference(case):
    from sam2consensus_amd.cli import run_text
    status, files = run_text(case["sam"], case["args"])
    assert status == case["status"]
    assert files == case["files"], sorted(files)


def _ws(hb, thresholds, min_depth=1, fill=b"-", keep_counts=False):
    from sam2consensus_amd.engine import DeviceBatch, Workspace, needs_dense_layers
    db = DeviceBatch(hb, dense_layers=needs_dense_layers(fill, keep_counts))
    return Workspace(db, thresholds, min_depth, fill, keep_counts)


@pytest.mark.parametrize("name,over", [("c1", {}), ("c2", {"n_refs": 18}), ("c5", {"ref_len": 400_000}),
                                       ("c5nd", {"ref_len": 400_000, "long_del_frac": 0.05}),
                                       ("c4", {"ref_len": 2000, "depth": 12000.0}),
                                       ("c4u", {"ref_len": 2000, "depth": 12000.0})])
def test_runs_and_counts_equal_batch_model(name, over):
    """k_reads' run records and the tile kernels' counts == the CPU restatement."""
    from sam2consensus_amd import configs
    hb = configs.synth_batch(name, **over)
    ws = _ws(hb, [0.25], keep_counts=True)
    got = ws.pileup_counts().astype(np.int64)
    runs, _ = bm.model_reads(hb)
    dev_runs = ws.runs[: 16 * hb.info.n_ops].view(torch_i32()).cpu().numpy().view(np.uint32).reshape(-1, 4)
    assert (dev_runs == runs[: hb.info.n_ops]).all()
    want = bm.model_counts(hb, runs)
    for r in range(hb.info.n_refs):
        a, L = int(hb.ref_off[r]), int(hb.ref_len[r])
        assert (got[:, a:a + L] == want[:, a:a + L]).all(), hb.names[r]
    if name.startswith("c4"):
        assert (hb.tiles[:, 3] & 1 == 1).any(), "deep config must exercise chunked (atomic) tiles"
    if name.startswith("c5"):
        assert hb.info.n_dense > 0


def torch_i32():
    import torch
    return torch.int32


def _first_diff(a, b):
    """Short description of the first differing byte (pytest's own diff of MB-sized bytes
    objects takes minutes)."""
    n = min(len(a), len(b))
    i = next((k for k in range(n) if a[k] != b[k]), n)
    return "lengths %d / %d, first difference at byte %d: %r vs %r" % (len(a), len(b), i, a[i:i + 16], b[i:i + 16])


def _sha_files(files):
    return {k.decode("latin-1"): hashlib.sha256(v).hexdigest() for k, v in files.items()}


@pytest.mark.parametrize("name", ["c1", "c2", "c4", "c4u", "c5", "c5nd", "c3"])
def test_config_fasta_byte_identical_to_reference(name):
    """Full-size BASELINE configs: every FASTA file's sha256 equals the reference's."""
    if name not in CONFIGS:
        pytest.skip("golden for %s not generated yet (oracle/gen_golden_configs.py)" % name)
    from sam2consensus_amd import configs
    from sam2consensus_amd.cli import consensus_batch
    g = CONFIGS[name]
    args = g["args"]
    opt = o.parse_argv(["-i", g["sam_file"]] + args)
    if name == "c3" and os.environ.get("S2C_TEST_C3_GZ", "1") != "0":   # the 2.3 GB BGZF .sam.gz through the product parser
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, g["sam_file"])
            configs.synth_write(name, p)
            from sam2consensus_amd.batch import parse_file
            hb = parse_file(p, opt.maxdel_active, 150)
    else:
        hb = configs.synth_batch(name)
    assert hb.info.reads_mapped == g["n_reads"]
    files = consensus_batch(hb, opt.thresholds, opt.prefix.encode(), opt.min_depth, opt.fill.encode(), opt.n)
    got = _sha_files(files)
    want = {k: v["sha256"] for k, v in g["files"].items()}
    assert got == want
    # size-independent property: Σ counts == counted aligned bases (no maxdel drops here)
    if name in ("c1", "c2", "c5", "c5nd"):
        ws = _ws(hb, opt.thresholds, keep_counts=True)
        cnt = ws.pileup_counts()
        tot = 0
        for r in range(hb.info.n_refs):
            a, L = int(hb.ref_off[r]), int(hb.ref_len[r])
            tot += int(cnt[:, a:a + L].astype(np.int64).sum())
        if name != "c5nd":   # c5nd drops the '-' of its long-deletion reads (:210)
            assert tot == hb.info.aligned_bases
        else:
            assert tot < hb.info.aligned_bases


def test_c3_samgz_bgzf_reduced_matches_oracle(tmp_path):
    """C3's record order and compression at 1/20 scale (250 kb x 1000x, 1.67 M reads): the
    .sam.gz is BGZF, so the CLI's parser inflates it block-parallel; the FASTA equals the C
    restatement's on the same file (the full-size golden: test_config_fasta_..., c3)."""
    import subprocess
    from sam2consensus_amd import configs
    from sam2consensus_amd.cli import main
    gz = str(tmp_path / "c3r.sam.gz")
    configs.synth_write("c3", gz, scale=0.05)
    with open(gz, "rb") as fh:
        h = fh.read(18)
    assert h[:4] == b"\x1f\x8b\x08\x04" and h[12:14] == b"BC", "expected a BGZF member"
    args = configs.cli_args("c3")
    out = tmp_path / "out"
    assert main(["-i", gz, "-o", str(out), "-p", "c3r"] + args) == 0
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(root, "oracle")], check=True)
    ref = tmp_path / "ref"
    r = subprocess.run([os.path.join(root, "oracle", "build", "s2c_oracle_mc"), "16", "-i", gz, "-o", str(ref),
                        "-p", "c3r"] + args, capture_output=True, text=True, timeout=300)
    assert "status: ok" in r.stdout, r.stdout[-500:]
    assert sorted(os.listdir(out)) == sorted(os.listdir(ref))
    for fn in os.listdir(ref):
        assert open(os.path.join(out, fn), "rb").read() == open(os.path.join(ref, fn), "rb").read()


@pytest.mark.parametrize("wl,scale,args", [
    ("c5", 0.05, ["-c", "0.1,0.5,0.9"]),
    ("c5", 0.05, ["-c", "0.25", "-m", "5", "-f", "N", "-n", "60"]),
    ("c5", 0.05, ["-c", "0.75", "-d", "3"]),
    ("c4", 0.02, ["-c", "0.2,0.6", "-m", "20"]),
    ("c5", 0.05, ["-c", "0.5"]),
    ("c2", 0.1, ["-c", "0.3,0.51,0.99", "-n", "70"]),
    ("c2", 0.1, ["-c", "0.3,0.51", "-n", "70"]),
], ids=["c5-3thr", "c5-m5-fN-n60", "c5-d3", "c4-m20", "c5-c50", "c2-3thr-n70", "c2-2thr-n70"])
def test_cli_options_match_c_restatement(tmp_path, wl, scale, args):
    """The CLI (HIP path) on reduced BASELINE configs under option sets their goldens do not
    use, against the C restatement (oracle/s2c_oracle_mc.c, itself pinned to the reference's
    outputs in test_oracle.py) on the same file: every FASTA byte-identical, or the same error
    (C5 with a 0.1 threshold reaches base sets the reference's IUPAC table lacks: KeyError)."""
    import subprocess
    from sam2consensus_amd import configs
    from sam2consensus_amd.cli import main
    sam = str(tmp_path / ("%s.sam" % wl))
    configs.synth_write(wl, sam, scale=scale)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(root, "oracle")], check=True)
    ref = tmp_path / "ref"
    r = subprocess.run([os.path.join(root, "oracle", "build", "s2c_oracle_mc"), "16", "-i", sam, "-o", str(ref),
                        "-p", wl] + args, capture_output=True, text=True, timeout=300)
    status = [ln for ln in r.stdout.splitlines() if ln.startswith("status: ")][-1][len("status: "):]
    out = tmp_path / "out"
    try:
        rc = main(["-i", sam, "-o", str(out), "-p", wl] + args)
        got = "ok" if rc == 0 else "rc %d" % rc
    except (KeyError, IndexError, ValueError, ZeroDivisionError, OverflowError) as e:
        got = type(e).__name__
    assert got == status, (got, status)   # (the reference's error where it raises one)
    if status != "ok":
        return
    assert sorted(os.listdir(out)) == sorted(os.listdir(ref)) and os.listdir(ref)
    for fn in os.listdir(ref):
        a, b = open(os.path.join(out, fn), "rb").read(), open(os.path.join(ref, fn), "rb").read()
        assert a == b, (fn, _first_diff(a, b))


def test_cli_end_to_end_c1(tmp_path):
    from sam2consensus_amd import configs
    from sam2consensus_amd.cli import main
    g = CONFIGS["c1"]
    sam = str(tmp_path / "c1.sam")
    configs.synth_write("c1", sam)
    out = tmp_path / "out"
    assert main(["-i", sam, "-o", str(out)] + g["args"]) == 0
    got = {fn: open(os.path.join(out, fn), "rb").read().decode("latin-1") for fn in os.listdir(out)}
    assert got == g["content"]


def test_cli_process_runs_without_torch(tmp_path):
    """The CLI process (sam2consensus.py, one GPU, whole file) never imports PyTorch — its
    device side is hiprun.py on the HIP runtime libs2c.so is bound to — and writes the
    reference's files: C1 against the golden content, a 5 %-scale C5 with -f N -n 60 -m 3
    against the C restatement (the lengths != 1 fill takes the dense tiles' layered path)."""
    import subprocess
    import sys
    from sam2consensus_amd import configs
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    run = ("import runpy, sys\n"
           "sys.argv = [%r] + sys.argv[1:]\n"
           "try:\n    runpy.run_path(%r, run_name='__main__')\n"
           "except SystemExit as e:\n    assert not e.code, e.code\n"
           "print('TORCH', 'torch' in sys.modules)\n") % (os.path.join(root, "sam2consensus.py"),
                                                         os.path.join(root, "sam2consensus.py"))
    g = CONFIGS["c1"]
    sam = str(tmp_path / "c1.sam")
    configs.synth_write("c1", sam)
    out = tmp_path / "out"
    r = subprocess.run([sys.executable, "-c", run, "-i", sam, "-o", str(out)] + g["args"], capture_output=True,
                       text=True, timeout=240, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "TORCH False" in r.stdout, r.stdout[-500:]
    got = {fn: open(os.path.join(out, fn), "rb").read().decode("latin-1") for fn in os.listdir(out)}
    assert got == g["content"]
    sam5 = str(tmp_path / "c5.sam")
    configs.synth_write("c5", sam5, scale=0.05)
    args = ["-c", "0.25,0.75", "-f", "N", "-n", "60", "-m", "3", "-p", "c5"]
    out5, ref5 = tmp_path / "out5", tmp_path / "ref5"
    r = subprocess.run([sys.executable, "-c", run, "-i", sam5, "-o", str(out5)] + args, capture_output=True,
                       text=True, timeout=240, cwd=root)
    assert r.returncode == 0 and "TORCH False" in r.stdout, r.stderr[-2000:]
    subprocess.run(["make", "-s", "-C", os.path.join(root, "oracle")], check=True)
    o = subprocess.run([os.path.join(root, "oracle", "build", "s2c_oracle_mc"), "16", "-i", sam5, "-o", str(ref5)] + args,
                       capture_output=True, text=True, timeout=300)
    assert "status: ok" in o.stdout, o.stdout[-500:]
    assert sorted(os.listdir(out5)) == sorted(os.listdir(ref5)) and os.listdir(ref5)
    for fn in os.listdir(ref5):
        assert open(os.path.join(out5, fn), "rb").read() == open(os.path.join(ref5, fn), "rb").read(), fn


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_exchange_at_world_one(tmp_path):
    """The multi-GPU exchange over RCCL with device tensors, on this box's one GPU: a 1-rank
    `nccl` process group with S2C_FORCE_COLLECTIVES=1, so the collectives that world size 1
    skips run anyway — dparse's all-reduces and all_to_all of the read blobs, shard.gather_results'
    reduce / all_gather / gather of the stats and bodies.  The merged C2 files == the reference's."""
    import json
    import subprocess
    import sys
    from sam2consensus_amd import configs
    g = CONFIGS["c2"]
    path = str(tmp_path / g["sam_file"])
    configs.synth_write("c2", path)
    opt = o.parse_argv(["-i", path] + g["args"])
    res = tmp_path / "sha.json"
    code = (
        "import hashlib, json, sys\n"
        "import torch.distributed as dist\n"
        "from sam2consensus_amd import cli\n"
        "files = cli.consensus_files_sharded(%r, %r, %r, %d, %r, %d, %r)\n"
        "assert not dist.is_initialized()\n"
        "json.dump({k.decode('latin-1'): hashlib.sha256(v).hexdigest() for k, v in files.items()}, open(%r, 'w'))\n"
        % (path, opt.thresholds, opt.prefix.encode(), opt.min_depth, opt.fill.encode(), opt.n, opt.maxdel_active,
           str(res)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), S2C_FORCE_COLLECTIVES="1", S2C_DIST_BACKEND="nccl",
               PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, timeout=240)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    assert json.load(open(res)) == {k: v["sha256"] for k, v in g["files"].items()}


def test_cli_torchrun_distributed_parse(tmp_path):
    """The multi-GPU CLI (2 ranks under torchrun, the file parsed once across them —
    sam2consensus_amd/dparse.py — each rank's tile range on the device, bodies gathered):
    C1 == the reference's files; a scaled C2 .sam.gz == the one-process CLI's files.  Both
    ranks share this box's one GPU, so the collectives run over gloo."""
    import subprocess
    import sys
    from sam2consensus_amd import configs
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, S2C_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")

    def torchrun(inp, out, args):
        # every rank's stdout / stderr kept in its own file (--log-dir, --redirects 3): a failing
        # rank's traceback is in the assertion, not only the launcher's summary
        logs = tmp_path / ("logs_" + os.path.basename(str(out)))
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               "--log-dir", str(logs), "--redirects", "3",
               os.path.join(root, "sam2consensus.py"), "-i", inp, "-o", str(out)] + args
        r = subprocess.run(cmd, env=env, capture_output=True, timeout=240)
        ranks = {}
        for dp, _, fns in os.walk(logs):
            for fn in fns:
                if fn in ("stdout.log", "stderr.log"):
                    rank = os.path.basename(dp)
                    ranks.setdefault(rank, {})[fn] = open(os.path.join(dp, fn), errors="replace").read()
        if r.returncode != 0:
            detail = "\n".join("rank %s %s:\n%s" % (k, f, v[-3000:]) for k, d in sorted(ranks.items())
                               for f, v in sorted(d.items()) if v.strip())
            raise AssertionError("torchrun exit %d\n%s\nlauncher:\n%s" % (r.returncode, detail,
                                                                           r.stderr.decode()[-1500:]))
        return "".join(d.get("stdout.log", "") for _, d in sorted(ranks.items())) + r.stdout.decode()

    g = CONFIGS["c1"]
    sam = str(tmp_path / "c1.sam")
    configs.synth_write("c1", sam)
    out = tmp_path / "o1"
    so = torchrun(sam, out, g["args"])
    got = {fn: open(os.path.join(out, fn), "rb").read().decode("latin-1") for fn in os.listdir(out)}
    assert got == g["content"]
    assert "reads processed." in so and "Done." in so
    from sam2consensus_amd.cli import main
    gz = str(tmp_path / "c2.sam.gz")
    configs.synth_write("c2", gz, scale=0.05)
    args = configs.cli_args("c2")
    o2, o1 = tmp_path / "o2", tmp_path / "o1p"
    torchrun(gz, o2, args)
    assert main(["-i", gz, "-o", str(o1)] + args) == 0
    assert sorted(os.listdir(o2)) == sorted(os.listdir(o1))
    for fn in os.listdir(o1):
        assert open(os.path.join(o2, fn), "rb").read() == open(os.path.join(o1, fn), "rb").read()


def test_cli_failure_writes_nothing(tmp_path):
    from sam2consensus_amd.cli import main
    p = tmp_path / "bad.sam"
    p.write_text("@SQ\tSN:g\tLN:5\nr\t0\tg\t1\t60\t5M\t*\t0\t0\tACGTA\t*\n")
    out = tmp_path / "o"
    with pytest.raises(KeyError):
        main(["-i", str(p), "-o", str(out), "-c", "0"])      # vote selects "" (:367)
    assert os.listdir(out) == []


@pytest.mark.parametrize("name,over", [("c2", {"scale": 0.03}), ("c4", {"ref_len": 2000, "depth": 12000.0})])
def test_repeated_runs_identical(name, over):
    """Workspace reuse (bench steps) gives identical bytes every time (no stale state): the
    insertion tables and (round 6) the deep tiles' HBM counts are left zero by every run —
    no zeroing launch before the next — also after the counts-only diagnostic filled them."""
    from sam2consensus_amd import configs
    hb = configs.synth_batch(name, **over)
    if name == "c4":
        assert hb.info.n_deep > 0, "the deep-tile path must run"
    ws = _ws(hb, [0.25, 0.5, 0.75], keep_counts=(name == "c4"))
    ws.run()
    a = ws.fetch()
    for k in range(3):
        if k == 1 and name == "c4":
            ws.pileup_counts()   # (fills the counts; the next run must not add to them)
        ws.run()
        b = ws.fetch()
        assert (a[0] == b[0]).all() and (a[1] == b[1]).all() and a[2] == b[2]
    if name == "c4":   # and the counts themselves are zero after a run
        assert int(np.count_nonzero(ws.counts_host())) == 0


@pytest.mark.parametrize("name,world", [("c1", 4), ("c2", 3), ("c5", 2), ("c3", 8), ("c4", 8)])
def test_sharded_on_device_matches_golden(name, world):
    """Tile-range shards (s2c_batch_shard) run through libs2c.so, merged == the reference.
    C3 and C4 split 8 ways as BASELINE.json runs them: deep and layered tiles cut by shard
    boundaries (each shard re-lays its pieces and layered windows)."""
    from sam2consensus_amd import configs, shard
    from sam2consensus_amd.engine import DeviceBatch, Workspace, needs_dense_layers
    g = CONFIGS[name]
    opt = o.parse_argv(["-i", g["sam_file"]] + g["args"])
    hb = configs.synth_batch(name)
    parts, stats = [], None
    for rank in range(world):
        sub = shard.sub_batch(hb, rank, world)
        ws = Workspace(DeviceBatch(sub, dense_layers=needs_dense_layers(opt.fill.encode())), opt.thresholds,
                       opt.min_depth, opt.fill.encode())
        ws.run()
        st, offs, out = ws.fetch()
        stats = st if stats is None else stats + st
        parts.append((sub.t0, sub.t1, offs, out))
    offs, out = shard.merge_outputs(parts, len(opt.thresholds))
    from sam2consensus_amd.records import build_records, render
    recs = build_records(hb, opt.thresholds, opt.prefix.encode(), stats, offs, out)
    got = {n + "__" + opt.prefix + ".fasta": hashlib.sha256(render(r, opt.n)).hexdigest() for n, r in recs.items()}
    assert got == {k: v["sha256"] for k, v in g["files"].items()}


@pytest.mark.parametrize("name,nbatch", [("c2", 8), ("c1", 5)])
def test_streamed_batches_on_device_match_golden(tmp_path, name, nbatch):
    """Coordinate-sorted SAM file fed in blocks, run as nbatch streamed tile ranges through
    libs2c.so (sam2consensus_amd/stream.py) == the reference's files."""
    from sam2consensus_amd import configs, stream
    from sam2consensus_amd.records import build_records, render
    g = CONFIGS[name]
    opt = o.parse_argv(["-i", g["sam_file"]] + g["args"])
    path = str(tmp_path / g["sam_file"])
    configs.synth_write(name, path)
    size = os.path.getsize(path)
    res = stream.stream_batches(stream.file_blocks(path, max(4096, size // (4 * nbatch))), opt.thresholds,
                                stream.device_runner(opt.thresholds, opt.min_depth, opt.fill.encode()),
                                opt.maxdel_active, 512, size // nbatch + 1)
    assert len(res.batches) >= nbatch - 1
    assert res.reads_mapped == g["n_reads"]
    recs = build_records(res.hb, opt.thresholds, opt.prefix.encode(), res.stats, res.offs, res.out)
    got = {n + "__" + opt.prefix + ".fasta": hashlib.sha256(render(r, opt.n)).hexdigest() for n, r in recs.items()}
    assert got == {k: v["sha256"] for k, v in g["files"].items()}


def test_cli_streamed_and_unsorted_fallback(tmp_path, monkeypatch):
    """S2C_STREAM turns on streamed batches in the CLI: C1 (sorted) streams; a shuffled
    .sam.gz (C3's record order, reduced, SO:unsorted) accumulates counts batch by batch, and so
    does the same text under a header claiming SO:coordinate, after the sorted pass detects it;
    all == the oracle."""
    from sam2consensus_amd import configs
    from sam2consensus_amd.cli import main
    monkeypatch.setenv("S2C_STREAM", "64K")
    g = CONFIGS["c1"]
    sam = str(tmp_path / "c1.sam")
    configs.synth_write("c1", sam)
    out = tmp_path / "out"
    assert main(["-i", sam, "-o", str(out)] + g["args"]) == 0
    got = {fn: open(os.path.join(out, fn), "rb").read().decode("latin-1") for fn in os.listdir(out)}
    assert got == g["content"]
    gz = str(tmp_path / "c3s.sam.gz")
    configs.synth_write("c3", gz, scale=0.004)
    out2 = tmp_path / "out2"
    assert main(["-i", gz, "-o", str(out2), "-m", "10", "-p", "c3s"]) == 0
    want, _ = o.run_path(gz, ["-m", "10", "-p", "c3s"])
    got = {fn: open(os.path.join(out2, fn), "rb").read().decode("latin-1") for fn in os.listdir(out2)}
    assert got == want
    # the same records under a header claiming SO:coordinate: the sorted pass runs, detects the
    # first read below an emitted tile (NotSorted) and the file is re-read in accumulation mode
    import gzip
    text = gzip.decompress(open(gz, "rb").read())
    assert text.startswith(b"@HD\tVN:1.6\tSO:unsorted\n")
    lie = str(tmp_path / "c3s_lie.sam")
    open(lie, "wb").write(text.replace(b"SO:unsorted", b"SO:coordinate", 1))
    out3 = tmp_path / "out3"
    assert main(["-i", lie, "-o", str(out3), "-m", "10", "-p", "c3s"]) == 0
    got = {fn: open(os.path.join(out3, fn), "rb").read().decode("latin-1") for fn in os.listdir(out3)}
    assert got == want


def test_unsorted_accumulation_on_device_kat():
    """Every KAT case through streamed batches of unsorted input on the device (counts added
    into HBM running totals, the last batch voted over them): the reference's bytes / class."""
    from sam2consensus_amd import stream
    from sam2consensus_amd.records import build_records, render
    for case in golden_io.load("kat"):
        opt = o.parse_argv(["-i", "in.sam"] + case["args"])
        data = case["sam"].encode("latin-1")
        blocks = (data[k:k + 29] for k in range(0, len(data), 29))
        try:
            res = stream.stream_unsorted(blocks, opt.thresholds,
                                         stream.DeviceAccumulator(opt.thresholds, opt.min_depth,
                                                                  opt.fill.encode("latin-1")),
                                         opt.maxdel_active, 60)
            recs = build_records(res.hb, opt.thresholds, opt.prefix, res.stats, res.offs, res.out)
            files = {n + "__" + opt.prefix + ".fasta": render(r, opt.n).decode("latin-1") for n, r in recs.items()}
        except (KeyError, IndexError, ValueError, ZeroDivisionError, OverflowError) as e:
            assert type(e).__name__ == case["status"], case["name"]
            continue
        assert case["status"] == "ok" and files == case["files"], case["name"]


@pytest.mark.parametrize("name,over,args", [
    ("c2", {"n_refs": 40, "shuffle": 1}, ["-c", "0.25,0.50,0.75"]),
    ("c5nd", {"ref_len": 300_000, "shuffle": 1, "long_del_frac": 0.05}, []),
    ("c4", {"ref_len": 3000, "depth": 10000.0, "shuffle": 1}, [])])
def test_unsorted_accumulation_on_device_configs(tmp_path, name, over, args):
    """Shuffled synthetic configs (insertions, maxdel drops, deep tiles) in 7+ streamed
    batches through s2c_accumulate == the oracle."""
    from sam2consensus_amd import configs, stream
    from sam2consensus_amd.records import build_records, render
    path = str(tmp_path / (name + ".sam"))
    configs.synth_write(name, path, **over)
    opt = o.parse_argv(["-i", path] + args)
    size = os.path.getsize(path)
    res = stream.stream_unsorted(stream.file_blocks(path, max(4096, size // 32)), opt.thresholds,
                                 stream.DeviceAccumulator(opt.thresholds, opt.min_depth, opt.fill.encode()),
                                 opt.maxdel_active, size // 7 + 1)
    assert len(res.batches) >= 7
    recs = build_records(res.hb, opt.thresholds, opt.prefix.encode(), res.stats, res.offs, res.out)
    got = {n + "__" + opt.prefix + ".fasta": render(r, opt.n).decode("latin-1") for n, r in recs.items()}
    want, _ = o.run_path(path, args)
    assert got == want


@pytest.mark.parametrize("name,over,thr,md,fill", [
    ("c2", {"n_refs": 6}, [0.25, 0.5, 0.75], 1, b"-"),
    # long insertions: > 1024 insertion columns in a tile → the HBM column path
    ("c2", {"n_refs": 2, "depth": 60.0, "ins_frac": 0.6, "ins_max": 60}, [0.1, 0.5], 1, b"-"),
    # deep tiles (several work items) with insertions: k_prep + k_consensus epilogue
    ("c2", {"n_refs": 1, "ref_len": 700, "depth": 9000.0, "ins_frac": 0.05, "ins_max": 6}, [0.25, 0.75], 1, b"-"),
    # 6 thresholds (two passes of 4), min depth with uncalled positions, a 100-byte fill (HBM)
    ("c2", {"n_refs": 3, "depth": 30.0}, [0.1, 0.3, 0.5, 0.6, 0.8, 0.95], 25, b"Nn" * 50),
    # empty fill: uncalled positions write nothing
    ("c2", {"n_refs": 2, "depth": 30.0}, [0.5], 25, b""),
    # thresholds outside (0, inf): the max-count shortcut is off, every vote in full
    ("c2", {"n_refs": 2, "depth": 40.0}, [0.0, 0.5, 1.0, 2.0], 1, b"-"),
    ("c2", {"n_refs": 2, "depth": 40.0}, [-0.5, float("inf"), 0.25], 1, b"?"),
    # the longest -f kept in LDS and one byte more (HBM)
    ("c2", {"n_refs": 2, "depth": 20.0}, [0.3, 0.7], 18, b"x" * 64),
    ("c2", {"n_refs": 2, "depth": 20.0}, [0.3, 0.7], 18, b"y" * 65),
    # low depth: ties and split votes everywhere (full closed form), 1-5 thresholds
    ("c2", {"n_refs": 4, "depth": 3.0}, [0.2, 0.4, 0.6, 0.8, 1.0], 1, b"N"),
    # many '-'/'N' entries per work item (> 1024: past the register prefetch, from HBM)
    ("c2", {"n_refs": 2, "del_frac": 0.6, "del_max": 8, "n_rate": 0.05}, [0.25, 0.5], 1, b"-"),
])
def test_device_pipeline_equals_batch_model(name, over, thr, md, fill):
    """stats / block offsets / bytes of the HIP stages == the batch model (tests/batch_model.py)."""
    from sam2consensus_amd import configs
    hb = configs.synth_batch(name, **over)
    if over.get("ins_max") == 60:
        assert (hb.tiles[:, 3] & 2 == 2).any(), "case must exercise general (k_consensus) tiles"
        assert int(hb.tiles[:, 9].max()) > 1024, "case must exercise long motifs and many columns"
    if over.get("depth") == 9000.0:
        assert hb.info.n_deep > 0 and hb.info.n_ins > 0
    ws = _ws(hb, thr, min_depth=md, fill=fill)
    want = bm.model_pipeline(hb, thr, md, fill)
    # the pinned oracle on the same SAM (the model shares the host packing with the kernels)
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "case.sam")
        configs.synth_write(name, p, **over)
        text = open(p, "rb").read().decode("latin-1")
    args = ["--consensus-thresholds=" + ",".join(repr(t) for t in thr), "-m", str(md), "--fill=" + fill.decode("latin-1")]
    ref = o.run_case(text, args, name="case.sam")
    for _ in range(2):   # second run: no state of the first may leak
        ws.run()
        st, offs, out = ws.fetch()
        assert (st == want[0]).all()
        assert (offs == want[1]).all()
        assert out == want[2], _first_diff(out, want[2])
    # the reference's files, or its exception class (:367 KeyError for thresholds that select
    # no symbol or ACGNT, :395 ZeroDivisionError for an empty record)
    import builtins
    from sam2consensus_amd.records import build_records, render
    if ref["status"] == "ok":
        recs = build_records(hb, thr, "case", st, offs, out)
        got = {n + "__case.fasta": render(r, 0).decode("latin-1") for n, r in recs.items()}
        assert got == ref["files"]
    else:
        with pytest.raises(getattr(builtins, ref["status"])):
            build_records(hb, thr, "case", st, offs, out)


@pytest.mark.parametrize("idx", range(len(golden_io.load("stdout"))))
def test_cli_stdout_matches_reference(idx, tmp_path, monkeypatch, capsys):
    """The whole CLI's stdout equals the reference's own captured stdout (tests/golden/
    stdout.json: the reference run in a scratch directory as `-i in.sam -o out`), failing
    cases included (the same exception class, stdout up to the raise): :143, :182, :194,
    :224-227, :420-426."""
    from sam2consensus_amd import cli
    from test_host import _stdout_case
    c = golden_io.load("stdout")[idx]
    sam, args = _stdout_case(c)
    (tmp_path / "in.sam").write_bytes(sam.encode("latin-1"))
    monkeypatch.chdir(tmp_path)
    status = "ok"
    try:
        cli.main(["-i", "in.sam", "-o", "out"] + list(args))
    except (KeyError, IndexError, ValueError, ZeroDivisionError, OverflowError) as e:
        status = type(e).__name__
    assert status == c["status"]
    assert capsys.readouterr().out == c["stdout"]


@pytest.mark.parametrize("idx", [0, 1])
def test_long_skip_on_device_matches_reference(idx):
    """A read whose seqout spans ≥ 2^24 positions (a 16.7 Mb N skip: a long piece, its runs
    from k_reads through the tile long lists, 27-bit run lengths) on the GPU equals the
    reference's files (tests/golden/longskip.json)."""
    from sam2consensus_amd.cli import run_text
    c = golden_io.load("longskip")[idx]
    status, files = run_text(c["sam"], c["args"])
    assert status == c["status"]
    got = {k: hashlib.sha256(v.encode("latin-1")).hexdigest() for k, v in files.items()}
    assert got == {k: v["sha256"] for k, v in c["files"].items()}


@pytest.mark.parametrize("idx", [0, 1])
def test_many_thresholds_on_device_match_reference(idx):
    """300 thresholds (more than round 3's 256-threshold limit): dense tiles loop the vote over
    them, k_tile's epilogue passes of 4, k_consensus reads them from HBM; the FASTA equals the
    reference's files (tests/golden/limits.json)."""
    from sam2consensus_amd.cli import run_text
    c = golden_io.load("limits")[idx]
    status, files = run_text(c["sam"], c["args"])
    assert status == c["status"]
    got = {k: hashlib.sha256(v.encode("latin-1")).hexdigest() for k, v in files.items()}
    assert got == {k: v["sha256"] for k, v in c["files"].items()}


@pytest.mark.timeout(600)
def test_bench_two_ranks_strong_split_line():
    """bench.py --gpus 2 as the driver runs it (no WORLD_SIZE: it starts torchrun as a child):
    the line says n_gpus 2; its value is the strong position split of C5 — two tile ranges,
    the shards' bodies gathered to rank 0 from device memory and byte-identical to the
    reference's file — with the exchange timed; the weak run rides in the same line.  Both
    ranks share this box's one GPU, so the collectives run over gloo."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, S2C_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world_size"] == 2 and d["backend"] == "gloo"
    assert d["scaling"] == "strong"
    assert d["parity"] == "byte-identical to reference (1 files, 2 shards)"
    ex = d["exchange"]
    for k in ("fetch_ms", "stats_reduce_ms", "meta_ms", "body_gather_ms", "merge_ms", "exchange_ms"):
        assert ex[k] >= 0.0, k
    assert ex["body_gather_bytes"] >= 60_000_000   # (C5: 64.4 MB of bodies)
    w = d["weak"]
    assert w["scaling"] == "weak" and w["parity"] == "byte-identical to reference (1 files)"
    assert d["value"] > 0 and w["value"] > 0


@pytest.mark.parametrize("ins_frac,ins_max", [(0.05, 12), (0.01, 20)])
def test_tile_events_and_k_reads_events_agree(tmp_path, ins_frac, ins_max):
    """Who hashes which insertion event is decided twice — on the host (mark_runs: the
    tile's walk records the short motifs of its finish tiles, k_reads the rest) and on the
    device (k_reads' skip test, k_tile's record test).  An event both skipped would be lost
    silently.  The CLI on workloads with insertions of up to 12 / 20 bases (both planned as
    a mix: most events recorded by the tiles, some hashed by k_reads — motifs > 16 bases,
    general tiles), N calls (S2C_PF_XFEW pieces) and events at tile edges, run with the
    tile-recorded events (the product plan) and with every event hashed by k_reads
    (S2C_DEBUG_PLAN=1 S2C_NO_TILE_EVENTS=1, its own process: the plan reads it once): both
    byte-identical to the C restatement."""
    import json
    import subprocess
    import sys
    from sam2consensus_amd import configs
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sam = str(tmp_path / "ins.sam")
    configs.synth_write("c2", sam, n_refs=24, ins_frac=ins_frac, ins_max=ins_max, n_rate=0.01)
    args = ["-c", "0.25,0.5,0.75"]
    subprocess.run(["make", "-s", "-C", os.path.join(root, "oracle")], check=True)
    ref = tmp_path / "ref"
    r = subprocess.run([os.path.join(root, "oracle", "build", "s2c_oracle_mc"), "16", "-i", sam, "-o", str(ref),
                        "-p", "ins"] + args, capture_output=True, text=True, timeout=300)
    assert "status: ok" in r.stdout, r.stdout[-500:]
    want = {fn: open(os.path.join(ref, fn), "rb").read() for fn in os.listdir(ref)}
    assert want
    for tag, extra in (("tile", {}), ("reads", {"S2C_DEBUG_PLAN": "1", "S2C_NO_TILE_EVENTS": "1"})):
        out = tmp_path / tag
        code = ("import json, sys\nfrom sam2consensus_amd import cli\nfrom sam2consensus_amd.batch import parse_file\n"
                "i = parse_file(%r, True, 150).info\n"
                "print(json.dumps([i.tile_events, i.n_rlist, i.n_rlist_run]))\n"
                "sys.exit(cli.main(%r))\n" % (sam, ["-i", sam, "-o", str(out), "-p", "ins"] + args))
        env = dict(os.environ, PYTHONPATH=root, **extra)
        rr = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
        assert rr.returncode == 0, (tag, rr.stderr[-3000:])
        te, nr, nrun = json.loads(rr.stdout.splitlines()[0])
        if tag == "tile":   # (a mix: the tiles record most events, k_reads hashes some)
            assert te == 1 and 0 < nrun < nr, (te, nr, nrun)
        else:
            assert te == 0
        got = {fn: open(os.path.join(out, fn), "rb").read() for fn in os.listdir(out)}
        assert sorted(got) == sorted(want), tag
        for fn in want:
            assert got[fn] == want[fn], (tag, fn, _first_diff(got[fn], want[fn]))
