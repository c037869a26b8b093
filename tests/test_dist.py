"""Multi-rank sharding (sam2consensus_amd/shard.py) on CPU: tile split, sub-batch slicing,
stats all-reduce and output gather must reproduce the single-shard result byte for byte.
The per-rank runner is the kernel-shaped CPU model (tests/batch_model.py); on GPU the
same sub-batches run through libs2c.so (tests/test_gpu.py::test_sharded_on_device)."""
import os
import socket

import numpy as np
import pytest

import batch_model as bm
import golden_io
import s2c_oracle as o
from sam2consensus_amd import batch, configs, records, shard


def _files(hb, opt, stats, offs, out):
    fastas = records.build_records(hb, opt.thresholds, opt.prefix, stats, offs, out)
    return {n + "__" + opt.prefix + ".fasta": records.render(r, opt.n).decode("latin-1") for n, r in fastas.items()}


def _virtual(hb, opt, world):
    parts, stats = [], None
    for rank in range(world):
        sub = shard.sub_batch(hb, rank, world)
        bm.check_plan_shard(sub)
        st, offs, out = bm.model_pipeline(sub, opt.thresholds, opt.min_depth, opt.fill.encode("latin-1"))
        stats = st if stats is None else stats + st
        parts.append((sub.t0, sub.t1, offs, out))
    offs, out = shard.merge_outputs(parts, len(opt.thresholds))
    return _files(hb, opt, stats, offs, out)


MULTI = golden_io.load("kat")


def _big_case():
    """Several refs with insertions, deletions, long (N) reads and POS=0 wrap."""
    sam = "@SQ\tSN:a\tLN:900\n@SQ\tSN:b\tLN:3000\n@SQ\tSN:c\tLN:40\n"
    rows = []
    for s in range(1, 760, 3):
        rows.append(("a", s, "60M2I50M", "ACGT" * 28))
    for s in range(1, 2800, 5):
        rows.append(("b", s, "40M3D60M", "TTGCA" * 20))
    rows.append(("b", 10, "10M2000N10M", "G" * 20))
    rows.append(("b", 1500, "5M2I", "GGGGGTT"))           # insertion keyed after the last base
    rows.append(("b", 2000, "3S4I", "AAACCCC"))            # events, nothing counted
    rows.append(("c", 0, "5M", "CCCCC"))
    rows.append(("c", 0, "1M2I3M", "AGGCCC"))              # POS=0 wrap with an insertion
    for r in rows:
        sam += "r\t0\t%s\t%d\t60\t%s\t*\t0\t0\t%s\t*\n" % r
    return sam


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_virtual_ranks_reproduce_reference(world):
    for case in [c for c in MULTI if c["status"] == "ok"][:12]:
        opt = o.parse_argv(["-i", "in.sam"] + case["args"])
        hb = batch.parse_text(case["sam"], opt.maxdel_active, 150)
        assert _virtual(hb, opt, world) == case["files"], case["name"]
    sam = _big_case()
    for args in ([], ["-c", "0.25,0.75"], ["-d", "9"]):
        opt = o.parse_argv(["-i", "in.sam"] + args)
        hb = batch.parse_text(sam, opt.maxdel_active, 150)
        assert _virtual(hb, opt, world) == o.run_case(sam, args)["files"]


def test_split_is_balanced_and_contiguous():
    hb = configs.synth_batch("c2", n_refs=40)
    for world in (2, 4, 8):
        rng = shard.split_tiles(hb, world)
        assert rng[0][0] == 0 and rng[-1][1] == hb.info.n_tiles
        assert all(rng[k][1] == rng[k + 1][0] for k in range(world - 1))
        w = shard.tile_weights(hb)
        loads = [w[a:b].sum() for a, b in rng]
        assert max(loads) < 1.3 * (sum(loads) / world)


def test_shard_keeps_the_instantiation_its_layers_were_cut_for():
    """Layers are cut for the k_tile instantiation planned for the whole batch (s2c.h
    S2C_CHUNK_QBYTES_OF: the non-queue one holds more plane bytes per layer), and a shard inherits
    its tiles' layer counts: a shard may drop the walk queue but never take it up when its parent
    was planned without it."""
    for name, over in (("c2", {"n_refs": 40}), ("c2", {"n_refs": 40, "ins_frac": 0.0, "del_frac": 0.004}),
                       ("c4", {"ref_len": 2000, "depth": 3000.0})):
        hb = configs.synth_batch(name, **over)
        for world in (2, 4):
            for r in range(world):
                sub = shard.sub_batch(hb, r, world)
                assert sub.info.walk_queue <= hb.info.walk_queue, (name, over, world, r)
                assert (sub.tiles[:, 19] == hb.tiles[sub.t0:sub.t1, 19]).all()
                sub.free()


def test_exchange_volumes_count_the_duplicated_reads():
    """shard.exchange_volumes (bench.py's dup_frac): the pieces summed over the
    shards are at least the workload's and exceed it by the reads reaching across a cut."""
    hb = configs.synth_batch("c2", n_refs=12)
    for world in (1, 2, 4):
        subs = [shard.sub_batch(hb, r, world) for r in range(world)]
        v = shard.exchange_volumes(hb, subs)
        assert v["pieces_total"] == hb.info.n_pieces
        assert v["pieces_over_shards"] >= v["pieces_total"]
        if world == 1:
            assert v["dup_frac"] == 1.0 and v["cuts"] == 0 and v["count_merge_bytes"] == 0
        else:
            assert 1.0 < v["dup_frac"] < 1.5 and v["cuts"] == world - 1 and v["dup_bytes"] > 0
        # (ABI 13) each shard uploads the per-word arrays over its own words (+ the window
        # lookback) only: together about one copy of the whole batch's, not `world` copies
        nw = int(hb.info.n_words)
        per_word = sum(int(s_.info.word_hi - s_.info.word_lo) for s_ in subs)
        assert per_word <= nw + world * (int(hb.info.kwin) + 2)
        for s_ in subs:
            lo, hi = int(s_.info.word_lo), int(s_.info.word_hi)
            assert 0 <= lo < hi <= nw and len(s_.device_view("rs")) == hi - lo + 1
            assert len(s_.device_view("wtile")) == hi - lo
            t = s_.tiles
            assert lo <= int(t[0, 0]) >> 5 and (int(t[-1, 1]) + 31) >> 5 <= hi
        for s_ in subs:
            s_.free()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, sam, args, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        opt = o.parse_argv(["-i", "in.sam"] + args)
        hb = batch.parse_text(sam, opt.maxdel_active, 150)
        sub = shard.sub_batch(hb, rank, world)
        tim = {}
        res = shard.gather_results(bm.model_pipeline(sub, opt.thresholds, opt.min_depth, opt.fill.encode("latin-1")),
                                   sub, rank, world, len(opt.thresholds), timing=tim)
        # every exchange step timed on every rank (bench.py's "exchange" record), merge on rank 0
        steps = ("stats_reduce", "meta", "body_gather") + (("merge",) if rank == 0 else ())
        assert all(tim[k + "_s"] >= 0 for k in steps), tim
        assert tim["body_gather_bytes"] >= 8 and tim["stats_reduce_bytes"] > 0
        if rank == 0:
            q.put(_files(hb, opt, *res))
    finally:
        dist.destroy_process_group()


def test_gloo_two_ranks_match_reference():
    import torch.multiprocessing as mp
    sam = _big_case()
    args = ["-c", "0.25,0.5"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, sam, args, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == o.run_case(sam, args)["files"]


# ---- distributed parse (sam2consensus_amd/dparse.py): every line parsed once, by one rank

def _dparse_worker(rank, world, port, cases, paths, block, q):
    import torch.distributed as dist

    from sam2consensus_amd import dparse
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = []
    try:
        for sam, args, path in [(s, a, None) for s, a in cases] + [(None, a, p) for p, a in paths]:
            opt = o.parse_argv(["-i", "in.sam"] + args)
            try:
                P = dparse.parse_distributed(path, rank, world, opt.maxdel_active,
                                             block=block if path is None else 1 << 20,
                                             text=None if sam is None else sam.encode("latin-1"))
                res = shard.gather_results(bm.model_pipeline(P.sub, opt.thresholds, opt.min_depth,
                                                             opt.fill.encode("latin-1")),
                                           P.sub, rank, world, len(opt.thresholds))
                got = ("ok", None, None)
                if rank == 0:
                    P.hb.ref_reads = P.ref_flags
                    got = ("ok", _files(P.hb, opt, *res), (P.header_lines, P.lines_total, P.reads_mapped))
            except Exception as e:  # noqa: BLE001 - compared with the reference's class
                got = (type(e).__name__, {}, None)
            out.append(got)
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


def _run_dparse(world, cases, paths, block):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dparse_worker, args=(r, world, port, cases, paths, block, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("world,block", [(2, 90), (3, 400)])
def test_distributed_parse_matches_reference(world, block, tmp_path):
    """KAT cases (errors included: the first failing line in file order, the insertion checks
    in reference order) and the multi-reference case, cut into many small blocks; plus a
    scaled C2 as .sam and .sam.gz files against the whole-file parse."""
    kat = golden_io.load("kat")
    cases = [(c["sam"], c["args"]) for c in kat]
    big = _big_case()
    cases += [(big, a) for a in ([], ["-c", "0.25,0.75"], ["-d", "9"])]
    want = [(c["status"], c["files"]) for c in kat]
    want += [("ok", o.run_case(big, a)["files"]) for a in ([], ["-c", "0.25,0.75"], ["-d", "9"])]
    # '@' lines in the body (skipped by the read pass, :195; never references): every block
    # boundary of the small block size falls on one of them somewhere
    body = []
    for k in range(40):
        body.append("r%d\t0\tg1\t%d\t60\t6M\t*\t0\t0\tACGTAC\t*\n" % (k, 1 + k % 20))
        if k % 3 == 1:
            body.append("@SQ\tSN:zz%d\tLN:9\n" % k if k % 2 else "@CO\tcomment %d\n" % k)
    at_body = "@HD\tVN:1.0\n@SQ\tSN:g1\tLN:30\n" + "".join(body)
    cases.append((at_body, []))
    ref = o.run_case(at_body, [])
    want.append((ref["status"], ref["files"]))
    paths = []
    for ext in (".sam", ".sam.gz"):   # (.sam.gz: BGZF, each rank inflates its own blocks)
        p = str(tmp_path / ("c2s" + ext))
        configs.synth_write("c2", p, scale=0.03 if world == 2 else 0.01)
        paths.append((p, configs.cli_args("c2")))
    if world == 3:   # a small BGZF file: few blocks per rank, lines cut at every range end
        p = str(tmp_path / "c1.sam.gz")
        configs.synth_write("c1", p)
        paths.append((p, configs.cli_args("c1")))
    got = _run_dparse(world, cases, paths, block)
    assert len(got) == len(want) + len(paths)
    for k, (g, w) in enumerate(zip(got, want)):
        assert g[0] == w[0], (k, g[0], w[0])
        if g[0] == "ok":
            assert g[1] == w[1], k
    for (p, args), g in zip(paths, got[len(want):]):
        opt = o.parse_argv(["-i", "in.sam"] + args)
        hb = batch.parse_file(p, opt.maxdel_active, 150)
        assert g[0] == "ok"
        assert g[1] == _virtual(hb, opt, 1)
        i = hb.info
        assert g[2] == (i.header_lines, i.lines_total, i.reads_mapped)


def test_forced_collectives_at_world_one(monkeypatch):
    """S2C_FORCE_COLLECTIVES=1 runs the exchange collectives that world size 1 skips (the
    path tests/test_gpu.py::test_rccl_exchange_at_world_one runs over RCCL on the GPU box):
    here over gloo, the distributed parse and the gather == the reference."""
    monkeypatch.setenv("S2C_FORCE_COLLECTIVES", "1")
    big = _big_case()
    cases = [(big, []), (big, ["-c", "0.25,0.75"])]
    got = _run_dparse(1, cases, [], 400)
    assert [g[0] for g in got] == ["ok", "ok"]
    for (sam, args), g in zip(cases, got):
        assert g[1] == o.run_case(sam, args)["files"]
