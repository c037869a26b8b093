"""Drop-in ``sam2consensus.py`` command line (reference sam2consensus.py:86-430).

Same flags, same outputs (``outfolder/REF__PREFIX.fasta``), same stdout text and the
same failure behaviour: the reference's exception class propagates (traceback, exit
status 1) and no FASTA file is written.  The pileup-and-vote work runs on the GPU
through libs2c.so; host SAM parsing runs in libs2c.so's C++ parser.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

__version__ = "2.1"
DESCRIPTION = """
+------------------------------------------------------------------+
| sam2consensus.py: extract the consensus sequence from a SAM file |
+------------------------------------------------------------------+

Consensus sequences (Geneious threshold rule, IUPAC ambiguity codes) from reads mapped
to one or more references (.sam or .sam.gz), one FASTA file per reference with one
record per consensus threshold.  MI355X implementation: pileup, insertion and vote run
as HIP kernels (libs2c.so); output is byte-identical to sam2consensus.py v2.1.
"""


def build_parser():
    p = argparse.ArgumentParser(description=DESCRIPTION, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("-i", "--input", action="store", dest="filename", required=True,
                   help="Name of the SAM file, SAM does not need to be sorted and can be compressed with gzip")
    p.add_argument("-c", "--consensus-thresholds", action="store", dest="thresholds", type=str, default="0.25",
                   help="List of consensus thresold(s) separated by commas, no spaces, example: -c 0.25,0.75,0.50, default=0.25")
    p.add_argument("-n", action="store", dest="n", type=int, default=0,
                   help="Split FASTA output sequences every n nucleotides, default=do not split sequence")
    p.add_argument("-o", "--outfolder", action="store", dest="outfolder", default="./",
                   help="Name of output folder, default=same folder as input")
    p.add_argument("-p", "--prefix", action="store", dest="prefix", default="",
                   help="Prefix for output file name, default=input filename without .sam extension")
    p.add_argument("-m", "--min-depth", action="store", dest="min_depth", type=int, default=1,
                   help="Minimum read depth at each site to report the nucleotide in the consensus, default=1")
    p.add_argument("-f", "--fill", action="store", dest="fill", default="-",
                   help="Character for padding regions not covered in the reference, default= - (gap)")
    # no type= on purpose (:102): a given -d stays a string, which Python 2 compares
    # as greater than every int, so the maxdel filter (:210) is then never applied.
    p.add_argument("-d", "--maxdel", action="store", dest="maxdel", default=150,
                   help="Ignore deletions longer than this value, default=150")
    return p


class RunResult:
    def __init__(self, files, timings, info, pending=None):
        self.files = files          # {filename: bytes}
        self.timings = timings      # phase → seconds
        self.info = info            # s2c_batch_info
        self.pending = pending      # the host batch's release, still running (HostBatch.free_async)

    def wait(self):
        """Join the batch's release (the CLI does, after writing its files)."""
        if self.pending is not None:
            self.pending.join()
            self.pending = None
        return self


def consensus_batch(hb, thresholds, prefix, min_depth=1, fill=b"-", nchar=0, device=None, timings=None):
    """Device pipeline on a parsed HostBatch → {``REF__PREFIX.fasta``: bytes}."""
    import torch

    from .engine import _UPLOADERS, DeviceBatch, Workspace, needs_dense_layers
    from .records import build_records, render

    t = timings if timings is not None else {}
    t0 = time.perf_counter()
    db = DeviceBatch(hb, device, dense_layers=needs_dense_layers(fill))
    t1 = time.perf_counter()
    ws = Workspace(db, thresholds, min_depth, fill)
    torch.cuda.synchronize(db.device)
    t["h2d"] = time.perf_counter() - t0
    t["h2d_issue"] = t1 - t0   # (layers + pinned staging + copies issued; the rest: workspace + drain)
    up = _UPLOADERS.get(db.device)
    if up is not None:   # (the pinned ring's cumulative host seconds: alloc, wait, pack, issue)
        t.update(("h2d_up_" + k, v) for k, v in up.timing.items())
    t0 = time.perf_counter()
    ws.run()
    torch.cuda.synchronize(db.device)
    t1 = time.perf_counter()
    stats, offs, out = ws.fetch()
    t["device"] = time.perf_counter() - t0
    t["device_run"] = t1 - t0   # (the launches to completion; the rest: the results' D2H)
    t0 = time.perf_counter()
    fastas = build_records(hb, thresholds, prefix, stats, offs, out)
    pre = prefix.encode("latin-1") if isinstance(prefix, str) else prefix
    files = {}
    for name, recs in fastas.items():
        files[name.encode("latin-1") + b"__" + pre + b".fasta"] = render(recs, nchar)
    t["format"] = time.perf_counter() - t0
    return files


PROGRESS_EVERY = 500000   # :224


def progress_lines(header_lines, lines_total):
    """The reference's progress lines (:182, :194, :224-225): its counter starts at
    -header_length, is incremented for every line of the data pass (header lines
    included) and a line is printed whenever it is a multiple of 500000 — "0 reads
    processed." right after a non-empty header, negative multiples for headers longer
    than 500000 lines."""
    lo, hi = 1 - header_lines, lines_total - header_lines   # counter values after each increment
    first = -((-lo) // PROGRESS_EVERY) * PROGRESS_EVERY      # smallest multiple >= lo
    return [str(v) + " reads processed." for v in range(first, hi + 1, PROGRESS_EVERY)]


def _log_summary(log, info):
    log("SAM header processed, " + str(info.n_refs) + " references found.\n")
    for line in progress_lines(info.header_lines, info.lines_total):
        log(line)
    log("A total of " + str(info.lines_total - info.header_lines) + " reads were processed, out of which, " +
        str(info.reads_mapped) + " reads were mapped.\n")


REF_ERRORS = (KeyError, IndexError, ValueError, ZeroDivisionError, OverflowError)


class _Partial:
    """_log_summary's fields from the parser's counters (a run that failed after the read pass)."""

    def __init__(self, n_refs, counters):
        self.n_refs = n_refs
        self.header_lines, self.lines_total, self.reads_mapped = counters[0], counters[1], counters[2]


def _log_failed_parse(log, parser):
    """What the reference has printed when the read pass or its insertion checks raise: its
    header line once the header is read (:182), the progress lines of the lines before the
    failing one (:224-225); after a clean read pass (an insertion check failed, :284-294) the
    whole summary (:227)."""
    ended, n_refs, header_lines, lines, err = parser.progress()
    if not err:
        _log_summary(log, _Partial(n_refs, parser.counters()))
        return
    if not ended:
        return   # (the header pass raised: nothing after "Processing file")
    log("SAM header processed, " + str(n_refs) + " references found.\n")
    for line in progress_lines(header_lines, lines - 1):
        log(line)


def _warm_session(sess, reserve, timing):
    """Bring up the HIP runtime and the device on a side thread (the first device call costs
    tenths of a second) so it overlaps the host parse, and reserve the batch's device buffer
    and pinned staging (``reserve`` bytes: a large input's estimate) there too; join() before
    the upload.  A failure is raised on the main thread by ``_join_session``."""
    import threading

    def run():
        try:
            sess.reserve(reserve)
        except Exception as e:  # noqa: BLE001 - re-raised by _join_session on the main thread
            sess.error = e
        timing.update(sess.timing)
    sess.error = None
    th = threading.Thread(target=run, daemon=True)
    th.start()
    return th


def _join_session(sess, th):
    th.join()
    if sess.error is not None:
        raise sess.error


def upload_estimate(filename):
    """A device block that holds the packed batch of a large input (0 below 64 MB of input):
    the batch is ≈ 0.42 of a plain SAM file's bytes on C5 (short reads, qualities dropped,
    bases in 2-bit planes) — 0.6 × the file (2.4 × a gzip file) leaves room for longer CIGARs."""
    try:
        size = os.path.getsize(filename)
    except OSError:
        return 0   # (the parser reports the reference's error for a missing file)
    if size < (64 << 20):
        return 0
    return int(size * (2.4 if filename.endswith(".gz") else 0.6))


def consensus_batch_hip(sess, hb, thresholds, prefix, min_depth=1, fill=b"-", nchar=0, timings=None):
    """consensus_batch through hiprun.Session (no PyTorch): the one-process CLI's device side."""
    from .records import build_records, render

    t = timings if timings is not None else {}
    t0 = time.perf_counter()
    stats, offs, out = sess.run(hb, thresholds, min_depth, fill, t)
    t["device"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    fastas = build_records(hb, thresholds, prefix, stats, offs, out)
    pre = prefix.encode("latin-1") if isinstance(prefix, str) else prefix
    files = {}
    for name, recs in fastas.items():
        files[name.encode("latin-1") + b"__" + pre + b".fasta"] = render(recs, nchar)
    t["format"] = time.perf_counter() - t0
    return files


def consensus_files(filename, thresholds, prefix, min_depth=1, fill=b"-", nchar=0, maxdel_active=True,
                    device=None, log=None):
    """Run the whole pipeline on one SAM/SAM.gz file; returns a RunResult whose
    ``files`` maps ``REF__PREFIX.fasta`` → content bytes (nothing written).  The device side
    runs through the HIP runtime directly (hiprun.py): this path never imports PyTorch."""
    from .batch import Parser
    from .hiprun import Session, device_index

    t = {}
    t0 = time.perf_counter()
    sess = Session(device_index(device))
    warm = _warm_session(sess, upload_estimate(filename), t)   # (the device comes up while the host parses)
    try:
        p = Parser(maxdel_active, 150)
        try:
            p.feed_file(filename)
            hb = p.finish()
        except REF_ERRORS:
            if log:
                _log_failed_parse(log, p)
            raise
        finally:
            p.close()
        t["parse"] = time.perf_counter() - t0
        _join_session(sess, warm)
        if log:
            _log_summary(log, hb.info)
        files = consensus_batch_hip(sess, hb, thresholds, prefix, min_depth, fill, nchar, t)
    finally:
        warm.join()
        sess.close()
    # the batch's host arrays (GBs for a large input: ~60 ms of munmap on the box) released
    # beside the caller's file writes
    return RunResult(files, t, hb.info, hb.free_async())


def run_text(sam_text, argv, device=None):
    """Library entry for tests: SAM text + CLI args (without -i) → (status, {fname: str}).
    status is "ok" or the reference's exception class name; nothing touches the disk."""
    from .batch import parse_text

    args = build_parser().parse_args(["-i", "in.sam"] + list(argv))
    try:
        thresholds = [float(i) for i in args.thresholds.split(",")]
        prefix = args.prefix or "in"
        hb = parse_text(sam_text, not isinstance(args.maxdel, str), 150)
        files = consensus_batch(hb, thresholds, os.fsencode(prefix), args.min_depth,
                                os.fsencode(args.fill), args.n, device)
    except (KeyError, IndexError, ValueError, ZeroDivisionError, OverflowError) as e:
        return type(e).__name__, {}
    return "ok", {k.decode("latin-1"): v.decode("latin-1") for k, v in files.items()}


def _dist_env():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), \
        int(os.environ.get("LOCAL_RANK", "0"))


class _Counters:
    """The summary counters of the distributed read pass (``_log_summary``'s fields)."""

    def __init__(self, n_refs, parsed):
        self.n_refs = n_refs
        self.header_lines, self.lines_total, self.reads_mapped = \
            parsed.header_lines, parsed.lines_total, parsed.reads_mapped


def consensus_files_sharded(filename, thresholds, prefix, min_depth, fill, nchar, maxdel_active, log=None):
    """One process per GPU (torchrun): the file is parsed once across the ranks and each
    rank receives the reads of its tile range (sam2consensus_amd.dparse), runs it, the
    stats are all-reduced and the FASTA bodies gathered over the process group (RCCL; the
    gloo backend with S2C_DIST_BACKEND=gloo); rank 0 returns the files, other ranks None."""
    import torch
    import torch.distributed as dist

    from .dparse import parse_distributed
    from .engine import DeviceBatch, Workspace, needs_dense_layers
    from .records import build_records, render
    from .shard import gather_device

    world, rank, local = _dist_env()
    backend = os.environ.get("S2C_DIST_BACKEND", "nccl")
    ndev = max(torch.cuda.device_count(), 1)
    if local >= ndev:
        if backend != "gloo":   # RCCL: one device per rank
            raise RuntimeError("LOCAL_RANK %d but %d GPU(s) visible: launch one process per GPU "
                               "(S2C_DIST_BACKEND=gloo lets ranks share a device)" % (local, ndev))
        local %= ndev   # (ranks sharing a device: gloo tests on one GPU)
    torch.cuda.set_device(local)
    from . import _lib
    _lib.plan_for_device(torch.device("cuda", local))
    owned = not dist.is_initialized()   # (this call's process group: destroyed on the way out)
    if owned:
        dist.init_process_group(backend, device_id=torch.device("cuda", local) if backend == "nccl" else None)
    try:
        P = parse_distributed(filename, rank, world, maxdel_active)
        if log and rank == 0:
            _log_summary(log, _Counters(P.hb.info.n_refs, P))
        ws = Workspace(DeviceBatch(P.sub, "cuda:%d" % local, dense_layers=needs_dense_layers(fill)), thresholds,
                       min_depth, fill)
        ws.run()
        res = gather_device(ws, P.sub, rank, world, len(thresholds))
    finally:
        if owned and dist.is_initialized():
            dist.destroy_process_group()
    if rank != 0:
        return None
    P.hb.ref_reads = P.ref_flags   # Σcoverage > 0 over every rank's reads (:334-341)
    fastas = build_records(P.hb, thresholds, prefix, *res)
    pre = prefix.encode("latin-1") if isinstance(prefix, str) else prefix
    return {n.encode("latin-1") + b"__" + pre + b".fasta": render(r, nchar) for n, r in fastas.items()}


def main(argv=None):
    args = build_parser().parse_args(argv)
    filename = args.filename
    thresholds = [float(i) for i in args.thresholds.split(",")]                # :117-118
    if args.prefix == "":
        prefix = "".join(args.filename.split("/")[-1]).split(".")[0]            # :121-122
    else:
        prefix = args.prefix
    outfolder = args.outfolder.rstrip("/")                                       # :127-130
    world, rank, _ = _dist_env()
    if rank == 0 and not os.path.exists(outfolder):   # (one process creates it: rank 0 writes the files)
        os.makedirs(outfolder)
    outfolder += "/"
    maxdel_active = not isinstance(args.maxdel, str)
    res = None
    if rank == 0:
        print("\nProcessing file " + filename + ":\n")
    if world > 1:
        files = consensus_files_sharded(filename, thresholds, os.fsencode(prefix), args.min_depth,
                                        os.fsencode(args.fill), args.n, maxdel_active, log=print)
        if files is None:
            return 0
    else:
        from .stream import consensus_files_streamed, stream_bytes_from_env
        sb = stream_bytes_from_env()
        if sb > 0:   # coordinate-sorted input in bounded host memory (stream.py)
            files = consensus_files_streamed(filename, thresholds, os.fsencode(prefix), args.min_depth,
                                             os.fsencode(args.fill), args.n, maxdel_active, log=print,
                                             batch_bytes=sb).files
        else:
            res = consensus_files(filename, thresholds, os.fsencode(prefix), args.min_depth,
                                  os.fsencode(args.fill), args.n, maxdel_active, log=lambda s: print(s))
            files = res.files
    for fname, body in files.items():                                             # :411-424
        path = os.fsencode(outfolder) + fname
        with open(path, "wb") as fh:
            fh.write(body)
        shown = os.fsdecode(path)
        if len(thresholds) == 1:
            print("Consensus sequence at " + str(int(thresholds[0] * 100)) + "% saved for " +
                  os.fsdecode(fname[: fname.rfind(b"__")]) + " in: " + shown)
        else:
            print("Consensus sequences at " + ",".join([str(int(i * 100)) + "%" for i in thresholds]) +
                  " saved for " + os.fsdecode(fname[: fname.rfind(b"__")]) + " in: " + shown)
    if res is not None:
        res.wait()
    print("Done.\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
