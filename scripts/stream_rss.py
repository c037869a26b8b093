"""Host memory of the whole-batch path vs streamed batches (stream.py) on one config's
coordinate-sorted SAM file: each mode runs in its own child process (peak RSS from
getrusage), and the FASTA bytes of both must agree.  `seconds` is the CLI's work: parse,
device, records, the FASTA files written (round 6: the writes and the whole batch's host
release are included; earlier rounds' figures stop before the writes).

    python scripts/stream_rss.py c5 [batch_MB] > gpurun_out/stream_rss_c5.json
"""
import hashlib
import json
import os
import resource
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(mode, path, name, batch_mb):
    from sam2consensus_amd import configs
    from sam2consensus_amd.cli import consensus_files
    from sam2consensus_amd.cli import build_parser
    from sam2consensus_amd.stream import consensus_files_streamed
    a = build_parser().parse_args(["-i", path] + configs.cli_args(name))
    thr = [float(x) for x in a.thresholds.split(",")]
    prefix = os.path.basename(path).split(".")[0].encode()
    common = (thr, prefix, a.min_depth, a.fill.encode(), a.n, not isinstance(a.maxdel, str))
    if os.environ.get("E2E_NO_RESERVE"):   # (A/B: the CLI's warm-up thread without the upload reservation)
        import sam2consensus_amd.cli as cli
        cli.upload_estimate = lambda filename: 0
    t0 = time.perf_counter()
    if mode == "whole":
        r = consensus_files(path, *common)
    else:
        batch_mb = int(os.environ.get("STREAM_BATCH_MB", batch_mb))
        r = consensus_files_streamed(path, *common, batch_bytes=batch_mb << 20)
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as od:   # (the CLI's file writes)
        t1 = time.perf_counter()
        for k, body in r.files.items():
            with open(os.path.join(os.fsencode(od), k), "wb") as fh:
                fh.write(body)
        r.timings["write"] = time.perf_counter() - t1
        if hasattr(r, "wait"):
            r.wait()   # (the whole batch's release, overlapped with the writes)
        r.timings["write_and_free"] = time.perf_counter() - t1
        dt = time.perf_counter() - t0
    h = hashlib.sha256()
    for k in sorted(r.files):
        h.update(k)
        h.update(r.files[k])
    print(json.dumps({"mode": mode, "seconds": round(dt, 3),
                      "peak_rss_mb": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0, 1),
                      "sha256": h.hexdigest(), "batches": len(getattr(r, "batches", [])) or 1,
                      "phases_s": {k: round(v, 3) for k, v in getattr(r, "timings", {}).items()},
                      "reads_held_max": getattr(r, "held_max", None)}))


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]))
        return 0
    name = sys.argv[1]
    batch_mb = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    from sam2consensus_amd import configs
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        path = os.path.join(td, name + (".sam.gz" if name == "c3" else ".sam"))   # C3 is a SAM.gz config
        n = configs.synth_write(name, path)
        size = os.path.getsize(path)
        res = {"config": name, "reads": n, "sam_bytes": size, "batch_mb": batch_mb}
        sys.stderr.write("wrote %d reads, %d bytes\n" % (n, size))
        sys.stderr.flush()
        # STREAM_VARIANTS="A=1,B=2;A=4": more streamed runs of the same file, each with those
        # environment settings (keys "stream:A=1,B=2", ...)
        runs = [("whole", {}), ("stream", {})]
        if os.environ.get("STREAM_WHOLE_ONLY"):   # (the whole-file CLI only, twice: box-to-box spread)
            runs = [("whole", {}), ("whole:again", {})]
        for v in filter(None, os.environ.get("STREAM_VARIANTS", "").split(";")):
            runs.append(("stream:" + v, dict(kv.split("=", 1) for kv in v.split(","))))
        # WHOLE_VARIANTS="A=1;A=2": whole-file runs with those settings, the set twice in turn
        # (with a plain run in each turn; keys "whole:A=1#1", ...)
        wv = list(filter(None, os.environ.get("WHOLE_VARIANTS", "").split(";")))
        if wv:
            runs = [(("whole:%s#%d" % (v, k)) if v else "whole" if k == 1 else "whole:#2",
                     dict(kv.split("=", 1) for kv in v.split(",")) if v else {}) for k in (1, 2) for v in [""] + wv]
        for key, env in runs:
            mode = key.split(":")[0]
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", mode, path, name,
                                  str(batch_mb)], capture_output=True, text=True, timeout=600,
                                 env=dict(os.environ, **env))
            if out.returncode != 0:
                sys.stderr.write(out.stderr)
                return out.returncode
            if os.environ.get("STREAM_LOG"):   # (the children's stderr, e.g. S2C_HOST_TIMING lines)
                with open(os.environ["STREAM_LOG"], "a") as f:
                    f.write("== %s\n%s" % (key, out.stderr))
            res[key] = json.loads(out.stdout.strip().splitlines()[-1])
            sys.stderr.write(key + " " + json.dumps(res[key]) + "\n")
            sys.stderr.flush()
        res["identical"] = all(res[k]["sha256"] == res["whole"]["sha256"] for k, _ in runs)
        print(json.dumps(res))
        return 0 if res["identical"] else 1


if __name__ == "__main__":
    sys.exit(main())
