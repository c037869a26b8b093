"""Host parse + plan time of one config's SAM file (libs2c.so: s2c_parser_feed_file, then
s2c_parser_finish) under environment variants, each in its own child process, best of R.

    python scripts/parse_time.py c5 'S2C_HUGEPAGES=0' 'S2C_HUGE_MIN_KB=1024' ... > out.json
(no variant: the defaults only).  S2C_HOST_TIMING=1 in a variant prints the plan's phases.
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
R = 3


def child(path):
    from sam2consensus_amd import configs  # noqa: F401  (loads libs2c.so)
    from sam2consensus_amd.batch import Parser
    best = None
    for _ in range(R):
        p = Parser(True, 150)
        t0 = time.perf_counter()
        p.feed_file(path)
        t1 = time.perf_counter()
        hb = p.finish()
        t2 = time.perf_counter()
        hb.free()
        p.close()
        r = (t1 - t0, t2 - t1)
        best = r if best is None or sum(r) < sum(best) else best
    print(json.dumps({"feed_s": round(best[0], 3), "finish_s": round(best[1], 3), "total_s": round(sum(best), 3)}))


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2])
        return 0
    wl, variants = sys.argv[1], [""] + sys.argv[2:]
    from sam2consensus_amd import configs
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        path = os.path.join(td, wl + ".sam")
        configs.synth_write(wl, path)
        res = {"config": wl, "bytes": os.path.getsize(path), "threads": os.environ.get("OMP_NUM_THREADS"), "runs": {}}
        for v in variants:
            env = dict(os.environ)
            for kv in v.split():
                k, _, val = kv.partition("=")
                env[k] = val
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", path], env=env,
                                 capture_output=True, text=True, timeout=600)
            if out.returncode:
                sys.stderr.write(out.stderr)
                return out.returncode
            res["runs"][v or "default"] = json.loads(out.stdout.strip().splitlines()[-1])
            sys.stderr.write(out.stderr[-2000:])
            sys.stderr.write("%s %s\n" % (v or "default", res["runs"][v or "default"]))
        print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
