"""Golden outputs of the REFERENCE on BASELINE.json's synthetic configs (test infra).

For each config: write the deterministic SAM (sam2consensus_amd.configs / s2c_synth.cpp),
run the reference (oracle/ref_harness.py, Python-2 semantics) on it, and record
  - sha256 of the SAM bytes (pins the generator),
  - sha256 of every FASTA file the reference wrote, and its size,
  - the full FASTA text for small configs (c1).
into tests/golden/configs.json (merged, so configs can be generated one at a time):

    python oracle/gen_golden_configs.py c1 c2          # ~1 min
    python oracle/gen_golden_configs.py c4 c3 c5       # long (reference is 1 core)
Build container only (needs /root/reference and libs2c.so built for the generator).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
import ref_harness  # noqa: E402
from sam2consensus_amd import configs  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "configs.json")


def sha_file(path):
    h = hashlib.sha256()
    with open(path, "rb") as fh:
        for chunk in iter(lambda: fh.read(1 << 22), b""):
            h.update(chunk)
    return h.hexdigest()


def run(name, workdir):
    ext = ".sam.gz" if name == "c3" else ".sam"
    sam = os.path.join(workdir, name + ext)
    t0 = time.time()
    n = configs.synth_write(name, sam)
    tgen = time.time() - t0
    out = os.path.join(workdir, "out_" + name)
    args = configs.cli_args(name)
    t0 = time.time()
    status, _ = ref_harness.run_file(sam, args, out)
    tref = time.time() - t0
    files = {}
    full = {}
    if status == "ok":
        for fn in sorted(os.listdir(out)):
            p = os.path.join(out, fn)
            files[fn] = {"sha256": sha_file(p), "size": os.path.getsize(p)}
            if name == "c1":
                full[fn] = open(p, "rb").read().decode("latin-1")
    rec = {"args": args, "n_reads": n, "sam_file": os.path.basename(sam), "sam_sha256": sha_file(sam),
           "status": status, "files": files, "reference_seconds": round(tref, 2),
           "generator_seconds": round(tgen, 2)}
    if full:
        rec["content"] = full
    return rec


def main(names):
    db = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for name in names:
        with tempfile.TemporaryDirectory(dir=os.environ.get("S2C_GOLD_TMP")) as td:
            rec = run(name, td)
        db[name] = rec
        print(name, rec["status"], rec["n_reads"], "reads, reference", rec["reference_seconds"], "s,",
              len(rec["files"]), "files", flush=True)
        with open(OUT, "w") as fh:
            json.dump(db, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:] or ["c1", "c2"])
