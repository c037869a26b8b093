"""Wall clock of the real CLI process on a config's SAM file (python startup, imports, parse,
device, files written) against `import torch` alone and the in-process phases (GPU box).

    python scripts/cli_wall.py [workload]
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def wall(cmd):
    t0 = time.perf_counter()
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, cwd=ROOT, timeout=600)
    return round(time.perf_counter() - t0, 3)


def main():
    from sam2consensus_amd import configs
    wl = sys.argv[1] if len(sys.argv) > 1 else "c5"
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        sam = os.path.join(td, wl + ".sam")
        configs.synth_write(wl, sam)
        res = {"workload": wl, "sam_bytes": os.path.getsize(sam), "runs": []}
        for _ in range(2):
            res["runs"].append({
                "python_startup_s": wall([sys.executable, "-c", "pass"]),
                "import_torch_s": wall([sys.executable, "-c", "import torch"]),
                "cli_s": wall([sys.executable, "sam2consensus.py", "-i", sam, "-o", os.path.join(td, "out")]
                              + configs.cli_args(wl)),
            })
        print(json.dumps(res))


if __name__ == "__main__":
    main()
