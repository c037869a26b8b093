"""The oracle (oracle/s2c_oracle.py) is pinned to the reference's own outputs."""
import random

import pytest

import golden_io
import s2c_oracle as o

CASES = golden_io.cases()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference(case):
    r = o.run_case(case["sam"], case["args"])
    assert r["status"] == case["status"]
    assert r["files"] == case["files"]


def test_amb_table_matches_reference_dict():
    amb = golden_io.load("amb")                      # sam2consensus.py:317-329 as data
    assert len(amb) == 62
    for m in range(64):
        key = o.mask_key(m)
        assert o.AMB_TABLE[m] == amb.get(key), key
    assert "ACGNT" not in amb and o.AMB_TABLE[0b111110] is None


def test_closed_form_vote_equals_group_sort():
    rng = random.Random(7)
    for _ in range(60000):
        c = [rng.choice([0, 0, 1, 2, 3, 5, 8, rng.randint(0, 60)]) for _ in range(6)]
        if rng.random() < 0.3:
            c[0] = rng.randint(-40, 3)          # insertion columns: '-' may be <= 0 (:294)
        cov = sum(c) + (rng.randint(0, 30) if rng.random() < 0.4 else 0)
        t = rng.choice([0.1, 0.25, 0.29, 0.5, 0.66, 0.75, 0.9, 1.0, 1.5, 0.0, -0.2])
        assert o.vote_groups(c, cov, t) == o.vote_closed(c, cov, t)


def test_py2_round_and_str():
    assert o.py2_str_float(o.py2_round(9 / 8.0)) == "1.13"      # Py3 round gives 1.12
    assert o.py2_str_float(o.py2_round(1.0)) == "1.0"
    assert o.py2_str_float(o.py2_round(100000.0)) == "100000.0"
    assert o.py2_str_float(o.py2_round(2 / 3.0)) == "0.67"
    assert o.py2_str_float(o.py2_round(-9 / 8.0)) == "-1.13"


def test_configs_c1_oracle_matches_reference_content():
    """The oracle reproduces the reference's C1 FASTA files byte for byte."""
    import hashlib
    from sam2consensus_amd import configs
    import tempfile, os
    g = golden_io.load("configs")["c1"]
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "c1.sam")
        configs.synth_write("c1", p)
        assert hashlib.sha256(open(p, "rb").read()).hexdigest() == g["sam_sha256"]
        text = open(p, "rb").read().decode("latin-1")
    r = o.run_case(text, g["args"], name="c1.sam")
    assert r["status"] == "ok"
    assert {k: v for k, v in r["files"].items()} == g["content"]


# ------------------------------------------------ the multi-threaded C restatement
ORACLE_DIR = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))), "oracle")


@pytest.fixture(scope="module")
def mc_bin():
    import os
    import subprocess
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return os.path.join(ORACLE_DIR, "build", "s2c_oracle_mc")


def run_mc(binary, sam_text, args, threads, name="in.sam"):
    """oracle/s2c_oracle_mc on SAM text → {"status", "files"} (the golden cases' form)."""
    import os
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, name)
        with open(p, "w", encoding="latin-1", newline="") as fh:
            fh.write(sam_text)
        out = os.path.join(td, "out")
        r = subprocess.run([binary, str(threads), "-i", p, "-o", out] + list(args), capture_output=True, text=True)
        status = r.stdout.split("status: ")[1].split()[0] if "status: " in r.stdout else "crash rc=%d" % r.returncode
        files = {}
        if status == "ok" and os.path.isdir(out):
            for f in sorted(os.listdir(out)):
                with open(os.path.join(out, f), encoding="latin-1", newline="") as fh:
                    files[f] = fh.read()
        return {"status": status, "files": files}


def test_c_oracle_matches_reference_cases(mc_bin):
    """Every KAT / fuzz case (reference outputs) through the C restatement, 1 and 3 threads."""
    bad = []
    for i, case in enumerate(CASES):
        for threads in ((1, 3) if i % 4 == 0 else (2,)):
            r = run_mc(mc_bin, case["sam"], case["args"], threads)
            if r["status"] != case["status"] or r["files"] != case["files"]:
                bad.append((case["name"], threads, r["status"], case["status"]))
    assert not bad, bad[:10]


@pytest.mark.parametrize("wl", ["c1", "c2s"])
def test_c_oracle_matches_python_oracle_on_configs(mc_bin, wl):
    """Synthetic configurations (insertions, deletions, N, several references): the C
    restatement on 4 threads equals the Python oracle."""
    import os
    import tempfile
    from sam2consensus_amd import configs
    name, kw = (wl, {}) if wl != "c2s" else ("c2", {"n_refs": 6, "depth": 40.0})
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, name + ".sam")
        configs.synth_write(name, p, **kw)
        text = open(p, "rb").read().decode("latin-1")
    args = configs.cli_args(name)
    want = o.run_case(text, args, name=name + ".sam")
    got = run_mc(mc_bin, text, args, 4, name=name + ".sam")
    assert got["status"] == want["status"] == "ok"
    assert got["files"] == want["files"]


@pytest.mark.parametrize("idx", [0, 1])
def test_oracle_many_thresholds_matches_reference(idx):
    """300 thresholds (-c; the reference takes any number, sam2consensus.py:117-118): the
    oracle equals the reference's files (tests/golden/limits.json, oracle/gen_golden_limits.py)."""
    import hashlib
    c = golden_io.load("limits")[idx]
    r = o.run_case(c["sam"], c["args"])
    assert r["status"] == c["status"]
    got = {k: hashlib.sha256(v.encode("latin-1")).hexdigest() for k, v in r["files"].items()}
    assert got == {k: v["sha256"] for k, v in c["files"].items()}
