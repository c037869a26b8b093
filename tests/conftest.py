"""pytest configuration: the `gpu` marker and import paths.

CPU tier (driver runs `pytest -m "not gpu"` in the build container): oracle vs the
reference's golden fixtures, host parser/packing/plan through a CPU model of the
kernels, the C-ABI export table, multi-rank sharding over gloo.
GPU tier (`pytest -m gpu` on an MI355X): HIP path vs golden fixtures / oracle.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels run)")
    config.addinivalue_line("markers", "slow: multi-minute CPU work")
