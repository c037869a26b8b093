"""Reference-run harness (TEST INFRASTRUCTURE ONLY — never shipped, never on the GPU box).

Runs the *unmodified algorithm* of the reference script
``/root/reference/sam2consensus.py`` (read-only, Python 2 only) under this
container's Python 3, restoring the Python 2 semantics the script depends on.
This is the recipe of SURVEY.md §8(c); it is used by ``oracle/gen_golden.py``
to produce the golden fixtures committed under ``tests/golden/``.

Nothing from the reference is copied: the source text is read from
``/root/reference`` at run time, four ``.iteritems()`` calls
(``sam2consensus.py:242,247,299,304``) are spelled ``.items()`` in memory, and
the code object is executed in a fresh namespace with these shims:

1. ``round`` → Python 2.7 ``round(x, n)``: correctly rounded, exact binary
   ties away from zero (CPython 2.7 ``_Py_double_round``), returning a float
   whose ``str`` is Python 2's ``'%.12g'`` + ``'.0'`` (``float_str``).
   Used at ``sam2consensus.py:395``.
2. ``argparse`` → when ``-d`` is given its value stays a ``str``
   (``sam2consensus.py:102`` has no ``type=``); Python 2 orders every int
   below every str, so ``count <= maxdel`` (``:210``) is always True.  The shim
   wraps that str so the comparison gives Python 2's answer.
3. ``open`` / ``gzip.open`` → byte-transparent text (latin-1, lines split on
   ``\\n`` only, no newline translation), as Python 2 ``str`` I/O.
"""
from __future__ import annotations

import argparse
import decimal
import gzip as _gzip
import io
import math
import os
import sys
import tempfile
import types

REF_PATH = "/root/reference/sam2consensus.py"


# ---------------------------------------------------------------- Py2 shims
class Py2Float(float):
    """float whose str() is CPython 2.7 ``float_str``: '%.12g', '.0' if integral-looking."""

    def __str__(self):  # noqa: D401
        r = "%.12g" % float(self)
        if r.lstrip("-").isdigit():
            r += ".0"
        return r


def py2_round(x, n=0):
    """CPython 2.7 round(): correctly rounded, exact ties away from zero."""
    x = float(x)
    if x == 0.0 or math.isnan(x) or math.isinf(x):
        return Py2Float(x)
    ctx = decimal.Context(prec=400, rounding=decimal.ROUND_HALF_UP)
    q = decimal.Decimal(1).scaleb(-n)
    d = decimal.Decimal(x).quantize(q, context=ctx)
    return Py2Float(float(d))


class _Py2MaxdelStr(str):
    """A ``-d`` value as Python 2 compares it: every int is < every str."""

    def __ge__(self, other):
        if isinstance(other, int):
            return True
        return str.__ge__(self, other)

    def __gt__(self, other):
        if isinstance(other, int):
            return True
        return str.__gt__(self, other)


class _Py2ArgumentParser(argparse.ArgumentParser):
    def parse_args(self, *a, **k):
        ns = super().parse_args(*a, **k)
        if isinstance(getattr(ns, "maxdel", None), str):
            ns.maxdel = _Py2MaxdelStr(ns.maxdel)
        return ns


def _py2_open(name, mode="r", *a, **k):
    if "w" in mode or "a" in mode:
        return open(name, mode.replace("b", ""), encoding="latin-1", newline="")
    return io.TextIOWrapper(open(name, "rb"), encoding="latin-1", newline="\n")


def _py2_gzip_open(name, mode="rb", *a, **k):
    return io.TextIOWrapper(_gzip.open(name, "rb"), encoding="latin-1", newline="\n")


def _load_code():
    with open(REF_PATH, "r", encoding="utf-8") as fh:
        src = fh.read()
    assert src.count(".iteritems()") == 4, "reference changed: expected 4 iteritems sites"
    return compile(src.replace(".iteritems()", ".items()"), REF_PATH, "exec")


_CODE = None


def run_reference(argv, cwd=None):
    """Run the reference ``main()`` with ``argv`` (list of CLI args, no program name).

    Returns ``(status, stdout_text)`` where status is ``"ok"`` or the name of the
    exception class the reference died with (``"KeyError"``, ``"IndexError"``, ...).
    """
    global _CODE
    if _CODE is None:
        _CODE = _load_code()
    g = {"__name__": "s2c_reference_under_harness", "__file__": REF_PATH}
    exec(_CODE, g)  # defines parsecigar/main, imports modules
    g["round"] = py2_round
    g["open"] = _py2_open
    g["gzip"] = types.SimpleNamespace(open=_py2_gzip_open)
    g["argparse"] = types.SimpleNamespace(
        ArgumentParser=_Py2ArgumentParser,
        RawDescriptionHelpFormatter=argparse.RawDescriptionHelpFormatter)
    old_argv, old_out, old_cwd = sys.argv, sys.stdout, os.getcwd()
    buf = io.StringIO()
    sys.argv = ["sam2consensus.py"] + list(argv)
    sys.stdout = buf
    status = "ok"
    try:
        if cwd:
            os.chdir(cwd)
        g["main"]()
    except SystemExit as e:  # argparse
        status = "SystemExit" if e.code not in (0, None) else "ok"
    except Exception as e:  # noqa: BLE001 - the class IS the result
        status = type(e).__name__
    finally:
        sys.argv, sys.stdout = old_argv, old_out
        os.chdir(old_cwd)
    return status, buf.getvalue()


def run_case(sam_text, args, name="in.sam", gz=False):
    """Write ``sam_text`` to a temp dir, run the reference, collect output files.

    Returns dict(status=..., files={filename: content_latin1_str}).
    """
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, name)
        data = sam_text.encode("latin-1")
        if gz:
            with _gzip.open(path, "wb") as fh:
                fh.write(data)
        else:
            with open(path, "wb") as fh:
                fh.write(data)
        out = os.path.join(td, "out")
        status, _ = run_reference(["-i", path, "-o", out] + list(args))
        files = {}
        if os.path.isdir(out):
            for fn in sorted(os.listdir(out)):
                with open(os.path.join(out, fn), "rb") as fh:
                    files[fn] = fh.read().decode("latin-1")
        return {"status": status, "files": files if status == "ok" else {}}


def run_file(path, args, outdir):
    """Run the reference on an existing SAM/SAM.gz file, writing into ``outdir``."""
    return run_reference(["-i", path, "-o", outdir] + list(args))


if __name__ == "__main__":  # pragma: no cover - manual use
    st, out = run_reference(sys.argv[1:])
    sys.stderr.write(out)
    print(st)
