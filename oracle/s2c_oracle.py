"""CPU restatement of sam2consensus's pileup-and-vote path (TEST INFRASTRUCTURE).

This module is the *oracle*: an independent, pure-Python restatement of the
reference algorithm (``/root/reference/sam2consensus.py`` v2.1), written from
SURVEY.md Appendix A and checked against golden fixtures produced by running
the reference itself (``oracle/gen_golden.py`` → ``tests/golden/``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it, and only as the checker / the timed CPU
baseline.  The product (``sam2consensus_amd``) never imports it.

Parity status: PINNED — every function below is exercised by
``tests/test_oracle.py`` against reference-generated fixtures.

Citations are ``sam2consensus.py:LINE`` of the reference.
"""
from __future__ import annotations

import decimal
import math
import os
import re

CODES = "-ACGNT"                      # sorted() order of the 6 symbols (:167, :367)
CODE = {c: i for i, c in enumerate(CODES)}
_VALID = frozenset(CODES)

# ------------------------------------------------------------------ IUPAC LUT
_IUPAC = {"A": "A", "C": "C", "G": "G", "T": "T", "AC": "M", "AG": "R", "AT": "W",
          "CG": "S", "CT": "Y", "GT": "K", "ACG": "V", "ACT": "H", "AGT": "D",
          "CGT": "B", "ACGT": "N"}


def amb_char(mask):
    """Char for a 6-bit symbol mask (bit i = CODES[i]); None where the reference's
    ``amb`` dict (:317-329) has no entry (→ KeyError).  Rule = SURVEY Appendix A S10."""
    if mask == 0:
        return None
    dash, n = bool(mask & 1), bool(mask & 16)
    b = "".join(c for i, c in enumerate(CODES) if mask >> i & 1 and c in "ACGT")
    if not b:
        return "n" if (dash and n) else ("-" if dash else "N")
    if b == "ACGT":
        if n and not dash:
            return None                          # "ACGNT" is absent from :317-329
        return "N"
    ch = _IUPAC[b]
    return ch.lower() if (dash or n) else ch


AMB_TABLE = [amb_char(m) for m in range(64)]


def mask_key(mask):
    """The dict key the reference builds: ``"".join(sorted(nucs))`` (:367)."""
    return "".join(c for i, c in enumerate(CODES) if mask >> i & 1)


# --------------------------------------------------------- Py2 number formats
def py2_round(x, n=2):
    """CPython 2.7 round(): correctly rounded, exact binary ties away from zero (:395)."""
    x = float(x)
    if x == 0.0 or math.isnan(x) or math.isinf(x):
        return x
    ctx = decimal.Context(prec=400, rounding=decimal.ROUND_HALF_UP)
    return float(decimal.Decimal(x).quantize(decimal.Decimal(1).scaleb(-n), context=ctx))


def py2_str_float(x):
    """CPython 2.7 str(float): '%.12g', with '.0' appended when it looks integral (:395)."""
    r = "%.12g" % x
    if r.lstrip("-").isdigit():
        r += ".0"
    return r


_PY2_WS = re.compile(r"[ \t\n\r\x0b\x0c]+")
_PY2_INT = re.compile(r"[ \t\n\r\x0b\x0c]*([+-]?[0-9]+)[ \t\n\r\x0b\x0c]*\Z")


def py2_split(s):
    """Python 2 ``str.split()`` with no argument (ASCII whitespace)."""
    return [t for t in _PY2_WS.split(s) if t]


def py2_int(s):
    """Python 2 ``int(str)``: ASCII whitespace, sign, decimal digits; else ValueError."""
    m = _PY2_INT.match(s)
    if not m:
        raise ValueError("invalid literal for int() with base 10: %r" % s)
    return int(m.group(1))


# ------------------------------------------------------------------- CIGAR
_CIGAR_RE = re.compile(r"([0-9]+)([MIDNSHPX=])")


def tokenize_cigar(cigar):
    """``re.findall(r"(\\d+)([MIDNSHPX=]{1})")`` (:58-59): non-matching text is skipped."""
    return [(op, int(n)) for n, op in _CIGAR_RE.findall(cigar)]


def parsecigar(cigarstring, seq, pos_ref):
    """Restates ``parsecigar`` (:46-82): returns (seqout, [(ref_pos, motif), ...]).

    M/=/X copy ``seq[start:start+l]`` (truncated when SEQ is short, :67),
    D/N/P emit ``l`` dashes (:71), I records (start_ref, inserted slice) (:74),
    S skips query (:77), H is ignored (:79)."""
    start = 0
    start_ref = pos_ref
    out = []
    ins = []
    for op, ln in tokenize_cigar(cigarstring):
        if op in "=XM":
            out.append(seq[start:start + ln])
            start += ln
            start_ref += ln
        elif op in "DNP":
            out.append("-" * ln)
            start_ref += ln
        elif op == "I":
            ins.append((start_ref, seq[start:start + ln]))
            start += ln
        elif op == "S":
            start += ln
    return "".join(out), ins


# -------------------------------------------------------------------- vote
def vote_groups(counts, cov, t):
    """The reference's vote, restated literally: invert counts into equal-value groups,
    sort descending (:241-251 / :298-308), take groups while acc < t*cov (:359-366)."""
    groups = {}
    for i, v in enumerate(counts):
        if v != 0:
            groups.setdefault(v, []).append(i)
    acc = 0
    mask = 0
    for v, idx in sorted(groups.items(), reverse=True):
        if acc < t * cov:
            for i in idx:
                mask |= 1 << i
            acc += v * len(idx)
        else:
            break
    return mask


def vote_closed(counts, cov, t):
    """Closed form: include i iff c_i != 0 and
    sum_{j: c_j > c_i} c_j < t*cov.  Equal to :vote_groups: (tests/test_oracle.py)."""
    mask = 0
    for i, ci in enumerate(counts):
        if ci == 0:
            continue
        s = sum(cj for cj in counts if cj > ci)
        if s < t * cov:
            mask |= 1 << i
    return mask


def vote_char(counts, cov, t):
    m = vote_groups(counts, cov, t)
    ch = AMB_TABLE[m]
    if ch is None:
        raise KeyError(mask_key(m))
    return ch


# ------------------------------------------------------------------ driver
class Options:
    """The CLI surface (:87-138)."""

    def __init__(self, filename, thresholds="0.25", n=0, outfolder="./", prefix="",
                 min_depth=1, fill="-", maxdel=None):
        self.filename = filename
        self.thresholds = [float(x) for x in thresholds.split(",")]        # :117-118
        self.n = int(n)
        self.outfolder = outfolder.rstrip("/") + "/"                       # :127-130
        self.prefix = prefix if prefix != "" else filename.split("/")[-1].split(".")[0]  # :121-122
        self.min_depth = int(min_depth)
        self.fill = fill
        # :102 -d has no type=: given → a str, and Py2 `int <= str` is always True (:210)
        self.maxdel_active = maxdel is None
        self.maxdel = 150


def parse_argv(argv):
    import argparse
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("-i", "--input", dest="filename", required=True)
    p.add_argument("-c", "--consensus-thresholds", dest="thresholds", default="0.25")
    p.add_argument("-n", dest="n", type=int, default=0)
    p.add_argument("-o", "--outfolder", dest="outfolder", default="./")
    p.add_argument("-p", "--prefix", dest="prefix", default="")
    p.add_argument("-m", "--min-depth", dest="min_depth", type=int, default=1)
    p.add_argument("-f", "--fill", dest="fill", default="-")
    p.add_argument("-d", "--maxdel", dest="maxdel", default=None)
    a = p.parse_args(argv)
    return Options(a.filename, a.thresholds, a.n, a.outfolder, a.prefix, a.min_depth, a.fill, a.maxdel)


def _lines(text):
    """Python-2 line iteration: lines end after each newline (kept); nothing else splits."""
    parts = text.split("\n")
    out = [q + "\n" for q in parts[:-1]]
    if parts[-1]:
        out.append(parts[-1])
    return out


def read_header(lines):
    """First pass (:149-172): leading '@' lines; @SQ → name (:163) and length (:164)."""
    refs = {}
    for line in lines:
        if not line.startswith("@"):
            break
        if line.startswith("@SQ"):
            f = line.split("\t")
            name = py2_split(f[1].replace("SN:", ""))[0]
            refs[name] = max(0, py2_int(f[2].replace("LN:", "")))
    return refs


def pileup(lines, refs, opt):
    """Second pass (:180-228): counts[ref][pos][code] and insertion lists."""
    counts = {r: [[0] * 6 for _ in range(L)] for r, L in refs.items()}
    inserts = {r: [] for r in refs}
    for line in lines:
        if line[0] == "@":                                   # :195
            continue
        f = line.split("\t")
        if len(f) < 6:
            raise IndexError("list index out of range")      # :195 [5]
        if f[5] == "*":
            continue
        tok = py2_split(f[2])
        if not tok:
            raise IndexError("list index out of range")      # :200
        rname = tok[0]
        pos = py2_int(f[3]) - 1                              # :201
        if len(f) < 10:
            raise IndexError("list index out of range")      # :206 [9]
        seqout, ins = parsecigar(f[5], f[9], pos)
        if rname not in counts:
            raise KeyError(rname)                            # :212/:217/:221
        cref = counts[rname]
        L = len(cref)
        drop = opt.maxdel_active and seqout.count("-") > opt.maxdel   # :210
        if not drop and 0 <= pos and pos + len(seqout) <= L and _VALID.issuperset(seqout):
            for ch in seqout:                                # :211-213, nothing can raise
                cref[pos][CODE[ch]] += 1
                pos += 1
            inserts[rname] += ins
            continue
        for ch in seqout:                                    # :211-218
            if not (drop and ch == "-"):
                if not (-L <= pos < L):
                    raise IndexError("list index out of range")
                if ch not in CODE:
                    raise KeyError(ch)
                cref[pos][CODE[ch]] += 1
            pos += 1
        inserts[rname] += ins                                # :221
    return counts, inserts


def insertion_columns(ins_list, cov):
    """:262-311 — {key: [6-count column, ...]} with '-' = cov[key] - sum(column) (:294)."""
    motifs = {}
    for key, motif in ins_list:                              # :264-271
        d = motifs.setdefault(key, {})
        d[motif] = d.get(motif, 0) + 1
    cols = {}
    for key in sorted(motifs):                               # :277-281
        cols[key] = [[0] * 6 for _ in range(max(len(m) for m in motifs[key]))]
    for key in sorted(motifs):                               # :284-287
        for motif, mult in motifs[key].items():
            for c, ch in enumerate(motif):
                if ch not in CODE:
                    raise KeyError(ch)
                cols[key][c][CODE[ch]] += mult
    L = len(cov)
    for key in sorted(cols):                                 # :290-294
        for col in cols[key]:
            if not (-L <= key < L):
                raise IndexError("list index out of range")
            col[0] = cov[key] - sum(col)
    return cols


def consensus(refs, counts, inserts, opt):
    """:232-406 — returns {refname: [(header, seq), ...]} for records kept."""
    covs = {}
    cols = {}
    for r in refs:                                           # :233-311
        covs[r] = [sum(c) for c in counts[r]]
        cols[r] = insertion_columns(inserts[r], covs[r]) if inserts[r] else {}
    fastas = {}
    for r in refs:
        cov = covs[r]
        if sum(cov) == 0:                                    # :334-341
            continue
        cr, ir = counts[r], cols[r]
        for t in opt.thresholds:                             # :348
            out = []
            sumcov = 0
            for p in range(len(cov)):                        # :355-389
                c = cov[p]
                if c == 0:
                    out.append(opt.fill)
                    continue
                sumcov += c
                if c >= opt.min_depth:
                    out.append(vote_char(cr[p], c, t))
                    if p in ir:
                        for col in ir[p]:
                            ch = vote_char(col, c, t)
                            if ch != "-":
                                out.append(ch)
                                sumcov += c
                else:
                    out.append(opt.fill)
            seq = "".join(out)
            tag = str(int(t * 100))                          # :394 (ValueError/OverflowError)
            cov_s = py2_str_float(py2_round(float(sumcov) / float(len(seq)), 2))  # :395
            nondash = len(seq.replace("-", ""))
            hdr = (">" + opt.prefix + "|c" + tag + " reference:" + r + " coverage:" + cov_s +
                   " length:" + str(nondash) + " consensus_threshold:" + tag + "%")
            if nondash > 0:                                  # :400-406
                fastas.setdefault(r, []).append((hdr, seq))
    return fastas


def render(fastas, opt):
    """:411-418 — {filename: file content}."""
    files = {}
    n = opt.n
    for r, recs in fastas.items():
        if n == 0:
            body = "\n".join(h + "\n" + s for h, s in recs) + "\n"
        else:
            body = "\n".join(h + "\n" + "\n".join(s[i:i + n] for i in range(0, len(s), n))
                             for h, s in recs) + "\n"
        files[r + "__" + opt.prefix + ".fasta"] = body
    return files


def run_text(sam_text, opt):
    """Whole pipeline on SAM text.  Returns {filename: content}; raises the reference's
    exception class on failure."""
    lines = _lines(sam_text)
    refs = read_header(lines)
    counts, inserts = pileup(lines, refs, opt)
    return render(consensus(refs, counts, inserts, opt), opt)


def run_case(sam_text, args, name="in.sam"):
    """Mirror of ``oracle/ref_harness.run_case``: status + files, no disk I/O."""
    opt = parse_argv(["-i", name] + list(args))
    try:
        files = run_text(sam_text, opt)
    except (KeyError, IndexError, ValueError, ZeroDivisionError, OverflowError) as e:
        return {"status": type(e).__name__, "files": {}}
    return {"status": "ok", "files": files}


def run_path(path, args):
    """Run on a SAM / SAM.gz path (bench cpu_baseline and large tests)."""
    import gzip
    opt = parse_argv(["-i", path] + list(args))
    raw = gzip.open(path, "rb").read() if path.endswith(".gz") else open(path, "rb").read()
    return run_text(raw.decode("latin-1"), opt), opt


if __name__ == "__main__":  # pragma: no cover
    import sys
    files, opt = run_path(sys.argv[1], sys.argv[2:])
    os.makedirs(opt.outfolder, exist_ok=True)
    for fn, body in files.items():
        with open(opt.outfolder + fn, "w", encoding="latin-1", newline="") as fh:
            fh.write(body)
