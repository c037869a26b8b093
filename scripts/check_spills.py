"""Fail the build when a kernel spills: reads the -Rpass-analysis=kernel-resource-usage
remarks hipcc wrote for one source (Makefile) and exits 1 if any kernel's ScratchSize is
not 0 (round 5: a spill of 416 bytes per lane in k_tile's walk-queue instantiation made C2
25 % slower without any other sign).  Other compiler output is passed through."""
import re
import sys


def main(path):
    name, bad = None, []
    with open(path) as f:
        for ln in f:
            if "remark:" not in ln:
                if not re.match(r"^\s*\d*\s*\|", ln) and "remark" not in ln:   # (the remarks' source context)
                    sys.stderr.write(ln)
                continue
            m = re.search(r"Function Name: (\S+)", ln)
            if m:
                name = m.group(1)
            m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", ln)
            if m and int(m.group(1)) > 0:
                bad.append((name, int(m.group(1))))
    for n, s in bad:
        sys.stderr.write("error: kernel %s spills %d bytes per lane to scratch\n" % (n, s))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
