"""Fail the build when a kernel spills: reads the -Rpass-analysis=kernel-resource-usage
remarks hipcc wrote for one source (Makefile) and exits 1 if any kernel's ScratchSize is
not 0 (round 5: a spill of 416 bytes per lane in k_tile's walk-queue instantiation made C2
25 % slower without any other sign).  Other compiler output is passed through."""
import re
import sys


# k_tile's workgroups per CU by LDS: 3 for tiles of <= 512 positions (NWP 8 / 16), 2 above.
# The share is the largest measured to keep 3: 53,536 bytes ran at 3 per CU, 54,176 (round 6,
# profiles/r06/d1_*, d2_*) and 54,560 (round 5) bytes ran C2 40-47 % slower with no other sign
# (the occupancy remark does not count the CU's reserved LDS or its allocation granules)
LDS_CAP = {"k_tileILi8E": 53536, "k_tileILi16E": 53536, "k_tileILi32E": 81920, "k_tileILi64E": 81920}


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
            m = re.search(r"LDS Size \[bytes/block\]: (\d+)", ln)
            if m and name:
                for k, cap in LDS_CAP.items():
                    if k in name and int(m.group(1)) > cap:
                        sys.stderr.write("error: kernel %s takes %s bytes of LDS, over its %d-byte share\n"
                                         % (name, m.group(1), cap))
                        bad.append((name, -1))
    for n, s in bad:
        if s < 0:
            continue
        sys.stderr.write("error: kernel %s uses %d bytes of scratch per lane (a register spill, or the kernel arguments copied for an out-of-line call)\n" % (n, s))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
