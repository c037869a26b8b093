#!/usr/bin/env python3
# -*- coding: utf-8 -*-
"""sam2consensus.py — drop-in replacement CLI (same flags and outputs as v2.1) whose
pileup-and-vote path runs as HIP kernels on an AMD Instinct MI355X.

    python sam2consensus.py -i reads.sam[.gz] [-c 0.25,0.5] [-n N] [-o DIR] [-p PREFIX]
                            [-m MIN_DEPTH] [-f FILL] [-d MAXDEL]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from sam2consensus_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
