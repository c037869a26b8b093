"""sam2consensus_amd — MI355X-native pileup-and-vote engine behind the sam2consensus.py CLI.

Layers:
  _lib      ctypes binding of libs2c.so (include/s2c.h C-ABI)
  batch     host SAM/SAM.gz parser → packed read batch (C++), parsecigar API mirror
  engine    device buffers (torch as allocator) + the HIP stages
  records   FASTA headers/bodies with the reference's Python-2 number formatting
  cli       the drop-in command line
  configs   BASELINE.json's synthetic workloads C1..C5
  shard     position-range sharding across GPUs (one process per GPU)
"""
from .batch import HostBatch, Parser, parse_file, parse_text, parsecigar  # noqa: F401

__version__ = "0.1.0"
