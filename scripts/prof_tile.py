"""Phase clocks of k_tile (diagnostic build): `make prof`, then on the GPU box
   S2C_LIB=libs2c_prof.so python scripts/prof_tile.py [workload]
prints the average s_memtime cycles per sampled workgroup (wave 0) of each phase."""
import ctypes as C
import os
import sys
import time

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
os.environ.setdefault("S2C_LIB", "libs2c_prof.so")
import torch  # noqa: E402

from sam2consensus_amd import _lib, configs  # noqa: E402
from sam2consensus_amd.engine import DeviceBatch, Workspace  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
t0 = time.time()
hb = configs.synth_batch(wl)
i = hb.info
print("batch %.1fs tiles %d items %d dense %d deep %d tile_max %d" % (time.time() - t0, i.n_tiles, i.n_items, i.n_dense,
                                                                     i.n_deep, i.tile_max), flush=True)
args = configs.cli_args(wl)
thr = [float(x) for x in args[args.index("-c") + 1].split(",")] if "-c" in args else [0.25]
ws = Workspace(DeviceBatch(hb), thr, int(args[args.index("-m") + 1]) if "-m" in args else 1, b"-")
f = _lib.lib.s2c_prof_tile
f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
abl = _lib.lib.s2c_prof_tile_ablate   # (1 walk, 2 count, 4 flush atomics; timing only)
abl.argtypes = [C.c_uint32]
abl(int(sys.argv[2]) if len(sys.argv) > 2 else 0)
buf = (C.c_ulonglong * 16)()
ws.run()
torch.cuda.synchronize()
f(buf, 1)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
ev[0].record()
ws.reads()
ev[1].record()
ws.pileup()
ev[2].record()
ws.consensus()
ev[3].record()
torch.cuda.synchronize()
f(buf, 0)
print("k_reads %.4f ms  pileup %.4f ms  consensus %.4f ms" % (ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]),
                                                            ev[2].elapsed_time(ev[3])))
n = max(buf[15], 1)
names = {0: "setup (zero LDS)", 1: "layer DMA + wait", 9: "walk: records, segments", 10: "walk: one-token pieces",
         8: "walk: op walks", 2: "walk: planes wait", 3: "count", 4: "long pieces + flush", 5: "reconstruct counts",
         11: "epilogue: LDS + layout", 6: "epilogue: votes / store"}
tot = sum(buf[k] for k in names)
for k, nm in names.items():
    print("  %-24s %9.0f cyc/wg  %5.1f%%" % (nm, buf[k] / n, 100.0 * buf[k] / max(tot, 1)))
print("  layers/wg %.1f" % (buf[14] / n))
