"""Phase clocks of k_tile_dense (diagnostic build): `make prof`, then on the GPU box
   S2C_LIB=libs2c_prof.so python scripts/prof_dense.py [workload] [ablation bits,...]
prints the average s_memtime cycles per wave of each phase (DMA wait, walk, count, fix-up +
transpose, vote + store) and the per-wave averages of groups, pieces and staged dwords."""
import ctypes as C
import os
import sys
import time

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
os.environ.setdefault("S2C_LIB", "libs2c_prof.so")
import torch  # noqa: E402

from sam2consensus_amd import _lib, configs  # noqa: E402
from sam2consensus_amd.engine import DeviceBatch, Workspace  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c5"
t0 = time.time()
hb = configs.synth_batch(wl)
print("batch %.1fs tiles %d dense %d tile_max %d dense_lds %d" % (time.time() - t0, hb.info.n_tiles, hb.info.n_dense,
                                                                  hb.info.tile_max, hb.info.dense_lds), flush=True)
ws = Workspace(DeviceBatch(hb), [0.25], 1, b"-")
f = _lib.lib.s2c_prof_dense
f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
abl = _lib.lib.s2c_prof_ablate
abl.argtypes = [C.c_uint32]
buf = (C.c_ulonglong * 16)()
names = ["prologue (tile loads, DMA, wait)", "walk fast", "walk slow", "walk N/-", "count", "fixup+transpose", "vote+store"]
bits_list = [int(b) for b in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
for bits in bits_list:
    abl(bits)
    ws.run()
    torch.cuda.synchronize()
    f(buf, 1)
    N = 5
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(N):
        ws.run()
    ev1.record()
    torch.cuda.synchronize()
    f(buf, 0)
    waves = max(buf[8], 1)
    tot = sum(buf[i] for i in range(len(names)))
    print("ablate %d (1 events, 2 count, 4 walk, 8 vote, 16 queued walk, 32 N/- events): step %.3f ms" % (bits, ev0.elapsed_time(ev1) / N))
    for i, nm in enumerate(names):
        print("  %-18s %9.0f cyc/wave  %5.1f%%" % (nm, buf[i] / waves, 100.0 * buf[i] / max(tot, 1)))
    print("  groups/wave %.1f pieces/wave %.1f staged dwords/wave %.0f slow/wave %.2f xq/wave %.2f" % (
        buf[9] / waves, buf[10] / waves, buf[11] / waves, buf[12] / waves, buf[13] / waves), flush=True)
abl(0)
