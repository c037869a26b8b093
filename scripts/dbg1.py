import sys,time; sys.path[:0]=['.','tests','oracle']
import torch
from sam2consensus_amd import configs
from sam2consensus_amd.engine import DeviceBatch, Workspace
name,over,thr,md,fill=("c2", {"n_refs": 3, "depth": 30.0}, [0.1, 0.3, 0.5, 0.6, 0.8, 0.95], 25, b"Nn" * 50)
for thr_, md_, fill_ in [([0.1,0.3],25,b"N"),([0.1,0.3],25,b"Nn"*50),(thr,1,b"-"),(thr,md,fill)]:
    hb=configs.synth_batch(name,**over)
    ws=Workspace(DeviceBatch(hb),thr_,md_,fill_)
    print("case", thr_, md_, len(fill_), flush=True)
    ws.reads(); torch.cuda.synchronize(); print(" reads ok", flush=True)
    ws.pileup(); torch.cuda.synchronize(); print(" pileup ok", flush=True)
    ws.consensus(); torch.cuda.synchronize(); print(" consensus ok", flush=True)
