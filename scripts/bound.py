"""What bounds the pileup kernels of a workload, from its PMC passes (scripts/pmc.sh).

    python scripts/bound.py <workload> <pmc dir, e.g. gpurun_out/pmc_c5> <evidence path>
Per launch of the tile kernels (k_tile_dense, k_tile, k_prep), summed: the VALU issue floor
(SQ_INSTS_VALU × 4 clocks per wave64 instruction on one of 1024 SIMDs at 2.4 GHz,
MI355X_MICROARCH.md) and the HBM floor (profiles/traffic_<wl>.json bytes ÷ 8 TB/s), each as
a fraction of the kernels' time under the counters.  The larger one is the bound; writes
profiles/bound_<wl>.json, which bench.py reports as roofline.bound."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TILE = ("s2c::k_tile_dense", "s2c::k_tile", "s2c::k_prep")


def main():
    wl, base, evidence = sys.argv[1], sys.argv[2], sys.argv[3]
    valu, dur = defaultdict(list), defaultdict(list)
    for f in glob.glob(os.path.join(base, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
                if name.split("<")[0] not in TILE:
                    continue
                if row["Counter_Name"] == "SQ_INSTS_VALU":
                    valu[name].append(float(row["Counter_Value"]))
                    dur[name].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
    v = sum(sum(x) / len(x) for x in valu.values())
    t = sum(sum(x) / len(x) for x in dur.values())
    valu_ms = v * 4 / 1024 / 2.4e9 * 1e3
    tr = None
    p = os.path.join(ROOT, "profiles", "traffic_%s.json" % wl)
    if os.path.exists(p):
        tr = json.load(open(p)).get("tile_hbm_bytes_per_launch")
    hbm_ms = tr / 8e12 * 1e3 if tr else None
    fv = valu_ms / t if t else None
    fh = hbm_ms / t if (t and hbm_ms) else None
    bound = "valu" if (fv and (fh is None or fv >= fh)) else "hbm"
    out = {"workload": wl, "bound": bound, "kernels": sorted(valu), "valu_insts_per_launch": v,
           "valu_floor_ms": valu_ms, "hbm_floor_ms": hbm_ms, "kernel_ms_under_counters": t,
           "valu_frac_of_time": fv, "hbm_frac_of_time": fh, "evidence": evidence}
    json.dump(out, open(os.path.join(ROOT, "profiles", "bound_%s.json" % wl), "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
