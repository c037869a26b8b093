"""Per-launch HBM traffic of the bench kernels from the PMC passes of scripts/pmc.sh.

    python scripts/traffic.py [workload] [round-tag]
Reads gpurun_out/pmc_<wl>/p3 (FETCH_SIZE) and p4 (WRITE_SIZE), averages every dispatch
of each kernel, applies the gfx950 correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE
reports half the bytes of a 16-B/lane streaming read: ×2) and writes
profiles/traffic_<wl>.json, which bench.py reports as roofline.traffic.  Units: the
rocprofv3 FETCH_SIZE / WRITE_SIZE values are KiB."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path_glob, counter):
    acc = defaultdict(list)
    for f in glob.glob(path_glob, recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter:
                    name = row["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
                    acc[name].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
    tag = sys.argv[2] if len(sys.argv) > 2 else ""
    base = os.path.join(ROOT, "gpurun_out", "pmc_%s" % wl)
    fetch = per_kernel(os.path.join(base, "p3", "**", "*counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(base, "p4", "**", "*counter_collection.csv"), "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f_raw, w_raw = fetch.get(k, 0.0), write.get(k, 0.0)
        kernels[k] = {"fetch_kib_raw": f_raw, "write_kib_raw": w_raw,
                      "hbm_bytes_per_launch": (2.0 * f_raw + w_raw) * 1024.0}
    # the pileup stage of one step: k_tile_dense + k_tile (+ k_prep), summed per launch
    tile = [v for k, v in kernels.items() if k.split("<")[0] in ("s2c::k_tile_dense", "s2c::k_tile", "s2c::k_prep")]
    pile = sum(v["hbm_bytes_per_launch"] for v in tile)
    # the ×2 holds for wide (16 B/lane) streaming reads only: the tile kernels read their
    # windows with buffer_load_dwordx4 … lds (wide) but their descriptors, piece lists and
    # HBM count rows with narrower loads, so the true bytes lie between the raw counter
    # (all reads narrow) and the doubled one (all reads wide); the doubled one is reported
    lo = sum((v["fetch_kib_raw"] + v["write_kib_raw"]) * 1024.0 for v in tile)
    out = {"workload": wl, "round": tag, "kernels": kernels,
           "tile_hbm_bytes_per_launch": pile or None,
           "tile_hbm_bytes_range": [lo, pile] if pile else None,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (scripts/pmc.sh); "
                     "bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 per dispatch, averaged; the x2 is the gfx950 "
                     "read correction of MI355X_MICROARCH.md for wide 16-B/lane reads (the window DMAs); "
                     "the tile kernels' narrower reads (descriptors, piece lists, count rows) make the "
                     "true figure lie in tile_hbm_bytes_range = [raw, doubled]; WRITE_SIZE is uncalibrated for byte stores/atomics. "
                     "Infinity Cache hits are included (a batch below 256 MiB, e.g. C2, is largely served from it)."}
    dst = os.path.join(ROOT, "profiles", "traffic_%s.json" % wl)
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: round(v["hbm_bytes_per_launch"] / 1e6, 3) for k, v in kernels.items()}))


if __name__ == "__main__":
    main()
