"""Per-launch HBM traffic of the fused K3s walk (k_tile_walk, lg_spread_tile_resource_topk_f64)
from scripts/gpu_traffic.sh (walk_d<D>/): FETCH_SIZE x 2 + WRITE_SIZE (the gfx950 corrections of
MI355X_MICROARCH.md, as scripts/pmc_summary.py for K1), averaged over the launches after the
first tile (whose list fill makes it atypical), recorded in profiles/pmc_traffic.json under
"<workload>/spread_walk" with the hash of csrc/spread_tiled.hip (bench.py uses it only for that
source). Usage: walk_traffic_summary.py TAG [WORKLOAD (c5-d64)] [DIR (gpurun_out/walk_traffic)]"""
import csv
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
D = os.path.join(REPO, "gpurun_out", "walk_traffic")


def rows(sub, name):
    p = os.path.join(D, sub, name)
    return [r for r in csv.DictReader(open(p)) if "k_tile_walk" in r["Kernel_Name"]]


def main(tag, workload="c5-d64"):
    t = rows("trace", "run_kernel_trace.csv")
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in t][1:]
    f = [float(r["Counter_Value"]) for r in rows("fetch", "run_counter_collection.csv")][1:]
    w = [float(r["Counter_Value"]) for r in rows("write", "run_counter_collection.csv")][1:]
    fk, wk = sum(f) / len(f), sum(w) / len(w)
    src = os.path.join(REPO, "light-graph-convolutional-recommendation-algorithm-based-on-"
                       "hybrid-spreading_amd", "csrc", "spread_tiled.hip")
    sha = hashlib.sha256(open(src, "rb").read()).hexdigest()[:16]
    e = {"kernel": "lg_spread_tile_resource_topk_f64", "source": tag, "kernel_sha": sha,
         "launches": len(dur), "avg_ms": sum(dur) / len(dur),
         "FETCH_SIZE_KiB_per_launch": fk, "WRITE_SIZE_KiB_per_launch": wk,
         "hbm_bytes_per_launch": (2 * fk + wk) * 1024}
    tp = os.path.join(REPO, "profiles", "pmc_traffic.json")
    d = json.load(open(tp)) if os.path.exists(tp) else {}
    d[f"{workload}/spread_walk"] = e
    json.dump(d, open(tp, "w"), indent=1)
    print(json.dumps(e, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 3:
        D = sys.argv[3]
    main(sys.argv[1] if len(sys.argv) > 1 else "r02", sys.argv[2] if len(sys.argv) > 2 else "c5-d64")
