"""Summarise rocprofv3 kernel-trace + PMC passes (scripts/gpu_traffic.sh output) into
profiles/: per-kernel average duration, FETCH_SIZE / WRITE_SIZE per launch and the HBM
traffic estimate bench.py reports as roofline.traffic.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) counts half the bytes of
16-B-per-lane streaming/gather reads -> x2; WRITE_SIZE (KiB) is exact for 16-B stores."""
import csv
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"k_spmm_layer": "lg_spmm_layer_f32", "k_score_topk": "lg_score_topk_f32",
        "k_topk_merge": "lg_score_topk_f32(merge)"}


def kernel_key(name):
    for k, v in KEYS.items():
        if k in name:
            return v
    return None


def main(out_dir, tag, workload="c5-d64", world=1, g=None):
    """Per kernel, the launch shape (grid size) with the most total time is the headline
    launch (the bench also runs side configurations); every statistic below is over the
    dispatches of that shape only. g: the passes' directory, holding trace/ fetch/ write/
    (scripts/gpu_traffic.sh: gpurun_out/<out>/k1_<workload>) or prof_trace/ prof_fetch/
    prof_write/ (scripts/profile.sh: gpurun_out)."""
    g = g or os.path.join(REPO, "gpurun_out")
    pre = "prof_" if os.path.isdir(os.path.join(g, "prof_trace")) else ""
    groups = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(g, pre + "trace", "run_kernel_trace.csv"))):
        k = kernel_key(r["Kernel_Name"])
        if k:
            groups[(k, int(r["Grid_Size_X"]))].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    head = {}
    for (k, grid), d in groups.items():
        if k not in head or sum(d) > sum(groups[(k, head[k])]):
            head[k] = grid
    stats = {}
    for k, grid in head.items():
        d = sorted(groups[(k, grid)])
        stats[k] = {"grid_size": grid, "calls": len(d), "avg_ms": sum(d) / len(d),
                    "min_ms": d[0], "max_ms": d[-1]}
    ctr = defaultdict(list)
    for sub in ("fetch", "write", "sq"):
        path = os.path.join(g, pre + sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            k = kernel_key(r["Kernel_Name"])
            if k and k in head and int(r["Grid_Size"]) == head[k]:
                ctr[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in ctr.items():
        unit = "_KiB_per_launch" if c.endswith("_SIZE") else "_per_launch"
        stats[k][c + unit] = sum(v) / len(v)
    for k, s in stats.items():
        # SQ_VALU_MFMA_BUSY_CYCLES = 32 cycles x MFMAs summed over all 1024 SIMDs;
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, SQ counters)
        busy, active = s.get("SQ_VALU_MFMA_BUSY_CYCLES_per_launch"), s.get("GRBM_GUI_ACTIVE_per_launch")
        if busy and active:
            s["mfma_busy_frac"] = busy / (1024 * active / 8)
            s["clock_ghz_profiled"] = active / 8 / (s["avg_ms"] * 1e6)
        if "FETCH_SIZE_KiB_per_launch" in s and "WRITE_SIZE_KiB_per_launch" in s:
            s["hbm_bytes_per_launch"] = (2 * s["FETCH_SIZE_KiB_per_launch"]
                                         + s["WRITE_SIZE_KiB_per_launch"]) * 1024
    os.makedirs(out_dir, exist_ok=True)
    tp = os.path.join(out_dir, "pmc_traffic.json")
    d = json.load(open(tp)) if os.path.exists(tp) else {}
    if "lg_spmm_layer_f32" in stats and "hbm_bytes_per_launch" in stats["lg_spmm_layer_f32"]:
        import hashlib  # the kernel source the counters were measured on (bench.py checks it)
        src = os.path.join(REPO, "light-graph-convolutional-recommendation-algorithm-based-on-"
                           "hybrid-spreading_amd", "csrc", "spmm.hip")
        sha = hashlib.sha256(open(src, "rb").read()).hexdigest()[:16]
        d[f"{workload}/n{world}"] = {"kernel": "lg_spmm_layer_f32", "source": tag,
                                     "kernel_sha": sha, **stats["lg_spmm_layer_f32"]}
    json.dump(d, open(tp, "w"), indent=1)
    print(json.dumps(stats, indent=1))


if __name__ == "__main__":
    # usage: pmc_summary.py TAG [WORKLOAD (c5-d64)] [DIR]
    main(os.path.join(REPO, "profiles"), sys.argv[1] if len(sys.argv) > 1 else "r05",
         sys.argv[2] if len(sys.argv) > 2 else "c5-d64",
         g=sys.argv[3] if len(sys.argv) > 3 else None)
