"""Propagation-only driver and PMC summary for a bench workload (the K1 record of
profiles/pmc_traffic.json for graphs whose forward runs more than one kernel per layer, e.g.
the Zipf(1.1) graph: k_spmm_layer for short rows + k_spmm_segments / k_spmm_long_reduce for
hub rows).
  python scripts/prop_pmc.py run WORKLOAD [STEPS]          (on the box, under rocprofv3)
  python scripts/prop_pmc.py summarize TAG WORKLOAD DIR     (DIR: trace/, fetch/, write/)
The summary sums, per forward layer, the average FETCH_SIZE x 2 + WRITE_SIZE (the gfx950
corrections of MI355X_MICROARCH.md) of the layer's kernels (their launches at the workload's
shape), and records it under '<WORKLOAD>/n1' with the hash of csrc/spmm.hip."""
import csv
import hashlib
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
KERNELS = ("k_spmm_layer", "k_spmm_segments", "k_spmm_long_reduce")


def run(workload, steps):
    import torch
    import bench
    from lgcnhs import _native as NV
    from lgcnhs.dist import RowShard
    dev = torch.device("cuda", 0)
    U, I, E, D, L = bench.WORKLOADS[workload]
    N = U + I
    rowptr, src, _ = bench.gen_graph(U, I, E, seed=3, dev=dev,
                                     dist=bench.GRAPH_DIST.get(workload, "uniform"))
    dis = torch.empty(N, dtype=torch.float32, device=dev)
    NV.check(NV.lib().lg_gcn_norm_f32(NV.ptr(rowptr), N, NV.ptr(dis), NV.stream_handle(dev)), "norm")
    w = torch.empty(src.numel(), dtype=torch.float32, device=dev)
    NV.check(NV.lib().lg_gcn_edge_weight_f32(NV.ptr(rowptr), NV.ptr(src), NV.ptr(dis), N, 0,
                                             NV.ptr(w), NV.stream_handle(dev)), "weights")
    shard = RowShard(rowptr, src, N, 0, 1, dev, weight=w, chunks=1)
    e0 = torch.randn(N, D, device=dev) * 0.1
    el, k_s, _ = bench.time_propagation(shard, shard.permute_rows(dis), e0, D, L, steps, 1, 1, dev)
    print(json.dumps({"workload": workload, "ms_per_step": el / steps * 1e3,
                      "layer_ms": k_s * 1e3}), flush=True)


def summarize(tag, workload, d):
    import bench
    U, I, E, D, L = bench.WORKLOADS[workload]
    dur = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_trace.csv"))):
        k = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
        if k:
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    ctr = defaultdict(lambda: defaultdict(list))
    for sub in ("fetch", "write"):
        for r in csv.DictReader(open(os.path.join(d, sub, "run_counter_collection.csv"))):
            k = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
            if k:
                ctr[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    per = {}
    for k in KERNELS:
        c = ctr.get(k)
        if not c:
            continue
        f = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
        wr = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
        per[k] = {"avg_ms": sum(dur[k]) / max(len(dur[k]), 1), "calls": len(dur[k]),
                  "FETCH_SIZE_KiB_per_launch": f, "WRITE_SIZE_KiB_per_launch": wr,
                  "hbm_bytes_per_launch": (2 * f + wr) * 1024}
    layer = {"hbm_bytes_per_launch": sum(v["hbm_bytes_per_launch"] for v in per.values()),
             "avg_ms": sum(v["avg_ms"] for v in per.values())}
    nnz = 2 * E
    alg = nnz * (8 + 4 * D) + (U + I) * (4 + 4 * D)
    src = os.path.join(REPO, "light-graph-convolutional-recommendation-algorithm-based-on-"
                       "hybrid-spreading_amd", "csrc", "spmm.hip")
    sha = hashlib.sha256(open(src, "rb").read()).hexdigest()[:16]
    tp = os.path.join(REPO, "profiles", "pmc_traffic.json")
    out = json.load(open(tp)) if os.path.exists(tp) else {}
    out[f"{workload}/n1"] = {"kernel": "lg_spmm_layer_f32 + lg_spmm_long_rows_f32 (one layer)",
                             "source": tag, "kernel_sha": sha, **layer,
                             "alg_bytes_per_launch": alg,
                             "traffic_over_alg": layer["hbm_bytes_per_launch"] / alg,
                             "kernels": per}
    json.dump(out, open(tp, "w"), indent=1)
    print(json.dumps(out[f"{workload}/n1"], indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 3)
    else:
        summarize(sys.argv[2], sys.argv[3], sys.argv[4])
