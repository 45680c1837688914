"""Probe: SpMM layer time of the C5 d=64 graph (same rowptr, same nnz) when every row's
neighbours are folded into a window of S nodes of the other half (src -> base + (src-base) % S).
S = 1M is the real graph; smaller S shows how much a gather set that fits the MALL /
L2 would buy, i.e. the upper bound of a column-slab (cache-blocked) propagation."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from lgcnhs import _native as NV  # noqa: E402
from lgcnhs.dist import RowShard  # noqa: E402

dev = torch.device("cuda")
U, I, E, D, L = bench.WORKLOADS["c5-d64"]
N = U + I
rowptr, src, keys = bench.gen_graph(U, I, E, 0, dev)
del keys
dis = torch.empty(N, dtype=torch.float32, device=dev)
NV.check(NV.lib().lg_gcn_norm_f32(NV.ptr(rowptr), N, NV.ptr(dis), NV.stream_handle(dev)), "n")
wgt = torch.empty(src.numel(), dtype=torch.float32, device=dev)
NV.check(NV.lib().lg_gcn_edge_weight_f32(NV.ptr(rowptr), NV.ptr(src), NV.ptr(dis), N, 0,
                                         NV.ptr(wgt), NV.stream_handle(dev)), "w")
e0 = torch.randn(N, D, device=dev) * 0.1
res = {}
for S in [int(a) for a in (sys.argv[1:] or ["1000000", "500000", "250000", "125000", "31250"])]:
    s64 = src.to(torch.int64)
    folded = torch.where(s64 >= U, U + (s64 - U) % S, s64 % S).to(torch.int32)
    del s64
    shard = RowShard(rowptr, folded, N, 0, 1, dev, weight=wgt, chunks=1)
    el, k, _ = bench.time_propagation(shard, dis, e0, D, L, 5, 2, 1, dev)
    b = shard.nnz * (8 + 4 * D) + shard.n_rows * (4 + 4 * D)
    res[S] = {"ms_layer_kernel": k * 1e3, "alg_GBs": b / k / 1e9,
              "window_MB": S * D * 4 / 2**20}
    print(S, res[S], file=sys.stderr, flush=True)
    del shard, folded
    torch.cuda.empty_cache()
print(json.dumps(res))
