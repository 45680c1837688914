"""Probe: per-GPU time of one full L-layer forward of the C5 graph when each GPU holds a
column slab of width dc of the embeddings (column-sharded propagation: d/dc GPUs, no
exchange). Prints ms per forward and per layer for each dc."""
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
U, I, E, _, L = bench.WORKLOADS["c5-d64"]
N = U + I
rowptr, src, keys = bench.gen_graph(U, I, E, 0, dev)
del keys
dis = torch.empty(N, dtype=torch.float32, device=dev)
NV.check(NV.lib().lg_gcn_norm_f32(NV.ptr(rowptr), N, NV.ptr(dis), NV.stream_handle(dev)), "n")
wgt = torch.empty(src.numel(), dtype=torch.float32, device=dev)
NV.check(NV.lib().lg_gcn_edge_weight_f32(NV.ptr(rowptr), NV.ptr(src), NV.ptr(dis), N, 0,
                                         NV.ptr(wgt), NV.stream_handle(dev)), "w")
shard = RowShard(rowptr, src, N, 0, 1, dev, weight=wgt, chunks=1)
res = {}
for dc in [int(a) for a in (sys.argv[1:] or ["8", "16", "32", "64"])]:
    e0 = torch.randn(N, dc, device=dev) * 0.1
    el, k = bench.time_propagation(shard, dis, e0, dc, L, 5, 2, 1, dev)
    b = shard.nnz * (8 + 4 * dc) + shard.n_rows * (4 + 4 * dc)
    res[dc] = {"ms_forward": el / 5 * 1e3, "ms_layer_kernel": k * 1e3,
               "alg_GBs": b / k / 1e9}
    print(dc, res[dc], file=sys.stderr, flush=True)
    del e0
print(json.dumps(res))
