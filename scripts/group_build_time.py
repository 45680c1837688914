"""Time the group build of the factored spreading (ops.TileWeights.build: lg_spread_group_*)
over the first --tiles item tiles of the C5 graph for each group size in --groups, so the
per-group cost (the gathers over every (item, user) pair) and the per-tile cost separate:
  python scripts/group_build_time.py --groups 2,4,8 --tiles 64"""
import argparse
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from lgcnhs import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--groups", default="2,4,8")
ap.add_argument("--tiles", type=int, default=64)
ap.add_argument("--tile", type=int, default=2048)
ap.add_argument("--workload", default="c5-d64")
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()
dev = torch.device("cuda:0")
U, I, E, D, _ = bench.WORKLOADS[a.workload]
_, _, keys = bench.gen_graph(U, I, E, 0, dev)
A = ops.Interactions.from_pairs(keys // I, keys % I, U, I, dev)
del keys
stop = min(I, a.tiles * a.tile)
ref = None
for g in [int(x) for x in a.groups.split(",")]:
    tw = ops.TileWeights(A, 0.5, a.tile, group=g)
    for rep in range(a.reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        h = torch.zeros((), dtype=torch.int64, device=dev)
        for j0 in range(0, stop, a.tile):
            tw.build(j0, stop=stop)
            if rep == 0:  # (a checksum of the tiles' words: every group size builds the same)
                h += (tw.lines[:I * 32].to(torch.int64) * 1000003 % 998244353).sum()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        if rep == 0:
            hv = int(h)
            ref = hv if ref is None else ref
            continue
        print(f"group {g}: {a.tiles} tiles in {dt * 1e3:.1f} ms = {dt * 1e3 / a.tiles:.3f} ms "
              f"per tile  (tile words checksum {hv}: {'same' if hv == ref else 'DIFFERENT'})",
              flush=True)
    del tw
