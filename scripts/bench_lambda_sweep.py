"""Time findLambda's loop (reference findLambda.py:74-114: 101 lambda values 0, 0.01, ..., 1,
each HybridS -> A @ W -> G * F -> filtered top-k) through ops.spread_lambda_sweep, which builds
general_W (dense) or the lambda-independent W tiles (tiled) once and only rescales per lambda.

  c3: Douban shape (600 users x 20,000 items, 60,000 Zipf interactions), dense fp64 path
  c4: 200K x 200K, 20M uniform interactions, item-tiled path (tiles cached on the device)

Prints one JSON line per shape: seconds for all lambdas, per lambda, and the first lambda
(which includes the general_W / tile build). Synthetic data, e0 ~ N(0, 0.1^2), d = 64, k = 20.
Usage: python scripts/bench_lambda_sweep.py [--shapes c3,c4] [--lambdas 101]"""
import argparse
import json
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lgcnhs import ops  # noqa: E402
from lgcnhs.synth import synth_graph_device, synth_interactions  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shapes", default="c3,c4")
ap.add_argument("--lambdas", type=int, default=101)
a = ap.parse_args()
dev = torch.device("cuda:0")
lams = np.linspace(0.0, 1.0, a.lambdas).round(2).tolist()
for shape in a.shapes.split(","):
    if shape == "c3":
        U, I, E = 600, 20_000, 60_000
        u, i = synth_interactions(U, I, E, seed=3, dist="zipf")
        A = ops.Interactions.from_pairs(torch.as_tensor(u), torch.as_tensor(i), U, I, dev)
        tiled = False
    else:
        U, I, E = 200_000, 200_000, 20_000_000
        _, _, keys = synth_graph_device(U, I, E, 0, dev)
        A = ops.Interactions.from_pairs(keys // I, keys % I, U, I, dev)
        del keys
        tiled = True
    g = torch.Generator(device=dev).manual_seed(42)
    eu = torch.randn(U, 64, device=dev, generator=g) * 0.1
    ei = torch.randn(I, 64, device=dev, generator=g) * 0.1
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    marks = []
    for lam, v, idx in ops.spread_lambda_sweep(A, lams, 20, A.by_user, True, eu, ei, tiled=tiled):
        torch.cuda.synchronize()
        marks.append(time.perf_counter() - t0)
    dt = marks[-1]
    print(json.dumps({"shape": shape, "users": U, "items": I, "interactions": E,
                      "path": "tiled (W tiles cached)" if tiled else "dense general_W",
                      "lambdas": len(lams), "seconds": dt, "first_lambda_s": marks[0],
                      "per_lambda_after_first_s": (dt - marks[0]) / max(1, len(lams) - 1)}),
          flush=True)
    del A, eu, ei
    torch.cuda.empty_cache()
