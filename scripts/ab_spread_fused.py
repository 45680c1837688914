"""A/B of the factored spreading top-K (K3s) at C5: two-kernel path (F tile through HBM +
16-user MFMA top-K) vs the fused resource+top-K kernel, with and without the G factor.
Usage: python scripts/ab_spread_fused.py [--users 65536] [--tile 2048]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from lgcnhs import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=65536)
    ap.add_argument("--tile", type=int, default=2048)
    ap.add_argument("--workload", default="c5-d64")
    a = ap.parse_args()
    dev = torch.device("cuda")
    U, I, E, D, _ = bench.WORKLOADS[a.workload]
    _, _, keys = bench.gen_graph(U, I, E, 0, dev)
    A = ops.Interactions.from_pairs(keys // I, keys % I, U, I, dev)
    del keys
    g = torch.Generator(device=dev).manual_seed(42)
    eu = torch.randn(U, D, device=dev, generator=g) * 0.1
    ei = torch.randn(I, D, device=dev, generator=g) * 0.1
    n = min(a.users, U)
    out = {"workload": a.workload, "users": n, "tile": a.tile}
    ref = {}
    for use_g in (False, True):
        for fused in (False, True):
            kw = dict(eu=eu, ei=ei) if use_g else {}
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            v, i = ops.spread_topk_tiled(A, 0.5, 20, A.by_user, users=slice(0, n),
                                         tile=a.tile, fused=fused, **kw)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            key = f"{'G' if use_g else 'noG'}_{'fused' if fused else 'two_kernel'}"
            out[key + "_s"] = dt
            if use_g in ref:
                out[key + "_equal"] = bool(torch.equal(i, ref[use_g][1]) and
                                           torch.equal(v.view(torch.int64),
                                                       ref[use_g][0].view(torch.int64)))
            else:
                ref[use_g] = (v, i)
            print(key, f"{dt:.3f}s", file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
