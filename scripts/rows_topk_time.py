"""Time lg_rows_topk_f64 (ops.rows_topk: the dense spreading path's filtered top-K of G * F)
at the C3 Douban shape (600 users x 20,000 items, k = 20, d = 64, ~100 excluded items per
user) and print a fingerprint of the lists (A/B builds must agree).
Usage: python scripts/rows_topk_time.py [--users 600] [--items 20000] [--k 20]"""
import argparse
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd")]
import torch  # noqa: E402

from lgcnhs import ops  # noqa: E402
from lgcnhs.graph import RowSets  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--users", type=int, default=600)
ap.add_argument("--items", type=int, default=20000)
ap.add_argument("--k", type=int, default=20)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(7)
U, I = a.users, a.items
F = torch.rand(U, I, device=dev, generator=g, dtype=torch.float64)
F = torch.round(F * 4096) / 4096  # (exact ties among F values)
eu = torch.randn(U, 64, device=dev, generator=g) * 0.1
ei = torch.randn(I, 64, device=dev, generator=g) * 0.1
ku = torch.unique(torch.randint(0, U, (U * 100,), device=dev, generator=g) * I +
                  torch.randint(0, I, (U * 100,), device=dev, generator=g))
ex = RowSets.from_pairs(ku // I, ku % I, U, I, dev)
for G in (False, True):
    kw = {"eu": eu, "ei": ei} if G else {}
    v, i = ops.rows_topk(F, a.k, ex, True, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        ops.rows_topk(F, a.k, ex, True, **kw)
    e1.record()
    torch.cuda.synchronize()
    fp = int((i.to(torch.float64) * torch.arange(1, a.k + 1, device=dev)).sum())
    print(f"G={G}: {e0.elapsed_time(e1) / a.reps:.3f} ms  lists fingerprint {fp} "
          f"values sum {float(v[torch.isfinite(v)].sum()):.17g}", flush=True)
