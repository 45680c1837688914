"""A/B check of lg_score_chunk_bound between two builds (LGCNHS_LIB_PATH of this process vs
the library named by --other, run in a child): the gb and q bytes must agree bit for bit.
Prints where they differ. Usage: python scripts/bound_ab_diff.py --other LIB [--users U]
[--width W] [--dim D]"""
import argparse
import os
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd")]
import numpy as np  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--other", default=None)
ap.add_argument("--users", type=int, default=300)
ap.add_argument("--width", type=int, default=333)
ap.add_argument("--dim", type=int, default=64)
ap.add_argument("--dump", default=None)
a = ap.parse_args()


def run(dump):
    import torch
    from lgcnhs import ops
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(5)
    eu = torch.randn(a.users, a.dim, generator=g) * 0.1
    ei = torch.randn(40 + a.width + 5, a.dim, generator=g) * 0.1
    ub, un = ops.bound_operands(eu.to(dev))
    ib, inn = ops.bound_operands(ei.to(dev))
    qs = -(-a.width // 256) * 256
    q = torch.zeros((a.users, qs), dtype=torch.uint8, device=dev)
    gb, q = ops.chunk_bounds(ub, un, ib, inn, a.dim, 40, a.width, qout=q)
    np.savez(dump, gb=gb.cpu().numpy(), q=q.cpu().numpy()[:, :a.width])


if a.dump:
    run(a.dump)
    sys.exit(0)
env = dict(os.environ, LGCNHS_LIB_PATH=a.other)
subprocess.run([sys.executable, __file__, "--users", str(a.users), "--width", str(a.width),
                "--dim", str(a.dim), "--dump", "/tmp/ab_other.npz"], env=env, check=True)
run("/tmp/ab_self.npz")
x, y = np.load("/tmp/ab_self.npz"), np.load("/tmp/ab_other.npz")
print("gb equal:", np.array_equal(x["gb"].view(np.int32), y["gb"].view(np.int32)))
d = x["q"] != y["q"]
print("q differ:", int(d.sum()), "of", d.size)
if d.any():
    r, c = np.nonzero(d)
    print("rows", np.unique(r)[:40], "n rows", len(np.unique(r)))
    print("cols mod 64 hist", np.bincount(c % 64, minlength=64))
    print("chunks", np.unique(c // 64))
    print("users mod 64 hist", np.bincount(r % 64, minlength=64))
    for i in range(min(12, len(r))):
        print(r[i], c[i], x["q"][r[i], c[i]], y["q"][r[i], c[i]])
