"""K3s v2 diagnostics on the C5 graph: tightness of the chunk score bounds (gb against the
true chunk maximum of the fp32 score) and walk timing without / with the G factor."""
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from lgcnhs import ops  # noqa: E402

dev = torch.device("cuda:0")
U, I, E, D, _ = bench.WORKLOADS["c5-d64"]
g = torch.Generator(device=dev).manual_seed(42)
eu = torch.randn(U, D, device=dev, generator=g) * 0.1
ei = torch.randn(I, D, device=dev, generator=g) * 0.1
ub, un = ops.bound_operands(eu[:4096])
ib, inn = ops.bound_operands(ei)
gb = ops.chunk_bounds(ub, un, ib, inn, D, 0, 2048)
G = eu[:4096] @ ei[:2048].T
gmax = G.view(4096, 32, 64).max(-1).values
d = gb - gmax
print(f"bound - chunk max: min {d.min().item():.4g} mean {d.mean().item():.4g} max {d.max().item():.4g}"
      f" (score sd {G.std().item():.4g}); violations {(d < 0).sum().item()}", flush=True)
_, _, keys = bench.gen_graph(U, I, E, 0, dev)
A = ops.Interactions.from_pairs(keys // I, keys % I, U, I, dev)
del keys
for label, kw in (("no G", {}), ("G", {"eu": eu, "ei": ei})):
    for rep in range(2):
        torch.cuda.synchronize()
        t = time.time()
        ops.spread_topk_tiled(A, 0.5, 20, A.by_user, tile=2048, items=slice(0, 16 * 2048), **kw)
        torch.cuda.synchronize()
        print(f"{label} rep {rep}: 16 tiles {time.time() - t:.3f} s", flush=True)
