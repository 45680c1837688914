"""Print the first rows where the tiled G walk and the dense path disagree (debug)."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd"), os.path.join(R, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lgcnhs import ops  # noqa: E402
from lgcnhs.synth import synth_interactions  # noqa: E402

DEV = "cuda"
U, I, d, k, tile, lam = 300, 1000, 64, int(sys.argv[1]) if len(sys.argv) > 1 else 10, 64, 0.4
u, i = synth_interactions(U, I, 9000, seed=11, dist="zipf")
A = ops.Interactions.from_pairs(torch.as_tensor(u), torch.as_tensor(i), U, I, DEV)
g = torch.Generator(device=DEV).manual_seed(3)
eu = torch.randn(U, d, device=DEV, generator=g) * 0.1
ei = torch.randn(I, d, device=DEV, generator=g) * 0.1
W = ops.hybrid_weight(ops.spread_general(A), A.k_item, lam)
v0, i0 = ops.spread_topk(A, W, k, A.by_user, drop=True, eu=eu, ei=ei)
v1, i1 = ops.spread_topk_tiled(A, lam, k, A.by_user, drop=True, tile=tile, eu=eu, ei=ei)
F = ops.spread_resource(A, W).cpu().numpy()
G = (eu @ ei.T).cpu().numpy().astype(np.float64)
v0, i0, v1, i1 = v0.cpu().numpy(), i0.cpu().numpy(), v1.cpu().numpy(), i1.cpu().numpy()
n = 0
for r in range(U):
    if np.allclose(v0[r], v1[r], rtol=1e-12, atol=0) and set(i0[r]) == set(i1[r]):
        continue
    print("row", r)
    print(" dense", list(zip(i0[r].tolist(), np.round(v0[r], 8).tolist())))
    print(" tiled", list(zip(i1[r].tolist(), np.round(v1[r], 8).tolist())))
    miss = sorted(set(i0[r]) - set(i1[r]))
    print(" missing", [(j, j // tile, F[r, j], G[r, j], G[r, j] * F[r, j]) for j in miss[:5]])
    n += 1
    if n >= 3:
        break
print("bad rows", n)
