"""Debug: the fused G walk over items [0, 128) for row 0 vs numpy ground truth."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lgcnhs import ops  # noqa: E402
from lgcnhs.synth import synth_interactions  # noqa: E402

DEV = "cuda"
U, I, d, k, tile, lam = 300, 1000, 64, 10, 64, 0.4
u, i = synth_interactions(U, I, 9000, seed=11, dist="zipf")
A = ops.Interactions.from_pairs(torch.as_tensor(u), torch.as_tensor(i), U, I, DEV)
g = torch.Generator(device=DEV).manual_seed(3)
eu = torch.randn(U, d, device=DEV, generator=g) * 0.1
ei = torch.randn(I, d, device=DEV, generator=g) * 0.1
W = ops.hybrid_weight(ops.spread_general(A), A.k_item, lam)
F = ops.spread_resource(A, W).cpu().numpy()
G = (eu @ ei.T).cpu().numpy().astype(np.float64)
rp, col = A.by_user.rowptr.cpu().numpy(), A.by_user.col.cpu().numpy()
for hi in (192, 256):
    v1, i1 = ops.spread_topk_tiled(A, lam, k, A.by_user, drop=True, tile=tile, eu=eu, ei=ei,
                                   items=slice(0, hi))
    r = int(os.environ.get('ROW', '1'))
    s = G[r, :hi] * F[r, :hi]
    s[col[rp[r]:rp[r + 1]][col[rp[r]:rp[r + 1]] < hi]] = -np.inf
    o = np.lexsort((np.arange(hi), -s))[:k]
    ok = set(o.tolist()) == set(i1[r].cpu().tolist())
    print(hi, "ok" if ok else "BAD", "walk", list(zip(i1[r].cpu().tolist(), np.round(v1[r].cpu().numpy(), 5).tolist())), "truth", list(zip(o.tolist(), np.round(s[o], 5).tolist())))
tw = ops.TileWalk(A, 0, U, 0, k, A.by_user, eu, ei, tile)
r = int(os.environ.get('ROW', '1'))
for t0 in (128, 192):
    gb, q = tw.bounds(t0, 64)
    gbn = gb[r].cpu().numpy()
    print("gb row", r, "tile", t0, gbn, "max G", G[r, t0:t0 + 64].max(), "argmax", t0 + G[r, t0:t0 + 64].argmax())
    print("  q row", None if q is None else q[r, :64].cpu().numpy())
sc = ops.HybridScale(A, lam)
print("rb 192..255 max", sc.rb[192:256].max().item(), "rb[204]", sc.rb[204].item())
print("G[r,204]", G[r, 204], "F[r,204]", F[r, 204])
print("excl row0", col[rp[0]:rp[1]][:30])
