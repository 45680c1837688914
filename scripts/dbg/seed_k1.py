"""debug: the seeded k=1 mismatch (tests/test_gpu_topk.py::test_seeded_topk_exclusions_in_seed_range)"""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [R, os.path.join(R, "tests"), os.path.join(R, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd")]
import numpy as np, torch
from test_gpu_topk import _emb, _rowsets, O
from lgcnhs import ops
k = int(sys.argv[1]) if len(sys.argv) > 1 else 1
U, I, d = 200, 65536, 64
eu, ei = _emb(U, d, 51 + k), _emb(I, d, 52)
ei[100:140] = ei[60:100]
g = torch.Generator().manual_seed(53)
eu *= torch.exp(torch.randn(U, 1, generator=g) * 1.5)
eu[9] = 0.0
n_seed = I // 16
G = O.chain_scores(eu.numpy(), ei[:n_seed].numpy())
us, its = [], []
for u in range(U):
    e = (u * 7) % 61
    top = np.argsort(-G[u], kind="stable")[:e]
    us += [u] * e; its += top.tolist()
rng = np.random.default_rng(54)
extra = rng.integers(0, I, 2000)
us += rng.integers(0, U, 2000).tolist(); its += extra.tolist()
rp, col = O.exclusion_csr(U, I, (np.array(us), np.array(its)))
ex = _rowsets(rp, col, U, I)
DEV = torch.device("cuda:0")
for ns in (1,):
    v, i = ops.score_topk(eu.to(DEV), ei.to(DEV), k, ex, n_splits=ns, screen=True)
    v0, i0 = ops.score_topk(eu.to(DEV), ei.to(DEV), k, ex, n_splits=ns, screen=False)
    bad = ((i != i0) | (v.view(torch.int32) != v0.view(torch.int32))).any(1).nonzero().flatten().tolist()
    print("ns", ns, "bad users", len(bad), bad[:10])
    for u in bad[:5]:
        print(" u", u, "E", int(rp[u + 1] - rp[u]), "screen", v[u].tolist()[:4], i[u].tolist()[:4],
              "plain", v0[u].tolist()[:4], i0[u].tolist()[:4])
