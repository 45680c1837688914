import os, sys
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [R, os.path.join(R, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd"), os.path.join(R, "tests")]
import numpy as np, torch
from lgcnhs import ops
from lgcnhs.synth import synth_interactions
U, I = 700, 900
u, i = synth_interactions(U, I, 12000, seed=5, dist="uniform")
A = ops.Interactions.from_pairs(torch.as_tensor(u), torch.as_tensor(i), U, I, "cuda")
stop = I - 37
a = ops.TileWeights(A, 0.5, 64, group=1)
b = ops.TileWeights(A, 0.5, 64, group=8)
for j0 in range(0, stop, 64):
    a.build(j0, stop); b.build(j0, stop)
    nw = a.n_units * 4
    x, y = a.ovf[:nw].cpu().numpy(), b.ovf[:nw].cpu().numpy()
    d = np.nonzero(x != y)[0]
    if d.size:
        print("tile", j0, "grp", b._grp[0], b._grp[2], b._grp[3], "units", a.n_units)
        print("g_base", b.g_base.cpu().numpy())
        bd = a.bound.cpu().numpy(); op = a.ovf_ptr.cpu().numpy(); opb = b.ovf_ptr.cpu().numpy()
        rows = np.nonzero(bd > 31)[0]
        G = b.g_ovf.cpu().numpy()
        base = (b.ovf.data_ptr() - b.g_ovf.data_ptr()) // 4
        for r in rows:
            ou = op[r]; n = x[ou * 4]
            runa = x[ou * 4: (ou + 1 + n) * 4]; runb = y[opb[r] * 4:(opb[r] + 1 + n) * 4]
            ok = np.array_equal(runa, runb)
            where = None
            if not ok:
                # search the run's first data unit anywhere in the group buffer
                pat = runa[4:8]
                for s in range(0, G.size - 4, 4):
                    if np.array_equal(G[s:s + 4], pat):
                        where = s // 4; break
            print(f"row {r} i//4={r//4} bound {bd[r]} ou a {ou} b {opb[r]} n {n} ok {ok} found_at_unit {where} (tile base unit {base//4})")
        break
else:
    print("all equal")
