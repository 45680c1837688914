"""LightGCNOpti (reference model/LightGCNOpti/model.py:14-96) against the reference's own
outputs (tests/golden/lightgcnopti_mid.npz, make_golden_opti.py): e0 = Linear(features)
under torch.manual_seed(42) (same RNG consumption as the reference's construction), and
the L-layer forward. CPU: construction + oracle forward; GPU: the HIP forward."""
import numpy as np
import pytest
import torch

from oracle import lgcn_oracle as O


def _model(g):
    from model.LightGCNOpti.model import LightGCNOpti
    torch.manual_seed(42)
    return LightGCNOpti(int(g["n_users"]), int(g["n_items"]), 64, 3,
                        torch.from_numpy(g["user_features"]),
                        torch.from_numpy(g["item_features"]))


def test_opti_init_matches_reference(golden):
    g = golden("lightgcnopti_mid")
    m = _model(g)
    assert np.array_equal(m.users_emb.weight.detach().numpy(), g["e0_u"])
    assert np.array_equal(m.items_emb.weight.detach().numpy(), g["e0_i"])


@pytest.mark.parametrize("L", [1, 2, 3])
def test_oracle_forward_on_opti_e0(golden, L):
    g = golden("lightgcnopti_mid")
    coo = torch.as_tensor(g["train_coo"].astype(np.int64))
    uf, itf = O.lightgcn_forward(coo, torch.from_numpy(g["e0_u"]), torch.from_numpy(g["e0_i"]), L)
    np.testing.assert_allclose(uf.numpy(), g[f"out_u_L{L}"], atol=1e-6, rtol=0)
    np.testing.assert_allclose(itf.numpy(), g[f"out_i_L{L}"], atol=1e-6, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("L", [1, 2, 3])
def test_gpu_opti_forward_matches_reference(golden, L):
    """north_star tolerance 1e-4 absolute (fp32); observed ~1e-7."""
    g = golden("lightgcnopti_mid")
    m = _model(g).cuda()
    m.layers = L
    uf, u0, itf, i0 = m.forward(torch.as_tensor(g["train_coo"].astype(np.int64)).cuda())
    assert np.abs(uf.detach().cpu().numpy() - g[f"out_u_L{L}"]).max() <= 1e-4
    assert np.abs(itf.detach().cpu().numpy() - g[f"out_i_L{L}"]).max() <= 1e-4
    assert np.array_equal(u0.detach().cpu().numpy(), g["e0_u"])


@pytest.mark.gpu
def test_gpu_spread_opti_douban_matches_reference(golden, monkeypatch, tmp_path):
    """BASELINE configs[2] (Douban-shaped SpreadLightGCNOpti, lambda = 0.5): the package's
    recommendSpreadLightGCNOpti (fused GPU spreading + e0 scores) against the reference's
    own getResourceMat + recommendForAllUser run (spread_opti_douban.npz,
    make_golden_c3.py), both on the untrained seeded LightGCNOpti. Tie-aware at 1e-12 of
    the largest boundary value (fp64 F, BLAS vs ordered sums)."""
    import pandas as pd
    from golden.make_golden_c3 import features
    from const import cfg
    from lgcnhs.synth import synth_dataframes
    import model.SpreadLightGCNOpti.model as SM
    from model.LightGCNOpti.model import LightGCNOpti
    from model.SpreadLightGCNOpti.recommend import recommendSpreadLightGCNOpti
    from _compare import compare_topk_sets
    g = golden("spread_opti_douban")
    U, I, E, k = int(g["n_users"]), int(g["n_items"]), int(g["n_edges"]), int(g["k"])
    rating_df, tr, va, te = synth_dataframes(U, I, E, seed=int(g["seed"]), dist="zipf")
    fu, fi = features(U, I)
    uf_df = pd.DataFrame({"user_id": np.arange(U), "user_features": [list(map(float, r)) for r in fu]})
    if_df = pd.DataFrame({"item_id": np.arange(I), "item_features": [list(map(float, r)) for r in fi]})

    made = []

    def untrained(user_num, item_num, edge_index, train_ei, val_ei, uf, itf, kk):
        torch.manual_seed(42)
        made.append(LightGCNOpti(user_num, item_num, 64, 3, uf, itf).cuda())
        return made[-1]

    monkeypatch.setattr(SM, "load_or_train_opti", untrained)
    saved = (dict(cfg.MODEL), dict(cfg.RECOMMEND))
    try:
        cfg.MODEL["name"] = "SpreadLightGCNOpti"
        cfg.MODEL["HyperParameter"] = {"lambda": float(g["lam"]), "seed": 42,
                                       "embedding_dim": 64, "layers": 3}
        cfg.RECOMMEND["k"] = k
        cfg.RECOMMEND["save_path"] = str(tmp_path) + "/"
        recs = recommendSpreadLightGCNOpti(U, I, rating_df, tr, va, te, uf_df, if_df)
    finally:
        cfg.MODEL.clear(); cfg.MODEL.update(saved[0])
        cfg.RECOMMEND.clear(); cfg.RECOMMEND.update(saved[1])
    got = np.array([recs[u] for u in range(U)])
    from model.SpreadLightGCN.recommend import spread_lightgcn_topk
    vals, idx = spread_lightgcn_topk(made[0], U, I, tr, va, float(g["lam"]), k)
    assert np.array_equal(idx.cpu().numpy(), got)
    gaps = g["gaps"]
    # users with fewer than k positive scores fill their lists with exact ties at 0.0 (F = 0
    # or G*F = -0.0), ordered arbitrarily by the reference's argsort: allowed, but their
    # positive-score prefix must match
    ties = compare_topk_sets(got, g["recs"], gaps, tol=1e-12 * np.nanmax(np.abs(gaps)),
                             max_tie_frac=1.0, got_vals=vals.cpu().numpy())
    exact_ties = int((gaps[:, 0] == gaps[:, 1]).sum())
    print(f"[C3 SpreadLightGCNOpti douban-shape] tie-affected users: {ties} of {U} "
          f"(exact 0.0 ties at the K boundary: {exact_ties})")
    # the exact-tie users (equal k-th / (k+1)-th reference values: any order is the
    # reference's) plus at most 1 % rounding-level ties
    assert ties <= exact_ties + max(1, U // 100)
