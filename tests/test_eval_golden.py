"""The validation API of training (reference model/LightGCN/evaluation.py:17-86 and the
periodic-eval block of model/LightGCN/train.py:147-180) against the reference's own run
(tests/golden/eval_mid.npz, make_golden_eval.py), plus the negative sampler's exactness.

CPU: the oracle's op sequence against the fixture; the sampler (device-agnostic torch ops).
GPU: getValRecommendations (lg_score_topk_f32, train-only mask), the val loss on the HIP
forward, the eval block's six metrics, and the training loop's eval rows / CSV."""
import numpy as np
import pytest
import torch

from oracle import lgcn_oracle as O
from _compare import compare_topk_sets


def _pairs(coo, U):
    coo = np.asarray(coo, np.int64)
    m = (coo[0] < U) & (coo[1] >= U)
    return coo[0][m], coo[1][m] - U


def test_oracle_val_recommendations_match_reference(golden):
    g = golden("eval_mid")
    U, I, k = int(g["n_users"]), int(g["n_items"]), int(g["k"])
    tp = _pairs(g["train_coo"], U)
    _, idx, _ = O.recommend_topk_torch(torch.from_numpy(g["e0_u"]), torch.from_numpy(g["e0_i"]),
                                       tp, None, k)
    compare_topk_sets(idx.numpy(), g["val_recs"], g["val_gaps"], tol=1e-6)


def test_oracle_val_loss_matches_reference(golden):
    g = golden("eval_mid")
    U = int(g["n_users"])
    coo = torch.as_tensor(g["val_coo"].astype(np.int64))
    uf, itf = O.lightgcn_forward(coo, torch.from_numpy(g["e0_u"]), torch.from_numpy(g["e0_i"]), 3)
    u, p, n = (torch.as_tensor(r.astype(np.int64)) for r in g["val_triples"])
    e0u, e0i = torch.from_numpy(g["e0_u"]), torch.from_numpy(g["e0_i"])
    loss = O.bpr_loss(uf[u], e0u[u], itf[p], e0i[p], itf[n], e0i[n], float(g["epsilon"]))
    assert round(float(loss), 5) == float(g["val_loss"])
    del U


# ---------------------------------------------------------------------- sampler (CPU)
def test_negatives_exact_for_users_with_few_free_items():
    """A user with 1 or 2 free items out of 200 defeats rejection sampling (64 rounds at
    p = 0.995 of hitting a positive); the exact complement draw must still return only
    free items, uniformly over them."""
    from model.LightGCN import loss as L
    I = 200
    u1 = np.zeros(199, np.int64)
    i1 = np.array([i for i in range(I) if i != 17])            # user 0: only 17 free
    u2 = np.ones(198, np.int64)
    i2 = np.array([i for i in range(I) if i not in (3, 150)])  # user 1: 3 and 150 free
    u3 = np.full(5, 2, np.int64)
    i3 = np.arange(5)
    users = torch.as_tensor(np.concatenate([u1, u2, u3]))
    items = torch.as_tensor(np.concatenate([i1, i2, i3]))
    keys = L._sorted_keys(users, items, I)
    g = torch.Generator().manual_seed(0)
    q = torch.as_tensor([0] * 500 + [1] * 2000 + [2] * 100)
    neg = L._negatives(q, keys, I, generator=g)
    n = neg.numpy()
    assert (n[:500] == 17).all()
    assert set(n[500:2500].tolist()) == {3, 150}
    assert abs(float((n[500:2500] == 3).mean()) - 0.5) < 0.06
    assert not np.isin(n[2500:], np.arange(5)).any()
    full_u = torch.zeros(I, dtype=torch.int64)
    full_keys = L._sorted_keys(full_u, torch.arange(I), I)
    with pytest.raises(ValueError):
        L._negatives(torch.zeros(3, dtype=torch.int64), full_keys, I, generator=g)


def test_structured_negative_sampling_never_returns_positives():
    from model.LightGCN.loss import sampleMiniBatch, structured_negative_sampling
    rng = np.random.default_rng(3)
    U, I = 50, 40
    A = rng.random((U, I)) < 0.9            # dense: most draws are positives
    A[:, 0] = False                         # every user has at least one free item
    uu, ii = np.nonzero(A)
    ei = torch.as_tensor(np.stack([uu, ii]))
    u, p, n = structured_negative_sampling(ei, I, generator=torch.Generator().manual_seed(1))
    assert not A[u.numpy(), n.numpy()].any()
    bu, bp, bn = sampleMiniBatch(4096, ei, I, generator=torch.Generator().manual_seed(2))
    assert A[bu.numpy(), bp.numpy()].all() and not A[bu.numpy(), bn.numpy()].any()


# ---------------------------------------------------------------------------- GPU
def _model(g, dev):
    from model.LightGCN.model import LightGCN
    U, I = int(g["n_users"]), int(g["n_items"])
    m = LightGCN(U, I, 64, 3)
    with torch.no_grad():
        m.users_emb.weight.copy_(torch.from_numpy(g["e0_u"]))
        m.items_emb.weight.copy_(torch.from_numpy(g["e0_i"]))
    return m.to(dev)


@pytest.mark.gpu
def test_gpu_val_recommendations_and_loss_match_reference(golden):
    from model.LightGCN.evaluation import getValRecommendations, val_loss_for_triples
    g = golden("eval_mid")
    U, I, k = int(g["n_users"]), int(g["n_items"]), int(g["k"])
    dev = torch.device("cuda")
    m = _model(g, dev)
    tr = torch.as_tensor(g["train_coo"].astype(np.int64))
    va = torch.as_tensor(g["val_coo"].astype(np.int64))
    recs = getValRecommendations(m, U, I, tr, va, k)
    assert recs.shape == (U, k) and recs.dtype == torch.int64 and recs.is_cuda
    compare_topk_sets(recs.cpu().numpy(), g["val_recs"], g["val_gaps"], tol=1e-6)
    rp, col = O.exclusion_csr(U, I, _pairs(g["train_coo"], U))
    _, oi = O.chain_topk(g["e0_u"], g["e0_i"], rp, col, k)
    np.testing.assert_array_equal(recs.cpu().numpy(), oi)  # the kernel's own chain order
    u, p, n = (torch.as_tensor(r.astype(np.int64), device=dev) for r in g["val_triples"])
    with torch.no_grad():
        vl = val_loss_for_triples(m, va.to(dev), u, p, n, float(g["epsilon"]))
    assert abs(vl - float(g["val_loss"])) <= 1e-5


@pytest.mark.gpu
def test_gpu_eval_block_metrics_match_reference(golden):
    """evaluate_epoch's P/R/F1/NDCG/H/I equal the reference's eval-block values on the
    same recommendations (the lists are tie-free at this fixture's K boundary)."""
    from model.LightGCN.train import ValidationState, evaluate_epoch
    from utils.graph import convertAdjMatrixToEdgeIndex
    g = golden("eval_mid")
    U, I, k = int(g["n_users"]), int(g["n_items"]), int(g["k"])
    dev = torch.device("cuda")
    m = _model(g, dev)
    tr = torch.as_tensor(g["train_coo"].astype(np.int64)).to(dev)
    va = torch.as_tensor(g["val_coo"].astype(np.int64)).to(dev)
    r_train = convertAdjMatrixToEdgeIndex(U, I, tr)
    st = ValidationState(U, I, r_train, va, dev)
    row = evaluate_epoch(m, U, I, tr, va, st, 0, 0.5, k, float(g["epsilon"]),
                         generator=torch.Generator(dev).manual_seed(0))
    got = [row[x] for x in ("val_precision", "val_recall", "val_f1", "val_ndcg", "val_H",
                            "val_I")]
    np.testing.assert_allclose(got, g["metrics"], rtol=0, atol=1.01e-5)
    assert np.isfinite(row["val_loss"])


@pytest.mark.gpu
def test_gpu_training_loop_runs_eval_block(tmp_path):
    from const import cfg
    from lgcnhs.synth import synth_dataframes
    from model.LightGCN.recommend import buildGraph
    from model.LightGCN.train import trainLightGCN
    saved = (dict(cfg.MODEL), dict(cfg.RECOMMEND), dict(cfg.PICTURES))
    try:
        cfg.MODEL["save_path"] = cfg.PICTURES["save_path"] = str(tmp_path) + "/"
        cfg.RECOMMEND["k"] = 10
        cfg.MODEL["HyperParameter"] = {"seed": 42, "embedding_dim": 64, "layers": 3,
                                       "lr": 1e-2, "gamma": 0.95, "epochs": 21,
                                       "epoch_per_eval": 10, "epoch_per_lr_decay": 20,
                                       "batch_size": 256, "epsilon": 1e-6}
        rating_df, tr, va, te = synth_dataframes(150, 220, 4000, seed=5)
        ei, tr_coo, va_coo, _ = buildGraph(150, 220, rating_df, tr, va, te)
        m = trainLightGCN(150, 220, ei, tr_coo, va_coo)
        rows = m.val_metrics
        assert [r["iters"] for r in rows] == [0, 10, 20]
        for r in rows:
            assert all(np.isfinite(r[x]) for x in r)
            assert 0 <= r["val_precision"] <= 1 and 0 <= r["val_H"] <= 1
        import pandas as pd
        df = pd.read_csv(tmp_path / "LightGCN_10_val_metrics.csv")
        assert list(df["iters"]) == [0, 10, 20] and len(df.columns) == 9
    finally:
        cfg.MODEL.clear(); cfg.MODEL.update(saved[0])
        cfg.RECOMMEND.clear(); cfg.RECOMMEND.update(saved[1])
        cfg.PICTURES.clear(); cfg.PICTURES.update(saved[2])
