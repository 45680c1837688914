"""Generate tests/golden/eval_mid.npz: the REFERENCE's validation functions
(model/LightGCN/evaluation.py:17-54 getValRecommendations, :56-86 calValLoss) and the
metrics of its periodic-eval block (model/LightGCN/train.py:147-170: getAccurateMetrics on
the val positives, getDiversityMetrics on the train interactions), run in this container
on top of pyg_restated.py (PyG 2.6.1 restated; see make_golden.py).

    python tests/golden/make_golden_eval.py [--ref /root/reference]

Inputs: the "mid" synthetic split of make_golden.py (300 users x 500 items, seed 2),
torch.manual_seed(42) before LightGCN(U, I, 64, 3), k = 20. calValLoss draws its negatives
with PyG's structured_negative_sampling, an RNG stream no device implementation
reproduces, so it is replaced by fixed negatives stored in the fixture (numpy
default_rng(9): one item per val edge that is not one of the user's val items, as PyG's
rejection does); everything else is the reference's code."""
from __future__ import annotations

import argparse
import importlib.util
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PKG = os.path.join(REPO, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd")
K, EPS = 20, 1e-6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default=os.environ.get("LGCN_REFERENCE", "/root/reference"))
    ap.add_argument("--out", default=HERE)
    args = ap.parse_args()
    spec = importlib.util.spec_from_file_location("lgcnhs_synth",
                                                  os.path.join(PKG, "lgcnhs", "synth.py"))
    synth = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(synth)
    out_dir = os.path.abspath(args.out)
    sys.path.insert(0, HERE)
    import pyg_restated
    pyg_restated.install()
    os.chdir(tempfile.mkdtemp(prefix="lgcn_golden_eval_"))
    sys.path.insert(0, os.path.abspath(args.ref))
    import const
    const.cfg.MODEL["HyperParameter"] = {"lambda": 0.5, "seed": 42, "embedding_dim": 64,
                                         "layers": 3}
    from model.LightGCN.recommend import buildGraph
    from model.LightGCN.model import LightGCN
    import model.LightGCN.evaluation as ref_eval
    from metrics.accurate import getAccurateMetrics
    from metrics.diversity import getDiversityMetrics
    from utils.graph import convertAdjMatrixToEdgeIndex
    from utils.trans import (getInteractionMatrixByEdgeIndex, getItemDegreeByUserPosItemDict,
                             getUserItemsDictByEdgeIndex)

    U, I, E, seed = 300, 500, 12000, 2
    rating_df, tr, va, te = synth.synth_dataframes(U, I, E, seed=seed)
    _, train_ei, val_ei, _ = buildGraph(U, I, rating_df, tr, va, te)

    torch.manual_seed(42)
    model = LightGCN(U, I, 64, 3)
    model.eval()
    with torch.no_grad():
        recs = ref_eval.getValRecommendations(model, U, I, train_ei, val_ei, K)
        # K-boundary gaps of the reference's masked score matrix (tie-aware comparison)
        score = torch.matmul(model.users_emb.weight, model.items_emb.weight.T)
        r_tr = convertAdjMatrixToEdgeIndex(U, I, train_ei)
        score[r_tr[0], r_tr[1]] = -(1 << 10)
        top = torch.topk(score, K + 1).values.numpy()
        gaps = top[:, K - 1:K + 1].astype(np.float64)

        # fixed negatives in place of PyG's structured_negative_sampling
        r_val = convertAdjMatrixToEdgeIndex(U, I, val_ei)
        vu, vp = r_val[0].numpy(), r_val[1].numpy()
        pos = {}
        for a, b in zip(vu, vp):
            pos.setdefault(int(a), set()).add(int(b))
        rng = np.random.default_rng(9)
        vn = rng.integers(0, I, vu.size)
        for t in range(vu.size):
            while int(vn[t]) in pos[int(vu[t])]:
                vn[t] = rng.integers(0, I)
        fixed = (torch.from_numpy(vu), torch.from_numpy(vp), torch.from_numpy(vn))
        ref_eval.structured_negative_sampling = lambda ei, contains_neg_self_loops=False: fixed
        val_loss = ref_eval.calValLoss(model, U, I, val_ei, EPS)

        # the eval block's metrics on these recommendations (train.py:115-122,158-160)
        val_pos = getUserItemsDictByEdgeIndex(r_val)
        train_pos = getUserItemsDictByEdgeIndex(r_tr)
        deg = getItemDegreeByUserPosItemDict(train_pos)
        mat = getInteractionMatrixByEdgeIndex(U, I, r_tr)
        P, R, F1, NDCG = getAccurateMetrics(val_pos, recs, K)
        H, Ival = getDiversityMetrics(recs, deg, mat, K)
    meta = np.array("reference=Alex-McAvoy/Light-Graph-Convolutional-Recommendation-"
                    "Algorithm-based-on-Hybrid-Spreading@2025-12-05 LightGCN evaluation; "
                    f"torch={torch.__version__}; PyG 2.6.1 restated (pyg_restated.py); "
                    f"k={K} epsilon={EPS}; val negatives fixed (numpy seed 9)")
    np.savez_compressed(
        os.path.join(out_dir, "eval_mid.npz"), meta=meta, n_users=U, n_items=I, seed=seed,
        k=K, epsilon=EPS, train_coo=train_ei.numpy().astype(np.int32),
        val_coo=val_ei.numpy().astype(np.int32),
        val_triples=np.stack([vu, vp, vn]).astype(np.int32),
        e0_u=model.users_emb.weight.detach().numpy().copy(),
        e0_i=model.items_emb.weight.detach().numpy().copy(),
        val_recs=recs.numpy().astype(np.int32), val_gaps=gaps, val_loss=np.float64(val_loss),
        metrics=np.array([P, R, F1, NDCG, H, Ival], np.float64))
    print("eval_mid done", {"val_loss": val_loss, "P": P, "R": R, "F1": F1, "NDCG": NDCG,
                            "H": H, "I": Ival})


if __name__ == "__main__":
    main()
