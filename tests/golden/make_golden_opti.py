"""Generate tests/golden/lightgcnopti_mid.npz from the REFERENCE's own LightGCNOpti
(model/LightGCNOpti/model.py:14-96: e0 = Linear(features), then the LightGCN forward),
run in this container on top of pyg_restated.py (PyG 2.6.1 restated; see make_golden.py).

    python tests/golden/make_golden_opti.py [--ref /root/reference]

Inputs: the "mid" synthetic split of make_golden.py (300 users x 500 items, seed 2) and
seeded feature matrices (numpy default_rng(4)); torch.manual_seed(42) before construction,
as train.py seeds it. Stores the features, the train COO, e0 and the L = 1..3 outputs."""
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
    os.chdir(tempfile.mkdtemp(prefix="lgcn_golden_opti_"))
    sys.path.insert(0, os.path.abspath(args.ref))
    import const
    const.cfg.MODEL["HyperParameter"] = {"lambda": 0.5, "seed": 42, "embedding_dim": 64,
                                         "layers": 3}
    from model.LightGCN.recommend import buildGraph
    from model.LightGCNOpti.model import LightGCNOpti

    U, I, E, seed = 300, 500, 12000, 2
    rating_df, tr, va, te = synth.synth_dataframes(U, I, E, seed=seed)
    _, train_ei, _, _ = buildGraph(U, I, rating_df, tr, va, te)
    rng = np.random.default_rng(4)
    fu = rng.standard_normal((U, 10)).astype(np.float32)
    fi = rng.random((I, 18)).astype(np.float32)
    torch.manual_seed(42)
    model = LightGCNOpti(U, I, 64, 3, torch.from_numpy(fu), torch.from_numpy(fi))
    res = {}
    with torch.no_grad():
        for L in (1, 2, 3):
            model.layers = L
            uf, u0, itf, i0 = model.forward(train_ei)
            res[f"out_u_L{L}"] = uf.numpy()
            res[f"out_i_L{L}"] = itf.numpy()
    meta = np.array("reference=Alex-McAvoy/Light-Graph-Convolutional-Recommendation-"
                    "Algorithm-based-on-Hybrid-Spreading@2025-12-05 LightGCNOpti; "
                    f"torch={torch.__version__}; PyG 2.6.1 restated (pyg_restated.py)")
    np.savez_compressed(os.path.join(out_dir, "lightgcnopti_mid.npz"), meta=meta, n_users=U,
                        n_items=I, seed=seed, user_features=fu, item_features=fi,
                        train_coo=train_ei.numpy().astype(np.int32),
                        e0_u=u0.detach().numpy(), e0_i=i0.detach().numpy(), **res)
    print("lightgcnopti_mid done")


if __name__ == "__main__":
    main()
