"""Generate tests/golden/train_mid.npz: two BPR training steps of the REFERENCE's own
LightGCN (model/LightGCN/train.py:26-59 getEmbeddingForBPR, model/LightGCN/loss.py:12-43
BPRLoss, the Adam step of train.py:104,148-151), run in this container on top of
pyg_restated.py (PyG 2.6.1 restated; see make_golden.py).

    python tests/golden/make_golden_train.py [--ref /root/reference]

The mini-batch sampler (loss.py:46-70: PyG structured_negative_sampling + random.choices)
draws from RNG streams that no device implementation reproduces, so the reference's
sampleMiniBatch is replaced by fixed (user, pos, neg) triples stored in the fixture (drawn
here with numpy default_rng(7): a train edge with replacement, a negative item that is not
one of the user's train items). Everything else is the reference's code: forward,
convertAdjMatrixToEdgeIndex, the gathers, BPRLoss (with its sign), backward, Adam.

Inputs: the "mid" synthetic split of make_golden.py (300 users x 500 items, seed 2),
torch.manual_seed(42) before LightGCN(U, I, 64, 3). Stores the loss of each step, the
gradients of step 1 and the parameters after each step."""
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

BATCH, LR, EPS = 512, 1e-3, 1e-6


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
    os.chdir(tempfile.mkdtemp(prefix="lgcn_golden_train_"))
    sys.path.insert(0, os.path.abspath(args.ref))
    import const
    const.cfg.MODEL["HyperParameter"] = {"lambda": 0.5, "seed": 42, "embedding_dim": 64,
                                         "layers": 3}
    from model.LightGCN.recommend import buildGraph
    from model.LightGCN.model import LightGCN
    from model.LightGCN.loss import BPRLoss
    import model.LightGCN.train as ref_train

    U, I, E, seed = 300, 500, 12000, 2
    rating_df, tr, va, te = synth.synth_dataframes(U, I, E, seed=seed)
    _, train_ei, _, _ = buildGraph(U, I, rating_df, tr, va, te)

    # fixed triples in place of the reference's RNG-driven sampler
    tu = tr["user_id"].to_numpy(np.int64)
    ti = tr["item_id"].to_numpy(np.int64)
    pos_sets = {}
    for a, b in zip(tu, ti):
        pos_sets.setdefault(int(a), set()).add(int(b))
    rng = np.random.default_rng(7)
    steps = []
    for _ in range(2):
        pick = rng.integers(0, tu.size, BATCH)
        u, p = tu[pick], ti[pick]
        n = rng.integers(0, I, BATCH)
        for t in range(BATCH):
            while int(n[t]) in pos_sets[int(u[t])]:
                n[t] = rng.integers(0, I)
        steps.append(np.stack([u, p, n]))
    it = iter(steps)
    ref_train.sampleMiniBatch = lambda batch_size, edge_index: tuple(
        torch.from_numpy(r) for r in next(it))

    torch.manual_seed(42)
    model = LightGCN(U, I, 64, 3)
    e0_u = model.users_emb.weight.detach().numpy().copy()
    e0_i = model.items_emb.weight.detach().numpy().copy()
    opt = torch.optim.Adam(model.parameters(), lr=LR)
    model.train()
    res = {}
    for s in range(2):
        batch = ref_train.getEmbeddingForBPR(model, U, I, train_ei, BATCH, torch.device("cpu"))
        loss = BPRLoss(*batch, EPS)
        opt.zero_grad()
        loss.backward()
        if s == 0:
            res["grad_u_1"] = model.users_emb.weight.grad.numpy().copy()
            res["grad_i_1"] = model.items_emb.weight.grad.numpy().copy()
        opt.step()
        res[f"loss_{s + 1}"] = np.float32(loss.item())
        res[f"emb_u_{s + 1}"] = model.users_emb.weight.detach().numpy().copy()
        res[f"emb_i_{s + 1}"] = model.items_emb.weight.detach().numpy().copy()
    meta = np.array("reference=Alex-McAvoy/Light-Graph-Convolutional-Recommendation-"
                    "Algorithm-based-on-Hybrid-Spreading@2025-12-05 LightGCN train step; "
                    f"torch={torch.__version__}; PyG 2.6.1 restated (pyg_restated.py); "
                    f"batch={BATCH} lr={LR} epsilon={EPS}; triples fixed (numpy seed 7)")
    np.savez_compressed(os.path.join(out_dir, "train_mid.npz"), meta=meta, n_users=U,
                        n_items=I, seed=seed, batch=BATCH, lr=LR, epsilon=EPS,
                        train_coo=train_ei.numpy().astype(np.int32),
                        triples=np.stack(steps).astype(np.int32), e0_u=e0_u, e0_i=e0_i, **res)
    print("train_mid done", {k: float(v) for k, v in res.items() if k.startswith("loss")})


if __name__ == "__main__":
    main()
