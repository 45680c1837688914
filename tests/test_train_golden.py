"""The LightGCN training step (reference model/LightGCN/train.py:26-59,148-151 and
model/LightGCN/loss.py:12-43) against the reference's own two BPR + Adam steps
(tests/golden/train_mid.npz, make_golden_train.py). The mini-batch sampler's RNG stream is
not reproducible across implementations, so both sides use the fixture's fixed
(user, pos, neg) triples; everything else (forward, gathers, BPR with the reference's sign,
backward, Adam) is compared. CPU: the oracle restatement; GPU: the package's
getEmbeddingForBPR + BPRLoss through the HIP forward/backward."""
import numpy as np
import pytest
import torch

from oracle import lgcn_oracle as O

LOSS_TOL = 1e-6      # fp32 loss, absolute
GRAD_TOL = 1e-8      # gradients are <= 1e-4 in magnitude; absolute
EMB_TOL = 1e-4       # north_star: embedding values within 1e-4 (fp32)


def _inputs(g):
    coo = torch.as_tensor(g["train_coo"].astype(np.int64))
    t = torch.as_tensor(g["triples"].astype(np.int64))
    return coo, t


def test_oracle_bpr_step_matches_reference(golden):
    g = golden("train_mid")
    coo, t = _inputs(g)
    loss, gu, gi = O.bpr_step(coo, torch.from_numpy(g["e0_u"]), torch.from_numpy(g["e0_i"]),
                              3, t[0, 0], t[0, 1], t[0, 2], float(g["epsilon"]))
    assert abs(float(loss) - float(g["loss_1"])) <= LOSS_TOL
    np.testing.assert_allclose(gu.numpy(), g["grad_u_1"], atol=GRAD_TOL, rtol=0)
    np.testing.assert_allclose(gi.numpy(), g["grad_i_1"], atol=GRAD_TOL, rtol=0)


@pytest.mark.gpu
def test_gpu_train_steps_match_reference(golden, monkeypatch):
    import model.LightGCN.train as T
    from model.LightGCN.loss import BPRLoss
    from model.LightGCN.model import LightGCN
    g = golden("train_mid")
    coo, t = _inputs(g)
    U, I = int(g["n_users"]), int(g["n_items"])
    dev = torch.device("cuda")
    steps = iter([tuple(r.to(dev) for r in t[s]) for s in range(t.shape[0])])
    monkeypatch.setattr(T, "sampleMiniBatch", lambda batch_size, edge_index, n_items=None: next(steps))
    m = LightGCN(U, I, 64, 3)
    with torch.no_grad():
        m.users_emb.weight.copy_(torch.from_numpy(g["e0_u"]))
        m.items_emb.weight.copy_(torch.from_numpy(g["e0_i"]))
    m = m.to(dev)
    opt = torch.optim.Adam(m.parameters(), lr=float(g["lr"]))
    m.train()
    coo_d = coo.to(dev)
    for s in range(2):
        batch = T.getEmbeddingForBPR(m, U, I, coo_d, int(g["batch"]), dev)
        loss = BPRLoss(*batch, float(g["epsilon"]))
        opt.zero_grad()
        loss.backward()
        if s == 0:
            np.testing.assert_allclose(m.users_emb.weight.grad.cpu().numpy(), g["grad_u_1"],
                                       atol=GRAD_TOL, rtol=0)
            np.testing.assert_allclose(m.items_emb.weight.grad.cpu().numpy(), g["grad_i_1"],
                                       atol=GRAD_TOL, rtol=0)
        opt.step()
        assert abs(loss.item() - float(g[f"loss_{s + 1}"])) <= LOSS_TOL
        assert np.abs(m.users_emb.weight.detach().cpu().numpy() - g[f"emb_u_{s + 1}"]).max() <= EMB_TOL
        assert np.abs(m.items_emb.weight.detach().cpu().numpy() - g[f"emb_i_{s + 1}"]).max() <= EMB_TOL


@pytest.mark.parametrize("seed", [0, 1])
def test_structured_negative_sampling_properties(seed):
    """The sampler (reference loss.py:46-70 via PyG structured_negative_sampling): users and
    positives are the edge list itself, every negative lies in the item range and is never
    one of that user's positives; sampleMiniBatch draws rows of that triple set. Its RNG
    stream differs from PyG's, so the properties are checked, not values (unpinned)."""
    from model.LightGCN.loss import sampleMiniBatch, structured_negative_sampling
    g = torch.Generator().manual_seed(seed)
    U, I = 50, 12                      # dense rows: rejection must loop several times
    keys = torch.unique(torch.randint(0, U * I, (400,), generator=g))
    ei = torch.stack([keys // I, keys % I])
    u, p, n = structured_negative_sampling(ei, I, generator=g)
    assert torch.equal(u, ei[0]) and torch.equal(p, ei[1])
    assert int(n.min()) >= 0 and int(n.max()) < I
    assert not bool(torch.isin(u * I + n, keys).any())
    bu, bp, bn = sampleMiniBatch(64, ei, I, generator=g)
    assert bu.shape == bp.shape == bn.shape == (64,)
    assert bool(torch.isin(bu * I + bp, keys).all())
    assert not bool(torch.isin(bu * I + bn, keys).any())
