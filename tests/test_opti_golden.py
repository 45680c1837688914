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
