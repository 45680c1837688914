"""Host-side glue on CPU (no kernels): the [U, k] -> dict conversion of the recommend
modules (reference model/*/recommend.py dict building)."""
from collections import defaultdict

import numpy as np
import torch


def test_topk_to_dict_trims_padding_and_keeps_order():
    from lgcnhs.recs import topk_to_dict
    idx = torch.tensor([[5, 3, 9], [7, -1, -1], [-1, -1, -1], [0, 1, 2]])
    d = topk_to_dict(idx)
    assert d == {0: [5, 3, 9], 1: [7], 2: [], 3: [0, 1, 2]}
    assert all(type(x) is int for v in d.values() for x in v)
    d2 = topk_to_dict(idx, n_rows=2, factory=defaultdict)
    assert isinstance(d2, defaultdict) and dict(d2) == {0: [5, 3, 9], 1: [7]}
    assert topk_to_dict(torch.zeros((0, 4), dtype=torch.int64)) == {}


def test_topk_to_dict_large_matches_loop():
    from lgcnhs.recs import topk_to_dict
    rng = np.random.default_rng(0)
    a = rng.integers(0, 1000, size=(5000, 20))
    pad = rng.integers(0, 21, size=5000)
    for u in range(5000):
        a[u, pad[u]:] = -1
    d = topk_to_dict(torch.as_tensor(a))
    for u in range(5000):
        assert d[u] == a[u][a[u] >= 0].tolist()


def test_saved_recs_round_trip_without_pickle(tmp_path):
    """save_recs writes the reference's .npy dict plus a pickle-free sidecar; load_recs (what
    main.py's Step 2 reads) returns the dict from the sidecar alone, and an unreadable or
    foreign cache raises one of the errors main.py turns into a recompute."""
    import pytest
    from lgcnhs.recs import CACHE_ERRORS, lists_path, load_recs, save_recs
    recs = {0: [5, 3, 9], 1: [7], 2: [], 3: [0, 1, 2]}
    path = str(tmp_path / "rec" / "all_user_recommend_dict_HybridS_3.npy")
    save_recs(recs, path)
    assert np.load(path, allow_pickle=True).item() == recs  # the reference's format
    got = load_recs(path)
    assert got == recs and all(type(x) is int for v in got.values() for x in v)
    with open(lists_path(path), "wb") as f:  # truncated / corrupt sidecar
        f.write(b"PK\x03\x04 not a zip")
    with pytest.raises(CACHE_ERRORS):
        load_recs(path)
    # a pickled object array under the sidecar's name is refused, never unpickled
    np.savez(lists_path(path), uids=np.array([{"x": 1}], dtype=object))
    with pytest.raises(CACHE_ERRORS):
        load_recs(path)
    with pytest.raises(CACHE_ERRORS):
        load_recs(str(tmp_path / "missing.npy"))


def test_saved_recs_sidecar_follows_its_npy(tmp_path):
    """Deleting the '.npy' (the reference's way to force a recompute) invalidates the sidecar;
    so does a '.npy' newer than it; a rewrite replaces the sidecar whole (no old lists served
    after a failed write)."""
    import os
    import pytest
    from lgcnhs.recs import CACHE_ERRORS, lists_path, load_recs, save_recs
    path = str(tmp_path / "rec" / "all_user_recommend_dict_LightGCN_3.npy")
    save_recs({0: [1, 2]}, path)
    assert load_recs(path) == {0: [1, 2]}
    os.remove(path)
    with pytest.raises(CACHE_ERRORS):
        load_recs(path)
    save_recs({0: [3]}, path)
    assert load_recs(path) == {0: [3]} and not os.path.exists(lists_path(path) + ".tmp.npz")
    t = os.path.getmtime(lists_path(path))
    os.utime(path, (t + 10, t + 10))  # the .npy rewritten after its sidecar
    with pytest.raises(CACHE_ERRORS):
        load_recs(path)


def test_topk_dispatch_guard_follows_the_measured_crossover():
    """ops.screen_pays: the default top-K takes the screened kernel only where it measured
    faster than the plain one (profiles/r06_topk_guard.log) -- the C5 bench shape and the
    2-rank rehearsal shape screen, few-user or small-catalog calls do not."""
    from lgcnhs import ops
    assert ops.screen_pays(32768, 1_000_000, 20) and ops.screen_pays(32768, 1_000_000, 100)
    assert ops.screen_pays(8192, 200_000, 20) and ops.screen_pays(8192, 200_000, 100)
    assert ops.screen_pays(2048, 1_000_000, 100)
    assert not ops.screen_pays(512, 1_000_000, 20)
    assert not ops.screen_pays(8192, 30_000, 20)
    assert not ops.screen_pays(8192, 100_000, 100)
    assert not ops.screen_pays(1, 10**9, 129)  # (beyond the screened kernel's k)
