"""Tie-aware top-k comparison: the reference's torch.topk / np.argsort
order ties unspecified and its BLAS rounds in its own order, so two correct top-k lists
may differ only where the k-th and (k+1)-th values are within `tol`."""
import numpy as np


def compare_topk_sets(got, ref, gaps=None, tol=0.0, max_tie_frac=0.01):
    """got/ref: [U, k] int arrays (-1 = padding). gaps: [U, 2] = (v_k, v_k+1) of the
    reference row (NaN second entry: fewer than k+1 candidates). Returns the number of
    tie-affected users; raises AssertionError on any other difference."""
    got = np.asarray(got)
    ref = np.asarray(ref)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    bad, ties = [], 0
    for u in range(ref.shape[0]):
        g = set(got[u][got[u] >= 0].tolist())
        r = set(ref[u][ref[u] >= 0].tolist())
        if g == r:
            continue
        if gaps is not None and not np.isnan(gaps[u, 1]) and abs(gaps[u, 0] - gaps[u, 1]) <= tol:
            ties += 1
            continue
        bad.append((u, sorted(g - r), sorted(r - g)))
    assert not bad, f"{len(bad)} users differ beyond ties, first: {bad[:3]}"
    assert ties <= max(1, int(max_tie_frac * ref.shape[0])), f"too many tie-affected users: {ties}"
    return ties
