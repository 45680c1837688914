"""Tie-aware top-k comparison: the reference's torch.topk / np.argsort
order ties unspecified and its BLAS rounds in its own order, so two correct top-k lists
may differ only where the k-th and (k+1)-th values are within `tol`."""
import numpy as np


def compare_topk_sets(got, ref, gaps=None, tol=0.0, max_tie_frac=0.01, got_vals=None):
    """got/ref: [U, k] int arrays (-1 = padding). gaps: [U, 2] = (v_k, v_k+1) of the
    reference row (NaN second entry: fewer than k+1 candidates). Returns the number of
    tie-affected users; raises AssertionError on any other difference. With got_vals
    ([U, k] values of got), a tie-affected user must still agree above the tie: the m items
    of got whose values exceed v_k + tol are the reference's first m items (as sets)."""
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
            if got_vals is not None:
                m = int(np.sum(np.asarray(got_vals[u]) > gaps[u, 0] + tol))
                if set(got[u][:m].tolist()) != set(ref[u][:m].tolist()):
                    bad.append((u, "above the tie", got[u][:m].tolist(), ref[u][:m].tolist()))
                    continue
            ties += 1
            continue
        bad.append((u, sorted(g - r), sorted(r - g)))
    assert not bad, f"{len(bad)} users differ beyond ties, first: {bad[:3]}"
    assert ties <= max(1, int(max_tie_frac * ref.shape[0])), f"too many tie-affected users: {ties}"
    return ties


def compare_topk_exact(got, ref, exact, tol, label=""):
    """Top-k sets against a reference computed in a different rounding order, judged by
    exact (fp64) scores. got/ref: [U, k] item ids (-1 = padding); exact(u, items) -> fp64
    exact scores of those items for user u; tol(u, items) -> a rigorous bound on how far
    either method's rounded score of each item can be from its exact score.

    A user whose two sets differ is *tie-affected* when every item in the symmetric
    difference has an exact score within its tolerance (plus the boundary item's) of the
    reference's k-th exact score: some rounding within the bounds orders it either way.
    Any other difference fails. Returns (tie-affected users, users compared) and prints
    the count (the north_star parity claim is "identical top-K sets except rounding-level
    ties", so the number is reported, not hidden)."""
    got = np.asarray(got)
    ref = np.asarray(ref)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    bad, ties = [], 0
    for u in range(ref.shape[0]):
        g = set(got[u][got[u] >= 0].tolist())
        r = set(ref[u][ref[u] >= 0].tolist())
        if g == r:
            continue
        rl = np.array(sorted(r), np.int64)
        er = exact(u, rl)
        b = int(np.argmin(er))
        eb, tb = er[b], tol(u, rl[b:b + 1])[0]
        diff = np.array(sorted(g ^ r), np.int64)
        ed, td = exact(u, diff), tol(u, diff)
        if np.all(np.abs(ed - eb) <= td + tb):
            ties += 1
            continue
        bad.append((u, sorted(g - r), sorted(r - g), float(np.max(np.abs(ed - eb) - td - tb))))
    print(f"[{label}] tie-affected users: {ties} of {ref.shape[0]}")
    assert not bad, f"{label}: {len(bad)} users differ beyond rounding ties, first: {bad[:3]}"
    return ties, ref.shape[0]


def compare_lists_close(got_v, got_i, ref_v, ref_i, rtol=1e-12, label=""):
    """Two sorted top-k lists of the same scores computed in different summation orders
    (e.g. the factored K3s walk against the dense spreading path): per row the same number
    of entries, values position-wise within rtol, and the same item sets except near-ties,
    where every differing item's value lies within rtol of the reference row's k-th value.
    Returns the number of tie-affected rows (printed)."""
    got_v, got_i = np.asarray(got_v), np.asarray(got_i)
    ref_v, ref_i = np.asarray(ref_v), np.asarray(ref_i)
    assert got_v.shape == ref_v.shape == got_i.shape == ref_i.shape
    ties, bad = 0, []
    for u in range(ref_v.shape[0]):
        mg, mr = got_i[u] >= 0, ref_i[u] >= 0
        if mg.sum() != mr.sum():
            bad.append((u, "lengths", int(mg.sum()), int(mr.sum())))
            continue
        vg, vr = got_v[u][mg], ref_v[u][mr]
        scale = np.maximum(np.abs(vr), np.finfo(np.float64).tiny)
        if not np.all(np.abs(vg - vr) <= rtol * scale):
            bad.append((u, "values", float(np.max(np.abs(vg - vr) / scale))))
            continue
        g, r = set(got_i[u][mg].tolist()), set(ref_i[u][mr].tolist())
        if g == r:
            continue
        vk = vr[-1]
        val = dict(zip(got_i[u][mg].tolist(), vg.tolist()))
        val.update(zip(ref_i[u][mr].tolist(), vr.tolist()))
        if all(abs(val[x] - vk) <= rtol * max(abs(vk), np.finfo(np.float64).tiny) for x in g ^ r):
            ties += 1
            continue
        bad.append((u, "items", sorted(g - r), sorted(r - g)))
    if label:
        print(f"[{label}] tie-affected rows: {ties} of {ref_v.shape[0]}")
    assert not bad, f"{label}: {len(bad)} rows differ beyond rounding, first: {bad[:3]}"
    return ties
