"""ORACLE — CPU restatement of the reference's hot path. TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the CPU baseline; the product package never
imports it (tests/test_no_oracle_in_product.py enforces that).

What it restates (reference = Alex-McAvoy/Light-Graph-Convolutional-Recommendation-
Algorithm-based-on-Hybrid-Spreading @ 2025-12-05; citations are file:line there):

* utils/graph.py:12-35     convertEdgeIndexToAdjMatrix -> coalesced symmetric COO
* PyG 2.6.1 (torch-geometric==2.6.1, environment.yaml:276; absent from this image, so its
  published algorithm is restated): gcn_norm(add_self_loops=False) and
  MessagePassing.propagate(aggr='add', flow='source_to_target') as called by
  model/LightGCN/model.py:53,62,84
* model/LightGCN/model.py:32-38,40-74  init + forward (stack/mean/split)
* model/LightGCN/recommend.py:83-114   e0 scoring, -1024 masks, torch.topk
* model/SpreadLightGCN/model.py:74-104,151  getAllocateMat, G * F
* model/SpreadMethod/model.py:14-99    getSpreadingGeneralMat, ProbS, HeatS, HybridS,
                                        getResource
* model/SpreadMethod/recommend.py:18-111 recommendForAllUser (argsort + filter, the
                                        ML-ProbS unfiltered quirk), recommendSpreadMethod
                                        (lambda / transpose overrides)
* utils/trans.py:13-29,51-80           interaction matrix and user->items dicts
* metrics/accurate.py:11-102           precision / recall / F1 / NDCG (its fp32 torch ops)
* metrics/diversity.py:15-115          Hamming distance, internal similarity (its loops)

Pinning: tests/golden/make_golden.py runs the reference's own importable modules
(SpreadMethod, utils/trans) unmodified, and its LightGCN modules on top of a PyG 2.6.1
restatement, to produce tests/golden/*.npz; tests/test_oracle_golden.py checks this
oracle against those fixtures.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
MASK = float(-(1 << 10))  # model/LightGCN/recommend.py:101,111


# ----------------------------------------------------------------------------------
# graph format: utils/graph.py:12-35
# ----------------------------------------------------------------------------------
def coo_adjacency(n_users: int, n_items: int, users, items) -> np.ndarray:
    """convertEdgeIndexToAdjMatrix: R[u][i] = 1 (duplicates collapse), the symmetric
    (U+I)^2 block matrix, ``to_sparse_coo().indices()``: int64 [2, nnz] sorted by
    (row, col) with items offset by U."""
    users = np.asarray(users, dtype=np.int64)
    items = np.asarray(items, dtype=np.int64) + n_users
    n = n_users + n_items
    rows = np.concatenate([users, items])
    cols = np.concatenate([items, users])
    keys = np.unique(rows * n + cols)
    return np.stack([keys // n, keys % n])


def coo_to_interactions(n_users: int, n_items: int, edge_index: np.ndarray) -> np.ndarray:
    """convertAdjMatrixToEdgeIndex (utils/graph.py:38-50): the user->item block of the
    symmetric COO back as a sorted [2, E] (user, item) array."""
    r, c = np.asarray(edge_index[0]), np.asarray(edge_index[1])
    m = (r < n_users) & (c >= n_users)
    keys = np.unique(r[m] * n_items + (c[m] - n_users))
    return np.stack([keys // n_items, keys % n_items])


# ----------------------------------------------------------------------------------
# PyG 2.6.1 restated (torch CPU, fp32)
# ----------------------------------------------------------------------------------
def gcn_norm(edge_index: torch.Tensor, num_nodes: int | None = None):
    """torch_geometric.nn.conv.gcn_conv.gcn_norm(edge_index, add_self_loops=False),
    flow='source_to_target': deg = scatter_add(ones, col); dis = deg.pow(-0.5);
    dis[inf] = 0; w = dis[row] * 1 * dis[col]."""
    if num_nodes is None:
        num_nodes = int(edge_index.max()) + 1 if edge_index.numel() else 0
    row, col = edge_index[0], edge_index[1]
    w = torch.ones(row.numel(), dtype=torch.float32)
    deg = torch.zeros(num_nodes, dtype=torch.float32).scatter_add_(0, col, w)
    dis = deg.pow(-0.5)
    dis.masked_fill_(dis == float("inf"), 0)
    return edge_index, dis[row] * w * dis[col]


def propagate(edge_index: torch.Tensor, w: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """MessagePassing.propagate, aggr='add': x_j = x.index_select(0, row);
    msg = w.view(-1,1) * x_j (model/LightGCN/model.py:84); out[col] += msg."""
    row, col = edge_index[0], edge_index[1]
    msg = w.view(-1, 1) * x.index_select(0, row)
    out = torch.zeros_like(x)
    out.index_add_(0, col, msg)
    return out


def lightgcn_init(n_users: int, n_items: int, dim: int, seed: int = 42):
    """model/LightGCN/model.py:32-38 under torch.manual_seed(seed)
    (model/LightGCN/train.py:91): Embedding(U) then Embedding(I) are constructed (each
    consuming its default N(0,1) init), then normal_(std=0.1) users, then items."""
    torch.manual_seed(seed)
    eu = torch.nn.Embedding(n_users, dim)
    ei = torch.nn.Embedding(n_items, dim)
    torch.nn.init.normal_(eu.weight, std=0.1)
    torch.nn.init.normal_(ei.weight, std=0.1)
    return eu.weight.detach().clone(), ei.weight.detach().clone()


def lightgcn_forward(edge_index: torch.Tensor, emb_u: torch.Tensor, emb_i: torch.Tensor,
                     layers: int):
    """model/LightGCN/model.py:53-74: (users_final, items_final)."""
    n_users = emb_u.shape[0]
    n = n_users + emb_i.shape[0]
    ei_norm, w = gcn_norm(edge_index, None)
    emb = torch.cat([emb_u, emb_i])
    embs = [emb]
    for _ in range(layers):
        emb = propagate(ei_norm, w, emb)
        embs.append(emb)
    final = torch.stack(embs, dim=1).mean(dim=1)
    del n
    return torch.split(final, [n_users, emb_i.shape[0]])


# ----------------------------------------------------------------------------------
# training step: model/LightGCN/train.py:26-59,148-151, model/LightGCN/loss.py:12-43
# ----------------------------------------------------------------------------------
def bpr_loss(uf, u0, pf, p0, nf, n0, lambda_val: float):
    """loss.py:28-43, with its sign: -mean(softplus(pos - neg)) + lambda * sum of squared
    L2 norms of the batch's e0 rows."""
    reg = lambda_val * (u0.norm(2).pow(2) + p0.norm(2).pow(2) + n0.norm(2).pow(2))
    pos = torch.sum(uf * pf, dim=-1)
    neg = torch.sum(uf * nf, dim=-1)
    return -torch.mean(torch.nn.functional.softplus(pos - neg)) + reg


def bpr_step(edge_index, emb_u, emb_i, layers: int, users, pos, neg, lambda_val: float):
    """One getEmbeddingForBPR + BPRLoss + backward on leaf copies of (emb_u, emb_i) for
    fixed (users, pos, neg) triples (train.py:50-57 gathers; item ids are 0-based):
    returns (loss, grad_u, grad_i)."""
    eu = emb_u.detach().clone().requires_grad_(True)
    ei = emb_i.detach().clone().requires_grad_(True)
    uf, itf = lightgcn_forward(edge_index, eu, ei, layers)
    loss = bpr_loss(uf[users], eu[users], itf[pos], ei[pos], itf[neg], ei[neg], lambda_val)
    loss.backward()
    return loss.detach(), eu.grad, ei.grad


# ----------------------------------------------------------------------------------
# e0 scoring + masks + topk: model/LightGCN/recommend.py:83-114
# ----------------------------------------------------------------------------------
def masked_scores_torch(eu: torch.Tensor, ei: torch.Tensor, train_pairs, val_pairs):
    """torch.matmul + the two -1024 index-puts (fp32, the reference's BLAS rounding)."""
    score = torch.matmul(eu, ei.T)
    for pairs in (train_pairs, val_pairs):
        if pairs is not None and len(pairs[0]):
            score[torch.as_tensor(pairs[0]), torch.as_tensor(pairs[1])] = MASK
    return score


def recommend_topk_torch(eu, ei, train_pairs, val_pairs, k: int):
    score = masked_scores_torch(eu, ei, train_pairs, val_pairs)
    vals, idx = torch.topk(score, k=k)
    return vals, idx, score


def exclusion_csr(n_users: int, n_items: int, *pair_sets):
    """Sorted, de-duplicated union of (user, item) pair sets as (rowptr int64, col int32)."""
    keys = [np.asarray(p[0], np.int64) * n_items + np.asarray(p[1], np.int64)
            for p in pair_sets if p is not None]
    keys = np.unique(np.concatenate(keys)) if keys else np.zeros(0, np.int64)
    u = keys // n_items
    rowptr = np.searchsorted(u, np.arange(n_users + 1), side="left").astype(np.int64)
    return rowptr, (keys % n_items).astype(np.int32)


# ----------------------------------------------------------------------------------
# exact fp32 chain scores (C): oracle/score_chain.c
# ----------------------------------------------------------------------------------
_C = None


def _clib():
    global _C
    if _C is None:
        # (ORACLE_LIB_PATH: the host-sanitized build of the sanitizer leg, oracle/Makefile asan)
        path = os.environ.get("ORACLE_LIB_PATH") or os.path.join(HERE, "build", "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.run(["make", "-C", HERE], check=True, capture_output=True)
        lib = ctypes.CDLL(path)
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        lib.oracle_score_matrix.argtypes = [vp, vp, i64, i64, ctypes.c_int, vp]
        lib.oracle_score_topk.argtypes = [vp, vp, i64, i64, ctypes.c_int, vp, vp,
                                          ctypes.c_float, ctypes.c_int, vp, vp]
        lib.oracle_score_topk.restype = ctypes.c_int
        _C = lib
    return _C


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else ctypes.c_void_p(0)


def chain_scores(eu: np.ndarray, ei: np.ndarray) -> np.ndarray:
    eu = np.ascontiguousarray(eu, np.float32)
    ei = np.ascontiguousarray(ei, np.float32)
    out = np.empty((eu.shape[0], ei.shape[0]), np.float32)
    _clib().oracle_score_matrix(_p(eu), _p(ei), eu.shape[0], ei.shape[0], eu.shape[1],
                                _p(out))
    return out


def chain_topk(eu, ei, ex_rowptr, ex_col, k: int, mask_value: float = MASK):
    eu = np.ascontiguousarray(eu, np.float32)
    ei = np.ascontiguousarray(ei, np.float32)
    nu = eu.shape[0]
    ov = np.empty((nu, k), np.float32)
    oi = np.empty((nu, k), np.int64)
    rp = None if ex_rowptr is None else np.ascontiguousarray(ex_rowptr, np.int64)
    cl = None if ex_col is None else np.ascontiguousarray(ex_col, np.int32)
    st = _clib().oracle_score_topk(_p(eu), _p(ei), nu, ei.shape[0], eu.shape[1], _p(rp),
                                   _p(cl), mask_value, k, _p(ov), _p(oi))
    assert st == 0
    return ov, oi


def chain_masked_matrix(eu, ei, ex_rowptr, ex_col, mask_value: float = MASK):
    g = chain_scores(eu, ei)
    for u in range(g.shape[0]):
        g[u, ex_col[ex_rowptr[u]:ex_rowptr[u + 1]]] = mask_value
    return g


# ----------------------------------------------------------------------------------
# hybrid spreading: model/SpreadMethod/model.py, utils/trans.py
# ----------------------------------------------------------------------------------
def interaction_matrix(n_users: int, n_items: int, users, items) -> np.ndarray:
    """getInteractionMatrixByDataframe (utils/trans.py:13-29): dense fp64 A, A[u,i] = 1."""
    A = np.zeros((n_users, n_items))
    A[np.asarray(users, np.int64), np.asarray(items, np.int64)] = 1
    return A


def spreading_general_mat(A: np.ndarray) -> np.ndarray:
    """getSpreadingGeneralMat (model/SpreadMethod/model.py:14-27)."""
    ud = np.sum(A, axis=1)
    ud[ud == 0] = 1
    return np.dot(A.T / ud, A)


def prob_s(A, gW):
    """ProbS (model/SpreadMethod/model.py:30-43; never called by the reference)."""
    kd = np.sum(A, axis=0)
    kd[kd == 0] = 1
    return gW / kd[np.newaxis, :]


def heat_s(A, gW):
    """HeatS (model/SpreadMethod/model.py:46-60; never called by the reference)."""
    kd = np.sum(A, axis=0)
    kd[kd == 0] = 1
    return gW / kd[:, np.newaxis]


def hybrid_s(A: np.ndarray, gW: np.ndarray, lam: float) -> np.ndarray:
    """HybridS (model/SpreadMethod/model.py:63-85)."""
    kd = np.sum(A, axis=0)
    den = np.power(kd, 1 - lam)[:, np.newaxis] * np.power(kd, lam)[np.newaxis, :]
    den[den == 0] = 1
    return gW / den


def get_resource(A, W):
    """getResource (model/SpreadMethod/model.py:88-99)."""
    return np.dot(A, W)


def spread_rows_sparse(user_rowptr, user_items, item_rowptr, item_users, n_items: int,
                       users, lam: float) -> np.ndarray:
    """Rows ``users`` of F = A @ HybridS(A, getSpreadingGeneralMat(A), lam) without the
    dense I x I matrices (model/SpreadMethod/model.py:14-27, :63-85, :88-99 restated over
    the interaction lists, fp64): for user u, every path u -> i -> v -> j with i in items(u),
    v in users(i), j in items(v) contributes A[v,i]/k_v to general_W[i,j]
    (``A.T / user_degrees``, k_v == 0 -> 1), W[i,j] = general_W[i,j] / den with
    den = k_i^(1-lam) * k_j^lam (den == 0 -> 1), and F[u,j] = sum_i W[i,j]. The sums run in
    path order, not BLAS order (a rounding-level difference: callers compare with a
    tolerance). Returns float64 [len(users), n_items]."""
    urp = np.asarray(user_rowptr, np.int64)
    uit = np.asarray(user_items, np.int64)
    irp = np.asarray(item_rowptr, np.int64)
    ius = np.asarray(item_users, np.int64)
    k_u = np.diff(urp).astype(np.float64)
    k_u[k_u == 0] = 1
    k_i = np.diff(irp).astype(np.float64)
    alpha = np.power(k_i, 1 - lam)
    beta = np.power(k_i, lam)
    out = np.zeros((len(users), n_items))
    for r, u in enumerate(users):
        its = uit[urp[u]:urp[u + 1]]
        if its.size == 0:
            continue
        nv = irp[its + 1] - irp[its]
        i_of = np.repeat(its, nv)
        v_of = ius[np.concatenate([np.arange(irp[i], irp[i + 1]) for i in its])]
        nj = urp[v_of + 1] - urp[v_of]
        i_p = np.repeat(i_of, nj)
        w_p = np.repeat(1.0 / k_u[v_of], nj)
        j_p = uit[np.concatenate([np.arange(urp[v], urp[v + 1]) for v in v_of])]
        key = i_p * n_items + j_p
        uk, inv = np.unique(key, return_inverse=True)
        gw = np.bincount(inv, weights=w_p)
        ii, jj = uk // n_items, uk % n_items
        den = alpha[ii] * beta[jj]
        den[den == 0] = 1
        out[r] = np.bincount(jj, weights=gw / den, minlength=n_items)
    return out


def _csr_gather(col: np.ndarray, starts: np.ndarray, counts: np.ndarray) -> np.ndarray:
    """col[starts[t] .. starts[t] + counts[t]) for every t, concatenated (vectorised)."""
    total = int(counts.sum())
    if total == 0:
        return np.zeros(0, col.dtype)
    base = np.repeat(starts - np.concatenate([[0], np.cumsum(counts)[:-1]]), counts)
    return col[base + np.arange(total)]


def spread_row_paths(urp, uit, irp, ius, n_items: int, u: int, lam: float,
                     inv_ku=None, alpha=None, beta=None) -> np.ndarray:
    """User u's row of F = A @ HybridS(A, getSpreadingGeneralMat(A), lam)
    (model/SpreadMethod/model.py:14-27, :63-85, :88-99) by enumerating its 3-hop paths
    u -> i -> v -> j in fp64: F[j] = (1 / k_j^lam) * sum over paths of
    (1 / k_v) / k_i^(1 - lam) -- the same sum as general_W[i, j] / (k_i^(1-lam) k_j^lam)
    summed over i, in path order instead of BLAS order (a rounding-level difference; the
    callers compare with a tolerance). k_v == 0 -> 1 and den == 0 -> 1 as the reference.
    ~10^6 paths per C5 user: vectorised gathers + one bincount (tens of ms)."""
    if inv_ku is None:
        k_u = np.diff(urp).astype(np.float64)
        k_u[k_u == 0] = 1
        inv_ku = 1.0 / k_u
    if alpha is None:
        k_i = np.diff(irp).astype(np.float64)
        alpha, beta = np.power(k_i, 1 - lam), np.power(k_i, lam)
        alpha[alpha == 0] = 1
        beta[beta == 0] = 1
    its = uit[urp[u]:urp[u + 1]]
    if its.size == 0:
        return np.zeros(n_items)
    nv = irp[its + 1] - irp[its]
    v_of = _csr_gather(ius, irp[its], nv)
    i_of = np.repeat(its, nv)
    nj = urp[v_of + 1] - urp[v_of]
    j_p = _csr_gather(uit, urp[v_of], nj)
    w_p = np.repeat(inv_ku[v_of] / alpha[i_of], nj)
    return np.bincount(j_p, weights=w_p, minlength=n_items) / beta


def spread_rows_spmv(urp, uit, irp, ius, n_items: int, users, lam: float) -> np.ndarray:
    """The rows ``users`` of F = A @ HybridS(A, getSpreadingGeneralMat(A), lam)
    (model/SpreadMethod/model.py:14-27, :63-85, :88-99) as two sparse products instead of
    the path enumeration of spread_row_paths: with X = A[users] / k_i^(1-lam) (one row per
    user), C = X A^T (the users' co-occurrence with every user v, weighted by 1/k_i^(1-lam)),
    F = (C / k_v) A / k_j^lam -- the same sum regrouped (v before j), fp64; for hub-heavy
    (Zipf) graphs, where a user's 3-hop paths run into the 10^9 (every hub item's users'
    items), it costs two SpMMs over the interactions per block. k == 0 -> 1 as the reference."""
    import scipy.sparse as sp
    urp, uit = np.asarray(urp, np.int64), np.asarray(uit, np.int64)
    irp = np.asarray(irp, np.int64)
    n_users = urp.size - 1
    k_u = np.diff(urp).astype(np.float64)
    k_u[k_u == 0] = 1
    k_i = np.diff(irp).astype(np.float64)
    alpha, beta = np.power(k_i, 1 - lam), np.power(k_i, lam)
    alpha[alpha == 0] = 1
    beta[beta == 0] = 1
    A = sp.csr_matrix((np.ones(uit.size), uit, urp), shape=(n_users, n_items))
    X = sp.diags(np.ones(len(users))) @ A[np.asarray(users, np.int64)] @ sp.diags(1.0 / alpha)
    C = (X @ A.T).toarray()                      # [len(users), n_users]
    C /= k_u[None, :]
    return np.asarray((A.T @ C.T).T) / beta[None, :]


def spread_parity(got_idx, users, urp, uit, irp, ius, n_items: int, lam: float, eu, ei,
                  k: int, dim_tol: int | None = None, block: int = 64,
                  method: str = "auto"):
    """LGCNHS (SpreadLightGCN, model/SpreadLightGCN/model.py:122-153 + recommend.py:18-52)
    top-k lists ``got_idx`` [len(users), k] of ``users`` against this oracle: S = G * F with
    F = spread_row_paths and G the e0 score (eu[u] . ei[j], judged in exact fp64), every
    item of the user's interactions dropped. The reference's top-k is taken by exact S over
    the candidates of an fp32 screen (the screen's rounding bound is checked to leave out no
    item that could rank in the top k). A user is *identical* if the sets agree,
    *tie-affected* if every differing item's exact S lies within the two methods' rounding
    bounds (G: 2 gamma_d sum|u_k i_k| for the fp32 dot of either side; F: 1e-12 relative) of
    the reference's k-th exact S, else *mismatched*. Returns the counts. F comes from
    spread_row_paths, or (method "spmv", or "auto" when a block's users have more than
    2 x 10^8 three-hop paths: hub-heavy graphs) from spread_rows_spmv."""
    urp, uit = np.asarray(urp, np.int64), np.asarray(uit, np.int64)
    irp, ius = np.asarray(irp, np.int64), np.asarray(ius, np.int64)
    eu, ei = np.asarray(eu, np.float32), np.asarray(ei, np.float32)
    d = eu.shape[1] if dim_tol is None else dim_tol
    u32 = 2.0 ** -24
    gam = 2.0 * (d * u32 / (1 - d * u32))
    k_u = np.diff(urp).astype(np.float64)
    k_u[k_u == 0] = 1
    k_i = np.diff(irp).astype(np.float64)
    alpha, beta = np.power(k_i, 1 - lam), np.power(k_i, lam)
    alpha[alpha == 0] = 1
    beta[beta == 0] = 1
    inv_ku = 1.0 / k_u
    ei_abs = np.abs(ei)
    users = np.asarray(users, np.int64)
    out = {"users": int(users.size), "k": k, "identical": 0, "tie_affected": 0,
           "mismatched": 0, "first_mismatch": None}
    # three-hop paths behind each user: sum over its items i of sum over i's users v of k_v
    p_item = np.add.reduceat(k_u[ius], irp[:-1]) if ius.size else np.zeros(n_items)
    p_item[np.diff(irp) == 0] = 0
    for b0 in range(0, users.size, block):
        ub = users[b0:b0 + block]
        G32 = eu[ub] @ ei.T                      # fp32 screen of G for the block
        Gb = np.abs(eu[ub]) @ ei_abs.T           # sum |u_k i_k| (fp32, rounded up below)
        paths = sum(float(p_item[uit[urp[u]:urp[u + 1]]].sum()) for u in ub.tolist())
        Fb = None
        if method == "spmv" or (method == "auto" and paths > 2e8):
            Fb = spread_rows_spmv(urp, uit, irp, ius, n_items, ub, lam)
        for r, u in enumerate(ub.tolist()):
            F = Fb[r] if Fb is not None else \
                spread_row_paths(urp, uit, irp, ius, n_items, u, lam, inv_ku, alpha, beta)
            own = uit[urp[u]:urp[u + 1]]
            gtol = gam * Gb[r].astype(np.float64) * (1 + 1e-6) + 1e-30
            s32 = G32[r].astype(np.float64) * F
            s32[own] = -np.inf
            # exact S on a candidate set that provably holds the exact top k
            m = min(n_items, 4 * k + 64)
            cand = np.argpartition(-s32, m - 1)[:m]
            ex = (ei[cand].astype(np.float64) @ eu[u].astype(np.float64)) * F[cand]
            stol = gtol[cand] * F[cand] + np.abs(ex) * 1e-12 + 1e-300
            order = np.lexsort((cand, -ex))
            ref = cand[order[:k]]
            kth = ex[order[k - 1]]
            outside = np.ones(n_items, bool)
            outside[cand] = False
            outside[own] = False
            if outside.any():
                # no item outside the candidates can reach the k-th exact score
                bound = s32[outside] + gtol[outside] * F[outside] + np.abs(s32[outside]) * 1e-12
                assert bound.max() < kth - stol[order[k - 1]], "candidate set too small"
            g = got_idx[b0 + r]
            gs, rs = set(g[g >= 0].tolist()), set(ref.tolist())
            if gs == rs:
                out["identical"] += 1
                continue
            diff = np.array(sorted(gs ^ rs), np.int64)
            exd = (ei[diff].astype(np.float64) @ eu[u].astype(np.float64)) * F[diff]
            tld = gtol[diff] * F[diff] + np.abs(exd) * 1e-12
            if np.all(np.abs(exd - kth) <= tld + stol[order[k - 1]]):
                out["tie_affected"] += 1
            else:
                out["mismatched"] += 1
                if out["first_mismatch"] is None:
                    out["first_mismatch"] = {"user": u, "got_only": sorted(gs - rs),
                                             "ref_only": sorted(rs - gs)}
    return out


def spread_overrides(method: str, dataset: str, lam: float, gW: np.ndarray):
    """model/SpreadMethod/recommend.py:86-111: the lambda / transpose per method."""
    if method == "ProbS" and dataset == "movielens":
        return 0.01, gW.T
    if method == "HeatS" and dataset == "douban":
        return 0.99, gW.T
    return lam, gW


def recommend_all_user(F_new: np.ndarray, n_users: int, excl: dict, k: int,
                       unfiltered: bool = False) -> dict:
    """recommendForAllUser (model/SpreadMethod/recommend.py:18-56) with the canonical tie
    order (value desc, item asc) in place of np.argsort's unspecified one."""
    out = {}
    for u in range(n_users):
        row = F_new[u]
        order = np.lexsort((np.arange(row.size), -row))
        if unfiltered:
            out[u] = order[:k].tolist()
            continue
        ex = set(excl.get(u, ()))
        out[u] = [int(i) for i in order if int(i) not in ex][:k]
    return out


def rows_topk(F: np.ndarray, k: int, ex_rowptr=None, ex_col=None, drop: bool = True):
    """Canonical (value desc, column asc) top-k per row with excluded columns dropped:
    what lg_rows_topk_f64 must return bit for bit on the same F."""
    n, m = F.shape
    ov = np.full((n, k), -np.inf)
    oi = np.full((n, k), -1, np.int64)
    for r in range(n):
        cols = np.arange(m)
        vals = F[r]
        if drop and ex_rowptr is not None:
            keep = np.ones(m, bool)
            keep[ex_col[ex_rowptr[r]:ex_rowptr[r + 1]]] = False
            cols, vals = cols[keep], vals[keep]
        order = np.lexsort((cols, -vals))[:k]
        ov[r, :order.size] = vals[order]
        oi[r, :order.size] = cols[order]
    return ov, oi


# ----------------------------------------------------------------------------------
# metrics: metrics/accurate.py:11-102, metrics/diversity.py:15-115 (the reference's own
# loop orders and dtypes, so the rounded results agree exactly on the fixtures)
# ----------------------------------------------------------------------------------
def _labels(pos: dict, recs: np.ndarray) -> np.ndarray:
    """metrics/accurate.py:24-31: membership of each recommended item in the user's list."""
    return np.array([[int(it) in set(int(x) for x in items) for it in recs[uid]]
                     for uid, items in pos.items()]).astype("float")


def precision_recall(pos: dict, recs: np.ndarray, k: int):
    """metrics/accurate.py:11-46 (fp32 torch reductions, rounded to 5 decimals)."""
    R = torch.Tensor(_labels(pos, recs))
    lens = torch.Tensor([len(v) for v in pos.values()])
    n = torch.sum(R, dim=-1)
    return round((torch.mean(n) / k).item(), 5), round(torch.mean(n / lens).item(), 5)


def f1_score(p: float, r: float) -> float:
    """metrics/accurate.py:48-56."""
    return round(2 * (p * r) / (p + r), 5)


def ndcg(pos: dict, recs: np.ndarray, k: int) -> float:
    """metrics/accurate.py:58-102: the ideal DCG counts min(len(list), k) ones, whatever
    the number of test items."""
    R = torch.Tensor(_labels(pos, recs))
    tmp = torch.zeros((len(R), k))
    for j, row in enumerate(R):
        tmp[j, :min(len(row), k)] = 1
    idcg = torch.sum(tmp * 1. / torch.log2(torch.arange(2, k + 2)), axis=1)
    dcg = torch.sum(R * (1. / torch.log2(torch.arange(2, k + 2))), axis=1)
    idcg[idcg == 0.] = 1.
    v = dcg / idcg
    v[torch.isnan(v)] = 0.
    return round(torch.mean(v).item(), 5)


def hamming_distance(recs: np.ndarray, k: int) -> float:
    """metrics/diversity.py:15-63: mean over ordered pairs u != v of 1 - |set & set| / k,
    summed in the reference's (u, v) order."""
    U = recs.shape[0]
    sets = [set(int(x) for x in r) for r in recs]
    total = 0.0
    for a in range(U):
        for b in range(U):
            if a != b:
                total += 1 - (len(sets[a] & sets[b]) / k)
    return round(round(total / (U * (U - 1)), 5), 5)


def internal_similarity(recs: np.ndarray, deg: dict, A: np.ndarray, k: int) -> float:
    """metrics/diversity.py:66-115: sum over users and ordered pairs of distinct items of
    nonzero degree of (A[:, i] . A[:, j]) / sqrt(k_i k_j), in the reference's order."""
    total = 0.0
    for row in recs:
        items = [int(x) for x in row]
        for i in items:
            for j in items:
                if i == j:
                    continue
                ki, kj = deg.get(i, 0), deg.get(j, 0)
                if ki == 0 or kj == 0:
                    continue
                total += np.dot(A[:, i], A[:, j]) / np.sqrt(ki * kj)
    return round(total / (recs.shape[0] * k * (k - 1)), 5)


def item_degrees(*pos_dicts: dict) -> dict:
    """utils/trans.py:94-115 getItemDegreeByUserPosItemDict."""
    d = {}
    for pd_ in pos_dicts:
        for items in pd_.values():
            for it in items:
                d[int(it)] = d.get(int(it), 0) + 1
    return d


def pos_dict(pairs: np.ndarray) -> dict:
    """utils/trans.py:51-63 getUserItemsDictByDataframe on a [2, n] (user, item) array."""
    d = {}
    for u, i in zip(pairs[0].tolist(), pairs[1].tolist()):
        d.setdefault(int(u), []).append(int(i))
    return d
