"""Benchmark: propagation edges/sec (+ full-catalog top-K recs/sec) on MI355X.

Workload (BASELINE.json north_star headline): synthetic uniform bipartite graph,
1M users x 1M items, 100M interactions (200M directed nnz of A_hat), dim 64, 3 LightGCN
layers. A "step" = one full 3-layer forward over the whole graph (gcn_norm cached, as the
graph is fixed), with the layer mean fused. N GPUs (--layout bipartite, the default): users
and items are sharded separately, each layer propagates one half then the other, and the
RCCL all-gather of one half's new rows runs on a high-priority stream behind the other
half's SpMM (strong scaling: the graph is fixed, value = all nnz x layers / max-over-ranks
time). "roofline" prices the SpMM kernel's algorithmic bytes against HBM peak with its own
HIP-event time on the stream it runs on.

Phases after the timed steps (each reported in its own key of the same JSON line):
  topk    masked full-catalog top-20 (e0 scores, -1024 exclusion of each user's train+val
          items) for a block of users per rank over all 1M items (recs/s over ranks);
  spread  SpreadLightGCN / LGCNHS for ALL users over all items: item-tiled factored HybridS
          spreading (no I x I matrix), G (.) F filtered top-20, item ranges sharded over
          ranks, per-range lists exchanged all-to-all and merged; then "eval": P/R/NDCG/H/I
          of those lists against a synthetic test split;
  train   (N=1) one LightGCN BPR training step on the same graph: HIP forward, a mini-batch
          with structured negatives, BPR, HIP backward, Adam;
  cpu_baseline*  the reference's op sequences (oracle restatement) on host cores, bounded
          samples (skip with --no-cpu-baseline).

Run: python bench.py [--gpus N --steps K --warmup W]. N > 1: one process per GPU, either
under the caller's torch.distributed.run (WORLD_SIZE must equal N) or started here as a child
torch.distributed.run when WORLD_SIZE is unset.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
F32_MFMA_PEAK_TF = 157.3    # dense fp32 MFMA (= fp32 vector) peak, same table
BF16_MFMA_PEAK_TF = 2500.0  # dense bf16 MFMA peak, same table
# chip-wide ds_add_f64 rate to random columns of a per-wave 2048-entry accumulator, 8 waves
# per CU (scripts/micro/lds_atomic.hip on the box, profiles/r03_lds_atomic.txt): the ceiling
# of the K3s walk, which adds every 3-hop path with one LDS atomic
LDS_F64_ADD_PEAK_G = 1584.4

WORKLOADS = {
    # name: (users, items, interactions, dim, layers)
    "c5-d64": (1_000_000, 1_000_000, 100_000_000, 64, 3),
    "c5-d128": (1_000_000, 1_000_000, 100_000_000, 128, 3),
    "c4": (200_000, 200_000, 20_000_000, 64, 3),
    "c2": (6_040, 3_706, 800_167, 64, 3),
    "tiny": (20_000, 20_000, 1_000_000, 64, 3),
    # the power-law secondary input of SURVEY.md §8(d) / BASELINE.md: Zipf(1.1) item
    # popularity, uniform users (lgcnhs.synth.synth_graph_device(dist="zipf"))
    "c5-zipf-d64": (1_000_000, 1_000_000, 100_000_000, 64, 3),
    "c4-zipf": (200_000, 200_000, 20_000_000, 64, 3),
}
GRAPH_DIST = {"c5-zipf-d64": "zipf", "c4-zipf": "zipf"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def gen_graph(U, I, E, seed, dev, dist="uniform"):
    """Exactly E unique (user, item) pairs on the device (items uniform or Zipf(1.1)); returns
    the symmetric CSR over U+I nodes (rowptr int64, src int32) plus the sorted interaction
    keys."""
    from lgcnhs.synth import synth_graph_device
    return synth_graph_device(U, I, E, seed, dev, dist=dist)


def cpu_threads():
    """Host threads for the CPU baselines: the job's CPU share
    (OMP_NUM_THREADS, which the GPU box sets to the CPUs it allots one job) or else
    os.cpu_count(); set explicitly with torch.set_num_threads. Returns (threads, host CPUs,
    CPU model)."""
    n = int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)
    torch.set_num_threads(n)
    model = platform.processor() or "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return n, os.cpu_count(), model


def cpu_baseline(rowptr, src, n, dim, layers, target_nnz=4_000_000, reps=5):
    """The oracle's PyG op sequence (index_select * w, index_add_) on the host cores over a
    bounded sample: the first rows of the graph until ~target_nnz edges, full-size x;
    median of `reps` after one warm-up."""
    from oracle import lgcn_oracle as O  # noqa: F401  (the port being timed)
    threads, host_cpus, model = cpu_threads()
    rp = rowptr.cpu()
    r_end = int(torch.searchsorted(rp, torch.tensor([target_nnz])).item())
    r_end = max(1, min(r_end, n))
    e_end = int(rp[r_end])
    s = src[:e_end].cpu().to(torch.int64)
    deg = (rp[1:r_end + 1] - rp[:r_end])
    t = torch.repeat_interleave(torch.arange(r_end), deg)
    ei = torch.stack([s, t])
    full_deg = (rp[1:] - rp[:-1]).float()
    dis = full_deg.pow(-0.5)
    dis.masked_fill_(dis == float("inf"), 0)
    w = dis[s] * dis[t]
    x = torch.randn(n, dim) * 0.1
    O.propagate(ei, w, x)  # warm-up
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        cur = x
        for _ in range(layers):
            cur = O.propagate(ei, w, cur)
        times.append(time.perf_counter() - t0)
    secs = sorted(times)[reps // 2]
    return {"value": e_end * layers / secs, "unit": "edge-layers/s", "cores": threads,
            "host_cpus": host_cpus, "cpu_model": model, "kind": "port",
            "sample": f"PyG op sequence (index_select*w, index_add_) over rows [0,{r_end}) = "
                      f"{e_end} directed nnz x {layers} layers, full {n}x{dim} x, median of "
                      f"{reps}"}


def cpu_baseline_topk(e0_orig, keys, U, I, k, n_users=4096, block=512):
    """The reference's e0 scoring + -1024 masks + torch.topk (model/LightGCN/recommend.py:
    83-114, restated by the oracle) on the host cores for a 4,096-user block x all items
    (BASELINE.md §3), in 512-user slices (a 4,096 x 1M fp32 score matrix is 16 GB).
    Returns the baseline line and the CPU lists (compared with the GPU's by the caller)."""
    from oracle import lgcn_oracle as O  # noqa: F401  (the port being timed)
    threads, host_cpus, model = cpu_threads()
    ei = e0_orig[U:U + I].cpu()
    O.recommend_topk_torch(e0_orig[:8].cpu(), ei, None, None, k)  # warm-up
    lists = []
    secs = 0.0
    for b0 in range(0, n_users, block):
        b1 = min(n_users, b0 + block)
        eu = e0_orig[b0:b1].cpu()
        blk = keys[(keys >= b0 * I) & (keys < b1 * I)].cpu()
        pairs = (blk // I - b0, blk % I)
        t0 = time.perf_counter()
        _, idx, _ = O.recommend_topk_torch(eu, ei, pairs, None, k)
        secs += time.perf_counter() - t0
        lists.append(idx)
    line = {"value": n_users / secs, "unit": "recs/s", "cores": threads,
            "host_cpus": host_cpus, "cpu_model": model, "kind": "port",
            "sample": f"torch.matmul + -1024 index-put + torch.topk(k={k}) for users "
                      f"[0,{n_users}) x {I} items in {block}-user slices (fp32, the "
                      f"reference's op sequence)"}
    return line, torch.cat(lists)


def topk_parity(gpu_idx, cpu_idx, e0_orig, U, D, k):
    """GPU top-k lists (lg_score_topk_f32's fp32 chain) against the CPU reference op
    sequence's (BLAS fp32) for the same users: identical sets, or tie-affected users whose
    differing items all have exact (fp64) scores within both methods' rounding bound
    (2 * gamma_d * sum |u_k i_k|) of the reference's k-th exact score. Returns counts."""
    g = gpu_idx.cpu().numpy()
    c = cpu_idx.cpu().numpy()
    n = c.shape[0]
    gam = 2.0 * D * 2.0 ** -24 / (1 - D * 2.0 ** -24)
    ties = bad = 0
    for u in range(n):
        sg, sc = set(g[u].tolist()), set(c[u].tolist())
        if sg == sc:
            continue
        eu = e0_orig[u].double().cpu()
        items = torch.tensor(sorted(sg | sc))
        ei = e0_orig[U + items].double().cpu()
        ex = ei @ eu
        tol = gam * (ei.abs() @ eu.abs())
        pos = {int(i): t for t, i in enumerate(items.tolist())}
        ref_ex = torch.tensor([float(ex[pos[int(i)]]) for i in c[u]])
        b = int(torch.argmin(ref_ex))
        eb, tb = float(ref_ex[b]), float(tol[pos[int(c[u][b])]])
        diff = sg ^ sc
        if all(abs(float(ex[pos[i]]) - eb) <= float(tol[pos[i]]) + tb for i in diff):
            ties += 1
        else:
            bad += 1
    return {"users": n, "k": k, "identical": n - ties - bad, "tie_affected": ties,
            "mismatched": bad,
            "rule": "sets equal, or every differing item's exact fp64 score within both "
                    "methods' fp32 rounding bound of the reference's k-th exact score"}


def cpu_baseline_spread(k, lam=0.5):
    """The reference's dense SpreadLightGCN op sequence (model/SpreadMethod/model.py:14-99,
    model/SpreadLightGCN/model.py:140-151, recommend.py:18-52; restated by the oracle in
    numpy fp64) on the host cores, at the Douban-shaped stand-in the GPU's c3_douban_shape
    line times: general_W, HybridS, F = A W, G (fp32 e0 scores) * F, filtered top-k."""
    import numpy as np
    from oracle import lgcn_oracle as O  # noqa: F401  (the port being timed)
    from lgcnhs.synth import synth_interactions
    cpu_threads()
    du, di, de = 600, 20_000, 60_000
    users, items = synth_interactions(du, di, de, seed=3, dist="zipf")
    g = torch.Generator().manual_seed(42)
    eu = torch.randn(du, 64, generator=g) * 0.1
    ei = torch.randn(di, 64, generator=g) * 0.1
    t0 = time.perf_counter()
    A = O.interaction_matrix(du, di, users, items)
    W = O.hybrid_s(A, O.spreading_general_mat(A), lam)
    F = O.get_resource(A, W)
    del W
    F = torch.matmul(eu, ei.T).numpy() * F
    rp = np.searchsorted(users, np.arange(du + 1))
    O.rows_topk(F, k, rp, items.astype(np.int32), True)
    secs = time.perf_counter() - t0
    threads, host_cpus, model = cpu_threads()
    return {"value": du / secs, "unit": "recs/s", "cores": threads, "host_cpus": host_cpus,
            "cpu_model": model, "kind": "port", "seconds": secs,
            "sample": f"dense fp64 numpy general_W / HybridS / A@W, G*F, filtered top-{k}: "
                      f"{du} users x {di} items, {de} Zipf interactions (c3_douban_shape)"}


def _sync(dev):
    if torch.device(dev).type == "cuda":
        torch.cuda.synchronize()


def time_propagation(shard, dis_l, e0_orig, D, L, steps, warmup, world, dev, layer_fn=None):
    """Time `steps` full L-layer forwards; returns (max-over-ranks seconds, average SpMM
    'launch' seconds = one layer's kernels on this rank, from HIP events on the stream, and
    at N > 1 the `comm` block). layer_fn: lgcnhs.dist's HIP layer unless given (the CPU
    launch check passes a host stand-in)."""
    from lgcnhs.dist import BipartitePropagation, SegmentShard, ShardedPropagation, exposed_wait_ms
    e0 = shard.permute_rows(e0_orig)  # chunk-major layout (identity at N=1)
    cls = BipartitePropagation if isinstance(shard, SegmentShard) else ShardedPropagation
    kw = {} if layer_fn is None else {"layer_fn": layer_fn}
    prop = cls(shard, dis_l, D, L, dev, **kw)
    for _ in range(warmup):
        prop.forward(e0)
    _sync(dev)
    cuda = torch.device(dev).type == "cuda"
    prop.events = [] if cuda else None
    prop.waits = []
    if world > 1:
        dist.barrier()
    _sync(dev)
    t1 = time.perf_counter()
    for _ in range(steps):
        prop.forward(e0)
    _sync(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t1
    kernel_ms = sum(s.elapsed_time(e) for s, e in prop.events) if cuda else 0.0  # SpMM only
    comm = None
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        wait = exposed_wait_ms(prop.waits, L, steps)
        prop.waits = None
        comm = time_exchange(prop, shard, D, world, dev)
        comm.update(exposure(wait, comm["allgather_ms_per_layer"], L, world, dev))
    del prop, e0
    return elapsed, kernel_ms / (steps * L) / 1e3, comm


def exposure(wait_ms, ag_ms, L, world, dev):
    """The part of the exchange the overlapped forward did not hide: per layer, the compute
    stream's stall on the gathers it awaited (lgcnhs.dist._WaitTimer; the stall of layer l is
    the wait for layer l-1's gathers), max over ranks; against the L - 1 layers' gathers timed
    alone (`allgather_ms_per_layer`): hidden_frac = 1 - exposed / isolated."""
    t = torch.tensor(wait_ms, dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    per = [float(v) for v in t.tolist()]
    iso = (L - 1) * ag_ms
    tot = sum(per)
    return {"exposed_wait_ms_per_layer": per, "exposed_wait_ms": tot,
            "isolated_allgather_ms_per_step": iso,
            "hidden_frac": (1.0 - tot / iso) if iso > 0 else None}


def time_exchange(prop, shard, D, world, dev, reps=5):
    """The all-gathers of one layer alone (no SpMM running): RCCL over xGMI, ms per layer.
    Rates as nccl-tests defines them for all_gather of a total output of S bytes (the padded
    [n, D] fp32 table): algbw = S / t, busbw = algbw (W - 1) / W -- what each GPU receives
    per second, the figure to hold against xGMI's per-link rate."""
    from lgcnhs.dist import SegmentShard, _gather_block, _gather_piece
    buf = prop.bufs[0]

    def once():
        hs = []
        if isinstance(shard, SegmentShard):
            for s_, ps in enumerate(shard.seg_pieces):
                for c in range(len(ps)):
                    hs.append(_gather_piece(buf, shard, s_, c, prop.group))
        else:
            for c in range(shard.chunks):
                hs.append(_gather_block(buf, shard, c, prop.group))
        for h in hs:
            h.wait()
    once()
    _sync(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    _sync(dev)
    dt = (time.perf_counter() - t0) / reps
    t = torch.tensor([dt], device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    size = shard.n_pad * D * 4
    recv = (world - 1) / world * size
    return {"allgather_ms_per_layer": dt * 1e3, "algbw_GBps": size / dt / 1e9,
            "busbw_GBps": recv / dt / 1e9, "recv_GBps_per_gpu": recv / dt / 1e9,
            "recv_bytes_per_gpu": recv, "pad_ratio": shard.pad_ratio}


def bench_other_graph(name, dev, steps, k, topk_users, cpu_parity=True, spread=False):
    """A second graph shape at N = 1 (SURVEY.md §8(d)'s power-law input): the propagation
    (K1 with the long-row pass for hub rows inside the timed forward) with its roofline and
    PMC traffic, the degree profile that drives it, and the masked top-K on the same graph's
    exclusion sets (hub items are in most users' histories), its lists checked against the
    reference op sequence on a CPU sample."""
    from lgcnhs import _native as NV
    from lgcnhs.dist import RowShard
    from lgcnhs.graph import LONG_ROW_THRESHOLD
    U, I, E, D, L = WORKLOADS[name]
    N = U + I
    t0 = time.time()
    rowptr, src, keys = gen_graph(U, I, E, seed=3, dev=dev, dist=GRAPH_DIST.get(name, "uniform"))
    nnz = int(src.numel())
    deg = rowptr[1:] - rowptr[:-1]
    long_rows = deg > LONG_ROW_THRESHOLD
    stats = {"dist": GRAPH_DIST.get(name, "uniform"), "zipf_s": 1.1, "users": U, "items": I,
             "interactions": E, "nnz": nnz, "max_item_degree": int(deg[U:].max()),
             "max_user_degree": int(deg[:U].max()),
             "long_rows": int(long_rows.sum()), "long_row_threshold": LONG_ROW_THRESHOLD,
             "long_row_nnz_share": float(deg[long_rows].sum()) / nnz}
    dis = torch.empty(N, dtype=torch.float32, device=dev)
    NV.check(NV.lib().lg_gcn_norm_f32(NV.ptr(rowptr), N, NV.ptr(dis), NV.stream_handle(dev)),
             "gcn_norm")
    wgt = torch.empty(nnz, dtype=torch.float32, device=dev)
    NV.check(NV.lib().lg_gcn_edge_weight_f32(NV.ptr(rowptr), NV.ptr(src), NV.ptr(dis), N, 0,
                                             NV.ptr(wgt), NV.stream_handle(dev)), "edge weights")
    shard = RowShard(rowptr, src, N, 0, 1, dev, weight=wgt, chunks=1)
    del wgt, rowptr, src
    gen = torch.Generator(device=dev).manual_seed(43)
    e0 = torch.randn(N, D, device=dev, generator=gen) * 0.1
    setup = time.time() - t0
    elapsed, k_s, _ = time_propagation(shard, shard.permute_rows(dis), e0, D, L, steps,
                                       max(1, steps // 3), 1, dev)
    alg = nnz * (8 + 4 * D) + N * (4 + 4 * D)
    traffic, tsrc = load_traffic(name, 1)
    prop = {"value": nnz * L * steps / elapsed, "unit": "edge-layers/s",
            "ms_per_step": elapsed / steps * 1e3,
            "roofline": {"bound": "hbm", "achieved": alg / k_s / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": alg / k_s / 1e9 / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_source": tsrc,
                         # (hub rows' sources are re-read from L2 / the Infinity Cache: the
                         # algorithmic rate can pass the HBM peak; the PMC bytes cannot)
                         "traffic_frac": (traffic / k_s / 1e9 / HBM_PEAK_GBS) if traffic else None,
                         "kernel": "lg_spmm_layer_f32 + lg_spmm_long_rows_f32 (one layer)",
                         "avg_launch_ms": k_s * 1e3, "alg_bytes_per_launch": alg}}
    del shard
    torch.cuda.empty_cache()
    out = {"workload": name, "graph": stats, "setup_s": setup, "propagation": prop}
    try:
        topk, lists = bench_topk(e0, keys, U, I, D, k, topk_users, 0, 1, dev)
        if cpu_parity and lists is not None:
            _, cpu_lists = cpu_baseline_topk(e0, keys, U, I, k, n_users=512)
            topk["parity_vs_cpu_reference"] = topk_parity(lists[:512], cpu_lists[:512], e0, U,
                                                          D, k)
        out["topk"] = topk
    except Exception as ex:  # a side measurement never hides the main result
        log(f"{name} topk bench failed: {ex!r}")
    if spread:  # LGCNHS on this graph (all users), its walk roofline, the V-row share, parity
        try:
            torch.cuda.empty_cache()
            out["spread"] = bench_spread(keys, U, I, e0, k, 0, 1, dev, extras=False,
                                         parity=cpu_parity)
        except Exception as ex:  # a side measurement never hides the main result
            log(f"{name} spread bench failed: {ex!r}")
    del e0, keys
    torch.cuda.empty_cache()
    return out


def bench_small_config(dev, k):
    """configs[1] (ML-1M shape: 6040 users x 3706 items, 800,167 train interactions, d=64,
    L=3) on one GPU: propagation eager and replayed from a captured hipGraph, and the full
    masked top-k for every user. Kernels of tens of microseconds: launch-bound."""
    from lgcnhs import ops
    from lgcnhs.graph import Adjacency, RowSets
    U, I, E, D, L = WORKLOADS["c2"]
    rowptr, src, keys = gen_graph(U, I, E, seed=1, dev=dev)
    users, items = keys // I, keys % I
    adj = Adjacency.from_interactions(users, items, U, I, dev)
    e0 = torch.randn(U + I, D, device=dev, generator=torch.Generator(device=dev).manual_seed(7)) * 0.1
    ops.propagate(adj, e0, L)
    pg = ops.PropagationGraph(adj, D, L)
    res = {"users": U, "items": I, "directed_nnz": adj.nnz, "dim": D, "layers": L}
    for name, fn in (("eager", lambda: ops.propagate(adj, e0, L)), ("graph", lambda: pg.run(e0))):
        fn()
        torch.cuda.synchronize()
        reps = 50
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        res[f"propagation_{name}_edge_layers_per_s"] = adj.nnz * L / dt
        res[f"forward_{name}_us"] = dt * 1e6
    excl = RowSets.from_pairs(users, items, U, I, dev)
    eu, ei = e0[:U].contiguous(), e0[U:].contiguous()
    ops.score_topk(eu, ei, k, excl)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        ops.score_topk(eu, ei, k, excl)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10
    res["topk_all_users_ms"] = dt * 1e3
    res["topk_recs_per_s"] = U / dt
    return res


def bench_train(rowptr, src, keys, U, I, e0_orig, D, L, dev, steps=3, batch=1024):
    """SURVEY.md §8 f2 on the north_star graph, one GPU: the reference's training step
    (model/LightGCN/train.py:26-59,148-151; loss.py:12-70) through the package's own path:
    a 1024-triple mini-batch of the interactions with structured negatives
    (model.LightGCN.loss.sampleMiniBatch), the HIP forward at the batch's rows
    (ops.propagate_rows: output-restricted layers, bitwise the full forward's rows), BPRLoss,
    backward (the
    HIP propagation with A_hat^T = A_hat) and one Adam step over all U+I embedding rows.
    The interactions here are the train|val positives the other phases exclude."""
    from lgcnhs import ops
    from lgcnhs.graph import Adjacency
    from model.LightGCN.loss import BPRLoss, sampleMiniBatch
    adj = Adjacency(rowptr, src, U + I, n_users=U, symmetric=True)
    e0 = torch.nn.Parameter(e0_orig.clone())
    opt = torch.optim.Adam([e0], lr=1e-3)
    r_edge = torch.stack([keys // I, keys % I])
    gen = torch.Generator(device=dev).manual_seed(42)

    def step():
        # (model/LightGCN/train.py getEmbeddingForBPR: the batch first, then the forward's
        # layers only where the batch's rows depend on them)
        u, p, n = sampleMiniBatch(batch, r_edge, I, generator=gen)
        f = ops.propagate_rows(adj, e0, L, torch.cat([u, U + p, U + n]))
        fu, fp, fn = torch.split(f, [batch, batch, batch])
        loss = BPRLoss(fu, e0[u], fp, e0[U + p], fn, e0[U + n], 1e-6)
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    res = {"ms_per_step": dt * 1e3, "steps_per_s": 1.0 / dt, "batch": batch,
           "interactions_sampled": int(keys.numel()), "loss": float(loss.item()),
           "what": "mini-batch with structured negatives over all interactions + HIP forward "
                   "restricted to the rows the batch depends on (layer 3 at the batch, layer 2 "
                   "at it and its neighbours, layer 1 in full) + BPR + HIP backward + Adam "
                   "over all embedding rows"}
    del opt, e0, r_edge, adj
    torch.cuda.empty_cache()
    return res


def bench_eval(idx, u0, u1, A, keys, U, I, k, rank, world, dev, n_test=10_000_000):
    """Full top-k evaluation of the C5 recommendations (metrics/accurate.py +
    metrics/diversity.py on the device, lgcnhs.metrics): P / R / NDCG against a synthetic
    test set (n_test random pairs outside train|val, seeded), Hamming distance over all user
    pairs (exact closed form; the lists are all-gathered) and internal similarity over A.
    This rank evaluates its user block; sums are all-reduced."""
    from lgcnhs import metrics as M
    from lgcnhs.graph import RowSets
    g = torch.Generator(device=dev).manual_seed(11)
    tk = torch.unique(torch.randint(0, U, (n_test,), device=dev, generator=g) * I +
                      torch.randint(0, I, (n_test,), device=dev, generator=g))
    pos = torch.searchsorted(keys, tk).clamp_max(keys.numel() - 1)
    tk = tk[keys[pos] != tk]                       # test items are never train|val items
    tk = tk[(tk >= u0 * I) & (tk < u1 * I)]        # this rank's users
    test = RowSets.from_pairs(tk // I - u0, tk % I, u1 - u0, I, dev)
    deg_item = A.by_item.degrees()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    acc = M.accuracy(idx, test, k)
    part = M.intra_similarity_parts(idx, A.by_item, deg_item)
    sums = torch.tensor([acc["precision"] * acc["n_eval"], acc["recall"] * acc["n_eval"],
                         acc["ndcg"] * acc["n_eval"], float(acc["n_eval"]),
                         float(part.sum())], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(sums)
        # every rank's lists (padded to equal blocks with -1, which match nothing)
        nmax = -(-U // world)
        mine = torch.full((nmax, k), -1, dtype=idx.dtype, device=dev)
        mine[:idx.shape[0]] = idx
        allr = torch.empty((world * nmax, k), dtype=idx.dtype, device=dev)
        dist.all_gather_into_tensor(allr, mine)
    else:
        allr = idx
    overlap = M.pair_overlap(allr, I)
    H = (U * (U - 1) - overlap / k) / (U * (U - 1))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    n = float(sums[3])
    return {"seconds": dt, "users": U, "test_pairs_evaluated_rank0": int(tk.numel()),
            "P": float(sums[0]) / n, "R": float(sums[1]) / n, "NDCG": float(sums[2]) / n,
            "H": H, "I": 2.0 * float(sums[4]) / (U * k * (k - 1)),
            "path": "lg_rec_hits + lg_rec_pair_overlap + lg_rec_intra_similarity_f64"}


def spread_parity_field(idx, u0, u1, A, eu, ei, lam, k, n=256, top=16, seed=11):
    """spread.parity_vs_oracle: ``n`` users of this rank's block (its `top` highest-degree
    users, the first and last, the rest at random) against the oracle's fp64 path-order
    restatement of S = G * F (oracle.spread_parity; the checker, run after the timed region
    on the host cores): identical / tie-affected / mismatched counts."""
    import numpy as np
    from oracle import lgcn_oracle as O  # noqa: F401  (the checker)
    nb = u1 - u0
    deg = A.by_user.degrees()[u0:u1].cpu().numpy()
    fixed = np.unique(np.concatenate([np.argsort(-deg, kind="stable")[:top], [0, nb - 1]]))
    rest = np.random.default_rng(seed).choice(np.setdiff1d(np.arange(nb), fixed),
                                              max(0, min(n, nb) - fixed.size), replace=False)
    rows = np.sort(np.concatenate([fixed, rest]))
    got = idx[torch.as_tensor(rows, device=idx.device)].cpu().numpy()
    t0 = time.perf_counter()
    r = O.spread_parity(got, rows + u0, A.by_user.rowptr.cpu().numpy(),
                        A.by_user.col.cpu().numpy(), A.by_item.rowptr.cpu().numpy(),
                        A.by_item.col.cpu().numpy(), A.n_items, lam, eu.cpu().numpy(),
                        ei.cpu().numpy(), k)
    r["seconds_cpu"] = time.perf_counter() - t0
    r["rule"] = ("sets equal, or every differing item's exact fp64 S = G*F within both "
                 "methods' rounding bounds (fp32 dot for G, 1e-12 rel for F) of the "
                 "oracle's k-th exact S; users: the 16 highest-degree, first, last, random")
    return r


def bench_spread(keys, U, I, e0_orig, k, rank, world, dev, lam=0.5, tile=2048, extras=True,
                 parity=True):
    """C5 LGCNHS recommendation for EVERY user (SpreadLightGCN, model/SpreadLightGCN/model.py:
    107-153 + recommend.py:18-52): per user, top-k of G * F with F = A @ HybridS(A, general_W,
    lam) and G the fp32 e0 score (width = e0_orig's), train|val items dropped, over the
    factored tile path. Sharded by item range (lgcnhs.dist.sharded_spread_topk): each rank
    builds only its own W tiles and scores all users on them, then one all-to-all + merge
    gives each rank the final lists of its user block. Timed end to end (max over ranks).
    With ``extras`` also the evaluation of the lists and the Douban-shaped dense path
    (configs[2]: SpreadLightGCNOpti, lam=0.5) at N=1; with ``parity`` (rank 0) the lists of
    256 sampled users against the oracle (after the timed region)."""
    from lgcnhs import ops
    from lgcnhs.dist import item_range, sharded_spread_topk
    A = ops.Interactions.from_pairs(keys // I, keys % I, U, I, dev)
    eu = e0_orig[:U].contiguous()
    ei = e0_orig[U:U + I].contiguous()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    st = {}  # paths added / row bytes gathered by the walk (the 3-hop paths of F = A W)
    (u0, u1), _, idx = sharded_spread_topk(A, lam, k, A.by_user, True, eu, ei, rank=rank,
                                           world=world, tile=tile, stats=st)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # the walk's paths / row bytes: counted from the tiles after the timed run (untimed)
    i0, i1 = item_range(I, tile, rank, world)
    st["w_paths"], st["w_bytes"], st["w_paths_v"] = ops.tile_traffic(A, tile,
                                                                   items=slice(i0, i1), hub=True)
    paths, nbytes = float(st["w_paths"]), float(st["w_bytes"])
    if world > 1:
        e = torch.tensor([paths, nbytes], dtype=torch.float64, device=dev)
        dist.all_reduce(e)
        paths, nbytes = float(e[0]), float(e[1])
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    filled = float((idx >= 0).float().mean().item())
    # roofline of the walk kernel (lg_spread_tile_resource_topk_f64), this rank, per launch.
    # Its binding resource is the LDS atomic unit (one ds_add_f64 per 3-hop path into the
    # user's fp64 accumulator): achieved = the useful paths it adds per second (padding slots
    # excluded), peak = the measured random-column ds_add_f64 rate. The HBM side is reported
    # beside it: algorithmic bytes = the W-row bytes gathered (one 128-B line per (user, item)
    # and tile + overflow units) + 12 B of item id / ra per (user, item) + the user's list
    # read and written (2 k 16 B) + its score bounds (qstride + 4 nch B) + 16 B of row
    # pointers; time = HIP events around each launch on its stream.
    walk = None
    if st.get("walk_launches"):
        nl = st["walk_launches"]
        per_user = 2 * k * 16 + st.get("qstride", 0) + 4 * st.get("nch", 0) + 16
        alg = (st["w_bytes"] + 12 * st["user_items"] + per_user * st["users"] * nl) / nl
        ms = st["t_walk_ms"] / nl
        traffic, traffic_src = (None, {"status": "PMC records are for the C5 walks (2048-col tiles)"})
        if (U, I) == (1_000_000, 1_000_000) and tile == 2048:
            wl = f"c5-d{int(eu.shape[1])}"
            traffic, traffic_src = load_traffic(wl, 1, "spread_tiled.hip", f"{wl}/spread_walk")
        gpaths = st["w_paths"] / nl / ms / 1e6
        walk = {"bound": "lds-atomic", "achieved": gpaths, "peak": LDS_F64_ADD_PEAK_G,
                "unit": "G path-adds/s", "frac": gpaths / LDS_F64_ADD_PEAK_G,
                "peak_source": "profiles/r03_lds_atomic.txt (ds_add_f64, random columns, 8 "
                               "waves per CU)",
                "kernel": "lg_spread_tile_resource_topk_f64", "avg_launch_ms": ms,
                "launches": nl, "paths_per_launch": st["w_paths"] / nl,
                "hbm": {"achieved": alg / ms / 1e6, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": alg / ms / 1e6 / HBM_PEAK_GBS, "alg_bytes_per_launch": alg,
                        "traffic": traffic, "traffic_source": traffic_src},
                "build_ms_per_tile": st["t_build_ms"] / nl,
                "bounds_ms_per_tile": st["t_bounds_ms"] / nl}
    res = {"recs_per_s": U / dt, "users": U, "dim": int(eu.shape[1]), "seconds": dt, "k": k,
           "lambda": lam, "paths_per_s": paths / dt, "row_bytes_GBps": nbytes / dt / 1e9,
           "tile": tile, "filled_frac_rank0": filled, "roofline": walk,
           # the paths' split between P rows (one 4-byte slot per (user, item) pair) and V
           # rows (hub items: merged general_W entries, one 16-byte unit per column)
           "paths_v_rows_share": (st["w_paths_v"] / st["w_paths"]) if st["w_paths"] else None,
           "sharding": f"item range x{world} + all-to-all of per-range top-k lists",
           "path": "lg_spread_group_{cursor,bound,rows} + lg_score_chunk_bound (bf16 MFMA) + "
                   "lg_spread_tile_resource_topk_f64 (fused walk) + lg_topk_lists_merge_f64"}
    if parity and rank == 0:
        try:
            res["parity_vs_oracle"] = spread_parity_field(idx, u0, u1, A, eu, ei, lam, k)
        except Exception as ex:  # the checker never hides the measured result
            log(f"spread parity failed: {ex!r}")
    if extras:
        try:
            res["eval"] = bench_eval(idx, u0, u1, A, keys, U, I, k, rank, world, dev)
        except Exception as ex:  # a side measurement never hides the main result
            log(f"eval bench failed: {ex!r}")
    del A, idx
    torch.cuda.empty_cache()
    if extras and world == 1:
        res["c3_douban_shape"] = bench_dense_spread(dev, k, lam)
        torch.cuda.empty_cache()
    return res


def bench_dense_spread(dev, k, lam):
    """configs[2] stand-in: Douban-like (U=600, I=20000, 60000 Zipf(1.1) interactions), the
    dense spreading path of spread_recommend (W as an fp64 I x I matrix built with general_W
    in one pass, fused G * F top-k), end to end and per kernel with HIP events, each against
    its roofline (algorithmic bytes / HBM peak; general_W + HybridS: the I x I write,
    resource: the W rows gathered per (user, item) + the F write, rows top-k: the F read)."""
    from lgcnhs import ops
    from lgcnhs.synth import synth_interactions
    du, di, de = 600, 20_000, 60_000
    users, items = synth_interactions(du, di, de, seed=3, dist="zipf")
    g = torch.Generator(device=dev).manual_seed(42)
    deu = torch.randn(du, 64, device=dev, generator=g) * 0.1
    dei = torch.randn(di, 64, device=dev, generator=g) * 0.1

    def dense(ev=None):
        mark = (lambda i: ev[i].record()) if ev else (lambda i: None)
        mark(0)
        Ad = ops.Interactions.from_pairs(torch.as_tensor(users), torch.as_tensor(items), du,
                                         di, dev)
        mark(1)
        W = ops.spread_hybrid(Ad, lam)  # general_W + HybridS, one pass (spread_recommend's)
        mark(2)
        F = ops.spread_resource(Ad, W)
        mark(3)
        out = ops.rows_topk(F, k, Ad.by_user, True, deu, dei)
        mark(4)
        return out
    dense()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    t0 = time.perf_counter()
    dense(ev)
    torch.cuda.synchronize()
    dd = time.perf_counter() - t0
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(4)]
    I2 = 8.0 * di * di
    kern = {
        "lg_spread_hybrid_f64": (ms[1], I2),
        "lg_spread_resource_f64": (ms[2], 8.0 * de * di + 8.0 * du * di),
        "lg_rows_topk_f64": (ms[3], 8.0 * du * di),
    }
    roof = {n: {"ms": t, "alg_bytes": b, "achieved_GBs": b / t / 1e6,
                "frac": b / t / 1e6 / HBM_PEAK_GBS} for n, (t, b) in kern.items()}
    return {"users": du, "items": di, "interactions": de, "seconds": dd, "recs_per_s": du / dd,
            "kernels": roof, "setup_ms": ms[0],
            "path": "lg_spread_hybrid_f64 + lg_spread_resource_f64 + lg_rows_topk_f64"}


def bench_topk(e0_orig, keys, U, I, D, k, nu, rank, world, dev):
    """Masked full-catalog top-k (lg_score_topk_f32) for a block of ``nu`` users per rank
    over all items: recs/s over ranks, MFMA fraction. Returns (line, GPU lists of users
    [0, nu) when this rank's block starts at user 0, else None)."""
    from lgcnhs import ops
    from lgcnhs.graph import RowSets
    nu = min(nu, U)
    u0 = (rank * nu) % max(1, U - nu + 1)
    eu = e0_orig[u0:u0 + nu].contiguous()
    ei = e0_orig[U:U + I].contiguous()
    ku = keys[(keys >= u0 * I) & (keys < (u0 + nu) * I)]  # this block's positives
    excl = RowSets.from_pairs(ku // I - u0, ku % I, nu, I, dev)
    def timed(screen, reps=3):
        ops.score_topk(eu, ei, k, excl, screen=screen)  # warm-up
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            ops.score_topk(eu, ei, k, excl, screen=screen)
        e.record()
        torch.cuda.synchronize()
        tk = s.elapsed_time(e) / 1e3 / reps
        if world > 1:
            t = torch.tensor([tk], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            tk = float(t.item())
        return tk
    tk = timed(True)
    tp = timed(False)
    flops = 2.0 * nu * I * D
    # the screened kernel (the product default): every score is a bf16 MFMA product, the
    # exact fp32 chain runs only on the 16-item tiles the bound cannot rule out; its bf16
    # MFMA share is priced against the dense bf16 peak. The plain fp32-MFMA kernel is timed
    # beside it (same lists bit for bit).
    line = {"recs_per_s": nu * world / tk, "users_per_rank": nu, "items": I, "k": k, "dim": D,
            "ms": tk * 1e3, "fp32_equiv_tflops_per_gpu": flops / tk / 1e12,
            "bf16_screen_mfma_frac": flops / tk / 1e12 / BF16_MFMA_PEAK_TF,
            "kernel": "lg_score_topk_screened_f32 (bf16 MFMA 16x16x32 screen, bound-side "
                      "lists ranked by the exact f32 MFMA 16x16x4 chain at the end)",
            "unscreened": {"ms": tp * 1e3, "recs_per_s": nu * world / tp,
                           "tflops_per_gpu": flops / tp / 1e12,
                           "mfma_frac": flops / tp / 1e12 / F32_MFMA_PEAK_TF,
                           "kernel": "lg_score_topk_f32 (f32 MFMA 16x16x4 + streaming top-k)"}}
    line["roofline"] = topk_roofline(nu, I, D, k, tk)
    lists = ops.score_topk(eu, ei, k, excl)[1] if u0 == 0 else None
    return line, lists


def topk_roofline(nu, I, D, k, tk):
    """roofline of the screened top-K (MFMA-bound): the MFMA work it executes priced against
    the dense bf16 peak (k_topk_ring, bound-side lists, every k): the bf16 screen of every
    (user, item), plus the seed pass's screen of the first 1/16 of the items (catalogs of
    >= 1024 k items); the exact fp32 chains run only on the surviving entries per user
    (~k + 9 at k = 20) and are counted from the PMC record (f32 MFMAs beyond the screen's)
    at the bf16 / fp32 peak ratio. The record (profiles/pmc_topk.json,
    scripts/gpu_topk_pmc.sh + scripts/topk_pmc_summary.py) is used only if taken on this
    csrc/topk.hip at this shape (users per rank, items, k); it also gives the PMC MFMA-busy
    fraction and HBM traffic. Without one (e.g. the N > 1 lines' per-rank user blocks) the
    frac counts the screen alone and says so in frac_basis."""
    import hashlib
    sha = hashlib.sha256(open(os.path.join(PKG, "csrc", "topk.hip"), "rb").read()).hexdigest()[:16]
    key = f"c5-d{D}/topk" + ("" if k == 20 else f"_k{k}")
    rec, status = None, f"no PMC record for {key}"
    try:
        rec = json.load(open(os.path.join(REPO, "profiles", "pmc_topk.json"))).get(key)
    except Exception:
        rec = None
    scale = 1.0  # the record's exact chains per launch -> this launch's
    if rec is not None:
        if rec.get("kernel_sha") != sha:
            rec, status = None, "stale: recorded on another topk.hip"
        elif (rec.get("items"), rec.get("k")) != (I, k):
            rec, status = None, "recorded at another shape"
        elif rec.get("users") != nu:
            # another user block of the same catalog and k (the N > 1 lines' per-rank share):
            # the exact chains per user are a property of the workload, scaled by users
            scale, status = nu / rec["users"], "measured at N = 1, scaled per user"
        else:
            status = "measured"
    seeded = I // 16 // 16 * 16 >= 64 * k
    bf16 = 2.0 * nu * I * D * (1.0 + (1.0 / 16 if seeded else 0.0))
    # fp32 MFMA flops of the exact chains: 16x16x4 f32 MFMA = 2048 flop each
    f32 = 2048.0 * rec["f32_mfma_per_launch"] * scale if rec else 0.0
    achieved = (bf16 + f32 * BF16_MFMA_PEAK_TF / F32_MFMA_PEAK_TF) / tk / 1e12
    return {"bound": "mfma", "achieved": achieved, "peak": BF16_MFMA_PEAK_TF,
            "unit": "TFLOP/s (bf16-equivalent MFMA work)", "frac": achieved / BF16_MFMA_PEAK_TF,
            "traffic": rec.get("hbm_bytes_per_launch") if rec else None,
            "kernel": "lg_score_topk_screened_f32", "avg_launch_ms": tk * 1e3,
            "frac_basis": ("bf16 screen + seed pass + the exact chains" if rec else
                           "bf16 screen + seed pass only (no exact-chain record for this shape)"),
            "exact_f32_mfma_per_launch": rec["f32_mfma_per_launch"] * scale if rec else None,
            "pmc_mfma_busy_frac": rec.get("mfma_busy_frac") if rec else None,
            "pmc_avg_ms": rec.get("avg_ms") if rec else None,
            "pmc_wave_parked_frac": rec.get("wave_parked_frac") if rec else None,
            "record_source": {"status": status, "kernel_sha": sha,
                              "source": rec.get("source") if rec else None}}


def load_traffic(workload, world, src_name="spmm.hip", key=None):
    """roofline.traffic: HBM bytes per launch of a kernel from the PMC pass recorded in
    profiles/pmc_traffic.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, FETCH x 2 per the
    gfx950 correction; K1: scripts/gpu_traffic.sh + scripts/pmc_summary.py under
    "<workload>/n<world>", the K3s walk: scripts/gpu_traffic.sh +
    scripts/walk_traffic_summary.py under "c5-d64/spread_walk"). The entry is used only if
    the kernel source it was measured on (sha256 of csrc/<src_name>) is the one built now;
    otherwise traffic is null and the reason is reported."""
    import hashlib
    src = os.path.join(PKG, "csrc", src_name)
    sha = hashlib.sha256(open(src, "rb").read()).hexdigest()[:16]
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    key = key or f"{workload}/n{world}"
    try:
        d = json.load(open(path))
    except Exception:
        return None, {"status": "no PMC record", "kernel_sha": sha}
    e = d.get(key)
    if e is None:
        return None, {"status": f"no PMC record for {key}", "kernel_sha": sha}
    if e.get("kernel_sha") != sha:
        return None, {"status": f"stale: recorded on another {src_name}",
                      "recorded_sha": e.get("kernel_sha"), "kernel_sha": sha,
                      "source": e.get("source")}
    return float(e["hbm_bytes_per_launch"]), {"status": "measured", "kernel_sha": sha,
                                               "source": e.get("source")}


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int | None:
    """--gpus N without a torch.distributed launcher around us: start N ranks as a CHILD
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) and return its exit
    code; rank 0's JSON line reaches our stdout through the inherited pipe. Nothing here
    touches the GPU (the parent never initialises HIP, and never execs). Returns None when
    this process is itself a rank (WORLD_SIZE set) or N == 1. A launcher whose WORLD_SIZE
    differs from --gpus is an error: the line would report the wrong n_gpus."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            log(f"bench: WORLD_SIZE={env_world} but --gpus {args.gpus}")
            return 2
        return None
    if args.gpus <= 1:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    log(f"bench: launching {args.gpus} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd, env=env).returncode


def wants_cpu_baseline(rank: int, args) -> bool:
    """Rank 0 times the CPU baselines at every N (not only N = 1), unless switched off."""
    return rank == 0 and not args.no_cpu_baseline


def _host_layer(shard, piece, dis, x, y, x0, acc, out, mode, denom):
    """Host (torch CPU) stand-in for lgcnhs.dist.hip_layer over one piece of a shard, for
    the CPU launch check only: the same modes as lg_spmm_layer_f32 (1 FIRST, 2 MID, 3 LAST,
    4 FIRST+LAST)."""
    lb, le, off = piece
    if le <= lb:
        return
    rp = shard.rowptr
    e0, e1 = int(rp[lb]), int(rp[le])
    srcs = shard.src[e0:e1].long()
    rows = torch.repeat_interleave(torch.arange(le - lb), (rp[lb + 1:le + 1] - rp[lb:le]))
    w = dis[srcs] * dis[rows + off]
    v = torch.zeros(le - lb, x.shape[1]).index_add_(0, rows, w[:, None] * x[srcs])
    g = slice(off, off + le - lb)
    if y is not None:
        y[g] = v
    if mode == 1:
        acc[g] = x0[g] + v
    elif mode == 2:
        acc[g] += v
    elif mode == 3:
        out[g] = (acc[g] + v) / denom
    elif mode == 4:
        out[g] = (x0[g] + v) / denom


def launch_check(world: int, rank: int, args) -> None:
    """--launch-check: the rank plumbing alone (process group, one all-reduce, rank 0's
    JSON line), no GPU work; what the CPU tests drive through launch_ranks(). Rank 0 also
    runs the propagation CPU baseline on a small CPU graph through the same function and
    rank rule as the real line, and at N > 1 every rank times the overlapped bipartite
    forward over gloo through time_propagation, so the N > 1 cpu_baseline and comm fields are
    exercised without a GPU."""
    t = torch.ones(1)
    if world > 1:
        dist.all_reduce(t)
    g = torch.Generator().manual_seed(0)  # a small symmetric bipartite CSR, built on CPU
    U, I = 300, 400
    keys = torch.unique(torch.randint(0, U, (5000,), generator=g) * I +
                        torch.randint(0, I, (5000,), generator=g))
    rows = torch.cat([keys // I, keys % I + U])
    cols = torch.cat([keys % I + U, keys // I])
    order = torch.argsort(rows * (U + I) + cols)
    rows, src = rows[order], cols[order].to(torch.int32)
    rp = torch.zeros(U + I + 1, dtype=torch.int64)
    rp[1:] = torch.cumsum(torch.bincount(rows, minlength=U + I), 0)
    comm = None
    if world > 1:
        # the N > 1 line's comm block through the real timing code: the bipartite shards and
        # the overlapped forward over gloo, a host stand-in for the HIP layer
        from lgcnhs.dist import SegmentShard
        shard = SegmentShard(rp, src, [0, U, U + I], rank, world, "cpu", chunks=2)
        deg = (rp[1:] - rp[:-1]).float()
        dis = torch.where(deg > 0, deg.pow(-0.5), torch.zeros_like(deg))
        e0 = torch.randn(U + I, 16, generator=g) * 0.1
        _, _, comm = time_propagation(shard, shard.permute_rows(dis), e0, 16, 3, 2, 1, world,
                                      "cpu", layer_fn=_host_layer)
    cpu = None
    if wants_cpu_baseline(rank, args):
        cpu = cpu_baseline(rp, src, U + I, 16, 3, target_nnz=4000, reps=1)
    if rank == 0:
        print(json.dumps({"metric": "launch-check", "n_gpus": world,
                          "ranks_seen": int(t.item()), "cpu_baseline": cpu, "comm": comm}),
              flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c5-d64", choices=sorted(WORKLOADS))
    ap.add_argument("--topk-users", type=int, default=32768, help="users per rank for the top-K phase")
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--k-long", type=int, default=100,
                    help="the topk_k100 leg's list length (0: no leg)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-topk", action="store_true")
    ap.add_argument("--no-spread", action="store_true")
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL) | gloo (rehearsal only)")
    ap.add_argument("--same-device", action="store_true",
                    help="map every rank to cuda:0 (multi-rank rehearsal on a 1-GPU box)")
    ap.add_argument("--no-small", action="store_true",
                    help="skip the ML-1M-shaped (configs[1]) side measurement at N=1")
    ap.add_argument("--extra-dims", type=int, nargs="*", default=[128],
                    help="also time the same graph's propagation at these embedding widths")
    ap.add_argument("--extra-dim-legs", type=int, nargs="*", default=[128],
                    help="... and its top-K and spread legs at these widths (C5: d=128)")
    ap.add_argument("--chunks", type=int, default=0,
                    help="sub-chunks per rank per layer (per half with --layout bipartite) "
                         "for comm/compute overlap (0 = auto)")
    ap.add_argument("--layout", default="bipartite", choices=["bipartite", "rows"],
                    help="N>1 row sharding: users and items sharded separately with "
                         "cross-layer overlap (bipartite) or contiguous node rows (rows)")
    ap.add_argument("--spread-graphs", nargs="*", default=["c4-zipf"],
                    help="N = 1: of --other-graphs, also run LGCNHS (all users) on these")
    ap.add_argument("--other-graphs", nargs="*", default=["c5-zipf-d64", "c4-zipf"],
                    help="N = 1: also measure these graph shapes (other_graphs; the Zipf(1.1) "
                         "power-law input of SURVEY.md §8(d))")
    ap.add_argument("--launch-check", action="store_true",
                    help="rank plumbing only (process group + one all-reduce), no GPU work")
    args = ap.parse_args()

    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_device:
        local = 0
    if args.launch_check:
        if world > 1:
            dist.init_process_group(args.backend if args.backend != "nccl" else "gloo")
        launch_check(world, rank, args)
        return
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            # RCCL on a high-priority stream: its all-gather workgroups are dispatched ahead
            # of the queued SpMM workgroups they overlap with
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
            dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                    pg_options=opts)
        else:
            dist.init_process_group(args.backend)
    dev = torch.device("cuda", local)

    from lgcnhs import ops
    from lgcnhs.dist import RowShard, SegmentShard
    from lgcnhs.graph import RowSets

    U, I, E, D, L = WORKLOADS[args.workload]
    N = U + I
    t0 = time.time()
    rowptr, src, keys = gen_graph(U, I, E, seed=0, dev=dev,
                                  dist=GRAPH_DIST.get(args.workload, "uniform"))
    nnz = int(src.numel())
    from lgcnhs import _native as NV
    dis = torch.empty(N, dtype=torch.float32, device=dev)
    NV.check(NV.lib().lg_gcn_norm_f32(NV.ptr(rowptr), N, NV.ptr(dis), NV.stream_handle(dev)),
             "gcn_norm")
    wgt = torch.empty(nnz, dtype=torch.float32, device=dev)
    NV.check(NV.lib().lg_gcn_edge_weight_f32(NV.ptr(rowptr), NV.ptr(src), NV.ptr(dis), N, 0,
                                             NV.ptr(wgt), NV.stream_handle(dev)), "edge weights")
    if world > 1 and args.layout == "bipartite":
        # users and items sharded separately: one half's all-gather hides behind the other
        # half's SpMM, across layer boundaries (lgcnhs.dist.BipartitePropagation)
        chunks = args.chunks if args.chunks else 2
        shard = SegmentShard(rowptr, src, [0, U, N], rank, world, dev, weight=wgt,
                             chunks=chunks)
    else:
        chunks = args.chunks if args.chunks else (1 if world == 1 else 4)
        shard = RowShard(rowptr, src, N, rank, world, dev, weight=wgt, chunks=chunks)
    del wgt
    dis_l = shard.permute_rows(dis)
    gen = torch.Generator(device=dev).manual_seed(42)
    e0_orig = torch.randn(N, D, device=dev, generator=gen) * 0.1
    # the reference's CPU path beside every N's line (north_star: "in the same run"), on rank 0
    # after the timed region (the other ranks wait at the closing barrier)
    cpu_rp, cpu_src = (rowptr, src) if wants_cpu_baseline(rank, args) else (None, None)
    train_graph = (rowptr, src) if (world == 1 and not args.no_train) else None
    del rowptr
    if cpu_src is None:
        del src
    torch.cuda.synchronize()
    log(f"[rank {rank}] graph U={U} I={I} nnz={nnz} rows {getattr(shard, 'ranges', None) or (shard.g0, shard.g1)} "
        f"setup {time.time() - t0:.1f}s")

    elapsed, avg_kernel_s, comm = time_propagation(shard, dis_l, e0_orig, D, L, args.steps,
                                                   args.warmup, world, dev)
    edge_layers = nnz * L * args.steps
    value = edge_layers / elapsed
    # algorithmic bytes per SpMM launch: nnz*(8+4d) + rows*(4+4d)
    alg_bytes = shard.nnz * (8 + 4 * D) + shard.n_rows * (4 + 4 * D)
    achieved = alg_bytes / avg_kernel_s / 1e9
    job_bytes = nnz * (8 + 4 * D) + N * (4 + 4 * D)  # one layer of the whole graph
    traffic, traffic_src = load_traffic(args.workload, world)

    # the same graph at the other embedding widths the configs name (C5: d=128): the
    # propagation, and (--extra-dim-legs) the e0 top-K and the LGCNHS spread leg at that width
    extra = {}
    for d2 in args.extra_dims:
        if d2 == D:
            continue
        e2 = torch.randn(N, d2, device=dev, generator=gen) * 0.1
        el2, k2, _ = time_propagation(shard, dis_l, e2, d2, L, max(2, args.steps // 2), 1,
                                      world, dev)
        b2 = shard.nnz * (8 + 4 * d2) + shard.n_rows * (4 + 4 * d2)
        wl2 = args.workload.rsplit("-d", 1)[0] + f"-d{d2}" if "-d" in args.workload else None
        tr2, tr2_src = load_traffic(wl2, world) if wl2 else (None, {"status": "no record"})
        extra[f"d{d2}"] = {"value": nnz * L * max(2, args.steps // 2) / el2,
                           "unit": "edge-layers/s", "ms_per_step": el2 / max(2, args.steps // 2) * 1e3,
                           "roofline_frac": b2 / k2 / 1e9 / HBM_PEAK_GBS,
                           "achieved_GBs": b2 / k2 / 1e9, "avg_launch_ms": k2 * 1e3,
                           "alg_bytes_per_launch": b2, "traffic": tr2,
                           "traffic_source": tr2_src}
        if d2 in args.extra_dim_legs:
            e2o = e2  # original node order (time_propagation permutes its own copy)
            if not args.no_topk:
                try:
                    extra[f"d{d2}"]["topk"], _ = bench_topk(e2o, keys, U, I, d2, args.k,
                                                            args.topk_users, rank, world, dev)
                except Exception as ex:
                    log(f"d{d2} topk bench failed: {ex!r}")
            if not args.no_spread:
                try:
                    extra[f"d{d2}"]["spread"] = bench_spread(
                        keys, U, I, e2o, args.k, rank, world, dev, extras=False,
                        parity=not args.no_cpu_baseline)
                except Exception as ex:
                    log(f"d{d2} spread bench failed: {ex!r}")
            del e2o
        del e2
        torch.cuda.empty_cache()

    other_graphs = {}
    if world == 1:
        for name in args.other_graphs:
            try:
                other_graphs[name.split("-d")[0].replace("c5-", "").replace("c4-", "c4_")] = \
                    bench_other_graph(name, dev, max(3, args.steps // 2), args.k,
                                      args.topk_users, cpu_parity=not args.no_cpu_baseline,
                                      spread=name in args.spread_graphs)
            except Exception as ex:  # a side measurement never hides the main result
                log(f"{name} bench failed: {ex!r}")
            torch.cuda.empty_cache()

    train = None
    if train_graph is not None:  # after the timed forwards: it leaves the caches cold
        try:
            train = bench_train(*train_graph, keys, U, I, e0_orig, D, L, dev)
        except Exception as ex:  # a side measurement never hides the main result
            log(f"train bench failed: {ex!r}")
        del train_graph
        torch.cuda.empty_cache()

    topk = topk_gpu_lists = None
    if not args.no_topk:
        topk, topk_gpu_lists = bench_topk(e0_orig, keys, U, I, D, args.k, args.topk_users,
                                          rank, world, dev)
    # the reference's production list length (const.py:433, k = 100) on the same users
    topk_k100 = topk_k100_lists = None
    if not args.no_topk and args.k_long and args.k_long != args.k:
        try:
            topk_k100, topk_k100_lists = bench_topk(e0_orig, keys, U, I, D, args.k_long,
                                                    args.topk_users, rank, world, dev)
        except Exception as ex:  # a side measurement never hides the main result
            log(f"k={args.k_long} topk bench failed: {ex!r}")

    spread = None
    if not args.no_spread:
        try:
            spread = bench_spread(keys, U, I, e0_orig, args.k, rank, world, dev,
                                  parity=not args.no_cpu_baseline)
        except Exception as ex:  # a side measurement never hides the main result
            log(f"spread bench failed: {ex!r}")

    small = None
    if world == 1 and not args.no_small:
        try:
            small = bench_small_config(dev, args.k)
        except Exception as ex:  # an auxiliary measurement never hides the main result
            log(f"small-config bench failed: {ex!r}")

    cpu = cpu_topk = cpu_spread = None
    if cpu_src is not None:
        try:
            cpu = cpu_baseline(cpu_rp, cpu_src, N, D, L)
            cpu_topk, cpu_lists = cpu_baseline_topk(e0_orig, keys, U, I, args.k)
            if topk is not None and topk_gpu_lists is not None:
                n_cmp = min(cpu_lists.shape[0], topk_gpu_lists.shape[0])
                topk["parity_vs_cpu_reference"] = topk_parity(
                    topk_gpu_lists[:n_cmp], cpu_lists[:n_cmp], e0_orig, U, D, args.k)
            if topk_k100 is not None and topk_k100_lists is not None:
                _, cpu_l100 = cpu_baseline_topk(e0_orig, keys, U, I, args.k_long, n_users=1024)
                topk_k100["parity_vs_cpu_reference"] = topk_parity(
                    topk_k100_lists[:1024], cpu_l100, e0_orig, U, D, args.k_long)
            cpu_spread = cpu_baseline_spread(args.k)
        except Exception as ex:  # the baseline must never hide the GPU result
            log(f"cpu baseline failed: {ex!r}")
    if rank == 0:
        line = {
            "metric": "propagation edges/sec + full-catalog top-K recs/sec, 1/2/4/8 MI355X",
            "value": value, "unit": "edge-layers/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic (uniform bipartite, seed 0; e0 ~ N(0, 0.1^2))",
            "config": {"workload": args.workload, "users": U, "items": I, "interactions": E,
                       "directed_nnz": nnz, "dim": D, "layers": L,
                       "parallelism": f"row-shard x{world} + RCCL all-gather per layer"
                                      + (f" ({args.layout} layout, {chunks} sub-chunks)"
                                         if world > 1 else "")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "lg_spmm_layer_f32",
                         "avg_launch_ms": avg_kernel_s * 1e3,
                         "alg_bytes_per_launch": alg_bytes,
                         # north_star's end-to-end figure: value (all ranks, all-gathers
                         # included) against N GPUs' HBM-roofline edge-layers/s for the
                         # whole graph's algorithmic bytes per edge-layer
                         "job_edge_layers_roofline": world * HBM_PEAK_GBS * 1e9 * nnz / job_bytes,
                         "job_frac": value / (world * HBM_PEAK_GBS * 1e9 * nnz / job_bytes)},
            "comm": comm,
            "topk": topk,
            "topk_k100": topk_k100,
            "spread": spread,
            "train": train,
            "other_dims": extra,
            "other_graphs": other_graphs,
            "c2_ml1m_shape": small,
            "cpu_baseline": cpu,
            "cpu_baseline_topk": cpu_topk,
            "cpu_baseline_spread": cpu_spread,
            "host": platform.node(),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
