"""Side benchmark of the factored LGCNHS spreading path (K3s, lgcnhs.ops.spread_topk_tiled)
at catalog sizes whose I x I matrices cannot exist (C4: 200K x 200K, C5: 1M x 1M).

Per item tile the work splits into a user-independent part (the tile of W, built once per
tile: cursor + bound + weight kernels) and a per-user part (F tile + G*F top-K merge). The
script times both over all tiles for a sample of users and reports the measured time for the
sample and the projection to a full user shard:
    t(users) = t_build(all tiles) + users * t_user.
Usage: python scripts/bench_spread.py [--workload c5-d64] [--users 16384] [--tile 2048]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from lgcnhs import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c5-d64", choices=["c5-d64", "c5-d128", "c4"])
    ap.add_argument("--users", type=int, default=16384)
    ap.add_argument("--tile", type=int, default=2048)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--lam", type=float, default=0.5)
    ap.add_argument("--scratch-gib", type=int, default=4)
    ap.add_argument("--max-tiles", type=int, default=0,
                    help="stop after this many tiles (quick kernel iteration / profiling); "
                         "the projection then scales the measured times to all tiles")
    a = ap.parse_args()
    dev = torch.device("cuda")
    U, I, E, D, _ = bench.WORKLOADS[a.workload]
    t0 = time.time()
    _, _, keys = bench.gen_graph(U, I, E, 0, dev)
    A = ops.Interactions.from_pairs(keys // I, keys % I, U, I, dev)
    del keys
    g = torch.Generator(device=dev).manual_seed(42)
    eu = torch.randn(U, D, device=dev, generator=g) * 0.1
    ei = torch.randn(I, D, device=dev, generator=g) * 0.1
    torch.cuda.synchronize()
    print(f"graph U={U} I={I} E={E} d={D} setup {time.time() - t0:.1f}s", file=sys.stderr,
          flush=True)

    n = min(a.users, U)
    tile = a.tile
    span = max(tile, a.scratch_gib * (1 << 30) // (n * 8) // tile * tile)
    span = min(span, -(-I // tile) * tile)
    vals = torch.full((n, a.k), float("-inf"), dtype=torch.float64, device=dev)
    idxs = torch.full((n, a.k), -1, dtype=torch.int64, device=dev)
    F = torch.empty((n, span), dtype=torch.float64, device=dev)
    tw = ops.TileWeights(A, a.lam, tile)
    ex = A.by_user.slice_rows(0, n)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    t_build = t_res = t_topk = 0.0
    entries = 0
    tiles = 0
    torch.cuda.synchronize()
    wall = time.time()
    last = wall
    I_run = I if a.max_tiles <= 0 else min(I, a.max_tiles * tile)
    for s0 in range(0, I_run, span):
        s1 = min(I_run, s0 + span)
        for j0 in range(s0, s1, tile):
            e0, e1, e2 = ev(), ev(), ev()
            e0.record()
            tw.build(j0)
            e1.record()
            tw.resource(0, n, F[:, j0 - s0:])
            e2.record()
            e2.synchronize()
            t_build += e0.elapsed_time(e1) / 1e3
            t_res += e1.elapsed_time(e2) / 1e3
            entries += int(tw.row_len[:I].sum())
            tiles += 1
        e0, e1 = ev(), ev()
        e0.record()
        ops.tile_topk(F, s0, s1 - s0, a.k, vals, idxs, s0 == 0, ex, True, eu[:n], ei)
        e1.record()
        e1.synchronize()
        t_topk += e0.elapsed_time(e1) / 1e3
        if time.time() - last > 30:
            print(f"  tile {tiles} build {t_build:.2f}s resource {t_res:.2f}s topk "
                  f"{t_topk:.2f}s", file=sys.stderr, flush=True)
            last = time.time()
    scale = -(-I // tile) / tiles
    t_build, t_res, t_topk = t_build * scale, t_res * scale, t_topk * scale
    t_user = t_res + t_topk
    wall = time.time() - wall
    per_user = t_user / n
    res = {
        "workload": a.workload, "users": U, "items": I, "interactions": E, "dim": D,
        "k": a.k, "lambda": a.lam, "tile": tile, "tiles": tiles, "sample_users": n,
        "span": span, "w_entries": entries, "t_build_s": t_build, "t_resource_s": t_res,
        "t_topk_s": t_topk, "t_users_s": t_user, "wall_s": wall,
        "per_user_us": per_user * 1e6,
        "sample_recs_per_s": n / (t_build + t_user),
        "projected": {f"{w}gpu": {"users_per_gpu": -(-U // w),
                                  "seconds": t_build + -(-U // w) * per_user,
                                  "recs_per_s_total": U / (t_build + -(-U // w) * per_user)}
                      for w in (1, 8)},
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
