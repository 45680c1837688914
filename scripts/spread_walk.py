"""Time ops.spread_topk_tiled (the pipelined tile walk) over the first --tiles item tiles
for all users of the C5 graph; with rocprofv3 --kernel-trace the timeline shows whether the
next tile's W build overlaps the current tile's resource pass (scripts/overlap.py)."""
import argparse
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from lgcnhs import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tiles", type=int, default=16)
ap.add_argument("--tile", type=int, default=2048)
ap.add_argument("--workload", default="c5-d64")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--no-g", action="store_true", help="no G factor (SpreadMethod)")
ap.add_argument("--count", action="store_true", help="count paths / row bytes (extra work)")
ap.add_argument("--no-col-bounds", action="store_true",
                help="chunk score bounds only (no per-column 8-bit bounds)")
ap.add_argument("--no-excl", action="store_true",
                help="no exclusion sets (timing of the walk without the per-user exclusion cursor)")
ap.add_argument("--identity-classes", action="store_true",
                help="class = degree (the walk_recip A/B variant computes fl(1/k) itself)")
a = ap.parse_args()
if a.identity_classes:
    def _identity_classes(deg):
        n = max(ops.INV_TAB, int(deg.max()) + 1)
        if n > ops.MAX_CLASSES:
            raise ValueError("degree too large for identity classes")
        inv = torch.zeros(n, dtype=torch.float64, device=deg.device)
        inv[1:] = 1.0 / torch.arange(1, n, dtype=torch.float64, device=deg.device)
        return deg.to(torch.int16).view(torch.uint16), inv
    ops.degree_classes = _identity_classes
dev = torch.device("cuda:0")
U, I, E, D, _ = bench.WORKLOADS[a.workload]
_, _, keys = bench.gen_graph(U, I, E, 0, dev, dist=bench.GRAPH_DIST.get(a.workload, "uniform"))
A = ops.Interactions.from_pairs(keys // I, keys % I, U, I, dev)
del keys
g = torch.Generator(device=dev).manual_seed(42)
eu = torch.randn(U, D, device=dev, generator=g) * 0.1
ei = torch.randn(I, D, device=dev, generator=g) * 0.1
kw = {} if a.no_g else {"eu": eu, "ei": ei, "col_bounds": not a.no_col_bounds}
for rep in range(a.reps):
    torch.cuda.synchronize()
    t = time.time()
    st = {}
    vals, idxs = ops.spread_topk_tiled(A, 0.5, 20, None if a.no_excl else A.by_user, tile=a.tile,
                          items=slice(0, a.tiles * a.tile),
                          stats=st if rep == 0 else None, count_paths=a.count, **kw)
    torch.cuda.synchronize()
    dt = time.time() - t
    print(f"rep {rep}: {a.tiles} tiles x {U} users: {dt:.3f} s"
          + (f"  paths {st.get('w_paths', 0):.3e} (V rows {st.get('w_paths_hub', 0):.3e})"
             f" bytes {st.get('w_bytes', 0):.3e}"
             f"  build {st.get('t_build_ms', 0):.1f} ms bounds {st.get('t_bounds_ms', 0):.1f} ms"
             f" walk {st.get('t_walk_ms', 0):.1f} ms" if st else ""), flush=True)
    h = (idxs.to(torch.float64) * torch.arange(1, 21, device=dev, dtype=torch.float64)).sum()
    print(f"  lists checksum {float(h):.17g} values sum {float(vals[torch.isfinite(vals)].sum()):.17g}",
          flush=True)
    if st.get("walk_ms_list"):
        wl = st["walk_ms_list"]
        h = len(wl) // 3
        print(f"  walk ms per tile: first {h} {sum(wl[:h]) / max(1, h):.3f}, "
              f"rest {sum(wl[h:]) / max(1, len(wl) - h):.3f}", flush=True)
