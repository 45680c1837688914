"""Time ops.score_topk over the C5 catalog (1M items, 32768 users, k=20 (--k), e0 ~ N(0, 0.1^2)):
the bf16-screened kernel against the plain fp32-MFMA one, lists compared bit for bit.
  --dims 64,128   embedding widths       --modes screen,plain   kernels
  --splits auto,1 item splits            --reps 3               timed calls per case"""
import argparse
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd")]
import torch  # noqa: E402

from lgcnhs import ops  # noqa: E402
from lgcnhs.graph import RowSets  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dims", default="64,128")
ap.add_argument("--modes", default="screen,plain")
ap.add_argument("--splits", default="auto,1")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--users", type=int, default=32768)
ap.add_argument("--k", type=int, default=20)
ap.add_argument("--items", type=int, default=1_000_000)
ap.add_argument("--no-excl", action="store_true", help="no exclusion sets")
args = ap.parse_args()
import ctypes  # noqa: E402
from lgcnhs import _native as NV  # noqa: E402
_lib = NV.lib()
counts = getattr(_lib, "lg_topk_counts", None)  # (measurement builds with -DLG_TOPK_COUNT)
if counts is not None:
    counts.argtypes, counts.restype = [ctypes.c_void_p], ctypes.c_int
    _buf = (ctypes.c_ulonglong * 16)()
    counts(_buf)

dev = torch.device("cuda:0")
U, I, k = args.users, args.items, args.k
for D in [int(x) for x in args.dims.split(",")]:
    g = torch.Generator(device=dev).manual_seed(42)
    eu = torch.randn(U, D, device=dev, generator=g) * 0.1
    ei = torch.randn(I, D, device=dev, generator=g) * 0.1
    ku = torch.unique(torch.randint(0, U, (U * 100,), device=dev, generator=g) * I +
                      torch.randint(0, I, (U * 100,), device=dev, generator=g))
    excl = None if args.no_excl else RowSets.from_pairs(ku // I, ku % I, U, I, dev)
    res = {}
    for mode in args.modes.split(","):
        screen = mode == "screen"
        for sp in args.splits.split(","):
            ns = None if sp == "auto" else int(sp)
            ops.score_topk(eu, ei, k, excl, n_splits=ns, screen=screen)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(args.reps):
                v, i = ops.score_topk(eu, ei, k, excl, n_splits=ns, screen=screen)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / args.reps
            res[(mode, sp)] = (v, i)
            if counts is not None and screen:
                counts(_buf)
                names = ["inserted", "hit_group_tiles", "compactions", "escapes", "excl_loads",
                         "final_entries", "users_finished"]
                c = [x / (args.reps + 1) for x in _buf[:7]]
                print("  counts per call: " + ", ".join(f"{n} {v:.4g}" for n, v in zip(names, c)) +
                      f"  (per user: inserted {c[0] / U:.1f}, compactions {c[2] / U:.2f}, "
                      f"escapes {c[3] / U:.3f}, excl loads {c[4] / U:.2f}, "
                      f"final entries {c[5] / max(c[6], 1):.1f})", flush=True)
                cyc = [x / (args.reps + 1) for x in _buf[:16]]
                if cyc[13]:
                    print("  cycles (share of the wave's): " + ", ".join(
                        f"{n} {cyc[i] / cyc[13]:.3f}" for n, i in (
                            ("ring", 8), ("(buffer-free wait", 14), ("dma+vmcnt+signal", 15),
                            ("arrival wait)", 7), ("screen+tests", 9), ("insertion", 10),
                            ("compaction", 11), ("final", 12))), flush=True)
            print(f"d={D} {mode} splits={sp}: {dt * 1e3:.2f} ms  "
                  f"{U / dt / 1e6:.2f} M users/s  {2 * U * I * D / dt / 1e12:.0f} fp32-equiv TFLOP/s",
                  flush=True)
    base = next(iter(res.values()))
    for key, (v, i) in res.items():
        same = torch.equal(i, base[1]) and torch.equal(v.view(torch.int32), base[0].view(torch.int32))
        print(f"  {key}: identical to {next(iter(res))} = {same}", flush=True)
