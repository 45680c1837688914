"""Time ops.score_topk over the C5 catalog (1M items, 32768 users, k=20, e0 ~ N(0, 0.1^2)):
the bf16-screened kernel against the plain fp32-MFMA one, lists compared bit for bit."""
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd")]
import torch  # noqa: E402

from lgcnhs import ops  # noqa: E402
from lgcnhs.graph import RowSets  # noqa: E402

dev = torch.device("cuda:0")
U, I, k = 32768, 1_000_000, 20
for D in (64, 128):
    g = torch.Generator(device=dev).manual_seed(42)
    eu = torch.randn(U, D, device=dev, generator=g) * 0.1
    ei = torch.randn(I, D, device=dev, generator=g) * 0.1
    ku = torch.unique(torch.randint(0, U, (U * 100,), device=dev, generator=g) * I +
                      torch.randint(0, I, (U * 100,), device=dev, generator=g))
    excl = RowSets.from_pairs(ku // I, ku % I, U, I, dev)
    res = {}
    for screen in (True, False):
        for ns in (None, 1):
            ops.score_topk(eu, ei, k, excl, n_splits=ns, screen=screen)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(3):
                v, i = ops.score_topk(eu, ei, k, excl, n_splits=ns, screen=screen)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / 3
            res[(screen, ns)] = (v, i)
            print(f"d={D} screen={screen} splits={ns}: {dt * 1e3:.2f} ms  "
                  f"{U / dt / 1e6:.2f} M users/s  {2 * U * I * D / dt / 1e12:.0f} fp32-equiv TFLOP/s",
                  flush=True)
    base = res[(False, None)]
    for key, (v, i) in res.items():
        same = torch.equal(i, base[1]) and torch.equal(v.view(torch.int32), base[0].view(torch.int32))
        print(f"  {key}: identical to plain = {same}", flush=True)
