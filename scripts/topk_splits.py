"""Screened top-K (C5 catalog, 32768 users, k=20) timed over item-range split counts: with
n_splits = 8 (16) the splits land one (two) per XCD (blockIdx % n_splits = split, blocks
dispatched round-robin over the 8 XCDs), so each XCD's L2 streams 1/8 of the item table."""
import os
import sys

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
    base = None
    for screen in (True, False):
        for ns in (None, 2, 4, 8, 16, 24, 32):
            v, i = ops.score_topk(eu, ei, k, excl, n_splits=ns, screen=screen)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(3):
                ops.score_topk(eu, ei, k, excl, n_splits=ns, screen=screen)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / 3
            if base is None:
                base = i
            print(f"d={D} screen={screen} n_splits={ns}: {ms:.2f} ms  {U / ms / 1e3:.2f} M users/s"
                  f"  same lists: {torch.equal(i, base)}", flush=True)
