"""A/B of lg_score_topk_f32 variants in ONE process (interleaved rounds, median), on the
bench's top-K shape: 32768 users x 1M items, d=64, k=20, random exclusions."""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd"))
import torch  # noqa: E402

from lgcnhs import ops  # noqa: E402
from lgcnhs.graph import RowSets  # noqa: E402

dev = torch.device("cuda")
U, I, D, K = int(os.environ.get("AB_USERS", 32768)), 1_000_000, 64, 20
g = torch.Generator(device=dev).manual_seed(0)
eu = torch.randn(U, D, device=dev, generator=g) * 0.1
ei = torch.randn(I, D, device=dev, generator=g) * 0.1
nex = U * 100
ex = RowSets.from_pairs(torch.randint(0, U, (nex,), device=dev, generator=g),
                        torch.randint(0, I, (nex,), device=dev, generator=g), U, I, dev)
variants = {v: os.environ.copy() for v in sys.argv[1:] or ["PF=1", "PF=2"]}
times = {v: [] for v in variants}
ref = None
for rnd in range(5):
    for v in variants:
        for kv in v.split(","):
            key, val = kv.split("=")
            os.environ["LGCNHS_TOPK_" + key] = val
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        val_, idx = ops.score_topk(eu, ei, K, ex)
        e.record()
        torch.cuda.synchronize()
        times[v].append(s.elapsed_time(e))
        if ref is None:
            ref = idx.clone()
        for kv in v.split(","):
            os.environ.pop("LGCNHS_TOPK_" + kv.split("=")[0], None)
        if "PROBE" not in v:
            assert torch.equal(idx, ref), f"variant {v} differs"
for v, t in times.items():
    ms = statistics.median(t[1:])
    print(f"{v}: median {ms:.2f} ms  min {min(t[1:]):.2f}  -> {U / ms * 1e3:.0f} users/s, "
          f"{2 * U * I * D / ms / 1e9:.1f} TFLOP/s")
