"""Where the screened top-K's time goes at C5 (1M items, 32768 users, k=20): the screened
kernel with the real margins, with every tile recomputed (margins +1e30: the exact chain on
every tile) and with the screen alone (margins -1e30: a tile is recomputed only while a
list can still take the mask value; the lists are then wrong -- timing only). The fraction
of tiles the real screen recomputes follows as (t_real - t_none) / (t_all - t_none)."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd")]
import torch  # noqa: E402

from lgcnhs import _native as N  # noqa: E402
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
    ub, un = ops.bound_operands(eu)
    ib, inorm = ops.bound_operands(ei)
    real = un * (inorm.max() * ops.SCREEN_MARGIN)
    ns = ops._splits_for(U, I, k, ops._resident_blocks(dev, k, True), True)
    wsb = N.lib().lg_score_topk_ws_bytes(U, I, D, k, ns)
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    val = torch.empty((U, k), dtype=torch.float32, device=dev)
    idx = torch.empty((U, k), dtype=torch.int64, device=dev)
    res = {}
    for name, m in (("real", real), ("all", torch.full_like(real, 1e30)),
                    ("none", torch.full_like(real, -1e30))):
        def run():
            N.check(N.lib().lg_score_topk_screened_f32(
                N.ptr(eu), N.ptr(ei), N.ptr(ub), N.ptr(ib), N.ptr(m), U, I, D,
                N.ptr(excl.rowptr), N.ptr(excl.col), float(ops.MASK_VALUE), k, ns, N.ptr(val),
                N.ptr(idx), N.ptr(ws), wsb, N.stream_handle(dev)), "screened")
        run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(3):
            run()
        e.record()
        torch.cuda.synchronize()
        res[name] = s.elapsed_time(e) / 3
    h = (res["real"] - res["none"]) / max(1e-9, res["all"] - res["none"])
    print(f"d={D} splits={ns}: real {res['real']:.2f} ms, every tile exact {res['all']:.2f} ms, "
          f"screen only {res['none']:.2f} ms -> recomputed fraction ~{h:.3f}", flush=True)
