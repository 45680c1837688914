"""Where the score-bound kernel's time goes at C5 (1M users, one 2048-column tile, D = 64):
lg_score_chunk_bound with the per-column q bytes, with gb only (no q), and a plain 2 GB
device write (torch fill_) as the HBM write ceiling for the q bytes. Prints one JSON line.
Usage: python scripts/micro_bound.py [--users 1000000] [--dim 64]"""
import argparse
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd")]
import torch  # noqa: E402

from lgcnhs import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--users", type=int, default=1_000_000)
ap.add_argument("--items", type=int, default=1_000_000)
ap.add_argument("--dim", type=int, default=64)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(1)
eu = torch.randn(a.users, a.dim, device=dev, generator=g) * 0.1
ei = torch.randn(a.items, a.dim, device=dev, generator=g) * 0.1
ub, un = ops.bound_operands(eu)
ib, inn = ops.bound_operands(ei)
T = 2048
gb = torch.empty(a.users * (T // 64), dtype=torch.float32, device=dev)
q = torch.empty(a.users, T, dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream(dev)


def timed(fn):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for r in range(a.reps):
        fn(r)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.reps


def with_q(r=0):
    ops.chunk_bounds(ub, un, ib, inn, a.dim, (r * T) % (a.items - T), T, out=gb, qout=q)


def gb_only(r=0):
    ops.chunk_bounds(ub, un, ib, inn, a.dim, (r * T) % (a.items - T), T, out=gb)


def fill(r=0):
    q.fill_(r & 255)


def strided(piece):
    # the q bytes written piece by piece: every row's `piece` bytes of one column block, then the
    # next block (the kernel's write pattern: at a time, one chunk of many users' rows)
    v = q.view(a.users, T // piece, piece)

    def f(r=0):
        for c in range(T // piece):
            v[:, c].fill_(r & 255)
    return f


def blocked(rows):
    # a [n / rows][chunk][rows][64 B] layout: per chunk, every block of `rows` rows as one
    # contiguous 64 rows-byte piece
    v = q.view(a.users // rows, T // 64, rows * 64)

    def f(r=0):
        for c in range(T // 64):
            v[:, c].fill_(r & 255)
    return f


res = {"users": a.users, "tile": T, "dim": a.dim,
       "fill_blk16_ms": timed(blocked(16)), "fill_blk64_ms": timed(blocked(64)),
       "with_q_ms": timed(with_q), "gb_only_ms": timed(gb_only), "fill_q_ms": timed(fill),
       "fill_64B_pieces_ms": timed(strided(64)), "fill_128B_pieces_ms": timed(strided(128)),
       "fill_256B_pieces_ms": timed(strided(256))}
with_q(0)  # bitwise fingerprint of one tile's bounds (A/B builds must agree)
torch.cuda.synchronize()
res["q_sum"] = int(q.to(torch.int64).sum())
res["gb_bits_sum"] = int(gb.view(torch.int32).to(torch.int64).sum())
qbytes = a.users * T
res["fill_GBps"] = qbytes / res["fill_q_ms"] / 1e6
res["with_q_write_GBps"] = (qbytes + gb.numel() * 4) / res["with_q_ms"] / 1e6
res["mfma_TFLOPs_with_q"] = 2 * a.users * T * a.dim / res["with_q_ms"] / 1e9
print(json.dumps(res), flush=True)
