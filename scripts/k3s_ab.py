"""A/B of walk-kernel variants (LGCNHS_WALK_UC) on the first 16 C5 tiles, no G factor."""
import os
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import os, sys, time
R = REPO_ROOT
sys.path[:0] = [R, os.path.join(R, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd")]
import torch, bench
from lgcnhs import ops
dev = torch.device("cuda:0")
U, I, E, D, _ = bench.WORKLOADS["c5-d64"]
_, _, keys = bench.gen_graph(U, I, E, 0, dev)
A = ops.Interactions.from_pairs(keys // I, keys % I, U, I, dev)
del keys
for rep in range(2):
    torch.cuda.synchronize(); t = time.time()
    ops.spread_topk_tiled(A, 0.5, 20, A.by_user, tile=2048, items=slice(0, 16 * 2048))
    torch.cuda.synchronize()
    print(f"variant {os.environ.get('LGCNHS_WALK_UC', '0')} rep {rep}: {time.time() - t:.3f} s", flush=True)
'''.replace("REPO_ROOT", repr(R))
for v in sys.argv[1:] or ["4", "2", "8"]:
    env = dict(os.environ, LGCNHS_WALK_UC=v)
    subprocess.run([sys.executable, "-u", "-c", code], env=env, check=True, timeout=200)
