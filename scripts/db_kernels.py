"""Per-(kernel, grid) summary of a rocprofv3 sqlite (.db) kernel trace.
Usage: python scripts/db_kernels.py <results.db> [top]"""
import re
import sqlite3
import sys
from collections import defaultdict

c = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
g = defaultdict(list)
for name, dur, grid, wg, vg, sg, lds, scr in c.execute(
        "select name, duration, grid_x, workgroup_x, vgpr_count, sgpr_count, lds_size, "
        "scratch_size from kernels"):
    m = re.search(r"(lg::[A-Za-z_0-9]+(<[^>]*>)?)", name)
    k = m.group(1) if m else name[:60]
    g[(k, grid, wg, vg, lds, scr)].append(dur / 1e6)
tot = sum(sum(v) for v in g.values())
print(f"all kernels {tot:.1f} ms")
for (k, grid, wg, vg, lds, scr), d in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{k:58s} grid={grid:8d} wg={wg:4d} vgpr={vg:3d} lds={lds:6d} scr={scr:4d} n={len(d):4d} "
          f"avg={sum(d) / len(d):8.3f} tot={sum(d):9.1f}")
