"""Overlap of kernel families in a rocprofv3 kernel trace: for each W-build kernel, the
fraction of its duration that runs concurrently with a resource / top-K kernel."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
big = [(s, e) for s, e, n in iv if "k_tile_resource" in n or "k_tile_topk" in n]
fam = {}
for s, e, n in iv:
    if any(x in n for x in ("k_tile_weight", "k_tile_bound", "k_tile_cursor")):
        ov = sum(max(0, min(e, e2) - max(s, s2)) for s2, e2 in big)
        key = n.split("(")[0].replace("void ", "")
        t, o = fam.get(key, (0, 0))
        fam[key] = (t + (e - s), o + ov)
for k, (t, o) in fam.items():
    print(f"{k}: {t / 1e6:.1f} ms total, {o / max(t, 1):.0%} overlapped with resource/top-K")
s0 = min(s for s, _, _ in iv); e0 = max(e for _, e, _ in iv)
busy = sum(e - s for s, e, _ in iv)
print(f"span {(e0 - s0) / 1e6:.1f} ms, kernel time {busy / 1e6:.1f} ms")
