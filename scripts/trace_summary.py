"""Per-(kernel, launch shape) summary of a rocprofv3 --kernel-trace run
(gpurun_out/<dir>/run_kernel_trace.csv) -> markdown + json under profiles/.
The bench runs side configurations too, so every lg:: kernel is split by grid size.
Usage: python scripts/trace_summary.py <trace_dir> <out_stem> [command]"""
import csv
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(lg::[A-Za-z_0-9]+(<[^>]*>)?)", name)
    if m:
        return m.group(1)
    m = re.search(r"_ZN2lg(\d+)([A-Za-z_0-9]+)", name)  # names the tracer left mangled
    if m:
        return "lg::" + m.group(2)[:int(m.group(1))]
    return None


def main(trace_dir, stem, command=""):
    groups = defaultdict(list)
    total = 0.0
    for r in csv.DictReader(open(os.path.join(trace_dir, "run_kernel_trace.csv"))):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        total += d
        k = short(r["Kernel_Name"])
        if k:
            groups[(k, int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))].append(d)
    rows = []
    for (k, grid, wg), d in groups.items():
        rows.append({"kernel": k, "grid_size": grid, "workgroup": wg, "calls": len(d),
                     "avg_ms": sum(d) / len(d), "min_ms": min(d), "max_ms": max(d),
                     "total_ms": sum(d)})
    rows.sort(key=lambda r: -r["total_ms"])
    out = {"command": command, "all_kernels_total_ms": total, "lg_kernels": rows}
    json.dump(out, open(stem + ".json", "w"), indent=1)
    with open(stem + ".md", "w") as f:
        f.write(f"# rocprofv3 kernel trace summary\n\n`{command}`\n\n")
        f.write(f"All kernels: {total:.1f} ms. lg:: kernels by launch shape "
                "(grid = work-items):\n\n")
        f.write("| kernel | grid | wg | calls | avg ms | min ms | max ms | total ms |\n")
        f.write("|---|---|---|---|---|---|---|---|\n")
        for r in rows:
            f.write(f"| `{r['kernel']}` | {r['grid_size']} | {r['workgroup']} | {r['calls']} | "
                    f"{r['avg_ms']:.4f} | {r['min_ms']:.4f} | {r['max_ms']:.4f} | "
                    f"{r['total_ms']:.1f} |\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
