"""Average every PMC counter per kernel name over the passes of profile_spread.sh."""
import csv
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]
dur = defaultdict(list)
p = os.path.join(d, "trace", "run_kernel_trace.csv")
if os.path.exists(p):
    for r in csv.DictReader(open(p)):
        dur[r["Kernel_Name"][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
ctr = defaultdict(list)
for sub in sorted(os.listdir(d)):
    p = os.path.join(d, sub, "run_counter_collection.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            ctr[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
out = {}
for k, v in dur.items():
    if "lg::" in k:
        out[k] = {"calls": len(v), "avg_us": sum(v) / len(v)}
for (k, c), v in ctr.items():
    if k in out:
        out[k][c] = sum(v) / len(v)
print(json.dumps(out, indent=1))
