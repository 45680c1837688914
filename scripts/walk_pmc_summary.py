"""Summarise scripts/gpu_walk_pmc.sh (rocprofv3 trace + PMC passes over the fused K3s walk,
k_tile_walk = lg_spread_tile_resource_topk_f64, at C5) into profiles/pmc_walk.json, keyed
"c5-d64/walk/<variant>", with the hash of csrc/spread_tiled.hip.

Per launch (averaged over the launches after the first tile, whose list fill is atypical):
the kernel's duration; wave states (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over
SQ_WAVE_CYCLES); the instruction mix; and the LDS pipe: SQ_LDS_IDX_ACTIVE (all LDS-array
cycles, MI355X_MICROARCH.md) over the CU-cycles of the launch (256 CUs x GRBM_GUI_ACTIVE / 8
XCDs) = the fraction of time the CUs' LDS arrays are busy, SQ_LDS_BANK_CONFLICT over
SQ_LDS_IDX_ACTIVE = the share of those cycles that are bank-conflict cycles, and
SQ_WAIT_INST_LDS over SQ_WAVE_CYCLES = the LDS issue stalls.
Usage: python scripts/walk_pmc_summary.py TAG DIR"""
import csv
import hashlib
import json
import os
import re
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAT = r"k_tile_walk"
CUS = 256


def launches(path, key):
    out = defaultdict(list)  # dispatch id -> values
    for r in csv.DictReader(open(path)):
        if re.search(PAT, r["Kernel_Name"]):
            out[int(r.get(key) or 0)].append(r)
    return out


def main(tag, d):
    sha = hashlib.sha256(open(os.path.join(
        REPO, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd",
        "csrc", "spread_tiled.hip"), "rb").read()).hexdigest()[:16]
    tp = os.path.join(REPO, "profiles", "pmc_walk.json")
    out = json.load(open(tp)) if os.path.exists(tp) else {}
    for v in sorted(os.listdir(d)):
        vd = os.path.join(d, v)
        if not os.path.isdir(vd) or not os.path.exists(os.path.join(vd, "trace")):
            continue
        tr = [r for r in csv.DictReader(open(os.path.join(vd, "trace", "run_kernel_trace.csv")))
              if re.search(PAT, r["Kernel_Name"])]
        ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in tr][1:]
        ctr = defaultdict(lambda: defaultdict(float))  # (pass, dispatch) -> counter -> value
        for p in ("p1", "p2", "p3"):
            f = os.path.join(vd, p, "run_counter_collection.csv")
            if not os.path.exists(f):
                continue
            for r in csv.DictReader(open(f)):
                if re.search(PAT, r["Kernel_Name"]):
                    ctr[(p, int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
        per = defaultdict(list)
        for p in ("p1", "p2", "p3"):
            ids = sorted(i for (q, i) in ctr if q == p)[1:]  # (the first tile's launch dropped)
            for i in ids:
                for n, x in ctr[(p, i)].items():
                    per[(p, n)].append(x)
        avg = {f"{n}@{p}": sum(x) / len(x) for (p, n), x in per.items()}
        g = lambda n, p: avg.get(f"{n}@{p}")  # noqa: E731
        wc = g("SQ_WAVE_CYCLES", "p1")
        cu_cycles = lambda p: CUS * g("GRBM_GUI_ACTIVE", p) / 8  # noqa: E731
        e = {"kernel": "lg_spread_tile_resource_topk_f64 (k_tile_walk)", "source": tag,
             "variant": v, "kernel_sha": sha, "launches": len(ms),
             "avg_ms": sum(ms) / len(ms) if ms else None,
             "wave_parked_frac": g("SQ_WAIT_ANY", "p1") / wc,
             "wave_issue_stall_frac": g("SQ_WAIT_INST_ANY", "p1") / wc,
             "wave_active_frac": g("SQ_ACTIVE_INST_ANY", "p1") / wc,
             "lds_busy_frac": g("SQ_LDS_IDX_ACTIVE", "p2") / cu_cycles("p2"),
             "lds_bank_conflict_share": g("SQ_LDS_BANK_CONFLICT", "p2") / g("SQ_LDS_IDX_ACTIVE", "p2"),
             "lds_issue_stall_frac": g("SQ_WAIT_INST_LDS", "p2") / wc,
             "lds_insts_per_launch": g("SQ_INSTS_LDS", "p2"),
             "lds_array_cycles_per_lds_inst": g("SQ_LDS_IDX_ACTIVE", "p2") / g("SQ_INSTS_LDS", "p2"),
             "valu_insts_per_launch": g("SQ_INSTS_VALU", "p2"),
             "salu_insts_per_launch": g("SQ_INSTS_SALU", "p2"),
             "vmem_rd_insts_per_launch": g("SQ_INSTS_VMEM_RD", "p2"),
             "clock_ghz_profiled": g("GRBM_GUI_ACTIVE", "p1") / 8 / (sum(ms) / len(ms) * 1e6) if ms else None,
             "counters_per_launch": avg}
        out[f"c5-d64/walk/{v}"] = e
        print(json.dumps({k: x for k, x in e.items() if k != "counters_per_launch"}, indent=1))
    json.dump(out, open(tp, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
