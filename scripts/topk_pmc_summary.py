"""Summarise scripts/gpu_r04_topk.sh (rocprofv3 kernel trace + PMC passes over the screened
top-K kernel k_score_topk_screen at C5: 32768 users x 1M items, k = 20, d = 64 and 128) into
profiles/pmc_topk.json, keyed "c5-d<D>/topk", with the hash of csrc/topk.hip (bench.py uses a
record only for the source it was measured on).

Per call: the kernel's average duration (main pass + seed pass; the PMC counters are the main
pass's), SQ_VALU_MFMA_BUSY_CYCLES as a fraction of the
SIMD cycles (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), and the share of (16-user group, 16-item
tile) pairs recomputed by the exact fp32 chain: SQ_INSTS_MFMA minus the screen's bf16 MFMAs
(waves x tiles x groups x D / 32, exactly known) = the exact chains' fp32 MFMAs, D / 4 per
recomputed group-tile. Also the wave-state split (SQ_WAIT_ANY / SQ_WAIT_INST_ANY /
SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES) and HBM traffic (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950
corrections of MI355X_MICROARCH.md).
Usage: python scripts/topk_pmc_summary.py TAG [DIR (gpurun_out/r04_topk)]"""
import csv
import hashlib
import json
import os
import re
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
USERS, ITEMS, K = 32768, 1_000_000, 20


def main(tag, d):
    # the main pass (..., true, false>) and, when the catalog is large enough, the seed pass
    # (..., true, true>: the lower-bound class maxima over the first 1/16 of the items) that
    # runs before it in the same lg_score_topk_screened_f32 call
    pat = r"k_score_topk_screen<(\d+), (\d+), (\d+), (\d+), true, (true|false)>"
    dur = defaultdict(list)
    seed_dur = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_trace.csv"))):
        m = re.search(pat, r["Kernel_Name"])
        if m:
            ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            (seed_dur if m.group(5) == "true" else dur)[int(m.group(1))].append(ms)
    ctr = defaultdict(lambda: defaultdict(list))
    for sub in sorted(os.listdir(d)):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            m = re.search(pat, r["Kernel_Name"])
            if m and m.group(5) == "false":
                ctr[int(m.group(1))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    sha = hashlib.sha256(open(os.path.join(
        REPO, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd",
        "csrc", "topk.hip"), "rb").read()).hexdigest()[:16]
    tp = os.path.join(REPO, "profiles", "pmc_topk.json")
    out = json.load(open(tp)) if os.path.exists(tp) else {}
    for D, c in sorted(ctr.items()):
        avg = {k: sum(v) / len(v) for k, v in c.items()}
        waves = avg["SQ_WAVES"]
        tiles_per_wave = ITEMS / 16 / (waves * 32 / USERS)  # items of a wave's split / 16
        groups = 2
        bf16_mfma = waves * tiles_per_wave * groups * (D // 32)
        f32_mfma = max(0.0, avg["SQ_INSTS_MFMA"] - bf16_mfma)
        exact_group_tiles = f32_mfma / (D // 4)
        simd_cycles = avg["GRBM_GUI_ACTIVE"] / 8 * 1024
        wc = avg["SQ_WAVE_CYCLES"]
        e = {"kernel": "lg_score_topk_screened_f32 (k_score_topk_screen)", "source": tag,
             "kernel_sha": sha, "users": USERS, "items": ITEMS, "k": K, "dim": D,
             "avg_ms": (sum(dur[D]) / len(dur[D]) if dur[D] else 0.0) +
                       (sum(seed_dur[D]) / len(seed_dur[D]) if seed_dur[D] else 0.0),
             "main_pass_avg_ms": sum(dur[D]) / len(dur[D]) if dur[D] else None,
             "seed_pass_avg_ms": sum(seed_dur[D]) / len(seed_dur[D]) if seed_dur[D] else None,
             "mfma_busy_frac": avg["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles,
             "exact_group_tile_share": exact_group_tiles / (waves * tiles_per_wave * groups),
             "bf16_mfma_per_launch": bf16_mfma, "f32_mfma_per_launch": f32_mfma,
             "wave_parked_frac": avg["SQ_WAIT_ANY"] / wc,
             "wave_issue_stall_frac": avg["SQ_WAIT_INST_ANY"] / wc,
             "wave_active_frac": avg["SQ_ACTIVE_INST_ANY"] / wc,
             "lds_bank_conflict_frac": avg.get("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, avg.get("SQ_LDS_IDX_ACTIVE", 1)),
             "clock_ghz_profiled": avg["GRBM_GUI_ACTIVE"] / 8 / (sum(dur[D]) / len(dur[D]) * 1e6) if dur[D] else None,
             "hbm_bytes_per_launch": (2 * avg.get("FETCH_SIZE", 0) + avg.get("WRITE_SIZE", 0)) * 1024,
             "counters_per_launch": avg}
        out[f"c5-d{D}/topk"] = e
        print(json.dumps({k: v for k, v in e.items() if k != "counters_per_launch"}, indent=1))
    json.dump(out, open(tp, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r04",
         sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "gpurun_out", "r04_topk"))
