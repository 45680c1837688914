"""Summarise scripts/gpu_topk_pmc.sh (rocprofv3 kernel trace + PMC passes over the screened
top-K at C5: 32768 users x 1M items, k = 20 (or K), d = 64 and 128) into
profiles/pmc_topk.json, keyed "c5-d<D>/topk" (k = 20) or "c5-d<D>/topk_k<K>", with the hash of csrc/topk.hip (bench.py uses a record only for the
source it was measured on).

The kernel is k_topk_ring<D, NG, WAVES, M, CAP, NBUF, LA, LAG, SEEDP> (csrc/topk.hip K2r): for
k <= 32 a seed pass (SEEDP = true, the first 1/16 of the items), then the main pass. Per call: the
kernels' average durations, SQ_VALU_MFMA_BUSY_CYCLES as a fraction of the SIMD cycles
(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) of the main pass, its instruction mix per wave and per
64-item chunk, the wave-state split (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over
SQ_WAVE_CYCLES) and HBM traffic (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 corrections of
MI355X_MICROARCH.md). The bf16 MFMAs beyond the screen's (waves x chunks x 16 at d = 64) are
the f32 MFMAs of the exact chains (the final ranking and mid-stream escapes).
Usage: python scripts/topk_pmc_summary.py TAG DIR [K]"""
import csv
import hashlib
import json
import os
import re
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
USERS, ITEMS, K = 32768, 1_000_000, 20
PAT = r"k_topk_ring<(\d+), (\d+), (\d+), \d+, \d+, \d+, \d+, \d+, (true|false)(?:, (?:true|false))?>"


def main(tag, d, K=K):
    dur = defaultdict(list)
    seed_dur = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_trace.csv"))):
        m = re.search(PAT, r["Kernel_Name"])
        if m:
            ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            (seed_dur if m.group(4) == "true" else dur)[int(m.group(1))].append(ms)
    ctr = defaultdict(lambda: defaultdict(list))
    shape = {}
    for sub in sorted(os.listdir(d)):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            m = re.search(PAT, r["Kernel_Name"])
            if m and m.group(4) == "false":
                D = int(m.group(1))
                shape[D] = (int(m.group(2)), int(m.group(3)))
                ctr[D][r["Counter_Name"]].append(float(r["Counter_Value"]))
    sha = hashlib.sha256(open(os.path.join(
        REPO, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd",
        "csrc", "topk.hip"), "rb").read()).hexdigest()[:16]
    tp = os.path.join(REPO, "profiles", "pmc_topk.json")
    out = json.load(open(tp)) if os.path.exists(tp) else {}
    for D, c in sorted(ctr.items()):
        avg = {k: sum(v) / len(v) for k, v in c.items()}
        NG, WAVES = shape[D]
        waves = avg["SQ_WAVES"]
        users_per_wave = 16 * NG
        items_per_wave = ITEMS * users_per_wave * waves / USERS / waves  # (the wave's split)
        splits = waves * users_per_wave / USERS
        chunk_items = (8192 if D >= 64 or WAVES >= 8 else 4096) // (2 * D)
        chunks = ITEMS / splits / chunk_items
        bf16_mfma = waves * chunks * (chunk_items // 16) * NG * (D // 32)
        f32_mfma = max(0.0, avg["SQ_INSTS_MFMA"] - bf16_mfma)
        simd_cycles = avg["GRBM_GUI_ACTIVE"] / 8 * 1024
        wc = avg["SQ_WAVE_CYCLES"]
        per = {n: avg[n] / waves / chunks for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU",
                                                   "SQ_INSTS_LDS", "SQ_INSTS_MFMA",
                                                   "SQ_INSTS_BRANCH") if n in avg}
        md = sum(dur[D]) / len(dur[D]) if dur[D] else None
        sd = sum(seed_dur[D]) / len(seed_dur[D]) if seed_dur[D] else None
        e = {"kernel": "lg_score_topk_screened_f32 (k_topk_ring: bound-side lists)",
             "source": tag, "kernel_sha": sha, "users": USERS, "items": ITEMS, "k": K, "dim": D,
             "waves_per_block": WAVES, "groups_per_wave": NG, "splits": splits,
             "avg_ms": (md or 0.0) + (sd or 0.0), "main_pass_avg_ms": md, "seed_pass_avg_ms": sd,
             "mfma_busy_frac": avg["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles,
             "bf16_mfma_per_launch": bf16_mfma, "f32_mfma_per_launch": f32_mfma,
             "exact_group_tile_share": None,
             "insts_per_wave_chunk": per,
             "wave_parked_frac": avg["SQ_WAIT_ANY"] / wc,
             "wave_issue_stall_frac": avg["SQ_WAIT_INST_ANY"] / wc,
             "wave_active_frac": avg["SQ_ACTIVE_INST_ANY"] / wc,
             "lds_bank_conflict_frac": avg.get("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, avg.get("SQ_LDS_IDX_ACTIVE", 1)),
             "clock_ghz_profiled": avg["GRBM_GUI_ACTIVE"] / 8 / (md * 1e6) if md else None,
             "hbm_bytes_per_launch": (2 * avg.get("FETCH_SIZE", 0) + avg.get("WRITE_SIZE", 0)) * 1024,
             "counters_per_launch": avg}
        out[f"c5-d{D}/topk" + ("" if K == 20 else f"_k{K}")] = e
        print(json.dumps({k: v for k, v in e.items() if k != "counters_per_launch"}, indent=1))
    json.dump(out, open(tp, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(int(a) for a in sys.argv[3:4]))
