"""bench.py --gpus N starts N ranks itself when no launcher set WORLD_SIZE (a child
torch.distributed.run, never an exec), and refuses a launcher whose world differs from N.
CPU only: --launch-check runs the rank plumbing (gloo process group, one all-reduce, rank 0's
JSON line) without GPU work."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def _run(args, env):
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=240, cwd=REPO)


def test_gpus_2_launches_two_ranks():
    p = _run(["--gpus", "2", "--backend", "gloo", "--launch-check"], _env())
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["ranks_seen"] == 2
    # rank 0 times the reference's CPU path at N > 1 too (north_star: every N's line)
    cpu = line["cpu_baseline"]
    assert cpu is not None and cpu["value"] > 0 and cpu["cores"] >= 1
    assert cpu["kind"] == "port" and cpu["unit"] == "edge-layers/s"


def test_no_cpu_baseline_flag_drops_it():
    p = _run(["--gpus", "2", "--backend", "gloo", "--launch-check", "--no-cpu-baseline"], _env())
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])
    assert line["n_gpus"] == 2 and line["cpu_baseline"] is None


def test_gpus_1_stays_single_process():
    p = _run(["--gpus", "1", "--launch-check"], _env())
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(p.stdout.strip().splitlines()[-1])["n_gpus"] == 1
    assert "launching" not in p.stderr


def test_world_size_must_match_gpus():
    p = _run(["--gpus", "2", "--launch-check"], _env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"))
    assert p.returncode != 0
    assert "WORLD_SIZE=3" in p.stderr


def test_topk_roofline_prices_the_screen_the_seed_pass_and_the_exact_chains():
    """bench.topk_roofline: bf16 work = the screen of every (user, item) plus, on a large
    catalog, the seed pass's screen of the first 1/16 of the items; the fp32 exact chains (the
    f32 MFMAs of the final ranking, from the PMC record of this topk.hip, profiles/
    pmc_topk.json) priced at the bf16 / fp32 MFMA peak ratio; another user block of the same
    catalog and k (an N > 1 rank's share) scales the record's chains per user; a shape without
    a record counts the screen alone and says so in frac_basis."""
    sys.path.insert(0, REPO)
    import bench
    nu, I, D, t = 32768, 1_000_000, 64, 0.0105
    r = bench.topk_roofline(nu, I, D, 20, t)
    base = 2.0 * nu * I * D
    f32 = r["exact_f32_mfma_per_launch"]
    if r["record_source"]["status"] == "measured":
        assert f32 is not None and 0 <= 2048.0 * f32 < 0.01 * base  # (~29 chains per user)
        assert "exact chains" in r["frac_basis"] and "only" not in r["frac_basis"]
        # a rank's quarter of the users: the same chains per user
        r4 = bench.topk_roofline(nu // 4, I, D, 20, t)
        assert r4["record_source"]["status"].startswith("measured at N = 1")
        assert abs(r4["exact_f32_mfma_per_launch"] - f32 / 4) < 1e-6 * f32
    want = (base * (1 + 1 / 16) + 2048.0 * (f32 or 0.0) * bench.BF16_MFMA_PEAK_TF /
            bench.F32_MFMA_PEAK_TF) / t / 1e12
    assert abs(r["achieved"] - want) < 1e-9 * want
    assert abs(r["frac"] - want / bench.BF16_MFMA_PEAK_TF) < 1e-12
    # a shape without a record (k = 33): the screen and the seed pass alone, flagged
    r2 = bench.topk_roofline(nu, I, D, 33, t)
    assert r2["exact_f32_mfma_per_launch"] is None
    assert r2["record_source"]["status"] != "measured" and "only" in r2["frac_basis"]
    assert abs(r2["achieved"] - base * (1 + 1 / 16) / t / 1e12) < 1e-9 * r2["achieved"]


def test_gpus_2_line_carries_the_exchange_exposure():
    """The N > 1 line's comm block (what the first SCALE run is read by): the all-gathers
    timed alone (allgather_ms_per_layer, algbw / busbw as nccl-tests define them), and the
    compute stream's stall on the gathers inside the overlapped forward, per layer
    (exposed_wait_ms_per_layer; none before layer 0, whose input is replicated) and in all,
    against the L - 1 layers' isolated gathers (hidden_frac)."""
    p = _run(["--gpus", "2", "--backend", "gloo", "--launch-check", "--no-cpu-baseline"], _env())
    assert p.returncode == 0, p.stderr[-2000:]
    comm = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])["comm"]
    assert comm["allgather_ms_per_layer"] > 0
    assert comm["busbw_GBps"] > 0 and abs(comm["busbw_GBps"] - comm["algbw_GBps"] / 2) < 1e-9 * comm["algbw_GBps"]
    per = comm["exposed_wait_ms_per_layer"]
    assert len(per) == 3 and per[0] == 0.0 and all(v >= 0 for v in per)
    assert abs(comm["exposed_wait_ms"] - sum(per)) < 1e-9
    assert abs(comm["isolated_allgather_ms_per_step"] - 2 * comm["allgather_ms_per_layer"]) < 1e-9
    assert comm["hidden_frac"] <= 1.0
