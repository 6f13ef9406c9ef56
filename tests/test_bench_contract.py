"""bench.py driver contract on CPU (gloo): one JSON line from rank 0 with the required keys, for a
single process and for two ranks launched through torch.distributed.run (table-wise + DP plan)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd, **extra_env):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", MASTER_ADDR="127.0.0.1", **extra_env)
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def _check(r, n):
    assert KEYS <= set(r), KEYS - set(r)
    assert r["n_gpus"] == n and r["steps"] == 2 and r["warmup"] == 1
    assert r["value"] > 0 and r["ms_per_step"] > 0 and r["higher_is_better"] is True
    assert r["scaling"] == "weak" and r["data"] == "synthetic"
    assert r["config"]["global_batch"] == 64 * n
    assert r["config"]["loss"] == r["config"]["loss"]   # not NaN
    # HBM preflight of the headline plan (simulator memory model vs the minimum free memory over
    # ranks; host memory on this CPU rehearsal)
    h = r["config"]["hbm"]
    assert h["need_gb"] >= 0 and h["free_gb"] > 0 and h["need_gb"] <= h["free_gb"]


def _check_three_plans(r, n):
    """The default N>1 record: the SOAP-searched plan is the headline, the hand plan it was seeded
    with is ``config.table``, pure DP is ``config.dp``; both speedups are value ratios."""
    c = r["config"]
    assert c["parallelism"] == f"soap-search{n}"
    s = c["search"]
    assert s["budget"] > 0 and s["iterations"] == s["budget"] and s["seconds"] >= 0 and s["speedup_vs_dp"] > 0
    tb, dp = c["table"], c["dp"]
    assert "emb" in tb["parallelism"] and tb["value"] > 0 and tb["ms_per_step"] > 0
    assert dp["parallelism"] == f"dp{n}" and dp["value"] > 0 and dp["ms_per_step"] > 0
    assert c["soap_speedup_vs_dp"] == round(r["value"] / dp["value"], 3)
    assert c["search_speedup_vs_table"] == round(r["value"] / tb["value"], 3)


def test_bench_single_process():
    r = _run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--config", "tiny",
              "--batch-per-gpu", "64"])
    _check(r, 1)


def test_bench_two_ranks():
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
              "--steps", "2", "--warmup", "1", "--config", "tiny", "--batch-per-gpu", "64"])
    _check(r, 2)
    _check_three_plans(r, 2)


@pytest.mark.multiproc
def test_bench_self_launches_eight_ranks():
    """``bench.py --gpus 8`` with no torchrun environment spawns its own 8 ranks (the driver may
    invoke it exactly so) and still prints ONE JSON line with n_gpus 8."""
    env_keys = ("WORLD_SIZE", "RANK", "LOCAL_RANK")
    saved = {k: os.environ.pop(k) for k in env_keys if k in os.environ}
    try:
        r = _run([sys.executable, "bench.py", "--gpus", "8", "--steps", "2", "--warmup", "1",
                  "--config", "mlperf", "--table-scale", "1e-4", "--batch-per-gpu", "64"])
    finally:
        os.environ.update(saved)
    _check(r, 8)
    assert r["config"]["process_world"] == 8 and r["config"]["backend"] == "gloo"
    _check_three_plans(r, 8)


def test_bench_refuses_world_mismatch():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--config", "tiny", "--batch-per-gpu", "8"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode != 0 and not [l for l in p.stdout.splitlines() if l.startswith("{")]


@pytest.mark.multiproc
@pytest.mark.parametrize("strategy", ["table", "dp", "search"])
def test_bench_eight_ranks_mlperf_plan(strategy):
    """The exact 8-GPU plan the driver's scaling run builds (mlperf widths: d=128, 26 tables,
    bottom 13-512-256-128, top 479-1024-1024-512-256-1; HBM-balanced column/table placement or
    pure DP or the SOAP search) compiled and stepped on 8 gloo ranks with scaled-down tables."""
    extra = ["--search-budget", "200"] if strategy == "search" else []
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
              "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "8",
              "--steps", "2", "--warmup", "1", "--config", "mlperf", "--table-scale", "1e-4",
              "--batch-per-gpu", "64", "--strategy", strategy] + extra)
    _check(r, 8)
    assert r["config"]["embedding_dim"] == 128 and r["config"]["mlp_top"] == [479, 1024, 1024, 512, 256, 1]
    if strategy == "dp":
        assert r["config"]["parallelism"] == "dp8" and "soap_speedup_vs_dp" not in r["config"]
    else:
        assert r["config"]["dp"]["parallelism"] == "dp8" and r["config"]["soap_speedup_vs_dp"] > 0
    if strategy == "search":
        sens = r["config"]["search"]["sensitivity"]
        assert sens["worst_ratio_vs_table"] > 0 and sens["threshold"] == 0.10 and sens["worst_corner"]
        assert r["config"]["parallelism"] == "soap-search8" + ("-robust-table" if sens["fallback_to_table"] else "")


@pytest.mark.multiproc
def test_bench_search_falls_back_to_the_robust_plan():
    """when the searched plan is not robust to the spec-based machine constants (here
    forced: --robust-threshold -1 rejects any pick), the 8-rank MLPerf headline runs the table plan
    the search was seeded with, labelled as such, with the corner table's worst case recorded."""
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
              "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "8",
              "--steps", "2", "--warmup", "1", "--config", "mlperf", "--table-scale", "1e-4",
              "--batch-per-gpu", "64", "--search-budget", "200", "--robust-threshold", "-1", "--no-dp"])
    _check(r, 8)
    c = r["config"]
    assert c["parallelism"] == "soap-search8-robust-table"
    assert c["search"]["sensitivity"]["fallback_to_table"] is True
    # the headline ran the table plan: same plan as the table comparison run, so their step times agree
    assert 0.5 < c["search_speedup_vs_table"] < 2.0


@pytest.mark.multiproc
def test_bench_comparison_failure_keeps_headline():
    """A comparison run that fails on ONE rank of eight (FM_BENCH_FAIL=dp@3: an exception in its
    build phase) becomes ``config.dp.error`` on every rank -- no hang in the next collective -- and
    the already-measured headline (and the table comparison) still come out as one JSON line."""
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
              "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "8",
              "--steps", "2", "--warmup", "1", "--config", "tiny", "--batch-per-gpu", "64",
              "--search-budget", "200"], FM_BENCH_FAIL="dp@3")
    _check(r, 8)
    c = r["config"]
    assert c["parallelism"] == "soap-search8"
    assert "error" in c["dp"] and "soap_speedup_vs_dp" not in c
    assert c["table"]["value"] > 0 and c["table"]["hbm"]["need_gb"] >= 0


def test_bench_wall_budget_skips_comparisons():
    """With no wall budget left after the headline, the comparison runs are skipped with a reason
    instead of being started (two gloo ranks)."""
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
              "--steps", "2", "--warmup", "1", "--config", "tiny", "--batch-per-gpu", "64", "--budget-s", "1"])
    _check(r, 2)
    for name in ("table", "dp"):
        assert "wall budget" in r["config"][name]["skipped"]


def test_bench_init_failure_keeps_headline():
    """a comparison run that fails on one rank AFTER the build agreement (FM_BENCH_FAIL
    dp@1:init -- device allocation / weight init) is agreed on by both ranks: ``config.dp.error``,
    the headline kept, no hang."""
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
              "--steps", "2", "--warmup", "1", "--config", "tiny", "--batch-per-gpu", "64",
              "--search-budget", "200"], FM_BENCH_FAIL="dp@1:init")
    _check(r, 2)
    assert "init" in r["config"]["dp"]["error"]      # rank 0 reports the other rank's init failure
    assert r["config"]["table"]["value"] > 0


def test_bench_step_failure_ends_the_job():
    """A failure inside a comparison run's steps (dp@1:step: the other rank may already wait in the
    step's collectives) ends the whole job with a non-zero exit within seconds instead of hanging."""
    import time
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", MASTER_ADDR="127.0.0.1", FM_BENCH_FAIL="dp@1:step")
    t0 = time.time()
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                        "--steps", "2", "--warmup", "1", "--config", "tiny", "--batch-per-gpu", "64",
                        "--search-budget", "200"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode != 0, p.stdout[-2000:]
    assert "failed inside its steps" in p.stderr
    assert time.time() - t0 < 200
