"""bench.py driver contract on CPU (gloo): one JSON line from rank 0 with the required keys, for a
single process and for two ranks launched through torch.distributed.run (table-wise + DP plan)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", MASTER_ADDR="127.0.0.1")
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


def test_bench_single_process():
    r = _run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--config", "tiny",
              "--batch-per-gpu", "64"])
    _check(r, 1)


def test_bench_two_ranks():
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
              "--steps", "2", "--warmup", "1", "--config", "tiny", "--batch-per-gpu", "64"])
    _check(r, 2)
    assert "table-wise" in r["config"]["parallelism"]
