"""Multi-GPU RCCL equivalence of the two N>1 defaults that only gloo has exercised so far (ADVICE
r3): sparse data parallelism for replicated tables (FLEXMI_SPARSE_DP=1 vs the dense replica
all-reduce 0) and the micro-batched embedding exchange (FLEXMI_XCHG_CHUNKS=auto vs 1), 2 ranks on
2 GPUs over RCCL.  Skipped on boxes with fewer than 2 GPUs."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ngpu():
    import torch
    return torch.cuda.device_count()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(tmp_path, strategy, env_extra, tag):
    out = str(tmp_path / f"{tag}.npz")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1", **env_extra)
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                        os.path.join(ROOT, "tests", "rccl_multi_worker.py"), strategy, out],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0 and "rccl multi ok" in p.stdout, (p.stdout[-2000:], p.stderr[-4000:])
    return [v for _, v in sorted(np.load(out).items(), key=lambda kv: int(kv[0].split("_")[1]))], p.stdout


@pytest.mark.skipif(_ngpu() < 2, reason="needs 2 GPUs")
def test_sparse_dp_matches_dense_replica_allreduce_on_rccl(tmp_path):
    a, _ = _launch(tmp_path, "dp", {"FLEXMI_SPARSE_DP": "0"}, "dense")
    b, _ = _launch(tmp_path, "dp", {"FLEXMI_SPARSE_DP": "1"}, "sparse")
    for x, y in zip(a, b):
        np.testing.assert_allclose(y, x, rtol=1e-4, atol=1e-6)


@pytest.mark.skipif(_ngpu() < 2, reason="needs 2 GPUs")
def test_chunked_exchange_matches_whole_batch_on_rccl(tmp_path):
    a, _ = _launch(tmp_path, "table", {"FLEXMI_XCHG_CHUNKS": "1"}, "whole")
    b, out = _launch(tmp_path, "table", {"FLEXMI_XCHG_CHUNKS": "auto"}, "chunked")
    assert "pipe=True" in out, out
    for x, y in zip(a, b):
        np.testing.assert_allclose(y, x, rtol=1e-4, atol=1e-6)
