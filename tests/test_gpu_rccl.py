"""RCCL on the GPU box: the native runner's collectives on a real ``nccl`` process group (world 1,
the only size a one-GPU box offers).  Runs in a child process so the communicator never touches
the pytest process; rank counts > 1 are covered on gloo by tests/test_distributed_cpu.py and on
the driver's 8-GPU node by bench.py."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_native_runner_collectives_on_rccl_world1():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "rccl_world1_worker.py"), str(_port())],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=150)
    assert p.returncode == 0 and "rccl world1 ok" in p.stdout, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
