"""The example suite (reference ``python/test.sh`` runs ~30 example scripts through
``flexflow_python``): every script under ``examples/python`` runs end-to-end as a subprocess --
through the ``python -m flexmi.run`` launcher -- on a reduced synthetic dataset.  Accuracy
thresholds are relaxed here (few samples, one epoch); ``test_mnist_mlp_reaches_threshold`` keeps
one real 90 % check like the reference's ``ModelAccuracy`` asserts."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples", "python")

KERAS = ["seq_mnist_mlp", "seq_mnist_cnn", "seq_reuters_mlp", "seq_cifar10_cnn", "seq_mnist_mlp_net2net",
         "seq_mnist_cnn_net2net", "seq_mnist_cnn_nested", "callback", "unary", "reshape", "func_mnist_mlp",
         "func_mnist_mlp_concat", "func_mnist_mlp_concat2", "func_mnist_cnn", "func_mnist_cnn_concat",
         "func_cifar10_cnn", "func_cifar10_cnn_nested", "func_cifar10_alexnet", "func_mnist_mlp_net2net",
         "func_cifar10_cnn_net2net", "func_cifar10_cnn_concat", "func_cifar10_cnn_concat_model",
         "func_cifar10_cnn_concat_seq_model"]
NATIVE = ["mnist_mlp", "mnist_mlp_attach", "mnist_cnn", "cifar10_cnn", "cifar10_cnn_attach", "cifar10_cnn_concat",
          "split", "print_layers", "tensor_attach", "print_input"]
SCRIPTS = ([f"keras/{k}.py" for k in KERAS] + ["keras/candle_uno/candle_uno.py"] +
           [f"native/{k}.py" for k in NATIVE] +
           [f"native/{k}.py" for k in ("alexnet", "inception", "resnet")] +
           [f"onnx/{k}.py" for k in ("mnist_mlp", "cifar10_cnn", "alexnet", "resnet")] +
           [f"pytorch/{k}.py" for k in ("mnist_mlp", "cifar10_cnn")])
HEAVY = {"keras/func_cifar10_alexnet.py", "onnx/alexnet.py"}


def run_example(script, tmp_path, args=(), samples=128, min_acc="0", device="cpu", nproc=1):
    env = dict(os.environ, FLEXMI_EXAMPLE_SAMPLES=str(samples), FLEXMI_EXAMPLE_EPOCHS="1",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), HSA_ENABLE_IPC_MODE_LEGACY="0")
    if min_acc is not None:
        env["FLEXMI_EXAMPLE_MIN_ACC"] = min_acc
    cmd = [sys.executable, "-m", "flexmi.run", "-ll:gpu", str(nproc), os.path.join(EX, script),
           "--device", device] + list(args)
    if device == "cpu":
        cmd += ["--dtype", "fp32"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, f"{script} failed:\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    return r.stdout


@pytest.mark.parametrize("script", SCRIPTS)
def test_example_runs(script, tmp_path):
    small = script.startswith("native/") and any(k in script for k in ("alexnet", "inception", "resnet"))
    args = ["-b", "8" if (small or script in HEAVY) else "32"] + (["--small", "--iterations", "1"] if small else [])
    out = run_example(script, tmp_path, args, samples=32 if script in HEAVY else 128)
    assert "Traceback" not in out


def test_mnist_mlp_reaches_threshold(tmp_path):
    out = run_example("native/mnist_mlp_attach.py", tmp_path, ["-b", "64", "-e", "3"], samples=4096, min_acc=None)
    assert "threshold 90.0%" in out


def test_example_two_ranks(tmp_path):
    """The launcher's SPMD path: 2 gloo ranks run the same script (reference -ll:gpu 2)."""
    out = run_example("keras/func_mnist_mlp.py", tmp_path, ["-b", "32"], nproc=2)
    assert out.count("THROUGHPUT") == 2


def test_launcher_flag_filtering():
    from flexmi.run import parse
    p = parse(["-ll:gpu", "4", "-ll:fsize", "2048", "-ll:zsize", "12192", "-ll:py", "1", "x.py", "-e", "5",
               "-lg:prof", "1"])
    assert p["nproc"] == 4 and p["script"] == "x.py"
    assert p["args"] == ["-ll:gpu", "4", "-e", "5"]


@pytest.mark.gpu
@pytest.mark.parametrize("script", ["native/mnist_mlp.py", "native/cifar10_cnn.py", "keras/func_mnist_mlp_concat2.py",
                                    "native/split.py", "onnx/resnet.py"])
def test_example_gpu(script, tmp_path):
    run_example(script, tmp_path, ["-b", "64"], samples=512, device="gpu")


def test_example_two_nodes(tmp_path):
    """Multi-node launch (X9/P12): two launcher processes, one per "node" (--nodes 2 --node-rank
    0/1, --nproc 2 each, rendezvous at --master 127.0.0.1) form ONE 4-rank job running the same
    SPMD plan: every rank trains and the per-rank results agree."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, FLEXMI_EXAMPLE_SAMPLES="128", FLEXMI_EXAMPLE_EPOCHS="1", FLEXMI_EXAMPLE_MIN_ACC="0",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), MASTER_PORT=str(port),
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = []
    for node in range(2):
        cmd = [sys.executable, "-m", "flexmi.run", "--nproc", "2", "--nodes", "2", "--node-rank", str(node),
               "--master", "127.0.0.1", os.path.join(EX, "keras/func_mnist_mlp.py"), "--device", "cpu",
               "--dtype", "fp32", "-b", "32"]
        procs.append(subprocess.Popen(cmd, cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=600)
        assert p.returncode == 0, f"node failed:\n{o[-2000:]}\n{e[-3000:]}"
        outs.append(o)
    assert sum(o.count("THROUGHPUT") for o in outs) == 4
