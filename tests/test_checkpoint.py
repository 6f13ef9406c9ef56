"""Checkpoint / resume with reshard-on-load, multi-rank over gloo.

A run that trains 2 steps under one strategy, checkpoints, and resumes for 2 more steps under a
DIFFERENT strategy / world size must end with exactly the parameters of an uninterrupted
4-step world-1 run (SGD with sparse embedding updates, and Adam with its m/v state and step
counters)."""
import os
import sys
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.multiproc


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(world, strategy, opt):
    from flexmi.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    from flexmi.models.dlrm import DLRMConfig, build_dlrm, dlrm_strategy
    from flexmi.parallel.layout import ParallelConfig
    cfg = FFConfig()
    cfg.device, cfg.compute_dtype, cfg.batchSize = "cpu", "fp32", 16
    if strategy.endswith("_zero"):        # ZeRO-1: optimizer state sharded over the replicas
        cfg.zero_stage, cfg.grad_bucket_mb = 1, 0.002
        strategy = strategy[:-5]
    m = FFModel(cfg)
    d, s, _ = build_dlrm(m, DLRMConfig.preset("tiny"))
    strat = {}
    if world > 1 and strategy == "table":
        strat = dlrm_strategy(m, world)
    elif world > 1 and strategy == "colsplit":
        strat = dlrm_strategy(m, world)
        strat["embedding0"] = ParallelConfig([world, 1], list(range(world)))
        strat["embedding2"] = ParallelConfig([world, 1], list(range(world)))
    m.strategies = strat
    o = SGDOptimizer(m, 0.1) if opt == "sgd" else AdamOptimizer(m, 0.01)
    m.compile(o, LossType.LOSS_BINARY_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
    m.strategies = strat
    return m, d, s


def _steps(m, d, s, first, n):
    from flexmi.models.dlrm import DLRMConfig
    rows = DLRMConfig.preset("tiny").embedding_size
    ex = m._ex()
    for it in range(first, first + n):
        rng = np.random.RandomState(100 + it)
        dd = np.zeros((16, d.dims[1]), np.float32)
        dd[:, :13] = rng.rand(16, 13)
        ex.scatter_from_host(d, dd)
        for t, r in zip(s, rows):
            ex.scatter_from_host(t, rng.randint(0, r, (16, 1)).astype(np.int64))
        ex.scatter_from_host(m.get_label_tensor(), rng.randint(0, 2, (16, 1)).astype(np.float32))
        ex.train_step()


def _job(rank, world, strategy, opt, ckpt, mode, out):
    m, d, s = _model(world, strategy, opt)
    m.init_layers()
    if mode == "full":
        _steps(m, d, s, 0, 4)
    elif mode == "save":
        _steps(m, d, s, 0, 2)
        m.save_checkpoint(ckpt)
    else:
        m.load_checkpoint(ckpt)
        _steps(m, d, s, 2, 2)
    params = [p.get_weights(m) for p in m.parameters]
    if rank == 0 and out:
        np.savez(out, *params)


def _worker(rank, world, port, *args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rc = 0
    try:
        _job(rank, world, *args)
    except BaseException:  # noqa: BLE001 -- reported through the exit code
        import traceback
        traceback.print_exc()
        rc = 1
    finally:
        dist.destroy_process_group()   # ordered teardown: normal interpreter exit afterwards
    sys.exit(rc)


def _launch(world, strategy, opt, ckpt, mode):
    out = tempfile.mktemp(suffix=".npz")
    if world == 1:
        _job(0, 1, strategy, opt, ckpt, mode, out)
    else:
        mp.start_processes(_worker, args=(world, _port(), strategy, opt, ckpt, mode, out), nprocs=world, join=True,
                           start_method="spawn")
    d = np.load(out)
    os.unlink(out)
    return [d[k] for k in sorted(d.files, key=lambda k: int(k.split("_")[1]))]


@pytest.mark.parametrize("opt", ["sgd", "adam"])
@pytest.mark.parametrize("save_w,save_s,load_w,load_s", [(2, "table", 1, "dp"), (1, "dp", 2, "colsplit"),
                                                         (2, "colsplit", 2, "table"), (2, "dp_zero", 1, "dp"),
                                                         (1, "dp", 2, "dp_zero"), (2, "table_zero", 2, "dp_zero")])
def test_resume_under_another_strategy(tmp_path, opt, save_w, save_s, load_w, load_s):
    ref = _launch(1, "dp", opt, None, "full")
    ck = str(tmp_path / "ck")
    _launch(save_w, save_s, opt, ck, "save")
    assert os.path.exists(os.path.join(ck, "manifest.json")) and os.path.exists(os.path.join(ck, "strategy.pb"))
    got = _launch(load_w, load_s, opt, ck, "load")
    assert len(got) == len(ref)
    # reduce-scatter sums in another order than the all-reduce: ZeRO runs agree to fp32 rounding
    tol = dict(rtol=1e-4, atol=1e-5) if "zero" in save_s + load_s else dict(rtol=1e-5, atol=1e-6)
    for a, b in zip(got, ref):
        np.testing.assert_allclose(a, b, **tol)
