"""Failure detection: debug-mode NaN/Inf guards, replica-divergence checks,
the progress watchdog, and fault injection into the collectives (delay / drop / corrupt /
kill a rank) -- every injected failure must surface as an exception, never as silent garbage
or a hang."""
import json
import os
import socket
import tempfile
import time

import numpy as np
import pytest
import torch.multiprocessing as mp


def _mlp(debug=True, watchdog=0.0, B=8):
    from flexmi.core import ActiMode, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    cfg = FFConfig()
    cfg.device, cfg.compute_dtype, cfg.batchSize = "cpu", "fp32", B
    cfg.debug = debug
    cfg.watchdog_s, cfg.watchdog_mode = watchdog, "raise"
    m = FFModel(cfg)
    x = m.create_tensor([B, 12], name="x")
    h = m.dense(x, 16, ActiMode.AC_MODE_RELU, name="fc1")
    o = m.dense(h, 4, name="fc2")
    o = m.softmax(o, name="sm")
    m.compile(SGDOptimizer(m, 0.1), LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
    return m, x


def _feed(m, x, it=0):
    rng = np.random.RandomState(it)
    ex = m._ex()
    ex.scatter_from_host(x, rng.rand(*x.dims).astype(np.float32))
    lab = m.get_label_tensor()
    ex.scatter_from_host(lab, rng.randint(0, 4, lab.dims).astype(np.int32))


def test_debug_mode_names_the_op_producing_nan():
    from flexmi.runtime.health import NumericalError
    m, x = _mlp()
    m.init_layers()
    w = m.get_layer_by_name("fc2").weights[0]
    a = w.get_weights(m)
    a[0, 0] = np.inf
    w.set_weights(m, a)
    _feed(m, x)
    with pytest.raises(NumericalError, match="fc2.fwd"):
        m.forward()


def test_debug_mode_clean_run_passes():
    m, x = _mlp()
    m.init_layers()
    for it in range(3):
        _feed(m, x, it)
        m._ex().train_step()


def test_watchdog_interrupts_a_stalled_step():
    from flexmi.runtime.health import WatchdogTimeout
    m, x = _mlp(debug=False, watchdog=0.5)
    ex = m.init_layers()
    assert ex.native_runner() is not None      # heartbeats are the native runner's per-step hooks
    _feed(m, x)
    op = m.get_layer_by_name("fc1")
    orig = op.forward

    def stalled(ctx):
        time.sleep(5.0)
        return orig(ctx)
    op.forward = stalled
    t0 = time.time()
    with pytest.raises(WatchdogTimeout, match="fc1"):
        ex.forward()
    assert time.time() - t0 < 4.5
    op.forward = orig
    ex.watchdog.stop()


# ---------------------------------------------------------------------- multi-rank faults
def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fault_worker(rank, world, port, fault, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import datetime
    import torch.distributed as dist
    # rendezvous through a file store in this run's private directory: no TCP port to race for
    # with the other multi-process tests running in parallel
    store = dist.FileStore(os.path.join(out_dir, "store"), world)
    dist.init_process_group("gloo", store=store, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    res = {"rank": rank, "error": None}
    try:
        from flexmi.runtime.health import FaultyComm
        m, x = _mlp(debug=True, watchdog=20.0)
        if rank == 1:
            # the native runner's collective #0 = step 1's gradient-bucket all-reduce (the runner
            # issues the program's collectives in program order; the metric reduction is not one
            # of them), so exactly one deterministic collective is faulted
            m.comm = FaultyComm(m.comm, {0: fault} if fault[0] != "none" else {})
        m.init_layers()
        nr = m._ex().native_runner()
        res["native"] = nr is not None
        res["steps"] = []
        for it in range(2):
            _feed(m, x, it)
            try:
                m._ex().train_step()
            finally:   # evidence for a failed expectation: collectives issued / faults consumed
                res["steps"].append({"collectives": nr.rt.collectives if nr else None,
                                     "fault_calls": nr.rt.fault_calls if nr else None,
                                     "programs": [nr.rt.describe(p) for p in range(nr.rt.num_programs())] if nr else None})
    except BaseException as e:  # noqa: BLE001 -- report every failure kind to the parent
        res["error"] = type(e).__name__
        res["msg"] = str(e)[:300]
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
        json.dump(res, f)
    # a faulted run's communicators cannot be torn down collectively (a peer may be dead or out
    # of step), so this worker -- and only this one -- leaves without interpreter finalisation
    os._exit(0)


def _run_faulty(fault, world=2, timeout=90):
    out = tempfile.mkdtemp()
    ctx = mp.get_context("spawn")
    port = _port()
    ps = [ctx.Process(target=_fault_worker, args=(r, world, port, fault, out)) for r in range(world)]
    for p in ps:
        p.start()
    deadline = time.time() + timeout
    for p in ps:
        p.join(max(1.0, deadline - time.time()))
    hung = [p.pid for p in ps if p.is_alive()]
    for p in ps:
        if p.is_alive():
            p.kill()
            p.join()
    res = {}
    for r in range(world):
        f = os.path.join(out, f"r{r}.json")
        if os.path.exists(f):
            res[r] = json.load(open(f))
    return res, hung, [p.exitcode for p in ps]


@pytest.mark.multiproc
def test_dropped_allreduce_is_detected_as_replica_divergence():
    res, hung, _ = _run_faulty(("drop",))
    assert not hung
    assert res[0]["error"] == "ReplicaDivergence" and res[1]["error"] == "ReplicaDivergence", res
    # detected in the step whose gradient all-reduce was dropped (the first), not later
    assert len(res[0]["steps"]) == 1 and len(res[1]["steps"]) == 1, res
    assert res[1]["steps"][0]["fault_calls"] >= 1, res
    # the fault was injected by the native step runner (flexmi._rt), the production path
    assert res[0]["native"] and res[1]["native"], res


@pytest.mark.multiproc
def test_corrupted_allreduce_is_detected_as_nonfinite_weights():
    res, hung, _ = _run_faulty(("corrupt",))
    assert not hung
    assert res[0]["error"] == "NumericalError" and res[1]["error"] == "NumericalError", res
    assert len(res[0]["steps"]) == 1 and len(res[1]["steps"]) == 1, res
    assert res[0]["native"] and res[1]["native"], res


@pytest.mark.multiproc
def test_killed_rank_surfaces_as_error_on_survivor():
    res, hung, codes = _run_faulty(("kill",))
    assert not hung, "survivor hung after peer death"
    assert codes[1] == 3 and 1 not in res
    assert res[0]["error"] is not None, res


@pytest.mark.multiproc
def test_no_fault_no_false_alarm():
    """The same 2-rank debug run without a fault trains both steps: replica checksums and
    finiteness checks cover the whole flat weight buffer, alignment gaps included."""
    res, hung, _ = _run_faulty(("none",))
    assert not hung
    assert res[0]["error"] is None and res[1]["error"] is None, res
    assert len(res[0]["steps"]) == 2 and len(res[1]["steps"]) == 2, res


def test_metrics_jsonl_log(tmp_path):
    """--metrics-log: one JSON record per training step with loss / accuracy / step time."""
    from flexmi.core import SingleDataLoader
    m, x = _mlp(debug=False)
    m.config.metrics_log = str(tmp_path / "run.jsonl")
    m.init_layers()
    rng = np.random.RandomState(0)
    n = 32
    xs = rng.rand(n, 12).astype(np.float32)
    ys = rng.randint(0, 4, (n, 1)).astype(np.int32)
    dl = [SingleDataLoader(m, x, xs, n), SingleDataLoader(m, m.get_label_tensor(), ys, n)]
    m.train(dl, epochs=2)
    recs = [json.loads(line) for line in open(m.config.metrics_log)]
    assert recs[0]["event"] == "start" and "config" in recs[0]
    steps = [r for r in recs if r["event"] == "step"]
    assert [r["step"] for r in steps] == list(range(1, 9))
    assert all(np.isfinite(r["loss"]) for r in steps) and "step_ms" in steps[1]
