"""Multi-rank correctness without GPUs: world_size 2/4 over gloo (SURVEY §7.6 "strategy
equivalence": any SOAP strategy must train exactly like data parallelism / world 1).

Each case builds the same model on every rank with a strategy, trains a few steps on the same
global batches and compares the FULL gathered parameters with a world-1 run."""
import os
import sys
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.multiproc


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _build(case, world):
    from flexmi.core import (ActiMode, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer, PoolType)
    from flexmi.parallel.layout import ParallelConfig
    from flexmi.models.dlrm import DLRMConfig, build_dlrm, dlrm_strategy
    cfg = FFConfig()
    cfg.device = "cpu"
    cfg.compute_dtype = "fp32"
    pipe = "+pipe" in case
    case = case.split("+pipe")[0]
    B = 128 if pipe else 16     # micro-batch pipelining: >= 8 rows per chunk on every rank
    cfg.batchSize = B
    m = FFModel(cfg)
    strat = {}
    inputs = {}
    if case == "mlp_tied":
        # tied weights (shared_op) under data parallelism: the bucketed all-reduce must wait for
        # BOTH uses' gradients
        x = m.create_tensor([B, 12], name="x")
        h = m.dense(x, 12, ActiMode.AC_MODE_RELU, name="fc1")
        h = m.dense(h, 12, ActiMode.AC_MODE_TANH, shared_op=h.owner_op, name="fc1_tied")
        o = m.softmax(m.dense(h, 4, name="fc3"), name="sm")
        loss = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY
        inputs["x"] = (x, (B, 12), "f")
    dp_small = case.endswith("_dpsmall")
    if dp_small:
        # pure DP (replicated tables, dense grads) with tiny buckets: a bucket may only be reduced
        # once the fused embedding group's backward has produced every member's gradient
        case = case[:-8]
        cfg.grad_bucket_mb = 0.002
    zero = case.endswith("_zero")
    if zero:
        # ZeRO-1: sharded optimizer state, reduce-scatter + all-gather instead of all-reduce;
        # tiny buckets so several padded buckets (and a padded tail) exist
        case = case[:-5]
        cfg.zero_stage = 1
        cfg.grad_bucket_mb = 0.002
    if case in ("nmt_reference", "nmt_pipeline"):
        # NMT seq2seq (2 layers, 3-step LSTM chunks) under the reference's chunk placement
        # (embeddings on GPUs 0 / 1, chunks data parallel) and under chunk (pipeline) placement
        from flexmi.models.nmt import NMTConfig, nmt, nmt_strategy
        ncfg = NMTConfig.small()
        cfg.batchSize = B = 4
        ins, out = nmt(m, ncfg)
        loss = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY
        for k, t in ins.items():
            inputs[k] = (t, tuple(t.dims), ("i", ncfg.vocab))
        if world > 1:
            strat = nmt_strategy(m, world, case.split("_")[1])
    if case == "mlp_subset":
        # ops placed on a device subset: fc1 / fc2 on ranks {0, 1} with swapped sample shards, so the
        # fc1 -> fc2 reshard involves only ranks 0 and 1 (its all_to_all runs on a 2-rank
        # communicator; ranks 2, 3 skip it)
        x = m.create_tensor([B, 12], name="x")
        h = m.dense(x, 16, ActiMode.AC_MODE_RELU, name="fc1")
        h = m.dense(h, 8, ActiMode.AC_MODE_TANH, name="fc2")
        o = m.softmax(m.dense(h, 4, name="fc3"), name="sm")
        loss = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY
        inputs["x"] = (x, (B, 12), "f")
        if world > 2:
            strat["fc1"] = ParallelConfig([1, 2], [0, 1])
            strat["fc2"] = ParallelConfig([1, 2], [1, 0])
    if case in ("mlp_dp", "mlp_channel"):
        x = m.create_tensor([B, 12], name="x")
        h = m.dense(x, 16, ActiMode.AC_MODE_RELU, name="fc1")
        h = m.dense(h, 8, ActiMode.AC_MODE_TANH, name="fc2")
        o = m.dense(h, 4, name="fc3")
        o = m.softmax(o, name="sm")
        loss = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY
        inputs["x"] = (x, (B, 12), "f")
        if case == "mlp_channel" and world > 1:
            # fc1: channel (parameter) split over all ranks; fc2: 2-D sample x channel split
            strat["fc1"] = ParallelConfig([world, 1], list(range(world)))
            if world % 2 == 0:
                strat["fc2"] = ParallelConfig([2, world // 2], list(range(world)))
    elif case in ("dlrm_mlperf8", "dlrm_shipped8"):
        # the 8-GPU plans bench.py / the reference use, rehearsed on 8 gloo ranks: the MLPerf table
        # set (rows scaled 1/20000, d=32 so the big tables column-split 8 ways into 4-float rows)
        # under dlrm_strategy(model, 8), and run_random (8 x 1e6 rows scaled to 1000) under the
        # reference's shipped src/runtime/dlrm_strategy_8embs_8gpus.pb
        if case == "dlrm_mlperf8":
            from flexmi.models.dlrm import MLPERF_TABLES
            dcfg = DLRMConfig(32, [max(3, r // 20000) for r in MLPERF_TABLES], [13, 64, 32], [0, 64, 32, 1], 1, -1, -1,
                              0.0, "dot", "", -1, "bce", "mlperf_scaled")
        else:
            dcfg = DLRMConfig.preset("run_random")
            dcfg.embedding_size = [1000] * 8
        d, s, p = build_dlrm(m, dcfg)
        loss = LossType.LOSS_BINARY_CROSSENTROPY if dcfg.loss == "bce" else LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE
        inputs["dense"] = (d, (B, dcfg.mlp_bot[0]), "f")
        for i, (t, r) in enumerate(zip(s, dcfg.embedding_size)):
            inputs[f"sparse{i}"] = (t, (B, 1), ("i", r))
        if world > 1:
            if case == "dlrm_mlperf8":
                strat = dlrm_strategy(m, world)
                assert sum(len(pc.device_ids) == world and pc.dims[0] == world for pc in strat.values()) >= 4
            else:
                from flexmi.parallel.strategy import load_strategies_from_file
                ref = "/root/reference/src/runtime/dlrm_strategy_8embs_8gpus.pb"
                if not os.path.exists(ref):
                    pytest.skip("reference strategy file not available")
                strat = load_strategies_from_file(ref)
    elif case.startswith("dlrm"):
        dcfg = DLRMConfig.preset("tiny")
        dcfg.arch_interaction_op = "dot" if case in ("dlrm_dot", "dlrm_dp", "dlrm_dpmix") else "cat"
        if case == "dlrm_dpmix":
            # one 3-row table: its dense replica all-reduce (48 words) is cheaper than the
            # touched-row all-gather, so it trains densely while the others go sparse
            dcfg.embedding_size = [100, 3, 200, 30]
        d, s, p = build_dlrm(m, dcfg)
        loss = LossType.LOSS_BINARY_CROSSENTROPY
        inputs["dense"] = (d, (B, 13), "f")
        for i, (t, r) in enumerate(zip(s, dcfg.embedding_size)):
            inputs[f"sparse{i}"] = (t, (B, 1), ("i", r))
        if world > 1 and not dp_small and case not in ("dlrm_dp", "dlrm_dpmix"):   # pure data parallelism
            strat = dlrm_strategy(m, world)
            if case == "dlrm_search":
                # strategy chosen by the MCMC search over the MI355X simulator (same seed on
                # every rank => identical strategy); must train exactly like world 1
                # (slow all-reduce in the machine model => replicated weights are expensive, so
                # the walk must leave data parallelism for table/column/channel placements)
                from flexmi.parallel.machine import MachineModel
                from flexmi.parallel.search import optimize
                m.optimizer = SGDOptimizer(m, 0.1)
                mach = MachineModel.mi355x(world, ar_busbw_GBps=1e-4, ar_lat_us=500.0)
                strat = dict(optimize(m, 400, 1.0, num_devices=world, machine=mach, seed=5, verbose=False).best)
                dp = ParallelConfig.data_parallel(2, world)
                assert sum(pc != dp for pc in strat.values()) >= 3, strat
            if case == "dlrm_rowsplit":
                # row split of a table: every rank holds a block of rows (partial outputs summed
                # by the exchange); on 4 ranks a second table is row x sample split (2 x 2)
                strat["embedding2"] = ParallelConfig([1, 1, world], list(range(world)))
                if world == 4:
                    strat["embedding0"] = ParallelConfig([1, 2, 2], [3, 1, 2, 0])
            if case == "dlrm_colsplit":
                # column (parameter-dim) split of one table across all ranks
                strat["embedding1"] = ParallelConfig([world, 1], list(range(world)))
    elif case == "inception8":
        # BASELINE config 3 rehearsed on 8 gloo ranks: InceptionV3 (75x75 images, the smallest the
        # stride-2 stages allow) under a strategy from the MCMC search over the MI355X simulator,
        # seeded with attribute (spatial h) splits of the stem and operator placement of the
        # first inception block's branches on device subsets (reference README.md:52-61,
        # examples/cpp/InceptionV3/inception.cc:26-174)
        from flexmi.models import cnn
        cfg.batchSize = B = 8
        x, o = cnn.inception_v3(m, image=75)
        loss = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY
        inputs["img"] = (x, (B, 3, 75, 75), "f")
        if world > 1:
            from flexmi.core.types import OperatorType
            convs = [op for op in m.layers if op.op_type == OperatorType.OP_CONV2D]
            pools = [op for op in m.layers if op.op_type == OperatorType.OP_POOL2D]
            hand = {}
            for op in convs[:3] + pools[:1]:          # stem: h split 2 x sample split 4
                hand[op.name] = ParallelConfig([1, 2, 1, world // 2], list(range(world)))
            half = world // 2
            blk = convs[5:12]                          # first inception_a block's branch convs
            for i, op in enumerate(blk):
                lo = 0 if i < 3 else half
                hand[op.name] = ParallelConfig([1, 1, 1, half], list(range(lo, lo + half)))
            from flexmi.parallel.search import optimize
            m.optimizer = SGDOptimizer(m, 0.1)
            r = optimize(m, 200, 1.0, num_devices=world, init=hand, seed=3, verbose=False)
            strat = dict(r.best)
            spatial = [k for k, pc in strat.items() if len(pc.dims) == 4 and (pc.dims[0] > 1 or pc.dims[1] > 1)]
            subset = [k for k, pc in strat.items() if len(set(pc.device_ids)) < world]
            assert spatial and subset, (spatial, subset)
    elif case == "cnn_spatial":
        x = m.create_tensor([4, 3, 12, 12], name="img")
        c = m.conv2d(x, 4, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU, name="conv1")
        c = m.pool2d(c, 3, 3, 2, 2, 1, 1, PoolType.POOL_MAX, name="pool1")
        c = m.conv2d(c, 4, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_NONE, name="conv2")
        f = m.flat(c, name="flat")
        o = m.dense(f, 3, name="fc")
        o = m.softmax(o, name="sm")
        loss = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY
        inputs["img"] = (x, (4, 3, 12, 12), "f")
        cfg.batchSize = 4
        if world > 1:
            # attribute (spatial) split: H split across ranks (exact, with halo exchange)
            strat["conv1"] = ParallelConfig([1, world, 1, 1], list(range(world)))
            strat["pool1"] = ParallelConfig([1, world, 1, 1], list(range(world)))
            strat["conv2"] = ParallelConfig([world, 1, 1, 1], list(range(world)))
    m.strategies = strat
    if zero and case == "mlp_dp":
        from flexmi.core import AdamOptimizer
        opt = AdamOptimizer(m, 0.01)
    elif zero:
        opt = SGDOptimizer(m, 0.1, momentum=0.9, weight_decay=0.01)
    else:
        opt = SGDOptimizer(m, 0.1)
    m.compile(opt, loss, [MetricsType.METRICS_ACCURACY])
    m.strategies = strat
    return m, inputs


def _run(case, world, rank, steps, out_path):
    from flexmi.runtime import executor as E
    p2p = case.endswith("+p2p")
    case = case.replace("+p2p", "")
    E.P2P_MODE = "1" if p2p else os.environ.get("FM_P2P", "auto")
    suffix = case.split("+pipe")[1] if "+pipe" in case else ""
    chunks = int(suffix) if suffix else 0
    E.XCHG_CHUNKS = str(chunks) if chunks else os.environ.get("FLEXMI_XCHG_CHUNKS", "auto")
    m, inputs = _build(case, world)
    ex = m.init_layers()
    if chunks and world > 1:
        # the exchange feeding the interaction + top MLP really is split into chunk all-to-alls,
        # forward and backward, and the tail runs chunk by chunk
        assert ex.pipe is not None and ex.pipe["K"] == chunks and ex.pipe["kb"] is not None, ex.pipe
        names = [it.name for it in ex.prog_fwd + ex.prog_bwd]
        for c in range(chunks):
            assert f"reshard.fwd.c{c}.a2a" in names and f"reshard.bwd.c{c}.a2a" in names, names
            assert any(n.endswith(f".c{c}.fwd") for n in names) and any(n.endswith(f".c{c}.bwd_dx") for n in names)
    case = case.split("+pipe")[0]
    for op in m.layers:  # the strategy must really be applied (no silent DP fallback)
        if op.name in m.strategies:
            assert ex.pcs[op.guid] == m.strategies[op.name], (op.name, ex.pcs[op.guid])
    rng = np.random.RandomState(7)
    for it in range(steps):
        for name, (t, shape, kind) in inputs.items():
            if kind == "f":
                a = rng.rand(*shape).astype(np.float32)
            else:
                a = rng.randint(0, kind[1], shape).astype(np.int64)
            ex.scatter_from_host(t, a)
        lab = m.get_label_tensor()
        if lab.data_type.name == "DT_INT32":
            la = rng.randint(0, m.layers[-1].outputs[0].dims[-1], lab.dims).astype(np.int32)
        else:
            la = rng.randint(0, 2, lab.dims).astype(np.float32)
        ex.scatter_from_host(lab, la)
        ex.train_step()
    if m.config.zero_stage and world > 1:
        zg = [g for g in ex.groups if g.zero]
        assert zg and all(len(g.buckets) > 1 for g in zg), "ZeRO groups / buckets missing"
        for g in zg:   # optimizer state really is sharded
            assert all(t.numel() * len(g.holders) == g.numel for t in g.state.values())
    if case in ("dlrm_dp", "dlrm_cat_dpsmall", "dlrm_dpmix") and world > 1:
        # sparse data parallelism: replicated tables train by touched-row all-gather (no
        # table-sized gradient, no dense all-reduce) where that moves fewer bytes than the dense
        # replica all-reduce (Embedding.sdp_prefer_sparse); the others stay in a dense group
        from flexmi.core.types import OperatorType
        embs = [e for e in ex.wentries.values() if e.op.op_type == OperatorType.OP_EMBEDDING]
        sp = [e for e in embs if ex._sdp_pays(e.op, e.layout)]
        dn = [e for e in embs if e not in sp]
        assert sp and all(e.sparse and e.group is None and e.grad is None for e in sp)
        assert all(e.op.sparse_dp == tuple(range(world)) for e in sp)
        dense_in_groups = [e for g in ex.groups for e in g.entries if e.op.op_type == OperatorType.OP_EMBEDDING]
        assert sorted(id(e) for e in dense_in_groups) == sorted(id(e) for e in dn)
        assert all(not e.sparse and e.op.sparse_dp is None for e in dn)
        if case == "dlrm_dpmix":
            assert [e.shape[0] for e in dn] == [3], [e.shape for e in dn]
        rep = ex.memory_report()
        assert rep["sparse_tables"] == sum(e.numel * 4 for e in sp) and rep["sparse_dp_payload"] > 0, rep
    params = [p.get_weights(m) for p in m.parameters]
    loss = m.get_perf_metrics().get_loss()
    nr = ex.native_runner()
    native_colls = nr.rt.collectives if nr is not None else -1
    if case == "mlp_subset" and world > 2:
        from flexmi.runtime.executor import FusedExchange
        subs = [x for x in nr.keep if isinstance(x, FusedExchange) and x.participants == [0, 1]]
        # a subset exchange runs on its own communicator or point-to-point on the world one
        assert subs and all((x.pg is not None) or x.p2p for x in subs), "subset exchange over the whole world"
        assert all(x.active == (rank in (0, 1)) for x in subs)
    if world > 1 and (p2p or (case == "cnn_spatial" and world >= 4)):
        # sparse exchanges (halos, chunk hand-offs) go point-to-point: grouped send/recv with
        # the real peers only, through the native runner
        from flexmi.runtime.executor import FusedExchange
        xs = [x for x in nr.keep if isinstance(x, FusedExchange)]
        assert any(x.p2p for x in xs), "no point-to-point exchange planned"
        assert any(k == "p2p" for pid in range(nr.rt.num_programs()) for k, _ in nr.rt.describe(pid))
    if rank == 0:
        np.savez(out_path, loss=loss, native_colls=native_colls, *params)


def _worker(rank, world, port, case, steps, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rc = 0
    try:
        _run(case, world, rank, steps, out_path)
    except BaseException:  # noqa: BLE001 -- reported through the exit code
        import traceback
        traceback.print_exc()
        rc = 1
    finally:
        # ordered teardown (flexmi.parallel.comm.shutdown_distributed): every backend thread is
        # joined before the interpreter finalises, so the rank exits normally
        dist.destroy_process_group()
    sys.exit(rc)


def _launch(case, world, steps=3):
    out = tempfile.mktemp(suffix=".npz")
    if world == 1:
        _run(case, 1, 0, steps, out)
    else:
        mp.start_processes(_worker, args=(world, _free_port(), case, steps, out), nprocs=world, join=True,
                           start_method="spawn")
    d = np.load(out)
    os.unlink(out)
    return d


@pytest.mark.parametrize("case,world", [("mlp_dp", 2), ("mlp_tied", 2), ("mlp_channel", 2), ("mlp_channel", 4), ("dlrm_dot", 2),
                                        ("dlrm_cat", 2), ("dlrm_colsplit", 2), ("cnn_spatial", 2),
                                        ("dlrm_search", 2), ("dlrm_search", 4), ("dlrm_rowsplit", 2),
                                        ("dlrm_rowsplit", 4), ("mlp_dp_zero", 2), ("dlrm_dot_zero", 2),
                                        ("mlp_dp_zero", 4), ("dlrm_cat_dpsmall", 2), ("dlrm_mlperf8", 8), ("mlp_subset", 4), ("nmt_reference", 2),
                                        ("nmt_pipeline", 2), ("nmt_pipeline", 4), ("cnn_spatial", 4),
                                        ("cnn_spatial+p2p", 2), ("dlrm_dot+p2p", 2),
                                        ("dlrm_shipped8", 8), ("dlrm_dp", 2), ("dlrm_dp", 4), ("dlrm_dp", 8), ("dlrm_dpmix", 2), ("dlrm_dpmix", 4),
                                        ("inception8", 8), ("dlrm_dot+pipe2", 2), ("dlrm_dot+pipe3", 2),
                                        ("dlrm_cat+pipe2", 4), ("dlrm_mlperf8+pipe2", 8)])
def test_strategy_equivalence(case, world):
    ref = _launch(case.replace("+p2p", "").split("+pipe")[0] + ("+pipe" if "+pipe" in case else ""), 1)
    got = _launch(case, world)
    keys = [k for k in ref.files if k.startswith("arr_")]
    assert len(keys) == len([k for k in got.files if k.startswith("arr_")])
    for k in keys:
        np.testing.assert_allclose(got[k], ref[k], rtol=1e-4, atol=1e-5, err_msg=f"{case} w{world} {k}")
    assert abs(float(got["loss"]) - float(ref["loss"])) < 1e-4
    try:
        import flexmi._rt  # noqa: F401
    except ImportError:
        return
    if os.environ.get("FLEXMI_NATIVE_RUNNER", "1") == "0":
        return
    # the steps ran through the native runner (flexmi._rt): its collectives were issued from C++
    assert int(got["native_colls"]) >= 0, "world>1 training did not go through the native step runner"
    if case != "dlrm_search":   # a searched strategy may need no collective at all
        assert int(got["native_colls"]) > 0
