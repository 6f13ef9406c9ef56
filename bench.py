#!/usr/bin/env python3
"""flexmi headline benchmark: DLRM training throughput (samples/s) on N MI355X GPUs.

Metric/config from BASELINE.json: "samples/sec DLRM (MLPerf-like) at 1/2/4/8 MI355X" on the
DLRM MLPerf-like configuration (13 dense + 26 sparse features, Criteo-Terabyte table sizes with
max-ind-range 40M = 187.8 M rows x 128 fp32 = 96 GB of tables, dot interaction, bottom MLP
13-512-256-128, top MLP 479-1024-1024-512-256-1, BCE loss, SGD), synthetic data of that shape and
random-init weights (no dataset/network).  Weak scaling: per-GPU batch fixed (default 8192, i.e.
the MLPerf global batch 65536 at 8 GPUs); the four ~40 M-row tables are split on the parameter
(column) dimension over all GPUs, the others placed whole on one GPU (table-wise model
parallelism, HBM-balanced: dlrm_strategy), and the MLPs are data parallel (RCCL all-to-all +
bucketed all-reduce).

    python bench.py --gpus N --steps K --warmup W          (N>1 under torch.distributed.run)

Precision: the headline ``value`` is the REFERENCE precision, fp32 end to end (the reference is
fp32 everywhere: cublasSgemm / cuDNN FLOAT) -- fp32 activations, fp32 weights, fp32
tables.  The big Linear GEMMs run the exact three-way split on the bf16 matrix cores (every fp32
operand split into three bf16 planes, the six products that matter, each exact in fp32, fp32
accumulation: csrc/kernels/gemm_x3.hip), the small ones the f32-input MFMA
(v_mfma_f32_16x16x4_f32); both are tested against float64 at the native fp32 kernel's accuracy
and the record names the engine in ``config.fp32_gemm``.  The bf16 fast mode (bf16 activations /
MFMA operands, fp32 master weights and accumulation) is measured afterwards in the same process
and reported as a secondary field ``config.bf16`` (``--dtype bf16`` makes it the headline,
``--no-secondary`` skips it).

Plans (N > 1): the headline is the SOAP-SEARCHED plan (``--strategy search``, the default): rank 0
runs the MCMC search over the MI355X execution simulator (budget ``--search-budget``, seeded with the
hand plan; the reference's FFModel::optimize, src/runtime/model.cc:1093-1144) and every rank trains
with that plan; ``config.search`` carries the simulated speedup, budget and wall seconds.  The hand
plan the search was seeded with (table-wise / column-split embeddings + DP MLPs, dlrm_strategy) is
then timed as ``config.table`` (``config.search_speedup_vs_table``).  Before training, the pick is
re-simulated against the table plan with every xGMI / all-reduce constant of the (spec-based)
machine model at 0.5x and 2x; if it loses more than ``--robust-threshold`` (10 %) in any corner the
headline runs the table plan instead (``config.search.sensitivity``, parallelism
``soap-searchN-robust-table``; profiles/search_sensitivity_mlperf.txt).

SOAP vs DP (N > 1): after the headline plan, the same model / precision / batch is built and timed
under pure data parallelism -- every table replicated on every GPU and trained by touched-row
exchange (each replica coalesces its lookups, one all-gather of (row, gradient) payloads, every
replica applies them in rank order; no table-sized gradient) -- and reported as ``config.dp``
with ``config.soap_speedup_vs_dp`` = value / dp.value (``--no-dp`` skips it).

Native engine (N = 1, fp32): the same model, batch, steps and warm-up trained by the C++ plan compiler and
HIP engine alone (apps/c/dlrm_native_bench.c through libflexmi_native_c, a child process with no
Python), reported as ``config.native_engine`` (``--no-native`` skips it).

Timed region: W untimed steps, then EXACTLY K full training steps (forward, backward, all
collectives, SGD update of every parameter incl. the sparse embedding rows) bracketed by a
barrier + device synchronize on both sides; the max over ranks is reported.  Prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "samples/sec DLRM (MLPerf-like) at 1/2/4/8 MI355X; SOAP speedup vs pure DP"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="mlperf", choices=["mlperf", "run_random", "criteo_kaggle", "summit", "summit_large", "kaggle_day1", "tiny"])
    ap.add_argument("--batch-per-gpu", type=int, default=8192)
    ap.add_argument("--no-graph", action="store_true", help="disable hipGraph capture of the step")
    ap.add_argument("--strategy", default=None, choices=["table", "dp", "search"],
                    help="search (default for N>1): MCMC SOAP search over the MI355X simulator, seeded with "
                         "'table' (the reference's FFModel::optimize, src/runtime/model.cc:1093-1144); table: "
                         "table-wise embedding placement + DP MLPs (the hand plan, dlrm_strategy); dp: pure data "
                         "parallel")
    ap.add_argument("--search-budget", type=int, default=10000)
    ap.add_argument("--robust-threshold", type=float, default=0.10,
                    help="N>1 search: fall back to the table plan when the searched plan simulates more than this "
                         "fraction slower than it on any machine corner (xGMI / all-reduce constants at 0.5x and 2x)")
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--table-scale", type=float, default=1.0, help="debug only: shrink tables (invalid for reporting)")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="headline compute precision (fp32 = the reference's precision)")
    ap.add_argument("--no-secondary", action="store_true", help="skip the secondary run in the other precision")
    ap.add_argument("--no-native", action="store_true",
                    help="N=1: skip the native-engine comparison (config.native_engine: the same model trained by the "
                         "C++ plan compiler + HIP engine alone, apps/c/dlrm_native_bench.c)")
    ap.add_argument("--no-dp", action="store_true",
                    help="N>1: skip the pure data-parallel comparison run (config.dp / config.soap_speedup_vs_dp)")
    ap.add_argument("--no-table", action="store_true",
                    help="N>1 with --strategy search: skip the hand-plan comparison run (config.table)")
    ap.add_argument("--budget-s", type=float, default=1200.0,
                    help="wall budget of the whole command: a comparison run whose estimated time no longer fits "
                         "is skipped (config.<run>.skipped) instead of risking the already-measured headline")
    a = ap.parse_args()
    if a.strategy is None:
        a.strategy = "search" if a.gpus > 1 else "table"
    return a


def launch_ranks(a) -> int:
    """``--gpus N`` without a torchrun environment: spawn the N rank processes ourselves (one per
    GPU, rendezvous on 127.0.0.1), like the reference's single ``-ll:gpu N`` command
    (examples/cpp/DLRM/run_random.sh:9).  This parent never touches the GPU (no torch import at
    all) and never execs: the ranks are children, rank 0 prints the JSON line on the inherited
    stdout, and the parent exits with the launcher's return code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    import torch
    import torch.distributed as dist
    from flexmi.parallel.comm import init_distributed
    comm = init_distributed()
    rank, world = comm.rank, comm.world
    if world != a.gpus:
        if rank == 0:
            print(f"[bench] error: --gpus {a.gpus} but the process group has {world} ranks", file=sys.stderr)
        sys.exit(3)
    if torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    cuda = torch.cuda.is_available()
    t_start = time.time()
    # the headline first: everything after it is a comparison whose failure must not lose it
    head = run_once(a, a.dtype, comm)
    runs = []
    if cuda and not a.no_secondary:
        other = "bf16" if a.dtype == "fp32" else "fp32"
        runs.append((other, other, None))
    if world > 1 and a.strategy == "search" and not a.no_table:
        # the hand-written plan the search was seeded with (table-wise / column embeddings + DP MLPs)
        runs.append(("table", a.dtype, "table"))
    if world > 1 and a.strategy != "dp" and not a.no_dp:
        # the second half of the BASELINE metric: the same model, precision and batch under pure
        # data parallelism (replicated tables trained by touched-row all-gather, DP MLPs)
        runs.append(("dp", a.dtype, "dp"))
    extra = {name: guarded_run(a, comm, name, dt, strat, head, t_start) for name, dt, strat in runs}
    native = None
    if cuda and world == 1 and not a.no_native and a.dtype == "fp32" and a.table_scale == 1.0:
        native = native_run(a, t_start)
    if rank == 0:
        rec = head["rec"]
        for name, r in extra.items():
            if "rec" not in r:                      # skipped or failed: say why, keep the headline
                rec["config"][name] = {k: v for k, v in r.items()}
                continue
            sub = {"value": r["rec"]["value"], "ms_per_step": r["rec"]["ms_per_step"], "loss": r["rec"]["config"]["loss"]}
            if name in ("table", "dp"):
                sub["parallelism"] = r["rec"]["config"]["parallelism"]
            sub["hbm"] = r["rec"]["config"].get("hbm")
            rec["config"][name] = sub
        if native is not None:
            rec["config"]["native_engine"] = native
        if "rec" in extra.get("table", {}):
            rec["config"]["search_speedup_vs_table"] = round(rec["value"] / extra["table"]["rec"]["value"], 3)
        if "rec" in extra.get("dp", {}):
            rec["config"]["soap_speedup_vs_dp"] = round(rec["value"] / extra["dp"]["rec"]["value"], 3)
        elif world == 1:
            rec["config"]["soap_speedup_vs_dp"] = 1.0   # one GPU: the searched plan IS data parallel
        print(f"ELAPSED TIME = {head['el']:.4f}s, THROUGHPUT = {rec['value']:.2f} samples/s", file=sys.stderr)
        print(json.dumps(rec), flush=True)
    if world > 1:
        backend = comm.backend
        # ordered teardown (barrier, native runners, subset and world communicators, reference
        # cycles; flexmi.parallel.comm.shutdown_distributed) -- then a normal interpreter exit
        dist.destroy_process_group()
        if backend == "nccl":
            # the JSON line is out and every communicator is destroyed; what remains is HIP/RCCL
            # runtime finalisation at exit, which is not part of the measurement and must not be
            # able to stall a finished rank of the driver's multi-GPU run
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(0)


class SkipRun(Exception):
    """A comparison run every rank agreed not to start (HBM preflight or wall budget)."""


class StepFailure(Exception):
    """An exception inside a run's training steps (after every agreement point)."""


def _agree(comm, ok: bool) -> bool:
    """True iff ``ok`` on every rank (one tiny all-reduce; ranks that failed still take part, so a
    failure on one rank becomes the same decision everywhere instead of a hang in the next
    collective)."""
    if comm.world == 1:
        return ok
    import torch
    import torch.distributed as dist
    dev = "cuda" if (torch.cuda.is_available() and comm.backend == "nccl") else "cpu"
    t = torch.tensor([0.0 if ok else 1.0], dtype=torch.float32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()) == 0.0


def _min_over_ranks(comm, v: float) -> float:
    if comm.world == 1:
        return v
    import torch
    import torch.distributed as dist
    dev = "cuda" if (torch.cuda.is_available() and comm.backend == "nccl") else "cpu"
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return float(t.item())


def _free_bytes():
    """Free device memory (HBM) on a GPU, available host memory on the CPU rehearsal."""
    import torch
    if torch.cuda.is_available():
        return float(torch.cuda.mem_get_info()[0])
    import psutil
    return float(psutil.virtual_memory().available)


def _hbm_need_bytes(model, strategies, world):
    """Per-device memory of this plan from the simulator's memory model (csrc/sim/simulator.cc
    Simulator::memory: activations + gradients, weights with their optimizer state, tables and
    sparse-DP receive buffers); the max over devices."""
    from flexmi.parallel.search import SimGraph
    g = SimGraph(model, world, max_cands=4, extra=strategies)
    return max(g.memory(g.assign_from(strategies)))


def _fail_injected(name, rank, phase="build"):
    """FM_BENCH_FAIL=<run>[@<rank>][:<phase>] (tests): raise in that phase of that run -- build
    (default), init (device allocation and weight init, after the build agreement) or step (the
    first warm-up step, which runs collectives)."""
    spec = os.environ.get("FM_BENCH_FAIL", "")
    for item in filter(None, spec.split(",")):
        item, _, ph = item.partition(":")
        run, _, r = item.partition("@")
        if run == name and (r == "" or int(r) == rank) and (ph or "build") == phase:
            raise RuntimeError(f"injected failure in the {name} run ({phase}) on rank {rank} (FM_BENCH_FAIL)")


def guarded_run(a, comm, name, dtype, strategy, head, t_start):
    """One comparison run that cannot lose the headline: skipped (with the reason) when the wall
    budget left cannot hold it (estimate: the headline run's wall time x 1.5 + 30 s, rank 0's
    clock) or when its HBM preflight fails.  An exception in the build or init phase becomes
    ``{"error": ...}`` on every rank (both phases end in an all-rank agreement); one inside the steps
    ends the job on every rank (StepFailure: the other ranks may be blocked in a collective)."""
    est = head["wall_s"] * 1.5 + 30.0
    left = a.budget_s - (time.time() - t_start)
    if not _agree(comm, left >= est if comm.rank == 0 else True):
        return {"skipped": f"wall budget: {left:.0f} s left of --budget-s {a.budget_s:.0f}, run estimated at {est:.0f} s"}
    try:
        return run_once(a, dtype, comm, strategy=strategy, name=name)
    except SkipRun as e:
        return {"skipped": str(e)}
    except StepFailure as e:
        # a failure inside the steps, whose collectives the other ranks may already be blocked in: no
        # agreement can reach them, so this rank ends the job (torch.distributed.run then stops every
        # rank) instead of leaving them hung -- non-zero exit, no record
        import traceback
        traceback.print_exc(file=sys.stderr)
        print(f"[bench] rank {comm.rank}: the {name} run failed inside its steps; aborting the job", file=sys.stderr,
              flush=True)
        if comm.world > 1:
            os._exit(17)
        _release_memory()
        return {"error": f"{type(e).__name__}: {e}"[:400]}
    except Exception as e:   # noqa: BLE001 -- reported in the record, the headline survives
        import traceback
        traceback.print_exc(file=sys.stderr)
        _release_memory()
        return {"error": f"{type(e).__name__}: {e}"[:400]}


def native_run(a, t_start, timeout_s=300.0):
    """The headline configuration trained by the native engine alone: apps/c/dlrm_native_bench.c (the C
    API's plan compiler + HIP engine, no Python in that process; same model, batch, fp32, steps and
    warm-up; its tables stay zero-initialised) built with gcc and run as a child process after this
    process released its models.  A comparison only: any failure is reported, never raised."""
    import json as _json
    import shutil
    import subprocess
    import tempfile
    root = os.path.dirname(os.path.abspath(__file__))
    lib_dir = os.path.join(root, "flexmi")
    src = os.path.join(root, "apps", "c", "dlrm_native_bench.c")
    if not os.path.exists(os.path.join(lib_dir, "libflexmi_native_c.so")) or not os.path.exists(src):
        return {"skipped": "libflexmi_native_c.so or apps/c/dlrm_native_bench.c missing"}
    if shutil.which("gcc") is None:
        return {"skipped": "no gcc to build apps/c/dlrm_native_bench.c"}
    left = a.budget_s - (time.time() - t_start)
    if left < timeout_s + 30:
        return {"skipped": f"wall budget: {left:.0f} s left of --budget-s {a.budget_s:.0f}"}
    _release_memory()
    tmp = tempfile.mkdtemp(prefix="flexmi_native_")
    try:
        exe = os.path.join(tmp, "dlrm_native_bench")
        subprocess.run(["gcc", "-O2", src, "-I" + os.path.join(root, "csrc", "capi"), "-L" + lib_dir,
                        "-Wl,-rpath," + lib_dir, "-lflexmi_native_c", "-o", exe], check=True, capture_output=True,
                       timeout=120)
        r = subprocess.run([exe, "hip", str(a.steps), str(a.warmup), str(a.batch_per_gpu)], capture_output=True,
                           text=True, timeout=timeout_s)
        if r.returncode != 0:
            return {"error": f"exit {r.returncode}: {r.stderr.strip()[-300:]}"}
        out = _json.loads(r.stdout.strip().splitlines()[-1])
        return {"engine": out["engine"], "value": out["samples_per_s"], "ms_per_step": out["ms_per_step"],
                "loss": out["loss"], "program": "apps/c/dlrm_native_bench.c"}
    except Exception as e:   # noqa: BLE001 -- reported in the record
        return {"error": f"{type(e).__name__}: {e}"[:300]}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def _release_memory():
    import gc
    import torch
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


def run_once(a, dtype, comm, strategy=None, name="head"):
    """Build, warm up and time one DLRM training configuration in compute precision ``dtype``
    under ``strategy`` (default ``--strategy``); frees the model before returning (the tables of
    two configurations never coexist).  The build phase (model, plan, compile, HBM preflight) ends
    in an all-rank agreement: a failure or a failed preflight on any rank stops the run on every
    rank before its first collective."""
    strategy = strategy or a.strategy
    import gc
    import torch
    import torch.distributed as dist
    rank, world = comm.rank, comm.world
    from flexmi.core import FFConfig, FFModel, SGDOptimizer, LossType, MetricsType
    from flexmi.models.dlrm import DLRMConfig, build_dlrm, dlrm_strategy, SyntheticDLRMData

    t_run = time.time()
    err = None
    try:
        _fail_injected(name, rank)
        model, cfg, dcfg, dense_in, sparse, strategies, search = _build(a, dtype, comm, strategy)
        need = _hbm_need_bytes(model, strategies, world)
    except Exception as e:   # noqa: BLE001 -- re-raised below, after every rank has heard of it
        err = e
    if not _agree(comm, err is None):
        if err is not None:
            raise err
        raise RuntimeError(f"the {name} run failed to build on another rank")
    free = _min_over_ranks(comm, _free_bytes())
    hbm = {"need_gb": round(need / 1e9, 3), "free_gb": round(free / 1e9, 3)}
    if need > 0.92 * free and name != "head":
        model = None
        _release_memory()
        raise SkipRun(f"HBM preflight: the plan needs {hbm['need_gb']} GB per device, {hbm['free_gb']} GB free")
    cuda = torch.cuda.is_available()
    sync = torch.cuda.synchronize if cuda else (lambda: None)   # CPU (gloo) rehearsal runs too
    # device allocation and weight init (no collectives: every rank initialises its shards from the
    # seeds) end in a second agreement -- an OOM on one rank stops the run everywhere before the
    # first step's collectives
    t0 = time.time()
    ex = None
    try:
        _fail_injected(name, rank, "init")
        ex = model.init_layers()
        sync()
    except Exception as e:   # noqa: BLE001 -- re-raised below, after every rank has heard of it
        err = e
    if not _agree(comm, err is None):
        ex = model = None
        _release_memory()
        if err is not None:
            raise err
        raise RuntimeError(f"the {name} run failed to initialise on another rank")
    t_init = time.time() - t0
    try:
        return _timed(a, comm, model, cfg, dcfg, dense_in, sparse, strategy, search, ex, t_init, hbm, t_run, name)
    except Exception as e:   # noqa: BLE001
        raise StepFailure(f"{type(e).__name__}: {e}") from e


def _build(a, dtype, comm, strategy):
    """The model, its plan and the compiled graph (no device memory beyond the model objects)."""
    import torch
    import torch.distributed as dist
    rank, world = comm.rank, comm.world
    from flexmi.core import FFConfig, FFModel, SGDOptimizer, LossType, MetricsType
    from flexmi.models.dlrm import DLRMConfig, build_dlrm, dlrm_strategy

    dcfg = DLRMConfig.preset(a.config)
    if a.table_scale != 1.0:
        dcfg.embedding_size = [max(2, int(r * a.table_scale)) for r in dcfg.embedding_size]
    cfg = FFConfig()
    cfg.batchSize = a.batch_per_gpu * world
    cfg.profiling = a.profile
    cfg.compute_dtype = dtype if torch.cuda.is_available() else "fp32"
    model = FFModel(cfg)
    dense_in, sparse, out = build_dlrm(model, dcfg)
    strategies = {}
    search = None
    if world > 1 and strategy in ("table", "search"):
        strategies = dlrm_strategy(model, world)
    if world > 1 and strategy == "search":
        cached = getattr(a, "_search_plan", None)
        if cached is None:
            # rank 0 searches (fixed budget and seed), every rank applies rank 0's plan
            plan = [None, None]
            if rank == 0:
                from flexmi.core import SGDOptimizer as _S
                from flexmi.parallel.search import optimize
                model.optimizer = _S(model, 0.01)
                res = optimize(model, a.search_budget, 1.0, num_devices=world, init=strategies, seed=0, verbose=True)
                summ = {k: round(v, 4) for k, v in res.summary().items()}
                summ["budget"] = a.search_budget
                best = dict(res.best)
                # sensitivity pass: the pick re-simulated against the table plan with every xGMI /
                # all-reduce constant at 0.5x and 2x; a pick that loses > robust_threshold to the
                # table plan in any corner is replaced by the table plan (the constants are spec-based
                # until an 8-GPU node calibrates them)
                from flexmi.parallel.search import sensitivity
                rows, worst = sensitivity(model, best, strategies, world)
                wc = max(rows, key=lambda r: r[3])
                fallback = worst > 1.0 + a.robust_threshold
                summ["sensitivity"] = {"worst_ratio_vs_table": round(worst, 4), "worst_corner": wc[0],
                                       "threshold": a.robust_threshold, "fallback_to_table": fallback}
                print(f"[bench] search sensitivity: worst pick/table {worst:.3f} at {wc[0]}"
                      f"{' -> table plan' if fallback else ''}", file=sys.stderr)
                if fallback:
                    best = dict(strategies)
                plan = [best, summ]
            dist.broadcast_object_list(plan, src=0)
            a._search_plan = cached = (plan[0], plan[1])
        strategies = dict(cached[0])
        search = cached[1]
    model.strategies = strategies
    loss = LossType.LOSS_BINARY_CROSSENTROPY if dcfg.loss == "bce" else LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE
    model.compile(SGDOptimizer(model, 0.01), loss, [MetricsType.METRICS_ACCURACY, MetricsType.METRICS_MEAN_SQUARED_ERROR])
    model.strategies = strategies
    return model, cfg, dcfg, dense_in, sparse, strategies, search


def _timed(a, comm, model, cfg, dcfg, dense_in, sparse, strategy, search, ex, t_init, hbm, t_run, name="head"):
    """Warm-up and the timed K steps of a built model; returns the record and frees the model."""
    import gc
    import torch
    import torch.distributed as dist
    from flexmi.models.dlrm import SyntheticDLRMData
    rank, world = comm.rank, comm.world
    cuda = torch.cuda.is_available()
    sync = torch.cuda.synchronize if cuda else (lambda: None)
    data = SyntheticDLRMData(model, dense_in, sparse, dcfg, num_batches=4, seed=rank)

    use_graph = (not a.no_graph) and torch.cuda.is_available() and not a.profile
    run_step = stage = None

    first = [True]

    def step_eager():
        if first[0]:
            first[0] = False
            _fail_injected(name, rank, "step")
        data.next_batch()
        ex.train_step()

    if use_graph:
        # warm the allocator / lazily created workspaces, then capture: one small graph per pooled
        # batch for input staging + the training step as hipGraph segments split at the RCCL
        # collectives (collectives stay eager between replays when world > 1)
        for _ in range(2):
            step_eager()
        torch.cuda.synchronize()
        gi = [0]
        if world > 1:
            # input staging as its own small graph per pooled batch, replayed before the step (N > 1:
            # one segmented step capture instead of one per pooled batch)
            stage = []
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            for k in range(data.nb):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.stream(s):
                    with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                        data.i = k
                        data.next_batch()
                stage.append(g)
            torch.cuda.current_stream().wait_stream(s)
            run_step = ex.capture_step()

            def step():
                stage[gi[0] % len(stage)].replay()
                run_step()
                gi[0] += 1
        else:
            # one step graph per pooled batch with that batch's input staging captured at its head
            # (one multi-copy launch): no second graph launch and no gap between the two per step
            def stage_fn(k):
                def f():
                    data.i = k
                    data.next_batch()
                return f
            runs = [ex.capture_step(pre=stage_fn(k)) for k in range(data.nb)]

            def step():
                runs[gi[0] % len(runs)]()
                gi[0] += 1
    else:
        step = step_eager

    for _ in range(a.warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    el = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device="cuda" if cuda else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    ms = el * 1e3 / a.steps
    gb = cfg.batchSize
    sps = gb * a.steps / el
    met = model.get_perf_metrics()
    rec = {
        "metric": METRIC,
        "value": round(sps, 1),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": cfg.compute_dtype,
        "data": "synthetic",
        "config": {
            "model": f"DLRM {dcfg.name} ({'MLPerf-like: 13 dense + 26 sparse, Criteo-TB tables (187.8M rows x 128, fp32), dot interaction' if dcfg.name == 'mlperf' else dcfg.name})",
            "global_batch": gb,
            "seq_len": 1,
            "parallelism": (f"dp{world}" if world == 1 or strategy == "dp" else
                            (f"soap-search{world}" + ("-robust-table" if (search or {}).get("sensitivity", {}).get(
                                "fallback_to_table") else "")) if strategy == "search" else
                            f"table+column-emb{world}+dp{world}-mlp"),
            "tables_rows": sum(dcfg.embedding_size),
            "embedding_dim": dcfg.sparse_feature_size,
            "mlp_bot": dcfg.mlp_bot,
            "mlp_top": dcfg.mlp_top,
            "interaction": dcfg.arch_interaction_op,
            "hip_graph": bool(use_graph),
            "init_s": round(t_init, 2),
            "loss": round(met.get_loss(), 5),
            "table_scale": a.table_scale,
            "backend": comm.backend if world > 1 else "none",
            "rccl_world": dist.get_world_size() if (world > 1 and comm.backend == "nccl") else None,
            "process_world": world,
            "hbm": hbm,
        },
    }
    if cuda and cfg.compute_dtype == "fp32":
        # how the fp32 GEMMs run (split mode, gemm_f32.hip): 3 = the exact three-way bf16 split kernel
        # (gemm_x3.hip, six bf16 products exact in fp32, fp32 accumulation) for the big layers, the
        # native v_mfma_f32_16x16x4_f32 kernel for the rest; 4 = as 3 with the scaled fp16 two-plane
        # split (three fp16 products, per-row / per-column power-of-two scales) on the forward and dX
        # GEMMs.  Both are float64-oracle tested at the native kernel's tolerance
        # (tests/test_gpu_fp32_split.py)
        from flexmi.ops import _kernels as _K
        rec["config"]["fp32_gemm"] = {0: "native-f32-mfma", 2: "bf16x3-split-all",
                                      3: "bf16x3-split-big+native-f32-mfma",
                                      4: "f16x2-scaled-split-fwd-dx+bf16x3-split-dw+native-f32-mfma",
                                      5: "f16x2-scaled-split-all"}.get(_K.C().gemm_f32_get_split(), "?")
        # measured per-shape GEMM configurations in use (flexmi/ops/gemm_tune.py; FM_GEMM_TUNE=0: none)
        from flexmi.ops import gemm_tune as _T
        rec["config"]["gemm_tuned_entries"] = len(_T.table())
        # operand staging of full GEMM / conv tiles: LDS-DMA (FM_GEMM_DMA=0: register staging)
        rec["config"]["gemm_staging"] = "lds-dma" if _K.C().gemm_dma_enabled() else "registers"
    if search is not None:
        rec["config"]["search"] = dict(search)
    if rank == 0 and a.profile:
        ex.timer.print_summary(file=sys.stderr)
    out = {"rec": rec, "el": el, "dtype": cfg.compute_dtype, "wall_s": time.time() - t_run}
    # release this configuration's device memory before the next one is built
    ex.release()
    ex = model = data = step = run_step = stage = None
    gc.collect()
    if cuda:
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    main()
