"""FFConfig: global run configuration and command-line flags.

Same flag spellings and defaults as the reference (``src/runtime/model.cc:1272-1381``,
``include/config.h:65-103``) plus MI355X-specific knobs.  In the SPMD design every rank is
one process bound to one GPU; ``workersPerNode`` is the number of GPUs (ranks) per node.
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch


def _dist_info():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


class FFConfig:
    """Run configuration.  Attribute names follow ``include/config.h:65-103``."""

    def __init__(self, argv=None):
        self.epochs = 1
        self.iterations = 1
        self.batchSize = 64             # GLOBAL batch size (reference semantics)
        self.printFreq = 0
        self.profiling = False
        self.debug = False              # serialising executor + NaN guards
        self.learningRate = 0.01
        self.weightDecay = 0.0001
        self.workSpaceSize = 1 << 30
        self.numNodes = 1
        self.loadersPerNode = 4
        self.workersPerNode = 0
        self.simulator_work_space_size = 2 << 30
        self.search_budget = 0
        self.search_alpha = 1.0
        self.search_overlap_backward_update = False
        self.import_strategy_file = ""
        self.export_strategy_file = ""
        self.dataset_path = ""
        self.syntheticInput = False
        self.seed = 0
        # MI355X knobs
        self.device = "auto"            # auto | cpu | gpu
        self.compute_dtype = "auto"     # auto | fp32 | bf16
        self.use_hip_graphs = False     # capture the steady-state iteration (Legion tracing analogue)
        self.grad_bucket_mb = 32.0      # all-reduce bucket size (xGMI ring: fewer, larger buckets)
        self.overlap_grad_sync = True
        self.zero_stage = 0             # 1: shard optimizer state over each replica set (ZeRO-1)
        self.machine_file = ""          # simulator machine model override (JSON)
        self.cost_db = ""               # measured per-op cost database (JSON)
        self.strategy_file = ""         # alias of --import (fixes reference caveat C12)
        self.watchdog_s = 0.0           # >0: abort a rank whose program makes no progress
        self.watchdog_mode = "exit"     # exit (EXIT_HANG, launcher tears the job down) | raise
        self.metrics_log = ""           # per-step JSONL metrics
        self.log_level = "INFO"
        self.rank, self.world_size = _dist_info()
        self._start = time.perf_counter()
        self._models = []               # FFModels built on this config (begin/end_trace targets)
        self.strategies = {}
        if argv is not None:
            self.parse_args(argv)
        self._finalize()

    # ------------------------------------------------------------------
    def parse_args(self, argv=None):
        """Parse the reference flag set (``model.cc:1313-1381``).  Unknown flags are ignored
        exactly like the reference (apps parse their own on top)."""
        if argv is None:
            argv = sys.argv
        i = 1
        n = len(argv)

        def nxt():
            nonlocal i
            i += 1
            return argv[i]

        while i < n:
            a = argv[i]
            if a in ("-e", "--epochs"):
                self.epochs = int(nxt())
            elif a in ("-i", "--iterations"):
                self.iterations = int(nxt())
            elif a in ("-b", "--batch-size"):
                self.batchSize = int(nxt())
            elif a in ("--lr", "--learning-rate"):
                self.learningRate = float(nxt())
            elif a in ("--wd", "--weight-decay"):
                self.weightDecay = float(nxt())
            elif a in ("-p", "--print-freq"):
                self.printFreq = int(nxt())
            elif a in ("-d", "--dataset"):
                self.dataset_path = nxt()
            elif a in ("--budget", "--search-budget"):
                self.search_budget = int(nxt())
            elif a in ("--alpha", "--search-alpha"):
                self.search_alpha = float(nxt())
            elif a in ("--import", "--import-strategy", "-s", "--strategy"):
                self.import_strategy_file = nxt()
            elif a in ("--export", "--export-strategy"):
                self.export_strategy_file = nxt()
            elif a == "-ll:gpu":
                self.workersPerNode = int(nxt())
            elif a == "--nodes":
                self.numNodes = int(nxt())
            elif a == "-ll:cpu":
                self.loadersPerNode = int(nxt())
            elif a == "--profiling":
                self.profiling = True
            elif a == "--debug":
                self.debug = True
            elif a == "--overlap":
                self.search_overlap_backward_update = True
            elif a == "--device":
                self.device = nxt()
            elif a == "--dtype":
                self.compute_dtype = nxt()
            elif a == "--hip-graphs":
                self.use_hip_graphs = True
            elif a == "--zero":
                self.zero_stage = 1
            elif a == "--zero-stage":
                self.zero_stage = int(nxt())
            elif a == "--bucket-mb":
                self.grad_bucket_mb = float(nxt())
            elif a == "--machine":
                self.machine_file = nxt()
            elif a == "--cost-db":
                self.cost_db = nxt()
            elif a == "--seed":
                self.seed = int(nxt())
            elif a == "--watchdog":
                self.watchdog_s = float(nxt())
            elif a == "--metrics-log":
                self.metrics_log = nxt()
            elif a == "--log-level":
                self.log_level = nxt()
            i += 1
        self._finalize()
        return self

    def _finalize(self):
        self.rank, self.world_size = _dist_info()
        if self.workersPerNode <= 0:
            self.workersPerNode = max(1, self.world_size // max(1, self.numNodes))
        if self.device == "auto":
            self.device = "gpu" if torch.cuda.is_available() else "cpu"
        if self.compute_dtype == "auto":
            self.compute_dtype = "bf16" if self.device == "gpu" else "fp32"

    # ------------------------------------------------------------------
    # python API of the reference (flexflow_cbinding.py:346-377)
    def get_batch_size(self):
        return self.batchSize

    def get_workers_per_node(self):
        return self.workersPerNode

    def get_num_nodes(self):
        return self.numNodes

    def get_epochs(self):
        return self.epochs

    def get_current_time(self):
        """Microseconds, like ``Realm::Clock::current_time_in_microseconds``."""
        if self.device == "gpu":
            torch.cuda.synchronize()
        return (time.perf_counter() - self._start) * 1e6

    def begin_trace(self, trace_id):
        """Legion tracing analogue (``flexflow_cbinding.py`` begin_trace): forwarded to the
        models built on this config, which replay a recorded training step as hipGraph segments
        (FFModel.begin_trace)."""
        for m in self._models:
            m.begin_trace(trace_id)

    def end_trace(self, trace_id):
        for m in self._models:
            m.end_trace(trace_id)

    @property
    def torch_device(self):
        if self.device == "gpu":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    @property
    def num_workers(self):
        return self.world_size

    def to_json(self):
        d = {k: v for k, v in self.__dict__.items() if not k.startswith("_") and k != "strategies"}
        return json.dumps(d, sort_keys=True)
