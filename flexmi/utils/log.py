"""Structured logging and per-step JSONL metrics.

The reference logged through Legion logger categories (``ff``, ``Mapper``, ``DLRM`` ...,
``src/runtime/model.cc:22``) plus ad-hoc printfs and ``[Metrics] accuracy: ...`` lines
(``src/metrics_functions/metrics_functions.cc:46-71``).  flexmi uses one ``logging`` hierarchy
(``flexmi.<category>``) whose records carry the rank, a level from ``--log-level`` /
``FLEXMI_LOG_LEVEL``, and a :class:`MetricsLogger` that appends one JSON object per step
(loss, accuracy, samples/s, step time, comm counters, HBM peak) to ``--metrics-log PATH``
(rank 0 only; ``{rank}`` in the path gives one file per rank).
"""
from __future__ import annotations

import json
import logging
import os
import shutil
import subprocess
import sys
import time

_CONFIGURED = False


def _rank():
    return int(os.environ.get("RANK", "0"))


class _RankFilter(logging.Filter):
    def filter(self, record):
        record.rank = _rank()
        return True


def get_logger(category="ff", level=None):
    """``flexmi.<category>`` logger; first call installs the rank-tagged stderr handler."""
    global _CONFIGURED
    root = logging.getLogger("flexmi")
    if not _CONFIGURED:
        h = logging.StreamHandler(sys.stderr)
        h.addFilter(_RankFilter())
        h.setFormatter(logging.Formatter("[%(asctime)s r%(rank)d %(name)s %(levelname)s] %(message)s", "%H:%M:%S"))
        root.addHandler(h)
        root.propagate = False
        root.setLevel(os.environ.get("FLEXMI_LOG_LEVEL", "WARNING").upper())
        _CONFIGURED = True
    if level is not None:
        root.setLevel(str(level).upper())
    return logging.getLogger(f"flexmi.{category}")


def device_snapshot():
    """One-shot device description for the run log (``amd-smi``/``rocm-smi`` when present)."""
    info = {"time": time.time(), "host": os.uname().nodename}
    try:
        import torch
        if torch.cuda.is_available():
            p = torch.cuda.get_device_properties(torch.cuda.current_device())
            info.update(device=p.name, gcn_arch=getattr(p, "gcnArchName", ""), hbm_bytes=p.total_memory,
                        cus=p.multi_processor_count)
    except Exception:
        pass
    for tool in ("amd-smi", "rocm-smi"):
        exe = shutil.which(tool)
        if exe:
            try:
                args = [exe, "static", "--json"] if tool == "amd-smi" else [exe, "--showproductname", "--json"]
                r = subprocess.run(args, capture_output=True, text=True, timeout=20)
                if r.returncode == 0:
                    info[tool] = r.stdout[:4000]
                    break
            except Exception:
                pass
    return info


class MetricsLogger:
    """Appends one JSON object per call of :meth:`step` to a JSONL file."""

    def __init__(self, path, config=None, rank=None, all_ranks=False):
        self.rank = _rank() if rank is None else rank
        self.enabled = bool(path) and (all_ranks or "{rank}" in str(path) or self.rank == 0)
        self.path = str(path).replace("{rank}", str(self.rank)) if path else ""
        self._f = None
        self._t_last = None
        if self.enabled:
            d = os.path.dirname(self.path)
            if d:
                os.makedirs(d, exist_ok=True)
            self._f = open(self.path, "a")
            head = {"event": "start", "rank": self.rank, "device": device_snapshot()}
            if config is not None:
                head["config"] = json.loads(config.to_json())
            self._write(head)

    def _write(self, obj):
        self._f.write(json.dumps(obj, default=str) + "\n")
        self._f.flush()

    def step(self, step, samples, perf=None, executor=None, **extra):
        if not self.enabled:
            return
        now = time.perf_counter()
        rec = {"event": "step", "step": int(step), "rank": self.rank}
        if self._t_last is not None:
            dt = now - self._t_last
            rec["step_ms"] = dt * 1e3
            rec["samples_per_s"] = samples / dt if dt > 0 else None
        self._t_last = now
        if perf is not None:
            rec["loss"] = perf.get_loss()
            rec["accuracy"] = perf.get_accuracy()
        if executor is not None:
            rec["comm_calls"] = executor.comm.calls
            rec["comm_bytes"] = executor.comm.bytes_sent
            try:
                import torch
                if executor.backend == "hip":
                    rec["hbm_peak_bytes"] = torch.cuda.max_memory_allocated()
            except Exception:
                pass
        rec.update(extra)
        self._write(rec)

    def event(self, name, **kw):
        if self.enabled:
            self._write({"event": name, "rank": self.rank, **kw})

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None
