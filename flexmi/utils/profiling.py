"""Per-op timing behind ``--profiling`` and roctx ranges.

Reference: every task bracketed its kernel with ``cudaEventRecord`` and printed
``"<Op> forward time = ..ms"`` when ``--profiling`` was set (``src/ops/linear.cu:499-531``).
flexmi records HIP events per op (no host sync in the loop; read on demand) and emits roctx
ranges so ``rocprofv3 --marker-trace`` timelines carry op names.
"""
from __future__ import annotations

import contextlib
import json
import time
from collections import defaultdict

import torch


class OpTimer:
    def __init__(self, enabled=False, gpu=False):
        self.enabled = enabled
        self.gpu = gpu
        self.events = defaultdict(list)
        self._host = defaultdict(float)
        self._count = defaultdict(int)

    @contextlib.contextmanager
    def scope(self, name):
        if not self.enabled:
            yield
            return
        if self.gpu:
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            try:
                torch.cuda.nvtx.range_push(name)
            except Exception:
                pass
            s.record()
            yield
            e.record()
            try:
                torch.cuda.nvtx.range_pop()
            except Exception:
                pass
            self.events[name].append((s, e))
        else:
            t0 = time.perf_counter()
            yield
            self._host[name] += (time.perf_counter() - t0) * 1e3
            self._count[name] += 1

    def summary(self):
        """{name: (calls, total_ms, mean_ms)}"""
        out = {}
        if self.gpu:
            torch.cuda.synchronize()
            for k, lst in self.events.items():
                tot = sum(s.elapsed_time(e) for s, e in lst)
                out[k] = (len(lst), tot, tot / max(1, len(lst)))
        for k, v in self._host.items():
            out[k] = (self._count[k], v, v / max(1, self._count[k]))
        return out

    def print_summary(self, file=None):
        for k, (n, tot, mean) in sorted(self.summary().items(), key=lambda kv: -kv[1][1]):
            print(f"{k}: calls={n} total={tot:.3f}ms mean={mean:.4f}ms", file=file)

    def reset(self):
        self.events.clear()
        self._host.clear()
        self._count.clear()

    def to_chrome_trace(self, path):
        """Chrome-trace JSON of the recorded op intervals (relative)."""
        evs = []
        t = 0.0
        for k, (n, tot, mean) in self.summary().items():
            evs.append({"name": k, "ph": "X", "ts": t * 1e3, "dur": tot * 1e3, "pid": 0, "tid": 0})
            t += tot
        with open(path, "w") as f:
            json.dump({"traceEvents": evs}, f)
