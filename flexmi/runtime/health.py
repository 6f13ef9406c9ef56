"""Failure detection, debug mode and fault injection.

The reference had none of this: errors were fatal ``exit(1)`` from ``checkCUDA`` macros
(``include/cuda_helper.h:6-36``) and Legion privileges ordered every access.  flexmi runs
SPMD with explicit streams and RCCL collectives, so it adds:

* **debug mode** (``--debug``): the executor synchronises after every program item and checks
  every op's outputs (forward) and input gradients (backward) for NaN/Inf, raising
  :class:`NumericalError` naming the op and phase; after every update it verifies that all
  replicas of every data-parallel weight group hold the same values (checksum all-reduce),
  raising :class:`ReplicaDivergence` -- catches a lost / corrupted gradient all-reduce.
* **watchdog** (``--watchdog SECONDS``): a heartbeat thread; when one program item (a kernel
  launch, a collective wait) makes no progress for the timeout it dumps all Python stacks and
  either raises :class:`WatchdogTimeout` in the main thread or terminates the rank with
  ``EXIT_HANG`` so the launcher tears the job down.  Recovery = restart from the last
  checkpoint (``flexmi.runtime.checkpoint`` reshard-on-load works for a new world size too).
* **fault injection**: :class:`FaultyComm` wraps a :class:`flexmi.parallel.comm.Comm` and
  delays / drops / corrupts the n-th collective or kills the rank there -- used by the tests to
  prove each failure is detected instead of silently training on garbage or hanging.
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time
from typing import Dict, Optional

import torch

EXIT_HANG = 75


class NumericalError(FloatingPointError):
    pass


class ReplicaDivergence(RuntimeError):
    pass


class WatchdogTimeout(RuntimeError):
    pass


# ---------------------------------------------------------------------- numerics guards
def first_nonfinite(tensors):
    """Index of the first tensor holding NaN/Inf (None if all finite)."""
    for i, t in enumerate(tensors):
        if t is None or not torch.is_tensor(t) or not t.is_floating_point() or t.numel() == 0:
            continue
        if not bool(torch.isfinite(t).all()):
            return i
    return None


def check_finite(where: str, tensors, kind="output"):
    i = first_nonfinite(tensors)
    if i is not None:
        t = tensors[i].float()
        n_nan = int(torch.isnan(t).sum())
        n_inf = int(torch.isinf(t).sum())
        raise NumericalError(f"{where}: {kind} {i} {tuple(t.shape)} has {n_nan} NaN and {n_inf} Inf values")


def replica_checksums(executor):
    """Per replicated sync group: (sum, sum|x|) of the fp32 master buffer."""
    out = []
    for g in executor.groups:
        if g.numel == 0 or not g.replicated:
            continue
        m = g.master.detach().double()
        out.append((g, torch.stack([m.sum(), m.abs().sum()])))
    return out


def check_replicas(executor, rtol=0.0):
    """All holders of every replicated weight group must agree bit-for-bit (every replica
    applies the same all-reduced gradient with the same kernel).  One MAX and one MIN
    all-reduce of a 2-double checksum per group."""
    if executor.world == 1:
        return
    for g, cs in replica_checksums(executor):
        hi, lo = cs.clone(), cs.clone()
        executor.comm.all_reduce_op(hi, g.holders, "max")
        executor.comm.all_reduce_op(lo, g.holders, "min")
        diff = float((hi - lo).abs().max())
        scale = float(hi.abs().max()) + 1e-30
        if diff > rtol * scale:
            names = ",".join(e.param.name or str(e.param.guid) for e in g.entries[:4])
            raise ReplicaDivergence(f"data-parallel replicas of weight group [{names}] diverged: checksum spread "
                                    f"{diff:.3e} (rel {diff / scale:.3e}) on ranks {list(g.holders)}")


# ---------------------------------------------------------------------- watchdog
class Watchdog:
    """Heartbeat watchdog.  ``beat(tag)`` marks progress; if no beat arrives for ``timeout_s``
    while armed, the stacks of all threads are dumped to stderr and ``mode`` decides:
    ``"raise"`` interrupts the main thread (re-raised as WatchdogTimeout by the executor),
    ``"exit"`` ends the process with EXIT_HANG (the launcher then stops the other ranks)."""

    def __init__(self, timeout_s: float, mode: str = "exit", poll_s: Optional[float] = None, stream=None):
        self.timeout_s = float(timeout_s)
        self.mode = mode
        self.poll_s = poll_s or min(1.0, self.timeout_s / 4)
        self.stream = stream or sys.stderr
        self._last = time.monotonic()
        self._tag = ""
        self._armed = False
        self.fired = False
        self.fired_tag = None
        self._stop = threading.Event()
        self._thr = threading.Thread(target=self._loop, name="flexmi-watchdog", daemon=True)
        self._thr.start()

    def beat(self, tag=""):
        self._last = time.monotonic()
        self._tag = tag

    def arm(self):
        self.beat(self._tag)
        self._armed = True

    def disarm(self):
        self._armed = False

    def stop(self):
        self._stop.set()
        self._thr.join(timeout=2)

    def _loop(self):
        while not self._stop.wait(self.poll_s):
            if not self._armed or self.fired:
                continue
            idle = time.monotonic() - self._last
            if idle < self.timeout_s:
                continue
            self.fired = True
            self.fired_tag = self._tag
            rank = os.environ.get("RANK", "0")
            print(f"[flexmi watchdog] rank {rank}: no progress for {idle:.1f}s in '{self._tag}'", file=self.stream,
                  flush=True)
            try:
                faulthandler.dump_traceback(file=self.stream, all_threads=True)
            except Exception:
                pass
            if self.mode == "exit":
                self.stream.flush()
                os._exit(EXIT_HANG)
            # a real SIGINT (not _thread.interrupt_main) so blocking sleeps / syscalls wake up
            import signal
            signal.pthread_kill(threading.main_thread().ident, signal.SIGINT)


# ---------------------------------------------------------------------- fault injection
class FaultyComm:
    """Wraps a Comm; counts collectives (all_to_all + all_reduce) and injects one fault per
    entry of ``faults``: ``{call_index: ("delay", secs) | ("drop",) | ("corrupt",) | ("kill",)}``.
    ``drop`` loses this rank's result of the collective (it runs on a scratch copy, so the rank
    keeps its local gradient while its peers get the sum -- no peer is left waiting), ``corrupt``
    writes NaN into the payload, ``kill`` ends this rank abruptly (exit code 3).  The executor
    hands ``faults`` to the native step runner (``flexmi._rt`` set_faults), so injection runs on
    the production path too."""

    def __init__(self, inner, faults: Dict[int, tuple]):
        self.inner = inner
        self.faults = dict(faults)
        self.n = 0
        self.log = []

    def __getattr__(self, k):
        return getattr(self.inner, k)

    def _fault(self):
        f = self.faults.get(self.n)
        self.n += 1
        if f is not None:
            self.log.append((self.n - 1, f[0]))
        return f

    def all_to_all(self, send, recv_numel, dtype, device):
        f = self._fault()
        if f and f[0] == "delay":
            time.sleep(f[1])
        if f and f[0] == "kill":
            os._exit(3)
        out = self.inner.all_to_all(send, recv_numel, dtype, device)
        if f and f[0] == "drop":
            out = [torch.zeros_like(o) for o in out]
        if f and f[0] == "corrupt":
            for o in out:
                if o.numel():
                    o.view(-1)[0] = float("nan")
                    break
        return out

    def all_reduce_async(self, t, ranks=None):
        f = self._fault()
        if f and f[0] == "delay":
            time.sleep(f[1])
        if f and f[0] == "kill":
            os._exit(3)
        if f and f[0] == "drop":
            return self.inner.all_reduce_async(t.clone(), ranks)
        if f and f[0] == "corrupt" and t.numel():
            t.view(-1)[0] = float("nan")
        return self.inner.all_reduce_async(t, ranks)

    def all_reduce(self, t, ranks=None):
        w = self.all_reduce_async(t, ranks)
        if w is not None:
            w.wait()
        return t
