"""Loss functions and training metrics.

Reference: ``src/loss_functions/loss_functions.cu`` (backward-only losses scaled by
``1/global_batch``, ``:141-181``) and ``src/metrics_functions/metrics_functions.cu`` (per-shard
atomics into ``PerfMetrics``, folded on the CPU, ``model.cc:1182-1205``).

MI355X: one fused kernel per step computes the logit gradient AND accumulates every requested
metric into a small device-resident fp64-free fp32 accumulator (``csrc/kernels/loss.hip``);
nothing is copied to the host until ``get_perf_metrics()`` is called, where the accumulators of
all ranks are summed with one all-reduce.  Fix vs the reference: with one
output class the accuracy is binary accuracy (threshold 0.5) instead of a hard-coded 100 %.
"""
from __future__ import annotations

import math

import torch

from .types import LossType, MetricsType

# accumulator slots
M_ALL, M_CORRECT, M_CCE, M_SCCE, M_MSE, M_RMSE, M_MAE, M_LOSS = range(8)
NUM_SLOTS = 8


class PerfMetrics:
    """Host view of the folded metrics (``include/metrics_functions.h:26-40``)."""

    def __init__(self, vals, metrics):
        self.train_all = int(vals[M_ALL])
        self.train_correct = int(vals[M_CORRECT])
        self.cce_loss = float(vals[M_CCE])
        self.sparse_cce_loss = float(vals[M_SCCE])
        self.mse_loss = float(vals[M_MSE])
        self.rmse_loss = float(vals[M_RMSE])
        self.mae_loss = float(vals[M_MAE])
        self.loss_sum = float(vals[M_LOSS])
        self.metrics = metrics

    def get_accuracy(self):
        return 100.0 * self.train_correct / max(1, self.train_all)

    def get_mse(self):
        return self.mse_loss / max(1, self.train_all)

    def get_loss(self):
        return self.loss_sum / max(1, self.train_all)

    def __str__(self):
        n = max(1, self.train_all)
        s = "[Metrics]"
        ms = set(int(m) for m in self.metrics)
        if MetricsType.METRICS_ACCURACY in ms:
            s += f" accuracy: {self.get_accuracy():.2f}% ({self.train_correct} / {self.train_all})"
        if MetricsType.METRICS_CATEGORICAL_CROSSENTROPY in ms:
            s += f" categorical_crossentropy: {self.cce_loss / n:.4f}"
        if MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY in ms:
            s += f" sparse_categorical_crossentropy: {self.sparse_cce_loss / n:.4f}"
        if MetricsType.METRICS_MEAN_SQUARED_ERROR in ms:
            s += f" mean_squared_error: {self.mse_loss / n:.4f}"
        if MetricsType.METRICS_ROOT_MEAN_SQUARED_ERROR in ms:
            s += f" root_mean_squared_error: {self.rmse_loss / n:.4f}"
        if MetricsType.METRICS_MEAN_ABSOLUTE_ERROR in ms:
            s += f" mean_absolute_error: {self.mae_loss / n:.4f}"
        return s


def metrics_mask(metrics):
    ms = set(int(m) for m in (metrics or []))
    mask = 0
    for bit, m in enumerate([MetricsType.METRICS_ACCURACY, MetricsType.METRICS_CATEGORICAL_CROSSENTROPY,
                             MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY,
                             MetricsType.METRICS_MEAN_SQUARED_ERROR,
                             MetricsType.METRICS_ROOT_MEAN_SQUARED_ERROR,
                             MetricsType.METRICS_MEAN_ABSOLUTE_ERROR]):
        if int(m) in ms:
            mask |= 1 << bit
    return mask


LOG_MIN = 1e-7


def loss_and_metrics_torch(loss_type, logits, labels, grad, scale, acc, mask, compute_grad=True, clamp=0.0):
    """fp32 reference implementation (CPU path and test oracle).  clamp in (0, 0.5): predictions
    clamped to [clamp, 1-clamp] before loss and metrics, no gradient through clamped ones (DLRM
    --loss-threshold)."""
    p = logits.float()
    B = p.shape[0]
    C = p.shape[-1] if p.dim() > 1 else 1
    p2 = p.reshape(B, -1)
    keep = None
    if clamp > 0.0:
        pc = p2.clamp(clamp, 1.0 - clamp)
        keep = (pc == p2).to(p2.dtype)
        p2 = pc
    lt = LossType(loss_type)
    if lt == LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY:
        lab = labels.reshape(B).long()
        onehot = torch.zeros_like(p2)
        onehot[torch.arange(B), lab] = 1.0
        y = onehot
    else:
        y = labels.float().reshape(B, -1)
    if compute_grad:
        if lt in (LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, LossType.LOSS_CATEGORICAL_CROSSENTROPY,
                  LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, LossType.LOSS_MEAN_SQUARED_ERROR_SUM_REDUCE):
            g = (p2 - y) * scale
        elif lt == LossType.LOSS_BINARY_CROSSENTROPY:
            # logits are sigmoid probabilities (DLRM top layer); d/dz of BCE(sigmoid(z)) = p - y
            g = (p2 - y) * scale
        else:
            raise ValueError(lt)
        if keep is not None:
            g = g * keep
        grad.reshape(B, -1).copy_(g)
    # metrics
    acc[M_ALL] += B
    if mask & 1:
        if C == 1:
            acc[M_CORRECT] += ((p2[:, 0] >= 0.5).float() == (y[:, 0] >= 0.5).float()).sum()
        else:
            acc[M_CORRECT] += (p2.argmax(1) == y.argmax(1)).sum()
    if mask & 2:
        acc[M_CCE] += (-(y * torch.log(p2.clamp_min(LOG_MIN)))).sum()
    if mask & 4:
        acc[M_SCCE] += (-(torch.log(p2.gather(1, y.argmax(1, keepdim=True)).clamp_min(LOG_MIN)))).sum()
    d = p2 - y
    se = (d * d).sum(1)
    if mask & 8:
        acc[M_MSE] += se.sum()
    if mask & 16:
        acc[M_RMSE] += se.sqrt().sum()
    if mask & 32:
        acc[M_MAE] += d.abs().sum()
    # loss value
    if lt == LossType.LOSS_BINARY_CROSSENTROPY:
        pc = p2.clamp(LOG_MIN, 1 - LOG_MIN)
        acc[M_LOSS] += (-(y * torch.log(pc) + (1 - y) * torch.log(1 - pc))).sum()
    elif lt in (LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, LossType.LOSS_CATEGORICAL_CROSSENTROPY):
        acc[M_LOSS] += (-(y * torch.log(p2.clamp_min(LOG_MIN)))).sum()
    else:
        acc[M_LOSS] += se.sum()


class Loss:
    def __init__(self, loss_type):
        self.loss_type = LossType(loss_type)


class Metrics:
    def __init__(self, loss_type, metrics):
        self.loss_type = LossType(loss_type)
        self.metrics = list(metrics or [])
        self.mask = metrics_mask(self.metrics)
