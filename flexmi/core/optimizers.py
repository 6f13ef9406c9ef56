"""SGD and Adam (``include/optimizer.h:26-74``, ``src/runtime/optimizer_kernel.cu``).

Reference: one single-point Legion task per parameter gathers every gradient replica to one GPU,
sums them and applies the update (``optimizer_kernel.cu:44-110``).  flexmi: gradients are
reduced by RCCL all-reduce (bucketed, overlapped with backward), then ONE multi-tensor kernel
updates every parameter shard of the rank in a single pass over flat fp32 buffers and
refreshes the bf16 compute copies in the same pass (``csrc/kernels/optim.hip``).
Update rules are bit-for-bit the reference's:

  SGD : g = ∇ + wd·W; V = μV + g; g = nesterov ? g + μV : V (only if μ>0); W -= lr·g
  Adam: β1ᵗ,β2ᵗ updated in ``next()``; α_t = α·sqrt(1-β2ᵗ)/(1-β1ᵗ);
        g = ∇ + wd·W; m = β1 m + (1-β1) g; v = β2 v + (1-β2) g²; W -= α_t·m/(sqrt(v)+ε)
"""
from __future__ import annotations

import math

import torch


class Optimizer:
    def __init__(self, ffmodel=None):
        self.model = ffmodel

    def next(self):
        pass

    def state_names(self):
        return []

    def state_dict(self):
        return {}

    def load_state_dict(self, d):
        pass


class SGDOptimizer(Optimizer):
    def __init__(self, ffmodel=None, lr=0.01, momentum=0.0, nesterov=False, weight_decay=0.0):
        super().__init__(ffmodel)
        self.lr = float(lr)
        self.momentum = float(momentum)
        self.nesterov = bool(nesterov)
        self.weight_decay = float(weight_decay)

    def set_learning_rate(self, learning_rate):
        self.lr = float(learning_rate)
        if self.model is not None and getattr(self.model, "executor", None) is not None:
            self.model.executor.set_lr(self.lr)

    def state_names(self):
        return ["v"] if self.momentum > 0 else []

    @property
    def sparse_capable(self):
        """Embedding rows can be updated in place (no dense grad) iff the update of an
        untouched row is the identity: no weight decay, no momentum."""
        return self.momentum == 0.0 and self.weight_decay == 0.0

    def update_torch(self, w, g, state):
        gt = g + self.weight_decay * w
        if self.momentum > 0:
            v = state["v"]
            v.mul_(self.momentum).add_(gt)
            gt = gt + self.momentum * v if self.nesterov else v
        w.sub_(self.lr * gt)

    def state_dict(self):
        return {"lr": self.lr}

    def load_state_dict(self, d):
        self.lr = d.get("lr", self.lr)


class AdamOptimizer(Optimizer):
    def __init__(self, ffmodel=None, alpha=0.001, beta1=0.9, beta2=0.999, weight_decay=0.0, epsilon=1e-8):
        super().__init__(ffmodel)
        self.alpha = float(alpha)
        self.beta1 = float(beta1)
        self.beta2 = float(beta2)
        self.weight_decay = float(weight_decay)
        self.epsilon = float(epsilon)
        self.beta1_t = 1.0
        self.beta2_t = 1.0
        self.alpha_t = self.alpha

    @property
    def lr(self):
        return self.alpha

    def set_learning_rate(self, learning_rate):
        self.alpha = float(learning_rate)

    sparse_capable = False

    def next(self):
        """``AdamOptimizer::next`` (``src/runtime/optimizer.cc:167-173``)."""
        self.beta1_t *= self.beta1
        self.beta2_t *= self.beta2
        self.alpha_t = self.alpha * math.sqrt(1 - self.beta2_t) / (1 - self.beta1_t)

    def state_names(self):
        return ["m", "v"]

    def update_torch(self, w, g, state):
        gt = g + self.weight_decay * w
        m, v = state["m"], state["v"]
        m.mul_(self.beta1).add_((1 - self.beta1) * gt)
        v.mul_(self.beta2).add_((1 - self.beta2) * gt * gt)
        w.sub_(self.alpha_t * m / (v.sqrt() + self.epsilon))

    def state_dict(self):
        return {"alpha": self.alpha, "beta1_t": self.beta1_t, "beta2_t": self.beta2_t, "alpha_t": self.alpha_t}

    def load_state_dict(self, d):
        for k, v in d.items():
            setattr(self, k, v)
