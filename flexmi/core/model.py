"""FFModel: graph builder + training lifecycle.

Public API follows the reference (C++ ``include/model.h:291-517``, Python
``python/flexflow/core/flexflow_cbinding.py:564-875``): layer builders return output Tensors,
``compile(optimizer, loss_type, metrics)`` picks the parallelization strategy (imported
``.pb``, MCMC search over the MI355X simulator, or data parallel), ``init_layers()`` builds the
per-rank executor, and the training loop is ``forward(); zero_gradients(); backward(); update()``.
Unlike the reference, a strategy found by search is *applied* to the run (caveat C6) and
``--strategy`` is accepted as an alias of ``--import`` (caveat C12).
"""
from __future__ import annotations

import sys
from typing import Dict, List

import numpy as np
import torch

from flexmi.core.config import FFConfig
from flexmi.core.loss_metrics import Loss, Metrics
from flexmi.core.optimizers import AdamOptimizer, Optimizer, SGDOptimizer
from flexmi.core.tensor import Parameter, Tensor
from flexmi.core.types import (ActiMode, AggrMode, DataType, LossType, MetricsType, OperatorType,
                               PoolType)
from flexmi.ops.conv import BatchNorm, Conv2D, Pool2D
from flexmi.ops.elementwise import ElementBinary, ElementUnary
from flexmi.ops.embedding import Embedding
from flexmi.ops.linear import Linear
from flexmi.ops.nn_ops import BatchMatmul, DotInteraction, Dropout, Softmax
from flexmi.ops.tensor_ops import Concat, Flat, Reshape, Reverse, Split, Transpose
from flexmi.parallel.comm import Comm
from flexmi.parallel.layout import ParallelConfig


class DeferredOp:
    """Functional "no-inout" op (``include/model.h:402-436``): built without its input
    (``ff.dense(in_dim, out_dim)``, ``ff.relu()``, ``ff.add()`` ...), connected later with
    ``init_inout(model, input)`` which creates the real op and returns its output tensor.
    After binding, attribute access (``get_weight_tensor`` ...) goes to the real op."""

    def __init__(self, model, builder, num_inputs=1, check=None, desc=""):
        self._model = model
        self._builder = builder
        self._num_inputs = num_inputs
        self._check = check
        self._desc = desc
        self.op = None

    def init_inout(self, model, input):
        assert self.op is None, f"{self._desc}: init_inout called twice"
        ins = list(input) if isinstance(input, (list, tuple)) else [input]
        assert len(ins) == self._num_inputs, f"{self._desc}: {self._num_inputs} input(s) expected, got {len(ins)}"
        if self._check is not None:
            self._check(*ins)
        out = self._builder(*ins)
        self.op = out.owner_op
        return out

    def __call__(self, *inputs):
        return self.init_inout(self._model, list(inputs) if len(inputs) > 1 else inputs[0])

    def __getattr__(self, name):
        op = self.__dict__.get("op")
        if op is None:
            raise AttributeError(f"{self.__dict__.get('_desc', 'op')} is not connected yet (call init_inout): {name}")
        return getattr(op, name)


def _is_tensor(x):
    return isinstance(x, Tensor)


class FFModel:
    def __init__(self, ffconfig: FFConfig = None):
        self.config = ffconfig or FFConfig()
        self.layers = []
        self.input_tensors: List[Tensor] = []
        self.parameters: List[Parameter] = []
        self.optimizer: Optimizer = None
        self.loss_op = None
        self.metrics_op = None
        self.label_tensor: Tensor = None
        self.executor = None
        self._trace = None                 # open trace: {"id", "calls", "defer"}
        self._traces = {}                  # trace id -> {"seq", "replay", "replayable"}
        if hasattr(self.config, "_models"):
            self.config._models.append(self)
        self.strategies: Dict[str, ParallelConfig] = {}
        self._seed = self.config.seed * 1000003 + 12345
        self._tracing_id = 200
        self.comm = Comm()
        self.search_result = None

    def _next_seed(self):
        self._seed = (self._seed * 1103515245 + 12345) & 0x7FFFFFFF
        return self._seed

    # ------------------------------------------------------------------ tensors
    def create_tensor(self, dims, data_type=DataType.DT_FLOAT, create_grad=True, name=None):
        if isinstance(data_type, str):
            # older reference spelling create_tensor(dims, name, data_type) (examples/python/onnx)
            name, data_type = (data_type or None), (create_grad if not isinstance(create_grad, bool)
                                                    else DataType.DT_FLOAT)
            create_grad = True
        t = Tensor(dims, data_type, None, 0, create_grad, self, name)
        self.input_tensors.append(t)
        return t

    def create_constant(self, dims, value, data_type=DataType.DT_FLOAT):
        t = self.create_tensor(dims, data_type, False)
        t.constant_value = value
        return t

    def _add(self, op):
        op.layer_id = len(self.layers)
        self.layers.append(op)
        have = {p.guid for p in self.parameters}
        self.parameters.extend(w for w in op.weights if w.guid not in have)   # shared weights once
        return op

    def add_layer(self, op_type, name):
        return None

    # ------------------------------------------------------------------ builders
    def exp(self, x=None, name=None):
        if x is None:
            return DeferredOp(self, lambda t: self.exp(t, name), 1, desc="exp")
        return self._add(ElementUnary(self, OperatorType.OP_EXP, x, name)).outputs[0]

    def relu(self, x=None, name=None):
        if x is None:
            return DeferredOp(self, lambda t: self.relu(t, name), 1, desc="relu")
        return self._add(ElementUnary(self, OperatorType.OP_RELU, x, name)).outputs[0]

    def sigmoid(self, x=None, name=None):
        if x is None:
            return DeferredOp(self, lambda t: self.sigmoid(t, name), 1, desc="sigmoid")
        return self._add(ElementUnary(self, OperatorType.OP_SIGMOID, x, name)).outputs[0]

    def tanh(self, x=None, name=None):
        if x is None:
            return DeferredOp(self, lambda t: self.tanh(t, name), 1, desc="tanh")
        return self._add(ElementUnary(self, OperatorType.OP_TANH, x, name)).outputs[0]

    def elu(self, x=None, name=None):
        if x is None:
            return DeferredOp(self, lambda t: self.elu(t, name), 1, desc="elu")
        return self._add(ElementUnary(self, OperatorType.OP_ELU, x, name)).outputs[0]

    def add(self, x=None, y=None, name=None):
        if x is None:
            return DeferredOp(self, lambda a, b: self.add(a, b, name), 2, desc="add")
        return self._add(ElementBinary(self, OperatorType.OP_EW_ADD, x, y, name)).outputs[0]

    def subtract(self, x=None, y=None, name=None):
        if x is None:
            return DeferredOp(self, lambda a, b: self.subtract(a, b, name), 2, desc="subtract")
        return self._add(ElementBinary(self, OperatorType.OP_EW_SUB, x, y, name)).outputs[0]

    def multiply(self, x=None, y=None, name=None):
        if x is None:
            return DeferredOp(self, lambda a, b: self.multiply(a, b, name), 2, desc="multiply")
        return self._add(ElementBinary(self, OperatorType.OP_EW_MUL, x, y, name)).outputs[0]

    def divide(self, x=None, y=None, name=None):
        if x is None:
            return DeferredOp(self, lambda a, b: self.divide(a, b, name), 2, desc="divide")
        return self._add(ElementBinary(self, OperatorType.OP_EW_DIV, x, y, name)).outputs[0]

    def conv2d(self, input, out_channels, kernel_h, kernel_w, stride_h, stride_w, padding_h, padding_w,
               activation=ActiMode.AC_MODE_NONE, use_bias=True, shared_op=None, kernel_initializer=None,
               bias_initializer=None, name=None, groups=1):
        if not _is_tensor(input):
            # functional form conv2d(in_channels, out_channels, kh, kw, sh, sw, ph, pw, act, use_bias,
            # kernel_init, bias_init) (include/model.h:411-420); shared_op slot = kernel_init here
            in_c = int(input)
            ki, bi = shared_op, kernel_initializer

            def chk(t):
                assert t.dims[1] == in_c, f"conv2d: input has {t.dims[1]} channels, op built for {in_c}"
            return DeferredOp(self, lambda t: self.conv2d(t, out_channels, kernel_h, kernel_w, stride_h, stride_w,
                                                          padding_h, padding_w, activation, use_bias, None, ki, bi,
                                                          name, groups), 1, chk, "conv2d")
        op = Conv2D(self, input, out_channels, kernel_h, kernel_w, stride_h, stride_w, padding_h, padding_w,
                    activation, use_bias, kernel_initializer, bias_initializer, name, groups)
        self._share(op, shared_op)
        return self._add(op).outputs[0]

    def embedding(self, input, num_entries, out_dim=None, aggr=AggrMode.AGGR_MODE_SUM, shared_op=None,
                  kernel_initializer=None, name=None):
        if not _is_tensor(input):
            # functional form embedding(num_entries, out_dim, aggr, kernel_init) (include/model.h:421-425)
            n_e, d = int(input), int(num_entries)
            ag = out_dim if out_dim is not None else AggrMode.AGGR_MODE_SUM
            ki = aggr if not isinstance(aggr, (int, AggrMode)) else None
            return DeferredOp(self, lambda t: self.embedding(t, n_e, d, ag, None, ki, name), 1, desc="embedding")
        op = Embedding(self, input, num_entries, out_dim, aggr, kernel_initializer, name)
        self._share(op, shared_op)
        return self._add(op).outputs[0]

    def pool2d(self, input, kernel_h, kernel_w, stride_h, stride_w, padding_h, padding_w=None,
               pool_type=PoolType.POOL_MAX, activation=ActiMode.AC_MODE_NONE, name=None):
        if not _is_tensor(input):
            # functional form pool2d(kh, kw, sh, sw, ph, pw, type, act) (include/model.h:426-431)
            args = (input, kernel_h, kernel_w, stride_h, stride_w, padding_h)
            pt = padding_w if padding_w is not None else PoolType.POOL_MAX
            ac = pool_type if pool_type in (ActiMode.AC_MODE_NONE, ActiMode.AC_MODE_RELU,
                                            ActiMode.AC_MODE_SIGMOID, ActiMode.AC_MODE_TANH) else ActiMode.AC_MODE_NONE
            return DeferredOp(self, lambda t: self.pool2d(t, *args, pt, ac, name), 1, desc="pool2d")
        return self._add(Pool2D(self, input, kernel_h, kernel_w, stride_h, stride_w, padding_h, padding_w,
                                pool_type, activation, name)).outputs[0]

    def batch_norm(self, input, relu=True, name=None):
        return self._add(BatchNorm(self, input, relu, name)).outputs[0]

    def batch_matmul(self, A, B, name=None):
        return self._add(BatchMatmul(self, A, B, name)).outputs[0]

    def dense(self, input, out_dim, activation=ActiMode.AC_MODE_NONE, use_bias=True, shared_op=None,
              kernel_initializer=None, bias_initializer=None, name=None):
        if not _is_tensor(input):
            # functional form dense(in_dim, out_dim, act, use_bias, kernel_init, bias_init)
            # (include/model.h:432-436: no shared_op slot -> the 5th/6th args are the initialisers)
            in_dim = int(input)
            ki, bi = shared_op, kernel_initializer

            def chk(t):
                assert t.dims[-1] == in_dim, f"dense: input has {t.dims[-1]} features, op built for {in_dim}"
            return DeferredOp(self, lambda t: self.dense(t, out_dim, activation, use_bias, None, ki, bi, name), 1, chk,
                              "dense")
        op = Linear(self, input, out_dim, activation, use_bias, kernel_initializer, bias_initializer, name)
        self._share(op, shared_op)
        return self._add(op).outputs[0]

    def concat(self, tensors, axis, name=None):
        return self._add(Concat(self, tensors, axis, name)).outputs[0]

    def split(self, input, sizes, axis, name=None):
        return list(self._add(Split(self, input, sizes, axis, name)).outputs)

    def flat(self, input=None, name=None):
        if input is None:
            return DeferredOp(self, lambda t: self.flat(t, name), 1, desc="flat")
        return self._add(Flat(self, input, name)).outputs[0]

    def softmax(self, input, name=None):
        return self._add(Softmax(self, input, name)).outputs[0]

    def reshape(self, input, shape, name=None):
        return self._add(Reshape(self, input, shape, name)).outputs[0]

    def transpose(self, input, perm, name=None):
        return self._add(Transpose(self, input, perm, name)).outputs[0]

    def reverse(self, input, axis, name=None):
        return self._add(Reverse(self, input, axis, name)).outputs[0]

    def dropout(self, input, rate, seed=0, name=None):
        return self._add(Dropout(self, input, rate, seed, name)).outputs[0]

    def lstm(self, input, hidden_size, h0=None, c0=None, name=None):
        """LSTM over [batch, time, features] (NMT, ``nmt/lstm.cu``); returns (y, h_T, c_T)."""
        from flexmi.ops.rnn import LSTM
        op = self._add(LSTM(self, input, hidden_size, h0, c0, name))
        return op.outputs[0], op.outputs[1], op.outputs[2]

    def dot_interaction(self, bottom, embs, self_interaction=False, name=None):
        """DLRM ``dot`` feature interaction (fixes reference caveat C3)."""
        return self._add(DotInteraction(self, bottom, embs, 16, self_interaction, name)).outputs[0]

    def _share(self, op, shared_op):
        """``shared_op`` (``src/runtime/model.cc:157-171``): the new op uses the weights of
        ``shared_op``.  The reference only reused the op NAME (so both ops got the same parallel
        config) and still created separate weights; flexmi ties the weights themselves --
        one set of Parameters, gradients of both ops summed, one optimizer update -- and runs
        the sharing op under the owner's parallel config so the weight shards coincide."""
        if shared_op is None:
            return
        if isinstance(shared_op, DeferredOp):
            shared_op = shared_op.op
        owner = getattr(shared_op, "shared_from", None) or shared_op
        assert type(owner) is type(op), f"shared_op must be a {type(op).__name__}, got {type(owner).__name__}"
        assert len(owner.weights) == len(op.weights) and all(
            a.dims == b.dims for a, b in zip(owner.weights, op.weights)), \
            f"shared_op weight shapes {[w.dims for w in owner.weights]} != {[w.dims for w in op.weights]}"
        op.weights = list(owner.weights)
        op.shared_from = owner

    # ------------------------------------------------------------------ lifecycle
    def set_sgd_optimizer(self, optimizer):
        self.optimizer = optimizer
        optimizer.model = self

    def set_adam_optimizer(self, optimizer):
        self.optimizer = optimizer
        optimizer.model = self

    def compile(self, optimizer=None, loss_type=None, metrics=None, comp_mode=None):
        """``FFModel::compile`` (``src/runtime/model.cc:995-1080``)."""
        if optimizer is not None:
            self.optimizer = optimizer
            optimizer.model = self
        if self.optimizer is None:
            self.optimizer = SGDOptimizer(self, self.config.learningRate)
        self.loss_type = LossType(loss_type) if loss_type is not None else LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE
        self.loss_op = Loss(self.loss_type)
        self.metrics_op = Metrics(self.loss_type, metrics or [])
        # ---- strategy --------------------------------------------------------
        from flexmi.parallel import strategy as S
        cfg = self.config
        path = cfg.import_strategy_file or cfg.strategy_file
        if path:
            self.strategies = S.resolve_reference_names(self, S.load_strategies_from_file(path))
        elif cfg.search_budget > 0:
            from flexmi.parallel.search import optimize
            self.search_result = optimize(self, cfg.search_budget, cfg.search_alpha,
                                          num_devices=max(cfg.world_size, cfg.workersPerNode * cfg.numNodes))
            self.strategies = dict(self.search_result.best)
            if cfg.export_strategy_file and cfg.rank == 0:
                S.save_strategies_to_file(cfg.export_strategy_file, self.strategies)
        # ---- label tensor (model.cc:1051-1076) -------------------------------
        final = self.layers[-1].outputs[0]
        if self.loss_type == LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY:
            self.label_tensor = Tensor((final.dims[0], 1), DataType.DT_INT32, model=self, name="label")
        else:
            self.label_tensor = Tensor(final.dims, DataType.DT_FLOAT, model=self, name="label")
        return self

    def init_layers(self):
        """``FFModel::init_layers``: build the per-rank executor (allocation + weight init)."""
        if self.executor is None:
            from flexmi.runtime.executor import Executor
            self.executor = Executor(self, self.strategies, self.comm, self.optimizer, self.loss_type,
                                     self.metrics_op, self.label_tensor)
            # host arrays mapped / attached before init (inline_map between compile and init)
            for t in list(self.input_tensors) + ([self.label_tensor] if self.label_tensor is not None else []):
                pend = getattr(t, "_pending", None)
                if pend is not None and t.guid in self.executor.home:
                    self.executor.scatter_from_host(t, pend)
                    t._pending = None
        return self.executor

    def _ex(self):
        if self.executor is None:
            self.init_layers()
        return self.executor

    def forward(self):
        if not self._traced("forward"):
            self._ex().forward()

    def backward(self):
        if not self._traced("backward"):
            self._ex().backward()

    def forward_op(self, op):
        """Run one op's forward compute on this rank (``Op::forward``, the C API's op_forward):
        the op's compute items of the compiled forward program; its inputs must be in place."""
        op = getattr(op, "op", None) or op
        ex = self._ex()
        prefix = op.name + "."
        for it in ex.prog_fwd:
            if it.kind == "compute" and (it.name == op.name or it.name.startswith(prefix)):
                it.fn()

    def update(self):
        if not self._traced("update"):
            self._ex().update()

    def zero_gradients(self):
        if not self._traced("zero_gradients"):
            self._ex().zero_gradients()

    # ---- Legion tracing analogue (reference: runtime->begin_trace/end_trace around every
    # iteration from epoch 1, examples/cpp/DLRM/dlrm.cc:178-185, Python trace ids 111/200) --------
    # The first traced iteration of an id runs eagerly and records its call sequence.  When that
    # sequence is one training step (forward, [zero_gradients,] backward, update) on MI355X, later
    # iterations of the id defer their calls and end_trace replays the step as hipGraph segments
    # (captured on the second iteration) -- the replay of a memoised trace.  Any other sequence,
    # or a CPU run, simply executes eagerly.
    def begin_trace(self, trace_id):
        st = self._traces.get(trace_id)
        self._trace = {"id": trace_id, "calls": [], "defer": bool(st and st["replayable"])}

    def end_trace(self, trace_id):
        tr, self._trace = self._trace, None
        if tr is None or tr["id"] != trace_id:
            return
        st = self._traces.get(trace_id)
        if st is None:
            calls = [c for c in tr["calls"] if c != "zero_gradients"]
            ex = self._ex()
            self._traces[trace_id] = {"seq": tr["calls"], "replay": None,
                                      "replayable": ex.backend == "hip" and calls == ["forward", "backward", "update"]}
            return
        if not tr["defer"]:
            return
        if tr["calls"] != st["seq"]:       # another sequence this time: run it eagerly, stop replaying
            st["replayable"] = False
            ex = self._ex()
            for c in tr["calls"]:
                getattr(ex, c)()
            return
        if st["replay"] is None:
            st["replay"] = self._ex().capture_step()
        st["replay"]()

    def _traced(self, name):
        tr = self._trace
        if tr is None:
            return False
        tr["calls"].append(name)
        return tr["defer"]

    def compute_metrics(self):
        self._ex().compute_metrics()

    def reset_metrics(self):
        self._ex().reset_metrics()

    def prefetch(self):
        return None

    def get_perf_metrics(self):
        return self._ex().perf_metrics()

    def train(self, dataloaders, epochs=1, batch_size=None):
        """``flexflow_cbinding.py:789-807``."""
        from flexmi.utils.log import MetricsLogger
        num_samples = dataloaders[0].get_num_samples()
        bs = self.config.get_batch_size()
        ex = self._ex()
        ex.training = True
        mlog = MetricsLogger(getattr(self.config, "metrics_log", ""), self.config)
        step = 0
        for epoch in range(epochs):
            for d in dataloaders:
                d.reset()
            self.reset_metrics()
            for _ in range(int(num_samples // bs)):
                for d in dataloaders:
                    d.next_batch(self)
                if epoch > 0:
                    self.begin_trace(200)      # reference trace id (flexflow_cbinding.py train)
                self.forward()
                self.zero_gradients()
                self.backward()
                self.update()
                if epoch > 0:
                    self.end_trace(200)
                step += 1
                if mlog.enabled:
                    mlog.step(step, bs, self.get_perf_metrics(), ex, epoch=epoch)
            if self.config.rank == 0 and self.config.printFreq:
                print(self.get_perf_metrics(), file=sys.stderr)
        mlog.close()

    def eval(self, dataloaders):
        num_samples = dataloaders[0].get_num_samples()
        bs = self.config.get_batch_size()
        ex = self._ex()
        ex.training = False
        for d in dataloaders:
            d.reset()
        self.reset_metrics()
        for _ in range(int(num_samples // bs)):
            for d in dataloaders:
                d.next_batch(self)
            self.forward()
            self.compute_metrics()
        ex.training = True

    # ------------------------------------------------------------------ introspection
    # ---- checkpoint / resume (reshard-on-load across strategies and world sizes)
    def save_checkpoint(self, path, extra=None):
        from flexmi.runtime.checkpoint import save_checkpoint
        return save_checkpoint(self, path, extra)

    def load_checkpoint(self, path, strict=True):
        from flexmi.runtime.checkpoint import load_checkpoint
        return load_checkpoint(self, path, strict)

    def get_layers(self):
        return {i: l for i, l in enumerate(self.layers)}

    def print_layers(self, id=-1):
        for i, l in enumerate(self.layers):
            if id == -1 or id == i:
                ins = ", ".join(str(list(t.dims)) for t in l.inputs)
                outs = ", ".join(str(list(t.dims)) for t in l.outputs)
                print(f"layer[{i}] {type(l).__name__} name={l.name} inputs=[{ins}] outputs=[{outs}] "
                      f"weights={[list(w.dims) for w in l.weights]}")

    def get_layer_by_id(self, layer_id):
        return self.layers[layer_id]

    def get_layer_by_name(self, layer_name):
        for l in self.layers:
            if l.name == layer_name:
                return l
        raise KeyError(layer_name)

    def get_tensor_by_id(self, id):
        return self.parameters[id]

    def get_parameter_by_id(self, id):
        return self.parameters[id]

    def get_label_tensor(self):
        return self.label_tensor

    def get_output_tensor(self):
        return self.layers[-1].outputs[0]
