"""Keras ``Model`` (functional) and ``Sequential`` (``python/flexflow/keras/models/*.py``).

``compile`` creates the FFModel (FFConfig parsed from the command line, so ``-b`` / strategy /
search flags apply exactly as for native scripts), lowers the layer graph in topological order,
and compiles it; ``fit`` builds one data loader per input plus the label loader and runs the
reference training loop with callbacks (``base_model.py:367-445``), printing the same
``THROUGHPUT`` line; ``evaluate`` runs forward + metrics only.
"""
from __future__ import annotations

import sys
import time
from typing import List

import numpy as np

from flexmi.core import FFConfig, FFModel, SingleDataLoader
from flexmi.core.types import DataType

from . import losses as L
from . import metrics as Mt
from .layers import InputLayer, KTensor, Layer
from .layers import _Merge as _MergeBase


class Model:
    def __init__(self, inputs=None, outputs=None, name=None, ffconfig=None):
        self.name = name or "model"
        self._inputs: List[KTensor] = list(inputs) if isinstance(inputs, (list, tuple)) else ([inputs] if inputs else [])
        self._output: KTensor = outputs
        self._ffconfig = ffconfig
        self.ffmodel = None
        self.optimizer = None
        self._loss = None
        self._metrics = []
        self._loaders = []
        self._label_loader = None

    # -- graph ------------------------------------------------------------------------
    @property
    def layers(self) -> List[Layer]:
        if getattr(self, "_snapshot", None) is not None:
            return [lay for lay, _, _ in self._snapshot]
        order, seen = [], set()

        def visit(t):
            lay = t.layer
            if lay is None or id(lay) in seen:
                return
            for u in lay.inputs:
                visit(u)
            seen.add(id(lay))
            order.append(lay)
        visit(self._output)
        return [lay for lay in order if not isinstance(lay, InputLayer)]

    # -- nesting: a model used as a layer replays its layers on the new inputs ----------
    def __call__(self, x):
        xs = list(x) if isinstance(x, (list, tuple)) else [x]
        if len(xs) != len(self._inputs):
            raise ValueError(f"model {self.name} takes {len(self._inputs)} inputs, got {len(xs)}")
        if getattr(self, "_snapshot", None) is None:
            # the layers get rebound to the caller's graph: remember this model's own wiring
            self._snapshot = [(lay, list(lay.inputs), list(lay.outputs)) for lay in self.layers]
        env = {id(t): u for t, u in zip(self._inputs, xs)}
        for lay, lins, louts in self._snapshot:
            ins = [env[id(t)] for t in lins]
            old = louts
            out = lay(ins if len(ins) > 1 or isinstance(lay, _MergeBase) else ins[0])
            new = out if isinstance(out, list) else [out]
            for o, n in zip(old, new):
                env[id(o)] = n
        return env[id(self._output)]

    @property
    def input(self):
        """Input tensors (a list, as the reference's ``model.input[0]`` expects)."""
        return list(self._inputs)

    @property
    def output(self):
        return self._output

    @property
    def input_shape(self):
        return self._inputs[0].shape if self._inputs else None

    def get_layer(self, name=None, index=None):
        lays = self.layers
        if index is not None:
            return lays[index]
        for lay in lays:
            if lay.name == name:
                return lay
        raise ValueError(f"no layer {name!r}")

    def summary(self):
        s = f'Model: "{self.name}"\n' + "".join(lay.get_summary() for lay in self.layers)
        return s

    # -- compile ----------------------------------------------------------------------
    def compile(self, optimizer, loss=None, metrics=None, batch_size=None, **kwargs):
        if loss is None:
            raise ValueError("loss is None")
        self._loss = loss if isinstance(loss, L.Loss) else L.get(loss)
        self._metrics = [m if isinstance(m, Mt.Metric) else Mt.get(m) for m in (metrics or [])]
        cfg = self._ffconfig or FFConfig()
        if self._ffconfig is None:
            cfg.parse_args(sys.argv)
        if batch_size is not None:
            cfg.batchSize = int(batch_size)
        self._ffconfig = cfg
        m = FFModel(cfg)
        self.ffmodel = m
        b = cfg.batchSize
        for t in self._inputs:
            t.ff = m.create_tensor([b] + list(t.shape), t.dtype, name=t.layer.name if t.layer else None)
        for lay in self.layers:
            ins = [t.ff for t in lay.inputs]
            if any(x is None for x in ins):
                raise ValueError(f"layer {lay.name} consumes a tensor that is not produced by the model inputs")
            out = lay.build_ff(m, ins)
            lay.ff_op = out.owner_op if all(out is not x for x in ins) else None
            outs = out if isinstance(out, list) else [out]
            for kt, ft in zip(lay.outputs, outs):
                kt.ff = ft
        self.optimizer = optimizer
        m.compile(optimizer.build(m), self._loss.type, [mt.type for mt in self._metrics])
        return self

    # -- data ---------------------------------------------------------------------------
    def _loaders_for(self, x, y):
        xs = x if isinstance(x, (list, tuple)) else [x]
        if len(xs) != len(self._inputs):
            raise ValueError(f"model has {len(self._inputs)} inputs, got {len(xs)} arrays")
        m = self.ffmodel
        n = len(xs[0])
        loaders = []
        for t, arr in zip(self._inputs, xs):
            arr = np.ascontiguousarray(arr, dtype=np.float32 if t.dtype == DataType.DT_FLOAT else np.int32)
            loaders.append(SingleDataLoader(m, t.ff, arr, n))
        lab = m.get_label_tensor()
        y = np.asarray(y)
        y = y.reshape(n, -1).astype(np.int32 if lab.data_type == DataType.DT_INT32 else np.float32)
        lab_loader = SingleDataLoader(m, lab, y, n)
        return loaders, lab_loader, n

    def fit(self, x=None, y=None, batch_size=None, epochs=1, callbacks=None, verbose=1, **kwargs):
        if batch_size is not None and batch_size != self._ffconfig.batchSize:
            raise ValueError("batch size is fixed at compile time (use -b or compile(batch_size=...))")
        self._loaders, self._label_loader, self._num_samples = self._loaders_for(x, y)
        self.ffmodel.init_layers()
        return self._train(epochs, callbacks or [], train=True, verbose=verbose)

    def evaluate(self, x=None, y=None, batch_size=None, callbacks=None, verbose=1, **kwargs):
        self._loaders, self._label_loader, self._num_samples = self._loaders_for(x, y)
        self.ffmodel.init_layers()
        return self._train(1, callbacks or [], train=False, verbose=verbose)

    def _train(self, epochs, callbacks, train, verbose):
        m = self.ffmodel
        for cb in callbacks:
            cb.set_model(self)
            cb.on_train_begin()
        bs = self._ffconfig.batchSize
        iters = self._num_samples // bs
        t0 = time.time()
        history = []
        epoch = 0
        while epoch < epochs:
            for cb in callbacks:
                cb.on_epoch_begin(epoch)
            for d in self._loaders:
                d.reset()
            self._label_loader.reset()
            m.reset_metrics()
            for it in range(iters):
                for cb in callbacks:
                    cb.on_batch_begin(it)
                for d in self._loaders:
                    d.next_batch(m)
                self._label_loader.next_batch(m)
                if train and epoch > 0:
                    m.begin_trace(100)         # reference Keras trace id (base_model.py _train)
                m.forward()
                if train:
                    m.zero_gradients()
                    m.backward()
                    m.update()
                    if epoch > 0:
                        m.end_trace(100)
                else:
                    m.compute_metrics()
                for cb in callbacks:
                    cb.on_batch_end(it)
            pm = m.get_perf_metrics()
            history.append({"accuracy": pm.get_accuracy(), "loss": pm.get_loss()})
            if verbose and self._ffconfig.rank == 0:
                print(f"epoch {epoch}: accuracy {pm.get_accuracy():.2f}% loss {pm.get_loss():.4f}", file=sys.stderr)
            stop = False
            for cb in callbacks:
                stop = bool(cb.on_epoch_end(epoch)) or stop
            epoch += 1
            if stop:
                break
        el = max(time.time() - t0, 1e-9)
        if verbose and self._ffconfig.rank == 0:
            print(f"epochs {epoch}, ELAPSED TIME = {el:.4f}s, interations {iters}, samples {self._num_samples}, "
                  f"THROUGHPUT = {self._num_samples * epoch / el:.2f} samples/s")
        for cb in callbacks:
            cb.on_train_end()
        return history


class Sequential(Model):
    def __init__(self, layers=None, name=None, ffconfig=None):
        super().__init__(name=name or "sequential", ffconfig=ffconfig)
        self._stack: List = []
        for lay in layers or []:
            self.add(lay)

    def add(self, layer):
        if isinstance(layer, KTensor):            # Input(...) placed first
            self._inputs = [layer]
            self._output = layer
            return
        if not self._inputs:
            if layer.input_shape is None:
                raise ValueError("the first layer needs input_shape (or start with Input(...))")
            from .layers import Input
            t = Input(shape=layer.input_shape)
            self._inputs = [t]
            self._output = t
        self._output = layer(self._output)
        self._stack.append(layer)

    def pop(self):
        raise NotImplementedError("Sequential.pop is not supported")
