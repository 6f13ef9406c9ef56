#!/usr/bin/env python3
"""Train any zoo model on synthetic data and print the reference's throughput line.

    python apps/train.py alexnet -b 256 -e 1 [--iterations 20] [--small] [--image-dir DIR] [reference FFConfig flags]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 apps/train.py inception_v3 -b 64 --budget 2000

Mirrors the reference apps (examples/cpp/{AlexNet,InceptionV3,ResNet,candle_uno,DLRM}): the random
input batch is loaded once and reused (alexnet.cc:106-111), the timed loop runs forward /
zero_gradients / backward / update, and the result is printed as
``ELAPSED TIME = ...s, THROUGHPUT = ... samples/s`` (alexnet.cc:129).  With ``--budget N`` the
strategy comes from the MCMC search over the MI355X simulator (``--export`` writes it as .pb).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(add_help=True)
    ap.add_argument("model")
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--iterations", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--graph", action="store_true", help="replay the step as hipGraph segments")
    ap.add_argument("--image-dir", default=None,
                    help="ImageNet-style folder (one sub-directory per class): decode + GPU-normalize a new "
                         "batch every iteration (flexmi.utils.images) instead of the reused random batch")
    a, rest = ap.parse_known_args(argv)

    import numpy as np
    import torch
    from flexmi.core import FFConfig, FFModel, SGDOptimizer, DataType
    from flexmi.models import zoo
    from flexmi.parallel.comm import init_distributed

    comm = init_distributed()
    cfg = FFConfig()
    cfg.parse_args(["train.py"] + rest)
    if torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    model = FFModel(cfg)
    built = zoo.build(a.model, model, small=a.small)
    model.optimizer = SGDOptimizer(model, cfg.learningRate if "--lr" in rest else built.lr)
    model.compile(model.optimizer, built.loss, built.metrics)
    ex = model.init_layers()
    rng = np.random.RandomState(comm.rank + 1)
    if "dlrm" in built.extra:
        from flexmi.models.dlrm import SyntheticDLRMData
        ins = list(built.inputs.values())
        data = SyntheticDLRMData(model, ins[0], ins[1:], built.extra["dlrm"], num_batches=1)
        data.next_batch()
    else:
        for t in built.inputs.values():
            if t.data_type in (DataType.DT_INT32, DataType.DT_INT64):
                arr = rng.randint(0, built.extra.get("int_range", 2), t.dims).astype(np.int32)
            else:
                arr = rng.rand(*t.dims).astype(np.float32)
            ex.scatter_from_host(t, arr)
        lab = model.get_label_tensor()
        if lab.data_type == DataType.DT_INT32:
            ncls = built.output.dims[-1]
            ex.scatter_from_host(lab, rng.randint(0, ncls, lab.dims).astype(np.int32))
        else:
            ex.scatter_from_host(lab, rng.rand(*lab.dims).astype(np.float32))
    sync = (lambda: torch.cuda.synchronize()) if ex.backend == "hip" else (lambda: None)
    loader = None
    if a.image_dir:
        from flexmi.utils.images import ImageFolderLoader
        img = next(t for t in built.inputs.values() if len(t.dims) == 4)
        loader = ImageFolderLoader(model, img, model.get_label_tensor(), a.image_dir, shuffle=True, seed=comm.rank,
                                   threads=16)
        loader.next_batch()
    for _ in range(a.warmup):
        ex.train_step()
    step = ex.train_step
    if a.graph and ex.backend == "hip":
        step = ex.capture_step()
    if loader is not None:
        inner = step

        def step():
            loader.next_batch()
            inner()
    sync()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(a.iterations):
        step()
    sync()
    comm.barrier()
    el = time.perf_counter() - t0
    samples = cfg.batchSize * a.iterations
    m = model.get_perf_metrics()
    if comm.rank == 0:
        print(f"[{a.model}] batch {cfg.batchSize} x {a.iterations} iterations on {comm.world} device(s), "
              f"loss {m.get_loss():.4f} accuracy {m.get_accuracy():.2f}%", file=sys.stderr)
        print(f"ELAPSED TIME = {el:.4f}s, THROUGHPUT = {samples / el:.2f} samples/s", flush=True)
        from flexmi.ops import _kernels as K
        for d, key, times, pick in K.CONV_TUNE_LOG:   # per-layer measured convolution forms
            print(f"[conv-tune] {d} x{list(key[0])} w{list(key[1])} s{key[2][0]}: " +
                  " ".join(f"{f}={t:.1f}us" for f, t in sorted(times.items(), key=lambda kv: kv[1])) + f" -> {pick}",
                  file=sys.stderr)
    if cfg.metrics_log:
        from flexmi.utils.log import MetricsLogger
        mlog = MetricsLogger(cfg.metrics_log, cfg)
        mlog.event("summary", model=a.model, world=comm.world, iterations=a.iterations, elapsed_s=el,
                   samples_per_s=samples / el, loss=m.get_loss(), accuracy=m.get_accuracy())
        mlog.close()
    return samples / el


if __name__ == "__main__":
    main()
