#!/usr/bin/env python3
"""The reference DLRM application (``examples/cpp/DLRM/dlrm.cc:77-199``) on flexmi.

    python apps/dlrm.py --arch-sparse-feature-size 64 --arch-embedding-size 1000000-1000000 \\
        --arch-mlp-bot 64-512-512-64 --arch-mlp-top 576-1024-1024-1024-1 -b 2048 -e 1 [--dataset f.h5]
    python apps/dlrm.py --preset summit_large -b 256 -e 1
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 apps/dlrm.py --preset run_random -b 2048 --strategy s.pb

Same flags as the reference (``parse_input_args`` dlrm.cc:201-264 + the FFConfig flag set):
``--dataset`` trains on the HDF5 file written by ``preprocess_hdf.py`` (native reader + prefetch
ring, ``HDF5DLRMData``), otherwise on random data of ``--data-size`` samples (default 256 x 4 x
GPUs, dlrm.cc:273-282); ``--loss-threshold t`` clamps predictions to [t, 1-t] in the loss.  The
loop is the reference's (dlrm.cc:160-195): per epoch ``num_samples / batch`` iterations of
next_batch / forward / zero_gradients / backward / update, traced with begin/end_trace(111),
then ``ELAPSED TIME = ..., THROUGHPUT = ... samples/s``.  ``--preset`` (mlperf, run_random,
criteo_kaggle, summit, summit_large, kaggle_day1, tiny) seeds the architecture flags.
"""
from __future__ import annotations

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    import torch
    from flexmi.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    from flexmi.models.dlrm import DLRMConfig, HDF5DLRMData, SyntheticDLRMData, build_dlrm
    from flexmi.parallel.comm import init_distributed

    comm = init_distributed()
    base = None
    if "--preset" in argv:
        k = argv.index("--preset")
        base = DLRMConfig.preset(argv[k + 1])
        del argv[k:k + 2]
    dcfg = DLRMConfig.parse_args(["dlrm"] + argv, base)
    cfg = FFConfig()
    cfg.parse_args(["dlrm"] + argv)
    if dcfg.dataset_path and not cfg.dataset_path:
        cfg.dataset_path = dcfg.dataset_path
    if torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    model = FFModel(cfg)
    dense_in, sparse, out = build_dlrm(model, dcfg)
    loss = LossType.LOSS_BINARY_CROSSENTROPY if dcfg.loss == "bce" else LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE
    model.compile(SGDOptimizer(model, cfg.learningRate), loss,
                  [MetricsType.METRICS_ACCURACY, MetricsType.METRICS_MEAN_SQUARED_ERROR])
    ex = model.init_layers()
    if dcfg.dataset_path:
        data = HDF5DLRMData(model, dense_in, sparse, dcfg)
        num_samples = data.num_samples
    else:
        num_samples = dcfg.data_size if dcfg.data_size > 0 else 256 * 4 * cfg.workersPerNode * cfg.numNodes
        num_samples = max(num_samples, cfg.batchSize)
        data = SyntheticDLRMData(model, dense_in, sparse, dcfg, num_batches=max(1, num_samples // cfg.batchSize),
                                 seed=comm.rank)
    iters = max(1, num_samples // cfg.batchSize)
    sync = torch.cuda.synchronize if ex.backend == "hip" else (lambda: None)
    # warm-up iteration (dlrm.cc:153-158), not timed
    data.next_batch()
    ex.train_step()
    sync()
    comm.barrier()
    t0 = time.perf_counter()
    for epoch in range(cfg.epochs):
        model.reset_metrics()
        for it in range(iters):
            if epoch > 0 or it > 0:
                model.begin_trace(111)
            data.next_batch()
            model.forward()
            model.zero_gradients()
            model.backward()
            model.update()
            if epoch > 0 or it > 0:
                model.end_trace(111)
    sync()
    comm.barrier()
    el = time.perf_counter() - t0
    m = model.get_perf_metrics()
    samples = num_samples * cfg.epochs
    if comm.rank == 0:
        print(f"[dlrm {dcfg.name}] {cfg.epochs} epoch(s) x {iters} iterations, batch {cfg.batchSize}, "
              f"{comm.world} device(s), {'dataset ' + dcfg.dataset_path if dcfg.dataset_path else 'random data'}: "
              f"loss {m.get_loss():.5f} accuracy {m.get_accuracy():.2f}%", file=sys.stderr)
        print(f"ELAPSED TIME = {el:.4f}s, THROUGHPUT = {samples / el:.2f} samples/s", flush=True)
    if hasattr(data, "close"):
        data.close()
    return samples / el, m


if __name__ == "__main__":
    main()
