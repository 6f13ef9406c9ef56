"""Worker of tests/test_gpu_rccl_multi.py (one rank per GPU, torch.distributed.run, RCCL): trains a
small DLRM for a few steps under ``strategy`` (table | dp) and saves rank 0's parameters.  The
sparse-DP and chunked-exchange switches (FLEXMI_SPARSE_DP, FLEXMI_XCHG_CHUNKS) come from the
environment -- module constants, so each variant is its own launch."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(strategy, out):
    import torch
    import torch.distributed as dist
    from flexmi.parallel.comm import init_distributed
    comm = init_distributed()
    rank, world = comm.rank, comm.world
    cuda = torch.cuda.is_available()
    if cuda:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    from flexmi.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    from flexmi.models.dlrm import DLRMConfig, build_dlrm, dlrm_strategy
    B = 2048 * world   # >= 1024 rows per rank: the auto exchange pipelining engages
    dcfg = DLRMConfig(64, [20000, 300, 12, 70000, 40, 5000], [13, 128, 64], [128, 64, 1], 1, -1, -1, 0.0, "dot", "", -1,
                      "bce", "rccl_multi")
    cfg = FFConfig()
    cfg.batchSize, cfg.compute_dtype, cfg.seed = B, "fp32", 3
    if not cuda:
        cfg.device = "cpu"   # gloo rehearsal of the same plan
    m = FFModel(cfg)
    d, s, _ = build_dlrm(m, dcfg)
    if strategy == "table":
        m.strategies = dlrm_strategy(m, world)
    m.compile(SGDOptimizer(m, 0.1), LossType.LOSS_BINARY_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
    if strategy == "table":
        m.strategies = dlrm_strategy(m, world)
    ex = m.init_layers()
    rng = np.random.RandomState(11)
    for _ in range(3):
        dd = np.zeros((B, d.dims[1]), np.float32)
        dd[:, :13] = rng.rand(B, 13)
        ex.scatter_from_host(d, dd)
        for t, r in zip(s, dcfg.embedding_size):
            ex.scatter_from_host(t, np.minimum(rng.zipf(1.3, (B, 1)) - 1, r - 1).astype(np.int64))
        ex.scatter_from_host(m.get_label_tensor(), rng.randint(0, 2, (B, 1)).astype(np.float32))
        ex.train_step()
    if cuda:
        torch.cuda.synchronize()
    params = [p.get_weights(m) for p in m.parameters]
    if rank == 0:
        np.savez(out, *params)
        print(f"rccl multi ok: {strategy} world {world} sparse_dp={os.environ.get('FLEXMI_SPARSE_DP', '1')} "
              f"chunks={os.environ.get('FLEXMI_XCHG_CHUNKS', 'auto')} pipe={ex.pipe is not None}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
