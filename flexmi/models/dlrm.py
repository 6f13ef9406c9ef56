"""DLRM (the reference's headline workload, ``examples/cpp/DLRM/dlrm.cc:26-199``).

Graph: dense input -> bottom MLP; every sparse feature -> embedding bag; feature interaction
(``cat`` as in the reference, or ``dot`` -- the DLRM/MLPerf interaction the reference left as a
TODO, caveat C3); top MLP ending in a sigmoid; MSE (reference) or BCE (MLPerf) loss; SGD.
Initialisers follow ``create_mlp``/``create_emb`` (``dlrm.cc:26-47``): MLP weights
N(0, sqrt(2/(in+out))), biases N(0, sqrt(2/out)), tables U(±sqrt(1/rows)).

Default strategy (``dlrm_strategy``): embedding tables placed whole on GPUs with a greedy
size/traffic-balanced assignment (the table-wise model parallelism of
``src/runtime/dlrm_strategy.cc:242-296``) + data-parallel MLPs; the exchange between the
table-placed embeddings and the sample-parallel interaction is ONE RCCL all-to-all per direction.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List

import numpy as np
import torch

from flexmi.core.initializers import NormInitializer, UniformInitializer
from flexmi.core.types import ActiMode, AggrMode, DataType, LossType, MetricsType
from flexmi.parallel.layout import ParallelConfig

# Criteo Terabyte feature cardinalities with --max-ind-range=40M (MLPerf DLRM v1 configuration)
MLPERF_TABLES = [39884406, 39043, 17289, 7420, 20263, 3, 7120, 1543, 63, 38532951, 2953546, 403346, 10, 2208,
                 11938, 155, 4, 976, 14, 39979771, 25641295, 39664984, 585935, 12972, 108, 36]
# run_criteo_kaggle.sh:8 (Kaggle cardinalities)
KAGGLE_TABLES = [1396, 550, 1761917, 507795, 290, 21, 11948, 608, 3, 58176, 5237, 1497287, 3127, 26, 12153, 1068715,
                 10, 4836, 2085, 4, 1312273, 17, 15, 110946, 91, 72655]


@dataclass
class DLRMConfig:
    """``struct DLRMConfig`` (``examples/cpp/DLRM/dlrm.h:24-42``) + flexmi knobs."""
    sparse_feature_size: int = 2
    embedding_size: List[int] = field(default_factory=lambda: [4])
    mlp_bot: List[int] = field(default_factory=lambda: [4, 2])
    mlp_top: List[int] = field(default_factory=lambda: [8, 2])
    embedding_bag_size: int = 1
    sigmoid_bot: int = -1
    sigmoid_top: int = -1
    loss_threshold: float = 0.0
    arch_interaction_op: str = "cat"
    dataset_path: str = ""
    data_size: int = -1
    loss: str = "mse"            # mse (reference) | bce (MLPerf)
    name: str = "custom"

    @staticmethod
    def preset(name):
        if name == "run_random":  # examples/cpp/DLRM/run_random.sh:9
            return DLRMConfig(64, [1000000] * 8, [64, 512, 512, 64], [576, 1024, 1024, 1024, 1], 1, -1, -1, 0.0,
                              "cat", "", -1, "mse", "run_random")
        if name == "mlperf":      # MLPerf DLRM (Criteo Terabyte): 13 dense + 26 sparse, dot, d=128
            return DLRMConfig(128, list(MLPERF_TABLES), [13, 512, 256, 128], [479, 1024, 1024, 512, 256, 1], 1, -1, -1,
                              0.0, "dot", "", -1, "bce", "mlperf")
        if name == "criteo_kaggle":  # run_criteo_kaggle.sh
            return DLRMConfig(16, list(KAGGLE_TABLES), [13, 512, 256, 64, 16], [224, 512, 256, 1], 1, -1, -1, 0.0,
                              "cat", "", -1, "mse", "criteo_kaggle")
        if name == "summit":      # run_summit.sh:3-13 (512 samples per GPU)
            return DLRMConfig(64, [1000000] * 8, [64, 512, 512, 64], [576, 1024, 1024, 1024, 1], 1, -1, -1, 0.0,
                              "cat", "", -1, "mse", "summit")
        if name == "summit_large":  # run_summit_large.sh:3-16 (bag 100, 256 samples per GPU)
            return DLRMConfig(64, [1000000] * 6, [2048, 4096, 4096, 4096, 4096, 4096],
                              [10240, 4096, 4096, 4096, 4096, 1], 100, -1, -1, 0.0, "cat", "", -1, "mse", "summit_large")
        if name == "kaggle_day1":  # run_dlrm_kaggle_day1.sh (batch 128, --dataset kaggle_day_1.h5); the script's
            # "--arch-sparse-feature-sie 13" is a typo the reference parser ignores -> d follows the bottom MLP (16)
            return DLRMConfig(16, list(KAGGLE_TABLES), [13, 512, 256, 64, 16], [512, 256, 1], 1, -1, -1, 0.0,
                              "cat", "", -1, "mse", "kaggle_day1")
        if name == "tiny":
            return DLRMConfig(16, [100, 50, 200, 30], [13, 32, 16], [64, 32, 1], 1, -1, -1, 0.0, "dot", "", -1, "bce", "tiny")
        raise KeyError(name)

    @staticmethod
    def parse_args(argv, base=None):
        """``parse_input_args`` of ``dlrm.cc:201-264`` (same flag spellings)."""
        c = base or DLRMConfig()
        i = 1
        while i < len(argv):
            a = argv[i]
            nx = argv[i + 1] if i + 1 < len(argv) else None
            if a == "--arch-sparse-feature-size":
                c.sparse_feature_size = int(nx); i += 1
            elif a == "--arch-embedding-size":
                c.embedding_size = [int(x) for x in nx.split("-")]; i += 1
            elif a == "--embedding-bag-size":
                c.embedding_bag_size = int(nx); i += 1
            elif a == "--arch-mlp-bot":
                c.mlp_bot = [int(x) for x in nx.split("-")]; i += 1
            elif a == "--arch-mlp-top":
                c.mlp_top = [int(x) for x in nx.split("-")]; i += 1
            elif a == "--loss-threshold":
                c.loss_threshold = float(nx); i += 1
            elif a == "--sigmoid-top":
                c.sigmoid_top = int(nx); i += 1
            elif a == "--sigmoid-bot":
                c.sigmoid_bot = int(nx); i += 1
            elif a == "--arch-interaction-op":
                c.arch_interaction_op = nx; i += 1
            elif a == "--dataset":
                c.dataset_path = nx; i += 1
            elif a == "--data-size":
                c.data_size = int(nx); i += 1
            elif a == "--dlrm-loss":
                c.loss = nx; i += 1
            i += 1
        return c


def create_mlp(model, x, ln, sigmoid_layer, seed_base=0):
    """``create_mlp`` (``dlrm.cc:26-39``).  If ``x`` is a zero-padded input (more columns than
    ln[0]), the first layer is initialised as the unpadded one (ColumnPaddedInitializer)."""
    from flexmi.core.initializers import ColumnPaddedInitializer
    t = x
    for i in range(len(ln) - 1):
        std = math.sqrt(2.0 / (ln[i + 1] + ln[i]))
        winit = NormInitializer(model._next_seed(), 0.0, std)
        if i == 0 and x.dims[-1] != ln[0]:
            winit = ColumnPaddedInitializer(winit, ln[0])
        binit = NormInitializer(model._next_seed(), 0.0, math.sqrt(2.0 / ln[i + 1]))
        act = ActiMode.AC_MODE_SIGMOID if i == sigmoid_layer else ActiMode.AC_MODE_RELU
        t = model.dense(t, ln[i + 1], act, True, None, winit, binit)
    return t


def create_emb(model, idx, rows, dim, i):
    r = math.sqrt(1.0 / rows)
    return model.embedding(idx, rows, dim, AggrMode.AGGR_MODE_SUM, None, UniformInitializer(model._next_seed(), -r, r),
                           name=f"embedding{i}")


def build_dlrm(model, c: DLRMConfig, pad_dense=True):
    """Returns (dense_input, sparse_inputs, output).  Dense input is padded to a multiple of 8
    columns (zeros) so its GEMM uses 16-B vector loads; the padding does not change the model.
    ``loss_threshold`` in (0, 1) clamps predictions to [t, 1-t] in the loss (the clamp the
    reference leaves as a TODO + assert, dlrm.cc:129-132)."""
    B = model.config.batchSize
    if 0.0 < c.loss_threshold < 1.0:
        model.loss_threshold = min(c.loss_threshold, 0.5)
    sparse = [model.create_tensor([B, c.embedding_bag_size], DataType.DT_INT64, name=f"sparse{i}")
              for i in range(len(c.embedding_size))]
    bot = list(c.mlp_bot)
    if pad_dense and model.config.device == "gpu":
        bot[0] = (bot[0] + 7) // 8 * 8   # 13 -> 16: 16-B aligned rows for the first GEMM (pad columns are 0)
    dense_in = model.create_tensor([B, bot[0]], DataType.DT_FLOAT, name="dense")
    dense_in.real_features = c.mlp_bot[0]
    x = create_mlp(model, dense_in, list(c.mlp_bot), c.sigmoid_bot)
    ly = [create_emb(model, sparse[i], c.embedding_size[i], c.sparse_feature_size, i) for i in range(len(sparse))]
    if c.arch_interaction_op == "cat":
        z = model.concat([x] + ly, 1, name="concat")
    elif c.arch_interaction_op == "dot":
        z = model.dot_interaction(x, ly, name="interaction")
    else:
        raise ValueError(c.arch_interaction_op)
    top = [z.dims[1]] + list(c.mlp_top[1:])
    sig = c.sigmoid_top if c.sigmoid_top >= 0 else len(top) - 2
    p = create_mlp(model, z, top, sig)
    return dense_in, sparse, p


def dlrm_strategy(model, num_gpus, table_sizes=None, split_factor=0.5):
    """Embedding placement + DP elsewhere (the reference's table-wise plan, ``dlrm_strategy.cc:242-296``,
    made HBM-balanced for MLPerf-size tables).

    * Tables holding more than ``split_factor`` x (total table bytes / num_gpus) are split on the
      PARAMETER (column) dimension over all GPUs -- ``ParallelConfig([num_gpus, 1])``: every GPU
      holds all rows x d/num_gpus columns, looks up the full global batch for its columns, and the
      exchange to the data-parallel interaction moves B x d/num_gpus per peer (an 8th of a row-split
      table's partial sums).  For the Criteo-TB set at 8 GPUs the four ~40 M-row tables become
      4 x 2.6 GB per GPU instead of 20.9 GB on one.
    * The other tables go whole to one GPU (table-wise model parallelism), greedily: the GPU with
      the fewest tables, then the least bytes.
    Returns {op name: ParallelConfig}."""
    from flexmi.core.types import OperatorType
    embs = [op for op in model.layers if op.op_type == OperatorType.OP_EMBEDDING]
    nbytes = [e.num_entries * e.out_dim * 4 for e in embs]
    total = sum(nbytes)
    strat = {}
    loads = [0.0] * num_gpus
    counts = [0] * num_gpus
    split = set()
    if num_gpus > 1:
        for i, e in enumerate(embs):
            cols_ok = e.out_dim % num_gpus == 0 and (e.out_dim // num_gpus) % 4 == 0
            if cols_ok and nbytes[i] > split_factor * total / num_gpus:
                split.add(i)
                strat[e.name] = ParallelConfig([num_gpus, 1], list(range(num_gpus)))
                for g in range(num_gpus):
                    loads[g] += nbytes[i] / num_gpus
    order = sorted((i for i in range(len(embs)) if i not in split), key=lambda i: -nbytes[i])
    for i in order:
        g = min(range(num_gpus), key=lambda k: (counts[k], loads[k]))
        loads[g] += nbytes[i]
        counts[g] += 1
        strat[embs[i].name] = ParallelConfig([1, 1], [g])
    return strat


def strategy_table_bytes(model, strategies, num_gpus):
    """Embedding-table bytes held by each GPU under ``strategies`` (HBM balance of a plan)."""
    from flexmi.core.types import OperatorType
    per = [0.0] * num_gpus
    for op in model.layers:
        if op.op_type != OperatorType.OP_EMBEDDING:
            continue
        b = op.num_entries * op.out_dim * 4.0
        pc = strategies.get(op.name)
        if pc is None:                              # data parallel: replicated everywhere
            for g in range(num_gpus):
                per[g] += b
            continue
        d = list(pc.dims) + [1] * (3 - len(pc.dims))
        c, n, r = int(d[0]), int(d[1]), int(d[2])
        for dev in pc.device_ids:
            per[dev] += b / (c * r)
    return per


class SyntheticDLRMData:
    """Random-data generator mirroring the reference's random mode (``dlrm.cc:355-424``: indices
    uniform in [0, rows), dense U[0,1), labels {0,1}); pools of batches are generated ONCE on the
    device (like ``--data-size``) and cycled, so the timed loop measures training, not RNG."""

    def __init__(self, model, dense_in, sparse, cfg: DLRMConfig, num_batches=4, seed=0):
        self.model = model
        self.dense_in, self.sparse, self.cfg = dense_in, sparse, cfg
        self.nb = num_batches
        ex = model._ex()
        dev = ex.device
        g = torch.Generator(device=dev)
        g.manual_seed(1234 + seed)
        B = model.config.batchSize
        self.pools = {}
        # each rank only materialises the rows of the tensors it holds (home layout)
        for t, rows in zip(sparse, cfg.embedding_size):
            buf = ex.local_buffer(t)
            if buf is None:
                continue
            lay = ex.home[t.guid]
            box = lay.local_box(ex.rank)
            n = box[0][1] - box[0][0]
            self.pools[t.guid] = torch.randint(0, rows, (num_batches, n, buf.shape[1]), generator=g, device=dev,
                                               dtype=buf.dtype)
        buf = ex.local_buffer(dense_in)
        if buf is not None:
            pool = torch.rand((num_batches,) + tuple(buf.shape), generator=g, device=dev)
            nreal = getattr(dense_in, "real_features", buf.shape[1])
            pool[..., nreal:] = 0.0        # zero padding columns: the model is unchanged
            self.pools[dense_in.guid] = pool.to(buf.dtype)
        lab = model.get_label_tensor()
        lbuf = ex.local_buffer(lab)
        if lbuf is not None:
            self.pools[lab.guid] = torch.randint(0, 2, (num_batches,) + tuple(lbuf.shape), generator=g, device=dev).to(lbuf.dtype)
        self.i = 0

    def next_batch(self):
        ex = self.model.executor
        k = self.i % self.nb
        ex.load_local_many([(ex.tensors[gid], pool[k]) for gid, pool in self.pools.items()])
        self.i += 1


class HDF5DLRMData:
    """``--dataset FILE``: the Criteo HDF5 layout written by ``preprocess_hdf.py`` (X_int float32
    [N, 13] = log(1+x), X_cat int64 [N, tables*bag], y float32 [N]) and loaded by the reference
    (``dlrm.cc:284-330`` shapes/classes checked, ``:425-483`` whole dataset read, ``:489-589``
    next_batch = consecutive samples).  flexmi memory-maps the datasets (native HDF5 reader,
    ``flexmi.utils.hdf5``) and streams batches through the native prefetch ring: each sparse
    input is a zero-copy column block of X_cat, the 13 dense features are zero-padded into the
    GPU's 16-wide input, every rank stages only its shard rows.  ``num_samples`` whole batches
    per epoch (``--data-size`` caps it), consecutive like the reference or shuffled."""

    def __init__(self, model, dense_in, sparse, cfg: DLRMConfig, path=None, shuffle=False, seed=0, depth=3, threads=2):
        from flexmi.core.dataloader import PrefetchLoader
        from flexmi.utils.hdf5 import open_h5
        path = path or cfg.dataset_path
        d = open_h5(path)
        for k in ("X_int", "X_cat", "y"):
            if k not in d:
                raise ValueError(f"{path}: dataset {k!r} missing (have {sorted(d)})")
        X_int, X_cat, y = d["X_int"], d["X_cat"], d["y"]
        if X_int.ndim != 2 or X_int.dtype.kind != "f" or X_int.shape[1] != cfg.mlp_bot[0]:
            raise ValueError(f"X_int must be float [N, {cfg.mlp_bot[0]}], got {X_int.dtype} {X_int.shape}")
        N = X_int.shape[0]
        bag = cfg.embedding_bag_size
        if X_cat.ndim != 2 or X_cat.dtype.kind not in "iu" or X_cat.shape != (N, len(sparse) * bag):
            raise ValueError(f"X_cat must be integer [N, {len(sparse) * bag}], got {X_cat.dtype} {X_cat.shape}")
        if y.shape[0] != N:
            raise ValueError("y must have one label per sample")
        self.num_samples = N if cfg.data_size <= 0 else min(N, cfg.data_size)
        B = model.config.batchSize
        if self.num_samples < B:
            raise ValueError(f"dataset has {self.num_samples} samples < batch {B}")
        self.arrays = d
        pairs = [(dense_in, X_int, (0, X_int.shape[1]))]
        pairs += [(t, X_cat, (i * bag, (i + 1) * bag)) for i, t in enumerate(sparse)]
        pairs.append((model.get_label_tensor(), y.reshape(N, 1), (0, 1)))
        self.loader = PrefetchLoader(model, pairs, self.num_samples, shuffle=shuffle, seed=seed, depth=depth,
                                     threads=threads)
        self.nb = self.num_samples // B

    def next_batch(self):
        self.loader.next_batch()

    def close(self):
        self.loader.close()
