"""DLRM workload surface: the native HDF5 reader (reference dataset path ``dlrm.cc:284-330``,
``preprocess_hdf.py``), the ``--dataset`` training path through the prefetch ring, the
``--loss-threshold`` clamp and the Summit / Kaggle-day-1 presets.  h5py is not installed, so the
files come from flexmi's own writer (h5py's default on-disk layout); real Criteo files are
parity-unpinned."""
import os

import numpy as np
import pytest
import torch


def _criteo_like(n, tables, bag=1, seed=0):
    rng = np.random.RandomState(seed)
    return {
        "X_int": np.log(rng.randint(0, 1000, (n, 13)).astype(np.float32) + 1),
        "X_cat": np.concatenate([rng.randint(0, r, (n, bag)) for r in tables], 1).astype(np.int64),
        "y": rng.randint(0, 2, n).astype(np.float32),
    }


def test_hdf5_roundtrip_dtypes_and_shapes(tmp_path, native):
    from flexmi.utils.hdf5 import list_datasets, open_h5, write_h5
    rng = np.random.RandomState(1)
    arrays = {"a_f4": rng.randn(7, 3).astype(np.float32), "b_f8": rng.randn(11).astype(np.float64),
              "c_i8": rng.randint(-9, 9, (2, 3, 4)).astype(np.int64), "d_i4": rng.randint(0, 9, (5,)).astype(np.int32),
              "e_u1": rng.randint(0, 255, (6, 2)).astype(np.uint8)}
    p = str(tmp_path / "x.h5")
    write_h5(p, arrays)
    info = list_datasets(p)
    assert set(info) == set(arrays)
    assert info["c_i8"][0] == "<i8" and info["c_i8"][1] == (2, 3, 4)
    assert info["e_u1"][0] == "<u1" and info["b_f8"][0] == "<f8"
    m = open_h5(p)
    for k, v in arrays.items():
        assert m[k].dtype == v.dtype and np.array_equal(m[k], v), k
    # every dataset's data is 512-B aligned and inside the file
    size = os.path.getsize(p)
    for k, (_, _, off, nb) in info.items():
        assert off % 512 == 0 and off + nb <= size


def test_hdf5_rejects_non_hdf5(tmp_path, native):
    from flexmi.utils.hdf5 import list_datasets
    p = tmp_path / "bad.h5"
    p.write_bytes(b"not an hdf5 file" * 64)
    with pytest.raises(RuntimeError, match="not an HDF5 file"):
        list_datasets(str(p))


def test_hdf5_rejects_truncated_and_corrupted(tmp_path, native):
    """Malformed files raise a clean error (no read past a buffer, no shift by >= 64 bits)."""
    from flexmi.utils.hdf5 import list_datasets, write_h5
    p = str(tmp_path / "ok.h5")
    write_h5(p, {"a": np.arange(4096, dtype=np.float32).reshape(64, 64)})
    good = open(p, "rb").read()
    info = list_datasets(p)
    off, nb = info["a"][2], info["a"][3]
    # data cut off: the dataset would extend past the end of the file
    t = tmp_path / "trunc.h5"
    t.write_bytes(good[:off + nb // 2])
    with pytest.raises(RuntimeError, match="past the end|read past"):
        list_datasets(str(t))
    # superblock offset size 0 / 16 (would make the address decoder shift by >= 64 bits)
    for bad in (0, 16):
        b = bytearray(good)
        b[9 if good[8] >= 2 else 13] = bad
        c = tmp_path / f"so{bad}.h5"
        c.write_bytes(bytes(b))
        with pytest.raises(RuntimeError, match="sizes"):
            list_datasets(str(c))
    # every single-byte corruption of the metadata either parses or raises (never crashes)
    rng = np.random.RandomState(0)
    for i in range(64):
        b = bytearray(good)
        pos = int(rng.randint(0, min(off, len(good))))
        b[pos] ^= int(rng.randint(1, 256))
        c = tmp_path / f"c{i}.h5"
        c.write_bytes(bytes(b))
        try:
            list_datasets(str(c))
        except RuntimeError:
            pass


def test_host_array_as_bf16_staging():
    """Column-block sources feeding a bf16 input are staged as bf16 bit patterns (numpy has no
    bfloat16): round to nearest even, same as torch's cast."""
    from flexmi.core.dataloader import _host_array_as
    x = np.random.RandomState(0).randn(33, 13).astype(np.float32)
    got = _host_array_as(x, torch.bfloat16)
    assert got.dtype == np.int16 and got.shape == x.shape and got.flags["C_CONTIGUOUS"]
    exp = torch.from_numpy(x).to(torch.bfloat16)
    assert torch.equal(torch.from_numpy(got).view(torch.bfloat16), exp)
    assert _host_array_as(x.astype(np.float64), torch.float32).dtype == np.float32
    assert _host_array_as(np.arange(6), torch.int32).dtype == np.int32


@pytest.mark.gpu
def test_dlrm_dataset_default_bf16_on_gpu(tmp_path, native):
    """apps/dlrm.py --dataset with the GPU default (bf16 compute): the dense column block is
    staged as bf16 and the step trains (this crashed in numpy)."""
    from flexmi.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    from flexmi.models.dlrm import DLRMConfig, HDF5DLRMData, build_dlrm
    from flexmi.utils.hdf5 import write_h5
    tables = [50, 20, 70, 9]
    dcfg = DLRMConfig(8, tables, [13, 16, 8], [40, 16, 1], 1, -1, -1, 0.0, "cat", "", -1, "mse", "h5")
    B, n = 32, 32 * 5
    arrays = _criteo_like(n, tables)
    path = str(tmp_path / "kaggle.h5")
    write_h5(path, arrays)
    cfg = FFConfig()
    cfg.batchSize = B
    m = FFModel(cfg)
    d, s, _ = build_dlrm(m, dcfg)
    m.compile(SGDOptimizer(m, 0.1), LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, [MetricsType.METRICS_ACCURACY])
    ex = m.init_layers()
    data = HDF5DLRMData(m, d, s, dcfg, path)
    for _ in range(6):
        data.next_batch()
        ex.train_step()
    torch.cuda.synchronize()
    data.close()
    dense = ex.local_buffer(d)
    assert dense.dtype == torch.bfloat16
    met = m.get_perf_metrics()
    assert met.train_all == 6 * B and np.isfinite(met.get_loss())


def _dlrm_model(dcfg, B, lt=0.0):
    from flexmi.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    from flexmi.models.dlrm import build_dlrm
    cfg = FFConfig()
    cfg.batchSize = B
    cfg.device = "cpu"
    cfg.compute_dtype = "fp32"
    cfg.seed = 3
    m = FFModel(cfg)
    dcfg.loss_threshold = lt
    d, s, p = build_dlrm(m, dcfg)
    m.compile(SGDOptimizer(m, 0.1), LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, [MetricsType.METRICS_ACCURACY])
    ex = m.init_layers()
    return m, ex, d, s


def test_dlrm_dataset_training_matches_manual_feed(tmp_path, native):
    """HDF5DLRMData (memory-mapped X_int / X_cat column blocks / y through the native ring) feeds
    exactly the consecutive batches the reference's next_batch copies (dlrm.cc:489-589)."""
    from flexmi.models.dlrm import DLRMConfig, HDF5DLRMData
    from flexmi.utils.hdf5 import write_h5
    tables = [50, 20, 70, 9]
    dcfg = DLRMConfig(8, tables, [13, 16, 8], [40, 16, 1], 1, -1, -1, 0.0, "cat", "", -1, "mse", "h5")
    B, n = 32, 32 * 5
    arrays = _criteo_like(n, tables)
    path = str(tmp_path / "kaggle.h5")
    write_h5(path, arrays)
    m, ex, d, s = _dlrm_model(dcfg, B)
    data = HDF5DLRMData(m, d, s, dcfg, path)
    assert data.num_samples == n and data.nb == 5
    for _ in range(7):        # wraps into the second epoch
        data.next_batch()
        ex.train_step()
    data.close()
    got = [p.get_weights(m) for p in m.parameters]
    m2, ex2, d2, s2 = _dlrm_model(DLRMConfig(8, tables, [13, 16, 8], [40, 16, 1], 1, -1, -1, 0.0, "cat", "", -1,
                                             "mse", "h5"), B)
    for it in range(7):
        k = it % 5
        rows = slice(k * B, (k + 1) * B)
        ex2.scatter_from_host(d2, arrays["X_int"][rows])
        for i, t in enumerate(s2):
            ex2.scatter_from_host(t, arrays["X_cat"][rows, i:i + 1])
        ex2.scatter_from_host(m2.get_label_tensor(), arrays["y"][rows].reshape(B, 1))
        ex2.train_step()
    exp = [p.get_weights(m2) for p in m2.parameters]
    for a, b in zip(got, exp):
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7)


def test_dlrm_dataset_shape_checks(tmp_path, native):
    from flexmi.models.dlrm import DLRMConfig, HDF5DLRMData
    from flexmi.utils.hdf5 import write_h5
    dcfg = DLRMConfig(8, [10, 10], [13, 8], [24, 1], 1, -1, -1, 0.0, "cat", "", -1, "mse", "h5")
    arrays = _criteo_like(64, [10, 10, 10])        # 3 sparse columns for a 2-table model
    path = str(tmp_path / "bad.h5")
    write_h5(path, arrays)
    m, ex, d, s = _dlrm_model(dcfg, 16)
    with pytest.raises(ValueError, match="X_cat"):
        HDF5DLRMData(m, d, s, dcfg, path)


def test_dlrm_app_dataset_and_presets(tmp_path, native):
    """apps/dlrm.py: reference flags + --dataset (HDF5) end to end, --data-size caps the epoch."""
    import importlib.util
    from flexmi.utils.hdf5 import write_h5
    spec = importlib.util.spec_from_file_location("dlrm_app", os.path.join(os.path.dirname(__file__), "..", "apps", "dlrm.py"))
    app = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(app)
    tables = [30, 40, 50]
    path = str(tmp_path / "day1.h5")
    write_h5(path, _criteo_like(256, tables))
    sps, met = app.main(["--arch-sparse-feature-size", "8", "--arch-embedding-size", "30-40-50",
                         "--arch-mlp-bot", "13-16-8", "--arch-mlp-top", "32-8-1", "--dataset", path,
                         "--data-size", "192", "-b", "64", "-e", "2", "--device", "cpu"])
    assert sps > 0 and met.train_all == 192 and met.get_loss() == met.get_loss()   # metrics reset per epoch


@pytest.mark.parametrize("preset", ["summit", "summit_large", "kaggle_day1"])
def test_reference_presets_build_and_step(preset):
    """run_summit.sh / run_summit_large.sh (bag 100, bottom 2048-4096x5, top ->4096x4-1) /
    run_dlrm_kaggle_day1.sh architectures (tables scaled down) train one step on CPU."""
    from flexmi.models.dlrm import DLRMConfig
    dcfg = DLRMConfig.preset(preset)
    dcfg.embedding_size = [min(r, 1000) for r in dcfg.embedding_size]
    if preset == "summit_large":
        assert dcfg.embedding_bag_size == 100 and dcfg.mlp_bot == [2048] + [4096] * 5
    m, ex, d, s = _dlrm_model(dcfg, 4)
    rng = np.random.RandomState(0)
    ex.scatter_from_host(d, rng.rand(*d.dims).astype(np.float32))
    for t, r in zip(s, dcfg.embedding_size):
        ex.scatter_from_host(t, rng.randint(0, r, t.dims).astype(np.int64))
    ex.scatter_from_host(m.get_label_tensor(), rng.randint(0, 2, (4, 1)).astype(np.float32))
    ex.train_step()
    assert np.isfinite(m.get_perf_metrics().get_loss())


def test_loss_threshold_clamps_predictions_and_gradient():
    """--loss-threshold t: predictions clamped to [t, 1-t], no gradient through clamped ones."""
    from flexmi.core.loss_metrics import NUM_SLOTS, loss_and_metrics_torch
    from flexmi.core.types import LossType
    p = torch.tensor([[0.001], [0.3], [0.999], [0.6]])
    y = torch.tensor([[0.0], [1.0], [1.0], [0.0]])
    g = torch.empty_like(p)
    acc = torch.zeros(NUM_SLOTS)
    loss_and_metrics_torch(LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, p, y, g, 1.0, acc, 0xFF, clamp=0.01)
    assert g[0, 0] == 0.0 and g[2, 0] == 0.0
    assert torch.allclose(g[1], torch.tensor([0.3 - 1.0])) and torch.allclose(g[3], torch.tensor([0.6]))
    se = (0.01 - 0.0) ** 2 + (0.3 - 1) ** 2 + (0.99 - 1) ** 2 + 0.6 ** 2
    assert abs(acc[4].item() - se) < 1e-6


def test_loss_threshold_model_level():
    from flexmi.models.dlrm import DLRMConfig
    dcfg = DLRMConfig(8, [20, 20], [13, 8], [24, 1], 1, -1, -1, 0.0, "cat", "", -1, "mse", "lt")
    m, ex, d, s = _dlrm_model(dcfg, 8, lt=0.25)
    assert m.loss_threshold == 0.25
    rng = np.random.RandomState(0)
    ex.scatter_from_host(d, rng.rand(*d.dims).astype(np.float32))
    for t in s:
        ex.scatter_from_host(t, rng.randint(0, 20, t.dims).astype(np.int64))
    ex.scatter_from_host(m.get_label_tensor(), rng.randint(0, 2, (8, 1)).astype(np.float32))
    ex.train_step()
    assert np.isfinite(m.get_perf_metrics().get_loss())


@pytest.mark.parametrize("gpus", [2, 4, 8])
def test_dlrm_strategy_hbm_balanced(gpus):
    """The default multi-GPU plan of the MLPerf table set: the ~40 M-row tables split on the
    parameter dim over all GPUs, the rest table-wise; per-GPU table bytes within 2x of each other
    (table-wise only at 8 GPUs: 20.9 GB vs 0.27 GB)."""
    from flexmi.core import FFConfig, FFModel
    from flexmi.models.dlrm import DLRMConfig, build_dlrm, dlrm_strategy, strategy_table_bytes
    cfg = FFConfig()
    cfg.batchSize, cfg.device = 64, "cpu"
    m = FFModel(cfg)
    build_dlrm(m, DLRMConfig.preset("mlperf"))
    st = dlrm_strategy(m, gpus)
    assert len(st) == 26
    per = strategy_table_bytes(m, st, gpus)
    assert abs(sum(per) - 187767399 * 128 * 4) / sum(per) < 1e-9
    assert max(per) / min(per) < 2.0, per
    assert max(per) < 288e9 * 0.5
