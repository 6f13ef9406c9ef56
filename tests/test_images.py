"""Image input pipeline (flexmi/utils/images.py, csrc/kernels/image.hip): folder listing, the
reference's nearest-neighbour resize and /256 normalization (src/runtime/model.cu:56-164), the
loader feeding a CNN on CPU, and the HIP normalize kernel against the torch fp32 formula."""
import numpy as np
import pytest
import torch

from flexmi.utils import images as I


def _folder(tmp_path, n_per_class=3, classes=("cat", "dog"), size=(20, 30)):
    from PIL import Image
    rng = np.random.RandomState(0)
    for c in classes:
        d = tmp_path / c
        d.mkdir()
        for k in range(n_per_class):
            arr = rng.randint(0, 256, size + (3,), dtype=np.uint8)
            Image.fromarray(arr).save(d / f"{k}.png")
    return tmp_path


def _ref_normalize(u8):
    x = u8.permute(0, 3, 1, 2).double() / 256.0
    m = torch.tensor(I.IMAGENET_MEAN, dtype=torch.float64).view(1, 3, 1, 1)
    s = torch.tensor(I.IMAGENET_STD, dtype=torch.float64).view(1, 3, 1, 1)
    return (x - m) / s


def test_list_and_decode(tmp_path):
    root = _folder(tmp_path)
    files, labels, classes = I.list_image_folder(str(root))
    assert classes == ["cat", "dog"] and len(files) == 6 and labels.tolist() == [0, 0, 0, 1, 1, 1]
    img = I.decode_image(files[0], 8, 12)
    assert img.shape == (8, 12, 3) and img.dtype == np.uint8
    from PIL import Image
    full = np.asarray(Image.open(files[0]).convert("RGB"))
    # reference sampling: row roundf(y * 20/8) clamped, column roundf(x * 30/12) clamped
    # (half away from zero: x = 5 -> 12.5 -> 13)
    for y, x in [(0, 0), (3, 5), (7, 11)]:
        sy, sx = min(int(np.floor(y * 20 / 8 + 0.5)), 19), min(int(np.floor(x * 30 / 12 + 0.5)), 29)
        assert (img[y, x] == full[sy, sx]).all()


def test_normalize_cpu():
    u8 = torch.randint(0, 256, (2, 5, 7, 3), dtype=torch.uint8)
    out = torch.empty(2, 3, 5, 7)
    I.normalize_images(u8, out)
    torch.testing.assert_close(out.double(), _ref_normalize(u8), rtol=1e-6, atol=1e-6)


def test_loader_trains_cnn_cpu(tmp_path):
    from flexmi.core import FFConfig, FFModel, SGDOptimizer
    from flexmi.core.types import ActiMode, LossType, MetricsType, PoolType
    root = _folder(tmp_path, n_per_class=4, size=(24, 18))
    cfg = FFConfig()
    cfg.batchSize = 4
    m = FFModel(cfg)
    x = m.create_tensor([4, 3, 16, 16], name="img")
    c = m.conv2d(x, 4, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
    c = m.pool2d(c, 2, 2, 2, 2, 0, 0, PoolType.POOL_MAX)
    o = m.softmax(m.dense(m.flat(c), 2))
    m.optimizer = SGDOptimizer(m, 0.01)
    m.compile(m.optimizer, LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
    ex = m.init_layers()
    ld = I.ImageFolderLoader(m, x, m.get_label_tensor(), str(root), shuffle=True, seed=1, threads=2)
    assert ld.get_num_samples() == 8
    ld.next_batch()
    # the input shard holds the normalized decoded images of this batch
    ids = ld.order[:4]
    u8 = torch.from_numpy(np.stack([I.decode_image(ld.files[i], 16, 16) for i in ids]))
    torch.testing.assert_close(ex.local_buffer(x).double(), _ref_normalize(u8), rtol=1e-6, atol=1e-6)
    assert ex.local_buffer(m.get_label_tensor()).view(-1).tolist() == ld.labels[ids].tolist()
    for _ in range(3):
        ex.train_step()
        ld.next_batch()
    assert np.isfinite(m.get_perf_metrics().get_loss())
    ld.close()


@pytest.mark.gpu
@pytest.mark.parametrize("dt,W", [(torch.float32, 224), (torch.bfloat16, 224), (torch.float32, 13)])
def test_normalize_hip(gpu, dt, W):
    u8 = torch.randint(0, 256, (3, 11, W, 3), dtype=torch.uint8, device=gpu)
    out = torch.empty(3, 3, 11, W, dtype=dt, device=gpu)
    I.normalize_images(u8, out)
    ref = _ref_normalize(u8.cpu())
    tol = 1e-6 if dt == torch.float32 else 8e-3
    torch.testing.assert_close(out.double().cpu(), ref, rtol=tol, atol=tol)


def test_nearest_resize_rounds_half_away_from_zero():
    # 5 -> 2 columns / rows: scale 2.5, output 1 samples source 2.5 exactly.  The reference's
    # roundf (model.cu:64-66) picks 3; numpy's rint (half to even) would pick 2.
    img = np.arange(5 * 5 * 3, dtype=np.uint8).reshape(5, 5, 3)
    out = I.nearest_resize_hwc(img, 2, 2)

    def ref_idx(n_out, n_in):
        scale = np.float32(n_in) / np.float32(n_out)
        return [min(int(np.floor(np.float32(i) * scale + np.float32(0.5))), n_in - 1) for i in range(n_out)]

    ys, xs = ref_idx(2, 5), ref_idx(2, 5)
    assert ys == [0, 3]
    np.testing.assert_array_equal(out, img[np.ix_(ys, xs)])
    # a generic shrink/enlarge keeps the min(.., n-1) clamp
    big = I.nearest_resize_hwc(img, 7, 11)
    assert big.shape == (7, 11, 3)
    np.testing.assert_array_equal(big[-1, -1], img[4, 4])


def test_roundf_near_half():
    """C roundf on float32: a value one ulp below k + 0.5 rounds DOWN (float32 x + 0.5 would
    tie-to-even up to k + 1), exact halves round away from zero."""
    import math
    below = np.nextafter(np.float32(0.5), np.float32(0.0))     # 0.5 - 2**-25
    vals = np.array([below, 0.5, 1.5, 2.5, np.nextafter(np.float32(2.5), np.float32(0.0)), 0.0, 3.49999],
                    dtype=np.float32)
    got = I.roundf(vals)
    # reference: exact decimal rounding of the float32 value, half away from zero
    want = [int(math.floor(float(v) + 0.5)) if float(v) - math.floor(float(v)) != 0.5 else int(math.floor(float(v))) + 1
            for v in vals]
    assert got.tolist() == want == [0, 1, 2, 3, 2, 0, 3]
    assert np.float32(below) + np.float32(0.5) == np.float32(1.0)   # the float32 pitfall it avoids
