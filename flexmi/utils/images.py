"""Image input pipeline: decode -> resize -> (GPU) normalize, straight into the input shard.

Reference: ``UtilityTasks::load_images_task`` (libjpeg decode + CPU nearest-neighbour resize into a
CHW uint8 region) and ``normalize_images_task`` / ``apply_normalize`` (GPU, ``x / 256 - mean`` over
``std`` with the ImageNet constants), ``src/runtime/model.cu:56-164``; the per-shard image / label
regions of ``include/model.h`` (``DataLoadMeta``: file names + labels of one shard).

flexmi: every rank decodes only the rows of ITS shard of the image input (the tensor's home
layout), in a thread pool (PIL's decoders release the GIL), resizes with the reference's
nearest-neighbour sampling (``round(y * scale)`` clamped to the last row/column) in HWC order --
no host transpose -- and ships the uint8 batch to the GPU, where ONE kernel
(``csrc/kernels/image.hip``) converts HWC -> CHW, scales and normalizes into the executor's input
buffer (fp32 or bf16).  3 bytes per pixel cross PCIe instead of 12.  CPU runs use the same math in
torch.
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
IMAGE_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


def list_image_folder(root):
    """ImageNet-style folder: one sub-directory per class (sorted names -> label ids).
    Returns (files, labels, classes)."""
    classes = sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
    files, labels = [], []
    for ci, c in enumerate(classes):
        for f in sorted(os.listdir(os.path.join(root, c))):
            if f.lower().endswith(IMAGE_EXTENSIONS):
                files.append(os.path.join(root, c, f))
                labels.append(ci)
    return files, np.asarray(labels, dtype=np.int32), classes


def roundf(x: np.ndarray) -> np.ndarray:
    """C ``roundf`` of float32 values (half away from zero) as int64.  The +-0.5 is added in
    float64, where it is exact for every float32 input: in float32, x = 0.5 - 2**-25 would give
    x + 0.5 = 1.0 by ties-to-even and round up, while roundf gives 0."""
    xd = np.asarray(x, dtype=np.float32).astype(np.float64)
    return np.trunc(xd + np.copysign(0.5, xd)).astype(np.int64)


def nearest_resize_hwc(img: np.ndarray, height: int, width: int) -> np.ndarray:
    """The reference's nearest-neighbour sampling (``model.cu:56-74``): source row
    ``min(roundf(y * scale), oh - 1)`` with a float32 ``scale = oh / h`` and roundf's half-away-
    from-zero rounding (not numpy's half-to-even), column likewise; HWC in, HWC out."""
    oh, ow = img.shape[:2]
    if (oh, ow) == (height, width):
        return img

    def src(n_out, n_in):
        scale = np.float32(n_in) / np.float32(n_out)
        pos = np.arange(n_out, dtype=np.float32) * scale   # the float32 product, as the reference
        return np.minimum(roundf(pos), n_in - 1)

    ys, xs = src(height, oh), src(width, ow)
    return img[ys[:, None], xs[None, :]]


def decode_image(path: str, height: int, width: int) -> np.ndarray:
    """Decode one file to uint8 RGB [height][width][3].  Non-RGB images are converted (the
    reference skips them)."""
    from PIL import Image
    with Image.open(path) as im:
        arr = np.asarray(im.convert("RGB"), dtype=np.uint8)
    return nearest_resize_hwc(arr, height, width)


def normalize_images(u8: torch.Tensor, out: torch.Tensor, mean=IMAGENET_MEAN, std=IMAGENET_STD):
    """uint8 [N][H][W][3] -> out [N][3][H][W] = (x / 256 - mean[c]) / std[c].  On the GPU one HIP
    kernel (layout change fused in); the extension must be present there."""
    if out.is_cuda:
        from flexmi.ops import _kernels as K
        K.C().image_normalize(u8.contiguous(), out, [float(m) for m in mean], [float(s) for s in std])
        return out
    x = u8.permute(0, 3, 1, 2).float() / 256.0
    m = torch.tensor(mean, dtype=torch.float32).view(1, 3, 1, 1)
    s = torch.tensor(std, dtype=torch.float32).view(1, 3, 1, 1)
    out.copy_((x - m) / s)
    return out


class ImageFolderLoader:
    """Image + label loader for an FFModel (the reference's ImageNet data loaders): each
    ``next_batch`` decodes this rank's rows of the next batch and writes the normalized images
    and labels into the executor's input / label shards.

    ``source``: a directory (one sub-directory per class) or a ``(files, labels)`` pair."""

    def __init__(self, ffmodel, image_tensor, label_tensor, source, shuffle=False, seed=0, threads=8,
                 mean=IMAGENET_MEAN, std=IMAGENET_STD):
        self.model = ffmodel
        self.image = image_tensor
        self.label = label_tensor
        if isinstance(source, (str, os.PathLike)):
            files, labels, self.classes = list_image_folder(source)
        else:
            files, labels = source
            self.classes = None
        if not files:
            raise ValueError("ImageFolderLoader: no images found")
        self.files = list(files)
        self.labels = np.asarray(labels, dtype=np.int32)
        n, c, h, w = image_tensor.dims
        if c != 3:
            raise ValueError("ImageFolderLoader: the image input must be [N][3][H][W]")
        self.batch_size, self.height, self.width = n, h, w
        self.mean, self.std = mean, std
        self.shuffle = shuffle
        self.rng = np.random.RandomState(seed)
        self.order = np.arange(len(self.files))
        self.next_index = 0
        self.pool = ThreadPoolExecutor(max_workers=max(1, threads))
        self._staging = None
        self._h2d_done = None
        self._next = None         # (batch ids, future of the decoded uint8 rows) of the NEXT batch

    def get_num_samples(self):
        return len(self.files)

    def reset(self):
        self.next_index = 0
        self._next = None
        if self.shuffle:
            self.rng.shuffle(self.order)

    def _batch_ids(self):
        if self.next_index + self.batch_size > len(self.files):
            self.reset()
        ids = self.order[np.arange(self.next_index, self.next_index + self.batch_size) % len(self.files)]
        self.next_index += self.batch_size
        return ids

    def _decode_rows(self, ids):
        """Decode a batch's rows in the thread pool; returns one future per row."""
        futs = [self.pool.submit(decode_image, self.files[i], self.height, self.width) for i in ids]
        return futs

    def next_batch(self, ffmodel=None):
        """Load the next batch.  The batch after it is decoded in the background (thread pool)
        while the caller trains on this one, so the host decode overlaps the GPU step."""
        m = ffmodel or self.model
        ex = m._ex()
        buf = ex.local_buffer(self.image)
        box = ex.home[self.image.guid].local_box(ex.rank) if buf is not None else None
        if self._next is None:
            ids = self._batch_ids()
            futs = self._decode_rows(ids[box[0][0]:box[0][1]]) if box is not None else []
        else:
            ids, futs = self._next
        nxt = self._batch_ids()
        self._next = (nxt, self._decode_rows(nxt[box[0][0]:box[0][1]]) if box is not None else [])
        if buf is not None:
            r0, r1 = box[0]
            u8 = torch.from_numpy(np.stack([f.result() for f in futs]))
            if buf.is_cuda:
                if self._staging is None or self._staging.shape != u8.shape:
                    self._staging = torch.empty(u8.shape, dtype=torch.uint8).pin_memory()
                    self._h2d_done = None
                if self._h2d_done is not None:      # the previous async H2D still reads the staging buffer
                    self._h2d_done.synchronize()
                self._staging.copy_(u8)
                u8 = self._staging.to(buf.device, non_blocking=True)
                self._h2d_done = torch.cuda.Event()
                self._h2d_done.record()
            full = tuple(box[1:]) == ((0, 3), (0, self.height), (0, self.width))
            if full and buf.is_contiguous():
                normalize_images(u8, buf, self.mean, self.std)
            else:   # a spatial / channel split of the image input: normalize, then take the box
                tmp = torch.empty((r1 - r0, 3, self.height, self.width), dtype=buf.dtype, device=buf.device)
                normalize_images(u8, tmp, self.mean, self.std)
                buf.copy_(tmp[(slice(None),) + tuple(slice(lo, hi) for lo, hi in box[1:])])
        lab = self.labels[ids].reshape((-1,) + tuple(self.label.dims[1:]))
        ex.load_batch(self.label, torch.from_numpy(lab.astype(np.int32)))

    def close(self):
        self.pool.shutdown(wait=False)
