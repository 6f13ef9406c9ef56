"""Attach a host numpy array to a tensor and read it back (reference
examples/python/native/tensor_attach.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from common import header  # noqa: E402

import numpy as np  # noqa: E402
from flexmi.core import DataType, FFConfig, FFModel  # noqa: E402


def main():
    cfg = FFConfig()
    cfg.parse_args()
    header(cfg)
    model = FFModel(cfg)
    t = model.create_tensor([8, 3, 10, 10], DataType.DT_FLOAT)
    src = np.arange(8 * 3 * 10 * 10, dtype=np.float32).reshape(8, 3, 10, 10)
    t.attach_numpy_array(cfg, src)
    print("mapped:", t.is_mapped())
    got = t.get_array(cfg, DataType.DT_FLOAT)
    assert np.array_equal(np.asarray(got).reshape(src.shape), src)
    t.detach_numpy_array(cfg)
    print("attach/detach ok", got.shape)


if __name__ == "__main__":
    print("tensor attach")
    main()
