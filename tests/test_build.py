"""Build checks that need no GPU: both native extensions load (all symbols resolve) and expose
the kernels the framework calls."""
import subprocess


def test_hip_extension_loads(native):
    import torch  # noqa: F401  (libtorch must be loaded first)
    import flexmi._C as C
    assert C.arch == "gfx950"
    for name in ("gemm", "embedding_fwd_multi", "embedding_bwd_multi", "dot_fwd", "dot_bwd", "sgd", "adam", "loss",
                 "im2col", "col2im", "transpose_batched", "pool_fwd", "pool_bwd", "bn_fwd", "bn_bwd", "skinny_fwd",
                 "skinny_bwd", "multi_copy", "softmax", "dropout", "permute", "init_fill"):
        assert hasattr(C, name), name
    out = subprocess.run(["nm", "-D", "--undefined-only", C.__file__], capture_output=True, text=True).stdout
    assert "fm_" not in out, "unresolved kernel launcher symbols:\n" + out


def test_native_runtime_loads(native):
    import flexmi._native as N
    for name in ("load_strategy", "save_strategy", "encode_strategy", "decode_strategy", "Simulator"):
        assert hasattr(N, name), name
