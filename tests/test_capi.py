"""C API (csrc/capi/flexmi_c.h; parity with the reference's python/flexflow_c.h): a C program
trains an MLP through the embedded runtime, and the same library works in-process via ctypes."""
import ctypes
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "flexmi", "libflexmi_c.so")


@pytest.mark.skipif(not shutil.which("gcc"), reason="needs a C compiler")
def test_c_program_trains_mlp(tmp_path):
    assert os.path.exists(LIB), "build the C API first (tools/build_ext.py)"
    exe = str(tmp_path / "mlp_c")
    subprocess.run(["gcc", os.path.join(ROOT, "apps", "c", "mlp_c.c"), f"-I{ROOT}/csrc/capi", f"-L{ROOT}/flexmi",
                    "-lflexmi_c", f"-Wl,-rpath,{ROOT}/flexmi", "-o", exe], check=True)
    r = subprocess.run([exe, "-b", "32", "-e", "6", "--device", "cpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    acc = float(r.stdout.split("accuracy")[1].split()[0])
    assert acc > 50.0, r.stdout
    assert "dense1 kernel elements 1024" in r.stdout and "THROUGHPUT" in r.stdout


def test_capi_in_process_ctypes():
    lib = ctypes.CDLL(LIB)
    lib.flexmi_init.argtypes = [ctypes.c_int, ctypes.c_void_p]
    assert lib.flexmi_init(0, None) == 0
    lib.flexmi_config_create.restype = ctypes.c_void_p
    lib.flexmi_config_get_batch_size.argtypes = [ctypes.c_void_p]
    lib.flexmi_config_set_batch_size.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.flexmi_config_destroy.argtypes = [ctypes.c_void_p]
    c = lib.flexmi_config_create()
    assert c
    assert lib.flexmi_config_get_batch_size(c) == 64          # reference default (model.cc:1274)
    assert lib.flexmi_config_set_batch_size(c, 96) == 0
    assert lib.flexmi_config_get_batch_size(c) == 96
    lib.flexmi_model_create.restype = ctypes.c_void_p
    lib.flexmi_model_create.argtypes = [ctypes.c_void_p]
    lib.flexmi_tensor_create.restype = ctypes.c_void_p
    lib.flexmi_tensor_create.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                         ctypes.c_int, ctypes.c_char_p]
    lib.flexmi_model_add_relu.restype = ctypes.c_void_p
    lib.flexmi_model_add_relu.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p]
    lib.flexmi_tensor_get_dims.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    lib.flexmi_last_error.restype = ctypes.c_char_p
    m = lib.flexmi_model_create(c)
    dims = (ctypes.c_int * 2)(96, 7)
    t = lib.flexmi_tensor_create(m, 2, dims, 40, 1, b"x")
    assert t, lib.flexmi_last_error()
    r = lib.flexmi_model_add_relu(m, t, None)
    out = (ctypes.c_int * 4)()
    assert lib.flexmi_tensor_get_dims(r, out) == 2 and list(out[:2]) == [96, 7]
    # errors are reported, not fatal
    bad = lib.flexmi_tensor_create(m, 2, dims, 999, 1, b"y")
    assert not bad and b"DataType" in lib.flexmi_last_error()
    lib.flexmi_config_destroy(c)


@pytest.mark.skipif(not shutil.which("gcc"), reason="needs a C compiler")
def test_c_program_functional_layers_and_4d_loaders(tmp_path):
    """apps/c/cnn_c.c: conv2d / pool2d / flat / dense built with the *_no_inout entry points and
    connected by op_init_inout; dataloader_4d_create_v2 over host tensors with attached raw
    pointers, the random-data dataloader_4d_create, inline_map + get_raw_ptr_float, op_forward."""
    exe = str(tmp_path / "cnn_c")
    subprocess.run(["gcc", os.path.join(ROOT, "apps", "c", "cnn_c.c"), f"-I{ROOT}/csrc/capi", f"-L{ROOT}/flexmi",
                    "-lflexmi_c", f"-Wl,-rpath,{ROOT}/flexmi", "-o", exe], check=True)
    r = subprocess.run([exe, "-b", "16", "-e", "2", "--device", "cpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    loss = float(r.stdout.split("loss")[1].split()[0])
    assert 0 < loss < 5 and "is_mapped 1" in r.stdout and "THROUGHPUT" in r.stdout


def test_capi_reference_name_parity():
    """Every function of the reference's python/flexflow_c.h has a flexmi_ counterpart (the
    reference's commented-out model_add_mse_loss excepted)."""
    hdr = open(os.path.join(ROOT, "csrc", "capi", "flexmi_c.h")).read()
    ref = "/root/reference/python/flexflow_c.h"
    if not os.path.exists(ref):
        pytest.skip("reference header not present")
    import re
    names = set(re.findall(r"^(?!\s*//)\s*flexflow_([a-z0-9_]+)\(", open(ref).read(), re.M))
    names |= set(re.findall(r"^flexflow_([a-z0-9_]+)\(", open(ref).read(), re.M))
    missing = sorted(n for n in names if f"flexmi_{n}(" not in hdr and n != "model_add_mse_loss")
    assert not missing, missing
