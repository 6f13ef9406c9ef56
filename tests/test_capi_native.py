"""The CPython-free native C API (csrc/capi/flexmi_native_c.h, flexmi/libflexmi_native_c.so): a C
program (tests/capi/native_demo.c) compiled with gcc drives the strategy codec (incl. the
reference's shipped dlrm_strategy_8embs_8gpus.pb), the sharding algebra, the simulator + MCMC
search, the HDF5 reader, the batch loader ring, the CPU embedding kernels and the graph planner -- and the library
must not link libpython."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "flexmi", "libflexmi_native_c.so")
REF_PB = "/root/reference/src/runtime/dlrm_strategy_8embs_8gpus.pb"


@pytest.fixture(scope="module")
def demo(tmp_path_factory):
    if not os.path.exists(LIB) or shutil.which("gcc") is None:
        pytest.skip("native C API library or gcc not available")
    d = tmp_path_factory.mktemp("capi_native")
    exe = str(d / "native_demo")
    subprocess.run(["gcc", "-O2", "-std=c11", f"-I{ROOT}/csrc/capi", os.path.join(ROOT, "tests", "capi", "native_demo.c"),
                    f"-L{ROOT}/flexmi", "-lflexmi_native_c", f"-Wl,-rpath,{ROOT}/flexmi", "-lm", "-o", exe],
                   check=True, capture_output=True)
    return d, exe


def test_native_c_api_has_no_python_dependency():
    if not os.path.exists(LIB):
        pytest.skip("not built")
    deps = subprocess.run(["ldd", LIB], capture_output=True, text=True).stdout
    assert "python" not in deps.lower(), deps
    syms = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    assert sum(1 for l in syms.splitlines() if " T fmn_" in l) >= 40


def test_native_c_program(demo):
    from flexmi.utils.hdf5 import write_h5
    d, exe = demo
    rng = np.random.RandomState(0)
    x = rng.rand(20, 13).astype(np.float32)
    h5 = str(d / "d.h5")
    write_h5(h5, {"X_int": x, "y": rng.rand(20).astype(np.float32)})
    args = [exe, str(d), h5] + ([REF_PB] if os.path.exists(REF_PB) else [])
    p = subprocess.run(args, capture_output=True, text=True, timeout=120, env=dict(os.environ, PYTHONHOME="/nonexistent"))
    assert p.returncode == 0, p.stdout + p.stderr
    out = p.stdout
    for area in ("strategies", "sharding", "simulator", "hdf5", "loader", "embedding", "planner"):
        assert f"ok {area}" in out, out
    s = float(out.split("X_int[3:5] sum")[1].split()[0])
    assert abs(s - float(x[3:5].sum())) < 1e-4
    assert "ALL OK" in out
