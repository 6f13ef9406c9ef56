#!/usr/bin/env python3
"""Build flexmi's native extensions IN-TREE with ninja (no hipify, gfx950 only).

  flexmi/_C*.so       HIP kernels (csrc/kernels/*.hip, hipcc --offload-arch=gfx950, no torch
                      headers) + torch/pybind11 bindings (csrc/bindings/hip_ops.cpp)
  flexmi/libflexmi_c.so  C API (csrc/capi/flexmi_c.h; embeds CPython for the model API)
  flexmi/libflexmi_native_c.so  native C API (csrc/capi/flexmi_native_c.h; C++ runtime, no Python)
  flexmi/_native*.so  C++ runtime: strategy .pb codec, sharding algebra, MI355X execution
                      simulator + MCMC search, data-loader ring (csrc/runtime/*.cc, g++ -O3,
                      pybind11; no GPU dependency -- usable on the CPU box)

  flexmi/_cpu*.so     native CPU kernels (csrc/cpu/*.cc: embedding bag / gradient / sparse SGD,
                      AVX2 + ATen thread pool) for the CPU backend and host-placed tables

Usage: python tools/build_ext.py [--only C|rt|cpu|native] [-j N] [--clean]
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "build")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
if ARCH != "gfx950":
    ARCH = "gfx950"  # MI355X only
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
TORCH_RUNTIME_SRCS = ("step_runner.cc",)   # csrc/runtime sources built into flexmi/_rt (torch + HIP)


def _torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(tdir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _py_includes():
    import pybind11
    return [sysconfig.get_paths()["include"], pybind11.get_include()]


def write_ninja(only=None):
    os.makedirs(BUILD, exist_ok=True)
    ext = sysconfig.get_config_var("EXT_SUFFIX")
    pyinc = " ".join(f"-I{p}" for p in _py_includes())
    lines = [
        "ninja_required_version = 1.5",
        f"hipcc = {ROCM}/bin/hipcc",
        "cxx = g++",
        f"hipflags = --offload-arch={ARCH} -O3 -std=c++17 -fPIC -Wno-unused-result -munsafe-fp-atomics "
        f"-mllvm -pragma-unroll-threshold=500000 -I{ROOT}/csrc/kernels",
        f"cxxflags = -O3 -std=c++17 -fPIC -Wall -Wno-sign-compare -I{ROOT}/csrc/runtime -I{ROOT}/csrc/sim {pyinc}",
        "rule hipcc",
        "  command = $hipcc $hipflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIPCC $in",
        "rule cxx",
        "  command = $cxx $cxxflags $extra -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule hiplink",
        "  command = $hipcc -shared -fPIC $in -o $out $ldflags",
        "  description = LINK $out",
        "rule cxxlink",
        "  command = $cxx -shared -fPIC $in -o $out $ldflags",
        "  description = LINK $out",
    ]
    targets = []
    if only in (None, "C"):
        tinc, tlib, abi = _torch_paths()
        incs = " ".join(f"-I{p}" for p in tinc)
        objs = []
        for src in sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip"))):
            o = os.path.join(BUILD, "k_" + os.path.basename(src).replace(".hip", ".o"))
            lines.append(f"build {o}: hipcc {src}")
            objs.append(o)
        b = os.path.join(BUILD, "hip_ops.o")
        bflags = (f"--offload-arch={ARCH} -O2 -std=c++17 -fPIC -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 "
                  f"-DTORCH_EXTENSION_NAME=_C -D_GLIBCXX_USE_CXX11_ABI={abi} {incs} {pyinc} -Wno-unused-result")
        lines.append(f"build {b}: hipcc {os.path.join(ROOT, 'csrc', 'bindings', 'hip_ops.cpp')}")
        lines.append(f"  hipflags = {bflags}")
        objs.append(b)
        out = os.path.join(ROOT, "flexmi", "_C" + ext)
        ld = f"-L{tlib} -Wl,-rpath,{tlib} -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -ltorch_python -L{ROCM}/lib -lamdhip64"
        lines.append(f"build {out}: hiplink {' '.join(objs)}")
        lines.append(f"  ldflags = {ld}")
        targets.append(out)
    if only in (None, "C", "rt"):
        # native step runner (csrc/runtime/step_runner.cc): host C++ against torch's c10d and the
        # HIP runtime API, compiled by g++ like torch itself so pybind11 shares torch's type
        # registry (the c10d ProcessGroup objects of torch.distributed pass straight through)
        tinc, tlib, abi = _torch_paths()
        incs = " ".join(f"-I{p}" for p in tinc)
        objs = []
        for name in TORCH_RUNTIME_SRCS:
            src = os.path.join(ROOT, "csrc", "runtime", name)
            o = os.path.join(BUILD, "rt_" + name.replace(".cc", ".o"))
            lines.append(f"build {o}: cxx {src}")
            lines.append(f"  extra = -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -DTORCH_EXTENSION_NAME=_rt "
                         f"-D_GLIBCXX_USE_CXX11_ABI={abi} {incs} -I{ROCM}/include -Wno-unused-parameter")
            objs.append(o)
        out = os.path.join(ROOT, "flexmi", "_rt" + ext)
        lines.append(f"build {out}: cxxlink {' '.join(objs)}")
        lines.append(f"  ldflags = -L{tlib} -Wl,-rpath,{tlib} -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip "
                     f"-ltorch_python -L{ROCM}/lib -Wl,-rpath,{ROCM}/lib -lamdhip64")
        targets.append(out)
    if only in (None, "cpu"):
        # native CPU kernels (csrc/cpu/*.cc): torch CPU extension, ATen intra-op thread pool
        tinc, tlib, abi = _torch_paths()
        incs = " ".join(f"-I{p}" for p in tinc)
        objs = []
        for src in sorted(glob.glob(os.path.join(ROOT, "csrc", "cpu", "*.cc"))):
            o = os.path.join(BUILD, "cpu_" + os.path.basename(src).replace(".cc", ".o"))
            lines.append(f"build {o}: cxx {src}")
            lines.append(f"  extra = -DTORCH_EXTENSION_NAME=_cpu -D_GLIBCXX_USE_CXX11_ABI={abi} {incs} "
                         f"-Wno-unused-parameter -fopenmp")
            objs.append(o)
        out = os.path.join(ROOT, "flexmi", "_cpu" + ext)
        lines.append(f"build {out}: cxxlink {' '.join(objs)}")
        lines.append(f"  ldflags = -L{tlib} -Wl,-rpath,{tlib} -lc10 -ltorch -ltorch_cpu -ltorch_python -fopenmp")
        targets.append(out)
    if only in (None, "native"):
        objs = []
        for src in sorted(glob.glob(os.path.join(ROOT, "csrc", "runtime", "*.cc")) +
                          glob.glob(os.path.join(ROOT, "csrc", "sim", "*.cc"))) + [
                os.path.join(ROOT, "csrc", "bindings", "native.cc")]:
            if not os.path.exists(src) or os.path.basename(src) in TORCH_RUNTIME_SRCS:
                continue
            o = os.path.join(BUILD, "n_" + os.path.basename(src).replace(".cc", ".o"))
            lines.append(f"build {o}: cxx {src}")
            objs.append(o)
        out = os.path.join(ROOT, "flexmi", "_native" + ext)
        lines.append(f"build {out}: cxxlink {' '.join(objs)}")
        lines.append("  ldflags = -pthread")
        targets.append(out)
        # native C API (csrc/capi/flexmi_native_c.h): the C++ runtime without Python
        nobjs = []
        for src in [os.path.join(ROOT, "csrc", "capi", "flexmi_native_c.cc"), os.path.join(ROOT, "csrc", "cpu", "emb_kernels.cc"),
                    os.path.join(ROOT, "csrc", "sim", "simulator.cc")] + [
                os.path.join(ROOT, "csrc", "runtime", n) for n in ("hdf5_lite.cc", "loader.cc", "planner.cc", "shard.cc", "strategy_pb.cc")]:
            o = os.path.join(BUILD, "nc_" + os.path.basename(src).replace(".cc", ".o"))
            lines.append(f"build {o}: cxx {src}")
            lines.append(f"  extra = -I{ROOT}/csrc/capi")
            nobjs.append(o)
        # the native model (csrc/runtime/native_model.cc) with its HIP engine (csrc/native/
        # native_hip.cc: flexmi's kernels + RCCL) -- libflexmi_kernels.so is the kernel objects
        # alone, no PyTorch
        for src in [os.path.join(ROOT, "csrc", "runtime", "native_model.cc"), os.path.join(ROOT, "csrc", "runtime", "host_comm.cc")]:
            o = os.path.join(BUILD, "nc_" + os.path.basename(src).replace(".cc", ".o"))
            lines.append(f"build {o}: cxx {src}")
            lines.append(f"  extra = -I{ROOT}/csrc/capi")
            nobjs.append(o)
        hip_o = os.path.join(BUILD, "nc_native_hip.o")
        lines.append(f"build {hip_o}: cxx {os.path.join(ROOT, 'csrc', 'native', 'native_hip.cc')}")
        lines.append(f"  extra = -D__HIP_PLATFORM_AMD__=1 -I{ROCM}/include -I{ROOT}/csrc/runtime")
        nobjs.append(hip_o)
        kobjs = [os.path.join(BUILD, "k_" + os.path.basename(src).replace(".hip", ".o"))
                 for src in sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")))]
        if only == "native":   # kernel objects come from the C target's rules otherwise
            for src in sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip"))):
                lines.append(f"build {os.path.join(BUILD, 'k_' + os.path.basename(src).replace('.hip', '.o'))}: hipcc {src}")
        klib = os.path.join(ROOT, "flexmi", "libflexmi_kernels.so")
        lines.append(f"build {klib}: hiplink {' '.join(kobjs)}")
        lines.append(f"  ldflags = -L{ROCM}/lib -Wl,-rpath,{ROCM}/lib -lamdhip64")
        targets.append(klib)
        nc = os.path.join(ROOT, "flexmi", "libflexmi_native_c.so")
        lines.append(f"build {nc}: cxxlink {' '.join(nobjs)} | {klib}")
        lines.append(f"  ldflags = -pthread -L{ROOT}/flexmi -Wl,-rpath,'$$ORIGIN' -lflexmi_kernels "
                     f"-L{ROCM}/lib -Wl,-rpath,{ROCM}/lib -lamdhip64 -lrccl -ldl")
        targets.append(nc)
        # C API (csrc/capi): embeds CPython, so it links libpython
        capi_src = os.path.join(ROOT, "csrc", "capi", "flexmi_c.cc")
        capi_o = os.path.join(BUILD, "capi_flexmi_c.o")
        pyver = sysconfig.get_config_var("LDVERSION") or sysconfig.get_python_version()
        pylib = sysconfig.get_config_var("LIBDIR")
        lines.append(f"build {capi_o}: cxx {capi_src}")
        lines.append(f"  extra = -I{ROOT}/csrc/capi")
        capi = os.path.join(ROOT, "flexmi", "libflexmi_c.so")
        lines.append(f"build {capi}: cxxlink {capi_o}")
        lines.append(f"  ldflags = -L{pylib} -lpython{pyver} -ldl -pthread")
        targets.append(capi)
    lines.append("default " + " ".join(targets))
    path = os.path.join(BUILD, "build.ninja")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return path


def build(only=None, jobs=None, verbose=False):
    path = write_ninja(only)
    cmd = ["ninja", "-f", path]
    j = jobs or int(os.environ.get("MAX_JOBS", "0") or 0) or min(16, os.cpu_count() or 4)
    cmd += ["-j", str(min(j, 16))]
    if verbose:
        cmd.append("-v")
    r = subprocess.run(cmd, cwd=BUILD)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed ({' '.join(cmd)})")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["C", "rt", "cpu", "native"], default=None)
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("-v", action="store_true")
    ap.add_argument("--clean", action="store_true")
    a = ap.parse_args()
    if a.clean:
        import shutil
        shutil.rmtree(BUILD, ignore_errors=True)
    build(a.only, a.j, a.v)


if __name__ == "__main__":
    main()
