"""Register-allocation guard for the hot GEMM kernels: the split-bf16 fp32 kernel
(csrc/kernels/gemm_x3.hip) runs at one block of 8 waves per CU with ~110-180 VGPRs, so any change
that pushes it over 256 spills to scratch and silently costs 2-3x (a timing knob with runtime
branches did exactly that: 221 spilled VGPRs, 8192x1024x1024 dW 99 -> 262 us); the native fp32
kernels (gemm_f32.hip) likewise.  Compiles both files for gfx950 concurrently (no GPU needed) and
checks hipcc's resource report for every instantiation: no spill, no scratch."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_big_gemm_kernels_do_not_spill(tmp_path):
    procs = {}
    for name in ("gemm_x3", "gemm_f32"):
        src = os.path.join(ROOT, "csrc", "kernels", name + ".hip")
        procs[name] = subprocess.Popen([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", src, "-o",
                                        str(tmp_path / (name + ".o")), "-Rpass-analysis=kernel-resource-usage"],
                                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    for name, p in procs.items():
        _, err = p.communicate(timeout=900)
        assert p.returncode == 0, err[-2000:]
        names = re.findall(r"Function Name: (\S+)", err)
        spills = [int(v) for v in re.findall(r"VGPRs Spill: (\d+)", err)]
        scratch = [int(v) for v in re.findall(r"ScratchSize \[bytes/lane\]: (\d+)", err)]
        assert names and len(spills) == len(names) == len(scratch), name
        assert not [(n, s) for n, s in zip(names, spills) if s], (name, "VGPR spill")
        assert not [(n, c) for n, c in zip(names, scratch) if c], (name, "scratch")
