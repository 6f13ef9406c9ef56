"""Register-allocation guard for the hot fp32 GEMM kernel: the split-bf16 kernel
(csrc/kernels/gemm_x3.hip) runs at one block of 8 waves per CU with ~220-240 VGPRs, so any change
that pushes it over 256 spills to scratch and silently costs 2-3x (a timing knob with runtime
branches did exactly that: 221 spilled VGPRs, 8192x1024x1024 dW 99 -> 262 us).  Compiles the file
for gfx950 (no GPU needed) and checks hipcc's resource report for every instantiation."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_split_gemm_kernels_do_not_spill(tmp_path):
    src = os.path.join(ROOT, "csrc", "kernels", "gemm_x3.hip")
    out = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", src, "-o", str(tmp_path / "x3.o"),
                          "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-2000:]
    names = re.findall(r"Function Name: (\S+)", out.stderr)
    spills = [int(v) for v in re.findall(r"VGPRs Spill: (\d+)", out.stderr)]
    scratch = [int(v) for v in re.findall(r"ScratchSize \[bytes/lane\]: (\d+)", out.stderr)]
    assert names and len(spills) == len(names) == len(scratch)
    bad = [(n, s, c) for n, s, c in zip(names, spills, scratch) if s or c]
    assert not bad, bad
