"""Race detection / sanitizers for the native runtime: the C++ components that have
no GPU dependency -- strategy .pb codec, sharding algebra, threaded data-loader ring -- are built
into a standalone self-test (csrc/tests/native_selftest.cc) under AddressSanitizer +
UndefinedBehaviorSanitizer and under ThreadSanitizer, and run on the host."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = ["csrc/tests/native_selftest.cc", "csrc/runtime/shard.cc", "csrc/runtime/strategy_pb.cc",
        "csrc/runtime/loader.cc"]


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_native_runtime_under_sanitizer(tmp_path, san):
    if shutil.which("g++") is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-pthread",
           "-I" + os.path.join(ROOT, "csrc", "runtime")] + [os.path.join(ROOT, s) for s in SRCS] + ["-o", exe]
    if "undefined" in san:
        cmd.insert(5, "-fno-sanitize-recover=undefined")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "native selftest ok" in r.stdout, (r.stdout[-2000:], r.stderr[-6000:])
