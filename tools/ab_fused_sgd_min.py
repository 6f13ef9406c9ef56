"""A/B: the smallest weight (elements) whose SGD is fused into its dW GEMM (executor FUSED_SGD_MIN) on the bench.

    python tools/ab_fused_sgd_min.py <elements>
"""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import flexmi.runtime.executor as E  # noqa: E402

E.FUSED_SGD_MIN = int(sys.argv[1])
sys.argv = ["bench.py", "--steps", "50", "--warmup", "10", "--no-native"]
runpy.run_path("bench.py", run_name="__main__")
