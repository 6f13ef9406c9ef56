"""A/B: the count / update embedding backward (Embedding.COUNT + fm_embedding_set_bwd_mode(1)) on the bench.

    python tools/ab_emb_count.py 0|1
"""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mode = sys.argv[1] == "1"
import flexmi.ops.embedding as E
from flexmi.ops import _kernels as K
E.Embedding.COUNT = mode
K.C().embedding_set_bwd_mode(mode)
sys.argv = ["bench.py", "--steps", "50", "--warmup", "10", "--no-secondary", "--no-native"]
runpy.run_path("bench.py", run_name="__main__")
