"""A/B: the owner-computes (claim / dup / owner) embedding backward vs per-lookup atomics for every
non-tiny table (Embedding.CLAIM) on the bench.

    python tools/ab_emb_claim.py 0|1
"""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
claim = sys.argv[1] == "1"
import flexmi.ops.embedding as E  # noqa: E402

E.Embedding.CLAIM = claim
sys.argv = ["bench.py", "--steps", "50", "--warmup", "10", "--no-native"] + sys.argv[2:]
runpy.run_path("bench.py", run_name="__main__")
