#!/usr/bin/env python3
"""Per-dispatch timeline of the last full training step in a rocprofv3 rocpd database
(kernels between the last two dispatches of the step's first kernel): start / end offset (us)
from the step's first kernel, HIP queue index, duration, launch geometry, name.
usage: prof_step.py run_results.db [first_kernel_substring[|alternative...]]"""
import sqlite3
import sys


def main(path, first="fm_emb_fwd_multi"):
    c = sqlite3.connect(path)
    cols = {r[1] for r in c.execute("pragma table_info(kernels)")}
    qcol = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else "0")
    rows = list(c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x, lds_size, vgpr_count, start, "
                          f"{qcol} from kernels order by start"))
    keys = first.split("|")   # alternatives, e.g. "fm_emb_fwd_multi<float|fm_emb_fwd_split<float"
    idx = [i for i, r in enumerate(rows) if any(k in r[0] for k in keys)]
    s, e = idx[-2], idx[-1]
    tot = 0
    t0 = rows[s][8]
    queues = {}
    for r in rows[s:e]:
        n = r[0].replace("(anonymous namespace)::", "")[:80]
        tot += r[1]
        q = queues.setdefault(r[9], len(queues))
        # start / end offsets from the step's first kernel and the queue (stream) index: kernels on
        # different queues with overlapping [start, end) ran concurrently
        print(f"{(r[8] - t0) / 1e3:8.2f} {(r[8] + r[1] - t0) / 1e3:8.2f} q{q} {r[1] / 1e3:7.2f}us "
              f"grid={r[2] // max(1, r[5])}x{r[3]}x{r[4]} wg={r[5]} lds={r[6]} vgpr={r[7]}  {n}")
    print(f"step kernel sum {tot / 1e3:.1f}us, span {(rows[e][8] - rows[s][8]) / 1e3:.1f}us")


if __name__ == "__main__":
    main(*sys.argv[1:])
