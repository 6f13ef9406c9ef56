"""``python -m flexmi.run`` -- the ``flexflow_python`` launcher (reference ``python/main.cc:47-100``,
``python/flexflow/core/flexflow_top.py``).

    python -m flexmi.run [-ll:gpu N | --nproc N] [--nodes M --node-rank R --master HOST] script.py [args]

The reference started one Legion process whose Python top-level task ran the script, with
``-ll:gpu N`` GPUs inside it.  flexmi is SPMD: ``N`` processes (one per GPU) each run the script;
the launcher is ``torch.distributed.run`` with the rendezvous on 127.0.0.1 for a single node.
``-ll:gpu N`` stays in the script's argv (FFConfig reads it as workersPerNode); other Legion
flags (``-ll:fsize``, ``-ll:zsize``, ``-ll:py``, ``-lg:*``, ``-dm:*``) are accepted and dropped.
With N == 1 the script runs in this process (``runpy``), like ``flexflow_python script.py``.
"""
from __future__ import annotations

import os
import runpy
import socket
import subprocess
import sys

_LEGION_VALUED = ("-ll:fsize", "-ll:zsize", "-ll:py", "-ll:cpu", "-ll:util", "-ll:csize", "-ll:dma",
                  "-ll:bgwork", "-ll:ahandlers", "-ll:pyimport")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def parse(argv):
    nproc, nodes, node_rank, master = 1, 1, 0, "127.0.0.1"
    out, script, i = [], None, 0
    while i < len(argv):
        a = argv[i]
        if script is None and a in ("--nproc", "-n"):
            nproc = int(argv[i + 1]); i += 2; continue
        if script is None and a == "--nodes":
            nodes = int(argv[i + 1]); i += 2; continue
        if script is None and a == "--node-rank":
            node_rank = int(argv[i + 1]); i += 2; continue
        if script is None and a == "--master":
            master = argv[i + 1]; i += 2; continue
        if a == "-ll:gpu":
            nproc = int(argv[i + 1])
            out += [a, argv[i + 1]]; i += 2; continue
        if a in _LEGION_VALUED:
            i += 2; continue
        if a.startswith(("-lg:", "-dm:", "-hl:")):
            i += 1 + (i + 1 < len(argv) and not argv[i + 1].startswith("-")); continue
        if script is None and not a.startswith("-"):
            script = a; i += 1; continue
        out.append(a); i += 1
    return dict(nproc=nproc, nodes=nodes, node_rank=node_rank, master=master, script=script, args=out)


def main(argv=None):
    p = parse(list(sys.argv[1:] if argv is None else argv))
    if p["script"] is None:
        print(__doc__)
        return 2
    if p["nproc"] <= 1 and p["nodes"] <= 1:
        sys.argv = [p["script"]] + p["args"]
        sys.path.insert(0, os.path.dirname(os.path.abspath(p["script"])))
        runpy.run_path(p["script"], run_name="__main__")
        return 0
    cmd = [sys.executable, "-m", "torch.distributed.run", f"--nnodes={p['nodes']}",
           f"--nproc-per-node={p['nproc']}", f"--node-rank={p['node_rank']}",
           f"--master-addr={p['master']}", f"--master-port={os.environ.get('MASTER_PORT') or _free_port()}",
           p["script"]] + p["args"]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


if __name__ == "__main__":
    sys.exit(main())
