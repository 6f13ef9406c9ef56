"""flexmi.cli: the DLRM strategy generator reproduces the reference's shipped strategy files
(src/runtime/dlrm_strategy_*.pb, decoded configs equal), the hetero generator, and the
standalone simulator / search commands."""
import json
import os

import pytest

from flexmi.cli import main
from flexmi.parallel.layout import ParallelConfig
from flexmi.parallel.strategy import load_strategies_from_file

REF = "/root/reference/src/runtime"


@pytest.mark.parametrize("name,emb,gpus", [("8embs_8gpus", 8, 8), ("16embs_8gpus", 16, 8), ("16embs_16gpus", 16, 16)])
def test_gen_dlrm_matches_shipped_files(tmp_path, name, emb, gpus):
    out = str(tmp_path / "s.pb")
    assert main(["gen-dlrm", "--gpus", str(gpus), "--emb", str(emb), "-o", out]) == 0
    got = load_strategies_from_file(out)
    ref_file = os.path.join(REF, f"dlrm_strategy_{name}.pb")
    if not os.path.exists(ref_file):
        pytest.skip("reference strategy files not available")
    assert got == load_strategies_from_file(ref_file)
    assert os.path.getsize(out) == os.path.getsize(ref_file)


def test_gen_dlrm_hetero(tmp_path):
    out = str(tmp_path / "h.pb")
    assert main(["gen-dlrm-hetero", "--emb", "8", "-o", out]) == 0
    st = load_strategies_from_file(out)
    assert all(st[f"embedding{i}"].device_type == ParallelConfig.CPU for i in range(8))
    assert st["linear"].device_ids == [0] and st["linear"].device_type == ParallelConfig.GPU


def test_simulate_and_search_cli(tmp_path, capsys):
    tr = str(tmp_path / "t.json")
    assert main(["simulate", "--model", "alexnet", "--small", "--gpus", "4", "--trace", tr]) == 0
    rec = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert rec["predicted_ms"] > 0 and abs(rec["speedup_vs_dp"] - 1.0) < 1e-6
    assert json.load(open(tr))["traceEvents"]
    pb = str(tmp_path / "best.pb")
    assert main(["search", "--model", "alexnet", "--small", "--gpus", "4", "--budget", "200", "--export", pb]) == 0
    out = capsys.readouterr().out.strip().splitlines()
    rec = json.loads([ln for ln in out if ln.startswith("{")][-1])
    assert rec["best_ms"] <= rec["dp_ms"] + 1e-9
    assert load_strategies_from_file(pb)
