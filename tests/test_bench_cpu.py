"""bench.py's launch contract on the CPU (no GPU): --gpus N spawns N ranks that join one process
group, and the row-sharded C5 config refuses a world it does not fit."""
from __future__ import annotations

import json
import os
import subprocess
import sys

from tests.conftest import ROOT


def _run(*args, timeout=180):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], cwd=ROOT, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_gpus_2_launches_two_ranks():
    p = _run("--gpus", "2", "--dry-run")
    assert p.returncode == 0, p.stderr[-2000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, p.stdout
    rec = json.loads(line[0])
    assert rec["n_gpus"] == 2 and rec["ranks_joined"] == 2


def test_c5_refuses_one_gpu_cleanly():
    """C5's planned per-rank HBM (bench.sharded_bytes_per_gpu: the buffers the pipelined row-sharded step
    allocates) exceeds one GPU's budget below 8 ranks: refused before anything touches a GPU."""
    for g in ("1", "4"):
        p = _run("--config", "c5", "--gpus", g, *(["--dry-run"] if g != "1" else []))
        assert p.returncode != 0, (g, p.stderr[-2000:])  # 2 (one rank) / the launcher's failure (ranks)
        assert "needs >= 8 GPUs" in p.stderr
        assert not any(x.startswith("{") for x in p.stdout.splitlines())


def test_c5_world8_dry_run_accepted():
    p = _run("--config", "c5", "--gpus", "8", "--dry-run")
    assert p.returncode == 0, p.stderr[-2000:]
    rec = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][0])
    assert rec["ranks_joined"] == 8 and rec["mode"] == "sharded" and rec["min_gpus"] == 8


def test_cpu_extrapolated_baseline_small():
    """The C4 CPU-baseline extrapolation on a small graph: the oracle step at two edge subsamples, then
    the remaining edges at the measured A . X per-edge cost (never below the larger measured step)."""
    import importlib

    sys.path.insert(0, str(ROOT))
    bench = importlib.import_module("bench")
    graph = importlib.import_module(bench.PKG + ".graph")
    U, E, inter, trip = graph.synthetic_ckg(4000, 30000, seed=3)
    lay = graph.build_layout(U, E, inter, trip)
    cfg = dict(dim=16, layers=[16, 8], batch=32, workload="tiny")
    rec = bench.cpu_extrapolated(lay, cfg, fracs=(0.2, 0.5))
    assert rec["extrapolated"] and rec["kind"] == "port" and rec["value"] > 0
    assert rec["per_edge_s"] >= 0 and rec["ms_per_step"] > 0
    assert "A.X per-edge cost" in rec["sample"]
