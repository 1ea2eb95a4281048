"""bench.py's --gpus launcher (config 5: one process per GPU).

The driver may run `python bench.py --gpus N` with no WORLD_SIZE (then bench.py starts the N ranks
itself) or under torchrun (WORLD_SIZE set, and it must equal --gpus).  These tests run on the CPU:
the decision table, and a real 2-rank spawn whose ranks rendezvous over gloo on 127.0.0.1 and
all-reduce (--launch-selftest stops before any GPU work).
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launch_mode_decision():
    assert bench.launch_mode(1, {}) == "run"
    assert bench.launch_mode(2, {}) == "spawn"
    assert bench.launch_mode(8, {"WORLD_SIZE": ""}) == "spawn"
    assert bench.launch_mode(8, {"WORLD_SIZE": "8", "RANK": "3"}) == "run"
    assert bench.launch_mode(1, {"WORLD_SIZE": "1"}) == "run"
    with pytest.raises(SystemExit):
        bench.launch_mode(8, {"WORLD_SIZE": "1"})   # torchrun with 1 proc but --gpus 8
    with pytest.raises(SystemExit):
        bench.launch_mode(1, {"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit):
        bench.launch_mode(0, {})


def _clean_env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR")}
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_spawned_ranks_rendezvous(n):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                        "--launch-selftest"], env=_clean_env(), capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 alone prints
    d = json.loads(lines[0])
    assert d == {"n_gpus": n, "rank_sum": n * (n - 1) // 2, "ranks": n, "master": "127.0.0.1"}


def test_world_size_mismatch_fails_nonzero():
    env = dict(_clean_env(), WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--launch-selftest"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=1 but --gpus 2" in r.stderr
