"""bench.py's --gpus contract on the CPU (no GPU needed): a launcher's
WORLD_SIZE must equal --gpus, and --gpus N > 1 without a launcher spawns N
ranks instead of silently running one."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launch_plan():
    assert bench.launch_plan(1, {}) == ("run", 1)
    assert bench.launch_plan(4, {}) == ("spawn", 4)
    assert bench.launch_plan(2, {"WORLD_SIZE": "2"}) == ("run", 2)
    with pytest.raises(SystemExit, match="must agree"):
        bench.launch_plan(2, {"WORLD_SIZE": "3"})
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {})


def test_mismatched_world_fails_loudly():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "must agree" in r.stderr
