"""bench.py's rank launch (no GPU): `--gpus N` without a launcher starts N
rank processes itself, a launcher whose WORLD_SIZE differs from --gpus is
refused, and the RCCL-id hand-over reaches every spawned rank.  --dry-run
stops each rank before its first HIP call."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

BENCH = os.path.join(REPO, "bench.py")


def _clean_env():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT", "RTAMD_RUN_ID",
              "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=_clean_env(), cwd=REPO)
    assert r.returncode == 0, r.stderr
    views = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    assert sorted(v["rank"] for v in views) == list(range(n))
    assert all(v["world"] == n and v["local_rank"] == v["rank"] and v["id_ok"] for v in views)


def test_single_gpu_runs_in_process():
    r = subprocess.run([sys.executable, BENCH, "--dry-run"], capture_output=True, text=True, timeout=120,
                       env=_clean_env(), cwd=REPO)
    assert r.returncode == 0, r.stderr
    (v,) = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    assert (v["rank"], v["world"]) == (0, 1)


def test_launcher_world_must_match_gpus():
    env = dict(_clean_env(), RANK="0", WORLD_SIZE="2", LOCAL_RANK="0", LOCAL_WORLD_SIZE="2", MASTER_PORT="1")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=env, cwd=REPO)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr
    assert not r.stdout.strip()


def test_multi_node_world_is_refused():
    env = dict(_clean_env(), RANK="0", WORLD_SIZE="2", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1", MASTER_PORT="1")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=env, cwd=REPO)
    assert r.returncode != 0 and "LOCAL_WORLD_SIZE" in r.stderr
