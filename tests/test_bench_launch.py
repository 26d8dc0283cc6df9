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


def _bench_module():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _check_ranks_block(blk, world, H):
    assert blk["rccl_world"] == [world]
    assert len(blk["kernel_ms"]["per_rank"]) == world
    assert blk["kernel_ms"]["min"] <= blk["kernel_ms"]["max"]
    assert sum(blk["rows"]) == H
    for key in ("reduce_device", "verdict_wait_host"):
        assert len(blk["agreement_ms"][key]) == world
    assert len(blk["gather_ms"]["per_rank"]) == world and len(blk["gather_ms"]["last_chunk_per_rank"]) == world
    assert set(blk["placement_ms"]) == {"root_total", "root_last_chunk"}
    assert len(blk["call_ms"]) == world and len(blk["tail_ms"]) == world
    json.dumps(blk)   # (goes into the JSON line)


def test_ranks_block_schema_synthetic():
    """The N > 1 line's per-rank block from synthetic rank values (no GPU)."""
    b = _bench_module()
    world, H = 3, 50
    splits = [[1.5 + r, 0.01, 0.02, 0.1, 0.3 if r == 0 else 0.0, 0.03, 0.05 if r == 0 else 0.0, 0.04, world,
               [18, 16, 16][r]] for r in range(world)]
    blk = b.ranks_block([1.0, 1.2, 1.1], [0.05] * 3, splits)
    _check_ranks_block(blk, world, H)
    assert blk["kernel_ms"]["max"] == 1.2 and blk["placement_ms"]["root_total"] == 0.3


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 8])
def test_ranks_block_from_thread_ranks(gpu, world):
    """The same block from real rank splits: world concurrent ranks on one GPU
    through the product's dist_frame (rt_test_dist_threads)."""
    import numpy as np

    import scenes

    b = _bench_module()
    sc = gpu.load_scene_from_json_text(scenes.config_json(4, dpi=40)[0])
    W, H = sc.width, sc.height
    split = np.zeros((2, world, 10))
    out, rc, ms, msg = gpu.dist_threads(sc, W, H, 0, world, frames=2, split_out=split)
    assert (rc == 0).all(), msg
    last = split[1]
    blk = b.ranks_block([1.0] * world, [0.0] * world, [list(x) for x in last])
    _check_ranks_block(blk, world, H)
    assert blk["placement_ms"]["root_total"] > 0 and all(g > 0 for g in blk["gather_ms"]["per_rank"])
    assert all(c > 0 for c in blk["call_ms"])
