"""bench.py's process model, without a GPU: `--gpus N` outside torchrun starts N
ranks (torch.distributed.run on 127.0.0.1) that split one global batch into
cell-balanced contiguous shards; a mismatched --gpus under torchrun fails."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=300, env=e)


def test_gpus_flag_spawns_ranks():
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert all(x["world"] == 2 and x["gather"] for x in lines)
    shards = sorted(tuple(x["shard"]) for x in lines)
    assert shards == [(0, 1_000_000), (1_000_000, 2_000_000)]      # weak: 1M pairs per GPU


def test_strong_workload_shards_one_global_batch():
    r = _run(["--gpus", "4", "--dry-run", "--workload", "semi"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    shards = sorted(tuple(x["shard"]) for x in lines)
    assert shards[0][0] == 0 and shards[-1][1] == 10_000_000 and len(shards) == 4
    assert all(b - a == 2_500_000 for a, b in shards)


def test_gpus_mismatch_under_torchrun_fails():
    r = _run(["--gpus", "8", "--dry-run"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
