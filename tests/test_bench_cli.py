"""bench.py's multi-GPU launch contract on CPU: `--gpus N` without WORLD_SIZE re-launches itself
under torch.distributed.run with N ranks; the dry run takes the collective path of the sharded
step (histogram all-reduce + exact-size gather to rank 0) over gloo and prints one JSON line."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    return p


@pytest.mark.parametrize("n", [2, 3])
def test_bench_spawns_n_ranks(n):
    p = _run(["--gpus", str(n), "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == n
    assert d["collectives_ok"] is True
    assert sum(d["slab_planes"]) == 512 and all(z % 8 == 0 for z in d["slab_planes"])


def test_bench_rejects_world_mismatch():
    p = _run(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr
