"""bench.py's multi-GPU plumbing on the CPU: `bench.py --gpus N` started bare
(no WORLD_SIZE) must start N ranks itself through torch.distributed.run and
forward rank 0's JSON line; under a launcher (WORLD_SIZE set) it must not
spawn again.  --dry-run keeps every rank off the GPU (gloo rendezvous and one
all-reduce only)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.strip().startswith("{")]


def test_launcher_cmd_plumbing():
    import bench
    cmd = bench.launcher_cmd(8, ["--gpus", "8", "--steps", "5"], 29555)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"]
    assert cmd[-5].endswith("bench.py")


@pytest.mark.parametrize("n,config,rows", [(2, "c2", 1_000_000_000), (4, "c5", 1_250_000_000)])
def test_bare_gpus_n_spawns_n_ranks(n, config, rows):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--config", config,
                        "--dry-run"], capture_output=True, text=True, timeout=180, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout  # only rank 0 prints, and the launcher forwards exactly that line
    d = lines[0]
    assert d["n_gpus"] == n
    assert d["rank_id_sum"] == n * (n + 1) // 2  # every rank joined the all-reduce
    assert d["config"]["rows_per_gpu"] == rows
    assert d["config"]["parallelism"] == f"row-range shards x{n}"


def test_under_launcher_does_not_respawn():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "[launcher]" not in p.stderr
    assert _json_lines(p.stdout)[0]["n_gpus"] == 1
