"""bench.py's multi-GPU plumbing on the CPU.

Default form (the product's path): `bench.py --gpus N` runs in ONE process that
opens devices 0..N-1 through the library's `gpu_devices` key (each listed
--shards-per-gpu times); under the driver's torch.distributed.run launch rank 0
drives every device and the other ranks only join the gloo barriers.
`--ranks`: `bench.py --ranks --gpus N` started bare (no WORLD_SIZE) starts N
ranks itself through torch.distributed.run and forwards rank 0's JSON line;
under a launcher (WORLD_SIZE set) it must not spawn again.  --dry-run keeps
every rank off the GPU (gloo rendezvous and one all-reduce only)."""
import json
import os
import subprocess
import sys
from types import SimpleNamespace

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.strip().startswith("{")]


def _bare_env():
    return {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}


def test_launcher_cmd_plumbing():
    import bench
    cmd = bench.launcher_cmd(8, ["--gpus", "8", "--steps", "5"], 29555)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"]
    assert cmd[-5].endswith("bench.py")


@pytest.mark.parametrize("gpus,spg,world,devices", [
    (1, 1, 1, [0]), (8, 1, 1, list(range(8))), (1, 2, 1, [0, 0]), (4, 2, 1, [0, 0, 1, 1, 2, 2, 3, 3]),
    (1, 1, 8, list(range(8))),  # the driver's launch: WORLD_SIZE decides the device count
])
def test_inlib_plan(gpus, spg, world, devices):
    import bench
    p = bench.inlib_plan(SimpleNamespace(gpus=gpus, shards_per_gpu=spg, rows=1_000_000_000), world)
    assert p["devices"] == devices
    assert p["nshards"] == len(devices)
    assert p["rows_total"] == 1_000_000_000 * p["ngpu"]  # weak scaling: 1e9 rows per GPU
    if len(devices) > 1:
        assert "gpu_devices=" + ",".join(map(str, devices)) in p["parallelism"]
        assert "in-library" in p["parallelism"]


@pytest.mark.parametrize("n,spg", [(4, 1), (2, 2)])
def test_bare_gpus_n_is_one_inlib_process(n, spg):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--shards-per-gpu",
                        str(spg), "--dry-run"], capture_output=True, text=True, timeout=180, env=_bare_env())
    assert p.returncode == 0, p.stderr[-2000:]
    assert "[launcher]" not in p.stderr  # no ranks spawned: the library shards in-process
    d = _json_lines(p.stdout)[0]
    assert d["mode"] == "in-library" and d["processes"] == 1 and d["n_gpus"] == n
    assert d["gpu_devices"] == [g for g in range(n) for _ in range(spg)]


@pytest.mark.parametrize("n,config,rows", [(2, "c2", 1_000_000_000), (4, "c5", 1_250_000_000)])
def test_bare_ranks_spawns_n_ranks(n, config, rows):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--ranks", "--gpus", str(n), "--config",
                        config, "--dry-run"], capture_output=True, text=True, timeout=180, env=_bare_env())
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout  # only rank 0 prints, and the launcher forwards exactly that line
    d = lines[0]
    assert d["n_gpus"] == n and d["mode"] == "ranks"
    assert d["rank_id_sum"] == n * (n + 1) // 2  # every rank joined the all-reduce
    assert d["config"]["rows_per_gpu"] == rows
    assert d["config"]["parallelism"].startswith(f"row-range shards x{n}")


def test_driver_launch_is_inlib_on_rank0():
    """The driver's `torch.distributed.run --nproc-per-node 2 bench.py --gpus 2`:
    both ranks join, rank 0 alone prints the in-library layout over devices 0, 1."""
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", "--master-port=29571", os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--dry-run"], capture_output=True, text=True, timeout=180, env=_bare_env())
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    d = lines[0]
    assert d["mode"] == "in-library" and d["processes"] == 2 and d["rank_id_sum"] == 3
    assert d["gpu_devices"] == [0, 1] and d["n_gpus"] == 2


def test_under_launcher_does_not_respawn():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--ranks", "--gpus", "8", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "[launcher]" not in p.stderr
    assert _json_lines(p.stdout)[0]["n_gpus"] == 1
