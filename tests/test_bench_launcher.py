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


@pytest.mark.parametrize("counts,world,ranks,form", [
    ([8] * 8, 8, False, "in-library"),   # a full node visible to every rank
    ([8, 1, 1, 1, 1, 1, 1, 1], 8, False, "in-library"),
    ([1] * 8, 8, False, "ranks"),        # one device per rank (per-rank visibility)
    ([2, 2], 4, False, "ranks"),
    ([8] * 8, 8, True, "ranks"),         # --ranks asks for it
    ([0, 1], 2, False, None),            # a rank without a GPU: no layout
])
def test_choose_form(counts, world, ranks, form):
    import bench
    f, reason = bench.choose_form(counts, world, ranks)
    assert f == form, reason
    assert reason


def _torchrun(n, port, extra_env, *args):
    env = dict(_bare_env(), **extra_env)
    return subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py")]
                          + list(args), capture_output=True, text=True, timeout=180, env=env)


@pytest.mark.parametrize("visible,form", [("2", "in-library"), ("1", "ranks")])
def test_driver_launch_follows_device_visibility(visible, form):
    """The driver's launch under the two visibilities an 8-GPU node can give:
    every rank sees all devices (one process drives them in-library) or only
    its own (one device per rank, RCCL combine); the choice, the counts and
    the reason are in config.form and config.parallelism."""
    p = _torchrun(2, 29573 if form == "ranks" else 29575, {"MBX_BENCH_VISIBLE_GPUS": visible},
                  "--gpus", "2", "--dry-run")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    d = lines[0]
    assert d["mode"] == form and d["processes"] == 2 and d["rank_id_sum"] == 3
    f = d["config"]["form"]
    assert f["form"] == form and f["visible_devices_per_rank"] == [int(visible)] * 2
    assert f["min"] == f["max"] == int(visible) and f["reason"]
    if form == "ranks":
        assert d["gpu_devices"] is None
        assert "one process per GPU" in d["config"]["parallelism"]
    else:
        assert d["gpu_devices"] == [0, 1] and "in-library" in d["config"]["parallelism"]


def test_driver_launch_without_gpus_fails_loudly():
    p = _torchrun(2, 29577, {"MBX_BENCH_VISIBLE_GPUS": "0"}, "--gpus", "2", "--dry-run")
    assert p.returncode != 0
    assert "see no GPU" in p.stderr


def test_gpus_1_is_unchanged():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run"], capture_output=True,
                       text=True, timeout=120, env=_bare_env())
    assert p.returncode == 0, p.stderr[-2000:]
    d = _json_lines(p.stdout)[0]
    assert d["n_gpus"] == 1 and d["mode"] == "in-library" and d["gpu_devices"] == [0]
    assert "form" not in d["config"]  # no vote without a launcher


def test_guarded_leg_times_out_and_reports():
    """The RCCL leg runs under a watchdog: a leg that never returns becomes an
    {"error": "timeout ..."} entry instead of hanging the headline line."""
    import threading
    import bench
    ev = threading.Event()
    r = bench.guarded(lambda: ev.wait(30) and {"ok": 1}, 0.2)
    assert r["error"].startswith("timeout")
    ev.set()
    assert bench.guarded(lambda: {"ok": 1}, 5) == {"ok": 1}
    r = bench.guarded(lambda: 1 // 0, 5)
    assert "division" in r["error"]


def test_stdout_carries_only_the_json_line():
    """Anything a library in the bench process writes to fd 1 (RCCL prints its
    version banner when a communicator is created) lands on stderr; the JSON
    line printed through sys.stdout is the only thing on stdout."""
    code = ("import os, sys, json; sys.path.insert(0, %r); import bench; bench.guard_stdout(); "
            "os.write(1, b'RCCL version : x\\n'); print(json.dumps({'metric': 'm', 'value': 1}), flush=True)" % ROOT)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert p.stdout.strip().splitlines() == ['{"metric": "m", "value": 1}'], p.stdout
    assert "RCCL version" in p.stderr


def test_dry_run_pins_the_multi_device_line_fields():
    """`--gpus 8` (the driver's SCALE point): the line's multi_device block
    carries the RCCL self-test over devices 0..7 (run before the connection),
    the combine's per-step collective counts and the communicators' RCCL
    evidence, and the 1 -> 8 curve from the same process."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--dry-run"],
                       capture_output=True, text=True, timeout=180, env=_bare_env())
    assert p.returncode == 0, p.stderr[-2000:]
    md = _json_lines(p.stdout)[0]["multi_device_plan"]
    assert md["rccl_selftest"]["devices"] == list(range(8))
    assert {"ran_rccl_steps", "ncclReduce_steps", "ncclAllGather_steps", "fallback_steps",
            "unsupported_steps"} <= set(md["combine"]["timed_loop"])
    assert {"ranks[].count", "ranks[].user_rank", "init_s", "first_wait_ms", "proves_n_ranks"} <= \
        set(md["combine"]["rccl"])
    pts = md["curve"]["points"]
    assert [x["gpus"] for x in pts] == [1, 2, 4, 8] and pts[-1]["the_headline"]
    assert [x["devices"] for x in pts[:3]] == [[0], [0, 1], [0, 1, 2, 3]]
    # one GPU: no multi-device block at all
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run"], capture_output=True,
                       text=True, timeout=120, env=_bare_env())
    assert "multi_device_plan" not in _json_lines(p.stdout)[0]


@pytest.mark.parametrize("ngpu,spg,pts", [
    (8, 1, [(1, [0]), (2, [0, 1]), (4, [0, 1, 2, 3])]), (2, 2, [(1, [0, 0])]), (1, 1, []),
    (6, 1, [(1, [0]), (2, [0, 1]), (4, [0, 1, 2, 3])])])
def test_curve_points(ngpu, spg, pts):
    import bench
    assert bench.curve_points(ngpu, spg) == pts


def test_rccl_evidence_proves_n_ranks_only_from_rccl_itself():
    import bench
    ranks = [{"device": d, "count": 4, "user_rank": d, "cu_device": d} for d in range(4)]
    e = bench.rccl_evidence({"state": "ready", "ranks": ranks}, [0, 1, 2, 3])
    assert e["proves_n_ranks"] and e["saw_nranks"] == [4]
    bad = [dict(r, count=1) for r in ranks]  # four one-rank communicators are not a 4-rank RCCL
    assert not bench.rccl_evidence({"ranks": bad}, [0, 1, 2, 3])["proves_n_ranks"]
    assert not bench.rccl_evidence({"state": "none"}, [0, 0])["proves_n_ranks"]  # same-device shards


class _FakeResult:
    def __init__(self, cells):
        self._cells = cells

    def column_count(self):
        return len(self._cells[0])

    def value(self, c, r):
        return self._cells[r][c]

    def cells(self):
        return [list(r) for r in self._cells], [[False] * len(r) for r in self._cells]

    def close(self):
        pass


class _FakeConn:
    """A sharded connection whose shards hold the given per-shard answers: the
    global answer is their combination, every shard_partial its own row."""

    def __init__(self, config, shards, devices, wrong_shard=None):
        self.config, self.shards, self.devices, self.wrong = config, shards, devices, wrong_shard
        self.steps = 0

    def query(self, sql):
        return SimpleNamespace(value=None)

    def _global(self):
        if self.config == "c3":
            acc = {}
            for sh in self.shards:
                for k, c, s in sh:
                    a = acc.get(k, (0, 0))
                    acc[k] = (a[0] + c, a[1] + s)
            return [(str(k), str(acc[k][1]), str(acc[k][0])) for k in sorted(acc)]
        return [tuple(str(sum(sh[i] for sh in self.shards)) for i in range(len(self.shards[0])))]

    def query_raw(self, sql):
        self.steps += 1
        return _FakeResult(self._global())

    def shard_partial(self, i):
        sh = self.shards[i]
        if self.config == "c3":
            rows = [(str(k), str(s), str(c + (1 if i == self.wrong else 0))) for k, c, s in sh]
            return _FakeResult(rows)
        return _FakeResult([tuple(str(v + (1 if i == self.wrong else 0)) for v in sh)])

    def profile_drain(self):
        name = "group_direct" if self.config == "c3" else "filter_agg"
        return [{"name": name, "ms": 1.0, "shard": i, "device": d} for i, d in enumerate(self.devices)]

    def rccl_stats(self):
        return dict(bench_zero(), rccl_combines=self.steps, rccl_reduces=self.steps)

    def rccl_info(self):
        n = len(self.devices)
        return {"state": "ready", "ranks": [{"device": d, "count": n, "user_rank": i, "cu_device": d}
                                            for i, d in enumerate(self.devices)]}

    def close(self):
        pass


def bench_zero():
    import bench
    return dict(bench.ZERO_RCCL_STATS)


@pytest.mark.parametrize("config", ["c2", "c5", "c3"])
def test_curve_legs_schema_and_parity_on_cpu(config, monkeypatch):
    """curve_legs over a fake library: one point per prefix (1, 2, 4 of 8
    GPUs) plus the headline's, each with value, kernel time, the combine's
    collective counts, RCCL's rank evidence and parity of the global answer
    and of every shard against the headline's per-shard oracle entries; a
    shard whose partial is off fails its point's parity."""
    import bench
    monkeypatch.setattr(bench, "time_steps", lambda step, k, w, b=None, s=None: (0.01 * k, [step() for _ in range(k)][-1]))
    nsh = 8
    if config == "c3":
        shard_par = [{"shard": i, "match": True, "oracle": [(k, 10 + i, 100 * k - i) for k in range(4)]}
                     for i in range(nsh)]
        per_shard = [e["oracle"] for e in shard_par]
    else:
        shard_par = [{"shard": i, "match": True, "oracle_count": 500 + i, "oracle_sum": 9000 + i}
                     for i in range(nsh)]
        per_shard = [[e["oracle_count"]] + ([e["oracle_sum"]] if config == "c5" else []) for e in shard_par]
    for wrong in (None, 1):
        made = []

        def connect(cfg):
            devs = [int(x) for x in cfg.kv.get("gpu_devices", cfg.kv.get("gpu_device", "0")).split(",")]
            c = _FakeConn(config, per_shard[:len(devs)], devs, wrong_shard=wrong)
            made.append(c)
            return SimpleNamespace(value=c)

        class Cfg:
            def __init__(self):
                self.kv = {}

            def set(self, k, v):
                self.kv[k] = v

        fake = SimpleNamespace(Config=SimpleNamespace(create=Cfg), connect_with_config=connect, Err=type("Err", (), {}))
        args = SimpleNamespace(config=config, rows=1000, warmup=1, steps=3)
        plan = {"ngpu": 8, "shards_per_gpu": 1, "devices": list(range(8)), "nshards": 8, "rows_total": 8000}
        result = {"ms_per_step": 1.2, "value": 6.6e12, "roofline": {"kernel_ms_avg": 1.1}, "parity": {"match": True}}
        out = bench.curve_legs(fake, args, plan, result, shard_par)
        pts = out["points"]
        assert [p["gpus"] for p in pts] == [1, 2, 4, 8], pts
        assert pts[-1]["the_headline"] and pts[-1]["value"] == 6.6e12
        for p in pts[:3]:
            assert "error" not in p, p
            assert p["rows"] == 1000 * p["gpus"] and p["unit"] == "rows/s" and p["kernel_ms_avg"] == 1.0
            assert p["combine"]["ran_rccl_steps"] == 3 and p["combine"]["ncclReduce_steps"] == 3
            if p["shards"] > 1:
                assert p["rccl"]["proves_n_ranks"], p["rccl"]
                assert p["parity"]["shards_match"] == (wrong is None), p
            assert p["parity"]["match"] == (wrong is None or p["shards"] == 1), p
        assert pts[0]["speedup_vs_1"] == 1.0
        assert [len(c.devices) for c in made] == [1, 2, 4]
