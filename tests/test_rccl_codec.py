"""The in-library RCCL combine's lane codec (csrc/combine.h), on the CPU.

mbx_combine=rccl sends each shard's partial row as int64 lanes {lo, hi,
non-NULL}; SUM (and COUNT) is an int128 add with the low word's carry, which
no RCCL reduction op provides, so the gathered lanes are combined by
CombineColumn on device 0.  The same function is exported to the host
(duckdb_mbx_combine_lanes); here it is checked against Python's exact
integers, including carries across 2^64, sign changes, the int128 extremes
and NULL partials."""
import random

import pytest


def _ref(parts, kinds):
    out = []
    for j, k in enumerate(kinds):
        vals = [p[j] for p in parts if p[j] is not None]
        if not vals:
            out.append(None)
        elif k == "sum":
            s = sum(vals)
            s &= (1 << 128) - 1  # two's complement wrap, as the device's int128 add
            out.append(s - (1 << 128) if s >> 127 else s)
        else:
            out.append(min(vals) if k == "min" else max(vals))
    return out


def test_carry_across_the_low_word(mbx):
    parts = [[(1 << 64) - 1], [1], [(1 << 64) - 1]]
    assert mbx.combine_lanes(parts, ["sum"]) == [(1 << 65) - 1]
    parts = [[-(1 << 64)], [1], [-1]]
    assert mbx.combine_lanes(parts, ["sum"]) == [-(1 << 64)]


def test_null_partials(mbx):
    assert mbx.combine_lanes([[None, None, None], [None, None, None]], ["sum", "min", "max"]) == [None] * 3
    assert mbx.combine_lanes([[None, 5, None], [7, None, -3]], ["sum", "min", "max"]) == [7, 5, -3]


@pytest.mark.parametrize("seed", range(20))
def test_random_partials_vs_python(mbx, seed):
    rng = random.Random(seed)
    nranks = rng.choice([1, 2, 3, 7, 8, 16])
    kinds = [rng.choice(["sum", "min", "max"]) for _ in range(rng.randint(1, 12))]
    pool = [0, 1, -1, (1 << 63) - 1, -(1 << 63), (1 << 64) - 1, 1 << 64, -(1 << 64), (1 << 126), -(1 << 126),
            (1 << 127) - 1, -(1 << 127)]

    def val():
        r = rng.random()
        if r < 0.1:
            return None
        if r < 0.4:
            return rng.choice(pool)
        return rng.randint(-(1 << 100), 1 << 100)

    parts = [[val() for _ in kinds] for _ in range(nranks)]
    assert mbx.combine_lanes(parts, kinds) == _ref(parts, kinds)


def test_c5_shape_sum_of_eight_shards(mbx):
    # C5: 8 shards of 1.25e9 rows, x in [1, 50]: per-shard SUM ~ 3e10, total ~ 2.5e11 (the
    # int128 path must agree with the plain sum); and shard sums of a value column near 2^62
    parts = [[1_250_000_000, 31_875_000_000 + r, (1 << 62) + r] for r in range(8)]
    got = mbx.combine_lanes(parts, ["sum", "sum", "sum"])
    assert got == [10_000_000_000, 8 * 31_875_000_000 + 28, 8 * (1 << 62) + 28]


def test_bad_arguments(mbx):
    with pytest.raises(ValueError):
        mbx.combine_lanes([], ["sum"])
    with pytest.raises(ValueError):
        mbx.combine_lanes([[1] * 33], ["sum"] * 33)


def test_loopback_combine_needs_the_experiments_opt_in(mbx):
    """mbx_combine=rccl_loopback (the test stand-in for the collectives) is a
    config value only under MBX_EXPERIMENTS=1: a MoonBit program's environment
    cannot turn the product's RCCL combine into device copies."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import importlib.util, sys\n"
        f"spec = importlib.util.spec_from_file_location('m', {os.path.join(root, 'duckdb.mbt_amd', '__init__.py')!r})\n"
        "m = importlib.util.module_from_spec(spec); sys.modules['m'] = m; spec.loader.exec_module(m)\n"
        "cfg = m.Config.create()\n"
        "print(type(cfg.set('mbx_combine', 'rccl_loopback')).__name__, type(cfg.set('mbx_combine', 'rccl')).__name__)\n"
    )
    env = {k: v for k, v in os.environ.items() if k != "MBX_EXPERIMENTS"}
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == ["Err", "Ok"], out.stdout
    cfg = mbx.Config.create()  # this process has the opt-in (conftest)
    assert isinstance(cfg.set("mbx_combine", "rccl_loopback"), mbx.Ok)
