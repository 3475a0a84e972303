"""The in-library RCCL combine (mbx_combine=rccl, SURVEY §8(e): a sharded global
aggregate's partials combined on the shard devices) run on the one-GPU test
box.  RCCL takes one rank per device, so same-device shards cannot open
communicators; the test-only loopback (mbx_combine=rccl_loopback, refused
without MBX_EXPERIMENTS=1) replaces the two collectives by device copies of
each shard's lane block into every rank's receive buffer.  Everything around
them is the product code that a multi-GPU node runs:
  * pack_lanes_kernel on every shard's stream (COUNT as one lane; SUM / MIN /
    MAX as {lo, hi, valid} of the int128 value; the device error word last);
  * the all-gather / reduce data movement, ordered after each pack;
  * combine_lanes_kernel on device 0 (carry-correct int128 sum, signed
    min/max, validity OR) and the one D2H;
  * the host decode (LanesValue, AVG finished as the emit kernel does) and the
    per-shard error words (raised naming the shard, cleared on every shard).
Each answer is checked against the CPU oracle / numpy over the oracle's
generator, and against the host merge of the same connection.
Reference path: /root/reference/src/duckdb_native.c:714-747 (Config::set)."""
import numpy as np
import pytest

from conftest import one, q

pytestmark = pytest.mark.gpu


def _conn(mbx, devices, combine="rccl_loopback"):
    cfg = mbx.Config.create()
    assert isinstance(cfg.set("gpu_devices", devices), mbx.Ok)
    assert isinstance(cfg.set("mbx_combine", combine), mbx.Ok)
    r = mbx.connect_with_config(cfg)
    assert isinstance(r, mbx.Ok), r.error.message
    return r.value


def _ran(c, before, kind="rccl_loopbacks"):
    st = c.rccl_stats()
    assert st["note"] == "", st
    return st[kind] - before[kind]


def _both(c, sql):
    """The query under the loopback RCCL combine and under the host merge."""
    st0 = c.rccl_stats()
    got = one(c, sql)
    assert _ran(c, st0) == 1, (sql, c.rccl_stats())
    c.set_combine("host")
    ref = one(c, sql)
    c.set_combine("rccl_loopback")
    assert got == ref, (sql, got, ref)
    return got


@pytest.mark.parametrize("devices", ["0,0", "0,0,0"])
def test_rccl_loopback_count_sum_minmax_avg(mbx, oracle, devices):
    n = 30_000_017
    c = _conn(mbx, devices)
    q(c, f"CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x, "
         f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range({n}) tbl(i)")
    x = oracle.synth_i64(n, 42, 0, 50, 1)
    v = oracle.synth_i64(n, 9, 0, 1 << 40, -(1 << 39))
    cnt, s = oracle.synth_filter_count(42, 0, n, 50, 1, 25, 2**63 - 1, 8)
    # COUNT only: the reduce form (one lane per column + the error word)
    assert _both(c, "SELECT COUNT(*) FROM t WHERE x > 24") == [str(cnt)]
    assert _both(c, "SELECT COUNT(*), COUNT(x) FROM t") == [str(n), str(n)]
    # COUNT + SUM(BIGINT) -> HUGEINT: the all-gather form and the combine kernel
    assert _both(c, "SELECT COUNT(*), SUM(x) FROM t WHERE x > 24") == [str(cnt), str(s)]
    # signed MIN / MAX over negative and positive partials, int128 sums of them
    m = x > 24
    got = _both(c, "SELECT SUM(v), MIN(v), MAX(v), COUNT(v) FROM t WHERE x > 24")
    assert got == [str(int(v[m].astype(object).sum())), str(v[m].min()), str(v[m].max()), str(int(m.sum()))]
    # AVG: SUM + COUNT partials, finished on the host as the emit kernel does
    avg = float(_both(c, "SELECT AVG(v) FROM t")[0])
    exact = int(v.astype(object).sum()) / n
    assert abs(avg - exact) <= 1e-9 * max(1.0, abs(exact))
    # every partial NULL (no row passes on any shard): SUM / MIN NULL, COUNT 0
    assert _both(c, "SELECT COUNT(*), SUM(x), MIN(x), MAX(v) FROM t WHERE x > 100") == ["0", "", "", ""]
    c.close()


def test_rccl_loopback_null_partials_on_some_shards(mbx):
    """Rows pass on the last shard only: the other ranks send {0, 0, invalid}
    lanes, and the combine keeps the valid rank's MIN / MAX / SUM."""
    n = 3_000_000
    c = _conn(mbx, "0,0,0")
    q(c, f"CREATE TABLE r AS SELECT i AS r, i - 2500000 AS w FROM range({n}) tbl(i)")
    lo = 2_500_000
    w = np.arange(lo, n, dtype=np.int64) - 2_500_000
    got = _both(c, f"SELECT SUM(w), MIN(w), MAX(w), COUNT(w) FROM r WHERE r >= {lo}")
    assert got == [str(int(w.sum())), str(w.min()), str(w.max()), str(len(w))]
    # and NULL-able values: a shard whose every value is NULL
    q(c, f"CREATE TABLE rn AS SELECT CASE WHEN i < 1000000 THEN NULL ELSE i END AS y FROM range({n}) tbl(i)")
    y = np.arange(1_000_000, n, dtype=np.int64)
    got = _both(c, "SELECT SUM(y), MIN(y), MAX(y), COUNT(y), COUNT(*) FROM rn")
    assert got == [str(int(y.sum())), str(y.min()), str(y.max()), str(len(y)), str(n)]
    c.close()


def test_rccl_loopback_int128_carry_and_decimal(mbx, oracle):
    """Partials whose int128 sums carry out of the low word across ranks, and
    SUM(DECIMAL(15,2)) -> DECIMAL(38,2)."""
    n = 4_000_000
    c = _conn(mbx, "0,0")
    q(c, f"CREATE TABLE b AS SELECT CAST(9223372036854775807 - mbx_synth(3, i, 1000) AS BIGINT) AS big, "
         f"CAST(mbx_synth(11, i, 100000) - 50000 AS DECIMAL(15,2)) AS d, "
         f"-9223372036854775807 + mbx_synth(5, i, 7) AS neg FROM range({n}) tbl(i)")
    big = 9223372036854775807 - oracle.synth_i64(n, 3, 0, 1000, 0).astype(object)
    d = oracle.synth_i64(n, 11, 0, 100000, -50000).astype(object)
    neg = -9223372036854775807 + oracle.synth_i64(n, 5, 0, 7, 0).astype(object)
    got = _both(c, "SELECT SUM(big), SUM(neg), MIN(neg), MAX(big) FROM b")
    assert got == [str(int(big.sum())), str(int(neg.sum())), str(int(neg.min())), str(int(big.max()))]
    sd = int(d.sum())
    sign = "-" if sd < 0 else ""
    assert _both(c, "SELECT SUM(d) FROM b") == [f"{sign}{abs(sd)}.00"]
    t_rccl = q(c, "SELECT SUM(d), SUM(big) FROM b").column_types
    c.set_combine("host")
    assert t_rccl == q(c, "SELECT SUM(d), SUM(big) FROM b").column_types == ["Decimal", "HugeInt"], t_rccl
    c.close()


def test_rccl_loopback_shard_error_is_raised_and_cleared(mbx):
    """A shard whose partial raises an overflow on its device: the error comes
    back naming that shard, and the next query on every shard is clean."""
    c = _conn(mbx, "0,0")
    q(c, "CREATE TABLE o AS SELECT i AS x FROM range(2000) tbl(i)")  # shard 0: 0..999, shard 1: 1000..1999
    m = 9_220_000_000_000_000  # 9.22e15: 1000·m fits in BIGINT, 1001·m does not
    assert 1000 * m < 2**63 <= 1001 * m
    st0 = c.rccl_stats()
    r = c.query(f"SELECT SUM(x * {m}) FROM o")
    assert not hasattr(r, "value"), r
    msg = r.error.message
    assert "Overflow" in msg and "shard 1" in msg, msg
    # no stale error word: the same connection answers the next queries exactly
    assert one(c, "SELECT COUNT(*), SUM(x) FROM o") == ["2000", str(sum(range(2000)))]
    assert one(c, f"SELECT SUM(x * {m}) FROM o WHERE x < 1000") == [str(m * sum(range(1000)))]
    st = c.rccl_stats()
    assert st["rccl_loopbacks"] - st0["rccl_loopbacks"] >= 2, st
    c.close()


def test_rccl_loopback_c5_shape(mbx, oracle):
    """The C5 query over 2 x 1.25e8 rows: COUNT and the int128 SUM of every
    shard combined on device 0, exact against the oracle over all rows."""
    n = 250_000_000
    c = _conn(mbx, "0,0")
    q(c, f"CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x FROM range({n}) tbl(i)")
    cnt, s = oracle.synth_filter_count(42, 0, n, 50, 1, 25, 2**63 - 1, 8)
    for _ in range(3):
        st0 = c.rccl_stats()
        assert one(c, "SELECT COUNT(*), SUM(x) FROM t WHERE x > 24") == [str(cnt), str(s)]
        assert _ran(c, st0) == 1
        st0 = c.rccl_stats()
        assert one(c, "SELECT COUNT(*) FROM t WHERE x > 24") == [str(cnt)]
        assert _ran(c, st0) == 1
    # per-shard partials as the all-gather delivered them, each against its
    # shard's row range; and the COUNT-only reduce keeps every rank's own count
    one(c, "SELECT COUNT(*), SUM(x) FROM t WHERE x > 24")
    for i in range(2):
        p = c.shard_partial(i)
        lo, hi = i * n // 2, (i + 1) * n // 2
        pc, ps = oracle.synth_filter_count(42, lo, hi - lo, 50, 1, 25, 2**63 - 1, 8)
        assert p.value(0, 0) == str(pc) and p.value(1, 0) == str(ps), (i, p.cells())
        p.close()
    one(c, "SELECT COUNT(*) FROM t WHERE x > 24")
    for i in range(2):
        p = c.shard_partial(i)
        lo, hi = i * n // 2, (i + 1) * n // 2
        pc, _ = oracle.synth_filter_count(42, lo, hi - lo, 50, 1, 25, 2**63 - 1, 8)
        assert p is not None and p.value(0, 0) == str(pc), i
        p.close()
    info = c.rccl_info()
    assert info["state"] == "loopback" and info["reduces"] >= 4 and info["allgathers"] >= 4, info
    assert info["last_collective"] == "loopback ncclReduce (int64 sum to device 0)", info
    c.close()


def test_rccl_without_distinct_devices_falls_back_with_note(mbx, oracle):
    """mbx_combine=rccl over same-device shards (no loopback): RCCL refuses
    two ranks on one device, so the host merge answers and says why."""
    n = 1_000_003
    c = _conn(mbx, "0,0", combine="rccl")
    q(c, f"CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x FROM range({n}) tbl(i)")
    cnt, s = oracle.synth_filter_count(42, 0, n, 50, 1, 25, 2**63 - 1, 8)
    st0 = c.rccl_stats()
    assert one(c, "SELECT COUNT(*), SUM(x) FROM t WHERE x > 24") == [str(cnt), str(s)]
    st = c.rccl_stats()
    assert st["rccl_combines"] == st0["rccl_combines"]
    # a layout RCCL never covers: counted apart from combines that failed
    assert st["rccl_unsupported"] == st0["rccl_unsupported"] + 1 and st["rccl_fallbacks"] == st0["rccl_fallbacks"]
    assert "not distinct" in st["note"], st
    info = c.rccl_info()
    assert info["state"] == "none" and not info["prepared_at_connect"] and info["mode"] == "rccl", info
    # shapes the RCCL combine does not cover say so too (a DOUBLE key, DOUBLE SUM)
    c.set_combine("rccl_loopback")
    q(c, "SELECT x / 2 AS g, COUNT(*) FROM t GROUP BY g")
    assert "not an integer" in c.rccl_stats()["note"], c.rccl_stats()
    q(c, "SELECT SUM(x / 2) FROM t")
    assert "floating-point" in c.rccl_stats()["note"]
    c.close()


def test_rccl_collective_failure_falls_back_to_host_merge(mbx, oracle, monkeypatch):
    """A collective that reports an error (injected, MBX_RCCL_TEST_FAIL): the
    statement is answered exactly by the host merge, the communicators are
    dropped, and the connection keeps the host merge for the next statements;
    the GROUP BY combine the same."""
    n = 2_000_003
    for sql, group in (("SELECT COUNT(*), SUM(x) FROM t WHERE x > 24", False),
                       ("SELECT k, COUNT(*), SUM(x) FROM t GROUP BY k", True)):
        c = _conn(mbx, "0,0")
        q(c, f"CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x, CAST(mbx_synth(7, i, 32) AS INTEGER) AS k "
             f"FROM range({n}) tbl(i)")
        c.set_combine("host")
        ref = q(c, sql).rows
        c.set_combine("rccl_loopback")
        monkeypatch.setenv("MBX_RCCL_TEST_FAIL", "1")
        st0 = c.rccl_stats()
        assert q(c, sql).rows == ref, sql
        st = c.rccl_stats()
        assert st["rccl_fallbacks"] > st0["rccl_fallbacks"], st
        assert st["rccl_loopbacks"] == st0["rccl_loopbacks"] and "host merge from now on" in st["note"], st
        monkeypatch.delenv("MBX_RCCL_TEST_FAIL")
        assert q(c, sql).rows == ref, sql
        assert c.rccl_stats()["rccl_loopbacks"] == st0["rccl_loopbacks"], c.rccl_stats()  # communicators dropped
        if not group:
            cnt, s = oracle.synth_filter_count(42, 0, n, 50, 1, 25, 2**63 - 1, 8)
            assert ref == [[str(cnt), str(s)]]
        c.close()


def test_rccl_library_calls_on_one_gpu(mbx):
    """The real RCCL calls the combine makes -- librccl opened by dlopen,
    ncclCommInitAll (on its helper thread, bounded), one ncclReduce and one
    ncclAllGather inside ncclGroupStart/End on a stream of the device -- on a
    one-rank communicator, the only one a one-GPU box allows; the lanes come
    back unchanged.  (Distinct-device ranks exchange data the same way.)"""
    r = mbx.rccl_selftest(0)
    assert r["ok"], r
    # twice: a second communicator in the same process; the device-list form
    # reports what RCCL itself says about its one rank
    r = mbx.rccl_selftest([0])
    assert r["ok"], r
    assert r["ranks"] == [{"device": 0, "count": 1, "user_rank": 0, "cu_device": 0}], r
    assert r["init_us"] > 0 and r["check_us"] > 0 and r["total_us"] >= r["init_us"], r
    # a device list RCCL cannot take (two ranks on one device) is refused before any RCCL call
    r = mbx.rccl_selftest([0, 0])
    assert not r["ok"] and "not distinct" in r["error"], r


def _group_both(c, sql):
    """A GROUP BY under the loopback RCCL combine (dense key slots) and under
    the host merge of the same connection: the same rows, in key order."""
    st0 = c.rccl_stats()
    got = q(c, sql).rows
    st = c.rccl_stats()
    assert st["note"] == "" and st["rccl_group_combines"] - st0["rccl_group_combines"] == 1, (sql, st)
    c.set_combine("host")
    ref = q(c, sql).rows
    c.set_combine("rccl_loopback")
    assert got == ref, (sql, got[:5], ref[:5])
    return got


@pytest.mark.parametrize("devices", ["0,0", "0,0,0"])
def test_rccl_loopback_group_by_c3_shape(mbx, oracle, devices):
    """C3 over sharded parts: each shard's 32 groups packed into dense key
    slots, all-gathered, combined on device 0; every group's COUNT and exact
    int128 SUM against the oracle, and every shard's partial against its range."""
    n = 40_000_003
    c = _conn(mbx, devices)
    q(c, f"CREATE TABLE g AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
         f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range({n}) tbl(i)")
    oc, osum = oracle.synth_groupby(7, 9, 0, n, 32, 1 << 40, -(1 << 39), 8)
    rows = _group_both(c, "SELECT k, SUM(v), COUNT(*) FROM g GROUP BY k")
    assert rows == [[str(k), str(osum[k]), str(oc[k])] for k in range(32) if oc[k]]
    nsh = devices.count(",") + 1
    for i in range(nsh):
        lo, hi = n * i // nsh, n * (i + 1) // nsh
        pc, ps = oracle.synth_groupby(7, 9, lo, hi - lo, 32, 1 << 40, -(1 << 39), 8)
        part = c.shard_partial(i)
        got, _ = part.cells()
        part.close()
        assert sorted((int(r[0]), int(r[1]), int(r[2])) for r in got) == \
            [(k, int(ps[k]), int(pc[k])) for k in range(32) if pc[k]], i
    # HAVING / ORDER BY / LIMIT over the combined groups
    top = q(c, "SELECT k, COUNT(*) AS n FROM g GROUP BY k HAVING COUNT(*) > 0 ORDER BY n DESC, k LIMIT 3").rows
    exp = sorted(((int(oc[k]), k) for k in range(32)), key=lambda t: (-t[0], t[1]))[:3]
    assert top == [[str(k), str(cn)] for cn, k in exp]
    c.close()


def test_rccl_loopback_group_by_nulls_sparse_keys(mbx):
    """Negative keys, a NULL key group, keys present on one shard only,
    MIN / MAX / AVG / COUNT(col) with NULL values, DECIMAL sums; against numpy
    and the host merge."""
    n = 3_000_000
    c = _conn(mbx, "0,0,0")
    q(c, f"CREATE TABLE s AS SELECT CASE WHEN i % 97 = 0 THEN NULL "
         f"WHEN i >= 2000000 THEN 100 + i % 5 ELSE i % 13 - 6 END AS k, "
         f"CASE WHEN i % 11 = 0 THEN NULL ELSE i - 1500000 END AS v, "
         f"CAST(i % 1000 AS DECIMAL(12,2)) AS d FROM range({n}) tbl(i)")
    i = np.arange(n, dtype=np.int64)
    knull = i % 97 == 0
    k = np.where(i >= 2_000_000, 100 + i % 5, i % 13 - 6)
    vnull = i % 11 == 0
    v = i - 1_500_000
    d = i % 1000
    rows = _group_both(c, "SELECT k, COUNT(*), COUNT(v), SUM(v), MIN(v), MAX(v), SUM(d) FROM s GROUP BY k")
    keys = sorted(set(k[~knull].tolist()))
    exp = []
    for kk in keys + [None]:
        m = knull if kk is None else (~knull & (k == kk))
        mv = m & ~vnull
        vs = v[mv]
        exp.append(["" if kk is None else str(kk), str(int(m.sum())), str(int(mv.sum())),
                    str(int(vs.sum())) if vs.size else "", str(vs.min()) if vs.size else "",
                    str(vs.max()) if vs.size else "", f"{int(d[m].sum())}.00"])
    assert rows == exp
    avg = _group_both(c, "SELECT k, AVG(v) FROM s GROUP BY k")
    for row, kk in zip(avg, keys + [None]):
        m = (knull if kk is None else (~knull & (k == kk))) & ~vnull
        assert abs(float(row[1]) - v[m].mean()) <= 1e-9 * max(1.0, abs(v[m].mean())), (kk, row)
    c.close()


def test_rccl_loopback_group_by_wide_keys_and_errors(mbx):
    """A key range wider than 4096 slots takes the host merge of the same
    partials (with its note); an overflow on one shard's partial is raised
    naming the shard, and the next GROUP BY on the connection is exact."""
    c = _conn(mbx, "0,0")
    q(c, "CREATE TABLE w AS SELECT i * 7 AS k, i AS x FROM range(10000) tbl(i)")
    st0 = c.rccl_stats()
    rows = q(c, "SELECT k, COUNT(*) FROM w GROUP BY k").rows
    assert len(rows) == 10000 and rows[0] == ["0", "1"] and rows[-1] == [str(9999 * 7), "1"]
    st = c.rccl_stats()
    assert "wider than 4096" in st["note"] and st["rccl_group_combines"] == st0["rccl_group_combines"], st
    m = 9_220_000_000_000_000
    q(c, "CREATE TABLE o AS SELECT i % 4 AS k, i AS x FROM range(2000) tbl(i)")
    r = c.query(f"SELECT k, SUM(x * {m}) FROM o GROUP BY k")
    assert not hasattr(r, "value"), r
    assert "Overflow" in r.error.message and "shard 1" in r.error.message, r.error.message
    got = q(c, "SELECT k, SUM(x), COUNT(*) FROM o GROUP BY k").rows
    assert got == [[str(kk), str(sum(range(kk, 2000, 4))), "500"] for kk in range(4)]
    assert c.rccl_stats()["note"] == ""
    c.close()
