"""GROUP BY with NULL keys and NULL-able value columns on the device-native
direct-index kernel (group_direct_lds, validity mask VM): a NULL key is its
own group (the last key slot, emitted last), COUNT(*) counts every row of a
group, COUNT(col) / SUM / MIN / MAX / AVG skip the column's NULLs, and a group
whose values are all NULL has SUM / MIN / MAX / AVG NULL and COUNT(col) 0.
The reference's NULL semantics: src/duckdb_fixture_cases.mbt:125-145 ("null
handling"), :223-228 ("null in values"); DuckDB puts all NULL keys in one
group.  Every answer is checked against the oracle's restatement over the same
generator (oracle.c orc_synth_groupby_nulls), and the kernel that ran is read
from the query profile: the run-time compiled jit_group no longer takes these
shapes."""
import pytest

from conftest import q

pytestmark = pytest.mark.gpu

SEEDS = [7, 19, 9, 23, 31, 29]  # k, k NULL, v, v NULL, w, w NULL
MODS = [32, 7, 1 << 40, 7, 1 << 40, 7]  # 32 keys, 1/7 NULL keys, values, 1/7 NULL values
ADDS = [-(1 << 39), -(1 << 39)]


def _setup(c, n, name="gnn", mods=MODS):
    kn = f"mbx_synth({SEEDS[1]}, i, {mods[1]}) = 0" if mods[1] else "false"
    vn = f"mbx_synth({SEEDS[3]}, i, {mods[3]}) = 0" if mods[3] else "false"
    wn = f"mbx_synth({SEEDS[5]}, i, {mods[5]}) = 0" if mods[5] else "false"
    q(c, f"CREATE TABLE {name} AS SELECT "
         f"CASE WHEN {kn} THEN NULL ELSE CAST(mbx_synth({SEEDS[0]}, i, {mods[0]}) AS INTEGER) END AS k, "
         f"CASE WHEN {vn} THEN NULL ELSE mbx_synth({SEEDS[2]}, i, {mods[2]}) + ({ADDS[0]}) END AS v, "
         f"CASE WHEN {wn} THEN NULL ELSE mbx_synth({SEEDS[4]}, i, {mods[4]}) + ({ADDS[1]}) END AS w, "
         f"mbx_synth(42, i, 50) + 1 AS x FROM range({n}) tbl(i)")


def _kernels(c):
    return [kk["name"] for kk in c.last_profile()["kernels"]]


def _cell(x):
    return "" if x is None else str(x)


def _conn(mbx, devices=None, combine=None):
    cfg = mbx.Config.create()
    cfg.set("mbx_profile", "true")
    if devices:
        assert isinstance(cfg.set("gpu_devices", devices), mbx.Ok)
    if combine:
        assert isinstance(cfg.set("mbx_combine", combine), mbx.Ok)
    r = mbx.connect_with_config(cfg)
    assert isinstance(r, mbx.Ok), r.error.message
    return r.value


SQL = "SELECT k, COUNT(*), COUNT(v), SUM(v), MIN(v), MAX(v), COUNT(w), SUM(w), MIN(w), MAX(w) FROM gnn GROUP BY k"


def _expect(groups, cols=(0, 1, 2, 3, 4, 5, 6, 7, 8, 9)):
    return [[_cell(g[i]) for i in cols] for g in groups]


@pytest.mark.parametrize("n", [1, 255, 257, 100_003, 1_000_003])
def test_null_keys_two_nullable_values(mbx, oracle, monkeypatch, n):
    c = _conn(mbx)
    _setup(c, n)
    exp = _expect(oracle.synth_groupby_nulls(SEEDS, MODS, ADDS, 0, n, 8))
    got = q(c, SQL).rows
    ks = _kernels(c)
    assert "group_direct" in ks and "jit_group" not in ks, ks
    assert got == exp, (n, got[-2:], exp[-2:])
    # the generic path (MBX_GD_NULLS=0: jit_group / compaction) agrees
    monkeypatch.setenv("MBX_GD_NULLS", "0")
    ref = q(c, SQL + " ORDER BY k").rows
    monkeypatch.delenv("MBX_GD_NULLS")
    assert "group_direct" not in _kernels(c)
    assert ref == got
    c.close()


def test_null_key_shapes_and_avg(mbx, oracle):
    """Every validity mask the kernel takes: the key alone (with COUNT(*) only,
    and with one value), one value alone, two values with either or both
    NULL-able; AVG over NULL-able values; a fused predicate on another column."""
    n = 300_007
    c = _conn(mbx)
    # k NULL-able; v, w never NULL
    _setup(c, n, "gk", [32, 7, 1 << 40, 0, 1 << 40, 0])
    g = oracle.synth_groupby_nulls(SEEDS, [32, 7, 1 << 40, 0, 1 << 40, 0], ADDS, 0, n, 8)
    for sql, cols in (("SELECT k, COUNT(*) FROM gk GROUP BY k", (0, 1)),
                      ("SELECT k, COUNT(*), SUM(v), MIN(v), MAX(v) FROM gk GROUP BY k", (0, 1, 3, 4, 5)),
                      ("SELECT k, SUM(v), SUM(w), COUNT(w) FROM gk GROUP BY k", (0, 3, 7, 6))):
        assert q(c, sql).rows == _expect(g, cols), sql
        assert "group_direct" in _kernels(c), (sql, _kernels(c))
    # v NULL-able, k and w not; and only w NULL-able
    for mods in ([32, 0, 1 << 40, 7, 1 << 40, 0], [32, 0, 1 << 40, 0, 1 << 40, 7], [32, 5, 1 << 40, 3, 1 << 40, 11]):
        q(c, "DROP TABLE IF EXISTS gm")
        _setup(c, n, "gm", mods)
        g = oracle.synth_groupby_nulls(SEEDS, mods, ADDS, 0, n, 8)
        sql = "SELECT k, COUNT(*), COUNT(v), SUM(v), MIN(v), MAX(v), COUNT(w), SUM(w), MIN(w), MAX(w) FROM gm GROUP BY k"
        assert q(c, sql).rows == _expect(g), mods
        assert "group_direct" in _kernels(c), (mods, _kernels(c))
        # AVG: DOUBLE of the exact sum / count, NULL for a group of NULLs
        for row, e in zip(q(c, "SELECT k, AVG(v), AVG(w) FROM gm GROUP BY k").rows, g):
            for cell, cnt, s in ((row[1], e[2], e[3]), (row[2], e[6], e[7])):
                if not cnt:
                    assert cell == ""
                else:
                    assert abs(float(cell) - s / cnt) <= 1e-9 * max(1.0, abs(s / cnt)), (mods, row, e)
    # a fused range predicate on a column of its own (x, never NULL)
    import numpy as np
    mods = [32, 7, 1 << 40, 7, 1 << 40, 7]
    q(c, "DROP TABLE IF EXISTS gm")
    _setup(c, n, "gm", mods)
    rows = q(c, "SELECT k, COUNT(*), COUNT(v), SUM(v) FROM gm WHERE x > 24 GROUP BY k").rows
    assert "group_direct" in _kernels(c), _kernels(c)
    k = oracle.synth_i64(n, 7, 0, 32, 0)
    kn = oracle.synth_i64(n, 19, 0, 7, 0) == 0
    v = oracle.synth_i64(n, 9, 0, 1 << 40, -(1 << 39))
    vn = oracle.synth_i64(n, 23, 0, 7, 0) == 0
    x = oracle.synth_i64(n, 42, 0, 50, 1)
    want = []
    for kk in list(range(32)) + [None]:
        m = (x > 24) & (kn if kk is None else (~kn & (k == kk)))
        if not m.any():
            continue
        vs = v[m & ~vn]
        want.append([_cell(kk), str(int(m.sum())), str(len(vs)), str(int(vs.astype(object).sum())) if len(vs) else ""])
    assert rows == want
    # every key NULL: one group
    q(c, f"CREATE TABLE an AS SELECT CAST(NULL AS INTEGER) AS k, i AS v FROM range(1000) tbl(i)")
    assert q(c, "SELECT k, COUNT(*), SUM(v) FROM an GROUP BY k").rows == [["", "1000", str(sum(range(1000)))]]
    c.close()


def test_null_keys_1e9_rows(mbx, oracle):
    """The shape at 1e9 rows (14 % NULL keys, 14 % NULL values in each of two
    INT64 columns): every group against the oracle over all rows."""
    import os
    n = 1_000_000_000
    c = _conn(mbx)
    _setup(c, n)
    got = q(c, SQL).rows
    assert "group_direct" in _kernels(c), _kernels(c)
    exp = _expect(oracle.synth_groupby_nulls(SEEDS, MODS, ADDS, 0, n, max(8, len(os.sched_getaffinity(0)))))
    assert got == exp
    c.close()


@pytest.mark.parametrize("combine", ["host", "rccl_loopback"])
def test_null_keys_sharded(mbx, oracle, combine):
    """The same GROUP BY over 3 row-range shards: each shard's partial groups
    (the NULL key among them) combined by the host merge or by the RCCL
    combine's dense key slots (loopback on one GPU); against the oracle, and
    every shard's partial against its own row range."""
    n = 3_000_017
    c = _conn(mbx, "0,0,0", combine)
    _setup(c, n)
    got = q(c, SQL).rows
    assert got == _expect(oracle.synth_groupby_nulls(SEEDS, MODS, ADDS, 0, n, 8))
    if combine == "rccl_loopback":
        st = c.rccl_stats()
        assert st["note"] == "" and st["rccl_group_combines"] >= 1, st
    for i in range(3):
        lo, hi = n * i // 3, n * (i + 1) // 3
        part = c.shard_partial(i)
        rows, _ = part.cells()
        part.close()
        exp = oracle.synth_groupby_nulls(SEEDS, MODS, ADDS, lo, hi - lo, 8)
        # partial columns: key, COUNT(*), then per value COUNT / SUM / MIN / MAX in the plan's order
        assert len(rows) == len(exp), i
        assert [r[0] for r in rows] == [_cell(e[0]) for e in exp], i
    c.close()


# ---------------------------------------------------------------------------
# F3: one integer key over a range too wide for the LDS tables (group_part.hip)
# ---------------------------------------------------------------------------
def _np_groups(k, cols, aggs):
    """numpy GROUP BY k (no NULLs): sorted keys and, per (agg, column), the
    exact per-key result as Python ints."""
    import numpy as np
    keys, inv = np.unique(k, return_inverse=True)
    out = [keys.tolist(), np.bincount(inv).tolist()]
    for a, x in aggs:
        v = cols[x]
        if a == "sum":
            acc = [0] * len(keys)
            order = np.argsort(inv, kind="stable")
            bounds = np.concatenate([[0], np.cumsum(np.bincount(inv))])
            vs = v[order].astype(object)
            for g in range(len(keys)):
                acc[g] = int(vs[bounds[g]:bounds[g + 1]].sum())
            out.append(acc)
        elif a == "min":
            m = np.full(len(keys), np.iinfo(np.int64).max)
            np.minimum.at(m, inv, v.astype(np.int64))
            out.append(m.tolist())
        elif a == "max":
            m = np.full(len(keys), np.iinfo(np.int64).min)
            np.maximum.at(m, inv, v.astype(np.int64))
            out.append(m.tolist())
    return out


@pytest.mark.parametrize("n,groups,ktype,vtype", [
    (3_000_017, 100_000, "BIGINT", "BIGINT"), (2_000_003, 5_000, "INTEGER", "INTEGER"),
    (1_000_001, 250_000, "BIGINT", "INTEGER"), (100_000, 60_000, "INTEGER", "BIGINT")])
def test_partitioned_group_by_wide_key_range(mbx, oracle, n, groups, ktype, vtype):
    """COUNT(*), SUM, MIN, MAX, AVG of two value columns per key, keys spread
    over a range wider than the LDS tables (negative minimum included), against
    numpy; the profile names group_part, not the hash path."""
    import numpy as np
    c = _conn(mbx)
    q(c, f"CREATE TABLE w AS SELECT CAST(mbx_synth(7, i, {groups}) * 3 - {groups} AS {ktype}) AS k, "
         f"CAST(mbx_synth(9, i, 2000000) - 1000000 AS {vtype}) AS v, "
         f"CAST(mbx_synth(11, i, 1000) AS {vtype}) AS u FROM range({n}) tbl(i)")
    k = oracle.synth_i64(n, 7, 0, groups, 0) * 3 - groups
    v = oracle.synth_i64(n, 9, 0, 2_000_000, -1_000_000)
    u = oracle.synth_i64(n, 11, 0, 1000, 0)
    rows = q(c, "SELECT k, COUNT(*), SUM(v), MIN(v), MAX(u), SUM(u) FROM w GROUP BY k").rows
    assert "group_part" in _kernels(c), _kernels(c)
    keys, cnt, sv, mnv, mxu, su = _np_groups(k, {"v": v, "u": u},
                                             [("sum", "v"), ("min", "v"), ("max", "u"), ("sum", "u")])
    assert rows == [[str(a), str(b), str(c_), str(d_), str(e_), str(f_)]
                    for a, b, c_, d_, e_, f_ in zip(keys, cnt, sv, mnv, mxu, su)]
    # COUNT(*) only, and AVG
    assert q(c, "SELECT k, COUNT(*) FROM w GROUP BY k").rows == [[str(a), str(b)] for a, b in zip(keys, cnt)]
    assert "group_part" in _kernels(c)
    for row, s_, n_ in zip(q(c, "SELECT k, AVG(v) FROM w GROUP BY k").rows, sv, cnt):
        assert abs(float(row[1]) - s_ / n_) <= 1e-9 * max(1.0, abs(s_ / n_)), row
    # HAVING / ORDER BY / LIMIT over the emitted groups
    top = q(c, "SELECT k, COUNT(*) AS c FROM w GROUP BY k ORDER BY c DESC, k LIMIT 5").rows
    want = sorted(zip(keys, cnt), key=lambda t: (-t[1], t[0]))[:5]
    assert top == [[str(a), str(b)] for a, b in want]
    c.close()


def test_partitioned_group_by_1e9_rows(mbx, oracle):
    """The c3h shape at 1e9 rows: 1e5 distinct INT64 keys, SUM(v) and COUNT(*)
    of every group against the oracle over all rows."""
    import os
    n, groups = 1_000_000_000, 100_000
    c = _conn(mbx)
    q(c, f"CREATE TABLE th AS SELECT mbx_synth(7, i, {groups}) AS k, "
         f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range({n}) tbl(i)")
    rr = c.query_raw("SELECT k, SUM(v), COUNT(*) FROM th GROUP BY k")
    rows, _ = rr.cells()
    rr.close()
    assert "group_part" in _kernels(c), _kernels(c)
    oc, osum = oracle.synth_groupby(7, 9, 0, n, groups, 1 << 40, -(1 << 39), min(32, max(8, len(os.sched_getaffinity(0)))))
    assert len(rows) == groups
    assert all(r[0] == str(g) and r[1] == str(osum[g]) and r[2] == str(oc[g]) for g, r in enumerate(rows))
    c.close()


def test_partitioned_group_by_unpacked_int64_values(mbx, oracle):
    """INT64 values whose zone map uses the top bits (|v| up to 2^49): the
    partition index cannot ride in the value, so keys and values travel as
    separate arrays; and values wide enough that no overflow-free piece size
    exists take the other GROUP BY paths -- both exact against numpy."""
    import numpy as np
    n, groups = 700_001, 20_000
    c = _conn(mbx)
    for span, kern in ((1 << 50, "group_part"), (1 << 60, None)):
        q(c, "DROP TABLE IF EXISTS wb")
        q(c, f"CREATE TABLE wb AS SELECT mbx_synth(7, i, {groups}) AS k, "
             f"mbx_synth(9, i, {span}) - {span // 2} AS v FROM range({n}) tbl(i)")
        k = oracle.synth_i64(n, 7, 0, groups, 0)
        v = oracle.synth_i64(n, 9, 0, span, -(span // 2))
        rows = q(c, "SELECT k, SUM(v), COUNT(*), MIN(v) FROM wb GROUP BY k ORDER BY k").rows
        if kern:
            assert kern in _kernels(c), _kernels(c)
        keys, cnt, sv, mnv = _np_groups(k, {"v": v}, [("sum", "v"), ("min", "v")])
        assert rows == [[str(a), str(s_), str(b), str(m)] for a, b, s_, m in zip(keys, cnt, sv, mnv)], span
    c.close()


# ---------------------------------------------------------------------------
# F3h: integer keys too sparse for dense states, hashed partitions
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("n,groups,mult,ktype", [
    (3_000_017, 100_000, 1_000_003, "BIGINT"), (2_000_003, 60_000, 20_011, "INTEGER"),
    (500_000, 400_000, -7_919_000_001, "BIGINT")])
def test_hashed_group_by_sparse_keys(mbx, oracle, n, groups, mult, ktype):
    """Keys spread over a range far wider than the rows (so no dense per-key
    states): rows hash-partitioned, each partition reduced in an LDS hash
    table, groups collected in a global hash table; against numpy, in any
    order (DuckDB's hash aggregate order is unspecified)."""
    c = _conn(mbx)
    q(c, f"CREATE TABLE hs AS SELECT CAST(mbx_synth(7, i, {groups}) * ({mult}) AS {ktype}) AS k, "
         f"mbx_synth(9, i, 2000000) - 1000000 AS v FROM range({n}) tbl(i)")
    k = oracle.synth_i64(n, 7, 0, groups, 0) * mult
    v = oracle.synth_i64(n, 9, 0, 2_000_000, -1_000_000)
    rows = q(c, "SELECT k, COUNT(*), SUM(v), MIN(v), MAX(v) FROM hs GROUP BY k").rows
    # F3h answered (no fallback to the hash path)
    assert "group_part_hashed" in _kernels(c) and "hash_group_assign" not in _kernels(c), _kernels(c)
    keys, cnt, sv, mnv, mxv = _np_groups(k, {"v": v}, [("sum", "v"), ("min", "v"), ("max", "v")])
    want = sorted([str(a), str(b), str(c_), str(d_), str(e_)] for a, b, c_, d_, e_ in zip(keys, cnt, sv, mnv, mxv))
    assert sorted(rows) == want
    assert sorted(q(c, "SELECT k, COUNT(*) FROM hs GROUP BY k").rows) == sorted([str(a), str(b)] for a, b in zip(keys, cnt))
    assert "group_part_hashed" in _kernels(c)
    c.close()


def test_hashed_group_by_edge_keys_and_overflow(mbx):
    """INT64_MIN (the key the tables keep apart), INT64_MAX, 0 and -1 as keys;
    and more groups than the hashed tables hold: the hash path answers, exact."""
    import numpy as np
    c = _conn(mbx)
    n = 1 << 17
    q(c, f"CREATE TABLE he AS SELECT CASE WHEN i % 5 = 0 THEN -9223372036854775807 - 1 "
         f"WHEN i % 5 = 1 THEN 9223372036854775807 WHEN i % 5 = 2 THEN 0 WHEN i % 5 = 3 THEN -1 "
         f"ELSE i * 1000003 END AS k, i AS v FROM range({n}) tbl(i)")
    i = np.arange(n, dtype=np.int64)
    k = np.where(i % 5 == 0, np.iinfo(np.int64).min, np.where(i % 5 == 1, np.iinfo(np.int64).max,
                 np.where(i % 5 == 2, 0, np.where(i % 5 == 3, -1, i * 1_000_003))))
    rows = q(c, "SELECT k, COUNT(*), SUM(v) FROM he GROUP BY k").rows
    assert "group_part_hashed" in _kernels(c) and "hash_group_assign" not in _kernels(c), _kernels(c)
    keys, cnt, sv = _np_groups(k, {"v": i}, [("sum", "v")])
    assert sorted(rows) == sorted([str(a), str(b), str(s_)] for a, b, s_ in zip(keys, cnt, sv))
    # 2.5M distinct sparse keys: beyond the hashed tables -> the hash path, still exact
    n2 = 2_500_000
    q(c, f"CREATE TABLE hb AS SELECT i * 1000003 AS k, i % 7 AS v FROM range({n2}) tbl(i)")
    r = c.query_raw("SELECT COUNT(*), SUM(c) FROM (SELECT k, COUNT(*) AS c FROM hb GROUP BY k) t")
    assert r.value(0, 0) == str(n2) and r.value(1, 0) == str(n2)
    r.close()
    assert "hash_group_assign" in _kernels(c), _kernels(c)  # the fallback answered
    c.close()


def test_hashed_group_by_1e9_rows(mbx, oracle):
    """1e9 rows, 1e5 distinct sparse INT64 keys (k = g x 2654435761): every
    group's COUNT and exact SUM against the oracle over all rows."""
    import os
    n, groups, mult = 1_000_000_000, 100_000, 2654435761
    c = _conn(mbx)
    q(c, f"CREATE TABLE th AS SELECT mbx_synth(7, i, {groups}) * {mult} AS k, "
         f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range({n}) tbl(i)")
    rr = c.query_raw("SELECT k, SUM(v), COUNT(*) FROM th GROUP BY k")
    rows, _ = rr.cells()
    rr.close()
    assert "group_part_hashed" in _kernels(c) and "hash_group_assign" not in _kernels(c), _kernels(c)
    oc, osum = oracle.synth_groupby(7, 9, 0, n, groups, 1 << 40, -(1 << 39), min(32, max(8, len(os.sched_getaffinity(0)))))
    got = sorted((int(r[0]), int(r[1]), int(r[2])) for r in rows)
    assert got == [(g * mult, osum[g], oc[g]) for g in range(groups)]
    c.close()


def test_hash_path_above_5e8_rows(mbx, oracle, monkeypatch):
    """The hash path itself at 6e8 rows (F3 / F3h off): its table is capped at
    2^30 entries, so the int32 scan over it holds (a 2^31-entry table returned no
    groups at all above 5.4e8 rows before round 6)."""
    import os
    n, groups = 600_000_000, 1000
    c = _conn(mbx)
    q(c, f"CREATE TABLE hp AS SELECT mbx_synth(7, i, {groups}) * 1000003 AS k, "
         f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range({n}) tbl(i)")
    monkeypatch.setenv("MBX_PART_GROUP", "0")
    rr = c.query_raw("SELECT k, SUM(v), COUNT(*) FROM hp GROUP BY k")
    rows, _ = rr.cells()
    rr.close()
    monkeypatch.delenv("MBX_PART_GROUP")
    assert "hash_group_assign" in _kernels(c), _kernels(c)
    oc, osum = oracle.synth_groupby(7, 9, 0, n, groups, 1 << 40, -(1 << 39), min(32, max(8, len(os.sched_getaffinity(0)))))
    assert sorted((int(r[0]), int(r[1]), int(r[2])) for r in rows) == [(g * 1000003, osum[g], oc[g]) for g in range(groups)]
    c.close()


@pytest.mark.parametrize("n,spread,mult,kern", [
    (50_001, 150_000, 1, "group_part"), (70_001, 150_000, 1_000_003, "group_part_hashed"),
    (4_097, 10_000, 1, "group_part"), (65_537, 9_000, -104_729, "group_part_hashed")])
def test_partitioned_group_by_skew_and_ragged(mbx, n, spread, mult, kern):
    """One key holding 90 % of the rows (one partition takes almost every row,
    so one partition spans many reduce pieces) and row counts just past a
    scatter tile, dense (F3) and sparse (F3h, from 2^16 rows) keys: exact
    against numpy."""
    import numpy as np
    c = _conn(mbx)
    q(c, f"CREATE TABLE sk AS SELECT CASE WHEN i % 10 = 0 THEN ((i * 7) % {spread}) * ({mult}) "
         f"ELSE CAST(4242 AS BIGINT) * ({mult}) END AS k, i % 1000 - 500 AS v FROM range({n}) tbl(i)")
    i = np.arange(n, dtype=np.int64)
    k = np.where(i % 10 == 0, ((i * 7) % spread) * mult, 4242 * mult)
    v = i % 1000 - 500
    rows = q(c, "SELECT k, COUNT(*), SUM(v), MIN(v), MAX(v) FROM sk GROUP BY k").rows
    assert kern in _kernels(c), _kernels(c)
    keys, cnt, sv, mnv, mxv = _np_groups(k, {"v": v}, [("sum", "v"), ("min", "v"), ("max", "v")])
    want = sorted([str(a), str(b), str(c_), str(d_), str(e_)] for a, b, c_, d_, e_ in zip(keys, cnt, sv, mnv, mxv))
    assert sorted(rows) == want
    c.close()
