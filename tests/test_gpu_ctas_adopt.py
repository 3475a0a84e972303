"""CREATE TABLE AS / INSERT ... SELECT into an empty table take over the
query's output blocks (executor.cpp AdoptResultColumn) instead of allocating
and copying.  These tests pin what must not change when they do: the values,
the NULLs, the zone map (read by the planner for direct GROUP BY tables and
narrow staging), later appends growing the adopted column, a result that
names one block twice (SELECT x, x), and blocks going back to the pool when
the table is replaced.  Expected values come from numpy over the same rows."""
import numpy as np
import pytest

from conftest import one, q

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def src(mbx):
    c = mbx.connect().value
    n = 3_000_017
    rng = np.random.default_rng(11)
    x = rng.integers(1, 5000, n).astype(np.int64)
    y = rng.integers(-40, 40, n).astype(np.int32)
    vy = rng.random(n) > 0.25
    q(c, "CREATE TABLE d (x BIGINT, y INTEGER)")
    ap = c.create_appender("main", "d").value
    assert isinstance(ap.append_column(0, x), mbx.Ok)
    assert isinstance(ap.append_column(1, y, vy.astype(np.uint8)), mbx.Ok)
    assert isinstance(ap.commit(n), mbx.Ok)
    ap.close()
    yield mbx, c, x, y, vy
    c.close()


def _sums(x, y, vy):
    return [str(len(x)), str(int(x.sum())), str(int(x.min())), str(int(x.max())), str(int(vy.sum())),
            str(int(y[vy].sum()))]


def test_ctas_adopted_values_nulls_and_stats(src):
    mbx, c, x, y, vy = src
    q(c, "CREATE TABLE a AS SELECT x, x AS x2, y FROM d WHERE x > 2400")
    m = x > 2400
    got = one(c, "SELECT COUNT(*), SUM(x), MIN(x), MAX(x), COUNT(y), SUM(y) FROM a")
    assert got == _sums(x[m], y[m], vy[m])
    assert one(c, "SELECT SUM(x2), MIN(x2), MAX(x2) FROM a") == [str(int(x[m].sum())), str(int(x[m].min())),
                                                                 str(int(x[m].max()))]
    # the zone map of the adopted INTEGER column drives a direct-index GROUP BY
    res = q(c, "SELECT y, COUNT(*), SUM(x) FROM a GROUP BY y ORDER BY y NULLS LAST").rows
    ym, xm, vm = y[m], x[m], vy[m]
    exp = [[str(v), str(int(((ym == v) & vm).sum())), str(int(xm[(ym == v) & vm].sum()))]
           for v in sorted(set(ym[vm].tolist()))]
    exp.append(["", str(int((~vm).sum())), str(int(xm[~vm].sum()))])
    assert res == exp
    # positions survive: a selection over the adopted table in row order
    got = q(c, "SELECT x FROM a WHERE x2 > 4990").rows
    assert [r[0] for r in got] == [str(v) for v in x[m][x[m] > 4990]]
    q(c, "DROP TABLE a")


def test_adopted_column_grows_on_later_appends(src):
    mbx, c, x, y, vy = src
    q(c, "CREATE TABLE g AS SELECT x, y FROM d WHERE x > 2500")
    q(c, "INSERT INTO g SELECT x, y FROM d WHERE x < 30")
    q(c, "INSERT INTO g VALUES (123456789012, NULL), (-5, 7)")
    ap = c.create_appender("main", "g").value
    extra = np.arange(70_001, dtype=np.int64) * 3
    ey = (np.arange(70_001) % 11).astype(np.int32)
    assert isinstance(ap.append_column(0, extra), mbx.Ok)
    assert isinstance(ap.append_column(1, ey), mbx.Ok)
    assert isinstance(ap.commit(len(extra)), mbx.Ok)
    ap.close()
    m1, m2 = x > 2500, x < 30
    xs = np.concatenate([x[m1], x[m2], [123456789012, -5], extra])
    ys = np.concatenate([y[m1], y[m2], [0, 7], ey]).astype(np.int64)
    vs = np.concatenate([vy[m1], vy[m2], [False, True], np.ones(len(extra), bool)])
    got = one(c, "SELECT COUNT(*), SUM(x), MIN(x), MAX(x), COUNT(y), SUM(y) FROM g")
    assert got == _sums(xs, ys, vs)
    # the appended rows' zone map folded into the adopted one
    assert one(c, "SELECT COUNT(*) FROM g WHERE x >= 123456789012") == ["1"]
    assert one(c, "SELECT COUNT(*) FROM g WHERE x < 0") == ["1"]
    q(c, "DROP TABLE g")


def test_replaced_tables_return_blocks_and_stay_exact(src):
    mbx, c, x, y, vy = src
    for lo in (2400, 1000, 2400, 4000, 2400):
        q(c, f"CREATE OR REPLACE TABLE r AS SELECT x, y FROM d WHERE x > {lo}")
        m = x > lo
        assert one(c, "SELECT COUNT(*), SUM(x), MIN(x), MAX(x), COUNT(y), SUM(y) FROM r") == \
            _sums(x[m], y[m], vy[m])
    # a selective filter keeps the copy (its block is sized for every input row)
    q(c, "CREATE OR REPLACE TABLE r AS SELECT x, y FROM d WHERE x = 7")
    m = x == 7
    assert one(c, "SELECT COUNT(*), SUM(x), MIN(x), MAX(x), COUNT(y), SUM(y) FROM r") == _sums(x[m], y[m], vy[m])
    q(c, "DROP TABLE r")


def test_kernel_zone_map_drives_narrow_staging(mbx):
    """select_rounds returns its outputs' zone maps for CREATE TABLE AS; a
    missed extreme would let a later selection stage the column as int32 and
    truncate it (narrow staging trusts the map), so the extremes sit in a few
    rows among 5e6 small values, NULLs mixed in."""
    c = mbx.connect().value
    n = 5_000_000
    rng = np.random.default_rng(3)
    x = rng.integers(-1000, 1000, n).astype(np.int64)
    idx = rng.choice(n, 6, replace=False)
    x[idx] = [2**40, -(2**41), 2**31, -(2**31) - 1, 2**62, -(2**62)]
    vx = rng.random(n) > 0.1
    vx[idx] = True
    q(c, "CREATE TABLE b (x BIGINT)")
    ap = c.create_appender("main", "b").value
    assert isinstance(ap.append_column(0, x, vx.astype(np.uint8)), mbx.Ok)
    assert isinstance(ap.commit(n), mbx.Ok)
    ap.close()
    for pred, m in (("x > -4611686018427387905", vx), ("x > -900", (x > -900) & vx),
                    ("x BETWEEN -2147483649 AND 2147483648", (x >= -(2**31) - 1) & (x <= 2**31) & vx)):
        q(c, f"CREATE OR REPLACE TABLE bz AS SELECT x FROM b WHERE {pred}")
        xm = x[m]
        for sel, mm in (("x > 999", xm > 999), ("x < -1000", xm < -1000)):
            got = q(c, f"SELECT x FROM bz WHERE {sel}").rows
            assert [int(r[0]) for r in got] == [int(v) for v in xm[mm]]
        assert one(c, "SELECT COUNT(*), COUNT(x), MIN(x), MAX(x), SUM(x) FROM bz") == \
            [str(len(xm)), str(len(xm)), str(int(xm.min())), str(int(xm.max())), str(int(xm.sum()))]
    c.close()


def test_ctas_of_table_columns_and_casts(src):
    mbx, c, x, y, vy = src
    # an unfiltered projection of table columns (no result block to take) and
    # a cast (a new block from the cast kernel) side by side
    q(c, "CREATE TABLE t2 AS SELECT x, CAST(y AS BIGINT) AS yb FROM d")
    assert one(c, "SELECT SUM(x), COUNT(yb), SUM(yb) FROM t2") == [str(int(x.sum())), str(int(vy.sum())),
                                                                  str(int(y[vy].astype(np.int64).sum()))]
    q(c, "DROP TABLE t2")


@pytest.mark.parametrize("shape", ["x", "x, k, y", "y", "k"])
def test_kernel_zone_map_folds_tail_rows(mbx, shape):
    """select_rounds' workgroup 0 writes the rows after the
    last full step (< 256 H of them) and must fold them into the zone map it
    hands CREATE TABLE AS.  The extremes sit in the last rows of an input
    whose size is not a multiple of 512: an INT64 beyond int32 (narrow
    staging), an INTEGER key far outside 0..31 (direct GROUP BY range) and
    INT32_MAX in a NULL-able BIGINT (the NULL sentinel of a narrow column)."""
    c = mbx.connect().value
    n = (1 << 22) + 300_311  # above select_rounds' 2^22-row floor; n % 512 != 0
    rng = np.random.default_rng(17)
    x = rng.integers(-1000, 1000, n).astype(np.int64)
    k = rng.integers(0, 32, n).astype(np.int32)
    y = rng.integers(-5000, 5000, n).astype(np.int64)
    vy = rng.random(n) > 0.2
    x[-1], x[-7] = 2**40, -(2**41)
    k[-2], k[-5] = 1000, -77
    y[-3], vy[-3] = 2**31 - 1, True
    y[-9], vy[-9] = -(2**31) + 1, True  # (INT32_MIN stays free: the sentinel a correct map picks)
    q(c, "CREATE TABLE s (x BIGINT, k INTEGER, y BIGINT)")
    ap = c.create_appender("main", "s").value
    assert isinstance(ap.append_column(0, x), mbx.Ok)
    assert isinstance(ap.append_column(1, k), mbx.Ok)
    assert isinstance(ap.append_column(2, y, vy.astype(np.uint8)), mbx.Ok)
    assert isinstance(ap.commit(n), mbx.Ok)
    ap.close()
    m = x != 12345  # every row but a handful: the selection runs, the tail is selected
    q(c, f"CREATE TABLE z AS SELECT {shape} FROM s WHERE x <> 12345")
    xm, km, ym, vm = x[m], k[m], y[m], vy[m]
    if "x" in shape:
        assert one(c, "SELECT MIN(x), MAX(x) FROM z") == [str(int(xm.min())), str(int(xm.max()))]
        got = q(c, "SELECT x FROM z WHERE x > 999").rows
        assert [int(r[0]) for r in got] == [int(v) for v in xm[xm > 999]]
        got = q(c, "SELECT x FROM z WHERE x < -1000").rows
        assert [int(r[0]) for r in got] == [int(v) for v in xm[xm < -1000]]
    if "k" in shape:
        res = q(c, "SELECT k, COUNT(*) FROM z GROUP BY k ORDER BY k").rows
        ks, cs = np.unique(km, return_counts=True)
        assert res == [[str(int(a)), str(int(b))] for a, b in zip(ks, cs)]
    if "y" in shape:
        yv = ym[vm]
        assert one(c, "SELECT COUNT(*), COUNT(y), MIN(y), MAX(y), SUM(y) FROM z") == \
            [str(len(ym)), str(len(yv)), str(int(yv.min())), str(int(yv.max())), str(int(yv.sum()))]
        got = q(c, "SELECT y FROM z WHERE y > 4999 OR y < -5000").rows
        assert [int(r[0]) for r in got] == [int(v) for v in yv[(yv > 4999) | (yv < -5000)]]
        if "x" in shape:
            # a narrow-staged NULL-able selection: INT32_MAX must stay a value, the NULLs NULL
            got = q(c, "SELECT y FROM z WHERE x > -2000000")
            sel = xm > -2000000
            assert [None if nl[0] else int(r[0]) for r, nl in zip(got.rows, got.nulls)] == \
                [int(v) if ok else None for v, ok in zip(ym[sel], vm[sel])]
    c.close()
