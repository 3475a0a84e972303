"""COUNT(DISTINCT ...) against numpy (the oracle of a set count).

The binder keeps DISTINCT only on COUNT (MIN/MAX DISTINCT are MIN/MAX; SUM /
AVG DISTINCT are rejected), and the device answers it with two aggregations
per distinct aggregate (the distinct (groups..., arg) pairs, then COUNT(arg)
of the pairs per group) merged by group key into the other aggregates.  Round
2 compared COUNT(DISTINCT) of a sharded table only with an unsharded
connection of the same engine, which hid that both returned COUNT(arg); these
tests pin it to independent numbers, NULLs (not counted) and VARCHAR
arguments included."""
import numpy as np
import pytest

from conftest import one, q

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dt(mbx):
    c = mbx.connect().value
    n = 2_000_003
    rng = np.random.default_rng(5)
    x = rng.integers(0, 5000, n).astype(np.int64)
    k = rng.integers(0, 7, n).astype(np.int32)
    y = rng.integers(-3, 3, n).astype(np.int32)
    vy = rng.random(n) > 0.2
    q(c, "CREATE TABLE d (x BIGINT, k INTEGER, y INTEGER)")
    ap = c.create_appender("main", "d").value
    assert isinstance(ap.append_column(0, x), mbx.Ok)
    assert isinstance(ap.append_column(1, k), mbx.Ok)
    assert isinstance(ap.append_column(2, y, vy.astype(np.uint8)), mbx.Ok)
    assert isinstance(ap.commit(n), mbx.Ok)
    ap.close()
    yield c, x, k, y, vy
    c.close()


def test_count_distinct_global(dt):
    c, x, k, y, vy = dt
    assert one(c, "SELECT COUNT(DISTINCT x) FROM d") == [str(len(np.unique(x)))]
    m = (x > 2400) & (k < 3)
    assert one(c, "SELECT COUNT(DISTINCT x) FROM d WHERE x > 2400 AND k < 3") == [str(len(np.unique(x[m])))]
    # NULLs are not counted; mixed with plain aggregates in one query
    got = one(c, "SELECT COUNT(DISTINCT y), COUNT(y), COUNT(*), SUM(x), COUNT(DISTINCT k) FROM d")
    assert got == [str(len(np.unique(y[vy]))), str(int(vy.sum())), str(len(x)), str(int(x.sum())),
                   str(len(np.unique(k)))]
    # nothing passes: 0, not NULL
    assert one(c, "SELECT COUNT(DISTINCT x), COUNT(*) FROM d WHERE x > 100000") == ["0", "0"]


def test_count_distinct_grouped(dt):
    c, x, k, y, vy = dt
    res = q(c, "SELECT k, COUNT(DISTINCT x), SUM(x), COUNT(DISTINCT y) FROM d GROUP BY k ORDER BY k").rows
    exp = [[str(g), str(len(np.unique(x[k == g]))), str(int(x[k == g].sum())),
            str(len(np.unique(y[(k == g) & vy])))] for g in range(7)]
    assert res == exp
    # HAVING over a distinct count
    res = q(c, "SELECT y, COUNT(DISTINCT k) AS nk FROM d WHERE x < 10 GROUP BY y HAVING COUNT(DISTINCT k) > 0 "
               "ORDER BY y NULLS LAST").rows
    m = x < 10
    exp = [[str(v), str(len(np.unique(k[m & vy & (y == v)])))] for v in sorted(set(y[m & vy].tolist()))]
    if (m & ~vy).any():
        exp.append(["", str(len(np.unique(k[m & ~vy])))])
    assert res == exp


def test_count_distinct_varchar(conn):
    q(conn, "CREATE TABLE s AS SELECT CASE WHEN i % 5 = 0 THEN NULL WHEN i % 3 = 0 THEN 'a' "
            "WHEN i % 3 = 1 THEN 'bb' ELSE 'c' END AS v, i % 4 AS g FROM range(100000) tbl(i)")
    assert one(conn, "SELECT COUNT(DISTINCT v), COUNT(v) FROM s") == ["3", "80000"]
    assert q(conn, "SELECT g, COUNT(DISTINCT v) FROM s GROUP BY g ORDER BY g").rows == \
        [[str(g), "3"] for g in range(4)]
