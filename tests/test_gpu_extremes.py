"""INT64 extremes through the fused LDS-DMA kernels at ring-path sizes.

The fused kernels fold a range predicate lo <= x <= hi into one unsigned
compare (x - lo, as uint64) <= span.  These tests put INT64_MIN / INT64_MAX and
their neighbours into columns of 4.5e6 rows (the ring kernels' sizes, and
above select_rounds' 2^22-row threshold) and check predicates at and next to
both bounds against numpy, through filter_agg_lds (one column), filter_multi
(a conjunction over two columns), group_direct_lds (the WHERE form) and
select_rounds (materialising).  The reference's own extremes fixtures are
"bigint extremes" / "integer extremes" (src/duckdb_fixture_cases.mbt:26-32,
:96-102), which hold three-row tables; these widen them to the kernels'
sizes.  Parity bar: bit-exact (COUNT, int128 SUM, every selected row)."""
import numpy as np
import pytest

from conftest import q

pytestmark = pytest.mark.gpu

MIN, MAX = -2**63, 2**63 - 1
N = 4_500_007
EDGES = np.array([MIN, MIN + 1, MIN + 2, -2, -1, 0, 1, 2, MAX - 2, MAX - 1, MAX], dtype=np.int64)

# (SQL predicate on column c, numpy mask builder)
PREDS = [
    ("{c} > 9223372036854775806", lambda a: a == MAX),
    ("{c} >= 9223372036854775807", lambda a: a == MAX),
    ("{c} < -9223372036854775807", lambda a: a == MIN),
    ("{c} <= -9223372036854775808", lambda a: a == MIN),
    ("{c} > -9223372036854775808", lambda a: a != MIN),
    ("{c} < 9223372036854775807", lambda a: a != MAX),
    ("{c} >= -9223372036854775807", lambda a: a > MIN),
    ("{c} BETWEEN -9223372036854775808 AND -9223372036854775806", lambda a: a <= MIN + 2),
    ("{c} BETWEEN 9223372036854775805 AND 9223372036854775807", lambda a: a >= MAX - 2),
    ("{c} > 0", lambda a: a > 0),
    ("{c} <= -1", lambda a: a <= -1),
    ("{c} BETWEEN -1 AND 1", lambda a: (a >= -1) & (a <= 1)),
    ("{c} < 9223372036854775808", lambda a: np.ones(len(a), bool)),  # HUGEINT literal above the range
    ("{c} > -9223372036854775809", lambda a: np.ones(len(a), bool)),
]


def _extreme_col(rng, n):
    a = rng.integers(MIN, MAX, n, dtype=np.int64, endpoint=True)
    # every edge value many times, spread over the whole column
    pos = rng.choice(n, size=len(EDGES) * 2000, replace=False)
    a[pos] = np.repeat(EDGES, 2000)
    a[:len(EDGES)] = EDGES
    a[-len(EDGES):] = EDGES[::-1]
    return a


def _exact_sum(a):
    """Exact int128 sum of int64 values (32-bit halves, no overflow)."""
    hi = int(np.sum(a >> 32))
    lo = int(np.sum(a & 0xFFFFFFFF))
    return (hi << 32) + lo


@pytest.fixture(scope="module")
def ext(mbx):
    rng = np.random.default_rng(2024)
    x = _extreme_col(rng, N)
    y = _extreme_col(rng, N)
    k = rng.integers(0, 32, N).astype(np.int32)
    v = rng.integers(-2**39, 2**39, N).astype(np.int64)
    cfg = mbx.Config.create()
    cfg.set("mbx_profile", "true")
    c = mbx.connect_with_config(cfg).value
    q(c, "CREATE TABLE e (x BIGINT, y BIGINT, k INTEGER, v BIGINT)")
    ap = c.create_appender("main", "e").value
    for j, col in enumerate((x, y, k, v)):
        assert isinstance(ap.append_column(j, col), mbx.Ok)
    assert isinstance(ap.commit(N), mbx.Ok)
    ap.close()
    yield c, x, y, k, v
    c.close()


def _kernels(c):
    return [kk["name"] for kk in c.last_profile()["kernels"]]


@pytest.mark.parametrize("pred,mask", PREDS, ids=[p for p, _ in PREDS])
def test_extremes_filter_agg(ext, pred, mask):
    c, x, y, k, v = ext
    m = mask(x)
    got = q(c, f"SELECT COUNT(*), SUM(x) FROM e WHERE {pred.format(c='x')}").rows[0]
    assert int(got[0]) == int(m.sum())
    assert (got[1] == "" and not m.any()) or int(got[1]) == _exact_sum(x[m])
    assert "filter_agg" in _kernels(c) or not m.any() or m.all(), _kernels(c)


@pytest.mark.parametrize("i", range(0, len(PREDS), 2))
def test_extremes_filter_multi(ext, i):
    """A conjunction over two full-range columns (filter_multi), aggregating a third."""
    c, x, y, k, v = ext
    px, mx = PREDS[i]
    py, my = PREDS[(i + 5) % len(PREDS)]
    m = mx(x) & my(y)
    got = q(c, f"SELECT COUNT(*), SUM(v) FROM e WHERE {px.format(c='x')} AND {py.format(c='y')}").rows[0]
    assert int(got[0]) == int(m.sum())
    assert (got[1] == "" and not m.any()) or int(got[1]) == int(v[m].sum())


@pytest.mark.parametrize("pred,mask", PREDS[:12], ids=[p for p, _ in PREDS[:12]])
def test_extremes_group_direct_where(ext, pred, mask):
    """GROUP BY a 32-value INT32 key WHERE a full-range INT64 predicate column
    (group_direct_lds with its predicate slice in the ring)."""
    c, x, y, k, v = ext
    m = mask(x)
    res = q(c, f"SELECT k, SUM(v), COUNT(*) FROM e WHERE {pred.format(c='x')} GROUP BY k ORDER BY k").rows
    cnt = np.bincount(k[m], minlength=32)
    exp = [[str(g), str(int(v[m & (k == g)].sum())), str(int(cnt[g]))] for g in range(32) if cnt[g]]
    assert res == exp
    if m.any():
        assert "group_direct" in _kernels(c), _kernels(c)


@pytest.mark.parametrize("pred,mask", [PREDS[i] for i in (0, 2, 4, 7, 8, 11)],
                         ids=[PREDS[i][0] for i in (0, 2, 4, 7, 8, 11)])
def test_extremes_select_rounds(ext, pred, mask):
    """The materialising one-pass compaction: every selected row, in order."""
    c, x, y, k, v = ext
    m = mask(x)
    a = c.query_arrow(f"SELECT x, v FROM e WHERE {pred.format(c='x')}").value
    assert a.row_count() == int(m.sum())
    kinds = _kernels(c)
    bx, bv = a._buf("int64", 0), a._buf("int64", 1)
    a.close()
    cnt = int.from_bytes(bx[:4], "little", signed=True)
    assert cnt == int(m.sum())  # whole wire buffers (< 2^28 bytes), not the MoonBit decoders' 1e6-row cap
    assert np.array_equal(np.frombuffer(bx[4:4 + 8 * cnt], dtype=np.int64), x[m])
    assert np.array_equal(np.frombuffer(bv[4:4 + 8 * cnt], dtype=np.int64), v[m])
    assert "select_rounds" in kinds, kinds
