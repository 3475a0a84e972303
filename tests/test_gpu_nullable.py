"""NULL-able columns on the fused filter-aggregate (filter_multi_lds: the
step's validity words ride the LDS-DMA ring) — the C2/C5 shapes over columns
with NULLs — checked against numpy on the oracle's generator arrays.  DuckDB
rules: a NULL fails a comparison; COUNT(x)/SUM/MIN/MAX skip NULLs; SUM of no
rows is NULL."""
import numpy as np
import pytest

from conftest import q

pytestmark = pytest.mark.gpu


def _num(cell):
    return None if cell is None or cell == "" else int(cell)


@pytest.mark.parametrize("n", [1, 255, 256, 257, 4097, 100_003, 2_000_011])
def test_filter_aggregate_nullable(mbx, oracle, n):
    cfg = mbx.Config.create()
    cfg.set("mbx_profile", "true")
    c = mbx.connect_with_config(cfg).value
    q(c, f"CREATE TABLE tn AS SELECT mbx_synth(42, i, 50) + 1 AS x, "
         f"CASE WHEN mbx_synth(13, i, 10) = 0 THEN NULL ELSE mbx_synth(42, i, 50) + 1 END AS xn, "
         f"CASE WHEN mbx_synth(17, i, 3) = 0 THEN NULL ELSE CAST(mbx_synth(7, i, 32) AS INTEGER) END AS kn, "
         f"CASE WHEN mbx_synth(19, i, 7) = 0 THEN NULL ELSE mbx_synth(9, i, 1099511627776) - 549755813888 END AS vn "
         f"FROM range({n}) tbl(i)")
    x = oracle.synth_i64(n, 42, 0, 50, 1)
    xv = oracle.synth_i64(n, 13, 0, 10, 0) != 0
    k = oracle.synth_i64(n, 7, 0, 32, 0)
    kv = oracle.synth_i64(n, 17, 0, 3, 0) != 0
    v = oracle.synth_i64(n, 9, 0, 2**40, -2**39)
    vv = oracle.synth_i64(n, 19, 0, 7, 0) != 0

    def agg(vals, m):
        sel = vals[m].astype(object)
        return [int(m.sum()), int(sel.sum()) if m.any() else None,
                int(vals[m].min()) if m.any() else None, int(vals[m].max()) if m.any() else None]

    cases = [
        # C2 / C5 shapes over a NULL-able column
        ("SELECT COUNT(*) FROM tn WHERE xn > 24", lambda: [int((xv & (x > 24)).sum())]),
        ("SELECT COUNT(*), SUM(xn), MIN(xn), MAX(xn) FROM tn WHERE xn > 24", lambda: agg(x, xv & (x > 24))),
        # NULL-able aggregated column without a predicate on it (no COUNT(*))
        ("SELECT COUNT(vn), SUM(vn), MIN(vn), MAX(vn) FROM tn WHERE x > 24", lambda: agg(v, vv & (x > 24))),
        # NULL-able predicate columns of two widths
        ("SELECT COUNT(vn), SUM(vn), MIN(vn), MAX(vn) FROM tn WHERE xn > 24 AND kn < 16",
         lambda: agg(v, vv & xv & (x > 24) & kv & (k < 16))),
        ("SELECT COUNT(*) FROM tn WHERE xn BETWEEN 10 AND 40 AND kn >= 3",
         lambda: [int((xv & (x >= 10) & (x <= 40) & kv & (k >= 3)).sum())]),
    ]
    for sql, want in cases:
        got = [_num(cell) for cell in q(c, sql).rows[0]]
        assert got == want(), (n, sql)
        names = [kk["name"] for kk in c.last_profile()["kernels"]]
        if n >= 4097:  # tiny tables may hold no NULLs at all (then no validity, the F1 kernel)
            assert "filter_multi" in names, (sql, names)
    # COUNT(*) next to an aggregate of a NULL-able column without a predicate on it:
    # another kernel answers (the two counts differ); the result must still be exact
    m = x > 24
    got = [_num(cell) for cell in q(c, "SELECT COUNT(*), COUNT(vn), SUM(vn) FROM tn WHERE x > 24").rows[0]]
    assert got == [int(m.sum()), int((m & vv).sum()), int(v[m & vv].astype(object).sum()) if (m & vv).any() else None]
    c.close()


@pytest.mark.parametrize("n", [1, 1000, 100_003, 3_000_017])
def test_filter_aggregate_minmax_int32_mode(conn, oracle, n):
    """MIN/MAX of the fused filter-aggregate run in int32 when the zone map
    bounds |value| below 2^31 (filter_agg_lds MM = 2): values at the int32
    edges, empty selections and a column just past the bound (int64 mode)."""
    v = oracle.synth_i64(n, 9, 0, 2**40, -2**39)
    x = oracle.synth_i64(n, 42, 0, 50, 1)
    for name, bound in (("edge", 2**31 - 1), ("past", 2**31)):
        # values spread over [-bound, bound] with both ends present
        vals = (v % (2 * bound + 1)) - bound
        vals[0] = bound
        if n > 1:
            vals[1] = -bound
        q(conn, "DROP TABLE IF EXISTS mm")
        q(conn, f"CREATE TABLE mm AS SELECT mbx_synth(42, i, 50) + 1 AS x, "
                f"(mbx_synth(9, i, 1099511627776) - 549755813888) % {2 * bound + 1} AS r FROM range({n}) tbl(i)")
        # the same values as numpy (truncated modulo, as in SQL), then shifted
        r = np.fmod(v, 2 * bound + 1)
        for sql, m in ((f"SELECT COUNT(*), SUM(r), MIN(r), MAX(r) FROM mm WHERE r > {-bound // 3}", r > -bound // 3),
                       ("SELECT COUNT(*), MIN(r), MAX(r) FROM mm WHERE r > 99999999999", r > 99999999999),
                       ("SELECT MIN(r), MAX(r) FROM mm", np.ones(n, bool))):
            got = [_num(c) for c in q(conn, sql).rows[0]]
            sel = r[m]
            mn = int(sel.min()) if m.any() else None
            mx = int(sel.max()) if m.any() else None
            if sql.startswith("SELECT COUNT(*), SUM"):
                want = [int(m.sum()), int(sel.astype(object).sum()) if m.any() else None, mn, mx]
            elif sql.startswith("SELECT COUNT(*), MIN"):
                want = [int(m.sum()), mn, mx]
            else:
                want = [mn, mx]
            assert got == want, (n, name, sql)
