"""A device result that reads table columns in place outlives the table's
buffers as they were: a plain projection (`SELECT v FROM t`) and a LIMIT /
OFFSET slice hand the table's own buffers to the Arrow result or stream, so an
append that regrows the column (a new buffer, the old one released) or a DROP
must not free memory such a result still reads.  The table buffers are
shared-owned (DevColumn::*_owner, DCol::pins); these tests read the results
after both and compare with the rows as they were when the query ran (the
full 64-bit wire values: the MoonBit decoders keep only the low word)."""
import numpy as np
import pytest

from conftest import q

pytestmark = pytest.mark.gpu


def _fill(mbx, c, name, v, vv):
    ap = c.create_appender("main", name).value
    assert isinstance(ap.append_column(0, v), mbx.Ok)
    assert isinstance(ap.append_column(1, v.astype(np.int64) * 3, vv.astype(np.uint8)), mbx.Ok)
    assert isinstance(ap.commit(len(v)), mbx.Ok)
    ap.close()


def _same(got, exp, what):
    got, exp = np.asarray(got, dtype=np.int64), np.asarray(exp, dtype=np.int64)
    assert got.shape == exp.shape, f"{what}: {got.shape} rows vs {exp.shape}"
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, f"{what}: {len(bad)} mismatches, first at {bad[0]}: {got[bad[0]]} vs {exp[bad[0]]}"


def test_results_outlive_regrow_and_drop(mbx):
    c = mbx.connect().value
    n = 200_000
    rng = np.random.default_rng(17)
    v = rng.integers(-10**12, 10**12, n).astype(np.int64)
    vv = rng.random(n) > 0.3
    q(c, "CREATE TABLE lt (v BIGINT, w BIGINT)")
    _fill(mbx, c, "lt", v, vv)
    q(c, "INSERT INTO lt VALUES (-1, NULL), (-1, NULL)")
    strs = "CASE WHEN i % 3 = 0 THEN 'a' WHEN i % 3 = 1 THEN 'bb' ELSE NULL END"
    q(c, f"CREATE TABLE ls AS SELECT {strs} AS s FROM range(200002) tbl(i)")
    ev = np.concatenate([v, [-1, -1]])
    ew = np.concatenate([v * 3, [0, 0]])
    evalid = np.concatenate([vv, [False, False]])
    whole = c.query_arrow("SELECT v FROM lt").value
    nul = c.query_arrow("SELECT w FROM lt").value
    sl = c.query_arrow("SELECT v, w FROM lt LIMIT 70000 OFFSET 640").value   # bitmap slice on a word
    sl2 = c.query_arrow("SELECT v FROM lt LIMIT 1000 OFFSET 333").value      # values only: any offset
    st = c.query_stream("SELECT s FROM ls").value
    _same(c.query_arrow("SELECT v FROM lt").value.raw_int64(0), ev, "before the appends")
    # regrow every column (200k -> 4.2M rows: new buffers, string offsets and
    # chars included), then drop the tables
    more = np.arange(4_000_000, dtype=np.int64)
    _fill(mbx, c, "lt", more, np.ones(len(more), bool))
    assert c.query("SELECT COUNT(*) FROM lt").value.rows == [[str(n + 2 + len(more))]]
    for _ in range(3):
        q(c, f"INSERT INTO ls SELECT {strs} FROM range(4000000) tbl(i)")
    q(c, "DROP TABLE lt")
    q(c, "DROP TABLE ls")
    q(c, "CREATE TABLE lt (v BIGINT, w BIGINT)")  # new buffers may land where the old ones were
    _fill(mbx, c, "lt", more[:300_000] * 7, np.ones(300_000, bool))
    _same(whole.raw_int64(0), ev, "whole")
    vals, valid = nul._nullable("int64", 0, 8, "q")
    _same(valid, evalid, "validity")
    _same(np.asarray(vals)[evalid], ew[evalid], "NULL-able values")
    _same(sl.raw_int64(0), ev[640:70640], "slice")
    vals, valid = sl._nullable("int64", 1, 8, "q")
    _same(valid, evalid[640:70640], "slice validity")
    _same(sl2.raw_int64(0), ev[333:1333], "slice at 333")
    got_s = []
    while True:
        ch = st.next().value
        if ch is None:
            break
        got_s += [r[0] for r in ch.rows]
    assert got_s == [["a", "bb", ""][i % 3] for i in range(200002)]
    for r in (whole, nul, sl, sl2):
        r.close()
    st.close()
    c.close()


def test_limit_offset_slices_match_numpy(mbx):
    c = mbx.connect().value
    n = 1_000_003
    rng = np.random.default_rng(23)
    v = rng.integers(-2**62, 2**62, n).astype(np.int64)
    vv = rng.random(n) > 0.1
    w = v * 3  # (wraps, as the appended column does)
    q(c, "CREATE TABLE ls (v BIGINT, w BIGINT)")
    _fill(mbx, c, "ls", v, vv)
    for lim, off in ((10, 0), (1000, 64), (12345, 999_990), (5, n + 10), (0, 5), (70_000, 777)):
        got = c.query(f"SELECT v, w FROM ls LIMIT {lim} OFFSET {off}").value.rows
        sel = slice(off, off + lim)
        assert [int(r[0]) for r in got] == v[sel].tolist()
        assert [r[1] for r in got] == [str(x) if ok else "" for x, ok in zip(w[sel], vv[sel])]
    # a slice inside a subquery still aggregates right (the subquery takes the gather)
    m = v[100:100_100]
    assert c.query("SELECT COUNT(*), SUM(v) FROM (SELECT v FROM ls LIMIT 100000 OFFSET 100) q").value.rows == \
        [[str(len(m)), str(sum(int(x) for x in m))]]  # HUGEINT sum: no int64 wrap
    c.close()
