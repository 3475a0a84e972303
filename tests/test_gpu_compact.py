"""Filter -> compaction against the CPU oracle's generator arrays: the
round-synchronous one-pass kernel (dev::SelectRounds; the default from
MBX_SR_MIN_ROWS rows, forced at every size with MBX_SR_MIN_ROWS=0), the
count-first two-pass form (dev::FilterCountChunks + scan +
dev::CompactRecompute, when every predicate column is an output; MBX_SL=0),
the ballot-bits two-pass form (dev::FilterBits + scan + dev::CompactColumns;
MBX_SL=0 MBX_CC=0) and the VM path (MBX_FC=0) must all give the selected rows of every
output column, in row order, bit for bit.  Sizes straddle the 256-row step,
the one-pass tiles (4 S steps per workgroup and round) and the grid-stride
(partial last step, one-row tail, many rounds per workgroup)."""
import numpy as np
import pytest

from conftest import one, q

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 255, 256, 257, 4095, 4096, 4097, 12_289, 1_000_003, 30_000_017]


def _col(conn, sql, kind, idx=0):
    a = conn.query_arrow(sql).value
    b = a._buf(kind, idx)
    a.close()
    n = int.from_bytes(b[:4], "little", signed=True) if len(b) >= 4 else 0
    return np.frombuffer(b[4:4 + n * (8 if kind in ("int64", "double") else 4)],
                         dtype=np.int64 if kind == "int64" else np.int32 if kind == "int32" else np.float64)


def _table(conn, oracle, n):
    q(conn, "DROP TABLE IF EXISTS fc")
    q(conn, f"CREATE TABLE fc AS SELECT mbx_synth(42, i, 50) + 1 AS x, CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
            f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v, "
            f"CAST(mbx_synth(11, i, 1000) - 500 AS SMALLINT) AS s, "
            f"CAST(mbx_synth(9, i, 1099511627776) - 549755813888 AS HUGEINT) * 1000000000000 AS h "
            f"FROM range({n}) tbl(i)")
    return (oracle.synth_i64(n, 42, 0, 50, 1), oracle.synth_i64(n, 7, 0, 32, 0),
            oracle.synth_i64(n, 9, 0, 2**40, -2**39), oracle.synth_i64(n, 11, 0, 1000, -500))


@pytest.mark.parametrize("n", SIZES)
def test_filter_compact_parity(conn, oracle, monkeypatch, n):
    x, k, v, s = _table(conn, oracle, n)
    cases = [
        ("SELECT x FROM fc WHERE x > 24", x > 24, [("int64", x)]),
        ("SELECT k, v FROM fc WHERE x > 24 AND k < 16", (x > 24) & (k < 16), [("int32", k), ("int64", v)]),
        ("SELECT v, x FROM fc WHERE x BETWEEN 10 AND 40 AND k >= 3 AND v > 0",
         (x >= 10) & (x <= 40) & (k >= 3) & (v > 0), [("int64", v), ("int64", x)]),
        ("SELECT x FROM fc WHERE x >= 1", np.ones(n, bool), [("int64", x)]),
    ]
    for sql, m, cols in cases:
        for i, (kind, arr) in enumerate(cols):
            got = _col(conn, sql, kind, i)
            assert np.array_equal(got, arr[m].astype(got.dtype)), (n, sql, i)
        # every other form: the same rows
        for envs in ({"MBX_SR_MIN_ROWS": "0"}, {"MBX_SL": "0"}, {"MBX_SL": "0", "MBX_CC": "0"},
                     {"MBX_FC": "0"}):
            for env, val in envs.items():
                monkeypatch.setenv(env, val)
            for i, (kind, arr) in enumerate(cols):
                got = _col(conn, sql, kind, i)
                assert np.array_equal(got, arr[m].astype(got.dtype)), (n, sql, i, envs)
            for env in envs:
                monkeypatch.delenv(env)
    # nothing passes: typed empty result
    r = q(conn, "SELECT x, k FROM fc WHERE x > 100")
    assert r.rows == [] and r.column_types == ["BigInt", "Integer"]
    # 2- and 16-byte outputs (SMALLINT, HUGEINT) through CTAS, checked by aggregates
    m = (x > 24) & (k < 16)
    q(conn, "CREATE OR REPLACE TABLE fc2 AS SELECT s, h, x FROM fc WHERE x > 24 AND k < 16")
    got = one(conn, "SELECT COUNT(*), SUM(s), SUM(h), SUM(x) FROM fc2")
    exp_h = int(v[m].astype(object).sum()) * 10**12
    assert [int(g) if g else 0 for g in got] == [int(m.sum()), int(s[m].sum()), exp_h, int(x[m].sum())], n
    if m.sum():
        first = np.flatnonzero(m)[0]
        assert q(conn, "SELECT s, h FROM fc2 LIMIT 1").rows[0] == [str(s[first]), str(int(v[first]) * 10**12)]


def test_filter_compact_decimal_predicate(conn, oracle):
    n = 100_003
    x = oracle.synth_i64(n, 42, 0, 50, 1)
    q(conn, "DROP TABLE IF EXISTS fcd")
    q(conn, f"CREATE TABLE fcd AS SELECT CAST(mbx_synth(42, i, 50) + 1 AS DECIMAL(15,2)) AS q, i AS r "
            f"FROM range({n}) tbl(i)")
    got = _col(conn, "SELECT r FROM fcd WHERE q > 24", "int64")  # DECIMAL literal folded to raw > 2400
    assert np.array_equal(got, np.flatnonzero(x > 24))
    got = _col(conn, "SELECT r FROM fcd WHERE q >= 24.5 AND q < 30", "int64")
    assert np.array_equal(got, np.flatnonzero((x >= 25) & (x < 30)))


def test_filter_compact_runs_the_hip_passes(mbx, oracle, monkeypatch):
    cfg = mbx.Config.create()
    cfg.set("mbx_profile", "true")
    c = mbx.connect_with_config(cfg).value
    n = 200_003
    x, k, v, s = _table(c, oracle, n)
    # a predicate column (x) that is not an output: ballot bits between the passes
    got = _col(c, "SELECT v, k FROM fc WHERE x > 24 AND k < 16", "int64")
    names = [kk["name"] for kk in c.last_profile()["kernels"]]
    assert "filter_bits" in names and "compact" in names, names
    assert np.array_equal(got, v[(x > 24) & (k < 16)])
    # every predicate column is an output: per-chunk counts, predicates re-evaluated in pass 2
    got = _col(c, "SELECT k, x FROM fc WHERE x > 24 AND k < 16", "int32")
    names = [kk["name"] for kk in c.last_profile()["kernels"]]
    assert "filter_count" in names and "compact" in names and "filter_bits" not in names, names
    assert np.array_equal(got, k[(x > 24) & (k < 16)])
    monkeypatch.setenv("MBX_SR_MIN_ROWS", "0")  # the round-synchronous one pass (default from 2^22 rows)
    for sql, col, m in (("SELECT v, k FROM fc WHERE x > 24 AND k < 16", v, (x > 24) & (k < 16)),
                        ("SELECT x FROM fc WHERE x > 24", x, x > 24)):
        got = _col(c, sql, "int64")
        names = [kk["name"] for kk in c.last_profile()["kernels"]]
        assert "select_rounds" in names and "filter_bits" not in names and "filter_count" not in names, names
        assert np.array_equal(got, col[m])
    c.close()


_SHAPE_CASES = [
    ("SELECT k FROM fc WHERE k < 5", lambda x, k, v: k < 5, ["k"]),
    ("SELECT x FROM fc WHERE x > 24", lambda x, k, v: x > 24, ["x"]),
    ("SELECT x, k FROM fc WHERE x > 24 AND k <= 16", lambda x, k, v: (x > 24) & (k <= 16), ["x", "k"]),
    ("SELECT v, x, k FROM fc WHERE v > 0 AND x < 30", lambda x, k, v: (v > 0) & (x < 30), ["v", "x", "k"]),
    ("SELECT k, v FROM fc WHERE x BETWEEN 10 AND 40 AND k >= 3 AND v > 0",
     lambda x, k, v: (x >= 10) & (x <= 40) & (k >= 3) & (v > 0), ["k", "v"]),
    ("SELECT x FROM fc WHERE x >= 1", lambda x, k, v: np.ones(len(x), bool), ["x"]),
]


@pytest.mark.parametrize("s_,depth,stg,sleep,h", [(2, 0, 0, 1, 2), (1, 2, 512, 0, 2), (1, 2, 256, 0, 1),
                                                  (2, 3, 1024, 4, 2), (8, 6, 2048, 1, 1), (4, 4, 4096, 2, 2),
                                                  (3, 3, 4096, 1, 1)])
def test_select_rounds_launch_shapes(mbx, oracle, monkeypatch, s_, depth, stg, sleep, h):
    """Every tile size (S steps per loader and round), sub-steps per step (H),
    ring depth, staging ring (one step: the loader waits on its storer every
    step when every row passes) and poll back-off of the round-synchronous
    kernel, over many rounds per workgroup (meta-slot reuse) and the 1..4-column
    loaded sets: exact rows in order."""
    monkeypatch.setenv("MBX_SR_MIN_ROWS", "0")
    monkeypatch.setenv("MBX_SR_H", str(h))
    monkeypatch.setenv("MBX_SR_S", str(s_))
    if depth:
        monkeypatch.setenv("MBX_SR_DEPTH", str(depth))
    if stg:
        monkeypatch.setenv("MBX_SR_STG", str(stg))
    monkeypatch.setenv("MBX_SR_SLEEP", str(sleep))
    cfg = mbx.Config.create()
    cfg.set("mbx_profile", "true")
    c = mbx.connect_with_config(cfg).value
    n = 20_000_077
    x, k, v, s = _table(c, oracle, n)
    arrs = {"x": ("int64", x), "k": ("int32", k), "v": ("int64", v)}
    for sql, mf, names in _SHAPE_CASES:
        m = mf(x, k, v)
        for i, nm in enumerate(names):
            kind, arr = arrs[nm]
            got = _col(c, sql, kind, i)
            if stg >= 512 or len(names) == 1:  # multi-column steps need 512 staging rows (H = 2)
                assert "select_rounds" in [kk["name"] for kk in c.last_profile()["kernels"]], sql
            assert np.array_equal(got, arr[m].astype(got.dtype)), (sql, i)
    c.close()


def test_select_rounds_abort_falls_back(mbx, oracle, monkeypatch):
    """A workgroup that never publishes (MBX_SR_TEST_STALL: as if it were never
    scheduled) makes every coordinator give up after 100 ms; the launch is
    reported aborted and the query answers through the two-pass form, exact."""
    monkeypatch.setenv("MBX_SR_MIN_ROWS", "0")
    cfg = mbx.Config.create()
    cfg.set("mbx_profile", "true")
    c = mbx.connect_with_config(cfg).value
    n = 5_000_011
    x, k, v, s = _table(c, oracle, n)
    st0 = c.engine_stats()
    for stall in ("0", "17"):
        monkeypatch.setenv("MBX_SR_TEST_STALL", stall)
        got = _col(c, "SELECT x FROM fc WHERE x > 24", "int64")
        names = [kk["name"] for kk in c.last_profile()["kernels"]]
        assert "select_rounds_abort" in names and "filter_count" in names, names
        assert np.array_equal(got, x[x > 24])
    st1 = c.engine_stats()  # the aborts are counted (duckdb_mbx_engine_stats)
    assert st1["select_rounds_aborts"] - st0["select_rounds_aborts"] == 2, (st0, st1)
    assert st1["select_rounds_launches"] - st0["select_rounds_launches"] >= 2
    monkeypatch.delenv("MBX_SR_TEST_STALL")
    got = _col(c, "SELECT x FROM fc WHERE x > 24", "int64")  # the next launch (fresh epoch) is clean
    names = [kk["name"] for kk in c.last_profile()["kernels"]]
    assert "select_rounds" in names and "select_rounds_abort" not in names, names
    assert np.array_equal(got, x[x > 24])
    c.close()


def test_filter_compact_any_width_outputs(mbx, oracle):
    # 1-, 2- and 16-byte outputs (BOOLEAN, SMALLINT, HUGEINT) take the generic
    # compaction kernel; values and order exact
    cfg = mbx.Config.create()
    cfg.set("mbx_profile", "true")
    c = mbx.connect_with_config(cfg).value
    for n in (1, 300, 70_001):
        q(c, "DROP TABLE IF EXISTS fw")
        q(c, f"CREATE TABLE fw AS SELECT mbx_synth(42, i, 50) + 1 AS x, (mbx_synth(13, i, 2) = 1) AS b, "
             f"CAST(mbx_synth(11, i, 1000) - 500 AS SMALLINT) AS s, "
             f"CAST(mbx_synth(9, i, 1099511627776) - 549755813888 AS HUGEINT) * 1000000000000 AS h, "
             f"CAST(mbx_synth(7, i, 32) AS TINYINT) AS t FROM range({n}) tbl(i)")
        x = oracle.synth_i64(n, 42, 0, 50, 1)
        b = oracle.synth_i64(n, 13, 0, 2, 0) == 1
        s_ = oracle.synth_i64(n, 11, 0, 1000, -500)
        v = oracle.synth_i64(n, 9, 0, 2**40, -2**39)
        t = oracle.synth_i64(n, 7, 0, 32, 0)
        m = x > 24
        got = q(c, "SELECT b, s, h, t, x FROM fw WHERE x > 24").rows
        if m.any():
            assert "compact" in [k["name"] for k in c.last_profile()["kernels"]]
        exp = [["true" if b[i] else "false", str(s_[i]), str(int(v[i]) * 10**12), str(t[i]), str(x[i])]
               for i in np.flatnonzero(m)]
        assert got == exp, n
    c.close()


def test_filter_compact_profile_and_stream(conn, oracle):
    n = 3_000_017
    x, k, v, s = _table(conn, oracle, n)
    m = x > 24
    st = conn.query_stream("SELECT v FROM fc WHERE x > 24").value
    got = []
    while True:
        r = st.next().value
        if r is None:
            break
        got.extend(int(row[0]) for row in r.rows)
    st.close()
    assert got == v[m].tolist()
    q(conn, "SELECT COUNT(*) FROM (SELECT v FROM fc WHERE x > 24) t")


def _ncol(conn, sql, kind, idx=0):
    # nullable wire buffer -> (values with NULLs zeroed, validity)
    a = conn.query_arrow(sql).value
    b = a._buf(kind, idx, nullable=True)
    a.close()
    n = int.from_bytes(b[:4], "little", signed=True) if len(b) >= 4 else 0
    w = 8 if kind == "int64" else 4
    vals = np.frombuffer(b[4:4 + n * w], dtype=np.int64 if w == 8 else np.int32)
    return vals, np.frombuffer(b[4 + n * w:4 + n * (w + 1)], dtype=np.uint8).astype(bool)


@pytest.mark.parametrize("path", ["auto", "rounds", "rounds_bytes", "twopass"])
@pytest.mark.parametrize("n", [1, 63, 64, 255, 257, 4097, 70_001, 1_000_003])
def test_filter_compact_nullable(mbx, oracle, monkeypatch, n, path):
    """NULLs in predicate columns (a NULL fails the row) and in output columns:
    the two-pass path (validity bits compacted by compact_validity) and the
    one-pass select_rounds (validity words in a second ring, one byte per
    output row packed by pack_validity), forced at every size with
    MBX_SR_MIN_ROWS=0; values and validity exact vs numpy and vs the VM path
    (MBX_FC=0)."""
    if path != "auto":
        monkeypatch.setenv("MBX_SR_MIN_ROWS", "0")
    if path == "twopass":
        monkeypatch.setenv("MBX_SR_NULLS", "0")
    cfg = mbx.Config.create()
    cfg.set("mbx_profile", "true")
    c = mbx.connect_with_config(cfg).value
    q(c, f"CREATE TABLE fn AS SELECT mbx_synth(42, i, 50) + 1 AS x, "
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
    cases = [
        ("SELECT vn FROM fn WHERE xn > 24", xv & (x > 24), [("int64", v, vv)]),
        ("SELECT vn, kn FROM fn WHERE x > 24", x > 24, [("int64", v, vv), ("int32", k, kv)]),
        ("SELECT kn, x FROM fn WHERE xn > 24 AND kn < 16", xv & (x > 24) & kv & (k < 16),
         [("int32", k, kv), ("int64", x, np.ones(n, bool))]),
    ]
    for sql, m, cols in cases:
        for i, (kind, arr, valid) in enumerate(cols):
            got, ok = _ncol(c, sql, kind, i)
            names = [kk["name"] for kk in c.last_profile()["kernels"]]
            # NULL-free loaded columns (tiny n) take the one-pass kernel
            assert "filter_bits" in names or "select" in names or "select_rounds" in names, (sql, names)
            if path.startswith("rounds"):
                assert "select_rounds" in names and "filter_bits" not in names, (sql, names)
                if i == 0 and not valid.all() and m.any():
                    assert "pack_validity" in names, (sql, names)
            elif i == 0 and not valid.all() and m.any() and "select_rounds" not in names:
                assert "compact_validity" in names, (sql, names)
            assert np.array_equal(ok, valid[m]), (n, sql, i)
            assert np.array_equal(got, np.where(valid[m], arr[m], 0).astype(got.dtype)), (n, sql, i)
            monkeypatch.setenv("MBX_FC", "0")
            got2, ok2 = _ncol(c, sql, kind, i)
            monkeypatch.delenv("MBX_FC")
            assert np.array_equal(ok2, ok) and np.array_equal(got2, got), (n, sql, i)
    c.close()


@pytest.mark.parametrize("sent", ["1", "0"])
def test_select_rounds_nullable_sentinel_extremes(mbx, monkeypatch, sent):
    """NULL-able outputs whose valid values reach the ends of the staged width:
    an INT64 column holding INT64_MIN and INT64_MAX leaves no sentinel (validity
    bytes are staged), an INTEGER column holding INT32_MAX and a narrow-staged
    BIGINT column holding INT32_MAX take INT32_MIN as the sentinel, and one
    holding INT32_MIN and INT32_MAX leaves none in 4 bytes.  Values (0 under
    NULL) and validity exact vs numpy, one-pass kernel forced (and, with
    sent=0, validity bytes everywhere)."""
    monkeypatch.setenv("MBX_SR_MIN_ROWS", "0")
    monkeypatch.setenv("MBX_SR_SENT", sent)
    n = 300_001
    i = np.arange(n, dtype=np.int64)
    ext = np.array([-2**63, 2**63 - 1, -2**63 + 1, 2**63 - 2, 0, -1], dtype=np.int64)
    e64 = ext[i % 6]
    e32 = np.array([2**31 - 1, -5, 7, 2**31 - 2], dtype=np.int64)[i % 4]
    f32 = np.array([2**31 - 1, -2**31, 3], dtype=np.int64)[i % 3]
    null = (i % 5) == 2
    cfg = mbx.Config.create()
    cfg.set("mbx_profile", "true")
    c = mbx.connect_with_config(cfg).value
    def case(col):
        return f"CASE WHEN i % 5 = 2 THEN NULL ELSE {col} END"
    e64_sql = ("CASE WHEN i % 6 = 0 THEN -9223372036854775808 WHEN i % 6 = 1 THEN 9223372036854775807 "
               "WHEN i % 6 = 2 THEN -9223372036854775807 WHEN i % 6 = 3 THEN 9223372036854775806 "
               "WHEN i % 6 = 4 THEN 0 ELSE -1 END")
    e32_sql = "CASE WHEN i % 4 = 0 THEN 2147483647 WHEN i % 4 = 1 THEN -5 WHEN i % 4 = 2 THEN 7 ELSE 2147483646 END"
    f32_sql = "CASE WHEN i % 3 = 0 THEN 2147483647 WHEN i % 3 = 1 THEN -2147483648 ELSE 3 END"
    m = (i % 3) != 1
    sel = i > 1000
    for col, kind, arr, expr in [("a", "int64", e64, e64_sql + "::BIGINT"), ("b", "int32", e32, e32_sql + "::INTEGER"),
                                 ("c", "int64", e32, e32_sql + "::BIGINT"), ("d", "int32", f32, f32_sql + "::INTEGER"),
                                 ("e", "int64", f32, f32_sql + "::BIGINT")]:
        # one table per column (the device VM caps the instructions of one CTAS)
        q(c, f"CREATE OR REPLACE TABLE se AS SELECT i AS x, {case(expr)} AS {col} FROM range({n}) tbl(i)")
        got, ok = _ncol(c, f"SELECT {col} FROM se WHERE x % 3 <> 1", kind)
        got2, ok2 = _ncol(c, f"SELECT {col}, x FROM se WHERE x > 1000", kind)
        names = [kk["name"] for kk in c.last_profile()["kernels"]]
        assert "select_rounds" in names, (col, names)
        assert np.array_equal(ok2, ~null[sel]), col
        assert np.array_equal(got2, np.where(null[sel], 0, arr[sel]).astype(got2.dtype)), col
        assert np.array_equal(ok, ~null[m]), col
        assert np.array_equal(got, np.where(null[m], 0, arr[m]).astype(got.dtype)), col
    c.close()


def test_nullable_selection_large_properties(mbx, oracle):
    """The sentinel-staged NULL-able selection at 2e8 rows (select_rounds with
    8 loaders, result adopted by CREATE TABLE AS with the storers' zone map):
    the result's COUNT(*), COUNT(vn), SUM(vn), MIN(vn), MAX(vn) against numpy
    over the same generators, in 5e7-row chunks; then every output value and
    validity bit of one 1e6-row slice in the middle."""
    n, chunk = 200_000_000, 50_000_000
    cfg = mbx.Config.create()
    cfg.set("mbx_profile", "true")
    c = mbx.connect_with_config(cfg).value
    q(c, f"CREATE TABLE fl AS SELECT mbx_synth(42, i, 50) + 1 AS x, "
         f"CASE WHEN mbx_synth(19, i, 7) = 0 THEN NULL ELSE mbx_synth(9, i, 1099511627776) - 549755813888 END AS vn "
         f"FROM range({n}) tbl(i)")
    q(c, "CREATE TABLE sl AS SELECT vn FROM fl WHERE x > 24")
    assert "select_rounds" in [k["name"] for k in c.last_profile()["kernels"]]
    cnt = cv = s = 0
    mn, mx = None, None
    for a in range(0, n, chunk):
        x = oracle.synth_i64(chunk, 42, a, 50, 1)
        v = oracle.synth_i64(chunk, 9, a, 2**40, -2**39)
        ok = oracle.synth_i64(chunk, 19, a, 7, 0) != 0
        m = x > 24
        sv = v[m & ok]
        cnt += int(m.sum())
        cv += int(sv.size)
        s += int(sv.sum(dtype=np.int64))
        mn = int(sv.min()) if mn is None else min(mn, int(sv.min()))
        mx = int(sv.max()) if mx is None else max(mx, int(sv.max()))
    assert one(c, "SELECT COUNT(*), COUNT(vn), SUM(vn), MIN(vn), MAX(vn) FROM sl") == [
        str(cnt), str(cv), str(s), str(mn), str(mx)]
    # one slice: rows [a0, a0 + 2e6) of fl hold the selected rows [off, off + len) of sl
    a0 = 100_000_000
    x = oracle.synth_i64(2_000_000, 42, a0, 50, 1)
    v = oracle.synth_i64(2_000_000, 9, a0, 2**40, -2**39)
    ok = oracle.synth_i64(2_000_000, 19, a0, 7, 0) != 0
    off = 0  # selected rows before a0, from the generator
    for a in range(0, a0, chunk):
        off += int((oracle.synth_i64(chunk, 42, a, 50, 1) > 24).sum())
    m = x > 24
    got, gv = _ncol(c, f"SELECT vn FROM sl LIMIT {int(m.sum())} OFFSET {off}", "int64")
    assert np.array_equal(gv, ok[m])
    assert np.array_equal(got, np.where(ok[m], v[m], 0))
    c.close()
