"""The reference's arrow tests (src/duckdb_arrow_test.mbt) plus byte-exact
checks of every wire buffer against the oracle's restatement of
duckdb_native.c:2285-2797."""
import pytest

from oracle import wire

pytestmark = pytest.mark.gpu


def arrow(conn, mbx, sql):
    r = conn.query_arrow(sql)
    assert isinstance(r, mbx.Ok), r.error.message
    return r.value


def test_arrow_basic_counts(conn, mbx):
    a = arrow(conn, mbx, "SELECT 1 AS x, 2 AS y")                       # :36-53
    assert (a.column_count(), a.row_count()) == (2, 1)
    a = arrow(conn, mbx, "SELECT * FROM RANGE(10)")                     # :56-73
    assert (a.column_count(), a.row_count()) == (1, 10)
    a = arrow(conn, mbx, "SELECT 42::INTEGER AS i, 3.14::DOUBLE AS d, true::BOOLEAN AS b, 'hello'::VARCHAR AS s")
    assert a.column_count() == 4
    a = arrow(conn, mbx, "SELECT * FROM RANGE(0)")                      # :95-112
    assert (a.column_count(), a.row_count()) == (1, 0)
    assert a.get_column_int64(0) == [] and mbx._take(mbx.lib.duckdb_mb_arrow_get_column_int64(a._h, 0)) == b""
    assert isinstance(conn.query_arrow("SELECT * FROM nonexistent_table"), mbx.Err)  # :115-125


def test_arrow_schema(conn, mbx):
    a = arrow(conn, mbx, "SELECT 42::INTEGER AS a, 3.14::DOUBLE AS b")   # :128-166
    s = a.get_schema().value
    assert [(f.name, f.type_id) for f in s.fields] == [("a", "int32"), ("b", "double")]
    a = arrow(conn, mbx, "SELECT 1::INTEGER AS i, 2::BIGINT AS bi, 3.0::DOUBLE AS d, true::BOOLEAN AS b, "
                         "'text'::VARCHAR AS s")                           # :169-207
    assert [f.type_id for f in a.get_schema().value.fields] == ["int32", "int64", "double", "bool", "string"]
    assert mbx._take(mbx.lib.duckdb_mb_arrow_schema(a._h)) == wire.schema(["i", "bi", "d", "b", "s"], [4, 5, 11, 1, 17])


def test_arrow_column_data(conn, mbx):
    a = arrow(conn, mbx, "SELECT * FROM RANGE(5)")
    assert a.get_column_int32(0) == [0, 1, 2, 3, 4]                      # :210-228
    assert arrow(conn, mbx, "SELECT 100::BIGINT AS x").get_column_int64(0) == [100]   # :231-247
    v = arrow(conn, mbx, "SELECT 3.14::DOUBLE AS x").get_column_double(0)
    assert len(v) == 1 and 3.13 < v[0] < 3.15                            # :250-269
    a = arrow(conn, mbx, "SELECT true::BOOLEAN AS t, false::BOOLEAN AS f")
    assert a.get_column_bool(0) == [True] and a.get_column_bool(1) == [False]   # :272-296
    assert arrow(conn, mbx, "SELECT 'hello'::VARCHAR AS s").get_column_string(0) == ["hello"]
    v = arrow(conn, mbx, "SELECT * FROM RANGE(100)").get_column_int32(0)
    assert len(v) == 100 and v[0] == 0 and v[99] == 99                   # :318-340


def test_arrow_nullable(conn, mbx):
    a = arrow(conn, mbx, "SELECT 1::INTEGER UNION ALL SELECT NULL::INTEGER UNION ALL SELECT 3::INTEGER "
                         "UNION ALL SELECT NULL::INTEGER UNION ALL SELECT 5::INTEGER")   # :343-371
    vals, valid = a.get_column_int32_nullable(0)
    assert valid == [True, False, True, False, True] and len(vals) == 5
    a = arrow(conn, mbx, "SELECT NULL::INTEGER UNION ALL SELECT NULL::INTEGER UNION ALL SELECT NULL::INTEGER")
    assert a.get_column_int32_nullable(0)[1] == [False, False, False]
    a = arrow(conn, mbx, "SELECT 1 UNION ALL SELECT 2 UNION ALL SELECT 3")
    assert a.get_column_int32_nullable(0)[1] == [True, True, True]


def test_arrow_wire_bytes_exact(conn, mbx):
    # a device-scanned relation with NULLs in every type, checked byte for byte
    conn.query("CREATE TABLE w (i INTEGER, b BIGINT, d DOUBLE, t BOOLEAN, s VARCHAR)")
    conn.query("INSERT INTO w VALUES (1, 10, 1.5, true, 'a'), (NULL, -7, NULL, false, NULL), "
               "(-3, NULL, 2.25, NULL, 'ccc'), (4, 9223372036854775807, -0.5, true, '')")
    a = arrow(conn, mbx, "SELECT * FROM w WHERE b IS NULL OR b <> 0")
    lib = mbx.lib
    I = [1, None, -3, 4]
    B = [10, -7, None, 9223372036854775807]
    D = [1.5, None, 2.25, -0.5]
    T = [True, False, None, True]
    S = ["a", None, "ccc", ""]
    for nullable in (False, True):
        suf = "_nullable" if nullable else ""
        get = lambda k, c: mbx._take(getattr(lib, f"duckdb_mb_arrow_get_column_{k}{suf}")(a._h, c))
        assert get("int32", 0) == wire.int32(I, nullable)
        assert get("int64", 1) == wire.int64(B, nullable)
        assert get("double", 2) == wire.double(D, nullable)
        assert get("bool", 3) == wire.boolean(T, nullable)
        assert get("string", 4) == wire.string(S, nullable)
    # int32 getter over BIGINT truncates like (int32_t) (duckdb_native.c:2384-2385)
    assert mbx._take(lib.duckdb_mb_arrow_get_column_int32(a._h, 1)) == wire.int32(B)
    # bad column index / arrow of strings as numbers -> defined empties / zeros
    assert mbx._take(lib.duckdb_mb_arrow_get_column_int64(a._h, 9)) == b""


def test_arrow_nullable_string_double_bool(conn, mbx):
    # duckdb_arrow_test.mbt:428-518
    a = arrow(conn, mbx, "SELECT 'a' UNION ALL SELECT NULL UNION ALL SELECT 'c' UNION ALL SELECT NULL UNION ALL SELECT 'e'")
    vals, valid = a.get_column_string_nullable(0)
    assert valid == [True, False, True, False, True] and len(vals) == 5 and vals[0] == "a" and vals[2] == "c"
    a = arrow(conn, mbx, "SELECT 1.5::DOUBLE UNION ALL SELECT NULL::DOUBLE UNION ALL SELECT 3.14::DOUBLE")
    vals, valid = a.get_column_double_nullable(0)
    assert valid == [True, False, True] and vals[0] == 1.5 and vals[2] == 3.14
    a = arrow(conn, mbx, "SELECT true::BOOLEAN UNION ALL SELECT NULL::BOOLEAN UNION ALL SELECT false::BOOLEAN")
    vals, valid = a.get_column_bool_nullable(0)
    assert valid == [True, False, True] and vals[0] is True and vals[2] is False


def test_arrow_device_columns_direct_and_materialized(conn, mbx):
    # device-resident results: plain columns take the direct-DMA getters, columns with
    # NULLs / other types the per-cell path; both must give the reference's buffers
    q = conn.query
    assert isinstance(q("CREATE TABLE ad AS SELECT CAST(i AS INTEGER) AS a, i * 3 AS b, CAST(i AS DOUBLE) / 4 AS d, "
                        "CASE WHEN i % 3 = 0 THEN NULL ELSE i END AS n FROM range(5000) tbl(i)"), mbx.Ok)
    a = arrow(conn, mbx, "SELECT a, b, d, n FROM ad")
    assert a.get_column_int32(0) == list(range(5000))
    assert a.get_column_int64(1) == [3 * i for i in range(5000)]
    assert a.get_column_double(2) == [i / 4 for i in range(5000)]
    vals, valid = a.get_column_int64_nullable(3)
    assert valid == [i % 3 != 0 for i in range(5000)]
    assert [v for v, ok in zip(vals, valid) if ok] == [i for i in range(5000) if i % 3]
    # int32 getter over BIGINT truncates like the reference's (int32_t) cast (duckdb_native.c:2384-2385)
    assert a.get_column_int32(1)[:3] == [0, 3, 6]


def test_arrow_nullable_device_wire_vs_host(conn, mbx):
    # nullable device columns of every fixed-width getter type: the device wire
    # kernel (values with NULLs zeroed + validity bytes, one DMA each) and the
    # host path (after the result was materialised by a string getter) must give
    # the same bytes, and both the oracle's (duckdb_native.c:2572-2797)
    n = 5003
    assert isinstance(conn.query(
        f"CREATE TABLE anw AS SELECT CASE WHEN i % 3 = 0 THEN NULL ELSE CAST(i - 2500 AS INTEGER) END AS a, "
        f"CASE WHEN i % 5 = 1 THEN NULL ELSE i * 1000000007 - 3 END AS b, "
        f"CASE WHEN i % 7 = 2 THEN NULL ELSE CAST(i AS DOUBLE) / 8 END AS d, "
        f"CASE WHEN i % 4 = 3 THEN NULL ELSE i % 2 = 0 END AS t FROM range({n}) tbl(i)"), mbx.Ok)
    A = [None if i % 3 == 0 else i - 2500 for i in range(n)]
    B = [None if i % 5 == 1 else i * 1000000007 - 3 for i in range(n)]
    D = [None if i % 7 == 2 else i / 8 for i in range(n)]
    T = [None if i % 4 == 3 else i % 2 == 0 for i in range(n)]
    want = {"int32": wire.int32, "int64": wire.int64, "double": wire.double, "bool": wire.boolean}
    cols = {"int32": (0, A), "int64": (1, B), "double": (2, D), "bool": (3, T)}
    sql = "SELECT a, b, d, t FROM anw"
    for host_first in (False, True):
        a = arrow(conn, mbx, sql)
        if host_first:
            assert a.get_column_string(0)[:2] == ["", "-2499"]  # materialises on the host
        for k, (c, vals) in cols.items():
            for nullable in (True, False):
                suf = "_nullable" if nullable else ""
                got = mbx._take(getattr(mbx.lib, f"duckdb_mb_arrow_get_column_{k}{suf}")(a._h, c))
                assert got == want[k](vals, nullable), (k, nullable, host_first)


@pytest.mark.parametrize("n", [1, 255, 1_000_000])
def test_arrow_string_getter_formats_on_device(mbx, oracle, n):
    """The string getters of integer / BOOLEAN / DECIMAL / HUGEINT device
    columns (DECIMAL and HUGEINT map to "string" in the reference,
    duckdb_native.c:2336-2338) are formatted by the text kernels: the wire
    buffer is byte-exact vs oracle/wire.py over oracle/fmt.py's spellings, NULLs
    included, and the kernels are the ones that ran."""
    from oracle import fmt
    cfg = mbx.Config.create()
    cfg.set("mbx_profile", "true")
    c = mbx.connect_with_config(cfg).value
    for q in (f"CREATE TABLE ts1 AS SELECT CASE WHEN mbx_synth(5, i, 7) = 0 THEN NULL ELSE "
              f"CAST(mbx_synth(11, i, 200000) - 100000 AS DECIMAL(15,2)) END AS d FROM range({n}) tbl(i)",
              f"CREATE TABLE ts2 AS SELECT CAST(mbx_synth(9, i, 1099511627776) - 549755813888 AS HUGEINT) * "
              f"100000000000000000000 AS h FROM range({n}) tbl(i)",
              f"CREATE TABLE ts3 AS SELECT mbx_synth(42, i, 50) - 25 AS b, CAST(mbx_synth(7, i, 32) - 16 AS INTEGER) AS k "
              f"FROM range({n}) tbl(i)",
              f"CREATE TABLE ts4 AS SELECT (mbx_synth(13, i, 2) = 1) AS f, CAST(mbx_synth(3, i, 9) AS DECIMAL(4,3)) AS s "
              f"FROM range({n}) tbl(i)"):
        r = c.query(q)
        assert isinstance(r, mbx.Ok), r.error.message
    d_valid = oracle.synth_i64(n, 5, 0, 7, 0) != 0
    d = oracle.synth_i64(n, 11, 0, 200000, -100000)
    h = oracle.synth_i64(n, 9, 0, 2**40, -2**39)
    b = oracle.synth_i64(n, 42, 0, 50, -25)
    k = oracle.synth_i64(n, 7, 0, 32, -16)
    f = oracle.synth_i64(n, 13, 0, 2, 0) == 1
    s3 = oracle.synth_i64(n, 3, 0, 9, 0)
    exp = {
        0: [fmt.decimal(int(x) * 100, 2) if v else None for x, v in zip(d, d_valid)],
        1: [str(int(x) * 10**20) for x in h],
        2: [str(int(x)) for x in b],
        3: [str(int(x)) for x in k],
        4: [fmt.boolean(bool(x)) for x in f],
        5: [fmt.decimal(int(x) * 1000, 3) for x in s3],
    }
    where = {0: ("ts1", "d"), 1: ("ts2", "h"), 2: ("ts3", "b"), 3: ("ts3", "k"), 4: ("ts4", "f"), 5: ("ts4", "s")}
    for col, vals in exp.items():
        a = c.query_arrow(f"SELECT {where[col][1]} FROM {where[col][0]}").value
        for nullable in (False, True):
            got = mbx._take((mbx.lib.duckdb_mb_arrow_get_column_string_nullable if nullable else
                             mbx.lib.duckdb_mb_arrow_get_column_string)(a._h, 0))
            want = wire.string(vals, nullable)
            if got != want:  # report the first difference (a full diff of MBs is too slow)
                i = next((j for j in range(min(len(got), len(want))) if got[j] != want[j]), min(len(got), len(want)))
                raise AssertionError(f"n={n} col={col} nullable={nullable} len {len(got)} vs {len(want)}, first "
                                     f"difference at byte {i}: got {got[max(0, i - 24):i + 24]!r} "
                                     f"want {want[max(0, i - 24):i + 24]!r}")
        a.close()
    names = [x["name"] for x in c.profile_drain()]
    assert "text_write" in names and "text_lengths" in names
    c.close()


def test_arrow_buffer_limit_is_the_moonbit_bytes_limit(mbx):
    """A MoonBit byte object holds < 2^28 bytes (its length is 28 bits of the
    header): the largest int64 column that fits (2^25 - 1 rows: 268 435 452
    bytes with the count) comes back whole and exact; one more row is refused
    with an error and an empty buffer instead of a truncated length."""
    import numpy as np
    c = mbx.connect().value
    n_ok = (1 << 25) - 1
    c.query(f"CREATE TABLE big AS SELECT i * 3 AS x FROM range({n_ok + 1}) tbl(i)")
    a = c.query_arrow(f"SELECT x FROM big LIMIT {n_ok}").value
    raw = a.raw_int64_bytes(0)
    a.close()
    assert len(raw) == 4 + 8 * n_ok
    got = np.frombuffer(raw, dtype=np.int64, offset=4)
    assert int.from_bytes(raw[:4], "little") == n_ok and got[0] == 0 and got[-1] == 3 * (n_ok - 1)
    assert np.array_equal(got, np.arange(n_ok, dtype=np.int64) * 3)  # through the host-link pool
    a = c.query_arrow("SELECT x FROM big").value
    raw = a.raw_int64_bytes(0)
    a.close()
    assert raw == b""
    assert "2^28" in mbx._last_error("")
    c.close()


@pytest.mark.parametrize("link", [{}, {"MBX_LINK_THREADS": "0"}, {"MBX_LINK_THREADS": "3", "MBX_LINK_MIN": "1"},
                                  {"MBX_LINK_HUGE": "0", "MBX_LINK_MIN": "1"}], ids=["pool", "runtime", "t3_min1", "nohuge"])
@pytest.mark.parametrize("n", [5, 3_000_017])
def test_arrow_host_link_copies_exact(mbx, monkeypatch, link, n):
    """Getter buffers copied by the host-link pool (csrc/hostlink.cpp: threads
    with pinned double buffers into huge-page-advised fresh Bytes) and by the
    runtime's own copy are byte-exact, for ragged sizes whose last chunk is
    partial: plain int64/int32/double columns (direct DMA), NULL-able ones
    (wire kernel + validity bytes) and device-formatted strings."""
    import numpy as np
    for k, v in link.items():
        monkeypatch.setenv(k, v)
    c = mbx.connect().value
    assert isinstance(c.query(
        f"CREATE TABLE hl AS SELECT i * 7 - 11 AS b, CAST(i % 100000 AS INTEGER) AS a, CAST(i AS DOUBLE) / 4 AS d, "
        f"CASE WHEN i % 3 = 0 THEN NULL ELSE i END AS nb FROM range({n}) tbl(i)"), mbx.Ok)
    i = np.arange(n, dtype=np.int64)
    a = c.query_arrow("SELECT b, a, d, nb FROM hl").value

    def raw(kind, col, nullable=False):
        return mbx._take(getattr(mbx.lib, f"duckdb_mb_arrow_get_column_{kind}{'_nullable' if nullable else ''}")(a._h, col))

    def body(b, dtype, count):
        assert int.from_bytes(b[:4], "little") == n
        return np.frombuffer(b, dtype=dtype, offset=4, count=count)

    assert np.array_equal(body(raw("int64", 0), np.int64, n), i * 7 - 11)
    assert np.array_equal(body(raw("int32", 1), np.int32, n), (i % 100000).astype(np.int32))
    assert np.array_equal(body(raw("double", 2), np.float64, n), i.astype(np.float64) / 4)
    nb = raw("int64", 3, nullable=True)
    valid = i % 3 != 0
    assert np.array_equal(body(nb, np.int64, n), np.where(valid, i, 0))
    assert np.array_equal(np.frombuffer(nb, dtype=np.uint8, offset=4 + 8 * n), valid.astype(np.uint8))
    if n <= 5:
        assert a.get_column_string(0) == [str(x * 7 - 11) for x in range(n)]
    else:
        s = raw("string", 0)
        nn, chars = int.from_bytes(s[:4], "little"), int.from_bytes(s[4:8], "little")
        assert nn == n
        text = s[8:8 + chars].split(b"\0")[:-1]
        assert len(text) == n and text[0] == b"-11" and text[-1] == str((n - 1) * 7 - 11).encode()
        assert text[n // 2] == str((n // 2) * 7 - 11).encode()
    a.close()
    c.close()


def test_arrow_host_link_concurrent_connections(mbx):
    """Two host threads pull >= 32 MiB getter buffers at once through two
    connections on the same device: the device's host-link pool serves one
    copy at a time and both results stay exact (ctypes drops the GIL, so the
    getters really overlap)."""
    import threading
    import numpy as np
    n = 5_000_003  # 40 MB of int64: above the pool's 32 MiB threshold
    conns = [mbx.connect().value for _ in range(2)]
    for j, c in enumerate(conns):
        assert isinstance(c.query(f"CREATE TABLE hc AS SELECT i * {j + 3} + 1 AS b FROM range({n}) tbl(i)"), mbx.Ok)
    errs = []

    def pull(j):
        try:
            for _ in range(3):
                a = conns[j].query_arrow("SELECT b FROM hc").value
                raw = mbx._take(mbx.lib.duckdb_mb_arrow_get_column_int64(a._h, 0))
                a.close()
                got = np.frombuffer(raw, dtype=np.int64, offset=4, count=n)
                if not np.array_equal(got, np.arange(n, dtype=np.int64) * (j + 3) + 1):
                    errs.append(f"connection {j}: values differ")
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(f"connection {j}: {e!r}")

    th = [threading.Thread(target=pull, args=(j,)) for j in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs, errs
    for c in conns:
        c.close()
