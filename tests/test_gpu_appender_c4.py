"""C4 (BASELINE.json configs[3]): Appender ingest of 1e8 INT64 rows into
device column vectors, then the values read back bit-exact through the
reference's three read paths — Arrow int64 buffers in <= 1e6-row slices (the
MoonBit decoders cap at 1e6, duckdb_arrow_native.mbt:474), query_stream
chunks, and to_typed (32-bit saturation, duckdb_parsing.mbt:203-237).
Generator: v_i = i * 2654435761 mod 2^63."""
import json
import os

import numpy as np
import pytest

from conftest import ROOT, one, q

pytestmark = pytest.mark.gpu

N = 100_000_000
BATCH = 10_000_000


def gen(start, n):
    i = np.arange(start, start + n, dtype=np.uint64)
    return ((i * np.uint64(2654435761)) & np.uint64(2**63 - 1)).astype(np.int64)


@pytest.fixture(scope="module")
def c4(mbx):
    conn = mbx.connect().value
    q(conn, "CREATE TABLE c4 (v BIGINT)")
    ap = conn.create_appender("main", "c4").value
    for s in range(0, N, BATCH):
        v = gen(s, BATCH)
        assert isinstance(ap.append_column(0, v), mbx.Ok)
        r = ap.commit(BATCH)
        assert isinstance(r, mbx.Ok), r.error.message
    ap.close()
    yield conn
    conn.close()


def test_c4_count_sum_minmax(c4):
    total = 0
    mn, mx = None, None
    for s in range(0, N, BATCH):
        v = gen(s, BATCH)
        total += int(v.astype(object).sum())
        mn = v.min() if mn is None else min(mn, v.min())
        mx = v.max() if mx is None else max(mx, v.max())
    assert one(c4, "SELECT COUNT(*), SUM(v), MIN(v), MAX(v) FROM c4") == [str(N), str(total), str(mn), str(mx)]


@pytest.mark.parametrize("offset", [0, 1_000_000, 49_999_999, 99_000_000])
def test_c4_arrow_slices_bit_exact(c4, mbx, offset):
    a = c4.query_arrow(f"SELECT v FROM c4 LIMIT 1000000 OFFSET {offset}").value
    buf = a.raw_int64_bytes(0)
    n = min(1_000_000, N - offset)
    assert np.frombuffer(buf[:4], dtype=np.int32)[0] == n
    got = np.frombuffer(buf[4:], dtype=np.int64)
    assert np.array_equal(got, gen(offset, n))
    a.close()


def test_c4_arrow_all_slices_checksum(c4, mbx):
    # every 1e6-row slice through the arrow path; checksum of checksums
    acc = 0
    exp = 0
    for k in range(0, N, 1_000_000):
        a = c4.query_arrow(f"SELECT v FROM c4 LIMIT 1000000 OFFSET {k}").value
        got = np.frombuffer(a.raw_int64_bytes(0)[4:], dtype=np.int64)
        a.close()
        acc = (acc * 31 + int(np.bitwise_xor.reduce(got))) % (2**61 - 1)
        exp = (exp * 31 + int(np.bitwise_xor.reduce(gen(k, 1_000_000)))) % (2**61 - 1)
    assert acc == exp


def test_c4_stream_roundtrip(c4, mbx):
    s = c4.query_stream("SELECT v FROM c4 WHERE v < 1000000000000").value
    exp = gen(0, N)
    exp = exp[exp < 10**12]
    got = []
    while True:
        r = s.next().value
        if r is None:
            break
        got.extend(int(x[0]) for x in r.rows)
    s.close()
    assert got == exp.tolist()


def test_c4_typed_roundtrip(c4, mbx):
    res = q(c4, "SELECT v FROM c4 LIMIT 1000 OFFSET 5")
    exp = gen(5, 1000)
    assert [int(r[0]) for r in res.rows] == exp.tolist()   # string cells exact
    typed = res.to_typed().get_int_column(0)               # MoonBit Int: saturating parse
    assert typed == [min(int(x), 2**31 - 1) for x in exp]


def test_row_appender_1e5(mbx):
    conn = mbx.connect().value
    q(conn, "CREATE TABLE r (id INTEGER, v BIGINT)")
    ap = conn.create_appender("main", "r").value
    n = 100_000
    v = gen(0, n)
    for i in range(n):
        ap.begin_row()
        ap.append_int(i)
        ap.append_bigint(int(v[i]))
        ap.end_row()
    ap.close()
    a = conn.query_arrow("SELECT v FROM r ORDER BY id").value
    assert np.array_equal(np.frombuffer(a.raw_int64_bytes(0)[4:], dtype=np.int64), v)
    conn.close()


def test_row_appender_partial_row_and_nulls(mbx):
    # values go straight into the batch columns: a row left half appended at
    # close never reaches the table; NULLs after fast-path values keep their rows
    conn = mbx.connect().value
    q(conn, "CREATE TABLE p (a BIGINT, b INTEGER)")
    ap = conn.create_appender("main", "p").value
    for i in range(3):
        ap.begin_row(); ap.append_bigint(10 * i); ap.append_int(i); ap.end_row()
    ap.begin_row(); ap.append_null(); ap.append_int(7); ap.end_row()
    ap.begin_row(); ap.append_bigint(99)             # partial row
    assert isinstance(ap.flush(), mbx.Err)           # "Incomplete append to row"
    ap.close()
    res = q(conn, "SELECT a, b FROM p")
    assert res.rows == [["0", "0"], ["10", "1"], ["20", "2"], ["", "7"]]
    assert res.nulls[3] == [True, False]
    conn.close()


def test_c4_row_appender_native_harness(mbx, tmp_path):
    # the reference's row-wise Appender driven from C (no Python per call)
    import subprocess
    exe = str(tmp_path / "mb_harness")
    lib = os.path.join(ROOT, "duckdb.mbt_amd")
    subprocess.run(["gcc", "-O2", "-std=c11", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c_harness", "mb_harness.c"), "-o", exe, "-L", lib,
                    "-lduckdb_mb_amd", f"-Wl,-rpath,{lib}"], check=True)
    p = subprocess.run([exe, "c4", "3000017"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["bit_exact"] and r["rows"] == 3000017
