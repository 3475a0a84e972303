"""Tables sharded inside the library ("gpu_devices"): every table
is split into contiguous row runs, one per shard, and a query over it runs on
every shard at once and is combined by the connection's first device.  On the
1-GPU test box the shards share device 0 ("0,0", "0,0,0"), which exercises the
same split / per-shard kernels / combine code as distinct devices.

Everything is checked against the CPU oracle or numpy over the oracle's
generator: aggregates (C2, C5, C3 shapes), row results, hash GROUP BY, HAVING,
AVG over DECIMAL / DOUBLE, streams, CTAS, appender ingest; with
mbx_force_peer the same-device shards also exchange rows by peer DMA."""
import numpy as np
import pytest

from conftest import one, q

pytestmark = pytest.mark.gpu


def _conn(mbx, devices, profile=False, shard_rows=None):
    cfg = mbx.Config.create()
    assert isinstance(cfg.set("gpu_devices", devices), mbx.Ok)
    if profile:
        cfg.set("mbx_profile", "true")
    if shard_rows is not None:
        assert isinstance(cfg.set("mbx_shard_rows", str(shard_rows)), mbx.Ok)
    r = mbx.connect_with_config(cfg)
    assert isinstance(r, mbx.Ok), r.error.message
    return r.value


@pytest.mark.parametrize("devices", ["0,0", "0,0,0"])
def test_sharded_c2_c5_aggregates(mbx, oracle, devices):
    n = 50_000_017
    c = _conn(mbx, devices, profile=True)
    q(c, f"CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x FROM range({n}) tbl(i)")
    assert one(c, "SELECT COUNT(*) FROM t") == [str(n)]
    cnt, s = oracle.synth_filter_count(42, 0, n, 50, 1, 25, 2**63 - 1, 8)
    assert one(c, "SELECT COUNT(*) FROM t WHERE x > 24") == [str(cnt)]                 # C2
    kinds = [k["name"] for k in c.last_profile()["kernels"]]
    assert kinds.count("filter_agg") == devices.count(",") + 1, kinds                  # one per shard
    got = one(c, "SELECT COUNT(*), SUM(x), MIN(x), MAX(x) FROM t WHERE x > 24")         # C5
    assert got == [str(cnt), str(s), "25", "50"]
    x = oracle.synth_i64(n, 42, 0, 50, 1)
    avg = float(one(c, "SELECT AVG(x) FROM t")[0])
    assert abs(avg - x.mean()) <= 1e-9 * abs(x.mean())
    assert one(c, "SELECT COUNT(*), SUM(x) FROM t WHERE x > 100") == ["0", ""]  # NULL cells read as ""
    c.close()


def test_sharded_c3_group_by(mbx, oracle):
    n = 40_000_003
    c = _conn(mbx, "0,0,0")
    q(c, f"CREATE TABLE g AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
         f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range({n}) tbl(i)")
    oc, osum = oracle.synth_groupby(7, 9, 0, n, 32, 1 << 40, -(1 << 39), 8)
    rows = q(c, "SELECT k, SUM(v), COUNT(*) FROM g GROUP BY k").rows
    assert rows == [[str(k), str(osum[k]), str(oc[k])] for k in range(32) if oc[k]]
    # HAVING / ORDER BY / LIMIT over the combined groups
    top = q(c, "SELECT k, COUNT(*) AS n FROM g GROUP BY k HAVING COUNT(*) > 0 ORDER BY n DESC, k LIMIT 3").rows
    exp = sorted(((int(oc[k]), k) for k in range(32)), key=lambda t: (-t[0], t[1]))[:3]
    assert top == [[str(k), str(cn)] for cn, k in exp]
    c.close()


@pytest.mark.parametrize("force_peer", [False, True])
def test_sharded_rows_and_hash_groups_vs_numpy(mbx, oracle, force_peer):
    """Row results, hash GROUP BY (VARCHAR / NULL keys, two keys), HAVING,
    ORDER BY / LIMIT, AVG / SUM over DECIMAL and DOUBLE, streams and CTAS over a
    2-shard table, each against numpy over the oracle's generator (not against
    another connection of the same engine)."""
    from oracle import fmt
    n = 1_000_003
    sql_t = (f"CREATE TABLE h AS SELECT mbx_synth(42, i, 50) + 1 AS x, "
             f"CASE WHEN mbx_synth(5, i, 9) = 0 THEN NULL WHEN mbx_synth(3, i, 3) = 0 THEN 'apple' "
             f"WHEN mbx_synth(3, i, 3) = 1 THEN 'kiwi' ELSE 'fig' END AS s, "
             f"CAST(mbx_synth(11, i, 100000) - 50000 AS DECIMAL(12,2)) AS d, mbx_synth(13, i, 1000) / 7 AS f, "
             f"i AS r FROM range({n}) tbl(i)")
    cfg = mbx.Config.create()
    assert isinstance(cfg.set("gpu_devices", "0,0"), mbx.Ok)
    if force_peer:
        assert isinstance(cfg.set("mbx_force_peer", "true"), mbx.Ok)
    c = mbx.connect_with_config(cfg).value
    q(c, sql_t)
    x = oracle.synth_i64(n, 42, 0, 50, 1)
    s5 = oracle.synth_i64(n, 5, 0, 9, 0)
    s3 = oracle.synth_i64(n, 3, 0, 3, 0)
    sv = np.where(s3 == 0, "apple", np.where(s3 == 1, "kiwi", "fig")).astype(object)
    sv[s5 == 0] = None
    snull = s5 == 0
    draw = (oracle.synth_i64(n, 11, 0, 100000, 0) - 50000) * 100  # DECIMAL(12,2) unscaled
    fv = oracle.synth_i64(n, 13, 0, 1000, 0) / 7.0
    r = np.arange(n, dtype=np.int64)

    def rows(sql):
        return q(c, sql).rows

    m = (x > 24) & (r % 3 == 0)
    assert rows("SELECT r, x FROM h WHERE x > 24 AND r % 3 = 0") == [[str(a), str(b)] for a, b in zip(r[m], x[m])]
    sel = np.sort(r[(x >= 10) & (x <= 12)])[::-1][5:1005]
    assert rows("SELECT r FROM h WHERE x BETWEEN 10 AND 12 ORDER BY r DESC LIMIT 1000 OFFSET 5") == \
        [[str(v)] for v in sel]
    exp = []
    for key in ["apple", "fig", "kiwi", None]:
        mk = snull if key is None else (~snull) & (sv == key)
        exp.append(["" if key is None else key, str(int(mk.sum())), str(int(x[mk].sum())), str(int(r[mk].min())),
                    str(int(r[mk].max()))])
    res = q(c, "SELECT s, COUNT(*), SUM(x), MIN(r), MAX(r) FROM h GROUP BY s ORDER BY s NULLS LAST")
    assert res.rows == exp
    assert res.column_types == ["Varchar", "BigInt", "HugeInt", "BigInt", "BigInt"]
    exp = []
    mr = r > 100
    for mm in range(7):
        for key in ["apple", "fig", "kiwi", None]:
            mk = mr & (x % 7 == mm) & (snull if key is None else (~snull) & (sv == key))
            if mk.any():
                exp.append([str(mm), "" if key is None else key, str(int(mk.sum()))])
    assert rows("SELECT x % 7 AS m, s, COUNT(*) FROM h WHERE r > 100 GROUP BY m, s ORDER BY m, s") == exp
    assert rows("SELECT COUNT(DISTINCT x) FROM h") == [[str(len(np.unique(x)))]]
    assert rows("SELECT COUNT(s), COUNT(*), MIN(x) FROM h WHERE s IS NOT NULL") == \
        [[str(int((~snull).sum())), str(int((~snull).sum())), str(int(x[~snull].min()))]]
    exp = [[str(v), str(int((x == v).sum()))] for v in range(1, 51) if int(r[x == v].sum()) > 10_000_000_000]
    assert rows("SELECT x, COUNT(*) FROM h GROUP BY x HAVING SUM(r) > 10000000000 ORDER BY x") == exp
    md = x < 30
    got = rows("SELECT AVG(d), SUM(d), MIN(d), MAX(d) FROM h WHERE x < 30")[0]
    ssum = int(draw[md].sum())
    assert got[1:] == [fmt.decimal(ssum, 2), fmt.decimal(int(draw[md].min()), 2), fmt.decimal(int(draw[md].max()), 2)]
    avg = float(ssum) / (float(md.sum()) * 100.0)
    assert abs(float(got[0]) - avg) <= 1e-12 * abs(avg)
    # DOUBLE sums: summation order differs between shards (stated tolerance 1e-9 relative)
    got = [float(v) for v in rows("SELECT SUM(f), AVG(f), MIN(f), MAX(f) FROM h")[0]]
    for u, w in zip(got, [float(fv.sum()), float(fv.mean()), float(fv.min()), float(fv.max())]):
        assert abs(u - w) <= 1e-9 * abs(w)
    # stream read-back of a sharded SELECT: the rows in part (= row) order
    st = c.query_stream("SELECT r FROM h WHERE x > 40").value
    got = []
    while True:
        ch = st.next().value
        if ch is None:
            break
        got.extend(int(row[0]) for row in ch.rows)
    st.close()
    assert got == r[x > 40].tolist()
    # CTAS from a sharded table stays sharded part by part; DROP removes every part
    q(c, "CREATE TABLE h2 AS SELECT r, x FROM h WHERE x > 24")
    assert rows("SELECT COUNT(*), SUM(r) FROM h2") == [[str(int((x > 24).sum())), str(int(r[x > 24].sum()))]]
    q(c, "DROP TABLE h2")
    assert isinstance(c.query("SELECT COUNT(*) FROM h2"), mbx.Err)
    if force_peer:
        assert c.shard_stats()["peer_copies"] > 0
    c.close()


def test_sharded_appender_fills_parts_in_order(mbx):
    # mbx_shard_rows = 300 000: 1 000 000 appended rows land 300k / 300k / 400k
    # over three parts; the table reads back in append order
    c = _conn(mbx, "0,0,0", shard_rows=300_000)
    q(c, "CREATE TABLE a (v BIGINT, w INTEGER)")
    n = 1_000_000
    v = (np.arange(n, dtype=np.int64) * 2654435761) & (2**62 - 1)
    w = (np.arange(n) % 1000).astype(np.int32)
    ap = c.create_appender("main", "a").value
    for s0 in range(0, n, 250_000):
        ap.append_column(0, v[s0:s0 + 250_000])
        ap.append_column(1, w[s0:s0 + 250_000])
        assert isinstance(ap.commit(250_000), mbx.Ok)
    ap.close()
    # the row-wise appender and INSERT go to the last part
    ap = c.create_appender("main", "a").value
    for i in range(5):
        ap.begin_row()
        ap.append_bigint(-i)
        ap.append_int(i)
        ap.end_row()
    ap.close()
    q(c, "INSERT INTO a VALUES (7, 7), (NULL, 8)")
    got = c.query_arrow("SELECT v FROM a LIMIT 1000000").value
    assert np.array_equal(np.frombuffer(got.raw_int64_bytes(0)[4:], dtype=np.int64), v)
    got.close()
    assert q(c, "SELECT v, w FROM a OFFSET 1000000").rows == \
        [[str(-i), str(i)] for i in range(5)] + [["7", "7"], ["", "8"]]
    assert one(c, "SELECT COUNT(*), COUNT(v), SUM(w) FROM a") == \
        [str(n + 7), str(n + 6), str(int(w.astype(np.int64).sum()) + 10 + 15)]
    c.close()


def test_sharded_empty_and_tiny_tables(mbx):
    c = _conn(mbx, "0,0,0")
    q(c, "CREATE TABLE e (x BIGINT)")
    assert one(c, "SELECT COUNT(*), SUM(x), MIN(x) FROM e") == ["0", "", ""]
    assert q(c, "SELECT x, COUNT(*) FROM e GROUP BY x").rows == []
    q(c, "CREATE TABLE t1 AS SELECT i AS x FROM range(2) tbl(i)")  # fewer rows than shards
    assert q(c, "SELECT x FROM t1").rows == [["0"], ["1"]]
    assert one(c, "SELECT SUM(x), AVG(x) FROM t1") == ["1", "0.5"]
    c.close()


@pytest.mark.parametrize("devices", ["0,0", "0,0,0"])
def test_sharded_select_rounds(mbx, oracle, monkeypatch, devices):
    """Row results of the one-pass compaction on every shard at once: shards
    that share a device take turns through the per-device lock (two persistent
    grids never compete for the CUs), rows come back in part order, exact."""
    monkeypatch.setenv("MBX_SR_MIN_ROWS", "0")
    n = 12_000_007
    c = _conn(mbx, devices, profile=True)
    q(c, f"CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x, CAST(mbx_synth(7, i, 32) AS INTEGER) AS k "
         f"FROM range({n}) tbl(i)")
    x = oracle.synth_i64(n, 42, 0, 50, 1)
    k = oracle.synth_i64(n, 7, 0, 32, 0)
    for _ in range(3):
        a = c.query_arrow("SELECT x, k FROM t WHERE x > 24 AND k < 16").value
        b = a._buf("int64", 0)
        a.close()
        cnt = int.from_bytes(b[:4], "little", signed=True)
        got = np.frombuffer(b[4:4 + 8 * cnt], dtype=np.int64)
        m = (x > 24) & (k < 16)
        assert np.array_equal(got, x[m])
        kinds = [kk["name"] for kk in c.last_profile()["kernels"]]
        assert kinds.count("select_rounds") == devices.count(",") + 1, kinds
    c.close()


def test_force_peer_rows_and_groups_vs_oracle(mbx, oracle):
    """mbx_force_peer sends row results of shards that share the test GPU
    through the multi-device move (hipMemcpyPeerAsync into the combining
    engine, one synchronisation for all parts), as distinct MI355X devices
    would; rows, the gathered COUNT(DISTINCT) path and GROUP BY are checked
    against the oracle (not against another connection of the same engine)."""
    n = 6_000_011
    cfg = mbx.Config.create()
    assert isinstance(cfg.set("gpu_devices", "0,0,0"), mbx.Ok)
    assert isinstance(cfg.set("mbx_force_peer", "true"), mbx.Ok)
    c = mbx.connect_with_config(cfg).value
    q(c, f"CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x, CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
         f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v, i AS r FROM range({n}) tbl(i)")
    x = oracle.synth_i64(n, 42, 0, 50, 1)
    k = oracle.synth_i64(n, 7, 0, 32, 0)
    st0 = c.shard_stats()
    assert st0["shards"] == 3
    # row result: every shard's passing rows moved by peer DMA, concatenated in part order
    a = c.query_arrow("SELECT r, x FROM t WHERE x > 24 AND k < 16").value
    br, bx = a._buf("int64", 0), a._buf("int64", 1)
    a.close()
    m = (x > 24) & (k < 16)
    cnt = int.from_bytes(br[:4], "little", signed=True)
    assert cnt == int(m.sum())
    assert np.array_equal(np.frombuffer(br[4:4 + 8 * cnt], dtype=np.int64), np.nonzero(m)[0])
    assert np.array_equal(np.frombuffer(bx[4:4 + 8 * cnt], dtype=np.int64), x[m])
    st1 = c.shard_stats()
    assert st1["peer_copies"] >= 3 * 2 and st1["peer_bytes"] >= cnt * 16, st1  # 2 columns from every shard
    # a shape that does not decompose: every part gathered by peer DMA first
    assert one(c, "SELECT COUNT(DISTINCT x) FROM t WHERE k < 3") == [str(len(np.unique(x[k < 3])))]
    assert c.shard_stats()["peer_copies"] > st1["peer_copies"]
    # C3 over the shards vs the oracle: finished on the host (no re-upload)
    oc, osum = oracle.synth_groupby(7, 9, 0, n, 32, 1 << 40, -(1 << 39), 8)
    h0 = c.shard_stats()["host_results"]
    assert q(c, "SELECT k, SUM(v), COUNT(*) FROM t GROUP BY k").rows == \
        [[str(g), str(osum[g]), str(oc[g])] for g in range(32) if oc[g]]
    assert c.shard_stats()["host_results"] == h0 + 1
    # the columns picked out of order, and HAVING (device path) agree
    assert q(c, "SELECT COUNT(*), k FROM t GROUP BY k").rows == [[str(oc[g]), str(g)] for g in range(32) if oc[g]]
    got = q(c, "SELECT k, COUNT(*) FROM t GROUP BY k HAVING COUNT(*) > 187500 ORDER BY k").rows
    assert got == [[str(g), str(oc[g])] for g in range(32) if oc[g] > 187500]
    c.close()


def test_sharded_float_keys_merge_like_one_device(mbx):
    """-0.0 and 0.0 (and every NaN) are one group on one device; the host merge
    of the shards' partial groups must not split them.  With
    mbx_shard_rows = 10, each 10-row INSERT fills the next part, so every
    shard holds 0.0, -0.0 and NaN keys."""
    vals = ["0.0", "-0.0", "NaN", "1.5", "-0.0", "NaN", "0.0", "2.5", "NaN", "-1.0"]
    out = []
    for devs in ("0,0,0", None):
        if devs:
            c = _conn(mbx, devs, shard_rows=10)
        else:
            c = mbx.connect().value
        q(c, "CREATE TABLE f (d DOUBLE, i BIGINT)")
        for part in range(3):
            q(c, "INSERT INTO f VALUES " + ", ".join(f"('{v}'::DOUBLE, {10 * part + j})" for j, v in enumerate(vals)))
        if devs:
            assert q(c, "SELECT COUNT(*) FROM f").rows == [["30"]]
        out.append(q(c, "SELECT d, COUNT(*), SUM(i) FROM f GROUP BY d ORDER BY d").rows)
        out.append(q(c, "SELECT COUNT(*), SUM(i) FROM f WHERE d = 0.0").rows)
        c.close()
    assert out[0] == out[2] and out[1] == out[3]
    assert len(out[2]) == 5, out[2]  # -1.0, 0.0, 1.5, 2.5, nan
    assert [r[1] for r in out[2]] == ["3", "12", "3", "3", "9"], out[2]


def test_sharded_rowwise_appender_across_parts(mbx):
    """The row-wise appender's pinned double buffer flushed across part
    boundaries (mbx_shard_rows smaller than a flush, flushes smaller than a
    part): a buffer is refilled only after its DMA to whichever shard took it
    has completed, so every value lands intact."""
    cfg = mbx.Config.create()
    assert isinstance(cfg.set("gpu_devices", "0,0,0,0"), mbx.Ok)
    assert isinstance(cfg.set("mbx_shard_rows", "25000"), mbx.Ok)
    assert isinstance(cfg.set("mbx_appender_flush_rows", "7001"), mbx.Ok)
    c = mbx.connect_with_config(cfg).value
    q(c, "CREATE TABLE a (v BIGINT, d DOUBLE)")
    n = 90_000
    v = (np.arange(n, dtype=np.int64) * 2654435761) & (2**62 - 1)
    ap = c.create_appender("main", "a").value
    for i in range(n):
        ap.begin_row()
        ap.append_bigint(int(v[i]))
        ap.append_double(float(i) * 0.5)
        ap.end_row()
    ap.close()
    got = c.query_arrow("SELECT v, d FROM a").value
    bv = got._buf("int64", 0)
    bd = got._buf("double", 1)
    got.close()
    assert np.array_equal(np.frombuffer(bv[4:], dtype=np.int64), v)
    assert np.array_equal(np.frombuffer(bd[4:], dtype=np.float64), np.arange(n) * 0.5)
    c.close()


def test_sharded_integer_key_merge_vs_numpy(mbx, oracle):
    """The host merge's integer-key path (MergeIntKeys): negative keys, NULL
    keys (last), two keys and a DECIMAL key over 4 shards, each group's
    COUNT / SUM / MIN / MAX / AVG against numpy, in key order with and without
    ORDER BY (the direct host result and the re-uploaded relation)."""
    n = 400_009
    c = _conn(mbx, "0,0,0,0")
    q(c, f"CREATE TABLE w AS SELECT CASE WHEN mbx_synth(5, i, 9) = 0 THEN NULL ELSE mbx_synth(7, i, 40) - 20 END AS kn, "
         f"CAST(mbx_synth(3, i, 3) AS INTEGER) AS k2, mbx_synth(42, i, 50) + 1 AS x, "
         f"CAST(mbx_synth(11, i, 7) - 3 AS DECIMAL(9,2)) AS dk FROM range({n}) tbl(i)")
    nul = oracle.synth_i64(n, 5, 0, 9, 0) == 0
    kn = oracle.synth_i64(n, 7, 0, 40, 0) - 20
    k2 = oracle.synth_i64(n, 3, 0, 3, 0)
    x = oracle.synth_i64(n, 42, 0, 50, 1)
    dk = oracle.synth_i64(n, 11, 0, 7, 0) - 3
    exp = []
    for key in list(range(-20, 20)) + [None]:
        mk = nul if key is None else (~nul) & (kn == key)
        if mk.any():
            exp.append(["" if key is None else str(key), str(int(mk.sum())), str(int(x[mk].sum())),
                        str(int(x[mk].min())), str(int(x[mk].max()))])
    assert q(c, "SELECT kn, COUNT(*), SUM(x), MIN(x), MAX(x) FROM w GROUP BY kn").rows == exp
    assert q(c, "SELECT kn, COUNT(*), SUM(x), MIN(x), MAX(x) FROM w GROUP BY kn ORDER BY kn NULLS LAST").rows == exp
    exp2 = []
    for key in list(range(-20, 20)) + [None]:
        for b in range(3):
            mk = (nul if key is None else (~nul) & (kn == key)) & (k2 == b)
            if mk.any():
                exp2.append(["" if key is None else str(key), str(b), str(int(mk.sum()))])
    assert q(c, "SELECT kn, k2, COUNT(*) FROM w GROUP BY kn, k2").rows == exp2
    got = q(c, "SELECT dk, COUNT(*), AVG(x) FROM w GROUP BY dk").rows
    assert [r[:2] for r in got] == [[f"{v}.00", str(int((dk == v).sum()))] for v in range(-3, 4)]
    for r, v in zip(got, range(-3, 4)):
        assert abs(float(r[2]) - x[dk == v].mean()) <= 1e-9 * x[dk == v].mean()
    c.close()
