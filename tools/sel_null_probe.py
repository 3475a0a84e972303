"""NULL-able materialising selections at 1e9 rows (GPU only): kernel ms of
each form (one-pass select_rounds with validity vs MBX_SR_NULLS=0, the
filter_bits + compact + compact_validity two-pass form), result kept in HBM
(query_arrow + row count); the two forms' results are compared through
COUNT / COUNT(col) / SUM(col) of a CREATE TABLE AS of each."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

m = ge._load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
cfg = m.Config.create()
cfg.set("mbx_profile", "true")
c = m.connect_with_config(cfg).value
c.query(f"CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x, "
        f"CASE WHEN mbx_synth(13, i, 10) = 0 THEN NULL ELSE mbx_synth(42, i, 50) + 1 END AS xn, "
        f"CASE WHEN mbx_synth(19, i, 7) = 0 THEN NULL ELSE mbx_synth(9, i, 1099511627776) - 549755813888 END AS vn, "
        f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range({n}) tbl(i)")
SHAPES = {
    "x_where_x": ("SELECT x FROM t WHERE x > 24", "x"),
    "v_where_x": ("SELECT v FROM t WHERE x > 24", "v"),
    "vn_where_x": ("SELECT vn FROM t WHERE x > 24", "vn"),
    "xn_where_xn": ("SELECT xn FROM t WHERE xn > 24", "xn"),
    "vn_where_xn": ("SELECT vn FROM t WHERE xn > 24", "vn"),
}
for name, (sql, col) in SHAPES.items():
    agg = {}
    for nulls in (os.environ.get("NULLS_GRID", "1,0").split(",")):
        os.environ["MBX_SR_NULLS"] = nulls
        ms, kern = [], None
        for i in range(5):
            a = c.query_arrow(sql).value
            rows = a.row_count()
            a.close()
            ks = c.last_profile()["kernels"]
            kern = [k["name"] for k in ks]
            if i:
                ms.append(sum(k["ms"] for k in ks if k["name"] != "text_lengths"))
                per = {k["name"]: round(k["ms"], 3) for k in ks}
        c.query("DROP TABLE IF EXISTS r")
        c.query(f"CREATE TABLE r AS {sql}")
        rr = c.query_raw(f"SELECT COUNT(*), COUNT({col}), SUM({col}) FROM r")
        agg[nulls] = [rr.value(j, 0) for j in range(3)]
        rr.close()
        print(json.dumps({"shape": name, "sql": sql, "MBX_SR_NULLS": nulls, "ms_median": statistics.median(ms),
                          "rows": rows, "kernels": per, "agg": agg[nulls]}), flush=True)
    if "1" in agg and "0" in agg:
        print(json.dumps({"shape": name, "same_result": agg["1"] == agg["0"]}), flush=True)
