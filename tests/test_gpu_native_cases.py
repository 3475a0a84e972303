"""Replays every assertion of the reference's native and arrow tests that
tests/golden/make_native_cases.py extracts into tests/golden/native_cases.json
(src/duckdb_test.mbt, src/duckdb_arrow_test.mbt), through the host mirror of
the MoonBit API over the C-ABI: the same SQL, the same statement / appender
calls in the same order, the same asserted cells, row counts, stream counts,
Arrow schema types and getter values.  Cases the extractor marks partial keep
the assertions it read (the rest is restated by hand in test_gpu_native.py /
test_gpu_arrow.py); helper-only and LIST/STRUCT/MAP cases have nothing to run
here (the CPU test below checks the classification)."""
import json
import os

import pytest

from conftest import q

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "native_cases.json")))["cases"]
RUNNABLE = ("stream", "prepare", "appender", "arrow", "query")
RUN = [c for c in CASES if c["kind"] in RUNNABLE and (c["kind"] != "query" or c["cells"] or "row_count" in c)]


def _arg(a):
    from oracle import mb
    if isinstance(a, dict) and "call" in a:
        return getattr(mb, a["call"])(*[_arg(x) for x in a["args"]])
    assert not isinstance(a, dict), f"unevaluated argument {a}"
    return a


def _check_cells(res, case):
    for r, c, want in case["cells"]:
        got = res.cell(r, c)
        if isinstance(want, dict) and "one_of" in want:
            assert got in want["one_of"], (case["name"], r, c, got, want)
        elif isinstance(want, dict):
            assert got is not None and want["contains"] in got, (case["name"], r, c, got)
        else:
            assert got == want, (case["name"], r, c, got, want)
    if "row_count" in case:
        assert res.row_count() == case["row_count"], case["name"]


def _check_values(got, facts, what):
    if "length" in facts:
        assert len(got) == facts["length"], what
    for i, v in facts.get("values", {}).items():
        assert got[int(i)] == v, (what, i, got[int(i)], v)
    for i, (lo, hi) in facts.get("ranges", {}).items():
        assert lo <= got[int(i)] <= hi, (what, i, got[int(i)])


@pytest.mark.gpu
@pytest.mark.parametrize("case", RUN, ids=[f'{c["file"].split("/")[-1]}:{c["line"]}' for c in RUN])
def test_reference_native_case(conn, mbx, case):
    k = case["kind"]
    if k == "stream":
        st = conn.query_stream(case["sql"][0]).value
        n = 0
        cols = st.columns()
        while True:
            r = st.next().value
            if r is None:
                break
            n += len(r.rows)
        st.close()
        s = case["stream"]
        assert n == s["count"] and len(cols) == s.get("ncols", len(cols))
        assert cols[:len(s.get("columns", []))] == s.get("columns", [])
    elif k == "prepare":
        st = conn.prepare(case["sql"][0]).value
        for name, args in case["ops"]:
            assert isinstance(getattr(st, name)(*[_arg(a) for a in args]), mbx.Ok), (case["name"], name)
        _check_cells(st.execute().value, case)
        st.close()
    elif k == "appender":
        q(conn, "DROP TABLE IF EXISTS test_table")
        q(conn, case["sql"][0])
        ap = conn.create_appender("main", "test_table").value
        for name, args in case["ops"]:
            assert isinstance(getattr(ap, name)(*[_arg(a) for a in args]), mbx.Ok), (case["name"], name)
        ap.close()  # close => flush (callback style, as the reference's Appender::close)
        _check_cells(q(conn, case["sql"][1]), case)
    elif k == "arrow":
        a = case["arrow"]
        r = conn.query_arrow(case["sql"][0])
        if a["expect_error"]:
            assert isinstance(r, mbx.Err)
            return
        res = r.value
        if "column_count" in a:
            assert res.column_count() == a["column_count"]
        if "row_count" in a:
            assert res.row_count() == a["row_count"]
        if "fields" in a or "types" in a or "names" in a:
            fields = res.get_schema().value.fields
            assert len(fields) == a.get("fields", len(fields))
            for i, t in a.get("types", {}).items():
                assert fields[int(i)].type_id == t, (case["name"], i)
            for i, nm in a.get("names", {}).items():
                assert fields[int(i)].name == nm, (case["name"], i)
        for g in a["getters"]:
            got = getattr(res, "get_column_" + g["getter"])(g["col"])
            if "validity" in g:
                vals, valid = got
                _check_values(vals, g["values"], (case["name"], "values"))
                _check_values(valid, g["validity"], (case["name"], "validity"))
            else:
                _check_values(got, g["values"], (case["name"], g["getter"]))
        res.close()
    else:  # query
        _check_cells(q(conn, case["sql"][0]), case)


def test_native_cases_cover_every_reference_test():
    # every test block of the two reference files is classified, and the
    # runnable ones carry at least one extracted assertion
    assert len(CASES) == 62
    kinds = {}
    for c in CASES:
        kinds[c["kind"]] = kinds.get(c["kind"], 0) + 1
    assert set(kinds) <= set(RUNNABLE) | {"helper", "out_of_scope"}, kinds
    for c in RUN:
        assert (c["cells"] or "row_count" in c or c.get("stream") or c.get("arrow")), c["name"]


def test_native_cases_match_the_reference_sources(tmp_path):
    # when the reference is present (development container), the committed JSON
    # is exactly what the extractor produces from it
    if not os.path.isdir("/root/reference/src"):
        pytest.skip("reference sources not present (GPU box)")
    import subprocess
    import sys
    gen = os.path.join(HERE, "golden", "make_native_cases.py")
    before = open(os.path.join(HERE, "golden", "native_cases.json")).read()
    subprocess.run([sys.executable, gen], check=True, capture_output=True)
    assert open(os.path.join(HERE, "golden", "native_cases.json")).read() == before
