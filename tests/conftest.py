"""Shared fixtures.  `-m gpu` tests need an MI355X (they run the kernels
through the C-ABI); everything else runs on the CPU of the dev container."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the tests set MBX_* tuning / fault-injection switches (monkeypatch); the
# library reads them only with this opt-in (csrc/knobs.h).  Set before the
# library is loaded: it is read once per process.
os.environ["MBX_EXPERIMENTS"] = "1"
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "duckdb.mbt_amd", "libduckdb_mb_amd.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


def _ensure_built():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(ROOT, "duckdb.mbt_amd")])
    olib = os.path.join(ROOT, "oracle", "build", "liboracle_mbx.so")
    if not os.path.exists(olib):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


def load_mbx():
    if "duckdb_mbt_amd" in sys.modules:
        return sys.modules["duckdb_mbt_amd"]
    _ensure_built()
    spec = importlib.util.spec_from_file_location("duckdb_mbt_amd", os.path.join(ROOT, "duckdb.mbt_amd", "__init__.py"))
    m = importlib.util.module_from_spec(spec)
    sys.modules["duckdb_mbt_amd"] = m
    spec.loader.exec_module(m)
    return m


@pytest.fixture(scope="session")
def mbx():
    return load_mbx()


@pytest.fixture(scope="session")
def oracle():
    _ensure_built()
    from oracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def fixtures():
    return json.load(open(os.path.join(ROOT, "tests", "golden", "fixtures.json")))["cases"]


@pytest.fixture()
def hostconn(mbx):
    """A connection without a GPU: only statements that touch no table rows
    (host-constant SELECTs, DDL) can run — used to test the front end."""
    cfg = mbx.Config.create()
    assert isinstance(cfg.set("mbx_allow_no_gpu", "true"), mbx.Ok)
    r = mbx.connect_with_config(cfg)
    assert isinstance(r, mbx.Ok), r
    yield r.value
    r.value.close()


@pytest.fixture()
def conn(mbx):
    r = mbx.connect()
    assert isinstance(r, mbx.Ok), r.error.message
    yield r.value
    r.value.close()


def q(conn, sql):
    """Runs a query through the mirror of Connection::query; raises on Err."""
    r = conn.query(sql)
    if not hasattr(r, "value"):
        raise AssertionError(f"query failed: {sql}: {r.error.message}")
    return r.value


def one(conn, sql):
    res = q(conn, sql)
    assert res.row_count() == 1, (sql, res.rows)
    return res.rows[0]
