"""The C-ABI boundary: the library loads and exports every symbol the
reference's MoonBit FFI binds (duckdb_native.mbt:10-411, :669-743;
duckdb_arrow_native.mbt:10-104) and every symbol include/duckdb_mb.h declares.
No compute calls here: runs without a GPU."""
import ctypes
import os
import re

import pytest

from conftest import LIB, ROOT

REF_SYMBOLS = [
    # the 89 names bound by the reference MoonBit driver (extern "C" fn ... = "duckdb_mb_*")
    "duckdb_mb_connect", "duckdb_mb_connect_with_config", "duckdb_mb_config_create", "duckdb_mb_config_destroy",
    "duckdb_mb_config_set", "duckdb_mb_config_error", "duckdb_mb_appender_create", "duckdb_mb_appender_destroy",
    "duckdb_mb_appender_error", "duckdb_mb_begin_row", "duckdb_mb_append_int", "duckdb_mb_append_bigint",
    "duckdb_mb_append_double", "duckdb_mb_append_varchar", "duckdb_mb_append_bool", "duckdb_mb_append_null",
    "duckdb_mb_end_row", "duckdb_mb_flush", "duckdb_mb_is_null_appender", "duckdb_mb_bind_date",
    "duckdb_mb_bind_timestamp", "duckdb_mb_append_date", "duckdb_mb_append_timestamp", "duckdb_mb_bind_blob",
    "duckdb_mb_append_blob", "duckdb_mb_bind_decimal", "duckdb_mb_append_decimal", "duckdb_mb_bind_interval",
    "duckdb_mb_append_interval", "duckdb_mb_bind_list_varchar", "duckdb_mb_bind_struct_varchar",
    "duckdb_mb_bind_map_varchar_varchar", "duckdb_mb_append_list_varchar", "duckdb_mb_append_struct_varchar",
    "duckdb_mb_append_map_varchar_varchar", "duckdb_mb_disconnect", "duckdb_mb_query", "duckdb_mb_query_stream",
    "duckdb_mb_result_destroy", "duckdb_mb_result_column_count", "duckdb_mb_result_row_count",
    "duckdb_mb_result_column_name", "duckdb_mb_result_column_type", "duckdb_mb_result_is_null",
    "duckdb_mb_result_value", "duckdb_mb_stream_destroy", "duckdb_mb_stream_column_count",
    "duckdb_mb_stream_column_name", "duckdb_mb_stream_fetch_chunk", "duckdb_mb_chunk_destroy",
    "duckdb_mb_chunk_row_count", "duckdb_mb_chunk_column_count", "duckdb_mb_chunk_is_null", "duckdb_mb_chunk_value",
    "duckdb_mb_last_error", "duckdb_mb_is_null_conn", "duckdb_mb_is_null_result", "duckdb_mb_is_null_stream",
    "duckdb_mb_is_null_chunk", "duckdb_mb_prepare", "duckdb_mb_statement_destroy", "duckdb_mb_statement_error",
    "duckdb_mb_bind_int", "duckdb_mb_bind_bigint", "duckdb_mb_bind_double", "duckdb_mb_bind_varchar",
    "duckdb_mb_bind_bool", "duckdb_mb_bind_null", "duckdb_mb_clear_bindings", "duckdb_mb_execute_prepared",
    "duckdb_mb_execute_prepared_stream", "duckdb_mb_is_null_statement", "duckdb_mb_query_arrow",
    "duckdb_mb_arrow_destroy", "duckdb_mb_arrow_column_count", "duckdb_mb_arrow_row_count", "duckdb_mb_arrow_schema",
    "duckdb_mb_arrow_get_column_int32", "duckdb_mb_arrow_get_column_int64", "duckdb_mb_arrow_get_column_double",
    "duckdb_mb_arrow_get_column_string", "duckdb_mb_arrow_get_column_bool",
    "duckdb_mb_arrow_get_column_int32_nullable", "duckdb_mb_arrow_get_column_int64_nullable",
    "duckdb_mb_arrow_get_column_double_nullable", "duckdb_mb_arrow_get_column_string_nullable",
    "duckdb_mb_arrow_get_column_bool_nullable", "duckdb_mb_is_null_arrow_result", "duckdb_mb_bytes_to_double",
]


def test_reference_symbol_list_is_89_distinct():
    assert len(REF_SYMBOLS) == 89 and len(set(REF_SYMBOLS)) == 89


def test_library_exports_reference_symbols(mbx):
    lib = ctypes.CDLL(LIB)
    missing = [s for s in REF_SYMBOLS if not hasattr(lib, s)]
    assert not missing, missing


def test_library_exports_every_header_declaration(mbx):
    hdr = open(os.path.join(ROOT, "include", "duckdb_mb.h")).read()
    names = set(re.findall(r"\b((?:duckdb_mbx?|moonbit)_[a-z0-9_]+)\s*\(", hdr))
    assert len(names) >= 89 + 10
    lib = ctypes.CDLL(LIB)
    missing = [s for s in sorted(names) if not hasattr(lib, s)]
    assert not missing, missing


def test_header_declares_all_reference_symbols():
    hdr = open(os.path.join(ROOT, "include", "duckdb_mb.h")).read()
    for s in REF_SYMBOLS:
        assert re.search(r"\b" + s + r"\s*\(", hdr), s


def test_moonbit_bytes_layout(mbx):
    # header {int32 rc; uint32 meta} precedes the payload; length = meta & (2^28-1)
    b = mbx.lib.duckdb_mbx_bytes_new(b"hello", 5)
    assert mbx.lib.duckdb_mbx_bytes_len(b) == 5
    base = ctypes.cast(b, ctypes.c_void_p).value
    meta = ctypes.c_uint32.from_address(base - 4).value
    rc = ctypes.c_int32.from_address(base - 8).value
    assert meta & ((1 << 28) - 1) == 5 and rc == 1
    assert ctypes.string_at(b, 5) == b"hello"
    mbx.lib.duckdb_mbx_bytes_free(b)
    e = mbx.lib.moonbit_make_bytes_raw(0)
    assert mbx.lib.duckdb_mbx_bytes_len(e) == 0
    mbx.lib.duckdb_mbx_bytes_free(e)


def test_null_handles_are_safe(mbx):
    lib = mbx.lib
    # reference: NULL handle -> 0 / empty / is_null 1 (duckdb_native.c:182-254, :440-535)
    assert lib.duckdb_mb_is_null_conn(None) == 1
    assert lib.duckdb_mb_is_null_result(None) == 1
    assert lib.duckdb_mb_result_column_count(None) == 0
    assert lib.duckdb_mb_result_row_count(None) == 0
    assert lib.duckdb_mb_result_is_null(None, 0, 0) == 1
    assert mbx._take(lib.duckdb_mb_result_value(None, 0, 0)) == b""
    assert lib.duckdb_mb_stream_column_count(None) == 0
    assert lib.duckdb_mb_chunk_row_count(None) == 0
    assert lib.duckdb_mb_arrow_column_count(None) == 0
    assert mbx._take(lib.duckdb_mb_arrow_schema(None)) == b"[]"
    assert mbx._take(lib.duckdb_mb_arrow_get_column_int64(None, 0)) == b""
    lib.duckdb_mb_result_destroy(None)
    lib.duckdb_mb_disconnect(None)
    lib.duckdb_mb_stream_destroy(None)
    lib.duckdb_mb_chunk_destroy(None)
    lib.duckdb_mb_statement_destroy(None)
    lib.duckdb_mb_appender_destroy(None)
    lib.duckdb_mb_arrow_destroy(None)
    assert lib.duckdb_mb_bind_int(None, 1, 1) == 0
    assert lib.duckdb_mb_append_int(None, 1) == 0
    a = mbx._Arg("select 1")
    assert lib.duckdb_mb_query(None, a.p) is None
    assert mbx._str(lib.duckdb_mb_last_error()) == "connection is null"
    assert lib.duckdb_mb_stream_fetch_chunk(None) is None
    assert mbx._str(lib.duckdb_mb_last_error()) == "stream is null"


def test_bytes_to_double(mbx):
    import struct
    buf = b"xxxx" + struct.pack("<d", 3.25)
    assert mbx.lib.duckdb_mb_bytes_to_double(buf, 4) == 3.25


def test_connect_without_gpu_fails_loudly(mbx):
    if mbx.device_count() > 0:
        pytest.skip("a GPU is visible")
    r = mbx.connect()
    assert isinstance(r, mbx.Err)
    assert "GPU" in r.error.message


def test_config_keys(mbx):
    c = mbx.Config.create()
    assert isinstance(c.set("threads", "4"), mbx.Ok)
    assert isinstance(c.set("memory_limit", "1GB"), mbx.Ok)
    assert isinstance(c.set("gpu_device", "0"), mbx.Ok)
    bad = c.set("no_such_option", "x")
    assert isinstance(bad, mbx.Err) and bad.error.message == "duckdb_set_config failed"
    assert isinstance(c.set("threads", "abc"), mbx.Err)
    # in-library sharding: a device list (a device may repeat), rows per part
    assert isinstance(c.set("gpu_devices", "0,1,2,3,4,5,6,7"), mbx.Ok)
    assert isinstance(c.set("gpu_devices", " 0, 0 "), mbx.Ok)
    for bad_list in ("", "0,", "a,b", "0,-1", "1;2"):
        assert isinstance(c.set("gpu_devices", bad_list), mbx.Err), bad_list
    assert isinstance(c.set("mbx_shard_rows", "1000000"), mbx.Ok)
    assert isinstance(c.set("mbx_shard_rows", "-1"), mbx.Err)
    r = mbx.lib.duckdb_mb_connect_with_config(mbx._Arg(":memory:").p, None)
    assert r is None and mbx._str(mbx.lib.duckdb_mb_last_error()) == "config is null"


def test_jit_kernels_compile_without_gpu(mbx):
    # the run-time specialised expression kernels (jit.cpp) compile for gfx950
    # through hipRTC on a host without a GPU
    import ctypes
    f = mbx.lib.duckdb_mbx_jit_selftest
    f.restype = ctypes.c_void_p
    r = f()
    if r:
        log = ctypes.string_at(r).decode(errors="replace")
        mbx.lib.duckdb_mbx_free(ctypes.c_void_p(r))
        raise AssertionError(log[:4000])


def test_rccl_info_and_selftest_refusals_without_gpu(mbx):
    # no handle: an empty object; the device-list self-test refuses a list RCCL
    # cannot take before any RCCL or HIP call (one rank per device)
    import json
    p = mbx.lib.duckdb_mbx_rccl_info(None)
    assert json.loads(ctypes.string_at(p).decode()) == {}
    mbx.lib.duckdb_mbx_free(p)
    r = mbx.rccl_selftest([1, 1])
    assert r["ok"] is False and "not distinct" in r["error"] and r["ranks"] == [], r
    r = mbx.rccl_selftest([])
    assert r["ok"] is False and "no device" in r["error"], r
    st = (ctypes.c_int64 * 9)()
    assert mbx.lib.duckdb_mbx_rccl_stats_ex(None, st, 9) == 0
