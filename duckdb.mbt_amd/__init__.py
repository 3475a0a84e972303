"""duckdb.mbt_amd — host-side mirror of the duckdb.mbt MoonBit API over the
MI355X C-ABI library (libduckdb_mb_amd.so, include/duckdb_mb.h).

The reference's host language (MoonBit, `moon` toolchain) is not available in
this image, so this module re-states the MoonBit driver layer on top of the
same 89 `duckdb_mb_*` entry points it binds:

  connect / Connection.query        /root/reference/src/duckdb_native.mbt:429-501
  Connection.query_stream / next    /root/reference/src/duckdb_native.mbt:504-582
  Config / connect_with_config      /root/reference/src/duckdb_native.mbt:608-662
  prepare / bind_* / execute        /root/reference/src/duckdb_native.mbt:760-938
  create_appender / Appender.*      /root/reference/src/duckdb_native.mbt:955-1076
  query_arrow / ArrowResult.*       /root/reference/src/duckdb_arrow_native.mbt:123-822
  QueryResult / Value / ColumnType  /root/reference/src/duckdb.mbt:49-278
  to_typed / TypedQueryResult       /root/reference/src/duckdb_typed_result.mbt:8-379
  column_type_from_id / parse_*     /root/reference/src/duckdb_parsing.mbt:8-257

Callbacks are invoked synchronously (as on the reference's native target).
Results are `Ok(value)` / `Err(DuckDBError)`.  MoonBit `Int` is 32-bit: the
typed layer saturates integers to int32 exactly like parse_int
(duckdb_parsing.mbt:203-237), and the Arrow decoders reject more than
1 000 000 rows (duckdb_arrow_native.mbt:435, :474, ...).

There is no CPU execution path: if the HIP library is missing, importing the
module raises.
"""
from __future__ import annotations

import atexit
import ctypes
import math
import os
import struct
from dataclasses import dataclass, field
from typing import Any, Callable, List, Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DUCKDB_MB_AMD_LIB", os.path.join(_HERE, "libduckdb_mb_amd.so"))


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libduckdb_mb_amd.so not found at {LIB_PATH}: run `make -C duckdb.mbt_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback"
        )
    return ctypes.CDLL(LIB_PATH)


lib = _load()

_P = ctypes.c_void_p
_B = ctypes.POINTER(ctypes.c_uint8)
_I = ctypes.c_int32
_L = ctypes.c_int64


def _sig(name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


# --- MoonBit bytes ----------------------------------------------------------
_sig("moonbit_make_bytes_raw", _B, _I)
_sig("duckdb_mbx_bytes_new", _B, ctypes.c_char_p, _I)
_sig("duckdb_mbx_bytes_len", _I, _B)
_sig("duckdb_mbx_bytes_free", None, _B)
_sig("duckdb_mbx_free", None, _P)
_sig("duckdb_mbx_device_count", _I)
_sig("duckdb_mbx_jit_join", None)
atexit.register(lib.duckdb_mbx_jit_join)  # before exit() tears hipRTC down (jit.h)
_sig("duckdb_mbx_explain", ctypes.c_void_p, _P, ctypes.c_char_p, _L)
_sig("duckdb_mbx_last_profile", ctypes.c_void_p, _P)
_sig("duckdb_mbx_profile_drain", ctypes.c_void_p, _P)
_sig("duckdb_mbx_result_raw", _I, _P, _I, _I, _P, _I)
_sig("duckdb_mbx_result_text", ctypes.c_void_p, _P, ctypes.POINTER(ctypes.c_int64))
_sig("duckdb_mbx_append_column", _I, _P, _I, _P, _P, _L)
_sig("duckdb_mbx_append_commit", _I, _P, _L)
_sig("duckdb_mbx_hbm_calibrate", _I, _P, _L, _I, ctypes.POINTER(ctypes.c_double))
_sig("duckdb_mbx_hbm_calibrate_ex", _I, _P, _L, _I, ctypes.POINTER(ctypes.c_double), _I)
_sig("duckdb_mbx_clock_stamps", _I, _P, ctypes.POINTER(ctypes.c_uint64), _I)
_sig("duckdb_mbx_set_link_mode", _I, _I)
_sig("duckdb_mbx_rccl_selftest", _I, _I, ctypes.POINTER(ctypes.c_double))
_sig("duckdb_mbx_rccl_selftest_ex", ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), _I)
_sig("duckdb_mbx_rccl_info", ctypes.c_void_p, _P)
_sig("duckdb_mbx_link_stats", ctypes.c_void_p)
_sig("duckdb_mbx_statement_plan_stats", _I, _P, ctypes.POINTER(ctypes.c_int64))
_sig("duckdb_mbx_shard_stats", _I, _P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double))
_sig("duckdb_mbx_engine_stats", _I, _P, ctypes.POINTER(ctypes.c_int64))
_sig("duckdb_mbx_shard_timings", _I, _P, ctypes.POINTER(ctypes.c_double), _I)
_sig("duckdb_mbx_shard_partial", _P, _P, _I)
_sig("duckdb_mbx_rccl_stats", _I, _P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double))
_sig("duckdb_mbx_rccl_note", ctypes.c_void_p, _P)
_sig("duckdb_mbx_set_combine", _I, _P, _I)
_sig("duckdb_mbx_rccl_stats_ex", _I, _P, ctypes.POINTER(ctypes.c_int64), _I)
_sig("duckdb_mbx_combine_lanes", _I, ctypes.POINTER(ctypes.c_int64), _I, _I, ctypes.POINTER(ctypes.c_int8),
     ctypes.POINTER(ctypes.c_int64))

for _n in ["duckdb_mb_connect"]:
    _sig(_n, _P, _B)
_sig("duckdb_mb_connect_with_config", _P, _B, _P)
_sig("duckdb_mb_disconnect", None, _P)
_sig("duckdb_mb_is_null_conn", _I, _P)
_sig("duckdb_mb_last_error", _B)
_sig("duckdb_mb_query", _P, _P, _B)
_sig("duckdb_mb_result_destroy", None, _P)
_sig("duckdb_mb_result_column_count", _I, _P)
_sig("duckdb_mb_result_row_count", _I, _P)
_sig("duckdb_mb_result_column_name", _B, _P, _I)
_sig("duckdb_mb_result_column_type", _I, _P, _I)
_sig("duckdb_mb_result_is_null", _I, _P, _I, _I)
_sig("duckdb_mb_result_value", _B, _P, _I, _I)
_sig("duckdb_mb_is_null_result", _I, _P)
_sig("duckdb_mb_query_stream", _P, _P, _B)
_sig("duckdb_mb_execute_prepared_stream", _P, _P)
_sig("duckdb_mb_stream_destroy", None, _P)
_sig("duckdb_mb_is_null_stream", _I, _P)
_sig("duckdb_mb_stream_column_count", _I, _P)
_sig("duckdb_mb_stream_column_name", _B, _P, _I)
_sig("duckdb_mb_stream_fetch_chunk", _P, _P)
_sig("duckdb_mb_chunk_destroy", None, _P)
_sig("duckdb_mb_is_null_chunk", _I, _P)
_sig("duckdb_mb_chunk_row_count", _I, _P)
_sig("duckdb_mb_chunk_column_count", _I, _P)
_sig("duckdb_mb_chunk_is_null", _I, _P, _I, _I)
_sig("duckdb_mb_chunk_value", _B, _P, _I, _I)
_sig("duckdb_mb_config_create", _P)
_sig("duckdb_mb_config_destroy", None, _P)
_sig("duckdb_mb_config_error", _B, _P)
_sig("duckdb_mb_config_set", _I, _P, _B, _B)
_sig("duckdb_mb_prepare", _P, _P, _B)
_sig("duckdb_mb_statement_destroy", None, _P)
_sig("duckdb_mb_statement_error", _B, _P)
_sig("duckdb_mb_bind_int", _I, _P, _I, _I)
_sig("duckdb_mb_bind_bigint", _I, _P, _I, _L)
_sig("duckdb_mb_bind_double", _I, _P, _I, ctypes.c_double)
_sig("duckdb_mb_bind_varchar", _I, _P, _I, _B)
_sig("duckdb_mb_bind_bool", _I, _P, _I, ctypes.c_bool)
_sig("duckdb_mb_bind_null", _I, _P, _I)
_sig("duckdb_mb_clear_bindings", _I, _P)
_sig("duckdb_mb_execute_prepared", _P, _P)
_sig("duckdb_mb_is_null_statement", _I, _P)
_sig("duckdb_mb_bind_date", _I, _P, _I, _I)
_sig("duckdb_mb_bind_timestamp", _I, _P, _I, _L)
_sig("duckdb_mb_bind_decimal", _I, _P, _I, ctypes.c_uint8, ctypes.c_uint8, _L, _L)
_sig("duckdb_mb_bind_interval", _I, _P, _I, _I, _I, _L)
_sig("duckdb_mb_appender_create", _P, _P, _B, _B)
_sig("duckdb_mb_appender_destroy", None, _P)
_sig("duckdb_mb_appender_error", _B, _P)
_sig("duckdb_mb_begin_row", _I, _P)
_sig("duckdb_mb_append_int", _I, _P, _I)
_sig("duckdb_mb_append_bigint", _I, _P, _L)
_sig("duckdb_mb_append_double", _I, _P, ctypes.c_double)
_sig("duckdb_mb_append_varchar", _I, _P, _B)
_sig("duckdb_mb_append_bool", _I, _P, ctypes.c_bool)
_sig("duckdb_mb_append_null", _I, _P)
_sig("duckdb_mb_end_row", _I, _P)
_sig("duckdb_mb_flush", _I, _P)
_sig("duckdb_mb_is_null_appender", _I, _P)
_sig("duckdb_mb_append_date", _I, _P, _I)
_sig("duckdb_mb_append_timestamp", _I, _P, _L)
_sig("duckdb_mb_append_decimal", _I, _P, ctypes.c_uint8, ctypes.c_uint8, _L, _L)
_sig("duckdb_mb_append_interval", _I, _P, _I, _I, _L)
_sig("duckdb_mb_query_arrow", _P, _P, _B)
_sig("duckdb_mb_arrow_destroy", None, _P)
_sig("duckdb_mb_arrow_column_count", _I, _P)
_sig("duckdb_mb_arrow_row_count", _I, _P)
_sig("duckdb_mb_arrow_schema", _B, _P)
for _n in ["int32", "int64", "double", "string", "bool"]:
    _sig(f"duckdb_mb_arrow_get_column_{_n}", _B, _P, _I)
    _sig(f"duckdb_mb_arrow_get_column_{_n}_nullable", _B, _P, _I)
_sig("duckdb_mb_is_null_arrow_result", _I, _P)
_sig("duckdb_mb_bytes_to_double", ctypes.c_double, ctypes.c_char_p, _I)


def _enc(s: str):
    b = s.encode("utf-8")
    return lib.duckdb_mbx_bytes_new(b, len(b))


def _take(bp) -> bytes:
    """Copies a returned MoonBit Bytes object and releases it."""
    if not bp:
        return b""
    n = lib.duckdb_mbx_bytes_len(bp)
    data = ctypes.string_at(bp, n)
    lib.duckdb_mbx_bytes_free(bp)
    return data


def _str(bp) -> str:
    return _take(bp).decode("utf-8", errors="replace")  # @encoding/utf8.decode_lossy


def _result_text(res):
    """(rows, nulls) of a materialized result: the strings and NULL flags that
    duckdb_mb_result_value / _is_null give cell by cell (the loop of
    Connection::query, duckdb_native.mbt:477-497), fetched in ONE C call
    (duckdb_mbx_result_text) instead of two ctypes calls per cell."""
    n = ctypes.c_int64(0)
    p = lib.duckdb_mbx_result_text(res, ctypes.byref(n))
    if not p:
        raise DuckDBError("duckdb_mbx_result_text failed")
    try:
        data = ctypes.string_at(p, n.value)
    finally:
        lib.duckdb_mbx_free(ctypes.c_void_p(p))
    nr, nc = struct.unpack_from("<qq", data, 0)
    ncell = nr * nc
    if ncell == 0:
        return [[] for _ in range(nr)], [[] for _ in range(nr)]
    head = 16 + ((ncell + 7) & ~7)
    offs = struct.unpack_from(f"<{ncell + 1}q", data, head)
    base = head + 8 * (ncell + 1)
    raw = data[base:base + offs[ncell]]
    if raw.isascii():  # one decode; byte offsets are then character offsets
        txt = raw.decode("ascii")
        vals = [txt[a:b] for a, b in zip(offs, offs[1:])]
    else:
        vals = [raw[a:b].decode("utf-8", errors="replace") for a, b in zip(offs, offs[1:])]
    fl = [f == 1 for f in data[16:16 + ncell]]
    rows = [vals[i:i + nc] for i in range(0, ncell, nc)]
    nulls = [fl[i:i + nc] for i in range(0, ncell, nc)]
    return rows, nulls


class _Arg:
    """A MoonBit Bytes argument owned by the caller (borrowed by the callee)."""

    def __init__(self, s: str):
        self.p = _enc(s)

    def __del__(self):
        if self.p:
            lib.duckdb_mbx_bytes_free(self.p)
            self.p = None


def device_count() -> int:
    return lib.duckdb_mbx_device_count()


# --- public types (src/duckdb.mbt) -----------------------------------------
class DuckDBError(Exception):
    """DuckDBError::Message(String)."""

    @property
    def message(self) -> str:
        return self.args[0]


@dataclass
class Ok:
    value: Any


@dataclass
class Err:
    error: DuckDBError


COLUMN_TYPES = {
    0: "Invalid", 1: "Boolean", 2: "TinyInt", 3: "SmallInt", 4: "Integer", 5: "BigInt", 6: "UTinyInt",
    7: "USmallInt", 8: "UInteger", 9: "UBigInt", 10: "Float", 11: "Double", 12: "Timestamp", 13: "Date",
    14: "Time", 15: "Interval", 16: "HugeInt", 17: "Varchar", 18: "Blob", 19: "Decimal", 20: "TimestampS",
    21: "TimestampMs", 22: "TimestampNs", 23: "Enum", 24: "List", 25: "Struct", 26: "Map", 27: "Uuid",
    28: "Union", 29: "Bit", 30: "TimeTz", 31: "TimestampTz", 32: "UHugeInt", 33: "Array", 34: "Any",
    35: "Bignum", 36: "SqlNull", 37: "StringLiteral", 38: "IntegerLiteral", 39: "TimeNs",
}


def column_type_from_id(i: int) -> str:
    """duckdb_parsing.mbt:8-52; unknown ids map to Unknown(id)."""
    return COLUMN_TYPES.get(i, f"Unknown({i})")


INT_MAX = 2**31 - 1
INT_MIN = -(2**31)


def parse_int(s: str) -> int:
    """duckdb_parsing.mbt:203-237: digits accumulate negatively, saturating at
    the 32-bit MoonBit Int range; non-digit characters are skipped."""
    result = 0
    negative = False
    start = 0
    if s:
        if s[0] == "-":
            negative, start = True, 1
        elif s[0] == "+":
            start = 1
    limit = INT_MIN if negative else -INT_MAX
    multmin = int(limit / 10)  # MoonBit Int division truncates
    for c in s[start:]:
        if "0" <= c <= "9":
            digit = ord(c) - 48
            if result < multmin:
                return INT_MIN if negative else INT_MAX
            result = result * 10
            nxt = result - digit
            if nxt < limit:
                return INT_MIN if negative else INT_MAX
            result = nxt
    return result if negative else -result


def is_integer(s: str) -> bool:
    if not s:
        return False
    start = 1 if s[0] in "+-" else 0
    body = s[start:]
    return len(body) > 0 and all("0" <= c <= "9" for c in body)


def is_double(s: str) -> bool:
    if not s:
        return False
    start = 1 if s[0] in "+-" else 0
    has_dot = has_digit = False
    for c in s[start:]:
        if c == ".":
            if has_dot:
                return False
            has_dot = True
        elif not ("0" <= c <= "9"):
            return False
        else:
            has_digit = True
    return has_digit and has_dot


def _parse_fractional(s: str) -> float:
    # duckdb_parsing.mbt parse_fractional: digit / 10^k accumulation
    v, scale = 0.0, 0.1
    for c in s:
        if "0" <= c <= "9":
            v += (ord(c) - 48) * scale
            scale /= 10.0
    return v


def parse_double(s: str) -> float:
    """duckdb_parsing.mbt:241-257."""
    idx = s.find(".")
    if idx >= 0:
        int_val = parse_int(s[:idx])
        frac_val = _parse_fractional(s[idx + 1:])
        sign = -1.0 if s and s[0] == "-" else 1.0
        return sign * (float(abs(int_val)) + frac_val)
    return float(parse_int(s))


SPECIAL_FLOATS = {"nan", "NaN", "inf", "Infinity", "-inf", "-Infinity"}


@dataclass
class Value:
    kind: str  # "Null" | "Bool" | "Int" | "Double" | "String" | "Date" | "Timestamp"
    value: Any = None

    def __eq__(self, o):
        return isinstance(o, Value) and self.kind == o.kind and self.value == o.value


def parse_value(s: str) -> Value:
    """duckdb_parsing.mbt:56-78 (date/timestamp detection kept as strings here)."""
    if s == "true":
        return Value("Bool", True)
    if s == "false":
        return Value("Bool", False)
    if is_integer(s):
        return Value("Int", parse_int(s))
    if is_double(s):
        return Value("Double", parse_double(s))
    return Value("String", s)


_INT_KINDS = {"TinyInt", "SmallInt", "Integer", "BigInt", "UTinyInt", "USmallInt", "UInteger", "UBigInt"}
_STR_KINDS = {"Varchar", "Enum", "Uuid", "StringLiteral", "Decimal", "HugeInt", "UHugeInt", "Interval", "List",
              "Struct", "Map", "Array", "Union", "Bit", "Time", "TimeTz", "TimeNs", "Any", "Bignum", "Blob",
              "SqlNull", "IntegerLiteral"}


def parse_value_with_type(s: str, column_type: str) -> Value:
    """duckdb_parsing.mbt:82-144."""
    if column_type == "Boolean":
        return Value("Bool", True) if s == "true" else Value("Bool", False) if s == "false" else Value("String", s)
    if column_type in _INT_KINDS:
        return Value("Int", parse_int(s))
    if column_type in ("Float", "Double"):
        return Value("String", s) if s in SPECIAL_FLOATS else Value("Double", parse_double(s))
    if column_type in _STR_KINDS:
        return Value("String", s)
    if column_type in ("Date",):
        return Value("Date", s)
    if column_type.startswith("Timestamp"):
        return Value("Timestamp", s)
    return parse_value(s)


@dataclass
class QueryResult:
    """src/duckdb.mbt:49-54: row-major strings + null mask + column types."""
    columns: List[str]
    column_types: List[str]
    rows: List[List[str]]
    nulls: List[List[bool]]

    def column_count(self) -> int:
        return len(self.columns)

    def row_count(self) -> int:
        return len(self.rows)

    def cell(self, row: int, col: int) -> Optional[str]:
        """duckdb.mbt:214-220: None for NULL / out of range."""
        if row < 0 or row >= len(self.rows) or col < 0 or col >= len(self.columns):
            return None
        if self.nulls[row][col]:
            return None
        return self.rows[row][col]

    def get_int(self, row: int, col: int) -> Optional[int]:
        c = self.cell(row, col)
        return None if c is None else parse_int(c)

    def to_typed(self) -> "TypedQueryResult":
        """duckdb_typed_result.mbt:8-43 (row-major strings -> column-major Values)."""
        cols = []
        for c in range(len(self.columns)):
            ct = self.column_types[c] if c < len(self.column_types) else "Invalid"
            col = []
            for r in range(len(self.rows)):
                col.append(Value("Null") if self.nulls[r][c] else parse_value_with_type(self.rows[r][c], ct))
            cols.append(col)
        return TypedQueryResult(self.columns, self.column_types, cols, len(self.rows))


@dataclass
class TypedQueryResult:
    columns: List[str]
    column_types: List[str]
    data: List[List[Value]]  # column-major
    nrows: int

    def get_value(self, row: int, col: int) -> Optional[Value]:
        if col < 0 or col >= len(self.data) or row < 0 or row >= self.nrows:
            return None
        return self.data[col][row]

    def get_int(self, row: int, col: int) -> Optional[int]:
        v = self.get_value(row, col)
        return v.value if v is not None and v.kind == "Int" else None

    def get_int_column(self, col: int) -> Optional[List[Optional[int]]]:
        if col < 0 or col >= len(self.data):
            return None
        return [v.value if v.kind == "Int" else None for v in self.data[col]]

    def get_double_column(self, col: int) -> Optional[List[Optional[float]]]:
        if col < 0 or col >= len(self.data):
            return None
        return [v.value if v.kind == "Double" else None for v in self.data[col]]

    def get_string_column(self, col: int) -> Optional[List[Optional[str]]]:
        if col < 0 or col >= len(self.data):
            return None
        return [v.value if v.kind == "String" else None for v in self.data[col]]


@dataclass
class DataChunk:
    columns: List[str]
    rows: List[List[str]]
    nulls: List[List[bool]]

    def row_count(self) -> int:
        return len(self.rows)


def _last_error(fallback: str) -> str:
    msg = _str(lib.duckdb_mb_last_error())
    return fallback if msg == "" else msg


# --- connection ----------------------------------------------------------------
class Connection:
    def __init__(self, handle):
        self._h = handle

    @property
    def handle(self):
        return self._h

    def close(self, on_done: Callable = None):
        if self._h:
            lib.duckdb_mb_disconnect(self._h)
            self._h = None
        if on_done:
            on_done(Ok(None))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # Connection::query (duckdb_native.mbt:454-501): row-major strings + NULL
    # flags of every cell.  The reference's per-cell loop (:477-497) costs two
    # native calls per cell; over ctypes that would be ~2 us per cell, so the
    # same strings come back in one call (_result_text).  query_percell keeps
    # the literal per-cell form over duckdb_mb_result_is_null/_value.
    def query(self, sql: str, on_done: Callable = None):
        return self._query(sql, on_done, _result_text)

    def query_percell(self, sql: str, on_done: Callable = None):
        return self._query(sql, on_done, _result_cells)

    def _query(self, sql, on_done, pull):
        a = _Arg(sql)
        res = lib.duckdb_mb_query(self._h, a.p)
        if lib.duckdb_mb_is_null_result(res):
            out = Err(DuckDBError(_last_error("duckdb_query failed")))
        else:
            ncol = lib.duckdb_mb_result_column_count(res)
            columns, types = [], []
            for c in range(ncol):
                columns.append(_str(lib.duckdb_mb_result_column_name(res, c)))
                types.append(column_type_from_id(lib.duckdb_mb_result_column_type(res, c)))
            try:
                rows, nulls = pull(res)
            finally:
                lib.duckdb_mb_result_destroy(res)
            out = Ok(QueryResult(columns, types, rows, nulls))
        if on_done:
            on_done(out)
        return out

    def query_stream(self, sql: str, on_done: Callable = None):
        a = _Arg(sql)
        s = lib.duckdb_mb_query_stream(self._h, a.p)
        out = Err(DuckDBError(_last_error("duckdb_stream failed"))) if lib.duckdb_mb_is_null_stream(s) \
            else Ok(ResultStream(s))
        if on_done:
            on_done(out)
        return out

    def prepare(self, sql: str, on_done: Callable = None):
        a = _Arg(sql)
        st = lib.duckdb_mb_prepare(self._h, a.p)
        out = Err(DuckDBError(_last_error("duckdb_prepare failed"))) if lib.duckdb_mb_is_null_statement(st) \
            else Ok(PreparedStatement(st))
        if on_done:
            on_done(out)
        return out

    def create_appender(self, schema: str, table: str, on_done: Callable = None):
        a, b = _Arg(schema), _Arg(table)
        ap = lib.duckdb_mb_appender_create(self._h, a.p, b.p)
        out = Err(DuckDBError("create_appender failed")) if lib.duckdb_mb_is_null_appender(ap) \
            else Ok(Appender(ap))
        if on_done:
            on_done(out)
        return out

    def query_arrow(self, sql: str, on_done: Callable = None):
        a = _Arg(sql)
        r = lib.duckdb_mb_query_arrow(self._h, a.p)
        out = Err(DuckDBError(_last_error("duckdb_query_arrow failed"))) if lib.duckdb_mb_is_null_arrow_result(r) \
            else Ok(ArrowResult(r))
        if on_done:
            on_done(out)
        return out

    # extensions
    def explain(self, sql: str) -> str:
        b = sql.encode()
        p = lib.duckdb_mbx_explain(self._h, b, len(b))
        if not p:
            raise DuckDBError(_last_error("explain failed"))
        s = ctypes.string_at(p).decode()
        lib.duckdb_mbx_free(p)
        return s

    def last_profile(self) -> dict:
        import json
        p = lib.duckdb_mbx_last_profile(self._h)
        s = ctypes.string_at(p).decode()
        lib.duckdb_mbx_free(p)
        return json.loads(s)

    def hbm_calibrate(self, nbytes: int = 2 << 30, iters: int = 5) -> dict:
        """This device's measured HBM ceilings (GB/s; a copy counts read + write)."""
        out = (ctypes.c_double * 8)()
        if lib.duckdb_mbx_hbm_calibrate_ex(self._h, nbytes, iters, out, 8) != 8:
            raise DuckDBError(_last_error("hbm_calibrate failed"))
        return {"copy_gbs": out[0], "read_nt_gbs": out[1], "read_gbs": out[2], "ring_read_gbs": out[3],
                "copy_nt4_gbs": out[4], "ring_copy_gbs": out[5], "ring_copy_half_gbs": out[6],
                "ring_read2_gbs": out[7], "bytes": nbytes}

    def clock_stamps(self, nwg: int) -> list:
        """In-kernel clock of each of the first `nwg` workgroups of the last
        filter_agg_lds / group_direct_lds / two-array ring launch, in GHz
        (d s_memtime / d s_memrealtime x 100 MHz around its main loop).  Only
        the diagnostic build (libduckdb_mb_amd_clk.so) stamps; [] otherwise."""
        out = (ctypes.c_uint64 * (4 * nwg))()
        n = lib.duckdb_mbx_clock_stamps(self._h, out, nwg)
        res = []
        for i in range(n):
            c0, r0, c1, r1 = out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]
            if r1 > r0 and c1 > c0:
                res.append({"ghz": (c1 - c0) / (r1 - r0) * 0.1, "loop_us": (r1 - r0) / 100.0, "r0": r0})
        return res

    def shard_stats(self) -> dict:
        """Counters of the in-library multi-device path (gpu_devices; extension)."""
        out = (ctypes.c_int64 * 6)()
        outd = (ctypes.c_double * 2)()
        lib.duckdb_mbx_shard_stats(self._h, out, outd)
        return {"shards": out[0], "peer_links": out[1], "dispatches": out[2], "peer_copies": out[3],
                "peer_bytes": out[4], "host_results": out[5], "last_dispatch_us": outd[0],
                "last_combine_us": outd[1]}

    def engine_stats(self) -> dict:
        """select_rounds outcomes (extension): launches, aborts, launch failures."""
        out = (ctypes.c_int64 * 3)()
        lib.duckdb_mbx_engine_stats(self._h, out)
        return {"select_rounds_launches": out[0], "select_rounds_aborts": out[1],
                "select_rounds_launch_failures": out[2]}

    def shard_timings(self) -> list:
        """The last sharded dispatch, per shard (extension): device and the us
        since the dispatch began at which the worker took the job (wake), its
        launches were queued (launch) and its result reached the host (done)."""
        cap = 256
        out = (ctypes.c_double * (4 * cap))()
        n = lib.duckdb_mbx_shard_timings(self._h, out, cap)
        return [{"shard": i, "device": int(out[4 * i]), "wake_us": out[4 * i + 1], "launch_us": out[4 * i + 2],
                 "done_us": out[4 * i + 3]} for i in range(min(n, cap))]

    def shard_partial(self, shard: int):
        """Shard `shard`'s partial aggregate row(s) of the last sharded aggregate
        as a RawResult (None if there is none)."""
        h = lib.duckdb_mbx_shard_partial(self._h, shard)
        return RawResult(h) if h else None

    def rccl_stats(self) -> dict:
        """mbx_combine=rccl counters (extension): RCCL combines, fallbacks to the
        host merge and why the last one fell back, the last collective's us."""
        out = (ctypes.c_int64 * 2)()
        us = (ctypes.c_double * 1)()
        lib.duckdb_mbx_rccl_stats(self._h, out, us)
        ex = (ctypes.c_int64 * 9)()
        lib.duckdb_mbx_rccl_stats_ex(self._h, ex, 9)
        p = lib.duckdb_mbx_rccl_note(self._h)
        note = ctypes.string_at(p).decode()
        lib.duckdb_mbx_free(p)
        return {"rccl_combines": out[0], "rccl_fallbacks": out[1], "rccl_loopbacks": ex[2], "rccl_errors": ex[3],
                "rccl_timeouts": ex[4], "rccl_group_combines": ex[5], "rccl_unsupported": ex[6],
                "rccl_reduces": ex[7], "rccl_allgathers": ex[8], "last_rccl_us": us[0], "note": note}

    def rccl_info(self) -> dict:
        """The RCCL combine's communicators (extension): state, whether their
        open started at connect, its ncclCommInitAll seconds and check us, the
        first combine's wait, every rank's ncclCommCount / ncclCommUserRank /
        ncclCommCuDevice, the counters and the last collective."""
        import json
        p = lib.duckdb_mbx_rccl_info(self._h)
        s = ctypes.string_at(p).decode()
        lib.duckdb_mbx_free(p)
        return json.loads(s)

    def set_combine(self, rccl) -> None:
        """Host merge (False / "host"), RCCL combine (True / "rccl") or, in tests
        with MBX_EXPERIMENTS=1, the RCCL combine over device copies instead of
        the collectives ("rccl_loopback"), from the next statement on."""
        mode = {"host": 0, "rccl": 1, "rccl_loopback": 2}[rccl] if isinstance(rccl, str) else (1 if rccl else 0)
        if not lib.duckdb_mbx_set_combine(self._h, mode):
            raise ValueError(f"mbx_combine mode {rccl!r} refused (the loopback needs MBX_EXPERIMENTS=1)")

    def profile_drain(self) -> list:
        import json
        p = lib.duckdb_mbx_profile_drain(self._h)
        s = ctypes.string_at(p).decode()
        lib.duckdb_mbx_free(p)
        return json.loads(s)

    def query_raw(self, sql: str):
        """Runs a query and returns the raw handle (caller destroys); raises on error."""
        a = _Arg(sql)
        res = lib.duckdb_mb_query(self._h, a.p)
        if lib.duckdb_mb_is_null_result(res):
            raise DuckDBError(_last_error("duckdb_query failed"))
        return RawResult(res)


class RawResult:
    """Direct access to a materialized result (no per-row Python lists)."""

    def __init__(self, h):
        self._h = h

    def close(self):
        if self._h:
            lib.duckdb_mb_result_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def row_count(self):
        return lib.duckdb_mb_result_row_count(self._h)

    def column_count(self):
        return lib.duckdb_mb_result_column_count(self._h)

    def column_type(self, c):
        return lib.duckdb_mb_result_column_type(self._h, c)

    def is_null(self, c, r):
        return bool(lib.duckdb_mb_result_is_null(self._h, c, r))

    def value(self, c, r) -> str:
        return _str(lib.duckdb_mb_result_value(self._h, c, r))

    def cells(self):
        """(rows, nulls): every cell's string and NULL flag in one call."""
        return _result_text(self._h)

    def raw(self, c, r) -> bytes:
        buf = ctypes.create_string_buffer(16)
        n = lib.duckdb_mbx_result_raw(self._h, c, r, buf, 16)
        return buf.raw[:n]


def rccl_selftest(device=0) -> dict:
    """The RCCL calls of the combine on hardware (extension): a fresh
    ncclCommInitAll over `device` (an int: one rank) or a list of distinct
    devices (one rank each), then the multi-rank check the combine is gated on
    (one grouped reduce and one all-gather, verified on every rank).  The dict
    has ok, error, us, and for a device list init_us / check_us and every
    rank's ncclCommCount / ncclCommUserRank / ncclCommCuDevice."""
    import json
    if isinstance(device, int):
        us = (ctypes.c_double * 1)()
        ok = lib.duckdb_mbx_rccl_selftest(device, us) == 1
        return {"ok": ok, "us": us[0], "error": "" if ok else _last_error("rccl self-test failed")}
    devs = (ctypes.c_int32 * max(1, len(device)))(*device)
    p = lib.duckdb_mbx_rccl_selftest_ex(devs, len(device))
    r = json.loads(ctypes.string_at(p).decode())
    lib.duckdb_mbx_free(p)
    r["us"] = r.get("total_us")
    return r


def set_link_mode(mode: int) -> None:
    """Arrow getter copies of 2-32 MiB, process-wide (extension): -1 the measured
    choice (default), 0 the runtime's copy, 1 a registered destination, 2 the
    pinned bounce."""
    lib.duckdb_mbx_set_link_mode(mode)


def link_stats() -> list:
    """Per device and size class of the 2-32 MiB getter copies: each method's
    trial medians (GB/s), the method kept, the calls served (extension)."""
    import json
    p = lib.duckdb_mbx_link_stats()
    s = ctypes.string_at(p).decode()
    lib.duckdb_mbx_free(p)
    return json.loads(s)


def connect(on_ready: Callable = None, path: str = ":memory:"):
    """connect (duckdb_native.mbt:429-442)."""
    a = _Arg(path)
    h = lib.duckdb_mb_connect(a.p)
    out = Err(DuckDBError(_last_error("duckdb_open failed"))) if lib.duckdb_mb_is_null_conn(h) else Ok(Connection(h))
    if on_ready:
        on_ready(out)
    return out


class Config:
    """Config::create / Config::set (duckdb_native.mbt:608-627)."""

    def __init__(self):
        self._h = lib.duckdb_mb_config_create()

    @staticmethod
    def create():
        return Config()

    def set(self, key: str, value: str):
        a, b = _Arg(key), _Arg(value)
        if lib.duckdb_mb_config_set(self._h, a.p, b.p):
            return Ok(None)
        msg = _str(lib.duckdb_mb_config_error(self._h))
        return Err(DuckDBError(msg or "config_set failed"))

    def __del__(self):
        if getattr(self, "_h", None):
            lib.duckdb_mb_config_destroy(self._h)
            self._h = None


def connect_with_config(config: Config, on_ready: Callable = None, path: str = ":memory:"):
    a = _Arg(path)
    h = lib.duckdb_mb_connect_with_config(a.p, config._h)
    out = Err(DuckDBError(_last_error("duckdb_open failed"))) if lib.duckdb_mb_is_null_conn(h) else Ok(Connection(h))
    if on_ready:
        on_ready(out)
    return out


class ResultStream:
    def __init__(self, h):
        self._h = h

    def column_count(self) -> int:
        return lib.duckdb_mb_stream_column_count(self._h)

    def columns(self) -> List[str]:
        return [_str(lib.duckdb_mb_stream_column_name(self._h, c)) for c in range(self.column_count())]

    def next(self, on_done: Callable = None):
        """ResultStream::next (duckdb_native.mbt:535-582)."""
        ch = lib.duckdb_mb_stream_fetch_chunk(self._h)
        if lib.duckdb_mb_is_null_chunk(ch):
            msg = _str(lib.duckdb_mb_last_error())
            out = Ok(None) if msg == "" else Err(DuckDBError(msg))
        else:
            nrow = lib.duckdb_mb_chunk_row_count(ch)
            ncol = lib.duckdb_mb_chunk_column_count(ch)
            if nrow <= 0 or ncol <= 0:
                lib.duckdb_mb_chunk_destroy(ch)
                out = Ok(None)
            else:
                cols = self.columns()
                rows, nulls = [], []
                for r in range(nrow):
                    rv, rn = [], []
                    for c in range(ncol):
                        isnull = bool(lib.duckdb_mb_chunk_is_null(ch, c, r))
                        rn.append(isnull)
                        rv.append("" if isnull else _str(lib.duckdb_mb_chunk_value(ch, c, r)))
                    rows.append(rv)
                    nulls.append(rn)
                lib.duckdb_mb_chunk_destroy(ch)
                out = Ok(DataChunk(cols, rows, nulls))
        if on_done:
            on_done(out)
        return out

    def next_count(self) -> Optional[int]:
        """Row count of the next chunk without per-cell pulls (None at end)."""
        ch = lib.duckdb_mb_stream_fetch_chunk(self._h)
        if lib.duckdb_mb_is_null_chunk(ch):
            msg = _str(lib.duckdb_mb_last_error())
            if msg:
                raise DuckDBError(msg)
            return None
        n = lib.duckdb_mb_chunk_row_count(ch)
        lib.duckdb_mb_chunk_destroy(ch)
        return n

    def close(self, on_done: Callable = None):
        if self._h:
            lib.duckdb_mb_stream_destroy(self._h)
            self._h = None
        if on_done:
            on_done(Ok(None))


class PreparedStatement:
    def __init__(self, h):
        self._h = h

    def _r(self, ok, what):
        if ok:
            return Ok(None)
        msg = _str(lib.duckdb_mb_statement_error(self._h))
        return Err(DuckDBError(msg or f"{what} failed"))

    def bind_int(self, i, v):
        return self._r(lib.duckdb_mb_bind_int(self._h, i, v), "bind_int")

    def bind_bigint(self, i, v):
        return self._r(lib.duckdb_mb_bind_bigint(self._h, i, v), "bind_bigint")

    def bind_double(self, i, v):
        return self._r(lib.duckdb_mb_bind_double(self._h, i, v), "bind_double")

    def bind_varchar(self, i, v):
        a = _Arg(v)
        return self._r(lib.duckdb_mb_bind_varchar(self._h, i, a.p), "bind_varchar")

    def bind_bool(self, i, v):
        return self._r(lib.duckdb_mb_bind_bool(self._h, i, bool(v)), "bind_bool")

    def bind_null(self, i):
        return self._r(lib.duckdb_mb_bind_null(self._h, i), "bind_null")

    def bind_date(self, i, days):
        return self._r(lib.duckdb_mb_bind_date(self._h, i, days), "bind_date")

    def bind_timestamp(self, i, micros):
        return self._r(lib.duckdb_mb_bind_timestamp(self._h, i, micros), "bind_timestamp")

    def bind_decimal(self, i, width, scale, value: int):
        lower = value & ((1 << 64) - 1)
        upper = value >> 64
        if lower >= 1 << 63:
            lower -= 1 << 64
        return self._r(lib.duckdb_mb_bind_decimal(self._h, i, width, scale, lower, upper), "bind_decimal")

    def clear_bindings(self):
        return self._r(lib.duckdb_mb_clear_bindings(self._h), "clear_bindings")

    def plan_stats(self) -> dict:
        """Bound-plan cache counters (extension): binds and plan reuses."""
        out = (ctypes.c_int64 * 2)()
        lib.duckdb_mbx_statement_plan_stats(self._h, out)
        return {"binds": out[0], "reuses": out[1]}

    def execute(self, on_done: Callable = None):
        res = lib.duckdb_mb_execute_prepared(self._h)
        if lib.duckdb_mb_is_null_result(res):
            out = Err(DuckDBError(_last_error("execute failed")))
        else:
            out = Ok(_materialize(res))
        if on_done:
            on_done(out)
        return out

    def execute_stream(self, on_done: Callable = None):
        s = lib.duckdb_mb_execute_prepared_stream(self._h)
        out = Err(DuckDBError(_last_error("execute_stream failed"))) if lib.duckdb_mb_is_null_stream(s) \
            else Ok(ResultStream(s))
        if on_done:
            on_done(out)
        return out

    def close(self, on_done: Callable = None):
        if self._h:
            lib.duckdb_mb_statement_destroy(self._h)
            self._h = None
        if on_done:
            on_done(Ok(None))


def _result_cells(res):
    """The reference's literal per-cell pull (duckdb_native.mbt:477-497)."""
    ncol = lib.duckdb_mb_result_column_count(res)
    nrow = lib.duckdb_mb_result_row_count(res)
    rows, nulls = [], []
    for r in range(nrow):
        rn = [bool(lib.duckdb_mb_result_is_null(res, c, r)) for c in range(ncol)]
        rv = ["" if rn[c] else _str(lib.duckdb_mb_result_value(res, c, r)) for c in range(ncol)]
        rows.append(rv)
        nulls.append(rn)
    return rows, nulls


def _materialize(res) -> QueryResult:
    ncol = lib.duckdb_mb_result_column_count(res)
    columns = [_str(lib.duckdb_mb_result_column_name(res, c)) for c in range(ncol)]
    types = [column_type_from_id(lib.duckdb_mb_result_column_type(res, c)) for c in range(ncol)]
    try:
        rows, nulls = _result_text(res)
    finally:
        lib.duckdb_mb_result_destroy(res)
    return QueryResult(columns, types, rows, nulls)


class Appender:
    def __init__(self, h):
        self._h = h

    def _r(self, ok, what):
        if ok:
            return Ok(None)
        msg = _str(lib.duckdb_mb_appender_error(self._h))
        return Err(DuckDBError(msg or f"{what} failed"))

    def begin_row(self):
        return self._r(lib.duckdb_mb_begin_row(self._h), "begin_row")

    def append_int(self, v):
        return self._r(lib.duckdb_mb_append_int(self._h, v), "append_int")

    def append_bigint(self, v):
        return self._r(lib.duckdb_mb_append_bigint(self._h, v), "append_bigint")

    def append_double(self, v):
        return self._r(lib.duckdb_mb_append_double(self._h, v), "append_double")

    def append_varchar(self, v):
        a = _Arg(v)
        return self._r(lib.duckdb_mb_append_varchar(self._h, a.p), "append_varchar")

    def append_bool(self, v):
        return self._r(lib.duckdb_mb_append_bool(self._h, bool(v)), "append_bool")

    def append_null(self):
        return self._r(lib.duckdb_mb_append_null(self._h), "append_null")

    def append_date(self, days):
        return self._r(lib.duckdb_mb_append_date(self._h, days), "append_date")

    def append_timestamp(self, micros):
        return self._r(lib.duckdb_mb_append_timestamp(self._h, micros), "append_timestamp")

    def append_decimal(self, width, scale, value: int):
        lower = value & ((1 << 64) - 1)
        upper = value >> 64
        if lower >= 1 << 63:
            lower -= 1 << 64
        return self._r(lib.duckdb_mb_append_decimal(self._h, width, scale, lower, upper), "append_decimal")

    def end_row(self):
        return self._r(lib.duckdb_mb_end_row(self._h), "end_row")

    def flush(self):
        return self._r(lib.duckdb_mb_flush(self._h), "flush")

    def append_column(self, col: int, array, validity=None):
        """Columnar bulk ingest (extension): `array` is a numpy array in the
        column's physical layout.  The library keeps only the pointers until
        commit(), so the (contiguous) arrays are held here until then."""
        import numpy as np
        array = np.ascontiguousarray(array)
        if validity is not None:
            validity = np.ascontiguousarray(validity, dtype=np.uint8)
        if not hasattr(self, "_held"):
            self._held = {}
        self._held[col] = (array, validity)
        vp = validity.ctypes.data if validity is not None else None
        return self._r(lib.duckdb_mbx_append_column(self._h, col, array.ctypes.data, vp, len(array)), "append_column")

    def commit(self, count: int):
        r = self._r(lib.duckdb_mbx_append_commit(self._h, count), "append_commit")
        self._held = {}  # the rows are on the device (or staged): the host arrays may go
        return r

    def close(self, on_done: Callable = None):
        if self._h:
            lib.duckdb_mb_appender_destroy(self._h)
            self._h = None
        if on_done:
            on_done(Ok(None))


# --- Arrow-style columnar read-back (duckdb_arrow_native.mbt) ---------------------
ARROW_MAX_ROWS = 1_000_000  # decoders return [] above this (duckdb_arrow_native.mbt:435, :474, :517, ...)


@dataclass
class ArrowField:
    name: str
    type_id: str
    nullable: bool


@dataclass
class ArrowSchema:
    fields: List[ArrowField] = field(default_factory=list)


def _i32(b: bytes, off: int) -> int:
    return struct.unpack_from("<i", b, off)[0]


def _mb_int(x: int) -> int:
    """The reference int64 decoder (duckdb_arrow_native.mbt:481-503) assembles
    8 bytes into a 32-bit MoonBit Int with shifts of 32..56, which MoonBit
    masks to 0..24: the result is (low word | high word) as Int.  Exact for
    every value in [-2^31, 2^31) (the range the reference tests use)."""
    lo = x & 0xFFFFFFFF
    hi = (x >> 32) & 0xFFFFFFFF
    v = lo | hi
    return v - (1 << 32) if v >= 1 << 31 else v


class ArrowResult:
    def __init__(self, h):
        self._h = h

    def column_count(self):
        return lib.duckdb_mb_arrow_column_count(self._h)

    def row_count(self):
        return lib.duckdb_mb_arrow_row_count(self._h)

    def get_schema(self):
        import json
        txt = _str(lib.duckdb_mb_arrow_schema(self._h))
        try:
            arr = json.loads(txt)
        except Exception as e:  # parse_arrow_schema_json error path
            return Err(DuckDBError(f"schema parse failed: {e}"))
        return Ok(ArrowSchema([ArrowField(f["name"], f["type_id"], f["nullable"]) for f in arr]))

    def _buf(self, kind, col, nullable=False):
        fn = getattr(lib, f"duckdb_mb_arrow_get_column_{kind}{'_nullable' if nullable else ''}")
        return _take(fn(self._h, col))

    def get_column_int32(self, col) -> List[int]:
        b = self._buf("int32", col)
        if len(b) < 4:
            return []
        n = _i32(b, 0)
        if n <= 0 or n > ARROW_MAX_ROWS:
            return []
        return list(struct.unpack_from(f"<{n}i", b, 4))

    def get_column_int64(self, col) -> List[int]:
        """duckdb_arrow_native.mbt:465-505 assembles each value into a 32-bit
        Int (low word); values keep their 64-bit wire form in `raw_int64`."""
        return [_mb_int(v) for v in self.raw_int64(col)]

    def raw_int64(self, col) -> List[int]:
        b = self._buf("int64", col)
        if len(b) < 4:
            return []
        n = _i32(b, 0)
        if n <= 0 or n > ARROW_MAX_ROWS:
            return []
        return list(struct.unpack_from(f"<{n}q", b, 4))

    def raw_int64_bytes(self, col) -> bytes:
        """The wire buffer itself: [int32 count][count x int64 LE]."""
        return self._buf("int64", col)

    def get_column_double(self, col) -> List[float]:
        b = self._buf("double", col)
        if len(b) < 4:
            return []
        n = _i32(b, 0)
        if n <= 0 or n > ARROW_MAX_ROWS:
            return []
        return list(struct.unpack_from(f"<{n}d", b, 4))

    def get_column_bool(self, col) -> List[bool]:
        b = self._buf("bool", col)
        if len(b) < 4:
            return []
        n = _i32(b, 0)
        if n <= 0 or n > ARROW_MAX_ROWS:
            return []
        return [x != 0 for x in b[4:4 + n]]

    def get_column_string(self, col) -> List[str]:
        b = self._buf("string", col)
        if len(b) < 8:
            return []
        n, tot = _i32(b, 0), _i32(b, 4)
        if n <= 0 or n > ARROW_MAX_ROWS:
            return []
        parts = b[8:8 + tot].split(b"\0")
        return [p.decode("utf-8", errors="replace") for p in parts[:n]]

    def _nullable(self, kind, col, width, fmt):
        b = self._buf(kind, col, True)
        if len(b) < 4:
            return [], []
        n = _i32(b, 0)
        if n <= 0 or n > ARROW_MAX_ROWS:
            return [], []
        vals = list(struct.unpack_from(f"<{n}{fmt}", b, 4)) if fmt else list(b[4:4 + n])
        valid = [x != 0 for x in b[4 + n * width:4 + n * width + n]]
        return vals, valid

    def get_column_int32_nullable(self, col):
        return self._nullable("int32", col, 4, "i")

    def get_column_int64_nullable(self, col):
        v, m = self._nullable("int64", col, 8, "q")
        return [_mb_int(x) for x in v], m

    def get_column_double_nullable(self, col):
        return self._nullable("double", col, 8, "d")

    def get_column_bool_nullable(self, col):
        v, m = self._nullable("bool", col, 1, None)
        return [x != 0 for x in v], m

    def get_column_string_nullable(self, col):
        b = self._buf("string", col, True)
        if len(b) < 8:
            return [], []
        n, tot = _i32(b, 0), _i32(b, 4)
        if n <= 0 or n > ARROW_MAX_ROWS:
            return [], []
        parts = b[8:8 + tot].split(b"\0")[:n]
        valid = [x != 0 for x in b[8 + tot:8 + tot + n]]
        return [p.decode("utf-8", errors="replace") for p in parts], valid

    def close(self, on_done: Callable = None):
        if self._h:
            lib.duckdb_mb_arrow_destroy(self._h)
            self._h = None
        if on_done:
            on_done(Ok(None))


def combine_lanes(parts, kinds):
    """The in-library RCCL combine's lane arithmetic run on the host
    (duckdb_mbx_combine_lanes; the device runs the same code, combine.h).
    parts[rank][j] = a partial value (int, up to int128) or None (NULL);
    kinds[j] = "sum" | "min" | "max".  Returns the combined value per column
    (None if every rank's is NULL)."""
    nr, nc = len(parts), len(kinds)
    lanes = (ctypes.c_int64 * (nr * (3 * nc + 1)))()
    m64 = (1 << 64) - 1
    for r, row in enumerate(parts):
        for j, v in enumerate(row):
            base = r * (3 * nc + 1) + 3 * j
            if v is None:
                lanes[base + 2] = 0
                continue
            u = v & ((1 << 128) - 1)
            lo, hi = u & m64, u >> 64
            lanes[base] = lo - (1 << 64) if lo >> 63 else lo
            lanes[base + 1] = hi - (1 << 64) if hi >> 63 else hi
            lanes[base + 2] = 1
    kk = (ctypes.c_int8 * nc)(*[{"sum": 0, "min": 1, "max": 2}[k] for k in kinds])
    out = (ctypes.c_int64 * (3 * nc))()
    if lib.duckdb_mbx_combine_lanes(lanes, nr, nc, kk, out) != 1:
        raise ValueError("combine_lanes: bad arguments")
    res = []
    for j in range(nc):
        if not out[3 * j + 2] & 1:
            res.append(None)
            continue
        v = ((out[3 * j + 1] & m64) << 64) | (out[3 * j] & m64)
        res.append(v - (1 << 128) if v >> 127 else v)
    return res
