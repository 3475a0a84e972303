"""TEST INFRASTRUCTURE: byte-exact restatement of the reference shim's
columnar ("arrow") read-back buffers, /root/reference/src/duckdb_native.c.

  int32   :2359-2390  [i32 count][count x i32]        NULL -> 0, value = (int32)int64
  int64   :2392-2422  [i32 count][count x i64]        NULL -> 0
  double  :2424-2454  [i32 count][count x f64]        NULL -> 0.0
  string  :2456-2514  [i32 count][i32 total][s0\\0 s1\\0 ...]   NULL -> "" (1 NUL byte)
  bool    :2516-2546  [i32 count][count x u8]         NULL -> 0
  *_nullable (:2572-2797): the same followed by count validity bytes (1 = valid)
  schema  :2285-2355  [{"name":..,"nullable":true,"type_id":..},...]
An empty buffer is returned for a bad column index or row_count <= 0.
"""
import struct

SCHEMA_TYPE = {1: "bool", 2: "int32", 3: "int32", 4: "int32", 5: "int64", 10: "double", 11: "double"}


def schema(names, type_ids):
    if not names:
        return b"[]"
    parts = []
    for n, t in zip(names, type_ids):
        parts.append('{"name":"%s","nullable":true,"type_id":"%s"}' % (n, SCHEMA_TYPE.get(t, "string")))
    return ("[" + ",".join(parts) + "]").encode()


def _trunc32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= 1 << 31 else v


def int32(values, nullable=False):
    if not values:
        return b""
    out = struct.pack("<i", len(values))
    out += b"".join(struct.pack("<i", 0 if v is None else _trunc32(v)) for v in values)
    if nullable:
        out += bytes(0 if v is None else 1 for v in values)
    return out


def int64(values, nullable=False):
    if not values:
        return b""
    out = struct.pack("<i", len(values)) + b"".join(struct.pack("<q", 0 if v is None else v) for v in values)
    if nullable:
        out += bytes(0 if v is None else 1 for v in values)
    return out


def double(values, nullable=False):
    if not values:
        return b""
    out = struct.pack("<i", len(values)) + b"".join(struct.pack("<d", 0.0 if v is None else v) for v in values)
    if nullable:
        out += bytes(0 if v is None else 1 for v in values)
    return out


def boolean(values, nullable=False):
    if not values:
        return b""
    out = struct.pack("<i", len(values)) + bytes(0 if v is None else (1 if v else 0) for v in values)
    if nullable:
        out += bytes(0 if v is None else 1 for v in values)
    return out


def string(values, nullable=False):
    if not values:
        return b""
    data = b"".join(((v or "").encode() + b"\0") for v in values)
    out = struct.pack("<ii", len(values), len(data)) + data
    if nullable:
        out += bytes(0 if v is None else 1 for v in values)
    return out
