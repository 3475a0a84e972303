"""TEST INFRASTRUCTURE: restatement of the MoonBit-side typed parsing the
reference applies to result strings (/root/reference/src/duckdb_parsing.mbt),
used to pin the host mirror in duckdb.mbt_amd/__init__.py."""

INT_MAX = 2**31 - 1
INT_MIN = -(2**31)


def parse_int(s: str) -> int:
    """duckdb_parsing.mbt:203-237 — saturates at the 32-bit Int range."""
    neg = s.startswith("-")
    digits = [c for c in (s[1:] if s[:1] in "+-" else s) if "0" <= c <= "9"]
    v = 0
    for c in digits:
        v = v * 10 + (ord(c) - 48)
        if v > 2**31:
            break
    v = -v if neg else v
    return max(INT_MIN, min(INT_MAX, v))


def column_type_from_id(i: int) -> str:
    names = ["Invalid", "Boolean", "TinyInt", "SmallInt", "Integer", "BigInt", "UTinyInt", "USmallInt", "UInteger",
             "UBigInt", "Float", "Double", "Timestamp", "Date", "Time", "Interval", "HugeInt", "Varchar", "Blob",
             "Decimal", "TimestampS", "TimestampMs", "TimestampNs", "Enum", "List", "Struct", "Map", "Uuid", "Union",
             "Bit", "TimeTz", "TimestampTz", "UHugeInt", "Array", "Any", "Bignum", "SqlNull", "StringLiteral",
             "IntegerLiteral", "TimeNs"]
    return names[i] if 0 <= i < len(names) else f"Unknown({i})"


def date_from_ymd(year: int, month: int, day: int) -> int:
    """duckdb_native.mbt:1188-1203 — days since 1970-01-01 (proleptic Gregorian)."""
    import datetime
    return (datetime.date(year, month, day) - datetime.date(1970, 1, 1)).days


def timestamp_from_ymd_hms(year: int, month: int, day: int, hour: int, minute: int, second: int) -> int:
    """duckdb_native.mbt:1250-1266 — microseconds since 1970-01-01 00:00:00."""
    return (date_from_ymd(year, month, day) * 86400 + hour * 3600 + minute * 60 + second) * 1_000_000
