"""TEST INFRASTRUCTURE: DuckDB's text rendering of values (what the
reference's duckdb_mb_result_value / duckdb_mb_chunk_value return,
/root/reference/src/duckdb_native.c:224-238, :537-667), restated in Python and
pinned by the golden fixtures (src/duckdb_fixture_cases.mbt)."""
import math


def integer(v: int) -> str:
    return str(int(v))


def decimal(unscaled: int, scale: int) -> str:
    if scale == 0:
        return str(unscaled)
    neg = unscaled < 0
    u = -unscaled if neg else unscaled
    ip, fp = divmod(u, 10 ** scale)
    return ("-" if neg else "") + str(ip) + "." + str(fp).rjust(scale, "0")


def double(x: float) -> str:
    """Shortest round-trip digits; fixed for exponents in [-4, 16), else
    scientific; integral values keep '.0' (the layout of Python's repr)."""
    if math.isnan(x):
        return "nan"
    if math.isinf(x):
        return "-inf" if x < 0 else "inf"
    return repr(float(x))


def boolean(b: bool) -> str:
    return "true" if b else "false"
