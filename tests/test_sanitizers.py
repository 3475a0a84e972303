"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer:
`make -C duckdb.mbt_amd asan` instruments the host side of every translation
unit (parser, binder, formatter, shim handles, executor host code); the C
harness (tests/c_harness/mb_harness.c) is linked against it with the same
runtime and drives, without a GPU, the host-constant checks, the
DataChunk/Vector handles, and every statement of the reference's 35 golden
fixtures plus malformed SQL (as a query, a prepared statement, and every
result cell).  Any sanitizer report fails the test."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "duckdb.mbt_amd")
ASAN_LIB = os.path.join(LIBDIR, "libduckdb_mb_amd_asan.so")
CLANG = "/opt/rocm/lib/llvm/bin/clang"

MALFORMED = [
    "SELEC 1", "SELECT", "SELECT 1 +", "SELECT (1", "SELECT '", "SELECT 'abc", "SELECT 1 FROM", "SELECT * FROM (",
    "SELECT 99999999999999999999999999999999999999999", "SELECT -9223372036854775808", "SELECT 1e400",
    "SELECT CAST('x' AS INTEGER)", "SELECT 1 / 0, 1 // 0, 1 % 0", "SELECT 9223372036854775807 + 1",
    "SELECT 123.4500::DECIMAL(38,10) * 1000000000000000000000000000", "SELECT ?, ?", "SELECT $3",
    "CREATE TABLE", "CREATE TABLE t (", "INSERT INTO nope VALUES (1)", "DROP TABLE nope",
    "SELECT CASE WHEN 1 THEN 2", "SELECT 'a' || NULL || 'b'", "SELECT LENGTH('héllo'), UPPER('ß'), LOWER('ÄB')",
    "SELECT 1 UNION ALL SELECT 'a'", "SELECT i FROM range(3) tbl(i) ORDER BY", "SELECT COUNT(DISTINCT 1)",
    "SELECT " + "1 + " * 2000 + "1", "SELECT " + "(" * 300 + "1" + ")" * 300, "SELECT '" + "x" * 70000 + "'",
]


def _ensure_asan():
    # always through make: a library older than its sources (e.g. lacking a
    # symbol the header gained) is rebuilt; an up-to-date one costs nothing
    subprocess.run(["make", "-s", "-j8", "-C", LIBDIR, "asan"], check=True, capture_output=True)


def _rt_dir():
    import glob
    d = glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so")
    return os.path.dirname(d[0]) if d else ""


def _harness(tmp_path):
    exe = str(tmp_path / "mb_harness_asan")
    subprocess.run([CLANG, "-O1", "-g", "-std=c11", "-fsanitize=address,undefined", "-shared-libasan",
                    "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c_harness", "mb_harness.c"), "-o", exe,
                    "-L", LIBDIR, "-lduckdb_mb_amd_asan", f"-Wl,-rpath,{LIBDIR}", f"-Wl,-rpath,{_rt_dir()}"],
                   check=True, capture_output=True, text=True)
    return exe


def _run(exe, *args):
    env = dict(os.environ)
    # leak checking is off: the HIP runtime keeps allocations until exit;
    # verify_asan_link_order=0 tolerates libraries the environment preloads
    env["ASAN_OPTIONS"] = "detect_leaks=0:verify_asan_link_order=0:halt_on_error=1:abort_on_error=0"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    def big_stack():  # ASan frames are several times larger than plain ones
        import resource
        resource.setrlimit(resource.RLIMIT_STACK, (256 << 20, 256 << 20))
    p = subprocess.run([exe, *args], capture_output=True, text=True, timeout=600, env=env, preexec_fn=big_stack)
    out = p.stdout + p.stderr
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-6000:]
    assert p.returncode == 0, out[-4000:]
    return out


def test_host_code_under_asan_ubsan(tmp_path):
    if not os.path.exists(CLANG):
        pytest.skip("ROCm clang not present")
    _ensure_asan()
    exe = _harness(tmp_path)
    assert "harness cpu: ok" in _run(exe, "cpu")
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "fixtures.json")))["cases"]
    sqlf = tmp_path / "stmts.sql"
    sqlf.write_text("\n".join([c["sql"].replace("\n", " ") for c in fx] + MALFORMED) + "\n")
    out = _run(exe, "sqlfile", str(sqlf))
    assert "sqlfile:" in out
