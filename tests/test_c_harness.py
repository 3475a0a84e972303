"""The drop-in boundary exercised from C, as MoonBit's native target links it:
tests/c_harness/mb_harness.c is compiled with gcc against include/duckdb_mb.h
and linked to libduckdb_mb_amd.so, with a stand-in MoonBit runtime whose
strong moonbit_make_bytes_raw must win over the library's weak one (every
returned Bytes is checked for the runtime's tag)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "duckdb.mbt_amd")


def _build(tmp_path):
    exe = str(tmp_path / "mb_harness")
    cmd = ["gcc", "-O1", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "c_harness", "mb_harness.c"), "-o", exe,
           "-L", LIBDIR, "-lduckdb_mb_amd", f"-Wl,-rpath,{LIBDIR}"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_c_harness_cpu(mbx, tmp_path):
    exe = _build(tmp_path)
    p = subprocess.run([exe, "cpu"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "harness cpu: ok" in p.stdout


@pytest.mark.gpu
def test_c_harness_gpu(mbx, oracle, tmp_path):
    exe = _build(tmp_path)
    n = 1_000_003
    p = subprocess.run([exe, "gpu", str(n)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    c, _ = oracle.synth_filter_count(42, 0, n, 50, 1, 25, 2**63 - 1, 4)
    assert f"count={c}" in p.stdout


@pytest.mark.gpu
def test_c_harness_c1_native(mbx, tmp_path):
    # C1 consumed natively: per-cell query loop and stream chunks, exact
    import json
    exe = _build(tmp_path)
    p = subprocess.run([exe, "c1", "1"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["exact"] and r["rows"] == 500000 and r["sum"] == 249999500000 and r["stream_chunks"] >= 245


@pytest.mark.gpu
def test_c_harness_c4_data_chunks(mbx, tmp_path):
    # f3: 1e8 INT64 rows ingested through duckdb_mb_append_data_chunk (2048-row
    # vectors, ref src/duckdb_native.c:2029-2132), read back bit-exact
    import json
    exe = _build(tmp_path)
    p = subprocess.run([exe, "c4chunk", "100000000"], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["bit_exact"] and r["rows"] == 100_000_000 and r["ingest_api"] == "append_data_chunk"
