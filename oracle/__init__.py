"""oracle — TEST INFRASTRUCTURE ONLY (checker for tests/, smoke(), and the
cpu_baseline leg of bench.py).  Nothing under duckdb.mbt_amd/ imports this.

Contents
  liboracle_mbx.so (oracle.c): multi-threaded C restatement of the hot-path
      arithmetic (synthetic generator, filter+COUNT/SUM/MIN/MAX, GROUP BY SUM,
      order-preserving selection SELECT x WHERE lo <= x <= hi).
  wire.py:   byte-exact restatement of the reference shim's "arrow" buffers
             (/root/reference/src/duckdb_native.c:2285-2797).
  mb.py:     restatement of the MoonBit-side parsing (duckdb_parsing.mbt) used
             to pin the typed-result behaviour.
  fmt.py:    DuckDB text rendering of values (what duckdb_value_varchar
             returns, pinned by src/duckdb_fixture_cases.mbt).

Parity status: pinned by the reference's own golden vectors — the 35 SQL
fixtures (tests/golden/fixtures.json, extracted from
src/duckdb_fixture_cases.mbt by tests/golden/make_fixtures.py), the native and
arrow test assertions (tests/golden/native_cases.json, extracted from
src/duckdb_test.mbt and src/duckdb_arrow_test.mbt by
tests/golden/make_native_cases.py and replayed by
tests/test_gpu_native_cases.py), and closed forms for
large N (e.g. COUNT(range(N) WHERE i%2=0) = ceil(N/2)).  libduckdb itself is
absent from /root/reference and from this image, so it cannot be executed.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle_mbx.so")


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", HERE])


def load():
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    u64, i64, i32, vp = ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p
    lib.orc_splitmix64.restype = u64
    lib.orc_splitmix64.argtypes = [u64]
    lib.orc_synth_i64.argtypes = [vp, i64, u64, i64, u64, i64]
    lib.orc_synth_i32.argtypes = [vp, i64, u64, i64, u64, i64]
    lib.orc_filter_agg_i64.argtypes = [vp, i64, i64, i64, ctypes.c_int, vp, vp, vp, vp]
    lib.orc_synth_filter_count.argtypes = [u64, i64, i64, u64, i64, i64, i64, ctypes.c_int, vp, vp]
    lib.orc_groupby_sum_i32_i64.argtypes = [vp, vp, i64, i32, ctypes.c_int, ctypes.c_int, vp, vp]
    lib.orc_synth_groupby.argtypes = [u64, u64, i64, i64, ctypes.c_int, u64, i64, ctypes.c_int, vp, vp]
    lib.orc_synth_groupby_nulls.argtypes = [vp, vp, vp, i64, i64, ctypes.c_int, vp, vp, vp]
    lib.orc_range_mod_select.restype = i64
    lib.orc_range_mod_select.argtypes = [i64, i64, i64, i64, vp, i64]
    lib.orc_select_i64.restype = i64
    lib.orc_select_i64.argtypes = [vp, i64, i64, i64, ctypes.c_int, vp]
    return lib


def i128_from(b: bytes) -> int:
    return int.from_bytes(b, "little", signed=True)


class Oracle:
    def __init__(self):
        self.lib = load()

    def splitmix64(self, z: int) -> int:
        return self.lib.orc_splitmix64(z & (2**64 - 1))

    def synth_i64(self, n, seed, start, m, add):
        import numpy as np
        out = np.empty(n, dtype=np.int64)
        self.lib.orc_synth_i64(out.ctypes.data, n, seed, start, m, add)
        return out

    def synth_i32(self, n, seed, start, m, add):
        import numpy as np
        out = np.empty(n, dtype=np.int32)
        self.lib.orc_synth_i32(out.ctypes.data, n, seed, start, m, add)
        return out

    def filter_agg_i64(self, x, lo, hi, threads=1):
        c = ctypes.c_uint64()
        s = ctypes.create_string_buffer(16)
        mn, mx = ctypes.c_int64(), ctypes.c_int64()
        self.lib.orc_filter_agg_i64(x.ctypes.data, len(x), lo, hi, threads, ctypes.byref(c), s,
                                    ctypes.byref(mn), ctypes.byref(mx))
        return c.value, i128_from(s.raw), mn.value, mx.value

    def synth_filter_count(self, seed, start, n, m, add, lo, hi, threads=1):
        c = ctypes.c_uint64()
        s = ctypes.create_string_buffer(16)
        self.lib.orc_synth_filter_count(seed, start, n, m, add, lo, hi, threads, ctypes.byref(c), s)
        return c.value, i128_from(s.raw)

    def groupby_sum(self, k, v, kmin, nk, threads=1):
        import numpy as np
        counts = np.zeros(nk, dtype=np.uint64)
        sums = ctypes.create_string_buffer(16 * nk)
        self.lib.orc_groupby_sum_i32_i64(k.ctypes.data, v.ctypes.data, len(k), kmin, nk, threads,
                                         counts.ctypes.data, sums)
        raw = sums.raw  # (one copy: .raw builds a new bytes object per access)
        return [int(c) for c in counts], [i128_from(raw[16 * i:16 * i + 16]) for i in range(nk)]

    def synth_groupby(self, seed_k, seed_v, start, n, nk, vm, vadd, threads=1):
        """C3 over the generator: per-key COUNT(*) and exact SUM(v) (no arrays)."""
        import numpy as np
        counts = np.zeros(nk, dtype=np.uint64)
        sums = ctypes.create_string_buffer(16 * nk)
        self.lib.orc_synth_groupby(seed_k, seed_v, start, n, nk, vm, vadd, threads, counts.ctypes.data, sums)
        raw = sums.raw  # (one copy: .raw builds a new bytes object per access)
        return [int(c) for c in counts], [i128_from(raw[16 * i:16 * i + 16]) for i in range(nk)]

    def synth_groupby_nulls(self, seeds, mods, adds, start, n, threads=1):
        """The C3 GROUP BY with NULL keys and two NULL-able value columns over
        the generator (oracle.c orc_synth_groupby_nulls): a list of groups in
        key order, the NULL key last, each (key or None, COUNT(*), COUNT(v),
        SUM(v) or None, MIN(v), MAX(v), COUNT(w), SUM(w), MIN(w), MAX(w))."""
        import numpy as np
        sd = np.array(seeds, dtype=np.uint64)
        md = np.array(mods, dtype=np.uint64)
        ad = np.array(adds, dtype=np.int64)
        nk = int(mods[0])
        ng = nk + 1
        counts = np.zeros(3 * ng, dtype=np.uint64)
        sums = ctypes.create_string_buffer(2 * ng * 16)
        mm = np.zeros(4 * ng, dtype=np.int64)
        self.lib.orc_synth_groupby_nulls(sd.ctypes.data, md.ctypes.data, ad.ctypes.data, start, n, threads,
                                         counts.ctypes.data, sums, mm.ctypes.data)
        out = []
        raw = sums.raw
        for g in range(ng):
            if not counts[3 * g]:
                continue
            row = [None if g == nk else g, int(counts[3 * g])]
            for c in range(2):
                cv = int(counts[3 * g + 1 + c])
                s = i128_from(raw[16 * (2 * g + c):16 * (2 * g + c) + 16])
                row += [cv, s if cv else None, int(mm[4 * g + 2 * c]) if cv else None,
                        int(mm[4 * g + 2 * c + 1]) if cv else None]
            out.append(tuple(row))
        return out

    def range_mod_select(self, n, k, c, mul):
        import numpy as np
        cap = n // k + 2
        out = np.empty(cap, dtype=np.int64)
        w = self.lib.orc_range_mod_select(n, k, c, mul, out.ctypes.data, cap)
        return out[:w]

    def select_i64(self, x, lo, hi, threads=1, out=None):
        """The passing values of x (lo <= x <= hi) in row order (out: optional
        preallocated int64 array with room for len(x) values)."""
        import numpy as np
        if out is None:
            out = np.empty(max(len(x), 1), dtype=np.int64)
        w = self.lib.orc_select_i64(x.ctypes.data, len(x), lo, hi, threads, out.ctypes.data)
        return out[:w]
