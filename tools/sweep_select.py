#!/usr/bin/env python3
"""Sweep of the filter -> compaction forms: count-first (filter_count + scan +
compact_recomp, the default when the predicate columns are outputs), ballot
bits (MBX_CC=0: filter_bits + scan + compact), one pass (MBX_SL=1) and launch
shapes of the count-first kernels; interleaved rounds, median kernel times
from the per-launch HIP events.  GPU only.  Usage: sweep_select.py [rows]"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

m = ge._load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
cfg = m.Config.create()
cfg.set("mbx_profile", "true")
c = m.connect_with_config(cfg).value
c.query(f"CREATE TABLE t AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
        f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v, mbx_synth(42, i, 50) + 1 AS x FROM range({n}) tbl(i)")
SQLS = {"sel": "SELECT x FROM t WHERE x > 24", "sel2": "SELECT k, v FROM t WHERE x > 24",
        "sel3": "SELECT v FROM t WHERE x > 24 AND k < 16", "sel4": "SELECT x, k FROM t WHERE x > 24 AND k < 16"}
sqls = {k: SQLS[k] for k in os.environ.get("SWEEP_SQLS", ",".join(SQLS)).split(",")}
variants = os.environ.get("SWEEP_VARIANTS", "count_first,bits,cf_g2,cf_g4,cf_d2,cf_d4").split(",")
rounds = int(os.environ.get("SWEEP_ROUNDS", "5"))
KN = ("select", "filter_bits", "filter_count", "compact")
SHAPES = {  # variant -> environment
    "count_first": {}, "bits": {"MBX_CC": "0"}, "one_pass": {"MBX_SL": "1"},
    "cf_g2": {"MBX_CR_BLOCKS_PER_CU": "2", "MBX_FK_BLOCKS_PER_CU": "2"},
    "cf_g4": {"MBX_CR_BLOCKS_PER_CU": "4", "MBX_FK_BLOCKS_PER_CU": "4"},
    "cf_d2": {"MBX_CR_DEPTH": "2"}, "cf_d4": {"MBX_CR_DEPTH": "4"}, "cf_d6": {"MBX_CR_DEPTH": "6"},
    "k8": {"MBX_FK_CHUNK": "8"}, "k8_g1": {"MBX_FK_CHUNK": "8", "MBX_FK_BLOCKS_PER_CU": "1"},
    "fk_g1": {"MBX_FK_BLOCKS_PER_CU": "1"}, "fk_g2": {"MBX_FK_BLOCKS_PER_CU": "2"},
    "fk_g1d4": {"MBX_FK_BLOCKS_PER_CU": "1", "MBX_FK_DEPTH": "4"},
    "cr_g1": {"MBX_CR_BLOCKS_PER_CU": "1"}, "cr_g1d6": {"MBX_CR_BLOCKS_PER_CU": "1", "MBX_CR_DEPTH": "6"},
}
ALLKEYS = sorted({k for v in SHAPES.values() for k in v})
res = {}
for name, sql in sqls.items():
    times = {v: {k: [] for k in KN} for v in variants}
    walls = {v: [] for v in variants}
    for rnd in range(rounds):
        for v in (variants if rnd % 2 == 0 else variants[::-1]):
            for key in ALLKEYS:
                os.environ.pop(key, None)
            os.environ.update(SHAPES[v])
            st = c.query_stream(sql).value  # the result stays in HBM
            st.close()
            prof = c.last_profile()
            walls[v].append(prof.get("total_ms", 0))
            for k in prof["kernels"]:
                if k["name"] in times[v]:
                    times[v][k["name"]].append(k["ms"])
    res[name] = {v: dict({kn: statistics.median(t) for kn, t in d.items() if t},
                         total_ms=statistics.median(walls[v])) for v, d in times.items()}
    print(name, json.dumps(res[name]), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump({"rows": n, "sweep": res}, open(os.path.join(ROOT, "gpurun_out", "sweep_select.json"), "w"), indent=1)
