#!/usr/bin/env python3
"""Turns a rocprofv3 `--pmc FETCH_SIZE [WRITE_SIZE]` counter_collection.csv into
per-launch HBM traffic for our kernels and merges it into
profiles/pmc_traffic.json (read by bench.py's roofline.traffic).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE is reported in KB and
counts exactly half the bytes of a wide (16 B/lane) coalesced streaming read,
so hbm_bytes = FETCH_SIZE * 1024 * 2.  WRITE_SIZE is exact for 16 B/lane
stores (x1024).  Usage: pmc_traffic.py <counter_collection.csv> <kernel-key=substring> ...
A key "<kernel>@<rows>" records a launch over that many rows (bench.py reads it
for lines at that size, e.g. filter_agg@1250000000 for C5).

Every entry it writes carries its provenance: the sha256 of the kernel and
executor sources it was measured with (csrc_digest(), the same digest
bench.py computes at run time), the git commit and the date.  bench.py
reports an entry's bytes as roofline.traffic only while the sources still
hash to that digest; otherwise traffic is null and traffic_source says why.
"""
import collections
import csv
import datetime
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import csrc_digest  # noqa: E402  (one definition of the digest)


def git_head():
    try:
        return subprocess.check_output(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], text=True).strip()
    except Exception:  # noqa: BLE001
        return None


def main():
    path = sys.argv[1]
    keys = dict(a.split("=", 1) for a in sys.argv[2:])
    out_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        for key, sub in keys.items():
            if sub in r["Kernel_Name"]:
                vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for key, counters in vals.items():
        # a FETCH_SIZE pass and a WRITE_SIZE pass (separate runs) merge into one entry
        e = dict(data.get(key, {})) if len(sys.argv) > 2 else {}
        e.update({"source": os.path.basename(path), "launches": max(len(v) for v in counters.values())})
        if "FETCH_SIZE" in counters:
            f = sum(counters["FETCH_SIZE"]) / len(counters["FETCH_SIZE"])
            e["fetch_size_kb_avg"] = f
            e["hbm_read_bytes_per_launch"] = f * 1024 * 2
        if "WRITE_SIZE" in counters:
            w = sum(counters["WRITE_SIZE"]) / len(counters["WRITE_SIZE"])
            e["write_size_kb_avg"] = w
            e["hbm_write_bytes_per_launch"] = w * 1024
        e["hbm_bytes_per_launch"] = e.get("hbm_read_bytes_per_launch", 0) + e.get("hbm_write_bytes_per_launch", 0)
        e["correction"] = "FETCH_SIZE x1024 x2 (gfx950 half-count of 16B/lane streaming reads), WRITE_SIZE x1024"
        if "@" in key:  # "<kernel>@<rows>": measured at that row count per launch
            e["rows"] = int(key.split("@", 1)[1])
        e["csrc_sha256"] = csrc_digest()
        e["git_head"] = git_head()
        e["date"] = datetime.date.today().isoformat()
        data[key] = e
    json.dump(data, open(out_path, "w"), indent=1)
    print(json.dumps(data, indent=1))


if __name__ == "__main__":
    main()
