#!/usr/bin/env python3
"""Extracts the reference's 35 golden SQL fixtures into tests/golden/fixtures.json.

Source: /root/reference/src/duckdb_fixture_cases.mbt:4-262 (generated upstream by
scripts/generate_duckdb_fixtures.js with @duckdb/node-api 1.4.3-r.3).  Only the
data (name, sql, expected columns / row strings / null masks) is kept; the
MoonBit record syntax is converted to JSON (keys quoted, trailing commas
dropped; MoonBit string escapes are JSON-compatible here).  Run it in the
development container where /root/reference exists; the GPU box only reads the
committed JSON.
"""
import json
import os
import re
import sys

SRC = "/root/reference/src/duckdb_fixture_cases.mbt"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures.json")


def main():
    text = open(SRC).read()
    body = text[text.index("= [") + 2:]
    body = body[: body.rindex("]") + 1]
    body = re.sub(r"\b(name|sql|columns|rows|nulls):", r'"\1":', body)
    body = re.sub(r",(\s*[\]}])", r"\1", body)
    cases = json.loads(body)
    for c in cases:
        assert set(c) == {"name", "sql", "columns", "rows", "nulls"}, c
    json.dump({"source": "src/duckdb_fixture_cases.mbt:4-262", "cases": cases}, open(OUT, "w"), indent=1)
    print(f"wrote {len(cases)} cases to {OUT}")


if __name__ == "__main__":
    sys.exit(main())
