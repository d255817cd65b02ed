#!/usr/bin/env python3
"""One-line summary of a bench.py JSON line: python3 scripts/bench_brief.py FILE."""
import json
import sys

j = json.load(open(sys.argv[1]))
out = {"config": j["config"]["workload"][:40], "value": j["value"], "ms": j["ms_per_step"]}
for k in ("depth_l1_vs_oracle",):
    if isinstance(j.get(k), dict):
        out["bit_exact"] = j[k].get("bit_exact")
if "roofline" in j:
    out["roofline"] = j["roofline"]["frac"]
rs = j.get("roofline_sweep") or {}
out["fused_ms_view"] = rs.get("avg_ms_per_view")
for k in ("reference_cost", "reference_defaults", "c3", "two_pass_variant", "view_sharded"):
    if isinstance(j.get(k), dict):
        v = j[k]
        out[k] = v.get("error") or (v.get("value"), v.get("ms_per_step"),
                                    (v.get("depth_l1_vs_oracle") or {}).get("bit_exact"))
print(json.dumps(out))
