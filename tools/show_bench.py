"""Summarise a bench.py JSON line (last line of the file given)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d.pop("secondary", {}) or {}
c = d.pop("cpu_baseline", None)
print("value %.1f  grad %.1f  ms/step %.4f  grad ms %.4f  roofline frac %.4f (kernel %.4f ms)" % (
    d["value"], d["grad_value"], d["ms_per_step"], d["grad_ms_per_step"], d["roofline"]["frac"],
    d["roofline"]["kernel_ms"]))
for k, v in s.items():
    if k.startswith("bands"):
        print("%-22s fwd max/mean %.4f adj %.4f  %s" % (k, v["fwd_max_over_mean"], v["adj_max_over_mean"],
                                                      [(b["fwd_ms"], b["adj_ms"]) for b in v["bands"]]))
    else:
        print("%-22s %s" % (k, json.dumps({a: b for a, b in v.items() if a != "workload"})[:300]))
if c:
    print("cpu", c["value"], c["grad_value"], c["value_1core"], c["cores"])
