"""Per-kernel durations from a rocprofv3 --kernel-trace CSV, split into the
launches that ran alone (no other launch of a trace kernel overlapping them:
bench.py's serial pass, whose HIP-event time is `roofline.kernel_ms`) and
those that overlapped another (the headline's frames-in-flight pass).

    python tools/prof_split.py gpurun_out/prof_X/run_kernel_trace.csv [out.json]
"""
import csv
import json
import sys
from collections import defaultdict


def main(path, out=None):
    rows = list(csv.DictReader(open(path)))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows]
    ev.sort()
    trace = [e for e in ev if "trace_kernel" in e[2]]
    res = defaultdict(lambda: {"alone": [], "overlapped": []})
    for i, (s, e, k) in enumerate(trace):
        over = any(o_s < e and s < o_e for j, (o_s, o_e, _) in enumerate(trace) if j != i and abs(j - i) <= 4)
        res[k]["overlapped" if over else "alone"].append((e - s) / 1e3)
    summary = {k: {kind: {"launches": len(v), "avg_us": round(sum(v) / len(v), 1) if v else None}
                   for kind, v in d.items()} for k, d in res.items()}
    print(json.dumps(summary, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump({"source": path, "kernels": summary}, f, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:3])
