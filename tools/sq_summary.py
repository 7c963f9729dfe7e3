"""Summarise an rocprofv3 --pmc SQ counter CSV per kernel."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    if "ipt" not in k:
        continue
    d = {c: sum(x) / len(x) for c, x in v.items()}
    print(k)
    if "SQ_ACTIVE_INST_VALU" in d and "SQ_THREAD_CYCLES_VALU" in d:
        print("  VALU lane utilisation      %.3f" % (d["SQ_THREAD_CYCLES_VALU"] / (d["SQ_ACTIVE_INST_VALU"] * 64)))
    if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d:
        print("  VALU insts / wave          %.4g   SALU/VALU %.3f   SMEM/VALU %.3f" % (
            d["SQ_INSTS_VALU"] / d["SQ_WAVES"], d.get("SQ_INSTS_SALU", 0) / d["SQ_INSTS_VALU"],
            d.get("SQ_INSTS_SMEM", 0) / d["SQ_INSTS_VALU"]))
    if "SQ_WAVE_CYCLES" in d:
        for c in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in d:
                print("  %-26s %.3f of wave cycles" % (c, d[c] / d["SQ_WAVE_CYCLES"]))
    print("  raw", {c: "%.4g" % x for c, x in d.items()})
