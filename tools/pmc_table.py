"""Per-kernel averages of every counter in one or more rocprofv3 --pmc runs
(the counter_collection.csv files under the given directories / globs).

    python tools/pmc_table.py 'gpurun_out/attr_r04b_*' [--json OUT]
"""
import argparse
import collections
import csv
import glob
import json
import os


def table(patterns):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for pat in patterns:
        for d in sorted(glob.glob(pat)):
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    for r in csv.DictReader(fh):
                        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
                        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: (sum(v) / len(v), len(v)) for c, v in cs.items()} for k, cs in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("patterns", nargs="+")
    ap.add_argument("--json")
    a = ap.parse_args()
    t = table(a.patterns)
    for k, cs in sorted(t.items()):
        if "ipt" not in k:
            continue
        print(k)
        for c, (v, n) in sorted(cs.items()):
            print("  %-40s %14.6g  (%d dispatches)" % (c, v, n))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump({k: {c: v for c, (v, n) in cs.items()} for k, cs in t.items() if "ipt" in k}, fh, indent=1)


if __name__ == "__main__":
    main()
