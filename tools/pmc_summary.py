"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs,
MI355X_MICROARCH.md "HBM [CDNA4]") into per-launch HBM bytes per kernel.

Corrections: rocprofv3 reports both counters in KB (1024 B); on gfx950
FETCH_SIZE counts half the bytes of wide coalesced reads, so it is doubled.
WRITE_SIZE is exact for 16-B stores and dword atomics.

    python tools/pmc_summary.py gpurun_out/pmc_fetch_r01 gpurun_out/pmc_write_r01 profiles/pmc_fwd_trace_kernel.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_kernel(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit("no counter_collection.csv under %s" % d)
    acc = defaultdict(list)
    with open(f[0]) as fh:
        for row in csv.DictReader(fh):
            if row["Counter_Name"] == counter:
                acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main(fetch_dir, write_dir, out):
    fe, wr = per_kernel(fetch_dir, "FETCH_SIZE"), per_kernel(write_dir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fe) | set(wr)):
        f_kb = fe.get(k, (0.0, 0))[0]
        w_kb = wr.get(k, (0.0, 0))[0]
        kernels[k] = {"fetch_kb_raw": round(f_kb, 3), "write_kb_raw": round(w_kb, 3),
                      "hbm_bytes_per_launch": int(round(2 * f_kb * 1024 + w_kb * 1024)),
                      "launches": max(fe.get(k, (0, 0))[1], wr.get(k, (0, 0))[1])}
    # the forward of the headline: the fused render (MODE_FWDM = 4), else the unfused trace kernel
    fwd = [k for k in kernels if "trace_kernel<4" in k] or [k for k in kernels if "trace_kernel<0" in k]
    res = {"source": [fetch_dir, write_dir], "correction": "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024",
           "kernels": kernels}
    if fwd:
        res["kernel"] = fwd[0]
        res["hbm_bytes_per_launch"] = kernels[fwd[0]]["hbm_bytes_per_launch"]
    # the gradient half of the headline: the adjoint (MODE_ADJW = 5, else MODE_ADJ = 2)
    adj = [k for k in kernels if "trace_kernel<5" in k] or [k for k in kernels if "trace_kernel<2" in k]
    if adj:
        res["grad_kernel"] = adj[0]
        res["grad_hbm_bytes_per_launch"] = kernels[adj[0]]["hbm_bytes_per_launch"]
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v["hbm_bytes_per_launch"] for k, v in kernels.items()}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
