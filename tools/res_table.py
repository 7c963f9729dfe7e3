"""Compact per-kernel register/scratch table from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (make asm / make variant .res):

    make -C inverse_path_tracer_amd/csrc asm 2> /tmp/res.txt; python tools/res_table.py /tmp/res.txt
"""
import re
import sys

MODES = {"0": "FWD", "1": "ADJ", "2": "GRAPH", "3": "ADJU", "4": "FWDM", "5": "ADJW"}
rows, cur = [], None
for line in open(sys.argv[1], errors="replace"):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/lane\]| \[waves/SIMD\]| \[bytes/block\])?: (\S+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
for r in rows:
    n = r["name"]
    m = re.search(r"trace_kernelILi(\d)ELb(\d)ELb(\d)E", n)
    label = "trace<%s,spec=%s,bvh=%s>" % (MODES[m.group(1)], m.group(2), m.group(3)) if m else n[:40]
    print("%-28s VGPR %4s  scratch %4s  VGPRspill %4s  SGPRspill %4s  occ %s" % (
        label, r.get("VGPRs"), r.get("ScratchSize"), r.get("VGPRs Spill"), r.get("SGPRs Spill"), r.get("Occupancy")))
