"""Per-kernel resources of the gfx950 code object inside a built library
(lib/libipt_amd.so by default), read from the code object's own metadata
notes -- no GPU needed:

    python tools/code_object_resources.py [LIB] > resources.json

For each kernel: VGPRs, SGPRs, VGPR/SGPR spill counts, scratch bytes per
lane (private_segment_fixed_size) and the LDS it declares statically.
tests/test_code_object.py holds the budgets of the shipping instances.
"""
import json
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
DEMANGLE = re.compile(r"_ZN3ipt12trace_kernelILi(\d)ELb([01])ELb([01])E")
FIELDS = {
    ".vgpr_count": "vgpr",
    ".sgpr_count": "sgpr",
    ".vgpr_spill_count": "vgpr_spill",
    ".sgpr_spill_count": "sgpr_spill",
    ".private_segment_fixed_size": "scratch_bytes_per_lane",
    ".group_segment_fixed_size": "static_lds_bytes",
}


def gfx950_object(lib):
    """The gfx950 entry of the library's clang offload bundle (raw ELF bytes)."""
    data = open(lib, "rb").read()
    i = data.find(b"__CLANG_OFFLOAD_BUNDLE__")
    if i < 0:
        raise ValueError("%s holds no offload bundle" % lib)
    n = struct.unpack_from("<Q", data, i + 24)[0]
    off = i + 32
    for _ in range(n):
        eo, es, il = struct.unpack_from("<QQQ", data, off)
        tid = data[off + 24:off + 24 + il].decode()
        off += 24 + il
        if tid.endswith("gfx950"):
            return data[i + eo:i + eo + es]
    raise ValueError("%s has no gfx950 code object" % lib)


def kernel_name(sym):
    m = DEMANGLE.match(sym)
    if m:
        return "ipt::trace_kernel<%s, %s, %s>" % (m.group(1), "true" if m.group(2) == "1" else "false",
                                                  "true" if m.group(3) == "1" else "false")
    return sym


def resources(lib=None):
    lib = lib or os.path.join(ROOT, "inverse_path_tracer_amd", "lib", "libipt_amd.so")
    with tempfile.NamedTemporaryFile(suffix=".elf") as f:
        f.write(gfx950_object(lib))
        f.flush()
        text = subprocess.run([READELF, "--notes", f.name], check=True, capture_output=True, text=True).stdout
    out, cur = {}, None
    for line in text.splitlines():
        s = line.strip().lstrip("- ").strip()
        if s.startswith(".name:"):
            cur = out.setdefault(kernel_name(s.split(":", 1)[1].strip()), {})
            continue
        key = s.split(":", 1)[0]
        if cur is not None and key in FIELDS:
            cur[FIELDS[key]] = int(s.split(":", 1)[1])
    return out


if __name__ == "__main__":
    r = resources(sys.argv[1] if len(sys.argv) > 1 else None)
    print(json.dumps({"source": "code object metadata (llvm-readelf --notes) of the built library",
                      "note": "trace_kernel<MODE,SPEC,BVH>: MODE 0 FWD, 1 ADJ, 2 GRAPH, 3 ADJU, 4 FWDM",
                      "kernels": r}, indent=1))
