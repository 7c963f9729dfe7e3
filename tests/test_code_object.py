"""Scratch budgets of the shipping kernel instances, read from the gfx950 code
object's metadata in the built library (no GPU).  A scratch access in the
trace loop costs a memory round trip per use; a refactor that makes the
compiler put a value on the stack (e.g. a select between two whole V3
structs, lowered to a pointer select into stack copies) shows up here before
it shows up as a slower kernel.

The diffuse brute-force instances (the C2 headline's forward, the fused
render, the adjoint, createGraph) and the BVH adjoints carry no scratch; the
unbounded adjoint has a few spilled VGPRs; the SPEC instances (Phong paths,
compiled only for scenes with Ks != 0) spill at most 32 B outside the BVH,
and the BVH forwards at 5 waves/SIMD spill by design (ipt_hip.hip,
IPT_MIN_BLOCKS_*)."""
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import code_object_resources as COR  # noqa: E402

LIB = os.path.join(ROOT, "inverse_path_tracer_amd", "lib", "libipt_amd.so")

# (MODE, SPEC, BVH) -> max scratch bytes per lane
BUDGET = {
    (0, False, False): 0,   # forward (sample buffer)
    (4, False, False): 0,   # fused render: the C2 headline
    (1, False, False): 0,   # adjoint: the C2 headline's gradient
    (5, False, False): 8,   # adjoint at 6 waves/SIMD (80 VGPRs, full-size launches): work item + Le in LDS
                            # (round 5: 16 B reloaded per pair block; 12 B for one build of the fp32 sin/cos, §12.11)
    (2, False, False): 0,   # createGraph
    (2, False, True): 0,
    (1, False, True): 0,    # BVH adjoint (2 waves/SIMD, 256 VGPRs allowed)
    (3, False, True): 0,
    (3, False, False): 12,  # unbounded adjoint: pool chunks (round 5: 8 B; round 6: 12 B with the uniform-region
                            # flag, DESIGN.md §12.9, under which this launch is 1.2-1.4% faster; 20 B with the fp32
                            # sin/cos before its quadrant select became sign flips, §12.11)
    (0, False, True): 0,    # BVH forward: the work item, source triangle and Le in LDS (round 5; was 44-52 B)
    # SPEC instances (materials with a Phong lobe): pow_d out of line keeps its
    # constants out of the trace loop (round 4: 164-292 B per lane)
    (0, True, False): 0,    # (16 B until the fp32 sin/cos, §12.11)
    (1, True, False): 0,
    (3, True, False): 32,
    (4, True, False): 32,
    (1, True, True): 0,
    (0, True, True): 16,    # BVH forward + Phong at 5 waves/SIMD (32 B until the fp32 sin/cos)
}


def name(mode, spec, bvh):
    return "ipt::trace_kernel<%d, %s, %s>" % (mode, "true" if spec else "false", "true" if bvh else "false")


@pytest.mark.skipif(not os.path.exists(COR.READELF), reason="llvm-readelf absent")
def test_trace_kernel_scratch_budgets():
    assert os.path.exists(LIB), "run __graft_entry__.build()"
    r = COR.resources(LIB)
    for key, cap in BUDGET.items():
        k = name(*key)
        assert k in r, k
        assert r[k]["scratch_bytes_per_lane"] <= cap, (k, r[k])
    # every trace_kernel instance is in the object (5 modes x SPEC x BVH, + the 6-wave adjoint)
    assert sum(1 for k in r if k.startswith("ipt::trace_kernel<")) == 21
