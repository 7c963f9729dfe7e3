// bvh.h -- host-side triangle BVH build (binned SAH) for the exact
// closest-hit traversal of ipt_device.h::closest_hit_bvh.
#pragma once
#include <string>
#include <vector>

#include "scene_io.h"

namespace ipt {

// Builds S->bvh_nodes / bvh_pairs / bvh_depth from S->isect, S->geom and the
// camera.  Returns false (S->bvh_status says why, the vectors stay empty)
// when the scene has a triangle whose acceptance region cannot be bounded
// exactly (non-finite fields, parallel edge planes): such scenes keep the
// brute-force loop.  Scenes with nT < 2 get no BVH either.
bool build_bvh(HostScene *S);

// Per-triangle box of the ACCEPTANCE region (the points at which the fp32
// hit test of ipt_device.h::hit_test can accept), padded for the rounding of
// the hit point and of the traversal's slab test.  lo/hi: 3 floats each.
// Returns 0 = bounded, 1 = never accepted (zero normal), -1 = unbounded.
// verts (nullable): the region's six vertices (the prism's two triangles).
int acceptance_box(const TriIsect &T, const TriGeom &G, double r_all, float lo[3], float hi[3],
                   double verts[6][3] = nullptr);

// Scene-wide coordinate bound used by the padding (max |vertex coordinate|,
// |camera origin|, plus one).
double scene_coord_bound(const HostScene &S);

// Acceptance boxes of the brute-force pair loop's pairs (2j, 2j+1), two pairs
// per record (scene_layout.h PairBox2), for the culled shadow cast of small
// scenes (ipt_device.h::shadow_hit_pairs_small).
std::vector<PairBox2> pair_boxes(const HostScene &S);
// Per (source triangle, emitter): the pairs that might occlude a shadow ray
// (bit j = pair j), nT * nE words; see bvh.cpp.
std::vector<uint32_t> shadow_occluder_masks(const HostScene &S);
// The same over an explicit pair list (2 triangle indices per pair; < 0 or
// >= nT = padding): the BVH scenes' large-triangle pairs.
std::vector<uint32_t> shadow_occluder_masks(const HostScene &S, const std::vector<int> &pair_tris);

}  // namespace ipt
