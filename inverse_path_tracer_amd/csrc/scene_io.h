// scene_io.h -- host scene ingest: scene records -> flattened HostScene.
#pragma once
#include <string>
#include <vector>

#include "scene_layout.h"

namespace ipt {

// One OBJECT block of a scene file (ipt_cuda.py:39-59 from_string / ObjParams).
struct ObjectRecord {
  float pos[3] = {0.f, 0.f, 0.f};
  float ori[3] = {0.f, 0.f, 0.f};
  float scl[3] = {1.f, 1.f, 1.f};
  std::string obj_file;
  std::string mtl_file;  // a path, or an inline "*Kd r g b*" material
};

struct HostScene {
  int nT = 0, nE = 0;
  std::vector<TriIsect> isect;
  std::vector<TriGeom> geom;
  std::vector<TriMat> mat;
  std::vector<float> kd;        // nT*3
  std::vector<int> emit_tri;    // nE
  std::vector<float> emit_cdf;  // nE
  std::vector<float> emit_pmf;  // nE
  std::vector<int> obj_first, obj_count;
  float cam[16];
  // triangle BVH (bvh.cpp); empty when the scene cannot use one exactly
  std::vector<BvhNode> bvh_nodes;
  std::vector<BvhPair> bvh_pairs;
  int bvh_depth = 0;           // inner-node levels (stack entries needed)
  // triangles tested by the unrolled brute-force pair loop before the BVH
  // (the few large ones, e.g. Cornell walls, that almost every ray reaches):
  // pairs in ascending original index, padded with zero triangles
  std::vector<TriPair> bvh_big_pairs;
  std::vector<int32_t> bvh_big_idx;  // 2 per pair; 0x7fffffff = padding
  std::vector<PairBox2> bvh_big_boxes;  // their acceptance boxes (culled shadow pre-pass)
  // the same tree collapsed to 8-wide nodes for the cooperative traversal
  std::vector<WideNode> bvh_wide;   // breadth-first, root 0
  std::vector<TriIsect> bvh_wtris;  // leaf triangles (pad[0] = original index)
  int bvh_wdepth = 0;               // wide levels
  float bvh_root_box[6] = {0, 0, 0, 0, 0, 0};  // lo xyz, hi xyz of the whole tree
  // tree entry tests (bvh.cpp tree_cull): bounding sphere (centre xyz,
  // padded radius^2) and per source triangle {face normal xyz, tau}
  float bvh_sphere[4] = {0, 0, 0, 0};
  std::vector<float> bvh_src_cull;
  std::string bvh_status;      // "ok" or why the BVH was not built
};

// Builds the scene (scene.h:89-117 Scene::Scene semantics).  Returns false
// and fills *err on failure (the reference exit(1)s instead).
bool build_scene(const std::vector<ObjectRecord> &objects, HostScene *out, std::string *err);

// Per-triangle export in the oracle's 57-float layout (for parity tests).
void export_triangles(const HostScene &s, float *out);
constexpr int kExportStride = 57;

}  // namespace ipt
