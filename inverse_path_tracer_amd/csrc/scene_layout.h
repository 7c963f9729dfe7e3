// scene_layout.h -- flattened, device-resident scene layout (host + device).
//
// The reference keeps a pointer-rich AoS scene in CUDA managed memory
// (Scene -> Object -> Mesh -> Triangle, scene.h:86-173, scene_basics.h:64-517)
// and recomputes per-triangle constants inside every ray test.  Here the
// scene is flattened once on the host into four SoA-of-records arrays that
// are uploaded to HBM and read by the kernels:
//
//   TriIsect[nT]  80 B  everything the closest-hit test reads (centre,
//                       face normal, three hoisted edge planes).  Read with a
//                       wave-uniform index -> scalar (SMEM) loads.
//   TriGeom[nT]  128 B  vertices, vertex normals, area, sampling frame R:
//                       read once per path vertex by the hit lane.
//   TriMat[nT]    32 B  Ks, shininess, Ke, flags.
//   kd[nT*3]            diffuse albedo -- the per-material parameter vector
//                       of getMaterials/setMaterials (scene.h:145-162); kept
//                       separate so a torch tensor can stand in for it.
//   emitters            global triangle index, CDF and pmf of the area-
//                       weighted light pick (path_trace.cu:39-51).
#pragma once
#include <stdint.h>

namespace ipt {

struct TriIsect {       // 20 floats
  float c[3];           // centre            (scene_basics.h:80-84)
  float n[3];           // face normal       (:86-91)
  float e0[4];          // edge plane (v0,v1): out.xyz, d  (signedDistance :497-503)
  float e1[4];          // edge plane (v1,v2)
  float e2[4];          // edge plane (v2,v0)
  float pad[2];
};
static_assert(sizeof(TriIsect) == 80, "TriIsect layout");

// Two consecutive triangles (2j, 2j+1) field-interleaved: every field is an
// (A, B) float pair, i.e. one 64-bit SGPR pair after the scalar load, which
// is exactly the operand a packed-FP32 instruction (v_pk_fma_f32) takes -- the
// closest-hit loop tests both triangles with one instruction per field.
// Field order: c[3], n[3], e0[4], e1[4], e2[4].  An odd count is padded with
// an all-zero triangle, which the |n.d| < eps test always rejects.
struct TriPair {
  float f[18][2];
};
static_assert(sizeof(TriPair) == 144, "TriPair layout");
inline void pack_pairs(const TriIsect *t, int nT, TriPair *out) {
  for (int j = 0; 2 * j < nT; ++j) {
    for (int h = 0; h < 2; ++h) {
      const int i = 2 * j + h;
      float src[18] = {0.f};
      if (i < nT) {
        const TriIsect &T = t[i];
        const float v[18] = {T.c[0], T.c[1], T.c[2], T.n[0], T.n[1], T.n[2], T.e0[0], T.e0[1], T.e0[2],
                             T.e0[3], T.e1[0], T.e1[1], T.e1[2], T.e1[3], T.e2[0], T.e2[1], T.e2[2], T.e2[3]};
        for (int k = 0; k < 18; ++k) src[k] = v[k];
      }
      for (int k = 0; k < 18; ++k) out[j].f[k][h] = src[k];
    }
  }
}

struct TriGeom {        // 32 floats
  float v[3][3];        // vertices
  float vn[3][3];       // vertex normals (columns of Triangle::normals)
  float area;
  float R[3][3];        // sampling frame, row-major (sampleNextDir)
  uint32_t flags;       // GEOM_AXIS_FLAT
  float pad[3];
};
static_assert(sizeof(TriGeom) == 128, "TriGeom layout");

// The three vertex normals are bitwise equal and axis-aligned (two components
// +-0, one +-1).  Triangle::getNormal's blend-and-renormalise then returns that
// normal EXACTLY: the zero components stay signed zeros, the +-1 component
// becomes +-s with s > 0, and RN(sqrt(RN(s*s))) == s in binary IEEE
// arithmetic, so +-s / s == +-1.  The kernels skip the blend for such
// triangles (every Cornell wall and every cube face) -- a bitwise identity,
// not an approximation.
enum : uint32_t { GEOM_AXIS_FLAT = 1u };

enum : uint32_t { MAT_HAS_KS = 1u, MAT_SPECULAR = 2u };

struct TriMat {         // 8 floats
  float ks[3];
  float shininess;
  float ke[3];
  uint32_t flags;
};
static_assert(sizeof(TriMat) == 32, "TriMat layout");

// ---- triangle BVH (bvh.cpp) for scenes past the brute-force size
// The reference's BVH (bvh.h:109-205) is over OBJECTS and, for the shipped
// scenes (<= 4 objects), a single leaf: its closest hit is brute force over
// every triangle with first-index ties (scene_basics.h:444, bvh.h:75).  This
// BVH is over triangles and returns exactly that hit: boxes bound the region
// where the fp32 hit test can ACCEPT a point (not the triangle itself), and
// the traversal keeps the lexicographic minimum of (t, triangle index).
//
// Binary node, Aila-Laine layout: both children's boxes live in the parent,
// so one 64-B fetch (four 16-B LDS reads) tests two boxes.
//   q[0] = lo0.x hi0.x lo0.y hi0.y   q[1] = lo0.z hi0.z lo1.x hi1.x
//   q[2] = lo1.y hi1.y lo1.z hi1.z   q[3] = child0 child1 (int bits) 0 0
// child >= 0: inner node index; child < 0: leaf, ~child = first_pair << 4 |
// (pairs - 1).  Nodes are stored breadth-first (root 0), so a prefix of the
// array is the top of the tree.
struct BvhNode {
  float q[4][4];
};
static_assert(sizeof(BvhNode) == 64, "BvhNode layout");
constexpr int kBvhLeafPairBits = 4;   // <= 16 triangle pairs per leaf
constexpr int kBvhMaxDepth = 32;      // traversal stack entries (u16, LDS)
// Leaf triangles, two per record in TriPair's field order, plus the ORIGINAL
// triangle indices (the tie-break key and the returned hit index).  An odd
// leaf is padded with an all-zero triangle (never accepted) of index
// 0x7fffffff.
struct BvhPair {
  float f[18][2];
  int32_t idx[2];
  int32_t pad[2];
};
static_assert(sizeof(BvhPair) == 160, "BvhPair layout");

// 8-wide node of the cooperative traversal (ipt_device.h::coop_cast): one
// 32-B slot per child -- lo.xyz, hi.xyz, ref, pad -- so lane j of an 8-lane
// group reads its child with two 16-B loads, the group's eight reads being one
// contiguous 256-B run.  ref >= 0: wide node; ref < 0: leaf, ~ref =
// first_triangle << 4 | (count - 1) into the leaf-triangle array; kWideEmpty:
// unused slot.  Leaf triangles are TriIsect records in leaf order with the
// ORIGINAL triangle index in pad[0] (int bits).
struct WideNode {
  float s[8][8];
};
static_assert(sizeof(WideNode) == 256, "WideNode layout");
constexpr int32_t kWideEmpty = (int32_t)0x80000000;

// Acceptance boxes (bvh.cpp) of the brute-force loop's triangle pairs, two
// pairs per record so one packed fma computes a slab parameter of both:
// f[k] = {pair 2J, pair 2J+1}, k = lo.x hi.x lo.y hi.y lo.z hi.z.  A pair's
// box is the union of its triangles' boxes; a triangle without a bounded
// acceptance region makes its pair's box infinite (never culled); a pair
// that can never be accepted gets {+inf, +inf} per axis (always culled).
struct PairBox2 {
  float f[6][2];
};
static_assert(sizeof(PairBox2) == 48, "PairBox2 layout");

// Device view of a loaded scene (all pointers are device pointers).
struct DevScene {
  int nT, nE;
  const TriIsect *isect;
  const TriGeom *geom;
  const TriMat *mat;
  const float *kd;
  const int *emit_tri;
  const float *emit_cdf;
  const float *emit_pmf;
  float cam[16];        // row-major 4x4 inverse view (scene.h:67-77)
};

// Explicit render parameters (the reference's compile-time constants,
// scene.h:3-13, made run-time; defaults reproduce them).
struct RenderParams;
inline int band_rows(const RenderParams &p);
struct RenderParams {
  int width, height, spp;
  int max_bounces;      // < 0: unbounded (reference semantics)
  uint64_t seed;
  int row_begin, row_end;
  // rows row_begin, row_begin + row_step, ... < row_end are traced (1 =
  // a contiguous band; world = the interleaved share of one rank)
  int row_step = 1;
  // scene batch: nscenes material sets over this geometry in one launch,
  // set b with seed + b * seed_stride (kd, outputs, adjoint image, gradient
  // at per-set strides)
  int nscenes = 1;
  uint64_t seed_stride = 0;
};
// number of image rows a launch traces
inline int band_rows(const RenderParams &p) {
  const int n = p.row_end - p.row_begin;
  return n <= 0 ? 0 : (p.row_step <= 1 ? n : (n + p.row_step - 1) / p.row_step);
}

}  // namespace ipt
