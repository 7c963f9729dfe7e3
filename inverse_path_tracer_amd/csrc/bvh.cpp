// bvh.cpp -- triangle BVH for the exact closest-hit traversal.
//
// What "exact" needs.  The reference's closest hit is the
// brute-force loop of Object::getIntersection (scene_basics.h:426-459) over
// every triangle in order with a strict `<`, i.e. the lexicographic minimum
// of (t, triangle index) over the triangles whose fp32 test accepts.  A BVH
// returns the same hit iff it never prunes a triangle that the fp32 test
// would accept with (t, i) below the current best.  Three facts make that so:
//
//  1. Acceptance region.  The test accepts a hit point q only if its three
//     computed edge-plane distances are <= 0 and q came from the plane
//     equation.  With unit rounding u = 2^-24 the computed distance of a
//     3-term fma chain is within ds = 2^-21 (|e3| + 3 Q) of the exact
//     distance (Q bounds |q|), and q lies within h = 2^-17 * 3 R of the
//     triangle's plane (R bounds every ray origin and hit point: the scene's
//     coordinates and the camera).  So q lies in the prism of the three
//     relaxed half-spaces e_k.x + e3_k <= ds_k cut by the slab
//     |n.(x - c)| <= h: a convex solid whose six vertices are solved below in
//     double precision (Cramer's rule).  A triangle whose relaxed region is
//     not bounded (edge planes not forming a triangle, non-finite fields)
//     makes the whole scene fall back to the brute-force loop.
//  2. Slab test.  The traversal computes each slab parameter as
//     fma(lo, 1/d, -p/d): the exact crossing parameter of a plane displaced
//     by at most 2u(|lo| + 2|p|) <= 6uR.  Boxes are padded by 2^-16 R (over
//     40x that, plus the u|q| between the rounded hit point and the exact ray
//     point), so the computed [entry, exit] always contains the parameter of
//     every acceptable hit.  Slabs with |d| < 2^-60 are dropped (NaN, ignored
//     by min/max): conservative.
//  3. Order.  The leaf test keeps (t, index) lexicographically; a box is
//     pruned only when its entry parameter exceeds the current best t.
//
// The build is a binned SAH (32 bins, pair-granular leaf cost) over the
// acceptance boxes; nodes are emitted breadth-first, leaves as field-
// interleaved triangle pairs in depth-first leaf order.
#include "bvh.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>

namespace ipt {

namespace {

constexpr int kBins = 32;
constexpr int kMaxLeafTris = 8;  // SAH may stop at <= 8 triangles (4 pairs)
constexpr double kCostNode = 1.0, kCostPair = 1.0;
// Triangles whose acceptance box has at least this fraction of the scene
// box's surface area (almost every ray reaches them: room walls) are tested
// by the unrolled brute-force pair loop ahead of the traversal, up to 2 *
// kBigPairs of them, instead of sitting in leaves that every ray visits.
#ifndef IPT_BVH_BIGFRAC  // (make variant DEFS=-DIPT_BVH_BIGFRAC=... for A/B timing)
#define IPT_BVH_BIGFRAC (1.0 / 64)
#endif
constexpr double kBigFrac = IPT_BVH_BIGFRAC;  // 1/32 left the cube of the north-star scene in the tree: fwd 5.27 -> 4.50 ms at 1/64 (profiles/r02_bigfrac_ab.log)
constexpr int kBigPairs = 16;  // = ipt_device.h kSmallPairs

struct Box {
  float lo[3] = {std::numeric_limits<float>::infinity(), std::numeric_limits<float>::infinity(),
                 std::numeric_limits<float>::infinity()};
  float hi[3] = {-std::numeric_limits<float>::infinity(), -std::numeric_limits<float>::infinity(),
                 -std::numeric_limits<float>::infinity()};
  void grow(const Box &b) {
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(lo[a], b.lo[a]);
      hi[a] = std::max(hi[a], b.hi[a]);
    }
  }
  void grow(const float *p) {
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(lo[a], p[a]);
      hi[a] = std::max(hi[a], p[a]);
    }
  }
  double area() const {
    if (!(hi[0] >= lo[0])) return 0.0;
    const double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }
};

struct Prim {
  Box box;
  float c[3];
  int tri;
};

struct TNode {  // build-time inner node
  Box box[2];
  int kid[2];   // >= 0 inner (build index); < 0: ~leaf id
};

struct Builder {
  std::vector<Prim> prims;
  std::vector<TNode> nodes;
  std::vector<std::pair<int, int>> leaves;  // [begin, end) into prims
  int max_depth = 0;
  bool too_deep = false;

  static int pairs_of(int n) { return (n + 1) / 2; }

  // Returns the child code for prims[b, e) and its box.
  int build(int b, int e, int depth, bool force_split, Box *out_box) {
    Box box, cbox;
    for (int i = b; i < e; ++i) {
      box.grow(prims[i].box);
      cbox.grow(prims[i].c);
    }
    *out_box = box;
    const int n = e - b;
    const double leaf_cost = kCostPair * pairs_of(n);
    const bool can_leaf = pairs_of(n) <= (1 << kBvhLeafPairBits);
    if (!force_split && n <= 2) return make_leaf(b, e);
    if (depth >= kBvhMaxDepth - 1) {
      if (can_leaf) return make_leaf(b, e);
      too_deep = true;
      return make_leaf(b, b + 1);  // build is discarded
    }
    // binned SAH over centroids
    int best_axis = -1, best_split = -1;
    double best_cost = std::numeric_limits<double>::infinity();
    const double parent_area = std::max(box.area(), 1e-30);
    for (int a = 0; a < 3; ++a) {
      const double lo = cbox.lo[a], ext = (double)cbox.hi[a] - lo;
      if (!(ext > 0.0)) continue;
      Box bb[kBins];
      int cnt[kBins] = {0};
      for (int i = b; i < e; ++i) {
        int k = (int)((prims[i].c[a] - lo) / ext * kBins);
        k = std::min(std::max(k, 0), kBins - 1);
        cnt[k]++;
        bb[k].grow(prims[i].box);
      }
      double right_area[kBins];
      int right_cnt[kBins];
      Box acc;
      int ac = 0;
      for (int k = kBins - 1; k > 0; --k) {
        acc.grow(bb[k]);
        ac += cnt[k];
        right_area[k] = acc.area();
        right_cnt[k] = ac;
      }
      Box lacc;
      int lc = 0;
      for (int k = 1; k < kBins; ++k) {
        lacc.grow(bb[k - 1]);
        lc += cnt[k - 1];
        if (lc == 0 || right_cnt[k] == 0) continue;
        const double cost = kCostNode + (lacc.area() * kCostPair * pairs_of(lc) +
                                         right_area[k] * kCostPair * pairs_of(right_cnt[k])) / parent_area;
        if (cost < best_cost) {
          best_cost = cost;
          best_axis = a;
          best_split = k;
        }
      }
    }
    if (!force_split && n <= kMaxLeafTris && leaf_cost <= best_cost) return make_leaf(b, e);
    int mid;
    if (best_axis >= 0) {
      const int a = best_axis;
      const double lo = cbox.lo[a], ext = (double)cbox.hi[a] - lo;
      auto it = std::partition(prims.begin() + b, prims.begin() + e, [&](const Prim &p) {
        int k = (int)((p.c[a] - lo) / ext * kBins);
        k = std::min(std::max(k, 0), kBins - 1);
        return k < best_split;
      });
      mid = (int)(it - prims.begin());
    } else {
      mid = b;  // all centroids equal
    }
    if (mid == b || mid == e) {  // degenerate: median by index along the widest axis
      int a = 0;
      for (int k = 1; k < 3; ++k)
        if ((double)cbox.hi[k] - cbox.lo[k] > (double)cbox.hi[a] - cbox.lo[a]) a = k;
      mid = b + n / 2;
      std::nth_element(prims.begin() + b, prims.begin() + mid, prims.begin() + e, [&](const Prim &x, const Prim &y) {
        return x.c[a] < y.c[a] || (x.c[a] == y.c[a] && x.tri < y.tri);
      });
    }
    const int id = (int)nodes.size();
    nodes.emplace_back();
    max_depth = std::max(max_depth, depth + 1);
    Box lb, rb;
    const int l = build(b, mid, depth + 1, false, &lb);
    const int r = build(mid, e, depth + 1, false, &rb);
    nodes[id].box[0] = lb;
    nodes[id].box[1] = rb;
    nodes[id].kid[0] = l;
    nodes[id].kid[1] = r;
    return id;
  }

  int make_leaf(int b, int e) {
    leaves.emplace_back(b, e);
    return ~(int)(leaves.size() - 1);
  }
};

void put_tri(BvhPair *P, int h, const TriIsect *T, int idx) {
  float v[18] = {0.f};
  if (T) {
    const float src[18] = {T->c[0], T->c[1], T->c[2], T->n[0], T->n[1], T->n[2], T->e0[0], T->e0[1], T->e0[2],
                           T->e0[3], T->e1[0], T->e1[1], T->e1[2], T->e1[3], T->e2[0], T->e2[1], T->e2[2], T->e2[3]};
    std::memcpy(v, src, sizeof v);
  }
  for (int k = 0; k < 18; ++k) P->f[k][h] = v[k];
  P->idx[h] = idx;
}

float round_down(double x) {
  float f = (float)x;
  if ((double)f > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
  return f;
}
float round_up(double x) {
  float f = (float)x;
  if ((double)f < x) f = std::nextafter(f, std::numeric_limits<float>::infinity());
  return f;
}

}  // namespace

double scene_coord_bound(const HostScene &S) {
  double m = 0.0;
  for (const TriGeom &g : S.geom)
    for (int j = 0; j < 3; ++j)
      for (int a = 0; a < 3; ++a) m = std::max(m, std::fabs((double)g.v[j][a]));
  for (int a = 0; a < 3; ++a) m = std::max(m, std::fabs((double)S.cam[4 * a + 3]));  // camera origin M*(0,0,0,1)
  return m + 1.0;
}

int acceptance_box(const TriIsect &T, const TriGeom &G, double r_all, float lo[3], float hi[3], double verts[6][3]) {
  const float *fields[5] = {T.c, T.n, T.e0, T.e1, T.e2};
  const int counts[5] = {3, 3, 4, 4, 4};
  for (int f = 0; f < 5; ++f)
    for (int k = 0; k < counts[f]; ++k)
      if (!std::isfinite(fields[f][k])) return -1;
  const double n[3] = {T.n[0], T.n[1], T.n[2]};
  if (n[0] == 0.0 && n[1] == 0.0 && n[2] == 0.0) return 1;  // |n.d| = 0 < 1e-4 for every ray
  double q = 0.0;
  for (int j = 0; j < 3; ++j)
    for (int a = 0; a < 3; ++a) q = std::max(q, std::fabs((double)G.v[j][a]));
  q += 1.0;
  const float *pl[3] = {T.e0, T.e1, T.e2};
  double e[3][3], d[3], ds[3];
  for (int k = 0; k < 3; ++k) {
    for (int a = 0; a < 3; ++a) e[k][a] = pl[k][a];
    d[k] = pl[k][3];
    ds[k] = std::ldexp(std::fabs(d[k]) + 3.0 * q, -21);
  }
  const double h = std::ldexp(3.0 * r_all, -17);
  const double nc = n[0] * T.c[0] + n[1] * T.c[1] + n[2] * T.c[2];
  auto cross = [](const double *a, const double *b, double *o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
  };
  auto dot = [](const double *a, const double *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
  auto norm = [&](const double *a) { return std::sqrt(dot(a, a)); };
  double blo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, bhi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
  for (int j = 0; j < 3; ++j) {
    const int k = (j + 1) % 3, i = (j + 2) % 3;
    double ejk[3], ekn[3], nej[3];
    cross(e[j], e[k], ejk);
    cross(e[k], n, ekn);
    cross(n, e[j], nej);
    const double det = dot(n, ejk);
    if (!(std::fabs(det) > 1e-9 * norm(n) * norm(e[j]) * norm(e[k]))) return -1;
    for (int s = -1; s <= 1; ++s) {
      const double b0 = nc + s * h, b1 = ds[j] - d[j], b2 = ds[k] - d[k];
      double x[3];
      for (int a = 0; a < 3; ++a) x[a] = (b0 * ejk[a] + b1 * ekn[a] + b2 * nej[a]) / det;
      if (s == 0) {  // bounded iff every vertex satisfies the third half-space
        if (!(dot(e[i], x) + d[i] <= ds[i] * (1.0 + 1e-9))) return -1;
      } else {
        for (int a = 0; a < 3; ++a) {
          blo[a] = std::min(blo[a], x[a]);
          bhi[a] = std::max(bhi[a], x[a]);
          if (verts) verts[2 * j + (s > 0 ? 1 : 0)][a] = x[a];
        }
      }
    }
  }
  const double pad = std::ldexp(r_all, -16);
  for (int a = 0; a < 3; ++a) {
    lo[a] = round_down(blo[a] - pad);
    hi[a] = round_up(bhi[a] + pad);
  }
  return 0;
}

std::vector<PairBox2> pair_boxes(const HostScene &S) {
  const float inf = std::numeric_limits<float>::infinity();
  const int nP = (S.nT + 1) / 2;
  std::vector<PairBox2> out((size_t)(nP + 1) / 2);
  const double r_all = scene_coord_bound(S);
  for (int j = 0; j < nP; ++j) {
    float lo[3] = {inf, inf, inf}, hi[3] = {-inf, -inf, -inf};
    bool any = false, unbounded = false;
    for (int h = 0; h < 2; ++h) {
      const int i = 2 * j + h;
      if (i >= S.nT) continue;  // the padding triangle is never accepted
      float l[3], u[3];
      const int rc = acceptance_box(S.isect[(size_t)i], S.geom[(size_t)i], r_all, l, u);
      if (rc < 0) unbounded = true;
      if (rc != 0) continue;
      any = true;
      for (int a = 0; a < 3; ++a) {
        lo[a] = std::min(lo[a], l[a]);
        hi[a] = std::max(hi[a], u[a]);
      }
    }
    float b[6];
    for (int a = 0; a < 3; ++a) {
      b[2 * a] = unbounded ? -inf : (any ? lo[a] : inf);
      b[2 * a + 1] = unbounded ? inf : (any ? hi[a] : inf);
    }
    for (int k = 0; k < 6; ++k) out[(size_t)j / 2].f[k][j & 1] = b[k];
  }
  if (nP & 1)  // the record's unused half: never tested (the loop stops at nP)
    for (int k = 0; k < 6; ++k) out.back().f[k][1] = inf;
  return out;
}

// Potential occluders of next-event shadow rays, per (source triangle S,
// emitter e): bit j = pair j might accept a shadow ray from a vertex on S to
// a point on emitter triangle E = emit_tri[e].  Every such ray has its origin
// p in S's acceptance box (p is the point S's test accepted), its target pt
// in E's vertex box (padded), d = unit(pt - p) within 2^-21 relative, and
// only t in [1e-2, t_E (1 + tiny)] matters.  A triangle w accepts only points
// q with |n_w.q - n_w.c_w| <= h (acceptance_box), and a computed q lies
// within eps << 2^-14 R of the exact line point p + t d.  Along the segment,
// f(x) = n_w.x - n_w.c_w = (1 - s) f(p) + s f(pt), s = t / |pt - p| in
// [1e-2 / L_max, 1]: affine in s, so when f keeps one sign with margin
// h + eps at both ends for every p and pt (box corners bound f), w cannot
// accept.  A pair is left out only if both its triangles are.  The emitter's
// own pair (coplanar partner) always stays; in a room, a wall on whose plane
// S ends (a neighbour) is left out thanks to the 1e-2 lower end.
std::vector<uint32_t> shadow_occluder_masks(const HostScene &S) {
  std::vector<int> tri((size_t)((S.nT + 1) / 2) * 2);
  for (size_t k = 0; k < tri.size(); ++k) tri[k] = (int)k < S.nT ? (int)k : -1;
  return shadow_occluder_masks(S, tri);
}

std::vector<uint32_t> shadow_occluder_masks(const HostScene &S, const std::vector<int> &pair_tris) {
  const int nT = S.nT, nE = S.nE, nP = (int)pair_tris.size() / 2;
  const uint32_t all = nP >= 32 ? 0xffffffffu : ((1u << nP) - 1u);
  std::vector<uint32_t> out((size_t)nT * (size_t)std::max(nE, 1), all);
  if (nP > 32 || nE == 0) return out;
  const double r_all = scene_coord_bound(S);
  const double h = std::ldexp(3.0 * r_all, -17), thr = h + std::ldexp(r_all, -14);
  struct B3 {
    double lo[3], hi[3];
    bool ok;
  };
  std::vector<B3> src((size_t)nT);
  for (int i = 0; i < nT; ++i) {
    float l[3], u[3];
    src[(size_t)i].ok = acceptance_box(S.isect[(size_t)i], S.geom[(size_t)i], r_all, l, u) == 0;
    for (int a = 0; a < 3; ++a) {
      src[(size_t)i].lo[a] = l[a];
      src[(size_t)i].hi[a] = u[a];
    }
  }
  auto corners = [](const B3 &b, int k, double x[3]) {
    for (int a = 0; a < 3; ++a) x[a] = (k >> a) & 1 ? b.hi[a] : b.lo[a];
  };
  for (int e = 0; e < nE; ++e) {
    const int et = S.emit_tri[(size_t)e];
    B3 E;
    E.ok = true;
    const double pad = std::ldexp(r_all, -18);
    for (int a = 0; a < 3; ++a) {
      E.lo[a] = HUGE_VAL;
      E.hi[a] = -HUGE_VAL;
      for (int j = 0; j < 3; ++j) {
        E.lo[a] = std::min(E.lo[a], (double)S.geom[(size_t)et].v[j][a]);
        E.hi[a] = std::max(E.hi[a], (double)S.geom[(size_t)et].v[j][a]);
      }
      E.lo[a] -= pad;
      E.hi[a] += pad;
    }
    for (int si = 0; si < nT; ++si) {
      const B3 &Sb = src[(size_t)si];
      if (!Sb.ok) continue;  // unbounded (or never accepted): every pair stays
      double lmax = 0.0;
      for (int k = 0; k < 8; ++k)
        for (int m = 0; m < 8; ++m) {
          double x[3], y[3];
          corners(Sb, k, x);
          corners(E, m, y);
          lmax = std::max(lmax, std::sqrt((x[0] - y[0]) * (x[0] - y[0]) + (x[1] - y[1]) * (x[1] - y[1]) +
                                          (x[2] - y[2]) * (x[2] - y[2])));
        }
      const double slo = 0.01 / (lmax * (1.0 + 1e-6) + 1e-30);
      uint32_t mask = 0;
      for (int j = 0; j < nP; ++j) {
        bool excluded = true;
        for (int hh = 0; hh < 2 && excluded; ++hh) {
          const int w = pair_tris[(size_t)(2 * j + hh)];
          if (w < 0 || w >= nT) continue;  // the padding triangle is never accepted
          const TriIsect &T = S.isect[(size_t)w];
          const double n[3] = {T.n[0], T.n[1], T.n[2]};
          if (n[0] == 0.0 && n[1] == 0.0 && n[2] == 0.0) continue;  // never accepted
          bool finite = true;
          for (int a = 0; a < 3; ++a) finite = finite && std::isfinite(n[a]) && std::isfinite(T.c[a]);
          if (!finite) {
            excluded = false;
            break;
          }
          const double nc = n[0] * T.c[0] + n[1] * T.c[1] + n[2] * T.c[2];
          auto frange = [&](const B3 &b, double &mn, double &mx) {
            mn = HUGE_VAL;
            mx = -HUGE_VAL;
            for (int k = 0; k < 8; ++k) {
              double x[3];
              corners(b, k, x);
              const double f = n[0] * x[0] + n[1] * x[1] + n[2] * x[2] - nc;
              mn = std::min(mn, f);
              mx = std::max(mx, f);
            }
          };
          double aS, AS, aE, AE;
          frange(Sb, aS, AS);
          frange(E, aE, AE);
          const bool pos = aE > thr && (1.0 - slo) * aS + slo * aE > thr;
          const bool neg = AE < -thr && (1.0 - slo) * AS + slo * AE < -thr;
          if (!(pos || neg)) excluded = false;
        }
        if (!excluded) mask |= 1u << j;
      }
      out[(size_t)si * nE + e] = mask;
    }
  }
  return out;
}

// Collapse the binary tree into 8-wide nodes: starting from a binary node's
// two children, repeatedly open the inner child with the largest box until
// the node has 8 children or only leaves remain.  An inner binary node whose
// subtree holds at most kWideLeafTris triangles is not opened but becomes one
// leaf with all of them: the cooperative traversal tests a leaf's triangles
// 8 at a time (one triangle per lane), so a leaf of 8 costs one round -- one
// dependent load -- where the binary SAH's leaves of ~2 (its cost counts
// pairs) cost a node level each.  Leaves are re-laid as single TriIsect
// records (<= 16 per leaf).  IPT_WIDE_LEAF_TRIS (a build-time define, make
// variant) sets the bound; 0 keeps the binary leaves.  North-star scene: 81 wide
// nodes of depth 4 -> 73 of depth 3, 214 leaves of 6 triangles on average;
// forward 3.843 -> 3.782 ms, adjoint 4.698 -> 4.623 (bound 16: 4.23 / 5.02,
// the leaves' boxes grow; profiles/r04/envab_wideleaf_r04n.log).
#ifndef IPT_WIDE_LEAF_TRIS
#define IPT_WIDE_LEAF_TRIS 8
#endif
static bool build_wide(HostScene *S) {
  const int fat = std::min(16, std::max(0, (int)IPT_WIDE_LEAF_TRIS));
  // triangles of a binary child code (leaf: its pairs' real triangles)
  std::vector<int> tris_of_node(S->bvh_nodes.size(), -1);
  std::function<int(int)> count = [&](int code) -> int {
    if (code < 0) {
      const int c = ~code, first = c >> kBvhLeafPairBits, np = (c & ((1 << kBvhLeafPairBits) - 1)) + 1;
      int n = 0;
      for (int j = first; j < first + np; ++j)
        for (int hh = 0; hh < 2; ++hh) n += S->bvh_pairs[(size_t)j].idx[hh] != 0x7fffffff;
      return n;
    }
    int &m = tris_of_node[(size_t)code];
    if (m < 0) {
      int kid[2];
      std::memcpy(kid, &S->bvh_nodes[(size_t)code].q[3][0], sizeof kid);
      m = count(kid[0]) + count(kid[1]);
    }
    return m;
  };
  std::function<void(int, std::vector<int> &)> gather = [&](int code, std::vector<int> &out) {
    if (code < 0) {
      const int c = ~code, first = c >> kBvhLeafPairBits, np = (c & ((1 << kBvhLeafPairBits) - 1)) + 1;
      for (int j = first; j < first + np; ++j)
        for (int hh = 0; hh < 2; ++hh)
          if (S->bvh_pairs[(size_t)j].idx[hh] != 0x7fffffff) out.push_back(S->bvh_pairs[(size_t)j].idx[hh]);
      return;
    }
    int kid[2];
    std::memcpy(kid, &S->bvh_nodes[(size_t)code].q[3][0], sizeof kid);
    gather(kid[0], out);
    gather(kid[1], out);
  };
  auto openable = [&](int code) { return code >= 0 && count(code) > fat; };
  struct Child {
    float lo[3], hi[3];
    int code;  // binary child code
  };
  auto child_of = [&](int n, int c) {
    const BvhNode &N = S->bvh_nodes[(size_t)n];
    Child ch;
    const float *q = &N.q[0][0];
    for (int a = 0; a < 3; ++a) {
      ch.lo[a] = q[6 * c + 2 * a];
      ch.hi[a] = q[6 * c + 2 * a + 1];
    }
    int kid[2];
    std::memcpy(kid, &N.q[3][0], sizeof kid);
    ch.code = kid[c];
    return ch;
  };
  auto area = [](const Child &c) {
    const double dx = (double)c.hi[0] - c.lo[0], dy = (double)c.hi[1] - c.lo[1], dz = (double)c.hi[2] - c.lo[2];
    return dx * dy + dy * dz + dz * dx;
  };
  S->bvh_wide.clear();
  S->bvh_wtris.clear();
  S->bvh_wdepth = 0;
  // root box
  {
    const Child c0 = child_of(0, 0), c1 = child_of(0, 1);
    for (int a = 0; a < 3; ++a) {
      S->bvh_root_box[a] = std::min(c0.lo[a], c1.lo[a]);
      S->bvh_root_box[3 + a] = std::max(c0.hi[a], c1.hi[a]);
    }
  }
  // breadth-first over wide nodes, each given by its binary node
  std::vector<std::pair<int, int>> queue;  // (binary node, wide depth)
  queue.push_back({0, 1});
  for (size_t h = 0; h < queue.size(); ++h) {
    const int bn = queue[h].first, depth = queue[h].second;
    S->bvh_wdepth = std::max(S->bvh_wdepth, depth);
    std::vector<Child> kids = {child_of(bn, 0), child_of(bn, 1)};
    while (kids.size() < 8) {
      int best = -1;
      for (size_t k = 0; k < kids.size(); ++k)
        if (openable(kids[k].code) && (best < 0 || area(kids[k]) > area(kids[(size_t)best]))) best = (int)k;
      if (best < 0) break;
      const int n = kids[(size_t)best].code;
      kids[(size_t)best] = child_of(n, 0);
      kids.push_back(child_of(n, 1));
    }
    WideNode W;
    std::memset(&W, 0, sizeof W);
    for (int k = 0; k < 8; ++k) {
      float *sl = W.s[k];
      int32_t ref = kWideEmpty;
      if (k < (int)kids.size()) {
        const Child &c = kids[(size_t)k];
        for (int a = 0; a < 3; ++a) {
          sl[a] = c.lo[a];
          sl[3 + a] = c.hi[a];
        }
        if (openable(c.code)) {
          ref = (int32_t)queue.size();  // wide node h is queue[h]: a child's index is its queue position
          queue.push_back({c.code, depth + 1});
        } else {  // a binary leaf, or a subtree of <= fat triangles: one leaf
          std::vector<int> ts;
          gather(c.code, ts);
          const int tfirst = (int)S->bvh_wtris.size();
          for (const int t : ts) {
            TriIsect T = S->isect[(size_t)t];
            std::memcpy(&T.pad[0], &t, sizeof t);
            S->bvh_wtris.push_back(T);
          }
          const int cnt = (int)S->bvh_wtris.size() - tfirst;
          if (cnt < 1 || cnt > 16 || tfirst >= (1 << 26)) {
            S->bvh_status = "leaf too large for the cooperative traversal";
            return false;
          }
          ref = ~((tfirst << 4) | (cnt - 1));
        }
      } else {
        for (int a = 0; a < 3; ++a) {  // empty slot: never hit
          sl[a] = 1.f;
          sl[3 + a] = -1.f;
        }
      }
      std::memcpy(&sl[6], &ref, sizeof ref);
    }
    // Front-to-back child order per ray-direction octant o (bit a set: d_a <
    // 0), kept in slot o's pad word as each child's RANK, 3 bits per child
    // (bits 3k: the rank of child k): rank by the centre's coordinate sum
    // signed by the octant, empty slots last.  Lane k of a traversal group
    // reads child k and this word at once (coop_cast); only the visit order
    // depends on it.
    for (int o = 0; o < 8; ++o) {
      int order[8];
      double key[8];
      for (int k = 0; k < 8; ++k) {
        order[k] = k;
        key[k] = k < (int)kids.size() ? 0.0 : HUGE_VAL;
        if (k < (int)kids.size())
          for (int a = 0; a < 3; ++a)
            key[k] += ((o >> a) & 1 ? -0.5 : 0.5) * ((double)kids[(size_t)k].lo[a] + kids[(size_t)k].hi[a]);
      }
      std::stable_sort(order, order + 8, [&](int x, int y) { return key[x] < key[y]; });
      uint32_t rank = 0;
      for (int r = 0; r < 8; ++r) rank |= (uint32_t)r << (3 * order[r]);
      std::memcpy(&W.s[o][7], &rank, sizeof rank);
    }
    S->bvh_wide.push_back(W);
  }
  return true;
}

// Two exact, conservative entry tests for the tree (ipt_device.h
// coop_root_test, tree_skip), computed from the acceptance regions A_w of the
// tree's triangles (the prisms acceptance_box bounds; convex, their six
// vertices below):
//  * bounding sphere: centre = the root box's centre (a float), radius = the
//    largest distance from it to a vertex of some A_w, padded by 2^-10 R --
//    over 100x the fp32 error of the kernel's ray-sphere test (|p|, |c| <= R,
//    squared terms <= 4R^2 with a few roundings of 2^-24 each).  A ray whose
//    origin is outside the padded sphere and whose line misses it accepts no
//    tree triangle.
//  * source plane: a ray leaving a point p that triangle s's test accepted
//    (|n_s.(p - c_s)| <= h, the acceptance slab) reaches, at any t >= 1e-2
//    (the test rejects smaller t), points with n_s.(x - c_s) >=
//    -h + 1e-2 (n_s.d); the computed hit point of a tree triangle w lies
//    within 2^-23 R of the exact ray point, and inside A_w, where n_s.(x -
//    c_s) <= M_s = the largest value over all A_w's vertices.  So when
//    1e-2 (n_s.d) > M_s + h + 2^-23 R, no tree triangle can accept the ray:
//    tau_s = (M_s + h + 2^-23 R) / 1e-2 + 2e-6 (the fp32 dot's error), and
//    at least 4e-6 (the bound needs n_s.d >= 0); the kernel skips the tree
//    when dot(n_s, d) >= tau_s.  Every tree triangle
//    behind s's plane -- a convex mesh's own faces seen from any of them, or
//    an object behind a wall -- gives tau_s < 1; otherwise tau_s = +inf.
//    (North-star scene: every path and shadow ray leaving the sphere.)
static void tree_cull(HostScene *S, const std::vector<Prim> &tree, double r_all) {
  const float inf = std::numeric_limits<float>::infinity();
  std::vector<double> vx;  // the tree triangles' region vertices, xyz
  vx.reserve(tree.size() * 18);
  for (const Prim &p : tree) {
    float l[3], u[3];
    double v[6][3];
    if (acceptance_box(S->isect[(size_t)p.tri], S->geom[(size_t)p.tri], r_all, l, u, v) != 0) continue;
    for (int k = 0; k < 6; ++k)
      for (int a = 0; a < 3; ++a) vx.push_back(v[k][a]);
  }
  const size_t nv = vx.size() / 3;
  float c[3];
  for (int a = 0; a < 3; ++a) c[a] = 0.5f * S->bvh_root_box[a] + 0.5f * S->bvh_root_box[3 + a];
  double rho2 = 0.0;
  for (size_t k = 0; k < nv; ++k) {
    double d2 = 0.0;
    for (int a = 0; a < 3; ++a) d2 += (vx[3 * k + a] - c[a]) * (vx[3 * k + a] - c[a]);
    rho2 = std::max(rho2, d2);
  }
  const double rho = std::sqrt(rho2) + std::ldexp(r_all, -10);
  for (int a = 0; a < 3; ++a) S->bvh_sphere[a] = c[a];
  S->bvh_sphere[3] = round_up(rho * rho * (1.0 + 1e-12));
  const double h = std::ldexp(3.0 * r_all, -17);
  S->bvh_src_cull.assign((size_t)S->nT * 4, 0.f);
  for (int si = 0; si < S->nT; ++si) {
    const TriIsect &T = S->isect[(size_t)si];
    const double n[3] = {T.n[0], T.n[1], T.n[2]};
    double m = -HUGE_VAL;
    bool finite = true;
    for (int a = 0; a < 3; ++a) finite = finite && std::isfinite(n[a]) && std::isfinite(T.c[a]);
    for (size_t k = 0; k < nv && finite; ++k)
      m = std::max(m, n[0] * (vx[3 * k] - T.c[0]) + n[1] * (vx[3 * k + 1] - T.c[1]) + n[2] * (vx[3 * k + 2] - T.c[2]));
    // (the bound used t (n_s.d) >= 1e-2 (n_s.d), i.e. n_s.d >= 0: tau is at
    // least 4e-6 even when the whole tree lies far behind s's plane -- a ray
    // leaving s backwards may well reach it)
    const double tau = std::max((m + h + std::ldexp(r_all, -23) + 1e-9 * r_all) / 1e-2 + 2e-6, 4e-6);
    for (int a = 0; a < 3; ++a) S->bvh_src_cull[(size_t)si * 4 + a] = T.n[a];
    S->bvh_src_cull[(size_t)si * 4 + 3] = (finite && nv > 0 && tau < 0.999) ? round_up(tau) : inf;
  }
}

bool build_bvh(HostScene *S) {
  S->bvh_nodes.clear();
  S->bvh_pairs.clear();
  S->bvh_big_pairs.clear();
  S->bvh_big_idx.clear();
  S->bvh_big_boxes.clear();
  S->bvh_depth = 0;
  const double r_all = scene_coord_bound(*S);
  Builder B;
  for (int i = 0; i < S->nT; ++i) {
    Prim p;
    const int rc = acceptance_box(S->isect[(size_t)i], S->geom[(size_t)i], r_all, p.box.lo, p.box.hi);
    if (rc < 0) {
      S->bvh_status = "triangle " + std::to_string(i) + " has no bounded acceptance region";
      return false;
    }
    if (rc == 1) continue;  // never accepted: left out of the tree
    for (int a = 0; a < 3; ++a) p.c[a] = 0.5f * p.box.lo[a] + 0.5f * p.box.hi[a];
    p.tri = i;
    B.prims.push_back(p);
  }
  // the large triangles go to the brute-force pre-pass
  {
    Box all;
    for (const Prim &p : B.prims) all.grow(p.box);
    const double lim = kBigFrac * all.area();
    std::vector<size_t> cand;
    for (size_t k = 0; k < B.prims.size(); ++k)
      if (B.prims[k].box.area() >= lim) cand.push_back(k);
    std::stable_sort(cand.begin(), cand.end(),
                     [&](size_t x, size_t y) { return B.prims[x].box.area() > B.prims[y].box.area(); });
    if (cand.size() > (size_t)(2 * kBigPairs)) cand.resize(2 * kBigPairs);
    std::vector<int> big;
    std::vector<char> drop(B.prims.size(), 0);
    for (size_t k : cand) {
      big.push_back(B.prims[k].tri);
      drop[k] = 1;
    }
    std::sort(big.begin(), big.end());
    std::vector<Prim> rest;
    for (size_t k = 0; k < B.prims.size(); ++k)
      if (!drop[k]) rest.push_back(B.prims[k]);
    B.prims.swap(rest);
    const int np = ((int)big.size() + 1) / 2;
    S->bvh_big_pairs.assign((size_t)np, TriPair());
    S->bvh_big_idx.assign((size_t)np * 2, 0x7fffffff);
    std::vector<TriIsect> recs((size_t)np * 2);
    for (auto &r : recs) std::memset(&r, 0, sizeof r);
    for (size_t k = 0; k < big.size(); ++k) {
      recs[k] = S->isect[(size_t)big[k]];
      S->bvh_big_idx[k] = big[k];
    }
    if (np > 0) pack_pairs(recs.data(), 2 * np, S->bvh_big_pairs.data());
    // acceptance boxes of the big pairs, two pairs per record (as pair_boxes)
    const float inf = std::numeric_limits<float>::infinity();
    S->bvh_big_boxes.assign((size_t)(np + 1) / 2, PairBox2());
    for (int j = 0; j < np; ++j) {
      float lo[3] = {inf, inf, inf}, hi[3] = {-inf, -inf, -inf};
      bool any = false;
      for (int h = 0; h < 2; ++h) {
        const size_t k = (size_t)(2 * j + h);
        if (k >= big.size()) continue;
        float l[3], u[3];
        if (acceptance_box(S->isect[(size_t)big[k]], S->geom[(size_t)big[k]], r_all, l, u) != 0) continue;
        any = true;
        for (int a = 0; a < 3; ++a) {
          lo[a] = std::min(lo[a], l[a]);
          hi[a] = std::max(hi[a], u[a]);
        }
      }
      for (int a = 0; a < 3; ++a) {
        S->bvh_big_boxes[(size_t)j / 2].f[2 * a][j & 1] = any ? lo[a] : inf;
        S->bvh_big_boxes[(size_t)j / 2].f[2 * a + 1][j & 1] = any ? hi[a] : inf;
      }
    }
    if (np & 1)
      for (int k = 0; k < 6; ++k) S->bvh_big_boxes.back().f[k][1] = inf;
  }
  if (B.prims.size() < 2) {
    S->bvh_status = "fewer than two hittable triangles outside the brute-force set";
    S->bvh_big_pairs.clear();
    S->bvh_big_idx.clear();
    S->bvh_big_boxes.clear();
    return false;
  }
  Box root_box;
  B.build(0, (int)B.prims.size(), 0, true, &root_box);
  if (B.too_deep || B.nodes.size() >= 65535) {
    S->bvh_status = "tree too deep or too large for the u16 traversal stack";
    return false;
  }
  // leaves -> pairs (depth-first leaf order)
  std::vector<int> leaf_code(B.leaves.size());
  for (size_t l = 0; l < B.leaves.size(); ++l) {
    const int b = B.leaves[l].first, e = B.leaves[l].second;
    const int first = (int)S->bvh_pairs.size();
    const int np = (e - b + 1) / 2;
    if (first >= (1 << (31 - kBvhLeafPairBits))) {
      S->bvh_status = "too many triangles for the leaf encoding";
      S->bvh_pairs.clear();
      return false;
    }
    for (int j = 0; j < np; ++j) {
      BvhPair P;
      std::memset(&P, 0, sizeof P);
      for (int h = 0; h < 2; ++h) {
        const int k = b + 2 * j + h;
        if (k < e) {
          const int t = B.prims[(size_t)k].tri;
          put_tri(&P, h, &S->isect[(size_t)t], t);
        } else {
          put_tri(&P, h, nullptr, 0x7fffffff);
        }
      }
      S->bvh_pairs.push_back(P);
    }
    leaf_code[l] = ~((first << kBvhLeafPairBits) | (np - 1));
  }
  // inner nodes -> breadth-first order
  std::vector<int> order, newid(B.nodes.size(), -1);
  order.push_back(0);
  newid[0] = 0;
  for (size_t h = 0; h < order.size(); ++h) {
    const TNode &t = B.nodes[(size_t)order[h]];
    for (int c = 0; c < 2; ++c)
      if (t.kid[c] >= 0) {
        newid[(size_t)t.kid[c]] = (int)order.size();
        order.push_back(t.kid[c]);
      }
  }
  S->bvh_nodes.resize(order.size());
  for (size_t h = 0; h < order.size(); ++h) {
    const TNode &t = B.nodes[(size_t)order[h]];
    BvhNode &N = S->bvh_nodes[h];
    std::memset(&N, 0, sizeof N);
    const Box &b0 = t.box[0], &b1 = t.box[1];
    const float q[12] = {b0.lo[0], b0.hi[0], b0.lo[1], b0.hi[1], b0.lo[2], b0.hi[2],
                         b1.lo[0], b1.hi[0], b1.lo[1], b1.hi[1], b1.lo[2], b1.hi[2]};
    std::memcpy(&N.q[0][0], q, sizeof q);
    int kid[2];
    for (int c = 0; c < 2; ++c) kid[c] = t.kid[c] >= 0 ? newid[(size_t)t.kid[c]] : leaf_code[(size_t)(~t.kid[c])];
    std::memcpy(&N.q[3][0], kid, sizeof kid);
  }
  S->bvh_depth = B.max_depth;
  if (!build_wide(S)) S->bvh_wide.clear();  // (build_wide sets bvh_status)
  if (S->bvh_wide.empty()) {
    S->bvh_nodes.clear();
    S->bvh_pairs.clear();
    S->bvh_big_pairs.clear();
    S->bvh_big_idx.clear();
    S->bvh_big_boxes.clear();
    return false;
  }
  tree_cull(S, B.prims, r_all);
  S->bvh_status = "ok";
  return true;
}

}  // namespace ipt
