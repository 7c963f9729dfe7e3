// scene_io.cpp -- host scene ingest for the MI355X path tracer.
//
// Restates, for the OBJ/MTL subset the reference's assets exercise, the
// semantics of the reference's vendored tinyobjloader and its Mesh /
// Triangle / Scene construction:
//   number parsing        utils.h:70-239 (tryParseDouble / parseReal)
//   face indices          utils.h:287-362 (fixIndex / parseTriple)
//   lines                 utils.h:412-444 (safeGetline: \n, \r, \r\n)
//   LoadObj               tiny_obj_loader.h:585-933
//   triangulation         tiny_obj_loader.h:179-583 (quad split on the
//                         shorter diagonal, ear clipping otherwise)
//   LoadMtl               material.h:383-772 (Kd, Ks, Ke, Ns; first name wins)
//   ParseFromString       scene_basics.h:207-289 (scene-supplied MTL stream,
//                         inline "*Kd r g b*", per-vertex normals only when
//                         #vn == #v)
//   Mesh transform        scene_basics.h:147-157 (T = translate*rotate*scale)
//   Triangle              scene_basics.h:74-96
//   Scene / setOffsets    scene.h:89-117, scene_basics.h:467-474
//   Camera                scene.h:15-84
// and hoists the per-ray-test constants of Object::signedDistance
// (scene_basics.h:497-503) and the sampling frame of sampleNextDir
// (path_trace.cu:98-103) into the flattened per-triangle records.
//
// Host arithmetic is unfused fp32 in Eigen's expression order (compiled with
// -ffp-contract=off); DESIGN.md §3.
#include "scene_io.h"

#include "bvh.h"

#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>

namespace ipt {
namespace {

inline bool is_space(char c) { return c == ' ' || c == '\t'; }
inline bool is_digit(char c) { return static_cast<unsigned>(c - '0') < 10u; }
inline bool is_eol(char c) { return c == '\r' || c == '\n' || c == '\0'; }

// ---------------------------------------------------------------- numbers
// Decimal parser with tinyobj's exact accumulation order (utils.h:70-200):
// mantissa digits accumulate in double, fractional digit k adds d*10^-k
// (table for k<8, pow otherwise), exponent applied as ldexp(m*5^e, e).
bool parse_decimal(const char *s, const char *end, double *out) {
  if (s >= end) return false;
  static const double kPow10[8] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
  const char *p = s;
  bool negative = false, frac_only = false;
  if (*p == '+' || *p == '-') {
    negative = (*p == '-');
    ++p;
    frac_only = (p != end && *p == '.');
  } else if (*p == '.') {
    frac_only = true;
  } else if (!is_digit(*p)) {
    return false;
  }
  double m = 0.0;
  int ndig = 0;
  if (!frac_only) {
    while (p != end && is_digit(*p)) {
      m *= 10;
      m += static_cast<int>(*p - '0');
      ++p;
      ++ndig;
    }
    if (ndig == 0) return false;
  }
  int e = 0;
  if (p != end) {
    bool exp_next = false;
    if (*p == '.') {
      ++p;
      int k = 1;
      while (p != end && is_digit(*p)) {
        m += static_cast<int>(*p - '0') * (k < 8 ? kPow10[k] : std::pow(10.0, -k));
        ++k;
        ++p;
      }
      exp_next = (p != end);
    } else if (*p == 'e' || *p == 'E') {
      exp_next = true;
    }
    if (exp_next && (*p == 'e' || *p == 'E')) {
      ++p;
      bool eneg = false;
      if (p != end && (*p == '+' || *p == '-')) {
        eneg = (*p == '-');
        ++p;
      } else if (!is_digit(*p)) {
        return false;
      }
      int nd = 0;
      while (p != end && is_digit(*p)) {
        if (e > 2147483647 / 10) return false;
        e = e * 10 + static_cast<int>(*p - '0');
        ++p;
        ++nd;
      }
      if (nd == 0) return false;
      if (eneg) e = -e;
    }
  }
  double mag = e ? std::ldexp(m * std::pow(5.0, e), e) : m;
  *out = (negative ? -1 : 1) * mag;
  return true;
}

struct Cursor {
  const char *p;
  void skip_ws() { p += std::strspn(p, " \t"); }
  float real(double dflt = 0.0) {
    skip_ws();
    const char *end = p + std::strcspn(p, " \t\r");
    double v = dflt;
    parse_decimal(p, end, &v);
    p = end;
    return static_cast<float>(v);
  }
  std::string word() {
    skip_ws();
    size_t n = std::strcspn(p, " \t\r");
    std::string s(p, n);
    p += n;
    return s;
  }
};

// ---------------------------------------------------------------- lines
class Lines {
 public:
  explicit Lines(std::string text) : buf_(std::move(text)), pos_(0) {}
  bool next(std::string *line) {
    if (pos_ >= buf_.size()) return false;
    size_t s = pos_;
    while (pos_ < buf_.size() && buf_[pos_] != '\n' && buf_[pos_] != '\r') ++pos_;
    line->assign(buf_, s, pos_ - s);
    if (pos_ < buf_.size()) {
      if (buf_[pos_] == '\r' && pos_ + 1 < buf_.size() && buf_[pos_ + 1] == '\n') pos_ += 2;
      else pos_ += 1;
    }
    return true;
  }

 private:
  std::string buf_;
  size_t pos_;
};

bool slurp(const std::string &path, std::string *out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::ostringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return true;
}

// ---------------------------------------------------------------- materials
struct Material {
  float kd[3] = {0.f, 0.f, 0.f};
  float ks[3] = {0.f, 0.f, 0.f};
  float ke[3] = {0.f, 0.f, 0.f};
  float shininess = 1.f;  // InitMaterial, material.h:317-367
};

class MtlLibrary {
 public:
  std::vector<Material> materials;
  int find(const std::string &name) const {
    auto it = index_.find(name);
    return it == index_.end() ? -1 : it->second;
  }
  void add(const std::string &name, const Material &m) {
    index_.emplace(name, static_cast<int>(materials.size()));  // first wins
    materials.push_back(m);
  }
  // LoadMtl, material.h:383-772 (only the fields the integrators read).
  void load(const std::string &text) {
    Lines lines(text);
    std::string line, name;
    Material cur;
    while (lines.next(&line)) {
      size_t last = line.find_last_not_of(" \t");
      line.resize(last == std::string::npos ? 0 : last + 1);
      if (!line.empty() && line.back() == '\n') line.pop_back();
      if (!line.empty() && line.back() == '\r') line.pop_back();
      if (line.empty()) continue;
      Cursor c{line.c_str()};
      c.skip_ws();
      const char *t = c.p;
      if (t[0] == '\0' || t[0] == '#') continue;
      if (std::strncmp(t, "newmtl", 6) == 0 && is_space(t[6])) {
        if (!name.empty()) add(name, cur);
        cur = Material();
        name.assign(t + 7);
        continue;
      }
      if (t[0] == 'K' && is_space(t[2]) && (t[1] == 'd' || t[1] == 's' || t[1] == 'e')) {
        float *dst = t[1] == 'd' ? cur.kd : (t[1] == 's' ? cur.ks : cur.ke);
        c.p = t + 2;
        for (int i = 0; i < 3; ++i) dst[i] = c.real();
        continue;
      }
      if (t[0] == 'N' && t[1] == 's' && is_space(t[2])) {
        c.p = t + 2;
        cur.shininess = c.real();
        continue;
      }
    }
    add(name, cur);  // flush last (even unnamed)
  }

 private:
  std::map<std::string, int> index_;
};

// ---------------------------------------------------------------- OBJ
struct Corner { int v, vt, vn; };

struct ObjMesh {
  std::vector<float> v, vn;
  int nvt = 0;
  std::vector<int> tri;      // 3 vertex indices per triangle, export order
  std::vector<int> tri_mat;  // material id per triangle (-1 = default)
};

bool to_index(int raw, int n, int *out) {  // fixIndex, utils.h:287-307
  if (raw > 0) { *out = raw - 1; return true; }
  if (raw == 0) return false;
  *out = n + raw;
  return true;
}

bool read_corner(const char **tok, const ObjMesh &m, Corner *out) {  // parseTriple
  Corner c{-1, -1, -1};
  const char *&p = *tok;
  const int nv = static_cast<int>(m.v.size() / 3), nn = static_cast<int>(m.vn.size() / 3);
  if (!to_index(std::atoi(p), nv, &c.v)) return false;
  p += std::strcspn(p, "/ \t\r");
  if (p[0] == '/') {
    ++p;
    if (p[0] == '/') {
      ++p;
      if (!to_index(std::atoi(p), nn, &c.vn)) return false;
      p += std::strcspn(p, "/ \t\r");
    } else {
      if (!to_index(std::atoi(p), m.nvt, &c.vt)) return false;
      p += std::strcspn(p, "/ \t\r");
      if (p[0] == '/') {
        ++p;
        if (!to_index(std::atoi(p), nn, &c.vn)) return false;
        p += std::strcspn(p, "/ \t\r");
      }
    }
  }
  *out = c;
  return true;
}

bool point_in_tri(const float *x, const float *y, float tx, float ty) {  // pnpoly
  bool in = false;
  for (int i = 0, j = 2; i < 3; j = i++) {
    if (((y[i] > ty) != (y[j] > ty)) && (tx < (x[j] - x[i]) * (ty - y[i]) / (y[j] - y[i]) + x[i]))
      in = !in;
  }
  return in;
}

// exportGroupsToShape with triangulate=true (tiny_obj_loader.h:179-583)
void triangulate(ObjMesh &m, const std::vector<std::vector<Corner>> &faces, int mat) {
  const std::vector<float> &v = m.v;
  const size_t vsize = v.size();
  auto emit = [&](const Corner &a, const Corner &b, const Corner &c) {
    m.tri.push_back(a.v);
    m.tri.push_back(b.v);
    m.tri.push_back(c.v);
    m.tri_mat.push_back(mat);
  };
  for (const auto &f : faces) {
    const size_t n = f.size();
    if (n < 3) continue;
    if (n == 4) {
      size_t i[4];
      for (int k = 0; k < 4; ++k) i[k] = static_cast<size_t>(f[k].v);
      bool bad = false;
      for (int k = 0; k < 4; ++k) bad |= (3 * i[k] + 2 >= vsize);
      if (bad) continue;
      float d02[3], d13[3];
      for (int a = 0; a < 3; ++a) {
        d02[a] = v[i[2] * 3 + a] - v[i[0] * 3 + a];
        d13[a] = v[i[3] * 3 + a] - v[i[1] * 3 + a];
      }
      float q02 = d02[0] * d02[0] + d02[1] * d02[1] + d02[2] * d02[2];
      float q13 = d13[0] * d13[0] + d13[1] * d13[1] + d13[2] * d13[2];
      if (q02 < q13) {
        emit(f[0], f[1], f[2]);
        emit(f[0], f[2], f[3]);
      } else {
        emit(f[0], f[1], f[3]);
        emit(f[1], f[2], f[3]);
      }
      continue;
    }
    // projection axes from the first non-degenerate corner
    size_t ax0 = 1, ax1 = 2;
    for (size_t k = 0; k < n; ++k) {
      size_t a = f[k % n].v, b = f[(k + 1) % n].v, c = f[(k + 2) % n].v;
      if (3 * a + 2 >= vsize || 3 * b + 2 >= vsize || 3 * c + 2 >= vsize) continue;
      float e0[3], e1[3];
      for (int t = 0; t < 3; ++t) {
        e0[t] = v[b * 3 + t] - v[a * 3 + t];
        e1[t] = v[c * 3 + t] - v[b * 3 + t];
      }
      float cx = std::fabs(e0[1] * e1[2] - e0[2] * e1[1]);
      float cy = std::fabs(e0[2] * e1[0] - e0[0] * e1[2]);
      float cz = std::fabs(e0[0] * e1[1] - e0[1] * e1[0]);
      if (cx > FLT_EPSILON || cy > FLT_EPSILON || cz > FLT_EPSILON) {
        if (!(cx > cy && cx > cz)) {
          ax0 = 0;
          if (cz > cx && cz > cy) ax1 = 1;
        }
        break;
      }
    }
    std::vector<Corner> poly(f);
    size_t guess = 0, budget = n, last_n = n;
    Corner ear[3];
    float ex[3], ey[3];
    while (poly.size() > 3 && budget > 0) {
      const size_t np = poly.size();
      if (guess >= np) guess -= np;
      if (last_n != np) {
        last_n = np;
        budget = np;
      } else {
        --budget;
      }
      for (size_t k = 0; k < 3; ++k) {
        ear[k] = poly[(guess + k) % np];
        size_t vi = static_cast<size_t>(ear[k].v);
        bool oob = (vi * 3 + ax0) >= vsize || (vi * 3 + ax1) >= vsize;
        ex[k] = oob ? 0.f : v[vi * 3 + ax0];
        ey[k] = oob ? 0.f : v[vi * 3 + ax1];
      }
      float cr = (ex[1] - ex[0]) * (ey[2] - ey[1]) - (ey[1] - ey[0]) * (ex[2] - ex[1]);
      float ar = (ex[0] * ey[1] - ey[0] * ex[1]) * 0.5f;
      if (cr * ar < 0.f) {
        ++guess;
        continue;
      }
      bool blocked = false;
      for (size_t o = 3; o < np && !blocked; ++o) {
        size_t idx = (guess + o) % np;
        if (idx >= poly.size()) continue;
        size_t ov = static_cast<size_t>(poly[idx].v);
        if ((ov * 3 + ax0) >= vsize || (ov * 3 + ax1) >= vsize) continue;
        blocked = point_in_tri(ex, ey, v[ov * 3 + ax0], v[ov * 3 + ax1]);
      }
      if (blocked) {
        ++guess;
        continue;
      }
      emit(ear[0], ear[1], ear[2]);
      poly.erase(poly.begin() + static_cast<long>((guess + 1) % np));
    }
    if (poly.size() == 3) emit(poly[0], poly[1], poly[2]);
  }
}

// LoadObj (tiny_obj_loader.h:585-933).  `mtl_text` is the scene-supplied
// material stream (nullptr = stream not readable).
bool load_obj(const std::string &text, const std::string *mtl_text, ObjMesh *m, MtlLibrary *lib,
              std::string *err) {
  Lines lines(text);
  std::string line;
  std::vector<std::vector<Corner>> pending;
  int material = -1;
  bool mtl_read = false;
  auto flush = [&]() {
    triangulate(*m, pending, material);
    pending.clear();
  };
  while (lines.next(&line)) {
    if (!line.empty() && line.back() == '\n') line.pop_back();
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line.empty()) continue;
    Cursor c{line.c_str()};
    c.skip_ws();
    const char *t = c.p;
    if (t[0] == '\0' || t[0] == '#') continue;
    if (t[0] == 'v' && is_space(t[1])) {
      c.p = t + 2;
      for (int i = 0; i < 3; ++i) m->v.push_back(c.real());
    } else if (t[0] == 'v' && t[1] == 'n' && is_space(t[2])) {
      c.p = t + 3;
      for (int i = 0; i < 3; ++i) m->vn.push_back(c.real());
    } else if (t[0] == 'v' && t[1] == 't' && is_space(t[2])) {
      m->nvt++;
    } else if (t[0] == 'f' && is_space(t[1])) {
      const char *p = t + 2;
      p += std::strspn(p, " \t");
      std::vector<Corner> face;
      while (!is_eol(p[0])) {
        Corner cn;
        if (!read_corner(&p, *m, &cn)) {
          *err = "failed to parse `f' line (zero face index)";
          return false;
        }
        face.push_back(cn);
        p += std::strspn(p, " \t\r");
      }
      pending.push_back(std::move(face));
    } else if (std::strncmp(t, "usemtl", 6) == 0) {
      c.p = t + 6;
      int id = lib->find(c.word());
      if (id != material) {
        flush();
        material = id;
      }
    } else if (std::strncmp(t, "mtllib", 6) == 0 && is_space(t[6])) {
      if (mtl_text && !mtl_read) lib->load(*mtl_text);
      mtl_read = true;
    } else if ((t[0] == 'g' || t[0] == 'o') && is_space(t[1])) {
      flush();
    }
  }
  flush();
  return true;
}

// ---------------------------------------------------------------- geometry
struct V3 { float x, y, z; };
inline V3 v3sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 v3add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline float hdot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
inline V3 hcross(V3 a, V3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline V3 hunit(V3 v) {
  float n2 = hdot(v, v);
  if (n2 > 0.f) {
    float s = std::sqrt(n2);
    v = {v.x / s, v.y / s, v.z / s};
  }
  return v;
}

// Quaternion::setFromTwoVectors((0,0,1), n).toRotationMatrix(), with the
// reference's exact -I shortcut (path_trace.cu:99-103).
void sampling_frame(V3 n, float R[3][3]) {
  if (n.z == -1.f) {
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) R[i][j] = i == j ? -1.f : 0.f;
    return;
  }
  const V3 z{0.f, 0.f, 1.f};
  V3 u = hunit(n);
  float c = hdot(u, z);
  float qx, qy, qz, qw;
  if (c < -1.f + 1e-5f) {  // Eigen's SVD branch; DESIGN.md §3.4
    c = c > -1.f ? c : -1.f;
    V3 ax = hcross(z, u);
    ax = hdot(ax, ax) > 0.f ? hunit(ax) : V3{1.f, 0.f, 0.f};
    float w2 = (1.f + c) * 0.5f;
    qw = std::sqrt(w2);
    float sv = std::sqrt(1.f - w2);
    qx = ax.x * sv;
    qy = ax.y * sv;
    qz = ax.z * sv;
  } else {
    V3 ax = hcross(z, u);
    float s = std::sqrt((1.f + c) * 2.f);
    float is = 1.f / s;
    qx = ax.x * is;
    qy = ax.y * is;
    qz = ax.z * is;
    qw = s * 0.5f;
  }
  float tx = 2.f * qx, ty = 2.f * qy, tz = 2.f * qz;
  float twx = tx * qw, twy = ty * qw, twz = tz * qw;
  float txx = tx * qx, txy = ty * qx, txz = tz * qx;
  float tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
  R[0][0] = 1.f - (tyy + tzz);
  R[0][1] = txy - twz;
  R[0][2] = txz + twy;
  R[1][0] = txy + twz;
  R[1][1] = 1.f - (txx + tzz);
  R[1][2] = tyz - twx;
  R[2][0] = txz - twy;
  R[2][1] = tyz + twx;
  R[2][2] = 1.f - (txx + tyy);
}

struct Tri {
  V3 v[3], vn[3], n, c;
  float area;
  Material m;
};

Tri make_tri(V3 a, V3 b, V3 c, const V3 *ns, const Material &m) {  // Triangle::Triangle
  Tri t;
  t.v[0] = a;
  t.v[1] = b;
  t.v[2] = c;
  V3 ctr{0.f, 0.f, 0.f};
  for (int j = 0; j < 3; ++j) {
    ctr.x = ctr.x + t.v[j].x / 3.f;
    ctr.y = ctr.y + t.v[j].y / 3.f;
    ctr.z = ctr.z + t.v[j].z / 3.f;
  }
  t.c = ctr;
  V3 nrm = hcross(v3sub(t.v[1], t.v[0]), v3sub(t.v[2], t.v[1]));
  t.area = std::sqrt(hdot(nrm, nrm)) / 2.f;
  t.n = hunit(nrm);
  for (int j = 0; j < 3; ++j) t.vn[j] = ns ? ns[j] : t.n;
  t.m = m;
  return t;
}

// GEOM_AXIS_FLAT (scene_layout.h): equal axis-aligned vertex normals on a
// triangle of positive finite area
bool axis_flat(const Tri &t) {
  if (!(t.area > 0.f) || !std::isfinite(t.area)) return false;
  for (int j = 1; j < 3; ++j)
    if (std::memcmp(&t.vn[j], &t.vn[0], sizeof(V3)) != 0) return false;
  const float c[3] = {t.vn[0].x, t.vn[0].y, t.vn[0].z};
  int zeros = 0, ones = 0;
  for (float x : c) {
    zeros += (x == 0.f);
    ones += (x == 1.f || x == -1.f);
  }
  return zeros == 2 && ones == 1;
}

// Mesh::Mesh + ParseFromString (scene_basics.h:147-289)
bool load_mesh(const ObjectRecord &rec, std::vector<Tri> *tris, std::string *err) {
  // T = translate(pos) * rotate(AngleAxis(|ori|, ori/|ori|)) * scale(scl)
  V3 o{rec.ori[0], rec.ori[1], rec.ori[2]};
  float angle = std::sqrt(hdot(o, o));
  o = hunit(o);
  float s = std::sin(angle), co = std::cos(angle), omc = 1.f - co;
  float R[3][3];
  {  // Eigen AngleAxis::toRotationMatrix
    V3 sa{s * o.x, s * o.y, s * o.z}, ca{omc * o.x, omc * o.y, omc * o.z};
    float tmp = ca.x * o.y;
    R[0][1] = tmp - sa.z;
    R[1][0] = tmp + sa.z;
    tmp = ca.x * o.z;
    R[0][2] = tmp + sa.y;
    R[2][0] = tmp - sa.y;
    tmp = ca.y * o.z;
    R[1][2] = tmp - sa.x;
    R[2][1] = tmp + sa.x;
    R[0][0] = ca.x * o.x + co;
    R[1][1] = ca.y * o.y + co;
    R[2][2] = ca.z * o.z + co;
  }
  float L[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) L[i][j] = R[i][j] * rec.scl[j];

  std::string obj_text;
  if (!slurp(rec.obj_file, &obj_text)) {
    *err = "Object File was not able to be opened: " + rec.obj_file;
    return false;
  }
  const bool inline_mtl = !rec.mtl_file.empty() && rec.mtl_file[0] == '*';
  std::string mtl_text;
  bool mtl_ok = !inline_mtl && slurp(rec.mtl_file, &mtl_text);
  ObjMesh mesh;
  MtlLibrary lib;
  if (!load_obj(obj_text, mtl_ok ? &mtl_text : nullptr, &mesh, &lib, err)) return false;

  Material fallback;  // faces without a material (scene_basics.h:249-283)
  if (inline_mtl) {
    std::string body = rec.mtl_file.size() >= 2 ? rec.mtl_file.substr(1, rec.mtl_file.size() - 2) : "";
    std::stringstream ss(body);
    std::string ln;
    while (std::getline(ss, ln, '\n')) {
      if (ln.size() >= 3 && ln[0] == 'K' && is_space(ln[2])) {
        Cursor c{ln.c_str() + 2};
        float r = c.real(), g = c.real(), b = c.real();
        if (ln[1] == 'd') {
          fallback.kd[0] = r;
          fallback.kd[1] = g;
          fallback.kd[2] = b;
        }
      }
    }
  }
  const size_t nv = mesh.v.size() / 3, nn = mesh.vn.size() / 3;
  std::vector<V3> vs(nv), ns(nn);
  for (size_t i = 0; i < nv; ++i) {
    float x = mesh.v[3 * i], y = mesh.v[3 * i + 1], z = mesh.v[3 * i + 2];
    float r[3];
    for (int k = 0; k < 3; ++k) r[k] = ((L[k][0] * x + L[k][1] * y) + L[k][2] * z) + rec.pos[k];
    vs[i] = {r[0], r[1], r[2]};
  }
  // normals by T.linear().transpose().inverse() (Eigen cofactor inverse)
  float A[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) A[i][j] = L[j][i];
  auto cof = [&](int i, int j) {
    return A[(i + 1) % 3][(j + 1) % 3] * A[(i + 2) % 3][(j + 2) % 3] -
           A[(i + 1) % 3][(j + 2) % 3] * A[(i + 2) % 3][(j + 1) % 3];
  };
  float c00 = cof(0, 0), c10 = cof(1, 0), c20 = cof(2, 0);
  float det = (c00 * A[0][0] + c10 * A[1][0]) + c20 * A[2][0];
  float inv = 1.f / det;
  float N[3][3] = {{c00 * inv, c10 * inv, c20 * inv},
                   {cof(0, 1) * inv, cof(1, 1) * inv, cof(2, 1) * inv},
                   {cof(0, 2) * inv, cof(1, 2) * inv, cof(2, 2) * inv}};
  for (size_t i = 0; i < nn; ++i) {
    float x = mesh.vn[3 * i], y = mesh.vn[3 * i + 1], z = mesh.vn[3 * i + 2];
    float r[3];
    for (int k = 0; k < 3; ++k) r[k] = (N[k][0] * x + N[k][1] * y) + N[k][2] * z;
    ns[i] = {r[0], r[1], r[2]};
  }
  const size_t nf = mesh.tri_mat.size();
  for (size_t f = 0; f < nf; ++f) {
    int ia = mesh.tri[3 * f], ib = mesh.tri[3 * f + 1], ic = mesh.tri[3 * f + 2];
    if (ia < 0 || ib < 0 || ic < 0 || static_cast<size_t>(ia) >= nv ||
        static_cast<size_t>(ib) >= nv || static_cast<size_t>(ic) >= nv) {
      *err = "face references a vertex out of range in " + rec.obj_file;
      return false;
    }
    int mid = mesh.tri_mat[f];
    const Material &m = mid != -1 ? lib.materials[static_cast<size_t>(mid)] : fallback;
    V3 tn[3];
    const V3 *pn = nullptr;
    if (nn == nv) {
      tn[0] = ns[ia];
      tn[1] = ns[ib];
      tn[2] = ns[ic];
      pn = tn;
    }
    tris->push_back(make_tri(vs[ia], vs[ib], vs[ic], pn, m));
  }
  return true;
}

void camera_matrix(float M[16]) {  // Camera(CameraParams_t(true)), scene.h:15-84
  const V3 eye{0.f, 0.f, 0.f}, look{0.f, 0.f, 1.f}, up0{0.f, 1.f, 0.f};
  const float ha = static_cast<float>(M_PI * static_cast<double>(90.f) / static_cast<double>(360.f));
  const float ar = 1.f;
  V3 dir = hunit(look), up = hunit(up0);
  V3 f = hunit(dir);
  V3 s = hunit(hcross(f, up));
  V3 u = hunit(hcross(s, f));
  const float V[4][4] = {{s.x, s.y, s.z, -hdot(s, eye)},
                         {u.x, u.y, u.z, -hdot(u, eye)},
                         {f.x, f.y, f.z, -hdot(f, eye)},
                         {0.f, 0.f, 0.f, 1.f}};
  const float S[4][4] = {{std::tan(ha), 0.f, 0.f, 0.f},
                         {0.f, std::tan(ha * ar), 0.f, 0.f},
                         {0.f, 0.f, 1.f, 0.f},
                         {0.f, 0.f, 0.f, 1.f}};
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)  // S * V^T
      M[4 * i + j] = ((S[i][0] * V[j][0] + S[i][1] * V[j][1]) + S[i][2] * V[j][2]) + S[i][3] * V[j][3];
}

}  // namespace

bool build_scene(const std::vector<ObjectRecord> &objects, HostScene *out, std::string *err) {
  std::vector<Tri> tris;
  HostScene &S = *out;
  S = HostScene();
  for (const auto &rec : objects) {
    size_t before = tris.size();
    if (!load_mesh(rec, &tris, err)) return false;
    S.obj_first.push_back(static_cast<int>(before));
    S.obj_count.push_back(static_cast<int>(tris.size() - before));
  }
  S.nT = static_cast<int>(tris.size());
  S.isect.resize(tris.size());
  S.geom.resize(tris.size());
  S.mat.resize(tris.size());
  S.kd.resize(tris.size() * 3);
  for (size_t i = 0; i < tris.size(); ++i) {
    const Tri &t = tris[i];
    TriIsect &I = S.isect[i];
    std::memset(&I, 0, sizeof I);
    I.c[0] = t.c.x; I.c[1] = t.c.y; I.c[2] = t.c.z;
    I.n[0] = t.n.x; I.n[1] = t.n.y; I.n[2] = t.n.z;
    float *planes[3] = {I.e0, I.e1, I.e2};
    for (int j = 0; j < 3; ++j) {
      V3 s0 = t.v[j], s1 = t.v[(j + 1) % 3];
      V3 o = hunit(hcross(v3sub(s1, s0), t.n));
      planes[j][0] = o.x;
      planes[j][1] = o.y;
      planes[j][2] = o.z;
      planes[j][3] = -hdot(o, v3add(s1, s0)) / 2.f;
    }
    TriGeom &G = S.geom[i];
    std::memset(&G, 0, sizeof G);
    for (int j = 0; j < 3; ++j) {
      G.v[j][0] = t.v[j].x; G.v[j][1] = t.v[j].y; G.v[j][2] = t.v[j].z;
      G.vn[j][0] = t.vn[j].x; G.vn[j][1] = t.vn[j].y; G.vn[j][2] = t.vn[j].z;
    }
    G.area = t.area;
    sampling_frame(t.n, G.R);
    G.flags = axis_flat(t) ? GEOM_AXIS_FLAT : 0u;
    TriMat &M = S.mat[i];
    for (int j = 0; j < 3; ++j) {
      M.ks[j] = t.m.ks[j];
      M.ke[j] = t.m.ke[j];
      S.kd[3 * i + j] = t.m.kd[j];
    }
    M.shininess = t.m.shininess;
    M.flags = 0;
    if (t.m.ks[0] != 0.f || t.m.ks[1] != 0.f || t.m.ks[2] != 0.f) {
      M.flags |= MAT_HAS_KS;
      if (t.m.shininess != 0.f) M.flags |= MAT_SPECULAR;  // path_trace.cu:132
    }
    if (t.m.ke[0] > 0.f || t.m.ke[1] > 0.f || t.m.ke[2] > 0.f)  // scene_basics.h:184
      S.emit_tri.push_back(static_cast<int>(i));
  }
  S.nE = static_cast<int>(S.emit_tri.size());
  float area_sum = 0.f;
  for (int e : S.emit_tri) area_sum += S.geom[static_cast<size_t>(e)].area;
  float acc = 0.f;
  for (int e : S.emit_tri) {
    float p = S.geom[static_cast<size_t>(e)].area / area_sum;
    acc += p;
    S.emit_cdf.push_back(acc);
    S.emit_pmf.push_back(p);
  }
  camera_matrix(S.cam);
  build_bvh(&S);  // no BVH (bvh_status says why) keeps the brute-force loop
  return true;
}

void export_triangles(const HostScene &s, float *out) {
  std::vector<int> idxE(static_cast<size_t>(s.nT), -1);
  for (int e = 0; e < s.nE; ++e) idxE[static_cast<size_t>(s.emit_tri[static_cast<size_t>(e)])] = e;
  for (int i = 0; i < s.nT; ++i) {
    const TriIsect &I = s.isect[static_cast<size_t>(i)];
    const TriGeom &G = s.geom[static_cast<size_t>(i)];
    const TriMat &M = s.mat[static_cast<size_t>(i)];
    float *o = out + static_cast<size_t>(i) * kExportStride;
    for (int j = 0; j < 3; ++j)
      for (int a = 0; a < 3; ++a) {
        o[3 * j + a] = G.v[j][a];
        o[9 + 3 * j + a] = G.vn[j][a];
      }
    for (int a = 0; a < 3; ++a) {
      o[18 + a] = I.n[a];
      o[21 + a] = I.c[a];
      o[25 + a] = s.kd[3 * static_cast<size_t>(i) + static_cast<size_t>(a)];
      o[28 + a] = M.ks[a];
      o[31 + a] = M.ke[a];
    }
    o[24] = G.area;
    o[34] = M.shininess;
    const float *planes[3] = {I.e0, I.e1, I.e2};
    for (int j = 0; j < 3; ++j)
      for (int a = 0; a < 4; ++a) o[35 + 4 * j + a] = planes[j][a];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) o[47 + 3 * a + b] = G.R[a][b];
    o[56] = static_cast<float>(idxE[static_cast<size_t>(i)]);
  }
}

}  // namespace ipt
