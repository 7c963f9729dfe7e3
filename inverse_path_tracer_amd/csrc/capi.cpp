// capi.cpp -- the C ABI (include/ipt.h): the reference's six FFI symbols plus
// the explicit-parameter API, over the HIP side in ipt_hip.hip.
#include <cmath>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <ctime>
#include <string>
#include <vector>

#include "../../include/ipt.h"
#include "gpu_api.h"
#include "png_io.h"
#include "scene_io.h"
#include "bvh.h"

using ipt::GpuScene;

namespace {

thread_local std::string g_err;

void fail(const std::string &e) { g_err = e; }

struct LegacyConfig {
  int width = 500, height = 500, spp = 100, max_bounces = -1;  // scene.h:8-11
  int64_t seed = -1;                                            // time(NULL)
} g_legacy;

ipt::RenderParams to_params(const ipt_params_t *p) {
  ipt::RenderParams r;
  r.width = p->width;
  r.height = p->height;
  r.spp = p->spp;
  r.max_bounces = p->max_bounces;
  r.seed = p->seed;
  r.row_begin = p->row_begin;
  r.row_end = p->row_end;
  r.row_step = p->row_step;
  return r;
}

ipt::RenderParams legacy_params() {
  ipt::RenderParams r;
  r.width = g_legacy.width;
  r.height = g_legacy.height;
  r.spp = g_legacy.spp;
  r.max_bounces = g_legacy.max_bounces;
  r.seed = g_legacy.seed >= 0 ? (uint64_t)g_legacy.seed : (uint64_t)time(nullptr);  // path_trace.cu:206
  r.row_begin = 0;
  r.row_end = r.height;
  return r;
}

int gpu_status(int rc) {
  if (rc) fail(ipt::gpu_last_error());
  return rc;
}

GpuScene *as_scene(void *p) {
  if (!p) fail("null scene handle");
  return static_cast<GpuScene *>(p);
}

void compress(int nT, const double *acc, float *data) {  // DataWrapper::compress, inv_scene.h:87-115
  const size_t sz = (size_t)(nT + 1) * nT;
  float *wts = data, *pix = data + sz, *lig = data + 4 * sz;
  std::vector<float> ws((size_t)nT);
  for (int dst = 0; dst <= nT; ++dst) {
    float total = 0.f;
    for (int src = 0; src < nT; ++src) {
      const double *e = acc + ((size_t)dst * nT + src) * 8;
      const float w = logf((float)e[0] + 1);  // Edge::normalize, inv_scene.h:38-47
      ws[(size_t)src] = w;
      total += w;
      const float fs = (float)e[1];
      const float den = (fs != 0.f) ? fs : 1.f;
      for (int i = 0; i < 3; ++i) {
        pix[((size_t)dst * nT + src) * 3 + i] = (float)e[2 + i] / den;
        lig[((size_t)dst * nT + src) * 3 + i] = (float)e[5 + i] / den;
      }
    }
    for (int src = 0; src < nT; ++src)
      wts[(size_t)dst * nT + src] = (total != 0.f) ? ws[(size_t)src] / total : 0.f;
  }
}

}  // namespace

extern "C" {

const char *ipt_last_error(void) { return g_err.c_str(); }
void ipt_clear_error(void) { g_err.clear(); }
int ipt_abi_version(void) { return 5; }
int ipt_device_count(void) { return ipt::gpu_device_count(); }
int ipt_selftest_math(uint64_t n, uint64_t seed, uint64_t *counts) {
  if (!counts) return -1;
  return gpu_status(ipt::gpu_selftest_math(n, seed, counts));
}
void ipt_debug_fail_launches(int n) { ipt::gpu_debug_fail_launches(n); }
void ipt_debug_adju_ring(int pool_chunks, int lds_slots) { ipt::gpu_debug_adju_ring(pool_chunks, lds_slots); }

void ipt_legacy_config(int width, int height, int spp, int max_bounces, int64_t seed) {
  g_legacy.width = width;
  g_legacy.height = height;
  g_legacy.spp = spp;
  g_legacy.max_bounces = max_bounces;
  g_legacy.seed = seed;
}

static int load_scene_impl(int n, const float *pos, const float *ori, const float *scl, const char **obj_files,
                           const char **mtl_files, void **scenePtr, bool device) {
  if (scenePtr) *scenePtr = nullptr;
  if (n < 0 || !scenePtr || (n > 0 && (!pos || !ori || !scl || !obj_files || !mtl_files))) {
    fail("ipt_load_scene: bad arguments");
    return -1;
  }
  std::vector<ipt::ObjectRecord> recs((size_t)n);
  for (int i = 0; i < n; ++i) {
    for (int k = 0; k < 3; ++k) {
      recs[(size_t)i].pos[k] = pos[3 * i + k];
      recs[(size_t)i].ori[k] = ori[3 * i + k];
      recs[(size_t)i].scl[k] = scl[3 * i + k];
    }
    if (!obj_files[i] || !mtl_files[i]) {
      fail("ipt_load_scene: null file name");
      return -1;
    }
    recs[(size_t)i].obj_file = obj_files[i];
    recs[(size_t)i].mtl_file = mtl_files[i];
  }
  ipt::HostScene host;
  std::string err;
  if (!ipt::build_scene(recs, &host, &err)) {
    fail(err);
    return -1;
  }
  GpuScene *s = device ? ipt::gpu_upload(host, &err) : ipt::gpu_host_only(host);
  if (!s) {
    fail(err);
    return -1;
  }
  *scenePtr = s;
  return host.nT;
}

int ipt_load_scene(int n, const float *pos, const float *ori, const float *scl, const char **obj_files,
                   const char **mtl_files, void **scenePtr) {
  return load_scene_impl(n, pos, ori, scl, obj_files, mtl_files, scenePtr, true);
}
int ipt_load_scene_host(int n, const float *pos, const float *ori, const float *scl, const char **obj_files,
                        const char **mtl_files, void **scenePtr) {
  return load_scene_impl(n, pos, ori, scl, obj_files, mtl_files, scenePtr, false);
}

int loadScene(float **poss, float **oris, float **scls, char **obj_fs, char **mtl_fs, int n, void **scenePtr) {
  if (n < 0 || !poss || !oris || !scls) {
    if (scenePtr) *scenePtr = nullptr;
    fail("loadScene: bad arguments");
    return -1;
  }
  std::vector<float> pos((size_t)n * 3), ori((size_t)n * 3), scl((size_t)n * 3);
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) {
      pos[(size_t)(3 * i + k)] = poss[i][k];
      ori[(size_t)(3 * i + k)] = oris[i][k];
      scl[(size_t)(3 * i + k)] = scls[i][k];
    }
  return ipt_load_scene(n, pos.data(), ori.data(), scl.data(), const_cast<const char **>(obj_fs),
                        const_cast<const char **>(mtl_fs), scenePtr);
}

void freeScene(void *scenePtr) { ipt::gpu_free(static_cast<GpuScene *>(scenePtr)); }

int ipt_scene_num_triangles(void *scene) {
  GpuScene *s = as_scene(scene);
  return s ? ipt::gpu_host(s).nT : -1;
}
int ipt_scene_num_emissives(void *scene) {
  GpuScene *s = as_scene(scene);
  return s ? ipt::gpu_host(s).nE : -1;
}
int ipt_scene_export_triangles(void *scene, float *out) {
  GpuScene *s = as_scene(scene);
  if (!s || !out) return -1;
  ipt::export_triangles(ipt::gpu_host(s), out);
  return 0;
}
int ipt_scene_camera(void *scene, float *out16) {
  GpuScene *s = as_scene(scene);
  if (!s || !out16) return -1;
  std::memcpy(out16, ipt::gpu_host(s).cam, 16 * sizeof(float));
  return 0;
}

int ipt_scene_bvh_info(void *scene, int32_t *info8) {
  GpuScene *s = as_scene(scene);
  if (!s || !info8) return -1;
  const ipt::HostScene &h = ipt::gpu_host(s);
  info8[0] = (int32_t)h.bvh_nodes.size();
  info8[1] = (int32_t)h.bvh_pairs.size();
  info8[2] = h.bvh_depth;
  info8[3] = ipt::gpu_accel_in_use(s);
  info8[4] = (int32_t)h.bvh_big_pairs.size();
  info8[5] = (int32_t)h.bvh_wide.size();  // 8-wide nodes of the cooperative traversal
  info8[6] = h.bvh_wdepth;
  info8[7] = (int32_t)h.bvh_wtris.size();
  if (h.bvh_nodes.empty()) fail("no BVH: " + h.bvh_status);
  return h.bvh_nodes.empty() ? 0 : 1;
}
int ipt_scene_export_bvh(void *scene, float *nodes, float *pairs, int32_t *big_idx) {
  GpuScene *s = as_scene(scene);
  if (!s) return -1;
  const ipt::HostScene &h = ipt::gpu_host(s);
  if (big_idx && !h.bvh_big_idx.empty())
    std::memcpy(big_idx, h.bvh_big_idx.data(), h.bvh_big_idx.size() * sizeof(int32_t));
  if (nodes && !h.bvh_nodes.empty()) std::memcpy(nodes, h.bvh_nodes.data(), h.bvh_nodes.size() * sizeof(ipt::BvhNode));
  if (pairs && !h.bvh_pairs.empty()) std::memcpy(pairs, h.bvh_pairs.data(), h.bvh_pairs.size() * sizeof(ipt::BvhPair));
  return 0;
}
int ipt_scene_export_wide(void *scene, float *wide) {
  GpuScene *s = as_scene(scene);
  if (!s) return -1;
  const ipt::HostScene &h = ipt::gpu_host(s);
  if (wide && !h.bvh_wide.empty()) std::memcpy(wide, h.bvh_wide.data(), h.bvh_wide.size() * sizeof(ipt::WideNode));
  return 0;
}
int ipt_scene_shadow_masks(void *scene, uint32_t *masks) {
  GpuScene *s = as_scene(scene);
  if (!s || !masks) return -1;
  const std::vector<uint32_t> m = ipt::shadow_occluder_masks(ipt::gpu_host(s));
  std::memcpy(masks, m.data(), m.size() * sizeof(uint32_t));
  return 0;
}
int ipt_scene_set_accel(void *scene, int mode) {
  GpuScene *s = as_scene(scene);
  if (!s) return -1;
  return gpu_status(ipt::gpu_set_accel(s, mode));
}
// The probe kernel indexes emitter and occluder-mask tables with these: a
// target >= 0 must be an emitter triangle, a source must lie in [-1, nT).
static bool probe_ids_ok(GpuScene *s, int64_t n, const int32_t *targets, const int32_t *sources, const char *who) {
  const ipt::HostScene &h = ipt::gpu_host(s);
  for (int64_t i = 0; i < n; ++i) {
    if (targets && targets[i] >= 0 &&
        std::find(h.emit_tri.begin(), h.emit_tri.end(), targets[i]) == h.emit_tri.end()) {
      fail(std::string(who) + ": target " + std::to_string(targets[i]) + " is not an emitter triangle");
      return false;
    }
    if (sources && (sources[i] < -1 || sources[i] >= h.nT)) {
      fail(std::string(who) + ": source " + std::to_string(sources[i]) + " outside [-1, nT)");
      return false;
    }
  }
  return true;
}
int ipt_closest_hit_host(void *scene, int64_t n, const float *origins, const float *dirs, const int32_t *targets,
                         float *t, int32_t *idx) {
  GpuScene *s = as_scene(scene);
  if (!s || n < 0 || (n > 0 && (!origins || !dirs || !t || !idx))) {
    if (s) fail("ipt_closest_hit_host: bad arguments");
    return -1;
  }
  if (!probe_ids_ok(s, n, targets, nullptr, "ipt_closest_hit_host")) return -1;
  return gpu_status(ipt::gpu_closest_hit_host(s, n, origins, dirs, targets, nullptr, t, idx));
}
int ipt_shadow_hit_host(void *scene, int64_t n, const float *origins, const float *dirs, const int32_t *targets,
                        const int32_t *sources, float *t, int32_t *idx) {
  GpuScene *s = as_scene(scene);
  if (!s || n < 0 || (n > 0 && (!origins || !dirs || !targets || !sources || !t || !idx))) {
    if (s) fail("ipt_shadow_hit_host: bad arguments");
    return -1;
  }
  if (!probe_ids_ok(s, n, targets, sources, "ipt_shadow_hit_host")) return -1;
  return gpu_status(ipt::gpu_closest_hit_host(s, n, origins, dirs, targets, sources, t, idx));
}
int ipt_closest_hit_dev(void *scene, int64_t n, const float *origins_dev, const float *dirs_dev,
                        const int32_t *targets_dev, float *t_dev, int32_t *idx_dev, void *stream) {
  GpuScene *s = as_scene(scene);
  if (!s || n < 0) return -1;
  return gpu_status(ipt::gpu_closest_hit(s, n, origins_dev, dirs_dev, targets_dev, nullptr, t_dev, idx_dev, stream));
}

int ipt_scene_get_materials(void *scene, float *kd) {
  GpuScene *s = as_scene(scene);
  if (!s || !kd) return -1;
  const auto &v = ipt::gpu_host(s).kd;
  std::memcpy(kd, v.data(), v.size() * sizeof(float));
  return 0;
}
int ipt_scene_set_materials(void *scene, const float *kd) {
  GpuScene *s = as_scene(scene);
  if (!s || !kd) return -1;
  return gpu_status(ipt::gpu_set_kd(s, kd));
}

void getMaterials(void *scenePtr, float *materials) {
  GpuScene *s = as_scene(scenePtr);
  if (!s || !materials) return;
  const auto &kd = ipt::gpu_host(s).kd;
  std::memcpy(materials, kd.data(), kd.size() * sizeof(float));
}

void setMaterials(void *scenePtr, float *materials) {
  GpuScene *s = as_scene(scenePtr);
  if (!s || !materials) return;
  gpu_status(ipt::gpu_set_kd(s, materials));
}

int ipt_render_samples_host(void *scene, const ipt_params_t *p, float *samples) {
  GpuScene *s = as_scene(scene);
  if (!s || !p || !samples) return -1;
  return gpu_status(ipt::gpu_render_samples_host(s, to_params(p), samples));
}

int ipt_render_host(void *scene, const ipt_params_t *p, float *hdr, uint8_t *ldr) {
  GpuScene *s = as_scene(scene);
  if (!s || !p || !hdr) return -1;
  return gpu_status(ipt::gpu_render_host(s, to_params(p), hdr, ldr));
}

int ipt_adjoint_host(void *scene, const ipt_params_t *p, const float *adj, double *grad) {
  GpuScene *s = as_scene(scene);
  if (!s || !p || !adj || !grad) return -1;
  return gpu_status(ipt::gpu_adjoint_host(s, to_params(p), adj, grad));
}

int ipt_compress(int nT, const double *acc, float *data) {
  if (nT < 0 || !acc || !data) {
    fail("ipt_compress: bad arguments");
    return -1;
  }
  compress(nT, acc, data);
  return 0;
}

int ipt_graph_host(void *scene, const ipt_params_t *p, const uint8_t *target, double *acc, float *data) {
  GpuScene *s = as_scene(scene);
  if (!s || !p || !target) return -1;
  const int nT = ipt::gpu_host(s).nT;
  std::vector<double> bins((size_t)(nT + 1) * nT * 8);
  if (gpu_status(ipt::gpu_graph_host(s, to_params(p), target, bins.data()))) return -1;
  if (acc) std::memcpy(acc, bins.data(), bins.size() * sizeof(double));
  if (data) compress(nT, bins.data(), data);
  return 0;
}

void createImage(void *scenePtr, char *img_file) {
  GpuScene *s = as_scene(scenePtr);
  if (!s || !img_file) return;
  const ipt::RenderParams p = legacy_params();
  std::vector<float> hdr((size_t)p.width * p.height * 3);
  std::vector<uint8_t> ldr((size_t)p.width * p.height * 3);
  if (gpu_status(ipt::gpu_render_host(s, p, hdr.data(), ldr.data()))) return;
  std::string err;
  if (!ipt::png_write_rgb8(img_file, p.width, p.height, ldr.data(), &err)) fail(err);
}

void createGraph(void *scenePtr, char *imgFile, float *data) {
  GpuScene *s = as_scene(scenePtr);
  if (!s || !imgFile || !data) return;
  const ipt::RenderParams p = legacy_params();
  int W = 0, H = 0;
  std::vector<uint8_t> target;
  std::string err;
  if (!ipt::png_read_rgb8(imgFile, &W, &H, &target, &err)) {
    fail(err);
    return;
  }
  if (W != p.width || H != p.height) {  // inv_scene.h:56-57 assumes IM_WIDTH x IM_HEIGHT
    fail("createGraph: target image is " + std::to_string(W) + "x" + std::to_string(H) + ", expected " +
         std::to_string(p.width) + "x" + std::to_string(p.height));
    return;
  }
  ipt_params_t q{p.width, p.height, p.spp, p.max_bounces, p.seed, 0, p.height, 1};
  ipt_graph_host(scenePtr, &q, target.data(), nullptr, data);
}

int ipt_render_dev(void *scene, const ipt_params_t *p, const float *kd_dev, float *hdr_dev, uint8_t *ldr_dev,
                   void *stream) {
  GpuScene *s = as_scene(scene);
  if (!s || !p || !hdr_dev) return -1;
  return gpu_status(ipt::gpu_render(s, to_params(p), kd_dev, hdr_dev, ldr_dev, stream));
}

int ipt_render_samples_dev(void *scene, const ipt_params_t *p, const float *kd_dev, float *samples_dev,
                           void *stream) {
  GpuScene *s = as_scene(scene);
  if (!s || !p || !samples_dev) return -1;
  return gpu_status(ipt::gpu_render_samples(s, to_params(p), kd_dev, samples_dev, stream));
}

int ipt_pixel_mean_dev(const float *samples_dev, int64_t npix, int spp, float *hdr_dev, uint8_t *ldr_dev,
                       void *stream) {
  if (!samples_dev || !hdr_dev || spp <= 0) {
    fail("ipt_pixel_mean_dev: bad arguments");
    return -1;
  }
  return gpu_status(ipt::gpu_pixel_mean(samples_dev, npix, spp, hdr_dev, ldr_dev, stream));
}

int ipt_render_samples_sm_dev(void *scene, const ipt_params_t *p, const float *kd_dev, float *samples_dev,
                              void *stream) {
  GpuScene *s = as_scene(scene);
  if (!s || !p || !samples_dev) return -1;
  return gpu_status(ipt::gpu_render_samples_sm(s, to_params(p), kd_dev, samples_dev, stream));
}

int ipt_pixel_mean_sm_dev(const float *samples_dev, int64_t npix, int spp, float *hdr_dev, uint8_t *ldr_dev,
                          void *stream) {
  if (!samples_dev || !hdr_dev || spp <= 0) {
    fail("ipt_pixel_mean_sm_dev: bad arguments");
    return -1;
  }
  return gpu_status(ipt::gpu_pixel_mean_sm(samples_dev, npix, spp, hdr_dev, ldr_dev, stream));
}

int ipt_adjoint_dev(void *scene, const ipt_params_t *p, const float *kd_dev, const float *adj_dev, double *grad_dev,
                    void *stream) {
  GpuScene *s = as_scene(scene);
  if (!s || !p || !adj_dev || !grad_dev) return -1;
  return gpu_status(ipt::gpu_adjoint(s, to_params(p), kd_dev, adj_dev, grad_dev, stream));
}

int ipt_render_batch_dev(void *scene, const ipt_params_t *p, int n_scenes, uint64_t seed_stride, const float *kd_dev,
                         float *hdr_dev, void *stream) {
  GpuScene *s = as_scene(scene);
  if (!s || !p || !kd_dev || !hdr_dev || n_scenes < 1) {
    if (s) fail("ipt_render_batch_dev: bad arguments (kd_dev and hdr_dev are required, n_scenes >= 1)");
    return -1;
  }
  ipt::RenderParams r = to_params(p);
  r.nscenes = n_scenes;
  r.seed_stride = seed_stride;
  return gpu_status(ipt::gpu_render(s, r, kd_dev, hdr_dev, nullptr, stream));
}

int ipt_adjoint_batch_dev(void *scene, const ipt_params_t *p, int n_scenes, uint64_t seed_stride, const float *kd_dev,
                          const float *adj_dev, double *grad_dev, void *stream) {
  GpuScene *s = as_scene(scene);
  if (!s || !p || !kd_dev || !adj_dev || !grad_dev || n_scenes < 1) {
    if (s) fail("ipt_adjoint_batch_dev: bad arguments (kd_dev, adj_dev and grad_dev are required, n_scenes >= 1)");
    return -1;
  }
  ipt::RenderParams r = to_params(p);
  r.nscenes = n_scenes;
  r.seed_stride = seed_stride;
  return gpu_status(ipt::gpu_adjoint(s, r, kd_dev, adj_dev, grad_dev, stream));
}

int ipt_graph_dev(void *scene, const ipt_params_t *p, const uint8_t *target_dev, double *acc_dev, void *stream) {
  GpuScene *s = as_scene(scene);
  if (!s || !p || !target_dev || !acc_dev) return -1;
  return gpu_status(ipt::gpu_graph(s, to_params(p), target_dev, acc_dev, stream));
}

int ipt_png_write(const char *path, int width, int height, const uint8_t *rgb) {
  std::string err;
  if (!path || !rgb || !ipt::png_write_rgb8(path, width, height, rgb, &err)) {
    fail(err.empty() ? "ipt_png_write: bad arguments" : err);
    return -1;
  }
  return 0;
}

int ipt_png_read(const char *path, int *width, int *height, uint8_t *rgb, int64_t capacity) {
  std::string err;
  int W = 0, H = 0;
  std::vector<uint8_t> img;
  if (!path || !ipt::png_read_rgb8(path, &W, &H, &img, &err)) {
    fail(err.empty() ? "ipt_png_read: bad arguments" : err);
    return -1;
  }
  if (width) *width = W;
  if (height) *height = H;
  if (rgb) {
    if (capacity < (int64_t)img.size()) {
      fail("ipt_png_read: buffer too small");
      return -1;
    }
    std::memcpy(rgb, img.data(), img.size());
  }
  return 0;
}

}  // extern "C"
