/*
 * ipt.h -- C ABI of the MI355X-native inverse path tracer
 * (inverse_path_tracer_amd/lib/libipt_amd.so, also installed as
 * build/libpt.so and build/libipt.so so the reference's ipt_cuda.py loads it
 * unchanged).
 *
 * Part 1 is the reference's own FFI surface, symbol for symbol, with the
 * reference's signatures (the reference's ctypes caller sets no argtypes, so
 * these are plain C ints and pointers).  Part 2 is the explicit-parameter API
 * the reference hard-codes at compile time (scene.h:3-13), plus the adjoint.
 *
 * Errors: the reference exit(1)s on bad input and ignores CUDA errors.  Here
 * no entry point exits; failures return -1 (or leave outputs untouched for the
 * void legacy symbols) and ipt_last_error() says why (thread-local).
 */
#ifndef IPT_H
#define IPT_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ */
/* Part 1: reference symbols                                           */
/* ------------------------------------------------------------------ */

/* Replaces scene.h:177-193 loadScene.  Builds the scene from n object
 * records (pos/ori/scl float[3] each, OBJ path, MTL path or inline
 * "*Kd r g b*") and uploads it to the current HIP device.  Returns the
 * triangle count nT (the reference's return value) or -1 on error, in which
 * case *scenePtr = NULL. */
int loadScene(float **poss, float **oris, float **scls, char **obj_fs, char **mtl_fs, int n,
              void **scenePtr);

/* Replaces scene.h:195-199 freeScene. */
void freeScene(void *scenePtr);

/* Replaces path_trace.cu:227-234 createImage: renders the legacy
 * configuration (500x500, 100 spp, unbounded bounces, seed = time(NULL)
 * unless ipt_legacy_config() set one) and writes an RGB8 PNG tonemapped
 * with 255*x/(1+x). */
void createImage(void *scenePtr, char *img_file);

/* Replaces inv_path_trace.cu:195-208 createGraph: renders the transport
 * graph against the target PNG (must match the legacy image size) and
 * writes (nT+1)*nT*7 floats: weights[(nT+1)*nT] | pixel[(nT+1)*nT*3] |
 * light[(nT+1)*nT*3] (ipt_cuda.py:145-163 layout; eye row last). */
void createGraph(void *scenePtr, char *imgFile, float *data);

/* Replace inv_path_trace.cu:210-221: per-triangle diffuse Kd, nT*3 floats,
 * object-major then triangle, RGB inner (scene.h:145-162). */
void getMaterials(void *scenePtr, float *materials);
void setMaterials(void *scenePtr, float *materials);

/* ------------------------------------------------------------------ */
/* Part 2: explicit API                                                */
/* ------------------------------------------------------------------ */

/* Render configuration.  max_bounces < 0 reproduces the reference
 * (paths end only by Russian roulette or a miss); max_bounces = B allows B
 * continuation rays and does next-event estimation at the (B+1)-th vertex.
 * Sample s of pixel (r,c) has global index (r*width + c)*spp + s and RNG
 * seed `seed + index` (curand_init(seed+index, 0, 0)).  Only rows
 * row_begin, row_begin + row_step, ... < row_end are traced (sharding:
 * row_step 1 = a contiguous band, row_step = world = a rank's interleaved
 * share); images and sample buffers hold those rows, in that order.
 * ABI 2 added row_step; ABI 3 dropped the quantised-node export of
 * ipt_scene_export_wide; ABI 4 added ipt_debug_fail_launches; ABI 5 added
 * ipt_debug_adju_ring (ipt_abi_version).  Bindings must check the version
 * before passing this struct. */
typedef struct ipt_params {
  int32_t width, height, spp, max_bounces;
  uint64_t seed;
  int32_t row_begin, row_end;
  int32_t row_step;
} ipt_params_t;

const char *ipt_last_error(void);
void ipt_clear_error(void);
int ipt_abi_version(void);            /* 5 */
int ipt_device_count(void);
/* Diagnostic: bitwise self-test of the kernels' in-range sqrt/division cores
 * against the IEEE operations over n random operands per test; counts[8]
 * receives mismatch counts (0 expected; counts[6] is the number of unit()
 * fast-path hits, not a mismatch).  No reference counterpart. */
int ipt_selftest_math(uint64_t n, uint64_t seed, uint64_t *counts);
/* Diagnostic (tests): the next n trace-kernel launches fail with an error
 * just before their kernel is enqueued -- after the launch's chunk counters
 * and scratch are allocated.  A later launch on the same stream must be
 * unaffected (the counters reset themselves on the device).  No reference
 * counterpart. */
void ipt_debug_fail_launches(int n);
/* Diagnostic (tests): the unbounded adjoint's record ring at reduced sizes --
 * pool_chunks 16-slot chunks per wave pool (1..63) and lds_slots LDS slots
 * per lane (>= 1); 0 restores the launch's own choice.  Small pools make
 * lanes find the pool empty and shorten their rings (replays), the paths the
 * default sizes almost never take.  Gradients are unchanged.  No reference
 * counterpart. */
void ipt_debug_adju_ring(int pool_chunks, int lds_slots);

/* Legacy-symbol configuration (defaults 500, 500, 100, -1, seed -1 = time). */
void ipt_legacy_config(int width, int height, int spp, int max_bounces, int64_t seed);

/* Same as loadScene with flat arrays (pos/ori/scl: n*3 floats). */
int ipt_load_scene(int n, const float *pos, const float *ori, const float *scl, const char **obj_files,
                   const char **mtl_files, void **scenePtr);
/* Host-only scene (no device buffers): export / materials only; render
 * entry points fail on it.  Lets CPU-only tooling check scene ingest. */
int ipt_load_scene_host(int n, const float *pos, const float *ori, const float *scl, const char **obj_files,
                        const char **mtl_files, void **scenePtr);
int ipt_scene_num_triangles(void *scene);
int ipt_scene_num_emissives(void *scene);
/* nT*57 floats: v0..v2, vertex normals, face normal, centre, area, Kd, Ks,
 * Ke, shininess, three edge planes, sampling frame, emissive index. */
int ipt_scene_export_triangles(void *scene, float *out);
/* getMaterials / setMaterials with a status (nT*3 floats, host memory). */
int ipt_scene_get_materials(void *scene, float *kd);
int ipt_scene_set_materials(void *scene, const float *kd);
int ipt_scene_camera(void *scene, float *out16);

/* Acceleration structure for closest-hit queries.  The reference's BVH
 * (bvh.h:109-205) is over objects and, for its <= 4-object scenes, one leaf:
 * brute force over all triangles, ties to the lowest index
 * (scene_basics.h:426-459, bvh.h:55-77).  Here scenes of >= 64 triangles
 * trace a triangle BVH that returns exactly the same hits;
 * AUTO picks it, BRUTE/BVH force either (BVH fails if the scene has none). */
#define IPT_ACCEL_AUTO 0
#define IPT_ACCEL_BRUTE 1
#define IPT_ACCEL_BVH 2
int ipt_scene_set_accel(void *scene, int mode);
/* info8 = {nodes, leaf pairs, depth, accel in use (IPT_ACCEL_BRUTE/BVH),
 * large-triangle pairs tested before the traversal, 8-wide nodes, 8-wide
 * levels, leaf triangles of the 8-wide tree}; returns 1 if
 * the scene has a BVH, 0 if not (ipt_last_error says why). */
int ipt_scene_bvh_info(void *scene, int32_t *info8);
/* nodes: info8[0]*16 floats (BvhNode), pairs: info8[1]*40 floats (BvhPair:
 * 18 field pairs, then 2 int32 triangle indices, 2 pad), big_idx:
 * info8[4]*2 int32 (the pre-pass triangles, 0x7fffffff = padding); each
 * nullable. */
int ipt_scene_export_bvh(void *scene, float *nodes, float *pairs, int32_t *big_idx);
/* The 8-wide nodes of the cooperative traversal (info8[5] of them): wide
 * receives info8[5]*64 floats (WideNode: per child lo.xyz, hi.xyz, ref bits,
 * pad; nullable). */
int ipt_scene_export_wide(void *scene, float *wide);
/* The shadow rays' potential occluders (bvh.cpp shadow_occluder_masks):
 * masks receives nT * max(nE, 1) words, word [s * nE + e] = the pairs (bit j
 * = triangles 2j, 2j+1) that may occlude a shadow ray from a vertex on
 * triangle s to a point on emitter e (all pairs when not bounded). */
int ipt_scene_shadow_masks(void *scene, uint32_t *masks);
/* Closest hit of n rays (origins, dirs: n*3 floats) through the kernels'
 * own cast: idx = triangle index or -1, t = its distance.  targets
 * (nullable, n ints): >= 0 marks a next-event shadow ray towards that
 * emitter triangle, for which only "idx == target" and then t are defined
 * (the BVH stops once the target is known to be occluded; small scenes use
 * the megakernel's culled shadow cast, which reports -1 when occluded);
 * < 0 a path ray through the megakernel's path cast (small scenes: the
 * culled pair loop).  Without targets small scenes run the full pair loop.
 * Directions need not be unit vectors (t is then in units of |dir|): the
 * BVH's tree-entry culls that assume |dir| = 1, as the megakernel's rays
 * have, are applied only to rays with |dot(dir, dir) - 1| <= 2^-20. */
int ipt_closest_hit_host(void *scene, int64_t n, const float *origins, const float *dirs, const int32_t *targets,
                         float *t, int32_t *idx);
int ipt_closest_hit_dev(void *scene, int64_t n, const float *origins_dev, const float *dirs_dev,
                        const int32_t *targets_dev, float *t_dev, int32_t *idx_dev, void *stream);
/* Rays exactly as the megakernel casts them from a path vertex:
 * sources[i] >= 0 is the triangle the origin lies on (a point its hit test
 * accepted), which selects the static potential-occluder mask of (source,
 * emitter) on top of the culled shadow cast, and in BVH scenes the tree's
 * source-plane skip; < 0 = none.  targets[i] >= 0 = a shadow ray towards that
 * emitter, < 0 = a bounce ray (the path cast), as in ipt_closest_hit_host
 * (both arrays required). */
int ipt_shadow_hit_host(void *scene, int64_t n, const float *origins, const float *dirs, const int32_t *targets,
                        const int32_t *sources, float *t, int32_t *idx);

/* Host-memory entry points (synchronous). */
int ipt_render_samples_host(void *scene, const ipt_params_t *p, float *samples); /* rows*W*spp*3 */
int ipt_render_host(void *scene, const ipt_params_t *p, float *hdr, uint8_t *ldr); /* rows*W*3 */
int ipt_adjoint_host(void *scene, const ipt_params_t *p, const float *adj /*H*W*3*/, double *grad /*nT*3*/);
int ipt_graph_host(void *scene, const ipt_params_t *p, const uint8_t *target /*H*W*3*/,
                   double *acc /*nullable, (nT+1)*nT*8*/, float *data /*nullable, (nT+1)*nT*7*/);
/* DataWrapper::compress (inv_scene.h:87-115) of fp64 accumulators. */
int ipt_compress(int nT, const double *acc, float *data);

/* Device-memory entry points: pointers are device pointers, `stream` a
 * hipStream_t (NULL = null stream); asynchronous.  kd_dev (nT*3) overrides
 * the scene's materials when non-NULL.  grad_dev / acc_dev ACCUMULATE (zero
 * them first). */
int ipt_render_dev(void *scene, const ipt_params_t *p, const float *kd_dev, float *hdr_dev, uint8_t *ldr_dev,
                   void *stream);
int ipt_render_samples_dev(void *scene, const ipt_params_t *p, const float *kd_dev, float *samples_dev,
                           void *stream);
int ipt_pixel_mean_dev(const float *samples_dev, int64_t npix, int spp, float *hdr_dev, uint8_t *ldr_dev,
                       void *stream);
/* The same two steps over a sample-major buffer ([s][pixel][3], rows*W*spp*3
 * floats): the layout ipt_render_dev uses internally (coalesced mean). */
int ipt_render_samples_sm_dev(void *scene, const ipt_params_t *p, const float *kd_dev, float *samples_dev,
                              void *stream);
int ipt_pixel_mean_sm_dev(const float *samples_dev, int64_t npix, int spp, float *hdr_dev, uint8_t *ldr_dev,
                          void *stream);
int ipt_adjoint_dev(void *scene, const ipt_params_t *p, const float *kd_dev, const float *adj_dev, double *grad_dev,
                    void *stream);
int ipt_graph_dev(void *scene, const ipt_params_t *p, const uint8_t *target_dev, double *acc_dev, void *stream);

/* Scene batch (BASELINE config C5 over scenes/0..99.txt, which share their
 * geometry and differ only in the cube's Kd; the reference renders them one
 * loadScene/createImage at a time, ipt_cuda.py:115-134): n_scenes material
 * sets over ONE loaded geometry in one launch.  Set b uses kd_dev + b*nT*3
 * and seed p->seed + b*seed_stride, and equals ipt_render_dev /
 * ipt_adjoint_dev of that kd and seed (images bit for bit, gradients to fp64
 * summation order).  hdr_dev: n_scenes*rows*W*3; adj_dev: n_scenes*H*W*3
 * (full frames, indexed by global pixel like ipt_adjoint_dev); grad_dev:
 * n_scenes*nT*3, accumulated. */
int ipt_render_batch_dev(void *scene, const ipt_params_t *p, int n_scenes, uint64_t seed_stride, const float *kd_dev,
                         float *hdr_dev, void *stream);
int ipt_adjoint_batch_dev(void *scene, const ipt_params_t *p, int n_scenes, uint64_t seed_stride, const float *kd_dev,
                          const float *adj_dev, double *grad_dev, void *stream);

/* PNG helpers (RGB8). ipt_png_read with rgb == NULL only reports the size. */
int ipt_png_write(const char *path, int width, int height, const uint8_t *rgb);
int ipt_png_read(const char *path, int *width, int *height, uint8_t *rgb, int64_t capacity);

#ifdef __cplusplus
}
#endif
#endif
