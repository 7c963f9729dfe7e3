/*
 * ipt_oracle.h -- CPU ORACLE for the inverse_path_tracer hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the
 * checker / the timed CPU baseline.  The product (inverse_path_tracer_amd)
 * never links or calls it.
 *
 * It is a plain-C restatement of the reference's algorithm
 * (/root/reference: path_trace.cu, inv_path_trace.cu, inv_scene.h, scene.h,
 * bvh.h, scene_basics.h, tiny_obj_loader.h, material.h, utils.h), written in
 * the reference's own shape (AoS triangles, per-sample loop, object-order
 * brute-force intersection).  Every function cites the reference file:line
 * it follows.  The arithmetic is the "canonical arithmetic" of DESIGN.md §3
 * (explicit fmaf where nvcc --fmad=true would contract, IEEE div/sqrt,
 * deterministic double-precision sin/cos/exp/log), so the HIP kernels can be
 * checked against it bit-for-bit.
 *
 * Parity status: the reference cannot be compiled or run in
 * this container (no nvcc / cuRAND / Eigen / stb); the oracle is pinned by the
 * reference's own fixtures: preds/0_true.png region statistics, temp.pt
 * triangle ordering, the scenes/ text files, and by the reference's compile-time
 * constants.  cuRAND XORWOW bit-parity is "parity unpinned" (no reference
 * vector exists); it follows the published curand_kernel.h algorithm.
 */
#ifndef IPT_ORACLE_H
#define IPT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Scene construction (scene.h:177-193 loadScene semantics). Returns NULL on
 * failure; oro_last_error() says why. */
void *oro_load_scene(int n, const float *poss, const float *oris,
                     const float *scls, const char **obj_files,
                     const char **mtl_files);
void oro_free_scene(void *scene);
const char *oro_last_error(void);
int oro_num_triangles(void *scene);
int oro_num_emissives(void *scene);

/* Per-triangle export, ORO_TRI_STRIDE floats per triangle:
 *  [0..8]   v0,v1,v2           [9..17] vertex normals n0,n1,n2
 *  [18..20] face normal        [21..23] centre       [24] area
 *  [25..27] Kd  [28..30] Ks  [31..33] Ke  [34] shininess
 *  [35..38] edge plane 0 (out.xyz, d)  [39..42] plane 1  [43..46] plane 2
 *  [47..55] sampling frame R (row-major)  [56] idxE (as float)            */
#define ORO_TRI_STRIDE 57
void oro_export_triangles(void *scene, float *out);
void oro_get_materials(void *scene, float *out);       /* nT*3 Kd */
void oro_set_materials(void *scene, const float *in);  /* nT*3 Kd */
void oro_camera_matrix(void *scene, float *out16);     /* row-major 4x4 */

/* Forward: per-sample radiance for global sample indices [s_begin,s_end)
 * (path_trace.cu:146-184).  out: (s_end-s_begin)*3 floats.  max_bounces<0
 * means unbounded (reference semantics).  casts (nullable) receives the
 * number of ray casts (camera/continuation + shadow).  Returns 0 on success. */
int oro_render_samples(void *scene, int W, int H, int spp, int max_bounces,
                       uint64_t seed, int64_t s_begin, int64_t s_end,
                       float *out, int64_t *casts);

/* toneMap mean (path_trace.cu:186-198): per-pixel sequential sum of v/spp.
 * samples: npix*spp*3, hdr: npix*3, u8 (nullable): npix*3. */
void oro_pixel_mean(const float *samples, int64_t npix, int spp, float *hdr,
                    uint8_t *u8);

/* Inverse graph (inv_path_trace.cu:109-191 + inv_scene.h:9-115).
 * target: H*W*3 RGB8.  acc (nullable): (nT+1)*nT*8 doubles
 * [w, f0, pix0 rgb, light0 rgb] per (dst,src).  data: (nT+1)*nT*7 floats in
 * the createGraph layout (ipt_cuda.py:145-163). */
int oro_graph_casts(void *scene, int W, int H, int spp, int max_bounces, uint64_t seed, int row_begin,
                    int row_end, int64_t *casts);
int oro_graph(void *scene, int W, int H, int spp, int max_bounces,
              uint64_t seed, int row_begin, int row_end,
              const uint8_t *target, double *acc, float *data);
void oro_compress(int nT, const double *acc, float *data);

/* Adjoint d(sum adj*I)/dKd of the forward estimator under common random
 * numbers (new capability).  adj: H*W*3, grad: nT*3
 * doubles.  Rows [row_begin,row_end) only.  Requires max_bounces >= 0. */
int oro_adjoint(void *scene, int W, int H, int spp, int max_bounces,
                uint64_t seed, int row_begin, int row_end, const float *adj,
                double *grad);

/* Closest hit (BVH::getIntersection over its single leaf, bvh.h:55-77 ->
 * Object::getIntersection, scene_basics.h:426-459) of n caller rays:
 * t[i] (INFINITY on a miss), idx[i] (-1 on a miss). */
int oro_closest_hit(void *scene, int64_t n, const float *org, const float *dir, float *t, int *idx);
/* Per-triangle acceptance of one ray (no best-t test): t_out[nT], NaN where
 * the triangle rejects the ray. */
int oro_hit_each(void *scene, const float *org, const float *dir, float *t_out);

/* Canonical scalar helpers, exported so the tests can pin them. */
float oro_uniform_at(uint64_t seed, int k); /* k-th curand_uniform draw */
void oro_sincos(float x, float *s, float *c);
double oro_log(double x);
double oro_exp(double x);
float oro_powf(float x, float y);

/* Threads used by the oracle (OpenMP); 0 = all. */
void oro_set_threads(int n);

#ifdef __cplusplus
}
#endif
#endif
