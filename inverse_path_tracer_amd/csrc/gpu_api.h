// gpu_api.h -- host-callable interface of the HIP side (ipt_hip.hip).
// Plain C++ (no HIP types) so the C-ABI layer compiles without HIP headers.
#pragma once
#include <stdint.h>

#include <string>

#include "../../include/ipt.h"  // IPT_ACCEL_* modes
#include "scene_io.h"

namespace ipt {

struct GpuScene;  // device-resident scene + workspace

GpuScene *gpu_upload(const HostScene &host, std::string *err);
// Host-only handle: no device buffers (export / materials only).
GpuScene *gpu_host_only(const HostScene &host);
bool gpu_on_device(const GpuScene *s);
void gpu_free(GpuScene *s);
const HostScene &gpu_host(const GpuScene *s);
HostScene &gpu_host_mut(GpuScene *s);
int gpu_set_kd(GpuScene *s, const float *kd_host);  // re-upload materials

// All `*_dev` pointers are device pointers; `stream` is a hipStream_t
// (nullptr = the null stream).  kd_dev == nullptr uses the scene's own Kd.
// Return 0 on success, -1 on error (gpu_last_error()).
int gpu_render_samples(GpuScene *s, const RenderParams &p, const float *kd_dev, float *samples_dev,
                       void *stream);
int gpu_pixel_mean(const float *samples_dev, int64_t npix, int spp, float *hdr_dev, uint8_t *ldr_dev,
                   void *stream);
// Same pair over a sample-major buffer [s][pixel][3] (what gpu_render uses).
int gpu_render_samples_sm(GpuScene *s, const RenderParams &p, const float *kd_dev, float *samples_dev,
                          void *stream);
int gpu_pixel_mean_sm(const float *samples_dev, int64_t npix, int spp, float *hdr_dev, uint8_t *ldr_dev,
                      void *stream);
int gpu_render(GpuScene *s, const RenderParams &p, const float *kd_dev, float *hdr_dev, uint8_t *ldr_dev,
               void *stream);
int gpu_adjoint(GpuScene *s, const RenderParams &p, const float *kd_dev, const float *adj_dev,
                double *grad_dev, void *stream);
int gpu_graph(GpuScene *s, const RenderParams &p, const uint8_t *target_dev, double *acc_dev, void *stream);

// Host-memory conveniences (allocate, copy, run, copy back, synchronize).
int gpu_render_samples_host(GpuScene *s, const RenderParams &p, float *samples);
int gpu_render_host(GpuScene *s, const RenderParams &p, float *hdr, uint8_t *ldr);
int gpu_adjoint_host(GpuScene *s, const RenderParams &p, const float *adj, double *grad);
int gpu_graph_host(GpuScene *s, const RenderParams &p, const uint8_t *target, double *acc);

// Acceleration structure (IPT_ACCEL_AUTO / _BRUTE / _BVH) and the one in use.
int gpu_set_accel(GpuScene *s, int mode);
int gpu_accel_in_use(const GpuScene *s);
// Closest hit of n caller-supplied rays (origins, directions: n*3 floats;
// targets: nullable, n ints, >= 0 = shadow ray towards that emitter;
// sources: nullable, n ints, >= 0 = the shadow ray starts on that triangle).
int gpu_closest_hit(GpuScene *s, int64_t n, const float *org_dev, const float *dir_dev, const int *targets_dev,
                    const int *sources_dev, float *t_dev, int *idx_dev, void *stream);
int gpu_closest_hit_host(GpuScene *s, int64_t n, const float *org, const float *dir, const int *targets,
                         const int *sources, float *t, int *idx);

int gpu_device_count();
int gpu_selftest_math(uint64_t n, uint64_t seed, uint64_t *counts);  // 8 mismatch counters
void gpu_debug_fail_launches(int n);  // the next n trace launches fail before their kernel is enqueued
void gpu_debug_adju_ring(int pool_chunks, int lds_slots);  // unbounded adjoint ring sizes (0: default)
const char *gpu_last_error();
void gpu_set_error(const std::string &e);

}  // namespace ipt
