// valu_rate.hip -- issue rate of the VALU operations the trace kernel mixes
// (gfx950): v_fma_f32, v_pk_fma_f32, v_fma_f64, v_sqrt_f32, v_rsq_f64,
// v_cvt_f64_f32.  Each lane runs 8 independent dependency chains (enough to
// hide the pipeline latency at 8 waves/SIMD), so time = issue slots.
// Build: hipcc -O3 --offload-arch=gfx950 tools/valu_rate.hip -o tools/valu_rate
// Prints one JSON line per op: wave-instructions per SIMD-cycle.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;
constexpr int kChains = 8;

typedef float f2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ __launch_bounds__(256) void rate_kernel(float *out, float seed) {
  const float x0 = seed + threadIdx.x * 1e-7f;
  if (OP == 0) {  // v_fma_f32
    float a[kChains];
    for (int c = 0; c < kChains; ++c) a[c] = x0 + c;
    for (int i = 0; i < kIters; ++i)
#pragma unroll
      for (int c = 0; c < kChains; ++c) a[c] = fmaf(a[c], 0.999f, 1e-3f);
    float s = 0.f;
    for (int c = 0; c < kChains; ++c) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  } else if (OP == 1) {  // v_pk_fma_f32
    f2 a[kChains];
    for (int c = 0; c < kChains; ++c) a[c] = f2{x0 + c, x0 - c};
    for (int i = 0; i < kIters; ++i)
#pragma unroll
      for (int c = 0; c < kChains; ++c) a[c] = __builtin_elementwise_fma(a[c], f2{0.999f, 0.998f}, f2{1e-3f, 2e-3f});
    float s = 0.f;
    for (int c = 0; c < kChains; ++c) s += a[c].x + a[c].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
  } else if (OP == 2) {  // v_fma_f64
    double a[kChains];
    for (int c = 0; c < kChains; ++c) a[c] = (double)x0 + c;
    for (int i = 0; i < kIters; ++i)
#pragma unroll
      for (int c = 0; c < kChains; ++c) a[c] = fma(a[c], 0.999, 1e-3);
    double s = 0.0;
    for (int c = 0; c < kChains; ++c) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = (float)s;
  } else if (OP == 3) {  // v_sqrt_f32 (raw)
    float a[kChains];
    for (int c = 0; c < kChains; ++c) a[c] = x0 + c + 1.f;
    for (int i = 0; i < kIters; ++i)
#pragma unroll
      for (int c = 0; c < kChains; ++c) a[c] = __builtin_amdgcn_sqrtf(a[c]) + 1.0f;
    float s = 0.f;
    for (int c = 0; c < kChains; ++c) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  } else if (OP == 4) {  // v_rsq_f64 (raw) + v_add_f64
    double a[kChains];
    for (int c = 0; c < kChains; ++c) a[c] = (double)x0 + c + 1.0;
    for (int i = 0; i < kIters; ++i)
#pragma unroll
      for (int c = 0; c < kChains; ++c) a[c] = __builtin_amdgcn_rsq(a[c]) + 1.0;
    double s = 0.0;
    for (int c = 0; c < kChains; ++c) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = (float)s;
  } else if (OP == 5) {  // v_add_f64 alone (the companion of OP 4)
    double a[kChains];
    for (int c = 0; c < kChains; ++c) a[c] = (double)x0 + c + 1.0;
    for (int i = 0; i < kIters; ++i)
#pragma unroll
      for (int c = 0; c < kChains; ++c) a[c] = a[c] + 1.0;
    double s = 0.0;
    for (int c = 0; c < kChains; ++c) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = (float)s;
  } else if (OP == 6) {  // v_cvt_f64_f32 + v_cvt_f32_f64 round trip with an add
    float a[kChains];
    for (int c = 0; c < kChains; ++c) a[c] = x0 + c;
    for (int i = 0; i < kIters; ++i)
#pragma unroll
      for (int c = 0; c < kChains; ++c) a[c] = (float)((double)a[c] + 1e-3);
    float s = 0.f;
    for (int c = 0; c < kChains; ++c) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  } else if (OP == 7) {  // v_mul_f64
    double a[kChains];
    for (int c = 0; c < kChains; ++c) a[c] = (double)x0 + c + 1.0;
    for (int i = 0; i < kIters; ++i)
#pragma unroll
      for (int c = 0; c < kChains; ++c) a[c] = a[c] * 0.9999999;
    double s = 0.0;
    for (int c = 0; c < kChains; ++c) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = (float)s;
  }
}

template <int OP>
static void run(const char *name, int ops_per_chain_step, float *out, int cus) {
  const int blocks = cus * 8;  // 8 blocks of 4 waves per CU: 8 waves per SIMD
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(rate_kernel<OP>, dim3(blocks), dim3(256), 0, 0, out, 1.0f);
  hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(rate_kernel<OP>, dim3(blocks), dim3(256), 0, 0, out, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  int clk_khz = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  const double waves_per_simd = (double)blocks * 4 / (cus * 4);
  const double insts = waves_per_simd * kIters * kChains * ops_per_chain_step * reps;  // per SIMD
  const double cycles = (ms * 1e-3) * clk_khz * 1e3;
  std::printf("{\"op\": \"%s\", \"ms\": %.4f, \"wave_insts_per_simd_cycle\": %.4f, \"clock_mhz\": %d}\n", name,
              ms / reps, insts / cycles, clk_khz / 1000);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float *out = nullptr;
  hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(float));
  run<0>("v_fma_f32", 1, out, cus);
  run<1>("v_pk_fma_f32", 1, out, cus);
  run<2>("v_fma_f64", 1, out, cus);
  run<3>("v_sqrt_f32+v_add_f32", 2, out, cus);
  run<4>("v_rsq_f64+v_add_f64", 2, out, cus);
  run<5>("v_add_f64", 1, out, cus);
  run<6>("cvt_f64_f32+add_f64+cvt_f32_f64", 3, out, cus);
  run<7>("v_mul_f64", 1, out, cus);
  hipFree(out);
  return 0;
}
