// ipt_hip.hip -- MI355X (gfx950) kernels of the inverse path tracer.
//
// One persistent megakernel traces paths for three integrators that share the
// reference's sampling (template MODE):
//   MODE_FWD    path_trace.cu:111-184  (renderSample/radiance): per-sample
//               radiance to a sample buffer, then pixel_mean_kernel
//               (path_trace.cu:186-198 toneMap) averages it;
//   MODE_ADJ    new: dLoss/dKd of the same estimator under common random
//               numbers (path replay with per-lane vertex records in LDS and
//               a backward sweep when the path ends);
//   MODE_GRAPH  inv_path_trace.cu:109-191 (createGraph): triangle->triangle
//               transport edges accumulated in LDS-privatised fp64 bins.
//
// MI355X-first structure:
//   * one ray per lane, 256-thread workgroups, a grid of exactly the resident
//     workgroups (persistent); each wave owns a contiguous range of global
//     sample indices and refills finished lanes from it with
//     ballot + mbcnt (wave-level compaction, no atomics), so lanes stay busy
//     whatever the path-length spread (the reference's one-thread-per-sample
//     launch idles a wave until its longest path ends);
//   * one loop iteration is one path vertex for the whole wave, in
//     wave-synchronous phases (path cast, shading with all of the vertex's
//     random numbers, shadow cast, emitter term, finish), so each phase --
//     above all the closest-hit loop -- runs once per iteration with most
//     lanes on;
//   * the closest-hit loop walks the triangle table with a wave-uniform
//     index: 80-B records arrive through scalar loads and the test is
//     branch-free per lane.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "bvh.h"
#include "gpu_api.h"
#include "ipt_device.h"

namespace ipt {

static thread_local std::string g_gpu_err;
void gpu_set_error(const std::string &e) { g_gpu_err = e; }
const char *gpu_last_error() { return g_gpu_err.c_str(); }
// ipt_debug_fail_launches(n): the next n trace launches fail just before
// their kernel is enqueued (after the chunk counters and the launch's scratch
// are allocated) -- the tests' way to check that a failed launch leaves
// nothing behind that a later launch on the stream depends on
static std::atomic<int> g_fail_launches{0};
void gpu_debug_fail_launches(int n) { g_fail_launches.store(n > 0 ? n : 0); }
// ipt_debug_adju_ring(chunks, slots): the unbounded adjoint's pool chunks per
// wave and LDS slots per lane forced small (0: the launch's choice) -- the
// tests' way to run the empty-pool and short-ring paths
static std::atomic<int> g_adju_pool{0}, g_adju_lds{0};
void gpu_debug_adju_ring(int pool_chunks, int lds_slots) {
  g_adju_pool.store(pool_chunks > 0 ? std::min(pool_chunks, 63) : 0);
  g_adju_lds.store(lds_slots > 0 ? lds_slots : 0);
}

#define HIP_TRY(expr)                                                                        \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess) {                                                                  \
      gpu_set_error(std::string(#expr) + ": " + hipGetErrorString(e_));                      \
      return -1;                                                                             \
    }                                                                                        \
  } while (0)

// MODE_ADJU: the adjoint of the reference's own estimator (no bounce cap,
// paths end by Russian roulette or a miss, path_trace.cu:172-181).  Vertex
// records live in an LDS ring of rec_cap slots; a path longer than the ring
// is swept in chunks from its end, each earlier chunk re-recorded by
// replaying the path from its camera ray (same seed, same draws, so the same
// floats) -- see trace_kernel.
// MODE_FWDM: MODE_FWD with the pixel mean fused in (gpu_render, TraceArgs::fused).
// MODE_ADJW: MODE_ADJ compiled for 6 waves/SIMD instead of 5 (80 VGPRs), for
// full-size launches (gpu_adjoint: C2 adjoint 1.914 -> 1.862 ms, scenes/0
// 2.316 -> 2.275; a C2 1/8 share is slower with it, 0.307 -> 0.320 ms,
// profiles/r04/variants_chain_adj6_r04l.log, envab_adjw_r04m.log); brute-force diffuse scenes only.
enum { MODE_FWD = 0, MODE_ADJ = 1, MODE_GRAPH = 2, MODE_ADJU = 3, MODE_FWDM = 4, MODE_ADJW = 5 };
template <int MODE>
constexpr bool is_badj() {  // the bounded adjoint (either occupancy)
  return MODE == MODE_ADJ || MODE == MODE_ADJW;
}
template <int MODE>
constexpr bool is_adj() {
  return is_badj<MODE>() || MODE == MODE_ADJU;
}
template <int MODE>
constexpr bool is_fwd() {
  return MODE == MODE_FWD || MODE == MODE_FWDM;
}
constexpr int kBlock = 256;
// Adjoint vertex record (per lane, in LDS): tri | et << 16, the emitter factor
// s (lo = Ke[et] * s is rebuilt bit-identically in the sweep; s = 0 when the
// shadow ray failed), coeff; with a Phong lobe also specd and speci.  The
// prefix throughputs are not recorded (3 more words per vertex cost a wave
// of occupancy and measured slower, profiles/r02_variants_adj_sweep.log):
// the sweep rebuilds them with the forward's own operations.
constexpr int kRecSD = 3;  // specd, then speci
constexpr int kRecFieldsDiffuse = 3;
constexpr int kRecFieldsSpec = kRecFieldsDiffuse + 2;
constexpr int kMaxAdjTris = 65535;  // tri and et share one 32-bit field
constexpr int kEdgeW = 8;      // graph bin: w, w*f, pix[3]*w*f, light[3]*w*f
// LDS form of the graph bins: 5 doubles per (dst, src) (w, w*f, pix[3]*w*f)
// plus 3 light doubles per (dst, emitter) -- only next-event updates, whose
// source is an emitter, touch the light fields.  60 -> 39 KB for scenes/0.txt
// (2 -> 4 workgroups per CU); flushed into the global kEdgeW-wide layout.
constexpr int kEdgeL = 5;
__host__ __device__ inline size_t graph_lds_doubles(int nT, int nE) {
  return (size_t)(nT + 1) * nT * kEdgeL + (size_t)(nT + 1) * (nE > 0 ? nE : 0) * 3;
}
constexpr int kMaxAdjBounces = 62;
// ADJU ring slots per lane (3 words each, like ADJ's records: tri | et,
// emitter factor, coeff; the prefix throughputs are rebuilt by the sweep's
// chain from the chunk's first one, Mlo).  Round 3 kept 64 six-word slots
// (with the recorded M_k) per lane in global memory (503 MB at C3 for 327 680
// resident lanes): the records of the live paths overflowed the XCDs' L2s --
// 7.5 GB fetched and 6.7 GB written per C3 launch, 48% L2 hits
// (profiles/r04/unbounded_pmc_r04g.txt) -- and the unbounded adjoint took 1.7x
// the unbounded forward.  Now the first IPT_ADJU_LDS_SLOTS slots of every lane
// are in LDS (a path of up to 8 vertices never touches global memory) and the
// rest of the ring is global, IPT_ADJU_RING = 63 slots in all (round 4: 56
// global slots per lane, 220 MB at C3 for 327 680 resident lanes; now pool
// chunks per wave, below).  The ring's size is what bounds the
// launch's tail: a path longer than the ring replays from its camera ray, and
// the longest paths of a launch (~65 vertices in 16.8 M Russian-roulette
// paths) then run alone at its end -- a 24-slot ring (64 MB) left the average
// wave idle for a quarter of the C3 launch; 63 slots: C3 4.32 -> 4.08 ms,
// Cornell 3.26 -> 3.08, north star 8.21 -> 8.00
// (profiles/r04/variants_adju_rings_r04x.log).  Only the slots a path reaches
// are ever written (the AoS layout below), so the HBM traffic follows the
// path lengths, not the allocation.  Chunks are aligned to the ring: a path of K vertices is swept in chunks
// [j R, min((j+1) R, K)), R = ring slots, the last one straight after the
// first pass (its prefix throughput captured there at vertex j R), every
// earlier one after a replay from the camera ray to its end (K = 30, R = 24:
// 24 replayed vertex traces; a path of K costs about K^2 / 2R, DESIGN.md
// §10.3).  Round 2 kept an 8-slot ring in LDS (24 KB
// per workgroup): every path longer than 8 vertices replayed, C3 unbounded
// adjoint 5.97 ms for a 2.73 ms forward.
#ifndef IPT_CHAIN_DPP  // the sweep's chain steps with the wave shifts fused into their VALU ops (ipt_device.h)
#define IPT_CHAIN_DPP 1
#endif
#ifndef IPT_ADJU_SHIFTED_CHAIN  // the bounded adjoint's chain form in MODE_ADJU too (A/B)
#define IPT_ADJU_SHIFTED_CHAIN 0
#endif
#ifndef IPT_ADJU_RING
#define IPT_ADJU_RING 63
#endif
// The ring's global slots come from a pool per wave, in chunks of
// kPoolSlots slots handed out as a lane's path reaches them (a lane holds at
// most kPoolMaxChunks, their ids packed 6 bits each in `ctab`, 63 = none).
// Most lanes never leave the LDS slots (a path of K vertices uses
// ceil((K - rec_lds) / 16) chunks), so a pool of up to 63 chunks
// (TraceArgs::pool_chunks, sized to IPT_ADJU_POOL_MB) serves 64 lanes: 12 KB
// per wave, 62 MB at C3 (5120 resident waves) for the 220 MB of round 4's
// per-lane ring.  A lane that finds the pool empty makes its current slot
// count its ring size for the rest of the path (its chunks stay aligned to it,
// the usual replays follow) -- with 4 LDS slots (the BVH instances) and 32
// chunks that happened to 0.8% of the paths of a q = 0.8 simulation, and the
// north star's unbounded adjoint lost 3%; with 48 or more, never
// (tests/test_adju_protocol.py models the hand-out).
constexpr int kPoolSlots = 16, kPoolMaxChunks = 4;
#ifndef IPT_ADJU_POOL_MB
#define IPT_ADJU_POOL_MB 64
#endif
// LDS ring slots only while the workgroup's LDS stays under this (bytes): at
// equal occupancy (5 blocks/CU) scenes/0's unbounded adjoint ran 4.33 ms with
// 8 slots (32.2 KB) and 4.10 with 6 (26.1 KB), Cornell's 3.26 with 8 (30.0 KB)
// and 3.40 with 6 (profiles/r04/envab_adjulds_r04w.log, _r04x.log)
#ifndef IPT_ADJU_LDS_CAP
#define IPT_ADJU_LDS_CAP (31 * 1024)
#endif
#ifndef IPT_ADJU_LDS_SLOTS
#define IPT_ADJU_LDS_SLOTS 8
#endif
// (BVH instance, at 4 waves/SIMD since round 5: 6 slots -- north-star 6.43
// -> 6.37 ms against 4; 7 loses the fourth workgroup, 7.13 ms;
// profiles/r05/variants_bvh_adju_lds_slots*.log)
#ifndef IPT_ADJU_LDS_SLOTS_BVH
#define IPT_ADJU_LDS_SLOTS_BVH 6
#endif
#ifndef IPT_ADJU_LDS_SLOTS_FIXED
#define IPT_ADJU_LDS_SLOTS_FIXED -1
#endif
constexpr int kAdjuRing = IPT_ADJU_RING;
// Sub-chunked sweep of the unbounded adjoint (IPT_ADJU_SUB = G > 0): a chunk
// is swept G vertices at a time from its end, one sub-chunk per loop
// iteration, the lane tracing nothing meanwhile (its suffix carried in Scar,
// as between chunks), so a sweep round's chain runs at most G - 1 steps
// instead of as long as the round's longest path.  The forward's M at every
// G-th slot of a chunk (k > 0) is captured to a per-lane global array
// (TraceArgs::mring, kMrEnt entries), which also replaces the chunk's Mlo
// register.  0: whole chunks per round (round 5).
#ifndef IPT_ADJU_SUB
#define IPT_ADJU_SUB 0
#endif
constexpr int kSub = IPT_ADJU_SUB;
constexpr int kMrEnt = kSub > 0 ? (kAdjuRing + kSub - 1) / kSub : 1;
// Dynamic work distribution across the waves of a launch (TraceArgs::chunk):
// static per-wave ranges left each launch's tail to the waves whose pixels
// hold the longest paths -- C2 forward 2.41 -> 2.11 ms, sphere 6.61 -> 4.63 ms,
// north-star 8.52 -> 5.79 ms, adjoints 1.16-1.63x
// (profiles/r02_variants_dynamic_chunks.log).  IPT_DYN_CHUNKS_PER_WAVE sets
// the chunk size (items per launch / waves / this, a multiple of 64).
#ifndef IPT_DYN_CHUNKS
#define IPT_DYN_CHUNKS 1
#endif
#ifndef IPT_DYN_CHUNKS_PER_WAVE
#define IPT_DYN_CHUNKS_PER_WAVE 32
#endif
#ifndef IPT_DYN_MIN_CHUNK
#define IPT_DYN_MIN_CHUNK 128
#endif
constexpr int kMaxTableTris = 512;  // kd/kd-over-pi LDS tables up to 12 KB
// (an LDS table of the emission Ke next to them -- vertex 0's Le, the
// emitter's lo, the sweep's lo -- measured neutral, profiles/r03/variants_ke_ring_r03n.log)
#ifndef IPT_LDS_GRAD_KB
#define IPT_LDS_GRAD_KB 12
#endif
// ADJ gradient bins in LDS (12 KB: all of them up to nT = 512, else the hot
// set).  12 rather than 16 KB lets the BVH adjoint (bins + vertex records +
// tree + group stacks) keep 3 workgroups per CU: sphere scene 16.3 -> 12.1 ms.
constexpr int kLdsGradBytes = IPT_LDS_GRAD_KB * 1024;
// Scenes of at least this many triangles trace through the BVH (auto mode).
// Below it the unrolled / packed brute-force loop wins (a few pairs per cast).
#ifndef IPT_BVH_MIN_TRIS
#define IPT_BVH_MIN_TRIS 64
#endif
constexpr int kBvhMinTris = IPT_BVH_MIN_TRIS;
#ifndef IPT_BVH_LDS_KB
#define IPT_BVH_LDS_KB 32
#endif
constexpr int kBvhLdsNodeBytes = IPT_BVH_LDS_KB * 1024;  // stage the whole tree in LDS up to 512 nodes

struct TraceArgs {
  int W, H, spp, max_bounces;
  uint64_t seed;
  uint64_t n_samples;
  int nT, nE;
  int lds_edges;  // GRAPH: bins privatised in LDS
  int sample_major;  // FWD: sample buffer [s][pixel][3] (else [pixel][s][3])
  int kd_tables;     // kd and kd/pi staged in LDS
  const float *kdpi_g;  // kd/pi in global memory (large scenes: no LDS tables), per launch
  int small_pairs;   // nT <= 2*kSmallPairs: unrolled closest-hit, plane offsets in LDS
  uint64_t npix;     // pixels of the launch (its rows x W)
  int row0, row_step;  // traced rows: row0, row0 + row_step, ... (row_step 1: a contiguous band)
  // index arithmetic: when every global sample index of the frame is below
  // 2^32, g / spp and pixel / W use Lemire's multiply-high division
  // (M = ceil(2^64 / d), exact for 32-bit n and d > 1) instead of the ~40
  // instruction 64-bit division sequence
  int idx32;
  uint64_t m_spp, m_W, m_npix;
  // BVH (BVH instances only): nodes staged in LDS (0: read from global),
  // traversal stack entries per lane
  int bvh_nbig;                 // large-triangle pairs tested before the traversal
  // cooperative traversal (IPT_BVH_COOP): 8-wide nodes (first bvh_wide_lds of
  // them staged in LDS: all or none), leaf triangles, group-stack entries
  const float4 *bvh_wide;  // WideNode or QWideNode records (kWideF4 float4 each)
  const TriIsect *bvh_wtris;
  int bvh_wide_lds, coop_stride;
  int bvh_big_lds;  // culled path pre-pass: the large pairs' LDS copy is built (launch_bvh chooses)
  float root_box[6];
  float tree_sphere[4];     // bvh.cpp tree_cull
  const float4 *src_cull;   // per triangle {face normal, tau} (ipt_device.h tree_skip)
  const TriPair *bvh_big;
  const int32_t *bvh_big_idx;
  const PairBox2 *bvh_big_boxes;
  // ADJ gradient bins: grad_slots triangles accumulate in LDS fp64 (all of
  // them when they fit, else the largest -- the most-hit -- ones, mapped by
  // grad_map[tri] -> slot or -1, slot_tri[slot] -> tri); the rest go to
  // global fp64 atomics directly
  int grad_slots;
  const int *grad_map;
  const int *slot_tri;
  float cam[16];
  float cam_org[3];
  // per emitter: 1/pmf when pmf is a power of two (then x * (1/pmf) == x / pmf
  // exactly), else 0 -- the emitter term's double division becomes a multiply
  const double *emit_pmfr;  // the camera origin M * (0,0,0,1) with camera_ray's own operations (host, same IEEE ops)
  // 1/spp when spp is a power of two (then x * rc_spp == x / spp for every
  // float x: both are the correctly rounded x * 2^-k), else 0
  float rc_spp;
  float rc_W, rc_H;  // 1/W, 1/H for power-of-two sizes, else 0 (camera_ray divides)
  int rec_cap;   // ADJ: vertex records per lane (max_bounces + 1); ADJU: ring slots
  // ADJU: ring slots 0 .. rec_lds-1 of every lane live in LDS ([field][slot]
  // [lane], like ADJ's records), slots rec_lds .. rec_cap-1 in pool chunks in
  // global memory (grec: grec_stride floats per wave, pool_chunks chunks)
  int rec_lds;
  float *grec;
  uint64_t grec_stride;
  int pool_chunks;  // ADJU: chunks per wave pool (<= 63)
  // ADJU with IPT_ADJU_SUB: per wave [kMrEnt][64 lanes][3] floats, entry e
  // = the forward's M before the update of the vertex in ring slot e * kSub
  float *mring;
  // scene batch (C5): blocks b, b + nscenes, ... (bps of them) trace material
  // set b -- interleaved, not contiguous ranges: the dispatcher fills a CU
  // with consecutive workgroups, so contiguous ranges gave some sets fewer
  // CUs and the launch waited on them (C5 forward 5.77 -> 4.81 ms, adjoint
  // 6.66 -> 5.29 ms, profiles/r02_batch_interleave.log) --
  // kd + b*3nT, seed + b*seed_stride, outputs at b * (out|adj)_stride,
  // gradient at b*3nT -- so each workgroup holds ONE set's tables and bins
  // (the single-scene LDS footprint) and every set is the single-scene
  // launch of its own kd and seed
  int nscenes, bps;
  uint64_t seed_stride, out_stride, adj_stride;
  // dynamic work distribution (IPT_DYN_CHUNKS): a wave starts with chunk
  // `wave` of `chunk` items and then takes chunk nwaves + atomicAdd(ctr[set])
  // until the launch's items are used up; chunk 0 = static per-wave ranges
  uint32_t chunk;
  // guided sizes: the first chunk_big_n chunks hold `chunk` units, the rest
  // chunk_small (units: work items, or pixels in MODE_FWDM), so a launch ends
  // on small chunks and its waves run dry close together (chunk_range)
  uint32_t chunk_small, chunk_big_n;
  // the launch's grab counters (one word per material set or XCD region).
  // Each wave grabs until one grab fails, so a word ends a launch at
  // `grabs` (launch_grabs: a function of the launch's shape, like the chunk
  // sizes); the wave whose grab returns grabs - 1 zeroes the word.  Each
  // launch on a stream thus starts from zeroed counters in stream order -- no
  // host-side copy of device state, no memset launch per launch, no extra
  // atomic (a count of finished waves cost 2% on the adjoints)
  uint32_t *chunk_ctr;  // word j at chunk_ctr[j * kCtrStride]
  uint32_t grabs;
  // small scenes: acceptance boxes of the pairs (culled shadow casts)
  const PairBox2 *pboxes;
  // small scenes: potential occluders per (source triangle, emitter), nT*nE
  // words (bvh.cpp shadow_occluder_masks), copied to LDS; nullptr = none
  const uint32_t *pomask;
  // BVH scenes: the same masks over the large-triangle pairs (nullptr = none)
  const uint32_t *big_pomask;
  // FWD with the pixel mean fused in (gpu_render, IPT_FUSED_MEAN): a chunk of
  // `chunk` (then chunk_small) launch-local pixels is issued in groups of
  // `group` pixels x spp samples;
  // each pixel of a group gets one of the wave's nslots LDS slots (spp x 3
  // floats), a finished sample goes to its pixel's slot, and a slot whose
  // last sample is in is summed in sample order (toneMap) into out_samples
  // (HDR, npix x 3) and ldr.  Per wave, at byte mean_off + wave *
  // mean_wstride * 4 of the dynamic LDS: the slots' unfinished counts
  // [nslots], their pixels [nslots], then the slots
  int fused;
  uint32_t group;
  uint32_t mean_off, mean_wstride;
  int nslots;
  uint8_t *ldr;
};
static_assert(alignof(TraceArgs) == 8, "TraceArgs sits right after the ten 8-B scene pointers in the kernarg segment");

__device__ __forceinline__ uint32_t udiv32(uint32_t n, uint64_t m, uint32_t d) {
  return d == 1u ? n : (uint32_t)__umul64hi(m, (uint64_t)n);
}

// Work item w of a launch -> (launch-local pixel lp, sample sj).  Pixel-major:
// w = lp * spp + sj (a wave traces consecutive samples of one pixel).
// Sample-major: w = sj * npix + lp (lane i of a wave writes slot base + i of a
// [s][pixel][3] buffer -- one contiguous store run).
__device__ __forceinline__ void item_split(const TraceArgs &a, uint64_t w, uint64_t &lp, uint64_t &sj) {
  if (a.idx32) {
    if (a.sample_major) {
      const uint32_t q = udiv32((uint32_t)w, a.m_npix, (uint32_t)a.npix);
      sj = q;
      lp = (uint32_t)w - q * (uint32_t)a.npix;
    } else {
      const uint32_t q = udiv32((uint32_t)w, a.m_spp, (uint32_t)a.spp);
      lp = q;
      sj = (uint32_t)w - q * (uint32_t)a.spp;
    }
  } else if (a.sample_major) {
    sj = w / a.npix;
    lp = w - sj * a.npix;
  } else {
    lp = w / (uint64_t)a.spp;
    sj = w - lp * (uint64_t)a.spp;
  }
}
// launch-local pixel -> image row and column
__device__ __forceinline__ void local_rc(const TraceArgs &a, uint64_t lp, int &r, int &c) {
  uint64_t lr;
  if (a.idx32) {
    const uint32_t q = udiv32((uint32_t)lp, a.m_W, (uint32_t)a.W);
    lr = q;
    c = (int)((uint32_t)lp - q * (uint32_t)a.W);
  } else {
    lr = lp / (uint64_t)a.W;
    c = (int)(lp - lr * (uint64_t)a.W);
  }
  r = a.row0 + (int)lr * a.row_step;
}

// Guided chunk sizes for the brute-force instances too (IPT_BF_BIG = the big
// chunks' size in small ones, > 1; see launch_inst): every grab is a
// device-scope atomic, performed at the memory side (the XCDs' L2s are not
// coherent), and the launch's grabs queue there -- C2 adjoint 131 072 -> 77 824
// grabs, 1.816 -> 1.764 ms, the sample-buffer forward 1.629 -> 1.525, scenes/0
// adjoint 2.276 -> 2.243; 3 or 4 (fewer grabs still) lose some of it, and the
// fused render's 256-sample grabs are neutral (profiles/r06/variants_bf_r06c.log,
// variants_ctr_stride_r06e.log)
#ifndef IPT_BF_BIG
#define IPT_BF_BIG 2
#endif
#ifndef IPT_BF_TAIL
#define IPT_BF_TAIL 4
#endif
// The grab counters' spacing in words: the device-scope atomics on one line
// are serialised at the memory side, so each word (material set) gets a
// 128-B line of its own.  Eight words on one line (round 6's XCD bands,
// DESIGN.md §12.2) doubled a C2 1/8 share's adjoint (0.31 -> 0.70 ms), one
// line each: 0.32; the C2 adjoint 1.796 -> 1.768 ms with it
// (profiles/r06/variants_bands_r06d.log, variants_ctr_stride_r06e.log,
// variants_grab_r06h.log)
#ifndef IPT_CTR_STRIDE
#define IPT_CTR_STRIDE 32
#endif
constexpr int kCtrStride = IPT_CTR_STRIDE;
template <bool BVH>
constexpr bool kGuided() {
  return BVH || IPT_BF_BIG > 1;
}
// Chunk g of a launch (TraceArgs::chunk_big_n) -> units [start, end).
// GUIDED: the BVH instances (guided_tail); the others take `chunk` units.
template <bool GUIDED>
__device__ __forceinline__ void chunk_range(const TraceArgs &a, uint64_t g, uint64_t units, uint64_t &start,
                                            uint64_t &end) {
  const uint64_t nb = a.chunk_big_n;
  uint64_t len;
  if (!GUIDED || g < nb) {
    start = g * a.chunk;
    len = a.chunk;
  } else {
    start = nb * a.chunk + (g - nb) * a.chunk_small;
    len = a.chunk_small;
  }
  end = start + len < units ? start + len : units;
}

// The failed grab that returned c: the launch's last grab of that word
// (TraceArgs::grabs) zeroes it.
__device__ __forceinline__ void grab_failed(uint32_t *word, uint32_t c, uint32_t grabs) {
  if (c + 1u == grabs) __hip_atomic_store(word, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// global pixel index (r * W + c) of this launch's work item w
__device__ __forceinline__ uint64_t item_pixel(const TraceArgs &a, uint64_t w) {
  uint64_t lp, sj;
  item_split(a, w, lp, sj);
  int r, c;
  local_rc(a, lp, r, c);
  if (a.idx32) return (uint32_t)r * (uint32_t)a.W + (uint32_t)c;
  return (uint64_t)r * (uint64_t)a.W + (uint64_t)c;
}

using namespace dev;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// Work item w of a launch -> global sample g, pixel (r, c), XORWOW state
// after the two camera draws and the camera ray (path_trace.cu:150-165); the
// enumeration is described in trace_kernel.
__device__ __forceinline__ void item_ray_ls(const TraceArgs &a, uint64_t seed, uint64_t lp, uint64_t sj, Rng &st, V3 &p,
                                            V3 &d, int &r, int &c) {
  local_rc(a, lp, r, c);
  uint64_t g;  // global sample index
  if (a.idx32) {  // every index of the frame fits 32 bits: one 32x32->64 multiply-add
    const uint32_t pixel = (uint32_t)r * (uint32_t)a.W + (uint32_t)c;
    g = (uint64_t)pixel * (uint32_t)a.spp + sj;
  } else {
    g = ((uint64_t)r * (uint64_t)a.W + (uint64_t)c) * (uint64_t)a.spp + sj;
  }
  rng_init(st, seed + g);
  camera_ray(a.cam, a.cam_org, st, r, c, a.W, a.H, a.rc_W, a.rc_H, p, d);
}
__device__ __forceinline__ void item_ray(const TraceArgs &a, uint64_t seed, uint64_t w, Rng &st, V3 &p, V3 &d, int &r,
                                         int &c) {
  uint64_t lp, sj;
  item_split(a, w, lp, sj);
  item_ray_ls(a, seed, lp, sj, st, p, d, r, c);
}

// ---------------------------------------------------------------------------
// Minimum resident 256-thread blocks per CU (= waves per SIMD) requested per
// integrator; 0 lets the compiler choose.  Round 1 measured 6 best (80 VGPRs,
// 20 B of cold spill); with the dynamic chunks, the culled shadow cast and
// the batch fields the 80-VGPR build spills 72-76 B per lane inside the loop
// and 5 (96 VGPRs, 12-20 B) wins: C2 forward 2.11 -> 1.98 ms, adjoint 2.49 ->
// 2.41, scenes/0 2.66 -> 2.53 / 2.98 -> 2.95; 4 (108-115 VGPRs, no spill)
// loses (profiles/r02_variants_occupancy.log).
#ifndef IPT_MIN_BLOCKS_FWD
#define IPT_MIN_BLOCKS_FWD 5
#endif
#ifndef IPT_MIN_BLOCKS_ADJ
#define IPT_MIN_BLOCKS_ADJ 5
#endif
#ifndef IPT_MIN_BLOCKS_ADJU
#define IPT_MIN_BLOCKS_ADJU 5
#endif
#ifndef IPT_MIN_BLOCKS_ADJW
#define IPT_MIN_BLOCKS_ADJW 6
#endif
#ifndef IPT_ADJW_LANE_LDS  // MODE_ADJW's work item and Le in LDS (trace_kernel's lane_ws)
#define IPT_ADJW_LANE_LDS 1
#endif
#ifndef IPT_MIN_BLOCKS_GRAPH
#define IPT_MIN_BLOCKS_GRAPH 0
#endif
// The BVH instances hold the traversal state on top (slab parameters, stack
// pointer, node) and their LDS (node copy + stack) caps residency anyway:
// 4 waves/SIMD, 128 VGPRs, no spill.
#ifndef IPT_MIN_BLOCKS_BVH
#define IPT_MIN_BLOCKS_BVH 4
#endif
// The adjoint's BVH instance: its LDS (gradient bins + vertex records + tree
// + group stacks, ~55 KB for the sphere scene) allows only 2 workgroups per
// CU, i.e. 2 waves/SIMD, so it may use up to 256 VGPRs without losing
// residency (at 4 waves/SIMD it spilled).
#ifndef IPT_MIN_BLOCKS_BVH_ADJ
#define IPT_MIN_BLOCKS_BVH_ADJ 2
#endif
// The unbounded adjoint's BVH instance: its LDS (4 ring slots, the gradient
// hot set, the tree stage) leaves room for 4 workgroups per CU, and at 131
// VGPRs it ran 3 waves/SIMD; held to 128 (4 waves) it spills nothing and the
// north-star unbounded adjoint runs 7.08 -> 6.4x ms.
#ifndef IPT_MIN_BLOCKS_BVH_ADJU
#define IPT_MIN_BLOCKS_BVH_ADJU 4
#endif
// The forward's BVH instance at 5 waves/SIMD (96 VGPRs, ~116 B of spill,
// mostly outside the casts) beats 4 (121 VGPRs, none): sphere scene 9.92 ->
// 9.48 ms (profiles/r01_variants_bvh_occupancy.log); 6 spills in the
// traversal and loses (14.5 ms).
#ifndef IPT_MIN_BLOCKS_BVH_FWD
#define IPT_MIN_BLOCKS_BVH_FWD 5
#endif
template <int MODE, bool BVH>
constexpr int min_blocks() {
  return BVH ? (MODE == MODE_ADJU ? IPT_MIN_BLOCKS_BVH_ADJU
                                  : (is_adj<MODE>() ? IPT_MIN_BLOCKS_BVH_ADJ
                                                    : (is_fwd<MODE>() ? IPT_MIN_BLOCKS_BVH_FWD : IPT_MIN_BLOCKS_BVH)))
             : (is_fwd<MODE>() ? IPT_MIN_BLOCKS_FWD
                                : (MODE == MODE_ADJU   ? IPT_MIN_BLOCKS_ADJU
                                   : MODE == MODE_ADJW ? IPT_MIN_BLOCKS_ADJW
                                                       : (is_adj<MODE>() ? IPT_MIN_BLOCKS_ADJ : IPT_MIN_BLOCKS_GRAPH)));
}
// Rejected and removed (round 3; the A/B logs under profiles/ keep the
// evidence): a traversal-server wave per workgroup fed through an LDS ray
// queue (r01_bvh_server.log: 21.0 vs 13.3 ms), the one-lane-per-ray binary
// traversal (r01_variants_coop_notrav.log), the per-lane backward sweep
// (r02_variants_adj_knobs_final.log: 7% slower), recorded prefix throughputs
// (r02_variants_adj_sweep.log), quantised wide nodes (r02_variants_qnodes.log),
// the forward's camera-ray ring (r02_variants_occupancy_after_cull.log), the
// shadow target tested with its pair partner (r02_variants_shadow_target_pair.log)
// the tolerance-mode fast cast (r02_variants_fastcast.log: fails the
// 1e-3 gradient bar), a per-wave LDS queue that parked the forward's path
// rays with their path state until a full cooperative round of 8 was waiting
// (r03/variants_queue_chsweep_r03f.log: north-star forward 4.70 vs 3.75 ms;
// r03/variants_r03e.log for the first form, 4.30 ms) and a channel-split
// adjoint sweep, lane 3i + c walking path i in channel c (same log: C2
// adjoint 2.33 vs 2.16 ms, north-star 6.57 vs 5.02 ms at one wave less);
// round 5: the four waves of a workgroup pooling their tree rays in an LDS
// queue and sharing out full rounds of 8 (two barriers per cast, the waves in
// step): north-star forward 3.71 -> 4.25 ms, unbounded adjoint 8.06 -> 13.6 --
// the lockstep waits cost more than the fuller rounds save
// (profiles/r05/variants_coop_wg_r05i.log, _r05j.log).
// Graph bins stay in LDS up to this size (KB), else global fp64 atomics.
#ifndef IPT_GRAPH_LDS_KB
#define IPT_GRAPH_LDS_KB 64
#endif
// Work enumeration of the adjoint and graph integrators.  Round 1 chose
// sample-major (a wave's 64 lanes trace 64 different pixels, so the LDS
// atomics of a vertex step hit different bins and few lanes need the BVH tree
// at once: C2 adjoint 3.29 -> 3.24 ms, sphere 23.8 -> 16.3 ms,
// profiles/r01_variants_adj_sample_major.log).  Since the culled casts and the
// wave-parallel sweep, pixel-major is the faster adjoint (a wave's coherent
// rays skip more pair blocks; C2 1.747 -> 1.734 ms, scenes/0 unbounded
// 3.554 -> 3.502, north star 3.905 -> 3.835, profiles/r06/variants_adj_enumeration_r06t.log)
// and each pixel's adjoint value is fetched by one chunk, i.e. one XCD's L2
// (DESIGN.md §12.10).  IPT_ADJ_PIXEL_MAJOR / IPT_GRAPH_PIXEL_MAJOR select it.
#ifndef IPT_ADJ_PIXEL_MAJOR
#define IPT_ADJ_PIXEL_MAJOR 1
#endif
#ifndef IPT_GRAPH_PIXEL_MAJOR
#define IPT_GRAPH_PIXEL_MAJOR 1
#endif
#define IPT_TRACE_BOUNDS __attribute__((amdgpu_flat_work_group_size(1, kBlock), amdgpu_waves_per_eu(min_blocks<MODE, BVH>() ? min_blocks<MODE, BVH>() : 1)))
// Profiling-only build (make variant DEFS=-DIPT_PHASE_TIMING): each wave
// accumulates s_memtime cycles per phase of the loop; read with
// ipt_debug_phase_cycles (tools/phase_timing.py).
#ifdef IPT_PHASE_TIMING
constexpr int kPhaseWords = 26;
__device__ unsigned long long g_phase_cycles[kPhaseWords];
// [8], [9]: the tree (coop_cast) part of phases 1 and 3 (BVH scenes);
// [10..21]: per phase, the lanes that take part summed over the wave
// iterations that run it, and those iterations (PHASE_LANES): refill,
// shade, shadow cast, emitter term, finalise, adjoint sweep rounds (valid
// tasks per round); [22] the sweep's chain steps (wave-level), [23] the
// rounds that run a chain, [24] the lanes' own chain steps summed (the
// useful part of [22] x 64); the path cast's lanes are [7]
#define PHASE_LANES(i, cond)                             \
  {                                                      \
    const uint64_t b_ = __ballot(cond);                  \
    if (b_) {                                            \
      tacc[i] += (uint64_t)__popcll(b_);                 \
      tacc[(i) + 1] += 1;                                \
    }                                                    \
  }
#define SUBPHASE_BEGIN const uint64_t ts_ = __builtin_amdgcn_s_memtime();
#define SUBPHASE_END(i) tacc[i] += __builtin_amdgcn_s_memtime() - ts_;
#define PHASE(i)                                     \
  {                                                  \
    const uint64_t tn_ = __builtin_amdgcn_s_memtime(); \
    tacc[i] += tn_ - tp_;                            \
    tp_ = tn_;                                       \
  }
#else
#define PHASE(i)
#define SUBPHASE_BEGIN
#define SUBPHASE_END(i)
#define PHASE_LANES(i, cond)
#endif

// Path ray of the brute-force scenes: the unrolled pair loop with plane
// offsets from LDS (nT <= 2 * kSmallPairs), else the packed pair loop.
__device__ __forceinline__ int cast_bf(const TriPair *__restrict__ pairs, const f2 *e3, int nT, V3 p, V3 d, float &t) {
  if (e3) return closest_hit_pairs_small(pairs, e3, nT, p, d, t);
  return closest_hit_pairs(pairs, nT, p, d, t);
}

// Entry i of the small-scene LDS table (kE3Floats per pair): the three
// edge-plane offsets of the pair as (A, B) float pairs.
__device__ __forceinline__ float small_table_entry(const TriPair *__restrict__ pairs, int i) {
  const int j = i / kE3Floats, k = i % kE3Floats, h = k & 1;
  return pairs[j].f[9 + 4 * (k >> 1)][h];
}

// LDS carve-out of the BVH instances (16-B aligned): wide nodes, large-pair
// copies, emitter records, group stacks.
__host__ __device__ inline size_t bvh_lds_offset(size_t base) { return (base + 15) & ~(size_t)15; }
// Bytes of the culled path pre-pass's LDS copy of the large pairs (16-B
// aligned, 36 floats per pair) and their original indices (2 ints per pair).
// The emitters' TriIsect records for the BVH shadow target test (nE <= 16).
constexpr int kEmitLdsMax = 16;
__host__ __device__ inline size_t emit_lds_bytes(int nE) {
  return nE > 0 && nE <= kEmitLdsMax ? (size_t)nE * sizeof(TriIsect) : 0;
}
__host__ __device__ inline size_t big_lds_bytes(int nbig) {
  return IPT_PATH_CULL && nbig > 0 ? 12 + (size_t)nbig * (sizeof(TriPair) + 2 * sizeof(int32_t)) : 0;
}
// Fill that copy at `at` (rounded up to 16 B from the LDS base); returns the
// first float after it.
__device__ __forceinline__ float *big_lds_copy(const TraceArgs &a, float *at, float *base, int tid, int nthr,
                                               BvhView &bv) {
  if (!(IPT_PATH_CULL && a.bvh_nbig > 0 && a.bvh_big_lds)) return at;
  float *pl = at + ((4 - (int)((at - base) & 3)) & 3);
  const float *g = reinterpret_cast<const float *>(a.bvh_big);
  for (int i = tid; i < 36 * a.bvh_nbig; i += nthr) pl[i] = g[i];
  int32_t *il = reinterpret_cast<int32_t *>(pl + 36 * a.bvh_nbig);
  for (int i = tid; i < 2 * a.bvh_nbig; i += nthr) il[i] = a.bvh_big_idx[i];
  bv.big_lds = pl;
  return at + big_lds_bytes(a.bvh_nbig) / sizeof(float);
}

// Wave-wide inclusive scans (GFX9 DPP: row_shr 1..8 inside each 16-lane
// row, then row_bcast:15 / row_bcast:31 carry the rows' totals; lanes a
// stage does not write add / max the identity 0).
// The adjoint sweep's task scan and owner search use them (an LDS scatter of
// owner markers + a max-scan) instead of six dependent ds_bpermute steps
// each: C2 adjoint 2.11 -> 2.05 ms, scenes/0 2.53 -> 2.47, north-star 4.96 ->
// 4.88 (profiles/r03/variants_ke_ring_r03n.log, `scan0`).
template <int CTRL, int ROW, int BANK>
__device__ __forceinline__ int dpp0(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROW, BANK, true);
}
__device__ __forceinline__ int wave_scan_add(int v) {
  int s = v + dpp0<0x111, 0xf, 0xf>(v);
  s += dpp0<0x112, 0xf, 0xf>(v);
  s += dpp0<0x113, 0xf, 0xf>(v);
  s += dpp0<0x114, 0xf, 0xe>(s);
  s += dpp0<0x118, 0xf, 0xc>(s);
  s += dpp0<0x142, 0xa, 0xf>(s);
  s += dpp0<0x143, 0xc, 0xf>(s);
  return s;
}
__device__ __forceinline__ uint32_t wave_scan_max(uint32_t v) {
  v = max(v, (uint32_t)dpp0<0x111, 0xf, 0xf>((int)v));
  v = max(v, (uint32_t)dpp0<0x112, 0xf, 0xf>((int)v));
  v = max(v, (uint32_t)dpp0<0x114, 0xf, 0xf>((int)v));
  v = max(v, (uint32_t)dpp0<0x118, 0xf, 0xf>((int)v));
  v = max(v, (uint32_t)dpp0<0x142, 0xa, 0xf>((int)v));
  v = max(v, (uint32_t)dpp0<0x143, 0xc, 0xf>((int)v));
  return v;
}

// TraceArgs is the kernel's FIRST parameter, so it sits at offset 0 of the
// kernarg segment -- the in-loop reload below depends on that (IPT_ARGS_RELOAD).
// The explicit arguments of trace_kernel as the kernarg segment holds them
// (in order, each at its natural alignment): karg() re-reads one of them at
// its point of use.  The adjoint's adj / grad pointers are used only by the
// sweep and the final flush; kept live across the loop they sit in SGPRs
// the pair loops need, and the compiler spills them to VGPR lanes and reloads
// them (v_readlane, VALU work) after every pair block.
struct TraceKernArgs {
  TraceArgs a;
  const TriIsect *isect;
  const TriPair *pairs;
  const TriGeom *geom;
  const TriMat *mat;
  const float *kd;
  const int *emit_tri;
  const float *emit_cdf;
  const float *emit_pmf;
  float *out_samples;
  const float *adj;
  double *grad;
  const uint8_t *target;
  double *edges;
};
static_assert(offsetof(TraceKernArgs, isect) == sizeof(TraceArgs), "pointers follow TraceArgs");
template <typename T>
__device__ __forceinline__ T karg(size_t off) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef __attribute__((address_space(4))) const char cst_char;
  typedef __attribute__((address_space(4))) const T cst_t;
  const cst_char *k = (const cst_char *)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(k));  // read here, not hoisted to the kernel's entry
  return *(const cst_t *)(k + off);
#else
  (void)off;
  return T();
#endif
}
template <int MODE, bool SPEC, bool BVH>
__global__ IPT_TRACE_BOUNDS void trace_kernel(
    const TraceArgs a, const TriIsect *__restrict__ isect, const TriPair *__restrict__ pairs,
    const TriGeom *__restrict__ geom, const TriMat *__restrict__ mat, const float *__restrict__ kd,
    const int *__restrict__ emit_tri, const float *__restrict__ emit_cdf, const float *__restrict__ emit_pmf,
    float *__restrict__ out_samples, const float *__restrict__ adj, double *__restrict__ grad,
    const uint8_t *__restrict__ target, double *__restrict__ edges) {
  extern __shared__ double lds[];
  const int tid = threadIdx.x;
  // scene batch: this workgroup's material set and its place among the set's blocks
  const int set = a.nscenes > 1 ? (int)(blockIdx.x % (uint32_t)a.nscenes) : 0;
  const uint32_t sblock = a.nscenes > 1 ? blockIdx.x / (uint32_t)a.nscenes : blockIdx.x;
  const uint32_t sgrid = a.nscenes > 1 ? (uint32_t)a.bps : gridDim.x;
  const uint64_t seed = a.seed + (uint64_t)set * a.seed_stride;
  if (a.nscenes > 1) {
    kd += (size_t)set * 3 * a.nT;
    if (is_fwd<MODE>()) out_samples += (size_t)set * a.out_stride;
    // (adj, grad: karg() at their uses, offset there)
  }
  const float *kdpi_g = a.kdpi_g ? a.kdpi_g + (size_t)set * 3 * a.nT : nullptr;
  constexpr int nthr = kBlock;
  const int nT = a.nT, nE = a.nE;
  const int vmax = a.rec_cap;  // ADJ record capacity per lane (ADJU: ring slots)
  // LDS: [fp64 accumulators][kd table][kd/pi table][ADJ vertex records]
  double *lds_acc = lds;               // ADJ: nT*3 grad; GRAPH: (nT+1)*nT*kEdgeW bins
  int n_acc = 0;
  if (is_adj<MODE>()) {
    n_acc = a.grad_slots * 3;
  } else if (MODE == MODE_GRAPH && a.lds_edges) {
    n_acc = (int)graph_lds_doubles(nT, nE);
  }
  // Per-triangle kd and kd/pi (the latter is BSDF's indirect `diffuse /=
  // M_PI`, path_trace.cu:15-17): computed once per workgroup with the same
  // IEEE division the per-vertex code would do, instead of three divisions
  // per vertex.  Falls back to global memory for large scenes.
  float *tab = reinterpret_cast<float *>(lds + n_acc);
  if (a.kd_tables) {
    for (int i = tid; i < 3 * nT; i += nthr) {
      const float v = kd[i];
      tab[i] = v;
      tab[3 * nT + i] = v / kPiF;
    }
  }
  // kd and kd/pi of triangle t, from the tables or from global memory by a
  // wave-uniform branch (a pointer that may point at either compiles to flat
  // loads: vector-memory latency and a vmcnt+lgkmcnt wait for LDS data)
  const lds_f32 *tab_l = (const lds_f32 *)tab;
  const gbl_f32 *kd_g = (const gbl_f32 *)kd;
  auto kd3 = [&](int t) -> V3 {
    if (a.kd_tables) return mk(tab_l[3 * t], tab_l[3 * t + 1], tab_l[3 * t + 2]);
    return mk(kd_g[3 * t], kd_g[3 * t + 1], kd_g[3 * t + 2]);
  };
  auto ke3 = [&](int t) -> V3 {  // TriMat::ke
    const gbl_f32 *q = (const gbl_f32 *)mat + (size_t)t * (sizeof(TriMat) / sizeof(float)) + offsetof(TriMat, ke) / sizeof(float);
    return mk(q[0], q[1], q[2]);
  };
  auto kdpi3 = [&](int t) -> V3 {
    if (a.kd_tables) return mk(tab_l[3 * nT + 3 * t], tab_l[3 * nT + 3 * t + 1], tab_l[3 * nT + 3 * t + 2]);
    const gbl_f32 *q = (const gbl_f32 *)kdpi_g + 3 * t;
    return mk(q[0], q[1], q[2]);
  };
  // edge-plane offsets of each triangle pair for the unrolled small-scene
  // closest-hit loop (ipt_device.h::closest_hit_pairs_small)
  const f2 *e3 = nullptr;
  float *lds_e3 = tab + (a.kd_tables ? 6 * nT : 0);
  const int nP = (nT + 1) >> 1;
  if (a.small_pairs) {
    for (int i = tid; i < kE3Floats * nP; i += nthr) lds_e3[i] = small_table_entry(pairs, i);
    e3 = reinterpret_cast<const f2 *>(lds_e3);
  }
  // small scenes: a copy of the TriIsect records (16-B aligned), read by the
  // culled shadow cast's per-lane target test from LDS instead of L2
  float *lds_is = lds_e3 + (a.small_pairs ? kE3Floats * nP : 0);
  lds_is += (4 - (int)((lds_is - reinterpret_cast<float *>(lds)) & 3)) & 3;
  if (a.small_pairs) {
    const float *g = reinterpret_cast<const float *>(isect);
    for (int i = tid; i < 20 * nT; i += nthr) lds_is[i] = g[i];
  }
  // small scenes, culled path cast (IPT_PATH_CULL): a copy of the TriPair
  // records (16-B aligned after the TriIsect copy), gathered per lane
  float *lds_pr = lds_is + (a.small_pairs ? 20 * nT : 0);
  if (a.small_pairs && IPT_PATH_CULL) {
    const float *g = reinterpret_cast<const float *>(pairs);
    for (int i = tid; i < 36 * nP; i += nthr) lds_pr[i] = g[i];
  }
  // ... and the shadow casts' potential-occluder masks (IPT_SHADOW_PO)
  uint32_t *lds_po = reinterpret_cast<uint32_t *>(lds_pr + (a.small_pairs && IPT_PATH_CULL ? 36 * nP : 0));
  const bool po = a.small_pairs && IPT_SHADOW_PO && a.pomask;
  if (po)
    for (int i = tid; i < nT * nE; i += nthr) lds_po[i] = a.pomask[i];
  float *lds_rec = a.small_pairs ? reinterpret_cast<float *>(lds_po) + (po ? nT * nE : 0) : lds_e3;
  // MODE_ADJ: one word per lane (the sweep's owner markers) in front of the
  // vertex records
  if (is_adj<MODE>()) lds_rec += kBlock;
  BvhView bv;
  bv.isect = isect;
  bv.big = nullptr;
  bv.big_idx = nullptr;
  bv.big_e3 = nullptr;
  bv.nbig = 0;
  bv.big_boxes = nullptr;
  bv.big_lds = nullptr;
  bv.emit_is = nullptr;
  // BVH forward (5 waves/SIMD, 96 VGPRs): the lane's work item, the triangle
  // its path ray leaves and its first emission Le live in LDS ([6][kBlock]
  // words: item lo, hi, source, Le xyz) instead of registers -- each is
  // touched a few times per path, and in registers the allocator spilled them
  // (and more) to scratch inside the loop
  // The 6-wave adjoint (MODE_ADJW, 80 VGPRs) likewise keeps its work item
  // and Le there (its path source is not needed): in registers they pushed
  // the culled path cast past 80 VGPRs and a ray-direction pair was reloaded
  // from scratch in every pair block (16 B/lane of scratch; IPT_ADJW_LANE_LDS)
  constexpr bool kLaneLds = (BVH && is_fwd<MODE>()) || (!BVH && MODE == MODE_ADJW && IPT_ADJW_LANE_LDS);
  lds_u32 *lane_ws = nullptr;
  if (!BVH && kLaneLds)  // after the vertex records ([6][kBlock] words, as the BVH forward's)
    lane_ws = (lds_u32 *)(lds_rec + (size_t)vmax * kRecFieldsDiffuse * kBlock);
  CoopView cv;
  cv.wn = nullptr;
  cv.wn_lds = false;
  cv.wt = a.bvh_wtris;
  cv.stk = nullptr;
  cv.stride = a.coop_stride;
  for (int k = 0; k < 6; ++k) cv.root[k] = a.root_box[k];
  for (int k = 0; k < 4; ++k) cv.sphere[k] = a.tree_sphere[k];
  if (BVH) {
    const size_t rec_words = is_badj<MODE>()    ? (size_t)vmax * (SPEC ? kRecFieldsSpec : kRecFieldsDiffuse) * kBlock
                             : MODE == MODE_ADJU ? (size_t)a.rec_lds * (SPEC ? kRecFieldsSpec : kRecFieldsDiffuse) * kBlock
                                                 : 0;
    char *base = reinterpret_cast<char *>(lds);
    const size_t off = bvh_lds_offset((size_t)(reinterpret_cast<char *>(lds_rec + rec_words) - base));
    float4 *lw = reinterpret_cast<float4 *>(base + off);
    cv.wn = a.bvh_wide;
    if (a.bvh_wide_lds > 0) {
      for (int i = tid; i < kWideF4 * a.bvh_wide_lds; i += nthr) lw[i] = a.bvh_wide[i];
      cv.wn = lw;
      cv.wn_lds = true;
    }
    float *be3 = reinterpret_cast<float *>(lw + kWideF4 * a.bvh_wide_lds);
    for (int i = tid; i < 6 * a.bvh_nbig; i += nthr) {
      const int j = i / 6, kf = (i % 6) >> 1, h = i & 1;
      be3[i] = a.bvh_big[j].f[9 + 4 * kf][h];
    }
    bv.big = a.bvh_big;
    bv.big_idx = a.bvh_big_idx;
    bv.big_boxes = a.bvh_big_boxes;
    bv.big_e3 = reinterpret_cast<const f2 *>(be3);
    bv.nbig = a.bvh_nbig;
    float *after = big_lds_copy(a, be3 + 6 * a.bvh_nbig, reinterpret_cast<float *>(lds), tid, nthr, bv);
    if (emit_lds_bytes(nE)) {
      for (int i = tid; i < 20 * nE; i += nthr) after[i] = reinterpret_cast<const float *>(isect)[20 * emit_tri[i / 20] + i % 20];
      bv.emit_is = after;
      after += 20 * nE;
    }
    cv.stk = reinterpret_cast<uint32_t *>(after) + (tid >> 6) * 8 * a.coop_stride;
    if (kLaneLds) lane_ws = (lds_u32 *)(reinterpret_cast<uint32_t *>(after) + (kBlock / 64) * 8 * a.coop_stride);
  }
  for (int i = tid; i < n_acc; i += nthr) lds_acc[i] = 0.0;
  __syncthreads();
  // fp64 bin updates go to LDS (ds_add_f64) or to global memory by a
  // wave-uniform (GRAPH) or per-lane (ADJ hot set) branch -- never through
  // one pointer that may be either: that compiles to flat atomics, which take
  // the vector-memory path even when the address is in LDS.
  // The pointers carry their address space in the type so that LLVM cannot
  // merge the two branches' atomics back into one through a selected pointer.
  auto bins_add = [&](bool in_lds, double *glob, size_t off, int n, const double *v) {
    if (in_lds) {
      lds_f64 *b = (lds_f64 *)lds_acc + off;
      for (int i = 0; i < n; ++i) __hip_atomic_fetch_add(b + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
      gbl_f64 *b = (gbl_f64 *)glob + off;
      for (int i = 0; i < n; ++i) __hip_atomic_fetch_add(b + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };

  // MODE_ADJU: the ring's global slots (TraceArgs::grec): this wave's pool of
  // pool_chunks chunks, [chunk][slot][field], a record's fields contiguous --
  // one 12-B store per vertex, and a sweep round reads an owner's consecutive
  // records as contiguous runs.  Round 4's first form, [field][slot][lane],
  // stored 4 B per field at a different place per lane: three write requests
  // per vertex, 767 MB written per C3 launch, profiles/r04/unbounded_pmc_r04l.txt)
  gbl_f32 *upool = nullptr;  // this wave's chunk pool ([chunk][slot][field])
  if (MODE == MODE_ADJU)
    upool = (gbl_f32 *)a.grec + ((size_t)blockIdx.x * (kBlock / 64) + (tid >> 6)) * a.grec_stride;
  gbl_f32 *umr = nullptr;  // this lane's captured prefix throughputs (IPT_ADJU_SUB), entry e at umr + e * 192
  if (MODE == MODE_ADJU && kSub > 0)
    umr = (gbl_f32 *)a.mring + ((size_t)blockIdx.x * (kBlock / 64) + (tid >> 6)) * (kMrEnt * 64 * 3) + (tid & 63) * 3;
  {  // the wave's persistent loop
  // wave-uniform sample range (static partition, regenerated per lane)
  const uint32_t wave = __builtin_amdgcn_readfirstlane((sblock * kBlock + tid) >> 6);
  const uint32_t nwaves = (sgrid * kBlock) >> 6;
  const TraceArgs &ar = a;
  // Work items w in [0, n_samples) of this launch (item_split): pixel-major
  // w = lp * spp + s, or sample-major w = s * npix + lp over the launch's
  // pixels lp.  Either way the sample's seed is seed + its global index g:
  // results do not depend on the enumeration or on the row partition.
  // Which wave traces which items only changes WHO computes a sample, never
  // its value.  Static ranges leave the launch's tail to the waves whose
  // pixels hold the longest paths; chunks taken from a per-launch counter
  // keep every wave busy to the end.
  const bool dyn = a.chunk != 0;
  uint64_t next, end;
  if (dyn) {
    chunk_range<kGuided<BVH>()>(ar, wave, ar.n_samples, next, end);
  } else {
    next = (ar.n_samples * wave) / nwaves;
    end = (ar.n_samples * (wave + 1)) / nwaves;
  }
  bool exhausted = !dyn;
  // fused pixel mean (MODE_FWDM), wave-uniform: the current group's first
  // launch-local pixel glp, pixel count gnp and slots gslots (4 bits per
  // pixel), fj = its samples issued so far (item j = sample j / gnp of pixel
  // glp + j % gnp: sample-major inside the group); sfree / sdone = the ring's
  // free slots / slots whose samples are all in but not yet summed.  A slot
  // is held by ONE pixel, so a long path keeps one pixel's slot, not a whole
  // chunk's: the ring also serves unbounded paths.
  uint32_t glp = 0, gnp = 0, gslots = 0, fj = 0, sdone = 0;
  uint64_t pl0 = 0, pl1 = 0;  // the grabbed chunk's pixels not yet in a group
  uint32_t sfree = MODE == MODE_FWDM ? (a.nslots >= 32 ? ~0u : (1u << a.nslots) - 1u) : 0u;
  bool started = false;

  bool active = false;
  Rng st;
  V3 p = mk(0.f, 0.f, 0.f), d = p;
  V3 L = p, Le_r = p, Ld = p, M = mk(1.f, 1.f, 1.f);
  // Le: the path's first emission (kLaneLds: in LDS words 3..5 of lane_ws)
  auto set_le = [&](V3 v) {
    if (kLaneLds) {
      ((lds_f32 *)lane_ws)[3 * kBlock + tid] = v.x;
      ((lds_f32 *)lane_ws)[4 * kBlock + tid] = v.y;
      ((lds_f32 *)lane_ws)[5 * kBlock + tid] = v.z;
    } else {
      Le_r = v;
    }
  };
  auto le = [&]() -> V3 {
    if (kLaneLds)
      return mk(((lds_f32 *)lane_ws)[3 * kBlock + tid], ((lds_f32 *)lane_ws)[4 * kBlock + tid],
                ((lds_f32 *)lane_ws)[5 * kBlock + tid]);
    return Le_r;
  };
  // ADJU (unbounded adjoint): suffix carried from the chunk after, replay
  // target (0 = first pass), next ring slot
  // and the prefix throughput at the chunk's first vertex (1 for a chunk
  // starting at vertex 0; captured while a replay passes its start)
  V3 Scar = mk(0.f, 0.f, 0.f), Mlo = mk(1.f, 1.f, 1.f);
  int rhi = 0, rslot = 0;
  // IPT_ADJU_SUB: the end of the sub-chunk this lane sweeps next (0: none);
  // such a lane is neither traced nor refilled until its chunk is swept
  int usub = 0;
  auto pending = [&]() { return MODE == MODE_ADJU && kSub > 0 && usub > 0; };
  // ADJU: the pool chunks this path holds and its ring size, in one word --
  // bits 6j..6j+5: the id of its chunk j (63: none), 24-29: the ring size
  // (a.rec_cap unless the pool ran dry) -- and the wave's free chunks
  constexpr uint32_t kNoChunks = 0x00ffffffu;
  uint32_t ctab = kNoChunks | ((uint32_t)vmax << 24);
  uint64_t pfree = MODE == MODE_ADJU ? (a.pool_chunks >= 64 ? ~0ull : (1ull << a.pool_chunks) - 1ull) : 0ull;
  auto vcap_of = [&]() { return (int)(ctab >> 24); };
  float weight = 1.f;  // GRAPH path weight
  V3 pix = p;          // GRAPH target pixel
  int k = 0, dst = 0;
  int ptri_r = -1;       // BVH: the triangle the path ray leaves (tree_skip), -1 = camera ray
  uint64_t witem_r = 0;  // this lane's work item (output slot / pixel source)
  auto set_item = [&](uint64_t w) {
    if (kLaneLds) {
      lane_ws[tid] = (uint32_t)w;
      lane_ws[kBlock + tid] = (uint32_t)(w >> 32);
    } else {
      witem_r = w;
    }
  };
  auto witem = [&]() -> uint64_t {
    if (kLaneLds) return (uint64_t)lane_ws[tid] | ((uint64_t)lane_ws[kBlock + tid] << 32);
    return witem_r;
  };
  auto set_ptri = [&](int t) {  // (read by the BVH instances' tree_skip only)
    if (!BVH) return;
    if (kLaneLds) lane_ws[2 * kBlock + tid] = (uint32_t)t;
    else ptri_r = t;
  };
  auto ptri = [&]() -> int { return kLaneLds ? (int)lane_ws[2 * kBlock + tid] : ptri_r; };
  // One iteration = one path vertex for the whole wave, in two
  // wave-synchronous phases: (1) every active lane casts its path ray and,
  // on a hit, shades the vertex and draws ALL of the vertex's random numbers
  // in the reference's order (NEE: emitter, r1, r2; then RR; then phi,
  // theta); (2) the lanes that need one cast their next-event shadow ray;
  // then every vertex lane finalises (L, M, records, next ray).  Each shading
  // block thus runs once per vertex with most lanes on, instead of path and
  // shadow lanes serialising each other's code every iteration.
#ifdef IPT_PHASE_TIMING
  uint64_t tacc[kPhaseWords] = {};
  uint64_t tp_ = __builtin_amdgcn_s_memtime();
#endif
  const int lane = tid & 63;
  // MODE_FWDM: this wave's slot table ([nslots] unfinished counts, [nslots]
  // pixels, padded to 16 B) and slots ([channel][sample] floats each)
  auto fused_tab = [&](const TraceArgs &A) -> lds_u32 * {
    return (lds_u32 *)(reinterpret_cast<char *>(lds) + A.mean_off) + (size_t)(tid >> 6) * A.mean_wstride;
  };
  auto fused_slots = [&](const TraceArgs &A) -> lds_f32 * {
    return (lds_f32 *)(fused_tab(A) + ((2 * A.nslots + 3) & ~3));
  };
  // Sum the slots of `mask` (wave-uniform, <= 16 of them): lanes 3i + c take
  // the i-th slot's channel c and add v_s / spp over s = 0 .. spp-1 in sample
  // order -- toneMap's operations (path_trace.cu:186-198), i.e.
  // pixel_mean_sm_kernel's -- then write the HDR (and 8-bit) pixel.
  auto fused_sum = [&](const TraceArgs &A, uint32_t mask) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the slots' sample writes before the sums
    __builtin_amdgcn_wave_barrier();
    const int m = __popc(mask);
    const int kq = (lane * 43) >> 7, ch = lane - 3 * kq;  // lane / 3 for lane < 64
    int slot = 0;
    uint32_t mm = mask;
    for (int i = 0; i < m; ++i) {  // wave-uniform: this lane's slot = the kq-th set bit
      const int b = __builtin_ctz(mm);
      mm &= mm - 1u;
      slot = kq == i ? b : slot;
    }
    if (lane < 3 * m) {
      const int spp = A.spp;
      const lds_f32 *v = fused_slots(A) + (size_t)(3 * slot + ch) * spp;
      float acc = 0.f;
      if (A.rc_spp != 0.f && (spp & 3) == 0) {  // x * (1/spp) == x / spp (power of two); 16-B reads
        const float rc = A.rc_spp;
        for (int s = 0; s < spp; s += 4) {
          const v4f w4 = *(const lds_v4 *)(v + s);
          acc += w4.x * rc;
          acc += w4.y * rc;
          acc += w4.z * rc;
          acc += w4.w * rc;
        }
      } else {
        const float fs = (float)spp;
        for (int s = 0; s < spp; ++s) acc += v[s] / fs;
      }
      const uint64_t px = fused_tab(A)[A.nslots + slot];
      out_samples[px * 3 + ch] = acc;
      if (A.ldr) A.ldr[(size_t)set * A.out_stride + px * 3 + ch] = (uint8_t)(255.f * acc / (1 + acc));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the sums' reads before the slots are refilled
    __builtin_amdgcn_wave_barrier();
  };
  for (;;) {
#if defined(__HIP_DEVICE_COMPILE__)  // (the host pass has no AS4 copy)
    // The launch arguments, re-read from the kernarg segment every iteration
    // through a pointer the compiler cannot see through: left alone it keeps
    // the loop-invariant fields (camera, divisors, pointers) in SGPRs for
    // the whole loop, runs out of them and spills them to VGPR lanes, paying
    // a v_readlane (a VALU instruction) at every use.  Scalar loads hit the
    // constant cache.  This `a` shadows the parameter inside the loop.
    typedef __attribute__((address_space(4))) const TraceArgs cst_args;
    const cst_args *apc = (const cst_args *)__builtin_amdgcn_kernarg_segment_ptr();  // first parameter: offset 0
    asm volatile("" : "+s"(apc));
    TraceArgs a = *apc;
#else
    TraceArgs a = ar;
#endif
    if (MODE == MODE_FWDM) {
      const uint32_t G = a.group;  // pixels per group (a chunk's last group may hold fewer)
      const bool issued = fj >= gnp * (uint32_t)a.spp;
      // sum the finished slots when a group's worth is waiting, when the next
      // group lacks free slots, or -- once the launch's work is handed out --
      // right away (lazily: one pass sums up to 16 pixels, 3 lanes each)
      if (sdone && ((uint32_t)__popc(sdone) >= G || exhausted || (issued && (uint32_t)__popc(sfree) < G))) {
        fused_sum(a, sdone);
        sfree |= sdone;
        sdone = 0;
      }
      // the next group of pixels (from the chunk in hand, else the wave's own
      // chunk, then the counter's) once the current one is fully issued and
      // G slots are free
      if (issued && !exhausted && (uint32_t)__popc(sfree) >= G) {
        if (pl0 >= pl1) {
          bool own = false;
          if (!started) {
            started = true;
            chunk_range<kGuided<BVH>()>(a, wave, a.npix, pl0, pl1);
            own = pl0 < a.npix;
          }
          if (!own) {
            uint32_t c = 0;
            if (lane == 0) c = atomicAdd(a.chunk_ctr + (size_t)set * kCtrStride, 1u);
            c = (uint32_t)__builtin_amdgcn_readfirstlane((int)c);  // lane 0 (full exec here)
            chunk_range<kGuided<BVH>()>(a, nwaves + c, a.npix, pl0, pl1);
            if (pl0 >= a.npix && lane == 0) grab_failed(a.chunk_ctr + (size_t)set * kCtrStride, c, a.grabs);
          }
        }
        if (pl0 < a.npix) {
          glp = (uint32_t)pl0;
          gnp = (uint32_t)(pl1 - pl0 < G ? pl1 - pl0 : G);
          pl0 += gnp;
          fj = 0;
          gslots = 0;
          uint32_t mm = sfree;
          for (uint32_t q = 0; q < gnp; ++q) {  // the lowest free slots, 4 bits per pixel
            gslots |= (uint32_t)__builtin_ctz(mm) << (4 * q);
            mm &= mm - 1u;
          }
          sfree = mm;
          if ((uint32_t)lane < gnp) {  // slot table: unfinished samples, pixel
            lds_u32 *tab = fused_tab(a);
            const uint32_t sl = (gslots >> (4 * lane)) & 15u;
            tab[sl] = (uint32_t)a.spp;
            tab[a.nslots + sl] = glp + (uint32_t)lane;
          }
        } else {
          exhausted = true;
        }
      }
    } else if (next >= end && !exhausted) {  // wave-uniform: the next chunk (full exec here)
      // One counter, grabbed when needed.  Measured against alternatives
      // (profiles/r02_variants_chunk_*.log): 8 counters on separate lines
      // with stealing and a grab prefetched one chunk ahead were both slower
      // (and round 6's XCD bands).
      uint32_t c = 0;
      if (lane == 0) c = atomicAdd(a.chunk_ctr + (size_t)set * kCtrStride, 1u);
      c = (uint32_t)__shfl((int)c, 0);
      uint64_t start, stop;
      chunk_range<kGuided<BVH>()>(a, nwaves + c, a.n_samples, start, stop);
      if (start < a.n_samples) {
        next = start;
        end = stop;
      } else {
        exhausted = true;
        if (lane == 0) grab_failed(a.chunk_ctr + (size_t)set * kCtrStride, c, a.grabs);
      }
    }
    // ---- refill finished lanes from the wave's range (ballot + mbcnt)
    const bool wants = !active && !pending();
    const uint64_t need = __ballot(wants);
#ifdef IPT_PHASE_TIMING
    const uint64_t act0_ = ~need;
#endif
    if (MODE == MODE_FWDM) {
      const uint32_t fn = gnp * (uint32_t)a.spp;
      if (need && fj < fn) {
        const uint32_t rank =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
        if (!active && fj + rank < fn) {
          const uint32_t j = fj + rank;
          const uint32_t s = (gnp & (gnp - 1u)) == 0u ? j >> __builtin_ctz(gnp) : j / gnp;
          const uint32_t q = j - s * gnp;
          int r, c;
          item_ray_ls(a, seed, glp + q, s, st, p, d, r, c);
          // the sample's LDS place: its pixel's slot, sample s
          set_item((uint64_t)((gslots >> (4 * q)) & 15u) | ((uint64_t)s << 4));
          L = mk(0.f, 0.f, 0.f);
          set_le(L);
          Ld = L;
          M = mk(1.f, 1.f, 1.f);
          k = 0;
          set_ptri(-1);
          active = true;
        }
        fj += (uint32_t)__popcll(need);
        fj = fj < fn ? fj : fn;
      }
    } else if (need) {
      const uint32_t rank =
          __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
      if (wants) {
        const uint64_t w = next + rank;
        if (w < end) {
          set_item(w);
          int r, c;
          item_ray(a, seed, w, st, p, d, r, c);
          L = mk(0.f, 0.f, 0.f);
          set_le(L);
          Ld = L;
          M = mk(1.f, 1.f, 1.f);
          k = 0;
          set_ptri(-1);
          if (MODE == MODE_ADJU) {
            rhi = 0;
            rslot = 0;
            if (!kSub) Mlo = mk(1.f, 1.f, 1.f);
            ctab = kNoChunks | ((uint32_t)vmax << 24);
          }
          if (MODE == MODE_GRAPH) {
            weight = 1.f;
            dst = nT;
            const uint8_t *px = target + ((size_t)r * a.W + c) * 3;
            pix = mk((float)px[0] / 255.0f, (float)px[1] / 255.0f, (float)px[2] / 255.0f);
          }
          active = true;
        }
      }
      next += (uint64_t)__popcll(need);
    }
    PHASE(0)
    PHASE_LANES(10, active && !((act0_ >> (tid & 63)) & 1ull))
    // (MODE_FWDM: the last finished slots are summed at the loop top first)
    if (__ballot(active || pending()) == 0 &&
        (MODE != MODE_FWDM || (exhausted && sdone == 0 && fj >= gnp * (uint32_t)a.spp)))
      break;
#ifdef IPT_PHASE_TIMING
    tacc[6] += 1;
    tacc[7] += __popcll(__ballot(active));
#endif

    // ================= phase 1: path ray (radiance, path_trace.cu:111-144)
    float t = 0.f;
    int hit = -1;
    if (BVH) {  // pre-pass per lane, the tree part by 8-lane groups
      bool qn = false;
      if (active) {
        bvh_prepass<false>(bv, p, d, t, hit, -1);
        qn = coop_root_test(cv, p, d, t) && !(IPT_TREE_SKIP && tree_skip(a.src_cull, ptri(), d));
      }
      SUBPHASE_BEGIN
      coop_cast<false>(cv, qn, p, d, t, hit);
      SUBPHASE_END(8)
    } else if (active) {
      if (IPT_PATH_CULL && e3)
        hit = closest_hit_pairs_culled((const lds_f32 *)lds_pr, a.pboxes, nT, p, d, t);
      else
        hit = cast_bf(pairs, e3, nT, p, d, t);
    }
    PHASE(1)
    const bool vertex = active && hit >= 0;
    bool finished = false, escaped = false;
    if (active && hit < 0) {  // miss: the stale L_e/L_d are re-added (F4)
      finished = true;
      escaped = (k > 0);
      if (MODE != MODE_GRAPH) {
        const V3 Le = le();
        L = mk(fmaf(M.x, Le.x + Ld.x, L.x), fmaf(M.y, Le.y + Ld.y, L.y), fmaf(M.z, Le.z + Ld.z, L.z));
      }
    }
    const int tri = hit;
    V3 nh = p, din = d, sd = d, nd = d;
    bool shadow = false, cont = false;
    int emitter = 0;
    float ct = 0.f, coeff = 0.f, speci = 0.f, specd = 0.f;
    if (vertex) {
      const V3 q = along(p, d, t);
      if (MODE == MODE_GRAPH) {
        (void)uniform(st);  // isSpecular = u < P_SPEC(0), inv_path_trace.cu:117
        const float wf = weight * 1.f;  // Edge::update, inv_scene.h:26-36
        const double v[5] = {(double)weight, (double)wf, (double)(wf * pix.x), (double)(wf * pix.y),
                             (double)(wf * pix.z)};
        const size_t bin = (size_t)dst * nT + tri;
        bins_add(a.lds_edges != 0, edges, a.lds_edges ? bin * kEdgeL : bin * kEdgeW, 5, v);
      } else if (k == 0) {
        set_le(ke3(tri));
      }
      nh = shading_normal(geom[tri], q);
      p = q;
      Ld = mk(0.f, 0.f, 0.f);
      if (nE > 0) {  // directLighting up to the shadow ray, path_trace.cu:30-71
        const float u = uniform(st);
        int ie = 0;
        while (ie < nE && !(emit_cdf[ie] >= u)) ++ie;
        ie = ie < nE ? ie : nE - 1;
        const float r1 = uniform(st), r2 = uniform(st);
        const double sq = dsqrt_core((double)r1);  // r1 >= 2^-33: sqrt's identity range
        const float ca = (float)(1.0 - sq);
        const float cb = (float)(sq * (double)(1.f - r2));
        const float cc = (float)((double)r2 * sq);
        const TriGeom &ge = geom[emit_tri[ie]];
        const V3 pt = mk(fmaf(cc, ge.v[2][0], fmaf(cb, ge.v[1][0], ca * ge.v[0][0])),
                         fmaf(cc, ge.v[2][1], fmaf(cb, ge.v[1][1], ca * ge.v[0][1])),
                         fmaf(cc, ge.v[2][2], fmaf(cb, ge.v[1][2], ca * ge.v[0][2])));
        sd = unit(sub(pt, q));
        ct = dot3(nh, sd);
        emitter = ie;
        shadow = !(ct < 0.f);
      }
      if (!(a.max_bounces >= 0 && k == a.max_bounces)) {
        const float pr = uniform(st);  // Russian roulette, path_trace.cu:130-131
        if (pr < kPRR) {                // sampleNextDir, path_trace.cu:91-109
          const TriMat &m = mat[tri];
          const bool spec = SPEC && (MODE != MODE_GRAPH) && (m.flags & MAT_SPECULAR);
          const float uphi = uniform(st);
          const float phi = (float)(2.0 * kPi * (double)uphi);
          const float ut = uniform(st);
          float cth, sth, psamp;
          if (!spec) {
            cth = sqrt_core(ut);  // == (float)sqrt((double)ut) (innocuous double rounding); ut >= 2^-33
            // sin(theta) = sqrt(1 - u) from the float 1 - u (rounds 1-6: from the
            // exact double 1 - u, 0.6% slower)
            const float omu = 1.0f - ut;  // 0 or >= 2^-24
            sth = omu > 0.f ? sqrt_core(omu) : 0.f;
            psamp = kInvPiF;
          } else {
            const double cd = pow_d((double)ut, 1.0 / ((double)m.shininess + 1.0));
            cth = (float)cd;
            sth = (float)sqrt(1.0 - cd * cd);
            psamp = pow_f((m.shininess + 1.f) * cth, m.shininess);
          }
          float sp, cp;
          sincos_f(phi, sp, cp);
          const V3 h = mk(sth * cp, sth * sp, cth);
          const TriGeom &g = geom[tri];
          nd = unit(mk(fmaf(g.R[0][2], h.z, fmaf(g.R[0][1], h.y, g.R[0][0] * h.x)),
                       fmaf(g.R[1][2], h.z, fmaf(g.R[1][1], h.y, g.R[1][0] * h.x)),
                       fmaf(g.R[2][2], h.z, fmaf(g.R[2][1], h.y, g.R[2][0] * h.x))));
          if (MODE != MODE_GRAPH) {
            if (SPEC && (m.flags & MAT_HAS_KS)) speci = phong(m.shininess, nh, din, nd);
            coeff = spec ? (dot3(nd, nh) / psamp) / kPRR : div_const<1>(div_const<0>(dot3(nd, nh)));  // psamp = kInvPiF
          }
          cont = true;
        }
      }
    }

    // ================= phase 2: next-event shadow ray (path_trace.cu:73-88)
    PHASE(2)
    PHASE_LANES(12, vertex)
    V3 lo = mk(0.f, 0.f, 0.f);
    float emit_s = 0.f;  // ADJ record: lo = Ke[emit_et] * emit_s
    int emit_et = 0;
    float ts = 0.f;
    int hs = -1;
    const int et = shadow ? emit_tri[emitter] : -1;
    if (__ballot(shadow)) {
      PHASE_LANES(14, shadow)
      if (BVH) {
        bool qn = false;
        if (shadow && bvh_prepass<true>(bv, p, sd, ts, hs, et,
                                        a.big_pomask ? a.big_pomask[tri * nE + emitter] : 0xffffffffu, emitter))
          qn = coop_root_test(cv, p, sd, ts) && !(IPT_TREE_SKIP && tree_skip(a.src_cull, tri, sd));
        SUBPHASE_BEGIN
        coop_cast<true>(cv, qn, p, sd, ts, hs);
        SUBPHASE_END(9)
      } else if (shadow) {
        if (IPT_SHADOW_CULL && e3)
          hs = shadow_hit_pairs_small((const lds_f32 *)lds_is, pairs, a.pboxes, e3, nT, p, sd, et, ts,
                                      po ? ((const lds_u32c *)lds_po)[tri * nE + emitter] : 0xffffffffu);
        else
          hs = cast_bf(pairs, e3, nT, p, sd, ts);
      }
      PHASE(3)
      if (shadow && hs == et) {  // must hit the sampled emitter itself
        const V3 ne = shading_normal(geom[et], along(p, sd, ts));
        const float ctp = -dot3(ne, sd);
        if (!(ctp < 0.f)) {
          const double td = (double)ts;
          const TriMat &me = mat[et];
          if (MODE == MODE_GRAPH) {
            const double q = (double)((weight * ct) * ctp) / (td * td), pr = a.emit_pmfr[emitter];
            double w2d;
            if (pr != 0.0)
              w2d = q * pr;
            else
              w2d = q / (double)emit_pmf[emitter];
            const float w2 = (float)w2d;
            const float wf = w2 * kInvPiF;  // BSDF(direct) factor 1/pi, inv_path_trace.cu:8
            const double v[8] = {(double)w2, (double)wf, (double)(wf * pix.x), (double)(wf * pix.y),
                                 (double)(wf * pix.z), (double)(wf * me.ke[0]), (double)(wf * me.ke[1]),
                                 (double)(wf * me.ke[2])};
            const size_t bin = (size_t)tri * nT + et;
            if (a.lds_edges) {
              bins_add(true, edges, bin * kEdgeL, 5, v);
              bins_add(true, edges, (size_t)(nT + 1) * nT * kEdgeL + ((size_t)tri * nE + emitter) * 3, 3, v + 5);
            } else {
              bins_add(false, edges, bin * kEdgeW, 8, v);
            }
          } else {
            const double q = (double)(ct * ctp) / (td * td), pr = a.emit_pmfr[emitter];
            double s64;
            if (pr != 0.0)
              s64 = q * pr;
            else
              s64 = q / (double)emit_pmf[emitter];
            const float s = (float)s64;
            const V3 kee = ke3(et);
            lo = mk(kee.x * s, kee.y * s, kee.z * s);
            emit_s = s;
            emit_et = et;
            const TriMat &m = mat[tri];
            if (SPEC && (m.flags & MAT_HAS_KS)) specd = phong(m.shininess, nh, din, sd);
            const V3 kt = kd3(tri);
            if (SPEC)
              Ld = mk((kt.x + m.ks[0] * specd) * lo.x, (kt.y + m.ks[1] * specd) * lo.y,
                      (kt.z + m.ks[2] * specd) * lo.z);
            else  // Ks = 0: kd + 0*0 == kd
              Ld = mk(kt.x * lo.x, kt.y * lo.y, kt.z * lo.z);
          }
        }
      }
    }

    PHASE(4)
    PHASE_LANES(16, shadow && hs == et)
    if (MODE == MODE_ADJU) {
      // a lane about to write the first slot of a pool chunk it does not hold
      // takes one (wave-uniform hand-out in lane order); none left: the ring
      // ends here for this path (rslot = k, no wrap yet, so the path's chunks
      // [j vcap, (j+1) vcap) stay aligned) and this record goes to slot 0
      const int gs = rslot - a.rec_lds;
      const int sh = 6 * (gs / kPoolSlots);
      const bool needc = vertex && gs >= 0 && (gs % kPoolSlots) == 0 && ((ctab >> sh) & 63u) == 63u;
      uint64_t want = __ballot(needc);
      if (want) {
        int got = -1;
        do {
          const int l = (int)__builtin_ctzll(want);
          want &= want - 1;
          const int c = pfree ? (int)__builtin_ctzll(pfree) : -1;
          pfree &= pfree - 1ull;
          if (lane == l) got = c;
        } while (want);
        if (needc) {
          if (got >= 0) {
            ctab = (ctab & ~(63u << sh)) | ((uint32_t)got << sh);
          } else {
            ctab = (ctab & 0x00ffffffu) | ((uint32_t)rslot << 24);
            rslot = 0;
          }
        }
      }
    }
    // ================= finalise the vertex
    PHASE_LANES(18, vertex)
    if (vertex) {
      if (is_badj<MODE>()) {  // vertex record k (layout [field][vertex][lane])
        float *rec = lds_rec + (size_t)k * kBlock + tid;
        const size_t fs = (size_t)vmax * kBlock;
        rec[0] = __uint_as_float((uint32_t)tri | ((uint32_t)emit_et << 16));
        rec[fs] = emit_s;
        rec[2 * fs] = coeff;
        if (SPEC) {
          rec[kRecSD * fs] = specd;
          rec[(kRecSD + 1) * fs] = speci;
        }
      }
      if (MODE == MODE_ADJU) {  // ring slot rslot = k % rec_cap: LDS or global (TraceArgs::rec_lds)
        constexpr int NF = SPEC ? kRecFieldsSpec : kRecFieldsDiffuse;
        float v[NF];
        v[0] = __uint_as_float((uint32_t)tri | ((uint32_t)emit_et << 16));
        v[1] = emit_s;
        v[2] = coeff;
        if (SPEC) {
          v[kRecSD] = specd;
          v[kRecSD + 1] = speci;
        }
        const int nl = a.rec_lds;
        if (rslot < nl) {  // LDS slot
          float *rec = lds_rec + (size_t)rslot * kBlock + tid;
          const size_t fs = (size_t)nl * kBlock;
#pragma unroll
          for (int f = 0; f < NF; ++f) rec[f * fs] = v[f];
        } else {  // global slot: pool chunk (rslot - nl) / kPoolSlots of this lane
          const int gs = rslot - nl;
          const uint32_t c = (ctab >> (6 * (gs / kPoolSlots))) & 63u;
          gbl_f32 *rec = upool + ((size_t)c * kPoolSlots + (size_t)(gs % kPoolSlots)) * NF;
#pragma unroll
          for (int f = 0; f < NF; ++f) rec[f] = v[f];
        }
        // a chunk starts at ring slot 0 (vertex j * ring size): the forward's M
        // before the update of its first vertex is the chunk's Mlo
        if (kSub > 0) {  // (vertex 0's M is 1: not stored)
          if (rslot % kSub == 0 && k > 0) {
            gbl_f32 *m = umr + (size_t)(rslot / kSub) * 192;
            m[0] = M.x;
            m[1] = M.y;
            m[2] = M.z;
          }
        } else if (rslot == 0) {
          Mlo = M;
        }
        rslot = (rslot + 1 == vcap_of()) ? 0 : rslot + 1;
      }
      if (MODE == MODE_GRAPH) {
        if (cont) {
          weight *= dot3(nd, nh);  // inv_path_trace.cu:144-145
          weight = (float)((double)weight * (((1.0 / (double)kInvPiF) / (double)kPRR) / 1.0));
          dst = tri;
        }
      } else {
        const V3 Le = le();
        L = mk(fmaf(M.x, Le.x + Ld.x, L.x), fmaf(M.y, Le.y + Ld.y, L.y), fmaf(M.z, Le.z + Ld.z, L.z));
        if (cont) {
          const V3 tp = kdpi3(tri);
          const float t0 = tp.x, t1 = tp.y, t2 = tp.z;
          if (SPEC) {
            const TriMat &m = mat[tri];
            M = mk((M.x * (t0 + m.ks[0] * speci)) * coeff, (M.y * (t1 + m.ks[1] * speci)) * coeff,
                   (M.z * (t2 + m.ks[2] * speci)) * coeff);
          } else {  // Ks = 0: kd/pi + 0*0 == kd/pi
            M = mk((M.x * t0) * coeff, (M.y * t1) * coeff, (M.z * t2) * coeff);
          }
        }
      }
      ++k;  // vertices so far
      if (BVH) set_ptri(tri);
      if (cont) d = nd;
      else finished = true;
      if (MODE == MODE_ADJU && rhi > 0 && k == rhi) finished = true;  // replay reached its target
    }

    // ADJU: the chunk [ulo, uhi) to sweep; uend = it ends the path (its escape
    // terms apply, uesc = the path escaped); urep = replay target (0: none)
    int uhi = 0, ulo = 0, urep = 0;
    bool uend = false, uesc = false;
    const bool upend = pending();  // a lane with sub-chunks of its chunk left (IPT_ADJU_SUB)
    if (upend) {  // the chunk of its last sweep: k, rslot, rhi and ctab are untouched since
      uhi = usub;
      ulo = rhi == 0 ? k - (rslot == 0 ? vcap_of() : rslot) : rhi - vcap_of();
      if (ulo > 0) urep = ulo;
    }
    if (finished) {
      active = false;
      if (MODE == MODE_FWDM) {  // slot [channel][sample]
        const uint64_t wi = witem();
        lds_f32 *o = fused_slots(a) + (uint32_t)(wi & 15u) * 3u * (uint32_t)a.spp + (uint32_t)(wi >> 4);
        o[0] = L.x;
        o[a.spp] = L.y;
        o[2 * a.spp] = L.z;
      } else if (MODE == MODE_FWD) {
        float *o = out_samples + witem() * 3;
        o[0] = L.x;
        o[1] = L.y;
        o[2] = L.z;
      } else if (MODE == MODE_ADJU) {
        // The first pass sweeps the path's last chunk [b, K), b = the last
        // multiple of rec_cap below K (its records are the ring's slots 0 ..
        // K - b - 1, its Mlo was captured at vertex b).  A replay to vertex b
        // (same seed, same draws, same floats) re-records [b - rec_cap, b) in
        // slots 0 .. rec_cap - 1 and captures that chunk's Mlo; it is swept with
        // the suffix carried from the chunk after (Scar), and so on to vertex 0.
        if (rhi == 0) {
          uhi = k;
          ulo = k > 0 ? k - (rslot == 0 ? vcap_of() : rslot) : 0;  // (rslot = K % ring size)
          uend = true;
          uesc = escaped;
        } else {
          uhi = rhi;
          ulo = rhi - vcap_of();
        }
        if (ulo > 0) urep = ulo;
      }
    }
    // IPT_ADJU_SUB: this iteration sweeps the chunk's last unswept sub-chunk
    // [uslo, uhi) (sub-chunks aligned to the chunk's start)
    const int uslo = (MODE == MODE_ADJU && kSub > 0 && uhi > ulo) ? ulo + kSub * ((uhi - 1 - ulo) / kSub) : ulo;
    if (MODE == MODE_FWDM && __ballot(finished)) {
      // fused pixel mean: each finished lane counts its sample off its slot's
      // table entry (LDS atomic, after the wave's sample writes: a wave's LDS
      // operations complete in order); the lane that takes a count to zero
      // marks the slot done.  Slots are summed lazily at the loop top.
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      uint32_t left = 0;
      if (finished)
        left = __hip_atomic_fetch_sub(fused_tab(a) + (uint32_t)(witem() & 15u), 1u, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
      uint64_t comp = __ballot(finished && left == 1u);
      while (comp) {  // wave-uniform: usually 0 or 1 slot per iteration
        const int l = (int)__builtin_ctzll(comp);
        comp &= comp - 1ull;
        sdone |= 1u << (__builtin_amdgcn_readlane((int)(witem() & 15u), l) & 31);
      }
    }
    if (is_adj<MODE>()) {
      // Wave-parallel backward sweep (oracle adjoint_sample).  The vertices of
      // the paths that finished in this iteration become tasks (path, vertex
      // kk), packed into rounds of <= 64 consecutive lanes without splitting a
      // path (K <= rec_cap <= 63).  Each task lane reads ITS vertex's record
      // once; the prefix throughputs M_kk then pass left to right and the
      // suffixes S_kk+1 right to left between neighbouring lanes (wave shifts),
      // every step with the forward's / the per-path sweep's own operations,
      // so each M_kk and S_kk+1 is the same float as in the oracle's single
      // sweep (only the order of the fp64 gradient atomics changes).  Round 2
      // recomputed both chains per task from the owner's LDS column (O(K^2)
      // record reads, loops as long as the wave's longest chain).
      // MODE_ADJU sweeps the chunk [ulo, uhi) of each finished lane the same
      // way, from its ring slots (LDS, then global): the prefix chain starts
      // from the chunk's captured Mlo, the last task's suffix is the chunk
      // after's (Scar) unless the chunk ends the path, and the suffix at ulo
      // goes back to the owner for its replay.
      const int Kf = is_badj<MODE>() ? ((finished && k > 0) ? k : 0) : (uhi > 0 ? uhi - uslo : 0);
      if (__ballot(Kf > 0)) {
        const int lane = tid & 63;
        const int inc = wave_scan_add(Kf);  // inclusive scan of the task counts over the wave
        const int T = __builtin_amdgcn_readlane(inc, 63);
        // per-wave LDS word per lane: the round's owner markers
        uint32_t *swl = reinterpret_cast<uint32_t *>(lds_rec) - kBlock + (tid & ~63);
        float wx = 0.f, wy = 0.f, wz = 0.f;  // the owner's adjoint weights dL/dI / spp
        if (Kf > 0) {
          const float *adj = karg<const float *>(offsetof(TraceKernArgs, adj)) +
                             (a.nscenes > 1 ? (size_t)set * a.adj_stride : 0);
          const uint64_t pixel = item_pixel(a, witem());
          if (a.rc_spp != 0.f) {
            wx = adj[pixel * 3 + 0] * a.rc_spp;
            wy = adj[pixel * 3 + 1] * a.rc_spp;
            wz = adj[pixel * 3 + 2] * a.rc_spp;
          } else {
            wx = adj[pixel * 3 + 0] / (float)a.spp;
            wy = adj[pixel * 3 + 1] / (float)a.spp;
            wz = adj[pixel * 3 + 2] / (float)a.spp;
          }
        }
        const size_t fs = (size_t)vmax * kBlock;  // ADJ record field stride (ADJU: per slot kind, below)
        int base = 0;
        while (base < T) {  // wave-uniform
          // this round: the whole paths whose tasks end by base + 64
          const uint64_t fit = __ballot(Kf > 0 && inc <= base + 64);
          const int next = __builtin_amdgcn_readlane(inc, 63 - (int)__builtin_clzll(fit));
          const int t = base + lane;
          const bool valid = t < next;
          PHASE_LANES(20, valid)
          // owners of this round mark their first task's lane with (start,
          // first pass, escaped, K, owner lane) + 1 -- start in the top bits,
          // so an inclusive max-scan leaves every task lane the marker of the
          // last owner starting at or before it: its own path
          swl[lane] = 0u;
          const int st0 = inc - Kf - base;
          const bool owns = Kf > 0 && inc <= next && st0 >= 0;
          const bool oend = is_badj<MODE>() || uend, oesc = is_badj<MODE>() ? escaped : uesc;
          // (ADJU: the sub-chunk's first ring slot, uslo - ulo, in bits 15-20)
          if (owns)
            swl[st0] = (((uint32_t)st0 << 21) | ((uint32_t)(MODE == MODE_ADJU ? uslo - ulo : 0) << 15) |
                        (oend ? 1u << 14 : 0u) | (oesc ? 1u << 13 : 0u) | ((uint32_t)Kf << 6) | (uint32_t)lane) + 1u;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          const uint32_t mk_ = wave_scan_max(swl[lane]) - 1u;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // read before the next round's marks
          __builtin_amdgcn_wave_barrier();
          const int ow = valid ? (int)(mk_ & 63u) : lane;
          const int KL = valid ? (int)((mk_ >> 6) & 127u) : 0;
          const int kk = valid ? lane - (int)(mk_ >> 21) : 0;  // task index inside the path's (sub-)chunk
          const bool esc = valid && ((mk_ >> 13) & 1u);
          const bool fst_o = is_badj<MODE>() || (valid && ((mk_ >> 14) & 1u));  // the chunk ends the path
          const int rr = valid ? KL - 1 - kk : 0;  // vertices after this one
          const V3 Lev = le();
          const V3 LeL = mk(__shfl(Lev.x, ow), __shfl(Lev.y, ow), __shfl(Lev.z, ow));
          // this task's record (lanes past the round read vertex 0 of a valid column)
          uint32_t f0;
          float es, ck, sdv = 0.f, si = 0.f;
          // the prefix throughput: the chunk's Mlo on its first task, passed
          // right by the chain below (ADJ: every chunk starts at vertex 0)
          V3 Mk = mk(1.f, 1.f, 1.f);
          V3 Sc = mk(0.f, 0.f, 0.f);  // ADJU: the owner's suffix from the chunk after
          if (is_badj<MODE>()) {
            const float *r = lds_rec + (tid & ~63) + (valid ? ow : lane) + (size_t)kk * kBlock;
            f0 = valid ? __float_as_uint(r[0]) : 0u;
            es = r[fs];
            ck = r[2 * fs];
            if (SPEC) {
              sdv = r[kRecSD * fs];
              si = r[(kRecSD + 1) * fs];
            }
          } else {
            // the vertex's ring slot (chunks start at slot 0; a sub-chunk at uslo - ulo)
            const int sl = kk + (valid ? (int)((mk_ >> 15) & 63u) : 0), nl = a.rec_lds;
            constexpr int NF = SPEC ? kRecFieldsSpec : kRecFieldsDiffuse;
            float rv[NF];
            uint32_t cto = 0;  // the owner's pool chunks (uniform branch: its ds_bpermute sees every lane)
            if (__ballot(sl >= nl)) cto = (uint32_t)__shfl((int)ctab, ow);
            if (sl < nl) {  // LDS slot (typed: ds_read, see bins_add)
              const lds_f32 *r = (const lds_f32 *)lds_rec + (tid & ~63) + (valid ? ow : lane) + (size_t)sl * kBlock;
              const size_t fl = (size_t)nl * kBlock;
#pragma unroll
              for (int f = 0; f < NF; ++f) rv[f] = r[f * fl];
            } else {  // global slot
              const int gs = sl - nl;
              const uint32_t c = (cto >> (6 * (gs / kPoolSlots))) & 63u;
              const gbl_f32 *r = upool + ((size_t)c * kPoolSlots + (size_t)(gs % kPoolSlots)) * NF;
#pragma unroll
              for (int f = 0; f < NF; ++f) rv[f] = r[f];
            }
            f0 = valid ? __float_as_uint(rv[0]) : 0u;
            es = rv[1];
            ck = rv[2];
            if (SPEC) {
              sdv = rv[kRecSD];
              si = rv[kRecSD + 1];
            }
            // (wave-uniform skips: a chunk from vertex 0 has Mlo = 1, and only
            // replay chunks, which paths longer than the ring make, read Scar)
            if (kSub > 0) {  // the sub-chunk's first M: captured by the forward (1 at vertex 0)
              if (__ballot(owns && uslo > 0)) {
                V3 m0 = mk(1.f, 1.f, 1.f);
                if (owns && uslo > 0) {
                  const gbl_f32 *m = umr + (size_t)((uslo - ulo) / kSub) * 192;
                  m0 = mk(m[0], m[1], m[2]);
                }
                Mk = mk(__shfl(m0.x, ow), __shfl(m0.y, ow), __shfl(m0.z, ow));
              }
            } else if (__ballot(owns && ulo > 0)) {
              Mk = mk(__shfl(Mlo.x, ow), __shfl(Mlo.y, ow), __shfl(Mlo.z, ow));
            }
            if (__ballot(owns && !uend)) Sc = mk(__shfl(Scar.x, ow), __shfl(Scar.y, ow), __shfl(Scar.z, ow));
          }
          // (the min()s keep a mis-indexed record from reaching global memory out of bounds)
          const int tk = min((int)(f0 & 0xffffu), nT - 1);
          const V3 kee = ke3(min((int)(f0 >> 16), nT - 1));
          const V3 lk = mk(kee.x * es, kee.y * es, kee.z * es);  // the forward's lo, same products
          V3 dj = kd3(tk), tv = kdpi3(tk);  // D = kd (+ Ks*specd), T = kd/pi (+ Ks*speci)
          if (SPEC) {
            const TriMat &mj = mat[tk];
            dj = mk(dj.x + mj.ks[0] * sdv, dj.y + mj.ks[1] * sdv, dj.z + mj.ks[2] * sdv);
            tv = mk(tv.x + mj.ks[0] * si, tv.y + mj.ks[1] * si, tv.z + mj.ks[2] * si);
          }
          // prefix (ADJ): M_0 = 1, M_s = (M_{s-1} * T_{s-1}) * c_{s-1} from the left neighbour
          // suffix: S_K = escaped ? Le + D_{K-1} lo_{K-1} : 0 (ADJU replay chunks: Scar),
          // S_j = (Le + D_j lo_j) + (T_j c_j) S_{j+1}
          const V3 A = mk(LeL.x + dj.x * lk.x, LeL.y + dj.y * lk.y, LeL.z + dj.z * lk.z);
          const V3 B = mk(tv.x * ck, tv.y * ck, tv.z * ck);
          V3 S = (esc && rr == 0) ? A : mk(0.f, 0.f, 0.f);
          if (MODE == MODE_ADJU && !fst_o && rr == 0) S = Sc;
          const int kkp = kk;  // prefix chain: task kk takes its left neighbour's M_kk-1 T c
          // both chains in one loop (max(K) - 1 steps instead of up to twice
          // that; two independent dependency chains per step: -0.2..0.6%,
          // profiles/r03/variants_merged_r03o.log)
          const int steps = valid ? max(kkp, rr) : 0;  // this lane's chain steps
          if (__ballot(steps > 0)) {
            // Every lane steps every round: lane i takes lane i-1's (M T) c and
            // lane i+1's A + B S, computed here from the neighbours' operands
            // (shifted once per round; the same float operations as in the
            // neighbour), except a path's first task keeps its M (Mlo / 1) and
            // its last keeps its S.  A lane's value is final after kk (M) / rr
            // (S) steps -- its neighbour's is by then -- and stays so.  (Round 3:
            // a select of the shifted product at step kk only; this form has no
            // per-step compares and one shift fewer per channel.)
            float mx = Mk.x, my = Mk.y, mz = Mk.z, sx = S.x, sy = S.y, sz = S.z;
            int s = 1;
            if (is_badj<MODE>() || IPT_ADJU_SHIFTED_CHAIN) {
              const V3 tvl = mk(wave_shr1(tv.x), wave_shr1(tv.y), wave_shr1(tv.z));
              const float ckl = wave_shr1(ck);
              const V3 Al = mk(wave_shl1(A.x), wave_shl1(A.y), wave_shl1(A.z));
              const V3 Bl = mk(wave_shl1(B.x), wave_shl1(B.y), wave_shl1(B.z));
              const bool keepM = kkp == 0, keepS = rr == 0;
#if IPT_CHAIN_DPP
              const uint64_t kM = __ballot(keepM), kS = __ballot(keepS);
              do {
                chain_step_shifted(mx, my, mz, sx, sy, sz, tvl, ckl, Al, Bl, kM, kS);
              } while (__ballot(steps > s++));
#else
              do {  // (a do-while: the loop-carried values need no copies per step)
                const float nx = (wave_shr1(mx) * tvl.x) * ckl, ny = (wave_shr1(my) * tvl.y) * ckl,
                            nz = (wave_shr1(mz) * tvl.z) * ckl;
                const float hx = Al.x + Bl.x * wave_shl1(sx), hy = Al.y + Bl.y * wave_shl1(sy),
                            hz = Al.z + Bl.z * wave_shl1(sz);
                mx = keepM ? mx : nx;
                my = keepM ? my : ny;
                mz = keepM ? mz : nz;
                sx = keepS ? sx : hx;
                sy = keepS ? sy : hy;
                sz = keepS ? sz : hz;
              } while (__ballot(steps > s++));
#endif
            } else {  // ADJU (register pressure: no pre-shifted operands; a lane takes its neighbour's value at step kk / rr)
#if IPT_CHAIN_DPP
              do {
                chain_step_select(mx, my, mz, sx, sy, sz, tv, ck, A, B, kkp, rr, s);
              } while (__ballot(steps > s++));
#else
              do {
                const float nx = wave_shr1((mx * tv.x) * ck), ny = wave_shr1((my * tv.y) * ck),
                            nz = wave_shr1((mz * tv.z) * ck);
                const float hx = wave_shl1(A.x + B.x * sx), hy = wave_shl1(A.y + B.y * sy),
                            hz = wave_shl1(A.z + B.z * sz);
                const bool tm = kkp == s, ts = rr == s;
                mx = tm ? nx : mx;
                my = tm ? ny : my;
                mz = tm ? nz : mz;
                sx = ts ? hx : sx;
                sy = ts ? hy : sy;
                sz = ts ? hz : sz;
              } while (__ballot(steps > s++));
#endif
            }
            Mk = mk(mx, my, mz);
            S = mk(sx, sy, sz);
#ifdef IPT_PHASE_TIMING
            tacc[22] += (uint64_t)(s - 1);  // chain steps of this round (s: one past the last)
            tacc[23] += 1;
            tacc[24] += (uint64_t)__builtin_amdgcn_readlane(wave_scan_add(steps), 63);
#endif
          }
          // (the owner's adjoint weights are taken only here: their global
          // loads, issued as the sweep starts, finish under the chain)
          const float ax = __shfl(wx, ow), ay = __shfl(wy, ow), az = __shfl(wz, ow);
          if (valid) {
            V3 dLd = Mk;
            if (esc && rr == 0) {  // the escape's stale re-add weights Ld by M_K = (M_K-1 T_K-1) c_K-1
              const V3 ML = mk((Mk.x * tv.x) * ck, (Mk.y * tv.y) * ck, (Mk.z * tv.z) * ck);
              dLd = mk(dLd.x + ML.x, dLd.y + ML.y, dLd.z + ML.z);
            }
            V3 gk = mk(dLd.x * lk.x, dLd.y * lk.y, dLd.z * lk.z);
            if (rr > 0 || esc || !fst_o) {
              const float cpi = div_const<2>(ck);  // ck / kPiF
              gk = mk(gk.x + (cpi * Mk.x) * S.x, gk.y + (cpi * Mk.y) * S.y, gk.z + (cpi * Mk.z) * S.z);
            }
            const int sl = a.grad_map ? a.grad_map[tk] : tk;
            const double v[3] = {(double)(ax * gk.x), (double)(ay * gk.y), (double)(az * gk.z)};
            double *grad = karg<double *>(offsetof(TraceKernArgs, grad)) + (a.nscenes > 1 ? (size_t)set * 3 * a.nT : 0);
            bins_add(sl >= 0, grad, sl >= 0 ? (size_t)sl * 3 : (size_t)tk * 3, 3, v);
          }
          if (MODE == MODE_ADJU && __ballot(owns && (urep > 0 || uslo > ulo))) {  // the suffix at the chunk's first vertex, S_lo = A + B S, back to its owner (for its replay)
            const V3 H = mk(A.x + B.x * S.x, A.y + B.y * S.y, A.z + B.z * S.z);
            const int sa = (owns ? st0 : lane) << 2;
            const V3 Hs = mk(bperm_f(sa, H.x), bperm_f(sa, H.y), bperm_f(sa, H.z));
            if (owns) Scar = Hs;
          }
          base = next;
        }
      }
      // IPT_ADJU_SUB: a lane whose chunk has sub-chunks left sweeps the next
      // one in the next iteration (neither traced nor refilled meanwhile)
      const bool umore = MODE == MODE_ADJU && kSub > 0 && (finished || upend) && uslo > ulo;
      if (MODE == MODE_ADJU && kSub > 0) usub = umore ? uslo : 0;
      if (MODE == MODE_ADJU) {  // a path swept to its first vertex gives its pool chunks back
        const bool rel = (finished || upend) && !umore && urep == 0 && (ctab & kNoChunks) != kNoChunks;
        uint64_t rm = __ballot(rel);
        if (rm) {
          uint64_t mine = 0;
#pragma unroll
          for (int j = 0; j < kPoolMaxChunks; ++j) {
            const uint32_t c = (ctab >> (6 * j)) & 63u;
            if (c != 63u) mine |= 1ull << c;
          }
          do {
            const int l = (int)__builtin_ctzll(rm);
            rm &= rm - 1;
            pfree |= (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mine, l) |
                     ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(mine >> 32), l) << 32);
          } while (rm);
          if (rel) ctab |= kNoChunks;
        }
      }
      if (MODE == MODE_ADJU && urep > 0 && !umore) {  // replay the path from its camera ray (see the chunk choice)
        int r, c;
        item_ray(a, seed, witem(), st, p, d, r, c);
        L = mk(0.f, 0.f, 0.f);
        set_le(L);
        Ld = L;
        M = mk(1.f, 1.f, 1.f);
        Mlo = M;
        k = 0;
        set_ptri(-1);
        rslot = 0;
        rhi = urep;
        active = true;
      }
    }
    PHASE(5)
  }
#ifdef IPT_PHASE_TIMING
  if ((tid & 63) == 0)
    for (int i = 0; i < kPhaseWords; ++i) atomicAdd(&g_phase_cycles[i], (unsigned long long)tacc[i]);
#endif
  }

  if (!is_fwd<MODE>()) {
    __syncthreads();
    if (n_acc > 0) {
      double *dstp = is_adj<MODE>() ? karg<double *>(offsetof(TraceKernArgs, grad)) + (a.nscenes > 1 ? (size_t)set * 3 * a.nT : 0)
                                    : edges;
      const int nb5 = (nT + 1) * nT * kEdgeL;
      for (int i = tid; i < n_acc; i += nthr) {
        const double v = lds_acc[i];
        int j = (is_adj<MODE>() && a.slot_tri) ? a.slot_tri[i / 3] * 3 + i % 3 : i;
        if (MODE == MODE_GRAPH) {  // LDS form -> kEdgeW-wide global bins
          if (i < nb5) {
            j = (i / kEdgeL) * kEdgeW + i % kEdgeL;
          } else {
            const int q = i - nb5, dst = q / (3 * nE), ie = (q / 3) % nE;
            j = (dst * nT + emit_tri[ie]) * kEdgeW + kEdgeL + q % 3;
          }
        }
        if (v != 0.0) atomicAdd(dstp + j, v);
      }
    }
  }
}

// toneMap over a sample-major buffer [s][pixel][3]: same per-pixel
// sequential sum, but lane l reads pixel base+l, so every load of a wave is
// one contiguous 768-byte run (the pixel-major form below strides 12*spp B).
__global__ __launch_bounds__(kBlock) void pixel_mean_sm_kernel(const float *__restrict__ samples, int64_t npix,
                                                               int spp, float *__restrict__ hdr,
                                                               uint8_t *__restrict__ ldr) {
  const int64_t px = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (px >= npix) return;
  // scene batch: blockIdx.y = material set, each with its own [s][pixel][3] buffer and image
  samples += (size_t)blockIdx.y * (size_t)npix * spp * 3;
  hdr += (size_t)blockIdx.y * (size_t)npix * 3;
  if (ldr) ldr += (size_t)blockIdx.y * (size_t)npix * 3;
  float tx = 0.f, ty = 0.f, tz = 0.f;
  const float fs = (float)spp;
  if ((spp & (spp - 1)) == 0 && spp <= (1 << 24)) {
    // x / spp == x * (1/spp) for a power of two (both the correctly rounded
    // x * 2^-k); the loads of 16 samples are issued before their sums (the
    // kernel is latency-bound: one pixel per thread, spp dependent adds)
    const float rc = 1.0f / fs;
    int i = 0;
    for (; i + 16 <= spp; i += 16) {
      float v[48];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const float *s = samples + ((int64_t)(i + u) * npix + px) * 3;
        v[3 * u] = s[0];
        v[3 * u + 1] = s[1];
        v[3 * u + 2] = s[2];
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        tx += v[3 * u] * rc;
        ty += v[3 * u + 1] * rc;
        tz += v[3 * u + 2] * rc;
      }
    }
    for (; i < spp; ++i) {
      const float *s = samples + ((int64_t)i * npix + px) * 3;
      tx += s[0] * rc;
      ty += s[1] * rc;
      tz += s[2] * rc;
    }
  } else {
    for (int i = 0; i < spp; ++i) {
      const float *s = samples + ((int64_t)i * npix + px) * 3;
      tx += s[0] / fs;
      ty += s[1] / fs;
      tz += s[2] / fs;
    }
  }
  hdr[px * 3] = tx;
  hdr[px * 3 + 1] = ty;
  hdr[px * 3 + 2] = tz;
  if (ldr) {
    ldr[px * 3] = (uint8_t)(255.f * tx / (1 + tx));
    ldr[px * 3 + 1] = (uint8_t)(255.f * ty / (1 + ty));
    ldr[px * 3 + 2] = (uint8_t)(255.f * tz / (1 + tz));
  }
}

// toneMap, path_trace.cu:186-198: sequential divide-then-sum per pixel.
__global__ __launch_bounds__(kBlock) void pixel_mean_kernel(const float *__restrict__ samples, int64_t npix,
                                                            int spp, float *__restrict__ hdr,
                                                            uint8_t *__restrict__ ldr) {
  const int64_t px = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (px >= npix) return;
  const float *s = samples + px * spp * 3;
  float tx = 0.f, ty = 0.f, tz = 0.f;
  const float fs = (float)spp;
  for (int i = 0; i < spp; ++i) {
    tx += s[3 * i] / fs;
    ty += s[3 * i + 1] / fs;
    tz += s[3 * i + 2] / fs;
  }
  hdr[px * 3] = tx;
  hdr[px * 3 + 1] = ty;
  hdr[px * 3 + 2] = tz;
  if (ldr) {
    ldr[px * 3] = (uint8_t)(255.f * tx / (1 + tx));
    ldr[px * 3 + 1] = (uint8_t)(255.f * ty / (1 + ty));
    ldr[px * 3 + 2] = (uint8_t)(255.f * tz / (1 + tz));
  }
}

// ---------------------------------------------------------------------------
// TraceArgs::emit_pmfr: 1/pmf for the power-of-two pmfs (exact multiply), else 0.
static std::vector<double> pmf_reciprocals(const std::vector<float> &pmf) {
  std::vector<double> r(pmf.size(), 0.0);
  for (size_t e = 0; e < pmf.size(); ++e) {
    int ex = 0;
    const double m = std::frexp((double)pmf[e], &ex);
    if (pmf[e] > 0.f && m == 0.5 && ex > -1000) r[e] = std::ldexp(1.0, 1 - ex);
  }
  return r;
}

struct GpuScene {
  HostScene host;
  int device = 0;
  bool on_device = false;
  TriIsect *isect = nullptr;
  TriPair *pairs = nullptr;
  TriGeom *geom = nullptr;
  TriMat *mat = nullptr;
  float *kd = nullptr;
  int *emit_tri = nullptr;
  float *emit_cdf = nullptr, *emit_pmf = nullptr;
  double *emit_pmfr = nullptr;  // TraceArgs::emit_pmfr
  bool has_ks = false;      // some material has a Phong lobe
  TriPair *big_pairs = nullptr;
  int32_t *big_idx = nullptr;
  PairBox2 *big_boxes = nullptr;
  float4 *wide = nullptr;  // WideNode records
  float4 *src_cull = nullptr;  // HostScene::bvh_src_cull
  TriIsect *wtris = nullptr;
  PairBox2 *pboxes = nullptr;  // pair acceptance boxes (small scenes' culled shadow casts)
  uint32_t *pomask = nullptr;  // shadow rays' potential occluders (small scenes)
  uint32_t *big_pomask = nullptr;  // ... over the large-triangle pairs (BVH scenes)
  int accel = IPT_ACCEL_AUTO;
  size_t adju_base = 0;  // gpu_adjoint's choice of LDS ring slots (unbounded, brute force) ...
  int adju_nl = 0;       // ... made for this LDS base
  int *grad_map = nullptr, *slot_tri = nullptr;  // ADJ hot-set LDS slots (large scenes)
  int grid[24] = {0};       // resident workgroups per (mode, spec, bvh) (0 = not queried)
  size_t grid_lds[24] = {0};
  size_t pick_base[24] = {0};  // launch_bvh's LDS choice per (mode, spec): base bytes it was made for
  size_t pick_tail[24] = {0};  // ... and the per-block tail (fused pixel mean slots) behind it
  int pick_opt[24] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
                      -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
  // dynamic-chunk counters per stream (stream_counters): `words` grab words,
  // zeroed once; every launch leaves them zero (TraceArgs::chunk_ctr)
  struct Counters {
    hipStream_t stream;
    int words;
    uint32_t *dev;
  };
  std::vector<Counters> counters;
  // buffers a grow replaced: a launch on another host thread may hold one it
  // took before the grow and not have enqueued its kernel yet, so they live
  // until gpu_free
  std::vector<uint32_t *> counters_retired;
  std::mutex counters_mu;
};

#ifdef IPT_PHASE_TIMING
extern "C" int ipt_debug_phase_cycles(unsigned long long *out) {  // read and reset (kPhaseWords words)
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase_cycles), kPhaseWords * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  unsigned long long z[kPhaseWords] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_phase_cycles), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif

#ifdef IPT_BVH_STATS
extern "C" int ipt_debug_bvh_stats(unsigned long long *out) {  // read and reset (kBvhStats counters)
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bvh_stats), kBvhStats * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  unsigned long long z[kBvhStats] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_bvh_stats), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif

const HostScene &gpu_host(const GpuScene *s) { return s->host; }
HostScene &gpu_host_mut(GpuScene *s) { return s->host; }

template <typename T>
static int upload(T **dst, const std::vector<T> &v) {
  const size_t n = std::max<size_t>(v.size(), 1) * sizeof(T);
  HIP_TRY(hipMalloc(reinterpret_cast<void **>(dst), n));
  if (!v.empty()) HIP_TRY(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}

template <typename T>
static int upload_as_f4(float4 **dst, const std::vector<T> &v) {
  static_assert(sizeof(T) % sizeof(float4) == 0, "record is not a whole number of float4");
  HIP_TRY(hipMalloc(reinterpret_cast<void **>(dst), std::max<size_t>(v.size(), 1) * sizeof(T)));
  if (!v.empty()) HIP_TRY(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}

static std::vector<float4> src_cull_f4(const HostScene &host) {
  std::vector<float4> v(host.bvh_src_cull.size() / 4);
  for (size_t i = 0; i < v.size(); ++i)
    v[i] = make_float4(host.bvh_src_cull[4 * i], host.bvh_src_cull[4 * i + 1], host.bvh_src_cull[4 * i + 2],
                       host.bvh_src_cull[4 * i + 3]);
  return v;
}

GpuScene *gpu_upload(const HostScene &host, std::string *err) {
  GpuScene *s = new GpuScene();
  s->host = host;
  if (hipGetDevice(&s->device) != hipSuccess) {
    *err = "no HIP device available";
    delete s;
    return nullptr;
  }
  std::vector<TriPair> pairs((host.isect.size() + 1) / 2);
  pack_pairs(host.isect.data(), (int)host.isect.size(), pairs.data());
  if (upload(&s->isect, host.isect) || upload(&s->pairs, pairs) || upload(&s->geom, host.geom) || upload(&s->mat, host.mat) ||
      upload(&s->kd, host.kd) || upload(&s->emit_tri, host.emit_tri) || upload(&s->emit_cdf, host.emit_cdf) ||
      upload(&s->emit_pmf, host.emit_pmf) || upload(&s->emit_pmfr, pmf_reciprocals(host.emit_pmf)) ||
      upload(&s->big_pairs, host.bvh_big_pairs) || upload(&s->big_idx, host.bvh_big_idx) ||
      upload(&s->big_boxes, host.bvh_big_boxes) ||
      upload_as_f4(&s->wide, host.bvh_wide) || upload(&s->src_cull, src_cull_f4(host)) ||
      upload(&s->wtris, host.bvh_wtris) || upload(&s->pboxes, pair_boxes(host)) ||
      upload(&s->pomask, shadow_occluder_masks(host)) ||
      upload(&s->big_pomask, host.bvh_big_idx.empty()
                                 ? std::vector<uint32_t>()
                                 : shadow_occluder_masks(host, std::vector<int>(host.bvh_big_idx.begin(),
                                                                                host.bvh_big_idx.end())))) {
    *err = gpu_last_error();
    gpu_free(s);
    return nullptr;
  }
  for (const TriMat &m : host.mat) s->has_ks |= (m.flags & MAT_HAS_KS) != 0;
  {  // keep stream-ordered scratch blocks in the pool between launches
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, s->device) == hipSuccess) {
      uint64_t keep = ~0ull;
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
  }
  if ((size_t)host.nT * 3 * sizeof(double) > (size_t)kLdsGradBytes) {
    // adjoint gradient bins: the largest triangles (most path vertices land on
    // them, so their bins are the contended ones) get LDS slots
    const int slots = kLdsGradBytes / (3 * (int)sizeof(double));
    std::vector<int> order(host.nT), map(host.nT, -1), inv(slots);
    for (int i = 0; i < host.nT; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(),
                     [&](int x, int y) { return host.geom[(size_t)x].area > host.geom[(size_t)y].area; });
    for (int k = 0; k < slots; ++k) {
      map[(size_t)order[(size_t)k]] = k;
      inv[(size_t)k] = order[(size_t)k];
    }
    if (upload(&s->grad_map, map) || upload(&s->slot_tri, inv)) {
      *err = gpu_last_error();
      gpu_free(s);
      return nullptr;
    }
  }
  s->on_device = true;
  return s;
}

GpuScene *gpu_host_only(const HostScene &host) {
  GpuScene *s = new GpuScene();
  s->host = host;
  return s;
}
bool gpu_on_device(const GpuScene *s) { return s->on_device; }

void gpu_free(GpuScene *s) {
  if (!s) return;
  if (!s->on_device) {
    delete s;
    return;
  }
  (void)hipFree(s->isect);
  (void)hipFree(s->pairs);
  (void)hipFree(s->geom);
  (void)hipFree(s->mat);
  (void)hipFree(s->kd);
  (void)hipFree(s->emit_tri);
  (void)hipFree(s->emit_cdf);
  (void)hipFree(s->emit_pmf);
  (void)hipFree(s->emit_pmfr);
  (void)hipFree(s->big_pairs);
  (void)hipFree(s->big_idx);
  (void)hipFree(s->big_boxes);
  (void)hipFree(s->wide);
  (void)hipFree(s->src_cull);
  (void)hipFree(s->wtris);
  (void)hipFree(s->pboxes);
  (void)hipFree(s->pomask);
  (void)hipFree(s->big_pomask);
  (void)hipFree(s->grad_map);
  (void)hipFree(s->slot_tri);
  for (auto &c : s->counters) (void)hipFree(c.dev);
  for (uint32_t *p : s->counters_retired) (void)hipFree(p);
  delete s;
}

int gpu_set_kd(GpuScene *s, const float *kd_host) {
  std::memcpy(s->host.kd.data(), kd_host, s->host.kd.size() * sizeof(float));
  if (!s->on_device) return 0;
  HIP_TRY(hipMemcpy(s->kd, kd_host, s->host.kd.size() * sizeof(float), hipMemcpyHostToDevice));
  return 0;
}

int gpu_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

static int check_params(const GpuScene *s, const RenderParams &p) {
  if (!s->on_device) {
    gpu_set_error("scene was loaded host-only (ipt_load_scene_host); it cannot be rendered");
    return -1;
  }
  if (p.width <= 0 || p.height <= 0 || p.spp <= 0 || p.row_begin < 0 || p.row_end > p.height ||
      p.row_begin > p.row_end || p.row_step < 1) {
    gpu_set_error("invalid render parameters (width/height/spp > 0, 0 <= row_begin <= row_end <= height, row_step >= 1)");
    return -1;
  }
  if ((uint64_t)p.width * (uint64_t)p.height * (uint64_t)p.spp >= (1ull << 40)) {
    gpu_set_error("too many samples (width*height*spp must be < 2^40)");
    return -1;
  }
  if (s->host.nT <= 0) {
    gpu_set_error("scene has no triangles");
    return -1;
  }
  if (p.nscenes < 1) {
    gpu_set_error("scene batch needs n_scenes >= 1");
    return -1;
  }
  return 0;
}

#ifndef IPT_DEBUG_GRID
#define IPT_DEBUG_GRID 0
#endif
template <int MODE, bool SPEC, bool BVH>
static int resident_grid(GpuScene *s, size_t lds_bytes, int *grid) {
  const int slot = MODE * 4 + (SPEC ? 2 : 0) + (BVH ? 1 : 0);
  if (s->grid[slot] == 0 || s->grid_lds[slot] != lds_bytes) {
    int per_cu = 0, cus = 0;
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, trace_kernel<MODE, SPEC, BVH>, kBlock,
                                                         lds_bytes));
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device));
    if (per_cu <= 0) {
      gpu_set_error("trace kernel cannot be resident (LDS request too large?)");
      return -1;
    }
    s->grid[slot] = per_cu * cus;
    s->grid_lds[slot] = lds_bytes;
    if (IPT_DEBUG_GRID)  // (make variant DEFS=-DIPT_DEBUG_GRID=1)
      std::fprintf(stderr, "[ipt] trace_kernel<%d,%d,%d>: %zu B LDS/block, %d blocks/CU x %d CUs\n", MODE, (int)SPEC,
                   (int)BVH, lds_bytes, per_cu, cus);
  }
  *grid = s->grid[slot];
  return 0;
}

static TraceArgs make_args(const GpuScene *s, const RenderParams &p);
static TraceArgs make_args_scene(const GpuScene *s) {
  RenderParams p;
  p.width = p.height = p.spp = 1;
  p.max_bounces = 0;
  p.seed = 0;
  p.row_begin = 0;
  p.row_end = 1;
  return make_args(s, p);
}
static TraceArgs make_args(const GpuScene *s, const RenderParams &p) {
  TraceArgs a;
  a.W = p.width;
  a.H = p.height;
  a.spp = p.spp;
  a.max_bounces = p.max_bounces < 0 ? -1 : p.max_bounces;
  a.seed = p.seed;
  const int rows = band_rows(p);
  a.n_samples = (uint64_t)rows * p.width * p.spp;
  a.nT = s->host.nT;
  a.nE = s->host.nE;
  a.lds_edges = 0;
  a.sample_major = 0;
  a.kdpi_g = nullptr;
  a.kd_tables = s->host.nT <= kMaxTableTris ? 1 : 0;
  a.small_pairs = s->host.nT <= 2 * kSmallPairs ? 1 : 0;
  a.npix = (uint64_t)rows * p.width;
  a.row0 = p.row_begin;
  a.row_step = p.row_step > 1 ? p.row_step : 1;
  const uint64_t total = (uint64_t)p.height * p.width * p.spp;
  a.idx32 = total <= 0xffffffffull ? 1 : 0;
  a.m_spp = p.spp > 1 ? ~0ull / (uint64_t)p.spp + 1 : 0;
  a.m_W = p.width > 1 ? ~0ull / (uint64_t)p.width + 1 : 0;
  a.m_npix = a.npix > 1 ? ~0ull / a.npix + 1 : 0;
  a.bvh_nbig = 0;
  a.bvh_big = nullptr;
  a.bvh_big_idx = nullptr;
  a.bvh_big_boxes = nullptr;
  a.bvh_wide = nullptr;
  a.bvh_wtris = nullptr;
  a.bvh_wide_lds = 0;
  a.bvh_big_lds = 0;
  a.coop_stride = 0;
  for (int k = 0; k < 6; ++k) a.root_box[k] = s->host.bvh_root_box[k];
  for (int k = 0; k < 4; ++k) a.tree_sphere[k] = s->host.bvh_sphere[k];
  a.src_cull = s->src_cull;
  a.grad_slots = 0;
  a.grad_map = nullptr;
  a.slot_tri = nullptr;
  std::memcpy(a.cam, s->host.cam, sizeof a.cam);
  a.emit_pmfr = s->emit_pmfr;
  for (int i = 0; i < 3; ++i) {  // camera_ray's pr[i], evaluated once: fmaf is the IEEE fma on host and device
    const float *M = a.cam + 4 * i;
    a.cam_org[i] = std::fmaf(M[3], 1.f, std::fmaf(M[2], 0.f, std::fmaf(M[1], 0.f, M[0] * 0.f)));
  }
  a.rec_cap = p.max_bounces >= 0 ? p.max_bounces + 1 : 0;
  a.rec_lds = 0;
  a.grec = nullptr;
  a.grec_stride = 0;
  a.pool_chunks = 0;
  a.mring = nullptr;
  a.chunk = 0;
  a.group = 0;
  a.chunk_small = 0;
  a.chunk_big_n = 0;
  a.chunk_ctr = nullptr;
  a.grabs = 0;
  a.pboxes = s->pboxes;
  a.pomask = s->host.nE > 0 ? s->pomask : nullptr;
  a.big_pomask = nullptr;  // set with the other BVH fields (bvh_lds)
  a.nscenes = p.nscenes > 1 ? p.nscenes : 1;
  a.bps = 1;
  a.seed_stride = p.seed_stride;
  a.out_stride = a.n_samples * 3;
  a.adj_stride = (uint64_t)p.width * p.height * 3;
  a.rc_spp = (p.spp > 0 && p.spp <= (1 << 24) && (p.spp & (p.spp - 1)) == 0) ? 1.0f / (float)p.spp : 0.f;
  a.rc_W = (p.width > 0 && (p.width & (p.width - 1)) == 0) ? 1.0f / (float)p.width : 0.f;
  a.rc_H = (p.height > 0 && (p.height & (p.height - 1)) == 0) ? 1.0f / (float)p.height : 0.f;
  a.fused = 0;
  a.mean_off = 0;
  a.mean_wstride = 0;
  a.nslots = 0;
  a.ldr = nullptr;
  return a;
}

// Acceleration structure of a launch: the BVH when the scene has one and is
// past the brute-force size (or the caller forced it), else the pair loop.
static bool use_bvh(const GpuScene *s) {
  if (s->host.bvh_nodes.empty()) return false;
  if (s->accel == IPT_ACCEL_BVH) return true;
  if (s->accel == IPT_ACCEL_BRUTE) return false;
  return s->host.nT >= kBvhMinTris;
}

// BVH LDS carve-out on top of `base` bytes; fills the args' BVH fields:
// [wide nodes if staged][large pairs' plane offsets][large pairs' copy if
// taken][emitter records][the wave's 8 group stacks].
static size_t bvh_lds(const GpuScene *s, TraceArgs &a, size_t base, bool stage = true, bool big_copy = true,
                      bool lane_words = false) {
  const size_t nw = s->host.bvh_wide.size();
  a.bvh_wide = s->wide;
  a.bvh_wtris = s->wtris;
  a.bvh_wide_lds = (stage && nw * kWideF4 * sizeof(float4) <= (size_t)kBvhLdsNodeBytes) ? (int)nw : 0;
  a.bvh_big_lds = big_copy && IPT_PATH_CULL ? 1 : 0;
  a.big_pomask = (IPT_SHADOW_PO && s->host.nE > 0 && !s->host.bvh_big_idx.empty()) ? s->big_pomask : nullptr;
  a.coop_stride = 7 * s->host.bvh_wdepth + 8;
  a.bvh_nbig = (int)s->host.bvh_big_pairs.size();
  a.bvh_big = s->big_pairs;
  a.bvh_big_idx = s->big_idx;
  a.bvh_big_boxes = s->big_boxes;
  const size_t head = bvh_lds_offset(base) + (size_t)a.bvh_wide_lds * kWideF4 * sizeof(float4) +
                      (size_t)a.bvh_nbig * 6 * sizeof(float) + (a.bvh_big_lds ? big_lds_bytes(a.bvh_nbig) : 0) +
                      emit_lds_bytes(s->host.nE);
  return head + (size_t)(kBlock / 64) * 8 * a.coop_stride * sizeof(uint32_t) +
         (lane_words ? (size_t)6 * kBlock * sizeof(uint32_t) : 0);  // (BVH forward: trace_kernel's lane_ws)
}

static size_t table_bytes(const TraceArgs &a) {
  return (a.kd_tables ? (size_t)6 * a.nT * sizeof(float) : 0) +
         (a.small_pairs ? (size_t)kE3Floats * ((a.nT + 1) / 2) * sizeof(float) + 12 + (size_t)a.nT * sizeof(TriIsect) +
                              (IPT_PATH_CULL ? (size_t)((a.nT + 1) / 2) * sizeof(TriPair) : 0) +
                              (IPT_SHADOW_PO && a.pomask ? (size_t)a.nT * a.nE * sizeof(uint32_t) : 0)
                        : 0);
}

// Per-launch scratch (the fused render's sample buffer, kd/pi of large
// scenes) is allocated in stream order on the launch's own stream and freed
// behind it: launches on different streams never share a buffer, and the
// device's default pool (release threshold raised in gpu_upload) recycles
// the blocks without a device-wide synchronisation.
struct StreamScratch {
  void *p = nullptr;
  hipStream_t st = nullptr;
  int alloc(size_t bytes, hipStream_t stream) {
    st = stream;
    HIP_TRY(hipMallocAsync(&p, std::max<size_t>(bytes, 16), st));
    return 0;
  }
  ~StreamScratch() {
    if (p) (void)hipFreeAsync(p, st);
  }
};

// The chunk counters of launches on stream `st` with `words` grab words:
// one buffer per (scene, stream), allocated and zeroed (on `st`, in stream
// order) at the stream's first launch and replaced by a larger one when a
// launch needs more words (the old one is kept until gpu_free: another host
// thread may have taken it for a launch it has not enqueued yet -- launches
// already queued on it leave it zeroed and never touch the new one, so no
// synchronisation is needed).  Every launch leaves them zeroed
// (TraceArgs::chunk_ctr), so the host keeps no copy of device state: a launch
// that fails before or after enqueueing changes nothing the next one depends
// on, and any kind of launch (single set, regions, scene batch) may follow any
// other on the stream.  Launches on one stream run in order; other streams
// get their own buffers.  A launch captured into a graph gets a zeroed buffer
// of its own inside the graph (*scratch, freed behind it), so a replay never
// shares words with launches on the capturing stream.
static int stream_counters(GpuScene *s, hipStream_t st, int words, uint32_t **out, void **scratch) {
  const size_t bytes = (size_t)words * sizeof(uint32_t);
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIP_TRY(hipStreamIsCapturing(st, &cap));
  if (cap != hipStreamCaptureStatusNone) {
    HIP_TRY(hipMallocAsync(scratch, bytes, st));
    HIP_TRY(hipMemsetAsync(*scratch, 0, bytes, st));
    *out = (uint32_t *)*scratch;
    return 0;
  }
  std::lock_guard<std::mutex> lk(s->counters_mu);
  GpuScene::Counters *c = nullptr;
  for (auto &e : s->counters)
    if (e.stream == st) c = &e;
  if (c && c->words < words) {  // grow: a new buffer; the old one is retired, not freed
    s->counters_retired.push_back(c->dev);
    c->dev = nullptr;
    c->words = 0;
  }
  if (!c || c->dev == nullptr) {
    const int w = std::max(words, 16);
    uint32_t *dev = nullptr;
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&dev), (size_t)w * sizeof(uint32_t)));
    // zeroed ON the launch stream: a blocking hipMemset goes to the null
    // stream, which a non-blocking stream (every torch stream) does not wait
    // for (round 4's race)
    HIP_TRY(hipMemsetAsync(dev, 0, (size_t)w * sizeof(uint32_t), st));
    if (c) {
      c->dev = dev;
      c->words = w;
    } else {
      s->counters.push_back({st, w, dev});
      c = &s->counters.back();
    }
  }
  *out = c->dev;
  return 0;
}

// Guided chunk sizes (TraceArgs::chunk_big_n), BVH instances: a launch hands
// out its last ~IPT_GUIDED_TAIL small chunks per wave (64 work items) after
// the big ones, so the waves that take the last chunks finish close to the
// others -- a BVH loop iteration is ~2.4x a brute-force one, so a big chunk
// taken at the end kept its wave busy long after the rest of the grid ran
// dry.  North-star 1/8 share: forward 0.814 -> 0.727 ms, adjoint 0.933 ->
// 0.850 (4 per wave; 1 and 2 less).  The brute-force scenes lose with it
// (C2 1/8 share 0.278 -> 0.297 ms at 2 per wave: the fused render's 64-sample
// chunks outrun its two LDS slots, and each extra grab is an atomic round
// trip the wave waits for), so their instances keep fixed chunks
// (profiles/r03/envab_r03j.log).
#ifndef IPT_GUIDED_TAIL
#define IPT_GUIDED_TAIL 4
#endif

// Grabs of one counter word in a launch (a set's or a region's; units, big
// chunks and waves as chunk_range and the kernel's loop see them): chunks 0 ..
// rw-1 are the waves' own, each later chunk is taken by one successful grab,
// and every wave ends with exactly one failed grab -- the non-fused loop
// grabs when its range is used up and stops at the first chunk past the end;
// the fused loop grabs when its chunk is used up, or at once when its own
// chunk is past the end.  Guided instances (BVH) hand out nb chunks of c
// units and then chunks of `small`, the others only chunks of c.
static uint32_t launch_grabs(bool guided, uint64_t units, uint64_t c, uint64_t small, uint64_t nb, uint64_t rw) {
  const uint64_t chunks = guided ? nb + (units - nb * c + small - 1) / small : (units + c - 1) / c;
  return (uint32_t)((chunks > rw ? chunks - rw : 0) + rw);
}
#ifndef IPT_DYN_SMALL_CHUNK
#define IPT_DYN_SMALL_CHUNK 64
#endif

template <int MODE, bool SPEC, bool BVH>
static int launch_inst(GpuScene *s, const TraceArgs &a, size_t lds, const float *kd_dev, float *out, const float *adj,
                       double *grad, const uint8_t *target, double *edges, hipStream_t st) {
  int grid = 0;
  if (lds > 160 * 1024) {
    gpu_set_error("LDS footprint of the launch exceeds 160 KiB");
    return -1;
  }
  if (resident_grid<MODE, SPEC, BVH>(s, lds, &grid)) return -1;
  if (a.n_samples == 0) return 0;
  TraceArgs b = a;
  if (a.nscenes > 1) {  // scene batch: an equal share of the resident blocks per material set
    b.bps = std::max(1, grid / a.nscenes);
    grid = b.bps * a.nscenes;
  }
  b.chunk = 0;
  b.chunk_ctr = nullptr;
  StreamScratch cap_ctr;  // only for a launch captured into a graph
  if (IPT_DYN_CHUNKS) {
    // ~IPT_DYN_CHUNKS_PER_WAVE chunks per wave, a multiple of 64 items, 64..4096
    const uint64_t waves = (uint64_t)(a.nscenes > 1 ? b.bps : grid) * (kBlock / 64);
    uint64_t c = (a.n_samples / (waves * IPT_DYN_CHUNKS_PER_WAVE) + 63) / 64 * 64;
    c = std::min<uint64_t>(std::max<uint64_t>(c, IPT_DYN_MIN_CHUNK), 4096);
    uint64_t units = a.n_samples, small = std::min<uint64_t>(c, IPT_DYN_SMALL_CHUNK);
    if (a.fused) {  // fused pixel mean: chunks of a.chunk pixels (all their samples), small ones of >= 64 samples
      // a launch with fewer chunks than waves (a thin band) halves them while
      // that gives the idle waves work and a chunk keeps >= 64 samples: C2's
      // 1/64 share 0.217 -> 0.10 ms (profiles/r03/launch_scaling_r03w.jsonl)
      c = a.chunk;
      while (c > 1 && (a.npix + c - 1) / c < waves && (c / 2) * (uint64_t)a.spp >= 64) c /= 2;
      b.group = std::min<uint32_t>(a.group, (uint32_t)c);
      small = std::min<uint64_t>(c, std::max<uint64_t>(1, 64 / (uint64_t)a.spp));
      units = a.npix;
    }
    // guided sizes: the last ~IPT_GUIDED_TAIL small chunks per wave end the launch
    // (non-guided instances: one size, chunk_small = chunk and no big-chunk count;
    // IPT_BF_BIG > 1: big chunks of IPT_BF_BIG x c, then IPT_BF_TAIL chunks of
    // c per wave -- fewer grabs for the same tail)
    if (!BVH) {
      small = c;
      c *= IPT_BF_BIG;
    }
    b.chunk = (uint32_t)c;
    b.chunk_small = (uint32_t)small;
    const uint64_t rw = waves;  // chunks 0 .. rw-1: the waves' own; every wave ends with one failed grab
    constexpr bool guided = kGuided<BVH>();
    const uint64_t tail = guided ? rw * (uint64_t)(BVH ? IPT_GUIDED_TAIL : IPT_BF_TAIL) * small : 0;
    const uint64_t nb = guided ? (units > tail ? (units - tail) / c : 0) : 0;
    b.chunk_big_n = (uint32_t)nb;
    b.grabs = launch_grabs(guided, units, c, small, nb, rw);
    cap_ctr.st = st;
    const int words = a.nscenes * kCtrStride;
    if (stream_counters(s, st, words, &b.chunk_ctr, &cap_ctr.p)) return -1;
  }
  StreamScratch grec, mring;  // ADJU: the vertex-record ring (TraceArgs::grec), freed behind the launch
  if (MODE == MODE_ADJU) {  // the ring's global slots: one chunk pool per wave
    const size_t fields = SPEC ? kRecFieldsSpec : kRecFieldsDiffuse;
    const size_t waves = (size_t)grid * (kBlock / 64), chunk = (size_t)kPoolSlots * fields * sizeof(float);
    b.pool_chunks = (int)std::max<size_t>(16, std::min<size_t>(63, ((size_t)IPT_ADJU_POOL_MB << 20) / (waves * chunk)));
    if (g_adju_pool.load() > 0) b.pool_chunks = g_adju_pool.load();
    b.grec_stride = (uint64_t)b.pool_chunks * kPoolSlots * fields;  // floats per wave
    b.rec_cap = std::min(kAdjuRing, a.rec_lds + kPoolMaxChunks * kPoolSlots);
    if (grec.alloc(waves * b.grec_stride * sizeof(float), st)) return -1;
    b.grec = (float *)grec.p;
    if (kSub > 0) {  // the captured prefix throughputs of the sub-chunked sweep
      if (mring.alloc(waves * (size_t)kMrEnt * 64 * 3 * sizeof(float), st)) return -1;
      b.mring = (float *)mring.p;
    }
  }
  // (tests: a launch that fails after its counters and scratch are allocated)
  if (g_fail_launches.load() > 0 && g_fail_launches.fetch_sub(1) > 0) {
    gpu_set_error("launch failed on request (ipt_debug_fail_launches)");
    return -1;
  }
  hipLaunchKernelGGL((trace_kernel<MODE, SPEC, BVH>), dim3(grid), dim3(kBlock), lds, st, b, s->isect, s->pairs, s->geom,
                     s->mat, kd_dev ? kd_dev : s->kd, s->emit_tri, s->emit_cdf, s->emit_pmf, out, adj, grad, target,
                     edges);
  HIP_TRY(hipGetLastError());
  return 0;
}

// The Phong paths (double-precision pow) are compiled only into the SPEC
// instance, used when some material has Ks != 0; the shipped scenes have
// none, and dropping the code lowers register pressure (occupancy).  The BVH
// instances carry the traversal (and its LDS) only for large scenes.
// kd / pi once per launch for scenes without LDS tables (the same IEEE
// division the per-vertex code would do three times per vertex)
__global__ __launch_bounds__(kBlock) void kdpi_kernel(const float *__restrict__ kd, int n, float *__restrict__ out) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i < n) out[i] = kd[i] / kPiF;
}

// BVH instances: the LDS extras (the wide nodes' stage, the large pairs' copy
// of the culled path pre-pass) are taken only as far as they cost no
// residency: of the four combinations, the first (most staged) with the most
// resident workgroups per CU.  North-star adjoint: the tree stage + records +
// bins sit just under 3 workgroups/CU, and the pair copy would tip it to 2
// (6.6 -> 7.9 ms).  Cached per scene and instance for the base LDS bytes.
template <int MODE, bool SPEC>
static int launch_bvh_pick(GpuScene *s, TraceArgs &a, size_t *lds, size_t tail) {
  const int slot = MODE * 4 + (SPEC ? 2 : 0);
  const bool opt[4][2] = {{true, true}, {true, false}, {false, true}, {false, false}};
  const size_t base = *lds;
  if (s->pick_opt[slot] < 0 || s->pick_base[slot] != base || s->pick_tail[slot] != tail) {
    int best = -1, best_per_cu = 0;
    for (int k = 0; k < 4; ++k) {
      TraceArgs b = a;
      const size_t l = bvh_lds_offset(bvh_lds(s, b, base, opt[k][0], opt[k][1], is_fwd<MODE>())) + tail;
      if (l > 160 * 1024) continue;
      int per_cu = 0;
      HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, trace_kernel<MODE, SPEC, true>,
                                                           kBlock, l));
      if (per_cu > best_per_cu) {
        best = k;
        best_per_cu = per_cu;
      }
    }
    if (best < 0) {
      gpu_set_error("BVH trace kernel cannot be resident (LDS request too large?)");
      return -1;
    }
    s->pick_opt[slot] = best;
    s->pick_base[slot] = base;
    s->pick_tail[slot] = tail;
  }
  const int k = s->pick_opt[slot];
  *lds = bvh_lds(s, a, base, opt[k][0], opt[k][1], is_fwd<MODE>());
  return 0;
}

// tail: bytes per workgroup placed after everything else (16-B aligned; the
// fused pixel mean's sample slots, TraceArgs::mean_off).
template <int MODE>
static int launch(GpuScene *s, TraceArgs a, size_t lds, const float *kd_dev, float *out, const float *adj,
                  double *grad, const uint8_t *target, double *edges, hipStream_t st, size_t tail = 0) {
  StreamScratch kdpi;
  if (MODE != MODE_GRAPH && !a.kd_tables && a.n_samples > 0) {
    const int n = 3 * s->host.nT * a.nscenes;
    if (kdpi.alloc((size_t)n * sizeof(float), st)) return -1;
    hipLaunchKernelGGL(kdpi_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, kd_dev ? kd_dev : s->kd, n,
                       (float *)kdpi.p);
    HIP_TRY(hipGetLastError());
    a.kdpi_g = (const float *)kdpi.p;
  }
  auto add_tail = [&]() {
    if (tail) {
      a.mean_off = (uint32_t)bvh_lds_offset(lds);
      lds = a.mean_off + tail;
    }
  };
  if constexpr (MODE == MODE_ADJW) {  // (gpu_adjoint: brute-force diffuse scenes only)
    add_tail();
    return launch_inst<MODE, false, false>(s, a, lds, kd_dev, out, adj, grad, target, edges, st);
  } else if (use_bvh(s)) {
    if (s->has_ks) {
      if (launch_bvh_pick<MODE, true>(s, a, &lds, tail)) return -1;
      add_tail();
      return launch_inst<MODE, true, true>(s, a, lds, kd_dev, out, adj, grad, target, edges, st);
    }
    if (launch_bvh_pick<MODE, false>(s, a, &lds, tail)) return -1;
    add_tail();
    return launch_inst<MODE, false, true>(s, a, lds, kd_dev, out, adj, grad, target, edges, st);
  } else {
    add_tail();
    if (s->has_ks) return launch_inst<MODE, true, false>(s, a, lds, kd_dev, out, adj, grad, target, edges, st);
    return launch_inst<MODE, false, false>(s, a, lds, kd_dev, out, adj, grad, target, edges, st);
  }
}

int gpu_render_samples(GpuScene *s, const RenderParams &p, const float *kd_dev, float *samples_dev, void *stream) {
  if (check_params(s, p)) return -1;
  const TraceArgs a = make_args(s, p);
  return launch<MODE_FWD>(s, a, table_bytes(a), kd_dev, samples_dev, nullptr, nullptr, nullptr, nullptr,
                          (hipStream_t)stream);
}

int gpu_pixel_mean(const float *samples_dev, int64_t npix, int spp, float *hdr_dev, uint8_t *ldr_dev, void *stream) {
  if (npix <= 0) return 0;
  const int blocks = (int)((npix + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(pixel_mean_kernel, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream, samples_dev, npix, spp,
                     hdr_dev, ldr_dev);
  HIP_TRY(hipGetLastError());
  return 0;
}

int gpu_render_samples_sm(GpuScene *s, const RenderParams &p, const float *kd_dev, float *samples_dev,
                          void *stream) {
  if (check_params(s, p)) return -1;
  TraceArgs a = make_args(s, p);
  a.sample_major = 1;
  return launch<MODE_FWD>(s, a, table_bytes(a), kd_dev, samples_dev, nullptr, nullptr, nullptr, nullptr,
                          (hipStream_t)stream);
}

static int pixel_mean_sm_sets(const float *samples_dev, int64_t npix, int spp, int nsets, float *hdr_dev,
                              uint8_t *ldr_dev, void *stream) {
  if (npix <= 0 || nsets <= 0) return 0;
  const int blocks = (int)((npix + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(pixel_mean_sm_kernel, dim3(blocks, nsets), dim3(kBlock), 0, (hipStream_t)stream, samples_dev,
                     npix, spp, hdr_dev, ldr_dev);
  HIP_TRY(hipGetLastError());
  return 0;
}

int gpu_pixel_mean_sm(const float *samples_dev, int64_t npix, int spp, float *hdr_dev, uint8_t *ldr_dev,
                      void *stream) {
  return pixel_mean_sm_sets(samples_dev, npix, spp, 1, hdr_dev, ldr_dev, stream);
}

// Fused pixel mean (IPT_FUSED_MEAN): the ring of one-pixel slots per wave
// (nslots, <= 16, spp x 3 floats each, IPT_FUSED_WAVE_BYTES of LDS per wave)
// and the pixels per group (a power of two, group x spp <= 256 samples, >= 32),
// or {0, 0} when the launch renders through the sample
// buffer + pixel_mean_sm_kernel instead.  A pixel's slot stays busy until its
// last sample is in, so the ring holds at least two groups (bounded paths of
// <= 8 bounces) or four (longer or unbounded paths: a few long paths then
// still leave the next groups their slots -- simulated lane use >= 99% for
// the reference's Russian roulette).  The index math needs
// < 2^32 samples per frame.  (The unfused path stays reachable through
// ipt_render_samples_sm_dev + ipt_pixel_mean_sm_dev; `make variant
// DEFS=-DIPT_FUSED_MEAN=0` builds a library without the fused render.)
#ifndef IPT_FUSED_MEAN
#define IPT_FUSED_MEAN 1
#endif
#ifndef IPT_FUSED_GRAB_SAMPLES  // samples handed out per counter grab (at least)
#define IPT_FUSED_GRAB_SAMPLES 256
#endif
#ifndef IPT_FUSED_WAVE_BYTES
#define IPT_FUSED_WAVE_BYTES 6144
#endif
struct FusedShape {
  int slots, group, per_grab;  // per_grab: groups per chunk (counter grab)
};
// BVH scenes keep the two-kernel render unless the library is built with
// IPT_FUSED_BVH=1 (make variant, A/B timing): their LDS already holds the
// tree stage, and slots beyond IPT_FUSED_BVH_WAVE_BYTES per wave cost
// residency (north-star 3.82 -> 4.10 ms fused,
// profiles/r04/envab_fusedbvh_r04e.log).
#ifndef IPT_FUSED_BVH
#define IPT_FUSED_BVH 0
#endif
#ifndef IPT_FUSED_BVH_WAVE_BYTES
#define IPT_FUSED_BVH_WAVE_BYTES 3072
#endif
static FusedShape fused_shape(const RenderParams &p, bool bvh) {
  const FusedShape none = {0, 0, 0};
  if (!IPT_FUSED_MEAN || !IPT_DYN_CHUNKS) return none;
  if ((uint64_t)p.width * (uint64_t)p.height * (uint64_t)p.spp > 0xffffffffull || p.spp > 256) return none;
  int bytes = IPT_FUSED_WAVE_BYTES;
  if (bvh) {
    if (!IPT_FUSED_BVH) return none;
    bytes = IPT_FUSED_BVH_WAVE_BYTES;
  }
  const int slots = std::min(16, bytes / (12 * p.spp));
  const bool long_paths = p.max_bounces < 0 || p.max_bounces > 8;
  const int cap = slots / (long_paths ? 4 : 2);  // groups the ring holds at once
  if (cap < 1) return none;
  int g = 1;
  while (2 * g <= cap && 2 * g * p.spp <= 256) g *= 2;
  if (g * p.spp < 32) return none;  // (tiny spp: a grab per few samples; the two-kernel render wins)
  // a grab hands out >= 256 samples (small groups -- spp > 128, or long
  // paths -- would otherwise grab per pixel: the legacy 100-spp createImage
  // issued 250 000 counter atomics, 8 MB of memory-side writes per frame)
  const int per_grab = std::min(8, (IPT_FUSED_GRAB_SAMPLES + g * p.spp - 1) / (g * p.spp));
  return {slots, g, per_grab};
}

int gpu_render(GpuScene *s, const RenderParams &p, const float *kd_dev, float *hdr_dev, uint8_t *ldr_dev,
               void *stream) {
  if (check_params(s, p)) return -1;
  const int64_t npix = (int64_t)band_rows(p) * p.width;
  const int sets = p.nscenes > 1 ? p.nscenes : 1;
  // (BVH scenes: two-kernel render by default, see fused_shape)
  const FusedShape fs = fused_shape(p, use_bvh(s));
  if (fs.group > 0) {
    TraceArgs a = make_args(s, p);
    a.fused = 1;
    a.group = (uint32_t)fs.group;
    a.chunk = (uint32_t)(fs.group * fs.per_grab);  // pixels per grab; launch_inst may halve it for thin launches
    a.nslots = fs.slots;
    a.mean_wstride = (uint32_t)(((2 * fs.slots + 3) & ~3) + 3 * fs.slots * p.spp + 3) & ~3u;  // floats per wave
    a.ldr = ldr_dev;
    a.out_stride = (uint64_t)npix * 3;  // per material set: its own HDR (and LDR) image
    const size_t tail = (size_t)(kBlock / 64) * a.mean_wstride * sizeof(float);
    return launch<MODE_FWDM>(s, a, table_bytes(a), kd_dev, hdr_dev, nullptr, nullptr, nullptr, nullptr,
                             (hipStream_t)stream, tail);
  }
  StreamScratch ws;
  if (ws.alloc((size_t)sets * npix * p.spp * 3 * sizeof(float), (hipStream_t)stream)) return -1;
  if (gpu_render_samples_sm(s, p, kd_dev, (float *)ws.p, stream)) return -1;
  return pixel_mean_sm_sets((const float *)ws.p, npix, p.spp, sets, hdr_dev, ldr_dev, stream);
}

// Bounded adjoint launches of at least this many samples (all material sets)
// use MODE_ADJW: C2 (16.8 M) gains 2.7%, a C2 1/8 share (2.1 M) loses 4%.
#ifndef IPT_ADJW_MIN_SAMPLES
#define IPT_ADJW_MIN_SAMPLES (8ull << 20)
#endif
int gpu_adjoint(GpuScene *s, const RenderParams &p, const float *kd_dev, const float *adj_dev, double *grad_dev,
                void *stream) {
  if (check_params(s, p)) return -1;
  if (p.max_bounces > kMaxAdjBounces) {
    gpu_set_error("adjoint requires max_bounces <= 62 (vertex records live in LDS); -1 = unbounded");
    return -1;
  }
  const bool unbounded = p.max_bounces < 0;
  if (s->host.nT > kMaxAdjTris) {
    gpu_set_error("adjoint supports at most 65535 triangles");
    return -1;
  }
  TraceArgs a = make_args(s, p);
  a.sample_major = IPT_ADJ_PIXEL_MAJOR ? 0 : 1;  // (see IPT_ADJ_PIXEL_MAJOR)
  if (s->grad_map) {
    a.grad_slots = kLdsGradBytes / (3 * (int)sizeof(double));
    a.grad_map = s->grad_map;
    a.slot_tri = s->slot_tri;
  } else {
    a.grad_slots = s->host.nT;
  }
  const size_t fields = (size_t)(s->has_ks ? kRecFieldsSpec : kRecFieldsDiffuse);
  const size_t base = (size_t)a.grad_slots * 3 * sizeof(double) + table_bytes(a) +
                      (size_t)kBlock * sizeof(uint32_t);  // + the sweep's owner markers
  if (unbounded) {
    // ring slots in LDS: up to IPT_ADJU_LDS_SLOTS (brute force) or
    // IPT_ADJU_LDS_SLOTS_BVH, as many as cost no resident workgroup (a
    // variant built with IPT_ADJU_LDS_SLOTS_FIXED >= 0 fixes the count, A/B
    // timing); the rest of the ring in global memory
    a.rec_cap = kAdjuRing;
    const bool bvh = use_bvh(s);
    int nl = bvh ? IPT_ADJU_LDS_SLOTS_BVH : IPT_ADJU_LDS_SLOTS;
    if (IPT_ADJU_LDS_SLOTS_FIXED >= 0) {
      nl = IPT_ADJU_LDS_SLOTS_FIXED;
    } else if (!bvh) {
      const size_t per = fields * kBlock * sizeof(float);
      if (s->adju_base != base) {  // cached per scene for this LDS base
        int occ0 = 0;
        HIP_TRY(s->has_ks ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ0, trace_kernel<MODE_ADJU, true, false>,
                                                                         kBlock, base)
                          : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ0, trace_kernel<MODE_ADJU, false, false>,
                                                                         kBlock, base));
        int best = 0;
        for (int k = nl; k > 0 && best == 0; --k) {
          int o = 0;
          HIP_TRY(s->has_ks ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, trace_kernel<MODE_ADJU, true, false>,
                                                                           kBlock, base + k * per)
                            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, trace_kernel<MODE_ADJU, false, false>,
                                                                           kBlock, base + k * per));
          if (o >= occ0 && base + k * per <= IPT_ADJU_LDS_CAP) best = k;
        }
        s->adju_base = base;
        s->adju_nl = best;
      }
      nl = s->adju_nl;
    }
    // (>= 1: a lane's first record never waits for a pool chunk -- with none
    // left it could not start its ring -- so a scene whose LDS base leaves no
    // room for one slot at full residency runs with one workgroup less; one
    // that leaves no room for one slot at all is refused below; launch_inst
    // sizes the global part)
    if (g_adju_lds.load() > 0) nl = g_adju_lds.load();
    a.rec_lds = std::max(1, std::min(nl, kAdjuRing - 1));
  }
  const size_t lds = base + (size_t)(unbounded ? a.rec_lds : a.rec_cap) * fields * kBlock * sizeof(float);
  if (lds > 160 * 1024) {
    gpu_set_error(unbounded ? "unbounded adjoint: the scene's LDS tables plus one record slot per lane exceed 160 KiB"
                            : "adjoint LDS footprint exceeds 160 KiB; lower max_bounces");
    return -1;
  }
  if (unbounded)
    return launch<MODE_ADJU>(s, a, lds, kd_dev, nullptr, adj_dev, grad_dev, nullptr, nullptr, (hipStream_t)stream);
  // the 6-wave instance for full-size launches whose LDS leaves room for a
  // sixth workgroup per CU (IPT_ADJW=0/1 in the environment forces the choice)
  const size_t lane_words = IPT_ADJW_LANE_LDS ? (size_t)6 * kBlock * sizeof(uint32_t) : 0;  // trace_kernel's lane_ws
  bool wide = !use_bvh(s) && !s->has_ks && 6 * (lds + lane_words) <= 160 * 1024 &&
              (uint64_t)a.n_samples * (uint64_t)std::max(1, a.nscenes) >= IPT_ADJW_MIN_SAMPLES;
  if (const char *e = std::getenv("IPT_ADJW")) wide = std::atoi(e) != 0 && !use_bvh(s) && !s->has_ks;
  if (wide)
    return launch<MODE_ADJW>(s, a, lds + lane_words, kd_dev, nullptr, adj_dev, grad_dev, nullptr, nullptr,
                             (hipStream_t)stream);
  return launch<MODE_ADJ>(s, a, lds, kd_dev, nullptr, adj_dev, grad_dev, nullptr, nullptr, (hipStream_t)stream);
}

int gpu_graph(GpuScene *s, const RenderParams &p, const uint8_t *target_dev, double *acc_dev, void *stream) {
  if (check_params(s, p)) return -1;
  TraceArgs a = make_args(s, p);
  const size_t bins = graph_lds_doubles(s->host.nT, s->host.nE) * sizeof(double);
  a.lds_edges = bins <= (size_t)IPT_GRAPH_LDS_KB * 1024 ? 1 : 0;
  a.kd_tables = 0;  // the graph integrator never reads albedo
  a.sample_major = IPT_GRAPH_PIXEL_MAJOR ? 0 : 1;  // (see IPT_ADJ_PIXEL_MAJOR)
  return launch<MODE_GRAPH>(s, a, (a.lds_edges ? bins : 0) + table_bytes(a), nullptr, nullptr, nullptr, nullptr, target_dev, acc_dev,
                            (hipStream_t)stream);
}

// ------------------------------------------------------------ math self-test
// Diagnostic for the exactness claims behind the in-range cores: each core is
// compared bitwise with the IEEE operation hipcc emits, over random operands
// drawn across the whole range the core is used in (and the guard boundaries
// of unit()).  counts[k] = mismatches of test k:
//   0 sqrt_core vs sqrtf          x in [2^-96, 2^127]
//   1 dsqrt_core vs sqrt (f64)    x in [2^-767, 2^1000]
//   2 div_inrange vs a/b          |a| in [2^-100, 2^60], |b| in [2^-60, 2^60], |a/b| in [2^-120, 2^120]
//   3 div_inrange, hit-test range |a| <= 2^20, |b| in [kMinDotUp, 1]
//   4 div3_core vs v/s            unit()'s fast-path operands
//   5 unit vs unit_ieee           vectors with zero / tiny / huge components (guard both ways)
//   6 fast-path hits of test 5    (not a mismatch: shows both paths were exercised)
//   7 camera division range       (2(c+u0))/W, c in [0, 2^16), W in [1, 2^16]
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float rand_exp_float(uint64_t r, int emin, int emax) {  // sign random
  const int e = emin + (int)((r >> 23) % (uint64_t)(emax - emin + 1));
  const uint32_t m = (uint32_t)r & 0x7fffffu;
  const uint32_t sgn = (uint32_t)(r >> 63) << 31;
  return __uint_as_float(sgn | ((uint32_t)(e + 127) << 23) | m);
}
__global__ __launch_bounds__(kBlock) void math_selftest_kernel(uint64_t n, uint64_t seed,
                                                               unsigned long long *counts) {
  unsigned long long c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const uint64_t r0 = mix64(seed ^ (i * 8 + 0)), r1 = mix64(seed ^ (i * 8 + 1)), r2 = mix64(seed ^ (i * 8 + 2));
    const uint64_t r3 = mix64(seed ^ (i * 8 + 3)), r4 = mix64(seed ^ (i * 8 + 4));
    {  // 0
      const float x = fabsf(rand_exp_float(r0, -96, 127));
      c[0] += __float_as_uint(sqrt_core(x)) != __float_as_uint(sqrtf(x));
    }
    {  // 1
      const int e = -767 + (int)((r1 >> 52) % 1768u);
      const double x = __longlong_as_double((long long)(((uint64_t)(e + 1023) << 52) | (r1 & 0xfffffffffffffull)));
      c[1] += __double_as_longlong(dsqrt_core(x)) != __double_as_longlong(sqrt(x));
    }
    {  // 2
      const float a = rand_exp_float(r2, -100, 60);  // nonzero: see div_inrange on zeros
      const float b = rand_exp_float(r3, -60, 60);
      const float q = a / b;
      if (fabsf(q) >= 0x1p-120f && fabsf(q) <= 0x1p120f)
        c[2] += __float_as_uint(div_inrange(a, b)) != __float_as_uint(q);
    }
    {  // 3
      const float a = rand_exp_float(r4, -40, 20);
      const float b = (r0 & 1 ? 1.f : -1.f) * (kMinDotUp + (1.f - kMinDotUp) * (float)(r3 >> 40) * 0x1p-24f);
      c[3] += __float_as_uint(div_inrange(a, b)) != __float_as_uint(a / b);
    }
    {  // 4, 5, 6
      V3 v;
      float comp[3];
      for (int k = 0; k < 3; ++k) {
        const uint64_t rk = mix64(r4 ^ (uint64_t)(k + 11));
        const int kind = (int)(rk & 15);
        if (kind == 0) comp[k] = 0.f;
        else if (kind == 1) comp[k] = (rk & 16) ? -0.f : 0.f;
        else if (kind == 2) comp[k] = rand_exp_float(rk, -149 + 23, -85);   // tiny: around the 2^-90 guard
        else if (kind == 3) comp[k] = rand_exp_float(rk, 25, 35);           // huge: around the 2^60 guard
        else if (kind == 4) comp[k] = rand_exp_float(rk, -6, -2);           // small: around the 2^-6 guard
        else comp[k] = rand_exp_float(rk, -30, 3);
      }
      v = mk(comp[0], comp[1], comp[2]);
      const V3 u = unit(v), w = unit_ieee(v);
      c[5] += (__float_as_uint(u.x) != __float_as_uint(w.x)) || (__float_as_uint(u.y) != __float_as_uint(w.y)) ||
              (__float_as_uint(u.z) != __float_as_uint(w.z));
      const float n2 = dot3(v, v);
      const uint32_t m = min(min((__float_as_uint(v.x) << 1) - 1u, (__float_as_uint(v.y) << 1) - 1u),
                             (__float_as_uint(v.z) << 1) - 1u);
      const bool fast = n2 >= 0x1p-6f && n2 <= 0x1p60f && m >= ((0x25u << 24) - 1u);
      c[6] += fast;
      if (fast) {
        const float sq = sqrtf(n2);
        const V3 q = div3_core(v, sq);
        c[4] += (__float_as_uint(q.x) != __float_as_uint(v.x / sq)) || (__float_as_uint(q.y) != __float_as_uint(v.y / sq)) ||
                (__float_as_uint(q.z) != __float_as_uint(v.z / sq));
      }
    }
    {  // 7
      const int W = 1 + (int)(r0 % 65536u), cc = (int)(r1 % (uint64_t)W);
      const float u0 = (float)(uint32_t)r2 * 2.3283064e-10f + 1.1641532e-10f;
      const float a = 2.f * ((float)cc + u0);
      c[7] += __float_as_uint(div_inrange(a, (float)W)) != __float_as_uint(a / (float)W);
    }
  }
  for (int k = 0; k < 8; ++k)
    if (c[k]) atomicAdd(&counts[k], c[k]);
}

int gpu_selftest_math(uint64_t n, uint64_t seed, uint64_t *counts_host) {
  unsigned long long *d = nullptr;
  HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d), 8 * sizeof(unsigned long long)));
  int rc = 0;
  if (hipMemset(d, 0, 8 * sizeof(unsigned long long)) != hipSuccess) rc = -1;
  if (!rc) {
    hipLaunchKernelGGL(math_selftest_kernel, dim3(2048), dim3(kBlock), 0, 0, n, seed, d);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = -1;
  }
  if (!rc && hipMemcpy(counts_host, d, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) rc = -1;
  (void)hipFree(d);
  if (rc) gpu_set_error("math self-test failed to run");
  return rc;
}

// ------------------------------------------------------------ closest-hit probe
// The cast() of the megakernel on caller-supplied rays: one ray per thread,
// the same LDS staging (small-scene plane offsets, BVH nodes + stack).
// targets[i] >= 0 makes ray i a shadow ray towards that emitter triangle
// (the BVH and the small scenes' culled shadow cast then answer only "is the
// closest hit the target, and at which t"); targets[i] < 0 runs the
// megakernel's path cast (the culled one in small scenes); without targets
// the brute-force loop returns the full closest hit.  Used by the exactness tests of the
// BVH and of the shadow cull against the brute-force loop.
// Potential-occluder mask of a shadow ray from a vertex on triangle `src`
// towards emitter triangle `target` (all pairs when unknown: src outside
// [0, nT), or target not an emitter).
__device__ __forceinline__ uint32_t probe_allow(const uint32_t *masks, const int *emit_tri, int nE, int nT, int src,
                                                int target) {
  if (!masks || src < 0 || src >= nT) return 0xffffffffu;
  for (int e = 0; e < nE; ++e)
    if (emit_tri[e] == target) return masks[src * nE + e];
  return 0xffffffffu;
}

template <bool BVH>
__global__ __launch_bounds__(kBlock) void closest_hit_kernel(const TriIsect *__restrict__ isect,
                                                             const TriPair *__restrict__ pairs, const TraceArgs a,
                                                             int small, int64_t n, const float *__restrict__ org,
                                                             const float *__restrict__ dir,
                                                             const int *__restrict__ targets,
                                                             const int *__restrict__ sources,
                                                             const int *__restrict__ emit_tri, float *__restrict__ t_out,
                                                             int *__restrict__ i_out) {
  extern __shared__ double lds[];
  const int tid = threadIdx.x;
  const int nT = a.nT;
  const int nP = (nT + 1) >> 1;
  float *lds_e3 = reinterpret_cast<float *>(lds);
  const f2 *e3 = nullptr;
  if (small) {
    for (int i = tid; i < kE3Floats * nP; i += kBlock) lds_e3[i] = small_table_entry(pairs, i);
    e3 = reinterpret_cast<const f2 *>(lds_e3);
  }
  // the culled shadow cast's LDS copy of the TriIsect records (!BVH, small)
  float *lds_is = lds_e3 + kE3Floats * nP;
  lds_is += (4 - (int)((lds_is - lds_e3) & 3)) & 3;
  float *lds_pr = lds_is + 20 * nT;  // the culled path cast's TriPair copy (!BVH, small)
  if (!BVH && small) {
    const float *g = reinterpret_cast<const float *>(isect);
    for (int i = tid; i < 20 * nT; i += kBlock) lds_is[i] = g[i];
    if (IPT_PATH_CULL) {
      const float *gp = reinterpret_cast<const float *>(pairs);
      for (int i = tid; i < 36 * nP; i += kBlock) lds_pr[i] = gp[i];
    }
  }
  BvhView bv;
  bv.isect = isect;
  bv.big = nullptr;
  bv.big_idx = nullptr;
  bv.big_e3 = nullptr;
  bv.nbig = 0;
  bv.big_boxes = nullptr;
  bv.big_lds = nullptr;
  bv.emit_is = nullptr;
  CoopView cv;
  cv.wn = a.bvh_wide;
  cv.wn_lds = false;
  cv.wt = a.bvh_wtris;
  cv.stk = nullptr;
  cv.stride = a.coop_stride;
  for (int k = 0; k < 6; ++k) cv.root[k] = a.root_box[k];
  for (int k = 0; k < 4; ++k) cv.sphere[k] = a.tree_sphere[k];
  if (BVH) {
    char *base = reinterpret_cast<char *>(lds);
    float4 *lw = reinterpret_cast<float4 *>(base + bvh_lds_offset((size_t)(small ? kE3Floats * nP : 0) * sizeof(float)));
    if (a.bvh_wide_lds > 0) {
      for (int i = tid; i < kWideF4 * a.bvh_wide_lds; i += kBlock) lw[i] = a.bvh_wide[i];
      cv.wn = lw;
      cv.wn_lds = true;
    }
    float *be3 = reinterpret_cast<float *>(lw + kWideF4 * a.bvh_wide_lds);
    for (int i = tid; i < 6 * a.bvh_nbig; i += kBlock) {
      const int j = i / 6, kf = (i % 6) >> 1, h = i & 1;
      be3[i] = a.bvh_big[j].f[9 + 4 * kf][h];
    }
    bv.big = a.bvh_big;
    bv.big_idx = a.bvh_big_idx;
    bv.big_boxes = a.bvh_big_boxes;
    bv.big_e3 = reinterpret_cast<const f2 *>(be3);
    bv.nbig = a.bvh_nbig;
    uint32_t *after = reinterpret_cast<uint32_t *>(
        big_lds_copy(a, be3 + 6 * a.bvh_nbig, reinterpret_cast<float *>(lds), tid, kBlock, bv));
    cv.stk = after + (tid >> 6) * 8 * a.coop_stride;
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kBlock + tid;
  const bool valid = i < n;  // no early return: the cooperative cast needs the whole wave
  V3 p = mk(0.f, 0.f, 0.f), d = mk(0.f, 0.f, 1.f);
  int target = -1, src = -1;
  if (valid) {
    p = mk(org[3 * i], org[3 * i + 1], org[3 * i + 2]);
    d = mk(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
    target = targets ? targets[i] : -1;
    src = sources ? sources[i] : -1;
    src = src < nT ? src : -1;
  }
  float t = 0.f;
  int h = -1;
  if (BVH) {
    bool qn = false;
    if (valid) {
      // the tree-entry culls (sphere, source plane) hold for the megakernel's
      // unit directions; a caller's ray of another length takes the box test
      // only, so the BVH answers the brute-force loop for any direction
      const bool unit = fabsf(dot3(d, d) - 1.f) <= 0x1p-20f;
      if (target >= 0) {
        const uint32_t allow = probe_allow(IPT_SHADOW_PO ? a.big_pomask : nullptr, emit_tri, a.nE, nT, src, target);
        if (bvh_prepass<true>(bv, p, d, t, h, target, allow))
          qn = coop_root_test(cv, p, d, t, unit) && !(IPT_TREE_SKIP && tree_skip(a.src_cull, src, d, unit));
      } else {  // (a path ray with a source: the megakernel's bounce ray leaving that triangle)
        bvh_prepass<false>(bv, p, d, t, h, -1);
        qn = coop_root_test(cv, p, d, t, unit) && !(IPT_TREE_SKIP && tree_skip(a.src_cull, src, d, unit));
      }
    }
    coop_cast<false>(cv, qn && target < 0, p, d, t, h);
    coop_cast<true>(cv, qn && target >= 0, p, d, t, h);
  } else if (valid) {
    if (IPT_SHADOW_CULL && small && target >= 0) {  // the megakernel's shadow cast of small scenes
      const uint32_t allow = probe_allow(IPT_SHADOW_PO ? a.pomask : nullptr, emit_tri, a.nE, nT, src, target);
      h = shadow_hit_pairs_small((const lds_f32 *)lds_is, pairs, a.pboxes, e3, nT, p, d, target, t, allow);
    } else if (IPT_PATH_CULL && small && targets && target < 0) {  // ... and its path cast
      h = closest_hit_pairs_culled((const lds_f32 *)lds_pr, a.pboxes, nT, p, d, t);
    } else {  // the full closest hit (brute-force pair loop)
      h = cast_bf(pairs, e3, nT, p, d, t);
    }
  }
  if (valid) {
    t_out[i] = t;
    i_out[i] = h;
  }
}

int gpu_set_accel(GpuScene *s, int mode) {
  if (mode != IPT_ACCEL_AUTO && mode != IPT_ACCEL_BRUTE && mode != IPT_ACCEL_BVH) {
    gpu_set_error("unknown acceleration mode");
    return -1;
  }
  if (mode == IPT_ACCEL_BVH && s->host.bvh_nodes.empty()) {
    gpu_set_error("scene has no BVH: " + s->host.bvh_status);
    return -1;
  }
  s->accel = mode;
  return 0;
}
int gpu_accel_in_use(const GpuScene *s) { return use_bvh(s) ? IPT_ACCEL_BVH : IPT_ACCEL_BRUTE; }

int gpu_closest_hit(GpuScene *s, int64_t n, const float *org_dev, const float *dir_dev, const int *targets_dev,
                    const int *sources_dev, float *t_dev, int *idx_dev, void *stream) {
  if (!s->on_device) {
    gpu_set_error("scene was loaded host-only (ipt_load_scene_host); it cannot be traced");
    return -1;
  }
  if (n <= 0) return 0;
  TraceArgs a = make_args_scene(s);
  const int small = s->host.nT <= 2 * kSmallPairs ? 1 : 0;
  const size_t base = small ? (size_t)kE3Floats * ((s->host.nT + 1) / 2) * sizeof(float) : 0;
  const int blocks = (int)((n + kBlock - 1) / kBlock);
  if (use_bvh(s)) {
    const size_t lds = bvh_lds(s, a, base);
    hipLaunchKernelGGL(closest_hit_kernel<true>, dim3(blocks), dim3(kBlock), lds, (hipStream_t)stream, s->isect,
                       s->pairs, a, small, n, org_dev, dir_dev, targets_dev, sources_dev, s->emit_tri, t_dev, idx_dev);
  } else {
    const size_t lds = base + (small ? 12 + (size_t)s->host.nT * sizeof(TriIsect) +
                                           (IPT_PATH_CULL ? (size_t)((s->host.nT + 1) / 2) * sizeof(TriPair) : 0)
                                     : 0);
    hipLaunchKernelGGL(closest_hit_kernel<false>, dim3(blocks), dim3(kBlock), lds, (hipStream_t)stream, s->isect,
                       s->pairs, a, small, n, org_dev, dir_dev, targets_dev, sources_dev, s->emit_tri, t_dev, idx_dev);
  }
  HIP_TRY(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------ host wrappers
namespace {
struct DevBuf {
  void *p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};
}  // namespace

int gpu_render_samples_host(GpuScene *s, const RenderParams &p, float *samples) {
  if (check_params(s, p)) return -1;
  const size_t n = (size_t)band_rows(p) * p.width * p.spp * 3;
  DevBuf b;
  HIP_TRY(hipMalloc(&b.p, std::max<size_t>(n, 1) * sizeof(float)));
  if (gpu_render_samples(s, p, nullptr, (float *)b.p, nullptr)) return -1;
  HIP_TRY(hipMemcpy(samples, b.p, n * sizeof(float), hipMemcpyDeviceToHost));
  return 0;
}

int gpu_render_host(GpuScene *s, const RenderParams &p, float *hdr, uint8_t *ldr) {
  if (check_params(s, p)) return -1;
  const size_t npix = (size_t)band_rows(p) * p.width;
  DevBuf h, l;
  HIP_TRY(hipMalloc(&h.p, std::max<size_t>(npix, 1) * 3 * sizeof(float)));
  if (ldr) HIP_TRY(hipMalloc(&l.p, std::max<size_t>(npix, 1) * 3));
  if (gpu_render(s, p, nullptr, (float *)h.p, (uint8_t *)l.p, nullptr)) return -1;
  HIP_TRY(hipMemcpy(hdr, h.p, npix * 3 * sizeof(float), hipMemcpyDeviceToHost));
  if (ldr) HIP_TRY(hipMemcpy(ldr, l.p, npix * 3, hipMemcpyDeviceToHost));
  return 0;
}

int gpu_adjoint_host(GpuScene *s, const RenderParams &p, const float *adj, double *grad) {
  if (check_params(s, p)) return -1;
  const size_t na = (size_t)p.width * p.height * 3, ng = (size_t)s->host.nT * 3;
  DevBuf a, g;
  HIP_TRY(hipMalloc(&a.p, na * sizeof(float)));
  HIP_TRY(hipMalloc(&g.p, ng * sizeof(double)));
  HIP_TRY(hipMemcpy(a.p, adj, na * sizeof(float), hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(g.p, 0, ng * sizeof(double)));
  if (gpu_adjoint(s, p, nullptr, (const float *)a.p, (double *)g.p, nullptr)) return -1;
  HIP_TRY(hipMemcpy(grad, g.p, ng * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

int gpu_closest_hit_host(GpuScene *s, int64_t n, const float *org, const float *dir, const int *targets,
                         const int *sources, float *t, int *idx) {
  if (n <= 0) return 0;
  DevBuf o, d, g, sr, tt, ii;
  const size_t n3 = (size_t)n * 3 * sizeof(float);
  HIP_TRY(hipMalloc(&o.p, n3));
  HIP_TRY(hipMalloc(&d.p, n3));
  HIP_TRY(hipMalloc(&tt.p, (size_t)n * sizeof(float)));
  HIP_TRY(hipMalloc(&ii.p, (size_t)n * sizeof(int)));
  HIP_TRY(hipMemcpy(o.p, org, n3, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(d.p, dir, n3, hipMemcpyHostToDevice));
  if (targets) {
    HIP_TRY(hipMalloc(&g.p, (size_t)n * sizeof(int)));
    HIP_TRY(hipMemcpy(g.p, targets, (size_t)n * sizeof(int), hipMemcpyHostToDevice));
  }
  if (sources) {
    HIP_TRY(hipMalloc(&sr.p, (size_t)n * sizeof(int)));
    HIP_TRY(hipMemcpy(sr.p, sources, (size_t)n * sizeof(int), hipMemcpyHostToDevice));
  }
  if (gpu_closest_hit(s, n, (const float *)o.p, (const float *)d.p, (const int *)g.p, (const int *)sr.p,
                      (float *)tt.p, (int *)ii.p, nullptr))
    return -1;
  HIP_TRY(hipMemcpy(t, tt.p, (size_t)n * sizeof(float), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(idx, ii.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost));
  return 0;
}

int gpu_graph_host(GpuScene *s, const RenderParams &p, const uint8_t *target, double *acc) {
  if (check_params(s, p)) return -1;
  const size_t nt = (size_t)p.width * p.height * 3;
  const size_t nb = (size_t)(s->host.nT + 1) * s->host.nT * kEdgeW;
  DevBuf t, e;
  HIP_TRY(hipMalloc(&t.p, nt));
  HIP_TRY(hipMalloc(&e.p, nb * sizeof(double)));
  HIP_TRY(hipMemcpy(t.p, target, nt, hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(e.p, 0, nb * sizeof(double)));
  if (gpu_graph(s, p, (const uint8_t *)t.p, (double *)e.p, nullptr)) return -1;
  HIP_TRY(hipMemcpy(acc, e.p, nb * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

}  // namespace ipt
