// pass_common.h — device-side data model and shared device functions of the PatchMatch pass.
//
// HBM layout (one reference image, pass resolution W x H, L = W*H, N images):
//   imgq[v]     float4 [(H+2)*(W+2)]  padded quad-texel image: element (X,Y) holds the four texels
//                                     (X-1,Y-1),(X,Y-1),(X-1,Y),(X,Y) with clamp -> one 16-B load per
//                                     bilinear tap (replaces the CUDA texture unit, DPE.cpp:919-935)
//   ref         f32 [L]               reference grey levels (exact texels, DPE.cu:585/722/734)
//   depth[v]    f32 [L]               source depth maps for the geometric term (DPE.cpp:826-843)
//   planes      float4 [L]            (n, d) hypotheses; snapshot copy for red/black reads
//   costs, sel  f32/u32 [L]           + snapshots
//   weak        u8 [L]                PixelState
//   vw          u8 [L*32]             view weights of the last sweep (DPE.cu:1548)
//   nb          short2 [L*9]          deformable neighbours, per pixel (reference: compacted by
//                                     neighbours_map, DPE.cpp:859-870; per-pixel costs 36 B/px
//                                     of the 288 GB and removes one indirection)
//   nearest, edge_neigh[8], lab_bound[8] short2 per pixel; complex f32, radius i32, fit float4
#pragma once
#include "device_math.h"
#include "bres_walk.h"
#include "../../include/dpe_mvs.h"

namespace dpe {

struct ViewConst { float M[9]; float b[3]; };

struct PassConst {
  int W, H, N, LW, LH;
  int half_rows;             // rows visited by the red/black grids (DPE.cu:3143)
  uint32_t seed32, salt;
  float kinv0, kinv4, kc2, kc5;
  float gn_cos, gn_sin, gn_thr;
  int gn_shift;
  uint32_t gn_shift_m;       // floor(2^32 / gn_shift) (2^32 - 1 for 1): x % gn_shift as a multiply (gn_mod)
  int weak_nn;               // side of the weak sweep's neighbour patches, (2 weak_radius) / weak_increment + 1 (0 if radius < 0)
  DpePatchMatchParams P;
  DpeCamera cams[DPE_MAX_IMAGES];
  ViewConst vc[DPE_MAX_IMAGES];
};

struct DevBufs {
  const float4* imgq[DPE_MAX_IMAGES];     // f32 quad-texel images (any grey levels)
  // 8-bit grey-level images as quad texels in the two layouts below (TEX_U8, TEX_F16), each with
  // all views in one allocation, view v at byte offset v * view bytes (< 4 GiB: 32-bit offsets)
  const uint8_t* img8; uint32_t img8_view;
  const uint8_t* img16; uint32_t img16_view;
  const uint8_t* imgp; uint32_t imgp_view;   // TEX_P16 column pairs, row stride W + 3
  const float* depth[DPE_MAX_IMAGES];
  const float* ref;
  float4* planes; float4* planes_snap; float4* fit_plane;
  const float4* planes0;                  // the staged initial planes (read by GenNeighbours)
  float* costs; float* costs_snap; float* complex_;
  uint32_t* sel; uint32_t* sel_snap;
  uint8_t* weak; uint8_t* weak_rel; uint8_t* vw;
  short2* nb; short2* nearest; short2* edge_neigh; short2* lab_bound;
  int* radius;
  const uint8_t* edge; const uint8_t* edge_low; const int* label;
  // algorithmic work counters of the launch class (nullptr unless counting):
  // [0] homographies (NCC set-ups), [1] bilinear taps, [2] geometric-consistency evaluations
  unsigned long long* cnt;
  unsigned long long* phase;              // DPE_PHASE_PROF builds only
  int xcd_rows;   // block rows per XCD chunk (0 = dispatcher order)
};

// Diagnostic builds, -DDPE_DIAG=<bits> (none of them changes a result; the product is DPE_DIAG=0):
//   1  phase cycle sums of the cooperative kernels (tools/phase_prof.py)
//   2  gather-line statistics of the fast tap loops (tools/line_stats.py)
//   4  weak-sweep path statistics (tools/weak_stats.py)
//   8  GenNeighbours per-pixel clocks and counts (tools/gn_times.py)
//  16  job-pool statistics of the cooperative kernels (tools/pool_stats.py)
//  32  TIMING ONLY, results wrong: the fast taps' texel loads replaced by values made from their
//      address bits (the gather path's share of a tap kernel, interleaved A/B with AB_NOCHECK=1)
#ifndef DPE_DIAG
#define DPE_DIAG 0
#endif
// DPE_UNCLAMPED=0 (A/B only): every fast Old-NCC patch keeps its tap clamps (taps_unclamped unused)
#ifndef DPE_UNCLAMPED
#define DPE_UNCLAMPED 1
#endif
#define DPE_POOL_STATS (((DPE_DIAG) >> 4) & 1)
#define DPE_PHASE_PROF ((DPE_DIAG) & 1)
#define DPE_LINE_STATS (((DPE_DIAG) >> 1) & 1)
#define DPE_WEAK_STATS (((DPE_DIAG) >> 2) & 1)
#define DPE_GN_TIMES (((DPE_DIAG) >> 3) & 1)
#define DPE_FAKE_GATHER (((DPE_DIAG) >> 5) & 1)
// Phase profiling (DPE_DIAG & 1): shader-clock cycles of each phase of a cooperative kernel,
// summed over waves into B.phase[k].
#if DPE_PHASE_PROF
#define PHASE_BEGIN() uint64_t ph_t_ = __builtin_readcyclecounter(), ph_acc_[16] = {}
#define PHASE(k)                                                                    \
  do {                                                                              \
    const uint64_t n_ = __builtin_readcyclecounter();                               \
    ph_acc_[k] += n_ - ph_t_;                                                       \
    ph_t_ = n_;                                                                     \
  } while (0)
// per-wave sums go to one of 32 copies of the counters (the host adds them up)
#define PHASE_END(kernel)                                                           \
  do {                                                                              \
    if ((threadIdx.x & 63) == 0 && B.phase)                                         \
      for (int k_ = 0; k_ < 16; ++k_)                                               \
        if (ph_acc_[k_]) atomicAdd(B.phase + ((blockIdx.x & 31) * 4 + (kernel)) * 16 + k_, (unsigned long long)ph_acc_[k_]); \
  } while (0)
// every lane adds its own sums (thread-per-item kernels whose lanes diverge)
#define PHASE_END_ALL(kernel)                                                       \
  do {                                                                              \
    if (B.phase)                                                                    \
      for (int k_ = 0; k_ < 16; ++k_)                                               \
        if (ph_acc_[k_]) atomicAdd(B.phase + ((blockIdx.x & 31) * 4 + (kernel)) * 16 + k_, (unsigned long long)ph_acc_[k_]); \
  } while (0)
#else
#define PHASE_BEGIN() do {} while (0)
#define PHASE(k) do {} while (0)
#define PHASE_END(kernel) do {} while (0)
#define PHASE_END_ALL(kernel) do {} while (0)
#endif
// Job-pool statistics (DPE_DIAG & 16): per pool, the jobs dealt, the 64-lane rounds they take and
// the waves (utilisation = jobs / (64 rounds)); pools: 0 strong cost vectors, 1 strong refinement,
// 2 weak candidates, 3 weak current / fit plane, 4 weak refinement, 5 weak final Old NCC.
#if DPE_POOL_STATS
static __device__ unsigned long long g_pool[8][3];
DEV void pool_stat(int k, int jobs) {
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&g_pool[k][0], (unsigned long long)jobs);
    atomicAdd(&g_pool[k][1], (unsigned long long)((jobs + 63) / 64));
    atomicAdd(&g_pool[k][2], 1ull);
  }
}
#define POOL_STAT(k, n) pool_stat(k, n)
// Old NCC patches read from LDS (ncc_old_lds): all, and those whose reciprocal range check failed
#define PATCH_STAT(ok) do { atomicAdd(&g_pool[6][0], 1ull); if (!(ok)) atomicAdd(&g_pool[6][1], 1ull); } while (0)
#else
#define POOL_STAT(k, n) do {} while (0)
#define PATCH_STAT(ok) do {} while (0)
#endif
DEV void count_work(const DevBufs& B, unsigned long long ncc, unsigned long long taps) {
  if (B.cnt) { atomicAdd(B.cnt + 0, ncc); atomicAdd(B.cnt + 1, taps); }
}

// XCD-aware workgroup order.  The dispatcher deals workgroups round-robin to the 8 XCDs, each with
// its own 4 MB L2 (MI355X_MICROARCH.md), so neighbouring tiles land on different L2s.  The remap
// gives XCD k every 8th chunk of `chunk` consecutive logical workgroups (a band of block rows):
// an XCD's in-flight tiles then share source-image footprints in its L2, while the interleave keeps
// spatially clustered work (the WEAK regions) spread over all XCDs.  Bijective; speed only.
DEV int xcd_remap(int b, int nb, int chunk) {
  if (chunk <= 0) return b;
  const int super = 8 * chunk;
  const int S = (nb / super) * super;
  if (b >= S) return b;
  const int xcd = b & 7, pos = b >> 3;
  return ((pos / chunk) * 8 + xcd) * chunk + (pos % chunk);
}

// ------------------------------------------------------------------------------ bits
DEV void setBit(uint32_t& v, unsigned n) { v |= (1u << n); }
DEV void unSetBit(uint32_t& v, unsigned n) { v &= (0xFFFFFFFEu << n); }   // clears bits 0..n (DPE.cu:77-80)
DEV int isSet(uint32_t v, unsigned n) { return (v >> n) & 1; }

// ------------------------------------------------------------------------------ geometry
DEV void normalize3(float4& v) {
  const float n2 = v.x * v.x + v.y * v.y + v.z * v.z;
  const float inv = d_rsqrtf(n2);
  v.x *= inv; v.y *= inv; v.z *= inv;
}
DEV void normalize2(float2& v) {
  const float n2 = v.x * v.x + v.y * v.y;
  const float inv = d_rsqrtf(n2);
  v.x *= inv; v.y *= inv;
}
DEV void get3d(const DpeCamera& c, int px, int py, float depth, float X[3]) {
  X[0] = depth * ((float)px - c.K[2]) / c.K[0];
  X[1] = depth * ((float)py - c.K[5]) / c.K[4];
  X[2] = depth;
}
DEV float4 view_direction(const DpeCamera& c, int px, int py, float depth) {
  float X[3]; get3d(c, px, py, depth, X);
  const float norm = __builtin_sqrtf(X[0] * X[0] + X[1] * X[1] + X[2] * X[2]);
  return make_float4(X[0] / norm, X[1] / norm, X[2] / norm, 0.0f);
}
DEV float dist2origin(const DpeCamera& c, int px, int py, float depth, const float4& n) {
  float X[3]; get3d(c, px, py, depth, X);
  return -(n.x * X[0] + n.y * X[1] + n.z * X[2]);
}
DEV float depth_from_plane(const DpeCamera& c, const float4& pl, int px, int py) {
  return -pl.w * c.K[0] / (((float)px - c.K[2]) * pl.x + (c.K[0] / c.K[4]) * ((float)py - c.K[5]) * pl.y + c.K[0] * pl.z);
}
DEV float4 transform_normal(const DpeCamera& c, const float4& p) {      // R^T n (DPE.cu:524-532)
  return make_float4(c.R[0] * p.x + c.R[3] * p.y + c.R[6] * p.z,
                     c.R[1] * p.x + c.R[4] * p.y + c.R[7] * p.z,
                     c.R[2] * p.x + c.R[5] * p.y + c.R[8] * p.z, p.w);
}
DEV float4 transform_normal_ref(const DpeCamera& c, const float4& p) {  // R n (DPE.cu:534-542)
  return make_float4(c.R[0] * p.x + c.R[1] * p.y + c.R[2] * p.z,
                     c.R[3] * p.x + c.R[4] * p.y + c.R[5] * p.z,
                     c.R[6] * p.x + c.R[7] * p.y + c.R[8] * p.z, p.w);
}
DEV float3 world_point(float x, float y, float depth, const DpeCamera& c) {   // DPE.cu:881-901
  float3 X, T;
  X.x = depth * (x - c.K[2]) / c.K[0];
  X.y = depth * (y - c.K[5]) / c.K[4];
  X.z = depth;
  T.x = c.R[0] * X.x + c.R[3] * X.y + c.R[6] * X.z;
  T.y = c.R[1] * X.x + c.R[4] * X.y + c.R[7] * X.z;
  T.z = c.R[2] * X.x + c.R[5] * X.y + c.R[8] * X.z;
  return make_float3(T.x + c.c[0], T.y + c.c[1], T.z + c.c[2]);
}
DEV float2 project_cam(const float3& X, const DpeCamera& c) {                 // DPE.cu:903-913
  const float tx = c.R[0] * X.x + c.R[1] * X.y + c.R[2] * X.z + c.t[0];
  const float ty = c.R[3] * X.x + c.R[4] * X.y + c.R[5] * X.z + c.t[1];
  const float tz = c.R[6] * X.x + c.R[7] * X.y + c.R[8] * X.z + c.t[2];
  const float d = c.K[6] * tx + c.K[7] * ty + c.K[8] * tz;
  return make_float2((c.K[0] * tx + c.K[1] * ty + c.K[2] * tz) / d, (c.K[3] * tx + c.K[4] * ty + c.K[5] * tz) / d);
}

// GenerateRandomNormal (DPE.cu:361-387)
DEV float4 random_normal(const DpeCamera& c, int px, int py, Rng& rs, float depth) {
  float q1 = 1.0f, q2 = 1.0f, s = 2.0f;
  while (s >= 1.0f) {
    q1 = 2.0f * rng_uniform(rs) - 1.0f;
    q2 = 2.0f * rng_uniform(rs) - 1.0f;
    s = q1 * q1 + q2 * q2;
  }
  const float sq = __builtin_sqrtf(1.0f - s);
  float4 n = make_float4(2.0f * q1 * sq, 2.0f * q2 * sq, 1.0f - 2.0f * s, 0.0f);
  const float4 vd = view_direction(c, px, py, depth);
  if (n.x * vd.x + n.y * vd.y + n.z * vd.z > 0.0f) { n.x = -n.x; n.y = -n.y; n.z = -n.z; }
  normalize3(n);
  return n;
}
// GeneratePerturbedNormal (DPE.cu:389-424)
DEV float4 perturbed_normal(const DpeCamera& c, int px, int py, const float4& normal, Rng& rs, float pert) {
  const float4 vd = view_direction(c, px, py, 1.0f);
  const float a1 = (rng_uniform(rs) - 0.5f) * pert;
  const float a2 = (rng_uniform(rs) - 0.5f) * pert;
  const float a3 = (rng_uniform(rs) - 0.5f) * pert;
  float s1, c1, s2, c2, s3, c3;
  d_sincosf(a1, &s1, &c1); d_sincosf(a2, &s2, &c2); d_sincosf(a3, &s3, &c3);
  const float R0 = c2 * c3, R1 = c3 * s1 * s2 - c1 * s3, R2 = s1 * s3 + c1 * c3 * s2;
  const float R3 = c2 * s3, R4 = c1 * c3 + s1 * s2 * s3, R5 = c1 * s2 * s3 - c3 * s1;
  const float R6 = -s2, R7 = c2 * s1, R8 = c1 * c2;
  float4 np = make_float4(R0 * normal.x + R1 * normal.y + R2 * normal.z,
                          R3 * normal.x + R4 * normal.y + R5 * normal.z,
                          R6 * normal.x + R7 * normal.y + R8 * normal.z, normal.w);
  if (np.x * vd.x + np.y * vd.y + np.z * vd.z >= 0.0f) np = normal;
  normalize3(np);
  return np;
}

// The refinement draws of PlaneHypothesisRefinement (DPE.cu:1081-1093: a uniform depth,
// GenerateRandomNormal, a uniform perturbed depth, GeneratePerturbedNormal's three angles) sit at
// fixed stream positions from word w0 on: the rejection loop's length depends on the draws only.
// So their data-independent part can be evaluated on other lanes, ahead of the data-dependent rest
// (the view-direction flips, the rotation of the accepted plane, normalisation): same values, same
// order of operations as random_normal / perturbed_normal.
struct RefineDraws {
  float u_depth;          // uniform of the random depth
  float n[3];             // random normal before the view-direction flip
  float u_pert;           // uniform of the perturbed depth
  uint32_t w_angles;      // stream word of the first angle
};
DEV RefineDraws refine_draws(const Rng& rs, uint32_t w0) {
  RefineDraws d;
  d.u_depth = u32_to_uniform(rng_word(rs, w0));
  uint32_t w = w0 + 1;
  float q1 = 1.0f, q2 = 1.0f, s = 2.0f;
  while (s >= 1.0f) {
    q1 = 2.0f * u32_to_uniform(rng_word(rs, w)) - 1.0f;
    q2 = 2.0f * u32_to_uniform(rng_word(rs, w + 1)) - 1.0f;
    s = q1 * q1 + q2 * q2;
    w += 2;
  }
  const float sq = __builtin_sqrtf(1.0f - s);
  d.n[0] = 2.0f * q1 * sq; d.n[1] = 2.0f * q2 * sq; d.n[2] = 1.0f - 2.0f * s;
  d.u_pert = u32_to_uniform(rng_word(rs, w));
  d.w_angles = w + 1;
  return d;
}
// angle k (0..2) of GeneratePerturbedNormal: its sine and cosine
DEV void refine_angle(const Rng& rs, uint32_t w_angles, int k, float pert, float* s, float* c) {
  const float a = (u32_to_uniform(rng_word(rs, w_angles + (uint32_t)k)) - 0.5f) * pert;
  d_sincosf(a, s, c);
}
// random_normal from its pre-flip normal
DEV float4 random_normal_from(const DpeCamera& c, int px, int py, const float* n0, float depth) {
  float4 n = make_float4(n0[0], n0[1], n0[2], 0.0f);
  const float4 vd = view_direction(c, px, py, depth);
  if (n.x * vd.x + n.y * vd.y + n.z * vd.z > 0.0f) { n.x = -n.x; n.y = -n.y; n.z = -n.z; }
  normalize3(n);
  return n;
}
// perturbed_normal from the angles' sines and cosines sc = {s1, c1, s2, c2, s3, c3}
DEV float4 perturbed_normal_from(const DpeCamera& c, int px, int py, const float4& normal, const float* sc) {
  const float4 vd = view_direction(c, px, py, 1.0f);
  const float s1 = sc[0], c1 = sc[1], s2 = sc[2], c2 = sc[3], s3 = sc[4], c3 = sc[5];
  const float R0 = c2 * c3, R1 = c3 * s1 * s2 - c1 * s3, R2 = s1 * s3 + c1 * c3 * s2;
  const float R3 = c2 * s3, R4 = c1 * c3 + s1 * s2 * s3, R5 = c1 * s2 * s3 - c3 * s1;
  const float R6 = -s2, R7 = c2 * s1, R8 = c1 * c2;
  float4 np = make_float4(R0 * normal.x + R1 * normal.y + R2 * normal.z,
                          R3 * normal.x + R4 * normal.y + R5 * normal.z,
                          R6 * normal.x + R7 * normal.y + R8 * normal.z, normal.w);
  if (np.x * vd.x + np.y * vd.y + np.z * vd.z >= 0.0f) np = normal;
  normalize3(np);
  return np;
}

// ------------------------------------------------------------------------------ homography
// H = M_v - b_v g^T, g = Kref^-T (n/w) (restatement of ComputeHomography, DPE.cu:453-513).
struct Homog { float h[9]; };
DEV Homog make_homography(const PassConst& pc, int v, const float4& pl) {
  const float iw = 1.0f / pl.w;
  const float qx = pl.x * iw, qy = pl.y * iw, qz = pl.z * iw;
  const float g0 = qx * pc.kinv0;
  const float g1 = qy * pc.kinv4;
  const float g2 = __builtin_fmaf(-qx, pc.kc2, __builtin_fmaf(-qy, pc.kc5, qz));
  const ViewConst& vc = pc.vc[v];
  Homog H;
  H.h[0] = __builtin_fmaf(-vc.b[0], g0, vc.M[0]);
  H.h[1] = __builtin_fmaf(-vc.b[0], g1, vc.M[1]);
  H.h[2] = __builtin_fmaf(-vc.b[0], g2, vc.M[2]);
  H.h[3] = __builtin_fmaf(-vc.b[1], g0, vc.M[3]);
  H.h[4] = __builtin_fmaf(-vc.b[1], g1, vc.M[4]);
  H.h[5] = __builtin_fmaf(-vc.b[1], g2, vc.M[5]);
  H.h[6] = __builtin_fmaf(-vc.b[2], g0, vc.M[6]);
  H.h[7] = __builtin_fmaf(-vc.b[2], g1, vc.M[7]);
  H.h[8] = __builtin_fmaf(-vc.b[2], g2, vc.M[8]);
  return H;
}
DEV float2 project_h(const Homog& H, float x, float y) {   // ComputeCorrespondingPoint (DPE.cu:515-522)
  const float px = __builtin_fmaf(H.h[1], y, __builtin_fmaf(H.h[0], x, H.h[2]));
  const float py = __builtin_fmaf(H.h[4], y, __builtin_fmaf(H.h[3], x, H.h[5]));
  const float pz = __builtin_fmaf(H.h[7], y, __builtin_fmaf(H.h[6], x, H.h[8]));
  const float iz = 1.0f / pz;
  return make_float2(px * iz, py * iz);
}

// True when every tap (x, y) of the rectangle [x0, x1] x [y0, y1] computes its projective
// denominator qz = fma(h7, y, fma(h6, x, h8)) with a biased exponent in [1, 252]: there the bare
// v_rcp_f32 (rcp_tap<true>) is the tap reciprocal of restatement choice 8 (the rcp_model / oracle
// o_rcp_tap table value) with no per-tap range test, and project_h_fast's d_rcp_fast is
// bit-identical to 1.0f / z.  qz is affine in (x, y): its exact values over the
// rectangle lie between the four corner values (evaluated here with the taps' own formula), and
// a tap's computed value is within 2^-22 * max(|bz|, |qz|) of the exact one.  Same sign at the
// corners, a minimum magnitude well above that error and above 2^-100, and magnitudes below 2^100
// give the range with a wide margin.  NaN/inf anywhere -> false.
DEV bool rcp_range_ok(const Homog& H, float x0, float x1, float y0, float y1) {
  const float b0 = __builtin_fmaf(H.h[6], x0, H.h[8]), b1 = __builtin_fmaf(H.h[6], x1, H.h[8]);
  const float q00 = __builtin_fmaf(H.h[7], y0, b0), q01 = __builtin_fmaf(H.h[7], y1, b0);
  const float q10 = __builtin_fmaf(H.h[7], y0, b1), q11 = __builtin_fmaf(H.h[7], y1, b1);
  const float mn = __builtin_fminf(__builtin_fminf(q00, q01), __builtin_fminf(q10, q11));
  const float mx = __builtin_fmaxf(__builtin_fmaxf(q00, q01), __builtin_fmaxf(q10, q11));
  const float amax = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(b0), __builtin_fabsf(b1)),
                                     __builtin_fmaxf(__builtin_fabsf(mn), __builtin_fabsf(mx)));
  const float lo = mn > 0.0f ? mn : -mx;
  return (mn > 0.0f || mx < 0.0f) && lo > amax * 9.5367431640625e-07f && lo > 7.888609052210118e-31f &&
         amax < 1.2676506002282294e+30f;
}

// Round 6: true when, besides rcp_range_ok, every tap (x, y) of the box [x0, x1] x [y0, y1] has its
// computed t = fma(Qx, iz, kTexMagic + 1) strictly inside the clamp range (kTexMagic, kTexMagic + W + 1)
// (and the same for y with H), so tex_t_fast's med3 returns t itself and the taps can skip it: the
// same bits.  Why it suffices (s = Qx / qz, the tap's exact coordinate; the clamp range is s in
// [-1, W]):
//  * qz, Qx, Qy are affine in (x, y) and qz keeps one sign over the box (rcp_range_ok), so each tap's
//    exact s lies between the exact corner values;
//  * each corner is tested with the taps' own FMAs: Qx >= 0 and fma(W - 1, qz, -Qx) >= 0 (times the
//    sign of qz), i.e. s in [0, W - 1] up to the rounding of those values, below 0.01 texel under
//    the two magnitude conditions below;
//  * a tap's computed t differs from s + kTexMagic + 1 by at most 0.15 texel: qz is one FMA of
//    (h7 y) and b = fma(h6, x, h8), so its relative error is <= 2^-24 (1 + |b| / |qz|) <= 2^-17 when
//    min |qz| >= 2^-6 max |b, qz| (condition 1); v_rcp_f32 adds 2^-22; Qx's absolute error is
//    <= 2^-24 (|Qx| + 2 |bx|) and |bx| <= 2^16 min |qz| (condition 2) makes it <= 2^-6.8 texel after
//    the division; |s| < 2^14 (images narrower than 16383 px) gives |s| 2^-16.9 < 0.14; the final
//    rounding of t adds 2^-9 -- the corner margin of one texel on each side covers all of it.
DEV bool taps_unclamped(const Homog& H, float x0, float x1, float y0, float y1, float wm1, float hm1) {
  const float b0 = __builtin_fmaf(H.h[6], x0, H.h[8]), b1 = __builtin_fmaf(H.h[6], x1, H.h[8]);
  const float q00 = __builtin_fmaf(H.h[7], y0, b0), q01 = __builtin_fmaf(H.h[7], y1, b0);
  const float q10 = __builtin_fmaf(H.h[7], y0, b1), q11 = __builtin_fmaf(H.h[7], y1, b1);
  const float mn = __builtin_fminf(__builtin_fminf(q00, q01), __builtin_fminf(q10, q11));
  const float mx = __builtin_fmaxf(__builtin_fmaxf(q00, q01), __builtin_fmaxf(q10, q11));
  const float amax = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(b0), __builtin_fabsf(b1)),
                                     __builtin_fmaxf(__builtin_fabsf(mn), __builtin_fabsf(mx)));
  const float sg = mn > 0.0f ? 1.0f : -1.0f;
  const float lo = mn > 0.0f ? mn : -mx;
  const float bx0 = __builtin_fmaf(H.h[0], x0, H.h[2]), bx1 = __builtin_fmaf(H.h[0], x1, H.h[2]);
  const float by0 = __builtin_fmaf(H.h[3], x0, H.h[5]), by1 = __builtin_fmaf(H.h[3], x1, H.h[5]);
  const float bmax = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(bx0), __builtin_fabsf(bx1)),
                                     __builtin_fmaxf(__builtin_fabsf(by0), __builtin_fabsf(by1)));
  bool ok = lo >= amax * 0.015625f && bmax <= lo * 65536.0f;
  const float bxs[2] = {bx0, bx1}, bys[2] = {by0, by1}, qs[4] = {q00, q01, q10, q11}, ys[2] = {y0, y1};
  float m = 3.40282347e+38f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float qz = qs[k] * sg;
    const float X = __builtin_fmaf(H.h[1], ys[k & 1], bxs[k >> 1]) * sg;
    const float Y = __builtin_fmaf(H.h[4], ys[k & 1], bys[k >> 1]) * sg;
    m = __builtin_fminf(m, __builtin_fminf(__builtin_fminf(X, Y),
                                           __builtin_fminf(__builtin_fmaf(wm1, qz, -X), __builtin_fmaf(hm1, qz, -Y))));
  }
  return ok && m >= 0.0f;
}

// ------------------------------------------------------------------------------ sampling
DEV float ref_texel(const float* ref, int W, int H, int x, int y) {
  x = x < 0 ? 0 : (x > W - 1 ? W - 1 : x);
  y = y < 0 ? 0 : (y > H - 1 ? H - 1 : y);
  return ref[y * W + x];
}
// ------------------------------------------------------------------------------ tap coordinates
// The texture unit's coordinate conversion (tex2D(x + 0.5) with linear filtering and clamp
// addressing, DPE.cpp:927-933), restated (round 3; oracle OracleSampleQ):
// a tap whose homography rows give (qx, qy, qz) reads the padded quad texel (Ux >> 8, Uy >> 8) with
// weights (Ux & 255) / 256, (Uy & 255) / 256, where
//     U = clamp(RN_even(Q * iz + 256), 0, 256 * lim + 256),   Q = 256 q (exact),  iz = rcp_tap(qz)
// (round 5, restatement choice 8: iz is gfx950's v_rcp_f32 of qz, within 1 ulp of 1/qz and not
// correctly rounded, for biased exponents 1..252; IEEE 1/qz outside; rounds 3-4 used RN(1 / qz))
// i.e. the coordinate s + 1 = q / qz + 1 in 1/256 units rounded to nearest ONCE.  The rows are
// pre-scaled by 256 (power of two: exact), and t = fma(Q, iz, 1.5·2^23 + 256) lands on the unit grid
// of [2^23, 2^24), so t's encoding minus that of 1.5·2^23 is U: one FMA per coordinate (round 2 used
// trunc(fma(q·iz, 256, 256.5)): a multiply, an FMA, a clamp and a half-rate conversion).  The clamp
// is taken on t (monotone; NaN -> the low end), and the bound |256 s + 256| < 2^22 for unclamped taps
// holds for images narrower than 16383 px (dpe_pm_stage checks).
// Round 3: the same U on the 1/256-unit grid of [2^15, 2^16) instead of the unit grid
// of [2^23, 2^24): t' = fma(q, iz, 1.5·2^15 + 1) = t / 256 exactly (scaling by a power of two commutes
// with the FMA's one rounding, and the row terms are no longer scaled), its encoding still differs
// from that of 1.5·2^15 by U, and the tap's weight (U & 255) / 256 is v_fract_f32(t') straight from
// the float (one full-rate op in place of v_cvt_f32_ubyte0 + a multiply per axis).
constexpr float kTexMagic = 49152.0f;             // 1.5 * 2^15
constexpr uint32_t kTexMagicBits = 0x47400000u;   // its encoding
constexpr uint32_t kTexMagicHi = 0x474000u;       // encoding >> 8: texel index bias of t >> 8
constexpr float kTexUnit = 1.0f;                  // one texel in t units
DEV float tex_tmax(int lim) { return kTexMagic + kTexUnit * (float)(lim + 1); }   // t of U = 256 lim + 256
// clamped t of a tap with scaled row value Q (generic path: NaN -> kTexMagic)
DEV float tex_t(float Q, float iz, float tmax) {
  const float t = __builtin_fmaf(Q, iz, kTexMagic + kTexUnit);
  return __builtin_fminf(__builtin_fmaxf(t, kTexMagic), tmax);
}
// bilinear weight (U & 255) / 256 of a clamped t whose encoding is `bits`
DEV float tex_frac(float t, uint32_t bits) {
  (void)bits;
  return __builtin_amdgcn_fractf(t);
}
// The taps' numerators Q = 256 q: the column coefficients h1, h4 scaled by 256 here, the row terms
// (h0 x + h2, h3 x + h5) scaled after their FMA (the oracle's OracleSampleQ caller does the same).
DEV Homog scale_cols(const Homog& H) {
  Homog S = H;
  S.h[1] = H.h[1] * kTexUnit;
  S.h[4] = H.h[4] * kTexUnit;
  return S;
}

// Bilinear sample with 8-bit weights on the padded quad image (see oracle OracleSampleQ), at the
// tap with scaled numerators (Qx, Qy) and reciprocal denominator iz.
DEV float sample_quad(const float4* __restrict__ q, int W, int H, float Qx, float Qy, float iz) {
  const float tx = tex_t(Qx, iz, tex_tmax(W)), ty = tex_t(Qy, iz, tex_tmax(H));
  const uint32_t ux = __float_as_uint(tx) - kTexMagicBits;
  const uint32_t uy = __float_as_uint(ty) - kTexMagicBits;
  const float ax = tex_frac(tx, ux);
  const float ay = tex_frac(ty, uy);
  const float4 t = q[(uy >> 8) * (W + 2) + (ux >> 8)];
  const float r0 = __builtin_fmaf(ax, t.y - t.x, t.x);
  const float r1 = __builtin_fmaf(ax, t.w - t.z, t.z);
  return __builtin_fmaf(ay, r1 - r0, r0);
}
// Source-image layouts, the kernels' `U8` template argument: TEX_F32 is the f32 quad image (any
// grey levels); the other two hold 8-bit grey levels.  A quad texel holds the 2x2 neighbourhood
// a=(x0,y0), b=(x1,y0), c=(x0,y1), d=(x1,y1) of its bilinear footprint:
//   TEX_U8:  4 B, bytes (a, b, c, d)
//   TEX_F16: 8 B, f16 (a, c, b-a, d-c): all exact (integers of magnitude <= 255), so each row
//     interpolation is one v_fma_mix_f32 on the loaded halves with the weight fx/256 (exact),
//     bit for bit the reference's fma(fx/256, b-a, a): 7 fewer VALU ops per tap than TEX_U8 for
//     twice the bytes.
//   TEX_P16: 4 B column pairs, f16 (g(X-1, Y-1), g(X-1, Y)) at (X, Y), row stride W + 3: the quad
//     texel (X, Y) is the 8 B at pair X (a, c) and pair X+1 (b, d), read with one unaligned 8-B
//     load; the row differences are one packed f16 subtraction (exact: integers <= 255), so each row
//     interpolation is again one v_fma_mix_f32, now with fx/256 (exact) times (b-a): 2 more VALU ops
//     per tap than TEX_F16 for half the footprint (and a layout whose windows copy as plain rows).
enum { TEX_F32 = 0, TEX_U8 = 1, TEX_F16 = 2, TEX_P16 = 3 };
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef uint2 uint2_a4 __attribute__((aligned(4)));
template <int T> DEV const uint8_t* tex_base(const DevBufs& B) {
  return T == TEX_F16 ? B.img16 : (T == TEX_P16 ? B.imgp : B.img8);
}
template <int T> DEV uint32_t tex_view(const DevBufs& B) {
  return T == TEX_F16 ? B.img16_view : (T == TEX_P16 ? B.imgp_view : B.img8_view);
}
template <int T> constexpr uint32_t tex_bytes() { return T == TEX_F16 ? 8u : 4u; }
template <int T> DEV uint32_t tex_stride(int W) { return (uint32_t)(W + (T == TEX_P16 ? 3 : 2)); }
// the two row interpolations (r0 at y0, r1 at y1) of the texel at `p` for the x weight ax = fx / 256
// texel loads of the fast taps; DPE_FAKE_GATHER (timing only): f16 values in [128, 256) / bytes made
// from the address bits instead of memory
#if DPE_FAKE_GATHER
DEV uint2 fake_texel2(const uint8_t* p) {
  const uint32_t a = (uint32_t)(uintptr_t)p;
  uint2 v; v.x = 0x58005800u | (a & 0x03FF03FFu); v.y = 0x58005800u | ((a >> 3) & 0x03FF03FFu);
  return v;
}
#define LD_TEXEL_P16(p) fake_texel2(p)
#define LD_TEXEL_F16(p) fake_texel2(p)
#define LD_TEXEL_U8(p) ((uint32_t)(uintptr_t)(p) & 0x7F7F7F7Fu)
#else
#define LD_TEXEL_P16(p) (*(const uint2_a4*)(p))
#define LD_TEXEL_F16(p) (*(const uint2*)(p))
#define LD_TEXEL_U8(p) (*(const uint32_t*)(p))
#endif
template <int T>
DEV void texel_rows(const uint8_t* p, float ax, float& r0, float& r1) {
  if constexpr (T == TEX_P16) {
    const uint2 t = LD_TEXEL_P16(p);                     // (a, c), (b, d)
    const h2v df = __builtin_bit_cast(h2v, t.y) - __builtin_bit_cast(h2v, t.x);
    const uint32_t d = __builtin_bit_cast(uint32_t, df);
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(r0) : "v"(ax), "v"(d), "v"(t.x));
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,1] op_sel_hi:[0,1,1]" : "=v"(r1) : "v"(ax), "v"(d), "v"(t.x));
  } else if constexpr (T == TEX_F16) {
    // v_fma_mix_f32 is fma(ax, (float)half, (float)half) with one rounding; the compiler only forms
    // it under f32 denormal flushing, which cannot matter here (|ax*d| >= 2^-8 or 0, a integer)
    const uint2 t = LD_TEXEL_F16(p);
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(r0) : "v"(ax), "v"(t.y), "v"(t.x));
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,1] op_sel_hi:[0,1,1]" : "=v"(r1) : "v"(ax), "v"(t.y), "v"(t.x));
  } else {
    const uint32_t t = LD_TEXEL_U8(p);
    const float t00 = (float)(t & 255u), t10 = (float)((t >> 8) & 255u);
    const float t01 = (float)((t >> 16) & 255u), t11 = (float)(t >> 24);
    r0 = __builtin_fmaf(ax, t10 - t00, t00);
    r1 = __builtin_fmaf(ax, t11 - t01, t01);
  }
}
// Same sampler on the 8-bit quad texels of one view: identical values to the f32 layout's.
template <int T>
DEV float sample_quad8(const uint8_t* __restrict__ q, int W, int H, float Qx, float Qy, float iz) {
  const float tx = tex_t(Qx, iz, tex_tmax(W)), ty = tex_t(Qy, iz, tex_tmax(H));
  const uint32_t ux = __float_as_uint(tx) - kTexMagicBits;
  const uint32_t uy = __float_as_uint(ty) - kTexMagicBits;
  const float ay = tex_frac(ty, uy);
  float r0, r1;
  texel_rows<T>(q + (size_t)((uy >> 8) * tex_stride<T>(W) + (ux >> 8)) * tex_bytes<T>(), tex_frac(tx, ux), r0, r1);
  return __builtin_fmaf(ay, r1 - r0, r0);
}
// The default 36-tap patch (strong radius 5, increment 2) that the tabulated fast paths serve.
// (a macro, not a function: the short-circuit keeps the second load behind a branch, as in round 4)
#define FAST_PATCH(pc) ((pc).P.strong_radius == 5 && (pc).P.strong_increment == 2)
// Minimum waves per SIMD the tap-heavy kernels are compiled for (register cap 512 / waves).
constexpr int kTapWaves = 4;

typedef float f2v __attribute__((ext_vector_type(2)));
DEV f2v f2s(float a) { return (f2v){a, a}; }
DEV f2v fma2(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }

// Gather-locality diagnostic (DPE_DIAG & 2; tools/line_stats.py): for every wave
// gather of a fast-path tap, the number of distinct 128-B lines and 64-B sectors its active lanes
// touch, summed per texel layout T in a per-translation-unit device array (read back with
// dpe_dbg_line_stats).  Off in the product.
#if DPE_LINE_STATS
static __device__ unsigned long long g_lstat[4][4];   // [T][loads, lines, quad lines, active lanes]
DEV void line_stat(int T, const void* p) {
  const uint64_t a = (uint64_t)p;
  uint64_t rem = __ballot(1);
  const int first = __builtin_ctzll(rem);
  const unsigned long long act = __popcll(rem);
  unsigned long long nl = 0, ns = 0;
  {   // the texture-address cost: sum over lane quads of the distinct lines each quad touches
    const int lane = threadIdx.x & 63, q0 = lane & ~3;
    bool firstl = true;
    for (int j = 0; j < 4; ++j) {
      const uint64_t o = __shfl(a >> 7, q0 + j);
      if (q0 + j < lane && ((rem >> (q0 + j)) & 1) && o == (a >> 7)) firstl = false;
    }
    ns = __popcll(__ballot(firstl));
  }
  uint64_t r = rem;
  while (r) {
    const int l = __builtin_ctzll(r);
    const uint64_t L = __shfl(a >> 7, l);
    r &= ~__ballot((a >> 7) == L);
    ++nl;
  }
  if ((int)(threadIdx.x & 63) == first) {
    atomicAdd(&g_lstat[T][0], 1ull); atomicAdd(&g_lstat[T][1], nl);
    atomicAdd(&g_lstat[T][2], ns); atomicAdd(&g_lstat[T][3], act);
  }
}
#define LINE_STAT(T, p) line_stat(T, p)
#else
#define LINE_STAT(T, p) do {} while (0)
#endif

// Fast-path tap constants of one (view, homography): the t clamps of the two axes and the view's
// byte offset biased so that the t encodings index texels directly:
//   offset = vofs + ((Uy >> 8) * stride + (Ux >> 8)) * bytes
//          = vadj + ((bits(ty) >> 8) * stride + (bits(tx) >> 8)) * bytes   (mod 2^32)
// with vadj = vofs - kTexMagicHi * (stride + 1) * bytes (bits(t) >> 8 = kTexMagicHi + (U >> 8) < 2^24,
// so __umul24 sees the whole operand; the true offset is below 2^32, so the wrap-around cancels).
DEV f2v tex_tmax2(int W, int H) { return (f2v){tex_tmax(W), tex_tmax(H)}; }
template <int T> DEV uint32_t tex_vadj(uint32_t vofs, uint32_t stride) {
  return vofs - kTexMagicHi * (stride + 1u) * tex_bytes<T>();
}
// clamped t of the fast path (no NaN there: rcp_range_ok)
DEV float tex_t_fast(float t, float tmax) { return __builtin_amdgcn_fmed3f(t, kTexMagic, tmax); }

// One bilinear tap of the 8-bit quad image (layout T) at the view offset `vadj` (tex_vadj), from
// the homography h with scaled column coefficients (scale_cols) and its row terms
// bxy = 256 (h0 x + h2, h3 x + h5), bz = h6 x + h8; column yf.  Bit-identical to sample_quad8 with
// rcp_model's reciprocal when the tap's qz has a biased exponent in [1, 252] (rcp_range_ok), where
// the bare v_rcp_f32 is restatement choice 8's tap reciprocal.
template <int T>
DEV float tap_u8_fast(const DevBufs& B, uint32_t vadj, uint32_t stride, f2v tmax, const float* h, f2v bxy, float bz,
                      float yf) {
  const f2v q = fma2((f2v){h[1], h[4]}, f2s(yf), bxy);
  const float iz = rcp_tap<true>(__builtin_fmaf(h[7], yf, bz));
  const f2v t = fma2(q, f2s(iz), f2s(kTexMagic + kTexUnit));
  const float ctx = tex_t_fast(t.x, tmax.x), cty = tex_t_fast(t.y, tmax.y);
  const uint32_t ux = __float_as_uint(ctx), uy = __float_as_uint(cty);
  const uint8_t* p = tex_base<T>(B) + (vadj + (__umul24(uy >> 8, stride) + (ux >> 8)) * tex_bytes<T>());
  LINE_STAT(T, p);
  const float ay = tex_frac(cty, uy);
  if constexpr (T == TEX_F16 || T == TEX_P16) {
    float r0, r1;
    texel_rows<T>(p, tex_frac(ctx, ux), r0, r1);
    return __builtin_fmaf(ay, r1 - r0, r0);
  } else {
    const uint32_t tt = LD_TEXEL_U8(p);
    const float ax = tex_frac(ctx, ux);
    const f2v lo = (f2v){(float)(tt & 255u), (float)((tt >> 16) & 255u)};
    const f2v hi = (f2v){(float)((tt >> 8) & 255u), (float)(tt >> 24)};
    const f2v r = fma2(f2s(ax), hi - lo, lo);
    return __builtin_fmaf(ay, r.y - r.x, r.x);
  }
}

// Two taps of one patch row (columns yf.x, yf.y) with the projection, reciprocal refinement and
// the coordinate FMAs packed across the two taps; per element the same operations as tap_u8_fast,
// so each result is bit-identical to it.
// `base` is the texel array the byte offsets index (tex_base of the layout; vadj selects the view).
template <int T, bool CLAMP = true>
DEV f2v tap2_at(const uint8_t* base, uint32_t vadj, uint32_t stride, f2v tmax, const float* h, f2v bxy, float bz, f2v yf) {
  const f2v qx = fma2(f2s(h[1]), yf, f2s(bxy.x));
  const f2v qy = fma2(f2s(h[4]), yf, f2s(bxy.y));
  const f2v qz = fma2(f2s(h[7]), yf, f2s(bz));
  const f2v iz = (f2v){rcp_tap<true>(qz.x), rcp_tap<true>(qz.y)};
  const f2v tx = fma2(qx, iz, f2s(kTexMagic + kTexUnit)), ty = fma2(qy, iz, f2s(kTexMagic + kTexUnit));
  // CLAMP = false: the caller proved every tap inside the clamp range (taps_unclamped), where the
  // clamp returns t itself
  const float cx0 = CLAMP ? tex_t_fast(tx.x, tmax.x) : tx.x, cx1 = CLAMP ? tex_t_fast(tx.y, tmax.x) : tx.y;
  const float cy0 = CLAMP ? tex_t_fast(ty.x, tmax.y) : ty.x, cy1 = CLAMP ? tex_t_fast(ty.y, tmax.y) : ty.y;
  const uint32_t ux0 = __float_as_uint(cx0), ux1 = __float_as_uint(cx1);
  const uint32_t uy0 = __float_as_uint(cy0), uy1 = __float_as_uint(cy1);
  const uint8_t* p0 = base + (vadj + (__umul24(uy0 >> 8, stride) + (ux0 >> 8)) * tex_bytes<T>());
  const uint8_t* p1 = base + (vadj + (__umul24(uy1 >> 8, stride) + (ux1 >> 8)) * tex_bytes<T>());
  LINE_STAT(T, p0);
  LINE_STAT(T, p1);
  const f2v ay = (f2v){tex_frac(cy0, uy0), tex_frac(cy1, uy1)};
  float a0, a1, b0, b1;
  texel_rows<T>(p0, tex_frac(cx0, ux0), a0, a1);
  texel_rows<T>(p1, tex_frac(cx1, ux1), b0, b1);
  const f2v r0 = (f2v){a0, b0}, r1 = (f2v){a1, b1};
  return fma2(ay, r1 - r0, r0);
}
template <int T>
DEV f2v tap2_fast(const DevBufs& B, uint32_t vadj, uint32_t stride, f2v tmax, const float* h, f2v bxy, float bz, f2v yf) {
  return tap2_at<T>(tex_base<T>(B), vadj, stride, tmax, h, bxy, bz, yf);
}

// Sample of view v at the tap with scaled numerators (Qx, Qy) and reciprocal denominator iz.
template <int U8> DEV float sample_src(const DevBufs& B, int v, int W, int H, float Qx, float Qy, float iz) {
  if constexpr (U8 != TEX_F32) return sample_quad8<U8>(tex_base<U8>(B) + (size_t)v * tex_view<U8>(B), W, H, Qx, Qy, iz);
  else return sample_quad(B.imgq[v], W, H, Qx, Qy, iz);
}

DEV float depth_texel(const float* d, int W, int H, float x, float y) {   // DPE.cu:936
  return ref_texel(d, W, H, f2i(x), f2i(y));
}

// ComputeBilateralWeight (DPE.cu:550-555)
DEV float bilateral_weight(int i, int j, float pix, float cpix, float ss, float sc) {
  const float xd = (float)i, yd = (float)j;
  const float sd = __builtin_sqrtf(xd * xd + yd * yd);
  const float cd = __builtin_fabsf(pix - cpix);
  return d_expf(-sd / (2.0f * ss * ss) - cd / (2.0f * sc * sc));
}

// The reference-patch half of ncc_finalize, computed once per patch: (1/s_w, s_ref/s_w, var_ref)
// with the same operations, so ncc_finalize_pre(pre..., src sums) == ncc_finalize(ref sums, src sums).
DEV void ncc_pre(float s_ref, float s_rr, float s_w, float& inv, float& mref, float& var_ref) {
  inv = 1.0f / s_w;
  mref = s_ref * inv;
  const float mrr = s_rr * inv;
  var_ref = mrr - mref * mref;
}
DEV float ncc_finalize_pre(float inv, float mref, float var_ref, float s_src, float s_ss, float s_rs) {
  s_src *= inv; s_ss *= inv; s_rs *= inv;
  const float var_src = s_ss - s_src * s_src;
  if (var_ref < 1e-5f || var_src < 1e-5f) return 2.0f;
  const float cov = s_rs - mref * s_src;
  const float vrs = __builtin_sqrtf(var_ref * var_src);
  return __builtin_fmaxf(0.0f, __builtin_fminf(2.0f, 1.0f - cov / vrs));
}
DEV float ncc_finalize(float s_ref, float s_rr, float s_w, float s_src, float s_ss, float s_rs) {
  const float inv = 1.0f / s_w;
  s_ref *= inv; s_rr *= inv; s_src *= inv; s_ss *= inv; s_rs *= inv;
  const float var_ref = s_rr - s_ref * s_ref;
  const float var_src = s_ss - s_src * s_src;
  if (var_ref < 1e-5f || var_src < 1e-5f) return 2.0f;
  const float cov = s_rs - s_ref * s_src;
  const float vrs = __builtin_sqrtf(var_ref * var_src);
  return __builtin_fmaxf(0.0f, __builtin_fminf(2.0f, 1.0f - cov / vrs));
}

// Generic bilateral NCC of one patch, weights computed per tap (NCC-New neighbour patches and
// non-default radius/increment).  Same arithmetic order as the oracle's PatchNCC.
template <int U8, bool FAST>
DEV void generic_taps(const PassConst& pc, const DevBufs& B, int v, const Homog& H0, int cx, int cy, float rcp,
                      int radius, int increment, float* acc) {
  const int W = pc.W, Hh = pc.H;
  const Homog H = scale_cols(H0);
  const float ss = pc.P.sigma_spatial, sc = pc.P.sigma_color;
  float s_ref = 0, s_rr = 0, s_src = 0, s_ss = 0, s_rs = 0, s_w = 0;
  for (int i = -radius; i <= radius; i += increment) {
    float r_ref = 0, r_src = 0, r_rr = 0, r_ss = 0, r_rs = 0, r_w = 0;
    const int x = cx + i;
    const float xf = (float)x;
    const float bx = __builtin_fmaf(H.h[0], xf, H.h[2]) * kTexUnit;
    const float by = __builtin_fmaf(H.h[3], xf, H.h[5]) * kTexUnit;
    const float bz = __builtin_fmaf(H.h[6], xf, H.h[8]);
    for (int j = -radius; j <= radius; j += increment) {
      const int y = cy + j;
      const float rp = ref_texel(B.ref, W, Hh, x, y);
      const float yf = (float)y;
      const float qx = __builtin_fmaf(H.h[1], yf, bx);
      const float qy = __builtin_fmaf(H.h[4], yf, by);
      const float iz = rcp_tap<FAST>(__builtin_fmaf(H.h[7], yf, bz));
      const float sp = sample_src<U8>(B, v, W, Hh, qx, qy, iz);
      const float w = bilateral_weight(i, j, rp, rcp, ss, sc);
      const float wr = w * rp;
      r_ref = r_ref + wr;
      r_rr = __builtin_fmaf(wr, rp, r_rr);
      r_src = __builtin_fmaf(w, sp, r_src);
      const float ws = w * sp;
      r_ss = __builtin_fmaf(ws, sp, r_ss);
      r_rs = __builtin_fmaf(wr, sp, r_rs);
      r_w = r_w + w;
    }
    s_ref += r_ref; s_rr += r_rr; s_src += r_src; s_ss += r_ss; s_rs += r_rs; s_w += r_w;
  }
  acc[0] = s_ref; acc[1] = s_rr; acc[2] = s_src; acc[3] = s_ss; acc[4] = s_rs; acc[5] = s_w;
}

// Generic bilateral NCC of one patch, weights computed per tap (NCC-New neighbour patches and
// non-default radius/increment).  Same arithmetic order as the oracle's PatchNCC.
template <int U8>
DEV float patch_ncc_generic(const PassConst& pc, const DevBufs& B, int v, const Homog& H,
                            int cx, int cy, float rcp, int radius, int increment) {
  float a[6];
  if (rcp_range_ok(H, (float)(cx - radius), (float)(cx + radius), (float)(cy - radius), (float)(cy + radius)))
    generic_taps<U8, true>(pc, B, v, H, cx, cy, rcp, radius, increment, a);
  else
    generic_taps<U8, false>(pc, B, v, H, cx, cy, rcp, radius, increment, a);
  if (B.cnt) { const unsigned long long n = (unsigned long long)(2 * radius / increment + 1); count_work(B, 0, n * n); }
  return ncc_finalize(a[0], a[1], a[5], a[2], a[3], a[4]);
}

// project_h with the exact 3-op reciprocal (callers guarantee rcp_range_ok over a box holding (x, y))
DEV float2 project_h_fast(const Homog& H, float x, float y) {
  const float px = __builtin_fmaf(H.h[1], y, __builtin_fmaf(H.h[0], x, H.h[2]));
  const float py = __builtin_fmaf(H.h[4], y, __builtin_fmaf(H.h[3], x, H.h[5]));
  const float pz = __builtin_fmaf(H.h[7], y, __builtin_fmaf(H.h[6], x, H.h[8]));
  const float iz = d_rcp_fast(pz);
  return make_float2(px * iz, py * iz);
}
template <bool FAST = false>
DEV bool center_outside(const PassConst& pc, int v, const Homog& H, int px, int py) {
  const float2 pt = FAST ? project_h_fast(H, (float)px, (float)py) : project_h(H, (float)px, (float)py);
  const DpeCamera& sc = pc.cams[v];
  return pt.x >= (float)sc.width || pt.x < 0.0f || pt.y >= (float)sc.height || pt.y < 0.0f;
}

// ComputeBilateralNCCOld (DPE.cu:692-778), weights per tap.
template <int U8>
DEV float ncc_old_generic(const PassConst& pc, const DevBufs& B, int px, int py, int v, const float4& pl) {
  const Homog H = make_homography(pc, v, pl);
  count_work(B, 1, 0);
  if (center_outside(pc, v, H, px, py)) return 2.0f;
  const float rc = ref_texel(B.ref, pc.W, pc.H, px, py);
  return patch_ncc_generic<U8>(pc, B, v, H, px, py, rc, pc.P.strong_radius, pc.P.strong_increment);
}

// Reference patch of the Old NCC with the default radius 5 / increment 2 (36 taps), precomputed
// once per pixel: weights and weight*ref are view- and plane-independent.
struct Patch36 {
  float w[36], wr[36];
  float s_ref, s_rr, s_w;
  int px, py;
};
DEV void make_patch36(Patch36& P, const PassConst& pc, const DevBufs& B, int px, int py) {
  const int W = pc.W, Hh = pc.H;
  const float ss = pc.P.sigma_spatial, sc = pc.P.sigma_color;
  const float rc = ref_texel(B.ref, W, Hh, px, py);
  P.px = px; P.py = py;
  float s_ref = 0, s_rr = 0, s_w = 0;
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    const int i = -5 + 2 * a;
    float r_ref = 0, r_rr = 0, r_w = 0;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const int j = -5 + 2 * b;
      const float rp = ref_texel(B.ref, W, Hh, px + i, py + j);
      const float w = bilateral_weight(i, j, rp, rc, ss, sc);
      const float wr = w * rp;
      r_ref = r_ref + wr;
      r_rr = __builtin_fmaf(wr, rp, r_rr);
      r_w = r_w + w;
      P.w[a * 6 + b] = w;
      P.wr[a * 6 + b] = wr;
    }
    s_ref += r_ref; s_rr += r_rr; s_w += r_w;
  }
  P.s_ref = s_ref; P.s_rr = s_rr; P.s_w = s_w;
}
template <int U8>
DEV void patch36_taps(const Patch36& P, const PassConst& pc, const DevBufs& B, int v, const Homog& H0, float* acc) {
  const int W = pc.W, Hh = pc.H;
  const Homog H = scale_cols(H0);
  float s_src = 0, s_ss = 0, s_rs = 0;
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    const float x = (float)(P.px - 5 + 2 * a);
    const float bx = __builtin_fmaf(H.h[0], x, H.h[2]) * kTexUnit;
    const float by = __builtin_fmaf(H.h[3], x, H.h[5]) * kTexUnit;
    const float bz = __builtin_fmaf(H.h[6], x, H.h[8]);
    float r_src = 0, r_ss = 0, r_rs = 0;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const float y = (float)(P.py - 5 + 2 * b);
      const float qx = __builtin_fmaf(H.h[1], y, bx);
      const float qy = __builtin_fmaf(H.h[4], y, by);
      const float iz = rcp_tap<true>(__builtin_fmaf(H.h[7], y, bz));
      const float sp = sample_src<U8>(B, v, W, Hh, qx, qy, iz);
      const float w = P.w[a * 6 + b], wr = P.wr[a * 6 + b];
      r_src = __builtin_fmaf(w, sp, r_src);
      const float ws = w * sp;
      r_ss = __builtin_fmaf(ws, sp, r_ss);
      r_rs = __builtin_fmaf(wr, sp, r_rs);
    }
    s_src += r_src; s_ss += r_ss; s_rs += r_rs;
  }
  acc[0] = s_src; acc[1] = s_ss; acc[2] = s_rs;
}
template <int U8>
DEV float ncc_old_patch36(const Patch36& P, const PassConst& pc, const DevBufs& B, int v, const float4& pl) {
  const Homog H = make_homography(pc, v, pl);
  if (center_outside(pc, v, H, P.px, P.py)) { count_work(B, 1, 0); return 2.0f; }
  count_work(B, 1, 36);
  float a[3];
  if (rcp_range_ok(H, (float)(P.px - 5), (float)(P.px + 5), (float)(P.py - 5), (float)(P.py + 5))) {
    patch36_taps<U8>(P, pc, B, v, H, a);
  } else {
    // the rare slow patch (per-tap reciprocal range test) through the rolled generic loop: the same
    // weights (bilateral_weight of the same texels) summed in the same order, so the same bits, and
    // the cached patch's 75 registers stay out of an unrolled slow loop (random init at occupancy 2)
    float g[6];
    generic_taps<U8, false>(pc, B, v, H, P.px, P.py, ref_texel(B.ref, pc.W, pc.H, P.px, P.py), pc.P.strong_radius,
                            pc.P.strong_increment, g);
    a[0] = g[2]; a[1] = g[3]; a[2] = g[4];
  }
  return ncc_finalize(P.s_ref, P.s_rr, P.s_w, a[0], a[1], a[2]);
}

// Old NCC through the cached patch when the pass uses the default 5/2 patch, else generic.
template <int U8>
DEV float ncc_old(const Patch36& P, bool fast, const PassConst& pc, const DevBufs& B, int v, const float4& pl) {
  if (fast) return ncc_old_patch36<U8>(P, pc, B, v, pl);
  return ncc_old_generic<U8>(pc, B, P.px, P.py, v, pl);
}

// ComputeBilateralNCCNew (DPE.cu:557-690)
template <int U8>
DEV float ncc_new(const PassConst& pc, const DevBufs& B, int px, int py, int v, const float4& pl) {
  const int W = pc.W, Hh = pc.H;
  const int center = px + py * W;
  const Homog H = make_homography(pc, v, pl);
  count_work(B, 1, 0);
  if (center_outside(pc, v, H, px, py)) return 2.0f;
  float cost = 0.0f;
  if (B.weak[center] != DPE_WEAK) return cost;
  const float rc = ref_texel(B.ref, W, Hh, px, py);
  float center_cost = 0.0f, strong_cost = 0.0f;
  int strong_count = 0;
  const short2* nb = B.nb + (size_t)center * 9;
  for (int k = 0; k < DPE_NEIGHBOUR_NUM; ++k) {
    const short2 np = nb[k];
    if (np.x == -1 || np.y == -1) continue;
    const float2 nsp = project_h(H, (float)np.x, (float)np.y);
    if (nsp.x < 0 || nsp.y < 0 || nsp.x >= (float)W || nsp.y >= (float)Hh) {
      if (k != 0) {
        const uint32_t vi = B.sel[np.x + np.y * W];
        if (isSet(vi, v - 1)) { strong_cost += 2.0f; strong_count++; }
        continue;
      }
      return 2.0f;
    }
    int radius = (k == 0 ? pc.P.strong_radius : pc.P.weak_radius);
    int increment = (k == 0 ? pc.P.strong_increment : pc.P.weak_increment);
    if (pc.P.use_radius && k == 0) {
      radius = B.radius[center];
      increment = MAXo(2, d2i(2.0 * radius / 5.0));
    }
    const float tc = patch_ncc_generic<U8>(pc, B, v, H, np.x, np.y, rc, radius, increment);
    if (k == 0) center_cost = tc;
    else { strong_cost += tc; strong_count++; }
  }
  if (strong_count == 0) cost = center_cost;
  else {
    strong_cost /= (float)strong_count;
    strong_cost = MINo(strong_cost, 2.0f);
    cost = (float)(0.25 * (double)center_cost + 0.75 * (double)strong_cost);
  }
  return cost;
}

// ComputeGeomConsistencyCost (DPE.cu:915-953), split where the view enters: the pixel's world point
// under the plane (depth_from_plane + Get3DPointonWorld) is the same for every source view, so a
// caller that scores one plane against several views computes it once (same operations, same bits).
DEV float3 geom_point(const PassConst& pc, int px, int py, const float4& pl) {
  const DpeCamera& rc = pc.cams[0];
  const float depth = depth_from_plane(rc, pl, px, py);
  return world_point((float)px, (float)py, depth, rc);
}
DEV float geom_cost_at(const PassConst& pc, const DevBufs& B, int px, int py, int v, const float3& fw) {
  if (B.cnt) atomicAdd(B.cnt + 2, 1ull);
  const DpeCamera& rc = pc.cams[0];
  const DpeCamera& sc = pc.cams[v];
  const float2 sp = project_cam(fw, sc);
  const float src_depth = depth_texel(B.depth[v], pc.W, pc.H, sp.x, sp.y);
  if (src_depth == 0.0f) return 3.0f;
  const float3 s3 = world_point(sp.x, sp.y, src_depth, sc);
  const float2 bp = project_cam(s3, rc);
  const float dc = (float)px - bp.x, dr = (float)py - bp.y;
  const float cc = __builtin_sqrtf(dc * dc + dr * dr);
  return __builtin_fminf(3.0f, cc);
}
DEV float geom_cost(const PassConst& pc, const DevBufs& B, int px, int py, int v, const float4& pl) {
  return geom_cost_at(pc, B, px, py, v, geom_point(pc, px, py, pl));
}

// ------------------------------------------------------------------------------ edges / triangles
DEV uint8_t low_edge_at(const PassConst& pc, const DevBufs& B, int idx) {
  if (idx < 0 || idx >= pc.LW * pc.LH) return 0;
  return B.edge_low[idx];
}
// BresenhamLine (DPE.cu:158-244).  The walk's positions do not depend on the map values, and the
// reference returns at the first edge pixel it meets, so the result is "any edge pixel among the
// positions the walk visits before it stops".  Positions are generated in batches of 8 and their
// loads issued together: one memory latency per batch instead of one per step.
constexpr int kBresBatch = 8;
DEV bool bresenham(const PassConst& pc, const DevBufs& B, int Ax, int Ay, int Bx, int By) {
  const int W = pc.W;
  if (B.edge[Ax + Ay * W] || B.edge[Bx + By * W]) return false;
  const float scale_x = 1.0f * pc.LW / (float)pc.W;
  const float scale_y = 1.0f * pc.LH / (float)pc.H;
  const int height = pc.LH, width = pc.LW;
  const int max_step = pc.P.high_res_img ? (int)__builtin_round(MAXo(height, width) / 60.0) : MAXo(height, width);
  for (int pass = 0; pass < 2; ++pass) {
    const int fx = pass == 0 ? Bx : Ax, fy = pass == 0 ? By : Ay;
    const int tx = pass == 0 ? Ax : Bx, ty = pass == 0 ? Ay : By;
    const int x0 = (int)MINo(__builtin_roundf(fx * scale_x), (float)(width - 1));
    const int y0 = (int)MINo(__builtin_roundf(fy * scale_y), (float)(height - 1));
    const int x1 = (int)MINo(__builtin_roundf(tx * scale_x), (float)(width - 1));
    const int y1 = (int)MINo(__builtin_roundf(ty * scale_y), (float)(height - 1));
    if (bres::walk_bytes_flat<kBresBatch>(x0, y0, x1, y1, max_step, B.edge_low, width, height)) return true;
  }
  return false;
}
// PointinTriangle (DPE.cu:135-156)
DEV bool point_in_triangle(short2 A, short2 Bp, short2 C, int Px, int Py) {
  const float ABx = (float)(Bp.x - A.x), ABy = (float)(Bp.y - A.y);
  const float BCx = (float)(C.x - Bp.x), BCy = (float)(C.y - Bp.y);
  const float CAx = (float)(A.x - C.x), CAy = (float)(A.y - C.y);
  const float AB_ = __builtin_sqrtf(ABx * ABx + ABy * ABy);
  const float BC_ = __builtin_sqrtf(BCx * BCx + BCy * BCy);
  const float CA_ = __builtin_sqrtf(CAx * CAx + CAy * CAy);
  if (AB_ <= 2 || BC_ <= 2 || CA_ <= 2) return false;
  if (!(AB_ + BC_ > CA_ && BC_ + CA_ > AB_ && AB_ + CA_ > BC_)) return false;
  const float PAx = (float)(A.x - Px), PAy = (float)(A.y - Py);
  const float PBx = (float)(Bp.x - Px), PBy = (float)(Bp.y - Py);
  const float PCx = (float)(C.x - Px), PCy = (float)(C.y - Py);
  const float t1 = PAx * PBy - PAy * PBx;
  const float t2 = PBx * PCy - PBy * PCx;
  const float t3 = PCx * PAy - PCy * PAx;
  return t1 * t2 >= 0 && t1 * t3 >= 0;
}

__device__ __constant__ static const int kDir[8][2] = {{0, -1}, {0, 1}, {-1, 0}, {1, 0}, {-1, -1}, {1, 1}, {-1, 1}, {1, -1}};

}  // namespace dpe
