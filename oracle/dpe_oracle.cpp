// dpe_oracle.cpp — TEST INFRASTRUCTURE: CPU restatement of DPE-MVS's PatchMatch pass.
//
// PARITY CHECKER ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
// load this library.  The product path (dpe-mvs_amd/) never links, imports or calls it.
//
// What it restates: csrc/DPE-MVS/DPE.cu (the whole `DPE::RunPatchMatch` pass, :3126-3249, and
// every kernel / device function it reaches), line by line, in scalar C++.  Each function cites
// the reference lines it follows.
//
// PARITY UNPINNED: the reference cannot be built here (needs nvcc, CUDA textures, cuRAND, OpenCV —
// SURVEY.md §8c) and holds no tests, golden vectors or fixtures for this path, so
// no reference output pins this restatement.  What pins it: the published Philox4x32-10 KATs
// (Random123), per-function known-answer / invariant tests (tests/test_oracle_kat.py,
// tests/test_oracle_functions.py: homography vs the literal float32 sequence, NCC-New, geometric
// cost, median filter, DepthToWeak classes, GetDepthandNormal, LocalRefine) and the
// self-generated golden fixtures that freeze it (tests/golden/).  See DESIGN.md §4.
//
// Deliberate, documented restatement choices:
//  1. Arithmetic primitives are those of oracle_math.h (the reference is --use_fast_math).
//  2. RNG: Philox4x32-10 keyed (pixel, seed), one counter stream per (kernel, iteration);
//     draw ORDER within a kernel follows the reference exactly.  In
//     `(curand()%2==0 ? 1 : -1) * curand() % shift` (DPE.cu:2182) the sign draw is first.
//  3. Homography: ComputeHomography (DPE.cu:453-513) is restated as H = M_v - b_v g^T with
//     per-view M_v = Ksrc·Rrel·Kref^-1, b_v = Ksrc·trel (computed once per pass in double, rounded
//     to float) and per-plane g = Kref^-T (n / w); projection x/z is x * (1/z).
//  4. Same-colour reads of the red/black sweep (the (-1,-1) edge direction, DPE.cu:1275,1312,
//     and the row-wrap of `center+1`, :1554) see the values from before the half-sweep
//     (snapshot semantics).  Out-of-range `selected_views` reads (:1554-1558) read 0.
//  5. Out-of-array reads of the low-resolution edge map by BresenhamLine's overshoot step
//     (DPE.cu:199-200) read 0.
//  6. Dead stores with no observable effect are not restated: RANSACToGetFitPlane's copy of the
//     plane into fit_plane for non-WEAK pixels (:2904-2906, only WEAK pixels ever read it) and
//     CheckerboardPropagationWeak's radius save/restore around the Old-NCC cost (:1845-1861,
//     Old NCC never reads the radius map).  NCCs whose result is multiplied by a zero view
//     weight are not evaluated when the product is provably +0 (cost vectors feeding only
//     `view_weights[j] * c` sums).
//  7. Bilinear taps: the fixed-point coordinate of the texture unit is RN(256 (q / qz) + 256), rounded
//     once from the 256-scaled homography numerator and the tap reciprocal iz (OracleSampleQ);
//     the reference's hardware conversion is unspecified beyond "8 fractional bits".
//  8. (round 5) The tap reciprocal iz is gfx950's v_rcp_f32, not the correctly rounded 1 / qz
//     (oracle_math.h o_rcp_tap: the instruction's table for biased exponents 1..252, IEEE outside);
//     the reference's own `pt.x / pt.z` under --use_fast_math is an approximate reciprocal too.
#include "oracle_math.h"
#include "../include/dpe_mvs.h"

// ORACLE_LITERAL (build/liboracle_dpe_literal*.so, tests/test_literal_drift.py only): restatement
// choices 3, 7 and 8 switched off, i.e. ComputeHomography / ComputeCorrespondingPoint / tex2D(pt + 0.5f)
// as the reference writes them, to measure what those choices move over whole passes.  1: IEEE
// division; 2: a * (1 / b) for every division there (a model of --use_fast_math's approximate one).
#ifndef ORACLE_LITERAL
#define ORACLE_LITERAL 0
#endif

#include <algorithm>
#include <cmath>
#include <cstring>
#include <atomic>
#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <chrono>
#include <vector>

using namespace oracle;

namespace {

struct short2_ { short x, y; };
struct int2_ { int x, y; };
struct float2_ { float x, y; };
struct float3_ { float x, y, z; };
struct float4_ { float x, y, z, w; };

static inline short2_ mk_s2(short x, short y) { short2_ r; r.x = x; r.y = y; return r; }

struct ViewConst {   // per source view, restatement choice 3
  float M[9];
  float b[3];
};

struct Pass {
  int W = 0, H = 0, N = 0;     // width, height, num_images
  int LW = 0, LH = 0;          // low-res edge size
  DpePatchMatchParams P;
  uint64_t seed = 0;
  uint32_t salt = 0;
  int nthreads = 1;
  std::vector<DpeCamera> cams;
  std::vector<std::vector<float>> img;     // [N][H*W]
  std::vector<std::vector<float>> dep;     // [N][H*W] (geom)
  std::vector<uint8_t> edge, edge_low;
  std::vector<int32_t> label;
  ViewConst vc[DPE_MAX_IMAGES];
  float kinv0 = 0, kinv4 = 0, kc2 = 0, kc5 = 0;
  // GenNeighbours constants (DPE.cu:2148-2152), computed in double like the reference
  float gn_cos = 0, gn_sin = 0, gn_thr = 0; int gn_shift = 1;
  // state (DataPassHelper buffers, DPE.h:52-86)
  std::vector<float4_> planes, fit_plane, planes_snap;
  std::vector<float> costs, costs_snap, complex_;
  std::vector<uint32_t> sel, sel_snap;
  std::vector<uint8_t> weak, weak_reliable, view_weight;   // view_weight [L*32]
  std::vector<short2_> neighbours;         // [L*9] (indexed per pixel instead of via neighbours_map)
  std::vector<short2_> nearest_strong;     // [L]
  std::vector<short2_> edge_neigh;         // [L*8]
  std::vector<short2_> label_boundary;     // [L*8]
  std::vector<int> radius;                 // [L]
};

template <class F>
static void parallel_rows(int H, int nthreads, F f) {
  if (nthreads <= 1) { for (int y = 0; y < H; ++y) f(y); return; }
  std::atomic<int> next(0);
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&]() { for (int y; (y = next.fetch_add(1)) < H;) f(y); });
  for (auto& t : th) t.join();
}

// ------------------------------------------------------------------ small helpers
static inline void setBit(uint32_t* v, unsigned n) { *v |= (1u << n); }                 // DPE.cu:72-75
static inline void unSetBit(uint32_t* v, unsigned n) { *v &= (0xFFFFFFFEu << n); }      // DPE.cu:77-80 (clears 0..n)
static inline int isSet(uint32_t v, unsigned n) { return (v >> n) & 1; }                 // DPE.cu:82-85

static void sort_small(float* d, int n) {                                                // DPE.cu:5-14
  int j;
  for (int i = 1; i < n; i++) {
    float tmp = d[i];
    for (j = i; j >= 1 && tmp < d[j - 1]; j--) d[j] = d[j - 1];
    d[j] = tmp;
  }
}
static void sort_small_weighted(short2_* pts, float* w, int n) {                         // DPE.cu:16-29
  int j;
  for (int i = 1; i < n; i++) {
    short2_ tmp = pts[i]; float tw = w[i];
    for (j = i; j >= 1 && tw < w[j - 1]; j--) { pts[j] = pts[j - 1]; w[j] = w[j - 1]; }
    pts[j] = tmp; w[j] = tw;
  }
}
static int FindMinCostIndex(const float* c, int n) {                                     // DPE.cu:46-57
  float m = c[0]; int mi = 0;
  for (int i = 1; i < n; ++i) if (c[i] <= m) { m = c[i]; mi = i; }
  return mi;
}
static void NormalizeVec3(float4_* v) {                                                  // DPE.cu:268-275
  const float n2 = v->x * v->x + v->y * v->y + v->z * v->z;
  const float inv = o_rsqrtf(n2);
  v->x *= inv; v->y *= inv; v->z *= inv;
}
static void NormalizeVec2(float2_* v) {                                                  // DPE.cu:285-291
  const float n2 = v->x * v->x + v->y * v->y;
  const float inv = o_rsqrtf(n2);
  v->x *= inv; v->y *= inv;
}
static void TransformPDFToCDF(float* p, int n) {                                         // DPE.cu:293-307
  float s = 0.0f;
  for (int i = 0; i < n; ++i) s += p[i];
  const float inv = 1.0f / s;
  float cum = 0.0f;
  for (int i = 0; i < n; ++i) { const float q = p[i] * inv; cum += q; p[i] = cum; }
}
static void Get3DPoint(const DpeCamera& c, int px, int py, float depth, float* X) {     // DPE.cu:309-321
  X[0] = depth * ((float)px - c.K[2]) / c.K[0];
  X[1] = depth * ((float)py - c.K[5]) / c.K[4];
  X[2] = depth;
}
static float4_ GetViewDirection(const DpeCamera& c, int px, int py, float depth) {      // DPE.cu:323-335
  float X[3]; Get3DPoint(c, px, py, depth, X);
  float norm = sqrtf(X[0] * X[0] + X[1] * X[1] + X[2] * X[2]);
  float4_ v; v.x = X[0] / norm; v.y = X[1] / norm; v.z = X[2] / norm; v.w = 0; return v;
}
static float GetDistance2Origin(const DpeCamera& c, int px, int py, float depth, const float4_& n) {  // :337-342
  float X[3]; Get3DPoint(c, px, py, depth, X);
  return -(n.x * X[0] + n.y * X[1] + n.z * X[2]);
}
static float ComputeDepthfromPlaneHypothesis(const DpeCamera& c, const float4_& pl, int px, int py) {  // :356-359
  return -pl.w * c.K[0] / (((float)px - c.K[2]) * pl.x + (c.K[0] / c.K[4]) * ((float)py - c.K[5]) * pl.y + c.K[0] * pl.z);
}
static float4_ GenerateRandomNormal(const DpeCamera& c, int px, int py, Philox* rs, float depth) {   // :361-387
  float4_ n;
  float q1 = 1.0f, q2 = 1.0f, s = 2.0f;
  while (s >= 1.0f) {
    q1 = 2.0f * rng_uniform(rs) - 1.0f;
    q2 = 2.0f * rng_uniform(rs) - 1.0f;
    s = q1 * q1 + q2 * q2;
  }
  const float sq = sqrtf(1.0f - s);
  n.x = 2.0f * q1 * sq; n.y = 2.0f * q2 * sq; n.z = 1.0f - 2.0f * s; n.w = 0;
  float4_ vd = GetViewDirection(c, px, py, depth);
  float dot = n.x * vd.x + n.y * vd.y + n.z * vd.z;
  if (dot > 0.0f) { n.x = -n.x; n.y = -n.y; n.z = -n.z; }
  NormalizeVec3(&n);
  return n;
}
static float4_ GeneratePerturbedNormal(const DpeCamera& c, int px, int py, const float4_& normal, Philox* rs, float pert) {  // :389-424
  float4_ vd = GetViewDirection(c, px, py, 1.0f);
  const float a1 = (rng_uniform(rs) - 0.5f) * pert;
  const float a2 = (rng_uniform(rs) - 0.5f) * pert;
  const float a3 = (rng_uniform(rs) - 0.5f) * pert;
  float s1, c1, s2, c2, s3, c3;
  o_sincosf(a1, &s1, &c1); o_sincosf(a2, &s2, &c2); o_sincosf(a3, &s3, &c3);
  float R[9];
  R[0] = c2 * c3;
  R[1] = c3 * s1 * s2 - c1 * s3;
  R[2] = s1 * s3 + c1 * c3 * s2;
  R[3] = c2 * s3;
  R[4] = c1 * c3 + s1 * s2 * s3;
  R[5] = c1 * s2 * s3 - c3 * s1;
  R[6] = -s2;
  R[7] = c2 * s1;
  R[8] = c1 * c2;
  float4_ np;
  np.x = R[0] * normal.x + R[1] * normal.y + R[2] * normal.z;
  np.y = R[3] * normal.x + R[4] * normal.y + R[5] * normal.z;
  np.z = R[6] * normal.x + R[7] * normal.y + R[8] * normal.z;
  np.w = normal.w;   // Mat33DotVec3 leaves w untouched (DPE.cu:87-92); w is overwritten by callers
  if (np.x * vd.x + np.y * vd.y + np.z * vd.z >= 0.0f) np = normal;
  NormalizeVec3(&np);
  return np;
}
static float4_ TransformNormal(const DpeCamera& c, const float4_& p) {                  // :524-532 (R^T n)
  float4_ t;
  t.x = c.R[0] * p.x + c.R[3] * p.y + c.R[6] * p.z;
  t.y = c.R[1] * p.x + c.R[4] * p.y + c.R[7] * p.z;
  t.z = c.R[2] * p.x + c.R[5] * p.y + c.R[8] * p.z;
  t.w = p.w; return t;
}
static float4_ TransformNormal2RefCam(const DpeCamera& c, const float4_& p) {           // :534-542 (R n)
  float4_ t;
  t.x = c.R[0] * p.x + c.R[1] * p.y + c.R[2] * p.z;
  t.y = c.R[3] * p.x + c.R[4] * p.y + c.R[5] * p.z;
  t.z = c.R[6] * p.x + c.R[7] * p.y + c.R[8] * p.z;
  t.w = p.w; return t;
}
static float3_ Get3DPointonWorld(float x, float y, float depth, const DpeCamera& c) {   // :881-901
  float3_ X, T;
  X.x = depth * (x - c.K[2]) / c.K[0];
  X.y = depth * (y - c.K[5]) / c.K[4];
  X.z = depth;
  T.x = c.R[0] * X.x + c.R[3] * X.y + c.R[6] * X.z;
  T.y = c.R[1] * X.x + c.R[4] * X.y + c.R[7] * X.z;
  T.z = c.R[2] * X.x + c.R[5] * X.y + c.R[8] * X.z;
  X.x = T.x + c.c[0]; X.y = T.y + c.c[1]; X.z = T.z + c.c[2];
  return X;
}
static void ProjectonCamera(const float3_& X, const DpeCamera& c, float2_* pt, float* d) {  // :903-913
  float3_ t;
  t.x = c.R[0] * X.x + c.R[1] * X.y + c.R[2] * X.z + c.t[0];
  t.y = c.R[3] * X.x + c.R[4] * X.y + c.R[5] * X.z + c.t[1];
  t.z = c.R[6] * X.x + c.R[7] * X.y + c.R[8] * X.z + c.t[2];
  *d = c.K[6] * t.x + c.K[7] * t.y + c.K[8] * t.z;
  pt->x = (c.K[0] * t.x + c.K[1] * t.y + c.K[2] * t.z) / *d;
  pt->y = (c.K[3] * t.x + c.K[4] * t.y + c.K[5] * t.z) / *d;
}

// ------------------------------------------------------------------ image sampling
// tex2D<float>(img, x + 0.5f, y + 0.5f) at integer (x, y): the texel, clamp addressing.
static inline float RefTexel(const Pass& S, const std::vector<float>& im, int x, int y) {
  x = x < 0 ? 0 : (x > S.W - 1 ? S.W - 1 : x);
  y = y < 0 ? 0 : (y > S.H - 1 ? S.H - 1 : y);
  return im[(size_t)y * S.W + x];
}
// tex2D<float>(img, sx + 0.5f, sy + 0.5f), linear filter, clamp addressing (DPE.cpp:927-933).
// Texture model (restatement choice 7): the tap's homography numerators are scaled by 256
// (Q = fma(256 h1, y, 256 fma(h0, x, h2)) = 256 q, exact) and the coordinate s + 1 = q / qz + 1 is converted to fixed point with 8
// fractional bits by ONE round-to-nearest-even, U = RN(Q * iz + 256) with iz = 1 / qz, evaluated
// as t = fma(Q, iz, 1.5*2^23 + 256) on the unit grid of [2^23, 2^24) so that U = t - 1.5*2^23;
// U is clamped to [0, 256 lim + 256] (clamp addressing: beyond that the filtered value is the
// border texel's), NaN -> 0.  Texel index i = (U >> 8) - 1, weight a = (U & 255) / 256.
static const float kTexMagic = 12582912.0f;   // 1.5 * 2^23
static inline uint32_t TexU(float Q, float iz, int lim) {
  const float t = fmaf(Q, iz, kTexMagic + 256.0f);
  const float tc = fminf(fmaxf(t, kTexMagic), kTexMagic + 256.0f * (float)(lim + 1));
  uint32_t u; std::memcpy(&u, &tc, 4);
  return u - 0x4B400000u;
}
static inline float OracleSampleU(const Pass& S, const std::vector<float>& im, uint32_t ux, uint32_t uy) {
  const float ax = (float)(ux & 255u) * 0.00390625f;
  const float ay = (float)(uy & 255u) * 0.00390625f;
  const int ix = (int)(ux >> 8) - 1, iy = (int)(uy >> 8) - 1;
  int x0 = ix < 0 ? 0 : (ix > S.W - 1 ? S.W - 1 : ix);
  int x1 = ix + 1 < 0 ? 0 : (ix + 1 > S.W - 1 ? S.W - 1 : ix + 1);
  int y0 = iy < 0 ? 0 : (iy > S.H - 1 ? S.H - 1 : iy);
  int y1 = iy + 1 < 0 ? 0 : (iy + 1 > S.H - 1 ? S.H - 1 : iy + 1);
  float t00 = im[(size_t)y0 * S.W + x0], t10 = im[(size_t)y0 * S.W + x1];
  float t01 = im[(size_t)y1 * S.W + x0], t11 = im[(size_t)y1 * S.W + x1];
  float r0 = fmaf(ax, t10 - t00, t00);
  float r1 = fmaf(ax, t11 - t01, t01);
  return fmaf(ay, r1 - r0, r0);
}
static inline float OracleSampleQ(const Pass& S, const std::vector<float>& im, float Qx, float Qy, float iz) {
  return OracleSampleU(S, im, TexU(Qx, iz, S.W), TexU(Qy, iz, S.H));
}
#if ORACLE_LITERAL
// Literal texture coordinate (ORACLE_LITERAL builds): tex2D(img, s + 0.5f) as DPE.cu:734-736 writes it
// (the float add rounded), then the CUDA guide's linear filter: x_B = x - 0.5 (rounded in float),
// 8 fractional bits taken as round-to-nearest of 256 x_B, clamp addressing; same U convention as
// TexU (texel (U >> 8) - 1, weight (U & 255) / 256, U clamped to [0, 256 lim + 256], NaN -> 0).
static inline uint32_t TexULiteral(float s, int lim) {
  const float xb = (s + 0.5f) - 0.5f;
  if (std::isnan(xb)) return 0;
  double u = std::floor((double)xb * 256.0 + 0.5) + 256.0;
  u = u < 0.0 ? 0.0 : (u > 256.0 * (lim + 1) ? 256.0 * (lim + 1) : u);
  return (uint32_t)u;
}
#endif
// tex2D<float>(depth, (int)x + 0.5f, (int)y + 0.5f) (DPE.cu:936): texel at the truncated coordinate.
static inline float DepthTexel(const Pass& S, const std::vector<float>& im, float x, float y) {
  int ix = o_f2i(x), iy = o_f2i(y);
  return RefTexel(S, im, ix, iy);
}

// ------------------------------------------------------------------ homography (choice 3)
static void ComputeViewConstants(Pass& S) {
  // DPE.cu:455-512 evaluated in double for the plane-independent part.
  const DpeCamera& rc = S.cams[0];
  double rK0 = rc.K[0], rK2 = rc.K[2], rK4 = rc.K[4], rK5 = rc.K[5];
  double refC[3];
  for (int j = 0; j < 3; ++j)
    refC[j] = -((double)rc.R[0 + j] * rc.t[0] + (double)rc.R[3 + j] * rc.t[1] + (double)rc.R[6 + j] * rc.t[2]);
  for (int v = 1; v < S.N; ++v) {
    const DpeCamera& sc = S.cams[v];
    double srcC[3], Rrel[9], Crel[3], trel[3];
    for (int j = 0; j < 3; ++j)
      srcC[j] = -((double)sc.R[0 + j] * sc.t[0] + (double)sc.R[3 + j] * sc.t[1] + (double)sc.R[6 + j] * sc.t[2]);
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c)
        Rrel[r * 3 + c] = (double)sc.R[r * 3 + 0] * rc.R[c * 3 + 0] + (double)sc.R[r * 3 + 1] * rc.R[c * 3 + 1] +
                          (double)sc.R[r * 3 + 2] * rc.R[c * 3 + 2];
    for (int j = 0; j < 3; ++j) Crel[j] = refC[j] - srcC[j];
    for (int r = 0; r < 3; ++r)
      trel[r] = (double)sc.R[r * 3 + 0] * Crel[0] + (double)sc.R[r * 3 + 1] * Crel[1] + (double)sc.R[r * 3 + 2] * Crel[2];
    double T[9];
    for (int r = 0; r < 3; ++r) {
      T[r * 3 + 0] = Rrel[r * 3 + 0] / rK0;
      T[r * 3 + 1] = Rrel[r * 3 + 1] / rK4;
      T[r * 3 + 2] = -Rrel[r * 3 + 0] * rK2 / rK0 - Rrel[r * 3 + 1] * rK5 / rK4 + Rrel[r * 3 + 2];
    }
    double sK0 = sc.K[0], sK2 = sc.K[2], sK4 = sc.K[4], sK5 = sc.K[5], sK8 = sc.K[8];
    for (int c = 0; c < 3; ++c) {
      S.vc[v].M[0 + c] = (float)(sK0 * T[0 + c] + sK2 * T[6 + c]);
      S.vc[v].M[3 + c] = (float)(sK4 * T[3 + c] + sK5 * T[6 + c]);
      S.vc[v].M[6 + c] = (float)(sK8 * T[6 + c]);
    }
    S.vc[v].b[0] = (float)(sK0 * trel[0] + sK2 * trel[2]);
    S.vc[v].b[1] = (float)(sK4 * trel[1] + sK5 * trel[2]);
    S.vc[v].b[2] = (float)(sK8 * trel[2]);
  }
  S.kinv0 = (float)(1.0 / rK0);
  S.kinv4 = (float)(1.0 / rK4);
  S.kc2 = (float)(rK2 / rK0);
  S.kc5 = (float)(rK5 / rK4);
}

struct Homog { float h[9]; };

#if ORACLE_LITERAL
// float division of the literal builds: IEEE (ORACLE_LITERAL 1) or a * (1 / b), a model of the
// approximate division --use_fast_math selects (ORACLE_LITERAL 2)
static inline float LDiv(float a, float b) { return ORACLE_LITERAL == 2 ? a * (1.0f / b) : a / b; }
// ComputeHomography (DPE.cu:453-513) statement by statement in float32, per call
static inline Homog MakeHomography(const Pass& S, int v, const float4_& pl) {
  const DpeCamera& rc = S.cams[0];
  const DpeCamera& sc = S.cams[v];
  float refC[3], srcC[3], Rr[9], Cr[3], tr[3], H[9], tmp[9];
  refC[0] = -(rc.R[0] * rc.t[0] + rc.R[3] * rc.t[1] + rc.R[6] * rc.t[2]);
  refC[1] = -(rc.R[1] * rc.t[0] + rc.R[4] * rc.t[1] + rc.R[7] * rc.t[2]);
  refC[2] = -(rc.R[2] * rc.t[0] + rc.R[5] * rc.t[1] + rc.R[8] * rc.t[2]);
  srcC[0] = -(sc.R[0] * sc.t[0] + sc.R[3] * sc.t[1] + sc.R[6] * sc.t[2]);
  srcC[1] = -(sc.R[1] * sc.t[0] + sc.R[4] * sc.t[1] + sc.R[7] * sc.t[2]);
  srcC[2] = -(sc.R[2] * sc.t[0] + sc.R[5] * sc.t[1] + sc.R[8] * sc.t[2]);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      Rr[r * 3 + c] = sc.R[r * 3 + 0] * rc.R[c * 3 + 0] + sc.R[r * 3 + 1] * rc.R[c * 3 + 1] + sc.R[r * 3 + 2] * rc.R[c * 3 + 2];
  for (int j = 0; j < 3; ++j) Cr[j] = refC[j] - srcC[j];
  for (int r = 0; r < 3; ++r) tr[r] = sc.R[r * 3 + 0] * Cr[0] + sc.R[r * 3 + 1] * Cr[1] + sc.R[r * 3 + 2] * Cr[2];
  const float pv[3] = {pl.x, pl.y, pl.z};
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) H[r * 3 + c] = Rr[r * 3 + c] - LDiv(tr[r] * pv[c], pl.w);
  for (int r = 0; r < 3; ++r) {
    tmp[r * 3 + 0] = LDiv(H[r * 3 + 0], rc.K[0]);
    tmp[r * 3 + 1] = LDiv(H[r * 3 + 1], rc.K[4]);
    tmp[r * 3 + 2] = LDiv(-H[r * 3 + 0] * rc.K[2], rc.K[0]) - LDiv(H[r * 3 + 1] * rc.K[5], rc.K[4]) + H[r * 3 + 2];
  }
  Homog o;
  for (int c = 0; c < 3; ++c) {
    o.h[0 + c] = sc.K[0] * tmp[0 + c] + sc.K[2] * tmp[6 + c];
    o.h[3 + c] = sc.K[4] * tmp[3 + c] + sc.K[5] * tmp[6 + c];
    o.h[6 + c] = sc.K[8] * tmp[6 + c];
  }
  return o;
}
// ComputeCorrespondingPoint (DPE.cu:515-522) as written: h0*x + h1*y + h2, then X / Z
static inline float2_ Project(const Homog& H, float x, float y) {
  const float X = H.h[0] * x + H.h[1] * y + H.h[2];
  const float Y = H.h[3] * x + H.h[4] * y + H.h[5];
  const float Z = H.h[6] * x + H.h[7] * y + H.h[8];
  float2_ r; r.x = LDiv(X, Z); r.y = LDiv(Y, Z); return r;
}
#else
static inline Homog MakeHomography(const Pass& S, int v, const float4_& pl) {
  const float iw = 1.0f / pl.w;
  const float qx = pl.x * iw, qy = pl.y * iw, qz = pl.z * iw;
  float g[3];
  g[0] = qx * S.kinv0;
  g[1] = qy * S.kinv4;
  g[2] = fmaf(-qx, S.kc2, fmaf(-qy, S.kc5, qz));
  Homog H;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) H.h[r * 3 + c] = fmaf(-S.vc[v].b[r], g[c], S.vc[v].M[r * 3 + c]);
  return H;
}
// ComputeCorrespondingPoint (DPE.cu:515-522): h0*x + h1*y + h2 evaluated as fma(h1, y, fma(h0, x, h2))
static inline float2_ Project(const Homog& H, float x, float y) {
  float px = fmaf(H.h[1], y, fmaf(H.h[0], x, H.h[2]));
  float py = fmaf(H.h[4], y, fmaf(H.h[3], x, H.h[5]));
  float pz = fmaf(H.h[7], y, fmaf(H.h[6], x, H.h[8]));
  float iz = 1.0f / pz;
  float2_ r; r.x = px * iz; r.y = py * iz; return r;
}
#endif

// ComputeBilateralWeight (DPE.cu:550-555)
static inline float BilateralWeight(const Pass& S, int i, int j, float pix, float cpix) {
  const float xd = (float)i, yd = (float)j;
  const float sd = sqrtf(xd * xd + yd * yd);
  const float cd = fabsf(pix - cpix);
  const float ss = S.P.sigma_spatial, sc = S.P.sigma_color;
  return o_expf(-sd / (2.0f * ss * ss) - cd / (2.0f * sc * sc));
}

// Bilateral-weighted NCC of one patch (body shared by ComputeBilateralNCCOld :715-775 and the
// per-point body of ComputeBilateralNCCNew :609-668).
static inline float PatchNCC(const Pass& S, const std::vector<float>& src, const Homog& H, int cx, int cy,
                             float ref_center_pix, int radius, int increment) {
  const std::vector<float>& ref = S.img[0];
  const float h1s = H.h[1] * 256.0f, h4s = H.h[4] * 256.0f;   // tap numerators Q = 256 q (choice 7)
  float s_ref = 0, s_rr = 0, s_src = 0, s_ss = 0, s_rs = 0, s_w = 0;
  for (int i = -radius; i <= radius; i += increment) {
    float r_ref = 0, r_src = 0, r_rr = 0, r_ss = 0, r_rs = 0, r_w = 0;
    for (int j = -radius; j <= radius; j += increment) {
      const int x = cx + i, y = cy + j;
      const float rp = RefTexel(S, ref, x, y);
      const float xf = (float)x, yf = (float)y;
#if ORACLE_LITERAL
      (void)h1s; (void)h4s;
      const float2_ st = Project(H, xf, yf);
      const float sp = OracleSampleU(S, src, TexULiteral(st.x, S.W), TexULiteral(st.y, S.H));
#else
      const float Qx = fmaf(h1s, yf, fmaf(H.h[0], xf, H.h[2]) * 256.0f);
      const float Qy = fmaf(h4s, yf, fmaf(H.h[3], xf, H.h[5]) * 256.0f);
      const float iz = o_rcp_tap(fmaf(H.h[7], yf, fmaf(H.h[6], xf, H.h[8])));   // choice 8
      const float sp = OracleSampleQ(S, src, Qx, Qy, iz);
#endif
      const float w = BilateralWeight(S, i, j, rp, ref_center_pix);
      const float wr = w * rp;
      r_ref = r_ref + wr;
      r_rr = fmaf(wr, rp, r_rr);
      r_src = fmaf(w, sp, r_src);
      const float ws = w * sp;
      r_ss = fmaf(ws, sp, r_ss);
      r_rs = fmaf(wr, sp, r_rs);
      r_w = r_w + w;
    }
    s_ref += r_ref; s_rr += r_rr; s_src += r_src; s_ss += r_ss; s_rs += r_rs; s_w += r_w;
  }
  const float inv = 1.0f / s_w;
  s_ref *= inv; s_rr *= inv; s_src *= inv; s_ss *= inv; s_rs *= inv;
  const float var_ref = s_rr - s_ref * s_ref;
  const float var_src = s_ss - s_src * s_src;
  const float kMinVar = 1e-5f;
  if (var_ref < kMinVar || var_src < kMinVar) return 2.0f;
  const float cov = s_rs - s_ref * s_src;
  const float vrs = sqrtf(var_ref * var_src);
  return fmaxf(0.0f, fminf(2.0f, 1.0f - cov / vrs));
}

// ComputeBilateralNCCOld (DPE.cu:692-778)
static float NCCOld(const Pass& S, int px, int py, int v, const float4_& pl) {
  Homog H = MakeHomography(S, v, pl);
  float2_ pt = Project(H, (float)px, (float)py);
  const DpeCamera& sc = S.cams[v];
  if (pt.x >= (float)sc.width || pt.x < 0.0f || pt.y >= (float)sc.height || pt.y < 0.0f) return 2.0f;
  const float rc = RefTexel(S, S.img[0], px, py);
  return PatchNCC(S, S.img[v], H, px, py, rc, S.P.strong_radius, S.P.strong_increment);
}

// GetNeighbourPoint (DPE.cu:544-548), stored per pixel
static inline short2_ Neighbour(const Pass& S, int center, int k) { return S.neighbours[(size_t)center * 9 + k]; }

// ComputeBilateralNCCNew (DPE.cu:557-690)
static float NCCNew(const Pass& S, int px, int py, int v, const float4_& pl) {
  const int W = S.W, Hh = S.H;
  const int center = px + py * W;
  Homog H = MakeHomography(S, v, pl);
  float2_ pt = Project(H, (float)px, (float)py);
  const DpeCamera& sc = S.cams[v];
  if (pt.x >= (float)sc.width || pt.x < 0.0f || pt.y >= (float)sc.height || pt.y < 0.0f) return 2.0f;
  float cost = 0.0f;
  if (S.weak[center] != DPE_WEAK) return cost;   // reference prints "error" and returns 0 (:685-687)
  const float rc = RefTexel(S, S.img[0], px, py);
  float center_cost = 0.0f, strong_cost = 0.0f;
  int strong_count = 0;
  for (int k = 0; k < DPE_NEIGHBOUR_NUM; ++k) {
    const short2_ np = Neighbour(S, center, k);
    if (np.x == -1 || np.y == -1) continue;
    float2_ nsp = Project(H, (float)np.x, (float)np.y);
    if (nsp.x < 0 || nsp.y < 0 || nsp.x >= (float)W || nsp.y >= (float)Hh) {
      if (k != 0) {
        uint32_t vi = S.sel[np.x + np.y * W];
        if (isSet(vi, v - 1)) { strong_cost += 2.0f; strong_count++; }
        continue;
      } else {
        return 2.0f;
      }
    }
    int radius = (k == 0 ? S.P.strong_radius : S.P.weak_radius);
    int increment = (k == 0 ? S.P.strong_increment : S.P.weak_increment);
    if (S.P.use_radius && k == 0) {
      radius = S.radius[center];
      increment = MAXo(2, o_d2i(2.0 * radius / 5.0));
    }
    const float tc = PatchNCC(S, S.img[v], H, np.x, np.y, rc, radius, increment);
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

// ComputeGeomConsistencyCost (DPE.cu:915-953)
static float GeomCost(const Pass& S, int px, int py, int v, const float4_& pl) {
  const DpeCamera& rc = S.cams[0];
  const DpeCamera& sc = S.cams[v];
  const float max_cost = 3.0f;
  float depth = ComputeDepthfromPlaneHypothesis(rc, pl, px, py);
  float3_ fw = Get3DPointonWorld((float)px, (float)py, depth, rc);
  float2_ sp; float sd;
  ProjectonCamera(fw, sc, &sp, &sd);
  const float src_depth = DepthTexel(S, S.dep[v], sp.x, sp.y);
  if (src_depth == 0.0f) return max_cost;
  float3_ s3 = Get3DPointonWorld(sp.x, sp.y, src_depth, sc);
  float2_ bp; float rd;
  ProjectonCamera(s3, rc, &bp, &rd);
  const float dc = (float)px - bp.x, dr = (float)py - bp.y;
  const float cc = sqrtf(dc * dc + dr * dr);
  return fminf(max_cost, cc);
}

// ------------------------------------------------------------------ BresenhamLine (DPE.cu:158-244)
static inline uint8_t LowEdgeAt(const Pass& S, int idx) {
  if (idx < 0 || idx >= S.LW * S.LH) return 0;   // restatement choice 5
  return S.edge_low[idx];
}
static bool BresenhamLine(const Pass& S, int Ax, int Ay, int Bx, int By) {
  const int W = S.W;
  if (S.edge[Ax + Ay * W] || S.edge[Bx + By * W]) return false;
  const float scale_x = 1.0f * S.LW / (float)S.W;
  const float scale_y = 1.0f * S.LH / (float)S.H;
  const int height = S.LH, width = S.LW;
  int max_step = S.P.high_res_img ? (int)std::round(MAXo(height, width) / 60.0) : MAXo(height, width);
  for (int pass = 0; pass < 2; ++pass) {
    int fx = pass == 0 ? Bx : Ax, fy = pass == 0 ? By : Ay;
    int tx = pass == 0 ? Ax : Bx, ty = pass == 0 ? Ay : By;
    int x0 = (int)MINo(roundf(fx * scale_x), (float)(width - 1));
    int y0 = (int)MINo(roundf(fy * scale_y), (float)(height - 1));
    int x1 = (int)MINo(roundf(tx * scale_x), (float)(width - 1));
    int y1 = (int)MINo(roundf(ty * scale_y), (float)(height - 1));
    int dx = abs(x1 - x0), sx = x0 < x1 ? 1 : -1;
    int dy = abs(y1 - y0), sy = y0 < y1 ? 1 : -1;
    int erro = (dx > dy ? dx : dy) / 2;
    int step = 0;
    bool tagx = true, tagy = true;
    while (tagx || tagy) {
      if (x0 == x1) tagx = false;
      if (y0 == y1) tagy = false;
      int e2 = erro;
      if (e2 > -dx) { erro -= dy; x0 += sx; }
      if (e2 < dy) { erro += dx; y0 += sy; }
      if (LowEdgeAt(S, x0 + y0 * width)) return true;
      step += 1;
      if (step >= max_step) break;
    }
  }
  return false;
}

// PointinTriangle (DPE.cu:135-156)
static bool PointinTriangle(short2_ A, short2_ B, short2_ C, int Px, int Py) {
  float2_ AB = {(float)(B.x - A.x), (float)(B.y - A.y)};
  float2_ BC = {(float)(C.x - B.x), (float)(C.y - B.y)};
  float2_ CA = {(float)(A.x - C.x), (float)(A.y - C.y)};
  float AB_ = sqrtf(AB.x * AB.x + AB.y * AB.y);
  float BC_ = sqrtf(BC.x * BC.x + BC.y * BC.y);
  float CA_ = sqrtf(CA.x * CA.x + CA.y * CA.y);
  if (AB_ <= 2 || BC_ <= 2 || CA_ <= 2) return false;
  if (!(AB_ + BC_ > CA_ && BC_ + CA_ > AB_ && AB_ + CA_ > BC_)) return false;
  float2_ PA = {(float)(A.x - Px), (float)(A.y - Py)};
  float2_ PB = {(float)(B.x - Px), (float)(B.y - Py)};
  float2_ PC = {(float)(C.x - Px), (float)(C.y - Py)};
  float t1 = PA.x * PB.y - PA.y * PB.x;
  float t2 = PB.x * PC.y - PB.y * PC.x;
  float t3 = PC.x * PA.y - PC.y * PA.x;
  return t1 * t2 >= 0 && t1 * t3 >= 0;
}

// ------------------------------------------------------------------ kernels
static const int kDir[8][2] = {{0, -1}, {0, 1}, {-1, 0}, {1, 0}, {-1, -1}, {1, 1}, {-1, 1}, {1, -1}};

// GenEdgeInform (DPE.cu:2483-2591)
static void GenEdgeInform(Pass& S, int x, int y) {
  const int W = S.W, H = S.H;
  const int center = x + y * W;
  if (S.P.use_edge) {
    short2_* en = &S.edge_neigh[(size_t)center * 8];
    for (int i = 0; i < 8; i++) {
      en[i] = mk_s2(-1, -1);
      int dx = kDir[i][0], dy = kDir[i][1];
      int nx = x + dx, ny = y + dy;
      while (true) {
        if (nx < 0 || nx >= W || ny < 0 || ny >= H) break;
        if (S.edge[nx + ny * W]) { en[i] = mk_s2((short)nx, (short)ny); break; }
        nx += dx; ny += dy;
      }
    }
    int radius = S.P.strong_radius;
    int edge_pix = 0, tot_pix = 0;
    for (int i = -radius; i <= radius; i++)
      for (int j = -radius; j <= radius; j++) {
        int nx = x + i, ny = y + j;
        if (nx < 0 || nx >= W || ny < 0 || ny >= H) continue;
        if (S.edge[ny * W + nx]) edge_pix++;
        tot_pix++;
      }
    float density = 1.0f * edge_pix / tot_pix;
    if (S.P.use_label) {
      int bound_pix = 0;
      for (int i = -radius; i <= radius; i++)
        for (int j = -radius; j <= radius; j++) {
          int nx = x + i, ny = y + j;
          if (nx < 0 || nx >= W || ny < 0 || ny >= H) continue;
          if (S.label[ny * W + nx] == 0) bound_pix++;
        }
      density = MAXo(density, (float)(bound_pix / tot_pix));   // integer division (:2551)
    }
    S.complex_[center] = (float)(1.0f / (1.0f + o_exp_d(-25.0 * ((double)density - 0.35))));
  }
  if (S.P.use_label && S.weak[center] == DPE_WEAK) {
    short2_* lb = &S.label_boundary[(size_t)center * 8];
    int cl = S.label[center];
    if (cl > 0) {
      for (int i = 0; i < 8; i++) {
        int dx = kDir[i][0], dy = kDir[i][1];
        int nx = x + dx, ny = y + dy;
        int lx = -1, ly = -1;
        while (true) {
          if (nx < 0 || nx >= W || ny < 0 || ny >= H) break;
          int nl = S.label[nx + ny * W];
          if (nl == cl) { lx = nx; ly = ny; }
          else if (nl == -1) break;
          nx += dx; ny += dy;
        }
        lb[i] = mk_s2((short)lx, (short)ly);
      }
    }
  }
}

// FindNearestStrongPoint (DPE.cu:2855-2889)
static void FindNearestStrongPoint(Pass& S, int x, int y) {
  const int W = S.W, H = S.H;
  const int center = x + y * W;
  S.nearest_strong[center] = mk_s2(-1, -1);
  if (S.weak[center] != DPE_WEAK) return;
  for (int r = 0; r <= 100; ++r)
    for (int dx = -r; dx <= r; ++dx)
      for (int dy = -r; dy <= r; ++dy) {
        if (abs(dx) != r && abs(dy) != r) continue;
        int nx = x + dx, ny = y + dy;
        if (nx < 0 || ny < 0 || nx >= W || ny >= H) continue;
        if (S.weak[nx + ny * W] == DPE_STRONG) { S.nearest_strong[center] = mk_s2((short)nx, (short)ny); return; }
      }
}

// GenNeighbours (DPE.cu:2103-2463)
static void GenNeighbours(Pass& S, int x, int y) {
  const int W = S.W, H = S.H;
  const int center = x + y * W;
  if (S.weak[center] != DPE_WEAK) return;
  const int max_pt_num = 64;
  const int min_margin = 6;
  const float depth_diff = S.P.depth_max - S.P.depth_min;
  const DpeCamera& camera = S.cams[0];
  Philox rs; rng_init(&rs, (uint32_t)center, S.seed, STREAM_GEN_NEIGHBOURS, S.salt);
  short2_* nb = &S.neighbours[(size_t)center * 9];
  for (int i = 0; i < 9; ++i) nb[i] = mk_s2(-1, -1);
  nb[0] = mk_s2((short)x, (short)y);
  short2_ strong_points[64];
  bool dir_valid[64];
  for (int i = 0; i < max_pt_num; ++i) { strong_points[i] = mk_s2(-1, -1); dir_valid[i] = false; }
  int origin_direction_index = -1;
  int strong_point_size = 0;
  const int rotate_time = S.P.rotate_time;
  const float cos_angle = S.gn_cos, sin_angle = S.gn_sin, threshhold = S.gn_thr;
  const int shift_range = S.gn_shift;
  const float ransac_threshold = S.P.ransac_threshold * depth_diff;

  bool edge_limit = false;
  if (S.P.use_limit) {
    edge_limit = true;
    if (S.P.use_edge) {
      float cv = S.complex_[center];
      const float rp = rng_uniform(&rs) - FLT_EPSILON;
      if (rp < cv) edge_limit = false;
      else S.complex_[center] = MAXo(0.99f, cv);
    }
  }

  for (int odx = -1; odx <= 1; ++odx) {
    for (int ody = -1; ody <= 1; ++ody) {
      if (odx == 0 && ody == 0) continue;
      float2_ od = {(float)odx, (float)ody};
      NormalizeVec2(&od);
      origin_direction_index++;
      for (int rotate_iter = 0; rotate_iter < rotate_time; ++rotate_iter) {
        int dir_index = origin_direction_index * 4 + rotate_iter;
        for (int radius = 2; radius <= 4096; radius = MINo(radius * 2, radius + 25)) {
          float2_ tp = {(float)x + od.x * radius, (float)y + od.y * radius};
          if (tp.x < 0 || tp.y < 0 || tp.x >= W || tp.y >= H) break;
          for (int radius_iter = 0; radius_iter < 4; ++radius_iter) {
            uint32_t r1 = rng_u32(&rs), r2 = rng_u32(&rs);
            int rxs = (int)(((r1 % 2 == 0) ? 1u : 0xFFFFFFFFu) * r2 % (uint32_t)shift_range);
            uint32_t r3 = rng_u32(&rs), r4 = rng_u32(&rs);
            int rys = (int)(((r3 % 2 == 0) ? 1u : 0xFFFFFFFFu) * r4 % (uint32_t)shift_range);
            float2_ dir = {od.x * 20 + (float)rxs, od.y * 20 + (float)rys};
            NormalizeVec2(&dir);
            short2_ np = mk_s2((short)o_f2i((float)x + dir.x * radius), (short)o_f2i((float)y + dir.y * radius));
            if (np.x < min_margin || np.y < min_margin || np.x >= W - min_margin || np.y >= H - min_margin) continue;
            int npc = np.x + np.y * W;
            if (S.weak[npc] != DPE_STRONG) {
              np = S.nearest_strong[npc];
              if (np.x == -1 || np.y == -1) continue;
              npc = np.x + np.y * W;
            }
            float2_ td = {(float)(np.x - x), (float)(np.y - y)};
            NormalizeVec2(&td);
            float ca = td.x * od.x + td.y * od.y;
            if (ca > threshhold && (!edge_limit || !BresenhamLine(S, x, y, np.x, np.y))) {
              strong_points[dir_index] = np;
              dir_valid[dir_index] = true;
              strong_point_size++;
              break;
            }
          }
          if (dir_valid[dir_index]) break;
        }
        {
          float2_ rd;
          rd.x = od.x * cos_angle - od.y * sin_angle;
          rd.y = od.x * sin_angle + od.y * cos_angle;
          NormalizeVec2(&rd);
          od = rd;
        }
      }
    }
  }

  int extend_index = 31;
  if (S.P.use_label && S.label[center] > 0) {
    const short2_* lb = &S.label_boundary[(size_t)center * 8];
    float bound_dist[8] = {0};
    int dir_step[8] = {0};
    for (int i = 0; i < 8; ++i) {
      short2_ bp = lb[i];
      float dist = 0.0f;
      if (bp.x != -1 && bp.y != -1) {
        double dxx = (double)(x - bp.x), dyy = (double)(y - bp.y);
        dist = (float)std::sqrt(dxx * dxx + dyy * dyy);
        if (i >= 4) dist = (float)((double)dist / std::sqrt(2.0));
      }
      bound_dist[i] = dist;
      if (i % 2 == 1) {
        // step = MIN(1, MAX(2*rotate_time-1, ...)) == 1 for rotate_time >= 1 (:2241)
        int step = 1;
        int opposite_step = 2 * rotate_time - step;
        dir_step[i - 1] = opposite_step;
        dir_step[i] = step;
      }
    }
    for (int i = 0; i < 8; ++i) {
      float dist = bound_dist[i];
      int gap_num = dir_step[i] + 1;
      int step_len = MAXo(1, o_d2i(floor(1.0 * dist / gap_num)));
      for (int step = 1; step <= dir_step[i]; ++step) {
        short2_ np = mk_s2((short)(x + step * step_len * kDir[i][0]), (short)(y + step * step_len * kDir[i][1]));
        if (np.x < min_margin || np.y < min_margin || np.x >= W - min_margin || np.y >= H - min_margin) continue;
        int npc = np.x + np.y * W;
        if (S.weak[npc] != DPE_STRONG) {
          np = S.nearest_strong[npc];
          if (np.x == -1 || np.y == -1) continue;
          npc = np.x + np.y * W;
        }
        if (S.label[npc] != 0 && S.label[npc] != S.label[center]) continue;
        extend_index++;
        strong_points[extend_index] = np;
        dir_valid[extend_index] = true;
        strong_point_size++;
      }
    }
  }

  if (strong_point_size <= 3) { S.weak_reliable[center] = 0; return; }

  float4_ best_plane = {0, 0, 0, 0};
  bool has_valid_plane = false;
  short2_ spv[64];
  float3_ spv3[64];
  float3_ spvn[64];
  int valid_count = 0;
  float X[3];
  Get3DPoint(camera, x, y, S.planes[center].w, X);
  float3_ cpw = {X[0], X[1], X[2]};
  for (int i = 0; i < max_pt_num; ++i) {
    spv[i] = mk_s2(-1, -1);
    if (dir_valid[i]) {
      const short2_ sp = strong_points[i];
      int spc = sp.x + sp.y * W;
      spv[valid_count] = sp;
      Get3DPoint(camera, sp.x, sp.y, S.planes[spc].w, X);
      spv3[valid_count] = {X[0], X[1], X[2]};
      float4_ n4 = TransformNormal2RefCam(camera, S.planes[spc]);
      spvn[valid_count] = {n4.x, n4.y, n4.z};
      valid_count++;
    }
  }
  {
    int iteration = 50, max_iter = S.P.high_res_img ? 200 : 125, max_count = 3;
    float min_cost = FLT_MAX, residuals[64];
    for (int i = 0; i < 64; ++i) residuals[i] = 0.0f;
    float temp_thr = ransac_threshold;
    static thread_local uint8_t edge_test[64][64];
    std::memset(edge_test, 0, sizeof(edge_test));
    bool has_consist_normal_plane = false;
    bool must_in_triangle = (S.P.use_label && S.label[center] > 0 && edge_limit) ? false : true;
    while (iteration > 0 && max_iter > 0) {
      max_iter--;
      int a = (int)(rng_u32(&rs) % (uint32_t)valid_count);
      int b = (int)(rng_u32(&rs) % (uint32_t)valid_count);
      int c = (int)(rng_u32(&rs) % (uint32_t)valid_count);
      if (a == b || b == c || a == c) continue;
      if (must_in_triangle && !PointinTriangle(spv[a], spv[b], spv[c], x, y)) continue;
      if (edge_limit) {
        if (edge_test[a][b] == 0) edge_test[a][b] = edge_test[b][a] = (BresenhamLine(S, spv[a].x, spv[a].y, spv[b].x, spv[b].y) ? 1 : 2);
        if (edge_test[b][c] == 0) edge_test[b][c] = edge_test[c][b] = (BresenhamLine(S, spv[b].x, spv[b].y, spv[c].x, spv[c].y) ? 1 : 2);
        if (edge_test[c][a] == 0) edge_test[c][a] = edge_test[a][c] = (BresenhamLine(S, spv[c].x, spv[c].y, spv[a].x, spv[a].y) ? 1 : 2);
        if (edge_test[a][b] == 1 || edge_test[b][c] == 1 || edge_test[c][a] == 1) continue;
      }
      bool normal_consistency = false;
      if (S.P.geom_consistency && edge_limit) {
        const float3_ &AN = spvn[a], &BN = spvn[b], &CN = spvn[c];
        normal_consistency = true;
        if ((double)(AN.x * BN.x + AN.y * BN.y + AN.z * BN.z) < 0.8660254 ||
            (double)(AN.x * CN.x + AN.y * CN.y + AN.z * CN.z) < 0.8660254 ||
            (double)(BN.x * CN.x + BN.y * CN.y + BN.z * CN.z) < 0.8660254)
          normal_consistency = false;
        if (has_consist_normal_plane && !normal_consistency) continue;
      }
      iteration--;
      const float3_ &A = spv3[a], &B = spv3[b], &C = spv3[c];
      float3_ A_C = {A.x - C.x, A.y - C.y, A.z - C.z};
      float3_ B_C = {B.x - C.x, B.y - C.y, B.z - C.z};
      float4_ cv;
      cv.x = A_C.y * B_C.z - B_C.y * A_C.z;
      cv.y = -(A_C.x * B_C.z - B_C.x * A_C.z);
      cv.z = A_C.x * B_C.y - B_C.x * A_C.y;
      if ((cv.x == 0 && cv.y == 0 && cv.z == 0) || std::isnan(cv.x) || std::isnan(cv.y) || std::isnan(cv.z)) continue;
      NormalizeVec3(&cv);
      cv.w = -(cv.x * A.x + cv.y * A.y + cv.z * A.z);
      int temp_count = 0;
      float strong_dist = 0.0f;
      for (int si = 0; si < valid_count; ++si) {
        const float3_& tp = spv3[si];
        const short2_& pos = spv[si];
        float fx = ((float)pos.x - camera.K[2]) / camera.K[0];
        float fy = ((float)pos.y - camera.K[5]) / camera.K[4];
        float fd = -cv.w / (cv.x * fx + cv.y * fy + cv.z);
        float dist = fabsf(fd - tp.z);
        residuals[si] = dist;
        if (dist < temp_thr) { temp_count++; strong_dist += dist; }
      }
      if (temp_count < 6) continue;
      if (temp_count > max_count) {
        if (!must_in_triangle && PointinTriangle(spv[a], spv[b], spv[c], x, y)) must_in_triangle = true;
        if (!has_consist_normal_plane && normal_consistency) has_consist_normal_plane = true;
        float fx = ((float)x - camera.K[2]) / camera.K[0];
        float fy = ((float)y - camera.K[5]) / camera.K[4];
        float fd = -cv.w / (cv.x * fx + cv.y * fy + cv.z);
        const float cd = fabsf(fd - cpw.z);
        best_plane = cv;
        max_count = temp_count;
        strong_dist /= temp_count;
        min_cost = cd;
        has_valid_plane = true;
        if ((double)temp_thr > (S.P.high_res_img ? 0.05 : 0.005)) {
          sort_small(residuals, valid_count);
          if (temp_thr < residuals[DPE_NEIGHBOUR_NUM]) continue;
          temp_thr = (float)((double)residuals[DPE_NEIGHBOUR_NUM] - 1e-6);
          temp_count = 0;
          for (int i = 0; i < valid_count; ++i) {
            if (residuals[i] < temp_thr) temp_count++;
            else break;
          }
          max_count = temp_count;
        }
      } else if (temp_count == max_count) {
        if (!must_in_triangle && PointinTriangle(spv[a], spv[b], spv[c], x, y)) must_in_triangle = true;
        float fx = ((float)x - camera.K[2]) / camera.K[0];
        float fy = ((float)y - camera.K[5]) / camera.K[4];
        float fd = -cv.w / (cv.x * fx + cv.y * fy + cv.z);
        const float cd = fabsf(fd - cpw.z);
        if (cd < min_cost) {
          best_plane = cv;
          max_count = temp_count;
          strong_dist /= temp_count;
          min_cost = cd;
        }
      }
    }
  }
  float weight[64];
  if (!has_valid_plane) { S.weak_reliable[center] = 0; return; }
  for (int i = 0; i < valid_count; ++i) {
    const float3_& tp = spv3[i];
    const short2_& pos = spv[i];
    float fx = ((float)pos.x - camera.K[2]) / camera.K[0];
    float fy = ((float)pos.y - camera.K[5]) / camera.K[4];
    float fd = -best_plane.w / (best_plane.x * fx + best_plane.y * fy + best_plane.z);
    float dist = fabsf(fd - tp.z);
    if (dist >= ransac_threshold) { spv[i] = mk_s2(-1, -1); weight[i] = FLT_MAX; continue; }
    weight[i] = dist;
  }
  sort_small_weighted(spv, weight, valid_count);
  for (int i = 1; i < DPE_NEIGHBOUR_NUM; ++i) nb[i] = spv[i - 1];
  S.weak_reliable[center] = 1;
}

// NeigbourUpdate (DPE.cu:2465-2481)
static void NeigbourUpdate(Pass& S, int x, int y) {
  const int c = x + y * S.W;
  if (S.weak[c] != DPE_WEAK) return;
  if (S.weak_reliable[c] != 1) S.weak[c] = DPE_UNKNOWN;
}

// ComputeMultiViewInitialCostandSelectedViews (DPE.cu:780-826)
// The selection half of ComputeMultiViewInitialCostandSelectedViews (DPE.cu:800-825): sort the
// cost vector (cv, zero-initialised past element 0 as `float cost_vector[32] = { 2.0f }`), average the
// top_k smallest valid costs, select every view whose unsorted cost is <= the k-th smallest.
static float TopKViews(float* cv, const float* cvc, int cost_count, int num_valid, int top_k_param, int nv,
                       uint32_t* sel) {
  const float cost_max = 2.0f;
  sort_small(cv, cost_count);
  *sel = 0;
  int top_k = std::min(num_valid, top_k_param);
  if (top_k > 0) {
    float cost = 0.0f;
    for (int i = 0; i < top_k; ++i) cost += cv[i];
    float thr = cv[top_k - 1];
    for (int i = 0; i < nv; ++i) if (cvc[i] <= thr) setBit(sel, i);
    return cost / top_k;
  }
  return cost_max;
}
static float InitialCostAndViews(Pass& S, int x, int y) {
  const int center = x + y * S.W;
  float4_ pl = S.planes[center];
  const float cost_max = 2.0f;
  float cv[32], cvc[32];
  for (int i = 0; i < 32; ++i) { cv[i] = 0.0f; cvc[i] = 0.0f; }
  cv[0] = 2.0f; cvc[0] = 2.0f;
  int cost_count = 0, num_valid = 0;
  for (int i = 1; i < S.N; ++i) {
    float c = NCCOld(S, x, y, i, pl);
    cv[i - 1] = c; cvc[i - 1] = c;
    cost_count++;
    if (c < cost_max) num_valid++;
  }
  return TopKViews(cv, cvc, cost_count, num_valid, S.P.top_k, S.N - 1, &S.sel[center]);
}

// ComputeMultiViewInitialCost (DPE.cu:828-857)
template <class CostF>
static float InitialCostOf(int N, uint32_t* sel, CostF ncc) {
  const float cost_max = 2.0f;
  int cost_count = 0;
  float cost = 0.0f;
  for (int i = 1; i < N; ++i) {
    if (isSet(*sel, i - 1)) {
      float c = ncc(i);
      if (c < cost_max) { cost_count++; cost += c; }
      else unSetBit(sel, i - 1);
    }
  }
  if (cost_count == 0) return cost_max;
  return cost / cost_count;
}
static float InitialCost(Pass& S, int x, int y) {
  const int center = x + y * S.W;
  float4_ pl = S.planes[center];
  return InitialCostOf(S.N, &S.sel[center], [&](int i) { return NCCOld(S, x, y, i, pl); });
}

// RandomInitialization (DPE.cu:1035-1063)
static void RandomInitialization(Pass& S, int x, int y) {
  const int center = x + y * S.W;
  const DpeCamera& c0 = S.cams[0];
  if (S.P.state == DPE_FIRST_INIT) {
    Philox rs; rng_init(&rs, (uint32_t)center, S.seed, STREAM_RANDOM_INIT, S.salt);
    // GenerateRandomPlaneHypothesis (:426-432)
    float depth = rng_uniform(&rs) * (S.P.depth_max - S.P.depth_min) + S.P.depth_min;
    float4_ ph = GenerateRandomNormal(c0, x, y, &rs, depth);
    ph.w = GetDistance2Origin(c0, x, y, depth, ph);
    S.planes[center] = ph;
    S.costs[center] = InitialCostAndViews(S, x, y);
  } else {
    float4_ ph = S.planes[center];
    ph = TransformNormal2RefCam(c0, ph);
    float depth = ph.w;
    ph.w = GetDistance2Origin(c0, x, y, depth, ph);
    S.planes[center] = ph;
    S.costs[center] = InitialCost(S, x, y);
  }
}

// Multi-hypothesis joint view selection shared by both sweeps (DPE.cu:1547-1615 / 1710-1779).
template <class DrawF>
static void ViewSelectionDraws(int nv, int iter, const float cost_array[8][32], const float* priors, DrawF draw,
                               uint8_t* vw, uint32_t* tsv, float* wnorm);
static void ViewSelection(Pass& S, int center, int iter, const float cost_array[8][32], const float* priors, Philox* rs,
                          uint8_t* vw, uint32_t* tsv, float* wnorm) {
  ViewSelectionDraws(S.N - 1, iter, cost_array, priors, [&]() { return rng_uniform(rs); }, vw, tsv, wnorm);
  (void)center;
}
template <class DrawF>
static void ViewSelectionDraws(int nv, int iter, const float cost_array[8][32], const float* priors, DrawF draw,
                               uint8_t* vw, uint32_t* tsv, float* wnorm) {
  for (int i = 0; i < DPE_MAX_IMAGES; ++i) vw[i] = 0;
  float sp[32];
  for (int i = 0; i < 32; ++i) sp[i] = 0.0f;
  const float cost_threshold = (float)(0.8 * (double)o_expf((float)(iter * iter) / (-90.0f)));
  for (int i = 0; i < nv; i++) {
    float count = 0; int count_false = 0; float tmpw = 0;
    for (int j = 0; j < 8; j++) {
      if (cost_array[j][i] < cost_threshold) { tmpw += o_expf(cost_array[j][i] * cost_array[j][i] / (-0.18f)); count++; }
      if (cost_array[j][i] > 1.2f) count_false++;
    }
    if (count > 2 && count_false < 3) sp[i] = tmpw / count;
    else if (count_false < 3) sp[i] = o_expf(cost_threshold * cost_threshold / (-0.32f));
    sp[i] = sp[i] * priors[i];
  }
  TransformPDFToCDF(sp, nv);
  for (int s = 0; s < 15; ++s) {
    const float rp = draw() - FLT_EPSILON;
    for (int id = 0; id < nv; ++id) {
      if (sp[id] > rp) { vw[id] += 1; break; }
    }
  }
  uint32_t t = 0; float wn = 0;
  for (int i = 0; i < nv; ++i) if (vw[i] > 0) { setBit(&t, i); wn += vw[i]; }
  *tsv = t; *wnorm = wn;
}

// PlaneHypothesisRefinementStrong (DPE.cu:1065-1118)
static void RefinementStrong(Pass& S, float4_* plane, float* depth, float* cost, Philox* rs, const uint8_t* vw, float wnorm,
                             int x, int y) {
  const float depth_perturbation = 0.02f, normal_perturbation = 0.02f;
  const DpeCamera& c0 = S.cams[0];
  const float dmin = S.P.depth_min, dmax = S.P.depth_max;
  float depth_rand = rng_uniform(rs) * (dmax - dmin) + dmin;
  float4_ prand = GenerateRandomNormal(c0, x, y, rs, *depth);
  float depth_perturbed = *depth;
  const float dminp = (1 - depth_perturbation) * depth_perturbed;
  const float dmaxp = (1 + depth_perturbation) * depth_perturbed;
  depth_perturbed = rng_uniform(rs) * (dmaxp - dminp) + dminp;   // do-while runs once (:1088-1090)
  float4_ ppert = GeneratePerturbedNormal(c0, x, y, *plane, rs, (float)(normal_perturbation * M_PI));
  const int num_planes = 5;
  float depths[5] = {depth_rand, *depth, depth_rand, *depth, depth_perturbed};
  float4_ normals[5] = {*plane, prand, prand, ppert, *plane};
  for (int i = 0; i < num_planes; ++i) {
    float4_ tp = normals[i];
    tp.w = GetDistance2Origin(c0, x, y, depths[i], tp);
    float tc = 0.0f;
    for (int j = 0; j < S.N - 1; ++j)
      if (vw[j] > 0) tc += vw[j] * NCCOld(S, x, y, j + 1, tp);
    tc /= wnorm;
    float db = ComputeDepthfromPlaneHypothesis(c0, tp, x, y);
    if (db >= dmin && db <= dmax && tc < *cost) { *depth = db; *plane = tp; *cost = tc; }
  }
}

// CheckerboardPropagationStrong (DPE.cu:1214-1666); reads of neighbours use the snapshot.
static void PropagationStrong(Pass& S, int x, int y, int iter) {
  const int W = S.W, H = S.H, N = S.N, nv = N - 1;
  const int center = y * W + x;
  const DpeCamera& c0 = S.cams[0];
  Philox rs; rng_init(&rs, (uint32_t)center, S.seed, STREAM_ITER_BASE + 4 * iter + 0, S.salt);
  const std::vector<float>& costs = S.costs_snap;
  const std::vector<float4_>& planes = S.planes_snap;
  float cost_array[8][32];
  for (int a = 0; a < 8; ++a) for (int b = 0; b < 32; ++b) cost_array[a][b] = 0.0f;
  cost_array[0][0] = 2.0f;   // `= { 2.0f }` initialises only [0][0] (:1236)
  bool flag[8] = {false};
  int positions[8] = {0};

  auto costvec = [&](const float4_& pl, float* out) { for (int i = 1; i < N; ++i) out[i - 1] = NCCOld(S, x, y, i, pl); };

  if (S.P.use_edge) {
    const short2_* en = &S.edge_neigh[(size_t)center * 8];
    const float max_edge_dist = MAXo(H, W) / 30.0f;
    const int min_step_len = 2;
    for (int d = 0; d < 8; ++d) {
      const int dx = kDir[d][0], dy = kDir[d][1];
      const int sx = MAXo(1, 5 - 2 * iter) * dx, sy = MAXo(1, 5 - 2 * iter) * dy;
      short2_ ep = en[d];
      double ex = (double)(ep.x - x), ey = (double)(ep.y - y);
      float dist = (float)std::sqrt(ex * ex + ey * ey);
      if (d >= 4) dist = (float)((double)dist / std::sqrt(2.0));
      if (S.edge[center]) dist = 11 * min_step_len;
      else if (ep.x == -1 || ep.y == -1 || dist > max_edge_dist) {
        dist = max_edge_dist;
        if (d >= 4) dist = (float)((double)dist / std::sqrt(2.0));
      }
      int step_num = MINo(MAXo(11, o_f2i(1.0f * dist / min_step_len)), 22);
      int step_len = MAXo(o_f2i(1.0f * dist / step_num), min_step_len);
      if (d < 4 && step_len % 2 == 1) step_len -= 1;
      int mx = 0, my = 0; float mc = FLT_MAX;
      for (int step = 0; step < step_num; ++step) {
        int fx = 0, fy = 0;
        if (d > 4) { if (d % 2) fx = dx; else fy = dy; }
        const int tx = x + sx + step * step_len * dx + fx, ty = y + sy + step * step_len * dy + fy;
        if (!(tx >= 0 && ty >= 0 && tx < W && ty < H)) continue;
        const int ptc = tx + ty * W;
        if (mc > costs[ptc]) { mx = tx; my = ty; mc = costs[ptc]; }
      }
      if (mc < FLT_MAX) {
        flag[d] = true;
        positions[d] = mx + my * W;
        costvec(planes[positions[d]], cost_array[d]);
      }
    }
    if (!S.edge[center]) {
      const float good_threshold = 0.8f * o_expf((float)(iter * iter) / (-90.0f));
      const float bad_threshold = 1.2f;
      for (int d = 0; d < 8; ++d) {
        const int dx = kDir[d][0], dy = kDir[d][1];
        const int sx = MAXo(1, 5 - 2 * iter) * dx, sy = MAXo(1, 5 - 2 * iter) * dy;
        bool hasResBefore = flag[d];
        float tca[32];
        for (int b = 0; b < 32; ++b) tca[b] = 0.0f;
        tca[0] = 2.0f;
        int mx = 0, my = 0; float mc = FLT_MAX;
        for (int step = 0; step < 11; ++step) {
          int fx = 0, fy = 0;
          if (d > 4) { if (d % 2) fx = dx; else fy = dy; }
          const int tx = x + sx + step * min_step_len * dx + fx, ty = y + sy + step * min_step_len * dy + fy;
          if (!(tx >= 0 && ty >= 0 && tx < W && ty < H)) continue;
          const int ptc = tx + ty * W;
          if (mc > costs[ptc]) { mx = tx; my = ty; mc = costs[ptc]; }
        }
        if (mc < FLT_MAX) {
          flag[d] = true;
          int tpos = mx + my * W;
          costvec(planes[tpos], tca);
          int good[2] = {0, 0}, bad[2] = {0, 0};
          for (int i = 0; i < 2; i++)
            for (int j = 0; j < nv; j++) {
              float val = (i == 0 ? cost_array[d][j] : tca[j]);
              if (val < good_threshold) good[i]++;
              if (val > bad_threshold) bad[i]++;
            }
          if (!hasResBefore || good[1] > good[0] || (good[1] == good[0] && bad[1] < bad[0])) {
            positions[d] = tpos;
            for (int j = 0; j < nv; j++) cost_array[d][j] = tca[j];
          }
        }
      }
    }
  } else {
    float costMin; int costMinPoint;
    int left_near = center - 1, left_far = center - 3, right_near = center + 1, right_far = center + 3;
    int up_near = center - W, up_far = center - 3 * W, down_near = center + W, down_far = center + 3 * W;
    if (y > 2) {
      flag[1] = true; costMin = costs[up_far]; costMinPoint = up_far;
      for (int i = 1; i < 11; ++i) if (y > 2 + 2 * i) { int pt = up_far - 2 * i * W; if (costs[pt] < costMin) { costMin = costs[pt]; costMinPoint = pt; } }
      up_far = costMinPoint; costvec(planes[up_far], cost_array[1]);
    }
    if (y < H - 3) {
      flag[3] = true; costMin = costs[down_far]; costMinPoint = down_far;
      for (int i = 1; i < 11; ++i) if (y < H - 3 - 2 * i) { int pt = down_far + 2 * i * W; if (costs[pt] < costMin) { costMin = costs[pt]; costMinPoint = pt; } }
      down_far = costMinPoint; costvec(planes[down_far], cost_array[3]);
    }
    if (x > 2) {
      flag[5] = true; costMin = costs[left_far]; costMinPoint = left_far;
      for (int i = 1; i < 11; ++i) if (x > 2 + 2 * i) { int pt = left_far - 2 * i; if (costs[pt] < costMin) { costMin = costs[pt]; costMinPoint = pt; } }
      left_far = costMinPoint; costvec(planes[left_far], cost_array[5]);
    }
    if (x < W - 3) {
      flag[7] = true; costMin = costs[right_far]; costMinPoint = right_far;
      for (int i = 1; i < 11; ++i) if (x < W - 3 - 2 * i) { int pt = right_far + 2 * i; if (costs[pt] < costMin) { costMin = costs[pt]; costMinPoint = pt; } }
      right_far = costMinPoint; costvec(planes[right_far], cost_array[7]);
    }
    if (y > 0) {
      flag[0] = true; costMin = costs[up_near]; costMinPoint = up_near;
      for (int i = 0; i < 3; ++i) {
        if (y > 1 + i && x > i) { int pt = up_near - (1 + i) * W - (1 + i); if (costs[pt] < costMin) { costMin = costs[pt]; costMinPoint = pt; } }
        if (y > 1 + i && x < W - 1 - i) { int pt = up_near - (1 + i) * W + (1 + i); if (costs[pt] < costMin) { costMin = costs[pt]; costMinPoint = pt; } }
      }
      up_near = costMinPoint; costvec(planes[up_near], cost_array[0]);
    }
    if (y < H - 1) {
      flag[2] = true; costMin = costs[down_near]; costMinPoint = down_near;
      for (int i = 0; i < 3; ++i) {
        if (y < H - 2 - i && x > i) { int pt = down_near + (1 + i) * W - (1 + i); if (costs[pt] < costMin) { costMin = costs[pt]; costMinPoint = pt; } }
        if (y < H - 2 - i && x < W - 1 - i) { int pt = down_near + (1 + i) * W + (1 + i); if (costs[pt] < costMin) { costMin = costs[pt]; costMinPoint = pt; } }
      }
      down_near = costMinPoint; costvec(planes[down_near], cost_array[2]);
    }
    if (x > 0) {
      flag[4] = true; costMin = costs[left_near]; costMinPoint = left_near;
      for (int i = 0; i < 3; ++i) {
        if (x > 1 + i && y > i) { int pt = left_near - (1 + i) - (1 + i) * W; if (costs[pt] < costMin) { costMin = costs[pt]; costMinPoint = pt; } }
        if (x > 1 + i && y < H - 1 - i) { int pt = left_near - (1 + i) + (1 + i) * W; if (costs[pt] < costMin) { costMin = costs[pt]; costMinPoint = pt; } }
      }
      left_near = costMinPoint; costvec(planes[left_near], cost_array[4]);
    }
    if (x < W - 1) {
      flag[6] = true; costMin = costs[right_near]; costMinPoint = right_near;
      for (int i = 0; i < 3; ++i) {
        if (x < W - 2 - i && y > i) { int pt = right_near + (1 + i) - (1 + i) * W; if (costs[pt] < costMin) { costMin = costs[pt]; costMinPoint = pt; } }
        if (x < W - 2 - i && y < H - 1 - i) { int pt = right_near + (1 + i) + (1 + i) * W; if (costs[pt] < costMin) { costMin = costs[pt]; costMinPoint = pt; } }
      }
      right_near = costMinPoint; costvec(planes[right_near], cost_array[6]);
    }
    positions[0] = up_near; positions[1] = up_far; positions[2] = down_near; positions[3] = down_far;
    positions[4] = left_near; positions[5] = left_far; positions[6] = right_near; positions[7] = right_far;
  }

  // priors from the 4-neighbourhood (:1552-1566); OOB index reads 0 (choice 4)
  uint8_t* vw = &S.view_weight[(size_t)center * DPE_MAX_IMAGES];
  float priors[32];
  for (int i = 0; i < 32; ++i) priors[i] = 0.0f;
  const long L = (long)W * H;
  long npos[4] = {(long)center - W, (long)center + W, (long)center - 1, (long)center + 1};
  for (int i = 0; i < 4; ++i) {
    if (flag[2 * i]) {
      uint32_t sv = (npos[i] >= 0 && npos[i] < L) ? S.sel_snap[npos[i]] : 0u;
      for (int j = 0; j < nv; ++j) priors[j] += isSet(sv, j) == 1 ? 0.9f : 0.1f;
    }
  }
  uint32_t tsv; float wnorm;
  ViewSelection(S, center, iter, cost_array, priors, &rs, vw, &tsv, &wnorm);

  float final_costs[8];
  for (int i = 0; i < 8; ++i) {
    final_costs[i] = 0.0f;
    for (int j = 0; j < nv; ++j) if (vw[j] > 0) final_costs[i] += vw[j] * cost_array[i][j];
    final_costs[i] /= wnorm;
  }
  const int mi = FindMinCostIndex(final_costs, 8);

  const float4_ cur = planes[center];
  float cost_now = 0.0f;
  for (int i = 0; i < nv; ++i) if (vw[i] > 0) cost_now += vw[i] * NCCOld(S, x, y, i + 1, cur);
  cost_now /= wnorm;
  const float cost_written = cost_now;
  S.costs[center] = cost_now;
  float depth_now = ComputeDepthfromPlaneHypothesis(c0, cur, x, y);
  float4_ pnow = cur;
  if (flag[mi]) {
    float db = ComputeDepthfromPlaneHypothesis(c0, planes[positions[mi]], x, y);
    if (db >= S.P.depth_min && db <= S.P.depth_max && final_costs[mi] < cost_now) {
      depth_now = db;
      pnow = planes[positions[mi]];
      cost_now = final_costs[mi];
      S.sel[center] = tsv;
    }
  }
  RefinementStrong(S, &pnow, &depth_now, &cost_now, &rs, vw, wnorm, x, y);
  if (S.P.state == DPE_REFINE_INIT) {
    if ((double)cost_now < (double)cost_written - 0.1) { S.costs[center] = cost_now; S.planes[center] = pnow; }
  } else {
    S.costs[center] = cost_now;
    S.planes[center] = pnow;
  }
}

// PlaneHypothesisRefinementWeak (DPE.cu:1120-1212)
static void RefinementWeak(Pass& S, float4_* plane, float* depth, float* cost, Philox* rs, const uint8_t* vw, float wnorm,
                           int x, int y) {
  const float depth_perturbation = 0.02f, normal_perturbation = 0.02f;
  const DpeCamera& c0 = S.cams[0];
  const float dmin = S.P.depth_min, dmax = S.P.depth_max;
  const int center = x + y * S.W;
  const int nv = S.N - 1;
  auto hyp_cost = [&](const float4_& tp) {
    float tc = 0.0f;
    for (int j = 0; j < nv; ++j) {
      if (vw[j] > 0) {
        float c = NCCNew(S, x, y, j + 1, tp);
        if (S.P.geom_consistency) tc += vw[j] * (c + S.P.geom_factor * GeomCost(S, x, y, j + 1, tp));
        else tc += vw[j] * c;
      }
    }
    return tc / wnorm;
  };
  if (S.weak[center] == DPE_WEAK) {
    float4_ fp = S.fit_plane[center];
    if (fp.x == 0 && fp.y == 0 && fp.z == 0) return;
    float tc = hyp_cost(fp);
    float db = ComputeDepthfromPlaneHypothesis(c0, fp, x, y);
    if (db >= dmin && db <= dmax && tc < *cost) { *depth = db; *plane = fp; *cost = tc; }
  }
  float depth_rand = rng_uniform(rs) * (dmax - dmin) + dmin;
  float4_ prand = GenerateRandomNormal(c0, x, y, rs, *depth);
  float depth_perturbed = *depth;
  const float dminp = (1 - depth_perturbation) * depth_perturbed;
  const float dmaxp = (1 + depth_perturbation) * depth_perturbed;
  depth_perturbed = rng_uniform(rs) * (dmaxp - dminp) + dminp;
  float4_ ppert = GeneratePerturbedNormal(c0, x, y, *plane, rs, (float)(normal_perturbation * M_PI));
  float depths[5] = {depth_rand, *depth, depth_rand, *depth, depth_perturbed};
  float4_ normals[5] = {*plane, prand, prand, ppert, *plane};
  for (int i = 0; i < 5; ++i) {
    float4_ tp = normals[i];
    tp.w = GetDistance2Origin(c0, x, y, depths[i], tp);
    float tc = hyp_cost(tp);
    float db = ComputeDepthfromPlaneHypothesis(c0, tp, x, y);
    if (db >= dmin && db <= dmax && tc < *cost) { *depth = db; *plane = tp; *cost = tc; }
  }
}

// CheckerboardPropagationWeak (DPE.cu:1668-1862)
static void PropagationWeak(Pass& S, int x, int y, int iter) {
  const int W = S.W, N = S.N, nv = N - 1;
  const int center = y * W + x;
  const DpeCamera& c0 = S.cams[0];
  Philox rs; rng_init(&rs, (uint32_t)center, S.seed, STREAM_ITER_BASE + 4 * iter + 2, S.salt);
  float cost_array[8][32];
  for (int a = 0; a < 8; ++a) for (int b = 0; b < 32; ++b) cost_array[a][b] = 0.0f;
  cost_array[0][0] = 2.0f;
  bool flag[8] = {false};
  int positions[8] = {0};
  float4_ nph[8];
  for (int i = 0; i < 8; ++i) {
    const short2_ np = Neighbour(S, center, i + 1);
    if (np.x == -1 || np.y == -1 || S.weak[np.x + np.y * W] != DPE_STRONG) { flag[i] = false; continue; }
    positions[i] = np.x + np.y * W;
    flag[i] = true;
    const float4_ pl = S.planes[positions[i]];
    for (int v = 1; v < N; ++v) cost_array[i][v - 1] = NCCNew(S, x, y, v, pl);
    nph[i] = pl;
  }
  uint8_t* vw = &S.view_weight[(size_t)center * DPE_MAX_IMAGES];
  float priors[32];
  for (int i = 0; i < 32; ++i) priors[i] = 0.0f;
  for (int i = 0; i < 8; ++i) {
    const short2_ np = Neighbour(S, center, i + 1);
    if (np.x == -1 || np.y == -1) continue;
    uint32_t sv = S.sel[np.x + np.y * W];
    for (int j = 0; j < nv; ++j) priors[j] += isSet(sv, j) == 1 ? 0.9f : 0.1f;
  }
  uint32_t tsv; float wnorm;
  ViewSelection(S, center, iter, cost_array, priors, &rs, vw, &tsv, &wnorm);

  float final_costs[8];
  for (int i = 0; i < 8; ++i) {
    final_costs[i] = 0.0f;
    for (int j = 0; j < nv; ++j) {
      if (vw[j] > 0) {
        if (S.P.geom_consistency) {
          if (flag[i]) final_costs[i] += vw[j] * (cost_array[i][j] + S.P.geom_factor * GeomCost(S, x, y, j + 1, S.planes[positions[i]]));
          else final_costs[i] += vw[j] * (cost_array[i][j] + S.P.geom_factor * 3.0f);
        } else {
          final_costs[i] += vw[j] * cost_array[i][j];
        }
      }
    }
    final_costs[i] /= wnorm;
  }
  const int mi = FindMinCostIndex(final_costs, 8);
  const float4_ cur = S.planes[center];
  float cost_now = 0.0f;
  for (int i = 0; i < nv; ++i) {
    if (vw[i] == 0) continue;   // exact: 0 * finite == +0 (choice 6)
    float c = NCCNew(S, x, y, i + 1, cur);
    if (S.P.geom_consistency) cost_now += vw[i] * (c + S.P.geom_factor * GeomCost(S, x, y, i + 1, cur));
    else cost_now += vw[i] * c;
  }
  cost_now /= wnorm;
  const float cost_written = cost_now;
  S.costs[center] = cost_now;
  float depth_now = ComputeDepthfromPlaneHypothesis(c0, cur, x, y);
  float4_ pnow = cur;
  if (flag[mi]) {
    float db = ComputeDepthfromPlaneHypothesis(c0, nph[mi], x, y);
    if (db >= S.P.depth_min && db <= S.P.depth_max && final_costs[mi] < cost_now) {
      depth_now = db; pnow = nph[mi]; cost_now = final_costs[mi]; S.sel[center] = tsv;
    }
  }
  RefinementWeak(S, &pnow, &depth_now, &cost_now, &rs, vw, wnorm, x, y);
  if (S.P.state == DPE_REFINE_INIT) {
    if ((double)cost_now < (double)cost_written - 0.1) { S.costs[center] = cost_now; S.planes[center] = pnow; }
  } else {
    S.costs[center] = cost_now; S.planes[center] = pnow;
  }
  // final cost with the Old NCC (:1845-1861)
  {
    const float4_ pl = S.planes[center];
    float c2 = 0.0f;
    for (int i = 0; i < nv; ++i) if (vw[i] > 0) c2 += vw[i] * NCCOld(S, x, y, i + 1, pl);
    c2 /= wnorm;
    S.costs[center] = c2;
  }
}

// RANSACToGetFitPlane (DPE.cu:2891-3124)
static void RANSACFitPlane(Pass& S, int x, int y, int iter) {
  const int W = S.W;
  const int center = x + y * W;
  if (S.weak[center] != DPE_WEAK) return;   // copy to fit_plane is dead (choice 6)
  Philox rs; rng_init(&rs, (uint32_t)center, S.seed, STREAM_ITER_BASE + 4 * iter + 1, S.salt);
  const DpeCamera& camera = S.cams[0];
  bool edge_limit = false;
  if (S.P.use_limit) {
    edge_limit = true;
    if (S.P.use_edge) {
      float cv = S.complex_[center];
      const float rp = rng_uniform(&rs) - FLT_EPSILON;
      if (rp < cv) edge_limit = false;
    }
  }
  short2_ sp[8]; float3_ sp3[8]; float3_ spn[8];
  int sc = 0;
  float X[3];
  for (int i = 1; i < DPE_NEIGHBOUR_NUM; ++i) {
    short2_ tp = Neighbour(S, center, i);
    if (tp.x == -1 || tp.y == -1) continue;
    sp[sc] = tp;
    const int tc = tp.x + tp.y * W;
    float depth = ComputeDepthfromPlaneHypothesis(camera, S.planes[tc], tp.x, tp.y);
    Get3DPoint(camera, tp.x, tp.y, depth, X);
    sp3[sc] = {X[0], X[1], X[2]};
    float4_ n4 = S.planes[tc];
    spn[sc] = {n4.x, n4.y, n4.z};
    sc++;
  }
  if (sc < 3) { S.fit_plane[center] = S.planes[center]; return; }
  int iteration = 50;
  int ua = -1, ub = -1, uc = -1;
  float min_cost = FLT_MAX;
  float4_ best = {0, 0, 0, 0};
  bool has_best = false, has_strong_plane = false;
  bool must_in_triangle = (S.P.use_label && S.label[center] > 0 && edge_limit) ? false : true;
  uint8_t edge_test[8][8];
  std::memset(edge_test, 0, sizeof(edge_test));
  while (iteration--) {
    int a = (int)(rng_u32(&rs) % (uint32_t)sc);
    int b = (int)(rng_u32(&rs) % (uint32_t)sc);
    int c = (int)(rng_u32(&rs) % (uint32_t)sc);
    if (a == b || b == c || a == c) continue;
    bool is_strong_plane = false;
    if (S.P.geom_consistency && edge_limit) {
      const float3_ &AN = spn[a], &BN = spn[b], &CN = spn[c];
      is_strong_plane = true;
      if ((double)(AN.x * BN.x + AN.y * BN.y + AN.z * BN.z) < 0.8660254 ||
          (double)(AN.x * CN.x + AN.y * CN.y + AN.z * CN.z) < 0.8660254 ||
          (double)(BN.x * CN.x + BN.y * CN.y + BN.z * CN.z) < 0.8660254)
        is_strong_plane = false;
      if (has_strong_plane && !is_strong_plane) continue;
    }
    if (must_in_triangle && !PointinTriangle(sp[a], sp[b], sp[c], x, y)) continue;
    if (edge_limit) {
      if (edge_test[a][b] == 0) edge_test[a][b] = edge_test[b][a] = (BresenhamLine(S, sp[a].x, sp[a].y, sp[b].x, sp[b].y) ? 1 : 2);
      if (edge_test[b][c] == 0) edge_test[b][c] = edge_test[c][b] = (BresenhamLine(S, sp[b].x, sp[b].y, sp[c].x, sp[c].y) ? 1 : 2);
      if (edge_test[c][a] == 0) edge_test[c][a] = edge_test[a][c] = (BresenhamLine(S, sp[c].x, sp[c].y, sp[a].x, sp[a].y) ? 1 : 2);
      if (edge_test[a][b] == 1 || edge_test[b][c] == 1 || edge_test[c][a] == 1) continue;
    }
    const float3_ &A = sp3[a], &B = sp3[b], &C = sp3[c];
    float3_ A_C = {A.x - C.x, A.y - C.y, A.z - C.z};
    float3_ B_C = {B.x - C.x, B.y - C.y, B.z - C.z};
    float4_ cv;
    cv.x = A_C.y * B_C.z - B_C.y * A_C.z;
    cv.y = -(A_C.x * B_C.z - B_C.x * A_C.z);
    cv.z = A_C.x * B_C.y - B_C.x * A_C.y;
    if ((cv.x == 0 && cv.y == 0 && cv.z == 0) || std::isnan(cv.x) || std::isnan(cv.y) || std::isnan(cv.z)) continue;
    NormalizeVec3(&cv);
    cv.w = -(cv.x * A.x + cv.y * A.y + cv.z * A.z);
    if (!has_strong_plane && is_strong_plane) has_strong_plane = true;
    float tcost = 0.0f;
    for (int si = 0; si < sc; ++si) {
      if (si == a || si == b || si == c) continue;
      const float3_& tp = sp3[si];
      const short2_& tpix = sp[si];
      float fx = ((float)tpix.x - camera.K[2]) / camera.K[0];
      float fy = ((float)tpix.y - camera.K[5]) / camera.K[4];
      float fd = -cv.w / (cv.x * fx + cv.y * fy + cv.z);
      tcost += fabsf(fd - tp.z);
    }
    if (tcost < min_cost) {
      if (!must_in_triangle && PointinTriangle(sp[a], sp[b], sp[c], x, y)) must_in_triangle = true;
      min_cost = tcost; best = cv; has_best = true; ua = a; ub = b; uc = c;
    }
  }
  if (has_best) {
    float depth = ComputeDepthfromPlaneHypothesis(camera, S.planes[center], x, y);
    float4_ vd = GetViewDirection(camera, x, y, depth);
    float dot = best.x * vd.x + best.y * vd.y + best.z * vd.z;
    if (dot > 0) { best.x = -best.x; best.y = -best.y; best.z = -best.z; best.w = -best.w; }
    S.fit_plane[center] = best;
    if (S.P.use_radius) {
      if (must_in_triangle) {
        const short2_ &A = sp[ua], &B = sp[ub], &C = sp[uc];
        float a = sqrtf((float)((A.x - B.x) * (A.x - B.x) + (A.y - B.y) * (A.y - B.y)));
        float b = sqrtf((float)((B.x - C.x) * (B.x - C.x) + (B.y - C.y) * (B.y - C.y)));
        float c = sqrtf((float)((C.x - A.x) * (C.x - A.x) + (C.y - A.y) * (C.y - A.y)));
        float p = (float)((double)(a + b + c) / 2.0);
        float Sarea = sqrtf(p * (p - a) * (p - b) * (p - c));
        int radius = o_d2i(floor((double)sqrtf(Sarea) / 2.0));
        float Ad = sqrtf((float)((A.x - x) * (A.x - x) + (A.y - y) * (A.y - y)));
        float Bd = sqrtf((float)((B.x - x) * (B.x - x) + (B.y - y) * (B.y - y)));
        float Cd = sqrtf((float)((C.x - x) * (C.x - x) + (C.y - y) * (C.y - y)));
        float min_dis = MINo(MINo(Ad, Bd), Cd);
        if (2.5 * (double)min_dis < (double)radius) radius = o_f2i(min_dis);
        if (edge_limit) {
          if (S.P.use_edge) {
            float med = FLT_MAX;
            const short2_* en = &S.edge_neigh[(size_t)center * 8];
            for (int d = 0; d < 8; ++d) {
              short2_ ep = en[d];
              if (ep.x == -1 || ep.y == -1) continue;
              float dist = sqrtf((float)((ep.x - x) * (ep.x - x) + (ep.y - y) * (ep.y - y)));
              med = MINo(med, dist);
            }
            if (med < (float)radius) radius = o_f2i(med);
          }
          if (S.P.use_label && S.label[center] > 0) {
            float mbd = FLT_MAX;
            const short2_* lb = &S.label_boundary[(size_t)center * 8];
            for (int d = 0; d < 8; ++d) {
              short2_ bp = lb[d];
              if (bp.x == -1 || bp.y == -1) continue;
              double dxx = (double)(x - bp.x), dyy = (double)(y - bp.y);
              float dist = (float)std::sqrt(dxx * dxx + dyy * dyy);
              mbd = MINo(mbd, dist);
            }
            if (mbd < (float)radius) radius = o_f2i(mbd);
          }
        }
        while ((radius << 1) % 5 != 0) radius--;
        if (!edge_limit) S.radius[center] = radius > S.P.strong_radius ? 0 : S.P.strong_radius;
        else S.radius[center] = radius > S.P.strong_radius ? radius : S.P.strong_radius;
      } else {
        S.radius[center] = S.P.strong_radius;
      }
    }
  } else {
    S.fit_plane[center] = {0, 0, 0, 0};
    if (S.P.use_radius) S.radius[center] = S.P.strong_radius;
  }
}

// GetDepthandNormal (DPE.cu:1940-1955)
static void GetDepthandNormal(Pass& S, int x, int y) {
  const int c = y * S.W + x;
  S.planes[c].w = ComputeDepthfromPlaneHypothesis(S.cams[0], S.planes[c], x, y);
  S.planes[c] = TransformNormal(S.cams[0], S.planes[c]);
}

// CheckerboardFilterStrong (DPE.cu:1957-2067)
static void FilterStrong(Pass& S, int x, int y) {
  const int W = S.W, H = S.H;
  const int center = y * W + x;
  if (S.weak[center] == DPE_WEAK) return;
  float filter[21];
  int index = 0;
  const std::vector<float4_>& P = S.planes;
  filter[index++] = P[center].w;
  const int left = center - 1, leftleft = center - 3, up = center - W, upup = center - 3 * W;
  const int down = center + W, downdown = center + 3 * W, right = center + 1, rightright = center + 3;
  if (S.costs[center] < 0.001f) return;
  auto st = [&](int i) { return S.weak[i] == DPE_STRONG; };
  if (y > 0 && st(up)) filter[index++] = P[up].w;
  if (y > 2 && st(upup)) filter[index++] = P[upup].w;
  if (y > 4 && st(upup - W * 2)) filter[index++] = P[upup - W * 2].w;
  if (y < H - 1 && st(down)) filter[index++] = P[down].w;
  if (y < H - 3 && st(downdown)) filter[index++] = P[downdown].w;
  if (y < H - 5 && st(downdown + W * 2)) filter[index++] = P[downdown + W * 2].w;
  if (x > 0 && st(left)) filter[index++] = P[left].w;
  if (x > 2 && st(leftleft)) filter[index++] = P[leftleft].w;
  if (x > 4 && st(leftleft - 2)) filter[index++] = P[leftleft - 2].w;
  if (x < W - 1 && st(right)) filter[index++] = P[right].w;
  if (x < W - 3 && st(rightright)) filter[index++] = P[rightright].w;
  if (x < W - 5 && st(rightright + 2)) filter[index++] = P[rightright + 2].w;
  if (y > 0 && x < W - 2 && st(up + 2)) filter[index++] = P[up + 2].w;
  if (y < H - 1 && x < W - 2 && st(down + 2)) filter[index++] = P[down + 2].w;
  if (y > 0 && x > 1 && st(up - 2)) filter[index++] = P[up - 2].w;
  if (y < H - 1 && x > 1 && st(down - 2)) filter[index++] = P[down - 2].w;
  if (x > 0 && y > 2 && st(left - W * 2)) filter[index++] = P[left - W * 2].w;
  if (x < W - 1 && y > 2 && st(right - W * 2)) filter[index++] = P[right - W * 2].w;
  if (x > 0 && y < H - 2 && st(left + W * 2)) filter[index++] = P[left + W * 2].w;
  if (x < W - 1 && y < H - 2 && st(right + W * 2)) filter[index++] = P[right + W * 2].w;
  sort_small(filter, index);
  int m = index / 2;
  if (index % 2 == 0) S.planes[center].w = (filter[m - 1] + filter[m]) / 2;
  else S.planes[center].w = filter[m];
}

// Baseline helper shared by DepthToWeak / LocalRefine (DPE.cu:2629-2648, 2776-2795)
struct CostNow { float cost_now, base_line, weight_normal; int valid; };

static CostNow CostAndBaseline(Pass& S, int x, int y, const float4_& op, float od) {
  const int center = x + y * S.W;
  const uint8_t* vw = &S.view_weight[(size_t)DPE_MAX_IMAGES * center];
  CostNow r = {0.0f, 0.0f, 0.0f, 0};
  for (int si = 1; si < S.N; ++si) {
    int vi = si - 1;
    if (isSet(S.sel[center], vi)) {
      float4_ tp = op;
      tp.w = GetDistance2Origin(S.cams[0], x, y, od, tp);
      float tc = NCCOld(S, x, y, si, tp);
      if (S.P.geom_consistency) tc += S.P.geom_factor * GeomCost(S, x, y, si, tp);
      r.cost_now += (tc * vw[vi]);
      r.weight_normal += vw[vi];
      float cd[3];
      cd[0] = S.cams[0].c[0] - S.cams[si].c[0];
      cd[1] = S.cams[0].c[1] - S.cams[si].c[1];
      cd[2] = S.cams[0].c[2] - S.cams[si].c[2];
      double tv = cd[0] * cd[0] + cd[1] * cd[1] + cd[2] * cd[2];
      r.base_line += sqrtf((float)tv);
      r.valid++;
    }
  }
  return r;
}

// DepthToWeak's classification (DPE.cu:2700-2745) of the 61-sample cost curve pc[pd + 30]
static uint8_t ClassifyCostCurve(const float* pc, int weak_peak_radius) {
  const int radius = 30, n = 2 * radius + 1;
  bool is_peak[61];
  for (int i = 0; i < n; ++i) is_peak[i] = false;
  int peak_count = 0, min_peak = 0;
  float min_cost = 2.0f;
  for (int i = 2; i < n - 2; ++i) {
    if (pc[i - 1] > pc[i] && pc[i + 1] > pc[i]) {
      is_peak[i] = true; peak_count++;
      if (pc[i] < min_cost) { min_peak = i; min_cost = pc[i]; }
    }
  }
  if (abs(min_peak - radius) > weak_peak_radius || pc[min_peak] > 0.5f) return DPE_WEAK;
  if (peak_count == 1) return pc[min_peak] <= 0.15f ? DPE_STRONG : DPE_WEAK;
  float var = 0.0f;
  for (int i = 2; i < n - 2; ++i) if (is_peak[i] && i != min_peak) { float d = pc[i] - min_cost; var += d * d; }
  var = sqrtf(var);
  var /= (peak_count - 1);
  return var > 0.2f ? DPE_STRONG : DPE_WEAK;
}

// DepthToWeak (DPE.cu:2593-2747)
static void DepthToWeak(Pass& S, int x, int y) {
  const int W = S.W, H = S.H;
  const int min_margin = 6;
  const int center = x + y * W;
  if (x < min_margin || y < min_margin || x >= W - min_margin || y >= H - min_margin) { S.weak[center] = DPE_UNKNOWN; return; }
  const DpeCamera& c0 = S.cams[0];
  const uint8_t* vw = &S.view_weight[(size_t)DPE_MAX_IMAGES * center];
  float4_ op = TransformNormal2RefCam(c0, S.planes[center]);
  float od = op.w;
  if (od == 0) { S.weak[center] = DPE_UNKNOWN; return; }
  CostNow cn = CostAndBaseline(S, x, y, op, od);
  if (cn.valid == 0) { S.weak[center] = DPE_UNKNOWN; return; }
  cn.cost_now /= cn.weight_normal;
  cn.base_line /= cn.valid;
  float disp = c0.K[0] * cn.base_line / od;
  const int radius = 30;
  float pc[61];
  for (int pd = -radius; pd <= radius; pd += 1) {
    float p_depth = c0.K[0] * cn.base_line / (disp + (float)pd);
    if (p_depth < S.P.depth_min || p_depth > S.P.depth_max) { pc[pd + radius] = 2.0f; continue; }
    float4_ tp = op;
    tp.w = GetDistance2Origin(c0, x, y, p_depth, tp);
    float p_cost = 0.0f;
    for (int si = 1; si < S.N; ++si) {
      int vi = si - 1;
      float tcst = 0.0f;
      if (isSet(S.sel[center], vi)) {
        tcst += NCCOld(S, x, y, si, tp);
        if (S.P.geom_consistency) tcst += S.P.geom_factor * GeomCost(S, x, y, si, tp);
        p_cost += (tcst * vw[vi]);
      }
    }
    p_cost /= cn.weight_normal;
    pc[pd + radius] = MINo(2.0f, p_cost);
  }
  S.weak[center] = ClassifyCostCurve(pc, S.P.weak_peak_radius);
}

// LocalRefine's choice (DPE.cu:2796-2834): the in-range hypothesis of least cost in pd order (first
// of equals), taken when it improves the current cost by more than 0.1 (compared in double).
static bool LocalRefineSelect(const float* tc, const int* ok, const float* p_depth, float cost_now, float od,
                              float* out_depth) {
  float min_cost = 2.0f, best_depth = od;
  for (int k = 0; k < 11; ++k) {
    if (!ok[k]) continue;
    if (tc[k] < min_cost) { min_cost = tc[k]; best_depth = p_depth[k]; }
  }
  *out_depth = best_depth;
  return (double)(cost_now - min_cost) > 0.1;
}

// LocalRefine (DPE.cu:2749-2835)
static void LocalRefine(Pass& S, int x, int y) {
  const int center = x + y * S.W;
  const DpeCamera& c0 = S.cams[0];
  const uint8_t* vw = &S.view_weight[(size_t)DPE_MAX_IMAGES * center];
  float4_ op = TransformNormal2RefCam(c0, S.planes[center]);
  float od = op.w;
  if (od == 0) return;
  CostNow cn = CostAndBaseline(S, x, y, op, od);
  if (cn.weight_normal == 0 || cn.valid == 0) return;
  cn.cost_now /= cn.weight_normal;
  cn.base_line /= cn.valid;
  float disp = c0.K[0] * cn.base_line / od;
  const int radius = 5;
  float tcs[11], depths[11];
  int ok[11];
  for (int pd = -radius; pd <= radius; ++pd) {
    float p_depth = c0.K[0] * cn.base_line / (disp + (float)pd);
    depths[pd + radius] = p_depth;
    ok[pd + radius] = !(p_depth < S.P.depth_min || p_depth > S.P.depth_max);
    tcs[pd + radius] = 2.0f;
    if (!ok[pd + radius]) continue;
    float4_ tp = op;
    tp.w = GetDistance2Origin(c0, x, y, p_depth, tp);
    float tc = 0.0f;
    for (int si = 1; si < S.N; ++si) {
      int vi = si - 1;
      if (isSet(S.sel[center], vi)) {
        tc += (NCCOld(S, x, y, si, tp) * vw[vi]);
        if (S.P.geom_consistency) tc += (S.P.geom_factor * GeomCost(S, x, y, si, tp) * vw[vi]);
      }
    }
    tc /= cn.weight_normal;
    tcs[pd + radius] = tc;
  }
  float best_depth;
  if (LocalRefineSelect(tcs, ok, depths, cn.cost_now, od, &best_depth)) S.planes[center].w = best_depth;
}

// half-sweep geometry (DPE.cu:1864-1938): Black = (x+y) even, Red = (x+y) odd.
// Rows covered by the half grid: grid_size_half.y = ((H/2)+15)/16 blocks of 16 rows of pairs
// (DPE.cu:3143), so for odd H with (H/2) % 16 == 0 the last row is never visited.
template <class F>
static void HalfSweep(Pass& S, int colour, F f) {
  const int rows = std::min(S.H, 2 * 16 * (((S.H / 2) + 15) / 16));
  parallel_rows(rows, S.nthreads, [&](int y) {
    for (int x = ((y + colour) & 1); x < S.W; x += 2) f(x, y);
  });
}
template <class F>
static void Full(Pass& S, F f) {
  parallel_rows(S.H, S.nthreads, [&](int y) { for (int x = 0; x < S.W; ++x) f(x, y); });
}

static int RunPass(Pass& S) {
  const int W = S.W;
  (void)W;
  ComputeViewConstants(S);
  {   // GenNeighbours constants (DPE.cu:2147-2152)
    const float angle = 45.0f / S.P.rotate_time;
    S.gn_cos = (float)cos((double)angle * M_PI / 180.f);
    S.gn_sin = (float)sin((double)angle * M_PI / 180.f);
    S.gn_thr = (float)cos((double)(angle / 2.0f) * M_PI / 180.0f);
    S.gn_shift = MAXo(o_d2i(tan((double)(angle / 2.0f) * M_PI / 180.0f) * 20), 1);
  }
  // ORACLE_PROFILE=1: wall time of each stage on stderr (where the checker's time goes)
  static const bool prof = [] { const char* e = getenv("ORACLE_PROFILE"); return e && atoi(e) != 0; }();
  auto t0 = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (!prof) return;
    const auto t1 = std::chrono::steady_clock::now();
    fprintf(stderr, "oracle %-16s %8.3f s\n", what, std::chrono::duration<double>(t1 - t0).count());
    t0 = t1;
  };
  // RunPatchMatch launch sequence (DPE.cu:3150-3226)
  Full(S, [&](int x, int y) { GenEdgeInform(S, x, y); });
  Full(S, [&](int x, int y) { FindNearestStrongPoint(S, x, y); });
  mark("edge+nearest");
  Full(S, [&](int x, int y) { GenNeighbours(S, x, y); });
  Full(S, [&](int x, int y) { NeigbourUpdate(S, x, y); });
  mark("gen_neighbours");
  Full(S, [&](int x, int y) { RandomInitialization(S, x, y); });
  mark("init");
  for (int it = 0; it < S.P.max_iterations; ++it) {
    for (int colour = 0; colour < 2; ++colour) {
      S.planes_snap = S.planes; S.costs_snap = S.costs; S.sel_snap = S.sel;
      HalfSweep(S, colour, [&](int x, int y) { if (S.weak[x + y * S.W] != DPE_WEAK) PropagationStrong(S, x, y, it); });
    }
    mark("strong");
    Full(S, [&](int x, int y) { RANSACFitPlane(S, x, y, it); });
    mark("ransac");
    for (int colour = 0; colour < 2; ++colour)
      HalfSweep(S, colour, [&](int x, int y) { if (S.weak[x + y * S.W] == DPE_WEAK) PropagationWeak(S, x, y, it); });
    mark("weak");
  }
  Full(S, [&](int x, int y) { GetDepthandNormal(S, x, y); });
  for (int colour = 0; colour < 2; ++colour) HalfSweep(S, colour, [&](int x, int y) { FilterStrong(S, x, y); });
  mark("filter");
  Full(S, [&](int x, int y) { DepthToWeak(S, x, y); });
  mark("depth_to_weak");
  Full(S, [&](int x, int y) { LocalRefine(S, x, y); });
  mark("local_refine");
  return 0;
}

static char g_err[512];

}  // namespace

extern "C" {

const char* oracle_last_error(void) { return g_err; }

// the tap reciprocal of restatement choice 8 (oracle_math.h o_rcp_tap) over n inputs
void oracle_rcp_tap(const float* z, float* out, long n) {
  for (long i = 0; i < n; ++i) out[i] = o_rcp_tap(z[i]);
}

// Runs one pass on the CPU.  Same structs and in/out semantics as dpe_pm_run (include/dpe_mvs.h).
int oracle_pm_run(const DpePassInput* in, const DpePassState* st, int nthreads) {
  g_err[0] = 0;
  if (!in || !st || !st->planes || !st->weak_info || !st->selected_views) { snprintf(g_err, sizeof g_err, "null arg"); return DPE_ERR_ARG; }
  if (in->num_images > DPE_MAX_IMAGES) { snprintf(g_err, sizeof g_err, "too many images"); return DPE_ERR_TOO_MANY; }
  if (in->num_images < 2 || in->width <= 0 || in->height <= 0) { snprintf(g_err, sizeof g_err, "bad shape"); return DPE_ERR_ARG; }
  Pass S;
  S.W = in->width; S.H = in->height; S.N = in->num_images;
  S.P = in->params;
  S.P.num_images = S.N;
  S.seed = in->seed; S.salt = in->pass_salt;
  S.nthreads = nthreads < 1 ? 1 : nthreads;
  const size_t L = (size_t)S.W * S.H;
  S.cams.assign(in->cams, in->cams + S.N);
  S.img.resize(S.N);
  for (int i = 0; i < S.N; ++i) S.img[i].assign(in->images[i], in->images[i] + L);
  if (S.P.geom_consistency) {
    if (!in->depths) { snprintf(g_err, sizeof g_err, "geom needs depths"); return DPE_ERR_ARG; }
    S.dep.resize(S.N);
    for (int i = 1; i < S.N; ++i) {
      if (!in->depths[i]) { snprintf(g_err, sizeof g_err, "missing depth %d", i); return DPE_ERR_ARG; }
      S.dep[i].assign(in->depths[i], in->depths[i] + L);
    }
  }
  if (S.P.use_edge || S.P.use_limit) {
    if (!in->edge || !in->edge_low_res || in->low_width <= 0 || in->low_height <= 0) { snprintf(g_err, sizeof g_err, "edges required"); return DPE_ERR_ARG; }
    S.edge.assign(in->edge, in->edge + L);
    S.LW = in->low_width; S.LH = in->low_height;
    S.edge_low.assign(in->edge_low_res, in->edge_low_res + (size_t)S.LW * S.LH);
  }
  if (S.P.use_label) {
    if (!in->label) { snprintf(g_err, sizeof g_err, "labels required"); return DPE_ERR_ARG; }
    S.label.assign(in->label, in->label + L);
  }
  S.planes.resize(L);
  std::memcpy(S.planes.data(), st->planes, L * sizeof(float4_));
  S.sel.assign(st->selected_views, st->selected_views + L);
  if (S.P.use_APD) S.weak.assign(st->weak_info, st->weak_info + L);
  else S.weak.assign(L, (uint8_t)DPE_STRONG);                // DPE.cpp:873-881
  S.costs.assign(L, 0.0f);
  S.fit_plane.assign(L, {0, 0, 0, 0});                        // cudaMemset (DPE.cpp:982)
  S.complex_.assign(L, 0.0f);
  S.weak_reliable.assign(L, 0);
  S.view_weight.assign(L * DPE_MAX_IMAGES, 0);
  S.neighbours.assign(L * 9, mk_s2(-1, -1));
  S.nearest_strong.assign(L, mk_s2(-1, -1));
  S.edge_neigh.assign(L * 8, mk_s2(-1, -1));
  S.label_boundary.assign(L * 8, mk_s2(-1, -1));
  S.radius.assign(L, 0);
  RunPass(S);
  std::memcpy(st->planes, S.planes.data(), L * sizeof(float4_));
  std::memcpy(st->weak_info, S.weak.data(), L);
  std::memcpy(st->selected_views, S.sel.data(), L * sizeof(uint32_t));
  if (st->costs) std::memcpy(st->costs, S.costs.data(), L * sizeof(float));
  return DPE_OK;
}

// ---- known-answer entry points for per-function tests ------------------------------------
// Old-NCC cost of one (pixel, source view, ref-frame plane) on the given pass inputs.
float oracle_ncc_old(const DpePassInput* in, int x, int y, int view, const float plane[4]) {
  Pass S;
  S.W = in->width; S.H = in->height; S.N = in->num_images; S.P = in->params;
  const size_t L = (size_t)S.W * S.H;
  S.cams.assign(in->cams, in->cams + S.N);
  S.img.resize(S.N);
  for (int i = 0; i < S.N; ++i) S.img[i].assign(in->images[i], in->images[i] + L);
  ComputeViewConstants(S);
  float4_ p = {plane[0], plane[1], plane[2], plane[3]};
  return NCCOld(S, x, y, view, p);
}
// Pass S from the inputs of a per-function test (images, cameras, params, depths when geom)
static void kat_pass(Pass& S, const DpePassInput* in) {
  S.W = in->width; S.H = in->height; S.N = in->num_images; S.P = in->params;
  const size_t L = (size_t)S.W * S.H;
  S.cams.assign(in->cams, in->cams + S.N);
  S.img.resize(S.N);
  for (int i = 0; i < S.N; ++i) if (in->images && in->images[i]) S.img[i].assign(in->images[i], in->images[i] + L);
  if (in->depths) {
    S.dep.resize(S.N);
    for (int i = 1; i < S.N; ++i) if (in->depths[i]) S.dep[i].assign(in->depths[i], in->depths[i] + L);
  }
  ComputeViewConstants(S);
}
// MakeHomography (restatement choice 3) of source view `view` for a reference-frame plane
void oracle_homography(const DpePassInput* in, int view, const float plane[4], float H[9]) {
  Pass S;
  kat_pass(S, in);
  const float4_ p = {plane[0], plane[1], plane[2], plane[3]};
  const Homog h = MakeHomography(S, view, p);
  for (int k = 0; k < 9; ++k) H[k] = h.h[k];
}
void oracle_project(const float H[9], float x, float y, float out[2]) {
  Homog h;
  for (int k = 0; k < 9; ++k) h.h[k] = H[k];
  const float2_ r = Project(h, x, y);
  out[0] = r.x; out[1] = r.y;
}
// ComputeBilateralNCCNew of (x, y) with the given pixel states, view masks, deformable neighbours
// (short2 [L][9]) and radius map
float oracle_ncc_new(const DpePassInput* in, const uint8_t* weak, const uint32_t* sel, const int16_t* neighbours,
                     const int32_t* radius, int x, int y, int view, const float plane[4]) {
  Pass S;
  kat_pass(S, in);
  const size_t L = (size_t)S.W * S.H;
  S.weak.assign(weak, weak + L);
  S.sel.assign(sel, sel + L);
  S.neighbours.resize(L * 9);
  std::memcpy(S.neighbours.data(), neighbours, L * 9 * sizeof(short2_));
  S.radius.assign(L, 0);
  if (radius) S.radius.assign(radius, radius + L);
  const float4_ p = {plane[0], plane[1], plane[2], plane[3]};
  return NCCNew(S, x, y, view, p);
}
// ComputeGeomConsistencyCost of (x, y) against the source depth map of `view`
float oracle_geom_cost(const DpePassInput* in, int x, int y, int view, const float plane[4]) {
  Pass S;
  kat_pass(S, in);
  const float4_ p = {plane[0], plane[1], plane[2], plane[3]};
  return GeomCost(S, x, y, view, p);
}
// CheckerboardFilterStrong at (x, y): the resulting depth (.w) of the pixel
float oracle_filter_strong(int W, int H, const float* planes, const uint8_t* weak, const float* costs, int x, int y) {
  Pass S;
  S.W = W; S.H = H;
  const size_t L = (size_t)W * H;
  S.planes.resize(L);
  std::memcpy(S.planes.data(), planes, L * sizeof(float4_));
  S.weak.assign(weak, weak + L);
  S.costs.assign(costs, costs + L);
  FilterStrong(S, x, y);
  return S.planes[(size_t)y * W + x].w;
}
int oracle_d2w_class(const float pc[61], int weak_peak_radius) { return ClassifyCostCurve(pc, weak_peak_radius); }
// GetDepthandNormal of one pixel: out = (world normal, depth)
void oracle_depth_normal(const DpeCamera* cam, const float plane[4], int x, int y, float out[4]) {
  Pass S;
  S.W = x + 1; S.H = y + 1;
  S.cams.assign(cam, cam + 1);
  S.planes.assign((size_t)S.W * S.H, {0, 0, 0, 0});
  S.planes[(size_t)y * S.W + x] = {plane[0], plane[1], plane[2], plane[3]};
  GetDepthandNormal(S, x, y);
  const float4_ r = S.planes[(size_t)y * S.W + x];
  out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = r.w;
}
int oracle_local_refine_select(const float tc[11], const int ok[11], const float p_depth[11], float cost_now, float od,
                               float* out_depth) {
  return LocalRefineSelect(tc, ok, p_depth, cost_now, od, out_depth) ? 1 : 0;
}
// top-k view selection of ComputeMultiViewInitialCostandSelectedViews (DPE.cu:780-826) on the given
// per-view costs (nv = num_images - 1); returns the cost, *sel the view mask
float oracle_topk_views(const float* costs, int nv, int top_k, uint32_t* sel) {
  float cv[32], cvc[32];
  for (int i = 0; i < 32; ++i) { cv[i] = 0.0f; cvc[i] = 0.0f; }
  cv[0] = 2.0f; cvc[0] = 2.0f;
  int num_valid = 0;
  for (int i = 0; i < nv; ++i) { cv[i] = costs[i]; cvc[i] = costs[i]; if (costs[i] < 2.0f) num_valid++; }
  return TopKViews(cv, cvc, nv, num_valid, top_k, nv, sel);
}
// ComputeMultiViewInitialCost (DPE.cu:828-857) on the given per-view costs; *sel in/out
float oracle_initial_cost(const float* costs, int nv, uint32_t* sel) {
  return InitialCostOf(nv + 1, sel, [&](int i) { return costs[i - 1]; });
}
// the joint view selection (DPE.cu:1547-1615) with cost_array [8][32], priors [32] and the 15 draws
// of curand_uniform given; vw [32] out
void oracle_view_select(const float* cost_array, const float* priors, int nv, int iter, const float* draws, uint8_t* vw,
                        uint32_t* tsv, float* wnorm) {
  float ca[8][32];
  std::memcpy(ca, cost_array, sizeof(ca));
  int k = 0;
  ViewSelectionDraws(nv, iter, ca, priors, [&]() { return draws[k++]; }, vw, tsv, wnorm);
}
// RANSACToGetFitPlane (DPE.cu:2891-3124) at (x, y) with the given planes [L][4], pixel states and
// deformable neighbours [L][9] (short2); no edge or label maps (all edges absent, labels 0,
// complexity 0).  out_plane: the fit plane, *out_radius: the radius map entry (strong_radius before).
void oracle_ransac_fit(const DpePassInput* in, const float* planes, const uint8_t* weak, const int16_t* neighbours,
                       int x, int y, int iter, float out_plane[4], int* out_radius) {
  Pass S;
  kat_pass(S, in);
  const size_t L = (size_t)S.W * S.H;
  S.planes.resize(L);
  std::memcpy(S.planes.data(), planes, L * sizeof(float4_));
  S.fit_plane.assign(L, {0, 0, 0, 0});
  S.weak.assign(weak, weak + L);
  S.neighbours.resize(L * 9);
  std::memcpy(S.neighbours.data(), neighbours, L * 9 * sizeof(short2_));
  S.complex_.assign(L, 0.0f);
  S.label.assign(L, 0);
  S.edge_neigh.assign(L * 8, mk_s2(-1, -1));
  S.label_boundary.assign(L * 8, mk_s2(-1, -1));
  S.LW = S.W; S.LH = S.H;
  S.edge.assign(L, 0);
  S.edge_low.assign(L, 0);
  S.radius.assign(L, S.P.strong_radius);
  RANSACFitPlane(S, x, y, iter);
  const float4_ f = S.fit_plane[(size_t)y * S.W + x];
  out_plane[0] = f.x; out_plane[1] = f.y; out_plane[2] = f.z; out_plane[3] = f.w;
  *out_radius = S.radius[(size_t)y * S.W + x];
}
float oracle_expf(float x) { return o_expf(x); }
float oracle_sinf(float x) { return o_sinf(x); }
float oracle_cosf(float x) { return o_cosf(x); }
double oracle_exp_d(double x) { return o_exp_d(x); }
void oracle_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1, uint32_t out[4]) {
  philox_block(c0, c1, c2, c3, k0, k1, out);
}
float oracle_sample(const float* img, int W, int H, float sx, float sy) {
  Pass S; S.W = W; S.H = H;
  std::vector<float> im(img, img + (size_t)W * H);
  return OracleSampleQ(S, im, sx * 256.0f, sy * 256.0f, 1.0f);   // the coordinate itself (iz = 1)
}

// dpe_pass_runner_fn (include/dpe_host.h) over the restatement, so tests can drive the C++ host
// pipeline with the oracle in place of the GPU; `user` points to the thread count (int).
int oracle_pass_runner(void* user, const DpePassInput* in, const DpePassState* st) {
  return oracle_pm_run(in, st, user ? *static_cast<int*>(user) : 1);
}

// ---- RunFusion (DPE.cpp:1220-1370) -----------------------------------------------------------
// Restated as the reference writes it.  fz_* follow Get3DPointonWorld / ProjectCamera
// (DPE.cpp:1170-1206) and GetAngle (:1208-1217) in single precision, expression order kept; the
// reprojection error's pow(float, int) (:1331) promotes to double.
namespace {
struct FzP { float x, y, z; };
FzP fz_world(int x, int y, float depth, const DpeCamera& cam) {
  FzP p, t, C;
  p.x = depth * (x - cam.K[2]) / cam.K[0];
  p.y = depth * (y - cam.K[5]) / cam.K[4];
  p.z = depth;
  t.x = cam.R[0] * p.x + cam.R[3] * p.y + cam.R[6] * p.z;
  t.y = cam.R[1] * p.x + cam.R[4] * p.y + cam.R[7] * p.z;
  t.z = cam.R[2] * p.x + cam.R[5] * p.y + cam.R[8] * p.z;
  C.x = -(cam.R[0] * cam.t[0] + cam.R[3] * cam.t[1] + cam.R[6] * cam.t[2]);
  C.y = -(cam.R[1] * cam.t[0] + cam.R[4] * cam.t[1] + cam.R[7] * cam.t[2]);
  C.z = -(cam.R[2] * cam.t[0] + cam.R[5] * cam.t[1] + cam.R[8] * cam.t[2]);
  return FzP{t.x + C.x, t.y + C.y, t.z + C.z};
}
void fz_project(const FzP& X, const DpeCamera& cam, float& px, float& py, float& depth) {
  const float tx = cam.R[0] * X.x + cam.R[1] * X.y + cam.R[2] * X.z + cam.t[0];
  const float ty = cam.R[3] * X.x + cam.R[4] * X.y + cam.R[5] * X.z + cam.t[1];
  const float tz = cam.R[6] * X.x + cam.R[7] * X.y + cam.R[8] * X.z + cam.t[2];
  depth = cam.K[6] * tx + cam.K[7] * ty + cam.K[8] * tz;
  px = (cam.K[0] * tx + cam.K[1] * ty + cam.K[2] * tz) / depth;
  py = (cam.K[3] * tx + cam.K[4] * ty + cam.K[5] * tz) / depth;
}
// int(v + 0.5f) inside [0, size): on the reference's x86 host an out-of-range / NaN conversion gives
// INT_MIN, i.e. outside; the float test below is that rule without the undefined conversion.
bool fz_pixel(float v, int size, int& out) {
  const float f = v + 0.5f;
  if (!(f > -1.0f && f < (float)size)) return false;
  out = (int)f;
  return true;
}
}  // namespace

// One view as RunFusion sees it (test-infrastructure struct, mirrored in oracle/oracle.py).
typedef struct OracleFusionView {
  int width, height;
  DpeCamera cam;
  const float* depth;      // [H][W]
  const float* normal;     // [H][W][3]
  const uint8_t* weak;     // [H][W] PixelState
  const uint8_t* bgr;      // [H][W][3]
  const uint8_t* block;    // [H][W] or NULL
  int image_id;
  int ns;
  const int* src_ids;      // pair.txt order
} OracleFusionView;

// RunFusion's serial loop (DPE.cpp:1286-1367) over `views` in problem order; writes up to `cap`
// points as (x, y, z, b, g, r) floats into `out` and returns the point count.
int oracle_run_fusion(const OracleFusionView* views, int n, float* out, int cap) {
  std::vector<std::vector<uint8_t>> masks(n);
  for (int i = 0; i < n; ++i) masks[i].assign((size_t)views[i].width * views[i].height, 0);
  auto idx_of = [&](int id) { for (int k = 0; k < n; ++k) if (views[k].image_id == id) return k; return 0; };
  int count = 0;
  for (int i = 0; i < n; ++i) {
    const int ref = idx_of(views[i].image_id);
    const OracleFusionView& R = views[ref];
    const int num_ngb = views[i].ns;
    std::vector<int> ux(num_ngb), uy(num_ngb);
    for (int r = 0; r < R.height; ++r)
      for (int c = 0; c < R.width; ++c) {
        const size_t rc = (size_t)r * R.width + c;
        if (R.block && R.block[rc] < 128) continue;
        if (masks[ref][rc] == 1) continue;
        const float ref_depth = R.depth[rc];
        if (ref_depth <= 0.0) continue;
        const float* rn = R.normal + 3 * rc;
        const FzP X = fz_world(c, r, ref_depth, R.cam);
        int num_consistent = 0;
        float dyn = 0.0f;
        for (int j = 0; j < num_ngb; ++j) {
          ux[j] = uy[j] = -1;
          const int s = idx_of(views[i].src_ids[j]);
          const OracleFusionView& S = views[s];
          float px, py, pd;
          fz_project(X, S.cam, px, py, pd);
          int src_r, src_c;
          if (!fz_pixel(py, S.height, src_r) || !fz_pixel(px, S.width, src_c)) continue;
          const size_t sc = (size_t)src_r * S.width + src_c;
          if (masks[s][sc] == 1) continue;
          const float src_depth = S.depth[sc];
          if (src_depth <= 0.0) continue;
          const FzP Y = fz_world(src_c, src_r, src_depth, S.cam);
          float tx, ty;
          fz_project(Y, R.cam, tx, ty, pd);
          const float dx = c - tx, dy = r - ty;
          // sqrt(pow(c - x, 2) + pow(r - y, 2)) (DPE.cpp:1331): pow(float, int) promotes to double
          const float reproj_error = (float)std::sqrt((double)dx * dx + (double)dy * dy);
          const float rel = std::fabs(pd - ref_depth) / ref_depth;
          const float* sn = S.normal + 3 * sc;
          const float dot = rn[0] * sn[0] + rn[1] * sn[1] + rn[2] * sn[2];
          float angle = std::acos(dot);
          if (angle != angle) angle = 0.0f;
          if (reproj_error < 2.0f && rel < 0.01f && angle < 0.174533f) {
            ux[j] = src_c; uy[j] = src_r;
            const float tmp_index = reproj_error + 200 * rel + angle * 10;
            dyn += std::exp(-tmp_index);
            num_consistent++;
          }
        }
        const float factor = R.weak[rc] == DPE_WEAK ? 0.45f : 0.3f;
        if (num_consistent >= 1 && dyn > factor * num_consistent) {
          float col[3] = {(float)R.bgr[3 * rc], (float)R.bgr[3 * rc + 1], (float)R.bgr[3 * rc + 2]};
          for (int j = 0; j < num_ngb; ++j) {
            if (ux[j] == -1) continue;
            const int s = idx_of(views[i].src_ids[j]);
            const size_t sc = (size_t)uy[j] * views[s].width + ux[j];
            masks[s][sc] = 1;
            col[0] += views[s].bgr[3 * sc]; col[1] += views[s].bgr[3 * sc + 1]; col[2] += views[s].bgr[3 * sc + 2];
          }
          for (float& v : col) v /= (num_consistent + 1);
          if (count < cap && out) {
            float* o = out + 6 * (size_t)count;
            o[0] = X.x; o[1] = X.y; o[2] = X.z; o[3] = col[0]; o[4] = col[1]; o[5] = col[2];
          }
          count++;
        }
      }
  }
  return count;
}

// dpe_fusion_fn (include/dpe_host.h) on the CPU: the per-(pixel, view) tests of RunFusion with the
// contract of dpe_fusion_candidates (include/dpe_mvs.h).  Checker of the HIP kernel.
int oracle_fusion_candidates(void* /*user*/, const DpeFusionView* views, int n, int ref, const int* src, int ns,
                             int32_t* idx, float* val) {
  if (!views || ref < 0 || ref >= n) return DPE_ERR_ARG;
  const DpeFusionView& R = views[ref];
  for (int r = 0; r < R.height; ++r)
    for (int c = 0; c < R.width; ++c) {
      const size_t p = (size_t)r * R.width + c;
      for (int j = 0; j < ns; ++j) {
        idx[p * ns + j] = -1;
        val[(p * ns + j) * 3] = val[(p * ns + j) * 3 + 1] = val[(p * ns + j) * 3 + 2] = 0.0f;
      }
      const float ref_depth = R.depth[p];
      if (!(ref_depth > 0.0f)) continue;
      const FzP X = fz_world(c, r, ref_depth, R.cam);
      const float* rn = R.normal + 3 * p;
      for (int j = 0; j < ns; ++j) {
        const DpeFusionView& S = views[src[j]];
        float px, py, pd;
        fz_project(X, S.cam, px, py, pd);
        int src_r, src_c;
        if (!fz_pixel(px, S.width, src_c) || !fz_pixel(py, S.height, src_r)) continue;
        const size_t sp = (size_t)src_r * S.width + src_c;
        const float sd = S.depth[sp];
        if (!(sd > 0.0f)) continue;
        const FzP Y = fz_world(src_c, src_r, sd, S.cam);
        float tx, ty, pd2;
        fz_project(Y, R.cam, tx, ty, pd2);
        const float dx = c - tx, dy = r - ty;
        const float re = (float)std::sqrt((double)dx * dx + (double)dy * dy);   // DPE.cpp:1331 (double pow)
        const float rl = std::fabs(pd2 - ref_depth) / ref_depth;
        if (re < 2.0f && rl < 0.01f) {
          idx[p * ns + j] = (int32_t)sp;
          const float* sn = S.normal + 3 * sp;
          float* v = val + (p * ns + j) * 3;
          v[0] = re; v[1] = rl; v[2] = rn[0] * sn[0] + rn[1] * sn[1] + rn[2] * sn[2];
        }
      }
    }
  return DPE_OK;
}

}  // extern "C"
