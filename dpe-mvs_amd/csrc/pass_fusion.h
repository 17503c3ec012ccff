// pass_fusion.h — RunFusion's per-pixel projection tests (DPE.cpp:1303-1343) on the GPU.
//
// RunFusion walks the reference pixels of every image in order, projects each into its source
// views, and keeps a point when enough views agree; a kept point masks the source pixels it used,
// so the walk is order-dependent.  Everything except the masks is independent per (pixel, view):
// the two projections, the reprojection error, the relative depth difference and the normal dot
// product.  This kernel computes exactly that part, one thread per reference pixel, in the
// reference's expression order and precision (-ffp-contract=off, IEEE division and sqrt; single
// precision except the reprojection error, whose pow() promotes to double), and
// the host finishes with the masks, the angle test (acosf), the weights (expf) and the colours in
// the reference's serial order (host/fusion.cpp).
#pragma once
#include "../../include/dpe_mvs.h"

namespace dpe {

struct FusionViewDev {
  const float* depth;
  const float* normal;
  int w, h;
};

struct FP3 { float x, y, z; };

// Get3DPointonWorld (DPE.cpp:1170-1194): camera centre from -R^T t
__device__ inline FP3 fz_world(int x, int y, float depth, const DpeCamera& cam) {
  FP3 p, t, C;
  p.x = depth * ((float)x - cam.K[2]) / cam.K[0];
  p.y = depth * ((float)y - cam.K[5]) / cam.K[4];
  p.z = depth;
  t.x = cam.R[0] * p.x + cam.R[3] * p.y + cam.R[6] * p.z;
  t.y = cam.R[1] * p.x + cam.R[4] * p.y + cam.R[7] * p.z;
  t.z = cam.R[2] * p.x + cam.R[5] * p.y + cam.R[8] * p.z;
  C.x = -(cam.R[0] * cam.t[0] + cam.R[3] * cam.t[1] + cam.R[6] * cam.t[2]);
  C.y = -(cam.R[1] * cam.t[0] + cam.R[4] * cam.t[1] + cam.R[7] * cam.t[2]);
  C.z = -(cam.R[2] * cam.t[0] + cam.R[5] * cam.t[1] + cam.R[8] * cam.t[2]);
  return FP3{t.x + C.x, t.y + C.y, t.z + C.z};
}

// ProjectCamera (DPE.cpp:1196-1206)
__device__ inline void fz_project(const FP3& X, const DpeCamera& cam, float& px, float& py, float& depth) {
  const float tx = cam.R[0] * X.x + cam.R[1] * X.y + cam.R[2] * X.z + cam.t[0];
  const float ty = cam.R[3] * X.x + cam.R[4] * X.y + cam.R[5] * X.z + cam.t[1];
  const float tz = cam.R[6] * X.x + cam.R[7] * X.y + cam.R[8] * X.z + cam.t[2];
  depth = cam.K[6] * tx + cam.K[7] * ty + cam.K[8] * tz;
  px = (cam.K[0] * tx + cam.K[1] * ty + cam.K[2] * tz) / depth;
  py = (cam.K[3] * tx + cam.K[4] * ty + cam.K[5] * tz) / depth;
}

// idx[p*ns + j]: source pixel (row-major) when the projection of reference pixel p lands inside
// source view src[j] on a positive depth with reprojection error < 2 and relative depth difference
// < 0.01, else -1.  val[(p*ns + j)*3 + {0, 1, 2}] = (reprojection error, relative depth difference,
// normal dot product) of those candidates.  `int(v + 0.5f)` of the reference is taken only for
// v + 0.5 in (-1, size): the in-range test on the float, so NaN / huge projections are rejected
// the same way as on the reference's host (where they convert to INT_MIN).
__global__ void __launch_bounds__(256) k_fusion_candidates(const DpeCamera* __restrict__ cams,
                                                          const FusionViewDev* __restrict__ views, int ref,
                                                          const int* __restrict__ src, int ns,
                                                          int32_t* __restrict__ idx, float* __restrict__ val) {
  const FusionViewDev R = views[ref];
  const int L = R.w * R.h;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= L) return;
  const int r = p / R.w, c = p - r * R.w;
  int32_t* oi = idx + (size_t)p * ns;
  float* ov = val + (size_t)p * ns * 3;
  const float ref_depth = R.depth[p];
  if (!(ref_depth > 0.0f)) {
    for (int j = 0; j < ns; ++j) oi[j] = -1;
    return;
  }
  const DpeCamera& rc = cams[ref];
  const FP3 X = fz_world(c, r, ref_depth, rc);
  const float n0 = R.normal[3 * (size_t)p], n1 = R.normal[3 * (size_t)p + 1], n2 = R.normal[3 * (size_t)p + 2];
  for (int j = 0; j < ns; ++j) {
    int32_t o = -1;
    float e = 0.0f, rel = 0.0f, dot = 0.0f;
    const int s = src[j];
    const FusionViewDev S = views[s];
    const DpeCamera& sc = cams[s];
    float px, py, pd;
    fz_project(X, sc, px, py, pd);
    const float fx = px + 0.5f, fy = py + 0.5f;
    if (fx > -1.0f && fx < (float)S.w && fy > -1.0f && fy < (float)S.h) {
      const int src_c = (int)fx, src_r = (int)fy;
      const int sp = src_r * S.w + src_c;
      const float sd = S.depth[sp];
      if (sd > 0.0f) {
        const FP3 Y = fz_world(src_c, src_r, sd, sc);
        float tx, ty, pd2;
        fz_project(Y, rc, tx, ty, pd2);
        const float dx = (float)c - tx, dy = (float)r - ty;
        // DPE.cpp:1331 sqrt(pow(c - x, 2) + pow(r - y, 2)): pow(float, int) promotes to double, so the
        // squares, the sum and the root are double, rounded to float once
        const float re = (float)__builtin_sqrt((double)dx * dx + (double)dy * dy);
        const float rl = __builtin_fabsf(pd2 - ref_depth) / ref_depth;
        if (re < 2.0f && rl < 0.01f) {
          o = sp; e = re; rel = rl;
          const float* sn = S.normal + 3 * (size_t)sp;
          dot = n0 * sn[0] + n1 * sn[1] + n2 * sn[2];
        }
      }
    }
    oi[j] = o;
    ov[3 * j] = e; ov[3 * j + 1] = rel; ov[3 * j + 2] = dot;
  }
}

}  // namespace dpe
