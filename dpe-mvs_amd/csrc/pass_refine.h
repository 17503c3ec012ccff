// pass_refine.h — wave-cooperative kernels: DepthToWeak, LocalRefine, FindNearestStrongPoint.
//
// DepthToWeak (DPE.cu:2593-2747) evaluates 61 disparity hypotheses per pixel and LocalRefine
// (:2749-2835) 11; the reference loops over them in one thread.  Here one wave owns one pixel
// (DepthToWeak: lane = hypothesis) or five pixels (LocalRefine: 12 lanes per pixel = 11
// hypotheses + the current depth), so the per-pixel state (view mask, weights, baseline) is
// wave-uniform and the 36-tap reference patch is built once per pixel, cooperatively, in LDS.
// Reductions whose floating-point order matters (the peak variance, the arg-min) are done
// serially by one lane in the reference's index order, so results stay bit-exact.
#pragma once
#include "pass_common.h"

namespace dpe {

// wave-local LDS hand-off (all lanes of one wave; no workgroup barrier)
DEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 36-tap reference patch in LDS: (w, w*grey) pairs [36][2], then rp[36] (grey level), pixel (px, py).
// Lane `t` of the group computes taps t, t+stride, ...
// (lane t of S lanes; all of a lane's texel loads are issued before the weights are computed)
template <int S>
DEV void patch_lds_build(float* pw, const PassConst& pc, const DevBufs& B, int px, int py, int t) {
  constexpr int R = (36 + S - 1) / S;
  const float rc = ref_texel(B.ref, pc.W, pc.H, px, py);
  float rp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int k = t + r * S < 36 ? t + r * S : 35;
    rp[r] = ref_texel(B.ref, pc.W, pc.H, px - 5 + 2 * (k / 6), py - 5 + 2 * (k % 6));
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int k = t + r * S;
    if (k >= 36) break;
    const int i = -5 + 2 * (k / 6), j = -5 + 2 * (k % 6);
    const float w = bilateral_weight(i, j, rp[r], rc, pc.P.sigma_spatial, pc.P.sigma_color);
    pw[2 * k] = w;
    pw[2 * k + 1] = w * rp[r];
    pw[72 + k] = rp[r];
  }
}
// reference sums in the row order of make_patch36 (bit-identical), returned as ncc_pre's
// (1/s_w, s_ref/s_w, var_ref), which is what every NCC of the patch needs
DEV void patch_lds_pre(const float* pw, float& p_inv, float& p_mref, float& p_var) {
  float a_ref = 0, a_rr = 0, a_w = 0;
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    float r_ref = 0, r_rr = 0, r_w = 0;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const float w = pw[2 * (a * 6 + b)], wr = pw[2 * (a * 6 + b) + 1], rp = pw[72 + a * 6 + b];
      r_ref = r_ref + wr;
      r_rr = __builtin_fmaf(wr, rp, r_rr);
      r_w = r_w + w;
    }
    a_ref += r_ref; a_rr += r_rr; a_w += r_w;
  }
  ncc_pre(a_ref, a_rr, a_w, p_inv, p_mref, p_var);
}
// The 36 taps of the packed fast path on the texel array `base` (texel (tx, ty) of the view at byte
// base + vofs + (ty * stride + tx) * texel bytes, 32-bit arithmetic).
// Packed form: (r_src, r_rs) accumulate as one pair; weights are (w, w*grey) pairs in LDS; the two
// taps of a row pair share each packed op (tap2_at).
template <int U8, bool CLAMP = true>
DEV void taps36_at(const float* pw, int px, int py, f2v tmax, const uint8_t* base, uint32_t vofs, uint32_t stride,
                   const Homog& H0, float* acc) {
    const Homog H = scale_cols(H0);
    const uint32_t vadj = tex_vadj<U8>(vofs, stride);
    // packed form: (r_src, r_rs) accumulate as one pair; weights are (w, w*grey) pairs in LDS
    const f2v* wp = (const f2v*)pw;
    f2v s_sr = f2s(0.0f);
    float s_ss = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      const float x = (float)(px - 5 + 2 * a);
      const f2v bxy = fma2((f2v){H.h[0], H.h[3]}, f2s(x), (f2v){H.h[2], H.h[5]}) * f2s(kTexUnit);
      const float bz = __builtin_fmaf(H.h[6], x, H.h[8]);
      f2v r_sr = f2s(0.0f);
      float r_ss = 0;
#pragma unroll
      for (int b = 0; b < 6; b += 2) {
        const f2v sp = tap2_at<U8, CLAMP>(base, vadj, stride, tmax, H.h, bxy, bz,
                                   (f2v){(float)(py - 5 + 2 * b), (float)(py - 3 + 2 * b)});
        const f2v w0 = wp[a * 6 + b], w1 = wp[a * 6 + b + 1];
        const float ws0 = w0.x * sp.x, ws1 = w1.x * sp.y;   // two plain multiplies: no operand packing
        r_sr = fma2(w0, f2s(sp.x), r_sr);
        r_ss = __builtin_fmaf(ws0, sp.x, r_ss);
        r_sr = fma2(w1, f2s(sp.y), r_sr);
        r_ss = __builtin_fmaf(ws1, sp.y, r_ss);
      }
      s_sr += r_sr; s_ss += r_ss;
    }
    acc[0] = s_sr.x; acc[1] = s_ss; acc[2] = s_sr.y;
}
// Old NCC with the patch read from LDS (same arithmetic as ncc_old_patch36).  FAST: the caller has
// checked the reciprocal range for the whole patch (rcp_range_ok).  A slow patch (rare: 2316 of
// 1.3e9 on the bench workload, profiles/r05d_pool_stats.log) goes through the rolled generic loop,
// which sums the same weights (bilateral_weight of the same texels) in the same order, so the same
// bits, and keeps an unrolled per-tap-tested loop out of every caller's register budget.
template <int U8, bool FAST, bool CLAMP = true>
DEV void lds_taps(const float* pw, int px, int py, const PassConst& pc, const DevBufs& B, int v, const Homog& H0,
                  float* acc) {
  const int W = pc.W, Hh = pc.H;
  if constexpr (U8 != TEX_F32 && FAST) {
    taps36_at<U8, CLAMP>(pw, px, py, tex_tmax2(W, Hh), tex_base<U8>(B), (uint32_t)v * tex_view<U8>(B),
                         tex_stride<U8>(W), H0, acc);
  } else if constexpr (!FAST) {
    float g[6];
    generic_taps<U8, false>(pc, B, v, H0, px, py, ref_texel(B.ref, W, Hh, px, py), pc.P.strong_radius,
                            pc.P.strong_increment, g);
    acc[0] = g[2]; acc[1] = g[3]; acc[2] = g[4];
  } else {
    const Homog H = scale_cols(H0);
    float s_src = 0, s_ss = 0, s_rs = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      const float x = (float)(px - 5 + 2 * a);
      const float bx = __builtin_fmaf(H.h[0], x, H.h[2]) * kTexUnit;
      const float by = __builtin_fmaf(H.h[3], x, H.h[5]) * kTexUnit;
      const float bz = __builtin_fmaf(H.h[6], x, H.h[8]);
      float r_src = 0, r_ss = 0, r_rs = 0;
#pragma unroll
      for (int b = 0; b < 6; ++b) {
        const float y = (float)(py - 5 + 2 * b);
        const float qx = __builtin_fmaf(H.h[1], y, bx);
        const float qy = __builtin_fmaf(H.h[4], y, by);
        const float iz = rcp_tap<true>(__builtin_fmaf(H.h[7], y, bz));
        const float sp = sample_src<U8>(B, v, W, Hh, qx, qy, iz);
        const float w = pw[2 * (a * 6 + b)], wr = pw[2 * (a * 6 + b) + 1];
        r_src = __builtin_fmaf(w, sp, r_src);
        const float ws = w * sp;
        r_ss = __builtin_fmaf(ws, sp, r_ss);
        r_rs = __builtin_fmaf(wr, sp, r_rs);
      }
      s_src += r_src; s_ss += r_ss; s_rs += r_rs;
    }
    acc[0] = s_src; acc[1] = s_ss; acc[2] = s_rs;
  }
}
// Row a of lds_taps<U8, FAST> with the same operations: (r_src, r_ss, r_rs) of taps (a, 0..5).
// lds_taps adds its six row triplets to zero in row order, so summing these in row order gives
// its result bit for bit; the strong sweep's pool uses this to split the jobs of a nearly empty
// last round over several lanes.
template <int U8, bool FAST>
DEV void lds_row(const float* pw, int px, int py, const PassConst& pc, const DevBufs& B, int v, const Homog& H0, int a,
                 float* r3) {
  const int W = pc.W, Hh = pc.H;
  const Homog H = scale_cols(H0);
  const float x = (float)(px - 5 + 2 * a);
  if constexpr (U8 != TEX_F32 && FAST) {
    const uint32_t stride = tex_stride<U8>(W), vadj = tex_vadj<U8>((uint32_t)v * tex_view<U8>(B), stride);
    const f2v tmax = tex_tmax2(W, Hh);
    const f2v* wp = (const f2v*)pw;
    const f2v bxy = fma2((f2v){H.h[0], H.h[3]}, f2s(x), (f2v){H.h[2], H.h[5]}) * f2s(kTexUnit);
    const float bz = __builtin_fmaf(H.h[6], x, H.h[8]);
    f2v r_sr = f2s(0.0f);
    float r_ss = 0;
#pragma unroll
    for (int b = 0; b < 6; b += 2) {
      const f2v sp = tap2_fast<U8>(B, vadj, stride, tmax, H.h, bxy, bz, (f2v){(float)(py - 5 + 2 * b), (float)(py - 3 + 2 * b)});
      const f2v w0 = wp[a * 6 + b], w1 = wp[a * 6 + b + 1];
      const float ws0 = w0.x * sp.x, ws1 = w1.x * sp.y;
      r_sr = fma2(w0, f2s(sp.x), r_sr);
      r_ss = __builtin_fmaf(ws0, sp.x, r_ss);
      r_sr = fma2(w1, f2s(sp.y), r_sr);
      r_ss = __builtin_fmaf(ws1, sp.y, r_ss);
    }
    r3[0] = r_sr.x; r3[1] = r_ss; r3[2] = r_sr.y;
  } else {
    const float bx = __builtin_fmaf(H.h[0], x, H.h[2]) * kTexUnit;
    const float by = __builtin_fmaf(H.h[3], x, H.h[5]) * kTexUnit;
    const float bz = __builtin_fmaf(H.h[6], x, H.h[8]);
    float r_src = 0, r_ss = 0, r_rs = 0;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const float y = (float)(py - 5 + 2 * b);
      const float qx = __builtin_fmaf(H.h[1], y, bx);
      const float qy = __builtin_fmaf(H.h[4], y, by);
      const float iz = rcp_tap<FAST>(__builtin_fmaf(H.h[7], y, bz));
      const float sp = sample_src<U8>(B, v, W, Hh, qx, qy, iz);
      const float w = pw[2 * (a * 6 + b)], wr = pw[2 * (a * 6 + b) + 1];
      r_src = __builtin_fmaf(w, sp, r_src);
      const float ws = w * sp;
      r_ss = __builtin_fmaf(ws, sp, r_ss);
      r_rs = __builtin_fmaf(wr, sp, r_rs);
    }
    r3[0] = r_src; r3[1] = r_ss; r3[2] = r_rs;
  }
}
template <int U8>
DEV float ncc_old_lds(const float* pw, float s_ref, float s_rr, float s_w, int px, int py, const PassConst& pc,
                      const DevBufs& B, int v, const float4& pl) {
  const Homog H = make_homography(pc, v, pl);
  if (center_outside(pc, v, H, px, py)) { count_work(B, 1, 0); return 2.0f; }
  count_work(B, 1, 36);
  float a[3];
  const bool ok = rcp_range_ok(H, (float)(px - 5), (float)(px + 5), (float)(py - 5), (float)(py + 5));
  PATCH_STAT(ok);
  if (ok) {
    // the clamp-free taps when every active lane's patch is inside the image with a texel to spare
    const bool ncl = taps_unclamped(H, (float)(px - 5), (float)(px + 5), (float)(py - 5), (float)(py + 5), (float)(pc.W - 1),
                                    (float)(pc.H - 1));
#if DPE_POOL_STATS   // tools/pool_stats.py: lanes failing the test, lanes tested, lanes on the clamp-free path
    atomicAdd(&g_pool[6][2], ncl ? 0ull : 1ull);
    atomicAdd(&g_pool[7][0], 1ull);
#endif
    if (DPE_UNCLAMPED && U8 != TEX_F32 && __all(ncl)) {
#if DPE_POOL_STATS
      atomicAdd(&g_pool[7][1], 1ull);
#endif
      lds_taps<U8, true, false>(pw, px, py, pc, B, v, H, a);
    } else
      lds_taps<U8, true>(pw, px, py, pc, B, v, H, a);
  } else
    lds_taps<U8, false>(pw, px, py, pc, B, v, H, a);
  return ncc_finalize_pre(s_ref, s_rr, s_w, a[0], a[1], a[2]);   // (inv, mref, var_ref) of patch_lds_pre
}

template <int U8>
DEV float ncc_old_any(bool fast, const float* pw, float s_ref, float s_rr, float s_w, int px, int py,
                      const PassConst& pc, const DevBufs& B, int v, const float4& pl) {
  if (fast) return ncc_old_lds<U8>(pw, s_ref, s_rr, s_w, px, py, pc, B, v, pl);
  return ncc_old_generic<U8>(pc, B, px, py, v, pl);
}

// Baseline part of DPE.cu:2629-2648 (without the cost, which DepthToWeak never uses).
DEV void baseline_and_weights(const PassConst& pc, uint32_t sel, const uint8_t* vw, float& base_line, float& weight_normal,
                              int& valid) {
  const DpeCamera& c0 = pc.cams[0];
  base_line = 0.0f; weight_normal = 0.0f; valid = 0;
  for (int si = 1; si < pc.N; ++si) {
    const int vi = si - 1;
    if (isSet(sel, vi)) {
      weight_normal += vw[vi];
      const DpeCamera& cs = pc.cams[si];
      const float d0 = c0.c[0] - cs.c[0], d1 = c0.c[1] - cs.c[1], d2 = c0.c[2] - cs.c[2];
      const float tv = d0 * d0 + d1 * d1 + d2 * d2;
      base_line += __builtin_sqrtf(tv);
      valid++;
    }
  }
}

// ------------------------------------------------------------------------------ DepthToWeak
// The classification of DPE.cu:2700-2745 from the 61-sample cost curve `pcs` and its local minima
// `is_peak` (bit i = sample i): the reference's in-order scan over the peaks (non-peaks never update
// it), then the single-peak / peak-variance rules.
DEV uint8_t d2w_class(const PassConst& pc, const float* pcs, uint64_t is_peak) {
  const int radius = 30;
  const int peak_count = __popcll(is_peak);
  int min_peak = 0;
  float min_cost = 2.0f;
  for (uint64_t m = is_peak; m; m &= m - 1) {
    const int i = __builtin_ctzll(m);
    if (pcs[i] < min_cost) { min_peak = i; min_cost = pcs[i]; }
  }
  uint8_t cls;
  if (abs(min_peak - radius) > pc.P.weak_peak_radius || pcs[min_peak] > 0.5f) cls = DPE_WEAK;
  else if (peak_count == 1) cls = pcs[min_peak] <= 0.15f ? DPE_STRONG : DPE_WEAK;
  else {
    float var = 0.0f;
    for (uint64_t m = is_peak; m; m &= m - 1) {
      const int i = __builtin_ctzll(m);
      if (i != min_peak) { const float d = pcs[i] - min_cost; var += d * d; }
    }
    var = __builtin_sqrtf(var);
    var /= (peak_count - 1);
    cls = var > 0.2f ? DPE_STRONG : DPE_WEAK;
  }
  return cls;
}

// grid: one wave per pixel, one wave per workgroup (DepthToWeak: 19.97 against 20.69 ms at 4 waves,
// profiles/r05ao_ab_wgsize2.log); LocalRefine 4 waves per 256-thread workgroup
constexpr int kBwD2W = 1, kBwLR = 4;
// LocalRefine fused into DepthToWeak's epilogue (LR = true).  For an interior pixel LocalRefine's 11
// hypotheses (p_disp -5..5, DPE.cu:2809-2831) are DepthToWeak's samples 25..35 (:2663-2686): same
// plane, depth, selected views and weights, so every per-view NCC and geometric term is the same
// value; only the sums differ (LocalRefine adds ncc*vw and gf*geom*vw as two terms, DepthToWeak
// (ncc + gf*geom)*vw), so lanes 25..35 keep both sums.  Lane 61 evaluates cost_now at the current
// depth (:2776-2795), whose sum is DepthToWeak's.  Both kernels read only their own pixel's plane
// and write only their own pixel (weak_info / plane.w), and the geometric term reads the source
// depth maps, so doing LocalRefine right after the classification of the same pixel gives the
// reference's results.  The 6-pixel border, where DepthToWeak stops at once (:2604-2607) but
// LocalRefine runs, goes to k_local_refine_jobs over the border pixels (border_pixel).
constexpr int kD2WMargin = 6;
// pixels outside DepthToWeak's interior (x or y within kD2WMargin of the edge), enumerated: top rows,
// bottom rows, then the left and right margins of the rows in between (every pixel if no interior)
__host__ __device__ inline long border_count(int W, int H) {
  constexpr int m = kD2WMargin;
  if (W <= 2 * m || H <= 2 * m) return (long)W * H;
  return 2L * m * W + 2L * m * (H - 2 * m);
}
DEV long border_pixel(long i, int W, int H) {
  constexpr int m = kD2WMargin;
  if (W <= 2 * m || H <= 2 * m) return i;
  const long top = (long)m * W;
  if (i < top) return i;
  if (i < 2 * top) return (long)(H - m) * W + (i - top);
  const long r = i - 2 * top;
  const int row = m + (int)(r / (2 * m)), c = (int)(r % (2 * m));
  return (long)row * W + (c < m ? c : W - 2 * m + c);
}
template <int U8, bool LR = false>
__global__ void __launch_bounds__(64 * kBwD2W, kTapWaves) k_depth_to_weak(const PassConst* __restrict__ pcp, DevBufs B) {   // DPE.cu:2593-2747
  __shared__ float s_patch[kBwD2W][108];
  __shared__ float s_pc[kBwD2W][64];              // [0..60] cost curve, [61] LocalRefine's cost_now
  __shared__ float s_lr[kBwD2W][11];              // LocalRefine's hypothesis costs (pd -5..5)
  const PassConst& pc = *pcp;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int W = pc.W, H = pc.H;
  const long pix = (long)xcd_remap(blockIdx.x, gridDim.x, B.xcd_rows * 16 * ((pc.W + kBwD2W - 1) / kBwD2W)) * kBwD2W + wave;
  if (pix >= (long)W * H) return;                 // wave-uniform
  const int x = (int)(pix % W), y = (int)(pix / W);
  const int center = (int)pix;
  const int min_margin = kD2WMargin;
  if (x < min_margin || y < min_margin || x >= W - min_margin || y >= H - min_margin) {
    if (lane == 0) B.weak[center] = DPE_UNKNOWN;
    return;
  }
  const DpeCamera& c0 = pc.cams[0];
  const float4 op = transform_normal_ref(c0, B.planes[center]);
  const float od = op.w;
  if (od == 0) { if (lane == 0) B.weak[center] = DPE_UNKNOWN; return; }
  PHASE_BEGIN();
  const uint32_t sel = B.sel[center];
  const uint8_t* vw = B.vw + (size_t)DPE_MAX_IMAGES * center;
  float base_line, weight_normal; int valid;
  baseline_and_weights(pc, sel, vw, base_line, weight_normal, valid);
  if (valid == 0) { if (lane == 0) B.weak[center] = DPE_UNKNOWN; return; }
  base_line /= valid;
  const float disp = c0.K[0] * base_line / od;
  const bool fast = FAST_PATCH(pc);
  float* pw = s_patch[wave];
  if (fast) patch_lds_build<64>(pw, pc, B, x, y, lane);
  wave_sync();
  float s_ref = 0, s_rr = 0, s_w = 0;
  if (fast) patch_lds_pre(pw, s_ref, s_rr, s_w);
  PHASE(0);
  const int radius = 30;
  constexpr int kNow = 2 * radius + 1;            // lane of LocalRefine's cost_now
  const bool lr_pix = LR && weight_normal != 0;   // LocalRefine skips the pixel otherwise (:2797)
  if (lane < 2 * radius + 1 || (lr_pix && lane == kNow)) {
    const int pd = lane - radius;
    const float p_depth = lane == kNow ? od : c0.K[0] * base_line / (disp + (float)pd);
    float val, lr = 0.0f;
    if (lane != kNow && (p_depth < pc.P.depth_min || p_depth > pc.P.depth_max)) val = 2.0f;
    else {
      float4 tp = op;
      tp.w = dist2origin(c0, x, y, p_depth, tp);
      const float3 fw = pc.P.geom_consistency ? geom_point(pc, x, y, tp) : make_float3(0.0f, 0.0f, 0.0f);
      float p_cost = 0.0f;
      for (int si = 1; si < pc.N; ++si) {
        const int vi = si - 1;
        // a selected view whose weight is 0 adds (ncc + gf*geom) * 0 = +0 (both terms are finite
        // and >= 0), so its NCC is not evaluated (restatement choice 6)
        if (isSet(sel, vi) && vw[vi] != 0) {
          float tcst = 0.0f;
          const float c = ncc_old_any<U8>(fast, pw, s_ref, s_rr, s_w, x, y, pc, B, si, tp);
          tcst += c;
          PHASE(1);
          if constexpr (LR) lr += (c * vw[vi]);                       // DPE.cu:2820
          if (pc.P.geom_consistency) {
            const float g = pc.P.geom_factor * geom_cost_at(pc, B, x, y, si, fw);
            tcst += g;
            if constexpr (LR) lr += (g * vw[vi]);                     // :2822
          }
          PHASE(2);
          p_cost += (tcst * vw[vi]);
        }
      }
      p_cost /= weight_normal;
      val = lane == kNow ? p_cost : MINo(2.0f, p_cost);              // cost_now is not clamped
      lr /= weight_normal;
    }
    s_pc[wave][lane] = val;
    if (LR && lane >= radius - 5 && lane <= radius + 5) s_lr[wave][lane - (radius - 5)] = lr;
  }
  wave_sync();
  PHASE(3);
  // local minima of the cost curve: one lane per sample, then the reference's in-order scan over
  // the (few) peaks only, which is the same scan since non-peaks never update it
  const float* pcs = s_pc[wave];
  const bool pk = lane >= 2 && lane < 59 && pcs[lane - 1] > pcs[lane] && pcs[lane + 1] > pcs[lane];
  const uint64_t is_peak = __ballot(pk);
  PHASE(4);
  PHASE_END(3);
  if (lane != 0) return;
  B.weak[center] = d2w_class(pc, pcs, is_peak);
  if (!lr_pix) return;
  // LocalRefine's choice (DPE.cu:2807-2834): the in-range hypothesis of least cost in pd order
  float min_cost = 2.0f, best_depth = od;
  for (int pd = -5; pd <= 5; ++pd) {
    const float p_depth = c0.K[0] * base_line / (disp + (float)pd);
    if (p_depth < pc.P.depth_min || p_depth > pc.P.depth_max) continue;
    const float tcv = s_lr[wave][pd + 5];
    if (tcv < min_cost) { min_cost = tcv; best_depth = p_depth; }
  }
  if ((double)(pcs[kNow] - min_cost) > 0.1) B.planes[center].w = best_depth;
}

// ------------------------------------------------------------------------------ LocalRefine
// LocalRefine with a flat job pool: a wave owns 4 pixels; every (pixel, hypothesis, selected view)
// NCC is one job, dealt round-robin over the 64 lanes, so lanes stay busy whatever the pixels'
// view counts are.  Per-hypothesis sums over views then run on one lane each, in ascending view
// order (the reference's si loop), and the arg-min on the pixel's first lane.
constexpr int kLrPix = 4;
template <int U8>
__global__ void __launch_bounds__(64 * kBwLR, kTapWaves) k_local_refine_jobs(const PassConst* __restrict__ pcp, DevBufs B,
                                                                                     int border) {   // DPE.cu:2749-2835
  constexpr int BW = kBwLR;
  __shared__ float s_patch[BW][kLrPix][108];
  __shared__ float s_sum[BW][kLrPix][3];
  __shared__ float4 s_hyp[BW][kLrPix][12];
  extern __shared__ float s_dyn[];                // [BW waves][kLrPix][12][nv][2] job results
  __shared__ float s_tc[BW][kLrPix][12];
  __shared__ float3 s_fw[BW][kLrPix][12];         // geometric-consistency world point of each hypothesis
  __shared__ uint8_t s_sel[BW][kLrPix][DPE_MAX_IMAGES];
  __shared__ int s_cnt[BW][kLrPix][2];          // [0] selected views, [1] hypothesis mask (bit 11 = current)
  __shared__ int s_xy[BW][kLrPix];              // pixel x | y << 16 (read by the job pool)
  const PassConst& pc = *pcp;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int W = pc.W;
  // border != 0: only the pixels outside DepthToWeak's interior (border_pixel), whose LocalRefine the
  // fused DepthToWeak does not do; else every pixel
  const long L = border ? border_count(W, pc.H) : (long)W * pc.H;
  const long base = border ? ((long)blockIdx.x * BW + wave) * kLrPix
                           : ((long)xcd_remap(blockIdx.x, gridDim.x, B.xcd_rows * 16 * ((pc.W + BW * kLrPix - 1) / (BW * kLrPix))) * BW + wave) * kLrPix;
  if (base >= L) return;                          // wave-uniform
  const DpeCamera& c0 = pc.cams[0];
  const bool fast = FAST_PATCH(pc);
  const uint32_t vmask = (pc.N - 1) >= 32 ? 0xFFFFFFFFu : ((1u << (pc.N - 1)) - 1u);
  const int nv = pc.N - 1;
  float* res = s_dyn + (size_t)wave * kLrPix * 12 * nv * 2;   // res[((p * 12 + h) * nv + k) * 2 + {0, 1}]
  // ---- per pixel set-up: 16 lanes per pixel
  const int gp = lane >> 4, gl = lane & 15;
  const bool act = base + gp < L;
  const long pix = !act ? 0 : border ? border_pixel(base + gp, W, pc.H) : base + gp;
  const int x = act ? (int)(pix % W) : 0, y = act ? (int)(pix / W) : 0;
  float4 op = make_float4(0, 0, 0, 0);
  float od = 0, base_line = 0, weight_normal = 0;
  int valid = 0;
  uint32_t sel = 0;
  bool go = act;
  if (go) { op = transform_normal_ref(c0, B.planes[pix]); od = op.w; if (od == 0) go = false; }
  const uint8_t* vw = B.vw + (size_t)DPE_MAX_IMAGES * (act ? pix : 0);
  if (go) {
    sel = B.sel[pix];
    baseline_and_weights(pc, sel, vw, base_line, weight_normal, valid);
    if (weight_normal == 0 || valid == 0) go = false;
  }
  float* pw = s_patch[wave][gp];
  if (go && fast) patch_lds_build<16>(pw, pc, B, x, y, gl);
  float disp = 0.0f;
  if (go) { base_line /= valid; disp = c0.K[0] * base_line / od; }
  if (go && gl < 12) {                             // hypothesis gl (11 = the current depth)
    bool ok = true;
    float4 tp = op;
    if (gl < 11) {
      const float p_depth = c0.K[0] * base_line / (disp + (float)(gl - 5));
      ok = !(p_depth < pc.P.depth_min || p_depth > pc.P.depth_max);
      tp.w = dist2origin(c0, x, y, p_depth, tp);
    } else {
      tp.w = dist2origin(c0, x, y, od, tp);
    }
    s_hyp[wave][gp][gl] = tp;
    if (pc.P.geom_consistency) s_fw[wave][gp][gl] = geom_point(pc, x, y, tp);
    const uint64_t m = __ballot(ok) >> (gp * 16);
    if (gl == 0) s_cnt[wave][gp][1] = (int)(m & 0xFFFu);
  }
  if (gl == 0) {
    int ns = 0;
    s_xy[wave][gp] = (int)((uint32_t)x | ((uint32_t)y << 16));
    if (go) for (uint32_t bits = sel & vmask; bits; bits &= bits - 1) s_sel[wave][gp][ns++] = (uint8_t)__builtin_ctz(bits);
    s_cnt[wave][gp][0] = ns;
    if (!go) s_cnt[wave][gp][1] = 0;
  }
  wave_sync();
  if (go && fast && gl == 0) patch_lds_pre(pw, s_sum[wave][gp][0], s_sum[wave][gp][1], s_sum[wave][gp][2]);
  wave_sync();
  // ---- flat job pool: (pixel, valid hypothesis, selected view)
  int total = 0;
#pragma unroll
  for (int p = 0; p < kLrPix; ++p) total += __popc((unsigned)s_cnt[wave][p][1]) * s_cnt[wave][p][0];
  for (int j = lane; j < total; j += 64) {
    int p = 0, r = j;
    for (;;) {
      const int njp = __popc((unsigned)s_cnt[wave][p][1]) * s_cnt[wave][p][0];
      if (r < njp) break;
      r -= njp; ++p;
    }
    const int ns = s_cnt[wave][p][0];
    unsigned m = (unsigned)s_cnt[wave][p][1];
    // view-major: a pixel's hypotheses (depths a disparity step apart, one normal) of one view sit
    // on adjacent lanes, so their taps gather from neighbouring texels
    const int nh = __popc(m);
    for (int q = r % nh; q > 0; --q) m &= m - 1;      // the (r % nh)-th valid hypothesis
    const int h = __builtin_ctz(m), k = r / nh;
    const uint32_t jxy = (uint32_t)s_xy[wave][p];
    const int jx = (int)(jxy & 0xFFFFu), jy = (int)(jxy >> 16);
    const int si = s_sel[wave][p][k] + 1;
    const float4 tp = s_hyp[wave][p][h];
    const float* sm = s_sum[wave][p];
    float* rr = res + ((p * 12 + h) * nv + k) * 2;
    rr[0] = ncc_old_any<U8>(fast, s_patch[wave][p], sm[0], sm[1], sm[2], jx, jy, pc, B, si, tp);
    if (pc.P.geom_consistency) rr[1] = geom_cost_at(pc, B, jx, jy, si, s_fw[wave][p][h]);
  }
  wave_sync();
  // ---- per-hypothesis sums over views in ascending order (DPE.cu:2776-2795, 2805-2818)
  if (go && gl < 12 && ((s_cnt[wave][gp][1] >> gl) & 1)) {
    const int ns = s_cnt[wave][gp][0];
    const bool geom = pc.P.geom_consistency;
    const float gf = pc.P.geom_factor;
    float tc = 0.0f;
    for (int k = 0; k < ns; ++k) {
      const int vi = s_sel[wave][gp][k];
      const float* rr = res + ((gp * 12 + gl) * nv + k) * 2;
      const float c = rr[0];
      if (gl < 11) {
        tc += (c * vw[vi]);
        if (geom) tc += (gf * rr[1] * vw[vi]);
      } else {
        float t = c;
        if (geom) t += gf * rr[1];
        tc += (t * vw[vi]);
      }
    }
    s_tc[wave][gp][gl] = tc / weight_normal;
  }
  wave_sync();
  if (!go || gl != 0) return;
  const float* t = s_tc[wave][gp];
  float min_cost = 2.0f, best_depth = od;
  for (int pd = -5; pd <= 5; ++pd) {
    const float p_depth = c0.K[0] * base_line / (disp + (float)pd);
    if (p_depth < pc.P.depth_min || p_depth > pc.P.depth_max) continue;
    const float tcv = t[pd + 5];
    if (tcv < min_cost) { min_cost = tcv; best_depth = p_depth; }
  }
  if ((double)(t[11] - min_cost) > 0.1) B.planes[pix].w = best_depth;
}

// (non-template kernels: defined only in the translation unit that launches them, dpe_mvs.hip)
#ifndef DPE_TAP_TU
// ------------------------------------------------------------------------------ FindNearestStrongPoint
// Ring search r = 0..100 (DPE.cu:2855-2889) in O(1) per ring with two tables:
//   next_right[y*W + x] = smallest x' >= x with weak(x', y) == STRONG (W if none)
//   next_down [y*W + x] = smallest y' >= y with weak(x, y') == STRONG (H if none)
// Ring order of the reference: column dx = -r (all dy ascending), then columns -r < dx < r
// (dy = -r before dy = +r), then column dx = +r -> first hit = same pixel.
// Both tables as line scans: one wave per row (next_right) or column (next_down), 64 positions per
// step from the far end, the nearest STRONG position at or after each lane by ballot bit arithmetic,
// the nearest one beyond the step carried (same tables as the two one-thread-per-line kernels below).
__global__ void __launch_bounds__(64) k_strong_tables_scan(const PassConst* __restrict__ pcp, DevBufs B,
                                                           int* __restrict__ next_right, int* __restrict__ next_down) {
  const PassConst& pc = *pcp;
  const int W = pc.W, H = pc.H, lane = threadIdx.x;
  const bool row = (int)blockIdx.x < H;
  const int line = row ? (int)blockIdx.x : (int)blockIdx.x - H;
  const int len = row ? W : H;
  int* out = row ? next_right : next_down;
  const unsigned long long from = ~0ull << lane;   // bits lane..63
  int carry = len;
  for (int t0 = ((len - 1) / 64) * 64; t0 >= 0; t0 -= 64) {
    const int t = t0 + lane;
    const int idx = row ? line * W + t : t * W + line;
    const bool st = t < len && B.weak[idx] == DPE_STRONG;
    const unsigned long long m = __ballot(st);
    const unsigned long long ge = m & from;
    if (t < len) out[idx] = ge ? t0 + __builtin_ctzll(ge) : carry;
    if (m) carry = t0 + __builtin_ctzll(m);
  }
}
__global__ void k_find_nearest_strong(const PassConst* __restrict__ pcp, DevBufs B, const int* __restrict__ next_right,
                                      const int* __restrict__ next_down) {
  const PassConst& pc = *pcp;
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y * blockDim.y + threadIdx.y;
  if (x >= pc.W || y >= pc.H) return;
  const int W = pc.W, H = pc.H;
  const int center = x + y * W;
  short2 res = make_short2(-1, -1);
  if (B.weak[center] == DPE_WEAK) {
    for (int r = 1; r <= 100; ++r) {   // r = 0 is the pixel itself, which is WEAK
      const int y0 = MAXo(y - r, 0), y1 = MINo(y + r, H - 1);
      // column dx = -r
      const int xl = x - r;
      if (xl >= 0) {
        const int yy = next_down[y0 * W + xl];
        if (yy <= y1) { res = make_short2((short)xl, (short)yy); break; }
      }
      // columns -r < dx < r on rows y - r and y + r
      const int xa = MAXo(x - r + 1, 0), xb = MINo(x + r - 1, W - 1);
      int best = W, besty = 0;
      if (xa <= xb) {
        if (y - r >= 0) { const int xx = next_right[(y - r) * W + xa]; if (xx <= xb) { best = xx; besty = y - r; } }
        if (y + r < H) { const int xx = next_right[(y + r) * W + xa]; if (xx <= xb && xx < best) { best = xx; besty = y + r; } }
      }
      if (best < W) { res = make_short2((short)best, (short)besty); break; }
      // column dx = +r
      const int xr = x + r;
      if (xr < W) {
        const int yy = next_down[y0 * W + xr];
        if (yy <= y1) { res = make_short2((short)xr, (short)yy); break; }
      }
    }
  }
  B.nearest[center] = res;
}

#endif  // DPE_TAP_TU

}  // namespace dpe
