// tap_launch.hip — launches of the strong sweep, DepthToWeak and LocalRefine on the 8-bit /
// quarter-integer texel layouts, their own translation unit; the f32-texel instantiations are in
// tap_f32.hip.
//
// A scheduler is chosen per compilation.  Rounds 2-4 compiled these kernels with LLVM's
// occupancy-first iterative scheduler (-mllvm -amdgpu-sched-strategy=iterative-maxocc): the
// default one then hoisted the unrolled 36-tap loop's gathers past 128 VGPRs and spilled.  Since
// round 5's tap reciprocal (no Newton step) and rolled slow-patch loop the default scheduler fits
// them in 113-124 VGPRs with no scratch, and is faster: strong 26.56 -> 25.99 ms, DepthToWeak
// 21.81 -> 20.94 ms, wall 67.63 -> 65.73 ms (profiles/r05ad_ab_tapsched.log, bit-identical).  The
// f32 instantiations still spill under the default (164-244 B/lane) and keep the iterative
// scheduler in tap_f32.hip.  The weak sweep stays in dpe_mvs.hip with the default.
#define DPE_TAP_TU 1
#include "tap_launch.h"
#include "pass_refine.h"
#include "pass_sweep.h"

namespace dpe {

void launch_strong(bool edge, int cls, unsigned grid, size_t lds, hipStream_t s, const PassConst* dpc,
                   const DevBufs& B, int it, const int* list, const int* count) {
  constexpr int T = 64 * kBwStrong;
  if (lds > 65536) {   // dynamic LDS beyond the default limit (gfx950 has 160 KB per CU)
    static bool once = false;
    if (!once) {
      once = true;
      (void)hipFuncSetAttribute((const void*)k_strong_coop<kTexStrong, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)k_strong_coop<kTexStrong, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    }
  }
  if (cls == IMG_F32) { launch_strong_f32(edge, grid, lds, s, dpc, B, it, list, count); return; }
  if (edge) k_strong_coop<kTexStrong, true><<<grid, T, lds, s>>>(dpc, B, it, list, count);
  else k_strong_coop<kTexStrong, false><<<grid, T, lds, s>>>(dpc, B, it, list, count);
}

void launch_depth_to_weak(int cls, long L, hipStream_t s, const PassConst* dpc, const DevBufs& B) {
  const unsigned g = (unsigned)((L + kBwD2W - 1) / kBwD2W);
  if (cls == IMG_F32) { launch_depth_to_weak_f32(g, s, dpc, B); return; }
  k_depth_to_weak<kTexD2W, true><<<g, 64 * kBwD2W, 0, s>>>(dpc, B);
}

void launch_local_refine(int cls, long L, int W, int H, int nv, hipStream_t s, const PassConst* dpc, const DevBufs& B) {
  // with the fused DepthToWeak only its border pixels are left
  const int border = 1;
  L = border_count(W, H);
  const unsigned g = (unsigned)((L + kBwLR * kLrPix - 1) / (kBwLR * kLrPix));
  if (g == 0) return;
  const size_t lds = (size_t)kBwLR * kLrPix * 12 * nv * 2 * sizeof(float);
  if (lds > 65536) {
    static bool once = false;
    if (!once) {
      once = true;
      (void)hipFuncSetAttribute((const void*)k_local_refine_jobs<kTexLR>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    }
  }
  if (cls == IMG_F32) { launch_local_refine_f32(g, lds, border, s, dpc, B); return; }
  k_local_refine_jobs<kTexLR><<<g, 64 * kBwLR, lds, s>>>(dpc, B, border);
}

}  // namespace dpe

#if DPE_POOL_STATS
extern "C" void dpe_dbg_pool_stats_tap(unsigned long long out[24], int reset) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(dpe::g_pool), sizeof(dpe::g_pool));
  if (reset) { unsigned long long z[24] = {}; (void)hipMemcpyToSymbol(HIP_SYMBOL(dpe::g_pool), z, sizeof(z)); }
}
#endif
#if DPE_LINE_STATS
extern "C" void dpe_dbg_line_stats_tap(unsigned long long out[16], int reset) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(dpe::g_lstat), sizeof(dpe::g_lstat));
  if (reset) { unsigned long long z[16] = {}; (void)hipMemcpyToSymbol(HIP_SYMBOL(dpe::g_lstat), z, sizeof(z)); }
}
#endif
