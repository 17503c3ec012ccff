// tap_launch.hip — launches of the strong sweep, DepthToWeak and LocalRefine, compiled as their own
// translation unit with LLVM's occupancy-first iterative scheduler
// (-mllvm -amdgpu-sched-strategy=iterative-maxocc, see the Makefile).
//
// A scheduler is chosen per compilation, so the kernels that gain from it live here.  At the
// 4 waves/SIMD of __launch_bounds__(256, kTapWaves) the default scheduler hoists the gathers of
// the unrolled 36-tap loop until it needs more than 128 VGPRs and spills (strong 56, DepthToWeak
// 68, LocalRefine 36 B/lane of scratch, whose stores reach HBM); the iterative scheduler fits the
// same code in 106-110 VGPRs with no scratch.  Interleaved A/B on the bench pass (bit-identical
// outputs): strong -0.4 / -0.6 ms, DepthToWeak -0.6 / -0.6 ms, LocalRefine +0.05 ms.  The weak
// sweep is slower under it (+1.2 ms, more scratch) and stays in dpe_mvs.hip with the default.
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
      (void)hipFuncSetAttribute((const void*)k_strong_coop<TEX_F32, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)k_strong_coop<kTexStrong, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)k_strong_coop<TEX_F32, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    }
  }
  if (edge) {
    if (cls != IMG_F32) k_strong_coop<kTexStrong, true><<<grid, T, lds, s>>>(dpc, B, it, list, count);
    else k_strong_coop<TEX_F32, true><<<grid, T, lds, s>>>(dpc, B, it, list, count);
  } else {
    if (cls != IMG_F32) k_strong_coop<kTexStrong, false><<<grid, T, lds, s>>>(dpc, B, it, list, count);
    else k_strong_coop<TEX_F32, false><<<grid, T, lds, s>>>(dpc, B, it, list, count);
  }
}

void launch_depth_to_weak(int cls, long L, hipStream_t s, const PassConst* dpc, const DevBufs& B) {
  const unsigned g = (unsigned)((L + kBwD2W - 1) / kBwD2W);
  if (cls != IMG_F32) k_depth_to_weak<kTexD2W, true><<<g, 64 * kBwD2W, 0, s>>>(dpc, B);
  else k_depth_to_weak<TEX_F32, true><<<g, 64 * kBwD2W, 0, s>>>(dpc, B);
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
      (void)hipFuncSetAttribute((const void*)k_local_refine_jobs<TEX_F32>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    }
  }
  if (cls != IMG_F32) k_local_refine_jobs<kTexLR><<<g, 64 * kBwLR, lds, s>>>(dpc, B, border);
  else k_local_refine_jobs<TEX_F32><<<g, 64 * kBwLR, lds, s>>>(dpc, B, border);
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
