// tap_f32.hip — the strong sweep, DepthToWeak and LocalRefine on f32 quad texels (images whose grey
// levels are not quarter-integers), compiled with LLVM's occupancy-first iterative scheduler
// (-mllvm -amdgpu-sched-strategy=iterative-maxocc, see the Makefile): under the default scheduler
// these instantiations spill 164-244 B/lane, under this one 0-176 (tools/ru.py).  The 8-bit /
// quarter-integer instantiations are in tap_launch.hip with the default scheduler.
#define DPE_TAP_TU 1
#include "tap_launch.h"
#include "pass_refine.h"
#include "pass_sweep.h"

namespace dpe {

void launch_strong_f32(bool edge, unsigned grid, size_t lds, hipStream_t s, const PassConst* dpc, const DevBufs& B,
                       int it, const int* list, const int* count) {
  constexpr int T = 64 * kBwStrong;
  if (lds > 65536) {   // dynamic LDS beyond the default limit (gfx950 has 160 KB per CU)
    static bool once = false;
    if (!once) {
      once = true;
      (void)hipFuncSetAttribute((const void*)k_strong_coop<TEX_F32, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)k_strong_coop<TEX_F32, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    }
  }
  if (edge) k_strong_coop<TEX_F32, true><<<grid, T, lds, s>>>(dpc, B, it, list, count);
  else k_strong_coop<TEX_F32, false><<<grid, T, lds, s>>>(dpc, B, it, list, count);
}

void launch_depth_to_weak_f32(unsigned grid, hipStream_t s, const PassConst* dpc, const DevBufs& B) {
  k_depth_to_weak<TEX_F32, true><<<grid, 64 * kBwD2W, 0, s>>>(dpc, B);
}

void launch_local_refine_f32(unsigned grid, size_t lds, int border, hipStream_t s, const PassConst* dpc,
                             const DevBufs& B) {
  if (lds > 65536) {
    static bool once = false;
    if (!once) {
      once = true;
      (void)hipFuncSetAttribute((const void*)k_local_refine_jobs<TEX_F32>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    }
  }
  k_local_refine_jobs<TEX_F32><<<grid, 64 * kBwLR, lds, s>>>(dpc, B, border);
}

}  // namespace dpe

// this unit's own copies of the DPE_DIAG counters (static __device__ in pass_common.h), summed by
// tools/pool_stats.py and tools/line_stats.py with the other two units'
#if DPE_POOL_STATS
extern "C" void dpe_dbg_pool_stats_f32(unsigned long long out[24], int reset) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(dpe::g_pool), sizeof(dpe::g_pool));
  if (reset) { unsigned long long z[24] = {}; (void)hipMemcpyToSymbol(HIP_SYMBOL(dpe::g_pool), z, sizeof(z)); }
}
#endif
#if DPE_LINE_STATS
extern "C" void dpe_dbg_line_stats_f32(unsigned long long out[16], int reset) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(dpe::g_lstat), sizeof(dpe::g_lstat));
  if (reset) { unsigned long long z[16] = {}; (void)hipMemcpyToSymbol(HIP_SYMBOL(dpe::g_lstat), z, sizeof(z)); }
}
#endif
