// tap_launch.h — source-image layout per kernel and the launchers of the tap kernels compiled in
// their own translation unit (tap_launch.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "pass_common.h"

// source-image layout of each kernel for 8-bit grey-level images (pass_common.h TEX_*): TEX_F16
// issues fewer VALU ops per tap, TEX_U8 touches half the bytes (better for scattered gathers),
// TEX_P16 is in between (half the bytes, 2 more ops per tap than TEX_F16, one unaligned 8-B load).
// A/B on the bench pass (two runs): P16 strong -0.85 / -0.32 ms; DepthToWeak -0.9 / +0.9 (noise),
// LocalRefine +0.2 / -0.2, weak +3 (the 8-B unaligned gathers of its scattered patches cost more)
#ifndef DPE_TEX_STRONG
#define DPE_TEX_STRONG TEX_P16
#endif
#ifndef DPE_TEX_WEAK
#define DPE_TEX_WEAK TEX_U8
#endif
#ifndef DPE_TEX_D2W
#define DPE_TEX_D2W TEX_F16
#endif
#ifndef DPE_TEX_LR
#define DPE_TEX_LR TEX_F16
#endif
#ifndef DPE_TEX_INIT
#define DPE_TEX_INIT TEX_F16
#endif

// Waves per workgroup of the tap kernels.  A workgroup's waves share one CU (and its L1), and its
// waves take consecutive pixels, so a larger workgroup keeps neighbouring pixels' gathers (whose
// patches overlap) in one L1.
#ifndef DPE_BW_STRONG
#define DPE_BW_STRONG 4
#endif
#ifndef DPE_BW_D2W
#define DPE_BW_D2W 4
#endif
#ifndef DPE_BW_LR
#define DPE_BW_LR 4
#endif

namespace dpe {
constexpr int kTexInit = DPE_TEX_INIT, kTexStrong = DPE_TEX_STRONG, kTexWeak = DPE_TEX_WEAK;
constexpr int kTexD2W = DPE_TEX_D2W, kTexLR = DPE_TEX_LR;

// Launchers (tap_launch.hip).  img8: the 8-bit texel layouts are staged (else the f32 quad image).
// CheckerboardPropagationStrong + refinement, one colour's list (edge: 4 pixels x 16 lanes per wave,
// else 8 x 8); the grid and dynamic LDS are the caller's (strong_lds_per_wave).
void launch_strong(bool edge, bool img8, unsigned grid, size_t lds, hipStream_t s, const PassConst* dpc,
                   const DevBufs& B, int it, const int* list, const int* count);
// DepthToWeak over the L pixels of the pass (one wave per pixel), with LocalRefine fused into its
// epilogue for interior pixels when DPE_FUSE_LR (default)
void launch_depth_to_weak(bool img8, long L, hipStream_t s, const PassConst* dpc, const DevBufs& B);
// LocalRefine (kLrPix pixels per wave), nv source views: over the L = W x H pixels, or with the
// fused DepthToWeak (DPE_FUSE_LR) over the border pixels it leaves
void launch_local_refine(bool img8, long L, int W, int H, int nv, hipStream_t s, const PassConst* dpc, const DevBufs& B);
}  // namespace dpe
