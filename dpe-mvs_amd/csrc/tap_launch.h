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
namespace dpe {
constexpr int kTexInit = TEX_F16, kTexStrong = TEX_P16, kTexWeak = TEX_U8;
constexpr int kTexD2W = TEX_F16, kTexLR = TEX_F16;

// Launchers (tap_launch.hip).  img8: the 8-bit texel layouts are staged (else the f32 quad image).
// CheckerboardPropagationStrong + refinement, one colour's list (edge: 4 pixels x 16 lanes per wave,
// else 8 x 8); the grid and dynamic LDS are the caller's (strong_lds_per_wave).
void launch_strong(bool edge, bool img8, unsigned grid, size_t lds, hipStream_t s, const PassConst* dpc,
                   const DevBufs& B, int it, const int* list, const int* count);
// DepthToWeak over the L pixels of the pass (one wave per pixel), with LocalRefine fused into its
// epilogue for interior pixels
void launch_depth_to_weak(bool img8, long L, hipStream_t s, const PassConst* dpc, const DevBufs& B);
// LocalRefine (kLrPix pixels per wave), nv source views, over the border pixels the fused
// DepthToWeak leaves
void launch_local_refine(bool img8, long L, int W, int H, int nv, hipStream_t s, const PassConst* dpc, const DevBufs& B);
}  // namespace dpe
