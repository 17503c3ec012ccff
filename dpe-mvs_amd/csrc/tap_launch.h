// tap_launch.h — source-image layout per kernel and the launchers of the tap kernels compiled in
// their own translation units (tap_launch.hip; the f32-texel instantiations in tap_f32.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "pass_common.h"

// source-image layout of each kernel for 8-bit grey-level images (pass_common.h TEX_*): TEX_F16
// issues fewer VALU ops per tap, TEX_U8 touches half the bytes (better for scattered gathers),
// TEX_P16 is in between (half the bytes, 2 more ops per tap than TEX_F16, one unaligned 8-B load).
// A/B on the bench pass (two runs): P16 strong -0.85 / -0.32 ms; DepthToWeak -0.9 / +0.9 (noise),
// LocalRefine +0.2 / -0.2, weak +3 (the 8-B unaligned gathers of its scattered patches cost more)
namespace dpe {
// Grey-level class of a pass's images (dpe_pm_stage): which texel layouts hold them exactly
enum ImgClass { IMG_F32 = 0, IMG_Q = 1, IMG_U8 = 2 };   // any / multiples of 1/4 in [0, 255] / integers
constexpr int kTexInit = TEX_F16, kTexStrong = TEX_P16, kTexWeak = TEX_U8;
constexpr int kTexD2W = TEX_F16, kTexLR = TEX_F16;

// Launchers (tap_launch.hip).  cls: ImgClass of the staged images (IMG_U8 / IMG_Q: the half-precision
// layouts are staged; IMG_F32: the f32 quad image only).
// CheckerboardPropagationStrong + refinement, one colour's list (edge: 4 pixels x 16 lanes per wave,
// else 8 x 8); the grid and dynamic LDS are the caller's (strong_lds_per_wave).
void launch_strong(bool edge, int cls, unsigned grid, size_t lds, hipStream_t s, const PassConst* dpc,
                   const DevBufs& B, int it, const int* list, const int* count);
// DepthToWeak over the L pixels of the pass (one wave per pixel), with LocalRefine fused into its
// epilogue for interior pixels
void launch_depth_to_weak(int cls, long L, hipStream_t s, const PassConst* dpc, const DevBufs& B);
// LocalRefine (kLrPix pixels per wave), nv source views, over the border pixels the fused
// DepthToWeak leaves
void launch_local_refine(int cls, long L, int W, int H, int nv, hipStream_t s, const PassConst* dpc, const DevBufs& B);
// the f32-texel instantiations of the three (tap_f32.hip, occupancy-first scheduler); the grid,
// dynamic LDS and arguments are the launchers' above
void launch_strong_f32(bool edge, unsigned grid, size_t lds, hipStream_t s, const PassConst* dpc, const DevBufs& B,
                       int it, const int* list, const int* count);
void launch_depth_to_weak_f32(unsigned grid, hipStream_t s, const PassConst* dpc, const DevBufs& B);
void launch_local_refine_f32(unsigned grid, size_t lds, int border, hipStream_t s, const PassConst* dpc,
                             const DevBufs& B);
}  // namespace dpe
