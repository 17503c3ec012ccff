// pass_edges.h — the data-parallel stages of EdgeSegment (DPE.cpp:129-291) on the device.
//
// EdgeSegment runs before the first pass of every image (GetProblemEdges, main.cpp:331-388) through
// OpenCV: cv::resize, cv::Canny(L2gradient, aperture 3), Roberts, cv::threshold, Connect and
// cv::HoughLinesP.  The per-pixel stages are restated here with the same integer / float operations
// as the host restatement (host/edges.cpp, host/hostio.cpp), so every output is bit-identical to it:
//   k_resize_linear_h / _v   cv::resize INTER_LINEAR, CV_32F (two separable passes, mul + mul + add)
//   k_resize_u8_h / _v       cv::resize INTER_LINEAR, CV_8U (11-bit fixed point; 16/8-lane vector
//                            formula of VResizeLinear below `xv`, the scalar FixedPtCast above it)
//   k_resize_u8_half         the INTER_AREA fast path cv::resize takes at exactly 1/2
//   k_canny_sobel            Sobel 3x3 (BORDER_REPLICATE, CV_16S) and the squared magnitude with a
//                            zero frame
//   k_canny_nms              non-maximum suppression (13573 / 2^15 tan 22.5 fixed point) into the
//                            candidate map of canny.cpp: 1 not an edge, 0 candidate, 2 strong
//   k_roberts_threshold      Roberts (DPE.cpp:9-25, frame t1 = t2 = 50, (uchar) of the truncated
//                            magnitude) followed by cv::threshold(THRESH_BINARY)
// The order-dependent parts stay on the host: Canny's 8-connected hysteresis walk (over the map the
// device produced), Connect (DPE.cpp:27-127, union-find in scan order), HoughLinesP (random point
// order of cv::RNG).
//
// Strong seeds: canny.cpp marks a strong candidate as a seed only when its left run and the pixel
// above hold no seed (prev_flag / pm[x - mapstep] != 2) and lets the hysteresis reach the others.
// Every strong candidate it skips is 8-connected through candidates to a seed (the run to its left,
// or the seed above), so the hysteresis closure is the same set; here every strong candidate is a
// seed, which needs no scan order.
#pragma once
#include "pass_common.h"

namespace dpe {

__global__ void k_resize_linear_h(const float* __restrict__ src, int w, int h, const int* __restrict__ s0,
                                  const int* __restrict__ s1, const float* __restrict__ a0, const float* __restrict__ a1,
                                  float* __restrict__ rows, int nw) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y * blockDim.y + threadIdx.y;
  if (x >= nw || y >= h) return;
  const float* s = src + (size_t)y * w;
  const float p = s[s0[x]] * a0[x];
  const float q = s[s1[x]] * a1[x];
  rows[(size_t)y * nw + x] = p + q;
}
__global__ void k_resize_linear_v(const float* __restrict__ rows, int nw, const int* __restrict__ s0,
                                  const int* __restrict__ s1, const float* __restrict__ a0, const float* __restrict__ a1,
                                  float* __restrict__ dst, int nh) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y * blockDim.y + threadIdx.y;
  if (x >= nw || y >= nh) return;
  const float p = rows[(size_t)s0[y] * nw + x] * a0[y];
  const float q = rows[(size_t)s1[y] * nw + x] * a1[y];
  dst[(size_t)y * nw + x] = p + q;
}

__global__ void k_resize_u8_half(const uint8_t* __restrict__ src, int w, uint8_t* __restrict__ dst, int nw, int nh) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y * blockDim.y + threadIdx.y;
  if (x >= nw || y >= nh) return;
  const uint8_t* s0 = src + (size_t)(2 * y) * w;
  const uint8_t* s1 = s0 + w;
  dst[(size_t)y * nw + x] = (uint8_t)((s0[2 * x] + s0[2 * x + 1] + s1[2 * x] + s1[2 * x + 1] + 2) >> 2);
}
// HResizeLinear<uchar, int, short, 2048>: taps (ofs, a0, a1); both taps below xmax
__global__ void k_resize_u8_h(const uint8_t* __restrict__ src, int w, int h, const int* __restrict__ ofs,
                              const short* __restrict__ a, int xmax, int* __restrict__ rows, int nw) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y * blockDim.y + threadIdx.y;
  if (x >= nw || y >= h) return;
  const uint8_t* s = src + (size_t)y * w;
  const int sx = ofs[x];
  rows[(size_t)y * nw + x] = x < xmax ? s[sx] * a[2 * x] + s[sx + 1] * a[2 * x + 1] : s[sx] * 2048;
}
DEV uint8_t sat_u8d(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }
DEV int clamp16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }
__global__ void k_resize_u8_v(const int* __restrict__ rows, int h, int nw, const int* __restrict__ ofs,
                              const short* __restrict__ a, int xv, uint8_t* __restrict__ dst, int nh) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y * blockDim.y + threadIdx.y;
  if (x >= nw || y >= nh) return;
  const int sy = ofs[y], sy1 = min(sy + 1, h - 1);
  const int b0 = a[2 * y], b1 = a[2 * y + 1];
  const int S0 = rows[(size_t)sy * nw + x], S1 = rows[(size_t)sy1 * nw + x];
  uint8_t r;
  if (x < xv) {   // VResizeLinearVec_32s8u
    const int p0 = (int)(int16_t)clamp16(S0 >> 4), p1 = (int)(int16_t)clamp16(S1 >> 4);
    const int v = (int)(int16_t)(((p0 * b0) >> 16) + ((p1 * b1) >> 16));
    r = sat_u8d((v + 2) >> 2);
  } else {        // FixedPtCast<int, uchar, 22>
    r = sat_u8d((S0 * b0 + S1 * b1 + (1 << 21)) >> 22);
  }
  dst[(size_t)y * nw + x] = r;
}

// Sobel (BORDER_REPLICATE) and the squared magnitude into a zero-framed (w + 2) x (h + 2) array
__global__ void k_canny_sobel(const uint8_t* __restrict__ src, int w, int h, int16_t* __restrict__ dx,
                              int16_t* __restrict__ dy, int* __restrict__ mag) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x - 1, y = blockIdx.y * blockDim.y + threadIdx.y - 1;
  if (x > w || y > h) return;
  const int ms = w + 2;
  if (x < 0 || y < 0 || x == w || y == h) { mag[(size_t)(y + 1) * ms + x + 1] = 0; return; }
  auto at = [&](int xx, int yy) -> int {
    xx = xx < 0 ? 0 : (xx >= w ? w - 1 : xx);
    yy = yy < 0 ? 0 : (yy >= h ? h - 1 : yy);
    return src[(size_t)yy * w + xx];
  };
  const int gx = (at(x + 1, y - 1) - at(x - 1, y - 1)) + 2 * (at(x + 1, y) - at(x - 1, y)) + (at(x + 1, y + 1) - at(x - 1, y + 1));
  const int gy = (at(x - 1, y + 1) - at(x - 1, y - 1)) + 2 * (at(x, y + 1) - at(x, y - 1)) + (at(x + 1, y + 1) - at(x + 1, y - 1));
  dx[(size_t)y * w + x] = (int16_t)gx;
  dy[(size_t)y * w + x] = (int16_t)gy;
  const int a = (int16_t)gx, b = (int16_t)gy;
  mag[(size_t)(y + 1) * ms + x + 1] = a * a + b * b;
}
// candidate map (w + 2) x (h + 2), frame 1: 1 not an edge, 0 candidate, 2 strong candidate (seed)
__global__ void k_canny_nms(const int16_t* __restrict__ dx, const int16_t* __restrict__ dy, const int* __restrict__ mag,
                            int w, int h, int low, int high, uint8_t* __restrict__ map) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x - 1, y = blockIdx.y * blockDim.y + threadIdx.y - 1;
  if (x > w || y > h) return;
  const int ms = w + 2;
  uint8_t* pm = map + (size_t)(y + 1) * ms + x + 1;
  if (x < 0 || y < 0 || x == w || y == h) { *pm = 1; return; }
  const int* ma = mag + (size_t)(y + 1) * ms + x + 1;
  const int* mp = ma - ms;
  const int* mn = ma + ms;
  const int m = ma[0];
  bool push = false;
  if (m > low) {
    constexpr int CANNY_SHIFT = 15;
    const int TG22 = (int)(0.4142135623730950488016887242097 * (1 << CANNY_SHIFT) + 0.5);
    const int xs = dx[(size_t)y * w + x], ys = dy[(size_t)y * w + x];
    const int ax = abs(xs);
    const int ay = abs(ys) << CANNY_SHIFT;
    const int tg22x = ax * TG22;
    if (ay < tg22x) {
      push = m > ma[-1] && m >= ma[1];
    } else {
      const int tg67x = tg22x + (ax << (CANNY_SHIFT + 1));
      if (ay > tg67x) {
        push = m > mp[0] && m >= mn[0];
      } else {
        const int s = (xs ^ ys) < 0 ? -1 : 1;
        push = m > mp[-s] && m > mn[s];
      }
    }
  }
  *pm = !push ? 1 : (m > high ? 2 : 0);
}

// Roberts (DPE.cpp:9-25) then cv::threshold(thr, 255, THRESH_BINARY)
__global__ void k_roberts_threshold(const uint8_t* __restrict__ src, int w, int h, int thr, uint8_t* __restrict__ dst) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x, i = blockIdx.y * blockDim.y + threadIdx.y;
  if (j >= w || i >= h) return;
  int t1 = 50, t2 = 50;
  if (i > 0 && i < h - 1 && j > 0 && j < w - 1) {
    t1 = src[(size_t)i * w + j] - src[(size_t)(i + 1) * w + j + 1];
    t2 = src[(size_t)(i + 1) * w + j] - src[(size_t)i * w + j + 1];
  }
  // (int)sqrt((double)n) for an integer n < 2^17: the exact integer square root
  const int n = t1 * t1 + t2 * t2;
  int r = (int)__builtin_sqrt((double)n);
  while ((r + 1) * (r + 1) <= n) ++r;
  while (r * r > n) --r;
  const uint8_t v = (uint8_t)r;
  dst[(size_t)i * w + j] = v > thr ? 255 : 0;
}

}  // namespace dpe
