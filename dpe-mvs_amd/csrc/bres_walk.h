// bres_walk.h — the Bresenham walk of GenNeighbours' / RANSACToGetFitPlane's edge test
// (BresenhamLine, DPE.cu:158-244) on the low-resolution edge map, in equivalent forms:
//   walk_bytes  positions in batches of 8, one byte load each, the batch's loads issued together
//               (walk_bytes_flat: the same with plain locals, the device form)
// (round 4 also measured 8x8 bit tiles of the map and a wave-cooperative closed-form walk; both
// were slower, DESIGN.md §8, and were removed.)  Both return "some position the walk visits before it stops holds an edge"; the positions do not
// depend on the map, so that equals the reference's return at the first edge pixel.
// Pure C++ (no HIP types): tests/test_bres_walk.py compiles it with g++ against a literal
// transcription of the reference loop.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define BW_HD __host__ __device__ __forceinline__
#else
#define BW_HD inline
#endif

namespace dpe {
namespace bres {

// one direction of the walk (from (x0, y0) towards (x1, y1)), the reference's loop state
struct Walk {
  int x0, y0, x1, y1, dx, dy, sx, sy, erro, step, max_step;
  bool tagx, tagy, more;
};

BW_HD Walk start(int x0, int y0, int x1, int y1, int max_step) {
  Walk w;
  w.x0 = x0; w.y0 = y0; w.x1 = x1; w.y1 = y1;
  w.dx = x1 > x0 ? x1 - x0 : x0 - x1; w.sx = x0 < x1 ? 1 : -1;
  w.dy = y1 > y0 ? y1 - y0 : y0 - y1; w.sy = y0 < y1 ? 1 : -1;
  w.erro = (w.dx > w.dy ? w.dx : w.dy) / 2;
  w.step = 0; w.max_step = max_step;
  w.tagx = true; w.tagy = true; w.more = true;
  return w;
}

// one step of the reference loop body: tags from the position before the move, then the move;
// returns false (and clears `more`) when the loop would not run this step
BW_HD bool advance(Walk& w) {
  if (!(w.more && (w.tagx || w.tagy))) { w.more = false; return false; }
  if (w.x0 == w.x1) w.tagx = false;
  if (w.y0 == w.y1) w.tagy = false;
  const int e2 = w.erro;
  if (e2 > -w.dx) { w.erro -= w.dy; w.x0 += w.sx; }
  if (e2 < w.dy) { w.erro += w.dx; w.y0 += w.sy; }
  w.step += 1;
  if (w.step >= w.max_step) w.more = false;
  return true;
}

template <int BATCH>
BW_HD bool walk_bytes(Walk w, const uint8_t* map, int width, int height) {
  const int n = width * height;
  while (w.more) {
    int idx[BATCH];
#pragma unroll
    for (int k = 0; k < BATCH; ++k) idx[k] = advance(w) ? w.x0 + w.y0 * width : -1;
    uint8_t hit = 0;
#pragma unroll
    for (int k = 0; k < BATCH; ++k) hit |= (idx[k] >= 0 && idx[k] < n) ? map[idx[k]] : (uint8_t)0;
    if (hit) return true;
  }
  return false;
}

// walk_bytes with the loop state in plain locals (the device default: the struct form costs
// GenNeighbours 7 VGPRs and its fifth wave per SIMD)
template <int BATCH>
BW_HD bool walk_bytes_flat(int x0, int y0, int x1, int y1, int max_step, const uint8_t* map, int width, int height) {
  const int dx = x1 > x0 ? x1 - x0 : x0 - x1, sx = x0 < x1 ? 1 : -1;
  const int dy = y1 > y0 ? y1 - y0 : y0 - y1, sy = y0 < y1 ? 1 : -1;
  int erro = (dx > dy ? dx : dy) / 2;
  int step = 0;
  bool tagx = true, tagy = true, more = true;
  while (more) {
    int idx[BATCH];
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      idx[k] = -1;
      if (more && (tagx || tagy)) {
        if (x0 == x1) tagx = false;
        if (y0 == y1) tagy = false;
        const int e2 = erro;
        if (e2 > -dx) { erro -= dy; x0 += sx; }
        if (e2 < dy) { erro += dx; y0 += sy; }
        idx[k] = x0 + y0 * width;
        step += 1;
        if (step >= max_step) more = false;
      } else {
        more = false;
      }
    }
    uint8_t hit = 0;
#pragma unroll
    for (int k = 0; k < BATCH; ++k) hit |= (idx[k] >= 0 && idx[k] < width * height) ? map[idx[k]] : (uint8_t)0;
    if (hit) return true;
  }
  return false;
}

}  // namespace bres
}  // namespace dpe
