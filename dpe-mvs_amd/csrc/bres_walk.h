// bres_walk.h — the Bresenham walk of GenNeighbours' / RANSACToGetFitPlane's edge test
// (BresenhamLine, DPE.cu:158-244) on the low-resolution edge map, in equivalent forms:
//   walk_bytes  positions in batches of 8, one byte load each, the batch's loads issued together
//               (walk_bytes_flat: the same with plain locals, the device default)
//   walk_tiles  the map as 8x8 bit tiles (one uint64 per tile, bit (y & 7) * 8 + (x & 7)); the walk
//               in chunks that touch at most NT tiles: one pass over the chunk collects its tiles,
//               their words are loaded together, a second pass tests the positions' bits
//   walk_pos    the closed-form position after k steps (the wave-cooperative walk, DPE_GN_COOP)
// All return "some position the walk visits before it stops holds an edge"; the positions do not
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

// tile of the 1-D map index the walk forms (x + y * width, the byte form's indexing and range rule)
// and its bit; -1 outside the map.  A step past the endpoint can leave [0, width) and wrap rows.
BW_HD int tile_of(int x, int y, int width, int height, int tw, int& bit) {
  const int idx = x + y * width;
  if (idx < 0 || idx >= width * height) return -1;
  int xi = x, yi = y;
  if (x < 0 || x >= width) { yi = idx / width; xi = idx - yi * width; }
  bit = (yi & 7) * 8 + (xi & 7);
  return (yi >> 3) * tw + (xi >> 3);
}

BW_HD void build_tile(const uint8_t* map, int width, int height, int t, uint64_t& word) {
  const int tw = (width + 7) >> 3;
  const int x0 = (t % tw) * 8, y0 = (t / tw) * 8;
  uint64_t m = 0;
  for (int yy = 0; yy < 8; ++yy)
    for (int xx = 0; xx < 8; ++xx)
      if (x0 + xx < width && y0 + yy < height && map[(y0 + yy) * width + x0 + xx]) m |= 1ull << (yy * 8 + xx);
  word = m;
}

template <int NT>
BW_HD bool walk_tiles(Walk w, const uint64_t* tiles, int width, int height) {
  const int tw = (width + 7) >> 3;
  while (w.more) {
    int tid[NT];
    int nt = 0, last = -1, n = 0;
    Walk c = w;
    while (n < 64) {                     // pass 1: the chunk's steps and distinct tiles
      Walk nx = c;
      if (!advance(nx)) { c.more = false; break; }
      int bit;
      const int t = tile_of(nx.x0, nx.y0, width, height, tw, bit);
      if (t >= 0 && t != last) {
        if (nt == NT) break;             // this step starts the next chunk
        tid[nt++] = t; last = t;
      }
      c = nx; ++n;
    }
    uint64_t wv[NT];
#pragma unroll
    for (int k = 0; k < NT; ++k) wv[k] = k < nt ? tiles[tid[k]] : 0ull;
    bool hit = false;
    int slot = -1;
    last = -1;
    for (int k = 0; k < n; ++k) {        // pass 2: the same steps, bits tested
      advance(w);
      int bit;
      const int t = tile_of(w.x0, w.y0, width, height, tw, bit);
      if (t >= 0) {
        if (t != last) { ++slot; last = t; }
        uint64_t word = 0;
#pragma unroll
        for (int q = 0; q < NT; ++q) word = q == slot ? wv[q] : word;
        hit |= ((word >> bit) & 1ull) != 0;
      }
    }
    if (hit) return true;
    w = c;
  }
  return false;
}

// Closed form of the walk: the position after k >= 1 steps, and the number of steps the loop runs
// (max(dx, dy) + 1: it stops one step past the endpoint -- the loop tests its tags before moving --
// or at max_step, at least 1).  With dx >= dy every step moves x and the error term stays in
// [0, dx), so y has moved ceil((k dy - dx/2) / dx) times; with dy > dx every step moves y and x has
// moved min(k, floor((dy/2 + dx - 1 + (k - 1) dx) / dy) + 1) times (the min covers the first steps,
// where the error term starts above its steady range; for a vertical line it is the reference's one
// step sideways).  tests/test_bres_walk.py checks it against advance() step by step.
BW_HD int div_floor(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }   // b > 0
BW_HD int div_ceil(int a, int b) { return a >= 0 ? (a + b - 1) / b : -((-a) / b); }   // b > 0
BW_HD int walk_steps(const Walk& w) {
  const int n = (w.dx > w.dy ? w.dx : w.dy) + 1;
  const int m = w.max_step < 1 ? 1 : w.max_step;
  return n < m ? n : m;
}
BW_HD void walk_pos(const Walk& w, int k, int& px, int& py) {
  if (w.dx == 0 && w.dy == 0) { px = w.x0; py = w.y0; return; }
  if (w.dx >= w.dy) {
    const int ys = div_ceil(k * w.dy - w.dx / 2, w.dx);
    px = w.x0 + k * w.sx; py = w.y0 + ys * w.sy;
  } else {
    int xs = div_floor(w.dy / 2 + w.dx - 1 + (k - 1) * w.dx, w.dy) + 1;
    xs = xs < k ? xs : k;
    px = w.x0 + xs * w.sx; py = w.y0 + k * w.sy;
  }
}

}  // namespace bres
}  // namespace dpe
