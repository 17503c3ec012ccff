// pass_kernels.h — the kernels of one PatchMatch pass (DPE::RunPatchMatch, DPE.cu:3126-3249).
//
// Launch structure: full-grid kernels run one thread per pixel on 16x16 workgroups; the red/black
// sweeps run one thread per pixel of the colour on 32x4 workgroups (a wave covers two rows of 64
// columns).  Per-pixel arrays that the reference keeps in registers/local memory
// (cost_array[8][32], DPE.cu:1236/1690; p_costs[61], :2660) are staged in LDS, view-major with the
// thread index fastest, so every access is bank-conflict free.  The 36-tap Old-NCC reference patch
// (weights and weight*grey, view- and plane-independent) is computed once per pixel and kept in
// registers for every NCC the pixel evaluates in that launch.
#pragma once
#include "pass_common.h"

namespace dpe {

#define PIX2D_FULL()                                                   \
  const int lb_ = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y, B.xcd_rows * gridDim.x); \
  const int x = (lb_ % gridDim.x) * blockDim.x + threadIdx.x;          \
  const int y = (lb_ / gridDim.x) * blockDim.y + threadIdx.y;          \
  if (x >= pc.W || y >= pc.H) return;                                  \
  const int center = x + y * pc.W;

// half-sweep pixel of colour `colour` (0 = black: (x+y) even, 1 = red), DPE.cu:1864-1938
#define PIX2D_HALF()                                                   \
  const int lb_ = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y, B.xcd_rows * gridDim.x); \
  const int y = (lb_ / gridDim.x) * blockDim.y + threadIdx.y;          \
  const int x = 2 * ((lb_ % gridDim.x) * blockDim.x + threadIdx.x) + ((y + colour) & 1); \
  if (x >= pc.W || y >= pc.H || y >= pc.half_rows) return;             \
  const int center = x + y * pc.W;

// ------------------------------------------------------------------------------ GenEdgeInform
// The (2r+1)^2 window counts of the edge density come from a byte tile of the block's footprint in
// LDS (bit 0 edge, bit 1 label 0, bit 2 inside the image) for r <= kEiTileR; the counts are
// integers, so the tile changes nothing but the number of global loads (r^2 per pixel -> ~1.6).
constexpr int kEiTileR = 8, kEiTile = 16 + 2 * kEiTileR;
// GenEdgeInform's 8 edge rays (DPE.cu:2497-2530: the first edge pixel along each direction, to the
// image border) as line scans: every pixel lies on one row, one column, one diagonal (x - y const)
// and one anti-diagonal (x + y const); along a line the ray in one direction is the nearest edge
// position after the pixel, in the other the nearest before it.  One wave per line, 64 consecutive
// positions per step: the edge bits of a step by ballot, the nearest set bit above / below each lane
// by bit arithmetic, the nearest edge beyond the step carried from the steps already done (the
// lines are walked once from each end).  Same positions as the per-pixel walks, O(L) loads in all.
__global__ void __launch_bounds__(64) k_edge_rays(const PassConst* __restrict__ pcp, DevBufs B) {
  const PassConst& pc = *pcp;
  const int W = pc.W, H = pc.H;
  const int lane = threadIdx.x;
  int line = blockIdx.x;
  // family f: 0 rows (kDir 2 / 3), 1 columns (0 / 1), 2 diagonals (4 / 5), 3 anti-diagonals (7 / 6);
  // position t along the line, pixel (x0 + t * sx, y0 + t * sy), t in [0, len)
  int f, x0, y0, sx, sy, len, iprev, inext;
  if (line < H) { f = 0; x0 = 0; y0 = line; sx = 1; sy = 0; len = W; iprev = 2; inext = 3; }
  else if ((line -= H) < W) { f = 1; x0 = line; y0 = 0; sx = 0; sy = 1; len = H; iprev = 0; inext = 1; }
  else if ((line -= W) < W + H - 1) {   // x - y = c, c = line - (H - 1), t = y - max(0, -c)
    f = 2; const int c = line - (H - 1);
    y0 = c < 0 ? -c : 0; x0 = c + y0; sx = 1; sy = 1; len = MINo(H - y0, W - x0); iprev = 4; inext = 5;
  } else {                              // x + y = s, t = y - max(0, s - W + 1)
    line -= W + H - 1; f = 3; const int sm = line;
    y0 = sm - (W - 1) > 0 ? sm - (W - 1) : 0; x0 = sm - y0; sx = -1; sy = 1; len = MINo(H - y0, x0 + 1); iprev = 7; inext = 6;
  }
  (void)f;
  const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const unsigned long long above = lane == 63 ? 0ull : (~0ull << (lane + 1));
  // forward: nearest edge before t (direction iprev)
  int carry = -1;
  for (int t0 = 0; t0 < len; t0 += 64) {
    const int t = t0 + lane;
    const int px = x0 + t * sx, py = y0 + t * sy;
    const bool e = t < len && B.edge[py * W + px] != 0;
    const unsigned long long m = __ballot(e);
    const unsigned long long lo = m & below;
    const int prev = lo ? t0 + 63 - __builtin_clzll(lo) : carry;
    if (t < len) {
      B.edge_neigh[(size_t)(py * W + px) * 8 + iprev] =
          prev < 0 ? make_short2(-1, -1) : make_short2((short)(x0 + prev * sx), (short)(y0 + prev * sy));
    }
    if (m) carry = t0 + 63 - __builtin_clzll(m);
  }
  // backward: nearest edge after t (direction inext)
  carry = -1;
  for (int t0 = ((len - 1) / 64) * 64; t0 >= 0; t0 -= 64) {
    const int t = t0 + lane;
    const int px = x0 + t * sx, py = y0 + t * sy;
    const bool e = t < len && B.edge[py * W + px] != 0;
    const unsigned long long m = __ballot(e);
    const unsigned long long hi = m & above;
    const int next = hi ? t0 + __builtin_ctzll(hi) : carry;
    if (t < len) {
      B.edge_neigh[(size_t)(py * W + px) * 8 + inext] =
          next < 0 ? make_short2(-1, -1) : make_short2((short)(x0 + next * sx), (short)(y0 + next * sy));
    }
    if (m) carry = t0 + __builtin_ctzll(m);
  }
}

__global__ void __launch_bounds__(256) k_gen_edge_inform(const PassConst* __restrict__ pcp, DevBufs B) {   // DPE.cu:2483-2591
  const PassConst& pc = *pcp;
  __shared__ uint8_t s_tile[kEiTile * kEiTile];
  __shared__ uint32_t s_hs[kEiTile][16];   // round 6: row sums of the packed flags over 2r + 1 columns
  const int radius = pc.P.strong_radius;
  const bool tiled = pc.P.use_edge && radius >= 0 && radius <= kEiTileR && blockDim.x == 16;
  if (tiled) {   // block-uniform; every thread of the block helps before any returns
    const int lb0 = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y, B.xcd_rows * gridDim.x);
    const int ox = (lb0 % gridDim.x) * blockDim.x - radius, oy = (lb0 / gridDim.x) * blockDim.y - radius;
    const int tw = blockDim.x + 2 * radius, th = blockDim.y + 2 * radius;
    for (int t = threadIdx.y * blockDim.x + threadIdx.x; t < tw * th; t += blockDim.x * blockDim.y) {
      const int nx = ox + t % tw, ny = oy + t / tw;
      uint8_t v = 0;
      if (nx >= 0 && nx < pc.W && ny >= 0 && ny < pc.H) {
        const int q = ny * pc.W + nx;
        v = 4 | (B.edge[q] ? 1 : 0) | ((pc.P.use_label && B.label[q] == 0) ? 2 : 0);
      }
      s_tile[t] = v;
    }
    __syncthreads();
    // the window counts are separable: each (tile row, output column) sums its 2r + 1 flags, packed
    // as edge | label 0 << 10 | inside << 20 (each count <= 17 x 17 < 1024), then a pixel adds 2r + 1
    // row sums -- the same integer counts as the 2-D loop
    for (int t = threadIdx.y * blockDim.x + threadIdx.x; t < th * 16; t += blockDim.x * blockDim.y) {
      const uint8_t* row = s_tile + (t / 16) * tw + t % 16;
      uint32_t acc = 0;
      for (int i = 0; i <= 2 * radius; i++) {
        const uint32_t v = row[i];
        acc += (v & 1u) | ((v & 2u) << 9) | ((v & 4u) << 18);
      }
      s_hs[t / 16][t % 16] = acc;
    }
    __syncthreads();
  }
  PIX2D_FULL();
  const int W = pc.W, H = pc.H;
  if (pc.P.use_edge) {   // the 8 edge rays come from k_edge_rays
    int edge_pix = 0, tot_pix = 0, bound_pix = 0;
    if (tiled) {
      uint32_t acc = 0;
      for (int j = 0; j <= 2 * radius; j++) acc += s_hs[threadIdx.y + j][threadIdx.x];
      edge_pix = (int)(acc & 1023u); bound_pix = (int)((acc >> 10) & 1023u); tot_pix = (int)(acc >> 20);
    } else {
      for (int i = -radius; i <= radius; i++)
        for (int j = -radius; j <= radius; j++) {
          const int nx = x + i, ny = y + j;
          if (nx < 0 || nx >= W || ny < 0 || ny >= H) continue;
          if (B.edge[ny * W + nx]) edge_pix++;
          if (pc.P.use_label && B.label[ny * W + nx] == 0) bound_pix++;
          tot_pix++;
        }
    }
    float density = 1.0f * edge_pix / tot_pix;
    if (pc.P.use_label) density = MAXo(density, (float)(bound_pix / tot_pix));   // integer division (:2551)
    B.complex_[center] = (float)(1.0f / (1.0f + d_exp_d(-25.0 * ((double)density - 0.35))));
  }
  if (pc.P.use_label && B.weak[center] == DPE_WEAK) {
    const int cl = B.label[center];
    if (cl > 0) {
      short2* lb = B.lab_bound + (size_t)center * 8;
      for (int i = 0; i < 8; i++) {
        // last pixel of the own label before the first -1 label (or the border); batches of 8 loads
        const int dx = kDir[i][0], dy = kDir[i][1];
        const int sx = dx > 0 ? W - 1 - x : (dx < 0 ? x : 1 << 30);
        const int sy = dy > 0 ? H - 1 - y : (dy < 0 ? y : 1 << 30);
        const int n = MINo(sx, sy);
        int lk = -1;
        bool stop = false;
        for (int k0 = 1; k0 <= n && !stop; k0 += 8) {
          int lab[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) lab[k] = (k0 + k <= n) ? B.label[(x + (k0 + k) * dx) + (y + (k0 + k) * dy) * W] : -1;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            if (stop) continue;
            if (k0 + k > n) { stop = true; continue; }
            if (lab[k] == cl) lk = k0 + k;
            else if (lab[k] == -1) stop = true;
          }
        }
        lb[i] = lk < 0 ? make_short2(-1, -1) : make_short2((short)(x + lk * dx), (short)(y + lk * dy));
      }
    }
  }
}

// ------------------------------------------------------------------------------ GenNeighbours
// One WEAK pixel of GenNeighbours with per-thread arrays (2.3 KB/lane of scratch): the fallback for
// the pixels k_gen_neighbours_lds defers (more support points than its LDS slots, or a NaN where its
// selections need an order), and for rotate_time > 4.
constexpr int kGnSpec = 4;   // probe attempts drawn and loaded together
DEV void gen_neighbours_px(const PassConst& pc, const DevBufs& B, int center) {   // DPE.cu:2103-2463
  const int W = pc.W, H = pc.H;
  PHASE_BEGIN();
  const int x = center % W, y = center / W;
  const int min_margin = 6;
  const float depth_diff = pc.P.depth_max - pc.P.depth_min;
  const DpeCamera& camera = pc.cams[0];
  Rng rs; rng_init(rs, (uint32_t)center, pc.seed32, STREAM_GEN_NEIGHBOURS, pc.salt);
  short2* nb = B.nb + (size_t)center * 9;
  nb[0] = make_short2((short)x, (short)y);
  for (int i = 1; i < 9; ++i) nb[i] = make_short2(-1, -1);
  short2 strong_points[64];
  uint64_t dir_valid = 0;
  int origin_direction_index = -1, strong_point_size = 0;
  const int rotate_time = pc.P.rotate_time;
  const float cos_angle = pc.gn_cos, sin_angle = pc.gn_sin, threshhold = pc.gn_thr;
  const int shift_range = pc.gn_shift;
  const float ransac_threshold = pc.P.ransac_threshold * depth_diff;
  bool edge_limit = false;
  if (pc.P.use_limit) {
    edge_limit = true;
    if (pc.P.use_edge) {
      const float cv = B.complex_[center];
      const float rp = rng_uniform(rs) - 1.1920929e-07f;
      if (rp < cv) edge_limit = false;
      else B.complex_[center] = MAXo(0.99f, cv);
    }
  }
  for (int odx = -1; odx <= 1; ++odx) {
    for (int ody = -1; ody <= 1; ++ody) {
      if (odx == 0 && ody == 0) continue;
      float2 od = make_float2((float)odx, (float)ody);
      normalize2(od);
      origin_direction_index++;
      for (int rotate_iter = 0; rotate_iter < rotate_time; ++rotate_iter) {
        const int dir_index = origin_direction_index * 4 + rotate_iter;
        for (int radius = 2; radius <= 4096; radius = MINo(radius * 2, radius + 25)) {
          const float tpx = (float)x + od.x * radius, tpy = (float)y + od.y * radius;
          if (tpx < 0 || tpy < 0 || tpx >= W || tpy >= H) break;
          // kGnSpec attempts at a time: their draws, targets and weak[] / nearest[] loads are all
          // issued first, then the attempts are tested in order; the stream is put back to just
          // after the attempt that succeeded, so the draws consumed are the serial loop's.
          bool found = false;
          for (int radius_iter = 0; radius_iter < 4 && !found; radius_iter += kGnSpec) {
            short2 cand[kGnSpec], nnv[kGnSpec];
            uint8_t wkv[kGnSpec];
            bool inm[kGnSpec];
            uint32_t rb[kGnSpec][4], rc[kGnSpec];
            int ri[kGnSpec];
#pragma unroll
            for (int q = 0; q < kGnSpec; ++q) {
              const uint32_t r1 = rng_u32(rs); const uint32_t r2 = rng_u32(rs);
              const int rxs = (int)(((r1 % 2 == 0) ? 1u : 0xFFFFFFFFu) * r2 % (uint32_t)shift_range);
              const uint32_t r3 = rng_u32(rs); const uint32_t r4 = rng_u32(rs);
              const int rys = (int)(((r3 % 2 == 0) ? 1u : 0xFFFFFFFFu) * r4 % (uint32_t)shift_range);
              rb[q][0] = rs.b0; rb[q][1] = rs.b1; rb[q][2] = rs.b2; rb[q][3] = rs.b3; rc[q] = rs.ctr; ri[q] = rs.idx;
              float2 dir = make_float2(od.x * 20 + (float)rxs, od.y * 20 + (float)rys);
              normalize2(dir);
              const short2 np = make_short2((short)f2i((float)x + dir.x * radius), (short)f2i((float)y + dir.y * radius));
              inm[q] = !(np.x < min_margin || np.y < min_margin || np.x >= W - min_margin || np.y >= H - min_margin);
              const int npc = inm[q] ? np.x + np.y * W : center;
              wkv[q] = B.weak[npc];
              nnv[q] = B.nearest[npc];
              cand[q] = np;
            }
#pragma unroll
            for (int q = 0; q < kGnSpec; ++q) {
              if (found || !inm[q]) continue;
              short2 np = cand[q];
              if (wkv[q] != DPE_STRONG) {
                np = nnv[q];
                if (np.x == -1 || np.y == -1) continue;
              }
              float2 td = make_float2((float)(np.x - x), (float)(np.y - y));
              normalize2(td);
              const float ca = td.x * od.x + td.y * od.y;
              if (ca > threshhold && (!edge_limit || !bresenham(pc, B, x, y, np.x, np.y))) {
                strong_points[dir_index] = np;
                dir_valid |= (1ull << dir_index);
                strong_point_size++;
                found = true;
                rs.b0 = rb[q][0]; rs.b1 = rb[q][1]; rs.b2 = rb[q][2]; rs.b3 = rb[q][3]; rs.ctr = rc[q]; rs.idx = ri[q];
              }
            }
          }
          if ((dir_valid >> dir_index) & 1ull) break;
        }
        float2 rd = make_float2(od.x * cos_angle - od.y * sin_angle, od.x * sin_angle + od.y * cos_angle);
        normalize2(rd);
        od = rd;
      }
    }
  }
  PHASE(0);
  int extend_index = 31;
  if (pc.P.use_label && B.label[center] > 0) {
    const short2* lb = B.lab_bound + (size_t)center * 8;
    float bound_dist[8];
    int dir_step[8];
    for (int i = 0; i < 8; ++i) {
      const short2 bp = lb[i];
      float dist = 0.0f;
      if (bp.x != -1 && bp.y != -1) {
        const double dxx = (double)(x - bp.x), dyy = (double)(y - bp.y);
        dist = (float)__builtin_sqrt(dxx * dxx + dyy * dyy);
        if (i >= 4) dist = (float)((double)dist / 1.4142135623730951);
      }
      bound_dist[i] = dist;
      if (i % 2 == 1) { dir_step[i - 1] = 2 * rotate_time - 1; dir_step[i] = 1; }
    }
    for (int i = 0; i < 8; ++i) {
      const float dist = bound_dist[i];
      const int gap_num = dir_step[i] + 1;
      const int step_len = MAXo(1, d2i(__builtin_floor(1.0 * dist / gap_num)));
      for (int step = 1; step <= dir_step[i]; ++step) {
        short2 np = make_short2((short)(x + step * step_len * kDir[i][0]), (short)(y + step * step_len * kDir[i][1]));
        if (np.x < min_margin || np.y < min_margin || np.x >= W - min_margin || np.y >= H - min_margin) continue;
        int npc = np.x + np.y * W;
        if (B.weak[npc] != DPE_STRONG) {
          np = B.nearest[npc];
          if (np.x == -1 || np.y == -1) continue;
          npc = np.x + np.y * W;
        }
        if (B.label[npc] != 0 && B.label[npc] != B.label[center]) continue;
        extend_index++;
        strong_points[extend_index] = np;
        dir_valid |= (1ull << extend_index);
        strong_point_size++;
      }
    }
  }
  PHASE(1);
  if (strong_point_size <= 3) { B.weak_rel[center] = 0; PHASE_END_ALL(2); return; }

  // support points compacted in place (strong_points doubles as spv[]); per point only the depth
  // is kept: its 3-D point and normal are recomputed from (pixel, depth) / planes[] when a, b, c
  // are drawn (same expressions, same bits), which halves the per-thread scratch.
  short2* spv = strong_points;
  float spd[64];
  int valid_count = 0;
  float X[3];
  get3d(camera, x, y, B.planes0[center].w, X);
  const float cpz = X[2];
  for (int i = 0; i < 64; ++i) {
    if ((dir_valid >> i) & 1ull) {
      const short2 sp = strong_points[i];
      spv[valid_count] = sp;
      spd[valid_count] = B.planes0[sp.x + sp.y * W].w;
      valid_count++;
    }
  }
  for (int i = valid_count; i < 64; ++i) spv[i] = make_short2(-1, -1);
  // normalised image coordinates of each support point: loop-invariant in the RANSAC iterations
  // below (same expression, same bits as evaluating it per iteration)
  float2 spf[64];
  for (int i = 0; i < valid_count; ++i)
    spf[i] = make_float2(((float)spv[i].x - camera.K[2]) / camera.K[0], ((float)spv[i].y - camera.K[5]) / camera.K[4]);
  auto point3 = [&](int i) -> float3 {
    float Y[3];
    get3d(camera, spv[i].x, spv[i].y, spd[i], Y);
    return make_float3(Y[0], Y[1], Y[2]);
  };
  auto normal3 = [&](int i) -> float3 {
    const float4 n4 = transform_normal_ref(camera, B.planes0[spv[i].x + spv[i].y * W]);
    return make_float3(n4.x, n4.y, n4.z);
  };
  PHASE(2);
  float4 best_plane = make_float4(0, 0, 0, 0);
  bool has_valid_plane = false;
  {
    int iteration = 50, max_iter = pc.P.high_res_img ? 200 : 125, max_count = 3;
    // residuals[i < valid_count] are written before every read; of the rest only index
    // DPE_NEIGHBOUR_NUM is ever read (as the reference's zero-initialised entry)
    float min_cost = 3.40282347e+38f, residuals[64];
    for (int i = valid_count; i <= DPE_NEIGHBOUR_NUM; ++i) residuals[i] = 0.0f;
    float temp_thr = ransac_threshold;
    // edge_test[64][64] (DPE.cu:2307) as two bit matrices: tested / crosses-an-edge
    // rows are zeroed on first use (row_live), not up front: a thread touches a few of the 64
    uint64_t tested[64], crosses[64], row_live = 0;
    bool has_consist_normal_plane = false;
    bool must_in_triangle = (pc.P.use_label && B.label[center] > 0 && edge_limit) ? false : true;
    auto edge_pair = [&](int a, int b) -> bool {   // returns edge_test[a][b] == 1
      if (!((row_live >> a) & 1ull)) { tested[a] = 0; crosses[a] = 0; row_live |= 1ull << a; }
      if (!((row_live >> b) & 1ull)) { tested[b] = 0; crosses[b] = 0; row_live |= 1ull << b; }
      if (!((tested[a] >> b) & 1ull)) {
        const bool c = bresenham(pc, B, spv[a].x, spv[a].y, spv[b].x, spv[b].y);
        tested[a] |= 1ull << b; tested[b] |= 1ull << a;
        if (c) { crosses[a] |= 1ull << b; crosses[b] |= 1ull << a; }
      }
      return (crosses[a] >> b) & 1ull;
    };
    while (iteration > 0 && max_iter > 0) {
      max_iter--;
      const int a = (int)(rng_u32(rs) % (uint32_t)valid_count);
      const int b = (int)(rng_u32(rs) % (uint32_t)valid_count);
      const int c = (int)(rng_u32(rs) % (uint32_t)valid_count);
      if (a == b || b == c || a == c) continue;
      if (must_in_triangle && !point_in_triangle(spv[a], spv[b], spv[c], x, y)) continue;
      if (edge_limit) {
        const bool eab = edge_pair(a, b);
        const bool ebc = edge_pair(b, c);
        const bool eca = edge_pair(c, a);
        if (eab || ebc || eca) continue;
      }
      bool normal_consistency = false;
      if (pc.P.geom_consistency && edge_limit) {
        const float3 AN = normal3(a), BN = normal3(b), CN = normal3(c);
        normal_consistency = true;
        if ((double)(AN.x * BN.x + AN.y * BN.y + AN.z * BN.z) < 0.8660254 ||
            (double)(AN.x * CN.x + AN.y * CN.y + AN.z * CN.z) < 0.8660254 ||
            (double)(BN.x * CN.x + BN.y * CN.y + BN.z * CN.z) < 0.8660254)
          normal_consistency = false;
        if (has_consist_normal_plane && !normal_consistency) continue;
      }
      iteration--;
      const float3 A = point3(a), Bq = point3(b), C = point3(c);
      const float ACx = A.x - C.x, ACy = A.y - C.y, ACz = A.z - C.z;
      const float BCx = Bq.x - C.x, BCy = Bq.y - C.y, BCz = Bq.z - C.z;
      float4 cv;
      cv.x = ACy * BCz - BCy * ACz;
      cv.y = -(ACx * BCz - BCx * ACz);
      cv.z = ACx * BCy - BCx * ACy;
      if ((cv.x == 0 && cv.y == 0 && cv.z == 0) || cv.x != cv.x || cv.y != cv.y || cv.z != cv.z) continue;
      normalize3(cv);
      cv.w = -(cv.x * A.x + cv.y * A.y + cv.z * A.z);
      // residual of support point si under cv (stored only when a new best plane needs the sort)
      auto resid = [&](int si) -> float {
        const float2 f = spf[si];
        const float fd = -cv.w / (cv.x * f.x + cv.y * f.y + cv.z);
        return __builtin_fabsf(fd - spd[si]);
      };
      int temp_count = 0;
      for (int si = 0; si < valid_count; ++si)
        if (resid(si) < temp_thr) temp_count++;
      if (temp_count < 6) continue;
      if (temp_count > max_count) {
        if (!must_in_triangle && point_in_triangle(spv[a], spv[b], spv[c], x, y)) must_in_triangle = true;
        if (!has_consist_normal_plane && normal_consistency) has_consist_normal_plane = true;
        const float fx = ((float)x - camera.K[2]) / camera.K[0];
        const float fy = ((float)y - camera.K[5]) / camera.K[4];
        const float fd = -cv.w / (cv.x * fx + cv.y * fy + cv.z);
        const float cd = __builtin_fabsf(fd - cpz);
        best_plane = cv; max_count = temp_count; min_cost = cd; has_valid_plane = true;
        if ((double)temp_thr > (pc.P.high_res_img ? 0.05 : 0.005)) {
          for (int si = 0; si < valid_count; ++si) residuals[si] = resid(si);
          // sort_small(residuals, valid_count) (DPE.cu:5-14)
          for (int i = 1; i < valid_count; i++) {
            const float tmp = residuals[i];
            int j = i;
            for (; j >= 1 && tmp < residuals[j - 1]; j--) residuals[j] = residuals[j - 1];
            residuals[j] = tmp;
          }
          if (temp_thr < residuals[DPE_NEIGHBOUR_NUM]) continue;
          temp_thr = (float)((double)residuals[DPE_NEIGHBOUR_NUM] - 1e-6);
          temp_count = 0;
          for (int i = 0; i < valid_count; ++i) {
            if (residuals[i] < temp_thr) temp_count++;
            else break;
          }
          max_count = temp_count;
        }
      } else if (temp_count == max_count) {
        if (!must_in_triangle && point_in_triangle(spv[a], spv[b], spv[c], x, y)) must_in_triangle = true;
        const float fx = ((float)x - camera.K[2]) / camera.K[0];
        const float fy = ((float)y - camera.K[5]) / camera.K[4];
        const float fd = -cv.w / (cv.x * fx + cv.y * fy + cv.z);
        const float cd = __builtin_fabsf(fd - cpz);
        if (cd < min_cost) { best_plane = cv; max_count = temp_count; min_cost = cd; }
      }
    }
  }
  PHASE(3);
  if (!has_valid_plane) { B.weak_rel[center] = 0; PHASE_END_ALL(2); return; }
  float* weight = spd;          // in place: weight[i] is written after spd[i] is read
  for (int i = 0; i < valid_count; ++i) {
    const float fx = spf[i].x, fy = spf[i].y;
    const float fd = -best_plane.w / (best_plane.x * fx + best_plane.y * fy + best_plane.z);
    const float dist = __builtin_fabsf(fd - spd[i]);
    if (dist >= ransac_threshold) { spv[i] = make_short2(-1, -1); weight[i] = 3.40282347e+38f; continue; }
    weight[i] = dist;
  }
  // sort_small_weighted (DPE.cu:16-29)
  for (int i = 1; i < valid_count; i++) {
    const short2 tp = spv[i]; const float tw = weight[i];
    int j = i;
    for (; j >= 1 && tw < weight[j - 1]; j--) { spv[j] = spv[j - 1]; weight[j] = weight[j - 1]; }
    spv[j] = tp; weight[j] = tw;
  }
  for (int i = 1; i < DPE_NEIGHBOUR_NUM; ++i) nb[i] = spv[i - 1];
  B.weak_rel[center] = 1;
  PHASE(4);
  PHASE_END_ALL(2);
}
// over `list`: a small persistent grid (kGnOvfBlocks x 256 threads) striding through the list, so
// that the usual empty overflow list costs one short launch (the round-4 full-grid launch took the
// aux stream for 0.7 ms)
constexpr int kGnOvfBlocks = 64;
__global__ void __launch_bounds__(256) k_gen_neighbours(const PassConst* __restrict__ pcp, DevBufs B,
                                                        const int* __restrict__ list, const int* __restrict__ nlist_p) {
  const PassConst& pc = *pcp;
  const int n = *nlist_p;
  for (int gi = blockIdx.x * blockDim.x + threadIdx.x; gi < n; gi += gridDim.x * blockDim.x)
    gen_neighbours_px(pc, B, list[gi]);
}

// ------------------------------------------------------------------------------ GenNeighbours, scratch-free
// The same GenNeighbours with no per-thread arrays (k_gen_neighbours keeps 2.3 KB/lane of them in
// scratch, re-read from HBM on every RANSAC try).  The support points are appended in probe order,
// which is the order of the reference's compaction of strong_points[] (dir_index grows through the
// probe loops, the label extension follows at 32+; rotate_time <= 4), so they go straight into an
// LDS column per thread: the packed pixel, K slots ([slot][thread], conflict-free; K = 16 x
// rotate_time rounded up to 32 / 64 holds the most a pixel can collect: 8 KB / 16 KB per 64-thread
// workgroup).  A point's depth is re-read from planes0[] and its normalised image
// coordinates come from per-column / per-row tables (`gtab`, the same expression per coordinate), so
// nothing else is stored.  The edge tests are recomputed instead of cached (BresenhamLine is a pure
// function of its end points; the reference's edge_test[][] only saves work), the probe batches
// re-position the Philox stream by its word index instead of saving its state, and the two sorts
// become order-statistic selections whose results equal the insertion sorts' whenever no residual
// or weight is NaN.  A pixel with more than K support points, or a NaN where a sort needs the
// order, writes nothing and is appended to `ovf` for k_gen_neighbours (its Philox stream is
// addressed by the pixel, so the rerun draws the same numbers).  96 VGPRs, 5 waves per SIMD.
constexpr int kGnBT = 64;   // threads per workgroup
// table of the normalised image coordinates: gtab[x] = (x - K[2]) / K[0], gtab[W + y] = (y - K[5]) / K[4]
__global__ void k_gn_tables(const PassConst* __restrict__ pcp, float* __restrict__ gtab) {
  const PassConst& pc = *pcp;
  const DpeCamera& camera = pc.cams[0];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < pc.W) gtab[i] = ((float)i - camera.K[2]) / camera.K[0];
  else if (i < pc.W + pc.H) gtab[i] = ((float)(i - pc.W) - camera.K[5]) / camera.K[4];
}
// the angle test of a probe, td = normalize(np - p), td . od > thr (DPE.cu:2196-2199)
DEV bool gn_angle_ok(float dxf, float dyf, float2 od, float thr) {
  float2 td = make_float2(dxf, dyf);
  normalize2(td);
  return td.x * od.x + td.y * od.y > thr;
}
// Per-pixel durations of the scratch-free GenNeighbours (DPE_DIAG & 8; tools/gn_times.py): shader
// clocks from the start to the end of the probes and to the pixel's end, at the pixel's list index
// (one wave = 64 consecutive indices).  Off in the product.
#if DPE_GN_TIMES
// + per-pixel counts: [0] radius steps of the direction walks, [1] Bresenham walks of the probes,
// [2] RANSAC tries, [3] Bresenham walks of the RANSAC, [4] / [5] shader clocks in the probes' / the
// RANSAC's Bresenham walks
static __device__ uint32_t g_gntime[2 << 20];
static __device__ uint32_t g_gncnt[6 << 20];
#define GN_T0() const uint64_t gn_t0_ = __builtin_readcyclecounter(); uint32_t gn_c_[6] = {0, 0, 0, 0, 0, 0}
#define GN_T(k) do { if (gi < (1 << 20)) { g_gntime[2 * gi + (k)] = (uint32_t)(__builtin_readcyclecounter() - gn_t0_); \
                       if ((k) == 1) for (int q_ = 0; q_ < 6; ++q_) g_gncnt[6 * gi + q_] = gn_c_[q_]; } } while (0)
#define GN_C(k, n) (gn_c_[k] += (n))
#define GN_CLK() __builtin_readcyclecounter()
#else
#define GN_T0() do {} while (0)
#define GN_T(k) do {} while (0)
#define GN_C(k, n) do {} while (0)
#define GN_CLK() 0ull
#endif
// The probe's walk pair runs from the pixel: BresenhamLine(A, B) is "an edge on the walk B -> A or
// on the walk A -> B", whichever is walked first; with the pixel as B the first walk starts at the
// pixel, where the edge that blocks a direction usually is, and stops there (round 4).
template <int K>
__global__ void __launch_bounds__(kGnBT) k_gen_neighbours_lds(const PassConst* __restrict__ pcp, DevBufs B,
                                                              const int* __restrict__ list, const int* __restrict__ nlist_p,
                                                              const float* __restrict__ gtab, int* __restrict__ ovf,
                                                              int* __restrict__ novf) {   // DPE.cu:2103-2463
  __shared__ uint32_t s_pt[K][kGnBT];           // support point (x | y << 16)
  const PassConst& pc = *pcp;
  const int t = threadIdx.x;
  const int gi = xcd_remap(blockIdx.x, gridDim.x, B.xcd_rows * 64) * kGnBT + t;
  if (gi >= *nlist_p) return;
  const int W = pc.W, H = pc.H;
  const int center = list[gi];
  const int x = center % W, y = center / W;
  const int min_margin = 6;
  const float depth_diff = pc.P.depth_max - pc.P.depth_min;
  const DpeCamera& camera = pc.cams[0];
  Rng rs; rng_init(rs, (uint32_t)center, pc.seed32, STREAM_GEN_NEIGHBOURS, pc.salt);
  PHASE_BEGIN();
  GN_T0();
  int valid_count = 0;
  bool overflow = false;
  auto push = [&](short2 np) {
    if (valid_count < K) s_pt[valid_count][t] = (uint32_t)(uint16_t)np.x | ((uint32_t)(uint16_t)np.y << 16);
    else overflow = true;
    valid_count++;
  };
  auto pt_at = [&](int i) -> short2 {
    const uint32_t v = s_pt[i][t];
    return make_short2((short)(v & 0xFFFFu), (short)(v >> 16));
  };
  const int rotate_time = pc.P.rotate_time;
  const float cos_angle = pc.gn_cos, sin_angle = pc.gn_sin, threshhold = pc.gn_thr;
  const int shift_range = pc.gn_shift;
  const float ransac_threshold = pc.P.ransac_threshold * depth_diff;
  auto crosses = [&](int ax, int ay, int bx, int by) -> bool { return bresenham(pc, B, ax, ay, bx, by); };
  bool edge_limit = false;
  float complex_new = -1.0f;                       // complex_[center] to write once the pixel is done
  if (pc.P.use_limit) {
    edge_limit = true;
    if (pc.P.use_edge) {
      const float cv = B.complex_[center];
      const float rp = rng_uniform(rs) - 1.1920929e-07f;
      if (rp < cv) edge_limit = false;
      else complex_new = MAXo(0.99f, cv);
    }
  }
  // The 8 x rotate_time direction walks as ONE loop per lane: a lane that ends a walk (support point
  // found, radius past the image or 4096) moves on to its next direction at once, so a wave's time
  // is its slowest lane's total walk, not the sum over directions of each direction's slowest walk.
  // Each lane's sequence of probes (and of Philox draws) is the nested loops' sequence.  One radius
  // of a walk is kGnSpec attempts at a time: their draws, targets and weak[] / nearest[] loads
  // issued first, then tested in order; the stream is then positioned just after the attempt that
  // succeeded (each attempt draws 4 words; the stream is position-addressable).
  {
    auto origin_od = [](int oi) -> float2 {   // odx -1..1 outer, ody -1..1 inner, (0, 0) skipped
      const int k = oi < 4 ? oi : oi + 1;
      float2 od = make_float2((float)(k / 3 - 1), (float)(k % 3 - 1));
      normalize2(od);
      return od;
    };
    int oi = 0, ri = 0, radius = 2;
    float2 od = origin_od(0);
    while (oi < 8) {
      bool next = radius > 4096;
      GN_C(0, 1);
      if (!next) {
        const float tpx = (float)x + od.x * radius, tpy = (float)y + od.y * radius;
        if (tpx < 0 || tpy < 0 || tpx >= W || tpy >= H) next = true;
      }
      if (!next) {
        bool dir_found = false;
        for (int ra = 0; ra < 4 && !dir_found; ra += kGnSpec) {
          short2 cand[kGnSpec], nnv[kGnSpec];
          uint8_t wkv[kGnSpec];
          bool inm[kGnSpec];
          const uint32_t pos0 = rs.idx == 4 ? rs.ctr * 4u : (rs.ctr - 1u) * 4u + (uint32_t)rs.idx;
#pragma unroll
          for (int q = 0; q < kGnSpec; ++q) {
            const uint32_t r1 = rng_u32(rs); const uint32_t r2 = rng_u32(rs);
            const uint32_t r3 = rng_u32(rs); const uint32_t r4 = rng_u32(rs);
            const int rxs = (int)(((r1 % 2 == 0) ? 1u : 0xFFFFFFFFu) * r2 % (uint32_t)shift_range);
            const int rys = (int)(((r3 % 2 == 0) ? 1u : 0xFFFFFFFFu) * r4 % (uint32_t)shift_range);
            float2 dir = make_float2(od.x * 20 + (float)rxs, od.y * 20 + (float)rys);
            normalize2(dir);
            const short2 np = make_short2((short)f2i((float)x + dir.x * radius), (short)f2i((float)y + dir.y * radius));
            inm[q] = !(np.x < min_margin || np.y < min_margin || np.x >= W - min_margin || np.y >= H - min_margin);
            const int npc = inm[q] ? np.x + np.y * W : center;
            wkv[q] = B.weak[npc];
            nnv[q] = B.nearest[npc];
            cand[q] = np;
          }
#pragma unroll
          for (int q = 0; q < kGnSpec; ++q) {
            if (dir_found || !inm[q]) continue;
            short2 np = cand[q];
            if (wkv[q] != DPE_STRONG) {
              np = nnv[q];
              if (np.x == -1 || np.y == -1) continue;
            }
            const bool ang = gn_angle_ok((float)(np.x - x), (float)(np.y - y), od, threshhold);
            if (ang && edge_limit) GN_C(1, 1);
            const uint64_t gn_b0_ = GN_CLK(); (void)gn_b0_;
            const bool pass_ = ang && (!edge_limit || !crosses(np.x, np.y, x, y));
            GN_C(4, (uint32_t)(GN_CLK() - gn_b0_));
            if (pass_) {
              push(np);
              dir_found = true;
              rng_seek(rs, pos0 + 4u * (uint32_t)(q + 1));
            }
          }
        }
        if (dir_found) next = true;
        else radius = MINo(radius * 2, radius + 25);
      }
      if (next) {
        radius = 2;
        if (++ri < rotate_time) {
          float2 rd = make_float2(od.x * cos_angle - od.y * sin_angle, od.x * sin_angle + od.y * cos_angle);
          normalize2(rd);
          od = rd;
        } else {
          ri = 0;
          if (++oi < 8) od = origin_od(oi);
        }
      }
    }
  }
  PHASE(0);
  if (pc.P.use_label && B.label[center] > 0) {
    const short2* lb = B.lab_bound + (size_t)center * 8;
    for (int i = 0; i < 8; ++i) {
      const short2 bp = lb[i];
      float dist = 0.0f;
      if (bp.x != -1 && bp.y != -1) {
        const double dxx = (double)(x - bp.x), dyy = (double)(y - bp.y);
        dist = (float)__builtin_sqrt(dxx * dxx + dyy * dyy);
        if (i >= 4) dist = (float)((double)dist / 1.4142135623730951);
      }
      const int nstep = (i % 2 == 0) ? 2 * rotate_time - 1 : 1;   // dir_step (DPE.cu:2236-2247)
      const int step_len = MAXo(1, d2i(__builtin_floor(1.0 * dist / (nstep + 1))));
      for (int step = 1; step <= nstep; ++step) {
        short2 np = make_short2((short)(x + step * step_len * kDir[i][0]), (short)(y + step * step_len * kDir[i][1]));
        if (np.x < min_margin || np.y < min_margin || np.x >= W - min_margin || np.y >= H - min_margin) continue;
        int npc = np.x + np.y * W;
        if (B.weak[npc] != DPE_STRONG) {
          np = B.nearest[npc];
          if (np.x == -1 || np.y == -1) continue;
          npc = np.x + np.y * W;
        }
        if (B.label[npc] != 0 && B.label[npc] != B.label[center]) continue;
        push(np);
      }
    }
  }
  PHASE(1);
  GN_T(0);
  auto defer = [&]() { ovf[atomicAdd(novf, 1)] = center; PHASE_END_ALL(2); GN_T(1); };
  auto finish_fail = [&]() {
    GN_T(1);
    if (complex_new >= 0.0f) B.complex_[center] = complex_new;
    short2* nb = B.nb + (size_t)center * 9;
    nb[0] = make_short2((short)x, (short)y);
    for (int i = 1; i < 9; ++i) nb[i] = make_short2(-1, -1);
    B.weak_rel[center] = 0;
    PHASE_END_ALL(2);
  };
  if (overflow) { defer(); return; }
  if (valid_count <= 3) { finish_fail(); return; }
  // depths of the support points (the reference's spv3[].z); the 3-D points and normals of the
  // drawn triples are recomputed from (pixel, depth) / planes0[] with the reference's expressions
  auto depth_at = [&](int i) -> float { const uint32_t v = s_pt[i][t]; return B.planes0[(v & 0xFFFFu) + (v >> 16) * W].w; };
  float X[3];
  get3d(camera, x, y, B.planes0[center].w, X);
  const float cpz = X[2];
  auto resid_of = [&](const float4& pl, int si) -> float {
    const uint32_t v = s_pt[si][t];
    const float fx = gtab[v & 0xFFFFu], fy = gtab[W + (v >> 16)];
    const float fd = -pl.w / (pl.x * fx + pl.y * fy + pl.z);
    return __builtin_fabsf(fd - depth_at(si));
  };
  PHASE(2);
  float4 best_plane = make_float4(0, 0, 0, 0);
  bool has_valid_plane = false, nan_sort = false;
  {
    int iteration = 50, max_iter = pc.P.high_res_img ? 200 : 125, max_count = 3;
    float min_cost = 3.40282347e+38f;
    float temp_thr = ransac_threshold;
    bool has_consist_normal_plane = false;
    bool must_in_triangle = (pc.P.use_label && B.label[center] > 0 && edge_limit) ? false : true;
    while (iteration > 0 && max_iter > 0) {
      max_iter--;
      GN_C(2, 1);
      const int a = (int)(rng_u32(rs) % (uint32_t)valid_count);
      const int b = (int)(rng_u32(rs) % (uint32_t)valid_count);
      const int c = (int)(rng_u32(rs) % (uint32_t)valid_count);
      if (a == b || b == c || a == c) continue;
      const short2 pa = pt_at(a), pb = pt_at(b), pcc = pt_at(c);
      if (must_in_triangle && !point_in_triangle(pa, pb, pcc, x, y)) continue;
      if (edge_limit) {
        bool eab, ebc, eca;
        const uint64_t gn_b1_ = GN_CLK(); (void)gn_b1_;
        eab = crosses(pa.x, pa.y, pb.x, pb.y);
        ebc = crosses(pb.x, pb.y, pcc.x, pcc.y);
        eca = crosses(pcc.x, pcc.y, pa.x, pa.y);
        GN_C(3, 3);
        GN_C(5, (uint32_t)(GN_CLK() - gn_b1_));
        if (eab || ebc || eca) continue;
      }
      bool normal_consistency = false;
      if (pc.P.geom_consistency && edge_limit) {
        const float4 a4 = transform_normal_ref(camera, B.planes0[pa.x + pa.y * W]);
        const float4 b4 = transform_normal_ref(camera, B.planes0[pb.x + pb.y * W]);
        const float4 c4 = transform_normal_ref(camera, B.planes0[pcc.x + pcc.y * W]);
        normal_consistency = true;
        if ((double)(a4.x * b4.x + a4.y * b4.y + a4.z * b4.z) < 0.8660254 ||
            (double)(a4.x * c4.x + a4.y * c4.y + a4.z * c4.z) < 0.8660254 ||
            (double)(b4.x * c4.x + b4.y * c4.y + b4.z * c4.z) < 0.8660254)
          normal_consistency = false;
        if (has_consist_normal_plane && !normal_consistency) continue;
      }
      iteration--;
      float A[3], Bq[3], C[3];
      get3d(camera, pa.x, pa.y, depth_at(a), A);
      get3d(camera, pb.x, pb.y, depth_at(b), Bq);
      get3d(camera, pcc.x, pcc.y, depth_at(c), C);
      const float ACx = A[0] - C[0], ACy = A[1] - C[1], ACz = A[2] - C[2];
      const float BCx = Bq[0] - C[0], BCy = Bq[1] - C[1], BCz = Bq[2] - C[2];
      float4 cv;
      cv.x = ACy * BCz - BCy * ACz;
      cv.y = -(ACx * BCz - BCx * ACz);
      cv.z = ACx * BCy - BCx * ACy;
      if ((cv.x == 0 && cv.y == 0 && cv.z == 0) || cv.x != cv.x || cv.y != cv.y || cv.z != cv.z) continue;
      normalize3(cv);
      cv.w = -(cv.x * A[0] + cv.y * A[1] + cv.z * A[2]);
      int temp_count = 0;
      for (int si = 0; si < valid_count; ++si)
        if (resid_of(cv, si) < temp_thr) temp_count++;
      if (temp_count < 6) continue;
      if (temp_count > max_count) {
        if (!must_in_triangle && point_in_triangle(pa, pb, pcc, x, y)) must_in_triangle = true;
        if (!has_consist_normal_plane && normal_consistency) has_consist_normal_plane = true;
        const float fx = ((float)x - camera.K[2]) / camera.K[0];
        const float fy = ((float)y - camera.K[5]) / camera.K[4];
        const float fd = -cv.w / (cv.x * fx + cv.y * fy + cv.z);
        const float cd = __builtin_fabsf(fd - cpz);
        best_plane = cv; max_count = temp_count; min_cost = cd; has_valid_plane = true;
        if ((double)temp_thr > (pc.P.high_res_img ? 0.05 : 0.005)) {
          // sort_small(residuals, valid_count) then residuals[DPE_NEIGHBOUR_NUM] (DPE.cu:5-14,
          // 2367-2376): the 10th smallest residual (0 when there are at most 9: the untouched entry);
          // the count that follows is the number of residuals below the new threshold, all of them
          // among those 10 smallest
          float top[DPE_NEIGHBOUR_NUM + 1];
#pragma unroll
          for (int k = 0; k <= DPE_NEIGHBOUR_NUM; ++k) top[k] = __builtin_inff();
          bool has_nan = false;
          for (int si = 0; si < valid_count; ++si) {
            float r = resid_of(cv, si);
            has_nan |= r != r;
#pragma unroll
            for (int k = 0; k <= DPE_NEIGHBOUR_NUM; ++k) {   // sorted insertion, static indices
              const float lo = __builtin_fminf(top[k], r), hi = __builtin_fmaxf(top[k], r);
              top[k] = lo; r = hi;
            }
          }
          if (has_nan) { nan_sort = true; break; }
          const float kth = valid_count > DPE_NEIGHBOUR_NUM ? top[DPE_NEIGHBOUR_NUM] : 0.0f;
          if (temp_thr < kth) continue;
          temp_thr = (float)((double)kth - 1e-6);
          temp_count = 0;
#pragma unroll
          for (int k = 0; k <= DPE_NEIGHBOUR_NUM; ++k)
            if (k < valid_count && top[k] < temp_thr) temp_count++;
          max_count = temp_count;
        }
      } else if (temp_count == max_count) {
        if (!must_in_triangle && point_in_triangle(pa, pb, pcc, x, y)) must_in_triangle = true;
        const float fx = ((float)x - camera.K[2]) / camera.K[0];
        const float fy = ((float)y - camera.K[5]) / camera.K[4];
        const float fd = -cv.w / (cv.x * fx + cv.y * fy + cv.z);
        const float cd = __builtin_fabsf(fd - cpz);
        if (cd < min_cost) { best_plane = cv; max_count = temp_count; min_cost = cd; }
      }
    }
  }
  PHASE(3);
  if (nan_sort) { defer(); return; }
  if (!has_valid_plane) { finish_fail(); return; }
  // weights (DPE.cu:2437-2449) in place of the depths, then sort_small_weighted (:16-29) and the
  // first 8 points: the insertion sort is stable, so with no NaN weight the k-th output is the k-th
  // smallest (weight, index) -- outliers carry FLT_MAX and the point (-1, -1)
  bool wnan = false;
  for (int i = 0; i < valid_count; ++i) { const float dist = resid_of(best_plane, i); wnan |= dist != dist; }
  auto weight_at = [&](int i) -> float {
    const float dist = resid_of(best_plane, i);
    return dist >= ransac_threshold ? 3.40282347e+38f : dist;
  };
  if (wnan) { defer(); return; }
  short2 out[DPE_NEIGHBOUR_NUM - 1];
  uint64_t taken = 0;
#pragma unroll
  for (int k = 0; k < DPE_NEIGHBOUR_NUM - 1; ++k) {
    int bi = -1; float bw = 0.0f;
    for (int i = 0; i < valid_count; ++i) {
      if ((taken >> i) & 1ull) continue;
      const float w = weight_at(i);
      if (bi < 0 || w < bw) { bi = i; bw = w; }
    }
    if (bi >= 0) { taken |= 1ull << bi; out[k] = bw >= ransac_threshold ? make_short2(-1, -1) : pt_at(bi); }
    else out[k] = make_short2(-1, -1);
  }
  if (complex_new >= 0.0f) B.complex_[center] = complex_new;
  short2* nb = B.nb + (size_t)center * 9;
  nb[0] = make_short2((short)x, (short)y);
#pragma unroll
  for (int k = 0; k < DPE_NEIGHBOUR_NUM - 1; ++k) nb[k + 1] = out[k];
  B.weak_rel[center] = 1;
  PHASE(4);
  PHASE_END_ALL(2);
  GN_T(1);
}

// ------------------------------------------------------------------------------ NeigbourUpdate
__global__ void k_neighbour_update(const PassConst* __restrict__ pcp, DevBufs B) {   // DPE.cu:2465-2481
  const PassConst& pc = *pcp;
  PIX2D_FULL();
  if (B.weak[center] != DPE_WEAK) return;
  if (B.weak_rel[center] != 1) B.weak[center] = DPE_UNKNOWN;
}

// ------------------------------------------------------------------------------ RandomInitialization
template <int U8>
__global__ void __launch_bounds__(256) k_random_init(const PassConst* __restrict__ pcp, DevBufs B) {   // DPE.cu:1035-1063
  const PassConst& pc = *pcp;
  PIX2D_FULL();
  const DpeCamera& c0 = pc.cams[0];
  const int N = pc.N;
  const bool fast = FAST_PATCH(pc);
  Patch36 P;
  if (fast) make_patch36(P, pc, B, x, y); else { P.px = x; P.py = y; }
  if (pc.P.state == DPE_FIRST_INIT) {
    Rng rs; rng_init(rs, (uint32_t)center, pc.seed32, STREAM_RANDOM_INIT, pc.salt);
    const float depth = rng_uniform(rs) * (pc.P.depth_max - pc.P.depth_min) + pc.P.depth_min;
    float4 ph = random_normal(c0, x, y, rs, depth);
    ph.w = dist2origin(c0, x, y, depth, ph);
    B.planes[center] = ph;
    // ComputeMultiViewInitialCostandSelectedViews (DPE.cu:780-826): sorted copy kept in registers
    float sorted[DPE_MAX_IMAGES];
    int cost_count = 0, num_valid = 0;
    for (int i = 1; i < N; ++i) {
      const float c = ncc_old<U8>(P, fast, pc, B, i, ph);
      // insertion into the sorted prefix == sort_small of the full vector afterwards
      int j = cost_count;
      for (; j >= 1 && c < sorted[j - 1]; j--) sorted[j] = sorted[j - 1];
      sorted[j] = c;
      cost_count++;
      if (c < 2.0f) num_valid++;
    }
    uint32_t sel = 0;
    const int top_k = MINo(num_valid, pc.P.top_k);
    float cost = 2.0f;
    if (top_k > 0) {
      float s = 0.0f;
      for (int i = 0; i < top_k; ++i) s += sorted[i];
      const float thr = sorted[top_k - 1];
      // second pass recomputes the (deterministic) per-view costs instead of keeping a copy
      for (int i = 1; i < N; ++i) if (ncc_old<U8>(P, fast, pc, B, i, ph) <= thr) setBit(sel, i - 1);
      cost = s / top_k;
    }
    B.sel[center] = sel;
    B.costs[center] = cost;
  } else {
    float4 ph = transform_normal_ref(c0, B.planes[center]);
    const float depth = ph.w;
    ph.w = dist2origin(c0, x, y, depth, ph);
    B.planes[center] = ph;
    // ComputeMultiViewInitialCost (DPE.cu:828-857)
    uint32_t sel = B.sel[center];
    int cc = 0; float cost = 0.0f;
    for (int i = 1; i < N; ++i) {
      if (isSet(sel, i - 1)) {
        const float c = ncc_old<U8>(P, fast, pc, B, i, ph);
        if (c < 2.0f) { cc++; cost += c; }
        else unSetBit(sel, i - 1);
      }
    }
    B.sel[center] = sel;
    B.costs[center] = cc == 0 ? 2.0f : cost / cc;
  }
}

// ------------------------------------------------------------------------------ RANSACToGetFitPlane
constexpr int kRansacThreads = 128;   // 1-D workgroups: 16 KB of LDS each
// One thread per entry of a weak list (the sweep's list of one colour), instead of the reference's
// full-grid launch with ~80 % of the threads returning at once.  Only the colour's own weak update
// reads a fit plane or radius, so the rows past the red/black grid (half_rows) need none.
__global__ void __launch_bounds__(kRansacThreads) k_ransac_fit(const PassConst* __restrict__ pcp, DevBufs B, int iter,
                                                               const int* __restrict__ list, const int* __restrict__ nlist_p) {   // DPE.cu:2891-3124
  const PassConst& pc = *pcp;
  const int gi = xcd_remap(blockIdx.x, gridDim.x, B.xcd_rows * 16) * kRansacThreads + (int)threadIdx.x;
  if (gi >= *nlist_p) return;
  const int center = list[gi];
  const int x = center % pc.W, y = center / pc.W;
  const int W = pc.W;
  if (B.weak[center] != DPE_WEAK) return;
  Rng rs; rng_init(rs, (uint32_t)center, pc.seed32, STREAM_ITER_BASE + 4 * iter + 1, pc.salt);
  const DpeCamera& camera = pc.cams[0];
  bool edge_limit = false;
  if (pc.P.use_limit) {
    edge_limit = true;
    if (pc.P.use_edge) {
      const float cv = B.complex_[center];
      const float rp = rng_uniform(rs) - 1.1920929e-07f;
      if (rp < cv) edge_limit = false;
    }
  }
  // support points in LDS (thread index fastest): the random draws index them, which a register
  // array cannot do without scratch memory.  Their normals are re-read from the planes when a try
  // needs them (nothing writes a plane during the fits): 128 B of LDS per thread instead of 224, so
  // 5 waves per SIMD instead of 3 and both colours' fits resident at once
  __shared__ short2 s_sp[8][kRansacThreads];
  __shared__ float3 s_sp3[8][kRansacThreads];
  const int tid = threadIdx.x;
  struct Col2 { short2* p; DEV short2& operator[](int i) const { return p[i * kRansacThreads]; } } sp{&s_sp[0][tid]};
  struct Col3 { float3* p; DEV float3& operator[](int i) const { return p[i * kRansacThreads]; } } sp3{&s_sp3[0][tid]};
  auto spn = [&](int i) -> float3 {
    const float4 pl = B.planes[sp[i].x + sp[i].y * W];
    return make_float3(pl.x, pl.y, pl.z);
  };
  int sc = 0;
  float X[3];
  const short2* nb = B.nb + (size_t)center * 9;
  for (int i = 1; i < DPE_NEIGHBOUR_NUM; ++i) {
    const short2 tp = nb[i];
    if (tp.x == -1 || tp.y == -1) continue;
    sp[sc] = tp;
    const float4 pl = B.planes[tp.x + tp.y * W];
    const float depth = depth_from_plane(camera, pl, tp.x, tp.y);
    get3d(camera, tp.x, tp.y, depth, X);
    sp3[sc] = make_float3(X[0], X[1], X[2]);
    sc++;
  }
  if (sc < 3) { B.fit_plane[center] = B.planes[center]; return; }
  int iteration = 50;
  int ua = -1, ub = -1, uc = -1;
  float min_cost = 3.40282347e+38f;
  float4 best = make_float4(0, 0, 0, 0);
  bool has_best = false, has_strong_plane = false;
  bool must_in_triangle = (pc.P.use_label && B.label[center] > 0 && edge_limit) ? false : true;
  // edge_test[8][8] (DPE.cu:2960) as two 64-bit matrices, bit a * 8 + b
  uint64_t tested = 0, crosses = 0;
  auto edge_pair = [&](int a, int b) -> bool {
    if (!((tested >> (a * 8 + b)) & 1ull)) {
      const bool c = bresenham(pc, B, sp[a].x, sp[a].y, sp[b].x, sp[b].y);
      tested |= (1ull << (a * 8 + b)) | (1ull << (b * 8 + a));
      if (c) crosses |= (1ull << (a * 8 + b)) | (1ull << (b * 8 + a));
    }
    return (crosses >> (a * 8 + b)) & 1ull;
  };
  while (iteration--) {
    const int a = (int)(rng_u32(rs) % (uint32_t)sc);
    const int b = (int)(rng_u32(rs) % (uint32_t)sc);
    const int c = (int)(rng_u32(rs) % (uint32_t)sc);
    if (a == b || b == c || a == c) continue;
    bool is_strong_plane = false;
    if (pc.P.geom_consistency && edge_limit) {
      const float3 AN = spn(a), BN = spn(b), CN = spn(c);
      is_strong_plane = true;
      if ((double)(AN.x * BN.x + AN.y * BN.y + AN.z * BN.z) < 0.8660254 ||
          (double)(AN.x * CN.x + AN.y * CN.y + AN.z * CN.z) < 0.8660254 ||
          (double)(BN.x * CN.x + BN.y * CN.y + BN.z * CN.z) < 0.8660254)
        is_strong_plane = false;
      if (has_strong_plane && !is_strong_plane) continue;
    }
    if (must_in_triangle && !point_in_triangle(sp[a], sp[b], sp[c], x, y)) continue;
    if (edge_limit) {
      const bool eab = edge_pair(a, b);
      const bool ebc = edge_pair(b, c);
      const bool eca = edge_pair(c, a);
      if (eab || ebc || eca) continue;
    }
    const float3 A = sp3[a], Bq = sp3[b], C = sp3[c];
    const float ACx = A.x - C.x, ACy = A.y - C.y, ACz = A.z - C.z;
    const float BCx = Bq.x - C.x, BCy = Bq.y - C.y, BCz = Bq.z - C.z;
    float4 cv;
    cv.x = ACy * BCz - BCy * ACz;
    cv.y = -(ACx * BCz - BCx * ACz);
    cv.z = ACx * BCy - BCx * ACy;
    if ((cv.x == 0 && cv.y == 0 && cv.z == 0) || cv.x != cv.x || cv.y != cv.y || cv.z != cv.z) continue;
    normalize3(cv);
    cv.w = -(cv.x * A.x + cv.y * A.y + cv.z * A.z);
    if (!has_strong_plane && is_strong_plane) has_strong_plane = true;
    float tcost = 0.0f;
    for (int si = 0; si < sc; ++si) {
      if (si == a || si == b || si == c) continue;
      const float fx = ((float)sp[si].x - camera.K[2]) / camera.K[0];
      const float fy = ((float)sp[si].y - camera.K[5]) / camera.K[4];
      const float fd = -cv.w / (cv.x * fx + cv.y * fy + cv.z);
      tcost += __builtin_fabsf(fd - sp3[si].z);
    }
    if (tcost < min_cost) {
      if (!must_in_triangle && point_in_triangle(sp[a], sp[b], sp[c], x, y)) must_in_triangle = true;
      min_cost = tcost; best = cv; has_best = true; ua = a; ub = b; uc = c;
    }
  }
  if (has_best) {
    const float depth = depth_from_plane(camera, B.planes[center], x, y);
    const float4 vd = view_direction(camera, x, y, depth);
    if (best.x * vd.x + best.y * vd.y + best.z * vd.z > 0) { best.x = -best.x; best.y = -best.y; best.z = -best.z; best.w = -best.w; }
    B.fit_plane[center] = best;
    if (pc.P.use_radius) {
      if (must_in_triangle) {
        const short2 A = sp[ua], Bq = sp[ub], C = sp[uc];
        const float a = __builtin_sqrtf((float)((A.x - Bq.x) * (A.x - Bq.x) + (A.y - Bq.y) * (A.y - Bq.y)));
        const float b = __builtin_sqrtf((float)((Bq.x - C.x) * (Bq.x - C.x) + (Bq.y - C.y) * (Bq.y - C.y)));
        const float c = __builtin_sqrtf((float)((C.x - A.x) * (C.x - A.x) + (C.y - A.y) * (C.y - A.y)));
        const float p = (float)((double)(a + b + c) / 2.0);
        const float Sarea = __builtin_sqrtf(p * (p - a) * (p - b) * (p - c));
        int radius = d2i(__builtin_floor((double)__builtin_sqrtf(Sarea) / 2.0));
        const float Ad = __builtin_sqrtf((float)((A.x - x) * (A.x - x) + (A.y - y) * (A.y - y)));
        const float Bd = __builtin_sqrtf((float)((Bq.x - x) * (Bq.x - x) + (Bq.y - y) * (Bq.y - y)));
        const float Cd = __builtin_sqrtf((float)((C.x - x) * (C.x - x) + (C.y - y) * (C.y - y)));
        const float min_dis = MINo(MINo(Ad, Bd), Cd);
        if (2.5 * (double)min_dis < (double)radius) radius = f2i(min_dis);
        if (edge_limit) {
          if (pc.P.use_edge) {
            float med = 3.40282347e+38f;
            const short2* en = B.edge_neigh + (size_t)center * 8;
            for (int d = 0; d < 8; ++d) {
              const short2 ep = en[d];
              if (ep.x == -1 || ep.y == -1) continue;
              const float dist = __builtin_sqrtf((float)((ep.x - x) * (ep.x - x) + (ep.y - y) * (ep.y - y)));
              med = MINo(med, dist);
            }
            if (med < (float)radius) radius = f2i(med);
          }
          if (pc.P.use_label && B.label[center] > 0) {
            float mbd = 3.40282347e+38f;
            const short2* lb = B.lab_bound + (size_t)center * 8;
            for (int d = 0; d < 8; ++d) {
              const short2 bp = lb[d];
              if (bp.x == -1 || bp.y == -1) continue;
              const double dxx = (double)(x - bp.x), dyy = (double)(y - bp.y);
              const float dist = (float)__builtin_sqrt(dxx * dxx + dyy * dyy);
              mbd = MINo(mbd, dist);
            }
            if (mbd < (float)radius) radius = f2i(mbd);
          }
        }
        while ((radius << 1) % 5 != 0) radius--;
        if (!edge_limit) B.radius[center] = radius > pc.P.strong_radius ? 0 : pc.P.strong_radius;
        else B.radius[center] = radius > pc.P.strong_radius ? radius : pc.P.strong_radius;
      } else {
        B.radius[center] = pc.P.strong_radius;
      }
    }
  } else {
    B.fit_plane[center] = make_float4(0, 0, 0, 0);
    if (pc.P.use_radius) B.radius[center] = pc.P.strong_radius;
  }
}

// ------------------------------------------------------------------------------ GetDepthandNormal
__global__ void k_depth_normal(const PassConst* __restrict__ pcp, DevBufs B) {   // DPE.cu:1940-1955
  const PassConst& pc = *pcp;
  PIX2D_FULL();
  float4 p = B.planes[center];
  p.w = depth_from_plane(pc.cams[0], p, x, y);
  B.planes[center] = transform_normal(pc.cams[0], p);
}

// ------------------------------------------------------------------------------ CheckerboardFilterStrong
// The up-to-21 candidates live in LDS, thread index fastest (conflict-free), so the insertion sort
// indexes them without scratch memory.  Launched with 128-thread (32 x 4) workgroups.
constexpr int kFilterThreads = 128;
__global__ void __launch_bounds__(kFilterThreads) k_filter(const PassConst* __restrict__ pcp, DevBufs B, int colour) {   // DPE.cu:1957-2101
  __shared__ float s_filter[21][kFilterThreads];
  const PassConst& pc = *pcp;
  PIX2D_HALF();
  const int W = pc.W, H = pc.H;
  if (B.weak[center] == DPE_WEAK) return;
  const float4* P = B.planes;
  struct Col {
    float* p;
    DEV float& operator[](int i) const { return p[i * kFilterThreads]; }
  } filter{&s_filter[0][threadIdx.y * blockDim.x + threadIdx.x]};
  int n = 0;
  filter[n++] = P[center].w;
  if (B.costs[center] < 0.001f) return;
  const int left = center - 1, leftleft = center - 3, up = center - W, upup = center - 3 * W;
  const int down = center + W, downdown = center + 3 * W, right = center + 1, rightright = center + 3;
  auto add = [&](bool cond, int idx) { if (cond && B.weak[idx] == DPE_STRONG) filter[n++] = P[idx].w; };
  add(y > 0, up); add(y > 2, upup); add(y > 4, upup - W * 2);
  add(y < H - 1, down); add(y < H - 3, downdown); add(y < H - 5, downdown + W * 2);
  add(x > 0, left); add(x > 2, leftleft); add(x > 4, leftleft - 2);
  add(x < W - 1, right); add(x < W - 3, rightright); add(x < W - 5, rightright + 2);
  add(y > 0 && x < W - 2, up + 2); add(y < H - 1 && x < W - 2, down + 2);
  add(y > 0 && x > 1, up - 2); add(y < H - 1 && x > 1, down - 2);
  add(x > 0 && y > 2, left - W * 2); add(x < W - 1 && y > 2, right - W * 2);
  add(x > 0 && y < H - 2, left + W * 2); add(x < W - 1 && y < H - 2, right + W * 2);
  for (int i = 1; i < n; i++) {
    const float tmp = filter[i];
    int j = i;
    for (; j >= 1 && tmp < filter[j - 1]; j--) filter[j] = filter[j - 1];
    filter[j] = tmp;
  }
  const int m = n / 2;
  B.planes[center].w = (n % 2 == 0) ? (filter[m - 1] + filter[m]) / 2 : filter[m];
}

// ------------------------------------------------------------------------------ staging kernels
// padded quad-texel images of 8-bit (or quarter-integer: q8 == nullptr) grey levels, both layouts
// (pass_common.h: TEX_U8, TEX_F16)
__global__ void k_build_quad8(const float* __restrict__ img, uint32_t* __restrict__ q8, uint2* __restrict__ q16,
                              int W, int H) {
  const int X = blockIdx.x * blockDim.x + threadIdx.x;
  const int Y = blockIdx.y * blockDim.y + threadIdx.y;
  if (X > W + 1 || Y > H + 1) return;
  auto cl = [](int v, int n) { return v < 0 ? 0 : (v > n - 1 ? n - 1 : v); };
  const int x0 = cl(X - 1, W), x1 = cl(X, W), y0 = cl(Y - 1, H), y1 = cl(Y, H);
  const float a = img[y0 * W + x0], b = img[y0 * W + x1], c = img[y1 * W + x0], d = img[y1 * W + x1];
  const size_t o = (size_t)Y * (W + 2) + X;
  if (q8) q8[o] = (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)c << 16) | ((uint32_t)d << 24);
  const h2v lo = (h2v){(_Float16)a, (_Float16)c};
  const h2v df = (h2v){(_Float16)(b - a), (_Float16)(d - c)};
  q16[o] = make_uint2(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, df));
}
// TEX_P16 column pairs (pass_common.h): (g(X-1, Y-1), g(X-1, Y)) as f16, X in [0, W+2], Y in [0, H+1]
__global__ void k_build_pair16(const float* __restrict__ img, uint32_t* __restrict__ qp, int W, int H) {
  const int X = blockIdx.x * blockDim.x + threadIdx.x;
  const int Y = blockIdx.y * blockDim.y + threadIdx.y;
  if (X > W + 2 || Y > H + 1) return;
  auto cl = [](int v, int n) { return v < 0 ? 0 : (v > n - 1 ? n - 1 : v); };
  const int x0 = cl(X - 1, W), y0 = cl(Y - 1, H), y1 = cl(Y, H);
  const h2v pr = (h2v){(_Float16)img[y0 * W + x0], (_Float16)img[y1 * W + x0]};
  qp[(size_t)Y * (W + 3) + X] = __builtin_bit_cast(uint32_t, pr);
}
// padded quad-texel image (see pass_common.h)
__global__ void k_build_quad(const float* __restrict__ img, float4* __restrict__ q, int W, int H) {
  const int X = blockIdx.x * blockDim.x + threadIdx.x;
  const int Y = blockIdx.y * blockDim.y + threadIdx.y;
  if (X > W + 1 || Y > H + 1) return;
  auto cl = [](int v, int n) { return v < 0 ? 0 : (v > n - 1 ? n - 1 : v); };
  const int x0 = cl(X - 1, W), x1 = cl(X, W), y0 = cl(Y - 1, H), y1 = cl(Y, H);
  q[Y * (W + 2) + X] = make_float4(img[y0 * W + x0], img[y0 * W + x1], img[y1 * W + x0], img[y1 * W + x1]);
}

}  // namespace dpe
