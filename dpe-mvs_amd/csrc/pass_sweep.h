// pass_sweep.h — cooperative red/black sweeps (CheckerboardPropagationStrong/Weak, DPE.cu:1214-1862).
//
// The reference runs one thread per pixel with cost_array[8][32] in local memory (DPE.cu:1236, 1690).
// Here a wave owns P pixels and gives each pixel C lanes:
//   strong sweep, edge mode      P = 4,  C = 16 (8 adaptive + 8 fixed 11-step candidates)
//   strong sweep, ACMH mode      P = 8,  C = 8  (near/far candidates)
//   weak sweep                   P = 8,  C = 8  (the 8 deformable neighbours)
// Candidate scans and the candidate x view NCC cost vectors run in parallel lanes; cost vectors
// live in LDS ([pixel][candidate][view], a few KB per wave, so occupancy is register-limited);
// the reference patch (weights, weight*grey) is built once per pixel in LDS.  Every step whose
// floating-point order or RNG order matters (CDF, the 15 view samples, cost sums over views,
// hypothesis acceptance) runs on the pixel's first lane in the reference's order, so results are
// bit-identical to the serial restatement.  Pixels come from per-colour compacted lists.
#pragma once
#include "pass_common.h"
#include "pass_refine.h"
#include "lds_layout.h"

namespace dpe {

// ------------------------------------------------------------------------------ pixel lists
// MODE 0: list[k] (k = colour*2 + weak?1:0) = pixels of that colour and class inside the red/black
//         grid (rows < half_rows), for the sweeps (built after NeigbourUpdate).
// MODE 1: one list of all WEAK pixels (rows < H), for GenNeighbours (built before it).
// MODE 2: colour-0 pixels of the red/black grid whose GenNeighbours failed (weak_rel == 0; the
//         pixels NeigbourUpdate turns UNKNOWN), for the iteration-0 colour-0 strong sweep that runs
//         beside GenNeighbours on the pre-GenNeighbours list (see dpe_pm_execute).
// Row-major order; one wave per row; ballot compaction keeps the order deterministic.
template <int MODE> constexpr int list_count() { return MODE == 0 ? 4 : 1; }
template <int MODE> DEV int list_rows(const PassConst& pc) { return MODE == 1 ? pc.H : pc.half_rows; }
template <int MODE> DEV int list_key(const PassConst& pc, const DevBufs& B, int x, int y) {
  if constexpr (MODE == 2) return (((x + y) & 1) == 0 && B.weak_rel[y * pc.W + x] == 0) ? 0 : -1;
  const bool wk = B.weak[y * pc.W + x] == DPE_WEAK;
  if constexpr (MODE == 1) return wk ? 0 : -1;
  else return (((x + y) & 1) << 1) | (wk ? 1 : 0);
}
template <int MODE>
__global__ void k_list_count(const PassConst* __restrict__ pcp, DevBufs B, int* __restrict__ row_counts) {
  constexpr int NL = list_count<MODE>();
  const PassConst& pc = *pcp;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int y = blockIdx.x * 4 + wave, rows = list_rows<MODE>(pc);
  if (y >= rows) return;
  int cnt[NL];
  for (int j = 0; j < NL; ++j) cnt[j] = 0;
  for (int x0 = 0; x0 < pc.W; x0 += 64) {
    const int x = x0 + lane;
    const int k = x < pc.W ? list_key<MODE>(pc, B, x, y) : -1;
#pragma unroll
    for (int j = 0; j < NL; ++j) cnt[j] += __popcll(__ballot(k == j));
  }
  if (lane == 0)
    for (int j = 0; j < NL; ++j) row_counts[j * rows + y] = cnt[j];
}
// exclusive scan of the row counts of each list: one wave per list, 64 rows per step
template <int MODE>
__global__ void k_list_scan(const PassConst* __restrict__ pcp, int* __restrict__ row_counts, int* __restrict__ totals) {
  const PassConst& pc = *pcp;
  const int j = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int rows = list_rows<MODE>(pc);
  if (j >= list_count<MODE>()) return;
  int acc = 0;
  for (int y0 = 0; y0 < rows; y0 += 64) {
    const int y = y0 + lane;
    const int c = y < rows ? row_counts[j * rows + y] : 0;
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(incl, o);
      if (lane >= o) incl += t;
    }
    if (y < rows) row_counts[j * rows + y] = acc + incl - c;
    acc += __shfl(incl, 63);
  }
  if (lane == 0) totals[j] = acc;
}
template <int MODE>
__global__ void k_list_fill(const PassConst* __restrict__ pcp, DevBufs B, const int* __restrict__ row_offsets,
                            int* __restrict__ lists, long list_stride) {
  constexpr int NL = list_count<MODE>();
  const PassConst& pc = *pcp;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int y = blockIdx.x * 4 + wave, rows = list_rows<MODE>(pc);
  if (y >= rows) return;
  int off[NL];
  for (int j = 0; j < NL; ++j) off[j] = row_offsets[j * rows + y];
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int x0 = 0; x0 < pc.W; x0 += 64) {
    const int x = x0 + lane;
    const int k = x < pc.W ? list_key<MODE>(pc, B, x, y) : -1;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const unsigned long long m = __ballot(k == j);
      if (k == j) lists[j * list_stride + off[j] + __popcll(m & below)] = y * pc.W + x;
      off[j] += __popcll(m);
    }
  }
}

// ------------------------------------------------------------------------------ weak list by patch side
// The weak sweep's NCC-New cost runs the pixel's centre patch at side n_c (6 at radius >= 5, 1 at the
// radius RANSACToGetFitPlane sets to 0; DPE.cu:1120-1212, 557-690), and a wave runs the sides of its
// pixels one after the other.  After the fits, each colour's weak list is stably partitioned into
// side >= 4 then side < 4 pixels (chunks of kPartChunk entries: count, scan, fill), so almost every
// wave holds one side.  Pixels of a half-sweep are independent, so the order changes no result.
constexpr int kPartChunk = 1024;
DEV int weak_side(const PassConst& pc, const DevBufs& B, int center) {
  const int rad = B.radius[center], inc = MAXo(2, d2i(2.0 * rad / 5.0));
  return rad >= 0 ? (2 * rad) / inc + 1 : 0;
}
DEV int part_key(const PassConst& pc, const DevBufs& B, int center) { return weak_side(pc, B, center) >= 4 ? 1 : 0; }
DEV int block_sum256(int v, int* s4) {   // sum over a 256-thread block (all threads call it)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) s4[threadIdx.x >> 6] = v;
  __syncthreads();
  const int t = s4[0] + s4[1] + s4[2] + s4[3];
  __syncthreads();
  return t;
}
static __global__ void __launch_bounds__(256) k_part_count(const PassConst* __restrict__ pcp, DevBufs B, const int* __restrict__ list,
                                                    const int* __restrict__ nlist_p, int* __restrict__ chunk_cnt) {
  const PassConst& pc = *pcp;
  const int n = *nlist_p, base = blockIdx.x * kPartChunk;
  if (base >= n) return;   // block-uniform
  __shared__ int s4[4];
  int cnt = 0;
  for (int i = base + (int)threadIdx.x; i < min(n, base + kPartChunk); i += 256) cnt += part_key(pc, B, list[i]);
  cnt = block_sum256(cnt, s4);
  if (threadIdx.x == 0) chunk_cnt[blockIdx.x] = cnt;
}
// exclusive scan of the chunk counts (one 256-thread block); total side->=4 count into *tot
static __global__ void __launch_bounds__(256) k_part_scan(const int* __restrict__ nlist_p, int* __restrict__ chunk_cnt,
                                                   int* __restrict__ tot) {
  __shared__ int s4[4];
  const int nch = (*nlist_p + kPartChunk - 1) / kPartChunk;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int acc = 0;
  for (int k0 = 0; k0 < nch; k0 += 256) {
    const int k = k0 + (int)threadIdx.x;
    const int c = k < nch ? chunk_cnt[k] : 0;
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(incl, o);
      if (lane >= o) incl += t;
    }
    if (lane == 63) s4[wave] = incl;
    __syncthreads();
    int before = acc;
    for (int w = 0; w < wave; ++w) before += s4[w];
    const int all = s4[0] + s4[1] + s4[2] + s4[3];
    __syncthreads();
    if (k < nch) chunk_cnt[k] = before + incl - c;
    acc += all;
  }
  if (threadIdx.x == 0) *tot = acc;
}
static __global__ void __launch_bounds__(256) k_part_fill(const PassConst* __restrict__ pcp, DevBufs B, const int* __restrict__ list,
                                                   const int* __restrict__ nlist_p, const int* __restrict__ chunk_off,
                                                   const int* __restrict__ tot, int* __restrict__ out) {
  const PassConst& pc = *pcp;
  const int n = *nlist_p, base = blockIdx.x * kPartChunk;
  if (base >= n) return;
  __shared__ int s4[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int offA = chunk_off[blockIdx.x], offB = *tot + (base - offA);
  const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  int runA = 0;   // side->=4 entries of this chunk before the current step
  for (int i0 = base; i0 < min(n, base + kPartChunk); i0 += 256) {
    const int i = i0 + (int)threadIdx.x;
    const int p = i < n ? list[i] : 0;
    const int k = i < n ? part_key(pc, B, p) : 0;
    const unsigned long long m = __ballot(k == 1);
    if (lane == 0) s4[wave] = __popcll(m);
    __syncthreads();
    int a = runA + __popcll(m & below);
    for (int w = 0; w < wave; ++w) a += s4[w];
    const int all = s4[0] + s4[1] + s4[2] + s4[3];
    __syncthreads();
    if (i < n) out[k ? offA + a : offB + (i - base) - a] = p;
    runA += all;
  }
}

// ------------------------------------------------------------------------------ view selection
// sampling probability of view i before the prior (DPE.cu:1568-1589), costs by candidate j.
template <class CostF>
DEV float view_prob_raw(CostF cost, int i, float cost_threshold) {
  float count = 0; int count_false = 0; float tmpw = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const float c = cost(j, i);
    if (c < cost_threshold) { tmpw += d_expf(c * c / (-0.18f)); count++; }
    if (c > 1.2f) count_false++;
  }
  float sp = 0.0f;
  if (count > 2 && count_false < 3) sp = tmpw / count;
  else if (count_false < 3) sp = d_expf(cost_threshold * cost_threshold / (-0.32f));
  return sp;
}

// Serial part of the joint view selection on one lane (DPE.cu:1592-1615): CDF over `sp`, 15 samples.
DEV void view_sample(const float* sp, int nv, Rng& rs, uint8_t* vw, uint32_t& tsv, float& wnorm) {
  for (int i = 0; i < DPE_MAX_IMAGES; ++i) vw[i] = 0;
  float psum = 0.0f;
  for (int i = 0; i < nv; ++i) psum += sp[i];
  const float inv = 1.0f / psum;
  float cdf[DPE_MAX_IMAGES];
  float cum = 0.0f;
  for (int i = 0; i < nv; ++i) { const float q = sp[i] * inv; cum += q; cdf[i] = cum; }
  for (int s = 0; s < 15; ++s) {
    const float rp = rng_uniform(rs) - 1.1920929e-07f;
    for (int id = 0; id < nv; ++id)
      if (cdf[id] > rp) { vw[id] += 1; break; }
  }
  uint32_t t = 0; float wn = 0;
  for (int i = 0; i < nv; ++i) if (vw[i] > 0) { setBit(t, i); wn += vw[i]; }
  tsv = t; wnorm = wn;
}

// The same sampling on the C lanes of one pixel: the CDF is built in the reference's order on lane
// 0 (in place of sp), the 15 draws (stream words 0..14) and their CDF searches run one per lane,
// and the per-view counts are LDS integer atomics (order-free).  cnt: nv ints of scratch.
// Leaves vwl[0..31] and the global copy vwg[0..31]; the caller's lane-0 stream is then positioned
// with rng_seek(rs, 15).  Every lane of the wave calls it (wave_sync inside).
DEV void view_sample_coop(float* sp, int* cnt, int nv, int c, int C, bool active, const Rng& rs, uint8_t* vwl,
                          uint8_t* vwg) {
  if (active) {
    if (c == 0) {
      float psum = 0.0f;
      for (int i = 0; i < nv; ++i) psum += sp[i];
      const float inv = 1.0f / psum;
      float cum = 0.0f;
      for (int i = 0; i < nv; ++i) { const float q = sp[i] * inv; cum += q; sp[i] = cum; }
    }
    for (int v = c; v < nv; v += C) cnt[v] = 0;
  }
  wave_sync();
  if (active) {
    for (int s = c; s < 15; s += C) {
      const float rp = u32_to_uniform(rng_word(rs, (uint32_t)s)) - 1.1920929e-07f;
      for (int id = 0; id < nv; ++id)
        if (sp[id] > rp) { atomicAdd(&cnt[id], 1); break; }
    }
  }
  wave_sync();
  if (active)
    for (int j = c; j < DPE_MAX_IMAGES; j += C) {
      const uint8_t w = j < nv ? (uint8_t)cnt[j] : (uint8_t)0;
      vwl[j] = w;
      vwg[j] = w;
    }
  wave_sync();
}

// ------------------------------------------------------------------------------ candidate scans
// Edge-adaptive (kind 0) and fixed 11-step (kind 1) scans of direction d (DPE.cu:1250-1292, 1297-1322).
DEV int edge_candidate(const PassConst& pc, const DevBufs& B, const float* __restrict__ costs, int x, int y, int center,
                       int iter, int d, int kind, bool on_edge) {
  const int W = pc.W, H = pc.H;
  const int dx = kDir[d][0], dy = kDir[d][1];
  const int s0 = MAXo(1, 5 - 2 * iter);
  const int min_step_len = 2;
  int step_num = 11, step_len = min_step_len;
  if (kind == 0) {
    const float max_edge_dist = MAXo(H, W) / 30.0f;
    const short2 ep = B.edge_neigh[(size_t)center * 8 + d];
    const double ex = (double)(ep.x - x), ey = (double)(ep.y - y);
    float dist = (float)__builtin_sqrt(ex * ex + ey * ey);
    if (d >= 4) dist = (float)((double)dist / 1.4142135623730951);
    if (on_edge) dist = 11 * min_step_len;
    else if (ep.x == -1 || ep.y == -1 || dist > max_edge_dist) {
      dist = max_edge_dist;
      if (d >= 4) dist = (float)((double)dist / 1.4142135623730951);
    }
    step_num = MINo(MAXo(11, f2i(1.0f * dist / min_step_len)), 22);
    step_len = MAXo(f2i(1.0f * dist / step_num), min_step_len);
    if (d < 4 && step_len % 2 == 1) step_len -= 1;
  }
  int fx = 0, fy = 0;
  if (d > 4) { if (d % 2) fx = dx; else fy = dy; }
  int mpos = -1; float mc = 3.40282347e+38f;
  // the loads of 8 steps are issued together, then scanned in step order (same first minimum)
  for (int s = 0; s < step_num; s += 8) {
    float cv[8]; int pv[8]; bool ok[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int step = s + u;
      const int tx = x + s0 * dx + step * step_len * dx + fx, ty = y + s0 * dy + step * step_len * dy + fy;
      ok[u] = step < step_num && tx >= 0 && ty >= 0 && tx < W && ty < H;
      pv[u] = tx + ty * W;
      cv[u] = ok[u] ? costs[pv[u]] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (ok[u] && mc > cv[u]) { mpos = pv[u]; mc = cv[u]; }
  }
  return mc < 3.40282347e+38f ? mpos : -1;
}

// ACMH near/far candidate of slot s (DPE.cu:1346-1544): 0 up_near, 1 up_far, 2 down_near,
// 3 down_far, 4 left_near, 5 left_far, 6 right_near, 7 right_far.  -1 if the slot is absent.
DEV int acmh_candidate(const PassConst& pc, const float* __restrict__ costs, int x, int y, int center, int s) {
  const int W = pc.W, H = pc.H;
  float costMin; int cmp;
  switch (s) {
    case 1: {
      if (!(y > 2)) return -1;
      const int up_far = center - 3 * W; costMin = costs[up_far]; cmp = up_far;
      for (int i = 1; i < 11; ++i) if (y > 2 + 2 * i) { const int pt = up_far - 2 * i * W; if (costs[pt] < costMin) { costMin = costs[pt]; cmp = pt; } }
      return cmp;
    }
    case 3: {
      if (!(y < H - 3)) return -1;
      const int down_far = center + 3 * W; costMin = costs[down_far]; cmp = down_far;
      for (int i = 1; i < 11; ++i) if (y < H - 3 - 2 * i) { const int pt = down_far + 2 * i * W; if (costs[pt] < costMin) { costMin = costs[pt]; cmp = pt; } }
      return cmp;
    }
    case 5: {
      if (!(x > 2)) return -1;
      const int left_far = center - 3; costMin = costs[left_far]; cmp = left_far;
      for (int i = 1; i < 11; ++i) if (x > 2 + 2 * i) { const int pt = left_far - 2 * i; if (costs[pt] < costMin) { costMin = costs[pt]; cmp = pt; } }
      return cmp;
    }
    case 7: {
      if (!(x < W - 3)) return -1;
      const int right_far = center + 3; costMin = costs[right_far]; cmp = right_far;
      for (int i = 1; i < 11; ++i) if (x < W - 3 - 2 * i) { const int pt = right_far + 2 * i; if (costs[pt] < costMin) { costMin = costs[pt]; cmp = pt; } }
      return cmp;
    }
    case 0: {
      if (!(y > 0)) return -1;
      const int up_near = center - W; costMin = costs[up_near]; cmp = up_near;
      for (int i = 0; i < 3; ++i) {
        if (y > 1 + i && x > i) { const int pt = up_near - (1 + i) * W - (1 + i); if (costs[pt] < costMin) { costMin = costs[pt]; cmp = pt; } }
        if (y > 1 + i && x < W - 1 - i) { const int pt = up_near - (1 + i) * W + (1 + i); if (costs[pt] < costMin) { costMin = costs[pt]; cmp = pt; } }
      }
      return cmp;
    }
    case 2: {
      if (!(y < H - 1)) return -1;
      const int down_near = center + W; costMin = costs[down_near]; cmp = down_near;
      for (int i = 0; i < 3; ++i) {
        if (y < H - 2 - i && x > i) { const int pt = down_near + (1 + i) * W - (1 + i); if (costs[pt] < costMin) { costMin = costs[pt]; cmp = pt; } }
        if (y < H - 2 - i && x < W - 1 - i) { const int pt = down_near + (1 + i) * W + (1 + i); if (costs[pt] < costMin) { costMin = costs[pt]; cmp = pt; } }
      }
      return cmp;
    }
    case 4: {
      if (!(x > 0)) return -1;
      const int left_near = center - 1; costMin = costs[left_near]; cmp = left_near;
      for (int i = 0; i < 3; ++i) {
        if (x > 1 + i && y > i) { const int pt = left_near - (1 + i) - (1 + i) * W; if (costs[pt] < costMin) { costMin = costs[pt]; cmp = pt; } }
        if (x > 1 + i && y < H - 1 - i) { const int pt = left_near - (1 + i) + (1 + i) * W; if (costs[pt] < costMin) { costMin = costs[pt]; cmp = pt; } }
      }
      return cmp;
    }
    default: {   // 6
      if (!(x < W - 1)) return -1;
      const int right_near = center + 1; costMin = costs[right_near]; cmp = right_near;
      for (int i = 0; i < 3; ++i) {
        if (x < W - 2 - i && y > i) { const int pt = right_near + (1 + i) - (1 + i) * W; if (costs[pt] < costMin) { costMin = costs[pt]; cmp = pt; } }
        if (x < W - 2 - i && y < H - 1 - i) { const int pt = right_near + (1 + i) + (1 + i) * W; if (costs[pt] < costMin) { costMin = costs[pt]; cmp = pt; } }
      }
      return cmp;
    }
  }
}

// ------------------------------------------------------------------------------ strong sweep
constexpr int kTailJobs = 16;   // a last round of at most this many jobs is split by patch rows
// the strong sweep's LDS carve per wave (lds_layout.h: P pixels, C candidate lanes, nv source views)
template <int P, int C> using StrongCarveT = lds::StrongCarve<P, C, kTailJobs>;
__host__ __device__ inline int strong_lds_per_wave(int P, int C, int nv) {
  return P == 4 && C == 16 ? StrongCarveT<4, 16>::total(nv) : StrongCarveT<8, 8>::total(nv);
}

// Job pools of a wave: the NCCs of all its pixels are dealt round-robin over the 64 lanes, so a
// lane's work does not depend on how many candidates / selected views its own pixel has.
// (pixel p, item i) <- flat job j, given per-pixel job counts cnt[p].
template <int P>
DEV bool job_decode(const int* cnt, int j, int& p, int& r) {
  r = j;
#pragma unroll
  for (int q = 0; q < P; ++q) {
    if (r < cnt[q]) { p = q; return true; }
    r -= cnt[q];
  }
  return false;
}

// waves per workgroup: 2 (4 before round 5's end; 2 fits the first half-sweep beside GenNeighbours
// better: wall -0.6 ms together with DepthToWeak at 1, profiles/r05ao_ab_wgsize2.log)
constexpr int kBwStrong = 2;
template <int U8, bool EDGE>
__global__ void __launch_bounds__(64 * kBwStrong, kTapWaves) k_strong_coop(const PassConst* __restrict__ pcp, DevBufs B, int iter,
                                                     const int* __restrict__ list, const int* __restrict__ nlist_p) {
  extern __shared__ float4 lds4[];
  float* lds = (float*)lds4;
  const int nlist = *nlist_p;
  constexpr int C = EDGE ? 16 : 8;
  constexpr int P = 64 / C;
  const PassConst& pc = *pcp;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ps = lane / C, c = lane % C;
  const int W = pc.W, nv = pc.N - 1;
  const DpeCamera& c0 = pc.cams[0];
  const int wbase = (xcd_remap(blockIdx.x, gridDim.x, B.xcd_rows * 16) * kBwStrong + wave) * P;
  if (wbase >= nlist) return;                          // wave-uniform tail
  const int gi = wbase + ps;
  const bool active = gi < nlist;
  const int center = active ? list[gi] : 0;
  const int x = center % W, y = center / W;
  // ---- LDS carve (per wave, lds_layout.h; arrays indexed by pixel q where another pixel's data is read)
  using SC = StrongCarveT<P, C>;
  float* wl = lds + (size_t)wave * SC::total(nv);
  float4* hyp_all = (float4*)(wl + SC::hyp());           // [P][5] float4
  float* pw_all = wl + SC::patch();                      // [P][108] patch
  float* cost_all = wl + SC::cost(nv);                   // [P][C + 1][nv]; slot C = the current plane
  float* sp = wl + SC::sp(nv) + ps * nv;                 // [P][nv]
  float* ref_all = wl + SC::ref(nv);                     // [P][5][nv] refinement NCCs
  float* fc = wl + SC::fc(nv) + ps * 8;                  // [P][8]  final costs
  float* sums_all = wl + SC::sums(nv);                   // [P][4]  patch sums s_ref, s_rr, s_w; wnorm
  uint8_t* vwl = (uint8_t*)(wl + SC::vw(nv)) + ps * 32;  // [P][32] view weights
  int* ib_all = (int*)(wl + SC::ib(nv));
  const int ibs = SC::ib_ints(nv);                       // ints per pixel
  int* ib = ib_all + ps * ibs;
  int* posl = ib + SC::IB_POS;                           // [C] candidate positions (-1 = none)
  int* fin = ib + SC::IB_FIN;                            // [8] final slot of direction d (-1 = zero vector)
  int* misc = ib + SC::IB_MISC;                          // [8] 0: nsel, 1: job slots (candidates + current)
  int* sel_list = ib + SC::IB_SEL;                       // [nv]
  int* slots = ib + SC::ib_slots(nv);                    // [C + 1] cost-vector jobs: candidate slots, then C
  float4* cpl_all = (float4*)(wl + SC::cpl(nv));         // [P][C + 1] candidate planes, slot C = current
  int* alias_all = (int*)(wl + SC::alias(nv));           // [P][C + 1]
  float* rnd = wl + SC::rnd(nv) + ps * 12;               // [P][12] refinement draws
  float4* cpl = cpl_all + ps * (C + 1);
  int* alias = alias_all + ps * (C + 1);
  float4* hyp = hyp_all + ps * 5;
  float* pw = pw_all + ps * 108;
  float* cost = cost_all + ps * (C + 1) * nv;
  float* ref = ref_all + ps * 5 * nv;

  const float* __restrict__ costs_s = B.costs_snap;
  const float4* __restrict__ planes_s = B.planes_snap;
  const bool fast = FAST_PATCH(pc);
  bool on_edge = false;
  PHASE_BEGIN();
  // ---- phase 1: reference patch + candidate scans
  if (active) {
    if (fast) patch_lds_build<C>(pw, pc, B, x, y, c);
    PHASE(14);
    int pos;
    if constexpr (EDGE) {
      on_edge = B.edge[center] != 0;
      const int d = c & 7, kind = c >> 3;
      pos = (kind == 1 && on_edge) ? -1 : edge_candidate(pc, B, costs_s, x, y, center, iter, d, kind, on_edge);
    } else {
      pos = acmh_candidate(pc, costs_s, x, y, center, c);
    }
    posl[c] = pos;
    auto phash = [](const float4& p) -> int {
      uint32_t h = __float_as_uint(p.x) * 0x9E3779B1u;
      h = (h ^ (h >> 15) ^ __float_as_uint(p.y)) * 0x85EBCA77u;
      h = (h ^ (h >> 13) ^ __float_as_uint(p.z)) * 0xC2B2AE3Du;
      h = (h ^ (h >> 16) ^ __float_as_uint(p.w)) * 0x27D4EB2Fu;
      return (int)((h ^ (h >> 15)) & 0x7FFFFFFFu);
    };
    if (pos >= 0) { const float4 pl = planes_s[pos]; cpl[c] = pl; alias[c] = phash(pl); }
    else alias[c] = (int)(0x80000000u | (uint32_t)c);
    if (c == 0) { const float4 pl = planes_s[center]; cpl[C] = pl; alias[C] = phash(pl); }
  }
  wave_sync();
  PHASE(0);
  // ---- phase 1b: bitwise-identical planes among the candidates and the current plane (a third of
  // the candidates in a converged map: propagation copies planes) share one cost vector.  alias[]
  // first holds a 31-bit hash of each valid slot's plane (absent slots: a unique value with the top
  // bit set); the earliest equal-hash slot is then confirmed bit by bit.
  auto same = [](const float4& a, const float4& b) {
    return __float_as_uint(a.x) == __float_as_uint(b.x) && __float_as_uint(a.y) == __float_as_uint(b.y) &&
           __float_as_uint(a.z) == __float_as_uint(b.z) && __float_as_uint(a.w) == __float_as_uint(b.w);
  };
  int al[2] = {-1, -1};
  if (active) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int sl = c + r * C;
      if (sl > C || (sl < C && posl[sl] < 0)) continue;
      const float4 me = cpl[sl];
      const uint32_t h = (uint32_t)alias[sl];
      uint32_t m = 0;
#pragma unroll
      for (int t = 0; t < C; ++t) m |= ((uint32_t)alias[t] == h && t < sl) ? (1u << t) : 0u;
      int a = sl;
      while (m) {
        const int t = __builtin_ctz(m);
        if (same(cpl[t], me)) { a = t; break; }
        m &= m - 1;
      }
      al[r] = a;
    }
  }
  wave_sync();
  if (active) {
    alias[c] = al[0];
    if (c == 0) alias[C] = al[1];
  }
  wave_sync();
  PHASE(1);
  if (c == 0) {
    int n = 0;
    if (active) {
      for (int k = 0; k <= C; ++k) if (alias[k] == k) slots[n++] = k;
      if (fast) patch_lds_pre(pw, sums_all[ps * 4 + 0], sums_all[ps * 4 + 1], sums_all[ps * 4 + 2]);
    }
    misc[SC::MI_JOBS] = n;
  }
  wave_sync();
  PHASE(2);
  // ---- phase 2: cost vectors of every candidate and of the current plane, one flat pool
  {
    // view-major order: the lanes of one round gather from the same source image (cache locality)
    int cnt[P], S = 0;
#pragma unroll
    for (int q = 0; q < P; ++q) { cnt[q] = ib_all[q * ibs + SC::IB_MISC + 1]; S += cnt[q]; }
    int q, r;
    const int total = S * nv, tail = total & 63;
    // a last round with at most kTailJobs jobs: each job's 6 patch rows go to 64 / tail lanes (rows
    // per lane 1 or 2), the row sums meet in LDS, and one lane per job adds them in row order
    const bool split = fast && tail > 0 && tail <= kTailJobs;
    POOL_STAT(0, total);
    const int jend = split ? total - tail : total;
    for (int j = lane; j < jend; j += 64) {
      job_decode<P>(cnt, j % S, q, r);
      const int* iq = ib_all + q * ibs;
      const int slot = iq[SC::ib_slots(nv) + r], v = j / S + 1;
      const int cq = list[wbase + q];
      const int qx = cq % W, qy = cq / W;
      const float4 pl = cpl_all[q * (C + 1) + slot];
      const float* sm = sums_all + q * 4;
      cost_all[(q * (C + 1) + slot) * nv + v - 1] =
          ncc_old_any<U8>(fast, pw_all + q * 108, sm[0], sm[1], sm[2], qx, qy, pc, B, v, pl);
    }
    if (split) {
      float* tb = wl + SC::tail(nv);                     // [job][row][3]
      const int rpp = 64 / tail >= 6 ? 1 : 2, npc = 6 / rpp;            // rows per lane, lanes per job
      if (lane < tail * npc) {
        const int j = jend + lane / npc, a0 = (lane % npc) * rpp;
        job_decode<P>(cnt, j % S, q, r);
        const int slot = ib_all[q * ibs + SC::ib_slots(nv) + r], v = j / S + 1;
        const int cq = list[wbase + q];
        const int qx = cq % W, qy = cq / W;
        const Homog H = make_homography(pc, v, cpl_all[q * (C + 1) + slot]);
        if (!center_outside(pc, v, H, qx, qy)) {
          const bool fr = rcp_range_ok(H, (float)(qx - 5), (float)(qx + 5), (float)(qy - 5), (float)(qy + 5));
          for (int a = a0; a < a0 + rpp; ++a) {
            float* r3 = tb + ((lane / npc) * 6 + a) * 3;
            if (fr) lds_row<U8, true>(pw_all + q * 108, qx, qy, pc, B, v, H, a, r3);
            else lds_row<U8, false>(pw_all + q * 108, qx, qy, pc, B, v, H, a, r3);
          }
        }
      }
      wave_sync();
      if (lane < tail) {
        const int j = jend + lane;
        job_decode<P>(cnt, j % S, q, r);
        const int slot = ib_all[q * ibs + SC::ib_slots(nv) + r], v = j / S + 1;
        const int cq = list[wbase + q];
        const Homog H = make_homography(pc, v, cpl_all[q * (C + 1) + slot]);
        float cst = 2.0f;
        if (center_outside(pc, v, H, cq % W, cq / W)) {
          count_work(B, 1, 0);
        } else {
          count_work(B, 1, 36);
          float s_src = 0, s_ss = 0, s_rs = 0;
          for (int a = 0; a < 6; ++a) {
            const float* r3 = tb + (lane * 6 + a) * 3;
            s_src += r3[0]; s_ss += r3[1]; s_rs += r3[2];
          }
          const float* sm = sums_all + q * 4;
          cst = ncc_finalize_pre(sm[0], sm[1], sm[2], s_src, s_ss, s_rs);
        }
        cost_all[(q * (C + 1) + slot) * nv + v - 1] = cst;
      }
    }
  }
  wave_sync();
  PHASE(3);
  if (active) {                                          // duplicates take their original's vector
    for (int sl = c; sl <= C; sl += C) {
      const int a = alias[sl];
      if (a >= 0 && a != sl)
        for (int v = 0; v < nv; ++v) cost[sl * nv + v] = cost[a * nv + v];
    }
  }
  wave_sync();
  PHASE(4);
  // ---- phase 3: arbitration of the two candidates of each direction (edge mode, DPE.cu:1323-1342)
  if (active && c < 8) {
    if constexpr (EDGE) {
      const int d = c;
      const bool hasA = posl[d] >= 0, hasB = !on_edge && posl[8 + d] >= 0;
      int f = hasA ? d : -1;
      if (hasB) {
        const float good_threshold = 0.8f * d_expf((float)(iter * iter) / (-90.0f));
        int g0 = 0, g1 = 0, b0 = 0, b1 = 0;
        for (int j = 0; j < nv; ++j) {
          // slot A as the reference sees it: its vector, or the zero-initialised row
          const float v0 = hasA ? cost[d * nv + j] : ((d == 0 && j == 0) ? 2.0f : 0.0f);
          if (v0 < good_threshold) g0++;
          if (v0 > 1.2f) b0++;
          const float v1 = cost[(8 + d) * nv + j];
          if (v1 < good_threshold) g1++;
          if (v1 > 1.2f) b1++;
        }
        if (!hasA || g1 > g0 || (g1 == g0 && b1 < b0)) f = 8 + d;
      }
      fin[d] = f;
    } else {
      fin[c] = posl[c] >= 0 ? c : -1;
    }
  }
  wave_sync();
  PHASE(5);
  // cost of (direction j, view i) as the reference's cost_array holds it
  auto cst = [&](int j, int i) -> float {
    const int f = fin[j];
    return f >= 0 ? cost[f * nv + i] : ((j == 0 && i == 0) ? 2.0f : 0.0f);
  };
  const float cost_threshold = (float)(0.8 * (double)d_expf((float)(iter * iter) / (-90.0f)));
  // ---- phase 4: per-view sampling probabilities with the 4-neighbour priors (DPE.cu:1552-1590)
  if (active) {
    const long Lp = (long)W * pc.H;
    uint32_t nsv[4];
    bool nfl[4];
    const long npos[4] = {(long)center - W, (long)center + W, (long)center - 1, (long)center + 1};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      nfl[i] = fin[2 * i] >= 0;
      nsv[i] = (nfl[i] && npos[i] >= 0 && npos[i] < Lp) ? B.sel_snap[npos[i]] : 0u;
    }
    for (int v = c; v < nv; v += C) {
      float prior = 0.0f;
#pragma unroll
      for (int i = 0; i < 4; ++i) if (nfl[i]) prior += isSet(nsv[i], v) == 1 ? 0.9f : 0.1f;
      sp[v] = view_prob_raw(cst, v, cost_threshold) * prior;
    }
  }
  wave_sync();
  PHASE(6);
  // ---- samples + view weights (cooperative), then the selected-view list on lane 0
  Rng rs;
  rng_init(rs, (uint32_t)center, pc.seed32, STREAM_ITER_BASE + 4 * iter + 0, pc.salt);
  view_sample_coop(sp, (int*)ref, nv, c, C, active, rs, vwl, B.vw + (size_t)center * DPE_MAX_IMAGES);
  PHASE(12);
  uint32_t tsv = 0; float wnorm = 0.0f;
  if (c == 0) {
    int ns = 0;
    if (active) {
      rng_seek(rs, 15);
      for (int i = 0; i < nv; ++i) if (vwl[i] > 0) { setBit(tsv, i); wnorm += vwl[i]; sel_list[ns++] = i; }
      sums_all[ps * 4 + 3] = wnorm;
    }
    misc[SC::MI_NSEL] = ns;
  }
  wave_sync();
  PHASE(7);
  const int nsel = active ? misc[SC::MI_NSEL] : 0;
  // ---- phase 5: final costs of the 8 directions
  if (active && c < 8) {
    float wn = 0.0f;
    for (int i = 0; i < nv; ++i) wn += vwl[i];   // == weight_norm (same order: sum of vw > 0)
    float f = 0.0f;
    for (int j = 0; j < nv; ++j) { const int w = vwl[j]; if (w > 0) f += w * cst(c, j); }
    fc[c] = f / wn;
  }
  wave_sync();
  PHASE(8);
  // ---- serial: propagation acceptance + refinement hypotheses (DPE.cu:1617-1654, 1065-1095)
  float cost_now = 0.0f, cost_written = 0.0f, depth_now = 0.0f;
  float4 pnow = make_float4(0, 0, 0, 0);
  const float pert = (float)(0.02f * 3.14159265358979323846);
  // lanes 1..4 evaluate the refinement draws (refine_draws: stream words 15.. after the view
  // sampling) while lane 0 runs the acceptance; lane 0 then finishes the hypotheses from them
  if (active && c >= 1 && c <= 4) {
    const RefineDraws d = refine_draws(rs, 15u);
    if (c == 1) { rnd[0] = d.u_depth; rnd[1] = d.n[0]; rnd[2] = d.n[1]; rnd[3] = d.n[2]; rnd[4] = d.u_pert; }
    else refine_angle(rs, d.w_angles, c - 2, pert, &rnd[5 + 2 * (c - 2)], &rnd[6 + 2 * (c - 2)]);
  }
  if (active && c == 0) {
    int mi = 0; float mcost = fc[0];
    for (int i = 1; i < 8; ++i) if (fc[i] <= mcost) { mcost = fc[i]; mi = i; }
    const float4 curp = planes_s[center];
    for (int k = 0; k < nsel; ++k) cost_now += vwl[sel_list[k]] * cost[C * nv + sel_list[k]];
    cost_now /= wnorm;
    cost_written = cost_now;
    B.costs[center] = cost_now;
    depth_now = depth_from_plane(c0, curp, x, y);
    pnow = curp;
    const int f = fin[mi];
    if (f >= 0) {
      const float4 cand = planes_s[posl[f]];
      const float db = depth_from_plane(c0, cand, x, y);
      if (db >= pc.P.depth_min && db <= pc.P.depth_max && fc[mi] < cost_now) {
        depth_now = db; pnow = cand; cost_now = fc[mi]; B.sel[center] = tsv;
      }
    }
  }
  wave_sync();
  if (active && c == 0) {
    const float dmin = pc.P.depth_min, dmax = pc.P.depth_max;
    const float depth_rand = rnd[0] * (dmax - dmin) + dmin;
    const float4 prand = random_normal_from(c0, x, y, rnd + 1, depth_now);
    const float dminp = (1 - 0.02f) * depth_now, dmaxp = (1 + 0.02f) * depth_now;
    const float depth_perturbed = rnd[4] * (dmaxp - dminp) + dminp;
    const float4 ppert = perturbed_normal_from(c0, x, y, pnow, rnd + 5);
    float4 h0 = pnow, h1 = prand, h2 = prand, h3 = ppert, h4 = pnow;
    h0.w = dist2origin(c0, x, y, depth_rand, h0);
    h1.w = dist2origin(c0, x, y, depth_now, h1);
    h2.w = dist2origin(c0, x, y, depth_rand, h2);
    h3.w = dist2origin(c0, x, y, depth_now, h3);
    h4.w = dist2origin(c0, x, y, depth_perturbed, h4);
    hyp[0] = h0; hyp[1] = h1; hyp[2] = h2; hyp[3] = h3; hyp[4] = h4;
  }
  wave_sync();
  PHASE(9);
  // ---- phase 6: refinement NCCs, one flat pool of (pixel, hypothesis, selected view)
  {
    int cnt[P];
#pragma unroll
    for (int q = 0; q < P; ++q) cnt[q] = 5 * ib_all[q * ibs + SC::IB_MISC];
    POOL_STAT(1, [&] { int t = 0; for (int q = 0; q < P; ++q) t += cnt[q]; return t; }());
    int q, r;
    for (int j = lane; job_decode<P>(cnt, j, q, r); j += 64) {
      const int* iq = ib_all + q * ibs;
      const int h = r % 5, k = r / 5;                      // the 5 hypotheses of one view adjacent
      const int cq = list[wbase + q];
      const float* sm = sums_all + q * 4;
      ref_all[(q * 5 + h) * nv + k] = ncc_old_any<U8>(fast, pw_all + q * 108, sm[0], sm[1], sm[2], cq % W, cq / W, pc,
                                                      B, iq[SC::IB_SEL + k] + 1, hyp_all[q * 5 + h]);
    }
  }
  wave_sync();
  PHASE(10);
  // ---- hypothesis costs and depths (one lane each), then sequential acceptance + write-back on
  // lane 0 (DPE.cu:1097-1117, 1656-1665)
  if (active && c < 5) {
    const int h = c;
    float tc = 0.0f;
    for (int k = 0; k < nsel; ++k) tc += vwl[sel_list[k]] * ref[h * nv + k];
    tc /= sums_all[ps * 4 + 3];
    fc[h] = tc;
    misc[SC::MI_DEPTH + h] = __float_as_int(depth_from_plane(c0, hyp[h], x, y));
  }
  wave_sync();
  PHASE(13);
  if (active && c == 0) {
    const float dmin = pc.P.depth_min, dmax = pc.P.depth_max;
    for (int h = 0; h < 5; ++h) {
      const float tc = fc[h], db = __int_as_float(misc[SC::MI_DEPTH + h]);
      if (db >= dmin && db <= dmax && tc < cost_now) { depth_now = db; pnow = hyp[h]; cost_now = tc; }
    }
    if (pc.P.state == DPE_REFINE_INIT) {
      if ((double)cost_now < (double)cost_written - 0.1) { B.costs[center] = cost_now; B.planes[center] = pnow; }
    } else {
      B.costs[center] = cost_now;
      B.planes[center] = pnow;
    }
  }
  PHASE(11);
  PHASE_END(0);
}

// ------------------------------------------------------------------------------ weak sweep
// The NCC-New cost of a weak pixel (DPE.cu:557-690) is 9 bilateral patches (its own, radius from
// the RANSAC radius map, and one around each deformable strong neighbour).  All tap weights are
// plane- and view-independent, so they are tabulated once per pixel in LDS together with the
// reference sums of each patch; an NCC job is then projection + bilinear fetch + 3 FMAs per tap.
struct WeakTab {
  const float* tc;                        // centre patch (w, w*grey) pairs [n_c^2][2]
  const float* tn;                        // neighbour k=1..8: pairs at [((k-1)*9 + t)*2]
  const float* sums;                      // [9][3]: ncc_pre (1/s_w, s_ref/s_w, var_ref) of each tabulated patch
  const short2* nbl;                      // [9] neighbour pixels (nb[0] = the pixel itself)
  const uint32_t* nsv;                    // [9] selected_views of the neighbours
  int rad_c, inc_c, n_c, rad_n, inc_n, n_n;
  bool tab_c, tab_n;
  float rc;                               // grey level of the pixel
  bool nb3;                               // neighbour patches are tabulated 3x3 and nbox is set
  float nbox[4];                          // x0, x1, y0, y1 of the union of the neighbour patches
};

// patch NCC with tabulated weights; the same tap order and arithmetic as patch_ncc_generic.
// NN > 0: the patch side n is the compile-time NN, so the tap loop unrolls and the gathers of a
// patch are in flight together (the weak sweep's patches are 3x3 and 4..6 square).
template <int U8, bool FAST, int NN = 0>
DEV void tab_taps(const PassConst& pc, const DevBufs& B, int v, const Homog& H0, int cx, int cy, int rad, int inc,
                  int n_rt, const float* __restrict__ tw, float* acc) {
  const int W = pc.W, Hh = pc.H;
  const Homog H = scale_cols(H0);
  const int n = NN > 0 ? NN : n_rt;
  const f2v* wp = (const f2v*)tw;            // (w, w*grey) pairs
  if constexpr (U8 != TEX_F32 && FAST) {
    const uint32_t stride = tex_stride<U8>(W), vadj = tex_vadj<U8>((uint32_t)v * tex_view<U8>(B), stride);
    const f2v tmax = tex_tmax2(W, Hh);
    f2v s_sr = f2s(0.0f);
    float s_ss = 0;
#pragma unroll
    for (int a = 0; a < (NN > 0 ? NN : n); ++a) {
      const float xf = (float)(cx - rad + a * inc);
      const f2v bxy = fma2((f2v){H.h[0], H.h[3]}, f2s(xf), (f2v){H.h[2], H.h[5]}) * f2s(kTexUnit);
      const float bz = __builtin_fmaf(H.h[6], xf, H.h[8]);
      f2v r_sr = f2s(0.0f);
      float r_ss = 0;
#pragma unroll
      for (int b = 0; b < (NN > 0 ? NN : n); ++b) {
        const float sp = tap_u8_fast<U8>(B, vadj, stride, tmax, H.h, bxy, bz, (float)(cy - rad + b * inc));
        const f2v w = wp[a * n + b];
        r_sr = fma2(w, f2s(sp), r_sr);
        const float ws = w.x * sp;
        r_ss = __builtin_fmaf(ws, sp, r_ss);
      }
      s_sr += r_sr; s_ss += r_ss;
    }
    acc[0] = s_sr.x; acc[1] = s_ss; acc[2] = s_sr.y;
  } else {
    float s_src = 0, s_ss = 0, s_rs = 0;
    for (int a = 0; a < n; ++a) {
      const float xf = (float)(cx - rad + a * inc);
      const float bx = __builtin_fmaf(H.h[0], xf, H.h[2]) * kTexUnit;
      const float by = __builtin_fmaf(H.h[3], xf, H.h[5]) * kTexUnit;
      const float bz = __builtin_fmaf(H.h[6], xf, H.h[8]);
      float r_src = 0, r_ss = 0, r_rs = 0;
      for (int b = 0; b < n; ++b) {
        const float yf = (float)(cy - rad + b * inc);
        const float qx = __builtin_fmaf(H.h[1], yf, bx);
        const float qy = __builtin_fmaf(H.h[4], yf, by);
        const float iz = rcp_tap<FAST>(__builtin_fmaf(H.h[7], yf, bz));
        const float sp = sample_src<U8>(B, v, W, Hh, qx, qy, iz);
        const f2v w = wp[a * n + b];
        r_src = __builtin_fmaf(w.x, sp, r_src);
        const float ws = w.x * sp;
        r_ss = __builtin_fmaf(ws, sp, r_ss);
        r_rs = __builtin_fmaf(w.y, sp, r_rs);
      }
      s_src += r_src; s_ss += r_ss; s_rs += r_rs;
    }
    acc[0] = s_src; acc[1] = s_ss; acc[2] = s_rs;
  }
}
// NMAX: the largest side the caller can pass (the neighbour patches are tabulated only up to 3)
template <int U8, int NMAX = 6>
DEV float patch_ncc_tab(const PassConst& pc, const DevBufs& B, int v, const Homog& H, int cx, int cy, int rad, int inc,
                        int n, const float* __restrict__ tw, const float* sm) {
  float a[3];
  if (rcp_range_ok(H, (float)(cx - rad), (float)(cx + rad), (float)(cy - rad), (float)(cy + rad))) {
    switch (n) {
      case 3: tab_taps<U8, true, 3>(pc, B, v, H, cx, cy, rad, inc, n, tw, a); break;
      case 4: tab_taps<U8, true, 4>(pc, B, v, H, cx, cy, rad, inc, n, tw, a); break;
      case 5: tab_taps<U8, true, 5>(pc, B, v, H, cx, cy, rad, inc, n, tw, a); break;
      case 6: tab_taps<U8, true, 6>(pc, B, v, H, cx, cy, rad, inc, n, tw, a); break;
      default: tab_taps<U8, true>(pc, B, v, H, cx, cy, rad, inc, n, tw, a); break;
    }
  } else {
    tab_taps<U8, false>(pc, B, v, H, cx, cy, rad, inc, n, tw, a);
  }
  count_work(B, 0, (unsigned long long)(n * n));
  return ncc_finalize_pre(sm[0], sm[1], sm[2], a[0], a[1], a[2]);
}

// Weak-sweep path statistics (DPE_DIAG & 4; tools/weak_stats.py): per NCC-New,
// the centre patch side and path, the neighbour-patch paths, and per wave the number of distinct
// centre-patch variants its lanes execute one after another.  Off in the product.
#if DPE_WEAK_STATS
// 0 jobs, 1 centre outside, 2..11 n_c histogram (n 0..9, 9 = larger), 12 centre generic (untabulated),
// 13 centre tabulated but slow reciprocal, 14 neighbour box fast, 15 neighbour patches, 16 neighbour
// generic, 17 sum of distinct centre variants per wave call, 18 wave calls, 19 active lanes per wave call
static __device__ unsigned long long g_wstat[24];
DEV void wstat(int k, unsigned long long n = 1) { atomicAdd(&g_wstat[k], n); }
DEV void wstat_variants(int variant) {
  uint64_t rem = __ballot(1);
  const int first = __builtin_ctzll(rem);
  const unsigned long long act = __popcll(rem);
  unsigned long long nv = 0;
  while (rem) {
    const int l = __builtin_ctzll(rem);
    const int V = __shfl(variant, l);
    rem &= ~__ballot(variant == V);
    ++nv;
  }
  if ((int)(threadIdx.x & 63) == first) { wstat(17, nv); wstat(18); wstat(19, act); }
}
#define WSTAT(...) wstat(__VA_ARGS__)
#else
#define WSTAT(...) do {} while (0)
#endif

// ComputeBilateralNCCNew (DPE.cu:557-690) of the tabulated weak pixel (px, py)
template <int U8>
DEV float ncc_new_tab(const PassConst& pc, const DevBufs& B, const WeakTab& T, int px, int py, int v, const float4& pl) {
  const int W = pc.W, Hh = pc.H;
  const Homog H = make_homography(pc, v, pl);
  count_work(B, 1, 0);
  WSTAT(0);
  if (center_outside(pc, v, H, px, py)) { WSTAT(1); return 2.0f; }
  float center_cost = 0.0f, strong_cost = 0.0f;
  int strong_count = 0;
  {   // k = 0: the pixel's own patch
    const short2 np = T.nbl[0];
    if (!(np.x == -1 || np.y == -1)) {
      const float2 nsp = project_h(H, (float)np.x, (float)np.y);
      if (nsp.x < 0 || nsp.y < 0 || nsp.x >= (float)W || nsp.y >= (float)Hh) return 2.0f;
#if DPE_WEAK_STATS
      WSTAT(2 + min(T.n_c, 9));
      if (!T.tab_c) WSTAT(12);
      else if (!rcp_range_ok(H, (float)(np.x - T.rad_c), (float)(np.x + T.rad_c), (float)(np.y - T.rad_c), (float)(np.y + T.rad_c))) WSTAT(13);
      wstat_variants(T.tab_c ? T.n_c : 100 + T.n_c);
#endif
      center_cost = T.tab_c ? patch_ncc_tab<U8>(pc, B, v, H, np.x, np.y, T.rad_c, T.inc_c, T.n_c, T.tc, T.sums)
                            : patch_ncc_generic<U8>(pc, B, v, H, np.x, np.y, T.rc, T.rad_c, T.inc_c);
    }
  }
  // k = 1..8; one range check over the union of the 3x3 neighbour patches selects the fast
  // reciprocal for all of them (it is exact on every tap inside that box)
  const bool nfast = T.nb3 && rcp_range_ok(H, T.nbox[0], T.nbox[1], T.nbox[2], T.nbox[3]);
  if (nfast) WSTAT(14);
#pragma unroll 1
  for (int k = 1; k < DPE_NEIGHBOUR_NUM; ++k) {
    const short2 np = T.nbl[k];
    if (np.x == -1 || np.y == -1) continue;
    const float2 nsp = nfast ? project_h_fast(H, (float)np.x, (float)np.y) : project_h(H, (float)np.x, (float)np.y);
    if (nsp.x < 0 || nsp.y < 0 || nsp.x >= (float)W || nsp.y >= (float)Hh) {
      if (isSet(T.nsv[k], v - 1)) { strong_cost += 2.0f; strong_count++; }
      continue;
    }
    float tc;
    WSTAT(15);
    if (!nfast && !T.tab_n) WSTAT(16);
    if (nfast) {
      float a[3];
      tab_taps<U8, true, 3>(pc, B, v, H, np.x, np.y, T.rad_n, T.inc_n, 3, T.tn + (k - 1) * 18, a);
      count_work(B, 0, 9ull);
      const float* sm = T.sums + 3 * k;
      tc = ncc_finalize_pre(sm[0], sm[1], sm[2], a[0], a[1], a[2]);
    } else {
      tc = T.tab_n ? patch_ncc_tab<U8, 6>(pc, B, v, H, np.x, np.y, T.rad_n, T.inc_n, T.n_n, T.tn + (k - 1) * 18,
                                       T.sums + 3 * k)
                   : patch_ncc_generic<U8>(pc, B, v, H, np.x, np.y, T.rc, T.rad_n, T.inc_n);
    }
    strong_cost += tc; strong_count++;
  }
  if (strong_count == 0) return center_cost;
  strong_cost /= (float)strong_count;
  strong_cost = MINo(strong_cost, 2.0f);
  return (float)(0.25 * (double)center_cost + 0.75 * (double)strong_cost);
}

// LDS floats per weak pixel (lds_layout.h WeakCarve: fixed part, then [8][nv] costs, [nv] sampling
// probabilities, [nv] selected views, [7][nv] hypothesis values; multiple of 4).  At 9 source views a
// pixel takes 636 floats, so four 4-wave workgroups (4 x 40.7 KB) fit a CU's LDS.
using WC = lds::WeakCarveT<true>;
constexpr int kWeakFixed = WC::FIXED;
__host__ __device__ inline int weak_lds_per_pixel(int nv) { return WC::per_pixel(nv); }

// CheckerboardPropagationWeak (DPE.cu:1668-1862) + PlaneHypothesisRefinementWeak (:1120-1212).
// C lanes per pixel, 64/C pixels per wave, blockDim.x/64 waves per workgroup.
template <int U8, int C>
__global__ void __launch_bounds__(256, kTapWaves) k_weak_coop(const PassConst* __restrict__ pcp, DevBufs B, int iter,
                                                   const int* __restrict__ list, const int* __restrict__ nlist_p) {
  extern __shared__ float4 lds4[];
  static_assert(C == 16 || C == 32, "the per-pixel phases give lanes 0..8 the patch sums and lanes 8..15 the alias rows");
  constexpr int P = 64 / C;
  const PassConst& pc = *pcp;
  const int nlist = *nlist_p;
  const int wpb = blockDim.x >> 6;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ps = lane / C, c = lane % C;
  const int W = pc.W, Hh = pc.H, nv = pc.N - 1;
  const DpeCamera& c0 = pc.cams[0];
  const int wgbase = xcd_remap(blockIdx.x, gridDim.x, B.xcd_rows * 16) * wpb * P;
  const int wbase = wgbase + wave * P;
  constexpr bool WGP = true;   // workgroup-wide job pools (false: each wave's own 4 pixels)
  if ((WGP ? wgbase : wbase) >= nlist) return;           // workgroup- (wave-) uniform tail
  const int gi = wbase + ps;
  const bool active = gi < nlist;
  const int center = active ? list[gi] : 0;
  const int x = center % W, y = center / W;
  // ---- LDS carve (per pixel, floats; lds_layout.h WeakCarve)
  const int S = weak_lds_per_pixel(nv);
  float* pb = (float*)lds4 + (size_t)(wave * P + ps) * S;
  float* pw = pb + WC::PW;                               // [108] Old-NCC patch (patch_lds_build)
  float* tcp = pb + WC::TC;                              // centre patch table, pairs [36][2]
  float* tnp = pb + WC::TN;                              // neighbour patch tables, pairs [8][9][2]
  float* sums = pb + WC::SUMS;                           // [9][3]
  float* osum = pb + WC::OSUM;                           // [3] Old-NCC patch sums
  float4* cpl = (float4*)(pb + WC::CPL);                 // [8] candidate planes
  float4* hyp = (float4*)(pb + WC::HYP);                 // [7] refinement hypotheses / final plane
  float* fc = pb + WC::FC;                               // [8] final candidate costs
  int* misc = (int*)(pb + WC::MISC);                     // WC::M_* slots (nsel, header, wnorm, candidate mask, flags)
  short2* nbl = (short2*)(pb + WC::NBL);                 // [9]
  uint32_t* nsv = (uint32_t*)(pb + WC::NSV);             // [9]
  int* alias = (int*)(pb + WC::ALIAS);                   // [8] earlier row with a bitwise-identical plane
  uint8_t* vwl = (uint8_t*)(pb + WC::VWL);               // [32] view weights
  // the pixel's header, read by the lanes of other pixels in the pooled phases: misc[M_RADC / M_INCC /
  // M_NC / M_NB3], the grey level at RC, nbox at NBOX_A[0..2] and NBOX_B; fit plane in hyp[6]
  float* cost = pb + WC::cost(nv);                       // [8][nv]
  float* sp = pb + WC::sp(nv);                           // [nv]
  int* sel_list = (int*)(pb + WC::sel(nv));              // [nv]
  float* hv = pb + WC::hv(nv);                           // [7][nv] hypothesis x selected-view values

  const bool geom = pc.P.geom_consistency;
  const float gf = pc.P.geom_factor;
  const bool fast_old = pc.P.strong_radius == 5 && pc.P.strong_increment == 2;
  WeakTab T;
  T.rad_c = pc.P.strong_radius; T.inc_c = pc.P.strong_increment;
  if (pc.P.use_radius && active) { T.rad_c = B.radius[center]; T.inc_c = MAXo(2, d2i(2.0 * T.rad_c / 5.0)); }
  T.rad_n = pc.P.weak_radius; T.inc_n = pc.P.weak_increment;
  T.n_c = T.rad_c >= 0 ? (2 * T.rad_c) / T.inc_c + 1 : 0;
  T.n_n = T.rad_n >= 0 ? (2 * T.rad_n) / T.inc_n + 1 : 0;
  T.tab_c = T.n_c >= 1 && T.n_c <= 6;
  T.tab_n = T.n_n >= 1 && T.n_n <= 3;
  // plain copies (round 5): references to T's fields under the selects below kept T in scratch
  // (32 B/lane); with the round-5 phase 1 and workgroup pools the copies are as fast and 0 B
  const int rad_c = T.rad_c, inc_c = T.inc_c, n_c = T.n_c, rad_n = T.rad_n, inc_n = T.inc_n, n_n = T.n_n;
  const bool tab_c = T.tab_c, tab_n = T.tab_n;
  T.rc = active ? ref_texel(B.ref, W, Hh, x, y) : 0.0f;
  T.tc = tcp; T.tn = tnp; T.sums = sums; T.nbl = nbl; T.nsv = nsv;
  const short2* nbg = B.nb + (size_t)center * 9;
  // pooled phases: the NCCs of all the workgroup's pixels are dealt round-robin over its lanes, so
  // a job carries its pixel q (0..npx-1, the workgroup's pixels in list order) and pix(q) is that
  // pixel's LDS block.  A pool's jobs fill whole waves first, so a wave with no job left skips
  // the round and its SIMD issues other waves (pools over one wave's 4 pixels left 27-46 of 64
  // lanes idle in the current-plane, refinement and final-cost rounds).  Each pixel's job count
  // sits in its misc[M_POOL]; a job index is decoded by a scan over the pool's pixels.
  const int npx = WGP ? wpb * P : P;
  float* const pool0 = (float*)lds4 + (size_t)(WGP ? 0 : wave * P) * S;
  const int pbase = WGP ? wgbase : wbase;                // list index of the pool's pixel 0
  const int pl_lane = WGP ? (int)threadIdx.x : lane, pl_n = WGP ? (int)blockDim.x : 64;
  auto pool_sync = [&]() { if constexpr (WGP) __syncthreads(); else wave_sync(); };
  auto pix = [&](int q) -> float* { return pool0 + (size_t)q * S; };
  auto pool_cnt = [&](int q) -> int { return ((const int*)(pix(q) + WC::MISC))[WC::M_POOL]; };
  auto pool_total = [&]() -> int { int t = 0; for (int q = 0; q < npx; ++q) t += pool_cnt(q); return t; };
  auto pool_decode = [&](int j, int& q, int& r) { q = 0; for (int cc; j >= (cc = pool_cnt(q)); ++q) j -= cc; r = j; };
  auto pool_stat_g = [&](int k, int jobs) {   // DPE_DIAG & 16: jobs, wave rounds with a job, waves
#if DPE_POOL_STATS
    if (pl_lane == 0) {
      atomicAdd(&g_pool[k][0], (unsigned long long)jobs);
      atomicAdd(&g_pool[k][1], (unsigned long long)((jobs + 63) / 64));
      atomicAdd(&g_pool[k][2], (unsigned long long)(pl_n / 64));
    }
#else
    (void)k; (void)jobs;
#endif
  };
  auto tab_of = [&](int q) -> WeakTab {
    const float* qb = pix(q);
    const int* h = (const int*)(qb + WC::MISC);
    WeakTab t;
    t.rad_c = h[WC::M_RADC]; t.inc_c = h[WC::M_INCC]; t.n_c = h[WC::M_NC]; t.nb3 = h[WC::M_NB3] != 0;
    t.rad_n = T.rad_n; t.inc_n = T.inc_n; t.n_n = T.n_n; t.tab_n = T.tab_n;
    t.tab_c = t.n_c >= 1 && t.n_c <= 6;
    t.rc = qb[WC::RC];
    t.nbox[0] = qb[WC::NBOX_A]; t.nbox[1] = qb[WC::NBOX_A + 1]; t.nbox[2] = qb[WC::NBOX_A + 2]; t.nbox[3] = qb[WC::NBOX_B];
    t.tc = qb + WC::TC; t.tn = qb + WC::TN; t.sums = qb + WC::SUMS;
    t.nbl = (const short2*)(qb + WC::NBL); t.nsv = (const uint32_t*)(qb + WC::NSV);
    return t;
  };
  // phase 1 by patch rows (the common case: centre side <= 6, 3x3 neighbour patches, C = 16)
  const bool rows1 = C == 16 && tab_c && tab_n && n_n == 3;

  PHASE_BEGIN();
  // ---- phase 1: neighbours, weight tables, Old-NCC patch, candidate rows
  if (active) {
    if (fast_old) patch_lds_build<C>(pw, pc, B, x, y, c);
    for (int k = c; k < 9; k += C) {
      const short2 np = nbg[k];
      nbl[k] = np;
      nsv[k] = (np.x == -1 || np.y == -1) ? 0u : B.sel[np.x + np.y * W];
    }
    const float ss = pc.P.sigma_spatial, sc = pc.P.sigma_color;
    if (rows1) {
      // the tables by patch rows with their reference sums (the order of phase 1b's loop): lanes
      // 0..n_c-1 a centre row each (row sums to RSUM, added in row order in phase 1b), lanes 8..15
      // a 3x3 neighbour patch each (sums complete); a lane's texel loads are issued together
      if (c < n_c) {
        const short2 np = nbg[0];
        if (!(np.x == -1 || np.y == -1)) {
          const int i = -rad_c + c * inc_c;
          float rp[6];
#pragma unroll
          for (int b = 0; b < 6; ++b) rp[b] = b < n_c ? ref_texel(B.ref, W, Hh, np.x + i, np.y - rad_c + b * inc_c) : 0.0f;
          float r_ref = 0, r_rr = 0, r_w = 0;
#pragma unroll
          for (int b = 0; b < 6; ++b) {
            if (b >= n_c) break;
            const float w = bilateral_weight(i, -rad_c + b * inc_c, rp[b], T.rc, ss, sc);
            const float wr = w * rp[b];
            tcp[2 * (c * n_c + b)] = w; tcp[2 * (c * n_c + b) + 1] = wr;
            r_ref = r_ref + wr;
            r_rr = __builtin_fmaf(wr, rp[b], r_rr);
            r_w = r_w + w;
          }
          float* rs3 = pb + WC::RSUM + 3 * c;
          rs3[0] = r_ref; rs3[1] = r_rr; rs3[2] = r_w;
        }
      } else if (c >= 8) {
        const int k = c - 7;
        const short2 np = nbg[k];
        if (!(np.x == -1 || np.y == -1)) {
          float rp[9];
#pragma unroll
          for (int t = 0; t < 9; ++t) rp[t] = ref_texel(B.ref, W, Hh, np.x - rad_n + (t / 3) * inc_n, np.y - rad_n + (t % 3) * inc_n);
          float* tp = tnp + (k - 1) * 18;
          float a_ref = 0, a_rr = 0, a_w = 0;
#pragma unroll
          for (int a = 0; a < 3; ++a) {
            float r_ref = 0, r_rr = 0, r_w = 0;
#pragma unroll
            for (int b = 0; b < 3; ++b) {
              const float w = bilateral_weight(-rad_n + a * inc_n, -rad_n + b * inc_n, rp[a * 3 + b], T.rc, ss, sc);
              const float wr = w * rp[a * 3 + b];
              tp[2 * (a * 3 + b)] = w; tp[2 * (a * 3 + b) + 1] = wr;
              r_ref = r_ref + wr;
              r_rr = __builtin_fmaf(wr, rp[a * 3 + b], r_rr);
              r_w = r_w + w;
            }
            a_ref += r_ref; a_rr += r_rr; a_w += r_w;
          }
          ncc_pre(a_ref, a_rr, a_w, sums[3 * k], sums[3 * k + 1], sums[3 * k + 2]);
        }
      }
    }
    const int ntc = tab_c && !rows1 ? n_c * n_c : 0, ntn = tab_n && !rows1 ? n_n * n_n : 0;
    for (int t = c; t < ntc + 8 * ntn; t += C) {
      int k, tt, n, rad, inc;
      if (t < ntc) { k = 0; tt = t; n = n_c; rad = rad_c; inc = inc_c; }
      else { k = 1 + (t - ntc) / ntn; tt = (t - ntc) % ntn; n = n_n; rad = rad_n; inc = inc_n; }
      const short2 np = nbg[k];
      if (np.x == -1 || np.y == -1) continue;
      const int i = -rad + (tt / n) * inc, j = -rad + (tt % n) * inc;
      const float rp = ref_texel(B.ref, W, Hh, np.x + i, np.y + j);
      const float w = bilateral_weight(i, j, rp, T.rc, ss, sc);
      float* dst = k == 0 ? tcp + 2 * tt : tnp + 2 * ((k - 1) * 9 + tt);
      dst[0] = w; dst[1] = w * rp;
    }
    for (int i = c; i < 8; i += C) {
      const short2 np = nbg[i + 1];
      const bool fl = !(np.x == -1 || np.y == -1) && B.weak[np.x + np.y * W] == DPE_STRONG;
      misc[WC::M_FLAGS + i] = fl ? 1 : 0;
      if (fl) cpl[i] = B.planes[np.x + np.y * W];
      else for (int v = 0; v < nv; ++v) cost[i * nv + v] = (i == 0 && v == 0) ? 2.0f : 0.0f;
    }
  }
  wave_sync();
  PHASE(0);
  // union box of the neighbour patches (k = 1..8) for the one-check fast path of ncc_new_tab
  T.nb3 = false;
  if (active && T.tab_n && T.n_n == 3) {
    int x0 = 0x7FFFFFFF, x1 = -0x7FFFFFFF, y0 = 0x7FFFFFFF, y1 = -0x7FFFFFFF;
    for (int k = 1; k < DPE_NEIGHBOUR_NUM; ++k) {
      const short2 np = nbl[k];
      if (np.x == -1 || np.y == -1) continue;
      x0 = min(x0, (int)np.x); x1 = max(x1, (int)np.x); y0 = min(y0, (int)np.y); y1 = max(y1, (int)np.y);
    }
    if (x0 <= x1) {
      T.nb3 = true;
      T.nbox[0] = (float)(x0 - T.rad_n); T.nbox[1] = (float)(x1 + T.rad_n);
      T.nbox[2] = (float)(y0 - T.rad_n); T.nbox[3] = (float)(y1 + T.rad_n);
    }
  }
  // ---- phase 1b: reference sums of every tabulated patch (tap order of patch_ncc_generic)
  if (active) {
    if (c == C - 2) {
      misc[WC::M_RADC] = T.rad_c; misc[WC::M_INCC] = T.inc_c; misc[WC::M_NC] = T.n_c; misc[WC::M_NB3] = T.nb3 ? 1 : 0;
      pb[WC::NBOX_A] = T.nbox[0]; pb[WC::NBOX_A + 1] = T.nbox[1]; pb[WC::NBOX_A + 2] = T.nbox[2]; pb[WC::NBOX_B] = T.nbox[3];
      pb[WC::RC] = T.rc;
    }
    if (rows1 && c == 0) {   // the centre patch's row sums in row order
      const short2 np = nbl[0];
      if (!(np.x == -1 || np.y == -1)) {
        float a_ref = 0, a_rr = 0, a_w = 0;
        for (int a = 0; a < n_c; ++a) {
          const float* rs3 = pb + WC::RSUM + 3 * a;
          a_ref += rs3[0]; a_rr += rs3[1]; a_w += rs3[2];
        }
        ncc_pre(a_ref, a_rr, a_w, sums[0], sums[1], sums[2]);
      }
    }
    for (int k = c; k < 9; k += C) {
      const short2 np = nbl[k];
      if (rows1 || np.x == -1 || np.y == -1 || !(k == 0 ? tab_c : tab_n)) continue;
      const int n = k == 0 ? n_c : n_n, rad = k == 0 ? rad_c : rad_n, inc = k == 0 ? inc_c : inc_n;
      const float* tp = k == 0 ? tcp : tnp + (k - 1) * 18;
      float a_ref = 0, a_rr = 0, a_w = 0;
      for (int a = 0; a < n; ++a) {
        float r_ref = 0, r_rr = 0, r_w = 0;
        for (int b = 0; b < n; ++b) {
          const float rp = ref_texel(B.ref, W, Hh, np.x - rad + a * inc, np.y - rad + b * inc);
          const float w = tp[2 * (a * n + b)], wr = tp[2 * (a * n + b) + 1];
          r_ref = r_ref + wr;
          r_rr = __builtin_fmaf(wr, rp, r_rr);
          r_w = r_w + w;
        }
        a_ref += r_ref; a_rr += r_rr; a_w += r_w;
      }
      ncc_pre(a_ref, a_rr, a_w, sums[3 * k], sums[3 * k + 1], sums[3 * k + 2]);
    }
    if (c == C - 1 && fast_old) patch_lds_pre(pw, osum[0], osum[1], osum[2]);
    // bitwise-identical neighbour planes share one cost vector: alias = first earlier flagged row
    // with the same plane (lanes 8..15; lanes 0..8 build the sums above)
    for (int i = c - 8; i >= 0 && i < 8; i += C) {
      int a = i;
      if (misc[WC::M_FLAGS + i]) {
        const float4 me = cpl[i];
        for (int t = 0; t < i; ++t)
          if (misc[WC::M_FLAGS + t] && __float_as_uint(cpl[t].x) == __float_as_uint(me.x) &&
              __float_as_uint(cpl[t].y) == __float_as_uint(me.y) && __float_as_uint(cpl[t].z) == __float_as_uint(me.z) &&
              __float_as_uint(cpl[t].w) == __float_as_uint(me.w)) { a = t; break; }
      }
      alias[i] = a;
    }
  }
  wave_sync();
  PHASE(1);
  // ---- phase 2: candidate cost vectors, jobs (unique flagged neighbour plane, view)
  if (active && c == 0) {
    uint32_t um = 0;
    for (int i = 0; i < 8; ++i) if (misc[WC::M_FLAGS + i] && alias[i] == i) um |= 1u << i;
    misc[WC::M_CMASK] = (int)um;
    misc[WC::M_POOL] = __builtin_popcount(um);
  }
  if (!active && c == 0) misc[WC::M_POOL] = 0;
  pool_sync();
  {
    const int Sj = pool_total();
    int q, r;
    pool_stat_g(2, Sj * nv);
    // view-major: the lanes of one round gather from the same source images
    for (int j = pl_lane; j < Sj * nv; j += pl_n) {
      pool_decode(j % Sj, q, r);
      const int v = j / Sj + 1;
      float* qb = pix(q);
      uint32_t m = (uint32_t)((const int*)(qb + WC::MISC))[WC::M_CMASK];
      for (; r > 0; --r) m &= m - 1;
      const int i = __builtin_ctz(m);
      const int cq = list[pbase + q];
      (qb + WC::cost(nv))[i * nv + v - 1] = ncc_new_tab<U8>(pc, B, tab_of(q), cq % W, cq / W, v, ((const float4*)(qb + WC::CPL))[i]);
    }
  }
  pool_sync();
  PHASE(2);
  if (active)
    for (int i = c; i < 8; i += C)
      if (misc[WC::M_FLAGS + i] && alias[i] != i)
        for (int v = 0; v < nv; ++v) cost[i * nv + v] = cost[alias[i] * nv + v];
  wave_sync();
  PHASE(3);
  // ---- phase 3: per-view probabilities with the deformable-neighbour priors (DPE.cu:1768-1790)
  const float cost_threshold = (float)(0.8 * (double)d_expf((float)(iter * iter) / (-90.0f)));
  if (active) {
    auto cst = [&](int j, int i) -> float { return cost[j * nv + i]; };
    for (int v = c; v < nv; v += C) {
      float prior = 0.0f;
      for (int i = 0; i < 8; ++i) {
        const short2 np = nbl[i + 1];
        if (np.x == -1 || np.y == -1) continue;
        prior += isSet(nsv[i + 1], v) == 1 ? 0.9f : 0.1f;
      }
      sp[v] = view_prob_raw(cst, v, cost_threshold) * prior;
    }
  }
  wave_sync();
  PHASE(4);
  Rng rs;
  rng_init(rs, (uint32_t)center, pc.seed32, STREAM_ITER_BASE + 4 * iter + 2, pc.salt);
  view_sample_coop(sp, (int*)hv, nv, c, C, active, rs, vwl, B.vw + (size_t)center * DPE_MAX_IMAGES);
  uint32_t tsv = 0; float wnorm = 0.0f;
  if (active && c == 0) {
    rng_seek(rs, 15);
    int ns = 0;
    for (int i = 0; i < nv; ++i) if (vwl[i] > 0) { setBit(tsv, i); wnorm += vwl[i]; sel_list[ns++] = i; }
    misc[WC::M_NSEL] = ns;
    misc[WC::M_WNORM] = __float_as_int(wnorm);
    const float4 f6 = B.fit_plane[center];
    hyp[6] = f6;
    misc[WC::M_POOL] = ((f6.x == 0 && f6.y == 0 && f6.z == 0) ? 1 : 2) * ns;   // current (+ fit) plane jobs
  }
  if (!active && c == 0) misc[WC::M_POOL] = 0;
  pool_sync();
  PHASE(5);
  const int nsel = active ? misc[WC::M_NSEL] : 0;
  const float wn = active ? __int_as_float(misc[WC::M_WNORM]) : 1.0f;
  const float4 cur = active ? B.planes[center] : make_float4(0, 0, 0, 1);
  const float4 fp = active ? B.fit_plane[center] : make_float4(0, 0, 0, 0);
  const bool has_fit = !(fp.x == 0 && fp.y == 0 && fp.z == 0);
  // ---- phase 4: current plane and fit plane over the selected views; final candidate costs
  // pixel q's hyp_cost term (DPE.cu:1140-1150) (view v, plane pl) into its hv row
  auto hyp_val_q = [&](int q, int v, const float4& pl) __attribute__((always_inline)) -> float {
    const int cq = list[pbase + q];
    const int qx = cq % W, qy = cq / W;
    const float cn = ncc_new_tab<U8>(pc, B, tab_of(q), qx, qy, v, pl);
    return geom ? cn + gf * geom_cost(pc, B, qx, qy, v, pl) : cn;
  };
  {
    const int tot = pool_total();
    pool_stat_g(3, tot);
    int q, r;
    for (int j = pl_lane; j < tot; j += pl_n) {
      pool_decode(j, q, r);
      float* qb = pix(q);
      const int ns = ((const int*)(qb + WC::MISC))[WC::M_NSEL];
      const int h = r / ns, k = r % ns;
      const int v = ((const int*)(qb + WC::sel(nv)))[k] + 1;
      (qb + WC::hv(nv))[h * nv + k] = hyp_val_q(q, v, h ? ((const float4*)(qb + WC::HYP))[6] : B.planes[list[pbase + q]]);
    }
  }
  PHASE(12);   // (phase 6 from here: the final candidate costs)
  if (active) {
    for (int i = c; i < 8; i += C) {
      const bool fl = misc[WC::M_FLAGS + i] != 0;
      const float3 fwi = (geom && fl) ? geom_point(pc, x, y, cpl[i]) : make_float3(0.0f, 0.0f, 0.0f);
      float f = 0.0f;
      for (int j = 0; j < nv; ++j) {
        const int w = vwl[j];
        if (w > 0) {
          if (geom) {
            if (fl) f += w * (cost[i * nv + j] + gf * geom_cost_at(pc, B, x, y, j + 1, fwi));
            else f += w * (cost[i * nv + j] + gf * 3.0f);
          } else {
            f += w * cost[i * nv + j];
          }
        }
      }
      fc[i] = f / wn;
    }
  }
  pool_sync();   // the current / fit-plane values of every pool pixel are in
  PHASE(6);
  // ---- serial: propagation acceptance, fit plane, refinement hypotheses (DPE.cu:1792-1843, 1120-1170)
  float cost_now = 0.0f, cost_written = 0.0f, depth_now = 0.0f;
  float4 pnow = cur;
  const float dmin = pc.P.depth_min, dmax = pc.P.depth_max;
  const float pert = (float)(0.02f * 3.14159265358979323846);
  // lanes 1..4 evaluate the refinement draws (refine_draws: stream words 15.. after the view
  // sampling) while lane 0 runs the acceptance; lane 0 then finishes the hypotheses from them
  float* rnd = pb + WC::RND;
  if (active && has_fit && c >= 1 && c <= 4) {
    const RefineDraws d = refine_draws(rs, 15u);
    if (c == 1) { rnd[0] = d.u_depth; rnd[1] = d.n[0]; rnd[2] = d.n[1]; rnd[3] = d.n[2]; rnd[4] = d.u_pert; }
    else refine_angle(rs, d.w_angles, c - 2, pert, &rnd[5 + 2 * (c - 2)], &rnd[6 + 2 * (c - 2)]);
  }
  if (active && c == 0) {
    int mi = 0; float mcost = fc[0];
    for (int i = 1; i < 8; ++i) if (fc[i] <= mcost) { mcost = fc[i]; mi = i; }
    for (int k = 0; k < nsel; ++k) cost_now += vwl[sel_list[k]] * hv[k];
    cost_now /= wnorm;
    cost_written = cost_now;
    depth_now = depth_from_plane(c0, cur, x, y);
    if (misc[WC::M_FLAGS + mi]) {
      const float4 cand_pl = cpl[mi];
      const float db = depth_from_plane(c0, cand_pl, x, y);
      if (db >= dmin && db <= dmax && fc[mi] < cost_now) {
        depth_now = db; pnow = cand_pl; cost_now = fc[mi]; B.sel[center] = tsv;
      }
    }
    if (has_fit) {
      float tc = 0.0f;
      for (int k = 0; k < nsel; ++k) tc += vwl[sel_list[k]] * hv[nv + k];
      tc /= wnorm;
      const float db = depth_from_plane(c0, fp, x, y);
      if (db >= dmin && db <= dmax && tc < cost_now) { depth_now = db; pnow = fp; cost_now = tc; }
    }
  }
  wave_sync();
  if (active && c == 0 && has_fit) {
    const float depth_rand = rnd[0] * (dmax - dmin) + dmin;
    const float4 prand = random_normal_from(c0, x, y, rnd + 1, depth_now);
    const float dminp = (1 - 0.02f) * depth_now, dmaxp = (1 + 0.02f) * depth_now;
    const float depth_perturbed = rnd[4] * (dmaxp - dminp) + dminp;
    const float4 ppert = perturbed_normal_from(c0, x, y, pnow, rnd + 5);
    float4 h0 = pnow, h1 = prand, h2 = prand, h3 = ppert, h4 = pnow;
    h0.w = dist2origin(c0, x, y, depth_rand, h0);
    h1.w = dist2origin(c0, x, y, depth_now, h1);
    h2.w = dist2origin(c0, x, y, depth_rand, h2);
    h3.w = dist2origin(c0, x, y, depth_now, h3);
    h4.w = dist2origin(c0, x, y, depth_perturbed, h4);
    hyp[0] = h0; hyp[1] = h1; hyp[2] = h2; hyp[3] = h3; hyp[4] = h4;
  }
  if (c == 0) misc[WC::M_POOL] = active && has_fit ? 5 * nsel : 0;
  pool_sync();
  PHASE(7);
  // ---- phase 5: refinement NCCs, jobs (hypothesis, selected view)
  {
    const int tot = pool_total();
    pool_stat_g(4, tot);
    int q, r;
    for (int j = pl_lane; j < tot; j += pl_n) {
      pool_decode(j, q, r);
      float* qb = pix(q);
      const int ns = ((const int*)(qb + WC::MISC))[WC::M_NSEL];
      const int h = r / ns, k = r % ns;
      const int v = ((const int*)(qb + WC::sel(nv)))[k] + 1;
      (qb + WC::hv(nv))[(2 + h) * nv + k] = hyp_val_q(q, v, ((const float4*)(qb + WC::HYP))[h]);
    }
  }
  pool_sync();
  PHASE(8);
  // ---- serial: sequential acceptance + write-back (DPE.cu:1190-1207, 1831-1843)
  if (active && c == 0) {
    if (has_fit) {
      for (int h = 0; h < 5; ++h) {
        const float4 tp = hyp[h];
        float tc = 0.0f;
        for (int k = 0; k < nsel; ++k) tc += vwl[sel_list[k]] * hv[(2 + h) * nv + k];
        tc /= wnorm;
        const float db = depth_from_plane(c0, tp, x, y);
        if (db >= dmin && db <= dmax && tc < cost_now) { depth_now = db; pnow = tp; cost_now = tc; }
      }
    }
    float4 fin = cur;
    if (pc.P.state == DPE_REFINE_INIT) {
      if ((double)cost_now < (double)cost_written - 0.1) { fin = pnow; B.planes[center] = pnow; }
    } else {
      fin = pnow;
      B.planes[center] = pnow;
    }
    hyp[5] = fin;
  }
  if (c == 0) misc[WC::M_POOL] = active ? nsel : 0;
  pool_sync();
  PHASE(9);
  // ---- phase 6: the stored cost is the Old NCC of the final plane (DPE.cu:1845-1861)
  {
    const int tot = pool_total();
    pool_stat_g(5, tot);
    int q, r;
    for (int j = pl_lane; j < tot; j += pl_n) {
      pool_decode(j, q, r);
      float* qb = pix(q);
      const int cq = list[pbase + q];
      const int v = ((const int*)(qb + WC::sel(nv)))[r] + 1;
      (qb + WC::hv(nv))[r] = ncc_old_any<U8>(fast_old, qb + WC::PW, qb[WC::OSUM], qb[WC::OSUM + 1], qb[WC::OSUM + 2], cq % W,
                                                   cq / W, pc, B, v, ((const float4*)(qb + WC::HYP))[5]);
    }
  }
  pool_sync();
  PHASE(10);
  if (active && c == 0) {
    float c2 = 0.0f;
    for (int k = 0; k < nsel; ++k) c2 += vwl[sel_list[k]] * hv[k];
    B.costs[center] = c2 / wnorm;
  }
  PHASE(11);
  PHASE_END(1);
}

}  // namespace dpe
