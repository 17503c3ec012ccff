// fusion.cpp — RunFusion (DPE.cpp:1220-1370, the variant RunDPEPipeline calls at main.cpp:579) and
// ExportPointCloud (DPE.cpp:532-572) over the pipeline's final per-image maps.
//
// Split in two:
//  * the per-(pixel, source view) projection tests, independent of everything else, run through a
//    dpe_fusion_fn (include/dpe_host.h): by default the HIP kernel behind dpe_fusion_candidates
//    (csrc/pass_fusion.h); tests inject the CPU restatement (oracle/);
//  * the order-dependent remainder runs here in the reference's serial order: problems in pair.txt
//    order, pixels row-major, source views in pair.txt order; skip masked / blocked reference
//    pixels, skip candidates on masked source pixels, angle test, consistency weight, colour, and
//    the masks of the source pixels a fused point used.
// The reference reads depths.dmb / normals.dmb / weak.bin back from disk; here the same final maps
// come from the pipeline's state.  Arithmetic is single precision in the reference's expression
// order; its host code is built with -ffast-math -march=native, whose contractions are not
// reproducible, so agreement with the reference binary is unpinned.
#include "host.h"

#include <cmath>
#include <cstring>
#include <fstream>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <thread>
#include <unordered_map>

namespace dpe_host {

// RunFusion's serial part (DPE.cpp:1286-1367) over the candidates of `fn`.
//
// Round 6, three changes that keep every result (tests/test_fusion.py: the PLY bit for bit):
//  * the next image's candidates are fetched on a worker thread while this image is fused (double
//    buffer; only one `fn` call runs at a time, and the fusion itself makes no `fn` call);
//  * the candidate buffers are allocated once, uninitialised (`fn` writes every index, and every
//    value the walk reads);
//  * what in the reference's loop does not depend on the masks -- the angle test (acos) and the
//    consistency weight (exp) of every candidate -- is evaluated first on host threads, with the
//    same float expressions, into a per-pixel bit set of the candidates that pass and their weights;
//    the serial walk then visits only those, in ascending view order, and adds the same weights in
//    the same order (the masks it tests and sets are exactly the reference's).
namespace {
int fusion_threads() {
  unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  if (const char* e = getenv("OMP_NUM_THREADS")) { const int v = atoi(e); if (v > 0) hw = std::min(hw, (unsigned)v); }
  return (int)std::min(16u, hw);
}
}  // namespace

bool run_fusion(std::vector<FusionView>& views, dpe_fusion_fn fn, void* user, std::vector<FusedPoint>& cloud,
                std::string& err) {
  const int n = (int)views.size();
  std::unordered_map<int, int> index;
  for (int i = 0; i < n; ++i) index.emplace(views[i].image_id, i);
  auto idx_of = [&](int id) { auto it = index.find(id); return it == index.end() ? 0 : it->second; };   // operator[]
  std::vector<DpeFusionView> dv(n);
  for (int i = 0; i < n; ++i) {
    dv[i] = views[i].view;
    views[i].mask.assign((size_t)views[i].view.width * views[i].view.height, 0);
  }
  std::vector<std::vector<int>> srcs(n);
  std::vector<int> refs(n);
  size_t cap = 1;
  for (int i = 0; i < n; ++i) {
    refs[i] = idx_of(views[i].image_id);
    for (int id : views[i].src_ids) srcs[i].push_back(idx_of(id));
    if (srcs[i].size() > 32) { err = "fusion: more than 32 source views"; return false; }
    const DpeFusionView& R = views[refs[i]].view;
    cap = std::max(cap, (size_t)R.width * R.height * srcs[i].size());
  }
  struct Cand {
    std::unique_ptr<int32_t[]> idx;
    std::unique_ptr<float[]> val;
    int rc = 0;
  };
  Cand buf[2];
  // page-locked when the runtime allows (the candidate copies are ~16 B per (pixel, source view))
  struct Pin {
    void* p = nullptr;
    void pin(void* q, size_t n) { if (dpe_host_pin(q, n) == DPE_OK) p = q; }
    ~Pin() { if (p) dpe_host_unpin(p); }
  } pins[4];
  // DPE_FUSION_PROFILE=1: seconds pinning, waiting for candidates, in the terms, the walk, the points
  static const bool prof = [] { const char* e = getenv("DPE_FUSION_PROFILE"); return e && atoi(e) != 0; }();
  // DPE_FUSION_PIN=0: pageable candidate buffers (A/B of the pinning)
  static const bool pin = [] { const char* e = getenv("DPE_FUSION_PIN"); return !(e && atoi(e) == 0); }();
  double t_wait = 0, t_terms = 0, t_walk = 0, t_points = 0, t_pin = 0;
  auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  {
    const double tp = now();
    for (int k = 0; k < 2; ++k) {
      buf[k].idx.reset(new int32_t[cap]);
      buf[k].val.reset(new float[cap * 3]);
      if (pin) {
        pins[2 * k].pin(buf[k].idx.get(), cap * sizeof(int32_t));
        pins[2 * k + 1].pin(buf[k].val.get(), cap * 3 * sizeof(float));
      }
    }
    t_pin = now() - tp;
  }
  auto fetch = [&](int i, Cand* b) {
    const int ns = (int)srcs[i].size();
    b->rc = ns > 0 ? fn(user, dv.data(), n, refs[i], srcs[i].data(), ns, b->idx.get(), b->val.get()) : 0;
  };
  const int nt = fusion_threads();
  // per image: the candidates whose angle test passes (bit j of pass[p]) and their weights
  struct Terms {
    std::vector<uint32_t> pass;
    std::vector<float> wgt;
  };
  Terms terms[2];
  auto make_terms = [&](int i, const Cand* b, Terms* tm, int threads) {   // DPE.cpp:1318-1343 without the masks
    const FusionView& R = views[refs[i]];
    const int ns = (int)srcs[i].size();
    const size_t L = (size_t)R.view.width * R.view.height;
    tm->pass.assign(L, 0u);
    tm->wgt.resize(L * (size_t)std::max(ns, 1));
    if (ns == 0) return;
    const int32_t* cidx = b->idx.get();
    const float* cval = b->val.get();
    uint32_t* pass = tm->pass.data();
    float* wgt = tm->wgt.data();
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t)
      pool.emplace_back([&, t]() {
        const size_t lo = L * t / threads, hi = L * (t + 1) / threads;
        for (size_t p = lo; p < hi; ++p) {
          if (!(R.view.depth[p] > 0.0f)) continue;
          if (!R.block.empty() && R.block[p] < 128) continue;     // skipped by the walk in any case
          uint32_t m = 0;
          for (int j = 0; j < ns; ++j) {
            if (cidx[p * ns + j] < 0) continue;
            const float* v = cval + (p * ns + j) * 3;
            float angle = std::acos(v[2]);                 // GetAngle (DPE.cpp:1208-1217)
            if (angle != angle) angle = 0.0f;
            if (angle < 0.174533f) {                       // reproj < 2, rel < 0.01 tested by the candidates
              const float tmp_index = v[0] + 200 * v[1] + angle * 10;
              wgt[p * ns + j] = std::exp(-tmp_index);
              m |= 1u << j;
            }
          }
          pass[p] = m;
        }
      });
    for (auto& th : pool) th.join();
  };
  // the fused pixels of one image in walk order: pixel, depth, the candidates it used (bit j)
  struct Fused {
    uint32_t p, used;
    float depth;
  };
  std::vector<Fused> fused;
  std::thread worker;
  double t0 = now();
  fetch(0, &buf[0]);
  if (buf[0].rc == 0) make_terms(0, &buf[0], &terms[0], nt);
  t_terms += now() - t0;
  for (int i = 0; i < n; ++i) {
    t0 = now();
    if (worker.joinable()) worker.join();
    t_wait += now() - t0;
    const Cand& b = buf[i & 1];
    if (b.rc != 0) {
      err = "fusion candidates failed (" + std::to_string(b.rc) + ")";
      return false;
    }
    // the next image's candidates and terms on the worker (its own threads) while this one is walked
    if (i + 1 < n)
      worker = std::thread([&, i]() {
        Cand* nb = &buf[(i + 1) & 1];
        fetch(i + 1, nb);
        if (nb->rc == 0) make_terms(i + 1, nb, &terms[(i + 1) & 1], std::max(1, nt - 1));
      });
    FusionView& R = views[refs[i]];
    const int cols = R.view.width, rows = R.view.height;
    const std::vector<int>& src = srcs[i];
    const int ns = (int)src.size();   // <= DPE_MAX_IMAGES - 1: one bit per view
    const int32_t* cidx = b.idx.get();
    const uint32_t* pass = terms[i & 1].pass.data();
    const float* wgt = terms[i & 1].wgt.data();
    t0 = now();
    uint8_t* smask[32];
    for (int j = 0; j < ns; ++j) smask[j] = views[src[j]].mask.data();
    fused.clear();
    for (int r = 0; r < rows; ++r)
      for (int c = 0; c < cols; ++c) {
        const size_t p = (size_t)r * cols + c;
        // no candidate passes the angle test (or the pixel is blocked / has no depth): the
        // reference's loop finds num_consistent = 0 and keeps nothing, whatever the masks say
        if (!pass[p]) continue;
        if (R.mask[p] == 1) continue;
        const float ref_depth = R.view.depth[p];
        int num_consistent = 0;
        uint32_t used = 0;
        float dyn = 0.0f;
        for (uint32_t m = pass[p]; m; m &= m - 1) {
          const int j = __builtin_ctz(m);
          const int32_t sp = cidx[p * ns + j];
          if (smask[j][sp] == 1) continue;
          used |= 1u << j;
          dyn += wgt[p * ns + j];
          num_consistent++;
        }
        const float factor = R.weak[p] == DPE_WEAK ? 0.45f : 0.3f;
        if (num_consistent >= 1 && dyn > factor * num_consistent) {
          for (uint32_t m = used; m; m &= m - 1) {
            const int j = __builtin_ctz(m);
            smask[j][cidx[p * ns + j]] = 1;
          }
          fused.push_back(Fused{(uint32_t)p, used, ref_depth});
        }
      }
    t_walk += now() - t0;
    // colours and 3-D points of the fused pixels (DPE.cpp:1345-1366): they read only the images'
    // colours, which nothing writes, so they run on host threads, each point at its walk position
    t0 = now();
    const size_t base = cloud.size(), nf = fused.size();
    cloud.resize(base + nf);
    {
      std::vector<std::thread> pool;
      const int th = (int)std::min<size_t>((size_t)nt, std::max<size_t>(1, nf / 4096));
      for (int t = 0; t < th; ++t)
        pool.emplace_back([&, t]() {
          for (size_t k = nf * t / th; k < nf * (t + 1) / th; ++k) {
            const Fused& f = fused[k];
            const size_t p = f.p;
            float col[3] = {(float)R.bgr[3 * p], (float)R.bgr[3 * p + 1], (float)R.bgr[3 * p + 2]};
            for (uint32_t m = f.used; m; m &= m - 1) {
              const int j = __builtin_ctz(m);
              const size_t sp = (size_t)cidx[p * ns + j];
              const FusionView& S = views[src[j]];
              col[0] += S.bgr[3 * sp];
              col[1] += S.bgr[3 * sp + 1];
              col[2] += S.bgr[3 * sp + 2];
            }
            const int num_consistent = __builtin_popcount(f.used);
            for (float& x : col) x /= (num_consistent + 1);
            cloud[base + k] = fusion_point((int)(p % cols), (int)(p / cols), f.depth, R.view.cam, col);
          }
        });
      for (auto& th2 : pool) th2.join();
    }
    t_points += now() - t0;
  }
  if (worker.joinable()) worker.join();
  if (prof)
    fprintf(stderr, "fusion: %d images, buffers + pinning %.3f s, wait for candidates + terms %.3f s, first image "
            "%.3f s, serial walk %.3f s, points %.3f s, %zu points\n", n, t_pin, t_wait, t_terms, t_walk, t_points,
            cloud.size());
  return true;
}

// Get3DPointonWorld (DPE.cpp:1170-1194), the point a fused pixel contributes
FusedPoint fusion_point(int x, int y, float depth, const DpeCamera& cam, const float* bgr) {
  float px = depth * (x - cam.K[2]) / cam.K[0];
  float py = depth * (y - cam.K[5]) / cam.K[4];
  float pz = depth;
  const float tx = cam.R[0] * px + cam.R[3] * py + cam.R[6] * pz;
  const float ty = cam.R[1] * px + cam.R[4] * py + cam.R[7] * pz;
  const float tz = cam.R[2] * px + cam.R[5] * py + cam.R[8] * pz;
  const float cx = -(cam.R[0] * cam.t[0] + cam.R[3] * cam.t[1] + cam.R[6] * cam.t[2]);
  const float cy = -(cam.R[1] * cam.t[0] + cam.R[4] * cam.t[1] + cam.R[7] * cam.t[2]);
  const float cz = -(cam.R[2] * cam.t[0] + cam.R[5] * cam.t[1] + cam.R[8] * cam.t[2]);
  return FusedPoint{tx + cx, ty + cy, tz + cz, bgr[0], bgr[1], bgr[2]};
}

// ExportPointCloud (DPE.cpp:532-572): binary little-endian PLY, xyz float + BGR uchar
bool export_point_cloud(const std::string& path, const std::vector<FusedPoint>& cloud, std::string& err) {
  std::ofstream out(path, std::ios::binary);
  if (!out) { err = "cannot write " + path; return false; }
  out << "ply\n" << "format binary_little_endian 1.0\n" << "element vertex " << int(cloud.size()) << "\n"
      << "property float x\n" << "property float y\n" << "property float z\n"
      << "property uchar diffuse_blue\n" << "property uchar diffuse_green\n" << "property uchar diffuse_red\n"
      << "end_header\n";
  for (const FusedPoint& p : cloud) {
    const float xyz[3] = {p.x, p.y, p.z};
    const uint8_t px[3] = {static_cast<uint8_t>(p.b), static_cast<uint8_t>(p.g), static_cast<uint8_t>(p.r)};
    out.write(reinterpret_cast<const char*>(xyz), sizeof(xyz));
    out.write(reinterpret_cast<const char*>(px), sizeof(px));
  }
  if (!out) { err = "write failed: " + path; return false; }
  return true;
}

}  // namespace dpe_host
