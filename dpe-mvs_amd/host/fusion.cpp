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
#include <unordered_map>

namespace dpe_host {

// RunFusion's serial part (DPE.cpp:1286-1367) over the candidates of `fn`.
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
  std::vector<int32_t> cidx;
  std::vector<float> cval;
  for (int i = 0; i < n; ++i) {
    const int ref = idx_of(views[i].image_id);
    FusionView& R = views[ref];
    const int cols = R.view.width, rows = R.view.height;
    std::vector<int> src;
    for (int id : views[i].src_ids) src.push_back(idx_of(id));
    const int ns = (int)src.size();
    cidx.assign((size_t)cols * rows * ns, -1);
    cval.assign((size_t)cols * rows * ns * 3, 0.0f);
    if (ns > 0) {
      const int rc = fn(user, dv.data(), n, ref, src.data(), ns, cidx.data(), cval.data());
      if (rc != 0) { err = "fusion candidates failed (" + std::to_string(rc) + ")"; return false; }
    }
    std::vector<int> used(ns);
    for (int r = 0; r < rows; ++r)
      for (int c = 0; c < cols; ++c) {
        const size_t p = (size_t)r * cols + c;
        if (!R.block.empty() && R.block[p] < 128) continue;
        if (R.mask[p] == 1) continue;
        const float ref_depth = R.view.depth[p];
        if (ref_depth <= 0.0) continue;
        int num_consistent = 0;
        float dyn = 0.0f;
        for (int j = 0; j < ns; ++j) {
          used[j] = -1;
          const int32_t sp = cidx[p * ns + j];
          if (sp < 0) continue;
          if (views[src[j]].mask[sp] == 1) continue;
          const float* v = cval.data() + (p * ns + j) * 3;
          float angle = std::acos(v[2]);                     // GetAngle (DPE.cpp:1208-1217)
          if (angle != angle) angle = 0.0f;
          if (angle < 0.174533f) {                           // reproj < 2, rel < 0.01 tested by the candidates
            used[j] = sp;
            const float tmp_index = v[0] + 200 * v[1] + angle * 10;
            dyn += std::exp(-tmp_index);
            num_consistent++;
          }
        }
        const float factor = R.weak[p] == DPE_WEAK ? 0.45f : 0.3f;
        if (num_consistent >= 1 && dyn > factor * num_consistent) {
          float col[3] = {(float)R.bgr[3 * p], (float)R.bgr[3 * p + 1], (float)R.bgr[3 * p + 2]};
          for (int j = 0; j < ns; ++j) {
            if (used[j] < 0) continue;
            FusionView& S = views[src[j]];
            S.mask[used[j]] = 1;
            col[0] += S.bgr[3 * (size_t)used[j]];
            col[1] += S.bgr[3 * (size_t)used[j] + 1];
            col[2] += S.bgr[3 * (size_t)used[j] + 2];
          }
          for (float& x : col) x /= (num_consistent + 1);
          const FusedPoint pt = fusion_point(c, r, ref_depth, R.view.cam, col);
          cloud.push_back(pt);
        }
      }
  }
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
