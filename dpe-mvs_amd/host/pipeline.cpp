// pipeline.cpp — RunDPEPipeline (main.cpp:474-600) over the C-ABI PatchMatch pass.
//
// Kept from the reference: the dense_folder contract (images/%08d.jpg, cams/%08d_cam.txt, pair.txt
// in; DPE/%08d/ results; edges_<s>.dmb / labels_<s>.dmb read from the result folders), the
// coarse-to-fine schedule and its per-pass parameters (main.cpp:490-570), InuputInitialization's
// rescaling rules (DPE.cpp:733-914), the ProcessProblem epilogue (main.cpp:423-446) and the final
// .npy outputs (main.cpp:99-260).
//
// Different by design: every image is decoded once and its pyramid levels cached; per-image state
// (depth, normal, weak, selected views) stays in memory between passes instead of .dmb round
// trips; problems are split in contiguous blocks over ranks (one process per GPU) and the depth
// maps are all-gathered after every pass; "reference" schedule = the reference's serial order,
// "jacobi" = each pass reads the previous pass's depths (forced when world_size > 1).
//
// GetProblemEdges (main.cpp:331-388) runs before the first pass as in the reference: edges_<s>.dmb /
// labels_<s>.dmb that are missing are computed by EdgeSegment (edges.cpp) and written.
// fusion = true runs RunFusion (fusion.cpp) on rank 0 after the outputs: the per-(pixel, view)
// projection tests on the GPU (dpe_fusion_candidates), the order-dependent rest on the host; with
// several ranks the final normals and pixel states are all-gathered first.  As in the reference the
// edges_/labels_ maps are deleted at the end unless keep_intermediate.  Not part of this build: the
// viz medium results (ignored).
#include "host.h"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <thread>

namespace fs = std::filesystem;

namespace dpe_host {
namespace {

thread_local std::string g_err;
const char* kOutName = "DPE";
// wall seconds of the last run's phases: total, decode, GetProblemEdges pre-pass, passes (incl. the
// exchanges), outputs + fusion, then (multi-rank) the depth exchanges alone, the pass work alone and
// RunFusion alone (rank 0, incl. the normal/weak exchange that feeds it)
constexpr int kNumTimes = 8;
double g_times[kNumTimes] = {0, 0, 0, 0, 0, 0, 0, 0};
double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

struct Problem {   // main.h:108-118
  int index = 0, ref_image_id = 0;
  std::vector<int> src_image_ids;
  std::string dense_folder, result_folder;
  int scale_size = 1;
  DpePatchMatchParams params;
  int iteration = 0;
};

struct DepthMap { int w = 0, h = 0; std::vector<float> d; };

struct ImageState {   // depths.dmb / normals.dmb / weak.bin / selected_views.bin of one image
  int w = 0, h = 0;
  std::vector<float> depth, normal;     // normal: [h][w][3]
  std::vector<uint8_t> weak;
  std::vector<uint32_t> sel;
};

int std_round(float v) { return (int)std::round(v); }   // std::round: half away from zero

bool generate_sample_list(const std::string& dense, std::vector<Problem>& probs, std::string& err) {   // main.cpp:264-308
  std::ifstream f(fs::path(dense) / "pair.txt");
  if (!f) { err = "cannot read pair.txt in " + dense; return false; }
  std::string line;
  std::getline(f, line);
  int n = 0;
  std::istringstream(line) >> n;
  for (int i = 0; i < n; ++i) {
    Problem p;
    dpe_params_default(&p.params);
    p.index = i;
    std::getline(f, line);
    std::istringstream(line) >> p.ref_image_id;
    p.dense_folder = dense;
    p.result_folder = (fs::path(dense) / kOutName / fmt_index(p.ref_image_id)).string();
    std::error_code ec;
    fs::create_directories(p.result_folder, ec);
    std::getline(f, line);
    std::istringstream is(line);
    int m = 0;
    is >> m;
    for (int j = 0; j < m; ++j) {
      int id; float score;
      is >> id >> score;
      if (score <= 0.0f) continue;
      p.src_image_ids.push_back(id);
    }
    probs.push_back(std::move(p));
  }
  return true;
}

class ImageCache {
 public:
  explicit ImageCache(std::string folder) : folder_(std::move(folder)) {}
  const std::vector<float>* full(int idx, int& w, int& h, std::string& err) {
    auto it = full_.find(idx);
    if (it == full_.end()) {
      GrayImage g;
      if (!read_gray((fs::path(folder_) / "images" / (fmt_index(idx) + ".jpg")).string(), g, err)) return nullptr;
      Level L{g.w, g.h, std::vector<float>(g.px.begin(), g.px.end())};
      it = full_.emplace(idx, std::move(L)).first;
    }
    w = it->second.w; h = it->second.h;
    return &it->second.px;
  }
  // decodes the images not cached yet on `nt` host threads (independent files; same pixels as full())
  bool prefetch(const std::vector<int>& ids, int nt, std::string& err) {
    std::vector<int> todo;
    for (int id : ids)
      if (!full_.count(id) && std::find(todo.begin(), todo.end(), id) == todo.end()) todo.push_back(id);
    std::vector<GrayImage> g(todo.size());
    std::vector<std::string> e(todo.size());
    nt = std::max(1, std::min<int>(nt, (int)todo.size()));
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t)
      pool.emplace_back([&, t]() {
        for (size_t k = t; k < todo.size(); k += nt)
          read_gray((fs::path(folder_) / "images" / (fmt_index(todo[k]) + ".jpg")).string(), g[k], e[k]);
      });
    for (auto& th : pool) th.join();
    for (size_t k = 0; k < todo.size(); ++k) {
      if (!e[k].empty()) { err = e[k]; return false; }
      full_.emplace(todo[k], Level{g[k].w, g[k].h, std::vector<float>(g[k].px.begin(), g[k].px.end())});
    }
    return true;
  }
  const std::vector<float>* level(int idx, int scale, int& w, int& h, std::string& err) {
    int fw, fh;
    const std::vector<float>* f = full(idx, fw, fh, err);
    if (!f) return nullptr;
    if (scale == 1) { w = fw; h = fh; return f; }
    const auto key = std::make_pair(idx, scale);
    auto it = lvl_.find(key);
    if (it == lvl_.end()) {
      const float factor = 1.0f / (float)scale;
      const int nw = std_round(fw * factor), nh = std_round(fh * factor);
      Level L{nw, nh, std::vector<float>((size_t)nw * nh)};
      resize_linear(f->data(), fw, fh, L.px.data(), nw, nh);
      it = lvl_.emplace(key, std::move(L)).first;
    }
    w = it->second.w; h = it->second.h;
    return &it->second.px;
  }

 private:
  struct Level { int w, h; std::vector<float> px; };
  std::string folder_;
  std::map<int, Level> full_;
  std::map<std::pair<int, int>, Level> lvl_;
};

int scale_index(int scale_size) { int s = 0; while ((1 << s) < scale_size) s++; return s; }

void pass_params(DpePatchMatchParams& p, int i, int j) {   // main.cpp:510-556 (j = -1: first pass of round i)
  if (j < 0) {
    if (i == 0) { p.state = DPE_FIRST_INIT; p.use_APD = false; p.use_edge = false; }
    else {
      p.state = DPE_REFINE_INIT; p.use_APD = true; p.use_edge = true;
      p.ransac_threshold = (float)(0.01 - i * 0.00125);
      p.rotate_time = std::min((int)std::pow(2, i), 4);
    }
    p.geom_consistency = false;
    p.max_iterations = 3;
    p.weak_peak_radius = 6;
  } else {
    p.state = DPE_REFINE_ITER;
    p.use_APD = i != 0; p.use_edge = i != 0;
    p.ransac_threshold = (float)(0.01 - i * 0.00125);
    p.rotate_time = std::min((int)std::pow(2, i), 4);
    p.geom_consistency = true;
    p.max_iterations = 3;
    p.weak_peak_radius = std::max(4 - 2 * j, 2);
  }
}

template <class T>
std::vector<T> rescaled(const std::vector<T>& src, int w, int h, int nw, int nh, int ch = 1) {
  if (w == nw && h == nh) return src;
  std::vector<T> dst((size_t)nw * nh * ch, T(0));
  rescale_nearest(src.data(), w, h, dst.data(), nw, nh, (int)sizeof(T) * ch);
  return dst;
}

bool read_support(const Problem& p, const std::string& name, Mat& m, std::string& err) {
  const std::string path = (fs::path(p.result_folder) / name).string();
  if (!fs::exists(path)) {
    err = path + " missing (GetProblemEdges writes it before the first pass)";
    return false;
  }
  return read_bin_mat(path, m, err);
}

struct Runner {
  dpe_pass_runner_fn fn = nullptr;
  void* user = nullptr;
  DpeContext* ctx = nullptr;
  ~Runner() { if (ctx) dpe_destroy(ctx); }
};
int native_runner(void* user, const DpePassInput* in, const DpePassState* st) {
  return dpe_pm_run(static_cast<DpeContext*>(user), in, st);
}

struct NativeFusion {
  DpeContext* ctx = nullptr;
  bool own = false;
  const DpeFusionView* staged = nullptr;
  std::string err;   // the library's message of a failed call (run_fusion calls from a worker thread,
                     // and dpe_last_error() is per thread)
  ~NativeFusion() { if (own && ctx) dpe_destroy(ctx); }
};
int native_fusion(void* user, const DpeFusionView* views, int n, int ref, const int* src, int ns, int32_t* idx,
                  float* val) {
  NativeFusion* f = static_cast<NativeFusion*>(user);
  if (f->staged != views) {
    const int r = dpe_fusion_stage(f->ctx, views, n);
    if (r != DPE_OK) { f->err = dpe_last_error(); return r; }
    f->staged = views;
  }
  const int r = dpe_fusion_candidates(f->ctx, ref, src, ns, idx, val);
  if (r != DPE_OK) f->err = dpe_last_error();
  return r;
}

// the per-pass intermediate maps of the reference (main.cpp:439-446)
bool write_state_maps(const Problem& p, const ImageState& s, std::string& err) {
  const int W = s.w, H = s.h;
  const size_t L = (size_t)W * H;
  Mat m;
  m.create(H, W, CV_32FC1); std::memcpy(m.data.data(), s.depth.data(), L * 4);
  if (!write_bin_mat((fs::path(p.result_folder) / "depths.dmb").string(), m, err)) return false;
  m.create(H, W, CV_32FC3); std::memcpy(m.data.data(), s.normal.data(), L * 12);
  if (!write_bin_mat((fs::path(p.result_folder) / "normals.dmb").string(), m, err)) return false;
  m.create(H, W, CV_8UC1); std::memcpy(m.data.data(), s.weak.data(), L);
  if (!write_bin_mat((fs::path(p.result_folder) / "weak.bin").string(), m, err)) return false;
  m.create(H, W, CV_32SC1); std::memcpy(m.data.data(), s.sel.data(), L * 4);
  if (!write_bin_mat((fs::path(p.result_folder) / "selected_views.bin").string(), m, err)) return false;
  return true;
}

// host copy of an image's HBM-resident state (depth_only: a state imported from another rank)
bool fetch_state(DpeContext* ctx, int id, ImageState& s, std::string& err, bool depth_only = false) {
  int w = 0, h = 0;
  if (dpe_state_fetch(ctx, id, &w, &h, nullptr, nullptr, nullptr, nullptr) != 0) { err = dpe_last_error(); return false; }
  const size_t L = (size_t)w * h;
  s.w = w; s.h = h;
  s.depth.resize(L);
  if (!depth_only) { s.normal.resize(L * 3); s.weak.resize(L); s.sel.resize(L); }
  const int rc = dpe_state_fetch(ctx, id, &w, &h, s.depth.data(), depth_only ? nullptr : s.normal.data(),
                                 depth_only ? nullptr : s.weak.data(), depth_only ? nullptr : s.sel.data());
  if (rc != 0) { err = dpe_last_error(); return false; }
  return true;
}

// InuputInitialization + SupportInitialization (DPE.cpp:733-914, 1025-1052), the pass, the epilogue
bool process_problem(Problem& p, ImageCache& cache, std::map<int, ImageState>& states,
                     const std::map<int, DepthMap>& depth_src, const DpePipelineOptions& opt, Runner& run,
                     std::string& err) {
  DpePatchMatchParams& P = p.params;
  std::vector<int> ids{p.ref_image_id};
  ids.insert(ids.end(), p.src_image_ids.begin(), p.src_image_ids.end());
  if ((int)ids.size() > DPE_MAX_IMAGES) { err = "Can't process so much images: " + std::to_string(ids.size()); return false; }
  int fw, fh;
  if (!cache.full(ids[0], fw, fh, err)) return false;
  std::vector<const float*> images;
  std::vector<DpeCamera> cams(ids.size());
  int W = 0, H = 0;
  for (size_t k = 0; k < ids.size(); ++k) {
    DpeCamera& cam = cams[k];
    if (!read_camera((fs::path(p.dense_folder) / "cams" / (fmt_index(ids[k]) + "_cam.txt")).string(), cam, err)) return false;
    cam.width = fw; cam.height = fh;
    int w, h;
    const std::vector<float>* img = cache.level(ids[k], p.scale_size, w, h, err);
    if (!img) return false;
    if (p.scale_size != 1) {
      const float sx = w / (float)fw, sy = h / (float)fh;
      cam.K[0] *= sx; cam.K[2] *= sx; cam.K[4] *= sy; cam.K[5] *= sy;
      cam.width = w; cam.height = h;
    }
    if (k == 0) { W = w; H = h; }
    images.push_back(img->data());
  }
  const size_t L = (size_t)W * H;
  P.depth_min = cams[0].depth_min * 0.6f;
  P.depth_max = cams[0].depth_max * 1.2f;
  P.num_images = (int)ids.size();
  // with the default runner the state stays in HBM (dpe_state_save / dpe_pm_stage_resident): the
  // prior, the source depths and the epilogue are all on the device, nothing is copied back per pass
  const bool resident = run.ctx != nullptr;
  std::vector<std::vector<float>> dep_store;
  std::vector<const float*> depths(ids.size(), nullptr);
  if (P.geom_consistency && !resident) {
    dep_store.reserve(ids.size());
    for (size_t k = 1; k < ids.size(); ++k) {
      auto it = depth_src.find(ids[k]);
      if (it == depth_src.end()) { err = "no depth map of source image " + std::to_string(ids[k]); return false; }
      dep_store.push_back(rescaled(it->second.d, it->second.w, it->second.h, W, H));
      depths[k] = dep_store.back().data();
    }
  }
  const ImageState* prev = (!resident && states.count(p.ref_image_id)) ? &states.at(p.ref_image_id) : nullptr;
  std::vector<float> planes(resident ? 0 : L * 4, 0.0f);
  std::vector<uint8_t> weak(resident ? 0 : L, DPE_STRONG);
  std::vector<uint32_t> sel(resident ? 0 : L, 0u);
  if (resident) {
    // nothing to build on the host
  } else if (P.use_APD) {
    if (!prev) { err = "Can't find weak info of image " + std::to_string(p.ref_image_id); return false; }
    weak = rescaled(prev->weak, prev->w, prev->h, W, H);
  }
  if (!resident && P.state != DPE_FIRST_INIT) {
    if (!prev) { err = "no prior depth/normal of image " + std::to_string(p.ref_image_id); return false; }
    const std::vector<float> d = rescaled(prev->depth, prev->w, prev->h, W, H);
    const std::vector<float> n = rescaled(prev->normal, prev->w, prev->h, W, H, 3);
    for (size_t i = 0; i < L; ++i) {
      planes[4 * i + 0] = n[3 * i + 0]; planes[4 * i + 1] = n[3 * i + 1]; planes[4 * i + 2] = n[3 * i + 2];
      planes[4 * i + 3] = d[i];
    }
    sel = rescaled(prev->sel, prev->w, prev->h, W, H);
  }
  DpePassInput in;
  std::memset(&in, 0, sizeof(in));
  in.width = W; in.height = H; in.num_images = (int)ids.size();
  in.images = images.data();
  in.cams = cams.data();
  in.depths = (P.geom_consistency && !resident) ? depths.data() : nullptr;
  Mat edge, edge_low, label;
  if (P.use_edge || P.use_limit) {
    const int s = scale_index(p.scale_size);
    const int max_s = P.high_res_img ? scale_index(P.max_scale_size) : s;
    if (!read_support(p, "edges_" + std::to_string(s) + ".dmb", edge, err)) return false;
    if (!read_support(p, "edges_" + std::to_string(max_s) + ".dmb", edge_low, err)) return false;
    if (edge.rows != H || edge.cols != W || edge.type != CV_8UC1) { err = "edge map size/type mismatch in " + p.result_folder; return false; }
    in.edge = edge.ptr<uint8_t>();
    in.edge_low_res = edge_low.ptr<uint8_t>();
    in.low_width = edge_low.cols; in.low_height = edge_low.rows;
  }
  if (P.use_label) {
    if (!read_support(p, "labels_" + std::to_string(scale_index(p.scale_size)) + ".dmb", label, err)) return false;
    if (label.rows != H || label.cols != W || label.type != CV_32SC1) { err = "label map size/type mismatch in " + p.result_folder; return false; }
    in.label = label.ptr<int32_t>();
  }
  in.params = P;
  in.seed = opt.base_seed ^ ((uint64_t)p.ref_image_id * 0x9E3779B97F4A7C15ull);
  in.pass_salt = (uint32_t)p.iteration;
  in.image_ids = ids.data();        // pyramid levels stay in HBM across passes (keyed by id and size)
  if (resident) {
    int rc = dpe_pm_stage_resident(run.ctx, &in, p.ref_image_id);
    if (rc == 0) rc = dpe_pm_execute(run.ctx, nullptr);
    if (rc == 0) rc = dpe_state_save(run.ctx, p.ref_image_id);
    if (rc != 0) { err = "PatchMatch pass failed (" + std::to_string(rc) + "): " + dpe_last_error(); return false; }
    if (opt.keep_intermediate) {
      ImageState s;
      if (!fetch_state(run.ctx, p.ref_image_id, s, err)) return false;
      if (!write_state_maps(p, s, err)) return false;
    }
    return true;
  }
  std::vector<float> costs(L);
  DpePassState st{planes.data(), weak.data(), sel.data(), costs.data()};
  const int rc = run.fn(run.user, &in, &st);
  if (rc != 0) {
    err = "PatchMatch pass failed (" + std::to_string(rc) + "): " + (run.ctx ? std::string(dpe_last_error()) : "runner");
    return false;
  }
  // epilogue (main.cpp:423-437): depth outside [dmin, dmax] -> 0 and UNKNOWN
  ImageState s;
  s.w = W; s.h = H;
  s.depth.resize(L); s.normal.resize(L * 3); s.weak = weak; s.sel = sel;
  for (size_t i = 0; i < L; ++i) {
    float d = planes[4 * i + 3];
    if (d < P.depth_min || d > P.depth_max) { d = 0.0f; s.weak[i] = DPE_UNKNOWN; }
    s.depth[i] = d;
    s.normal[3 * i + 0] = planes[4 * i + 0]; s.normal[3 * i + 1] = planes[4 * i + 1]; s.normal[3 * i + 2] = planes[4 * i + 2];
  }
  if (opt.keep_intermediate && !write_state_maps(p, s, err)) return false;
  states[p.ref_image_id] = std::move(s);
  return true;
}

bool write_outputs(const Problem& p, const ImageState& s, const DpePipelineOptions& opt, std::string& err) {   // main.cpp:572-578
  const std::vector<int64_t> hw{s.h, s.w};
  const fs::path rf(p.result_folder);
  if (opt.depth) {
    std::vector<float> d = s.depth;
    for (size_t i = 0; i < d.size(); ++i) if (s.weak[i] == DPE_UNKNOWN) d[i] = 0.0f;   // ZeroDepthForUnknown
    if (!write_npy((rf / "depth.npy").string(), d.data(), hw, "<f4", 4, err)) return false;
  }
  if (opt.normal && !write_npy((rf / "normal.npy").string(), s.normal.data(), {s.h, s.w, 3}, "<f4", 4, err)) return false;
  if (opt.weak) {
    std::vector<int8_t> e(s.weak.size());
    for (size_t i = 0; i < e.size(); ++i) e[i] = s.weak[i] == DPE_WEAK ? 1 : (s.weak[i] == DPE_STRONG ? 2 : 0);
    if (!write_npy((rf / "weak.npy").string(), e.data(), hw, "|i1", 1, err)) return false;
  }
  if (opt.edge) {
    for (int idx = 0; idx < 8; ++idx) {
      const fs::path ep = rf / ("edges_" + std::to_string(idx) + ".dmb");
      if (!fs::exists(ep)) continue;
      Mat m;
      if (!read_bin_mat(ep.string(), m, err)) return false;
      std::vector<int8_t> b(m.data.size());
      for (size_t i = 0; i < b.size(); ++i) b[i] = m.data[i] > 0 ? 1 : 0;
      if (!write_npy((rf / "edge.npy").string(), b.data(), {m.rows, m.cols}, "|i1", 1, err)) return false;
      break;
    }
  }
  return true;
}

int run(const char* dense_folder, const DpePipelineOptions& opt) {
  std::string& err = g_err;
  err.clear();
  const double t_start = now_s();
  for (double& t : g_times) t = 0.0;
  const int world = std::max(1, opt.world_size), rank = opt.rank;
  if (world > 1 && !opt.allgather) { err = "world_size > 1 needs an all-gather"; return 1; }
  if (rank < 0 || rank >= world) { err = "bad rank"; return 1; }
  const bool jacobi = world > 1 || opt.schedule == DPE_SCHEDULE_JACOBI;
  const std::string dense(dense_folder);
  std::error_code ec;
  fs::create_directories(fs::path(dense) / kOutName, ec);
  std::vector<Problem> problems;
  if (!generate_sample_list(dense, problems, err)) return 1;
  ImageCache cache(dense);
  double t_mark = now_s();
  {   // every image of the run decoded once, on the host threads
    std::vector<int> ids;
    for (const Problem& p : problems) {
      ids.push_back(p.ref_image_id);
      for (int s : p.src_image_ids) ids.push_back(s);
    }
    const int nt = (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
    std::string perr;
    if (!cache.prefetch(ids, nt, perr)) { err = "Images may error, check it! " + perr; std::cerr << "Images may error, check it!\n"; return 1; }
  }
  {   // CheckImages (main.cpp:310-329)
    int w0 = 0, h0 = 0;
    bool ok = !problems.empty();
    for (size_t i = 0; ok && i < problems.size(); ++i) {
      int w, h;
      if (!cache.full(problems[i].ref_image_id, w, h, err)) ok = false;
      else if (i == 0) { w0 = w; h0 = h; }
      else if (w != w0 || h != h0) ok = false;
    }
    if (!ok) { err = "Images may error, check it! " + err; std::cerr << "Images may error, check it!\n"; return 1; }
  }
  const int n = (int)problems.size();
  // every rank reads the same pair.txt, so every rank takes this exit together (no collective yet)
  if (world > n) { err = "world_size " + std::to_string(world) + " exceeds the " + std::to_string(n) + " problems"; return 1; }
  std::vector<std::vector<int>> blocks(world);
  for (int r = 0; r < world; ++r) for (int i = r * n / world; i < (r + 1) * n / world; ++i) blocks[r].push_back(i);
  // Multi-rank failure handling: a rank whose own work fails keeps joining the collectives with a
  // failure flag in its message, so every rank sees it at the same exchange and all return 1 together
  // (an early return on one rank would leave the others blocked in the all-gather).
  bool failed = false;
  std::string first_err;
  auto fail = [&](const std::string& e) { if (!failed) { failed = true; first_err = e; } };
  // A collective that fails on this rank may leave peers waiting in theirs: the optional abort hook
  // (ncclCommAbort in bin/dpe) makes them fail fast instead of waiting for RCCL's timeout.  Without
  // one (torch / gloo hooks from Python) the peers wait for their backend's own timeout.
  auto abort_peers = [&]() { if (opt.abort_collectives) (void)opt.abort_collectives(opt.abort_user); };
  // all-gather of `per` floats per rank plus one status float; false (err set) when any rank failed
  auto exchange = [&](std::vector<float>& send, std::vector<float>& recv) -> bool {
    const size_t per = send.size();
    send.push_back(failed ? 1.0f : 0.0f);
    recv.assign((per + 1) * world, 0.0f);
    if (opt.allgather(opt.allgather_user, send.data(), per + 1, recv.data()) != 0) {
      err = "all-gather failed";
      abort_peers();
      return false;
    }
    send.pop_back();
    std::vector<float> packed(per * world);
    int bad = -1;
    for (int r = 0; r < world; ++r) {
      std::memcpy(packed.data() + (size_t)r * per, recv.data() + (size_t)r * (per + 1), per * sizeof(float));
      if (bad < 0 && recv[(size_t)r * (per + 1) + per] != 0.0f) bad = r;
    }
    recv.swap(packed);
    if (bad >= 0) {
      err = bad == rank ? first_err : "rank " + std::to_string(bad) + " failed";
      return false;
    }
    return true;
  };
  // the ranks' failure flags, one float each over the host hook; false (err set) when any rank failed
  auto status_exchange = [&]() -> bool {
    float flag = failed ? 1.0f : 0.0f;
    std::vector<float> all(world, 0.0f);
    if (opt.allgather(opt.allgather_user, &flag, 1, all.data()) != 0) { err = "all-gather failed"; abort_peers(); return false; }
    for (int r = 0; r < world; ++r)
      if (all[r] != 0.0f) { err = r == rank ? first_err : "rank " + std::to_string(r) + " failed"; return false; }
    return true;
  };
  // DPE_FAULT_INJECT="before:R" / "after:R" (tests): rank R fails locally just before / after the
  // first resident depth exchange's collectives (read per run)
  const std::pair<int, int> fault = [] {
    const char* e = std::getenv("DPE_FAULT_INJECT");
    if (!e) return std::make_pair(-1, -1);
    const std::string v(e);
    const size_t c = v.find(':');
    if (c == std::string::npos) return std::make_pair(-1, -1);
    return std::make_pair(v.compare(0, c, "before") == 0 ? 0 : (v.compare(0, c, "after") == 0 ? 1 : -1), std::atoi(v.c_str() + c + 1));
  }();
  bool fault_done = false;
  auto fault_at = [&](int when, int r) -> bool {
    if (fault_done || fault.first != when || fault.second != r) return false;
    fault_done = true;
    return true;
  };
  Runner runner;
  if (opt.runner) { runner.fn = opt.runner; runner.user = opt.runner_user; }
  else {
    runner.ctx = dpe_create(opt.gpu_index);
    if (!runner.ctx) fail(std::string("dpe_create: ") + dpe_last_error());
    else { runner.fn = native_runner; runner.user = runner.ctx; }
    if (world == 1 && failed) { err = first_err; return 1; }
  }
  int w0, h0;
  cache.full(problems[0].ref_image_id, w0, h0, err);
  int round_num = 1, max_size = std::max(w0, h0);   // ComputeRoundNum (main.cpp:390-408)
  while (max_size > 800) { max_size /= 2; round_num++; }
  round_num = std::max(round_num, 2);
  if (opt.verbose && rank == 0) {
    // std::cout as main.cpp:489, 504 (the pybind module redirects it into sys.stdout)
    std::cout << "There are " << n << " images to be processed!" << std::endl;
    std::cout << "There are " << round_num << " resolution stages for coarse-to-fine processing!" << std::endl;
    std::cout << "Iteration nums: " << round_num * 4 << std::endl;
  }
  g_times[1] = now_s() - t_mark;
  t_mark = now_s();
  roctxRangePushA("GetProblemEdges");
  {   // GetProblemEdges for every scale of the schedule (main.cpp:494-501); images are independent,
      // so a pool of host threads takes them round-robin (the decode cache is filled first)
    std::vector<GrayImage> grey(blocks[rank].size());
    for (size_t k = 0; k < blocks[rank].size(); ++k) {
      int fw, fh;
      const std::vector<float>* f = cache.full(problems[blocks[rank][k]].ref_image_id, fw, fh, err);
      if (!f) return 1;   // decoded in CheckImages above: cannot fail here
      grey[k].w = fw; grey[k].h = fh;
      grey[k].px.resize(f->size());
      for (size_t q = 0; q < f->size(); ++q) grey[k].px[q] = (uint8_t)(*f)[q];
    }
    const int nt = (int)std::max<size_t>(1, std::min<size_t>({grey.size(), (size_t)16,
                                                              (size_t)std::max(1u, std::thread::hardware_concurrency())}));
    // the data-parallel stages (resize, Sobel / NMS, Roberts) on the runner's GPU, the scan-order and
    // RNG-order parts (hysteresis walk, Connect, HoughLinesP) on the host threads
    std::mutex edge_mu;
    EdgeDevice edev{runner.ctx, &edge_mu};
    std::vector<std::string> terr(nt);
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t)
      pool.emplace_back([&, t]() {
        for (size_t k = t; k < grey.size(); k += nt) {
          const Problem& p = problems[blocks[rank][k]];
          for (int i = 0; i < round_num && terr[t].empty(); ++i)
            if (!get_problem_edges(grey[k], (int)std::pow(2, round_num - 1 - i), p.result_folder, p.params.use_edge,
                                   p.params.use_label, p.params.high_res_img, terr[t], &edev) && terr[t].empty())
              terr[t] = "EdgeSegment failed";
        }
      });
    for (auto& th : pool) th.join();
    for (auto& e : terr) if (!e.empty()) { fail(e); break; }
    roctxRangePop();
    if (world == 1 && failed) return 1;
  }
  g_times[2] = now_s() - t_mark;
  t_mark = now_s();
  for (auto& p : problems) p.params.max_scale_size = std::max(1, (int)std::pow(2, round_num - 1));
  std::map<int, ImageState> states;
  std::map<int, DepthMap> depth_cur;
  int iteration_index = 0;
  const bool resident = runner.ctx != nullptr;
  double t_pass = 0.0, t_xchg = 0.0;   // g_times[6] / [5]
  for (int i = 0; i < round_num; ++i) {
    for (int j = -1; j < 3; ++j) {
      const double tp0 = now_s();
      if (resident && jacobi && !failed && dpe_state_snapshot(runner.ctx) != 0) fail(dpe_last_error());
      const std::map<int, DepthMap> snapshot = (jacobi && !resident) ? depth_cur : std::map<int, DepthMap>{};
      const auto& depth_src = jacobi ? snapshot : depth_cur;
      // pass size: ImageCache::level's rounding of the first image (CheckImages: all the same size)
      const int scale = (int)std::pow(2, round_num - 1 - i);
      const int pw = scale == 1 ? w0 : std_round(w0 * (1.0f / (float)scale));
      const int ph = scale == 1 ? h0 : std_round(h0 * (1.0f / (float)scale));
      for (int pi : blocks[rank]) {
        if (failed) break;
        Problem& p = problems[pi];
        p.iteration = iteration_index;
        p.scale_size = scale;
        p.params.scale_size = p.scale_size;
        pass_params(p.params, i, j);
        if (opt.max_iterations > 0) p.params.max_iterations = opt.max_iterations;
        if (opt.photometric_only) p.params.geom_consistency = false;
        std::string perr;
        const std::string rname = "ProcessProblem round " + std::to_string(i) + " pass " + std::to_string(j + 1) +
                                  " image " + std::to_string(p.ref_image_id);
        roctxRangePushA(rname.c_str());
        const bool ok = process_problem(p, cache, states, depth_src, opt, runner, perr);
        roctxRangePop();
        if (!ok) { fail(perr); break; }
        if (!resident) {
          const ImageState& s = states[p.ref_image_id];
          depth_cur[p.ref_image_id] = DepthMap{s.w, s.h, s.depth};
        }
      }
      // the pass round's GPU work is finished before its clock stops (and, multi-rank, before the
      // exchange's clock starts): with one rank the passes are otherwise only enqueued here
      if (resident && !failed && dpe_sync(runner.ctx) != 0) fail(dpe_last_error());
      if (world == 1 && failed) { err = first_err; return 1; }
      const double tx0 = now_s();
      t_pass += tx0 - tp0;
      if (world > 1 && resident) {   // all-gather of the depth maps from / into the HBM-resident states
        // Two collectives per exchange, both joined by every rank whatever happened locally:
        //  1. the ranks' status flags over the host hook (one float each).  A local error before it
        //     (the pass, the exchange buffers, the export) raises the flag and every rank returns 1
        //     at this exchange;
        //  2. the depth maps (nmax maps per rank), device to device, or one device -> host -> device
        //     hop through the host hook.  An error after (1) can no longer stop the others, who are
        //     committed to (2): the rank still joins (2), records the error and reports it at the
        //     next exchange's (1) or at the final status exchange after the passes.
        size_t nmax = 0;
        for (auto& b : blocks) nmax = std::max(nmax, b.size());
        const size_t per = (size_t)pw * ph, cnt = nmax * per;
        float* dsend = dpe_device_buffer(runner.ctx, 0, cnt);
        float* drecv = dsend ? dpe_device_buffer(runner.ctx, 1, cnt * world) : nullptr;
        bool dev_ok = drecv != nullptr;
        if (!dev_ok) fail(dpe_last_error());
        for (size_t k = 0; dev_ok && !failed && k < blocks[rank].size(); ++k)
          if (dpe_state_export_depth(runner.ctx, problems[blocks[rank][k]].ref_image_id, dsend + k * per, nullptr) != 0)
            fail(dpe_last_error());
        // the exports run on the context's stream; the collective reads dsend from another one
        if (dev_ok && !failed && dpe_sync(runner.ctx) != 0) fail(dpe_last_error());
        if (fault_at(0, rank)) fail("injected fault before the exchange");
        if (!status_exchange()) return 1;
        if (opt.allgather_device) {
          if (opt.allgather_device(opt.allgather_device_user, dsend, cnt, drecv) != 0) {
            err = "all-gather failed";
            abort_peers();
            return 1;
          }
        } else {   // host hook: one device -> host -> device hop of the packed maps
          std::vector<float> hs(cnt, 0.0f), hr(cnt * world, 0.0f);
          if (dpe_device_copy(runner.ctx, hs.data(), dsend, cnt * sizeof(float), 1) != 0) fail(dpe_last_error());
          if (opt.allgather(opt.allgather_user, hs.data(), cnt, hr.data()) != 0) {
            err = "all-gather failed";
            abort_peers();
            return 1;
          }
          if (!failed && dpe_device_copy(runner.ctx, drecv, hr.data(), hr.size() * sizeof(float), 0) != 0)
            fail(dpe_last_error());
        }
        if (fault_at(1, rank)) fail("injected fault after the exchange");
        for (int r = 0; r < world; ++r) {
          if (r == rank) continue;
          for (size_t k = 0; k < blocks[r].size(); ++k)
            if (!failed && dpe_state_import_depth(runner.ctx, problems[blocks[r][k]].ref_image_id, pw, ph,
                                                  drecv + (size_t)r * cnt + k * per, nullptr) != 0)
              fail(dpe_last_error());   // reported at the next exchange's status step
        }
        if (!failed && dpe_sync(runner.ctx) != 0) fail(dpe_last_error());   // imports done: the exchange's end
      } else if (world > 1) {   // all-gather of the depth maps (the pass's only cross-image data)
        size_t nmax = 0;
        for (auto& b : blocks) nmax = std::max(nmax, b.size());
        const size_t per = (size_t)pw * ph;
        std::vector<float> send(nmax * per, 0.0f), recv;
        for (size_t k = 0; !failed && k < blocks[rank].size(); ++k) {
          const auto& d = depth_cur[problems[blocks[rank][k]].ref_image_id];
          std::memcpy(send.data() + k * per, d.d.data(), per * 4);
        }
        if (!exchange(send, recv)) return 1;
        for (int r = 0; r < world; ++r)
          for (size_t k = 0; k < blocks[r].size(); ++k) {
            const float* src = recv.data() + ((size_t)r * nmax + k) * per;
            depth_cur[problems[blocks[r][k]].ref_image_id] = DepthMap{pw, ph, std::vector<float>(src, src + per)};
          }
      }
      if (world > 1) t_xchg += now_s() - tx0;
      if (opt.verbose && rank == 0) std::cout << "Iteration " << iteration_index + 1 << " / " << round_num * 4 << " done" << std::endl;
      iteration_index++;
    }
  }
  g_times[3] = now_s() - t_mark;
  g_times[5] = t_xchg;
  g_times[6] = t_pass;
  t_mark = now_s();
  if (resident && !failed)   // the final states come back from HBM once
    for (int pi : blocks[rank]) {
      std::string ferr;
      if (!fetch_state(runner.ctx, problems[pi].ref_image_id, states[problems[pi].ref_image_id], ferr)) { fail(ferr); break; }
    }
  if (!failed) {   // each image's .npy files on their own host thread (independent files)
    const auto& blk = blocks[rank];
    const int nt = (int)std::min<size_t>(blk.size(), std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency())));
    std::vector<std::string> werr(blk.size());
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t)
      pool.emplace_back([&, t]() {
        for (size_t k = t; k < blk.size(); k += nt) {
          const Problem& p = problems[blk[k]];
          if (!write_outputs(p, states.at(p.ref_image_id), opt, werr[k]) && werr[k].empty()) werr[k] = "write failed";
        }
      });
    for (auto& th : pool) th.join();
    for (auto& e : werr) if (!e.empty()) { fail(e); break; }
  }
  // every rank learns here whether any rank failed after its last exchange (a rank returning alone
  // would leave the others' next collective, or their success, inconsistent with it)
  if (world > 1 && !status_exchange()) return 1;
  if (failed) { err = first_err; return 1; }
  const double t_fusion0 = now_s();
  g_times[7] = 0.0;
  if (opt.fusion) {   // RunFusion (main.cpp:578-580)
    std::map<int, ImageState> all;
    for (int pi : blocks[rank]) all[problems[pi].ref_image_id] = states[problems[pi].ref_image_id];
    if (world > 1) {   // the final normals and pixel states of every image (depths are in depth_cur)
      const ImageState& s0 = states[problems[blocks[rank][0]].ref_image_id];
      const size_t per = (size_t)s0.w * s0.h;
      size_t nmax = 0;
      for (auto& b : blocks) nmax = std::max(nmax, b.size());
      std::vector<float> send(nmax * per * 4, 0.0f), recv(send.size() * world);
      for (size_t k = 0; k < blocks[rank].size(); ++k) {
        const ImageState& st = states[problems[blocks[rank][k]].ref_image_id];
        float* o = send.data() + k * per * 4;
        std::memcpy(o, st.normal.data(), per * 12);
        for (size_t i = 0; i < per; ++i) o[3 * per + i] = (float)st.weak[i];
      }
      if (!exchange(send, recv)) return 1;
      for (int r = 0; r < world; ++r)
        for (size_t k = 0; k < blocks[r].size(); ++k) {
          const int id = problems[blocks[r][k]].ref_image_id;
          if (all.count(id)) continue;
          const float* src = recv.data() + ((size_t)r * nmax + k) * per * 4;
          ImageState st;
          st.w = s0.w; st.h = s0.h;
          if (resident) {
            ImageState d;
            if (!fetch_state(runner.ctx, id, d, err, true)) return 1;
            st.depth = std::move(d.depth);
          } else {
            st.depth = depth_cur[id].d;
          }
          st.normal.assign(src, src + 3 * per);
          st.weak.resize(per);
          for (size_t i = 0; i < per; ++i) st.weak[i] = (uint8_t)src[3 * per + i];
          all[id] = std::move(st);
        }
    }
    if (rank == 0) {
      std::vector<FusionView> views(problems.size());
      const bool use_block = fs::exists(fs::path(dense) / "blocks");
      // each view's camera, colour image (decode + RescaleImageAndCamera) and block mask on its own
      // host thread (independent files, independent outputs)
      std::vector<std::string> verr(problems.size());
      auto load_view = [&](size_t i) -> bool {
        std::string& err = verr[i];
        const Problem& p = problems[i];
        FusionView& v = views[i];
        const ImageState& st = all.at(p.ref_image_id);
        v.image_id = p.ref_image_id;
        v.src_ids = p.src_image_ids;
        DpeCamera cam;
        if (!read_camera((fs::path(dense) / "cams" / (fmt_index(p.ref_image_id) + "_cam.txt")).string(), cam, err)) return false;
        ColorImage img;
        if (!read_bgr((fs::path(dense) / "images" / (fmt_index(p.ref_image_id) + ".jpg")).string(), img, err)) return false;
        if (img.w != st.w || img.h != st.h) {   // RescaleImageAndCamera (DPE.cpp:1123-1144), per channel
          const float sx = st.w / (float)img.w, sy = st.h / (float)img.h;
          std::vector<uint8_t> ch((size_t)img.w * img.h), och((size_t)st.w * st.h);
          v.bgr.assign((size_t)st.w * st.h * 3, 0);
          for (int k = 0; k < 3; ++k) {
            for (size_t q = 0; q < ch.size(); ++q) ch[q] = img.bgr[3 * q + k];
            resize_u8(ch.data(), img.w, img.h, och.data(), st.w, st.h);
            for (size_t q = 0; q < och.size(); ++q) v.bgr[3 * q + k] = och[q];
          }
          cam.K[0] *= sx; cam.K[2] *= sx; cam.K[4] *= sy; cam.K[5] *= sy;
        } else {
          v.bgr = std::move(img.bgr);
        }
        cam.width = st.w; cam.height = st.h;
        if (use_block) {
          GrayImage b;
          if (!read_gray((fs::path(dense) / "blocks" / ("mask_" + std::to_string(p.ref_image_id) + ".jpg")).string(), b, err)) return false;
          if (b.w != st.w || b.h != st.h) { err = "block mask size differs from the depth map"; return false; }
          v.block = std::move(b.px);
        }
        v.view.width = st.w; v.view.height = st.h;
        v.view.cam = cam;
        v.view.depth = st.depth.data();
        v.view.normal = st.normal.data();
        v.weak = st.weak.data();
        return true;
      };
      {
        const size_t nv = problems.size();
        const int nt = (int)std::min<size_t>(nv, std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency())));
        std::vector<std::thread> pool;
        for (int t = 0; t < nt; ++t)
          pool.emplace_back([&, t]() {
            for (size_t i = t; i < nv; i += nt)
              if (!load_view(i) && verr[i].empty()) verr[i] = "fusion view load failed";
          });
        for (auto& th : pool) th.join();
        for (auto& e : verr) if (!e.empty()) { err = e; return 1; }
      }
      NativeFusion nf;
      dpe_fusion_fn ffn = opt.fusion_runner;
      void* fuser = opt.fusion_user;
      if (!ffn) {
        nf.ctx = runner.ctx;
        if (!nf.ctx) {
          nf.ctx = dpe_create(opt.gpu_index);
          if (!nf.ctx) { err = std::string("dpe_create: ") + dpe_last_error(); return 1; }
          nf.own = true;
        }
        ffn = native_fusion; fuser = &nf;
      }
      std::vector<FusedPoint> cloud;
      if (!run_fusion(views, ffn, fuser, cloud, err)) {
        if (!opt.fusion_runner) err += std::string(": ") + (nf.err.empty() ? std::string(dpe_last_error()) : nf.err);
        return 1;
      }
      if (!export_point_cloud((fs::path(dense) / kOutName / "DPE.ply").string(), cloud, err)) return 1;
      if (opt.verbose) std::cout << "Fused " << cloud.size() << " points" << std::endl;
    }
    g_times[7] = now_s() - t_fusion0;
  }
  if (!opt.keep_intermediate)   // the reference's clean-up (main.cpp:581-595)
    for (int pi : blocks[rank])
      for (int j = 0; j < round_num; j++) {
        std::error_code ec2;
        fs::remove(fs::path(problems[pi].result_folder) / ("edges_" + std::to_string(j) + ".dmb"), ec2);
        fs::remove(fs::path(problems[pi].result_folder) / ("labels_" + std::to_string(j) + ".dmb"), ec2);
      }
  if (opt.verbose && rank == 0) std::cout << "All done" << std::endl;
  g_times[4] = now_s() - t_mark;
  g_times[0] = now_s() - t_start;
  return 0;
}

}  // namespace
}  // namespace dpe_host

extern "C" {

void dpe_pipeline_default_options(DpePipelineOptions* o) {
  std::memset(o, 0, sizeof(*o));
  o->gpu_index = 0;
  o->verbose = true; o->fusion = false; o->viz = false;
  o->depth = true; o->normal = false; o->weak = false; o->edge = false;
  o->schedule = DPE_SCHEDULE_REFERENCE;
  o->rank = 0; o->world_size = 1;
  o->base_seed = 0x5EED;
}

int dpe_run_pipeline(const char* dense_folder, const DpePipelineOptions* opt) {
  DpePipelineOptions o;
  if (opt) o = *opt; else dpe_pipeline_default_options(&o);
  try {
    return dpe_host::run(dense_folder, o);
  } catch (const std::exception& e) {
    dpe_host::g_err = e.what();
    return 1;
  }
}

const char* dpe_pipeline_last_error(void) { return dpe_host::g_err.c_str(); }

int dpe_pipeline_last_timings(double* out, int n) {
  int k = 0;
  for (; k < n && k < dpe_host::kNumTimes; ++k) out[k] = dpe_host::g_times[k];
  return k;
}

}  // extern "C"
