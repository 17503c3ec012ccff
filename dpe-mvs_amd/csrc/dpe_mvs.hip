// dpe_mvs.hip — the C-ABI library (include/dpe_mvs.h): context, HBM staging and the launch
// sequence of one PatchMatch pass on gfx950.
//
// Replaces DPE::CudaSpaceInitialization / SetDataPassHelperInCuda / RunPatchMatch / getters
// (DPE.cpp:916-1121, DPE.cu:3126-3249).  Differences by design:
//   * no per-launch cudaDeviceSynchronize: the 26 launches are queued on one stream;
//   * device buffers persist in the context across passes (resized only when W/H/N grow);
//   * the bilinear texture path is a padded quad-texel image in HBM (one 16-B load per tap);
//   * cuRAND states (48 B/px + curand_init) are replaced by counter-based Philox;
//   * errors are return codes (no exit()).
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <map>
#include <vector>

#include "pass_kernels.h"
#include "pass_refine.h"
#include "pass_fusion.h"
#include "pass_sweep.h"
#include "pass_edges.h"
#include "tap_launch.h"

using namespace dpe;

static const int kDefaultXcdRows = 1;
static constexpr int kWeakLanes = 16;   // lanes per weak pixel in k_weak_coop

namespace {

thread_local std::string g_err;

// roctx ranges (SURVEY.md §5 tracing): host-side enqueue regions of the pass, visible in
// `rocprofv3 --marker-trace` beside the kernel trace
struct Range {
  explicit Range(const char* m) { roctxRangePushA(m); }
  ~Range() { roctxRangePop(); }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;
};

#define HIPC(expr)                                                                  \
  do {                                                                              \
    hipError_t e_ = (expr);                                                         \
    if (e_ != hipSuccess) {                                                         \
      g_err = std::string(#expr) + ": " + hipGetErrorString(e_);                    \
      return DPE_ERR_HIP;                                                           \
    }                                                                               \
  } while (0)

template <class T>
struct DevArr {
  T* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t count) {
    if (count <= n && p) return hipSuccess;
    if (p) { (void)hipFree(p); p = nullptr; n = 0; }
    hipError_t e = hipMalloc((void**)&p, count * sizeof(T) + 256);
    if (e == hipSuccess) n = count;
    return e;
  }
  void release() { if (p) (void)hipFree(p); p = nullptr; n = 0; }
};

}  // namespace

// An image kept in HBM across passes (DpePassInput.image_ids): its f32 grey levels and the gather
// layouts built from them.
struct CachedImage {
  int id = 0, W = 0, H = 0;
  int cls = IMG_F32;          // ImgClass of the grey levels
  DevArr<float> plain;
  DevArr<uint32_t> q8;      // TEX_U8 quad texels (8-bit images)
  DevArr<uint2> q16;        // TEX_F16 quad texels (8-bit images)
  DevArr<uint32_t> qp;      // TEX_P16 column pairs (8-bit images)
  DevArr<float4> qf;        // f32 quad texels (built on demand)
  uint64_t last_use = 0;
  size_t bytes() const { return plain.n * 4 + q8.n * 4 + q16.n * 8 + qp.n * 4 + qf.n * 16; }
  void release() { plain.release(); q8.release(); q16.release(); qp.release(); qf.release(); }
};

// Per-image pipeline state kept in HBM between passes (the reference's depths.dmb / normals.dmb /
// weak.bin / selected_views.bin round trip, main.cpp:439-446 -> DPE.cpp:826-911).
struct ResState {
  int w = 0, h = 0;
  bool full = false;          // planes / weak / sel of a pass of this image; false: depth only (imported)
  DevArr<float4> planes;      // (world normal xyz, depth) after the ProcessProblem epilogue
  DevArr<uint8_t> weak;
  DevArr<uint32_t> sel;
  DevArr<float> snap;         // depth snapshot for the Jacobi schedule (dpe_state_snapshot)
  int snap_w = 0, snap_h = 0;
  bool has_snap = false;
  void release() { planes.release(); weak.release(); sel.release(); snap.release(); }
};

struct DpeContext {
  int device = 0;
  std::map<int, ResState*> rstore;
  DevArr<float> xbuf[2];             // dpe_device_buffer: exchange buffers of the multi-rank schedule
  // EdgeSegment stages (dpe_canny / dpe_resize_* / dpe_roberts_threshold): scratch
  DevArr<uint8_t> e_a, e_b, e_map;
  DevArr<float> e_fa, e_fb;
  DevArr<int> e_rows, e_mag, e_itab;
  DevArr<int16_t> e_dx, e_dy;
  DevArr<float> e_ftab;
  DevArr<short> e_stab;
  bool snap_mode = false;            // stage_resident reads source depths from the Jacobi snapshots
  std::vector<CachedImage*> icache;
  uint64_t icache_clock = 0;
  hipStream_t stream = nullptr;
  hipStream_t aux = nullptr;         // GenNeighbours beside the first strong half-sweep
  hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_ei = nullptr;
  hipEvent_t ev_done = nullptr;      // end of the last dpe_pm_execute's work on its stream
  bool pending = false;              // ev_done recorded and not yet waited for
  bool staged = false;
  bool gn_done_for_stage = false;    // DPE_DBG_GN_ONCE (timing experiments): GenNeighbours' outputs kept
  bool timing = false;
  bool counting = false;
  int gn_slots = 0;                  // DPE_OPT_GN_SLOTS (0 = by rotate_time)
  float timings[DPE_NUM_CLASSES + 1] = {0};
  int launches[DPE_NUM_CLASSES + 1] = {0};
  unsigned long long counts[DPE_NUM_CLASSES * 4] = {0};
  std::vector<hipEvent_t> ev;        // timing: (start, end) per launch class slot
  hipEvent_t ev_start = nullptr;     // timing: start of the pass
  DevArr<unsigned long long> cnt;
  DevArr<unsigned long long> phase;  // DPE_PHASE_PROF builds: per-phase cycle sums
  PassConst hc;                  // host copy of the pass constants
  DevArr<PassConst> dc;
  // inputs
  DevArr<float> img_plain[DPE_MAX_IMAGES];  // plain f32 images (ref used directly)
  DevArr<float4> imgq[DPE_MAX_IMAGES];
  DevArr<uint32_t> imgq8_all;        // all 8-bit quad images, TEX_U8 layout, one allocation
  DevArr<uint2> imgq16_all;          //   and TEX_F16 layout (32-bit tap offsets)
  DevArr<uint32_t> imgqp_all;        //   and TEX_P16 column pairs
  int img_cls = IMG_F32;             // ImgClass of the pass (the widest class of its views)
  DevArr<float> depth[DPE_MAX_IMAGES];
  DevArr<uint8_t> edge, edge_low;
  DevArr<int> label;
  // staged initial state
  DevArr<float4> planes0;
  DevArr<uint8_t> weak0;
  DevArr<uint32_t> sel0;
  // working state
  DevArr<float4> planes, planes_snap, fit_plane;
  DevArr<float> costs, costs_snap, complex_;
  DevArr<uint32_t> sel, sel_snap;
  DevArr<uint8_t> weak, weak_rel, vw;
  DevArr<short2> nb, nearest, edge_neigh, lab_bound;
  DevArr<int> radius;
  DevArr<int> tab_right, tab_down;   // FindNearestStrongPoint tables
  DevArr<int> gn_ovf;                // GenNeighbours pixels left to the scratch kernel (k_gen_neighbours_lds)
  DevArr<float> gn_complex;          // DPE_DBG_GN_ONCE: complex_ after GenNeighbours
  DevArr<float> gn_tab;              // normalised image coordinates per column / row (k_gn_tables)
  DevArr<int> lists, row_counts, list_totals;   // per-colour pixel lists for the sweeps
  DevArr<int> part_cnt;                          // per colour: chunk counts / offsets of the weak-list partition
  DevBufs bufs;
  // fusion (dpe_fusion_stage / dpe_fusion_candidates)
  std::vector<DevArr<float>> fz_depth, fz_normal;
  std::vector<FusionViewDev> fz_host;
  DevArr<FusionViewDev> fz_views;
  DevArr<DpeCamera> fz_cams;
  DevArr<int> fz_src;
  DevArr<int32_t> fz_idx;
  DevArr<float> fz_val;
  int fz_n = 0;
};

extern "C" {

void dpe_params_default(DpePatchMatchParams* p) {   // main.h:78-106
  p->max_iterations = 3;
  p->num_images = 5;
  p->sigma_spatial = 5.0f;
  p->sigma_color = 3.0f;
  p->top_k = 4;
  p->depth_min = 0.0f;
  p->depth_max = 1.0f;
  p->geom_consistency = false;
  p->strong_radius = 5;
  p->strong_increment = 2;
  p->weak_radius = 5;
  p->weak_increment = 5;
  p->use_APD = true;
  p->use_edge = true;
  p->use_limit = true;
  p->use_label = true;
  p->use_radius = true;
  p->high_res_img = true;
  p->max_scale_size = 1;
  p->scale_size = 1;
  p->weak_peak_radius = 2;
  p->rotate_time = 4;
  p->ransac_threshold = 0.005f;
  p->geom_factor = 0.2f;
  p->state = DPE_FIRST_INIT;
}

const char* dpe_last_error(void) { return g_err.c_str(); }

DpeContext* dpe_create(int device) {
  g_err.clear();
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
    g_err = "dpe_create: no such HIP device";
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) { g_err = "dpe_create: hipSetDevice failed"; return nullptr; }
  DpeContext* c = new DpeContext();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    g_err = "dpe_create: stream"; delete c; return nullptr;
  }
  if (hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_ei, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreate(&c->ev_start) != hipSuccess) {
    g_err = "dpe_create: aux stream";
    if (c->ev_start) (void)hipEventDestroy(c->ev_start);
    if (c->ev_done) (void)hipEventDestroy(c->ev_done);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->ev_ei) (void)hipEventDestroy(c->ev_ei);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->aux) (void)hipStreamDestroy(c->aux);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return nullptr;
  }
  return c;
}

// Host-waits for the work of the last dpe_pm_execute, which may have been enqueued on a caller
// stream: staging, fetching and freeing must not overwrite or release buffers that pass still uses.
static hipError_t wait_pending(DpeContext* c) {
  hipError_t e = hipSuccess;
  if (c->pending) { e = hipEventSynchronize(c->ev_done); c->pending = false; }
  return e;
}

void dpe_image_cache_clear(DpeContext* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)wait_pending(c);
  (void)hipStreamSynchronize(c->stream);
  for (CachedImage* e : c->icache) { e->release(); delete e; }
  c->icache.clear();
}

void dpe_destroy(DpeContext* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)wait_pending(c);
  (void)hipStreamSynchronize(c->stream);
  (void)hipStreamSynchronize(c->aux);
  dpe_image_cache_clear(c);
  for (auto& a : c->fz_depth) a.release();
  for (auto& a : c->fz_normal) a.release();
  c->fz_views.release(); c->fz_cams.release(); c->fz_src.release(); c->fz_idx.release(); c->fz_val.release();
  for (auto& e : c->ev) (void)hipEventDestroy(e);
  (void)hipEventDestroy(c->ev_start);
  (void)hipEventDestroy(c->ev_done);
  c->dc.release();
  for (int i = 0; i < DPE_MAX_IMAGES; ++i) { c->img_plain[i].release(); c->imgq[i].release(); c->depth[i].release(); }
  c->imgq8_all.release();
  c->imgq16_all.release();
  c->imgqp_all.release();
  c->edge.release(); c->edge_low.release(); c->label.release();
  c->planes0.release(); c->weak0.release(); c->sel0.release();
  c->planes.release(); c->planes_snap.release(); c->fit_plane.release();
  c->costs.release(); c->costs_snap.release(); c->complex_.release();
  c->sel.release(); c->sel_snap.release();
  c->weak.release(); c->weak_rel.release(); c->vw.release();
  c->nb.release(); c->nearest.release(); c->edge_neigh.release(); c->lab_bound.release();
  c->radius.release();
  for (auto& kv : c->rstore) { kv.second->release(); delete kv.second; }
  c->rstore.clear();
  c->xbuf[0].release(); c->xbuf[1].release();
  c->e_a.release(); c->e_b.release(); c->e_map.release(); c->e_fa.release(); c->e_fb.release();
  c->e_rows.release(); c->e_mag.release(); c->e_itab.release(); c->e_dx.release(); c->e_dy.release();
  c->e_ftab.release(); c->e_stab.release();
  c->cnt.release();
  c->tab_right.release(); c->tab_down.release(); c->gn_ovf.release(); c->gn_tab.release(); c->gn_complex.release();
  c->lists.release(); c->row_counts.release(); c->list_totals.release(); c->part_cnt.release();
  (void)hipStreamSynchronize(c->aux);
  (void)hipEventDestroy(c->ev_fork); (void)hipEventDestroy(c->ev_join); (void)hipEventDestroy(c->ev_ei);
  (void)hipStreamDestroy(c->aux);
  (void)hipStreamDestroy(c->stream);
  delete c;
}

void dpe_set_timing(DpeContext* c, int enable) { if (c) c->timing = enable != 0; }

}  // extern "C"

// Per-pass constants (restatement of ComputeHomography's plane-independent part, DPE.cu:455-512,
// evaluated in double and rounded once; GenNeighbours' angle constants, DPE.cu:2147-2152).
static void compute_pass_constants(PassConst& pc) {
  const DpeCamera& rc = pc.cams[0];
  const double rK0 = rc.K[0], rK2 = rc.K[2], rK4 = rc.K[4], rK5 = rc.K[5];
  double refC[3];
  for (int j = 0; j < 3; ++j)
    refC[j] = -((double)rc.R[0 + j] * rc.t[0] + (double)rc.R[3 + j] * rc.t[1] + (double)rc.R[6 + j] * rc.t[2]);
  for (int v = 1; v < pc.N; ++v) {
    const DpeCamera& sc = pc.cams[v];
    double srcC[3], Rrel[9], Crel[3], trel[3], T[9];
    for (int j = 0; j < 3; ++j)
      srcC[j] = -((double)sc.R[0 + j] * sc.t[0] + (double)sc.R[3 + j] * sc.t[1] + (double)sc.R[6 + j] * sc.t[2]);
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c)
        Rrel[r * 3 + c] = (double)sc.R[r * 3 + 0] * rc.R[c * 3 + 0] + (double)sc.R[r * 3 + 1] * rc.R[c * 3 + 1] +
                          (double)sc.R[r * 3 + 2] * rc.R[c * 3 + 2];
    for (int j = 0; j < 3; ++j) Crel[j] = refC[j] - srcC[j];
    for (int r = 0; r < 3; ++r)
      trel[r] = (double)sc.R[r * 3 + 0] * Crel[0] + (double)sc.R[r * 3 + 1] * Crel[1] + (double)sc.R[r * 3 + 2] * Crel[2];
    for (int r = 0; r < 3; ++r) {
      T[r * 3 + 0] = Rrel[r * 3 + 0] / rK0;
      T[r * 3 + 1] = Rrel[r * 3 + 1] / rK4;
      T[r * 3 + 2] = -Rrel[r * 3 + 0] * rK2 / rK0 - Rrel[r * 3 + 1] * rK5 / rK4 + Rrel[r * 3 + 2];
    }
    const double sK0 = sc.K[0], sK2 = sc.K[2], sK4 = sc.K[4], sK5 = sc.K[5], sK8 = sc.K[8];
    for (int c = 0; c < 3; ++c) {
      pc.vc[v].M[0 + c] = (float)(sK0 * T[0 + c] + sK2 * T[6 + c]);
      pc.vc[v].M[3 + c] = (float)(sK4 * T[3 + c] + sK5 * T[6 + c]);
      pc.vc[v].M[6 + c] = (float)(sK8 * T[6 + c]);
    }
    pc.vc[v].b[0] = (float)(sK0 * trel[0] + sK2 * trel[2]);
    pc.vc[v].b[1] = (float)(sK4 * trel[1] + sK5 * trel[2]);
    pc.vc[v].b[2] = (float)(sK8 * trel[2]);
  }
  pc.kinv0 = (float)(1.0 / rK0);
  pc.kinv4 = (float)(1.0 / rK4);
  pc.kc2 = (float)(rK2 / rK0);
  pc.kc5 = (float)(rK5 / rK4);
  const float angle = 45.0f / pc.P.rotate_time;
  pc.gn_cos = (float)cos((double)angle * M_PI / 180.f);
  pc.gn_sin = (float)sin((double)angle * M_PI / 180.f);
  pc.gn_thr = (float)cos((double)(angle / 2.0f) * M_PI / 180.0f);
  const double sr = tan((double)(angle / 2.0f) * M_PI / 180.0f) * 20;
  const int sri = (sr != sr) ? 0 : (int)sr;
  pc.gn_shift = sri < 1 ? 1 : sri;
  pc.half_rows = std::min(pc.H, 2 * 16 * (((pc.H / 2) + 15) / 16));
  pc.weak_nn = pc.P.weak_radius >= 0 && pc.P.weak_increment > 0 ? (2 * pc.P.weak_radius) / pc.P.weak_increment + 1 : 0;
}

// where a stage takes the initial state and the source depths from: host buffers (dpe_pm_stage) or
// the resident store (dpe_pm_stage_resident)
struct StageSrc {
  const DpePassState* st = nullptr;   // host initial state
  const ResState* prior = nullptr;    // resident initial state (nullptr: none, FIRST_INIT)
  const ResState* dep[DPE_MAX_IMAGES] = {};   // resident source depths (index 1..N-1)
  bool dep_snap = false;              // read the depths' Jacobi snapshots
};
static int stage_impl(DpeContext* c, const DpePassInput* in, const StageSrc& src);

#if DPE_POOL_STATS
extern "C" void dpe_dbg_pool_stats_main(unsigned long long out[24], int reset) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(dpe::g_pool), sizeof(dpe::g_pool));
  if (reset) { unsigned long long z[24] = {}; (void)hipMemcpyToSymbol(HIP_SYMBOL(dpe::g_pool), z, sizeof(z)); }
}
#endif
#if DPE_LINE_STATS
extern "C" void dpe_dbg_line_stats_main(unsigned long long out[16], int reset) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(dpe::g_lstat), sizeof(dpe::g_lstat));
  if (reset) { unsigned long long z[16] = {}; (void)hipMemcpyToSymbol(HIP_SYMBOL(dpe::g_lstat), z, sizeof(z)); }
}
#endif
#if DPE_GN_TIMES
extern "C" void dpe_dbg_gn_times(unsigned int* out, int n) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(dpe::g_gntime), sizeof(unsigned int) * (size_t)(n < (2 << 20) ? n : (2 << 20)));
}
extern "C" void dpe_dbg_gn_counts(unsigned int* out, int n) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(dpe::g_gncnt), sizeof(unsigned int) * (size_t)(n < (6 << 20) ? n : (6 << 20)));
}
#endif
#if DPE_WEAK_STATS
extern "C" void dpe_dbg_weak_stats(unsigned long long out[24], int reset) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(dpe::g_wstat), sizeof(dpe::g_wstat));
  if (reset) { unsigned long long z[24] = {}; (void)hipMemcpyToSymbol(HIP_SYMBOL(dpe::g_wstat), z, sizeof(z)); }
}
#endif

extern "C" int dpe_pm_stage(DpeContext* c, const DpePassInput* in, const DpePassState* st) {
  g_err.clear();
  if (!c || !in || !st || !in->images || !in->cams || !st->planes || !st->weak_info || !st->selected_views) {
    g_err = "dpe_pm_stage: null argument"; return DPE_ERR_ARG;
  }
  if (in->params.geom_consistency) {
    if (!in->depths) { g_err = "dpe_pm_stage: geom_consistency needs depths"; return DPE_ERR_ARG; }
    for (int i = 1; i < in->num_images; ++i) if (!in->depths[i]) { g_err = "dpe_pm_stage: missing source depth"; return DPE_ERR_ARG; }
  }
  StageSrc src;
  src.st = st;
  return stage_impl(c, in, src);
}

template <class T>
__global__ void k_rescale_nearest(const T* __restrict__ src, int w, int h, T* __restrict__ dst, int nw, int nh, T zero) {
  // RescaleMatToTargetSize (DPE.cpp:1146-1165) with its swapped factors, as host rescale_nearest
  const int c = blockIdx.x * blockDim.x + threadIdx.x, r = blockIdx.y * blockDim.y + threadIdx.y;
  if (c >= nw || r >= nh) return;
  const float scale_x = nw / (float)w, scale_y = nh / (float)h;
  const int o_r = (int)(r / scale_x), o_c = (int)(c / scale_y);
  dst[(size_t)r * nw + c] = (o_r < 0 || o_c < 0 || o_r >= h || o_c >= w) ? zero : src[(size_t)o_r * w + o_c];
}
__global__ void k_rescale_depth(const float4* __restrict__ src, int w, int h, float* __restrict__ dst, int nw, int nh) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x, r = blockIdx.y * blockDim.y + threadIdx.y;
  if (c >= nw || r >= nh) return;
  const float scale_x = nw / (float)w, scale_y = nh / (float)h;
  const int o_r = (int)(r / scale_x), o_c = (int)(c / scale_y);
  dst[(size_t)r * nw + c] = (o_r < 0 || o_c < 0 || o_r >= h || o_c >= w) ? 0.0f : src[(size_t)o_r * w + o_c].w;
}

extern "C" int dpe_pm_stage_resident(DpeContext* c, const DpePassInput* in, int prior_id) {
  g_err.clear();
  if (!c || !in || !in->images || !in->cams) { g_err = "dpe_pm_stage_resident: null argument"; return DPE_ERR_ARG; }
  const DpePatchMatchParams& P = in->params;
  StageSrc src;
  auto find = [&](int id) -> ResState* { auto it = c->rstore.find(id); return it == c->rstore.end() ? nullptr : it->second; };
  if (P.state != DPE_FIRST_INIT || P.use_APD) {
    src.prior = find(prior_id);
    if (!src.prior || !src.prior->full) {
      g_err = "dpe_pm_stage_resident: no resident state of image " + std::to_string(prior_id); return DPE_ERR_STATE;
    }
  }
  if (P.geom_consistency) {
    if (!in->image_ids) { g_err = "dpe_pm_stage_resident: geom_consistency needs image_ids"; return DPE_ERR_ARG; }
    for (int i = 1; i < in->num_images && i < DPE_MAX_IMAGES; ++i) {
      src.dep[i] = find(in->image_ids[i]);
      if (!src.dep[i]) { g_err = "no depth map of source image " + std::to_string(in->image_ids[i]); return DPE_ERR_STATE; }
    }
    src.dep_snap = c->snap_mode;
    if (src.dep_snap)
      for (int i = 1; i < in->num_images && i < DPE_MAX_IMAGES; ++i)
        if (!src.dep[i]->has_snap) { g_err = "no depth snapshot of source image " + std::to_string(in->image_ids[i]); return DPE_ERR_STATE; }
  }
  return stage_impl(c, in, src);
}

static int stage_impl(DpeContext* c, const DpePassInput* in, const StageSrc& src) {
  g_err.clear();
  Range range_(src.st ? "dpe_pm_stage" : "dpe_pm_stage_resident");
  const DpePassState* st = src.st;
  if (in->num_images > DPE_MAX_IMAGES) { g_err = "dpe_pm_stage: num_images > 32 (DPE.cpp:762)"; return DPE_ERR_TOO_MANY; }
  if (in->num_images < 2 || in->width <= 0 || in->height <= 0) { g_err = "dpe_pm_stage: bad shape"; return DPE_ERR_ARG; }
  if (in->width > 32000 || in->height > 32000) { g_err = "dpe_pm_stage: image too large for short2 coordinates"; return DPE_ERR_ARG; }
  // tap coordinates on the unit grid of [2^23, 2^24) (pass_common.h kTexMagic): 256 (lim + 1) < 2^22
  if (in->width > 16000 || in->height > 16000) { g_err = "dpe_pm_stage: image wider or taller than 16000 px"; return DPE_ERR_ARG; }
  const DpePatchMatchParams& P = in->params;
  if (P.rotate_time < 1 || P.rotate_time > 4) { g_err = "dpe_pm_stage: rotate_time must be in [1,4]"; return DPE_ERR_ARG; }
  if (P.strong_increment <= 0 || P.weak_increment <= 0) { g_err = "dpe_pm_stage: increments must be > 0"; return DPE_ERR_ARG; }
  for (int i = 0; i < in->num_images; ++i) if (!in->images[i]) { g_err = "dpe_pm_stage: missing image"; return DPE_ERR_ARG; }
  if ((P.use_edge || P.use_limit) && (!in->edge || !in->edge_low_res || in->low_width <= 0 || in->low_height <= 0)) {
    g_err = "dpe_pm_stage: use_edge/use_limit need edge and edge_low_res"; return DPE_ERR_ARG;
  }
  if (P.use_label && !in->label) { g_err = "dpe_pm_stage: use_label needs label"; return DPE_ERR_ARG; }
  HIPC(hipSetDevice(c->device));
  HIPC(wait_pending(c));   // an earlier execute on a caller stream may still read what is overwritten here
  const int W = in->width, H = in->height, N = in->num_images;
  const size_t L = (size_t)W * H;
  PassConst& pc = c->hc;
  std::memset(&pc, 0, sizeof(pc));
  pc.W = W; pc.H = H; pc.N = N;
  pc.P = P; pc.P.num_images = N;
  pc.seed32 = (uint32_t)in->seed ^ (uint32_t)(in->seed >> 32);
  pc.salt = in->pass_salt;
  for (int i = 0; i < N; ++i) pc.cams[i] = in->cams[i];
  compute_pass_constants(pc);
  HIPC(c->dc.ensure(1));
  HIPC(hipMemcpyAsync(c->dc.p, &pc, sizeof(PassConst), hipMemcpyHostToDevice, c->stream));

  DevBufs& B = c->bufs;
  std::memset(&B, 0, sizeof(B));
  const dim3 qb(16, 16), qg((W + 2 + 15) / 16, (H + 2 + 15) / 16);
  // The half-precision layouts hold every grey level exactly when it is a multiple of 1/4 in
  // [0, 255] (IMG_Q: the exact 1/2 and 1/4 INTER_LINEAR downscales of an 8-bit image, the coarse
  // pyramid levels of every BASELINE config; the differences b - a of the F16 / P16 texels are then
  // exact too); the u8 layout needs integers (IMG_U8: images decoded from 8-bit files).  Identical
  // sample values in every layout; the smaller ones gather fewer bytes.
  auto image_class = [&](const float* im) -> int {
    bool integer = true;
    for (size_t k = 0; k < L; ++k) {
      const float v = im[k];
      if (!(v >= 0.0f && v <= 255.0f)) return IMG_F32;
      const float v4 = v * 4.0f;   // exact (power of two)
      if (v4 != (float)(int)v4) return IMG_F32;
      integer = integer && v == (float)(int)v;
    }
    return integer ? IMG_U8 : IMG_Q;
  };
  const size_t plane = (size_t)(W + 2) * (H + 2);
  const size_t pplane = (size_t)(W + 3) * (H + 2);        // TEX_P16
  const dim3 pg((W + 3 + 15) / 16, (H + 2 + 15) / 16);
  if (in->image_ids) {   // device-resident images: upload and build layouts once per (id, size)
    CachedImage* ent[DPE_MAX_IMAGES];
    const uint64_t call_clock = c->icache_clock;   // entries used by this call have last_use > call_clock
    for (int i = 0; i < N; ++i) {
      CachedImage* e = nullptr;
      for (CachedImage* q : c->icache)
        if (q->id == in->image_ids[i] && q->W == W && q->H == H) { e = q; break; }
      if (!e) {
        size_t total = 0;   // keep the cache under 64 GiB: evict least recently used entries, never one
        for (CachedImage* q : c->icache) total += q->bytes();   // this call already placed in ent[]
        while (total > (64ull << 30)) {
          auto lru = c->icache.end();
          for (auto it = c->icache.begin(); it != c->icache.end(); ++it)
            if ((*it)->last_use <= call_clock && (lru == c->icache.end() || (*it)->last_use < (*lru)->last_use)) lru = it;
          if (lru == c->icache.end()) break;   // only this pass's own views are cached: keep them
          HIPC(hipStreamSynchronize(c->stream));
          total -= (*lru)->bytes();
          (*lru)->release(); delete *lru; c->icache.erase(lru);
        }
        e = new CachedImage();
        e->id = in->image_ids[i]; e->W = W; e->H = H;
        e->cls = image_class(in->images[i]);
        c->icache.push_back(e);
        HIPC(e->plain.ensure(L));
        HIPC(hipMemcpyAsync(e->plain.p, in->images[i], L * sizeof(float), hipMemcpyHostToDevice, c->stream));
        if (e->cls != IMG_F32) {
          if (e->cls == IMG_U8) HIPC(e->q8.ensure(plane));
          HIPC(e->q16.ensure(plane)); HIPC(e->qp.ensure(pplane));
          k_build_quad8<<<qg, qb, 0, c->stream>>>(e->plain.p, e->cls == IMG_U8 ? e->q8.p : nullptr, e->q16.p, W, H);
          k_build_pair16<<<pg, qb, 0, c->stream>>>(e->plain.p, e->qp.p, W, H);
          HIPC(hipGetLastError());
        }
      }
      e->last_use = ++c->icache_clock;
      ent[i] = e;
    }
    int cls = (size_t)(W + 2) * (H + 2) * 8 * N < (1ull << 32) ? IMG_U8 : IMG_F32;   // 32-bit tap offsets
    for (int i = 0; i < N; ++i) cls = std::min(cls, ent[i]->cls);
    c->img_cls = cls;
    if (cls != IMG_F32) {
      if (cls == IMG_U8) HIPC(c->imgq8_all.ensure(plane * N));
      HIPC(c->imgq16_all.ensure(plane * N));
      HIPC(c->imgqp_all.ensure(pplane * N));
      for (int i = 0; i < N; ++i) {   // the per-pass views in one allocation (32-bit tap offsets)
        if (cls == IMG_U8)
          HIPC(hipMemcpyAsync(c->imgq8_all.p + plane * i, ent[i]->q8.p, plane * 4, hipMemcpyDeviceToDevice, c->stream));
        HIPC(hipMemcpyAsync(c->imgq16_all.p + plane * i, ent[i]->q16.p, plane * 8, hipMemcpyDeviceToDevice, c->stream));
        HIPC(hipMemcpyAsync(c->imgqp_all.p + pplane * i, ent[i]->qp.p, pplane * 4, hipMemcpyDeviceToDevice, c->stream));
      }
      if (cls == IMG_U8) { B.img8 = (const uint8_t*)c->imgq8_all.p; B.img8_view = (uint32_t)(plane * 4); }
      B.img16 = (const uint8_t*)c->imgq16_all.p; B.img16_view = (uint32_t)(plane * 8);
      B.imgp = (const uint8_t*)c->imgqp_all.p; B.imgp_view = (uint32_t)(pplane * 4);
    } else {
      for (int i = 0; i < N; ++i) {
        if (!ent[i]->qf.p) {
          HIPC(ent[i]->qf.ensure(plane));
          k_build_quad<<<qg, qb, 0, c->stream>>>(ent[i]->plain.p, ent[i]->qf.p, W, H);
          HIPC(hipGetLastError());
        }
        B.imgq[i] = ent[i]->qf.p;
      }
    }
    B.ref = ent[0]->plain.p;
  }
  int cls = IMG_U8;
  for (int i = 0; i < N && cls != IMG_F32 && !in->image_ids; ++i) cls = std::min(cls, image_class(in->images[i]));
  if ((size_t)(W + 2) * (H + 2) * 8 * N >= (1ull << 32)) cls = IMG_F32;   // 32-bit tap offsets
  if (!in->image_ids) c->img_cls = cls;
  for (int i = 0; i < N && !in->image_ids; ++i) {
    HIPC(c->img_plain[i].ensure(L));
    HIPC(hipMemcpyAsync(c->img_plain[i].p, in->images[i], L * sizeof(float), hipMemcpyHostToDevice, c->stream));
    if (cls != IMG_F32) {
      if (cls == IMG_U8) HIPC(c->imgq8_all.ensure(plane * N));
      HIPC(c->imgq16_all.ensure(plane * N));
      HIPC(c->imgqp_all.ensure(pplane * N));
      k_build_quad8<<<qg, qb, 0, c->stream>>>(c->img_plain[i].p, cls == IMG_U8 ? c->imgq8_all.p + plane * i : nullptr,
                                              c->imgq16_all.p + plane * i, W, H);
      k_build_pair16<<<pg, qb, 0, c->stream>>>(c->img_plain[i].p, c->imgqp_all.p + pplane * i, W, H);
      if (cls == IMG_U8) {
        B.img8 = (const uint8_t*)c->imgq8_all.p;
        B.img8_view = (uint32_t)(plane * 4);
      }
      B.img16 = (const uint8_t*)c->imgq16_all.p;
      B.img16_view = (uint32_t)(plane * 8);
      B.imgp = (const uint8_t*)c->imgqp_all.p;
      B.imgp_view = (uint32_t)(pplane * 4);
    } else {
      HIPC(c->imgq[i].ensure((size_t)(W + 2) * (H + 2)));
      k_build_quad<<<qg, qb, 0, c->stream>>>(c->img_plain[i].p, c->imgq[i].p, W, H);
      B.imgq[i] = c->imgq[i].p;
    }
    HIPC(hipGetLastError());
  }
  if (!in->image_ids) B.ref = c->img_plain[0].p;
  const dim3 rb2(32, 8), rg2((W + 31) / 32, (H + 7) / 8);
  if (P.geom_consistency) {
    for (int i = 1; i < N; ++i) {
      HIPC(c->depth[i].ensure(L));
      if (st) {
        HIPC(hipMemcpyAsync(c->depth[i].p, in->depths[i], L * sizeof(float), hipMemcpyHostToDevice, c->stream));
      } else {
        const ResState* r = src.dep[i];
        if (src.dep_snap)
          k_rescale_nearest<float><<<rg2, rb2, 0, c->stream>>>(r->snap.p, r->snap_w, r->snap_h, c->depth[i].p, W, H, 0.0f);
        else
          k_rescale_depth<<<rg2, rb2, 0, c->stream>>>(r->planes.p, r->w, r->h, c->depth[i].p, W, H);
        HIPC(hipGetLastError());
      }
      B.depth[i] = c->depth[i].p;
    }
  }
  if (P.use_edge || P.use_limit) {
    pc.LW = in->low_width; pc.LH = in->low_height;
    HIPC(c->edge.ensure(L));
    HIPC(c->edge_low.ensure((size_t)pc.LW * pc.LH));
    HIPC(hipMemcpyAsync(c->edge.p, in->edge, L, hipMemcpyHostToDevice, c->stream));
    HIPC(hipMemcpyAsync(c->edge_low.p, in->edge_low_res, (size_t)pc.LW * pc.LH, hipMemcpyHostToDevice, c->stream));
    B.edge = c->edge.p; B.edge_low = c->edge_low.p;
    HIPC(hipMemcpyAsync(c->dc.p, &pc, sizeof(PassConst), hipMemcpyHostToDevice, c->stream));
  }
  if (P.use_label) {
    HIPC(c->label.ensure(L));
    HIPC(hipMemcpyAsync(c->label.p, in->label, L * sizeof(int), hipMemcpyHostToDevice, c->stream));
    B.label = c->label.p;
  }
  HIPC(c->planes0.ensure(L)); HIPC(c->weak0.ensure(L)); HIPC(c->sel0.ensure(L));
  if (st) {
    HIPC(hipMemcpyAsync(c->planes0.p, st->planes, L * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    if (P.use_APD) HIPC(hipMemcpyAsync(c->weak0.p, st->weak_info, L, hipMemcpyHostToDevice, c->stream));
    else HIPC(hipMemsetAsync(c->weak0.p, DPE_STRONG, L, c->stream));   // DPE.cpp:873-881
    HIPC(hipMemcpyAsync(c->sel0.p, st->selected_views, L * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
  } else {   // InuputInitialization's prior (DPE.cpp:845-911) from the resident state, rescaled on device
    const ResState* r = src.prior;
    if (P.state != DPE_FIRST_INIT) {
      k_rescale_nearest<float4><<<rg2, rb2, 0, c->stream>>>(r->planes.p, r->w, r->h, c->planes0.p, W, H, make_float4(0, 0, 0, 0));
      k_rescale_nearest<uint32_t><<<rg2, rb2, 0, c->stream>>>(r->sel.p, r->w, r->h, c->sel0.p, W, H, 0u);
    } else {
      HIPC(hipMemsetAsync(c->planes0.p, 0, L * sizeof(float4), c->stream));
      HIPC(hipMemsetAsync(c->sel0.p, 0, L * sizeof(uint32_t), c->stream));
    }
    if (P.use_APD) k_rescale_nearest<uint8_t><<<rg2, rb2, 0, c->stream>>>(r->weak.p, r->w, r->h, c->weak0.p, W, H, (uint8_t)0);
    else HIPC(hipMemsetAsync(c->weak0.p, DPE_STRONG, L, c->stream));
    HIPC(hipGetLastError());
  }
  HIPC(c->planes.ensure(L)); HIPC(c->planes_snap.ensure(L)); HIPC(c->fit_plane.ensure(L));
  HIPC(c->costs.ensure(L)); HIPC(c->costs_snap.ensure(L)); HIPC(c->complex_.ensure(L));
  HIPC(c->sel.ensure(L)); HIPC(c->sel_snap.ensure(L));
  HIPC(c->weak.ensure(L)); HIPC(c->weak_rel.ensure(L)); HIPC(c->vw.ensure(L * DPE_MAX_IMAGES));
  HIPC(c->nb.ensure(L * 9)); HIPC(c->nearest.ensure(L)); HIPC(c->edge_neigh.ensure(L * 8)); HIPC(c->lab_bound.ensure(L * 8));
  HIPC(c->radius.ensure(L));
  HIPC(c->tab_right.ensure(L)); HIPC(c->tab_down.ensure(L));
  HIPC(c->gn_ovf.ensure(L + 64)); HIPC(c->gn_tab.ensure((size_t)W + H));
  HIPC(c->lists.ensure(6 * (L / 2 + 64) + 3 * (L + 64))); HIPC(c->row_counts.ensure(4 * (size_t)H + 4)); HIPC(c->list_totals.ensure(16));
  HIPC(c->part_cnt.ensure(2 * ((L / 2 + 1) / kPartChunk + 2)));
  B.planes = c->planes.p; B.planes_snap = c->planes_snap.p; B.fit_plane = c->fit_plane.p;
  B.planes0 = c->planes0.p;
  B.costs = c->costs.p; B.costs_snap = c->costs_snap.p; B.complex_ = c->complex_.p;
  B.sel = c->sel.p; B.sel_snap = c->sel_snap.p;
  B.weak = c->weak.p; B.weak_rel = c->weak_rel.p; B.vw = c->vw.p;
  B.nb = c->nb.p; B.nearest = c->nearest.p; B.edge_neigh = c->edge_neigh.p; B.lab_bound = c->lab_bound.p;
  B.radius = c->radius.p;
  HIPC(hipStreamSynchronize(c->stream));
  c->staged = true;
  c->gn_done_for_stage = false;
  return DPE_OK;
}

// the pass's initial state in one launch: planes, weak_info and selected views from the staged
// copies, costs and view weights cleared
static_assert(DPE_MAX_IMAGES == 32, "k_pass_init clears 32 view-weight bytes per pixel");
__global__ void __launch_bounds__(256) k_pass_init(const uint4* __restrict__ planes0, const uint8_t* __restrict__ weak0,
                                                   const uint32_t* __restrict__ sel0, uint4* __restrict__ planes,
                                                   uint8_t* __restrict__ weak, uint32_t* __restrict__ sel,
                                                   uint32_t* __restrict__ costs, uint4* __restrict__ vw, size_t L) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= L) return;
  planes[i] = planes0[i];
  weak[i] = weak0[i];
  sel[i] = sel0[i];
  costs[i] = 0u;
  const uint4 z = make_uint4(0u, 0u, 0u, 0u);
  vw[2 * i] = z;
  vw[2 * i + 1] = z;
}

// the state a strong half-sweep reads its neighbours from (planes, costs, selected views before the
// sweep: the red/black same-colour semantics), the three copies in one launch
__global__ void __launch_bounds__(256) k_snapshot(const uint4* __restrict__ planes, const uint32_t* __restrict__ costs,
                                                  const uint32_t* __restrict__ sel, uint4* __restrict__ planes_s,
                                                  uint32_t* __restrict__ costs_s, uint32_t* __restrict__ sel_s, size_t L) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= L) return;
  planes_s[i] = planes[i];
  costs_s[i] = costs[i];
  sel_s[i] = sel[i];
}

extern "C" int dpe_pm_execute(DpeContext* c, void* stream_) {
  g_err.clear();
  if (!c) { g_err = "dpe_pm_execute: null context"; return DPE_ERR_ARG; }
  if (!c->staged) { g_err = "dpe_pm_execute: call dpe_pm_stage first"; return DPE_ERR_STATE; }
  Range range_("dpe_pm_execute");
  HIPC(hipSetDevice(c->device));
  hipStream_t s = stream_ ? (hipStream_t)stream_ : c->stream;
  // a previous execute, possibly on another stream, still uses the working buffers this one resets
  if (c->pending) HIPC(hipStreamWaitEvent(s, c->ev_done, 0));
  const PassConst& pc = c->hc;
  const PassConst* dpc = c->dc.p;
  const int W = pc.W, H = pc.H, nv = pc.N - 1;
  const size_t L = (size_t)W * H;
  DevBufs B = c->bufs;
  B.cnt = nullptr;
  {   // tuning knob: block rows per XCD chunk (see xcd_remap); DPE_XCD_ROWS=0 disables
    const char* e = getenv("DPE_XCD_ROWS");
    B.xcd_rows = e ? atoi(e) : kDefaultXcdRows;
  }
#if DPE_PHASE_PROF
  HIPC(c->phase.ensure(32 * 64));
  HIPC(hipMemsetAsync(c->phase.p, 0, 32 * 64 * sizeof(unsigned long long), s));
  B.phase = c->phase.p;
#endif
  if (c->counting) {
    HIPC(c->cnt.ensure(DPE_NUM_CLASSES * 4));
    HIPC(hipMemsetAsync(c->cnt.p, 0, DPE_NUM_CLASSES * 4 * sizeof(unsigned long long), s));
  }
  // per-launch events: slot pairs (start, end) + class id; one slot per class section of the
  // launch sequence (setup, init, 5 per iteration, filter, DepthToWeak, LocalRefine)
  const bool timing = c->timing;
  const int max_slots = 5 + 5 * std::max(0, pc.P.max_iterations);
  if (timing && (int)c->ev.size() < 2 * max_slots) {
    const size_t have = c->ev.size();
    c->ev.resize(2 * max_slots, nullptr);
    for (size_t k = have; k < c->ev.size(); ++k) HIPC(hipEventCreate(&c->ev[k]));
  }
  int nev = 0;
  bool slot_overflow = false;   // more timed sections than slots: fail the timed execute loudly
  std::vector<int> ev_class(timing ? max_slots : 0);
  for (int k = 0; k <= DPE_NUM_CLASSES; ++k) c->launches[k] = 0;
  static const char* const kClassName[DPE_NUM_CLASSES] = {"setup", "init", "strong", "ransac", "weak", "filter",
                                                           "depth_to_weak", "local_refine"};
  auto begin = [&](int cls) -> DevBufs {
    roctxRangePushA(kClassName[cls]);
    DevBufs Bc = B;
    if (c->counting) Bc.cnt = c->cnt.p + 4 * cls;
    c->launches[cls]++;
    if (timing && nev < max_slots) { ev_class[nev] = cls; (void)hipEventRecord(c->ev[2 * nev], s); }
    else if (timing) slot_overflow = true;
    return Bc;
  };
  auto end = [&]() {
    if (timing && nev < max_slots) { (void)hipEventRecord(c->ev[2 * nev + 1], s); nev++; }
    roctxRangePop();
  };

  if (timing) (void)hipEventRecord(c->ev_start, s);
  // DPE_DBG_GN_ONCE=1 (timing experiments only): GenNeighbours runs in the first execute after a stage
  // and its outputs (nb, weak_rel and complex_, which GenEdgeInform rewrites: restored after it) are kept for the next executes of the same staged state,
  // which then skip it -- the same results (GenNeighbours depends only on the staged state), and the
  // pass time without GenNeighbours on the critical path
  static const bool gn_once = [] { const char* e = getenv("DPE_DBG_GN_ONCE"); return e && atoi(e) == 1; }();
  const bool gn_skip = gn_once && c->gn_done_for_stage;
  // initial state (the reference uploads it in CudaSpaceInitialization, DPE.cpp:964-1015)
  k_pass_init<<<(unsigned)((L + 255) / 256), 256, 0, s>>>((const uint4*)c->planes0.p, c->weak0.p, c->sel0.p, (uint4*)B.planes,
                                                          B.weak, B.sel, (uint32_t*)B.costs, (uint4*)B.vw, L);
  // the rest of the initial state is first read by the setup chain (or, after it joins the pass
  // stream, by RANSACToGetFitPlane and the weak sweeps): it is cleared on the setup chain's stream
  auto clear_setup_state = [&](hipStream_t q) -> int {
    HIPC(hipMemsetAsync(B.fit_plane, 0, L * sizeof(float4), q));
    HIPC(hipMemsetAsync(B.complex_, 0, L * sizeof(float), q));
    if (!gn_skip) HIPC(hipMemsetAsync(B.weak_rel, 0xFF, L, q));   // GenNeighbours writes 0 / 1 for every WEAK pixel
    if (!gn_skip) HIPC(hipMemsetAsync(B.nb, 0xFF, L * 9 * sizeof(short2), q));
    HIPC(hipMemsetAsync(B.nearest, 0xFF, L * sizeof(short2), q));
    HIPC(hipMemsetAsync(B.edge_neigh, 0xFF, L * 8 * sizeof(short2), q));
    HIPC(hipMemsetAsync(B.lab_bound, 0xFF, L * 8 * sizeof(short2), q));
    HIPC(hipMemsetAsync(B.radius, 0, L * sizeof(int), q));
    return DPE_OK;
  };

  const dim3 fb(16, 16), fg((W + 15) / 16, (H + 15) / 16);
  const dim3 rb(16, kRansacThreads / 16), rg((W + 15) / 16, (H + rb.y - 1) / rb.y);
  const dim3 hb(32, 4), hg((((W + 1) / 2) + 31) / 32, (pc.half_rows + 3) / 4);

  DevBufs Bc;

  // RunPatchMatch launch sequence (DPE.cu:3150-3226)
  // DPE_OVERLAP=0 keeps one stream (profiling runs whose per-kernel durations must not overlap);
  // timed / counting executes keep one stream too (per-class events)
  static const bool overlap_env = [] { const char* e = getenv("DPE_OVERLAP"); return !(e && atoi(e) == 0); }();
  // (the join into `s` sits in the first strong half-sweep, so a pass without iterations keeps one stream)
  const bool overlap = overlap_env && !timing && !c->counting && pc.P.max_iterations >= 1;
  const long list_stride = (long)(L / 2 + 64);
  int* weak_list = c->lists.p + 4 * list_stride;     // all WEAK pixels (list_totals slot 4)
  int* failed_list = weak_list + L + 64;             // colour-0 pixels whose GenNeighbours failed (slot 5)
  int* side_lists = failed_list + list_stride;       // per colour: the weak list partitioned by patch side
  // The whole setup chain (GenEdgeInform, FindNearestStrongPoint's tables, the WEAK list,
  // GenNeighbours, NeigbourUpdate) runs on the aux stream `a`, forked at the start of the pass beside
  // RandomInitialization; the first strong half-sweep waits for GenEdgeInform's edge rays only.
  // GenNeighbours + NeigbourUpdate only decide which WEAK pixels join the strong lists; nothing the
  // first strong half-sweep (iteration 0, colour 0) or RandomInitialization reads is written by them,
  // and GenNeighbours reads the staged planes, not the ones those two rewrite.  So that half-sweep
  // runs over the pre-GenNeighbours colour-0 strong list, and the colour-0 pixels whose GenNeighbours
  // failed (NeigbourUpdate makes them UNKNOWN) get the same half-sweep (same snapshot) once the
  // streams join.  Pixels of one half-sweep are independent, so this is the reference's order of
  // results (GPU test test_overlapped_and_sequential_schedules_agree).
  const hipStream_t a = overlap ? c->aux : s;
  auto sweep_lists = [&](const DevBufs& Bl) {   // per-colour strong / weak lists of the sweeps
    k_list_count<0><<<(pc.half_rows + 3) / 4, 256, 0, s>>>(dpc, Bl, c->row_counts.p);
    k_list_scan<0><<<1, 256, 0, s>>>(dpc, c->row_counts.p, c->list_totals.p);
    k_list_fill<0><<<(pc.half_rows + 3) / 4, 256, 0, s>>>(dpc, Bl, c->row_counts.p, c->lists.p, list_stride);
  };
  Bc = begin(DPE_CLASS_SETUP);
  if (overlap) {   // pre-GenNeighbours sweep lists (the colour-0 strong list is the one used)
    sweep_lists(Bc);
    HIPC(hipEventRecord(c->ev_fork, s));
    HIPC(hipStreamWaitEvent(a, c->ev_fork, 0));
  }
  if (const int rc = clear_setup_state(a); rc != DPE_OK) return rc;
  k_gen_edge_inform<<<fg, fb, 0, a>>>(dpc, Bc);
  if (pc.P.use_edge) k_edge_rays<<<(unsigned)(3 * (W + H) - 2), 64, 0, a>>>(dpc, Bc);
  if (gn_skip) HIPC(hipMemcpyAsync(B.complex_, c->gn_complex.p, L * sizeof(float), hipMemcpyDeviceToDevice, a));
  if (overlap) HIPC(hipEventRecord(c->ev_ei, a));
  k_strong_tables_scan<<<(unsigned)(W + H), 64, 0, a>>>(dpc, Bc, c->tab_right.p, c->tab_down.p);
  k_find_nearest_strong<<<fg, fb, 0, a>>>(dpc, Bc, c->tab_right.p, c->tab_down.p);
  // list of all WEAK pixels, then GenNeighbours one thread per WEAK pixel
  k_list_count<1><<<(H + 3) / 4, 256, 0, a>>>(dpc, Bc, c->row_counts.p + 2 * (size_t)H + 2);
  k_list_scan<1><<<1, 64, 0, a>>>(dpc, c->row_counts.p + 2 * (size_t)H + 2, c->list_totals.p + 4);
  k_list_fill<1><<<(H + 3) / 4, 256, 0, a>>>(dpc, Bc, c->row_counts.p + 2 * (size_t)H + 2, weak_list, (long)L);
  if (gn_skip) {
  } else if (pc.P.rotate_time <= 4) {
    // the scratch-free kernel; pixels with more support points than its LDS slots (none at the
    // BASELINE workloads) or a NaN go to the scratch kernel, a small persistent grid that loops over
    // that overflow list (list_totals slot 6)
    k_gn_tables<<<(unsigned)((W + H + 255) / 256), 256, 0, a>>>(dpc, c->gn_tab.p);
    HIPC(hipMemsetAsync(c->list_totals.p + 6, 0, sizeof(int), a));
    const unsigned gg = (unsigned)((L + kGnBT - 1) / kGnBT);
    const int* cnt = c->list_totals.p + 4;
    if (c->gn_slots == 8)   // test setting: most pixels overflow into the scratch kernel
      k_gen_neighbours_lds<8><<<gg, kGnBT, 0, a>>>(dpc, Bc, weak_list, cnt, c->gn_tab.p, c->gn_ovf.p, c->list_totals.p + 6);
    else if (pc.P.rotate_time <= 2 && c->gn_slots != 64)   // at most 16 x rotate_time support points
      k_gen_neighbours_lds<32><<<gg, kGnBT, 0, a>>>(dpc, Bc, weak_list, cnt, c->gn_tab.p, c->gn_ovf.p, c->list_totals.p + 6);
    else
      k_gen_neighbours_lds<64><<<gg, kGnBT, 0, a>>>(dpc, Bc, weak_list, cnt, c->gn_tab.p, c->gn_ovf.p, c->list_totals.p + 6);
    k_gen_neighbours<<<kGnOvfBlocks, 256, 0, a>>>(dpc, Bc, c->gn_ovf.p, c->list_totals.p + 6);
  } else {
    k_gen_neighbours<<<kGnOvfBlocks, 256, 0, a>>>(dpc, Bc, weak_list, c->list_totals.p + 4);
  }
  if (gn_once && !gn_skip) {
    HIPC(c->gn_complex.ensure(L));
    HIPC(hipMemcpyAsync(c->gn_complex.p, B.complex_, L * sizeof(float), hipMemcpyDeviceToDevice, a));
    c->gn_done_for_stage = true;
  }
  k_neighbour_update<<<fg, fb, 0, a>>>(dpc, Bc);
  if (overlap) {
    k_list_count<2><<<(pc.half_rows + 3) / 4, 256, 0, a>>>(dpc, Bc, c->row_counts.p);
    k_list_scan<2><<<1, 64, 0, a>>>(dpc, c->row_counts.p, c->list_totals.p + 5);
    k_list_fill<2><<<(pc.half_rows + 3) / 4, 256, 0, a>>>(dpc, Bc, c->row_counts.p, failed_list, list_stride);
    HIPC(hipEventRecord(c->ev_join, a));
  } else {
    sweep_lists(Bc);   // weak_info is fixed from here until DepthToWeak
  }
  end();
  Bc = begin(DPE_CLASS_INIT);
  if (c->img_cls != IMG_F32) k_random_init<kTexInit><<<fg, fb, 0, s>>>(dpc, Bc); else k_random_init<TEX_F32><<<fg, fb, 0, s>>>(dpc, Bc);
  end();
  if (overlap) HIPC(hipStreamWaitEvent(s, c->ev_ei, 0));   // the strong sweeps read GenEdgeInform's rays
  HIPC(hipGetLastError());
  auto strong_sweep = [&](const DevBufs& Bs, int it, const int* lst, const int* cnt) {
    const bool edge = pc.P.use_edge;
    const int P = edge ? 4 : 8, C = edge ? 16 : 8;
    const size_t lds = (size_t)kBwStrong * strong_lds_per_wave(P, C, nv) * sizeof(float);
    const unsigned grid = (unsigned)((L / 2 + 1 + kBwStrong * P - 1) / (kBwStrong * P));
    launch_strong(edge, c->img_cls, grid, lds, s, dpc, Bs, it, lst, cnt);
  };
  for (int it = 0; it < pc.P.max_iterations; ++it) {
    for (int colour = 0; colour < 2; ++colour) {
      k_snapshot<<<(unsigned)((L + 255) / 256), 256, 0, s>>>((const uint4*)B.planes, (const uint32_t*)B.costs, B.sel,
                                                          (uint4*)B.planes_snap, (uint32_t*)B.costs_snap, B.sel_snap, L);
      Bc = begin(DPE_CLASS_STRONG);
      strong_sweep(Bc, it, c->lists.p + (colour * 2 + 0) * list_stride, c->list_totals.p + colour * 2 + 0);
      if (overlap && it == 0 && colour == 0) {
        // the colour-0 pixels whose GenNeighbours failed (UNKNOWN after NeigbourUpdate), same snapshot
        HIPC(hipStreamWaitEvent(s, c->ev_join, 0));
        strong_sweep(Bc, it, failed_list, c->list_totals.p + 5);
        sweep_lists(Bc);   // the sweep lists after NeigbourUpdate (weak_info is fixed until DepthToWeak)
      }
      end();
    }
    HIPC(hipGetLastError());
    // The two colours' weak sweeps read only STRONG pixels' state besides their own pixel (planes and
    // selected views of the GenNeighbours support points, DPE.cu:1690-1725; the NCC-New patches come
    // from the images), and write only their own pixel, so they are independent: the colour-1 sweep
    // runs on the aux stream beside the colour-0 one (the launch tails overlap).  Each colour's
    // RANSACToGetFitPlane over that colour's weak list runs on that colour's stream just before its
    // sweep (a fit reads STRONG pixels and writes its own pixel's fit plane, which only its own weak
    // update reads).
    const unsigned rl_grid = (unsigned)((L / 2 + 1 + kRansacThreads - 1) / kRansacThreads);
    if (overlap) {   // fork first: the colour-1 fit must not wait for the colour-0 one
      HIPC(hipEventRecord(c->ev_fork, s));
      HIPC(hipStreamWaitEvent(c->aux, c->ev_fork, 0));
    }
    Bc = begin(DPE_CLASS_RANSAC);
    for (int colour = 1; colour >= 0; --colour) {
      const hipStream_t sr = colour == 1 ? a : s;
      k_ransac_fit<<<rl_grid, kRansacThreads, 0, sr>>>(dpc, Bc, it, c->lists.p + (colour * 2 + 1) * list_stride,
                                                        c->list_totals.p + colour * 2 + 1);
    }
    end();
    for (int colour = 0; colour < 2; ++colour) {
      Bc = begin(DPE_CLASS_WEAK);
      {
        const hipStream_t sw = colour == 1 ? a : s;
        const int* lst = c->lists.p + (colour * 2 + 1) * list_stride;
        const int* cnt = c->list_totals.p + colour * 2 + 1;
        if (pc.P.use_radius) {   // the fits just set the radii: partition the list by centre-patch side
          const unsigned pg = (unsigned)((L / 2 + 1 + kPartChunk - 1) / kPartChunk);
          int* pcnt = c->part_cnt.p + colour * (pg + 2);
          int* out = side_lists + colour * list_stride;
          k_part_count<<<pg, 256, 0, sw>>>(dpc, Bc, lst, cnt, pcnt);
          k_part_scan<<<1, 256, 0, sw>>>(cnt, pcnt, c->list_totals.p + 8 + colour);
          k_part_fill<<<pg, 256, 0, sw>>>(dpc, Bc, lst, cnt, pcnt, c->list_totals.p + 8 + colour, out);
          lst = out;
        }
        constexpr int C = kWeakLanes, P = 64 / C;
        const size_t per_wave = (size_t)P * weak_lds_per_pixel(nv) * sizeof(float);
        const int wpb = per_wave * 4 <= 64 * 1024 ? 4 : (per_wave * 2 <= 64 * 1024 ? 2 : 1);
        const unsigned grid = (unsigned)((L / 2 + 1 + wpb * P - 1) / (wpb * P));
        // U8 texels for 8-bit images; F16 (exact for quarter-integer grey levels) for the coarse levels
        if (c->img_cls == IMG_U8) k_weak_coop<kTexWeak, C><<<grid, 64 * wpb, per_wave * wpb, sw>>>(dpc, Bc, it, lst, cnt);
        else if (c->img_cls == IMG_Q) k_weak_coop<TEX_F16, C><<<grid, 64 * wpb, per_wave * wpb, sw>>>(dpc, Bc, it, lst, cnt);
        else k_weak_coop<TEX_F32, C><<<grid, 64 * wpb, per_wave * wpb, sw>>>(dpc, Bc, it, lst, cnt);
      }
      end();
    }
    if (overlap) {
      HIPC(hipEventRecord(c->ev_join, c->aux));
      HIPC(hipStreamWaitEvent(s, c->ev_join, 0));
    }
    HIPC(hipGetLastError());
  }
  Bc = begin(DPE_CLASS_FILTER);
  k_depth_normal<<<fg, fb, 0, s>>>(dpc, Bc);
  for (int colour = 0; colour < 2; ++colour) k_filter<<<hg, hb, 0, s>>>(dpc, Bc, colour);   // hb: 32 x 4 = kFilterThreads
  end();
  // LocalRefine on the 6-px border (which DepthToWeak leaves to it) reads and writes only its own
  // pixel's plane besides the images and source depths (DPE.cu:2749-2835), and DepthToWeak writes
  // only interior pixels: the two are independent, so the border kernel runs on the aux stream
  // beside DepthToWeak (launched first: it is small and would otherwise wait for DepthToWeak's slots)
  if (overlap) {
    HIPC(hipEventRecord(c->ev_fork, s));
    HIPC(hipStreamWaitEvent(a, c->ev_fork, 0));
    Bc = begin(DPE_CLASS_LOCAL_REFINE);
    launch_local_refine(c->img_cls, (long)L, W, H, nv, a, dpc, Bc);
    end();
    HIPC(hipEventRecord(c->ev_join, a));
  }
  Bc = begin(DPE_CLASS_DEPTH_TO_WEAK);
  launch_depth_to_weak(c->img_cls, (long)L, s, dpc, Bc);
  end();
  if (overlap) {
    HIPC(hipStreamWaitEvent(s, c->ev_join, 0));
  } else {
    Bc = begin(DPE_CLASS_LOCAL_REFINE);
    launch_local_refine(c->img_cls, (long)L, W, H, nv, s, dpc, Bc);
    end();
  }
  HIPC(hipGetLastError());
  if (slot_overflow) {   // per-class times would silently miss launches
    HIPC(hipStreamSynchronize(s));
    g_err = "dpe_pm_execute: more timed launch sections than timing slots (" + std::to_string(max_slots) + ")";
    return DPE_ERR_STATE;
  }
  if (timing && nev > 0) {
    HIPC(hipEventSynchronize(c->ev[2 * nev - 1]));
    for (int k = 0; k <= DPE_NUM_CLASSES; ++k) c->timings[k] = 0.0f;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, c->ev_start, c->ev[2 * nev - 1]);
    c->timings[0] = ms;
    for (int e = 0; e < nev; ++e) {
      (void)hipEventElapsedTime(&ms, c->ev[2 * e], c->ev[2 * e + 1]);
      c->timings[1 + ev_class[e]] += ms;
    }
  }
#if DPE_PHASE_PROF
  {
    unsigned long long ph32[32 * 64], ph[64] = {};
    HIPC(hipMemcpyAsync(ph32, c->phase.p, sizeof(ph32), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    for (int k = 0; k < 32 * 64; ++k) ph[k % 64] += ph32[k];
    unsigned long long tot[4] = {0, 0, 0, 0};
    for (int k = 0; k < 64; ++k) tot[k / 16] += ph[k];
    for (int k = 0; k < 64; ++k)
      if (ph[k]) fprintf(stderr, "PHASE %d.%d %.4e cycles %.1f%%\n", k / 16, k % 16, (double)ph[k], 100.0 * ph[k] / tot[k / 16]);
  }
#endif
  if (c->counting) {
    HIPC(hipMemcpyAsync(c->counts, c->cnt.p, sizeof(c->counts), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    for (int k = 0; k < DPE_NUM_CLASSES; ++k) c->counts[4 * k + 3] = (unsigned long long)c->launches[k];
  }
  HIPC(hipEventRecord(c->ev_done, s));
  c->pending = true;
  return DPE_OK;
}

extern "C" int dpe_pm_fetch(DpeContext* c, const DpePassState* st) {
  g_err.clear();
  if (!c || !st) { g_err = "dpe_pm_fetch: null argument"; return DPE_ERR_ARG; }
  if (!c->staged) { g_err = "dpe_pm_fetch: nothing staged"; return DPE_ERR_STATE; }
  HIPC(hipSetDevice(c->device));
  Range range_("dpe_pm_fetch");
  const size_t L = (size_t)c->hc.W * c->hc.H;
  HIPC(wait_pending(c));
  HIPC(hipStreamSynchronize(c->stream));
  if (st->planes) HIPC(hipMemcpy(st->planes, c->bufs.planes, L * sizeof(float4), hipMemcpyDeviceToHost));
  if (st->weak_info) HIPC(hipMemcpy(st->weak_info, c->bufs.weak, L, hipMemcpyDeviceToHost));
  if (st->selected_views) HIPC(hipMemcpy(st->selected_views, c->bufs.sel, L * sizeof(uint32_t), hipMemcpyDeviceToHost));
  if (st->costs) HIPC(hipMemcpy(st->costs, c->bufs.costs, L * sizeof(float), hipMemcpyDeviceToHost));
  return DPE_OK;
}

extern "C" int dpe_pm_run(DpeContext* c, const DpePassInput* in, const DpePassState* st) {
  int r = dpe_pm_stage(c, in, st);
  if (r) return r;
  r = dpe_pm_execute(c, nullptr);
  if (r) return r;
  return dpe_pm_fetch(c, st);
}

extern "C" void* dpe_pm_device_planes(DpeContext* c) { return (c && c->staged) ? (void*)c->bufs.planes : nullptr; }

__global__ void k_export_depth(const float4* __restrict__ p, float* __restrict__ d, size_t L) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < L) d[i] = p[i].w;
}

extern "C" int dpe_pm_export_depth(DpeContext* c, float* dev_dst, void* stream_) {
  g_err.clear();
  if (!c || !dev_dst) { g_err = "dpe_pm_export_depth: null argument"; return DPE_ERR_ARG; }
  if (!c->staged) { g_err = "dpe_pm_export_depth: nothing staged"; return DPE_ERR_STATE; }
  HIPC(hipSetDevice(c->device));
  hipStream_t s = stream_ ? (hipStream_t)stream_ : c->stream;
  if (c->pending) HIPC(hipStreamWaitEvent(s, c->ev_done, 0));   // after the pass that writes the planes
  const size_t L = (size_t)c->hc.W * c->hc.H;
  k_export_depth<<<(unsigned)((L + 255) / 256), 256, 0, s>>>(c->bufs.planes, dev_dst, L);
  HIPC(hipGetLastError());
  return DPE_OK;
}

// ------------------------------------------------------------------------------ resident state
// ProcessProblem's epilogue (main.cpp:423-437) on the pass outputs, into the image's resident state
__global__ void k_state_save(const float4* __restrict__ planes, const uint8_t* __restrict__ weak,
                             const uint32_t* __restrict__ sel, float dmin, float dmax, float4* __restrict__ op,
                             uint8_t* __restrict__ ow, uint32_t* __restrict__ os, size_t L) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= L) return;
  float4 p = planes[i];
  uint8_t w = weak[i];
  if (p.w < dmin || p.w > dmax) { p.w = 0.0f; w = DPE_UNKNOWN; }
  op[i] = p; ow[i] = w; os[i] = sel[i];
}
__global__ void k_depth_of(const float4* __restrict__ p, float* __restrict__ d, size_t L) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < L) d[i] = p[i].w;
}
__global__ void k_depth_into(const float* __restrict__ d, float4* __restrict__ p, size_t L) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < L) p[i].w = d[i];
}

static ResState* state_slot(DpeContext* c, int id) {
  auto it = c->rstore.find(id);
  if (it != c->rstore.end()) return it->second;
  ResState* r = new ResState();
  c->rstore[id] = r;
  return r;
}

extern "C" int dpe_state_save(DpeContext* c, int image_id) {
  g_err.clear();
  if (!c) { g_err = "dpe_state_save: null context"; return DPE_ERR_ARG; }
  if (!c->staged) { g_err = "dpe_state_save: nothing staged"; return DPE_ERR_STATE; }
  HIPC(hipSetDevice(c->device));
  Range range_("dpe_state_save");
  const int W = c->hc.W, H = c->hc.H;
  const size_t L = (size_t)W * H;
  if (c->pending) HIPC(hipStreamWaitEvent(c->stream, c->ev_done, 0));   // after the pass that wrote the outputs
  ResState* r = state_slot(c, image_id);
  HIPC(r->planes.ensure(L)); HIPC(r->weak.ensure(L)); HIPC(r->sel.ensure(L));
  r->w = W; r->h = H; r->full = true;
  k_state_save<<<(unsigned)((L + 255) / 256), 256, 0, c->stream>>>(c->bufs.planes, c->bufs.weak, c->bufs.sel, c->hc.P.depth_min,
                                                                  c->hc.P.depth_max, r->planes.p, r->weak.p, r->sel.p, L);
  HIPC(hipGetLastError());
  HIPC(hipEventRecord(c->ev_done, c->stream));   // the next execute / stage waits for the save too
  c->pending = true;
  return DPE_OK;
}

extern "C" int dpe_state_fetch(DpeContext* c, int image_id, int* w, int* h, float* depth, float* normal, uint8_t* weak,
                               uint32_t* sel) {
  g_err.clear();
  if (!c) { g_err = "dpe_state_fetch: null context"; return DPE_ERR_ARG; }
  auto it = c->rstore.find(image_id);
  if (it == c->rstore.end()) { g_err = "dpe_state_fetch: no state of image " + std::to_string(image_id); return DPE_ERR_STATE; }
  ResState* r = it->second;
  if (w) *w = r->w;
  if (h) *h = r->h;
  const size_t L = (size_t)r->w * r->h;
  HIPC(hipSetDevice(c->device));
  HIPC(wait_pending(c));
  HIPC(hipStreamSynchronize(c->stream));
  if (depth || normal) {
    std::vector<float4> p(L);
    HIPC(hipMemcpy(p.data(), r->planes.p, L * sizeof(float4), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < L; ++i) {
      if (depth) depth[i] = p[i].w;
      if (normal) { normal[3 * i] = p[i].x; normal[3 * i + 1] = p[i].y; normal[3 * i + 2] = p[i].z; }
    }
  }
  if (weak || sel) {
    if (!r->full) { g_err = "dpe_state_fetch: image " + std::to_string(image_id) + " holds a depth map only"; return DPE_ERR_STATE; }
    if (weak) HIPC(hipMemcpy(weak, r->weak.p, L, hipMemcpyDeviceToHost));
    if (sel) HIPC(hipMemcpy(sel, r->sel.p, L * sizeof(uint32_t), hipMemcpyDeviceToHost));
  }
  return DPE_OK;
}

extern "C" int dpe_state_snapshot(DpeContext* c) {
  g_err.clear();
  if (!c) { g_err = "dpe_state_snapshot: null context"; return DPE_ERR_ARG; }
  HIPC(hipSetDevice(c->device));
  if (c->pending) HIPC(hipStreamWaitEvent(c->stream, c->ev_done, 0));
  for (auto& kv : c->rstore) {
    ResState* r = kv.second;
    const size_t L = (size_t)r->w * r->h;
    HIPC(r->snap.ensure(L));
    k_depth_of<<<(unsigned)((L + 255) / 256), 256, 0, c->stream>>>(r->planes.p, r->snap.p, L);
    r->snap_w = r->w; r->snap_h = r->h;
    r->has_snap = true;
  }
  HIPC(hipGetLastError());
  HIPC(hipEventRecord(c->ev_done, c->stream));
  c->pending = true;
  c->snap_mode = true;
  return DPE_OK;
}

extern "C" int dpe_state_export_depth(DpeContext* c, int image_id, float* dev_dst, void* stream_) {
  g_err.clear();
  if (!c || !dev_dst) { g_err = "dpe_state_export_depth: null argument"; return DPE_ERR_ARG; }
  auto it = c->rstore.find(image_id);
  if (it == c->rstore.end()) { g_err = "dpe_state_export_depth: no state of image " + std::to_string(image_id); return DPE_ERR_STATE; }
  HIPC(hipSetDevice(c->device));
  hipStream_t s = stream_ ? (hipStream_t)stream_ : c->stream;
  if (c->pending) HIPC(hipStreamWaitEvent(s, c->ev_done, 0));
  const size_t L = (size_t)it->second->w * it->second->h;
  k_depth_of<<<(unsigned)((L + 255) / 256), 256, 0, s>>>(it->second->planes.p, dev_dst, L);
  HIPC(hipGetLastError());
  return DPE_OK;
}

extern "C" int dpe_state_import_depth(DpeContext* c, int image_id, int w, int h, const float* dev_src, void* stream_) {
  g_err.clear();
  if (!c || !dev_src || w <= 0 || h <= 0) { g_err = "dpe_state_import_depth: bad argument"; return DPE_ERR_ARG; }
  HIPC(hipSetDevice(c->device));
  hipStream_t s = stream_ ? (hipStream_t)stream_ : c->stream;
  if (c->pending) HIPC(hipStreamWaitEvent(s, c->ev_done, 0));   // an execute may still read this state's depth
  ResState* r = state_slot(c, image_id);
  const size_t L = (size_t)w * h;
  if (r->w != w || r->h != h) {
    HIPC(r->planes.ensure(L));
    HIPC(hipMemsetAsync(r->planes.p, 0, L * sizeof(float4), s));
    r->w = w; r->h = h; r->full = false;
  }
  k_depth_into<<<(unsigned)((L + 255) / 256), 256, 0, s>>>(dev_src, r->planes.p, L);
  HIPC(hipGetLastError());
  if (s != c->stream) {   // later stages on the context stream read it
    HIPC(hipEventRecord(c->ev_done, s));
    c->pending = true;
  }
  return DPE_OK;
}

extern "C" float* dpe_device_buffer(DpeContext* c, int slot, size_t count) {
  g_err.clear();
  if (!c || slot < 0 || slot > 1) { g_err = "dpe_device_buffer: bad argument"; return nullptr; }
  if (hipSetDevice(c->device) != hipSuccess) { g_err = "dpe_device_buffer: hipSetDevice"; return nullptr; }
  if (c->xbuf[slot].n < count) {
    if (wait_pending(c) != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) { g_err = "dpe_device_buffer: sync"; return nullptr; }
    if (c->xbuf[slot].ensure(count) != hipSuccess) { g_err = "dpe_device_buffer: hipMalloc"; return nullptr; }
  }
  return c->xbuf[slot].p;
}

extern "C" int dpe_sync(DpeContext* c) {
  g_err.clear();
  if (!c) { g_err = "dpe_sync: null context"; return DPE_ERR_ARG; }
  HIPC(hipSetDevice(c->device));
  HIPC(wait_pending(c));
  HIPC(hipStreamSynchronize(c->stream));
  return DPE_OK;
}

extern "C" int dpe_device_copy(DpeContext* c, void* dst, const void* src, size_t bytes, int kind) {
  g_err.clear();
  if (!c || !dst || !src || kind < 0 || kind > 2) { g_err = "dpe_device_copy: bad argument"; return DPE_ERR_ARG; }
  HIPC(hipSetDevice(c->device));
  HIPC(wait_pending(c));
  HIPC(hipStreamSynchronize(c->stream));
  const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : (kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice);
  HIPC(hipMemcpy(dst, src, bytes, k));
  return DPE_OK;
}

// ------------------------------------------------------------------------------ EdgeSegment stages
namespace {
// cv::resize INTER_LINEAR CV_32F taps (host/hostio.cpp linear_taps)
void f32_taps(int n_src, int n_dst, int* s0, int* s1, float* a0, float* a1) {
  const double scale = 1.0 / ((double)n_dst / n_src);
  for (int d = 0; d < n_dst; ++d) {
    float f = (float)((d + 0.5) * scale - 0.5);
    int sidx = (int)std::floor(f);
    f -= (float)sidx;
    if (sidx < 0) { f = 0; sidx = 0; }
    if (sidx >= n_src - 1) { f = 0; sidx = n_src - 1; }
    s0[d] = sidx; s1[d] = std::min(sidx + 1, n_src - 1);
    a0[d] = 1.0f - f; a1[d] = f;
  }
}
// cv::resize INTER_LINEAR CV_8U taps (host/edges.cpp lin_tab): 11-bit weights, cvRound half to even
int u8_taps(int ssize, int dsize, int* ofs, short* a) {
  const double scale = 1.0 / ((double)dsize / ssize);
  int xmax = dsize;
  for (int d = 0; d < dsize; ++d) {
    float f = (float)((d + 0.5) * scale - 0.5);
    int sidx = (int)std::floor(f);
    f -= (float)sidx;
    if (sidx < 0) { f = 0; sidx = 0; }
    if (sidx + 1 >= ssize) {
      xmax = std::min(xmax, d);
      if (sidx >= ssize - 1) { f = 0; sidx = ssize - 1; }
    }
    ofs[d] = sidx;
    const float c0 = 1.0f - f, c1 = f;
    a[2 * d] = (short)std::min(32767, std::max(-32768, (int)std::nearbyint(c0 * 2048.0f)));
    a[2 * d + 1] = (short)std::min(32767, std::max(-32768, (int)std::nearbyint(c1 * 2048.0f)));
  }
  return xmax;
}
}  // namespace

extern "C" int dpe_resize_linear(DpeContext* c, const float* src, int w, int h, float* dst, int nw, int nh) {
  g_err.clear();
  if (!c || !src || !dst || w < 1 || h < 1 || nw < 1 || nh < 1) { g_err = "dpe_resize_linear: bad argument"; return DPE_ERR_ARG; }
  if (w == nw && h == nh) { std::memcpy(dst, src, sizeof(float) * (size_t)w * h); return DPE_OK; }
  HIPC(hipSetDevice(c->device));
  std::vector<int> it(2 * (size_t)(nw + nh));
  std::vector<float> ft(2 * (size_t)(nw + nh));
  f32_taps(w, nw, it.data(), it.data() + nw, ft.data(), ft.data() + nw);
  f32_taps(h, nh, it.data() + 2 * nw, it.data() + 2 * nw + nh, ft.data() + 2 * nw, ft.data() + 2 * nw + nh);
  HIPC(c->e_fa.ensure((size_t)w * h)); HIPC(c->e_fb.ensure((size_t)nw * nh));
  HIPC(c->e_rows.ensure((size_t)h * nw));   // f32 rows stored in the int scratch (same size)
  HIPC(c->e_itab.ensure(it.size())); HIPC(c->e_ftab.ensure(ft.size()));
  HIPC(hipMemcpyAsync(c->e_fa.p, src, sizeof(float) * (size_t)w * h, hipMemcpyHostToDevice, c->stream));
  HIPC(hipMemcpyAsync(c->e_itab.p, it.data(), it.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
  HIPC(hipMemcpyAsync(c->e_ftab.p, ft.data(), ft.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
  float* rows = (float*)c->e_rows.p;
  const dim3 b(32, 8);
  k_resize_linear_h<<<dim3((nw + 31) / 32, (h + 7) / 8), b, 0, c->stream>>>(c->e_fa.p, w, h, c->e_itab.p, c->e_itab.p + nw,
                                                                            c->e_ftab.p, c->e_ftab.p + nw, rows, nw);
  k_resize_linear_v<<<dim3((nw + 31) / 32, (nh + 7) / 8), b, 0, c->stream>>>(rows, nw, c->e_itab.p + 2 * nw,
                                                                             c->e_itab.p + 2 * nw + nh, c->e_ftab.p + 2 * nw,
                                                                             c->e_ftab.p + 2 * nw + nh, c->e_fb.p, nh);
  HIPC(hipGetLastError());
  HIPC(hipMemcpyAsync(dst, c->e_fb.p, sizeof(float) * (size_t)nw * nh, hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  return DPE_OK;
}

// device-to-device core of dpe_resize_u8 (src / dst in the context's scratch)
static int resize_u8_dev(DpeContext* c, const uint8_t* dsrc, int w, int h, uint8_t* ddst, int nw, int nh) {
  const dim3 b(32, 8);
  if (w == nw && h == nh) { HIPC(hipMemcpyAsync(ddst, dsrc, (size_t)w * h, hipMemcpyDeviceToDevice, c->stream)); return DPE_OK; }
  const double scale_x = 1.0 / ((double)nw / w), scale_y = 1.0 / ((double)nh / h);
  const int isx = (int)std::lround(scale_x), isy = (int)std::lround(scale_y);
  const bool area_fast = std::fabs(scale_x - isx) < 2.220446049250313e-16 && std::fabs(scale_y - isy) < 2.220446049250313e-16;
  if (area_fast && isx == 2 && isy == 2) {   // INTER_LINEAR at exactly 1/2 = INTER_AREA's fast path
    k_resize_u8_half<<<dim3((nw + 31) / 32, (nh + 7) / 8), b, 0, c->stream>>>(dsrc, w, ddst, nw, nh);
    HIPC(hipGetLastError());
    return DPE_OK;
  }
  std::vector<int> ofs((size_t)nw + nh);
  std::vector<short> a(2 * ((size_t)nw + nh));
  const int xmax = u8_taps(w, nw, ofs.data(), a.data());
  (void)u8_taps(h, nh, ofs.data() + nw, a.data() + 2 * nw);
  int xv = 0;                                 // VResizeLinear: 16-lane, then 8-lane vector blocks
  for (; xv <= nw - 16; xv += 16) {}
  for (; xv < nw - 8; xv += 8) {}
  HIPC(c->e_rows.ensure((size_t)h * nw)); HIPC(c->e_itab.ensure(ofs.size())); HIPC(c->e_stab.ensure(a.size()));
  HIPC(hipMemcpyAsync(c->e_itab.p, ofs.data(), ofs.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
  HIPC(hipMemcpyAsync(c->e_stab.p, a.data(), a.size() * sizeof(short), hipMemcpyHostToDevice, c->stream));
  k_resize_u8_h<<<dim3((nw + 31) / 32, (h + 7) / 8), b, 0, c->stream>>>(dsrc, w, h, c->e_itab.p, c->e_stab.p, xmax,
                                                                        c->e_rows.p, nw);
  k_resize_u8_v<<<dim3((nw + 31) / 32, (nh + 7) / 8), b, 0, c->stream>>>(c->e_rows.p, h, nw, c->e_itab.p + nw,
                                                                         c->e_stab.p + 2 * nw, xv, ddst, nh);
  HIPC(hipGetLastError());
  return DPE_OK;
}

extern "C" int dpe_resize_u8(DpeContext* c, const uint8_t* src, int w, int h, uint8_t* dst, int nw, int nh) {
  g_err.clear();
  if (!c || !src || !dst || w < 1 || h < 1 || nw < 1 || nh < 1) { g_err = "dpe_resize_u8: bad argument"; return DPE_ERR_ARG; }
  HIPC(hipSetDevice(c->device));
  HIPC(c->e_a.ensure((size_t)w * h)); HIPC(c->e_b.ensure((size_t)nw * nh));
  HIPC(hipMemcpyAsync(c->e_a.p, src, (size_t)w * h, hipMemcpyHostToDevice, c->stream));
  const int r = resize_u8_dev(c, c->e_a.p, w, h, c->e_b.p, nw, nh);
  if (r != DPE_OK) return r;
  HIPC(hipMemcpyAsync(dst, c->e_b.p, (size_t)nw * nh, hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  return DPE_OK;
}

extern "C" int dpe_roberts_threshold(DpeContext* c, const uint8_t* src, int w, int h, int thr, uint8_t* dst) {
  g_err.clear();
  if (!c || !src || !dst || w < 1 || h < 1) { g_err = "dpe_roberts_threshold: bad argument"; return DPE_ERR_ARG; }
  HIPC(hipSetDevice(c->device));
  HIPC(c->e_a.ensure((size_t)w * h)); HIPC(c->e_b.ensure((size_t)w * h));
  HIPC(hipMemcpyAsync(c->e_a.p, src, (size_t)w * h, hipMemcpyHostToDevice, c->stream));
  k_roberts_threshold<<<dim3((w + 31) / 32, (h + 7) / 8), dim3(32, 8), 0, c->stream>>>(c->e_a.p, w, h, thr, c->e_b.p);
  HIPC(hipGetLastError());
  HIPC(hipMemcpyAsync(dst, c->e_b.p, (size_t)w * h, hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  return DPE_OK;
}

extern "C" int dpe_canny(DpeContext* c, const uint8_t* src, int w, int h, double low_thresh, double high_thresh, uint8_t* dst) {
  g_err.clear();
  if (!c || !src || !dst || w < 1 || h < 1) { g_err = "dpe_canny: bad argument"; return DPE_ERR_ARG; }
  HIPC(hipSetDevice(c->device));
  Range range_("dpe_canny");
  if (low_thresh > high_thresh) std::swap(low_thresh, high_thresh);   // canny.cpp threshold handling
  low_thresh = std::min(32767.0, low_thresh);
  high_thresh = std::min(32767.0, high_thresh);
  if (low_thresh > 0) low_thresh *= low_thresh;
  if (high_thresh > 0) high_thresh *= high_thresh;
  const int low = (int)std::floor(low_thresh), high = (int)std::floor(high_thresh);
  const int ms = w + 2;
  const size_t L = (size_t)w * h, M = (size_t)ms * (h + 2);
  HIPC(c->e_a.ensure(L)); HIPC(c->e_dx.ensure(L)); HIPC(c->e_dy.ensure(L)); HIPC(c->e_mag.ensure(M)); HIPC(c->e_map.ensure(M));
  HIPC(hipMemcpyAsync(c->e_a.p, src, L, hipMemcpyHostToDevice, c->stream));
  const dim3 b(32, 8), g((ms + 31) / 32, (h + 2 + 7) / 8);
  k_canny_sobel<<<g, b, 0, c->stream>>>(c->e_a.p, w, h, c->e_dx.p, c->e_dy.p, c->e_mag.p);
  k_canny_nms<<<g, b, 0, c->stream>>>(c->e_dx.p, c->e_dy.p, c->e_mag.p, w, h, low, high, c->e_map.p);
  HIPC(hipGetLastError());
  std::vector<uint8_t> map(M);
  HIPC(hipMemcpyAsync(map.data(), c->e_map.p, M, hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  // hysteresis: 8-connected growth through candidates from every strong candidate (any order: the
  // closure is the same set)
  std::vector<size_t> stack;
  stack.reserve(L / 8 + 16);
  for (size_t i = 0; i < M; ++i) if (map[i] == 2) stack.push_back(i);
  const long off[8] = {-ms - 1, -ms, -ms + 1, -1, 1, ms - 1, ms, ms + 1};
  while (!stack.empty()) {
    const size_t i = stack.back();
    stack.pop_back();
    for (long o : off) {
      const size_t j = (size_t)((long)i + o);
      if (!map[j]) { map[j] = 2; stack.push_back(j); }
    }
  }
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) dst[(size_t)y * w + x] = map[(size_t)(y + 1) * ms + x + 1] == 2 ? 255 : 0;
  return DPE_OK;
}

extern "C" void dpe_state_clear(DpeContext* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)wait_pending(c);
  (void)hipStreamSynchronize(c->stream);
  for (auto& kv : c->rstore) { kv.second->release(); delete kv.second; }
  c->rstore.clear();
  c->snap_mode = false;
}

extern "C" int dpe_host_pin(void* ptr, size_t bytes) {
  if (!ptr || bytes == 0) return DPE_ERR_ARG;
  return hipHostRegister(ptr, bytes, hipHostRegisterDefault) == hipSuccess ? DPE_OK : DPE_ERR_HIP;
}
extern "C" int dpe_host_unpin(void* ptr) {
  if (!ptr) return DPE_ERR_ARG;
  return hipHostUnregister(ptr) == hipSuccess ? DPE_OK : DPE_ERR_HIP;
}

extern "C" int dpe_fusion_stage(DpeContext* c, const DpeFusionView* views, int n) {
  g_err.clear();
  if (!c || !views || n < 1) { g_err = "dpe_fusion_stage: bad argument"; return DPE_ERR_ARG; }
  HIPC(hipSetDevice(c->device));
  c->fz_depth.resize(n); c->fz_normal.resize(n); c->fz_host.assign(n, FusionViewDev{});
  std::vector<DpeCamera> cams(n);
  for (int i = 0; i < n; ++i) {
    const DpeFusionView& v = views[i];
    if (v.width < 1 || v.height < 1 || !v.depth || !v.normal) { g_err = "dpe_fusion_stage: bad view"; return DPE_ERR_ARG; }
    const size_t L = (size_t)v.width * v.height;
    HIPC(c->fz_depth[i].ensure(L));
    HIPC(c->fz_normal[i].ensure(3 * L));
    HIPC(hipMemcpyAsync(c->fz_depth[i].p, v.depth, L * 4, hipMemcpyHostToDevice, c->stream));
    HIPC(hipMemcpyAsync(c->fz_normal[i].p, v.normal, 3 * L * 4, hipMemcpyHostToDevice, c->stream));
    c->fz_host[i] = FusionViewDev{c->fz_depth[i].p, c->fz_normal[i].p, v.width, v.height};
    cams[i] = v.cam;
  }
  HIPC(c->fz_views.ensure(n));
  HIPC(c->fz_cams.ensure(n));
  HIPC(hipMemcpyAsync(c->fz_views.p, c->fz_host.data(), n * sizeof(FusionViewDev), hipMemcpyHostToDevice, c->stream));
  HIPC(hipMemcpyAsync(c->fz_cams.p, cams.data(), n * sizeof(DpeCamera), hipMemcpyHostToDevice, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  c->fz_n = n;
  return DPE_OK;
}

extern "C" int dpe_fusion_candidates(DpeContext* c, int ref, const int* src, int ns, int32_t* idx, float* val) {
  g_err.clear();
  if (!c || !src || !idx || !val || ns < 0) { g_err = "dpe_fusion_candidates: bad argument"; return DPE_ERR_ARG; }
  if (c->fz_n < 1) { g_err = "dpe_fusion_candidates: nothing staged"; return DPE_ERR_STATE; }
  if (ref < 0 || ref >= c->fz_n) { g_err = "dpe_fusion_candidates: bad reference view"; return DPE_ERR_ARG; }
  for (int j = 0; j < ns; ++j)
    if (src[j] < 0 || src[j] >= c->fz_n) { g_err = "dpe_fusion_candidates: bad source view"; return DPE_ERR_ARG; }
  if (ns == 0) return DPE_OK;
  HIPC(hipSetDevice(c->device));
  const size_t L = (size_t)c->fz_host[ref].w * c->fz_host[ref].h;
  HIPC(c->fz_src.ensure(ns));
  HIPC(c->fz_idx.ensure(L * ns));
  HIPC(c->fz_val.ensure(L * ns * 3));
  HIPC(hipMemcpyAsync(c->fz_src.p, src, ns * sizeof(int), hipMemcpyHostToDevice, c->stream));
  k_fusion_candidates<<<(unsigned)((L + 255) / 256), 256, 0, c->stream>>>(c->fz_cams.p, c->fz_views.p, ref, c->fz_src.p, ns,
                                                                         c->fz_idx.p, c->fz_val.p);
  HIPC(hipGetLastError());
  HIPC(hipMemcpyAsync(idx, c->fz_idx.p, L * ns * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIPC(hipMemcpyAsync(val, c->fz_val.p, L * ns * 3 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  return DPE_OK;
}

extern "C" int dpe_pm_last_timings(DpeContext* c, float* out, int n) {
  if (!c || !out) return 0;
  const int m = n < DPE_NUM_CLASSES + 1 ? n : DPE_NUM_CLASSES + 1;
  for (int i = 0; i < m; ++i) out[i] = c->timings[i];
  return m;
}

extern "C" void dpe_set_counting(DpeContext* c, int enable) { if (c) c->counting = enable != 0; }

extern "C" int dpe_set_option(DpeContext* c, int option, int value) {
  g_err.clear();
  if (!c) { g_err = "dpe_set_option: null context"; return DPE_ERR_ARG; }
  if (option == DPE_OPT_GN_SLOTS && (value == 0 || value == 8 || value == 32 || value == 64)) { c->gn_slots = value; return DPE_OK; }
  g_err = "dpe_set_option: unknown option or value";
  return DPE_ERR_ARG;
}

extern "C" long long dpe_pm_last_stat(DpeContext* c, int stat) {
  if (c && c->staged && stat == DPE_STAT_TEX_CLASS) return c->img_cls;
  if (!c || !c->staged || stat != DPE_STAT_GN_DEFERRED || !c->list_totals.p) return -1;
  int v = 0;   // waits for this context's pass only (not the whole device)
  if (hipSetDevice(c->device) != hipSuccess || wait_pending(c) != hipSuccess || hipStreamSynchronize(c->aux) != hipSuccess ||
      hipMemcpyAsync(&v, c->list_totals.p + 6, sizeof(int), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return -1;
  return v;
}

extern "C" int dpe_pm_last_counts(DpeContext* c, unsigned long long* out, int n) {
  if (!c || !out) return 0;
  const int m = n < DPE_NUM_CLASSES * 4 ? n : DPE_NUM_CLASSES * 4;
  for (int i = 0; i < m; ++i) out[i] = c->counts[i];
  return m;
}
