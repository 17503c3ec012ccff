/*
 * dpe_mvs.h — C-ABI of the MI355X-native PatchMatch pass (the DPE-MVS hot path).
 *
 * This header is the drop-in boundary.  It replaces the inner seam of the reference's
 * per-image host object `class DPE`:
 *
 *   reference                                   replaced by
 *   ------------------------------------------  ------------------------------------------
 *   DPE::CudaSpaceInitialization  DPE.cpp:916   dpe_pm_stage()   (H2D, layout, workspaces)
 *   DPE::SetDataPassHelperInCuda  DPE.cpp:1054  (internal: device pointer bundle)
 *   DPE::RunPatchMatch            DPE.cu:3126   dpe_pm_execute() (the 26-launch pass)
 *   DPE::GetPlaneHypothesis       DPE.cpp:1091  dpe_pm_fetch()   (D2H of planes /
 *   DPE::GetPixelStates           DPE.cpp:1099                     weak_info / selected_views)
 *   DPE::GetSelectedViews         DPE.cpp:1103
 *   DPE::~DPE                     DPE.cpp:679   dpe_destroy()
 *   CudaSafeCall -> exit()        DPE.cpp:633   return codes + dpe_last_error()
 *
 * The caller (host orchestration, the reference's ProcessProblem main.cpp:411-446) keeps
 * doing InuputInitialization (DPE.cpp:733-914: image decode/resize, camera read, depth range
 * x0.6/x1.2, prior rescale) and the epilogue (main.cpp:427-446).
 *
 * Types are plain C: no torch, no HIP types.  `DpeCamera` and `DpePatchMatchParams` are
 * layout-compatible with the reference's `Camera` (main.h:50-59) and `PatchMatchParams`
 * (main.h:78-106); enum values match `RunState` / `PixelState` (main.h:66-76).
 */
#ifndef DPE_MVS_H_
#define DPE_MVS_H_

#include <stdint.h>
#include <stddef.h>
#ifndef __cplusplus
#include <stdbool.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define DPE_ABI_VERSION 1
#define DPE_MAX_IMAGES 32      /* main.h:40  MAX_IMAGES     */
#define DPE_NEIGHBOUR_NUM 9    /* main.h:41  NEIGHBOUR_NUM  */

/* main.h:66-70 RunState */
enum { DPE_FIRST_INIT = 0, DPE_REFINE_INIT = 1, DPE_REFINE_ITER = 2 };
/* main.h:72-76 PixelState */
enum { DPE_WEAK = 0, DPE_STRONG = 1, DPE_UNKNOWN = 2 };

/* Error codes (the reference exits the process instead, DPE.cpp:633-641, :762-765). */
enum {
  DPE_OK = 0,
  DPE_ERR_ARG = -1,       /* bad argument / shape */
  DPE_ERR_HIP = -2,       /* HIP runtime error */
  DPE_ERR_NOMEM = -3,     /* allocation failed */
  DPE_ERR_STATE = -4,     /* call order (execute before stage, ...) */
  DPE_ERR_TOO_MANY = -5   /* num_images > DPE_MAX_IMAGES (DPE.cpp:762) */
};

/* main.h:50-59 struct Camera (112 bytes) */
typedef struct DpeCamera {
  float K[9];
  float R[9];
  float t[3];
  float c[3];
  int height;
  int width;
  float depth_min;
  float depth_max;
} DpeCamera;

/* main.h:78-106 struct PatchMatchParams, same field order and C types. */
typedef struct DpePatchMatchParams {
  int max_iterations;     /* 3 */
  int num_images;         /* 1 ref + Ns src */
  float sigma_spatial;    /* 5 */
  float sigma_color;      /* 3 */
  int top_k;              /* 4 */
  float depth_min;
  float depth_max;
  bool geom_consistency;
  int strong_radius;      /* 5 */
  int strong_increment;   /* 2 */
  int weak_radius;        /* 5 */
  int weak_increment;     /* 5 */
  bool use_APD;
  bool use_edge;
  bool use_limit;
  bool use_label;
  bool use_radius;
  bool high_res_img;
  int max_scale_size;
  int scale_size;
  int weak_peak_radius;   /* 2 */
  int rotate_time;        /* 4 */
  float ransac_threshold; /* 0.005 */
  float geom_factor;      /* 0.2 */
  int state;              /* RunState */
} DpePatchMatchParams;

/* Fills `p` with the defaults of main.h:78-106. */
void dpe_params_default(DpePatchMatchParams* p);

/*
 * Inputs of one PatchMatch pass for one reference image, all HOST pointers, row-major.
 * Index 0 is the reference image, 1..num_images-1 the source images (DPE.cpp:743-761).
 */
typedef struct DpePassInput {
  int width, height;               /* pass resolution (after the caller's rescale) */
  int num_images;                  /* <= DPE_MAX_IMAGES */
  const float* const* images;      /* [num_images] -> f32 [H][W] grey levels (DPE.cpp:745-757) */
  const DpeCamera* cams;           /* [num_images], K already scale-adjusted (DPE.cpp:814-819) */
  const float* const* depths;      /* [num_images] -> f32 [H][W], NULL unless geom (DPE.cpp:826-843);
                                      entry 0 may be NULL (the ref depth is never sampled) */
  const uint8_t* edge;             /* [H][W] {0,255} edges_<scale>.dmb, or NULL (DPE.cpp:1032) */
  int low_width, low_height;       /* size of edge_low_res */
  const uint8_t* edge_low_res;     /* [lh][lw] edges_<max_scale>.dmb (DPE.cpp:1042), or NULL */
  const int32_t* label;            /* [H][W] labels_<scale>.dmb, or NULL (DPE.cpp:1049) */
  DpePatchMatchParams params;      /* params.num_images / depth_min / depth_max set by caller */
  uint64_t seed;                   /* Philox key (the reference seeds cuRAND from clock64()) */
  uint32_t pass_salt;              /* distinguishes passes that reuse a seed */
  const int32_t* image_ids;        /* [num_images] or NULL.  With ids, each image's device copy and its
                                      gather layouts stay resident in HBM keyed by (id, width, height)
                                      and later passes skip the upload (the caller promises that an
                                      id at a size always has the same pixels); NULL: upload every pass */
} DpePassInput;

/*
 * Per-pixel state, in/out, HOST pointers.
 *  planes:         float4 [H][W]; in: (world normal xyz, depth w) prior unless FIRST_INIT
 *                  (DPE.cpp:896-903); out: (world normal xyz, depth w) (DPE.cu:1940-1955).
 *  weak_info:      u8 [H][W] PixelState; in: weak.bin (ignored, all STRONG, when !use_APD,
 *                  DPE.cpp:873-881); out: DepthToWeak classification (DPE.cu:2593-2747).
 *  selected_views: u32 [H][W] view bit-mask, in/out (DPE.cpp:906-911).
 *  costs:          f32 [H][W] optional output (NULL to skip); not in the reference's readback.
 */
typedef struct DpePassState {
  float* planes;
  uint8_t* weak_info;
  uint32_t* selected_views;
  float* costs;
} DpePassState;

typedef struct DpeContext DpeContext;

/* Context = one HIP device + its workspaces.  One context per thread. */
DpeContext* dpe_create(int device);
void dpe_destroy(DpeContext* ctx);

/* Last error message of the calling thread ("" if none). */
const char* dpe_last_error(void);

/* Uploads inputs and the initial state (H2D), builds the device layouts. Synchronous.  Waits first
 * for the work of the previous dpe_pm_execute (on whatever stream it was enqueued), so stage(A);
 * execute(A, s); stage(B) never overwrites inputs pass A still reads. */
int dpe_pm_stage(DpeContext* ctx, const DpePassInput* in, const DpePassState* state);

/*
 * Runs the whole pass (DPE.cu:3150-3226) on device-resident data on `stream` (a hipStream_t,
 * NULL = the context's stream).  Every call starts from the staged initial state, so repeated
 * calls are idempotent.  Asynchronous w.r.t. the host; ordered after the previous execute (the stream
 * waits on its completion event), and dpe_pm_stage / dpe_pm_fetch / dpe_destroy wait for it.
 * Part of the pass runs on the context's second (aux) stream, forked from and joined back into
 * `stream` with events, so all work is complete when `stream` reaches the end of the call's
 * enqueued work (environment DPE_OVERLAP=0, timing or counting keep everything on `stream`).
 * The aux stream runs the setup chain: GenEdgeInform and its edge-ray line scans,
 * FindNearestStrongPoint's tables and search, the WEAK-pixel list, GenNeighbours (the scratch-free
 * kernel, its coordinate tables and the scratch kernel for its overflow pixels) and NeigbourUpdate.
 * Beside it `stream` runs
 * RandomInitialization (reads planes/sel/images, writes planes/costs/sel) and the iteration-0
 * colour-0 strong half-sweep, which waits for GenEdgeInform's event only (it reads the edge rays;
 * it must not read nearest, nb, weak_rel or radius, which the aux stream is still writing); every
 * later launch waits for the join.  tests/test_gpu_parity.py checks the forked and one-stream
 * schedules bit for bit, including weak, sel and costs.
 */
int dpe_pm_execute(DpeContext* ctx, void* stream);

/* D2H of the outputs (DPE.cu:3245-3247).  Synchronous. */
int dpe_pm_fetch(DpeContext* ctx, const DpePassState* state);

/* stage + execute + fetch. */
int dpe_pm_run(DpeContext* ctx, const DpePassInput* in, const DpePassState* state);

/* Drops every image kept by `image_ids` (frees their HBM). */
void dpe_image_cache_clear(DpeContext* ctx);

/* Device pointer of the working planes buffer (float4 [H][W]) for device-side consumers
 * (e.g. the depth all-gather of the multi-GPU schedule).  NULL before dpe_pm_stage. */
void* dpe_pm_device_planes(DpeContext* ctx);

/* Copies depth (planes.w) into a caller device buffer f32 [H][W] on `stream`. */
int dpe_pm_export_depth(DpeContext* ctx, float* dev_dst, void* stream);

/*
 * HBM-resident pipeline state: the reference writes each image's depths.dmb / normals.dmb / weak.bin /
 * selected_views.bin after a pass (main.cpp:439-446) and its next pass, or a neighbour's geometric
 * term, reads them back (DPE.cpp:826-911).  Here they stay on the device, keyed by image id.
 *
 * dpe_state_save:      after dpe_pm_execute, applies ProcessProblem's epilogue (main.cpp:423-437: depth
 *                      outside [params.depth_min, depth_max] -> 0 and UNKNOWN) on the device and keeps
 *                      (world normal, depth, weak, selected views) as image_id's state.
 * dpe_pm_stage_resident: dpe_pm_stage whose initial state (planes unless FIRST_INIT, weak when use_APD,
 *                      selected views unless FIRST_INIT) comes from prior_id's state, and whose source depths
 *                      (geom_consistency) come from the states of in->image_ids[1..]: each rescaled on the
 *                      device with RescaleMatToTargetSize's nearest rule (DPE.cpp:1146-1165), exactly as the
 *                      host path rescales them.  in->depths is ignored; in->image_ids is required for geom.
 * dpe_state_snapshot:  copies every state's depth into its snapshot and makes later resident stages read
 *                      source depths from the snapshots (the Jacobi schedule: every pass of a round sees the
 *                      previous round's depths).
 * dpe_state_fetch:     host copies of a state (any output pointer may be NULL); w, h receive its size.
 * dpe_state_export_depth / dpe_state_import_depth: the depth map of a state to / from a caller device
 *                      buffer f32 [h][w] on `stream` (the multi-rank all-gather; an imported id without a
 *                      pass of its own holds a depth map only).
 * dpe_state_clear:     frees every state.
 */
int dpe_state_save(DpeContext* ctx, int image_id);
int dpe_pm_stage_resident(DpeContext* ctx, const DpePassInput* in, int prior_id);
int dpe_state_snapshot(DpeContext* ctx);
int dpe_state_fetch(DpeContext* ctx, int image_id, int* w, int* h, float* depth, float* normal, uint8_t* weak,
                    uint32_t* selected_views);
int dpe_state_export_depth(DpeContext* ctx, int image_id, float* dev_dst, void* stream);
int dpe_state_import_depth(DpeContext* ctx, int image_id, int w, int h, const float* dev_src, void* stream);
void dpe_state_clear(DpeContext* ctx);
/* Context-owned device scratch of `count` floats (slot 0 or 1; grows, kept until dpe_destroy) and a
 * synchronous copy (kind 0 host->device, 1 device->host, 2 device->device) after all work of the
 * context: the exchange buffers of the multi-rank schedule without HIP in the caller. */
float* dpe_device_buffer(DpeContext* ctx, int slot, size_t count);
int dpe_device_copy(DpeContext* ctx, void* dst, const void* src, size_t bytes, int kind);
/* Blocks until every operation queued on the context (pass, state exports / imports) has finished,
 * e.g. before a caller's collective reads a buffer an export filled.  DPE_OK or an error code. */
int dpe_sync(DpeContext* ctx);

/*
 * EdgeSegment's data-parallel stages on the device (DPE.cpp:129-291 calls them through OpenCV; the
 * host restatement is host/edges.cpp, and these are bit-identical to it).  HOST buffers, synchronous,
 * on the context's stream (use one context per thread, or serialise the calls).
 *   dpe_resize_linear      cv::resize(INTER_LINEAR) of CV_32FC1             == dpe_host_resize_linear
 *   dpe_resize_u8          cv::resize(INTER_LINEAR) of CV_8UC1 (INTER_AREA fast path at exactly 1/2)
 *                                                                          == dpe_host_resize_u8
 *   dpe_canny              cv::Canny(L2gradient, aperture 3): Sobel, magnitude, non-maximum
 *                          suppression and the strong candidates on the device, the 8-connected
 *                          hysteresis walk on the host                      == dpe_host_canny
 *   dpe_roberts_threshold  Roberts (DPE.cpp:9-25) + cv::threshold(thr, 255, THRESH_BINARY)
 * Connect (DPE.cpp:27-127) and HoughLinesP are scan-order / RNG-order dependent and stay on the host.
 */
int dpe_resize_linear(DpeContext* ctx, const float* src, int w, int h, float* dst, int nw, int nh);
int dpe_resize_u8(DpeContext* ctx, const uint8_t* src, int w, int h, uint8_t* dst, int nw, int nh);
int dpe_canny(DpeContext* ctx, const uint8_t* src, int w, int h, double low, double high, uint8_t* dst);
int dpe_roberts_threshold(DpeContext* ctx, const uint8_t* src, int w, int h, int thr, uint8_t* dst);

/* Kernel classes of one pass, for timing and work accounting. */
enum {
  DPE_CLASS_SETUP = 0,        /* GenEdgeInform, FindNearestStrongPoint, GenNeighbours, NeigbourUpdate */
  DPE_CLASS_INIT = 1,         /* RandomInitialization */
  DPE_CLASS_STRONG = 2,       /* Black/RedPixelUpdateStrong */
  DPE_CLASS_RANSAC = 3,       /* RANSACToGetFitPlane */
  DPE_CLASS_WEAK = 4,         /* Black/RedPixelUpdateWeak */
  DPE_CLASS_FILTER = 5,       /* GetDepthandNormal + Black/RedPixelFilterStrong */
  DPE_CLASS_DEPTH_TO_WEAK = 6,/* DepthToWeak */
  DPE_CLASS_LOCAL_REFINE = 7, /* LocalRefine */
  DPE_NUM_CLASSES = 8
};

/* Enables hipEvent timing of every launch of the following dpe_pm_execute calls. */
void dpe_set_timing(DpeContext* ctx, int enable);
/* ms[0] = whole pass (first to last event), ms[1 + c] = summed kernel time of class c.
 * Returns the number of entries written (<= n, at most 1 + DPE_NUM_CLASSES). */
int dpe_pm_last_timings(DpeContext* ctx, float* ms, int n);

/* Enables algorithmic work counters (device atomics; a counting run is slower and is never the
 * timed run).  out[4*c + k] for class c: k=0 homography set-ups (NCC evaluations), k=1 bilinear
 * taps, k=2 geometric-consistency evaluations, k=3 launches.  Returns entries written. */
void dpe_set_counting(DpeContext* ctx, int enable);
int dpe_pm_last_counts(DpeContext* ctx, unsigned long long* out, int n);

/* Diagnostic knobs and statistics of the pass (not part of the reference's surface; tests).
 * DPE_OPT_GN_SLOTS: support-point slots per WEAK pixel of the scratch-free GenNeighbours
 *   (k_gen_neighbours_lds): 0 = by rotate_time (32 up to 2, else 64, enough for every pixel), 8 = a
 *   test setting that sends every pixel with more points through the overflow path (the scratch
 *   kernel).  Results are the same for every setting.
 * DPE_STAT_GN_DEFERRED: WEAK pixels the scratch-free GenNeighbours of the last execute handed to the
 *   scratch kernel (more points than slots, or a NaN in its sorts).  Synchronises with the pass.
 * DPE_STAT_TEX_CLASS: texel layouts of the staged images: 2 = every grey level an integer in
 *   [0, 255] (u8 / f16 texels), 1 = every grey level a multiple of 1/4 in [0, 255] (the exact 1/2
 *   and 1/4 downscales of the coarse pyramid levels: f16 texels), 0 = f32 texels.
 * dpe_set_option returns DPE_OK or DPE_ERR_ARG; dpe_pm_last_stat returns the value or -1. */
enum { DPE_OPT_GN_SLOTS = 1 };
enum { DPE_STAT_GN_DEFERRED = 1, DPE_STAT_TEX_CLASS = 2 };
int dpe_set_option(DpeContext* ctx, int option, int value);
long long dpe_pm_last_stat(DpeContext* ctx, int stat);

/*
 * RunFusion (DPE.cpp:1220-1370): the per-(pixel, source view) projection tests on the GPU.  The
 * order-dependent rest (the masks of already fused pixels, the angle test, the consistency weights,
 * colours) stays with the caller, in the reference's serial order (the host pipeline's fusion).
 */
typedef struct DpeFusionView {
  int width, height;
  DpeCamera cam;              /* ReadCamera, scaled to the map size (RescaleImageAndCamera, DPE.cpp:1123) */
  const float* depth;         /* f32 [H][W] final depth (depths.dmb; <= 0: no depth) */
  const float* normal;        /* f32 [H][W][3] final world normals (normals.dmb) */
} DpeFusionView;

/* Uploads every view's depth and normal map (H2D); they stay resident for dpe_fusion_candidates. */
int dpe_fusion_stage(DpeContext* ctx, const DpeFusionView* views, int n_views);

/* For reference view `ref` and its source views src[0..ns-1] (indices into the staged views),
 * pixel p (row-major) and source j (DPE.cpp:1303-1343 without the masks):
 *   idx[p*ns + j] = row-major source pixel int(y+.5)*W + int(x+.5) of the projection when it lies
 *                   inside the source view on a depth > 0 with reprojection error < 2 and relative
 *                   depth difference < 0.01; else -1;
 *   val[(p*ns + j)*3 + k] = (reprojection error, relative depth difference, n_ref . n_src).
 * HOST output buffers of W*H*ns int32 / W*H*ns*3 floats.  Synchronous. */
int dpe_fusion_candidates(DpeContext* ctx, int ref, const int* src, int ns, int32_t* idx, float* val);

/* Page-locks (pins) / releases a caller's host buffer so that device -> host copies into it run at
 * full PCIe rate (hipHostRegister; the host fusion pins its candidate buffers).  Nonzero when the
 * runtime refuses (no device, limits): the buffer then stays pageable and every call still works. */
int dpe_host_pin(void* ptr, size_t bytes);
int dpe_host_unpin(void* ptr);

#ifdef __cplusplus
}
#endif
#endif /* DPE_MVS_H_ */
