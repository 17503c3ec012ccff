/*
 * dpe_host.h — C-ABI of the host pipeline (libdpe_host.so): the reference's RunDPEPipeline
 * (main.cpp:474-600) and the helpers it is built from, around the PatchMatch pass of dpe_mvs.h.
 *
 *   reference                                    replaced by
 *   -------------------------------------------  ------------------------------------------
 *   int RunDPEPipeline(path, gpu, bool x7)       dpe_run_pipeline(dense_folder, options)
 *     main.h:120, main.cpp:474
 *   ProcessProblem / DPE::InuputInitialization   (internal: one pass of one reference image)
 *     main.cpp:411-446, DPE.cpp:733-914
 *   cv::imread(IMREAD_GRAYSCALE)                 dpe_host_read_gray (JPEG islow luma / PGM)
 *   cv::resize(INTER_LINEAR)  DPE.cpp:808        dpe_host_resize_linear
 *   RescaleMatToTargetSize    DPE.cpp:1146       dpe_host_rescale_nearest
 *   EdgeSegment               DPE.cpp:129-291    dpe_host_edge_segment (GetProblemEdges, main.cpp:331,
 *                                                runs inside dpe_run_pipeline for missing maps)
 *   cv::Canny(L2, aperture 3) DPE.cpp:226        dpe_host_canny
 *   cv::resize INTER_LINEAR 8U DPE.cpp:145,230   dpe_host_resize_u8
 *   Connect                   DPE.cpp:27-127     dpe_host_connect
 *   RunFusion / ExportPointCloud DPE.cpp:1220,532 inside dpe_run_pipeline (fusion = true): projection
 *                                                tests on the GPU (dpe_fusion_candidates), serial rest
 *   cv::imread(IMREAD_COLOR)  DPE.cpp:1253       dpe_host_read_bgr
 *   cv::HoughLinesP           DPE.cpp:186        dpe_host_hough_lines_p
 *
 * Additions for the one-process-per-GPU deployment: a pass runner hook (default: the HIP library
 * on `gpu_index`) and an all-gather hook for the depth maps (RCCL in the CLI, torch.distributed
 * from Python).  Plain C types only.
 */
#ifndef DPE_HOST_H_
#define DPE_HOST_H_

#include <stddef.h>
#include <stdint.h>
#ifndef __cplusplus
#include <stdbool.h>
#endif

#include "dpe_mvs.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Runs one PatchMatch pass: same contract as dpe_pm_run (stage + execute + fetch). */
typedef int (*dpe_pass_runner_fn)(void* user, const DpePassInput* in, const DpePassState* state);
/* All-gather of `count` floats per rank into recv[world * count], rank-major.  0 = success. */
typedef int (*dpe_allgather_fn)(void* user, const float* send, size_t count, float* recv);
/* The same all-gather on DEVICE buffers of the pipeline's GPU (RCCL over xGMI in the CLI); the hook
 * returns once recv is complete.  With the default runner the depth maps then go from each rank's
 * HBM-resident state to the others' without a host copy. */
typedef int (*dpe_allgather_dev_fn)(void* user, const float* dev_send, size_t count, float* dev_recv);
/* Optional: called once when one of this rank's collectives failed, before dpe_run_pipeline returns,
 * so that peers blocked in theirs fail fast (bin/dpe: ncclCommAbort).  Return value ignored. */
typedef int (*dpe_abort_fn)(void* user);

/* Fusion projection tests of one reference view: same contract as dpe_fusion_candidates
 * (include/dpe_mvs.h) over the given views (the default runs the HIP kernel on gpu_index). */
typedef int (*dpe_fusion_fn)(void* user, const DpeFusionView* views, int n_views, int ref, const int* src, int ns,
                             int32_t* idx, float* val);

enum { DPE_SCHEDULE_REFERENCE = 0, DPE_SCHEDULE_JACOBI = 1 };

typedef struct DpePipelineOptions {
  int gpu_index;            /* device of the default runner */
  bool verbose, fusion, viz, depth, normal, weak, edge;   /* RunDPEPipeline's flags */
  int schedule;             /* DPE_SCHEDULE_*: reference = serial order (later images see this
                               pass's depths of earlier ones); jacobi = depths of the previous pass */
  int rank, world_size;     /* problems are split in contiguous blocks; world > 1 forces jacobi */
  dpe_allgather_fn allgather; void* allgather_user;   /* required when world_size > 1 */
  dpe_pass_runner_fn runner; void* runner_user;       /* NULL: libdpe_mvs on gpu_index */
  uint64_t base_seed;       /* Philox key of image i: base_seed ^ (i * 0x9E3779B97F4A7C15) */
  bool keep_intermediate;   /* also write depths.dmb / normals.dmb / weak.bin / selected_views.bin and
                               keep edges_<s>.dmb / labels_<s>.dmb (the reference deletes them) */
  dpe_fusion_fn fusion_runner; void* fusion_user;     /* NULL: the HIP kernel on gpu_index */
  int max_iterations;       /* PatchMatch iterations per pass; 0 = the reference's 3 (main.cpp:527, 554) */
  bool photometric_only;    /* geom_consistency = false on every pass (BASELINE config 2; the
                               reference always runs its geometric passes, main.cpp:549) */
  dpe_allgather_dev_fn allgather_device; void* allgather_device_user;   /* optional (see above); with the
                               default runner it is used instead of `allgather` for the depth maps */
  dpe_abort_fn abort_collectives; void* abort_user;   /* optional (see dpe_abort_fn) */
} DpePipelineOptions;

void dpe_pipeline_default_options(DpePipelineOptions* opt);
/* RunDPEPipeline: 0 on success, nonzero on failure (message in dpe_pipeline_last_error()). */
int dpe_run_pipeline(const char* dense_folder, const DpePipelineOptions* opt);
const char* dpe_pipeline_last_error(void);
/* Wall seconds of the last successful dpe_run_pipeline on this process: [0] total, [1] image decode,
 * [2] the GetProblemEdges pre-pass (EdgeSegment), [3] the passes (with the depth exchanges),
 * [4] outputs + fusion, [5] the depth exchanges alone (multi-rank: status all-gather, export,
 * all-gather, import, summed over the pass rounds; 0 for one rank), [6] the pass work alone (each
 * pass round up to its GPU work's end, on one rank too), [7] RunFusion (part of [4]; with several
 * ranks it includes the exchange of the final normals / pixel states; 0 without fusion).  Returns
 * the number of entries written (<= n, at most 8). */
int dpe_pipeline_last_timings(double* out, int n);

/* Grey-level decode of a JPEG (baseline/extended, luma plane) or binary PGM.  Writes up to `cap`
 * bytes into `out` (pass NULL/0 to query the size) and the size into *w, *h.  0 on success. */
int dpe_host_read_gray(const char* path, uint8_t* out, size_t cap, int* w, int* h);
/* Colour decode (cv::imread IMREAD_COLOR): 8-bit BGR, up to `cap` bytes; size query with out = NULL. */
int dpe_host_read_bgr(const char* path, uint8_t* out, size_t cap, int* w, int* h);
/* ReadCamera (DPE.cpp:341-382): extrinsic, intrinsic, "dmin interval num dmax" line.  0 on success. */
int dpe_host_read_camera(const char* path, DpeCamera* cam);
/* cv::resize INTER_LINEAR of a CV_32FC1 image (float weights, horizontal then vertical pass). */
void dpe_host_resize_linear(const float* src, int w, int h, float* dst, int nw, int nh);
/* RescaleMatToTargetSize: nearest with the reference's swapped factors; `elem` bytes per pixel;
 * destination pixels whose source falls outside keep their (caller-initialised) value. */
void dpe_host_rescale_nearest(const void* src, int w, int h, void* dst, int nw, int nh, int elem);

/* EdgeSegment (DPE.cpp:129-291): mode 0 = edges (uint8 0/255, same size as src, use_canny = 1 in the
 * reference's call), mode 1 = labels (int32: -1 small region, 0 boundary, > 0 region; size
 * round(src / 2^scale), use_canny = 0).  Writes up to `cap` bytes into `out` (NULL: size query via
 * *ow, *oh).  0 on success. */
int dpe_host_edge_segment(int scale, const uint8_t* src, int w, int h, int mode, int use_canny, int high_res, void* out,
                          size_t cap, int* ow, int* oh);
/* cv::Canny(src, dst, low, high, 3, L2gradient = true): dst uint8 0/255.  0 on success. */
int dpe_host_canny(const uint8_t* src, int w, int h, double low, double high, uint8_t* dst);
/* cv::resize(INTER_LINEAR) of a CV_8UC1 image (exact 1/2: INTER_AREA fast path).  0 on success. */
int dpe_host_resize_u8(const uint8_t* src, int w, int h, uint8_t* dst, int nw, int nh);
/* Connect (DPE.cpp:27-127): labels of the 4-connected zero regions (255 -> 0); returns the label
 * count (label_cnt entries, written up to cnt_cap) or -1. */
int dpe_host_connect(const uint8_t* img, int w, int h, int* label, int* cnt, int cnt_cap);
/* cv::HoughLinesP: writes up to `cap` segments (x0, y0, x1, y1) into `lines`; returns the count or -1. */
int dpe_host_hough_lines_p(const uint8_t* img, int w, int h, double rho, double theta, int threshold, double min_len,
                           double max_gap, int* lines, int cap);

#ifdef __cplusplus
}
#endif
#endif /* DPE_HOST_H_ */
