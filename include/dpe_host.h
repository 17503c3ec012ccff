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
  bool keep_intermediate;   /* also write depths.dmb / normals.dmb / weak.bin / selected_views.bin */
} DpePipelineOptions;

void dpe_pipeline_default_options(DpePipelineOptions* opt);
/* RunDPEPipeline: 0 on success, nonzero on failure (message in dpe_pipeline_last_error()). */
int dpe_run_pipeline(const char* dense_folder, const DpePipelineOptions* opt);
const char* dpe_pipeline_last_error(void);

/* Grey-level decode of a JPEG (baseline/extended, luma plane) or binary PGM.  Writes up to `cap`
 * bytes into `out` (pass NULL/0 to query the size) and the size into *w, *h.  0 on success. */
int dpe_host_read_gray(const char* path, uint8_t* out, size_t cap, int* w, int* h);
/* ReadCamera (DPE.cpp:341-382): extrinsic, intrinsic, "dmin interval num dmax" line.  0 on success. */
int dpe_host_read_camera(const char* path, DpeCamera* cam);
/* cv::resize INTER_LINEAR of a CV_32FC1 image (float weights, horizontal then vertical pass). */
void dpe_host_resize_linear(const float* src, int w, int h, float* dst, int nw, int nh);
/* RescaleMatToTargetSize: nearest with the reference's swapped factors; `elem` bytes per pixel;
 * destination pixels whose source falls outside keep their (caller-initialised) value. */
void dpe_host_rescale_nearest(const void* src, int w, int h, void* dst, int nw, int nh, int elem);

#ifdef __cplusplus
}
#endif
#endif /* DPE_HOST_H_ */
