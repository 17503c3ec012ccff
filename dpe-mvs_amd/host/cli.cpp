// cli.cpp — the `dpe` command line, same positional arguments as the reference's `DPE` binary
// (main.cpp:602-635):
//
//     dpe dense_folder [gpu_index] [verbose] [viz] [fusion] [depth] [normal] [weak] [edge]
//
// One process per GPU: launched under torchrun (or any launcher that sets RANK / WORLD_SIZE /
// LOCAL_RANK), each rank takes a contiguous block of reference images on GPU LOCAL_RANK and the
// depth maps are all-gathered after every pass with RCCL over xGMI.  The RCCL unique id goes from
// rank 0 to the others over a TCP socket at MASTER_ADDR, port DPE_RDZV_PORT (default MASTER_PORT + 1,
// beside the launcher's own store): nothing is written to the dataset folder and a stale id from an
// earlier run cannot be read.  Rank 0 listens on MASTER_ADDR only and answers a rank only after its
// hello (rank + run token) checks out.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <string>
#include <thread>

#include "../../include/dpe_host.h"
#include "rdzv.h"

namespace {

struct Rccl {
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  float* dsend = nullptr;   // host all-gather staging, kStageFloats per rank
  float* drecv = nullptr;
  int world = 1;
};

// Host buffers (the per-exchange status flags, the runner-hook path, fusion's one-off exchange).
// Every call enters the same collectives on every rank whatever fails locally, so a peer is never
// left waiting in ncclAllGather: the staging buffers are allocated once at start-up (rccl_init,
// before the rendezvous) and a count beyond them goes in chunks of that fixed size, which every
// rank derives the same way.
constexpr size_t kStageFloats = 1u << 20;   // 4 MB send + world x 4 MB receive
int rccl_allgather(void* user, const float* send, size_t count, float* recv) {
  Rccl* r = static_cast<Rccl*>(user);
  bool ok = true;
  for (size_t off = 0; off < count; off += kStageFloats) {
    const size_t n = std::min(kStageFloats, count - off);
    ok = hipMemcpyAsync(r->dsend, send + off, n * sizeof(float), hipMemcpyHostToDevice, r->stream) == hipSuccess && ok;
    ok = ncclAllGather(r->dsend, r->drecv, n, ncclFloat, r->comm, r->stream) == ncclSuccess && ok;
    ok = hipMemcpy2DAsync(recv + off, count * sizeof(float), r->drecv, n * sizeof(float), n * sizeof(float), r->world,
                          hipMemcpyDeviceToHost, r->stream) == hipSuccess && ok;
    ok = hipStreamSynchronize(r->stream) == hipSuccess && ok;
  }
  return ok ? 0 : -1;
}

// device buffers on both sides: the depth maps go from HBM to HBM over xGMI with no host copy
int rccl_allgather_dev(void* user, const float* dsend, size_t count, float* drecv) {
  Rccl* r = static_cast<Rccl*>(user);
  if (ncclAllGather(dsend, drecv, count, ncclFloat, r->comm, r->stream) != ncclSuccess) return -1;
  return hipStreamSynchronize(r->stream) == hipSuccess ? 0 : -1;
}

// a failed collective on this rank: abort the communicator so that peers blocked in theirs fail
// fast (dpe_abort_fn) instead of waiting for RCCL's timeout
int rccl_abort(void* user) {
  Rccl* r = static_cast<Rccl*>(user);
  if (r->comm) { (void)ncclCommAbort(r->comm); r->comm = nullptr; }
  return 0;
}

bool rccl_init(Rccl& r, int rank, int world, int device) {
  r.world = world;
  if (hipSetDevice(device) != hipSuccess) return false;
  // the host all-gather's staging buffers, before any rank commits to a collective
  if (hipMalloc(&r.dsend, kStageFloats * sizeof(float)) != hipSuccess) return false;
  if (hipMalloc(&r.drecv, kStageFloats * sizeof(float) * world) != hipSuccess) return false;
  ncclUniqueId id;
  std::memset(&id, 0, sizeof(id));
  if (rank == 0 && ncclGetUniqueId(&id) != ncclSuccess) return false;
  if (!dpe_rdzv::exchange_blob(&id, sizeof(id), rank, world)) return false;
  if (hipStreamCreate(&r.stream) != hipSuccess) return false;
  return ncclCommInitRank(&r.comm, world, id, rank) == ncclSuccess;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "USAGE: DPE dense_folder\n");
    return EXIT_FAILURE;
  }
  DpePipelineOptions o;
  dpe_pipeline_default_options(&o);
  if (argc >= 3) o.gpu_index = std::atoi(argv[2]);
  if (argc >= 4) o.verbose = std::atoi(argv[3]);
  if (argc >= 5) o.viz = std::atoi(argv[4]);
  if (argc >= 6) o.fusion = std::atoi(argv[5]);
  if (argc >= 7) o.depth = std::atoi(argv[6]);
  if (argc >= 8) o.normal = std::atoi(argv[7]);
  if (argc >= 9) o.weak = std::atoi(argv[8]);
  if (argc >= 10) o.edge = std::atoi(argv[9]);
  const char* ws = std::getenv("WORLD_SIZE");
  Rccl rccl;
  if (ws && std::atoi(ws) > 1) {
    o.world_size = std::atoi(ws);
    o.rank = std::atoi(std::getenv("RANK") ? std::getenv("RANK") : "0");
    o.gpu_index = std::atoi(std::getenv("LOCAL_RANK") ? std::getenv("LOCAL_RANK") : "0");
    if (!rccl_init(rccl, o.rank, o.world_size, o.gpu_index)) {
      std::fprintf(stderr, "RCCL initialisation failed\n");
      return EXIT_FAILURE;
    }
    o.allgather = rccl_allgather;          // host buffers (runner hooks, fusion's one-off exchange)
    o.allgather_user = &rccl;
    o.allgather_device = rccl_allgather_dev;   // the per-pass depth maps, HBM to HBM
    o.allgather_device_user = &rccl;
    o.abort_collectives = rccl_abort;
    o.abort_user = &rccl;
  }
  const int rc = dpe_run_pipeline(argv[1], &o);
  if (rc != 0) std::fprintf(stderr, "DPE pipeline failed: %s\n", dpe_pipeline_last_error());
  if (rccl.comm) ncclCommDestroy(rccl.comm);
  return rc == 0 ? EXIT_SUCCESS : EXIT_FAILURE;
}
