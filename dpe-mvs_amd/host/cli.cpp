// cli.cpp — the `dpe` command line, same positional arguments as the reference's `DPE` binary
// (main.cpp:602-635):
//
//     dpe dense_folder [gpu_index] [verbose] [viz] [fusion] [depth] [normal] [weak] [edge]
//
// One process per GPU: launched under torchrun (or any launcher that sets RANK / WORLD_SIZE /
// LOCAL_RANK), each rank takes a contiguous block of reference images on GPU LOCAL_RANK and the
// depth maps are all-gathered after every pass with RCCL over xGMI.  The RCCL unique id is handed
// from rank 0 to the others through a file in <dense_folder>/DPE/.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <string>
#include <thread>

#include "../../include/dpe_host.h"

namespace fs = std::filesystem;

namespace {

struct Rccl {
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  float* dsend = nullptr;
  float* drecv = nullptr;
  size_t cap = 0;
  int world = 1;
};

int rccl_allgather(void* user, const float* send, size_t count, float* recv) {
  Rccl* r = static_cast<Rccl*>(user);
  if (count > r->cap) {
    if (r->dsend) { (void)hipFree(r->dsend); (void)hipFree(r->drecv); }
    if (hipMalloc(&r->dsend, count * sizeof(float)) != hipSuccess) return -1;
    if (hipMalloc(&r->drecv, count * sizeof(float) * r->world) != hipSuccess) return -1;
    r->cap = count;
  }
  if (hipMemcpyAsync(r->dsend, send, count * sizeof(float), hipMemcpyHostToDevice, r->stream) != hipSuccess) return -1;
  if (ncclAllGather(r->dsend, r->drecv, count, ncclFloat, r->comm, r->stream) != ncclSuccess) return -1;
  if (hipMemcpyAsync(recv, r->drecv, count * sizeof(float) * r->world, hipMemcpyDeviceToHost, r->stream) != hipSuccess) return -1;
  return hipStreamSynchronize(r->stream) == hipSuccess ? 0 : -1;
}

bool rccl_init(Rccl& r, int rank, int world, int device, const std::string& dense) {
  r.world = world;
  if (hipSetDevice(device) != hipSuccess) return false;
  const char* port = std::getenv("MASTER_PORT");
  const fs::path dir = fs::path(dense) / "DPE";
  std::error_code ec;
  fs::create_directories(dir, ec);
  const fs::path idfile = dir / (std::string(".rccl_uid_") + (port ? port : "0"));
  ncclUniqueId id;
  if (rank == 0) {
    if (ncclGetUniqueId(&id) != ncclSuccess) return false;
    const fs::path tmp = idfile.string() + ".tmp";
    { std::ofstream o(tmp, std::ios::binary); o.write(reinterpret_cast<const char*>(&id), sizeof(id)); }
    fs::rename(tmp, idfile, ec);
    if (ec) return false;
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      std::ifstream in(idfile, std::ios::binary);
      if (in && in.read(reinterpret_cast<char*>(&id), sizeof(id))) break;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) return false;
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
  }
  if (hipStreamCreate(&r.stream) != hipSuccess) return false;
  if (ncclCommInitRank(&r.comm, world, id, rank) != ncclSuccess) return false;
  if (rank == 0) fs::remove(idfile, ec);
  return true;
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
    if (!rccl_init(rccl, o.rank, o.world_size, o.gpu_index, argv[1])) {
      std::fprintf(stderr, "RCCL initialisation failed\n");
      return EXIT_FAILURE;
    }
    o.allgather = rccl_allgather;
    o.allgather_user = &rccl;
  }
  const int rc = dpe_run_pipeline(argv[1], &o);
  if (rc != 0) std::fprintf(stderr, "DPE pipeline failed: %s\n", dpe_pipeline_last_error());
  if (rccl.comm) ncclCommDestroy(rccl.comm);
  return rc == 0 ? EXIT_SUCCESS : EXIT_FAILURE;
}
