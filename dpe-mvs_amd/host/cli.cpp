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
// earlier run cannot be read.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

#include "../../include/dpe_host.h"

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

// device buffers on both sides: the depth maps go from HBM to HBM over xGMI with no host copy
int rccl_allgather_dev(void* user, const float* dsend, size_t count, float* drecv) {
  Rccl* r = static_cast<Rccl*>(user);
  if (ncclAllGather(dsend, drecv, count, ncclFloat, r->comm, r->stream) != ncclSuccess) return -1;
  return hipStreamSynchronize(r->stream) == hipSuccess ? 0 : -1;
}

bool send_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    const ssize_t k = ::send(fd, c, n, 0);
    if (k <= 0) return false;
    c += k; n -= (size_t)k;
  }
  return true;
}
bool recv_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k <= 0) return false;
    c += k; n -= (size_t)k;
  }
  return true;
}

// Rank 0 serves the id to world - 1 connections; the others connect (retrying for up to 120 s while
// rank 0 starts).  Every socket call is bounded, so a missing peer ends in an error, not a hang.
bool exchange_unique_id(ncclUniqueId& id, int rank, int world) {
  const char* addr = std::getenv("MASTER_ADDR");
  const char* rp = std::getenv("DPE_RDZV_PORT");
  const char* mp = std::getenv("MASTER_PORT");
  const int port = rp ? std::atoi(rp) : (mp ? std::atoi(mp) + 1 : 29501);
  timeval tv{120, 0};
  if (rank == 0) {
    const int srv = ::socket(AF_INET, SOCK_STREAM, 0);
    if (srv < 0) return false;
    const int one = 1;
    ::setsockopt(srv, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    ::setsockopt(srv, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
    sa.sin_port = htons((uint16_t)port);
    bool ok = ::bind(srv, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) == 0 && ::listen(srv, world) == 0;
    for (int k = 1; ok && k < world; ++k) {
      const int c = ::accept(srv, nullptr, nullptr);   // SO_RCVTIMEO bounds the wait
      if (c < 0) { ok = false; break; }
      ::setsockopt(c, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
      ok = send_all(c, &id, sizeof(id));
      ::close(c);
    }
    ::close(srv);
    return ok;
  }
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (::getaddrinfo(addr ? addr : "127.0.0.1", std::to_string(port).c_str(), &hints, &res) != 0 || !res) return false;
  const auto t0 = std::chrono::steady_clock::now();
  bool ok = false;
  while (!ok && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(120)) {
    const int c = ::socket(AF_INET, SOCK_STREAM, 0);
    if (c < 0) break;
    ::setsockopt(c, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    if (::connect(c, res->ai_addr, res->ai_addrlen) == 0) ok = recv_all(c, &id, sizeof(id));
    ::close(c);
    if (!ok) std::this_thread::sleep_for(std::chrono::milliseconds(100));
  }
  ::freeaddrinfo(res);
  return ok;
}

bool rccl_init(Rccl& r, int rank, int world, int device) {
  r.world = world;
  if (hipSetDevice(device) != hipSuccess) return false;
  ncclUniqueId id;
  std::memset(&id, 0, sizeof(id));
  if (rank == 0 && ncclGetUniqueId(&id) != ncclSuccess) return false;
  if (!exchange_unique_id(id, rank, world)) return false;
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
  }
  const int rc = dpe_run_pipeline(argv[1], &o);
  if (rc != 0) std::fprintf(stderr, "DPE pipeline failed: %s\n", dpe_pipeline_last_error());
  if (rccl.comm) ncclCommDestroy(rccl.comm);
  return rc == 0 ? EXIT_SUCCESS : EXIT_FAILURE;
}
