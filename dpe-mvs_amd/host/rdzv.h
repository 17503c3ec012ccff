// rdzv.h — the `dpe` command line's rendezvous: rank 0 hands an opaque id (the RCCL unique id) to
// ranks 1..world-1 over TCP at MASTER_ADDR:port (DPE_RDZV_PORT, default MASTER_PORT + 1).
// Header-only so that tests/test_rdzv.py can drive it without a GPU (tests/rdzv_driver.cpp).
#pragma once
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

namespace dpe_rdzv {

inline bool send_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    const ssize_t k = ::send(fd, c, n, 0);
    if (k <= 0) return false;
    c += k; n -= (size_t)k;
  }
  return true;
}
inline bool recv_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k <= 0) return false;
    c += k; n -= (size_t)k;
  }
  return true;
}

// The hello a rank sends before rank 0 hands it the id: magic, rank and a run token (a hash of
// TORCHELASTIC_RUN_ID, else of MASTER_ADDR:MASTER_PORT), so that a port scan, a health probe or a
// leftover rank of another job cannot take a slot or receive this job's communicator id.
struct Hello {
  uint32_t magic;
  int32_t rank;
  uint64_t token;
};
constexpr uint32_t kHelloMagic = 0x44504531u;   // "DPE1"

inline uint64_t run_token() {
  const char* id = std::getenv("TORCHELASTIC_RUN_ID");
  std::string t = id ? std::string("run:") + id : std::string();
  if (t.empty()) {
    const char* a = std::getenv("MASTER_ADDR");
    const char* p = std::getenv("MASTER_PORT");
    t = std::string("addr:") + (a ? a : "127.0.0.1") + ":" + (p ? p : "");
  }
  uint64_t h = 1469598103934665603ull;            // FNV-1a
  for (unsigned char c : t) { h ^= c; h *= 1099511628211ull; }
  return h;
}

// Rank 0 listens on MASTER_ADDR (not INADDR_ANY) and serves the id to each rank 1..world-1 once,
// after checking its hello; connections that fail the check are dropped and do not use up a slot.
// The others connect (retrying for up to 120 s while rank 0 starts).  Every socket call is
// bounded, so a missing peer ends in an error, not a hang.
inline bool exchange_blob(void* id, size_t id_bytes, int rank, int world) {
  const char* addr = std::getenv("MASTER_ADDR");
  const char* rp = std::getenv("DPE_RDZV_PORT");
  const char* mp = std::getenv("MASTER_PORT");
  const int port = rp ? std::atoi(rp) : (mp ? std::atoi(mp) + 1 : 29501);
  const uint64_t token = run_token();
  timeval tv{120, 0};
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (::getaddrinfo(addr ? addr : "127.0.0.1", std::to_string(port).c_str(), &hints, &res) != 0 || !res) return false;
  const auto t0 = std::chrono::steady_clock::now();
  const auto left = [&]() { return std::chrono::seconds(120) - (std::chrono::steady_clock::now() - t0); };
  if (rank == 0) {
    const int srv = ::socket(AF_INET, SOCK_STREAM, 0);
    if (srv < 0) { ::freeaddrinfo(res); return false; }
    const int one = 1;
    ::setsockopt(srv, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    ::setsockopt(srv, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    bool ok = ::bind(srv, res->ai_addr, res->ai_addrlen) == 0 && ::listen(srv, world) == 0;
    ::freeaddrinfo(res);
    std::string seen((size_t)world, '\0');
    int served = 0;
    while (ok && served < world - 1 && left().count() > 0) {
      const int c = ::accept(srv, nullptr, nullptr);   // SO_RCVTIMEO bounds the wait
      if (c < 0) { ok = false; break; }
      timeval hv{5, 0};                                  // a silent peer cannot stall the others long
      ::setsockopt(c, SOL_SOCKET, SO_RCVTIMEO, &hv, sizeof(hv));
      ::setsockopt(c, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
      Hello h{};
      if (recv_all(c, &h, sizeof(h)) && h.magic == kHelloMagic && h.token == token && h.rank > 0 && h.rank < world &&
          !seen[(size_t)h.rank] && send_all(c, id, id_bytes)) {
        seen[(size_t)h.rank] = 1;
        ++served;
      }
      ::close(c);
    }
    ::close(srv);
    return ok && served == world - 1;
  }
  bool ok = false;
  const Hello h{kHelloMagic, (int32_t)rank, token};
  while (!ok && left().count() > 0) {
    const int c = ::socket(AF_INET, SOCK_STREAM, 0);
    if (c < 0) break;
    ::setsockopt(c, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    if (::connect(c, res->ai_addr, res->ai_addrlen) == 0) ok = send_all(c, &h, sizeof(h)) && recv_all(c, id, id_bytes);
    ::close(c);
    if (!ok) std::this_thread::sleep_for(std::chrono::milliseconds(100));
  }
  ::freeaddrinfo(res);
  return ok;
}

}  // namespace dpe_rdzv
