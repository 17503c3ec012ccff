// rdzv.h — the `dpe` command line's rendezvous: rank 0 hands an opaque id (the RCCL unique id) to
// ranks 1..world-1 over TCP at MASTER_ADDR:port (DPE_RDZV_PORT, default MASTER_PORT + 1).
// Header-only so that tests/test_rdzv.py can drive it without a GPU (tests/rdzv_driver.cpp).
#pragma once
#include <arpa/inet.h>
#include <netdb.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <vector>

#include <algorithm>
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

// The hello a rank sends before rank 0 hands it the id: magic, rank and a run token, so that a port
// scan, a health probe or a leftover rank of another job cannot take a slot or receive this job's
// communicator id.  The token hashes DPE_RDZV_SECRET when the launcher sets one (a random value handed
// to every rank of the job: then only holders of the secret get the id, i.e. the rendezvous is
// authenticated); without it the token hashes TORCHELASTIC_RUN_ID, else MASTER_ADDR:MASTER_PORT, which
// are not secret: that token tells jobs apart, it does not authenticate a peer.
struct Hello {
  uint32_t magic;
  int32_t rank;
  uint64_t token;
};
constexpr uint32_t kHelloMagic = 0x44504531u;   // "DPE1"

inline uint64_t run_token() {
  const char* sec = std::getenv("DPE_RDZV_SECRET");
  const char* id = std::getenv("TORCHELASTIC_RUN_ID");
  std::string t = sec && *sec ? std::string("secret:") + sec : (id ? std::string("run:") + id : std::string());
  if (t.empty()) {
    const char* a = std::getenv("MASTER_ADDR");
    const char* p = std::getenv("MASTER_PORT");
    t = std::string("addr:") + (a ? a : "127.0.0.1") + ":" + (p ? p : "");
  }
  uint64_t h = 1469598103934665603ull;            // FNV-1a
  for (unsigned char c : t) { h ^= c; h *= 1099511628211ull; }
  return h;
}

// The address rank 0 listens on, given MASTER_ADDR (`addr`) and the address it resolved to
// (`resolved`, host order).  Normally that address.  The one exception: MASTER_ADDR is a host NAME
// (not a numeric literal, not "localhost") that resolves to a loopback address (/etc/hosts often
// maps a host's own name to 127.0.1.1) while some ranks may run on other hosts (LOCAL_WORLD_SIZE
// unset or below the world size): remote ranks could then never connect, so rank 0 listens on
// every interface -- but only when the launcher gave the ranks DPE_RDZV_SECRET, which makes the
// hello token a secret.  Without it the run token is built from non-secret values, so widening
// would hand the communicator id to anyone on the network who guesses them: the listener stays on
// loopback and a warning says why.  A numeric loopback literal or "localhost" never widens.
inline uint32_t listen_addr(const char* addr, uint32_t resolved, int world, bool* warned = nullptr) {
  if (warned) *warned = false;
  if ((resolved >> 24) != 127) return resolved;
  const char* lws = std::getenv("LOCAL_WORLD_SIZE");
  if (lws && std::atoi(lws) >= world) return resolved;
  in_addr tmp;
  if (!addr || ::inet_pton(AF_INET, addr, &tmp) == 1 || std::strcmp(addr, "localhost") == 0) return resolved;
  const char* sec = std::getenv("DPE_RDZV_SECRET");
  if (!(sec && *sec)) {
    if (warned) *warned = true;
    std::fprintf(stderr, "dpe rendezvous: MASTER_ADDR %s resolves to a loopback address; remote ranks cannot reach it, "
                         "and without DPE_RDZV_SECRET rank 0 does not listen on every interface\n", addr);
    return resolved;
  }
  return INADDR_ANY;
}

// Rank 0 listens (listen_addr) and serves the id to each rank 1..world-1 once, after checking its
// hello; connections that fail the check are dropped and do not use up a slot.  Pending connections
// are served concurrently (poll), each with a 2 s budget for its hello, so connections that send
// nothing cannot use up the 120 s window of the legitimate ranks.  The others connect (retrying for
// up to 120 s while rank 0 starts).  Every socket call is bounded, so a missing peer ends in an
// error, not a hang.
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
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  const auto left = [&]() { return std::chrono::seconds(120) - (clock::now() - t0); };
  if (rank == 0) {
    const int srv = ::socket(AF_INET, SOCK_STREAM, 0);
    if (srv < 0) { ::freeaddrinfo(res); return false; }
    const int one = 1;
    ::setsockopt(srv, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in sa;
    std::memcpy(&sa, res->ai_addr, sizeof(sa));
    ::freeaddrinfo(res);
    sa.sin_addr.s_addr = htonl(listen_addr(addr, ntohl(sa.sin_addr.s_addr), world));
    bool ok = ::bind(srv, (const sockaddr*)&sa, sizeof(sa)) == 0 && ::listen(srv, 64) == 0 &&
              ::fcntl(srv, F_SETFL, ::fcntl(srv, F_GETFL) | O_NONBLOCK) == 0;
    struct Pending { int fd; clock::time_point deadline; Hello h; size_t got; };
    std::vector<Pending> pend;
    std::string seen((size_t)world, '\0');
    int served = 0;
    const timeval sv{2, 0};
    while (ok && served < world - 1 && left().count() > 0) {
      std::vector<pollfd> fds(1 + pend.size());
      fds[0] = {srv, POLLIN, 0};
      auto wait = std::chrono::duration_cast<std::chrono::milliseconds>(left());
      for (size_t i = 0; i < pend.size(); ++i) {
        fds[1 + i] = {pend[i].fd, POLLIN, 0};
        wait = std::min(wait, std::chrono::duration_cast<std::chrono::milliseconds>(pend[i].deadline - clock::now()));
      }
      if (::poll(fds.data(), fds.size(), (int)std::max<long long>(0, std::min<long long>(wait.count(), 1000))) < 0 && errno != EINTR) {
        ok = false;
        break;
      }
      for (size_t i = 0; i < pend.size(); ++i) {   // hellos in progress
        Pending& q = pend[i];
        bool done = false;
        if (fds[1 + i].revents) {
          const ssize_t k = ::recv(q.fd, reinterpret_cast<char*>(&q.h) + q.got, sizeof(Hello) - q.got, MSG_DONTWAIT);
          if (k > 0) q.got += (size_t)k;
          else if (k == 0 || (errno != EAGAIN && errno != EWOULDBLOCK)) done = true;
          if (q.got == sizeof(Hello)) {
            const Hello& h = q.h;
            if (h.magic == kHelloMagic && h.token == token && h.rank > 0 && h.rank < world && !seen[(size_t)h.rank]) {
              ::setsockopt(q.fd, SOL_SOCKET, SO_SNDTIMEO, &sv, sizeof(sv));
              const int fl = ::fcntl(q.fd, F_GETFL);
              ::fcntl(q.fd, F_SETFL, fl & ~O_NONBLOCK);
              if (send_all(q.fd, id, id_bytes)) { seen[(size_t)h.rank] = 1; ++served; }
            }
            done = true;
          }
        }
        if (done || clock::now() >= q.deadline) { ::close(q.fd); q.fd = -1; }
      }
      pend.erase(std::remove_if(pend.begin(), pend.end(), [](const Pending& q) { return q.fd < 0; }), pend.end());
      if (fds[0].revents & POLLIN)   // new connections: each gets 2 s to say hello
        for (int c; (c = ::accept(srv, nullptr, nullptr)) >= 0;) {
          ::fcntl(c, F_SETFL, ::fcntl(c, F_GETFL) | O_NONBLOCK);
          if (pend.size() >= 256) { ::close(c); continue; }
          pend.push_back(Pending{c, clock::now() + std::chrono::seconds(2), Hello{}, 0});
        }
    }
    for (Pending& q : pend) ::close(q.fd);
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
