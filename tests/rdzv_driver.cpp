// Test driver of dpe-mvs_amd/host/rdzv.h (tests/test_rdzv.py): `rdzv_driver rank world`; rank 0
// serves a fixed 128-byte id, every rank prints the id it ends with as hex (or FAIL).
// `rdzv_driver bind MASTER_ADDR RESOLVED_IPV4 world` prints the address rank 0 would listen on.
#include <cstdio>
#include <cstdlib>
#include <string>
#include "../dpe-mvs_amd/host/rdzv.h"

int main(int argc, char** argv) {
  if (argc == 5 && std::string(argv[1]) == "bind") {
    in_addr a;
    if (::inet_pton(AF_INET, argv[3], &a) != 1) return 2;
    in_addr o;
    o.s_addr = htonl(dpe_rdzv::listen_addr(argv[2], ntohl(a.s_addr), std::atoi(argv[4])));
    char buf[INET_ADDRSTRLEN];
    std::printf("%s\n", ::inet_ntop(AF_INET, &o, buf, sizeof(buf)));
    return 0;
  }
  if (argc < 3) return 2;
  const int rank = std::atoi(argv[1]), world = std::atoi(argv[2]);
  unsigned char id[128];
  for (int i = 0; i < 128; ++i) id[i] = rank == 0 ? (unsigned char)(i * 37 + 11) : 0;
  if (!dpe_rdzv::exchange_blob(id, sizeof(id), rank, world)) { std::printf("FAIL\n"); return 1; }
  for (int i = 0; i < 128; ++i) std::printf("%02x", id[i]);
  std::printf("\n");
  return 0;
}
