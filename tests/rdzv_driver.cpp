// Test driver of dpe-mvs_amd/host/rdzv.h (tests/test_rdzv.py): `rdzv_driver rank world`; rank 0
// serves a fixed 128-byte id, every rank prints the id it ends with as hex (or FAIL).
#include <cstdio>
#include <cstdlib>
#include "../dpe-mvs_amd/host/rdzv.h"

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const int rank = std::atoi(argv[1]), world = std::atoi(argv[2]);
  unsigned char id[128];
  for (int i = 0; i < 128; ++i) id[i] = rank == 0 ? (unsigned char)(i * 37 + 11) : 0;
  if (!dpe_rdzv::exchange_blob(id, sizeof(id), rank, world)) { std::printf("FAIL\n"); return 1; }
  for (int i = 0; i < 128; ++i) std::printf("%02x", id[i]);
  std::printf("\n");
  return 0;
}
