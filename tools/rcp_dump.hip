// Dumps v_rcp_f32 over every mantissa at biased exponent 127 (z in [1, 2)) for the oracle's model
// of the tap reciprocal (oracle/oracle_math.h o_rcp_hw, restatement choice 8), and checks the two
// facts that model rests on: rcp(-z) == -rcp(z), and rcp(m * 2^k) == rcp(m) * 2^-k for every
// biased exponent 1..252 (all 2^23 mantissas each).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/rcp_dump.hip -o /tmp/rcp_dump && /tmp/rcp_dump out.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void dump(uint32_t* out) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= (1u << 23)) return;
  out[m] = __float_as_uint(__builtin_amdgcn_rcpf(__uint_as_float((127u << 23) | m)));
}
// bad[0]: (exponent, sign) pairs x mantissas whose rcp is not the exponent-127 result scaled
__global__ void check(const uint32_t* base, unsigned long long* bad) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= (1u << 23)) return;
  unsigned long long n = 0;
  for (uint32_t e = 1; e <= 252; ++e)
    for (uint32_t s = 0; s < 2; ++s) {
      const float z = __uint_as_float((s << 31) | (e << 23) | m);
      const uint32_t r = __float_as_uint(__builtin_amdgcn_rcpf(z));
      const uint32_t expect = (base[m] + (uint32_t)((127 - (int)e) * (1 << 23))) | (s << 31);
      n += r != expect;
    }
  if (n) atomicAdd(bad, n);
}

int main(int argc, char** argv) {
  uint32_t* d; unsigned long long* b;
  (void)hipMalloc(&d, (1u << 23) * 4);
  (void)hipMalloc(&b, 8);
  (void)hipMemset(b, 0, 8);
  dump<<<(1 << 23) / 256, 256>>>(d);
  check<<<(1 << 23) / 256, 256>>>(d, b);
  std::vector<uint32_t> h(1u << 23);
  unsigned long long bad = 0;
  (void)hipMemcpy(h.data(), d, (1u << 23) * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(&bad, b, 8, hipMemcpyDeviceToHost);
  printf("exponents 1..252, both signs: %llu results differ from the scaled exponent-127 table\n", bad);
  if (argc > 1) {
    FILE* f = fopen(argv[1], "wb");
    if (!f || fwrite(h.data(), 4, h.size(), f) != h.size()) { printf("write failed\n"); return 1; }
    fclose(f);
  }
  return bad != 0;
}
