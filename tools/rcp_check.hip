// Exhaustive check: is rcp + one FMA Newton step a correctly rounded 1/z (== IEEE 1.0f/z)?
// Counts mismatches over every float mantissa for a set of exponents.  Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/rcp_check.hip -o /tmp/rcp_check && /tmp/rcp_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float rcp_a(float z) {
  const float r = __builtin_amdgcn_rcpf(z);
  const float e = __builtin_fmaf(-z, r, 1.0f);
  return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ float rcp_b(float z) {
  const float r1 = rcp_a(z);
  const float e = __builtin_fmaf(-z, r1, 1.0f);
  return __builtin_fmaf(e, r1, r1);
}

__global__ void check(int exp_bias, unsigned sign, unsigned long long* bad) {   // bad[2]: raw v_rcp_f32 != 1/z
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= (1u << 23)) return;
  const uint32_t bits = sign | ((uint32_t)exp_bias << 23) | m;
  const float z = __uint_as_float(bits);
  const float ref = 1.0f / z;
  const float a = rcp_a(z), b = rcp_b(z);
  if (__float_as_uint(a) != __float_as_uint(ref)) atomicAdd(bad + 0, 1ull);
  if (__float_as_uint(b) != __float_as_uint(ref)) atomicAdd(bad + 1, 1ull);
  if (__float_as_uint(__builtin_amdgcn_rcpf(z)) != __float_as_uint(ref)) atomicAdd(bad + 2, 1ull);
}

int main() {
  unsigned long long* d;
  (void)hipMalloc(&d, 24);
  // every biased exponent 0..255, both signs: report the exponents where A differs from IEEE 1/z
  unsigned long long tot[2] = {0, 0}, in_range = 0;
  for (int e = 0; e < 256; ++e) for (unsigned s = 0; s < 2; ++s) {
    (void)hipMemset(d, 0, 24);
    check<<<(1 << 23) / 256, 256>>>(e, s << 31, d);
    unsigned long long h[3];
    (void)hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
    if (e == 127 && s == 0) printf("raw v_rcp_f32 != IEEE 1/z for %llu of 2^23 mantissas at exponent 127\n", h[2]);
    if (h[0] || h[1]) printf("exp %3d sign %u: mismatches A %llu  B %llu\n", e, s, h[0], h[1]);
    if (e >= 1 && e <= 252) in_range += h[0];
    tot[0] += h[0]; tot[1] += h[1];
  }
  printf("TOTAL A %llu B %llu; A mismatches with biased exponent in [1, 252]: %llu\n", tot[0], tot[1], in_range);
  return 0;
}
