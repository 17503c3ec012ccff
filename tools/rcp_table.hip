// Characterises v_rcp_f32 for a restatement that would use it without the Newton step (DESIGN §8
// "Next"): (1) is its result a function of the input mantissa alone, i.e. rcp(m * 2^k) ==
// rcp(m) * 2^-k bit for bit across exponents, for normal inputs and results; (2) how far is it from
// the correctly rounded 1/z (ulp histogram, direction).  Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/rcp_table.hip -o /tmp/rcp_table && /tmp/rcp_table
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

// out[0]: mantissas whose rcp at exponent e differs from the scaled rcp at exponent 127;
// out[1..5]: ulp difference of rcp(1.m) from IEEE 1/(1.m): -2, -1, 0, +1, +2 (out of range -> 0/6)
__global__ void check(int e, unsigned long long* out) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= (1u << 23)) return;
  const float z0 = __uint_as_float((127u << 23) | m);
  const float z = __uint_as_float(((uint32_t)e << 23) | m);
  const uint32_t r0 = __float_as_uint(__builtin_amdgcn_rcpf(z0));
  const uint32_t r = __float_as_uint(__builtin_amdgcn_rcpf(z));
  // scaling by 2^(127-e) moves the exponent field by (127 - e): same mantissa bits expected
  const uint32_t expect = r0 + (uint32_t)((127 - e) * (1 << 23));
  if (r != expect) atomicAdd(out + 0, 1ull);
  if (e == 127) {
    const int32_t d = (int32_t)r0 - (int32_t)__float_as_uint(1.0f / z0);
    const int k = d < -2 ? 0 : (d > 2 ? 6 : d + 3);
    atomicAdd(out + 1 + k, 1ull);
  }
}

int main() {
  unsigned long long* d;
  (void)hipMalloc(&d, 8 * sizeof(unsigned long long));
  const int exps[] = {1, 2, 64, 100, 126, 127, 128, 150, 200, 250, 252, 253};
  for (int e : exps) {
    (void)hipMemset(d, 0, 8 * sizeof(unsigned long long));
    check<<<(1 << 23) / 256, 256>>>(e, d);
    unsigned long long h[8];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("biased exponent %3d: %llu of 2^23 mantissas differ from the scaled exponent-127 result\n", e, h[0]);
    if (e == 127)
      printf("rcp(1.m) - RN(1/1.m) in ulps: <-2 %llu, -2 %llu, -1 %llu, 0 %llu, +1 %llu, +2 %llu, >+2 %llu\n", h[1], h[2], h[3], h[4],
             h[5], h[6], h[7]);
  }
  return 0;
}
