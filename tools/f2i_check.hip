// Checks that gfx950's v_cvt_i32_f32 equals dpe::f2i (device_math.h: saturating, NaN -> 0, and
// 2147483520.0f -> INT_MAX) except where f2i's explicit INT_MAX threshold differs, over special
// values and 2^24 random bit patterns.  Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/f2i_check tools/f2i_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
__device__ int f2i_ref(float f) {
  if (f != f) return 0;
  if (f >= 2147483520.0f) return 2147483647;
  if (f <= -2147483648.0f) return (int)0x80000000;
  return (int)f;
}
__device__ int f2i_hw(float f) {
  int r;
  asm volatile("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(f));
  return f == 2147483520.0f ? 2147483647 : r;
}
__global__ void k(const uint32_t* in, int n, int* bad, uint32_t* first) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float f = __uint_as_float(in[i]);
  if (f2i_ref(f) != f2i_hw(f)) { if (atomicAdd(bad, 1) == 0) *first = in[i]; }
}
int main() {
  std::vector<uint32_t> v;
  const float sp[] = {0.f, -0.f, 1.f, -1.f, 0.5f, -0.5f, 0.99999994f, -0.99999994f, 2147483520.f, -2147483520.f,
                      2147483648.f, -2147483648.f, 4294967296.f, -4294967296.f, 1e30f, -1e30f, 1e-45f, -1e-45f,
                      16777216.f, 8388607.5f};
  for (float f : sp) { uint32_t u; memcpy(&u, &f, 4); v.push_back(u); }
  const uint32_t specials[] = {0x7F800000u, 0xFF800000u, 0x7FC00000u, 0xFFC00000u, 0x7F800001u, 0x7FFFFFFFu};
  for (uint32_t u : specials) v.push_back(u);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < (1 << 24); ++i) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; v.push_back((uint32_t)s); }
  for (uint32_t e = 0; e < 256; ++e) for (uint32_t m = 0; m < 4096; ++m) v.push_back((e << 23) | (m << 11) | (m & 1 ? 0x80000000u : 0));
  uint32_t* d; int* bad; uint32_t* first;
  hipMalloc(&d, v.size() * 4); hipMalloc(&bad, 4); hipMalloc(&first, 4);
  hipMemcpy(d, v.data(), v.size() * 4, hipMemcpyHostToDevice); hipMemset(bad, 0, 4); hipMemset(first, 0, 4);
  k<<<(unsigned)((v.size() + 255) / 256), 256>>>(d, (int)v.size(), bad, first);
  int hb = -1; uint32_t hf = 0;
  hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost); hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
  printf("f2i_check: %zu inputs, %d mismatches%s", v.size(), hb, hb ? "" : "\n");
  if (hb) printf(" (first 0x%08x)\n", hf);
  return hb == 0 ? 0 : 1;
}
