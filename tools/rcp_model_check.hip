// Device side of tests/test_gpu_rcp.py::test_rcp_model_matches_oracle: the tap reciprocal the
// kernels use (device_math.h rcp_model / rcp_tap) over a fixed input set, written to a file that the
// test compares with the oracle's model (oracle_math.h o_rcp_tap) bit for bit.  Input set (the order
// the test regenerates): every mantissa at biased exponents 1, 127, 252, both signs; every 64th
// mantissa at exponents 0 (zero and denormals), 253, 254, 255 (inf / NaN), both signs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../dpe-mvs_amd/csrc/device_math.h"

__global__ void eval(const uint32_t* in, float* model, float* fast, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float z = __uint_as_float(in[i]);
  model[i] = dpe::rcp_model(z);
  fast[i] = dpe::rcp_tap<true>(z);
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  std::vector<uint32_t> in;
  for (uint32_t e : {1u, 127u, 252u})
    for (uint32_t s = 0; s < 2; ++s)
      for (uint32_t m = 0; m < (1u << 23); ++m) in.push_back((s << 31) | (e << 23) | m);
  for (uint32_t e : {0u, 253u, 254u, 255u})
    for (uint32_t s = 0; s < 2; ++s)
      for (uint32_t m = 0; m < (1u << 23); m += 64) in.push_back((s << 31) | (e << 23) | m);
  const long n = (long)in.size();
  uint32_t* din; float *dm, *df;
  if (hipMalloc(&din, n * 4) != hipSuccess || hipMalloc(&dm, n * 4) != hipSuccess || hipMalloc(&df, n * 4) != hipSuccess) return 1;
  (void)hipMemcpy(din, in.data(), n * 4, hipMemcpyHostToDevice);
  eval<<<(unsigned)((n + 255) / 256), 256>>>(din, dm, df, n);
  std::vector<float> m(n), f(n);
  if (hipMemcpy(m.data(), dm, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  if (hipMemcpy(f.data(), df, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  FILE* o = fopen(argv[1], "wb");
  if (!o || fwrite(m.data(), 4, n, o) != (size_t)n || fwrite(f.data(), 4, n, o) != (size_t)n) return 1;
  fclose(o);
  printf("%ld inputs\n", n);
  return 0;
}
