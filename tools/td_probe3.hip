// td_probe3.hip — gfx950 gather cost per wave load vs the load width (4 / 8 / 16 B per lane) at a
// fixed line pattern (diagnostic): does a wider load per tap cost the same texture-path cycles as
// an 8-B one (cost = lane-quad lines) or proportionally more (cost = bytes returned)?
// Per-lane offsets come from a table in global memory (opaque to the compiler); each iteration
// moves the pattern by an opaque stride inside the workgroup's 16 KB region (L1-resident).
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/td_probe3 tools/td_probe3.hip ; run: /tmp/td_probe3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int ITERS = 256, REGION = 16384;

template <int BYTES>
__global__ void __launch_bounds__(256) probe(const uint8_t* __restrict__ buf, const uint32_t* __restrict__ ofs,
                                             const uint32_t* __restrict__ shift_p, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const uint8_t* base = buf + (size_t)blockIdx.x * REGION;
  const uint32_t o0 = ofs[lane], sh = *shift_p;
  float acc = 0.0f;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      // aligned to the load width and inside the region: o + BYTES <= REGION
      const uint32_t o = (o0 + (uint32_t)(it * 8 + u) * sh) & (uint32_t)(REGION - 1) & ~(uint32_t)(BYTES - 1);
      if constexpr (BYTES == 4) {
        acc += __uint_as_float(*(const uint32_t*)(base + o) & 0x3FFFFFFFu);
      } else if constexpr (BYTES == 8) {
        const uint2 v = *(const uint2*)(base + o);
        acc += __uint_as_float((v.x ^ v.y) & 0x3FFFFFFFu);
      } else {
        const uint4 v = *(const uint4*)(base + o);
        acc += __uint_as_float((v.x ^ v.y ^ v.z ^ v.w) & 0x3FFFFFFFu);
      }
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

static int cus = 0; static double ghz = 0;
template <int BYTES>
void run(const char* name, const std::vector<uint32_t>& o, uint32_t shift, const uint8_t* buf, uint32_t* dofs, uint32_t* dsh, float* out, int blocks) {
  hipMemcpy(dofs, o.data(), 64 * 4, hipMemcpyHostToDevice);
  hipMemcpy(dsh, &shift, 4, hipMemcpyHostToDevice);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  probe<BYTES><<<blocks, 256>>>(buf, dofs, dsh, out);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) probe<BYTES><<<blocks, 256>>>(buf, dofs, dsh, out);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms = 0; hipEventElapsedTime(&ms, a, b);
  const double insts = 5.0 * blocks * 4 * ITERS * 8, cyc = ms * 1e-3 * ghz * 1e9 * cus;
  std::printf("%-48s %2d B  %7.2f CU-cycles per wave load\n", name, BYTES, cyc / insts);
  hipEventDestroy(a); hipEventDestroy(b);
}

int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  cus = p.multiProcessorCount; ghz = p.clockRate / 1e6;
  const int blocks = cus * 8;
  std::printf("%d CUs, %.2f GHz nominal\n", cus, ghz);
  uint8_t* buf; float* out; uint32_t *dofs, *dsh;
  hipMalloc(&buf, (size_t)blocks * REGION); hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipMalloc(&dofs, 256); hipMalloc(&dsh, 4);
  hipMemset(buf, 1, (size_t)blocks * REGION);
  char name[128];
  const uint32_t sh = 128u * 2 * 64;
  for (int k : {1, 4, 16, 64}) {
    // k lines; "quad-local": lane l on line (l / 4) % k, so a lane quad shares one line (16 quad-lines
    // whatever k); "interleaved": lane l on line l % k (min(k, 4) lines per quad)
    std::vector<uint32_t> q(64), il(64);
    for (int l = 0; l < 64; ++l) {
      q[l] = (uint32_t)(((l / 4) % k) * 256 + (l % 4) * 16);
      il[l] = (uint32_t)((l % k) * 256 + ((l / k) * 16) % 128);
    }
    std::snprintf(name, sizeof name, "%2d lines, quad shares a line", k);
    run<4>(name, q, sh, buf, dofs, dsh, out, blocks);
    run<8>(name, q, sh, buf, dofs, dsh, out, blocks);
    run<16>(name, q, sh, buf, dofs, dsh, out, blocks);
    std::snprintf(name, sizeof name, "%2d lines, interleaved lanes", k);
    run<4>(name, il, sh, buf, dofs, dsh, out, blocks);
    run<8>(name, il, sh, buf, dofs, dsh, out, blocks);
    run<16>(name, il, sh, buf, dofs, dsh, out, blocks);
  }
  hipFree(buf); hipFree(out); hipFree(dofs); hipFree(dsh);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
