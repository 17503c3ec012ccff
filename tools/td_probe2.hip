// td_probe2.hip — gfx950 gather cost per wave load as a function of the number of distinct 128-B
// lines the 64 lanes touch, and of how those lines are spread over the lanes (diagnostic).
// Per-lane offsets come from a table in global memory (opaque to the compiler); each iteration
// moves the whole pattern by an opaque stride inside the workgroup's 16 KB region (L1-resident).
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/td_probe2 tools/td_probe2.hip ; run: /tmp/td_probe2
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
      const uint32_t o = (o0 + (uint32_t)(it * 8 + u) * sh) & (REGION - 1) & ~3u;
      if (BYTES == 4) acc += __uint_as_float(*(const uint32_t*)(base + o) & 0x3FFFFFFFu);
      else { typedef uint2 u2a __attribute__((aligned(4))); const uint2 v = *(const u2a*)(base + o); acc += __uint_as_float((v.x ^ v.y) & 0x3FFFFFFFu); }
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
  std::printf("%-44s %d B  %7.2f CU-cycles per wave load\n", name, BYTES, cyc / insts);
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
  for (int k : {1, 2, 4, 8, 16, 32, 64}) {
    std::vector<uint32_t> g(64), il(64);
    for (int l = 0; l < 64; ++l) {
      const int per = 64 / k;                                 // lanes per line
      g[l] = (uint32_t)((l / per) * 128 * 2 + (l % per) * 128 / (per > 16 ? 16 : per) % 128);   // contiguous lane groups, stride 2 lines
      il[l] = (uint32_t)((l % k) * 128 * 2 + ((l / k) * 8) % 128);                              // interleaved lanes
    }
    std::snprintf(name, sizeof name, "%2d lines, lane groups", k); run<8>(name, g, 128u * 2 * 64, buf, dofs, dsh, out, blocks);
    std::snprintf(name, sizeof name, "%2d lines, interleaved lanes", k); run<8>(name, il, 128u * 2 * 64, buf, dofs, dsh, out, blocks);
  }
  // 4-B aligned (unaligned for 8 B) offsets: the P16 tap pattern, 8 lines of 8 lanes, 4-B steps
  {
    std::vector<uint32_t> o(64);
    for (int l = 0; l < 64; ++l) o[l] = (uint32_t)((l / 8) * 256 + (l % 8) * 12 + 4);
    run<8>("8 lines x 8 lanes, 12-B steps, +4 misaligned", o, 128u * 2 * 64, buf, dofs, dsh, out, blocks);
    for (int l = 0; l < 64; ++l) o[l] = (uint32_t)((l / 8) * 256 + (l % 8) * 12);
    run<8>("8 lines x 8 lanes, 12-B steps", o, 128u * 2 * 64, buf, dofs, dsh, out, blocks);
    run<4>("8 lines x 8 lanes, 12-B steps", o, 128u * 2 * 64, buf, dofs, dsh, out, blocks);
    // a line straddle per lane: 8 B at offset 124 of a line
    for (int l = 0; l < 64; ++l) o[l] = (uint32_t)((l / 8) * 256 + 124);
    run<8>("8 lines, every load straddles two lines", o, 128u * 2 * 64, buf, dofs, dsh, out, blocks);
  }
  hipFree(buf); hipFree(out); hipFree(dofs); hipFree(dsh);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
