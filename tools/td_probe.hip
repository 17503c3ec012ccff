// td_probe.hip — vector-memory gather cost on gfx950 by access pattern (diagnostic microbenchmark).
// Every wave issues ITERS x 8 independent loads whose per-lane byte offsets follow one pattern
// inside its workgroup's private 16 KB region (L1-resident after the first touch).  Reported:
// CU-cycles per wave load instruction = elapsed * clock * CUs / (load instructions issued).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/td_probe tools/td_probe.hip ; run: tools/td_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITERS = 256, REGION = 16384;

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

template <int PAT, int BYTES>
__global__ void __launch_bounds__(256) probe(const uint8_t* __restrict__ buf, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const uint8_t* base = buf + (size_t)blockIdx.x * REGION;
  float acc = 0.0f;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t k = (uint32_t)(it * 8 + u);
      uint32_t o;
      if (PAT == 0) o = (k * 64u) % REGION;                                   // all lanes one address
      else if (PAT == 1) o = (lane * BYTES + k * 1024u) % REGION;              // consecutive lanes
      else if (PAT == 2) o = (lane * 64u + k * 256u) % REGION;                 // 64-B stride
      else if (PAT == 3) o = (lane * 128u + k * 512u) % REGION;                // one 128-B line per lane
      else if (PAT == 4) o = hash32(lane * 977u + k * 131u + threadIdx.x) % (REGION / BYTES) * BYTES;   // random
      else if (PAT == 5) o = ((lane >> 1) * BYTES + k * 1024u) % REGION;       // lane pairs share a texel
      else o = ((lane & 15) * BYTES + (lane >> 4) * 1024u + k * 64u) % REGION; // 4 rows of 16 consecutive
      o &= ~(uint32_t)(BYTES - 1);
      if (BYTES == 4) acc += __uint_as_float(*(const uint32_t*)(base + o) & 0x3FFFFFFFu);
      else if (BYTES == 8) { const uint2 v = *(const uint2*)(base + o); acc += __uint_as_float((v.x ^ v.y) & 0x3FFFFFFFu); }
      else { const uint4 v = *(const uint4*)(base + o); acc += __uint_as_float((v.x ^ v.y ^ v.z ^ v.w) & 0x3FFFFFFFu); }
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// the same patterns served from LDS (the region copied in first)
template <int PAT, int BYTES>
__global__ void __launch_bounds__(256) probe_lds(const uint8_t* __restrict__ buf, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[REGION];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < REGION / 16; i += 256) ((uint4*)lds)[i] = ((const uint4*)(buf + (size_t)blockIdx.x * REGION))[i];
  __syncthreads();
  float acc = 0.0f;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t k = (uint32_t)(it * 8 + u);
      uint32_t o;
      if (PAT == 1) o = (lane * BYTES + k * 1024u) % REGION;
      else if (PAT == 4) o = hash32(lane * 977u + k * 131u + threadIdx.x) % (REGION / BYTES) * BYTES;
      else o = ((lane & 15) * BYTES + (lane >> 4) * 1024u + k * 64u) % REGION;
      o &= ~(uint32_t)(BYTES - 1);
      if (BYTES == 4) acc += __uint_as_float(*(const uint32_t*)(lds + o) & 0x3FFFFFFFu);
      else { const uint2 v = *(const uint2*)(lds + o); acc += __uint_as_float((v.x ^ v.y) & 0x3FFFFFFFu); }
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int PAT, int BYTES, bool LDS = false>
void run(const char* name, const uint8_t* buf, float* out, int blocks, double ghz, int cus) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  auto k = LDS ? probe_lds<PAT, BYTES> : probe<PAT, BYTES>;
  k<<<blocks, 256>>>(buf, out);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) k<<<blocks, 256>>>(buf, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double insts = 5.0 * blocks * 4 * ITERS * 8;      // wave load instructions
  const double cyc = ms * 1e-3 * ghz * 1e9 * cus;
  std::printf("%-4s %-34s %2d B  %8.3f ms  %6.2f CU-cycles per wave load (%.2f per lane)\n", LDS ? "LDS" : "HBM", name, BYTES, ms / 5, cyc / insts,
              cyc / insts / 64);
  hipEventDestroy(a); hipEventDestroy(b);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const double ghz = p.clockRate / 1e6;
  const int blocks = cus * 8;                   // 8 workgroups x 4 waves = 32 waves per CU
  std::printf("%s: %d CUs, clock %.2f GHz (nominal; the chip may run lower)\n", p.name, cus, ghz);
  uint8_t* buf; float* out;
  if (hipMalloc(&buf, (size_t)blocks * REGION) != hipSuccess || hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
  hipMemset(buf, 1, (size_t)blocks * REGION);
  run<0, 8>("uniform (all lanes one address)", buf, out, blocks, ghz, cus);
  run<1, 4>("consecutive lanes", buf, out, blocks, ghz, cus);
  run<1, 8>("consecutive lanes", buf, out, blocks, ghz, cus);
  run<1, 16>("consecutive lanes", buf, out, blocks, ghz, cus);
  run<5, 8>("lane pairs share a texel", buf, out, blocks, ghz, cus);
  run<6, 8>("4 rows x 16 consecutive", buf, out, blocks, ghz, cus);
  run<2, 8>("64-B stride", buf, out, blocks, ghz, cus);
  run<3, 8>("128-B stride (line per lane)", buf, out, blocks, ghz, cus);
  run<3, 4>("128-B stride (line per lane)", buf, out, blocks, ghz, cus);
  run<4, 4>("random in 16 KB", buf, out, blocks, ghz, cus);
  run<4, 8>("random in 16 KB", buf, out, blocks, ghz, cus);
  run<4, 16>("random in 16 KB", buf, out, blocks, ghz, cus);
  run<1, 8, true>("consecutive lanes", buf, out, blocks, ghz, cus);
  run<6, 8, true>("4 rows x 16 consecutive", buf, out, blocks, ghz, cus);
  run<4, 8, true>("random in 16 KB", buf, out, blocks, ghz, cus);
  run<4, 4, true>("random in 16 KB", buf, out, blocks, ghz, cus);
  hipFree(buf); hipFree(out);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
