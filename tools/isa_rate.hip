// Issue-rate microbenchmark for the VALU instructions of the bilinear tap (gfx950).
// Each kernel runs 8 independent chains of one instruction per lane, 256-thread blocks, enough
// blocks for 4 waves per SIMD on every CU; reports shader cycles per wave-instruction per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/isa_rate tools/isa_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP 256
#define CHAINS 8

#define KERNEL(name, body)                                                           \
  __global__ void __launch_bounds__(256) name(float* out, float seed) {              \
    float a[CHAINS];                                                                 \
    for (int i = 0; i < CHAINS; ++i) a[i] = seed + threadIdx.x + i;                  \
    float b = seed * 0.5f, c = seed * 0.25f;                                         \
    for (int r = 0; r < REP; ++r) {                                                  \
      _Pragma("unroll") for (int i = 0; i < CHAINS; ++i) { body; }                  \
    }                                                                                \
    float s = 0;                                                                     \
    for (int i = 0; i < CHAINS; ++i) s += a[i];                                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                  \
  }

KERNEL(k_fma, asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c)))
KERNEL(k_mul, asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
KERNEL(k_add, asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
KERNEL(k_med3, asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c)))
KERNEL(k_cvt_i32, asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(a[i])))
KERNEL(k_cvt_ubyte, asm volatile("v_cvt_f32_ubyte0 %0, %0" : "+v"(a[i])))
KERNEL(k_lshr, asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(a[i])))
KERNEL(k_mad24, asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c)))
KERNEL(k_lshl_add, asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(a[i]) : "v"(b)))
KERNEL(k_fma_mix, asm volatile("v_fma_mix_f32 %0, %0, %1, %2 op_sel_hi:[0,1,1]" : "+v"(a[i]) : "v"(b), "v"(c)))
KERNEL(k_rcp, asm volatile("v_rcp_f32 %0, %0" : "+v"(a[i])))
KERNEL(k_and, asm volatile("v_and_b32 %0, 0xff, %0" : "+v"(a[i])))
KERNEL(k_cndmask, asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b)))
KERNEL(k_mul_hi, asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
KERNEL(k_mul_lo, asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
KERNEL(k_mul_u24, asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
KERNEL(k_xor, asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
// 32 x 32 -> 64-bit product (both halves of a Philox round's product in one instruction)
__global__ void __launch_bounds__(256) k_mad64(float* out, float seed) {
  unsigned long long a[CHAINS];
  for (int i = 0; i < CHAINS; ++i) a[i] = (unsigned long long)(seed + threadIdx.x + i);
  const unsigned b = (unsigned)seed | 1u;
  for (int r = 0; r < REP; ++r) {
#pragma unroll
    for (int i = 0; i < CHAINS; ++i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"((unsigned)a[i]), "v"(b) : "vcc");
  }
  unsigned long long s = 0;
  for (int i = 0; i < CHAINS; ++i) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (float)s;
}
KERNEL(k_xad, asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c)))
KERNEL(k_sqrt, asm volatile("v_sqrt_f32 %0, %0" : "+v"(a[i])))
KERNEL(k_cvt_u32, asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(a[i])))
KERNEL(k_min_u32, asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))

typedef float f2 __attribute__((ext_vector_type(2)));
#define KERNEL2(name, body)                                                          \
  __global__ void __launch_bounds__(256) name(float* out, float seed) {              \
    f2 a[CHAINS];                                                                    \
    for (int i = 0; i < CHAINS; ++i) a[i] = (f2){seed + threadIdx.x + i, seed - i};  \
    f2 b = (f2){seed * 0.5f, seed}, c = (f2){seed * 0.25f, seed};                    \
    for (int r = 0; r < REP; ++r) {                                                  \
      _Pragma("unroll") for (int i = 0; i < CHAINS; ++i) { body; }                  \
    }                                                                                \
    float s = 0;                                                                     \
    for (int i = 0; i < CHAINS; ++i) s += a[i].x + a[i].y;                           \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                  \
  }
KERNEL2(k_pk_fma, asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c)))
KERNEL2(k_pk_mul, asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
KERNEL2(k_pk_add, asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))

typedef void (*kfn)(float*, float);
int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 4 * 4;          // 16 waves per CU = 4 per SIMD
  float* out;
  hipMalloc(&out, sizeof(float) * blocks * 256);
  struct { const char* name; kfn f; } ks[] = {
      {"v_fma_f32", k_fma}, {"v_mul_f32", k_mul}, {"v_add_f32", k_add}, {"v_med3_f32", k_med3},
      {"v_cvt_i32_f32", k_cvt_i32}, {"v_cvt_f32_ubyte0", k_cvt_ubyte}, {"v_lshrrev_b32", k_lshr},
      {"v_mad_u32_u24", k_mad24}, {"v_lshl_add_u32", k_lshl_add}, {"v_fma_mix_f32", k_fma_mix},
      {"v_rcp_f32", k_rcp}, {"v_and_b32", k_and}, {"v_cndmask_b32", k_cndmask},
      {"v_mul_hi_u32", k_mul_hi}, {"v_mul_lo_u32", k_mul_lo}, {"v_mul_u32_u24", k_mul_u24}, {"v_xor_b32", k_xor}, {"v_mad_u64_u32", k_mad64},
      {"v_xad_u32", k_xad}, {"v_sqrt_f32", k_sqrt}, {"v_cvt_u32_f32", k_cvt_u32}, {"v_min_u32", k_min_u32},
      {"v_pk_fma_f32", k_pk_fma}, {"v_pk_mul_f32", k_pk_mul}, {"v_pk_add_f32", k_pk_add}};
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  int clk_khz = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  printf("CUs %d, clock %d MHz (nominal), %d blocks of 256\n", cus, clk_khz / 1000, blocks);
  for (auto& k : ks) {
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1.0f);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    const int iters = 20;
    for (int it = 0; it < iters; ++it) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double waves_per_simd = (double)blocks * 4 / (cus * 4);
    const double instr_per_simd = waves_per_simd * REP * CHAINS * iters;
    const double cycles = ms * 1e-3 * 2.4e9;
    printf("%-20s %.2f cycles per wave-instruction per SIMD (at 2.4 GHz)\n", k.name, cycles / instr_per_simd);
  }
  hipFree(out);
  return 0;
}
