// device_math.h — gfx950 arithmetic primitives of the PatchMatch pass.
//
// Every primitive is a fixed sequence of IEEE-754 operations (compiled with -ffp-contract=off,
// all FMAs explicit) so that the pass is bit-reproducible: the same inputs and Philox seed give
// the same bits on any MI355X, and the CPU restatement in oracle/ reproduces them.
// Reference semantics restated (csrc/DPE-MVS/DPE.cu, compiled --use_fast_math there):
//   expf/__expf (:554,:1576,:1587) -> d_expf      sin/cos (:397-402)  -> d_sincosf
//   exp(double) (:2554)            -> d_exp_d     rsqrtf (:271,:288)  -> 1/sqrtf
//   curand / curand_uniform        -> Philox4x32-10 counter streams (no per-pixel state buffer)
//   tex2D linear filter            -> sample_quad() on the padded quad-texel image layout
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __device__ __forceinline__

namespace dpe {

DEV float pow2i(int k) { return __uint_as_float((uint32_t)(k + 127) << 23); }
DEV double pow2i_d(int k) { return __longlong_as_double((long long)((uint64_t)(k + 1023) << 52)); }

DEV float d_expf(float x) {
  if (x != x) return x;
  if (x > 88.7228394f) return __builtin_inff();
  if (x < -103.972084f) return 0.0f;
  float k = __builtin_rintf(x * 1.44269502f);
  float r = __builtin_fmaf(k, -0.693145752f, x);
  r = __builtin_fmaf(k, -1.42860677e-06f, r);
  float p = 1.98412698e-4f;
  p = __builtin_fmaf(p, r, 1.38888889e-3f);
  p = __builtin_fmaf(p, r, 8.33333377e-3f);
  p = __builtin_fmaf(p, r, 4.16666679e-2f);
  p = __builtin_fmaf(p, r, 1.66666672e-1f);
  p = __builtin_fmaf(p, r, 0.5f);
  p = __builtin_fmaf(p, r, 1.0f);
  p = __builtin_fmaf(p, r, 1.0f);
  int ki = (int)k;
  if (ki < -125) { p = p * 5.42101086e-20f; ki += 64; }
  if (ki > 127) { p = p * 2.0f; ki -= 1; }
  return p * pow2i(ki);
}

DEV void d_sincosf(float x, float* s, float* c) {
  float k = __builtin_rintf(x * 0.636619747f);
  float r = __builtin_fmaf(k, -1.5703125f, x);
  r = __builtin_fmaf(k, -4.83751297e-04f, r);
  r = __builtin_fmaf(k, -7.54978995e-08f, r);
  float r2 = r * r;
  float ps = -1.98412698e-4f;
  ps = __builtin_fmaf(ps, r2, 8.33333377e-3f);
  ps = __builtin_fmaf(ps, r2, -1.66666672e-1f);
  ps = ps * r2;
  float sr = __builtin_fmaf(ps, r, r);
  float pc = 2.48015876e-5f;
  pc = __builtin_fmaf(pc, r2, -1.38888892e-3f);
  pc = __builtin_fmaf(pc, r2, 4.16666679e-2f);
  pc = __builtin_fmaf(pc, r2, -0.5f);
  float cr = __builtin_fmaf(pc, r2, 1.0f);
  int q = ((int)k) & 3;
  float so, co;
  if (q == 0) { so = sr; co = cr; }
  else if (q == 1) { so = cr; co = -sr; }
  else if (q == 2) { so = -sr; co = -cr; }
  else { so = -cr; co = sr; }
  *s = so; *c = co;
}

DEV double d_exp_d(double x) {
  if (x != x) return x;
  if (x > 709.0) return __builtin_inf();
  if (x < -708.0) return 0.0;
  double k = __builtin_rint(x * 1.4426950408889634);
  double r = __builtin_fma(k, -6.93147180369123816490e-01, x);
  r = __builtin_fma(k, -1.90821492927058770002e-10, r);
  double p = 1.0 / 479001600.0;
  p = __builtin_fma(p, r, 1.0 / 39916800.0);
  p = __builtin_fma(p, r, 1.0 / 3628800.0);
  p = __builtin_fma(p, r, 1.0 / 362880.0);
  p = __builtin_fma(p, r, 1.0 / 40320.0);
  p = __builtin_fma(p, r, 1.0 / 5040.0);
  p = __builtin_fma(p, r, 1.0 / 720.0);
  p = __builtin_fma(p, r, 1.0 / 120.0);
  p = __builtin_fma(p, r, 1.0 / 24.0);
  p = __builtin_fma(p, r, 1.0 / 6.0);
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  p = __builtin_fma(p, r, 1.0);
  return p * pow2i_d((int)k);
}

// Correctly rounded 1/z (== IEEE 1.0f / z, bit for bit) in 3 VALU ops instead of the ~10-op
// div_scale/div_fmas/div_fixup sequence: v_rcp_f32 + one FMA Newton step.  Verified exhaustively on
// gfx950 for every float whose biased exponent is in [1, 252], both signs (tools/rcp_check.hip,
// tests/test_gpu_rcp.py).  Callers must guarantee that range (see rcp_range_ok); outside it (zero,
// denormals, |z| >= 2^126, inf, NaN) only the IEEE division is exact.
DEV float d_rcp_fast(float z) {
  const float r = __builtin_amdgcn_rcpf(z);
  return __builtin_fmaf(__builtin_fmaf(-z, r, 1.0f), r, r);
}
// The tap reciprocal (restatement choice 8): the hardware's v_rcp_f32 for every
// denominator whose biased exponent is in [1, 252] (results normal; the result is a function of
// the mantissa alone there, within 1 ulp of 1/z, and the oracle carries its table), IEEE 1.0f / z
// otherwise (zero, denormals, |z| >= 2^126, inf, NaN).  The reference divides under
// --use_fast_math (CMakeLists.txt:72), itself an approximate reciprocal (DPE.cu:515-522).
// FAST: the caller has checked the range for the whole patch (rcp_range_ok), so no per-tap test.
DEV float rcp_model(float z) {
  const uint32_t e = (__float_as_uint(z) >> 23) & 0xFFu;
  float r = __builtin_amdgcn_rcpf(z);
  if (__builtin_expect(e - 1u >= 252u, 0)) r = 1.0f / z;   // rare: a branch, not a select
  return r;
}
template <bool FAST> DEV float rcp_tap(float z) {
  if constexpr (FAST) return __builtin_amdgcn_rcpf(z);
  else return rcp_model(z);
}
DEV float d_rsqrtf(float x) { return 1.0f / __builtin_sqrtf(x); }

// float -> int with cvt.rzi.s32 semantics (saturating, NaN -> 0): written explicitly so the
// CPU restatement matches.
DEV int f2i(float f) {
  if (f != f) return 0;
  if (f >= 2147483520.0f) return 2147483647;
  if (f <= -2147483648.0f) return (int)0x80000000;
  return (int)f;
}
DEV int d2i(double f) {
  if (f != f) return 0;
  if (f >= 2147483647.0) return 2147483647;
  if (f <= -2147483648.0) return (int)0x80000000;
  return (int)f;
}

// OpenCV cvdef.h MIN / MAX as used throughout DPE.cu
template <class A, class B> DEV auto MINo(A a, B b) -> decltype(a + b) { return (a > b) ? b : a; }
template <class A, class B> DEV auto MAXo(A a, B b) -> decltype(a + b) { return (a < b) ? b : a; }

// ------------------------------------------------------------------------------ Philox4x32-10
struct Rng {
  uint32_t k0, k1, stream, salt, ctr;
  uint32_t b0, b1, b2, b3;
  int idx;
};

DEV void philox10(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // each round's two 32x32 products as one 64-bit product (v_mad_u64_u32) each
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    const uint32_t n0 = hi1 ^ c1 ^ k0;
    const uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

DEV void rng_init(Rng& s, uint32_t pixel, uint32_t seed32, uint32_t stream, uint32_t salt) {
  s.k0 = pixel; s.k1 = seed32; s.stream = stream; s.salt = salt; s.ctr = 0; s.idx = 4;
  s.b0 = s.b1 = s.b2 = s.b3 = 0;
}
DEV uint32_t rng_u32(Rng& s) {
  if (s.idx == 4) {
    uint32_t c0 = s.ctr, c1 = s.stream, c2 = s.salt, c3 = 0u;
    philox10(c0, c1, c2, c3, s.k0, s.k1);
    s.b0 = c0; s.b1 = c1; s.b2 = c2; s.b3 = c3;
    s.ctr++; s.idx = 0;
  }
  const int i = s.idx++;
  return i == 0 ? s.b0 : (i == 1 ? s.b1 : (i == 2 ? s.b2 : s.b3));
}
DEV float u32_to_uniform(uint32_t u) { return (float)u * 2.32830644e-10f + 1.16415322e-10f; }
DEV float rng_uniform(Rng& s) { return u32_to_uniform(rng_u32(s)); }
// word n of the stream (draws are position-addressable: word n = word n%4 of Philox block n/4)
DEV uint32_t rng_word(const Rng& s, uint32_t n) {
  uint32_t c0 = n >> 2, c1 = s.stream, c2 = s.salt, c3 = 0u;
  philox10(c0, c1, c2, c3, s.k0, s.k1);
  const uint32_t i = n & 3u;
  return i == 0 ? c0 : (i == 1 ? c1 : (i == 2 ? c2 : c3));
}
// position the stream so that the next draw is word n
DEV void rng_seek(Rng& s, uint32_t n) {
  s.ctr = n >> 2; s.idx = 4;
  if (n & 3u) { (void)rng_u32(s); s.idx = (int)(n & 3u); }
}

enum { STREAM_GEN_NEIGHBOURS = 1, STREAM_RANDOM_INIT = 2, STREAM_ITER_BASE = 16 };

}  // namespace dpe
