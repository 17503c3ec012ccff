// exact_div.h — the correctly rounded f32 quotient a / b from a reciprocal yb = RN(1/b), in 5 FMA-unit
// operations instead of the 11 of the IEEE division sequence (v_div_scale x2, v_rcp, 5 FMAs,
// v_div_fmas, v_div_fixup).  Used by the geometric-consistency term (project / back-project,
// DPE.cu:881-913), whose divisions are by per-camera constants (K[0], K[4]: yb from the host) or by
// one per-lane denominator shared by two quotients (yb from the exact 3-op reciprocal).
//
// q0 = RN(a yb) is within ~2 ulps of a/b; one correction q1 = RN(q0 + RN(a - b q0) yb) is faithful
// (error <= 1/2 ulp + O(2^-46) relative); then Markstein's theorem (yb within 1/2 ulp of 1/b, q1
// within 1 ulp of a/b => the FMA remainder r1 = a - b q1 is exact and RN(q1 + r1 yb) = RN(a/b)) gives
// the IEEE quotient.  The theorem needs no underflow or overflow anywhere: div_in_range() admits
// |a| and |b| in [2^-60, 2^60] (so the quotient, the remainders and yb are far from both ends); zero,
// subnormal, huge, infinite and NaN operands go to the IEEE division (zero for its sign: -0 / b).
// Pure C++ (no HIP types): tests/test_exact_div.py checks it against IEEE division with g++.
#pragma once

#if defined(__HIPCC__)
#define XD_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#define XD_HD inline
#endif

namespace dpe {
namespace xdiv {

XD_HD float fma_(float a, float b, float c) {
#if defined(__HIPCC__)
  return __builtin_fmaf(a, b, c);
#else
  return std::fma(a, b, c);
#endif
}
XD_HD float fabs_(float a) { return a < 0.0f ? -a : a; }

// |x| in [2^-60, 2^60]; false for 0, NaN and infinities
XD_HD bool div_in_range(float x) {
  const float m = fabs_(x);
  return m >= 0x1p-60f && m <= 0x1p60f;
}

// RN(a / b) for a, b in range, yb = RN(1 / b)
XD_HD float div_markstein(float a, float b, float yb) {
  const float q0 = a * yb;
  const float r0 = fma_(-q0, b, a);
  const float q1 = fma_(r0, yb, q0);
  const float r1 = fma_(-q1, b, a);
  return fma_(r1, yb, q1);
}

}  // namespace xdiv
}  // namespace dpe
