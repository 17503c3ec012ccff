"""The FMA quotient of dpe-mvs_amd/csrc/exact_div.h (the geometric-consistency term's divisions,
DPE.cu:881-913) against IEEE float32 division: random operands over the admitted range (every
exponent pairing, uniformly random mantissas), mantissas next to powers of two and to all-ones
(the hard cases of reciprocal-based division), exact quotients, the 1600x1200 camera regime the
pass divides in, and the range gate (zero, subnormal, huge, infinite, NaN operands are refused and
go to the IEEE division).  The header is pure C++, compiled here with g++; x86 float division and
std::fma are correctly rounded, the same operations the device runs."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "dpe-mvs_amd", "csrc", "exact_div.h")

HARNESS = r"""
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cmath>
#include <random>
#include "%s"
using namespace dpe::xdiv;

static float from_bits(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
static uint32_t bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
static long bad = 0, checked = 0;
static void check(float a, float b) {
  if (!div_in_range(a) || !div_in_range(b)) return;
  const float yb = 1.0f / b;
  const float q = div_markstein(a, b, yb), e = a / b;
  ++checked;
  if (bits(q) != bits(e)) {
    if (bad < 10) std::printf("MISMATCH a=%%a b=%%a got %%a want %%a\n", a, b, q, e);
    ++bad;
  }
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? std::atol(argv[1]) : 20000000;
  std::mt19937_64 rng(20261017);
  // 1: random mantissas and signs, exponents over the whole admitted range
  for (long i = 0; i < n; ++i) {
    const uint64_t r = rng();
    const uint32_t ea = 67 + (uint32_t)(r %% 121), eb = 67 + (uint32_t)((r >> 8) %% 121);
    const uint32_t ma = (uint32_t)(r >> 16) & 0x7FFFFFu, mb = (uint32_t)(r >> 40) & 0x7FFFFFu;
    const float a = from_bits((uint32_t)((r >> 63) << 31) | (ea << 23) | ma);
    const float b = from_bits((uint32_t)(((r >> 62) & 1) << 31) | (eb << 23) | mb);
    check(a, b);
  }
  // 2: mantissas near 1.0 and near 2.0 (all-ones) for both operands
  for (uint32_t da = 0; da < 512; ++da)
    for (uint32_t db = 0; db < 512; ++db) {
      const uint32_t ma[2] = {da, 0x7FFFFFu - da}, mb[2] = {db, 0x7FFFFFu - db};
      for (int s = 0; s < 2; ++s)
        for (int t = 0; t < 2; ++t) {
          check(from_bits((127u << 23) | ma[s]), from_bits((127u << 23) | mb[t]));
          check(from_bits((140u << 23) | ma[s]), from_bits((121u << 23) | mb[t]));
        }
    }
  // 3: exact quotients a = b * k (k small integers and powers of two) and their neighbours
  for (long i = 0; i < n / 20; ++i) {
    const float b = from_bits((uint32_t)(100 + rng() %% 55) << 23 | ((uint32_t)rng() & 0x7FFFFFu));
    const float k = (float)(1 + rng() %% 4096);
    const float a = b * k;
    check(a, b);
    check(std::nextafter(a, 0.0f), b);
    check(std::nextafter(a, 1e30f), b);
  }
  // 4: the pass's regime: pixel offsets x depth over focal lengths, projections over depths
  for (long i = 0; i < n / 4; ++i) {
    std::uniform_real_distribution<float> px(-0.5f, 1600.5f), dep(0.3f, 1000.0f), fk(500.0f, 4000.0f);
    const float cx = px(rng), d = dep(rng), k0 = fk(rng);
    check(d * (px(rng) - cx), k0);
    check(k0 * px(rng) + 3.0f * d, d);
  }
  // 5: the gate
  const float refused[] = {0.0f, -0.0f, 0x1p-61f, 0x1p61f, INFINITY, -INFINITY, NAN, from_bits(1u), 0x1p-127f};
  for (float x : refused) if (div_in_range(x)) { std::printf("GATE admits %%a\n", x); return 1; }
  if (!div_in_range(0x1p-60f) || !div_in_range(-0x1p60f)) { std::printf("GATE refuses its ends\n"); return 1; }
  std::printf("checked %%ld bad %%ld\n", checked, bad);
  return bad == 0 ? 0 : 1;
}
"""


def test_markstein_quotient_is_ieee_division(tmp_path):
    src = tmp_path / "xdiv.cpp"
    src.write_text(HARNESS % HDR)
    exe = tmp_path / "xdiv"
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-o", str(exe), str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe), "20000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert int(r.stdout.split()[1]) > 25000000, r.stdout
