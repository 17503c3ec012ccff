/* Exhaustive check of GenNeighbours' multiply-modulo (csrc/pass_kernels.h gn_mod, the constant from
 * dpe_mvs.hip compute_pass_constants): x % d for every 32-bit x and d = 1..8.  "old" is the first
 * version (x * ceil(2^35 / d) >> 35), whose 64-bit product overflows -- out-of-range residues, the
 * cause of the round-4 call-G memory fault in the direction-table build; "new" must report 0.
 * gcc -O2 -fopenmp -o /tmp/check_gn_mod tools/check_gn_mod.c && /tmp/check_gn_mod   (~20 s, 8 threads) */
#include <stdio.h>
#include <stdint.h>
#include <math.h>
int main(void) {
  for (uint32_t d = 1; d <= 8; ++d) {
    uint64_t m = ((1ull << 35) + d - 1) / d;
    uint64_t bad_old = 0, bad_new = 0;
    uint32_t M = d == 1 ? 0xFFFFFFFFu : (uint32_t)((1ull << 32) / d);
    #pragma omp parallel for reduction(+:bad_old,bad_new)
    for (int64_t xi = 0; xi < (1ll << 32); ++xi) {
      uint32_t x = (uint32_t)xi;
      uint32_t q = (uint32_t)(((uint64_t)x * m) >> 35);
      uint32_t r = x - q * d;
      if (r != x % d) bad_old++;
      uint32_t q2 = (uint32_t)(((uint64_t)x * M) >> 32);
      uint32_t r2 = x - q2 * d;
      r2 = r2 >= d ? r2 - d : r2;
      if (r2 != x % d) bad_new++;
    }
    printf("d=%u old_bad=%llu new_bad=%llu\n", d, (unsigned long long)bad_old, (unsigned long long)bad_new);
  }
  return 0;
}
