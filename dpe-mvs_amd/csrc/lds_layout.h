// lds_layout.h — compile-time layouts of the sweeps' LDS carves (the per-thread cost_array[8][32]
// and patch registers of the reference, DPE.cu:1236, 1690, become per-wave / per-pixel LDS blocks).
//
// Every region is (offset, length, alignment) in floats.  regions_ok() checks at compile time that
// each region lies inside its block, is aligned, and overlaps no other region; the carves depend on
// the source-view count nv only through closed forms, so the checks run for every nv the ABI allows
// (1..DPE_MAX_IMAGES-1).  Pure C++ (no HIP types): tests/test_lds_layout.py compiles it with g++, and
// shows that an overlapping layout does not compile.
#pragma once

#if defined(__HIPCC__)
#define LDS_HD __host__ __device__
#else
#define LDS_HD
#endif

namespace dpe {
namespace lds {

constexpr int kMaxViews = 31;   // DPE_MAX_IMAGES - 1 source views

struct Region {
  int off, len, align;
};

template <int N>
constexpr bool regions_ok(const Region (&r)[N], int total) {
  for (int i = 0; i < N; ++i) {
    if (r[i].len < 0 || r[i].off < 0 || r[i].off + r[i].len > total) return false;
    if (r[i].align > 1 && r[i].off % r[i].align != 0) return false;
    for (int j = i + 1; j < N; ++j)
      if (r[i].len > 0 && r[j].len > 0 && r[i].off < r[j].off + r[j].len && r[j].off < r[i].off + r[i].len) return false;
  }
  return true;
}

// ------------------------------------------------------------------ strong sweep (k_strong_coop)
// Per wave: P pixels x C candidate lanes.  Arrays indexed [pixel] are read across pixels by the
// wave's job pools.
template <int P, int C, int TAIL_JOBS>
struct StrongCarve {
  static constexpr int kPatch = 108;                                          // patch_lds_build: [36][2] + [36]
  LDS_HD static constexpr int ib_ints(int nv) { return 2 * C + 17 + nv; }     // per pixel, see IB_* below
  LDS_HD static constexpr int hyp() { return 0; }                             // [P][5] float4 refinement hypotheses
  LDS_HD static constexpr int patch() { return P * 20; }                      // [P][108]
  LDS_HD static constexpr int cost(int) { return P * 128; }                   // [P][C + 1][nv] cost vectors (slot C = current)
  LDS_HD static constexpr int sp(int nv) { return P * (128 + (C + 1) * nv); } // [P][nv] view probabilities
  LDS_HD static constexpr int ref(int nv) { return P * (128 + (C + 2) * nv); }   // [P][5][nv] refinement NCCs (+ sampling counts)
  LDS_HD static constexpr int fc(int nv) { return P * (128 + (C + 7) * nv); }    // [P][8] final costs
  LDS_HD static constexpr int sums(int nv) { return P * (136 + (C + 7) * nv); }  // [P][4] s_ref, s_rr, s_w, wnorm
  LDS_HD static constexpr int vw(int nv) { return P * (140 + (C + 7) * nv); }    // [P][32] u8 view weights
  LDS_HD static constexpr int ib(int nv) { return P * (148 + (C + 7) * nv); }    // [P][ib_ints] ints
  LDS_HD static constexpr int base(int nv) { return (ib(nv) + P * ib_ints(nv) + 3) & ~3; }
  LDS_HD static constexpr int cpl(int nv) { return base(nv); }                // [P][C + 1] float4 candidate planes
  LDS_HD static constexpr int alias(int nv) { return base(nv) + P * (C + 1) * 4; }   // [P][C + 1] ints
  LDS_HD static constexpr int tail(int nv) { return alias(nv) + P * (C + 1); }       // [TAIL_JOBS][6][3] row sums
  LDS_HD static constexpr int rnd(int nv) { return tail(nv) + TAIL_JOBS * 18; }      // [P][12] refinement draws
  LDS_HD static constexpr int total(int nv) { return rnd(nv) + P * 12; }
  // ints of a pixel's ib block
  static constexpr int IB_POS = 0;            // [C] candidate positions (-1 = none)
  static constexpr int IB_FIN = C;            // [8] final slot of direction d
  static constexpr int IB_MISC = C + 8;       // [8] 0: nsel, 1: cost-vector jobs, 2..6: hypothesis depths
  static constexpr int IB_SEL = C + 16;       // [nv] selected views
  LDS_HD static constexpr int ib_slots(int nv) { return C + 16 + nv; }   // [C + 1] cost-vector job slots
  static constexpr int MI_NSEL = 0, MI_JOBS = 1, MI_DEPTH = 2;          // IB_MISC ints (MI_DEPTH + 0..4)

  static constexpr bool ok(int nv) {
    const Region r[] = {{hyp(), P * 20, 4},        {patch(), P * kPatch, 1}, {cost(nv), P * (C + 1) * nv, 1},
                        {sp(nv), P * nv, 1},       {ref(nv), P * 5 * nv, 1}, {fc(nv), P * 8, 1},
                        {sums(nv), P * 4, 1},      {vw(nv), P * 8, 1},       {ib(nv), P * ib_ints(nv), 1},
                        {cpl(nv), P * (C + 1) * 4, 4}, {alias(nv), P * (C + 1), 1}, {tail(nv), TAIL_JOBS * 18, 1},
                        {rnd(nv), P * 12, 1}};
    // the sampling counts (view_sample_coop) reuse a pixel's ref block as nv ints; the ib block's
    // sub-arrays must fit its ints
    return regions_ok(r, total(nv)) && ib_slots(nv) + C + 1 == ib_ints(nv) && P * C == 64 && MI_DEPTH + 5 <= 8;
  }
  static constexpr bool ok_all() {
    for (int nv = 1; nv <= kMaxViews; ++nv) if (!ok(nv)) return false;
    return true;
  }
};

// ------------------------------------------------------------------ weak sweep (k_weak_coop)
// Per pixel, a fixed part (tables, planes, header) and an nv-dependent tail.  The header the pooled
// phases read from other pixels' blocks has named slots.  PRE: the layout of the DPE_WEAK_PRE build,
// whose refinement draws (12 floats, RND) reuse the alias rows once the cost vectors are shared
// (ALIAS is dead from phase 3 on) plus 4 more floats; ALIAS and VWL trade places so that the 12
// floats are contiguous.
template <bool PRE>
struct WeakCarveT {
  static constexpr int PW = 0;          // [108] Old-NCC patch (patch_lds_build)
  static constexpr int TC = 108;        // centre patch table, (w, w*grey) pairs [36][2]
  static constexpr int TN = 180;        // neighbour patch tables, pairs [8][9][2]
  static constexpr int SUMS = 324;      // [9][3] ncc_pre of each tabulated patch
  static constexpr int RC = 351;        // grey level of the pixel (header)
  static constexpr int OSUM = 352;      // [3] Old-NCC patch sums
  static constexpr int CPL = 356;       // [8] float4 candidate planes
  static constexpr int HYP = 388;       // [7] float4 refinement hypotheses; [5] final plane, [6] fit plane
  static constexpr int RSUM = HYP;      // phases 1-1b: [6][3] row sums of the centre patch (over HYP)
  static constexpr int FC = 416;        // [8] final candidate costs
  static constexpr int MISC = 424;      // [16] ints, slots M_* below
  static constexpr int NBL = 440;       // [9] short2 neighbour pixels
  static constexpr int NBOX_A = 449;    // nbox[0..2] (header)
  static constexpr int NSV = 452;       // [9] u32 selected views of the neighbours
  static constexpr int NBOX_B = 461;    // nbox[3] (header)
  static constexpr int ALIAS = PRE ? 472 : 464;   // [8] ints (phases 1b-3)
  static constexpr int VWL = PRE ? 464 : 472;     // [32] u8 view weights
  static constexpr int RND = 472;       // PRE: [12] refinement draws (phase 7), over ALIAS and 4 more floats
  static constexpr int FIXED = PRE ? 484 : 480;
  // misc ints
  static constexpr int M_NSEL = 0, M_RADC = 1, M_INCC = 2, M_NC = 3, M_WNORM = 4, M_CMASK = 5, M_NB3 = 6, M_POOL = 7, M_FLAGS = 8;
  // nv-dependent tail
  LDS_HD static constexpr int cost(int) { return FIXED; }                 // [8][nv]
  LDS_HD static constexpr int sp(int nv) { return FIXED + 8 * nv; }       // [nv]
  LDS_HD static constexpr int sel(int nv) { return FIXED + 9 * nv; }      // [nv] ints
  LDS_HD static constexpr int hv(int nv) { return FIXED + 10 * nv; }      // [7][nv]
  LDS_HD static constexpr int per_pixel(int nv) { return (FIXED + 17 * nv + 3) & ~3; }

  static constexpr bool ok(int nv) {
    // ALIAS lies inside RND in the PRE layout (a deliberate reuse, listed as the one region RND)
    const Region r[] = {{PW, 108, 1},   {TC, 72, 1},      {TN, 144, 1},    {SUMS, 27, 1},       {RC, 1, 1},
                        {OSUM, 3, 1},   {CPL, 32, 4},     {HYP, 28, 4},    {FC, 8, 1},          {MISC, 16, 1},
                        {NBL, 9, 1},    {NBOX_A, 3, 1},   {NSV, 9, 1},     {NBOX_B, 1, 1},
                        {PRE ? RND : ALIAS, PRE ? 12 : 8, 1},
                        {VWL, 8, 1},    {cost(nv), 8 * nv, 1}, {sp(nv), nv, 1}, {sel(nv), nv, 1}, {hv(nv), 7 * nv, 1}};
    return regions_ok(r, per_pixel(nv)) && per_pixel(nv) % 4 == 0 && M_FLAGS + 8 <= 16 &&
           (!PRE || (ALIAS >= RND && ALIAS + 8 <= RND + 12));
  }
  static constexpr bool ok_all() {
    for (int nv = 1; nv <= kMaxViews; ++nv) if (!ok(nv)) return false;
    return true;
  }
};
using WeakCarve = WeakCarveT<false>;

static_assert(StrongCarve<4, 16, 16>::ok_all(), "strong-sweep LDS carve (edge mode): overlap, alignment or bounds");
static_assert(StrongCarve<8, 8, 16>::ok_all(), "strong-sweep LDS carve (ACMH mode): overlap, alignment or bounds");
static_assert(WeakCarveT<false>::ok_all(), "weak-sweep LDS carve: overlap, alignment or bounds");
static_assert(WeakCarveT<true>::ok_all(), "weak-sweep LDS carve (DPE_WEAK_PRE): overlap, alignment or bounds");
// LDS budgets (160 KB per CU on gfx950).  Strong sweep: 4 waves per workgroup at the largest view
// count must fit one workgroup per CU at least (the dynamic-LDS attribute raises the 64 KB default).
static_assert(4 * StrongCarve<4, 16, 16>::total(kMaxViews) * 4 <= 160 * 1024, "strong-sweep workgroup LDS (edge)");
static_assert(4 * StrongCarve<8, 8, 16>::total(kMaxViews) * 4 <= 160 * 1024, "strong-sweep workgroup LDS (ACMH)");
// Weak sweep: at the headline 9 source views four 4-wave workgroups of 4 pixels per wave must fit
// a CU (4 resident waves per SIMD), i.e. <= 40 KB per workgroup.
static_assert(4 * (4 * 4 * WeakCarveT<false>::per_pixel(9) * 4) <= 160 * 1024, "weak-sweep LDS: 4 workgroups per CU at 9 views");
static_assert(4 * (4 * 4 * WeakCarveT<true>::per_pixel(9) * 4) <= 160 * 1024, "weak-sweep LDS (DPE_WEAK_PRE): 4 workgroups per CU at 9 views");

}  // namespace lds
}  // namespace dpe
