// TEST INFRASTRUCTURE (SURVEY.md §5 "ASan/UBSan on the CPU transcription"): drives the oracle's
// restatement of DPE.cu through every pass type on a small procedural scene, inside an executable
// built with -fsanitize=address,undefined (oracle/Makefile target `sanitize`).  Exits 0 when every
// pass returns and the sanitizers report nothing (they abort the process otherwise).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/dpe_mvs.h"

extern "C" int oracle_pm_run(const DpePassInput* in, const DpePassState* st, int nthreads);

namespace {
void params_main_h(DpePatchMatchParams* p) {   // the initialisers of main.h:78-106
  std::memset(p, 0, sizeof(*p));
  p->max_iterations = 3; p->num_images = 5; p->sigma_spatial = 5.0f; p->sigma_color = 3.0f; p->top_k = 4;
  p->depth_min = 0.0f; p->depth_max = 1.0f; p->geom_consistency = false;
  p->strong_radius = 5; p->strong_increment = 2; p->weak_radius = 5; p->weak_increment = 5;
  p->use_APD = true; p->use_edge = true; p->use_limit = true; p->use_label = true; p->use_radius = true;
  p->high_res_img = true; p->max_scale_size = 1; p->scale_size = 1; p->weak_peak_radius = 2; p->rotate_time = 4;
  p->ransac_threshold = 0.005f; p->geom_factor = 0.2f; p->state = DPE_FIRST_INIT;
}
uint32_t g_state = 12345u;
float frand() { g_state = g_state * 1664525u + 1013904223u; return (float)(g_state >> 8) / 16777216.0f; }
}  // namespace

int main() {
  const int W = 48, H = 36, N = 4;
  const size_t L = (size_t)W * H;
  std::vector<std::vector<float>> img(N, std::vector<float>(L));
  for (int i = 0; i < N; ++i)
    for (int y = 0; y < H; ++y)
      for (int x = 0; x < W; ++x) {
        const float v = 128.0f + 60.0f * std::sin(0.37f * (x + 2 * i)) * std::cos(0.29f * y) + 20.0f * frand();
        img[i][(size_t)y * W + x] = std::floor(std::fmin(255.0f, std::fmax(0.0f, v)));
      }
  for (size_t k = 0; k < L / 5; ++k) img[0][k] = 140.0f;   // a textureless band (WEAK pixels)
  std::vector<DpeCamera> cams(N);
  for (int i = 0; i < N; ++i) {
    DpeCamera& c = cams[i];
    std::memset(&c, 0, sizeof(c));
    const float f = 1.2f * W;
    c.K[0] = f; c.K[2] = W / 2.0f; c.K[4] = f; c.K[5] = H / 2.0f; c.K[8] = 1.0f;
    c.R[0] = c.R[4] = c.R[8] = 1.0f;
    c.t[0] = -0.15f * i; c.t[1] = 0.02f * i;
    c.c[0] = -c.t[0]; c.c[1] = -c.t[1];
    c.width = W; c.height = H; c.depth_min = 3.0f; c.depth_max = 7.0f;
  }
  std::vector<const float*> ip(N);
  for (int i = 0; i < N; ++i) ip[i] = img[i].data();
  std::vector<std::vector<float>> dep(N, std::vector<float>(L));
  std::vector<const float*> dp(N, nullptr);
  for (int i = 1; i < N; ++i) {
    for (size_t k = 0; k < L; ++k) dep[i][k] = 5.0f + 0.3f * frand();
    dp[i] = dep[i].data();
  }
  std::vector<uint8_t> edge(L, 0), edge_low((size_t)(W / 2) * (H / 2), 0);
  std::vector<int32_t> label(L, 1);
  for (int y = 0; y < H; ++y) { edge[(size_t)y * W + W / 3] = 255; label[(size_t)y * W + W / 3] = 0; }
  for (int y = 0; y < H / 2; ++y) edge_low[(size_t)y * (W / 2) + W / 6] = 255;
  for (size_t k = 0; k < L; ++k) if (k % W > W / 3) label[k] = 2;

  std::vector<float> planes(L * 4, 0.0f), costs(L, 0.0f);
  std::vector<uint8_t> weak(L, DPE_STRONG);
  std::vector<uint32_t> sel(L, 0u);
  const int states[3] = {DPE_FIRST_INIT, DPE_REFINE_INIT, DPE_REFINE_ITER};
  for (int pass = 0; pass < 3; ++pass) {
    DpePassInput in;
    std::memset(&in, 0, sizeof(in));
    in.width = W; in.height = H; in.num_images = N;
    in.images = ip.data(); in.cams = cams.data();
    in.edge = edge.data(); in.edge_low_res = edge_low.data(); in.low_width = W / 2; in.low_height = H / 2;
    in.label = label.data();
    params_main_h(&in.params);
    DpePatchMatchParams& P = in.params;
    P.state = states[pass];
    P.num_images = N;
    P.depth_min = 3.0f * 0.6f; P.depth_max = 7.0f * 1.2f;
    P.max_iterations = 2;
    P.use_APD = pass > 0; P.use_edge = pass > 0;
    P.geom_consistency = pass == 2;
    in.depths = pass == 2 ? dp.data() : nullptr;
    in.seed = 7; in.pass_salt = (uint32_t)pass;
    if (pass == 1) for (size_t k = 0; k < L; ++k) if (weak[k] == DPE_UNKNOWN) weak[k] = DPE_WEAK;
    DpePassState st{planes.data(), weak.data(), sel.data(), costs.data()};
    const int rc = oracle_pm_run(&in, &st, 2);
    if (rc != 0) { std::fprintf(stderr, "pass %d failed: %d\n", pass, rc); return 1; }
    int nw = 0;
    for (size_t k = 0; k < L; ++k) nw += weak[k] == DPE_WEAK;
    std::printf("pass %d ok (%d WEAK pixels)\n", pass, nw);
  }
  return 0;
}
