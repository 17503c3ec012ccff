// TEST INFRASTRUCTURE (SURVEY.md §5 sanitizers): the host pipeline's image code -- JPEG decode,
// EdgeSegment with its restated OpenCV operations, the resamplers -- in an executable built with
// -fsanitize=address,undefined (dpe-mvs_amd/Makefile target `sanitize-host`).  Usage:
//   host_sanitize <grey.jpg> <colour.jpg>    exits 0 when the sanitizers report nothing
#include <cstdio>
#include <string>
#include <vector>

#include "../../dpe-mvs_amd/host/host.h"

using namespace dpe_host;

int main(int argc, char** argv) {
  if (argc < 3) { std::fprintf(stderr, "usage: host_sanitize grey.jpg colour.jpg\n"); return 2; }
  std::string err;
  GrayImage g;
  if (!read_gray(argv[1], g, err)) { std::fprintf(stderr, "read_gray: %s\n", err.c_str()); return 1; }
  ColorImage c;
  if (!read_bgr(argv[2], c, err)) { std::fprintf(stderr, "read_bgr: %s\n", err.c_str()); return 1; }
  const int w = g.w, h = g.h;
  std::vector<uint8_t> e((size_t)w * h);
  canny_l2(g.px.data(), w, h, 30, 90, e.data());
  canny_l2(g.px.data(), w, h, 90, 30, e.data());
  for (int s = 0; s < 2; ++s)
    for (int mode = 0; mode < 2; ++mode)
      for (int hr = 0; hr < 2; ++hr) {
        Mat m;
        if (!edge_segment(s, g.px.data(), w, h, mode, mode == 0, hr != 0, m, err)) {
          std::fprintf(stderr, "edge_segment(%d, %d, %d): %s\n", s, mode, hr, err.c_str());
          return 1;
        }
      }
  const int sizes[][2] = {{w / 2, h / 2}, {w * 2 / 3, h * 3 / 4}, {w + 7, h + 5}, {3, 2}};
  for (auto& sz : sizes) {
    std::vector<uint8_t> r((size_t)sz[0] * sz[1]);
    resize_u8(g.px.data(), w, h, r.data(), sz[0], sz[1]);
    std::vector<float> f(g.px.begin(), g.px.end()), rf((size_t)sz[0] * sz[1]);
    resize_linear(f.data(), w, h, rf.data(), sz[0], sz[1]);
    std::vector<uint32_t> src((size_t)w * h, 7u), dst((size_t)sz[0] * sz[1], 0u);
    rescale_nearest(src.data(), w, h, dst.data(), sz[0], sz[1], 4);
  }
  std::vector<int> lab((size_t)w * h), cnt;
  threshold_binary(e.data(), e.size(), 127);
  connect(e.data(), w, h, lab.data(), cnt);
  std::vector<std::array<int, 4>> lines;
  hough_lines_p(e.data(), w, h, 1, 3.14159265358979323846 / 180, 10, 10, 3, lines);
  for (const auto& l : lines) draw_line(e.data(), w, h, l[0], l[1], l[2], l[3], 255);
  std::printf("host sanitize ok: %dx%d, %zu labels, %zu segments, colour %dx%d\n", w, h, cnt.size(), lines.size(), c.w, c.h);
  return 0;
}
