"""The Bresenham edge walk of GenNeighbours / RANSACToGetFitPlane (BresenhamLine, DPE.cu:158-244)
in the device forms of dpe-mvs_amd/csrc/bres_walk.h -- byte batches (walk_bytes, and
walk_bytes_flat, the form GenNeighbours runs) -- against a literal transcription of the reference loop, on random edge
maps, endpoints and map sizes (non-multiple-of-8 widths, steps past the endpoint that wrap rows,
max_step of both resolution classes).  The header is pure C++, compiled here with g++."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "dpe-mvs_amd", "csrc", "bres_walk.h")

HARNESS = r"""
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include <random>
#include "%s"
using namespace dpe::bres;

// DPE.cu:158-244 for one direction: the loop as written (tags, move, test, step limit); an index
// outside the map reads no edge (the restatement's range rule)
static bool ref_dir(int x0, int y0, int x1, int y1, int max_step, const std::vector<unsigned char>& e, int w, int h) {
  const int dx = std::abs(x1 - x0), sx = x0 < x1 ? 1 : -1;
  const int dy = std::abs(y1 - y0), sy = y0 < y1 ? 1 : -1;
  int erro = (dx > dy ? dx : dy) / 2, step = 0;
  bool tagx = true, tagy = true;
  while (tagx || tagy) {
    if (x0 == x1) tagx = false;
    if (y0 == y1) tagy = false;
    const int e2 = erro;
    if (e2 > -dx) { erro -= dy; x0 += sx; }
    if (e2 < dy) { erro += dx; y0 += sy; }
    const long pc = (long)x0 + (long)y0 * w;
    if (pc >= 0 && pc < (long)w * h && e[pc]) return true;
    step += 1;
    if (step >= max_step) break;
  }
  return false;
}

int main(int argc, char** argv) {
  std::mt19937 rng(12345);
  long walks = 0, hits = 0;
  for (int m = 0; m < 60; ++m) {
    const int W = 64 + rng() %% 1700, H = 48 + rng() %% 1300;
    const int w = 8 + rng() %% (W / 2 + 1), h = 8 + rng() %% (H / 2 + 1);
    const double dens = m %% 3 == 0 ? 0.0005 : (m %% 3 == 1 ? 0.01 : 0.08);
    std::vector<unsigned char> e((size_t)w * h);
    for (auto& v : e) v = (rng() %% 1000000) < dens * 1000000 ? (unsigned char)(1 + rng() %% 255) : 0;
    const float scale_x = 1.0f * w / (float)W, scale_y = 1.0f * h / (float)H;
    for (int hr = 0; hr < 2; ++hr) {
      const int max_step = hr ? (int)std::round((w > h ? w : h) / 60.0) : (w > h ? w : h);
      for (int q = 0; q < 1500; ++q) {
        int ax = rng() %% W, ay = rng() %% H, bx = rng() %% W, by = rng() %% H;
        if (q %% 10 == 0) { bx = W - 1 - rng() %% 3; }             // endpoints on the last columns:
        if (q %% 10 == 1) { ax = W - 1; ay = rng() %% H; }          // steps past them wrap rows
        if (q %% 10 == 2) { bx = ax; }                              // vertical
        if (q %% 10 == 3) { by = ay; }                              // horizontal
        if (q %% 10 == 4) { bx = ax; by = ay; }                     // degenerate
        for (int pass = 0; pass < 2; ++pass) {
          const int fx = pass == 0 ? bx : ax, fy = pass == 0 ? by : ay;
          const int tx = pass == 0 ? ax : bx, ty = pass == 0 ? ay : by;
          const int x0 = (int)std::fmin(std::roundf(fx * scale_x), (float)(w - 1));
          const int y0 = (int)std::fmin(std::roundf(fy * scale_y), (float)(h - 1));
          const int x1 = (int)std::fmin(std::roundf(tx * scale_x), (float)(w - 1));
          const int y1 = (int)std::fmin(std::roundf(ty * scale_y), (float)(h - 1));
          const bool r = ref_dir(x0, y0, x1, y1, max_step, e, w, h);
          const Walk wk = start(x0, y0, x1, y1, max_step);
          const bool b8 = walk_bytes<8>(wk, e.data(), w, h) && walk_bytes_flat<8>(x0, y0, x1, y1, max_step, e.data(), w, h);
          if (walk_bytes_flat<8>(x0, y0, x1, y1, max_step, e.data(), w, h) != walk_bytes<8>(wk, e.data(), w, h)) {
            std::printf("FLAT %%d,%%d -> %%d,%%d\n", x0, y0, x1, y1); return 1;
          }
          ++walks; hits += r;
          if (b8 != r) {
            std::printf("MISMATCH map %%d (%%dx%%d low %%dx%%d) %%d,%%d -> %%d,%%d max_step %%d: ref %%d bytes %%d\n",
                        m, W, H, w, h, x0, y0, x1, y1, max_step, r, b8);
            return 1;
          }
        }
      }
    }
  }
  std::printf("ok %%ld walks, %%ld hit an edge\n", walks, hits);
  return 0;
}
"""


def test_walk_forms_match_reference_loop(tmp_path):
    src = tmp_path / "bres.cpp"
    src.write_text(HARNESS % HDR)
    exe = tmp_path / "bres"
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe), str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    walks, hits = int(r.stdout.split()[1]), int(r.stdout.split()[3])
    assert walks == 360000 and 0.05 * walks < hits < 0.95 * walks, r.stdout
