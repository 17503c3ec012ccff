// edges.cpp — the edge / label precompute of DPE-MVS: EdgeSegment, Roberts and Connect
// (DPE.cpp:9-291) driven by GetProblemEdges (main.cpp:331-388), with the OpenCV operations they call
// restated here (OpenCV is not a dependency of this build):
//   cv::resize INTER_LINEAR, 8-bit  -> resize_u8   (exact 2x downscale = INTER_AREA fast path,
//                                                  otherwise the 11-bit fixed-point bilinear)
//   cv::Canny(L2gradient, aperture 3) -> canny_l2  (Sobel with replicated border, squared-magnitude
//                                                  non-maximum suppression, 8-connected hysteresis)
//   cv::HoughLinesP                   -> hough_lines_p (progressive probabilistic Hough, cv::RNG)
//   cv::line(thickness 1, LINE_8)     -> draw_line (LineIterator's Bresenham, left to right)
//   cv::threshold(THRESH_BINARY)      -> threshold_binary
// The restatements follow OpenCV 4.x's published algorithms (imgproc canny.cpp, hough.cpp,
// resize.cpp, drawing.cpp); no OpenCV build exists in this environment, so agreement with a real
// OpenCV is "parity unpinned" — the tests pin each piece with known answers instead.
#include "host.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <filesystem>

namespace fs = std::filesystem;

namespace dpe_host {

namespace {
// cvRound: round half to even (SSE2 cvtsd2si under the default rounding mode)
inline int cv_round(double v) { return (int)std::nearbyint(v); }
inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// Horizontal / vertical taps of OpenCV's resize for INTER_LINEAR (resize.cpp, ksize 2)
struct LinTab {
  std::vector<int> ofs;          // left source index
  std::vector<short> a;          // 11-bit fixed-point weights (1 - f, f)
  int xmin = 0, xmax = 0;        // [xmin, xmax): both taps inside
};
LinTab lin_tab(int ssize, int dsize) {
  LinTab t;
  t.ofs.resize(dsize); t.a.resize(2 * (size_t)dsize);
  const double scale = 1.0 / ((double)dsize / ssize);
  t.xmin = 0; t.xmax = dsize;
  for (int d = 0; d < dsize; ++d) {
    float f = (float)((d + 0.5) * scale - 0.5);
    int s = (int)std::floor(f);
    f -= (float)s;
    if (s < 0) { t.xmin = d + 1; f = 0; s = 0; }
    if (s + 1 >= ssize) {
      t.xmax = std::min(t.xmax, d);
      if (s >= ssize - 1) { f = 0; s = ssize - 1; }
    }
    t.ofs[d] = s;
    const float c0 = 1.0f - f, c1 = f;
    t.a[2 * d] = (short)std::min(32767, std::max(-32768, cv_round(c0 * 2048.0f)));
    t.a[2 * d + 1] = (short)std::min(32767, std::max(-32768, cv_round(c1 * 2048.0f)));
  }
  return t;
}
}  // namespace

// cv::resize(src, dst, Size(nw, nh), 0, 0, INTER_LINEAR) on CV_8UC1.
void resize_u8(const uint8_t* src, int w, int h, uint8_t* dst, int nw, int nh) {
  if (w == nw && h == nh) { std::memcpy(dst, src, (size_t)w * h); return; }
  const double scale_x = 1.0 / ((double)nw / w), scale_y = 1.0 / ((double)nh / h);
  const int isx = (int)std::lround(scale_x), isy = (int)std::lround(scale_y);
  const bool area_fast = std::fabs(scale_x - isx) < 2.220446049250313e-16 && std::fabs(scale_y - isy) < 2.220446049250313e-16;
  if (area_fast && isx == 2 && isy == 2) {   // INTER_LINEAR at exactly 1/2 is INTER_AREA's fast path
    for (int y = 0; y < nh; ++y) {
      const uint8_t* s0 = src + (size_t)(2 * y) * w;
      const uint8_t* s1 = s0 + w;
      for (int x = 0; x < nw; ++x)
        dst[(size_t)y * nw + x] = (uint8_t)((s0[2 * x] + s0[2 * x + 1] + s1[2 * x] + s1[2 * x + 1] + 2) >> 2);
    }
    return;
  }
  const LinTab tx = lin_tab(w, nw), ty = lin_tab(h, nh);
  std::vector<int> rows((size_t)h * nw);   // HResizeLinear<uchar, int, short, 2048>
  for (int y = 0; y < h; ++y) {
    const uint8_t* s = src + (size_t)y * w;
    int* d = rows.data() + (size_t)y * nw;
    for (int x = 0; x < nw; ++x) {
      const int sx = tx.ofs[x];
      d[x] = x < tx.xmax ? s[sx] * tx.a[2 * x] + s[sx + 1] * tx.a[2 * x + 1] : s[sx] * 2048;
    }
  }
  for (int y = 0; y < nh; ++y) {   // VResizeLinear: 16/8-lane vector formula, scalar FixedPtCast tail
    const int sy = ty.ofs[y], sy1 = std::min(sy + 1, h - 1);
    const int* S0 = rows.data() + (size_t)sy * nw;
    const int* S1 = rows.data() + (size_t)sy1 * nw;
    const int b0 = ty.a[2 * y], b1 = ty.a[2 * y + 1];
    uint8_t* d = dst + (size_t)y * nw;
    auto vec = [&](int x) {
      const int p0 = (int)(int16_t)std::min(32767, std::max(-32768, S0[x] >> 4));
      const int p1 = (int)(int16_t)std::min(32767, std::max(-32768, S1[x] >> 4));
      const int v = (int)(int16_t)(((p0 * b0) >> 16) + ((p1 * b1) >> 16));
      return sat_u8((v + 2) >> 2);
    };
    int x = 0;
    for (; x <= nw - 16; x += 16) for (int k = 0; k < 16; ++k) d[x + k] = vec(x + k);
    for (; x < nw - 8; x += 8) for (int k = 0; k < 8; ++k) d[x + k] = vec(x + k);
    for (; x < nw; ++x) d[x] = sat_u8((S0[x] * b0 + S1[x] * b1 + (1 << 21)) >> 22);
  }
}

// cv::threshold(src, dst, thr, 255, THRESH_BINARY) on 8-bit data (in place allowed)
void threshold_binary(uint8_t* img, size_t n, int thr) {
  for (size_t i = 0; i < n; ++i) img[i] = img[i] > thr ? 255 : 0;
}

// cv::Canny(src, dst, low, high, 3, true): 0/255 edge map.
void canny_l2(const uint8_t* src, int w, int h, double low_thresh, double high_thresh, uint8_t* dst) {
  if (low_thresh > high_thresh) std::swap(low_thresh, high_thresh);
  low_thresh = std::min(32767.0, low_thresh);
  high_thresh = std::min(32767.0, high_thresh);
  if (low_thresh > 0) low_thresh *= low_thresh;
  if (high_thresh > 0) high_thresh *= high_thresh;
  const int low = (int)std::floor(low_thresh), high = (int)std::floor(high_thresh);
  // Sobel 3x3, BORDER_REPLICATE, CV_16S
  std::vector<int16_t> dx((size_t)w * h), dy((size_t)w * h);
  auto at = [&](int x, int y) -> int {
    x = x < 0 ? 0 : (x >= w ? w - 1 : x);
    y = y < 0 ? 0 : (y >= h ? h - 1 : y);
    return src[(size_t)y * w + x];
  };
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const int gx = (at(x + 1, y - 1) - at(x - 1, y - 1)) + 2 * (at(x + 1, y) - at(x - 1, y)) + (at(x + 1, y + 1) - at(x - 1, y + 1));
      const int gy = (at(x - 1, y + 1) - at(x - 1, y - 1)) + 2 * (at(x, y + 1) - at(x, y - 1)) + (at(x + 1, y + 1) - at(x + 1, y - 1));
      dx[(size_t)y * w + x] = (int16_t)gx;
      dy[(size_t)y * w + x] = (int16_t)gy;
    }
  // squared magnitude with a zero frame: mag[(y+1)*(w+2) + x+1]
  const int ms = w + 2;
  std::vector<int> mag((size_t)ms * (h + 2), 0);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const int a = dx[(size_t)y * w + x], b = dy[(size_t)y * w + x];
      mag[(size_t)(y + 1) * ms + x + 1] = a * a + b * b;
    }
  // map: 0 = may be an edge, 1 = not an edge, 2 = edge; frame of 1s
  std::vector<uint8_t> map((size_t)ms * (h + 2), 1);
  std::vector<size_t> stack;
  stack.reserve((size_t)w * h / 8 + 16);
  constexpr int CANNY_SHIFT = 15;
  const int TG22 = (int)(0.4142135623730950488016887242097 * (1 << CANNY_SHIFT) + 0.5);
  for (int y = 0; y < h; ++y) {
    const int* mp = mag.data() + (size_t)y * ms + 1;        // row above
    const int* ma = mag.data() + (size_t)(y + 1) * ms + 1;  // this row
    const int* mn = mag.data() + (size_t)(y + 2) * ms + 1;  // row below
    uint8_t* pm = map.data() + (size_t)(y + 1) * ms + 1;
    int prev_flag = 0;
    for (int x = 0; x < w; ++x) {
      const int m = ma[x];
      bool push = false;
      if (m > low) {
        const int xs = dx[(size_t)y * w + x], ys = dy[(size_t)y * w + x];
        const int ax = std::abs(xs);
        const int ay = std::abs(ys) << CANNY_SHIFT;
        const int tg22x = ax * TG22;
        if (ay < tg22x) {
          push = m > ma[x - 1] && m >= ma[x + 1];
        } else {
          const int tg67x = tg22x + (ax << (CANNY_SHIFT + 1));
          if (ay > tg67x) {
            push = m > mp[x] && m >= mn[x];
          } else {
            const int s = (xs ^ ys) < 0 ? -1 : 1;
            push = m > mp[x - s] && m > mn[x + s];
          }
        }
      }
      if (!push) { prev_flag = 0; pm[x] = 1; continue; }
      if (!prev_flag && m > high && pm[x - ms] != 2) {
        pm[x] = 2; stack.push_back((size_t)(pm + x - map.data()));
        prev_flag = 1;
      } else {
        pm[x] = 0;
      }
    }
  }
  while (!stack.empty()) {   // hysteresis: 8-connected growth from the strong seeds
    const size_t i = stack.back();
    stack.pop_back();
    const long off[8] = {-ms - 1, -ms, -ms + 1, -1, 1, ms - 1, ms, ms + 1};
    for (long o : off) {
      const size_t j = (size_t)((long)i + o);
      if (!map[j]) { map[j] = 2; stack.push_back(j); }
    }
  }
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) dst[(size_t)y * w + x] = map[(size_t)(y + 1) * ms + x + 1] == 2 ? 255 : 0;
}

// Roberts (DPE.cpp:9-25): the frame gets t1 = t2 = 50; (uchar) of the truncated magnitude
void roberts(const uint8_t* src, int w, int h, uint8_t* dst) {
  for (int i = 0; i < h; ++i)
    for (int j = 0; j < w; ++j) {
      int t1 = 50, t2 = 50;
      if (i > 0 && i < h - 1 && j > 0 && j < w - 1) {
        t1 = src[(size_t)i * w + j] - src[(size_t)(i + 1) * w + j + 1];
        t2 = src[(size_t)(i + 1) * w + j] - src[(size_t)i * w + j + 1];
      }
      dst[(size_t)i * w + j] = (uint8_t)(int)std::sqrt((double)(t1 * t1 + t2 * t2));
    }
}

// Connect (DPE.cpp:27-127): 4-connected components of the zero pixels (255 -> label 0), labels
// renumbered 1.. in first-seen order of their roots; label_cnt[k] = pixels of label k.
void connect(const uint8_t* img, int w, int h, int* label, std::vector<int>& label_cnt) {
  auto px = [&](int y, int x) { return img[(size_t)y * w + x]; };
  std::vector<int> conn{0};
  int cnt = 1;
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      int& L = label[(size_t)y * w + x];
      if (px(y, x) == 255) { L = 0; continue; }
      const bool left_n = x > 0 && px(y, x) == 0 && px(y, x - 1) == 0;
      const bool up_n = y > 0 && px(y, x) == 0 && px(y - 1, x) == 0;
      bool left = false, up = false;
      if (left_n) { L = label[(size_t)y * w + x - 1]; left = true; }
      if (up_n) { L = label[(size_t)(y - 1) * w + x]; up = true; }
      if (!left && !up) {
        L = cnt; conn.push_back(cnt); cnt++;
      } else if (left && up) {
        const int ll = label[(size_t)y * w + x - 1], ul = label[(size_t)(y - 1) * w + x];
        if (ll > ul) { conn[ll] = ul; L = ul; }
        else if (ll < ul) { conn[ul] = ll; L = ll; }
      }
    }
  for (size_t i = 1; i < conn.size(); ++i) {
    int cur = conn[i], pre = conn[cur];
    while (pre != cur) { cur = pre; pre = conn[pre]; }
    conn[i] = cur;
  }
  int label_num = 1;
  std::vector<int> mapping{0};
  for (size_t i = 1; i < conn.size(); ++i) {
    mapping.push_back(0);
    if (conn[i] == (int)i) mapping[i] = label_num++;
  }
  for (size_t i = 1; i < conn.size(); ++i) conn[i] = mapping[conn[i]];
  label_cnt.assign(label_num, 0);
  for (size_t i = 0; i < (size_t)w * h; ++i) {
    const int l = label[i];
    label[i] = conn[l];
    label_cnt[conn[l]]++;
  }
}

// cv::line(img, p0, p1, 255, 1, LINE_8): LineIterator (8-connected Bresenham, left to right);
// the endpoints come from HoughLinesP and lie inside the image.
void draw_line(uint8_t* img, int w, int h, int x0, int y0, int x1, int y1, uint8_t value) {
  if (x0 < 0 || x1 < 0 || y0 < 0 || y1 < 0 || x0 >= w || x1 >= w || y0 >= h || y1 >= h) return;
  int dx = x1 - x0, dy = y1 - y0;
  int s = dx < 0 ? -1 : 0;
  dx = (dx ^ s) - s;
  dy = (dy ^ s) - s;
  int px = x0, py = y0;
  if (s) { px = x1; py = y1; }                 // start at the left end
  long istep = w, bt_pix = 1;
  s = dy < 0 ? -1 : 0;
  dy = (dy ^ s) - s;
  istep = (istep ^ s) - s;
  s = dy > dx ? -1 : 0;
  dx ^= dy & s; dy ^= dx & s; dx ^= dy & s;     // swap if steep
  bt_pix ^= istep & s; istep ^= bt_pix & s; bt_pix ^= istep & s;
  int err = dx - (dy + dy);
  const int plus_delta = dx + dx, minus_delta = -(dy + dy);
  const long plus_step = istep, minus_step = bt_pix;
  long p = (long)py * w + px;
  for (int i = 0; i <= dx; ++i) {
    img[p] = value;
    const int mask = err < 0 ? -1 : 0;
    err += minus_delta + (plus_delta & mask);
    p += minus_step + (plus_step & mask);
  }
}

// cv::HoughLinesP(img, lines, rho, theta, threshold, minLineLength, maxLineGap)
// (HoughLinesProbabilistic: random point order from cv::RNG((uint64)-1)).
void hough_lines_p(const uint8_t* img, int width, int height, double rho_d, double theta_d, int threshold,
                   double min_len_d, double max_gap_d, std::vector<std::array<int, 4>>& lines) {
  const float rho = (float)rho_d, theta = (float)theta_d;
  const int lineLength = cv_round(min_len_d), lineGap = cv_round(max_gap_d);
  const float irho = 1 / rho;
  uint64_t state = ~0ull;                                    // cv::RNG((uint64)-1)
  auto next = [&]() -> uint32_t {
    state = (uint64_t)(uint32_t)state * 4164903690u + (uint32_t)(state >> 32);
    return (uint32_t)state;
  };
  int numangle = (int)std::floor(3.14159265358979323846 / theta) + 1;   // computeNumangle(0, pi, theta)
  if (numangle > 1 && std::fabs(3.14159265358979323846 - (numangle - 1) * (double)theta) < theta / 2.0) --numangle;
  const int numrho = cv_round(((width + height) * 2 + 1) / rho);
  std::vector<int> accum((size_t)numangle * numrho, 0);
  std::vector<uint8_t> mask((size_t)width * height);
  std::vector<float> ttab(2 * (size_t)numangle);
  for (int n = 0; n < numangle; ++n) {
    ttab[2 * n] = (float)(std::cos((double)n * theta) * irho);
    ttab[2 * n + 1] = (float)(std::sin((double)n * theta) * irho);
  }
  std::vector<std::array<int, 2>> nz;   // (x, y)
  for (int y = 0; y < height; ++y)
    for (int x = 0; x < width; ++x) {
      if (img[(size_t)y * width + x]) { mask[(size_t)y * width + x] = 1; nz.push_back({x, y}); }
      else mask[(size_t)y * width + x] = 0;
    }
  auto rbin = [&](int j, int i, int n) {
    const float v = (float)j * ttab[2 * n] + (float)i * ttab[2 * n + 1];
    return (int)std::nearbyint(v) + (numrho - 1) / 2;
  };
  const int shift = 16;
  for (int count = (int)nz.size(); count > 0; count--) {
    const int idx = (int)(next() % (uint32_t)count);         // rng.uniform(0, count)
    int max_val = threshold - 1, max_n = 0;
    const std::array<int, 2> point = nz[idx];
    int lx[2] = {0, 0}, ly[2] = {0, 0};
    const int i = point[1], j = point[0];
    nz[idx] = nz[count - 1];
    if (!mask[(size_t)i * width + j]) continue;
    for (int n = 0; n < numangle; ++n) {
      const int val = ++accum[(size_t)n * numrho + rbin(j, i, n)];
      if (max_val < val) { max_val = val; max_n = n; }
    }
    if (max_val < threshold) continue;
    const float a = -ttab[2 * max_n + 1], b = ttab[2 * max_n];
    int x0 = j, y0 = i, dx0, dy0;
    bool xflag;
    if (std::fabs(a) > std::fabs(b)) {
      xflag = true;
      dx0 = a > 0 ? 1 : -1;
      dy0 = (int)std::nearbyint(b * (float)(1 << shift) / std::fabs(a));
      y0 = (y0 << shift) + (1 << (shift - 1));
    } else {
      xflag = false;
      dy0 = b > 0 ? 1 : -1;
      dx0 = (int)std::nearbyint(a * (float)(1 << shift) / std::fabs(b));
      x0 = (x0 << shift) + (1 << (shift - 1));
    }
    for (int k = 0; k < 2; ++k) {
      int gap = 0, x = x0, y = y0, dx = dx0, dy = dy0;
      if (k > 0) { dx = -dx; dy = -dy; }
      for (;; x += dx, y += dy) {
        const int j1 = xflag ? x : x >> shift, i1 = xflag ? y >> shift : y;
        if (j1 < 0 || j1 >= width || i1 < 0 || i1 >= height) break;
        if (mask[(size_t)i1 * width + j1]) { gap = 0; ly[k] = i1; lx[k] = j1; }
        else if (++gap > lineGap) break;
      }
    }
    const bool good = std::abs(lx[1] - lx[0]) >= lineLength || std::abs(ly[1] - ly[0]) >= lineLength;
    for (int k = 0; k < 2; ++k) {
      int x = x0, y = y0, dx = dx0, dy = dy0;
      if (k > 0) { dx = -dx; dy = -dy; }
      for (;; x += dx, y += dy) {
        const int j1 = xflag ? x : x >> shift, i1 = xflag ? y >> shift : y;
        uint8_t& m = mask[(size_t)i1 * width + j1];
        if (m) {
          if (good)
            for (int n = 0; n < numangle; ++n) accum[(size_t)n * numrho + rbin(j1, i1, n)]--;
          m = 0;
        }
        if (i1 == ly[k] && j1 == lx[k]) break;
      }
    }
    if (good) lines.push_back({lx[0], ly[0], lx[1], ly[1]});
  }
}

namespace {
// the frame rule after the final threshold (DPE.cpp:238-249)
void fix_frame(uint8_t* d, int cols, int rows) {
  for (int y = 0; y < rows; ++y) {
    if (d[y * cols + 1] == 0) d[y * cols] = 0;
    if (d[y * cols + cols - 2] == 0) d[y * cols + cols - 1] = 0;
  }
  for (int x = 0; x < cols; ++x) {
    if (d[1 * cols + x] == 0) d[x] = 0;
    if (d[(rows - 2) * cols + x] == 0) d[(rows - 1) * cols + x] = 0;
  }
}
}  // namespace

namespace {
// the data-parallel stages on the device when one is given (bit-identical), else on the host
bool stage_resize_u8(const EdgeDevice* dev, const uint8_t* src, int w, int h, uint8_t* dst, int nw, int nh, std::string& err) {
  if (!dev || !dev->ctx) { resize_u8(src, w, h, dst, nw, nh); return true; }
  std::lock_guard<std::mutex> lk(*dev->mu);
  if (dpe_resize_u8(dev->ctx, src, w, h, dst, nw, nh) != 0) { err = dpe_last_error(); return false; }
  return true;
}
bool stage_canny(const EdgeDevice* dev, const uint8_t* src, int w, int h, double low, double high, uint8_t* dst, std::string& err) {
  if (!dev || !dev->ctx) { canny_l2(src, w, h, low, high, dst); return true; }
  std::lock_guard<std::mutex> lk(*dev->mu);
  if (dpe_canny(dev->ctx, src, w, h, low, high, dst) != 0) { err = dpe_last_error(); return false; }
  return true;
}
bool stage_roberts_threshold(const EdgeDevice* dev, const uint8_t* src, int w, int h, int thr, uint8_t* dst, std::string& err) {
  if (!dev || !dev->ctx) { roberts(src, w, h, dst); threshold_binary(dst, (size_t)w * h, thr); return true; }
  std::lock_guard<std::mutex> lk(*dev->mu);
  if (dpe_roberts_threshold(dev->ctx, src, w, h, thr, dst) != 0) { err = dpe_last_error(); return false; }
  return true;
}
bool stage_resize_linear(const EdgeDevice* dev, const float* src, int w, int h, float* dst, int nw, int nh, std::string& err) {
  if (!dev || !dev->ctx) { resize_linear(src, w, h, dst, nw, nh); return true; }
  std::lock_guard<std::mutex> lk(*dev->mu);
  if (dpe_resize_linear(dev->ctx, src, w, h, dst, nw, nh) != 0) { err = dpe_last_error(); return false; }
  return true;
}
}  // namespace

// EdgeSegment (DPE.cpp:129-291) for mode 0 (edges: CV_8UC1 0/255) and mode 1 (labels: CV_32SC1,
// -1 = small region, 0 = boundary, > 0 region).
bool edge_segment(int scale, const uint8_t* src, int cols, int rows, int mode, bool use_canny, bool high_res, Mat& out,
                  std::string& err, const EdgeDevice* dev) {
  if (cols < 4 || rows < 4) { err = "EdgeSegment: image too small"; return false; }
  const int robthr = high_res ? 4 : 6;
  const int weak_tex_num = (int)(1.0 * rows * cols / (1024 << scale << scale));
  std::vector<uint8_t> dst;
  int dw = 0, dh = 0;
  if (!use_canny) {
    std::vector<uint8_t> down(src, src + (size_t)cols * rows);
    int w = cols, h = rows;
    if (high_res) {
      std::vector<uint8_t> t((size_t)(w / 2) * (h / 2));
      if (!stage_resize_u8(dev, down.data(), w, h, t.data(), w / 2, h / 2, err)) return false;
      down.swap(t); w /= 2; h /= 2;
    }
    {
      std::vector<uint8_t> t((size_t)(w / 2) * (h / 2));
      if (!stage_resize_u8(dev, down.data(), w, h, t.data(), w / 2, h / 2, err)) return false;
      down.swap(t); w /= 2; h /= 2;
    }
    const int mn = std::min(w, h);
    const int houthr = (int)(mn / 30.0), min_line_length = (int)(mn / 30.0), max_line_gap = (int)(mn / 30.0);
    dst.resize((size_t)w * h);
    if (!stage_roberts_threshold(dev, down.data(), w, h, robthr, dst.data(), err)) return false;
    std::vector<int> lab0((size_t)w * h);
    std::vector<int> cnt0;
    connect(dst.data(), w, h, lab0.data(), cnt0);
    std::vector<uint8_t> weak((size_t)w * h);
    for (size_t k = 1; k < cnt0.size(); ++k) {
      if (cnt0[k] < weak_tex_num) continue;
      const int wi = (int)k;
      std::fill(weak.begin(), weak.end(), 0);
      for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
          if (lab0[(size_t)y * w + x] == wi) continue;
          const bool border = (x > 0 && lab0[(size_t)y * w + x - 1] == wi) || (x < w - 1 && lab0[(size_t)y * w + x + 1] == wi) ||
                              (y > 0 && lab0[(size_t)(y - 1) * w + x] == wi) || (y < h - 1 && lab0[(size_t)(y + 1) * w + x] == wi);
          if (border) weak[(size_t)y * w + x] = 255;
        }
      std::vector<std::array<int, 4>> lines;
      hough_lines_p(weak.data(), w, h, 1, 3.14159265358979323846 / 180, houthr, min_line_length, max_line_gap, lines);
      for (const auto& l : lines) draw_line(dst.data(), w, h, l[0], l[1], l[2], l[3], 255);
    }
    dw = w; dh = h;
  } else {
    float histogram[256] = {0};
    for (size_t i = 0; i < (size_t)cols * rows; ++i) histogram[src[i]]++;
    const int half = rows * cols / 2;
    int median_val = -1, temp_sum = 0;
    for (int i = 0; i < 255; ++i) {
      temp_sum = (int)((float)temp_sum + histogram[i]);
      if (temp_sum > half) { median_val = i; break; }
    }
    const float sigma = 0.67f;
    const int t1 = (int)((1 - sigma) * (float)median_val), t2 = median_val;
    dst.resize((size_t)cols * rows);
    if (!stage_canny(dev, src, cols, rows, t1, t2, dst.data(), err)) return false;
    dw = cols; dh = rows;
  }
  int ow, oh;
  if (mode == 0) { ow = cols; oh = rows; }
  else {
    const float factor = 1.0f / (float)(1 << scale);
    ow = (int)std::round(cols * factor); oh = (int)std::round(rows * factor);
  }
  std::vector<uint8_t> rs((size_t)ow * oh);
  if (!stage_resize_u8(dev, dst.data(), dw, dh, rs.data(), ow, oh, err)) return false;
  threshold_binary(rs.data(), rs.size(), robthr);
  fix_frame(rs.data(), ow, oh);
  if (mode == 0) {
    out.create(oh, ow, CV_8UC1);
    std::memcpy(out.data.data(), rs.data(), rs.size());
    return true;
  }
  out.create(oh, ow, CV_32SC1);
  int* lab = out.ptr<int>();
  std::vector<int> cnt;
  connect(rs.data(), ow, oh, lab, cnt);
  for (size_t i = 0; i < (size_t)ow * oh; ++i)
    if (cnt[lab[i]] <= weak_tex_num && lab[i] != 0) lab[i] = -1;
  return true;
}

// GetProblemEdges (main.cpp:331-388): edges_<s>.dmb from the scaled image (32-bit float resize,
// then round to 8 bits), labels_<s>.dmb from the full-resolution image; files that exist are kept.
bool get_problem_edges(const GrayImage& full, int scale_size, const std::string& result_folder, bool use_edge,
                       bool use_label, bool high_res, std::string& err, const EdgeDevice* dev) {
  int scale = 0;
  while ((1 << scale) < scale_size) scale++;
  const fs::path rf(result_folder);
  std::error_code ec;
  fs::create_directories(rf, ec);
  if (use_edge) {
    const fs::path ep = rf / ("edges_" + std::to_string(scale) + ".dmb");
    if (!fs::exists(ep)) {
      const float factor = 1.0f / (float)scale_size;
      const int nw = (int)std::round(full.w * factor), nh = (int)std::round(full.h * factor);
      std::vector<float> f(full.px.begin(), full.px.end()), g((size_t)nw * nh);
      if (!stage_resize_linear(dev, f.data(), full.w, full.h, g.data(), nw, nh, err)) return false;
      std::vector<uint8_t> s(g.size());
      for (size_t i = 0; i < g.size(); ++i) s[i] = sat_u8(cv_round(g[i]));
      Mat m;
      if (!edge_segment(scale, s.data(), nw, nh, 0, true, high_res, m, err, dev)) return false;
      if (!write_bin_mat(ep.string(), m, err)) return false;
    }
  }
  if (use_label) {
    const fs::path lp = rf / ("labels_" + std::to_string(scale) + ".dmb");
    if (!fs::exists(lp)) {
      Mat m;
      if (!edge_segment(scale, full.px.data(), full.w, full.h, 1, false, high_res, m, err, dev)) return false;
      if (!write_bin_mat(lp.string(), m, err)) return false;
    }
  }
  return true;
}

}  // namespace dpe_host

extern "C" {

int dpe_host_canny(const uint8_t* src, int w, int h, double low, double high, uint8_t* dst) {
  if (!src || !dst || w < 1 || h < 1) return 1;
  dpe_host::canny_l2(src, w, h, low, high, dst);
  return 0;
}

int dpe_host_resize_u8(const uint8_t* src, int w, int h, uint8_t* dst, int nw, int nh) {
  if (!src || !dst || w < 1 || h < 1 || nw < 1 || nh < 1) return 1;
  dpe_host::resize_u8(src, w, h, dst, nw, nh);
  return 0;
}

int dpe_host_connect(const uint8_t* img, int w, int h, int* label, int* cnt, int cnt_cap) {
  if (!img || !label || w < 1 || h < 1) return -1;
  std::vector<int> c;
  dpe_host::connect(img, w, h, label, c);
  if (cnt) for (int i = 0; i < cnt_cap && i < (int)c.size(); ++i) cnt[i] = c[i];
  return (int)c.size();
}

int dpe_host_hough_lines_p(const uint8_t* img, int w, int h, double rho, double theta, int threshold, double min_len,
                           double max_gap, int* lines, int cap) {
  if (!img || w < 1 || h < 1) return -1;
  std::vector<std::array<int, 4>> l;
  dpe_host::hough_lines_p(img, w, h, rho, theta, threshold, min_len, max_gap, l);
  if (lines) for (int i = 0; i < cap && i < (int)l.size(); ++i) for (int k = 0; k < 4; ++k) lines[4 * i + k] = l[i][k];
  return (int)l.size();
}

int dpe_host_edge_segment(int scale, const uint8_t* src, int w, int h, int mode, int use_canny, int high_res, void* out,
                          size_t cap, int* ow, int* oh) {
  dpe_host::Mat m;
  std::string err;
  if (!src || !dpe_host::edge_segment(scale, src, w, h, mode, use_canny != 0, high_res != 0, m, err)) return 1;
  if (ow) *ow = m.cols;
  if (oh) *oh = m.rows;
  if (out) {
    if (cap < m.data.size()) return 2;
    std::memcpy(out, m.data.data(), m.data.size());
  }
  return 0;
}

}  // extern "C"
