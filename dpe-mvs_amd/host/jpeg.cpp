// jpeg.cpp — baseline / extended-sequential JPEG decoder: the luma plane, or BGR colour.
//
// Stands in for cv::imread(path, IMREAD_GRAYSCALE) (DPE.cpp:745, 755; main.cpp:316, 337), which
// asks libjpeg for JCS_GRAYSCALE output: the decoded Y component, no colour conversion; and for
// cv::imread(path, IMREAD_COLOR) (RunFusion, DPE.cpp:1253): libjpeg's default "fancy" triangular
// chroma upsampling (h2v1 / h2v2, edge rows and columns replicated) and its fixed-point YCbCr->RGB
// tables (16-bit scale, round half up), delivered as BGR.  The
// inverse DCT is the IJG "islow" integer algorithm (the libjpeg / libjpeg-turbo default), written
// from its published description: Loeffler-Ligtenberg-Moschytz 8-point IDCT, 13-bit constants,
// 2 extra bits of precision between the column and row passes, descale with rounding, +128 and
// clamp.  tests/test_host.py checks the output bit-for-bit against PIL (libjpeg-turbo) on
// grey, 4:4:4 and 4:2:0 colour files with and without restart intervals.
//
// Supported: 8-bit SOF0/SOF1 Huffman-coded, 1 or 3 components, any sampling factors where the
// first (luma) component has the largest ones, restart markers.  Progressive / arithmetic /
// 12-bit / lossless files are rejected with an error (the reference's datasets are baseline).
#include "host.h"

#include <cstdio>
#include <cstring>

namespace dpe_host {
namespace {

struct Huff {
  // canonical Huffman table: for each code length, the first code, count and value offset
  int mincode[17], maxcode[18], valptr[17];
  uint8_t vals[256];
  bool present = false;
};

struct Comp {
  int id, h, v, tq, td, ta;
  int bw, bh;          // blocks per line / column of the component (padded to the MCU grid)
  int dc_pred;
};

struct Reader {
  const uint8_t* p;
  size_t n, pos = 0;
  uint32_t bitbuf = 0;
  int bits = 0;
  bool marker_hit = false;
  int byte() { return pos < n ? p[pos++] : -1; }
  int u16() { int a = byte(), b = byte(); return (a < 0 || b < 0) ? -1 : (a << 8) | b; }
  // entropy-coded segment bit reader (0xFF00 stuffing; a marker stops the stream: zeros are fed)
  void fill() {
    while (bits <= 24) {
      int c = 0;
      if (!marker_hit) {
        if (pos >= n) { marker_hit = true; }
        else {
          c = p[pos];
          if (c == 0xFF) {
            const int c2 = pos + 1 < n ? p[pos + 1] : 0;
            if (c2 == 0x00) { pos += 2; }
            else { marker_hit = true; c = 0; }
          } else {
            pos++;
          }
        }
      }
      bitbuf |= (uint32_t)(c & 0xFF) << (24 - bits);
      bits += 8;
    }
  }
  int getbits(int k) {
    if (k == 0) return 0;
    fill();
    const int v = (int)(bitbuf >> (32 - k));
    bitbuf <<= k; bits -= k;
    return v;
  }
  int getbit() { return getbits(1); }
  void reset_bits() { bitbuf = 0; bits = 0; marker_hit = false; }
};

int decode_huff(Reader& r, const Huff& h) {
  int code = 0;
  for (int l = 1; l <= 16; ++l) {
    code = (code << 1) | r.getbit();
    if (h.maxcode[l] >= 0 && code <= h.maxcode[l] && code >= h.mincode[l]) return h.vals[h.valptr[l] + code - h.mincode[l]];
  }
  return -1;   // corrupt
}

int extend(int v, int t) { return (t == 0) ? 0 : (v < (1 << (t - 1)) ? v - (1 << t) + 1 : v); }

const int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                         12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                         35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                         58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// ---- islow IDCT
constexpr int CONST_BITS = 13, PASS1_BITS = 2;
constexpr int64_t F_0_298631336 = 2446, F_0_390180644 = 3196, F_0_541196100 = 4433, F_0_765366865 = 6270,
                  F_0_899976223 = 7373, F_1_175875602 = 9633, F_1_501321110 = 12299, F_1_847759065 = 15137,
                  F_1_961570560 = 16069, F_2_053119869 = 16819, F_2_562915447 = 20995, F_3_072711026 = 25172;
inline int64_t descale(int64_t x, int n) { return (x + ((int64_t)1 << (n - 1))) >> n; }
inline uint8_t clamp8(int64_t v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

void idct_islow(const int* coef /* dequantised, natural order */, uint8_t* out, int stride) {
  int64_t ws[64];
  for (int c = 0; c < 8; ++c) {                     // pass 1: columns
    const int* in = coef + c;
    if (in[8] == 0 && in[16] == 0 && in[24] == 0 && in[32] == 0 && in[40] == 0 && in[48] == 0 && in[56] == 0) {
      const int64_t dc = (int64_t)in[0] * (1 << PASS1_BITS);   // LEFT_SHIFT as a multiply: no UB on negatives
      for (int r = 0; r < 8; ++r) ws[r * 8 + c] = dc;
      continue;
    }
    int64_t z2 = in[16], z3 = in[48];
    int64_t z1 = (z2 + z3) * F_0_541196100;
    int64_t tmp2 = z1 + z3 * (-F_1_847759065);
    int64_t tmp3 = z1 + z2 * F_0_765366865;
    z2 = in[0]; z3 = in[32];
    int64_t tmp0 = (z2 + z3) * ((int64_t)1 << CONST_BITS);
    int64_t tmp1 = (z2 - z3) * ((int64_t)1 << CONST_BITS);
    const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    tmp0 = in[56]; tmp1 = in[40]; tmp2 = in[24]; tmp3 = in[8];
    z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2;
    int64_t z4 = tmp1 + tmp3;
    const int64_t z5 = (z3 + z4) * F_1_175875602;
    tmp0 *= F_0_298631336; tmp1 *= F_2_053119869; tmp2 *= F_3_072711026; tmp3 *= F_1_501321110;
    z1 *= -F_0_899976223; z2 *= -F_2_562915447; z3 *= -F_1_961570560; z4 *= -F_0_390180644;
    z3 += z5; z4 += z5;
    tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
    constexpr int s = CONST_BITS - PASS1_BITS;
    ws[0 * 8 + c] = descale(tmp10 + tmp3, s); ws[7 * 8 + c] = descale(tmp10 - tmp3, s);
    ws[1 * 8 + c] = descale(tmp11 + tmp2, s); ws[6 * 8 + c] = descale(tmp11 - tmp2, s);
    ws[2 * 8 + c] = descale(tmp12 + tmp1, s); ws[5 * 8 + c] = descale(tmp12 - tmp1, s);
    ws[3 * 8 + c] = descale(tmp13 + tmp0, s); ws[4 * 8 + c] = descale(tmp13 - tmp0, s);
  }
  for (int r = 0; r < 8; ++r) {                     // pass 2: rows
    const int64_t* w = ws + r * 8;
    uint8_t* o = out + r * stride;
    constexpr int s = CONST_BITS + PASS1_BITS + 3;
    if (w[1] == 0 && w[2] == 0 && w[3] == 0 && w[4] == 0 && w[5] == 0 && w[6] == 0 && w[7] == 0) {
      const uint8_t v = clamp8(descale(w[0], PASS1_BITS + 3) + 128);
      for (int c = 0; c < 8; ++c) o[c] = v;
      continue;
    }
    int64_t z2 = w[2], z3 = w[6];
    int64_t z1 = (z2 + z3) * F_0_541196100;
    int64_t tmp2 = z1 + z3 * (-F_1_847759065);
    int64_t tmp3 = z1 + z2 * F_0_765366865;
    int64_t tmp0 = (w[0] + w[4]) * ((int64_t)1 << CONST_BITS);
    int64_t tmp1 = (w[0] - w[4]) * ((int64_t)1 << CONST_BITS);
    const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    tmp0 = w[7]; tmp1 = w[5]; tmp2 = w[3]; tmp3 = w[1];
    z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2;
    int64_t z4 = tmp1 + tmp3;
    const int64_t z5 = (z3 + z4) * F_1_175875602;
    tmp0 *= F_0_298631336; tmp1 *= F_2_053119869; tmp2 *= F_3_072711026; tmp3 *= F_1_501321110;
    z1 *= -F_0_899976223; z2 *= -F_2_562915447; z3 *= -F_1_961570560; z4 *= -F_0_390180644;
    z3 += z5; z4 += z5;
    tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
    o[0] = clamp8(descale(tmp10 + tmp3, s) + 128); o[7] = clamp8(descale(tmp10 - tmp3, s) + 128);
    o[1] = clamp8(descale(tmp11 + tmp2, s) + 128); o[6] = clamp8(descale(tmp11 - tmp2, s) + 128);
    o[2] = clamp8(descale(tmp12 + tmp1, s) + 128); o[5] = clamp8(descale(tmp12 - tmp1, s) + 128);
    o[3] = clamp8(descale(tmp13 + tmp0, s) + 128); o[4] = clamp8(descale(tmp13 - tmp0, s) + 128);
  }
}

}  // namespace

namespace {
// fancy upsampling of one chroma plane (jdsample.c h2v1 / h2v2), replication for other ratios
void upsample_plane(const std::vector<uint8_t>& P, int st, int dw, int dh, int fx, int fy, int W, int H,
                    std::vector<uint8_t>& out) {
  out.assign((size_t)W * H, 0);
  auto at = [&](int x, int y) { return (int)P[(size_t)y * st + x]; };
  if (fx == 1 && fy == 1) {
    for (int y = 0; y < H; ++y) for (int x = 0; x < W; ++x) out[(size_t)y * W + x] = (uint8_t)at(x, y);
    return;
  }
  std::vector<int> row((size_t)2 * dw + 2);
  if (fx == 2 && fy == 1) {
    for (int y = 0; y < H && y < dh; ++y) {
      int* o = row.data();
      int v = at(0, y);
      *o++ = v;
      *o++ = (v * 3 + at(1, y) + 2) >> 2;
      for (int i = 1; i <= dw - 2; ++i) {
        v = at(i, y) * 3;
        *o++ = (v + at(i - 1, y) + 1) >> 2;
        *o++ = (v + at(i + 1, y) + 2) >> 2;
      }
      const int i = dw - 1;
      v = at(i, y);
      *o++ = (v * 3 + at(i > 0 ? i - 1 : 0, y) + 1) >> 2;
      *o++ = v;
      for (int x = 0; x < W; ++x) out[(size_t)y * W + x] = (uint8_t)row[x];
    }
    return;
  }
  if (fx == 2 && fy == 2) {
    for (int yi = 0; yi < dh; ++yi)
      for (int v = 0; v < 2; ++v) {
        const int oy = 2 * yi + v;
        if (oy >= H) break;
        const int y1 = v == 0 ? (yi > 0 ? yi - 1 : 0) : (yi + 1 < dh ? yi + 1 : dh - 1);   // context rows replicated
        auto cs = [&](int x) { return at(x, yi) * 3 + at(x, y1); };
        int* o = row.data();
        int thiscs = cs(0), nextcs = cs(1);
        *o++ = (thiscs * 4 + 8) >> 4;
        *o++ = (thiscs * 3 + nextcs + 7) >> 4;
        int lastcs = thiscs; thiscs = nextcs;
        for (int i = 2; i <= dw - 1; ++i) {
          nextcs = cs(i);
          *o++ = (thiscs * 3 + lastcs + 8) >> 4;
          *o++ = (thiscs * 3 + nextcs + 7) >> 4;
          lastcs = thiscs; thiscs = nextcs;
        }
        *o++ = (thiscs * 3 + lastcs + 8) >> 4;
        *o++ = (thiscs * 4 + 7) >> 4;
        for (int x = 0; x < W; ++x) out[(size_t)oy * W + x] = (uint8_t)row[x];
      }
    return;
  }
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) out[(size_t)y * W + x] = (uint8_t)at(std::min(x / fx, dw - 1), std::min(y / fy, dh - 1));
}
}  // namespace

bool decode_jpeg(const uint8_t* data, size_t size, bool color, GrayImage* gray, ColorImage* bgr, std::string& err) {
  Reader r{data, size};
  if (r.u16() != 0xFFD8) { err = "not a JPEG file"; return false; }
  uint16_t qt[4][64];
  bool qt_ok[4] = {false, false, false, false};
  Huff hdc[4], hac[4];
  std::vector<Comp> comps;
  int W = 0, H = 0, restart = 0, hmax = 1, vmax = 1;
  for (;;) {
    int m = r.byte();
    while (m == 0xFF) m = r.byte();
    if (m < 0) { err = "truncated JPEG"; return false; }
    if (m == 0xD9) { err = "no scan"; return false; }
    if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
    const int len = r.u16();
    if (len < 2 || r.pos + len - 2 > size) { err = "bad JPEG segment"; return false; }
    const size_t end = r.pos + len - 2;
    if (m == 0xDB) {                                   // DQT
      while (r.pos < end) {
        const int pq = r.byte(), tq = pq & 15, prec = pq >> 4;
        if (tq > 3) { err = "bad DQT"; return false; }
        for (int i = 0; i < 64; ++i) qt[tq][kZigzag[i]] = (uint16_t)(prec ? r.u16() : r.byte());
        qt_ok[tq] = true;
      }
    } else if (m == 0xC4) {                            // DHT
      while (r.pos < end) {
        const int tc = r.byte(), th = tc & 15, cls = tc >> 4;
        if (th > 3 || cls > 1) { err = "bad DHT"; return false; }
        Huff& h = cls ? hac[th] : hdc[th];
        int counts[17] = {0}, total = 0;
        for (int l = 1; l <= 16; ++l) { counts[l] = r.byte(); total += counts[l]; }
        if (total > 256) { err = "bad DHT"; return false; }
        for (int i = 0; i < total; ++i) h.vals[i] = (uint8_t)r.byte();
        int code = 0, k = 0;
        for (int l = 1; l <= 16; ++l) {
          h.valptr[l] = k; h.mincode[l] = code;
          code += counts[l]; k += counts[l];
          h.maxcode[l] = counts[l] ? code - 1 : -1;
          code <<= 1;
        }
        h.maxcode[17] = 0x7FFFFFFF;
        h.present = true;
      }
    } else if (m == 0xC0 || m == 0xC1) {               // SOF0 / SOF1
      if (r.byte() != 8) { err = "only 8-bit JPEG is supported"; return false; }
      H = r.u16(); W = r.u16();
      const int nc = r.byte();
      if (nc != 1 && nc != 3) { err = "unsupported JPEG component count"; return false; }
      for (int i = 0; i < nc; ++i) {
        Comp c{};
        c.id = r.byte();
        const int hv = r.byte();
        c.h = hv >> 4; c.v = hv & 15; c.tq = r.byte();
        if (c.h < 1 || c.v < 1 || c.h > 4 || c.v > 4 || c.tq > 3) { err = "bad SOF"; return false; }
        comps.push_back(c);
        hmax = std::max(hmax, c.h); vmax = std::max(vmax, c.v);
      }
      if (nc == 1) { comps[0].h = comps[0].v = 1; hmax = vmax = 1; }   // single-component scan: 1-block MCUs
      if (comps[0].h != hmax || comps[0].v != vmax) { err = "luma must have the largest sampling factors"; return false; }
    } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      err = "progressive / arithmetic / lossless JPEG is not supported"; return false;
    } else if (m == 0xDD) {                            // DRI
      restart = r.u16();
    } else if (m == 0xDA) {                            // SOS: decode and stop
      if (comps.empty() || W <= 0 || H <= 0) { err = "SOS before SOF"; return false; }
      const int ns = r.byte();
      std::vector<int> sc(ns);
      for (int i = 0; i < ns; ++i) {
        const int cid = r.byte(), t = r.byte();
        int idx = -1;
        for (size_t k = 0; k < comps.size(); ++k) if (comps[k].id == cid) idx = (int)k;
        if (idx < 0) { err = "bad SOS component"; return false; }
        comps[idx].td = t >> 4; comps[idx].ta = t & 15;
        sc[i] = idx;
      }
      r.pos = end;
      if (ns != (int)comps.size()) { err = "non-interleaved multi-scan JPEG is not supported"; return false; }
      const int mcux = (W + 8 * hmax - 1) / (8 * hmax), mcuy = (H + 8 * vmax - 1) / (8 * vmax);
      const int lw = mcux * hmax * 8, lh = mcuy * vmax * 8;   // padded luma plane
      std::vector<uint8_t> plane((size_t)lw * lh);
      const bool chroma = color && comps.size() == 3;
      std::vector<std::vector<uint8_t>> cplane(comps.size());
      std::vector<int> cst(comps.size(), 0);
      if (chroma)
        for (size_t k = 1; k < comps.size(); ++k) {
          cst[k] = mcux * comps[k].h * 8;
          cplane[k].assign((size_t)cst[k] * mcuy * comps[k].v * 8, 0);
        }
      for (auto& c : comps) {
        c.dc_pred = 0;
        if (!qt_ok[c.tq] || !hdc[c.td].present || !hac[c.ta].present) { err = "missing JPEG table"; return false; }
      }
      int coef[64], zz[64];
      int mcus_left = restart;
      r.reset_bits();
      for (int my = 0; my < mcuy; ++my) {
        for (int mx = 0; mx < mcux; ++mx) {
          if (restart && mcus_left == 0) {             // RSTn: byte-align, skip marker, reset predictors
            r.reset_bits();
            while (r.pos + 1 < size && !(r.p[r.pos] == 0xFF && r.p[r.pos + 1] >= 0xD0 && r.p[r.pos + 1] <= 0xD7)) r.pos++;
            r.pos += 2;
            for (auto& c : comps) c.dc_pred = 0;
            mcus_left = restart;
          }
          for (int ci : sc) {
            Comp& c = comps[ci];
            for (int by = 0; by < c.v; ++by) {
              for (int bx = 0; bx < c.h; ++bx) {
                std::memset(zz, 0, sizeof(zz));
                const int t = decode_huff(r, hdc[c.td]);
                if (t < 0 || t > 11) { err = "corrupt JPEG data"; return false; }
                c.dc_pred += extend(r.getbits(t), t);
                zz[0] = c.dc_pred;
                for (int k = 1; k < 64;) {
                  const int rs = decode_huff(r, hac[c.ta]);
                  if (rs < 0) { err = "corrupt JPEG data"; return false; }
                  const int rr = rs >> 4, ss = rs & 15;
                  if (ss == 0) { if (rr == 15) { k += 16; continue; } break; }
                  k += rr;
                  if (k > 63) { err = "corrupt JPEG data"; return false; }
                  zz[k++] = extend(r.getbits(ss), ss);
                }
                if (ci != 0 && !chroma) continue;      // grey output: chroma entropy-decoded and dropped
                for (int k = 0; k < 64; ++k) coef[kZigzag[k]] = zz[k] * (int)qt[c.tq][kZigzag[k]];
                const int ox = (mx * c.h + bx) * 8, oy = (my * c.v + by) * 8;
                if (ci == 0) idct_islow(coef, plane.data() + (size_t)oy * lw + ox, lw);
                else idct_islow(coef, cplane[ci].data() + (size_t)oy * cst[ci] + ox, cst[ci]);
              }
            }
          }
          if (restart) mcus_left--;
        }
      }
      if (!color) {
        gray->w = W; gray->h = H;
        gray->px.resize((size_t)W * H);
        for (int y = 0; y < H; ++y) std::memcpy(gray->px.data() + (size_t)y * W, plane.data() + (size_t)y * lw, W);
        return true;
      }
      bgr->w = W; bgr->h = H;
      bgr->bgr.resize((size_t)W * H * 3);
      if (!chroma) {                                   // grey file: B = G = R = Y
        for (int y = 0; y < H; ++y)
          for (int x = 0; x < W; ++x) {
            const uint8_t v = plane[(size_t)y * lw + x];
            uint8_t* o = bgr->bgr.data() + 3 * ((size_t)y * W + x);
            o[0] = o[1] = o[2] = v;
          }
        return true;
      }
      std::vector<uint8_t> cb, cr;
      for (int k = 1; k <= 2; ++k) {
        const Comp& c = comps[k];
        if (hmax % c.h || vmax % c.v) { err = "unsupported chroma sampling"; return false; }
        const int dw = (W * c.h + hmax - 1) / hmax, dh = (H * c.v + vmax - 1) / vmax;
        upsample_plane(cplane[k], cst[k], dw, dh, hmax / c.h, vmax / c.v, W, H, k == 1 ? cb : cr);
      }
      // jdcolor.c build_ycc_rgb_table / ycc_rgb_convert (SCALEBITS 16)
      constexpr int SB = 16;
      constexpr int64_t HALF = (int64_t)1 << (SB - 1);
      auto FIX = [](double x) { return (int64_t)(x * (1L << SB) + 0.5); };
      int cr_r[256], cb_b[256];
      int64_t cr_g[256], cb_g[256];
      for (int i = 0; i < 256; ++i) {
        const int64_t x = i - 128;
        cr_r[i] = (int)((FIX(1.40200) * x + HALF) >> SB);
        cb_b[i] = (int)((FIX(1.77200) * x + HALF) >> SB);
        cr_g[i] = -FIX(0.71414) * x;
        cb_g[i] = -FIX(0.34414) * x + HALF;
      }
      auto lim = [](int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); };
      for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
          const size_t i = (size_t)y * W + x;
          const int Y = plane[(size_t)y * lw + x], b = cb[i], r = cr[i];
          uint8_t* o = bgr->bgr.data() + 3 * i;
          o[2] = lim(Y + cr_r[r]);
          o[1] = lim(Y + (int)((cb_g[b] + cr_g[r]) >> SB));
          o[0] = lim(Y + cb_b[b]);
        }
      return true;
    }
    r.pos = end;
  }
}

bool decode_jpeg_luma(const uint8_t* data, size_t size, GrayImage& img, std::string& err) {
  return decode_jpeg(data, size, false, &img, nullptr, err);
}
bool decode_jpeg_bgr(const uint8_t* data, size_t size, ColorImage& img, std::string& err) {
  return decode_jpeg(data, size, true, nullptr, &img, err);
}

}  // namespace dpe_host
