// hostio.cpp — file formats and resampling of the host pipeline.
//   .dmb      ReadBinMat / WriteBinMat (DPE.cpp:293-339)
//   .npy      WriteMatToNpy (main.cpp:47-96)
//   cams      ReadCamera (DPE.cpp:341-382)
//   images    cv::imread(IMREAD_GRAYSCALE): JPEG luma (jpeg.cpp) or binary PGM
//   resize    cv::resize INTER_LINEAR, float path (DPE.cpp:798-822)
//   rescale   RescaleMatToTargetSize (DPE.cpp:1146-1168), swapped x/y factors kept
#include "host.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>

namespace dpe_host {

std::string fmt_index(int i) {
  char b[32];
  std::snprintf(b, sizeof(b), "%08d", i);
  return b;
}

int Mat::elem_size(int type) {
  switch (type) {
    case CV_8UC1: case CV_8SC1: return 1;
    case CV_32SC1: case CV_32FC1: return 4;
    case CV_32FC3: return 12;
    default: return 0;
  }
}

bool read_bin_mat(const std::string& path, Mat& m, std::string& err) {
  std::ifstream in(path, std::ios::binary);
  if (!in) { err = "Error opening file: " + path; return false; }
  int32_t hdr[4];
  if (!in.read(reinterpret_cast<char*>(hdr), sizeof(hdr))) { err = "truncated .dmb header: " + path; return false; }
  if (hdr[0] != 1) { err = "Version error: " + path; return false; }
  if (Mat::elem_size(hdr[3]) == 0 || hdr[1] < 0 || hdr[2] < 0) { err = "unsupported .dmb type: " + path; return false; }
  m.create(hdr[1], hdr[2], hdr[3]);
  if (!in.read(reinterpret_cast<char*>(m.data.data()), (std::streamsize)m.data.size())) {
    err = "truncated .dmb data: " + path; return false;
  }
  return true;
}

bool write_bin_mat(const std::string& path, const Mat& m, std::string& err) {
  std::ofstream out(path, std::ios::binary);
  if (!out) { err = "Error opening file: " + path; return false; }
  const int32_t hdr[4] = {1, m.rows, m.cols, m.type};
  out.write(reinterpret_cast<const char*>(hdr), sizeof(hdr));
  out.write(reinterpret_cast<const char*>(m.data.data()), (std::streamsize)m.data.size());
  if (!out) { err = "write failed: " + path; return false; }
  return true;
}

bool write_npy(const std::string& path, const void* data, const std::vector<int64_t>& shape, const char* descr,
               size_t elem, std::string& err) {
  std::string sh = "(";
  size_t n = 1;
  for (size_t i = 0; i < shape.size(); ++i) {
    sh += std::to_string(shape[i]);
    if (i + 1 < shape.size()) sh += ", ";
    n *= (size_t)shape[i];
  }
  if (shape.size() == 1) sh += ",";
  sh += ")";
  std::string header = std::string("{'descr': '") + descr + "', 'fortran_order': False, 'shape': " + sh + ", }";
  const size_t padding = (16 - ((10 + header.size() + 1) % 16)) % 16;
  header.append(padding, ' ');
  header.push_back('\n');
  std::ofstream out(path, std::ios::binary);
  if (!out) { err = "Failed to open npy for writing: " + path; return false; }
  out.write("\x93NUMPY", 6);
  out.put(1); out.put(0);
  const uint16_t hl = (uint16_t)header.size();
  out.write(reinterpret_cast<const char*>(&hl), 2);
  out.write(header.data(), (std::streamsize)header.size());
  out.write(reinterpret_cast<const char*>(data), (std::streamsize)(n * elem));
  if (!out) { err = "Failed while writing npy: " + path; return false; }
  return true;
}

bool read_camera(const std::string& path, DpeCamera& cam, std::string& err) {
  std::ifstream in(path);
  if (!in) { err = "Error opening camera: " + path; return false; }
  std::memset(&cam, 0, sizeof(cam));
  std::string word;
  in >> word;                                        // "extrinsic"
  for (int i = 0; i < 3; ++i) in >> cam.R[3 * i + 0] >> cam.R[3 * i + 1] >> cam.R[3 * i + 2] >> cam.t[i];
  float tmp[4];
  in >> tmp[0] >> tmp[1] >> tmp[2] >> tmp[3];
  in >> word;                                        // "intrinsic"
  for (int i = 0; i < 3; ++i) in >> cam.K[3 * i + 0] >> cam.K[3 * i + 1] >> cam.K[3 * i + 2];
  if (!in) { err = "malformed camera file: " + path; return false; }
  for (int j = 0; j < 3; ++j)   // camera centre -R^T t, products in double
    cam.c[j] = -(float)((double)cam.R[0 + j] * (double)cam.t[0] + (double)cam.R[3 + j] * (double)cam.t[1] +
                        (double)cam.R[6 + j] * (double)cam.t[2]);
  float interval = 0, depth_num = 0;
  cam.depth_min = cam.depth_max = 0;                 // a failed extraction leaves 0 (C++11 streams)
  in >> cam.depth_min >> interval >> depth_num >> cam.depth_max;
  if (in.fail()) { /* 2-number DTU line: depth_max stays 0 */ }
  return true;
}

bool read_gray(const std::string& path, GrayImage& img, std::string& err) {
  std::ifstream in(path, std::ios::binary);
  if (!in) { err = "cannot read image: " + path; return false; }
  std::vector<uint8_t> buf((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  if (buf.size() >= 2 && buf[0] == 0xFF && buf[1] == 0xD8) {
    if (!decode_jpeg_luma(buf.data(), buf.size(), img, err)) { err = path + ": " + err; return false; }
    return true;
  }
  if (buf.size() >= 2 && buf[0] == 'P' && buf[1] == '5') {      // binary 8-bit PGM
    std::istringstream hs(std::string(buf.begin(), buf.begin() + std::min<size_t>(buf.size(), 256)));
    std::string magic; int w, h, maxv;
    hs >> magic >> w >> h >> maxv;
    const size_t off = (size_t)hs.tellg() + 1;
    if (!hs || maxv > 255 || off + (size_t)w * h > buf.size()) { err = "bad PGM: " + path; return false; }
    img.w = w; img.h = h;
    img.px.assign(buf.begin() + off, buf.begin() + off + (size_t)w * h);
    return true;
  }
  err = "unsupported image format (JPEG or binary PGM expected): " + path;
  return false;
}

bool read_bgr(const std::string& path, ColorImage& img, std::string& err) {   // cv::imread(IMREAD_COLOR)
  std::ifstream in(path, std::ios::binary);
  if (!in) { err = "cannot read image: " + path; return false; }
  std::vector<uint8_t> buf((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  if (buf.size() >= 2 && buf[0] == 0xFF && buf[1] == 0xD8) {
    if (!decode_jpeg_bgr(buf.data(), buf.size(), img, err)) { err = path + ": " + err; return false; }
    return true;
  }
  GrayImage g;
  if (!read_gray(path, g, err)) return false;
  img.w = g.w; img.h = g.h;
  img.bgr.resize(g.px.size() * 3);
  for (size_t i = 0; i < g.px.size(); ++i) img.bgr[3 * i] = img.bgr[3 * i + 1] = img.bgr[3 * i + 2] = g.px[i];
  return true;
}

namespace {
struct Taps { std::vector<int> s0, s1; std::vector<float> a0, a1; };
Taps linear_taps(int n_src, int n_dst) {
  Taps t;
  t.s0.resize(n_dst); t.s1.resize(n_dst); t.a0.resize(n_dst); t.a1.resize(n_dst);
  const double scale = 1.0 / ((double)n_dst / n_src);
  for (int d = 0; d < n_dst; ++d) {
    float f = (float)((d + 0.5) * scale - 0.5);
    int s = (int)std::floor(f);
    f -= (float)s;
    if (s < 0) { f = 0; s = 0; }
    if (s >= n_src - 1) { f = 0; s = n_src - 1; }
    t.s0[d] = s; t.s1[d] = std::min(s + 1, n_src - 1);
    t.a0[d] = 1.0f - f; t.a1[d] = f;
  }
  return t;
}
}  // namespace

void resize_linear(const float* src, int w, int h, float* dst, int nw, int nh) {
  if (w == nw && h == nh) { std::memcpy(dst, src, sizeof(float) * (size_t)w * h); return; }
  const Taps tx = linear_taps(w, nw), ty = linear_taps(h, nh);
  std::vector<float> rows((size_t)h * nw);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < nw; ++x) {
      const float* s = src + (size_t)y * w;
      const float p = s[tx.s0[x]] * tx.a0[x];
      const float q = s[tx.s1[x]] * tx.a1[x];
      rows[(size_t)y * nw + x] = p + q;
    }
  for (int y = 0; y < nh; ++y)
    for (int x = 0; x < nw; ++x) {
      const float p = rows[(size_t)ty.s0[y] * nw + x] * ty.a0[y];
      const float q = rows[(size_t)ty.s1[y] * nw + x] * ty.a1[y];
      dst[(size_t)y * nw + x] = p + q;
    }
}

void rescale_nearest(const void* src, int w, int h, void* dst, int nw, int nh, int elem) {
  const float scale_x = nw / (float)w, scale_y = nh / (float)h;
  const uint8_t* s = static_cast<const uint8_t*>(src);
  uint8_t* d = static_cast<uint8_t*>(dst);
  for (int r = 0; r < nh; ++r)
    for (int c = 0; c < nw; ++c) {
      const int o_r = (int)(r / scale_x), o_c = (int)(c / scale_y);   // swapped factors (DPE.cpp:1157-1158)
      if (o_r < 0 || o_c < 0 || o_r >= h || o_c >= w) continue;
      std::memcpy(d + ((size_t)r * nw + c) * elem, s + ((size_t)o_r * w + o_c) * elem, elem);
    }
}

}  // namespace dpe_host

extern "C" {

int dpe_host_read_gray(const char* path, uint8_t* out, size_t cap, int* w, int* h) {
  dpe_host::GrayImage img;
  std::string err;
  if (!dpe_host::read_gray(path, img, err)) return -1;
  if (w) *w = img.w;
  if (h) *h = img.h;
  if (out && cap) std::memcpy(out, img.px.data(), std::min(cap, img.px.size()));
  return 0;
}

int dpe_host_read_bgr(const char* path, uint8_t* out, size_t cap, int* w, int* h) {
  dpe_host::ColorImage img;
  std::string err;
  if (!path || !dpe_host::read_bgr(path, img, err)) return 1;
  if (w) *w = img.w;
  if (h) *h = img.h;
  if (out) {
    if (cap < img.bgr.size()) return 2;
    std::memcpy(out, img.bgr.data(), img.bgr.size());
  }
  return 0;
}

int dpe_host_read_camera(const char* path, DpeCamera* cam) {
  std::string err;
  return dpe_host::read_camera(path, *cam, err) ? 0 : -1;
}

void dpe_host_resize_linear(const float* src, int w, int h, float* dst, int nw, int nh) {
  dpe_host::resize_linear(src, w, h, dst, nw, nh);
}

void dpe_host_rescale_nearest(const void* src, int w, int h, void* dst, int nw, int nh, int elem) {
  dpe_host::rescale_nearest(src, w, h, dst, nw, nh, elem);
}

}  // extern "C"
