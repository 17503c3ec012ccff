// host.h — internal interfaces of the host pipeline (libdpe_host.so).  Plain C++17, no HIP: the
// device work goes through the C-ABI of dpe_mvs.h.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/dpe_host.h"

namespace dpe_host {

struct GrayImage {
  int w = 0, h = 0;
  std::vector<uint8_t> px;
};
bool decode_jpeg_luma(const uint8_t* data, size_t size, GrayImage& img, std::string& err);
bool read_gray(const std::string& path, GrayImage& img, std::string& err);

// cv::Mat as the .dmb files carry it: OpenCV type code + raw rows (DPE.cpp:293-339)
enum { CV_8UC1 = 0, CV_8SC1 = 1, CV_32SC1 = 4, CV_32FC1 = 5, CV_32FC3 = 21 };
struct Mat {
  int rows = 0, cols = 0, type = CV_8UC1;
  std::vector<uint8_t> data;
  static int elem_size(int type);
  void create(int r, int c, int t) { rows = r; cols = c; type = t; data.assign((size_t)r * c * elem_size(t), 0); }
  template <class T> T* ptr() { return reinterpret_cast<T*>(data.data()); }
  template <class T> const T* ptr() const { return reinterpret_cast<const T*>(data.data()); }
  bool empty() const { return rows == 0 || cols == 0; }
};
bool read_bin_mat(const std::string& path, Mat& m, std::string& err);
bool write_bin_mat(const std::string& path, const Mat& m, std::string& err);
// .npy v1.0 (main.cpp:47-96); descr "<f4" / "|i1" / "|u1"
bool write_npy(const std::string& path, const void* data, const std::vector<int64_t>& shape, const char* descr,
               size_t elem, std::string& err);

bool read_camera(const std::string& path, DpeCamera& cam, std::string& err);   // DPE.cpp:341-382

void resize_linear(const float* src, int w, int h, float* dst, int nw, int nh);
void rescale_nearest(const void* src, int w, int h, void* dst, int nw, int nh, int elem);

std::string fmt_index(int i);   // ToFormatIndex: %08d

}  // namespace dpe_host
