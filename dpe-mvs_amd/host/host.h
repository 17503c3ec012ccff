// host.h — internal interfaces of the host pipeline (libdpe_host.so).  Plain C++17, no HIP: the
// device work goes through the C-ABI of dpe_mvs.h.
#pragma once
#include <array>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/dpe_host.h"

namespace dpe_host {

struct GrayImage {
  int w = 0, h = 0;
  std::vector<uint8_t> px;
};
struct ColorImage {                 // cv::imread(IMREAD_COLOR): 8-bit BGR, row-major
  int w = 0, h = 0;
  std::vector<uint8_t> bgr;
};
bool decode_jpeg(const uint8_t* data, size_t size, bool color, GrayImage* gray, ColorImage* bgr, std::string& err);
bool decode_jpeg_luma(const uint8_t* data, size_t size, GrayImage& img, std::string& err);
bool decode_jpeg_bgr(const uint8_t* data, size_t size, ColorImage& img, std::string& err);
bool read_gray(const std::string& path, GrayImage& img, std::string& err);
bool read_bgr(const std::string& path, ColorImage& img, std::string& err);

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

// edges.cpp: EdgeSegment and the OpenCV operations it uses (DPE.cpp:9-291, main.cpp:331-388)
void resize_u8(const uint8_t* src, int w, int h, uint8_t* dst, int nw, int nh);
void threshold_binary(uint8_t* img, size_t n, int thr);
void canny_l2(const uint8_t* src, int w, int h, double low, double high, uint8_t* dst);
void roberts(const uint8_t* src, int w, int h, uint8_t* dst);
void connect(const uint8_t* img, int w, int h, int* label, std::vector<int>& label_cnt);
void draw_line(uint8_t* img, int w, int h, int x0, int y0, int x1, int y1, uint8_t value);
void hough_lines_p(const uint8_t* img, int w, int h, double rho, double theta, int threshold, double min_len,
                   double max_gap, std::vector<std::array<int, 4>>& lines);
// The device for EdgeSegment's data-parallel stages (dpe_resize_linear / dpe_resize_u8 / dpe_canny /
// dpe_roberts_threshold, bit-identical to the host functions above): one context shared by the host
// threads behind `mu`.  ctx == nullptr: every stage on the host.
struct EdgeDevice {
  DpeContext* ctx = nullptr;
  std::mutex* mu = nullptr;
};
bool edge_segment(int scale, const uint8_t* src, int cols, int rows, int mode, bool use_canny, bool high_res, Mat& out,
                  std::string& err, const EdgeDevice* dev = nullptr);
bool get_problem_edges(const GrayImage& full, int scale_size, const std::string& result_folder, bool use_edge,
                       bool use_label, bool high_res, std::string& err, const EdgeDevice* dev = nullptr);

// fusion.cpp: RunFusion (DPE.cpp:1220-1370) / ExportPointCloud (DPE.cpp:532-572)
struct FusionView {
  int image_id = 0;
  std::vector<int> src_ids;          // pair.txt order
  DpeFusionView view{};              // size, camera, depth, normal (borrowed pointers)
  const uint8_t* weak = nullptr;     // PixelState [H][W]
  std::vector<uint8_t> bgr;          // colour image at the map size
  std::vector<uint8_t> block;        // blocks/mask_<id>.jpg at the map size, or empty
  std::vector<uint8_t> mask;         // fusion masks (set by run_fusion)
};
struct FusedPoint { float x, y, z, b, g, r; };
bool run_fusion(std::vector<FusionView>& views, dpe_fusion_fn fn, void* user, std::vector<FusedPoint>& cloud,
                std::string& err);
FusedPoint fusion_point(int x, int y, float depth, const DpeCamera& cam, const float* bgr);
bool export_point_cloud(const std::string& path, const std::vector<FusedPoint>& cloud, std::string& err);

}  // namespace dpe_host
