// Minimal PNG codec for the host pipeline (see png.cpp).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace mvs_host {

struct Image {
  int W = 0, H = 0;
  std::vector<uint8_t> rgbx;  // [H][W][4], s0=R s1=G s2=B s3=0 (loadImageIn, file_handler.cpp:6-14)
};

bool read_png(const std::string& path, Image& img, std::string& err);
bool write_png_gray8(const std::string& path, int W, int H, const uint8_t* g, std::string& err);

}  // namespace mvs_host
