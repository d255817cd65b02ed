// Minimal PNG codec on zlib for the host pipeline (mvs_cli).
//
// The reference reads its camera images with OpenCV imread and writes its
// depth maps with imwrite (file_handler.cpp:6-57, depth_refinement.cpp:1473-
// 1495); OpenCV is not part of this build, so the loader decodes the PNG
// subset those files use: 8-bit grey / grey+alpha / RGB / RGBA, non-interlaced,
// all five scanline filters.  The writer emits 8-bit greyscale.
#include "png.h"

#include <zlib.h>

#include <cstdio>
#include <cstring>
#include <new>
#include <fstream>
#include <iterator>

namespace mvs_host {
namespace {

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

void put_be32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back((uint8_t)(x >> 24));
  v.push_back((uint8_t)(x >> 16));
  v.push_back((uint8_t)(x >> 8));
  v.push_back((uint8_t)x);
}

int paeth(int a, int b, int c) {
  int p = a + b - c, pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

const uint8_t kSig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};

void chunk(std::vector<uint8_t>& out, const char* type, const uint8_t* data, size_t n) {
  put_be32(out, (uint32_t)n);
  size_t at = out.size();
  out.insert(out.end(), type, type + 4);
  if (n) out.insert(out.end(), data, data + n);
  put_be32(out, (uint32_t)crc32(0L, out.data() + at, (uInt)(n + 4)));
}

}  // namespace

bool read_png(const std::string& path, Image& img, std::string& err) {
  std::ifstream f(path, std::ios::binary);
  if (!f) {
    err = "cannot open " + path;
    return false;
  }
  std::vector<uint8_t> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (b.size() < 8 || std::memcmp(b.data(), kSig, 8) != 0) {
    err = path + ": not a PNG file";
    return false;
  }
  int W = 0, H = 0, depth = 0, ctype = -1, interlace = 0;
  std::vector<uint8_t> z;
  size_t p = 8;
  bool end = false;
  while (p + 12 <= b.size() && !end) {
    uint32_t n = be32(&b[p]);
    if (p + 12 + (size_t)n > b.size()) break;
    const char* t = (const char*)&b[p + 4];
    const uint8_t* d = &b[p + 8];
    if (!std::memcmp(t, "IHDR", 4) && n >= 13) {
      W = (int)be32(d);
      H = (int)be32(d + 4);
      depth = d[8];
      ctype = d[9];
      interlace = d[12];
    } else if (!std::memcmp(t, "IDAT", 4)) {
      z.insert(z.end(), d, d + n);
    } else if (!std::memcmp(t, "IEND", 4)) {
      end = true;
    }
    p += 12 + n;
  }
  int ch = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
  if (W <= 0 || H <= 0 || depth != 8 || ch == 0 || interlace != 0) {
    err = path + ": unsupported PNG (need 8-bit grey/RGB/RGBA, non-interlaced)";
    return false;
  }
  // the C-ABI's own limit (capi.cpp bad_dims: W*H*16 bytes of Lab < 2^31), checked
  // before anything is sized from the untrusted header
  if ((long long)W * H > (1LL << 31) / 16) {
    err = path + ": image too large (" + std::to_string(W) + "x" + std::to_string(H) + ")";
    return false;
  }
  const size_t stride = (size_t)W * ch;
  std::vector<uint8_t> raw;
  try {
    raw.resize((stride + 1) * H);
  } catch (const std::bad_alloc&) {
    err = path + ": out of host memory";
    return false;
  }
  uLongf len = (uLongf)raw.size();
  if (uncompress(raw.data(), &len, z.data(), (uLong)z.size()) != Z_OK || len != raw.size()) {
    err = path + ": corrupt image data";
    return false;
  }
  std::vector<uint8_t> px(stride * H);
  for (int y = 0; y < H; y++) {
    const uint8_t* s = &raw[(stride + 1) * y + 1];
    uint8_t* o = &px[stride * y];
    const uint8_t* up = y ? &px[stride * (y - 1)] : nullptr;
    const int ft = raw[(stride + 1) * y];
    for (size_t i = 0; i < stride; i++) {
      int a = i >= (size_t)ch ? o[i - ch] : 0, u = up ? up[i] : 0, c = (up && i >= (size_t)ch) ? up[i - ch] : 0;
      int pred = ft == 0 ? 0 : ft == 1 ? a : ft == 2 ? u : ft == 3 ? (a + u) / 2 : ft == 4 ? paeth(a, u, c) : -1;
      if (pred < 0) {
        err = path + ": bad scanline filter";
        return false;
      }
      o[i] = (uint8_t)(s[i] + pred);
    }
  }
  img.W = W;
  img.H = H;
  img.rgbx.assign((size_t)W * H * 4, 0);
  for (size_t i = 0; i < (size_t)W * H; i++) {
    const uint8_t* s = &px[i * ch];
    uint8_t* o = &img.rgbx[i * 4];
    if (ch <= 2) {
      o[0] = o[1] = o[2] = s[0];
    } else {
      o[0] = s[0];
      o[1] = s[1];
      o[2] = s[2];
    }
  }
  return true;
}

bool write_png_gray8(const std::string& path, int W, int H, const uint8_t* g, std::string& err) {
  std::vector<uint8_t> raw(((size_t)W + 1) * H);
  for (int y = 0; y < H; y++) {
    raw[((size_t)W + 1) * y] = 0;  // filter: none
    std::memcpy(&raw[((size_t)W + 1) * y + 1], g + (size_t)W * y, (size_t)W);
  }
  uLongf zl = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zl);
  if (compress2(z.data(), &zl, raw.data(), (uLong)raw.size(), 6) != Z_OK) {
    err = "deflate failed";
    return false;
  }
  std::vector<uint8_t> out(kSig, kSig + 8);
  uint8_t ihdr[13];
  const uint32_t w = (uint32_t)W, h = (uint32_t)H;
  for (int i = 0; i < 4; i++) {
    ihdr[i] = (uint8_t)(w >> (24 - 8 * i));
    ihdr[4 + i] = (uint8_t)(h >> (24 - 8 * i));
  }
  ihdr[8] = 8;   // bit depth
  ihdr[9] = 0;   // greyscale
  ihdr[10] = ihdr[11] = ihdr[12] = 0;
  chunk(out, "IHDR", ihdr, 13);
  chunk(out, "IDAT", z.data(), zl);
  chunk(out, "IEND", nullptr, 0);
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) {
    err = "cannot write " + path;
    return false;
  }
  bool ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
  ok = std::fclose(f) == 0 && ok;
  if (!ok) err = "write failed: " + path;
  return ok;
}

}  // namespace mvs_host
