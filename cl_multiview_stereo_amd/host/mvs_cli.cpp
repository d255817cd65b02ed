// mvs_cli -- the reference's host program (clMVDE.cpp main + pipeline.cpp)
// on libmvs.so: camera/image loader, the SLIC -> superpixel plane sweep ->
// refinement -> fusion pipeline, and its depth-map output format.
//
//   mvs_cli --data data.txt --array 3x3 [--spixl-size 8] [--min-disp 30]
//           [--max-disp 60] [--bl-ratio 1.0359] [--out DIR] [...]
//
// data.txt lists one image path per line (relative paths are relative to the
// list file), row-major over the camera array (read_image_array,
// file_handler.cpp:30-57).  Settings mirror system_settings (header.h:55-77)
// with main()'s defaults (clMVDE.cpp:14-36).  Outputs in DIR:
//   depth.f32       float32 [V][H][W] disparity (the fused depth maps)
//   fus <k>.png     8-bit maps floor((d - min) / (max - min) * 255), clamped
//                   to [0, 255] (plot_full_image, depth_refinement.cpp:1473-1495)
//   init <k>.png    (--dump-init) the superpixel initial disparity
//   filtered.f32    (--filter) after the cross-view consistency filter
//
// Test modes (no GPU): --png-decode IN OUT.raw (RGBx bytes) and
// --png-encode-gray W H IN.raw OUT.png.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "mvs.h"
#include "png.h"

namespace {

struct Settings {  // system_settings, clMVDE.cpp:14-36 defaults
  int spixl_size = 8;
  float slic_color_weight = 0.6f;
  int array_width = 3, array_height = 3;
  int no_iter = 5;
  bool enforce_connectivity = false;
  int edge_enable = 0;  // system_settings::edge_enable (header.h:61); 2 = the intended form (mvs.h)
  int search = 0;       // mvs_slic_params::search: 1 = the 3x3 candidate loop (clcode.cl:496-516)
  int neib_hor = 1, neib_ver = 1;
  int min_disp = 30, max_disp = 60, inc = 1;
  float bl_ratio = 1.03590f;
  int kernel_size = 1080, kernel_step = 13;
  float fuse = 1.0f, gamma = 2.0f, alpha = 6.0f;
  int no_prop = 5;
  bool fusion_compat = true, filter = false, dump_init = false, quiet = false;
  int device = 0;
  std::string data = "data.txt", out = ".";
};

int usage() {
  std::fprintf(stderr,
               "usage: mvs_cli --data LIST --array WxH [--spixl-size S] [--color-weight w] [--no-iter n]\n"
               "               [--connectivity] [--edge | --edge-intended] [--search3x3] [--min-disp a] [--max-disp b] [--inc i] [--neib-hor h]\n"
               "               [--neib-ver v] [--bl-ratio r] [--kernel-size k] [--kernel-step s] [--fuse f]\n"
               "               [--gamma g] [--alpha a] [--no-prop p] [--final-state] [--filter] [--dump-init]\n"
               "               [--device d] [--out DIR] [--quiet]\n"
               "       mvs_cli --png-decode IN.png OUT.raw | --png-encode-gray W H IN.raw OUT.png\n");
  return 2;
}

bool read_file(const std::string& p, std::vector<uint8_t>& b) {
  std::ifstream f(p, std::ios::binary);
  if (!f) return false;
  b.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  return true;
}

bool write_file(const std::string& p, const void* d, size_t n) {
  FILE* f = std::fopen(p.c_str(), "wb");
  if (!f) return false;
  bool ok = std::fwrite(d, 1, n, f) == n;
  return std::fclose(f) == 0 && ok;
}

int fail(const char* what) {
  std::fprintf(stderr, "mvs_cli: %s: %s\n", what, mvs_last_error());
  return 1;
}

// plot_full_image's scaling, clamped
void to_gray(const float* d, size_t n, int lo, int hi, std::vector<uint8_t>& g) {
  g.resize(n);
  if (hi == lo) {  // one disparity level: the reference's plot divides by zero; draw a flat map
    std::fill(g.begin(), g.end(), (uint8_t)0);
    return;
  }
  for (size_t i = 0; i < n; i++) {
    float v = std::floor(((d[i] - (float)lo) / (float)(hi - lo)) * 255.0f);
    g[i] = (uint8_t)std::min(255.0f, std::max(0.0f, v));
  }
}

double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

}  // namespace

int main(int argc, char** argv) {
  Settings st;
  std::vector<std::string> args(argv + 1, argv + argc);
  // ---- codec test modes ----------------------------------------------------
  if (args.size() == 3 && args[0] == "--png-decode") {
    mvs_host::Image im;
    std::string err;
    if (!mvs_host::read_png(args[1], im, err)) {
      std::fprintf(stderr, "mvs_cli: %s\n", err.c_str());
      return 1;
    }
    std::printf("%d %d\n", im.W, im.H);
    return write_file(args[2], im.rgbx.data(), im.rgbx.size()) ? 0 : 1;
  }
  if (args.size() == 5 && args[0] == "--png-encode-gray") {
    int W = std::atoi(args[1].c_str()), H = std::atoi(args[2].c_str());
    std::vector<uint8_t> raw;
    std::string err;
    if (W <= 0 || H <= 0 || !read_file(args[3], raw) || raw.size() != (size_t)W * H) return usage();
    if (!mvs_host::write_png_gray8(args[4], W, H, raw.data(), err)) {
      std::fprintf(stderr, "mvs_cli: %s\n", err.c_str());
      return 1;
    }
    return 0;
  }
  // ---- settings ------------------------------------------------------------
  for (size_t i = 0; i < args.size(); i++) {
    const std::string& a = args[i];
    auto val = [&]() -> const char* { return i + 1 < args.size() ? args[++i].c_str() : nullptr; };
    const char* v = nullptr;
    if (a == "--connectivity") st.enforce_connectivity = true;
    else if (a == "--final-state") st.fusion_compat = false;
    else if (a == "--filter") st.filter = true;
    else if (a == "--dump-init") st.dump_init = true;
    else if (a == "--quiet") st.quiet = true;
    else if (a == "--edge") st.edge_enable = 1;  // edge_enable = true, as the reference behaves
    else if (a == "--edge-intended") st.edge_enable = 2;
    else if (a == "--search3x3") st.search = 1;
    else if (!(v = val())) return usage();
    else if (a == "--data") st.data = v;
    else if (a == "--out") st.out = v;
    else if (a == "--array") {
      if (std::sscanf(v, "%dx%d", &st.array_width, &st.array_height) != 2) return usage();
    } else if (a == "--spixl-size") st.spixl_size = std::atoi(v);
    else if (a == "--color-weight") st.slic_color_weight = (float)std::atof(v);
    else if (a == "--no-iter") st.no_iter = std::atoi(v);
    else if (a == "--min-disp") st.min_disp = std::atoi(v);
    else if (a == "--max-disp") st.max_disp = std::atoi(v);
    else if (a == "--inc") st.inc = std::atoi(v);
    else if (a == "--neib-hor") st.neib_hor = std::atoi(v);
    else if (a == "--neib-ver") st.neib_ver = std::atoi(v);
    else if (a == "--bl-ratio") st.bl_ratio = (float)std::atof(v);
    else if (a == "--kernel-size") st.kernel_size = std::atoi(v);
    else if (a == "--kernel-step") st.kernel_step = std::atoi(v);
    else if (a == "--fuse") st.fuse = (float)std::atof(v);
    else if (a == "--gamma") st.gamma = (float)std::atof(v);
    else if (a == "--alpha") st.alpha = (float)std::atof(v);
    else if (a == "--no-prop") st.no_prop = std::atoi(v);
    else if (a == "--device") st.device = std::atoi(v);
    else return usage();
  }
  if (st.inc <= 0 || st.max_disp < st.min_disp || st.array_width <= 0 || st.array_height <= 0) return usage();
  const int V = st.array_width * st.array_height;

  // ---- read_image_array (file_handler.cpp:30-57) ---------------------------
  std::vector<std::string> files;
  {
    std::ifstream lf(st.data);
    if (!lf) {
      std::fprintf(stderr, "mvs_cli: cannot open %s\n", st.data.c_str());
      return 1;
    }
    std::string dir = st.data.find('/') == std::string::npos ? "" : st.data.substr(0, st.data.rfind('/') + 1);
    std::string line;
    while (std::getline(lf, line)) {
      while (!line.empty() && (line.back() == '\r' || line.back() == ' ')) line.pop_back();
      if (line.empty()) continue;
      files.push_back(line[0] == '/' ? line : dir + line);
    }
  }
  if ((int)files.size() < V) {
    std::fprintf(stderr, "mvs_cli: %s lists %zu images, the %dx%d array needs %d\n", st.data.c_str(), files.size(),
                 st.array_width, st.array_height, V);
    return 1;
  }
  std::vector<mvs_host::Image> imgs(V);
  for (int v = 0; v < V; v++) {
    std::string err;
    if (!mvs_host::read_png(files[v], imgs[v], err)) {
      std::fprintf(stderr, "mvs_cli: %s\n", err.c_str());
      return 1;
    }
    if (imgs[v].W != imgs[0].W || imgs[v].H != imgs[0].H) {
      std::fprintf(stderr, "mvs_cli: %s: image size differs from the first view\n", files[v].c_str());
      return 1;
    }
  }
  const int W = imgs[0].W, H = imgs[0].H, S = st.spixl_size;
  const int mw = (int)std::ceil((float)W / (float)S), mh = (int)std::ceil((float)H / (float)S);  // pipeline.cpp:18-19
  const size_t P = (size_t)W * H, M = (size_t)mw * mh;

  mvs_ctx* ctx = nullptr;
  if (mvs_create(st.device, &ctx) != MVS_OK) return fail("mvs_create");

  // ---- pipeline::perform_segmentation (pipeline.cpp:67-101) ----------------
  std::vector<float> lab(V * P * 4), spixl(V * M * 8, 0.0f);
  std::vector<uint32_t> labels(V * P);
  mvs_slic_params sp{sizeof(mvs_slic_params), S, st.slic_color_weight, st.no_iter,
                     st.enforce_connectivity ? 1 : 0, st.edge_enable, st.search};
  for (int v = 0; v < V; v++) {
    auto t0 = std::chrono::steady_clock::now();
    if (mvs_do_super_pixel_seg(ctx, imgs[v].rgbx.data(), W, H, &sp, &lab[v * P * 4], &spixl[v * M * 8],
                               &labels[v * P]) != MVS_OK)
      return fail("mvs_do_super_pixel_seg");
    if (!st.quiet) std::printf("Time of SLIC = %.3f ms\n", ms_since(t0));
  }

  // ---- pipeline::perform_depth_est (pipeline.cpp:108-151) ------------------
  std::vector<float> levels;
  for (int i = 0; i <= (st.max_disp - st.min_disp) / st.inc; i++) levels.push_back((float)(st.min_disp + i * st.inc));
  std::vector<int32_t> vs((size_t)V * V, 0), sn(V, 0);
  for (int i = 0; i < V; i++) {
    int n = 0;
    for (int x = i % st.array_width - st.neib_hor; x <= i % st.array_width + st.neib_hor; x++)
      for (int y = i / st.array_width - st.neib_ver; y <= i / st.array_width + st.neib_ver; y++) {
        int idx = y * st.array_width + x;
        if (x >= 0 && x < st.array_width && y >= 0 && y < st.array_height && idx != i) vs[(size_t)i * V + n++] = idx;
      }
    sn[i] = n;
  }
  mvs_array arr{V, st.array_width, st.bl_ratio, levels.data(), (int)levels.size(), vs.data(), sn.data()};
  std::vector<uint8_t> rep(V * M * 8);
  auto t1 = std::chrono::steady_clock::now();
  if (mvs_do_initial_depth_estimation(ctx, W, H, S, spixl.data(), rep.data(), lab.data(), labels.data(), &arr) !=
      MVS_OK)
    return fail("mvs_do_initial_depth_estimation");
  if (!st.quiet) std::printf("Time of initial depth estimation = %.3f ms\n", ms_since(t1));

  std::vector<float> disp(V * P);
  mvs_refine_params rp{sizeof(mvs_refine_params), st.gamma, st.alpha, st.fuse, st.kernel_step, st.kernel_size,
                       st.no_prop, st.fusion_compat ? 1 : 0, 0};
  auto t2 = std::chrono::steady_clock::now();
  if (mvs_do_refinement(ctx, W, H, S, spixl.data(), labels.data(), rep.data(), &arr, &rp, nullptr, disp.data()) !=
      MVS_OK)
    return fail("mvs_do_refinement");
  if (!st.quiet) std::printf("Time of refinement + fusion = %.3f ms\n", ms_since(t2));

  // ---- outputs -------------------------------------------------------------
  const std::string od = st.out + "/";
  if (!write_file(od + "depth.f32", disp.data(), disp.size() * sizeof(float))) {
    std::fprintf(stderr, "mvs_cli: cannot write %sdepth.f32\n", od.c_str());
    return 1;
  }
  std::vector<uint8_t> g;
  std::string err;
  for (int v = 0; v < V; v++) {
    to_gray(&disp[v * P], P, st.min_disp, st.max_disp, g);
    if (!mvs_host::write_png_gray8(od + "fus " + std::to_string(v) + ".png", W, H, g.data(), err)) {
      std::fprintf(stderr, "mvs_cli: %s\n", err.c_str());
      return 1;
    }
  }
  if (st.dump_init) {
    std::vector<float> init(P);
    for (int v = 0; v < V; v++) {
      for (size_t p = 0; p < P; p++) init[p] = spixl[(v * M + labels[v * P + p]) * 8 + 7];
      to_gray(init.data(), P, st.min_disp, st.max_disp, g);
      if (!mvs_host::write_png_gray8(od + "init " + std::to_string(v) + ".png", W, H, g.data(), err)) {
        std::fprintf(stderr, "mvs_cli: %s\n", err.c_str());
        return 1;
      }
    }
  }
  if (st.filter) {
    std::vector<float> filt(V * P);
    if (mvs_do_consistency_filter(ctx, V, W, H, st.array_width, st.bl_ratio, st.fuse, disp.data(), filt.data()) !=
        MVS_OK)
      return fail("mvs_do_consistency_filter");
    if (!write_file(od + "filtered.f32", filt.data(), filt.size() * sizeof(float))) return 1;
  }
  mvs_destroy(ctx);
  if (!st.quiet) std::printf("wrote %d depth maps (%dx%d) to %s\n", V, W, H, st.out.c_str());
  return 0;
}
