// Drives clmvde_adapter.h the way the reference's pipeline drives its stage
// classes (pipeline.cpp:7-28, 68-104, 108-175): SLIC per view, levels and
// neighbour lists, initial depth, refinement with the pipeline's
// pre-squared gamma/alpha and halved kernel_size.  Test infrastructure.
//
//   pipeline_driver W H AW AH S MIN MAX BL NH NV stack.rgbx out_disp.f32 out_spixl.f32
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <vector>

#include "ref_types.h"
#include "clmvde_adapter.h"

int main(int argc, char** argv) {
  if (argc != 14) {
    std::fprintf(stderr, "usage: pipeline_driver W H AW AH S MIN MAX BL NH NV stack out_disp out_spixl\n");
    return 2;
  }
  system_settings s;  // main(), clMVDE.cpp:14-36, with the test's geometry
  int W = std::atoi(argv[1]), H = std::atoi(argv[2]);
  s.array_width = std::atoi(argv[3]);
  s.array_height = std::atoi(argv[4]);
  s.spixl_size = std::atoi(argv[5]);
  s.min_disp = std::atoi(argv[6]);
  s.max_disp = std::atoi(argv[7]);
  s.bl_ratio = (float)std::atof(argv[8]);
  s.neib_hor = std::atoi(argv[9]);
  s.neib_ver = std::atoi(argv[10]);
  s.slic_color_weight = 0.6f;
  s.no_iter = 5;
  s.inc = 1;
  s.kernel_size = 1080;
  s.kernel_step = 13;
  s.fuse = 1;
  s.gamma = 2;
  s.alpha = 6;
  s.no_prop = 5;
  int V = s.array_width * s.array_height;
  cl_int2 img{};
  img.x = W;
  img.y = H;
  cl_int2 map{};
  map.x = (int)std::ceil((float)W / (float)s.spixl_size);  // pipeline.cpp:18-19
  map.y = (int)std::ceil((float)H / (float)s.spixl_size);
  size_t P = (size_t)W * H, M = (size_t)map.x * map.y;
  std::vector<vec3u> in(V * P);
  std::ifstream f(argv[11], std::ios::binary);
  if (!f.read((char*)in.data(), (std::streamsize)(in.size() * sizeof(vec3u)))) return 1;
  std::vector<vec3f> cvt(V * P);
  std::vector<cl_uint> idx(V * P);
  std::vector<vec8f> spixl(V * M);
  cl::Program program;
  try {
    clSLIC slic(program, &s, img, map);  // pipeline.cpp:73-95
    for (int i = 0; i < V; i++) slic.do_super_pixel_seg(&in[i * P], &cvt[i * P], &spixl[i * M], &idx[i * P]);
    std::vector<float> levels;  // pipeline.cpp:121-124
    for (int i = 0; i <= (s.max_disp - s.min_disp) / s.inc; i++) levels.push_back((float)(s.min_disp + i * s.inc));
    std::vector<std::vector<int> > subset(V);  // pipeline.cpp:130-142
    for (int i = 0; i < V; i++)
      for (int x = i % s.array_width - s.neib_hor; x <= i % s.array_width + s.neib_hor; x++)
        for (int y = i / s.array_width - s.neib_ver; y <= i / s.array_width + s.neib_ver; y++) {
          int k = y * s.array_width + x;
          if (x >= 0 && x < s.array_width && y >= 0 && y < s.array_height && k != i) subset[i].push_back(k);
        }
    std::vector<vec8u> rep(V * M);
    clPhotoConsistency pc(program, V, s.spixl_size, (int)levels.size(), img, map);  // pipeline.cpp:156-157
    pc.do_initial_depth_estimation(spixl.data(), rep.data(), cvt.data(), idx.data(), s.array_width, s.bl_ratio,
                                   subset, levels);
    float gamma = (float)(2 * std::pow(s.gamma, 2));  // pipeline.cpp:164-167
    float alpha = (float)(2 * std::pow(s.alpha, 2));
    int kernel_size = s.kernel_size / 2;
    vec2i cam{};
    cam.x = s.array_width;
    cam.y = s.array_height;
    clDepthRefinement dr(program, img, map, cam, cvt.data(), spixl.data(), idx.data(), rep.data(), subset,
                         s.spixl_size, s.bl_ratio);  // pipeline.cpp:170-173
    dr.do_refinement(gamma, alpha, s.fuse, s.kernel_step, kernel_size, s.no_prop);
    std::ofstream o(argv[12], std::ios::binary);
    o.write((const char*)dr.disp(), (std::streamsize)(sizeof(float) * V * P));
    std::ofstream o2(argv[13], std::ios::binary);
    o2.write((const char*)spixl.data(), (std::streamsize)(sizeof(vec8f) * V * M));
  } catch (const std::exception& e) {
    std::fprintf(stderr, "pipeline_driver: %s\n", e.what());
    return 1;
  }
  return 0;
}
