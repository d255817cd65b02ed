// Test-only declarations of the host types the reference's stage classes use
// (OpenCL C++ wrapper types and clMVDE's system_settings, header.h:55-77), so
// that cl_multiview_stereo_amd/host/clmvde_adapter.h can be compiled and run
// without OpenCL / OpenCV.  Layouts follow the OpenCL host ABI: cl_int2 is
// 8 B, cl_uchar3 4 B, cl_float3 16 B, cl_float8 32 B, cl_uchar8 8 B.
#pragma once
#include <cstdint>

typedef uint32_t cl_uint;
typedef union { int32_t s[2]; struct { int32_t x, y; }; } cl_int2;
typedef union { uint8_t s[4]; struct { uint8_t x, y, z, w; }; } cl_uchar3;
typedef union { float s[4]; struct { float x, y, z, w; }; } cl_float3;
typedef union { float s[8]; } cl_float8;
typedef union { uint8_t s[8]; } cl_uchar8;

typedef cl_float8 vec8f;
typedef cl_float3 vec3f;
typedef cl_int2 vec2i;
typedef cl_uchar8 vec8u;
typedef cl_uchar3 vec3u;

namespace cl {
struct Program {};  // the adapter ignores it
}

struct system_settings {
  int spixl_size;
  float slic_color_weight;
  int array_width, array_height;
  int no_iter;
  bool enforce_connectivity = false;
  bool edge_enable = false;
  int num_disp_levels;
  int neib_hor, neib_ver, min_disp, max_disp, inc;
  float bl_ratio;
  int kernel_size, kernel_step;
  float fuse, gamma, alpha;
  int no_prop;
};
