// clmvde_adapter.h -- drop-in replacements for the reference's three OpenCL
// stage classes (clSLIC, clPhotoConsistency, clDepthRefinement) on libmvs.so.
//
// A maintainer of clMVDE includes this header instead of clSLIC.h,
// photo_consistency.h and depth_refinement.h; every call site in
// pipeline.cpp (lines 73, 88, 156-157, 170-173) stays as it is.  The
// cl::Program argument is accepted and ignored (the kernels are in
// libmvs.so).  The reference's types (vec2i, vec3u, vec3f, vec8f, vec8u,
// cl_int2, cl_uint, system_settings, cl::Program; header.h + CL/cl.hpp) must
// be declared before this header, as clMVDE's header.h does.
//
// Errors: the reference prints cl_int codes and continues (errorHandler,
// file_handler.cpp:97-113); these classes throw std::runtime_error with
// mvs_last_error() instead.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "mvs.h"

namespace mvs_adapter {

inline void check(int rc, const char* what) {
  if (rc != MVS_OK) throw std::runtime_error(std::string(what) + ": " + mvs_last_error());
}

// one context per process (device 0), as the reference's one OpenCL context
inline mvs_ctx* context() {
  struct Holder {
    mvs_ctx* c = nullptr;
    Holder() { check(mvs_create(0, &c), "mvs_create"); }
    ~Holder() { mvs_destroy(c); }
  };
  static Holder h;
  return h.c;
}

// view_subset (vector of neighbour lists) -> the V x V matrix + counts the
// kernels take (photo_consistency.cpp:38-47, depth_refinement.cpp:22-31)
struct Subsets {
  std::vector<int32_t> mat, num;
  Subsets(const std::vector<std::vector<int> >& vs, int V) : mat((size_t)V * V, 0), num(V, 0) {
    for (int i = 0; i < V; i++) {
      num[i] = (int32_t)vs[i].size();
      for (size_t j = 0; j < vs[i].size(); j++) mat[(size_t)i * V + j] = vs[i][j];
    }
  }
};

}  // namespace mvs_adapter

// clSLIC.h:11-19 -- clSLIC(program, settings, img_size, map_size);
// do_super_pixel_seg(in_img, cvt_img, spixl_map, idx_img)
class clSLIC {
 public:
  clSLIC(cl::Program, system_settings* s, cl_int2 img_size, cl_int2 /*map_size*/)
      : W_(img_size.x), H_(img_size.y) {
    p_.struct_size = sizeof(mvs_slic_params);
    p_.spixl_size = s->spixl_size;
    p_.color_weight = s->slic_color_weight;
    p_.no_iter = s->no_iter;
    p_.enforce_connectivity = s->enforce_connectivity ? 1 : 0;
    p_.edge_enable = s->edge_enable ? 1 : 0;  // as the reference behaves (mvs.h)
    p_.search = 0;                            // clcode.cl's active candidate loop
  }
  void do_super_pixel_seg(vec3u* in_img, vec3f* cvt_img, vec8f* spixl_map, cl_uint* idx_img) {
    mvs_adapter::check(mvs_do_super_pixel_seg(mvs_adapter::context(), (const uint8_t*)in_img, W_, H_, &p_,
                                              (float*)cvt_img, (float*)spixl_map, (uint32_t*)idx_img),
                       "clSLIC::do_super_pixel_seg");
  }

 private:
  int W_, H_;
  mvs_slic_params p_{};
};

// photo_consistency.h:8-19 -- clPhotoConsistency(program, view_count,
// spixl_size, num_disp_levels, img_size, map_size);
// do_initial_depth_estimation(spixel_map, spixel_rep, cvt_img, idx_img,
// array_width, bl_ratio, view_subset, disp_levels)
class clPhotoConsistency {
 public:
  clPhotoConsistency(cl::Program, int view_count, int spixl_size, int /*num_disp_levels*/, vec2i img_size,
                     vec2i /*map_size*/)
      : V_(view_count), S_(spixl_size), W_(img_size.x), H_(img_size.y) {}
  void do_initial_depth_estimation(vec8f* spixel_map, vec8u* spixel_rep, vec3f* cvt_img, cl_uint* idx_img,
                                   int array_width, float bl_ratio, std::vector<std::vector<int> >& view_subset,
                                   std::vector<float>& disp_levels) {
    mvs_adapter::Subsets sub(view_subset, V_);
    mvs_array a{V_, array_width, bl_ratio, disp_levels.data(), (int)disp_levels.size(), sub.mat.data(),
                sub.num.data()};
    mvs_adapter::check(mvs_do_initial_depth_estimation(mvs_adapter::context(), W_, H_, S_, (float*)spixel_map,
                                                       (uint8_t*)spixel_rep, (const float*)cvt_img,
                                                       (const uint32_t*)idx_img, &a),
                       "clPhotoConsistency::do_initial_depth_estimation");
  }

 private:
  int V_, S_, W_, H_;
};

// depth_refinement.h:6-9 -- clDepthRefinement(program, img_size, map_size,
// camera_array_size, cvt_img, spixl_map, idx_img, spixl_rep, view_subset_vec,
// spixl_size, bl_ratio); do_refinement(gamma, alpha, fuse, kernel_step,
// kernel_size, no_prop).  pipeline.cpp:164-173 calls do_refinement with
// gamma' = 2 gamma^2, alpha' = 2 alpha^2 and kernel_size / 2 already applied,
// so the parameters go to libmvs with prescaled = 1.  The fused disparity
// stays inside the object, as the reference's private disp_img
// (depth_refinement.cpp:1458); disp() exposes it.
class clDepthRefinement {
 public:
  clDepthRefinement(cl::Program, vec2i img_size, vec2i map_size, vec2i camera_array_size, vec3f* /*cvt_img*/,
                    vec8f* spixl_map, cl_uint* idx_img, vec8u* spixl_rep,
                    std::vector<std::vector<int> > view_subset_vec, int spixl_size, float bl_ratio)
      : W_(img_size.x), H_(img_size.y), S_(spixl_size), aw_(camera_array_size.x),
        V_(camera_array_size.x * camera_array_size.y), bl_(bl_ratio), spixl_(spixl_map), idx_(idx_img),
        rep_(spixl_rep), sub_(view_subset_vec, camera_array_size.x * camera_array_size.y),
        disp_((size_t)V_ * img_size.x * img_size.y) {
    (void)map_size;
  }
  void do_refinement(float gamma, float alpha, float fuse, int kernel_step, int kernel_size, int no_prop) {
    mvs_refine_params p{};
    p.struct_size = sizeof(mvs_refine_params);
    p.gamma = gamma;
    p.alpha = alpha;
    p.fuse = fuse;
    p.kernel_step = kernel_step;
    p.kernel_size = kernel_size;
    p.no_prop = no_prop;
    p.fusion_compat = 1;  // fusion renders current_state_dev (depth_refinement.cpp:1352)
    p.prescaled = 1;
    float no_levels = 0.0f;  // the refinement reads no disparity levels; mvs_array wants one
    mvs_array a{V_, aw_, bl_, &no_levels, 1, sub_.mat.data(), sub_.num.data()};
    mvs_adapter::check(mvs_do_refinement(mvs_adapter::context(), W_, H_, S_, (const float*)spixl_,
                                         (const uint32_t*)idx_, (const uint8_t*)rep_, &a, &p, nullptr,
                                         disp_.data()),
                       "clDepthRefinement::do_refinement");
  }
  const float* disp() const { return disp_.data(); }

 private:
  int W_, H_, S_, aw_, V_;
  float bl_;
  vec8f* spixl_;
  cl_uint* idx_;
  vec8u* rep_;
  mvs_adapter::Subsets sub_;
  std::vector<float> disp_;
};
