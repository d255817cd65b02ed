// Internal helpers shared by the HIP translation units of libmvs.so.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdint>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mvs.h"
#include "../../include/mvs_detmath.h"

struct mvs_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  // persistent scratch (grown on demand)
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  // device copy of the last mvs_array metadata
  float* d_levels = nullptr;
  int* d_vs = nullptr;
  int* d_sn = nullptr;
  size_t cap_levels = 0, cap_vs = 0, cap_sn = 0;
  std::vector<float> h_levels;
  std::vector<int> h_vs, h_sn;
  // small host-built launch plans (e.g. the NCC shift tables), uploaded once
  // per distinct content and kept for the life of the context
  std::map<std::vector<int32_t>, int32_t*> plans;
  // NCC sweep variant override (mvs_set_ncc_variant; 0 = automatic) and the
  // variant of the last launch {K, TH, DPW, NW, BW, PAR, FUSE, NB} (DPW 16: the matrix-core form)
  int ncc_nw = 0, ncc_dpw = 0, ncc_bw = 0, ncc_general = 0;
  int ncc_last[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // kernel timing (mvs_set_kernel_timing): the fused NCC sweep's launches carry
  // start / stop events of their own dispatch (hipExtLaunchKernel), pooled
  bool ktime = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> kev;
  size_t kev_used = 0;
};

namespace mvs {

// the next timed launch's event pair (null, null: timing off or no events)
inline std::pair<hipEvent_t, hipEvent_t> kernel_events(mvs_ctx* ctx) {
  if (!ctx->ktime) return {nullptr, nullptr};
  if (ctx->kev_used == ctx->kev.size()) {
    hipEvent_t a = nullptr, b = nullptr;
    if (hipEventCreate(&a) != hipSuccess) return {nullptr, nullptr};
    if (hipEventCreate(&b) != hipSuccess) {
      hipEventDestroy(a);
      return {nullptr, nullptr};
    }
    ctx->kev.push_back({a, b});
  }
  return ctx->kev[ctx->kev_used++];
}

// Raise kern's dynamic-LDS limit to lds bytes on ctx's device when above the
// 64 KB default.  HIP keeps the attribute per device, so the raise is cached
// per (kernel, device) -- a context on a second GPU raises it there too --
// under a mutex (contexts may launch from several host threads).
inline hipError_t raise_lds(mvs_ctx* ctx, const void* kern, size_t lds) {
  if (lds <= 64 * 1024) return hipSuccess;
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, size_t> done;
  std::lock_guard<std::mutex> lock(mu);
  size_t& have = done[{kern, ctx->device}];
  if (lds <= have) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e == hipSuccess) have = lds;
  return e;
}

void set_error(const std::string& msg);
int hip_fail(hipError_t e, const char* what);
int arg_fail(const char* what);
void* scratch(mvs_ctx* ctx, size_t bytes, int* rc);
const int32_t* plan_upload(mvs_ctx* ctx, const std::vector<int32_t>& table, int* rc);

inline int map_dim(int n, int S) {
  // (int)ceil((float)n / (float)S), pipeline.cpp:18-19
  return (int)__builtin_ceilf((float)n / (float)S);
}

constexpr int kLocal = 16;  // LOCAL_SIZE_UPDATE, header.h:37-38

#define MVS_LAUNCH_CHECK(what)                          \
  do {                                                  \
    hipError_t _e = hipGetLastError();                  \
    if (_e != hipSuccess) return mvs::hip_fail(_e, what); \
  } while (0)

#define MVS_HIP(call, what)                              \
  do {                                                   \
    hipError_t _e = (call);                              \
    if (_e != hipSuccess) return mvs::hip_fail(_e, what); \
  } while (0)

// ---- launchers implemented in the .hip files (device pointers) ------------
int launch_cvt(hipStream_t s, const uint8_t* rgbx, long npix, float* lab, uint8_t* l8);
int launch_init_centers(hipStream_t s, const float* lab, int V, int W, int H, int S, float* spixl);
int launch_grid_labels(hipStream_t s, int V, int W, int H, int S, uint32_t* labels);
int launch_edge_step(hipStream_t s, float* lab, int V, int W, int H, int S, int edge_enable, float* spixl,
                     float* edge);
int launch_assign(hipStream_t s, const float* lab, const float* spixl, int V, int W, int H, int S, float xy_n,
                  float col_n, float weight, int search, uint32_t* labels, uint16_t* lb16 = nullptr);
size_t update_scratch_bytes(int V, int W, int H, int S);
int launch_assign_tiles(hipStream_t s, const float* lab, const float* spixl, int V, int W, int H, int S, float xy_n,
                        float col_n, float weight, int search, uint32_t* labels, float* part);
int launch_update_finalize(hipStream_t s, const float* part, int V, int W, int H, int S, float* spixl);
int launch_update(hipStream_t s, const float* lab, const uint32_t* labels, int V, int W, int H, int S,
                  float* spixl, float* part, const uint16_t* lb16 = nullptr);
int launch_suppress(hipStream_t s, const uint32_t* in, uint32_t* out, int V, int W, int H);

int launch_boundary(hipStream_t s, int V, int W, int H, int S, const float* spixl, const uint32_t* labels,
                    uint8_t* rep);
int launch_sweep_spixl(mvs_ctx* ctx, int V, int W, int H, int S, const float* lab, float* spixl,
                       const uint8_t* rep, const float* levels, int D, const int* vs, const int* sn, int aw,
                       float bl, int z0, int z1);
int launch_sweep_pixel_sad(mvs_ctx* ctx, int V, int W, int H, const float* lab, const float* levels_host, int D,
                           const int* vs_host, const int* sn_host, int aw, float bl, int z0, int z1, float* disp);
int launch_box_stats(hipStream_t s, const uint8_t* l8, int V, int W, int H, int K, int32_t* box, int z0, int z1);
int launch_ncc_volume(mvs_ctx* ctx, int V, int W, int H, const int32_t* box, const float* levels_host, int D,
                      const int* vs_host, const int* sn_host, int aw, float bl, int K, int z, float* vol,
                      const float* levels_dev = nullptr, float* disp = nullptr, float* conf = nullptr);
int launch_ncc_refs(mvs_ctx* ctx, int V, int W, int H, const int32_t* box, const float* levels_host, int D,
                    const int* vs_host, const int* sn_host, int aw, float bl, int K, int z0, int z1, float* vol,
                    const float* levels_dev, float* disp, float* conf);
int launch_wta(hipStream_t s, int W, int H, int D, const float* vol, const float* levels, float* disp,
               float* conf);

int launch_flatness(hipStream_t s, int V, int mw, int mh, const float* spixl, float gamma, float* flat);
// labels: uint32, or uint16 when lbits == 16 (16-bit gathered maps)
int launch_init_state(hipStream_t s, int V, int W, int H, int S, int aw, float bl, const float* spixl,
                      const void* labels, int lbits, const uint8_t* rep, const float* flat, const int* vs,
                      const int* sn, float gamma, float alpha, int nks, float kss, float fuse, float* state,
                      int z0, int z1);
int launch_propagate(hipStream_t s, int V, int W, int H, int S, int aw, float bl, const float* spixl,
                     const void* labels, int lbits, const uint8_t* rep, const float* flat, const int* vs,
                     const int* sn, int iter, float alpha, float gamma, float fuse, int nks, float kss,
                     const float* st_in, float* st_out, int z0, int z1,
                     int max_nbr);  // the largest neighbour count of views [z0, z1)
int launch_spixl_to_image(hipStream_t s, int V, int W, int H, int S, const float* spixl,
                          const void* labels, int lbits, const float* state, float* disp);
int launch_filter(hipStream_t s, int V, int W, int H, int aw, float bl, float fuse, const float* full,
                  float* proj, float* out, int z0, int z1);
int launch_proj_inv(hipStream_t s, int V, int W, int H, int aw, float bl, const float* full, float* proj, int z0,
                    int z1, int ya, int yb, bool band);
int launch_remove_incons(hipStream_t s, int V, int W, int H, int aw, float bl, float fuse, const float* full,
                         const float* proj, float* out, int z0, int z1, int ya, int yb, bool band);

}  // namespace mvs
