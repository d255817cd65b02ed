// C-ABI of libmvs.so (include/mvs.h): context management, argument checking,
// metadata upload and the stage orchestration that the reference's host stage
// classes perform (clSLIC, clPhotoConsistency, clDepthRefinement).
#include <algorithm>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "mvs_internal.h"

namespace {
thread_local std::string g_err;

template <class T>
int ensure_dev(T** p, size_t* cap, size_t n) {
  if (*cap >= n && *p) return 0;
  if (*p) hipFree(*p);
  *p = nullptr;
  *cap = 0;
  if (hipMalloc((void**)p, sizeof(T) * (n ? n : 1)) != hipSuccess) {
    mvs::set_error("hipMalloc failed for metadata");
    return MVS_E_NOMEM;
  }
  *cap = n;
  return 0;
}

int check_array(const mvs_array* a) {
  if (!a || a->view_count <= 0 || a->array_width <= 0 || !a->levels || a->num_levels <= 0 || !a->view_subset ||
      !a->subset_num)
    return mvs::arg_fail("mvs_array: null pointer or non-positive size");
  for (int z = 0; z < a->view_count; z++) {
    int n = a->subset_num[z];
    if (n < 0 || n > a->view_count) return mvs::arg_fail("mvs_array: subset_num out of range");
    for (int k = 0; k < n; k++) {
      int v = a->view_subset[a->view_count * z + k];
      if (v < 0 || v >= a->view_count) return mvs::arg_fail("mvs_array: view_subset entry out of range");
    }
  }
  return 0;
}

// Upload levels / view_subset / subset_num when they differ from the cached copy.
int upload_meta(mvs_ctx* c, const mvs_array* a) {
  int rc = check_array(a);
  if (rc) return rc;
  int V = a->view_count, D = a->num_levels;
  bool same = (int)c->h_levels.size() == D && (int)c->h_sn.size() == V &&
              std::memcmp(c->h_levels.data(), a->levels, sizeof(float) * D) == 0 &&
              std::memcmp(c->h_vs.data(), a->view_subset, sizeof(int) * V * V) == 0 &&
              std::memcmp(c->h_sn.data(), a->subset_num, sizeof(int) * V) == 0;
  if (same) return 0;
  if ((rc = ensure_dev(&c->d_levels, &c->cap_levels, (size_t)D))) return rc;
  if ((rc = ensure_dev(&c->d_vs, &c->cap_vs, (size_t)V * V))) return rc;
  if ((rc = ensure_dev(&c->d_sn, &c->cap_sn, (size_t)V))) return rc;
  c->h_levels.assign(a->levels, a->levels + D);
  c->h_vs.assign(a->view_subset, a->view_subset + (size_t)V * V);
  c->h_sn.assign(a->subset_num, a->subset_num + V);
  MVS_HIP(hipMemcpyAsync(c->d_levels, c->h_levels.data(), sizeof(float) * D, hipMemcpyHostToDevice, c->stream),
          "upload levels");
  MVS_HIP(hipMemcpyAsync(c->d_vs, c->h_vs.data(), sizeof(int) * V * V, hipMemcpyHostToDevice, c->stream),
          "upload view_subset");
  MVS_HIP(hipMemcpyAsync(c->d_sn, c->h_sn.data(), sizeof(int) * V, hipMemcpyHostToDevice, c->stream),
          "upload subset_num");
  // the host vectors are the copy sources: finish before they can change
  MVS_HIP(hipStreamSynchronize(c->stream), "upload sync");
  return 0;
}

bool bad_dims(int W, int H) { return W <= 0 || H <= 0 || (long)W * H > (1L << 31) / 16; }

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) hipFree(p);
  }
  int alloc(size_t n) {
    if (hipMalloc(&p, n ? n : 1) != hipSuccess) {
      mvs::set_error("hipMalloc failed");
      return MVS_E_NOMEM;
    }
    return 0;
  }
  template <class T>
  T* as() {
    return (T*)p;
  }
};

}  // namespace

namespace mvs {
void set_error(const std::string& msg) { g_err = msg; }
int hip_fail(hipError_t e, const char* what) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return MVS_E_HIP;
}
int arg_fail(const char* what) {
  g_err = what;
  return MVS_E_ARG;
}
const int32_t* plan_upload(mvs_ctx* ctx, const std::vector<int32_t>& table, int* rc) {
  *rc = 0;
  auto it = ctx->plans.find(table);
  if (it != ctx->plans.end()) return it->second;
  if (ctx->plans.size() >= 256) {  // bound the cache: drop everything once in-flight work is done
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) { *rc = hip_fail(hipGetLastError(), "plan sync"); return nullptr; }
    for (auto& kv : ctx->plans) hipFree(kv.second);
    ctx->plans.clear();
  }
  int32_t* d = nullptr;
  size_t bytes = sizeof(int32_t) * (table.empty() ? 1 : table.size());
  if (hipMalloc(&d, bytes) != hipSuccess) {
    set_error("plan allocation failed");
    *rc = MVS_E_NOMEM;
    return nullptr;
  }
  auto ins = ctx->plans.emplace(table, d).first;  // the map's key is the (stable) copy source
  hipError_t e = hipMemcpyAsync(d, ins->first.data(), sizeof(int32_t) * table.size(), hipMemcpyHostToDevice,
                                ctx->stream);
  if (e != hipSuccess) { *rc = hip_fail(e, "plan upload"); return nullptr; }
  return d;
}

void* scratch(mvs_ctx* ctx, size_t bytes, int* rc) {
  *rc = 0;
  if (ctx->scratch_bytes >= bytes && ctx->scratch) return ctx->scratch;
  if (ctx->scratch) {
    hipStreamSynchronize(ctx->stream);
    hipFree(ctx->scratch);
  }
  ctx->scratch = nullptr;
  ctx->scratch_bytes = 0;
  if (hipMalloc(&ctx->scratch, bytes) != hipSuccess) {
    *rc = MVS_E_NOMEM;
    g_err = "scratch allocation failed";
    return nullptr;
  }
  ctx->scratch_bytes = bytes;
  return ctx->scratch;
}
}  // namespace mvs

#define RC(x)           \
  do {                  \
    int _r = (x);       \
    if (_r) return _r;  \
  } while (0)

extern "C" {

const char* mvs_last_error(void) { return g_err.c_str(); }
const char* mvs_version(void) { return "mvs-mi355x 0.7 (gfx950)"; }

int mvs_create(int device, mvs_ctx** out) {
  if (!out) return mvs::arg_fail("mvs_create: out is null");
  int n = 0;
  MVS_HIP(hipGetDeviceCount(&n), "hipGetDeviceCount");
  if (device < 0 || device >= n) return mvs::arg_fail("mvs_create: no such device");
  MVS_HIP(hipSetDevice(device), "hipSetDevice");
  mvs_ctx* c = new mvs_ctx();
  c->device = device;
  *out = c;
  return 0;
}

void mvs_destroy(mvs_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  if (c->scratch) hipFree(c->scratch);
  if (c->d_levels) hipFree(c->d_levels);
  if (c->d_vs) hipFree(c->d_vs);
  if (c->d_sn) hipFree(c->d_sn);
  for (auto& kv : c->plans) hipFree(kv.second);
  for (auto& ev : c->kev) {
    hipEventDestroy(ev.first);
    hipEventDestroy(ev.second);
  }
  if (c->own_stream) hipStreamDestroy(c->stream);
  delete c;
}

int mvs_set_stream(mvs_ctx* c, void* s) {
  if (!c) return mvs::arg_fail("null context");
  c->stream = (hipStream_t)s;
  return 0;
}

int mvs_synchronize(mvs_ctx* c) {
  if (!c) return mvs::arg_fail("null context");
  MVS_HIP(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
  return 0;
}

// ---- device-pointer API ------------------------------------------------------
int mvs_cvt_d(mvs_ctx* c, const uint8_t* rgbx, int V, int W, int H, float* lab, uint8_t* l8) {
  if (!c || !rgbx || !lab || V <= 0 || bad_dims(W, H)) return mvs::arg_fail("mvs_cvt_d: bad arguments");
  return mvs::launch_cvt(c->stream, rgbx, (long)V * W * H, lab, l8);
}

int mvs_grid_d(mvs_ctx* c, const float* lab, int V, int W, int H, int S, float* spixl, uint32_t* labels) {
  if (!c || !lab || !spixl || !labels || V <= 0 || S <= 0 || bad_dims(W, H))
    return mvs::arg_fail("mvs_grid_d: bad arguments");
  RC(mvs::launch_init_centers(c->stream, lab, V, W, H, S, spixl));
  return mvs::launch_grid_labels(c->stream, V, W, H, S, labels);
}

int mvs_slic_d(mvs_ctx* c, float* lab, int V, int W, int H, const mvs_slic_params* p, float* spixl,
               uint32_t* labels) {
  if (!c || !lab || !spixl || !labels || !p || V <= 0 || bad_dims(W, H))
    return mvs::arg_fail("mvs_slic_d: bad arguments");
  if (p->struct_size != sizeof(mvs_slic_params))
    return mvs::arg_fail("mvs_slic_d: struct_size != sizeof(mvs_slic_params) (caller built against another mvs.h)");
  int S = p->spixl_size;
  if (S < 6 || S > 96) return mvs::arg_fail("mvs_slic_d: spixl_size must be in [6, 96] (3S/16 > 0)");
  if (p->no_iter < 0) return mvs::arg_fail("mvs_slic_d: no_iter < 0");
  if (p->edge_enable < 0 || p->edge_enable > 2) return mvs::arg_fail("mvs_slic_d: edge_enable must be 0, 1 or 2");
  if (p->search != 0 && p->search != 1) return mvs::arg_fail("mvs_slic_d: search must be 0 or 1");
  // clSLIC ctor, clSLIC.cpp:15-18 (host float arithmetic)
  float xy = 1.0f / (1.4242f * (float)S);
  float col = 15.0f / (1.7321f * 128.0f);
  xy = xy * xy;
  col = col * col;
  hipStream_t s = c->stream;
  // one scratch for the update partials and the connectivity pass
  // (the edge step's magnitude plane uses it before the first assignment)
  size_t sb = std::max(mvs::update_scratch_bytes(V, W, H, S),
                       p->enforce_connectivity ? sizeof(uint32_t) * (size_t)V * W * H : (size_t)0);
  if (p->edge_enable) sb = std::max(sb, sizeof(float) * (size_t)V * W * H);
  // the window-walk update (S % 16 != 0) reads 16-bit copies of the labels
  // that each assignment writes beside them (labels < 65536); the scratch is
  // free then (the edge plane is consumed before the first assignment, the
  // connectivity pass runs after the last)
  const bool l16 = S % 16 != 0 && p->no_iter > 0 && (long)mvs::map_dim(W, S) * mvs::map_dim(H, S) <= 65536;
  if (l16) sb = std::max(sb, sizeof(uint16_t) * (size_t)V * W * H);
  int rc = 0;
  void* scr = sb ? mvs::scratch(c, sb, &rc) : nullptr;
  if (rc) return rc;
  float* part = mvs::update_scratch_bytes(V, W, H, S) ? (float*)scr : nullptr;
  RC(mvs::launch_init_centers(s, lab, V, W, H, S, spixl));
  RC(mvs::launch_edge_step(s, lab, V, W, H, S, p->edge_enable, spixl, (float*)scr));
  if (part && S % 16 == 0) {
    // assign -> (update -> assign) x no_iter with each update's tile partials
    // produced by the assign pass before it (one Lab read per iteration)
    // (an assignment an update follows stores no labels: the update reads its partials only)
    RC(mvs::launch_assign_tiles(s, lab, spixl, V, W, H, S, xy, col, p->color_weight, p->search,
                                p->no_iter > 0 ? nullptr : labels, p->no_iter > 0 ? part : nullptr));
    for (int i = 0; i < p->no_iter; i++) {
      RC(mvs::launch_update_finalize(s, part, V, W, H, S, spixl));
      const bool more = i + 1 < p->no_iter;
      RC(mvs::launch_assign_tiles(s, lab, spixl, V, W, H, S, xy, col, p->color_weight, p->search,
                                  more ? nullptr : labels, more ? part : nullptr));
    }
  } else {
    uint16_t* lb16 = l16 ? (uint16_t*)scr : nullptr;
    // with the 16-bit copies, an assignment an update follows writes only them
    // (the updates read nothing else); the last one writes the 32-bit labels
    RC(mvs::launch_assign(s, lab, spixl, V, W, H, S, xy, col, p->color_weight, p->search, lb16 ? nullptr : labels,
                          lb16));
    for (int i = 0; i < p->no_iter; i++) {
      RC(mvs::launch_update(s, lab, labels, V, W, H, S, spixl, part, lb16));
      const bool more = i + 1 < p->no_iter;
      RC(mvs::launch_assign(s, lab, spixl, V, W, H, S, xy, col, p->color_weight, p->search,
                            more && lb16 ? nullptr : labels, more ? lb16 : nullptr));
    }
  }
  if (p->enforce_connectivity) {
    uint32_t* tmp = (uint32_t*)scr;
    RC(mvs::launch_suppress(s, labels, tmp, V, W, H));
    RC(mvs::launch_suppress(s, tmp, labels, V, W, H));
  }
  return 0;
}

int mvs_boundary_d(mvs_ctx* c, int V, int W, int H, int S, const float* spixl, const uint32_t* labels,
                   uint8_t* rep) {
  if (!c || !spixl || !labels || !rep || V <= 0 || S <= 0 || bad_dims(W, H))
    return mvs::arg_fail("mvs_boundary_d: bad arguments");
  if (S > 256) return mvs::arg_fail("mvs_boundary_d: extents are uint8 (S <= 256)");
  return mvs::launch_boundary(c->stream, V, W, H, S, spixl, labels, rep);
}

int mvs_sweep_spixl_d(mvs_ctx* c, int W, int H, int S, const float* lab, float* spixl, const uint8_t* rep,
                      const mvs_array* a, int z0, int z1) {
  if (!c || !lab || !spixl || !rep || S <= 0 || bad_dims(W, H)) return mvs::arg_fail("mvs_sweep_spixl_d: bad arguments");
  RC(upload_meta(c, a));
  if (z0 < 0 || z1 > a->view_count || z0 > z1) return mvs::arg_fail("mvs_sweep_spixl_d: bad view range");
  return mvs::launch_sweep_spixl(c, a->view_count, W, H, S, lab, spixl, rep, c->d_levels, a->num_levels,
                                 c->d_vs, c->d_sn, a->array_width, a->bl_ratio, z0, z1);
}

int mvs_sweep_pixel_sad_d(mvs_ctx* c, int W, int H, const float* lab, const mvs_array* a, int z0, int z1,
                          float* disp) {
  if (!c || !lab || !disp || bad_dims(W, H)) return mvs::arg_fail("mvs_sweep_pixel_sad_d: bad arguments");
  RC(upload_meta(c, a));
  if (z0 < 0 || z1 > a->view_count || z0 > z1) return mvs::arg_fail("mvs_sweep_pixel_sad_d: bad view range");
  return mvs::launch_sweep_pixel_sad(c, a->view_count, W, H, lab, a->levels, a->num_levels, a->view_subset,
                                     a->subset_num, a->array_width, a->bl_ratio, z0, z1, disp);
}

int mvs_box_stats_d(mvs_ctx* c, const uint8_t* l8, int V, int W, int H, int K, int32_t* box) {
  if (!c || !l8 || !box || V <= 0 || bad_dims(W, H) || (K != 5 && K != 7))
    return mvs::arg_fail("mvs_box_stats_d: bad arguments (K must be 5 or 7)");
  return mvs::launch_box_stats(c->stream, l8, V, W, H, K, box, 0, V);
}

int mvs_box_stats_range_d(mvs_ctx* c, const uint8_t* l8, int V, int W, int H, int K, int z0, int z1, int32_t* box) {
  if (!c || !l8 || !box || V <= 0 || bad_dims(W, H) || (K != 5 && K != 7) || z0 < 0 || z1 > V || z0 > z1)
    return mvs::arg_fail("mvs_box_stats_range_d: bad arguments (K must be 5 or 7, 0 <= z0 <= z1 <= V)");
  return mvs::launch_box_stats(c->stream, l8, V, W, H, K, box, z0, z1);
}

int mvs_set_ncc_variant(mvs_ctx* c, int waves, int levels_per_wave, int band_w, int general_rows) {
  if (!c) return mvs::arg_fail("null context");
  if ((waves != 0 && waves != 4 && waves != 8) || (levels_per_wave != 0 && levels_per_wave != 1 &&
      levels_per_wave != 2 && levels_per_wave != 4) ||
      (band_w != 0 && band_w != 64 && band_w != 80 && band_w != 96 && band_w != 128 && band_w != 192 &&
       band_w != 256))
    return mvs::arg_fail(
        "mvs_set_ncc_variant: waves 0|4|8, levels_per_wave 0|1|2|4, band_w 0|64|80|96|128|192|256");
  c->ncc_nw = waves;
  c->ncc_dpw = levels_per_wave;
  c->ncc_bw = band_w;
  c->ncc_general = general_rows ? 1 : 0;
  return 0;
}

int mvs_set_kernel_timing(mvs_ctx* c, int on) {
  if (!c) return mvs::arg_fail("mvs_set_kernel_timing: null context");
  c->ktime = on != 0;
  c->kev_used = 0;
  return 0;
}

int mvs_kernel_times(mvs_ctx* c, float* ms, int cap, int* n) {
  if (!c || !n || (cap > 0 && !ms)) return mvs::arg_fail("mvs_kernel_times: bad arguments");
  const int k = (int)c->kev_used;
  *n = k;
  // more launches than the caller's buffer holds: fail and keep the record
  // (a truncated list divided by every swept view would read low)
  if (k > cap) return mvs::arg_fail("mvs_kernel_times: more launches recorded than cap");
  for (int i = 0; i < k; i++) {
    MVS_HIP(hipEventSynchronize(c->kev[i].second), "hipEventSynchronize(kernel timing)");
    float t = 0.0f;
    MVS_HIP(hipEventElapsedTime(&t, c->kev[i].first, c->kev[i].second), "hipEventElapsedTime(kernel timing)");
    ms[i] = t;
  }
  c->kev_used = 0;
  return 0;
}

int mvs_ncc_last_variant(mvs_ctx* c, int32_t* out7) {
  if (!c || !out7) return mvs::arg_fail("mvs_ncc_last_variant: null argument");
  for (int i = 0; i < 7; i++) out7[i] = c->ncc_last[i];  // the 0.5 report: seven slots, as its callers size it
  return 0;
}

int mvs_ncc_last_variant_n(mvs_ctx* c, int32_t* out, int cap) {
  if (!c || (cap > 0 && !out) || cap < 0) return mvs::arg_fail("mvs_ncc_last_variant_n: bad arguments");
  const int k = cap < 8 ? cap : 8;
  for (int i = 0; i < k; i++) out[i] = c->ncc_last[i];
  return 8;
}

int mvs_ncc_volume_d(mvs_ctx* c, int W, int H, const uint8_t* l8, const int32_t* box, const mvs_array* a, int K,
                     int z, float* vol) {
  if (!c || !l8 || !box || !vol || bad_dims(W, H)) return mvs::arg_fail("mvs_ncc_volume_d: bad arguments");
  RC(upload_meta(c, a));
  if (z < 0 || z >= a->view_count) return mvs::arg_fail("mvs_ncc_volume_d: bad reference view");
  return mvs::launch_ncc_volume(c, a->view_count, W, H, box, a->levels, a->num_levels, a->view_subset,
                                a->subset_num, a->array_width, a->bl_ratio, K, z, vol);
}

int mvs_ncc_wta_d(mvs_ctx* c, int W, int H, const uint8_t* l8, const int32_t* box, const mvs_array* a, int K,
                  int z, float* disp, float* conf) {
  if (!c || !l8 || !box || !disp || bad_dims(W, H)) return mvs::arg_fail("mvs_ncc_wta_d: bad arguments");
  RC(upload_meta(c, a));
  if (z < 0 || z >= a->view_count) return mvs::arg_fail("mvs_ncc_wta_d: bad reference view");
  return mvs::launch_ncc_volume(c, a->view_count, W, H, box, a->levels, a->num_levels, a->view_subset,
                                a->subset_num, a->array_width, a->bl_ratio, K, z, nullptr, c->d_levels, disp, conf);
}

int mvs_ncc_wta_range_d(mvs_ctx* c, int W, int H, const uint8_t* l8, const int32_t* box, const mvs_array* a, int K,
                        int z0, int z1, float* disp, float* conf) {
  if (!c || !l8 || !box || !disp || bad_dims(W, H)) return mvs::arg_fail("mvs_ncc_wta_range_d: bad arguments");
  RC(upload_meta(c, a));
  if (z0 < 0 || z1 > a->view_count || z0 > z1) return mvs::arg_fail("mvs_ncc_wta_range_d: bad view range");
  return mvs::launch_ncc_refs(c, a->view_count, W, H, box, a->levels, a->num_levels, a->view_subset, a->subset_num,
                              a->array_width, a->bl_ratio, K, z0, z1, nullptr, c->d_levels, disp, conf);
}

int mvs_wta_d(mvs_ctx* c, int W, int H, int D, const float* vol, const float* levels, float* disp, float* conf) {
  if (!c || !vol || !levels || !disp || D <= 0 || bad_dims(W, H)) return mvs::arg_fail("mvs_wta_d: bad arguments");
  return mvs::launch_wta(c->stream, W, H, D, vol, levels, disp, conf);
}

int mvs_flatness_d(mvs_ctx* c, int V, int mw, int mh, const float* spixl, float gamma, float* flat) {
  if (!c || !spixl || !flat || V <= 0 || mw <= 0 || mh <= 0) return mvs::arg_fail("mvs_flatness_d: bad arguments");
  return mvs::launch_flatness(c->stream, V, mw, mh, spixl, gamma, flat);
}

int mvs_init_state_d(mvs_ctx* c, int W, int H, int S, const float* spixl, const uint32_t* labels, const uint8_t* rep,
                     const float* flat, const mvs_array* a, float gamma, float alpha, int kernel_steps, float kss,
                     float fuse, float* state) {
  if (!c || !spixl || !labels || !rep || !flat || !state || S <= 0 || bad_dims(W, H))
    return mvs::arg_fail("mvs_init_state_d: bad arguments");
  RC(upload_meta(c, a));
  return mvs::launch_init_state(c->stream, a->view_count, W, H, S, a->array_width, a->bl_ratio, spixl, labels, 32,
                                rep, flat, c->d_vs, c->d_sn, gamma, alpha, kernel_steps, kss, fuse, state, 0,
                                a->view_count);
}

// The refinement / fusion entry points over uint32 labels (lbits 32) or the
// 16-bit maps of a narrowed all-gather (lbits 16: every label < mw * mh must
// fit, so mw * mh <= 2^16 is required).
static int labels_ok(int lbits, int W, int H, int S) {
  return lbits == 32 || (lbits == 16 && (long)mvs::map_dim(W, S) * mvs::map_dim(H, S) <= (1L << 16));
}

static int init_state_range(mvs_ctx* c, int W, int H, int S, const float* spixl, const void* labels, int lbits,
                            const uint8_t* rep, const float* flat, const mvs_array* a, float gamma, float alpha,
                            int kernel_steps, float kss, float fuse, int z0, int z1, float* state, const char* fn) {
  if (!c || !spixl || !labels || !rep || !flat || !state || S <= 0 || bad_dims(W, H) || !labels_ok(lbits, W, H, S))
    return mvs::arg_fail((std::string(fn) + ": bad arguments").c_str());
  RC(upload_meta(c, a));
  if (z0 < 0 || z1 > a->view_count || z0 > z1) return mvs::arg_fail((std::string(fn) + ": bad view range").c_str());
  return mvs::launch_init_state(c->stream, a->view_count, W, H, S, a->array_width, a->bl_ratio, spixl, labels, lbits,
                                rep, flat, c->d_vs, c->d_sn, gamma, alpha, kernel_steps, kss, fuse, state, z0, z1);
}

int mvs_init_state_range_d(mvs_ctx* c, int W, int H, int S, const float* spixl, const uint32_t* labels,
                           const uint8_t* rep, const float* flat, const mvs_array* a, float gamma, float alpha,
                           int kernel_steps, float kss, float fuse, int z0, int z1, float* state) {
  return init_state_range(c, W, H, S, spixl, labels, 32, rep, flat, a, gamma, alpha, kernel_steps, kss, fuse, z0, z1,
                          state, "mvs_init_state_range_d");
}

int mvs_init_state_range_l16_d(mvs_ctx* c, int W, int H, int S, const float* spixl, const uint16_t* labels,
                               const uint8_t* rep, const float* flat, const mvs_array* a, float gamma, float alpha,
                               int kernel_steps, float kss, float fuse, int z0, int z1, float* state) {
  return init_state_range(c, W, H, S, spixl, labels, 16, rep, flat, a, gamma, alpha, kernel_steps, kss, fuse, z0, z1,
                          state, "mvs_init_state_range_l16_d");
}

static int propagate(mvs_ctx* c, int W, int H, int S, const float* spixl, const void* labels, int lbits,
                     const uint8_t* rep, const float* flat, const mvs_array* a, int iter, float alpha, float gamma,
                     float fuse, int kernel_steps, float kss, const float* st_in, float* st_out, int z0, int z1,
                     const char* fn) {
  if (!c || !spixl || !labels || !rep || !flat || !st_in || !st_out || S <= 0 || bad_dims(W, H) ||
      !labels_ok(lbits, W, H, S))
    return mvs::arg_fail((std::string(fn) + ": bad arguments").c_str());
  RC(upload_meta(c, a));
  if (z0 < 0 || z1 > a->view_count || z0 > z1) return mvs::arg_fail((std::string(fn) + ": bad view range").c_str());
  int max_nbr = 0;
  for (int z = z0; z < z1; z++) max_nbr = std::max(max_nbr, (int)a->subset_num[z]);
  return mvs::launch_propagate(c->stream, a->view_count, W, H, S, a->array_width, a->bl_ratio, spixl, labels, lbits,
                               rep, flat, c->d_vs, c->d_sn, iter, alpha, gamma, fuse, kernel_steps, kss, st_in,
                               st_out, z0, z1, max_nbr);
}

int mvs_propagate_d(mvs_ctx* c, int W, int H, int S, const float* spixl, const uint32_t* labels, const uint8_t* rep,
                    const float* flat, const mvs_array* a, int iter, float alpha, float gamma, float fuse,
                    int kernel_steps, float kss, const float* st_in, float* st_out, int z0, int z1) {
  return propagate(c, W, H, S, spixl, labels, 32, rep, flat, a, iter, alpha, gamma, fuse, kernel_steps, kss, st_in,
                   st_out, z0, z1, "mvs_propagate_d");
}

int mvs_propagate_l16_d(mvs_ctx* c, int W, int H, int S, const float* spixl, const uint16_t* labels,
                        const uint8_t* rep, const float* flat, const mvs_array* a, int iter, float alpha, float gamma,
                        float fuse, int kernel_steps, float kss, const float* st_in, float* st_out, int z0, int z1) {
  return propagate(c, W, H, S, spixl, labels, 16, rep, flat, a, iter, alpha, gamma, fuse, kernel_steps, kss, st_in,
                   st_out, z0, z1, "mvs_propagate_l16_d");
}

int mvs_spixl_to_image_d(mvs_ctx* c, int V, int W, int H, int S, const float* spixl, const uint32_t* labels,
                         const float* state, float* disp) {
  if (!c || !spixl || !labels || !state || !disp || V <= 0 || S <= 0 || bad_dims(W, H))
    return mvs::arg_fail("mvs_spixl_to_image_d: bad arguments");
  return mvs::launch_spixl_to_image(c->stream, V, W, H, S, spixl, labels, 32, state, disp);
}

int mvs_spixl_to_image_l16_d(mvs_ctx* c, int V, int W, int H, int S, const float* spixl, const uint16_t* labels,
                             const float* state, float* disp) {
  if (!c || !spixl || !labels || !state || !disp || V <= 0 || S <= 0 || bad_dims(W, H) || !labels_ok(16, W, H, S))
    return mvs::arg_fail("mvs_spixl_to_image_l16_d: bad arguments");
  return mvs::launch_spixl_to_image(c->stream, V, W, H, S, spixl, labels, 16, state, disp);
}

// clDepthRefinement::do_refinement + fusion (depth_refinement.cpp:91-118, 1318-1370)
int mvs_refine_d(mvs_ctx* c, int W, int H, int S, const float* spixl, const uint32_t* labels, const uint8_t* rep,
                 const mvs_array* a, const mvs_refine_params* p, float* flat, float* state, float* state2,
                 float* disp) {
  if (!c || !p || !flat || !state || !state2) return mvs::arg_fail("mvs_refine_d: bad arguments");
  if (p->struct_size != sizeof(mvs_refine_params))
    return mvs::arg_fail("mvs_refine_d: struct_size != sizeof(mvs_refine_params) (caller built against another mvs.h)");
  if (p->prescaled != 0 && p->prescaled != 1) return mvs::arg_fail("mvs_refine_d: prescaled must be 0 or 1");
  RC(upload_meta(c, a));
  int V = a->view_count;
  int mw = mvs::map_dim(W, S), mh = mvs::map_dim(H, S);
  // pipeline::refine_depth_map, pipeline.cpp:164-166 (skipped when the caller
  // passes the values do_refinement receives)
  float gamma_ = p->prescaled ? p->gamma : (float)(2.0 * std::pow((double)p->gamma, 2.0));
  float alpha_ = p->prescaled ? p->alpha : (float)(2.0 * std::pow((double)p->alpha, 2.0));
  int kernel_size = p->prescaled ? p->kernel_size : p->kernel_size / 2;
  int nks = p->kernel_step;
  if (nks <= 0) return mvs::arg_fail("mvs_refine_d: kernel_step must be > 0");
  int kss_i = kernel_size / nks * S;
  float kss = (float)(kss_i > 1 ? kss_i : 1);
  float fuse = (float)(0.5 * (double)p->fuse);
  RC(mvs_flatness_d(c, V, mw, mh, spixl, (float)(1.0 / (double)gamma_), flat));
  RC(mvs_init_state_d(c, W, H, S, spixl, labels, rep, flat, a, 1.0f / gamma_, 1.0f / alpha_, nks, kss, fuse, state));
  float pg = (float)(1.0 / (double)gamma_), pa = (float)(1.0 / (double)alpha_);
  size_t sb = sizeof(float) * 6 * (size_t)V * mw * mh;
  if (p->no_prop > 0) MVS_HIP(hipMemcpyAsync(state2, state, sb, hipMemcpyDeviceToDevice, c->stream), "copy state");
  for (int it = 0; it < p->no_prop; it++) {
    float* out = (it % 2 == 0) ? state2 : state;
    const float* in = (it % 2 == 0) ? state : state2;
    RC(mvs_propagate_d(c, W, H, S, spixl, labels, rep, flat, a, it, pa, pg, fuse, nks / (it + 1),
                       kss / (float)(it + 1), in, out, 0, V));
  }
  // fusion renders current_state_dev (= `state`): the last odd iteration
  // (reference behaviour, Appendix A #13); non-compat renders the final one.
  const float* src = state;
  if (!p->fusion_compat && p->no_prop > 0) src = ((p->no_prop - 1) % 2 == 0) ? state2 : state;
  if (disp) RC(mvs_spixl_to_image_d(c, V, W, H, S, spixl, labels, src, disp));
  return 0;
}

int mvs_filter_d(mvs_ctx* c, int V, int W, int H, int array_width, float bl_ratio, float fuse, const float* disp_full,
                 float* proj, float* out, int z0, int z1) {
  if (!c || !disp_full || !proj || !out || V <= 0 || array_width <= 0 || bad_dims(W, H) || z0 < 0 || z1 > V ||
      z0 > z1)
    return mvs::arg_fail("mvs_filter_d: bad arguments");
  return mvs::launch_filter(c->stream, V, W, H, array_width, bl_ratio, (float)(0.5 * (double)fuse), disp_full, proj,
                            out, z0, z1);
}

int mvs_proj_inv_d(mvs_ctx* c, int V, int W, int H, int array_width, float bl_ratio, const float* disp_full,
                   float* proj, int z0, int z1) {
  if (!c || !disp_full || !proj || V <= 0 || array_width <= 0 || bad_dims(W, H) || z0 < 0 || z1 > V || z0 > z1)
    return mvs::arg_fail("mvs_proj_inv_d: bad arguments");
  return mvs::launch_proj_inv(c->stream, V, W, H, array_width, bl_ratio, disp_full, proj, z0, z1, 0, H, false);
}

int mvs_proj_inv_rows_d(mvs_ctx* c, int V, int W, int H, int array_width, float bl_ratio, const float* disp_full,
                        float* proj, int proj_band, int z0, int z1, int y0, int y1) {
  if (!c || !disp_full || (!proj && y1 > y0) || V <= 0 || array_width <= 0 || bad_dims(W, H) || z0 < 0 || z1 > V || z0 > z1 ||
      y0 < 0 || y1 > H || y0 > y1)
    return mvs::arg_fail("mvs_proj_inv_rows_d: bad arguments");
  return mvs::launch_proj_inv(c->stream, V, W, H, array_width, bl_ratio, disp_full, proj, z0, z1, y0, y1,
                              proj_band != 0);
}

int mvs_remove_inconsistency_d(mvs_ctx* c, int V, int W, int H, int array_width, float bl_ratio, float fuse,
                               const float* disp_full, const float* proj, float* out, int z0, int z1) {
  if (!c || !disp_full || !proj || !out || V <= 0 || array_width <= 0 || bad_dims(W, H) || z0 < 0 || z1 > V ||
      z0 > z1)
    return mvs::arg_fail("mvs_remove_inconsistency_d: bad arguments");
  return mvs::launch_remove_incons(c->stream, V, W, H, array_width, bl_ratio, (float)(0.5 * (double)fuse), disp_full,
                                   proj, out, z0, z1, 0, H, false);
}

int mvs_remove_inconsistency_rows_d(mvs_ctx* c, int V, int W, int H, int array_width, float bl_ratio, float fuse,
                                    const float* disp_full, const float* proj, int proj_band, float* out, int z0,
                                    int z1, int y0, int y1) {
  if (!c || !disp_full || (!proj && y1 > y0) || !out || V <= 0 || array_width <= 0 || bad_dims(W, H) || z0 < 0 || z1 > V ||
      z0 > z1 || y0 < 0 || y1 > H || y0 > y1)
    return mvs::arg_fail("mvs_remove_inconsistency_rows_d: bad arguments");
  return mvs::launch_remove_incons(c->stream, V, W, H, array_width, bl_ratio, (float)(0.5 * (double)fuse), disp_full,
                                   proj, out, z0, z1, y0, y1, proj_band != 0);
}

// ---- host-pointer API (reference stage methods) ----------------------------------
int mvs_do_super_pixel_seg(mvs_ctx* c, const uint8_t* rgbx, int W, int H, const mvs_slic_params* p, float* lab,
                           float* spixl, uint32_t* labels) {
  if (!c || !rgbx || !p || bad_dims(W, H) || p->spixl_size <= 0) return mvs::arg_fail("mvs_do_super_pixel_seg: bad arguments");
  size_t P = (size_t)W * H;
  int mw = mvs::map_dim(W, p->spixl_size), mh = mvs::map_dim(H, p->spixl_size);
  size_t M = (size_t)mw * mh;
  DevBuf din, dlab, dsp, dlb;
  RC(din.alloc(P * 4));
  RC(dlab.alloc(P * 16));
  RC(dsp.alloc(M * 32));
  RC(dlb.alloc(P * 4));
  hipStream_t s = c->stream;
  MVS_HIP(hipMemsetAsync(dsp.p, 0, M * 32, s), "memset");
  MVS_HIP(hipMemcpyAsync(din.p, rgbx, P * 4, hipMemcpyHostToDevice, s), "H2D rgbx");
  RC(mvs_cvt_d(c, din.as<uint8_t>(), 1, W, H, dlab.as<float>(), nullptr));
  RC(mvs_slic_d(c, dlab.as<float>(), 1, W, H, p, dsp.as<float>(), dlb.as<uint32_t>()));
  if (lab) MVS_HIP(hipMemcpyAsync(lab, dlab.p, P * 16, hipMemcpyDeviceToHost, s), "D2H lab");
  if (spixl) MVS_HIP(hipMemcpyAsync(spixl, dsp.p, M * 32, hipMemcpyDeviceToHost, s), "D2H spixl");
  if (labels) MVS_HIP(hipMemcpyAsync(labels, dlb.p, P * 4, hipMemcpyDeviceToHost, s), "D2H labels");
  MVS_HIP(hipStreamSynchronize(s), "sync");
  return 0;
}

int mvs_do_initial_depth_estimation(mvs_ctx* c, int W, int H, int S, float* spixl, uint8_t* rep, const float* lab,
                                    const uint32_t* labels, const mvs_array* a) {
  if (!c || !spixl || !lab || !labels || S <= 0 || bad_dims(W, H)) return mvs::arg_fail("mvs_do_initial_depth_estimation: bad arguments");
  RC(check_array(a));
  int V = a->view_count;
  size_t P = (size_t)W * H;
  int mw = mvs::map_dim(W, S), mh = mvs::map_dim(H, S);
  size_t M = (size_t)mw * mh;
  DevBuf dlab, dsp, dlb, drep;
  RC(dlab.alloc(V * P * 16));
  RC(dsp.alloc(V * M * 32));
  RC(dlb.alloc(V * P * 4));
  RC(drep.alloc(V * M * 8));
  hipStream_t s = c->stream;
  MVS_HIP(hipMemcpyAsync(dlab.p, lab, V * P * 16, hipMemcpyHostToDevice, s), "H2D lab");
  MVS_HIP(hipMemcpyAsync(dsp.p, spixl, V * M * 32, hipMemcpyHostToDevice, s), "H2D spixl");
  MVS_HIP(hipMemcpyAsync(dlb.p, labels, V * P * 4, hipMemcpyHostToDevice, s), "H2D labels");
  RC(mvs_boundary_d(c, V, W, H, S, dsp.as<float>(), dlb.as<uint32_t>(), drep.as<uint8_t>()));
  RC(mvs_sweep_spixl_d(c, W, H, S, dlab.as<float>(), dsp.as<float>(), drep.as<uint8_t>(), a, 0, V));
  MVS_HIP(hipMemcpyAsync(spixl, dsp.p, V * M * 32, hipMemcpyDeviceToHost, s), "D2H spixl");
  if (rep) MVS_HIP(hipMemcpyAsync(rep, drep.p, V * M * 8, hipMemcpyDeviceToHost, s), "D2H rep");
  MVS_HIP(hipStreamSynchronize(s), "sync");
  return 0;
}

int mvs_do_refinement(mvs_ctx* c, int W, int H, int S, const float* spixl, const uint32_t* labels, const uint8_t* rep,
                      const mvs_array* a, const mvs_refine_params* p, float* state_out, float* disp) {
  if (!c || !spixl || !labels || !rep || !p || S <= 0 || bad_dims(W, H)) return mvs::arg_fail("mvs_do_refinement: bad arguments");
  RC(check_array(a));
  int V = a->view_count;
  size_t P = (size_t)W * H;
  int mw = mvs::map_dim(W, S), mh = mvs::map_dim(H, S);
  size_t M = (size_t)mw * mh;
  DevBuf dsp, dlb, drep, dfl, dst, dst2, ddisp;
  RC(dsp.alloc(V * M * 32));
  RC(dlb.alloc(V * P * 4));
  RC(drep.alloc(V * M * 8));
  RC(dfl.alloc(V * M * 8));
  RC(dst.alloc(V * M * 24));
  RC(dst2.alloc(V * M * 24));
  RC(ddisp.alloc(V * P * 4));
  hipStream_t s = c->stream;
  MVS_HIP(hipMemcpyAsync(dsp.p, spixl, V * M * 32, hipMemcpyHostToDevice, s), "H2D spixl");
  MVS_HIP(hipMemcpyAsync(dlb.p, labels, V * P * 4, hipMemcpyHostToDevice, s), "H2D labels");
  MVS_HIP(hipMemcpyAsync(drep.p, rep, V * M * 8, hipMemcpyHostToDevice, s), "H2D rep");
  RC(mvs_refine_d(c, W, H, S, dsp.as<float>(), dlb.as<uint32_t>(), drep.as<uint8_t>(), a, p, dfl.as<float>(),
                  dst.as<float>(), dst2.as<float>(), disp ? ddisp.as<float>() : nullptr));
  if (state_out) {
    const void* src = dst.p;
    if (!p->fusion_compat && p->no_prop > 0) src = ((p->no_prop - 1) % 2 == 0) ? dst2.p : dst.p;
    MVS_HIP(hipMemcpyAsync(state_out, src, V * M * 24, hipMemcpyDeviceToHost, s), "D2H state");
  }
  if (disp) MVS_HIP(hipMemcpyAsync(disp, ddisp.p, V * P * 4, hipMemcpyDeviceToHost, s), "D2H disp");
  MVS_HIP(hipStreamSynchronize(s), "sync");
  return 0;
}

int mvs_do_consistency_filter(mvs_ctx* c, int V, int W, int H, int array_width, float bl_ratio, float fuse,
                              const float* disp_full, float* out) {
  if (!c || !disp_full || !out || V <= 0 || array_width <= 0 || bad_dims(W, H))
    return mvs::arg_fail("mvs_do_consistency_filter: bad arguments");
  size_t n = (size_t)V * W * H * sizeof(float);
  DevBuf din, dproj, dout;
  RC(din.alloc(n));
  RC(dproj.alloc(n));
  RC(dout.alloc(n));
  hipStream_t s = c->stream;
  MVS_HIP(hipMemcpyAsync(din.p, disp_full, n, hipMemcpyHostToDevice, s), "H2D disparity");
  RC(mvs_filter_d(c, V, W, H, array_width, bl_ratio, fuse, din.as<float>(), dproj.as<float>(), dout.as<float>(), 0,
                  V));
  MVS_HIP(hipMemcpyAsync(out, dout.p, n, hipMemcpyDeviceToHost, s), "D2H filtered");
  MVS_HIP(hipStreamSynchronize(s), "sync");
  return 0;
}

}  // extern "C"
