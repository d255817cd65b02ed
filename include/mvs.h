/* mvs.h -- C-ABI of the MI355X multi-view-stereo depth engine (libmvs.so).
 *
 * Drop-in boundary for the reference's hot path.  The reference has no plugin
 * API: its host stage classes enqueue OpenCL kernels by name.  Each entry point
 * below replaces one of those stage methods / kernel groups (file:line of the
 * reference interface in the comment), takes the reference's data layouts
 *  as plain pointers + sizes, and returns 0 or a negative
 * MVS_E_* status (the reference prints cl_int errors and carries on;
 * errorHandler, file_handler.cpp:97-113 -- here every failure is returned).
 *
 * Two flavours:
 *   mvs_*      host pointers; copy in, run on the context's GPU, copy out,
 *              synchronous (what the reference stage methods do).
 *   mvs_*_d    device pointers, enqueued on the context's HIP stream, async.
 *
 * Layouts (all arrays view-major, row-major):
 *   rgbx   uint8 [V][H][W][4]  s0=R, s1=G, s2=B (loadImageIn, file_handler.cpp:6-14)
 *   lab    float [V][H][W][4]  CIE-Lab + pad  (cl_float3)
 *   l8     uint8 [V][H][W]     8-bit intensity for the NCC cost (build-defined)
 *   spixl  float [V][mh][mw][8] {id, cx, cy, L, a, b, count, disparity}
 *   labels uint32 [V][H][W]    per-view superpixel index y*mw+x
 *   rep    uint8 [V][mh][mw][8] ray extents {NW,W,SW,N,S,NE,E,SE}
 *   levels float [D]           disparity hypotheses
 *   view_subset int32 [V][V] (row z = neighbour list of z), subset_num int32 [V]
 *   state  float [V][mh][mw][6] {d, sm, cs, nx, ny, nz}
 *   disp   float [V][H][W]     disparity in pixels (depth-map output)
 *   mw = ceil(W/S), mh = ceil(H/S) (pipeline.cpp:18-19)
 *
 * Not thread-safe per context.  One context per GPU; one process per GPU.
 */
#ifndef MVS_H
#define MVS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  MVS_OK = 0,
  MVS_E_ARG = -1,      /* invalid argument / shape */
  MVS_E_HIP = -2,      /* HIP runtime error */
  MVS_E_NOMEM = -3,    /* device allocation failed */
  MVS_E_UNSUPPORTED = -4
};

typedef struct mvs_ctx mvs_ctx;

/* SLIC parameters: system_settings fields used by clSLIC (header.h:55-77).
 * ABI 0.3 (mvs_version): struct_size must be sizeof(mvs_slic_params) -- a
 * caller built against an older mvs.h (0.1: four ints, no size field) is
 * refused with MVS_E_ARG instead of having its fields misread. */
typedef struct {
  uint32_t struct_size;      /* = sizeof(mvs_slic_params) */
  int spixl_size;            /* S */
  float color_weight;        /* slic_color_weight (clMVDE.cpp:16 = 0.6) */
  int no_iter;               /* update/assign iterations (5) */
  int enforce_connectivity;  /* supress_local_lable x2 (clSLIC.cpp:373-411) */
  int edge_enable;           /* apply_edge_values (clSLIC.cpp:84-86, 186-233; clcode.cl:161-248):
                              * 0 off (the reference's default, header.h:61);
                              * 1 the reference's path as it behaves: the edge magnitude
                              *   overwrites the Lab image (L = a = b = e) and no centre moves
                              *   (apply_edge_alternative reads the never-written edge_img,
                              *   pinned as zeros);
                              * 2 the intended path: Lab kept, each centre moves to its
                              *   least-edge 8-neighbour and takes its colour. */
  int search;                /* candidate centres of find_center_association:
                              * 0 the active loop (clcode.cl:474-494: 2x2 cells, x/y
                              *   deltas swapped) -- the reference's default;
                              * 1 the 3x3 loop behind the reference's comment switch
                              *   (clcode.cl:496-516), with which its kept depth outputs
                              *   were produced. */
} mvs_slic_params;

/* Camera array / hypothesis set (pipeline::perform_depth_est).  Its arrays are
 * small metadata and are HOST pointers in both API flavours; the context keeps
 * a device copy (re-uploaded only when the contents change). */
typedef struct {
  int view_count;            /* V */
  int array_width;           /* cameras per row */
  float bl_ratio;            /* vertical / horizontal baseline ratio */
  const float* levels;       /* [D] host pointer */
  int num_levels;            /* D */
  const int32_t* view_subset;/* [V][V] */
  const int32_t* subset_num; /* [V] */
} mvs_array;

/* Refinement parameters (system_settings; clDepthRefinement::do_refinement).
 * ABI 0.3: struct_size must be sizeof(mvs_refine_params). */
typedef struct {
  uint32_t struct_size;      /* = sizeof(mvs_refine_params) */
  float gamma;               /* settings->gamma (2), or gamma' with prescaled = 1 */
  float alpha;               /* settings->alpha (6), or alpha' with prescaled = 1 */
  float fuse;                /* settings->fuse (1) */
  int kernel_step;           /* settings->kernel_step (13) */
  int kernel_size;           /* settings->kernel_size (1080), or its half with prescaled = 1 */
  int no_prop;               /* propagate iterations (5) */
  int fusion_compat;         /* 1: render current_state_dev as the reference does */
  int prescaled;             /* 0: the library applies pipeline::refine_depth_map's derivation
                              *    (pipeline.cpp:164-166: gamma' = 2 gamma^2, alpha' = 2 alpha^2,
                              *    kernel_size / 2);
                              * 1: gamma, alpha, kernel_size already are those values -- the
                              *    arguments clDepthRefinement::do_refinement receives
                              *    (depth_refinement.h:9), for a drop-in of that method */
} mvs_refine_params;

/* ---- context ----------------------------------------------------------- */
int mvs_create(int device, mvs_ctx** out);
void mvs_destroy(mvs_ctx* ctx);
const char* mvs_last_error(void);
int mvs_set_stream(mvs_ctx* ctx, void* hip_stream);   /* NULL = default stream */
int mvs_synchronize(mvs_ctx* ctx);
const char* mvs_version(void);

/* ---- device-pointer stage API ------------------------------------------ */
/* cvt kernel (clcode.cl:125-151) over V views; l8 may be NULL. */
int mvs_cvt_d(mvs_ctx* ctx, const uint8_t* rgbx, int V, int W, int H, float* lab, uint8_t* l8);

/* SLIC on V views of lab (clSLIC::do_super_pixel_seg, clSLIC.cpp:67-122,
 * minus the cvt it starts with).  spixl [V][mh][mw][8], labels [V][H][W].
 * lab is read only, except with p->edge_enable == 1, where the reference's
 * edge step overwrites it (as clSLIC's lab_img_dev).  Every spixl word is
 * written; s7 (disparity, untouched by the reference's SLIC on its zeroed
 * buffer) is set to 0. */
int mvs_slic_d(mvs_ctx* ctx, float* lab, int V, int W, int H, const mvs_slic_params* p,
               float* spixl, uint32_t* labels);

/* SLIC-off grid mode: init_cluster_centers + init_label_per_pixl
 * (clcode.cl:259-294, 341-353). */
int mvs_grid_d(mvs_ctx* ctx, const float* lab, int V, int W, int H, int S, float* spixl, uint32_t* labels);

/* find_super_pixel_boundary (clcode.cl:791-855; photo_consistency.cpp:88-110). */
int mvs_boundary_d(mvs_ctx* ctx, int V, int W, int H, int S, const float* spixl, const uint32_t* labels,
                   uint8_t* rep);

/* initial_depth_estimation_v2 for reference views [z0, z1): writes spixl.s7
 * (clcode.cl:972-1069; photo_consistency.cpp:113-140). */
int mvs_sweep_spixl_d(mvs_ctx* ctx, int W, int H, int S, const float* lab, float* spixl, const uint8_t* rep,
                      const mvs_array* a, int z0, int z1);

/* The same sweep evaluated at S=1 grid semantics (per-pixel SAD, reference
 * parity mode) without materialising spixl: disp [z1-z0][H][W]. */
int mvs_sweep_pixel_sad_d(mvs_ctx* ctx, int W, int H, const float* lab, const mvs_array* a, int z0, int z1,
                          float* disp);

/* Build-defined per-pixel NCC KxK plane sweep (definition: csrc/ncc.hip).
 * box int32 [2][V][Hp][W][2] (Hp = H rounded up to even; 16 B/px), from
 * mvs_box_stats_d, rows stored pairwise interleaved: plane 0 per row pair
 * (2m, 2m+1) and column x the float4 {a(2m), a(2m+1), b(2m), b(2m+1)} with
 * s = 1/sqrt(n*sum q^2 - (sum q)^2) (0 if textureless, NaN if the window
 * leaves the image), a = n*s, b = (sum q - 128 n)*s; plane 1 the centred
 * packed intensities q-128 of columns x-R .. x-R+7 of each pixel's row (two
 * little-endian dwords at uint2 index ((y>>1)*W + x)*2 + (y&1)).
 * vol [D][H][W] float cost of reference view z = 1 - max(-1, best NCC over
 * valid neighbour windows); l8 is validated only. */
int mvs_box_stats_d(mvs_ctx* ctx, const uint8_t* l8, int V, int W, int H, int K, int32_t* box);
/* The same planes for views [z0, z1) only of a V-view box buffer (a view shard
 * converts just its block and the block's neighbours). */
int mvs_box_stats_range_d(mvs_ctx* ctx, const uint8_t* l8, int V, int W, int H, int K, int z0, int z1,
                          int32_t* box);
int mvs_ncc_volume_d(mvs_ctx* ctx, int W, int H, const uint8_t* l8, const int32_t* box, const mvs_array* a,
                     int K, int z, float* vol);
/* Winner-take-all over vol [D][H][W]: disp = levels[first argmin], conf =
 * (min cost outside best+-1) - best cost.  conf may be NULL. */
int mvs_wta_d(mvs_ctx* ctx, int W, int H, int D, const float* vol, const float* levels, float* disp, float* conf);
/* mvs_ncc_volume_d + mvs_wta_d fused: the cost volume never reaches HBM.
 * disp/conf [H][W] are bit-identical to the two-pass result (levels from a->levels);
 * conf may be NULL. */
int mvs_ncc_wta_d(mvs_ctx* ctx, int W, int H, const uint8_t* l8, const int32_t* box, const mvs_array* a,
                  int K, int z, float* disp, float* conf);
/* mvs_ncc_wta_d for reference views [z0, z1) into disp/conf [z1 - z0][H][W]:
 * runs of views that share a sweep variant go in one launch (bit-identical to
 * one mvs_ncc_wta_d per view; clPhotoConsistency enqueues one sweep per
 * reference view, photo_consistency.cpp:133). */
int mvs_ncc_wta_range_d(mvs_ctx* ctx, int W, int H, const uint8_t* l8, const int32_t* box, const mvs_array* a,
                        int K, int z0, int z1, float* disp, float* conf);
/* Tuning / test hook: the NCC sweep variant this context tries first (0 =
 * automatic): waves per workgroup 4|8, levels per wave 1|2|4,
 * minimum LDS band width 64|80|96|128|192|256 columns, general_rows 1 = the kernel
 * that handles band rows starting on either row parity even when all start
 * on a pair.  Variants that do not fit the LDS fall back as in the default
 * chain.  mvs_ncc_last_variant reports the last launch as
 * {K, TH, levels per wave, waves, band width, row parity (0 mixed, 1 every band
 * row pair-aligned, 2 every pk row odd and stats row even), fused}: seven
 * int32 (the 0.5 report).  mvs_ncc_last_variant_n (0.7) writes the first
 * min(cap, 8) of those eight -- the eighth: band buffers (1 single-buffered,
 * 2 double-buffered) -- and returns 8, the slots it has. */
int mvs_set_ncc_variant(mvs_ctx* ctx, int waves, int levels_per_wave, int band_w, int general_rows);
int mvs_ncc_last_variant(mvs_ctx* ctx, int32_t* out7);
int mvs_ncc_last_variant_n(mvs_ctx* ctx, int32_t* out, int cap);
/* Kernel timing (a measurement aid, no reference counterpart): with timing on,
 * every fused NCC sweep launch (mvs_ncc_wta_d / mvs_ncc_wta_range_d) records
 * start / stop events of its own dispatch (hipExtLaunchKernel), so the time is
 * the kernel's alone -- an event recorded on the stream before a call can fire
 * while the previous kernel is still running.  mvs_kernel_times waits for the
 * recorded launches and returns their times in ms (*n = how many were
 * recorded), then starts a new record; switching timing on also does.  When
 * more launches were recorded than cap it fails (MVS_E_ARG) with *n set and the
 * record kept, so the caller can retry with a buffer of *n. */
int mvs_set_kernel_timing(mvs_ctx* ctx, int on);
int mvs_kernel_times(mvs_ctx* ctx, float* ms, int cap, int* n);

/* Superpixel-plane refinement (clDepthRefinement, depth_refinement.cpp:91-1470).
 * flat [V][mh][mw][2] and state/state2 [V][mh][mw][6] are caller-provided
 * workspaces; the final state is returned in *state (compat: see mvs_refine_params). */
int mvs_flatness_d(mvs_ctx* ctx, int V, int mw, int mh, const float* spixl, float gamma, float* flat);
int mvs_init_state_d(mvs_ctx* ctx, int W, int H, int S, const float* spixl, const uint32_t* labels,
                     const uint8_t* rep, const float* flat, const mvs_array* a, float gamma, float alpha,
                     int kernel_steps, float kss, float fuse, float* state);
/* init_current_state for views [z0, z1) only (state rows of other views untouched). */
int mvs_init_state_range_d(mvs_ctx* ctx, int W, int H, int S, const float* spixl, const uint32_t* labels,
                           const uint8_t* rep, const float* flat, const mvs_array* a, float gamma, float alpha,
                           int kernel_steps, float kss, float fuse, int z0, int z1, float* state);
int mvs_propagate_d(mvs_ctx* ctx, int W, int H, int S, const float* spixl, const uint32_t* labels,
                    const uint8_t* rep, const float* flat, const mvs_array* a, int iter, float alpha,
                    float gamma, float fuse, int kernel_steps, float kss, const float* st_in, float* st_out,
                    int z0, int z1);
int mvs_spixl_to_image_d(mvs_ctx* ctx, int V, int W, int H, int S, const float* spixl, const uint32_t* labels,
                         const float* state, float* disp);
/* ABI 0.5: the same three passes over 16-bit label maps (uint16 [V][H][W], the
 * view-sharded pipeline's narrowed labels all-gather; requires
 * mw * mh <= 65536, else MVS_E_ARG).  Results are identical to the uint32
 * entry points on the same label values. */
int mvs_init_state_range_l16_d(mvs_ctx* ctx, int W, int H, int S, const float* spixl, const uint16_t* labels,
                               const uint8_t* rep, const float* flat, const mvs_array* a, float gamma, float alpha,
                               int kernel_steps, float kss, float fuse, int z0, int z1, float* state);
int mvs_propagate_l16_d(mvs_ctx* ctx, int W, int H, int S, const float* spixl, const uint16_t* labels,
                        const uint8_t* rep, const float* flat, const mvs_array* a, int iter, float alpha,
                        float gamma, float fuse, int kernel_steps, float kss, const float* st_in, float* st_out,
                        int z0, int z1);
int mvs_spixl_to_image_l16_d(mvs_ctx* ctx, int V, int W, int H, int S, const float* spixl, const uint16_t* labels,
                             const float* state, float* disp);
int mvs_refine_d(mvs_ctx* ctx, int W, int H, int S, const float* spixl, const uint32_t* labels,
                 const uint8_t* rep, const mvs_array* a, const mvs_refine_params* p, float* flat,
                 float* state, float* state2, float* disp);

/* Cross-view consistency filter (clcode.cl:1995-2101, pinned order):
 * project_to_reference_inv for all views, then remove_view_inconsistency for
 * reference views [z0, z1).  proj/out [V][H][W]. */
int mvs_filter_d(mvs_ctx* ctx, int V, int W, int H, int array_width, float bl_ratio, float fuse,
                 const float* disp_full, float* proj, float* out, int z0, int z1);
/* The filter's two passes separately, for view sharding: project_to_reference_inv
 * (clcode.cl:1995-2034) writes proj slices [z0, z1); remove_view_inconsistency
 * (clcode.cl:2037-2101) for references [z0, z1) reads EVERY proj slice, so a
 * shard all-gathers proj in between.  mvs_filter_d == proj_inv(0, V) +
 * remove_inconsistency(z0, z1). */
int mvs_proj_inv_d(mvs_ctx* ctx, int V, int W, int H, int array_width, float bl_ratio, const float* disp_full,
                   float* proj, int z0, int z1);
int mvs_remove_inconsistency_d(mvs_ctx* ctx, int V, int W, int H, int array_width, float bl_ratio, float fuse,
                               const float* disp_full, const float* proj, float* out, int z0, int z1);
/* The same two passes over image rows [y0, y1) only (0 <= y0 <= y1 <= H), for
 * a shard that pipelines the proj all-gather in row bands: the removal at a
 * pixel reads the proj slices at that pixel only (clcode.cl:2054-2056), so a
 * band's removal can start once that band's proj rows have arrived.  The
 * disparity stack is read in full by both (reprojected gathers).  proj_band
 * 0: proj is the full [V][H][W] stack; 1: proj is the band alone,
 * [V][y1 - y0][W] (what a row band's all-gather delivers; the projection
 * writes its block's rows straight into the band buffer).  ABI 0.4: proj_band
 * added to mvs_proj_inv_rows_d. */
int mvs_proj_inv_rows_d(mvs_ctx* ctx, int V, int W, int H, int array_width, float bl_ratio, const float* disp_full,
                        float* proj, int proj_band, int z0, int z1, int y0, int y1);
int mvs_remove_inconsistency_rows_d(mvs_ctx* ctx, int V, int W, int H, int array_width, float bl_ratio, float fuse,
                                    const float* disp_full, const float* proj, int proj_band, float* out, int z0,
                                    int z1, int y0, int y1);

/* ---- host-pointer stage API (mirrors the reference stage methods) ------- */
/* clSLIC::do_super_pixel_seg(in_img, lab_out, spixl_out, idx_out), one view. */
int mvs_do_super_pixel_seg(mvs_ctx* ctx, const uint8_t* rgbx, int W, int H, const mvs_slic_params* p,
                           float* lab, float* spixl, uint32_t* labels);
/* clPhotoConsistency::do_initial_depth_estimation(spixl_inout, rep_out, lab,
 * idx, array_width, bl_ratio, view_subset, disp_levels), all V views. */
int mvs_do_initial_depth_estimation(mvs_ctx* ctx, int W, int H, int S, float* spixl, uint8_t* rep,
                                    const float* lab, const uint32_t* labels, const mvs_array* a);
/* clDepthRefinement(...)->do_refinement(...) + fusion output disp [V][H][W]. */
int mvs_do_refinement(mvs_ctx* ctx, int W, int H, int S, const float* spixl, const uint32_t* labels,
                      const uint8_t* rep, const mvs_array* a, const mvs_refine_params* p, float* state_out,
                      float* disp);

/* project_to_reference_inv + remove_view_inconsistency over all V views
 * (clcode.cl:1995-2101; the reference's disabled call site
 * depth_refinement.cpp:1398-1451), host pointers [V][H][W]. */
int mvs_do_consistency_filter(mvs_ctx* ctx, int V, int W, int H, int array_width, float bl_ratio, float fuse,
                              const float* disp_full, float* out);

#ifdef __cplusplus
}
#endif
#endif /* MVS_H */
