// Superpixel-plane refinement + fusion + cross-view filter for gfx950.
//
//  k_flatness        compute_flatness          clcode.cl:1076-1132
//  k_init_state      init_current_state        clcode.cl:1136-1404
//  k_propagate       propagate (+update, spatialRefinement, compute_smoothness,
//                    compute_consistency)       clcode.cl:1407-1900
//  k_spixl_to_image  spixl_to_image            clcode.cl:1906-1931
//  k_proj_inv /      project_to_reference_inv / remove_view_inconsistency
//  k_remove_incons   clcode.cl:1995-2101 (pinned order)
//
// Refinement is a latency-bound gather workload: one lane per
// (superpixel, view), candidate plane evaluations in the reference's order.
// The per-superpixel inputs are packed once per launch into 32-B records so a
// gather touches one cache line.  Numerics follow include/mvs_detmath.h.
#include <cstdlib>

#include "mvs_internal.h"

namespace mvs {
namespace {

struct RArgs {
  int V, W, H, S, mw, mh, aw;
  float bl, fuse, alpha, gamma;
};

__device__ __forceinline__ float expf_neg_sq(float diff, float k) { return mvs_expf(((-diff) * diff) * k); }

// roundf(v) as truncf(v + copysignf(0.49999997f, v)): equal for every non-NaN
// float (checked exhaustively over all 2^32 encodings, tests/test_oracle_cpu.py
// test_round_half_away_identity); 3 VALU instead of ~6.  NaN stays NaN.
__device__ __forceinline__ float round_ha(float v) {
  return truncf(v + copysignf(__int_as_float(0x3effffff), v));
}

// c - round_ha(v) as an int, for integral c: (int)(fc - round_ha(v)) without
// the float subtract and truncate.  Equal wherever either lands in an image
// ([0, 2^24)): round_ha(v) is then integral and exact, and outside it both are
// out of range (the convert saturates; NaN converts to 0 either way, and a NaN
// candidate votes 0 wherever it reads).
__device__ __forceinline__ int sub_round_ha(int c, float v) {
  return (int)((unsigned)c - (unsigned)(int)(v + copysignf(__int_as_float(0x3effffff), v)));
}

__device__ __forceinline__ float plane_at(float nx, float ny, float nz, float cx, float cy, float d, float px,
                                          float py) {
  float t = nx * (cx - px);
  t = t + ny * (cy - py);
  t = t + nz * d;
  return t / nz;
}

// plane_at with the divisor's reciprocal at hand (callers compute 1/nz once).
// The quotient is the IEEE division: a shared-reciprocal form (t*y, one FMA
// remainder, one FMA correction, IEEE fallback outside [1e-30, 1e30)) is
// bit-identical, but the compiler if-converts its fallback and evaluates the
// whole divide sequence for every lane anyway -- measured 1 % slower than the
// plain divide on the reference-defaults step (15.05 vs 14.90 ms), and 3 %
// slower with the fallback forced into a real branch.
__device__ __forceinline__ float plane_at_r(float nx, float ny, float nz, float rnz, float cx, float cy, float d,
                                            float px, float py) {
  (void)rnz;
  return plane_at(nx, ny, nz, cx, cy, d, px, py);
}

__device__ __forceinline__ int step_size_of(float flx, float kss) {
  int s = (int)((double)(flx * kss) + 0.5);
  return s > 1 ? s : 1;
}

// ---- compute_flatness ------------------------------------------------------
__global__ void k_flatness(const float* __restrict__ spixl, int mw, int mh, float gamma, float2* __restrict__ flat) {
  int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, z = blockIdx.z;
  if (x >= mw) return;
  long M = (long)mw * mh;
  long idx = M * z + (long)mw * y + x;
  const float* c0 = spixl + 8 * idx + 3;
  float fl = 1.0f;
  long nb[4] = {idx - 1, idx + 1, idx + mw, idx - mw};
  bool ok[4] = {x - 1 >= 0, x + 1 < mw, y + 1 < mh, y - 1 >= 0};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (!ok[k]) continue;
    const float* c1 = spixl + 8 * nb[k] + 3;
    float diff = (c1[0] - c0[0]) * (c1[0] - c0[0]);
    diff = diff + (c1[1] - c0[1]) * (c1[1] - c0[1]);
    diff = diff + (c1[2] - c0[2]) * (c1[2] - c0[2]);
    fl = fl + diff;
  }
  flat[idx] = make_float2(mvs_expf((-fl) * gamma), (float)(1.0 - mvs_exp((-0.25 * (double)fl) * (double)gamma)));
}

// ---- init_smoothness + initialize_consistency + init_current_state ---------
__device__ __forceinline__ float init_smoothness(const RArgs& c, const float* __restrict__ spixl, const float* sp, float2 fl, int x,
                                 int y, int z, int nks, float kss) {
  long M = (long)c.mw * c.mh;
  float sm = 0.0f, wn = 0.0f;
  float cl0 = sp[3], cl1 = sp[4], cl2 = sp[5], disp = sp[7];
  for (int i = -1; i <= 1; i++)
    for (int j = -1; j <= 1; j++) {
      int px = x + i, py = y + j;
      if (px >= 0 && py >= 0 && px < c.mw && py < c.mh && (i != 0 || j != 0)) {
        const float* s = spixl + 8 * (M * z + (long)c.mw * py + px);
        float diff = mvs_distance3(s[3], s[4], s[5], cl0, cl1, cl2);
        float simi = expf_neg_sq(diff, c.gamma);
        diff = disp - s[7];
        sm = sm + simi * expf_neg_sq(diff, c.alpha);
        wn = wn + simi;
      }
    }
  int ss = step_size_of(fl.x, kss);
  for (int i = 1; i <= nks; i++) {
    float gi = c.gamma * (float)(1 + i);
    int step = i * ss;
    int cx[4] = {x - (step + 1), x + (step + 1), x, x};
    int cy[4] = {y, y, y - step - 1, y + step + 1};
    bool ok[4] = {x > step, x < c.mw - step - 1, y > step, y < c.mh - step - 1};
    for (int k = 0; k < 4; k++) {
      if (!ok[k]) continue;
      const float* s = spixl + 8 * (M * z + (long)c.mw * cy[k] + cx[k]);
      float diff = mvs_distance3(cl0, cl1, cl2, s[3], s[4], s[5]);
      float simi = expf_neg_sq(diff, gi);
      diff = disp - s[7];
      sm = sm + simi * expf_neg_sq(diff, c.alpha);
      wn = wn + simi;
    }
  }
  return wn > 0 ? sm / wn : 0.000001f;
}

__device__ __forceinline__ void samples_of(const uint8_t* r, int* s) {
  s[0] = r[0]; s[1] = r[1]; s[2] = r[2]; s[3] = r[3]; s[4] = 0;
  s[5] = r[4]; s[6] = r[5]; s[7] = r[6]; s[8] = r[7];
}

__device__ __forceinline__ float finish_consistency(float cons, int vc) {
  float margin = 0.01f;
  return vc > 0 ? fmaxf(margin, cons / (float)vc) : margin;
}

// Label maps are uint32 (the reference's layout) or uint16 (LT): the
// view-sharded pipeline all-gathers them as 16-bit values when every label
// (< mw * mh <= 2^16) fits, and the refinement and fusion read them as they
// arrive instead of after a widening pass.
template <typename LT>
__device__ __forceinline__ uint32_t label_at(const void* labels, long i) {
  return ((const LT*)labels)[i];
}

template <typename LT>
__device__ __forceinline__ float init_consistency(const RArgs& c, const float* __restrict__ spixl, const void* __restrict__ labels,
                                  const uint8_t* rp, const int* __restrict__ vs, const int* __restrict__ sn, int z,
                                  const float* color, float cxf, float cyf, float d, float2 fl) {
  long M = (long)c.mw * c.mh, P = (long)c.W * c.H;
  float cons = 0.0f;
  int vc = 0;
  int camx = z % c.aw, camy = z / c.aw;
  int smp[9];
  samples_of(rp, smp);
  for (int n = 0; n < sn[z]; n++) {
    int view = vs[z * c.V + n];
    int vx = view % c.aw, vy = view / c.aw;
    float vis_w = 0.0f, occ_w = 0.0f, num = 0.0f, visibility = 0.0f, visible = 0.0f;
    // the view's 9 label gathers, then the 9 records they name, are issued
    // before the ordered sums (two memory latencies per view instead of 18);
    // record (ip % mw, ip / mw) is record ip
    bool okv[9];
    uint32_t ipv[9];
#pragma unroll
    for (int t = 0; t < 9; t++) {
      const int i = t / 3 - 1, j = t % 3 - 1;
      const int xr = (int)cxf + smp[t] * i;
      const int yr = (int)cyf + smp[t] * j;
      const int xp = (int)((float)xr - roundf(d * (float)(vx - camx)));
      const int yp = (int)((float)yr - roundf((c.bl * d) * (float)(vy - camy)));
      okv[t] = xp >= 0 && yp >= 0 && xp < c.W && yp < c.H;
      ipv[t] = label_at<LT>(labels, P * view + (okv[t] ? (long)c.W * yp + xp : 0));
    }
    float r3[9], r4[9], r5[9], r7[9];
#pragma unroll
    for (int t = 0; t < 9; t++) {
      const float* s = spixl + 8 * (M * view + (okv[t] ? (long)ipv[t] : 0));
      r3[t] = s[3]; r4[t] = s[4]; r5[t] = s[5]; r7[t] = s[7];
    }
#pragma unroll
    for (int t = 0; t < 9; t++) {
        if (okv[t]) {
          float diff = r7[t] - d;
          float wv = fabsf(diff) < c.fuse ? 1.0f : 0.0f;
          visible = visible + wv * expf_neg_sq(diff, c.alpha);
          vis_w = vis_w + wv;
          occ_w = occ_w + (1.0f - wv);
          diff = mvs_distance3(r3[t], r4[t], r5[t], color[0], color[1], color[2]);
          visibility = visibility + expf_neg_sq(diff, c.gamma);
          num = num + 1.0f;
        }
      }
    if (num > 0) {
      vc++;
      if (vis_w > 0) cons = cons + ((vis_w / num) * (visibility / vis_w)) * (visible / vis_w);
      if (occ_w > 0) cons = (float)((double)cons + 0.5 * (double)fl.y);
    }
  }
  return finish_consistency(cons, vc);
}

template <typename LT>
__global__ __launch_bounds__(256) void k_init_state(RArgs c, const float* __restrict__ spixl,
                                                    const void* __restrict__ labels,
                                                    const uint8_t* __restrict__ rep, const float2* __restrict__ flat,
                                                    const int* __restrict__ vs, const int* __restrict__ sn, int nks,
                                                    float kss, int z0, float* __restrict__ state) {
  int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, z = z0 + blockIdx.z;
  if (x >= c.mw) return;
  long M = (long)c.mw * c.mh;
  long idx = M * z + (long)c.mw * y + x;
  const float* sp = spixl + 8 * idx;
  float2 fl = flat[idx];
  float sm = init_smoothness(c, spixl, sp, fl, x, y, z, nks, kss);
  float color[3] = {sp[3], sp[4], sp[5]};
  float cs = init_consistency<LT>(c, spixl, labels, rep + 8 * idx, vs, sn, z, color, sp[1], sp[2], sp[7], fl);
  float* o = state + 6 * idx;
  o[0] = sp[7]; o[1] = sm; o[2] = cs; o[3] = 0.0f; o[4] = 0.0f; o[5] = 1.0f;
}

// ---- propagate -------------------------------------------------------------
struct PState {
  float d, sm, cs, nx, ny, nz;
};

struct PCtx {
  RArgs c;
  const float* spixl;
  const void* labels;  // uint32 or uint16 (the reader's LT)
  const int* vs;
  const int* sn;
  const float* st;
  int smp[9];
  int x, y, z, iter, nks;
  float kss;
  float cx, cy, col[3];
  float2 fl;
};

__device__ __forceinline__ float comp_smoothness(const PCtx& p, float d, float nx, float ny, float nz) {
  const RArgs& c = p.c;
  long M = (long)c.mw * c.mh;
  float sm = 0.0f, wn = 0.0f;
  for (int i = -1; i <= 1; i++)
    for (int j = -1; j <= 1; j++) {
      int px = p.x + i, py = p.y + j;
      if (px >= 0 && py >= 0 && px < c.mw && py < c.mh && (i != 0 || j != 0)) {
        long q = M * p.z + (long)c.mw * py + px;
        const float* s = p.spixl + 8 * q;
        float diff = mvs_distance3(p.col[0], p.col[1], p.col[2], s[3], s[4], s[5]);
        float simi = expf_neg_sq(diff, c.gamma);
        float di = plane_at(nx, ny, nz, p.cx, p.cy, d, s[1], s[2]);
        diff = di - p.st[6 * q];
        sm = sm + simi * expf_neg_sq(diff, c.alpha);
        wn = wn + simi;
      }
    }
  int ss = step_size_of(p.fl.x, p.kss);
  for (int i = 1; i <= p.nks; i++) {
    float gi = c.gamma * (float)(1 + i);
    int step = i * ss;
    int cxs[4] = {p.x - (step + 1), p.x + (step + 1), p.x, p.x};
    int cys[4] = {p.y, p.y, p.y - (step + 1), p.y + (step + 1)};
    bool ok[4] = {p.x > step, p.x < c.mw - step - 1, p.y > step, p.y < c.mh - step - 1};
    for (int k = 0; k < 4; k++) {
      if (!ok[k]) continue;
      long q = M * p.z + (long)c.mw * cys[k] + cxs[k];
      const float* s = p.spixl + 8 * q;
      float diff = mvs_distance3(s[3], s[4], s[5], p.col[0], p.col[1], p.col[2]);
      float simi = expf_neg_sq(diff, gi);
      float de = plane_at(nx, ny, nz, p.cx, p.cy, d, s[1], s[2]);
      diff = de - p.st[6 * q];
      sm = sm + simi * expf_neg_sq(diff, c.alpha);
      wn = wn + simi;
    }
  }
  return wn > 0 ? sm / wn : 0.000001f;
}

// compute_consistency (clcode.cl:1471-1565).  The candidate plane's disparity
// at the 9 sample points does not depend on the view: evaluated once.  Per
// view, all 9 label gathers are issued before the record gathers that depend
// on them, and the accumulation is branch-free (a sample outside the image
// leaves every sum unchanged), so the gathers overlap instead of forming 9
// round trips.  A label is the superpixel index y*mw + x, so the record is at
// view * M + label (the reference's % and / recombine to it exactly).
template <typename LT>
__device__ __forceinline__ float comp_consistency(const PCtx& p, float d, float nx, float ny, float nz) {
  const RArgs& c = p.c;
  const long M = (long)c.mw * c.mh, P = (long)c.W * c.H;
  float cons = 0.0f;
  int vc = 0;
  const int camx = p.z % c.aw, camy = p.z / c.aw;
  const int cxi = (int)p.cx, cyi = (int)p.cy;
  const float rnz = 1.0f / nz;
  float sxf[9], syf[9], di[9];
#pragma unroll
  for (int s = 0; s < 9; s++) {  // (i, j) = (s / 3 - 1, s % 3 - 1): i outer, j inner
    sxf[s] = (float)(cxi + p.smp[s] * (s / 3 - 1));
    syf[s] = (float)(cyi + p.smp[s] * (s % 3 - 1));
    di[s] = plane_at_r(nx, ny, nz, rnz, p.cx, p.cy, d, sxf[s], syf[s]);
  }
  for (int k = 0; k < p.sn[p.z]; k++) {
    const int view = p.vs[c.V * p.z + k];
    const float fdx = (float)(view % c.aw - camx), fdy = (float)(view / c.aw - camy);
    const long lv = P * view;
    int xp[9], yp[9];
    bool ok[9];
    uint32_t ip[9];
#pragma unroll
    for (int s = 0; s < 9; s++) {
      xp[s] = (int)(sxf[s] - roundf(di[s] * fdx));
      yp[s] = (int)(syf[s] - roundf((c.bl * di[s]) * fdy));
      ok[s] = xp[s] >= 0 && yp[s] >= 0 && xp[s] < c.W && yp[s] < c.H;
      ip[s] = label_at<LT>(p.labels, lv + (ok[s] ? (long)c.W * yp[s] + xp[s] : 0));
    }
    float vis_w = 0.0f, occ_w = 0.0f, num = 0.0f, visibility = 0.0f, visible = 0.0f;
#pragma unroll
    for (int s = 0; s < 9; s++) {
      const long q = M * view + ip[s];
      const float4 sa = *(const float4*)(p.spixl + 8 * q);      // s0..s3
      const float2 sb = *(const float2*)(p.spixl + 8 * q + 4);  // s4, s5
      const float* sq = p.st + 6 * q;
      const float2 t0 = *(const float2*)(sq);      // sq0 (d)
      const float2 t1 = *(const float2*)(sq + 2);  // sq3 (nx)
      const float2 t2 = *(const float2*)(sq + 4);  // sq4, sq5 (ny, nz)
      float dip = plane_at(t1.y, t2.x, t2.y, sa.y, sa.z, t0.x, (float)xp[s], (float)yp[s]);
      float diff = dip - di[s];
      const float wv = fabsf(diff) < c.fuse ? 1.0f : 0.0f;
      const float t_vis = wv * expf_neg_sq(diff, c.alpha);
      diff = mvs_distance3(sa.w, sb.x, sb.y, p.col[0], p.col[1], p.col[2]);
      const float t_col = expf_neg_sq(diff, c.gamma);
      if (ok[s]) {
        visible = visible + t_vis;
        vis_w = vis_w + wv;
        occ_w = occ_w + (1.0f - wv);
        visibility = visibility + t_col;
        num = num + 1.0f;
      }
    }
    if (num > 0) {
      vc++;
      if (vis_w > 0) cons = cons + ((vis_w / num) * (visibility / vis_w)) * (visible / vis_w);
      if (occ_w > 0) cons = (float)((double)cons + 0.5 * (double)p.fl.y);
    }
  }
  return finish_consistency(cons, vc);
}

// compute_consistency's per-sample terms dealt over a candidate's 8 lanes
// (k_propagate's lane-parallel phase): task = 9 * view slot + sample; lane r takes tasks
// r, r + 8, ... -- ceil(9 nv / 8) samples per lane instead of one view's 9, so
// a corner view (3 neighbours) keeps all 8 lanes busy.  The tasks run in
// batches of 3 (the label gathers of a batch issued before its record
// gathers) with a wave-uniform trip count ceil(ceil(9 nv / 8) / 3): 2 batches
// for nv <= 5, 3 for nv = 8 -- a fixed, predicated 9-task loop (the first
// form of this change) executed all 9 task slots for every view count and
// was 2 % slower than one view per lane.  Per task the view's camera offsets
// and the sample's offsets come from per-wave LDS tables; each sample's
// (t_vis, t_col) and (ok, wv) go to LDS, and view_sum adds a view's 9 samples
// in order (each view's sums start at 0, as in the reference).  Same
// arithmetic as comp_consistency, bit for bit.
template <typename LT>
__device__ __forceinline__ void view_tasks(const PCtx& p, int r, int L, int nv, const int2* toff,
                                           const float4* tview, const float* sdi, float2* samp, uint8_t* sflg) {
  const RArgs& c = p.c;
  const long M = (long)c.mw * c.mh, P = (long)c.W * c.H;
  const int cxi = (int)p.cx, cyi = (int)p.cy;
  const int ntask = 9 * nv;
  constexpr int TB = 3;  // tasks per batch (2 measured the same)
  const int nb = ((ntask + L - 1) / L + TB - 1) / TB;  // batches per lane (uniform)
  for (int b = 0; b < nb; b++) {
    int xp[TB], yp[TB], vw[TB];
    bool ok[TB];
    uint32_t ip[TB];
    float di[TB];
#pragma unroll
    for (int i = 0; i < TB; i++) {
      const int tk = r + L * (TB * b + i);
      xp[i] = yp[i] = vw[i] = 0;
      ok[i] = false;
      ip[i] = 0;
      di[i] = 0.0f;
      if (tk < ntask) {
        const int k = tk / 9, sm = tk - 9 * k;
        const int2 o = toff[sm];
        const float4 tv = tview[k];
        const int view = __float_as_int(tv.x);
        const float sxf = (float)(cxi + o.x), syf = (float)(cyi + o.y);
        di[i] = sdi[sm];  // the candidate plane at sample sm (view-independent, computed once)
        xp[i] = (int)(sxf - round_ha(di[i] * tv.y));
        yp[i] = (int)(syf - round_ha((c.bl * di[i]) * tv.z));
        ok[i] = xp[i] >= 0 && yp[i] >= 0 && xp[i] < c.W && yp[i] < c.H;
        ip[i] = label_at<LT>(p.labels, P * view + (ok[i] ? (long)c.W * yp[i] + xp[i] : 0));
        vw[i] = view;
      }
    }
#pragma unroll
    for (int i = 0; i < TB; i++) {
      const int tk = r + L * (TB * b + i);
      if (tk >= ntask) continue;
      const long q = M * vw[i] + ip[i];
      const float4 sa = *(const float4*)(p.spixl + 8 * q);
      const float2 sb = *(const float2*)(p.spixl + 8 * q + 4);
      const float* sq = p.st + 6 * q;
      const float2 t0 = *(const float2*)(sq);
      const float2 t1 = *(const float2*)(sq + 2);
      const float2 t2 = *(const float2*)(sq + 4);
      const float dip = plane_at(t1.y, t2.x, t2.y, sa.y, sa.z, t0.x, (float)xp[i], (float)yp[i]);
      float diff = dip - di[i];
      const bool wv = fabsf(diff) < c.fuse;
      const float t_vis = (wv ? 1.0f : 0.0f) * expf_neg_sq(diff, c.alpha);
      diff = mvs_distance3(sa.w, sb.x, sb.y, p.col[0], p.col[1], p.col[2]);
      samp[tk] = make_float2(t_vis, expf_neg_sq(diff, c.gamma));
      sflg[tk] = (uint8_t)((ok[i] ? 1 : 0) | (wv ? 2 : 0));
    }
  }
}
// one view's sums {num, vis_w, occ_w, visibility, visible} from its 9 task
// results, samples in order, finished into what compute_consistency adds for
// the view: o = {num, ((vis_w/num)*(visibility/vis_w))*(visible/vis_w) (0 if
// vis_w == 0), vis_w > 0, occ_w > 0} -- the three divides run here, one lane
// per view, instead of serially on the candidate's lane 8t
__device__ __forceinline__ void view_sum(const float2* samp, const uint8_t* sflg, float* o) {
  float vis_w = 0.0f, occ_w = 0.0f, num = 0.0f, visibility = 0.0f, visible = 0.0f;
#pragma unroll
  for (int s = 0; s < 9; s++) {
    const int f = sflg[s];
    if (f & 1) {
      const float2 v = samp[s];
      const float wv = (f & 2) ? 1.0f : 0.0f;
      visible = visible + v.x;
      vis_w = vis_w + wv;
      occ_w = occ_w + (1.0f - wv);
      visibility = visibility + v.y;
      num = num + 1.0f;
    }
  }
  o[0] = num;
  o[1] = vis_w > 0 ? ((vis_w / num) * (visibility / vis_w)) * (visible / vis_w) : 0.0f;
  o[2] = vis_w > 0 ? 1.0f : 0.0f;
  o[3] = occ_w > 0 ? 1.0f : 0.0f;
}

// One WAVE per superpixel.  The reference evaluates its candidate planes one
// after another, but a candidate's (sm, cs) never depends on the running
// state -- only the accept test does -- so lanes evaluate the candidates in
// parallel (plane candidates in batches of 64, then the 8 spatial-refinement
// triangles, whose normals use the post-plane depth) and the accept tests run
// in the reference's order over the broadcast results: bit-identical, with
// the superpixel count of waves in flight instead of that many threads.
// k is wave-uniform at every call: a v_readlane into an SGPR, not an LDS permute
constexpr int kTriViews = 8;  // views the lane-parallel triangle phase keeps in LDS
__device__ __forceinline__ float bcast(float v, int k) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}

// FAST: the host knows every superpixel of the launch takes the lane-parallel
// path (nks <= 13, so 9 + 4 nks <= 64 smoothness terms, and every view of
// [z0, z1) has <= kTriViews neighbours): the one-lane-per-candidate fallback is
// not compiled in, and its unrolled 9-sample consistency arrays no longer set
// the register allocation of the path that runs (reference defaults, C3, C4)
template <typename LT, bool FAST>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_propagate(RArgs c, const float* __restrict__ spixl,
                                                   const void* __restrict__ labels,
                                                   const uint8_t* __restrict__ rep, const float2* __restrict__ flat,
                                                   const int* __restrict__ vs, const int* __restrict__ sn, int iter,
                                                   int nks, float kss, const float* __restrict__ st_in,
                                                   float* __restrict__ st_out, int z0, long nsp) {
  const int lane = threadIdx.x & 63;
  const long g = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= nsp) return;  // whole wave; no barriers in this kernel
  const long M = (long)c.mw * c.mh;
  const int z = z0 + (int)(g / M);
  const int x = (int)(g % M) % c.mw, y = (int)(g % M) / c.mw;
  const long idx = M * z + (long)c.mw * y + x;
  PCtx p;
  p.c = c; p.spixl = spixl; p.labels = labels; p.vs = vs; p.sn = sn; p.st = st_in;
  p.x = x; p.y = y; p.z = z; p.iter = iter; p.nks = nks; p.kss = kss;
  const float* sp = spixl + 8 * idx;
  p.cx = sp[1]; p.cy = sp[2]; p.col[0] = sp[3]; p.col[1] = sp[4]; p.col[2] = sp[5];
  p.fl = flat[idx];
  samples_of(rep + 8 * idx, p.smp);
  const float* si = st_in + 6 * idx;
  PState cur{si[0], si[1], si[2], si[3], si[4], si[5]};

  // compute_smoothness terms (clcode.cl:1407-1470) whose neighbour, colour
  // similarity and neighbour depth do not depend on the candidate plane: lane t
  // holds term t (the 8 neighbours, then left/right/up/down at each far step),
  // computed once; each candidate then only evaluates its plane at the
  // neighbour centres.  Sums keep the reference's term order.
  const int ss = step_size_of(p.fl.x, kss);
  const int nterm = 9 + 4 * nks;
  const bool fast_sm = FAST || nterm <= 64;
  float t_simi = 0.f, t_sx = 0.f, t_sy = 0.f, t_sd = 0.f, wn = 0.f;
  unsigned long long t_valid = 0ull;
  if (fast_sm) {
    long q = -1;
    float gi = c.gamma;
    const int k = lane;
    if (k < 9) {
      const int i = k / 3 - 1, j = k % 3 - 1, px = x + i, py = y + j;
      if (px >= 0 && py >= 0 && px < c.mw && py < c.mh && (i != 0 || j != 0)) q = M * z + (long)c.mw * py + px;
    } else if (k < nterm) {
      const int i = (k - 9) / 4 + 1, dir = (k - 9) % 4, step = i * ss;
      gi = c.gamma * (float)(1 + i);
      const int qx[4] = {x - (step + 1), x + (step + 1), x, x};
      const int qy[4] = {y, y, y - (step + 1), y + (step + 1)};
      const bool ok[4] = {x > step, x < c.mw - step - 1, y > step, y < c.mh - step - 1};
      if (ok[dir]) q = M * z + (long)c.mw * qy[dir] + qx[dir];
    }
    if (q >= 0) {
      const float* sq = spixl + 8 * q;
      // neighbour terms: distance(own colour, neighbour); far terms the reverse (same bits)
      const float diff = k < 9 ? mvs_distance3(p.col[0], p.col[1], p.col[2], sq[3], sq[4], sq[5])
                               : mvs_distance3(sq[3], sq[4], sq[5], p.col[0], p.col[1], p.col[2]);
      t_simi = expf_neg_sq(diff, gi);
      t_sx = sq[1];
      t_sy = sq[2];
      t_sd = st_in[6 * q];
    }
    t_valid = __ballot(q >= 0);
    for (int l = 0; l < nterm; l++)
      if ((t_valid >> l) & 1ull) wn = wn + bcast(t_simi, l);
  }
  auto smooth = [&](float d, float nx, float ny, float nz) -> float {
    if (!fast_sm) return comp_smoothness(p, d, nx, ny, nz);
    float sm = 0.0f;
    const float rnz = 1.0f / nz;
    for (int l = 0; l < nterm; l++) {
      if (!((t_valid >> l) & 1ull)) continue;
      const float di = plane_at_r(nx, ny, nz, rnz, p.cx, p.cy, d, bcast(t_sx, l), bcast(t_sy, l));
      const float diff = di - bcast(t_sd, l);
      sm = sm + bcast(t_simi, l) * expf_neg_sq(diff, c.alpha);
    }
    return wn > 0 ? sm / wn : 0.000001f;
  };

  // plane candidates in the reference order (clcode.cl:1772-1805): the 8
  // neighbours, then for i = 1..nks up, down, left, right at offset i*(int)kss
  const int ssz = (int)kss;
  auto cand = [&](int k) -> long {  // superpixel of candidate slot k, -1 if out of the map
    if (k < 9) {
      const int i = k / 3 - 1, j = k % 3 - 1, px = x + i, py = y + j;
      return (px >= 0 && py >= 0 && px < c.mw && py < c.mh && !(i == 0 && j == 0)) ? M * z + (long)c.mw * py + px
                                                                                     : -1;
    }
    const int i = (k - 9) / 4 + 1, dir = (k - 9) % 4, off = i * ssz;
    if (dir == 0) return y > off ? M * z + (long)c.mw * (y - (off + 1)) + x : -1;
    if (dir == 1) return y < c.mh - off - 1 ? M * z + (long)c.mw * (y + off + 1) + x : -1;
    if (dir == 2) return x > off ? M * z + (long)c.mw * y + (x - off - 1) : -1;
    return x < c.mw - off - 1 ? M * z + (long)c.mw * y + (x + off + 1) : -1;
  };
  const int nslot = 9 + 4 * nks;
  const int nv = sn[z];
  if (FAST || (fast_sm && nv <= kTriViews)) {
    // Lane-parallel evaluation in groups of 8 candidates: lane 8t + r works
    // for candidate t of the group (L lanes per candidate in general: 8, or
    // more for a partial last group, see below).  The smoothness products simi_l * exp(...)
    // are computed by lanes r = l mod 8 into LDS and summed in term order by
    // lane 8t; each view's consistency sums (9 samples in order) by lane
    // r = view mod 8, combined in view order by lane 8t -- every float sum in
    // the reference's order, so bit-identical to the one-lane-per-candidate
    // forms kept below.  Groups: the valid plane candidates (compacted, slot
    // order), then the 8 spatial-refinement triangles (clcode.cl:1676-1723,
    // 1808-1820), whose normals use the depth after every plane candidate.
    // At S = 8 most far candidates leave the map, so one group of 8 neighbour
    // planes keeps all 64 lanes busy instead of 8.
    __shared__ float s_prod[4][8][64];
    __shared__ float s_view[4][8][kTriViews][4];
    __shared__ int s_slot[4][64];
    __shared__ float2 s_samp[4][8][9 * kTriViews];   // view_tasks results per candidate
    __shared__ uint8_t s_sflg[4][8][9 * kTriViews];
    __shared__ int2 s_toff[4][9];                     // sample offsets of this superpixel
    __shared__ float4 s_tview[4][kTriViews];          // {view, dx, dy} of each neighbour slot
    __shared__ int s_term[4][64];                     // the valid smoothness terms, in term order
    __shared__ float s_di[4][8][9];                   // the candidate's plane at the 9 sample points
    const int w = threadIdx.x >> 6;
    // compacted smoothness terms: the far terms that leave the superpixel map
    // (most of them at S = 8 in the first iterations: 61 terms, ~8 valid) take
    // no loop trips; products stored and summed by compacted index, i.e. in the
    // reference's term order over the valid terms
    const int nvt = __popcll(t_valid);
    if ((t_valid >> lane) & 1ull) s_term[w][__popcll(t_valid & ((1ull << lane) - 1ull))] = lane;
    if (lane < 9) {  // samples_of: extents 0..3, the centre, extents 4..7
      const int e = lane == 4 ? 0 : (int)rep[8 * idx + (lane < 4 ? lane : lane - 1)];
      s_toff[w][lane] = make_int2(e * (lane / 3 - 1), e * (lane % 3 - 1));
    }
    if (lane < nv) {
      const int view = vs[c.V * z + lane];
      s_tview[w][lane] = make_float4(__int_as_float(view), (float)(view % c.aw - z % c.aw),
                                     (float)(view / c.aw - z / c.aw), 0.0f);
    }
    const long qk = lane < nslot ? cand(lane) : -1;
    const unsigned long long vmask = __ballot(qk >= 0);
    if (qk >= 0) s_slot[w][__popcll(vmask & ((1ull << lane) - 1ull))] = lane;
    const int nvalid = __popcll(vmask);
    const int ngrp = (nvalid + 7) / 8;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int nbx[8] = {x - 1, x - 1, x, x + 1, x + 1, x + 1, x, x - 1};
    const int nby[8] = {y, y - 1, y - 1, y - 1, y, y + 1, y + 1, y + 1};
    for (int gi = 0; gi <= ngrp; gi++) {
      const bool tri = gi == ngrp;
      // lanes per candidate: 8, or 16 / 32 / 64 for a plane group of at most
      // 4 / 2 / 1 candidates (the last group: at S = 8 most iterations have 9-13
      // valid candidates, so a full group of 8 and a partial one)
      const int ncg = tri ? 8 : min(8, nvalid - 8 * gi);
      const int lg = ncg > 4 ? 3 : ncg > 2 ? 4 : ncg > 1 ? 5 : 6, L = 1 << lg;
      const int t = lane >> lg, r = lane & (L - 1);
      bool ok;
      float pd = cur.d, n0 = 0.f, n1 = 0.f, n2 = 1.f, ksimi = 0.f;
      if (!tri) {  // plane candidate: update(), clcode.cl:1635-1673, minus the accept test
        const int j = gi * 8 + t;
        ok = j < nvalid;
        if (ok) {
          const long q = cand(s_slot[w][j]);
          const float* s1 = st_in + 6 * q;
          n0 = s1[3]; n1 = s1[4]; n2 = s1[5];
          const float* sc = spixl + 8 * q;
          float tt = n0 * (sc[1] - p.cx);
          tt = tt + n1 * (sc[2] - p.cy);
          tt = tt + n2 * s1[0];
          pd = tt / n2;
          const float diff = mvs_distance3(p.col[0], p.col[1], p.col[2], sc[3], sc[4], sc[5]);
          ksimi = expf_neg_sq(diff, c.gamma);
        }
      } else {  // triangle t: normalize(cross(c_t - c, c_{t+1} - c)) at the current depth
        const int u = (t + 1) % 8;
        ok = nbx[t] > -1 && nby[t] > -1 && nbx[t] < c.mw && nby[t] < c.mh && nbx[u] > -1 && nby[u] > -1 &&
             nbx[u] < c.mw && nby[u] < c.mh;
        n2 = 0.f;
        if (ok) {
          const long q1 = M * z + (long)c.mw * nby[t] + nbx[t], q2 = M * z + (long)c.mw * nby[u] + nbx[u];
          const float* a1 = spixl + 8 * q1;
          const float* a2 = spixl + 8 * q2;
          const float v1x = a1[1] - p.cx, v1y = a1[2] - p.cy, v1z = st_in[6 * q1] - cur.d;
          const float v2x = a2[1] - p.cx, v2y = a2[2] - p.cy, v2z = st_in[6 * q2] - cur.d;
          n0 = v1y * v2z - v1z * v2y;
          n1 = v2x * v1z - v1x * v2z;
          n2 = v1x * v2y - v1y * v2x;
          float ss = n0 * n0;
          ss = ss + n1 * n1;
          ss = ss + n2 * n2;
          ss = ss + 0.0f * 0.0f;
          if (ss != 0.0f) {
            const float rr = sqrtf(ss);
            n0 = n0 / rr; n1 = n1 / rr; n2 = n2 / rr;
          }
        }
      }
      const float rn2 = 1.0f / n2;
      // smoothness products over the compacted valid terms; uniform trip count so
      // every lane takes part in the shuffles
      for (int i = 0; i < (nvt + L - 1) >> lg; i++) {
        const int j = r + L * i;
        const int ls = j < nvt ? s_term[w][j] : 0;
        const float simi = __shfl(t_simi, ls), sx = __shfl(t_sx, ls), sy = __shfl(t_sy, ls), sd = __shfl(t_sd, ls);
        if (ok && j < nvt) {
          const float di = plane_at_r(n0, n1, n2, rn2, p.cx, p.cy, pd, sx, sy);
          const float diff = di - sd;
          s_prod[w][t][j] = simi * expf_neg_sq(diff, c.alpha);
        }
      }
      // the candidate plane at the 9 sample points (plane_at_r, as comp_consistency)
      for (int sm = r; sm < 9; sm += L)
        if (ok) {
          const int2 o = s_toff[w][sm];
          s_di[w][t][sm] = plane_at_r(n0, n1, n2, rn2, p.cx, p.cy, pd, (float)((int)p.cx + o.x),
                                      (float)((int)p.cy + o.y));
        }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (ok) view_tasks<LT>(p, r, L, nv, s_toff[w], s_tview[w], s_di[w][t], s_samp[w][t], s_sflg[w][t]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (int k = r; k < nv; k += L)
        if (ok) view_sum(s_samp[w][t] + 9 * k, s_sflg[w][t] + 9 * k, s_view[w][t][k]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      float sm1 = 0.f, cs1 = 0.f;
      if (ok && r == 0) {
        float sm = 0.0f;
        for (int j = 0; j < nvt; j++) sm = sm + s_prod[w][t][j];
        sm1 = wn > 0 ? sm / wn : 0.000001f;
        float cons = 0.0f;
        int vc = 0;
        for (int k = 0; k < nv; k++) {
          const float* o = s_view[w][t][k];
          if (o[0] > 0) {  // num > 0
            vc++;
            if (o[2] != 0.0f) cons = cons + o[1];                               // vis_w > 0
            if (o[3] != 0.0f) cons = (float)((double)cons + 0.5 * (double)p.fl.y);  // occ_w > 0
          }
        }
        cs1 = finish_consistency(cons, vc);
      }
      // lane 8t's reads of this group's LDS sums are done before the next group writes
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const unsigned long long valid = __ballot(ok && r == 0);
      for (int l = 0; l < (64 >> lg); l++) {  // accept tests in candidate order
        if (!((valid >> (L * l)) & 1ull)) continue;
        const float ksm = bcast(sm1, L * l), kcs = bcast(cs1, L * l);
        if (!tri) {
          const float ksi = bcast(ksimi, L * l);
          if ((iter < 4 && ksm * ksi > cur.sm) || kcs * ksm > cur.sm * cur.cs) {
            cur.d = bcast(pd, L * l); cur.sm = ksm; cur.cs = kcs;
            cur.nx = bcast(n0, L * l); cur.ny = bcast(n1, L * l); cur.nz = bcast(n2, L * l);
          }
        } else if ((iter < 4 && ksm > cur.sm) || ksm * kcs > cur.sm * cur.cs) {
          cur.sm = ksm; cur.cs = kcs; cur.nx = bcast(n0, L * l); cur.ny = bcast(n1, L * l); cur.nz = bcast(n2, L * l);
        }
      }
    }
  } else if (!FAST) {
    // one lane per plane candidate, in batches of 64
    for (int b = 0; b < nslot; b += 64) {
      const int k = b + lane;
      const long q = k < nslot ? cand(k) : -1;
      float di = 0.f, sm1 = 0.f, cs1 = 0.f, simi = 0.f, nx = 0.f, ny = 0.f, nz = 1.f;
      if (q >= 0) {  // update(), clcode.cl:1635-1673, minus the accept test
        const float* s1 = st_in + 6 * q;
        nx = s1[3]; ny = s1[4]; nz = s1[5];
        const float* sc = spixl + 8 * q;
        float t = nx * (sc[1] - p.cx);
        t = t + ny * (sc[2] - p.cy);
        t = t + nz * s1[0];
        di = t / nz;
        sm1 = smooth(di, nx, ny, nz);
        cs1 = comp_consistency<LT>(p, di, nx, ny, nz);
        const float diff = mvs_distance3(p.col[0], p.col[1], p.col[2], sc[3], sc[4], sc[5]);
        simi = expf_neg_sq(diff, c.gamma);
      }
      const unsigned long long valid = __ballot(q >= 0);
      for (int l = 0; l < 64 && b + l < nslot; l++) {  // accept tests in order, on every lane
        if (!((valid >> l) & 1ull)) continue;
        const float ksm = bcast(sm1, l), kcs = bcast(cs1, l), ksi = bcast(simi, l);
        if ((iter < 4 && ksm * ksi > cur.sm) || kcs * ksm > cur.sm * cur.cs) {
          cur.d = bcast(di, l); cur.sm = ksm; cur.cs = kcs;
          cur.nx = bcast(nx, l); cur.ny = bcast(ny, l); cur.nz = bcast(nz, l);
        }
      }
    }

    // spatialRefinement, one lane per triangle
    {
      const int t = lane & 7;
      const int nbx[8] = {x - 1, x - 1, x, x + 1, x + 1, x + 1, x, x - 1};
      const int nby[8] = {y, y - 1, y - 1, y - 1, y, y + 1, y + 1, y + 1};
      const int u = (t + 1) % 8;
      const bool ok = lane < 8 && nbx[t] > -1 && nby[t] > -1 && nbx[t] < c.mw && nby[t] < c.mh && nbx[u] > -1 &&
                      nby[u] > -1 && nbx[u] < c.mw && nby[u] < c.mh;
      float sm1 = 0.f, cs1 = 0.f, n0 = 0.f, n1 = 0.f, n2 = 0.f;
      if (ok) {
        const long q1 = M * z + (long)c.mw * nby[t] + nbx[t], q2 = M * z + (long)c.mw * nby[u] + nbx[u];
        const float* a1 = spixl + 8 * q1;
        const float* a2 = spixl + 8 * q2;
        const float v1x = a1[1] - p.cx, v1y = a1[2] - p.cy, v1z = st_in[6 * q1] - cur.d;
        const float v2x = a2[1] - p.cx, v2y = a2[2] - p.cy, v2z = st_in[6 * q2] - cur.d;
        n0 = v1y * v2z - v1z * v2y;
        n1 = v2x * v1z - v1x * v2z;
        n2 = v1x * v2y - v1y * v2x;
        float ss = n0 * n0;
        ss = ss + n1 * n1;
        ss = ss + n2 * n2;
        ss = ss + 0.0f * 0.0f;
        if (ss != 0.0f) {
          const float rr = sqrtf(ss);
          n0 = n0 / rr; n1 = n1 / rr; n2 = n2 / rr;
        }
        sm1 = smooth(cur.d, n0, n1, n2);
        cs1 = comp_consistency<LT>(p, cur.d, n0, n1, n2);
      }
      const unsigned long long valid = __ballot(ok);
      for (int l = 0; l < 8; l++) {
        if (!((valid >> l) & 1ull)) continue;
        const float ksm = bcast(sm1, l), kcs = bcast(cs1, l);
        if ((iter < 4 && ksm > cur.sm) || ksm * kcs > cur.sm * cur.cs) {
          cur.sm = ksm; cur.cs = kcs; cur.nx = bcast(n0, l); cur.ny = bcast(n1, l); cur.nz = bcast(n2, l);
        }
      }
    }
  }
  if (lane == 0) {
    float* o = st_out + 6 * idx;
    o[0] = cur.d; o[1] = cur.sm; o[2] = cur.cs; o[3] = cur.nx; o[4] = cur.ny; o[5] = cur.nz;
  }
}

// ---- spixl_to_image ----------------------------------------------------------
template <typename LT>
__global__ void k_spixl_to_image(const float* __restrict__ spixl, const LT* __restrict__ labels,
                                 const float* __restrict__ st, int W, int H, int mw, int mh,
                                 float* __restrict__ disp) {
  int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, z = blockIdx.z;
  if (x >= W) return;
  long M = (long)mw * mh, P = (long)W * H;
  int id = (int)labels[P * z + (long)W * y + x];
  int sx = id % mw, sy = id / mw;
  long q = M * z + (long)mw * sy + sx;
  const float* s = spixl + 8 * q;
  const float* t = st + 6 * q;
  float v = t[3] * (s[1] - (float)x);
  v = v + t[4] * (s[2] - (float)y);
  v = v + t[5] * t[0];
  disp[P * z + (long)W * y + x] = v / t[5];
}

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x3 __attribute__((ext_vector_type(3)));

// The same map, 4 consecutive pixels per thread (W % 4 == 0): one 16-B (u32
// labels) or 8-B (u16) label load and one 16-B store per thread, the record gathers as buffer loads
// with 32-bit offsets inside view z's records (a label is the superpixel
// index sy * mw + sx, so the record is at M * z + label, as in
// comp_consistency).  Same arithmetic per pixel.
template <typename LT>
__global__ __launch_bounds__(256) void k_spixl_to_image4(const float* __restrict__ spixl,
                                                         const LT* __restrict__ labels,
                                                         const float* __restrict__ st, int W, int H, int mw, int mh,
                                                         float* __restrict__ disp) {
  const int x = 4 * (blockIdx.x * blockDim.x + threadIdx.x), y = blockIdx.y, z = blockIdx.z;
  if (x >= W) return;
  const long M = (long)mw * mh, P = (long)W * H, p = P * z + (long)W * y + x;
  const __amdgpu_buffer_rsrc_t rsp = __builtin_amdgcn_make_buffer_rsrc((void*)(spixl + 8 * M * z), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rst = __builtin_amdgcn_make_buffer_rsrc((void*)(st + 6 * M * z), 0, 0x7fffffff, 0x00020000);
  unsigned ids[4];
  if (sizeof(LT) == 4) {
    const uint4 id4 = *(const uint4*)(labels + p);
    ids[0] = id4.x, ids[1] = id4.y, ids[2] = id4.z, ids[3] = id4.w;
  } else {
    const uint2 id4 = *(const uint2*)(labels + p);
    ids[0] = id4.x & 0xffffu, ids[1] = id4.x >> 16, ids[2] = id4.y & 0xffffu, ids[3] = id4.y >> 16;
  }
  // three gathers per pixel, (x, y) of the centre, d, and the normal: the
  // kernel is bound by the gather instructions' address processing, not by
  // their bytes (six dword gathers per pixel: 0.17 ms at C4)
  float s1[4], s2[4], t0[4], t3[4], t4[4], t5[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int os = (int)ids[k] * 32, ot = (int)ids[k] * 24;
    const u32x2 sxy = __builtin_amdgcn_raw_buffer_load_b64(rsp, os + 4, 0, 0);
    const u32x3 tn = __builtin_amdgcn_raw_buffer_load_b96(rst, ot + 12, 0, 0);
    s1[k] = __uint_as_float(sxy.x);
    s2[k] = __uint_as_float(sxy.y);
    t0[k] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rst, ot, 0, 0));
    t3[k] = __uint_as_float(tn.x);
    t4[k] = __uint_as_float(tn.y);
    t5[k] = __uint_as_float(tn.z);
  }
  float o[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    float v = t3[k] * (s1[k] - (float)(x + k));
    v = v + t4[k] * (s2[k] - (float)y);
    v = v + t5[k] * t0[k];
    o[k] = v / t5[k];
  }
  *(float4*)(disp + p) = make_float4(o[0], o[1], o[2], o[3]);
}

// ---- cross-view filter -------------------------------------------------------
// Filter grid orders.  RM = false: (x tiles, rows, reference groups), so a
// reference group streams the whole disparity stack before the next one
// starts.  RM = true: (x tiles x reference groups, rows): every reference of
// a row band is in flight together, sharing the views' rows they gather
// around in L2.  Measured at C4 for k_remove_incons_q: 14.2 (RM) vs 14.6 ms.
struct FGrid {
  int xb, y, g;
};
template <bool RM>
__device__ __forceinline__ FGrid fgrid(int tiles_x, int y0) {
  if (RM) return {(int)blockIdx.x % tiles_x, y0 + (int)blockIdx.y, (int)blockIdx.x / tiles_x};
  return {(int)blockIdx.x, y0 + (int)blockIdx.y, (int)blockIdx.z};
}
// project_to_reference_inv: per (reference r, pixel) the running maximum md
// over the other views i of full[i] at the pixel projected with md itself
// (clcode.cl:1995-2034) -- a chain of dependent gathers, one thread per
// (reference, pixel).  Per-view buffer resources (scalar), so an out-of-image
// tap reads 0 through a load past the end and is skipped, as in the
// reference, without a branch.  Measured (C4, 32 references): 3.4 ms;
// issuing blocks of 4 / 8 views' gathers speculatively with the block's
// starting maximum (re-gathered once it moves) 4.1 / 4.4 ms, and a
// row-major grid (every reference of a row in flight together) 6.0 ms.
__global__ __launch_bounds__(256) void k_proj_inv(const float* __restrict__ full, int V, int W, int H, int aw,
                                                  float bl, int z0, float* __restrict__ proj, long PO, int ya) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = ya + blockIdx.y, r = z0 + blockIdx.z;
  if (x >= W) return;
  const long P = (long)W * H, p = (long)y * W + x;
  const int crx = r % aw, cry = r / aw;
  const float xf = (float)x, yf = (float)y;
  float md = full[P * r + p];
  // camera column / row of view i kept incrementally (scalar): i % aw and i / aw
  // per view were ~25 SALU instructions each, 0.86 G per C4 launch -- as many
  // SALU cycles per CU as the loop's VALU cycles per SIMD
  int cx = 0, cy = 0;
  const float* vb = full;
  for (int i = 0; i < V; i++, vb += P) {
    if (i != r) {
      const int xp = (int)(xf - round_ha(md * (float)(crx - cx)));
      const int yp = (int)(yf - round_ha((bl * md) * (float)(cry - cy)));
      const bool in = (unsigned)xp < (unsigned)W && (unsigned)yp < (unsigned)H;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)vb, 0, 0x7fffffff, 0x00020000);
      const int off = in ? (int)((unsigned)yp * (unsigned)W + (unsigned)xp) * 4 : 0x7fffffff;
      const float cd = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
      if (in && md < cd) md = cd;
    }
    if (++cx == aw) {
      cx = 0;
      cy++;
    }
  }
  proj[PO * r + p] = md;  // PO: proj's view stride (W H, or a band's rows x W)
}
__global__ void k_remove_incons(const float* __restrict__ proj, const float* __restrict__ full, int V, int W, int H,
                                int aw, float bl, float fuse, int z0, float* __restrict__ out, int y0, long PP) {
  int x = blockIdx.x * blockDim.x + threadIdx.x, y = y0 + blockIdx.y, r = z0 + blockIdx.z;
  if (x >= W) return;
  long P = (long)W * H, p = (long)y * W + x;
  int crx = r % aw, cry = r / aw;
  float dest = 0.0f;
  for (int i = 0; i < V; i++) {
    float d = proj[PP * i + p];
    if (d != 0) {
      float stab = 0.0f;
      for (int j = 0; j < V; j++) {
        float dc = proj[PP * j + p];
        if (dc != 0) {
          float diff = dc - d;
          if (fabsf(diff) > fuse) stab = stab - 1.0f;
          if (fabsf(diff) <= fuse) stab = stab + 1.0f;
        }
      }
      for (int j = 0; j < V; j++) {
        int cx = j % aw, cy = j / aw;
        int xx = (int)((float)x - roundf(d * (float)(cx - crx)));
        int yy = (int)((float)y - roundf((bl * d) * (float)(cy - cry)));
        if (xx >= 0 && yy >= 0 && xx < W && yy < H) {
          float dc = full[P * j + (long)W * yy + xx];
          float diff = dc - d;
          if (fabsf(diff) > fuse) stab = stab - 1.0f;
          if (fabsf(diff) < fuse) stab = stab + 1.0f;
        }
      }
      if (stab >= 0 && (dest == 0 || dest < d)) dest = d;
    }
  }
  out[P * r + p] = dest;
}

// The same output by candidate selection.  A candidate's stability depends
// only on its disparity d (and the pixel and reference view), and the
// reference keeps the largest d != 0 whose stability is >= 0 (its
// `dest == 0 || dest < d` update).  So the candidates are tried from the
// largest d down, every view holding that d retired together, and the first
// stable one is the answer: usually one or two stability evaluations per
// pixel instead of V, i.e. O(V) instead of O(V^2) work at V = 32 (C4).
// The views' camera offsets from the reference come from an LDS table (the
// block's reference is uniform), the reprojection rounds with round_ha and
// the gathers are 32-bit buffer loads (the launcher checks V * P * 4 < 2^31):
// the per-view integer divisions and 64-bit address arithmetic made the
// kernel VALU-bound (C3, V = 5: 443 us for 5 references).
template <int MAXV>
__global__ __launch_bounds__(256) void k_remove_incons_sel(const float* __restrict__ proj, const float* __restrict__ full,
                                                           int V, int W, int H, int aw, float bl, float fuse, int z0,
                                                           float* __restrict__ out, int y0, long PP) {
  __shared__ float2 s_off[MAXV];  // (float)(cx - crx), (float)(cy - cry) of view j
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = y0 + blockIdx.y, r = z0 + blockIdx.z;
  if ((int)threadIdx.x < MAXV)
    s_off[threadIdx.x] = make_float2((float)((int)threadIdx.x % aw - r % aw), (float)((int)threadIdx.x / aw - r / aw));
  __syncthreads();
  if (x >= W) return;
  const long P = (long)W * H, p = (long)y * W + x;
  const unsigned P4 = (unsigned)(P * 4);
  const float xf = (float)x, yf = (float)y;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)full, 0, 0x7fffffff, 0x00020000);
  float pv[MAXV];
  unsigned long long live = 0ull;  // candidates not yet tried: d != 0
#pragma unroll
  for (int i = 0; i < MAXV; i++) {
    pv[i] = i < V ? proj[PP * i + p] : 0.0f;
    if (pv[i] != 0) live |= 1ull << i;
  }
  float dest = 0.0f;
  while (live) {
    float d = 0.0f;
    bool any = false;
#pragma unroll
    for (int i = 0; i < MAXV; i++)
      if (((live >> i) & 1ull) && (!any || pv[i] > d)) { d = pv[i]; any = true; }
#pragma unroll
    for (int i = 0; i < MAXV; i++)
      if (pv[i] == d) live &= ~(1ull << i);
    float stab = 0.0f;
#pragma unroll
    for (int j = 0; j < MAXV; j++) {
      if (j < V && pv[j] != 0) {
        const float diff = pv[j] - d;
        if (fabsf(diff) > fuse) stab = stab - 1.0f;
        if (fabsf(diff) <= fuse) stab = stab + 1.0f;
      }
    }
    // each remaining view adds at most +1: stop once stab >= 0 is out of reach
    // (stab counts exactly, so this only skips work).  Views go in blocks of
    // 8 whose gathers are all in flight together; the bound is checked
    // between blocks (a few extra views at most, one round trip per block).
    const float bd = bl * d;
    for (int j0 = 0; j0 < V && stab + (float)(V - j0) >= 0.0f; j0 += 8) {
      float dc[8];
      bool in[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int j = j0 + u;
        const float2 o = s_off[j < MAXV ? j : 0];
        const int xx = (int)(xf - round_ha(d * o.x));
        const int yy = (int)(yf - round_ha(bd * o.y));
        in[u] = j < V && (unsigned)xx < (unsigned)W && (unsigned)yy < (unsigned)H;
        // every lane issues its load (a skipped tap reads 0 past the buffer)
        const int off = in[u] ? (int)((unsigned)j * P4 + (__umul24((unsigned)yy, (unsigned)W) + (unsigned)xx) * 4u)
                              : 0x7fffffff;
        dc[u] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        if (in[u]) {
          const float diff = dc[u] - d;
          if (fabsf(diff) > fuse) stab = stab - 1.0f;
          if (fabsf(diff) < fuse) stab = stab + 1.0f;
        }
      }
    }
    if (stab >= 0) {
      dest = d;
      break;
    }
  }
  out[P * r + p] = dest;
}

// Per-pixel form for several references at once.  A candidate's first
// stability term (the proj slices at the pixel) does not depend on the
// reference, so each thread owns one pixel: it sorts the V candidates once
// (bitonic network in registers, static indices), counts that term once per
// candidate, and then walks the sorted candidates for every reference of the
// shard -- the reference's answer is the largest d != 0 with stability >= 0.
// Measured at C4 (32 views): ~86 % of (reference, pixel) pairs have no stable
// candidate, so every candidate is tried; the selection kernel above repeats
// the O(V^2) candidate bookkeeping per reference and per try.
template <int N>
__device__ __forceinline__ void sort_desc(float (&v)[N]) {
#pragma unroll
  for (int k = 2; k <= N; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
      for (int i = 0; i < N; i++) {
        const int l = i ^ j;
        if (l > i) {
          const float a = v[i], b = v[l];
          const bool desc = (i & k) == 0;  // this half sorted descending
          v[i] = desc ? fmaxf(a, b) : fminf(a, b);
          v[l] = desc ? fminf(a, b) : fmaxf(a, b);
        }
      }
}

template <int MAXV, int FB>  // FB: views per gather block (gathers in flight together)
__global__ __launch_bounds__(256) void k_remove_incons_px(const float* __restrict__ proj, const float* __restrict__ full,
                                                          int V, int W, int H, int aw, float bl, float fuse, int z0,
                                                          int z1, float* __restrict__ out, int y0, long PP) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = y0 + blockIdx.y;
  if (x >= W) return;
  const long P = (long)W * H, p = (long)y * W + x;
  float pv[MAXV], sv[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; i++) {
    pv[i] = i < V ? proj[PP * i + p] : 0.0f;
    sv[i] = pv[i] != 0 ? pv[i] : -INFINITY;  // non-candidates sort last
  }
  sort_desc<MAXV>(sv);
  // first stability term of each sorted candidate (reference-independent)
  float A[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; k++) {
    float a = 0.0f;
#pragma unroll
    for (int j = 0; j < MAXV; j++) {
      if (j < V && pv[j] != 0) {
        const float diff = pv[j] - sv[k];
        if (fabsf(diff) > fuse) a = a - 1.0f;
        if (fabsf(diff) <= fuse) a = a + 1.0f;
      }
    }
    A[k] = a;
  }
  for (int r = z0; r < z1; r++) {
    const int crx = r % aw, cry = r / aw;
    float dest = 0.0f;
#pragma unroll
    for (int k = 0; k < MAXV; k++) {
      const float d = sv[k];
      if (d == -INFINITY) break;           // no candidates left
      if (k > 0 && d == sv[k - 1]) continue;  // views holding the same d: one evaluation
      float stab = A[k];
      for (int j0 = 0; j0 < V && stab + (float)(V - j0) >= 0.0f; j0 += FB) {
        float dc[FB];
        bool in[FB];
#pragma unroll
        for (int u = 0; u < FB; u++) {
          const int j = j0 + u;
          const int cx = j % aw, cy = j / aw;
          const int xx = (int)((float)x - roundf(d * (float)(cx - crx)));
          const int yy = (int)((float)y - roundf((bl * d) * (float)(cy - cry)));
          in[u] = j < V && xx >= 0 && yy >= 0 && xx < W && yy < H;
          dc[u] = in[u] ? full[P * j + (long)W * yy + xx] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < FB; u++) {
          if (in[u]) {
            const float diff = dc[u] - d;
            if (fabsf(diff) > fuse) stab = stab - 1.0f;
            if (fabsf(diff) < fuse) stab = stab + 1.0f;
          }
        }
      }
      if (stab >= 0) {
        dest = d;
        break;
      }
    }
    out[P * r + p] = dest;
  }
}

constexpr int RI_MAXV = 32;  // views of the per-lane queue walk

// The same answer with one work queue per lane.  The round-2 lock-step form
// (removed) walked candidates together: a wave runs every candidate until the LAST of its
// 64 lanes has given it up, so it pays, per candidate, the longest of the 64
// walks (measured at C4: 31.4 candidate rounds per wave against 20.5 per
// pixel, and most of a round's gather blocks idle).  Here each lane carries
// its own walk state and every pass of the loop does one gather block per
// slot: a lane whose candidate dies takes its next one in the next pass, so a
// wave runs the max over lanes of the passes a lane needs instead of the sum
// over candidates of the per-candidate maximum.
// NS slots per lane walk NS candidates at once (NS x FB gathers in flight per
// pass; the walk is bound by gather round trips, not by VALU).  Candidates
// are handed to the slots in descending order; `best` is the smallest index
// found stable so far, and a candidate above it is never started or is
// dropped -- the answer, the first stable candidate in descending order, is
// the reference's largest d != 0 with stability >= 0.
// Preparation (wave 0, registers with static indices): the proj values are
// sorted descending; the first stability term of candidate d is
// 2 C - nnz with C = #{nonzero pj : |RN(pj - d)| <= fuse}.  RN(pj - d) is
// monotone in pj, so in the sorted list that set is one contiguous run around
// d: it is counted in a window of +-RI_WIN neighbours, and counted in full
// (over the sorted list kept in LDS) when the run reaches the window's edge.
// Distinct candidates are compacted into LDS (views holding the same d: one
// evaluation).
// ROWB (aw % FB == 0): a gather block's FB views lie in one camera row, so
// their offsets are (kx + u, ky): one LDS read and one row projection per
// block.  Disparities are finite (as for the lds/px forms; NaN inputs: the
// generic k_remove_incons).
constexpr int RI_WIN = 5;
constexpr int8_t RI_OVER = -128;  // first term not yet counted (|term| <= 32)
// reference-independent per-pixel candidate lists (see k_remove_incons_q)
struct RiShared {
  float sv[RI_MAXV][64];  // distinct candidates, descending
  union {
    float srt[RI_MAXV][64];     // the sorted list (preparation only)
    uint32_t iv[RI_MAXV][64];   // then each distinct candidate's in-image camera offsets (ri_span_ends)
  };
  int8_t a[RI_MAXV][64];   // first stability term of each distinct candidate
  int nd[64];              // distinct candidates per pixel
};
// wave 0 of the workgroup, lane = pixel
__device__ __forceinline__ void ri_prep(RiShared& S, const float* __restrict__ proj, long P, long p, bool xin, int V,
                                        float fuse, int lane) {
  float sv[RI_MAXV];
  int nnz = 0;
#pragma unroll
  for (int j = 0; j < RI_MAXV; j++) {
    const float v = (xin && j < V) ? proj[P * j + p] : 0.0f;
    nnz += v != 0;
    sv[j] = v != 0 ? v : -INFINITY;  // non-candidates sort last
  }
  sort_desc<RI_MAXV>(sv);
#pragma unroll
  for (int j = 0; j < RI_MAXV; j++) S.srt[j][lane] = sv[j];
  int nd = 0;
#pragma unroll
  for (int k = 0; k < RI_MAXV; k++) {
    const float d = sv[k];
    if (k < nnz && (k == 0 || d != sv[k > 0 ? k - 1 : 0])) {
      int c = 0;
#pragma unroll
      for (int i = k - RI_WIN; i <= k + RI_WIN; i++)
        if (i >= 0 && i < RI_MAXV) c += (i < nnz && fabsf(sv[i] - d) <= fuse) ? 1 : 0;
      // the run reaches the window's edge.  (The empty asm keeps this
      // compiler from dropping the whole preparation: with both edge tests
      // feeding one boolean it deleted the loop at -O3, ROCm 7.2 clang.)
      int ov = 0;
      if (k - RI_WIN - 1 >= 0) ov |= fabsf(sv[k - RI_WIN - 1 >= 0 ? k - RI_WIN - 1 : 0] - d) <= fuse ? 1 : 0;
      if (k + RI_WIN + 1 < RI_MAXV)
        ov |= (k + RI_WIN + 1 < nnz && fabsf(sv[k + RI_WIN + 1 < RI_MAXV ? k + RI_WIN + 1 : 0] - d) <= fuse) ? 2 : 0;
      asm volatile("" : "+v"(ov));
      S.sv[nd][lane] = d;
      S.a[nd][lane] = ov != 0 ? RI_OVER : (int8_t)(2 * c - nnz);
      nd++;
    }
  }
  // runs reaching the window's edge (marked RI_OVER): counted in full over
  // the sorted list (each lane reads only its own column)
  for (int q = 0; q < nd; q++) {
    if (S.a[q][lane] != RI_OVER) continue;
    const float d = S.sv[q][lane];
    int c = 0;
    for (int i = 0; i < nnz; i++) c += fabsf(S.srt[i][lane] - d) <= fuse ? 1 : 0;
    S.a[q][lane] = (int8_t)(2 * c - nnz);
  }
  S.nd[lane] = nd;
}

// An upper bound on #{k in [k0, k1] : 0 <= p - round(fl(dd * k)) <= lim - 1},
// the camera columns (rows) whose reprojection of pixel coordinate p lands in
// the image.  round(v) in [p - lim + 1, p] needs v in [p - lim + 0.5, p + 0.5],
// and round(fl(dd * k)) is monotone in k, so the valid k are one interval;
// its ends come from one reciprocal with a 1e-3 margin (dd * k is within
// 2^-23 of the product, and only |k| <= 8 matters), so the count can only
// come out high.  dd != 0 (candidates are nonzero).
// The interval's ends do not depend on the reference view (k0, k1 do): they
// are computed once per (pixel, candidate) for the workgroup's references,
// as int8 (|k0|, |k1| < RI_MAXV, so clamping the ends to [-128, 127] changes
// no count), packed (ceil end, floor end) in the low 16 bits.
__device__ __forceinline__ uint32_t ri_span_ends(float dd, float p, int lim) {
  const float r = __builtin_amdgcn_rcpf(dd);
  float lo = (p - (float)lim + 0.5f) * r, hi = (p + 0.5f) * r;
  if (dd < 0.0f) {
    const float t = lo;
    lo = hi;
    hi = t;
  }
  lo = fminf(fmaxf(lo - 1e-3f, -128.0f), 127.0f);
  hi = fminf(fmaxf(hi + 1e-3f, -128.0f), 127.0f);
  return ((uint32_t)(int)ceilf(lo) & 0xffu) | ((uint32_t)(int)floorf(hi) & 0xffu) << 8;
}
__device__ __forceinline__ int ri_span_count(uint32_t e, int k0, int k1) {
  const int kl = max(k0, (int)(int8_t)(e & 0xffu)), kh = min(k1, (int)(int8_t)((e >> 8) & 0xffu));
  return max(0, kh - kl + 1);
}

template <int RG, int FB, int NS, bool ROWB, bool RM>
__global__ __launch_bounds__(64 * RG) void k_remove_incons_q(const float* __restrict__ proj,
                                                             const float* __restrict__ full, int V, int W, int H,
                                                             int aw, float bl, float fuse, int z0, int z1,
                                                             float* __restrict__ out, int y0, long PP, int inb) {
  __shared__ RiShared S;
  __shared__ float2 s_off[RG][RI_MAXV];  // per wave: view j's camera offset from the reference (dx, dy)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const FGrid fg = fgrid<RM>((W + 63) / 64, y0);
  const int x = fg.xb * 64 + lane, y = fg.y;
  const bool xin = x < W;
  const long P = (long)W * H, p = (long)y * W + (xin ? x : 0);
  {
    const int r = z0 + RG * fg.g + wave;
    if (lane < RI_MAXV)  // (float)(cx - crx), (float)(cy - cry) as the reference evaluates them
      s_off[wave][lane] = make_float2((float)(lane % aw - r % aw), (float)(lane / aw - r / aw));
  }
  if (wave == 0) ri_prep(S, proj, PP, p, xin, V, fuse, lane);
  __syncthreads();
  if (inb) {  // the candidates' in-image intervals (over srt: the preparation is done), dealt over the waves
    const int ndl = S.nd[lane];
    for (int q = wave; q < ndl; q += RG) {
      const float dv = S.sv[q][lane];
      S.iv[q][lane] = ri_span_ends(dv, (float)x, W) | ri_span_ends(bl * dv, (float)y, H) << 16;
    }
    __syncthreads();
  }
  const int r = z0 + RG * fg.g + wave;
  if (r >= z1 || !xin) return;  // after the barriers
  const unsigned P4 = (unsigned)(P * 4);  // the launcher checks V * P * 4 < 2^31
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)full, 0, 0x7fffffff, 0x00020000);
  const int nd = S.nd[lane];
  int best = nd;  // smallest candidate index found stable (nd: none yet)
  int nxt = 0;    // next candidate to hand to a slot
  int k[NS], j[NS], st[NS];
  int left[NS];     // upper bound on the in-image views the slot has still to visit
  unsigned jo[NS];  // j * P4: byte offset of view j
  float d[NS], bd[NS];
  // inb: the walk's bounds count only views whose reprojection is inside the
  // image (an outside one never votes): a candidate with a + (in-image views)
  // < 0 is given up without a gather, and a slot stops once its stability is
  // decided either way.  The camera grid is aw x (V / aw) (inb = 0 otherwise).
  const int cr = z0 + RG * fg.g + wave;
  const int crx = cr % aw, cry = cr / aw, ah = V / aw;
  auto bound = [&](int c) {
    if (!inb) return V;
    const uint32_t e = S.iv[c][lane];
    return ri_span_count(e, -crx, aw - 1 - crx) * ri_span_count(e >> 16, -cry, ah - 1 - cry);
  };
  auto take = [&](int s) {  // hand candidate nxt to slot s (k = nd: idle)
    k[s] = nd;
    while (nxt < best && nxt < nd) {
      const int c = nxt++;
      const float dv = S.sv[c][lane];
      const int a = S.a[c][lane];
      const float bdv = bl * dv;
      const int nb = bound(c);
      if (a + nb < 0) continue;  // unstable whatever the gathers say
      k[s] = c;
      d[s] = dv;
      st[s] = a;
      bd[s] = bdv;
      left[s] = nb;
      break;
    }
    j[s] = 0;
    jo[s] = 0;
  };
#pragma unroll
  for (int s = 0; s < NS; s++) take(s);
  while (k[0] < best || (NS > 1 && k[NS > 1 ? 1 : 0] < best)) {
    float dc[NS][FB];
    bool in[NS][FB];
#pragma unroll
    for (int s = 0; s < NS; s++) {
      const bool live = k[s] < best;
      if (ROWB) {
        const float2 o = s_off[wave][j[s]];
        const int yy = sub_round_ha(y, bd[s] * o.y);
        const bool yok = live && (unsigned)yy < (unsigned)H;
        const unsigned ro = jo[s] + __umul24((unsigned)yy, (unsigned)W) * 4u;
#pragma unroll
        for (int u = 0; u < FB; u++) {
          const int xx = sub_round_ha(x, d[s] * (u == 0 ? o.x : o.x + (float)u));  // dx integral: + 0 is exact
          in[s][u] = yok && j[s] + u < V && (unsigned)xx < (unsigned)W;
          // every lane issues its load (a skipped tap reads 0 past the buffer),
          // so the pass's gathers are in flight together
          const int off = in[s][u] ? (int)(ro + (unsigned)u * P4 + (unsigned)xx * 4u) : 0x7fffffff;
          dc[s][u] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
        }
      } else {
#pragma unroll
        for (int u = 0; u < FB; u++) {
          const float2 o = s_off[wave][min(j[s] + u, V - 1)];
          const int xx = sub_round_ha(x, d[s] * o.x);
          const int yy = sub_round_ha(y, bd[s] * o.y);
          in[s][u] = live && j[s] + u < V && (unsigned)xx < (unsigned)W && (unsigned)yy < (unsigned)H;
          const int off =
              in[s][u] ? (int)(jo[s] + (unsigned)u * P4 + (__umul24((unsigned)yy, (unsigned)W) + (unsigned)xx) * 4u) : 0x7fffffff;
          dc[s][u] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
        }
      }
    }
#pragma unroll
    for (int s = 0; s < NS; s++) {
#pragma unroll
      for (int u = 0; u < FB; u++) {
        const float ad = fabsf(dc[s][u] - d[s]);
        st[s] += in[s][u] ? (ad < fuse ? 1 : 0) - (ad > fuse ? 1 : 0) : 0;
        left[s] -= in[s][u] ? 1 : 0;
      }
      j[s] += FB;
      jo[s] += FB * P4;
    }
#pragma unroll
    for (int s = 0; s < NS; s++) {
      if (k[s] >= best) continue;
      // each remaining in-image view adds +1 at most and -1 at least: the
      // candidate is decided once stab >= 0 is out of reach or assured (stab
      // counts exactly: this only skips work).  left never undercounts: it
      // started at an upper bound and drops by the in-image views visited.
      const int rem = min(V - j[s], left[s]);
      const bool fin = j[s] >= V;
      if ((fin || st[s] - rem >= 0) && st[s] >= 0) {
        best = k[s];  // stable; every slot above it is dropped by the loop test
        k[s] = nd;
      } else if (fin || st[s] + rem < 0) {
        take(s);
      }
    }
  }
  out[P * r + p] = best < nd ? S.sv[best][lane] : 0.0f;
}

}  // namespace

int launch_flatness(hipStream_t s, int V, int mw, int mh, const float* spixl, float gamma, float* flat) {
  hipLaunchKernelGGL(k_flatness, dim3((mw + 63) / 64, mh, V), dim3(64), 0, s, spixl, mw, mh, gamma, (float2*)flat);
  MVS_LAUNCH_CHECK("k_flatness");
  return 0;
}

int launch_init_state(hipStream_t s, int V, int W, int H, int S, int aw, float bl, const float* spixl,
                      const void* labels, int lbits, const uint8_t* rep, const float* flat, const int* vs,
                      const int* sn, float gamma, float alpha, int nks, float kss, float fuse, float* state,
                      int z0, int z1) {
  if (z1 <= z0) return 0;
  RArgs c{V, W, H, S, map_dim(W, S), map_dim(H, S), aw, bl, fuse, alpha, gamma};
  hipLaunchKernelGGL(lbits == 16 ? k_init_state<uint16_t> : k_init_state<uint32_t>, dim3((c.mw + 63) / 64, c.mh, z1 - z0), dim3(64), 0, s, c, spixl, labels, rep,
                     (const float2*)flat, vs, sn, nks, kss, z0, state);
  MVS_LAUNCH_CHECK("k_init_state");
  return 0;
}

int launch_propagate(hipStream_t s, int V, int W, int H, int S, int aw, float bl, const float* spixl,
                     const void* labels, int lbits, const uint8_t* rep, const float* flat, const int* vs,
                     const int* sn, int iter, float alpha, float gamma, float fuse, int nks, float kss,
                     const float* st_in, float* st_out, int z0, int z1, int max_nbr) {
  if (z1 <= z0) return 0;
  RArgs c{V, W, H, S, map_dim(W, S), map_dim(H, S), aw, bl, fuse, alpha, gamma};
  const long nsp = (long)c.mw * c.mh * (z1 - z0);
  const bool fast = nks <= 13 && max_nbr <= kTriViews;  // see k_propagate's FAST
  auto kern = lbits == 16 ? (fast ? k_propagate<uint16_t, true> : k_propagate<uint16_t, false>)
                          : (fast ? k_propagate<uint32_t, true> : k_propagate<uint32_t, false>);
  hipLaunchKernelGGL(kern, dim3((unsigned)((nsp + 3) / 4)), dim3(256), 0, s, c, spixl, labels, rep,
                     (const float2*)flat, vs, sn, iter, nks, kss, st_in, st_out, z0, nsp);
  MVS_LAUNCH_CHECK("k_propagate");
  return 0;
}

int launch_spixl_to_image(hipStream_t s, int V, int W, int H, int S, const float* spixl, const void* labels,
                          int lbits, const float* state, float* disp) {
  int mw = map_dim(W, S), mh = map_dim(H, S);
  // the 4-pixel form needs aligned 4-label loads, 16-B aligned stores and
  // 32-bit record offsets
  const bool l16 = lbits == 16;
  const uintptr_t la = (uintptr_t)labels & (l16 ? 7 : 15);
  const bool four = W % 4 == 0 && (long)mw * mh * 32 < (1L << 31) && la == 0 && ((uintptr_t)disp & 15) == 0;
  const dim3 g4((W / 4 + 255) / 256, H, V), g1((W + 255) / 256, H, V);
  if (four && l16)
    hipLaunchKernelGGL(k_spixl_to_image4<uint16_t>, g4, dim3(256), 0, s, spixl, (const uint16_t*)labels, state, W, H,
                       mw, mh, disp);
  else if (four)
    hipLaunchKernelGGL(k_spixl_to_image4<uint32_t>, g4, dim3(256), 0, s, spixl, (const uint32_t*)labels, state, W, H,
                       mw, mh, disp);
  else if (l16)
    hipLaunchKernelGGL(k_spixl_to_image<uint16_t>, g1, dim3(256), 0, s, spixl, (const uint16_t*)labels, state, W, H,
                       mw, mh, disp);
  else
    hipLaunchKernelGGL(k_spixl_to_image<uint32_t>, g1, dim3(256), 0, s, spixl, (const uint32_t*)labels, state, W, H,
                       mw, mh, disp);
  MVS_LAUNCH_CHECK("k_spixl_to_image");
  return 0;
}

// project_to_reference_inv for reference views [z0, z1): proj slices z0..z1-1
int launch_proj_inv(hipStream_t s, int V, int W, int H, int aw, float bl, const float* full, float* proj, int z0,
                    int z1, int ya, int yb, bool band) {
  const int NR = yb - ya;  // rows [ya, yb) (the caller checks 0 <= ya <= yb <= H)
  if (z1 <= z0 || NR <= 0) return 0;
  // band: proj holds rows [ya, yb) only, [V][yb - ya][W] (as launch_remove_incons)
  const long PO = band ? (long)NR * W : (long)W * H;
  if (band) proj -= (long)ya * W;
  hipLaunchKernelGGL(k_proj_inv, dim3((W + 255) / 256, NR, z1 - z0), dim3(256), 0, s, full, V, W, H, aw, bl, z0, proj,
                     PO, ya);
  MVS_LAUNCH_CHECK("k_proj_inv");
  return 0;
}

// remove_view_inconsistency for reference views [z0, z1): reads every proj
// slice (all V must be filled) and the full disparity stack
int launch_remove_incons(hipStream_t s, int V, int W, int H, int aw, float bl, float fuse, const float* full,
                         const float* proj, float* out, int z0, int z1, int ya, int yb, bool band) {
  const int NR = yb - ya;  // rows [ya, yb) only (the caller checks 0 <= ya <= yb <= H)
  // band: proj holds rows [ya, yb) only, as [V][yb - ya][W] (the kernels index
  // proj[PP * view + y * W + x], so the band's base moves up by ya rows)
  const long PP = band ? (long)NR * W : (long)W * H;
  if (band) proj -= (long)ya * W;
  if (z1 > z0 && NR > 0) {
    const dim3 g((W + 255) / 256, NR, z1 - z0);
    const dim3 gp((W + 255) / 256, NR);
    // few views: one thread per (reference, pixel) keeps more threads in flight
    // (measured at V = 5: 350 vs 395 us); many views: one thread per pixel
    const bool off32 = (long)V * W * H * 4 < (1L << 31);  // 32-bit gather offsets (the sel / q kernels)
    if (V <= 8 && off32)
      hipLaunchKernelGGL(k_remove_incons_sel<8>, g, dim3(256), 0, s, proj, full, V, W, H, aw, bl, fuse, z0, out, ya, PP);
    else if (V <= 16)
      hipLaunchKernelGGL((k_remove_incons_px<16, 8>), gp, dim3(256), 0, s, proj, full, V, W, H, aw, bl, fuse, z0, z1,
                         out, ya, PP);
    else if (V <= 32 && (long)V * W * H * 4 < (1L << 31) &&
             !(getenv("MVS_FILTER_KERNEL") && std::string(getenv("MVS_FILTER_KERNEL")) == "px")) {
      // 32-bit gather offsets: one work queue per lane (k_remove_incons_q,
      // MVS_FILTER_NS candidates at once, MVS_FILTER_FB views per gather block,
      // both read per call); MVS_FILTER_KERNEL=px: the per-pixel form below.
      // Measured at C4, all 32 references with k_proj_inv
      // (scripts/bench_filter.py): q 18.1 ms (NS 2, FB 2); the lane-balanced
      // hand-out of (pixel, candidate) items 21.1 ms and the lock-step walk
      // 27.9 ms (both removed in round 3).
      constexpr int RG = 4;
      const dim3 gl((W + 63) / 64, NR, (z1 - z0 + RG - 1) / RG);
      {
        const char* fb = getenv("MVS_FILTER_FB");
        const int nfb = fb ? atoi(fb) : 2;
#define MVS_RIQ(FBV, NSV)                                                                                         \
  if (aw % FBV == 0 && rmo)                                                                                       \
    hipLaunchKernelGGL((k_remove_incons_q<RG, FBV, NSV, true, true>), glr, dim3(64 * RG), 0, s, proj, full, V, W, \
                       H, aw, bl, fuse, z0, z1, out, ya, PP, inb);                                                        \
  else if (aw % FBV == 0)                                                                                         \
    hipLaunchKernelGGL((k_remove_incons_q<RG, FBV, NSV, true, false>), gl, dim3(64 * RG), 0, s, proj, full, V, W, \
                       H, aw, bl, fuse, z0, z1, out, ya, PP, inb);                                                        \
  else if (rmo)                                                                                                   \
    hipLaunchKernelGGL((k_remove_incons_q<RG, FBV, NSV, false, true>), glr, dim3(64 * RG), 0, s, proj, full, V,   \
                       W, H, aw, bl, fuse, z0, z1, out, ya, PP, inb);                                                     \
  else                                                                                                            \
    hipLaunchKernelGGL((k_remove_incons_q<RG, FBV, NSV, false, false>), gl, dim3(64 * RG), 0, s, proj, full, V,   \
                       W, H, aw, bl, fuse, z0, z1, out, ya, PP, inb);
        // MVS_FILTER_BOUND=0 (read per call): the walk's bounds over every view (A/B)
        const char* fbd = getenv("MVS_FILTER_BOUND");
        const int inb = (V % aw == 0 && !(fbd && atoi(fbd) == 0)) ? 1 : 0;
        const bool rmo = !(getenv("MVS_FILTER_ORDER") && std::string(getenv("MVS_FILTER_ORDER")) == "ref");
        const dim3 glr(((W + 63) / 64) * ((z1 - z0 + RG - 1) / RG), NR);
        const char* ns = getenv("MVS_FILTER_NS");  // candidate slots per lane (1 | 2)
        const int nns = ns ? atoi(ns) : 2;
        if (nns == 1) {
          if (nfb == 4) {
            MVS_RIQ(4, 1)
          } else {
            MVS_RIQ(2, 1)
          }
        } else if (nfb == 4) {
          MVS_RIQ(4, 2)
        } else {
          MVS_RIQ(2, 2)
        }
#undef MVS_RIQ
      }
    } else if (V <= 32) {
      // MVS_FILTER_FB: views per gather block (A/B; read per call).  Measured at
      // C4 (scripts/bench_filter.py): blocks of 8 gathers 54 ms for all 32
      // references, 4: 35 ms, 2: 35 ms -- a candidate's early exit comes after
      // ~3 gathers, so 8-wide blocks fetched twice what the vote needed
      const char* fb = getenv("MVS_FILTER_FB");
      const int nfb = fb ? atoi(fb) : 4;
      if (nfb == 4)
        hipLaunchKernelGGL((k_remove_incons_px<32, 4>), gp, dim3(256), 0, s, proj, full, V, W, H, aw, bl, fuse, z0,
                           z1, out, ya, PP);
      else if (nfb == 2)
        hipLaunchKernelGGL((k_remove_incons_px<32, 2>), gp, dim3(256), 0, s, proj, full, V, W, H, aw, bl, fuse, z0,
                           z1, out, ya, PP);
      else
        hipLaunchKernelGGL((k_remove_incons_px<32, 8>), gp, dim3(256), 0, s, proj, full, V, W, H, aw, bl, fuse, z0,
                           z1, out, ya, PP);
    }
    else if (V <= 64 && off32)
      hipLaunchKernelGGL(k_remove_incons_sel<64>, g, dim3(256), 0, s, proj, full, V, W, H, aw, bl, fuse, z0, out, ya, PP);
    else
      hipLaunchKernelGGL(k_remove_incons, g, dim3(256), 0, s, proj, full, V, W, H, aw, bl, fuse, z0, out, ya, PP);
    MVS_LAUNCH_CHECK("k_remove_incons");
  }
  return 0;
}

// pinned order: every projection, then the removal
int launch_filter(hipStream_t s, int V, int W, int H, int aw, float bl, float fuse, const float* full,
                  float* proj, float* out, int z0, int z1) {
  int rc = launch_proj_inv(s, V, W, H, aw, bl, full, proj, 0, V, 0, H, false);
  if (rc) return rc;
  return launch_remove_incons(s, V, W, H, aw, bl, fuse, full, proj, out, z0, z1, 0, H, false);
}

}  // namespace mvs
