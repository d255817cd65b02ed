// Photo-consistency plane-sweep kernels for gfx950 (CDNA4, wave64).
//
//  k_boundary        find_super_pixel_boundary           clcode.cl:791-855
//  k_sweep_spixl     initial_depth_estimation_v2          clcode.cl:972-1069
//                    (one wave per superpixel, lanes over hypotheses,
//                    exact first-minimum WTA by a (cost, index) wave reduction)
//  k_sweep_pixel_sad the same sweep at S=1 grid semantics (reference-parity
//                    per-pixel mode): 32x32 output tile per workgroup, the
//                    per-tap absolute differences of one (d, neighbour) staged
//                    in LDS as (c, a) pairs so the reference's
//                    val+=30 / val-=30 / val+=AD sequence is three branch-free
//                    adds per tap, summed in the reference's window order.
//  (the NCC cost-volume kernels are in ncc.hip)
//  k_wta             winner-take-all + confidence over the materialised volume
//                    (the HBM-streaming pass the roofline is quoted on).
#include <cstdlib>

#include "mvs_internal.h"

namespace mvs {
namespace {

// ---- find_super_pixel_boundary, clcode.cl:791-855 -------------------------
__global__ void k_boundary(const float* __restrict__ spixl, const uint32_t* __restrict__ labels, int W, int H,
                           int S, int mw, int mh, uint8_t* __restrict__ rep) {
  int tx = blockIdx.x * blockDim.x + threadIdx.x, ty = blockIdx.y, z = blockIdx.z;
  if (tx >= mw) return;
  long M = (long)mw * mh, P = (long)W * H;
  long s = (long)ty * mw + tx;
  const float* sp = spixl + 8 * (z * M + s);
  int cx = (int)sp[1], cy = (int)sp[2];
  if (cx < S) cx += (S - cx);
  if (cx + S > W) cx -= S;
  if (cy < S) cy += (S - cy);
  if (cy + S > H) cy -= S;
  uint32_t id = (uint32_t)(ty * mw + tx);
  const uint32_t* L = labels + z * P;
  auto lbl = [&](int yy, int xx) -> uint32_t {
    return (yy >= 0 && yy < H && xx >= 0 && xx < W) ? L[(long)yy * W + xx] : 0xFFFFFFFFu;
  };
  uint32_t d0 = 0, d1 = 0, d2 = 0, d3 = 0, d4 = 0, d5 = 0, d6 = 0, d7 = 0;
  for (int i = 1; i < S; i++) {
    if (id == lbl(cy - i, cx - i) && cx - i >= 0 && cy - i >= 0) d0 = i - 1;
    if (id == lbl(cy, cx - i) && cx - i >= 0) d1 = i - 1;
    if (id == lbl(cy + i, cx - i) && cx - i >= 0 && cy + i < H) d2 = i - 1;
    if (id == lbl(cy - i, cx) && cy - i >= 0) d3 = i - 1;
    if (id == lbl(cy + i, cx) && cy + i < H) d4 = i - 1;
    if (id == lbl(cy - i, cx + i) && cx + i < W && cy - i >= 0) d5 = i - 1;
    if (id == lbl(cy, cx + i) && cx + i < W) d6 = i - 1;
    if (id == lbl(cy + i, cx + i) && cx + i < W && cy + i < H) d7 = i - 1;
  }
  uint2 packed;
  packed.x = (d0 & 0xff) | ((d1 & 0xff) << 8) | ((d2 & 0xff) << 16) | ((d3 & 0xff) << 24);
  packed.y = (d4 & 0xff) | ((d5 & 0xff) << 8) | ((d6 & 0xff) << 16) | ((d7 & 0xff) << 24);
  *(uint2*)(rep + 8 * (z * M + s)) = packed;
}

// ---- initial_depth_estimation_v2, clcode.cl:972-1069 ----------------------
struct SweepArgs {
  int V, W, H, mw, mh, D, aw, z;
  float bl;
};

// One workgroup = 4 waves; each superpixel is shared by wps waves (wps =
// ceil(D/64) up to 4), wave h taking levels lane + 64 (h + wps p), and all
// reference views of the call run in one launch (blockIdx.y), so the GPU is
// filled even at a few thousand superpixels per view.  The per-wave first
// minima are combined in (cost, index) lexicographic order -- the reference's
// strict-< scan over levels in index order -- through LDS.  LPS = 32 (D <= 32,
// e.g. the reference's default 31 levels): two superpixels per wave, one per
// 32-lane half, so no lane idles past the last level.
template <int LPS>
__global__ __launch_bounds__(256) void k_sweep_spixl(const float4* __restrict__ lab, float* __restrict__ spixl,
                                                     const uint8_t* __restrict__ rep,
                                                     const float* __restrict__ levels, const int* __restrict__ vs,
                                                     const int* __restrict__ sn, SweepArgs a, int wps) {
  __shared__ float4 refc[8][25];
  __shared__ int2 refxy[8][25];
  __shared__ float wbest[4];
  __shared__ int wbi[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ll = lane & (LPS - 1);                              // level lane within the superpixel's lanes
  const int spb = LPS == 64 ? 4 / wps : 8, h = LPS == 64 ? w % wps : 0;
  const int slot = LPS == 64 ? w / wps : 2 * w + (lane >> 5);  // superpixel of this block
  const int z = a.z + blockIdx.y;
  const long M = (long)a.mw * a.mh, P = (long)a.W * a.H;
  // XCD-aware order: blocks are dealt round-robin over the 8 XCDs; give each
  // XCD a contiguous run of superpixels so the neighbour rows its gathers
  // touch are shared within one L2 instead of being fetched by all eight
  const long nb = (M + spb - 1) / spb, per = (nb + 7) / 8;
  const long blk = (long)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  const long s = blk * spb + slot;
  const bool active = blk < nb && s < M && slot < spb;
  const long idx = z * M + (active ? s : 0);
  const uint8_t* dr = rep + 8 * idx;
  int bl_ = max((int)dr[0], max((int)dr[1], (int)dr[2]));
  int br_ = max((int)dr[5], max((int)dr[6], (int)dr[7]));
  int bt_ = max((int)dr[0], max((int)dr[3], (int)dr[5]));
  int bb_ = max((int)dr[2], max((int)dr[4], (int)dr[7]));
  float stx = (float)fmax(1.0, 0.25 * (double)(float)(bl_ + br_));
  float sty = (float)fmax(1.0, 0.25 * (double)(float)(bt_ + bb_));
  float cx = spixl[8 * idx + 1], cy = spixl[8 * idx + 2];
  const float4* labz = lab + (long)z * P;
  if (ll < 25 && (LPS == 32 || h == 0)) {
    int i = ll / 5 - 2, j = ll % 5 - 2;  // tap order: i (x) outer, j (y) inner
    int xr = (int)(cx + (float)i * stx);
    int yr = (int)(cy + (float)j * sty);
    refxy[slot][ll] = make_int2(xr, yr);
    bool in = xr >= 0 && yr >= 0 && xr < a.W && yr < a.H;
    refc[slot][ll] = in ? labz[(long)yr * a.W + xr] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  int rx = z % a.aw, ry = z / a.aw;
  int nn = sn[z];
  float best = 1000000.0f;
  int bi = 0x7fffffff;
  for (int dl = ll + LPS * h; dl < a.D; dl += LPS * wps) {
    float d = levels[dl];
    float mn = 1000000.0f;
    for (int n = 0; n < nn; n++) {
      int view = vs[a.V * z + n];
      int vx = view % a.aw, vy = view / a.aw;
      float fdx = d * (float)(vx - rx);
      float fdy = (a.bl * d) * (float)(vy - ry);
      const float4* labv = lab + (long)view * P;
      float val = 0.0f;
      // branch-free taps: every load is issued (out-of-image taps read pixel 0
      // and are dropped by the select), so the 25 gathers of a neighbour are
      // independent and in flight together instead of one per branch
#pragma unroll 5
      for (int t = 0; t < 25; t++) {
        int2 r = refxy[slot][t];
        int xp = (int)((float)r.x - fdx);
        int yp = (int)((float)r.y - fdy);
        const bool in = r.x >= 0 && r.y >= 0 && xp >= 0 && yp >= 0 && r.x < a.W && r.y < a.H && xp < a.W && yp < a.H;
        const float4 B = labv[in ? yp * a.W + xp : 0];
        const float4 A = refc[slot][t];
        float ad = fabsf(A.x - B.x) + fabsf(A.y - B.y);
        ad = ad + fabsf(A.z - B.z);
        const float v30 = val + 30.0f;  // the reference's val += 30; val -= 30; val += AD
        val = in ? (v30 - 30.0f) + ad : v30;
      }
      if (val < mn) mn = val;
    }
    if (mn < best) {
      best = mn;
      bi = dl;
    }
  }
  // first minimum across the superpixel's lanes: (cost, index) lexicographic
#pragma unroll
  for (int o = LPS / 2; o >= 1; o >>= 1) {
    float ob = __shfl_xor(best, o, 64);
    int oi = __shfl_xor(bi, o, 64);
    if (ob < best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  if (LPS == 32) {
    if (active && ll == 0) spixl[8 * idx + 7] = (bi != 0x7fffffff && best < 1000000.0f) ? levels[bi] : 0.0f;
    return;
  }
  if (lane == 0) {
    wbest[w] = best;
    wbi[w] = bi;
  }
  __syncthreads();
  if (active && h == 0 && lane == 0) {
    for (int k = 1; k < wps; k++) {
      const float ob = wbest[w + k];
      const int oi = wbi[w + k];
      if (ob < best || (ob == best && oi < bi)) {
        best = ob;
        bi = oi;
      }
    }
    spixl[8 * idx + 7] = (bi != 0x7fffffff && best < 1000000.0f) ? levels[bi] : 0.0f;
  }
}

// ---- per-pixel SAD sweep (S=1 grid semantics of initial_depth_estimation_v2)
constexpr int PT = 32;           // output tile edge
constexpr int PR = PT + 4;       // region edge (2-pixel halo)
constexpr int PREG = PR * PR;    // 1296 region pixels
constexpr int PPT = (PREG + 255) / 256;  // region pixels per thread (6)

__global__ __launch_bounds__(256) void k_sweep_pixel_sad(const float4* __restrict__ lab,
                                                         const float* __restrict__ levels,
                                                         const int* __restrict__ vs, const int* __restrict__ sn,
                                                         SweepArgs a, float* __restrict__ disp) {
  __shared__ float2 ca[PR][PR];  // (c, a): valid -> (30, AD), invalid -> (0, 0)
  const int tid = threadIdx.x;
  const int x0 = blockIdx.x * PT, y0 = blockIdx.y * PT;
  const long P = (long)a.W * a.H;
  const float4* labz = lab + (long)a.z * P;
  // reference colours of this thread's region pixels (constant over d, n)
  float3 rc[PPT];
  int rxy[PPT];
#pragma unroll
  for (int k = 0; k < PPT; k++) {
    int r = tid + 256 * k;
    int gx = x0 - 2 + r % PR, gy = y0 - 2 + r / PR;
    bool in = r < PREG && gx >= 0 && gy >= 0 && gx < a.W && gy < a.H;
    float4 c = in ? labz[(long)gy * a.W + gx] : make_float4(0.f, 0.f, 0.f, 0.f);
    rc[k] = make_float3(c.x, c.y, c.z);
    rxy[k] = in ? r : -1;
  }
  const int tx = tid & 31, ty0 = (tid >> 5) * 4;
  const int rx = a.z % a.aw, ry = a.z / a.aw;
  const int nn = sn[a.z];
  float cost[4], dsp[4];
#pragma unroll
  for (int o = 0; o < 4; o++) {
    cost[o] = 1000000.0f;
    dsp[o] = 0.0f;
  }
  for (int dl = 0; dl < a.D; dl++) {
    const float d = levels[dl];
    float mn[4];
#pragma unroll
    for (int o = 0; o < 4; o++) mn[o] = 1000000.0f;
    for (int n = 0; n < nn; n++) {
      const int view = vs[a.V * a.z + n];
      const int vx = view % a.aw, vy = view / a.aw;
      const float fdx = d * (float)(vx - rx);
      const float fdy = (a.bl * d) * (float)(vy - ry);
      const float4* labv = lab + (long)view * P;
      __syncthreads();  // previous (d, n) reads of ca done
#pragma unroll
      for (int k = 0; k < PPT; k++) {
        int r = tid + 256 * k;
        if (r < PREG) {
          float2 v = make_float2(0.0f, 0.0f);
          if (rxy[k] >= 0) {
            int gx = x0 - 2 + r % PR, gy = y0 - 2 + r / PR;
            int xp = (int)((float)gx - fdx);
            int yp = (int)((float)gy - fdy);
            if (xp >= 0 && yp >= 0 && xp < a.W && yp < a.H) {
              float4 B = labv[(long)yp * a.W + xp];
              float ad = fabsf(rc[k].x - B.x) + fabsf(rc[k].y - B.y);
              ad = ad + fabsf(rc[k].z - B.z);
              v = make_float2(30.0f, ad);
            }
          }
          ca[r / PR][r % PR] = v;
        }
      }
      __syncthreads();
      float val[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int i = 0; i < 5; i++) {  // window column (x offset) outer
        float2 col[8];
#pragma unroll
        for (int q = 0; q < 8; q++) col[q] = ca[ty0 + q][tx + i];
#pragma unroll
        for (int o = 0; o < 4; o++)
#pragma unroll
          for (int j = 0; j < 5; j++) {  // window row (y offset) inner
            float t = val[o] + 30.0f;
            t = t - col[o + j].x;
            val[o] = t + col[o + j].y;
          }
      }
#pragma unroll
      for (int o = 0; o < 4; o++)
        if (val[o] < mn[o]) mn[o] = val[o];
    }
#pragma unroll
    for (int o = 0; o < 4; o++)
      if (mn[o] < cost[o]) {
        cost[o] = mn[o];
        dsp[o] = d;
      }
  }
#pragma unroll
  for (int o = 0; o < 4; o++) {
    int x = x0 + tx, y = y0 + ty0 + o;
    if (x < a.W && y < a.H) disp[(long)y * a.W + x] = dsp[o];
  }
}

// ---- winner-take-all + confidence ----------------------------------------
// the 4 smallest (cost, level) of one pixel in lexicographic order
struct Top4 {
  float v0 = 1000000.0f, v1 = 1000000.0f, v2 = 1000000.0f, v3 = 1000000.0f;
  int i0 = -1, i1 = -1, i2 = -1, i3 = -1;
  __device__ __forceinline__ void insert(float cc, int ci) {
    if (cc < v3) {
      if (cc < v2) {
        v3 = v2; i3 = i2;
        if (cc < v1) {
          v2 = v1; i2 = i1;
          if (cc < v0) { v1 = v0; i1 = i0; v0 = cc; i0 = ci; }
          else { v1 = cc; i1 = ci; }
        } else { v2 = cc; i2 = ci; }
      } else { v3 = cc; i3 = ci; }
    }
  }
  __device__ __forceinline__ void emit(const float* levels, float* disp, float* conf, long p) const {
    disp[p] = i0 >= 0 ? levels[i0] : 0.0f;
    if (conf) {
      float c2 = 1000000.0f;
      if (i1 >= 0 && (i1 < i0 - 1 || i1 > i0 + 1)) c2 = v1;
      else if (i2 >= 0 && (i2 < i0 - 1 || i2 > i0 + 1)) c2 = v2;
      else if (i3 >= 0 && (i3 < i0 - 1 || i3 > i0 + 1)) c2 = v3;
      conf[p] = (i0 < 0 || c2 == 1000000.0f) ? 0.0f : c2 - v0;
    }
  }
};

// One lane per NP consecutive pixels (NP-wide non-temporal vector loads, so a
// wave streams 256 NP contiguous bytes per level), UNR levels in flight.
template <int NP, int UNR>
__global__ __launch_bounds__(256) void k_wta(const float* __restrict__ vol, const float* __restrict__ levels, long P,
                                             int D, float* __restrict__ disp, float* __restrict__ conf) {
  typedef float vec __attribute__((ext_vector_type(NP)));
  const long p = (blockIdx.x * (long)blockDim.x + threadIdx.x) * NP;
  if (p >= P) return;
  Top4 t[NP];
  const vec* col = (const vec*)(vol + p);
  const long Pv = P / NP;
  int dl = 0;
  for (; dl + UNR <= D; dl += UNR) {
    vec c[UNR];
#pragma unroll
    for (int u = 0; u < UNR; u++) c[u] = __builtin_nontemporal_load(col + (long)(dl + u) * Pv);
#pragma unroll
    for (int u = 0; u < UNR; u++)
#pragma unroll
      for (int k = 0; k < NP; k++) t[k].insert(c[u][k], dl + u);
  }
  for (; dl < D; dl++) {
    const vec c = col[(long)dl * Pv];
#pragma unroll
    for (int k = 0; k < NP; k++) t[k].insert(c[k], dl);
  }
#pragma unroll
  for (int k = 0; k < NP; k++) t[k].emit(levels, disp, conf, p + k);
}

}  // namespace

int launch_boundary(hipStream_t s, int V, int W, int H, int S, const float* spixl, const uint32_t* labels,
                    uint8_t* rep) {
  int mw = map_dim(W, S), mh = map_dim(H, S);
  hipLaunchKernelGGL(k_boundary, dim3((mw + 63) / 64, mh, V), dim3(64), 0, s, spixl, labels, W, H, S, mw, mh, rep);
  MVS_LAUNCH_CHECK("k_boundary");
  return 0;
}

int launch_sweep_spixl(hipStream_t s, int V, int W, int H, int S, const float* lab, float* spixl,
                       const uint8_t* rep, const float* levels, int D, const int* vs, const int* sn, int aw,
                       float bl, int z0, int z1) {
  if (z1 <= z0) return 0;
  int mw = map_dim(W, S), mh = map_dim(H, S);
  long M = (long)mw * mh;
  int wps = (D + 63) / 64;
  wps = wps >= 3 ? 4 : wps;  // waves per superpixel: 1, 2 or 4
  const bool half = D <= 32;  // two superpixels per wave
  const int spb = half ? 8 : 4 / wps;
  SweepArgs a{V, W, H, mw, mh, D, aw, z0, bl};
  const long nb = (M + spb - 1) / spb;
  hipLaunchKernelGGL(half ? k_sweep_spixl<32> : k_sweep_spixl<64>, dim3((unsigned)(8 * ((nb + 7) / 8)),
                     (unsigned)(z1 - z0)), dim3(256), 0, s, (const float4*)lab, spixl, rep, levels, vs, sn, a, wps);
  MVS_LAUNCH_CHECK("k_sweep_spixl");
  return 0;
}

int launch_sweep_pixel_sad(hipStream_t s, int V, int W, int H, const float* lab, const float* levels, int D,
                           const int* vs, const int* sn, const int* sn_host, int aw, float bl, int z0, int z1,
                           float* disp) {
  (void)sn_host;
  long P = (long)W * H;
  for (int z = z0; z < z1; z++) {
    SweepArgs a{V, W, H, W, H, D, aw, z, bl};
    hipLaunchKernelGGL(k_sweep_pixel_sad, dim3((W + PT - 1) / PT, (H + PT - 1) / PT), dim3(256), 0, s,
                       (const float4*)lab, levels, vs, sn, a, disp + (long)(z - z0) * P);
    MVS_LAUNCH_CHECK("k_sweep_pixel_sad");
  }
  return 0;
}

int launch_wta(hipStream_t s, int W, int H, int D, const float* vol, const float* levels, float* disp,
               float* conf) {
  long P = (long)W * H;
  // one pixel per lane, 8 levels in flight (wider per-lane vectors measured no faster)
  hipLaunchKernelGGL((k_wta<1, 8>), dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, vol, levels, P, D, disp,
                     conf);
  MVS_LAUNCH_CHECK("k_wta");
  return 0;
}

}  // namespace mvs
