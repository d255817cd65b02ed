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
//  k_box_stats       build-defined NCC: K x K window sums of l8 and l8^2
//  k_ncc_volume      build-defined NCC K x K cost volume: one wave = 64 image
//                    columns (64-2r outputs), rows slid in registers, the
//                    horizontal K-sum of q_ref*q_nbr by DPP wave shifts, integer
//                    sums (exact), IEEE f32 finish; cost = min over neighbours.
//  k_wta             winner-take-all + confidence over the materialised volume
//                    (the HBM-streaming pass the roofline is quoted on).
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

__global__ __launch_bounds__(256) void k_sweep_spixl(const float4* __restrict__ lab, float* __restrict__ spixl,
                                                     const uint8_t* __restrict__ rep,
                                                     const float* __restrict__ levels, const int* __restrict__ vs,
                                                     const int* __restrict__ sn, SweepArgs a) {
  __shared__ float4 refc[4][25];
  __shared__ int2 refxy[4][25];
  int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  long M = (long)a.mw * a.mh, P = (long)a.W * a.H;
  long s = (long)blockIdx.x * 4 + w;
  bool active = s < M;
  long idx = a.z * M + (active ? s : 0);
  const uint8_t* dr = rep + 8 * idx;
  int bl_ = max((int)dr[0], max((int)dr[1], (int)dr[2]));
  int br_ = max((int)dr[5], max((int)dr[6], (int)dr[7]));
  int bt_ = max((int)dr[0], max((int)dr[3], (int)dr[5]));
  int bb_ = max((int)dr[2], max((int)dr[4], (int)dr[7]));
  float stx = (float)fmax(1.0, 0.25 * (double)(float)(bl_ + br_));
  float sty = (float)fmax(1.0, 0.25 * (double)(float)(bt_ + bb_));
  float cx = spixl[8 * idx + 1], cy = spixl[8 * idx + 2];
  const float4* labz = lab + (long)a.z * P;
  if (lane < 25) {
    int i = lane / 5 - 2, j = lane % 5 - 2;  // tap order: i (x) outer, j (y) inner
    int xr = (int)(cx + (float)i * stx);
    int yr = (int)(cy + (float)j * sty);
    refxy[w][lane] = make_int2(xr, yr);
    bool in = xr >= 0 && yr >= 0 && xr < a.W && yr < a.H;
    refc[w][lane] = in ? labz[(long)yr * a.W + xr] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  int rx = a.z % a.aw, ry = a.z / a.aw;
  int nn = sn[a.z];
  float best = 1000000.0f;
  int bi = 0x7fffffff;
  for (int dl = lane; dl < a.D; dl += 64) {
    float d = levels[dl];
    float mn = 1000000.0f;
    for (int n = 0; n < nn; n++) {
      int view = vs[a.V * a.z + n];
      int vx = view % a.aw, vy = view / a.aw;
      float fdx = d * (float)(vx - rx);
      float fdy = (a.bl * d) * (float)(vy - ry);
      const float4* labv = lab + (long)view * P;
      float val = 0.0f;
#pragma unroll 5
      for (int t = 0; t < 25; t++) {
        int2 r = refxy[w][t];
        int xp = (int)((float)r.x - fdx);
        int yp = (int)((float)r.y - fdy);
        val = val + 30.0f;
        if (r.x >= 0 && r.y >= 0 && xp >= 0 && yp >= 0 && r.x < a.W && r.y < a.H && xp < a.W && yp < a.H) {
          val = val - 30.0f;
          float4 A = refc[w][t];
          float4 B = labv[(long)yp * a.W + xp];
          float ad = fabsf(A.x - B.x) + fabsf(A.y - B.y);
          ad = ad + fabsf(A.z - B.z);
          val = val + ad;
        }
      }
      if (val < mn) mn = val;
    }
    if (mn < best) {
      best = mn;
      bi = dl;
    }
  }
  // first minimum across lanes: (cost, index) lexicographic
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    float ob = __shfl_xor(best, o, 64);
    int oi = __shfl_xor(bi, o, 64);
    if (ob < best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  if (active && lane == 0) spixl[8 * idx + 7] = (bi != 0x7fffffff && best < 1000000.0f) ? levels[bi] : 0.0f;
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

// ---- NCC: window sums of l8 / l8^2 ----------------------------------------
__global__ void k_box_stats(const uint8_t* __restrict__ q, int W, int H, int K, int2* __restrict__ box) {
  int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, z = blockIdx.z;
  if (x >= W) return;
  int r = K / 2;
  long P = (long)W * H;
  const uint8_t* Q = q + z * P;
  int s = 0, ss = 0;
  if (x - r >= 0 && x + r < W && y - r >= 0 && y + r < H) {
    for (int j = -r; j <= r; j++)
      for (int i = -r; i <= r; i++) {
        int v = Q[(long)(y + j) * W + x + i];
        s += v;
        ss += v * v;
      }
  }
  box[z * P + (long)y * W + x] = make_int2(s, ss);
}

// ---- NCC K x K cost volume -----------------------------------------------
constexpr int kMaxNbr = 16;
struct NccArgs {
  int W, H, D, nn, z, d0, d1;
  int view[kMaxNbr];
  float fdx[kMaxNbr];  // dx as float
  float fdy[kMaxNbr];  // dy as float
  float bl;
};

__device__ __forceinline__ int hsum5(int p) {
  // P(l-2)+P(l-1)+P(l)+P(l+1)+P(l+2) with DPP wave shifts (symmetric, exact)
  int a1 = __builtin_amdgcn_update_dpp(0, p, 0x138, 0xf, 0xf, false);   // wave_shr:1
  int a2 = __builtin_amdgcn_update_dpp(0, a1, 0x138, 0xf, 0xf, false);
  int b1 = __builtin_amdgcn_update_dpp(0, p, 0x130, 0xf, 0xf, false);   // wave_shl:1
  int b2 = __builtin_amdgcn_update_dpp(0, b1, 0x130, 0xf, 0xf, false);
  return (((p + a1) + a2) + b1) + b2;
}
__device__ __forceinline__ int hsum7(int p) {
  int a1 = __builtin_amdgcn_update_dpp(0, p, 0x138, 0xf, 0xf, false);
  int a2 = __builtin_amdgcn_update_dpp(0, a1, 0x138, 0xf, 0xf, false);
  int a3 = __builtin_amdgcn_update_dpp(0, a2, 0x138, 0xf, 0xf, false);
  int b1 = __builtin_amdgcn_update_dpp(0, p, 0x130, 0xf, 0xf, false);
  int b2 = __builtin_amdgcn_update_dpp(0, b1, 0x130, 0xf, 0xf, false);
  int b3 = __builtin_amdgcn_update_dpp(0, b2, 0x130, 0xf, 0xf, false);
  return (((((p + a1) + a2) + a3) + b1) + b2) + b3;
}

template <int K, int TH>
__global__ __launch_bounds__(256) void k_ncc_volume(const uint8_t* __restrict__ q, const int2* __restrict__ box,
                                                    const float* __restrict__ levels_dev, NccArgs a,
                                                    float* __restrict__ vol) {
  constexpr int R = K / 2;
  constexpr int OUT = 64 - 2 * R;  // output columns per wave
  constexpr int NR = TH + 2 * R;   // rows streamed per (d, n)
  constexpr int NK = K * K;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int x = blockIdx.x * OUT - R + lane;
  const int yb = (blockIdx.y * 4 + wave) * TH;
  if (yb >= a.H) return;  // wave-uniform
  const long P = (long)a.W * a.H;
  const int W = a.W, H = a.H;
  const int xc = min(max(x, 0), W - 1);
  const uint8_t* Qz = q + (long)a.z * P;
  // reference column, rows yb-R .. yb+TH+R-1
  int qr[NR];
#pragma unroll
  for (int k = 0; k < NR; k++) {
    int yy = min(max(yb - R + k, 0), H - 1);
    qr[k] = Qz[(long)yy * W + xc];
  }
  const bool out_lane = lane >= R && lane < 64 - R && x < W;
  const bool xin = x >= R && x < W - R;
  int Sr[TH];
  float vrf[TH];
  unsigned rmask = 0;  // bit o: reference window valid and textured
  unsigned rvalid = 0;
#pragma unroll
  for (int o = 0; o < TH; o++) {
    int y = yb + o;
    int yc = min(y, H - 1);
    int2 b = box[(long)a.z * P + (long)yc * W + xc];
    Sr[o] = b.x;
    int vr = NK * b.y - b.x * b.x;
    vrf[o] = (float)vr;
    bool v = xin && y >= R && y < H - R;
    rvalid |= (v ? 1u : 0u) << o;
    rmask |= ((v && vr != 0) ? 1u : 0u) << o;
  }
  for (int dl = a.d0; dl < a.d1; dl++) {
    const float d = levels_dev[dl];
    float mn[TH];
#pragma unroll
    for (int o = 0; o < TH; o++) mn[o] = 1000000.0f;
    for (int n = 0; n < a.nn; n++) {
      const int tx = (int)roundf(d * a.fdx[n]);
      const int ty = (int)roundf((a.bl * d) * a.fdy[n]);
      const int xp = x - tx;
      const int xpc = min(max(xp, 0), W - 1);
      const bool xpin = xp >= R && xp < W - R;
      const uint8_t* Qv = q + (long)a.view[n] * P;
      const int2* Bv = box + (long)a.view[n] * P;
      // issue every load of this (d, n) first: clamped addresses, no branches
      int qpv[NR];
#pragma unroll
      for (int k = 0; k < NR; k++) {
        int yy = min(max(yb - R + k - ty, 0), H - 1);
        qpv[k] = Qv[(long)yy * W + xpc];
      }
      int2 bp[TH];
#pragma unroll
      for (int o = 0; o < TH; o++) {
        int yy = min(max(yb + o - ty, 0), H - 1);
        bp[o] = Bv[(long)yy * W + xpc];
      }
      int hs[NR];
#pragma unroll
      for (int k = 0; k < NR; k++) {
        int p = (int)__umul24(qr[k], qpv[k]);
        hs[k] = (K == 5) ? hsum5(p) : hsum7(p);
      }
      int srp = 0;
#pragma unroll
      for (int k = 0; k < 2 * R; k++) srp += hs[k];
#pragma unroll
      for (int o = 0; o < TH; o++) {
        srp += hs[o + 2 * R];
        const int yp = yb + o - ty;
        const bool pin = xpin && yp >= R && yp < H - R;
        // all factors < 2^24: 24-bit multiplies are full rate (v_mul_u32_u24)
        const int vp = NK * bp[o].y - (int)__umul24(bp[o].x, bp[o].x);
        const int num = NK * srp - (int)__umul24(Sr[o], bp[o].x);
        const float fa = (float)num;
        const float bb = fa * fabsf(fa);
        const float cc = vrf[o] * (float)vp;
        const float cost = 1.0f - bb / cc;
        const bool valid = ((rvalid >> o) & 1u) && pin;
        const bool textured = ((rmask >> o) & 1u) && vp != 0;
        const float c = !valid ? 2.0f : (!textured ? 1.0f : cost);
        mn[o] = c < mn[o] ? c : mn[o];
        srp -= hs[o];
      }
    }
    if (out_lane) {
      float* vd = vol + (long)dl * P;
#pragma unroll
      for (int o = 0; o < TH; o++) {
        int y = yb + o;
        if (y < H) vd[(long)y * W + x] = mn[o];
      }
    }
  }
}

// ---- winner-take-all + confidence ----------------------------------------
__global__ __launch_bounds__(256) void k_wta(const float* __restrict__ vol, const float* __restrict__ levels, long P,
                                             int D, float* __restrict__ disp, float* __restrict__ conf) {
  long p = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (p >= P) return;
  // 4 smallest (cost, index) in lexicographic order
  float v0 = 1000000.0f, v1 = 1000000.0f, v2 = 1000000.0f, v3 = 1000000.0f;
  int i0 = -1, i1 = -1, i2 = -1, i3 = -1;
  const float* col = vol + p;
  int dl = 0;
  for (; dl + 4 <= D; dl += 4) {
    float c[4];
#pragma unroll
    for (int u = 0; u < 4; u++) c[u] = __builtin_nontemporal_load(col + (long)(dl + u) * P);
#pragma unroll
    for (int u = 0; u < 4; u++) {
      float cc = c[u];
      int ci = dl + u;
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
  }
  for (; dl < D; dl++) {
    float cc = col[(long)dl * P];
    int ci = dl;
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
  disp[p] = i0 >= 0 ? levels[i0] : 0.0f;
  if (conf) {
    float c2 = 1000000.0f;
    if (i1 >= 0 && (i1 < i0 - 1 || i1 > i0 + 1)) c2 = v1;
    else if (i2 >= 0 && (i2 < i0 - 1 || i2 > i0 + 1)) c2 = v2;
    else if (i3 >= 0 && (i3 < i0 - 1 || i3 > i0 + 1)) c2 = v3;
    conf[p] = (i0 < 0 || c2 == 1000000.0f) ? 0.0f : c2 - v0;
  }
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
  int mw = map_dim(W, S), mh = map_dim(H, S);
  long M = (long)mw * mh;
  for (int z = z0; z < z1; z++) {
    SweepArgs a{V, W, H, mw, mh, D, aw, z, bl};
    hipLaunchKernelGGL(k_sweep_spixl, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, s, (const float4*)lab, spixl,
                       rep, levels, vs, sn, a);
    MVS_LAUNCH_CHECK("k_sweep_spixl");
  }
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

int launch_box_stats(hipStream_t s, const uint8_t* l8, int V, int W, int H, int K, int32_t* box) {
  hipLaunchKernelGGL(k_box_stats, dim3((W + 255) / 256, H, V), dim3(256), 0, s, l8, W, H, K, (int2*)box);
  MVS_LAUNCH_CHECK("k_box_stats");
  return 0;
}

int launch_ncc_volume(hipStream_t s, int V, int W, int H, const uint8_t* l8, const int32_t* box,
                      const float* levels_dev, int D, const int* vs_host, const int* sn_host, int aw, float bl,
                      int K, int z, float* vol) {
  constexpr int TH = 16;
  NccArgs a{};
  a.W = W; a.H = H; a.D = D; a.z = z; a.bl = bl;
  a.nn = sn_host[z];
  if (a.nn > kMaxNbr) return arg_fail("NCC sweep supports at most 16 neighbours per reference view");
  int rx = z % aw, ry = z / aw;
  for (int n = 0; n < a.nn; n++) {
    int v = vs_host[V * z + n];
    if (v < 0 || v >= V) return arg_fail("view_subset entry out of range");
    a.view[n] = v;
    a.fdx[n] = (float)(v % aw - rx);
    a.fdy[n] = (float)(v / aw - ry);
  }
  if (K != 5 && K != 7) return arg_fail("NCC window must be 5 or 7");
  int R = K / 2, OUT = 64 - 2 * R;
  // split the hypotheses so the grid holds enough waves to fill 256 CUs
  long tiles = (long)((W + OUT - 1) / OUT) * ((H + 4 * TH - 1) / (4 * TH));
  int chunks = (int)((4096 + tiles - 1) / tiles);
  if (chunks < 1) chunks = 1;
  if (chunks > D) chunks = D;
  int per = (D + chunks - 1) / chunks;
  for (int c = 0; c < chunks; c++) {
    a.d0 = c * per;
    a.d1 = min(D, (c + 1) * per);
    if (a.d0 >= a.d1) break;
    dim3 g((W + OUT - 1) / OUT, (H + 4 * TH - 1) / (4 * TH));
    if (K == 5)
      hipLaunchKernelGGL((k_ncc_volume<5, TH>), g, dim3(256), 0, s, l8, (const int2*)box, levels_dev, a, vol);
    else
      hipLaunchKernelGGL((k_ncc_volume<7, TH>), g, dim3(256), 0, s, l8, (const int2*)box, levels_dev, a, vol);
    MVS_LAUNCH_CHECK("k_ncc_volume");
  }
  return 0;
}

int launch_wta(hipStream_t s, int W, int H, int D, const float* vol, const float* levels, float* disp,
               float* conf) {
  long P = (long)W * H;
  hipLaunchKernelGGL(k_wta, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, vol, levels, P, D, disp, conf);
  MVS_LAUNCH_CHECK("k_wta");
  return 0;
}

}  // namespace mvs
