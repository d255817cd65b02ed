// SLIC superpixel kernels for gfx950 (CDNA4, wave64).
//
// Semantics restate clMVDE/clcode.cl (file:line at each kernel) under the
// numerical definition of include/mvs_detmath.h; layouts are the reference's.
// Design: pixel kernels are HBM-streaming (one lane per pixel, 16-B Lab
// loads/stores); the centre update is one workgroup per superpixel that walks
// the reference's 16x16 window tiles with one wave per tile and reproduces the
// reference LDS tree (stride 128..1) with two in-lane steps + six cross-lane
// shuffles, then sums the tile partials in tile order in the same workgroup
// (update_cluster_center and finalize_reduction_result fused: no accum_map
// round trip through HBM).
#include "mvs_internal.h"

namespace mvs {
namespace {

// mvs_powrf(x, third) (third = (float)(1/3): the definition's exp(third * log x)
// in double, rounded to float) for x in rgb2lab's range (0.008856, 1.09]
// without double arithmetic.  A = cbrt(x) * x^(third - 1/3) as an unevaluated
// float sum c + lo: c the hardware log2/exp2 estimate (relative error e0 ~
// 2^-22, two 1-ulp ops), lo = c (delta ln x) - (one Newton correction).  The
// correction's residual c^3 - x is formed exactly enough with FMAs (c^2 =
// p + pe exactly; p c - x rounded once, ~2^-44 x), so A's error is e0^2 plus
// the residual's and the reciprocal's roundings, together ~1.2e-13; the
// definition's double lies within ~1e-15 of x^third.  The float sums
// c + (lo -+ 1e-12 c) round A(1 -+ 1e-12) once each (their inner roundings
// move the ends by ~3e-14 c), so when they agree the definition rounds to
// the same float (rounding is monotone); otherwise (about 2 in 10^5 inputs)
// the definition itself is evaluated.  Checked on every 8-bit RGB colour --
// the kernel's whole input domain -- against the oracle
// (tests/test_gpu_parity.py).  (Round 4 formed A in double with two Newton
// steps: ~half of k_cvt's VALU.)
__device__ __forceinline__ float powr_third(float x) {
  const float l2 = __builtin_amdgcn_logf(x);  // log2 x, v_log_f32
  const float c = __builtin_amdgcn_exp2f(l2 * (1.0f / 3.0f));
  const float p = c * c;
  const float pe = fmaf(c, c, -p);                   // c^2 = p + pe
  const float r = fmaf(pe, c, fmaf(p, c, -x));       // c^3 - x
  const float dlt = r * __builtin_amdgcn_rcpf(3.0f * p);  // Newton: cbrt(x) = c - dlt
  constexpr float kDelta = (float)((double)(1.0f / 3.0f) - 1.0 / 3.0);  // 9.934e-9
  const float lo = fmaf(c, kDelta * (l2 * 0.693147182f), -dlt);     // A = c + lo
  const float m = 1e-12f * c;
  const float a0 = c + (lo - m), a1 = c + (lo + m);
  return a0 == a1 ? a0 : mvs_powrf(x, 1.0f / 3.0f);
}

// x / c for rgb2lab's constant divisors: q = x RN(1/c), its remainder by one
// FMA and one FMA correction -- the IEEE quotient for every operand rgb2lab
// forms (all 2^24 colours checked against the oracle's divisions,
// tests/test_gpu_parity.py test_cvt_every_rgb_colour), in 3 VALU instead of
// the ~10 of the general IEEE divide sequence
__device__ __forceinline__ float div_by(float x, float c, float rc) {
  const float q = x * rc;
  return fmaf(fmaf(-q, c, x), rc, q);
}

// ---- rgb2lab + cvt, clcode.cl:21-59, 125-151 (s0 read as blue) -----------
__device__ __forceinline__ float4 rgb2lab(uint32_t px) {
  float _b = (float)(px & 0xffu) * 0.0039216f;
  float _g = (float)((px >> 8) & 0xffu) * 0.0039216f;
  float _r = (float)((px >> 16) & 0xffu) * 0.0039216f;
  float x = _r * 0.412453f + _g * 0.357580f + _b * 0.180423f;
  float y = _r * 0.212671f + _g * 0.715160f + _b * 0.072169f;
  float z = _r * 0.019334f + _g * 0.119193f + _b * 0.950227f;
  const float epsilon = 0.008856f, kappa = 903.3f;
  float xr = div_by(x, 0.950456f, 1.0f / 0.950456f), yr = y, zr = div_by(z, 1.088754f, 1.0f / 1.088754f);
  const float third = 1.0f / 3.0f;
  (void)third;  // powr_third(v) == mvs_powrf(v, third)
  float fx = xr > epsilon ? powr_third(xr) : div_by(kappa * xr + 16.0f, 116.0f, 1.0f / 116.0f);
  float fy = yr > epsilon ? powr_third(yr) : div_by(kappa * yr + 16.0f, 116.0f, 1.0f / 116.0f);
  float fz = zr > epsilon ? powr_third(zr) : div_by(kappa * zr + 16.0f, 116.0f, 1.0f / 116.0f);
  return make_float4(116.0f * fy - 16.0f, 500.0f * (fx - fy), 200.0f * (fy - fz), 0.0f);
}

// Each wave converts 256 consecutive pixels per pass, lane l taking pixels
// l, l + 64, l + 128, l + 192: four independent conversions in flight per
// thread, every load and store still wave-contiguous.
__global__ __launch_bounds__(256) void k_cvt(const uint32_t* __restrict__ rgbx, long n, float4* __restrict__ lab,
                                             uint8_t* __restrict__ l8) {
  const long stride = (long)gridDim.x * 1024;
  for (long c = ((long)blockIdx.x * 256 + (threadIdx.x & ~63)) * 4 + (threadIdx.x & 63); c < n; c += stride) {
    uint32_t px[4];
#pragma unroll
    for (int u = 0; u < 4; u++) px[u] = c + 64 * u < n ? __builtin_nontemporal_load(rgbx + c + 64 * u) : 0u;
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const long i = c + 64 * u;
      if (i >= n) break;
      const float4 v = rgb2lab(px[u]);
      lab[i] = v;
      if (l8) {
        // build-defined NCC intensity: clamp((int)(L*2.55f + 0.5f), 0, 255)
        float t = v.x * 2.55f;
        t = t + 0.5f;
        const int q = (int)t;
        l8[i] = (uint8_t)(q < 0 ? 0 : (q > 255 ? 255 : q));
      }
    }
  }
}

// ---- init_cluster_centers, clcode.cl:259-294 -----------------------------
__global__ void k_init_centers(const float4* __restrict__ lab, int W, int H, int S, int mw, int mh,
                               float* __restrict__ spixl) {
  int col = blockIdx.x * blockDim.x + threadIdx.x, row = blockIdx.y, z = blockIdx.z;
  if (col >= mw || row >= mh) return;
  int ci = row * mw + col;
  int cx = col * S + S / 2, cy = row * S + S / 2;
  if (cx > W) cx = (col * S + W) / 2;
  if (cy > H) cy = (row * S + H) / 2;
  long P = (long)W * H;
  float* o = spixl + 8 * ((long)z * mw * mh + ci);
  o[0] = (float)ci;
  o[1] = (float)cx;
  o[2] = (float)cy;
  long p = (long)cy * W + cx;  // cx == W reads the next row (reference); past the end pinned to 0
  float4 c = p < P ? lab[(long)z * P + p] : make_float4(0.f, 0.f, 0.f, 0.f);
  o[3] = c.x;
  o[4] = c.y;
  o[5] = c.z;
  o[6] = 0.0f;
  o[7] = 0.0f;  // s7 (disparity) is never written by the reference's SLIC: its buffer starts at 0
}

// ---- edge_compute_alternative, clcode.cl:161-195 -------------------------
// Magnitude of the reference's Sobel-like operator over the clamped 3x3
// neighbourhood (its DX uses the centre c4 where a Sobel has c8: kept), left
// to right without contraction; dot(v, 1) = (v.x + v.y) + v.z.  Written to
// `edge` (the reference writes cvt_img in place while other work-items still
// read it; here every read precedes the store pass k_edge_store).
__global__ __launch_bounds__(256) void k_edge(const float4* __restrict__ lab, int W, int H,
                                              float* __restrict__ edge) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, z = blockIdx.z;
  if (x >= W) return;
  const float4* L = lab + (long)z * W * H;
  float4 c[9];
#pragma unroll
  for (int yo = -1; yo <= 1; yo++)
#pragma unroll
    for (int xo = -1; xo <= 1; xo++) {
      const int xx = min(max(x + xo, 0), W - 1), yy = min(max(y + yo, 0), H - 1);
      c[(yo + 1) * 3 + xo + 1] = L[(long)yy * W + xx];
    }
  auto mag2 = [&](float c0, float c1, float c2, float c3, float c4, float c5, float c6, float c7) {
    float dx = -1.0f * c0 + c2;
    dx = dx - 2.0f * c3;
    dx = dx + 2.0f * c4;
    dx = dx - c5;
    dx = dx + c7;
    float dy = -1.0f * c0 - 2.0f * c1;
    dy = dy - c2;
    dy = dy + c5;
    dy = dy + 2.0f * c6;
    dy = dy + c7;
    const float dx2 = dx * dx, dy2 = dy * dy;
    return dx2 + dy2;
  };
  const float sx = mag2(c[0].x, c[1].x, c[2].x, c[3].x, c[4].x, c[5].x, c[6].x, c[7].x);
  const float sy = mag2(c[0].y, c[1].y, c[2].y, c[3].y, c[4].y, c[5].y, c[6].y, c[7].y);
  const float sz = mag2(c[0].z, c[1].z, c[2].z, c[3].z, c[4].z, c[5].z, c[6].z, c[7].z);
  edge[((long)z * H + y) * W + x] = sqrtf((sx * 1.0f + sy * 1.0f) + sz * 1.0f);
}

// edge_enable = 1: the magnitude lands in the Lab image as the reference's
// float -> float3 store does (L, a, b <- e; the 4th float is untouched)
__global__ __launch_bounds__(256) void k_edge_store(const float* __restrict__ edge, long n, float4* __restrict__ lab) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float e = edge[i];
    float4 v = lab[i];
    v.x = e;
    v.y = e;
    v.z = e;
    lab[i] = v;
  }
}

// ---- apply_edge_alternative, clcode.cl:204-248 ---------------------------
// edge_enable = 2: each centre moves to its 8-neighbour of least edge value
// (strict <, first in the reference's dxy order) and takes that pixel's
// colour.  A centre outside the image (degenerate sizes) stays put.
__global__ void k_apply_edge(const float4* __restrict__ lab, const float* __restrict__ edge, int W, int H, int mw,
                             int mh, float* __restrict__ spixl) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x, row = blockIdx.y, z = blockIdx.z;
  if (col >= mw) return;
  float* sp = spixl + 8 * ((long)z * mw * mh + (long)row * mw + col);
  const int cx = (int)sp[1], cy = (int)sp[2];
  if (cx < 0 || cy < 0 || cx >= W || cy >= H) return;
  const long P = (long)W * H;
  const float* E = edge + z * P;
  const int dxs[8] = {-1, -1, 0, 1, 1, 1, 0, -1}, dys[8] = {0, -1, -1, -1, 0, 1, 1, 1};
  float ev = E[(long)cy * W + cx];
  int bx = -1, by = -1;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int nx = cx + dxs[i], ny = cy + dys[i];
    if (nx >= 0 && ny >= 0 && nx < W && ny < H) {
      const float ne = E[(long)ny * W + nx];
      if (ne < ev) {
        ev = ne;
        bx = nx;
        by = ny;
      }
    }
  }
  if (bx >= 0) {
    const float4 c = lab[z * P + (long)by * W + bx];
    sp[1] = (float)bx;
    sp[2] = (float)by;
    sp[3] = c.x;
    sp[4] = c.y;
    sp[5] = c.z;
  }
}

// ---- init_label_per_pixl, clcode.cl:341-353 ------------------------------
__global__ void k_grid_labels(int W, int H, int S, int mw, uint32_t* __restrict__ labels) {
  int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, z = blockIdx.z;
  if (x >= W) return;
  labels[((long)z * H + y) * W + x] = (uint32_t)(mw * (y / S) + x / S);
}

// ---- slic_distance_function + find_center_association, clcode.cl:422-520 -
// the argument of the reference's sqrt; the distance is sqrtf(slic_dist2)
__device__ __forceinline__ float slic_dist2(float4 px, int y, int x, float4 c, float cb, float weight, float sn,
                                            float cn) {
  // c = (cx, cy, L, a), cb = b of the centre (spixl fields 1..5)
  float a = (px.x - c.z) * (px.x - c.z);
  a = a + (px.y - c.w) * (px.y - c.w);
  a = a + (px.z - cb) * (px.z - cb);
  float b = ((float)x - c.x) * ((float)x - c.x);
  b = b + ((float)y - c.y) * ((float)y - c.y);
  return (a * cn) + weight * (b * sn);
}

// A workgroup assigns a 64 x 16 pixel block; the centres of every cell that
// can be a candidate of its pixels (one cell around the block's cells) are
// staged in LDS once, so the per-pixel candidate reads are LDS broadcasts.
// S3 = false: the reference's active candidate loop (clcode.cl:474-494: the
// 2x2 cells toward the pixel, x/y deltas swapped); S3 = true: the 3x3 loop the
// reference keeps behind its comment switch (clcode.cl:496-516), the one its
// kept Beer-Garden depth outputs were run with.
template <bool S3>
__device__ __forceinline__ void slic_cand(int ii, int jj, int dX, int dY, int& ox, int& oy) {
  if (S3) {  // i over y outer, j over x inner
    ox = jj - 1;
    oy = ii - 1;
  } else {  // i spans the x delta but offsets y (Appendix A #2)
    ox = jj - 1 + dY;
    oy = ii - 1 + dX;
  }
}

constexpr int AS_TW = 64, AS_TH = 16, AS_MAXC = 128;
template <bool S3>
__global__ __launch_bounds__(256) void k_assign(const float4* __restrict__ lab, const float* __restrict__ spixl,
                                                int W, int H, int S, int mw, int mh, float xy_n, float col_n,
                                                float weight, uint32_t* __restrict__ labels,
                                                uint16_t* __restrict__ lb16) {
  __shared__ float4 cxyla[AS_MAXC];  // (cx, cy, L, a)
  __shared__ float cbb[AS_MAXC];     // b
  const int x0 = blockIdx.x * AS_TW, y0 = blockIdx.y * AS_TH, z = blockIdx.z;
  const int cx0 = x0 / S - 1, cy0 = y0 / S - 1;
  const int ncx = min(x0 + AS_TW - 1, W - 1) / S - x0 / S + 3;
  const int ncy = min(y0 + AS_TH - 1, H - 1) / S - y0 / S + 3;
  const float* sp = spixl + 8L * z * mw * mh;
  const int col = x0 + (threadIdx.x & 63);
  const long P = (long)W * H;
  constexpr int NRW = AS_TH / 4;
  float4 pxs[NRW];  // the thread's pixels, loaded before the centre staging
#pragma unroll
  for (int r = 0; r < NRW; r++) {
    const int row = min(y0 + (threadIdx.x >> 6) + 4 * r, H - 1);
    pxs[r] = lab[(long)z * P + (long)row * W + min(col, W - 1)];
  }
  for (int e = threadIdx.x; e < ncx * ncy; e += 256) {
    const int cx = cx0 + e % ncx, cy = cy0 + e / ncx;
    if (cx >= 0 && cy >= 0 && cx < mw && cy < mh) {
      const float* c = sp + 8 * (cy * mw + cx);
      cxyla[e] = make_float4(c[1], c[2], c[3], c[4]);
      cbb[e] = c[5];
    }
  }
  __syncthreads();
  if (col >= W) return;
  // n / S as a multiply-high with M = ceil(2^32 / S): exact for n < 2^16, S <= 96
  const unsigned M = 0xffffffffu / (unsigned)S + 1u;
  auto divS = [&](int n) { return (int)__umulhi((unsigned)n, M); };
  const int cxg = divS(col), dX = divS(col + S / 2) - cxg;
#pragma unroll
  for (int r = 0; r < NRW; r++) {
    const int row = y0 + (threadIdx.x >> 6) + 4 * r;
    if (row >= H) break;
    const long pid = (long)z * P + (long)row * W + col;
    const float4 px = pxs[r];
    const int cyg = divS(row), dY = divS(row + S / 2) - cyg;
    // The reference keeps the smallest sqrt(d2) (strict <, first in loop
    // order).  sqrt is monotone, so a candidate with d2 >= the best d2 never
    // wins, and one below it by more than 2^-20 relative always does; only a
    // near tie needs the two correctly rounded square roots compared.
    float min_id = -1.0f;
    constexpr int NC = S3 ? 3 : 2;
    // the reference's loop, square roots and all
    auto exact = [&]() {
      float best2 = 0.0f, mid = -1.0f;
      bool have = false;
#pragma unroll
      for (int ii = 0; ii < NC; ii++)
#pragma unroll
        for (int jj = 0; jj < NC; jj++) {
          int ox, oy;
          slic_cand<S3>(ii, jj, dX, dY, ox, oy);
          const int cx = cxg + ox, cy = cyg + oy;
          const bool ok = cx >= 0 && cy >= 0 && cx < mw && cy < mh;
          const int e = ok ? (cy - cy0) * ncx + (cx - cx0) : 0;
          const float d2 = slic_dist2(px, row, col, cxyla[e], cbb[e], weight, xy_n, col_n);
          bool take;
          if (!have) {
            take = d2 < 9.0e11f || sqrtf(d2) < 999999.9999f;  // the reference's initial min_dist
          } else if (d2 >= best2) {
            take = false;
          } else if (d2 < best2 * 0.99999905f) {
            take = true;
          } else {
            take = sqrtf(d2) < sqrtf(best2);
          }
          take = take && ok;
          best2 = take ? d2 : best2;
          mid = take ? (float)(cy * mw + cx) : mid;
          have = have || take;
        }
      return mid;
    };
    if constexpr (S3) {
      min_id = exact();
    } else {
      // (k_assign_tiles4's test) the loop keeps the first candidate of least
      // d2 unless another d2 lies within the sqrt rounding above the least
      // (d2 * 0.99999905 <= least) or the least is not below 9e11: such a
      // pixel runs the loop itself.  A candidate outside the map takes a NaN
      // d2: never the least, never a near tie.
      float d2[4], cid[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        int ox, oy;
        slic_cand<false>(i >> 1, i & 1, dX, dY, ox, oy);
        const int cx = cxg + ox, cy = cyg + oy;
        const bool ok = cx >= 0 && cy >= 0 && cx < mw && cy < mh;
        const int e = ok ? (cy - cy0) * ncx + (cx - cx0) : 0;
        const float v = slic_dist2(px, row, col, cxyla[e], cbb[e], weight, xy_n, col_n);
        d2[i] = ok ? v : __builtin_nanf("");
        cid[i] = (float)(cy * mw + cx);
      }
      float lo, lo01;
      asm("v_min_f32 %0, %1, %2" : "=v"(lo01) : "v"(d2[0]), "v"(d2[1]));
      asm("v_min3_f32 %0, %1, %2, %3" : "=v"(lo) : "v"(lo01), "v"(d2[2]), "v"(d2[3]));
      bool amb = !(lo < 9.0e11f);
#pragma unroll
      for (int i = 0; i < 4; i++) amb |= (d2[i] > lo) & (d2[i] * 0.99999905f <= lo);
      min_id = d2[3] == lo ? cid[3] : -1.0f;
      min_id = d2[2] == lo ? cid[2] : min_id;
      min_id = d2[1] == lo ? cid[1] : min_id;
      min_id = d2[0] == lo ? cid[0] : min_id;
      if (amb) min_id = exact();
    }
    if (labels) labels[pid] = (uint32_t)min_id;  // (null: an update follows, reading only the copy)
    if (lb16) lb16[pid] = (uint16_t)min_id;      // the next k_update's 16-bit copy (mw * mh <= 65536)
  }
}

// ---- update_cluster_center + finalize_reduction_result -------------------
// clcode.cl:533-611 (per-tile LDS tree) and 719-773 (in-order partial sum),
// launch shape clSLIC.cpp:307-370.  One workgroup per (superpixel, view).
__device__ __forceinline__ float wave_tree(float v0, float v1, float v2, float v3) {
  // local_idx k = lane + 64*m holds v_m.  stride 128: k<128 gets k+128; stride
  // 64: k<64 gets k+64; strides 32..1 stay inside the wave, lane k adding lane
  // k+i without LDS: v_permlane32_swap (i=32), v_permlane16_swap (i=16), DPP
  // row_shl:i (i=8..1).  Only lane 0's result is used.
  float s = (v0 + v2) + (v1 + v3);
  unsigned u = __float_as_uint(s);
  s = s + __uint_as_float(__builtin_amdgcn_permlane32_swap(u, u, false, false)[1]);
  u = __float_as_uint(s);
  s = s + __uint_as_float(__builtin_amdgcn_permlane16_swap(u, u, false, false)[1]);
  s = s + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s), 0x108, 0xf, 0xf, true));
  s = s + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s), 0x104, 0xf, 0xf, true));
  s = s + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s), 0x102, 0xf, 0xf, true));
  s = s + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s), 0x101, 0xf, 0xf, true));
  return s;
}

// The same tree shape over uint32 (integer sums: any order gives the same value).
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3) {
  uint32_t s = (v0 + v2) + (v1 + v3);
  s = s + __builtin_amdgcn_permlane32_swap(s, s, false, false)[1];
  s = s + __builtin_amdgcn_permlane16_swap(s, s, false, false)[1];
  s = s + (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0x108, 0xf, 0xf, true);
  s = s + (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0x104, 0xf, 0xf, true);
  s = s + (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0x102, 0xf, 0xf, true);
  s = s + (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0x101, 0xf, 0xf, true);
  return s;
}

// wave_tree for several channels at once, from their in-lane sums sX =
// (v0 + v2) + (v1 + v3).  The two-register lane swaps pair the channels up
// instead of swapping each with itself: v_permlane32_swap(A, B) leaves the
// stride-32 sums of A in lanes 0-31 and of B in lanes 32-63, and
// v_permlane16_swap of two such registers puts the stride-16 sums of A, C, B,
// D in the four 16-lane rows, so one DPP row_shl chain finishes all four.
// Every channel's additions are wave_tree's, in its order.  Result lanes:
// A 0, C 16, B 32, D 48 (wave_tree2s: A 0, B 32).
__device__ __forceinline__ float dpp_rows_sum(float s) {
  s = s + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s), 0x108, 0xf, 0xf, true));
  s = s + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s), 0x104, 0xf, 0xf, true));
  s = s + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s), 0x102, 0xf, 0xf, true));
  s = s + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s), 0x101, 0xf, 0xf, true));
  return s;
}
__device__ __forceinline__ float halves_sum(float a, float b) {  // A in lanes 0-31, B in 32-63
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ float wave_tree4s(float sA, float sB, float sC, float sD) {
  const float X = halves_sum(sA, sB), Z = halves_sum(sC, sD);
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(X), __float_as_uint(Z), false, false);
  return dpp_rows_sum(__uint_as_float(r[0]) + __uint_as_float(r[1]));
}
__device__ __forceinline__ float wave_tree2s(float sA, float sB) {
  const float X = halves_sum(sA, sB);
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(X), __float_as_uint(X), false, false);
  return dpp_rows_sum(__uint_as_float(r[0]) + __uint_as_float(r[1]));
}
// two integer sums (any order gives the same value): A in lane 0, B in lane 32
__device__ __forceinline__ uint32_t wave_sum2_u32(uint32_t sA, uint32_t sB) {
  const auto p = __builtin_amdgcn_permlane32_swap(sA, sB, false, false);
  uint32_t s = p[0] + p[1];
  const auto r = __builtin_amdgcn_permlane16_swap(s, s, false, false);
  s = r[0] + r[1];
  s = s + (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0x108, 0xf, 0xf, true);
  s = s + (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0x104, 0xf, 0xf, true);
  s = s + (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0x102, 0xf, 0xf, true);
  s = s + (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0x101, 0xf, 0xf, true);
  return s;
}

// One WAVE per superpixel (4 per workgroup): the wave walks the G window
// tiles in order, each tile's 256 pixels as 4 per lane, tree-reduced in the
// reference's order (wave_tree), and lane 0 sums the tile partials in tile
// order -- no LDS, no barriers, and no idle waves when G < 4 (S = 8: G = 3,
// the third tile entirely outside the 3S window).
// UT = tiles per chunk (below): 4 when the window has many tiles (C5, S = 40:
// G = 57, update 39.1 -> 38.1 ms per C5 step), 1 for a few (S = 8: G = 3,
// where the chunk's registers cost more occupancy than the latencies it hides).
// LT: the label type read -- uint16_t when the previous assignment also wrote
// a 16-bit copy (every label < 65536): each window pixel's label is read by
// ~9 superpixels' walks, so halving it takes the C5 update from 3.0x its
// compulsory bytes to ~1.8x
template <int UT, typename LT = uint32_t>
__global__ __launch_bounds__(256) void k_update(const float4* __restrict__ lab, const LT* __restrict__ labels,
                                                int W, int H, int S, int mw, int mh, int G, int cpl,
                                                float* __restrict__ spixl) {
  const int lane = threadIdx.x & 63;
  const int sp = blockIdx.x * 4 + (threadIdx.x >> 6), z = blockIdx.y;
  if (sp >= mw * mh) return;  // whole wave; no barriers
  const int gx = sp % mw, gy = sp / mw;
  const long P = (long)W * H;
  const float4* L = lab + (long)z * P;
  const LT* I = labels + (long)z * P;
  const int lx = lane & 15, ly0 = lane >> 4;
  float acc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // tiles in chunks of UT: every label of the chunk is gathered before any
  // test, then every member's colour, so a chunk costs two memory latencies
  // instead of two per tile; the trees and the partial sums keep tile order
  for (int t0 = 0; t0 < G; t0 += UT) {
    LT lb[UT][4];
    int pix[UT][4], bx[UT], by[UT];
#pragma unroll
    for (int u = 0; u < UT; u++) {
      const int t = t0 + u, nbx = t % cpl, nby = t / cpl;
      bx[u] = gx * S - S + nbx * kLocal;
      by[u] = gy * S - S + nby * kLocal;
#pragma unroll
      for (int m = 0; m < 4; m++) {
        const int pxo = nbx * kLocal + lx, pyo = nby * kLocal + ly0 + 4 * m;
        const int px = bx[u] + lx, py = by[u] + ly0 + 4 * m;
        const bool in = t < G && pyo < S * 3 && pxo < S * 3 && py >= 0 && px >= 0 && px < W && py < H;
        pix[u][m] = in ? py * W + px : -1;
        lb[u][m] = I[in ? py * W + px : 0];
      }
    }
    float4 c[UT][4];
#pragma unroll
    for (int u = 0; u < UT; u++)
#pragma unroll
      for (int m = 0; m < 4; m++) {
        const bool mem = pix[u][m] >= 0 && lb[u][m] == (LT)sp;
        c[u][m] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (mem) c[u][m] = L[pix[u][m]];
      }
#pragma unroll
    for (int u = 0; u < UT; u++) {
      if (t0 + u >= G) break;
      float v[4][3];
      uint32_t pk[4];
      bool any = false;
#pragma unroll
      for (int m = 0; m < 4; m++) {
        const bool mem = pix[u][m] >= 0 && lb[u][m] == (LT)sp;
        // x, y, count: one packed integer tree of tile-local fields (as k_assign_tiles)
        pk[m] = mem ? (uint32_t)lx | (uint32_t)(ly0 + 4 * m) << 12 | 1u << 24 : 0u;
        v[m][0] = c[u][m].x;
        v[m][1] = c[u][m].y;
        v[m][2] = c[u][m].z;
        any |= mem;
      }
      float r[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (__any(any)) {
        const uint32_t q = wave_sum_u32(pk[0], pk[1], pk[2], pk[3]);
        const int cnt = (q >> 24) ? (int)(q >> 24) : 256;
        r[0] = (float)((int)(q & 0xfffu) + cnt * bx[u]);  // = the sum of member x: exact below 2^24
        r[1] = (float)((int)((q >> 12) & 0xfffu) + cnt * by[u]);
#pragma unroll
        for (int ch = 0; ch < 3; ch++) r[2 + ch] = wave_tree(v[0][ch], v[1][ch], v[2][ch], v[3][ch]);
        r[5] = (float)cnt;
      }
#pragma unroll
      for (int ch = 0; ch < 6; ch++) acc[ch] = acc[ch] + r[ch];  // lane 0 holds the tile partial
    }
  }
  if (lane == 0) {
    float* o = spixl + 8 * ((long)z * mw * mh + sp);
    const float n = acc[5];
    o[0] = (float)sp;
    if (n != 0) {
      // x * RN(1/n): the reference device's division, as its kept overlays
      // show (oracle orc_update)
      const float r = 1.0f / n;
      o[1] = acc[0] * r;
      o[2] = acc[1] * r;
      o[3] = acc[2] * r;
      o[4] = acc[3] * r;
      o[5] = acc[4] * r;
      o[6] = n;
    } else {
      o[1] = o[2] = o[3] = o[4] = o[5] = o[6] = 0.0f;
    }
  }
}

// k_update's window walk with the per-tile work cut to what the window
// needs (C5, S = 40: k_update<4, uint16_t> executed ~131 VALU and ~72 SALU
// per window tile, 296 M + 162 M per launch, VALU-issue-bound at 568 us):
//  * the tile coordinates advance incrementally (t % cpl, t / cpl were SALU
//    division sequences), and every address is a 32-bit buffer offset: the
//    tile origin (scalar) plus the lane's fixed offset, one add per load and
//    no select -- the view's buffer resource bounds it, and a pixel outside
//    the window or the image is dropped by its in-test as before;
//  * a pixel is tested with three compares (column: once per tile; the row
//    against the window and the image; the label);
//  * a colour is gathered for members only: a non-member's load is sent
//    past the buffer's records (no memory access, 0 -- the exact zero the
//    tree adds for it);
//  * the three colour trees run together (wave_tree4s: each channel's
//    additions are wave_tree's, in its order), accumulated in their result
//    lanes (0: L, 32: a, 16: b), x / y / count as k_update's integer tree.
// Bit-identical to k_update (the same per-tile trees, the same tile order).
typedef unsigned u32x3 __attribute__((ext_vector_type(3)));
template <int UT, typename LT>
__global__ __launch_bounds__(256) void k_update_walk(const float4* __restrict__ lab, const LT* __restrict__ labels,
                                                     int W, int H, int S, int mw, int mh, int G, int cpl,
                                                     float* __restrict__ spixl) {
  const int lane = threadIdx.x & 63;
  const int sp = blockIdx.x * 4 + (threadIdx.x >> 6), z = blockIdx.y;
  if (sp >= mw * mh) return;  // whole wave; no barriers
  const int gx = sp % mw, gy = sp / mw;
  const long P = (long)W * H;
  // the launcher checks P * 16 < 2^31
  const __amdgpu_buffer_rsrc_t rl =
      __builtin_amdgcn_make_buffer_rsrc((void*)(labels + z * P), 0, (int)(P * sizeof(LT)), 0x00020000);
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void*)(lab + z * P), 0, (int)(P * 16), 0x00020000);
  const int lx = lane & 15, ly0 = lane >> 4, S3 = 3 * S;
  const int x0 = gx * S - S, y0 = gy * S - S;  // the window's origin
  const int loff = ly0 * W + lx;                // the lane's pixel offset in a tile (row m: + 4 m W)
  const unsigned loffl = (unsigned)loff * (unsigned)sizeof(LT), loffc = (unsigned)loff * 16u;  // in bytes
  const uint32_t lpk = (uint32_t)lx | (uint32_t)ly0 << 12 | 1u << 24;
  float acc3 = 0.0f;                        // colour partial sums: lane 0 L, 32 a, 16 b
  float accx = 0.0f, accy = 0.0f, accn = 0.0f;  // lane 0
  int nbx = 0, nby = 0;                     // window tile of t0
  for (int t0 = 0; t0 < G; t0 += UT) {
    LT lb[UT][4];
    int tb[UT], bxs[UT], bys[UT], nys[UT];
    bool inx[UT];
#pragma unroll
    for (int u = 0; u < UT; u++) {
      bxs[u] = x0 + nbx * kLocal;
      bys[u] = y0 + nby * kLocal;
      nys[u] = nby * kLocal;
      tb[u] = bys[u] * W + bxs[u];  // tile origin's pixel offset (may be negative: dropped lanes)
      inx[u] = t0 + u < G && (unsigned)(bxs[u] + lx) < (unsigned)W && nbx * kLocal + lx < S3;
#pragma unroll
      for (int m = 0; m < 4; m++) {
        // scalar tile-row offset + the lane's pre-scaled offset: one add per load
        const unsigned o = (unsigned)(tb[u] + 4 * m * W) * (unsigned)sizeof(LT) + loffl;
        if (sizeof(LT) == 2)
          lb[u][m] = (LT)__builtin_amdgcn_raw_buffer_load_b16(rl, (int)o, 0, 0);
        else
          lb[u][m] = (LT)__builtin_amdgcn_raw_buffer_load_b32(rl, (int)o, 0, 0);
      }
      if (++nbx == cpl) {
        nbx = 0;
        nby++;
      }
    }
    // membership without short-circuit branches; a non-member's colour load
    // is sent past the records (no memory access, reads 0: the exact zero the
    // tree needs), so only members move colour bytes
    bool mem[UT][4], anyt[UT];
    u32x3 c[UT][4];
#pragma unroll
    for (int u = 0; u < UT; u++) {
      bool any = false;
#pragma unroll
      for (int m = 0; m < 4; m++) {
        const int py = bys[u] + ly0 + 4 * m;
        mem[u][m] = inx[u] & (nys[u] + ly0 + 4 * m < S3) & ((unsigned)py < (unsigned)H) & (lb[u][m] == (LT)sp);
        any |= mem[u][m];
        const unsigned oc = (unsigned)(tb[u] + 4 * m * W) * 16u + loffc;
        c[u][m] = __builtin_amdgcn_raw_buffer_load_b96(rc, mem[u][m] ? (int)oc : 0x7fffffff, 0, 0);
      }
      anyt[u] = __any(any);
    }
#pragma unroll
    for (int u = 0; u < UT; u++) {
      if (t0 + u >= G) break;
      float rx = 0.0f, ry = 0.0f, rn = 0.0f, r3 = 0.0f;
      if (anyt[u]) {
        uint32_t pk[4];
        float v[3][4];
#pragma unroll
        for (int m = 0; m < 4; m++) {
          pk[m] = mem[u][m] ? lpk + ((uint32_t)(4 * m) << 12) : 0u;
          v[0][m] = __uint_as_float(c[u][m].x);  // (0 for a non-member: its load read nothing)
          v[1][m] = __uint_as_float(c[u][m].y);
          v[2][m] = __uint_as_float(c[u][m].z);
        }
        const uint32_t q = wave_sum_u32(pk[0], pk[1], pk[2], pk[3]);
        const int cnt = (q >> 24) ? (int)(q >> 24) : 256;
        rx = (float)((int)(q & 0xfffu) + cnt * bxs[u]);  // the sum of member x: exact below 2^24
        ry = (float)((int)((q >> 12) & 0xfffu) + cnt * bys[u]);
        rn = (float)cnt;
        float sc[3];
#pragma unroll
        for (int ch = 0; ch < 3; ch++) sc[ch] = (v[ch][0] + v[ch][2]) + (v[ch][1] + v[ch][3]);
        r3 = wave_tree4s(sc[0], sc[1], sc[2], 0.0f);  // lanes 0: L, 32: a, 16: b
      }
      accx = accx + rx;
      accy = accy + ry;
      acc3 = acc3 + r3;
      accn = accn + rn;
    }
  }
  const float aL = __shfl(acc3, 0), aa = __shfl(acc3, 32), ab = __shfl(acc3, 16);
  if (lane == 0) {
    float* o = spixl + 8 * ((long)z * mw * mh + sp);
    const float n = accn;
    o[0] = (float)sp;
    if (n != 0) {
      const float r = 1.0f / n;  // x * RN(1/n), as k_update
      o[1] = accx * r;
      o[2] = accy * r;
      o[3] = aL * r;
      o[4] = aa * r;
      o[5] = ab * r;
      o[6] = n;
    } else {
      o[1] = o[2] = o[3] = o[4] = o[5] = o[6] = 0.0f;
    }
  }
}

// ---- the same update when S is a multiple of 16 --------------------------
// Every superpixel window then starts on the global 16x16 tile grid, so each
// image tile is tile t = nby*cpl + nbx of exactly the 3x3 superpixels whose
// windows cover it.  One wave per image tile reads its 256 pixels ONCE (the
// per-superpixel kernel above reads each pixel 9 times) and reduces, for each
// of those superpixels, its members with the reference's LDS tree order
// (wave_tree); non-members and other superpixels contribute exact zeros.
// k_update_finalize then sums each superpixel's G partials in tile order --
// bit-identical to k_update.
__global__ __launch_bounds__(256) void k_update_tiles(const float4* __restrict__ lab,
                                                      const uint32_t* __restrict__ labels, int W, int H, int S,
                                                      int mw, int mh, int G, int cpl, int ntx, int nty,
                                                      float* __restrict__ part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tile = blockIdx.x * 4 + wave, z = blockIdx.y;
  if (tile >= ntx * nty) return;  // no barriers below
  const int TX = tile % ntx, TY = tile / ntx, s16 = S / 16;
  const long P = (long)W * H;
  const float4* L = lab + (long)z * P;
  const uint32_t* I = labels + (long)z * P;
  const int lx = lane & 15, ly0 = lane >> 4;  // local index k = lane + 64*m, as the reference tile
  uint32_t lbl[4];
  float4 c[4];
  float fx[4], fy[4];
#pragma unroll
  for (int m = 0; m < 4; m++) {
    const int px = TX * 16 + lx, py = TY * 16 + ly0 + 4 * m;
    const bool in = px < W && py < H;
    lbl[m] = in ? I[(long)py * W + px] : 0xffffffffu;
    c[m] = in ? L[(long)py * W + px] : make_float4(0.f, 0.f, 0.f, 0.f);
    fx[m] = (float)px;
    fy[m] = (float)py;
  }
  float* out = part + (long)z * mw * mh * G * 6;
  for (int gy = TY / s16 - 1; gy <= TY / s16 + 1; gy++) {
    if (gy < 0 || gy >= mh) continue;
    for (int gx = TX / s16 - 1; gx <= TX / s16 + 1; gx++) {
      if (gx < 0 || gx >= mw) continue;
      const uint32_t sp = (uint32_t)(gy * mw + gx);
      const int t = (TY - (gy - 1) * s16) * cpl + (TX - (gx - 1) * s16);
      bool mem[4], any = false;
#pragma unroll
      for (int m = 0; m < 4; m++) {
        mem[m] = lbl[m] == sp;
        any |= mem[m];
      }
      float r[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (__any(any)) {
        r[0] = wave_tree(mem[0] ? fx[0] : 0.f, mem[1] ? fx[1] : 0.f, mem[2] ? fx[2] : 0.f, mem[3] ? fx[3] : 0.f);
        r[1] = wave_tree(mem[0] ? fy[0] : 0.f, mem[1] ? fy[1] : 0.f, mem[2] ? fy[2] : 0.f, mem[3] ? fy[3] : 0.f);
        r[2] = wave_tree(mem[0] ? c[0].x : 0.f, mem[1] ? c[1].x : 0.f, mem[2] ? c[2].x : 0.f, mem[3] ? c[3].x : 0.f);
        r[3] = wave_tree(mem[0] ? c[0].y : 0.f, mem[1] ? c[1].y : 0.f, mem[2] ? c[2].y : 0.f, mem[3] ? c[3].y : 0.f);
        r[4] = wave_tree(mem[0] ? c[0].z : 0.f, mem[1] ? c[1].z : 0.f, mem[2] ? c[2].z : 0.f, mem[3] ? c[3].z : 0.f);
        r[5] = wave_tree(mem[0] ? 1.f : 0.f, mem[1] ? 1.f : 0.f, mem[2] ? 1.f : 0.f, mem[3] ? 1.f : 0.f);
      }
      if (lane == 0) {  // the tree's result lives in lane 0
#pragma unroll
        for (int ch = 0; ch < 6; ch++) out[((long)sp * G + t) * 6 + ch] = r[ch];
      }
    }
  }
}

// ---- assignment fused with the next update's tile partials ----------------
// (S % 16 == 0) One wave per 16x16 image tile: the tile lies inside one
// superpixel cell, so every candidate centre of its pixels is one of the 3x3
// cells around it (staged in LDS per wave).  The wave assigns its 256 pixels
// exactly as k_assign (same arithmetic, same tie rule), stores the labels
// and, when part != nullptr, reduces the tile for each covering superpixel
// exactly as k_update_tiles would from those labels -- one read of Lab per
// SLIC iteration instead of two.
template <bool S3>
__global__ __launch_bounds__(256) void k_assign_tiles(const float4* __restrict__ lab,
                                                      const float* __restrict__ spixl, int W, int H, int S, int mw,
                                                      int mh, float xy_n, float col_n, float weight, int G, int cpl,
                                                      int ntx, int nty, uint32_t* __restrict__ labels,
                                                      float* __restrict__ part) {
  __shared__ float4 cxyla[4][9];  // (cx, cy, L, a) of the 3x3 cells around the tile's cell
  __shared__ float cbb[4][9];     // b
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile = blockIdx.x * 4 + wave, z = blockIdx.y;
  if (tile >= ntx * nty) return;  // whole wave; no workgroup barriers below
  const int TX = tile % ntx, TY = tile / ntx, s16 = S / 16;
  const int cxg = TX / s16, cyg = TY / s16;  // the tile's cell
  const long P = (long)W * H;
  const float4* L = lab + (long)z * P;
  const float* sp = spixl + 8L * z * mw * mh;
  if (lane < 9) {
    const int cx = cxg - 1 + lane % 3, cy = cyg - 1 + lane / 3;
    if (cx >= 0 && cy >= 0 && cx < mw && cy < mh) {
      const float* c = sp + 8 * (cy * mw + cx);
      cxyla[wave][lane] = make_float4(c[1], c[2], c[3], c[4]);
      cbb[wave][lane] = c[5];
    }
  }
  const int lx = lane & 15, ly0 = lane >> 4;  // local index k = lane + 64*m, as the reference tile
  uint32_t lbl[4];
  float4 c[4];
  float fx[4], fy[4];
#pragma unroll
  for (int m = 0; m < 4; m++) {
    const int px = TX * 16 + lx, py = TY * 16 + ly0 + 4 * m;
    const bool in = px < W && py < H;
    c[m] = in ? L[(long)py * W + px] : make_float4(0.f, 0.f, 0.f, 0.f);
    fx[m] = (float)px;
    fy[m] = (float)py;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const unsigned M = 0xffffffffu / (unsigned)S + 1u;  // n / S, exact for n < 2^16, S <= 96
  auto divS = [&](int n) { return (int)__umulhi((unsigned)n, M); };
#pragma unroll
  for (int m = 0; m < 4; m++) {
    const int col = TX * 16 + lx, row = TY * 16 + ly0 + 4 * m;
    lbl[m] = 0xffffffffu;
    if (col >= W || row >= H) continue;
    const int dX = divS(col + S / 2) - cxg, dY = divS(row + S / 2) - cyg;
    float best2 = 0.0f, min_id = -1.0f;
    bool have = false;
    constexpr int NC = S3 ? 3 : 2;
#pragma unroll
    for (int ii = 0; ii < NC; ii++)
#pragma unroll
      for (int jj = 0; jj < NC; jj++) {  // the candidate order of k_assign
        int ox, oy;
        slic_cand<S3>(ii, jj, dX, dY, ox, oy);
        const int cx = cxg + ox, cy = cyg + oy;
        const bool ok = cx >= 0 && cy >= 0 && cx < mw && cy < mh;
        const int e = (oy + 1) * 3 + (ox + 1);
        const float d2 = slic_dist2(c[m], row, col, cxyla[wave][e], cbb[wave][e], weight, xy_n, col_n);
        bool take;
        if (!have) {
          take = d2 < 9.0e11f || sqrtf(d2) < 999999.9999f;
        } else if (d2 >= best2) {
          take = false;
        } else if (d2 < best2 * 0.99999905f) {
          take = true;
        } else {
          take = sqrtf(d2) < sqrtf(best2);
        }
        take = take && ok;
        best2 = take ? d2 : best2;
        min_id = take ? (float)(cy * mw + cx) : min_id;
        have = have || take;
      }
    lbl[m] = (uint32_t)min_id;
    if (labels) labels[(long)z * P + (long)row * W + col] = lbl[m];  // (null: an update follows)
  }
  if (!part) return;
  float* out = part + (long)z * mw * mh * G * 6;
  for (int gy = cyg - 1; gy <= cyg + 1; gy++) {
    if (gy < 0 || gy >= mh) continue;
    for (int gx = cxg - 1; gx <= cxg + 1; gx++) {
      if (gx < 0 || gx >= mw) continue;
      const uint32_t spi = (uint32_t)(gy * mw + gx);
      const int t = (TY - (gy - 1) * s16) * cpl + (TX - (gx - 1) * s16);
      bool mem[4], any = false;
#pragma unroll
      for (int m = 0; m < 4; m++) {
        mem[m] = lbl[m] == spi;
        any |= mem[m];
      }
      float r[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (__any(any)) {
        // x, y and count are integers whose float trees are exact (sums < 2^24), so
        // they come from one integer tree of packed tile-local fields: sum of
        // x - 16 TX (<= 3840, bits 0-11), of y - 16 TY (bits 12-23) and the count
        // (bits 24-31; 256 wraps to 0, and a tree only runs with a member present)
        uint32_t pk[4];
#pragma unroll
        for (int m = 0; m < 4; m++) pk[m] = mem[m] ? (uint32_t)lx | (uint32_t)(ly0 + 4 * m) << 12 | 1u << 24 : 0u;
        const uint32_t q = wave_sum_u32(pk[0], pk[1], pk[2], pk[3]);
        const int cnt = (q >> 24) ? (int)(q >> 24) : 256;
        r[0] = (float)((int)(q & 0xfffu) + cnt * 16 * TX);
        r[1] = (float)((int)((q >> 12) & 0xfffu) + cnt * 16 * TY);
        r[2] = wave_tree(mem[0] ? c[0].x : 0.f, mem[1] ? c[1].x : 0.f, mem[2] ? c[2].x : 0.f, mem[3] ? c[3].x : 0.f);
        r[3] = wave_tree(mem[0] ? c[0].y : 0.f, mem[1] ? c[1].y : 0.f, mem[2] ? c[2].y : 0.f, mem[3] ? c[3].y : 0.f);
        r[4] = wave_tree(mem[0] ? c[0].z : 0.f, mem[1] ? c[1].z : 0.f, mem[2] ? c[2].z : 0.f, mem[3] ? c[3].z : 0.f);
        r[5] = (float)cnt;
      }
      if (lane == 0) {
#pragma unroll
        for (int ch = 0; ch < 6; ch++) out[((long)spi * G + t) * 6 + ch] = r[ch];
      }
    }
  }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x3 __attribute__((ext_vector_type(3)));

// The same wave per tile for the reference's active 2x2 loop when S = 32 or
// 64 (C2-C4's S = 32).  The tile's candidate cells are then the same four for
// all its pixels: dX = (col + S/2) / S - cxg cannot change inside a 16-column
// tile when S/2 is a multiple of 16 (likewise dY), so
//  * the pixel test is branch-free: a candidate is taken when d2 is below the
//    best d2 by more than the sqrt rounding can hide, or, for the first one,
//    below 9e11 (k_assign's fast tests); only a lane meeting a near tie (or a
//    huge d2) re-runs k_assign's exact loop with its square roots;
//  * the update reduces only the four candidate cells, their trees
//    interleaved (16 independent chains per wave instead of one cell's four at
//    a time behind a branch); the other in-image cells of the 3x3 around the
//    tile, which no pixel of the tile can join, get the exact zeros k_update_tiles
//    would write for them.
// (The 9-cell loop measured 71-83 us per C2 launch: 40 % of its wave cycles
// stalled on instruction dependencies, 632 SALU instructions per wave.)
// S16 = S / 16 (2: S = 32, 4: S = 64): divisions by constants.  Grid
// ((ntx + 3) / 4, nty, V): the tile is (4 blockIdx.x + wave, blockIdx.y).
template <int S16>
__global__ __launch_bounds__(256) void k_assign_tiles4(const float4* __restrict__ lab,
                                                       const float* __restrict__ spixl, int W, int H, int mw,
                                                       int mh, float xy_n, float col_n, float weight, int G, int cpl,
                                                       int ntx, uint32_t* __restrict__ labels,
                                                       float* __restrict__ part) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int TX = blockIdx.x * 4 + wave, TY = blockIdx.y, z = blockIdx.z;
  if (TX >= ntx) return;  // whole wave; no workgroup barriers below
  constexpr int s16 = S16;
  const int cxg = TX / S16, cyg = TY / S16;  // the tile's cell
  // (16 TX + S/2) / S with S = 16 S16
  const int dX = (TX + S16 / 2) / S16 - cxg, dY = (TY + S16 / 2) / S16 - cyg;
  const long P = (long)W * H;
  const float4* L = lab + (long)z * P;
  const float* sp = spixl + 8L * z * mw * mh;
  // candidate i = 2 ii + jj in k_assign's loop order (slic_cand<false>)
  int ccx[4], ccy[4];
  bool cok[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    int ox, oy;
    slic_cand<false>(i >> 1, i & 1, dX, dY, ox, oy);
    ccx[i] = cxg + ox;
    ccy[i] = cyg + oy;
    cok[i] = ccx[i] >= 0 && ccy[i] >= 0 && ccx[i] < mw && ccy[i] < mh;
  }
  // the candidates' centres, wave-uniform, as pairs (0, 1) and (2, 3) for the
  // packed two-candidate distance below; a cell outside the map gets a NaN
  // centre, so its d2 is NaN: never taken, never a near tie
  f32x2 ccxp[2], ccyp[2], cLp[2], cap[2], cbp[2];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    float v[5];
    const float* cc = sp + 8 * (cok[i] ? ccy[i] * mw + ccx[i] : 0);
#pragma unroll
    for (int f = 0; f < 5; f++) v[f] = cc[1 + f];  // (cell 0 stands in for an outside one)
#pragma unroll
    for (int f = 0; f < 5; f++) v[f] = cok[i] ? v[f] : __builtin_nanf("");
    ccxp[i >> 1][i & 1] = v[0];
    ccyp[i >> 1][i & 1] = v[1];
    cLp[i >> 1][i & 1] = v[2];
    cap[i >> 1][i & 1] = v[3];
    cbp[i >> 1][i & 1] = v[4];
  }
  const int lx = lane & 15, ly0 = lane >> 4;  // local index k = lane + 64*m, as the reference tile
  // the tile's L, a, b as buffer loads: a pixel outside the image reads
  // zeros (an offset past the view's records), with no branch around it
  // (the launcher checks W H 16 < 2^31)
  const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc((void*)L, 0, (int)(P * 16), 0x00020000);
  float4 c[4];
#pragma unroll
  for (int m = 0; m < 4; m++) {
    const int px = TX * 16 + lx, py = TY * 16 + ly0 + 4 * m;
    const bool in = px < W && py < H;
    const u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(rl, in ? (py * W + px) * 16 : 0x7fffffff, 0, 0);
    c[m] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), 0.f);
  }
  float cid[4];  // the candidates' labels as k_assign forms them
#pragma unroll
  for (int i = 0; i < 4; i++) cid[i] = (float)(ccy[i] * mw + ccx[i]);
  // labels null (an update follows: its partials are all it reads): no records, every store dropped
  const __amdgpu_buffer_rsrc_t rlb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(labels ? labels + (long)z * P : nullptr), 0, labels ? (int)(P * 4) : 0, 0x00020000);
  uint32_t lbl[4];
  int win[4];  // the pixel's candidate (-1: none, or outside the image)
  // the lane's column is the same for its 4 pixels: (x - cx)^2 of each
  // candidate once (the same product slic_dist2 forms, so the same bits)
  float bcx[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const float dx = __fsub_rn((float)(TX * 16 + lx), ccxp[i >> 1][i & 1]);
    bcx[i] = __fmul_rn(dx, dx);
  }
#pragma unroll
  for (int m = 0; m < 4; m++) {
    const int col = TX * 16 + lx, row = TY * 16 + ly0 + 4 * m;
    // slic_dist2 per candidate, the same operations in the same order, in
    // scalar f32 (v_pk_*_f32 measured slower in the NCC kernels)
    float d2[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int h = i >> 1, k = i & 1;
      const float dl = __fsub_rn(c[m].x, cLp[h][k]);
      float ac = __fmul_rn(dl, dl);
      const float da = __fsub_rn(c[m].y, cap[h][k]);
      ac = __fadd_rn(ac, __fmul_rn(da, da));
      const float db = __fsub_rn(c[m].z, cbp[h][k]);
      ac = __fadd_rn(ac, __fmul_rn(db, db));
      const float dy = __fsub_rn((float)row, ccyp[h][k]);
      const float bc = __fadd_rn(bcx[i], __fmul_rn(dy, dy));
      d2[i] = __fadd_rn(__fmul_rn(ac, col_n), __fmul_rn(weight, __fmul_rn(bc, xy_n)));
    }
    // k_assign's loop keeps the first candidate of least sqrtf(d2) (strict <),
    // sqrtf being monotone: the first of least d2, unless a later-looking d2
    // lies so close above the least that the square roots may round together
    // (d2 * 0.99999905 <= least: k_assign's own near-tie test), or the least
    // is not below the 9e11 the first take is sure of.  Such a lane re-runs
    // k_assign's loop.  NaN (outside-map) candidates drop out of the min.
    // v_min3 / v_min (IEEE minNum: a quiet-NaN operand drops out, as in fminf;
    // as asm, without the canonicalising v_max fminf brings along)
    float lo, lo01;
    asm("v_min_f32 %0, %1, %2" : "=v"(lo01) : "v"(d2[0]), "v"(d2[1]));
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(lo) : "v"(lo01), "v"(d2[2]), "v"(d2[3]));
    int w = d2[3] == lo ? 3 : -1;
    w = d2[2] == lo ? 2 : w;
    w = d2[1] == lo ? 1 : w;
    w = d2[0] == lo ? 0 : w;
    // (bitwise, not short-circuit logic, which compiled to a branch per
    // candidate: the compares combine as lane masks on the scalar unit)
    bool amb = !(lo < 9.0e11f);
#pragma unroll
    for (int i = 0; i < 4; i++) amb |= (d2[i] > lo) & (d2[i] * 0.99999905f <= lo);
    float min_id = w == 0 ? cid[0] : w == 1 ? cid[1] : w == 2 ? cid[2] : w == 3 ? cid[3] : -1.0f;
    if (amb) {  // k_assign's loop, square roots and all
      float best2 = 0.0f;
      bool have = false;
      min_id = -1.0f;
      w = -1;
      for (int i = 0; i < 4; i++) {
        bool take;
        if (!have) {
          take = d2[i] < 9.0e11f || sqrtf(d2[i]) < 999999.9999f;
        } else if (d2[i] >= best2) {
          take = false;
        } else if (d2[i] < best2 * 0.99999905f) {
          take = true;
        } else {
          take = sqrtf(d2[i]) < sqrtf(best2);
        }
        take = take && cok[i];
        best2 = take ? d2[i] : best2;
        min_id = take ? cid[i] : min_id;
        w = take ? i : w;
        have = have || take;
      }
    }
    const bool in = col < W && row < H;
    lbl[m] = in ? (uint32_t)min_id : 0xffffffffu;
    win[m] = in ? w : -1;
    // buffer stores throughout: a lane with nothing to store writes past the
    // records (dropped), so no branch per store
    __builtin_amdgcn_raw_buffer_store_b32(lbl[m], rlb, in ? (row * W + col) * 4 : 0x7fffffff, 0, 0);
  }
  if (!part) return;
  float* out = part + (long)z * mw * mh * G * 6;
  const __amdgpu_buffer_rsrc_t rpt = __builtin_amdgcn_make_buffer_rsrc((void*)out, 0, mw * mh * G * 24, 0x00020000);
  constexpr int kOob = 0x7fffffff;
  // the candidate cells some pixel of the tile joined (a wave-uniform mask)
  unsigned pres = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const bool mi = win[0] == i || win[1] == i || win[2] == i || win[3] == i;
    pres |= __ballot(mi) != 0 ? 1u << i : 0u;
  }
  pres = __builtin_amdgcn_readfirstlane(pres);
  const unsigned joined_mask = pres;
  // the present cells' tile partials, two cells' trees interleaved per pass
  // (one pass for a tile inside one or two superpixels, the usual case)
  while (pres) {
    const int i0 = __builtin_ctz(pres);
    pres &= pres - 1;
    const int i1 = pres ? __builtin_ctz(pres) : i0;  // i1 == i0: a second copy, not stored
    pres &= pres ? pres - 1 : 0u;
    float sL[2] = {0.f, 0.f}, sa[2] = {0.f, 0.f}, sb[2] = {0.f, 0.f};
    uint32_t sq[2] = {0u, 0u};
    const bool two = i1 != i0;  // (uniform) a single cell: its second copy is neither summed nor stored
#pragma unroll
    for (int h = 0; h < 2; h++) {  // the in-lane step of the trees
      if (h == 1 && !two) break;
      const int i = h == 0 ? i0 : i1;
      bool mem[4];
#pragma unroll
      for (int m = 0; m < 4; m++) mem[m] = win[m] == i;
      uint32_t pk[4];
      float vL[4], va[4], vb[4];
#pragma unroll
      for (int m = 0; m < 4; m++) {
        pk[m] = mem[m] ? (uint32_t)lx | (uint32_t)(ly0 + 4 * m) << 12 | 1u << 24 : 0u;
        vL[m] = mem[m] ? c[m].x : 0.f;
        va[m] = mem[m] ? c[m].y : 0.f;
        vb[m] = mem[m] ? c[m].z : 0.f;
      }
      sq[h] = (pk[0] + pk[2]) + (pk[1] + pk[3]);
      sL[h] = (vL[0] + vL[2]) + (vL[1] + vL[3]);
      sa[h] = (va[0] + va[2]) + (va[1] + va[3]);
      sb[h] = (vb[0] + vb[2]) + (vb[1] + vb[3]);
    }
    const float T1 = wave_tree4s(sL[0], sa[0], sb[0], sL[1]);  // lanes 0: L0, 32: a0, 16: b0, 48: L1
    const float T2 = two ? wave_tree2s(sa[1], sb[1]) : 0.f;    // lanes 0: a1, 32: b1
    const uint32_t Q = wave_sum2_u32(sq[0], sq[1]);            // lane 32 h: cell h's x, y, count
    int base[2];  // (records of one view: the launcher checks the size)
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int i = h == 0 ? i0 : i1;
      const int gx = i == 0 ? ccx[0] : i == 1 ? ccx[1] : i == 2 ? ccx[2] : ccx[3];
      const int gy = i == 0 ? ccy[0] : i == 1 ? ccy[1] : i == 2 ? ccy[2] : ccy[3];
      const int t = (TY - (gy - 1) * s16) * cpl + (TX - (gx - 1) * s16);
      base[h] = ((gy * mw + gx) * G + t) * 6;
    }
    // each result stored from the lane holding it
    {
      const int cnt = (Q >> 24) ? (int)(Q >> 24) : 256;  // present: at least one member
      const bool qs = lane == 0 || (lane == 32 && two);
      const int ob = qs ? (lane == 0 ? base[0] : base[1]) * 4 : kOob;
      const float fx = (float)((int)(Q & 0xfffu) + cnt * 16 * TX), fy = (float)((int)((Q >> 12) & 0xfffu) + cnt * 16 * TY);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(fx), rpt, ob, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(fy), rpt, qs ? ob + 4 : kOob, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)cnt), rpt, qs ? ob + 20 : kOob, 0, 0);
      const bool s1 = lane == 0 || lane == 16 || lane == 32 || (lane == 48 && two);
      const int o1 = lane == 0 ? base[0] + 2 : lane == 16 ? base[0] + 4 : lane == 32 ? base[0] + 3 : base[1] + 2;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(T1), rpt, s1 ? o1 * 4 : kOob, 0, 0);
      const bool s2 = two && (lane == 0 || lane == 32);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(T2), rpt, s2 ? (lane == 0 ? base[1] + 3 : base[1] + 4) * 4 : kOob,
                                            0, 0);
    }
  }
  // exact zeros for every other in-image cell of the 3x3 around the tile (no
  // pixel of the tile joined it): lane 6 j + ch, cell j
  {
    const int j = lane / 6, ch = lane - 6 * j;
    const int gx = cxg - 1 + j % 3, gy = cyg - 1 + j / 3;
    bool joined = false;
#pragma unroll
    for (int i = 0; i < 4; i++) joined = joined || (((joined_mask >> i) & 1u) && gx == ccx[i] && gy == ccy[i]);
    const bool zw = lane < 54 && !joined && gx >= 0 && gy >= 0 && gx < mw && gy < mh;
    const int t = (TY - (gy - 1) * s16) * cpl + (TX - (gx - 1) * s16);
    __builtin_amdgcn_raw_buffer_store_b32(0u, rpt, zw ? (((gy * mw + gx) * G + t) * 6 + ch) * 4 : kOob, 0, 0);
  }
}

// 8 lanes per superpixel, lane c < 6 summing channel c of the G partials in
// tile order (the reference's order; a tile outside the image adds an exact
// +0, which leaves the running sum unchanged: it starts at +0 and a sum is
// -0 only when both terms are).  All G loads are independent of the sums,
// so they are issued ahead -- one thread walking all six channels was
// load-latency-bound (14 us per launch at C2).
// CPL > 0: cpl = CPL (G = CPL^2; S = 32: 6), every partial's load issued
// before the sum (9.2 us per C2 launch with four in flight)
template <int CPL>
__global__ __launch_bounds__(256) void k_update_finalize(const float* __restrict__ part, int mw, int mh, int S,
                                                         int G, int cpl, int ntx, int nty,
                                                         float* __restrict__ spixl) {
  const int c = threadIdx.x & 7, sp = blockIdx.x * 32 + (threadIdx.x >> 3), z = blockIdx.y;
  const bool live = sp < mw * mh;  // no early exit: lanes exchange the count below
  const int spc = live ? sp : 0;
  const int gx = spc % mw, gy = spc / mw, s16 = S / 16;
  const float* pp = part + ((long)z * mw * mh + spc) * G * 6 + (c < 6 ? c : 5);
  float acc = 0.f;
  if (CPL > 0) {
    constexpr int GT = CPL > 0 ? CPL * CPL : 1;
    float v[GT];
#pragma unroll
    for (int t = 0; t < GT; t++) v[t] = pp[t * 6];
#pragma unroll
    for (int t = 0; t < GT; t++) {
      const int TX = (gx - 1) * s16 + t % CPL, TY = (gy - 1) * s16 + t / CPL;
      const bool in = TX >= 0 && TY >= 0 && TX < ntx && TY < nty;  // outside the image: the reference adds 0
      acc = acc + (in ? v[t] : 0.f);
    }
  } else {
    int tx = 0, ty = 0;
#pragma unroll 4
    for (int t = 0; t < G; t++) {
      const int TX = (gx - 1) * s16 + tx, TY = (gy - 1) * s16 + ty;
      const bool in = TX >= 0 && TY >= 0 && TX < ntx && TY < nty;  // outside the image: the reference adds 0
      const float v = pp[t * 6];
      acc = acc + (in ? v : 0.f);
      if (++tx == cpl) { tx = 0; ty++; }
    }
  }
  const float n = __shfl(acc, (threadIdx.x & 63 & ~7) + 5);
  if (!live || c > 6) return;
  float* o = spixl + 8 * ((long)z * mw * mh + sp);
  if (c == 6) {
    o[0] = (float)sp;
  } else if (c == 5) {
    o[6] = n;
  } else {
    o[1 + c] = n != 0 ? acc * (1.0f / n) : 0.0f;  // x * RN(1/n), as k_update
  }
}

// ---- supress_local_lable, clcode.cl:676-711 ------------------------------
__global__ void k_suppress(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int W, int H) {
  int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, z = blockIdx.z;
  if (x >= W) return;
  long base = (long)z * W * H;
  long idx = base + (long)y * W + x;
  int cl = (int)in[idx];
  if (x <= 1 || y <= 1 || x >= W - 2 || y >= H - 2) {
    out[idx] = (uint32_t)cl;
    return;
  }
  int cnt = 0, dl = -1;
  for (int j = -2; j <= 2; j++)
    for (int i = -2; i <= 2; i++) {
      int nl = (int)in[base + (long)(y + j) * W + (x + i)];
      if (nl != cl) {
        dl = nl;
        cnt++;
      }
    }
  out[idx] = (uint32_t)(cnt >= 16 ? dl : cl);
}

}  // namespace

int launch_cvt(hipStream_t s, const uint8_t* rgbx, long npix, float* lab, uint8_t* l8) {
  if (npix <= 0) return 0;
  long blocks = (npix + 1023) / 1024;  // 1024 pixels per 256-thread block and pass
  if (blocks > 256L * 32) blocks = 256L * 32;
  hipLaunchKernelGGL(k_cvt, dim3((unsigned)blocks), dim3(256), 0, s, (const uint32_t*)rgbx, npix, (float4*)lab, l8);
  MVS_LAUNCH_CHECK("k_cvt");
  return 0;
}

int launch_init_centers(hipStream_t s, const float* lab, int V, int W, int H, int S, float* spixl) {
  int mw = map_dim(W, S), mh = map_dim(H, S);
  hipLaunchKernelGGL(k_init_centers, dim3((mw + 63) / 64, mh, V), dim3(64), 0, s, (const float4*)lab, W, H, S, mw,
                     mh, spixl);
  MVS_LAUNCH_CHECK("k_init_centers");
  return 0;
}

// clSLIC::apply_edge_values (clSLIC.cpp:186-233); edge = V*W*H floats scratch
int launch_edge_step(hipStream_t s, float* lab, int V, int W, int H, int S, int edge_enable, float* spixl,
                     float* edge) {
  if (edge_enable != 1 && edge_enable != 2) return 0;
  hipLaunchKernelGGL(k_edge, dim3((W + 255) / 256, H, V), dim3(256), 0, s, (const float4*)lab, W, H, edge);
  MVS_LAUNCH_CHECK("k_edge");
  if (edge_enable == 1) {
    // the reference's path: magnitude into the Lab image; apply_edge_alternative
    // then reads the never-written edge_img (pinned as zeros): no centre moves
    const long n = (long)V * W * H;
    hipLaunchKernelGGL(k_edge_store, dim3((unsigned)std::min<long>((n + 255) / 256, 8192)), dim3(256), 0, s, edge, n,
                       (float4*)lab);
    MVS_LAUNCH_CHECK("k_edge_store");
    return 0;
  }
  const int mw = map_dim(W, S), mh = map_dim(H, S);
  hipLaunchKernelGGL(k_apply_edge, dim3((mw + 63) / 64, mh, V), dim3(64), 0, s, (const float4*)lab, edge, W, H, mw,
                     mh, spixl);
  MVS_LAUNCH_CHECK("k_apply_edge");
  return 0;
}

int launch_grid_labels(hipStream_t s, int V, int W, int H, int S, uint32_t* labels) {
  int mw = map_dim(W, S);
  hipLaunchKernelGGL(k_grid_labels, dim3((W + 255) / 256, H, V), dim3(256), 0, s, W, H, S, mw, labels);
  MVS_LAUNCH_CHECK("k_grid_labels");
  return 0;
}

int launch_assign(hipStream_t s, const float* lab, const float* spixl, int V, int W, int H, int S, float xy_n,
                  float col_n, float weight, int search, uint32_t* labels, uint16_t* lb16) {
  int mw = map_dim(W, S), mh = map_dim(H, S);
  if (!labels && !(lb16 && (long)mw * mh <= 65536)) return arg_fail("SLIC assign: no label output");
  if ((AS_TW / S + 4) * (AS_TH / S + 4) > AS_MAXC) return arg_fail("SLIC assign: spixl_size too small");
  hipLaunchKernelGGL(search ? k_assign<true> : k_assign<false>, dim3((W + AS_TW - 1) / AS_TW, (H + AS_TH - 1) / AS_TH, V), dim3(256), 0, s,
                     (const float4*)lab, spixl, W, H, S, mw, mh, xy_n, col_n, weight, labels,
                     (long)mw * mh <= 65536 ? lb16 : nullptr);
  MVS_LAUNCH_CHECK("k_assign");
  return 0;
}

int launch_assign_tiles(hipStream_t s, const float* lab, const float* spixl, int V, int W, int H, int S, float xy_n,
                        float col_n, float weight, int search, uint32_t* labels, float* part) {
  if (S % 16 != 0) return arg_fail("SLIC fused assign needs spixl_size % 16 == 0");
  int mw = map_dim(W, S), mh = map_dim(H, S);
  int G = (3 * S / kLocal) * (3 * S / kLocal), cpl = S * 3 / kLocal;
  int ntx = (W + 15) / 16, nty = (H + 15) / 16;
  // MVS_SLIC_TILES9=1 (read per call): the 9-cell kernel for S % 32 == 0 too (A/B)
  const char* t9 = getenv("MVS_SLIC_TILES9");
  if (!search && (S == 32 || S == 64) && (long)W * H * 16 < (1L << 31) && (long)mw * mh * G * 24 < (1L << 31) &&
      !(t9 && atoi(t9) == 1))
    hipLaunchKernelGGL(S == 32 ? k_assign_tiles4<2> : k_assign_tiles4<4>, dim3((ntx + 3) / 4, nty, V), dim3(256), 0,
                       s, (const float4*)lab, spixl, W, H, mw, mh, xy_n, col_n, weight, G, cpl, ntx, labels, part);
  else
    hipLaunchKernelGGL(search ? k_assign_tiles<true> : k_assign_tiles<false>, dim3((ntx * nty + 3) / 4, V), dim3(256), 0, s, (const float4*)lab, spixl, W,
                       H, S, mw, mh, xy_n, col_n, weight, G, cpl, ntx, nty, labels, part);
  MVS_LAUNCH_CHECK("k_assign_tiles");
  return 0;
}

int launch_update_finalize(hipStream_t s, const float* part, int V, int W, int H, int S, float* spixl) {
  int mw = map_dim(W, S), mh = map_dim(H, S);
  int G = (3 * S / kLocal) * (3 * S / kLocal), cpl = S * 3 / kLocal;
  int ntx = (W + 15) / 16, nty = (H + 15) / 16;
  hipLaunchKernelGGL(cpl == 6 ? k_update_finalize<6> : k_update_finalize<0>, dim3((mw * mh + 31) / 32, V), dim3(256),
                     0, s, part, mw, mh, S, G, cpl, ntx, nty, spixl);
  MVS_LAUNCH_CHECK("k_update_finalize");
  return 0;
}

size_t update_scratch_bytes(int V, int W, int H, int S) {
  if (S % 16 != 0) return 0;
  int mw = map_dim(W, S), mh = map_dim(H, S);
  int G = (3 * S / kLocal) * (3 * S / kLocal);
  return sizeof(float) * 6 * (size_t)G * mw * mh * V;
}

int launch_update(hipStream_t s, const float* lab, const uint32_t* labels, int V, int W, int H, int S,
                  float* spixl, float* part, const uint16_t* lb16) {
  int mw = map_dim(W, S), mh = map_dim(H, S);
  int G = (int)__builtin_ceilf((float)(S * S * 9) / (float)(kLocal * kLocal));
  int cpl = S * 3 / kLocal;
  if (cpl <= 0) return arg_fail("SLIC update needs spixl_size >= 6 (cluster_per_line = 3S/16 > 0)");
  if (part && S % 16 == 0) {  // tile-grid path (each pixel read once)
    int ntx = (W + 15) / 16, nty = (H + 15) / 16;
    hipLaunchKernelGGL(k_update_tiles, dim3((ntx * nty + 3) / 4, V), dim3(256), 0, s, (const float4*)lab, labels,
                       W, H, S, mw, mh, G, cpl, ntx, nty, part);
    MVS_LAUNCH_CHECK("k_update_tiles");
    hipLaunchKernelGGL(cpl == 6 ? k_update_finalize<6> : k_update_finalize<0>, dim3((mw * mh + 31) / 32, V),
                       dim3(256), 0, s, part, mw, mh, S, G, cpl, ntx, nty, spixl);
    MVS_LAUNCH_CHECK("k_update_finalize");
    return 0;
  }
  // k_update_walk (32-bit buffer offsets: P * 16 < 2^31); MVS_SLIC_UPDATE=0
  // (read per call): k_update (A/B)
  const char* ue = getenv("MVS_SLIC_UPDATE");
  const bool walk = (long)W * H * 16 < (1L << 31) && !(ue && atoi(ue) == 0);
  if (walk) {
    const bool l16 = lb16 && (long)mw * mh <= 65536;
    const dim3 g((mw * mh + 3) / 4, V);
    if (l16) {
      auto kw = G > 4 ? k_update_walk<4, uint16_t> : k_update_walk<1, uint16_t>;
      hipLaunchKernelGGL(kw, g, dim3(256), 0, s, (const float4*)lab, lb16, W, H, S, mw, mh, G, cpl, spixl);
    } else {
      auto kw = G > 4 ? k_update_walk<4, uint32_t> : k_update_walk<1, uint32_t>;
      hipLaunchKernelGGL(kw, g, dim3(256), 0, s, (const float4*)lab, labels, W, H, S, mw, mh, G, cpl, spixl);
    }
    MVS_LAUNCH_CHECK("k_update_walk");
    return 0;
  }
  if (lb16 && (long)mw * mh <= 65536) {  // the 16-bit copy the previous launch_assign wrote
    auto k16 = G > 4 ? k_update<4, uint16_t> : k_update<1, uint16_t>;
    hipLaunchKernelGGL(k16, dim3((mw * mh + 3) / 4, V), dim3(256), 0, s, (const float4*)lab, lb16, W, H, S, mw, mh,
                       G, cpl, spixl);
  } else {
    hipLaunchKernelGGL(G > 4 ? k_update<4> : k_update<1>, dim3((mw * mh + 3) / 4, V), dim3(256), 0, s,
                       (const float4*)lab, labels, W, H, S, mw, mh, G, cpl, spixl);
  }
  MVS_LAUNCH_CHECK("k_update");
  return 0;
}

int launch_suppress(hipStream_t s, const uint32_t* in, uint32_t* out, int V, int W, int H) {
  hipLaunchKernelGGL(k_suppress, dim3((W + 255) / 256, H, V), dim3(256), 0, s, in, out, W, H);
  MVS_LAUNCH_CHECK("k_suppress");
  return 0;
}

}  // namespace mvs
