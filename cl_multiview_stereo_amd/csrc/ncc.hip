// Build-defined per-pixel NCC K x K plane sweep: the cost-volume producer.
//
// Definition (no reference counterpart; restated in oracle/mvs_oracle.c
// orc_ncc_volume): q = 8-bit intensity (clamp(int(L*2.55+0.5))), window K x K,
// shift of neighbour n at level d: (tx, ty) = (roundf(d*dx), roundf((bl*d)*dy)),
// window valid iff every tap of the reference and the shifted window is inside
// the image; with n = K*K and integer sums
//   num = n*Srp - Sr*Sp,  vr = n*Srr - Sr^2,  vp = n*Spp - Sp^2
// ivr = vr ? 1/(float)vr : 0 and ivp likewise (per pixel, in the box plane),
// cost = 2 (invalid) | 1 - ((a*|a|)*ivr)*ivp with a = (float)num (1 - signed
// squared NCC; 1 on textureless windows); vol[d][y][x] = min over neighbours
// (strict <, init 1e6).
//
// Kernel design (gfx950, wave64):
//   * a workgroup = 4 waves on one tile of 64 image columns (64-2R outputs) x
//     TH rows and a chunk of 4*DPW hypotheses; wave w owns levels w, w+4, ...
//   * per neighbour the workgroup stages in LDS the neighbour's intensity band
//     and its window statistics (Sp, (float)vp) covering every shift of the
//     chunk, so the inner loops touch only LDS and registers;
//   * per (d, n) a lane walks its column down TH+2R rows: product
//     q_ref*q_nbr (24-bit multiply), horizontal K-sum across lanes by DPP
//     wave shifts, vertical K-sum by a register sliding window -- all integer,
//     so exact in any order; the IEEE f32 finish is branch-free;
//   * the min over neighbours stays in registers (DPW x TH per lane) and the
//     chunk's costs are written once, 64-column coalesced rows of the volume.
#include <algorithm>

#include "mvs_internal.h"

namespace mvs {
namespace {

// ---- window statistics: (S, (float)(n*SS - S^2)) of l8, 0 outside ---------
__global__ void k_box_stats(const uint8_t* __restrict__ q, int W, int H, int K, int* __restrict__ boxS,
                            float* __restrict__ boxI) {
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
  int v = K * K * ss - s * s;
  float iv = v != 0 ? 1.0f / (float)v : 0.0f;  // reciprocal window variance, 0 if textureless
  boxS[z * P + (long)y * W + x] = s;
  boxI[z * P + (long)y * W + x] = iv;
}

constexpr int kMaxNbr = 16;
struct NccArgs {
  int W, H, D, nn, z;
  int view[kMaxNbr];
  float fdx[kMaxNbr];
  float fdy[kMaxNbr];
  float bl;
  int band_w, band_h, box_h;  // LDS band extents (host-computed maxima)
  int monotone;               // levels non-decreasing (shift extents from the chunk ends)
};

// wave_shr:1 / wave_shl:1 with bound_ctrl (edge lanes read 0); the compiler
// folds them into the following v_add as a DPP source modifier
__device__ __forceinline__ int dpp_shr1(int v) { return __builtin_amdgcn_mov_dpp(v, 0x138, 0xf, 0xf, true); }
__device__ __forceinline__ int dpp_shl1(int v) { return __builtin_amdgcn_mov_dpp(v, 0x130, 0xf, 0xf, true); }

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gptr_t;
// LDS-DMA: lane l's element lands at dst + l*size (dst wave-uniform)
// (the ubyte form zero-extends into a 4-byte slot per lane, measured on gfx950)
__device__ __forceinline__ void glds_u8(const uint8_t* src, uint32_t* dst) {
  __builtin_amdgcn_global_load_lds((gptr_t)src, (lds_ptr_t)dst, 1, 0, 0);
}
__device__ __forceinline__ void glds_b32(const void* src, void* dst) {
  __builtin_amdgcn_global_load_lds((gptr_t)src, (lds_ptr_t)dst, 4, 0, 0);
}

// bits [lo, hi] set (clamped to [0, 31])
__device__ __forceinline__ unsigned bit_range(int lo, int hi) {
  lo = max(lo, 0);
  hi = min(hi, 31);
  if (hi < lo) return 0u;
  unsigned up = hi >= 31 ? 0xffffffffu : ((1u << (hi + 1)) - 1u);
  return up & ~((1u << lo) - 1u);
}

template <int R>
__device__ __forceinline__ int hsum(int p) {
  // sum of lanes l-R .. l+R (DPP wave shifts; symmetric and exact)
  int s = p, a = p, b = p;
#pragma unroll
  for (int i = 0; i < R; i++) {
    a = dpp_shr1(a);
    b = dpp_shl1(b);
    s = s + a;
    s = s + b;
  }
  return s;
}

__device__ __forceinline__ int shift_x(float d, float fdx) { return (int)roundf(d * fdx); }
__device__ __forceinline__ int shift_y(float bl, float d, float fdy) { return (int)roundf((bl * d) * fdy); }

template <int K, int TH, int DPW>
__global__ __launch_bounds__(256) void k_ncc_volume(const uint8_t* __restrict__ q, const int* __restrict__ boxS,
                                                    const float* __restrict__ boxI,
                                                    const float* __restrict__ levels, NccArgs a,
                                                    float* __restrict__ vol) {
  constexpr int R = K / 2;
  constexpr int OUT = 64 - 2 * R;
  constexpr int NR = TH + 2 * R;
  constexpr int NK = K * K;
  constexpr int DC = 4 * DPW;
  extern __shared__ __align__(16) uint8_t smem[];
  const int bwp = a.band_w;                        // band width, multiple of 64
  int* rS = (int*)smem;                            // [TH][64] window sums, reference
  float* rI = (float*)(rS + TH * 64);              // [TH][64] reciprocal variances
  const int nbuf = 2 * a.box_h * bwp + a.band_h * bwp;  // dwords per neighbour buffer
  uint32_t* rq = (uint32_t*)(rI + TH * 64);        // [NR][64] intensities, reference (1 dword/px)
  uint32_t* nbase = rq + NR * 64;                  // 2 x {nS[box_h][bwp], nI[box_h][bwp], nq[band_h][bwp]}

  // wave id made provably uniform: its level loads become scalar (SMEM), so no
  // vector-memory wait can drain the in-flight LDS-DMA prefetch
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int W = a.W, H = a.H;
  const long P = (long)W * H;
  const int x0 = blockIdx.x * OUT - R;  // image column of lane 0
  const int y0 = blockIdx.y * TH;
  const int d_lo = blockIdx.z * DC, d_hi = min(a.D, d_lo + DC);
  const int x = x0 + lane;

  // extents of the chunk's shifts for neighbour n (uniform)
  auto extents = [&](int n, int& txmin, int& txmax, int& tymin, int& tymax) {
    if (a.monotone) {  // non-decreasing levels: roundf(d*c) is monotone in d
      float d0 = levels[d_lo], d1 = levels[d_hi - 1];
      int t0 = shift_x(d0, a.fdx[n]), t1 = shift_x(d1, a.fdx[n]);
      int u0 = shift_y(a.bl, d0, a.fdy[n]), u1 = shift_y(a.bl, d1, a.fdy[n]);
      txmin = min(t0, t1); txmax = max(t0, t1);
      tymin = min(u0, u1); tymax = max(u0, u1);
      return;
    }
    txmin = 1 << 30; txmax = -(1 << 30); tymin = 1 << 30; tymax = -(1 << 30);
    for (int dl = d_lo; dl < d_hi; dl++) {
      float d = levels[dl];
      int tx = shift_x(d, a.fdx[n]), ty = shift_y(a.bl, d, a.fdy[n]);
      txmin = min(txmin, tx); txmax = max(txmax, tx);
      tymin = min(tymin, ty); tymax = max(tymax, ty);
    }
  };
  // LDS-DMA staging of neighbour n's bands into buffer b: (row, 64-column
  // block) pieces dealt to the 4 waves, asynchronous until the next barrier
  auto stage = [&](int n, int b) {
    int txmin, txmax, tymin, tymax;
    extents(n, txmin, txmax, tymin, tymax);
    const int nblk = (64 + txmax - txmin + 63) >> 6;
    const int bh = NR + tymax - tymin, bxh = TH + tymax - tymin;
    const int bx0 = x0 - txmax, by0 = y0 - R - tymax, bby0 = y0 - tymax;
    const uint8_t* Qv = q + (long)a.view[n] * P;
    const int* BSv = boxS + (long)a.view[n] * P;
    const float* BIv = boxI + (long)a.view[n] * P;
    uint32_t* buf = nbase + b * nbuf;
    int* nS = (int*)buf;
    float* nI = (float*)(buf + a.box_h * bwp);
    uint32_t* nq = buf + 2 * a.box_h * bwp;
    for (int cb = 0; cb < nblk; cb++) {  // wave w stages rows w, w+4, ...
      const int xx = min(max(bx0 + cb * 64 + lane, 0), W - 1);
      for (int r = wave; r < bh; r += 4)
        glds_u8(Qv + (long)min(max(by0 + r, 0), H - 1) * W + xx, nq + r * bwp + cb * 64);
      for (int r = wave; r < bxh; r += 4) {
        const long row = (long)min(max(bby0 + r, 0), H - 1) * W + xx;
        glds_b32(BSv + row, nS + r * bwp + cb * 64);
        glds_b32(BIv + row, nI + r * bwp + cb * 64);
      }
    }
  };

  // ---- reference band + statistics: LDS-DMA, one 64-lane row per instruction
  const uint8_t* Qz = q + (long)a.z * P;
  const int* BSz = boxS + (long)a.z * P;
  const float* BIz = boxI + (long)a.z * P;
  {
    const int xx = min(max(x, 0), W - 1);
    for (int r = wave; r < NR; r += 4)
      glds_u8(Qz + (long)min(max(y0 - R + r, 0), H - 1) * W + xx, rq + r * 64);
    for (int r = wave; r < TH; r += 4) {
      const long row = (long)min(y0 + r, H - 1) * W + xx;
      glds_b32(BSz + row, rS + r * 64);
      glds_b32(BIz + row, rI + r * 64);
    }
  }
  if (a.nn > 0) stage(0, 0);
  const bool xin = x >= R && x < W - R;
  const unsigned rrows = bit_range(R - y0, H - 1 - R - y0);  // reference rows with a full window
  float mn[DPW][TH];
#pragma unroll
  for (int j = 0; j < DPW; j++)
#pragma unroll
    for (int o = 0; o < TH; o++) mn[j][o] = 1000000.0f;
  __syncthreads();
  int qr[NR];
#pragma unroll
  for (int k = 0; k < NR; k++) qr[k] = rq[k * 64 + lane];

  for (int n = 0; n < a.nn; n++) {
    // prefetch the next neighbour's bands while this one is computed
    if (n + 1 < a.nn) stage(n + 1, (n + 1) & 1);
    const float fdx = a.fdx[n], fdy = a.fdy[n];
    int txmin, txmax, tymin, tymax;
    extents(n, txmin, txmax, tymin, tymax);
    const uint32_t* buf = nbase + (n & 1) * nbuf;
    const int* nS = (const int*)buf;
    const float* nI = (const float*)(buf + a.box_h * bwp);
    const uint32_t* nq = buf + 2 * a.box_h * bwp;
#pragma unroll
    for (int j = 0; j < DPW; j++) {
      const int dl = d_lo + wave + 4 * j;
      if (dl >= d_hi) break;  // wave-uniform
      const float d = levels[dl];
      const int tx = shift_x(d, fdx), ty = shift_y(a.bl, d, fdy);
      const int col = lane + txmax - tx;          // band column of x - tx
      const int rowq = tymax - ty;                // band row offset of y0-R-ty
      const int xp = x - tx;
      const bool xpin = xp >= R && xp < W - R;
      // bit o: both K x K windows of output row o lie inside the image
      const unsigned vmask = (xin && xpin) ? (rrows & bit_range(R - y0 + ty, H - 1 - R - y0 + ty)) : 0u;
      const uint32_t* nqp = nq + rowq * bwp + col;
      int hs[NR];
#pragma unroll
      for (int k = 0; k < NR; k++) {
        int qp = nqp[0];
        nqp += bwp;
        hs[k] = hsum<R>((int)__umul24(qr[k], qp));
      }
      int srp = 0;
#pragma unroll
      for (int k = 0; k < 2 * R; k++) srp += hs[k];
      const int nb = rowq * bwp + col;
#pragma unroll
      for (int o = 0; o < TH; o++) {
        srp += hs[o + 2 * R];
        const int sr = rS[o * 64 + lane], sp = nS[nb + o * bwp];
        const float ivr = rI[o * 64 + lane], ivp = nI[nb + o * bwp];
        const bool valid = (vmask >> o) & 1u;
        const int num = __mul24(NK, srp) - (int)__umul24(sr, sp);
        const float fa = (float)num;
        float e = fa * fabsf(fa);
        e = e * ivr;
        e = e * ivp;
        const float c = valid ? 1.0f - e : 2.0f;
        mn[j][o] = c < mn[j][o] ? c : mn[j][o];
        srp -= hs[o];
      }
    }
    __syncthreads();  // next bands landed (vmcnt 0); this buffer free for n+2
  }
  const bool out_lane = lane >= R && lane < 64 - R && x < W;
#pragma unroll
  for (int j = 0; j < DPW; j++) {
    const int dl = d_lo + wave + 4 * j;
    if (dl >= d_hi) break;
    float* vd = vol + (long)dl * P;
    if (out_lane) {
#pragma unroll
      for (int o = 0; o < TH; o++)
        if (y0 + o < H) vd[(long)(y0 + o) * W + x] = mn[j][o];
    }
  }
}

template <int K, int TH, int DPW>
int launch_ncc_t(hipStream_t s, const uint8_t* l8, const int* boxS, const float* boxI, const float* levels_dev,
                 NccArgs& a,
                 const float* levels_host, float* vol) {
  constexpr int R = K / 2, OUT = 64 - 2 * R, NR = TH + 2 * R, DC = 4 * DPW;
  int spx = 0, spy = 0;
  for (int d0 = 0; d0 < a.D; d0 += DC)
    for (int n = 0; n < a.nn; n++) {
      int txmin = 1 << 30, txmax = -(1 << 30), tymin = 1 << 30, tymax = -(1 << 30);
      for (int dl = d0; dl < std::min(a.D, d0 + DC); dl++) {
        float d = levels_host[dl];
        int tx = (int)roundf(d * a.fdx[n]), ty = (int)roundf((a.bl * d) * a.fdy[n]);
        txmin = std::min(txmin, tx); txmax = std::max(txmax, tx);
        tymin = std::min(tymin, ty); tymax = std::max(tymax, ty);
      }
      spx = std::max(spx, txmax - txmin);
      spy = std::max(spy, tymax - tymin);
    }
  a.band_w = (64 + spx + 63) & ~63;  // whole 64-lane LDS-DMA pieces per row
  a.band_h = NR + spy;
  a.box_h = TH + spy;
  size_t lds = 4 * (2 * TH * 64 + NR * 64 + 2 * (2 * (size_t)a.box_h * a.band_w + (size_t)a.band_h * a.band_w));
  lds = (lds + 15) & ~(size_t)15;
  if (lds > 160 * 1024) return -1;  // caller retries with a smaller chunk
  dim3 g((a.W + OUT - 1) / OUT, (a.H + TH - 1) / TH, (a.D + DC - 1) / DC);
  if (lds > 64 * 1024)
    MVS_HIP(hipFuncSetAttribute((const void*)k_ncc_volume<K, TH, DPW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds), "hipFuncSetAttribute(ncc lds)");
  hipLaunchKernelGGL((k_ncc_volume<K, TH, DPW>), g, dim3(256), lds, s, l8, boxS, boxI, levels_dev, a, vol);
  MVS_LAUNCH_CHECK("k_ncc_volume");
  return 0;
}

}  // namespace

int launch_box_stats(hipStream_t s, const uint8_t* l8, int V, int W, int H, int K, int32_t* box) {
  hipLaunchKernelGGL(k_box_stats, dim3((W + 255) / 256, H, V), dim3(256), 0, s, l8, W, H, K, box,
                     (float*)(box + (long)V * W * H));
  MVS_LAUNCH_CHECK("k_box_stats");
  return 0;
}

int launch_ncc_volume(hipStream_t s, int V, int W, int H, const uint8_t* l8, const int32_t* box,
                      const float* levels_dev, const float* levels_host, int D, const int* vs_host,
                      const int* sn_host, int aw, float bl, int K, int z, float* vol) {
  constexpr int TH = 16;
  NccArgs a{};
  a.W = W; a.H = H; a.D = D; a.z = z; a.bl = bl;
  a.nn = sn_host[z];
  if (a.nn > kMaxNbr) return arg_fail("NCC sweep supports at most 16 neighbours per reference view");
  a.monotone = 1;
  for (int i = 1; i < D; i++)
    if (!(levels_host[i] >= levels_host[i - 1])) a.monotone = 0;
  int rx = z % aw, ry = z / aw;
  for (int n = 0; n < a.nn; n++) {
    int v = vs_host[V * z + n];
    if (v < 0 || v >= V) return arg_fail("view_subset entry out of range");
    a.view[n] = v;
    a.fdx[n] = (float)(v % aw - rx);
    a.fdy[n] = (float)(v / aw - ry);
  }
  const int* bS = box;                                   // plane 0: window sums
  const float* bI = (const float*)(box + (long)V * W * H);  // plane 1: reciprocal variances
  int rc = -1;
  static const int dpw_env = [] {
    const char* e = getenv("MVS_NCC_DPW");
    return e ? atoi(e) : 4;
  }();
  if (K == 5) {
    if (dpw_env >= 4) rc = launch_ncc_t<5, TH, 4>(s, l8, bS, bI, levels_dev, a, levels_host, vol);
    if (rc < 0 && dpw_env >= 2) rc = launch_ncc_t<5, TH, 2>(s, l8, bS, bI, levels_dev, a, levels_host, vol);
    if (rc < 0) rc = launch_ncc_t<5, TH, 1>(s, l8, bS, bI, levels_dev, a, levels_host, vol);
  } else if (K == 7) {
    if (dpw_env >= 4) rc = launch_ncc_t<7, TH, 4>(s, l8, bS, bI, levels_dev, a, levels_host, vol);
    if (rc < 0 && dpw_env >= 2) rc = launch_ncc_t<7, TH, 2>(s, l8, bS, bI, levels_dev, a, levels_host, vol);
    if (rc < 0) rc = launch_ncc_t<7, TH, 1>(s, l8, bS, bI, levels_dev, a, levels_host, vol);
  } else {
    return arg_fail("NCC window must be 5 or 7");
  }
  if (rc < 0) return arg_fail("NCC sweep: neighbour shifts too large for the LDS band");
  return rc;
}

}  // namespace mvs
