// Build-defined per-pixel NCC K x K plane sweep: the cost-volume producer.
//
// Definition (no reference counterpart; restated in oracle/mvs_oracle.c
// orc_ncc_volume): q = 8-bit intensity (clamp(int(L*2.55+0.5))), window K x K,
// shift of neighbour n at level d: (tx, ty) = (roundf(d*dx), roundf((bl*d)*dy)),
// window valid iff every tap of the reference and the shifted window is inside
// the image; with n = K*K and integer sums
//   num = n*Srp - Sr*Sp,  vr = n*Srr - Sr^2,  vp = n*Spp - Sp^2
// ivr = vr ? 1/(float)vr : 0 and ivp likewise (per pixel),
// e_n = ((a*|a|)*ivr)*ivp with a = (float)num (signed squared NCC) for valid
// windows; vol[d][y][x] = 1 - max(-1, max over valid neighbours e_n): 1 minus
// the best signed squared correlation, 2 when no neighbour window is valid.
//
// Data layout (mvs_box_stats_d, per view, 16 B/px in two planes):
//   stats [V][H][W] {S, bits(ivr)}: window sum and reciprocal variance, with
//                   ivr = NaN where the window leaves the image;
//   pk    [V][H][W] {lo, hi}: the 8 intensities q(x-R .. x-R+7) of row y
//                   packed little-endian (0 outside the image).
// Validity is carried by the data: an invalid window anywhere makes e NaN and
// v_max_f32 (IEEE maxNum) drops it -- no per-cell bounds logic.
//
// Kernel (gfx950, wave64, 4 waves per workgroup):
//   * tile = 64 image columns (one per lane) x TH rows x a chunk of 4*DPW
//     hypotheses; wave w owns levels w, w+4, ...;
//   * the reference's packed rows and window stats live in registers;
//   * per neighbour, the pk and stats bands covering every shift of the chunk
//     are staged in LDS by 16-byte LDS-DMA (2 px per lane), double-buffered so
//     the next neighbour's bands land while this one is computed;
//   * per (level, neighbour) a lane walks its column: per band row one
//     ds_read_b64 and two v_dot4_u32_u8 give the exact horizontal K-tap
//     correlation, a register sliding window the vertical K-sum, then 7 VALU
//     ops finish the cell (integer num, IEEE f32 e, v_max_f32);
//   * the chunk's costs are written once, 64-column coalesced rows.
#include <algorithm>
#include <cstdlib>

#include "mvs_internal.h"

namespace mvs {
namespace {

// ---- window statistics + packed intensities ------------------------------
// one workgroup = 64 columns x 16 rows of one view; the (16+2R) x (64+2R)
// byte tile is staged in LDS once.
constexpr int BS_TW = 64, BS_TH = 16;
template <int R>
__global__ __launch_bounds__(256) void k_box_stats(const uint8_t* __restrict__ q, int W, int H,
                                                   uint2* __restrict__ stats, uint2* __restrict__ pk) {
  constexpr int K = 2 * R + 1, NK = K * K;
  constexpr int TW = BS_TW + 8, TR = BS_TH + 2 * R;  // tile covers columns x0-R .. x0+63-R+7
  __shared__ uint8_t t[TR][TW + 4];
  const int x0 = blockIdx.x * BS_TW, y0 = blockIdx.y * BS_TH, z = blockIdx.z;
  const long P = (long)W * H;
  const uint8_t* Q = q + z * P;
  for (int i = threadIdx.x; i < TR * TW; i += 256) {
    int r = i / TW, c = i % TW;
    int yy = y0 - R + r, xx = x0 - R + c;
    t[r][c] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? Q[(long)yy * W + xx] : 0;
  }
  __syncthreads();
  const int lx = threadIdx.x & 63, ly0 = (threadIdx.x >> 6) * 4;  // 4 rows per thread
  const int x = x0 + lx;
  if (x >= W) return;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int ly = ly0 + k, y = y0 + ly;
    if (y >= H) break;
    int s = 0, ss = 0;
#pragma unroll
    for (int j = 0; j < K; j++)
#pragma unroll
      for (int i = 0; i < K; i++) {
        int v = t[ly + j][lx + i];
        s += v;
        ss += v * v;
      }
    const bool valid = x - R >= 0 && x + R < W && y - R >= 0 && y + R < H;
    const int var = NK * ss - s * s;
    const float iv = !valid ? __int_as_float(0x7fc00000) : (var != 0 ? 1.0f / (float)var : 0.0f);
    const long o = z * P + (long)y * W + x;
    stats[o] = make_uint2((unsigned)(valid ? s : 0), (unsigned)__float_as_int(iv));
    const uint8_t* row = &t[ly + R][lx];
    unsigned lo = row[0] | (row[1] << 8) | (row[2] << 16) | ((unsigned)row[3] << 24);
    unsigned hi = row[4] | (row[5] << 8) | (row[6] << 16) | ((unsigned)row[7] << 24);
    pk[o] = make_uint2(lo, hi);
  }
}

constexpr int kMaxNbr = 16;
struct NccArgs {
  int W, H, D, nn, z;
  int view[kMaxNbr];
  int band_h, box_h;  // LDS band heights (rows); the row stride is the template BW
};
// host-built plan (device memory, cached per context), passed as separate
// __restrict__ kernel parameters so its loads are scalar (SMEM: they never
// wait on the vector-memory counter that the LDS-DMA prefetch runs under):
//   chunk[c][n] = {txmax, tymax, bh (pk rows to stage), sh (stats rows) | nblk << 16}
//   lvl[n][dl]  = {txmax - tx, tymax - ty} of level dl in its chunk

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gptr_t;
// 16-byte LDS-DMA: lane l's 16 bytes land at dst + 16*l (dst wave-uniform)
__device__ __forceinline__ void glds_b128(const void* src, void* dst) {
  __builtin_amdgcn_global_load_lds((gptr_t)src, (lds_ptr_t)dst, 16, 0, 0);
}

// v_max_f32 (IEEE maxNum: a quiet-NaN operand is dropped).  Inline asm so the
// compiler does not re-canonicalise the loop-carried accumulators every pass.
__device__ __forceinline__ float vmax(float acc, float e) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(acc), "v"(e));
  return r;
}

template <int K, int TH, int DPW, int BW>
__global__ __launch_bounds__(256) void k_ncc_volume(const uint2* __restrict__ stats, const uint2* __restrict__ pk,
                                                    const int4* __restrict__ plan_chunk,
                                                    const int2* __restrict__ plan_lvl, NccArgs a,
                                                    float* __restrict__ vol) {
  constexpr int R = K / 2;
  constexpr int NR = TH + 2 * R;
  constexpr int NK = K * K;
  constexpr int DC = 4 * DPW;
  // taps x-R .. x-R+3 in lo, x-R+4 .. x+R in the low K-4 bytes of hi
  constexpr unsigned HI_MASK = (K - 4) >= 4 ? 0xffffffffu : ((1u << (8 * (K - 4))) - 1u);
  extern __shared__ __align__(16) uint8_t smem[];
  const int nbuf = (a.band_h + a.box_h) * BW;  // uint2 per neighbour buffer
  uint2* nbase = (uint2*)smem;                 // 2 x {npk[band_h][BW], nst[box_h][BW]}

  // wave id made provably uniform: plan loads become scalar (SMEM), so no
  // vector-memory wait drains the in-flight LDS-DMA prefetch
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int W = a.W, H = a.H;
  const long P = (long)W * H;
  const int x0 = blockIdx.x * 64;
  const int y0 = blockIdx.y * TH;
  const int c = blockIdx.z;
  const int d_lo = c * DC, d_hi = min(a.D, d_lo + DC);
  const int x = x0 + lane;
  const int4* chunk = plan_chunk + c * a.nn;

  // LDS-DMA staging of neighbour n's bands into buffer b.  Band column j is
  // image column x0 - txmax + j; band row r of pk is image row y0-R-tymax+r,
  // of stats y0-tymax+r.  Columns and rows are clamped into the image: an
  // edge pixel's window is invalid (NaN ivr) for R >= 1, so clamped cells
  // never contribute.  A lane moves 2 px (16 B); pairs are clamped as a pair.
  auto stage = [&](int n, int b) {
    const int4 e = chunk[n];
    const int bh = e.z, sh = e.w & 0xffff, nblk = e.w >> 16;
    const int bx0 = x0 - e.x, by0 = y0 - R - e.y, sy0 = y0 - e.y;
    const long vo = (long)a.view[n] * P;
    uint2* npk = nbase + b * nbuf;
    uint2* nst = npk + a.band_h * BW;
    for (int cb = 0; cb < nblk; cb++) {
      const uint2* gpk = pk + vo + min(max(bx0 + cb * 128 + 2 * lane, 0), W - 2);
      const uint2* gst = stats + vo + min(max(bx0 + cb * 128 + 2 * lane, 0), W - 2);
      for (int r = wave; r < bh; r += 4)
        glds_b128(gpk + (long)min(max(by0 + r, 0), H - 1) * W, npk + r * BW + cb * 128);
      for (int r = wave; r < sh; r += 4)
        glds_b128(gst + (long)min(max(sy0 + r, 0), H - 1) * W, nst + r * BW + cb * 128);
    }
  };

  if (a.nn > 0) stage(0, 0);
  // reference: packed rows y0-R .. y0+TH+R-1 and window stats of rows y0 .. y0+TH-1
  const long zo = (long)a.z * P;
  const int xc = min(x, W - 1);
  unsigned qlo[NR], qhi[NR];
#pragma unroll
  for (int k = 0; k < NR; k++) {
    const uint2 v = pk[zo + (long)min(max(y0 - R + k, 0), H - 1) * W + xc];
    qlo[k] = v.x;
    qhi[k] = v.y & HI_MASK;
  }
  int nsr[TH];  // -Sr, so num = n*Srp + (-Sr)*Sp is one mul24 + one mad24
  float ivr[TH];
#pragma unroll
  for (int o = 0; o < TH; o++) {
    const uint2 v = stats[zo + (long)min(y0 + o, H - 1) * W + xc];
    nsr[o] = -(int)v.x;
    ivr[o] = __int_as_float((int)v.y);
  }
  float E[DPW][TH];
#pragma unroll
  for (int j = 0; j < DPW; j++)
#pragma unroll
    for (int o = 0; o < TH; o++) E[j][o] = -1.0f;
  __syncthreads();

  for (int n = 0; n < a.nn; n++) {
    if (n + 1 < a.nn) stage(n + 1, (n + 1) & 1);  // prefetch while computing n
    const uint2* npk = nbase + (n & 1) * nbuf;
    const uint2* nst = npk + a.band_h * BW;
    const int2* lv = plan_lvl + n * a.D;
#pragma unroll
    for (int j = 0; j < DPW; j++) {
      const int dl = d_lo + wave + 4 * j;
      if (dl >= d_hi) break;  // wave-uniform
      const int2 sh = lv[dl];  // {band column of x0 - tx, band row of y0 - R - ty}
      const uint2* p = npk + sh.y * BW + sh.x + lane;
      int hs[NR];
#pragma unroll
      for (int k = 0; k < NR; k++) {
        const uint2 v = p[k * BW];
        hs[k] = (int)__builtin_amdgcn_udot4(qhi[k], v.y, __builtin_amdgcn_udot4(qlo[k], v.x, 0u, false), false);
      }
      const uint2* s = nst + sh.y * BW + sh.x + lane;
      int srp = 0;
#pragma unroll
      for (int k = 0; k < 2 * R; k++) srp += hs[k];
#pragma unroll
      for (int o = 0; o < TH; o++) {
        srp += hs[o + 2 * R];
        const uint2 st = s[o * BW];
        const int num = __mul24(NK, srp) + __mul24(nsr[o], (int)st.x);
        const float fa = (float)num;
        float e = fa * fabsf(fa);
        e = e * ivr[o];
        e = e * __int_as_float((int)st.y);
        E[j][o] = vmax(E[j][o], e);
        srp -= hs[o];
      }
    }
    __syncthreads();  // next bands landed (vmcnt 0); this buffer free for n+2
  }
  if (x >= W) return;
#pragma unroll
  for (int j = 0; j < DPW; j++) {
    const int dl = d_lo + wave + 4 * j;
    if (dl >= d_hi) break;
    float* vd = vol + (long)dl * P;
#pragma unroll
    for (int o = 0; o < TH; o++)
      if (y0 + o < H) vd[(long)(y0 + o) * W + x] = 1.0f - E[j][o];
  }
}

// Host side: the chunk/level shift plan (every roundf of the definition is
// evaluated here, once per distinct configuration) and the launch.
struct NccPlan {
  std::vector<int32_t> table;  // chunk int4 [nchunks][nn], then lvl int2 [nn][D]
  int band_w = 0, band_h = 0, box_h = 0;
};

template <int K, int TH, int DPW>
NccPlan make_plan(const float* levels, int D, int nn, const float* fdx, const float* fdy, float bl) {
  constexpr int R = K / 2, NR = TH + 2 * R, DC = 4 * DPW;
  const int nch = (D + DC - 1) / DC;
  NccPlan p;
  p.table.assign((size_t)nch * nn * 4 + (size_t)nn * D * 2, 0);
  int32_t* ch = p.table.data();
  int32_t* lv = ch + (size_t)nch * nn * 4;
  int spx = 0, spy = 0;
  for (int c = 0; c < nch; c++)
    for (int n = 0; n < nn; n++) {
      int txmin = 1 << 30, txmax = -(1 << 30), tymin = 1 << 30, tymax = -(1 << 30);
      for (int dl = c * DC; dl < std::min(D, c * DC + DC); dl++) {
        const float d = levels[dl];
        const int tx = (int)roundf(d * fdx[n]), ty = (int)roundf((bl * d) * fdy[n]);
        txmin = std::min(txmin, tx); txmax = std::max(txmax, tx);
        tymin = std::min(tymin, ty); tymax = std::max(tymax, ty);
      }
      for (int dl = c * DC; dl < std::min(D, c * DC + DC); dl++) {
        const float d = levels[dl];
        const int tx = (int)roundf(d * fdx[n]), ty = (int)roundf((bl * d) * fdy[n]);
        lv[2 * ((size_t)n * D + dl)] = txmax - tx;
        lv[2 * ((size_t)n * D + dl) + 1] = tymax - ty;
      }
      const int nblk = (64 + txmax - txmin + 127) >> 7;
      int32_t* e = ch + 4 * ((size_t)c * nn + n);
      e[0] = txmax;
      e[1] = tymax;
      e[2] = NR + tymax - tymin;
      e[3] = (TH + tymax - tymin) | (nblk << 16);
      spx = std::max(spx, txmax - txmin);
      spy = std::max(spy, tymax - tymin);
    }
  p.band_w = (64 + spx + 127) & ~127;  // whole 128-px LDS-DMA pieces per row
  p.band_h = NR + spy;
  p.box_h = TH + spy;
  return p;
}

template <int K, int TH, int DPW, int BW>
int launch_ncc_bw(hipStream_t s, const uint2* stats, const uint2* pk, const int4* chunk, const int2* lvl,
                  NccArgs& a, float* vol, size_t lds) {
  constexpr int DC = 4 * DPW;
  dim3 g((a.W + 63) / 64, (a.H + TH - 1) / TH, (a.D + DC - 1) / DC);
  if (lds > 64 * 1024)
    MVS_HIP(hipFuncSetAttribute((const void*)k_ncc_volume<K, TH, DPW, BW>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "hipFuncSetAttribute(ncc lds)");
  hipLaunchKernelGGL((k_ncc_volume<K, TH, DPW, BW>), g, dim3(256), lds, s, stats, pk, chunk, lvl, a, vol);
  MVS_LAUNCH_CHECK("k_ncc_volume");
  return 0;
}

// returns 1 if this variant does not fit the LDS (caller tries a smaller one)
template <int K, int TH, int DPW>
int launch_ncc_t(mvs_ctx* ctx, const uint2* stats, const uint2* pk, NccArgs& a, const float* levels_host,
                 const float* fdx, const float* fdy, float bl, float* vol) {
  NccPlan p = make_plan<K, TH, DPW>(levels_host, a.D, a.nn, fdx, fdy, bl);
  const size_t lds = 2 * 8 * (size_t)(p.band_h + p.box_h) * p.band_w;
  if (lds > 160 * 1024 || (p.band_w != 128 && p.band_w != 256)) return 1;
  int rc = 0;
  const int32_t* dev = plan_upload(ctx, p.table, &rc);
  if (rc) return rc;
  a.band_h = p.band_h;
  a.box_h = p.box_h;
  const int nch = (a.D + 4 * DPW - 1) / (4 * DPW);
  const int4* chunk = (const int4*)dev;
  const int2* lvl = (const int2*)(dev + (size_t)nch * a.nn * 4);
  if (p.band_w == 128) return launch_ncc_bw<K, TH, DPW, 128>(ctx->stream, stats, pk, chunk, lvl, a, vol, lds);
  return launch_ncc_bw<K, TH, DPW, 256>(ctx->stream, stats, pk, chunk, lvl, a, vol, lds);
}

}  // namespace

int launch_box_stats(hipStream_t s, const uint8_t* l8, int V, int W, int H, int K, int32_t* box) {
  uint2* stats = (uint2*)box;
  uint2* pk = stats + (long)V * W * H;
  dim3 g((W + BS_TW - 1) / BS_TW, (H + BS_TH - 1) / BS_TH, V);
  if (K == 5)
    hipLaunchKernelGGL(k_box_stats<2>, g, dim3(256), 0, s, l8, W, H, stats, pk);
  else
    hipLaunchKernelGGL(k_box_stats<3>, g, dim3(256), 0, s, l8, W, H, stats, pk);
  MVS_LAUNCH_CHECK("k_box_stats");
  return 0;
}

int launch_ncc_volume(mvs_ctx* ctx, int V, int W, int H, const int32_t* box, const float* levels_host, int D,
                      const int* vs_host, const int* sn_host, int aw, float bl, int K, int z, float* vol) {
  if (W < 2) return arg_fail("NCC sweep needs W >= 2");
  NccArgs a{};
  a.W = W; a.H = H; a.D = D; a.z = z;
  a.nn = sn_host[z];
  if (a.nn > kMaxNbr) return arg_fail("NCC sweep supports at most 16 neighbours per reference view");
  float fdx[kMaxNbr], fdy[kMaxNbr];
  int rx = z % aw, ry = z / aw;
  for (int n = 0; n < a.nn; n++) {
    int v = vs_host[V * z + n];
    if (v < 0 || v >= V) return arg_fail("view_subset entry out of range");
    a.view[n] = v;
    fdx[n] = (float)(v % aw - rx);
    fdy[n] = (float)(v / aw - ry);
  }
  const uint2* stats = (const uint2*)box;
  const uint2* pk = stats + (long)V * W * H;
  // tile height and levels per wave: MVS_NCC_TH (8|16), MVS_NCC_DPW (1|2|4)
  static const int dpw_env = [] {
    const char* e = getenv("MVS_NCC_DPW");
    return e ? atoi(e) : 4;
  }();
  static const int th_env = [] {
    const char* e = getenv("MVS_NCC_TH");
    return e ? atoi(e) : 8;
  }();
  int rc = 1;
#define MVS_NCC_TRY(KK, TT, PP)                                                                     \
  if (rc == 1) rc = launch_ncc_t<KK, TT, PP>(ctx, stats, pk, a, levels_host, fdx, fdy, bl, vol);
  if (K == 5) {
    if (th_env == 16) {
      if (dpw_env >= 4) MVS_NCC_TRY(5, 16, 4)
      if (dpw_env >= 2) MVS_NCC_TRY(5, 16, 2)
    }
    if (dpw_env >= 4) MVS_NCC_TRY(5, 8, 4)
    if (dpw_env >= 2) MVS_NCC_TRY(5, 8, 2)
    MVS_NCC_TRY(5, 8, 1)
  } else if (K == 7) {
    if (th_env == 16) {
      if (dpw_env >= 4) MVS_NCC_TRY(7, 16, 4)
      if (dpw_env >= 2) MVS_NCC_TRY(7, 16, 2)
    }
    if (dpw_env >= 4) MVS_NCC_TRY(7, 8, 4)
    if (dpw_env >= 2) MVS_NCC_TRY(7, 8, 2)
    MVS_NCC_TRY(7, 8, 1)
  } else {
    return arg_fail("NCC window must be 5 or 7");
  }
#undef MVS_NCC_TRY
  if (rc == 1) return arg_fail("NCC sweep: neighbour shifts too large for the LDS band");
  return rc;
}

}  // namespace mvs
