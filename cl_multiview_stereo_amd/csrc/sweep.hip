// Photo-consistency plane-sweep kernels for gfx950 (CDNA4, wave64).
//
//  k_boundary        find_super_pixel_boundary           clcode.cl:791-855
//  k_sweep_spixl     initial_depth_estimation_v2          clcode.cl:972-1069
//                    (one wave per superpixel, lanes over hypotheses,
//                    exact first-minimum WTA by a (cost, index) wave reduction)
//  k_sad_band        the same sweep at S=1 grid semantics (reference-parity
//                    per-pixel mode): per (chunk of levels, neighbour) the
//                    neighbour's Lab band is staged in LDS once (LDS-DMA,
//                    double-buffered) and serves every level of the chunk; per
//                    level pair a lane forms its column's absolute differences
//                    and the 25-tap sums run in the reference's order as
//                    v_pk_add_f32 over the two levels, the window columns
//                    passed lane to lane by DPP wave_shr (systolic)
//                    or through an LDS plane (the first, two-phase form).
//  k_sweep_pixel_sad the first per-pixel form (every (d, neighbour) region
//                    gathered from global memory): kept for level sets with
//                    fractional column shifts.
//  (the NCC cost-volume kernels are in ncc.hip)
//  k_wta             winner-take-all + confidence over the materialised volume
//                    (the HBM-streaming pass the roofline is quoted on).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mvs_internal.h"

namespace mvs {
namespace {

// ---- find_super_pixel_boundary, clcode.cl:791-855 -------------------------
// One wave per superpixel.  The reference walks i = 1 .. S-1 along 8
// directions from the (clamped) centre and keeps, per direction, i - 1 of the
// last i whose pixel still carries the superpixel's label: a maximum over
// independent tests.  Lane 8k + j tests direction k at i = 1 + j + 8m, so the
// 8 (S - 1) label gathers issue together instead of as one thread's chain
// (C2: 30 -> see DESIGN.md), and an xor-butterfly takes each direction's
// maximum.  Integer results: identical.
__global__ __launch_bounds__(256) void k_boundary(const float* __restrict__ spixl,
                                                  const uint32_t* __restrict__ labels, int W, int H, int S, int mw,
                                                  int mh, uint8_t* __restrict__ rep) {
  const int lane = threadIdx.x & 63;
  const long s = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int z = blockIdx.y;
  const long M = (long)mw * mh, P = (long)W * H;
  if (s >= M) return;  // whole wave
  const float* sp = spixl + 8 * (z * M + s);
  int cx = (int)sp[1], cy = (int)sp[2];
  if (cx < S) cx += (S - cx);
  if (cx + S > W) cx -= S;
  if (cy < S) cy += (S - cy);
  if (cy + S > H) cy -= S;
  const uint32_t id = (uint32_t)s;
  const uint32_t* L = labels + z * P;
  const int k = lane >> 3, j = lane & 7;
  // direction k: (dx, dy) in the reference's order d0 .. d7
  const int dx = k < 3 ? -1 : (k < 5 ? 0 : 1);
  const int dy = (k == 0 || k == 3 || k == 5) ? -1 : ((k == 1 || k == 6) ? 0 : 1);
  int d = 0;
  for (int i0 = 1; i0 < S; i0 += 32) {
    uint32_t v[4];
    bool in[4];
#pragma unroll
    for (int m = 0; m < 4; m++) {  // unconditional (clamped) loads: all four in flight together
      const int i = i0 + j + 8 * m, xx = cx + dx * i, yy = cy + dy * i;
      in[m] = i < S && xx >= 0 && xx < W && yy >= 0 && yy < H;
      v[m] = L[in[m] ? (long)yy * W + xx : 0];
    }
#pragma unroll
    for (int m = 0; m < 4; m++)
      if (in[m] && v[m] == id) d = i0 + j + 8 * m - 1;  // i grows: the last hit is the largest
  }
  d = max(d, __shfl_xor(d, 1));
  d = max(d, __shfl_xor(d, 2));
  d = max(d, __shfl_xor(d, 4));
  uint32_t w = (uint32_t)(d & 0xff) << (8 * (k & 3));
  w |= __shfl_xor(w, 8);
  w |= __shfl_xor(w, 16);  // lane 0: directions 0-3, lane 32: directions 4-7
  const uint32_t hi = __shfl(w, 32);
  if (lane == 0) *(uint2*)(rep + 8 * (z * M + s)) = make_uint2(w, hi);
}

// 16-byte LDS-DMA: lane l's 16 bytes land at dst + 16 l (dst wave-uniform)
typedef __attribute__((address_space(3))) void* lds_vptr_t;
typedef const __attribute__((address_space(1))) void* glb_vptr_t;
__device__ __forceinline__ void glds16(const void* src, void* dst) {
  __builtin_amdgcn_global_load_lds((glb_vptr_t)src, (lds_vptr_t)dst, 16, 0, 0);
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
// Vertical and diagonal neighbours: lane = level puts 64 levels' taps on 64
// different rows -- 64 cache lines per gather instruction, 16 B used of each
// 128 (measured at C4, 8x4 array, 5 nearest neighbours, all 32 views:
// TCC_MISS 271 M per launch against 175 M hits, 4.66 ms).  labT (optional)
// holds such neighbour views re-laid so that consecutive levels' taps are
// consecutive elements: at labT + tslot[4 * view + kind] * tstride
// of kind 1 (same camera column: transposed, element (x, y) at x H + y),
// 2 (dx == dy: sheared, at (x - y + H - 1) H + y) or 3 (dx == -dy: at
// (x + y) H + y).  With bl != 1 the diagonal shifts drift apart by a row
// every 1/|bl - 1| levels: still a few lines per instruction instead of 64.
// TL = false (no re-laid views in this call, e.g. a horizontal array): the
// row-major addressing folds to yp W + xp at compile time -- the general
// form's extra multiply-add per tap cost C2 (5x1 array) 173 -> 224 us.
// HZ (every neighbour of the launch's references in the same camera row, every
// level x column offset an integer below 2^24, no re-laid views): the shift
// is an integer, so (int)((float)xr - d dx) = xr - (int)(d dx) exactly, the
// tap's row yr = (int)(r.y - 0) is the reference tap's own (inside the image
// whenever the reference tap is) and its offset yr W is stored with the tap.
// A tap then costs one integer subtract, one compare and one shift-add before
// its gather, and the gather needs no select: the view's buffer resource
// bounds every offset (a tap outside the image reads some pixel of the view,
// or 0, and is dropped as before).  The absolute differences and the
// reference's val += 30; val -= 30; val += AD are single-issue asm, as the
// compiler's SLP pairing put them in v_pk_add_f32 with the |.| as separate
// v_and_b32.  C2: see DESIGN.md section 3.
typedef unsigned u32x3 __attribute__((ext_vector_type(3)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float tap_ad(const float4& A, const u32x3& bv) {
  float t0, t1, t2, r;
  asm("v_sub_f32 %0, %1, %2" : "=v"(t0) : "v"(A.x), "v"(__uint_as_float(bv.x)));
  asm("v_sub_f32 %0, %1, %2" : "=v"(t1) : "v"(A.y), "v"(__uint_as_float(bv.y)));
  asm("v_add_f32 %0, |%1|, |%2|" : "=v"(r) : "v"(t0), "v"(t1));  // fabsf(dL) + fabsf(da)
  asm("v_sub_f32 %0, %1, %2" : "=v"(t2) : "v"(A.z), "v"(__uint_as_float(bv.z)));
  asm("v_add_f32 %0, %1, |%2|" : "=v"(r) : "v"(r), "v"(t2));  // + fabsf(db)
  return r;
}
// val = in ? ((val + 30) - 30) + ad : val + 30
__device__ __forceinline__ float tap_acc(float val, float ad, bool in) {
  float v30, t;
  asm("v_add_f32 %0, 0x41f00000, %1" : "=v"(v30) : "v"(val));
  asm("v_add_f32 %0, 0xc1f00000, %1" : "=v"(t) : "v"(v30));
  asm("v_add_f32 %0, %1, %2" : "=v"(t) : "v"(t), "v"(ad));
  return in ? t : v30;
}
template <int LPS, bool TL, bool HZ = false>
__global__ __launch_bounds__(256) void k_sweep_spixl(const float4* __restrict__ lab, float* __restrict__ spixl,
                                                     const uint8_t* __restrict__ rep,
                                                     const float* __restrict__ levels, const int* __restrict__ vs,
                                                     const int* __restrict__ sn, SweepArgs a, int wps,
                                                     const float4* __restrict__ labT,
                                                     const int* __restrict__ tslot, long tstride) {
  __shared__ float4 refc[8][25];
  __shared__ float2 refxy[8][25];  // (float)xr, (float)yr; xr = -1e9 for a tap outside the image
                                   // (HZ: int xr (-2^30 outside), int yr W)
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
    bool in = xr >= 0 && yr >= 0 && xr < a.W && yr < a.H;
    // (float)xr is exact; an outside reference tap projects outside too
    if (HZ)
      refxy[slot][ll] = make_float2(__int_as_float(in ? xr : -(1 << 30)), __int_as_float(in ? yr * a.W : 0));
    else
      refxy[slot][ll] = make_float2(in ? (float)xr : -1.0e9f, (float)yr);
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
      const int ddx = vx - rx, ddy = vy - ry;
      if (HZ) {
        const int sh = (int)fdx;  // exact (the launcher checked the levels)
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(lab + (long)view * P), 0, (int)(P * 16), 0x00020000);
        float val = 0.0f;
#pragma unroll 5
        for (int t = 0; t < 25; t++) {
          const float2 rf = refxy[slot][t];
          const int xp = __float_as_int(rf.x) - sh;
          const bool in = (unsigned)xp < (unsigned)a.W;
          const unsigned bo = (unsigned)(__float_as_int(rf.y) + xp) << 4;
          const u32x3 bv = __builtin_amdgcn_raw_buffer_load_b96(rs, (int)bo, 0, 0);
          val = tap_acc(val, tap_ad(refc[slot][t], bv), in);
        }
        if (val < mn) mn = val;
        continue;
      }
      const int kind = !TL ? 0 : ddx == 0 ? 1 : ddx == ddy ? 2 : ddx == -ddy ? 3 : 0;
      const int ts = TL && kind ? tslot[4 * view + kind] : -1;
      const float4* labv = TL && ts >= 0 ? labT + (long)ts * tstride : lab + (long)view * P;
      // 32-bit byte offsets into the view's layout (the launcher checks the
      // size): one address add per tap instead of 64-bit index arithmetic
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)labv, 0, 0x7fffffff, 0x00020000);
      // element index = off + x sxs + y sys in the view's layout
      const int sxs = !TL || ts < 0 ? 1 : a.H;
      const int sys = !TL || ts < 0 ? a.W : kind == 1 ? 1 : kind == 2 ? 1 - a.H : a.H + 1;
      const int off = TL && ts >= 0 && kind == 2 ? (a.H - 1) * a.H : 0;
      float val = 0.0f;
      // branch-free taps: every load is issued (out-of-image taps read pixel 0
      // and are dropped by the select), so the 25 gathers of a neighbour are
      // independent and in flight together instead of one per branch
#pragma unroll 5
      for (int t = 0; t < 25; t++) {
        const float2 r = refxy[slot][t];
        const int xp = (int)(r.x - fdx);
        const int yp = (int)(r.y - fdy);
        const bool in = (unsigned)xp < (unsigned)a.W && (unsigned)yp < (unsigned)a.H;
        const int bo = in ? (off + yp * sys + xp * sxs) * 16 : 0;  // an outside tap reads pixel 0, dropped below
        const u32x3 bv = __builtin_amdgcn_raw_buffer_load_b96(rs, bo, 0, 0);
        const float3 B = make_float3(__uint_as_float(bv.x), __uint_as_float(bv.y), __uint_as_float(bv.z));
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

// ---- the HZ sweep from LDS-staged rows (k_sweep_spixl_ring) ---------------
// The HZ gather form is texture-address-bound, not VALU-bound (C2, PMC: TA
// busy 74 % of the kernel, ~15 L2 requests per 64-lane gather: the 64 levels
// of one tap hit 64 pixels dx apart, a partial line each, and the 5 taps of a
// row re-read the same pixels at other levels).  Here a wave (64 levels of
// one superpixel) stages, per neighbour and tap row, the union of the columns
// its 5 taps reach at its 64 levels -- [min xr - max sh, max xr - min sh],
// clamped to the image, at most kSwU columns -- into LDS by whole-line
// LDS-DMA (one 1 KiB piece per 64 columns), and reads every tap from there.
// Rows go through a two-slot ring per wave: row k+2 is staged while row k+1
// lands and row k is computed (s_waitcnt vmcnt(pieces of row k+1) before
// row k); no barrier, the ring is the wave's own.  A tap's absolute
// differences are k_sweep_spixl's; its out-of-image flag rides as ad = -1
// (ad >= 0 otherwise), and the reference's val += 30; val -= 30; val += AD
// chain runs in tap order (i outer, j inner) once the neighbour's 25 taps
// are in.  The launcher takes this form only when every window fits kSwU
// columns: 2 (S - 1) + 2 + |dx| x the levels' range over any 64 consecutive
// levels (stx <= (S - 1) / 2), else the HZ gathers.
constexpr int kSwU = 336;  // C5 (S = 40, |dx| <= 4): 78 + 2 + 252 = 332
__device__ __forceinline__ void wait_vm(int n) {  // s_waitcnt vmcnt(n), n in [0, 6]
  switch (n) {
    case 0: __builtin_amdgcn_s_waitcnt(0x0f70); break;
    case 1: __builtin_amdgcn_s_waitcnt(0x0f71); break;
    case 2: __builtin_amdgcn_s_waitcnt(0x0f72); break;
    case 3: __builtin_amdgcn_s_waitcnt(0x0f73); break;
    case 4: __builtin_amdgcn_s_waitcnt(0x0f74); break;
    case 5: __builtin_amdgcn_s_waitcnt(0x0f75); break;
    default: __builtin_amdgcn_s_waitcnt(0x0f76); break;
  }
}
__device__ __forceinline__ float wave_min_f(float v) {
  v = fminf(v, __shfl_xor(v, 32));
  v = fminf(v, __shfl_xor(v, 16));
  v = fminf(v, __shfl_xor(v, 8));
  v = fminf(v, __shfl_xor(v, 4));
  v = fminf(v, __shfl_xor(v, 2));
  v = fminf(v, __shfl_xor(v, 1));
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
template <int WPS>
__global__ __launch_bounds__(256) void k_sweep_spixl_ring(const float4* __restrict__ lab, float* __restrict__ spixl,
                                                          const uint8_t* __restrict__ rep,
                                                          const float* __restrict__ levels, const int* __restrict__ vs,
                                                          const int* __restrict__ sn, SweepArgs a) {
  constexpr int SPB = 4 / WPS;
  __shared__ __align__(16) float4 ring[4][2][kSwU];  // per wave: two row slots
  __shared__ float4 refc[SPB][25];
  __shared__ int rxr[SPB][5], ryr[SPB][5];           // tap columns (i) and rows (j), possibly outside
  __shared__ unsigned rvm[SPB];                       // bit 5 i + j: tap (i, j) inside the image
  __shared__ float wbest[4];
  __shared__ int wbi[4];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = w % WPS, slot = w / WPS;
  const int z = a.z + blockIdx.y;
  const long M = (long)a.mw * a.mh, P = (long)a.W * a.H;
  const long nbk = (M + SPB - 1) / SPB, per = (nbk + 7) / 8;  // XCD-aware order, as k_sweep_spixl
  const long blk = (long)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  const long s = blk * SPB + slot;
  const bool active = blk < nbk && s < M;
  const long idx = z * M + (active ? s : 0);
  if (h == 0) {
    const uint8_t* dr = rep + 8 * idx;
    const int bl_ = max((int)dr[0], max((int)dr[1], (int)dr[2]));
    const int br_ = max((int)dr[5], max((int)dr[6], (int)dr[7]));
    const int bt_ = max((int)dr[0], max((int)dr[3], (int)dr[5]));
    const int bb_ = max((int)dr[2], max((int)dr[4], (int)dr[7]));
    const float stx = (float)fmax(1.0, 0.25 * (double)(float)(bl_ + br_));
    const float sty = (float)fmax(1.0, 0.25 * (double)(float)(bt_ + bb_));
    const float cx = spixl[8 * idx + 1], cy = spixl[8 * idx + 2];
    const int i = lane / 5 - 2, j = lane % 5 - 2;  // tap t = lane: i (x) outer, j (y) inner
    const int xr = (int)(cx + (float)i * stx);
    const int yr = (int)(cy + (float)j * sty);
    const bool in = lane < 25 && xr >= 0 && yr >= 0 && xr < a.W && yr < a.H;
    if (lane < 25) {
      // .w: the tap's column, or -2^30 for a tap outside the image (its projection is outside too)
      float4 rc = in ? lab[(long)z * P + (long)yr * a.W + xr] : make_float4(0.f, 0.f, 0.f, 0.f);
      rc.w = __int_as_float(in ? xr : -(1 << 30));
      refc[slot][lane] = rc;
      if (j == -2) rxr[slot][i + 2] = xr;
      if (i == -2) ryr[slot][j + 2] = yr;
    }
    const unsigned long long bal = __ballot(in);
    if (lane == 0) rvm[slot] = (unsigned)bal;
  }
  __syncthreads();
  const unsigned vm = __builtin_amdgcn_readfirstlane(rvm[slot]);
  int xr[5], yr[5];
#pragma unroll
  for (int q = 0; q < 5; q++) {
    xr[q] = rxr[slot][q];
    yr[q] = ryr[slot][q];
  }
  // the union of the inside taps' columns (any row), and the rows holding one
  int xlo = 1 << 30, xhi = -(1 << 30);
#pragma unroll
  for (int q = 0; q < 5; q++)
    if ((vm >> (5 * q)) & 0x1fu) {
      xlo = min(xlo, xr[q]);
      xhi = max(xhi, xr[q]);
    }
  const int rx = z % a.aw;  // (every neighbour in the reference's camera row)
  // the taps' columns (-2^30 outside), uniform, and the LDS byte addresses of
  // this wave's ring and this superpixel's reference colours
  int rcol[25];
#pragma unroll
  for (int t = 0; t < 25; t++) rcol[t] = __float_as_int(refc[slot][t].w);  // (VGPRs: the LDS caps the waves, not these)
  const unsigned ring_base = (unsigned)(uintptr_t)(lds_vptr_t)&ring[w][0][0];
  const unsigned refc_base = (unsigned)(uintptr_t)(lds_vptr_t)&refc[slot][0];
  const int nn = sn[z];
  float best = 1000000.0f;
  int bi = 0x7fffffff;
  for (int p0 = 64 * h; p0 < a.D; p0 += 64 * WPS) {
    const int dl = p0 + lane;
    const bool act = dl < a.D;
    const float d = levels[act ? dl : a.D - 1];
    // the pass's level range: (int)(d dx) is monotone in d, so a neighbour's
    // shift range comes from its ends
    const float dlo = wave_min_f(d), dhi = -wave_min_f(-d);
    // the staging window of neighbour n: columns [ulo, ulo + U) of its view
    auto window = [&](int n, int& ulo, int& U, int& sh) {
      const int view = vs[a.V * z + n];
      const float fdx = (float)(view % a.aw - rx);
      sh = (int)(d * fdx);  // exact (the launcher checked the levels)
      const int s0 = (int)(dlo * fdx), s1 = (int)(dhi * fdx);
      const int shmin = min(s0, s1), shmax = max(s0, s1);
      ulo = max(xlo - shmax, 0);
      U = min(xhi - shmin, a.W - 1) - ulo + 1;
    };
    // stage row k = 5 n + j into slot k & 1; returns its LDS-DMA pieces (0:
    // nothing staged -- no inside tap on the row, an empty or too wide window)
    auto stage = [&](int n, int j, int k, int ulo, int U) -> int {
      if (U <= 0 || !((vm >> j) & 0x108421u)) return 0;
      U = min(U, kSwU);  // (the launcher's bound makes this a no-op; never past the slot)
      const int view = vs[a.V * z + n];
      const float4* row = lab + (long)view * P + (long)yr[j] * a.W + ulo;
      const int np = (U + 63) >> 6;
      for (int q = 0; q < np; q++) {
        const int c0 = U >= 64 ? min(q * 64, U - 64) : 0;  // the last piece ends at U (U < 64: lanes past U re-read column U - 1)
        glds16(row + min(c0 + lane, U - 1), &ring[w][k & 1][c0]);
      }
      return np;
    };
    float mn = 1000000.0f;
    if (nn > 0) {
      int ulo0, U0, sh0;
      window(0, ulo0, U0, sh0);
      int pcn = stage(0, 0, 0, ulo0, U0);  // pieces of the row after the one computed next
      pcn = stage(0, 1, 1, ulo0, U0);
      int ulo_c = ulo0, sh_c = sh0;  // the neighbour being computed
      int ulo_s = ulo0, U_s = U0;              // the neighbour being staged (rows k + 2)
      for (int n = 0; n < nn; n++) {
        float ad[25];
#pragma unroll
        for (int j = 0; j < 5; j++) {
          const int k = 5 * n + j;
          wait_vm(k + 1 < 5 * nn ? pcn : 0);  // row k landed (row k + 1 may still be in flight)
          // the row's 5 taps: their columns (refc .w), then the 5 ring reads
          // and the 5 reference colours in one asm block closed by
          // lgkmcnt(0) -- the compiler would put vmcnt(0) (every LDS-DMA in
          // flight, row k + 1's included) before plain LDS reads here
          int xp[5];
          unsigned ra[5];
#pragma unroll
          for (int i = 0; i < 5; i++) {
            xp[i] = rcol[i * 5 + j] - sh_c;
            const bool in = (unsigned)xp[i] < (unsigned)a.W;
            ra[i] = ring_base + (unsigned)(k & 1) * (kSwU * 16u) + (in ? (unsigned)(xp[i] - ulo_c) * 16u : 0u);
          }
          const unsigned rb = refc_base + (unsigned)j * 16u;
          u32x3 Bv[5];
          f32x4 Av[5];
          asm volatile(
              "ds_read_b96 %0, %10\n\t"
              "ds_read_b96 %1, %11\n\t"
              "ds_read_b96 %2, %12\n\t"
              "ds_read_b96 %3, %13\n\t"
              "ds_read_b96 %4, %14\n\t"
              "ds_read_b128 %5, %15\n\t"
              "ds_read_b128 %6, %15 offset:80\n\t"
              "ds_read_b128 %7, %15 offset:160\n\t"
              "ds_read_b128 %8, %15 offset:240\n\t"
              "ds_read_b128 %9, %15 offset:320\n\t"
              "s_waitcnt lgkmcnt(0)"
              : "=&v"(Bv[0]), "=&v"(Bv[1]), "=&v"(Bv[2]), "=&v"(Bv[3]), "=&v"(Bv[4]), "=&v"(Av[0]), "=&v"(Av[1]),
                "=&v"(Av[2]), "=&v"(Av[3]), "=&v"(Av[4])
              : "v"(ra[0]), "v"(ra[1]), "v"(ra[2]), "v"(ra[3]), "v"(ra[4]), "v"(rb)
              : "memory");
#pragma unroll
          for (int i = 0; i < 5; i++) {
            const bool in = (unsigned)xp[i] < (unsigned)a.W;
            const float v = tap_ad(make_float4(Av[i].x, Av[i].y, Av[i].z, 0.f), Bv[i]);
            ad[5 * i + j] = in ? v : -1.0f;
          }
          // stage row k + 2 (the next neighbour's rows 0 and 1 from j = 3 on)
          const int k2 = k + 2;
          int pc2 = 0;
          if (k2 < 5 * nn) {
            const int n2 = k2 / 5, j2 = k2 - 5 * n2;
            if (j2 == 0) {
              int sh2;
              window(n2, ulo_s, U_s, sh2);
            }
            pc2 = stage(n2, j2, k2, ulo_s, U_s);
          }
          pcn = pc2;
        }
        float val = 0.0f;
#pragma unroll
        for (int t = 0; t < 25; t++) val = tap_acc(val, ad[t], ad[t] >= 0.0f);
        mn = val < mn ? val : mn;
        if (n + 1 < nn) {  // the next neighbour's window (staged from j = 3 of this one)
          ulo_c = ulo_s;
          const int view = vs[a.V * z + n + 1];
          sh_c = (int)(d * (float)(view % a.aw - rx));
        }
      }
    }
    if (act && mn < best) {
      best = mn;
      bi = dl;
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob < best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  if (lane == 0) {
    wbest[w] = best;
    wbi[w] = bi;
  }
  __syncthreads();
  if (active && h == 0 && lane == 0) {
    for (int k = 1; k < WPS; k++) {
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

// ---- per-pixel SAD sweep on LDS bands (S=1 grid semantics) -----------------
// Tile: 60 output columns x TH rows; its 64 x (TH+4) tap region (2-pixel
// halo) has one region column per lane.  Steps t = (chunk c of DC = 8*PPW
// levels, neighbour n): the neighbour's Lab rows and columns reachable from
// the region at any level of the chunk are staged in LDS once per step and
// serve every level of the chunk.  The next step's band is loaded into
// registers at the start of a step and written to the other LDS buffer after
// the step's compute, so its latency hides behind the compute.  Wave w takes
// the chunk's level pairs w*PPW .. w*PPW+PPW-1; per pair:
//   A. each lane forms its region column's taps a = |dL|+|da|+|db| of both
//      levels from its reference colours (registers) and the band, or 30 for
//      a tap outside the image (ref or projection), into a wave-private LDS
//      plane of float2 {level 2p, level 2p+1};
//   B. each lane sums its output pixel's 25 taps, x offset outer and y offset
//      inner as the reference does, val = ((val + 30) - 30) + a, as three
//      v_pk_add_f32 over the pair.  (An out-of-image tap with a = 30 gives
//      RN(RN(RN(val+30) - 30) + 30) = RN(val+30): RN(val+30) - 30 is exact for
//      val >= 0, so this is the reference's lone val += 30, bit for bit.)
// The per-level minimum over neighbours folds into a first-minimum WTA in
// level order; the 4 waves' (cost, level) winners are merged
// lexicographically at the end.
constexpr int SB_TW = 60;   // output columns per tile
constexpr int SB_NBLK = 2;  // 64-column blocks per band row (band columns <= 128)
constexpr float SB_INIT = 1000000.0f;
// row-table entry of a row outside the image: a valid entry (yp-by0)*bw - bx0
// is negative on the band's first row whenever bx0 > 0, so no -1 sentinel
constexpr int SB_NOROW = -0x40000000;

struct SadArgs {
  int W, H, D, nn, z;
  int tiles_x, ntiles, tiles_per_xcd, nch;
  int bw, brows;  // LDS band pitch (pixels) and rows per buffer
};
// host-built plan, one record per step (c, n), read by scalar loads
struct alignas(16) SadRec {
  int view, sxmin, sxmax, pad0;
  float fdymin, fdymax;
  int pad1[2];
  int sx[16];     // per level j of the chunk: column shift d*dx (integral)
  float fdy[16];  // per level j: (bl*d)*dy, the reference's float row shift
};

// the band of step record e for the tile at (x0, y0): every neighbour pixel a
// valid tap of the region can project to at any level of the chunk
struct SadBand {
  int bx0, by0, nrows, ncols;
};
template <int TH>
__device__ __forceinline__ SadBand sad_band_of(const SadRec& e, int x0, int y0, int W, int H) {
  SadBand g;
  g.bx0 = min(max(x0 - 2 - e.sxmax, 0), W - 1);
  const int bx1 = min(max(x0 + SB_TW + 1 - e.sxmin, 0), W - 1);
  g.by0 = min(max((int)((float)(y0 - 2) - e.fdymax), 0), H - 1);
  const int by1 = min(max((int)((float)(y0 + TH + 1) - e.fdymin), 0), H - 1);
  g.nrows = by1 - g.by0 + 1;
  g.ncols = bx1 - g.bx0 + 1;
  return g;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));


// The 25-tap sums run as a systolic chain across lanes (round 2's two-phase
// form staged the AD plane in LDS per wave and re-read it per tap: 3.35 ms
// per C2 view against 2.42; it was removed in round 3 with the other A/B
// variants).  An output's 25-tap chain takes its 5 window columns in order (x offset outer),
// and window column i of output x is region column x-2+i = lane (x-x0)+i.  So
// every lane runs the 5-row inner chains of its OWN column's taps (kept in
// registers) on the partial sums it receives from the lane to its left
// (DPP wave_shr:1, folded into the first add of each column): after the 5th
// column, lane l holds the output of image column x0 + l - 4.  The AD plane,
// its LDS writes/reads and the wave barriers of the two-phase form disappear.
// AFF: every level's row shift is integral, so region row r of
// level j reads band row r + (y0 - 2 - fdy_j - by0) exactly and is valid on
// one interval of r: the rows are addressed by immediate offsets r * BWT from
// one per-level lane address, and validity is a scalar interval test -- no
// row table reads, no per-row address arithmetic or compares.  BWT = the band
// pitch (a.bw) as a compile-time constant (0: runtime, the table path).
template <int TH, int PPW, bool AFF = false, int BWT = 0>
__global__ __launch_bounds__(256) void k_sad_band(const float4* __restrict__ lab, const float* __restrict__ levels,
                                                  const SadRec* __restrict__ plan, SadArgs a,
                                                  float* __restrict__ disp) {
  constexpr int RR = TH + 4, DC = 8 * PPW;
  extern __shared__ __align__(16) uint8_t smem[];
  float4* band = (float4*)smem;                // [2][brows][bw]
  int* rtab = (int*)(band + 2 * a.brows * a.bw);  // [2][DC][RR] (the row-table form)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware tile map (as k_ncc_volume): each XCD a contiguous strip of tiles
  const int bid = blockIdx.x, grp = bid & 7;
  const int tile = grp * a.tiles_per_xcd + (bid >> 3);
  if (tile >= a.ntiles) return;
  const int W = a.W, H = a.H;
  const int x0 = (tile % a.tiles_x) * SB_TW, y0 = (tile / a.tiles_x) * TH;
  const long P = (long)W * H;
  const int gx = x0 - 2 + lane;  // this lane's region column
  const bool gxok = gx >= 0 && gx < W;
  float rL[RR], ra[RR], rb[RR];
  {
    const float4* labz = lab + (long)a.z * P;
#pragma unroll
    for (int r = 0; r < RR; r++) {
      const int gy = y0 - 2 + r;
      const bool in = gxok && gy >= 0 && gy < H;
      const float4 c = labz[in ? (long)gy * W + gx : 0];
      rL[r] = c.x;
      ra[r] = c.y;
      rb[r] = c.z;
    }
  }
  const int T = a.nch * a.nn;

  SadBand pg{0, 0, 0, 0};
  // step t's band into LDS buffer b by 16-byte LDS-DMA (lane l's pixel lands
  // at 16 l past the wave-uniform row address), wave w taking rows w, w+4, ...
  // No registers hold the band: the register-staged prefetch this replaces
  // (12 float4 per lane) spilled to scratch, and the spill store waited for
  // the prefetch loads before the step could compute.  Columns past the band
  // (pitch a.bw is a multiple of 64) get a clamped copy nothing reads.
  auto stage = [&](int t, int b) {
    const SadRec& e = plan[t];
    pg = sad_band_of<TH>(e, x0, y0, W, H);
    const float4* src = lab + (long)e.view * P + (long)pg.by0 * W + pg.bx0;
    float4* dst = band + b * a.brows * a.bw;
    const int nblk = (pg.ncols + 63) >> 6;
    for (int cb = 0; cb < nblk; cb++) {
      const int col = min(cb * 64 + lane, pg.ncols - 1);
      for (int i = wave; i < pg.nrows; i += 4)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + (long)i * W + col),
                                         (__attribute__((address_space(3))) void*)(dst + i * a.bw + cb * 64), 16, 0, 0);
    }
  };
  // step t's row table into buffer b: per (level j, region row r) the band
  // index of row yp minus bx0 (so + xp gives the pixel), or SB_NOROW when the
  // reference row or the projected row leaves the image
  auto commit = [&](int t, int b) {
    const SadRec& e = plan[t];
    int* tb = rtab + b * DC * RR;
    const int c = t / a.nn;
    for (int k = tid; k < DC * RR; k += 256) {
      const int j = k / RR, r = k - j * RR;
      const int gy = y0 - 2 + r;
      int v = SB_NOROW;
      if (c * DC + j < a.D) {
        const int yp = (int)((float)gy - e.fdy[j]);
        if (gy >= 0 && gy < H && yp >= 0 && yp < H) v = (yp - pg.by0) * a.bw - pg.bx0;
      }
      tb[k] = v;
    }
  };

  float best[TH];
  int bidx[TH];
#pragma unroll
  for (int o = 0; o < TH; o++) {
    best[o] = SB_INIT;
    bidx[o] = -1;
  }
  f32x2 mn[PPW][TH];
  if (T > 0) {
    stage(0, 0);
    if (!AFF) commit(0, 0);
  }
  __syncthreads();
  // chunks outer, neighbours inner (step t = c * nn + n): the chunk's reset
  // and WTA fold sit outside the per-step body.  As one flat step loop the
  // compiler if-converted them into every step (exec-masked compares and
  // selects issued nn times per chunk)
  int t = 0;
  for (int c = 0; c < (a.nn > 0 ? a.nch : 0); c++) {
#pragma unroll
  for (int q = 0; q < PPW; q++)
#pragma unroll
    for (int o = 0; o < TH; o++) mn[q][o] = f32x2{SB_INIT, SB_INIT};
  for (int n = 0; n < a.nn; n++, t++) {
    // step t+1's band lands in the other buffer (last read in step t-1, before
    // the previous barrier) while this step computes
    if (t + 1 < T) stage(t + 1, (t + 1) & 1);
    const SadRec& e = plan[t];
    const float4* bnd = band + (t & 1) * a.brows * a.bw;
    const int* tb = rtab + (t & 1) * DC * RR;
#pragma unroll
    for (int q = 0; q < PPW; q++) {
      const int j0 = (wave * PPW + q) * 2;
      const int xp0 = gx - e.sx[j0], xp1 = gx - e.sx[j0 + 1];
      const bool xok0 = gxok && xp0 >= 0 && xp0 < W, xok1 = gxok && xp1 >= 0 && xp1 < W;
      const f32x2 k30 = f32x2{30.0f, 30.0f};
      // A. taps of the lane's region column, both levels
      f32x2 ad[RR];
      if constexpr (AFF) {
        const SadBand g = sad_band_of<TH>(e, x0, y0, W, H);  // this step's band (pg is step t+1's)
        const int off0 = (int)e.fdy[j0], off1 = (int)e.fdy[j0 + 1];
        const int rlo0 = max(max(0, 2 - y0), 2 - y0 + off0), rhi0 = min(min(RR - 1, H + 1 - y0), H + 1 - y0 + off0);
        const int rlo1 = max(max(0, 2 - y0), 2 - y0 + off1), rhi1 = min(min(RR - 1, H + 1 - y0), H + 1 - y0 + off1);
        const int b0 = xok0 ? (y0 - 2 - off0 - g.by0) * BWT + xp0 - g.bx0 : 0;
        const int b1 = xok1 ? (y0 - 2 - off1 - g.by0) * BWT + xp1 - g.bx0 : 0;
#pragma unroll
        for (int r = 0; r < RR; r++) {
          const bool v0 = xok0 && r >= rlo0 && r <= rhi0, v1 = xok1 && r >= rlo1 && r <= rhi1;
          const float4 n0 = bnd[b0 + r * BWT], n1 = bnd[b1 + r * BWT];
          asm volatile("" ::"v"(n0.w), "v"(n1.w));  // keep the full 16-B ds_read_b128
          float d0 = fabsf(rL[r] - n0.x) + fabsf(ra[r] - n0.y);
          d0 = d0 + fabsf(rb[r] - n0.z);
          float d1 = fabsf(rL[r] - n1.x) + fabsf(ra[r] - n1.y);
          d1 = d1 + fabsf(rb[r] - n1.z);
          ad[r] = f32x2{v0 ? d0 : 30.0f, v1 ? d1 : 30.0f};
        }
      } else {
#pragma unroll
      for (int r = 0; r < RR; r++) {
        const int t0 = tb[j0 * RR + r], t1 = tb[(j0 + 1) * RR + r];
        const bool v0 = xok0 && t0 != SB_NOROW, v1 = xok1 && t1 != SB_NOROW;
        const float4 n0 = bnd[v0 ? t0 + xp0 : 0], n1 = bnd[v1 ? t1 + xp1 : 0];
        asm volatile("" ::"v"(n0.w), "v"(n1.w));  // keep the full 16-B ds_read_b128 (b96 is 3x slower)
        float d0 = fabsf(rL[r] - n0.x) + fabsf(ra[r] - n0.y);
        d0 = d0 + fabsf(rb[r] - n0.z);
        float d1 = fabsf(rL[r] - n1.x) + fabsf(ra[r] - n1.y);
        d1 = d1 + fabsf(rb[r] - n1.z);
        ad[r] = f32x2{v0 ? d0 : 30.0f, v1 ? d1 : 30.0f};
      }
      }
      // B'. systolic: column 0 starts the chains (first tap: ((0+30)-30)+a = a
      // exactly), columns 1..4 continue the left neighbour's partials
      f32x2 p[TH];
      float c30;  // 30.0f in a VGPR: the DPP add's second source
      asm volatile("v_mov_b32 %0, 0x41f00000" : "=v"(c30));
#pragma unroll
      for (int o = 0; o < TH; o++) {
        p[o] = ad[o];
#pragma unroll
        for (int jj = 1; jj < 5; jj++) p[o] = ((p[o] + k30) - k30) + ad[o + jj];
      }
#pragma unroll
      for (int i = 1; i < 5; i++) {
        // the shift folded into the first add of the column: v_add_f32 with a
        // DPP wave_shr:1 source (lane 0 reads 0 by bound_ctrl: 0 + 30), four
        // rows per asm block.  The block's leading s_nop 1 gives the two wait
        // states a DPP read of a VALU result needs (the compiler does not see
        // inside inline asm); the pk ops below still pair the results.
        float sx[TH], sy[TH];
#pragma unroll
        for (int o = 0; o < TH; o += 4)
          asm volatile(
              "s_nop 1\n\t"
              "v_add_f32_dpp %0, %8, %16 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
              "v_add_f32_dpp %1, %9, %16 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
              "v_add_f32_dpp %2, %10, %16 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
              "v_add_f32_dpp %3, %11, %16 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
              "v_add_f32_dpp %4, %12, %16 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
              "v_add_f32_dpp %5, %13, %16 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
              "v_add_f32_dpp %6, %14, %16 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
              "v_add_f32_dpp %7, %15, %16 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
              : "=&v"(sx[o]), "=&v"(sy[o]), "=&v"(sx[o + 1]), "=&v"(sy[o + 1]), "=&v"(sx[o + 2]), "=&v"(sy[o + 2]),
                "=&v"(sx[o + 3]), "=&v"(sy[o + 3])
              : "v"(p[o].x), "v"(p[o].y), "v"(p[o + 1].x), "v"(p[o + 1].y), "v"(p[o + 2].x), "v"(p[o + 2].y),
                "v"(p[o + 3].x), "v"(p[o + 3].y), "v"(c30));
#pragma unroll
        for (int o = 0; o < TH; o++) {
          f32x2 v = f32x2{sx[o], sy[o]};
          v = (v - k30) + ad[o];
#pragma unroll
          for (int jj = 1; jj < 5; jj++) v = ((v + k30) - k30) + ad[o + jj];
          p[o] = v;
        }
      }
      // v_min_f32 as asm: fminf made the compiler canonicalise the
      // loop-carried minima (a v_max_f32 x, x each) every step; no NaN here
#pragma unroll
      for (int o = 0; o < TH; o++) {
        asm("v_min_f32 %0, %1, %2" : "=v"(mn[q][o].x) : "v"(mn[q][o].x), "v"(p[o].x));
        asm("v_min_f32 %0, %1, %2" : "=v"(mn[q][o].y) : "v"(mn[q][o].y), "v"(p[o].y));
      }
    }
    // step t+1's row table (its rows were last read in step t-1); the barrier
    // (vmcnt(0) first) publishes the table and the landed band
    if (t + 1 < T && !AFF) commit(t + 1, (t + 1) & 1);
    __syncthreads();
  }
  // chunk complete: first-minimum WTA in level order
#pragma unroll
  for (int q = 0; q < PPW; q++) {
    const int dl = c * DC + (wave * PPW + q) * 2;
#pragma unroll
    for (int o = 0; o < TH; o++) {
      if (dl < a.D && mn[q][o].x < best[o]) {
        best[o] = mn[q][o].x;
        bidx[o] = dl;
      }
      if (dl + 1 < a.D && mn[q][o].y < best[o]) {
        best[o] = mn[q][o].y;
        bidx[o] = dl + 1;
      }
    }
  }
  }
  // merge the 4 waves' winners: lexicographic (cost, level)
  float* mb = (float*)smem;
  int* mi = (int*)(mb + 4 * TH * 64);
#pragma unroll
  for (int o = 0; o < TH; o++) {
    mb[(wave * TH + o) * 64 + lane] = best[o];
    mi[(wave * TH + o) * 64 + lane] = bidx[o];
  }
  __syncthreads();
  for (int k = tid; k < TH * 64; k += 256) {
    const int o = k >> 6, l = k & 63;
    const int x = x0 + l - 4, y = y0 + o;  // lane l holds column x0 + l - 4
    if (l < 4 || x >= W || y >= H) continue;
    float bv = mb[k];
    int bi = mi[k];
#pragma unroll
    for (int w = 1; w < 4; w++) {
      const float v = mb[w * TH * 64 + k];
      const int i = mi[w * TH * 64 + k];
      if (i >= 0 && (v < bv || (v == bv && (bi < 0 || i < bi)))) {
        bv = v;
        bi = i;
      }
    }
    disp[(long)y * W + x] = (bi >= 0 && bv < SB_INIT) ? levels[bi] : 0.0f;
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
  hipLaunchKernelGGL(k_boundary, dim3((mw * mh + 3) / 4, V), dim3(256), 0, s, spixl, labels, W, H, S, mw, mh, rep);
  MVS_LAUNCH_CHECK("k_boundary");
  return 0;
}

// lab view `view` re-laid for the superpixel sweep (see k_sweep_spixl): KIND 1
// transposed, 2 / 3 sheared along x - y / x + y; 32 x 32 tiles through LDS,
// written along the output's contiguous direction (columns, or diagonals)
template <int KIND>
__global__ __launch_bounds__(256) void k_relayout_lab(const float4* __restrict__ lab, int W, int H, int view,
                                                      float4* __restrict__ out) {
  __shared__ float4 t[32][33];
  const int x0 = blockIdx.x * 32, y0 = blockIdx.y * 32, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const float4* src = lab + (long)view * W * H;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int y = y0 + ty + 8 * k, x = x0 + tx;
    if (x < W && y < H) t[ty + 8 * k][tx] = src[(long)y * W + x];
  }
  __syncthreads();
  if (KIND == 1) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int x = x0 + ty + 8 * k, y = y0 + tx;
      if (x < W && y < H) out[(long)x * H + y] = t[tx][ty + 8 * k];
    }
    return;
  }
  // the tile's 63 diagonals, 8 per pass; lane tx = the row within the tile
  for (int d0 = 0; d0 < 63; d0 += 8) {
    const int dd = d0 + ty, yl = tx;
    const int xl = KIND == 2 ? yl + dd - 31 : dd - yl;
    const int x = x0 + xl, y = y0 + yl;
    if (dd < 63 && xl >= 0 && xl < 32 && x < W && y < H)
      out[KIND == 2 ? (long)(x - y + H - 1) * H + y : (long)(x + y) * H + y] = t[yl][xl];
  }
}

int launch_sweep_spixl(mvs_ctx* ctx, int V, int W, int H, int S, const float* lab, float* spixl,
                       const uint8_t* rep, const float* levels, int D, const int* vs, const int* sn, int aw,
                       float bl, int z0, int z1) {
  if (z1 <= z0) return 0;
  // k_sweep_spixl's 32-bit byte offsets within a view (a re-laid one spans
  // at most (W + H) H elements)
  if ((long)(W + H) * H * 16 >= (1L << 31)) return arg_fail("superpixel sweep: image too large for 32-bit offsets");
  hipStream_t s = ctx->stream;
  int mw = map_dim(W, S), mh = map_dim(H, S);
  long M = (long)mw * mh;
  int wps = (D + 63) / 64;
  wps = wps >= 3 ? 4 : wps;  // waves per superpixel: 1, 2 or 4
  // MVS_SWEEP_WPS=1|2|4 (read per call): another wave count per superpixel (A/B)
  const char* we = getenv("MVS_SWEEP_WPS");
  const int wps_env = (we && D > 32 && (atoi(we) == 1 || atoi(we) == 2 || atoi(we) == 4)) ? atoi(we) : 0;
  if (wps_env) wps = wps_env;
  const bool half = D <= 32;  // two superpixels per wave
  const int spb = half ? 8 : 4 / wps;
  SweepArgs a{V, W, H, mw, mh, D, aw, z0, bl};
  const long nb = (M + spb - 1) / spb;
  // the vertical and diagonal neighbours of the references, re-laid into the
  // context scratch; MVS_SWEEP_TRANSPOSE (read per call) = 0: row-major
  // gathers only, 1: vertical neighbours only, 2 (default): both (A/B)
  // Slot offsets are in units of H elements (tstride = H): a transposed slot
  // takes W units, a sheared one W + H - 1.  If the scratch cannot be had, the
  // row-major kernel runs instead (same results, slower gathers).
  const float4* labT = nullptr;
  const int* tslot = nullptr;
  const long tstride = H;
  const char* te = getenv("MVS_SWEEP_TRANSPOSE");
  const int tmode = te ? atoi(te) : 2;
  if (tmode > 0) {
    std::vector<int32_t> slot(4 * (size_t)V, -1);
    long units = 0;
    for (int z = z0; z < z1; z++)
      for (int k = 0; k < ctx->h_sn[z]; k++) {
        const int v = ctx->h_vs[(size_t)V * z + k];
        if (v < 0 || v >= V) continue;
        const int dx = v % aw - z % aw, dy = v / aw - z / aw;
        const int kind = dx == 0 ? 1 : tmode < 2 ? 0 : dx == dy ? 2 : dx == -dy ? 3 : 0;
        if (kind && slot[4 * v + kind] < 0 && units + W + H <= INT32_MAX) {
          slot[4 * v + kind] = (int32_t)units;
          units += kind == 1 ? W : W + H - 1;
        }
      }
    if (units > 0) {
      int rc = 0;
      float4* buf = (float4*)scratch(ctx, (size_t)units * tstride * sizeof(float4), &rc);
      if (rc == MVS_E_NOMEM) {
        (void)hipGetLastError();  // the failed hipMalloc must not fail the next launch check
        units = 0;
      } else if (rc) {
        return rc;
      }
      if (units > 0) tslot = plan_upload(ctx, slot, &rc);
      if (rc) return rc;
      const dim3 tg((W + 31) / 32, (H + 31) / 32);
      for (int v = 0; v < V && units > 0; v++)
        for (int kind = 1; kind < 4; kind++) {
          const int sl = slot[4 * v + kind];
          if (sl < 0) continue;
          float4* o = buf + (long)sl * tstride;
          if (kind == 1)
            hipLaunchKernelGGL(k_relayout_lab<1>, tg, dim3(256), 0, s, (const float4*)lab, W, H, v, o);
          else if (kind == 2)
            hipLaunchKernelGGL(k_relayout_lab<2>, tg, dim3(256), 0, s, (const float4*)lab, W, H, v, o);
          else
            hipLaunchKernelGGL(k_relayout_lab<3>, tg, dim3(256), 0, s, (const float4*)lab, W, H, v, o);
        }
      MVS_LAUNCH_CHECK("k_relayout_lab");
      if (units > 0) labT = buf;
    }
  }
  // HZ: every neighbour of [z0, z1) in the reference's camera row and every
  // level x column offset an integer of magnitude below 2^24 (MVS_SWEEP_HZ=0,
  // read per call: the general form, A/B)
  bool hz = !labT && (long)W * H * 16 < (1L << 31) && !(getenv("MVS_SWEEP_HZ") && atoi(getenv("MVS_SWEEP_HZ")) == 0);
  for (int z = z0; z < z1 && hz; z++)
    for (int k = 0; k < ctx->h_sn[z] && hz; k++) {
      const int v = ctx->h_vs[(size_t)V * z + k];
      if (v / aw != z / aw) hz = false;
      const float fdxv = (float)(v % aw - z % aw);
      for (int l = 0; l < D && hz; l++) {
        const float f = ctx->h_levels[l] * fdxv;  // the kernel's d * (float)(vx - rx)
        if (!(fabsf(f) < 16777216.0f) || f != truncf(f)) hz = false;
      }
    }
  // HZ with 64 levels per wave: the LDS-staged rows (MVS_SWEEP_RING=0, read per call: the gathers)
  const char* re = getenv("MVS_SWEEP_RING");
  bool ring_ok = hz && !half && !(re && atoi(re) == 0);
  if (ring_ok) {  // every staged window fits kSwU columns (see k_sweep_spixl_ring)
    float rng = 0.0f;
    for (int c0 = 0; c0 < D; c0 += 64) {
      float lo = ctx->h_levels[c0], hi = lo;
      for (int l = c0; l < std::min(D, c0 + 64); l++) {
        lo = std::min(lo, ctx->h_levels[l]);
        hi = std::max(hi, ctx->h_levels[l]);
      }
      rng = std::max(rng, hi - lo);
    }
    int mdx = 0;
    for (int z = z0; z < z1; z++)
      for (int k = 0; k < ctx->h_sn[z]; k++) mdx = std::max(mdx, std::abs(ctx->h_vs[(size_t)V * z + k] % aw - z % aw));
    if (2.0 * (S - 1) + 2.0 + (double)rng * mdx + 1.0 > (double)kSwU) ring_ok = false;
  }
  if (ring_ok) {
    // one wave per superpixel, its 64-level passes in turn: the ring form's
    // cost is per staged row and level, not per wave, and four superpixels per
    // workgroup share its setup and tail (C5, D = 256: 1.19 ms per launch
    // against 1.42 with four waves per superpixel; C2 alike at 1 and 2:
    // profiles/r06/sweep_ring_waves.txt)
    const int rw = wps_env ? wps_env : 1;
    const long nbr = (M + 4 / rw - 1) / (4 / rw);
    const dim3 g((unsigned)(8 * ((nbr + 7) / 8)), (unsigned)(z1 - z0));
    if (rw == 1)
      hipLaunchKernelGGL(k_sweep_spixl_ring<1>, g, dim3(256), 0, s, (const float4*)lab, spixl, rep, levels, vs, sn, a);
    else if (rw == 2)
      hipLaunchKernelGGL(k_sweep_spixl_ring<2>, g, dim3(256), 0, s, (const float4*)lab, spixl, rep, levels, vs, sn, a);
    else
      hipLaunchKernelGGL(k_sweep_spixl_ring<4>, g, dim3(256), 0, s, (const float4*)lab, spixl, rep, levels, vs, sn, a);
    MVS_LAUNCH_CHECK("k_sweep_spixl_ring");
    return 0;
  }
  auto kern = labT ? (half ? k_sweep_spixl<32, true> : k_sweep_spixl<64, true>)
              : hz ? (half ? k_sweep_spixl<32, false, true> : k_sweep_spixl<64, false, true>)
                   : (half ? k_sweep_spixl<32, false> : k_sweep_spixl<64, false>);
  hipLaunchKernelGGL(kern, dim3((unsigned)(8 * ((nb + 7) / 8)), (unsigned)(z1 - z0)), dim3(256), 0, s,
                     (const float4*)lab, spixl, rep, levels, vs, sn, a, wps, labT, tslot, tstride);
  MVS_LAUNCH_CHECK("k_sweep_spixl");
  return 0;
}

namespace {
// Band-staged SAD sweep: host plan + launch for one reference view.  Returns 1
// when the level set has fractional column shifts or the bands do not fit
// the LDS (the caller then uses k_sweep_pixel_sad).
template <int TH, int PPW>
int launch_sad_band_t(mvs_ctx* ctx, int V, int W, int H, const float* lab, const float* levels_host, int D,
                      const int* vs_host, const int* sn_host, int aw, float bl, int z, float* disp) {
  bool aff = getenv("MVS_SAD_AFF") == nullptr;  // MVS_SAD_AFF set: the row-table path (A/B)
  constexpr int RR = TH + 4, DC = 8 * PPW;
  const int nn = sn_host[z];
  const int nch = (D + DC - 1) / DC;
  const int rx = z % aw, ry = z / aw;
  constexpr int RW = sizeof(SadRec) / 4;
  std::vector<int32_t> table((size_t)std::max(1, nch * nn) * RW, 0);
  int span_x = 0;
  float span_y = 0.0f;
  for (int c = 0; c < nch; c++)
    for (int n = 0; n < nn; n++) {
      SadRec e{};
      const int view = vs_host[V * z + n];
      const int dx = view % aw - rx, dy = view / aw - ry;
      e.view = view;
      e.sxmin = 1 << 30;
      e.sxmax = -(1 << 30);
      e.fdymin = INFINITY;
      e.fdymax = -INFINITY;
      for (int j = 0; j < DC; j++) {
        const int dl = std::min(c * DC + j, D - 1);  // past the end: the last level (rows masked)
        const float d = levels_host[dl];
        const float fdx = d * (float)dx;  // the reference's float shifts (clcode.cl:1033-1034)
        const float fdy = (bl * d) * (float)dy;
        if (fdx != std::trunc(fdx) || std::fabs(fdx) > 1e6f) return 1;
        e.sx[j] = (int)fdx;
        e.fdy[j] = fdy;
        if (fdy != std::trunc(fdy) || std::fabs(fdy) > 1e6f) aff = false;
        if (c * DC + j < D) {
          e.sxmin = std::min(e.sxmin, e.sx[j]);
          e.sxmax = std::max(e.sxmax, e.sx[j]);
          e.fdymin = std::min(e.fdymin, fdy);
          e.fdymax = std::max(e.fdymax, fdy);
        }
      }
      span_x = std::max(span_x, e.sxmax - e.sxmin);
      span_y = std::max(span_y, e.fdymax - e.fdymin);
      std::memcpy(table.data() + ((size_t)c * nn + n) * RW, &e, sizeof(SadRec));
    }
  SadArgs a{};
  a.W = W; a.H = H; a.D = D; a.nn = nn; a.z = z; a.nch = nch;
  a.bw = (64 + span_x + 63) & ~63;  // whole 64-pixel LDS-DMA pieces per band row
  // a step's band spans at most RR + ceil(span_y) rows (sad_band_of: the
  // truncated ends differ by < RR + span_y); one spare row for the float
  // rounding of fractional shifts, none when every shift is integral
  a.brows = RR + (int)std::ceil(span_y) + (aff ? 0 : 1);
  const size_t lds = 16 * 2 * (size_t)a.brows * a.bw + (aff ? 0 : 4 * 2 * (size_t)DC * RR);
  // band columns: SB_NBLK pieces of 64 at most (the systolic tile's reach)
  if (a.bw > 64 * SB_NBLK) return 1;
  if (lds > 160 * 1024 || (size_t)4 * TH * 64 * 8 > 16 * 2 * (size_t)a.brows * a.bw) return 1;
  int rc = 0;
  const int32_t* dev = plan_upload(ctx, table, &rc);
  if (rc) return rc;
  a.tiles_x = (W + SB_TW - 1) / SB_TW;
  a.ntiles = a.tiles_x * ((H + TH - 1) / TH);
  a.tiles_per_xcd = (a.ntiles + 7) / 8;
  auto kern = k_sad_band<TH, PPW>;
  if (aff) kern = a.bw == 64 ? k_sad_band<TH, PPW, true, 64> : k_sad_band<TH, PPW, true, 128>;
  MVS_HIP(raise_lds(ctx, (const void*)kern, lds), "hipFuncSetAttribute(sad lds)");
  hipLaunchKernelGGL(kern, dim3(8 * a.tiles_per_xcd), dim3(256), lds, ctx->stream, (const float4*)lab,
                     ctx->d_levels, (const SadRec*)dev, a, disp);
  MVS_LAUNCH_CHECK("k_sad_band");
  return 0;
}

}  // namespace

int launch_sweep_pixel_sad(mvs_ctx* ctx, int V, int W, int H, const float* lab, const float* levels_host, int D,
                           const int* vs_host, const int* sn_host, int aw, float bl, int z0, int z1, float* disp) {
  // MVS_SAD_KERNEL: "sys8x2", "sys8", "gather" (A/B and tests).  Without it:
  // 16-level chunks, else 8-level chunks (taller bands: vertical neighbours),
  // else the gather kernel.  A band variant named explicitly never falls back
  // (MVS_E_UNSUPPORTED), so a test of it cannot pass on another.
  const char* kv = getenv("MVS_SAD_KERNEL");
  const std::string kind = kv ? kv : "auto";
  const bool strict = kv != nullptr && kind != "gather";
  const long P = (long)W * H;
  for (int z = z0; z < z1; z++) {
    float* out = disp + (long)(z - z0) * P;
    int rc = 1;
    if (kind == "auto") {
      rc = launch_sad_band_t<8, 2>(ctx, V, W, H, lab, levels_host, D, vs_host, sn_host, aw, bl, z, out);
      if (rc == 1) rc = launch_sad_band_t<8, 1>(ctx, V, W, H, lab, levels_host, D, vs_host, sn_host, aw, bl, z, out);
    } else if (kind == "sys8")
      rc = launch_sad_band_t<8, 1>(ctx, V, W, H, lab, levels_host, D, vs_host, sn_host, aw, bl, z, out);
    else if (kind == "sys8x2")
      rc = launch_sad_band_t<8, 2>(ctx, V, W, H, lab, levels_host, D, vs_host, sn_host, aw, bl, z, out);
    if (rc < 0) return rc;
    if (rc == 1 && strict) {
      set_error("k_sad_band variant " + kind + " cannot stage this geometry (MVS_SAD_KERNEL set explicitly)");
      return MVS_E_UNSUPPORTED;
    }
    if (rc == 1) {
      SweepArgs a{V, W, H, W, H, D, aw, z, bl};
      hipLaunchKernelGGL(k_sweep_pixel_sad, dim3((W + PT - 1) / PT, (H + PT - 1) / PT), dim3(256), 0, ctx->stream,
                         (const float4*)lab, ctx->d_levels, ctx->d_vs, ctx->d_sn, a, out);
      MVS_LAUNCH_CHECK("k_sweep_pixel_sad");
    }
  }
  return 0;
}

int launch_wta(hipStream_t s, int W, int H, int D, const float* vol, const float* levels, float* disp,
               float* conf) {
  long P = (long)W * H;
  // one pixel per lane, 16 levels in flight (C2: 0.185 -> 0.182 ms against 8; 32 no faster;
  // wider per-lane vectors measured no faster)
  hipLaunchKernelGGL((k_wta<1, 16>), dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, vol, levels, P, D, disp,
                     conf);
  MVS_LAUNCH_CHECK("k_wta");
  return 0;
}

}  // namespace mvs
