// Build-defined per-pixel NCC K x K plane sweep: the cost-volume producer.
//
// Definition (no reference counterpart; restated in oracle/mvs_oracle.c
// orc_ncc_volume): q = 8-bit intensity (clamp(int(L*2.55+0.5))), window K x K,
// shift of neighbour n at level d: (tx, ty) = (roundf(d*dx), roundf((bl*d)*dy)),
// window valid iff every tap of the reference and the shifted window is inside
// the image; with n = K*K and integer sums
//   num = n*Srp - Sr*Sp,  vr = n*Srr - Sr^2,  vp = n*Spp - Sp^2
// ivr = vr ? 1/(float)vr : 0 and ivp likewise (per pixel),
// e_n = (a*|a|)*ivp with a = (float)num for valid windows, m = max_n e_n
// (-inf if none), vol[d][y][x] = 1 - max(-1, m*ivr): 1 minus the best signed
// squared correlation, 2 when no neighbour window is valid.  (ivr after the
// maximum: rounding is monotone, so m*ivr = max_n (e_n*ivr).)  Every sum is
// invariant under centring the intensities (q - 128), which the planes do.
//
// Data layout (mvs_box_stats_d, per view, 16 B/px in two planes):
//   stats [V][H][W] {S', bits(ivr)}: centred window sum S' = S - 128 n (K=5:
//                   as a float, K=7: as an int) and reciprocal variance, with
//                   ivr = NaN where the window leaves the image;
//   pk    [V][H][W] {lo, hi}: the 8 centred intensities q-128 (int8) of
//                   columns x-R .. x-R+7 of row y, packed little-endian.
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
//     ds_read_b64 and two v_dot4_i32_i8 give the exact horizontal K-tap
//     centred correlation, a prefix sum the vertical K-sum, then 6 VALU ops
//     finish the cell (num, IEEE f32 e, v_max_f32);
//   * the chunk's costs are written once, 64-column coalesced rows.
#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "mvs_internal.h"

namespace mvs {
namespace {

// Row-pair interleaved planes: element (y, x) of a view lives at uint2 index
// ((y >> 1) * W + x) * 2 + (y & 1), over Hp = H rounded up to even rows, so
// one 16-byte access returns rows 2m and 2m+1 of one column.
__host__ __device__ __forceinline__ long pair_index(int y, int x, int W) {
  return (((long)(y >> 1) * W + x) << 1) + (y & 1);
}

// ---- window statistics + packed intensities ------------------------------
// one workgroup = 64 columns x 16 rows of one view; the (16+2R) x (64+8)
// byte tile is staged in LDS once.  The dummy row H of an odd-height image
// is written as an invalid window.
constexpr int BS_TW = 64, BS_TH = 16;
template <int R>
__global__ __launch_bounds__(256) void k_box_stats(const uint8_t* __restrict__ q, int W, int H,
                                                   uint2* __restrict__ stats, uint2* __restrict__ pk) {
  constexpr int K = 2 * R + 1, NK = K * K;
  constexpr int TW = BS_TW + 8, TR = BS_TH + 2 * R;  // tile covers columns x0-R .. x0+63-R+7
  __shared__ uint8_t t[TR][TW + 4];
  const int x0 = blockIdx.x * BS_TW, y0 = blockIdx.y * BS_TH, z = blockIdx.z;
  const int Hp = H + (H & 1);
  const long Pv = (long)W * Hp;  // plane elements per view
  const uint8_t* Q = q + z * (long)W * H;
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
    if (y >= Hp) break;
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
    const long o = z * Pv + pair_index(y, x, W);
    // centred window sum S - 128 n: K = 5 as a float (exact) for the FP32
    // finish of the sweeps, K = 7 as an int
    const int sc = (valid ? s : 0) - 128 * NK;
    const unsigned sw = R == 2 ? (unsigned)__float_as_int((float)sc) : (unsigned)sc;
    stats[o] = make_uint2(sw, (unsigned)__float_as_int(iv));
    const uint8_t* row = &t[ly + R][lx];
    unsigned lo = row[0] | (row[1] << 8) | (row[2] << 16) | ((unsigned)row[3] << 24);
    unsigned hi = row[4] | (row[5] << 8) | (row[6] << 16) | ((unsigned)row[7] << 24);
    // q - 128 as int8 is q ^ 0x80
    pk[o] = y < H ? make_uint2(lo ^ 0x80808080u, hi ^ 0x80808080u) : make_uint2(0u, 0u);
  }
}

constexpr int kMaxNbr = 16;
struct NccArgs {
  int W, H, D, nn, z;
  int tiles_x, ntiles, tiles_per_xcd, nch;  // XCD-aware work map (see k_ncc_volume)
  int view[kMaxNbr];
  int pk_pairs, st_pairs;  // LDS band heights in row pairs; the pair-row stride is the template BW
};
// host-built plan (device memory, cached per context): one 128-B record per
// (chunk c, neighbour n, wave w), read with one scalar load per neighbour.
// A __restrict__ kernel parameter, so the loads are SMEM and never wait on
// the vector-memory counter the LDS-DMA prefetch runs under.
struct alignas(128) NccRec {
  int txmax, tymax;  // band origin: image column x0 - txmax; pk pair (y0-R-tymax)>>1, stats pair (y0-tymax)>>1
  int bhp, shp;      // pk pair rows to stage, stats pair rows | (64-px blocks per row) << 16
  int lv[16];        // per level j of wave w: {txmax - tx, pk start row | stats start row << 16 (band-relative)}
  int pad[12];
};

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

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// N consecutive band rows starting at band row r0 of a row-pair band (pair
// row stride BW, one column): ds_read_b128 per pair; an odd start takes the
// first and last rows as ds_read_b64 halves.  N even.
template <int N, int BW, bool EVEN>
__device__ __forceinline__ void read_rows(const u32x4* col, int r0, u32x2 (&v)[N]) {
  const u32x4* p = col + (r0 >> 1) * BW;
  if (EVEN || (r0 & 1) == 0) {
#pragma unroll
    for (int i = 0; i < N / 2; i++) {
      const u32x4 t = p[i * BW];
      v[2 * i] = t.xy;
      v[2 * i + 1] = t.zw;
    }
  } else {
    v[0] = ((const u32x2*)p)[1];
#pragma unroll
    for (int i = 1; i < N / 2; i++) {
      const u32x4 t = p[i * BW];
      v[2 * i - 1] = t.xy;
      v[2 * i] = t.zw;
    }
    v[N - 1] = ((const u32x2*)(p + (N / 2) * BW))[0];
  }
}

// EVEN: every level's band rows start on a pair boundary (all horizontal
// neighbours with even R + tymax): branch-free pair reads.
template <int K, int TH, int DPW, int BW, bool EVEN>
__global__ __launch_bounds__(256) void k_ncc_volume(const uint2* __restrict__ stats, const uint2* __restrict__ pk,
                                                    const NccRec* __restrict__ plan, NccArgs a,
                                                    float* __restrict__ vol) {
  constexpr int R = K / 2;
  constexpr int NR = TH + 2 * R;
  constexpr int NK = K * K;
  constexpr int DC = 4 * DPW;
  static_assert(TH % 2 == 0 && NR % 2 == 0, "row pairs");
  constexpr bool FPF = K == 5;  // FP32 finish (see the reference loads below)
  // taps x-R .. x-R+3 in lo, x-R+4 .. x+R in the low K-4 bytes of hi
  constexpr unsigned HI_MASK = (K - 4) >= 4 ? 0xffffffffu : ((1u << (8 * (K - 4))) - 1u);
  extern __shared__ __align__(16) uint8_t smem[];
  const int nbuf = (a.pk_pairs + a.st_pairs) * BW;  // uint4 per neighbour buffer
  u32x4* nbase = (u32x4*)smem;                      // 2 x {npk[pk_pairs][BW], nst[st_pairs][BW]}

  // wave id made provably uniform: plan loads become scalar (SMEM), so no
  // vector-memory wait drains the in-flight LDS-DMA prefetch
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int W = a.W, H = a.H;
  const int Hp2 = (H + 1) >> 1;  // row pairs per view
  const long Pv = (long)W * Hp2 * 2;
  const long P = (long)W * H;
  // One workgroup per 64 x TH tile, looping over every level chunk c and
  // neighbour n: a single pipeline of (c, n) steps whose neighbour bands are
  // LDS-DMA double-buffered, so the reference rows are loaded once per tile
  // and only the first band's latency is exposed.
  // XCD-aware map: blocks are dealt round-robin over the 8 XCDs, so block b
  // works in XCD-group b % 8; each group takes a contiguous strip of tiles,
  // whose neighbour bands and halos then overlap in its L2.
  const int bid = blockIdx.x, grp = bid & 7;
  const int tile = grp * a.tiles_per_xcd + (bid >> 3);
  if (tile >= a.ntiles) return;  // padding block (whole workgroup, before any barrier)
  const int x0 = (tile % a.tiles_x) * 64;
  const int y0 = (tile / a.tiles_x) * TH;  // even
  const int x = x0 + lane;
  const int nn = a.nn, T = a.nch * nn;   // pipeline steps
  const NccRec* rec = plan + wave;       // record of step t = c*nn + n for this wave at rec[4 * t]

  // LDS-DMA staging of step t's neighbour bands into buffer b.  Band column j
  // is image column x0 - txmax + j; band pair row i of pk holds image rows
  // 2(pm0+i), 2(pm0+i)+1 with pm0 = (y0-R-tymax)>>1 (stats: (y0-tymax)>>1).
  // Columns and pairs are clamped into the image: edge pixels' windows are
  // invalid (NaN ivr) for R >= 2, so clamped cells never contribute.
  auto stage = [&](int t, int n, int b) {
    const NccRec& e = rec[4 * t];
    const int bhp = e.bhp, shp = e.shp & 0xffff, nblk = e.shp >> 16;
    const int pm0 = (y0 - R - e.tymax) >> 1, sm0 = (y0 - e.tymax) >> 1;
    const long vo = (long)a.view[n] * Pv;
    u32x4* npk = nbase + b * nbuf;
    u32x4* nst = npk + a.pk_pairs * BW;
    for (int cb = 0; cb < nblk; cb++) {
      const int xx = min(max(x0 - e.txmax + cb * 64 + lane, 0), W - 1);
      const uint2* gpk = pk + vo + 2 * xx;
      const uint2* gst = stats + vo + 2 * xx;
      for (int i = wave; i < bhp; i += 4)
        glds_b128(gpk + 2L * W * min(max(pm0 + i, 0), Hp2 - 1), npk + i * BW + cb * 64);
      for (int i = wave; i < shp; i += 4)
        glds_b128(gst + 2L * W * min(max(sm0 + i, 0), Hp2 - 1), nst + i * BW + cb * 64);
    }
  };
  float E[DPW][TH];
  float ivr[TH];
  auto reset = [&]() {
#pragma unroll
    for (int j = 0; j < DPW; j++)
#pragma unroll
      for (int o = 0; o < TH; o++) E[j][o] = -INFINITY;
  };
  // cost = 1 - max(-1, E ivr) of chunk c's levels (v_max_f32 drops the NaN of
  // -inf * 0 and of an invalid reference window); partial tiles/chunks masked
  auto store = [&](int c) {
    if (x >= W) return;
#pragma unroll
    for (int j = 0; j < DPW; j++) {
      const int dl = c * DC + wave + 4 * j;
      if (dl >= a.D) break;
      float* vd = vol + (long)dl * P;  // scalar base; 32-bit per-lane offsets (saddr stores)
      const int off0 = y0 * W + x;
#pragma unroll
      for (int o = 0; o < TH; o++)
        if (y0 + o < H) {
          // streaming store: the volume must not evict the neighbour bands
          // from L2 / MALL (measured: the WTA pass after it also runs faster)
          __builtin_nontemporal_store(1.0f - vmax(E[j][o] * ivr[o], -1.0f), vd + off0 + o * W);
        }
    }
  };

  reset();
  if (T == 0) {  // no neighbours: every window invalid, cost 2
#pragma unroll
    for (int o = 0; o < TH; o++) ivr[o] = __int_as_float(0x7fc00000);
    for (int c = 0; c < a.nch; c++) store(c);
    return;
  }
  stage(0, 0, 0);
  // reference: packed rows y0-R .. y0+TH+R-1 and window stats of rows y0 .. y0+TH-1
  const long zo = (long)a.z * Pv;
  const int xc = min(x, W - 1);
  unsigned qlo[NR], qhi[NR];
#pragma unroll
  for (int k = 0; k < NR; k++) {
    const uint2 v = pk[zo + pair_index(min(max(y0 - R + k, 0), H - 1), xc, W)];
    qlo[k] = v.x;
    qhi[k] = v.y & HI_MASK;
  }
  // K = 5 (FPF): num = n*Srp' - Sr'*Sp' on centred sums (|n Srp'|,
  //   |Sr' Sp'| <= 10.24M), every intermediate an integer below 2^24 and one
  //   rounding at the final fma: bit-identical to (float)num, at the FP32
  //   issue rate (integer VALU ops issue at half rate on gfx950).  K = 7
  //   exceeds 2^24: integer finish.
  // rs[o]: -Sr' (FPF as float, else as int bits)
  float rs[TH];
#pragma unroll
  for (int o = 0; o < TH; o++) {
    const uint2 v = stats[zo + pair_index(min(y0 + o, H - 1), xc, W)];
    rs[o] = FPF ? -__int_as_float((int)v.x) : __int_as_float(-(int)v.x);
    ivr[o] = __int_as_float((int)v.y);
  }
  __syncthreads();

  int n = 0, c = 0;
  for (int t = 0; t < T; t++) {
    const int n1 = n + 1 == nn ? 0 : n + 1;
    if (t + 1 < T) stage(t + 1, n1, (t + 1) & 1);  // prefetch step t+1 while computing t
    const u32x4* npk = nbase + (t & 1) * nbuf;
    const u32x4* nst = npk + a.pk_pairs * BW;
    int lvv[2 * DPW];  // one scalar load of this wave's level shifts for step t
#pragma unroll
    for (int i = 0; i < 2 * DPW; i++) lvv[i] = rec[4 * t].lv[i];
    // levels past the end of the last chunk carry in-band dummy shifts: they
    // are computed and dropped at the store, so the loop is straight-line
#pragma unroll
    for (int j = 0; j < DPW; j++) {
      const int colo = lvv[2 * j], rows = lvv[2 * j + 1];
      u32x2 pv[NR];
      if (EVEN)
        read_rows<NR, BW, true>(npk + colo + lane, rows & 0xffff, pv);
      else
        read_rows<NR, BW, false>(npk + colo + lane, rows & 0xffff, pv);
      // prefix sums over band rows of the horizontal K-tap centred
      // correlation: the dot4 accumulator input carries the running sum
      // (two independent chains over the upper and lower halves of the band
      // rows, joined by one add each, for twice the instruction-level parallelism)
      constexpr int NH = NR / 2;
      int ps[NR];
      int acc0 = 0, acc1 = 0;
#pragma unroll
      for (int k = 0; k < NH; k++) {
        acc0 = __builtin_amdgcn_sdot4((int)qhi[k], (int)pv[k].y,
                                      __builtin_amdgcn_sdot4((int)qlo[k], (int)pv[k].x, acc0, false), false);
        acc1 = __builtin_amdgcn_sdot4((int)qhi[k + NH], (int)pv[k + NH].y,
                                      __builtin_amdgcn_sdot4((int)qlo[k + NH], (int)pv[k + NH].x, acc1, false), false);
        ps[k] = acc0;
        ps[k + NH] = acc1;
      }
#pragma unroll
      for (int k = NH; k < NR; k++) ps[k] += ps[NH - 1];
      u32x2 sv[TH];
      if (EVEN)
        read_rows<TH, BW, true>(nst + colo + lane, rows >> 16, sv);
      else
        read_rows<TH, BW, false>(nst + colo + lane, rows >> 16, sv);
      float pf[NR];
      if (FPF) {
#pragma unroll
        for (int k = 0; k < NR; k++) pf[k] = (float)ps[k];  // < 2^24: exact
      }
#pragma unroll
      for (int o = 0; o < TH; o++) {
        float fa;
        if (FPF) {
          const float spc = __int_as_float((int)sv[o].x);
          const float srp = o > 0 ? pf[o + 2 * R] - pf[o - 1] : pf[2 * R];  // Srp', exact
          fa = __builtin_fmaf(rs[o], spc, (float)NK * srp);                 // (float)num
        } else {
          const int srp = o > 0 ? ps[o + 2 * R] - ps[o - 1] : ps[2 * R];
          fa = (float)(__mul24(NK, srp) + __mul24(__float_as_int(rs[o]), (int)sv[o].x));
        }
        float e = fa * fabsf(fa);
        e = e * __int_as_float((int)sv[o].y);
        E[j][o] = vmax(E[j][o], e);
      }
    }
    if (n1 == 0) {  // chunk c complete
      store(c);
      reset();
      c++;
    }
    n = n1;
    __syncthreads();  // step t+1's bands landed (vmcnt 0); this buffer free for t+2
  }
}

// ---- matrix-core sweep for horizontal camera arrays -----------------------
// When every neighbour's shift is horizontal and linear in the level index,
// tx(l) = t0 + l*delta (integer levels, ty = 0), the centred correlations of
// one image row are a banded integer GEMM:
//   Srp'(x_i, c_j) = sum_k A[i][k] B[k][j],  A[i][k] = window tap k of the
//   reference at pixel x_i,  B[k][j] = tap k of the neighbour at column c_j,
// and level l of pixel x_i is column c = x_i - t0 - l*delta.  With pixels and
// columns taken in one residue class mod s = |delta| (x_i = xa + s i,
// c_j = cb + s j) the needed (i, j) form the diagonal band j - i in
// [0, D-1] of a 16 x (D+15) tile strip: one v_mfma_i32_16x16x64_i8 per 16 x 16
// tile (the K x K window as 8-byte rows of the packed plane, K-group h of a
// lane = one row pair of its 16-byte slot), ~89% of its outputs used at D=128.
// The per-cell finish is the same FP32/integer arithmetic as k_ncc_volume;
// the maximum over neighbours is an LDS float max (ds_max_f32) into the
// workgroup's [level][pixel] tile; cells of the two band-edge N-tiles that
// fall outside [0, D) are clamped into a dump row on either side.
//
// Work: M-tiles (neighbour n, residue rho, tile m; a host table of 16-byte
// records, one per lane, read back with v_readlane) dealt round-robin to the
// 4 waves; a wave loads an M-tile's reference operand and row sums once and
// walks its N-tiles nt = 0 .. NT-1 (the band), prefetching the next N-tile's
// neighbour operand while the current one is multiplied and finished.
constexpr int MF_X = 64;      // pixels per workgroup tile (one image row)
constexpr int MF_PITCH = 65;  // LDS row pitch (floats)
constexpr int MF_LOFF = 1;    // dump rows: one before level 0, one after D-1
struct MfArgs {
  int W, H, D, nmt, nt, z, tiles_x, ntiles, tiles_per_xcd;
};
// w0 = view | s << 16 | (delta < 0) << 24;  w1 = A row 0 pixel - x0 (xo);
// w2 = B column 0 - x0 at nt = 0;  w3 = last row of the M-tile inside the tile
typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int K>
__global__ __launch_bounds__(256) void k_ncc_mfma(const uint2* __restrict__ stats, const uint2* __restrict__ pk,
                                                  const i32x4* __restrict__ mtiles, MfArgs a,
                                                  float* __restrict__ vol) {
  constexpr int R = K / 2, NK = K * K;
  constexpr bool FPF = K == 5;
  constexpr unsigned HI_MASK = ((1u << (8 * (K - 4))) - 1u);
  extern __shared__ float lacc[];  // [D + 2 MF_LOFF][MF_PITCH]
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int W = a.W, H = a.H, D = a.D, NT = a.nt;
  const int Hp2 = (H + 1) >> 1;
  const long Pv = (long)W * Hp2 * 2;
  const long P = (long)W * H;
  const int bid = blockIdx.x, grp = bid & 7;
  const int tile = grp * a.tiles_per_xcd + (bid >> 3);
  if (tile >= a.ntiles) return;
  const int x0 = (tile % a.tiles_x) * MF_X, y = tile / a.tiles_x;
  const int x = x0 + lane;
  const long zo = (long)a.z * Pv;
  const uint2 rst = stats[zo + pair_index(y, min(x, W - 1), W)];
  const float ivr = __int_as_float((int)rst.y);
  const bool row_valid = y >= R && y + R < H;  // otherwise every window is invalid: cost 2

  if (row_valid) {
    for (int i = tid; i < D * MF_X; i += 256) lacc[(i / MF_X + MF_LOFF) * MF_PITCH + (i % MF_X)] = -INFINITY;
    // K-group of this lane: the 16-byte slot (row pair) it reads and which of
    // its two 8-byte rows belong to the window (the A mask zeroes the rest)
    const int h = lane >> 4, g = h, jj = lane & 15;
    const int first = y - R;
    int slot;
    unsigned m0 = 0u, m1 = 0u, m2 = 0u, m3 = 0u;
    if (h < R) {  // a full pair of window rows
      slot = ((first + (first & 1)) >> 1) + h;
      m0 = m2 = 0xffffffffu;
      m1 = m3 = HI_MASK;
    } else if (h == R) {  // the single remaining row: the last (first even) or the first (first odd)
      if ((first & 1) == 0) {
        slot = (y + R) >> 1;
        m0 = 0xffffffffu; m1 = HI_MASK;
      } else {
        slot = first >> 1;
        m2 = 0xffffffffu; m3 = HI_MASK;
      }
    } else {
      slot = 0;
    }
    slot = min(max(slot, 0), Hp2 - 1);
    const u32x4* pkrow = (const u32x4*)pk + (long)slot * W;  // + view * Pv/2 + column
    const unsigned boff = (unsigned)slot * (unsigned)W * 16u;  // byte offset of this lane's slot row
    const long st_row = (long)(y >> 1) * W * 2 + (y & 1);   // stats (uint2) index of (y, column 0)
    const i32x4 batch = mtiles[min(wave + 4 * lane, a.nmt - 1)];
    __syncthreads();

    struct Bop {
      i32x4 B;
      uint2 sb;
    };
    const int nw = a.nmt > wave ? (a.nmt - wave + 3) >> 2 : 0;  // this wave's M-tiles (<= 64)
    const uint2* rstats = stats + zo + st_row;
    // M-tile k's reference operand and row sums, loaded one M-tile ahead
    struct Mt {
      int view, s, neg, xo, co0, imax;
    };
    auto decode = [&](int k) {
      Mt m;
      const int w0 = __builtin_amdgcn_readlane(batch.x, k);
      m.view = w0 & 0xffff;
      m.s = (w0 >> 16) & 0xff;
      m.neg = (w0 >> 24) & 1;
      m.xo = __builtin_amdgcn_readlane(batch.y, k);
      m.co0 = __builtin_amdgcn_readlane(batch.z, k);
      m.imax = __builtin_amdgcn_readlane(batch.w, k);
      return m;
    };
    struct Mload {
      u32x4 av;
      int sv[4];
    };
    auto mload = [&](const Mt& m, Mload& o) {
      // rows past the tile repeat its last pixel: their LDS maxima are
      // duplicates, so partial M-tiles need no masking
      o.av = pkrow[(zo >> 1) + min(x0 + m.xo + m.s * min(jj, m.imax), W - 1)];
#pragma unroll
      for (int q = 0; q < 4; q++) o.sv[q] = (int)rstats[2 * min(x0 + m.xo + m.s * min(4 * g + q, m.imax), W - 1)].x;
    };
    Mload ml;
    if (nw > 0) mload(decode(0), ml);
    for (int k = 0; k < nw; k++) {
      const Mt mt = decode(k);
      const int view = mt.view, s = mt.s, neg = mt.neg, xo = mt.xo, co0 = mt.co0, imax = mt.imax;
      const i32x4 A = i32x4{(int)(ml.av.x & m0), (int)(ml.av.y & m1), (int)(ml.av.z & m2), (int)(ml.av.w & m3)};
      // this lane's output rows i = 4g + q: row sums and LDS addresses; level
      // of (i, jj) at N-tile nt is D-1 + i - jj - 16 nt, or jj - i + 16 nt (delta < 0)
      float nsr[4];
      int aq[4], dq[4], cq[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int ic = min(4 * g + q, imax);  // a duplicate of row imax past the tile
        cq[q] = xo + s * ic;
        nsr[q] = FPF ? -__int_as_float(ml.sv[q]) : __int_as_float(-ml.sv[q]);
        dq[q] = neg ? 4 * g - ic : ic - 4 * g;
        aq[q] = (dq[q] + MF_LOFF) * MF_PITCH + cq[q];
      }
      if (k + 1 < nw) mload(decode(k + 1), ml);  // next M-tile's operands, in flight during this one
      const int rbr = neg ? (jj - 4 * g) : (D - 1 + 4 * g - jj);  // level of (4g, jj) at nt = 0
      const int rb = rbr * MF_PITCH;
      const int rstep = neg ? 16 : -16;  // level step per N-tile
      // N-tiles holding levels outside [0, D): the first and the last one or two
      const int nt_hi_edge = max(1, min(NT, neg ? D / 16 : (D - 16) / 16 + 1));
      // neighbour operand of N-tile nt: 32-bit byte offsets from wave-uniform bases
      const char* bbase = (const char*)((const u32x4*)pk + (long)view * (Pv >> 1));
      const char* sbase = (const char*)(stats + (long)view * Pv + st_row);
      const int cb = x0 + co0 + s * jj, cstep = 16 * s;
      auto loadb = [&](int nt, Bop& o) {
        int c = cb + cstep * nt;
        asm("v_med3_i32 %0, %1, 0, %2" : "=v"(c) : "v"(c), "s"(W - 1));
        const u32x4 bv = *(const u32x4*)(bbase + (boff + ((unsigned)c << 4)));
        o.B = i32x4{(int)bv.x, (int)bv.y, (int)bv.z, (int)bv.w};
        o.sb = *(const uint2*)(sbase + ((unsigned)c << 4));
      };
      // finish of two N-tiles, in lockstep across their 8 outputs (independent
      // chains interleaved).  EDGE: N-tiles whose band cells may fall outside
      // [0, D), clamped into the dump rows.
      auto finish2 = [&](auto edge_tag, const i32x4& accA, const uint2& sbA, int ntA, const i32x4& accB,
                         const uint2& sbB, int ntB) {
        constexpr bool EDGE = decltype(edge_tag)::value;
        float f[8];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          f[q] = (float)accA[q];
          f[4 + q] = (float)accB[q];
        }
        if (FPF) {
#pragma unroll
          for (int q = 0; q < 8; q++) f[q] = (float)NK * f[q];
#pragma unroll
          for (int q = 0; q < 4; q++) {
            f[q] = __builtin_fmaf(nsr[q], __int_as_float((int)sbA.x), f[q]);
            f[4 + q] = __builtin_fmaf(nsr[q], __int_as_float((int)sbB.x), f[4 + q]);
          }
        } else {
#pragma unroll
          for (int q = 0; q < 4; q++) {
            f[q] = (float)(__mul24(NK, accA[q]) + __mul24(__float_as_int(nsr[q]), (int)sbA.x));
            f[4 + q] = (float)(__mul24(NK, accB[q]) + __mul24(__float_as_int(nsr[q]), (int)sbB.x));
          }
        }
#pragma unroll
        for (int q = 0; q < 8; q++) f[q] = f[q] * fabsf(f[q]);
#pragma unroll
        for (int q = 0; q < 4; q++) {
          f[q] = f[q] * __int_as_float((int)sbA.y);
          f[4 + q] = f[4 + q] * __int_as_float((int)sbB.y);
        }
        // an invalid neighbour window gives NaN: ds_max_f32 keeps the stored
        // value then (IEEE maxNum, as v_max_f32; pinned by the border cells of
        // the parity tests)
        int ad[8];
#pragma unroll
        for (int u = 0; u < 2; u++) {
          const int nt = u ? ntB : ntA;
#pragma unroll
          for (int q = 0; q < 4; q++) {
            if (EDGE) {
              int row = rbr + rstep * nt + dq[q];
              asm("v_med3_i32 %0, %1, -1, %2" : "=v"(row) : "v"(row), "s"(D));
              ad[4 * u + q] = (row + MF_LOFF) * MF_PITCH + cq[q];
            } else {
              ad[4 * u + q] = rb + rstep * MF_PITCH * nt + aq[q];
            }
          }
        }
#pragma unroll
        for (int q = 0; q < 8; q++)
          __hip_atomic_fetch_max(lacc + ad[q], f[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      };
      // N-tiles 0 .. NT-1, two per step: both products issued before either
      // finish, the next pair's operands loaded into the other register pair
      // (4 operand sets, so no load lands in a register still in use); an odd
      // count repeats the last N-tile, which the maximum absorbs
      auto pair = [&](const Bop& x0p, const Bop& x1p, Bop& y0p, Bop& y1p, int nt) {
        const int nt1 = min(nt + 1, NT - 1);
        const i32x4 acc0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, x0p.B, i32x4{0, 0, 0, 0}, 0, 0, 0);
        const i32x4 acc1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, x1p.B, i32x4{0, 0, 0, 0}, 0, 0, 0);
        loadb(min(nt + 2, NT - 1), y0p);
        loadb(min(nt + 3, NT - 1), y1p);
        if (nt == 0 || nt1 >= nt_hi_edge)
          finish2(std::true_type{}, acc0, x0p.sb, nt, acc1, x1p.sb, nt1);
        else
          finish2(std::false_type{}, acc0, x0p.sb, nt, acc1, x1p.sb, nt1);
        // keep the next pair's products below these finishes: hoisted, they
        // would wait on the loads just issued
        __builtin_amdgcn_sched_barrier(0);
      };
      Bop b0, b1, b2, b3;
      loadb(0, b0);
      loadb(min(1, NT - 1), b1);
      int nt = 0;
      for (; nt + 2 < NT; nt += 4) {
        pair(b0, b1, b2, b3, nt);
        pair(b2, b3, b0, b1, nt + 2);
      }
      if (nt < NT) pair(b0, b1, b2, b3, nt);
    }
    __syncthreads();
  }
  // cost = 1 - max(-1, m ivr) per level, 64-column coalesced rows
  if (x >= W) return;
  float* vy = vol + (long)y * W + x;
  const float ivr_e = row_valid ? ivr : __int_as_float(0x7fc00000);
  int l = wave;
  for (; l + 12 < D; l += 16) {
    float m[4];
#pragma unroll
    for (int u = 0; u < 4; u++) m[u] = row_valid ? lacc[(l + 4 * u + MF_LOFF) * MF_PITCH + lane] : -INFINITY;
#pragma unroll
    for (int u = 0; u < 4; u++) vy[(long)(l + 4 * u) * P] = 1.0f - vmax(m[u] * ivr_e, -1.0f);
  }
  for (; l < D; l += 4) {
    const float m = row_valid ? lacc[(l + MF_LOFF) * MF_PITCH + lane] : -INFINITY;
    vy[(long)l * P] = 1.0f - vmax(m * ivr_e, -1.0f);
  }
}

// M-tile table + launch; returns 1 when the neighbour set is not eligible.
template <int K>
int launch_ncc_mfma(mvs_ctx* ctx, const uint2* stats, const uint2* pk, int W, int H, int D, int z, int nn,
                    const int* view, const float* levels, const float* fdx, const float* fdy, float bl,
                    float* vol) {
  std::vector<int32_t> tab;
  for (int n = 0; n < nn; n++) {
    const int t0 = (int)roundf(levels[0] * fdx[n]);
    const int delta = D > 1 ? (int)roundf(levels[1] * fdx[n]) - t0 : 1;
    if (delta == 0 || view[n] > 0xffff) return 1;
    for (int l = 0; l < D; l++)
      if ((int)roundf(levels[l] * fdx[n]) != t0 + l * delta || (int)roundf((bl * levels[l]) * fdy[n]) != 0) return 1;
    const int s = delta < 0 ? -delta : delta;
    if (s > 16) return 1;  // wider strides leave most MFMA rows idle
    const int J0 = delta > 0 ? D - 1 : 0;
    for (int rho = 0; rho < s; rho++) {
      const int cnt = (MF_X - rho + s - 1) / s;  // pixels of the residue class in the tile
      for (int m = 0; 16 * m < cnt; m++) {
        const int xo = rho + 16 * s * m;
        const int32_t e[4] = {view[n] | (s << 16) | (delta < 0 ? 1 << 24 : 0), xo, xo - t0 - s * J0,
                              std::min(15, cnt - 16 * m - 1)};
        tab.insert(tab.end(), e, e + 4);
      }
    }
  }
  const int nmt = (int)(tab.size() / 4);
  if (nmt > 256) return 1;  // one 64-record batch per wave
  int rc = 0;
  const i32x4* dev = (const i32x4*)plan_upload(ctx, tab, &rc);
  if (rc) return rc;
  MfArgs a{};
  a.W = W; a.H = H; a.D = D; a.z = z;
  a.nmt = nmt;
  a.nt = (D + 15 + 15) / 16;  // N-tiles covering the band j - i in [0, D-1]
  a.tiles_x = (W + MF_X - 1) / MF_X;
  a.ntiles = a.tiles_x * H;
  a.tiles_per_xcd = (a.ntiles + 7) / 8;
  const size_t lds = sizeof(float) * (size_t)(D + 2 * MF_LOFF) * MF_PITCH;
  if (lds > 160 * 1024) return 1;
  auto kern = k_ncc_mfma<K>;
  if (lds > 64 * 1024)
    MVS_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
            "hipFuncSetAttribute(ncc mfma lds)");
  hipLaunchKernelGGL(kern, dim3(8 * a.tiles_per_xcd), dim3(256), lds, ctx->stream, stats, pk, dev, a, vol);
  MVS_LAUNCH_CHECK("k_ncc_mfma");
  return 0;
}

// Host side: the chunk/level shift plan (every roundf of the definition is
// evaluated here, once per distinct configuration) and the launch.
struct NccPlan {
  std::vector<int32_t> table;  // NccRec [nchunks][nn][4 waves] as int32
  int band_w = 0, pk_pairs = 0, st_pairs = 0;
  bool even = true;  // every level's band rows start on a pair boundary
};

inline int floor_half(int v) { return v >> 1; }  // arithmetic: floor(v / 2)

template <int K, int TH, int DPW>
NccPlan make_plan(const float* levels, int D, int nn, const float* fdx, const float* fdy, float bl) {
  constexpr int R = K / 2, NR = TH + 2 * R, DC = 4 * DPW;
  static_assert(DPW <= 8, "NccRec holds 8 levels per wave");
  constexpr int RW = sizeof(NccRec) / 4;
  const int nch = (D + DC - 1) / DC;
  NccPlan p;
  p.table.assign((size_t)nch * nn * 4 * RW, 0);
  int spx = 0;
  auto tx_of = [&](int dl, int n) { return (int)roundf(levels[dl] * fdx[n]); };
  auto ty_of = [&](int dl, int n) { return (int)roundf((bl * levels[dl]) * fdy[n]); };
  // y0 is even (TH even), so every row parity below is independent of y0
  for (int c = 0; c < nch; c++)
    for (int n = 0; n < nn; n++) {
      int txmin = 1 << 30, txmax = -(1 << 30), tymin = 1 << 30, tymax = -(1 << 30);
      for (int dl = c * DC; dl < std::min(D, c * DC + DC); dl++) {
        txmin = std::min(txmin, tx_of(dl, n)); txmax = std::max(txmax, tx_of(dl, n));
        tymin = std::min(tymin, ty_of(dl, n)); tymax = std::max(tymax, ty_of(dl, n));
      }
      const int pb = -R - tymax, sb = -tymax;            // band first image row - y0
      const int pr = pb - 2 * floor_half(pb), sr = sb - 2 * floor_half(sb);  // its parity in the pair band
      const int bhp = (pr + NR + tymax - tymin + 1) >> 1;  // pairs covering every level's rows
      const int shp = (sr + TH + tymax - tymin + 1) >> 1;
      const int nblk = (64 + txmax - txmin + 63) >> 6;
      for (int w = 0; w < 4; w++) {
        int32_t* e = p.table.data() + (((size_t)c * nn + n) * 4 + w) * RW;
        e[0] = txmax;
        e[1] = tymax;
        e[2] = bhp;
        e[3] = shp | (nblk << 16);
        for (int j = 0; j < DPW; j++) {
          const int dl = c * DC + w + 4 * j;
          if (dl >= D) {  // dummy level past the end: the band origin's even rows
            e[4 + 2 * j] = 0;
            e[5 + 2 * j] = pr | (sr << 16);
            continue;
          }
          const int ty = ty_of(dl, n);
          e[4 + 2 * j] = txmax - tx_of(dl, n);
          e[5 + 2 * j] = (pr + tymax - ty) | ((sr + tymax - ty) << 16);
          if (((pr + tymax - ty) | (sr + tymax - ty)) & 1) p.even = false;
        }
      }
      spx = std::max(spx, txmax - txmin);
      p.pk_pairs = std::max(p.pk_pairs, bhp);
      p.st_pairs = std::max(p.st_pairs, shp);
    }
  p.band_w = (64 + spx + 63) & ~63;  // whole 64-column LDS-DMA pieces per pair row
  return p;
}

template <int K, int TH, int DPW, int BW, bool EVEN>
int launch_ncc_bw(hipStream_t s, const uint2* stats, const uint2* pk, const NccRec* plan, NccArgs& a, float* vol,
                  size_t lds) {
  constexpr int DC = 4 * DPW;
  a.tiles_x = (a.W + 63) / 64;
  a.ntiles = a.tiles_x * ((a.H + TH - 1) / TH);
  a.tiles_per_xcd = (a.ntiles + 7) / 8;
  a.nch = (a.D + DC - 1) / DC;
  dim3 g(8 * a.tiles_per_xcd);
  auto kern = k_ncc_volume<K, TH, DPW, BW, EVEN>;
  if (lds > 64 * 1024)
    MVS_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
            "hipFuncSetAttribute(ncc lds)");
  hipLaunchKernelGGL(kern, g, dim3(256), lds, s, stats, pk, plan, a, vol);
  MVS_LAUNCH_CHECK("k_ncc_volume");
  return 0;
}

// returns 1 if this variant does not fit the LDS (caller tries a smaller one)
template <int K, int TH, int DPW>
int launch_ncc_t(mvs_ctx* ctx, const uint2* stats, const uint2* pk, NccArgs& a, const float* levels_host,
                 const float* fdx, const float* fdy, float bl, float* vol, size_t lds_cap) {
  NccPlan p = make_plan<K, TH, DPW>(levels_host, a.D, a.nn, fdx, fdy, bl);
  const size_t lds = 2 * 16 * (size_t)(p.pk_pairs + p.st_pairs) * p.band_w;
  if (lds > lds_cap || p.band_w > 256) return 1;
  int rc = 0;
  const int32_t* dev = plan_upload(ctx, p.table, &rc);
  if (rc) return rc;
  a.pk_pairs = p.pk_pairs;
  a.st_pairs = p.st_pairs;
  const NccRec* plan = (const NccRec*)dev;
  if (p.even) {
    if (p.band_w <= 128) return launch_ncc_bw<K, TH, DPW, 128, true>(ctx->stream, stats, pk, plan, a, vol, lds);
    if (p.band_w <= 192) return launch_ncc_bw<K, TH, DPW, 192, true>(ctx->stream, stats, pk, plan, a, vol, lds);
    return launch_ncc_bw<K, TH, DPW, 256, true>(ctx->stream, stats, pk, plan, a, vol, lds);
  }
  if (p.band_w <= 128) return launch_ncc_bw<K, TH, DPW, 128, false>(ctx->stream, stats, pk, plan, a, vol, lds);
  if (p.band_w <= 192) return launch_ncc_bw<K, TH, DPW, 192, false>(ctx->stream, stats, pk, plan, a, vol, lds);
  return launch_ncc_bw<K, TH, DPW, 256, false>(ctx->stream, stats, pk, plan, a, vol, lds);
}

}  // namespace

int launch_box_stats(hipStream_t s, const uint8_t* l8, int V, int W, int H, int K, int32_t* box) {
  const int Hp = H + (H & 1);
  uint2* stats = (uint2*)box;
  uint2* pk = stats + (long)V * W * Hp;
  dim3 g((W + BS_TW - 1) / BS_TW, (Hp + BS_TH - 1) / BS_TH, V);
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
  const uint2* pk = stats + (long)V * W * (H + (H & 1));
  // MVS_NCC_MFMA=1: the matrix-core sweep for horizontal arrays with integer
  // level steps (bit-identical; measured slower than the vector sweep on
  // MI355X), else the vector sweep
  const char* mf = getenv("MVS_NCC_MFMA");
  if (mf && mf[0] == '1' && a.nn > 0) {
    const int rc = K == 5 ? launch_ncc_mfma<5>(ctx, stats, pk, W, H, D, z, a.nn, a.view, levels_host, fdx, fdy, bl, vol)
                 : K == 7 ? launch_ncc_mfma<7>(ctx, stats, pk, W, H, D, z, a.nn, a.view, levels_host, fdx, fdy, bl, vol)
                          : 1;
    if (rc != 1) return rc;
  }
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
  // first the widest variant whose double-buffered bands leave room for two
  // workgroups per CU (vertical shifts grow the bands: fewer levels per step
  // then beat a single resident workgroup), then any that fits the LDS
#define MVS_NCC_TRY(KK, TT, PP)                                                                     \
  if (rc == 1) rc = launch_ncc_t<KK, TT, PP>(ctx, stats, pk, a, levels_host, fdx, fdy, bl, vol, cap);
  for (size_t cap : {(size_t)80 * 1024, (size_t)160 * 1024}) {
    if (K == 5) {
      if (th_env == 16) {
        if (dpw_env >= 4) MVS_NCC_TRY(5, 16, 4)
        if (dpw_env >= 2) MVS_NCC_TRY(5, 16, 2)
      }
      if (dpw_env >= 8) MVS_NCC_TRY(5, 8, 8)
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
  }
#undef MVS_NCC_TRY
  if (rc == 1) return arg_fail("NCC sweep: neighbour shifts too large for the LDS band");
  return rc;
}

}  // namespace mvs
