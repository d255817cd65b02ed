// Build-defined per-pixel NCC K x K plane sweep: the cost-volume producer.
//
// Definition (no reference counterpart; restated in oracle/mvs_oracle.c
// orc_ncc_volume): q = 8-bit intensity (clamp(int(L*2.55+0.5))), q' = q - 128,
// window K x K, n = K*K, shift of neighbour n at level d:
// (tx, ty) = (roundf(d*dx), roundf((bl*d)*dy)); window valid iff every tap of
// the reference and the shifted window is inside the image.  With centred
// integer sums Sr', Sp', Srp' and var = n*Sqq - Sq^2:
//   s = var ? 1/sqrtf((float)var) : 0 per window,
//   a = n*s, b = Sp'*s per neighbour pixel (the box planes below),
//   x = fma(-Sr', b, Srp'*a)            (= NCC * sqrt(var_r)),
//   m = max over valid neighbours of x (-inf if none),
//   vol[d][y][x] = 1 - max(-1, m*s_r):  1 minus the best NCC; 1 on a
//   textureless reference window, 2 when no neighbour window is valid.
// (s_r after the maximum: rounding is monotone, so m*s_r = max_n (x_n*s_r).)
//
// Data layout (mvs_box_stats_d, per view, 16 B/px in two planes of row pairs):
//   stats [V][Hp/2][W] float4 {a(2m), a(2m+1), b(2m), b(2m+1)}: rows 2m, 2m+1
//                   of column x, NaN where the window leaves the image;
//   pk    [V][H][W] {lo, hi}: the 8 centred intensities q' (int8) of columns
//                   x-R .. x-R+7 of row y, packed little-endian, stored at
//                   uint2 index ((y >> 1) * W + x) * 2 + (y & 1).
// Validity is carried by the data: an invalid neighbour window makes x NaN
// and v_max_f32 (IEEE maxNum) drops it -- no per-cell bounds logic.
//
// Kernel (gfx950, wave64, NW = 4 or 8 waves per workgroup):
//   * tile = 64 image columns (one per lane) x TH rows x a chunk of NW*DPW
//     hypotheses; wave w owns levels w, w+NW, ...;
//   * the reference's packed rows live in registers, its window sums and s_r
//     are computed from them once per tile;
//   * per neighbour, the pk and stats bands covering every shift of the chunk
//     are staged in LDS by 16-byte LDS-DMA, double-buffered so the next
//     neighbour's bands land while this one is computed;
//   * per (level, neighbour) a lane walks its column: per band row two
//     VOP3P v_dot4_i32_i8 extend one prefix-sum chain of the horizontal K-tap
//     centred correlation (no accumulator copies; the chain starts at the
//     bits of 1.5 * 2^23, so two prefix sums read as floats differ by exactly
//     Srp': one float subtract per output row, no integer convert), and per PAIR of output rows one
//     v_pk_mul_f32 + one v_pk_fma_f32 give x (rows 2m, 2m+1 of the stats
//     plane are one 16-byte LDS read), then v_max_f32 per cell;
//   * the chunk's costs are written once, 64-column coalesced rows.
#include <algorithm>
#include <array>
#include <vector>
#include <type_traits>
#include <cstdlib>

#include "ncc_common.h"

namespace mvs {
namespace {
using namespace ncc;


// ---- window statistics + packed intensities ------------------------------
// one workgroup = 64 columns x 16 rows of one view; the (16+2R) x 76 byte
// tile (image columns x0-4 .. x0+71) is staged in LDS once, by aligned 4-byte
// loads when W % 4 == 0.  A thread owns one column and two row pairs: per
// tile row it takes the 8 bytes starting at its window's left column (three
// LDS dwords + v_alignbyte), whose first K give the horizontal sums
// (v_sad_u8 against 0) and sums of squares (v_dot4_u32_u8 with itself); the
// vertical sums slide over those rows.  Each row pair is written as one
// 16-byte store per plane (rows 2m, 2m+1 are adjacent in the pair layout).
// All sums are exact integers, so the planes are the ones the per-tap loop
// made.  The dummy row H of an odd-height image is written as an invalid
// window.
constexpr int BS_TW = 64, BS_TH = 16;
template <int R>
__global__ __launch_bounds__(256) void k_box_stats(const uint8_t* __restrict__ q, int W, int H,
                                                   int z0, uint2* __restrict__ stats, uint2* __restrict__ pk) {
  constexpr int K = 2 * R + 1, NK = K * K, NR = 4 + 2 * R;
  constexpr int TW = BS_TW + 12, TR = BS_TH + 2 * R, ND = TW / 4, OFF = 4 - R;
  static_assert(R <= 3, "the window's K taps must fit the 8 bytes a thread takes per row");
  __shared__ uint32_t t[TR][ND + 1];  // byte column c of a row = image column x0 - 4 + c
  const int x0 = blockIdx.x * BS_TW, y0 = blockIdx.y * BS_TH, z = z0 + blockIdx.z;
  const int Hp = H + (H & 1);
  const long Pv = (long)W * Hp;  // plane elements per view
  const uint8_t* Q = q + z * (long)W * H;
  if ((W & 3) == 0 && ((uintptr_t)q & 3) == 0) {  // rows start on 4-byte boundaries: a dword is wholly in or out
    for (int i = threadIdx.x; i < TR * ND; i += 256) {
      const int r = i / ND, d = i - r * ND;
      const int yy = y0 - R + r, xx = x0 - 4 + 4 * d;
      t[r][d] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? *(const uint32_t*)(Q + (long)yy * W + xx) : 0u;
    }
  } else {
    for (int i = threadIdx.x; i < TR * ND; i += 256) {
      const int r = i / ND, d = i - r * ND;
      const int yy = y0 - R + r;
      uint32_t v = 0;
      if (yy >= 0 && yy < H) {
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const int xx = x0 - 4 + 4 * d + b;
          if (xx >= 0 && xx < W) v |= (uint32_t)Q[(long)yy * W + xx] << (8 * b);
        }
      }
      t[r][d] = v;
    }
  }
  __syncthreads();
  const int lx = threadIdx.x & 63, ly0 = (threadIdx.x >> 6) * 4;  // two row pairs per thread
  const int x = x0 + lx;
  if (x >= W) return;
  const int c0 = lx + OFF, dw = c0 >> 2, sh = c0 & 3;  // image column x - R
  constexpr uint32_t hmask = K == 7 ? 0x00ffffffu : K == 5 ? 0x000000ffu : 0u;
  uint32_t lo[NR], hi[NR];
  int hs[NR], hq[NR];
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const uint32_t d0 = t[ly0 + r][dw], d1 = t[ly0 + r][dw + 1], d2 = t[ly0 + r][dw + 2];
    lo[r] = __builtin_amdgcn_alignbyte(d1, d0, sh);
    hi[r] = __builtin_amdgcn_alignbyte(d2, d1, sh);
    const uint32_t hk = K == 3 ? 0u : hi[r] & hmask;
    const uint32_t lk = K == 3 ? lo[r] & 0x00ffffffu : lo[r];
    hs[r] = (int)__builtin_amdgcn_sad_u8(hk, 0u, __builtin_amdgcn_sad_u8(lk, 0u, 0u));
    hq[r] = (int)__builtin_amdgcn_udot4(hk, hk, __builtin_amdgcn_udot4(lk, lk, 0u, false), false);
  }
#pragma unroll
  for (int m = 0; m < 2; m++) {
    const int y = y0 + ly0 + 2 * m;
    if (y >= Hp) break;  // Hp and y are even: a pair is wholly in or out
    float av[2], bv[2];
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 2; e++) {
      const int k = 2 * m + e, yy = y + e;
      int s = 0, ss = 0;
#pragma unroll
      for (int j = 0; j < K; j++) {
        s += hs[k + j];
        ss += hq[k + j];
      }
      const bool valid = x - R >= 0 && x + R < W && yy - R >= 0 && yy + R < H;
      const int var = NK * ss - s * s;
      const float sv = !valid ? __int_as_float(0x7fc00000) : (var != 0 ? 1.0f / sqrtf((float)var) : 0.0f);
      av[e] = (float)NK * sv;
      bv[e] = (float)(s - 128 * NK) * sv;  // centred window sum Sp' * s
      // q - 128 as int8 is q ^ 0x80
      const bool in = yy < H;
      w[2 * e] = in ? lo[k + R] ^ 0x80808080u : 0u;
      w[2 * e + 1] = in ? hi[k + R] ^ 0x80808080u : 0u;
    }
    const long pi = ((long)(y >> 1) * W + x) << 1;  // pair_index(y, x, W), y even
    *(float4*)((float*)stats + z * Pv * 2 + 2 * pi) = make_float4(av[0], av[1], bv[0], bv[1]);
    *(uint4*)(pk + z * Pv + pi) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}


// PAR: the bands' row parity (kParEven / kParOdd: branch-free pair reads).
// FUSE: instead of writing the volume, every wave folds its levels' costs into
// a per-pixel (smallest cost, its level, second smallest cost) in level order;
// the workgroup then merges its waves through LDS into disp/conf.  A wave's
// levels are NW >= 4 apart, so at most one of them lies in best+-1: the
// smallest cost outside best+-1 is, per wave, its second smallest if its best
// level is in that window, else its smallest -- exactly what k_wta's top-4
// yields (ties resolved to the lower level by the strict < in level order).
// NB: band buffers.  2: step t+1's bands land while step t computes.  1: one
// buffer, staged at the start of each step behind a barrier (the other
// resident workgroup computes meanwhile) -- the form that lets 32-level chunks
// with tall vertical / diagonal bands keep two workgroups per CU (C4's 5-NN lists)
template <int K, int TH, int DPW, int NW, int BW, int PAR, bool FUSE, int NB = 2>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(4))) void k_ncc_volume(const uint2* __restrict__ stats, const uint2* __restrict__ pk,
                                                    const NccRec* __restrict__ plan, NccArgs a,
                                                    float* __restrict__ vol, WtaOut wo) {
  static_assert(!FUSE || NW >= 3, "fused WTA needs a wave's levels >= 3 apart");
  constexpr int R = K / 2;
  constexpr int NR = TH + 2 * R;
  constexpr int NK = K * K;
  constexpr int DC = NW * DPW;
  static_assert(TH % 2 == 0 && NR % 2 == 0, "row pairs");
  // taps x-R .. x-R+3 in lo, x-R+4 .. x+R in the low K-4 bytes of hi
  constexpr unsigned HI_MASK = (K - 4) >= 4 ? 0xffffffffu : ((1u << (8 * (K - 4))) - 1u);
  extern __shared__ __align__(16) uint8_t smem[];
  const int nbuf = (a.pk_pairs + a.st_pairs) * BW;  // uint4 per neighbour buffer
  u32x4* nbase = (u32x4*)smem;                      // NB x {npk[pk_pairs][BW], nst[st_pairs][BW]}

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
  // Several reference views per launch (fused sweep): the tiles of reference
  // r of the launch are r * ntiles .. r * ntiles + ntiles - 1, one kernel
  // boundary for the run instead of one per view.
  const int bid = blockIdx.x, grp = bid & 7;
  const int tg = grp * a.tiles_per_xcd + (bid >> 3);
  if (tg >= a.ntiles * a.nref) return;  // padding block (whole workgroup, before any barrier)
  const int ref = tg / a.ntiles, tile = tg - ref * a.ntiles;
  const int x0 = (tile % a.tiles_x) * 64;
  const int y0 = (tile / a.tiles_x) * TH;  // even
  const int x = x0 + lane;
  const int nn = a.nn[ref], T = a.nch * nn;  // pipeline steps
  const NccRec* rec = plan + a.plan[ref] + wave;  // record of step t = c*nn + n for this wave at rec[NW * t]

  // LDS-DMA staging of step t's neighbour bands into buffer b.  Band column j
  // is image column x0 - txmax + j; band pair row i of pk holds image rows
  // 2(pm0+i), 2(pm0+i)+1 with pm0 = (y0-R-tymax)>>1 (stats: (y0-tymax)>>1).
  // Columns and pairs are clamped into the image: edge pixels' windows are
  // invalid (NaN ivr) for R >= 2, so clamped cells never contribute.  A pair
  // row takes 64 + span columns (span: this neighbour's column-shift range
  // over the chunk) in 64-column DMA pieces at columns 0, 64, ..., the last
  // one moved back to end at column 64 + span: it never writes past the row,
  // so the row pitch BW need only hold 64 + the widest span (not a multiple
  // of 64), and the overlapped columns get the same bytes twice.
  // A view plane under 2 GB (plane32) is staged through buffer descriptors:
  // the lane's 32-bit offset (clamped column x 16 B) fixed per piece, the
  // clamped pair row as the scalar offset -- no per-lane 64-bit address per row
  // (C4's tall bands stage up to ~40 pair rows per step)
  auto stage = [&](int t, int n, int b) {
    const NccRec& e = rec[NW * t];
    const int bhp = e.bhp, shp = e.shp & 0xffff, span = e.shp >> 16, nblk = (span + 127) >> 6;
    const int pm0 = (y0 - R - e.tymax) >> 1, sm0 = (y0 - e.tymax) >> 1;
    const long vo = (long)a.view[ref][n] * Pv;
    u32x4* npk = nbase + b * nbuf;
    u32x4* nst = npk + a.pk_pairs * BW;
    if (a.plane32) {
      const int pb = 16 * W;  // bytes per pair row
      const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc((void*)(pk + vo), 0, pb * Hp2, 0x00020000);
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(stats + vo), 0, pb * Hp2, 0x00020000);
      for (int cb = 0; cb < nblk; cb++) {
        const int c0 = min(cb * 64, span);
        const int voff = 16 * min(max(x0 - e.txmax + c0 + lane, 0), W - 1);
        for (int i = wave; i < bhp; i += NW)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rp, (lds_ptr_t)(npk + i * BW + c0), 16, voff,
                                                   pb * min(max(pm0 + i, 0), Hp2 - 1), 0, 0);
        for (int i = wave; i < shp; i += NW)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(nst + i * BW + c0), 16, voff,
                                                   pb * min(max(sm0 + i, 0), Hp2 - 1), 0, 0);
      }
      return;
    }
    for (int cb = 0; cb < nblk; cb++) {
      const int c0 = min(cb * 64, span);
      const int xx = min(max(x0 - e.txmax + c0 + lane, 0), W - 1);
      const uint2* gpk = pk + vo + 2 * xx;
      const uint2* gst = stats + vo + 2 * xx;
      for (int i = wave; i < bhp; i += NW)
        glds_b128(gpk + 2L * W * min(max(pm0 + i, 0), Hp2 - 1), npk + i * BW + c0);
      for (int i = wave; i < shp; i += NW)
        glds_b128(gst + 2L * W * min(max(sm0 + i, 0), Hp2 - 1), nst + i * BW + c0);
    }
  };
  float E[DPW][TH];
  float sr[TH];  // reference 1/sqrt(var) per output row (NaN: invalid window)
  // FUSE: sr lives in LDS during the step loop (lane-major [64][TH], after
  // the band buffers and the merge area), read back at each chunk's fold --
  // 8 fewer long-lived VGPRs, so the loop needs no scratch reload (a VMEM
  // load there waits behind the in-flight band LDS-DMA)
  float* srl = (float*)(smem + 16 * (size_t)max(NB * nbuf, FUSE ? 3 * NW * TH * 64 / 4 : 0));
  float wv0[TH], wv1[TH];  // FUSE: this wave's smallest and second smallest cost per row
  int wi0[TH];             //       level of the smallest
  // fused K = 7: the levels of rows 2m, 2m+1 as the halves of one register
  // (0xffff: none yet).  With one register per row the fold went past the
  // 128-VGPR cap (r03: 96 B of scratch, three of them spilled and reloaded at
  // every chunk's fold -- C5's fused launch moved 40 GB of scratch writes
  // against 0.5 GB of output); a half-select costs one v_bfi_b32 more per cell
  constexpr bool PKI = FUSE && (K == 7 || (PAR == kParMixed && DPW == 4));  // (K = 5: the mixed-parity 4-level kernels, C4)
  unsigned wi0p[TH / 2];
  if (FUSE) {
#pragma unroll
    for (int o = 0; o < TH; o++) {
      wv0[o] = kWtaInit;
      wv1[o] = kWtaInit;
      wi0[o] = -1;
    }
#pragma unroll
    for (int m = 0; m < TH / 2; m++) wi0p[m] = 0xffffffffu;
  }
  auto reset = [&]() {
#pragma unroll
    for (int j = 0; j < DPW; j++)
#pragma unroll
      for (int o = 0; o < TH; o++) E[j][o] = -INFINITY;
  };
  // cost = 1 - max(-1, m s_r) of chunk c's levels (v_max_f32 drops the NaN of
  // -inf * 0 and of an invalid reference window); partial tiles/chunks masked
  auto store = [&](int c) {
    if (x >= W) return;
    if (FUSE) {
      // the fold, one quad of rows at a time: s_r of 4 rows (one ds_read_b128)
      // folded for every level before the next quad's are loaded, so at most 4
      // s_r registers are live beside E and the triple (at K = 7 the whole
      // tile's 8 pushed the fold past the 128-VGPR cap: r03, 96 B of scratch,
      // three accumulators spilled and reloaded at every chunk's fold -- C5's
      // fused launch moved 40 GB of scratch writes against 0.5 GB of output)
      const int ln = lane_now();
#pragma unroll
      for (int q = 0; q < TH; q += 4) {
        const f32x4 sq = *(const f32x4*)(srl + ln * TH + q);
#pragma unroll
        for (int j = 0; j < DPW; j++) {
          const int dl = c * DC + wave + NW * j;
          if (dl >= a.D) break;
          const unsigned dl2 = (unsigned)dl * 0x10001u;
#pragma unroll
          for (int o = q; o < q + 4; o += 2) {
            const f32x2 e = f32x2{E[j][o], E[j][o + 1]} * f32x2{sq[o - q], sq[o - q + 1]};
            const f32x2 r = f32x2{1.0f, 1.0f} - f32x2{vmax_m1(e.x), vmax_m1(e.y)};
#pragma unroll
            for (int h = 0; h < 2; h++) {
              const float cc = r[h];
              wv1[o + h] = vmed3(wv0[o + h], wv1[o + h], cc);  // second smallest
              if (PKI) {
                const unsigned hm = h ? 0xffff0000u : 0x0000ffffu;
                wi0p[o >> 1] = cc < wv0[o + h] ? (wi0p[o >> 1] & ~hm) | (dl2 & hm) : wi0p[o >> 1];
              } else {
                wi0[o + h] = cc < wv0[o + h] ? dl : wi0[o + h];
              }
              wv0[o + h] = vmin(wv0[o + h], cc);
            }
          }
        }
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < DPW; j++) {
      const int dl = c * DC + wave + NW * j;
      if (dl >= a.D) break;
      // buffer stores: the level plane as a buffer resource (scalar), the lane's
      // byte offset fixed for the tile, the row offset scalar -- no address VALU
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(vol + (long)dl * P, 0, (int)(P * 4), 0x00020000);
      const int off0 = (y0 * W + x) * 4;
      // cost pairs: m*s_r as one v_pk_mul_f32, 1 - c as one v_pk_add_f32
      float cst[TH];
#pragma unroll
      for (int o = 0; o < TH; o += 2) {
        const f32x2 e = f32x2{E[j][o], E[j][o + 1]} * f32x2{sr[o], sr[o + 1]};
        const f32x2 m = f32x2{vmax_m1(e.x), vmax_m1(e.y)};
        const f32x2 r = f32x2{1.0f, 1.0f} - m;
        cst[o] = r.x;
        cst[o + 1] = r.y;
      }
      // streaming (nt) stores: the volume must not evict the neighbour bands
      // from L2 / MALL (measured: the WTA pass after it also runs faster)
#pragma unroll
      for (int o = 0; o < TH; o++)
        if (y0 + TH <= H || y0 + o < H)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(cst[o]), rs, off0, o * W * 4, kCPolNT);
    }
  };

  if (T == 0) {  // no neighbours: every window invalid, cost 2
    reset();
#pragma unroll
    for (int o = 0; o < TH; o++) sr[o] = __int_as_float(0x7fc00000);
    if (FUSE) {  // the fused store reads s_r from LDS
      if (wave == 0)
#pragma unroll
        for (int o = 0; o < TH; o += 4) *(f32x4*)(srl + lane * TH + o) = f32x4{sr[o], sr[o + 1], sr[o + 2], sr[o + 3]};
      __syncthreads();
    }
    for (int c = 0; c < a.nch; c++) store(c);
  } else {
  stage(0, 0, 0);
  // reference: packed rows y0-R .. y0+TH+R-1 in registers; its centred window
  // sums Sr' and 1/sqrt(var_r) from them (dot4 with ones / with itself)
  const long zo = (long)a.z[ref] * Pv;
  const int xc = min(x, W - 1);
  unsigned qlo[NR], qhi[NR];
  int rsum[NR];
#pragma unroll
  for (int k = 0; k < NR; k++) {
    const uint2 v = pk[zo + pair_index(min(max(y0 - R + k, 0), H - 1), xc, W)];
    qlo[k] = v.x;
    qhi[k] = v.y & HI_MASK;
    rsum[k] = dot4(qlo[k], 0x01010101u, dot4(qhi[k], 0x01010101u, 0));
  }
  f32x2 rsn[TH / 2];  // -Sr' of output rows (2m, 2m+1)
#pragma unroll
  for (int o = 0; o < TH; o++) {
    int s1 = 0;
#pragma unroll
    for (int k = 0; k < K; k++) s1 += rsum[o + k];
    rsn[o >> 1][o & 1] = -(float)s1;
  }
  // fused: only wave 0 needs s_r (it publishes it in LDS), so the other waves
  // skip the squares and the correctly rounded sqrt + divide of every row
  if (!FUSE || wave == 0) {
    int rsq[NR];
#pragma unroll
    for (int k = 0; k < NR; k++) rsq[k] = dot4(qlo[k], qlo[k], dot4(qhi[k], qhi[k], 0));
#pragma unroll
    for (int o = 0; o < TH; o++) {
      int s1 = 0, s2 = 0;
#pragma unroll
      for (int k = 0; k < K; k++) {
        s1 += rsum[o + k];
        s2 += rsq[o + k];
      }
      const int y = y0 + o;
      const bool valid = x - R >= 0 && x + R < W && y - R >= 0 && y + R < H;
      const int var = NK * s2 - s1 * s1;
      sr[o] = !valid ? __int_as_float(0x7fc00000) : (var != 0 ? 1.0f / sqrtf((float)var) : 0.0f);
    }
  }
  if (FUSE && wave == 0) {
#pragma unroll
    for (int o = 0; o < TH; o += 4) *(f32x4*)(srl + lane * TH + o) = f32x4{sr[o], sr[o + 1], sr[o + 2], sr[o + 3]};
  }
  __syncthreads();

  // one pipeline step t = c * nn + n: prefetch step t+1's bands, then this
  // step's correlations into E.  FIRST (the chunk's first neighbour) assigns
  // E instead of max-ing into it, so no -inf reset of the 8 DPW accumulators
  // per chunk and no max for the first neighbour: v_max_f32 drops a NaN
  // (invalid neighbour window), so max(-inf, x) and x differ only when x is
  // NaN, and a NaN that survives to the store gives the same cost 2 as -inf
  // (both clamp to -1 there), while a later finite x replaces it either way.
  // Only the K = 5 EVEN kernels (horizontal neighbours: the C2 headline) are
  // peeled.  The others keep the flat loop: their second copy of the step
  // spilled at the 128-VGPR cap (fused K = 7 scratch 104 -> 532 bytes, K = 5
  // non-EVEN DPW 4 72 -> 452)
  constexpr bool PEEL = K == 5 && PAR == kParEven;
  auto step = [&](int t, int n, int cprev, auto first) {
    constexpr bool FIRST = decltype(first)::value;
    const int n1 = n + 1 == nn ? 0 : n + 1;
    if (NB == 2 && t + 1 < T) stage(t + 1, n1, (t + 1) & 1);  // prefetch step t+1 while computing t
    if (NB == 1 && t > 0) {  // this step's bands into the one buffer (step 0's: before the loop)
      stage(t, n, 0);
      __syncthreads();  // vmcnt(0): landed, for every wave
    }
    // the previous chunk's costs are written here (its E, before this step
    // overwrites it), after this step's prefetch is issued and a whole step
    // before the barrier's vmcnt(0) (which also waits for stores): the write
    // latency hides behind the compute.  (FUSE: the register fold.)
    if ((FIRST || !PEEL) && cprev >= 0) {
      store(cprev);
      if (!PEEL) reset();
    }
    const u32x4* npk = nbase + (NB == 2 ? (t & 1) * nbuf : 0);
    const u32x4* nst = npk + a.pk_pairs * BW;
    const int ln = lane_now();
    int lvv[2 * DPW];  // one scalar load of this wave's level shifts for step t
#pragma unroll
    for (int i = 0; i < 2 * DPW; i++) lvv[i] = rec[NW * t].lv[i];
    // levels past the end of the last chunk carry in-band dummy shifts: they
    // are computed and dropped at the store, so the loop is straight-line
#pragma unroll
    for (int j = 0; j < DPW; j++) {
      const int colo = lvv[2 * j], rows = lvv[2 * j + 1];
      u32x2 pv[NR];
      read_rows<NR, BW, PAR>(npk + colo + ln, rows & 0xffff, pv);
      // prefix sums over band rows of the horizontal K-tap centred correlation
      // prefix sums biased by kMagic: as floats they are 1.5 * 2^23 + the sum
      // (|sum| < 2^22), so a difference of two is the exact integer window sum
      // as a float -- one v_sub_f32 per row instead of v_sub_u32 + v_cvt
      int ps[NR];
      ps[0] = dot4(qlo[0], pv[0].x, dot4(qhi[0], pv[0].y, kMagicI));
#pragma unroll
      for (int k = 1; k < NR; k++) ps[k] = dot4(qlo[k], pv[k].x, dot4(qhi[k], pv[k].y, ps[k - 1]));
      f32x4 sv[TH / 2];
      read_stat_pairs<TH, BW, PAR>(nst + colo + ln, rows >> 16, sv);
#pragma unroll
      for (int m = 0; m < TH / 2; m++) {
        const int o = 2 * m;
        // Srp' of rows o, o+1 (exact)
        const float f0 = __int_as_float(ps[o + 2 * R]) - (o > 0 ? __int_as_float(ps[o - 1]) : kMagicF);
        const float f1 = __int_as_float(ps[o + 1 + 2 * R]) - __int_as_float(ps[o]);
        const f32x2 f = f32x2{f0, f1};
        const f32x2 xv = __builtin_elementwise_fma(rsn[m], f32x2{sv[m].z, sv[m].w}, f * f32x2{sv[m].x, sv[m].y});
        if (FIRST) {
          E[j][o] = xv.x;
          E[j][o + 1] = xv.y;
        } else {
          E[j][o] = vmax(E[j][o], xv.x);
          E[j][o + 1] = vmax(E[j][o + 1], xv.y);
        }
      }
    }
    __syncthreads();  // step t+1's bands landed (vmcnt 0); this buffer free for t+2
  };
  if (PEEL) {  // chunks outer, neighbours inner, the first neighbour peeled
    int t = 0;
    for (int c = 0; c < a.nch; c++) {
      step(t++, 0, c - 1, std::true_type{});
      for (int n = 1; n < nn; n++) step(t++, n, -1, std::false_type{});
    }
  } else {  // one flat step loop, E reset after each chunk's store
    reset();
    for (int t = 0, n = 0, c = 0; t < T; t++) {
      step(t, n, n == 0 && t > 0 ? c - 1 : -1, std::false_type{});
      if (++n == nn) {
        n = 0;
        c++;
      }
    }
  }
  store(a.nch - 1);
  }
  if (FUSE) {
    // merge the NW waves' partials of each of the tile's 64 x TH pixels; the
    // band buffers are free (every wave passed the loop's last barrier)
    constexpr int TP = TH * 64;
    float* m0 = (float*)smem;
    float* m1 = m0 + NW * TP;
    int* mi = (int*)(m1 + NW * TP);
    if (PKI)
#pragma unroll
      for (int o = 0; o < TH; o++) {
        const unsigned v = (o & 1) ? wi0p[o >> 1] >> 16 : wi0p[o >> 1] & 0xffffu;
        wi0[o] = v == 0xffffu ? -1 : (int)v;
      }
    __syncthreads();
#pragma unroll
    for (int o = 0; o < TH; o++) {
      m0[wave * TP + o * 64 + lane] = wv0[o];
      m1[wave * TP + o * 64 + lane] = wv1[o];
      mi[wave * TP + o * 64 + lane] = wi0[o];
    }
    __syncthreads();
    for (int q = tid; q < TP; q += NW * 64) {
      const int xx = x0 + (q & 63), yy = y0 + (q >> 6);
      // every wave's entries read up front (one LDS latency, not one per
      // wave) and compared without branches, in wave order as before
      float v0s[NW], v1s[NW];
      int is[NW];
#pragma unroll
      for (int w = 0; w < NW; w++) {
        v0s[w] = m0[w * TP + q];
        is[w] = mi[w * TP + q];
        v1s[w] = m1[w * TP + q];
      }
      float bv = v0s[0];
      int bi = is[0];
#pragma unroll
      for (int w = 1; w < NW; w++) {
        const bool tk = (v0s[w] < bv) | ((v0s[w] == bv) & (is[w] >= 0) & (is[w] < bi));
        bv = tk ? v0s[w] : bv;
        bi = tk ? is[w] : bi;
      }
      float c2 = kWtaInit;
#pragma unroll
      for (int w = 0; w < NW; w++) {
        const float v = ((is[w] >= bi - 1) & (is[w] <= bi + 1)) ? v1s[w] : v0s[w];
        c2 = vmin(c2, v);
      }
      if (xx < W && yy < H) {
        const long p = P * ref + (long)yy * W + xx;  // disp / conf of reference r of the launch
        wo.disp[p] = bi >= 0 ? wo.levels[bi] : 0.0f;
        if (wo.conf) wo.conf[p] = (bi < 0 || c2 == kWtaInit) ? 0.0f : c2 - bv;
      }
    }
  }
}

// Host side: the chunk/level shift plan (every roundf of the definition is
// evaluated here, once per distinct configuration) and the launch.
struct NccPlan {
  std::vector<int32_t> table;  // NccRec [nchunks][nn][NW waves] as int32
  int band_w = 0, pk_pairs = 0, st_pairs = 0;
  bool even = true;  // every level's band rows start on a pair boundary (kParEven)
  bool odd = true;   // every pk start odd, every stats start even (kParOdd)
  int par() const { return even ? kParEven : odd ? kParOdd : kParMixed; }
};

inline int floor_half(int v) { return v >> 1; }  // arithmetic: floor(v / 2)

template <int K, int TH, int DPW, int NW>
NccPlan make_plan(const float* levels, int D, int nn, const float* fdx, const float* fdy, float bl) {
  constexpr int R = K / 2, NR = TH + 2 * R, DC = NW * DPW;
  static_assert(DPW <= 8, "NccRec holds 8 levels per wave");
  constexpr int RW = sizeof(NccRec) / 4;
  const int nch = (D + DC - 1) / DC;
  NccPlan p;
  p.table.assign((size_t)nch * nn * NW * RW, 0);
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
      for (int w = 0; w < NW; w++) {
        int32_t* e = p.table.data() + (((size_t)c * nn + n) * NW + w) * RW;
        e[0] = txmax;
        e[1] = tymax;
        e[2] = bhp;
        e[3] = shp | ((txmax - txmin) << 16);  // stage(): pieces of 64 columns covering 64 + span
        for (int j = 0; j < DPW; j++) {
          const int dl = c * DC + w + NW * j;
          if (dl >= D) {  // dummy level past the end: the band origin's even rows
            e[4 + 2 * j] = 0;
            e[5 + 2 * j] = pr | (sr << 16);  // same parity as the real levels'
            continue;
          }
          const int ty = ty_of(dl, n);
          e[4 + 2 * j] = txmax - tx_of(dl, n);
          e[5 + 2 * j] = (pr + tymax - ty) | ((sr + tymax - ty) << 16);
          if (((pr + tymax - ty) | (sr + tymax - ty)) & 1) p.even = false;
          if (!((pr + tymax - ty) & 1) || ((sr + tymax - ty) & 1)) p.odd = false;
        }
      }
      spx = std::max(spx, txmax - txmin);
      p.pk_pairs = std::max(p.pk_pairs, bhp);
      p.st_pairs = std::max(p.st_pairs, shp);
    }
  p.band_w = 64 + spx;  // columns per pair row (stage() never writes past them)
  return p;
}

template <int K, int TH, int DPW, int NW, int BW, int PAR, int NB = 2>
int launch_ncc_bw(mvs_ctx* ctx, const uint2* stats, const uint2* pk, const NccRec* plan, NccArgs& a, float* vol,
                  const WtaOut& wo, size_t lds) {
  hipStream_t s = ctx->stream;
  const int variant[8] = {K, TH, DPW, NW, BW, PAR, vol ? 0 : 1, NB};
  std::copy(variant, variant + 8, ctx->ncc_last);
  constexpr int DC = NW * DPW;
  a.tiles_x = (a.W + 63) / 64;
  a.ntiles = a.tiles_x * ((a.H + TH - 1) / TH);
  a.tiles_per_xcd = (a.nref * a.ntiles + 7) / 8;
  a.nch = (a.D + DC - 1) / DC;
  dim3 g(8 * a.tiles_per_xcd);
  auto kern = vol ? k_ncc_volume<K, TH, DPW, NW, BW, PAR, false, NB> : k_ncc_volume<K, TH, DPW, NW, BW, PAR, true, NB>;
  if (!vol) lds = std::max(lds, (size_t)3 * 4 * NW * TH * 64) + 4 * TH * 64;  // WTA partials; + s_r [64][TH]
  MVS_HIP(raise_lds(ctx, (const void*)kern, lds), "hipFuncSetAttribute(ncc lds)");
  const auto ev = vol ? std::pair<hipEvent_t, hipEvent_t>{nullptr, nullptr} : kernel_events(ctx);  // (the fused sweep only)
  hipExtLaunchKernelGGL(kern, g, dim3(NW * 64), lds, s, ev.first, ev.second, 0, stats, pk, plan, a, vol, wo);
  MVS_LAUNCH_CHECK(vol ? "k_ncc_volume" : "k_ncc_volume (fused WTA)");
  return 0;
}

// One reference view's variant: its shift plan for (K, TH = 8, DPW, NW) and
// the band pair-row stride, if its double-buffered bands fit `cap` bytes of LDS.
struct NccChoice {
  int dpw = 0, nw = 0, bwt = 0, nb = 2;  // nb: band buffers (k_ncc_volume's NB)
  size_t cap = 0;
  NccPlan plan;
};
template <int K, int DPW, int NW>
bool try_plan(const mvs_ctx* ctx, const float* levels, int D, int nn, const float* fdx, const float* fdy, float bl,
              size_t cap, NccChoice& o, int nb = 2) {
  NccPlan p = make_plan<K, 8, DPW, NW>(levels, D, nn, fdx, fdy, bl);
  // the band's pair-row stride is the template BW: the smallest of 64 / 80 /
  // 96 / 128 / 192 / 256 holding band_w, or a wider one forced through
  // mvs_set_ncc_variant.  A vertical-only list needs 64, a diagonal or
  // horizontal neighbour 64 + the chunk's shift range (C4: 71 / 79 / 95)
  const int bw = std::max(p.band_w, ctx->ncc_bw);
  const int bwt = bw <= 64 ? 64 : bw <= 80 ? 80 : bw <= 96 ? 96 : bw <= 128 ? 128 : bw <= 192 ? 192 : 256;
  const size_t lds = nb * 16 * (size_t)(p.pk_pairs + p.st_pairs) * bwt;
  if (lds > cap || bw > 256) return false;
  o.nb = nb;
  o.dpw = DPW;
  o.nw = NW;
  o.bwt = bwt;
  o.cap = cap;
  o.plan = std::move(p);
  return true;
}
// waves per workgroup and levels per wave: MVS_NCC_NW (4|8), MVS_NCC_DPW
// (1|2|4), or the context's override (mvs_set_ncc_variant), tried first.
// Then the widest variant whose double-buffered bands leave room for two
// workgroups per CU (vertical shifts grow the bands: fewer levels per step
// then beat a single resident workgroup), then any that fits the LDS.
template <int K>
bool choose_variant(const mvs_ctx* ctx, const float* levels, int D, int nn, const float* fdx, const float* fdy,
                    float bl, NccChoice& o) {
  static const int dpw_env = [] {
    const char* e = getenv("MVS_NCC_DPW");
    return e ? atoi(e) : 4;
  }();
  static const int nw_env = [] {
    const char* e = getenv("MVS_NCC_NW");
    return e ? atoi(e) : 8;
  }();
  const int dpw_pref = ctx->ncc_dpw ? ctx->ncc_dpw : dpw_env;
  const int nw_pref = ctx->ncc_nw ? ctx->ncc_nw : nw_env;
  bool ok = false;
#define MVS_NCC_TRY(DD, WW) \
  if (!ok) ok = try_plan<K, DD, WW>(ctx, levels, D, nn, fdx, fdy, bl, cap, o);
  if (ctx->ncc_nw || ctx->ncc_dpw) {  // a forced variant is tried first, at the full LDS
    const size_t cap = (size_t)160 * 1024;
    if (nw_pref >= 8 && dpw_pref >= 4) {
      MVS_NCC_TRY(4, 8)
    } else if (nw_pref >= 8 && dpw_pref >= 2) {
      MVS_NCC_TRY(2, 8)
    } else if (dpw_pref >= 4) {
      MVS_NCC_TRY(4, 4)
    } else if (dpw_pref >= 2) {
      MVS_NCC_TRY(2, 4)
    } else {
      MVS_NCC_TRY(1, 4)
    }
  }
  // A K = 5 list whose double-buffered 32-level bands miss two workgroups per
  // CU (C4's 5-NN lists: vertical and diagonal bands) tries them single-
  // buffered before halving the chunk (k_ncc_volume's NB), and a list too
  // tall even for that (C4's corner views: a neighbour two rows away) takes
  // 8 waves x 2 levels single-buffered before 4 waves: C4 step 48.1 -> 46.6 ms,
  // fused sweep 0.71 -> 0.66 ms per view (interleaved A/B,
  // profiles/r04/abenv_c4_nb1_corner.txt).  MVS_NCC_NB=2 (read per call)
  // keeps the double-buffered forms.
  const char* nbe = getenv("MVS_NCC_NB");
  const bool nb1 = K == 5 && !(nbe && atoi(nbe) == 2);
  for (size_t cap : {(size_t)80 * 1024, (size_t)160 * 1024}) {
    if (nw_pref >= 8 && dpw_pref >= 4) MVS_NCC_TRY(4, 8)
    if (nb1 && cap <= 80 * 1024 && nw_pref >= 8 && dpw_pref >= 4 && !ok)
      ok = try_plan<K, 4, 8>(ctx, levels, D, nn, fdx, fdy, bl, cap, o, 1);
    if (nw_pref >= 8 && dpw_pref >= 2) MVS_NCC_TRY(2, 8)
    if (nb1 && cap <= 80 * 1024 && nw_pref >= 8 && dpw_pref >= 2 && !ok)  // (C4's corner views)
      ok = try_plan<K, 2, 8>(ctx, levels, D, nn, fdx, fdy, bl, cap, o, 1);
    if (dpw_pref >= 4) MVS_NCC_TRY(4, 4)
    if (dpw_pref >= 2) MVS_NCC_TRY(2, 4)
    MVS_NCC_TRY(1, 4)
  }
#undef MVS_NCC_TRY
  return ok;
}

template <int K, int DPW, int NW, int PAR, int NB = 2>
int launch_bw(mvs_ctx* ctx, int bwt, const uint2* stats, const uint2* pk, const NccRec* plan, NccArgs& a, float* vol,
              const WtaOut& wo, size_t lds) {
  if (bwt == 64) return launch_ncc_bw<K, 8, DPW, NW, 64, PAR, NB>(ctx, stats, pk, plan, a, vol, wo, lds);
  if (bwt == 80) return launch_ncc_bw<K, 8, DPW, NW, 80, PAR, NB>(ctx, stats, pk, plan, a, vol, wo, lds);
  if (bwt == 96) return launch_ncc_bw<K, 8, DPW, NW, 96, PAR, NB>(ctx, stats, pk, plan, a, vol, wo, lds);
  if (bwt == 128) return launch_ncc_bw<K, 8, DPW, NW, 128, PAR, NB>(ctx, stats, pk, plan, a, vol, wo, lds);
  if (bwt == 192) return launch_ncc_bw<K, 8, DPW, NW, 192, PAR, NB>(ctx, stats, pk, plan, a, vol, wo, lds);
  return launch_ncc_bw<K, 8, DPW, NW, 256, PAR, NB>(ctx, stats, pk, plan, a, vol, wo, lds);
}
// the parity-specific kernels only where they occur: kParEven for K = 5
// (horizontal bands, R = 2), kParOdd for K = 7 (R = 3)
template <int K, int DPW, int NW>
int launch_bw_par(mvs_ctx* ctx, int bwt, int par, const uint2* stats, const uint2* pk, const NccRec* plan,
                  NccArgs& a, float* vol, const WtaOut& wo, size_t lds, int nb) {
  constexpr int KPAR = K == 5 ? kParEven : kParOdd;
  if constexpr (K == 5 && DPW >= 2 && NW == 8)  // single-buffered bands: C4's tall 5-NN bands (any parity)
    if (nb == 1) return launch_bw<K, DPW, NW, kParMixed, 1>(ctx, bwt, stats, pk, plan, a, vol, wo, lds);
  if (par == KPAR && !ctx->ncc_general) return launch_bw<K, DPW, NW, KPAR>(ctx, bwt, stats, pk, plan, a, vol, wo, lds);
  return launch_bw<K, DPW, NW, kParMixed>(ctx, bwt, stats, pk, plan, a, vol, wo, lds);
}
template <int K>
int launch_variant(mvs_ctx* ctx, const NccChoice& c, int bwt, int par, const uint2* stats, const uint2* pk,
                   const NccRec* plan, NccArgs& a, float* vol, const WtaOut& wo, size_t lds) {
  if (c.dpw == 4 && c.nw == 8) return launch_bw_par<K, 4, 8>(ctx, bwt, par, stats, pk, plan, a, vol, wo, lds, c.nb);
  if (c.dpw == 2 && c.nw == 8) return launch_bw_par<K, 2, 8>(ctx, bwt, par, stats, pk, plan, a, vol, wo, lds, c.nb);
  if (c.dpw == 4) return launch_bw_par<K, 4, 4>(ctx, bwt, par, stats, pk, plan, a, vol, wo, lds, c.nb);
  if (c.dpw == 2) return launch_bw_par<K, 2, 4>(ctx, bwt, par, stats, pk, plan, a, vol, wo, lds, c.nb);
  return launch_bw_par<K, 1, 4>(ctx, bwt, par, stats, pk, plan, a, vol, wo, lds, c.nb);
}

}  // namespace

// window planes of views [z0, z1) of a V-view box buffer
int launch_box_stats(hipStream_t s, const uint8_t* l8, int V, int W, int H, int K, int32_t* box, int z0, int z1) {
  if (z1 <= z0) return 0;
  const int Hp = H + (H & 1);
  uint2* stats = (uint2*)box;
  uint2* pk = stats + (long)V * W * Hp;
  dim3 g((W + BS_TW - 1) / BS_TW, (Hp + BS_TH - 1) / BS_TH, z1 - z0);
  if (K == 5)
    hipLaunchKernelGGL(k_box_stats<2>, g, dim3(256), 0, s, l8, W, H, z0, stats, pk);
  else
    hipLaunchKernelGGL(k_box_stats<3>, g, dim3(256), 0, s, l8, W, H, z0, stats, pk);
  MVS_LAUNCH_CHECK("k_box_stats");
  return 0;
}

// Reference views [z0, z1): each view's variant is chosen on its own shifts;
// runs of consecutive views with the same (DPW, NW) whose merged bands still
// fit every member's LDS cap share one launch (up to kMaxRef views, fused
// sweep only: a cost volume holds one view), with the widest band stride and
// a parity-specific kernel only when every member has that parity -- the same arithmetic,
// one kernel boundary (~11 us between two of these launches) per run.
int launch_ncc_refs(mvs_ctx* ctx, int V, int W, int H, const int32_t* box, const float* levels_host, int D,
                    const int* vs_host, const int* sn_host, int aw, float bl, int K, int z0, int z1, float* vol,
                    const float* levels_dev, float* disp, float* conf) {
  if (!vol && (!levels_dev || !disp)) return arg_fail("fused NCC sweep needs levels and disp");
  if (vol && z1 - z0 != 1) return arg_fail("the NCC cost volume holds one reference view");
  if (W < 2) return arg_fail("NCC sweep needs W >= 2");
  if (K != 5 && K != 7) return arg_fail("NCC window must be 5 or 7");
  if (!vol && D > 65535) return arg_fail("fused NCC sweep: at most 65535 levels");  // K = 7 packs levels in 16 bits
  const int n = z1 - z0;
  if (n <= 0) return 0;
  std::vector<NccChoice> ch(n);
  std::vector<std::array<int, kMaxNbr>> views(n);
  // the matrix-core form (k_ncc_mfma) for fused K = 5 views: horizontal lists
  // (every vertical shift 0) in 32-level double-buffered chunks; lists with
  // vertical / diagonal neighbours (VERT) in the first of 32-level double- /
  // single-buffered, 16-level double- / single-buffered chunks whose bands
  // leave two workgroups per CU (80 KB).  MVS_NCC_MFMA=0 (read per call) or a
  // forced variant (mvs_set_ncc_variant) keeps the scalar kernels.  VERT
  // lists take the matrix-core form by default (MVS_NCC_MFMA_V unset or 1:
  // the launcher's choice under two workgroups per CU; 22 | 21 | 12 | 11:
  // that form; 0: the scalar kernels).  Since its finish went scalar f32 it
  // runs C4's 5-NN lists ~1 % faster than the scalar kernels
  // K = 7 (C5): horizontal lists in 16-level chunks (its 2 x 8-pixel blocks'
  // operands take 32 VGPRs); MVS_NCC_MFMA7=0 keeps the scalar kernels (A/B)
  const char* mfe = getenv("MVS_NCC_MFMA");
  const char* mfv = getenv("MVS_NCC_MFMA_V");
  const char* mf7 = getenv("MVS_NCC_MFMA7");
  // (its band DMA addresses one view's plane by 32-bit byte offsets)
  const bool mf_on = !vol && (K == 5 || (K == 7 && !(mf7 && atoi(mf7) == 0))) && !(mfe && atoi(mfe) == 0) &&
                     !ctx->ncc_nw && !ctx->ncc_dpw && !ctx->ncc_general && !ctx->ncc_bw &&
                     (long)W * (H + (H & 1)) * 8 < 0x7fffffffL;
  const int mfv_form = mfv ? atoi(mfv) : 1;  // 0: off, 1: automatic (default), else the form
  std::vector<char> mf(n, 0);
  std::vector<NccPlanM> mplan(n);
  std::vector<int> mnb(n, 2);
  for (int r = 0; r < n; r++) {
    const int z = z0 + r, nn = sn_host[z];
    if (nn > kMaxNbr) return arg_fail("NCC sweep supports at most 16 neighbours per reference view");
    float fdx[kMaxNbr], fdy[kMaxNbr];
    const int rx = z % aw, ry = z / aw;
    bool horiz = true;
    for (int k = 0; k < nn; k++) {
      const int v = vs_host[V * z + k];
      if (v < 0 || v >= V) return arg_fail("view_subset entry out of range");
      views[r][k] = v;
      fdx[k] = (float)(v % aw - rx);
      fdy[k] = (float)(v / aw - ry);
      if (fdy[k] != 0.0f) horiz = false;
    }
    if (mf_on && horiz && nn > 0) {
      const int ndb = K == 5 ? 2 : 1;
      mplan[r] = make_plan_mfma(levels_host, D, nn, fdx, fdy, bl, ndb, K);
      // the run keeps every step's level offsets in LDS (tmax = chunks x
      // neighbours): past the 160 KB of a CU (large D with many neighbours)
      // the scalar kernels take the view
      const int tm = ((D + 16 * ndb - 1) / (16 * ndb)) * nn;
      if (mplan[r].band_w <= 192 && mfma_lds_bytes(mplan[r], mplan[r].band_w, 2, tm, D) <= (size_t)160 * 1024) {
        mf[r] = 1;
        continue;
      }
    }
    if (mf_on && K == 5 && !horiz && nn > 0 && mfv_form != 0) {
      static const int forms[4][2] = {{2, 2}, {2, 1}, {1, 2}, {1, 1}};
      for (const auto& f : forms) {
        const bool forced = mfv_form > 1;
        if (forced && mfv_form != 10 * f[0] + f[1]) continue;
        NccPlanM pm = make_plan_mfma(levels_host, D, nn, fdx, fdy, bl, f[0]);
        const int tm = ((D + 16 * f[0] - 1) / (16 * f[0])) * nn;
        const size_t cap = forced ? (size_t)160 * 1024 : (size_t)80 * 1024;
        if (pm.band_w <= 128 && mfma_lds_bytes(pm, pm.band_w, f[1], tm, D) <= cap) {
          mplan[r] = std::move(pm);
          mnb[r] = f[1];
          mf[r] = 1;
          break;
        }
      }
      if (mf[r]) continue;
    }
    const bool ok = K == 5 ? choose_variant<5>(ctx, levels_host, D, nn, fdx, fdy, bl, ch[r])
                           : choose_variant<7>(ctx, levels_host, D, nn, fdx, fdy, bl, ch[r]);
    if (!ok) return arg_fail("NCC sweep: neighbour shifts too large for the LDS band");
  }
  const uint2* stats = (const uint2*)box;
  const uint2* pk = stats + (long)V * W * (H + (H & 1));
  constexpr int RW = sizeof(NccRec) / 4;
  const long P = (long)W * H;
  // MVS_NCC_RUN (read per call): views per launch at most (A/B; default kMaxRef)
  const char* re = getenv("MVS_NCC_RUN");
  const int maxrun = re ? std::max(1, std::min(kMaxRef, atoi(re))) : kMaxRef;
  for (int i = 0; i < n;) {
    if (mf[i]) {  // a run of matrix-core views of one form: one launch, the widest band, the tallest bands
      const bool vert = mplan[i].vert;
      const int ndb = mplan[i].ndb, nb = mnb[i];
      int j = i, bw = 0, tmax = 0;
      NccArgs a{};
      a.W = W;
      a.H = H;
      a.D = D;
      std::vector<int32_t> table;
      NccPlanM run;  // the run's band extents (LDS check)
      run.ndb = ndb;
      run.vert = vert;
      while (j < n && mf[j] && j - i < maxrun && mplan[j].vert == vert && mplan[j].ndb == ndb && mnb[j] == nb) {
        const int z = z0 + j;
        run.pk_pairs = std::max(run.pk_pairs, mplan[j].pk_pairs);
        run.st_pairs = std::max(run.st_pairs, mplan[j].st_pairs);
        const int bw2 = std::max(bw, mplan[j].band_w);
        const int tm2 = std::max(tmax, ((D + 16 * ndb - 1) / (16 * ndb)) * sn_host[z]);
        if (j > i && mfma_lds_bytes(run, bw2, nb, tm2, D) > (size_t)(vert ? 80 : 160) * 1024) break;
        bw = bw2;
        tmax = tm2;
        a.z[j - i] = z;
        a.nn[j - i] = sn_host[z];
        a.plan[j - i] = (int)(table.size() / 32);  // 128-B NccMRec records
        for (int k = 0; k < sn_host[z]; k++) a.view[j - i][k] = views[j][k];
        // each record's neighbour plane as a byte offset (words 22, 23): the
        // kernel rebases its band DMA on it with no per-step multiply
        const size_t r0 = table.size();
        table.insert(table.end(), mplan[j].table.begin(), mplan[j].table.end());
        for (size_t rr = r0; rr < table.size(); rr += 32) {
          const int nloc = (int)((rr - r0) / 32) % sn_host[z];
          const unsigned long long off = (unsigned long long)views[j][nloc] * (unsigned long long)W *
                                         (unsigned long long)((H + 1) >> 1) * 16ull;  // Pv uint2 = 16 B per (pair row, column)
          table[rr + 22] = (int32_t)(off & 0xffffffffull);
          table[rr + 23] = (int32_t)(off >> 32);
          a.txmax_all = std::max(a.txmax_all, table[rr]);
        }
        j++;
      }
      a.nref = j - i;
      a.pk_pairs = 0;
      a.st_pairs = 0;
      for (int r = i; r < j; r++) {
        a.pk_pairs = std::max(a.pk_pairs, mplan[r].pk_pairs);
        a.st_pairs = std::max(a.st_pairs, mplan[r].st_pairs);
      }
      int rc = 0;
      const int32_t* dev = plan_upload(ctx, table, &rc);
      if (rc) return rc;
      const WtaOut wo{levels_dev, disp + P * i, conf ? conf + P * i : nullptr};
      rc = launch_ncc_mfma(ctx, stats, pk, dev, a, wo, bw, tmax, vert, ndb, nb, K);
      if (rc) return rc;
      i = j;
      continue;
    }
    int bwt = ch[i].bwt, pkp = ch[i].plan.pk_pairs, stp = ch[i].plan.st_pairs;
    int par = ch[i].plan.par();
    size_t cap = ch[i].cap;
    int j = i + 1;
    while (!vol && j < n && !mf[j] && j - i < maxrun && ch[j].dpw == ch[i].dpw && ch[j].nw == ch[i].nw &&
           ch[j].nb == ch[i].nb) {
      const int b2 = std::max(bwt, ch[j].bwt);
      const int p2 = std::max(pkp, ch[j].plan.pk_pairs), s2 = std::max(stp, ch[j].plan.st_pairs);
      const size_t c2 = std::min(cap, ch[j].cap);
      if (ch[i].nb * 16 * (size_t)(p2 + s2) * b2 > c2) break;
      bwt = b2;
      pkp = p2;
      stp = s2;
      cap = c2;
      if (ch[j].plan.par() != par) par = kParMixed;
      j++;
    }
    NccArgs a{};
    a.W = W;
    a.H = H;
    a.D = D;
    // (band DMA by 32-bit buffer offsets; MVS_NCC_PLANE32=0, read per call: the 64-bit addresses, A/B)
    const char* p32 = getenv("MVS_NCC_PLANE32");
    a.plane32 = (long)W * (H + (H & 1)) * 8 < 0x7fffffffL && !(p32 && atoi(p32) == 0);
    a.nref = j - i;
    a.pk_pairs = pkp;
    a.st_pairs = stp;
    std::vector<int32_t> table;
    for (int r = i; r < j; r++) {
      const int z = z0 + r;
      a.z[r - i] = z;
      a.nn[r - i] = sn_host[z];
      a.plan[r - i] = (int)(table.size() / RW);
      for (int k = 0; k < sn_host[z]; k++) a.view[r - i][k] = views[r][k];
      table.insert(table.end(), ch[r].plan.table.begin(), ch[r].plan.table.end());
    }
    int rc = 0;
    const int32_t* dev = plan_upload(ctx, table, &rc);
    if (rc) return rc;
    const WtaOut wo{levels_dev, disp ? disp + P * i : nullptr, conf ? conf + P * i : nullptr};
    const size_t lds = ch[i].nb * 16 * (size_t)(pkp + stp) * bwt;
    rc = K == 5 ? launch_variant<5>(ctx, ch[i], bwt, par, stats, pk, (const NccRec*)dev, a, vol, wo, lds)
                : launch_variant<7>(ctx, ch[i], bwt, par, stats, pk, (const NccRec*)dev, a, vol, wo, lds);
    if (rc) return rc;
    i = j;
  }
  return 0;
}

int launch_ncc_volume(mvs_ctx* ctx, int V, int W, int H, const int32_t* box, const float* levels_host, int D,
                      const int* vs_host, const int* sn_host, int aw, float bl, int K, int z, float* vol,
                      const float* levels_dev, float* disp, float* conf) {
  return launch_ncc_refs(ctx, V, W, H, box, levels_host, D, vs_host, sn_host, aw, bl, K, z, z + 1, vol, levels_dev,
                         disp, conf);
}

}  // namespace mvs
