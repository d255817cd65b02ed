// Matrix-core form of the fused NCC sweep + WTA (K = 5): the definition and
// the outputs are ncc.hip's (k_ncc_volume with FUSE), bit for bit;
// launch_ncc_refs (ncc.hip) picks it per reference view.  See the comment at
// NccMRec for the formulation.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "ncc_common.h"

#ifndef MVS_MFMA_SPLIT
#define MVS_MFMA_SPLIT 1
#endif

namespace mvs {
namespace ncc {
namespace {

// ---- matrix-core form of the fused sweep (K = 5) ----
//
// The correlation Srp'(x, y, d) = sum_{j, i} r'(x+i, y+j) p'(x+i-tx(d), y+j)
// as a GEMM whose output lands in the SAME (pixel, level) layout for every
// neighbour, so the neighbour maximum stays in registers:
//   C[m][n] = sum_k A[m][k] B[k][n],   m = (xx, yy) of a 4 x 4 pixel block,
//   n = level d0 + n of a 16-level block, k = (row, column) of the block's
//   8 x 8 window footprint (rows y0b-2 .. y0b+5, columns x0b-2 .. x0b+5);
//   A[m][k] = r'(column, row) where the tap lies in pixel m's 5 x 5 window, else 0
//             (the REFERENCE, banded: built once per tile, reused for every
//             neighbour and level);
//   B[k][n] = p'(column - tx(d0+n), row)   (the neighbour: its row-pair pk entry
//             at column x0b - tx, i.e. one aligned 16-byte LDS read per lane).
// k = 64 = 4 row pairs x 16 bytes is exactly one v_mfma_i32_16x16x64_i8 and
// exactly the pk plane's row-pair entry, so a lane's B operand for row pair g
// is ONE ds_read_b128 from the band the LDS-DMA stages anyway.  The MFMA's
// accumulator starts at the bits of 1.5 * 2^23: read as a float the result is
// 1.5 * 2^23 + Srp' exactly (|Srp'| < 2^22), one v_sub_f32 per cell (scalar
// f32 throughout the finish and fold: v_pk_*_f32 measured slower, C2 -1.3 %,
// C5 -3.2 %, profiles/r06/ab_scalar_f32_finish.txt).
// Per lane the output is C[4 (l >> 4) + r][l & 15]: pixel column xx = l >> 4,
// rows yy = r = 0..3, level l & 15 -- a fixed pixel column and level per lane,
// so the neighbour stats (a, b of rows y0b..y0b+3 at column x - tx) are two
// ds_read_b128 per lane, and the finish x = fma(-Sr', b, Srp' a) and the
// maximum are the scalar kernel's operations in the same order (bit-identical).
// Per wave and neighbour step: 4 pixel blocks (8 columns x 8 rows) x 2 level
// blocks = 8 MFMAs for 2,048 view-cells, against 192 dot4 of the scalar form.
// Lane l holds the levels of class l & 15 (16 apart): the fold keeps the same
// (smallest, its level, second smallest) triple per cell, and the 16 classes
// of a pixel are merged through LDS as the scalar kernel merges its waves.
//
// VERT (lists with vertical / diagonal neighbours, C4): level j also shifts
// rows by ty(j), so its footprint starts o_j = tymax - ty(j) + (tymax & 1)
// rows into the band (the pk and stats bands start o_j's parity apart from
// a pair boundary alike).  At an odd o_j a lane's two footprint rows (and a
// pixel's stats rows) straddle two band pair entries: the B operand is two
// ds_read_b64 (row 2g + o_j, row 2g + o_j + 1) and the stats four (a, b)
// pairs, per-lane addresses fixed for the step -- the MFMA and the finish
// are unchanged.  The bands are staged per step (their rows depend on the
// step's tymax), 16 NDB levels per chunk.
struct alignas(128) NccMRec {
  int txmax, tymax;  // band origin, as NccRec
  int bhp, shp;      // pk pair rows to stage; stats pair rows (bits 0..7) | the stats bank shift (signed,
                     // bits 8..15) | column span << 16 | the odd pk rows' bank shift (signed) << 24
  int colo[16];      // 32 x int16: per level j of the chunk, txmax - tx(j) (band column of reference column x0)
                     // | o_j << 8 (VERT: band row of the level's footprint)
  int pad0[2];
  unsigned off_lo, off_hi;  // the neighbour's plane: byte offset from the stack's first (set by the launcher)
  int pad[8];
};
static_assert(sizeof(NccMRec) == 128, "one 128-B record per (chunk, neighbour)");
typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr int kMfMergeStride = 257;  // LDS merge rows: 256 pixels + 1 (16 classes on distinct banks)

// A tile is 64 columns x 8 rows: a wave owns 8 columns x 8 rows = 4 pixel
// blocks (K = 5: 4 x 4 pixels, one MFMA per level block; K = 7: 2 columns x
// 8 rows, whose 8-column x 16-row footprint is 8 row pairs = two MFMAs, the
// second accumulating onto the first).  TAIL: D % DC != 0, the last chunk carries dummy levels past the
// end.  NDB: 16-level blocks per chunk (DC = 16 NDB levels per step).  NB:
// band buffers (2: step t+1's bands land while step t computes; 1: staged at
// the start of each step, the other resident workgroup computing meanwhile).
// DBG (timing probe only, MVS_NCC_MFMA_DBG): 1 skips the MFMAs and the
// finish (band DMA, barriers, fold and merge stay), 2 skips the band DMA
template <int K, int BW, bool TAIL, bool VERT, int NDB, int NB, int DBG = 0>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void k_ncc_mfma(
    const uint2* __restrict__ stats, const uint2* __restrict__ pk, const NccMRec* __restrict__ plan, NccArgs a,
    WtaOut wo) {
  static_assert(NDB == 1 || NDB == 2, "one or two 16-level blocks per chunk");
  static_assert(K == 5 || K == 7, "5 x 5 or 7 x 7 windows");
  static_assert(K == 5 || !VERT, "K = 7: horizontal lists only");
  static_assert(VERT || NB == 2 || NB == 3, "the horizontal form is double- or triple-buffered");
  static_assert(VERT || NDB == (K == 5 ? 2 : 1), "horizontal chunks: 32 levels (K = 5), 16 (K = 7: A takes 32 VGPRs)");
  constexpr int R = K / 2, NW = 8, TH = 8, DC = 16 * NDB, NK = K * K;
  // pixel blocks per wave: XB across (BXW columns each) x NYB down; MF MFMAs per block and level block
  constexpr int XB = K == 5 ? 2 : 4, NYB = K == 5 ? TH / 4 : 1, NBL = XB * NYB, MF = K == 5 ? 1 : 2;
  constexpr int BXW = 8 / XB;
  // band row pitch: BW + 1 columns of 16 B, so a lane group's B reads in two
  // rows (row pairs g, g + 1) fall on different banks when the shift per level
  // is even (|dx| = 2: conflict-free instead of 2-way)
  constexpr int BWP = BW + 1;
  constexpr bool SPLIT = MVS_MFMA_SPLIT;
  extern __shared__ __align__(16) uint8_t smem[];
  const int nbuf = (a.pk_pairs + a.st_pairs) * BWP;  // uint4 per neighbour buffer
  u32x4* nbase = (u32x4*)smem;                      // 2 x {npk[pk_pairs][BW], nst[st_pairs][BW]}
  const int band_bytes = max(NB * nbuf * 16, 3 * 16 * kMfMergeStride * 4);
  float* rsn_l = (float*)(smem + band_bytes);  // [64][TH] -Sr' of the tile's pixels (column-major)
  float* srl = rsn_l + 64 * TH;                 // [64][TH] s_r
  short* colo_l = (short*)(srl + 64 * TH);      // [T][DC] band column (| row) offsets per step and level

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int W = a.W, H = a.H;
  const int Hp2 = (H + 1) >> 1;
  const long Pv = (long)W * Hp2 * 2;
  const long P = (long)W * H;
  const int bid = blockIdx.x, grp = bid & 7;  // XCD-aware tile map, as k_ncc_volume
  const int tg = grp * a.tiles_per_xcd + (bid >> 3);
  if (tg >= a.ntiles * a.nref) return;
  const int ref = tg / a.ntiles, tile = tg - ref * a.ntiles;
  const int x0 = (tile % a.tiles_x) * 64;
  const int y0 = (tile / a.tiles_x) * TH;  // even
  const int nn = a.nn[ref], T = a.nch * nn;
  const NccMRec* rec = plan + a.plan[ref];

  // LDS-DMA staging of step t's bands (k_ncc_volume's stage, one record per
  // step).  Horizontal lists: every step's band rows are the same image rows,
  // so wave w stages pk pair row w (w < bhp) and stats pair row w (w < shp),
  // whose clamped row offsets are computed once per tile.  VERT: the rows
  // start at the step's tymax, the waves take the pair rows in turn
  // pk band: K = 5 rows y0 - 2 .. y0 + TH + 1 (pair (y0 - 2) / 2 on); K = 7 the
  // 8 pairs from (y0 - 4) / 2 (rows y0 - 4 .. y0 + TH + 3: every block's
  // 16-row footprint, its first and last rows masked off in A)
  const int bhp = K == 5 ? (TH + 4) / 2 : (TH + 8) / 2, shp = TH / 2;
  const long pk_row = 2L * W * min(max((y0 >> 1) - (K == 5 ? 1 : 2) + wave, 0), Hp2 - 1);
  const long st_row = 2L * W * min(max(y0 / 2 + wave, 0), Hp2 - 1);
  // Horizontal lists: a step's scalars (band origin, column span, neighbour
  // view) are loaded two steps ahead and carried, so no step waits on a
  // scalar load; its DMA goes through buffer descriptors rebased per step
  // (base = the neighbour's plane row, 32-bit lane offsets: the clamped
  // column x 16 B), no per-lane 64-bit address arithmetic.
  struct StepInfo {
    int tx, shp;      // raw record words: nothing computed on them until they are used
    unsigned lo, hi;  // the neighbour plane's byte offset
  };
  auto load_info = [&](int t, int n) -> StepInfo {
    const NccMRec& e = rec[t];
    return StepInfo{e.txmax, e.shp, e.off_lo, e.off_hi};
  };
  const int lane_x = x0 + lane;
  auto stage_h = [&](const StepInfo& e, int b) {
    if (DBG == 2) return;
    const int span = (e.shp >> 16) & 0xff, nblk = (span + 127) >> 6;
    const unsigned long long vo = (unsigned long long)e.hi << 32 | e.lo;
    // odd pk pair rows land sh columns along, and (K = 7) stats pair rows 2, 3
    // st columns along (the step's bank shifts, see step())
    u32x4* npk = nbase + b * nbuf + ((wave & 1) ? (e.shp >> 24) : 0);
    u32x4* nst = nbase + b * nbuf + a.pk_pairs * BWP + ((K == 7 && wave >= 2) ? ((e.shp << 16) >> 24) : 0);
    // the wave's roles (pk row w < bhp, stats row w < shp) decided once per step, not per piece
    if (wave < shp) {
      const __amdgpu_buffer_rsrc_t rp =
          __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)pk + vo + 8 * pk_row), 0, 16 * W, 0x00020000);
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)stats + vo + 8 * st_row), 0, 16 * W, 0x00020000);
      for (int cb = 0; cb < nblk; cb++) {
        const int c0 = min(cb * 64, span);
        const int voff = 16 * min(max(lane_x - e.tx + c0, 0), W - 1);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rp, (lds_ptr_t)(npk + wave * BWP + c0), 16, voff, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(nst + wave * BWP + c0), 16, voff, 0, 0, 0);
      }
    } else if (wave < bhp) {
      const __amdgpu_buffer_rsrc_t rp =
          __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)pk + vo + 8 * pk_row), 0, 16 * W, 0x00020000);
      for (int cb = 0; cb < nblk; cb++) {
        const int c0 = min(cb * 64, span);
        const int voff = 16 * min(max(lane_x - e.tx + c0, 0), W - 1);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rp, (lds_ptr_t)(npk + wave * BWP + c0), 16, voff, 0, 0, 0);
      }
    }
  };
  auto stage = [&](int t, int n, int b) {
    if (DBG == 2) return;
    const NccMRec& e = rec[t];
    const int span = (e.shp >> 16) & 0xff, nblk = (span + 127) >> 6;  // (VERT: no odd-row shift)
    const long vo = (long)a.view[ref][n] * Pv;
    u32x4* npk = nbase + b * nbuf;
    u32x4* nst = npk + a.pk_pairs * BWP;
    const int xb0 = x0 - e.txmax + lane;
    if constexpr (!VERT) {
      for (int cb = 0; cb < nblk; cb++) {
        const int c0 = min(cb * 64, span);
        const int xx = min(max(xb0 + c0, 0), W - 1);
        if (wave < bhp) glds_b128(pk + vo + pk_row + 2 * xx, npk + wave * BWP + c0);
        if (wave < shp) glds_b128(stats + vo + st_row + 2 * xx, nst + wave * BWP + c0);
      }
    } else {
      const int ebh = e.bhp, esh = e.shp & 0xff;
      const int pm0 = (y0 - R - e.tymax) >> 1, sm0 = (y0 - e.tymax) >> 1;  // floor: arithmetic shifts
      for (int cb = 0; cb < nblk; cb++) {
        const int c0 = min(cb * 64, span);
        const int xx = min(max(xb0 + c0, 0), W - 1);
        const uint2* gpk = pk + vo + 2 * xx;
        const uint2* gst = stats + vo + 2 * xx;
        for (int i = wave; i < ebh; i += NW) glds_b128(gpk + 2L * W * min(max(pm0 + i, 0), Hp2 - 1), npk + i * BWP + c0);
        for (int i = wave; i < esh; i += NW) glds_b128(gst + 2L * W * min(max(sm0 + i, 0), Hp2 - 1), nst + i * BWP + c0);
      }
    }
  };

  // the steps' level -> band column offsets, into LDS (before the pipeline)
  for (int i = tid; i < T * DC / 2; i += NW * 64) ((int*)colo_l)[i] = rec[i / (DC / 2)].colo[i % (DC / 2)];
  // step t's scalars (cur) and step t+1's (nxt); horizontal lists only
  // NB = 3 (horizontal): nx2 = step t+2's, staged at step t, two steps ahead
  auto nmod = [&](int v) { return v >= nn ? v - nn : v; };  // (v < 2 nn)
  StepInfo cur{}, nxt{}, nx2{};
  if constexpr (!VERT) {
    cur = load_info(0, 0);
    if (T > 1) nxt = load_info(1, nmod(1 % nn));
    if (NB == 3 && T > 2) nx2 = load_info(2, nmod(2 % nn));
    stage_h(cur, 0);
    if (NB == 3 && T > 1) stage_h(nxt, 1);
  } else {
    stage(0, 0, 0);
  }
  const long zo = (long)a.z[ref] * Pv;
  // -Sr' and s_r of the tile's 64 x TH pixels (lane = column), as k_ncc_volume:
  // wave w takes rows w, w + 8, ... (one correctly rounded sqrt + divide per
  // row and lane, spread over the waves instead of TH of them on wave 0)
  for (int o = wave; o < TH; o += NW) {
    const int x = x0 + lane, xc = min(x, W - 1), y = y0 + o;
    int s1 = 0, s2 = 0;
#pragma unroll
    for (int k = 0; k < 2 * R + 1; k++) {
      const uint2 v = pk[zo + pair_index(min(max(y - R + k, 0), H - 1), xc, W)];
      const unsigned lo = v.x, hi = v.y & (K == 5 ? 0xffu : 0xffffffu);  // the window's K bytes
      s1 = dot4(lo, 0x01010101u, dot4(hi, 0x01010101u, s1));
      s2 = dot4(lo, lo, dot4(hi, hi, s2));
    }
    const bool valid = x - R >= 0 && x + R < W && y - R >= 0 && y + R < H;
    const int var = NK * s2 - s1 * s1;
    srl[lane * TH + o] = !valid ? __int_as_float(0x7fc00000) : (var != 0 ? 1.0f / sqrtf((float)var) : 0.0f);
    rsn_l[lane * TH + o] = -(float)s1;
  }
  // the reference operands.  K = 5: pixel block (xb, yb) of this wave =
  // columns x0 + 8 wave + 4 xb .. +3, rows y0 + 4 yb .. +3; lane l supplies
  // row m = l & 15 (pixel xx = m >> 2, yy = m & 3) and row pair g = l >> 4 of
  // the footprint: the 16-byte pk entry at column x0b, masked to the pixel's
  // window (bytes xx .. xx+4 of a row; footprint rows yy .. yy+4).  K = 7:
  // block xb = columns x0 + 8 wave + 2 xb, +1, rows y0 .. y0 + 7; m = 8 xx + yy,
  // the footprint rows y0 - 4 .. y0 + 11 (pairs g and g + 4: the block's two
  // MFMAs), bytes xx .. xx+6, footprint rows yy + 1 .. yy + 7
  i32x4 A[NBL][MF];
  {
    const int mA = lane & 15, g = lane >> 4;
    const int xxA = K == 5 ? mA >> 2 : mA >> 3, yyA = K == 5 ? mA & 3 : mA & 7;
    unsigned msk[MF][4];
#pragma unroll
    for (int mf = 0; mf < MF; mf++)
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int h = k >> 1, rr = 2 * (g + 4 * mf) + h;
        unsigned mk = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const int t = 4 * (k & 1) + b;
          const bool in = K == 5 ? (t >= xxA && t <= xxA + 4 && rr >= yyA && rr <= yyA + 4)
                                 : (t >= xxA && t <= xxA + 6 && rr >= yyA + 1 && rr <= yyA + 7);
          if (in) mk |= 0xffu << (8 * b);
        }
        msk[mf][k] = mk;
      }
#pragma unroll
    for (int xb = 0; xb < XB; xb++)
#pragma unroll
      for (int yb = 0; yb < NYB; yb++)
#pragma unroll
        for (int mf = 0; mf < MF; mf++) {
          const int xcol = min(x0 + 8 * wave + BXW * xb, W - 1);
          const int pr = min(max(K == 5 ? (y0 >> 1) - 1 + 2 * yb + g : (y0 >> 1) - 2 + g + 4 * mf, 0), Hp2 - 1);
          const u32x4 v = *(const u32x4*)(pk + zo + (((long)pr * W + xcol) << 1));
          A[xb * NYB + yb][mf] = i32x4{(int)(v.x & msk[mf][0]), (int)(v.y & msk[mf][1]), (int)(v.z & msk[mf][2]),
                                       (int)(v.w & msk[mf][3])};
        }
  }
  // this lane's output pixels of block (xb, yb): column 8 wave + pcol, rows
  // prow .. prow + 3 of the tile (the MFMA's C[4 (l >> 4) + r][l & 15])
  auto pcol = [&](int xb, int g) { return BXW * xb + (K == 5 ? g : g >> 1); };
  auto prow = [&](int yb, int g) { return K == 5 ? 4 * yb : 4 * (g & 1); };
  __syncthreads();

  float E[NBL][NDB][4];  // [block][level block][row]: max over the neighbours so far
  float wv0[NBL][4], wv1[NBL][4];
  unsigned wi0p[NBL][2];  // level of the smallest, rows (2p, 2p+1) as the halves of one register (0xffff: none)
#pragma unroll
  for (int k = 0; k < NBL; k++) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      wv0[k][r] = kWtaInit;
      wv1[k][r] = kWtaInit;
    }
    wi0p[k][0] = wi0p[k][1] = 0xffffffffu;
  }
  const i32x4 bias = i32x4{kMagicI, kMagicI, kMagicI, kMagicI};

  // fold chunk c's levels into the per-cell triples (k_ncc_volume's fold; this
  // lane's levels are c * DC + 16 db + (l & 15), in increasing order)
  auto fold = [&](int c) {
    const int ln = lane_now();
    // dummy levels past the end (TAIL kernels, last chunk): +inf costs change nothing
    float kill[NDB];
#pragma unroll
    for (int db = 0; db < NDB; db++) kill[db] = 0.0f;
    if (TAIL && c == a.nch - 1)
#pragma unroll
      for (int db = 0; db < NDB; db++) kill[db] = c * DC + 16 * db + (ln & 15) >= a.D ? INFINITY : 0.0f;
#pragma unroll
    for (int xb = 0; xb < XB; xb++)
#pragma unroll
      for (int yb = 0; yb < NYB; yb++) {
        const int kb = xb * NYB + yb;
        const f32x4 sq = *(const f32x4*)(srl + (8 * wave + pcol(xb, ln >> 4)) * TH + prow(yb, ln >> 4));
        // NDB = 2: this lane's two levels of the chunk, dl0 < dl1 = dl0 + 16,
        // folded as a pair: with lo / hi their smaller / larger cost, the
        // triple's new second smallest is min(max(v0, lo), v1, hi) (the second
        // of the multiset {v0 <= v1, c0, c1}), its smallest min(v0, lo), and its
        // level the pair's first argmin (dl1 only if c1 < c0) when lo < v0: the
        // sequential fold's results in fewer instructions per level
        const int dl0 = c * DC + (ln & 15);
        const unsigned d0 = (unsigned)dl0 * 0x10001u, d1 = (unsigned)(dl0 + 16) * 0x10001u;
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          f32x2 cst[NDB];
#pragma unroll
          for (int db = 0; db < NDB; db++) {
            f32x2 e;
            e.x = __fmul_rn(E[kb][db][r], sq[r]);
            e.y = __fmul_rn(E[kb][db][r + 1], sq[r + 1]);
            // NDB = 2: 1 - m without the clamp max(-1, m) -- a cost above 2 or
            // NaN (no valid neighbour window at the level) stands for the
            // clamped 2, restored at the merge; the pair fold below treats NaN
            // as absent.  (NDB = 1 keeps the clamp: its med3 fold would not.)
            if constexpr (NDB == 2) {
              cst[db].x = __fsub_rn(1.0f, e.x);
              cst[db].y = __fsub_rn(1.0f, e.y);
            } else {
              cst[db].x = __fsub_rn(1.0f, vmax_m1(e.x));
              cst[db].y = __fsub_rn(1.0f, vmax_m1(e.y));
            }
            if (TAIL) {  // costs are >= 0: x + 0 = x, x + inf = inf
              cst[db].x = __fadd_rn(cst[db].x, kill[db]);
              cst[db].y = __fadd_rn(cst[db].y, kill[db]);
            }
          }
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const unsigned hm = h ? 0xffff0000u : 0x0000ffffu;
            unsigned& wp = wi0p[kb][r >> 1];
            float& v0 = wv0[kb][r + h];
            float& v1 = wv1[kb][r + h];
            if constexpr (NDB == 2) {
              const float c0 = cst[0][h], c1 = cst[NDB - 1][h];  // NaN: absent (the clamped 2)
              const float lo = vmin3(c0, c1, INFINITY);  // the smaller present cost (+inf: none)
              const float hi = vmaximum3(c0, c1, c1);    // the larger, NaN if either is absent
              const unsigned idx = lo == c0 ? d0 : d1;   // a tie keeps the lower level
              v1 = vmin3(vmax(v0, lo), v1, hi);          // (a NaN hi drops out of the min)
              wp = lo < v0 ? (wp & ~hm) | (idx & hm) : wp;
              v0 = vmin(v0, lo);
            } else {  // one level: the sequential fold
              const float cc = cst[0][h];
              v1 = vmed3(v0, v1, cc);
              wp = cc < v0 ? (wp & ~hm) | (d0 & hm) : wp;
              v0 = vmin(v0, cc);
            }
          }
        }
      }
  };

  int bt = 0;  // NB = 3: the buffer of step t (t % 3)
  // one pipeline step t = c * nn + n (chunks outer, neighbours inner; the
  // chunk's first neighbour assigns E, as k_ncc_volume's PEEL)
  auto step = [&](int t, int n, int cprev, auto first) {
    constexpr bool FIRST = decltype(first)::value;
    const int n1 = n + 1 == nn ? 0 : n + 1;
    StepInfo pf{};  // step t+NB's scalars, issued now, used NB - 1 steps on
    if constexpr (!VERT) {
      const int n2 = n1 + 1 == nn ? 0 : n1 + 1;
      if (t + NB < T) pf = load_info(t + NB, NB == 2 ? n2 : nmod(n2 + 1));
    }
    if (NB == 1 && t > 0) {  // this step's bands into the one buffer (step 0's: before the loop)
      stage(t, n, 0);
      __syncthreads();  // vmcnt(0): landed, for every wave
    }
    u32x4* const nbuf_t = nbase + (NB == 2 ? (t & 1) : NB == 3 ? bt : 0) * nbuf;
    // A block's B entry sits at column x0b - tx, up to 3 columns left of its
    // cells' neighbour pixels: a valid cell (neighbour column 2, xx = 3) reads
    // the entry of image column -1, which the clamped DMA filled with column
    // 0's.  Where the band holds column -1 (tiles at the left image edge),
    // that entry becomes the pk plane's definition: column 0's bytes one place
    // later (its bytes 0..2 lie outside the image and meet masked taps only).
    // (K = 7: a block's entry column is its 2-wide block's first column - tx,
    // never left of a valid cell's neighbour column - 1 >= 2: nothing to fix)
    if (K == 5 && (VERT || x0 < a.txmax_all)) {  // (tiles right of every shift: never)
      const int jf = (VERT ? rec[t].txmax : cur.tx) - x0 - 1;  // band column of image column -1 (scalar)
      const int esh = VERT ? rec[t].shp : cur.shp;
      if (jf >= 0 && jf + 1 < 64 + ((esh >> 16) & 0xff)) {  // inside the band's 64 + span columns
        if (tid < a.pk_pairs) {
          u32x4* e = nbuf_t + tid * BWP + jf + ((tid & 1) ? (esh >> 24) : 0);
          const u32x4 v = e[1];
          *e = u32x4{v.x << 8, (v.y << 8) | (v.x >> 24), v.z << 8, (v.w << 8) | (v.z >> 24)};
        }
        __syncthreads();
      }
    }
    int pieces = 0;  // NB = 3: this wave's LDS-DMA pieces of step t+2 (the barrier's count)
    if constexpr (!VERT && NB == 2) {
      if (t + 1 < T) stage_h(nxt, (t + 1) & 1);
    } else if constexpr (!VERT) {
      if (t + 2 < T) {
        stage_h(nx2, bt == 0 ? 2 : bt - 1);  // (t + 2) % 3
        const int nb2 = (((nx2.shp >> 16) & 0xff) + 127) >> 6;
        pieces = (wave < bhp ? nb2 : 0) + (wave < shp ? nb2 : 0);
      }
    } else {
      if (NB == 2 && t + 1 < T) stage(t + 1, n1, (t + 1) & 1);
    }
    if (FIRST && cprev >= 0) fold(cprev);
    const u32x4* npk = nbuf_t;
    const u32x4* nst = npk + a.pk_pairs * BWP;
    const int ln = lane_now();
    const int g = ln >> 4;
    // per level block: the band column of the lane's level (horizontal), or
    // (VERT) the lane's B-row and stats-row addresses for block (0, 0): uint2
    // index of footprint rows o + 2g, o + 2g + 1 and float index of the a of
    // pixel rows o, o + 1 (b two floats on; rows + 2: the next pair row)
    int cl[NDB], iB0[NDB], iB1[NDB], iS0[NDB], iS1[NDB];
#pragma unroll
    for (int db = 0; db < NDB; db++) {
      const int v = colo_l[t * DC + 16 * db + (ln & 15)];
      if constexpr (!VERT) {
        cl[db] = v;
      } else {
        const int col = 8 * wave + (v & 0xff), o = v >> 8;
        const int r0 = o + 2 * g, r1 = r0 + 1, s1 = o + 1;
        iB0[db] = 2 * ((r0 >> 1) * BWP + col) + (r0 & 1);
        iB1[db] = 2 * ((r1 >> 1) * BWP + col) + (r1 & 1);
        iS0[db] = 4 * ((o >> 1) * BWP + col + g) + (o & 1);
        iS1[db] = 4 * ((s1 >> 1) * BWP + col + g) + (s1 & 1);
      }
    }
    // The lanes reading odd pk pair rows (g odd) find them sh columns along,
    // the step's bank shift: with the pitch BW + 1, lanes of one ds_read_b128
    // group read two rows 1 + sh bank quads apart, and the host picks sh per
    // step so that the column shift per level (|dx| = 1, 3 want sh = -1; 2
    // wants 0) puts their 16-byte entries on distinct quads.  K = 7: the odd-g
    // lanes' stats pairs (2, 3) likewise, st columns along
    const int sg = (!VERT && (g & 1)) ? (cur.shp >> 24) : 0;
    const int tg = (K == 7 && (g & 1)) ? ((cur.shp << 16) >> 24) : 0;
    auto bread = [&](int xb, int yb, int db, int mf) -> i32x4 {
      if constexpr (!VERT) {  // K = 5: pair 2 yb + g of the band; K = 7: pair g + 4 mf (parity g & 1 alike)
        const int pr = K == 5 ? 2 * yb + g : g + 4 * mf;
        return __builtin_bit_cast(i32x4, npk[pr * BWP + 8 * wave + BXW * xb + cl[db] + sg]);
      } else {
        const uint2* b2 = (const uint2*)npk;
        const int off = 2 * (2 * yb * BWP + 4 * xb);
        const uint2 lo = b2[iB0[db] + off], hi = b2[iB1[db] + off];
        return i32x4{(int)lo.x, (int)lo.y, (int)hi.x, (int)hi.y};
      }
    };
    // {a, a, b, b} of pixel rows 0, 1 (s0) and rows 2, 3 (s1) of the block
    auto sread = [&](int xb, int yb, int db, f32x4& s0, f32x4& s1) {
      if constexpr (!VERT) {
        const int colS = 8 * wave + pcol(xb, g) + cl[db] + tg;  // stats band column of this lane's pixel column
        const int sp = prow(yb, g) >> 1;                    // stats band pair of its first row
        s0 = __builtin_bit_cast(f32x4, nst[sp * BWP + colS]);
        s1 = __builtin_bit_cast(f32x4, nst[(sp + 1) * BWP + colS]);
      } else {
        const float* f = (const float*)nst;
        const int off = 4 * (2 * yb * BWP + 4 * xb);
        const int q0 = iS0[db] + off, q1 = iS1[db] + off, q2 = q0 + 4 * BWP, q3 = q1 + 4 * BWP;
        s0 = f32x4{f[q0], f[q1], f[q0 + 2], f[q1 + 2]};
        s1 = f32x4{f[q2], f[q3], f[q2 + 2], f[q3 + 2]};
      }
    };
    auto finish = [&](int xb, int yb, int db, const i32x4& acc, const f32x4& nsr, const f32x4& s0,
                      const f32x4& s1) {
#pragma unroll
      for (int p = 0; p < 2; p++) {
        const f32x4 sv = p ? s1 : s0;
        f32x2 xv;
        xv.x = __fmaf_rn(nsr[2 * p], sv.z, __fmul_rn(__fsub_rn(__int_as_float(acc[2 * p]), kMagicF), sv.x));
        xv.y = __fmaf_rn(nsr[2 * p + 1], sv.w, __fmul_rn(__fsub_rn(__int_as_float(acc[2 * p + 1]), kMagicF), sv.y));
        const int kb = xb * NYB + yb;
        if (FIRST) {
          E[kb][db][2 * p] = xv.x;
          E[kb][db][2 * p + 1] = xv.y;
        } else {
          E[kb][db][2 * p] = vmax(E[kb][db][2 * p], xv.x);
          E[kb][db][2 * p + 1] = vmax(E[kb][db][2 * p + 1], xv.y);
        }
      }
    };
    // one level block at a time (at the 128-VGPR cap the paired form spilled 16-40 B)
#pragma unroll
    for (int k = 0; k < (DBG == 1 ? 0 : NBL); k++) {
      const int xb = k / NYB, yb = k % NYB;
      const f32x4 nsr = *(const f32x4*)(rsn_l + (8 * wave + pcol(xb, g)) * TH + prow(yb, g));
#pragma unroll
      for (int db = 0; db < NDB; db++) {
        // the block's operand(s) and its neighbour stats issued together, ahead
        // of the MFMA: one LDS latency per block on the wave's chain, not two
        i32x4 bv[MF];
#pragma unroll
        for (int mf = 0; mf < MF; mf++) bv[mf] = bread(xb, yb, db, mf);
        f32x4 s0, s1;
        sread(xb, yb, db, s0, s1);
        if (SPLIT) __builtin_amdgcn_sched_barrier(0);
        i32x4 acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[k][0], bv[0], bias, 0, 0, 0);
        if constexpr (MF == 2) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[k][1], bv[1], acc, 0, 0, 0);
        finish(xb, yb, db, acc, nsr, s0, s1);
      }
    }
    if constexpr (!VERT && NB == 3) {
      // step t+1's bands landed (this wave's pieces of it are older than its
      // `pieces` of step t+2: loads retire in order), then the barrier: every
      // wave's; buffer t % 3 is free for step t+3 (staged at step t+1)
      wait_vm_barrier(pieces);  // (a memory clobber: no LDS access moves across it; no vmcnt(0) added)
    } else {
      __syncthreads();  // NB = 2: step t+1's bands landed, this buffer free for t+2; NB = 1: free for t+1
    }
    if constexpr (!VERT) {
      cur = nxt;
      if constexpr (NB == 3) {
        nxt = nx2;
        nx2 = pf;
        bt = bt == 2 ? 0 : bt + 1;
      } else {
        nxt = pf;
      }
    }
  };
  {
    int t = 0;
    for (int c = 0; c < a.nch; c++) {
      step(t++, 0, c - 1, std::true_type{});
      for (int n = 1; n < nn; n++) step(t++, n, -1, std::false_type{});
    }
  }
  fold(a.nch - 1);

  // merge the 16 level classes of every pixel through LDS (the band buffers
  // are free: every wave passed the loop's last barrier), one half tile of
  // 64 x 4 pixels at a time; one thread per pixel, k_ncc_volume's merge
  float* m0 = (float*)smem;
  float* m1 = m0 + 16 * kMfMergeStride;
  int* mi = (int*)(m1 + 16 * kMfMergeStride);
#pragma unroll
  for (int yb = 0; yb < TH / 4; yb++) {  // tile rows 4 yb .. 4 yb + 3
    {
      const int ln = lane_now(), cls = ln & 15, g = ln >> 4;
      // K = 5: block row yb; K = 7: the lanes whose rows are these (g & 1 == yb)
      const int kyb = K == 5 ? yb : 0;
      if (K == 5 || (g & 1) == yb) {
#pragma unroll
        for (int xb = 0; xb < XB; xb++)
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int kb = xb * NYB + kyb;
            const int q = cls * kMfMergeStride + r * 64 + 8 * wave + pcol(xb, g);
            const unsigned v = (r & 1) ? wi0p[kb][r >> 1] >> 16 : wi0p[kb][r >> 1] & 0xffffu;
            m0[q] = wv0[kb][r];
            m1[q] = wv1[kb][r];
            mi[q] = v == 0xffffu ? -1 : (int)v;
          }
      }
    }
    __syncthreads();
    if (tid < 256) {
      const int q = tid, xx = x0 + (q & 63), yy = y0 + 4 * yb + (q >> 6);
      // lexicographic (cost, level) minimum; "no level" (-1) compares as the
      // largest level (it only ever comes with the initial cost 1e6, which no
      // real level has).  Costs can be slightly negative (NCC rounding past 1),
      // so they are compared as floats.
      // every class's entries read up front (one LDS latency, not one per
      // class), the minimum as a branch-free tree (the order is immaterial:
      // the classes' levels are distinct, so no two entries tie in both keys)
      float v0s[16], v1s[16];
      unsigned is[16];
#pragma unroll
      for (int w = 0; w < 16; w++) {
        v0s[w] = m0[w * kMfMergeStride + q];
        is[w] = (unsigned)mi[w * kMfMergeStride + q];
        v1s[w] = m1[w * kMfMergeStride + q];
      }
      float tv[16];
      unsigned ti[16];
#pragma unroll
      for (int w = 0; w < 16; w++) {
        tv[w] = v0s[w];
        ti[w] = is[w];
      }
#pragma unroll
      for (int h = 8; h >= 1; h >>= 1)
#pragma unroll
        for (int w = 0; w < h; w++) {
          const bool tk = (tv[w + h] < tv[w]) | ((tv[w + h] == tv[w]) & (ti[w + h] < ti[w]));
          tv[w] = tk ? tv[w + h] : tv[w];
          ti[w] = tk ? ti[w + h] : ti[w];
        }
      const float bv = tv[0];
      const unsigned bi = ti[0];
      float c2 = kWtaInit;
#pragma unroll
      for (int w = 0; w < 16; w++) {
        const float v = (unsigned)((int)is[w] - (int)bi + 1) <= 2u ? v1s[w] : v0s[w];
        c2 = vmin(c2, v);
      }
      // The fold skipped the clamp (cost = 1 - max(-1, m) = min(2, 1 - m)).
      // If the smallest cost is below 2 the clamp changes neither it nor its
      // level, and the second smallest outside bi +- 1 is min(2, that) whenever
      // such a level exists; otherwise every level costs 2 and the first level
      // wins with confidence 0 (k_wta's strict <, in level order).
      const bool all2 = !(bv < 2.0f);
      const int b = (int)bi;
      if (!all2 && a.D > min(b + 1, a.D - 1) - max(b - 1, 0) + 1) c2 = vmin(c2, 2.0f);
      if (xx < W && yy < H) {
        const long p = P * ref + (long)yy * W + xx;
        wo.disp[p] = a.D <= 0 ? 0.0f : wo.levels[all2 ? 0 : b];
        if (wo.conf) wo.conf[p] = (all2 || c2 == kWtaInit) ? 0.0f : c2 - bv;
      }
    }
    __syncthreads();
  }
}


template <int K, int BW, bool TAIL, bool VERT, int NDB, int NB, int DBG = 0>
int launch_mfma_bw(mvs_ctx* ctx, const uint2* stats, const uint2* pk, const NccMRec* plan, NccArgs& a,
                   const WtaOut& wo, int tmax) {
  constexpr int TH = 8, DC = 16 * NDB;
  const int variant[8] = {K, TH, DC, 8, BW, VERT ? kParMixed : (K == 5 ? kParEven : kParOdd), 1, NB};
  std::copy(variant, variant + 8, ctx->ncc_last);
  a.tiles_x = (a.W + 63) / 64;
  a.ntiles = a.tiles_x * ((a.H + TH - 1) / TH);
  a.tiles_per_xcd = (a.nref * a.ntiles + 7) / 8;
  a.nch = (a.D + DC - 1) / DC;
  const size_t lds = std::max((size_t)NB * 16 * (a.pk_pairs + a.st_pairs) * (BW + 1), (size_t)3 * 16 * kMfMergeStride * 4) +
                     2 * 64 * TH * 4 + (size_t)tmax * DC * 2;
  auto kern = k_ncc_mfma<K, BW, TAIL, VERT, NDB, NB, DBG>;
  MVS_HIP(raise_lds(ctx, (const void*)kern, lds), "hipFuncSetAttribute(ncc mfma lds)");
  const auto ev = kernel_events(ctx);  // (timing off: plain launch)
  hipExtLaunchKernelGGL(kern, dim3(8 * a.tiles_per_xcd), dim3(512), lds, ctx->stream, ev.first, ev.second, 0, stats, pk,
                        plan, a, wo);
  MVS_LAUNCH_CHECK("k_ncc_mfma (fused WTA)");
  return 0;
}

// the band pitch template a VERT launch takes
int vert_bw(int band_w, bool tail) { return tail ? 128 : band_w <= 80 ? 80 : band_w <= 96 ? 96 : 128; }

template <bool TAIL, int NDB, int NB>
int launch_vert(mvs_ctx* ctx, const uint2* stats, const uint2* pk, const NccMRec* pl, NccArgs& a, const WtaOut& wo,
                int bw, int tmax) {
  const int bwt = vert_bw(bw, TAIL);  // (the tail kernels: one pitch)
  if (!TAIL && NDB == 1 && NB == 2 && bwt == 80) {  // timing probe (C4's interior lists): MVS_NCC_MFMA_DBG=1 | 2
    const char* dbg = getenv("MVS_NCC_MFMA_DBG");
    const int dv = dbg ? atoi(dbg) : 0;
    if (dv == 1) return launch_mfma_bw<5, 80, false, true, 1, 2, 1>(ctx, stats, pk, pl, a, wo, tmax);
    if (dv == 2) return launch_mfma_bw<5, 80, false, true, 1, 2, 2>(ctx, stats, pk, pl, a, wo, tmax);
  }
  if (TAIL || bwt == 128) return launch_mfma_bw<5, 128, TAIL, true, NDB, NB>(ctx, stats, pk, pl, a, wo, tmax);
  return bwt == 80 ? launch_mfma_bw<5, 80, TAIL, true, NDB, NB>(ctx, stats, pk, pl, a, wo, tmax)
                   : launch_mfma_bw<5, 96, TAIL, true, NDB, NB>(ctx, stats, pk, pl, a, wo, tmax);
}

}  // namespace

// LDS cycles of the B-operand / stats ds_read_b128 of one step (MI355X_MICROARCH.md,
// LDS table): 4 groups of 16 lanes, one cycle per group plus one per further
// distinct 16-byte entry on a busy bank quad (entry index mod 16; identical
// entries broadcast); summed over the chunk's level blocks and the 16
// residues c of the block column.  Lane l = 16 g + n reads entry
// row(g) (BW + 1) + sh (g & 1) + col(g) + c + colo[n], BW + 1 = 1 mod 16 for
// every horizontal pitch (129, 193): B operands row(g) = g, col(g) = 0;
// K = 7 stats row(g) = 2 (g & 1), col(g) = g >> 1.  (K = 5 stats: every lane
// of a read on one row, column g -- no shift changes them.)
static int bank_cycles(const int16_t* colo, int dc, int sh, bool k7_stats) {
  static const int grp[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                 {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                 {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                 {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
  // (a residue c adds to every entry alike: it rotates the quads and leaves
  // the count unchanged, so c = 0 stands for all 16)
  int cyc = 0;
  for (int b0 = 0; b0 < dc; b0 += 16)
      for (const auto& gr : grp) {
        int ent[16], most = 1;
        for (int i = 0; i < 16; i++) {
          const int l = gr[i], g = l >> 4;
          const int row = k7_stats ? 2 * (g & 1) : g, col = k7_stats ? g >> 1 : 0;
          ent[i] = row * 129 + sh * (g & 1) + col + (colo[b0 + (l & 15)] & 0xff) + 64;
        }
        for (int q = 0; q < 16; q++) {  // distinct entries on bank quad q
          int n = 0;
          for (int i = 0; i < 16; i++) {
            if ((ent[i] & 15) != q) continue;
            bool dup = false;
            for (int k = 0; k < i; k++) dup |= ent[k] == ent[i];
            n += !dup;
          }
          most = std::max(most, n);
        }
        cyc += most;
      }
  return cyc;
}
// the shift of fewest cycles among those the band's slack allows (a shifted
// row must stay inside its BW + 1 slot: |sh| <= BW + 1 - band_w; ties: the
// smaller |sh|, then the negative one)
static int bank_shift_eval(const int16_t* colo, int dc, bool k7_stats, int slack) {
  int best = 0, best_cyc = bank_cycles(colo, dc, 0, k7_stats);
  for (int sh : {-1, 1, -2, 2}) {
    if (std::abs(sh) > slack) continue;
    const int c = bank_cycles(colo, dc, sh, k7_stats);
    if (c < best_cyc) {
      best_cyc = c;
      best = sh;
    }
  }
  return best;
}
// memoised: the plan is rebuilt per call, and a level block's offsets repeat
// from call to call (a pure function of them, shared by every context)
static int bank_shift(const int16_t* colo, int dc, bool k7_stats, int slack) {
  static std::mutex mu;
  static std::map<std::vector<int16_t>, int> memo;
  std::vector<int16_t> key(colo, colo + dc);
  key.push_back((int16_t)(k7_stats ? 1 : 0));
  key.push_back((int16_t)std::min(slack, 2));  // (shifts beyond 2 are never tried)
  std::lock_guard<std::mutex> lock(mu);
  const auto it = memo.find(key);
  if (it != memo.end()) return it->second;
  const int v = bank_shift_eval(colo, dc, k7_stats, slack);
  if (memo.size() >= (1u << 16)) memo.clear();  // bounded: ~64 K level blocks (a few MB)
  memo.emplace(std::move(key), v);
  return v;
}

// the matrix-core form's plan: one NccMRec per (chunk of 16 ndb levels, neighbour)
NccPlanM make_plan_mfma(const float* levels, int D, int nn, const float* fdx, const float* fdy, float bl, int ndb,
                        int K) {
  constexpr int TH = 8, RW = sizeof(NccMRec) / 4;
  const int R = K / 2, NR = TH + 2 * R;
  const int DC = 16 * ndb;
  const int nch = (D + DC - 1) / DC;
  NccPlanM p;
  p.ndb = ndb;
  p.table.assign((size_t)nch * nn * RW, 0);
  int spx = 0;
  // k_ncc_volume's shifts (make_plan in ncc.hip)
  auto tx_of = [&](int dl, int n) { return (int)roundf(levels[dl] * fdx[n]); };
  auto ty_of = [&](int dl, int n) { return (int)roundf((bl * levels[dl]) * fdy[n]); };
  for (int n = 0; n < nn; n++)
    if (fdy[n] != 0.0f) p.vert = true;
  for (int c = 0; c < nch; c++)
    for (int n = 0; n < nn; n++) {
      int txmin = 1 << 30, txmax = -(1 << 30), tymin = 1 << 30, tymax = -(1 << 30);
      for (int dl = c * DC; dl < std::min(D, c * DC + DC); dl++) {
        txmin = std::min(txmin, tx_of(dl, n));
        txmax = std::max(txmax, tx_of(dl, n));
        tymin = std::min(tymin, ty_of(dl, n));
        tymax = std::max(tymax, ty_of(dl, n));
      }
      const int par = tymax & 1;  // the bands' first row (y0 - R - tymax, y0 - tymax) is o_j's parity off a pair
      // (K = 7, horizontal only: the 8 pairs of rows y0 - 4 .. y0 + TH + 3)
      const int bhp = K == 7 ? (TH + 8) / 2 : (par + NR + tymax - tymin + 1) >> 1;
      const int shp = (par + TH + tymax - tymin + 1) >> 1;
      int32_t* e = p.table.data() + ((size_t)c * nn + n) * RW;
      e[0] = txmax;
      e[1] = tymax;
      e[2] = bhp;                                  // pk pair rows: every level's y0-2 .. y0+TH+1 shifted
      e[3] = shp | ((txmax - txmin) << 16);       // stats pair rows | the chunk's column span
      int16_t* co = (int16_t*)(e + 4);
      for (int j = 0; j < DC; j++) {
        const int dl = c * DC + j;
        // a dummy level past the end: the band origin (in-band)
        co[j] = (int16_t)(dl < D ? (txmax - tx_of(dl, n)) | ((par + tymax - ty_of(dl, n)) << 8) : par << 8);
      }
      // horizontal lists: the odd pk rows' shift (bits 24..31 of word 3) and,
      // K = 7, the stats rows' (bits 8..15) that leave step()'s reads the
      // fewest LDS cycles.  Slack: the band pitch BW + 1 (129 | 193, the
      // horizontal templates) less this step's 64 + span columns
      if (!p.vert) {
        const int bw = 64 + txmax - txmin, slack = (bw <= 128 ? 129 : 193) - bw;
        e[3] |= (bank_shift(co, DC, false, slack) & 0xff) << 24;
        if (K == 7) e[3] |= (bank_shift(co, DC, true, slack) & 0xff) << 8;
      }
      spx = std::max(spx, txmax - txmin);
      p.pk_pairs = std::max(p.pk_pairs, bhp);
      p.st_pairs = std::max(p.st_pairs, shp);
    }
  p.band_w = 64 + spx;
  return p;
}

size_t mfma_lds_bytes(const NccPlanM& p, int band_w, int nb, int tmax, int D) {
  const bool tail = D % (16 * p.ndb) != 0;
  // the band pitch template launch_ncc_mfma picks: VERT by vert_bw, horizontal 128 | 192
  const int bwt = p.vert ? vert_bw(band_w, tail) : (tail || band_w > 128 ? 192 : 128);
  return std::max((size_t)nb * 16 * (p.pk_pairs + p.st_pairs) * (bwt + 1), (size_t)3 * 16 * kMfMergeStride * 4) +
         2 * 64 * 8 * 4 + (size_t)tmax * 16 * p.ndb * 2;
}

// the LDS bytes of a launch with these band heights, pitch bw (+1), nb buffers, dc levels per chunk
static size_t mfma_lds_bytes_nb(const NccArgs& a, int bw, int nb, int tmax, int dc) {
  return std::max((size_t)nb * 16 * (a.pk_pairs + a.st_pairs) * (bw + 1), (size_t)3 * 16 * kMfMergeStride * 4) +
         2 * 64 * 8 * 4 + (size_t)tmax * dc * 2;
}

int launch_ncc_mfma(mvs_ctx* ctx, const uint2* stats, const uint2* pk, const int32_t* plan_dev, NccArgs& a,
                    const WtaOut& wo, int bw, int tmax, bool vert, int ndb, int nb, int K) {
  const NccMRec* pl = (const NccMRec*)plan_dev;
  const bool tail = a.D % (16 * ndb) != 0;
  // timing probe (MVS_NCC_MFMA_DBG=1: no MFMA / finish, 2: no band DMA), C2's and C5's forms
  const char* dbg = getenv("MVS_NCC_MFMA_DBG");
  const int dv = dbg ? atoi(dbg) : 0;
  if (dv && !vert && !tail) {
    if (K == 7 && bw <= 128)
      return dv == 1 ? launch_mfma_bw<7, 128, false, false, 1, 2, 1>(ctx, stats, pk, pl, a, wo, tmax)
                     : launch_mfma_bw<7, 128, false, false, 1, 2, 2>(ctx, stats, pk, pl, a, wo, tmax);
    if (K == 5 && bw > 128)
      return dv == 1 ? launch_mfma_bw<5, 192, false, false, 2, 2, 1>(ctx, stats, pk, pl, a, wo, tmax)
                     : launch_mfma_bw<5, 192, false, false, 2, 2, 2>(ctx, stats, pk, pl, a, wo, tmax);
  }
  if (K == 7) {  // horizontal lists, 16-level chunks
    // the 128-column pitch triple-buffered (bands two steps ahead; 2 x 3
    // buffers of 24.8 KB keep two workgroups per CU), else double-buffered;
    // MVS_NCC_MFMA7_NB=3 (read per call): the triple-buffered form (measured slower, opt-in)
    const char* nbe = getenv("MVS_NCC_MFMA7_NB");
    const bool nb3 = nbe && atoi(nbe) == 3 && mfma_lds_bytes_nb(a, 128, 3, tmax, 16) <= (size_t)80 * 1024;
    if (tail) return launch_mfma_bw<7, 192, true, false, 1, 2>(ctx, stats, pk, pl, a, wo, tmax);
    if (bw <= 128)
      return nb3 ? launch_mfma_bw<7, 128, false, false, 1, 3>(ctx, stats, pk, pl, a, wo, tmax)
                 : launch_mfma_bw<7, 128, false, false, 1, 2>(ctx, stats, pk, pl, a, wo, tmax);
    return launch_mfma_bw<7, 192, false, false, 1, 2>(ctx, stats, pk, pl, a, wo, tmax);
  }
  if (vert) {
    if (ndb == 2 && nb == 2)
      return tail ? launch_vert<true, 2, 2>(ctx, stats, pk, pl, a, wo, bw, tmax)
                  : launch_vert<false, 2, 2>(ctx, stats, pk, pl, a, wo, bw, tmax);
    if (ndb == 2)
      return tail ? launch_vert<true, 2, 1>(ctx, stats, pk, pl, a, wo, bw, tmax)
                  : launch_vert<false, 2, 1>(ctx, stats, pk, pl, a, wo, bw, tmax);
    if (nb == 2)
      return tail ? launch_vert<true, 1, 2>(ctx, stats, pk, pl, a, wo, bw, tmax)
                  : launch_vert<false, 1, 2>(ctx, stats, pk, pl, a, wo, bw, tmax);
    return tail ? launch_vert<true, 1, 1>(ctx, stats, pk, pl, a, wo, bw, tmax)
                : launch_vert<false, 1, 1>(ctx, stats, pk, pl, a, wo, bw, tmax);
  }
  if (tail) return launch_mfma_bw<5, 192, true, false, 2, 2>(ctx, stats, pk, pl, a, wo, tmax);
  return bw <= 128 ? launch_mfma_bw<5, 128, false, false, 2, 2>(ctx, stats, pk, pl, a, wo, tmax)
                   : launch_mfma_bw<5, 192, false, false, 2, 2>(ctx, stats, pk, pl, a, wo, tmax);
}

}  // namespace ncc
}  // namespace mvs
