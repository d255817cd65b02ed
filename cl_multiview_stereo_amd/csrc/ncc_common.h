// Shared by the NCC sweep kernels (ncc.hip: scalar forms and the window
// planes; ncc_mfma.hip: the matrix-core form): row-pair plane indexing, the
// launch arguments, the LDS-DMA and the exact min / max / med3 helpers.
#pragma once
#include <cstdint>
#include <vector>
#include "mvs_internal.h"

namespace mvs {
namespace ncc {

// Row-pair interleaved planes: element (y, x) of a view lives at uint2 index
// ((y >> 1) * W + x) * 2 + (y & 1), over Hp = H rounded up to even rows, so
// one 16-byte access returns rows 2m and 2m+1 of one column.
__host__ __device__ __forceinline__ long pair_index(int y, int x, int W) {
  return (((long)(y >> 1) * W + x) << 1) + (y & 1);
}

constexpr int kMaxNbr = 16;
constexpr int kMaxRef = 8;  // reference views per launch (the fused sweep takes a run of them)
constexpr int kCPolNT = 2;  // buffer cache policy: non-temporal (CPol::NT on gfx940+)
struct NccArgs {
  int W, H, D, nref;
  int tiles_x, ntiles, tiles_per_xcd, nch;  // XCD-aware work map over nref x ntiles tiles (see k_ncc_volume)
  int pk_pairs, st_pairs;  // LDS band heights in row pairs; the pair-row stride is the template BW
  int txmax_all;           // (matrix-core runs) the largest band origin shift of any step: tiles with
                           // x0 >= it never hold image column -1 in a band
  int plane32;             // (scalar kernels) a view plane is under 2 GB: band DMA by buffer descriptors
  // per reference view r of the launch: view id, neighbour count, first plan
  // record, neighbour view ids
  int z[kMaxRef], nn[kMaxRef], plan[kMaxRef];
  int view[kMaxRef][kMaxNbr];
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
// max(-1, e) with -1.0 as an inline constant (no VGPR holding it)
__device__ __forceinline__ float vmax_m1(float e) {
  float r;
  asm("v_max_f32 %0, -1.0, %1" : "=v"(r) : "v"(e));
  return r;
}
__device__ __forceinline__ float vmin(float acc, float e) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(acc), "v"(e));
  return r;
}
__device__ __forceinline__ float vmin3(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// IEEE 754-2019 maximum of three (gfx950): NaN when any operand is NaN
__device__ __forceinline__ float vmaximum3(float a, float b, float c) {
  float r;
  asm("v_maximum3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// median of three: with lo <= hi, med3(lo, hi, c) = min(hi, max(lo, c))
__device__ __forceinline__ float vmed3(float lo, float hi, float c) {
  float r;
  asm("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(lo), "v"(hi), "v"(c));
  return r;
}

// Fused winner-take-all outputs (k_ncc_volume<..., FUSE = true>): the volume
// is never written.  Same results as k_wta over the materialised volume.
struct WtaOut {
  const float* levels;  // device [D]
  float* disp;          // [H][W]
  float* conf;          // [H][W] or null
};
constexpr float kWtaInit = 1000000.0f;  // k_wta's Top4 initial cost (sweep.hip)

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Row-parity modes of a launch's bands (k_ncc_volume's PAR; the plan knows it):
//   kParEven  every level's pk and stats rows start on a pair boundary (K = 5
//             with horizontal neighbours: R + tymax even)
//   kParOdd   every pk start is odd and every stats start even (K = 7 with
//             horizontal neighbours: R = 3)
//   kParMixed either, per level (vertical / diagonal neighbours): a run-time test
constexpr int kParMixed = 0, kParEven = 1, kParOdd = 2;

// N consecutive band rows starting at band row r0 of a row-pair band (pair
// row stride BW, one column): ds_read_b128 per pair; an odd start takes the
// first and last rows as ds_read_b64 halves.  N even.
template <int N, int BW, int PAR>
__device__ __forceinline__ void read_rows(const u32x4* col, int r0, u32x2 (&v)[N]) {
  const u32x4* p = col + (r0 >> 1) * BW;
  if (PAR == kParEven || (PAR == kParMixed && (r0 & 1) == 0)) {
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

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// The N/2 stats row pairs (o, o+1), o even, of a band column starting at band
// row r0: {a(o), a(o+1), b(o), b(o+1)}.  An odd start joins the second row of
// one stored pair with the first row of the next.
template <int N, int BW, int PAR>
__device__ __forceinline__ void read_stat_pairs(const u32x4* col, int r0, f32x4 (&v)[N / 2]) {
  const u32x4* p = col + (r0 >> 1) * BW;
  if (PAR != kParMixed || (r0 & 1) == 0) {
#pragma unroll
    for (int i = 0; i < N / 2; i++) v[i] = __builtin_bit_cast(f32x4, p[i * BW]);
  } else {
    // only the 16 needed dwords, as ds_read2_b32 pairs ({a, b} of one stored
    // row): no stored pair held whole, so the odd path needs no more registers
    // than the even one (the whole-pair form kept N/2 + 1 pairs live, and the
    // fused mixed-parity kernels spilled their fold accumulators for it)
    const float* f = (const float*)p;
#pragma unroll
    for (int i = 0; i < N / 2; i++) {
      const float* q0 = f + i * BW * 4;        // stored pair i: second rows (y, w)
      const float* q1 = f + (i + 1) * BW * 4;  // stored pair i + 1: first rows (x, z)
      v[i] = f32x4{q0[1], q1[0], q0[3], q1[2]};
    }
  }
}

// v_dot4_i32_i8 is the VOP3P form (separate destination): a prefix-sum chain
// keeps every partial sum without the accumulator copies the VOP2 v_dot4c
// form forces.  The Makefile builds this file with the dot6 feature (v_dot4c)
// off, so the compiler selects the VOP3P form and still tracks its hazards.
// s_waitcnt vmcnt(min(n, 6)) (n >= 0; a count above 6 waits for 6: still
// correct for a caller that needs at most n outstanding, only earlier)
__device__ __forceinline__ void wait_vm_le(int n) {
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

// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 6] (n > 6: vmcnt(6)), then
// s_barrier -- the selection inside one asm block, so the compiler sees no
// branch (a C-level switch split the step and spilled the fold's registers)
__device__ __forceinline__ void wait_vm_barrier(int n) {
  asm volatile(
      "s_cmp_eq_u32 %0, 0\n\ts_cbranch_scc1 10f\n\t"
      "s_cmp_eq_u32 %0, 1\n\ts_cbranch_scc1 11f\n\t"
      "s_cmp_eq_u32 %0, 2\n\ts_cbranch_scc1 12f\n\t"
      "s_cmp_eq_u32 %0, 3\n\ts_cbranch_scc1 13f\n\t"
      "s_cmp_eq_u32 %0, 4\n\ts_cbranch_scc1 14f\n\t"
      "s_cmp_eq_u32 %0, 5\n\ts_cbranch_scc1 15f\n\t"
      "s_waitcnt vmcnt(6)\n\ts_branch 19f\n"
      "10:\n\ts_waitcnt vmcnt(0)\n\ts_branch 19f\n"
      "11:\n\ts_waitcnt vmcnt(1)\n\ts_branch 19f\n"
      "12:\n\ts_waitcnt vmcnt(2)\n\ts_branch 19f\n"
      "13:\n\ts_waitcnt vmcnt(3)\n\ts_branch 19f\n"
      "14:\n\ts_waitcnt vmcnt(4)\n\ts_branch 19f\n"
      "15:\n\ts_waitcnt vmcnt(5)\n"
      "19:\n\ts_barrier"
      :
      : "s"(n)
      : "memory", "scc");
}

// the lane id, recomputed where it is used (volatile: never hoisted, so it is
// never a long-lived value the register allocator would spill)
__device__ __forceinline__ int lane_now() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

constexpr int kMagicI = 0x4B400000;  // the bits of 12582912.0f = 1.5 * 2^23
constexpr float kMagicF = 12582912.0f;
__device__ __forceinline__ int dot4(unsigned a, unsigned b, int c) {
  return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
}

// the matrix-core fused sweep (ncc_mfma.hip): its plan (one 128-B record per
// chunk of 16 NDB levels and neighbour) and one launch over a run of
// reference views.  vert: some neighbour shifts rows (the general form:
// per-level band rows, pair reads split at odd offsets); NB: band buffers
struct NccPlanM {
  std::vector<int32_t> table;
  int band_w = 0;                // columns per band pair row: 64 + the widest chunk span
  int pk_pairs = 0, st_pairs = 0;  // band heights in row pairs (the tallest step)
  int ndb = 2;                   // 16-level blocks per chunk
  bool vert = false;
};
NccPlanM make_plan_mfma(const float* levels, int D, int nn, const float* fdx, const float* fdy, float bl, int ndb,
                        int K = 5);
// the LDS bytes of one workgroup of the matrix-core form
size_t mfma_lds_bytes(const NccPlanM& p, int band_w, int nb, int tmax, int D);
int launch_ncc_mfma(mvs_ctx* ctx, const uint2* stats, const uint2* pk, const int32_t* plan_dev, NccArgs& a,
                    const WtaOut& wo, int bw, int tmax, bool vert, int ndb, int nb, int K);

}  // namespace ncc
}  // namespace mvs
