// VALU issue-rate probe (round 5): cycles per wave64 VALU instruction per SIMD
// at 1, 2, 4 and 8 waves per SIMD, counted in shader clocks by s_memtime inside
// each wave (independent of the clock the chip runs at), with every measured
// instruction written as inline asm so the compiler cannot pair scalar FP32 ops
// into v_pk_* forms (what made an earlier probe read "FP32 at 2 cycles").
//
// Layout: one workgroup per CU (96 KB of dynamic LDS) of 4*w waves for w <= 4,
// two workgroups of 16 waves (72 KB each) for w = 8; 8 independent
// accumulator chains per lane; the measured loop is 32 instructions per trip.
// Each wave records s_memtime at the start (after the workgroup barrier) and
// at the end of its loop and its SIMD (HW_ID bits 5:4).  The hardware does not
// deal a workgroup's waves evenly over the 4 SIMDs, so the rate is taken per
// SIMD: cycles/instr = (last end - first start of that SIMD's waves) /
// (waves on it x instructions per wave), median over every (CU, SIMD) with
// exactly w waves (and over all SIMDs, in the second column).  The clock is the
// s_memtime delta over the s_memrealtime (100 MHz) delta of the same wave.
//
//   hipcc -O3 --offload-arch=gfx950 valu_rate3.hip -o valu_rate3 && ./valu_rate3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <array>
#include <map>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ __launch_bounds__(1024) void k(unsigned long long* out, unsigned a, unsigned b, int iters) {
  extern __shared__ unsigned char lds_pad[];
  unsigned v[8];
  f2 p[8];
  for (int i = 0; i < 8; i++) {
    v[i] = threadIdx.x * (i + 1);
    p[i] = f2{(float)v[i], (float)(v[i] + 1)};
  }
  const float fa = __int_as_float(a);
  unsigned long long msk = __builtin_amdgcn_read_exec() & (unsigned long long)(a * 0x9e3779b97f4a7c15ull), m2 = 0;
  const f2 pa = f2{fa, fa};
  if (threadIdx.x == 1u << 30) lds_pad[0] = 1;  // keep the LDS allocation
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; it++) {
#define STEP(i)                                                                                                  \
    if (OP == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(fa), "v"(fa));                        \
    if (OP == 1) asm volatile("v_dot4_i32_i8 %0, %1, %2, %0" : "+v"(v[i]) : "v"(a), "v"(b));                      \
    if (OP == 2) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[i]) : "v"(pa), "v"(pa));                     \
    if (OP == 3) asm volatile("v_add_f32 %0, %1, %0" : "+v"(v[i]) : "v"(fa));                                     \
    if (OP == 4) asm volatile("v_max_f32 %0, %1, %0" : "+v"(v[i]) : "v"(fa));                                     \
    if (OP == 5) asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(p[i]) : "v"(pa));                                  \
    if (OP == 6) asm volatile("v_mov_b32 %0, %1" : "=v"(v[i]) : "v"(v[(i + 1) & 7]));                            \
    if (OP == 7) asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(p[i]) : "v"(pa));                                  \
    if (OP == 8) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(v[i]) : "v"(a));                                      \
    if (OP == 9) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(v[i]) : "v"(fa));                                     \
    if (OP == 10) asm volatile("v_add_f32_e64 %0, %1, %0" : "+v"(v[i]) : "v"(fa));                                \
    if (OP == 11) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(v[i]) : "v"(fa), "v"(fa));                          \
    if (OP == 12) asm volatile("v_med3_f32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(fa), "v"(fa));                      \
    if (OP == 13) asm volatile("v_max_i32 %0, %1, %0" : "+v"(v[i]) : "v"(a));                                    \
    if (OP == 14) asm volatile("v_max3_f32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(fa), "v"(fa));                     \
    if (OP == 15) asm volatile("v_min_f32 %0, %1, %0" : "+v"(v[i]) : "v"(fa));                                   \
    if (OP == 16) asm volatile("v_max_f32_e64 %0, %1, %0" : "+v"(v[i]) : "v"(fa));                               \
    if (OP == 17) asm volatile("v_sub_f32 %0, %1, %0" : "+v"(v[i]) : "v"(fa));                                   \
    if (OP == 18) asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(v[i]) : "v"(a));                           \
    if (OP == 19) asm volatile("v_min3_f32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(fa), "v"(fa));                     \
    if (OP == 20) asm volatile("v_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(v[i]) : "v"(a), "s"(msk));              \
    if (OP == 21) asm volatile("v_cmp_lt_f32 vcc, %1, %0\n\tv_cndmask_b32 %0, %1, %0, vcc" : "+v"(v[i]) : "v"(fa) : "vcc"); \
    if (OP == 22) asm volatile("v_bfi_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(a), "v"(fa));                       \
    if (OP == 23) asm volatile("v_cmp_lt_f32_e64 %1, %2, %0\n\tv_cndmask_b32_e64 %0, %2, %0, %1" : "+v"(v[i]), "=s"(m2) : "v"(fa));
#pragma unroll
    for (int u = 0; u < 4; u++) { REP8(STEP) }
#undef STEP
  }
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_HW_ID, 32 bits
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID
  unsigned s = 0;
  for (int i = 0; i < 8; i++) s += v[i] + __float_as_uint(p[i].x) + __float_as_uint(p[i].y);
  s += (unsigned)m2 + (unsigned)msk;
  const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if ((threadIdx.x & 63) == 0) {
    out[5 * wave + 0] = t0;
    out[5 * wave + 1] = t1;
    out[5 * wave + 2] = r1 - r0;
    out[5 * wave + 3] = ((unsigned long long)(xcc & 0xf) << 32) | hw;
    out[5 * wave + 4] = s;
  }
}

struct Res { double cyc_exact_w, cyc_all, clock_ghz, event_ms, cyc_at_nominal; int simds_w, simds; };

template <int OP>
Res run(unsigned long long* out, int cus, int w, unsigned a, unsigned b, int iters) {
  const int wgs = w == 8 ? 2 * cus : cus;
  const int threads = w == 8 ? 1024 : 256 * w;  // 4 SIMDs x w waves x 64 lanes per CU
  const size_t lds = w == 8 ? 72 * 1024 : 96 * 1024;  // one (two for w = 8) workgroup(s) per CU of 160 KB
  hipFuncSetAttribute((const void*)k<OP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 3; rep++) {  // the last of three (clock and caches settled)
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<OP>, dim3(wgs), dim3(threads), lds, 0, out, a, b, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
  }
  if (hipGetLastError() != hipSuccess) { printf("launch failed\n"); exit(1); }
  const int waves = wgs * threads / 64;
  std::vector<unsigned long long> h(5 * (size_t)waves);
  hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost);
  // per (xcc, se, sh, cu, simd): first start, last end, wave count
  std::map<unsigned long long, std::array<unsigned long long, 3>> simd;
  std::vector<double> clk(waves);
  for (int i = 0; i < waves; i++) {
    const unsigned long long t0 = h[5 * i], t1 = h[5 * i + 1], id = h[5 * i + 3];
    const unsigned hw = (unsigned)id;
    const unsigned long long key = ((id >> 32) << 16) | (((hw >> 13) & 7) << 12) | (((hw >> 12) & 1) << 11) |
                                   (((hw >> 8) & 15) << 4) | ((hw >> 4) & 3);
    auto it = simd.find(key);
    if (it == simd.end()) simd[key] = {t0, t1, 1};
    else { it->second[0] = std::min(it->second[0], t0); it->second[1] = std::max(it->second[1], t1); it->second[2]++; }
    clk[i] = (double)(t1 - t0) / ((double)h[5 * i + 2] / 100e6) / 1e9;  // s_memrealtime: 100 MHz
  }
  const double per_wave = (double)iters * 32;  // instructions per wave
  std::vector<double> exact, all;
  for (auto& kv : simd) {
    const double c = (double)(kv.second[1] - kv.second[0]) / (kv.second[2] * per_wave);
    all.push_back(c);
    if ((int)kv.second[2] == w) exact.push_back(c);
  }
  std::sort(exact.begin(), exact.end());
  std::sort(all.begin(), all.end());
  std::sort(clk.begin(), clk.end());
  Res r;
  r.cyc_exact_w = exact.empty() ? 0 : exact[exact.size() / 2];
  r.cyc_all = all[all.size() / 2];
  r.simds_w = (int)exact.size();
  r.simds = (int)all.size();
  r.clock_ghz = clk[waves / 2];
  r.event_ms = ms;
  r.cyc_at_nominal = ms * 1e-3 * 2.4e9 / (w * per_wave);
  return r;
}

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  unsigned long long* out;
  hipMalloc(&out, 5 * 8 * (size_t)cus * 32);
  const int iters = 4096;
  printf("# %s, %d CUs; 8 independent chains per lane, inline-asm ops, one workgroup per CU\n", prop.gcnArchName, cus);
  printf("# cyc_w: median over SIMDs holding exactly w waves of (SIMD's s_memtime span) / (waves x instructions);\n");
  printf("# cyc_all: the same over every SIMD; simds: SIMDs with exactly w waves / all; cyc@2.4: event time at 2.4 GHz\n");
  printf("%-16s %5s %8s %8s %11s %10s %9s %9s\n", "op", "w/SIMD", "cyc_w", "cyc_all", "simds", "clock_GHz",
         "event_ms", "cyc@2.4");
  auto rep = [&](const char* n, int w, Res r) {
    printf("%-16s %5d %8.3f %8.3f %5d/%-5d %10.3f %9.3f %9.3f\n", n, w, r.cyc_exact_w, r.cyc_all, r.simds_w, r.simds,
           r.clock_ghz, r.event_ms, r.cyc_at_nominal);
    fflush(stdout);
  };
  for (int w : {1, 2, 4, 8}) {
    rep("v_fma_f32", w, run<0>(out, cus, w, 0x3f800001u, 7u, iters));
    rep("v_dot4_i32_i8", w, run<1>(out, cus, w, 0x01020304u, 7u, iters));
    rep("v_pk_fma_f32", w, run<2>(out, cus, w, 0x3f800001u, 7u, iters));
    rep("v_add_f32", w, run<3>(out, cus, w, 0x3f800001u, 7u, iters));
    rep("v_max_f32", w, run<4>(out, cus, w, 0x3f800001u, 7u, iters));
    rep("v_pk_mul_f32", w, run<5>(out, cus, w, 0x3f800001u, 7u, iters));
    rep("v_mov_b32", w, run<6>(out, cus, w, 3u, 7u, iters));
    rep("v_pk_add_f32", w, run<7>(out, cus, w, 0x3f800001u, 7u, iters));
    rep("v_sub_u32", w, run<8>(out, cus, w, 3u, 7u, iters));
    rep("v_mul_f32", w, run<9>(out, cus, w, 0x3f800001u, 7u, iters));
    rep("v_add_f32_e64", w, run<10>(out, cus, w, 0x3f800001u, 7u, iters));
    rep("v_fmac_f32", w, run<11>(out, cus, w, 0x3f800001u, 7u, iters));
    rep("v_med3_f32", w, run<12>(out, cus, w, 0x3f800001u, 7u, iters));
    rep("v_max_i32", w, run<13>(out, cus, w, 3u, 7u, iters));
    rep("v_max3_f32", w, run<14>(out, cus, w, 0x3f800001u, 7u, iters));
    rep("v_min_f32", w, run<15>(out, cus, w, 0x3f800001u, 7u, iters));
    rep("v_max_f32_e64", w, run<16>(out, cus, w, 0x3f800001u, 7u, iters));
    rep("v_sub_f32", w, run<17>(out, cus, w, 0x3f800001u, 7u, iters));
    rep("v_cndmask_b32", w, run<18>(out, cus, w, 3u, 7u, iters));
    rep("v_min3_f32", w, run<19>(out, cus, w, 0x3f800001u, 7u, iters));
    rep("cndmask_e64_s", w, run<20>(out, cus, w, 3u, 7u, iters));
    rep("cmp+cndmask_vcc", w, run<21>(out, cus, w, 0x3f800001u, 7u, iters));
    rep("v_bfi_b32", w, run<22>(out, cus, w, 3u, 7u, iters));
    rep("cmp+cndmask_s", w, run<23>(out, cus, w, 0x3f800001u, 7u, iters));
  }
  return 0;
}
