// VALU issue-rate probe (round 5): cycles per wave64 VALU instruction per SIMD
// at 1, 2, 4 and 8 waves per SIMD, counted in shader clocks by s_memtime inside
// each wave (independent of the clock the chip runs at), with every measured
// instruction written as inline asm so the compiler cannot pair scalar FP32 ops
// into v_pk_* forms (what made an earlier probe read "FP32 at 2 cycles").
//
// Layout: one workgroup per CU (96 KB of dynamic LDS), 4*w waves per workgroup,
// so w waves on each SIMD; 8 independent accumulator chains per lane; the
// measured loop is 8 x UNR instructions per trip.  cycles/instr/SIMD =
// (wave's s_memtime delta) / (w * instructions per wave).  The clock is the
// s_memtime delta over the s_memrealtime (100 MHz) delta of the same wave.
//
//   hipcc -O3 --offload-arch=gfx950 valu_rate3.hip -o valu_rate3 && ./valu_rate3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

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
    if (OP == 8) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(v[i]) : "v"(a));
#pragma unroll
    for (int u = 0; u < 4; u++) { REP8(STEP) }
#undef STEP
  }
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  unsigned s = 0;
  for (int i = 0; i < 8; i++) s += v[i] + __float_as_uint(p[i].x) + __float_as_uint(p[i].y);
  const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if ((threadIdx.x & 63) == 0) {
    out[3 * wave + 0] = t1 - t0;
    out[3 * wave + 1] = r1 - r0;
    out[3 * wave + 2] = s;
  }
}

struct Res { double cyc_per_instr, clock_ghz, event_ms, cyc_at_nominal; };

template <int OP>
Res run(unsigned long long* out, int cus, int w, unsigned a, unsigned b, int iters) {
  const int threads = 256 * w;  // 4 SIMDs x w waves x 64 lanes
  const size_t lds = 96 * 1024;  // one workgroup per CU (160 KB LDS per CU)
  hipFuncSetAttribute((const void*)k<OP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 3; rep++) {  // the last of three (clock and caches settled)
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<OP>, dim3(cus), dim3(threads), lds, 0, out, a, b, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
  }
  const int waves = cus * threads / 64;
  std::vector<unsigned long long> h(3 * (size_t)waves);
  hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> cyc(waves), clk(waves);
  for (int i = 0; i < waves; i++) {
    cyc[i] = (double)h[3 * i];
    clk[i] = (double)h[3 * i] / ((double)h[3 * i + 1] / 100e6) / 1e9;  // s_memrealtime: 100 MHz
  }
  std::sort(cyc.begin(), cyc.end());
  std::sort(clk.begin(), clk.end());
  const double per_wave = (double)iters * 32;  // instructions per wave
  Res r;
  r.cyc_per_instr = cyc[waves / 2] / (w * per_wave);  // median wave
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
  hipMalloc(&out, 3 * 8 * (size_t)cus * 32);
  const int iters = 4096;
  printf("# %s, %d CUs; 8 independent chains per lane, inline-asm ops, one workgroup per CU\n", prop.gcnArchName, cus);
  printf("# cyc = median wave's s_memtime delta / (waves per SIMD x instructions per wave)\n");
  printf("%-16s %5s %10s %10s %10s %12s\n", "op", "w/SIMD", "cyc/instr", "clock_GHz", "event_ms", "cyc@2.4GHz");
  auto rep = [&](const char* n, int w, Res r) {
    printf("%-16s %5d %10.3f %10.3f %10.3f %12.3f\n", n, w, r.cyc_per_instr, r.clock_ghz, r.event_ms, r.cyc_at_nominal);
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
  }
  return 0;
}
