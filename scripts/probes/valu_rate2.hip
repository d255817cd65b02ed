// Micro-probe 2: issue cost per wave-instruction per SIMD of candidate NCC
// inner-loop ops (8 independent accumulator chains per lane, 32 waves per CU):
// the integer dot4 forms vs the f16/bf16 dot2 forms (exact for |q| <= 128).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef short bf16x2_t __attribute__((ext_vector_type(2)));
template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned a, unsigned b, int iters) {
  unsigned v[8];
  float f[8];
  for (int i = 0; i < 8; i++) { v[i] = threadIdx.x * (i + 1); f[i] = (float)v[i]; }
  const half2_t ha = __builtin_bit_cast(half2_t, a), hb = __builtin_bit_cast(half2_t, b);
  const bf16x2_t ba = __builtin_bit_cast(bf16x2_t, a), bb = __builtin_bit_cast(bf16x2_t, b);
  const float fa = __int_as_float(a);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (OP == 0) v[i] = (unsigned)__builtin_amdgcn_sdot4((int)a, (int)b, (int)v[i], false);
      if (OP == 1) { unsigned r; asm volatile("v_dot4_i32_i8 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(v[i])); v[i] = r; }
      if (OP == 2) f[i] = __builtin_amdgcn_fdot2(ha, hb, f[i], false);
      if (OP == 3) f[i] = __builtin_amdgcn_fdot2_f32_bf16(ba, bb, f[i], false);
      if (OP == 4) f[i] = f[i] - fa;
      if (OP == 5) { float r; asm volatile("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(f[i]), "v"(fa)); f[i] = r; }
      if (OP == 6) { unsigned r; asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v[i])); v[i] = r; }
      if (OP == 7) { float r; asm volatile("v_dot2_f32_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(f[i])); f[i] = r; }
      if (OP == 8) { float r; asm volatile("v_dot2c_f32_bf16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b), "0"(f[i])); f[i] = r; }
      if (OP == 9) v[i] = v[i] - a;
      if (OP == 10) { typedef float f2 __attribute__((ext_vector_type(2))); f2 t = {f[i], __int_as_float(v[i])};
        t = __builtin_elementwise_fma(t, f2{fa, fa}, f2{fa, fa}); f[i] = t.x; v[i] = __float_as_int(t.y); }
      if (OP == 11) f[i] = __builtin_fmaf(f[i], fa, fa);
      if (OP == 12) f[i] = f[i] / (fa + (float)i);
      if (OP == 13) f[i] = sqrtf(f[i] + fa);
    }
  }
  unsigned s = 0;
  for (int i = 0; i < 8; i++) s += v[i] + __float_as_int(f[i]);
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int OP>
float run(unsigned* out, unsigned a, unsigned b, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 2; rep++) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<OP>, dim3(8192), dim3(256), 0, 0, out, a, b, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
  }
  return ms;
}
int main() {
  unsigned* out;
  hipMalloc(&out, 4 * 256 * 8192);
  const int iters = 2048;
  const double instrs = 8192.0 * 4 * iters * 8;
  auto rep = [&](const char* n, float ms) {
    printf("%-22s %.3f ms  %.2f cycles per wave-instruction per SIMD (at 2.4 GHz)\n", n, ms,
           ms * 1e-3 * 2.4e9 / (instrs / 1024.0));
  };
  rep("v_dot4c_i32_i8", run<0>(out, 0x01020304u, 7u, iters));
  rep("v_dot4_i32_i8 (VOP3P)", run<1>(out, 0x01020304u, 7u, iters));
  rep("v_dot2_f32_f16", run<2>(out, 0x3c003c00u, 0x3c003c00u, iters));
  rep("v_dot2_f32_bf16", run<3>(out, 0x3f803f80u, 0x3f803f80u, iters));
  rep("v_sub_f32", run<4>(out, 0x3f800001u, 7u, iters));
  rep("v_max_f32", run<5>(out, 0x3f800001u, 7u, iters));
  rep("v_mov_b32", run<6>(out, 3u, 7u, iters));
  rep("v_dot2_f32_f16 (asm)", run<7>(out, 0x3c003c00u, 0x3c003c00u, iters));
  rep("v_dot2c_f32_bf16 (asm)", run<8>(out, 0x3f803f80u, 0x3f803f80u, iters));
  rep("v_sub_u32", run<9>(out, 3u, 7u, iters));
  rep("v_pk_fma_f32 (2 values)", run<10>(out, 0x3f800001u, 7u, iters));
  rep("v_fma_f32", run<11>(out, 0x3f800001u, 7u, iters));
  rep("IEEE f32 divide (sequence)", run<12>(out, 0x3f800001u, 7u, iters));
  rep("IEEE f32 sqrt (sequence)", run<13>(out, 0x3f800001u, 7u, iters));
  return 0;
}
