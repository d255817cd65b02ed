// Micro-probe: issue cost per wave-instruction per SIMD of the VALU ops the
// NCC finish uses (8 independent chains per lane, 32 waves per CU).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef float float2_t __attribute__((ext_vector_type(2)));
template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned a, unsigned b, int iters) {
  unsigned v[8];
  float f[8];
  float2_t p[8];
  for (int i = 0; i < 8; i++) { v[i] = threadIdx.x * (i + 1); f[i] = (float)v[i]; p[i] = float2_t{f[i], f[i] + 1}; }
  const float fa = __int_as_float(a), fb = __int_as_float(b);
  half2_t ha = __builtin_bit_cast(half2_t, a);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (OP == 0) v[i] = __builtin_amdgcn_udot4(v[i], a, b, false);
      if (OP == 1) v[i] = (unsigned)__builtin_amdgcn_sdot4((int)v[i], (int)a, (int)b, false);
      if (OP == 2) f[i] = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, v[i] + it), ha, f[i], false);
      if (OP == 3) v[i] = v[i] + a;
      if (OP == 4) f[i] = f[i] * fa;
      if (OP == 5) f[i] = __builtin_fmaf(f[i], fa, fb);
      if (OP == 6) { int t = (int)v[i]; v[i] = (unsigned)__float_as_int((float)t); }
      if (OP == 7) p[i] = p[i] * float2_t{fa, fb};
      if (OP == 8) v[i] = __mul24(v[i], a);
    }
  }
  unsigned s = 0;
  for (int i = 0; i < 8; i++) s += v[i] + __float_as_int(f[i]) + __float_as_int(p[i].x + p[i].y);
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
  const int iters = 4096;
  const double instrs = 8192.0 * 4 * iters * 8;
  auto rep = [&](const char* n, float ms) {
    printf("%-18s %.3f ms  %.2f cycles per wave-instruction per SIMD\n", n, ms, ms * 1e-3 * 2.4e9 / (instrs / 1024.0));
  };
  rep("v_dot4_u32_u8", run<0>(out, 0x01020304u, 7u, iters));
  rep("v_dot4_i32_i8", run<1>(out, 0x01020304u, 7u, iters));
  rep("v_dot2_f32_f16", run<2>(out, 0x3c003c00u, 7u, iters));
  rep("v_add_u32", run<3>(out, 3u, 7u, iters));
  rep("v_mul_f32", run<4>(out, 0x3f800001u, 7u, iters));
  rep("v_fma_f32", run<5>(out, 0x3f800001u, 0x3f800000u, iters));
  rep("v_cvt_f32_i32", run<6>(out, 3u, 7u, iters));
  rep("v_pk_mul_f32", run<7>(out, 0x3f800001u, 0x3f800001u, iters));
  rep("v_mul_u32_u24", run<8>(out, 3u, 7u, iters));
  return 0;
}
