// Probe: operand/result lane maps of v_mfma_i32_16x16x64_i8 on gfx950 (checked
// on the host against A[l&15][16(l>>4)+j], B[16(l>>4)+j][l&15], C[4(l>>4)+r][l&15]),
// and LDS float atomic max (ds_max_f32) on -inf / mixed-sign / NaN operands.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef int i32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const i32x4* a, const i32x4* b, i32x4* c, const float* mv, float* mo) {
  int l = threadIdx.x;
  c[l] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[l], b[l], i32x4{0, 0, 0, 0}, 0, 0, 0);
  __shared__ float s[8];
  if (l < 8) s[l] = -INFINITY;
  __syncthreads();
  __hip_atomic_fetch_max(&s[l & 7], mv[l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __syncthreads();
  if (l < 8) mo[l] = s[l];
}
int main() {
  signed char A[64][16], B[64][16];
  srand(1);
  for (int l = 0; l < 64; l++)
    for (int j = 0; j < 16; j++) { A[l][j] = (signed char)(rand() % 256 - 128); B[l][j] = (signed char)(rand() % 256 - 128); }
  float mv[64];
  for (int l = 0; l < 64; l++) mv[l] = (l & 7) == 0 ? NAN : (float)((l * 37) % 19) - 9.5f;
  mv[7] = NAN; mv[15] = NAN; mv[23] = NAN; mv[31] = NAN; mv[39] = NAN; mv[47] = NAN; mv[55] = NAN; mv[63] = NAN;  // slot 7 all NaN
  i32x4 *da, *db, *dc; float *dmv, *dmo;
  hipMalloc(&da, 1024); hipMalloc(&db, 1024); hipMalloc(&dc, 1024); hipMalloc(&dmv, 256); hipMalloc(&dmo, 32);
  hipMemcpy(da, A, 1024, hipMemcpyHostToDevice); hipMemcpy(db, B, 1024, hipMemcpyHostToDevice);
  hipMemcpy(dmv, mv, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dc, dmv, dmo);
  int C[64][4]; float mo[8];
  hipMemcpy(C, dc, 1024, hipMemcpyDeviceToHost); hipMemcpy(mo, dmo, 32, hipMemcpyDeviceToHost);
  // hypothesis
  int Am[16][64], Bm[64][16];
  for (int l = 0; l < 64; l++) for (int j = 0; j < 16; j++) { Am[l & 15][16 * (l >> 4) + j] = A[l][j]; Bm[16 * (l >> 4) + j][l & 15] = B[l][j]; }
  int bad = 0;
  for (int l = 0; l < 64; l++) for (int r = 0; r < 4; r++) {
    int row = 4 * (l >> 4) + r, col = l & 15, s = 0;
    for (int k = 0; k < 64; k++) s += Am[row][k] * Bm[k][col];
    if (s != C[l][r]) bad++;
  }
  printf("mfma_i32_16x16x64_i8 layout mismatches: %d of 256\n", bad);
  for (int i = 0; i < 8; i++) {
    float ref = -INFINITY;
    for (int l = i; l < 64; l += 8) if (!std::isnan(mv[l]) && mv[l] > ref) ref = mv[l];
    printf("ds_max slot %d: got %g, maxNum %g\n", i, mo[i], ref);
  }
}
