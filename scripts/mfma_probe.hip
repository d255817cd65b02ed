#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
// variant 0: lane l holds A[l&31][16*(l>>5) + j], j=0..15 ; B[16*(l>>5)+j][l&31]
// variant 1: lane l holds A[l&31][8*(l>>5) + j] j<8 and A[..][16 + 8*(l>>5) + (j-8)] j>=8
__global__ void k(const int8_t* A, const int8_t* B, int* D, int variant) {
  int l = threadIdx.x, r = l & 31, h = l >> 5;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; j++) {
    int kk = variant == 0 ? 16 * h + j : (j < 8 ? 8 * h + j : 16 + 8 * h + (j - 8));
    a[j] = A[r * 32 + kk];
    b[j] = B[kk * 32 + r];
  }
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  v16i c = {0};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
  for (int reg = 0; reg < 16; reg++) {
    int row = (reg & 3) + 8 * (reg >> 2) + 4 * h, col = r;
    D[row * 32 + col] = c[reg];
  }
}
int main() {
  int8_t A[1024], B[1024];
  srand(1);
  for (int i = 0; i < 1024; i++) { A[i] = (int8_t)(rand() % 256 - 128); B[i] = (int8_t)(rand() % 256 - 128); }
  int ref[1024];
  for (int i = 0; i < 32; i++) for (int j = 0; j < 32; j++) { int s = 0; for (int k = 0; k < 32; k++) s += A[i*32+k]*B[k*32+j]; ref[i*32+j] = s; }
  int8_t *dA, *dB; int* dD; int D[1024];
  hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dD, 4096);
  hipMemcpy(dA, A, 1024, hipMemcpyHostToDevice); hipMemcpy(dB, B, 1024, hipMemcpyHostToDevice);
  for (int v = 0; v < 2; v++) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD, v);
    hipMemcpy(D, dD, 4096, hipMemcpyDeviceToHost);
    int bad = 0; for (int i = 0; i < 1024; i++) bad += D[i] != ref[i];
    printf("variant %d: %d mismatches\n", v, bad);
  }
  return 0;
}
