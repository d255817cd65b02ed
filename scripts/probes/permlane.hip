// Probe: lane mapping of v_permlane16/32_swap (gfx950) as exposed by the
// clang builtins (both results), and DPP row_shl.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* o) {
  int l = threadIdx.x;
  auto a = __builtin_amdgcn_permlane32_swap(l, l + 100, false, false);
  auto b = __builtin_amdgcn_permlane16_swap(l, l + 100, false, false);
  o[l] = a[0]; o[64 + l] = a[1]; o[128 + l] = b[0]; o[192 + l] = b[1];
  o[256 + l] = __builtin_amdgcn_mov_dpp(l, 0x101, 0xf, 0xf, true);  // row_shl:1
}
int main() {
  int* d; hipMalloc(&d, 4 * 320);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[320]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* n[] = {"p32[0]", "p32[1]", "p16[0]", "p16[1]", "shl1"};
  for (int r = 0; r < 5; r++) { printf("%s:", n[r]); for (int i = 0; i < 64; i++) printf(" %d", h[r * 64 + i]); printf("\n"); }
}
