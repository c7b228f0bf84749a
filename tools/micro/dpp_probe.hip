// Prints what __builtin_amdgcn_update_dpp returns per lane for row_shr:1 / row_shl:1 with an "old"
// operand (bound_ctrl false): documents the lane mapping gdfn.hip's column shifts rely on.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(int* out) {
  const int l = threadIdx.x;
  out[l] = __builtin_amdgcn_update_dpp(1000 + l, l, 0x111, 0xf, 0xf, false);
  out[64 + l] = __builtin_amdgcn_update_dpp(1000 + l, l, 0x101, 0xf, 0xf, false);
  float v = (float)l, o = 1000.f + l;
  out[128 + l] = (int)__builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, o), __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, false));
}

int main() {
  int* d;
  if (hipMalloc(&d, 192 * sizeof(int)) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  int h[192];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  for (int k = 0; k < 3; ++k) {
    printf("%s:", k == 0 ? "shr1" : k == 1 ? "shl1" : "shr1f");
    for (int l = 0; l < 20; ++l) printf(" %d", h[64 * k + l]);
    printf("\n");
  }
  return 0;
}
