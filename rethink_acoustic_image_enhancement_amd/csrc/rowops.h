// Row operations shared by the GEMM kernels (gemm.hip) and the fused feed-forward half (ffn.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace kdlae {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// LayerNorm over channels of RT row subtiles held in registers (lane (li, lq): pixel li, channels
// 16 g + 4 lq .. + 3 of k-group g; the 4 lanes of a pixel reduce with xor-shuffles over lq), BiasFree
// (ln 1: x / sqrt(var + eps), KDLAE_model.py:50-52) or WithBias (ln 2: (x - mean) / ..., :67-70); the
// LN weight / bias are folded into the next GEMM.  Only the first `kgroups` k-groups count in the
// variance (padding groups hold zeros).  No fp contraction: every kernel that normalises a row must
// round the variance and the shift the same way, whatever code surrounds it (with hipcc's default
// fp-contract=fast the split-MFMA kernels contracted d.x * d.x + d.y * d.y differently from one another).
template <int KG, int RT>
__device__ __forceinline__ void ln_rows(int ln, int lnC, int kgroups, f32x4 (&a)[RT][KG]) {
#pragma clang fp contract(off)
  const float wb = (ln == 2) ? 1.f : 0.f;
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < KG; ++g) s += (a[r][g].x + a[r][g].y) + (a[r][g].z + a[r][g].w);
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    const float mean = s / (float)lnC;
    float v2 = 0.f;
#pragma unroll
    for (int g = 0; g < KG; ++g) {
      const f32x4 d = a[r][g] - mean;
      const float dd = (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
      v2 += (g < kgroups) ? dd : 0.f;
    }
    v2 += __shfl_xor(v2, 16);
    v2 += __shfl_xor(v2, 32);
    const float rstd = 1.0f / sqrtf(v2 / (float)lnC + 1e-5f);
    const float sh = mean * wb;
#pragma unroll
    for (int g = 0; g < KG; ++g) a[r][g] = (a[r][g] - sh) * rstd;
  }
}

}  // namespace kdlae
