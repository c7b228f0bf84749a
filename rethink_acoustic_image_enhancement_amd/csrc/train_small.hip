// Weight gradient of the training step's 3x3 convs with a 3- or 4-channel side (gfx950): the image
// heads output / output2 / outputen (Cout = 3, KDLAE_model.py:258,261,268) and the cen / patch_embed
// / output_param inputs (Cin = 3 / 4, :173,:259,:265).  As a tiled GEMM these are M or N = 3 of a
// 64-wide tile (the 393216-pixel outputen dW took 450 us, 0.3 TF/s); here a lane owns one channel of
// the wide side and accumulates its 9 x S products over a run of pixels on the VALU:
//   SMALL_OUT (Cout = S): dW[s][c][t] += dY[p][s] * X[p + off_t][c]    (X is the wide side)
//   else      (Cin  = S): dW[c][s][t] += dY[p][c] * X[p + off_t][s]    (dY is the wide side)
// Zero padding = dil.  Threads of a block are (pixel lane, channel) with channels fastest, so every
// wide-side load is a coalesced row segment; a block walks a contiguous pixel range, the pixel lanes
// are summed in fixed order in LDS and the block's [Cout][Cin][9] partial is written to part[block]
// for the caller's fixed-order column reduce: deterministic, no atomics.
#include "train_kernels.h"

namespace kdlae {
namespace train {

namespace {

constexpr int kPU = 4;  // pixels per lane per step: their loads are issued together (memory-level parallelism)

template <int S, bool SMALL_OUT>
__global__ __launch_bounds__(256) void dw3_small_kernel(const float* __restrict__ dy, int ldd,
                                                        const float* __restrict__ x, int ldx, int Cb, int H, int W,
                                                        int dil, long long P, long long per_block,
                                                        float* __restrict__ part) {
  __shared__ float red[256 * 9];  // one small channel's [G][Cb][9] partials at a time (G * Cb <= 256)
  const int G = 256 / Cb;         // pixel lanes (blockDim = G * Cb rounded up to whole waves)
  const int tid = threadIdx.x;
  const int c = tid % Cb, pl = tid / Cb;
  const bool act = pl < G;
  const long long p0 = blockIdx.x * per_block, p1 = min(P, p0 + per_block);
  const long long HW = (long long)H * W;
  float acc[S][9];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[s][t] = 0.f;
  if (act) {
    for (long long pb = p0 + pl; pb < p1; pb += (long long)kPU * G) {
      // the wide side's 9 taps (SMALL_OUT: X; else dY once) and the narrow side's values of kPU pixels
      float big[kPU][SMALL_OUT ? 9 : 1], nar[kPU][SMALL_OUT ? 1 : 9][S];
#pragma unroll
      for (int u = 0; u < kPU; ++u) {
        const long long p = pb + (long long)u * G;
        const bool pv = p < p1;
        const long long pc = pv ? p : p0;
        // 32-bit index math (the launcher checks P < 2^31): 64-bit division is a long call per pixel
        const unsigned pu = (unsigned)pc;
        const unsigned img = pu / (unsigned)HW;
        const int rem = (int)(pu - img * (unsigned)HW);
        const int y = rem / W, xx0 = rem - y * W;
        const float* xi = x + (long long)img * HW * ldx;
        if constexpr (SMALL_OUT) {
#pragma unroll
          for (int s = 0; s < S; ++s) nar[u][0][s] = pv ? dy[pc * ldd + s] : 0.f;
#pragma unroll
          for (int t = 0; t < 9; ++t) {
            const int yy = y + (t / 3 - 1) * dil, xx = xx0 + (t % 3 - 1) * dil;
            const bool ok = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
            big[u][t] = ok ? xi[((long long)yy * W + xx) * ldx + c] : 0.f;
          }
        } else {
          big[u][0] = pv ? dy[pc * ldd + c] : 0.f;
#pragma unroll
          for (int t = 0; t < 9; ++t) {
            const int yy = y + (t / 3 - 1) * dil, xx = xx0 + (t % 3 - 1) * dil;
            const bool ok = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
            const float* xr = xi + (ok ? ((long long)yy * W + xx) * ldx : 0);
#pragma unroll
            for (int s = 0; s < S; ++s) nar[u][t][s] = ok ? xr[s] : 0.f;
          }
        }
      }
      // accumulate in pixel order (a fixed order for a given launch shape)
#pragma unroll
      for (int u = 0; u < kPU; ++u)
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int s = 0; s < S; ++s)
            acc[s][t] = SMALL_OUT ? fmaf(nar[u][0][s], big[u][t], acc[s][t]) : fmaf(big[u][0], nar[u][t][s], acc[s][t]);
    }
  }
  // fixed-order sum over the pixel lanes, one small channel at a time through LDS
  float* out = part + (long long)blockIdx.x * Cb * S * 9;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    __syncthreads();
    if (act)
#pragma unroll
      for (int t = 0; t < 9; ++t) red[(pl * Cb + c) * 9 + t] = acc[s][t];
    __syncthreads();
    for (int i = tid; i < Cb * 9; i += blockDim.x) {
      float v = 0.f;
      for (int g = 0; g < G; ++g) v += red[g * Cb * 9 + i];
      const int cc = i / 9, t = i - (i / 9) * 9;
      // dW[co][ci][t]: (s, cc) when the output side is small, else (cc, s)
      out[(SMALL_OUT ? (s * Cb + cc) : (cc * S + s)) * 9 + t] = v;
    }
  }
}

}  // namespace

// instances: the released heads' shapes (3-channel images: Cout 3 heads, Cin 3 cen / patch_embed,
// Cin 4 output_param on cat[out, denoise_rate]); any other narrow side takes the tiled GEMM
bool dw3_small_ok(int Cin, int Cout) {
  if (Cout == 3) return Cin >= 1 && Cin <= 256;
  return (Cin == 3 || Cin == 4) && Cout >= 1 && Cout <= 256;
}

int dw3_small_blocks(long long P, int Cin, int Cout, size_t part_cap) {
  const long long ncols = (long long)Cin * Cout * 9;
  long long nb = (P + 47) / 48;  // >= 48 pixels per block: enough blocks to fill the chip several times
  if (nb > 2048) nb = 2048;
  const long long cap = (long long)(part_cap / (size_t)ncols);
  if (nb > cap) nb = cap;
  return nb < 1 ? 1 : (int)nb;
}

hipError_t launch_dw3_small(const float* dy, int ldd, const float* x, int ldx, int Cin, int Cout, int Bn, int H, int W,
                            int dil, float* part, int nblk, hipStream_t s) {
  if (!dw3_small_ok(Cin, Cout) || nblk < 1) return hipErrorInvalidValue;
  const long long P = (long long)Bn * H * W;
  if (P >= (1LL << 31)) return hipErrorInvalidValue;
  const long long per = (P + nblk - 1) / nblk;
  const bool so = Cout == 3;
  const int S = so ? Cout : Cin, Cb = so ? Cin : Cout;
  const int threads = ((256 / Cb) * Cb + 63) / 64 * 64;  // whole waves over the (pixel lane, channel) grid
  if (so)
    hipLaunchKernelGGL((dw3_small_kernel<3, true>), dim3(nblk), dim3(threads), 0, s, dy, ldd, x, ldx, Cb, H, W, dil, P,
                       per, part);
  else if (S == 3)
    hipLaunchKernelGGL((dw3_small_kernel<3, false>), dim3(nblk), dim3(threads), 0, s, dy, ldd, x, ldx, Cb, H, W, dil, P,
                       per, part);
  else
    hipLaunchKernelGGL((dw3_small_kernel<4, false>), dim3(nblk), dim3(threads), 0, s, dy, ldd, x, ldx, Cb, H, W, dil, P,
                       per, part);
  return hipGetLastError();
}

}  // namespace train
}  // namespace kdlae
