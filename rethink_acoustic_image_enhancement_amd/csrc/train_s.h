// Launch interface of the KDLAE-S training kernels (train_s.hip).  NDHWC views: [B][F][H][W] pixels,
// channels contiguous at a pixel stride.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>

namespace kdlae {
namespace train {

// Xcol[p][tap * C + c] = x[p + off(tap)][c] (zero padding 1 in frames, rows, columns); [P][27 C]
hipError_t launch_im2col3d(const float* x, int ldx, int C, int B, int F, int H, int W, float* col, hipStream_t s);
// dx[q][c] (+)= sum_tap dcol[q - off(tap)][tap * C + c]
hipError_t launch_col2im3d(const float* dcol, int C, int B, int F, int H, int W, float* dx, int lddx, int accumulate,
                           hipStream_t s);
// Conv3d weight order: dir 0 [O][C][27] (OIDHW) -> [O][27][C] (the column order); dir 1 back
hipError_t launch_wperm(const float* src, float* dst, int O, int C, int dir, hipStream_t s);
// packed (fragment-order, k = tap * in_pad + c) weights of a Conv3d 3x3x3 [cout][cin][27] for the inference
// conv kernels: dx = 0 the forward conv (cout outputs), dx = 1 the input-gradient conv (cin outputs, taps
// flipped); ceil(nout/16) * 27 in_pad/16 * 256 floats
hipError_t launch_pack_conv(const float* w, int cout, int cin, int dx, float* wp, hipStream_t s);
hipError_t launch_relu(float* y, int ld, int C, long long P, hipStream_t s);
// dy *= (y > 0)
hipError_t launch_relu_mask(float* dy, int ldd, const float* y, int ldy, int C, long long P, hipStream_t s);
// MaxPool3d (1,2,2) backward over the pooled grid [B][F][h][w]: din = dskip (or 0) + dout routed to the
// window's first maximum of `in`
hipError_t launch_maxpool2_bwd(const float* in, int ldi, const float* dout, int ldo, const float* dskip, int lds,
                               float* din, int ldd, int C, int B, int F, int h, int w, hipStream_t s);
// ConvTranspose3d (1,2,2) s (1,2,2) output + bias + skip: D[2y+i][2x+j][o] = U[y][x][4o+2i+j] + b[o] + skip
// (H, W: the output grid)
hipError_t launch_upshuffle_add(const float* U, int ldu, const float* bias, const float* skip, int lds, float* D,
                                int ldd, int C, int B, int F, int H, int W, hipStream_t s);
// L1LossForVideoFrames (losses.py:409-526) with reduction 'mean' (sum_reduction 0) or 'sum'
int l1frames_scratch_floats();
hipError_t launch_l1frames(const float* pred, const float* tgt, int N, int Cf, long long HW, float l1_weight,
                           float temporal_weight, float binary, int sum_reduction, float* dpred, float* loss,
                           float* scratch, hipStream_t s);

}  // namespace train
}  // namespace kdlae
