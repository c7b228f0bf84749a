// KDLAE-S training kernels (gfx950): the data-movement and elementwise pieces of the student's
// backward that are not GEMMs (kdlae_st.cpp sequences them around the training GEMM, train.hip).
//
// Activations are NDHWC: [B][F][H][W] pixels, channels contiguous at pixel stride ld.  The Conv3d
// 3x3x3 (padding 1, KDLAE/KDLAE_model.py:386-393) goes through an explicit column matrix
//   Xcol[p][tap * C + c],  tap = dt * 9 + dy * 3 + dx,  source pixel (f + dt - 1, y + dy - 1, x + dx - 1)
// tap-major, so consecutive threads touch consecutive channels of one source pixel (coalesced on both
// sides; a channel-major order made im2col / col2im 75% of the step).  The weights are permuted to the
// same order per step ([Cout][27][Cin], launch_wperm), so the forward is Xcol . W'^T, the weight
// gradient dZ^T . Xcol (permuted back into the OIDHW gradient) and the input gradient col2im(dZ . W').
#include "train_kernels.h"
#include "train_s.h"

namespace kdlae {
namespace train {

namespace {

struct Geo {
  int B, F, H, W;
  __device__ void coords(long long p, int& b, int& f, int& y, int& x) const {
    x = (int)(p % W);
    long long r = p / W;
    y = (int)(r % H);
    r /= H;
    f = (int)(r % F);
    b = (int)(r / F);
  }
};

constexpr int kThreads = 256;

inline unsigned grid_for(long long n, int per_block = kThreads) {
  long long g = (n + per_block - 1) / per_block;
  if (g > (1LL << 20)) g = 1LL << 20;  // grid-stride loops cover the rest
  return (unsigned)(g < 1 ? 1 : g);
}

// 32-bit pixel coordinates (P < 2^31; only addresses are 64-bit: 64-bit division is a long software
// sequence on CDNA and dominated the first version of these kernels)
struct Geo32 {
  int F, H, W;
  __device__ void coords(int p, int& bf, int& f, int& y, int& x) const {
    x = p % W;
    int r = p / W;
    y = r % H;
    r /= H;
    f = r % F;
    bf = r - f;  // b * F
  }
};

template <int V> struct VecT;
template <> struct VecT<1> { using T = float; };
template <> struct VecT<4> { using T = float4; };

// Xcol rows are K = 27 C floats; a thread owns V consecutive channels of one (tap, channel group) column
// slot, fixed for the whole launch, and walks pixels.  With KV = 27 C / V <= 256 slots a block covers
// 256 / KV pixels per step; otherwise each block covers one pixel per step and threads stride the row.
template <int V>
__global__ __launch_bounds__(kThreads) void im2col3d_kernel(const float* __restrict__ x, int ldx, int C, Geo32 g,
                                                            int P, float* __restrict__ col) {
  using T = typename VecT<V>::T;
  const int CV = C / V, KV = 27 * CV;
  const int ppb = KV <= kThreads ? kThreads / KV : 1;
  const int sub = KV <= kThreads ? (int)threadIdx.x / KV : 0;
  if (sub >= ppb) return;
  const int kv0 = KV <= kThreads ? (int)threadIdx.x - sub * KV : (int)threadIdx.x;
  // 64-bit loop index: p + the grid stride must not wrap for P close to 2^31
  for (long long pl = (long long)blockIdx.x * ppb + sub; pl < P; pl += (long long)gridDim.x * ppb) {
    const int p = (int)pl;
    int bf, f, y, xx;
    g.coords(p, bf, f, y, xx);
    T* dst = reinterpret_cast<T*>(col + (long long)p * 27 * C);
    for (int kv = kv0; kv < KV; kv += kThreads) {
      const int tap = kv / CV, c = (kv - tap * CV) * V;
      const int ff = f + tap / 9 - 1, yy = y + (tap / 3) % 3 - 1, xs = xx + tap % 3 - 1;
      T v;
      if ((unsigned)ff < (unsigned)g.F && (unsigned)yy < (unsigned)g.H && (unsigned)xs < (unsigned)g.W)
        v = *reinterpret_cast<const T*>(x + ((long long)((bf + ff) * g.H + yy) * g.W + xs) * ldx + c);
      else
        v = T{};
      dst[kv] = v;
    }
  }
}

// dX[q][c] (+)= sum over taps of dcol[q - off(tap)][tap * C + c] (the pixels whose window put q at that
// tap): a gather, so every dX element is written once, in a fixed order (deterministic, no atomics).
// One thread per (pixel, V-channel group).
template <int V>
__global__ __launch_bounds__(kThreads) void col2im3d_kernel(const float* __restrict__ dcol, int C, Geo32 g, int P,
                                                            float* __restrict__ dx, int lddx, int accumulate) {
  using T = typename VecT<V>::T;
  const int CV = C / V;
  const int n = P * CV;  // < 2^31 (checked by the launcher)
  const long long K = 27LL * C;
  // 64-bit loop index: i + the grid stride (up to 2^28) must not wrap for n close to 2^31
  for (long long il = (long long)blockIdx.x * kThreads + threadIdx.x; il < n; il += (long long)gridDim.x * kThreads) {
    const int i = (int)il;
    const int q = i / CV;
    const int c = (i - q * CV) * V;
    int bf, f, y, x;
    g.coords(q, bf, f, y, x);
    T s{};
#pragma unroll
    for (int tap = 0; tap < 27; ++tap) {
      // source pixel p with p + off(tap) = q
      const int pf = f - (tap / 9 - 1), py = y - ((tap / 3) % 3 - 1), px = x - (tap % 3 - 1);
      if ((unsigned)pf < (unsigned)g.F && (unsigned)py < (unsigned)g.H && (unsigned)px < (unsigned)g.W) {
        const int p = ((bf + pf) * g.H + py) * g.W + px;
        s += *reinterpret_cast<const T*>(dcol + p * K + tap * C + c);
      }
    }
    T* d = reinterpret_cast<T*>(dx + (long long)q * lddx + c);
    *d = accumulate ? *d + s : s;
  }
}

// dir 0: w [O][C][27] -> wp [O][27][C]; dir 1: the inverse
__global__ __launch_bounds__(kThreads) void wperm_kernel(const float* __restrict__ src, float* __restrict__ dst, int O,
                                                         int C, int dir) {
  const int n = O * C * 27;
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
    const int o = i / (27 * C), r = i - o * 27 * C;
    const int c = r / 27, t = r - c * 27;  // i = OIDHW index
    const int j = (o * 27 + t) * C + c;    // tap-major index
    if (dir == 0) dst[j] = src[i];
    else dst[i] = src[j];
  }
}

// Fragment-order weights (gemm.hip's packed layout: record (t, g) = [64 lanes][4], lane (li, lq)
// holding output channel 16t + li, k = 16g + 4lq + e) of a Conv3d 3x3x3 weight W [cout][cin][27] for the
// inference conv kernels (conv3d_c16 / conv_lds), k = tap * in_pad + c:
//   dx = 0: the forward conv, out channel o, in channel c:  W[o][c][tap]
//   dx = 1: the input-gradient conv dX[q][c] = sum_{tap, o} dZ[q + off(tap)][o] W[o][c][26 - tap]
//           (the transposed conv is the forward conv of dZ with the taps flipped, channel roles swapped)
__global__ __launch_bounds__(kThreads) void pack_conv_kernel(const float* __restrict__ w, int cout, int cin, int dx,
                                                             int nout, int nin, int in_pad, int ntiles, int kgroups,
                                                             float* __restrict__ wp) {
  const int n_all = ntiles * kgroups * 256;
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < n_all; i += gridDim.x * kThreads) {
    const int t = i / (kgroups * 256), r = i - t * kgroups * 256;
    const int g = r >> 8, lane = (r >> 2) & 63, e = r & 3;
    const int n = 16 * t + (lane & 15), k = 16 * g + 4 * (lane >> 4) + e;
    const int tap = k / in_pad, ci = k - tap * in_pad;
    float v = 0.f;
    if (n < nout && ci < nin && tap < 27)
      v = dx ? w[((long long)ci * cin + n) * 27 + (26 - tap)] : w[((long long)n * cin + ci) * 27 + tap];
    wp[i] = v;
  }
}

__global__ __launch_bounds__(kThreads) void relu_kernel(float* __restrict__ y, int ld, int C, long long P) {
  const long long n = P * C;
  for (long long i = blockIdx.x * (long long)kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads) {
    const long long p = i / C;
    float* v = y + p * ld + (i - p * C);
    *v = fmaxf(*v, 0.f);
  }
}

// dz = dy * (y > 0): ReLU backward (y is the ReLU output; y > 0 <=> the pre-activation > 0)
__global__ __launch_bounds__(kThreads) void relu_mask_kernel(float* __restrict__ dy, int ldd, const float* __restrict__ y,
                                                             int ldy, int C, long long P) {
  const long long n = P * C;
  for (long long i = blockIdx.x * (long long)kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads) {
    const long long p = i / C;
    const int c = (int)(i - p * C);
    if (!(y[p * ldy + c] > 0.f)) dy[p * ldd + c] = 0.f;
  }
}

// MaxPool3d (1,2,2) backward (KDLAE_model.py:366): each pooled element's gradient goes to the first
// maximal input of its 2 x 2 window in (row, column) order — PyTorch's tie rule (ReLU zeros tie often) —
// or to the last NaN of the window (PyTorch's `val > max || isnan(val)`);
// din = dskip (the same tensor's gradient through the decoder's skip add, or 0) + that routed gradient.
__global__ __launch_bounds__(kThreads) void maxpool2_bwd_kernel(const float* __restrict__ in, int ldi,
                                                                const float* __restrict__ dout, int ldo,
                                                                const float* __restrict__ dskip, int lds,
                                                                float* __restrict__ din, int ldd, int C, Geo lo) {
  const long long n = (long long)lo.B * lo.F * lo.H * lo.W * C;
  const int Wi = 2 * lo.W, Hi = 2 * lo.H;
  for (long long i = blockIdx.x * (long long)kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads) {
    const long long pl = i / C;
    const int c = (int)(i - pl * C);
    int b, f, y, x;
    lo.coords(pl, b, f, y, x);
    const long long p0 = (((long long)b * lo.F + f) * Hi + 2 * y) * Wi + 2 * x;
    const long long ps[4] = {p0, p0 + 1, p0 + Wi, p0 + Wi + 1};
    int am = 0;
    float mx = in[ps[0] * ldi + c];
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      const float v = in[ps[j] * ldi + c];
      if (v > mx || v != v) {
        mx = v;
        am = j;
      }
    }
    const float g = dout[pl * ldo + c];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float base = dskip ? dskip[ps[j] * lds + c] : 0.f;
      din[ps[j] * ldd + c] = base + (j == am ? g : 0.f);
    }
  }
}

// ConvTranspose3d (1,2,2) stride (1,2,2) epilogue (KDLAE_model.py:378-379, :416-417):
// D[b, f, 2y + i, 2x + j, o] = U[b, f, y, x, 4 o + 2 i + j] + bias[o] + skip[b, f, 2y + i, 2x + j, o]
__global__ __launch_bounds__(kThreads) void upshuffle_add_kernel(const float* __restrict__ U, int ldu,
                                                                 const float* __restrict__ bias,
                                                                 const float* __restrict__ skip, int lds,
                                                                 float* __restrict__ D, int ldd, int C, Geo hi) {
  const long long n = (long long)hi.B * hi.F * hi.H * hi.W * C;
  const int Wl = hi.W / 2, Hl = hi.H / 2;
  for (long long i = blockIdx.x * (long long)kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads) {
    const long long p = i / C;
    const int o = (int)(i - p * C);
    int b, f, y, x;
    hi.coords(p, b, f, y, x);
    const long long pl = (((long long)b * hi.F + f) * Hl + (y >> 1)) * Wl + (x >> 1);
    float v = U[pl * ldu + 4 * o + 2 * (y & 1) + (x & 1)];
    if (bias) v += bias[o];
    v += skip[p * lds + o];
    D[p * ldd + o] = v;
  }
}

// L1LossForVideoFrames (Train/basicsr/models/losses/losses.py:409-526), pred / target [N][Cf][HW]:
// part[blk] = (sum |p - t|, sum |bin(p) - bin(t)|, sum |(p_f+1 - p_f) - (t_f+1 - t_f)|), and the
// gradient of  w_l1 (S_l1 + S_bin) / n1 + w_t S_t / n2  (torch.where's binarisation carries none;
// d|u| = sign(u), sign(0) = 0)
constexpr int kLossBlocks = 1024;
__global__ __launch_bounds__(kThreads) void l1frames_kernel(const float* __restrict__ pred, const float* __restrict__ tgt,
                                                            int N, int Cf, long long HW, float binary, float g1,
                                                            float gt, float* __restrict__ dpred,
                                                            float* __restrict__ part) {
  const long long n = (long long)N * Cf * HW;
  float s1 = 0.f, sb = 0.f, st = 0.f;
  for (long long i = blockIdx.x * (long long)kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads) {
    const long long s = i % HW;
    const long long nf = i / HW;
    const int f = (int)(nf % Cf);
    const float p = pred[i], t = tgt[i];
    const float d = p - t;
    s1 += fabsf(d);
    sb += fabsf((p > binary ? 1.f : 0.f) - (t > binary ? 1.f : 0.f));
    float g = g1 * (float)((d > 0.f) - (d < 0.f));
    if (f + 1 < Cf) {  // temporal term of the pair (f, f + 1)
      const float u = (pred[i + HW] - p) - (tgt[i + HW] - t);
      st += fabsf(u);
      g -= gt * (float)((u > 0.f) - (u < 0.f));
    }
    if (f > 0) {  // ... and of the pair (f - 1, f)
      const float u = (p - pred[i - HW]) - (t - tgt[i - HW]);
      g += gt * (float)((u > 0.f) - (u < 0.f));
    }
    (void)s;
    dpred[i] = g;
  }
  __shared__ float red[3][kThreads];
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = sb;
  red[2][threadIdx.x] = st;
  __syncthreads();
  for (int w = kThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int j = 0; j < 3; ++j) red[j][threadIdx.x] += red[j][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < 3) part[blockIdx.x * 3 + threadIdx.x] = red[threadIdx.x][0];
}

__global__ void l1frames_final_kernel(const float* __restrict__ part, int nblk, float w1, float wt, double inv1,
                                      double inv2, float* __restrict__ loss) {
  if (threadIdx.x) return;
  double a = 0, b = 0, c = 0;
  for (int i = 0; i < nblk; ++i) {
    a += part[3 * i];
    b += part[3 * i + 1];
    c += part[3 * i + 2];
  }
  loss[0] = (float)(w1 * ((a + b) * inv1) + (inv2 > 0 ? wt * (c * inv2) : 0.0));
}

}  // namespace

bool vec4_ok(const void* a, int ld, int C) { return C % 4 == 0 && ld % 4 == 0 && ((uintptr_t)a & 15) == 0; }

hipError_t launch_im2col3d(const float* x, int ldx, int C, int B, int F, int H, int W, float* col, hipStream_t s) {
  const long long P = (long long)B * F * H * W;
  if (P >= (1LL << 31)) return hipErrorInvalidValue;
  const Geo32 g{F, H, W};
  if (vec4_ok(x, ldx, C) && ((uintptr_t)col & 15) == 0) {
    const int KV = 27 * C / 4, ppb = KV <= kThreads ? kThreads / KV : 1;
    hipLaunchKernelGGL(im2col3d_kernel<4>, dim3(grid_for(P, ppb)), dim3(kThreads), 0, s, x, ldx, C, g, (int)P, col);
  } else {
    const int KV = 27 * C, ppb = KV <= kThreads ? kThreads / KV : 1;
    hipLaunchKernelGGL(im2col3d_kernel<1>, dim3(grid_for(P, ppb)), dim3(kThreads), 0, s, x, ldx, C, g, (int)P, col);
  }
  return hipGetLastError();
}

hipError_t launch_col2im3d(const float* dcol, int C, int B, int F, int H, int W, float* dx, int lddx, int accumulate,
                           hipStream_t s) {
  const long long P = (long long)B * F * H * W;
  if (P * C >= (1LL << 31)) return hipErrorInvalidValue;
  const Geo32 g{F, H, W};
  // float4 only: the training handle admits widths divisible by 4 only (kdlae_st.cpp), so a scalar
  // instance would be dead code (r06 kernel coverage: never launched)
  if (!vec4_ok(dx, lddx, C) || ((uintptr_t)dcol & 15) != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(col2im3d_kernel<4>, dim3(grid_for(P * C / 4)), dim3(kThreads), 0, s, dcol, C, g, (int)P, dx,
                     lddx, accumulate);
  return hipGetLastError();
}

hipError_t launch_wperm(const float* src, float* dst, int O, int C, int dir, hipStream_t s) {
  hipLaunchKernelGGL(wperm_kernel, dim3(grid_for((long long)O * C * 27)), dim3(kThreads), 0, s, src, dst, O, C, dir);
  return hipGetLastError();
}

hipError_t launch_pack_conv(const float* w, int cout, int cin, int dx, float* wp, hipStream_t s) {
  const int nout = dx ? cin : cout, nin = dx ? cout : cin;
  const int in_pad = (nin + 15) / 16 * 16, ntiles = (nout + 15) / 16, kgroups = 27 * in_pad / 16;
  hipLaunchKernelGGL(pack_conv_kernel, dim3(grid_for((long long)ntiles * kgroups * 256)), dim3(kThreads), 0, s, w,
                     cout, cin, dx, nout, nin, in_pad, ntiles, kgroups, wp);
  return hipGetLastError();
}

hipError_t launch_relu(float* y, int ld, int C, long long P, hipStream_t s) {
  hipLaunchKernelGGL(relu_kernel, dim3(grid_for(P * C)), dim3(kThreads), 0, s, y, ld, C, P);
  return hipGetLastError();
}

hipError_t launch_relu_mask(float* dy, int ldd, const float* y, int ldy, int C, long long P, hipStream_t s) {
  hipLaunchKernelGGL(relu_mask_kernel, dim3(grid_for(P * C)), dim3(kThreads), 0, s, dy, ldd, y, ldy, C, P);
  return hipGetLastError();
}

hipError_t launch_maxpool2_bwd(const float* in, int ldi, const float* dout, int ldo, const float* dskip, int lds,
                               float* din, int ldd, int C, int B, int F, int h, int w, hipStream_t s) {
  const long long n = (long long)B * F * h * w * C;
  hipLaunchKernelGGL(maxpool2_bwd_kernel, dim3(grid_for(n)), dim3(kThreads), 0, s, in, ldi, dout, ldo, dskip, lds,
                     din, ldd, C, Geo{B, F, h, w});
  return hipGetLastError();
}

hipError_t launch_upshuffle_add(const float* U, int ldu, const float* bias, const float* skip, int lds, float* D,
                                int ldd, int C, int B, int F, int H, int W, hipStream_t s) {
  const long long n = (long long)B * F * H * W * C;
  hipLaunchKernelGGL(upshuffle_add_kernel, dim3(grid_for(n)), dim3(kThreads), 0, s, U, ldu, bias, skip, lds, D, ldd,
                     C, Geo{B, F, H, W});
  return hipGetLastError();
}

int l1frames_scratch_floats() { return 3 * kLossBlocks; }

hipError_t launch_l1frames(const float* pred, const float* tgt, int N, int Cf, long long HW, float l1_weight,
                           float temporal_weight, float binary, int sum_reduction, float* dpred, float* loss,
                           float* scratch, hipStream_t s) {
  const long long n = (long long)N * Cf * HW;
  const long long n2 = (long long)N * (Cf - 1) * HW;
  const double inv1 = sum_reduction ? 1.0 : 1.0 / (double)n;
  const double inv2 = Cf > 1 ? (sum_reduction ? 1.0 : 1.0 / (double)n2) : 0.0;
  const float g1 = (float)(l1_weight * inv1), gt = (float)(temporal_weight * inv2);
  const unsigned blocks = (unsigned)std::min<long long>(kLossBlocks, (n + kThreads - 1) / kThreads);
  hipLaunchKernelGGL(l1frames_kernel, dim3(blocks), dim3(kThreads), 0, s, pred, tgt, N, Cf, HW, binary, g1, gt, dpred,
                     scratch);
  hipLaunchKernelGGL(l1frames_final_kernel, dim3(1), dim3(64), 0, s, scratch, (int)blocks, l1_weight,
                     temporal_weight, inv1, inv2, loss);
  return hipGetLastError();
}

}  // namespace train
}  // namespace kdlae
