// 3x3 convolutions whose input or output has <= 4 channels: small-in as a K <= 36 MFMA GEMM,
// small-out on the VALU.
//
//   small-in  (Cin <= 4,  Cout % 16 == 0): patch_embed 3->48 (KDLAE_model.py:173),
//             output_param 4->96 dilation 2 on cat[out, denoise_rate] (:259, :316), cen 3->96 (:265)
//   small-out (Cout <= 4, Cin % 4 == 0):  output 96->3 (:258, :314), output2 96->3 + inp_img (:261,
//             :319-321), outputen 48->3 (:268, :329)
// Zero padding = dilation.  Input of small-in is any strided 4-D tensor (NCHW or NHWC view);
// output of small-out is NCHW (optionally + NCHW residual) or an NHWC view that also receives an
// extra NCHW channel — the torch.cat([out, denoise_rate]) of :316 folded into the producer.
#include "kernels.h"

namespace kdlae {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// MFMA form (r02): out[p][n] = bias[n] + sum_k W[n][k] im2col[p][k], k = ci * taps + tap (K <= 36,
// zero past Cin * taps), as v_mfma_f32_16x16x4_f32 with W as the A operand and 16 pixels as B.  Each
// lane's k index is fixed per k-step (k = 4 s + lane / 16), so its tap offsets and weight fragments
// are computed once: the W fragments of every output tile (NTO x 9 VGPRs) stay in registers and a
// k-step costs the lane one gathered load per 16 pixels.  The accumulator of output tile t holds
// channels 16 t + 4 (lane / 16) .. + 3 of pixel lane % 16 -> one 16 B NHWC store.  A wave walks
// 64-pixel chunks (4 independent 16-pixel sub-tiles in flight).  r01's VALU kernel read all 16 x 36
// weights of a thread's output group from LDS per pixel: 1.2 ms per 4M-pixel launch, ~5x its HBM floor.
template <int KT, int NTO>
__global__ __launch_bounds__(256) void conv_small_in_kernel(SmallInParams p) {
  constexpr int taps = 9 * KT;
  constexpr int KS = 9;  // k-steps of 4 (K <= 36)
  const int lane = threadIdx.x & 63, li = lane & 15, lq = lane >> 4;
  const int vh = p.vh ? p.vh : p.H, vw = p.vw ? p.vw : p.W;
  const int K = p.Cin * taps;
  // this lane's k per step: channel, tap offsets (frame, row, column) and the offset from the pixel
  int kdt[KS], kdy[KS], kdx[KS];
  long long koff[KS];
  bool kok[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 4 * s + lq;
    kok[s] = k < K;
    const int kk = kok[s] ? k : 0;
    const int ci = kk / taps, tap = kk - (kk / taps) * taps;
    const int t9 = tap % 9;
    kdt[s] = KT == 3 ? tap / 9 - 1 : 0;
    kdy[s] = (t9 / 3 - 1) * p.dil;
    kdx[s] = (t9 % 3 - 1) * p.dil;
    koff[s] = ci * p.sc + kdt[s] * p.st + kdy[s] * p.sy + kdx[s] * p.sx;
  }
  // W fragments: A[i = out channel li of tile t][k = 4 s + lq]
  float wf[NTO][KS];
  f32x4 bq[NTO];
#pragma unroll
  for (int t = 0; t < NTO; ++t) {
    const int co = 16 * t + li;
    const bool cok = co < p.Cout;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = 4 * s + lq;
      // wt: transposed conv's weight [Cin][wt][3][3], flipped taps (kt 1: k = ci * 9 + tap)
      const int wi = p.wt ? ((k / 9) * p.wt + co) * 9 + 8 - k % 9 : co * K + k;
      wf[t][s] = (cok && kok[s]) ? p.w[wi] : 0.f;
    }
    const int cb = 16 * t + 4 * lq;
    bq[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (p.bias && cb < p.Cout) bq[t] = f32x4{p.bias[cb], p.bias[cb + 1], p.bias[cb + 2], p.bias[cb + 3]};
  }
  const int fhw = p.H * p.W;
  const int HW = p.F * fhw;
  const long long P = (long long)p.Bn * HW;
  const long long nchunks = (P + 63) / 64;
  const long long wave_id = blockIdx.x * 4LL + (threadIdx.x >> 6);
  const long long nwaves = gridDim.x * 4LL;
  for (long long c = wave_id; c < nchunks; c += nwaves) {
    float bv[4][KS];
    long long pix[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pix[j] = c * 64 + 16 * j + li;
      const long long pc = pix[j] < P ? pix[j] : P - 1;
      const int b = (int)(pc / HW);
      const int pl = (int)(pc - (long long)b * HW);
      const int t0 = pl / fhw;
      const int rem = pl - t0 * fhw;
      const int y = rem / p.W, x = rem - (rem / p.W) * p.W;
      const long long base = b * p.sb + t0 * p.st + y * p.sy + x * p.sx;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int tt = t0 + kdt[s], yy = y + kdy[s], xx = x + kdx[s];
        const bool ok = kok[s] && (unsigned)tt < (unsigned)p.F && (unsigned)yy < (unsigned)vh &&
                        (unsigned)xx < (unsigned)vw;
        const long long off = ok ? base + koff[s] : 0;
        float v = p.in[off];
        if (p.in_sub) v -= p.in_sub[off];
        bv[j][s] = ok ? v : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 acc[NTO];
#pragma unroll
      for (int t = 0; t < NTO; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int t = 0; t < NTO; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[t][s], bv[j][s], acc[t], 0, 0, 0);
      if (pix[j] >= P) continue;
      float* o = p.out + pix[j] * p.ldo + 4 * lq;
#pragma unroll
      for (int t = 0; t < NTO; ++t) {
        if (16 * t >= p.Cout) continue;
        f32x4 r = acc[t] + bq[t];
        if (p.relu) r = f32x4{fmaxf(r.x, 0.f), fmaxf(r.y, 0.f), fmaxf(r.z, 0.f), fmaxf(r.w, 0.f)};
        *reinterpret_cast<f32x4*>(o + 16 * t) = r;
      }
    }
  }
}

template <int KT>
static void launch_small_in_nt(const SmallInParams& p, unsigned blocks, hipStream_t s) {
  const int nto = p.Cout / 16;
  if (nto <= 2) hipLaunchKernelGGL((conv_small_in_kernel<KT, 2>), dim3(blocks), dim3(256), 0, s, p);
  else if (nto <= 3) hipLaunchKernelGGL((conv_small_in_kernel<KT, 3>), dim3(blocks), dim3(256), 0, s, p);
  else if (nto <= 4) hipLaunchKernelGGL((conv_small_in_kernel<KT, 4>), dim3(blocks), dim3(256), 0, s, p);
  else if (nto <= 6) hipLaunchKernelGGL((conv_small_in_kernel<KT, 6>), dim3(blocks), dim3(256), 0, s, p);
  else hipLaunchKernelGGL((conv_small_in_kernel<KT, 8>), dim3(blocks), dim3(256), 0, s, p);
}

hipError_t launch_conv_small_in(const SmallInParams& p, hipStream_t s) {
  if (p.Cin * 9 * p.kt > 36 || p.Cout % 16 || (p.kt != 1 && p.kt != 3) || (p.wt && (p.kt != 1 || p.wt < p.Cout)))
    return hipErrorInvalidValue;
  const long long chunks = ((long long)p.Bn * p.F * p.H * p.W + 63) / 64;
  long long blocks = (chunks + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  const int K = p.Cin * 9 * p.kt;
  for (int co0 = 0; co0 < p.Cout; co0 += 128) {  // up to 8 output tiles per pass
    SmallInParams q = p;
    q.w = p.w + (p.wt ? (size_t)co0 * 9 : (size_t)co0 * K);
    q.bias = p.bias ? p.bias + co0 : nullptr;
    q.out = p.out + co0;
    q.Cout = p.Cout - co0 < 128 ? p.Cout - co0 : 128;
    if (p.kt == 3) launch_small_in_nt<3>(q, (unsigned)blocks, s);
    else launch_small_in_nt<1>(q, (unsigned)blocks, s);
  }
  return hipGetLastError();
}

// 4 lanes per pixel, each owning a quarter of the input channels (coalesced 16 B per lane along
// channels); weights transposed in LDS to [tap][ci][4 outputs]; partial sums combined with two
// butterfly shuffles.  A wave covers 16 pixels.
__global__ __launch_bounds__(256) void conv_small_out_kernel(SmallOutParams p) {
  extern __shared__ __attribute__((aligned(16))) float wso[];  // [taps][Cin][4]
  const int taps = p.ks * p.ks;
  const int nw = taps * p.Cin * 4;
  for (int i = threadIdx.x; i < nw; i += 256) {
    const int o = i & 3, ci = (i >> 2) % p.Cin, t = (i >> 2) / p.Cin;
    wso[i] = o < p.Cout ? p.w[p.wt ? (ci * p.Cout + o) * taps + taps - 1 - t : (o * p.Cin + ci) * taps + t] : 0.f;
  }
  __syncthreads();
  const int fhw = p.H * p.W;
  const int HW = p.F * fhw;
  const long long P = (long long)p.Bn * HW;
  const int cs = threadIdx.x & 3;
  const int cq = p.Cin >> 2;  // channels per lane (multiple of 4)
  for (long long pix = (blockIdx.x * 256LL + threadIdx.x) >> 2; pix < P + 0; pix += (long long)gridDim.x * 64) {
    const bool pv = pix < P;
    const long long pc = pv ? pix : 0;
    const int b = (int)(pc / HW);
    const int pl = (int)(pc - (long long)b * HW);
    const int tf = pl / fhw;
    const int rem = pl - tf * fhw;
    const int y = rem / p.W, x = rem - (rem / p.W) * p.W;
    const float* Xb = p.in + ((long long)b * HW + (long long)tf * fhw) * p.ld + cs * cq;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < taps; ++t) {
      const int yy = p.ks == 3 ? y + t / 3 - 1 : y, xx = p.ks == 3 ? x + t % 3 - 1 : x;
      const bool ok = (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W;
      const float* xr = Xb + (ok ? (yy * p.W + xx) * p.ld : 0);
      const f32x4* wt = reinterpret_cast<const f32x4*>(wso + (t * p.Cin + cs * cq) * 4);
      f32x4 part = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int c = 0; c < cq; c += 4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(xr + c);
        part += v.x * wt[c] + v.y * wt[c + 1] + v.z * wt[c + 2] + v.w * wt[c + 3];
      }
      acc += ok ? part : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[e] += __shfl_xor(acc[e], 1);
      acc[e] += __shfl_xor(acc[e], 2);
    }
    if (!pv || cs != 0) continue;
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      if (o >= p.Cout) break;
      float v = acc[o] + (p.bias ? p.bias[o] : 0.f);
      if (p.out_nchw) {
        const long long oi = ((long long)b * p.Cout + o) * HW + pl;
        if (p.res) v += p.res[oi];
        p.out[oi] = v;
      } else {
        if (p.res_nhwc) v += p.res_nhwc[pix * p.ldr + o];
        p.out[pix * p.ldo + o] = v;
      }
    }
    if (!p.out_nchw && p.extra) p.out[pix * p.ldo + p.Cout] = p.extra[(long long)b * HW + pl];
  }
}

// 3x3 / Cout <= 4 / single-frame head conv, LDS-tiled: a 256-thread block owns a 16 x 32 output tile,
// thread = (column, pair of rows).  The 18 x 34 input halo is staged 16 channels at a time in
// quad-planar LDS ([4 quads][612 px], conflict-free column reads), the next chunk's global loads are
// in flight in registers meanwhile; weights sit in LDS as float4 (4 outputs) per (tap, channel).
// Each input element is read from HBM ~1.1x instead of 9x through L2.
constexpr int kSoTW = 16, kSoTH = 32, kSoHW = kSoTW + 2, kSoHH = kSoTH + 2, kSoPx = kSoHW * kSoHH;  // 612
constexpr int kSoItems = kSoPx * 4;                                   // float4 per 16-channel chunk
constexpr int kSoPer = (kSoItems + 255) / 256;                         // 10 per thread

__global__ __launch_bounds__(256) void conv_small_out_tiled_kernel(SmallOutParams p) {
  __shared__ f32x4 st[4][kSoPx];
  extern __shared__ __attribute__((aligned(16))) f32x4 wq[];           // [9][Cin] (4 outputs each)
  const int tid = threadIdx.x;
  for (int i = tid; i < 9 * p.Cin; i += 256) {
    const int t = i / p.Cin, ci = i - t * p.Cin;
    f32x4 w4;
#pragma unroll
    for (int o = 0; o < 4; ++o) w4[o] = o < p.Cout ? p.w[p.wt ? (ci * p.Cout + o) * 9 + 8 - t : (o * p.Cin + ci) * 9 + t] : 0.f;
    wq[i] = w4;
  }
  const int tx_n = (p.W + kSoTW - 1) / kSoTW, ty_n = (p.H + kSoTH - 1) / kSoTH;
  int bid = blockIdx.x;
  const int tx = bid % tx_n;
  bid /= tx_n;
  const int ty = bid % ty_n;
  const int b = bid / ty_n;
  const int x0 = tx * kSoTW, y0 = ty * kSoTH;
  const long long HW = (long long)p.H * p.W;
  const float* X = p.in + (long long)b * HW * p.ld;
  const int cx = tid & 15, r0 = 2 * (tid >> 4);                       // rows r0, r0 + 1 of the tile
  f32x4 pf[kSoPer];
  auto fetch = [&](int c0) {
#pragma unroll
    for (int j = 0; j < kSoPer; ++j) {
      const int it = tid + 256 * j;
      const int px = it >> 2, q = it & 3;
      const int hy = px / kSoHW, hx = px - hy * kSoHW;
      const int yy = y0 - 1 + hy, xx = x0 - 1 + hx;
      const bool ok = it < kSoItems && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W;
      const f32x4 v = *reinterpret_cast<const f32x4*>(X + (ok ? ((long long)yy * p.W + xx) * p.ld + c0 + 4 * q : 0));
      pf[j] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto put = [&]() {
#pragma unroll
    for (int j = 0; j < kSoPer; ++j) {
      const int it = tid + 256 * j;
      if (it < kSoItems) st[it & 3][it >> 2] = pf[j];
    }
  };
  f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
  fetch(0);
  for (int c0 = 0; c0 < p.Cin; c0 += 16) {
    __syncthreads();                                                   // previous chunk consumed
    put();
    __syncthreads();
    if (c0 + 16 < p.Cin) fetch(c0 + 16);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        f32x4 v[4];                                                    // halo rows r0 .. r0 + 3
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) v[rr] = st[q][(r0 + rr) * kSoHW + cx + kx];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const f32x4* w = wq + (ky * 3 + kx) * p.Cin + c0 + 4 * q;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const f32x4 w4 = w[e];
            a0 += v[ky][e] * w4;
            a1 += v[ky + 1][e] * w4;
          }
        }
      }
    }
  }
  const int xo = x0 + cx;
  if (xo >= p.W) return;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int yo = y0 + r0 + k;
    if (yo >= p.H) continue;
    const f32x4 acc = k ? a1 : a0;
    const long long pl = (long long)yo * p.W + xo, pix = (long long)b * HW + pl;
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      if (o >= p.Cout) break;
      float v = acc[o] + (p.bias ? p.bias[o] : 0.f);
      if (p.out_nchw) {
        const long long oi = ((long long)b * p.Cout + o) * HW + pl;
        if (p.res) v += p.res[oi];
        p.out[oi] = v;
      } else {
        if (p.res_nhwc) v += p.res_nhwc[pix * p.ldr + o];
        p.out[pix * p.ldo + o] = v;
      }
    }
    if (!p.out_nchw && p.extra) p.out[pix * p.ldo + p.Cout] = p.extra[pix];
  }
}

hipError_t launch_conv_small_out(const SmallOutParams& p, hipStream_t s) {
  if (p.Cin % 16 || (p.ks != 1 && p.ks != 3) || (p.wt && p.ks != 3)) return hipErrorInvalidValue;
  if (p.ks == 3 && p.F == 1 && p.ld % 4 == 0 && p.Cin <= 256) {
    const long long blocks = (long long)p.Bn * ((p.H + kSoTH - 1) / kSoTH) * ((p.W + kSoTW - 1) / kSoTW);
    const size_t lds = (size_t)9 * p.Cin * sizeof(f32x4);
    hipLaunchKernelGGL(conv_small_out_tiled_kernel, dim3((unsigned)blocks), dim3(256), lds, s, p);
    return hipGetLastError();
  }
  const long long P = (long long)p.Bn * p.F * p.H * p.W;
  long long blocks = (P + 63) / 64;
  if (blocks > 16384) blocks = 16384;
  const size_t lds = (size_t)p.ks * p.ks * p.Cin * 4 * sizeof(float);
  hipLaunchKernelGGL(conv_small_out_kernel, dim3((unsigned)blocks), dim3(256), lds, s, p);
  return hipGetLastError();
}

// MaxPool (1,2,2) (KDLAE_model.py:366) / MaxPool2d(2) (ASDQE_model.py:41), NHWC float4 per thread.
__global__ __launch_bounds__(256) void maxpool2_kernel(const float* __restrict__ in, int ldi, float* __restrict__ out,
                                                       int ldo, int C, long long nframes, int H, int W) {
  const int Ho = H >> 1, Wo = W >> 1, c4n = C >> 2;
  const long long total = nframes * Ho * Wo * c4n;
  for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    const int c = (int)(idx % c4n) * 4;
    long long r = idx / c4n;
    const int xo = (int)(r % Wo);
    r /= Wo;
    const int yo = (int)(r % Ho);
    const long long f = r / Ho;
    const float* base = in + ((f * H + 2 * yo) * W + 2 * xo) * (long long)ldi + c;
    const f32x4 a = *reinterpret_cast<const f32x4*>(base);
    const f32x4 b = *reinterpret_cast<const f32x4*>(base + ldi);
    const f32x4 d = *reinterpret_cast<const f32x4*>(base + (long long)W * ldi);
    const f32x4 e = *reinterpret_cast<const f32x4*>(base + (long long)W * ldi + ldi);
    f32x4 m;
    m.x = fmaxf(fmaxf(a.x, b.x), fmaxf(d.x, e.x));
    m.y = fmaxf(fmaxf(a.y, b.y), fmaxf(d.y, e.y));
    m.z = fmaxf(fmaxf(a.z, b.z), fmaxf(d.z, e.z));
    m.w = fmaxf(fmaxf(a.w, b.w), fmaxf(d.w, e.w));
    *reinterpret_cast<f32x4*>(out + ((f * Ho + yo) * Wo + xo) * (long long)ldo + c) = m;
  }
}

hipError_t launch_maxpool2(const float* in, int ldi, float* out, int ldo, int C, long long nframes, int H, int W,
                           hipStream_t s) {
  if (C % 4) return hipErrorInvalidValue;
  const long long total = nframes * (H / 2) * (W / 2) * (C / 4);
  long long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(maxpool2_kernel, dim3((unsigned)blocks), dim3(256), 0, s, in, ldi, out, ldo, C, nframes, H, W);
  return hipGetLastError();
}

}  // namespace kdlae
