// Fully fused FeedForward (GDFN) of a TransformerBlock (KDLAE/KDLAE_model.py:89-106, :161):
//   y = x + project_out( gelu_erf(dw3x3(h1)) * dw3x3(h2) ),   [h1 | h2] = project_in( LN(x) )
// in ONE pass: x is read once (plus its 1-pixel halo) and y written once; the 2*hid-channel
// project_in output and the gated hid-channel tensor never reach HBM.  r01 ran this as a
// project_in GEMM writing 2*hidS floats per pixel (1 KiB at C = 48, 2 KiB at C = 96) and the
// gdfn_out kernel reading them back; at C = 48 / 1024^2 both halves were HBM-bound.
//
// Tile: 16 wide x 8 tall output pixels per workgroup (8 waves; wave w owns tile row w).
// project_in must be evaluated on the 18 x 10 halo (the depthwise conv zero-pads ITS output), so
// the halo's 180 pixels are 12 groups of 16: waves 0-3 own groups w and w + 8, waves 4-7 group w,
// which gives every SIMD (waves w and w + 4) the same 3 groups.  A wave keeps its groups' LN'd x
// rows in VGPRs for the whole tile as MFMA B operands (lane (li, lq): pixel li of the group,
// channels 16 kg + 4 lq .. +3) — exactly the r01 GEMM's A-row layout.  (A 16 x 16 tile has the
// same MFMA work per pixel — its 21 halo groups leave one SIMD 3 groups heavier — but needs ~60
// more VGPRs per lane than the 256 two waves per SIMD allow.)
//
// Per hidden chunk c (16 channels of h1 and the same 16 of h2; hidS / 16 chunks):
//   project_in(c)   MFMA 16x16x4 f32, A = packed W_in records (the project_in GEMM's own packing,
//                   LN weight folded in), B = x rows -> D^T = 4 channels of one halo pixel per lane;
//                   + folded bias, zero for halo pixels outside the image, written to a halo image
//                   in LDS laid out [pixel][quad ^ (pixel & 7)] (the gdfn.hip stencil layout);
//   gate(c)         the gdfn.hip depthwise 3x3 + exact-erf gate (A&S 7.1.26), 2 tile rows x 4
//                   channels per lane, producing the project_out B operand in registers;
//   project_out(c)  MFMA with the packed W_out records, accumulated over all chunks.
// Software pipeline with ONE barrier per chunk: iteration c runs project_in(c) into hidden buffer
// c & 1 and then gate(c - 1) + project_out(c - 1) from buffer (c - 1) & 1, so the gate VALU and
// both MFMA phases sit in one basic block.  Weights for chunk c + 1 (W_in, W_out, dw: 3 CT + 2
// DMA pieces of 1 KiB) arrive by LDS-DMA into a 3-slot ring while chunk c is computed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "kernels.h"

namespace kdlae {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int kTW = 16, kTH = 8;    // output tile (columns x rows); wave w computes row w
constexpr int kH = kTW + 2;         // halo row length (18)
constexpr int kHP = kH * (kTH + 2); // 180 halo pixels
constexpr int kNG = (kHP + 15) / 16;  // 12 pixel groups
constexpr int kWaves = 8;
constexpr int kGPW = (kNG + kWaves - 1) / kWaves;  // 2 groups per wave at most
constexpr int kHidF4 = kHP * 8;     // one hidden halo image: [pixel][8 quads] float4
constexpr int kDwF4 = 128;          // per-chunk dw block (gdfn.hip layout): [9][8] weights, [8] bias, pad

template <int CT>
struct Lay {
  static constexpr int win = 2 * CT * 64;            // W_in records of the chunk: h1 tile, h2 tile
  static constexpr int wout = CT * 64;               // W_out records (one per output tile)
  static constexpr int slot = win + wout + kDwF4;
  static constexpr int pieces = 3 * CT + 2;          // 1 KiB DMA wave-instructions per chunk
  static constexpr int ring = 2 * kHidF4;            // after the two hidden buffers
  static constexpr int bin = ring + 3 * slot;        // folded project_in bias, [chunk][8] float4
  static constexpr int per_wave(int w) { return (pieces - w + kWaves - 1) / kWaves; }
};

__device__ __forceinline__ float gelu_erf(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float poly = fmaf(1.061405429f, t, -1.453152027f);
  poly = fmaf(poly, t, 1.421413741f);
  poly = fmaf(poly, t, -0.284496736f);
  poly = fmaf(poly, t, 0.254829592f);
  poly *= t;
  const float e = 1.0f - poly * __expf(-z * z);  // erf(|x| / sqrt 2), |error| <= 1.5e-7
  return 0.5f * x * (1.0f + copysignf(e, x));
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
__device__ __forceinline__ void dma16(const void* src, f32x4* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ f32x4 buf_load4(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
__device__ __forceinline__ void buf_store4(__amdgpu_buffer_rsrc_t r, unsigned off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)off, 0, 0);
}
constexpr unsigned kOOB = 0x80000000u;

// every wave: all its VMEM (the DMAs of the next chunk were issued one iteration ago) and LDS ops
// done, then the workgroup barrier
__device__ __forceinline__ void sync_all() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

}  // namespace

// BPC = workgroups per CU the register budget is declared for: 1 at C = 96 (<= 256 VGPRs),
// 2 at C = 48 (<= 128 VGPRs; two 79 KiB workgroups share the 160 KiB of LDS)
template <int CT, int BPC>
__global__ __launch_bounds__(64 * kWaves, 2 * BPC) void ffn_fused_kernel(FfnParams p) {
  using LY = Lay<CT>;
  extern __shared__ __attribute__((aligned(16))) f32x4 lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lq = lane >> 4;   // project_in / LN lane roles
  const int cx = li, q = lq;                  // gate / project_out lane roles (column, channel quad)
  const int kch = p.hidS >> 4;

  // XCD-aware tile order (gdfn.hip): logical tiles [k*per, (k+1)*per) run on XCD k
  const int tx_n = (p.W + kTW - 1) / kTW, ty_n = (p.H + kTH - 1) / kTH;
  const int ntiles = p.Bn * tx_n * ty_n;
  const int per = (int)(gridDim.x >> 3);
  int bid = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (bid >= ntiles) return;
  const int tx = bid % tx_n;
  bid /= tx_n;
  const int ty = bid % ty_n;
  const int b = bid / ty_n;
  const int x0 = tx * kTW, y0 = ty * kTH;
  const long long HW = (long long)p.H * p.W;

  // ---- weights of chunk c -> ring slot c % 3 (LDS-DMA, no VGPRs); piece k is issued by wave k % 8
  const f32x4* Win = reinterpret_cast<const f32x4*>(p.Win);
  const f32x4* Wout = reinterpret_cast<const f32x4*>(p.Wout);
  const f32x4* Dw = reinterpret_cast<const f32x4*>(p.dw);
  auto issue = [&](int c) {
    f32x4* sl = lds + LY::ring + (c % 3) * LY::slot;
#pragma unroll
    for (int j = 0; j < (LY::pieces + kWaves - 1) / kWaves; ++j) {
      const int k = wave + kWaves * j;
      if (k >= LY::pieces) break;
      const f32x4* src;
      if (k < 2 * CT) src = Win + ((size_t)(2 * c) * CT + k) * 64;               // tiles 2c, 2c+1 contiguous
      else if (k < 3 * CT) src = Wout + ((size_t)(k - 2 * CT) * kch + c) * 64;   // output tile k - 2 CT
      else src = Dw + (size_t)c * kDwF4 + (k - 3 * CT) * 64;
      dma16(src + lane, sl + 64 * k);
    }
  };
  issue(0);

  // ---- folded project_in bias -> LDS [chunk][8 quads] (zeros when the layer has no bias)
  for (int i = tid; i < 2 * kch * 4; i += 64 * kWaves)
    lds[LY::bin + i] = p.bin ? *reinterpret_cast<const f32x4*>(p.bin + 4 * i) : f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- x rows of this wave's halo groups (LN'd in registers)
  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.x + (long long)b * HW * p.ldx), 0,
                                        (int)(HW * p.ldx * 4), 0x00020000);
  f32x4 xf[kGPW][CT];
  bool hv[kGPW];                      // halo pixel inside the image (hidden value kept), per lane
  int hpx[kGPW];                      // halo pixel index of this lane in group gi
#pragma unroll
  for (int gi = 0; gi < kGPW; ++gi) {
    const int hp = (wave + kWaves * gi) * 16 + li;
    const int hy = hp / kH, hx = hp - (hp / kH) * kH;
    const int yy = y0 - 1 + hy, xx = x0 - 1 + hx;
    hpx[gi] = hp;
    hv[gi] = hp < kHP && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W;
    const unsigned base = hv[gi] ? (unsigned)((yy * p.W + xx) * p.ldx + 4 * lq) * 4u : kOOB;
#pragma unroll
    for (int kg = 0; kg < CT; ++kg) xf[gi][kg] = buf_load4(rx, base + 64u * kg);
  }
  // LayerNorm over the C channels of each pixel (the four lq lanes of a pixel hold C/4 each):
  // BiasFree x / sqrt(var + 1e-5) (:50-52), WithBias (x - mu) / sqrt(var + 1e-5) (:67-70); the
  // LN weight is folded into W_in, the WithBias shift into the folded bias
  const float inv_c = 1.0f / (float)(16 * CT);
#pragma unroll
  for (int gi = 0; gi < kGPW; ++gi) {
    float s = 0.f;
#pragma unroll
    for (int kg = 0; kg < CT; ++kg) s += (xf[gi][kg].x + xf[gi][kg].y) + (xf[gi][kg].z + xf[gi][kg].w);
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    const float mean = s * inv_c;
    float v2 = 0.f;
#pragma unroll
    for (int kg = 0; kg < CT; ++kg) {
      const f32x4 d = xf[gi][kg] - mean;
      v2 += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
    }
    v2 += __shfl_xor(v2, 16);
    v2 += __shfl_xor(v2, 32);
    const float rstd = 1.0f / sqrtf(v2 * inv_c + 1e-5f);
    const float sh = p.ln == 2 ? mean : 0.f;
#pragma unroll
    for (int kg = 0; kg < CT; ++kg) xf[gi][kg] = (xf[gi][kg] - sh) * rstd;
  }

  f32x4 acc[CT];                      // project_out accumulators: tile row w, output tiles t
#pragma unroll
  for (int t = 0; t < CT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c = 0; c <= kch; ++c) {
    sync_all();                       // chunk c's weights landed; hidden buffer c & 1 free
    if (c + 1 < kch) issue(c + 1);
    if (c < kch) {
      // ---- project_in(c) on this wave's halo groups
      const f32x4* wl = lds + LY::ring + (c % 3) * LY::slot;
      f32x4 ah[kGPW][2];
#pragma unroll
      for (int gi = 0; gi < kGPW; ++gi) ah[gi][0] = ah[gi][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kg = 0; kg < CT; ++kg) {
        const f32x4 w0 = wl[kg * 64 + lane], w1 = wl[(CT + kg) * 64 + lane];
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int gi = 0; gi < kGPW; ++gi) {
            if (wave + kWaves * gi >= kNG) continue;   // wave-uniform: the 21st..24th groups do not exist
            ah[gi][0] = mfma4(w0[s], xf[gi][kg][s], ah[gi][0]);
            ah[gi][1] = mfma4(w1[s], xf[gi][kg][s], ah[gi][1]);
          }
      }
      f32x4* hid = lds + (c & 1) * kHidF4;
      const f32x4 b1 = lds[LY::bin + c * 8 + lq], b2 = lds[LY::bin + c * 8 + 4 + lq];
#pragma unroll
      for (int gi = 0; gi < kGPW; ++gi) {
        if (wave + kWaves * gi >= kNG) continue;
        const int hp = hpx[gi];
        if (hp >= kHP) continue;
        const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
        hid[hp * 8 + (lq ^ (hp & 7))] = hv[gi] ? ah[gi][0] + b1 : z;
        hid[hp * 8 + ((4 + lq) ^ (hp & 7))] = hv[gi] ? ah[gi][1] + b2 : z;
      }
    }
    if (c > 0) {
      // ---- gate(c - 1): depthwise 3x3 + gate for tile row w, column cx, channel quad q
      const int g = c - 1;
      const f32x4* sl = lds + ((g & 1) * kHidF4);
      const f32x4* dw = lds + LY::ring + (g % 3) * LY::slot + LY::win + LY::wout;
      f32x4 d[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) d[h] = dw[72 + 4 * h + q];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            const int px = (wave + i) * kH + cx + j;
            d[h] = sl[px * 8 + ((4 * h + q) ^ (px & 7))] * dw[(3 * i + j) * 8 + 4 * h + q] + d[h];
          }
      f32x4 gb;
      gb.x = gelu_erf(d[0].x) * d[1].x;
      gb.y = gelu_erf(d[0].y) * d[1].y;
      gb.z = gelu_erf(d[0].z) * d[1].z;
      gb.w = gelu_erf(d[0].w) * d[1].w;
      // ---- project_out(c - 1)
      const f32x4* wo = lds + LY::ring + (g % 3) * LY::slot + LY::win;
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        const f32x4 w = wo[t * 64 + lane];
        acc[t] = mfma4(w.x, gb.x, acc[t]);
        acc[t] = mfma4(w.y, gb.y, acc[t]);
        acc[t] = mfma4(w.z, gb.z, acc[t]);
        acc[t] = mfma4(w.w, gb.w, acc[t]);
      }
    }
  }

  // ---- epilogue: y = x + project_out + bias for the tile's own pixels (x itself is not written)
  const int xo = x0 + cx, yo = y0 + wave;
  const __amdgpu_buffer_rsrc_t ry =
      __builtin_amdgcn_make_buffer_rsrc(p.y + (long long)b * HW * p.ldy, 0, (int)(HW * p.ldy * 4), 0x00020000);
  const bool ok = xo < p.W && yo < p.H;
  const unsigned bx = ok ? (unsigned)((yo * p.W + xo) * p.ldx + 4 * q) * 4u : kOOB;
  const unsigned by = ok ? (unsigned)((yo * p.W + xo) * p.ldy + 4 * q) * 4u : kOOB;
  f32x4 res[CT];
#pragma unroll
  for (int t = 0; t < CT; ++t) res[t] = buf_load4(rx, bx == kOOB ? kOOB : bx + 64u * t);
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    const f32x4 bo = p.bout ? *reinterpret_cast<const f32x4*>(p.bout + 16 * t + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
    buf_store4(ry, by == kOOB ? kOOB : by + 64u * t, acc[t] + res[t] + bo);
  }
}

bool ffn_fused_supported(int C, int hidS) { return (C == 48 || C == 96) && hidS % 16 == 0 && hidS <= 256; }

static size_t ffn_lds_bytes(int CT, int hidS) {
  const size_t slot = (size_t)3 * CT * 64 + kDwF4;
  return (2 * (size_t)kHidF4 + 3 * slot + (size_t)(hidS / 16) * 8) * sizeof(f32x4);
}

hipError_t launch_ffn_fused(const FfnParams& p, hipStream_t s) {
  if (!ffn_fused_supported(p.C, p.hidS) || p.ldx % 4 || p.ldy % 4 || p.x == p.y) return hipErrorInvalidValue;
  if ((long long)p.H * p.W * p.ldx * 4 >= (1LL << 31) || (long long)p.H * p.W * p.ldy * 4 >= (1LL << 31))
    return hipErrorInvalidValue;
  const long long tiles = (long long)p.Bn * ((p.H + kTH - 1) / kTH) * ((p.W + kTW - 1) / kTW);
  const long long grid = (tiles + 7) / 8 * 8;
  const int CT = p.C / 16;
  const size_t lds = ffn_lds_bytes(CT, p.hidS);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  static size_t attr[64][2] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  const void* f = CT == 3 ? reinterpret_cast<const void*>(&ffn_fused_kernel<3, 1>)
                          : reinterpret_cast<const void*>(&ffn_fused_kernel<6, 1>);
  if (lds > attr[dev][CT == 6]) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr[dev][CT == 6] = lds;
  }
  if (CT == 3) hipLaunchKernelGGL((ffn_fused_kernel<3, 1>), dim3((unsigned)grid), dim3(64 * kWaves), lds, s, p);
  else hipLaunchKernelGGL((ffn_fused_kernel<6, 1>), dim3((unsigned)grid), dim3(64 * kWaves), lds, s, p);
  return hipGetLastError();
}

// strided copy of C floats per pixel (a stage whose fused FFNs ended in the alternate buffer)
__global__ __launch_bounds__(256) void copy_view_kernel(const float* __restrict__ src, int lds_, float* __restrict__ dst,
                                                        int ldd, int C4, long long P) {
  const long long n = P * C4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long px = i / C4;
    const int c = (int)(i - px * C4);
    *reinterpret_cast<f32x4*>(dst + px * ldd + 4 * c) = *reinterpret_cast<const f32x4*>(src + px * lds_ + 4 * c);
  }
}

hipError_t launch_copy_view(const float* src, int ld_src, float* dst, int ld_dst, int C, long long P, hipStream_t s) {
  if (C % 4 || ld_src % 4 || ld_dst % 4) return hipErrorInvalidValue;
  const long long n = P * (C / 4);
  long long blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(copy_view_kernel, dim3((unsigned)std::max(1LL, blocks)), dim3(256), 0, s, src, ld_src, dst, ld_dst,
                     C / 4, P);
  return hipGetLastError();
}

}  // namespace kdlae
