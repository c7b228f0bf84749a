// MDTA (transposed channel attention) and GDFN (gated dwconv FFN) kernels, NHWC fp32.
//
// Reference math (KDLAE/KDLAE_model.py):
//   Attention.forward :124-145   qkv_dwconv -> chunk(q,k,v) -> per head q^=q/max(|q|_HW,1e-12),
//                                 k^ likewise -> A = softmax(q^ k^T * temperature) -> A v -> project_out
//   FeedForward.forward :101-106  dwconv -> chunk(x1,x2) -> gelu_erf(x1) * x2
//
// MDTA is restated as three passes so that q and k never touch HBM:
//   1. dwconv_gram: depthwise 3x3 of q,k,v for a run of pixels, v written out, and per head the
//      UN-normalised Gram G = q k^T (v_mfma_f32_16x16x4_f32, pixels as the reduction index) and
//      the squared norms |q_c|^2, |k_c|^2 accumulated -> one partial slot per workgroup.
//   2. gram_reduce: deterministic fixed-order sum of the slots (no float atomics).
//   3. attn_fold: A = softmax(G / (max(|q|,eps) max(|k|,eps)) * temp); M = W_proj . blockdiag(A)
//      written directly in the packed GEMM fragment order, so "A v then project_out" is ONE GEMM
//      (conv_gemm with per-image weights M and the residual add in its epilogue).
#include <type_traits>
#include <utility>

#include "kernels.h"
#include "mfma3.h"
#include "lds_dma.h"

namespace kdlae {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// --------------------------------------------------------------------------- LN statistics
// (mean, rstd) per pixel over C channels (BiasFree/WithBias LN, :50-52 / :67-70), two-pass from
// registers; one wave per pixel, float4 per lane.  Used when a LN-fused GEMM needs K-chunking.
__global__ __launch_bounds__(256) void ln_stats_kernel(const float* __restrict__ x, int ld, int C,
                                                       long long P, float* __restrict__ stats) {
  const int lane = threadIdx.x & 63;
  const long long wave = (blockIdx.x * 256LL + threadIdx.x) >> 6;
  const long long nw = (gridDim.x * 256LL) >> 6;
  const int c4 = C >> 2;
  for (long long pix = wave; pix < P; pix += nw) {
    const float* row = x + pix * ld;
    f32x4 v0 = f32x4{0.f, 0.f, 0.f, 0.f}, v1 = v0;
    if (lane < c4) v0 = *reinterpret_cast<const f32x4*>(row + 4 * lane);
    if (lane + 64 < c4) v1 = *reinterpret_cast<const f32x4*>(row + 4 * (lane + 64));
    float s = (v0.x + v0.y + v0.z + v0.w) + (v1.x + v1.y + v1.z + v1.w);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    const float mean = s / (float)C;
    f32x4 d0 = v0 - mean, d1 = v1 - mean;
    float q = 0.f;
    if (lane < c4) q += d0.x * d0.x + d0.y * d0.y + d0.z * d0.z + d0.w * d0.w;
    if (lane + 64 < c4) q += d1.x * d1.x + d1.y * d1.y + d1.z * d1.z + d1.w * d1.w;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) q += __shfl_xor(q, o);
    if (lane == 0) {
      stats[2 * pix] = mean;
      stats[2 * pix + 1] = 1.0f / sqrtf(q / (float)C + 1e-5f);
    }
  }
}

hipError_t launch_ln_stats(const float* x, int ld, int C, long long P, float* stats, hipStream_t s) {
  long long blocks = (P + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(ln_stats_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, ld, C, P, stats);
  return hipGetLastError();
}

// --------------------------------------------------------------------------- dwconv + Gram
// grid (nslots, heads, B), 256 threads (4 waves); LDS-staged per 64-pixel step.
//  phase 1: wave w computes the depthwise 3x3 of q, k, v for the 16-pixel unit 4*step + w:
//           lane (i = lane & 15, q = lane >> 4) -> channel 16 ct + i at pixels 16u + 4q + s;
//           v goes to HBM, q and k to LDS [64 px][S] (S = Ch padded to 16 mod 32 -> the MFMA
//           operand reads below are bank-conflict free), squared norms accumulate in registers.
//  phase 2: the CT x CT Gram tiles of this head are dealt to the 4 waves; each wave runs
//           v_mfma_f32_16x16x4_f32 over the 64 staged pixels (16 k-steps) from LDS.
template <int CT>
__global__ __launch_bounds__(256) void dwconv_gram_kernel(GramParams p) {
  constexpr int Ch = CT * 16;
  constexpr int S = (Ch % 32 == 16) ? Ch : Ch + 16;
  constexpr int PPW = (CT * CT + 3) / 4;  // Gram tile pairs per wave
  __shared__ float qs[64 * S];
  __shared__ float ks[64 * S];
  __shared__ float nacc[4][4][2 * Ch];  // [wave][lane>>4][q|k channel] running squared norms
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int slot = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int HW = p.H * p.W;
  const int C = p.C;
  const float* __restrict__ X = p.qkv + (long long)b * HW * p.ld;
  float* __restrict__ V = p.v_out + (long long)b * HW * p.ldv;

  const int steps_total = (HW + 63) >> 6;
  const int st_begin = (int)((long long)steps_total * slot / p.nslots);
  const int st_end = (int)((long long)steps_total * (slot + 1) / p.nslots);

  // uniform neighbour deltas (in floats) for the 9 taps
  int dofs[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) dofs[t] = ((t / 3 - 1) * p.W + (t % 3 - 1)) * p.ld;

  f32x4 acc[PPW];
#pragma unroll
  for (int k = 0; k < PPW; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int i = li; i < 2 * Ch; i += 16) nacc[wave][lq][i] = 0.f;

  for (int st = st_begin; st < st_end; ++st) {
    // ---- phase 1: depthwise conv of this wave's unit
    const int u = st * 4 + wave;
    int base[4];
    unsigned okm[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int pix = u * 16 + 4 * lq + s;
      const int y = pix / p.W, x = pix - (pix / p.W) * p.W;
      unsigned m = 0;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
        const bool ok = pix < HW && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W;
        m |= ok ? (1u << t) : 0u;
      }
      okm[s] = m;
      base[s] = (pix < HW ? pix : 0) * p.ld;
    }
#pragma unroll 1
    for (int ct = 0; ct < CT; ++ct) {
      const int cq = h * Ch + ct * 16 + li;
      float n2q = 0.f, n2k = 0.f;
#pragma unroll 1
      for (int part = 0; part < 3; ++part) {
        const int c = cq + part * C;
        float w[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) w[t] = p.wdw[t * 3 * C + c];
        const float bias = p.bdw ? p.bdw[c] : 0.f;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          float a = bias;
#pragma unroll
          for (int t = 0; t < 9; ++t) {
            const bool ok = (okm[s] >> t) & 1u;
            const float xv = X[(ok ? base[s] + dofs[t] : 0) + c];
            a = fmaf(ok ? xv : 0.f, w[t], a);
          }
          const int pix = u * 16 + 4 * lq + s;
          const bool valid = pix < HW;
          a = valid ? a : 0.f;
          const int lp = wave * 16 + 4 * lq + s;
          if (part == 0) {
            qs[lp * S + ct * 16 + li] = a;
            n2q = fmaf(a, a, n2q);
          } else if (part == 1) {
            ks[lp * S + ct * 16 + li] = a;
            n2k = fmaf(a, a, n2k);
          } else if (valid) {
            V[pix * p.ldv + cq] = a;
          }
        }
      }
      nacc[wave][lq][ct * 16 + li] += n2q;
      nacc[wave][lq][Ch + ct * 16 + li] += n2k;
    }
    __syncthreads();
    // ---- phase 2: Gram tiles of this wave over the 64 staged pixels
#pragma unroll
    for (int k = 0; k < PPW; ++k) {
      const int pi = wave * PPW + k;
      if (pi < CT * CT) {
        const int i = pi / CT, j = pi - (pi / CT) * CT;
#pragma unroll
        for (int ks4 = 0; ks4 < 16; ++ks4) {
          const int lp = ks4 * 4 + lq;
          acc[k] = mfma4(qs[lp * S + 16 * i + li], ks[lp * S + 16 * j + li], acc[k]);
        }
      }
    }
    __syncthreads();
  }

  // ---- write this block's slot: Gram tiles in accumulator layout, then norms
  float* out = p.partial + (((long long)b * p.heads + h) * p.nslots + slot) * p.slot_floats;
#pragma unroll
  for (int k = 0; k < PPW; ++k) {
    const int pi = wave * PPW + k;
    if (pi < CT * CT) *reinterpret_cast<f32x4*>(out + (pi * 64 + lane) * 4) = acc[k];
  }
__syncthreads();
  for (int idx = threadIdx.x; idx < 2 * Ch; idx += 256) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int g = 0; g < 4; ++g) t += nacc[w][g][idx];
    out[CT * CT * 256 + idx] = t;
  }
}

// Row-sweep variant (W % 16 == 0): block = (16-column strip, row segment) of one head.
//  * the 3*CT (part, channel-tile) stencil jobs are dealt to the 4 waves; lane (i, q) of a job
//    computes channel 16 ct + i at pixels x0 + 4q + s (s = 0..3) and keeps a rolling 3-row x
//    6-column window, so a new row costs 6 scalar loads per 4 outputs;
//  * per row, q and k go to LDS [16 px][S], v to HBM; then the CT x CT Gram tiles (dealt to the
//    waves) take 4 MFMA k-steps over the row's 16 pixels.  One slot per block.
// waves per block for the sweep kernel: balances the 3*CT stencil jobs and CT^2 Gram tiles while
// keeping per-wave VGPRs low enough for >= 2 waves per SIMD
__host__ __device__ constexpr int gram_waves(int ct) {
  return ct == 1 ? 3 : ct == 2 ? 6 : ct == 3 ? 9 : ct == 4 ? 12 : ct == 5 ? 15 : ct == 6 ? 9 : ct == 7 ? 7 : 12;
}
// Ch = 96 ring: 12 waves (one block per CU).  The DMA waves are the ones without a v job, and at 10
// waves only 2 of the 18 jobs' waves qualified: each issued 11 of the row's 21 LDS-DMA pieces, and that
// issue (60-185 cycles a piece beside MFMAs) paced the row.  At 12 waves the v jobs ride as second jobs
// on waves 0-5, waves 6-11 are DMA waves with 4 pieces each: 2170 -> 1847 us per C96@512^2 launch
// (r04 same-box probe, gpurun_out/ring6b; 13 waves 1954, 14 1947, 16 2032)
constexpr auto KDLAE_RING6_WAVES = 12;
// r03 A/B (profiles/r03_gram_ab_probe.txt, retired): a stencil window rolled in registers across rows
// (6 LDS reads per job and row instead of 18) and q / k staged transposed with a quad swizzle
// (ds_read_b128 operands) were both no faster; neither LDS traffic nor issue is this kernel's limit
// waves per block for the LDS-DMA ring kernel (one block per CU at CT = 6)
constexpr auto KDLAE_RING3_WAVES = 9;
__host__ __device__ constexpr int gram_ring_waves(int ct) {
  return ct == 6 ? KDLAE_RING6_WAVES : ct == 3 ? KDLAE_RING3_WAVES : gram_waves(ct);
}

template <int CT>
__global__ __launch_bounds__(64 * gram_waves(CT)) void dwconv_gram_sweep_kernel(GramParams p, int nseg, int seg_rows) {
  constexpr int NW = gram_waves(CT);
  constexpr int Ch = CT * 16;
  constexpr int S = (Ch % 32 == 16) ? Ch : Ch + 16;
  constexpr int NJ = 3 * CT;               // stencil jobs
  constexpr int JPW = (NJ + NW - 1) / NW;  // jobs per wave
  constexpr int PPW = (CT * CT + NW - 1) / NW;   // Gram tile pairs per wave
  __shared__ float qs[2][16 * S];
  __shared__ float ks[2][16 * S];
  __shared__ float nred[2 * Ch];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int strips = p.W >> 4;
  const int slot = blockIdx.x;
  const int strip = slot % strips, seg = slot / strips;
  const int h = blockIdx.y, b = blockIdx.z;
  const int HW = p.H * p.W;
  const int C = p.C;
  const float* __restrict__ X = p.qkv + (long long)b * HW * p.ld;
  float* __restrict__ V = p.v_out + (long long)b * HW * p.ldv;
  const int x0 = strip * 16 + 4 * lq;      // this lane's first pixel column
  const int y0 = seg * seg_rows, y1 = min(y0 + seg_rows, p.H);

  int chan[JPW], part[JPW];
  float w[JPW][9], bias[JPW], win[JPW][3][6], nxt[JPW][6], n2[JPW];
#pragma unroll
  for (int j = 0; j < JPW; ++j) {
    const int jb = wave + NW * j;
    const int job = jb < NJ ? jb : 0;
    part[j] = job / CT;
    const int ct = job - part[j] * CT;
    chan[j] = part[j] * C + h * Ch + ct * 16 + li;
#pragma unroll
    for (int t = 0; t < 9; ++t) w[j][t] = p.wdw[t * 3 * C + chan[j]];
    bias[j] = p.bdw ? p.bdw[chan[j]] : 0.f;
    n2[j] = 0.f;
  }
  auto load_row = [&](int yy) {  // -> nxt
    const bool oky = (unsigned)yy < (unsigned)p.H;
#pragma unroll
    for (int c6 = 0; c6 < 6; ++c6) {
      const int xx = x0 - 1 + c6;
      const bool ok = oky && (unsigned)xx < (unsigned)p.W;
      const int off = ok ? (yy * p.W + xx) * p.ld : 0;
#pragma unroll
      for (int j = 0; j < JPW; ++j) {
        const float v = X[off + chan[j]];
        nxt[j][c6] = ok ? v : 0.f;
      }
    }
  };
  auto put_row = [&](int slotr) {
#pragma unroll
    for (int j = 0; j < JPW; ++j)
#pragma unroll
      for (int c6 = 0; c6 < 6; ++c6) win[j][slotr][c6] = nxt[j][c6];
  };
  f32x4 acc[PPW];
#pragma unroll
  for (int k = 0; k < PPW; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};

  // rolling window rows y-1, y, y+1 in win[.][0..2]; row y+2 is prefetched into nxt while row y
  // is computed, so one memory latency overlaps a row of work instead of stalling every row
  load_row(y0 - 1);
  put_row(0);
  load_row(y0);
  put_row(1);
  load_row(y0 + 1);
  put_row(2);
  int buf = 0;
  for (int y = y0; y < y1; ++y) {
    load_row(y + 2);
#pragma unroll
    for (int j = 0; j < JPW; ++j) {
      if (wave + NW * j < NJ) {
        const int ct = (wave + NW * j) % CT;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          float a = bias[j];
#pragma unroll
          for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) a = fmaf(win[j][r][s + dx], w[j][3 * r + dx], a);
          const int lp = 4 * lq + s;
          if (part[j] == 0) {
            qs[buf][lp * S + ct * 16 + li] = a;
            n2[j] = fmaf(a, a, n2[j]);
          } else if (part[j] == 1) {
            ks[buf][lp * S + ct * 16 + li] = a;
            n2[j] = fmaf(a, a, n2[j]);
          } else {
            V[(y * p.W + x0 + s) * p.ldv + h * Ch + ct * 16 + li] = a;
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int c6 = 0; c6 < 6; ++c6) win[j][r][c6] = win[j][r + 1][c6];
    }
    put_row(2);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PPW; ++k) {
      const int pi = wave * PPW + k;
      if (pi < CT * CT) {
        const int i = pi / CT, jj = pi - (pi / CT) * CT;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int lp = 4 * lq + s;
          acc[k] = mfma4(qs[buf][lp * S + 16 * i + li], ks[buf][lp * S + 16 * jj + li], acc[k]);
        }
      }
    }
    buf ^= 1;  // double-buffered staging: the next row's writes go to the other buffer
  }

  float* out = p.partial + (((long long)b * p.heads + h) * p.nslots + slot) * p.slot_floats;
#pragma unroll
  for (int k = 0; k < PPW; ++k) {
    const int pi = wave * PPW + k;
    if (pi < CT * CT) *reinterpret_cast<f32x4*>(out + (pi * 64 + lane) * 4) = acc[k];
  }
#pragma unroll
  for (int j = 0; j < JPW; ++j) {
    float t = n2[j];
    t += __shfl_xor(t, 16);
    t += __shfl_xor(t, 32);
    const int jb = wave + NW * j;
    if (jb < NJ && part[j] < 2 && lq == 0) nred[part[j] * Ch + (jb % CT) * 16 + li] = t;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 2 * Ch; idx += 64 * NW) out[CT * CT * 256 + idx] = nred[idx];
}

// DMA-ring row sweep (same blocking as the sweep kernel: 16-column strip x row segment of one
// head).  Rows of the block's input arrive by LDS-DMA into a 6-row ring, and the work is software-
// pipelined by one row: iteration y runs the Gram MFMAs of row y (staging buffer buf) interleaved,
// per k-step, with the depthwise stencil of row y+1 (ring rows y..y+2 -> buffer buf^1), while rows
// y+3, y+4 are in flight and row y+5 is issued.  One barrier per row.
//  * ring row = 18 pixels (strip columns -1..16) x [q | k | v of this head | 1 pad float4];
//    the pad makes the pixel stride 3 Ch + 4 floats, so the stencil's column reads (16 channels x
//    4 pixel groups per wave) fall on 64 distinct banks.  Pad items and out-of-image pixels read
//    p.zeros;
//  * two wave classes.  "DMA waves" (those whose stencil jobs are all q/k) issue every ring DMA,
//    PPD or PPD - 1 pieces each per row (a compile-time count per instantiation; r03 re-issued the
//    last piece of the short waves instead), and their only VMEM ops are those DMAs, so "row y+2
//    has landed" is the compile-time s_waitcnt vmcnt(count * rows issued after it).  The other waves store v and never
//    wait on vmcnt: the barrier after the DMA waves' wait covers them.  The loop body is
//    instantiated per class, so neither carries the other's branches;
//  * Gram MFMA k-step s takes pixel 4 s + (lane >> 4), so the q/k operand reads are
//    bank-conflict-free (S = Ch padded to 16 mod 32).
// f(std::integral_constant<int, J>) for J = 0 .. N-1 (compile-time job slots)
template <int... J, class F>
__device__ __forceinline__ void for_each_int(std::integer_sequence<int, J...>, F&& f) {
  (f(std::integral_constant<int, J>{}), ...);
}

template <int CT>
struct GramRing {
  static constexpr int Ch = CT * 16;
  static constexpr int NW = gram_ring_waves(CT);
  static constexpr int NJ = 3 * CT;
  static constexpr int PS4 = 3 * Ch / 4 + 1;          // float4 per ring pixel
  static constexpr int PS = 4 * PS4;                  // floats per ring pixel
  static constexpr int Items = 18 * PS4;
  static constexpr int Pieces = (Items + 63) / 64;    // 1 KiB DMA wave-instructions per row
  static constexpr int RowF4 = Pieces * 64;
  static constexpr int NSlot = 6;
  static constexpr int S = (Ch % 32 == 16) ? Ch : Ch + 16;
  static constexpr int Stage = 16 * S;  // floats per staging buffer
  static constexpr size_t lds_bytes = (size_t)NSlot * RowF4 * 16 + 4 * Stage * 4 + 2 * Ch * 4;
  // DMA waves: the waves none of whose jobs (w, w + NW, ...) is a v job (job >= 2 CT); with
  // NW > 2 CT these are the trailing waves (the leading ones carry a second, v, job)
  static constexpr bool has_v(int w) {
    for (int jb = w; jb < NJ; jb += NW)
      if (jb >= 2 * CT) return true;
    return false;
  }
  static constexpr int dma_waves() {
    int n = 0;
    for (int w = 0; w < NW; ++w) n += has_v(w) ? 0 : 1;
    return n;
  }
  // rank of wave w among the DMA waves
  static constexpr int dma_rank(int w) {
    int n = 0;
    for (int v = 0; v < w; ++v) n += has_v(v) ? 0 : 1;
    return n;
  }
  static constexpr int NDW = dma_waves();
  static constexpr int PPD = (Pieces + NDW - 1) / NDW;  // pieces per DMA wave per row
  // what stencil job slot j is for every wave of a class (D: the DMA waves, !D: the v waves), so the
  // row loop carries no per-job branches: 0 no wave of the class has the slot, 1 q or k (-> LDS
  // staging) for every wave that has it, 2 v (-> HBM) for every wave that has it, 3 mixed
  static constexpr int job_kind(bool D, int j) {
    bool any = false, lds = false, v = false;
    for (int w = 0; w < NW; ++w) {
      if (has_v(w) == D) continue;
      const int jb = w + NW * j;
      if (jb >= NJ) continue;
      any = true;
      (jb / CT == 2 ? v : lds) = true;
    }
    return !any ? 0 : (lds && v) ? 3 : lds ? 1 : 2;
  }
  // every wave of the class has job slot j
  static constexpr bool job_all(bool D, int j) {
    for (int w = 0; w < NW; ++w)
      if (has_v(w) != D && w + NW * j >= NJ) return false;
    return true;
  }
};

constexpr auto KDLAE_RING_XCD = 1;
template <int CT>
__global__ __launch_bounds__(64 * gram_ring_waves(CT)) void dwconv_gram_ring_kernel(GramParams p, int seg_rows) {
  using R = GramRing<CT>;
  using dma::f32x4;
  constexpr int NW = R::NW, NJ = R::NJ, NDW = R::NDW, PPD = R::PPD;
  constexpr int Ch = R::Ch, S = R::S, PS = R::PS, PS4 = R::PS4;
  constexpr int JPW = (NJ + NW - 1) / NW;
  constexpr int PPW = (CT * CT + NW - 1) / NW;
  static_assert(NDW >= 1 && 3 * PPD < 64, "ring DMA accounting");
  extern __shared__ __attribute__((aligned(16))) dma::f32x4 gring[];
  float* ringf = reinterpret_cast<float*>(gring);
  constexpr int ST = R::Stage;
  float* qs = ringf + R::NSlot * R::RowF4 * 4;  // [2][ST]
  float* ks = qs + 2 * ST;                      // [2][ST]
  float* nred = ks + 2 * ST;                    // [2 Ch]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, lq = lane >> 4;
  const int strips = p.W >> 4;
  // XCD-aware slot order: XCD k (blockIdx.x & 7; nslots % 8 == 0 keeps the 3-D grid's linear ids
  // congruent) walks the slot range [k n / 8, (k+1) n / 8), so neighbouring strips, whose 2 halo
  // columns overlap, are read on the same L2 at about the same time
  const int slot = (KDLAE_RING_XCD && p.nslots % 8 == 0)
                       ? (int)(blockIdx.x & 7) * (p.nslots >> 3) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  const int strip = slot % strips, seg = slot / strips;
  const int h = blockIdx.y, b = blockIdx.z;
  const int HW = p.H * p.W;
  const int C = p.C;
  const float* __restrict__ X = p.qkv + (long long)b * HW * p.ld;
  float* __restrict__ V = p.v_out + (long long)b * HW * p.ldv;
  const int xs = strip * 16;
  const int y0 = seg * seg_rows, y1 = min(y0 + seg_rows, p.H);

  // stencil jobs (part, channel tile) dealt round-robin; weights in registers before any DMA
  int part[JPW], ctj[JPW];
  float w[JPW][9], bias[JPW], n2[JPW];
#pragma unroll
  for (int j = 0; j < JPW; ++j) {
    const int jb = wave + NW * j;
    const int job = jb < NJ ? jb : 0;
    part[j] = job / CT;
    ctj[j] = job - part[j] * CT;
    const int c = part[j] * C + h * Ch + ctj[j] * 16 + li;
#pragma unroll
    for (int t = 0; t < 9; ++t) w[j][t] = p.wdw[t * 3 * C + c];
    bias[j] = p.bdw ? p.bdw[c] : 0.f;
    n2[j] = 0.f;
  }
  // DMA sources (DMA waves): piece k covers ring items 64k..64k+63; byte offset of the item's
  // column within an image row, ~0u -> zero line
  const bool dma_wave = !R::has_v(wave);
  const int drank = R::dma_rank(wave);
  // (issue priority of either wave class: r05 A/B, DMA waves +4%, v waves +-1%: default priority,
  // profiles/r05p3_ring_prio_ab.txt)
  unsigned colo[PPD];
#pragma unroll
  for (int j = 0; j < PPD; ++j) {
    const int k = min(drank + NDW * j, R::Pieces - 1);
    const int it = k * 64 + lane;
    const int px = it / PS4, r = it - (it / PS4) * PS4;
    const int xx = xs - 1 + px;
    const int pt = r / (Ch / 4), c4 = r - pt * (Ch / 4);
    const bool ok = it < R::Items && r < PS4 - 1 && (unsigned)xx < (unsigned)p.W;
    colo[j] = ok ? (unsigned)((xx * p.ld + pt * C + h * Ch + 4 * c4) * 4) : ~0u;
  }
  const unsigned rowbytes = (unsigned)p.W * (unsigned)p.ld * 4u;
  const char* Xb = reinterpret_cast<const char*>(X);
  // a DMA wave issues N = PPD or PPD - 1 pieces per row (ranks below Pieces % NDW carry the extra
  // one), a compile-time count per instantiation of the loop body so its vmcnt waits stay exact
  auto issue = [&](int yy, auto ntag) {
    constexpr int N = decltype(ntag)::value;
    f32x4* sl = gring + ((yy + R::NSlot) % R::NSlot) * R::RowF4;
    const bool oky = (unsigned)yy < (unsigned)p.H;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const int k = min(drank + NDW * j, R::Pieces - 1);
      const void* src = (oky && colo[j] != ~0u) ? (const void*)(Xb + (unsigned)yy * rowbytes + colo[j])
                                                 : (const void*)p.zeros;
      dma::dma16(src, sl + 64 * k);
    }
  };
  // DMA waves: wait until only the DMAs of the `ra` youngest rows are outstanding
  auto wait_rows = [&](int ra, auto ntag) {
    constexpr int N = decltype(ntag)::value;
    if (ra >= 3) dma::wait_vmcnt<3 * N>();
    else if (ra == 2) dma::wait_vmcnt<2 * N>();
    else if (ra == 1) dma::wait_vmcnt<N>();
    else dma::wait_vmcnt<0>();
  };

  f32x4 acc[PPW];
#pragma unroll
  for (int k = 0; k < PPW; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};

  dma::wait_vmcnt<0>();  // the weight loads above, so the first stencil does not drain the ring

  auto run = [&](auto dma_wave, auto ntag) {
    constexpr bool D = decltype(dma_wave)::value;
    // stencil of output pixel s (of this lane's 4) of ring row r for every job; q/k -> staging
    // buffer sb, v -> HBM (non-DMA waves only)
    float win[JPW][3][6];
    auto load_win = [&](int r) {
      const float* rm = ringf + ((r + 5) % R::NSlot) * R::RowF4 * 4 + 4 * lq * PS + li;
      const float* r0 = ringf + (r % R::NSlot) * R::RowF4 * 4 + 4 * lq * PS + li;
      const float* rp = ringf + ((r + 1) % R::NSlot) * R::RowF4 * 4 + 4 * lq * PS + li;
#pragma unroll
      for (int j = 0; j < JPW; ++j) {
        if (R::job_kind(D, j) == 0) continue;  // no wave of this class has job slot j
        const int co = part[j] * Ch + ctj[j] * 16;
#pragma unroll
        for (int c6 = 0; c6 < 6; ++c6) {
          win[j][0][c6] = rm[c6 * PS + co];
          win[j][1][c6] = r0[c6 * PS + co];
          win[j][2][c6] = rp[c6 * PS + co];
        }
      }
    };
    auto stencil = [&](int r, int sb, int s) {
      const int lp = 4 * lq + s;
      auto one = [&](auto jtag) {
        constexpr int j = decltype(jtag)::value;
        constexpr int K = R::job_kind(D, j);
        if constexpr (K != 0) {
          if (R::job_all(D, j) || wave + NW * j < NJ) {
            float a = bias[j];
#pragma unroll
            for (int rr = 0; rr < 3; ++rr)
#pragma unroll
              for (int dx = 0; dx < 3; ++dx) a = fmaf(win[j][rr][s + dx], w[j][3 * rr + dx], a);
            auto to_lds = [&]() {
              float* dst = part[j] == 0 ? qs : ks;
              dst[sb * 16 * S + lp * S + ctj[j] * 16 + li] = a;
              n2[j] = fmaf(a, a, n2[j]);
            };
            auto to_v = [&]() { V[(r * p.W + xs + lp) * p.ldv + h * Ch + ctj[j] * 16 + li] = a; };
            if constexpr (K == 1) {
              to_lds();
            } else if constexpr (K == 2) {
              to_v();
            } else if (part[j] < 2) {
              to_lds();
            } else {
              to_v();
            }
          }
        }
      };
      for_each_int(std::make_integer_sequence<int, JPW>{}, one);
    };

    // prologue: rows y0-1 .. min(y0+4, y1) in flight; stencil(y0) once rows y0-1..y0+1 landed
    if (D)
      for (int yy = y0 - 1; yy <= min(y0 + 4, y1); ++yy) issue(yy, ntag);
    if (y0 < y1) {
      if (D) wait_rows(max(0, min(y0 + 4, y1) - (y0 + 1)), ntag);
      dma::barrier_lds();
      load_win(y0);
#pragma unroll
      for (int s = 0; s < 4; ++s) stencil(y0, 0, s);
    }
    int buf = 0;
    for (int y = y0; y < y1; ++y) {
      const bool st = y + 1 < y1;
      // rows y..y+2 landed: the younger DMAs are rows y+3 .. min(y+4, y1)
      if (D && st) wait_rows(max(0, min(y + 4, y1) - (y + 2)), ntag);
      dma::barrier_lds();
      if (D && y + 5 <= y1) issue(y + 5, ntag);  // into the slot of row y-1, last read by stencil(y)
      float qv[PPW][4], kv[PPW][4];
#pragma unroll
      for (int k = 0; k < PPW; ++k) {
        const int pi = (CT * CT) % NW == 0 ? wave * PPW + k : min(wave * PPW + k, CT * CT - 1);
        const int i = pi / CT, jj = pi - (pi / CT) * CT;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int lp = 4 * s + lq;
          qv[k][s] = qs[buf * 16 * S + lp * S + 16 * i + li];
          kv[k][s] = ks[buf * 16 * S + lp * S + 16 * jj + li];
        }
      }
      if (st) load_win(y + 1);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int k = 0; k < PPW; ++k)
          if ((CT * CT) % NW == 0 || wave * PPW + k < CT * CT) acc[k] = mfma4(qv[k][s], kv[k][s], acc[k]);
        if (st) stencil(y + 1, buf ^ 1, s);
      }
      buf ^= 1;
    }
  };
  constexpr int PX = R::Pieces % NDW;  // DMA ranks below PX issue PPD pieces, the rest PPD - 1
  if (!dma_wave) run(std::false_type{}, std::integral_constant<int, 0>{});
  else if (PX == 0 || drank < PX) run(std::true_type{}, std::integral_constant<int, PPD>{});
  else run(std::true_type{}, std::integral_constant<int, (PX == 0 ? PPD : PPD - 1)>{});

  float* out = p.partial + (((long long)b * p.heads + h) * p.nslots + slot) * p.slot_floats;
#pragma unroll
  for (int k = 0; k < PPW; ++k) {
    const int pi = wave * PPW + k;
    if (pi < CT * CT) *reinterpret_cast<f32x4*>(out + (pi * 64 + lane) * 4) = acc[k];
  }
#pragma unroll
  for (int j = 0; j < JPW; ++j) {
    float t = n2[j];
    t += __shfl_xor(t, 16);
    t += __shfl_xor(t, 32);
    const int jb = wave + NW * j;
    if (jb < NJ && part[j] < 2 && lq == 0) nred[part[j] * Ch + ctj[j] * 16 + li] = t;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 2 * Ch; idx += 64 * NW) out[CT * CT * 256 + idx] = nred[idx];
}

// generic: the 64-pixel-step kernel whatever the width (self-test route; production takes it only
// for W % 16 != 0 or a slot count that does not tile the strips)
template <int CT>
static void launch_gram_ct(const GramParams& p, bool generic, hipStream_t s) {
  if (generic) {
    hipLaunchKernelGGL(dwconv_gram_kernel<CT>, dim3(p.nslots, p.heads, p.Bn), dim3(256), 0, s, p);
    return;
  }
  if constexpr (CT <= 6) {
    using R = GramRing<CT>;
    if (p.zeros && p.W % 16 == 0 && p.nslots % (p.W / 16) == 0 && p.ld % 4 == 0 && p.C % 4 == 0 &&
        (unsigned long long)p.H * p.W * p.ld * 4 < (1ull << 32)) {
      const int nseg = p.nslots / (p.W / 16);
      const int seg_rows = (p.H + nseg - 1) / nseg;
      hipLaunchKernelGGL(dwconv_gram_ring_kernel<CT>, dim3(p.nslots, p.heads, p.Bn), dim3(64 * gram_ring_waves(CT)),
                         R::lds_bytes, s, p, seg_rows);
      return;
    }
  }
  if (p.W % 16 == 0 && p.nslots % (p.W / 16) == 0) {
    const int nseg = p.nslots / (p.W / 16);
    const int seg_rows = (p.H + nseg - 1) / nseg;
    hipLaunchKernelGGL(dwconv_gram_sweep_kernel<CT>, dim3(p.nslots, p.heads, p.Bn), dim3(64 * gram_waves(CT)), 0, s,
                       p, nseg, seg_rows);
  } else {
    hipLaunchKernelGGL(dwconv_gram_kernel<CT>, dim3(p.nslots, p.heads, p.Bn), dim3(256), 0, s, p);
  }
}

hipError_t launch_dwconv_gram(const GramParams& p, hipStream_t s) { return launch_dwconv_gram_route(p, 0, s); }

hipError_t launch_dwconv_gram_route(const GramParams& p, int route, hipStream_t s) {
  const bool g = route == 2;
  switch (p.Ch / 16) {
    case 1: launch_gram_ct<1>(p, g, s); break;
    case 2: launch_gram_ct<2>(p, g, s); break;
    case 3: launch_gram_ct<3>(p, g, s); break;
    case 4: launch_gram_ct<4>(p, g, s); break;
    case 5: launch_gram_ct<5>(p, g, s); break;
    case 6: launch_gram_ct<6>(p, g, s); break;
    case 7: launch_gram_ct<7>(p, g, s); break;
    case 8: launch_gram_ct<8>(p, g, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// --------------------------------------------------------------------------- slot reduction
// reduced[bh][i] = sum over the nslots partial slots, in a fixed order and in float64 (each slot is
// an f32 sum over <= 1024 pixels; the HW-long sum over slots is where f32 loses the most: torch's
// f32 q.k^T over all HW pixels is what puts the reference's own f32 output 3e-3 from its f64 output
// on the config-1 MDD input, profiles/r03_config1_precision.txt): wave w of a block sums the
// slot range [w n / 8, (w+1) n / 8) sequentially for 64 consecutive floats (one 256 B line per
// load), then lane i adds the 8 wave sums in wave order.  Deterministic and batch-invariant (the
// slot partition depends on the image size only).  r01's kernel gave each float one thread that
// walked all slots (160 blocks at 1024^2: a latency-bound 64 us per launch).
constexpr int kRedWaves = 8;
__global__ __launch_bounds__(64 * kRedWaves) void gram_reduce_kernel(const float* __restrict__ partial,
                                                                     float* __restrict__ reduced, int nslots,
                                                                     int slot_floats) {
  __shared__ double part[kRedWaves][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int idx = blockIdx.x * 64 + lane;
  const long long bh = blockIdx.y;
  const int k0 = wave * nslots / kRedWaves, k1 = (wave + 1) * nslots / kRedWaves;
  double s = 0.0;
  if (idx < slot_floats) {
    const float* src = partial + bh * nslots * (long long)slot_floats + idx;
#pragma unroll 8
    for (int k = k0; k < k1; ++k) s += (double)src[(long long)k * slot_floats];
  }
  part[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && idx < slot_floats) {
    double t = part[0][lane];
#pragma unroll
    for (int w = 1; w < kRedWaves; ++w) t += part[w][lane];
    reduced[bh * slot_floats + idx] = (float)t;
  }
}

hipError_t launch_gram_reduce(const float* partial, float* reduced, int Bn, int heads, int nslots,
                              int slot_floats, hipStream_t s) {
  dim3 grid((slot_floats + 63) / 64, Bn * heads);
  hipLaunchKernelGGL(gram_reduce_kernel, grid, dim3(64 * kRedWaves), 0, s, partial, reduced, nslots, slot_floats);
  return hipGetLastError();
}

// --------------------------------------------------------------------------- softmax + fold
// grid (C/16, heads, B).  Each block rebuilds A for (b, h) in LDS, then computes 16 rows of
// M[n][h*Ch + c2] = sum_c1 Wproj[n][h*Ch + c1] * A[c1][c2], stored in split fragment order (the GEMM
// kernels' weight format, mfma3.h).
__global__ __launch_bounds__(256) void attn_fold_kernel(const float* __restrict__ reduced, int slot_floats,
                                                        const float* __restrict__ proj,
                                                        const float* __restrict__ temp,
                                                        float* __restrict__ Mp, int C, int heads) {
  extern __shared__ float sm[];
  const int Ch = C / heads;
  const int CT = Ch / 16;
  float* A = sm;                  // [Ch][Ch + 1]
  float* nrm = sm + Ch * (Ch + 1);  // [2 Ch]: 1/max(|q|,eps), 1/max(|k|,eps)
  const int nb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const float* G = reduced + ((long long)b * heads + h) * slot_floats;
  const int ldA = Ch + 1;
  // decode the accumulator layout: G[(i*CT + j)*256 + lane*4 + e] = Gram[16i + 4(lane>>4) + e][16j + (lane&15)]
  for (int idx = threadIdx.x; idx < CT * CT * 256; idx += 256) {
    const int e = idx & 3, lane = (idx >> 2) & 63, ij = idx >> 8;
    const int i = ij / CT, j = ij - (ij / CT) * CT;
    A[(16 * i + 4 * (lane >> 4) + e) * ldA + 16 * j + (lane & 15)] = G[idx];
  }
  for (int c = threadIdx.x; c < 2 * Ch; c += 256) {
    const float n2 = G[CT * CT * 256 + c];
    nrm[c] = 1.0f / fmaxf(sqrtf(n2), 1e-12f);
  }
  __syncthreads();
  const float tp = temp[h];
  for (int r = threadIdx.x; r < Ch; r += 256) {
    float* row = A + r * ldA;
    const float sq = nrm[r];
    float mx = -INFINITY;
    for (int c = 0; c < Ch; ++c) {
      const float l = (row[c] * sq * nrm[Ch + c]) * tp;
      row[c] = l;
      mx = fmaxf(mx, l);
    }
    float sum = 0.f;
    for (int c = 0; c < Ch; ++c) {
      const float e = expf(row[c] - mx);
      row[c] = e;
      sum += e;
    }
    const float inv = 1.0f / sum;
    for (int c = 0; c < Ch; ++c) row[c] *= inv;
  }
  __syncthreads();
  // M in split fragment order (mfma3.h): element (n, k) is bf16 j of lane (n & 15) + 16 q in the three
  // planes of record (n >> 4, k >> 5), with kk = k & 31, q = (kk & 15) >> 2, j = 4 (kk >> 4) + (kk & 3)
  const int kgroups = C / 16, kpt = (kgroups + 1) / 2;
  __bf16* Mb = reinterpret_cast<__bf16*>(Mp + (long long)b * split3_floats(kgroups, kgroups));
  auto put = [&](int n, int k, float v) {
    const int kk = k & 31;
    const int lane = (n & 15) + 16 * ((kk & 15) >> 2), j = 4 * (kk >> 4) + (kk & 3);
    const long long slot = ((long long)((n >> 4) * kpt + (k >> 5)) * 3) * 64 + lane;
    __bf16 vh, vm, vl;
    split1(v, vh, vm, vl);
    Mb[slot * 8 + j] = vh;
    Mb[(slot + 64) * 8 + j] = vm;
    Mb[(slot + 128) * 8 + j] = vl;
  };
  for (int idx = threadIdx.x; idx < 16 * Ch; idx += 256) {
    const int nl = idx / Ch, c2 = idx - (idx / Ch) * Ch;
    const int n = nb * 16 + nl;
    const float* wr = proj + (long long)n * C + h * Ch;
    float s = 0.f;
    for (int c1 = 0; c1 < Ch; ++c1) s = fmaf(wr[c1], A[c1 * ldA + c2], s);
    put(n, h * Ch + c2, s);
  }
  // an odd k-group count: the last pair's upper half (k = C .. C + 15) is zero
  if ((kgroups & 1) && h == heads - 1)
    for (int idx = threadIdx.x; idx < 256; idx += 256) put(nb * 16 + (idx >> 4), C + (idx & 15), 0.f);
}

hipError_t launch_attn_fold(const float* reduced, int slot_floats, const float* proj, const float* temp,
                            float* Mpacked, int Bn, int C, int heads, hipStream_t s) {
  const int Ch = C / heads;
  const size_t lds = (size_t)(Ch * (Ch + 1) + 2 * Ch) * sizeof(float);
  dim3 grid(C / 16, heads, Bn);
  hipLaunchKernelGGL(attn_fold_kernel, grid, dim3(256), lds, s, reduced, slot_floats, proj, temp, Mpacked,
                     C, heads);
  return hipGetLastError();
}

// --------------------------------------------------------------------------- GDFN dwconv + gate
// out[p][c] = gelu_erf(dw(x1)[p][c]) * dw(x2)[p][c], c < hidS; float4 of channels per thread.
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

// Vertical sweep: thread = (channel quad c of x1 and the same quad of x2, one column x) walking a
// segment of rows.  The 3x3 weights of its 8 channels sit in registers for the whole sweep and a
// rolling 3-row x 3-column window of float4s means each new output row costs 6 float4 loads
// (3 columns x {x1, x2}); the column neighbours are the adjacent lanes' loads (L1 hits), so HBM
// sees each input element ~once.  Lanes run along channels -> coalesced 16 B per lane.
constexpr int kGateRows = 32;

__global__ __launch_bounds__(256) void dwconv_gate_kernel(GateParams p) {
  extern __shared__ __attribute__((aligned(16))) f32x4 wsh[];  // [9][2][256 quads] of this block's channels
  const int c4n = p.hidS >> 2;                     // channel quads per half
  const int cols_per_block = 256 / c4n > 0 ? 256 / c4n : 1;
  const int tid = threadIdx.x;
  const int cq_groups = (c4n + 255) / 256;         // >1 only when hidS > 1024
  const int col_groups = (p.W + cols_per_block - 1) / cols_per_block;
  const int segs = (p.H + kGateRows - 1) / kGateRows;
  // XCD-aware remap (blocks b and b+8 share an XCD's L2): consecutive logical blocks — adjacent
  // column groups whose halo columns overlap — land on the same XCD.  Grid is padded to 8k.
  const int nb = p.Bn * segs * col_groups * cq_groups;
  const int per = (int)(gridDim.x >> 3);
  int bid = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (bid >= nb) return;
  const int cqg = bid % cq_groups; bid /= cq_groups;
  const int colg = bid % col_groups; bid /= col_groups;
  const int seg = bid % segs; bid /= segs;
  const int b = bid;
  const int nq = min(256, c4n - cqg * 256);        // channel quads handled by this block
  const int two = 2 * p.hidS;
  for (int i = tid; i < 9 * 2 * nq; i += 256) {
    const int t = i / (2 * nq), rem = i - t * 2 * nq, half = rem / nq, q = rem - half * nq;
    wsh[(t * 2 + half) * 256 + q] =
        *reinterpret_cast<const f32x4*>(p.w + t * two + half * p.hidS + 4 * (cqg * 256 + q));
  }
  __syncthreads();
  const int ql = c4n >= 256 ? tid : tid % c4n;
  const int c4 = cqg * 256 + ql;
  const int x = colg * cols_per_block + (c4n >= 256 ? 0 : tid / c4n);
  if (b >= p.Bn || ql >= nq || x >= p.W) return;
  if (c4n < 256 && tid >= cols_per_block * c4n) return;
  const int c = 4 * c4;
  const int HW = p.H * p.W;
  const float* __restrict__ X = p.x + (long long)b * HW * p.ld;
  float* __restrict__ O = p.out + (long long)b * HW * p.ldo;
  const f32x4 b1 = p.b ? *reinterpret_cast<const f32x4*>(p.b + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 b2 = p.b ? *reinterpret_cast<const f32x4*>(p.b + p.hidS + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool okl = x > 0, okr = x + 1 < p.W;
  // window rows: [0] = y-1, [1] = y, [2] = y+1 (all landed); nx = row y+2 (in flight)
  f32x4 r1[3][3], r2[3][3], n1[3], n2[3];
  auto load_row = [&](int yy, f32x4 (&d1)[3], f32x4 (&d2)[3]) {
    const bool oky = (unsigned)yy < (unsigned)p.H;
    const int base = (oky ? yy : 0) * p.W;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const bool ok = oky && (j == 0 ? okl : (j == 2 ? okr : true));
      const int off = (ok ? base + x + j - 1 : 0) * p.ld + c;
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(X + off);
      const f32x4 v2 = *reinterpret_cast<const f32x4*>(X + off + p.hidS);
      d1[j] = ok ? v1 : z;
      d2[j] = ok ? v2 : z;
    }
  };
  const int y0 = seg * kGateRows;
  const int y1 = min(y0 + kGateRows, p.H);
  load_row(y0 - 1, r1[0], r2[0]);
  load_row(y0, r1[1], r2[1]);
  load_row(y0 + 1, r1[2], r2[2]);
  for (int y = y0; y < y1; ++y) {
    load_row(y + 2, n1, n2);  // prefetch; consumed next iteration
    asm volatile("" ::: "memory");  // keep the weight reads in LDS (no hoisting into 72 VGPRs)
    f32x4 a1 = b1, a2 = b2;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        a1 = r1[i][j] * wsh[((3 * i + j) * 2 + 0) * 256 + ql] + a1;
        a2 = r2[i][j] * wsh[((3 * i + j) * 2 + 1) * 256 + ql] + a2;
      }
      __builtin_amdgcn_sched_barrier(0);  // at most one window row of weights live at a time
    }
    f32x4 o;
    o.x = gelu_erf(a1.x) * a2.x;
    o.y = gelu_erf(a1.y) * a2.y;
    o.z = gelu_erf(a1.z) * a2.z;
    o.w = gelu_erf(a1.w) * a2.w;
    *reinterpret_cast<f32x4*>(O + (y * p.W + x) * p.ldo + c) = o;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      r1[0][j] = r1[1][j]; r2[0][j] = r2[1][j];
      r1[1][j] = r1[2][j]; r2[1][j] = r2[2][j];
      r1[2][j] = n1[j];    r2[2][j] = n2[j];
    }
  }
}

hipError_t launch_dwconv_gate(const GateParams& p, hipStream_t s) {
  const int c4n = p.hidS / 4;
  const int cols_per_block = 256 / c4n > 0 ? 256 / c4n : 1;
  long long blocks = (long long)p.Bn * ((p.H + kGateRows - 1) / kGateRows) *
                     ((p.W + cols_per_block - 1) / cols_per_block) * ((c4n + 255) / 256);
  blocks = (blocks + 7) / 8 * 8;  // XCD remap needs a multiple of 8
  const size_t lds = (size_t)9 * 2 * 256 * sizeof(f32x4);
  hipLaunchKernelGGL(dwconv_gate_kernel, dim3((unsigned)blocks), dim3(256), lds, s, p);
  return hipGetLastError();
}

}  // namespace kdlae
