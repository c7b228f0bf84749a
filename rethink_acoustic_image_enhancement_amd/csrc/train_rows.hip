// Row-streaming MFMA GEMM of the training step (gfx950): C(m, n) = sum_k A(m, k) B(k, n) [+ bias[n]]
// [+ rs[n] R(m, n)] for the tall, narrow contractions — the 1x1 conv forward (A = activations, B = W^T)
// and dX (A = dY, B = W), and the MDTA per-(image, head) products A v, dv = dout A, dq, dk
// (KDLAE_model.py:99-106, :124-145 and their derivatives).
//
// The inference GEMM's layout (gemm.hip) with the weights taken raw: a block stages its NT output
// tiles' weights for the whole K into LDS once, split into bf16 planes in split fragment order
// (mfma3.h: record (tile t, k-group pair G) = planes h, m, l of lane (li, lq) holding
// B(32G + 4lq + j, 16t + li), j < 4, and B(32G + 16 + 4lq + j - 4, 16t + li), j >= 4), straight from
// the caller's B (the flat parameter buffer, or an attention matrix) — no packed copy to refresh after
// an optimizer step.  A rows stream HBM -> VGPRs as float4 (lane: pixel li, channels 16g + 4lq..+3);
// two k-groups' float4 split in registers ARE the v_mfma_f32_16x16x32_bf16 B operand, so A never
// touches LDS; the next (row tile, k-chunk)'s A registers load while the current one's MFMAs run.
// The accumulator of (tile t, subtile r) holds output channels 16t + 4lq..+3 of pixel 16r + li: one
// float4 store per lane.  A block walks row tiles with a grid stride, so the weight staging is paid
// once per block, not per tile.
// Products: the split-bf16 form of every inference GEMM (mfma3.h: six bf16 MFMAs per 32-deep pair,
// as accurate as an fp32 fma chain, 2.67x the f32 MFMA rate).  Summation order per output: pair
// ascending, mfma6 term order; bias, then the residual added after the K sum.
#include <stdint.h>

#include "mfma3.h"
#include "train_kernels.h"

namespace kdlae {
namespace train {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;            // 4 waves
constexpr int kRT = 2;                   // 16-row subtiles per wave
constexpr int kTileRows = 4 * kRT * 16;  // 128 rows per block tile
constexpr int kKC = 4;                   // k-groups (of 16) per A chunk

struct RowsArgs {
  TGemm g;
  int ncb, gx;    // column blocks, row-block slots (grid.x = ncb * gx rounded up to 8)
  int kg;         // k-groups: ceil(K / 16)
  int kp;         // k-group pairs: ceil(kg / 2)
  int nchunk;     // ceil(kg / kKC)
  int row_tiles;  // ceil(M / kTileRows)
  int klast;      // K - 16 (kg - 1): valid k in the last group (16 = full)
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* base, long long bytes) {
  const long long cap = 0x7fffff00LL;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, (int)(bytes < cap ? bytes : cap), 0x00020000);
}
constexpr unsigned kOOB = 0x80000000u;  // past every descriptor's range: loads give 0, stores drop

// Every global access in the streaming loop is an unconditional buffer op (out-of-range rows /
// columns / k-groups take the kOOB offset), so each iteration issues the same number of vector
// memory ops and the compiler's vmcnt waits for the current chunk's A registers stay exact instead
// of draining the next chunk's prefetch (and the previous tile's stores).
// (2 waves per SIMD: the r03 sweep measured a 1-wave-per-SIMD register budget slower)
template <int NT, bool HASR, bool VECC>
__global__ __launch_bounds__(kThreads, 2) void tgemm_rows_kernel(RowsArgs a) {
  // [NT][kp] split records (3 KiB), then [NT][4] bias and [NT][4] residual scale
  extern __shared__ __attribute__((aligned(16))) f32x4 wl[];
  const TGemm& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int kg = a.kg;
  // dispatch d runs on XCD d % 8: logical slot L = (d % 8) * (grid / 8) + d / 8 puts consecutive L
  // on one XCD, and the column blocks of a row block are consecutive L — they stream the same A
  // rows through that XCD's L2 at about the same time
constexpr auto KDLAE_ROWS_XCD = 1;
  const int per = (int)(gridDim.x >> 3);
  const int L = KDLAE_ROWS_XCD ? (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  if (L >= a.ncb * a.gx) return;
  const int cbk = L % a.ncb, rbk = L / a.ncb;
  const int n0 = cbk * NT * 16;
  const int z = blockIdx.z, z1 = z / g.nz2, z2 = z - z1 * g.nz2;

  // ---- stage this block's weight records (split), bias and residual scale
  const int kp = a.kp;
  const float* B = g.B + z1 * g.bB1 + z2 * g.bB2;
  const bool bk1 = g.sbk == 1 && ((uintptr_t)B & 15) == 0 && (g.sbn & 3) == 0;
  for (int idx = tid; idx < NT * kp * 64; idx += kThreads) {
    const int l = idx & 63, tg = idx >> 6;
    const int t = tg / kp, G = tg - t * kp;
    const int n = n0 + 16 * t + (l & 15);
    f32x4 v[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 32 * G + 16 * h + 4 * (l >> 4);
      v[h] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (n < g.N) {
        if (bk1 && k + 3 < g.K) {
          v[h] = *reinterpret_cast<const f32x4*>(B + (long long)n * g.sbn + k);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (k + e < g.K) v[h][e] = B[(long long)(k + e) * g.sbk + (long long)n * g.sbn];
        }
      }
    }
    const F3 w = split3(v[0], v[1]);
    f32x4* rec = wl + (long long)(t * kp + G) * kRec3 + l;
    rec[0] = __builtin_bit_cast(f32x4, w.h);
    rec[64] = __builtin_bit_cast(f32x4, w.m);
    rec[128] = __builtin_bit_cast(f32x4, w.l);
  }
  f32x4* bl = wl + NT * kp * kRec3;
  const float* rs = g.rs ? g.rs + z1 * g.brs1 + z2 * g.brs2 : nullptr;
  for (int idx = tid; idx < NT * 8; idx += kThreads) {
    const int which = idx / (NT * 4), qi = idx - which * NT * 4;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = n0 + 4 * qi + e;
      if (n < g.N) v[e] = which == 0 ? (g.bias ? g.bias[n] : 0.f) : (rs ? rs[n] : 1.f);
    }
    bl[idx] = v;
  }
  __syncthreads();

  // ---- stream A
  const float* A = g.A + z1 * g.bA1 + z2 * g.bA2;
  const __amdgpu_buffer_rsrc_t ra = rsrc(A, (long long)g.M * g.sam * 4);
  const unsigned lda4 = (unsigned)g.sam * 4u;
  const int nmine = (a.row_tiles - rbk + a.gx - 1) / a.gx;
  const int items = nmine * a.nchunk;
  // valid elements of this lane's quad in the last k-group (K % 16 != 0: the pad columns of a
  // ld-rounded view may hold anything; the zero weights there must not meet an Inf / NaN)
  const int kv_last = a.klast - 4 * lq;

  float* C = g.C + z1 * g.bC1 + z2 * g.bC2;
  const __amdgpu_buffer_rsrc_t rc = rsrc(C, (long long)g.M * g.scm * 4);
  [[maybe_unused]] __amdgpu_buffer_rsrc_t rr;
  if constexpr (HASR) rr = rsrc(g.R + z1 * g.bR1 + z2 * g.bR2, (long long)g.M * g.srm * 4);
  // per output tile t: this lane's column quad n0 + 16t + 4lq; its byte offset within a row, or
  // kOOB (VECC: whole quad past N) — per element for the scalar-store path
  unsigned coff[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n = n0 + 16 * t + 4 * lq;
    coff[t] = n < g.N ? 4u * (unsigned)n : kOOB;
  }

  auto load = [&](int i, f32x4 (&dst)[kRT][kKC]) {
    const int tile = rbk + a.gx * (i / a.nchunk), ch = i % a.nchunk;
    const int row0 = tile * kTileRows + wave * (kRT * 16);
#pragma unroll
    for (int r = 0; r < kRT; ++r) {
      const int m = row0 + 16 * r + li;
      const unsigned base = m < g.M ? (unsigned)m * lda4 + 16u * lq : kOOB;
#pragma unroll
      for (int gi = 0; gi < kKC; ++gi) {
        const int gg = ch * kKC + gi;
        const unsigned off = gg < kg ? base + 64u * gg : kOOB;
        dst[r][gi] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, (int)off, 0, 0));
      }
    }
  };
  // residual of item i's tile (every item issues it; only a tile's last chunk reads real rows),
  // issued before the prefetch that precedes the item's MFMAs
  auto load_res = [&](int i, f32x4 (&dst)[NT][kRT]) {
    const int tile = rbk + a.gx * (i / a.nchunk);
    const bool closes = i % a.nchunk == a.nchunk - 1;
    const int row0 = tile * kTileRows + wave * (kRT * 16);
#pragma unroll
    for (int r = 0; r < kRT; ++r) {
      const int m = row0 + 16 * r + li;
      const unsigned rb = (unsigned)m * (unsigned)g.srm * 4u;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const unsigned off = (closes && m < g.M && coff[t] != kOOB) ? rb + coff[t] : kOOB;
        dst[t][r] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, (int)off, 0, 0));
      }
    }
  };

  f32x4 acc[NT][kRT];
  [[maybe_unused]] f32x4 res[NT][kRT];

  auto compute = [&](int i, f32x4 (&av)[kRT][kKC]) {
    const int tile = rbk + a.gx * (i / a.nchunk), ch = i % a.nchunk;
    if (ch == 0) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < kRT; ++r) acc[t][r] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (a.klast < 16 && ch == a.nchunk - 1) {
      const int gl = kg - 1 - ch * kKC;  // the last k-group's slot in this chunk
#pragma unroll
      for (int gi = 0; gi < kKC; ++gi)
        if (gi == gl)
#pragma unroll
          for (int r = 0; r < kRT; ++r)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (e >= kv_last) av[r][gi][e] = 0.f;
    }
#pragma unroll
    for (int pi = 0; pi < kKC / 2; ++pi) {
      const int G = ch * (kKC / 2) + pi;  // (k-groups past kg were loaded as zeros)
      if (G < kp) {
        F3 xs[kRT];
#pragma unroll
        for (int r = 0; r < kRT; ++r) xs[r] = split3(av[r][2 * pi], av[r][2 * pi + 1]);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const F3 w = load_w3(wl + (t * kp + G) * kRec3, lane);
#pragma unroll
          for (int r = 0; r < kRT; ++r) acc[t][r] = mfma6(w, xs[r], acc[t][r]);
        }
      }
    }
    // epilogue of a tile's last chunk (an unconditional epilogue with the earlier chunks' stores
    // sent to kOOB measured up to 25% slower): lane (li, lq) of (t, r) holds channels
    // n0 + 16t + 4lq .. +3 of row 16r + li
    const bool closes = ch == a.nchunk - 1;
    if (!closes) return;
    const int row0 = tile * kTileRows + wave * (kRT * 16);
#pragma unroll
    for (int r = 0; r < kRT; ++r) {
      const int m = row0 + 16 * r + li;
      const unsigned cb = (closes && m < g.M) ? (unsigned)m * (unsigned)g.scm * 4u : kOOB;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        f32x4 v = acc[t][r] + bl[4 * t + lq];
        if constexpr (HASR) v += bl[NT * 4 + 4 * t + lq] * res[t][r];
        const unsigned off = (cb != kOOB && coff[t] != kOOB) ? cb + coff[t] : kOOB;
        if constexpr (VECC) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rc, (int)off, 0, 0);
        } else {
          const int n = n0 + 16 * t + 4 * lq;
          // (the element goes through a named scalar: __builtin_bit_cast of the vector-element
          // lvalue v[e] itself compiled to element 0 for every e — all four stores got v.x)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float ve = v[e];
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, ve), rc,
                                                  (int)(n + e < g.N ? off + 4u * e : kOOB), 0, 0);
          }
        }
      }
    }
  };

  if (items <= 0) return;
  f32x4 a0[kRT][kKC], a1[kRT][kKC];
  load(0, a0);
  for (int i = 0; i < items; i += 2) {
    if constexpr (HASR) load_res(i, res);
    if (i + 1 < items) load(i + 1, a1);
    compute(i, a0);
    if (i + 1 >= items) break;
    if constexpr (HASR) load_res(i + 1, res);
    if (i + 2 < items) load(i + 2, a0);
    compute(i + 1, a1);
  }
}

static inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
static inline bool m4(long long v) { return (v & 3) == 0; }

// resident blocks per CU for this variant at this LDS size (hipOccupancy..., cached per variant and
// LDS KiB) times the CU count: the grid is one full round of them, each block walking its row
// tiles (r03 sweep, tools/micro/rows_bench.cpp: a fixed 1024-block grid was 10-45% slower on the
// shapes whose LDS or VGPRs allow one or two blocks per CU — the second partial round ran alone)
static int g_cus = 0;
template <int NT, bool HASR, bool VECC>
int slots(size_t lds) {
  static int cache[161] = {};
  const int kb = (int)((lds + 1023) / 1024);
  if (kb > 160) return 0;
  if (!cache[kb]) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(&tgemm_rows_kernel<NT, HASR, VECC>),
                                                     kThreads, lds) != hipSuccess || n < 1)
      n = 1;
    cache[kb] = n;
  }
  if (!g_cus) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || cus < 1)
      cus = 256;
    g_cus = cus;
  }
  return cache[kb] * g_cus;
}

template <int NT, bool HASR, bool VECC>
hipError_t launch_nt(RowsArgs a, int nz, size_t lds, hipStream_t s) {
  static size_t attr[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (lds > attr[dev]) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&tgemm_rows_kernel<NT, HASR, VECC>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr[dev] = lds;
  }
  const long long units = (long long)a.ncb * nz;
  long long gx = (slots<NT, HASR, VECC>(lds) + units - 1) / units;
  if (gx > a.row_tiles) gx = a.row_tiles;
  if (gx < 1) gx = 1;
  a.gx = (int)gx;
  const dim3 grid((unsigned)((a.ncb * gx + 7) / 8 * 8), 1, (unsigned)nz);
  hipLaunchKernelGGL((tgemm_rows_kernel<NT, HASR, VECC>), grid, dim3(kThreads), lds, s, a);
  return hipGetLastError();
}

template <int NT>
hipError_t launch_nt(const RowsArgs& a, bool hasr, bool vecc, int nz, size_t lds, hipStream_t s) {
  if constexpr (NT <= 4) {  // residual variants only up to NT = 4 (wider ones spill)
    if (hasr) return vecc ? launch_nt<NT, true, true>(a, nz, lds, s) : launch_nt<NT, true, false>(a, nz, lds, s);
  } else {
    if (hasr) return hipErrorInvalidValue;
  }
  return vecc ? launch_nt<NT, false, true>(a, nz, lds, s) : launch_nt<NT, false, false>(a, nz, lds, s);
}

}  // namespace

bool tgemm_rows_eligible(const TGemm& g) {
  if (g.amode != 0 || g.bmode != 0 || g.alpha != 1.f || g.sak != 1) return false;
  if (g.M <= 0 || g.N <= 0 || g.K <= 0) return false;
  if (!al16(g.A) || !m4(g.sam) || !m4(g.bA1) || !m4(g.bA2)) return false;
  if (g.scn != 1) return false;
  if (g.R && (g.srn != 1 || !al16(g.R) || !m4(g.srm) || !m4(g.bR1) || !m4(g.bR2) || g.N % 4)) return false;
  if ((long long)g.M * g.sam * 4 >= (1LL << 31) - 64 || (long long)g.M * g.scm * 4 >= (1LL << 31) - 64 ||
      (g.R && (long long)g.M * g.srm * 4 >= (1LL << 31) - 64))
    return false;
  const int kp = (g.K + 31) / 32;
  if (kp > 48) return false;  // NT = 1 keeps at most 144 KiB of split records
  return true;
}

hipError_t launch_tgemm_rows(const TGemm& g, hipStream_t s) {
  if (!tgemm_rows_eligible(g)) return hipErrorInvalidValue;
  RowsArgs a;
  a.g = g;
  a.kg = (g.K + 15) / 16;
  a.kp = (a.kg + 1) / 2;
  a.nchunk = (a.kg + kKC - 1) / kKC;
  a.row_tiles = (g.M + kTileRows - 1) / kTileRows;
  a.klast = g.K - 16 * (a.kg - 1);
  // float4 stores: aligned rows, and whole quads (N % 4 == 0, or a private row pad to write into)
  const bool vecc = al16(g.C) && m4(g.scm) && m4(g.bC1) && m4(g.bC2) &&
                    (g.N % 4 == 0 || (g.c_pad_ok && g.scm >= (g.N + 3) / 4 * 4));
  // output tiles per block: one column block when the N tiles fit (A read once), else the width
  // with the least padding; LDS for the split records <= KDLAE_ROWS_LDS_KB KiB (3 NT kp KiB)
  const int ntiles = (g.N + 15) / 16;
  // (residual variants: NT <= 4, the residual registers of wider tiles spill)
  static const int nts[] = {8, 6, 4, 3, 2, 1};
constexpr auto KDLAE_ROWS_LDS_KB = 144;  // split-record LDS budget per block (KiB); r05 A/B: 96 116.5, 120 116.6, 144 119.6, 156 119.7 img/s
constexpr auto KDLAE_ROWS_NTMAX = 8;
  const int ntmax = g.R ? 4 : KDLAE_ROWS_NTMAX;
  int NT = 1;
  if (ntiles <= ntmax) {
    for (int c : nts)
      if (c <= ntmax && c >= ntiles && 3 * c * a.kp <= KDLAE_ROWS_LDS_KB) NT = c;
  }
  if (NT < ntiles) {
    int best = -1, best_pad = 1 << 30;
    for (int c : nts) {
      if (c > ntmax || (3 * c * a.kp > KDLAE_ROWS_LDS_KB && c > 1)) continue;
      const int pad = (ntiles + c - 1) / c * c;
      if (pad < best_pad) best = c, best_pad = pad;
    }
    NT = best;
  }
  const int ncb = (ntiles + NT - 1) / NT;
  const int nz = g.nz1 * g.nz2;
  const size_t lds = (size_t)NT * a.kp * 3072 + (size_t)NT * 128;
  a.ncb = ncb;
  a.gx = 1;
#define NTCASE(n)                                                            \
  case n:                                                                    \
    return launch_nt<n>(a, g.R != nullptr, vecc, nz, lds, s);
  switch (NT) {
    NTCASE(1)
    NTCASE(2)
    NTCASE(3)
    NTCASE(4)
    NTCASE(6)
    NTCASE(8)
    default:
      return hipErrorInvalidValue;
  }
#undef NTCASE
}

}  // namespace train
}  // namespace kdlae
