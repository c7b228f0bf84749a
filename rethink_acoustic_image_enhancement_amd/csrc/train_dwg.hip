// Fused depthwise-3x3 kernels of the training step (gfx950): the GDFN middle
// (KDLAE_model.py:101-105: x1, x2 = dwconv(project_in(x)).chunk(2); gelu(x1) * x2) and the MDTA qkv
// dwconv (:127), forward and backward, each in one pass over HBM.
//
//   dwgate_fwd : yd = dw(y) (+ bias) for both halves, g = gelu_erf(yd1) * yd2 — y read once, g
//                written (and yd, the stored-yd backward's gate input, under KDLAE_DEBUG=train_keep_yd);
//                the separate dwconv + gate kernels read yd a second time.
//   dwgate_bwd_rc: the GDFN backward recomputing yd from y (below).
//   dw_bwd     : from dyd (GATE: dyd = gate_bwd(dg, yd) computed on the fly), dy = dw^T(dyd) (the
//                flipped-tap conv) and the weight / bias gradient partials sum dyd * y_in(shifted),
//                sum dyd — dyd is never written; the unfused chain wrote it and read it twice.
//
// Layout: NHWC views, channels contiguous; the GDFN's y / yd hold x1 at [0, hid), x2 at
// [hid, 2 hid) (hid odd for the released widths, so the halves are not float4-aligned: one channel
// per lane, 64 consecutive channels = 256 B per load).  A block is 4 waves = 4 column groups of 4
// columns (16 columns) x TY rows of one image x 64 channels; a thread walks its 4 columns down the
// rows with a 3-row x 6-column register window per tensor (each input row is loaded once per walk;
// the 2 halo columns are the neighbouring wave's, L1 hits).  Accumulation order per output: bias,
// then taps row-major (as dw_tile_fwd_kernel), every multiply-add an explicit fma (so the recomputing
// backward reproduces the forward's yd and the stored-yd backward's arithmetic exactly).  Weight gradient partials: the block's 4 waves in
// fixed order -> part[spatial block][c * 9 + t] and part[..][9 C + c] (C = all channels), summed
// over spatial blocks in fixed order by part_reduce: deterministic.
#include <math.h>

#include <algorithm>

#include "train_kernels.h"

namespace kdlae {
namespace train {

namespace {

constexpr auto KDLAE_DWG_U = 4;
constexpr auto KDLAE_DWG_TY = 16;
constexpr auto KDLAE_DWG_PF = 1;
constexpr int kU = KDLAE_DWG_U;  // columns per thread
// rows are loaded one row ahead of their use, so the next row's loads overlap this row's arithmetic
// (r03 A/B at 6 x 128^2: qkv dwconv backward 3.32 -> 2.41 ms per step, GDFN forward 3.95 -> 3.74,
// the VALU-bound GDFN backward 5.06 -> 4.98; 99.5 -> 101.2 img/s)
constexpr bool kPF = KDLAE_DWG_PF != 0;
constexpr int kTX = 4 * kU;   // columns per block
// rows per block: 16, or 8 / 4 on the small levels so the grid still has >= 256 spatial blocks (the
// 16^2 latent: 6 blocks per channel group at 16 rows, 0.7-1.0 TB/s)
int rows_per_block(int Bn, int H, int W) {
  const int tx = (W + kTX - 1) / kTX;
  int ty = KDLAE_DWG_TY;
  while (ty > 4 && (long long)Bn * tx * ((H + ty - 1) / ty) < 256) ty >>= 1;
  return ty;
}

// erf(|x| / sqrt 2) by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, as the inference GDFN's
// gelu_erf_g), returning exp(-x^2 / 2) as well: the GELU derivative's Gaussian pdf is the same
// exponential, so the backward pays one __expf per element instead of libm's erff + expf (r03 PMC:
// the fused gate backward was VALU-bound, SQ_ACTIVE_INST_VALU ~1.3 of wave cycles).
__device__ __forceinline__ float erf_half(float x, float& ex) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float poly = fmaf(1.061405429f, t, -1.453152027f);
  poly = fmaf(poly, t, 1.421413741f);
  poly = fmaf(poly, t, -0.284496736f);
  poly = fmaf(poly, t, 0.254829592f);
  poly *= t;
  ex = __expf(-z * z);
  return copysignf(fmaf(-poly, ex, 1.0f), x);
}

// forward GELU with libm's erff (measured 5% faster here than the A&S form, which pays off only
// where its exponential is shared)
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

struct Geo {
  int b, x0, y0, y1, c;
  long long img0;
  bool live;
};

__device__ __forceinline__ Geo geo(int C, int H, int W, int tiles_x, int ty) {
  Geo o;
  const int t = blockIdx.x;
  o.b = blockIdx.z;
  o.x0 = (t % tiles_x) * kTX + (threadIdx.x >> 6) * kU;
  o.y0 = (t / tiles_x) * ty;
  o.y1 = min(H, o.y0 + ty);
  o.c = blockIdx.y * 64 + (threadIdx.x & 63);
  o.live = o.c < C;
  o.img0 = (long long)o.b * H * W;
  return o;
}

// Image-relative buffer accesses: a descriptor per (tensor, image) (uniform), a row offset per row
// (uniform) plus a loop-invariant column offset per lane, instead of a 64-bit address per element
// (the flat form spent ~4 VALU address instructions per load).  Out-of-image rows / columns and
// channels past C take kOOBU, one "out of range" unit: a row and a column unit together stay below
// 2^32 and past every image's byte count (< kOOBU, checked by the launchers), so the hardware
// returns the conv's zero padding on loads and drops stores.
constexpr unsigned kOOBU = 0x40000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t img_rsrc(const float* p, int ld, const Geo& o, int H, int W) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p + o.img0 * ld), 0, H * W * ld * 4, 0x00020000);
}
__device__ __forceinline__ unsigned row_off(int yy, int H, int W, int ld) {
  return (yy >= 0 && yy < H) ? (unsigned)(yy * W) * (unsigned)ld * 4u : kOOBU;
}
__device__ __forceinline__ unsigned col_off(const Geo& o, int xx, int W, int ld, int off) {
  return (o.live && xx >= 0 && xx < W) ? ((unsigned)xx * (unsigned)ld + (unsigned)off) * 4u : kOOBU;
}
__device__ __forceinline__ float ld_img(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
__device__ __forceinline__ void st_img(__amdgpu_buffer_rsrc_t r, unsigned off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)off, 0, 0);
}
bool img_bytes_ok(int H, int W, int ld) { return (long long)H * W * ld * 4 < (long long)kOOBU; }

// row yy, columns x0 - 1 .. x0 + kU of channel off (zero outside the image / past the channels)
__device__ __forceinline__ void load_row(const float* __restrict__ p, int ld, const Geo& o, int H, int W, int yy,
                                         int off, float (&r)[kU + 2]) {
  const __amdgpu_buffer_rsrc_t rs = img_rsrc(p, ld, o, H, W);
  const unsigned ro = row_off(yy, H, W, ld);
#pragma unroll
  for (int j = 0; j < kU + 2; ++j) r[j] = ld_img(rs, col_off(o, o.x0 - 1 + j, W, ld, off) + ro);
}

__global__ __launch_bounds__(256) void dwgate_fwd_kernel(const float* __restrict__ y, int ldi,
                                                         const float* __restrict__ w, const float* __restrict__ bias,
                                                         int hid, int H, int W, int tiles_x, int ty,
                                                         float* __restrict__ yd, int ldyd, float* __restrict__ g,
                                                         int ldg) {
  const Geo o = geo(hid, H, W, tiles_x, ty);
  const int c = o.c;
  float w1[9], w2[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    w1[t] = o.live ? w[c * 9 + t] : 0.f;
    w2[t] = o.live ? w[(hid + c) * 9 + t] : 0.f;
  }
  const float b1 = (o.live && bias) ? bias[c] : 0.f, b2 = (o.live && bias) ? bias[hid + c] : 0.f;
  const __amdgpu_buffer_rsrc_t rg = img_rsrc(g, ldg, o, H, W);
  [[maybe_unused]] const __amdgpu_buffer_rsrc_t ryd = img_rsrc(yd ? yd : g, yd ? ldyd : ldg, o, H, W);
  float a[3][kU + 2], v[3][kU + 2];  // rows y-1, y, y+1 of halves 1 and 2
  load_row(y, ldi, o, H, W, o.y0 - 1, c, a[0]);
  load_row(y, ldi, o, H, W, o.y0, c, a[1]);
  load_row(y, ldi, o, H, W, o.y0 - 1, hid + c, v[0]);
  load_row(y, ldi, o, H, W, o.y0, hid + c, v[1]);
  [[maybe_unused]] float an[kU + 2], vn[kU + 2];  // kPF: the row after next, in flight during this row
  if constexpr (kPF) {
    load_row(y, ldi, o, H, W, o.y0 + 1, c, an);
    load_row(y, ldi, o, H, W, o.y0 + 1, hid + c, vn);
  }
  for (int yy = o.y0; yy < o.y1; ++yy) {
    if constexpr (kPF) {
#pragma unroll
      for (int j = 0; j < kU + 2; ++j) {
        a[2][j] = an[j];
        v[2][j] = vn[j];
      }
      load_row(y, ldi, o, H, W, yy + 2, c, an);
      load_row(y, ldi, o, H, W, yy + 2, hid + c, vn);
    } else {
      load_row(y, ldi, o, H, W, yy + 1, c, a[2]);
      load_row(y, ldi, o, H, W, yy + 1, hid + c, v[2]);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      float s1 = b1, s2 = b2;
#pragma unroll
      for (int ty = 0; ty < 3; ++ty)
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) {
          s1 = fmaf(w1[ty * 3 + tx], a[ty][u + tx], s1);
          s2 = fmaf(w2[ty * 3 + tx], v[ty][u + tx], s2);
        }
      const int xx = o.x0 + u;
      if (yd) {  // (null: the backward recomputes yd, dwgate_bwd_rc_kernel)
        const unsigned ro = row_off(yy, H, W, ldyd);
        st_img(ryd, col_off(o, xx, W, ldyd, c) + ro, s1);
        st_img(ryd, col_off(o, xx, W, ldyd, hid + c) + ro, s2);
      }
      st_img(rg, col_off(o, xx, W, ldg, c) + row_off(yy, H, W, ldg), gelu_erf(s1) * s2);
    }
#pragma unroll
    for (int j = 0; j < kU + 2; ++j) {
      a[0][j] = a[1][j];
      a[1][j] = a[2][j];
      v[0][j] = v[1][j];
      v[1][j] = v[2][j];
    }
  }
}

// GATE: two halves, dyd from (dg, yd); else one tensor of C = `hid` channels, dyd read as given.
// GATE carries the two halves of a channel as one float2 (x: first half, y: second half) so the
// transposed conv and the weight-gradient FMAs issue as packed v_pk_fma_f32 (two per instruction;
// the fused GDFN backward is VALU-bound).
typedef float f2 __attribute__((ext_vector_type(2)));
template <bool GATE> struct DwType { using T = float; };
template <> struct DwType<true> { using T = f2; };

template <bool GATE>
__global__ __launch_bounds__(256) void dw_bwd_kernel(const float* __restrict__ dg, int ldg,
                                                     const float* __restrict__ yd, int ldyd,
                                                     const float* __restrict__ yin, int ldi,
                                                     const float* __restrict__ w, int hid, int H, int W, int tiles_x,
                                                     int ty, float* __restrict__ dy, int lddy,
                                                     float* __restrict__ part) {
  using T = typename DwType<GATE>::T;
  constexpr int NH = GATE ? 2 : 1;
  __shared__ float red[4][64][10 * NH];
  const Geo o = geo(hid, H, W, tiles_x, ty);
  const int c = o.c;
  auto comp = [](const T& v, int h) -> float {
    if constexpr (GATE) return h ? v.y : v.x;
    else return v;
  };
  auto pack = [](float a, float b) -> T {
    if constexpr (GATE) return f2{a, b};
    else return a;
  };
  const __amdgpu_buffer_rsrc_t rdy = img_rsrc(dy, lddy, o, H, W);
  T wf[9];  // flipped taps (the transposed conv)
#pragma unroll
  for (int t = 0; t < 9; ++t)
    wf[t] = pack(o.live ? w[c * 9 + 8 - t] : 0.f, (GATE && o.live) ? w[(hid + c) * 9 + 8 - t] : 0.f);
  T acc[10];
#pragma unroll
  for (int t = 0; t < 10; ++t) acc[t] = pack(0.f, 0.f);
  T d[3][kU + 2], x[3][kU + 2];
  // raw inputs of one row (GATE: dg, yd1, yd2; else dyd in r1) and the layer input rows
  float rg[GATE ? kU + 2 : 1], r1[kU + 2], r2[GATE ? kU + 2 : 1], rx[NH][kU + 2];
  auto load_raw = [&](int yy) {
    if constexpr (GATE) {
      load_row(dg, ldg, o, H, W, yy, c, rg);
      load_row(yd, ldyd, o, H, W, yy, hid + c, r2);
    }
    load_row(yd, ldyd, o, H, W, yy, c, r1);
#pragma unroll
    for (int h = 0; h < NH; ++h) load_row(yin, ldi, o, H, W, yy, h * hid + c, rx[h]);
  };
  // dyd of the raw row for both halves: gate backward of (dg, yd1, yd2), or the given gradient
  auto row_d = [&](T (&dd)[kU + 2]) {
#pragma unroll
    for (int j = 0; j < kU + 2; ++j) {
      if constexpr (GATE) {
        float ex;
        const float cdf = 0.5f * (1.f + erf_half(r1[j], ex));
        const float pdf = 0.39894228040143268f * ex;
        dd[j] = pack((rg[j] * r2[j]) * fmaf(r1[j], pdf, cdf), (rg[j] * r1[j]) * cdf);
      } else {
        dd[j] = r1[j];
      }
    }
  };
  auto take_x = [&](int slot) {
#pragma unroll
    for (int j = 0; j < kU + 2; ++j) x[slot][j] = pack(rx[0][j], rx[NH - 1][j]);
  };
  load_raw(o.y0 - 1);
  row_d(d[0]);
  take_x(0);
  load_raw(o.y0);
  row_d(d[1]);
  take_x(1);
  if constexpr (kPF) load_raw(o.y0 + 1);  // kPF: row yy + 1's loads are in flight during row yy - 1
  for (int yy = o.y0; yy < o.y1; ++yy) {
    if constexpr (!kPF) load_raw(yy + 1);
    row_d(d[2]);
    take_x(2);
    if constexpr (kPF) load_raw(yy + 2);
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int xx = o.x0 + u;
      T s = pack(0.f, 0.f);
#pragma unroll
      for (int ty = 0; ty < 3; ++ty)
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) s = __builtin_elementwise_fma(wf[ty * 3 + tx], d[ty][u + tx], s);
      {
        const unsigned ro = row_off(yy, H, W, lddy);
#pragma unroll
        for (int h = 0; h < NH; ++h) st_img(rdy, col_off(o, xx, W, lddy, h * hid + c) + ro, comp(s, h));
      }
      // weight / bias gradient: centre dyd times the input at each tap (zero past the image)
      const T dc = d[1][u + 1];
#pragma unroll
      for (int ty = 0; ty < 3; ++ty)
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) acc[ty * 3 + tx] = __builtin_elementwise_fma(dc, x[ty][u + tx], acc[ty * 3 + tx]);
      acc[9] += dc;
    }
#pragma unroll
    for (int j = 0; j < kU + 2; ++j) {
      d[0][j] = d[1][j];
      d[1][j] = d[2][j];
      x[0][j] = x[1][j];
      x[1][j] = x[2][j];
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int t = 0; t < 10; ++t) red[wv][lane][h * 10 + t] = comp(acc[t], h);
  __syncthreads();
  if (wv != 0 || !o.live) return;
  const int Ctot = NH * hid;
  float* pr = part + ((long long)o.b * gridDim.x + blockIdx.x) * 10 * Ctot;
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int t = 0; t < 10; ++t) {
      const float s = ((red[0][lane][h * 10 + t] + red[1][lane][h * 10 + t]) + red[2][lane][h * 10 + t]) +
                      red[3][lane][h * 10 + t];
      const int ch = h * hid + c;
      if (t < 9) pr[ch * 9 + t] = s;
      else pr[9 * Ctot + ch] = s;
    }
}

// The GDFN backward without a stored yd: yd = dw(y) (+ bias) is recomputed from the layer input y,
// which the weight gradient reads anyway, so the forward writes only g (1.5 instead of 2.5 KiB per
// pixel at hid = 127) and the backward reads dg and y (2.5 instead of 3.5 KiB).  The recomputation
// is the forward's arithmetic (bias, then taps row-major, fused multiply-adds), so yd, and with it
// every gradient, has the same bits as the stored-yd kernel's.
// A thread walks its kU columns down the rows with a 4-row x (kU + 4)-column window of y (both
// halves packed as one float2) and a 3-row x (kU + 2)-column window of dyd: output row yy needs dyd
// rows yy - 1 .. yy + 1, dyd row r needs yd row r, and yd row r needs y rows r - 1 .. r + 1.
__global__ __launch_bounds__(256) void dwgate_bwd_rc_kernel(const float* __restrict__ dg, int ldg,
                                                            const float* __restrict__ yin, int ldi,
                                                            const float* __restrict__ w,
                                                            const float* __restrict__ bias, int hid, int H, int W,
                                                            int tiles_x, int ty, float* __restrict__ dy, int lddy,
                                                            float* __restrict__ part) {
  constexpr int NY = kU + 4, ND = kU + 2;
  __shared__ float red[4][64][20];
  const Geo o = geo(hid, H, W, tiles_x, ty);
  const int c = o.c;
  f2 wv[9];  // forward taps; the transposed conv reads them flipped
#pragma unroll
  for (int t = 0; t < 9; ++t) wv[t] = o.live ? f2{w[c * 9 + t], w[(hid + c) * 9 + t]} : f2{0.f, 0.f};
  const f2 bv = (o.live && bias) ? f2{bias[c], bias[hid + c]} : f2{0.f, 0.f};
  f2 acc[10];
#pragma unroll
  for (int t = 0; t < 10; ++t) acc[t] = f2{0.f, 0.f};
  // y row yy, columns x0 - 2 .. x0 + kU + 1 (zero outside the image / past the channels)
  const __amdgpu_buffer_rsrc_t ryin = img_rsrc(yin, ldi, o, H, W), rdy = img_rsrc(dy, lddy, o, H, W);
  auto load_y = [&](int yy, f2 (&r)[NY]) {
    const unsigned ro = row_off(yy, H, W, ldi);
#pragma unroll
    for (int j = 0; j < NY; ++j) {
      const int xx = o.x0 - 2 + j;
      r[j] = f2{ld_img(ryin, col_off(o, xx, W, ldi, c) + ro), ld_img(ryin, col_off(o, xx, W, ldi, hid + c) + ro)};
    }
  };
  // dyd row from dg (columns x0 - 1 .. x0 + kU) and the y rows r - 1, r, r + 1: yd as the forward
  // computed it, then the gate backward (dg = 0 outside the image, so dyd is the transposed conv's
  // zero padding there)
  auto row_d = [&](const float (&rg)[ND], const f2 (&ya)[NY], const f2 (&yb)[NY], const f2 (&yc)[NY], f2 (&dd)[ND]) {
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      f2 s = bv;
#pragma unroll
      for (int tx = 0; tx < 3; ++tx) s = __builtin_elementwise_fma(wv[tx], ya[j + tx], s);
#pragma unroll
      for (int tx = 0; tx < 3; ++tx) s = __builtin_elementwise_fma(wv[3 + tx], yb[j + tx], s);
#pragma unroll
      for (int tx = 0; tx < 3; ++tx) s = __builtin_elementwise_fma(wv[6 + tx], yc[j + tx], s);
      float ex;
      const float cdf = 0.5f * (1.f + erf_half(s.x, ex));
      const float pdf = 0.39894228040143268f * ex;
      dd[j] = f2{(rg[j] * s.y) * fmaf(s.x, pdf, cdf), (rg[j] * s.x) * cdf};
    }
  };
  f2 Y[4][NY], D[3][ND];
  f2 y4[NY];
  float rg[ND];
  load_y(o.y0 - 2, y4);
  load_y(o.y0 - 1, Y[0]);
  load_y(o.y0, Y[1]);
  load_y(o.y0 + 1, Y[2]);
  load_y(o.y0 + 2, Y[3]);
  load_row(dg, ldg, o, H, W, o.y0 - 1, c, rg);
  row_d(rg, y4, Y[0], Y[1], D[0]);
  load_row(dg, ldg, o, H, W, o.y0, c, rg);
  row_d(rg, Y[0], Y[1], Y[2], D[1]);
  load_row(dg, ldg, o, H, W, o.y0 + 1, c, rg);
  row_d(rg, Y[1], Y[2], Y[3], D[2]);
  // rows yy + 3 (y) and yy + 2 (dg) are in flight during row yy
  load_y(o.y0 + 3, y4);
  load_row(dg, ldg, o, H, W, o.y0 + 2, c, rg);
  for (int yy = o.y0; yy < o.y1; ++yy) {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int xx = o.x0 + u;
      f2 s = f2{0.f, 0.f};
#pragma unroll
      for (int ty2 = 0; ty2 < 3; ++ty2)
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) s = __builtin_elementwise_fma(wv[8 - (ty2 * 3 + tx)], D[ty2][u + tx], s);
      {
        const unsigned ro = row_off(yy, H, W, lddy);
        st_img(rdy, col_off(o, xx, W, lddy, c) + ro, s.x);
        st_img(rdy, col_off(o, xx, W, lddy, hid + c) + ro, s.y);
      }
      // weight / bias gradient: centre dyd times the input at each tap (y at column x0 + u + tx - 1)
      const f2 dc = D[1][u + 1];
#pragma unroll
      for (int ty2 = 0; ty2 < 3; ++ty2)
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) acc[ty2 * 3 + tx] = __builtin_elementwise_fma(dc, Y[ty2][u + tx + 1], acc[ty2 * 3 + tx]);
      acc[9] += dc;
    }
    if (yy + 1 >= o.y1) break;
#pragma unroll
    for (int j = 0; j < NY; ++j) {
      Y[0][j] = Y[1][j];
      Y[1][j] = Y[2][j];
      Y[2][j] = Y[3][j];
      Y[3][j] = y4[j];
    }
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      D[0][j] = D[1][j];
      D[1][j] = D[2][j];
    }
    row_d(rg, Y[1], Y[2], Y[3], D[2]);  // dyd row yy + 2
    load_y(yy + 4, y4);
    load_row(dg, ldg, o, H, W, yy + 3, c, rg);
  }
  const int lane = threadIdx.x & 63, wv_ = threadIdx.x >> 6;
#pragma unroll
  for (int t = 0; t < 10; ++t) {
    red[wv_][lane][t] = acc[t].x;
    red[wv_][lane][10 + t] = acc[t].y;
  }
  __syncthreads();
  if (wv_ != 0 || !o.live) return;
  const int Ctot = 2 * hid;
  float* pr = part + ((long long)o.b * gridDim.x + blockIdx.x) * 10 * Ctot;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int t = 0; t < 10; ++t) {
      const float s = ((red[0][lane][h * 10 + t] + red[1][lane][h * 10 + t]) + red[2][lane][h * 10 + t]) +
                      red[3][lane][h * 10 + t];
      const int ch = h * hid + c;
      if (t < 9) pr[ch * 9 + t] = s;
      else pr[9 * Ctot + ch] = s;
    }
}

}  // namespace

int dwg_blocks(int Bn, int H, int W) {
  const int ty = rows_per_block(Bn, H, W);
  return Bn * ((W + kTX - 1) / kTX) * ((H + ty - 1) / ty);
}

hipError_t launch_dwgate_fwd(const float* y, int ldi, const float* w, const float* b, int hid, int Bn, int H, int W,
                             float* yd, int ldyd, float* g, int ldg, hipStream_t s) {
  if (!img_bytes_ok(H, W, std::max(ldi, std::max(ldyd, ldg)))) return hipErrorInvalidValue;
  const int ty = rows_per_block(Bn, H, W), tx = (W + kTX - 1) / kTX, nty = (H + ty - 1) / ty;
  hipLaunchKernelGGL(dwgate_fwd_kernel, dim3(tx * nty, (hid + 63) / 64, Bn), dim3(256), 0, s, y, ldi, w, b, hid, H, W,
                     tx, ty, yd, ldyd, g, ldg);
  return hipGetLastError();
}

hipError_t launch_dwgate_bwd(const float* dg, int ldg, const float* yd, int ldyd, const float* yin, int ldi,
                             const float* w, int hid, int Bn, int H, int W, float* dy, int lddy, float* part,
                             hipStream_t s) {
  if (!img_bytes_ok(H, W, std::max(std::max(ldg, ldyd), std::max(ldi, lddy)))) return hipErrorInvalidValue;
  const int ty = rows_per_block(Bn, H, W), tx = (W + kTX - 1) / kTX, nty = (H + ty - 1) / ty;
  hipLaunchKernelGGL(dw_bwd_kernel<true>, dim3(tx * nty, (hid + 63) / 64, Bn), dim3(256), 0, s, dg, ldg, yd, ldyd,
                     yin, ldi, w, hid, H, W, tx, ty, dy, lddy, part);
  return hipGetLastError();
}

hipError_t launch_dwgate_bwd_rc(const float* dg, int ldg, const float* yin, int ldi, const float* w, const float* b,
                                int hid, int Bn, int H, int W, float* dy, int lddy, float* part, hipStream_t s) {
  if (!img_bytes_ok(H, W, std::max(ldg, std::max(ldi, lddy)))) return hipErrorInvalidValue;
  const int ty = rows_per_block(Bn, H, W), tx = (W + kTX - 1) / kTX, nty = (H + ty - 1) / ty;
  hipLaunchKernelGGL(dwgate_bwd_rc_kernel, dim3(tx * nty, (hid + 63) / 64, Bn), dim3(256), 0, s, dg, ldg, yin, ldi, w, b,
                     hid, H, W, tx, ty, dy, lddy, part);
  return hipGetLastError();
}

hipError_t launch_dw_bwd(const float* dyd, int ldd, const float* yin, int ldi, const float* w, int C, int Bn, int H,
                         int W, float* dy, int lddy, float* part, hipStream_t s) {
  if (!img_bytes_ok(H, W, std::max(ldd, std::max(ldi, lddy)))) return hipErrorInvalidValue;
  const int ty = rows_per_block(Bn, H, W), tx = (W + kTX - 1) / kTX, nty = (H + ty - 1) / ty;
  hipLaunchKernelGGL(dw_bwd_kernel<false>, dim3(tx * nty, (C + 63) / 64, Bn), dim3(256), 0, s, nullptr, 0, dyd, ldd,
                     yin, ldi, w, C, H, W, tx, ty, dy, lddy, part);
  return hipGetLastError();
}

}  // namespace train
}  // namespace kdlae
