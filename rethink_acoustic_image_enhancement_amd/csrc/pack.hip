// Device execution of a handle's pack program (runtime.h PEx / PDot / PDer): packs the live fp32
// parameters (flat, state_dict key order) into the MFMA fragment-order arena the forward kernels
// read.  Three launches on the caller's stream, no host synchronisation:
//   derive  BatchNorm scale / shift values (ASDQE), written after the parameters,
//   gather  one packed float per thread: src[a] (x src[b], the LayerNorm weight folded into W),
//   dot     folded biases: conv bias + W . (WithBias LayerNorm bias), accumulated in double,
//   split   the GEMM weight blocks again in split fragment order (mfma3.h) into the split arena.
// HBM-bound: per packed float 8 B of program + the gathered source floats + 4 B written.
#include "runtime.h"

namespace kdlae {

namespace {

__device__ __forceinline__ float fetch(const float* __restrict__ src, int64_t nsrc, const float* __restrict__ ext,
                                       int32_t i) {
  return i < nsrc ? src[i] : ext[i - nsrc];
}

__global__ __launch_bounds__(256) void pack_derive_kernel(const PDer* __restrict__ der, int n, int kind,
                                                          const float* __restrict__ src, int64_t nsrc,
                                                          float* __restrict__ ext) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const PDer d = der[j];
  if (d.kind != kind) return;
  if (kind == 0) {
    ext[j] = fetch(src, nsrc, ext, d.a) / sqrtf(fetch(src, nsrc, ext, d.b) + 1e-5f);
  } else {
    ext[j] = (fetch(src, nsrc, ext, d.a) - fetch(src, nsrc, ext, d.b)) * fetch(src, nsrc, ext, d.c) +
             fetch(src, nsrc, ext, d.d);
  }
}

__global__ __launch_bounds__(256) void pack_gather_kernel(const PEx* __restrict__ ex, int64_t n,
                                                          const float* __restrict__ src, int64_t nsrc,
                                                          const float* __restrict__ ext, float* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const PEx e = ex[i];
    float v = 0.f;
    if (e.a >= 0) {
      v = fetch(src, nsrc, ext, e.a);
      if (e.b >= 0) v *= fetch(src, nsrc, ext, e.b);
    }
    out[i] = v;
  }
}

__global__ __launch_bounds__(256) void pack_dot_kernel(const PDot* __restrict__ dots, int n,
                                                       const float* __restrict__ src, int64_t nsrc,
                                                       const float* __restrict__ ext, float* __restrict__ out) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const PDot d = dots[j];
  double acc = d.base >= 0 ? (double)fetch(src, nsrc, ext, d.base) : 0.0;
  for (int k = 0; k < d.K; ++k)
    acc += (double)fetch(src, nsrc, ext, d.w + k) * (double)fetch(src, nsrc, ext, d.v + k);
  out[d.dst] = (float)acc;
}

// one work item = (split record, lane): the lane's float4 of k-groups 2G and 2G + 1 -> 3 x 16 B
__device__ __forceinline__ void split_record(const float* __restrict__ src, float* __restrict__ dst, int kgroups,
                                             long long rec, int lane) {
  const int kg2 = (kgroups + 1) / 2;
  const long long t = rec / kg2;
  const int G = (int)(rec - t * kg2);
  typedef float f4 __attribute__((ext_vector_type(4)));
  const f4* s4 = reinterpret_cast<const f4*>(src) + (t * kgroups + 2 * G) * 64 + lane;
  const f4 lo = s4[0];
  const f4 hi = 2 * G + 1 < kgroups ? s4[64] : f4{0.f, 0.f, 0.f, 0.f};
  const F3 w = split3(lo, hi);
  f4* d4 = reinterpret_cast<f4*>(dst) + rec * kRec3 + lane;
  d4[0] = __builtin_bit_cast(f4, w.h);
  d4[64] = __builtin_bit_cast(f4, w.m);
  d4[128] = __builtin_bit_cast(f4, w.l);
}

__global__ __launch_bounds__(256) void pack_split_kernel(const PSplit* __restrict__ d, int nd, int64_t items,
                                                         const float* __restrict__ arena, float* __restrict__ dev3) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < items; i += stride) {
    int lo = 0, hi = nd - 1;  // the last descriptor with first <= i
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (d[mid].first <= i) lo = mid;
      else hi = mid - 1;
    }
    const PSplit ds = d[lo];
    const int64_t r = i - ds.first;
    split_record(arena + ds.src, dev3 + ds.dst, ds.kgroups, r >> 6, (int)(r & 63));
  }
}

__global__ __launch_bounds__(256) void split3_kernel(const float* __restrict__ src, float* __restrict__ dst, int kgroups,
                                                     long long recs, long long src_img, long long dst_img) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= recs * 64) return;
  const int img = blockIdx.y;
  split_record(src + img * src_img, dst + img * dst_img, kgroups, i >> 6, (int)(i & 63));
}

}  // namespace

hipError_t launch_split3(const float* src, float* dst, int ntiles, int kgroups, int nimg, long long src_img_stride,
                         long long dst_img_stride, hipStream_t s) {
  const long long recs = (long long)ntiles * ((kgroups + 1) / 2);
  hipLaunchKernelGGL(split3_kernel, dim3((unsigned)((recs * 64 + 255) / 256), (unsigned)nimg), dim3(256), 0, s, src, dst,
                     kgroups, recs, src_img_stride, dst_img_stride);
  return hipGetLastError();
}

int DeviceWeights::upload_program(const PackProgram& p) {
  release();
  HIPCHK(hipGetDevice(&device));
  n = std::max<size_t>(p.ex.size(), 64);
  nsrc = p.nsrc;
  n_dots = (int)p.dots.size();
  n_der = (int)p.der.size();
  std::vector<PEx> ex(p.ex);
  ex.resize(n);
  HIPCHK(hipMalloc(&dev, n * sizeof(float)));
  HIPCHK(hipMalloc(&this->ex, n * sizeof(PEx)));
  HIPCHK(hipMemcpy(this->ex, ex.data(), n * sizeof(PEx), hipMemcpyHostToDevice));
  if (n_dots) {
    HIPCHK(hipMalloc(&dots, n_dots * sizeof(PDot)));
    HIPCHK(hipMemcpy(dots, p.dots.data(), n_dots * sizeof(PDot), hipMemcpyHostToDevice));
  }
  n_splits = (int)p.splits.size();
  n3 = (size_t)std::max<int64_t>(p.n3, 64);
  split_items = p.splits.empty() ? 0 : p.splits.back().first + (int64_t)p.splits.back().ntiles *
                                                                    ((p.splits.back().kgroups + 1) / 2) * 64;
  HIPCHK(hipMalloc(&dev3, n3 * sizeof(float)));
  HIPCHK(hipMemset(dev3, 0, n3 * sizeof(float)));
  if (n_splits) {
    HIPCHK(hipMalloc(&splits, n_splits * sizeof(PSplit)));
    HIPCHK(hipMemcpy(splits, p.splits.data(), n_splits * sizeof(PSplit), hipMemcpyHostToDevice));
  }
  if (n_der) {
    HIPCHK(hipMalloc(&der, n_der * sizeof(PDer)));
    HIPCHK(hipMemcpy(der, p.der.data(), n_der * sizeof(PDer), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&ext, n_der * sizeof(float)));
  }
  return KDLAE_OK;
}

int DeviceWeights::run(const float* params, hipStream_t s) const {
  if (!dev || !ex) return fail(KDLAE_ESTATE, "pack program not built");
  if (!params) return fail(KDLAE_ESTATE, "null parameter buffer");
  if (n_der) {
    const int g = (n_der + 255) / 256;
    for (int kind = 0; kind < 2; ++kind)
      hipLaunchKernelGGL(pack_derive_kernel, dim3(g), dim3(256), 0, s, der, n_der, kind, params, nsrc, ext);
  }
  const int64_t blocks = std::min<int64_t>((int64_t)(n + 255) / 256, 4096);
  hipLaunchKernelGGL(pack_gather_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ex, (int64_t)n, params, nsrc,
                     (const float*)ext, dev);
  if (n_dots)
    hipLaunchKernelGGL(pack_dot_kernel, dim3((n_dots + 255) / 256), dim3(256), 0, s, dots, n_dots, params, nsrc,
                       (const float*)ext, dev);
  if (n_splits)
    hipLaunchKernelGGL(pack_split_kernel, dim3((unsigned)std::min<int64_t>((split_items + 255) / 256, 4096)), dim3(256),
                       0, s, splits, n_splits, split_items, (const float*)dev, dev3);
  HIPCHK(hipGetLastError());
  return KDLAE_OK;
}

int DeviceWeights::run_host(const std::vector<float>& params, hipStream_t s) {
  if ((int64_t)params.size() != nsrc) return fail(KDLAE_ESTATE, "flat parameter count mismatch");
  if (!src) HIPCHK(hipMalloc(&src, std::max<int64_t>(nsrc, 1) * sizeof(float)));
  HIPCHK(hipMemcpyAsync(src, params.data(), nsrc * sizeof(float), hipMemcpyHostToDevice, s));
  int rc = run(src, s);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(s));  // the host vector may go away after this call
  return KDLAE_OK;
}

void DeviceWeights::release() {
  for (void* p : {(void*)dev, (void*)ex, (void*)dots, (void*)der, (void*)ext, (void*)src, (void*)dev3, (void*)splits})
    if (p) (void)hipFree(p);
  dev = nullptr;
  dev3 = nullptr;
  splits = nullptr;
  n3 = 0;
  n_splits = 0;
  split_items = 0;
  ex = nullptr;
  dots = nullptr;
  der = nullptr;
  ext = nullptr;
  src = nullptr;
  n = 0;
  n_dots = n_der = 0;
}

}  // namespace kdlae
