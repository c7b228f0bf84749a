// Device execution of a handle's pack program (runtime.h PEx / PDot / PDer): packs the live fp32
// parameters (flat, state_dict key order) into the MFMA fragment-order arena the forward kernels
// read.  Three launches on the caller's stream, no host synchronisation:
//   derive  BatchNorm scale / shift values (ASDQE), written after the parameters,
//   gather  one packed float per thread: src[a] (x src[b], the LayerNorm weight folded into W),
//   dot     folded biases: conv bias + W . (WithBias LayerNorm bias), accumulated in double.
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

}  // namespace

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
  for (void* p : {(void*)dev, (void*)ex, (void*)dots, (void*)der, (void*)ext, (void*)src})
    if (p) (void)hipFree(p);
  dev = nullptr;
  ex = nullptr;
  dots = nullptr;
  der = nullptr;
  ext = nullptr;
  src = nullptr;
  n = 0;
  n_dots = n_der = 0;
}

}  // namespace kdlae
