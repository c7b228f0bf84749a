// Shared host runtime for the KDLAE-T / KDLAE-S / ASDQE handles: error state, packed-weight
// descriptors, GEMM tile-variant selection, the weight arena and a GEMM launcher over NHWC views.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/kdlae.h"
#include "kernels.h"
#include "mfma3.h"

namespace kdlae {

extern thread_local std::string g_err;
int fail(int code, const std::string& msg);
// Debug switches, read when a handle builds its layer plan: KDLAE_DEBUG is a comma-separated list
// of flag names (include/kdlae.h lists them).  They select between kernel schedules that give the
// same bits (the GPU tests compare them); nothing else in the library reads the environment.
bool debug_flag(const char* name);

#define HIPCHK(x)                                                                                  \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) return ::kdlae::fail(KDLAE_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

inline int ru16(int x) { return (x + 15) / 16 * 16; }
inline long long ceil_div(long long a, long long b) { return (a + b - 1) / b; }
constexpr size_t kNone = (size_t)-1;

// packed 1x1 / implicit-GEMM weights (offsets in floats into a device weight arena)
struct Gemm {
  size_t w = kNone, bias = kNone;
  size_t w3 = kNone;  // the same weights in split fragment order (mfma3.h), offset into the split arena
  size_t w3t = kNone;  // 3x3x3 convs (kt = 3): split records of tap pairs (conv_lds.hip), see kdlae_s.cpp
  int ntiles = 0, kgroups = 0, N = 0, K = 0, ksize = 1, cg_per_tap = 0, kt = 1;
  int out_mode = 0;  // store map the variant must support (0 plain, 1 unshuffle, 2 shuffle)
  int NT = 0, KG = 0, group_tiles = 0, WPE = 2;
  int n_true = 0, k_true = 0;  // un-padded sizes (FLOP accounting)
  bool has_res = false;         // launched with a residual epilogue (variant choice)
};
struct SmallW {
  size_t w = kNone, bias = kNone;
  int Cout = 0, Cin = 0;
};

void choose_variant(Gemm& g, bool prefer_single_k = false);

// Packed weights are not computed on the host.  Each packed float is recorded as a gather from the
// flat parameter vector (every state_dict entry in key order, fp32), and the device executes that
// "pack program" (pack.hip) whenever the caller hands it the live parameters — so the packed copy
// can never go stale, whatever wrote the parameters (load_state_dict, an optimizer, `.data` edits).
struct PEx {                  // arena[i] = a < 0 ? 0 : src[a] * (b < 0 ? 1 : src[b])
  int32_t a = -1, b = -1;
};
struct PDot {                 // arena[dst] = (base < 0 ? 0 : src[base]) + sum_k src[w + k] * src[v + k]
  int64_t dst = 0;
  int32_t base = -1, w = 0, v = 0, K = 0;
};
struct PDer {                 // derived source value src[nsrc + j], computed before the gathers
  int32_t kind = 0;           // 0: src[a] / sqrt(src[b] + 1e-5)     (BatchNorm scale)
  int32_t a = -1, b = -1, c = -1, d = -1;  // 1: (src[a] - src[b]) * src[c] + src[d]  (BatchNorm shift)
};
struct PSplit {               // split arena [dst, +split3_floats) = split3 of the f32 records at arena[src]
  int64_t src = 0, dst = 0, first = 0;  // first: index of the descriptor's first work item (record x lane)
  int32_t ntiles = 0, kgroups = 0;
};
struct PackProgram {
  std::vector<PEx> ex;        // one per arena float
  std::vector<PDot> dots;
  std::vector<PDer> der;
  std::vector<PSplit> splits;  // run after the gathers and dots
  int64_t n3 = 0;              // floats in the split arena
  int64_t nsrc = 0;           // floats in the flat parameter vector
  size_t add(const std::vector<PEx>& v) {
    size_t off = (ex.size() + 63) / 64 * 64;
    ex.resize(off + v.size());
    std::copy(v.begin(), v.end(), ex.begin() + off);
    return off;
  }
  size_t copy(int32_t base, size_t n) {  // plain copy of n source floats
    std::vector<PEx> v(n);
    for (size_t i = 0; i < n; ++i) v[i].a = base + (int32_t)i;
    return add(v);
  }
  // the split-fragment-order copy of the f32 fragment block at arena offset w (ntiles x kgroups records)
  size_t split(size_t w, int ntiles, int kgroups) {
    PSplit d;
    d.src = (int64_t)w;
    d.dst = n3;
    d.ntiles = ntiles;
    d.kgroups = kgroups;
    d.first = splits.empty() ? 0 : splits.back().first + (int64_t)splits.back().ntiles * ((splits.back().kgroups + 1) / 2) * 64;
    splits.push_back(d);
    n3 += (split3_floats(ntiles, kgroups) + 63) / 64 * 64;
    return (size_t)d.dst;
  }
  int32_t derive(const PDer& d) {
    der.push_back(d);
    return (int32_t)(nsrc + (int64_t)der.size() - 1);
  }
};

// fragment-order pack: Wf(n, k) over [ntiles*16] x [kgroups*16]
template <class F>
std::vector<PEx> pack_fragments(int ntiles, int kgroups, F Wf) {
  std::vector<PEx> v((size_t)ntiles * kgroups * 256);
  for (int t = 0; t < ntiles; ++t)
    for (int g = 0; g < kgroups; ++g)
      for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 4; ++e) {
          const int n = 16 * t + (l & 15), k = 16 * g + 4 * (l >> 4) + e;
          v[(((size_t)t * kgroups + g) * 64 + l) * 4 + e] = Wf(n, k);
        }
  return v;
}

// expected state_dict keys (flat offsets in key order) + host copies staged through *_set_param
struct ParamStore {
  std::vector<std::pair<std::string, int64_t>> keys;
  std::vector<int64_t> offset;
  int64_t total = 0;
  std::unordered_map<std::string, int> index;
  std::unordered_map<std::string, std::vector<float>> staged;
  void add(const std::string& k, int64_t n) {
    index[k] = (int)keys.size();
    keys.emplace_back(k, n);
    offset.push_back(total);
    total += n;
  }
  int set(const char* name, const float* data, int64_t numel);
  int info(int i, const char** name, int64_t* numel) const;
  int check_complete() const;
  int32_t base(const std::string& k, int* err) const;  // flat offset of a key (-1 + err if unknown)
  std::vector<float> flat() const;                       // staged entries in key order
};

// Device side of a handle's weights: the packed arena plus the pack program that fills it.
struct DeviceWeights {
  float* dev = nullptr;       // packed arena
  size_t n = 0;
  float* dev3 = nullptr;      // split arena (GEMM weights in split fragment order, mfma3.h)
  size_t n3 = 0;
  PSplit* splits = nullptr;
  int n_splits = 0;
  int64_t split_items = 0;
  PEx* ex = nullptr;
  PDot* dots = nullptr;
  PDer* der = nullptr;
  float* ext = nullptr;       // derived values
  float* src = nullptr;       // flat parameters staged from the host (set_param/commit path)
  int64_t nsrc = 0;
  int n_dots = 0, n_der = 0;
  int device = -1;
  int upload_program(const PackProgram& p);                 // allocates; synchronous, once per layout
  int run(const float* params, hipStream_t s) const;        // enqueues the pack on `s`
  int run_host(const std::vector<float>& params, hipStream_t s);  // host copy of the flat vector
  void release();
  const float* P(size_t off) const { return off == kNone ? nullptr : dev + off; }
  const float* P3(size_t off) const { return off == kNone ? nullptr : dev3 + off; }
};

// Restores the caller's current device when it goes out of scope.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

struct View {
  float* p;
  int ld;
};

// One GEMM launch over NHWC views; geometry (B, F, H, W) of the input grid.
struct GemmCall {
  const Gemm* g = nullptr;
  const float* W = nullptr;
  long long w_img_stride = 0;
  const float* bias = nullptr;
  View in{nullptr, 0}, out{nullptr, 0};
  int B = 1, F = 1, H = 1, Wd = 1;
  int out_mode = 0;
  const float* R = nullptr;
  int ldr = 0;
  int relu = 0;
  int ln = 0, ln_C = 0;
  float* stats_buf = nullptr;  // scratch [P][2] used when LN needs precomputed row stats
  // fused attention output (GemmParams::Wm): in = v, R = x, out1 = where x1 goes (x itself)
  const float* Wm = nullptr;
  long long wm_img_stride = 0;
  const float* bias_m = nullptr;
  View out1{nullptr, 0};
};
int run_gemm(const GemmCall& c, hipStream_t s);
// Compute units of the current device (256 on MI355X) and the tail-aware GEMM grid split.
int device_cu_count();  // of the current device
int gemm_tiles_per_block(int total_tiles, int gy, bool resident, int wpe);

}  // namespace kdlae
