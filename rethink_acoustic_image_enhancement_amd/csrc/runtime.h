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

namespace kdlae {

extern thread_local std::string g_err;
int fail(int code, const std::string& msg);

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
  int ntiles = 0, kgroups = 0, N = 0, K = 0, ksize = 1, cg_per_tap = 0, kt = 1;
  int out_mode = 0;  // store map the variant must support (0 plain, 1 unshuffle, 2 shuffle)
  int NT = 0, KG = 0, group_tiles = 0, WPE = 2;
  int n_true = 0, k_true = 0;  // un-padded sizes (FLOP accounting)
};
struct SmallW {
  size_t w = kNone, bias = kNone;
  int Cout = 0, Cin = 0;
};

void choose_variant(Gemm& g, bool prefer_single_k = false);

struct Arena {
  std::vector<float> h;
  size_t add(const std::vector<float>& v) {
    size_t off = (h.size() + 63) / 64 * 64;
    h.resize(off + v.size());
    std::copy(v.begin(), v.end(), h.begin() + off);
    return off;
  }
};

// fragment-order pack: Wf(n, k) over [ntiles*16] x [kgroups*16]
template <class F>
std::vector<float> pack_fragments(int ntiles, int kgroups, F Wf) {
  std::vector<float> v((size_t)ntiles * kgroups * 256, 0.f);
  for (int t = 0; t < ntiles; ++t)
    for (int g = 0; g < kgroups; ++g)
      for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 4; ++e) {
          const int n = 16 * t + (l & 15), k = 16 * g + 4 * (l >> 4) + e;
          v[(((size_t)t * kgroups + g) * 64 + l) * 4 + e] = Wf(n, k);
        }
  return v;
}

// expected state_dict keys + host copies staged through *_set_param (strict, like load_state_dict)
struct ParamStore {
  std::vector<std::pair<std::string, int64_t>> keys;
  std::unordered_map<std::string, int> index;
  std::unordered_map<std::string, std::vector<float>> staged;
  void add(const std::string& k, int64_t n) {
    index[k] = (int)keys.size();
    keys.emplace_back(k, n);
  }
  int set(const char* name, const float* data, int64_t numel);
  int info(int i, const char** name, int64_t* numel) const;
  int check_complete() const;
  const std::vector<float>* get(const std::string& k, int* err) const;
};

// device weight arena owned by a handle
struct DeviceWeights {
  float* dev = nullptr;
  size_t n = 0;
  int upload(Arena& a, hipStream_t s);
  void release();
  const float* P(size_t off) const { return off == kNone ? nullptr : dev + off; }
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
};
int run_gemm(const GemmCall& c, hipStream_t s);
// Compute units of the current device (256 on MI355X) and the tail-aware GEMM grid split.
int device_cu_count();
int gemm_tiles_per_block(int total_tiles, int gy, bool resident, int wpe);

}  // namespace kdlae
