// Shared host runtime (see runtime.h).
#include "runtime.h"

#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

namespace kdlae {

thread_local std::string g_err;
int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

bool debug_flag(const char* name) {
  const char* e = getenv("KDLAE_DEBUG");
  if (!e) return false;
  const std::string s(e), n(name);
  size_t i = 0;
  while (i <= s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    if (s.compare(i, j - i, n) == 0 && j - i == n.size()) return true;
    i = j + 1;
  }
  return false;
}

// Tile-shape selection.  Resident schedule when a variant with KG == kgroups exists: the weights
// are split into groups that fit the LDS budget (one group per grid.y), and NT (accumulator tiles
// per pass) minimises padding inside a group.  Otherwise the chunked schedule over (NT, KG).
// Weights sit in LDS in split fragment order (mfma3.h): 3 KiB per output tile and k-group pair.
static constexpr int kLdsBudgetKB = 152;
static long long tile_lds_bytes(int kgroups) { return (long long)((kgroups + 1) / 2) * 3072 + 64; }

void choose_variant(Gemm& g, bool /*prefer_single_k*/) {
  static const int nts[] = {1, 2, 3, 4, 6, 8, 9, 12};
  static const int kgs[] = {2, 3, 4, 6, 8, 9, 12, 16};  // (12 x 8 and wider only on the r01 chunked kernel)
  g.group_tiles = 0;
  g.WPE = 2;
  if (g.ksize == 1) {
    int best_nt = 0, best_w = 2;
    double best = 1e30;
// r05: weigh one or two more weight groups than the LDS budget needs, counting every computed tile
// (the last group's padding too).  A/B (profiles/r05zx_gemm_groups_ab.txt): C192 qkv (36 tiles) as
// 6 groups of 6 instead of 5 of 8 (the last half empty): 588 -> 382 us per launch at 16 x 128^2.
constexpr auto KDLAE_GEMM_GROUPS_ALT = 1;
    int best_groups = 0;
    for (int w : {2}) {
      // two resident blocks per CU at 4 waves/SIMD -> half the LDS budget each
      const int budget_kb = w == 4 ? 76 : kLdsBudgetKB;
      const int budget = (int)std::max<long long>(1, budget_kb * 1024LL / tile_lds_bytes(g.kgroups));
      const int ngroups0 = (int)ceil_div(g.ntiles, budget);
      for (int ngroups = ngroups0; ngroups <= ngroups0 + (KDLAE_GEMM_GROUPS_ALT ? 2 : 0); ++ngroups) {
      const int gt = (int)ceil_div(g.ntiles, ngroups);
      if (ngroups > ngroups0 && (int)ceil_div(g.ntiles, gt) != ngroups) continue;
      for (int nt : nts) {
        if (!gemm_has_variant(nt, g.kgroups, false, w, true, g.out_mode)) continue;
        const long long padded = ceil_div(gt, nt) * nt;
        // split weights + the group's bias (64 B per tile) must fit 160 KiB
        if (padded * tile_lds_bytes(g.kgroups) > (w == 4 ? 80 : 158) * 1024LL) continue;
        // default policy: 2 waves/SIMD.  4 waves/SIMD used to win on the store-heavy K <= 48 shapes
        // while every epilogue load drained the stores; with that fixed, 2 waves measure 10-15%
        // faster on all of them (r01 probe: C48 project_in @1024^2 5864 -> 5099 us)
        double cost = (double)padded / gt + 0.01 * (12 - nt) + (ngroups - 1) * 0.05;
        // an odd NT leaves each k-group's last tile alone with 2 independent accumulator chains:
        // C96 qkv (18 tiles) measured 2% faster as 3 chunks of 6 than as 2 chunks of 9 on two boxes
        // (profiles/r02_gemm_odd_nt_probe.txt); riding that tile along with the first pair instead
        // measured no gain
        if (nt % 2) cost += 0.05;
        if (KDLAE_GEMM_GROUPS_ALT) {
          // (with an odd-NT penalty of 0.10 the C96 qkv took 3 groups of 6 and lost 2-8%)
          const double computed = (double)ngroups * padded / g.ntiles;
          cost = computed * (1.0 + 0.05 * (ngroups - 1)) + 0.01 * (12 - nt) + ((nt % 2) ? 0.05 : 0.0);
        }
        if (cost < best) {
          best = cost;
          best_nt = nt;
          best_w = w;
          best_groups = ngroups;
        }
      }
      }
    }
    if (best_nt) {
      g.NT = best_nt;
      g.KG = g.kgroups;
      g.WPE = best_w;
      g.group_tiles = (int)ceil_div(g.ntiles, best_groups);
      return;
    }
  }
  double best = 1e30;
  for (int nt : nts)
    for (int kg : kgs) {
      if (!gemm_has_variant2(nt, kg, g.ksize == 3, g.out_mode) || (g.has_res && nt * kg >= 36)) continue;
      const long long nch = ceil_div(g.ntiles, nt), kch = ceil_div(g.kgroups, kg);
      if (kch > 1 && kg % 2) continue;  // split pairs may not straddle k-chunks (mfma3.h)
      const double waste = (double)(nch * nt) * (kch * kg) / ((double)g.ntiles * g.kgroups);
      // every k-chunk restages weights behind two barriers; every n-chunk re-reads A.
      // 1x1 (r01 v15 probe): n-chunks cost more than k-chunks; with penalties 0.06 / 0.02 the
      // K = 510/1021 FFN project_out and the C384 GEMMs take 12x8 chunks (72 -> 85 and 76 -> 90 TF/s)
      // 3x3 (r01 probe): an n-chunk re-gathers the whole im2col A (12x3 beat 6x12 at N = 384, 768);
      // with 12-tile chunks, halving the k-chunks (12x6) saved 2%; with 3-tile chunks 3x6 lost 12%
constexpr auto KDLAE_NPEN_1X1 = 0.06;
constexpr auto KDLAE_NPEN_3X3 = 0.12;
      const double npen = g.ksize == 3 ? KDLAE_NPEN_3X3 : KDLAE_NPEN_1X1;
constexpr auto KDLAE_KPEN_1X1 = 0.02;
      const double kpen = g.ksize == 3 ? (nt >= 12 ? 0.01 : 0.0) : KDLAE_KPEN_1X1;
      double cost = waste * (1.0 + npen * (nch - 1) + kpen * (kch - 1));
      if (cost < best - 1e-9) {
        best = cost;
        g.NT = nt;
        g.KG = kg;
      }
    }
}


int ParamStore::set(const char* name, const float* data, int64_t numel) {
  auto it = index.find(name);
  if (it == index.end()) return fail(KDLAE_EPARAM, std::string("unexpected key in state_dict: ") + name);
  if (keys[it->second].second != numel)
    return fail(KDLAE_EPARAM, std::string("size mismatch for ") + name + ": expected " +
                                  std::to_string(keys[it->second].second) + " got " + std::to_string(numel));
  staged[name].assign(data, data + numel);
  return KDLAE_OK;
}

int ParamStore::info(int i, const char** name, int64_t* numel) const {
  if (i < 0 || i >= (int)keys.size()) return fail(KDLAE_EPARAM, "param index out of range");
  if (name) *name = keys[i].first.c_str();
  if (numel) *numel = keys[i].second;
  return KDLAE_OK;
}

int ParamStore::check_complete() const {
  for (auto& kv : keys)
    if (!staged.count(kv.first)) return fail(KDLAE_EPARAM, "missing state_dict entry: " + kv.first);
  return KDLAE_OK;
}


int32_t ParamStore::base(const std::string& k, int* err) const {
  auto it = index.find(k);
  if (it == index.end()) {
    if (err && *err == KDLAE_OK) *err = fail(KDLAE_EPARAM, "missing state_dict entry: " + k);
    return -1;
  }
  return (int32_t)offset[it->second];
}

std::vector<float> ParamStore::flat() const {
  std::vector<float> v((size_t)total, 0.f);
  for (size_t i = 0; i < keys.size(); ++i) {
    auto it = staged.find(keys[i].first);
    if (it != staged.end()) std::copy(it->second.begin(), it->second.end(), v.begin() + offset[i]);
  }
  return v;
}

int run_gemm(const GemmCall& c, hipStream_t s) {
  const Gemm& g = *c.g;
  const long long HW = (long long)c.F * c.H * c.Wd;
  const int ldmax = std::max({c.in.ld, c.out.ld, c.ldr, c.out1.ld});
  if (HW * ldmax * (c.out_mode == 2 ? 4 : 1) >= (1LL << 31))
    return fail(KDLAE_EINVAL_SHAPE, "image too large for 32-bit in-image offsets");
  GemmParams p{};
  p.A = c.in.p;
  p.lda = c.in.ld;
  p.cg_per_tap = g.cg_per_tap;
  p.kgroups = g.kgroups;
  p.ksize = g.ksize;
  p.dil = 1;
  p.Wp = c.W;
  p.w_img_stride = c.w_img_stride;
  p.ntiles = g.ntiles;
  p.N = g.N;
  p.bias = c.bias;
  p.out = c.out.p;
  p.ldo = c.out.ld;
  p.R = c.R;
  p.ldr = c.ldr;
  p.ln = c.ln;
  p.ln_C = c.ln_C;
  p.relu = c.relu;
  p.Bn = c.B;
  p.H = c.H;
  p.W = c.Wd;
  p.F = c.F;
  p.kt = g.kt;
  p.out_mode = c.out_mode;
  p.tiles_per_img = (int)ceil_div(HW, kGemmRows);
  p.total_tiles = c.B * p.tiles_per_img;
  p.kchunks = g.group_tiles ? 1 : (int)ceil_div(g.kgroups, g.KG);
  p.group_tiles = g.group_tiles;
  p.Wm = c.Wm;
  p.wm_img_stride = c.wm_img_stride;
  p.bias_m = c.bias_m;
  p.out1 = c.out1.p;
  p.ldo1 = c.out1.ld;
  p.stats = nullptr;
  if (c.ln && (p.kchunks > 1 || g.kgroups * 16 != c.ln_C)) {
    if (!c.stats_buf) return fail(KDLAE_ESTATE, "LN GEMM needs a stats buffer");
    HIPCHK(launch_ln_stats(c.in.p, c.in.ld, c.ln_C, (long long)c.B * HW, c.stats_buf, s));
    p.stats = c.stats_buf;
  }
  const int gy = g.group_tiles ? (int)ceil_div(g.ntiles, g.group_tiles) : (int)ceil_div(g.ntiles, g.NT);
  p.tiles_per_block = gemm_tiles_per_block(p.total_tiles, gy, g.group_tiles != 0, g.WPE);
  const int gx = (int)ceil_div(p.total_tiles, p.tiles_per_block);
  HIPCHK(launch_gemm(p, g.NT, g.KG, g.WPE, gx, s));
  return KDLAE_OK;
}

int device_cu_count() {
  static std::mutex mu;
  static std::map<int, int> per_device;  // a process may drive several GPUs (nn.DataParallel-style)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  std::lock_guard<std::mutex> lock(mu);
  auto it = per_device.find(dev);
  if (it != per_device.end()) return it->second;
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
  per_device[dev] = v;
  return v;
}

// Tiles per block for a GEMM grid of ceil(T / tpb) x gy equal-work blocks.  One 8-wave block fills
// a CU at 2 waves/SIMD (two at 4), so the launch runs in ceil(blocks / slots) rounds and its
// makespan is rounds x tpb tile-times.  The old "about 512 blocks" rule could land a handful of
// blocks past a round (C192 project_in: 516 blocks = 3 rounds of 12 tiles for 24 tiles of work per
// CU).  Resident blocks also restage their weight group once (about half a tile-time, from L2).
int gemm_tiles_per_block(int total_tiles, int gy, bool resident, int wpe) {
  thread_local std::map<std::tuple<int, int, bool, int, int>, int> memo;  // a forward repeats ~30 shapes
  const int cus = device_cu_count();
  const auto key = std::make_tuple(total_tiles, gy, resident, wpe, cus);
  auto it = memo.find(key);
  if (it != memo.end()) return it->second;
  const long long slots = (long long)cus * (wpe == 4 ? 2 : 1);
  const int target = resident ? 256 * wpe : 1024;  // previous heuristic: the tie-break
  const int gx0 = (int)std::min<long long>(total_tiles, std::max<long long>(1, ceil_div(target, gy)));
  int best = (int)ceil_div(total_tiles, gx0);
  auto cost = [&](int tpb) {
    const long long blocks = ceil_div(total_tiles, tpb) * gy;
    const long long rounds = ceil_div(blocks, slots);
    return (double)rounds * (tpb + (resident ? 0.5 : 0.0));
  };
  double best_cost = cost(best);
  for (int tpb = 1; tpb <= total_tiles; ++tpb) {
    const double c = cost(tpb);
    if (c < best_cost * 0.98) {
      best_cost = c;
      best = tpb;
    }
  }
  memo[key] = best;
  return best;
}

}  // namespace kdlae
