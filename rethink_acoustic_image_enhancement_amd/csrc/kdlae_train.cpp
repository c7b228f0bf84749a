// KDLAE-T training engine (C ABI kdlae_tt_*, include/kdlae.h): forward with saved activations and
// the hand-sequenced backward of KDLAE_teacher (KDLAE/KDLAE_model.py:204-336) on the train.hip
// kernels, plus the L1LossSr and clip_grad_norm_ + AdamW steps of BasicSR's ImageCleanModel
// (Train/basicsr/models/image_restoration_model.py:198-218).
//
// Parameters and their gradients live in two flat caller-owned device buffers laid out in
// state_dict order, each key 16-byte aligned (kdlae_tt_param_info gives each key's offset), so the optimizer is one kernel
// over one buffer and the DDP gradient all-reduce is one RCCL call over one buffer.
//
// Workspace: [split-K partials][reduction partials][saved forward activations][backward scratch].
// The same code runs in a dry mode (no launches) to size it, so the size is exact.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/kdlae.h"
#include "runtime.h"
#include "train_kernels.h"

using kdlae::fail;
namespace tr = kdlae::train;

namespace {

constexpr size_t kSplitCap = 8u << 20;  // floats of split-K partials
constexpr size_t kRedCap = 8u << 20;    // floats of reduction partials

struct BlockRec {
  std::string p;
  int C = 0, heads = 0, hid = 0, Bn = 0, H = 0, W = 0;
  float *x = nullptr, *xn1 = nullptr, *st1 = nullptr, *qkv = nullptr, *qkvd = nullptr, *sumsq = nullptr, *G = nullptr,
        *A = nullptr, *ao = nullptr, *x1 = nullptr, *xn2 = nullptr, *st2 = nullptr, *y = nullptr, *yd = nullptr,
        *g = nullptr, *out = nullptr;
  float* wpo = nullptr;  // ffn.project_out weight with rows padded to ld4(hid) (odd hid only), zero pads
};

struct Saved {
  int B = 0, H = 0, W = 0;
  const void* ws = nullptr;
  size_t fwd_end = 0;
  bool valid = false;
  float *img_h = nullptr, *pe = nullptr, *enc1 = nullptr, *dn1c = nullptr, *enc2 = nullptr, *dn2c = nullptr,
        *enc3 = nullptr, *dn3c = nullptr, *lat = nullptr, *cat3 = nullptr, *dec3 = nullptr, *cat2 = nullptr,
        *dec2 = nullptr, *cat1 = nullptr, *dec1 = nullptr, *ref = nullptr, *catp = nullptr, *ro = nullptr,
        *hq_h = nullptr, *cenc = nullptr, *enh = nullptr;
  std::unordered_map<std::string, std::vector<BlockRec>> stages;
};

}  // namespace

struct kdlae_tt_handle {
  kdlae_t_config cfg{};
  int device = 0;
  std::vector<std::pair<std::string, int64_t>> keys;
  std::unordered_map<std::string, int64_t> off;
  int64_t total = 0;
  Saved sv;
  int ws_B = -1, ws_H = -1, ws_W = -1;  // last kdlae_tt_workspace_bytes query (its dry run is cached)
  int64_t ws_bytes = -1;
  // gradient-ready marks of the last kdlae_tt_backward_marked: mark_slot[m] = index of the event
  // recorded at backward mark m (-1: not a bucket boundary), mark_lo[j] = first flat offset of the
  // suffix [mark_lo[j], total) whose gradients are final once event j has completed
  std::vector<int> mark_slot;
  std::vector<int64_t> mark_lo;
  std::vector<hipEvent_t> mark_ev;
  // the marks and the backward's workspace peak depend only on (has_dsr, B, H, W, forward end):
  // cached, so a training step does not repeat the host-side dry run
  int mk_dsr = -1, mk_B = -1, mk_H = -1, mk_W = -1;
  size_t mk_fwd_end = 0, mk_peak = 0;
  // per key offset the backward writes (dry run): the (first, last) mark at which it is written
  std::map<int64_t, std::pair<int, int>> mk_touch;
  // KDLAE_DEBUG=train_trace: per-launch event pairs of the current call, dumped to KDLAE_PROBE_DUMP
  struct TraceRec {
    std::string tag;
    hipEvent_t a, b;
  };
  std::vector<TraceRec> trace;
  // backward side stream (non-blocking) and its fork / join events: the weight-gradient GEMMs and
  // bias column sums run there, beside the input-gradient chain on the caller's stream
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // stage_bwd's lagged synchronisation: recorded after each block's last side launch (its scratch
  // region and gradient buffers are reused two blocks later)
  hipEvent_t ev_blk[2] = {nullptr, nullptr};
  ~kdlae_tt_handle() {
    for (hipEvent_t e : mark_ev) (void)hipEventDestroy(e);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_join) (void)hipEventDestroy(ev_join);
    for (hipEvent_t e : {ev_blk[0], ev_blk[1]})
      if (e) (void)hipEventDestroy(e);
    if (side) (void)hipStreamDestroy(side);
  }
};

namespace {

int hid_of(const kdlae_t_config& c, int dim) { return (int)((double)dim * c.ffn_expansion_factor); }

// state_dict order of KDLAE_teacher (KDLAE_model.py:220-268; TransformerBlock :150-157)
void build_keys(kdlae_tt_handle* h) {
  const kdlae_t_config& c = h->cfg;
  // every key starts on a 16-byte boundary (pad floats stay zero), so the weight operands of the
  // training GEMMs (temperature [heads] and ffn.dwconv [2 hid * 9] break 4-float alignment
  // otherwise) qualify for the vectorised kernel
  auto add = [&](const std::string& k, int64_t n) {
    h->off[k] = h->total;
    h->keys.emplace_back(k, n);
    h->total += (n + 3) & ~int64_t(3);
  };
  auto conv = [&](const std::string& n, int co, int ci, int k, bool b) {
    add(n + ".weight", (int64_t)co * ci * k * k);
    if (b) add(n + ".bias", co);
  };
  auto block = [&](const std::string& p, int dim, int heads) {
    const int hid = hid_of(c, dim);
    add(p + ".norm1.body.weight", dim);
    if (!c.layernorm_biasfree) add(p + ".norm1.body.bias", dim);
    add(p + ".attn.temperature", heads);
    conv(p + ".attn.qkv", 3 * dim, dim, 1, c.bias);
    conv(p + ".attn.qkv_dwconv", 3 * dim, 1, 3, c.bias);
    conv(p + ".attn.project_out", dim, dim, 1, c.bias);
    add(p + ".norm2.body.weight", dim);
    if (!c.layernorm_biasfree) add(p + ".norm2.body.bias", dim);
    conv(p + ".ffn.project_in", 2 * hid, dim, 1, c.bias);
    conv(p + ".ffn.dwconv", 2 * hid, 1, 3, c.bias);
    conv(p + ".ffn.project_out", dim, hid, 1, c.bias);
  };
  auto stage = [&](const std::string& n, int cnt, int dim, int heads) {
    for (int i = 0; i < cnt; ++i) block(n + "." + std::to_string(i), dim, heads);
  };
  const int d = c.dim, *nb = c.num_blocks, *hd = c.heads, nr = c.num_refinement_blocks;
  conv("patch_embed.proj", d, c.inp_channels, 3, false);
  stage("encoder_level1", nb[0], d, hd[0]);
  conv("down1_2.body.0", d / 2, d, 3, false);
  stage("encoder_level2", nb[1], 2 * d, hd[1]);
  conv("down2_3.body.0", d, 2 * d, 3, false);
  stage("encoder_level3", nb[2], 4 * d, hd[2]);
  conv("down3_4.body.0", 2 * d, 4 * d, 3, false);
  stage("latent", nb[3], 8 * d, hd[3]);
  conv("up4_3.body.0", 16 * d, 8 * d, 3, false);
  conv("reduce_chan_level3", 4 * d, 8 * d, 1, c.bias);
  stage("decoder_level3", nb[2], 4 * d, hd[2]);
  conv("up3_2.body.0", 8 * d, 4 * d, 3, false);
  conv("reduce_chan_level2", 2 * d, 4 * d, 1, c.bias);
  stage("decoder_level2", nb[1], 2 * d, hd[1]);
  conv("up2_1.body.0", 4 * d, 2 * d, 3, false);
  stage("decoder_level1", nb[0], 2 * d, hd[0]);
  stage("refinement", nr, 2 * d, hd[0]);
  conv("output", c.out_channels, 2 * d, 3, c.bias);
  conv("output_param", 2 * d, c.out_channels + 1, 3, c.bias);
  stage("refinement_out", nr, 2 * d, hd[0]);
  conv("output2", c.out_channels, 2 * d, 3, c.bias);
  if (c.static_train) {
    const int hc = 2 * d;
    conv("cen", hc, c.out_channels, 3, c.bias);
    conv("upen.body.0", 2 * hc, hc, 3, false);
    stage("enhance", nr, hc / 2, hd[0]);
    conv("outputen", c.out_channels, hc / 2, 3, c.bias);
  }
}

int validate(const kdlae_t_config& c) {
  if (c.dual_pixel_task)
    return fail(KDLAE_ENOTIMPL, "dual_pixel_task=True: the reference forward raises NameError (KDLAE_model.py:305-321)");
  if (c.dim <= 0 || c.dim % 2 || 8 * c.dim > 512)
    return fail(KDLAE_EINVAL_CONFIG, "training path: dim must be even and 8*dim <= 512 (LayerNorm wave kernel)");
  if (c.inp_channels < 1 || c.inp_channels != c.out_channels)
    return fail(KDLAE_EINVAL_CONFIG, "inp_channels must equal out_channels (hq = out + inp_img, KDLAE_model.py:321)");
  for (int i = 0; i < 4; ++i)
    if (c.num_blocks[i] < 0 || c.heads[i] <= 0) return fail(KDLAE_EINVAL_CONFIG, "bad num_blocks/heads");
  if (c.num_refinement_blocks < 0) return fail(KDLAE_EINVAL_CONFIG, "bad num_refinement_blocks");
  auto head_ok = [](int C, int heads) { return C % heads == 0 && C / heads <= 120; };
  const int d = c.dim;
  const int lv[4] = {d, 2 * d, 4 * d, 8 * d};
  for (int i = 0; i < 4; ++i)
    if (!head_ok(lv[i], c.heads[i]))
      return fail(KDLAE_EINVAL_CONFIG, "training path: channels per head must divide C and be <= 120");
  if (!head_ok(2 * d, c.heads[0]) || (c.static_train && !head_ok(d, c.heads[0])))
    return fail(KDLAE_EINVAL_CONFIG, "training path: channels per head must divide C and be <= 120");
  if (c.ffn_expansion_factor <= 0) return fail(KDLAE_EINVAL_CONFIG, "bad ffn_expansion_factor");
  return KDLAE_OK;
}

struct Ctx {
  const kdlae_tt_handle* h;
  const float* th = nullptr;
  float* gr = nullptr;
  char* base = nullptr;
  size_t off = 0, cap = 0, peak = 0;
  bool dry = true;
  hipStream_t s = nullptr;  // the stream launches go to: main_s, or side_s inside a side segment
  float* splitk = nullptr;   // split-K partials of the current stream (splitk_main / splitk_side)
  // backward side stream (kdlae_tt_backward*): a side segment (side_begin .. side_end) holds
  // launches that only READ buffers the main stream does not write until the next join.  Every
  // segment starts with a fork (the side stream waits for the main stream's current point), so side
  // work is ordered after all earlier main work, including reduction flushes; the main stream waits
  // for the side stream (join) at every flush, mark and block end, before a write to a buffer a
  // pending side launch reads, and before scratch is released.  side_s == nullptr: one stream.
  hipStream_t main_s = nullptr, side_s = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_blk[2] = {nullptr, nullptr};
  bool blk_rec[2] = {false, false};  // ev_blk[p] holds a record of this call (stage_bwd)
  float* splitk_main = nullptr;
  float* splitk_side = nullptr;
  bool in_side = false, side_pending = false;
  // gradient-ready marks (kdlae_tt_backward_marked): the dry run records, per key offset, the first
  // and last mark index at which its gradient was written; the real run records an event per mark
  std::map<int64_t, std::pair<int, int>>* touch = nullptr;
  int cur_mark = 0;
  bool record_marks = false;
  // launch trace (diagnostics only: KDLAE_DEBUG=train_trace); tag = the layer being sequenced
  std::vector<kdlae_tt_handle::TraceRec>* trace = nullptr;
  std::string tag;
  // queued partial reductions of the backward, one list per stream (partials written on the side
  // stream are reduced on it, those of the main stream on the main stream, so a flush never waits
  // for the other stream): one batched launch at the next flush (a full queue, the end of a
  // TransformerBlock, a mark, the end); red_off = floats of the stream's `red` buffer in use
  struct RedList {
    std::vector<tr::RedDesc> pend;
    float* red = nullptr;
    size_t red_off = 0;
  } rl[2];  // [0] main stream, [1] side segments
  RedList& cur_rl() { return rl[in_side ? 1 : 0]; }

  size_t red_cap = 0;  // floats of each `red` buffer (red_floats(): the largest single reduction's partials)
  int red_err = KDLAE_OK;  // why the last red_take returned nullptr
  float* alloc(size_t n) {
    off = (off + 255) / 256 * 256;
    float* p = reinterpret_cast<float*>(base + off);
    off += n * sizeof(float);
    if (off > peak) peak = off;
    return p;
  }
  const float* W(const std::string& k) const {
    auto it = h->off.find(k);
    return it == h->off.end() ? nullptr : th + it->second;
  }
  float* G(const std::string& k) const {
    auto it = h->off.find(k);
    if (it == h->off.end()) return nullptr;
    if (touch) {
      auto t = touch->find(it->second);
      if (t == touch->end()) touch->emplace(it->second, std::make_pair(cur_mark, cur_mark));
      else t->second.second = cur_mark;
    }
    return gr + it->second;
  }
};

int flush_reduce(Ctx& c);
int flush_all(Ctx& c);

int hip_fail(hipError_t e, const char* what) {
  return fail(KDLAE_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

// enter a side segment: the side stream waits for everything enqueued on the main stream so far
int side_begin(Ctx& c) {
  if (c.in_side) return KDLAE_OK;
  c.splitk = c.splitk_side;
  c.in_side = true;
  if (c.dry || !c.side_s) {
    c.splitk = c.splitk_main;  // one stream: the main stream's partials
    return KDLAE_OK;
  }
  hipError_t e = hipEventRecord(c.ev_fork, c.main_s);
  if (e == hipSuccess) e = hipStreamWaitEvent(c.side_s, c.ev_fork, 0);
  if (e != hipSuccess) return hip_fail(e, "side stream fork");
  c.s = c.side_s;
  c.side_pending = true;
  return KDLAE_OK;
}

void side_end(Ctx& c) {
  c.in_side = false;
  c.s = c.main_s;
  c.splitk = c.splitk_main;
}

// the main stream waits for every side launch enqueued so far
int join(Ctx& c) {
  if (c.in_side) side_end(c);
  if (!c.side_pending) return KDLAE_OK;
  c.side_pending = false;
  hipError_t e = hipEventRecord(c.ev_join, c.side_s);
  if (e == hipSuccess) e = hipStreamWaitEvent(c.main_s, c.ev_join, 0);
  return e == hipSuccess ? KDLAE_OK : hip_fail(e, "side stream join");
}

// record ev on the side stream after every side launch enqueued so far (no-op on one stream)
int side_record(Ctx& c, hipEvent_t ev) {
  if (c.dry || !c.side_s || !ev) return KDLAE_OK;
  hipError_t e = hipEventRecord(ev, c.side_s);
  return e == hipSuccess ? KDLAE_OK : hip_fail(e, "side stream event");
}

// the main stream waits for a side-stream event recorded earlier (typically long complete)
int main_wait(Ctx& c, hipEvent_t ev) {
  if (c.dry || !c.side_s || !ev) return KDLAE_OK;
  hipError_t e = hipStreamWaitEvent(c.main_s, ev, 0);
  return e == hipSuccess ? KDLAE_OK : hip_fail(e, "side stream wait");
}

// a region of the reduction buffer for a queued reduction's partials (flushes when full)
// Returns nullptr with c.red_err set (and the message in kdlae_last_error) when the flush fails
// (a HIP error) or when one request alone exceeds the buffer (a sizing bug: KDLAE_ESTATE).
float* red_take(Ctx& c, size_t n) {
  n = (n + 63) / 64 * 64;
  if (c.cur_rl().red_off + n > c.red_cap) {
    const int rc = flush_reduce(c);
    if (rc != KDLAE_OK) {
      c.red_err = rc;
      return nullptr;
    }
  }
  if (n > c.red_cap) {  // red_floats() must cover every reduction of the step
    c.red_err = fail(KDLAE_ESTATE, "internal: a reduction needs " + std::to_string(n) +
                                       " partial floats but the reduction buffer holds " +
                                       std::to_string(c.red_cap) + " (red_floats() misses it)");
    return nullptr;
  }
  Ctx::RedList& l = c.cur_rl();
  float* p = l.red + l.red_off;
  l.red_off += n;
  return p;
}

// A point in the backward after which some parameters' gradients are final (one TransformerBlock,
// one head conv, ...).  kdlae_tt_backward_marked records an event at the marks that close a suffix
// of the flat buffer, so the caller can all-reduce that suffix while the backward continues.
int mark(Ctx& c) {
  int rc = flush_all(c);  // the gradients this mark declares final (joins the side stream)
  if (rc) return rc;
  if (c.record_marks && !c.dry && c.cur_mark < (int)c.h->mark_slot.size()) {
    const int j = c.h->mark_slot[c.cur_mark];
    if (j >= 0) {
      hipError_t e = hipEventRecord(c.h->mark_ev[j], c.s);
      if (e != hipSuccess) return fail(KDLAE_EHIP, std::string("hipEventRecord: ") + hipGetErrorString(e));
    }
  }
  ++c.cur_mark;
  return KDLAE_OK;
}

hipEvent_t trace_begin(Ctx& c) {
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) == hipSuccess) (void)hipEventRecord(e, c.s);
  return e;
}

void trace_end(Ctx& c, hipEvent_t a, const char* what) {
  hipEvent_t b = nullptr;
  if (!a || hipEventCreate(&b) != hipSuccess) return;
  (void)hipEventRecord(b, c.s);
  std::string w(what);
  const size_t paren = w.find('(');
  if (paren != std::string::npos) w.resize(paren);
  if (w.rfind("tr::", 0) == 0) w = w.substr(4);
  c.trace->push_back({c.tag + "," + w, a, b});
}

#define LAUNCH(x)                                                                                    \
  do {                                                                                               \
    if (!c.dry) {                                                                                    \
      hipEvent_t ta_ = c.trace ? trace_begin(c) : nullptr;                                           \
      hipError_t e_ = (x);                                                                           \
      if (c.trace) trace_end(c, ta_, #x);                                                            \
      if (e_ != hipSuccess) return fail(KDLAE_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    }                                                                                                \
  } while (0)
#define TRY(x)                  \
  do {                          \
    int r_ = (x);               \
    if (r_ != KDLAE_OK) return r_; \
  } while (0)

inline int ld4(int n) { return (n + 3) / 4 * 4; }

// the current stream's queued reductions, on that stream (its partials were written there, and its
// later writes to the same `red` buffer follow the flush in stream order)
int flush_reduce(Ctx& c) {
  Ctx::RedList& l = c.cur_rl();
  if (!l.pend.empty()) LAUNCH(tr::launch_part_reduce_multi(l.pend.data(), (int)l.pend.size(), c.s));
  l.pend.clear();
  l.red_off = 0;
  return KDLAE_OK;
}

// every queued reduction (the side list on the side stream), then the main stream joins the side
// stream: all gradients so far are final on the main stream
int flush_all(Ctx& c) {
  const bool was_side = c.in_side;
  Ctx::RedList& sl = c.rl[1];
  if (!sl.pend.empty()) {
    hipStream_t keep = c.s;
    c.s = c.side_s && !c.dry ? c.side_s : c.main_s;
    if (c.side_s && !c.dry) c.side_pending = true;
    LAUNCH(tr::launch_part_reduce_multi(sl.pend.data(), (int)sl.pend.size(), c.s));
    c.s = keep;
  }
  sl.pend.clear();
  sl.red_off = 0;
  TRY(join(c));
  TRY(flush_reduce(c));
  if (was_side) TRY(side_begin(c));
  return KDLAE_OK;
}

// queue out[0, ncols) = sum over nblk rows (stride pstride) of part; flushed in one batched launch
int queue_reduce(Ctx& c, const float* part, int nblk, int ncols, int pstride, float* out) {
  if (!out || ncols <= 0) return KDLAE_OK;
  tr::RedDesc d;
  d.part = part;
  d.out = out;
  d.nblk = nblk;
  d.ncols = ncols;
  d.pstride = pstride;
  Ctx::RedList& l = c.cur_rl();
  l.pend.push_back(d);
  if ((int)l.pend.size() == tr::kRedBatch) return flush_reduce(c);
  return KDLAE_OK;
}

// Forward / input-gradient GEMMs of the deep low-resolution levels (M = 1536..6144 pixels at
// 6 x 128^2, K up to 2042) fill a few hundred 64 x 64 tiles: under one wave of blocks on 256 CUs.
// The K >= 1024 ones take the split-K partials too (launch_tgemm splits only where the grid is short).
// r04 trace A/B (gpurun_out/trab): dX 1536 x 384 K 2042 0.544 -> 0.386 ms, 6144 x 192 K 1020 0.688 ->
// 0.660; at K = 510 / 576 the partial round trip lost (0.42 -> 0.53, 0.42 -> 0.50 ms).
constexpr auto KDLAE_TRAIN_LAG = 1;  // stage_bwd's lagged side-stream synchronisation (0: join per block)
constexpr auto KDLAE_TRAIN_SPLIT_SMALL = 1;
constexpr long long kSplitSmallRows = 24576;  // below the row-streaming kernel's threshold
constexpr int kSplitSmallK = 1000;

// one tgemm launch; `what` (+ the shape) labels it in the launch trace
int gemm(Ctx& c, const tr::TGemm& g0, size_t cap, const std::string& what) {
  tr::TGemm g = g0;
  if (KDLAE_TRAIN_SPLIT_SMALL && cap == 0 && !g.partial && (long long)g.M * g.nz1 * g.nz2 < kSplitSmallRows &&
      g.K >= kSplitSmallK) {
    g.partial = c.splitk;
    cap = kSplitCap;
  }
  if (c.trace) {
    const std::string keep = c.tag;
    c.tag += " " + what + " M" + std::to_string(g.M) + " N" + std::to_string(g.N) + " K" + std::to_string(g.K) + " z" +
             std::to_string(g.nz1 * g.nz2);
    LAUNCH(tr::launch_tgemm(g, cap, c.s));
    c.tag = keep;
    return KDLAE_OK;
  }
  LAUNCH(tr::launch_tgemm(g, cap, c.s));
  return KDLAE_OK;
}

constexpr auto KDLAE_LN_BWD_MAXB = 2048;
constexpr auto KDLAE_LN_BWD_ROWS = 32;
int nblk_for(long long rows, long long ncols, int maxb = 1024, int rows_per_blk = 128) {
  long long nb = rows / rows_per_blk;
  if (nb > maxb) nb = maxb;
  const long long cap = (long long)(kRedCap / (size_t)(ncols > 0 ? ncols : 1));
  if (nb > cap) nb = cap;
  return nb < 1 ? 1 : (int)nb;
}

// ---- convolutions over NHWC views (weights OIHW straight from the flat parameter buffer)
struct V {
  float* p;
  int ld;
};

// wp (optional): the weight as [Cout][ldw] rows (a padded copy), else the flat buffer's [Cout][Cin]
// pad_ok: `out` is a private ld-rounded buffer whose row pad may be overwritten (TGemm::c_pad_ok)
int conv1(Ctx& c, const std::string& n, V x, int Cin, int Cout, long long P, V out, const float* R = nullptr,
          int ldr = 0, V wp = {nullptr, 0}, bool pad_ok = false) {
  tr::TGemm g;
  g.A = x.p; g.sam = x.ld; g.sak = 1;
  g.B = wp.p ? wp.p : c.W(n + ".weight"); g.sbk = 1; g.sbn = wp.p ? wp.ld : Cin;
  g.C = out.p; g.scm = out.ld; g.scn = 1;
  g.bias = c.W(n + ".bias");
  g.R = R; g.srm = ldr; g.srn = 1;
  g.M = (int)P; g.N = Cout; g.K = Cin;
  g.c_pad_ok = pad_ok;
  TRY(gemm(c, g, 0, n + " fwd"));
  return KDLAE_OK;
}

int bias_grad(Ctx& c, V dy, int N, long long P, float* out) {
  if (!out) return KDLAE_OK;
  const int nb = nblk_for(P, N);
  float* part = red_take(c, (size_t)nb * N);
  if (!part) return c.red_err;
  LAUNCH(tr::launch_colsum(dy.p, dy.ld, N, P, 1, 0, part, nb, c.s));
  return queue_reduce(c, part, nb, N, N, out);
  return KDLAE_OK;
}

// dW = dY^T X, db = colsum dY, dX = dY W (+R)
int conv1_bwd(Ctx& c, const std::string& n, V x, V dy, int Cin, int Cout, long long P, V dx, const float* R = nullptr,
              int ldr = 0, V wp = {nullptr, 0}, bool pad_ok = false) {
  tr::TGemm g;
  g.A = dy.p; g.sam = 1; g.sak = dy.ld;
  g.B = x.p; g.sbk = x.ld; g.sbn = 1;
  g.C = c.G(n + ".weight"); g.scm = Cin; g.scn = 1;
  g.M = Cout; g.N = Cin; g.K = (int)P;
  TRY(side_begin(c));  // dW and db only read x and dy
  g.partial = c.splitk;
  TRY(gemm(c, g, kSplitCap, n + " dW"));
  TRY(bias_grad(c, dy, Cout, P, c.G(n + ".bias")));
  side_end(c);
  if (dx.p) {
    tr::TGemm d;
    d.A = dy.p; d.sam = dy.ld; d.sak = 1;
    d.B = wp.p ? wp.p : c.W(n + ".weight"); d.sbk = wp.p ? wp.ld : Cin; d.sbn = 1;
    d.C = dx.p; d.scm = dx.ld; d.scn = 1;
    d.R = R; d.srm = ldr; d.srn = 1;
    d.M = (int)P; d.N = Cin; d.K = Cout;
    d.c_pad_ok = pad_ok;
    TRY(gemm(c, d, 0, n + " dX"));
  }
  return KDLAE_OK;
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// A 3x3 conv with a narrow side (<= 4 channels: the image heads and the 3- / 4-channel inputs) is a
// 64-wide GEMM tile that is mostly padding; those run on the inference path's small-channel kernels
// (conv_small.hip): narrow input -> the MFMA small-input kernel (K = 9 Cin <= 36), narrow output ->
// the LDS-tiled VALU head kernel.  `wt` selects the transposed-conv (dX) weight view of the same
// OIHW weight.  Returns 1 when it launched, 0 when the shape is not one of theirs.
int conv3_narrow(Ctx& c, const float* w, const float* bias, V in, int Cin, int Cout, int Bn, int H, int W, int dil,
                 V out, const float* R, int ldr, bool transposed, int* done) {
  *done = 0;
  if (!R && Cin * 9 <= 36 && Cout % 16 == 0 && out.ld % 4 == 0 && al16(out.p)) {
    kdlae::SmallInParams p{};
    p.in = in.p;
    p.sb = (long long)H * W * in.ld;
    p.sc = 1;
    p.sy = (long long)W * in.ld;
    p.sx = in.ld;
    p.Cin = Cin;
    p.Cout = Cout;
    p.dil = dil;
    p.w = w;
    p.wt = transposed ? Cout : 0;
    p.bias = bias;
    p.out = out.p;
    p.ldo = out.ld;
    p.Bn = Bn;
    p.H = H;
    p.W = W;
    p.F = 1;
    p.kt = 1;
    LAUNCH(kdlae::launch_conv_small_in(p, c.s));
    *done = 1;
    return KDLAE_OK;
  }
  if (Cout <= 4 && Cin % 16 == 0 && Cin <= 256 && dil == 1 && in.ld % 4 == 0 && al16(in.p)) {
    kdlae::SmallOutParams p{};
    p.in = in.p;
    p.ld = in.ld;
    p.Cin = Cin;
    p.Cout = Cout;
    p.w = w;
    p.wt = transposed ? 1 : 0;
    p.bias = bias;
    p.Bn = Bn;
    p.H = H;
    p.W = W;
    p.F = 1;
    p.ks = 3;
    p.out = out.p;
    p.out_nchw = 0;
    p.ldo = out.ld;
    p.res_nhwc = R;
    p.ldr = ldr;
    LAUNCH(kdlae::launch_conv_small_out(p, c.s));
    *done = 1;
  }
  return KDLAE_OK;
}

// the implicit-GEMM 3x3 conv's B operand repacked from the OIHW weights into a [9 Cg][N] matrix in the
// workspace (bmode 2 / 3 -> 0): float4 B loads in the tiled kernel instead of per-element index math
// (KDLAE_DEBUG=train_w3_raw keeps the OIHW operand; same bits)
int pack_w3(Ctx& c, tr::TGemm& g, int N) {
  if (kdlae::debug_flag("train_w3_raw") || N % 4) return KDLAE_OK;
  float* wp = c.alloc((size_t)9 * g.Cg * N);
  LAUNCH(tr::launch_pack_w3(g.B, g.Cg, N, g.bmode, wp, c.s));
  g.B = wp;
  g.bmode = 0;
  g.sbk = N;
  g.sbn = 1;
  return KDLAE_OK;
}

int conv3(Ctx& c, const std::string& n, V x, int Cin, int Cout, int Bn, int H, int W, int dil, V out,
          const float* R = nullptr, int ldr = 0) {
  int done = 0;
  TRY(conv3_narrow(c, c.W(n + ".weight"), c.W(n + ".bias"), x, Cin, Cout, Bn, H, W, dil, out, R, ldr, false, &done));
  if (done) return KDLAE_OK;
  tr::TGemm g;
  g.A = x.p; g.amode = 1; g.lda = x.ld; g.Cg = Cin;
  g.B = c.W(n + ".weight"); g.bmode = 2;
  TRY(pack_w3(c, g, Cout));
  g.C = out.p; g.scm = out.ld; g.scn = 1;
  g.bias = c.W(n + ".bias");
  g.R = R; g.srm = ldr; g.srn = 1;
  g.M = Bn * H * W; g.N = Cout; g.K = 9 * Cin;
  g.Bn = Bn; g.H = H; g.W = W; g.dil = dil;
  // split-K when the pixel tiles alone leave the chip idle (the 16^2 / 32^2 Upsample convs: 72-144
  // tiles, K up to 3456); launch_tgemm only splits where that fills it
  g.partial = c.splitk;
  TRY(gemm(c, g, kSplitCap, n + " fwd3"));
  return KDLAE_OK;
}

int conv3_bwd(Ctx& c, const std::string& n, V x, V dy, int Cin, int Cout, int Bn, int H, int W, int dil, V dx,
              const float* R = nullptr, int ldr = 0) {
  const long long P = (long long)Bn * H * W;
  float* gw = c.G(n + ".weight");
  TRY(side_begin(c));  // dW and db only read x and dy (dx may alias R, never x or dy)
  if (tr::dw3_small_ok(Cin, Cout) && gw) {
    // narrow side: per-block [Cout][Cin][9] partials on the VALU (train_small.hip)
    const int ncols = Cin * Cout * 9;
    const int nb = tr::dw3_small_blocks(P, Cin, Cout, c.red_cap);
    float* part = red_take(c, (size_t)nb * ncols);
    if (!part) return c.red_err;
    LAUNCH(tr::launch_dw3_small(dy.p, dy.ld, x.p, x.ld, Cin, Cout, Bn, H, W, dil, part, nb, c.s));
    TRY(queue_reduce(c, part, nb, ncols, ncols, gw));
  } else {
    tr::TGemm g;  // dW[co][ci][t] = sum_p dY[p,co] X[p + off_t, ci]
    g.A = dy.p; g.sam = 1; g.sak = dy.ld;
    g.B = x.p; g.bmode = 1; g.ldb = x.ld;
    g.C = gw; g.scm = (long long)Cin * 9; g.scn = 9; g.bC2 = 1;
    g.nz2 = 9;
    g.M = Cout; g.N = Cin; g.K = (int)P;
    g.Bn = Bn; g.H = H; g.W = W; g.dil = dil;
    g.partial = c.splitk;
    TRY(gemm(c, g, kSplitCap, n + " dW3"));
  }
  TRY(bias_grad(c, dy, Cout, P, c.G(n + ".bias")));
  side_end(c);
  if (dx.p) {
    // the transposed conv: Cout -> Cin channels (flipped taps), narrow-side kernels where they apply
    int done = 0;
    TRY(conv3_narrow(c, c.W(n + ".weight"), nullptr, dy, Cout, Cin, Bn, H, W, dil, dx, R, ldr, true, &done));
    if (done) return KDLAE_OK;
    tr::TGemm d;  // transposed conv: flipped taps, channels swapped
    d.A = dy.p; d.amode = 1; d.lda = dy.ld; d.Cg = Cout;
    d.B = c.W(n + ".weight"); d.bmode = 3;
    TRY(pack_w3(c, d, Cin));
    d.C = dx.p; d.scm = dx.ld; d.scn = 1;
    d.R = R; d.srm = ldr; d.srn = 1;
    d.M = (int)P; d.N = Cin; d.K = 9 * Cout;
    d.Bn = Bn; d.H = H; d.W = W; d.dil = dil;
    d.partial = c.splitk;
    TRY(gemm(c, d, kSplitCap, n + " dX3"));
  }
  return KDLAE_OK;
}

// ---- TransformerBlock (KDLAE_model.py:150-163)
int block_fwd(Ctx& c, BlockRec& r) {
  const kdlae_t_config& cf = c.h->cfg;
  const int C = r.C, C3 = 3 * C, hid = r.hid, heads = r.heads, Ch = C / heads, Bn = r.Bn;
  const long long HW = (long long)r.H * r.W, P = Bn * HW;
  const int bf = cf.layernorm_biasfree;
  const std::string& p = r.p;
  c.tag = p;
  r.xn1 = c.alloc(P * C);
  r.st1 = c.alloc(2 * P);
  LAUNCH(tr::launch_ln_fwd(r.x, C, c.W(p + ".norm1.body.weight"), c.W(p + ".norm1.body.bias"), C, P, bf, r.xn1, C,
                           r.st1, c.s));
  r.qkv = c.alloc(P * C3);
  TRY(conv1(c, p + ".attn.qkv", {r.xn1, C}, C, C3, P, {r.qkv, C3}));
  r.qkvd = c.alloc(P * C3);
  LAUNCH(tr::launch_dw_fwd(r.qkv, C3, c.W(p + ".attn.qkv_dwconv.weight"), c.W(p + ".attn.qkv_dwconv.bias"), 0, C3,
                           Bn, r.H, r.W, r.qkvd, C3, c.s));
  // ||q||^2, ||k||^2 per image and channel (F.normalize over HW, :135-136)
  r.sumsq = c.alloc((size_t)Bn * 2 * C);
  {
    const int nb = nblk_for(HW, (long long)2 * C * Bn, 256);
    LAUNCH(tr::launch_colsum(r.qkvd, C3, 2 * C, HW, Bn, 1, c.rl[0].red, nb, c.s));
    LAUNCH(tr::launch_part_reduce(c.rl[0].red, nb, 2 * C, Bn, r.sumsq, 0, 1.f, c.s));
  }
  const size_t mats = (size_t)Bn * heads * Ch * Ch;
  r.G = c.alloc(mats);
  {
    tr::TGemm g;  // G = q^T k per (image, head), un-normalised
    g.A = r.qkvd; g.sam = 1; g.sak = C3; g.bA1 = HW * C3; g.bA2 = Ch;
    g.B = r.qkvd + C; g.sbk = C3; g.sbn = 1; g.bB1 = HW * C3; g.bB2 = Ch;
    g.C = r.G; g.scm = Ch; g.scn = 1; g.bC1 = (long long)heads * Ch * Ch; g.bC2 = (long long)Ch * Ch;
    g.M = Ch; g.N = Ch; g.K = (int)HW; g.nz1 = Bn; g.nz2 = heads;
    g.partial = c.splitk;
    TRY(gemm(c, g, kSplitCap, "gram"));
  }
  r.A = c.alloc(mats);
  LAUNCH(tr::launch_attn_softmax(r.G, r.sumsq, c.W(p + ".attn.temperature"), Bn, C, heads, r.A, c.s));
  r.ao = c.alloc(P * C);
  {
    tr::TGemm g;  // out = A v  (per pixel: ao[p,i] = sum_j A[i,j] v[p,j])
    g.A = r.qkvd + 2 * C; g.sam = C3; g.sak = 1; g.bA1 = HW * C3; g.bA2 = Ch;
    g.B = r.A; g.sbk = 1; g.sbn = Ch; g.bB1 = (long long)heads * Ch * Ch; g.bB2 = (long long)Ch * Ch;
    g.C = r.ao; g.scm = C; g.scn = 1; g.bC1 = HW * C; g.bC2 = Ch;
    g.M = (int)HW; g.N = Ch; g.K = Ch; g.nz1 = Bn; g.nz2 = heads;
    TRY(gemm(c, g, 0, "av"));
  }
  r.x1 = c.alloc(P * C);
  TRY(conv1(c, p + ".attn.project_out", {r.ao, C}, C, C, P, {r.x1, C}, r.x, C));
  r.xn2 = c.alloc(P * C);
  r.st2 = c.alloc(2 * P);
  LAUNCH(tr::launch_ln_fwd(r.x1, C, c.W(p + ".norm2.body.weight"), c.W(p + ".norm2.body.bias"), C, P, bf, r.xn2, C,
                           r.st2, c.s));
  // hidden-width buffers get a pixel stride rounded up to 4 floats so GEMM rows stay float4-aligned
  const int L2 = ld4(2 * hid), L1 = ld4(hid);
  r.y = c.alloc(P * L2);
  TRY(conv1(c, p + ".ffn.project_in", {r.xn2, C}, C, 2 * hid, P, {r.y, L2}, nullptr, 0, {nullptr, 0}, true));
  // yd (the dwconv output) is not kept: the backward recomputes it from y, which its weight gradient
  // reads anyway (1 KiB per pixel less written here and read there); KDLAE_DEBUG=train_keep_yd stores
  // it for the stored-yd backward (A/B; same bits)
  r.yd = kdlae::debug_flag("train_keep_yd") ? c.alloc(P * L2) : nullptr;
  r.g = c.alloc(P * L1);
  // dwconv + GELU gate in one pass (train_dwg.hip): g for project_out
  LAUNCH(tr::launch_dwgate_fwd(r.y, L2, c.W(p + ".ffn.dwconv.weight"), c.W(p + ".ffn.dwconv.bias"), hid, Bn, r.H,
                               r.W, r.yd, L2, r.g, L1, c.s));
  r.out = c.alloc(P * C);
  if (hid % 4) {
    // row stride hid is not a multiple of 4 floats: a zero-padded [C][ld4(hid)] copy lets the forward
    // and dX GEMMs use the vectorised kernel (kept until the backward: theta is unchanged in between)
    r.wpo = c.alloc((size_t)C * L1);
    LAUNCH(tr::launch_copy_cols(c.W(p + ".ffn.project_out.weight"), hid, r.wpo, L1, hid, C, 0, c.s, L1));
  }
  TRY(conv1(c, p + ".ffn.project_out", {r.g, L1}, hid, C, P, {r.out, C}, r.x1, C, {r.wpo, L1}));
  return KDLAE_OK;
}

// sum the nb partial rows [9 C weights | C bias] of a depthwise conv's gradient into its keys
int dw_reduce(Ctx& c, const float* part, int nb, int C, const std::string& n) {
  // partial columns: [9 C weights | C bias]; one reduce when the bias key directly follows the
  // weight key in the flat buffer (keys are 16-byte aligned, so only when 9 C % 4 == 0)
  float* gw = c.G(n + ".weight");
  float* gb = c.G(n + ".bias");
  if (!gb || gb == gw + 9LL * C) return queue_reduce(c, part, nb, gb ? 10 * C : 9 * C, 10 * C, gw);
  TRY(queue_reduce(c, part, nb, 9 * C, 10 * C, gw));
  return queue_reduce(c, part + 9LL * C, nb, C, 10 * C, gb);
}

int ln_bwd(Ctx& c, const float* dy, const float* x, const float* st, int C, long long P, const std::string& n,
           const float* R, float* dx) {
  const int bf = c.h->cfg.layernorm_biasfree;
  const int ncol = bf ? C : 2 * C;
  // 32 pixels per block (8 per wave: one or two steps of the lane-group loop, whose loads are used
  // right away, so the kernel is latency-bound and wants many waves in flight), up to 2048 blocks
  const int nb = nblk_for(P, ncol, KDLAE_LN_BWD_MAXB, KDLAE_LN_BWD_ROWS);
  float* part = red_take(c, (size_t)nb * ncol);
  if (!part) return c.red_err;
  LAUNCH(tr::launch_ln_bwd(dy, C, x, C, c.W(n + ".weight"), st, C, P, bf, R, C, dx, C, part, nb, c.s));
  // partial columns: [C weight | C bias (WithBias)], split when the keys are not adjacent
  float* gw = c.G(n + ".weight");
  float* gb = bf ? nullptr : c.G(n + ".bias");
  if (!gb || gb == gw + C) return queue_reduce(c, part, nb, ncol, ncol, gw);
  TRY(queue_reduce(c, part, nb, C, ncol, gw));
  return queue_reduce(c, part + C, nb, C, ncol, gb);
}

// d: [P][C] gradient of the block output on entry, of the block input on exit
// d_in: [P][C] gradient of the block output; d_out: of the block input (a different buffer).
// Synchronisation with the side stream (stage_bwd passes lag = true): the main stream never waits for
// the block's own side launches.  The side launches read d_in (project_out weight gradient) and this
// block's scratch (the dW GEMMs' dy, dx1, dqkv and the bias sums); stage_bwd rotates three gradient
// buffers and alternates two scratch regions, so neither is written again before the block after
// next, whose start waits for this block's side launches.  lag = false: a join before the last
// LayerNorm backward and a full flush + join at the end.  *extent: end of the block's scratch.
int block_bwd(Ctx& c, const BlockRec& r, const float* d_in, float* d_out, bool lag, size_t* extent) {
  float* d = const_cast<float*>(d_in);
  const int C = r.C, C3 = 3 * C, hid = r.hid, heads = r.heads, Ch = C / heads, Bn = r.Bn;
  const long long HW = (long long)r.H * r.W, P = Bn * HW;
  const std::string& p = r.p;
  c.tag = p;
  const size_t mark = c.off;
  // ffn (KDLAE_model.py:101-106)
  const int L2 = ld4(2 * hid), L1 = ld4(hid);
  float* dg = c.alloc(P * L1);
  TRY(conv1_bwd(c, p + ".ffn.project_out", {r.g, L1}, {d, C}, hid, C, P, {dg, L1}, nullptr, 0, {r.wpo, L1}, true));
  float* dy = c.alloc(P * L2);
  {
    // gate backward + transposed dwconv + dwconv weight gradient in one pass (train_dwg.hip)
    const int nb = tr::dwg_blocks(Bn, r.H, r.W);
    float* part = red_take(c, (size_t)nb * 10 * 2 * hid);
    if (!part) return c.red_err;
    if (r.yd) {
      LAUNCH(tr::launch_dwgate_bwd(dg, L1, r.yd, L2, r.y, L2, c.W(p + ".ffn.dwconv.weight"), hid, Bn, r.H, r.W, dy,
                                   L2, part, c.s));
    } else {
      LAUNCH(tr::launch_dwgate_bwd_rc(dg, L1, r.y, L2, c.W(p + ".ffn.dwconv.weight"), c.W(p + ".ffn.dwconv.bias"), hid,
                                      Bn, r.H, r.W, dy, L2, part, c.s));
    }
    TRY(dw_reduce(c, part, nb, 2 * hid, p + ".ffn.dwconv"));
  }
  float* dxn2 = c.alloc(P * C);
  TRY(conv1_bwd(c, p + ".ffn.project_in", {r.xn2, C}, {dy, L2}, C, 2 * hid, P, {dxn2, C}));
  float* dx1 = c.alloc(P * C);
  TRY(ln_bwd(c, dxn2, r.x1, r.st2, C, P, p + ".norm2.body", d, dx1));
  // attention (KDLAE_model.py:124-145)
  float* dao = c.alloc(P * C);
  TRY(conv1_bwd(c, p + ".attn.project_out", {r.ao, C}, {dx1, C}, C, C, P, {dao, C}));
  const size_t mats = (size_t)Bn * heads * Ch * Ch;
  float* dA = c.alloc(mats);
  float* dqkvd = c.alloc(P * C3);
  {
    tr::TGemm g;  // dA[i,j] = sum_p dao[p,i] v[p,j]
    g.A = dao; g.sam = 1; g.sak = C; g.bA1 = HW * C; g.bA2 = Ch;
    g.B = r.qkvd + 2 * C; g.sbk = C3; g.sbn = 1; g.bB1 = HW * C3; g.bB2 = Ch;
    g.C = dA; g.scm = Ch; g.scn = 1; g.bC1 = (long long)heads * Ch * Ch; g.bC2 = (long long)Ch * Ch;
    g.M = Ch; g.N = Ch; g.K = (int)HW; g.nz1 = Bn; g.nz2 = heads;
    g.partial = c.splitk;
    TRY(gemm(c, g, kSplitCap, "dA"));
  }
  {
    tr::TGemm g;  // dv[p,j] = sum_i dao[p,i] A[i,j]
    g.A = dao; g.sam = C; g.sak = 1; g.bA1 = HW * C; g.bA2 = Ch;
    g.B = r.A; g.sbk = Ch; g.sbn = 1; g.bB1 = (long long)heads * Ch * Ch; g.bB2 = (long long)Ch * Ch;
    g.C = dqkvd + 2 * C; g.scm = C3; g.scn = 1; g.bC1 = HW * C3; g.bC2 = Ch;
    g.M = (int)HW; g.N = Ch; g.K = Ch; g.nz1 = Bn; g.nz2 = heads;
    TRY(gemm(c, g, 0, "dv"));
  }
  float* Mq = c.alloc(mats);
  float* cq = c.alloc((size_t)Bn * heads * Ch);
  float* ck = c.alloc((size_t)Bn * heads * Ch);
  float* dtp = c.alloc((size_t)Bn * heads);
  LAUNCH(tr::launch_attn_bwd(r.G, r.sumsq, c.W(p + ".attn.temperature"), r.A, dA, Bn, C, heads, Mq, cq, ck, dtp, c.s));
  float* gtemp = c.G(p + ".attn.temperature");  // outside LAUNCH: the dry run must record the write
  TRY(queue_reduce(c, dtp, Bn, heads, heads, gtemp));
  {
    tr::TGemm g;  // dq[p,i] = sum_j Mq[i,j] k[p,j] + cq[i] q[p,i]
    g.A = r.qkvd + C; g.sam = C3; g.sak = 1; g.bA1 = HW * C3; g.bA2 = Ch;
    g.B = Mq; g.sbk = 1; g.sbn = Ch; g.bB1 = (long long)heads * Ch * Ch; g.bB2 = (long long)Ch * Ch;
    g.C = dqkvd; g.scm = C3; g.scn = 1; g.bC1 = HW * C3; g.bC2 = Ch;
    g.R = r.qkvd; g.srm = C3; g.srn = 1; g.bR1 = HW * C3; g.bR2 = Ch;
    g.rs = cq; g.brs1 = (long long)heads * Ch; g.brs2 = Ch;
    g.M = (int)HW; g.N = Ch; g.K = Ch; g.nz1 = Bn; g.nz2 = heads;
    TRY(gemm(c, g, 0, "dq"));
    g.A = r.qkvd;  // dk[p,j] = sum_i Mq[i,j] q[p,i] + ck[j] k[p,j]
    g.B = Mq; g.sbk = Ch; g.sbn = 1;
    g.C = dqkvd + C;
    g.R = r.qkvd + C;
    g.rs = ck;
    TRY(gemm(c, g, 0, "dk"));
  }
  float* dqkv = c.alloc(P * C3);
  {
    const int nb = tr::dwg_blocks(Bn, r.H, r.W);
    float* part = red_take(c, (size_t)nb * 10 * C3);
    if (!part) return c.red_err;
    LAUNCH(tr::launch_dw_bwd(dqkvd, C3, r.qkv, C3, c.W(p + ".attn.qkv_dwconv.weight"), C3, Bn, r.H, r.W, dqkv, C3,
                             part, c.s));
    TRY(dw_reduce(c, part, nb, C3, p + ".attn.qkv_dwconv"));
  }
  float* dxn1 = c.alloc(P * C);
  TRY(conv1_bwd(c, p + ".attn.qkv", {r.xn1, C}, {dqkv, C3}, C, C3, P, {dxn1, C}));
  if (!lag) TRY(join(c));
  TRY(ln_bwd(c, dxn1, r.x, r.st1, C, P, p + ".norm1.body", dx1, d_out));
  TRY(flush_reduce(c));  // the main list, before the block's scratch (dtp) is released
  if (!lag) TRY(flush_all(c));
  if (extent) *extent = c.off;
  c.off = mark;
  return KDLAE_OK;
}

int stage_fwd(Ctx& c, const std::string& name, int n, int C, int heads, int Bn, int H, int W, float* x, float** out) {
  std::vector<BlockRec>& recs = const_cast<kdlae_tt_handle*>(c.h)->sv.stages[name];
  recs.assign(n, BlockRec{});
  for (int i = 0; i < n; ++i) {
    BlockRec& r = recs[i];
    r.p = name + "." + std::to_string(i);
    r.C = C; r.heads = heads; r.hid = hid_of(c.h->cfg, C); r.Bn = Bn; r.H = H; r.W = W;
    r.x = x;
    TRY(block_fwd(c, r));
    x = r.out;
  }
  *out = x;
  return KDLAE_OK;
}

// The blocks of a stage share one shape, so their scratch regions alternate between [base, e0) and
// [e0, e0 + size), and block k reads gradient buffer k % 3 and writes (k + 1) % 3 (0 = d): before
// block k reuses the region and the buffer of block k - 2, the main stream waits for the event
// recorded after block k - 2's side launches (by then complete, as a rule), instead of joining the
// side stream at every block (r05 trace: 240 joins, ≈13 µs of idle main stream each, plus waits for
// the last weight gradients).  The marked backward keeps a full flush + join per block (the
// gradient-ready marks need them); the stage ends with one either way, the result copied into d.
int stage_bwd(Ctx& c, const std::string& name, float* d) {
  const auto& recs = c.h->sv.stages.at(name);
  const bool lag = !c.record_marks && !c.dry && c.side_s && KDLAE_TRAIN_LAG;
  const BlockRec& r0 = recs.front();
  const size_t dn = (size_t)r0.Bn * r0.H * r0.W * r0.C;
  const size_t off0 = c.off;
  float* dbuf[3] = {d, c.alloc(dn), c.alloc(dn)};
  const size_t base = c.off;
  size_t e0 = base;
  c.blk_rec[0] = c.blk_rec[1] = false;
  for (int i = (int)recs.size() - 1, k = 0; i >= 0; --i, ++k) {
    const int par = k & 1;
    c.off = par ? e0 : base;  // the same layout with or without lag, so the dry run sizes it
    if (lag && c.blk_rec[par]) TRY(main_wait(c, c.ev_blk[par]));
    size_t ext = 0;
    TRY(block_bwd(c, recs[i], dbuf[k % 3], dbuf[(k + 1) % 3], lag, &ext));
    if (par == 0) e0 = ext;
    if (lag) {
      TRY(side_record(c, c.ev_blk[par]));
      c.blk_rec[par] = true;
      ++c.cur_mark;  // mark() without its flush and join
    } else {
      TRY(mark(c));
    }
  }
  if (lag) TRY(flush_all(c));
  const float* res = dbuf[recs.size() % 3];
  if (res != d) LAUNCH(hipMemcpyAsync(d, res, dn * sizeof(float), hipMemcpyDeviceToDevice, c.s));
  c.off = off0;
  return KDLAE_OK;
}

// ---- whole network (KDLAE_model.py:270-336)
int net_fwd(Ctx& c, const float* img, const float* rate, float* hq, float* sr) {
  kdlae_tt_handle* h = const_cast<kdlae_tt_handle*>(c.h);
  Saved& s = h->sv;
  const kdlae_t_config& cf = h->cfg;
  const int B = s.B, H = s.H, W = s.W, d = cf.dim, oc = cf.out_channels, ic = cf.inp_channels;
  const int* nb = cf.num_blocks;
  const int* hd = cf.heads;
  const int nr = cf.num_refinement_blocks;
  const long long P1 = (long long)B * H * W, P2 = P1 / 4, P3 = P1 / 16, P4 = P1 / 64;
  const int H2 = H / 2, W2 = W / 2, H3 = H / 4, W3 = W / 4, H4 = H / 8, W4 = W / 8;

  c.tag = "net";
  s.img_h = c.alloc(P1 * ic);
  LAUNCH(tr::launch_nchw_to_nhwc(img, ic, B, (long long)H * W, s.img_h, ic, 0, c.s));
  s.pe = c.alloc(P1 * d);
  TRY(conv3(c, "patch_embed.proj", {s.img_h, ic}, ic, d, B, H, W, 1, {s.pe, d}));
  TRY(stage_fwd(c, "encoder_level1", nb[0], d, hd[0], B, H, W, s.pe, &s.enc1));
  s.dn1c = c.alloc(P1 * (d / 2));
  TRY(conv3(c, "down1_2.body.0", {s.enc1, d}, d, d / 2, B, H, W, 1, {s.dn1c, d / 2}));
  float* dn1 = c.alloc(P2 * 2 * d);
  LAUNCH(tr::launch_shuffle(s.dn1c, d / 2, dn1, 2 * d, d / 2, B, H2, W2, 0, c.s));
  TRY(stage_fwd(c, "encoder_level2", nb[1], 2 * d, hd[1], B, H2, W2, dn1, &s.enc2));
  s.dn2c = c.alloc(P2 * d);
  TRY(conv3(c, "down2_3.body.0", {s.enc2, 2 * d}, 2 * d, d, B, H2, W2, 1, {s.dn2c, d}));
  float* dn2 = c.alloc(P3 * 4 * d);
  LAUNCH(tr::launch_shuffle(s.dn2c, d, dn2, 4 * d, d, B, H3, W3, 0, c.s));
  TRY(stage_fwd(c, "encoder_level3", nb[2], 4 * d, hd[2], B, H3, W3, dn2, &s.enc3));
  s.dn3c = c.alloc(P3 * 2 * d);
  TRY(conv3(c, "down3_4.body.0", {s.enc3, 4 * d}, 4 * d, 2 * d, B, H3, W3, 1, {s.dn3c, 2 * d}));
  float* dn3 = c.alloc(P4 * 8 * d);
  LAUNCH(tr::launch_shuffle(s.dn3c, 2 * d, dn3, 8 * d, 2 * d, B, H4, W4, 0, c.s));
  TRY(stage_fwd(c, "latent", nb[3], 8 * d, hd[3], B, H4, W4, dn3, &s.lat));
  // decoder level 3: cat [up4_3(latent), enc3] -> reduce_chan_level3 (KDLAE_model.py:288-291)
  float* u43 = c.alloc(P4 * 16 * d);
  TRY(conv3(c, "up4_3.body.0", {s.lat, 8 * d}, 8 * d, 16 * d, B, H4, W4, 1, {u43, 16 * d}));
  s.cat3 = c.alloc(P3 * 8 * d);
  LAUNCH(tr::launch_shuffle(u43, 16 * d, s.cat3, 8 * d, 4 * d, B, H4, W4, 1, c.s));
  LAUNCH(tr::launch_copy_cols(s.enc3, 4 * d, s.cat3 + 4 * d, 8 * d, 4 * d, P3, 0, c.s));
  float* rc3 = c.alloc(P3 * 4 * d);
  TRY(conv1(c, "reduce_chan_level3", {s.cat3, 8 * d}, 8 * d, 4 * d, P3, {rc3, 4 * d}));
  TRY(stage_fwd(c, "decoder_level3", nb[2], 4 * d, hd[2], B, H3, W3, rc3, &s.dec3));
  // decoder level 2 (:293-296)
  float* u32 = c.alloc(P3 * 8 * d);
  TRY(conv3(c, "up3_2.body.0", {s.dec3, 4 * d}, 4 * d, 8 * d, B, H3, W3, 1, {u32, 8 * d}));
  s.cat2 = c.alloc(P2 * 4 * d);
  LAUNCH(tr::launch_shuffle(u32, 8 * d, s.cat2, 4 * d, 2 * d, B, H3, W3, 1, c.s));
  LAUNCH(tr::launch_copy_cols(s.enc2, 2 * d, s.cat2 + 2 * d, 4 * d, 2 * d, P2, 0, c.s));
  float* rc2 = c.alloc(P2 * 2 * d);
  TRY(conv1(c, "reduce_chan_level2", {s.cat2, 4 * d}, 4 * d, 2 * d, P2, {rc2, 2 * d}));
  TRY(stage_fwd(c, "decoder_level2", nb[1], 2 * d, hd[1], B, H2, W2, rc2, &s.dec2));
  // decoder level 1 (:298-300), refinement (:302)
  float* u21 = c.alloc(P2 * 4 * d);
  TRY(conv3(c, "up2_1.body.0", {s.dec2, 2 * d}, 2 * d, 4 * d, B, H2, W2, 1, {u21, 4 * d}));
  s.cat1 = c.alloc(P1 * 2 * d);
  LAUNCH(tr::launch_shuffle(u21, 4 * d, s.cat1, 2 * d, d, B, H2, W2, 1, c.s));
  LAUNCH(tr::launch_copy_cols(s.enc1, d, s.cat1 + d, 2 * d, d, P1, 0, c.s));
  TRY(stage_fwd(c, "decoder_level1", nb[0], 2 * d, hd[0], B, H, W, s.cat1, &s.dec1));
  TRY(stage_fwd(c, "refinement", nr, 2 * d, hd[0], B, H, W, s.dec1, &s.ref));
  // output heads (:314-321)
  s.hq_h = c.alloc(P1 * oc);
  if (cf.params_cat) {
    s.catp = c.alloc(P1 * (oc + 1));
    TRY(conv3(c, "output", {s.ref, 2 * d}, 2 * d, oc, B, H, W, 1, {s.catp, oc + 1}));
    LAUNCH(tr::launch_nchw_to_nhwc(rate, 1, B, (long long)H * W, s.catp + oc, oc + 1, 0, c.s));
    float* op = c.alloc(P1 * 2 * d);
    TRY(conv3(c, "output_param", {s.catp, oc + 1}, oc + 1, 2 * d, B, H, W, 2, {op, 2 * d}));
    TRY(stage_fwd(c, "refinement_out", nr, 2 * d, hd[0], B, H, W, op, &s.ro));
    TRY(conv3(c, "output2", {s.ro, 2 * d}, 2 * d, oc, B, H, W, 1, {s.hq_h, oc}, s.img_h, ic));
  } else {
    TRY(conv3(c, "output", {s.ref, 2 * d}, 2 * d, oc, B, H, W, 1, {s.hq_h, oc}, s.img_h, ic));
  }
  LAUNCH(tr::launch_nhwc_to_nchw(s.hq_h, oc, nullptr, oc, B, (long long)H * W, hq, c.s));
  // super-resolution branch (:324-329)
  if (cf.static_train) {
    const int hc = 2 * d;
    s.cenc = c.alloc(P1 * hc);
    TRY(conv3(c, "cen", {s.hq_h, oc}, oc, hc, B, H, W, 1, {s.cenc, hc}));
    float* upc = c.alloc(P1 * 2 * hc);
    TRY(conv3(c, "upen.body.0", {s.cenc, hc}, hc, 2 * hc, B, H, W, 1, {upc, 2 * hc}));
    float* ups = c.alloc(P1 * 4 * (hc / 2));
    LAUNCH(tr::launch_shuffle(upc, 2 * hc, ups, hc / 2, hc / 2, B, H, W, 1, c.s));
    TRY(stage_fwd(c, "enhance", nr, hc / 2, hd[0], B, 2 * H, 2 * W, ups, &s.enh));
    float* srh = c.alloc(P1 * 4 * oc);
    TRY(conv3(c, "outputen", {s.enh, hc / 2}, hc / 2, oc, B, 2 * H, 2 * W, 1, {srh, oc}));
    LAUNCH(tr::launch_nhwc_to_nchw(srh, oc, nullptr, oc, B, 4LL * H * W, sr, c.s));
  }
  return KDLAE_OK;
}

// has_dsr: the sr branch is differentiated (dsr given); the dry sizing pass always takes it
int net_bwd(Ctx& c, const float* dhq, const float* dsr, bool has_dsr) {
  const Saved& s = c.h->sv;
  const kdlae_t_config& cf = c.h->cfg;
  const int B = s.B, H = s.H, W = s.W, d = cf.dim, oc = cf.out_channels, ic = cf.inp_channels;
  const long long P1 = (long long)B * H * W, P2 = P1 / 4, P3 = P1 / 16, P4 = P1 / 64;
  const int H2 = H / 2, W2 = W / 2, H3 = H / 4, W3 = W / 4, H4 = H / 8, W4 = W / 8;

  c.tag = "net";
  float* dhq_h = c.alloc(P1 * oc);
  if (dhq) LAUNCH(tr::launch_nchw_to_nhwc(dhq, oc, B, (long long)H * W, dhq_h, oc, 0, c.s));
  else LAUNCH(hipMemsetAsync(dhq_h, 0, P1 * oc * sizeof(float), c.s));
  if (cf.static_train && has_dsr) {
    const int hc = 2 * d;
    float* dsr_h = c.alloc(P1 * 4 * oc);
    LAUNCH(tr::launch_nchw_to_nhwc(dsr, oc, B, 4LL * H * W, dsr_h, oc, 0, c.s));
    float* denh = c.alloc(P1 * 4 * (hc / 2));
    TRY(conv3_bwd(c, "outputen", {s.enh, hc / 2}, {dsr_h, oc}, hc / 2, oc, B, 2 * H, 2 * W, 1, {denh, hc / 2}));
    TRY(mark(c));
    TRY(stage_bwd(c, "enhance", denh));
    float* dupc = c.alloc(P1 * 2 * hc);
    LAUNCH(tr::launch_shuffle(denh, hc / 2, dupc, 2 * hc, hc / 2, B, H, W, 0, c.s));
    // upen's input (cenc) is recomputed-free: it was saved in the forward
    float* dcen = c.alloc(P1 * hc);
    TRY(conv3_bwd(c, "upen.body.0", {s.cenc, hc}, {dupc, 2 * hc}, hc, 2 * hc, B, H, W, 1, {dcen, hc}));
    TRY(mark(c));
    TRY(conv3_bwd(c, "cen", {s.hq_h, oc}, {dcen, hc}, oc, hc, B, H, W, 1, {dhq_h, oc}, dhq_h, oc));
    TRY(mark(c));
  } else if (cf.static_train) {
    // sr unused by the loss: its parameters get zero gradients (grad buffer is zeroed up front)
  }
  // hq = out + img: d(out) = dhq
  float* dref = c.alloc(P1 * 2 * d);
  if (cf.params_cat) {
    float* dro = c.alloc(P1 * 2 * d);
    TRY(conv3_bwd(c, "output2", {s.ro, 2 * d}, {dhq_h, oc}, 2 * d, oc, B, H, W, 1, {dro, 2 * d}));
    TRY(mark(c));
    TRY(stage_bwd(c, "refinement_out", dro));
    float* dcatp = c.alloc(P1 * (oc + 1));
    TRY(conv3_bwd(c, "output_param", {s.catp, oc + 1}, {dro, 2 * d}, oc + 1, 2 * d, B, H, W, 2, {dcatp, oc + 1}));
    TRY(mark(c));
    TRY(conv3_bwd(c, "output", {s.ref, 2 * d}, {dcatp, oc + 1}, 2 * d, oc, B, H, W, 1, {dref, 2 * d}));
    TRY(mark(c));
  } else {
    TRY(conv3_bwd(c, "output", {s.ref, 2 * d}, {dhq_h, oc}, 2 * d, oc, B, H, W, 1, {dref, 2 * d}));
    TRY(mark(c));
  }
  TRY(stage_bwd(c, "refinement", dref));
  TRY(stage_bwd(c, "decoder_level1", dref));  // dref now holds d(cat1) = [d up2_1 | d enc1]
  float* de1 = c.alloc(P1 * d);
  LAUNCH(tr::launch_copy_cols(dref + d, 2 * d, de1, d, d, P1, 0, c.s));
  float* du21 = c.alloc(P2 * 4 * d);
  LAUNCH(tr::launch_shuffle(dref, 2 * d, du21, 4 * d, d, B, H2, W2, 0, c.s));
  float* ddec2 = c.alloc(P2 * 2 * d);
  TRY(conv3_bwd(c, "up2_1.body.0", {s.dec2, 2 * d}, {du21, 4 * d}, 2 * d, 4 * d, B, H2, W2, 1, {ddec2, 2 * d}));
  TRY(mark(c));
  TRY(stage_bwd(c, "decoder_level2", ddec2));
  float* dcat2 = c.alloc(P2 * 4 * d);
  TRY(conv1_bwd(c, "reduce_chan_level2", {s.cat2, 4 * d}, {ddec2, 2 * d}, 4 * d, 2 * d, P2, {dcat2, 4 * d}));
  TRY(mark(c));
  float* de2 = c.alloc(P2 * 2 * d);
  LAUNCH(tr::launch_copy_cols(dcat2 + 2 * d, 4 * d, de2, 2 * d, 2 * d, P2, 0, c.s));
  float* du32 = c.alloc(P3 * 8 * d);
  LAUNCH(tr::launch_shuffle(dcat2, 4 * d, du32, 8 * d, 2 * d, B, H3, W3, 0, c.s));
  float* ddec3 = c.alloc(P3 * 4 * d);
  TRY(conv3_bwd(c, "up3_2.body.0", {s.dec3, 4 * d}, {du32, 8 * d}, 4 * d, 8 * d, B, H3, W3, 1, {ddec3, 4 * d}));
  TRY(mark(c));
  TRY(stage_bwd(c, "decoder_level3", ddec3));
  float* dcat3 = c.alloc(P3 * 8 * d);
  TRY(conv1_bwd(c, "reduce_chan_level3", {s.cat3, 8 * d}, {ddec3, 4 * d}, 8 * d, 4 * d, P3, {dcat3, 8 * d}));
  TRY(mark(c));
  float* de3 = c.alloc(P3 * 4 * d);
  LAUNCH(tr::launch_copy_cols(dcat3 + 4 * d, 8 * d, de3, 4 * d, 4 * d, P3, 0, c.s));
  float* du43 = c.alloc(P4 * 16 * d);
  LAUNCH(tr::launch_shuffle(dcat3, 8 * d, du43, 16 * d, 4 * d, B, H4, W4, 0, c.s));
  float* dlat = c.alloc(P4 * 8 * d);
  TRY(conv3_bwd(c, "up4_3.body.0", {s.lat, 8 * d}, {du43, 16 * d}, 8 * d, 16 * d, B, H4, W4, 1, {dlat, 8 * d}));
  TRY(mark(c));
  TRY(stage_bwd(c, "latent", dlat));
  // encoder, deepest first; each Downsample's dX accumulates into the skip gradient
  float* ddn3c = c.alloc(P3 * 2 * d);
  LAUNCH(tr::launch_shuffle(dlat, 8 * d, ddn3c, 2 * d, 2 * d, B, H4, W4, 1, c.s));
  TRY(conv3_bwd(c, "down3_4.body.0", {s.enc3, 4 * d}, {ddn3c, 2 * d}, 4 * d, 2 * d, B, H3, W3, 1, {de3, 4 * d}, de3,
                4 * d));
  TRY(mark(c));
  TRY(stage_bwd(c, "encoder_level3", de3));
  float* ddn2c = c.alloc(P2 * d);
  LAUNCH(tr::launch_shuffle(de3, 4 * d, ddn2c, d, d, B, H3, W3, 1, c.s));
  TRY(conv3_bwd(c, "down2_3.body.0", {s.enc2, 2 * d}, {ddn2c, d}, 2 * d, d, B, H2, W2, 1, {de2, 2 * d}, de2, 2 * d));
  TRY(mark(c));
  TRY(stage_bwd(c, "encoder_level2", de2));
  float* ddn1c = c.alloc(P1 * (d / 2));
  LAUNCH(tr::launch_shuffle(de2, 2 * d, ddn1c, d / 2, d / 2, B, H2, W2, 1, c.s));
  TRY(conv3_bwd(c, "down1_2.body.0", {s.enc1, d}, {ddn1c, d / 2}, d, d / 2, B, H, W, 1, {de1, d}, de1, d));
  TRY(mark(c));
  TRY(stage_bwd(c, "encoder_level1", de1));
  TRY(conv3_bwd(c, "patch_embed.proj", {s.img_h, ic}, {de1, d}, ic, d, B, H, W, 1, {nullptr, 0}));
  TRY(mark(c));
  return KDLAE_OK;
}

// floats the reduction buffer needs: kRedCap, or the largest fused depthwise backward's partials
// ([dwg_blocks][10 C] at each level's resolution, C = 2 hid or 3 dim) when that is larger
size_t red_floats(const kdlae_t_config& cf, int B, int H, int W) {
  size_t need = kRedCap;
  auto level = [&](int C, int h, int w) {
    const size_t nb = (size_t)tr::dwg_blocks(B, h, w);
    const int hid = hid_of(cf, C);
    need = std::max(need, nb * 10 * (size_t)std::max(2 * hid, 3 * C) + 64);
  };
  const int d = cf.dim;
  level(d, H, W);
  level(2 * d, H, W);  // decoder_level1 / refinement / refinement_out
  level(2 * d, H / 2, W / 2);
  level(4 * d, H / 4, W / 4);
  level(8 * d, H / 8, W / 8);
  if (cf.static_train) level(d, 2 * H, 2 * W);  // enhance
  return need;
}

void ctx_init(Ctx& c, const kdlae_tt_handle* h, void* ws, size_t ws_bytes, bool dry, hipStream_t s, int B, int H,
              int W) {
  c.h = h;
  c.dry = dry;
  c.s = s;
  c.base = dry ? nullptr : static_cast<char*>(ws);
  c.cap = ws_bytes;
  c.off = 0;
  c.main_s = s;
  c.splitk_main = c.splitk = c.alloc(kSplitCap);
  c.splitk_side = c.alloc(kSplitCap);
  c.red_cap = red_floats(h->cfg, B, H, W);
  c.rl[0].red = c.alloc(c.red_cap);
  c.rl[1].red = c.alloc(c.red_cap);
}

// the backward's side stream (created once per handle, on its device); KDLAE_DEBUG=train_serial
// keeps every launch on the caller's stream (A/B and diagnostics: same results either way)
int use_side_stream(Ctx& c, kdlae_tt_handle* h) {
  if (kdlae::debug_flag("train_serial")) return KDLAE_OK;
  if (!h->side) {
    hipError_t e = hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming);
    for (hipEvent_t* ev : {&h->ev_blk[0], &h->ev_blk[1]})
      if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    if (e != hipSuccess) return hip_fail(e, "backward side stream");
  }
  c.side_s = h->side;
  c.ev_fork = h->ev_fork;
  c.ev_join = h->ev_join;
  c.ev_blk[0] = h->ev_blk[0];
  c.ev_blk[1] = h->ev_blk[1];
  return KDLAE_OK;
}

// KDLAE_DEBUG=train_trace: wait for the call's launches and append "phase,layer,kernel,ms" rows to
// the KDLAE_PROBE_DUMP file (diagnostics; the launches are the same, each bracketed by two events)
void trace_dump(kdlae_tt_handle* h, hipStream_t s, const char* phase) {
  if (h->trace.empty()) return;
  (void)hipStreamSynchronize(s);
  const char* path = getenv("KDLAE_PROBE_DUMP");
  FILE* f = path ? fopen(path, "a") : nullptr;
  for (auto& t : h->trace) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, t.a, t.b);
    if (f) fprintf(f, "%s,%s,%.5f\n", phase, t.tag.c_str(), ms);
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  if (f) fclose(f);
  h->trace.clear();
}

}  // namespace

extern "C" {

int kdlae_tt_create(const kdlae_t_config* cfg, int device, kdlae_tt_handle** out) {
  if (!cfg || !out) return fail(KDLAE_EINVAL_CONFIG, "null argument");
  int rc = validate(*cfg);
  if (rc) return rc;
  auto* h = new kdlae_tt_handle();
  h->cfg = *cfg;
  h->device = device;
  build_keys(h);
  *out = h;
  return KDLAE_OK;
}

int kdlae_tt_destroy(kdlae_tt_handle* h) {
  delete h;
  return KDLAE_OK;
}

int kdlae_tt_num_params(const kdlae_tt_handle* h) { return h ? (int)h->keys.size() : 0; }

int kdlae_tt_param_info(const kdlae_tt_handle* h, int index, const char** name, int64_t* numel, int64_t* offset) {
  if (!h || index < 0 || index >= (int)h->keys.size()) return fail(KDLAE_EPARAM, "param index out of range");
  if (name) *name = h->keys[index].first.c_str();
  if (numel) *numel = h->keys[index].second;
  if (offset) *offset = h->off.at(h->keys[index].first);
  return KDLAE_OK;
}

int64_t kdlae_tt_num_floats(const kdlae_tt_handle* h) { return h ? h->total : -1; }

static int check_shape(int B, int H, int W) {
  if (B <= 0 || H <= 0 || W <= 0) return fail(KDLAE_EINVAL_SHAPE, "B, H, W must be positive");
  if (H % 8 || W % 8)
    return fail(KDLAE_EINVAL_SHAPE, "H and W must be divisible by 8 (pixel_unshuffle x3, KDLAE_model.py:186-187)");
  if ((long long)B * H * W * 4 > (1LL << 31) - 1) return fail(KDLAE_EINVAL_SHAPE, "too many pixels for one step");
  return KDLAE_OK;
}

int64_t kdlae_tt_workspace_bytes(kdlae_tt_handle* h, int B, int H, int W) {
  if (!h) return -1;
  if (check_shape(B, H, W)) return -1;
  // the dry run walks the whole step on the host: cache it per shape (every training step asks)
  if (h->ws_B == B && h->ws_H == H && h->ws_W == W) return h->ws_bytes;
  Saved keep = h->sv;
  Ctx c;
  ctx_init(c, h, nullptr, 0, true, nullptr, B, H, W);
  h->sv = Saved{};
  h->sv.B = B; h->sv.H = H; h->sv.W = W;
  int rc = net_fwd(c, nullptr, nullptr, nullptr, nullptr);
  if (rc == KDLAE_OK) rc = net_bwd(c, nullptr, nullptr, h->cfg.static_train != 0);
  h->sv = keep;
  if (rc != KDLAE_OK) return -1;
  h->ws_B = B;
  h->ws_H = H;
  h->ws_W = W;
  h->ws_bytes = (int64_t)c.peak;
  return h->ws_bytes;
}

int kdlae_tt_forward(kdlae_tt_handle* h, const float* theta, const float* img, const float* rate, int B, int H, int W,
                     float* hq, float* sr, void* ws, size_t ws_bytes, void* stream) {
  if (!h || !theta || !img || !hq || !ws) return fail(KDLAE_EINVAL_CONFIG, "null argument");
  int rc = check_shape(B, H, W);
  if (rc) return rc;
  if (h->cfg.params_cat && !rate) return fail(KDLAE_EINVAL_CONFIG, "params='cat' needs denoise_rate");
  if (h->cfg.static_train && !sr) return fail(KDLAE_EINVAL_CONFIG, "static='train' needs the sr output");
  const int64_t need = kdlae_tt_workspace_bytes(h, B, H, W);
  if (need < 0 || (size_t)need > ws_bytes) return fail(KDLAE_ESTATE, "training workspace too small");
  kdlae::DeviceGuard dg(h->device);
  Ctx c;
  ctx_init(c, h, ws, ws_bytes, false, (hipStream_t)stream, B, H, W);
  c.th = theta;
  if (kdlae::debug_flag("train_trace")) c.trace = &h->trace;
  h->sv = Saved{};
  h->sv.B = B; h->sv.H = H; h->sv.W = W;
  rc = net_fwd(c, img, rate, hq, sr);
  trace_dump(h, c.s, "fwd");
  if (rc) return rc;
  h->sv.ws = ws;
  h->sv.fwd_end = c.off;
  h->sv.valid = true;
  return KDLAE_OK;
}

int kdlae_tt_backward(kdlae_tt_handle* h, const float* theta, const float* dhq, const float* dsr, float* grad, void* ws,
                      size_t ws_bytes, void* stream) {
  if (!h || !theta || !grad || !ws) return fail(KDLAE_EINVAL_CONFIG, "null argument");
  if (!h->sv.valid || h->sv.ws != ws)
    return fail(KDLAE_ESTATE, "kdlae_tt_backward needs a preceding kdlae_tt_forward on the same workspace");
  const bool has_dsr = h->cfg.static_train && dsr;
  {  // size the backward before launching anything
    Ctx d;
    ctx_init(d, h, nullptr, 0, true, nullptr, h->sv.B, h->sv.H, h->sv.W);
    d.off = h->sv.fwd_end;
    int rc = net_bwd(d, dhq, dsr, has_dsr);
    if (rc) return rc;
    if (d.peak > ws_bytes) return fail(KDLAE_ESTATE, "training workspace too small for the backward");
  }
  kdlae::DeviceGuard dg(h->device);
  Ctx c;
  ctx_init(c, h, ws, ws_bytes, false, (hipStream_t)stream, h->sv.B, h->sv.H, h->sv.W);
  c.th = theta;
  c.gr = grad;
  c.off = h->sv.fwd_end;
  if (kdlae::debug_flag("train_trace")) c.trace = &h->trace;
  int rc = use_side_stream(c, h);
  if (rc) return rc;
  hipError_t e = hipMemsetAsync(grad, 0, (size_t)h->total * sizeof(float), (hipStream_t)stream);
  if (e != hipSuccess) return fail(KDLAE_EHIP, hipGetErrorString(e));
  rc = net_bwd(c, dhq, dsr, has_dsr);
  if (rc == KDLAE_OK) rc = flush_all(c);
  if (rc != KDLAE_OK) (void)join(c);  // leave no side launch unjoined, even on an error path
  trace_dump(h, c.s, "bwd");
  return rc;
}

int kdlae_tt_backward_marked(kdlae_tt_handle* h, const float* theta, const float* dhq, const float* dsr, float* grad,
                             void* ws, size_t ws_bytes, void* stream) {
  if (!h || !theta || !grad || !ws) return fail(KDLAE_EINVAL_CONFIG, "null argument");
  if (!h->sv.valid || h->sv.ws != ws)
    return fail(KDLAE_ESTATE, "kdlae_tt_backward_marked needs a preceding kdlae_tt_forward on the same workspace");
  const bool has_dsr = h->cfg.static_train && dsr;
  const bool cached = h->mk_dsr == (int)has_dsr && h->mk_B == h->sv.B && h->mk_H == h->sv.H && h->mk_W == h->sv.W &&
                      h->mk_fwd_end == h->sv.fwd_end;
  if (!cached) {
    std::map<int64_t, std::pair<int, int>> touch;
    int nmarks = 0;
    {  // size the backward and find, per mark, which suffix of the flat buffer is final there
      Ctx d;
      ctx_init(d, h, nullptr, 0, true, nullptr, h->sv.B, h->sv.H, h->sv.W);
      d.off = h->sv.fwd_end;
      d.gr = grad;
      d.touch = &touch;
      int rc = net_bwd(d, dhq, dsr, has_dsr);
      if (rc) return rc;
      nmarks = d.cur_mark;
      h->mk_peak = d.peak;
    }
    // mark m closes the suffix [lo, total) when lo = the lowest offset written by mark m and every
    // key at or above lo is untouched (its gradient is the zero fill) or last written by mark m.
    // One pass from the end of the flat buffer: closed[m] <=> max over keys >= lo of last-write <= m
    h->mark_slot.assign(nmarks, -1);
    h->mark_lo.clear();
    h->mk_touch = touch;
    std::vector<int64_t> first_lo(nmarks, h->total);  // lowest offset first written at or before mark m
    for (const auto& kv : touch) {
      for (int m = kv.second.first; m < nmarks && kv.first < first_lo[m]; ++m) first_lo[m] = kv.first;
    }
    int64_t prev_lo = h->total;
    for (int m = 0; m < nmarks; ++m) {
      const int64_t lo = first_lo[m];
      if (lo >= prev_lo) continue;
      bool closed = true;
      for (auto it = touch.lower_bound(lo); it != touch.end(); ++it)
        if (it->second.second > m) { closed = false; break; }
      if (!closed) continue;
      h->mark_slot[m] = (int)h->mark_lo.size();
      h->mark_lo.push_back(lo);
      prev_lo = lo;
    }
    h->mk_dsr = (int)has_dsr;
    h->mk_B = h->sv.B;
    h->mk_H = h->sv.H;
    h->mk_W = h->sv.W;
    h->mk_fwd_end = h->sv.fwd_end;
  }
  if (h->mk_peak > ws_bytes) return fail(KDLAE_ESTATE, "training workspace too small for the backward");
  kdlae::DeviceGuard dg(h->device);
  while (h->mark_ev.size() < h->mark_lo.size()) {
    hipEvent_t e;
    hipError_t er = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (er != hipSuccess) return fail(KDLAE_EHIP, hipGetErrorString(er));
    h->mark_ev.push_back(e);
  }
  Ctx c;
  ctx_init(c, h, ws, ws_bytes, false, (hipStream_t)stream, h->sv.B, h->sv.H, h->sv.W);
  c.th = theta;
  c.gr = grad;
  c.off = h->sv.fwd_end;
  c.record_marks = true;
  std::map<int64_t, std::pair<int, int>> written;  // what the real run writes, checked against the marks
  c.touch = &written;
  if (kdlae::debug_flag("train_trace")) c.trace = &h->trace;
  int rc = use_side_stream(c, h);
  if (rc) return rc;
  hipError_t e = hipMemsetAsync(grad, 0, (size_t)h->total * sizeof(float), (hipStream_t)stream);
  if (e != hipSuccess) return fail(KDLAE_EHIP, hipGetErrorString(e));
  rc = net_bwd(c, dhq, dsr, has_dsr);
  if (rc == KDLAE_OK) rc = flush_all(c);
  if (rc != KDLAE_OK) (void)join(c);
  trace_dump(h, c.s, "bwd");
  if (rc) return rc;
  // every gradient the launches wrote must have been written by the dry run the marks came from, at
  // the same (first, last) marks: a write it missed, or one moved past the mark that declares its key
  // final, could be all-reduced before it lands
  if (written != h->mk_touch) {
    for (const auto& kv : written) {
      auto it = h->mk_touch.find(kv.first);
      if (it == h->mk_touch.end())
        return fail(KDLAE_ESTATE, "internal: the backward wrote gradient offset " + std::to_string(kv.first) +
                                      " that the gradient-ready marks never saw");
      if (it->second != kv.second)
        return fail(KDLAE_ESTATE, "internal: gradient offset " + std::to_string(kv.first) + " written at marks [" +
                                      std::to_string(kv.second.first) + ", " + std::to_string(kv.second.second) +
                                      "] but the marks were planned for [" + std::to_string(it->second.first) +
                                      ", " + std::to_string(it->second.second) + "]");
    }
    return fail(KDLAE_ESTATE, "internal: gradient-ready marks disagree with the keys the backward writes");
  }
  return KDLAE_OK;
}

int kdlae_tt_mark_count(const kdlae_tt_handle* h) { return h ? (int)h->mark_lo.size() : -1; }

int64_t kdlae_tt_mark_lo(const kdlae_tt_handle* h, int j) {
  return (h && j >= 0 && j < (int)h->mark_lo.size()) ? h->mark_lo[j] : -1;
}

int kdlae_tt_mark_wait(kdlae_tt_handle* h, int j, void* stream) {
  if (!h || j < 0 || j >= (int)h->mark_lo.size()) return fail(KDLAE_EPARAM, "mark index out of range");
  kdlae::DeviceGuard dg(h->device);
  hipError_t e = hipStreamWaitEvent((hipStream_t)stream, h->mark_ev[j], 0);
  return e == hipSuccess ? KDLAE_OK : fail(KDLAE_EHIP, hipGetErrorString(e));
}

int kdlae_tt_mark_sync(kdlae_tt_handle* h, int j) {
  if (!h || j < 0 || j >= (int)h->mark_lo.size()) return fail(KDLAE_EPARAM, "mark index out of range");
  kdlae::DeviceGuard dg(h->device);
  hipError_t e = hipEventSynchronize(h->mark_ev[j]);
  return e == hipSuccess ? KDLAE_OK : fail(KDLAE_EHIP, hipGetErrorString(e));
}

int64_t kdlae_train_l1sr_scratch_floats(void) { return 4 * 1024; }

int kdlae_train_l1sr(const float* pred_hq, const float* gt_hq, int64_t n_hq, const float* pred_sr, const float* gt_sr,
                     int64_t n_sr, float* dhq, float* dsr, float* loss, float* scratch, void* stream) {
  if (!pred_hq || !gt_hq || !loss || !scratch || n_hq <= 0) return fail(KDLAE_EINVAL_CONFIG, "null argument");
  hipStream_t s = (hipStream_t)stream;
  const int nb = 1024;
  float* p0 = scratch;
  float* p1 = scratch + 2 * nb;
  // L1LossSr (losses.py:159-170): 0.5 l1(hq) + 0.25 l1(sr) + 0.25 (shadow(hq) + shadow(sr))
  hipError_t e = tr::launch_l1sr(pred_hq, gt_hq, n_hq, 0.5f, dhq, p0, nb, s);
  if (e == hipSuccess && pred_sr) e = tr::launch_l1sr(pred_sr, gt_sr, n_sr, 0.25f, dsr, p1, nb, s);
  if (e == hipSuccess)
    e = tr::launch_l1sr_final(p0, nb, n_hq, 0.5f, 0.25f, pred_sr ? p1 : nullptr, pred_sr ? nb : 0, pred_sr ? n_sr : 1,
                              0.25f, 0.25f, loss, s);
  if (e != hipSuccess) return fail(KDLAE_EHIP, hipGetErrorString(e));
  return KDLAE_OK;
}

int64_t kdlae_train_adamw_scratch_floats(void) { return 2048 + 2; }

int kdlae_train_clip_adamw(float* theta, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float gscale,
                           float max_norm, float lr, float beta1, float beta2, float eps, float weight_decay, int step,
                           const int64_t* ranges, int nranges, float* scratch, void* stream) {
  if (!theta || !grad || !exp_avg || !exp_avg_sq || !scratch || n <= 0 || step < 1 || nranges < 0 ||
      (nranges > 0 && !ranges))
    return fail(KDLAE_EINVAL_CONFIG, "bad argument");
  for (int r = 0; r < nranges; ++r)
    if (ranges[2 * r] < 0 || ranges[2 * r] > ranges[2 * r + 1] || ranges[2 * r + 1] > n)
      return fail(KDLAE_EINVAL_CONFIG, "bad parameter range");
  hipStream_t s = (hipStream_t)stream;
  const int nb = 2048;
  float* state = scratch + nb;  // [0] = grad norm, [1] = applied grad scale
  // the norm covers every gradient (clip_grad_norm_ over net_g.parameters()); the update only the
  // parameters that received a gradient (torch.optim skips p.grad is None, e.g. output_param when
  // params != 'cat')
  hipError_t e = tr::launch_sumsq(grad, n, scratch, nb, s);
  if (e == hipSuccess) e = tr::launch_clip_coef(scratch, nb, gscale, max_norm, state, s);
  const int64_t whole[2] = {0, n};
  const int64_t* rg = nranges ? ranges : whole;
  for (int r = 0; r < (nranges ? nranges : 1) && e == hipSuccess; ++r) {
    const int64_t b = rg[2 * r], len = rg[2 * r + 1] - b;
    if (len > 0)
      e = tr::launch_adamw(theta + b, grad + b, exp_avg + b, exp_avg_sq + b, len, state, lr, beta1, beta2, eps,
                           weight_decay, step, s);
  }
  if (e != hipSuccess) return fail(KDLAE_EHIP, hipGetErrorString(e));
  return KDLAE_OK;
}

int kdlae_train_mixup(const float* in, float* out, int B, int64_t per_sample, const int* perm, float lam,
                      void* stream) {
  if (!in || !out || !perm || B <= 0 || per_sample <= 0 || in == out) return fail(KDLAE_EINVAL_CONFIG, "bad argument");
  hipError_t e = tr::launch_mixup(in, out, B, per_sample, perm, lam, (hipStream_t)stream);
  if (e != hipSuccess) return fail(KDLAE_EHIP, hipGetErrorString(e));
  return KDLAE_OK;
}

int kdlae_train_ema(float* ema, const float* theta, int64_t n, float decay, void* stream) {
  if (!ema || !theta || n <= 0) return fail(KDLAE_EINVAL_CONFIG, "bad argument");
  hipError_t e = tr::launch_ema(ema, theta, n, decay, (hipStream_t)stream);
  if (e != hipSuccess) return fail(KDLAE_EHIP, hipGetErrorString(e));
  return KDLAE_OK;
}

}  // extern "C"
