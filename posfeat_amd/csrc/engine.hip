// engine.hip -- whole-model extraction engine: PoSFeat.extract on gfx950.
//
// Replaces networks/PoSFeat_model.py:91-134 (PoSFeat.extract) for the
// effective extraction model (configs/train_desc.yaml:16-31):
//   ResUNet(resnet50, coarse 128, fine 128)   networks/DescNet.py:12-84
//   KeypointDet(192, 1, 'identity', 'Softplus') networks/DeteNet.py:9-121
// The host side only sequences launches on the caller's stream; every byte of
// arithmetic is in the gfx950 kernels (conv.hip, fmap.hip).  Activations live
// in one caller-provided workspace, NHWC fp32, with concat buffers laid out
// so each producer writes straight into its channel slice:
//   headcat [b][h/4][w/4][192] = [local_map(128) | local_map_small(64)]
//   cat2    [b][h/4][w/4][512] = [upconv2 out(256) | layer1 out(256)]
//   cat3    [b][h/8][w/8][1024]= [upconv3 out(512) | layer2 out(512)]
//   c1raw   [b][h/4][w/4][192] = conv1, then PReLU(IN(conv1)) in place (the
//                                 low-res map head.conv2 reads per bilinear phase)
//   g64     [b][h][w][64]      = IN(convimg)
#include <algorithm>
#include <functional>
#include <cstdio>
#include <cstring>
#include <cmath>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "common.h"
#include "fmap.h"
#include "train.h"

int pf_sample_desc(const float* fmap, int b, int c, int h, int w, int cs, const float* coord,
                   int npts, const int32_t* n_valid, int normalize, float* out, hipStream_t st);

namespace {

struct Spec {
  std::string name;
  int cout, cin, kh, kw;
  long long w_off, b_off;
};

struct SpecTable {
  std::vector<Spec> v;
  long long total = 0;
  SpecTable() {
    auto add = [&](const std::string& n, int co, int ci, int k) {
      Spec s{n, co, ci, k, k, 0, 0};
      const int kpad = posfeat_conv_packed_k(ci, k, k);
      s.w_off = total;
      total += ((long long)co * kpad + 63) / 64 * 64;
      s.b_off = total;
      total += (co + 63) / 64 * 64;
      v.push_back(s);
    };
    add("firstconv", 64, 3, 7);
    const int planes[3] = {64, 128, 256}, blocks[3] = {3, 4, 6};
    int inpl = 64;
    for (int l = 0; l < 3; ++l) {
      for (int bi = 0; bi < blocks[l]; ++bi) {
        const std::string p = "layer" + std::to_string(l + 1) + "." + std::to_string(bi);
        add(p + ".conv1", planes[l], inpl, 1);
        add(p + ".conv2", planes[l], planes[l], 3);
        add(p + ".conv3", planes[l] * 4, planes[l], 1);
        if (bi == 0) add(p + ".downsample", planes[l] * 4, inpl, 1);
        inpl = planes[l] * 4;
      }
    }
    add("conv_coarse", 128, 1024, 1);
    add("upconv3.conv", 512, 1024, 3);
    add("iconv3", 512, 1024, 3);
    add("upconv2.conv", 256, 512, 3);
    add("iconv2", 256, 512, 3);
    add("conv_fine", 128, 256, 1);
    add("head.conv1", 192, 192, 3);
    add("head.convimg", 64, 3, 3);
    add("head.conv2", 128, 256, 3);
    add("head.conv3", 1, 128, 1);
    Spec pr{"head.prelu", 1, 0, 0, 0, total, total};
    total += 64;
    v.push_back(pr);
  }
  const Spec* find(const std::string& n) const {
    for (auto& s : v)
      if (s.name == n) return &s;
    return nullptr;
  }
};

const SpecTable& specs() {
  static SpecTable t;
  return t;
}

struct Buf {
  size_t off = 0, floats = 0;
  bool persist = false;  // in the derived-weight store (posfeat_wstore), not the workspace
};

}  // namespace

// Derived weights of one weight blob (its bf16 planes; the Winograd-domain
// weights of every Winograd layer, F(4x4) and F(2x2) forms in separate
// slots), built once and shared by every extraction instance created with
// posfeat_model_create_shared from one another: an engine meeting many image
// sizes builds them once instead of once per instance, and an instance
// leaving the engine's LRU frees no device memory (hipFree synchronises the
// device).  The layout depends on the weight blob layout only, not the shape.
// Reference-counted by its instances; freed with the last.
struct posfeat_wstore {
  char* base = nullptr;  // allocated by the first forward that needs it
  size_t bytes = 0;
  const float* wts = nullptr;
  bool wsplit = false, bf6p = false;  // the layout's mode: sharers must agree
  bool wpl_done = false;
  std::set<std::string> wino_done;  // "<layer>/4" (F(4x4)) or "<layer>/2"
  hipEvent_t ev = nullptr;          // recorded after the last build
  // the side stream + fork / join events of image_branch, shared by the
  // instances: one per new shape cost a stream creation, and LRU eviction a
  // hipStreamDestroy (which waits for the stream) in the middle of a stream
  hipStream_t side_st = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  int refs = 0;
};

struct posfeat_model {
  int B, H, W;
  const float* wts;
  // layout
  size_t ws_bytes = 0;
  Buf img4, stem, headcat, t1, t2, ds, oa, ob, cat2, cat3, l3out, gmap, up3, d3, up2, d2;
  Buf c1raw, hcat, c2raw, yraw;
  Buf g64, wph, up4ws;             // phase-decomposed head.conv2 (conv.hip conv_up4_kernel)
  bool up4 = true;
  // keypoint-head training (config 5): forward keeps what the backward reads
  // (raw conv1 output, the materialised conv2 input `hcat`, per-layer IN stats)
  bool train = false;
  Buf dy3, dc2, dhcat, upt, dc1, wt2, wgws, inbws, tailws;
  // ... on the extraction path (POSFEAT_TRAINTAP=0: the materialised conv2
  // input + direct convs): conv2's upsampled part by the low-res tap GEMM,
  // its backward as the combine's adjoint D + two GEMMs on the h x w grid,
  // the image branch through the 32-channel tap image (headgrad.hip)
  bool traintap = false;
  Buf Lbuf, gram, x32, tapwT, dwtap, Aimg, imgbrws;
  Buf st_mean, st_rstd, st_part;  // instance-norm scratch (floats / doubles)
  Buf st_mean1, st_rstd1;
  Buf splitk;                      // split-K partial slabs (max over layers)
  // Winograd F(2x2,3x3) for the four decoder 3x3 convs (wino.hip): transformed
  // weights (rebuilt each forward: the blob may change between calls) + V/M
  bool wino = true;
  Buf wino_u, wino_ws;
  // head.conv2's G part as a per-image 5x5 conv of the image (gfuse.hip)
  bool gfuse = true;
  // head.conv2's upsampled part as a low-res Winograd F(4x4) conv (wino.hip)
  bool up4wino = true;
  Buf u4u, u4ws;
  // head.conv2's upsampled part with the channel mixing on the low-res grid:
  // nine 1x1 convs (one GEMM) + the interpolation/tap combine (up4tap.hip)
  bool up4tap = true;
  Buf tapw, tapP, tappart;
  bool bf6p = false;  // conv precision mode 2 (pre-split Winograd / tap GEMM operands)
  // bf16x6 with pre-split weights (conv_bf6b_kernel, the default in mode 1;
  // POSFEAT_BF6B=0 off): the weight blob is split into three bf16 planes at
  // the start of every forward, Winograd U and the tap weights as planes
  bool wsplit = false;
  Buf wpl;
  // each stage's first bottleneck: conv3 + downsample as one two-source GEMM
  // (pf_conv_dual) on [cout][k1 + k2] planes + summed biases built with wpl
  // (A/B: POSFEAT_DSFUSE=0 -- the downsample conv, then conv3 with it as residual)
  bool dsfuse = false;
  Buf dsw;
  // head.conv2's tap GEMM + combine in chunks of hchunk images reusing one P
  // slab (A/B: POSFEAT_HEAD_CHUNK=G; 0 = the whole batch per launch)
  int hchunk = 0;
  // head.conv1's IN + PReLU applied inside the tap GEMM's A loads (conv1's raw
  // output read directly; A/B only, POSFEAT_NPFUSE=1: the tap GEMM slower by
  // more than in_apply costs)
  bool npfuse = false;
  // head.conv1's IN statistics from its F(6x6) output transform (A/B:
  // POSFEAT_W6STATS=0 -- a statistics pass over conv1's output)
  bool w6stats = true;
  // conv_fine's epilogue writes local_map NCHW too (A/B only,
  // POSFEAT_NCHWSINK=1: measured even with the layout pass)
  bool nchwsink = false;
  // head.conv2's tap GEMM on the weight-stationary persistent kernel
  // (pf_tap_gemm_ws; A/B: POSFEAT_TAPWS=0 -- the tuned bf6x tile)
  bool tapws = false;
  // the short-K dense 1x1 convs on the same kernel (pf_gemm_ws): by default
  // (3) only where it measured faster than the tuned tiles, layer1's K = 256,
  // N = 64 conv1 (0.20 -> 0.18 ms at B = 32; conv3 with its residual and the
  // N = 128 / 1024 convs slower). A/B: POSFEAT_WS1X1=1 every
  // instantiated shape, 2 those without a residual, 0 none
  int ws1x1 = 0;
  // the stem on it too (pf_gemm_ws_stem, the G4 gather; A/B only,
  // POSFEAT_WSSTEM=1: bit-identical, but 0.447 -> 0.557 ms at B = 32, r16zs)
  bool wsstem = false;
  bool tapb = false;  // bf16x6 tap GEMM on pre-split planes (POSFEAT_BF6=2)
  Buf tapwb, tapLb;
  Buf gf_w, gf_b, gf_wp;
  // the G part computed inside the tap combine (up4tap_gcombine_kernel; the
  // default with bf16x6 and the tap form, POSFEAT_HEADFUSE=0 off): no G pass
  // over y, the border ring's G values in their own small buffer
  bool hfuse = false;
  Buf gring;
  // convimg's IN statistics from the image's tap moments instead of running
  // convimg (gfuse.hip): the full-res 64-channel map is never computed
  bool imgstats = true;
  Buf imws;
  size_t splitk_need = 0;
  // the image branch of KeypointDet (convimg + its IN statistics + the folded
  // G part of head.conv2 + head.conv2's weight transforms) depends on the
  // image only: it runs on a second stream, overlapping the ResUNet, and
  // joins before head.conv2's border/upsampled part (POSFEAT_SIDE=0: serial).
  // Set in plan() before the dry pass so the planning forward follows the
  // path that actually runs.
  bool side = false;
  int side_at = 0;
  unsigned tuned_modes = 0;  // bit per Mode: its first forward (autotune) ran, serially
  hipStream_t side_st = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  Buf splitk2;  // the side stream's own split-K / statistics scratch
  // per-layer conv tile chosen by timing the legal candidates on the first
  // forward of this shape (results do not depend on the tile)
  std::map<std::string, int> tuned;
  bool autotune = true;
  // derived weights (the blob's bf16 planes, the Winograd U) of an
  // extraction instance live in a store (posfeat_wstore) it may share with
  // the other instances of its engine, allocated by the first forward and
  // built once: by the first forward that needs them, again after
  // posfeat_model_weights_changed (training instances rebuild them every
  // forward in their workspace: their weights move every step)
  bool wcache = false;
  posfeat_wstore* store = nullptr;
  size_t p_bytes = 0;
  size_t wino_u_f2 = 0;        // floats: the F(2x2) slots after the F(4x4) ones
  size_t wino_u_f6 = 0;        // floats: the F(6x6) slots after those
  bool wino6 = true;           // F(6x6) for the decoder + head.conv1 (POSFEAT_WINO6=0: F(4x4))
  bool wprep_pending = false;  // built this forward: record the store's event at its end
  // timing
  bool timing = false;
  struct Ev {
    std::string label;
    double flops;
    int arith = 0;  // PF_ARITH_* mask of the label's MFMA launches
    hipEvent_t a, b;
  };
  std::vector<Ev> evs;
  size_t ev_used = 0;
};

namespace {

struct Ctx {
  posfeat_model* m;
  char* ws;
  hipStream_t st;
  bool dry = false;  // planning pass: record scratch needs, launch nothing
  bool side = false;  // running on the model's side stream (own scratch)
  char* base(const Buf& b) const { return (b.persist ? m->store->base : ws) + b.off; }
  float* f(const Buf& b) const { return reinterpret_cast<float*>(base(b)); }
  double* d(const Buf& b) const { return reinterpret_cast<double*>(base(b)); }
  const float* W(const std::string& n) const { return m->wts + specs().find(n)->w_off; }
  // the bf16 planes of blob weights w (posfeat_model::wsplit), else nothing
  void wplanes_of(const float* w, const unsigned short** wb, long long* wplane) const;
  const float* Bi(const std::string& n) const { return m->wts + specs().find(n)->b_off; }
};

void Ctx::wplanes_of(const float* w, const unsigned short** wb, long long* wplane) const {
  *wb = nullptr;
  *wplane = 0;
  const long long total = specs().total;
  if (!m->wsplit || w < m->wts || w >= m->wts + total) return;
  *wb = reinterpret_cast<const unsigned short*>(base(m->wpl)) + (w - m->wts);
  *wplane = total;
}

// record-and-run helper for optional per-launch timing
template <class F>
int timed(Ctx& c, const std::string& label, double flops, F&& fn) {
  posfeat_model* m = c.m;
  if (c.dry) return POSFEAT_OK;
  if (!m->timing) return fn();
  if (m->ev_used == m->evs.size()) {
    posfeat_model::Ev e;
    if (hipEventCreate(&e.a) != hipSuccess || hipEventCreate(&e.b) != hipSuccess)
      return POSFEAT_E_HIP;
    m->evs.push_back(e);
  }
  auto& e = m->evs[m->ev_used++];
  // side-stream launches overlap the main stream: keep them out of the
  // main-stream prefixes ("conv:", "head.conv2", ...) the bench sums
  e.label = c.side ? "side:" + label : label;
  e.flops = flops;
  if (hipEventRecord(e.a, c.st) != hipSuccess) return POSFEAT_E_HIP;
  const int outer = pf_arith_mask();  // (labels may nest)
  pf_arith_mask() = 0;
  const int r = fn();
  e.arith = pf_arith_mask();
  pf_arith_mask() = outer | e.arith;
  if (hipEventRecord(e.b, c.st) != hipSuccess) return POSFEAT_E_HIP;
  return r;
}

// Time each legal tile for this conv (1 warm-up + 3 timed launches on the
// layer's real inputs) and return the fastest; -1 (default plan) if only one.
template <class Run>
int tune(const std::string& name, const posfeat_conv_desc& d, hipStream_t st, Run&& run,
         bool wplanes) {
  static const bool log = [] {
    const char* e = getenv("POSFEAT_AUTOTUNE_LOG");
    return e && e[0] == '1';
  }();
  int cand[16];
  const int nc = pf_conv_candidates(&d, cand, 16, wplanes);
  if (nc <= 1) return -1;
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return -1;
  if (hipEventCreate(&e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    return -1;
  }
  int best = -1;
  float best_ms = 1e30f;
  for (int i = 0; i < nc; ++i) {
    if (run(cand[i]) != POSFEAT_OK) continue;  // e.g. stats unsupported for this tile
    if (hipEventRecord(e0, st) != hipSuccess) break;
    bool ok = true;
    for (int r = 0; r < 3 && ok; ++r) ok = run(cand[i]) == POSFEAT_OK;
    float ms = 0.f;
    if (!ok || hipEventRecord(e1, st) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
        hipEventElapsedTime(&ms, e0, e1) != hipSuccess)
      continue;
    if (log) fprintf(stderr, "[autotune] %-24s tile %2d  %8.4f ms\n", name.c_str(), cand[i], ms / 3);
    if (ms < best_ms) {
      best_ms = ms;
      best = cand[i];
    }
  }
  if (log) fprintf(stderr, "[autotune] %-24s -> tile %d\n", name.c_str(), best);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return best;
}

// Process-wide tile choices, keyed by the conv's full descriptor (and
// whether a residual is read): a new instance -- another batch size or image
// size, or a new engine -- times only the convs it has not met before.  A conv
// met before with the same class (everything but n, h, w) and a GEMM M
// (= n * oh * ow) within 25 % reuses that tile without timing (HPatches and
// Aachen images come in many sizes; POSFEAT_TUNE_SIMILAR=0 turns this off).
// An extraction conv's candidates share one arithmetic, so its results never
// depend on the tile; the training step's direct convs do (pf_conv_tuned_run).
struct TileCache {
  std::mutex mu;
  std::map<std::string, int> exact;
  std::map<std::string, std::vector<std::pair<double, int>>> by_class;  // (M, tile)
};
TileCache& tile_cache() {
  static TileCache t;
  return t;
}
std::string desc_class(const posfeat_conv_desc& d, bool res, bool wplanes) {
  char b[160];
  // the calling thread's tile scope too (PfDense32Scope / PfHaloFp32Scope
  // change the legal candidates: a training instance's choice must not be
  // reused by an extraction engine)
  snprintf(b, sizeof b, "%d/%d/%d/%dx%d/s%d/p%d/%d/%d/a%d/r%d/P%d%s/x%d%d", d.cin, d.x_cstride,
           d.cout, d.kh, d.kw, d.stride, d.pad, d.y_cstride, d.res_cstride, d.act, res ? 1 : 0,
           pf_conv_precision(), wplanes ? "B" : "", pf_bf6x_on() ? 1 : 0, pf_halo_bf6_on() ? 1 : 0);
  return b;
}
double desc_m(const posfeat_conv_desc& d) {
  const int oh = (d.h + 2 * d.pad - d.kh) / d.stride + 1, ow = (d.w + 2 * d.pad - d.kw) / d.stride + 1;
  return (double)d.n * oh * ow;
}
bool tile_lookup(const posfeat_conv_desc& d, bool res, bool wplanes, int* tile,
                 bool exact_only = false) {
  static const bool similar = [] {
    const char* e = pf_ab_getenv("POSFEAT_TUNE_SIMILAR");
    return !(e && e[0] == '0');
  }();
  const std::string cls = desc_class(d, res, wplanes);
  char nhw[48];
  snprintf(nhw, sizeof nhw, "|%d/%d/%d", d.n, d.h, d.w);
  TileCache& t = tile_cache();
  std::lock_guard<std::mutex> g(t.mu);
  auto it = t.exact.find(cls + nhw);
  if (it != t.exact.end()) {
    // an imported entry (records/tile_db.txt, tuned on another machine or
    // build) must still be a legal candidate here
    if (it->second >= 0) {
      int cand[16];
      const int nc = pf_conv_candidates(&d, cand, 16, wplanes);
      if (std::find(cand, cand + nc, it->second) == cand + nc) return false;
    }
    *tile = it->second;
    return true;
  }
  if (!similar || exact_only) return false;
  auto ct = t.by_class.find(cls);
  if (ct == t.by_class.end()) return false;
  const double m = desc_m(d);
  double best = 1e30;
  int bt = -2;
  for (auto& e : ct->second) {
    const double r = std::fabs(std::log(e.first / m));
    if (r < best) {
      best = r;
      bt = e.second;
    }
  }
  if (best > std::log(1.25)) return false;
  if (bt >= 0) {  // the tile must be legal for this shape too
    int cand[16];
    const int nc = pf_conv_candidates(&d, cand, 16, wplanes);
    if (std::find(cand, cand + nc, bt) == cand + nc) return false;
  }
  *tile = bt;
  return true;
}
void tile_store(const posfeat_conv_desc& d, bool res, bool wplanes, int tile) {
  const std::string cls = desc_class(d, res, wplanes);
  char nhw[48];
  snprintf(nhw, sizeof nhw, "|%d/%d/%d", d.n, d.h, d.w);
  TileCache& t = tile_cache();
  std::lock_guard<std::mutex> g(t.mu);
  if (t.exact.emplace(cls + nhw, tile).second) t.by_class[cls].push_back({desc_m(d), tile});
}

// The process-wide tile choices as text, one "<class>|<n>/<h>/<w> <tile>"
// line per entry (posfeat_tile_cache_export), and back
// (posfeat_tile_cache_import): a tuning database the caller keeps between
// processes, so a stream of image sizes is not timed conv by conv again
// (managers/extractor.py: records/tile_db.txt).  The similar-shape reuse then
// covers every shape within 25 % of a stored M.
std::string tile_cache_text() {
  TileCache& t = tile_cache();
  std::lock_guard<std::mutex> g(t.mu);
  std::string out;
  for (auto& e : t.exact) out += e.first + " " + std::to_string(e.second) + "\n";
  return out;
}
int tile_cache_load(const char* text) {
  int n = 0;
  const char* p = text;
  while (p && *p) {
    const char* eol = strchr(p, '\n');
    const std::string line(p, eol ? eol - p : strlen(p));
    p = eol ? eol + 1 : nullptr;
    const size_t sp = line.rfind(' '), bar = line.rfind('|');
    if (sp == std::string::npos || bar == std::string::npos || bar > sp) continue;
    int nn, hh, ww;
    if (sscanf(line.c_str() + bar + 1, "%d/%d/%d", &nn, &hh, &ww) != 3) continue;
    const std::string key = line.substr(0, sp), cls = line.substr(0, bar);
    const int tile = atoi(line.c_str() + sp + 1);
    // M of the entry from its class's kernel and stride: (h + 2p - k) / s + 1 per side
    int kh = 1, kw = 1, st = 1, pad = 0;
    if (sscanf(cls.c_str(), "%*d/%*d/%*d/%dx%d/s%d/p%d", &kh, &kw, &st, &pad) != 4) continue;
    const double m = (double)nn * ((hh + 2 * pad - kh) / st + 1) * ((ww + 2 * pad - kw) / st + 1);
    TileCache& t = tile_cache();
    std::lock_guard<std::mutex> g(t.mu);
    if (t.exact.emplace(key, tile).second) {
      t.by_class[cls].push_back({m, tile});
      ++n;
    }
  }
  return n;
}

// run (autotuned on the first forward of the instance, keyed by `key`) one
// conv described by d with packed weights w
// wb / wplane: the weights' bf16 planes (default: w's planes in the
// per-forward split of the weight blob, when w lies in the blob)
int conv_desc_run(Ctx& c, const std::string& key, const posfeat_conv_desc& d, const float* x,
                  const float* w, const float* bias, const float* res, float* y, double flops,
                  const unsigned short* wb = nullptr, long long wplane = 0) {
  const size_t need = posfeat_conv2d_workspace(&d);
  if (c.dry) {
    if (need > c.m->splitk_need) c.m->splitk_need = need;
    return POSFEAT_OK;
  }
  if (!wb) c.wplanes_of(w, &wb, &wplane);
  const Buf& sk = c.side ? c.m->splitk2 : c.m->splitk;
  float* part = c.f(sk);
  const size_t have = sk.floats * sizeof(float);
  auto run = [&](int tile) {
    return pf_conv_run_tile(&d, x, w, bias, res, y, part, have, tile, c.st, wb, wplane);
  };
  const bool wp = wb != nullptr;
  int tile = -1;
  auto it = c.m->tuned.find(key);
  if (it != c.m->tuned.end()) {
    tile = it->second;
  } else if (c.m->autotune) {
    if (!tile_lookup(d, res != nullptr, wp, &tile)) {
      tile = tune(key, d, c.st, run, wp);
      tile_store(d, res != nullptr, wp, tile);
    }
    c.m->tuned[key] = tile;
  }
  return timed(c, "conv:" + key, flops, [&] { return run(tile); });
}

int conv(Ctx& c, const std::string& name, const float* x, int n, int h, int w, int xcs, float* y,
         int ycs, int stride, int act, const float* res = nullptr, int rcs = 0) {
  const Spec* s = specs().find(name);
  if (!s) return POSFEAT_E_INVALID;
  posfeat_conv_desc d;
  d.n = n;
  d.h = h;
  d.w = w;
  d.cin = (s->cin + 3) / 4 * 4;
  d.x_cstride = xcs;
  d.cout = s->cout;
  d.kh = s->kh;
  d.kw = s->kw;
  d.stride = stride;
  d.pad = (s->kh - 1) / 2;
  d.y_cstride = ycs;
  d.res_cstride = rcs;
  d.act = act;
  const int oh = (h + 2 * d.pad - d.kh) / stride + 1, ow = (w + 2 * d.pad - d.kw) / stride + 1;
  const double flops = 2.0 * n * oh * ow * (double)s->cout * s->cin * s->kh * s->kw;
  // a short-K 1x1 conv: the weight-stationary GEMM (its three planes resident
  // in LDS, A streamed once per column tile; the bf6x tile's six terms in the
  // same order). Not under conv_fine's NCHW sink (the tile epilogue's)
  if (c.m->wsstem && !c.dry && s->kh == 7 && s->kw == 7 && d.cin == 4 && xcs == 4 &&
      s->cout == 64 && pf_bf6x_on()) {
    const unsigned short* wb = nullptr;
    long long wplane = 0;
    c.wplanes_of(c.W(name), &wb, &wplane);
    if (wb)
      return timed(c, "conv:" + name, flops, [&] {
        return pf_gemm_ws_stem(x, n, h, w, oh, ow, stride, d.pad, wb, wplane,
                               (d.kh * d.kw * 4 + 31) / 32 * 32, s->cout, c.Bi(name), act, y, ycs,
                               c.st);
      });
  }
  const int wsm = c.m->ws1x1;
  if (wsm && !(wsm >= 2 && res) && !(wsm == 3 && s->cout != 64) && !c.dry && s->kh == 1 && s->kw == 1 && stride == 1 && s->cin % 32 == 0 &&
      pf_bf6x_on() && pf_ws_gemm_ok(s->cin, s->cout) && !(c.m->nchwsink && name == "conv_fine")) {
    const unsigned short* wb = nullptr;
    long long wplane = 0;
    c.wplanes_of(c.W(name), &wb, &wplane);
    // (pf_gemm_ws's operand alignment: else the tiles)
    if (wb && wplane % 8 == 0 && xcs % 4 == 0 &&
        ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(wb)) & 15) == 0)
      return timed(c, "conv:" + name, flops, [&] {
        return pf_gemm_ws(x, xcs, n * h * w, s->cin, wb, wplane, s->cout, c.Bi(name), res, rcs,
                          act, y, ycs, c.st);
      });
  }
  return conv_desc_run(c, name, d, x, c.W(name), c.Bi(name), res, y, flops);
}

int head_forward(Ctx& c, float* img4, float* local_point, bool side);

// what one forward computes: PoSFeat.extract (ResUNet + KeypointDet),
// ResUNet.forward alone (DescNet.py:64-84), or KeypointDet.forward([x, img])
// alone (DeteNet.py:102-121) with x = cat[local_map, local_map_small] given
enum Mode { MODE_FULL = 0, MODE_BACKBONE = 1, MODE_HEAD = 2 };
int forward(Ctx& c, const float* img, posfeat_extract_out* out, int mode = MODE_FULL,
            const float* xhead = nullptr);

// The decoder's 3x3 stride-1 convs (DescNet.py:41-45) through Winograd
// F(4x4,3x3) / F(2x2,3x3) when enabled (default; POSFEAT_WINO=0 for the
// direct conv); then (POSFEAT_WINO_ENC, below) the encoder's stride-1 bottleneck
// conv2 layers, with their resolution divisor
const char* const kWinoLayers[16] = {"upconv3.conv", "iconv3",          "upconv2.conv",
                                     "iconv2",       "head.conv1",      "layer1.0.conv2",
                                     "layer1.1.conv2", "layer1.2.conv2", "layer2.1.conv2",
                                     "layer2.2.conv2", "layer2.3.conv2", "layer3.1.conv2",
                                     "layer3.2.conv2", "layer3.3.conv2", "layer3.4.conv2",
                                     "layer3.5.conv2"};
const int kWinoDiv[16] = {8, 8, 4, 4, 4, 4, 4, 4, 8, 8, 8, 16, 16, 16, 16, 16};
// Which encoder stages take Winograd (POSFEAT_WINO_ENC: "0" none, "1" all,
// else the stage digits; default "23").  Measured per layer (r5f, halo bf16x6
// tiles vs Winograd, B = 32 / 8): layer2 conv2 0.275 -> 0.24 / 0.111 -> 0.091
// ms (F(4x4) at 60x80), layer3 0.45 -> 0.36 / 0.125 -> 0.113 ms (F(2x2) at
// 30x40, whose halo tiles underfill), but layer1 0.333 -> 0.40 / 0.099 -> 0.13
// (its K = 64 GEMMs are too short for the transform round trip to pay)
unsigned wino_enc_mask() {
  static const unsigned mask = [] {
    const char* e = pf_ab_getenv("POSFEAT_WINO_ENC");
    if (!e) return 6u;
    if (e[0] == '1' && e[1] == 0) return 7u;
    unsigned m = 0;
    for (const char* q = e; *q; ++q)
      if (*q >= '1' && *q <= '3') m |= 1u << (*q - '1');
    return m;
  }();
  return mask;
}
bool wino_enc_on() { return wino_enc_mask() != 0; }
// `p`: the bottleneck prefix "layer<k>.<block>"
bool wino_enc_layer(const std::string& p) {
  return p.size() > 5 && p[5] >= '1' && p[5] <= '3' && ((wino_enc_mask() >> (p[5] - '1')) & 1u);
}

long long wino_u_offset(const std::string& name, bool planes) {
  long long off = 0;
  for (const char* n : kWinoLayers) {
    if (name == n) return off;
    const Spec* s = specs().find(n);
    off += (long long)(planes ? 54 : 36) * s->cout * s->cin;  // bf16x6: three planes
  }
  return -1;
}

// F(6x6) (1.27x fewer transform-domain MACs and 0.79x the V / M bytes of
// F(4x4); 2.25x fewer than F(2x2), which layer3's 30x40 maps took) for the
// decoder + head.conv1 and the encoder stages in POSFEAT_WINO6_ENC (A/B
// build; default "23": layer2 / layer3 conv2)
unsigned wino6_enc_mask() {
  static const unsigned mask = [] {
    const char* e = pf_ab_getenv("POSFEAT_WINO6_ENC");
    if (!e) return 6u;
    unsigned m = 0;
    for (const char* q = e; *q; ++q)
      if (*q >= '1' && *q <= '3') m |= 1u << (*q - '1');
    return m;
  }();
  return mask;
}
constexpr int kWino6Layers = 16;  // slots for every kWinoLayers entry
long long wino6_u_offset(const std::string& name, bool planes) {
  long long off = 0;
  for (int i = 0; i < kWino6Layers; ++i) {
    if (name == kWinoLayers[i]) {
      if (i >= 5 && !((wino6_enc_mask() >> (name[5] - '1')) & 1u)) return -1;
      return off;
    }
    const Spec* s = specs().find(kWinoLayers[i]);
    off += (long long)pf_wino6_weights_floats(s->cin, s->cout, planes);
  }
  return -1;
}

// up2: x is the (h/2, w/2) map and the conv input its x2 align_corners
// upsample (DescNet.py:182-190 upconv), interpolated inside the F(4x4)
// input transform (POSFEAT_UP2FUSE=0: materialised by the upsample kernel);
// xup: the full-res buffer for the unfused forms
bool up2fuse_on() {
  static const bool on = [] {
    const char* e = pf_ab_getenv("POSFEAT_UP2FUSE");
    return !(e && e[0] == '0');
  }();
  return on;
}

// stats (act none, F(6x6) only): the output transform also writes the
// instance-norm partials of y (pf_wino6_conv); *stats_done says whether it did
int conv3x3(Ctx& c, const std::string& name, const float* x, int n, int h, int w, int xcs, float* y,
            int ycs, int act, int up2 = 0, float* xup = nullptr, double* stats = nullptr,
            bool* stats_done = nullptr) {
  posfeat_model* m = c.m;
  if (stats_done) *stats_done = false;
  const long long uo6 = wino6_u_offset(name, m->wsplit);
  if (m->wino && m->wino6 && !m->bf6p && uo6 >= 0 && (!up2 || up2fuse_on())) {
    const Spec* s = specs().find(name);
    if (c.dry) return POSFEAT_OK;
    if (stats && (act != POSFEAT_ACT_NONE || s->cout % 64)) stats = nullptr;
    if (stats_done) *stats_done = stats != nullptr;
    float* U = c.f(m->wino_u) + m->wino_u_f6 + uo6;
    const std::string ukey = name + "/6";
    if (!(m->wcache && m->store && m->store->wino_done.count(ukey))) {
      PF_TRY(timed(c, "wino:weights", 0, [&] {
        return pf_wino6_weights(c.W(name), s->cout, s->cin, U, c.st, m->wsplit);
      }));
      if (m->wcache) {
        m->store->wino_done.insert(ukey);
        m->wprep_pending = true;
      }
    }
    const double T = (double)n * ((h + 5) / 6) * ((w + 5) / 6);
    auto stage = [&](int st_bits) {
      return pf_wino6_conv(x, xcs, n, h, w, s->cin, U, c.Bi(name), s->cout, act, y, ycs,
                           c.f(m->wino_ws), m->wino_ws.floats * sizeof(float), c.st, st_bits,
                           m->wsplit ? 1 : 0, up2, nullptr, (st_bits & 4) ? stats : nullptr);
    };
    PF_TRY(timed(c, "wino:in:" + name, 0, [&] { return stage(1); }));
    PF_TRY(timed(c, "conv:" + name + ".wino", 2.0 * T * 64 * s->cin * s->cout,
                 [&] { return stage(2); }));
    return timed(c, "wino:out:" + name, 0, [&] { return stage(4); });
  }
  const long long uo = wino_u_offset(name, m->bf6p || m->wsplit);
  const bool f4ok = m->wino && uo >= 0 && h % 4 == 0 && w % 4 == 0 &&
                    !(pf_ab_getenv("POSFEAT_WINO") && pf_ab_getenv("POSFEAT_WINO")[0] == '1');
  if (up2 && !(f4ok && up2fuse_on())) {  // materialise the upsample, then the plain conv
    PF_TRY(timed(c, "upsample2x", 0, [&] {
      return pf_upsample2x_ac(x, n, h / 2, w / 2, xcs, xcs, xup, xcs, c.st);
    }));
    return conv3x3(c, name, xup, n, h, w, xcs, y, ycs, act);
  }
  if (!m->wino || uo < 0 || (h & 1) || (w & 1))
    return conv(c, name, x, n, h, w, xcs, y, ycs, 1, act);
  const Spec* s = specs().find(name);
  if (c.dry) return POSFEAT_OK;
  // executed transform-domain MACs: F(4x4) 36 per 4x4 tile, F(2x2) 16 per 2x2 tile
  const bool f4 = h % 4 == 0 && w % 4 == 0 && !(pf_ab_getenv("POSFEAT_WINO") && pf_ab_getenv("POSFEAT_WINO")[0] == '1');
  // the cached U of this layer in its F(4x4) or F(2x2) slot
  float* U = c.f(m->wino_u) + uo + (f4 ? 0 : m->wino_u_f2);
  const std::string ukey = name + (f4 ? "/4" : "/2");
  if (!(m->wcache && m->store && m->store->wino_done.count(ukey))) {
    PF_TRY(timed(c, "wino:weights", 0,
                 [&] {
                   return pf_wino_weights_hw(c.W(name), s->cout, s->cin, h, w, U, c.st,
                                             m->bf6p || m->wsplit);
                 }));
    if (!c.dry && m->wcache) {
      m->store->wino_done.insert(ukey);
      m->wprep_pending = true;
    }
  }
  const double T = f4 ? (double)n * (h / 4) * (w / 4) : (double)n * (h / 2) * (w / 2);
  // three launches, timed apart: the input transform, the batched GEMMs
  // (the MFMA work), the output transform (+ bias, activation)
  auto stage = [&](int st_bits) {
    return pf_wino_conv(x, xcs, n, h, w, s->cin, U, c.Bi(name), s->cout, act, y, ycs,
                        c.f(m->wino_ws), m->wino_ws.floats * sizeof(float), c.st, st_bits,
                        m->bf6p ? 2 : m->wsplit ? 1 : 0, up2);
  };
  PF_TRY(timed(c, "wino:in:" + name, 0, [&] { return stage(1); }));
  PF_TRY(timed(c, "conv:" + name + ".wino", 2.0 * T * (f4 ? 36 : 16) * s->cin * s->cout,
               [&] { return stage(2); }));
  return timed(c, "wino:out:" + name, 0, [&] { return stage(4); });
}

// conv whose epilogue also produces the InstanceNorm mean/rstd of its output
// (falls back to a separate statistics pass when a tile could span >2 images)
int conv_in(Ctx& c, const std::string& name, const float* x, int n, int h, int w, int xcs,
            float* y, int ycs, float* mean, float* rstd) {
  const Spec* s = specs().find(name);
  if (!s) return POSFEAT_E_INVALID;
  posfeat_conv_desc d;
  d.n = n;
  d.h = h;
  d.w = w;
  d.cin = (s->cin + 3) / 4 * 4;
  d.x_cstride = xcs;
  d.cout = s->cout;
  d.kh = s->kh;
  d.kw = s->kw;
  d.stride = 1;
  d.pad = (s->kh - 1) / 2;
  d.y_cstride = ycs;
  d.res_cstride = 0;
  d.act = POSFEAT_ACT_NONE;
  const size_t need = pf_conv_stats_ws_max(&d);
  if (need == 0 || c.dry) {
    if (c.dry) {
      if (need > c.m->splitk_need) c.m->splitk_need = need;
      return POSFEAT_OK;
    }
    PF_TRY(conv(c, name, x, n, h, w, xcs, y, ycs, 1, POSFEAT_ACT_NONE));
    return timed(c, "instnorm", 0, [&] {
      return pf_in_stats(y, n, h * w, s->cout, ycs, mean, rstd,
                         c.side ? c.d(c.m->splitk2) : c.d(c.m->st_part), c.st);
    });
  }
  const double flops = 2.0 * n * h * w * (double)s->cout * s->cin * s->kh * s->kw;
  const Buf& sk = c.side ? c.m->splitk2 : c.m->splitk;
  float* part = c.f(sk);
  const size_t have = sk.floats * sizeof(float);
  // No autotuning here: the fused statistics are per-tile partial sums, so a
  // different tile would change mean/rstd in the last bits and make results
  // depend on a timing race.  The default plan is the tuned winner for these
  // layers anyway (profiles/r01/autotune_choices_b8_480x640.txt).
  const unsigned short* wb = nullptr;
  long long wplane = 0;
  c.wplanes_of(c.W(name), &wb, &wplane);
  return timed(c, "conv:" + name, flops, [&] {
    return pf_conv_stats_run_tile(&d, x, c.W(name), c.Bi(name), y, part, have, mean, rstd, 1e-5f,
                                  -1, c.st, wb, wplane);
  });
}

// input-gradient conv of head.conv2: d(conv2 out) (128 ch) -> d(cat) (256 ch)
posfeat_conv_desc dgrad_desc(const posfeat_model* m) {
  posfeat_conv_desc d;
  d.n = m->B;
  d.h = m->H;
  d.w = m->W;
  d.cin = 128;
  d.x_cstride = 128;
  d.cout = 256;
  d.kh = d.kw = 3;
  d.stride = 1;
  d.pad = 1;
  d.y_cstride = 256;
  d.res_cstride = 0;
  d.act = POSFEAT_ACT_NONE;
  return d;
}

// dL/dL-map of head.conv2's upsampled part: D (1152 ch) x WtT^T -> 192 ch, 1x1
posfeat_conv_desc dl_desc(const posfeat_model* m) {
  posfeat_conv_desc d;
  d.n = m->B;
  d.h = m->H / 4;
  d.w = m->W / 4;
  d.cin = 9 * 128;
  d.x_cstride = 9 * 128;
  d.cout = 192;
  d.kh = d.kw = 1;
  d.stride = 1;
  d.pad = 0;
  d.y_cstride = 192;
  d.res_cstride = 0;
  d.act = POSFEAT_ACT_NONE;
  return d;
}

// the fused conv3 + downsample weights of stage l (dsw): planes at u16 offset
// off, then the summed biases at float offset boff
struct DualLayout {
  int cout, k1, k2;
  size_t off, boff;
};
DualLayout dual_layout(int l) {
  const int planes[3] = {64, 128, 256}, inpl[3] = {64, 256, 512};
  size_t off = 0;
  DualLayout d{};
  for (int i = 0; i <= l; ++i) {
    d.cout = planes[i] * 4;
    d.k1 = planes[i];
    d.k2 = inpl[i];
    d.off = off;
    off += pf_align((size_t)3 * d.cout * (d.k1 + d.k2) * 2, 256) / 2;
    d.boff = off / 2;
    off += pf_align((size_t)d.cout * 4, 256) / 2;
  }
  return d;
}
size_t dual_floats() {
  const DualLayout d = dual_layout(2);
  return d.boff + pf_align((size_t)d.cout * 4, 256) / 4;
}

void plan(posfeat_model* m) {
  size_t cur = 0, pcur = 0;
  auto alloc = [&](Buf& b, size_t floats, size_t elem = 4) {
    b.off = cur;
    b.floats = floats;
    b.persist = false;
    cur += pf_align(floats * elem, 256);
  };
  // derived weights: the instance's own memory when they are cached
  auto palloc = [&](Buf& b, size_t floats) {
    if (!m->wcache) return alloc(b, floats);
    b.off = pcur;
    b.floats = floats;
    b.persist = true;
    pcur += pf_align(floats * 4, 256);
  };
  const size_t B = m->B, H = m->H, W = m->W;
  const size_t h2 = H / 2, w2 = W / 2, h4 = H / 4, w4 = W / 4, h8 = H / 8, w8 = W / 8,
               h16 = H / 16, w16 = W / 16;
  alloc(m->img4, B * H * W * 4);
  alloc(m->stem, B * h2 * w2 * 64);
  alloc(m->headcat, B * h4 * w4 * 192);
  alloc(m->t1, B * h4 * w4 * 256);
  alloc(m->t2, B * h4 * w4 * 256);
  alloc(m->ds, B * h4 * w4 * 256);
  alloc(m->oa, B * h4 * w4 * 256);
  alloc(m->ob, B * h4 * w4 * 256);
  alloc(m->cat2, B * h4 * w4 * 512);
  alloc(m->cat3, B * h8 * w8 * 1024);
  alloc(m->l3out, B * h16 * w16 * 1024);
  alloc(m->gmap, B * h16 * w16 * 128);
  alloc(m->up3, B * h8 * w8 * 1024);
  alloc(m->d3, B * h8 * w8 * 512);
  alloc(m->up2, B * h4 * w4 * 512);
  alloc(m->d2, B * h4 * w4 * 256);
  alloc(m->c1raw, B * h4 * w4 * 192);
  {
    const char* e = pf_ab_getenv("POSFEAT_HEAD_UP4");  // 0: materialise the x4 upsample (A/B only)
    m->up4 = !(e && e[0] == '0');
    const char* t = getenv("POSFEAT_AUTOTUNE");  // 0: heuristic tiles only
    m->autotune = !(t && t[0] == '0');
    const char* wv = pf_ab_getenv("POSFEAT_WINO");  // 0: direct conv for the decoder 3x3 layers
    m->wino = !(wv && wv[0] == '0');
    const char* w6 = pf_ab_getenv("POSFEAT_WINO6");  // 0: F(4x4) for the decoder / head.conv1
    m->wino6 = !(w6 && w6[0] == '0') && !(wv && wv[0] == '1');
    const char* gv = pf_ab_getenv("POSFEAT_GFUSE");  // 0: conv2's G part as the 64-ch 3x3 conv
    m->gfuse = !(gv && gv[0] == '0');
    const char* uv = pf_ab_getenv("POSFEAT_UP4WINO");  // 0: conv_up4_kernel (bilinear phases)
    m->up4wino = !(uv && uv[0] == '0') && H % 16 == 0 && W % 16 == 0;
    const char* tv = pf_ab_getenv("POSFEAT_UP4TAP");  // 0: the low-res Winograd / phase forms
    m->up4tap = !(tv && tv[0] == '0') && H % 16 == 0 && W % 16 == 0;
    const char* iv = pf_ab_getenv("POSFEAT_IMGSTATS");  // 0: convimg conv + fused statistics
    m->imgstats = !(iv && iv[0] == '0');
    const char* tt = pf_ab_getenv("POSFEAT_TRAINTAP");  // 0: training on the materialised conv2 input
    m->traintap = m->train && !(tt && tt[0] == '0') && m->up4 && m->gfuse && m->up4tap;
  }
  if (m->up4 && m->gfuse) {
    alloc(m->gf_w, B * 128 * 128);
    alloc(m->gf_b, B * 128 + 9 * 64 * 128);  // + the transposed W2 G slice (gfuse.hip)
    alloc(m->gf_wp, pf_gfuse_wplanes_bytes((int)B) / 4 + 4);  // pre-split K = 80 weights
    const char* e = pf_ab_getenv("POSFEAT_HEADFUSE");
    m->hfuse = !(e && e[0] == '0') && m->up4tap && pf_conv_precision() >= 1;
    if (m->hfuse) alloc(m->gring, pf_gfuse_ring_floats((int)B, (int)H, (int)W));
  }
  if (!(m->up4 && m->gfuse) || (m->train && !m->traintap)) m->imgstats = false;
  if (m->traintap) m->imgstats = true;  // the backward contracts the image moments
  if (m->imgstats) alloc(m->imws, pf_gfuse_imgstats_ws_bytes((int)B, (int)H) / 4 + 4);
  m->bf6p = pf_bf6p_on();  // fixed for the instance: buffer sizes depend on it
  {
    const char* e = pf_ab_getenv("POSFEAT_BF6B");
    m->wsplit = pf_conv_precision() == 1 && !(e && e[0] == '0') && specs().total % 4 == 0;
  }
  if (m->wsplit) palloc(m->wpl, (size_t)specs().total * 3 / 2 + 4);
  {
    const char* e = pf_ab_getenv("POSFEAT_DSFUSE");
    m->dsfuse = m->wsplit && !m->train && pf_bf6x_on() && !(e && e[0] == '0');
  }
  if (m->dsfuse) palloc(m->dsw, dual_floats());
  {
    const char* e = pf_ab_getenv("POSFEAT_HEAD_CHUNK");
    m->hchunk = e ? std::max(0, atoi(e)) : 0;
    const char* f = pf_ab_getenv("POSFEAT_NPFUSE");
    m->npfuse = m->wsplit && !m->train && f && f[0] == '1';
    const char* g = pf_ab_getenv("POSFEAT_W6STATS");
    m->w6stats = !(g && g[0] == '0');
    const char* k = pf_ab_getenv("POSFEAT_NCHWSINK");
    m->nchwsink = k && k[0] == '1';
    const char* tw = pf_ab_getenv("POSFEAT_TAPWS");
    m->tapws = m->wsplit && !m->train && !(tw && tw[0] == '0');
    const char* ws = pf_ab_getenv("POSFEAT_WSSTEM");
    m->wsstem = m->wsplit && !m->train && ws && ws[0] == '1';
    const char* w1 = pf_ab_getenv("POSFEAT_WS1X1");
    m->ws1x1 = !m->wsplit || m->train || (w1 && w1[0] == '0') ? 0
               : w1 && (w1[0] == '1' || w1[0] == '2')   ? w1[0] - '0'
                                                        : 3;
  }
  if (m->wino) {
    size_t uf = 0, wb = 0;
    const int nl = wino_enc_on() ? 16 : 5;
    for (int i = 0; i < nl; ++i) {
      const Spec* s = specs().find(kWinoLayers[i]);
      uf += (size_t)(m->bf6p || m->wsplit ? 54 : 36) * s->cout * s->cin;
      wb = std::max(wb, pf_wino_ws_bytes((int)B, (int)H / kWinoDiv[i], (int)W / kWinoDiv[i],
                                         s->cin, s->cout));
    }
    size_t uf6 = 0;
    if (m->wino6 && !m->bf6p)
      for (int i = 0; i < nl; ++i) {
        const Spec* s = specs().find(kWinoLayers[i]);
        uf6 += pf_wino6_weights_floats(s->cin, s->cout, m->wsplit);
        wb = std::max(wb, pf_wino6_ws_bytes((int)B, (int)H / kWinoDiv[i], (int)W / kWinoDiv[i],
                                            s->cin, s->cout));
      }
    // cached: F(4x4) slots, then F(2x2) slots (a shared store serves every
    // shape), then the F(6x6) slots
    palloc(m->wino_u, (m->wcache ? 2 * uf : uf) + uf6);
    m->wino_u_f2 = m->wcache ? uf : 0;
    m->wino_u_f6 = m->wcache ? 2 * uf : uf;
    alloc(m->wino_ws, wb / 4 + 4);
  }
  if (m->train && !m->traintap) m->up4 = false;  // the backward reads the materialised conv2 input
  {
    const char* e = pf_ab_getenv("POSFEAT_SIDE");
    m->side = !(e && e[0] == '0') && m->up4 && m->gfuse && (!m->train || m->traintap);
    const char* a = pf_ab_getenv("POSFEAT_SIDE_AT");
    m->side_at = a ? std::min(4, std::max(0, atoi(a))) : 2;
  }
  if (m->up4) {
    if (!m->imgstats) alloc(m->g64, B * H * W * 64);
    alloc(m->wph, posfeat_conv2_up4_weights_floats());
    alloc(m->up4ws, posfeat_conv2_up4_workspace((int)B, (int)H, (int)W) / 4 + 4);
    if (m->up4tap) {
      alloc(m->tapw, pf_up4tap_weights_floats());
      m->tapb = m->bf6p;
      if (m->tapb || m->wsplit)  // three bf16 planes of the tap weights
        alloc(m->tapwb, pf_up4tap_weights_floats() * 3 / 2);
      if (m->tapb)  // ... and of L
        alloc(m->tapLb, (size_t)B * h4 * w4 * 192 * 3 / 2);
      alloc(m->tapP, pf_up4tap_p_floats((int)B, (int)H, (int)W));
      alloc(m->tappart, pf_up4tap_part_bytes((int)B, (int)H, (int)W) / 4 + 4);
    } else if (m->up4wino) {
      alloc(m->u4u, pf_up4_wino_weights_floats());
      alloc(m->u4ws, pf_up4_wino_ws_bytes((int)B, (int)H, (int)W) / 4 + 4);
    }
  } else {
    alloc(m->hcat, B * H * W * 256);
  }
  alloc(m->c2raw, B * H * W * 128);
  alloc(m->yraw, B * H * W);
  // instance-norm statistics, one slot of B*256 per layer: conv1, convimg, conv2
  alloc(m->st_mean, B * 256 * 3);
  alloc(m->st_rstd, B * 256 * 3);
  if (m->train) {
    alloc(m->dy3, B * H * W);
    alloc(m->dc2, B * H * W * 128);
    alloc(m->dc1, B * h4 * w4 * 192);
    size_t wg = pf_conv_wgrad_ws_bytes((int)B, (int)h4, (int)w4, 192, 192, 3, 3, 1);
    if (m->traintap) {
      alloc(m->Lbuf, B * h4 * w4 * 192);
      alloc(m->gram, B * 32 * 32, sizeof(double));
      alloc(m->x32, B * H * W * 32);
      alloc(m->tapwT, pf_up4tap_weights_floats());
      alloc(m->dwtap, pf_up4tap_weights_floats());
      alloc(m->Aimg, B * 128 * 288);
      alloc(m->imgbrws, pf_imgbr_grad_ws_bytes((int)B) / 4 + 4);
      wg = std::max(wg, pf_conv_wgrad_ws_bytes((int)B, (int)h4, (int)w4, 192, 9 * 128, 1, 1, 1));
      wg = std::max(wg, pf_conv_wgrad_per_image_ws_bytes((int)B, (int)H, (int)W, 32, 128));
    } else {
      alloc(m->dhcat, B * H * W * 256);
      alloc(m->upt, B * H * w4 * 192);
      alloc(m->wt2, (size_t)256 * posfeat_conv_packed_k(128, 3, 3));
      wg = std::max(wg, pf_conv_wgrad_ws_bytes((int)B, (int)H, (int)W, 256, 128, 3, 3, 1));
      wg = std::max(wg, pf_conv_wgrad_ws_bytes((int)B, (int)H, (int)W, 4, 64, 3, 3, 1));
    }
    alloc(m->wgws, wg / 4 + 4);
    const size_t ib = std::max(pf_in_bwd_ws_bytes((int)B, (int)(H * W), 64),
                               pf_in_bwd_ws_bytes((int)B, (int)(h4 * w4), 192));
    alloc(m->inbws, ib / 4 + 4);
    alloc(m->tailws, pf_tail_bwd_ws_bytes((int)B, (int)(H * W)) / 4 + 4);
  }
  alloc(m->st_mean1, B * 4);
  alloc(m->st_rstd1, B * 4);
  const size_t part = pf_in_stats_ws_bytes((int)B, (int)(H * W), 256);
  alloc(m->st_part, part / 4 + 1);
  // split-K scratch: sized by a dry pass over the forward
  m->splitk_need = 0;
  {
    Ctx c{m, nullptr, nullptr, true};
    posfeat_extract_out o{};
    o.local_point = reinterpret_cast<float*>(16);
    forward(c, reinterpret_cast<const float*>(16), &o);
  }
  if (m->train) {
    const posfeat_conv_desc d = m->traintap ? dl_desc(m) : dgrad_desc(m);
    m->splitk_need = std::max(m->splitk_need, posfeat_conv2d_workspace(&d));
  }
  alloc(m->splitk, m->splitk_need / 4 + 4);
  if (m->side) alloc(m->splitk2, std::max(m->splitk_need, part) / 4 + 4);
  m->ws_bytes = cur;
  m->p_bytes = pcur;
}

// torchvision Bottleneck at (n, h, w): in -> out (out may be a concat slice)
int bottleneck(Ctx& c, const std::string& p, const float* in, int n, int h, int w, int ics,
               int planes, int stride, bool has_ds, float* out, int ocs) {
  posfeat_model* m = c.m;
  const int oh = (h - 1) / stride + 1, ow = (w - 1) / stride + 1;
  float* t1 = c.f(m->t1);
  float* t2 = c.f(m->t2);
  PF_TRY(conv(c, p + ".conv1", in, n, h, w, ics, t1, planes, 1, POSFEAT_ACT_RELU));
  if (stride == 1 && c.m->wino && wino_enc_layer(p) && !c.side)
    PF_TRY(conv3x3(c, p + ".conv2", t1, n, h, w, planes, t2, planes, POSFEAT_ACT_RELU));
  else
    PF_TRY(conv(c, p + ".conv2", t1, n, h, w, planes, t2, planes, stride, POSFEAT_ACT_RELU));
  const float* res = in;
  int rcs = ics;
  if (has_ds && m->dsfuse && pf_bf6x_on()) {  // (a tile scope may have turned bf6x off)
    const int l = planes == 64 ? 0 : planes == 128 ? 1 : 2;
    const DualLayout d = dual_layout(l);
    if (c.dry) return POSFEAT_OK;
    const double flops = 2.0 * n * oh * ow * (double)d.cout * (d.k1 + d.k2);
    return timed(c, "conv:" + p + ".conv3ds", flops, [&] {
      return pf_conv_dual(n, oh, ow, t2, planes, d.k1, in, ics, h, w, stride, d.k2, d.cout,
                          reinterpret_cast<const unsigned short*>(c.f(m->dsw)) + d.off,
                          (long long)d.cout * (d.k1 + d.k2), c.f(m->dsw) + d.boff,
                          POSFEAT_ACT_RELU, out, ocs, c.st);
    });
  }
  if (has_ds) {
    float* ds = c.f(m->ds);
    PF_TRY(conv(c, p + ".downsample", in, n, h, w, ics, ds, planes * 4, stride, POSFEAT_ACT_NONE));
    res = ds;
    rcs = planes * 4;
  }
  PF_TRY(conv(c, p + ".conv3", t2, n, oh, ow, planes, out, ocs, 1, POSFEAT_ACT_RELU, res, rcs));
  return POSFEAT_OK;
}

int run_layer(Ctx& c, int li, const float* in, int n, int h, int w, int ics, float* out, int ocs) {
  posfeat_model* m = c.m;
  const int planes[3] = {64, 128, 256}, blocks[3] = {3, 4, 6};
  const int stride = li == 0 ? 1 : 2;
  const int pl = planes[li];
  const int oh = (h - 1) / stride + 1, ow = (w - 1) / stride + 1;
  const float* x = in;
  int xcs = ics;
  int ch = h, cw = w;
  for (int bi = 0; bi < blocks[li]; ++bi) {
    const std::string p = "layer" + std::to_string(li + 1) + "." + std::to_string(bi);
    const bool last = bi == blocks[li] - 1;
    float* dst = last ? out : ((bi & 1) ? c.f(m->ob) : c.f(m->oa));
    const int dcs = last ? ocs : pl * 4;
    PF_TRY(bottleneck(c, p, x, n, ch, cw, xcs, pl, bi == 0 ? stride : 1, bi == 0, dst, dcs));
    x = dst;
    xcs = dcs;
    ch = oh;
    cw = ow;
  }
  return POSFEAT_OK;
}

// the G part of head.conv2 runs inside the tap combine (posfeat_model::hfuse;
// the precision is read per call, as the conv tiles do)
bool hfuse_now(const posfeat_model* m) { return m->hfuse && pf_conv_precision() >= 1; }

// head.conv2's G part from the image (gfuse.hip) once convimg's IN statistics
// and the folded weights exist: into y (c2) by the folded 5x5 conv, or -- the
// fused head -- only the weight planes and the border ring's values, the
// interior being computed by pf_up4tap_gcombine
int gpart(Ctx& c, const float* img4, const float* g64, float* c2) {
  posfeat_model* m = c.m;
  const int B = m->B, H = m->H, W = m->W;
  const size_t SL = (size_t)B * 256;
  const float* meanI = c.f(m->st_mean) + SL;
  const float* rstdI = c.f(m->st_rstd) + SL;
  unsigned short* wp = reinterpret_cast<unsigned short*>(c.f(m->gf_wp));
  if (hfuse_now(m))
    return timed(c, "head.conv2.gprep", 0, [&] {
      return pf_gfuse_prep(img4, g64, 64, B, H, W, c.f(m->gf_w), c.f(m->gf_b), meanI, rstdI,
                           c.Bi("head.conv2"), c.W("head.convimg"), c.Bi("head.convimg"), wp,
                           c.f(m->gring), c.st);
    });
  return timed(c, "conv:head.conv2.g", 2.0 * B * H * W * 128.0 * 4 * 26, [&] {
    return pf_gfuse_conv(img4, g64, 64, B, H, W, c.f(m->gf_w), c.f(m->gf_b), meanI, rstdI,
                         c.W("head.conv2"), c.Bi("head.conv2"), c2, 128, c.st,
                         c.W("head.convimg"), c.Bi("head.convimg"), wp);
  });
}

// KeypointDet's image branch on the side stream (see posfeat_model::side):
// convimg + IN statistics (DeteNet.py:110-111), the folded G part of
// head.conv2 into y (gfuse.hip), head.conv2's phase and Winograd weights
int image_branch(Ctx& c, const float* img4) {
  posfeat_model* m = c.m;
  const int B = m->B, H = m->H, W = m->W;
  Ctx s = c;
  s.side = true;
  if (!c.dry) {
    // the engine's shared store holds them when there is one (posfeat_wstore)
    hipStream_t& side_st = m->store ? m->store->side_st : m->side_st;
    hipEvent_t& ev_fork = m->store ? m->store->ev_fork : m->ev_fork;
    hipEvent_t& ev_join = m->store ? m->store->ev_join : m->ev_join;
    if (!side_st) {
      // commit the stream and both events together (a partial set would make
      // every later extract fail on a null event)
      hipStream_t st = nullptr;
      hipEvent_t ef = nullptr, ej = nullptr;
      // (the side stream at the lowest priority was measured within noise, r5w)
      if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess ||
          hipEventCreateWithFlags(&ef, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&ej, hipEventDisableTiming) != hipSuccess) {
        if (ef) (void)hipEventDestroy(ef);
        if (st) (void)hipStreamDestroy(st);
        return POSFEAT_E_HIP;
      }
      side_st = st;
      ev_fork = ef;
      ev_join = ej;
    }
    m->side_st = side_st;  // this run's handles (owned by the store when shared)
    m->ev_fork = ev_fork;
    m->ev_join = ev_join;
    if (hipEventRecord(m->ev_fork, c.st) != hipSuccess ||
        hipStreamWaitEvent(m->side_st, m->ev_fork, 0) != hipSuccess)
      return POSFEAT_E_HIP;
    s.st = m->side_st;
  }
  const size_t SL = (size_t)B * 256;
  float* meanI = c.f(m->st_mean) + SL;
  float* rstdI = c.f(m->st_rstd) + SL;
  float* g64 = m->imgstats ? nullptr : c.f(m->g64);
  float* c2 = c.f(m->c2raw);
  if (m->imgstats)
    PF_TRY(timed(s, "head.convimg.stats", 0, [&] {
      return pf_gfuse_imgstats(img4, B, H, W, s.W("head.convimg"), s.Bi("head.convimg"), meanI,
                               rstdI, s.f(m->imws), m->imws.floats * sizeof(float), s.st,
                               m->traintap ? s.d(m->gram) : nullptr);
    }));
  else
    PF_TRY(conv_in(s, "head.convimg", img4, B, H, W, 4, g64, 64, meanI, rstdI));
  if (!m->up4tap)
    PF_TRY(timed(s, "head.conv2.weights", 0, [&] {
      return posfeat_conv2_up4_weights(s.W("head.conv2"), s.f(m->wph), s.st);
    }));
  else
    PF_TRY(timed(s, "head.conv2.tapw", 0, [&] {
      PF_TRY(pf_up4tap_weights(s.W("head.conv2"), s.f(m->tapw), s.st));
      return m->tapb || m->wsplit
                 ? pf_split3_rows(s.f(m->tapw), 1152, 192, 192,
                                  reinterpret_cast<unsigned short*>(s.f(m->tapwb)), s.st)
                 : POSFEAT_OK;
    }));
  PF_TRY(timed(s, "head.conv2.gfuse_w", 0, [&] {
    return pf_gfuse_weights(s.W("head.conv2"), s.Bi("head.conv2"), s.W("head.convimg"),
                            s.Bi("head.convimg"), meanI, rstdI, B, s.f(m->gf_w), s.f(m->gf_b),
                            s.st);
  }));
  PF_TRY(gpart(s, img4, g64, c2));
  if (m->up4wino && !m->up4tap)
    PF_TRY(timed(s, "head.conv2.up4w", 0, [&] {
      return pf_up4_wino_weights(s.f(m->wph), s.f(m->u4u), s.st);
    }));
  if (!c.dry && hipEventRecord(m->ev_join, s.st) != hipSuccess) return POSFEAT_E_HIP;
  return POSFEAT_OK;
}

int forward(Ctx& c, const float* img, posfeat_extract_out* out, int mode, const float* xhead) {
  posfeat_model* m = c.m;
  // the keypoint-head training instance keeps the 32x32x16 dense tiles
  // (the head gradient's fixture case is ill-conditioned)
  const PfDense32Scope dense32(m->train);
  const int B = m->B, H = m->H, W = m->W;
  const int h2 = H / 2, w2 = W / 2, h4 = H / 4, w4 = W / 4, h8 = H / 8, w8 = W / 8, h16 = H / 16,
            w16 = W / 16;
  float* img4 = c.f(m->img4);
  float* headcat = c.f(m->headcat);
  bool lm_nchw = false;  // conv_fine wrote local_map NCHW (PfNchwSink)
  // ---- ResUNet (DescNet.py:64-84) -----------------------------------------
  // (the planning pass runs before the instance has its store)
  if (m->wsplit && !(m->wcache && m->store && m->store->wpl_done)) {  // the blob's bf16 planes
    PF_TRY(timed(c, "weights.split", 0, [&] {
      PF_TRY(pf_split3_rows(m->wts, specs().total / 4, 4, 4,
                            reinterpret_cast<unsigned short*>(c.f(m->wpl)), c.st));
      if (!m->dsfuse) return POSFEAT_OK;
      const unsigned short* wpl = reinterpret_cast<const unsigned short*>(c.f(m->wpl));
      unsigned short* dsw = reinterpret_cast<unsigned short*>(c.f(m->dsw));
      for (int l = 0; l < 3; ++l) {
        const DualLayout d = dual_layout(l);
        const std::string p = "layer" + std::to_string(l + 1) + ".0";
        PF_TRY(pf_dual_weights(wpl + specs().find(p + ".conv3")->w_off, d.k1,
                               wpl + specs().find(p + ".downsample")->w_off, d.k2, specs().total,
                               d.cout, c.Bi(p + ".conv3"), c.Bi(p + ".downsample"), dsw + d.off,
                               c.f(m->dsw) + d.boff, c.st));
      }
      return POSFEAT_OK;
    }));
    if (!c.dry && m->wcache) m->store->wpl_done = m->wprep_pending = true;
  }
  PF_TRY(timed(c, "layout:img", 0, [&] { return pf_nchw_to_nhwc(img, B, 3, H, W, 4, img4, c.st); }));
  // the first forward of a shape autotunes every main-stream conv by timing
  // it: run it serially so the side stream's kernels do not contend with
  // the candidates being timed (the tile choice would depend on that race)
  const bool side = m->side && mode != MODE_BACKBONE &&
                    (c.dry || ((m->tuned_modes >> mode) & 1u) || !m->autotune);
  // where the image branch forks (POSFEAT_SIDE_AT): 0 after the image layout,
  // 1 before layer2, 2 before layer3 (default: the 60x80 layers underfill the
  // chip; overlapping layer1 slowed its convs 2-4x), 3 before the decoder,
  // 4 before the head (beside head.conv1 and the tap GEMM)
  const int side_at = mode == MODE_HEAD ? 0 : m->side_at;
  if (side && side_at == 0) PF_TRY(image_branch(c, img4));
  if (mode == MODE_HEAD) {
    // KeypointDet's own input: fine_maps[0] = cat[local_map, local_map_small]
    // (PoSFeat_model.py:97-102), NCHW 192 channels at H/4 x W/4
    PF_TRY(timed(c, "layout:head_in", 0, [&] {
      return pf_nchw_to_nhwc(xhead, B, 192, h4, w4, 192, headcat, c.st);
    }));
  } else {
  PF_TRY(conv(c, "firstconv", img4, B, H, W, 4, c.f(m->stem), 64, 2, POSFEAT_ACT_RELU));
  PF_TRY(timed(c, "maxpool", 0, [&] {
    return pf_maxpool3s2(c.f(m->stem), B, h2, w2, 64, 64, headcat + 128, 192, c.st);
  }));
  float* cat2 = c.f(m->cat2);
  float* cat3 = c.f(m->cat3);
  PF_TRY(run_layer(c, 0, headcat + 128, B, h4, w4, 192, cat2 + 256, 512));  // layer1 -> cat2[256:]
  if (side && side_at == 1) PF_TRY(image_branch(c, img4));
  PF_TRY(run_layer(c, 1, cat2 + 256, B, h4, w4, 512, cat3 + 512, 1024));    // layer2 -> cat3[512:]
  if (side && side_at == 2) PF_TRY(image_branch(c, img4));
  PF_TRY(run_layer(c, 2, cat3 + 512, B, h8, w8, 1024, c.f(m->l3out), 1024));
  if (side && side_at == 3) PF_TRY(image_branch(c, img4));
  PF_TRY(conv(c, "conv_coarse", c.f(m->l3out), B, h16, w16, 1024, c.f(m->gmap), 128, 1,
              POSFEAT_ACT_ELU));
  // upconv (DescNet.py:182-190): x2 upsample + conv, the upsample inside
  // the Winograd input transform
  PF_TRY(conv3x3(c, "upconv3.conv", c.f(m->l3out), B, h8, w8, 1024, cat3, 1024, POSFEAT_ACT_ELU,
                 1, c.f(m->up3)));
  PF_TRY(conv3x3(c, "iconv3", cat3, B, h8, w8, 1024, c.f(m->d3), 512, POSFEAT_ACT_ELU));
  PF_TRY(conv3x3(c, "upconv2.conv", c.f(m->d3), B, h4, w4, 512, cat2, 512, POSFEAT_ACT_ELU, 1,
                 c.f(m->up2)));
  PF_TRY(conv3x3(c, "iconv2", cat2, B, h4, w4, 512, c.f(m->d2), 256, POSFEAT_ACT_ELU));
  // conv_fine also writes local_map NCHW from its epilogue when the caller
  // wants it (PfNchwSink; else the layout pass below)
  {
    const PfNchwSink sink(out && out->local_map && !c.dry && m->nchwsink ? out->local_map : nullptr);
    PF_TRY(conv(c, "conv_fine", c.f(m->d2), B, h4, w4, 256, headcat, 192, 1, POSFEAT_ACT_ELU));
    lm_nchw = sink.done();
  }
  }
  if (side && side_at == 4 && mode != MODE_HEAD) PF_TRY(image_branch(c, img4));
  if (mode != MODE_BACKBONE) PF_TRY(head_forward(c, img4, out->local_point, side));
  // ---- outputs -------------------------------------------------------------
  if (mode != MODE_HEAD) {
    if (out->global_feat)
      PF_TRY(timed(c, "global_feat", 0, [&] {
        return pf_global_feat(c.f(m->gmap), B, h16 * w16, 128, out->global_feat, c.st);
      }));
    if (out->local_map && !lm_nchw)
      PF_TRY(timed(c, "layout:out", 0, [&] {
        return pf_nhwc_to_nchw(headcat, B, 128, h4, w4, 192, out->local_map, c.st);
      }));
    if (out->local_map_small)
      PF_TRY(timed(c, "layout:out", 0, [&] {
        return pf_nhwc_to_nchw(headcat + 128, B, 64, h4, w4, 192, out->local_map_small, c.st);
      }));
    if (out->global_map)
      PF_TRY(timed(c, "layout:out", 0, [&] {
        return pf_nhwc_to_nchw(c.f(m->gmap), B, 128, h16, w16, 128, out->global_map, c.st);
      }));
  }
  out->local_map_nhwc = headcat;
  out->local_map_cstride = 192;
  return POSFEAT_OK;
}

// KeypointDet (DeteNet.py:102-121) on headcat = cat[local_map, local_map_small]
// and the NHWC4 image; `side`: the image branch was forked to the side stream
int head_forward(Ctx& c, float* img4, float* local_point, bool side) {
  posfeat_model* m = c.m;
  const int B = m->B, H = m->H, W = m->W, h4 = H / 4, w4 = W / 4;
  const float* slope = m->wts + specs().find("head.prelu")->b_off;
  float* headcat = c.f(m->headcat);
  // ---- KeypointDet (DeteNet.py:102-121), identity prior == exact 1.0 -------
  // IN statistics slots: conv1, convimg, conv2 (the backward reads all three)
  const size_t SL = (size_t)B * 256;
  float* mean = c.f(m->st_mean) + 2 * SL;
  float* rstd = c.f(m->st_rstd) + 2 * SL;
  float* mean1 = c.f(m->st_mean);
  float* rstd1 = c.f(m->st_rstd);
  float* meanI = c.f(m->st_mean) + SL;
  float* rstdI = c.f(m->st_rstd) + SL;
  double* part = c.d(m->st_part);
  float* c1 = c.f(m->c1raw);
  float* c2 = c.f(m->c2raw);
  if (m->wino && h4 % 2 == 0 && w4 % 2 == 0) {
    // Winograd conv (bias, no act); its output transform also sums the IN
    // statistics when it can (F(6x6): pf_wino6_conv stats, A/B
    // POSFEAT_W6STATS=0), else a separate statistics pass
    const size_t need = (size_t)B * pf_wino6_stats_groups(h4, w4) * 192 * 2;
    double* sp = m->w6stats && need <= m->st_part.floats / 2 ? c.d(m->st_part) : nullptr;
    bool done = false;
    PF_TRY(conv3x3(c, "head.conv1", headcat, B, h4, w4, 192, c1, 192, POSFEAT_ACT_NONE, 0,
                   nullptr, sp, &done));
    if (done)
      PF_TRY(timed(c, "instnorm", 0, [&] {
        return pf_in_finalize(sp, B, pf_wino6_stats_groups(h4, w4), h4 * w4, 192, mean1, rstd1,
                              c.st);
      }));
    else
      PF_TRY(timed(c, "instnorm", 0, [&] {
        return pf_in_stats(c1, B, h4 * w4, 192, 192, mean1, rstd1, c.d(m->st_part), c.st);
      }));
  } else {
    PF_TRY(conv_in(c, "head.conv1", headcat, B, h4, w4, 192, c1, 192, mean1, rstd1));
  }
  if (m->up4) {
    // L = PReLU(IN(conv1)) stays at 1/4 resolution; conv2 reads it per phase
    // (training keeps the raw conv1 output for the backward: L in its own buffer)
    float* L = m->traintap ? c.f(m->Lbuf) : c1;
    if (m->traintap)
      PF_TRY(timed(c, "train:keep_c1", 0, [&] {
        return hipMemcpyAsync(L, c1, (size_t)B * h4 * w4 * 192 * sizeof(float),
                              hipMemcpyDeviceToDevice, c.st) == hipSuccess
                   ? POSFEAT_OK
                   : POSFEAT_E_HIP;
      }));
    // npf: the tap GEMM normalises conv1's output on load (below)
    const bool npf = m->npfuse && !m->traintap && !m->tapb && m->up4tap && hfuse_now(m) &&
                     !(m->hchunk > 0 && m->hchunk < B) && pf_bf6x_on();
    auto norm_prelu = [&] {
      return timed(c, "norm_prelu", 0, [&] {
        return pf_in_apply(L, B, h4 * w4, 192, 192, mean1, rstd1, slope, c.st);
      });
    };
    if (!npf) PF_TRY(norm_prelu());
    float* g64 = m->imgstats ? nullptr : c.f(m->g64);
    if (!side && m->imgstats)
      PF_TRY(timed(c, "head.convimg.stats", 0, [&] {
        return pf_gfuse_imgstats(img4, B, H, W, c.W("head.convimg"), c.Bi("head.convimg"), meanI,
                                 rstdI, c.f(m->imws), m->imws.floats * sizeof(float), c.st,
                                 m->traintap ? c.d(m->gram) : nullptr);
      }));
    else if (!side)
      PF_TRY(conv_in(c, "head.convimg", img4, B, H, W, 4, g64, 64, meanI, rstdI));
    if (!m->gfuse)
      PF_TRY(timed(c, "instnorm_apply", 0, [&] {
        return pf_in_apply(g64, B, H * W, 64, 64, meanI, rstdI, nullptr, c.st);
      }));
    // executed MFMA work: 64 full-res channels x 9 taps, 192 low-res channels
    // x 6.25 taps on average over the 16 phases (the reference layer: 256 x 9)
    const float* wph = c.f(m->wph);
    if (!side && !m->up4tap)
      PF_TRY(timed(c, "head.conv2.weights", 0, [&] {
        return posfeat_conv2_up4_weights(c.W("head.conv2"), c.f(m->wph), c.st);
      }));
    if (!side && m->up4tap)
      PF_TRY(timed(c, "head.conv2.tapw", 0, [&] {
        PF_TRY(pf_up4tap_weights(c.W("head.conv2"), c.f(m->tapw), c.st));
        return m->tapb || m->wsplit
                   ? pf_split3_rows(c.f(m->tapw), 1152, 192, 192,
                                    reinterpret_cast<unsigned short*>(c.f(m->tapwb)), c.st)
                   : POSFEAT_OK;
      }));
    if (side) {
      // join the image branch (it wrote the G part into y)
      if (!c.dry && hipStreamWaitEvent(c.st, m->ev_join, 0) != hipSuccess) return POSFEAT_E_HIP;
    } else if (m->gfuse) {
      // G = IN(convimg(img)) folded into a per-image 5x5 conv of the image
      // (+ the exact one-pixel border ring); g64 holds the raw convimg output
      PF_TRY(timed(c, "head.conv2.gfuse_w", 0, [&] {
        return pf_gfuse_weights(c.W("head.conv2"), c.Bi("head.conv2"), c.W("head.convimg"),
                                c.Bi("head.convimg"), meanI, rstdI, B, c.f(m->gf_w),
                                c.f(m->gf_b), c.st);
      }));
      PF_TRY(gpart(c, img4, g64, c2));
    } else {
      PF_TRY(timed(c, "conv:head.conv2.g", 2.0 * B * H * W * 128.0 * 64 * 9, [&] {
        return pf_up4_gconv(B, H, W, g64, 64, wph, c.Bi("head.conv2"), c2, 128, c.st);
      }));
    }
    if (m->up4tap) {
      // P_k = W_k[:, :192] . L on the low-res grid (one 1x1-conv GEMM,
      // N = 9 taps x 128), then y += the tap-summed x4 interpolation of P,
      // with the instance-norm statistics of the finished conv2 output
      posfeat_conv_desc d;
      d.n = B;
      d.h = h4;
      d.w = w4;
      d.cin = 192;
      d.x_cstride = 192;
      d.cout = 9 * 128;
      d.kh = d.kw = 1;
      d.stride = 1;
      d.pad = 0;
      d.y_cstride = 9 * 128;
      d.res_cstride = 0;
      d.act = POSFEAT_ACT_NONE;
      if (m->tapb) {  // bf16x6 on pre-split planes (gemm6.hip)
        const long long M = (long long)B * h4 * w4;
        unsigned short* Lb = reinterpret_cast<unsigned short*>(c.f(m->tapLb));
        PF_TRY(timed(c, "head.conv2.split", 0,
                     [&] { return pf_split3_rows(L, M, 192, 192, Lb, c.st); }));
        PF_TRY(timed(c, "conv:head.conv2.up4tap", 2.0 * M * 1152.0 * 192, [&] {
          return pf_gemm_bf6p(Lb, 192, M * 192, 0,
                              reinterpret_cast<const unsigned short*>(c.f(m->tapwb)), 192,
                              1152LL * 192, 0, c.f(m->tapP), 1152, 0, 1, (int)M, 1152, 192, c.st);
        }));
      } else if (m->hchunk > 0 && m->hchunk < B && hfuse_now(m)) {
        // chunks of G images through one P slab (its lines may still be in
        // the memory-side cache when the combine reads them)
        const int G = m->hchunk;
        const size_t wpi = pf_gfuse_wplanes_bytes(1) / 2, rpi = pf_gfuse_ring_image_floats(H, W);
        for (int b0 = 0; b0 < B; b0 += G) {
          const int g = std::min(G, B - b0);
          d.n = g;
          PF_TRY(conv_desc_run(c, "head.conv2.up4tap", d, L + (size_t)b0 * h4 * w4 * 192,
                               c.f(m->tapw), nullptr, nullptr, c.f(m->tapP),
                               2.0 * g * h4 * w4 * 1152.0 * 192,
                               m->wsplit ? reinterpret_cast<const unsigned short*>(c.f(m->tapwb))
                                         : nullptr,
                               1152LL * 192));
          PF_TRY(timed(c, "head.conv2.gcombine", 0, [&] {
            return pf_up4tap_gcombine(
                g, H, W, c.f(m->tapP), img4 + (size_t)b0 * H * W * 4,
                reinterpret_cast<const unsigned short*>(c.f(m->gf_wp)) + b0 * wpi,
                c.f(m->gf_b) + (size_t)b0 * 128, c.f(m->gring) + b0 * rpi,
                c2 + (size_t)b0 * H * W * 128, 128, c.d(m->tappart), mean + (size_t)b0 * 128,
                rstd + (size_t)b0 * 128, c.st);
          }));
        }
      } else {
        int rc = POSFEAT_E_UNSUPPORTED;
        if (m->tapws && !npf && !c.dry && pf_bf6x_on()) {  // (16x16x32 terms: the bf6x family)
          const int M = B * h4 * w4;
          rc = timed(c, "conv:head.conv2.up4tap", 2.0 * M * 1152.0 * 192, [&] {
            return pf_tap_gemm_ws(L, 192, M, reinterpret_cast<const unsigned short*>(c.f(m->tapwb)),
                                  1152LL * 192, 1152, c.f(m->tapP), 1152, c.st);
          });
          if (rc != POSFEAT_OK && rc != POSFEAT_E_INVALID && rc != POSFEAT_E_UNSUPPORTED) return rc;
        }
        if (rc != POSFEAT_OK && npf && !c.dry) {
          // the tuned tile if there is one (else the DB's / the default plan)
          int tile = -1;
          auto it = m->tuned.find("head.conv2.up4tap");
          if (it != m->tuned.end())
            tile = it->second;
          else if (!tile_lookup(d, false, true, &tile))
            tile = -1;
          rc = timed(c, "conv:head.conv2.up4tap", 2.0 * B * h4 * w4 * 1152.0 * 192, [&] {
            return pf_conv_run_tile_np(&d, c1, c.f(m->tapw), c.f(m->tapP), tile, c.st,
                                       reinterpret_cast<const unsigned short*>(c.f(m->tapwb)),
                                       1152LL * 192, mean1, rstd1, slope);
          });
          if (rc != POSFEAT_OK && rc != POSFEAT_E_UNSUPPORTED) return rc;
        }
        if (rc != POSFEAT_OK) {  // (the planning pass, or a tile without the fused load)
          if (npf) PF_TRY(norm_prelu());
          PF_TRY(conv_desc_run(c, "head.conv2.up4tap", d, L, c.f(m->tapw), nullptr, nullptr,
                               c.f(m->tapP), 2.0 * B * h4 * w4 * 1152.0 * 192,
                               m->wsplit ? reinterpret_cast<const unsigned short*>(c.f(m->tapwb))
                                         : nullptr,
                               1152LL * 192));
        }
      }
      if (m->hchunk > 0 && m->hchunk < B && hfuse_now(m) && !m->tapb) {
        // (done above, chunk by chunk)
      } else if (hfuse_now(m))
        PF_TRY(timed(c, "head.conv2.gcombine", 0, [&] {
          return pf_up4tap_gcombine(B, H, W, c.f(m->tapP), img4,
                                    reinterpret_cast<const unsigned short*>(c.f(m->gf_wp)),
                                    c.f(m->gf_b), c.f(m->gring), c2, 128, c.d(m->tappart), mean,
                                    rstd, c.st);
        }));
      else
        PF_TRY(timed(c, "head.conv2.combine", 0, [&] {
          return pf_up4tap_combine(B, H, W, c.f(m->tapP), c2, 128, c.d(m->tappart), mean, rstd,
                                   c.st);
        }));
    } else {
    PF_TRY(timed(c, "head.conv2.border", 0, [&] {
      return pf_up4_border(B, H, W, c1, 192, wph, c2, 128, c.st);
    }));
    if (m->up4wino) {
      // executed: 36 transform-domain MACs per 4x4 low-res tile, 2048 phase
      // channels x 192 (vs 6.25 taps per full-res pixel for the phase kernel)
      if (!side)
        PF_TRY(timed(c, "head.conv2.up4w", 0, [&] {
          return pf_up4_wino_weights(wph, c.f(m->u4u), c.st);
        }));
      auto up4w = [&](int stages) {
        return pf_up4_wino(B, H, W, c1, 192, c.f(m->u4u), c2, 128, c.f(m->u4ws),
                           m->u4ws.floats * sizeof(float), c.st, stages);
      };
      PF_TRY(timed(c, "head.conv2.up4.vt", 0, [&] { return up4w(1); }));
      PF_TRY(timed(c, "conv:head.conv2.up4", 2.0 * 36 * B * (H / 16) * (W / 16) * 2048.0 * 192,
                   [&] { return up4w(2); }));
      // output transform + the instance-norm statistics of the finished conv2 output
      PF_TRY(timed(c, "head.conv2.up4.ot", 0, [&] {
        return pf_up4_wino(B, H, W, c1, 192, c.f(m->u4u), c2, 128, c.f(m->u4ws),
                           m->u4ws.floats * sizeof(float), c.st, 4, mean, rstd);
      }));
    } else {
      PF_TRY(timed(c, "conv:head.conv2.up4", 2.0 * B * H * W * 128.0 * 192 * 6.25, [&] {
        return pf_up4_main(B, H, W, c1, 192, wph, c2, 128, c.f(m->up4ws),
                           m->up4ws.floats * sizeof(float), mean, rstd, 1e-5f, c.st);
      }));
    }
    }
  } else {
    float* hcat = c.f(m->hcat);
    PF_TRY(timed(c, "norm_prelu_up4", 0, [&] {
      return pf_norm_prelu_upsample(c1, B, h4, w4, 192, 192, mean1, rstd1, slope, H, W, hcat, 256,
                                    c.st);
    }));
    PF_TRY(conv_in(c, "head.convimg", img4, B, H, W, 4, hcat + 192, 256, meanI, rstdI));
    PF_TRY(timed(c, "instnorm_apply", 0, [&] {
      return pf_in_apply(hcat + 192, B, H * W, 64, 256, meanI, rstdI, nullptr, c.st);
    }));
    PF_TRY(conv_in(c, "head.conv2", hcat, B, H, W, 256, c2, 128, mean, rstd));
  }
  PF_TRY(timed(c, "head_tail", 2.0 * B * H * W * 128, [&] {
    return pf_head_tail(c2, B, H * W, 128, mean, rstd, slope, c.W("head.conv3"),
                        c.Bi("head.conv3"), c.f(m->yraw), local_point, c.f(m->st_mean1),
                        c.f(m->st_rstd1), part, c.st);
  }));
  return POSFEAT_OK;
}

const Spec& spec(const char* n) { return *specs().find(n); }
long long head_offset() { return spec("head.conv1").w_off; }

// The rest of the KeypointDet backward on the extraction path's factorisation
// of head.conv2 (traintap), from dc2 = dL/d(conv2 out):
//   upsampled part: y += sum_k shift_k(up4(P_k)), P_k = W_k[:, :192] L, so
//     D = dL/dP (the combine's adjoint, up4tap.hip), dW_k = D_k^T L and
//     dL = sum_k D_k W_k -- two GEMMs on the h x w grid (1/16 of the full-res
//     weight / input gradients' MACs);
//   image part + convimg: contractions of the per-image 3x3 weight gradient
//     of dc2 against the 32-channel tap image (headgrad.hip) -- no G map;
//   conv1: IN/PReLU backward + weight gradient as before.
int head_backward_tap(Ctx& c, float* grad, double* t2s, int t2n) {
  posfeat_model* m = c.m;
  const int B = m->B, H = m->H, W = m->W, h4 = H / 4, w4 = W / 4;
  const long long hoff = head_offset();
  auto G = [&](const char* n) { return grad + (spec(n).w_off - hoff); };
  auto GB = [&](const char* n) { return grad + (spec(n).b_off - hoff); };
  const float* slope = m->wts + spec("head.prelu").b_off;
  const size_t SL = (size_t)B * 256;
  const float* mean1 = c.f(m->st_mean);
  const float* rstd1 = c.f(m->st_rstd);
  float* dc1 = c.f(m->dc1);
  float* dc2 = c.f(m->dc2);
  float* D = c.f(m->tapP);  // P is dead after the forward
  const size_t wgb = m->wgws.floats * sizeof(float);
  PF_TRY(timed(c, "bwd:up4tap_adjoint", 0,
               [&] { return pf_up4tap_adjoint(B, H, W, dc2, 128, D, c.st); }));
  // WtT (+ its bf16 planes in the forward's tap-weight plane buffer, free
  // after the forward) for the pre-split bf16x6 tiles
  unsigned short* wtTb = m->wsplit ? reinterpret_cast<unsigned short*>(c.f(m->tapwb)) : nullptr;
  PF_TRY(timed(c, "bwd:tapw_t", 0, [&] {
    PF_TRY(pf_up4tap_weights_t(c.W("head.conv2"), c.f(m->tapwT), c.st));
    return wtTb ? pf_split3_rows(c.f(m->tapwT), 192, 1152, 1152, wtTb, c.st) : POSFEAT_OK;
  }));
  PF_TRY(timed(c, "bwdconv:head.conv2.tap_wgrad", 2.0 * B * h4 * w4 * 1152.0 * 192, [&] {
    return pf_conv_wgrad(D, 1152, c.f(m->Lbuf), 192, B, h4, w4, 192, 1152, 1, 1, 1, c.f(m->dwtap),
                         nullptr, 0, c.f(m->wgws), wgb, c.st);
  }));
  {
    const posfeat_conv_desc d = dl_desc(m);
    PF_TRY(conv_desc_run(c, "bwd.head.conv2.tap_dgrad", d, D, c.f(m->tapwT), nullptr, nullptr, dc1,
                         2.0 * B * h4 * w4 * 1152.0 * 192, wtTb, 192LL * 1152));
  }
  PF_TRY(timed(c, "bwd:img_taps", 0,
               [&] { return pf_img_taps32(c.f(m->img4), B, H, W, c.f(m->x32), c.st); }));
  PF_TRY(timed(c, "bwdconv:head.imgbranch.wgrad", 2.0 * B * H * W * 128.0 * 288, [&] {
    return pf_conv_wgrad_per_image(dc2, 128, c.f(m->x32), 32, B, H, W, 32, 128, c.f(m->Aimg),
                                   c.f(m->wgws), wgb, c.st);
  }));
  PF_TRY(timed(c, "bwd:imgbranch_grads", 0, [&] {
    return pf_imgbr_grad(c.f(m->Aimg), B, H * W, c.W("head.conv2"), c.W("head.convimg"),
                         c.Bi("head.convimg"), c.f(m->st_mean) + SL, c.f(m->st_rstd) + SL,
                         c.d(m->gram), c.f(m->dwtap), G("head.conv2"), GB("head.conv2"),
                         G("head.convimg"), GB("head.convimg"), c.f(m->imgbrws),
                         m->imgbrws.floats * sizeof(float), c.st);
  }));
  double* c1s = nullptr;
  int c1n = 0;
  PF_TRY(timed(c, "bwd:in_conv1", 0, [&] {
    return pf_in_backward(c.f(m->c1raw), 192, dc1, 192, B, h4 * w4, 192, mean1, rstd1, slope, dc1,
                          192, c.f(m->inbws), &c1s, &c1n, c.st);
  }));
  PF_TRY(timed(c, "bwdconv:head.conv1.wgrad", 2.0 * B * h4 * w4 * 192.0 * 192 * 9, [&] {
    return pf_conv_wgrad(dc1, 192, c.f(m->headcat), 192, B, h4, w4, 192, 192, 3, 3, 1,
                         G("head.conv1"), GB("head.conv1"), 0, c.f(m->wgws), wgb, c.st);
  }));
  PF_TRY(timed(c, "bwd:scalars", 0, [&] {
    return pf_head_scalars(t2s, t2n, c1s, c1n, GB("head.conv3"), GB("head.prelu"), c.st);
  }));
  return POSFEAT_OK;
}

// KeypointDet backward (networks/DeteNet.py:102-121 under autograd, as
// managers/trainer.py:331 runs it for configs/train_kp.yaml): given dL/d
// local_point of the last forward on this workspace, writes dL/d(every head
// parameter) into `grad`, laid out like the weight blob from head.conv1 on.
int head_backward(Ctx& c, const float* dlp, float* grad) {
  posfeat_model* m = c.m;
  const int B = m->B, H = m->H, W = m->W, h4 = H / 4, w4 = W / 4;
  const long long hoff = head_offset();
  auto G = [&](const char* n) { return grad + (spec(n).w_off - hoff); };
  auto GB = [&](const char* n) { return grad + (spec(n).b_off - hoff); };
  const float* slope = m->wts + spec("head.prelu").b_off;
  const size_t SL = (size_t)B * 256;
  const float* mean1 = c.f(m->st_mean);
  const float* rstd1 = c.f(m->st_rstd);
  const float* mean2 = c.f(m->st_mean) + 2 * SL;
  const float* rstd2 = c.f(m->st_rstd) + 2 * SL;
  float* hcat = c.f(m->hcat);
  float* dhcat = c.f(m->dhcat);
  float* dc1 = c.f(m->dc1);
  float* dc2 = c.f(m->dc2);
  const size_t wgb = m->wgws.floats * sizeof(float);
  PF_TRY(timed(c, "bwd:zero", 0, [&] {
    return hipMemsetAsync(grad, 0, (specs().total - hoff) * sizeof(float), c.st) == hipSuccess
               ? POSFEAT_OK
               : POSFEAT_E_HIP;
  }));
  // Softplus / norm3 / conv3 / PReLU / norm2  ->  d(conv2 out)
  double* t2s = nullptr;
  int t2n = 0;
  PF_TRY(timed(c, "bwd:tail", 0, [&] {
    return pf_tail_backward(dlp, c.f(m->yraw), c.f(m->st_mean1), c.f(m->st_rstd1), c.f(m->c2raw),
                            128, mean2, rstd2, slope, c.W("head.conv3"), B, H * W, c.f(m->dy3),
                            dc2, 128, G("head.conv3"), c.f(m->tailws), &t2s, &t2n, c.st);
  }));
  if (m->traintap) return head_backward_tap(c, grad, t2s, t2n);
  // conv2: weight gradient over the materialised cat[up4(L), IN(convimg)]
  PF_TRY(timed(c, "bwdconv:head.conv2.wgrad", 2.0 * B * H * W * 128.0 * 256 * 9, [&] {
    return pf_conv_wgrad(dc2, 128, hcat, 256, B, H, W, 256, 128, 3, 3, 1, G("head.conv2"),
                         GB("head.conv2"), 0, c.f(m->wgws), wgb, c.st);
  }));
  // conv2: input gradient = conv of dc2 with the flipped, transposed kernel
  PF_TRY(timed(c, "bwd:dgrad_weights", 0, [&] {
    return pf_dgrad_weights(c.W("head.conv2"), 128, 256, 3, 3, c.f(m->wt2), c.st);
  }));
  {
    const posfeat_conv_desc d = dgrad_desc(m);
    PF_TRY(timed(c, "bwdconv:head.conv2.dgrad", 2.0 * B * H * W * 128.0 * 256 * 9, [&] {
      return posfeat_conv2d_nhwc_ws(&d, dc2, c.f(m->wt2), nullptr, nullptr, dhcat,
                                    c.f(m->splitk), m->splitk.floats * sizeof(float), c.st);
    }));
  }
  // image branch: normimg backward in place on channels 192..255, then convimg dW
  PF_TRY(timed(c, "bwd:in_img", 0, [&] {
    return pf_in_backward(hcat + 192, 256, dhcat + 192, 256, B, H * W, 64, nullptr,
                          c.f(m->st_rstd) + SL, nullptr, dhcat + 192, 256, c.f(m->inbws), nullptr,
                          nullptr, c.st);
  }));
  PF_TRY(timed(c, "bwdconv:head.convimg.wgrad", 2.0 * B * H * W * 64.0 * 3 * 9, [&] {
    return pf_conv_wgrad(dhcat + 192, 256, c.f(m->img4), 4, B, H, W, 4, 64, 3, 3, 1,
                         G("head.convimg"), GB("head.convimg"), 0, c.f(m->wgws), wgb, c.st);
  }));
  // x4 upsample adjoint of the 192 upsampled channels -> d PReLU(IN(conv1))
  PF_TRY(timed(c, "bwd:up4_adjoint", 0, [&] {
    return pf_up4_adjoint(dhcat, 256, B, H, W, h4, w4, 192, c.f(m->upt), dc1, 192, c.st);
  }));
  double* c1s = nullptr;
  int c1n = 0;
  PF_TRY(timed(c, "bwd:in_conv1", 0, [&] {
    return pf_in_backward(c.f(m->c1raw), 192, dc1, 192, B, h4 * w4, 192, mean1, rstd1, slope, dc1,
                          192, c.f(m->inbws), &c1s, &c1n, c.st);
  }));
  PF_TRY(timed(c, "bwdconv:head.conv1.wgrad", 2.0 * B * h4 * w4 * 192.0 * 192 * 9, [&] {
    return pf_conv_wgrad(dc1, 192, c.f(m->headcat), 192, B, h4, w4, 192, 192, 3, 3, 1,
                         G("head.conv1"), GB("head.conv1"), 0, c.f(m->wgws), wgb, c.st);
  }));
  PF_TRY(timed(c, "bwd:scalars", 0, [&] {
    return pf_head_scalars(t2s, t2n, c1s, c1n, GB("head.conv3"), GB("head.prelu"), c.st);
  }));
  return POSFEAT_OK;
}

}  // namespace

// The tile of a conv the training step runs itself (bbtrain.hip: forward
// convs, stride-1 input gradients, stride-2 phase convs).  Its direct convs
// are not all bit-identical across tiles (the pre-split tiles' sums differ
// from the fp32 ones, and the BatchNorm epilogue's fp64 partials follow the
// tile), so a choice timed live would make the step's numerics depend on a
// timing race -- between two runs, and between DDP ranks.  The
// training step therefore takes a tile only from an EXACT entry of the tile
// database every rank loads (records/tile_db.txt; its training entries are
// made by `tools/tile_db.py --train`, which sets POSFEAT_TRAIN_TUNE_LIVE=1 to
// time the candidates live), and runs the default plan for a conv it does not
// hold.  `run(tile)` launches the conv with that tile (-1: default plan).
static bool train_tune_live() {
  static const bool v = [] {
    const char* e = getenv("POSFEAT_TRAIN_TUNE_LIVE");
    return e && e[0] == '1';
  }();
  return v;
}

int pf_conv_tuned_run(const posfeat_conv_desc* d, bool res, bool wplanes, hipStream_t st,
                      const std::function<int(int)>& run) {
  int tile = -1;
  if (!tile_lookup(*d, res, wplanes, &tile, /*exact_only=*/true)) {
    tile = -1;
    if (train_tune_live()) {
      tile = tune("train", *d, st, run, wplanes);
      tile_store(*d, res, wplanes, tile);
    }
  }
  return run(tile);
}

extern "C" long long posfeat_model_head_offset(void) { return head_offset(); }
extern "C" long long posfeat_model_head_floats(void) { return specs().total - head_offset(); }

extern "C" int posfeat_model_create_train(int batch, int h, int w, const float* weights,
                                          posfeat_model** out) {
  if (!out || !weights || batch <= 0 || h < 16 || w < 16 || h % 16 || w % 16)
    return POSFEAT_E_INVALID;
  posfeat_model* m = new (std::nothrow) posfeat_model();
  if (!m) return POSFEAT_E_INVALID;
  m->B = batch;
  m->H = h;
  m->W = w;
  m->wts = weights;
  m->train = true;
  plan(m);
  *out = m;
  return POSFEAT_OK;
}

extern "C" int posfeat_model_head_backward(posfeat_model* m, const float* dlocal_point,
                                           float* grad, void* ws, size_t ws_bytes, void* stream) {
  if (!m || !dlocal_point || !grad || !ws) return POSFEAT_E_INVALID;
  if (!m->train) return POSFEAT_E_UNSUPPORTED;
  if (ws_bytes < m->ws_bytes) return POSFEAT_E_WORKSPACE;
  if (reinterpret_cast<uintptr_t>(ws) & 255) return POSFEAT_E_INVALID;
  Ctx c{m, static_cast<char*>(ws), pf_stream(stream)};
  const PfDense32Scope dense32(true);
  return head_backward(c, dlocal_point, grad);
}

extern "C" int posfeat_model_num_specs(void) { return (int)specs().v.size(); }

extern "C" int posfeat_model_conv_spec(int i, const char** name, int* cout, int* cin, int* kh,
                                       int* kw, long long* w_off, long long* b_off) {
  const auto& v = specs().v;
  if (i < 0 || i >= (int)v.size()) return POSFEAT_E_INVALID;
  const Spec& s = v[i];
  if (name) *name = s.name.c_str();
  if (cout) *cout = s.cout;
  if (cin) *cin = s.cin;
  if (kh) *kh = s.kh;
  if (kw) *kw = s.kw;
  if (w_off) *w_off = s.w_off;
  if (b_off) *b_off = s.b_off;
  return POSFEAT_OK;
}

extern "C" long long posfeat_model_weight_floats(void) { return specs().total; }

static void wstore_release(posfeat_wstore* s) {
  if (!s || --s->refs > 0) return;
  if (s->ev_fork) (void)hipEventDestroy(s->ev_fork);
  if (s->ev_join) (void)hipEventDestroy(s->ev_join);
  if (s->side_st) (void)hipStreamDestroy(s->side_st);
  if (s->ev) (void)hipEventDestroy(s->ev);
  if (s->base) (void)hipFree(s->base);
  delete s;
}

extern "C" int posfeat_model_create_shared(int batch, int h, int w, const float* weights,
                                           posfeat_model* share, posfeat_model** out) {
  if (!out || !weights || batch <= 0 || h < 16 || w < 16 || h % 16 || w % 16)
    return POSFEAT_E_INVALID;
  if (share && (!share->wcache || share->wts != weights)) return POSFEAT_E_INVALID;
  posfeat_model* m = new (std::nothrow) posfeat_model();
  if (!m) return POSFEAT_E_INVALID;
  m->B = batch;
  m->H = h;
  m->W = w;
  m->wts = weights;
  m->wcache = true;
  plan(m);  // host only: the derived-weight memory is allocated by the first forward
  posfeat_wstore* st = share ? share->store : nullptr;
  if (st && (st->bytes != m->p_bytes || st->wsplit != m->wsplit || st->bf6p != m->bf6p))
    st = nullptr;  // another layout (precision mode changed between the two): own store
  if (!st) {
    st = new (std::nothrow) posfeat_wstore();
    if (!st) {
      delete m;
      return POSFEAT_E_INVALID;
    }
    st->bytes = m->p_bytes;
    st->wts = weights;
    st->wsplit = m->wsplit;
    st->bf6p = m->bf6p;
  }
  ++st->refs;
  m->store = st;
  *out = m;
  return POSFEAT_OK;
}

extern "C" int posfeat_model_create(int batch, int h, int w, const float* weights,
                                    posfeat_model** out) {
  return posfeat_model_create_shared(batch, h, w, weights, nullptr, out);
}

// a forward that built derived weights records where they are complete; a
// later forward of any instance sharing the store (maybe on another stream)
// orders itself after that point
static int wprep_begin(posfeat_model* m, hipStream_t st) {
  if (!m->wcache) return POSFEAT_OK;
  posfeat_wstore* s = m->store;
  if (s->bytes && !s->base) {
    if (hipMalloc(reinterpret_cast<void**>(&s->base), s->bytes) != hipSuccess) {
      s->base = nullptr;
      return POSFEAT_E_HIP;
    }
    if (!s->ev && hipEventCreateWithFlags(&s->ev, hipEventDisableTiming) != hipSuccess)
      return POSFEAT_E_HIP;
  }
  if (s->ev && (s->wpl_done || !s->wino_done.empty()))
    if (hipStreamWaitEvent(st, s->ev, 0) != hipSuccess) return POSFEAT_E_HIP;
  return POSFEAT_OK;
}
static int wprep_end(posfeat_model* m, hipStream_t st, int r) {
  if (m->wprep_pending) {
    m->wprep_pending = false;
    if (r == POSFEAT_OK && hipEventRecord(m->store->ev, st) != hipSuccess) return POSFEAT_E_HIP;
    if (r != POSFEAT_OK) {  // a failed forward: build them again next time
      m->store->wpl_done = false;
      m->store->wino_done.clear();
    }
  }
  return r;
}

extern "C" int posfeat_model_weights_changed(posfeat_model* m) {
  if (!m) return POSFEAT_E_INVALID;
  if (m->store) {  // every instance sharing the store rebuilds
    m->store->wpl_done = false;
    m->store->wino_done.clear();
  }
  return POSFEAT_OK;
}

extern "C" size_t posfeat_model_workspace(const posfeat_model* m) { return m ? m->ws_bytes : 0; }

extern "C" int posfeat_tile_cache_export(char* buf, size_t cap, size_t* len) {
  const std::string t = tile_cache_text();
  if (len) *len = t.size() + 1;
  if (!buf) return POSFEAT_OK;
  if (cap < t.size() + 1) return POSFEAT_E_WORKSPACE;
  memcpy(buf, t.c_str(), t.size() + 1);
  return POSFEAT_OK;
}

extern "C" int posfeat_tile_cache_import(const char* text) {
  if (!text) return POSFEAT_E_INVALID;
  return tile_cache_load(text);
}

extern "C" int posfeat_model_extract(posfeat_model* m, const float* img_nchw,
                                     posfeat_extract_out* out, void* ws, size_t ws_bytes,
                                     void* stream) {
  if (!m || !img_nchw || !out || !out->local_point || !ws) return POSFEAT_E_INVALID;
  if (ws_bytes < m->ws_bytes) return POSFEAT_E_WORKSPACE;
  if (reinterpret_cast<uintptr_t>(ws) & 255) return POSFEAT_E_INVALID;
  Ctx c{m, static_cast<char*>(ws), pf_stream(stream)};
  m->ev_used = 0;
  PF_TRY(wprep_begin(m, c.st));
  const int r = wprep_end(m, c.st, forward(c, img_nchw, out));
  if (r == POSFEAT_OK) m->tuned_modes |= 1u << MODE_FULL;
  return r;
}

extern "C" int posfeat_model_backbone(posfeat_model* m, const float* img_nchw,
                                      posfeat_extract_out* out, void* ws, size_t ws_bytes,
                                      void* stream) {
  if (!m || !img_nchw || !out || !ws || m->train) return m && m->train ? POSFEAT_E_UNSUPPORTED
                                                                        : POSFEAT_E_INVALID;
  if (ws_bytes < m->ws_bytes) return POSFEAT_E_WORKSPACE;
  if (reinterpret_cast<uintptr_t>(ws) & 255) return POSFEAT_E_INVALID;
  Ctx c{m, static_cast<char*>(ws), pf_stream(stream)};
  m->ev_used = 0;
  PF_TRY(wprep_begin(m, c.st));
  const int r = wprep_end(m, c.st, forward(c, img_nchw, out, MODE_BACKBONE));
  if (r == POSFEAT_OK) m->tuned_modes |= 1u << MODE_BACKBONE;
  return r;
}

extern "C" int posfeat_model_keypointdet(posfeat_model* m, const float* x_nchw,
                                         const float* img_nchw, float* local_point, void* ws,
                                         size_t ws_bytes, void* stream) {
  if (!m || !x_nchw || !img_nchw || !local_point || !ws) return POSFEAT_E_INVALID;
  if (m->train) return POSFEAT_E_UNSUPPORTED;
  if (ws_bytes < m->ws_bytes) return POSFEAT_E_WORKSPACE;
  if (reinterpret_cast<uintptr_t>(ws) & 255) return POSFEAT_E_INVALID;
  Ctx c{m, static_cast<char*>(ws), pf_stream(stream)};
  m->ev_used = 0;
  posfeat_extract_out o{};
  o.local_point = local_point;
  PF_TRY(wprep_begin(m, c.st));
  const int r = wprep_end(m, c.st, forward(c, img_nchw, &o, MODE_HEAD, x_nchw));
  if (r == POSFEAT_OK) m->tuned_modes |= 1u << MODE_HEAD;
  return r;
}

extern "C" int posfeat_model_set_timing(posfeat_model* m, int enable) {
  if (!m) return POSFEAT_E_INVALID;
  m->timing = enable != 0;
  return POSFEAT_OK;
}

extern "C" int posfeat_model_timing(posfeat_model* m, const char* prefix, double* ms,
                                    double* flops, int* launches) {
  if (!m || !prefix) return POSFEAT_E_INVALID;
  double t = 0, f = 0;
  int k = 0;
  const size_t pl = strlen(prefix);
  for (size_t i = 0; i < m->ev_used; ++i) {
    auto& e = m->evs[i];
    if (e.label.compare(0, pl, prefix) != 0) continue;
    if (hipEventSynchronize(e.b) != hipSuccess) return POSFEAT_E_HIP;
    float dt = 0.f;
    if (hipEventElapsedTime(&dt, e.a, e.b) != hipSuccess) return POSFEAT_E_HIP;
    t += dt;
    f += e.flops;
    ++k;
  }
  if (ms) *ms = t;
  if (flops) *flops = f;
  if (launches) *launches = k;
  return POSFEAT_OK;
}

extern "C" int posfeat_model_timing_event(posfeat_model* m, int i, const char** label, double* ms,
                                          double* flops) {
  if (!m || i < 0 || (size_t)i >= m->ev_used) return POSFEAT_E_INVALID;
  auto& e = m->evs[i];
  if (hipEventSynchronize(e.b) != hipSuccess) return POSFEAT_E_HIP;
  float dt = 0.f;
  if (hipEventElapsedTime(&dt, e.a, e.b) != hipSuccess) return POSFEAT_E_HIP;
  if (label) *label = e.label.c_str();
  if (ms) *ms = dt;
  if (flops) *flops = e.flops;
  return POSFEAT_OK;
}

extern "C" void posfeat_model_destroy(posfeat_model* m) {
  if (!m) return;
  for (auto& e : m->evs) {
    (void)hipEventDestroy(e.a);
    (void)hipEventDestroy(e.b);
  }
  if (!m->store) {  // else the store's (released with its last instance)
    if (m->ev_fork) (void)hipEventDestroy(m->ev_fork);
    if (m->ev_join) (void)hipEventDestroy(m->ev_join);
    if (m->side_st) (void)hipStreamDestroy(m->side_st);
  }
  wstore_release(m->store);
  delete m;
}

extern "C" const char* posfeat_strerror(int code) {
  switch (code) {
    case POSFEAT_OK: return "ok";
    case POSFEAT_E_INVALID: return "posfeat: invalid argument or unsupported shape";
    case POSFEAT_E_HIP: return "posfeat: HIP runtime error";
    case POSFEAT_E_WORKSPACE: return "posfeat: workspace too small";
    case POSFEAT_E_UNSUPPORTED: return "posfeat: unsupported option";
    default: return "posfeat: unknown error";
  }
}

extern "C" int posfeat_abi_version(void) { return 1; }

extern "C" int posfeat_device_ok(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) return 0;
  return strncmp(p.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

// 1 in the A/B build (make ab: the POSFEAT_* path switches are read), 0 in
// the shipped library (common.h pf_ab_getenv)
extern "C" int posfeat_ab_build(void) { return POSFEAT_AB ? 1 : 0; }

// the PF_ARITH_* mask of the i-th timed label's MFMA launches (1: fp32 MFMA,
// 2: bf16x6, 3: both, 0: none), for bench.py's rooflines
extern "C" int posfeat_model_timing_event_arith(posfeat_model* m, int i) {
  if (!m || i < 0 || (size_t)i >= m->ev_used) return POSFEAT_E_INVALID;
  return m->evs[i].arith;
}
