// bbtrain.hip -- train-mode ResUNet forward / backward and Adam for the
// descriptor-training step (configs/train_desc.yaml: optimal_modules
// ['backbone'], Adam lr 1e-4; managers/trainer.py:293-331).
//
// Network: networks/DescNet.py:11-84 (ResNet-50 encoder cut after layer3,
// U-Net decoder; conv = Conv2d -> BatchNorm2d -> ELU at 167-179, upconv =
// bilinear x2 align_corners=True -> conv at 182-190) with BatchNorm in
// training mode: batch statistics over (N, H, W) of each forward call and a
// running-stat update (momentum 0.1, unbiased variance), as torch.nn.BatchNorm2d
// does under backbone.train() (trainer.py:293-296).  PoSFeat.forward runs the
// backbone once per image batch (PoSFeat_model.py:144-145), so im1 and im2
// each get their own statistics: one activation workspace per batch.
//
// Forward: every conv writes its raw output y (NHWC, compact); the BN
// statistics are fp64 partial sums in a fixed order (deterministic); the apply
// pass writes act(gamma (y - mean) rstd + beta [+ residual]) straight into the
// channel slices of the decoder's concat buffers.  Everything the backward
// reads stays resident (~6 GB per 8 x 480 x 640 batch; 288 GB of HBM).
//
// Backward of one conv + BN + act layer:
//   g  = da * act'(a)                      (ReLU: a > 0; ELU: a > 0 ? 1 : a + 1)
//   dgamma = sum g x^, dbeta = sum g,  dy = gamma rstd (g - E[g] - x^ E[g x^])
//   dW, db  = MFMA weight gradient (train.hip, stride 1 or 2)
//   dx      = forward conv of dy with flipped, channel-transposed weights
//             (stride 2: dy zero-inserted onto the input grid first)
// Max-pool (ATen first-max rule) and the x2 align_corners upsample have
// gather adjoints: no atomics, bit-reproducible.  Kernels: bbtrain_kernels.h.
//
// The keypoint head is not run: in this config its output feeds neither the
// loss (EpipolarLoss_full reads local_map only) nor any state (InstanceNorm
// keeps no running statistics, the head is not optimised).  conv_coarse gets
// no gradient (global_map is read at losses/preprocess.py:28-29 and never
// used) but its BN running statistics are updated, as the reference forward does.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "bbtrain_kernels.h"
#include "group.h"
#include "common.h"
#include "fmap.h"
#include "train.h"

using namespace bbt;

namespace {

// ------------------------------------------------------------------ layer table
struct TLayer {
  std::string name;  // engine naming (weights.conv_sources maps it to state-dict keys)
  int cin, cout, k, stride, act;
  bool bias;
  long long w_off, b_off, g_off, be_off;  // parameter / gradient blob (floats); b_off -1: no bias
  long long rm_off, rv_off;               // running-statistics blob
};

struct TTable {
  std::vector<TLayer> v;
  long long params = 0, stats = 0;
  int first, coarse, up3, ic3, up2, ic2, fine;
  TTable() {
    auto take = [&](long long nf) {
      const long long o = params;
      params += (nf + 63) / 64 * 64;
      return o;
    };
    auto add = [&](const std::string& n, int ci, int co, int k, int s, int act, bool bias) {
      TLayer L{n, ci, co, k, s, act, bias, 0, -1, 0, 0, 0, 0};
      L.w_off = take((long long)co * posfeat_conv_packed_k(ci, k, k));
      if (bias) L.b_off = take(co);
      L.g_off = take(co);
      L.be_off = take(co);
      L.rm_off = stats;
      stats += (co + 63) / 64 * 64;
      L.rv_off = stats;
      stats += (co + 63) / 64 * 64;
      v.push_back(L);
      return (int)v.size() - 1;
    };
    first = add("firstconv", 3, 64, 7, 2, ACT_RELU, false);
    const int planes[3] = {64, 128, 256}, blocks[3] = {3, 4, 6};
    int inpl = 64;
    for (int l = 0; l < 3; ++l)
      for (int bi = 0; bi < blocks[l]; ++bi) {
        const std::string p = "layer" + std::to_string(l + 1) + "." + std::to_string(bi);
        const int s = (bi == 0 && l > 0) ? 2 : 1;
        add(p + ".conv1", inpl, planes[l], 1, 1, ACT_RELU, false);
        add(p + ".conv2", planes[l], planes[l], 3, s, ACT_RELU, false);
        add(p + ".conv3", planes[l], planes[l] * 4, 1, 1, ACT_RELU, false);  // ReLU after + residual
        if (bi == 0) add(p + ".downsample", inpl, planes[l] * 4, 1, s, ACT_NONE, false);
        inpl = planes[l] * 4;
      }
    coarse = add("conv_coarse", 1024, 128, 1, 1, ACT_ELU, true);
    up3 = add("upconv3.conv", 1024, 512, 3, 1, ACT_ELU, true);
    ic3 = add("iconv3", 1024, 512, 3, 1, ACT_ELU, true);
    up2 = add("upconv2.conv", 512, 256, 3, 1, ACT_ELU, true);
    ic2 = add("iconv2", 512, 256, 3, 1, ACT_ELU, true);
    fine = add("conv_fine", 256, 128, 1, 1, ACT_ELU, true);
  }
  int find(const std::string& n) const {
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i].name == n) return (int)i;
    return -1;
  }
};

const TTable& tab() {
  static TTable t;
  return t;
}

struct BnGrid {
  int qpb, gy, R, chunk, nchunk;
};

// chunking of bn_partial_kernel: ~1024 blocks, chunk a multiple of the row count
BnGrid bn_grid(long long P, int C) {
  BnGrid g;
  const int c4n = C / 4;
  g.qpb = std::min(c4n, 64);
  g.gy = c4n / g.qpb;
  g.R = 256 / g.qpb;
  long long want = std::max(1LL, (1024LL + g.gy - 1) / g.gy);
  const long long rows = (P + g.R - 1) / g.R;
  want = std::min(want, rows);
  long long chunk = (P + want - 1) / want;
  chunk = (chunk + g.R - 1) / g.R * g.R;
  g.chunk = (int)chunk;
  g.nchunk = (int)((P + chunk - 1) / chunk);
  return g;
}

int grid_for(long long total, int block) {
  long long g = (total + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

struct Buf {
  size_t off = 0, bytes = 0;
};

}  // namespace

// ------------------------------------------------------------------ handle
struct posfeat_bbtrain {
  int B, H, W;
  // activation workspace (one per image batch)
  size_t act_bytes = 0;
  Buf img4, a0, mp, mpidx, cat2, cat3, l3out, up3, i3a, up2, i2a, fa;
  std::vector<Buf> y, st;         // per layer: raw conv output, mean|rstd
  std::vector<Buf> vk;            // per F(6x6) decoder layer: the forward's V
  std::vector<Buf> a1, a2, bout;  // per bottleneck
  // scratch (shared by the batches: forward transients + backward)
  size_t scr_bytes = 0;
  Buf dsn, part, coef, ga, gb, gc, gd, gres, dy, dz, dcat2, dcat3, dup, upt, wgws, splitk;
  // SyncBatchNorm (posfeat_bbtrain_set_group): statistics summed over the
  // group's ranks; bnsum holds [local | group] sums of one layer
  posfeat_group* group = nullptr;
  Buf bnsum;
  // Winograd F(2x2,3x3) for the decoder's 3x3 convs, forward and input
  // gradient (wino.hip; POSFEAT_WINO=0: direct conv)
  bool wino = true;
  bool wino6 = true;  // F(6x6) forward + input gradient (POSFEAT_TRAIN_WINO6=0, A/B: F(4x4))
  bool wino6_wg = true;  // F(6x6) weight gradient (POSFEAT_TRAIN_WINO6_WGRAD=0, A/B: F(4x4))
  // BatchNorm forward statistics from the conv epilogue (fp64 per-tile sums of
  // y; POSFEAT_TRAIN_BN_EPI=0, A/B: the separate bn_partial_kernel<0> pass)
  bool bn_epi = true;
  // the direct convs on the tile database's tiles (engine.hip
  // pf_conv_tuned_run: exact entries only, never timed live unless
  // POSFEAT_TRAIN_TUNE_LIVE=1; POSFEAT_TRAIN_TUNE=0, A/B: the default plan)
  bool tune = true;
  bool bf6p = false;     // conv precision mode 2 at create (pre-split Winograd operands)
  bool s2phase = true;  // stride-2 input gradients by output phases (POSFEAT_S2PHASE=0: zero insertion)
  Buf wu, wino_ws;
  // pre-split bf16x6 operands (conv precision 1, POSFEAT_BF6B=0: off): the
  // parameter blob's three bf16 planes (split at the start of each forward:
  // Adam moves the parameters between calls) and those of the transposed
  // input-gradient weights, so the row-tile convs run conv_bf6b_kernel
  // (weights read ready-made) instead of splitting both operands per wave --
  // the same products in the same order: bit-identical results
  bool wsplit = false;
  Buf wpl;
  // the input-gradient weights of every layer (transposed / phase weights,
  // their bf16 planes, the Winograd U): derived by an accumulate = 0
  // backward, reused by the accumulate = 1 call of the same step.  bw_valid
  // records that they were derived from `bw_params` into `bw_scratch` with no
  // forward since (a forward starts a new step: the parameters may have moved);
  // an accumulate = 1 call without that rebuilds them
  Buf bw;
  bool bw_valid = false, derive_now = true;
  const float* bw_params = nullptr;
  const void* bw_scratch = nullptr;
  std::vector<size_t> bw_wt, bw_wtp, bw_u;  // float offsets into bw
  // optional per-launch timing (labels "fwd:conv", "bwd:wgrad", ...)
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

struct Blk {
  int li, bi, pl, stride, inpl;
  bool ds;
  int c1, c2, c3, cds;  // layer indices
};

const std::vector<Blk>& blocks() {
  static const std::vector<Blk> v = [] {
    std::vector<Blk> r;
    const int planes[3] = {64, 128, 256}, nb[3] = {3, 4, 6};
    int inpl = 64;
    for (int l = 0; l < 3; ++l)
      for (int bi = 0; bi < nb[l]; ++bi) {
        Blk b;
        b.li = l;
        b.bi = bi;
        b.pl = planes[l];
        b.stride = (bi == 0 && l > 0) ? 2 : 1;
        b.inpl = inpl;
        b.ds = bi == 0;
        const std::string p = "layer" + std::to_string(l + 1) + "." + std::to_string(bi);
        b.c1 = tab().find(p + ".conv1");
        b.c2 = tab().find(p + ".conv2");
        b.c3 = tab().find(p + ".conv3");
        b.cds = b.ds ? tab().find(p + ".downsample") : -1;
        r.push_back(b);
        inpl = planes[l] * 4;
      }
    return r;
  }();
  return v;
}

struct Ctx {
  posfeat_bbtrain* m;
  char* act;
  char* scr;
  hipStream_t st;
  const float* prm;
  float* f(const Buf& b) const { return reinterpret_cast<float*>(act + b.off); }
  float* s(const Buf& b) const { return reinterpret_cast<float*>(scr + b.off); }
  double* sd(const Buf& b) const { return reinterpret_cast<double*>(scr + b.off); }
  unsigned short* su(const Buf& b) const { return reinterpret_cast<unsigned short*>(scr + b.off); }
};

template <class F>
int timed(Ctx& c, const std::string& label, double flops, F&& fn) {
  posfeat_bbtrain* m = c.m;
  if (!m->timing) return fn();
  if (m->ev_used == m->evs.size()) {
    posfeat_bbtrain::Ev e;
    if (hipEventCreate(&e.a) != hipSuccess || hipEventCreate(&e.b) != hipSuccess)
      return POSFEAT_E_HIP;
    m->evs.push_back(e);
  }
  auto& e = m->evs[m->ev_used++];
  e.label = label;
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

posfeat_conv_desc make_desc(int n, int h, int w, int cin, int xcs, int cout, int k, int stride,
                            int ycs, int rcs) {
  posfeat_conv_desc d;
  d.n = n;
  d.h = h;
  d.w = w;
  d.cin = (cin + 3) / 4 * 4;
  d.x_cstride = xcs;
  d.cout = cout;
  d.kh = d.kw = k;
  d.stride = stride;
  d.pad = (k - 1) / 2;
  d.y_cstride = ycs;
  d.res_cstride = rcs;
  d.act = POSFEAT_ACT_NONE;
  return d;
}

inline int out_dim(int h, int k, int s) { return (h + 2 * ((k - 1) / 2) - k) / s + 1; }

// the decoder's 3x3 stride-1 convs go through Winograd F(2x2,3x3)
bool use_wino(const posfeat_bbtrain* m, int li, int h, int w) {
  const TTable& T = tab();
  return m->wino && (li == T.up3 || li == T.ic3 || li == T.up2 || li == T.ic2) && !(h & 1) &&
         !(w & 1);
}

// a decoder layer whose F(6x6) forward keeps V for its F(6x6) weight gradient
bool vkeep_layer(const posfeat_bbtrain* m, int li) {
  const TLayer& L = tab().v[li];
  return m->wino && m->wino6 && m->wino6_wg && L.cin % 128 == 0 && L.cout % 128 == 0;
}

// input spatial size of every layer (forward order of DescNet.py:64-84)
void layer_inputs(int H, int W, std::vector<int>& ih, std::vector<int>& iw) {
  const TTable& T = tab();
  ih.assign(T.v.size(), 0);
  iw.assign(T.v.size(), 0);
  ih[T.first] = H;
  iw[T.first] = W;
  int h = H / 4, w = W / 4;
  for (const Blk& b : blocks()) {
    const int oh = (h - 1) / b.stride + 1, ow = (w - 1) / b.stride + 1;
    ih[b.c1] = ih[b.c2] = h;
    iw[b.c1] = iw[b.c2] = w;
    ih[b.c3] = oh;
    iw[b.c3] = ow;
    if (b.ds) {
      ih[b.cds] = h;
      iw[b.cds] = w;
    }
    h = oh;
    w = ow;
  }
  ih[T.coarse] = H / 16;
  iw[T.coarse] = W / 16;
  ih[T.up3] = ih[T.ic3] = H / 8;
  iw[T.up3] = iw[T.ic3] = W / 8;
  ih[T.up2] = ih[T.ic2] = ih[T.fine] = H / 4;
  iw[T.up2] = iw[T.ic2] = iw[T.fine] = W / 4;
}

void plan(posfeat_bbtrain* m) {
  const TTable& T = tab();
  const size_t B = m->B, H = m->H, W = m->W;
  const size_t h2 = H / 2, w2 = W / 2, h4 = H / 4, w4 = W / 4, h8 = H / 8, w8 = W / 8, h16 = H / 16,
               w16 = W / 16;
  size_t cur = 0;
  auto alloc = [&](Buf& b, size_t bytes) {
    b.off = cur;
    b.bytes = bytes;
    cur += pf_align(bytes, 256);
  };
  auto fl = [](size_t n) { return n * sizeof(float); };
  std::vector<int> lih, liw;
  layer_inputs(m->H, m->W, lih, liw);
  {  // path switches (A/B build), fixed for the handle: buffer sizes depend on them
    const char* e = pf_ab_getenv("POSFEAT_WINO");
    m->wino = !(e && e[0] == '0');
    const char* s2 = pf_ab_getenv("POSFEAT_S2PHASE");
    m->s2phase = !(s2 && s2[0] == '0');
    m->bf6p = pf_bf6p_on();
    const char* w6 = pf_ab_getenv("POSFEAT_TRAIN_WINO6");
    m->wino6 = !(w6 && w6[0] == '0') && !m->bf6p;
    const char* g = pf_ab_getenv("POSFEAT_TRAIN_WINO6_WGRAD");
    m->wino6_wg = !(g && g[0] == '0');
    const char* be = pf_ab_getenv("POSFEAT_TRAIN_BN_EPI");
    m->bn_epi = !(be && be[0] == '0');
    const char* tu = pf_ab_getenv("POSFEAT_TRAIN_TUNE");
    m->tune = !(tu && tu[0] == '0');
  }
  // ---- activations
  alloc(m->img4, fl(B * H * W * 4));
  alloc(m->a0, fl(B * h2 * w2 * 64));
  alloc(m->mp, fl(B * h4 * w4 * 64));
  alloc(m->mpidx, fl(B * h4 * w4 * 16));  // arg-max taps, one byte per channel
  alloc(m->cat2, fl(B * h4 * w4 * 512));
  alloc(m->cat3, fl(B * h8 * w8 * 1024));
  alloc(m->l3out, fl(B * h16 * w16 * 1024));
  alloc(m->up3, fl(B * h8 * w8 * 1024));
  alloc(m->i3a, fl(B * h8 * w8 * 512));
  alloc(m->up2, fl(B * h4 * w4 * 512));
  alloc(m->i2a, fl(B * h4 * w4 * 256));
  alloc(m->fa, fl(B * h4 * w4 * 128));
  const auto& bl = blocks();
  m->a1.assign(bl.size(), Buf());
  m->a2.assign(bl.size(), Buf());
  m->bout.assign(bl.size(), Buf());
  for (size_t i = 0; i < bl.size(); ++i) {
    const Blk& b = bl[i];
    const size_t ih = lih[b.c1], iw = liw[b.c1], oh = lih[b.c3], ow = liw[b.c3];
    alloc(m->a1[i], fl(B * ih * iw * b.pl));
    alloc(m->a2[i], fl(B * oh * ow * b.pl));
    const bool last = i + 1 == bl.size() || bl[i + 1].li != b.li;
    if (!last) alloc(m->bout[i], fl(B * oh * ow * b.pl * 4));
  }
  m->y.assign(T.v.size(), Buf());
  m->st.assign(T.v.size(), Buf());
  for (size_t li = 0; li < T.v.size(); ++li) {
    const TLayer& L = T.v[li];
    const size_t oh = out_dim(lih[li], L.k, L.stride), ow = out_dim(liw[li], L.k, L.stride);
    alloc(m->y[li], fl(B * oh * ow * L.cout));
    alloc(m->st[li], fl(2 * (size_t)L.cout));
  }
  // the F(6x6) decoder layers' transformed inputs V, kept from the forward for
  // their weight gradient (pf_wino6_conv vkeep -> pf_wino6_wgrad vpre)
  m->vk.assign(T.v.size(), Buf());
  for (int li : {T.up3, T.ic3, T.up2, T.ic2})
    if (vkeep_layer(m, li))
      alloc(m->vk[li], fl(pf_wino6_v_floats((int)B, lih[li], liw[li], T.v[li].cin)));
  m->act_bytes = cur;
  // ---- scratch
  cur = 0;
  const size_t MAXG = B * h4 * w4 * 256;  // largest gradient map (= B*h2*w2*64)
  alloc(m->dsn, fl(MAXG));
  alloc(m->part, 2 * 1100 * 1024 * sizeof(double));
  alloc(m->coef, fl(3 * 1024));
  alloc(m->bnsum, 2 * BN_SUM_SLOT * sizeof(double));
  alloc(m->ga, fl(MAXG));
  alloc(m->gb, fl(MAXG));
  alloc(m->gc, fl(MAXG));
  alloc(m->gd, fl(MAXG));
  alloc(m->gres, fl(MAXG));
  alloc(m->dy, fl(MAXG));

  alloc(m->dcat2, fl(B * h4 * w4 * 512));
  alloc(m->dcat3, fl(B * h8 * w8 * 1024));
  alloc(m->dup, fl(std::max(B * h4 * w4 * 512, B * h8 * w8 * 1024)));
  alloc(m->upt, fl(std::max(B * h4 * w8 * 512, B * h8 * w16 * 1024)));
  size_t wg = 0, sk = 0, dzf = 0;
  for (size_t li = 0; li < T.v.size(); ++li) {
    const TLayer& L = T.v[li];
    const int cinp = (L.cin + 3) / 4 * 4;
    wg = std::max(wg, pf_conv_wgrad_ws_bytes((int)B, lih[li], liw[li], cinp, L.cout, L.k, L.k,
                                             L.stride));
    posfeat_conv_desc d = make_desc((int)B, lih[li], liw[li], L.cin, cinp, L.cout, L.k, L.stride,
                                    L.cout, 0);
    sk = std::max(sk, posfeat_conv2d_workspace(&d));
    if ((int)li != T.first) {
      if (L.stride == 2 && L.k == 3) {
        posfeat_conv_desc e2 = make_desc((int)B, lih[li] / 2, liw[li] / 2, L.cout, L.cout,
                                         4 * L.cin, 2, 1, 4 * L.cin, 0);
        e2.pad = 1;
        sk = std::max(sk, posfeat_conv2d_workspace(&e2));
        dzf = std::max(dzf, (size_t)B * (lih[li] / 2 + 1) * (liw[li] / 2 + 1) * 4 * L.cin);
      }
      posfeat_conv_desc e = make_desc((int)B, lih[li], liw[li], L.cout, L.cout, L.cin, L.k, 1,
                                      L.cin, L.cin);
      sk = std::max(sk, posfeat_conv2d_workspace(&e));
    }
  }
  {
    const char* e = pf_ab_getenv("POSFEAT_BF6B");
    m->wsplit = pf_conv_precision() == 1 && !(e && e[0] == '0') && T.params % 4 == 0;
  }
  if (m->wsplit) alloc(m->wpl, (size_t)T.params * 6);
  alloc(m->dz, fl(std::max(dzf, 2 * MAXG)));
  alloc(m->wgws, wg);
  alloc(m->splitk, std::max<size_t>(sk, 256));
  if (m->wino) {
    size_t uf = 0, wb = 0;
    for (int li : {T.up3, T.ic3, T.up2, T.ic2}) {
      const TLayer& L = T.v[li];
      uf = std::max(uf, (size_t)(m->bf6p || m->wsplit ? 54 : 36) * L.cin * L.cout);
      if (m->wino6) {
        uf = std::max(uf, pf_wino6_weights_floats(L.cin, L.cout, m->wsplit));
        wb = std::max(wb, pf_wino6_ws_bytes((int)B, lih[li], liw[li], L.cin, L.cout));
        wb = std::max(wb, pf_wino6_ws_bytes((int)B, lih[li], liw[li], L.cout, L.cin));
      }
      wb = std::max(wb, pf_wino_ws_bytes((int)B, lih[li], liw[li], L.cin, L.cout));
      wb = std::max(wb, pf_wino_ws_bytes((int)B, lih[li], liw[li], L.cout, L.cin));
      if (lih[li] % 4 == 0 && liw[li] % 4 == 0)
        wb = std::max(wb, pf_wino_wgrad_ws_bytes((int)B, lih[li], liw[li], L.cin, L.cout));
      if (m->wino6_wg && L.cin % 128 == 0 && L.cout % 128 == 0)
        wb = std::max(wb, pf_wino6_wgrad_ws_bytes((int)B, lih[li], liw[li], L.cin, L.cout));
    }
    alloc(m->wu, fl(uf));
    alloc(m->wino_ws, wb);
  }
  {  // per-layer input-gradient weights (layer_bwd), 64-float aligned slots
    size_t tot = 0;
    auto slot = [&](size_t floats) {
      const size_t o = tot;
      tot += (floats + 63) / 64 * 64;
      return o;
    };
    m->bw_wt.assign(T.v.size(), 0);
    m->bw_wtp.assign(T.v.size(), 0);
    m->bw_u.assign(T.v.size(), 0);
    for (size_t li = 0; li < T.v.size(); ++li) {
      if ((int)li == T.first) continue;
      const TLayer& L = T.v[li];
      const bool s2k3 = L.stride == 2 && m->s2phase && L.k == 3;
      const size_t rows = s2k3 ? 4 * (size_t)L.cin : L.cin;
      const size_t cols = s2k3 ? posfeat_conv_packed_k(L.cout, 2, 2)
                               : posfeat_conv_packed_k(L.cout, L.k, L.k);
      m->bw_wt[li] = slot(rows * cols);
      if (m->wsplit) m->bw_wtp[li] = slot(rows * cols * 3 / 2 + 64);
      if (m->wino && (li == (size_t)T.up3 || li == (size_t)T.ic3 || li == (size_t)T.up2 ||
                      li == (size_t)T.ic2))
        m->bw_u[li] = slot(std::max(pf_wino6_weights_floats(L.cout, L.cin, m->wsplit),
                                    (size_t)54 * L.cin * L.cout));
    }
    alloc(m->bw, fl(tot));
  }
  m->scr_bytes = cur;
}

// executed transform-domain MACs x2 of a Winograd layer: F(4x4) 36 per 4x4
// tile, F(2x2) 16 per 2x2 tile (what the MFMA units run, for the rooflines)
double wino_flops(int n, int h, int w, int cin, int cout, bool wgrad = false) {
  const char* e = pf_ab_getenv("POSFEAT_WINO");
  const bool f4 = h % 4 == 0 && w % 4 == 0 && (wgrad || !(e && e[0] == '1'));
  const double T = f4 ? (double)n * (h / 4) * (w / 4) : (double)n * (h / 2) * (w / 2);
  return 2.0 * T * (f4 ? 36 : 16) * cin * cout;
}

// ------------------------------------------------------------------ layer passes
// conv -> BN (batch statistics, running update) -> act(. + res) into out (cs ocs);
// out == nullptr: statistics only (conv_coarse)
int layer_fwd(Ctx& c, int li, const float* x, int xcs, int h, int w, float* out, int ocs,
              float* stats, float mom, const float* res = nullptr, int rcs = 0) {
  const TLayer& L = tab().v[li];
  posfeat_bbtrain* m = c.m;
  const int oh = out_dim(h, L.k, L.stride), ow = out_dim(w, L.k, L.stride);
  const long long P = (long long)m->B * oh * ow;
  float* y = c.f(m->y[li]);
  posfeat_conv_desc d = make_desc(m->B, h, w, L.cin, xcs, L.cout, L.k, L.stride, L.cout, 0);
  if (use_wino(m, li, h, w) && m->wino6) {
    float* U = c.s(m->wu);
    const double T6 = (double)m->B * ((h + 5) / 6) * ((w + 5) / 6);
    PF_TRY(timed(c, std::string("fwd:conv:") + L.name, 2.0 * T6 * 64 * L.cin * L.cout, [&] {
      PF_TRY(pf_wino6_weights(c.prm + L.w_off, L.cout, L.cin, U, c.st, m->wsplit));
      return pf_wino6_conv(x, xcs, m->B, h, w, L.cin, U, c.prm + L.b_off, L.cout, ACT_NONE, y,
                           L.cout, c.s(m->wino_ws), m->wino_ws.bytes, c.st, 7, m->wsplit ? 1 : 0,
                           0, vkeep_layer(m, li) ? c.f(m->vk[li]) : nullptr);
    }));
  } else if (use_wino(m, li, h, w)) {
    float* U = c.s(m->wu);
    PF_TRY(timed(c, std::string("fwd:conv:") + L.name, wino_flops(m->B, h, w, L.cin, L.cout), [&] {
      PF_TRY(pf_wino_weights_hw(c.prm + L.w_off, L.cout, L.cin, h, w, U, c.st,
                                m->bf6p || m->wsplit));
      return pf_wino_conv(x, xcs, m->B, h, w, L.cin, U, c.prm + L.b_off, L.cout, ACT_NONE, y,
                          L.cout, c.s(m->wino_ws), m->wino_ws.bytes, c.st, 7,
                          m->bf6p ? 2 : m->wsplit ? 1 : 0);
    }));
  }
  // BN statistics: the conv epilogue's per-tile fp64 sums when the direct
  // conv produced them (nparts > 0), else the statistics pass over y
  int nparts = 0;
  if (!use_wino(m, li, h, w)) {
    PF_TRY(timed(c, std::string("fwd:conv:") + L.name, 2.0 * P * L.cout * L.cin * L.k * L.k, [&] {
      const unsigned short* wb = m->wsplit ? c.su(m->wpl) + L.w_off : nullptr;
      const float* bias = L.bias ? c.prm + L.b_off : nullptr;
      auto run = [&](int tile) {
        if (m->bn_epi)
          return pf_conv_run_tile_bn(&d, x, c.prm + L.w_off, bias, y, c.s(m->splitk),
                                     m->splitk.bytes, tile, c.st, wb, tab().params,
                                     c.sd(m->part), m->part.bytes, &nparts);
        return pf_conv_run_tile(&d, x, c.prm + L.w_off, bias, nullptr, y, c.s(m->splitk),
                                m->splitk.bytes, tile, c.st, wb, tab().params);
      };
      return m->tune ? pf_conv_tuned_run(&d, false, wb != nullptr, c.st, run) : run(-1);
    }));
  }
  float* mean = c.f(m->st[li]);
  float* rstd = mean + L.cout;
  const BnGrid g = bn_grid(P, L.cout);
  const int nchunk = nparts > 0 ? nparts : g.nchunk;
  const int c4n = L.cout / 4;
  const int world = pf_group_world(m->group);
  return timed(c, "fwd:bn", 0, [&] {
    if (nparts == 0)
      hipLaunchKernelGGL(bn_partial_kernel<0>, dim3(g.nchunk, g.gy), dim3(256), 0, c.st, y, P,
                         L.cout, g.chunk, nullptr, 0, nullptr, 0, 0, nullptr, nullptr, nullptr,
                         nullptr, c.sd(m->part));
    if (world == 1) {
      hipLaunchKernelGGL(bn_stats_final_kernel, dim3((L.cout + 3) / 4), dim3(256), 0, c.st,
                         c.sd(m->part), nchunk, L.cout, P, mom, mean, rstd,
                         stats ? stats + L.rm_off : nullptr, stats ? stats + L.rv_off : nullptr);
    } else {  // SyncBatchNorm: sums and pixel counts over the group
      double* sums = c.sd(m->bnsum);
      hipLaunchKernelGGL(bn_sums_kernel, dim3((L.cout + 3) / 4), dim3(256), 0, c.st,
                         c.sd(m->part), nchunk, L.cout, (double)P, sums, nullptr);
      PF_CHECK_LAUNCH();
      PF_TRY(pf_group_allreduce(m->group, sums, 2 * L.cout + 1, c.st));
      hipLaunchKernelGGL(bn_stats_from_sums_kernel, dim3((L.cout + 255) / 256), dim3(256), 0,
                         c.st, sums, L.cout, mom, mean, rstd,
                         stats ? stats + L.rm_off : nullptr, stats ? stats + L.rv_off : nullptr);
    }
    if (out)
      hipLaunchKernelGGL(bn_apply_kernel, dim3(grid_for(P * c4n, 256)), dim3(256), 0, c.st, y, P,
                         c4n, mean, rstd, c.prm + L.g_off, c.prm + L.be_off, res, rcs, L.act, out,
                         ocs);
    PF_CHECK_LAUNCH();
    return POSFEAT_OK;
  });
}

int upsample_adjoint(Ctx& c, const float* g, int gcs, int h, int w, int C, float* d, int dcs) {
  const int OH = 2 * h, OW = 2 * w, c4n = C / 4, B = c.m->B;
  float* t = c.s(c.m->upt);
  return timed(c, "bwd:misc", 0, [&] {
    hipLaunchKernelGGL(up2_adj_x_kernel, dim3(grid_for((long long)B * OH * w * c4n, 256)),
                       dim3(256), 0, c.st, g, gcs, B, OH, OW, w, c4n, t);
    hipLaunchKernelGGL(up2_adj_y_kernel, dim3(grid_for((long long)B * h * w * c4n, 256)), dim3(256),
                       0, c.st, t, B, OH, h, w, c4n, d, dcs);
    PF_CHECK_LAUNCH();
    return POSFEAT_OK;
  });
}

// Backward of conv li (input x at h x w) + BN + act, given da = dL/d(act out).
// gres: optional copy of g (the residual branch's gradient, conv3).
// dx (cs dxcs): input gradient (+ add, cs addcs) when non-null.
int layer_bwd(Ctx& c, int li, const float* x, int xcs, int h, int w, const float* a, int acs,
              const float* da, int dacs, float* grad, int acc, float* gres, float* dx, int dxcs,
              const float* add, int addcs, bool residual = false) {
  const TLayer& L = tab().v[li];
  posfeat_bbtrain* m = c.m;
  const int B = m->B;
  // act'(a) of a non-residual layer from y (a = act(BN(y)), recomputed exactly
  // as the forward did) rather than another read of the stored activation
  const float* as = residual ? a : nullptr;
  const int oh = out_dim(h, L.k, L.stride), ow = out_dim(w, L.k, L.stride);
  const long long P = (long long)B * oh * ow;
  const int C = L.cout, c4n = C / 4;
  const float* y = c.f(m->y[li]);
  const float* mean = c.f(m->st[li]);
  const float* rstd = mean + C;
  float* coef = c.s(m->coef);
  float* dy = c.s(m->dy);
  const BnGrid g = bn_grid(P, C);
  PF_TRY(timed(c, "bwd:bn", 0, [&] {
    hipLaunchKernelGGL(bn_partial_kernel<1>, dim3(g.nchunk, g.gy), dim3(256), 0, c.st, y, P, C,
                       g.chunk, as, acs, da, dacs, L.act, mean, rstd, c.prm + L.g_off,
                       c.prm + L.be_off, c.sd(m->part));
    const int world = pf_group_world(m->group);
    if (world == 1) {
      hipLaunchKernelGGL(bn_bwd_final_kernel, dim3((C + 3) / 4), dim3(256), 0, c.st,
                         c.sd(m->part), g.nchunk, C, P, c.prm + L.g_off, rstd, grad + L.g_off,
                         grad + L.be_off, acc, coef);
    } else {  // SyncBatchNorm backward: E[g], E[g x^] over the group's count
      double* loc = c.sd(m->bnsum);
      double* grp = loc + BN_SUM_SLOT;
      hipLaunchKernelGGL(bn_sums_kernel, dim3((C + 3) / 4), dim3(256), 0, c.st, c.sd(m->part),
                         g.nchunk, C, (double)P, loc, grp);
      PF_CHECK_LAUNCH();
      PF_TRY(pf_group_allreduce(m->group, grp, 2 * C + 1, c.st));
      hipLaunchKernelGGL(bn_bwd_from_sums_kernel, dim3((C + 255) / 256), dim3(256), 0, c.st, loc,
                         grp, C, c.prm + L.g_off, rstd, grad + L.g_off,
                         grad + L.be_off, acc, coef);
    }
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_for(P * c4n, 256)), dim3(256), 0, c.st, y, P,
                       c4n, as, acs, da, dacs, L.act, mean, rstd, c.prm + L.g_off, c.prm + L.be_off,
                       coef, dy, gres);
    PF_CHECK_LAUNCH();
    return POSFEAT_OK;
  }));
  const double flops = 2.0 * P * C * L.cin * L.k * L.k;
  const int cinp = (L.cin + 3) / 4 * 4;
  if (use_wino(m, li, h, w) && m->wino6_wg && L.cin % 128 == 0 && C % 128 == 0) {
    const double T6 = (double)B * ((h + 5) / 6) * ((w + 5) / 6);
    PF_TRY(timed(c, std::string("bwd:wgrad:") + L.name, 2.0 * T6 * 64 * L.cin * C, [&] {
      return pf_wino6_wgrad(dy, C, x, xcs, B, h, w, L.cin, C, grad + L.w_off,
                            L.bias ? grad + L.b_off : nullptr, acc, c.s(m->wino_ws),
                            m->wino_ws.bytes, c.st,
                            vkeep_layer(m, li) ? c.f(m->vk[li]) : nullptr);
    }));
  } else if (use_wino(m, li, h, w) && h % 4 == 0 && w % 4 == 0 && L.cin % 128 == 0 &&
             C % 128 == 0) {
    PF_TRY(timed(c, std::string("bwd:wgrad:") + L.name, wino_flops(B, h, w, L.cin, C, true), [&] {
      return pf_wino_wgrad(dy, C, x, xcs, B, h, w, L.cin, C, grad + L.w_off,
                           L.bias ? grad + L.b_off : nullptr, acc, c.s(m->wino_ws),
                           m->wino_ws.bytes, c.st);
    }));
  } else {
    PF_TRY(timed(c, std::string("bwd:wgrad:") + L.name, flops, [&] {
      return pf_conv_wgrad(dy, C, x, xcs, B, h, w, cinp, C, L.k, L.k, L.stride, grad + L.w_off,
                           L.bias ? grad + L.b_off : nullptr, acc, c.s(m->wgws), m->wgws.bytes,
                           c.st);
    }));
  }
  if (!dx) return POSFEAT_OK;
  // the input-gradient weights: derived here on an accumulate = 0 call, the
  // accumulate = 1 call of the same step (same parameters, same scratch) reuses
  // them (posfeat_bbtrain_backward)
  const bool derive = m->derive_now;
  float* wt = c.s(m->bw) + m->bw_wt[li];
  unsigned short* wtp = reinterpret_cast<unsigned short*>(c.s(m->bw) + m->bw_wtp[li]);
  float* Ud = c.s(m->bw) + m->bw_u[li];
  if (L.stride == 2 && m->s2phase) {
    // output-phase input gradient (bbtrain_kernels.h): 1x1 -> compact GEMM,
    // 3x3 -> one 2x2 pad-1 conv with 4 Cin phase channels; then one scatter
    if ((h & 1) || (w & 1) || L.cin % 32 || C % 32 || (L.k != 1 && L.k != 3))
      return POSFEAT_E_UNSUPPORTED;
    const int oh2 = h / 2, ow2 = w / 2;
    float* dz = c.s(m->dz);
    const bool k3 = L.k == 3;
    // the derived weights and (pre-split tiles) their bf16 planes in one pass
    if (derive) PF_TRY(timed(c, "bwd:misc", 0, [&] {
      if (!k3)
        return pf_dgrad_weights(c.prm + L.w_off, C, L.cin, 1, 1, wt, c.st,
                                m->wsplit ? wtp : nullptr);
      hipLaunchKernelGGL(s2_phase_weights_kernel,
                         dim3(grid_for(16LL * L.cin * C, 256)), dim3(256), 0, c.st,
                         c.prm + L.w_off, C, L.cin, wt, m->wsplit ? wtp : nullptr);
      PF_CHECK_LAUNCH();
      return (int)POSFEAT_OK;
    }));
    posfeat_conv_desc d = make_desc(B, oh2, ow2, C, C, k3 ? 4 * L.cin : L.cin, k3 ? 2 : 1, 1,
                                    k3 ? 4 * L.cin : L.cin, 0);
    d.pad = k3 ? 1 : 0;
    const double pf = k3 ? 2.0 * B * (oh2 + 1) * (ow2 + 1) * 4 * C * 4 * L.cin
                         : 2.0 * B * oh2 * ow2 * C * L.cin;
    const long long wrows = k3 ? 4LL * L.cin : L.cin, wcols = posfeat_conv_packed_k(C, d.kh, d.kw);
    PF_TRY(timed(c, std::string("bwd:dgrad:") + L.name, pf, [&] {
      auto run = [&](int tile) {
        return pf_conv_run_tile(&d, dy, wt, nullptr, nullptr, dz, c.s(m->splitk),
                                m->splitk.bytes, tile, c.st, m->wsplit ? wtp : nullptr,
                                wrows * wcols);
      };
      return m->tune ? pf_conv_tuned_run(&d, false, m->wsplit, c.st, run) : run(-1);
    }));
    return timed(c, "bwd:misc", 0, [&] {
      hipLaunchKernelGGL(s2_scatter_kernel, dim3(grid_for((long long)B * h * w * (L.cin / 4), 256)),
                         dim3(256), 0, c.st, dz, k3 ? 1 : 0, B, h, w, L.cin / 4, add, addcs, dx,
                         dxcs);
      PF_CHECK_LAUNCH();
      return (int)POSFEAT_OK;
    });
  }
  const float* src = dy;
  PF_TRY(timed(c, "bwd:misc", 0, [&] {
    // the direct input gradient's bf16 planes with the derived weights (one pass)
    const bool direct = add || !use_wino(m, li, h, w);
    if (derive)
      PF_TRY(pf_dgrad_weights(c.prm + L.w_off, C, L.cin, L.k, L.k, wt, c.st,
                              m->wsplit && direct ? wtp : nullptr));
    if (L.stride == 2) {
      if ((h & 1) || (w & 1)) return (int)POSFEAT_E_UNSUPPORTED;
      float* dz = c.s(m->dz);
      hipLaunchKernelGGL(zero_insert_kernel, dim3(grid_for((long long)B * h * w * c4n, 256)),
                         dim3(256), 0, c.st, dy, B, h, w, c4n, dz);
      PF_CHECK_LAUNCH();
      src = dz;
    }
    return (int)POSFEAT_OK;
  }));
  if (!add && use_wino(m, li, h, w) && m->wino6) {
    float* U = Ud;
    const double T6 = (double)B * ((h + 5) / 6) * ((w + 5) / 6);
    return timed(c, std::string("bwd:dgrad:") + L.name, 2.0 * T6 * 64 * C * L.cin, [&] {
      if (derive) PF_TRY(pf_wino6_weights(wt, L.cin, C, U, c.st, m->wsplit));
      return pf_wino6_conv(src, C, B, h, w, C, U, nullptr, L.cin, ACT_NONE, dx, dxcs,
                           c.s(m->wino_ws), m->wino_ws.bytes, c.st, 7, m->wsplit ? 1 : 0);
    });
  }
  if (!add && use_wino(m, li, h, w)) {
    float* U = Ud;
    return timed(c, std::string("bwd:dgrad:") + L.name, wino_flops(B, h, w, C, L.cin), [&] {
      if (derive) PF_TRY(pf_wino_weights_hw(wt, L.cin, C, h, w, U, c.st, m->bf6p || m->wsplit));
      return pf_wino_conv(src, C, B, h, w, C, U, nullptr, L.cin, ACT_NONE, dx, dxcs,
                          c.s(m->wino_ws), m->wino_ws.bytes, c.st, 7,
                          m->bf6p ? 2 : m->wsplit ? 1 : 0);
    });
  }
  posfeat_conv_desc d = make_desc(B, h, w, C, C, L.cin, L.k, 1, dxcs, add ? addcs : 0);
  const long long wcols = posfeat_conv_packed_k(C, L.k, L.k);
  return timed(c, std::string("bwd:dgrad:") + L.name, flops, [&] {
    auto run = [&](int tile) {
      return pf_conv_run_tile(&d, src, wt, nullptr, add, dx, c.s(m->splitk), m->splitk.bytes,
                              tile, c.st, m->wsplit ? wtp : nullptr, (long long)L.cin * wcols);
    };
    return m->tune ? pf_conv_tuned_run(&d, add != nullptr, m->wsplit, c.st, run) : run(-1);
  });
}

// ------------------------------------------------------------------ forward / backward
struct BlkIO {
  const float* x;
  int xcs;
  float* out;
  int ocs;
};

std::vector<BlkIO> block_io(Ctx& c) {
  posfeat_bbtrain* m = c.m;
  const auto& bl = blocks();
  std::vector<BlkIO> io(bl.size());
  const float* x = c.f(m->mp);
  int xcs = 64;
  for (size_t i = 0; i < bl.size(); ++i) {
    const bool last = i + 1 == bl.size() || bl[i + 1].li != bl[i].li;
    float* out;
    int ocs;
    if (!last) {
      out = c.f(m->bout[i]);
      ocs = bl[i].pl * 4;
    } else if (bl[i].li == 0) {
      out = c.f(m->cat2) + 256;  // layer1 -> cat2[:, 256:512]  (skipconnect(x1, .))
      ocs = 512;
    } else if (bl[i].li == 1) {
      out = c.f(m->cat3) + 512;  // layer2 -> cat3[:, 512:1024]
      ocs = 1024;
    } else {
      out = c.f(m->l3out);
      ocs = 1024;
    }
    io[i] = {x, xcs, out, ocs};
    x = out;
    xcs = ocs;
  }
  return io;
}

int forward(Ctx& c, const float* img, float* stats, float mom) {
  posfeat_bbtrain* mm = c.m;
  if (mm->wsplit)  // the parameters' bf16 planes for this call's row-tile convs
    PF_TRY(timed(c, "fwd:misc", 0, [&] {
      return pf_split3_rows(c.prm, tab().params / 4, 4, 4, c.su(mm->wpl), c.st);
    }));
  posfeat_bbtrain* m = c.m;
  const TTable& T = tab();
  const int B = m->B, H = m->H, W = m->W;
  const int h2 = H / 2, w2 = W / 2, h4 = H / 4, w4 = W / 4, h8 = H / 8, w8 = W / 8, h16 = H / 16,
            w16 = W / 16;
  std::vector<int> lih, liw;
  layer_inputs(H, W, lih, liw);
  PF_TRY(timed(c, "fwd:misc", 0,
               [&] { return pf_nchw_to_nhwc(img, B, 3, H, W, 4, c.f(m->img4), c.st); }));
  PF_TRY(layer_fwd(c, T.first, c.f(m->img4), 4, H, W, c.f(m->a0), 64, stats, mom));
  PF_TRY(timed(c, "fwd:misc", 0, [&] {
    hipLaunchKernelGGL(maxpool3s2_idx_kernel, dim3(grid_for((long long)B * h4 * w4 * 16, 256)),
                       dim3(256), 0, c.st, c.f(m->a0), 64, B, h2, w2, 16, h4, w4, c.f(m->mp), 64,
                       reinterpret_cast<unsigned*>(c.f(m->mpidx)));
    PF_CHECK_LAUNCH();
    return (int)POSFEAT_OK;
  }));
  const auto& bl = blocks();
  const auto io = block_io(c);
  for (size_t i = 0; i < bl.size(); ++i) {
    const Blk& b = bl[i];
    const int ih = lih[b.c1], iw = liw[b.c1], oh = lih[b.c3], ow = liw[b.c3];
    float* a1 = c.f(m->a1[i]);
    float* a2 = c.f(m->a2[i]);
    PF_TRY(layer_fwd(c, b.c1, io[i].x, io[i].xcs, ih, iw, a1, b.pl, stats, mom));
    PF_TRY(layer_fwd(c, b.c2, a1, b.pl, ih, iw, a2, b.pl, stats, mom));
    const float* res = io[i].x;
    int rcs = io[i].xcs;
    if (b.ds) {
      float* dsn = c.s(m->dsn);
      PF_TRY(layer_fwd(c, b.cds, io[i].x, io[i].xcs, ih, iw, dsn, b.pl * 4, stats, mom));
      res = dsn;
      rcs = b.pl * 4;
    }
    PF_TRY(layer_fwd(c, b.c3, a2, b.pl, oh, ow, io[i].out, io[i].ocs, stats, mom, res, rcs));
  }
  // decoder (DescNet.py:72-82)
  PF_TRY(layer_fwd(c, T.coarse, c.f(m->l3out), 1024, h16, w16, nullptr, 0, stats, mom));
  PF_TRY(timed(c, "fwd:misc", 0, [&] {
    return pf_upsample2x_ac(c.f(m->l3out), B, h16, w16, 1024, 1024, c.f(m->up3), 1024, c.st);
  }));
  PF_TRY(layer_fwd(c, T.up3, c.f(m->up3), 1024, h8, w8, c.f(m->cat3), 1024, stats, mom));
  PF_TRY(layer_fwd(c, T.ic3, c.f(m->cat3), 1024, h8, w8, c.f(m->i3a), 512, stats, mom));
  PF_TRY(timed(c, "fwd:misc", 0, [&] {
    return pf_upsample2x_ac(c.f(m->i3a), B, h8, w8, 512, 512, c.f(m->up2), 512, c.st);
  }));
  PF_TRY(layer_fwd(c, T.up2, c.f(m->up2), 512, h4, w4, c.f(m->cat2), 512, stats, mom));
  PF_TRY(layer_fwd(c, T.ic2, c.f(m->cat2), 512, h4, w4, c.f(m->i2a), 256, stats, mom));
  return layer_fwd(c, T.fine, c.f(m->i2a), 256, h4, w4, c.f(m->fa), 128, stats, mom);
}

int backward(Ctx& c, const float* dfa, int dfcs, float* grad, int acc) {
  posfeat_bbtrain* m = c.m;
  const TTable& T = tab();
  const int B = m->B, H = m->H, W = m->W;
  const int h2 = H / 2, w2 = W / 2, h4 = H / 4, w4 = W / 4, h8 = H / 8, w8 = W / 8, h16 = H / 16,
            w16 = W / 16;
  std::vector<int> lih, liw;
  layer_inputs(H, W, lih, liw);
  float* ga = c.s(m->ga);
  float* gb = c.s(m->gb);
  float* dcat2 = c.s(m->dcat2);
  float* dcat3 = c.s(m->dcat3);
  float* dup = c.s(m->dup);
  // decoder, top down
  PF_TRY(layer_bwd(c, T.fine, c.f(m->i2a), 256, h4, w4, c.f(m->fa), 128, dfa, dfcs, grad, acc,
                   nullptr, ga, 256, nullptr, 0));
  PF_TRY(layer_bwd(c, T.ic2, c.f(m->cat2), 512, h4, w4, c.f(m->i2a), 256, ga, 256, grad, acc,
                   nullptr, dcat2, 512, nullptr, 0));
  PF_TRY(layer_bwd(c, T.up2, c.f(m->up2), 512, h4, w4, c.f(m->cat2), 512, dcat2, 512, grad, acc,
                   nullptr, dup, 512, nullptr, 0));
  PF_TRY(upsample_adjoint(c, dup, 512, h8, w8, 512, ga, 512));
  PF_TRY(layer_bwd(c, T.ic3, c.f(m->cat3), 1024, h8, w8, c.f(m->i3a), 512, ga, 512, grad, acc,
                   nullptr, dcat3, 1024, nullptr, 0));
  PF_TRY(layer_bwd(c, T.up3, c.f(m->up3), 1024, h8, w8, c.f(m->cat3), 1024, dcat3, 1024, grad, acc,
                   nullptr, dup, 1024, nullptr, 0));
  PF_TRY(upsample_adjoint(c, dup, 1024, h16, w16, 1024, ga, 1024));
  // encoder blocks in reverse; `cur` holds d(block output)
  const auto& bl = blocks();
  const auto io = block_io(c);
  float* cur = ga;
  int ccs = 1024;
  for (int i = (int)bl.size() - 1; i >= 0; --i) {
    const Blk& b = bl[i];
    const int ih = lih[b.c1], iw = liw[b.c1], oh = lih[b.c3], ow = liw[b.c3];
    float* dst = cur == ga ? gb : ga;
    const int dcs = b.inpl;
    // the block input's other consumer: the decoder skip (layer2 -> cat3, layer1 -> cat2)
    const float* extra = nullptr;
    int ecs = 0;
    if (b.bi == 0 && b.li == 2) {
      extra = dcat3 + 512;
      ecs = 1024;
    } else if (b.bi == 0 && b.li == 1) {
      extra = dcat2 + 256;
      ecs = 512;
    }
    float* gres = c.s(m->gres);
    float* d2 = c.s(m->gd);  // d a2
    float* d1 = c.s(m->gc);  // d a1
    PF_TRY(layer_bwd(c, b.c3, c.f(m->a2[i]), b.pl, oh, ow, io[i].out, io[i].ocs, cur, ccs, grad,
                     acc, gres, d2, b.pl, nullptr, 0, true));
    PF_TRY(layer_bwd(c, b.c2, c.f(m->a1[i]), b.pl, ih, iw, c.f(m->a2[i]), b.pl, d2, b.pl, grad,
                     acc, nullptr, d1, b.pl, nullptr, 0));
    const float* radd;
    int rcs;
    if (b.ds) {
      float* dsg = d2;  // free again
      PF_TRY(layer_bwd(c, b.cds, io[i].x, io[i].xcs, ih, iw, nullptr, 0, gres, b.pl * 4, grad, acc,
                       nullptr, dsg, b.inpl, extra, ecs));
      radd = dsg;
      rcs = b.inpl;
    } else {
      radd = gres;  // identity shortcut
      rcs = b.pl * 4;
    }
    PF_TRY(layer_bwd(c, b.c1, io[i].x, io[i].xcs, ih, iw, c.f(m->a1[i]), b.pl, d1, b.pl, grad, acc,
                     nullptr, dst, dcs, radd, rcs));
    cur = dst;
    ccs = dcs;
  }
  // stem: cur = d(maxpool output)
  float* da0 = cur == ga ? gb : ga;
  PF_TRY(timed(c, "bwd:misc", 0, [&] {
    hipLaunchKernelGGL(maxpool_adjoint_idx_kernel,
                       dim3(grid_for((long long)B * h2 * w2 * 16, 256)), dim3(256), 0, c.st,
                       reinterpret_cast<const unsigned*>(c.f(m->mpidx)), B, h2, w2, 16, cur, ccs,
                       h4, w4, da0, 64);
    PF_CHECK_LAUNCH();
    return POSFEAT_OK;
  }));
  return layer_bwd(c, T.first, c.f(m->img4), 4, H, W, c.f(m->a0), 64, da0, 64, grad, acc, nullptr,
                   nullptr, 0, nullptr, 0);
}

}  // namespace

// ------------------------------------------------------------------ C ABI
extern "C" int posfeat_bbtrain_num_layers(void) { return (int)tab().v.size(); }

extern "C" int posfeat_bbtrain_layer(int i, const char** name, int* cin, int* cout, int* k,
                                     int* stride, int* has_bias, long long* offs) {
  if (i < 0 || i >= (int)tab().v.size()) return POSFEAT_E_INVALID;
  const TLayer& L = tab().v[i];
  if (name) *name = L.name.c_str();
  if (cin) *cin = L.cin;
  if (cout) *cout = L.cout;
  if (k) *k = L.k;
  if (stride) *stride = L.stride;
  if (has_bias) *has_bias = L.bias ? 1 : 0;
  if (offs) {
    offs[0] = L.w_off;
    offs[1] = L.b_off;
    offs[2] = L.g_off;
    offs[3] = L.be_off;
    offs[4] = L.rm_off;
    offs[5] = L.rv_off;
  }
  return POSFEAT_OK;
}

extern "C" long long posfeat_bbtrain_param_floats(void) { return tab().params; }
extern "C" long long posfeat_bbtrain_stat_floats(void) { return tab().stats; }

extern "C" int posfeat_bbtrain_create(int batch, int h, int w, posfeat_bbtrain** out) {
  if (!out || batch <= 0 || h <= 0 || w <= 0) return POSFEAT_E_INVALID;
  // multiples of 16: the skipconnect pads are zero (DescNet.py:50-62) and
  // every stride-2 input is even
  if (h % 16 || w % 16) return POSFEAT_E_UNSUPPORTED;
  posfeat_bbtrain* m = new posfeat_bbtrain();
  m->B = batch;
  m->H = h;
  m->W = w;
  plan(m);
  *out = m;
  return POSFEAT_OK;
}

extern "C" size_t posfeat_bbtrain_act_bytes(const posfeat_bbtrain* m) { return m ? m->act_bytes : 0; }
extern "C" size_t posfeat_bbtrain_scratch_bytes(const posfeat_bbtrain* m) {
  return m ? m->scr_bytes : 0;
}

// POSFEAT_TRAIN_HALO_BF6=1 (A/B build): the 3x3 stride-1 convs on their
// bf16x6 halo tiles instead of fp32 MFMA (speed / fixture-error probe)
static bool train_halo_fp32() {
  static const bool fp32 = [] {
    const char* e = pf_ab_getenv("POSFEAT_TRAIN_HALO_BF6");
    return !(e && e[0] == '1');
  }();
  return fp32;
}

extern "C" int posfeat_bbtrain_forward(posfeat_bbtrain* m, const float* params, float* stats,
                                       float momentum, const float* img_nchw, void* act,
                                       void* scratch, float** local_map_nhwc, void* stream) {
  if (!m || !params || !img_nchw || !act || !scratch) return POSFEAT_E_INVALID;
  if ((reinterpret_cast<uintptr_t>(act) & 255) || (reinterpret_cast<uintptr_t>(scratch) & 255) ||
      (reinterpret_cast<uintptr_t>(params) & 15) || (reinterpret_cast<uintptr_t>(stats) & 15))
    return POSFEAT_E_INVALID;
  Ctx c{m, static_cast<char*>(act), static_cast<char*>(scratch), pf_stream(stream), params};
  // fp32 halo tiles: the fixture-validated numerics
  const PfHaloFp32Scope halo32(train_halo_fp32());
  m->bw_valid = false;  // a new step: the next backward derives its weights again
  PF_TRY(forward(c, img_nchw, stats, momentum));
  if (local_map_nhwc) *local_map_nhwc = c.f(m->fa);
  return POSFEAT_OK;
}

extern "C" int posfeat_bbtrain_backward(posfeat_bbtrain* m, const float* params, const void* act,
                                        const float* dlocal_map_nhwc, int dcs, float* grad,
                                        int accumulate, void* scratch, void* stream) {
  if (!m || !params || !act || !dlocal_map_nhwc || !grad || !scratch || dcs < 128 || dcs % 4)
    return POSFEAT_E_INVALID;
  if ((reinterpret_cast<uintptr_t>(act) & 255) || (reinterpret_cast<uintptr_t>(scratch) & 255) ||
      (reinterpret_cast<uintptr_t>(dlocal_map_nhwc) & 15) || (reinterpret_cast<uintptr_t>(grad) & 15))
    return POSFEAT_E_INVALID;
  Ctx c{m, static_cast<char*>(const_cast<void*>(act)), static_cast<char*>(scratch),
        pf_stream(stream), params};
  const PfHaloFp32Scope halo32(train_halo_fp32());
  // reuse the input-gradient weights only when an accumulate = 0 call of this
  // step derived them from the same parameters into the same scratch
  m->derive_now = !accumulate || !m->bw_valid || m->bw_params != params || m->bw_scratch != scratch;
  m->bw_valid = false;
  const int rc = backward(c, dlocal_map_nhwc, dcs, grad, accumulate ? 1 : 0);
  if (rc == POSFEAT_OK) {
    m->bw_valid = true;
    m->bw_params = params;
    m->bw_scratch = scratch;
  }
  return rc;
}

extern "C" int posfeat_bbtrain_set_timing(posfeat_bbtrain* m, int enable) {
  if (!m) return POSFEAT_E_INVALID;
  m->timing = enable != 0;
  m->ev_used = 0;
  return POSFEAT_OK;
}

extern "C" int posfeat_bbtrain_timing(posfeat_bbtrain* m, const char* prefix, double* ms,
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

// the i-th timed launch of the last timed step: label ("fwd:conv:<layer>",
// "bwd:wgrad:<layer>", ...), ms, flops; POSFEAT_E_INVALID past the last
extern "C" int posfeat_bbtrain_timing_event(posfeat_bbtrain* m, int i, const char** label,
                                            double* ms, double* flops) {
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

extern "C" int posfeat_bbtrain_set_group(posfeat_bbtrain* m, posfeat_group* g) {
  if (!m) return POSFEAT_E_INVALID;
  m->group = g;
  return POSFEAT_OK;
}

extern "C" void posfeat_bbtrain_destroy(posfeat_bbtrain* m) {
  if (!m) return;
  for (auto& e : m->evs) {
    (void)hipEventDestroy(e.a);
    (void)hipEventDestroy(e.b);
  }
  delete m;
}

extern "C" int posfeat_adam(float* p, const float* g, float* m, float* v, long long n, float lr,
                            float beta1, float beta2, float eps, float weight_decay, long long step,
                            float grad_scale, void* stream) {
  if (!p || !g || !m || !v || n < 0 || step < 1) return POSFEAT_E_INVALID;
  if (n == 0) return POSFEAT_OK;
  const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
  const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
  const float neg_step = (float)(-(double)lr / bc1);
  const float bc2s = (float)std::sqrt(bc2);
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n, 256)), dim3(256), 0, pf_stream(stream), p, g, m,
                     v, n, neg_step, beta1, beta2, eps, bc2s, grad_scale, weight_decay);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// the PF_ARITH_* mask of the i-th timed label's MFMA launches (1: fp32 MFMA,
// 2: bf16x6, 3: both, 0: none), for bench.py's rooflines
extern "C" int posfeat_bbtrain_timing_event_arith(posfeat_bbtrain* m, int i) {
  if (!m || i < 0 || (size_t)i >= m->ev_used) return POSFEAT_E_INVALID;
  return m->evs[i].arith;
}
