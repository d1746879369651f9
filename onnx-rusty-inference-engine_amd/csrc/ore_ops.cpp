// C ABI: context, memory, reference geometry and the per-op entry points that replace the
// functions behind `node_inference` (model_inference.rs:137-161).
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <cstdlib>

#include "ore_internal.h"

namespace {
thread_local std::string g_global_err;
}

namespace ore {

ore_status set_error(ore_ctx* ctx, ore_status st, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (ctx) ctx->err = buf;
  g_global_err = buf;
  return st;
}

// get_padding_size (convolution_op.rs:519-557 == max_pool_op.rs:363-401).  The reference
// returns (pad_h, pad_w, pad_bottom, pad_top, pad_right, pad_left) into variables named
// (pad_num_h, pad_num_w, pad_top, pad_bottom, pad_left, pad_right): the larger half lands on
// the top/left, for SAME_UPPER and SAME_LOWER alike.
static ore_status same_padding(ore_ctx* ctx, int64_t H, int64_t W, int64_t sh, int64_t sw, int64_t kh, int64_t kw,
                               Window* w) {
  const int64_t ph = (H % sh == 0) ? kh - sh : kh - (H % sh);
  const int64_t pw = (W % sw == 0) ? kw - sw : kw - (W % sw);
  if (ph < 0 || pw < 0)  // usize underflow in the reference
    return set_error(ctx, ORE_ERR_UNSUPPORTED, "SAME padding with kernel smaller than stride/remainder");
  w->pb = ph / 2;
  w->pt = ph - w->pb;
  w->pr = pw / 2;
  w->pl = pw - w->pr;
  return ORE_OK;
}

ore_status resolve_window(ore_ctx* ctx, int auto_pad, const int64_t* pads, int n_pads, int64_t H, int64_t W,
                          int64_t kh, int64_t kw, int64_t sh, int64_t sw, Window* out) {
  *out = Window{};
  if (sh <= 0 || sw <= 0 || kh <= 0 || kw <= 0)
    return set_error(ctx, ORE_ERR_INVALID, "non-positive kernel/stride");
  switch (auto_pad) {
    case ORE_PAD_SAME_UPPER:
    case ORE_PAD_SAME_LOWER:
      // H' = ceil(H / stride), computed in f32 as the reference does (:297-310)
      out->Ho = int64_t(std::ceil(float(H) / float(sh)));
      out->Wo = int64_t(std::ceil(float(W) / float(sw)));
      return same_padding(ctx, H, W, sh, sw, kh, kw, out);
    case ORE_PAD_NOTSET: {
      if (n_pads < 4) return set_error(ctx, ORE_ERR_INVALID, "auto_pad NOTSET needs 4 pads");
      out->pt = pads[0]; out->pl = pads[1]; out->pb = pads[2]; out->pr = pads[3];
      if (out->pt < 0 || out->pl < 0 || out->pb < 0 || out->pr < 0)
        return set_error(ctx, ORE_ERR_INVALID, "negative pads");
      if (H + out->pt + out->pb < kh || W + out->pl + out->pr < kw)
        return set_error(ctx, ORE_ERR_INVALID, "window larger than padded input");
      out->Ho = (H - kh + out->pt + out->pb) / sh + 1;  // floor (:312-317)
      out->Wo = (W - kw + out->pl + out->pr) / sw + 1;
      return ORE_OK;
    }
    case ORE_PAD_VALID:
      if (H < kh || W < kw) return set_error(ctx, ORE_ERR_INVALID, "window larger than input");
      out->Ho = (H - kh) / sh + 1;
      out->Wo = (W - kw) / sw + 1;
      return ORE_OK;
    default:
      return set_error(ctx, ORE_ERR_UNSUPPORTED, "unknown auto_pad %d", auto_pad);
  }
}

static int64_t nstride_of(const ore_tensor* t) {
  if (t->nstride) return t->nstride;
  int64_t s = 1;
  for (int i = 1; i < t->ndim; ++i) s *= t->dims[i];
  return s;
}

static int64_t numel(const ore_tensor* t) {
  int64_t s = 1;
  for (int i = 0; i < t->ndim; ++i) s *= t->dims[i];
  return s;
}

static bool contiguous(const ore_tensor* t) {
  if (!t->nstride) return true;
  int64_t s = 1;
  for (int i = 1; i < t->ndim; ++i) s *= t->dims[i];
  return t->nstride == s;
}

static bool fits_i32(int64_t v) { return v >= 0 && v < (int64_t(1) << 31); }

// The kernels address activations through buffer resources (32-bit byte offsets, plus up to a few KB
// read before x by the 3x3 tap loads): a batch whose input or output extent does not fit is launched
// in image chunks that do.  Returns the images per chunk (0: one image alone is too large).
constexpr int64_t CHUNK_LIMIT = (int64_t(1) << 31) - (int64_t(1) << 21);
static int64_t image_chunk(int64_t N, int64_t x_nstride, int64_t x_img_bytes, int x_es, int64_t y_nstride,
                           int64_t y_img_bytes, int y_es) {
  auto fits = [&](int64_t nb) {
    return (nb - 1) * x_nstride * x_es + x_img_bytes < CHUNK_LIMIT && (nb - 1) * y_nstride * y_es + y_img_bytes < CHUNK_LIMIT;
  };
  if (!fits(1)) return 0;
  int64_t nb = N;
  while (nb > 1 && !fits(nb)) nb = (nb + 1) / 2;
  return nb;
}

ConvPlan conv_plan(int64_t M, int64_t C, int64_t H, int64_t W, int64_t kh, int64_t kw, int64_t sh, int64_t sw,
                   const Window& win, bool f16, int xmode, bool wino, int forced) {
  return plan_conv(int(M), int(C), int(H), int(W), int(kh), int(kw), int(sh), int(sw), int(win.pt), int(win.pl),
                   int(win.Ho), int(win.Wo), kh == 1 && kw == 1, f16, xmode, wino, forced);
}

size_t packed_bytes(const ConvPlan& pln) { return conv_packed_bytes(pln) + size_t(pln.krows) * sizeof(int2); }

float* pack_to_scratch(ore_ctx* ctx, const ConvPlan& pln, const float* w, bool kmajor_src, int64_t M, int64_t C,
                       int64_t kh, int64_t kw, int64_t H, int64_t W, const int2** ktab) {
  const size_t need = packed_bytes(pln);
  if (need > ctx->scratch_bytes) {
    if (ctx->scratch) {
      (void)hipStreamSynchronize(ctx->stream);
      (void)hipFree(ctx->scratch);
    }
    ctx->scratch = nullptr;
    ctx->scratch_bytes = 0;
    if (hipMalloc(reinterpret_cast<void**>(&ctx->scratch), need) != hipSuccess) {
      set_error(ctx, ORE_ERR_OOM, "weight scratch allocation (%zu bytes) failed", need);
      return nullptr;
    }
    ctx->scratch_bytes = need;
  }
  launch_pack(w, kmajor_src, int(M), int(C), int(kh), int(kw), pln, ctx->scratch, ctx->stream);
  int2* kt = reinterpret_cast<int2*>(reinterpret_cast<char*>(ctx->scratch) + conv_packed_bytes(pln));
  launch_ktab(kt, int(C * kh * kw), int(kh), int(kw), int(H * W), int(W), ctx->stream);
  if (hipGetLastError() != hipSuccess) {
    set_error(ctx, ORE_ERR_HIP, "weight packing launch failed");
    return nullptr;
  }
  *ktab = kt;
  return ctx->scratch;
}

ore_status run_conv(ore_ctx* ctx, const ConvPlan& pln, const float* x, int64_t N, int64_t C, int64_t H, int64_t W,
                    int64_t x_nstride, const float* wp, const int2* ktab, int64_t M, int64_t kh, int64_t kw,
                    const float* bias, const Window& win, int64_t sh, int64_t sw, bool relu, float* y,
                    int64_t y_nstride, int64_t x_ps, int64_t y_ps, int x_es) {
  if (N == 0) return ORE_OK;
  if (pln.f16 || x_es != 4) return set_error(ctx, ORE_ERR_INVALID, "internal: run_conv takes f32 plans and inputs");
  if (x_ps == 0) x_ps = H * W;
  if (y_ps == 0) y_ps = win.Ho * win.Wo;
  ConvParams p{};
  p.x = x; p.wp = wp; p.ktab = ktab; p.bias = bias; p.y = y;
  p.N = int(N); p.C = int(C); p.H = int(H); p.W = int(W);
  p.M = int(M); p.kh = int(kh); p.kw = int(kw); p.sh = int(sh); p.sw = int(sw);
  p.pt = int(win.pt); p.pl = int(win.pl);
  p.Ho = int(win.Ho); p.Wo = int(win.Wo);
  p.K = int(C * kh * kw);
  p.P = int(win.Ho * win.Wo);
  p.x_ps = int(x_ps);
  p.y_ps = int(y_ps);
  p.Ntot = N * y_ps;
  p.x_nstride = x_nstride;
  p.y_nstride = y_nstride;
  p.relu = relu ? 1 : 0;
  p.Mp = pln.Mp;
  p.x_f32 = 1;
  // 16-B epilogue stores of 4 floats
  p.vec_out = (y_ps % 4 == 0 && y_nstride % 4 == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0) ? 1 : 0;
  p.is1x1 = (kh == 1 && kw == 1 && sh == 1 && sw == 1 && win.pt == 0 && win.pl == 0 && win.Ho == H && win.Wo == W &&
             x_ps == y_ps);
  {  // mapped bytes before x: the rest of x's 4 KiB page, or the walker's arena lead
    const char* xc = reinterpret_cast<const char*>(x);
    int64_t g = int64_t(reinterpret_cast<uintptr_t>(x) & 4095);
    if (ctx->mapped_lo && xc >= ctx->mapped_lo && xc < ctx->mapped_hi) g = std::max<int64_t>(g, std::min<int64_t>(xc - ctx->mapped_lo, 1 << 20));
    p.x_guard = int(g);
  }
  if (x_ps < H * W || y_ps < win.Ho * win.Wo) return set_error(ctx, ORE_ERR_INVALID, "plane stride below plane size");
  if (!fits_i32(x_nstride * N + 256) || !fits_i32(y_nstride * N + 256) || !fits_i32(int64_t(pln.krows) * pln.Mp) ||
      !fits_i32(p.Ntot + 256) || (p.Ntot + 127) / 128 * ((M + 31) / 32) >= (int64_t(1) << 31))
    return set_error(ctx, ORE_ERR_INVALID, "conv geometry exceeds 32-bit indexing");
  if (!pln.wino && !p.is1x1 && !ktab) return set_error(ctx, ORE_ERR_INVALID, "internal: gather table missing");
  // image chunks whose x and y extents fit 32-bit byte offsets (the output may be a slice of a wider
  // concat buffer, e.g. an expand3x3 writing channels 256..511 of 512)
  const int64_t nb = image_chunk(N, x_nstride, C * x_ps * 4, 4, y_nstride, M * y_ps * 4, 4);
  if (nb == 0) return set_error(ctx, ORE_ERR_UNSUPPORTED, "conv: one image exceeds 2 GiB");
  for (int64_t i0 = 0; i0 < N; i0 += nb) {
    const int64_t nc = std::min(nb, N - i0);
    ConvParams q = p;
    q.x = x + i0 * x_nstride;
    q.y = y + i0 * y_nstride;
    q.N = int(nc);
    q.Ntot = nc * y_ps;
    q.x_bytes = ((nc - 1) * x_nstride + C * x_ps) * 4;
    ConvPlan qp = pln;
    if (pln.wino && !conv_wino_eligible(q, qp.cfg - WINO_TILE_BASE)) {  // the first tile that takes it
      int t = 0;
      while (t < WINO_TILES_N && !conv_wino_eligible(q, t)) ++t;
      if (t == WINO_TILES_N) return set_error(ctx, ORE_ERR_UNSUPPORTED, "Winograd conv: no tile takes this layout");
      qp.cfg = WINO_TILE_BASE + t;
    }
    launch_conv(q, qp, ctx->stream);
    ORE_HIP_CHECK(ctx, hipGetLastError());
  }
  return ORE_OK;
}

ore_status run_fire(ore_ctx* ctx, const float* x, int64_t N, int64_t C, int64_t H, int64_t W, int64_t x_nstride,
                    int64_t x_ps, const float* w1, const float* b1, int64_t E1, const float* w3, const float* b3,
                    int64_t E3, const float* ws, int64_t Msp, const float* bs, int64_t Ms, float* y, int64_t y_nstride,
                    int64_t y_ps, const Window* pool) {
  if (N == 0) return ORE_OK;
  FireParams p{};
  p.x = x; p.w1 = w1; p.b1 = b1; p.w3 = w3; p.b3 = b3; p.ws = ws; p.bs = bs; p.y = y;
  p.N = int(N); p.C = int(C); p.H = int(H); p.W = int(W);
  p.E1 = int(E1); p.E3 = int(E3); p.Ms = int(Ms); p.Msp = int(Msp);
  p.x_ps = int(x_ps); p.y_ps = int(y_ps);
  p.x_nstride = x_nstride; p.y_nstride = y_nstride;
  p.Ntot = N * y_ps;
  if (pool) {
    p.pool = 1;
    p.Hp = int(pool->Ho); p.Wp = int(pool->Wo); p.ppt = int(pool->pt); p.ppl = int(pool->pl);
    if (!fire_pool_plan(&p)) return set_error(ctx, ORE_ERR_INVALID, "internal: no band shape for the pooled fire module");
  }
  {  // mapped bytes before x (as run_conv): the rest of x's page or the walker's arena lead
    const char* xc = reinterpret_cast<const char*>(x);
    int64_t g = int64_t(reinterpret_cast<uintptr_t>(x) & 4095);
    if (ctx->mapped_lo && xc >= ctx->mapped_lo && xc < ctx->mapped_hi)
      g = std::max<int64_t>(g, std::min<int64_t>(xc - ctx->mapped_lo, 1 << 20));
    p.x_guard = int(g);
  }
  p.x_lead = int(((W + 1) * 4 + 15) & ~int64_t(15));
  if (x_ps < H * W || y_ps < (pool ? pool->Ho * pool->Wo : H * W) || !fits_i32(x_nstride * N + 256) || !fits_i32(y_nstride * N + 256) ||
      !fits_i32(p.Ntot + 256))
    return set_error(ctx, ORE_ERR_INVALID, "fire geometry exceeds 32-bit indexing");
  // the kernels address x through a buffer resource (32-bit byte offsets, plus the x_lead bytes before
  // it): a batch whose input extent does not fit runs in image chunks that do
  const int64_t nb = image_chunk(N, x_nstride, C * x_ps * 4, 4, y_nstride, Ms * y_ps * 4, 4);
  if (nb == 0) return set_error(ctx, ORE_ERR_UNSUPPORTED, "fused fire module: one image exceeds 2 GiB");
  for (int64_t i0 = 0; i0 < N; i0 += nb) {
    const int64_t nc = std::min(nb, N - i0);
    FireParams q = p;
    q.x = x + i0 * x_nstride;
    q.y = y + i0 * y_nstride;
    q.N = int(nc);
    q.Ntot = nc * y_ps;
    q.x_bytes = ((nc - 1) * x_nstride + C * x_ps) * 4;
    if (!fire_eligible(q)) return set_error(ctx, ORE_ERR_INVALID, "internal: fused fire module on an unsupported layout");
    launch_fire(q, ctx->stream);
    ORE_HIP_CHECK(ctx, hipGetLastError());
  }
  return ORE_OK;
}

ore_status run_fire_f16(ore_ctx* ctx, const void* x, int64_t N, int64_t C, int64_t H, int64_t W, int64_t x_nstride,
                        int64_t x_cs, const void* w1, const float* b1, int64_t E1, const void* w3, const float* b3,
                        int64_t E3, const void* ws, const float* bs, int64_t Ms, void* y, int64_t y_nstride,
                        int64_t y_cs, const Window* pool) {
  if (N == 0) return ORE_OK;
  if (!fits_i32(N) || !fits_i32(H * W) || !fits_i32(x_cs) || !fits_i32(y_cs))
    return set_error(ctx, ORE_ERR_INVALID, "fire geometry exceeds 32-bit indexing");
  FireF16Params p{};
  p.x = x; p.w1 = w1; p.b1 = b1; p.w3 = w3; p.b3 = b3; p.ws = ws; p.bs = bs; p.y = y;
  p.N = int(N); p.C = int(C); p.H = int(H); p.W = int(W);
  p.E1 = int(E1); p.E3 = int(E3); p.Ms = int(Ms); p.Msp = int((Ms + 31) / 32 * 32);
  p.x_cs = int(x_cs); p.y_cs = int(y_cs);
  p.x_nstride = x_nstride; p.y_nstride = y_nstride;
  if (pool) {
    p.pool = 1;
    p.Hp = int(pool->Ho); p.Wp = int(pool->Wo); p.ppt = int(pool->pt); p.ppl = int(pool->pl);
    if (!fire_pool_f16_plan(&p)) return set_error(ctx, ORE_ERR_INVALID, "internal: no band shape for the pooled f16 fire module");
  }
  if (!fire_f16_eligible(p)) return set_error(ctx, ORE_ERR_INVALID, "internal: f16 fire module on an unsupported layout");
  launch_fire_f16(p, ctx->stream);
  ORE_HIP_CHECK(ctx, hipGetLastError());
  return ORE_OK;
}

double epool_tile(int64_t Ho, int64_t Wo, int64_t pkh, int64_t pkw, int64_t psh, int64_t psw, const Window& pwin,
                  int* tr, int* tc) {
  // the kernel's pooled epilogue is specialised for 3x3 / stride-2 windows (every SqueezeNet pool)
  if (pkh != 3 || pkw != 3 || psh != 2 || psw != 2 || Ho * Wo == 0 || pwin.Ho <= 0 || pwin.Wo <= 0) return 0.0;
  *tr = int((pwin.Ho + EPOOL_TILE_PR - 1) / EPOOL_TILE_PR);
  *tc = int((pwin.Wo + EPOOL_TILE_PC - 1) / EPOOL_TILE_PC);
  return double(int64_t(*tr) * *tc * CONV_EPOOL_BN) / double(Ho * Wo);
}

ore_status run_conv_epool(ore_ctx* ctx, const ConvPlan& pln, const float* x, int64_t N, int64_t C, int64_t H, int64_t W,
                          int64_t x_nstride, int64_t x_ps, const float* wp, const int2* ktab, int64_t M, int64_t kh,
                          int64_t kw, const float* bias, const Window& win, int64_t sh, int64_t sw, bool relu,
                          int64_t pkh, int64_t pkw, int64_t psh, int64_t psw, const Window& pwin, float* y,
                          int64_t y_nstride, int64_t y_ps, const float* wc1, const C1SqueezeF32* sq1) {
  if (N == 0) return ORE_OK;
  if (pln.f16) return set_error(ctx, ORE_ERR_INVALID, "internal: the pooled epilogue is f32 gather only");
  if (x_ps == 0) x_ps = H * W;
  if (y_ps == 0) y_ps = pwin.Ho * pwin.Wo;
  int tr = 0, tc = 0;
  if (epool_tile(win.Ho, win.Wo, pkh, pkw, psh, psw, pwin, &tr, &tc) == 0.0)
    return set_error(ctx, ORE_ERR_INVALID, "internal: the pooled epilogue takes 3x3 / stride-2 pools");
  ConvParams p{};
  p.x = x; p.wp = wp; p.ktab = ktab; p.bias = bias; p.y = y;
  p.N = int(N); p.C = int(C); p.H = int(H); p.W = int(W);
  p.M = int(M); p.kh = int(kh); p.kw = int(kw); p.sh = int(sh); p.sw = int(sw);
  p.pt = int(win.pt); p.pl = int(win.pl);
  p.Ho = int(win.Ho); p.Wo = int(win.Wo);
  p.K = int(C * kh * kw);
  p.P = int(win.Ho * win.Wo);
  p.x_ps = int(x_ps);
  p.y_ps = int(y_ps);
  p.x_nstride = x_nstride;
  p.y_nstride = y_nstride;
  p.relu = relu ? 1 : 0;
  p.Mp = pln.Mp;
  p.x_f32 = 1;
  p.is1x1 = (kh == 1 && kw == 1 && sh == 1 && sw == 1 && win.pt == 0 && win.pl == 0 && win.Ho == H && win.Wo == W &&
             x_ps == H * W);
  p.ep_pt = int(pwin.pt); p.ep_pl = int(pwin.pl); p.ep_Ho = int(pwin.Ho); p.ep_Wo = int(pwin.Wo);
  p.ep_tr = tr; p.ep_tc = tc;
  p.ep_variant = pln.epv;
  p.wc1 = wc1;
  p.sq1 = sq1;
  {  // mapped bytes before x (as run_conv): the row-walking 3x3 kernel reads a few of them, masked
    const char* xc = reinterpret_cast<const char*>(x);
    int64_t g = int64_t(reinterpret_cast<uintptr_t>(x) & 4095);
    if (ctx->mapped_lo && xc >= ctx->mapped_lo && xc < ctx->mapped_hi)
      g = std::max<int64_t>(g, std::min<int64_t>(xc - ctx->mapped_lo, 1 << 20));
    p.x_guard = int(g);
  }
  p.Ntot = N * int64_t(p.ep_tr) * p.ep_tc * CONV_EPOOL_BN;
  if (x_ps < H * W || y_ps < pwin.Ho * pwin.Wo) return set_error(ctx, ORE_ERR_INVALID, "plane stride below plane size");
  if (!fits_i32(x_nstride * N + 256) || !fits_i32(y_nstride * N + 256) || !fits_i32(int64_t(pln.krows) * pln.Mp) ||
      !fits_i32(p.Ntot + 256) || N * p.ep_tr * p.ep_tc * ((M + 31) / 32) >= (int64_t(1) << 31))
    return set_error(ctx, ORE_ERR_INVALID, "conv geometry exceeds 32-bit indexing");
  if (!p.is1x1 && !ktab) return set_error(ctx, ORE_ERR_INVALID, "internal: gather table missing");
  const int64_t y_img = sq1 ? (sq1->M * int64_t(sq1->y_ps)) * 4 : M * y_ps * 4;
  const int64_t nb = image_chunk(N, x_nstride, C * x_ps * 4, 4, sq1 ? sq1->y_nstride : y_nstride, y_img, 4);
  if (nb == 0) return set_error(ctx, ORE_ERR_UNSUPPORTED, "pooled conv: one image exceeds 2 GiB");
  for (int64_t i0 = 0; i0 < N; i0 += nb) {
    const int64_t nc = std::min(nb, N - i0);
    ConvParams q = p;
    C1SqueezeF32 sq{};
    q.x = x + i0 * x_nstride;
    if (y) q.y = y + i0 * y_nstride;
    if (sq1) {
      sq = *sq1;
      sq.y = sq1->y + i0 * sq1->y_nstride;
      q.sq1 = &sq;
    }
    q.N = int(nc);
    q.Ntot = nc * int64_t(p.ep_tr) * p.ep_tc * CONV_EPOOL_BN;
    q.x_bytes = ((nc - 1) * x_nstride + C * x_ps) * 4;
    launch_conv_epool(q, ctx->stream);
    ORE_HIP_CHECK(ctx, hipGetLastError());
    if (sq1 && last_conv_tile != EPOOL_WIN_TILE && last_conv_tile != EPOOL_BAND_TILE)
      return set_error(ctx, ORE_ERR_INVALID, "internal: the fused first conv + squeeze declined its launch");
  }
  return ORE_OK;
}

ore_status run_conv_pool(ore_ctx* ctx, const ConvPlan& pln, const float* x, int64_t N, int64_t C, int64_t pH,
                         int64_t pW, int64_t x_nstride, int64_t x_ps, const Window& pwin, int64_t psh, int64_t psw,
                         const float* wp, int64_t M, const float* bias, bool relu, float* y, int64_t y_nstride,
                         int64_t y_ps, int x_es, const PoolExpand* pe) {
  if (N == 0) return ORE_OK;
  if (x_ps == 0) x_ps = pH * pW;
  const int64_t P = pwin.Ho * pwin.Wo;
  if (y_ps == 0) y_ps = P;
  if (pln.f16 || pln.wino || x_es != 4)
    return set_error(ctx, ORE_ERR_INVALID, "internal: the pooled 1x1 conv is f32 direct only");
  // 3x3 / stride-2 pools (the window is implied by the walker's pass, kernel_shape 3x3):
  // pool_conv1x1_f32_kernel (LDS-staged rows, MFMA squeeze)
  PoolConvParams q{};
  q.x = x; q.wp = wp; q.bias = bias; q.y = y;
  q.N = int(N); q.C = int(C); q.H = int(pH); q.W = int(pW); q.Hp = int(pwin.Ho); q.Wp = int(pwin.Wo);
  q.pt = int(pwin.pt); q.pl = int(pwin.pl); q.M = int(M); q.Mp = pln.Mp; q.Kp = pln.krows;
  q.x_ps = int(x_ps); q.y_ps = int(y_ps); q.x_nstride = x_nstride; q.y_nstride = y_nstride;
  q.relu = relu ? 1 : 0;
  if (pe) {
    q.s = pe->s; q.w1 = pe->w1; q.b1 = pe->b1; q.C1 = pe->C1; q.E1 = pe->E1; q.w1_Mp = pe->w1_Mp;
    q.s_ps = int(pe->s_ps); q.s_nstride = pe->s_nstride;
    if (!fits_i32(pe->s_nstride * N + 256) || !fits_i32(pe->s_ps))
      return set_error(ctx, ORE_ERR_INVALID, "internal: recomputed expand input past 2 GiB");
  }
  if (psh != 2 || psw != 2 || pwin.Ho <= 0 || !fits_i32(x_nstride * N + 256) || !fits_i32(y_nstride * N + 256) ||
      !pool_conv1x1_f32_eligible(q))
    return set_error(ctx, ORE_ERR_INVALID, "internal: pooled 1x1 conv outside pool_conv1x1_f32_kernel's limits");
  launch_pool_conv1x1_f32(q, ctx->stream);
  ORE_HIP_CHECK(ctx, hipGetLastError());
  return ORE_OK;
}

ore_status run_conv_pair_pool_f16(ore_ctx* ctx, const ConvPlan& pln, const float* x, int64_t N, int64_t C, int64_t H,
                                  int64_t W, int64_t x_nstride, int64_t x_ps, const void* wp, int64_t M, int64_t kh,
                                  int64_t kw, const float* bias, const Window& win, int64_t sh, int64_t sw, bool relu,
                                  void* y, int64_t y_nstride, int64_t y_ps, const F16Epool& ep, bool* ran,
                                  const C1Squeeze* sq) {
  *ran = false;
  if (N == 0 || !pln.f16 || pln.xmode != F16_X_NHWC_PAIR) return ORE_OK;
  if (x_ps == 0) x_ps = H * W;
  if (y_ps == 0) y_ps = M;
  int tr = 0, tc = 0;
  if (epool_tile(win.Ho, win.Wo, ep.kh, ep.kw, ep.sh, ep.sw, ep.win, &tr, &tc) == 0.0) return ORE_OK;
  if (!fits_i32(N * int64_t(tr) * tc) || !fits_i32(C * x_ps) || !fits_i32(y_ps * ep.win.Ho * ep.win.Wo) || x_ps < H * W)
    return ORE_OK;
  ConvParams p{};
  p.x = x; p.wp = static_cast<const float*>(wp); p.bias = bias; p.y = static_cast<float*>(y);
  p.N = int(N); p.C = int(C); p.H = int(H); p.W = int(W);
  p.M = int(M); p.kh = int(kh); p.kw = int(kw); p.sh = int(sh); p.sw = int(sw);
  p.pt = int(win.pt); p.pl = int(win.pl); p.Ho = int(win.Ho); p.Wo = int(win.Wo);
  p.K = f16_conv_k(pln.xmode, int(C), int(kh), int(kw));
  p.x_ps = int(x_ps); p.y_ps = int(y_ps);
  p.x_nstride = x_nstride; p.y_nstride = y_nstride;
  p.relu = relu ? 1 : 0;
  p.Mp = pln.Mp;
  p.ep_pt = int(ep.win.pt); p.ep_pl = int(ep.win.pl); p.ep_Ho = int(ep.win.Ho); p.ep_Wo = int(ep.win.Wo);
  p.ep_tr = tr; p.ep_tc = tc;
  if (!conv_pair_pool_f16_eligible(p, sq)) return ORE_OK;
  if (pln.epv == C1_BAND_F16_VARIANT && sq && conv_band_pool_f16_eligible(p, sq)) {  // the band walker (round 6)
    launch_conv_band_pool_f16(p, *sq, ctx->stream);
    last_conv_tile = C1_BAND_F16_TILE;
  } else {
    launch_conv_pair_pool_f16(p, sq, ctx->stream);
    last_conv_tile = C1_POOL_F16_TILE;
  }
  ORE_HIP_CHECK(ctx, hipGetLastError());
  *ran = true;
  return ORE_OK;
}

ore_status run_conv_f16(ore_ctx* ctx, const ConvPlan& pln, const void* x, int64_t N, int64_t C, int64_t H, int64_t W,
                        int64_t x_nstride, int64_t x_ps, const void* wp, const int2* ktab, int64_t M, int64_t kh,
                        int64_t kw, const float* bias, const Window& win, int64_t sh, int64_t sw, bool relu, void* y,
                        int64_t y_nstride, int64_t y_ps, const F16Epool* ep) {
  if (N == 0) return ORE_OK;
  if (!pln.f16) return set_error(ctx, ORE_ERR_INVALID, "internal: run_conv_f16 needs an f16 plan");
  const bool nchw = pln.xmode == F16_X_NCHW32;
  if (x_ps == 0) x_ps = nchw ? H * W : C;
  if (y_ps == 0) y_ps = M;
  if (nchw ? x_ps < H * W : x_ps < C) return set_error(ctx, ORE_ERR_INVALID, "input stride below its extent");
  if (y_ps < M) return set_error(ctx, ORE_ERR_INVALID, "output pixel stride below the channel count");
  if (pln.xmode == F16_X_NHWC_VEC &&
      (C % 8 || x_ps % 8 || x_nstride % 8 || (reinterpret_cast<uintptr_t>(x) & 15)))
    return set_error(ctx, ORE_ERR_INVALID, "internal: 16-B NHWC gather needs C, strides %% 8 == 0 and an aligned input");
  if (pln.xmode == F16_X_NHWC_PAIR && (C > 4 || x_ps != 4 || x_nstride % 4 || (reinterpret_cast<uintptr_t>(x) & 7)))
    return set_error(ctx, ORE_ERR_INVALID, "internal: the tap-pair gather needs an NHWC4 input");
  if (!ktab) return set_error(ctx, ORE_ERR_INVALID, "internal: gather table missing");
  ConvParams p{};
  p.x = static_cast<const float*>(x); p.wp = static_cast<const float*>(wp); p.ktab = ktab; p.bias = bias;
  p.y = static_cast<float*>(y);
  p.N = int(N); p.C = int(C); p.H = int(H); p.W = int(W);
  p.M = int(M); p.kh = int(kh); p.kw = int(kw); p.sh = int(sh); p.sw = int(sw);
  p.pt = int(win.pt); p.pl = int(win.pl);
  p.Ho = int(win.Ho); p.Wo = int(win.Wo);
  p.K = f16_conv_k(pln.xmode, int(C), int(kh), int(kw));
  p.P = int(win.Ho * win.Wo);
  p.x_ps = int(x_ps);
  p.y_ps = int(y_ps);
  p.Ntot = N * p.P;
  p.x_nstride = x_nstride;
  p.y_nstride = y_nstride;
  p.relu = relu ? 1 : 0;
  p.Mp = pln.Mp;
  p.x_f32 = nchw ? 1 : 0;
  p.vec_out = (M % 8 == 0 && y_ps % 8 == 0 && y_nstride % 8 == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0) ? 1 : 0;
  if (ep) {  // pooled epilogue: y is the pool's NHWC output [pwin.Ho][pwin.Wo]
    int tr = 0, tc = 0;
    if (epool_tile(win.Ho, win.Wo, ep->kh, ep->kw, ep->sh, ep->sw, ep->win, &tr, &tc) == 0.0)
      return set_error(ctx, ORE_ERR_INVALID, "internal: the pooled epilogue takes 3x3 / stride-2 pools");
    p.ep_pt = int(ep->win.pt); p.ep_pl = int(ep->win.pl); p.ep_Ho = int(ep->win.Ho); p.ep_Wo = int(ep->win.Wo);
    p.ep_tr = tr; p.ep_tc = tc;
    p.Ntot = N * int64_t(tr) * tc * CONV_EPOOL_BN;
  }
  if (!fits_i32(x_nstride * N + 256) || !fits_i32(y_nstride * N + 256) || !fits_i32(int64_t(pln.krows) * pln.Mp) ||
      !fits_i32(p.Ntot + 256) || (p.Ntot + 127) / 128 * ((M + 31) / 32) >= (int64_t(1) << 31))
    return set_error(ctx, ORE_ERR_INVALID, "conv geometry exceeds 32-bit indexing");
  // image chunks whose extents fit the kernels' 32-bit byte offsets (the NHWC_VEC kernel reads x
  // through a buffer resource)
  const int xes = nchw ? 4 : 2;
  const int64_t x_img = (nchw ? C * x_ps : H * W * x_ps) * xes;
  const int64_t y_img = (ep ? ep->win.Ho * ep->win.Wo : win.Ho * win.Wo) * y_ps * 2;
  const int64_t nb = image_chunk(N, x_nstride, x_img, xes, y_nstride, y_img, 2);
  if (nb == 0) return set_error(ctx, ORE_ERR_UNSUPPORTED, "f16 conv: one image exceeds 2 GiB");
  for (int64_t i0 = 0; i0 < N; i0 += nb) {
    const int64_t nc = std::min(nb, N - i0);
    ConvParams q = p;
    q.x = reinterpret_cast<const float*>(static_cast<const char*>(x) + i0 * x_nstride * xes);
    q.y = reinterpret_cast<float*>(static_cast<char*>(y) + i0 * y_nstride * 2);
    q.N = int(nc);
    q.Ntot = ep ? nc * int64_t(p.ep_tr) * p.ep_tc * CONV_EPOOL_BN : nc * p.P;
    q.x_bytes = (nc - 1) * x_nstride * xes + x_img;
    if (ep)
      launch_conv_f16_epool(q, pln.xmode, ctx->stream);
    else
      launch_conv(q, pln, ctx->stream);
    ORE_HIP_CHECK(ctx, hipGetLastError());
  }
  return ORE_OK;
}

ore_status run_maxpool_nhwc(ore_ctx* ctx, const void* x, int64_t N, int64_t C, int64_t H, int64_t W, int64_t x_nstride,
                            int64_t x_cs, int64_t kh, int64_t kw, const Window& win, int64_t sh, int64_t sw, void* y,
                            int64_t y_nstride, int64_t y_cs) {
  if (N == 0) return ORE_OK;
  NhwcPoolParams p{};
  p.x = static_cast<const _Float16*>(x); p.y = static_cast<_Float16*>(y);
  p.N = int(N); p.C = int(C); p.H = int(H); p.W = int(W);
  p.kh = int(kh); p.kw = int(kw); p.sh = int(sh); p.sw = int(sw);
  p.pt = int(win.pt); p.pl = int(win.pl);
  p.Ho = int(win.Ho); p.Wo = int(win.Wo);
  p.x_cs = int(x_cs ? x_cs : C); p.y_cs = int(y_cs ? y_cs : C);
  p.x_nstride = x_nstride; p.y_nstride = y_nstride;
  launch_maxpool_nhwc(p, ctx->stream);
  ORE_HIP_CHECK(ctx, hipGetLastError());
  return ORE_OK;
}

ore_status run_maxpool(ore_ctx* ctx, const float* x, int64_t N, int64_t C, int64_t H, int64_t W,
                       int64_t x_nstride, int64_t kh, int64_t kw, const Window& win, int64_t sh, int64_t sw,
                       float* y, int64_t y_nstride, int64_t x_ps, int64_t y_ps, int es) {
  if (N == 0) return ORE_OK;
  PoolParams p{};
  p.es = es;
  p.variant = ctx->pool_variant;
  p.x_ps = int(x_ps ? x_ps : H * W);
  p.y_ps = int(y_ps ? y_ps : win.Ho * win.Wo);
  p.x = x; p.y = y;
  p.N = int(N); p.C = int(C); p.H = int(H); p.W = int(W);
  p.kh = int(kh); p.kw = int(kw); p.sh = int(sh); p.sw = int(sw);
  p.pt = int(win.pt); p.pl = int(win.pl);
  p.Ho = int(win.Ho); p.Wo = int(win.Wo);
  p.x_nstride = x_nstride; p.y_nstride = y_nstride;
  launch_maxpool(p, ctx->stream);
  ORE_HIP_CHECK(ctx, hipGetLastError());
  return ORE_OK;
}

}  // namespace ore

using namespace ore;

// =================================================================================== C ABI
extern "C" {

int32_t ore_abi_version(void) { return ORE_ABI_VERSION; }

const char* ore_last_error(ore_ctx* ctx) { return ctx ? ctx->err.c_str() : g_global_err.c_str(); }

ore_status ore_ctx_create(int32_t device, ore_ctx** out) {
  if (!out) return set_error(nullptr, ORE_ERR_INVALID, "null out");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) return set_error(nullptr, ORE_ERR_HIP, "no HIP device available");
  if (device < 0 || device >= n) return set_error(nullptr, ORE_ERR_INVALID, "device %d out of range", device);
  ORE_HIP_CHECK(nullptr, hipSetDevice(device));
  ore_ctx* c = new ore_ctx();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return set_error(nullptr, ORE_ERR_HIP, "hipStreamCreate failed");
  }
  c->stream = c->own_stream;
  *out = c;
  return ORE_OK;
}

ore_status ore_ctx_destroy(ore_ctx* ctx) {
  if (!ctx) return ORE_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  else (void)hipDeviceSynchronize();
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->own_stream) {
    (void)hipStreamSynchronize(ctx->own_stream);
    (void)hipStreamDestroy(ctx->own_stream);
  }
  delete ctx;
  return ORE_OK;
}

ore_status ore_ctx_set_conv_algo(ore_ctx* ctx, int32_t algo) {
  if (!ctx) return set_error(nullptr, ORE_ERR_INVALID, "null context");
  if (algo != ORE_CONV_ALGO_DIRECT && algo != ORE_CONV_ALGO_WINOGRAD)
    return set_error(ctx, ORE_ERR_INVALID, "unknown conv algorithm %d", int(algo));
  ctx->conv_algo = algo;
  return ORE_OK;
}

ore_status ore_ctx_set_conv_tile(ore_ctx* ctx, int32_t tile) {
  if (!ctx) return set_error(nullptr, ORE_ERR_INVALID, "null context");
  const bool sp = tile >= CONV_TILE_SP && tile < CONV_TILE_SP + CONV_TILES_SP;
  if (conv_tile_retired(tile)) return set_error(ctx, ORE_ERR_UNSUPPORTED, "conv tile %d was retired (ABI 2)", int(tile));
  if (!sp && (tile < -1 || tile >= WINO_TILE_BASE + WINO_TILES_N))
    return set_error(ctx, ORE_ERR_INVALID, "conv tile %d is not a conv tile id", int(tile));
  ctx->conv_tile = tile;
  return ORE_OK;
}

ore_status ore_ctx_set_pool_variant(ore_ctx* ctx, int32_t variant) {
  if (!ctx) return set_error(nullptr, ORE_ERR_INVALID, "null context");
  if (variant == 1) return set_error(ctx, ORE_ERR_UNSUPPORTED, "MaxPool variant 1 was retired (ABI 2)");
  if (variant != 0 && (variant < 2 || variant > 5)) return set_error(ctx, ORE_ERR_INVALID, "unknown MaxPool variant %d", int(variant));
  ctx->pool_variant = variant;
  return ORE_OK;
}

ore_status ore_ctx_set_stream(ore_ctx* ctx, void* s) {
  if (!ctx) return set_error(nullptr, ORE_ERR_INVALID, "null ctx");
  ctx->stream = reinterpret_cast<hipStream_t>(s);
  return ORE_OK;
}

void* ore_ctx_get_stream(ore_ctx* ctx) { return ctx ? reinterpret_cast<void*>(ctx->stream) : nullptr; }

ore_status ore_sync(ore_ctx* ctx) {
  if (!ctx) return set_error(nullptr, ORE_ERR_INVALID, "null ctx");
  ORE_HIP_CHECK(ctx, hipSetDevice(ctx->device));
  ORE_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
  return ORE_OK;
}

ore_status ore_malloc(ore_ctx* ctx, size_t bytes, void** dptr) {
  if (!ctx || !dptr) return set_error(ctx, ORE_ERR_INVALID, "null argument");
  ORE_HIP_CHECK(ctx, hipSetDevice(ctx->device));
  if (hipMalloc(dptr, bytes ? bytes : 1) != hipSuccess) return set_error(ctx, ORE_ERR_OOM, "hipMalloc(%zu) failed", bytes);
  return ORE_OK;
}

ore_status ore_free(ore_ctx* ctx, void* dptr) {
  if (!ctx) return set_error(nullptr, ORE_ERR_INVALID, "null ctx");
  if (dptr) ORE_HIP_CHECK(ctx, hipFree(dptr));
  return ORE_OK;
}

ore_status ore_upload(ore_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!ctx) return set_error(nullptr, ORE_ERR_INVALID, "null ctx");
  ORE_HIP_CHECK(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  ORE_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
  return ORE_OK;
}

ore_status ore_download(ore_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!ctx) return set_error(nullptr, ORE_ERR_INVALID, "null ctx");
  ORE_HIP_CHECK(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  ORE_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
  return ORE_OK;
}

// ----------------------------------------------------------------------------- shapes
static ore_status conv_geometry(ore_ctx* ctx, const int64_t xd[4], const int64_t wd[4], const ore_conv_attrs* a,
                                Window* win) {
  if (!a) return set_error(ctx, ORE_ERR_INVALID, "null conv attrs");
  if (a->group != 1 || xd[1] != wd[1])  // assert at convolution_op.rs:252
    return set_error(ctx, ORE_ERR_UNSUPPORTED, "Conv: group must be 1 and Cin must match the weights");
  if (a->dilations[0] != 1 || a->dilations[1] != 1)
    return set_error(ctx, ORE_ERR_UNSUPPORTED, "Conv: dilation > 1 is not supported by the reference path");
  int auto_pad = a->auto_pad;
  if (a->n_pads >= 4 && (a->pads[0] > 0 || a->pads[1] > 0 || a->pads[2] > 0 || a->pads[3] > 0))
    auto_pad = ORE_PAD_NOTSET;  // convolution_op.rs:169-173
  return resolve_window(ctx, auto_pad, a->pads, a->n_pads, xd[2], xd[3], wd[2], wd[3], a->strides[0],
                        a->strides[1], win);
}

ore_status ore_conv_out_shape(const int64_t x_dims[4], const int64_t w_dims[4], const ore_conv_attrs* a,
                              int64_t y_dims[4], int64_t pads_tlbr[4]) {
  Window win;
  ore_status st = conv_geometry(nullptr, x_dims, w_dims, a, &win);
  if (st) return st;
  y_dims[0] = x_dims[0]; y_dims[1] = w_dims[0]; y_dims[2] = win.Ho; y_dims[3] = win.Wo;
  if (pads_tlbr) { pads_tlbr[0] = win.pt; pads_tlbr[1] = win.pl; pads_tlbr[2] = win.pb; pads_tlbr[3] = win.pr; }
  return ORE_OK;
}

ore_status ore_pool_out_shape(const int64_t x_dims[4], const ore_pool_attrs* a, int64_t y_dims[4],
                              int64_t pads_tlbr[4]) {
  if (!a) return set_error(nullptr, ORE_ERR_INVALID, "null pool attrs");
  Window win;
  ore_status st = resolve_window(nullptr, a->auto_pad, a->pads, a->n_pads, x_dims[2], x_dims[3], a->kernel[0],
                                 a->kernel[1], a->strides[0], a->strides[1], &win);
  if (st) return st;
  y_dims[0] = x_dims[0]; y_dims[1] = x_dims[1]; y_dims[2] = win.Ho; y_dims[3] = win.Wo;
  if (pads_tlbr) { pads_tlbr[0] = win.pt; pads_tlbr[1] = win.pl; pads_tlbr[2] = win.pb; pads_tlbr[3] = win.pr; }
  return ORE_OK;
}

// ----------------------------------------------------------------------------- ops
ore_status ore_conv2d_f32(ore_ctx* ctx, const ore_tensor* x, const ore_tensor* w, const ore_tensor* bias,
                          const ore_conv_attrs* a, ore_tensor* y) {
  if (!ctx || !x || !w || !y || !a) return set_error(ctx, ORE_ERR_INVALID, "null argument");
  if (x->ndim != 4 || w->ndim != 4 || y->ndim != 4) return set_error(ctx, ORE_ERR_INVALID, "Conv expects 4-D x, w, y");
  if (!contiguous(w)) return set_error(ctx, ORE_ERR_INVALID, "Conv weights must be contiguous");
  Window win;
  ore_status st = conv_geometry(ctx, x->dims, w->dims, a, &win);
  if (st) return st;
  if (bias && (bias->ndim != 1 || bias->dims[0] != w->dims[0]))
    return set_error(ctx, ORE_ERR_INVALID, "Bias array has the wrong shape");  // add_bias :710
  if (y->dims[0] != x->dims[0] || y->dims[1] != w->dims[0] || y->dims[2] != win.Ho || y->dims[3] != win.Wo)
    return set_error(ctx, ORE_ERR_INVALID, "Conv output dims mismatch: expected [%lld,%lld,%lld,%lld]",
                     (long long)x->dims[0], (long long)w->dims[0], (long long)win.Ho, (long long)win.Wo);
  if (x->dims[0] == 0) return ORE_OK;
  const int2* kt = nullptr;
  const ConvPlan pln = conv_plan(w->dims[0], w->dims[1], x->dims[2], x->dims[3], w->dims[2], w->dims[3], a->strides[0],
                                 a->strides[1], win, false, 0, ctx->conv_algo == ORE_CONV_ALGO_WINOGRAD,
                                 ctx->conv_tile);
  float* wp = pack_to_scratch(ctx, pln, w->data, false, w->dims[0], w->dims[1], w->dims[2], w->dims[3], x->dims[2],
                              x->dims[3], &kt);
  if (!wp) return ORE_ERR_OOM;
  return run_conv(ctx, pln, x->data, x->dims[0], x->dims[1], x->dims[2], x->dims[3], nstride_of(x), wp, kt, w->dims[0],
                  w->dims[2], w->dims[3], bias ? bias->data : nullptr, win, a->strides[0], a->strides[1],
                  a->fuse_relu != 0, y->data, nstride_of(y));
}

ore_status ore_maxpool2d_f32(ore_ctx* ctx, const ore_tensor* x, const ore_pool_attrs* a, ore_tensor* y) {
  if (!ctx || !x || !y || !a) return set_error(ctx, ORE_ERR_INVALID, "null argument");
  if (x->ndim != 4 || y->ndim != 4) return set_error(ctx, ORE_ERR_INVALID, "MaxPool expects 4-D tensors");
  Window win;
  ore_status st = resolve_window(ctx, a->auto_pad, a->pads, a->n_pads, x->dims[2], x->dims[3], a->kernel[0],
                                 a->kernel[1], a->strides[0], a->strides[1], &win);
  if (st) return st;
  if (y->dims[0] != x->dims[0] || y->dims[1] != x->dims[1] || y->dims[2] != win.Ho || y->dims[3] != win.Wo)
    return set_error(ctx, ORE_ERR_INVALID, "MaxPool output dims mismatch");
  return run_maxpool(ctx, x->data, x->dims[0], x->dims[1], x->dims[2], x->dims[3], nstride_of(x), a->kernel[0],
                     a->kernel[1], win, a->strides[0], a->strides[1], y->data, nstride_of(y));
}

ore_status ore_relu_f32(ore_ctx* ctx, const ore_tensor* x, ore_tensor* y) {
  if (!ctx || !x || !y) return set_error(ctx, ORE_ERR_INVALID, "null argument");
  if (numel(x) != numel(y)) return set_error(ctx, ORE_ERR_INVALID, "Relu size mismatch");
  if (!contiguous(x) || !contiguous(y)) return set_error(ctx, ORE_ERR_INVALID, "Relu expects contiguous tensors");
  launch_relu(x->data, y->data, numel(x), ctx->stream);
  ORE_HIP_CHECK(ctx, hipGetLastError());
  return ORE_OK;
}

ore_status ore_add_f32(ore_ctx* ctx, const ore_tensor* a, const ore_tensor* b, ore_tensor* y) {
  if (!ctx || !a || !b || !y) return set_error(ctx, ORE_ERR_INVALID, "null argument");
  if (b->ndim > a->ndim || a->ndim > 4 || a->ndim < 1) return set_error(ctx, ORE_ERR_INVALID, "Add: rank mismatch");
  if (!contiguous(a) || !contiguous(b) || !contiguous(y) || numel(a) != numel(y))
    return set_error(ctx, ORE_ERR_INVALID, "Add expects contiguous, same-size a and y");
  AddParams p{};
  p.a = a->data; p.b = b->data; p.y = y->data;
  int64_t bd[4] = {1, 1, 1, 1};
  for (int i = 0; i < 4; ++i) p.d[i] = 1;
  for (int i = 0; i < a->ndim; ++i) p.d[4 - a->ndim + i] = a->dims[i];
  for (int i = 0; i < b->ndim; ++i) bd[4 - b->ndim + i] = b->dims[i];
  int64_t s = 1;
  for (int i = 3; i >= 0; --i) {
    if (bd[i] != 1 && bd[i] != p.d[i]) return set_error(ctx, ORE_ERR_INVALID, "Add: shapes not broadcastable");
    p.bs[i] = bd[i] == 1 ? 0 : s;
    s *= bd[i];
  }
  if (numel(a) == 0) return ORE_OK;
  launch_add_bcast(p, ctx->stream);
  ORE_HIP_CHECK(ctx, hipGetLastError());
  return ORE_OK;
}

ore_status ore_softmax_f32(ore_ctx* ctx, const ore_tensor* x, ore_tensor* y) {
  if (!ctx || !x || !y) return set_error(ctx, ORE_ERR_INVALID, "null argument");
  if (!contiguous(x) || !contiguous(y) || numel(x) != numel(y))
    return set_error(ctx, ORE_ERR_INVALID, "Softmax expects contiguous same-size tensors");
  const int64_t rows = x->dims[0];
  if (rows == 0) return ORE_OK;
  const int64_t D = numel(x) / rows;
  if (D <= 0 || D >= (int64_t(1) << 31)) return set_error(ctx, ORE_ERR_INVALID, "Softmax row length");
  launch_softmax(x->data, y->data, rows, int(D), ctx->stream);
  ORE_HIP_CHECK(ctx, hipGetLastError());
  return ORE_OK;
}

ore_status ore_matmul_f32(ore_ctx* ctx, const ore_tensor* a, const ore_tensor* b, ore_tensor* y) {
  if (!ctx || !a || !b || !y) return set_error(ctx, ORE_ERR_INVALID, "null argument");
  if (a->ndim != 2 || b->ndim != 2 || y->ndim != 2 || a->dims[1] != b->dims[0] || y->dims[0] != a->dims[0] ||
      y->dims[1] != b->dims[1])
    return set_error(ctx, ORE_ERR_INVALID, "MatMul expects a[M,K] . b[K,N] -> y[M,N]");
  if (!contiguous(a) || !contiguous(b) || !contiguous(y))
    return set_error(ctx, ORE_ERR_INVALID, "MatMul expects contiguous tensors");
  // y[m][n] = sum_k a[m][k] b[k][n]  ==  1x1 conv over "images" m with Cin = K, Cout = N and
  // K-major weights b: the MFMA implicit-GEMM kernel, columns = rows of a.
  Window win;
  win.Ho = 1; win.Wo = 1;
  if (a->dims[0] == 0) return ORE_OK;
  const int2* kt = nullptr;
  const ConvPlan pln = conv_plan(b->dims[1], b->dims[0], 1, 1, 1, 1, 1, 1, win, false, 0, false, ctx->conv_tile);
  float* wp = pack_to_scratch(ctx, pln, b->data, true, b->dims[1], b->dims[0], 1, 1, 1, 1, &kt);
  if (!wp) return ORE_ERR_OOM;
  return run_conv(ctx, pln, a->data, a->dims[0], a->dims[1], 1, 1, a->dims[1], wp, kt, b->dims[1], 1, 1, nullptr, win, 1, 1,
                  false, y->data, y->dims[1]);
}

ore_status ore_gap_f32(ore_ctx* ctx, const ore_tensor* x, ore_tensor* y) {
  if (!ctx || !x || !y) return set_error(ctx, ORE_ERR_INVALID, "null argument");
  if (x->ndim != 4 || !contiguous(x) || !contiguous(y) || numel(y) != x->dims[0] * x->dims[1])
    return set_error(ctx, ORE_ERR_INVALID, "GlobalAveragePool expects contiguous [N,C,H,W] -> [N,C,1,1]");
  const int64_t HW = x->dims[2] * x->dims[3];
  if (HW <= 0 || HW >= (int64_t(1) << 31)) return set_error(ctx, ORE_ERR_INVALID, "GAP spatial size");
  launch_gap(x->data, 4, y->data, x->dims[0] * x->dims[1], int(HW), int(HW), ctx->stream);
  ORE_HIP_CHECK(ctx, hipGetLastError());
  return ORE_OK;
}

ore_status ore_concat_f32(ore_ctx* ctx, const ore_tensor* a, const ore_tensor* b, int64_t axis, ore_tensor* y) {
  if (!ctx || !a || !b || !y) return set_error(ctx, ORE_ERR_INVALID, "null argument");
  if (a->ndim != 4 || b->ndim != 4 || y->ndim != 4 || axis < 0 || axis > 3)
    return set_error(ctx, ORE_ERR_INVALID, "Concat expects 4-D tensors and axis in [0,3]");
  for (int i = 0; i < 4; ++i) {
    const int64_t want = (i == axis) ? a->dims[i] + b->dims[i] : a->dims[i];
    if ((i != axis && a->dims[i] != b->dims[i]) || y->dims[i] != want)
      return set_error(ctx, ORE_ERR_INVALID, "Concat shape mismatch");
  }
  if (!contiguous(a) || !contiguous(b) || !contiguous(y))
    return set_error(ctx, ORE_ERR_INVALID, "Concat expects contiguous tensors");
  int64_t outer = 1, ia = 1, ib = 1;
  for (int i = 0; i < axis; ++i) outer *= a->dims[i];
  for (int i = int(axis); i < 4; ++i) { ia *= a->dims[i]; ib *= b->dims[i]; }
  if (outer * (ia + ib) == 0) return ORE_OK;
  launch_concat(a->data, b->data, y->data, 4, outer, ia, ib, ctx->stream);
  ORE_HIP_CHECK(ctx, hipGetLastError());
  return ORE_OK;
}

ore_status ore_dropout_f32(ore_ctx* ctx, const ore_tensor* x, ore_tensor* y) {
  if (!ctx || !x || !y) return set_error(ctx, ORE_ERR_INVALID, "null argument");
  if (numel(x) != numel(y) || !contiguous(x) || !contiguous(y))
    return set_error(ctx, ORE_ERR_INVALID, "Dropout size mismatch");
  if (x->data == y->data) return ORE_OK;
  ORE_HIP_CHECK(ctx, hipMemcpyAsync(y->data, x->data, size_t(numel(x)) * 4, hipMemcpyDeviceToDevice, ctx->stream));
  return ORE_OK;
}

ore_status ore_reshape(const ore_tensor* x, const int64_t* shape, int32_t n_shape, ore_tensor* y) {
  if (!x || !shape || !y) return set_error(nullptr, ORE_ERR_INVALID, "null argument");
  if (n_shape != 2) return set_error(nullptr, ORE_ERR_UNSUPPORTED, "Reshape produces 2-D only (reshape_op.rs:87-91)");
  if (!contiguous(x)) return set_error(nullptr, ORE_ERR_INVALID, "Reshape of a strided view");
  int64_t ns[2] = {shape[0], shape[1]};
  for (int i = 0; i < 2; ++i)
    if (ns[i] == 0) ns[i] = x->dims[i];  // allowzero = 0 (:69-83)
  if (ns[0] < 0 || ns[1] < 0 || ns[0] * ns[1] != numel(x))
    return set_error(nullptr, ORE_ERR_INVALID, "Reshape element count mismatch");
  *y = ore_tensor{};
  y->data = x->data;
  y->ndim = 2;
  y->dims[0] = ns[0];
  y->dims[1] = ns[1];
  return ORE_OK;
}

}  // extern "C"
