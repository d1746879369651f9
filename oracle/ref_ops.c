/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called from the product
 * path (libore.so / the `ore` Python package).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may use it, and only as the checker / the CPU baseline.
 *
 * Plain-C restatement of the reference's fp32 op algorithms
 * (jackperlo/onnx-rusty-inference-engine, src/inference_fp32_ops/ *.rs), extended from the
 * reference's batch-1 to batch N by running the reference's per-image algorithm on each image.
 * Arithmetic ORDER follows the reference so results are as close to bit-identical as the
 * unpinned third-party pieces allow:
 *   - Conv:   out = 0; for cin: out += ndarray_sum(row_mul[k*k]); then out + bias
 *             (convolution_op.rs:407-516, add_bias :705-726).  row_mul is an f32 product per
 *             element (:461-464), summed by ndarray 0.15 `unrolled_fold` (8 partial sums).
 *   - GAP:    sequential Iterator::sum then / count (global_average_pool_op.rs:44-48).
 *   - Softmax: fold max from -inf, subtract, expf, ndarray sum_axis (unrolled_fold), divide
 *             (softmax_op.rs:45-57).
 *   - MatMul: ndarray Array2::dot -> matrixmultiply sgemm (mul_op.rs:23).  matrixmultiply's
 *             micro-kernel order is unpinned (Cargo.lock is git-ignored); restated as a plain
 *             k-ordered sum — tolerance parity only.
 * ndarray 0.15.x `numeric_util::unrolled_fold` is restated from its published source (8
 * accumulators p0..p7 over chunks of 8; acc = 0 + (p0+p4), + (p1+p5), + (p2+p6), + (p3+p7);
 * then the <8 tail sequentially).  Version unpinned: ndarray "0.15.3" semver range in
 * Cargo.toml:17, Cargo.lock ignored (.gitignore:5).
 *
 * The `faithful` flag reproduces the reference's COST structure (not its arithmetic, which is
 * identical either way): a fresh zeroed heap buffer for every per-(oc, pixel, cin) row product
 * (`Array1::zeros`, convolution_op.rs:461), a full im2col + ker2col materialisation per image
 * (:326-390), the zero-padded input copy (:351-362).  Used for the CPU baseline.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ref_ops.h"

/* ndarray 0.15 numeric_util::unrolled_fold(xs, A::zero, A::add) — see header comment. */
float oref_ndarray_sum(const float* xs, int64_t n) {
  float acc = 0.0f;
  float p0 = 0.0f, p1 = 0.0f, p2 = 0.0f, p3 = 0.0f, p4 = 0.0f, p5 = 0.0f, p6 = 0.0f, p7 = 0.0f;
  while (n >= 8) {
    p0 = p0 + xs[0];
    p1 = p1 + xs[1];
    p2 = p2 + xs[2];
    p3 = p3 + xs[3];
    p4 = p4 + xs[4];
    p5 = p5 + xs[5];
    p6 = p6 + xs[6];
    p7 = p7 + xs[7];
    xs += 8;
    n -= 8;
  }
  acc = acc + (p0 + p4);
  acc = acc + (p1 + p5);
  acc = acc + (p2 + p6);
  acc = acc + (p3 + p7);
  for (int64_t i = 0; i < n && i < 7; ++i) acc = acc + xs[i];
  return acc;
}

/* get_padding_size (convolution_op.rs:519-557, max_pool_op.rs:363-401): the larger half of the
 * SAME padding goes to the TOP/LEFT (the reference swaps them on return, :547-556).  usize
 * arithmetic: kernel < stride would underflow (panic in debug) -> error. */
int oref_same_padding(int64_t in_h, int64_t in_w, int64_t sh, int64_t sw, int64_t kh, int64_t kw,
                      int64_t pads_tlbr[4]) {
  int64_t ph, pw;
  if (sh <= 0 || sw <= 0) return -1;
  if (in_h % sh == 0) ph = kh - sh; else ph = kh - (in_h % sh);
  if (in_w % sw == 0) pw = kw - sw; else pw = kw - (in_w % sw);
  if (ph < 0 || pw < 0) return -1;
  int64_t top_small = ph / 2, left_small = pw / 2;
  pads_tlbr[0] = ph - top_small;  /* pad_top    <- returned "pad_bottom" */
  pads_tlbr[1] = pw - left_small; /* pad_left   <- returned "pad_right"  */
  pads_tlbr[2] = top_small;       /* pad_bottom <- returned "pad_top"    */
  pads_tlbr[3] = left_small;      /* pad_right  <- returned "pad_left"   */
  return 0;
}

/* Output size + resolved padding for Conv (convolution_op.rs:266-324, 334-350) and MaxPool
 * (max_pool_op.rs:188-264).  auto_pad: 0 NotSet, 1 SameUpper, 2 SameLower, 3 Valid.
 * pads_attr is ONNX order [h_begin, w_begin, h_end, w_end] (read at :267-278). */
int oref_resolve_window(int auto_pad, const int64_t* pads_attr, int n_pads, int64_t H, int64_t W,
                        int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t pads_tlbr[4],
                        int64_t* Ho, int64_t* Wo) {
  if (sh <= 0 || sw <= 0 || kh <= 0 || kw <= 0) return -1;
  pads_tlbr[0] = pads_tlbr[1] = pads_tlbr[2] = pads_tlbr[3] = 0;
  switch (auto_pad) {
    case 1:
    case 2:
      *Ho = (int64_t)ceilf((float)H / (float)sh);
      *Wo = (int64_t)ceilf((float)W / (float)sw);
      return oref_same_padding(H, W, sh, sw, kh, kw, pads_tlbr);
    case 0: {
      if (n_pads < 4) return -1; /* pads_arr.get(k).unwrap() panics */
      int64_t ht = pads_attr[0], hb = pads_attr[2], wl = pads_attr[1], wr = pads_attr[3];
      if (ht < 0 || hb < 0 || wl < 0 || wr < 0) return -1;
      if (H + ht + hb < kh || W + wl + wr < kw) return -1;
      *Ho = (H - kh + (ht + hb)) / sh + 1;
      *Wo = (W - kw + (wl + wr)) / sw + 1;
      pads_tlbr[0] = ht; pads_tlbr[1] = wl; pads_tlbr[2] = hb; pads_tlbr[3] = wr;
      return 0;
    }
    case 3:
      if (H < kh || W < kw) return -1;
      *Ho = (H - kh) / sh + 1;
      *Wo = (W - kw) / sw + 1;
      return 0;
    default:
      return -1;
  }
}

/* Zero-padded copy of image n (convolution_op.rs:351-362). */
static float* padded_copy(const float* img, int64_t C, int64_t H, int64_t W, const int64_t p[4],
                          int64_t* Hp, int64_t* Wp) {
  *Hp = H + p[0] + p[2];
  *Wp = W + p[1] + p[3];
  float* out = (float*)calloc((size_t)(C * *Hp * *Wp), sizeof(float));
  for (int64_t c = 0; c < C; ++c)
    for (int64_t h = 0; h < H; ++h)
      memcpy(out + (c * *Hp + h + p[0]) * *Wp + p[1], img + (c * H + h) * W, (size_t)W * sizeof(float));
  return out;
}

/* im2col_ref (convolution_op.rs:560-663 None/dilation-1 branch, max_pool_op.rs:403-449):
 * rows k*P + i*new_w + j, each row the kh x kw patch flattened row-major. */
static float* im2col(const float* img, int64_t C, int64_t Hp, int64_t Wp, int64_t kh, int64_t kw,
                     int64_t sh, int64_t sw, int64_t* P_out) {
  int64_t nh = (Hp - kh) / sh + 1, nw = (Wp - kw) / sw + 1, P = nh * nw, kk = kh * kw;
  float* cols = (float*)calloc((size_t)(C * P * kk), sizeof(float));
  int64_t cont = 0;
  for (int64_t k = 0; k < C; ++k)
    for (int64_t i = 0; i < nh; ++i)
      for (int64_t j = 0; j < nw; ++j, ++cont) {
        float* row = cols + cont * kk;
        for (int64_t a = 0; a < kh; ++a)
          for (int64_t b = 0; b < kw; ++b)
            row[a * kw + b] = img[(k * Hp + i * sh + a) * Wp + j * sw + b];
      }
  *P_out = P;
  return cols;
}

/* ker2col_ref (convolution_op.rs:666-703) after new_onnx_tensor_flow's [1,0,3,2] permute
 * (:57-71): row oc*C + cin holds W[oc, cin, :, :] flattened in (kh, kw) order. */
static float* ker2col(const float* w, int64_t M, int64_t C, int64_t kh, int64_t kw) {
  int64_t kk = kh * kw;
  float* out = (float*)calloc((size_t)(M * C * kk), sizeof(float));
  /* permuted[c][m][b][a] = w[m][c][a][b]; ker2col reads permuted[w=cin][k=oc][j-1][i-1] */
  for (int64_t oc = 0; oc < M; ++oc)
    for (int64_t cin = 0; cin < C; ++cin)
      for (int64_t a = 0; a < kh; ++a)
        for (int64_t b = 0; b < kw; ++b)
          out[(oc * C + cin) * kk + a * kw + b] = w[((oc * C + cin) * kh + a) * kw + b];
  return out;
}

/* conv2d (convolution_op.rs:224-517) for every image of the batch; y is [N, M, Ho, Wo]. */
int oref_conv2d(const float* x, int64_t N, int64_t C, int64_t H, int64_t W, const float* w, int64_t M,
                int64_t kh, int64_t kw, const float* bias, const int64_t pads_tlbr[4], int64_t sh,
                int64_t sw, int64_t Ho, int64_t Wo, float* y, int faithful) {
  int64_t kk = kh * kw;
  float* kcol = ker2col(w, M, C, kh, kw);
  float* scratch = (float*)malloc((size_t)kk * sizeof(float));
  for (int64_t n = 0; n < N; ++n) {
    const float* img = x + n * C * H * W;
    int64_t Hp, Wp, P;
    float* padded = padded_copy(img, C, H, W, pads_tlbr, &Hp, &Wp);
    float* cols = im2col(padded, C, Hp, Wp, kh, kw, sh, sw, &P);
    free(padded);
    if (P != Ho * Wo) { free(cols); free(kcol); free(scratch); return -1; }
    float* out = y + n * M * P;
    memset(out, 0, (size_t)(M * P) * sizeof(float)); /* Array4::zeros (:401) */
    for (int64_t oc = 0; oc < M; ++oc) {
      for (int64_t p = 0; p < P; ++p) {
        float acc = 0.0f;
        for (int64_t cin = 0; cin < C; ++cin) {
          const float* im_row = cols + (cin * P + p) * kk;
          const float* ker_row = kcol + (oc * C + cin) * kk;
          float* row_mul = faithful ? (float*)calloc((size_t)kk, sizeof(float)) : scratch;
          for (int64_t i = 0; i < kk; ++i) row_mul[i] = im_row[i] * ker_row[i];
          acc = acc + oref_ndarray_sum(row_mul, kk);
          if (faithful) free(row_mul);
        }
        out[oc * P + p] = acc;
      }
    }
    if (bias)
      for (int64_t oc = 0; oc < M; ++oc)
        for (int64_t p = 0; p < P; ++p) out[oc * P + p] = out[oc * P + p] + bias[oc];
    free(cols);
  }
  free(kcol);
  free(scratch);
  return 0;
}

/* max_pool2d (max_pool_op.rs:157-360): zero padding (:265-276), fold from f32::MIN (:337). */
int oref_maxpool2d(const float* x, int64_t N, int64_t C, int64_t H, int64_t W, int64_t kh, int64_t kw,
                   const int64_t pads_tlbr[4], int64_t sh, int64_t sw, int64_t Ho, int64_t Wo,
                   float* y, int faithful) {
  (void)faithful;
  int64_t kk = kh * kw;
  for (int64_t n = 0; n < N; ++n) {
    int64_t Hp, Wp, P;
    float* padded = padded_copy(x + n * C * H * W, C, H, W, pads_tlbr, &Hp, &Wp);
    float* cols = im2col(padded, C, Hp, Wp, kh, kw, sh, sw, &P);
    free(padded);
    if (P != Ho * Wo) { free(cols); return -1; }
    for (int64_t c = 0; c < C; ++c)
      for (int64_t p = 0; p < P; ++p) {
        const float* row = cols + (c * P + p) * kk;
        float m = -FLT_MAX;
        for (int64_t i = 0; i < kk; ++i) m = fmaxf(m, row[i]);
        y[(n * C + c) * P + p] = m;
      }
    free(cols);
  }
  return 0;
}

/* relu_wrapper (relu_op.rs:31-33): val.max(0.0) — Rust f32::max = IEEE maxNum = fmaxf. */
void oref_relu(const float* x, int64_t n, float* y) {
  for (int64_t i = 0; i < n; ++i) y[i] = fmaxf(x[i], 0.0f);
}

/* add (add_op.rs:74-84): ndarray broadcasting of b (rank rb, right-aligned) onto a (rank ra). */
int oref_add_bcast(const float* a, const int64_t* adims, int ra, const float* b, const int64_t* bdims,
                   int rb, float* y) {
  if (rb > ra || ra > 4) return -1;
  int64_t bd[4] = {1, 1, 1, 1}, ad[4] = {1, 1, 1, 1};
  for (int i = 0; i < ra; ++i) ad[4 - ra + i] = adims[i];
  for (int i = 0; i < rb; ++i) bd[4 - rb + i] = bdims[i];
  for (int i = 0; i < 4; ++i)
    if (bd[i] != 1 && bd[i] != ad[i]) return -1;
  int64_t bs[4], s = 1;
  for (int i = 3; i >= 0; --i) { bs[i] = (bd[i] == 1) ? 0 : s; s *= bd[i]; }
  int64_t idx = 0;
  for (int64_t i0 = 0; i0 < ad[0]; ++i0)
    for (int64_t i1 = 0; i1 < ad[1]; ++i1)
      for (int64_t i2 = 0; i2 < ad[2]; ++i2)
        for (int64_t i3 = 0; i3 < ad[3]; ++i3, ++idx)
          y[idx] = a[idx] + b[i0 * bs[0] + i1 * bs[1] + i2 * bs[2] + i3 * bs[3]];
  return 0;
}

/* softmax_wrapper (softmax_op.rs:45-57) over rows of length D. */
void oref_softmax_rows(const float* x, int64_t rows, int64_t D, float* y) {
  for (int64_t r = 0; r < rows; ++r) {
    const float* xr = x + r * D;
    float* yr = y + r * D;
    float m = -INFINITY;
    for (int64_t i = 0; i < D; ++i) m = fmaxf(xr[i], m);
    for (int64_t i = 0; i < D; ++i) yr[i] = expf(xr[i] - m);
    float s = oref_ndarray_sum(yr, D);
    for (int64_t i = 0; i < D; ++i) yr[i] = yr[i] / s;
  }
}

/* mul (mul_op.rs:23): Array2::dot, k-ordered sum (see header). */
void oref_matmul(const float* a, const float* b, int64_t M, int64_t K, int64_t Ncols, float* y) {
  for (int64_t i = 0; i < M; ++i)
    for (int64_t j = 0; j < Ncols; ++j) {
      float acc = 0.0f;
      for (int64_t k = 0; k < K; ++k) acc = acc + a[i * K + k] * b[k * Ncols + j];
      y[i * Ncols + j] = acc;
    }
}

/* global_average_pool_wrapper (global_average_pool_op.rs:33-51). */
void oref_gap(const float* x, int64_t N, int64_t C, int64_t HW, float* y) {
  for (int64_t nc = 0; nc < N * C; ++nc) {
    const float* s = x + nc * HW;
    float acc = 0.0f;
    for (int64_t i = 0; i < HW; ++i) acc = acc + s[i];
    y[nc] = acc / (float)HW;
  }
}

/* ndarray::concatenate(Axis(axis), [a, b]) (concatenate_op.rs:31-32) for 4-D row-major. */
int oref_concat2(const float* a, const int64_t* ad, const float* b, const int64_t* bd, int axis,
                 float* y) {
  if (axis < 0 || axis > 3) return -1;
  for (int i = 0; i < 4; ++i)
    if (i != axis && ad[i] != bd[i]) return -1;
  int64_t outer = 1, inner_a = 1, inner_b = 1;
  for (int i = 0; i < axis; ++i) outer *= ad[i];
  for (int i = axis; i < 4; ++i) { inner_a *= ad[i]; inner_b *= bd[i]; }
  for (int64_t o = 0; o < outer; ++o) {
    memcpy(y + o * (inner_a + inner_b), a + o * inner_a, (size_t)inner_a * sizeof(float));
    memcpy(y + o * (inner_a + inner_b) + inner_a, b + o * inner_b, (size_t)inner_b * sizeof(float));
  }
  return 0;
}
