/*
 * oracle.c — CPU restatement of the reference's RRAM fault-simulation hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (rram-caffe-simulation_amd/)
 * links, loads or calls this file; only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, as the checker.
 *
 * Each function cites the reference file:line it restates (paths relative to
 * fightingnoble/rram-caffe-simulation).  Compiled with -ffp-contract=off so the
 * fp32 arithmetic is the plain IEEE sequence the reference's CPU loop performs.
 *
 * Pinning: the fault arithmetic (fail_apply, fault_threshold) has no golden
 * vectors in the reference ("Fault-injection tests: none") and the
 * reference cannot be built here (no protobuf/glog/boost/cblas), so it is
 * pinned by the reference's own source semantics plus hand-derived known-answer
 * cases in tests/golden/ (see tests/golden/make_golden.py).  The GEMM restatement
 * is pinned by the reference's known-answer test test_util_blas.cpp:20-89; the
 * convolution restatement is a transcription of the reference's own test oracle
 * caffe_conv (test_convolution_layer.cpp:21-139).  The Philox stream is pinned by
 * the published Random123 known-answer vectors.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

/* ---------------------------------------------------------------- Philox */
typedef struct { uint32_t x, y, z, w; } u32x4;

/* Philox4x32-10 (Salmon et al., SC'11; Random123 philox4x32_R with R = 10). */
u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    u32x4 n;
    n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
    n.y = (uint32_t)p1;
    n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
    n.w = (uint32_t)p0;
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

void oracle_philox(const uint32_t* ctr, const uint32_t* key, uint32_t* out) {
  u32x4 c = {ctr[0], ctr[1], ctr[2], ctr[3]};
  u32x4 r = philox4x32_10(c, key[0], key[1]);
  out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = r.w;
}

/* Counter layout of the product's fault draws (documented in DESIGN.md §3). */
static u32x4 draw(uint64_t seed, uint64_t index, uint32_t map_id, uint32_t layer_id, uint32_t purpose) {
  u32x4 c = {(uint32_t)index, (uint32_t)(index >> 32), map_id, (layer_id << 4) | (purpose & 15u)};
  return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}
enum { P_FAULT = 0, P_VAR = 1, P_PAIR = 2, P_PAIRVAR = 3, P_ENDUR = 4 };

static float u01_open0(uint32_t r) { return ((float)(r >> 8) + 1.0f) * (1.0f / 16777216.0f); }
static float u01(uint32_t r) { return (float)(r >> 8) * (1.0f / 16777216.0f); }
static void box_muller(uint32_t a, uint32_t b, float* z0, float* z1) {
  float u1 = u01_open0(a), u2 = u01(b);
  float r = sqrtf(-2.0f * logf(u1));
  float th = 6.28318530717958647692f * u2;
  *z0 = r * cosf(th);
  *z1 = r * sinf(th);
}

/* ------------------------------------------------------- fault model a1 */
/* failure_maker.cu:5-16 (FailureThresholdKernel) / failure_maker.cpp:37-48 */
void oracle_fault_threshold(float* v, int64_t n, float split1, float split2) {
  for (int64_t j = 0; j < n; ++j) {
    if (v[j] < split1) v[j] = -1;
    else if (v[j] < split2) v[j] = 0;
    else v[j] = 1;
  }
}

static float stuck_value(uint32_t r, uint64_t thr_neg, uint64_t thr_zero) {
  return ((uint64_t)r < thr_neg) ? -1.0f : (((uint64_t)r < thr_zero) ? 0.0f : 1.0f);
}

/* Restates the GaussianFailureMaker constructor draws (failure_maker.cpp:5-52)
 * on the product's counter-based stream: endurance = mean + std*z, stuck value
 * from a uniform word and the (neg, zero, pos) split. */
void oracle_fault_init(float* e, float* v, int64_t n, float mean, float std, uint64_t thr_neg,
                       uint64_t thr_zero, uint64_t seed, uint32_t map_id, uint32_t layer_id) {
  for (int64_t p = 0; 2 * p < n; ++p) {
    u32x4 re = draw(seed, (uint64_t)p, map_id, layer_id, P_ENDUR);
    u32x4 rf = draw(seed, (uint64_t)p, map_id, layer_id, P_FAULT);
    float z0, z1;
    box_muller(re.x, re.y, &z0, &z1);
    e[2 * p] = fmaf(std, z0, mean);
    v[2 * p] = stuck_value(rf.y, thr_neg, thr_zero);
    if (2 * p + 1 < n) {
      e[2 * p + 1] = fmaf(std, z1, mean);
      v[2 * p + 1] = stuck_value(rf.w, thr_neg, thr_zero);
    }
  }
}

/* ------------------------------------------------------- fault model a2 */
/* GaussianFailureMaker::Fail_cpu, failure_maker.cpp:55-81 (identical arithmetic
 * to FailKernel, failure_maker.cu:23-41):
 *   if (iters <= 0) data = value;
 *   else { if (fabs(diff) < epsilon) continue; iters -= 100; if (iters <= 0) data = value; }
 * Returns the number of cells with iters <= 0 afterwards (the count the
 * reference computes and discards in failure_maker.hpp:37-55). */
int64_t oracle_fail_apply(const float* dw, float* w, float* e, const float* v, int64_t n,
                          float decrement, float eps) {
  int64_t broken = 0;
  for (int64_t j = 0; j < n; ++j) {
    if (e[j] <= 0) {
      w[j] = v[j];
    } else {
      if (fabsf(dw[j]) < eps) {
        /* not a write: no endurance consumed */
      } else {
        e[j] -= decrement;
        if (e[j] <= 0) w[j] = v[j];
      }
    }
    broken += (e[j] <= 0);
  }
  return broken;
}

/* ------------------------------------------------ Monte-Carlo injection */
typedef struct {
  uint64_t thr_fault, thr_neg, thr_zero, thr_sa1;
  float stuck_scale, g_max;
  int32_t quant_levels;
  float var_sigma;
  int32_t cell_mode, reserved;
} oracle_inject_cfg; /* layout == rram_inject_cfg */

static float quant_sym(float w, int L, float gmax, float delta, float inv) {
  float t = (w + gmax) * inv;
  t = rintf(t);
  t = fminf(fmaxf(t, 0.0f), (float)(L - 1));
  return fmaf(t, delta, -gmax);
}
static float quant_pos(float x, int L, float delta, float inv) {
  float t = x * inv;
  t = rintf(t);
  t = fminf(fmaxf(t, 0.0f), (float)(L - 1));
  return t * delta;
}

/* One Monte-Carlo fault map: the reference's "endurance <= 0 at the first
 * Fail()" stuck-at state (failure_maker.cpp:64-66) drawn as
 * Bernoulli(p) per cell, plus the build's extensions (quantisation, lognormal
 * variation, differential pair; parity unpinned vs the reference). */
int64_t oracle_inject(const float* src, float* dst, int64_t n, const oracle_inject_cfg* c,
                      uint64_t seed, uint32_t map_id, uint32_t layer_id) {
  int64_t nb = 0;
  const int L = c->quant_levels >= 2 ? c->quant_levels : 0;
  if (c->cell_mode == 1) {
    float delta = 0.f, inv = 0.f;
    if (L) { delta = c->g_max / (float)(L - 1); inv = 1.0f / delta; }
    for (int64_t i = 0; i < n; ++i) {
      float w = src[i];
      float gp = fmaxf(w, 0.0f), gn = fmaxf(-w, 0.0f);
      if (L) { gp = quant_pos(gp, L, delta, inv); gn = quant_pos(gn, L, delta, inv); }
      u32x4 r = draw(seed, (uint64_t)i, map_id, layer_id, P_PAIR);
      int bp = (uint64_t)r.x < c->thr_fault, bn = (uint64_t)r.z < c->thr_fault;
      if (c->var_sigma > 0.f && !(bp && bn)) {
        u32x4 rz = draw(seed, (uint64_t)i, map_id, layer_id, P_PAIRVAR);
        float z0, z1;
        box_muller(rz.x, rz.y, &z0, &z1);
        gp = gp * expf(c->var_sigma * z0);
        gn = gn * expf(c->var_sigma * z1);
      }
      if (bp) gp = ((uint64_t)r.y < c->thr_sa1) ? c->g_max : 0.0f;
      if (bn) gn = ((uint64_t)r.w < c->thr_sa1) ? c->g_max : 0.0f;
      nb += bp + bn;
      dst[i] = gp - gn;
    }
    return nb;
  }
  float delta = 0.f, inv = 0.f;
  if (L) { delta = (2.0f * c->g_max) / (float)(L - 1); inv = 1.0f / delta; }
  for (int64_t i = 0; i < n; ++i) {
    uint64_t pr = (uint64_t)i >> 1;
    int odd = (int)(i & 1);
    u32x4 r = draw(seed, pr, map_id, layer_id, P_FAULT);
    uint32_t rf = odd ? r.z : r.x, rv = odd ? r.w : r.y;
    float w = src[i];
    if (L) w = quant_sym(w, L, c->g_max, delta, inv);
    int b = (uint64_t)rf < c->thr_fault;
    if (b) {
      w = stuck_value(rv, c->thr_neg, c->thr_zero) * c->stuck_scale;
    } else if (c->var_sigma > 0.f) {
      u32x4 rz = draw(seed, pr, map_id, layer_id, P_VAR);
      float z, t;
      if (odd) box_muller(rz.z, rz.w, &z, &t);
      else box_muller(rz.x, rz.y, &z, &t);
      w = w * expf(c->var_sigma * z);
    }
    nb += b;
    dst[i] = w;
  }
  return nb;
}

/* ------------------------------------------------ strategy / solver a3 a4 */
/* ThresholdFailureStrategy::Apply inner loop, strategy.cpp:20-29 */
int64_t oracle_threshold(float* dw, int64_t n, float thr) {
  int64_t cleared = 0;
  for (int64_t j = 0; j < n; ++j)
    if (fabsf(dw[j]) <= thr) { dw[j] = 0; ++cleared; }
  return cleared;
}

/* SGDUpdate, sgd_solver.cu:9-11: g = h = momentum*h + local_rate*g */
void oracle_sgd_update(float* g, float* h, int64_t n, float momentum, float local_rate) {
  for (int64_t i = 0; i < n; ++i) {
    float v = momentum * h[i] + local_rate * g[i];
    g[i] = v;
    h[i] = v;
  }
}

/* Solver::Step tail in reference order (solver.cpp:300-305): Regularize L2
 * (sgd_solver.cpp:160-166), ComputeUpdateValue (:216-231), threshold strategy
 * (strategy.cpp:7-33), ApplyUpdate -> Blob::Update (blob.cpp:156-179), Fail. */
int64_t oracle_fused_update_fail(float* w, float* g, float* h, float* e, const float* v, int64_t n,
                                 float decay, float mom, float lr, int apply_thr, float thr,
                                 float dec, float eps) {
  int64_t nb = 0;
  for (int64_t i = 0; i < n; ++i) {
    float wi = w[i], gi = g[i];
    if (decay != 0.0f) gi = decay * wi + gi;
    gi = mom * h[i] + lr * gi;
    h[i] = gi;
    if (apply_thr && fabsf(gi) <= thr) gi = 0.0f;
    g[i] = gi;
    wi = wi - gi;
    if (e) {
      if (e[i] <= 0) wi = v[i];
      else if (!(fabsf(gi) < eps)) {
        e[i] -= dec;
        if (e[i] <= 0) wi = v[i];
      }
      nb += (e[i] <= 0);
    }
    w[i] = wi;
  }
  return nb;
}

/* ------------------------------------------------------------- GEMM a8 */
/* caffe_cpu_gemm semantics, math_functions.cpp:12-32 (cblas_sgemm RowMajor,
 * lda = TransA ? M : K, ldb = TransB ? K : N, ldc = N).  fp32 accumulation in
 * k order. */
void oracle_gemm(int ta, int tb, int M, int N, int K, float alpha, const float* A, const float* B,
                 float beta, float* C) {
  for (int m = 0; m < M; ++m)
    for (int n = 0; n < N; ++n) {
      float s = 0.0f;
      for (int k = 0; k < K; ++k) {
        float a = ta ? A[(int64_t)k * M + m] : A[(int64_t)m * K + k];
        float b = tb ? B[(int64_t)n * K + k] : B[(int64_t)k * N + n];
        s += a * b;
      }
      C[(int64_t)m * N + n] = alpha * s + (beta != 0.0f ? beta * C[(int64_t)m * N + n] : 0.0f);
    }
}

/* --------------------------------------------------------- im2col a6 */
/* im2col_cpu, im2col.cpp:18-55 (col is [C*kh*kw][Ho*Wo]) */
void oracle_im2col(const float* im, int C, int H, int W, int kh, int kw, int ph, int pw, int sh,
                   int sw, int dh, int dw, float* col) {
  int Ho = (H + 2 * ph - (dh * (kh - 1) + 1)) / sh + 1;
  int Wo = (W + 2 * pw - (dw * (kw - 1) + 1)) / sw + 1;
  int64_t o = 0;
  for (int c = 0; c < C; ++c)
    for (int a = 0; a < kh; ++a)
      for (int b = 0; b < kw; ++b)
        for (int y = 0; y < Ho; ++y) {
          int iy = -ph + a * dh + y * sh;
          for (int x = 0; x < Wo; ++x) {
            int ix = -pw + b * dw + x * sw;
            col[o++] = ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
                           ? im[((int64_t)c * H + iy) * W + ix] : 0.0f;
          }
        }
}

/* col2im_cpu, im2col.cpp:127-163: accumulate columns back into a zeroed image */
void oracle_col2im(const float* col, int C, int H, int W, int kh, int kw, int ph, int pw, int sh,
                   int sw, int dh, int dw, float* im) {
  int Ho = (H + 2 * ph - (dh * (kh - 1) + 1)) / sh + 1;
  int Wo = (W + 2 * pw - (dw * (kw - 1) + 1)) / sw + 1;
  memset(im, 0, sizeof(float) * (size_t)C * H * W);
  int64_t o = 0;
  for (int c = 0; c < C; ++c)
    for (int a = 0; a < kh; ++a)
      for (int b = 0; b < kw; ++b)
        for (int y = 0; y < Ho; ++y) {
          int iy = -ph + a * dh + y * sh;
          for (int x = 0; x < Wo; ++x, ++o) {
            int ix = -pw + b * dw + x * sw;
            if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
              im[((int64_t)c * H + iy) * W + ix] += col[o];
          }
        }
}

/* ---------------------------------------------------- convolution a5 */
/* caffe_conv, test_convolution_layer.cpp:21-139 (2-D case): explicit loops
 * over n, g, o, k, y, x, p, q; then bias. out must be zeroed by the caller. */
void oracle_conv(const float* in, int N, int C, int H, int W, const float* wt, const float* bias,
                 int Cout, int kh, int kw, int ph, int pw, int sh, int sw, int dh, int dw,
                 int group, float* out) {
  int Ho = (H + 2 * ph - (dh * (kh - 1) + 1)) / sh + 1;
  int Wo = (W + 2 * pw - (dw * (kw - 1) + 1)) / sw + 1;
  int o_g = Cout / group, k_g = C / group;
  for (int n = 0; n < N; ++n)
    for (int g = 0; g < group; ++g)
      for (int o = 0; o < o_g; ++o)
        for (int k = 0; k < k_g; ++k)
          for (int y = 0; y < Ho; ++y)
            for (int x = 0; x < Wo; ++x)
              for (int p = 0; p < kh; ++p)
                for (int q = 0; q < kw; ++q) {
                  int iy = y * sh - ph + p * dh, ix = x * sw - pw + q * dw;
                  if (iy >= 0 && iy < H && ix >= 0 && ix < W)
                    out[(((int64_t)n * Cout + o + o_g * g) * Ho + y) * Wo + x] +=
                        in[(((int64_t)n * C + k + k_g * g) * H + iy) * W + ix] *
                        wt[(((int64_t)(o + o_g * g) * k_g + k) * kh + p) * kw + q];
                }
  if (bias)
    for (int n = 0; n < N; ++n)
      for (int o = 0; o < Cout; ++o)
        for (int i = 0; i < Ho * Wo; ++i) out[((int64_t)n * Cout + o) * Ho * Wo + i] += bias[o];
}
