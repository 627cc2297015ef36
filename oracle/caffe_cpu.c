/*
 * caffe_cpu.c — Caffe CPU mode, restated in C for the CPU baseline.
 *
 * TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg and tests/): the
 * product never links or calls this file.
 *
 * Restates the reference's CPU forward path layer for layer, in the
 * reference's own order and granularity, so the baseline costs what Caffe's
 * `caffe test` / Solver::Test would on these host cores:
 *   Convolution  conv_layer.cpp:7-24 -> base_conv_layer.cpp:256-290: per image
 *                im2col_cpu (im2col.cpp:18-55) then one sgemm per group, then
 *                the bias as a rank-1 sgemm with bias_multiplier_.
 *   InnerProduct inner_product_layer.cpp:83-96: one sgemm (NoTrans, Trans)
 *                plus the rank-1 bias sgemm.
 *   ReLU         relu_layer.cpp:9-19 (scalar loop).
 *   LRN          lrn_layer.cpp:108-155 CrossChannelForward_cpu (padded square,
 *                sliding window of axpy, powx, mul).
 *   Pooling MAX  pooling_layer.cpp:133-176 (scalar loop with argmax mask).
 *   Softmax      softmax_layer.cpp:24-59 (max, subtract, exp, sum, divide).
 * sgemm is cblas_sgemm RowMajor (math_functions.cpp:12-32) from a BLAS the
 * caller names at run time: numpy's bundled OpenBLAS (ILP64, symbol prefix
 * scipy_, mode 0) or an LP64 `cblas_sgemm` such as MKL's libmkl_rt (mode 1).
 * Layers other than sgemm are single-threaded, as in the reference.
 */
#include <dlfcn.h>
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { RowMajor = 101, NoTrans = 111, Trans = 112 };
typedef void (*sgemm64_t)(int, int, int, int64_t, int64_t, int64_t, float, const float*, int64_t, const float*,
                          int64_t, float, float*, int64_t);
typedef void (*sgemm32_t)(int, int, int, int, int, int, float, const float*, int, const float*, int, float,
                          float*, int);
typedef void (*setthreads_t)(int64_t);

static sgemm64_t g_sgemm64;
static sgemm32_t g_sgemm32;

/* Returns 0 on success.  mode 0: ILP64 scipy_-prefixed OpenBLAS; 1: LP64 cblas_sgemm. */
int cc_init(const char* blas_path, int mode, int threads) {
  void* h = dlopen(blas_path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return -1;
  g_sgemm64 = NULL;
  g_sgemm32 = NULL;
  if (mode == 0) {
    g_sgemm64 = (sgemm64_t)dlsym(h, "scipy_cblas_sgemm64_");
    setthreads_t st = (setthreads_t)dlsym(h, "scipy_openblas_set_num_threads64_");
    if (st && threads > 0) st(threads);
    return g_sgemm64 ? 0 : -2;
  }
  g_sgemm32 = (sgemm32_t)dlsym(h, "cblas_sgemm");
  void (*mkl_threads)(int) = (void (*)(int))dlsym(h, "MKL_Set_Num_Threads");
  if (mkl_threads && threads > 0) mkl_threads(threads);
  return g_sgemm32 ? 0 : -2;
}

/* caffe_cpu_gemm (math_functions.cpp:12-32): row-major, lda = ta ? M : K,
 * ldb = tb ? K : N, ldc = N. */
static void gemm(int ta, int tb, int M, int N, int K, float alpha, const float* A, const float* B, float beta,
                 float* C) {
  const int lda = ta ? M : K, ldb = tb ? K : N;
  if (g_sgemm64)
    g_sgemm64(RowMajor, ta ? Trans : NoTrans, tb ? Trans : NoTrans, M, N, K, alpha, A, lda, B, ldb, beta, C, N);
  else
    g_sgemm32(RowMajor, ta ? Trans : NoTrans, tb ? Trans : NoTrans, M, N, K, alpha, A, lda, B, ldb, beta, C, N);
}

void cc_gemm(int ta, int tb, int M, int N, int K, float alpha, const float* A, const float* B, float beta,
             float* C) {
  gemm(ta, tb, M, N, K, alpha, A, B, beta, C);
}

/* im2col_cpu, im2col.cpp:18-55 */
static void im2col(const float* im, int C, int H, int W, int k, int pad, int stride, float* col) {
  const int Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  for (int c = 0; c < C; ++c)
    for (int a = 0; a < k; ++a)
      for (int b = 0; b < k; ++b)
        for (int y = 0; y < Ho; ++y) {
          const int iy = -pad + a + y * stride;
          if ((unsigned)iy >= (unsigned)H) {
            memset(col, 0, sizeof(float) * Wo);
            col += Wo;
            continue;
          }
          for (int x = 0; x < Wo; ++x) {
            const int ix = -pad + b + x * stride;
            *col++ = ((unsigned)ix < (unsigned)W) ? im[((int64_t)c * H + iy) * W + ix] : 0.0f;
          }
        }
}

/* ConvolutionLayer::Forward_cpu: per image im2col + group sgemms + bias sgemm.
 * col: scratch of C*k*k*Ho*Wo floats; ones: Ho*Wo ones (bias_multiplier_). */
void cc_conv_forward(const float* x, int N, int C, int H, int W, const float* w, const float* bias, int Cout,
                     int k, int pad, int stride, int group, float* y, float* col, const float* ones) {
  const int Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  const int og = Cout / group, kd = C / group * k * k, sp = Ho * Wo;
  for (int n = 0; n < N; ++n) {
    const float* xn = x + (int64_t)n * C * H * W;
    float* yn = y + (int64_t)n * Cout * sp;
    const float* cb = xn;
    if (!(k == 1 && pad == 0 && stride == 1)) {
      im2col(xn, C, H, W, k, pad, stride, col);
      cb = col;
    }
    for (int g = 0; g < group; ++g)
      gemm(0, 0, og, sp, kd, 1.0f, w + (int64_t)g * og * kd, cb + (int64_t)g * kd * sp, 0.0f,
           yn + (int64_t)g * og * sp);
    if (bias) gemm(0, 0, Cout, sp, 1, 1.0f, bias, ones, 1.0f, yn);
  }
}

/* InnerProductLayer::Forward_cpu: top = bottom * W^T + 1 * b^T */
void cc_ip_forward(const float* x, int M, int K, const float* w, const float* bias, int N, float* y,
                   const float* ones) {
  gemm(0, 1, M, N, K, 1.0f, x, w, 0.0f, y);
  if (bias) gemm(0, 0, M, N, 1, 1.0f, ones, bias, 1.0f, y);
}

void cc_relu(float* x, int64_t n) {
  for (int64_t i = 0; i < n; ++i) x[i] = x[i] > 0.0f ? x[i] : 0.0f;
}

/* CrossChannelForward_cpu; scale / padded: scratch of n*C*H*W and (C+size-1)*H*W floats */
void cc_lrn(const float* x, float* y, int num, int C, int H, int W, int size, float alpha, float beta, float k,
            float* scale, float* padded) {
  const int64_t hw = (int64_t)H * W, chw = C * hw;
  const int pre = (size - 1) / 2;
  const float aos = alpha / size;
  for (int64_t i = 0; i < num * chw; ++i) scale[i] = k;
  memset(padded, 0, sizeof(float) * (C + size - 1) * hw);
  for (int n = 0; n < num; ++n) {
    const float* xn = x + n * chw;
    float* sn = scale + n * chw;
    for (int64_t i = 0; i < chw; ++i) padded[pre * hw + i] = xn[i] * xn[i];
    for (int c = 0; c < size; ++c)
      for (int64_t i = 0; i < hw; ++i) sn[i] += aos * padded[c * hw + i];
    for (int c = 1; c < C; ++c) {
      float* s = sn + c * hw;
      memcpy(s, s - hw, sizeof(float) * hw);
      for (int64_t i = 0; i < hw; ++i) s[i] += aos * padded[(c + size - 1) * hw + i];
      for (int64_t i = 0; i < hw; ++i) s[i] += -aos * padded[(c - 1) * hw + i];
    }
  }
  for (int64_t i = 0; i < num * chw; ++i) y[i] = x[i] * powf(scale[i], -beta);
}

/* PoolingLayer::Forward_cpu, MAX (ceil output rule, pad 0) */
void cc_maxpool(const float* x, float* y, int* mask, int num, int C, int H, int W, int k, int stride) {
  const int PH = (int)ceilf((float)(H - k) / stride) + 1, PW = (int)ceilf((float)(W - k) / stride) + 1;
  for (int64_t nc = 0; nc < (int64_t)num * C; ++nc) {
    const float* xp = x + nc * H * W;
    float* yp = y + nc * PH * PW;
    int* mp = mask + nc * PH * PW;
    for (int ph = 0; ph < PH; ++ph)
      for (int pw = 0; pw < PW; ++pw) {
        const int hs = ph * stride, ws = pw * stride;
        const int he = hs + k < H ? hs + k : H, we = ws + k < W ? ws + k : W;
        float m = -FLT_MAX;
        int mi = -1;
        for (int h = hs; h < he; ++h)
          for (int w = ws; w < we; ++w)
            if (xp[h * W + w] > m) {
              m = xp[h * W + w];
              mi = h * W + w;
            }
        yp[ph * PW + pw] = m;
        mp[ph * PW + pw] = mi;
      }
  }
}

/* PoolingLayer::Forward_cpu with padding, MAX (method 0, pooling_layer.cpp:
 * 131-171: window clipped to the image, -FLT_MAX start, strict ">") or AVE
 * (method 1, :172-200: divisor = the window clipped to the padded image).
 * PH / PW from the caller (pool_out: ceil rule + the padded clip). */
void cc_pool(const float* x, float* y, int num, int C, int H, int W, int PH, int PW, int k, int stride, int pad,
             int method) {
  for (int64_t nc = 0; nc < (int64_t)num * C; ++nc) {
    const float* xp = x + nc * H * W;
    float* yp = y + nc * PH * PW;
    for (int ph = 0; ph < PH; ++ph)
      for (int pw = 0; pw < PW; ++pw) {
        int hs = ph * stride - pad, ws = pw * stride - pad;
        if (method == 0) {
          const int he = hs + k < H ? hs + k : H, we = ws + k < W ? ws + k : W;
          hs = hs > 0 ? hs : 0;
          ws = ws > 0 ? ws : 0;
          float m = -FLT_MAX;
          for (int h = hs; h < he; ++h)
            for (int w = ws; w < we; ++w)
              if (xp[h * W + w] > m) m = xp[h * W + w];
          yp[ph * PW + pw] = m;
        } else {
          int he = hs + k < H + pad ? hs + k : H + pad, we = ws + k < W + pad ? ws + k : W + pad;
          const int size = (he - hs) * (we - ws);
          hs = hs > 0 ? hs : 0;
          ws = ws > 0 ? ws : 0;
          he = he < H ? he : H;
          we = we < W ? we : W;
          float a = 0.0f;
          for (int h = hs; h < he; ++h)
            for (int w = ws; w < we; ++w) a += xp[h * W + w];
          yp[ph * PW + pw] = a / size;
        }
      }
  }
}

/* SoftmaxLayer::Forward_cpu over [outer, C] */
void cc_softmax(const float* x, float* y, int outer, int C) {
  for (int o = 0; o < outer; ++o) {
    const float* xo = x + (int64_t)o * C;
    float* yo = y + (int64_t)o * C;
    float m = xo[0];
    for (int c = 1; c < C; ++c) m = xo[c] > m ? xo[c] : m;
    float s = 0.0f;
    for (int c = 0; c < C; ++c) {
      yo[c] = expf(xo[c] - m);
      s += yo[c];
    }
    for (int c = 0; c < C; ++c) yo[c] /= s;
  }
}
