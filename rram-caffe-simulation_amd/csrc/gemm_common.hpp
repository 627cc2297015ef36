// Shared pieces of the fp32 GEMM / convolution kernels (gemm.hip) and the
// bf16x6 convolution kernels (x6.hip): operand views, convolution
// geometry, epilogue parameters, raw-buffer LDS-DMA helpers and the MFMA
// 32x32 accumulator epilogue.  Included into an anonymous namespace by each
// translation unit.
#pragma once
#include <stdint.h>

#include "rram_common.hpp"

namespace rram {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// K-tile depth is a template parameter KB (16 or 32); LDS rows are padded to
// KB + 4 floats (80 / 144 B: 16-B aligned, conflict-free ds_read_b128 for 16
// consecutive rows).  BK is the split-K chunk granularity (multiple of both).
constexpr int BK = 32;
template <int KB>
constexpr int ldk_of() { return KB + 4; }

// KCV = KC with 16-byte global loads (row stride, base and K all multiples of 4 floats)
// CONVT = CONV with a per-k offset/tap table (conv_table below) read by scalar
// loads: no (c, kh, kw) stepping and no multiplies in the gather.
// CONVT64: the same with a 64-bit tap mask (kh*kw <= 63, e.g. 7 x 7 with padding)
// KCU = KC with 16-byte raw buffer loads at any 4-byte alignment (row stride K
// not a multiple of 4, e.g. AlexNet conv1 K = 363): a float4 may run into the
// next row (or past the buffer end, where the per-dword range check returns
// 0); the elements at k >= K are zeroed when the tile is written to LDS.
// IM2T = the transposed column matrix of a convolution's weight gradient,
// gathered from the input (no im2col pass): row = reduction index (c, kh,
// kw) of the column matrix (row K = the folded bias gradient's ones row),
// k = output position (image, ho, wo); per-row {offset, kh*dh | kw*dw << 16}
// table (im2t_table), per-thread position decoded once per K-tile.
enum Mode : int { KC = 0, RC = 1, CONV = 2, NCHW = 3, NCHWT = 4, KCV = 5, CONVT = 6, CONVT64 = 7, KCU = 8, IM2T = 9 };
enum OutMode : int { OUT_ROWMAJOR = 0, OUT_NCHW = 1 };

// Fast unsigned division by a runtime constant (x < 2^31).
struct FastDiv {
  uint32_t d, m, s;
};
static FastDiv make_fastdiv(uint32_t d) {
  FastDiv f{d, 0, 0};
  if (d <= 1) {
    f.m = 0;
    f.s = 0;
    return f;
  }
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = static_cast<uint32_t>(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}
// d == 1 is encoded as m = 0, s = 0, so no branch is needed
__device__ __forceinline__ uint32_t fdiv(uint32_t x, const FastDiv& f) {
  const uint32_t t = __umulhi(x, f.m);
  return (t + x) >> f.s;
}

// Operand view: element (row, k).
struct View {
  const float* p;
  int64_t ld;        // KC: row stride; RC: k stride; NCHW(T): channel stride (= HW)
  int64_t img;       // NCHW/NCHWT/CONV: image stride
  int rows, kdim;    // logical extent
  FastDiv hw;        // NCHW/NCHWT: spatial size
};

struct ConvGeom {
  int C, H, W, KH, KW, ph, pw, sh, sw, dh, dw, Ho, Wo;
  FastDiv khkw, kw_div, howo, wo_div;
  int64_t chw;  // image stride of the input (C*H*W)
  int in_bytes; // bytes addressable from the group's input base (buffer range)
  const int2* tbl;  // CONVT: per k {4*(c*H*W + kh*dh*W + kw*dw), tap}; tap 31 = never valid
  int taps;         // CONVT: kh*kw taps tracked in the per-column validity mask (0: pad-free)
  int tpitch;       // octet kernels: positions per tile (0: the tile width; else whole output rows of
                    // an image, or whole images; the columns past it computed and dropped)
};

struct Epi {
  float* C;
  int64_t ldc;       // ROWMAJOR: row stride; NCHW: channel stride (= HW)
  int64_t cimg;      // NCHW: image stride (Cout*HW)
  FastDiv hw;        // NCHW: spatial size
  float alpha, beta;
  const float* bias;
  int bias_mode;
  int relu;
};

struct Params {
  View a, b;
  ConvGeom cv;
  Epi e;
  int M, N, K;
  int k_chunk;               // split-K chunk length (multiple of BK)
  float* ws;                 // split-K partials [split][M][N] (nullptr: direct)
  int64_t grp_a, grp_b, grp_c;  // per-group pointer offsets (z = group)
  int64_t grp_bias;
  int split;                 // number of K splits (z = split when > 1)
  int tiles_m, tiles_n, tiles_z;
};

// Per-thread constant data of the B loader for the CONV view.
struct ConvCol {
  int64_t base;  // image offset of this thread's column (n*C*H*W)
  int hb, wb;    // ho*sh - ph, wo*sw - pw
  bool valid;
  int pbase;     // n*C*H*W + hb*W + wb (element offset inside the group's input)
  __amdgpu_buffer_rsrc_t rsrc;  // raw buffer over the group's input (OOB loads return 0)
  uint32_t bad;     // CONVT: bit t set = tap t of this column reads padding (bit 31 always set)
  uint32_t bad_hi;  // CONVT64: taps 32..63 (bit 63 always set)
};

template <int ROWS, int KB>
struct Loader {
  static constexpr int EPT = ROWS * KB / 256;
  float v[EPT];
  int kn[EPT / 4 > 0 ? EPT / 4 : 1];  // KCU: valid elements of float4 i (K - k, may be <= 0 or >= 4)
  int2 rt[EPT];                       // IM2T: the table entries of this thread's rows (fixed per block)
};

// 16-byte zero block that guarded loads and bias selects read for out-of-range elements
__device__ __attribute__((aligned(16))) float g_zero4[4] = {0.f, 0.f, 0.f, 0.f};

__device__ __forceinline__ float pick(const float4& q, int s) {
  return (s & 3) == 0 ? q.x : (s & 3) == 1 ? q.y : (s & 3) == 2 ? q.z : q.w;
}

// Epilogue of one wave's MI x NI tiles of 32x32 (v_mfma_f32_32x32x2_f32
// accumulator layout): acc[i][j][r] -> row = mwave + 32 i + (r&3) + 8*(r>>2) + 4*lh,
// col = nwave + 32 j + lr.  Shared by k_gemm and k_gemm2.
template <int MI, int NI, int OM>
__device__ __forceinline__ void gemm_epilogue(floatx16 (&acc)[MI][NI], const Params& P, const Epi& ep, float* part,
                                              int mwave, int nwave, int lr, int lh) {
  // Every mode flag is block-uniform, so each loop below is free of
  // per-element waits: bias values are fetched with address selects (a select
  // on a loaded value makes the compiler branch around each load and wait for
  // it: one L2 round trip per output element), alpha and the row bias are
  // folded into the accumulators once per row, and only edge tiles mask rows.
  const int mw = mwave + 4 * lh;                       // this lane's first row
  const bool rows_full = mwave + MI * 32 <= P.M;
  if (part != nullptr) {                               // split-K partial slab [M][N]
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int n = nwave + j * 32 + lr;
      if (n >= P.N) continue;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mw + i * 32 + (r & 3) + 8 * (r >> 2);
          if (rows_full || m < P.M) part[(int64_t)m * P.N + n] = acc[i][j][r];
        }
    }
    return;
  }
  const bool row_bias = ep.bias_mode == RRAM_BIAS_ROW, col_bias = ep.bias_mode == RRAM_BIAS_COL;
  const bool relu = ep.relu != 0;
  const float alpha = ep.alpha, beta = ep.beta;
  if (beta == 0.0f) {
    // o = alpha*v + bias: one bias load per row, shared by the NI column tiles
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mw + i * 32 + (r & 3) + 8 * (r >> 2);
        const float b = *((row_bias && m < P.M) ? ep.bias + m : g_zero4);
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j][r] = alpha * acc[i][j][r] + b;
      }
  }
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int n = nwave + j * 32 + lr;
    if (n >= P.N) continue;
    const float cb = *(col_bias ? ep.bias + n : g_zero4);
    float* cj;
    if (OM == OUT_NCHW) {
      const uint32_t im = fdiv(static_cast<uint32_t>(n), ep.hw);
      const uint32_t sp = static_cast<uint32_t>(n) - im * ep.hw.d;
      cj = ep.C + (int64_t)im * ep.cimg + sp;
    } else {
      cj = ep.C + n;
    }
    const int64_t ld = ep.ldc;
    if (beta != 0.0f) {
      // accumulate into C (backward GEMMs): ((alpha*v) + beta*C) + bias
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mw + i * 32 + (r & 3) + 8 * (r >> 2);
          if (!rows_full && m >= P.M) continue;
          float* dst = cj + (int64_t)m * ld;
          float o = alpha * acc[i][j][r] + beta * *dst;
          o += *(row_bias ? ep.bias + m : g_zero4) + cb;
          *dst = relu ? fmaxf(o, 0.0f) : o;
        }
    } else if (rows_full) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mw + i * 32 + (r & 3) + 8 * (r >> 2);
          const float o = acc[i][j][r] + cb;
          cj[(int64_t)m * ld] = relu ? fmaxf(o, 0.0f) : o;
        }
    } else {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mw + i * 32 + (r & 3) + 8 * (r >> 2);
          const float o = acc[i][j][r] + cb;
          if (m < P.M) cj[(int64_t)m * ld] = relu ? fmaxf(o, 0.0f) : o;
        }
    }
  }
}

// Epilogue of the bf16x6 convolution kernels (beta = 0, no split-K, NCHW
// output): the same arithmetic as gemm_epilogue's beta = 0 path, stored with
// raw buffer stores whose row offsets are wave-uniform (scalar soffset: the
// lane's rows are mwave + 4 h + (r & 3) + 8 (r >> 2) + 32 i), so a store
// costs no per-element address arithmetic (the generic epilogue spent
// ~3000 VALU per wave on 64-bit addresses, exposed at one wave per SIMD).
// acc is left holding the stored values before the ReLU.  ep.C == nullptr:
// nothing stored (the 1x1 kernels' convolution-output fold: only the octet
// companion, from acc, is written).
template <int MI, int NI>
__device__ __forceinline__ void conv_epilogue_nchw(floatx16 (&acc)[MI][NI], const Params& P, const Epi& ep,
                                                   int mwave, int nwave, int lr, int lh, int nlim = 0x7FFFFFFF) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(ep.C, 0, 0x7FFFFFFF, 0x00020000);
  const int HWo = static_cast<int>(ep.hw.d);
  const int mw = mwave + 4 * lh;  // this lane's first row
  const bool rows_full = mwave + MI * 32 <= P.M;
  const bool row_bias = ep.bias_mode == RRAM_BIAS_ROW, col_bias = ep.bias_mode == RRAM_BIAS_COL;
  const bool relu = ep.relu != 0;
  const float alpha = ep.alpha;
  float bz[MI][16];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = mw + i * 32 + (r & 3) + 8 * (r >> 2);
      bz[i][r] = *((row_bias && m < P.M) ? ep.bias + m : g_zero4);
    }
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int n = nwave + j * 32 + lr;
    if (n >= P.N || n >= nlim) continue;  // nlim: a tile's last column + 1 (per-image tiles)
    const float cb = *(col_bias ? ep.bias + n : g_zero4);
    const uint32_t im = fdiv(static_cast<uint32_t>(n), ep.hw);
    const uint32_t sp = static_cast<uint32_t>(n) - im * ep.hw.d;
    const uint32_t base = static_cast<uint32_t>((im * ep.cimg + sp + static_cast<int64_t>(mw) * HWo) * 4);
    float ov[MI][16];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float o = (alpha * acc[i][j][r] + bz[i][r]) + cb;
        acc[i][j][r] = o;  // the stored value before the ReLU (k_conv_cb_x6's octet companion splits it)
        ov[i][r] = relu ? fmaxf(o, 0.0f) : o;
      }
    if (ep.C == nullptr) continue;
    if (rows_full) {  // uniform: no per-store exec masking
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, ov[i][r]), rs, static_cast<int>(base),
                                                (i * 32 + (r & 3) + 8 * (r >> 2)) * HWo * 4, 0);
    } else {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int dr = i * 32 + (r & 3) + 8 * (r >> 2);
          if (mw + dr < P.M)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, ov[i][r]), rs, static_cast<int>(base),
                                                  dr * HWo * 4, 0);
        }
    }
  }
}

Epi make_epi(float* C, int64_t ldc, float alpha, float beta, const float* bias, int bias_mode,
             int relu) {
  Epi e{};
  e.C = C;
  e.ldc = ldc;
  e.cimg = 0;
  e.hw = make_fastdiv(1);
  e.alpha = alpha;
  e.beta = beta;
  e.bias = bias;
  e.bias_mode = bias ? bias_mode : RRAM_BIAS_NONE;
  e.relu = relu;
  return e;
}

View make_view(const float* p, int64_t ld, int rows, int kdim) {
  View v{};
  v.p = p;
  v.ld = ld;
  v.img = 0;
  v.rows = rows;
  v.kdim = kdim;
  v.hw = make_fastdiv(1);
  return v;
}

// split-K reduction + epilogue (row-major C only)
// sum of the split-K partials of element idx in split order (s += p_0, p_1,
// ...): the loads of 8 partials are issued together, the adds stay
// sequential, so the result is the plain loop's bit for bit
__device__ __forceinline__ float splitk_sum(const float* __restrict__ ws, int split, int64_t total, int64_t idx) {
  float s = 0.0f;
  int z = 0;
  for (; z + 8 <= split; z += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ws[(int64_t)(z + u) * total + idx];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; z < split; ++z) s += ws[(int64_t)z * total + idx];
  return s;
}

__global__ void __launch_bounds__(256) k_splitk_reduce(const float* __restrict__ ws, int split, int M,
                                                       int N, Epi ep) {
  const int64_t total = (int64_t)M * N;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const float s = splitk_sum(ws, split, total, idx);
    const int m = static_cast<int>(idx / N);
    const int n = static_cast<int>(idx - (int64_t)m * N);
    float* dst = ep.C + (int64_t)m * ep.ldc + n;
    float o = ep.alpha * s;
    if (ep.beta != 0.0f) o += ep.beta * *dst;
    if (ep.bias_mode == RRAM_BIAS_ROW) o += ep.bias[m];
    else if (ep.bias_mode == RRAM_BIAS_COL) o += ep.bias[n];
    if (ep.relu) o = fmaxf(o, 0.0f);
    *dst = o;
  }
}

// k_splitk_reduce for an NCHW convolution output (column n = image * HW +
// position): partials summed in split order, then bias (per row) and ReLU as
// gemm_epilogue's beta = 0 path
__global__ void __launch_bounds__(256) k_splitk_reduce_nchw(const float* __restrict__ ws, int split, int M, int N,
                                                            Epi ep) {
  const int64_t total = (int64_t)M * N;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const float s = splitk_sum(ws, split, total, idx);
    const int m = static_cast<int>(idx / N);
    const uint32_t n = static_cast<uint32_t>(idx - (int64_t)m * N);
    const uint32_t im = fdiv(n, ep.hw), sp = n - im * ep.hw.d;
    const float o = ep.alpha * s + (ep.bias_mode == RRAM_BIAS_ROW ? ep.bias[m] : 0.0f);
    ep.C[(int64_t)im * ep.cimg + (int64_t)m * ep.ldc + sp] = ep.relu ? fmaxf(o, 0.0f) : o;
  }
}

// k_splitk_reduce of the weight gradient with the bias folded in (N = K + 1
// columns): column K goes to db, the rest to dw [M][K]; dst += sum in split
// order, as k_splitk_reduce's alpha = beta = 1 path
__global__ void __launch_bounds__(256) k_splitk_reduce_dwdb(const float* __restrict__ ws, int split, int M, int K,
                                                            float* __restrict__ dw, float* __restrict__ db) {
  const int N = K + 1;
  const int64_t total = (int64_t)M * N;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const float s = splitk_sum(ws, split, total, idx);
    const int m = static_cast<int>(idx / N);
    const int n = static_cast<int>(idx - (int64_t)m * N);
    float* dst = n < K ? dw + (int64_t)m * K + n : db + m;
    float o = 1.0f * s;
    o += 1.0f * *dst;
    *dst = o;
  }
}

// The weight-gradient split-K reduce for few outputs over many splits
// (CIFAR-10 conv1: 32 x 76 outputs, 256 partials each): one wave per output
// element, lane l summing partials l, l + 64, ... in order, then a fixed xor
// tree (deterministic; a different order than the sequential reduce's).
// dst += sum: dw [M][K] for n < K, db (nullable: K + 1 columns) for n == K.
__global__ void __launch_bounds__(256) k_splitk_reduce_wave(const float* __restrict__ ws, int split, int M, int K,
                                                            int ncols, float* __restrict__ dw,
                                                            float* __restrict__ db) {
  const int lane = threadIdx.x & 63;
  const int64_t total = (int64_t)M * ncols;
  const int64_t idx = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (idx >= total) return;
  float s = 0.0f;
  for (int z = lane; z < split; z += 64) s += ws[(int64_t)z * total + idx];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) {
    const int m = static_cast<int>(idx / ncols);
    const int n = static_cast<int>(idx - (int64_t)m * ncols);
    float* dst = n < K ? dw + (int64_t)m * K + n : db + m;
    float o = 1.0f * s;
    o += 1.0f * *dst;
    *dst = o;
  }
}

namespace g2 {
typedef int int4v __attribute__((ext_vector_type(4)));

// Raw buffer descriptor as four SGPR words (base, stride 0, byte range, raw
// untyped dword format): offsets at or past the range load zeros.
__device__ __forceinline__ int4v make_rsrc(const float* p, uint32_t range) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  int4v r;
  r.x = static_cast<int>(static_cast<uint32_t>(a));
  r.y = static_cast<int>(static_cast<uint32_t>(a >> 32) & 0xFFFFu);
  r.z = static_cast<int>(range);
  r.w = 0x00020000;
  return r;
}
// LDS-DMA loads (buffer_load ... lds) in inline asm: the compiler then neither
// drains the ring with vmcnt(0) before every ds_read (it cannot tell the DMA
// destination from the stage being read) nor demotes the uniform table loads
// to vector loads.  Their completion is tracked by hand (wait_vm + barrier).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma_b128(const int4v& rs, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs), "s"(lds)
               : "m0");
}
__device__ __forceinline__ void dma_b32(const int4v& rs, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dword %0, %1, 0 offen lds" ::"v"(voff), "s"(rs), "s"(lds)
               : "m0");
}
#pragma clang diagnostic pop

// wait until at most N of this wave's vector-memory operations (LDS-DMA
// included) are outstanding
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
}  // namespace g2

}  // namespace
}  // namespace rram
