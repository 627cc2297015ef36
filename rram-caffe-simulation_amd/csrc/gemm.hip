// fp32 GEMM and implicit-GEMM convolution on gfx950 MFMA
// (v_mfma_f32_32x32x2_f32: exact fp32, 64 FLOP/clk/SIMD).
//
// One templated kernel serves every contraction of the conv/IP path:
//   C[m][n] = sum_k A(m,k) * B(n,k)
// A and B are "operand views" (loader modes) so the same MFMA core runs
//   - Caffe GEMM with any transpose combination  (KC / KCV / RC views),
//   - implicit-im2col convolution forward         (CONV view: gather into LDS),
//   - NCHW activations / gradients spanning images (NCHW / NCHWT views).
// Block: 256 threads = 4 waves; each wave owns MI x NI tiles of 32x32.
// LDS holds both operands k-contiguous ([row][BK+4]), double-buffered and
// register-staged: the global loads of K-tile t+1 are issued before the MFMAs
// of tile t and written to the other LDS buffer after them (one barrier per
// K-tile).  Inside a tile K is consumed in a permuted order (lane half h at
// step s of sub-block q uses k = 16q + 8h + s) so each lane reads its
// fragments with 16-byte LDS reads; A and B use the same permutation, so the
// contraction is unchanged.  Blocks are remapped so that each XCD (own L2)
// receives a contiguous run of tiles that share operand panels.
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <array>
#include <map>
#include <tuple>
#include <mutex>
#include <type_traits>
#include <vector>

#include "gemm_common.hpp"

namespace rram {
namespace {


// Branch-free guarded loads: an out-of-range element loads from the view's
// base (always valid) and is replaced by 0, so the load stream has no
// exec-mask branches.
// The guard selects the ADDRESS (a 16-byte zero block for out-of-range
// elements), never the loaded value: a select on the value would force an
// s_waitcnt right after the load and serialise the prefetch behind it.
__device__ __forceinline__ float ld_guard(const float* p, int64_t off, bool ok) {
  return *(ok ? p + off : g_zero4);
}
__device__ __forceinline__ float ld_kc(const View& vw, int row, int k, bool kok) {
  const bool ok = kok && row < vw.rows;
  return ld_guard(vw.p, (int64_t)row * vw.ld + k, ok);
}
__device__ __forceinline__ float ld_rc(const View& vw, int row, int k, bool kok) {
  const bool ok = kok && row < vw.rows;
  return ld_guard(vw.p, (int64_t)k * vw.ld + row, ok);
}
// NCHW: row = channel, k = flattened (image, spatial)
__device__ __forceinline__ float ld_nchw(const View& vw, int row, int k, bool kok) {
  const bool ok = kok && row < vw.rows;
  const uint32_t im = fdiv(static_cast<uint32_t>(k), vw.hw);
  const uint32_t s = static_cast<uint32_t>(k) - im * vw.hw.d;
  return ld_guard(vw.p, (int64_t)im * vw.img + (int64_t)row * vw.ld + s, ok);
}
// NCHWT: row = flattened (image, spatial), k = channel
__device__ __forceinline__ float ld_nchwt(const View& vw, int row, int k, bool kok) {
  const bool ok = kok && row < vw.rows;
  const uint32_t im = fdiv(static_cast<uint32_t>(row), vw.hw);
  const uint32_t s = static_cast<uint32_t>(row) - im * vw.hw.d;
  return ld_guard(vw.p, (int64_t)im * vw.img + (int64_t)k * vw.ld + s, ok);
}

// Element e of a ROWS x BK tile -> (row, k) for a scalar view mode.  KC / NCHW
// are k-fastest (memory is contiguous along k); the others are row-fastest.
template <int MODE, int ROWS, int KB>
__device__ __forceinline__ void tile_coord(int e, int& row, int& k) {
  if (MODE == KC || MODE == NCHW || MODE == IM2T) {
    row = e / KB;
    k = e % KB;
  } else {
    row = e % ROWS;
    k = e / ROWS;
  }
}

// float4 q of a KCV tile -> (row, float4 column).  With 16-deep K-tiles a row
// is 4 float4 and LDK = 20 dwords, so 16 consecutive lanes on 4 consecutive
// rows span 80 dwords and wrap onto the same banks (2-way conflicts on every
// ds_write_b128 of the tile, measured as ~20 % of the LDS cycles of the KB = 16
// GEMMs).  Lanes are instead dealt to rows b, b+4, b+8, b+12 of a 16-row block
// (20 * 4 = 80 = 16 mod 64: disjoint bank quads); a wave still covers the same
// 16 rows, so the global loads touch the same cache lines.
template <int ROWS, int KB>
__device__ __forceinline__ void kcv_coord(int q, int& r, int& k4) {
  if (KB == 16 && ROWS % 16 == 0) {
    const int g = q >> 4;
    r = (g >> 2) * 16 + ((q >> 2) & 3) * 4 + (g & 3);
    k4 = q & 3;
  } else {
    r = q / (KB / 4);
    k4 = q % (KB / 4);
  }
}

template <int MODE, int ROWS, int KB>
__device__ __forceinline__ void load_tile(Loader<ROWS, KB>& L, const View& vw, const ConvGeom& cv,
                                          const ConvCol& col, int row0, int k0, int kend) {
  constexpr int EPT = Loader<ROWS, KB>::EPT;
  if (MODE == KCV) {
    // 16-byte loads: float4 q -> (row = q / (KB/4), k4 = q % (KB/4)); K-range
    // ends are multiples of 4 so a float4 is entirely in or out of range
#pragma unroll
    for (int i = 0; i < EPT / 4; ++i) {
      const int q = threadIdx.x + i * 256;
      int r, k4;
      kcv_coord<ROWS, KB>(q, r, k4);
      const int k = k0 + 4 * k4;
      const bool ok = row0 + r < vw.rows && k < kend;
      const float4 x = *reinterpret_cast<const float4*>(ok ? vw.p + (int64_t)(row0 + r) * vw.ld + k : g_zero4);
      L.v[4 * i] = x.x;
      L.v[4 * i + 1] = x.y;
      L.v[4 * i + 2] = x.z;
      L.v[4 * i + 3] = x.w;
    }
    return;
  }
  if (MODE == KCU) {
    // float4 q -> (row = q / (KB/4), k4 = q % (KB/4)) as KCV, but the row
    // stride is only 4-byte aligned: raw buffer loads over the operand
    // (uniform descriptor, exact byte range), rows past the view get an
    // all-ones offset (out of range: zeros)
    const uint32_t range = static_cast<uint32_t>(((int64_t)(vw.rows - 1) * vw.ld + vw.kdim) * 4);
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(vw.p), 0, static_cast<int>(range), 0x00020000);
#pragma unroll
    for (int i = 0; i < EPT / 4; ++i) {
      const int q = threadIdx.x + i * 256;
      const int r = q / (KB / 4);
      const int k = k0 + 4 * (q % (KB / 4));
      const bool ok = row0 + r < vw.rows;
      const uint32_t off = static_cast<uint32_t>(((int64_t)(row0 + r) * vw.ld + k) * 4) | (ok ? 0u : 0xFFFFFFFFu);
      // whole-vector bit cast: extracting the u32 lanes one by one made this
      // ROCm 7.2 clang shrink the load to one dword while still reading
      // four registers (observed on gfx950)
      const floatx4 x = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
      L.v[4 * i] = x.x;
      L.v[4 * i + 1] = x.y;
      L.v[4 * i + 2] = x.z;
      L.v[4 * i + 3] = x.w;
      L.kn[i] = kend - k;
    }
    return;
  }
  if (MODE == CONVT || MODE == CONVT64) {
    // implicit im2col from the table: thread = one output position x EPT
    // consecutive k; the k segment is wave-uniform, so each table entry is a
    // scalar load, and per element the VALU does one add, one bit extract
    // (0 or -1: this column's tap reads padding / k past K) and one or that
    // turns the offset into an out-of-range one (the buffer load returns 0).
    const int seg = threadIdx.x / ROWS;
    const int ks = __builtin_amdgcn_readfirstlane(k0 + seg * EPT);
    const int2* te = cv.tbl + ks;
    // descriptor rebuilt here from uniform values so it provably lives in SGPRs
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(vw.p), 0, cv.in_bytes, 0x00020000);
    const uint32_t pb4 = static_cast<uint32_t>(col.pbase) * 4u;
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int2 t = te[i];
      const uint32_t word = (MODE == CONVT64 && t.y >= 32) ? col.bad_hi : col.bad;
      const uint32_t bad = static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(word), t.y & 31, 1));
      L.v[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, (pb4 + static_cast<uint32_t>(t.x)) | bad, 0, 0));
    }
    return;
  }
  if constexpr (MODE == IM2T) {
    // the column matrix of the weight gradient, transposed and gathered: the
    // thread's position k0 + tid % KB is fixed for the tile (k-fastest tile
    // order, 256 % KB == 0), its rows step by 256 / KB.  Per element: one
    // table load (the row's input offset and kernel offsets), two bounds
    // compares, one add; an invalid element's offset is pushed out of the
    // buffer's range (the load returns 0).  The ones row (table y = -1) is
    // set to 1.0 in store_tile (after the MFMAs, where the loads are waited
    // for anyway), recorded in kn[0]'s bits.
    static_assert(256 % KB == 0 && EPT <= 32, "IM2T tile");
    const int p = k0 + static_cast<int>(threadIdx.x) % KB;
    const bool pv = p < kend;
    const uint32_t im = fdiv(static_cast<uint32_t>(p), cv.howo);
    const uint32_t sp = static_cast<uint32_t>(p) - im * cv.howo.d;
    const uint32_t ho = fdiv(sp, cv.wo_div);
    const int hb = static_cast<int>(ho) * cv.sh - cv.ph;
    const int wb = static_cast<int>(sp - ho * cv.wo_div.d) * cv.sw - cv.pw;
    const uint32_t pb4 = static_cast<uint32_t>((static_cast<int64_t>(im) * cv.chw + hb * cv.W + wb) * 4);
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(vw.p), 0, cv.in_bytes, 0x00020000);
    uint32_t ones = 0;
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int2 t = L.rt[i];  // (loaded once per block: the thread's rows do not move)
      const bool ok = pv && static_cast<unsigned>(hb + (t.y & 0xFFFF)) < static_cast<unsigned>(cv.H) &&
                      static_cast<unsigned>(wb + (t.y >> 16)) < static_cast<unsigned>(cv.W);
      L.v[i] = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, (pb4 + static_cast<uint32_t>(t.x)) | (ok ? 0u : 0xFFFFFFFFu), 0, 0));
      ones |= (pv && t.y == -1) ? (1u << i) : 0u;
    }
    L.kn[0] = static_cast<int>(ones);
    return;
  }
  if (MODE == CONV) {
    // implicit im2col: thread = one output position (row) x EPT consecutive k.
    // The k segment start is wave-uniform (ROWS >= 64), so (c, kh, kw) is
    // decomposed once per tile on the scalar unit and stepped incrementally;
    // per element the VALU does two bounds compares and one offset add, and
    // the load is a raw buffer load whose out-of-range offset returns 0.
    const int seg = threadIdx.x / ROWS;
    const int ks = __builtin_amdgcn_readfirstlane(k0 + seg * EPT);
    uint32_t c = fdiv(static_cast<uint32_t>(ks), cv.khkw);
    const uint32_t rem = static_cast<uint32_t>(ks) - c * cv.khkw.d;
    uint32_t kh = fdiv(rem, cv.kw_div);
    uint32_t kw = rem - kh * cv.kw_div.d;
    const int HW = cv.H * cv.W;
    const uint32_t KW = cv.kw_div.d, KH = cv.khkw.d / (KW ? KW : 1u);
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int khd = static_cast<int>(kh) * cv.dh, kwd = static_cast<int>(kw) * cv.dw;
      const bool ok = col.valid && (ks + i) < kend &&
                      static_cast<unsigned>(col.hb + khd) < static_cast<unsigned>(cv.H) &&
                      static_cast<unsigned>(col.wb + kwd) < static_cast<unsigned>(cv.W);
      const int soff = static_cast<int>(c) * HW + khd * cv.W + kwd;  // wave-uniform
      // offset computed unconditionally and OR-ed with an all-ones mask when
      // out of range: a select, never an exec-mask branch, so the loads stay
      // in one basic block with the MFMAs they are interleaved with
      const uint32_t boff = (static_cast<uint32_t>(col.pbase + soff) * 4u) | (ok ? 0u : 0xFFFFFFFFu);
      L.v[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(col.rsrc, boff, 0, 0));
      // step (c, kh, kw) by one k, branch-free (scalar selects)
      kw += 1u;
      const uint32_t cw = kw == KW;
      kw = cw ? 0u : kw;
      kh += cw;
      const uint32_t ch = kh == KH;
      kh = ch ? 0u : kh;
      c += ch;
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int e = threadIdx.x + i * 256;
    int r, kk;
    tile_coord<MODE, ROWS, KB>(e, r, kk);
    const int row = row0 + r;
    const int k = k0 + kk;
    float x;
    if (MODE == KC) {
      x = ld_kc(vw, row, k, k < kend);
    } else if (MODE == RC) {
      x = ld_rc(vw, row, k, k < kend);
    } else if (MODE == NCHW) {
      x = ld_nchw(vw, row, k, k < kend);
    } else {
      x = ld_nchwt(vw, row, k, k < kend);
    }
    L.v[i] = x;
  }
}

// global load instructions one thread issues per K-tile
template <int MODE, int ROWS, int KB>
constexpr int vmem_per_tile() {
  return (MODE == KCV || MODE == KCU) ? Loader<ROWS, KB>::EPT / 4 : Loader<ROWS, KB>::EPT;
}

template <int MODE, int ROWS, int KB>
__device__ __forceinline__ void store_tile(const Loader<ROWS, KB>& L, float* lds) {
  constexpr int EPT = Loader<ROWS, KB>::EPT;
  constexpr int LDK = ldk_of<KB>();
  if (MODE == CONV || MODE == CONVT || MODE == CONVT64) {
    // EPT consecutive k of one row: 16-byte LDS writes (row stride 36 dwords
    // puts the 8 lanes of a ds_write_b128 group on distinct bank quads)
    float* dst = lds + (threadIdx.x % ROWS) * LDK + (threadIdx.x / ROWS) * EPT;
#pragma unroll
    for (int i = 0; i < EPT / 4; ++i)
      *reinterpret_cast<float4*>(dst + 4 * i) = make_float4(L.v[4 * i], L.v[4 * i + 1], L.v[4 * i + 2], L.v[4 * i + 3]);
    return;
  }
  if (MODE == KCU) {
    // the K tail (and the next row's elements a float4 ran into) become 0;
    // selected here, after the MFMAs, so the loads are not waited on early
#pragma unroll
    for (int i = 0; i < EPT / 4; ++i) {
      const int q = threadIdx.x + i * 256;
      const int n = L.kn[i];
      *reinterpret_cast<float4*>(lds + (q / (KB / 4)) * LDK + 4 * (q % (KB / 4))) =
          make_float4(n > 0 ? L.v[4 * i] : 0.0f, n > 1 ? L.v[4 * i + 1] : 0.0f, n > 2 ? L.v[4 * i + 2] : 0.0f,
                      n > 3 ? L.v[4 * i + 3] : 0.0f);
    }
    return;
  }
  if (MODE == KCV) {
#pragma unroll
    for (int i = 0; i < EPT / 4; ++i) {
      const int q = threadIdx.x + i * 256;
      int r, k4;
      kcv_coord<ROWS, KB>(q, r, k4);
      *reinterpret_cast<float4*>(lds + r * LDK + 4 * k4) =
          make_float4(L.v[4 * i], L.v[4 * i + 1], L.v[4 * i + 2], L.v[4 * i + 3]);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int e = threadIdx.x + i * 256;
    int r, kk;
    tile_coord<MODE, ROWS, KB>(e, r, kk);
    lds[r * LDK + kk] = (MODE == IM2T && ((static_cast<uint32_t>(L.kn[0]) >> i) & 1u)) ? 1.0f : L.v[i];
  }
}


// Occupancy target 4 waves per SIMD: the 128 x 128 / KB = 16 conv tile then
// keeps its accumulators in VGPRs (116 VGPRs, no AGPRs, no spills) instead of
// 80 VGPRs + 64 AGPRs at 3 waves; 4 blocks x 40 KB fill the 160 KB LDS.
// Measured on MI355X (scripts/gpu_variants.sh): AlexNet b256 GEMMs 3.760 ->
// 3.667 ms.  RRAM_V_WPE_OFF builds the compiler's own choice for A/B runs.
#ifndef RRAM_V_WPE_OFF
// wave tiles of more than 4 accumulators (MI * NI > 4) need > 128 VGPRs: they
// target 2 waves per SIMD instead of spilling
#define RRAM_GEMM_OCC __attribute__((amdgpu_waves_per_eu(MI * NI > 4 ? 2 : 4)))
#else
#define RRAM_GEMM_OCC
#endif
template <int WM, int WN, int MI, int NI, int AM, int BMODE, int OM, int KB>
__global__ void __launch_bounds__(256) RRAM_GEMM_OCC k_gemm(Params P) {
  constexpr int BMr = WM * MI * 32;
  constexpr int BNr = WN * NI * 32;
  constexpr int LDK = ldk_of<KB>();
  static_assert(WM * WN == 4, "4 waves per block");
  static_assert(KB == 16 || KB == 32, "K-tile depth");
  static_assert(BMr * KB % 1024 == 0 && BNr * KB % 1024 == 0, "tile/threads");
  // Table-gather convolutions with 32-deep K-tiles (AlexNet conv1, the CIFAR /
  // LeNet convolutions) use ONE LDS buffer: two barriers per K-tile, but half
  // the LDS, so 4 blocks per CU instead of 2 hide the strided gather's latency
  // (MI355X: conv1 0.720 -> 0.672 ms).  The IP GEMMs measured slower that way
  // (VGPR spills at 4 waves) and the 16-deep tiles already fit 4 blocks.
  // RRAM_V_DOUBLE keeps every kernel double-buffered for A/B runs.
#ifndef RRAM_V_DOUBLE
  constexpr int NBUF = (KB == 32 && (BMODE == CONVT || BMODE == CONVT64)) ? 1 : 2;
#else
  constexpr int NBUF = 2;
#endif
  __shared__ __attribute__((aligned(16))) float As[NBUF][BMr * LDK];
  __shared__ __attribute__((aligned(16))) float Bs[NBUF][BNr * LDK];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave / WN;
  const int wn = wave % WN;

  // XCD-aware tile order (cdna_hip_programming.md §5.5 T1, bijective form):
  // dispatch deals blocks round-robin over 8 XCDs, so give every XCD a
  // contiguous range of tiles; within it the m-tiles of one n-tile are
  // adjacent (they share the B panel) and consecutive n-tiles follow.
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, loc = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int tid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  // integer division by a runtime divisor is expanded on the VALU; pin the
  // (block-uniform) results to SGPRs so the operand pointers and the buffer
  // descriptor derived from them stay scalar
  const int tm = __builtin_amdgcn_readfirstlane(tid % P.tiles_m);
  const int tn = __builtin_amdgcn_readfirstlane((tid / P.tiles_m) % P.tiles_n);
  const int z = __builtin_amdgcn_readfirstlane(tid / (P.tiles_m * P.tiles_n));
  const int n0 = tn * BNr;
  const int m0 = tm * BMr;

  View va = P.a, vb = P.b;
  Epi ep = P.e;
  int kbeg = 0, kend = P.K;
  float* part = nullptr;
  if (P.split > 1) {
    kbeg = z * P.k_chunk;
    kend = min(P.K, kbeg + P.k_chunk);
    part = P.ws + (int64_t)z * P.M * P.N;
  } else if (z > 0) {  // conv group
    va.p += z * P.grp_a;
    vb.p += z * P.grp_b;
    ep.C += z * P.grp_c;
    if (ep.bias) ep.bias += z * P.grp_bias;
  }

  // CONV column precompute (B operand rows = output positions; fixed per thread)
  ConvCol col{0, 0, 0, false};
  if (BMODE == CONV || BMODE == CONVT || BMODE == CONVT64) {
    int r, kk;
    tile_coord<CONV, BNr, KB>(threadIdx.x, r, kk);
    const int p = n0 + r;
    if (p < P.N) {
      const uint32_t im = fdiv(static_cast<uint32_t>(p), P.cv.howo);
      const uint32_t s = static_cast<uint32_t>(p) - im * P.cv.howo.d;
      const uint32_t ho = fdiv(s, P.cv.wo_div);
      const uint32_t wo = s - ho * P.cv.wo_div.d;
      col.base = (int64_t)im * P.cv.chw;
      col.hb = static_cast<int>(ho) * P.cv.sh - P.cv.ph;
      col.wb = static_cast<int>(wo) * P.cv.sw - P.cv.pw;
      col.valid = true;
      col.pbase = static_cast<int>(col.base) + col.hb * P.cv.W + col.wb;
    }
    if (BMODE == CONVT || BMODE == CONVT64) {
      // validity of every kernel tap for this column, once per block
      uint64_t good = 0;
      if (P.cv.taps == 0) {
        good = col.valid ? 1u : 0u;  // pad-free: every tap is inside the image
      } else if (col.valid) {
        for (int t = 0; t < P.cv.taps; ++t) {
          const int kh = t / P.cv.KW, kw = t - kh * P.cv.KW;
          good |= static_cast<uint64_t>(static_cast<unsigned>(col.hb + kh * P.cv.dh) < static_cast<unsigned>(P.cv.H) &&
                                        static_cast<unsigned>(col.wb + kw * P.cv.dw) < static_cast<unsigned>(P.cv.W))
                  << t;
        }
      }
      if (BMODE == CONVT) {
        col.bad = ~static_cast<uint32_t>(good) | 0x80000000u;
      } else {
        col.bad = ~static_cast<uint32_t>(good);
        col.bad_hi = ~static_cast<uint32_t>(good >> 32) | 0x80000000u;
      }
    }
    // group base pointer, range = the whole remaining input (host checks < 2^32 bytes)
    col.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(vb.p), 0, P.cv.in_bytes, 0x00020000);
  }

#ifdef RRAM_V_MFMA16
  // v_mfma_f32_16x16x4_f32 variant: the wave tile as (2 MI) x (2 NI) 16x16 tiles
  floatx4 acc[2 * MI][2 * NI];
#pragma unroll
  for (int i = 0; i < 2 * MI; ++i)
#pragma unroll
    for (int j = 0; j < 2 * NI; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.0f;
  const int l16 = threadIdx.x & 15, g16 = (threadIdx.x & 63) >> 4;
#else
  floatx16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
#endif

  Loader<BMr, KB> la;
  Loader<BNr, KB> lb;
  if constexpr (BMODE == IM2T) {
#pragma unroll
    for (int i = 0; i < Loader<BNr, KB>::EPT; ++i)
      lb.rt[i] = P.cv.tbl[n0 + static_cast<int>(threadIdx.x) / KB + i * (256 / KB)];
  }
  const int ntiles = (kend - kbeg + KB - 1) / KB;
  if (ntiles > 0) {
    load_tile<AM, BMr, KB>(la, va, P.cv, col, m0, kbeg, kend);
    load_tile<BMODE, BNr, KB>(lb, vb, P.cv, col, n0, kbeg, kend);
    store_tile<AM, BMr, KB>(la, As[0]);
    store_tile<BMODE, BNr, KB>(lb, Bs[0]);
  }
  __syncthreads();

#ifndef RRAM_V_MFMA16
  const int lr = lane & 31;
  const int lh = lane >> 5;
#else
  (void)lane;  // measured 6 % slower than the 32x32x2 form on AlexNet b256 (scripts/gpu_variants.sh)
#endif
  for (int t = 0; t < ntiles; ++t) {
    const int cur = NBUF == 2 ? (t & 1) : 0;
    const bool more = (t + 1) < ntiles;
#ifdef RRAM_V_PRIO
    __builtin_amdgcn_s_setprio(1);
#endif
    {
      // unconditional (no basic-block split): past the last tile every
      // element is out of range and the guarded loads return zeros
      const int kn = kbeg + (t + 1) * KB;
      load_tile<AM, BMr, KB>(la, va, P.cv, col, m0, kn, kend);
      load_tile<BMODE, BNr, KB>(lb, vb, P.cv, col, n0, kn, kend);
    }
#ifdef RRAM_V_MFMA16
    // lane group g at step s of sub-block q uses k = 16q + 4g + s (A and B alike)
#pragma unroll
    for (int q = 0; q < KB / 16; ++q) {
      float4 af[2 * MI], bf[2 * NI];
#pragma unroll
      for (int i = 0; i < 2 * MI; ++i)
        af[i] = *reinterpret_cast<const float4*>(&As[cur][(wm * MI * 32 + i * 16 + l16) * LDK + q * 16 + g16 * 4]);
#pragma unroll
      for (int j = 0; j < 2 * NI; ++j)
        bf[j] = *reinterpret_cast<const float4*>(&Bs[cur][(wn * NI * 32 + j * 16 + l16) * LDK + q * 16 + g16 * 4]);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int i = 0; i < 2 * MI; ++i)
#pragma unroll
          for (int j = 0; j < 2 * NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(pick(af[i], s4), pick(bf[j], s4), acc[i][j], 0, 0, 0);
    }
#else
#pragma unroll
    for (int q = 0; q < KB / 16; ++q) {
      float4 af[MI][2], bf[NI][2];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const float* pa = &As[cur][(wm * MI * 32 + i * 32 + lr) * LDK + q * 16 + lh * 8];
        af[i][0] = *reinterpret_cast<const float4*>(pa);
        af[i][1] = *reinterpret_cast<const float4*>(pa + 4);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const float* pb = &Bs[cur][(wn * NI * 32 + j * 32 + lr) * LDK + q * 16 + lh * 8];
        bf[j][0] = *reinterpret_cast<const float4*>(pb);
        bf[j][1] = *reinterpret_cast<const float4*>(pb + 4);
      }
#pragma unroll
      for (int s = 0; s < 8; ++s) {
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const float a = pick(af[i][s >> 2], s);
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, pick(bf[j][s >> 2], s), acc[i][j], 0, 0, 0);
        }
      }
    }
#endif
    // Interleave the next tile's global loads with the first MFMAs (a wave
    // issues VALU / VMEM while its MFMAs run): one load, then NMF MFMAs.
#ifndef RRAM_V_NOSCHED
    {
      constexpr int NVM = vmem_per_tile<AM, BMr, KB>() + vmem_per_tile<BMODE, BNr, KB>();
      constexpr int NMF_TOT = MI * NI * KB / 2;
#ifdef RRAM_V_SPREAD
      constexpr int NMF = NMF_TOT / NVM > 0 ? NMF_TOT / NVM : 1;
#else
      constexpr int NMF = NMF_TOT / (2 * NVM) > 0 ? NMF_TOT / (2 * NVM) : 1;
#endif
#pragma unroll
      for (int v = 0; v < NVM; ++v) {
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);    // VMEM read
        __builtin_amdgcn_sched_group_barrier(0x008, NMF, 0);  // MFMA
      }
    }
#endif
    // the LDS writes of the staged tile stay behind every MFMA
    __builtin_amdgcn_sched_barrier(0);
#ifdef RRAM_V_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    if (NBUF == 1) __syncthreads();  // every wave is done reading the single buffer
    if (more) {
      store_tile<AM, BMr, KB>(la, As[NBUF == 2 ? cur ^ 1 : 0]);
      store_tile<BMODE, BNr, KB>(lb, Bs[NBUF == 2 ? cur ^ 1 : 0]);
    }
    __syncthreads();
  }

#ifdef RRAM_V_MFMA16
  // epilogue: acc[i][j][r] -> row = 16 i + 4 g + r, col = 16 j + l16
#pragma unroll
  for (int j = 0; j < 2 * NI; ++j) {
    const int n = n0 + wn * NI * 32 + j * 16 + l16;
    if (n >= P.N) continue;
    int64_t cbase = 0;
    if (OM == OUT_NCHW && part == nullptr) {
      const uint32_t im = fdiv(static_cast<uint32_t>(n), ep.hw);
      const uint32_t s = static_cast<uint32_t>(n) - im * ep.hw.d;
      cbase = (int64_t)im * ep.cimg + s;
    }
#pragma unroll
    for (int i = 0; i < 2 * MI; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * MI * 32 + i * 16 + 4 * g16 + r;
        if (m >= P.M) continue;
        const float v = acc[i][j][r];
        if (part != nullptr) {
          part[(int64_t)m * P.N + n] = v;
          continue;
        }
        float* dst = (OM == OUT_NCHW) ? (ep.C + cbase + (int64_t)m * ep.ldc)
                                      : (ep.C + (int64_t)m * ep.ldc + n);
        float o = ep.alpha * v;
        if (ep.beta != 0.0f) o += ep.beta * *dst;
        if (ep.bias_mode == RRAM_BIAS_ROW) o += ep.bias[m];
        else if (ep.bias_mode == RRAM_BIAS_COL) o += ep.bias[n];
        if (ep.relu) o = fmaxf(o, 0.0f);
        *dst = o;
      }
    }
  }
#else
  gemm_epilogue<MI, NI, OM>(acc, P, ep, part, m0 + wm * MI * 32, n0 + wn * NI * 32, lr, lh);
#endif
}

// ---------------------------------------------------------------------------
// k_gemm2: the same contraction at one 128 x 128 tile per 4-wave workgroup and
// ONE wave per SIMD (3-stage LDS ring, ~97 KB: one workgroup per CU), for the
// 16-byte operands (A = KCV; B = KCV or the CONVT gather).  What it changes
// against k_gemm (hipBLASLt's fp32 kernels run the same regime: 1 WG/CU,
// 128x128, K-tiles of 64, pipelined loads; 128-133 TFLOP/s on this box):
//   * 32-deep K-tiles loaded as whole 128-byte row pieces (k_gemm's 16-deep
//     tiles fetch every row line in two halves, in two K-tiles);
//   * LDS-DMA (buffer_load ... lds): no staging VGPRs, no ds_write pass; an
//     out-of-range offset (rows past M/N, k past the chunk, padding taps) lands
//     zeros;
//   * tiles are issued NST-1 ahead and only the oldest is waited for (counted
//     vmcnt + raw s_barrier: __syncthreads() would drain the ring);
//   * one barrier per K-tile, in the middle of it: the fragments of the next
//     tile's first half are read while the second half's MFMAs run.
// Stage images (one __shared__ array):
//   A      [128 rows][32 k], 16-byte quad q of row r at quad position q ^ ((r>>1)&7)
//          (conflict-free ds_read_b128 for 16 consecutive rows; the swizzle is
//          applied on the global source address, the DMA destination stays
//          lane-linear);
//   B KCV  the same image;
//   B CONVT [32 k][130]: column n at n, rows padded so the two lane halves
//          (k and k + 16) read disjoint bank halves with ds_read_b32.
// K order inside a tile: lane half h at step s uses k = 16 h + s (A and B).
namespace g2 {
constexpr int BM = 128, BN = 128, KT = 32, LDN = 130;
constexpr int A_FL = BM * KT;
template <int BMODE>
constexpr int b_fl() { return BMODE == CONVT ? KT * LDN : BN * KT; }
template <int BMODE>
constexpr int stage_fl() { return A_FL + b_fl<BMODE>(); }
// LDS-DMA instructions one wave issues per K-tile: A 4 pieces of 1 KB; B 4 more
// (KCV) or 16 gathered rows of 64 columns x 4 B (CONVT)
template <int BMODE>
constexpr int vm_per_tile() { return 4 + (BMODE == CONVT ? 16 : 4); }


// Loader of a K-contiguous operand (rows x k): this lane's byte offset of row
// r = 32 w + 8 i + (lane >> 3) for piece i (bit 31 set when the row is out of
// range) and the k offset (floats) of the quad it fetches.
struct RowLd {
  int4v rsrc;
  uint32_t rb[4];
  int kq[4];
};
__device__ __forceinline__ RowLd make_rowld(const View& vw, int row0, int wave, int lane) {
  RowLd L;
  L.rsrc = make_rsrc(vw.p, static_cast<uint32_t>(((int64_t)(vw.rows - 1) * vw.ld + vw.kdim) * 4));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 32 * wave + 8 * i + (lane >> 3);
    const int q = (lane & 7) ^ ((r >> 1) & 7);
    const bool ok = row0 + r < vw.rows;
    L.rb[i] = ok ? static_cast<uint32_t>((int64_t)(row0 + r) * vw.ld * 4) : 0x80000000u;
    L.kq[i] = 4 * q;
  }
  return L;
}
// piece i of the tile at k0 into the image at LDS byte address img
__device__ __forceinline__ void issue_row_piece(const RowLd& L, uint32_t img, int wave, int i, int k0, int kend) {
  const int k = k0 + L.kq[i];
  const uint32_t off = (L.rb[i] + static_cast<uint32_t>(k) * 4u) | (k < kend ? 0u : 0x80000000u);
  dma_b128(L.rsrc, off, img + static_cast<uint32_t>((32 * wave + 8 * i) * KT * 4));
}

// Gather loader (CONVT): this lane's two columns n0 + 64 h + lane.
struct ColLd {
  int4v rsrc;
  uint32_t pb4[2];  // byte offset of the column's (image, ho*sh - ph, wo*sw - pw) input corner
  uint32_t bad[2];  // bit t: tap t reads padding (bit 31 always set; all set past N)
};
__device__ __forceinline__ ColLd make_colld(const Params& P, const float* base, int n0, int lane) {
  ColLd C;
  C.rsrc = make_rsrc(base, static_cast<uint32_t>(P.cv.in_bytes));
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int p = n0 + 64 * h + lane;
    C.pb4[h] = 0;
    C.bad[h] = 0xFFFFFFFFu;
    if (p < P.N) {
      const uint32_t im = fdiv(static_cast<uint32_t>(p), P.cv.howo);
      const uint32_t sp = static_cast<uint32_t>(p) - im * P.cv.howo.d;
      const uint32_t ho = fdiv(sp, P.cv.wo_div);
      const uint32_t wo = sp - ho * P.cv.wo_div.d;
      const int hb = static_cast<int>(ho) * P.cv.sh - P.cv.ph;
      const int wb = static_cast<int>(wo) * P.cv.sw - P.cv.pw;
      C.pb4[h] = static_cast<uint32_t>(static_cast<int>(im * P.cv.chw) + hb * P.cv.W + wb) * 4u;
      uint32_t good = 1u;  // pad-free: every tap is inside the image
      if (P.cv.taps > 0) {
        good = 0;
        for (int t = 0; t < P.cv.taps; ++t) {
          const int kh = t / P.cv.KW, kw = t - kh * P.cv.KW;
          good |= static_cast<uint32_t>(static_cast<unsigned>(hb + kh * P.cv.dh) < static_cast<unsigned>(P.cv.H) &&
                                        static_cast<unsigned>(wb + kw * P.cv.dw) < static_cast<unsigned>(P.cv.W))
                  << t;
        }
      }
      C.bad[h] = ~good | 0x80000000u;
    }
  }
  return C;
}
// k-row 8 w + kk of the tile, 64-column half h (table entry t, wave-uniform)
__device__ __forceinline__ void issue_col_row(const ColLd& C, int2 t, uint32_t img, int wave, int kk, int h) {
  const uint32_t bad = static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(C.bad[h]), t.y & 31, 1));
  dma_b32(C.rsrc, (C.pb4[h] + static_cast<uint32_t>(t.x)) | bad,
          img + static_cast<uint32_t>(((8 * wave + kk) * LDN + 64 * h) * 4));
}

// the wave's 8 gather-table entries of a K-tile, as one scalar load into
// SGPRs (inline asm: the memory-clobbering waits below would otherwise turn
// the uniform loads into vector loads); completed by the next lgkmcnt(0)
typedef int int16v __attribute__((ext_vector_type(16)));
__device__ __forceinline__ int16v sload_table(const int2* p) {
  int16v r;
  asm volatile("s_load_dwordx16 %0, %1, 0x0" : "=s"(r) : "s"(p));
  return r;
}
__device__ __forceinline__ int2 tentry(const int16v& v, int kk) {
  return make_int2(v[2 * kk], v[2 * kk + 1]);
}


// fragments of one K-half (8 k-steps) of a wave's 64 x 64 tile
template <int BMODE>
struct Frag {
  float4 a[2][2];
  float4 b[2][2];   // KCV
  float bc[2][8];   // CONVT
};
// fragment read item e of a K-half: A quads (4), then B quads (4, KCV) or
// B k-rows (16, CONVT, two per step)
template <int BMODE>
constexpr int frag_items() { return BMODE == CONVT ? 20 : 8; }
template <int BMODE>
__device__ __forceinline__ void read_item(Frag<BMODE>& F, const float* As, const float* Bs, int wm, int wn, int lr,
                                          int lh, int hf, int e) {
  if (e < 4) {
    const int i = e >> 1, u = e & 1;
    const int m = wm * 64 + i * 32 + lr;
    F.a[i][u] = *reinterpret_cast<const float4*>(As + m * KT + (((4 * lh + 2 * hf + u) ^ ((m >> 1) & 7)) << 2));
  } else if constexpr (BMODE == CONVT) {
    const int j = (e - 4) >> 3, sx = (e - 4) & 7;
    F.bc[j][sx] = Bs[(16 * lh + 8 * hf + sx) * LDN + wn * 64 + j * 32 + lr];
  } else {
    const int j = (e - 4) >> 1, u = (e - 4) & 1;
    const int n = wn * 64 + j * 32 + lr;
    F.b[j][u] = *reinterpret_cast<const float4*>(Bs + n * KT + (((4 * lh + 2 * hf + u) ^ ((n >> 1) & 7)) << 2));
  }
}
// MFMA pair p (0..15) of a K-half: step p >> 1, row tile p & 1, both column tiles
template <int BMODE>
__device__ __forceinline__ void mfma_pair(floatx16 (&acc)[2][2], const Frag<BMODE>& F, int p) {
  const int sx = p >> 1, i = p & 1;
  const float a = pick(F.a[i][sx >> 2], sx);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float b = BMODE == CONVT ? F.bc[j][sx] : pick(F.b[j][sx >> 2], sx);
    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i][j], 0, 0, 0);
  }
}
}  // namespace g2

template <int AM, int BMODE, int OM, int NST>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) k_gemm2(Params P) {
  using namespace g2;
  static_assert(AM == KCV && (BMODE == KCV || BMODE == CONVT), "k_gemm2 operand modes");
  static_assert(NST == 2 || NST == 3, "stages");
  constexpr int SF = stage_fl<BMODE>();
  constexpr int NVM = vm_per_tile<BMODE>();
  constexpr int NFR = frag_items<BMODE>();
  __shared__ __attribute__((aligned(16))) float smem[NST * SF];
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)smem));

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = lane & 31, lh = lane >> 5;

  // XCD-aware tile order, as k_gemm
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, loc = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int tid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int tm = __builtin_amdgcn_readfirstlane(tid % P.tiles_m);
  const int tn = __builtin_amdgcn_readfirstlane((tid / P.tiles_m) % P.tiles_n);
  const int z = __builtin_amdgcn_readfirstlane(tid / (P.tiles_m * P.tiles_n));
  const int n0 = tn * BN;
  const int m0 = tm * BM;

  View va = P.a, vb = P.b;
  Epi ep = P.e;
  int kbeg = 0, kend = P.K;
  float* part = nullptr;
  if (P.split > 1) {
    kbeg = z * P.k_chunk;
    kend = min(P.K, kbeg + P.k_chunk);
    part = P.ws + (int64_t)z * P.M * P.N;
  } else if (z > 0) {  // conv group
    va.p += z * P.grp_a;
    vb.p += z * P.grp_b;
    ep.C += z * P.grp_c;
    if (ep.bias) ep.bias += z * P.grp_bias;
  }

  const RowLd la = make_rowld(va, m0, wave, lane);
  RowLd lb;
  ColLd lc;
  if constexpr (BMODE == CONVT) lc = make_colld(P, vb.p, n0, lane);
  else lb = make_rowld(vb, n0, wave, lane);

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  const int nt = (kend - kbeg + KT - 1) / KT;
  // load item e (0 .. NVM-1) of K-tile at k0 into the stage at LDS address img;
  // te: the tile's gather-table entries for k-rows 8 w .. 8 w + 7 (SGPRs)
  auto item = [&](int e, uint32_t img, int k0, const int16v& te) {
    if (e < 4) {
      issue_row_piece(la, img, wave, e, k0, kend);
    } else if constexpr (BMODE == CONVT) {
      issue_col_row(lc, tentry(te, (e - 4) >> 1), img + A_FL * 4, wave, (e - 4) >> 1, (e - 4) & 1);
    } else {
      issue_row_piece(lb, img + A_FL * 4, wave, e - 4, k0, kend);
    }
  };
  auto table = [&](int k0) {
    int16v v{};
    if constexpr (BMODE == CONVT) v = sload_table(P.cv.tbl + k0 + 8 * wave);
    return v;
  };

  Frag<BMODE> f1, f2;
  int16v tnext{};  // table entries of the tile the next phase A issues
  if (nt > 0) {
    {
      const int16v te = table(kbeg);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int e = 0; e < NVM; ++e) item(e, lds0, kbeg, te);
    }
    if (NST == 3 && nt > 1) {
      const int16v te = table(kbeg + KT);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int e = 0; e < NVM; ++e) item(e, lds0 + SF * 4, kbeg + KT, te);
    }
    if (NST - 1 < nt) tnext = table(kbeg + (NST - 1) * KT);
    if (NST == 3 && nt > 1) wait_vm<NVM>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int e = 0; e < NFR; ++e) read_item<BMODE>(f1, smem, smem + A_FL, wm, wn, lr, lh, 0, e);
  }
  int st = 0;                 // stage of tile t
  int sn = NST == 3 ? 2 : 1;  // stage the next issued tile goes to
  // One K-tile.  LOADS: issue tile t + NST - 1 (phase A); NEXT: tile t + 1
  // exists (phase B waits for it, with WAITN younger tiles still in flight).
  auto step = [&](int t, auto loads_c, auto next_c, auto waitn_c) {
    constexpr bool LOADS = decltype(loads_c)::value;
    constexpr bool NEXT = decltype(next_c)::value;
    constexpr int WAITN = decltype(waitn_c)::value;
    const float* As = smem + st * SF;
    // phase A: first-half MFMAs of tile t (16 slots of one MFMA pair), the
    // DMA items of tile t + NST - 1 spread over them, and from slot 8 on the
    // second-half fragment reads
    const int kn = kbeg + (t + NST - 1) * KT;
    const uint32_t img = lds0 + static_cast<uint32_t>(sn * SF * 4);
    const int16v te = tnext;
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      mfma_pair<BMODE>(acc, f1, p);
      if constexpr (LOADS) {
#pragma unroll
        for (int e = (p * NVM + 15) / 16; e < ((p + 1) * NVM + 15) / 16; ++e) item(e, img, kn, te);
      }
      if (p >= 8) {
#pragma unroll
        for (int e = (p - 8) * NFR / 8; e < (p - 7) * NFR / 8; ++e)
          read_item<BMODE>(f2, As, As + A_FL, wm, wn, lr, lh, 1, e);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // phase B: the next tile is complete and visible; its first half is read
    // while this tile's second half runs
    const int st1 = st + 1 == NST ? 0 : st + 1;
    if constexpr (NEXT) {
      if (LOADS && t + NST < nt) tnext = table(kbeg + (t + NST) * KT);
      wait_vm<WAITN>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      const float* An = smem + st1 * SF;
#pragma unroll
      for (int p = 0; p < 16; ++p) {
#pragma unroll
        for (int e = p * NFR / 16; e < (p + 1) * NFR / 16; ++e)
          read_item<BMODE>(f1, An, An + A_FL, wm, wn, lr, lh, 0, e);
        mfma_pair<BMODE>(acc, f2, p);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int p = 0; p < 16; ++p) mfma_pair<BMODE>(acc, f2, p);
    }
    st = st1;
    sn = sn + 1 == NST ? 0 : sn + 1;
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  // steady state: every tile issues the one NST - 1 ahead
  int t = 0;
  for (; t + NST - 1 < nt; ++t) step(t, T_{}, T_{}, std::integral_constant<int, NST == 3 ? NVM : 0>{});
  // drain: no more loads; the last tile has no successor
  if (NST == 3 && t + 1 < nt) {
    step(t, F_{}, T_{}, std::integral_constant<int, 0>{});
    ++t;
  }
  if (t < nt) step(t, F_{}, F_{}, std::integral_constant<int, 0>{});
  gemm_epilogue<2, 2, OM>(acc, P, ep, part, m0 + wm * 64, n0 + wn * 64, lr, lh);
}

// ---------------------------------------------------------------------------
// k_conv_patch: stride-1 convolution with the input staged in LDS as a
// padded patch instead of an im2col gather.  A 128-position tile of one or two
// images needs only the input rows those positions touch (+ KH - 1), so per
// K-tile (2 CPH input channels) it loads ~2 CPH x rows x (W + 2 pw) floats
// where the table gather loads 128 x 2 CPH x KH x KW (5-10x fewer, and in
// whole rows).  The weights are repacked once per call into K-tile slabs
// ([group][m-tile][k-tile][64 MI rows][RL]: the 2 CPH x KH x KW taps of the
// K-tile split in two lane halves of HP floats, padded) so their tile is one
// linear LDS-DMA copy.  Structure as k_gemm2: one 4-wave workgroup per CU,
// 3-stage ring, one barrier in the middle of each K-tile.
// K order: lane half h at step s = (cc, kh, kw) uses input channel
// kt*2CPH + h*CPH + cc and tap (kh, kw), in A and B alike.
namespace cp {
constexpr int BN = 128;
template <int KH, int KW, int CPH>
struct Shape {
  static constexpr int T = KH * KW;
  static constexpr int S = CPH * T;                              // MFMA steps per K-tile
  static constexpr int S1 = (S / 2) / 4 * 4;                     // steps of the first half
  static constexpr int HP = (S + 3) / 4 * 4;                     // packed half (floats)
  static constexpr int RL = ((2 * HP / 4) % 2 == 0) ? 2 * HP + 4 : 2 * HP;  // row: RL/4 odd = conflict-free b128
  static constexpr int Q0 = 0, Q1 = S1 / 4, QE = (S + 3) / 4;   // A quads of the halves
};
// per-tile patch geometry (uniform)
struct PatchGeo {
  int img0, a0, rows0, img1;  // segment 0: image, first output row, patch rows; segment 1 starts at row 0
};
}  // namespace cp

template <int KH, int KW, int CPH, int MI, int PD, int NST>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NST == 2 ? 2 : 1, NST == 2 ? 2 : 1)))
k_conv_patch(Params P, const float* __restrict__ wpack, int PW, int CS) {
  using namespace g2;
  using Sh = cp::Shape<KH, KW, CPH>;
  constexpr int BMc = 64 * MI;
  constexpr int A_FL = BMc * Sh::RL;
  constexpr int A_DMA = ((A_FL + 255) / 256 + 3) / 4;   // x4 pieces per wave
  constexpr int A_REG = A_DMA * 4 * 256;                // floats reserved for A in a stage
  constexpr int P_REG = PD * 4 * 64;                    // patch floats per stage (PD dword pieces per wave)
  constexpr int SF = A_REG + P_REG;
  constexpr int NVM = A_DMA + PD;
  static_assert(NST == 2 || NST == 3, "stages");
  static_assert(NST * SF * 4 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) float smem[NST * SF];
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)smem));

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = lane & 31, lh = lane >> 5;

  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, loc = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int tid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int tm = __builtin_amdgcn_readfirstlane(tid % P.tiles_m);
  const int tn = __builtin_amdgcn_readfirstlane((tid / P.tiles_m) % P.tiles_n);
  const int z = __builtin_amdgcn_readfirstlane(tid / (P.tiles_m * P.tiles_n));
  const int n0 = tn * cp::BN;
  const int m0 = tm * BMc;

  const ConvGeom& cv = P.cv;
  const int HW = cv.howo.d, OW = cv.wo_div.d;
  const int ktiles = cv.C / (2 * CPH);
  const float* xin = P.b.p + z * P.grp_b;
  Epi ep = P.e;
  if (z > 0) {
    ep.C += z * P.grp_c;
    if (ep.bias) ep.bias += z * P.grp_bias;
  }
  // A: this tile's packed slabs, one per K-tile, each A_FL floats
  const float* abase = wpack + ((int64_t)z * P.tiles_m + tm) * ktiles * A_FL;
  const int4v arsrc = make_rsrc(abase, static_cast<uint32_t>((int64_t)ktiles * A_FL * 4));
  uint32_t aoff[A_DMA];
#pragma unroll
  for (int i = 0; i < A_DMA; ++i) {
    const int f = (wave * A_DMA + i) * 256 + lane * 4;
    aoff[i] = f < A_FL ? static_cast<uint32_t>(f * 4) : 0x80000000u;
  }

  // patch geometry of this tile (positions n0 .. n0 + 127, at most two images)
  const int plast = min(n0 + cp::BN, P.N) - 1;
  const int img0 = n0 / HW, img1 = plast / HW;
  const int a0 = (n0 - img0 * HW) / OW;
  const int b0 = img1 == img0 ? (plast - img0 * HW) / OW : cv.Ho - 1;
  const int rows0 = b0 - a0 + KH;
  const int rows1 = img1 == img0 ? 0 : (plast - img1 * HW) / OW + KH;
  const int R = rows0 + rows1;
  // per-lane source of the patch pieces: patch float f = (ch, prow, pcol)
  const int4v xrsrc = make_rsrc(xin, static_cast<uint32_t>(cv.in_bytes));
  const uint32_t HW4 = static_cast<uint32_t>(cv.H * cv.W * 4);
  uint32_t poff[PD];
#pragma unroll
  for (int i = 0; i < PD; ++i) {
    const int f = (wave * PD + i) * 64 + lane;
    const int ch = f / CS, w = f - ch * CS;
    const int prow = w / PW, pcol = w - prow * PW;
    uint32_t off = 0x80000000u;
    if (ch < 2 * CPH && prow < R) {
      const bool s1 = prow >= rows0;
      const int img = s1 ? img1 : img0;
      const int y = (s1 ? prow - rows0 : a0 + prow) - cv.ph;
      const int x = pcol - cv.pw;
      if (y >= 0 && y < cv.H && x >= 0 && x < cv.W)
        off = static_cast<uint32_t>((int64_t)img * cv.chw * 4) + static_cast<uint32_t>(ch) * HW4 +
              static_cast<uint32_t>((y * cv.W + x) * 4);
    }
    poff[i] = off;
  }
  // per-lane B fragment base (floats) of columns j = 0, 1 inside the patch
  int pb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = min(n0 + wn * 64 + j * 32 + lr, plast);
    const int img = n / HW, sp = n - img * HW;
    const int oh = sp / OW, ow = sp - oh * OW;
    const int prow = img == img0 ? oh - a0 : rows0 + oh;
    pb[j] = prow * PW + ow + lh * CPH * CS;
  }

  floatx16 acc[MI][2];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  auto issue = [&](int kt, int stg, int e) {  // DMA item e of K-tile kt into stage stg
    const uint32_t img = lds0 + static_cast<uint32_t>(stg * SF * 4);
    if (e < A_DMA) {
      dma_b128(arsrc, aoff[e] + static_cast<uint32_t>(kt * A_FL * 4),
               img + static_cast<uint32_t>((wave * A_DMA + e) * 1024));
    } else {
      const int i = e - A_DMA;
      dma_b32(xrsrc, poff[i] + static_cast<uint32_t>(kt * 2 * CPH) * HW4,
              img + static_cast<uint32_t>((A_REG + (wave * PD + i) * 64) * 4));
    }
  };
  // fragments: A quads [q0, q1) and B steps [s0, s1) of one half
  constexpr int QA = Sh::QE - Sh::Q1 > Sh::Q1 ? Sh::QE - Sh::Q1 : Sh::Q1;
  constexpr int SB = Sh::S - Sh::S1 > Sh::S1 ? Sh::S - Sh::S1 : Sh::S1;
  struct Fr {
    float4 a[MI][QA];
    float b[2][SB];
  };
  auto read_a = [&](Fr& F, const float* st, int q, int qb) {  // quad q into slot q - qb
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = wm * 32 * MI + i * 32 + lr;
      F.a[i][q - qb] = *reinterpret_cast<const float4*>(st + m * Sh::RL + lh * Sh::HP + 4 * q);
    }
  };
  auto read_b = [&](Fr& F, const float* st, int sx, int sb) {  // step sx into slot sx - sb
    const int cc = sx / Sh::T, tp = sx - cc * Sh::T, kh = tp / KW, kw = tp - kh * KW;
#pragma unroll
    for (int j = 0; j < 2; ++j) F.b[j][sx - sb] = st[A_REG + pb[j] + cc * CS + kh * PW + kw];
  };
  auto mfma_step = [&](const Fr& F, int sx, int qb, int sb) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const float a = pick(F.a[i][(sx >> 2) - qb], sx);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, F.b[j][sx - sb], acc[i][j], 0, 0, 0);
    }
  };

  Fr f1, f2;
  const int nt = ktiles;
  if (nt > 0) {
#pragma unroll
    for (int e = 0; e < NVM; ++e) issue(0, 0, e);
    if (NST == 3 && nt > 1) {
#pragma unroll
      for (int e = 0; e < NVM; ++e) issue(1, 1, e);
      wait_vm<NVM>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int q = Sh::Q0; q < Sh::Q1; ++q) read_a(f1, smem, q, Sh::Q0);
#pragma unroll
    for (int sx = 0; sx < Sh::S1; ++sx) read_b(f1, smem, sx, 0);
  }
  int st = 0, sn = NST - 1;
  auto step = [&](int t, auto loads_c, auto next_c, auto waitn_c) {
    constexpr bool LOADS = decltype(loads_c)::value;
    constexpr bool NEXT = decltype(next_c)::value;
    constexpr int WAITN = decltype(waitn_c)::value;
    const float* cur = smem + st * SF;
    // phase A: first-half MFMAs, DMA of tile t + 2, second-half reads
#pragma unroll
    for (int sx = 0; sx < Sh::S1; ++sx) {
      mfma_step(f1, sx, Sh::Q0, 0);
      if constexpr (LOADS) {
#pragma unroll
        for (int e = (sx * NVM + Sh::S1 - 1) / Sh::S1; e < ((sx + 1) * NVM + Sh::S1 - 1) / Sh::S1; ++e)
          issue(t + NST - 1, sn, e);
      }
      if (sx == Sh::S1 / 2) {
#pragma unroll
        for (int q = Sh::Q1; q < Sh::QE; ++q) read_a(f2, cur, q, Sh::Q1);
      }
      if (sx >= Sh::S1 / 2) {
#pragma unroll
        for (int u = Sh::S1 + (sx - Sh::S1 / 2) * (Sh::S - Sh::S1) / (Sh::S1 - Sh::S1 / 2);
             u < Sh::S1 + (sx + 1 - Sh::S1 / 2) * (Sh::S - Sh::S1) / (Sh::S1 - Sh::S1 / 2); ++u)
          read_b(f2, cur, u, Sh::S1);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    const int st1 = st + 1 == NST ? 0 : st + 1;
    if constexpr (NEXT) {
      wait_vm<WAITN>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      const float* nx = smem + st1 * SF;
      constexpr int S2 = Sh::S - Sh::S1;
#pragma unroll
      for (int sx = Sh::S1; sx < Sh::S; ++sx) {
        const int v = sx - Sh::S1;
        if (v == 0) {
#pragma unroll
          for (int q = Sh::Q0; q < Sh::Q1; ++q) read_a(f1, nx, q, Sh::Q0);
        }
#pragma unroll
        for (int u = v * Sh::S1 / S2; u < (v + 1) * Sh::S1 / S2; ++u) read_b(f1, nx, u, 0);
        mfma_step(f2, sx, Sh::Q1, Sh::S1);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int sx = Sh::S1; sx < Sh::S; ++sx) mfma_step(f2, sx, Sh::Q1, Sh::S1);
    }
    st = st1;
    sn = sn + 1 == NST ? 0 : sn + 1;
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  int t = 0;
  for (; t + NST - 1 < nt; ++t) step(t, T_{}, T_{}, std::integral_constant<int, NST == 3 ? NVM : 0>{});
  if (NST == 3 && t + 1 < nt) {
    step(t, F_{}, T_{}, std::integral_constant<int, 0>{});
    ++t;
  }
  if (t < nt) step(t, F_{}, F_{}, std::integral_constant<int, 0>{});
  gemm_epilogue<MI, 2, OUT_NCHW>(acc, P, ep, nullptr, m0 + wm * 32 * MI, n0 + wn * 64, lr, lh);
}

// Weight repack for k_conv_patch: w [G*M][C*T] -> [G][tiles_m][ktiles][64 MI][RL],
// row layout [half 0: CPH*T taps, zero pad to HP][half 1 ...][pad to RL].
__global__ void __launch_bounds__(256) k_conv_patch_pack(const float* __restrict__ w, float* __restrict__ out, int G,
                                                         int M, int C, int T, int CPH, int HP, int RL, int BMc,
                                                         int tiles_m, int ktiles, int64_t total) {
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = idx;
    const int col = static_cast<int>(r % RL);
    r /= RL;
    const int row = static_cast<int>(r % BMc);
    r /= BMc;
    const int kt = static_cast<int>(r % ktiles);
    r /= ktiles;
    const int tm = static_cast<int>(r % tiles_m);
    const int g = static_cast<int>(r / tiles_m);
    const int m = tm * BMc + row;
    const int h = col / HP, u = col - h * HP;
    float v = 0.0f;
    if (h < 2 && u < CPH * T && m < M) {
      const int c = kt * 2 * CPH + h * CPH + u / T;
      v = w[((int64_t)g * M + m) * C * T + (int64_t)c * T + (u % T)];
    }
    out[idx] = v;
  }
}


// y = alpha * op(A) x + beta * y, one wave per output element row
__global__ void __launch_bounds__(256) k_gemv(int trans, int M, int N, float alpha,
                                              const float* __restrict__ A,
                                              const float* __restrict__ x, float beta,
                                              float* __restrict__ y) {
  // non-trans: y[M] = A[M][N] x[N];  trans: y[N] = A[M][N]^T x[M]
  const int outs = trans ? N : M;
  const int red = trans ? M : N;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int nw = (gridDim.x * blockDim.x) >> 6;
  for (int o = wave; o < outs; o += nw) {
    float s = 0.0f;
    for (int r = lane; r < red; r += 64) {
      const float a = trans ? A[(int64_t)r * N + o] : A[(int64_t)o * N + r];
      s += a * x[r];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) y[o] = alpha * s + (beta != 0.0f ? beta * y[o] : 0.0f);
  }
}

// im2col for `nimg` images written into a [K][ldcol] matrix at column offset
// img*HoWo (ldcol >= nimg*HoWo).  Grid: y = column-matrix row (c, kh, kw),
// block-uniform, so its decomposition is scalar; x strides over the output
// positions (n, ho, wo) with 32-bit magic-number divisions; stores are
// coalesced along the row.
__global__ void __launch_bounds__(256)
    k_im2col(const float* __restrict__ im, int64_t im_img, int nimg, int C, int H, int W, int KH,
             int KW, int ph, int pw, int sh, int sw, int dh, int dw, int Ho, int Wo,
             float* __restrict__ col, int64_t ldcol, FastDiv howo, FastDiv wo_div) {
  const int krow = blockIdx.y;
  const int kw = krow % KW, kh = (krow / KW) % KH, c = krow / (KW * KH);
  const int HoWo = Ho * Wo;
  const int P = nimg * HoWo;
  float* dst = col + (int64_t)krow * ldcol;
  if (krow == C * KH * KW) {  // the ones row (im2col_core ones_row: bias gradient in the dW GEMM)
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x) dst[p] = 1.0f;
    return;
  }
  const float* src = im + (int64_t)c * H * W;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x) {
    const uint32_t n = fdiv(static_cast<uint32_t>(p), howo);
    const uint32_t r = static_cast<uint32_t>(p) - n * howo.d;
    const uint32_t ho = fdiv(r, wo_div);
    const uint32_t wo = r - ho * wo_div.d;
    const int iy = static_cast<int>(ho) * sh - ph + kh * dh;
    const int ix = static_cast<int>(wo) * sw - pw + kw * dw;
    float v = 0.0f;
    if (static_cast<unsigned>(iy) < static_cast<unsigned>(H) && static_cast<unsigned>(ix) < static_cast<unsigned>(W))
      v = src[n * im_img + iy * W + ix];
    dst[p] = v;
  }
}

// im2col, four consecutive output positions per thread and one 16-byte store
// (HoWo % 4 == 0, ldcol % 4 == 0, col 16-byte aligned: a quad never spans two
// images; it may wrap output rows when Wo % 4 != 0)
__global__ void __launch_bounds__(256)
    k_im2col4(const float* __restrict__ im, int64_t im_img, int nimg, int C, int H, int W, int KH,
              int KW, int ph, int pw, int sh, int sw, int dh, int dw, int Ho, int Wo,
              float* __restrict__ col, int64_t ldcol, FastDiv howo, FastDiv wo_div) {
  const int krow = blockIdx.y;
  const int kw = krow % KW, kh = (krow / KW) % KH, c = krow / (KW * KH);
  const int P4 = nimg * Ho * Wo / 4;
  float4* dst = reinterpret_cast<float4*>(col + (int64_t)krow * ldcol);
  if (krow == C * KH * KW) {  // the ones row (see k_im2col)
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < P4; q += gridDim.x * blockDim.x)
      dst[q] = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
    return;
  }
  const float* src = im + (int64_t)c * H * W;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < P4; q += gridDim.x * blockDim.x) {
    const uint32_t p = 4u * static_cast<uint32_t>(q);
    const uint32_t n = fdiv(p, howo);
    const uint32_t r = p - n * howo.d;
    int ho = static_cast<int>(fdiv(r, wo_div));
    int wo = static_cast<int>(r) - ho * Wo;
    const float* img = src + n * im_img;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int iy = ho * sh - ph + kh * dh;
      const int ix = wo * sw - pw + kw * dw;
      const bool ok = static_cast<unsigned>(iy) < static_cast<unsigned>(H) && static_cast<unsigned>(ix) < static_cast<unsigned>(W);
      v[j] = ok ? img[iy * W + ix] : 0.0f;
      if (++wo == Wo) {
        wo = 0;
        ++ho;
      }
    }
    dst[q] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// col2im: one thread per image pixel, gathers all column entries that map to it
__global__ void __launch_bounds__(256)
    k_col2im(const float* __restrict__ col, int64_t ldcol, int nimg, int C, int H, int W, int KH,
             int KW, int ph, int pw, int sh, int sw, int dh, int dw, int Ho, int Wo,
             float* __restrict__ im, int64_t im_img, int accumulate) {
  const int64_t total = (int64_t)nimg * C * H * W;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int64_t t = idx;
    const int x = t % W; t /= W;
    const int y = t % H; t /= H;
    const int c = t % C; t /= C;
    const int n = static_cast<int>(t);
    float s = 0.0f;
    for (int kh = 0; kh < KH; ++kh) {
      const int yy = y + ph - kh * dh;
      if (yy < 0 || yy % sh) continue;
      const int ho = yy / sh;
      if (ho >= Ho) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int xx = x + pw - kw * dw;
        if (xx < 0 || xx % sw) continue;
        const int wo = xx / sw;
        if (wo >= Wo) continue;
        const int64_t krow = ((int64_t)c * KH + kh) * KW + kw;
        s += col[krow * ldcol + (int64_t)n * Ho * Wo + (int64_t)ho * Wo + wo];
      }
    }
    float* dst = im + n * im_img + ((int64_t)c * H + y) * W + x;
    *dst = accumulate ? *dst + s : s;
  }
}


template <int WM, int WN, int MI, int NI, int AM, int BMODE, int OM, int KB>
int launch_cfg(Params P, int gz, hipStream_t s) {
  constexpr int BMr = WM * MI * 32, BNr = WN * NI * 32;
  P.tiles_m = (P.M + BMr - 1) / BMr;
  P.tiles_n = (P.N + BNr - 1) / BNr;
  P.tiles_z = gz;
  const int64_t nwg = (int64_t)P.tiles_m * P.tiles_n * gz;
  RRAM_REQUIRE(nwg < (1ll << 31), "gemm: grid too large");
  hipLaunchKernelGGL((k_gemm<WM, WN, MI, NI, AM, BMODE, OM, KB>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, P);
  return launch_status("gemm");
}

// Tile choice.  BN = 128 with BM in {192, 128, 96, 64} picked to minimise the
// padded rows of M (AlexNet: conv1 M = 96, conv4 M = 192 per group) as long as
// the grid keeps >= 2 blocks per CU; 64x64 when even that grid is too small.
// force_big: split-K grids (128x128).
template <int AM, int BMODE, int OM, int KB>
int launch(const Params& P, int gz, hipStream_t s, bool force_big) {
  if (force_big) {
#ifndef RRAM_SPLIT_THIN32
#define RRAM_SPLIT_THIN32 1
#endif
    // split-K grids with M <= 32 and N > 64 (the CIFAR-10 weight gradients:
    // Cout = 32, N = 76 / 801): 32 x 128 tiles, which waste no MFMA rows (64 x
    // 64 padded half): C4 0.362 -> 0.348 ms per iteration.  Not for N <= 64
    // (LeNet conv1, N = 26: 0.199 -> 0.204 ms, the 128-wide B tile gathers
    // mostly padding), profiles/r05_ab_split_thin32.txt
    if constexpr (KB == 32) {
      if (RRAM_SPLIT_THIN32 && P.M <= 32 && P.N > 64) return launch_cfg<1, 4, 1, 1, AM, BMODE, OM, KB>(P, gz, s);
    }
    // split-K grids: 64 x 64 tiles when an operand is that thin (conv weight gradients)
    if (P.M <= 64 || P.N <= 64) return launch_cfg<2, 2, 1, 1, AM, BMODE, OM, KB>(P, gz, s);
    return launch_cfg<2, 2, 2, 2, AM, BMODE, OM, KB>(P, gz, s);
  }
  // thin M (CIFAR / LeNet convolutions, M = 20..32): a 32 x 128 tile wastes no
  // MFMA rows (64 x 64 would pad half of them)
  if constexpr (KB == 32) {
    if (P.M <= 32)
      return launch_cfg<1, 4, 1, 1, AM, BMODE, OM, KB>(P, gz, s);
  }
  // 128 x 256 at 2 waves per SIMD (8 accumulators per wave: half the LDS and
  // L2 bytes per MFMA of 128 x 128) when M fills whole 128-row tiles and the
  // grid still gives every CU >= 2 rounds of its 2 resident blocks.  MI355X,
  // AlexNet b256: conv2 (M = 128 per group, N = 186,624) 1.08 -> 1.04 ms;
  // conv3 (507 such tiles, one round) 0.70 -> 0.69 ms is within noise, and
  // conv4 / conv5 / conv1 (fewer tiles or M % 128 != 0) are slower, so they
  // keep the policy below.
  if (KB == 16 && P.M % 128 == 0 && (int64_t)(P.M / 128) * ((P.N + 255) / 256) * gz >= 1024)
    return launch_cfg<2, 2, 2, 4, AM, BMODE, OM, KB>(P, gz, s);
  const int64_t ntn = (P.N + 127) / 128;
  const int cands[4] = {128, 192, 96, 64};  // ties keep 128 (2 blocks per CU)
  int best = 0;
  int64_t best_pad = -1;
  for (int c : cands) {
    const int64_t tiles_m = (P.M + c - 1) / c;
    if (tiles_m * ntn * gz < 512 && c != 64) continue;
    const int64_t pad = tiles_m * c - P.M;
    if (best_pad < 0 || pad < best_pad) {
      best = c;
      best_pad = pad;
    }
  }
  if (KB == 16 && P.M % 128 != 0 && P.M % 64 == 0 && ntn * (P.M / 64) * gz >= 512)
    best = 64;  // e.g. M = 192: three unpadded 64-row tiles beat one 192-row tile at KB = 16
  if (best == 64 && ntn * ((P.M + 63) / 64) * gz < 256)
    return launch_cfg<2, 2, 1, 1, AM, BMODE, OM, KB>(P, gz, s);  // 64 x 64: twice the blocks
  switch (best) {
    case 192: return launch_cfg<2, 2, 3, 2, AM, BMODE, OM, KB>(P, gz, s);  // 192 x 128
    case 128: return launch_cfg<2, 2, 2, 2, AM, BMODE, OM, KB>(P, gz, s);  // 128 x 128
    case 96:
      if constexpr (KB == 16) return launch_cfg<2, 2, 2, 2, AM, BMODE, OM, KB>(P, gz, s);  // 96 x 16 splits float4s
      else return launch_cfg<1, 4, 3, 1, AM, BMODE, OM, KB>(P, gz, s);   //  96 x 128
    default: return launch_cfg<1, 4, 2, 1, AM, BMODE, OM, KB>(P, gz, s);   //  64 x 128
  }
}

template <int AM, int BMODE, int OM>
int launch2(Params P, int gz, hipStream_t s) {
  P.tiles_m = (P.M + g2::BM - 1) / g2::BM;
  P.tiles_n = (P.N + g2::BN - 1) / g2::BN;
  P.tiles_z = gz;
  const int64_t nwg = (int64_t)P.tiles_m * P.tiles_n * gz;
  RRAM_REQUIRE(nwg < (1ll << 31), "gemm: grid too large");
  hipLaunchKernelGGL((k_gemm2<AM, BMODE, OM, 3>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, P);
  return launch_status("gemm2");
}

// k_gemm2 policy (3 LDS stages): 16-byte A and B (the IP layers), M padded by
// at most 1/8 in 128-row tiles, N > 64, and operands addressable with 32-bit
// buffer offsets.  MI355X, AlexNet b256 (kbench): fc6 111 -> 119 TFLOP/s, fc7
// 100 -> 109.  The table-gather convolutions stay on k_gemm: at one wave per
// SIMD the gather's 16 four-byte LDS-DMA issues per wave and K-tile cap it at
// 68 % MFMA busy (conv3 109 -> 100 TFLOP/s measured).
bool gemm2_ok(int am, int bm, const Params& P) {
  if (am != KCV || bm != KCV) return false;
  const int64_t mt = (P.M + g2::BM - 1) / g2::BM * g2::BM;
  if (P.N <= 64 || (mt - P.M) * 8 > mt) return false;
  auto fits = [](const View& v) { return ((int64_t)(v.rows - 1) * v.ld + v.kdim) * 4 < (1ll << 31); };
  if (!fits(P.a)) return false;
  if (bm == KCV && !fits(P.b)) return false;
  return true;
}

// K-tile depth of the implicit-GEMM convolution
// Measured on MI355X (scripts/gpu_sweep.sh, AlexNet b256): K >= 1024 runs
// faster with 16-deep K-tiles (half the LDS and loader registers: 3 waves per
// SIMD instead of 2), short K (conv1, K = 363) with 32.
int conv_kb(int K) {
  return K >= 1024 ? 16 : 32;
}

int dispatch(int am, int bm, int om, const Params& P, int gz, hipStream_t s, bool force_big = false) {
  if (gemm2_ok(am, bm, P)) {
    if (om == OUT_ROWMAJOR) return launch2<KCV, KCV, OUT_ROWMAJOR>(P, gz, s);
  }
  if (bm == CONV && om == OUT_NCHW && conv_kb(P.K) == 16) {
    if (am == KC) return launch<KC, CONV, OUT_NCHW, 16>(P, gz, s, force_big);
    if (am == KCV) return launch<KCV, CONV, OUT_NCHW, 16>(P, gz, s, force_big);
  }
  if (bm == CONVT && om == OUT_NCHW && conv_kb(P.K) == 16) {
    if (am == KC) return launch<KC, CONVT, OUT_NCHW, 16>(P, gz, s, force_big);
    if (am == KCV) return launch<KCV, CONVT, OUT_NCHW, 16>(P, gz, s, force_big);
    if (am == KCU) return launch<KCU, CONVT, OUT_NCHW, 16>(P, gz, s, force_big);
  }
  if (bm == CONVT64 && om == OUT_NCHW && conv_kb(P.K) == 16) {
    if (am == KC) return launch<KC, CONVT64, OUT_NCHW, 16>(P, gz, s, force_big);
    if (am == KCV) return launch<KCV, CONVT64, OUT_NCHW, 16>(P, gz, s, force_big);
  }
#define RRAM_D(A_, B_, O_) \
  if (am == A_ && bm == B_ && om == O_) return launch<A_, B_, O_, 32>(P, gz, s, force_big);
  RRAM_D(KC, KC, OUT_ROWMAJOR)
  RRAM_D(KCV, KC, OUT_ROWMAJOR)
  RRAM_D(KC, KCV, OUT_ROWMAJOR)
  RRAM_D(KCV, KCV, OUT_ROWMAJOR)
  RRAM_D(KC, RC, OUT_ROWMAJOR)
  RRAM_D(KCV, RC, OUT_ROWMAJOR)
  RRAM_D(RC, KC, OUT_ROWMAJOR)
  RRAM_D(RC, KCV, OUT_ROWMAJOR)
  RRAM_D(RC, RC, OUT_ROWMAJOR)
  RRAM_D(KC, CONV, OUT_NCHW)
  RRAM_D(KCV, CONV, OUT_NCHW)
  RRAM_D(KC, CONVT, OUT_NCHW)
  RRAM_D(KCV, CONVT, OUT_NCHW)
  RRAM_D(KCU, CONVT, OUT_NCHW)
  RRAM_D(KC, CONVT64, OUT_NCHW)
  RRAM_D(KCV, CONVT64, OUT_NCHW)
  RRAM_D(NCHW, KC, OUT_ROWMAJOR)
  RRAM_D(NCHW, KCV, OUT_ROWMAJOR)
  RRAM_D(NCHW, IM2T, OUT_ROWMAJOR)
  RRAM_D(RC, NCHWT, OUT_ROWMAJOR)
#undef RRAM_D
  set_error("gemm: unsupported operand combination %d/%d/%d", am, bm, om);
  return RRAM_EUNSUPPORTED;
}

// KC view eligible for 16-byte loads (also for every group offset)
bool vec_ok(const float* p, int64_t ld, int K, int64_t grp = 0) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0 && (ld & 3) == 0 && (K & 3) == 0 && (grp & 3) == 0;
}

// Per-geometry gather table of the CONVT loader, built once per process and
// cached (a few KB per conv geometry; never freed).  Entry k < K holds the
// input offset of reduction index k = (c, kh, kw) in bytes and its tap
// kh*KW + kw (0 for pad-free convolutions, whose taps are always inside the
// image); entries past K (the last tile's tail and the one-tile prefetch
// overrun) hold tap 31, which no column marks valid.
// Keyed by the current HIP device too: the table lives in that device's HBM.
std::mutex& conv_table_mutex() {
  static std::mutex mu;
  return mu;
}
std::map<std::array<int, 11>, int2*>& conv_table_cache() {
  static std::map<std::array<int, 11>, int2*> cache;
  return cache;
}

const int2* conv_table(const ConvGeom& cv, int K, bool padded, bool wide, hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  auto& cache = conv_table_cache();
  const std::array<int, 11> key{dev, cv.C, cv.H, cv.W, cv.KH, cv.KW, cv.dh, cv.dw, padded ? 1 : 0, K, wide ? 1 : 0};
  std::lock_guard<std::mutex> g(conv_table_mutex());
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  const int len = (K + BK - 1) / BK * BK + 2 * BK;
  std::vector<int2> h(len, int2{0, wide ? 63 : 31});  // the never-valid tap
  for (int k = 0; k < K; ++k) {
    const int c = k / (cv.KH * cv.KW), r = k % (cv.KH * cv.KW);
    const int kh = r / cv.KW, kw = r % cv.KW;
    h[k].x = 4 * (c * cv.H * cv.W + kh * cv.dh * cv.W + kw * cv.dw);
    h[k].y = padded ? r : 0;
  }
  int2* d = nullptr;
  if (hipMalloc(&d, len * sizeof(int2)) != hipSuccess) return nullptr;
  if (hipMemcpyAsync(d, h.data(), len * sizeof(int2), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    (void)hipFree(d);
    return nullptr;
  }
  cache[key] = d;
  return d;
}

// Row table of the IM2T loader (cached with the CONVT tables): entry n < K
// holds row n = (c, kh, kw) of the column matrix as {4 (c H W + kh dh W +
// kw dw), kh dh | kw dw << 16}; entry K the ones row {0, -1} when `ones`;
// the rest (tile padding) {0, 0x7FFF7FFF}, never inside the image.
const int2* im2t_table(const ConvGeom& cv, int K, bool ones, int rows_pad, hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  auto& cache = conv_table_cache();
  const int len = (K + 1 + rows_pad - 1) / rows_pad * rows_pad + rows_pad;
  const std::array<int, 11> key{dev, cv.C, cv.H, cv.W, cv.KH, cv.KW, cv.dh, cv.dw, len, K, ones ? 3 : 2};
  std::lock_guard<std::mutex> g(conv_table_mutex());
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  std::vector<int2> h(len, int2{0, 0x7FFF7FFF});
  for (int k = 0; k < K; ++k) {
    const int c = k / (cv.KH * cv.KW), r = k % (cv.KH * cv.KW);
    const int kh = r / cv.KW, kw = r % cv.KW;
    h[k].x = 4 * (c * cv.H * cv.W + kh * cv.dh * cv.W + kw * cv.dw);
    h[k].y = (kh * cv.dh) | ((kw * cv.dw) << 16);
  }
  if (ones) h[K] = int2{0, -1};
  int2* d = nullptr;
  if (hipMalloc(&d, len * sizeof(int2)) != hipSuccess) return nullptr;
  if (hipMemcpyAsync(d, h.data(), len * sizeof(int2), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    (void)hipFree(d);
    return nullptr;
  }
  cache[key] = d;
  return d;
}

}  // namespace

// bumped whenever internal scratch is freed (rram_scratch_generation)
std::atomic<uint64_t>& scratch_gen() {
  static std::atomic<uint64_t> g{0};
  return g;
}

// Frees every cached gather table (all devices).  Called by
// rram_release_caches(); the caller guarantees no launch still reads them.
int release_conv_tables() {
  std::lock_guard<std::mutex> g(conv_table_mutex());
  scratch_gen().fetch_add(1);
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (auto& kv : conv_table_cache()) {
    (void)hipSetDevice(kv.first[0]);
    (void)hipDeviceSynchronize();
    (void)hipFree(kv.second);
  }
  conv_table_cache().clear();
  (void)hipSetDevice(cur);
  return RRAM_OK;
}

// Shared by the C-ABI entry points in conv_api.hip.
int gemm_x6_nt(int M, int N, int K, float alpha, const float* A, int lda, const float* B, int ldb, float beta,
               float* C, int ldc, const float* bias, int bias_mode, int relu, void* ws, size_t ws_bytes,
               hipStream_t s, const void* a_rows = nullptr, char* y_rows = nullptr, int y_bmc = 0);

int gemm_core(int trans_a, int trans_b, int M, int N, int K, float alpha, const float* A, int lda,
              const float* B, int ldb, float beta, float* C, int ldc, const float* bias,
              int bias_mode, int relu, void* ws, size_t ws_bytes, hipStream_t s) {
  RRAM_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gemm: negative size");
  if (M == 0 || N == 0) return RRAM_OK;
  RRAM_REQUIRE(C != nullptr, "gemm: C is NULL");
  RRAM_REQUIRE(K == 0 || (A && B), "gemm: A/B NULL");
  RRAM_REQUIRE(ldc >= N, "gemm: ldc < N");
  RRAM_REQUIRE(trans_a ? lda >= M : lda >= K || K == 0, "gemm: lda too small");
  RRAM_REQUIRE(trans_b ? ldb >= K || K == 0 : ldb >= N, "gemm: ldb too small");
  if (!trans_a && trans_b) {  // InnerProduct forward: the bf16x6 engine when it covers the shape
    const int rc = gemm_x6_nt(M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, bias, bias_mode, relu, ws, ws_bytes, s);
    if (rc != 0) return rc < 0 ? rc : RRAM_OK;
  }
  Params P{};
  P.a = make_view(A, lda, M, K);
  P.b = make_view(B, ldb, N, K);
  P.e = make_epi(C, ldc, alpha, beta, bias, bias_mode, relu);
  P.M = M;
  P.N = N;
  P.K = K;
  P.split = 1;
  P.k_chunk = K;
  // op(A)(m,k) = trans_a ? A[k*lda+m] : A[m*lda+k]; op(B)(k,n) = trans_b ? B[n*ldb+k] : B[k*ldb+n]
  int am = trans_a ? RC : KC;
  int bm = trans_b ? KC : RC;
  if (am == KC && vec_ok(A, lda, K)) am = KCV;
  if (bm == KC && vec_ok(B, ldb, K)) bm = KCV;
  // split-K when the 128x128 grid is far below the CU count and K is long
  const int64_t tiles = (int64_t)((N + 127) / 128) * ((M + 127) / 128);
  int split = 1;
  // split-K target grid (blocks; 512 measured neutral, profiles/r04_ab_tail_batched.txt)
  constexpr int target = 256;
  // (kept for tiny products too: CIFAR-10 ip1 without the split measured
  // slower, 8.1k -> 7.3k maps/s, profiles/r04_ab_tail_batched.txt).
  // the least K that splits, and half of it the least K per split (rounds
  // 1-4: 1024; 256 since LeNet ip1 / ip2, K = 800 / 500: a lone workgroup
  // walking K is all latency, profiles/r04_ab_tail_batched.txt)
  constexpr int mink = 256;
  if (ws != nullptr && tiles < target && K >= mink) {
    split = static_cast<int>(target / (tiles > 0 ? tiles : 1));
    if (split > target / 16) split = target / 16;
    while (split > 1 && (K / split) < std::min(256, mink / 2)) --split;
    while (split > 1 && (size_t)split * M * N * sizeof(float) > ws_bytes) --split;
  }
  if (split > 1) {
    int chunk = (K + split - 1) / split;
    chunk = (chunk + BK - 1) / BK * BK;
    split = (K + chunk - 1) / chunk;
    P.split = split;
    P.k_chunk = chunk;
    P.ws = static_cast<float*>(ws);
    int rc = dispatch(am, bm, OUT_ROWMAJOR, P, split, s, true);
    if (rc) return rc;
    hipLaunchKernelGGL(k_splitk_reduce, dim3(stream_blocks((int64_t)M * N)), dim3(256), 0, s,
                       P.ws, split, M, N, P.e);
    return launch_status("gemm splitk reduce");
  }
  return dispatch(am, bm, OUT_ROWMAJOR, P, 1, s);
}


// Packed-weight buffers of k_conv_patch, one per (device, stream), grown on
// demand and reused by every later call on that stream (stream order keeps a
// launch from overwriting a buffer an earlier launch still reads).
std::mutex& pack_mutex() {
  static std::mutex mu;
  return mu;
}
// key: (device, stream, slot); slot 0 = pack buffers, 1 = conv split-K partials
std::map<std::tuple<int, hipStream_t, int>, std::pair<float*, size_t>>& pack_cache() {
  static std::map<std::tuple<int, hipStream_t, int>, std::pair<float*, size_t>> cache;
  return cache;
}

float* stream_buffer(int slot, size_t floats, hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> g(pack_mutex());
  auto& e = pack_cache()[{dev, s, slot}];
  if (e.second >= floats) return e.first;
  if (e.first) {
    if (hipStreamSynchronize(s) != hipSuccess) return nullptr;
    (void)hipFree(e.first);
    e = {nullptr, 0};
    scratch_gen().fetch_add(1);
  }
  float* p = nullptr;
  if (hipMalloc(&p, floats * sizeof(float)) != hipSuccess) return nullptr;
  e = {p, floats};
  return p;
}
float* pack_buffer(size_t floats, hipStream_t s) { return stream_buffer(0, floats, s); }

template <int KH, int KW, int CPH, int MI, int PD>
int launch_patch(Params P, const float* wpack, int PW, int CS, int gz, hipStream_t s) {
  // LDS stages: 2 (two workgroups per CU, 2 waves per SIMD) whenever two
  // workgroups' 2-stage rings fit the 160 KB LDS, else 3
  using Sh = cp::Shape<KH, KW, CPH>;
  constexpr int a_reg = ((64 * MI * Sh::RL + 255) / 256 + 3) / 4 * 4 * 256;
  constexpr int sf = a_reg + PD * 4 * 64;
  constexpr bool two_fit = 2 * 2 * sf * 4 <= 160 * 1024;
  const int nst = two_fit ? 2 : 3;
  P.tiles_m = (P.M + 64 * MI - 1) / (64 * MI);
  P.tiles_n = (P.N + cp::BN - 1) / cp::BN;
  P.tiles_z = gz;
  const int64_t nwg = (int64_t)P.tiles_m * P.tiles_n * gz;
  RRAM_REQUIRE(nwg < (1ll << 31), "conv: grid too large");
  bool done = false;
  if constexpr (two_fit) {
    if (nst == 2) {
      hipLaunchKernelGGL((k_conv_patch<KH, KW, CPH, MI, PD, 2>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, P,
                         wpack, PW, CS);
      done = true;
    }
  }
  if (!done)
    hipLaunchKernelGGL((k_conv_patch<KH, KW, CPH, MI, PD, 3>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, P,
                       wpack, PW, CS);
  return launch_status("conv patch");
}

// k_conv_patch for a stride-1, undilated 3x3 / 5x5 convolution whose output
// planes hold >= 128 positions.  Returns 1 when it ran, 0 when the shape is
// not covered (the caller falls back to the implicit-im2col GEMM), < 0 on
// error.
int conv_patch_fwd(const rram_conv_desc* d, const float* w, Params& P, hipStream_t s) {
  const int KH = d->kernel_h, KW = d->kernel_w;
  if (d->stride_h != 1 || d->stride_w != 1 || d->dilation_h != 1 || d->dilation_w != 1) return 0;
  if (!((KH == 3 && KW == 3) || (KH == 5 && KW == 5))) return 0;
  const int CPH = KH == 3 ? 2 : 1;
  const int G = d->group, Cg = d->channels / G, M = d->num_output / G;
  const int HW = d->out_h * d->out_w, OW = d->out_w, OH = d->out_h;
  if (HW < 128 || Cg % (2 * CPH) != 0 || Cg == 0) return 0;
  if ((reinterpret_cast<uintptr_t>(w) & 3u) != 0) return 0;
  // M tile: 128 or 192 rows, whichever pads less (<= 1/8 padded rows)
  const int t128 = (M + 127) / 128 * 128, t192 = (M + 191) / 192 * 192;
  const int MI = (t192 - M) < (t128 - M) ? 3 : 2;
  const int BMc = 64 * MI, mt = MI == 3 ? t192 : t128;
  if ((mt - M) * 8 > mt) return 0;
  // patch rows: the most any 128-position tile needs
  const int N = P.N;
  int rmax = 0;
  for (int n0 = 0; n0 < N; n0 += cp::BN) {
    const int pl = std::min(n0 + cp::BN, N) - 1;
    const int i0 = n0 / HW, i1 = pl / HW;
    if (i1 > i0 + 1) return 0;
    const int a0 = (n0 - i0 * HW) / OW;
    const int b0 = i1 == i0 ? (pl - i0 * HW) / OW : OH - 1;
    const int r = (b0 - a0 + KH) + (i1 == i0 ? 0 : (pl - i1 * HW) / OW + KH);
    rmax = std::max(rmax, r);
  }
  const int PW = d->width + 2 * d->pad_w;
  // channel stride: >= rmax * PW, with CPH * CS = 32 (mod 64) so the two lane
  // halves read disjoint bank halves
  int CS = rmax * PW;
  while ((CPH * CS) % 64 != 32) ++CS;
  const int pfl = 2 * CPH * CS;
  const int PD = pfl <= 1024 ? 4 : pfl <= 1536 ? 6 : pfl <= 2048 ? 8 : 0;
  if (PD == 0) return 0;
  if (KH == 5 && MI == 3 && PD != 4) return 0;  // LDS
  // repack the weights
  const int T = KH * KW, S = CPH * T, HP = (S + 3) / 4 * 4;
  const int RL = ((2 * HP / 4) % 2 == 0) ? 2 * HP + 4 : 2 * HP;
  const int tiles_m = mt / BMc, ktiles = Cg / (2 * CPH);
  const int64_t total = (int64_t)G * tiles_m * ktiles * BMc * RL;
  RRAM_REQUIRE(total * 4 < (1ll << 31), "conv: packed weights must be < 2 GiB");
  float* wp = pack_buffer(static_cast<size_t>(total), s);
  RRAM_REQUIRE(wp != nullptr, "conv: packed-weight buffer allocation failed");
  hipLaunchKernelGGL(k_conv_patch_pack, dim3(stream_blocks(total)), dim3(256), 0, s, w, wp, G, M, Cg, T, CPH, HP, RL,
                     BMc, tiles_m, ktiles, total);
  int rc = launch_status("conv weight pack");
  if (rc) return rc;
#define RRAM_P(KH_, CPH_, MI_, PD_) \
  if (KH == KH_ && MI == MI_ && PD == PD_) rc = launch_patch<KH_, KH_, CPH_, MI_, PD_>(P, wp, PW, CS, G, s); else
  RRAM_P(3, 2, 2, 4) RRAM_P(3, 2, 2, 6) RRAM_P(3, 2, 2, 8) RRAM_P(3, 2, 3, 4) RRAM_P(3, 2, 3, 6) RRAM_P(3, 2, 3, 8)
  RRAM_P(5, 1, 2, 4) RRAM_P(5, 1, 2, 6) RRAM_P(5, 1, 2, 8) RRAM_P(5, 1, 3, 4)
  return 0;
#undef RRAM_P
  return rc ? rc : 1;
}

// split-K factor of the fp32 implicit-GEMM convolution forward (1: none):
// ungrouped, M <= 64, K >= 256 and fewer than 256 output tiles of 32 or 64
// rows x 128 positions, split toward 1024 workgroups (512 / 2048 measured
// slower, profiles/r04_ab_conv_split.txt and the round-4 sweep of
// scripts/r04/gpu_r04_aq.sh) with >= 128 K per split
int conv_fwd_split(const rram_conv_desc* d, int M, int N, int K) {
  constexpr int target = 1024;
  if (d->group != 1 || M > 64 || K < 256) return 1;
  const int64_t tiles = (int64_t)((M + 31) / 32) * ((N + 127) / 128);
  if (tiles >= 256) return 1;
  int split = static_cast<int>((target + tiles - 1) / tiles);
  split = std::min(split, std::max(1, K / 128));
  return std::min(split, 16);
}

int conv_fwd_core(const rram_conv_desc* d, const float* x, const float* w, const float* bias,
                  float* y, int relu, hipStream_t s, int64_t y_img) {
  {
    WPack wk;
    wk.y_img = y_img;
    const int rc = conv_x6_fwd(d, x, nullptr, w, bias, y, nullptr, relu, s, wk);  // x6.hip
    if (rc != 0) return rc < 0 ? rc : RRAM_OK;
  }
  const int g = d->group;
  const int cin_g = d->channels / g, cout_g = d->num_output / g;
  const int K = cin_g * d->kernel_h * d->kernel_w;
  const int HoWo = d->out_h * d->out_w;
  Params P{};
  P.M = cout_g;
  P.N = d->num * HoWo;
  P.K = K;
  P.split = 1;
  P.k_chunk = K;
  P.a = make_view(w, K, cout_g, K);
  P.b = make_view(x, 0, P.N, K);
  ConvGeom& cv = P.cv;
  cv.C = cin_g;
  cv.H = d->height;
  cv.W = d->width;
  cv.KH = d->kernel_h;
  cv.KW = d->kernel_w;
  cv.ph = d->pad_h;
  cv.pw = d->pad_w;
  cv.sh = d->stride_h;
  cv.sw = d->stride_w;
  cv.dh = d->dilation_h;
  cv.dw = d->dilation_w;
  cv.Ho = d->out_h;
  cv.Wo = d->out_w;
  cv.khkw = make_fastdiv(d->kernel_h * d->kernel_w);
  cv.kw_div = make_fastdiv(d->kernel_w);
  cv.howo = make_fastdiv(HoWo);
  cv.wo_div = make_fastdiv(d->out_w);
  cv.chw = (int64_t)d->channels * d->height * d->width;
  RRAM_REQUIRE((int64_t)d->num * cv.chw * 4 < (1ll << 31), "conv2d_fwd: input must be < 2 GiB (32-bit buffer offsets)");
  cv.in_bytes = static_cast<int>((int64_t)d->num * cv.chw * 4);
  P.e = make_epi(y, HoWo, 1.0f, 0.0f, bias, RRAM_BIAS_ROW, relu);
  P.e.cimg = y_img > 0 ? y_img : (int64_t)d->num_output * HoWo;
  P.e.hw = make_fastdiv(HoWo);
  P.grp_a = (int64_t)cout_g * K;
  P.grp_b = (int64_t)cin_g * d->height * d->width;
  P.grp_c = (int64_t)cout_g * HoWo;
  P.grp_bias = cout_g;
  {
    const int rc = conv_patch_fwd(d, w, P, s);
    if (rc != 0) return rc < 0 ? rc : RRAM_OK;
  }
  // table-driven gather when the taps fit the 31-bit (or 63-bit) validity mask (or no padding)
  const bool padded = d->pad_h > 0 || d->pad_w > 0;
  const int taps = d->kernel_h * d->kernel_w;
  const bool wide = padded && taps > 31;
  int bmode = CONV;
  if ((!padded || taps <= 63) &&
      (int64_t)cin_g * d->height * d->width * 4 < (1ll << 31)) {
    cv.tbl = conv_table(cv, K, padded, wide, s);
    cv.taps = padded ? taps : 0;
    if (cv.tbl) bmode = wide ? CONVT64 : CONVT;
  }
  // A: 16-byte loads when the rows are 16-byte aligned; else (K % 4 != 0) the
  // unaligned raw-buffer form for the table gather
  int amode = vec_ok(w, K, K, P.grp_a) ? KCV : KC;
  if (amode == KC && bmode == CONVT && (reinterpret_cast<uintptr_t>(w) & 3u) == 0 &&
      (int64_t)g * cout_g * K * 4 < (1ll << 31))
    amode = KCU;
  // thin, short-grid convolutions (CIFAR-10 conv2 / conv3, LeNet conv2 at
  // batch 100: M = 32..64, a few hundred K, 50-200 tiles of 32/64 x 128) leave
  // most CUs idle for K / KB serial K-tiles: split K toward ~1024 workgroups,
  // partials summed in order by k_splitk_reduce_nchw
  {
    const int split = conv_fwd_split(d, P.M, P.N, K);
    if (split > 1) {
      const int kb = conv_kb(K);
      const int kc = ((K + split - 1) / split + kb - 1) / kb * kb;
      const int sp = (K + kc - 1) / kc;
      float* ws = stream_buffer(1, (size_t)sp * P.M * P.N, s);
      RRAM_REQUIRE(ws != nullptr, "conv2d_fwd: split-K buffer allocation failed");
      P.split = sp;
      P.k_chunk = kc;
      P.ws = ws;
      int rc = dispatch(amode, bmode, OUT_NCHW, P, sp, s);
      if (rc) return rc;
      hipLaunchKernelGGL(k_splitk_reduce_nchw, dim3(stream_blocks((int64_t)P.M * P.N)), dim3(256), 0, s, ws, sp, P.M,
                         P.N, P.e);
      return launch_status("conv fwd split-K reduce");
    }
  }
  return dispatch(amode, bmode, OUT_NCHW, P, g, s);
}

// Split-K factor of the weight-gradient GEMM: M = Cout/g and N = Cin/g*kh*kw
// are small while K = images*Ho*Wo is long (CIFAR conv1: 32 x 75 x 102400),
// so without a split the grid is a couple of blocks.  Aim for ~1024 blocks of
// 64 x 64 (or 128 x 128) tiles with >= 512 K per split, <= 64 splits and
// <= 256 MB of partials.
// Rounds 3-4 capped it at 64 splits of >= 512 K; the partials' reduce is
// cheap since k_splitk_reduce_wave, so the split goes to 256 with >= 256 K
// per split (CIFAR-10 conv1's dW: 128 -> 512 workgroups; cap / min-K sweep in
// profiles/r04_ab_tail_batched.txt)
int bwd_weight_split(int M, int N, int64_t K) {
  constexpr int cap = 256, mink = 256;
  const int64_t t = (M <= 64 || N <= 64) ? (int64_t)((M + 63) / 64) * ((N + 63) / 64)
                                         : (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  int64_t sp = 1024 / (t > 0 ? t : 1);
  if (sp > cap) sp = cap;
  while (sp > 1 && K / sp < mink) --sp;
  while (sp > 1 && sp * M * N * 4 > (256ll << 20)) --sp;
  return static_cast<int>(sp < 1 ? 1 : sp);
}

// dW_g[co][k] += sum_p dY_g[co][p] col_g[k][p]   (col: [Cin*kh*kw][ldcol]);
// part (nullable): part_bytes of split-K partials (see bwd_weight_split)
// db (nullable; ungrouped only, part required): the bias gradient as one more
// GEMM column against the ones row im2col_core wrote after the K column rows,
// always split (>= 2), the reduce routing column K to db
// The weight gradient with the column matrix gathered inside the GEMM (IM2T,
// no im2col pass and no column buffer): dW_g[co][k] += sum_p dY_g[co][p]
// x_g[k, p] over all d->num images; db (group 1 only) as the ones row's
// column of the same split GEMM.  part: the split-K partials (required:
// these are long-K GEMMs); 0 when not covered (the caller falls back to the
// column path), < 0 on error.  The same K-tiles, split and element values as
// the im2col + KC path, so the same bits.
bool conv_bwd_weight_im2t_ok(const rram_conv_desc* d, size_t part_bytes) {
  const int g = d->group;
  const int cout_g = d->num_output / g, K = d->channels / g * d->kernel_h * d->kernel_w;
  const int64_t P_all = (int64_t)d->num * d->out_h * d->out_w;
  const int64_t in_elems = (int64_t)d->num * d->channels * d->height * d->width;
  return P_all >= 2 * BK && P_all < (1ll << 31) && in_elems * 4 < (1ll << 31) && K + 1 < (1 << 24) &&
         (d->kernel_h - 1) * d->dilation_h < 32768 && (d->kernel_w - 1) * d->dilation_w < 32768 &&
         part_bytes >= 2 * (size_t)cout_g * (K + 1) * sizeof(float);
}
int conv_bwd_weight_im2t(const rram_conv_desc* d, const float* x, const float* dy, float* dw, float* db, void* part,
                         size_t part_bytes, hipStream_t s) {
  const int g = d->group;
  const int cin_g = d->channels / g, cout_g = d->num_output / g;
  const int K = cin_g * d->kernel_h * d->kernel_w;
  const int HoWo = d->out_h * d->out_w;
  const int64_t P_all = (int64_t)d->num * HoWo;
  const int64_t in_elems = (int64_t)d->num * d->channels * d->height * d->width;
  RRAM_REQUIRE(part != nullptr && conv_bwd_weight_im2t_ok(d, part_bytes) && (db == nullptr || g == 1),
               "conv bwd weight (gathered): shape or workspace not covered");
  ConvGeom cv{};
  cv.C = cin_g;
  cv.H = d->height;
  cv.W = d->width;
  cv.KH = d->kernel_h;
  cv.KW = d->kernel_w;
  cv.ph = d->pad_h;
  cv.pw = d->pad_w;
  cv.sh = d->stride_h;
  cv.sw = d->stride_w;
  cv.dh = d->dilation_h;
  cv.dw = d->dilation_w;
  cv.Ho = d->out_h;
  cv.Wo = d->out_w;
  cv.howo = make_fastdiv(HoWo);
  cv.wo_div = make_fastdiv(d->out_w);
  cv.chw = (int64_t)d->channels * d->height * d->width;
  cv.tbl = im2t_table(cv, K, db != nullptr, 256, s);
  RRAM_REQUIRE(cv.tbl != nullptr, "conv bwd weight: gather table allocation failed");
  const int N = K + (db ? 1 : 0);
  for (int gi = 0; gi < g; ++gi) {
    Params P{};
    P.M = cout_g;
    P.N = N;
    P.K = static_cast<int>(P_all);
    P.a = make_view(dy + (int64_t)gi * cout_g * HoWo, HoWo, cout_g, P.K);
    P.a.img = (int64_t)d->num_output * HoWo;
    P.a.hw = make_fastdiv(HoWo);
    P.b = make_view(x + (int64_t)gi * cin_g * d->height * d->width, 0, N, P.K);
    P.cv = cv;
    P.cv.in_bytes = static_cast<int>((in_elems - (int64_t)gi * cin_g * d->height * d->width) * 4);
    P.e = make_epi(dw + (int64_t)gi * cout_g * K, K, 1.0f, 1.0f, nullptr, 0, 0);
    int split = std::max(2, bwd_weight_split(P.M, P.N, P.K));
    while (split > 2 && (size_t)split * P.M * P.N * sizeof(float) > part_bytes) --split;
    int chunk = (P.K + split - 1) / split;
    chunk = (chunk + BK - 1) / BK * BK;
    split = (P.K + chunk - 1) / chunk;
    RRAM_REQUIRE(split >= 2 && (size_t)split * P.M * P.N * sizeof(float) <= part_bytes,
                 "conv bwd weight (gathered): split-K partials do not fit");
    P.split = split;
    P.k_chunk = chunk;
    P.ws = static_cast<float*>(part);
    int rc = dispatch(NCHW, IM2T, OUT_ROWMAJOR, P, split, s, true);
    if (rc) return rc;
    if (split >= 32)
      hipLaunchKernelGGL(k_splitk_reduce_wave, dim3(static_cast<unsigned>(((int64_t)P.M * P.N + 3) / 4)), dim3(256), 0,
                         s, P.ws, split, P.M, K, P.N, P.e.C, db);
    else if (db)
      hipLaunchKernelGGL(k_splitk_reduce_dwdb, dim3(stream_blocks((int64_t)P.M * P.N)), dim3(256), 0, s, P.ws, split,
                         P.M, K, P.e.C, db);
    else
      hipLaunchKernelGGL(k_splitk_reduce, dim3(stream_blocks((int64_t)P.M * P.N)), dim3(256), 0, s, P.ws, split,
                         P.M, P.N, P.e);
    rc = launch_status("conv bwd weight (gathered) split-K reduce");
    if (rc) return rc;
  }
  return RRAM_OK;
}

int conv_bwd_weight_core(const rram_conv_desc* d, int nimg, const float* dy, const float* col,
                         int64_t ldcol, float* dw, void* part, size_t part_bytes, hipStream_t s, float* db) {
  const int g = d->group;
  const int cin_g = d->channels / g, cout_g = d->num_output / g;
  const int K = cin_g * d->kernel_h * d->kernel_w;
  const int HoWo = d->out_h * d->out_w;
  RRAM_REQUIRE(db == nullptr || (g == 1 && part != nullptr), "conv bwd weight: folded bias needs group 1 + partials");
  if (db) {
    Params P{};
    P.M = cout_g;
    P.N = K + 1;
    P.K = nimg * HoWo;
    P.a = make_view(dy, HoWo, cout_g, P.K);
    P.a.img = (int64_t)d->num_output * HoWo;
    P.a.hw = make_fastdiv(HoWo);
    P.b = make_view(col, ldcol, K + 1, P.K);
    P.e = make_epi(dw, K, 1.0f, 1.0f, nullptr, 0, 0);
    const int bm = vec_ok(P.b.p, ldcol, P.K) ? KCV : KC;
    int split = std::max(2, bwd_weight_split(P.M, P.N, P.K));
    while (split > 2 && (size_t)split * P.M * P.N * sizeof(float) > part_bytes) --split;
    int chunk = (P.K + split - 1) / split;
    chunk = (chunk + BK - 1) / BK * BK;
    split = (P.K + chunk - 1) / chunk;
    RRAM_REQUIRE(split >= 2 && (size_t)split * P.M * P.N * sizeof(float) <= part_bytes,
                 "conv bwd weight: folded bias needs >= 2 K splits");
    P.split = split;
    P.k_chunk = chunk;
    P.ws = static_cast<float*>(part);
    int rc = dispatch(NCHW, bm, OUT_ROWMAJOR, P, split, s, true);
    if (rc) return rc;
    if (split >= 32)
      hipLaunchKernelGGL(k_splitk_reduce_wave, dim3(static_cast<unsigned>(((int64_t)P.M * P.N + 3) / 4)), dim3(256), 0,
                         s, P.ws, split, P.M, K, P.N, dw, db);
    else
      hipLaunchKernelGGL(k_splitk_reduce_dwdb, dim3(stream_blocks((int64_t)P.M * P.N)), dim3(256), 0, s, P.ws, split,
                         P.M, K, dw, db);
    return launch_status("conv bwd weight + bias split-K reduce");
  }
  for (int gi = 0; gi < g; ++gi) {
    Params P{};
    P.M = cout_g;
    P.N = K;
    P.K = nimg * HoWo;
    P.split = 1;
    P.k_chunk = P.K;
    P.a = make_view(dy + (int64_t)gi * cout_g * HoWo, HoWo, cout_g, P.K);
    P.a.img = (int64_t)d->num_output * HoWo;
    P.a.hw = make_fastdiv(HoWo);
    P.b = make_view(col + (int64_t)gi * K * ldcol, ldcol, K, P.K);
    P.e = make_epi(dw + (int64_t)gi * cout_g * K, K, 1.0f, 1.0f, nullptr, 0, 0);
    const int bm = vec_ok(P.b.p, ldcol, P.K) ? KCV : KC;
    int split = part ? bwd_weight_split(P.M, P.N, P.K) : 1;
    while (split > 1 && (size_t)split * P.M * P.N * sizeof(float) > part_bytes) --split;
    if (split > 1) {
      int chunk = (P.K + split - 1) / split;
      chunk = (chunk + BK - 1) / BK * BK;
      split = (P.K + chunk - 1) / chunk;
      P.split = split;
      P.k_chunk = chunk;
      P.ws = static_cast<float*>(part);
      int rc = dispatch(NCHW, bm, OUT_ROWMAJOR, P, split, s, true);
      if (rc) return rc;
      // dw += sum of the partials (beta = 1), fixed summation order
      if (split >= 32)  // (dw of group gi: P.e.C)
        hipLaunchKernelGGL(k_splitk_reduce_wave, dim3(static_cast<unsigned>(((int64_t)P.M * P.N + 3) / 4)), dim3(256),
                           0, s, P.ws, split, P.M, P.N, P.N, P.e.C, nullptr);
      else
        hipLaunchKernelGGL(k_splitk_reduce, dim3(stream_blocks((int64_t)P.M * P.N)), dim3(256), 0, s, P.ws, split,
                           P.M, P.N, P.e);
      rc = launch_status("conv bwd weight split-K reduce");
      if (rc) return rc;
      continue;
    }
    const int rc = dispatch(NCHW, bm, OUT_ROWMAJOR, P, 1, s);
    if (rc) return rc;
  }
  return RRAM_OK;
}

// dcol_g[k][p] = sum_co W_g[co][k] dY_g[co][p]
int conv_bwd_data_col_core(const rram_conv_desc* d, int nimg, const float* w, const float* dy,
                           float* col, int64_t ldcol, hipStream_t s) {
  const int g = d->group;
  const int cin_g = d->channels / g, cout_g = d->num_output / g;
  const int K = cin_g * d->kernel_h * d->kernel_w;
  const int HoWo = d->out_h * d->out_w;
  for (int gi = 0; gi < g; ++gi) {
    Params P{};
    P.M = K;
    P.N = nimg * HoWo;
    P.K = cout_g;
    P.split = 1;
    P.k_chunk = P.K;
    P.a = make_view(w + (int64_t)gi * cout_g * K, K, K, cout_g);  // RC: A(k_row, co) = W[co*K + k]
    P.b = make_view(dy + (int64_t)gi * cout_g * HoWo, HoWo, P.N, cout_g);
    P.b.img = (int64_t)d->num_output * HoWo;
    P.b.hw = make_fastdiv(HoWo);
    P.e = make_epi(col + (int64_t)gi * K * ldcol, ldcol, 1.0f, 0.0f, nullptr, 0, 0);
    const int rc = dispatch(RC, NCHWT, OUT_ROWMAJOR, P, 1, s);
    if (rc) return rc;
  }
  return RRAM_OK;
}

int im2col_core(const float* im, int64_t im_img, int nimg, const rram_conv_desc* d, float* col,
                int64_t ldcol, hipStream_t s, int ones_row) {
  const int64_t total = (int64_t)nimg * d->channels * d->kernel_h * d->kernel_w * d->out_h * d->out_w;
  if (total == 0) return RRAM_OK;
  // ones_row: one more row of 1.0 after the Cin*kh*kw column rows
  const int rows = d->channels * d->kernel_h * d->kernel_w + (ones_row ? 1 : 0);
  const int64_t P = (int64_t)nimg * d->out_h * d->out_w;
  RRAM_REQUIRE(P < (1ll << 31) && (int64_t)nimg * im_img < (1ll << 31) && rows < 65536,
               "im2col: more than 2^31 positions / input elements or 65535 rows is not supported");
  if ((d->out_h * d->out_w) % 4 == 0 && ldcol % 4 == 0 && (reinterpret_cast<uintptr_t>(col) & 15u) == 0) {
    const int gx4 = static_cast<int>(std::min<int64_t>((P / 4 + 255) / 256, 64));
    hipLaunchKernelGGL(k_im2col4, dim3(gx4, rows), dim3(256), 0, s, im, im_img, nimg,
                       d->channels, d->height, d->width, d->kernel_h, d->kernel_w, d->pad_h,
                       d->pad_w, d->stride_h, d->stride_w, d->dilation_h, d->dilation_w, d->out_h,
                       d->out_w, col, ldcol, make_fastdiv(d->out_h * d->out_w), make_fastdiv(d->out_w));
    return launch_status("im2col");
  }
  const int gx = static_cast<int>(std::min<int64_t>((P + 255) / 256, 64));
  hipLaunchKernelGGL(k_im2col, dim3(gx, rows), dim3(256), 0, s, im, im_img, nimg,
                     d->channels, d->height, d->width, d->kernel_h, d->kernel_w, d->pad_h,
                     d->pad_w, d->stride_h, d->stride_w, d->dilation_h, d->dilation_w, d->out_h,
                     d->out_w, col, ldcol, make_fastdiv(d->out_h * d->out_w), make_fastdiv(d->out_w));
  return launch_status("im2col");
}

int col2im_core(const float* col, int64_t ldcol, int nimg, const rram_conv_desc* d, float* im,
                int64_t im_img, int accumulate, hipStream_t s) {
  const int64_t total = (int64_t)nimg * d->channels * d->height * d->width;
  if (total == 0) return RRAM_OK;
  hipLaunchKernelGGL(k_col2im, dim3(stream_blocks(total)), dim3(256), 0, s, col, ldcol, nimg,
                     d->channels, d->height, d->width, d->kernel_h, d->kernel_w, d->pad_h,
                     d->pad_w, d->stride_h, d->stride_w, d->dilation_h, d->dilation_w, d->out_h,
                     d->out_w, im, im_img, accumulate);
  return launch_status("col2im");
}

int gemv_core(int trans, int M, int N, float alpha, const float* A, const float* x, float beta,
              float* y, hipStream_t s) {
  RRAM_REQUIRE(M >= 0 && N >= 0, "gemv: negative size");
  const int outs = trans ? N : M;
  if (outs == 0) return RRAM_OK;
  RRAM_REQUIRE(A && x && y, "gemv: NULL");
  const int blocks = (outs + 3) / 4 < 2048 ? (outs + 3) / 4 : 2048;
  hipLaunchKernelGGL(k_gemv, dim3(blocks), dim3(256), 0, s, trans, M, N, alpha, A, x, beta, y);
  return launch_status("gemv");
}

}  // namespace rram
