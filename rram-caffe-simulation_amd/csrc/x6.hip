// Convolution forward with fp32 products on the bf16 matrix cores
// (RRAM_ENGINE_BF16X6, include/rram_kernels.h): the LDS-patch convolution of
// gemm.hip's k_conv_patch re-tiled for v_mfma_f32_32x32x16_bf16.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <type_traits>

#include "gemm_common.hpp"
#include "split3.hpp"

namespace rram {
namespace {

// ---------------------------------------------------------------------------
// k_conv_patch_x6: the patch convolution with each fp32 product formed on the
// bf16 matrix cores.  Every fp32 operand is split exactly into three bf16
// terms, x = xh + xm + xl (round-to-nearest at each step; the remainders are
// exact in fp32 and the third term holds the last 8 significand bits), and
// a*b is accumulated in fp32 as the six terms
//   al*bh + ah*bl + am*bm + am*bh + ah*bm + ah*bh
// (v_mfma_f32_32x32x16_bf16: a product of two bf16 is exact in fp32).  The
// dropped terms am*bl, al*bm, al*bl are at most 2^-24, 2^-24, 2^-32 |a*b| with independent
// signs, under the fp32 rounding of the accumulation itself, so the result
// carries fp32 accuracy (tests compare it with a float64 evaluation at the
// same bound as the fp32-MFMA kernels) while a 32x32x16 bf16 MFMA does the
// work of eight 32x32x2 fp32 MFMAs in half their cycles: six of them cost
// 192 cycles where the fp32 form of the same 32x32x16 block costs 512.
// The weights are split once per call by the repack kernel (three bf16
// planes, fragment order); the activations are split in registers after the
// LDS reads of the patch (4-5 VALU per element, hidden between MFMAs).
// K order: a K-tile holds 2 CPH input channels (half h: channels
// kt*2CPH + h*CPH + cc) x KH*KW taps = S steps per half, padded to G8 groups
// of 8; MFMA group g takes steps 8g .. 8g+7 of both halves (lane half h holds
// k = 8h + j of the 32x32x16 operand).  Padded steps have zero weights and
// read no activations.
// RRAM_X6_DROP = k (1..5) leaves out the k-th product below.  Guard
// validation only (profiles/r04_fp32_guard.txt: a build with a term dropped
// must fail tests/test_gpu_fp32_guard.py); the product build has it 0.
#ifndef RRAM_X6_DROP
#define RRAM_X6_DROP 0
#endif
namespace x6 {
__device__ __forceinline__ floatx16 mfma6(const Parts& a, const Parts& b, floatx16 c) {
  if (RRAM_X6_DROP != 1) c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.l, b.h, c, 0, 0, 0);
  if (RRAM_X6_DROP != 2) c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.l, c, 0, 0, 0);
  if (RRAM_X6_DROP != 3) c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.m, c, 0, 0, 0);
  if (RRAM_X6_DROP != 4) c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.h, c, 0, 0, 0);
  if (RRAM_X6_DROP != 5) c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.m, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.h, c, 0, 0, 0);
}
template <int KH, int KW, int CPH>
struct Shape {
  static constexpr int T = KH * KW;
  static constexpr int S = CPH * T;         // steps per half
  static constexpr int G8 = (S + 7) / 8;    // MFMA groups per K-tile
  static constexpr int RLB = G8 * 96 + 16;  // bytes per packed weight row ([g][half][term][8 bf16] + pad: RLB/16 odd)
};
constexpr int BN = 256;  // workgroup tile columns (rows: 32 MI, MI = 3 | 4)
}  // namespace x6

template <int KH, int KW, int CPH, int MI, int PD>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_conv_patch_x6(Params P, const uint16_t* __restrict__ wpack, int PW, int CS) {
  using namespace g2;
  using Sh = x6::Shape<KH, KW, CPH>;
  // 32 MI x 256 tile; wave w owns all 32 MI rows x columns 64 w .. 64 w + 63,
  // so the B split (the VALU of the main loop) is shared by MI row blocks and
  // each weight byte staged in LDS feeds 256 columns
  constexpr int BMc = 32 * MI, BNc = x6::BN;
  constexpr int A_B = BMc * Sh::RLB;                    // weight slab bytes per K-tile
  constexpr int A_DMA = ((A_B + 1023) / 1024 + 3) / 4;  // 1 KB pieces per wave
  constexpr int A_REGB = A_DMA * 4 * 1024;
  constexpr int SFB = A_REGB + PD * 4 * 64 * 4;         // stage bytes (weights + patch)
  constexpr int NVM = A_DMA + PD;
  constexpr int G8 = Sh::G8;
  static_assert(2 * SFB <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[2 * SFB];
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem));

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lr = lane & 31, lh = lane >> 5;

  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, loc = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int tid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int tm = __builtin_amdgcn_readfirstlane(tid % P.tiles_m);
  const int tn = __builtin_amdgcn_readfirstlane((tid / P.tiles_m) % P.tiles_n);
  const int z = __builtin_amdgcn_readfirstlane(tid / (P.tiles_m * P.tiles_n));
  const int n0 = tn * BNc;
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
  const uint16_t* abase = wpack + ((int64_t)z * P.tiles_m + tm) * ktiles * (A_B / 2);
  const int4v arsrc = make_rsrc(reinterpret_cast<const float*>(abase), static_cast<uint32_t>((int64_t)ktiles * A_B));
  uint32_t aoff[A_DMA];
#pragma unroll
  for (int i = 0; i < A_DMA; ++i) {
    const int f = ((wave * A_DMA + i) * 64 + lane) * 16;
    aoff[i] = f < A_B ? static_cast<uint32_t>(f) : 0x80000000u;
  }

  // patch: positions n0 .. plast cover images img0 .. img0 + nseg - 1 (<= 3);
  // segment s holds output rows f_s .. l_s of its image plus the KH - 1 halo,
  // at patch rows p_s .. p_{s+1} - 1
  const int plast = min(n0 + BNc, P.N) - 1;
  const int img0 = n0 / HW, nseg = plast / HW - img0 + 1;
  const int f0 = (n0 - img0 * HW) / OW;
  auto seg_last = [&](int s) { return s == nseg - 1 ? (plast - (img0 + s) * HW) / OW : cv.Ho - 1; };
  const int p1 = seg_last(0) - f0 + KH;
  const int p2 = p1 + (nseg > 1 ? seg_last(1) + KH : 0);
  const int R = p2 + (nseg > 2 ? seg_last(2) + KH : 0);
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
      const int sg = prow >= p2 ? 2 : prow >= p1 ? 1 : 0;
      const int y = (sg == 0 ? f0 + prow : prow - (sg == 1 ? p1 : p2)) - cv.ph;
      const int x = pcol - cv.pw;
      if (y >= 0 && y < cv.H && x >= 0 && x < cv.W)
        off = static_cast<uint32_t>((int64_t)(img0 + sg) * cv.chw * 4) + static_cast<uint32_t>(ch) * HW4 +
              static_cast<uint32_t>((y * cv.W + x) * 4);
    }
    poff[i] = off;
  }
  int pb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = min(n0 + wave * 64 + j * 32 + lr, plast);
    const int img = n / HW, sp = n - img * HW;
    const int oh = sp / OW, ow = sp - oh * OW;
    const int sg = img - img0;
    const int prow = sg == 0 ? oh - f0 : (sg == 1 ? p1 : p2) + oh;
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
    const uint32_t img = lds0 + static_cast<uint32_t>(stg * SFB);
    if (e < A_DMA) {
      dma_b128(arsrc, aoff[e] + static_cast<uint32_t>(kt * A_B), img + static_cast<uint32_t>((wave * A_DMA + e) * 1024));
    } else {
      const int i = e - A_DMA;
      dma_b32(xrsrc, poff[i] + static_cast<uint32_t>(kt * 2 * CPH) * HW4,
              img + static_cast<uint32_t>(A_REGB + (wave * PD + i) * 64 * 4));
    }
  };
  // weight fragments (this lane's 8 k of rows 32 i + lr: high, middle, low
  // terms) are single-buffered: row block i of the next group is read as soon
  // as both column blocks of the current group have consumed it
  x6::bf16x8 fa[MI][3];
  struct Fr {
    float b[2][8];        // raw activations of columns j
    x6::Parts bp[2];      // their split
  };
  auto read_a = [&](const char* st, int g, int i) {
    const char* p = st + (i * 32 + lr) * Sh::RLB + (g * 2 + lh) * 48;
#pragma unroll
    for (int t = 0; t < 3; ++t) fa[i][t] = *reinterpret_cast<const x6::bf16x8*>(p + 16 * t);
  };
  auto read_b = [&](Fr& F, const char* st, int g) {
    const float* pt = reinterpret_cast<const float*>(st + A_REGB);
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int sx = 8 * g + jj;
      if (sx < Sh::S) {
        const int cc = sx / Sh::T, tp = sx - cc * Sh::T, kh = tp / KW, kw = tp - kh * KW;
#pragma unroll
        for (int j = 0; j < 2; ++j) F.b[j][jj] = pt[pb[j] + cc * CS + kh * PW + kw];
      } else {
#pragma unroll
        for (int j = 0; j < 2; ++j) F.b[j][jj] = 0.0f;
      }
    }
  };

  const int nt = ktiles;  // >= 1 (host)
  // fragments ping-pong between F[0] and F[1] by group parity (compile-time
  // indices, no register copies); with an odd group count tiles go in pairs
  Fr F[2];
#pragma unroll
  for (int e = 0; e < NVM; ++e) issue(0, 0, e);
  wait_vm<0>();
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int i = 0; i < MI; ++i) read_a(smem, 0, i);
  read_b(F[0], smem, 0);
#pragma unroll
  for (int j = 0; j < 2; ++j) x6::split8_safe(F[0].b[j], F[0].bp[j]);

  // one K-tile; PAR: parity of its first group's fragments; MORE: tile t + 1 exists
  auto tile = [&](int t, auto par_c, auto more_c) {
    constexpr int PAR = decltype(par_c)::value;
    constexpr bool MORE = decltype(more_c)::value;
    const char* cur = smem + (t & 1) * SFB;
    const char* nxt = smem + ((t + 1) & 1) * SFB;
#pragma unroll
    for (int g = 0; g < G8; ++g) {
      Fr& fc = F[(g + PAR) & 1];
      Fr& fn = F[(g + 1 + PAR) & 1];
      const bool last = g == G8 - 1;
      // the next group's fragments: this tile's group g + 1, or group 0 of
      // tile t + 1 once its DMA has landed (wait + barrier: every wave is then
      // also done reading the stage the next DMA overwrites)
      if (last && MORE) {
        wait_vm<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
      const bool rd = !last || MORE;
      const char* src = last ? nxt : cur;
      const int gn = last ? 0 : g + 1;
      constexpr int NB = 2 * MI;  // MFMA blocks (6 MFMAs each) of a group
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const int i = q >> 1, j = q & 1;
        acc[i][j] = x6::mfma6(x6::Parts{fa[i][0], fa[i][1], fa[i][2]}, fc.bp[j], acc[i][j]);
        if (rd) {
          if (q == 0) read_b(fn, src, gn);
          if (j == 1) read_a(src, gn, i);
          if (q == NB - 3) x6::split8_safe(fn.b[0], fn.bp[0]);
          if (q == NB - 1) x6::split8_safe(fn.b[1], fn.bp[1]);
        }
        // DMA of tile t + 1 spread over the blocks of groups 0 .. G8-2
        if (!last && MORE) {
          constexpr int SL = (G8 - 1) * NB;
          const int sl = g * NB + q;
#pragma unroll
          for (int e = 0; e < NVM; ++e)
            if ((e * SL) / NVM == sl) issue(t + 1, (t + 1) & 1, e);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  if constexpr (G8 % 2 == 0) {
    int t = 0;
    for (; t + 1 < nt; ++t) tile(t, P0{}, T_{});
    tile(t, P0{}, F_{});
  } else {
    int t = 0;
    for (; t + 2 < nt; t += 2) {
      tile(t, P0{}, T_{});
      tile(t + 1, P1{}, T_{});
    }
    if (t + 1 < nt) {
      tile(t, P0{}, T_{});
      tile(t + 1, P1{}, F_{});
    } else {
      tile(t, P0{}, F_{});
    }
  }
  conv_epilogue_nchw<MI, 2>(acc, P, ep, m0, n0 + wave * 64, lr, lh);
}


// ---------------------------------------------------------------------------
// k_conv_cb_x6: stride-1 KH x KW convolution on the bf16x6 engine with the
// activations split ONCE, outside the main loop, into a channel-octet layout
// (k_pack_octets_x6: [img][C/8][H][W][term][8 channels] bf16), so the main
// loop does no VALU split and no per-element gather: every B fragment term is
// one ds_read_b128 of 8 channels at one tap, and a K-tile is 16 channels x
// all KH*KW taps (no padded steps; k_conv_patch_x6 pads 5x5's 25 taps to 32).
// K order: MFMA group (kt, s) = channels 16 kt .. 16 kt + 15 at tap s; lane
// half h holds channel octet 2 kt + h.
// Tile 32 WR x 32 NB (4 / WR): wave w owns rows 32 (w % WR) .. + 31 and
// columns 32 NB (w / WR) .. + 32 NB - 1.  Its weight fragments (pre-split and
// fragment-ordered by k_conv_cb_pack_x6, 3 KB per group) come straight from
// L2 into registers one group ahead; the input patch of a K-tile (both
// octet planes, R rows x RPC 16-byte chunks) is LDS-DMA'd into a 2-stage
// ring, one barrier per K-tile.  A position is 3 16-byte chunks; the patch
// row pitch RPC (chunks) is >= 3 PW with RPC = 3 OW (mod 16), so the chunk of
// output column n is 3 n (mod 16) and the 16 consecutive columns of a
// ds_read_b128 lane group hit 16 disjoint bank quads (across row wraps too).  Per group a wave issues NB x 6 MFMAs, 3 NB ds_read_b128 and 3
// global loads: the loop is MFMA-paced.
namespace cbx6 {
constexpr int FRAG = 3 * 64;  // bf16x8 units per pre-split weight fragment (3 terms x 64 lanes)
// Patch segment shift (chunks).  Within one image's rows the B column n of a
// lane group sits at chunk 3 n + const (mod 16) (RPC = 3 OW mod 16), so the 16
// lanes of a ds_read_b128 group hit 16 bank quads.  The next image's segment
// starts KH halo rows later, which breaks that sequence (AlexNet conv3 / conv4:
// 14 % of the B reads' LDS cycles were 2-way conflicts); shifting segment s by
// s * dlt chunks restores it: dlt = 3 OW (1 - KH) (mod 16).  The gap chunks
// hold nothing (their DMA lanes load out of range: zero).  The host sizes the
// octet plane for the two shifts (up to 30 chunks).
__device__ __forceinline__ int seg_shift(int OW, int KH) { return (3 * OW * (1 - KH)) & 15; }
// column n of a lane past the tile's last position: the same column mod 16
// inside the tile (its value is never stored), so a lane group keeps 16
// distinct bank quads (clamping to plast made them collide in short tiles)
__device__ __forceinline__ int clamp_col(int n, int n0, int plast) {
  return n <= plast ? n : max(n0, n - (((n - plast) + 15) & ~15));
}
// first patch piece of K-tile kt + 1 staged at tap s (pieces spread evenly
// over taps 0 .. T - 2)
constexpr int piece_lo(int s, int PD, int T) { return s >= T - 1 ? PD : (s * PD + T - 2) / (T - 1); }
// the same over taps 0 .. T - 1 - SD (pieces loaded at tap s, stored at s + SD)
constexpr int piece_lo_d(int s, int PD, int T, int SD) { return s >= T - SD ? PD : (s * PD + T - SD - 1) / (T - SD); }
}  // namespace cbx6

// The loop's global reads are compiler-visible register loads: weights
// straight into the fragment registers one group ahead, patch pieces into
// staging registers, written to LDS one tap later.  (An LDS-DMA weight ring
// with hand-counted vmcnt measured slower: each DMA piece costs ~100 cycles
// of issue among the MFMAs, and the ring paid 3 per group.)
template <int KH, int KW, int WR, int NB, int PD, int OCC>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC)))
k_conv_cb_x6(Params P, const x6::bf16x8* __restrict__ wpack, const uint16_t* __restrict__ xpack, int octb, int rpc,
             uint32_t xrange, int ximg, char* __restrict__ yoct, int cout8, FastDiv oct_div, FastDiv rpc_div,
             int tpi) {
  using namespace g2;
  constexpr int T = KH * KW, WC = 4 / WR, BMc = 32 * WR, BNc = 32 * NB * WC, SFB = PD * 4 * 1024;
  static_assert(2 * SFB <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[2 * SFB];
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem));

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int wr = wave % WR, wc = wave / WR;

  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, loc = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int tid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int tm = __builtin_amdgcn_readfirstlane(tid % P.tiles_m);
  const int tn = __builtin_amdgcn_readfirstlane((tid / P.tiles_m) % P.tiles_n);
  const int z = __builtin_amdgcn_readfirstlane(tid / (P.tiles_m * P.tiles_n));
  const int m0 = tm * BMc;

  const ConvGeom& cv = P.cv;
  const int HW = cv.howo.d, OW = cv.wo_div.d;
  // tpi > 0: per-image tiles (tpi of them per image, the last one short), so
  // no tile spans two images and the patch carries one halo (the 5 x 5 patch
  // then fits the LDS of two workgroups per CU); tpi = 0: tiles of BNc
  // consecutive positions across images
  const int timg = tpi > 0 ? tn / tpi : 0;
  const int tpc = cv.tpitch > 0 ? cv.tpitch : BNc;  // positions per tile
  const int n0 = tpi > 0 ? timg * HW + (tn - timg * tpi) * tpc : tn * tpc;
  const int KT = cv.C >> 4;                      // K-tiles of 16 channels (>= 1, host)
  const uint32_t PL = static_cast<uint32_t>(cv.H * cv.W * 48);  // bytes per octet plane of the packed input
  Epi ep = P.e;
  if (z > 0) {
    ep.C += z * P.grp_c;
    if (ep.bias) ep.bias += z * P.grp_bias;
  }
  // this group's octets start at octet z C/8 of every image
  const uint16_t* xg = xpack + (int64_t)z * (cv.C >> 3) * (PL >> 1);
  const int4v xrsrc = make_rsrc(reinterpret_cast<const float*>(xg), xrange - static_cast<uint32_t>(z * (cv.C >> 3)) * PL);

  // patch: positions n0 .. plast cover images img0 .. img0 + nseg - 1 (<= 3);
  // segment s holds output rows f_s .. l_s of its image plus the KH - 1 halo
  const int plast = min(n0 + tpc, tpi > 0 ? (timg + 1) * HW : P.N) - 1;
  const int img0 = n0 / HW, nseg = plast / HW - img0 + 1;
  const int f0 = (n0 - img0 * HW) / OW;
  auto seg_last = [&](int s) { return s == nseg - 1 ? (plast - (img0 + s) * HW) / OW : cv.Ho - 1; };
  const int p1 = seg_last(0) - f0 + KH;
  const int p2 = p1 + (nseg > 1 ? seg_last(1) + KH : 0);
  const int R = p2 + (nseg > 2 ? seg_last(2) + KH : 0);
  const int PW = cv.W + 2 * cv.pw;
  const int dlt = cbx6::seg_shift(OW, KH);
  // LDS stage = [octet h][patch row: rpc chunks = positions x 3 terms + pad];
  // chunk c (16 B) of piece i of this wave = DMA lane's slot
  uint32_t poff[PD];
#pragma unroll
  for (int i = 0; i < PD; ++i) {
    const int c = (wave * PD + i) * 64 + lane;
    const int h = static_cast<int>(fdiv(static_cast<uint32_t>(c), oct_div)), rem = c - h * (octb >> 4);
    // segment of this chunk (segment s starts s * dlt chunks late), then its row
    const int sg = (nseg > 2 && rem >= p2 * rpc + 2 * dlt) ? 2 : (nseg > 1 && rem >= p1 * rpc + dlt) ? 1 : 0;
    const int r2 = rem - sg * dlt;
    const int prow = static_cast<int>(fdiv(static_cast<uint32_t>(r2), rpc_div)), pc = r2 - prow * rpc;
    const int pcol = pc / 3, t = pc - pcol * 3;
    uint32_t off = 0x80000000u;
    if (h < 2 && prow < (sg == 0 ? p1 : sg == 1 ? p2 : R) && prow < R && pcol < PW) {
      const int y = (sg == 0 ? f0 + prow : prow - (sg == 1 ? p1 : p2)) - cv.ph;
      const int x = pcol - cv.pw;
      if (y >= 0 && y < cv.H && x >= 0 && x < cv.W)
        off = static_cast<uint32_t>(img0 + sg) * static_cast<uint32_t>(ximg) + static_cast<uint32_t>(h) * PL +
              static_cast<uint32_t>((y * cv.W + x) * 48 + t * 16);
    }
    poff[i] = off;
  }
  // B fragment bases (bytes into a stage) of this lane's column in block j
  int bb[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int n = cbx6::clamp_col(n0 + wc * 32 * NB + 32 * j + lr, n0, plast);
    const int img = static_cast<int>(fdiv(static_cast<uint32_t>(n), cv.howo)), sp = n - img * HW;
    const int oh = static_cast<int>(fdiv(static_cast<uint32_t>(sp), cv.wo_div)), ow = sp - oh * OW;
    const int sg = img - img0;
    const int prow = sg == 0 ? oh - f0 : (sg == 1 ? p1 : p2) + oh;
    bb[j] = lh * octb + (prow * rpc + sg * dlt) * 16 + ow * 48;
  }
  floatx16 acc[1][NB];
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[0][j][r] = 0.0f;

  auto issue = [&](int kt, int stg, int i) {
    dma_b128(xrsrc, poff[i] + static_cast<uint32_t>(kt) * 2u * PL,
             lds0 + static_cast<uint32_t>(stg * SFB + (wave * PD + i) * 1024));
  };
  x6::bf16x8 fa[2][3], fb[2][3];
  auto read_b = [&](x6::bf16x8 (&f)[3], const char* st, int s, int j) {
    const int kh = s / KW, kw = s - kh * KW;
    const char* p = st + bb[j] + kh * rpc * 16 + kw * 48;
#pragma unroll
    for (int t = 0; t < 3; ++t) f[t] = *reinterpret_cast<const x6::bf16x8*>(p + 16 * t);
  };

  {
    const x6::bf16x8* ap = wpack + ((int64_t)((z * P.tiles_m + tm) * WR + wr) * KT) * T * cbx6::FRAG + lane;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t*>(xg), 0, static_cast<int>(xrange - static_cast<uint32_t>(z * (cv.C >> 3)) * PL), 0x00020000);
    auto load_a = [&](x6::bf16x8 (&f)[3], int q) {
#pragma unroll
      for (int t = 0; t < 3; ++t) f[t] = ap[q * cbx6::FRAG + t * 64];
    };
    // the next K-tile's patch pieces: loaded into staging registers at tap s,
    // stored to the next stage SD taps later (SD = 2: a load has two taps of
    // MFMAs, >= 1.5k cycles, to land; the input companion is mostly L2 misses)
    constexpr int SD = T >= 4 ? 2 : 1;
    constexpr int PMAX = (PD + T - SD - 1) / (T - SD);  // patch pieces per tap
    typedef int int4x __attribute__((ext_vector_type(4)));
    int4x stg[SD + 1][PMAX];
#pragma unroll
    for (int i = 0; i < PD; ++i) issue(0, 0, i);
    load_a(fa[0], 0);
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    read_b(fb[0], smem, 0, 0);
    auto vtile = [&](int kt, auto par_c, auto more_c) {
      constexpr int PAR = decltype(par_c)::value;
      constexpr bool MORE = decltype(more_c)::value;
      const char* cur = smem + (kt & 1) * SFB;
      const char* nxt = smem + ((kt + 1) & 1) * SFB;
      char* nst = smem + ((kt + 1) & 1) * SFB + wave * PD * 1024 + lane * 16;
#pragma unroll
      for (int s = 0; s < T; ++s) {
        const int pa = (s + PAR) & 1;
        const int q = kt * T + s;
        if (MORE) {
          // block 0: the pieces loaded at tap s - SD into the next stage, this
          // tap's pieces into staging registers
          if (s >= SD) {
            const int s0 = s - SD;
#pragma unroll
            for (int i = cbx6::piece_lo_d(s0, PD, T, SD); i < cbx6::piece_lo_d(s0 + 1, PD, T, SD); ++i)
              *reinterpret_cast<int4x*>(nst + i * 1024) = stg[s0 % (SD + 1)][i - cbx6::piece_lo_d(s0, PD, T, SD)];
          }
#pragma unroll
          for (int i = cbx6::piece_lo_d(s, PD, T, SD); i < cbx6::piece_lo_d(s + 1, PD, T, SD); ++i)
            stg[s % (SD + 1)][i - cbx6::piece_lo_d(s, PD, T, SD)] = __builtin_bit_cast(
                int4x, __builtin_amdgcn_raw_buffer_load_b128(
                           xr, static_cast<int>(poff[i] + static_cast<uint32_t>(kt + 1) * 2u * PL), 0, 0));
        }
        if (s + 1 < T || MORE) load_a(fa[pa ^ 1], q + 1);
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const bool last = s == T - 1 && j == NB - 1;
          if (last && MORE) {  // the next stage is complete
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
          }
          if (!last)
            read_b(fb[(j + 1) & 1], cur, j + 1 < NB ? s : s + 1, j + 1 < NB ? j + 1 : 0);
          else if (MORE)
            read_b(fb[0], nxt, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          acc[0][j] = x6::mfma6(x6::Parts{fa[pa][0], fa[pa][1], fa[pa][2]},
                                x6::Parts{fb[j & 1][0], fb[j & 1][1], fb[j & 1][2]}, acc[0][j]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    if constexpr (T % 2 == 0) {
      int kt = 0;
      for (; kt + 1 < KT; ++kt) vtile(kt, P0{}, T_{});
      vtile(kt, P0{}, F_{});
    } else {
      int kt = 0;
      for (; kt + 2 < KT; kt += 2) {
        vtile(kt, P0{}, T_{});
        vtile(kt + 1, P1{}, T_{});
      }
      if (kt + 1 < KT) {
        vtile(kt, P0{}, T_{});
        vtile(kt + 1, P1{}, F_{});
      } else {
        vtile(kt, P0{}, F_{});
      }
    }
  }
  conv_epilogue_nchw<1, NB>(acc, P, ep, m0 + 32 * wr, n0 + wc * 32 * NB, lr, lh, plast + 1);
  if (yoct != nullptr) {
    // the output's channel-octet companion (the next convolution's input,
    // k_pack_octets_x6 layout): the split of the stored values (bias and
    // ReLU applied; conv_epilogue_nchw left them in acc).  Lane (lr, h)
    // holds channels 8 k + 4 h .. + 3 of octets k = 0..3 of its 32 rows; the
    // two halves trade halves (lane ^ 32) so that half 0 owns octets 0, 1 and
    // half 1 octets 2, 3, whole.
    const int mw = m0 + 32 * wr;
    const bool relu = ep.relu != 0;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int n = n0 + wc * 32 * NB + 32 * j + lr;
      float o[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) o[r] = relu ? fmaxf(acc[0][j][r], 0.0f) : acc[0][j][r];
      float rcv[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) rcv[r] = __shfl_xor(lh ? o[r] : o[8 + r], 32);
      if (n > plast) continue;
      const uint32_t im = fdiv(static_cast<uint32_t>(n), ep.hw);
      const int sp = n - static_cast<int>(im) * HW;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int k = 2 * lh + u;
        if (mw + 8 * k >= P.M) continue;
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = lh ? rcv[4 * u + e] : o[4 * u + e];
          v[4 + e] = lh ? o[8 + 4 * u + e] : rcv[4 * u + e];
        }
        const int oct = (z * P.M + mw) / 8 + k;
        x6::store_terms8(v, yoct + (((int64_t)im * cout8 + oct) * HW + sp) * 48);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// k_conv_cb16_x6: k_conv_cb_x6 on v_mfma_f32_16x16x32_bf16.  Same input
// octet companion, patch ring, DMA / staging schedule and tile order; the
// matrix-core shape differs.  MI355X_MICROARCH.md (DVFS give-back, item 7):
// at equal cycles per FLOP a 16x16x32 loop on random data holds a higher
// clock than a 32x32x16 one (1.12-1.15x the FLOP/s, LDS-fed).
// K order: a K-tile is still 16 channels (two octets) x all T taps; an MFMA
// group's lane group g = lane >> 4 of the operands holds octet g & 1 at one
// tap (lower half g < 2, upper half g >= 2): taps 2p, 2p + 1 of one K-tile,
// or tap T - 1 of two consecutive K-tiles (the cross group, see the loop).
// Wave tile = 32 rows (two 16-row blocks) x 32 NB columns (2 NB 16-column
// blocks), the accumulators the same 64 floats per lane as the 32x32 form.
// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}
namespace cb16 {
constexpr int FRAG = 3 * 64;  // bf16x8 units per fragment (3 terms x 64 lanes): 16 rows x 32 k
}  // namespace cb16
namespace x6 {
__device__ __forceinline__ floatx4 mfma6_16(const Parts& a, const Parts& b, floatx4 c) {
  if (RRAM_X6_DROP != 1) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.l, b.h, c, 0, 0, 0);
  if (RRAM_X6_DROP != 2) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.l, c, 0, 0, 0);
  if (RRAM_X6_DROP != 3) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, b.m, c, 0, 0, 0);
  if (RRAM_X6_DROP != 4) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, b.h, c, 0, 0, 0);
  if (RRAM_X6_DROP != 5) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.m, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.h, c, 0, 0, 0);
}
}  // namespace x6

// Epilogue of MI x NJ 16x16 accumulator blocks (v_mfma_f32_16x16x32 layout:
// col = lane & 15, row = 4 (lane >> 4) + r): conv_epilogue_nchw's arithmetic
// and raw buffer stores, the lane's row group folded into its base address.
// acc is left holding the stored values before the ReLU.  ep.C == nullptr
// (the convolution-output fold: the only reader takes the octet companion)
// computes the values and stores nothing.
template <int MI, int NJ>
__device__ __forceinline__ void conv_epilogue_nchw16(floatx4 (&acc)[MI][NJ], const Params& P, const Epi& ep, int mwave,
                                                     int nwave, int c16, int g, int nlim) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(ep.C, 0, 0x7FFFFFFF, 0x00020000);
  const int HWo = static_cast<int>(ep.hw.d);
  const int mw = mwave + 4 * g;
  const bool rows_full = mwave + MI * 16 <= P.M;
  // (every octet-kernel launch passes a row bias or none: no column bias)
  const bool row_bias = ep.bias_mode == RRAM_BIAS_ROW;
  const bool relu = ep.relu != 0;
  const bool store = ep.C != nullptr;  // uniform
  const float alpha = ep.alpha;
  // The wave's 16 MI row biases by scalar loads (the constant address space;
  // whole blocks when every row is in range), each lane taking its row
  // group's, before the first store (round 5 loaded a value per column block
  // between the stores, each load waiting in the in-order vmcnt for every
  // store before it; time unchanged, profiles/r06_ab_cb16_epilogue.txt)
  float bz[MI][4];
  if (row_bias) {
    const int mb = __builtin_amdgcn_readfirstlane(mwave);
    typedef const __attribute__((address_space(4))) float cfloat;
    typedef float float8v __attribute__((ext_vector_type(8)));
    typedef const __attribute__((address_space(4))) float8v cfloat8;
    float sv[16 * MI];
    if (rows_full) {
#pragma unroll
      for (int b = 0; b < 2 * MI; ++b) {
        const float8v v = *(cfloat8*)((cfloat*)ep.bias + mb + 8 * b);
#pragma unroll
        for (int e = 0; e < 8; ++e) sv[8 * b + e] = v[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 16 * MI; ++e) {
        const float v = ((cfloat*)ep.bias)[min(mb + e, P.M - 1)];
        sv[e] = mb + e < P.M ? v : 0.0f;
      }
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float* s = sv + 16 * i + r;
        bz[i][r] = g == 0 ? s[0] : g == 1 ? s[4] : g == 2 ? s[8] : s[12];
      }
  } else {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) bz[i][r] = 0.0f;
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = nwave + 16 * j + c16;
    if (n >= P.N || n >= nlim) continue;
    const uint32_t im = fdiv(static_cast<uint32_t>(n), ep.hw);
    const uint32_t sp = static_cast<uint32_t>(n) - im * ep.hw.d;
    const uint32_t base = static_cast<uint32_t>((im * ep.cimg + sp + static_cast<int64_t>(mw) * HWo) * 4);
    float ov[MI][4];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float o = (alpha * acc[i][j][r] + bz[i][r]) + 0.0f;  // (+ the absent column bias: -0 -> +0 as before)
        acc[i][j][r] = o;
        ov[i][r] = relu ? fmaxf(o, 0.0f) : o;
      }
    if (!store) continue;
    if (rows_full) {  // uniform: no per-store exec masking
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, ov[i][r]), rs, static_cast<int>(base),
                                                (16 * i + r) * HWo * 4, 0);
    } else {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (mw + 16 * i + r < P.M)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, ov[i][r]), rs, static_cast<int>(base),
                                                  (16 * i + r) * HWo * 4, 0);
    }
  }
}

// RRAM_CB_STAMP (diagnostic build only, never the product): per-group
// s_memtime cycle sums of k_conv_cb16_x6 (slots 0 .. 2H:
// the groups of an (even, odd) K-tile pair, 2H + 1: the end-of-K-tile
// barriers, 2H + 2: the barrier after an odd K-tile's cross group, 2H + 3:
// the prologue, 2H + 4: the epilogue, 2H + 5: wave-tiles), summed over waves
// into g_cb_stamp (read by rram_debug_cb_stamps)
#ifdef RRAM_CB_STAMP
__device__ unsigned long long g_cb_stamp[64];
__device__ __forceinline__ unsigned long long cb_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#endif

// RRAM_CB16_ABLATE (diagnostic builds only, wrong results), a bit mask of
// the parts left out: 1 the K loop's B fragment reads (the MFMAs reuse the
// prologue's), 2 its weight loads, 4 the next K-tile's patch staging (loads
// and LDS stores), 8 its barriers, 16 the epilogue's stores.  Read with care:
// stale operands (1, 2) and unwritten outputs (16: the layers after it then
// multiply zeros) lower the chip's power and raise its clock, so part of
// those savings is DVFS, not the removed work (profiles/r06_ab_cb16_ablate.txt)
#ifndef RRAM_CB16_ABLATE
#define RRAM_CB16_ABLATE 0
#endif
// KTO = KT & 1 (the K-tile count's parity, host-checked): one tail shape per
// instantiation.  With both tails in one kernel (a runtime branch after the
// K-tile pair loop) the register allocator could not keep the loop's values
// in place and the two-workgroups-per-CU forms spilled 12-68 bytes per lane
// (conv2's 5 x 5: ~176 MB of scratch traffic per b256 launch, round 4);
// per parity they take 184-188 VGPRs and no scratch.
template <int KH, int KW, int WR, int NB, int PD, int OCC, int KTO>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC)))
k_conv_cb16_x6(Params P, const x6::bf16x8* __restrict__ wpack, const uint16_t* __restrict__ xpack, int octb, int rpc,
               uint32_t xrange, int ximg, char* __restrict__ yoct, int cout8, FastDiv oct_div, FastDiv rpc_div,
               int tpi) {
  using namespace g2;
  constexpr int T = KH * KW, PP = (T + 1) / 2, WC = 4 / WR, BMc = 32 * WR, BNc = 32 * NB * WC, SFB = PD * 4 * 1024;
  constexpr int MI = 2, NJ = 2 * NB;
  static_assert(2 * SFB <= 160 * 1024, "LDS");
  static_assert(PP >= 2, "pair groups");
#ifdef RRAM_CB_STAMP
  constexpr bool STAMP = true;
  __shared__ unsigned long long cst_lds[4][32];
  if ((threadIdx.x & 63) < 32) cst_lds[threadIdx.x >> 6][threadIdx.x & 63] = 0;
  unsigned long long ctprev = cb_stamp();
  auto cstamp = [&](int slot) __attribute__((always_inline)) {
    if constexpr (STAMP) {
      const unsigned long long tn = cb_stamp();
      if ((threadIdx.x & 63) == 0) cst_lds[threadIdx.x >> 6][slot] += tn - ctprev;
      ctprev = tn;
    }
  };
#define RRAM_CB_ST(slot) cstamp(slot)
#else
#define RRAM_CB_ST(slot)
#endif
  __shared__ __attribute__((aligned(16))) char smem[2 * SFB];
  // the patch pieces' source offsets, one word per (piece, thread): read per
  // refill instead of held in PD registers (at two workgroups per CU the
  // 5x5 form otherwise spills)
  __shared__ uint32_t poff_lds[PD * 256];
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem));

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c16 = lane & 15, g = lane >> 4, up = g >> 1;
  const int wr = wave % WR, wc = wave / WR;

  // Persistent (round 6): the grid holds at most two workgroups per CU.  XCD
  // x owns the contiguous tile range [xs, xe) (row tiles of a column tile
  // consecutive: they share its patch; a band order, 48 column tiles per band
  // so one row block's weights stay in L2, raised conv3 / conv4 traffic
  // 403 -> 461 / 389 -> 528 MB: profiles/r05_ab_cb16_sd_band.txt) and its
  // workgroups take every wx-th tile of it.  After a tile's last MFMA group
  // the next tile's patch pieces (K-tile 0) are DMA'd into the stage that
  // K-tile leaves free and its first weight group is loaded, so that
  // prologue's latency runs under this tile's epilogue stores instead of in
  // front of the next tile's MFMAs (K-tile kt's stage is (kt ^ sp) & 1, sp
  // flipping per tile when KT is odd).
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, loc = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int wx = q8 + (xcd < r8 ? 1 : 0);  // workgroups on this XCD
  const int ntiles = P.tiles_z * P.tiles_m * P.tiles_n;
  const int qt = ntiles >> 3, rt = ntiles & 7;
  const int xs = xcd * qt + min(xcd, rt), xe = xs + qt + (xcd < rt ? 1 : 0);

  const ConvGeom& cv = P.cv;
  const int HW = cv.howo.d, OW = cv.wo_div.d;
  const int KT = cv.C >> 4;
  const uint32_t PL = static_cast<uint32_t>(cv.H * cv.W * 48);
  const int PW = cv.W + 2 * cv.pw;
  const int dlt = cbx6::seg_shift(OW, KH);
  const int NQ = (KT * T + 1) / 2;  // MFMA groups of the whole K
  // one tile's geometry (uniform)
  struct TileGeo {
    int z, tm, m0, n0, plast, img0, nseg, f0, p1, p2, R;
  };
  auto geo = [&](int tid) __attribute__((always_inline)) {
    TileGeo tg;
    tg.z = __builtin_amdgcn_readfirstlane(tid / (P.tiles_m * P.tiles_n));
    const int r_ = tid - tg.z * P.tiles_m * P.tiles_n;
    tg.tm = __builtin_amdgcn_readfirstlane(r_ % P.tiles_m);
    const int tn = __builtin_amdgcn_readfirstlane(r_ / P.tiles_m);
    tg.m0 = tg.tm * BMc;
    const int timg = tpi > 0 ? tn / tpi : 0;
    const int tpc = cv.tpitch > 0 ? cv.tpitch : BNc;  // positions per tile
    tg.n0 = tpi > 0 ? timg * HW + (tn - timg * tpi) * tpc : tn * tpc;
    tg.plast = min(tg.n0 + tpc, tpi > 0 ? (timg + 1) * HW : P.N) - 1;
    tg.img0 = tg.n0 / HW;
    tg.nseg = tg.plast / HW - tg.img0 + 1;
    tg.f0 = (tg.n0 - tg.img0 * HW) / OW;
    auto seg_last = [&](int s) { return s == tg.nseg - 1 ? (tg.plast - (tg.img0 + s) * HW) / OW : cv.Ho - 1; };
    tg.p1 = seg_last(0) - tg.f0 + KH;
    tg.p2 = tg.p1 + (tg.nseg > 1 ? seg_last(1) + KH : 0);
    tg.R = tg.p2 + (tg.nseg > 2 ? seg_last(2) + KH : 0);
    return tg;
  };
  // the patch pieces' source offsets, one word per (piece, thread), each
  // thread reading only its own (no barrier between a write and its reads)
  // (scalar arguments: with the geometry struct behind a reference the
  // compiler kept it in scratch and indexed it per segment)
  auto set_poff = [&](int nseg, int p1, int p2, int R, int f0, int img0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PD; ++i) {
      const int c = (wave * PD + i) * 64 + lane;
      const int h = static_cast<int>(fdiv(static_cast<uint32_t>(c), oct_div)), rem = c - h * (octb >> 4);
      // segment of this chunk (segment s starts s * dlt chunks late), then its row
      const bool s2 = nseg > 2 && rem >= p2 * rpc + 2 * dlt, s1 = !s2 && nseg > 1 && rem >= p1 * rpc + dlt;
      const int sg = s2 ? 2 : s1 ? 1 : 0;
      const int r2 = rem - sg * dlt;
      const int prow = static_cast<int>(fdiv(static_cast<uint32_t>(r2), rpc_div)), pc = r2 - prow * rpc;
      const int pcol = pc / 3, t = pc - pcol * 3;
      const int plim = s2 ? R : s1 ? p2 : p1;
      const int y = (s2 ? prow - p2 : s1 ? prow - p1 : f0 + prow) - cv.ph;
      const int x = pcol - cv.pw;
      uint32_t off = 0x80000000u;
      if (h < 2 && prow < plim && prow < R && pcol < PW && y >= 0 && y < cv.H && x >= 0 && x < cv.W)
        off = static_cast<uint32_t>(img0 + sg) * static_cast<uint32_t>(ximg) + static_cast<uint32_t>(h) * PL +
              static_cast<uint32_t>((y * cv.W + x) * 48 + t * 16);
      poff_lds[i * 256 + threadIdx.x] = off;
    }
  };
  auto poff = [&](int i) { return poff_lds[i * 256 + threadIdx.x]; };
  // this group's octets start at octet z C/8 of every image
  auto xg_of = [&](int z) { return xpack + (int64_t)z * (cv.C >> 3) * (PL >> 1); };
  auto xbytes_of = [&](int z) { return xrange - static_cast<uint32_t>(z * (cv.C >> 3)) * PL; };
  // K-tile kt's patch piece i of tile geometry tg into stage stg (LDS-DMA)
  // (K-tile 0 of a tile: every offset read before the first DMA -- a DMA
  // writes LDS, so the compiler kept each offset read behind the DMA before
  // it, one LDS round trip per piece)
  auto issue_kt0 = [&](const int4v& rs, int stg) {
    uint32_t po[PD];
#pragma unroll
    for (int i = 0; i < PD; ++i) po[i] = poff(i);
#pragma unroll
    for (int i = 0; i < PD; ++i) dma_b128(rs, po[i], lds0 + static_cast<uint32_t>(stg * SFB + (wave * PD + i) * 1024));
  };
  // this wave's weight fragments through a buffer resource: the group's
  // offset is uniform (SGPR soffset), the lane's 16 bytes the only VGPR
  // (64-bit per-load addresses cost the registers this kernel spills)
  auto a_rsrc = [&](const TileGeo& tg) {
    const x6::bf16x8* ap = wpack + ((int64_t)((tg.z * P.tiles_m + tg.tm) * WR + wr) * NQ) * MI * cb16::FRAG;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<x6::bf16x8*>(ap), 0, NQ * MI * cb16::FRAG * 16, 0x00020000);
  };
  const int alane = lane * 16;
  auto load_a_from = [&](const __amdgpu_buffer_rsrc_t& rs, x6::bf16x8 (&f)[MI][3], int q) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int t = 0; t < 3; ++t)
        f[i][t] = __builtin_bit_cast(
            x6::bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, alane, (q * MI + i) * cb16::FRAG * 16 + t * 1024, 0));
  };

  // K order (T odd: 3x3, 5x5): K-tiles alternate even / odd.  An even K-tile
  // runs H = T / 2 pair groups (taps 2p, 2p + 1: lower / upper half) and
  // leaves tap T - 1; the odd K-tile after it starts with the cross group
  // (lower half: the even K-tile's tap T - 1 from the stage before, upper
  // half: its own tap T - 1), then its H pairs.  So no MFMA group is padded,
  // except a last even K-tile's tap T - 1 (odd KT): its upper half is zero
  // weights (pack) and zero B, so a non-finite input never meets a zero
  // weight.  The cross group reads the stage the odd K-tile's refill writes
  // next: a barrier after it (odd K-tiles only) orders the refill behind it.
  constexpr int H = T / 2;
  static_assert(T % 2 == 1, "odd tap counts (3x3, 5x5)");
  // a tile's last group runs on fa[0] (the next tile's first weights go to fa[1])
  static_assert((H & 1) == 0 || KTO == 0, "last group's A parity");
  const int rowb = rpc * 16;
  auto toff = [&](int s) { return (s / KW) * rowb + (s % KW) * 48; };  // uniform
  // (opaque to the compiler: hoisted out of the K-tile loop, the NJ x H sums
  // bb[j] + pair_off(s0) would each hold a register)
  auto pair_off = [&](int s0) {
    int o = toff(s0) + (up ? toff(s0 + 1) - toff(s0) : 0);
    asm volatile("" : "+v"(o));
    return o;
  };
  x6::bf16x8 fa[2][MI][3], fb[2][3];
  int bb[NJ];
  // group kinds: 0 pair (s0, s0 + 1), 1 cross (tap T - 1 of two K-tiles), 2 padded (tap T - 1, upper zero)
  auto read_b = [&](x6::bf16x8 (&f)[3], const char* lo, const char* hi, int kind, int s0, int j) {
    const char* st = kind == 1 ? (up ? hi : lo) : lo;
    const int to = kind == 0 ? pair_off(s0) : toff(T - 1);
    const char* q = st + bb[j] + to;
#pragma unroll
    for (int t = 0; t < 3; ++t) f[t] = *reinterpret_cast<const x6::bf16x8*>(q + 16 * t);
    if (kind == 2) {
#pragma unroll
      for (int t = 0; t < 3; ++t) f[t] = up ? x6::bf16x8{} : f[t];
    }
  };
  // staging distance (groups): the next K-tile's patch pieces are loaded at
  // group g and stored to the next stage at g + SD; SD = 2 where the K-tile
  // has >= 4 groups: the 3x3 forms (H = 4: +0.5 % maps/s, conv3 / conv4
  // -1 %, profiles/r05_ab_cb16_sd_band.txt) and, since H = 12 there, the
  // 5x5 form too (the r05 A/B's "5x5 keeps 1" described a build
  // that never shipped; RRAM_CB16_SD5 = 1 is that variant: no difference,
  // profiles/r06_ab_conv_y_fold_sd5.txt)
#ifndef RRAM_CB16_SD5
#define RRAM_CB16_SD5 2
#endif
  constexpr int SD = KH == 5 ? RRAM_CB16_SD5 : (H >= 4 ? 2 : 1);
  constexpr int PMAX = (PD + H - SD - 1) / (H - SD);  // patch pieces per group (the shortest K-tile spreads them over H - SD groups)
  static_assert(H >= 2, "pair groups");
  typedef int int4x __attribute__((ext_vector_type(4)));
  int4x stg[SD + 1][PMAX];
  floatx4 acc[MI][NJ];

  int t = xs + loc;
  if (t >= xe) return;  // (uniform; the host launches no such workgroup)
  TileGeo cur = geo(t);
  int sp = 0;
  set_poff(cur.nseg, cur.p1, cur.p2, cur.R, cur.f0, cur.img0);
  {
    const int4v rs0 = make_rsrc(reinterpret_cast<const float*>(xg_of(cur.z)), xbytes_of(cur.z));
    issue_kt0(rs0, 0);
    load_a_from(a_rsrc(cur), fa[0], 0);
  }
  for (;;) {
    const int tnext = t + wx;
    const bool more_tiles = tnext < xe;  // uniform
    Epi ep = P.e;
    if (cur.z > 0) {
      if (ep.C) ep.C += cur.z * P.grp_c;  // (NULL: the convolution-output fold stores no y, for any group)
      if (ep.bias) ep.bias += cur.z * P.grp_bias;
    }
    const __amdgpu_buffer_rsrc_t ar = a_rsrc(cur);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t*>(xg_of(cur.z)), 0, static_cast<int>(xbytes_of(cur.z)), 0x00020000);
    // B fragment bases (bytes into a stage) of this lane's column in block j,
    // at tap 0 of its octet (g & 1)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = cbx6::clamp_col(cur.n0 + wc * 32 * NB + 16 * j + c16, cur.n0, cur.plast);
      const int img = static_cast<int>(fdiv(static_cast<uint32_t>(n), cv.howo)), sp_ = n - img * HW;
      const int oh = static_cast<int>(fdiv(static_cast<uint32_t>(sp_), cv.wo_div)), ow = sp_ - oh * OW;
      const int sg = img - cur.img0;
      const int prow = sg == 0 ? oh - cur.f0 : (sg == 1 ? cur.p1 : cur.p2) + oh;
      bb[j] = (g & 1) * octb + (prow * rpc + sg * dlt) * 16 + ow * 48;
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.0f;
    auto load_a = [&](x6::bf16x8 (&f)[MI][3], int q) { load_a_from(ar, f, q); };
    const char* smem0 = smem + sp * SFB;
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    // the first K-tile is even: pair (0, 1), or the padded group when T == 1 ... (T >= 9 here)
    read_b(fb[0], smem0, smem0, 0, 0, 0);
    // K-tile kt of kind ODD (0 even, 1 odd); q0 = its first global group;
    // MORE: a next K-tile exists; PADT: the padded group ends it (last even K-tile)
    auto ktile = [&](int kt, int q0, auto odd_c, auto more_c, auto padt_c) {
      constexpr bool ODD = decltype(odd_c)::value, MORE = decltype(more_c)::value, PADT = decltype(padt_c)::value;
      constexpr int NG = ODD ? H + 1 : H + (PADT ? 1 : 0);
      constexpr int PAR = ODD ? (H & 1) : 0;  // A parity: an (even, odd) pair of K-tiles runs 2 H + 1 groups
      const int ks = (kt ^ sp) & 1;
      const char* cur_st = smem + ks * SFB;
      const char* oth = smem + (ks ^ 1) * SFB;  // the stage before = the stage refilled next
      char* nst = smem + (ks ^ 1) * SFB + wave * PD * 1024 + lane * 16;
      static_for<0, NG>([&](auto gc) {
        constexpr int gi = decltype(gc)::value;
        constexpr int KIND = ODD ? (gi == 0 ? 1 : 0) : (gi < H ? 0 : 2);
        constexpr int S0 = ODD ? 2 * (gi - 1) : 2 * gi;
        constexpr int pa = (gi + PAR) & 1;
        // the group after this one (same K-tile)
        constexpr int NKIND = ODD ? 0 : (gi + 1 < H ? 0 : 2);
        constexpr int NS0 = ODD ? 2 * gi : 2 * (gi + 1);
        const int q = q0 + gi;
        if (MORE && !(RRAM_CB16_ABLATE & 4)) {
          if (gi >= SD) {
            constexpr int g0 = gi - SD;
#pragma unroll
            for (int i = cbx6::piece_lo_d(g0, PD, NG, SD); i < cbx6::piece_lo_d(g0 + 1, PD, NG, SD); ++i)
              *reinterpret_cast<int4x*>(nst + i * 1024) = stg[g0 % (SD + 1)][i - cbx6::piece_lo_d(g0, PD, NG, SD)];
          }
#pragma unroll
          for (int i = cbx6::piece_lo_d(gi, PD, NG, SD); i < cbx6::piece_lo_d(gi + 1, PD, NG, SD); ++i)
            stg[gi % (SD + 1)][i - cbx6::piece_lo_d(gi, PD, NG, SD)] = __builtin_bit_cast(
                int4x, __builtin_amdgcn_raw_buffer_load_b128(
                           xr, static_cast<int>(poff(i) + static_cast<uint32_t>(kt + 1) * 2u * PL), 0, 0));
        }
        if ((gi + 1 < NG || MORE) && !(RRAM_CB16_ABLATE & 2)) load_a(fa[pa ^ 1], q + 1);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const bool last = gi == NG - 1 && j == NJ - 1;
          if (last && MORE && !(RRAM_CB16_ABLATE & 8)) {  // the next stage is complete
            RRAM_CB_ST(ODD ? H + gi : gi);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            RRAM_CB_ST(2 * H + 1);
          }
          if (RRAM_CB16_ABLATE & 1) {
          } else if (!last) {
            if (j + 1 < NJ)  // (the cross group: lower half from the stage before)
              read_b(fb[(j + 1) & 1], KIND == 1 ? oth : cur_st, cur_st, KIND, S0, j + 1);
            else
              read_b(fb[(j + 1) & 1], cur_st, cur_st, NKIND, NS0, 0);
          } else if (MORE) {
            // the next K-tile's first group: after an even K-tile the cross
            // group (lower half here, upper half in the new stage), after an
            // odd one the pair (0, 1) of the new stage
            if (ODD)
              read_b(fb[0], oth, oth, 0, 0, 0);
            else
              read_b(fb[0], cur_st, oth, 1, 0, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < MI; ++i)
            acc[i][j] = x6::mfma6_16(x6::Parts{fa[pa][i][0], fa[pa][i][1], fa[pa][i][2]},
                                     x6::Parts{fb[j & 1][0], fb[j & 1][1], fb[j & 1][2]}, acc[i][j]);
          __builtin_amdgcn_sched_barrier(0);
        }
        RRAM_CB_ST(ODD ? H + gi : gi);
        // every wave is past the cross group: the refill -- or, after the
        // tile's last K-tile, the next tile's patch -- may overwrite `oth`
        if (ODD && gi == 0 && (MORE || more_tiles) && !(RRAM_CB16_ABLATE & 8)) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          __builtin_amdgcn_sched_barrier(0);
          RRAM_CB_ST(2 * H + 2);
        }
      });
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    RRAM_CB_ST(2 * H + 3);
    int kt = 0;
    for (; kt + 2 < KT; kt += 2) {
      const int q0 = (kt / 2) * (2 * H + 1);
      ktile(kt, q0, F_{}, T_{}, F_{});
      ktile(kt + 1, q0 + H, T_{}, T_{}, F_{});
      // the pair ran 2 H + 1 groups: the next A sits in fa[1]
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int t2 = 0; t2 < 3; ++t2) fa[0][i][t2] = fa[1][i][t2];
    }
    {
      const int q0 = (kt / 2) * (2 * H + 1);
      if constexpr (KTO == 0) {
        ktile(kt, q0, F_{}, T_{}, F_{});
        ktile(kt + 1, q0 + H, T_{}, F_{}, F_{});
      } else {
        ktile(kt, q0, F_{}, F_{}, T_{});
      }
    }
    // the next tile's prologue, in flight under this tile's epilogue: its
    // patch pieces of K-tile 0 into the stage the last K-tile left free (the
    // last K-tile reads only its own stage, bar an odd one's cross group,
    // which the barrier after it covers), its first weight group into fa[1]
    // (the last group ran on fa[0])
    TileGeo nxt = cur;
    if (more_tiles) {
      nxt = geo(tnext);
      set_poff(nxt.nseg, nxt.p1, nxt.p2, nxt.R, nxt.f0, nxt.img0);
      const int4v rsn = make_rsrc(reinterpret_cast<const float*>(xg_of(nxt.z)), xbytes_of(nxt.z));
      const int sfree = (KT ^ sp) & 1;
      issue_kt0(rsn, sfree);
      load_a_from(a_rsrc(nxt), fa[1], 0);
    }
    const int mwave = cur.m0 + 32 * wr, nwave = cur.n0 + wc * 32 * NB;
    if (RRAM_CB16_ABLATE & 16) {  // keep the sums alive: one store under a condition never true at run time
      float sum = 0.0f;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) sum += acc[i][j][r];
      if (ep.relu == 12345 && ep.C != nullptr) ep.C[lane] = sum;
      ep.C = nullptr;
    }
    conv_epilogue_nchw16<MI, NJ>(acc, P, ep, mwave, nwave, c16, g, cur.plast + 1);
    if (yoct != nullptr && !(RRAM_CB16_ABLATE & 16)) {
      // the output's octet companion: lane group g holds rows 4 g .. 4 g + 3 of
      // both 16-row blocks; lanes g, g ^ 1 (lane ^ 16) trade one block so that
      // an even g stores octet g / 2 of block 0 and an odd g octet (g - 1) / 2
      // of block 1, each whole (8 consecutive rows).
      const bool relu = ep.relu != 0;
      const bool ev = (g & 1) == 0;
      const int orow = mwave + 16 * (g & 1) + 8 * (g >> 1);  // first row of the lane's octet
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = nwave + 16 * j + c16;
        float o0[4], o1[4], rcv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o0[r] = relu ? fmaxf(acc[0][j][r], 0.0f) : acc[0][j][r];
          o1[r] = relu ? fmaxf(acc[1][j][r], 0.0f) : acc[1][j][r];
          rcv[r] = __shfl_xor(ev ? o1[r] : o0[r], 16);
        }
        if (n > cur.plast || orow >= P.M) continue;
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = ev ? o0[r] : rcv[r];
          v[4 + r] = ev ? rcv[r] : o1[r];
        }
        const uint32_t im = fdiv(static_cast<uint32_t>(n), ep.hw);
        const int sp_ = n - static_cast<int>(im) * HW;
        const int oct = (cur.z * P.M + orow) / 8;
        x6::store_terms8(v, yoct + (((int64_t)im * cout8 + oct) * HW + sp_) * 48);
      }
    }
    RRAM_CB_ST(2 * H + 4);
#ifdef RRAM_CB_STAMP
    if constexpr (STAMP)
      if ((threadIdx.x & 63) == 0) cst_lds[threadIdx.x >> 6][2 * H + 5] += 1;
#endif
    if (!more_tiles) break;
    // the next tile's first weight group moves to fa[0]
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int t2 = 0; t2 < 3; ++t2) fa[0][i][t2] = fa[1][i][t2];
    cur = nxt;
    t = tnext;
    sp ^= KTO;
  }
#ifdef RRAM_CB_STAMP
  if constexpr (STAMP)
    if ((threadIdx.x & 63) == 0)
      for (int k = 0; k < 2 * H + 6; ++k) atomicAdd(&g_cb_stamp[k], cst_lds[threadIdx.x >> 6][k]);
#endif
}
#undef RRAM_CB_ST

// w [G*M][Cg][T] -> k_conv_cb16_x6 fragments [G][rblocks][NQ][2][term][64 lanes][8],
// NQ = ceil(KT T / 2) groups in the kernel's K order: per (even, odd) pair
// of K-tiles, H = T / 2 pairs of the even one, the cross group, H pairs of
// the odd one (an odd KT ends with the padded group).  Lane l of fragment
// (q, i) holds row 32 rb + 16 i + (l & 15), channel octet (l >> 4) & 1 of its
// half's K-tile at its half's tap (l >> 5: upper half); zero on padding.
__global__ void __launch_bounds__(256) k_conv_cb16_pack_x6(const float* __restrict__ w, char* __restrict__ out, int M,
                                                           int Cg, int T, int rblocks, int units) {
  const int KT = Cg >> 4, H = T / 2, NQ = (KT * T + 1) / 2;
  for (int u = blockIdx.x * blockDim.x + threadIdx.x; u < units; u += gridDim.x * blockDim.x) {
    const int lane = u & 63, up = lane >> 5;
    int r = u >> 6;
    const int i = r & 1;
    r >>= 1;
    const int q = r % NQ;
    r /= NQ;
    const int rb = r % rblocks;
    const int gz = r / rblocks;
    // (K-tile, tap) of this lane's half in group q
    const int a = q / (2 * H + 1), gq = q - a * (2 * H + 1);
    int kt, s;
    if (gq < H) {                   // pair of the even K-tile 2a
      kt = 2 * a;
      s = 2 * gq + up;
    } else if (gq == H) {           // cross group (or the padded one at an odd KT's end)
      kt = 2 * a + up;
      s = T - 1;
    } else {                        // pair of the odd K-tile 2a + 1
      kt = 2 * a + 1;
      s = 2 * (gq - H - 1) + up;
    }
    const int m = rb * 32 + 16 * i + (lane & 15), c0 = kt * 16 + ((lane >> 4) & 1) * 8;
    const bool ok = m < M && kt < KT;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = ok ? w[((int64_t)gz * M + m) * Cg * T + (int64_t)(c0 + e) * T + s] : 0.0f;
    x6::Parts t;
    x6::split8_safe(v, t);
    char* f = out + (int64_t)(u >> 6) * 3072 + lane * 16;
    *reinterpret_cast<x6::bf16x8*>(f) = t.h;
    *reinterpret_cast<x6::bf16x8*>(f + 1024) = t.m;
    *reinterpret_cast<x6::bf16x8*>(f + 2048) = t.l;
  }
}

// x [img][C][H][W] fp32 -> bf16 terms [img][C/8][H][W][3][8] (k_conv_cb_x6's
// input).  One thread per (image, octet, position): 8 strided loads (coalesced
// across the threads), 48 bytes out.
__global__ void __launch_bounds__(256) k_pack_octets_x6(const float* __restrict__ x, char* __restrict__ out, int C8,
                                                        int HWi, int units) {
  for (int u = blockIdx.x * blockDim.x + threadIdx.x; u < units; u += gridDim.x * blockDim.x) {
    const int r = u / HWi, p = u - r * HWi;  // r = img C8 + octet
    const float* src = x + (int64_t)r * 8 * HWi + p;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = src[(int64_t)e * HWi];
    x6::store_terms8(v, out + (int64_t)u * 48);
  }
}

// The output's channel-octet companion from a 32x32-accumulator epilogue
// (k_pack_octets_x6 layout, the next convolution's pre-split input): the split
// of the stored values (bias and ReLU applied; conv_epilogue_nchw left the
// pre-ReLU values in acc).  Row block i of the wave: lane (lr, h) holds
// channels 8 k + 4 h .. + 3 of octets k = 0..3 of its 32 rows; the two lane
// halves trade halves (lane ^ 32) so half 0 owns octets 0, 1 and half 1
// octets 2, 3, whole (k_conv_cb_x6's epilogue, per row block).
template <int MI, int NB>
__device__ __forceinline__ void octet_epilogue(floatx16 (&acc)[MI][NB], const Params& P, const Epi& ep, int mwave,
                                               int nwave, int lr, int lh, char* __restrict__ yoct, int cout8) {
  const int HW = static_cast<int>(ep.hw.d);
  const bool relu = ep.relu != 0;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int mw = mwave + 32 * i;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int n = nwave + 32 * j + lr;
      float o[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) o[r] = relu ? fmaxf(acc[i][j][r], 0.0f) : acc[i][j][r];
      float rcv[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) rcv[r] = __shfl_xor(lh ? o[r] : o[8 + r], 32);
      if (n >= P.N) continue;
      const uint32_t im = fdiv(static_cast<uint32_t>(n), ep.hw);
      const int sp = n - static_cast<int>(im) * HW;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int k = 2 * lh + u;
        if (mw + 8 * k >= P.M) continue;
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = lh ? rcv[4 * u + e] : o[4 * u + e];
          v[4 + e] = lh ? o[8 + 4 * u + e] : rcv[4 * u + e];
        }
        x6::store_terms8(v, yoct + (((int64_t)im * cout8 + mw / 8 + k) * HW + sp) * 48);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// k_conv1x1_x6: the 1 x 1, stride-1, pad-free convolution (GoogLeNet's
// inception 1x1 / 3x3_reduce / 5x5_reduce / pool_proj layers,
// conv_layer.cu:9-30 with kernel 1) on the bf16x6 engine.  Per image
// Y (Cout x HW) = W (Cout x C) . X (C x HW), X read straight from NCHW fp32:
// no input pack pass and no octet companion, so the 4 bytes per input element
// are the kernel's only HBM read of it (once per M-tile).
//  - Weights: pre-split fragments (k_conv_cb_pack_x6 with T = 1, cached per
//    fault map), straight from L2 into registers one K-tile ahead.
//  - Activations: a K-tile is 16 channels x BNc positions; RING K-tiles are
//    in flight in registers ahead of the one written to the 2-stage LDS tile
//    [16 channels][BNc positions] fp32 (one barrier per K-tile).  A wave's B
//    fragment (8 channels of one position) is 8 conflict-free ds_read_b32,
//    split in registers once and shared by the wave's MI row blocks.
// Tile 32 MI WR x 32 NB (4 / WR): wave (wr, wc) owns rows 32 MI wr .. + 32 MI - 1
// and columns 32 NB wc .. + 32 NB - 1.  VEC = 4: 16-byte loads of 4
// consecutive positions (HW % 4 == 0, 16-byte aligned input); VEC = 1:
// 4-byte loads (any HW: the 7 x 7 layers).
namespace c1x1 {
constexpr int RING = 4;  // K-tiles loaded ahead (registers); a multiple of 2
}  // namespace c1x1
template <int MI, int NB, int WR, int VEC>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, MI * NB <= 4 ? 2 : 1)))
k_conv1x1_x6(Params P, const x6::bf16x8* __restrict__ wpack, const float* __restrict__ x, uint32_t xrange,
             char* __restrict__ yoct, int cout8) {
  using namespace g2;
  constexpr int WC = 4 / WR, BMc = 32 * MI * WR, BNc = 32 * NB * WC;
  constexpr int STG = 16 * BNc;           // floats per LDS stage
  constexpr int LPT = STG / VEC / 256;    // loads per thread per K-tile
  constexpr int RING = c1x1::RING;
  static_assert(LPT >= 1 && STG % (VEC * 256) == 0, "tile");
  typedef int int4x __attribute__((ext_vector_type(4)));
  using SV = typename std::conditional<VEC == 4, int4x, int>::type;
  __shared__ __attribute__((aligned(16))) float smem[2 * STG];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int wr = wave % WR, wc = wave / WR;
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, loc = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int tid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int tm = __builtin_amdgcn_readfirstlane(tid % P.tiles_m);
  const int tn = __builtin_amdgcn_readfirstlane(tid / P.tiles_m);
  const int m0 = tm * BMc, n0 = tn * BNc;
  const int HW = static_cast<int>(P.cv.howo.d), C = P.cv.C, KT = C >> 4;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), 0, static_cast<int>(xrange),
                                                                      0x00020000);
  // byte offset of load i at K-tile 0 (past the range: zeros)
  uint32_t loff[LPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) {
    const int e = i * 256 + static_cast<int>(threadIdx.x);
    const int c = e / (BNc / VEC), n = n0 + (e - c * (BNc / VEC)) * VEC;
    uint32_t off = 0x80000000u;
    if (n < P.N) {
      const uint32_t img = fdiv(static_cast<uint32_t>(n), P.cv.howo);
      const uint32_t sp = static_cast<uint32_t>(n) - img * static_cast<uint32_t>(HW);
      off = ((img * static_cast<uint32_t>(C) + static_cast<uint32_t>(c)) * static_cast<uint32_t>(HW) + sp) * 4u;
    }
    loff[i] = off;
  }
  const uint32_t kstep = static_cast<uint32_t>(HW) * 64u;  // bytes per K-tile (16 channel planes)
  SV stg[RING][LPT];
  auto load_b = [&](SV (&r)[LPT], int kt, bool ok) {  // !ok: past the range (zeros, no traffic)
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int o = static_cast<int>(ok ? loff[i] + static_cast<uint32_t>(kt) * kstep : 0x80000000u);
      if constexpr (VEC == 4)
        r[i] = __builtin_bit_cast(int4x, __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0));
      else
        r[i] = __builtin_bit_cast(int, __builtin_amdgcn_raw_buffer_load_b32(xr, o, 0, 0));
    }
  };
  auto store_b = [&](const SV (&r)[LPT], int stage) {
#pragma unroll
    for (int i = 0; i < LPT; ++i)
      *reinterpret_cast<SV*>(smem + stage * STG + (i * 256 + static_cast<int>(threadIdx.x)) * VEC) = r[i];
  };
  // weight fragments of row block rb = tm (BMc / 32) + MI wr + i, K-tile kt
  const x6::bf16x8* ap = wpack + (int64_t)(tm * (BMc / 32) + MI * wr) * KT * cbx6::FRAG + lane;
  x6::Parts fa[2][MI];
  auto load_a = [&](x6::Parts (&f)[MI], int kt) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const x6::bf16x8* q = ap + ((int64_t)i * KT + kt) * cbx6::FRAG;
      f[i].h = q[0];
      f[i].m = q[64];
      f[i].l = q[128];
    }
  };
  floatx16 acc[MI][NB];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  // Every load is issued unconditionally (K-tiles past the end read zeros
  // past the buffer range, weight fragments re-read the last K-tile): vmcnt
  // counts in issue order, and a load the compiler cannot prove issued (one
  // under a branch) makes it drain the whole ring at the next wait.
  // prologue: K-tiles 0 .. RING - 1 in flight, K-tile 0 in LDS stage 0
#pragma unroll
  for (int q = 0; q < RING; ++q) load_b(stg[q], q, q < KT);
  load_a(fa[0], 0);
  __builtin_amdgcn_sched_barrier(0);
  store_b(stg[0], 0);
  __syncthreads();

  const int colw = 32 * NB * wc + lr;
  // K-tile kt (kt % RING == PH): its B from LDS stage PH & 1.  K-tiles
  // KT .. KTP - 1 only keep the load stream uniform.
  auto step = [&](int kt, auto ph_c) {
    constexpr int PH = decltype(ph_c)::value;
    // this step's loads go out before any MFMA (the scheduler would otherwise
    // sink them next to their uses)
    load_b(stg[PH], kt + RING, kt + RING < KT);
    load_a(fa[(PH + 1) & 1], min(kt + 1, KT - 1));
    __builtin_amdgcn_sched_barrier(0);
    if (kt < KT) {
      const float* bs = smem + (PH & 1) * STG + 8 * lh * BNc + colw;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = bs[e * BNc + 32 * j];
        x6::Parts bp;
        x6::split8_safe(v, bp);
#pragma unroll
        for (int i = 0; i < MI; ++i) acc[i][j] = x6::mfma6(fa[PH & 1][i], bp, acc[i][j]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < KT) store_b(stg[(PH + 1) % RING], (PH + 1) & 1);
    __syncthreads();
  };
  const int KTP = (KT + RING - 1) / RING * RING;
  for (int kt = 0; kt < KTP; kt += RING)
    static_for<0, RING>([&](auto ph) { step(kt + decltype(ph)::value, ph); });
  Epi ep = P.e;
  conv_epilogue_nchw<MI, NB>(acc, P, ep, m0 + 32 * MI * wr, n0 + 32 * NB * wc, lr, lh);
  if (yoct != nullptr) octet_epilogue<MI, NB>(acc, P, ep, m0 + 32 * MI * wr, n0 + 32 * NB * wc, lr, lh, yoct, cout8);
}

// k_conv1x1_dma_x6: the same contraction with every operand LDS-DMA'd
// (buffer_load ... lds) into an NS-stage ring, NS - 1 K-tiles ahead: per
// K-tile the weight fragments of the tile's row blocks (3 KB each) and the
// fp32 activation tile [16 channels][BNc positions].  The wait for K-tile
// kt + 1 is a hand-counted vmcnt (every wave issues the same number of
// pieces, OOB dummies included), so no weight load issued after the next
// activation tile forces that tile to land early (the register-ring form's
// in-order vmcnt did: about one K-tile of latency hiding).
namespace c1x1 {
constexpr int NS = 4;  // LDS stages
}  // namespace c1x1
template <int MI, int NB, int WR, int VEC>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_conv1x1_dma_x6(Params P, const x6::bf16x8* __restrict__ wpack, const float* __restrict__ x, uint32_t xrange,
                 uint32_t wrange, char* __restrict__ yoct, int cout8) {
  using namespace g2;
  constexpr int WC = 4 / WR, BMc = 32 * MI * WR, BNc = 32 * NB * WC, RBL = BMc / 32;
  constexpr int NS = c1x1::NS;
  constexpr int A_BYTES = RBL * 3072, B_BYTES = 64 * BNc, STB = A_BYTES + B_BYTES;
  constexpr int NA = RBL * 3;                         // 1 KB weight pieces per K-tile
  constexpr int PIECE_B = VEC == 4 ? 1024 : 256;      // bytes per activation piece
  constexpr int NBP = B_BYTES / PIECE_B;
  constexpr int PA = (NA + 3) / 4, PB = (NBP + 3) / 4, PPW = PA + PB;
  static_assert(NS * STB + 1024 <= 160 * 1024, "LDS");
  static_assert((NS - 2) * PPW <= 63, "vmcnt");
  __shared__ __attribute__((aligned(16))) char smem[NS * STB + 1024];  // + the dummy pieces' landing pad
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem));

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int wr = wave % WR, wc = wave / WR;
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, loc = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int tid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int tm = __builtin_amdgcn_readfirstlane(tid % P.tiles_m);
  const int tn = __builtin_amdgcn_readfirstlane(tid / P.tiles_m);
  const int m0 = tm * BMc, n0 = tn * BNc;
  const int HW = static_cast<int>(P.cv.howo.d), C = P.cv.C, KT = C >> 4;
  const int4v xrs = make_rsrc(x, xrange);
  const int4v wrs = make_rsrc(reinterpret_cast<const float*>(wpack), wrange);
  // weight piece a = wave + 4 i: row block a / 3, term a % 3 of K-tile kt at
  // (((tm RBL + a / 3) KT + kt) 3072 + (a % 3) 1024) + 16 lane
  uint32_t aoff[PA], alds[PA];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int a = wave + 4 * i;
    const bool ok = a < NA;
    aoff[i] = ok ? static_cast<uint32_t>(((tm * RBL + a / 3) * KT) * 3072 + (a % 3) * 1024 + lane * 16) : 0x80000000u;
    alds[i] = ok ? static_cast<uint32_t>((a / 3 * 3 + a % 3) * 1024) : 0xFFFFFFFFu;
  }
  // activation piece q = wave + 4 i: floats q PIECE_B / 4 .. of the stage's
  // [16][BNc] tile, this lane's VEC of them at element q PIECE_B / 4 + VEC lane
  uint32_t boff[PB], blds[PB];
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int q = wave + 4 * i;
    uint32_t off = 0x80000000u;
    if (q < NBP) {
      const int e = q * (PIECE_B / 4) + lane * VEC;
      const int c = e / BNc, n = n0 + (e - c * BNc);
      if (n < P.N) {
        const uint32_t img = fdiv(static_cast<uint32_t>(n), P.cv.howo);
        const uint32_t sp = static_cast<uint32_t>(n) - img * static_cast<uint32_t>(HW);
        off = ((img * static_cast<uint32_t>(C) + static_cast<uint32_t>(c)) * static_cast<uint32_t>(HW) + sp) * 4u;
      }
    }
    boff[i] = off;
    blds[i] = q < NBP ? static_cast<uint32_t>(A_BYTES + q * PIECE_B) : 0xFFFFFFFFu;
  }
  const uint32_t kstep = static_cast<uint32_t>(HW) * 64u;  // activation bytes per K-tile
  // every wave issues PPW pieces per K-tile (past the end: OOB, zeros into the pad)
  auto issue = [&](int kt) {
    const bool ok = kt < KT;
    const uint32_t st = lds0 + static_cast<uint32_t>((kt % NS) * STB);
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const bool real = ok && alds[i] != 0xFFFFFFFFu;
      dma_b128(wrs, real ? aoff[i] + static_cast<uint32_t>(kt) * 3072u : 0x80000000u,
               real ? st + alds[i] : lds0 + static_cast<uint32_t>(NS * STB));
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const bool real = ok && blds[i] != 0xFFFFFFFFu;
      const uint32_t vo = real && boff[i] != 0x80000000u ? boff[i] + static_cast<uint32_t>(kt) * kstep : 0x80000000u;
      const uint32_t dst = real ? st + blds[i] : lds0 + static_cast<uint32_t>(NS * STB);
      if constexpr (VEC == 4)
        dma_b128(xrs, vo, dst);
      else
        dma_b32(xrs, vo, dst);
    }
  };
  floatx16 acc[MI][NB];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

#pragma unroll
  for (int t = 0; t < NS - 1; ++t) issue(t);
  wait_vm<(NS - 2) * PPW>();
  __builtin_amdgcn_s_barrier();
  const int colw = 32 * NB * wc + lr;
  for (int kt = 0; kt < KT; ++kt) {
    issue(kt + NS - 1);
    const char* st = smem + (kt % NS) * STB;
    x6::Parts fa[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const char* f = st + (MI * wr + i) * 3072 + lane * 16;
      fa[i].h = *reinterpret_cast<const x6::bf16x8*>(f);
      fa[i].m = *reinterpret_cast<const x6::bf16x8*>(f + 1024);
      fa[i].l = *reinterpret_cast<const x6::bf16x8*>(f + 2048);
    }
    const float* bs = reinterpret_cast<const float*>(st + A_BYTES) + 8 * lh * BNc + colw;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = bs[e * BNc + 32 * j];
      x6::Parts bp;
      x6::split8_safe(v, bp);
#pragma unroll
      for (int i = 0; i < MI; ++i) acc[i][j] = x6::mfma6(fa[i], bp, acc[i][j]);
    }
    wait_vm<(NS - 2) * PPW>();  // this wave's pieces of K-tile kt + 1 have landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // ... and every wave's; stage kt % NS is free
    __builtin_amdgcn_sched_barrier(0);
  }
  Epi ep = P.e;
  conv_epilogue_nchw<MI, NB>(acc, P, ep, m0 + 32 * MI * wr, n0 + 32 * NB * wc, lr, lh);
  if (yoct != nullptr) octet_epilogue<MI, NB>(acc, P, ep, m0 + 32 * MI * wr, n0 + 32 * NB * wc, lr, lh, yoct, cout8);
}

// w [G*M][Cg][T] -> fragments [G][tiles_m][WR][Cg/16][T][term][64 lanes][8]:
// lane (lr, h) of fragment (kt, s) holds row 32 (tm WR + wr) + lr, channels
// 16 kt + 8 h .. + 7 at tap s.  One thread per (fragment, lane).
__global__ void __launch_bounds__(256) k_conv_cb_pack_x6(const float* __restrict__ w, char* __restrict__ out, int M,
                                                         int Cg, int T, int rblocks, int units) {
  const int KT = Cg >> 4;
  for (int u = blockIdx.x * blockDim.x + threadIdx.x; u < units; u += gridDim.x * blockDim.x) {
    const int lane = u & 63;
    int r = u >> 6;
    const int s = r % T;
    r /= T;
    const int kt = r % KT;
    r /= KT;
    const int rb = r % rblocks;  // tm WR + wr
    const int g = r / rblocks;
    const int m = rb * 32 + (lane & 31), c0 = kt * 16 + (lane >> 5) * 8;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e)
      v[e] = m < M ? w[((int64_t)g * M + m) * Cg * T + (int64_t)(c0 + e) * T + s] : 0.0f;
    x6::Parts t;
    x6::split8_safe(v, t);
    char* f = out + (int64_t)(u >> 6) * 3072 + lane * 16;
    *reinterpret_cast<x6::bf16x8*>(f) = t.h;
    *reinterpret_cast<x6::bf16x8*>(f + 1024) = t.m;
    *reinterpret_cast<x6::bf16x8*>(f + 2048) = t.l;
  }
}


// ---------------------------------------------------------------------------
// k_conv1_ring_x6: AlexNet conv1 (3 x 11 x 11, stride 4, 227 x 227 input, 96
// filters) as a persistent kernel whose input is split ONCE per element and
// whose B fragments are plain 8-byte LDS reads.
//
// One workgroup per CU walks tiles of 96 filters x 256 output positions of
// one image.  Its LDS holds three channel slots; slot c is the tile's input
// rows of channel c (32 rows: 6 output rows x stride 4 + 12 kernel rows),
// each element already split into its three bf16 terms, stored as plain rows
// [term][row][ic] (ROWE elements per row, columns >= W zero).
// K order ("quads"): a kernel row is padded to 12 columns = 3 quads of 4
// consecutive columns (column 11 has zero weights); the 99 quads (channel,
// kernel row, quad) are taken four per MFMA group, lane half h reading quads
// 4g + h and 4g + 2 + h of group g (25 groups; the 100th quad is padding).
// The im2col values of one quad at output column ow are input columns
// 4 ow + 4 kq .. + 3 of one row: 4 consecutive bf16 = one ds_read_b64 at a
// compile-time offset from a per-lane base (half 1 adds its own compile-time
// quad distance, one select per quad pair), and consecutive lanes (output
// columns) read consecutive 8-byte words, so a B fragment term is two
// ds_read_b64 with no gather VALU.  The padding costs 25 groups where 363
// items need 23 (round 3 padded the kernel rows to 12 as well: 27 groups).
// The slots are refilled for the next tile while this one computes: slot 0
// once group 8 (the last reader of channel 0) is done, slot 1 after group 16,
// slot 2 at the start of the tile it serves (read from group 16 on); three
// barriers per tile.  The weight fragments come from L2 into registers two
// groups ahead (fragment order, k_conv1_pack_x6).
namespace c1x6 {
constexpr int BM = 96, BN = 256;
// K in quads: (channel, kernel row, quad of 4 kernel columns; column 11 is
// the padding) = 3 x 11 x 3 = 99 quads, group g = quads 4g .. 4g + 3 (lane
// half h takes 4g + h and 4g + 2 + h): 25 groups, the last with one padded quad
constexpr int KR = 11, KQ = 3, C = 3, NQ = C * KR * KQ, G = (NQ + 3) / 4;
constexpr int ROWS = 32;                 // slot rows
// elements per slot row (>= 228: the last quad of output column 54 reads
// input column 227, which is zero).  ROWE = 24 (mod 32) 8-byte words: a
// 32-lane ds_read_b64 that wraps from output column 54 of one row to column 0
// four input rows down continues on the next bank pair but one (2-way on one
// pair at most), and rows stay 16-byte aligned for the staging writes
constexpr int ROWE = 248;
constexpr int TERMB = ROWS * ROWE * 2;   // bytes per term plane
constexpr int SLOTB = 3 * TERMB;         // bytes per slot
constexpr int QP = ROWE / 8;             // 8-column chunks per row
constexpr int CHUNKS = ROWS * QP;        // chunks per slot
constexpr int CPT = (CHUNKS + 255) / 256;  // chunks per thread
static_assert(3 * SLOTB + BM * 4 <= 160 * 1024, "LDS");
// first / last group reading channel c (quads 33 c .. 33 c + 32)
constexpr int first_group(int c) { return (c * KR * KQ) / 4; }
constexpr int last_group(int c) { return (c * KR * KQ + KR * KQ - 1) / 4; }
// LDS byte offset of quad q (relative to the lane's base): channel, row, column
constexpr int quad_off(int q) {
  return (q / (KR * KQ)) * SLOTB + (((q / KQ) % KR) * ROWE + 4 * (q % KQ)) * 2;
}
// the lane half 1 reads quad q + 1 where half 0 reads quad q (q = 4g + 2e):
// its extra byte offset (0 for the padded quad, which reads quad q again)
constexpr int half_delta(int q) { return q + 1 < NQ ? quad_off(q + 1) - quad_off(q) : 0; }
// mask of a quad's upper dword: column 11 (element 3 of a row's last quad)
// is padding; the padded quad is zero altogether
constexpr uint32_t hi_mask(int q) { return q >= NQ ? 0u : (q % KQ == KQ - 1 ? 0x0000FFFFu : 0xFFFFFFFFu); }
constexpr uint32_t lo_mask(int q) { return q >= NQ ? 0u : 0xFFFFFFFFu; }
}  // namespace c1x6

// RRAM_C1_STAMP (diagnostic build only, never the product): per-group
// s_memtime cycle sums of k_conv1_ring_x6 (slots 0 .. G - 1: group g's
// compute, G .. G + 2: the three barriers, G + 3: per-tile setup, G + 4: tile
// count), summed over waves into g_c1_stamp (read by rram_debug_c1_stamps)
#ifdef RRAM_C1_STAMP
__device__ unsigned long long g_c1_stamp[64];
__device__ __forceinline__ unsigned long long c1_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#endif
template <int W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_conv1_ring_x6(Params P, const uint16_t* __restrict__ wpack, int tiles_per_img, int tiles) {
  using namespace c1x6;
#ifdef RRAM_C1_STAMP
  __shared__ unsigned long long st_lds[4][32];
  if ((threadIdx.x & 63) < 32) st_lds[threadIdx.x >> 6][threadIdx.x & 63] = 0;
  unsigned long long tprev = 0;
  auto stamp_to = [&](int slot) __attribute__((always_inline)) {
    const unsigned long long tn = c1_stamp();
    if ((threadIdx.x & 63) == 0) st_lds[threadIdx.x >> 6][slot] += tn - tprev;
    tprev = tn;
  };
#define RRAM_C1_ST(slot) stamp_to(slot)
#else
#define RRAM_C1_ST(slot)
#endif
  constexpr int OW = (W - 11) / 4 + 1, MI = 3;
  static_assert(4 * (OW - 1) + 4 * KQ <= ROWE, "slot rows too short");
  __shared__ __attribute__((aligned(16))) char smem[3 * SLOTB];
  __shared__ float bias_lds[BM];
  if (threadIdx.x < BM)
    bias_lds[threadIdx.x] = (P.e.bias != nullptr && (int)threadIdx.x < P.M) ? P.e.bias[threadIdx.x] : 0.0f;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int HWo = P.cv.howo.d, H = P.cv.H;
  const int nwg = gridDim.x;
  // (the lambdas below capture these, never P: a by-reference capture of the
  // kernel-argument struct copies all of it into private memory)
  const float* const xin = P.b.p;
  const int in_bytes = static_cast<int>(P.cv.in_bytes);

  // ---- staging: chunk k of this thread = (slot row, 8 input columns) ----
  float sv[2][8];  // two chunks in flight
  // branch-free: an element outside the image row (ic >= W), a row at or past
  // H (kernel row 11 of the last output row: zero weights, so it must hold no
  // Inf / NaN), or a chunk of a tile that does not exist (t >= tiles: the
  // refill then writes zeros into a slot no later group reads) loads from past
  // the buffer's range, i.e. zero
  struct TileRef {
    int img, f;
  };
  auto tile_ref = [&](int t) __attribute__((always_inline)) {
    TileRef r;
    const int img = t / tiles_per_img, tin = t - img * tiles_per_img;
    r.img = __builtin_amdgcn_readfirstlane(t < tiles ? img : -1);
    r.f = __builtin_amdgcn_readfirstlane((tin * BN) / OW);
    return r;
  };
  // chunk index: the last thread group's extra chunks (q >= CHUNKS) redo chunk
  // CHUNKS - 1 (same loads, same values, same LDS bytes: a benign duplicate
  // write), so the refill has no branch for the scheduler to stop at
  auto chunk_of = [&](int k) __attribute__((always_inline)) { return min((int)threadIdx.x + k * 256, CHUNKS - 1); };
  auto stage_load = [&](const TileRef& tr, int c, int k, float (&v)[8]) {
    const int q = chunk_of(k);
    const int ri = q / QP, qp = q - ri * QP;
    const bool ok = tr.img >= 0 && 4 * tr.f + ri < H;
    const int rowoff = (((tr.img * 3 + c) * H + 4 * tr.f + ri) * W + 8 * qp) * 4;
    const uint32_t voff = ok ? static_cast<uint32_t>(rowoff) : 0x80000000u;
    // (built here from the kernel argument: a descriptor captured by reference
    // lands in private memory and every load becomes a waterfall loop)
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xin), 0, in_bytes, 0x00020000);
#ifdef RRAM_C1_LOAD128
    // (A/B: two 16-byte loads at 4-byte alignment per chunk instead of eight 4-byte loads)
    typedef float float4x __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4x q = __builtin_bit_cast(
          float4x, __builtin_amdgcn_raw_buffer_load_b128(xrs, static_cast<int>(voff + 16 * h), 0, 0));
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * h + e] = q[e];
    }
#else
#pragma unroll
    for (int e = 0; e < 8; ++e)
      v[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xrs, static_cast<int>(voff + 4 * e), 0, 0));
#endif
  };
  auto stage_store = [&](int c, int k, float (&v)[8]) {
    const int q = chunk_of(k);
    const int ri = q / QP, qp = q - ri * QP;
    // columns past the image row loaded the next row's (or, past the buffer,
    // zero) values: zero them (kernel column 11's weights are zero, and an
    // Inf there would make 0 * Inf = NaN)
    const int nv = W - 8 * qp;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = e < nv ? v[e] : 0.0f;
    char* base = smem + c * SLOTB + (ri * ROWE + 8 * qp) * 2;
    x6::Parts t;
    x6::split8_safe(v, t);
    *reinterpret_cast<x6::bf16x8*>(base) = t.h;
    *reinterpret_cast<x6::bf16x8*>(base + TERMB) = t.m;
    *reinterpret_cast<x6::bf16x8*>(base + 2 * TERMB) = t.l;
  };
  // whole slot at once (first tile)
  auto fill_slot = [&](const TileRef& tr, int c) __attribute__((always_inline)) {
    for (int k = 0; k < CPT; ++k) {
      stage_load(tr, c, k, sv[0]);
      stage_store(c, k, sv[0]);
    }
  };
  // spread refill: step 0 loads chunks 0, 1; step 1 stores them and loads 2, 3; step 2 stores 2, 3
  static_assert(CPT <= 4, "refill schedule covers 4 chunks per thread");
  // one register set u of refill step `step`: store the chunk it loaded in
  // the previous step, then load its chunk of this step
  auto refill_part = [&](const TileRef& tr, int c, int step, int u) __attribute__((always_inline)) {
    if (step > 0 && 2 * (step - 1) + u < CPT) stage_store(c, 2 * (step - 1) + u, sv[u]);
    if (step < 2 && 2 * step + u < CPT) stage_load(tr, c, 2 * step + u, sv[u]);
  };

  // the weight fragments are the same for every tile: the base address is
  // laundered once per tile so the tile loop does not hoist all groups'
  // loads out of itself.  (With the round-5 refill schedule the allocator
  // kept 20 bytes of scratch at 512 registers; the round-6 one-chunk-per-
  // group refill needs 483 and none)
  const x6::bf16x8* ap = reinterpret_cast<const x6::bf16x8*>(wpack) + lane;
  auto launder_a = [&]() __attribute__((always_inline)) {
    int z = 0;
    asm volatile("" : "+s"(z));
    ap = reinterpret_cast<const x6::bf16x8*>(wpack) + lane + z;
  };
  auto load_a = [&](x6::bf16x8 (&f)[MI][3], int g) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int tt = 0; tt < 3; ++tt) f[i][tt] = ap[((g * MI + i) * 3 + tt) * 64];
  };
  auto lds_barrier = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes done
    __builtin_amdgcn_s_barrier();
  };

  int t = blockIdx.x;
  if (t < tiles) {
    const TileRef tr = tile_ref(t);
    fill_slot(tr, 0);
    fill_slot(tr, 1);
    fill_slot(tr, 2);
  }
  lds_barrier();
  // Accumulators double-buffered across tiles: tile t computes into acc[c]
  // while its first 12 groups store tile t - nwg's acc[1 - c] (8 values per
  // group, between the MFMAs), so the epilogue is not a serial tail per tile.
  // Stores of lanes past the image's last position, and of the tile before
  // the first, go to an out-of-range offset (dropped by the buffer range check).
  floatx16 acc[2][MI][2];
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(P.e.C, 0, 0x7FFFFFFF, 0x00020000);
  const bool relu = P.e.relu != 0;
  const int mw = 4 * lh;
  uint32_t obase[2] = {0x80000000u, 0x80000000u};  // per column block: previous tile's output offset (bytes)
  auto store_part = [&](const floatx16 (&pa)[MI][2], int s8) __attribute__((always_inline)) {
    // values 8 s8 .. 8 s8 + 7 of the 96 (s8 < 12; block (i, j) = v / 16, row r = v % 16)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int v = 8 * s8 + e, i = (v >> 4) / 2, j = (v >> 4) & 1, r = v & 15;
      const int dr = i * 32 + (r & 3) + 8 * (r >> 2);
      const float o = pa[i][j][r] + bias_lds[mw + dr];
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, relu ? fmaxf(o, 0.0f) : o), ors,
                                            static_cast<int>(obase[j]), dr * HWo * 4, 0);
    }
  };
  auto tile_body = [&](auto cc, int t) __attribute__((always_inline)) {
    constexpr int CUR = decltype(cc)::value;
#ifdef RRAM_C1_STAMP
    tprev = c1_stamp();
    if ((threadIdx.x & 63) == 0) st_lds[threadIdx.x >> 6][G + 4] += 1;
#endif
    const TileRef cur = tile_ref(t), nxt = tile_ref(t + nwg);
    const int img = cur.img, sp0 = (t - img * tiles_per_img) * BN, f = cur.f;
    // per-lane slot byte offsets (term 0, quad 0) of this wave's two 32-column blocks
    uint32_t lb[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int sp = min(sp0 + wave * 64 + j * 32 + lr, HWo - 1);
      const int oh = sp / OW, ow = sp - oh * OW;
      lb[j] = static_cast<uint32_t>((4 * (oh - f) * ROWE + 4 * ow) * 2);
    }
    // B fragment term tt of column block j for group g: quads 2g, 2g + 1 =
    // two ds_read_b64 at compile-time offsets, issued one group ahead
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    // the padded K items (kernel column 11, the 100th quad) carry zero
    // weights but read real input elements; their B values are zeroed too,
    // so a non-finite input outside the 11 x 11 window never meets a zero
    // weight (0 * Inf = NaN where fp32 has no such product).  Lane half h
    // reads quads 4g + 2e + h: its offset and masks are the half's own
    // compile-time constants, picked per lane once per quad pair.
    auto pick = [&](uint32_t h0, uint32_t h1) __attribute__((always_inline)) { return lh ? h1 : h0; };
    auto mask_q = [&](u32x2 v, int q0) __attribute__((always_inline)) {
      if (lo_mask(q0) != 0xFFFFFFFFu || lo_mask(q0 + 1) != 0xFFFFFFFFu) v[0] &= pick(lo_mask(q0), lo_mask(q0 + 1));
      if (hi_mask(q0) != 0xFFFFFFFFu || hi_mask(q0 + 1) != 0xFFFFFFFFu) v[1] &= pick(hi_mask(q0), hi_mask(q0 + 1));
      return v;
    };
    auto read_part = [&](x6::Parts (&F)[2], int g, int part) __attribute__((always_inline)) {
      const int j = part / 3, tt = part % 3;
      const int qa = 4 * g, qb = 4 * g + 2;
      const char* ba = smem + lb[j] + (lh ? half_delta(qa) : 0) + tt * TERMB;
      const char* bb = smem + lb[j] + (lh ? half_delta(qb) : 0) + tt * TERMB;
      const u32x2 lo = mask_q(*reinterpret_cast<const u32x2*>(ba + quad_off(qa)), qa);
      const u32x2 hi = mask_q(*reinterpret_cast<const u32x2*>(bb + quad_off(qb)), qb);
      const x6::bf16x8 v = __builtin_bit_cast(x6::bf16x8, u32x4{lo[0], lo[1], hi[0], hi[1]});
      if (tt == 0) F[j].h = v;
      else if (tt == 1) F[j].m = v;
      else F[j].l = v;
    };
    floatx16 (&ac)[MI][2] = acc[CUR];
    const floatx16 (&ap_)[MI][2] = acc[1 - CUR];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) ac[i][j][r] = 0.0f;
    x6::bf16x8 fg[3][MI][3];
    launder_a();
    load_a(fg[0], 0);
    load_a(fg[1], 1);
    x6::Parts F[2][2];
#pragma unroll
    for (int part = 0; part < 6; ++part) read_part(F[0], 0, part);
    RRAM_C1_ST(G + 3);
    static_for<0, G>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      x6::Parts (&fc)[2] = F[g & 1];
      x6::Parts (&fn)[2] = F[(g + 1) & 1];
      if (g + 2 < G) load_a(fg[(g + 2) % 3], g + 2);
      // slot refills (see the header): channel 2 of this tile at groups 1, 3, 5;
      // channel 0 / 1 of the next tile two, four and six groups after their last reader
#ifndef RRAM_C1_SPREAD
#define RRAM_C1_SPREAD 1
#endif
#if !RRAM_C1_SPREAD
      auto refill = [&](int u) __attribute__((always_inline)) {
        // (unconditional: the first tile re-fills slot 2 with what the prologue
        // put there; past the last tile the loads return zeros into dead slots)
        if (g >= 1 && g <= 5 && (g & 1)) refill_part(cur, 2, (g - 1) / 2, u);
        constexpr int d0 = g - last_group(0) - 1, d1 = g - last_group(1) - 1;
        if (d0 >= 0 && d0 <= 4 && (d0 & 1) == 0) refill_part(nxt, 0, d0 / 2, u);
        if (d1 >= 0 && d1 <= 4 && (d1 & 1) == 0) refill_part(nxt, 1, d1 / 2, u);
      };
#else
      // round 6: one chunk per group over CPT + 1 consecutive groups per slot
      // -- load chunk s at step s, store it at step s + 1 -- instead of two
      // per step on every other group (RRAM_C1_SPREAD=0); the same windows:
      // slot 2 before the barrier after group last_group(0), slots 0 / 1
      // before the next barriers.  483 VGPRs and no scratch (was 512 + 20 B),
      // conv1 -0.6 % (profiles/r06_ab_conv1.txt)
      auto refill1 = [&](const TileRef& tr, int c, int st) __attribute__((always_inline)) {
        if (st > 0 && st - 1 < CPT) stage_store(c, st - 1, sv[(st - 1) & 1]);
        if (st < CPT) stage_load(tr, c, st, sv[st & 1]);
      };
      auto refill = [&](int u) __attribute__((always_inline)) {
        if (u != 0) return;
        if (g >= 1 && g <= 1 + CPT) refill1(cur, 2, g - 1);
        constexpr int d0 = g - last_group(0) - 1, d1 = g - last_group(1) - 1;
        if (d0 >= 0 && d0 <= CPT) refill1(nxt, 0, d0);
        if (d1 >= 0 && d1 <= CPT) refill1(nxt, 1, d1);
      };
#endif
#pragma unroll
      for (int q = 0; q < 2 * MI; ++q) {
        const int i = q >> 1, j = q & 1;
        const auto& fa = fg[g % 3][i];
        ac[i][j] = x6::mfma6(x6::Parts{fa[0], fa[1], fa[2]}, fc[j], ac[i][j]);
        // the next group's B fragment part q under MFMA6 block q
        if (g + 1 < G) read_part(fn, g + 1, q);
        if (q == 1) refill(0);
        if (q == 4) refill(1);
        // the previous tile's outputs: groups 0 .. 11, 8 values per group
        if (g < 12 && q == 3) store_part(ap_, g);
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
          __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // VALU
          __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
          __builtin_amdgcn_sched_group_barrier(0x020, 3, 0);  // VMEM read
          __builtin_amdgcn_sched_group_barrier(0x040, 1, 0);  // VMEM write
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      // barriers: after the last readers of channel 0 / 1 (their slots are then
      // refilled) and at the end of the tile
      RRAM_C1_ST(g);
      if (g == last_group(0) || g == last_group(1) || g == G - 1) {
        lds_barrier();
        RRAM_C1_ST(G + (g == last_group(0) ? 0 : g == last_group(1) ? 1 : 2));
      }
    });
    // this tile's output offsets, stored under the next tile (bias + ReLU:
    // conv_epilogue_nchw's arithmetic; the bias from LDS)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int sp = sp0 + wave * 64 + j * 32 + lr;
      obase[j] = sp < HWo ? static_cast<uint32_t>(((int64_t)img * P.e.cimg + sp + (int64_t)mw * HWo) * 4)
                          : 0x80000000u;
    }
  };
  for (; t < tiles; t += 2 * nwg) {
    tile_body(std::integral_constant<int, 0>{}, t);
    if (t + nwg >= tiles) {
#pragma unroll
      for (int s8 = 0; s8 < 12; ++s8) store_part(acc[0], s8);
#ifdef RRAM_C1_STAMP
      if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < G + 5; ++k) atomicAdd(&g_c1_stamp[k], st_lds[threadIdx.x >> 6][k]);
#endif
      return;
    }
    tile_body(std::integral_constant<int, 1>{}, t + nwg);
  }
  if (t - nwg < tiles && t != (int)blockIdx.x) {
#pragma unroll
    for (int s8 = 0; s8 < 12; ++s8) store_part(acc[1], s8);
  }
#ifdef RRAM_C1_STAMP
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < G + 5; ++k) atomicAdd(&g_c1_stamp[k], st_lds[threadIdx.x >> 6][k]);
#endif
}
#undef RRAM_C1_ST

// Weight repack for k_conv1_ring_x6: w [M][3][11][11] -> fragments
// [27 groups][3 row blocks][3 terms][64 lanes][8 bf16]; lane (lr, h) of
// fragment (g, i): row 32 i + lr, items j of half h = quads 2 g, 2 g + 1 in
// the kernel's quad order (kernel row 6 h + (qi / 3) % 6, columns 4 (qi % 3)
// .. + 3; row 11 and column 11 zero).
__global__ void __launch_bounds__(256) k_conv1_pack_x6(const float* __restrict__ w, char* __restrict__ out, int M,
                                                       int units) {
  using namespace c1x6;
  for (int u = blockIdx.x * blockDim.x + threadIdx.x; u < units; u += gridDim.x * blockDim.x) {
    const int lane = u & 63, i = (u >> 6) % 3, g = (u >> 6) / 3;
    const int row = 32 * i + (lane & 31), h = lane >> 5;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int q = 4 * g + 2 * (j >> 2) + h;  // the quad lane half h reads for items j
      const int c = q / (KR * KQ), kh = (q / KQ) % KR, kw = 4 * (q % KQ) + (j & 3);
      v[j] = (row < M && q < NQ && kw < 11) ? w[((row * 3 + c) * 11 + kh) * 11 + kw] : 0.0f;
    }
    x6::Parts t;
    x6::split8_safe(v, t);
    char* f = out + (int64_t)(u >> 6) * 3072 + lane * 16;
    *reinterpret_cast<x6::bf16x8*>(f) = t.h;
    *reinterpret_cast<x6::bf16x8*>(f + 1024) = t.m;
    *reinterpret_cast<x6::bf16x8*>(f + 2048) = t.l;
  }
}

// ---------------------------------------------------------------------------
// k_conv_s2_x6: GoogLeNet conv1 (3 channels, 7 x 7, stride 2, 64 filters) on
// the bf16x6 engine; the fp32 table-gather GEMM ran it before (round 6).
//
// A workgroup computes one tile of 64 filters x 256 output positions of one
// image, two workgroups per CU (one stages while the other computes).  The
// tile's input rows (4 output rows at most: 6 + 7 = 13 input rows per
// channel) are staged once, split into their three bf16 terms, as plain rows
// [channel][term][row][element], element e = input column e - pw (padding and
// columns past the row zero).  K order: a K row is (channel, kernel row), 21
// of them, each padded to 8 kernel columns (column 7 has zero weights and
// masked B values); MFMA group g takes rows 2g (lane half 0) and 2g + 1 (half
// 1), 11 groups, row 21 padding.  The im2col values of one K row at output
// column ow are the 8 consecutive elements 2 ow .. 2 ow + 7 of one slot row:
// a B fragment term is 16 bytes at a 4-byte aligned per-lane offset (two
// ds_read2_b32), consecutive lanes 4 bytes apart.  The weight fragments come
// from L2 into registers two groups ahead (fragment order, k_conv_s2_pack_x6).
namespace c7x6 {
constexpr int C = 3, KS = 7, S = 2, KC = 8;
constexpr int R = C * KS;            // K rows (channel, kernel row)
constexpr int G = (R + 1) / 2;       // MFMA groups (row 21 is padding)
constexpr int BM = 64, MI = 2;
constexpr int ROWE = 232;            // elements per slot row: S (OW - 1) + KC <= ROWE
constexpr int QR = ROWE / 4;         // 4-element staging chunks per row
static_assert((ROWE * 2) % 8 == 0, "8-byte staging stores");
// tile of 64 filters x 128 NBW positions (each wave NBW 32-column blocks)
template <int NBW>
struct Tile {
  static constexpr int BN = 128 * NBW;
  static constexpr int OR = NBW == 2 ? 4 : 3;     // output rows a tile may touch (host: OW large enough)
  static constexpr int SR = S * (OR - 1) + KS;    // slot rows per channel: 13 / 11
  static constexpr int TERMB = SR * ROWE * 2;     // bytes per (channel, term) plane
  static constexpr int CHB = 3 * TERMB;           // bytes per channel
  static constexpr int NCH = C * SR * QR;         // staging chunks per tile
  static constexpr int CPT = (NCH + 255) / 256;
  static constexpr int WGS = NBW == 2 ? 2 : 3;    // workgroups per CU
  static_assert(WGS * (C * CHB + BM * 4) <= 160 * 1024, "LDS");
  // LDS byte offset of K row rr (0 for the padding row, whose B values are masked)
  static constexpr int row_off(int rr) { return rr < R ? (rr / KS) * CHB + (rr % KS) * ROWE * 2 : 0; }
};
}  // namespace c7x6

template <int NBW>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NBW == 2 ? 2 : 3, NBW == 2 ? 2 : 3)))
k_conv_s2_x6(Params P, const x6::bf16x8* __restrict__ wpack, int tiles_per_img, int tiles) {
  using namespace c7x6;
  using T = Tile<NBW>;
  constexpr int BN = T::BN, SR = T::SR, TERMB = T::TERMB, CHB = T::CHB, NCH = T::NCH, CPT = T::CPT;
  __shared__ __attribute__((aligned(16))) char smem[C * CHB];
  __shared__ float bias_lds[BM];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  // XCD-aware order: consecutive tiles (which share input rows) on one XCD
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, loc = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int t = __builtin_amdgcn_readfirstlane((xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc);
  if (t >= tiles) return;  // (uniform per workgroup; nwg == tiles)
  const int img = t / tiles_per_img, sp0 = (t - img * tiles_per_img) * BN;
  const int HWo = P.cv.howo.d, OW = P.cv.Wo, H = P.cv.H, W = P.cv.W;
  const int f = sp0 / OW;
  if (threadIdx.x < BM)
    bias_lds[threadIdx.x] = (P.e.bias != nullptr && (int)threadIdx.x < P.M) ? P.e.bias[threadIdx.x] : 0.0f;

  // ---- staging: chunk q = (channel, slot row, 4 elements), one 4-byte load
  // per element (an element outside the image, in a row outside it or in the
  // left / right padding loads from past the buffer's range, i.e. zero)
  {
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(P.b.p), 0, static_cast<int>(P.cv.in_bytes), 0x00020000);
    const int row0 = S * f - P.cv.ph;
    float v[CPT][4];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int q = min((int)threadIdx.x + 256 * k, NCH - 1);  // (extra chunks redo the last: same bytes)
      const int c = q / (SR * QR), rem = q - c * (SR * QR), ri = rem / QR, e4 = rem - ri * QR;
      const int row = row0 + ri, col0 = 4 * e4 - P.cv.pw;
      const bool rok = static_cast<unsigned>(row) < static_cast<unsigned>(H);
      const int base = ((img * C + c) * H + row) * W + col0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool ok = rok && static_cast<unsigned>(col0 + e) < static_cast<unsigned>(W);
        v[k][e] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(xrs, ok ? 4 * (base + e) : static_cast<int>(0x80000000u), 0, 0));
      }
    }
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int q = min((int)threadIdx.x + 256 * k, NCH - 1);
      const int c = q / (SR * QR), rem = q - c * (SR * QR), ri = rem / QR, e4 = rem - ri * QR;
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      u32x2 hw, mw, lw;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const x6::float2v xv = {v[k][2 * p], v[k][2 * p + 1]};
        x6::bf16x2 h;
        const x6::float2v r1 = x6::bf16_high_safe(xv, h);
        const x6::bf16x2 m = __builtin_convertvector(x6::clamp_bf16(r1), x6::bf16x2);
        const x6::float2v r2 = r1 - __builtin_convertvector(m, x6::float2v);
        const x6::bf16x2 l = __builtin_convertvector(r2, x6::bf16x2);
        hw[p] = __builtin_bit_cast(uint32_t, h);
        mw[p] = __builtin_bit_cast(uint32_t, m);
        lw[p] = __builtin_bit_cast(uint32_t, l);
      }
      char* dst = smem + c * CHB + (ri * ROWE + 4 * e4) * 2;
      *reinterpret_cast<u32x2*>(dst) = hw;
      *reinterpret_cast<u32x2*>(dst + TERMB) = mw;
      *reinterpret_cast<u32x2*>(dst + 2 * TERMB) = lw;
    }
  }
  __syncthreads();

  // ---- K loop: 11 groups x (2 row blocks x 2 column blocks) x 6 MFMAs ----
  uint32_t lb[NBW];  // per-lane slot byte offset of column block j (K row 0)
#pragma unroll
  for (int j = 0; j < NBW; ++j) {
    const int sp = min(sp0 + wave * 32 * NBW + j * 32 + lr, HWo - 1);
    const int oh = sp / OW, ow = sp - oh * OW;
    lb[j] = static_cast<uint32_t>((S * (oh - f) * ROWE + S * ow) * 2);
  }
  const x6::bf16x8* ap = wpack + lane;
  auto load_a = [&](x6::bf16x8 (&fr)[MI][3], int g) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int tt = 0; tt < 3; ++tt) fr[i][tt] = ap[((g * MI + i) * 3 + tt) * 64];
  };
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  // B term tt of column block j for group g: K row 2 g + lh; kernel column 7
  // (the upper half of dword 3) and the padding row are zeroed, so a
  // non-finite input never meets a padded zero weight.  The raw reads are
  // issued a group ahead and masked at use, so no wait for them sits in
  // front of the current group's MFMAs
  auto read_b = [&](u32x4 (&Bq)[NBW][3], int g) __attribute__((always_inline)) {
    const uint32_t ho = lh ? static_cast<uint32_t>(T::row_off(2 * g + 1)) : static_cast<uint32_t>(T::row_off(2 * g));
#pragma unroll
    for (int j = 0; j < NBW; ++j)
#pragma unroll
      for (int tt = 0; tt < 3; ++tt) {
        const uint32_t* p = reinterpret_cast<const uint32_t*>(smem + lb[j] + ho + tt * TERMB);
        Bq[j][tt] = u32x4{p[0], p[1], p[2], p[3]};
      }
  };
  auto parts_b = [&](const u32x4 (&Bq)[NBW][3], int j, int g) __attribute__((always_inline)) {
    const uint32_t m3 = (2 * g + 1 < R || lh == 0) ? 0x0000FFFFu : 0u;
    const uint32_t m02 = (2 * g + 1 < R || lh == 0) ? 0xFFFFFFFFu : 0u;
    x6::bf16x8 t[3];
#pragma unroll
    for (int tt = 0; tt < 3; ++tt) {
      u32x4 d = Bq[j][tt];
      asm volatile("" : "+v"(d));  // (keeps the masks here: hoisted to the reads they wait for them)
      if (2 * g + 1 >= R) {
        d[0] &= m02;
        d[1] &= m02;
        d[2] &= m02;
      }
      d[3] &= m3;
      t[tt] = __builtin_bit_cast(x6::bf16x8, d);
    }
    return x6::Parts{t[0], t[1], t[2]};
  };
  floatx16 acc[MI][NBW];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NBW; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  x6::bf16x8 fa[3][MI][3];
  load_a(fa[0], 0);
  load_a(fa[1], 1);
  u32x4 Bq[2][NBW][3];
  read_b(Bq[0], 0);
  // (scheduling barriers keep the prefetches where they are issued: left to
  // itself the scheduler sinks each weight load next to its first MFMA and
  // waits the full L2 latency there)
  __builtin_amdgcn_sched_barrier(0);
  static_for<0, G>([&](auto gc) {
    constexpr int g = decltype(gc)::value;
    if (g + 2 < G) load_a(fa[(g + 2) % 3], g + 2);
    if (g + 1 < G) read_b(Bq[(g + 1) & 1], g + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      const x6::Parts b = parts_b(Bq[g & 1], j, g);
#pragma unroll
      for (int i = 0; i < MI; ++i)
        acc[i][j] = x6::mfma6(x6::Parts{fa[g % 3][i][0], fa[g % 3][i][1], fa[g % 3][i][2]}, b, acc[i][j]);
    }
    __builtin_amdgcn_sched_barrier(0);
  });

  // ---- epilogue: bias + ReLU (conv_epilogue_nchw's arithmetic), NCHW ----
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(P.e.C, 0, 0x7FFFFFFF, 0x00020000);
  const bool relu = P.e.relu != 0;
  float bv[MI][16];  // (all bias reads before the first store: a store between them orders each read)
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) bv[i][r] = bias_lds[i * 32 + 4 * lh + (r & 3) + 8 * (r >> 2)];
#pragma unroll
  for (int j = 0; j < NBW; ++j) {
    const int sp = sp0 + wave * 32 * NBW + j * 32 + lr;
    const uint32_t ob = sp < HWo ? static_cast<uint32_t>(((int64_t)img * P.e.cimg + sp) * 4) : 0x80000000u;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = i * 32 + 4 * lh + (r & 3) + 8 * (r >> 2);
        const float o = acc[i][j][r] + bv[i][r];
        if (m < P.M)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, relu ? fmaxf(o, 0.0f) : o), ors,
                                                static_cast<int>(ob), m * HWo * 4, 0);
      }
  }
}

// Weight repack for k_conv_s2_x6: w [M][3][7][7] -> fragments
// [11 groups][2 row blocks][3 terms][64 lanes][8 bf16]; lane (lr, h) of
// fragment (g, i): filter 32 i + lr, K row 2 g + h = (channel, kernel row),
// items = kernel columns 0 .. 7 (column 7, row 21 and filters >= M zero).
__global__ void __launch_bounds__(256) k_conv_s2_pack_x6(const float* __restrict__ w, char* __restrict__ out, int M,
                                                         int units) {
  using namespace c7x6;
  for (int u = blockIdx.x * blockDim.x + threadIdx.x; u < units; u += gridDim.x * blockDim.x) {
    const int lane = u & 63, i = (u >> 6) % MI, g = (u >> 6) / MI;
    const int m = 32 * i + (lane & 31), rr = 2 * g + (lane >> 5);
    const int c = rr / KS, kr = rr % KS;
    float v[8];
#pragma unroll
    for (int kc = 0; kc < 8; ++kc)
      v[kc] = (m < M && rr < R && kc < KS) ? w[((m * C + c) * KS + kr) * KS + kc] : 0.0f;
    x6::Parts tp;
    x6::split8_safe(v, tp);
    char* o = out + (int64_t)(u >> 6) * 3072 + lane * 16;
    *reinterpret_cast<x6::bf16x8*>(o) = tp.h;
    *reinterpret_cast<x6::bf16x8*>(o + 1024) = tp.m;
    *reinterpret_cast<x6::bf16x8*>(o + 2048) = tp.l;
  }
}

// Weight repack for k_conv_patch_x6: w [G*M][C*T] -> bf16 terms
// [G][tiles_m][ktiles][64 MI][RLB]: row = [group g][half h][term][8 steps] + pad.
// One thread per (row, group, half): 8 weights in, 48 bytes out.
__global__ void __launch_bounds__(256) k_conv_patch_pack_x6(const float* __restrict__ w, char* __restrict__ out, int G,
                                                            int M, int C, int T, int CPH, int G8, int RLB, int BMc,
                                                            int tiles_m, int ktiles, int units) {
  for (int u = blockIdx.x * blockDim.x + threadIdx.x; u < units; u += gridDim.x * blockDim.x) {
    int r = u;
    const int h = r & 1;
    r >>= 1;
    const int gg = r % G8;
    r /= G8;
    const int row = r % BMc;
    r /= BMc;
    const int kt = r % ktiles;
    r /= ktiles;
    const int tm = r % tiles_m;
    const int g = r / tiles_m;
    const int m = tm * BMc + row;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int sx = 8 * gg + j;
      v[j] = 0.0f;
      if (sx < CPH * T && m < M) {
        const int c = kt * 2 * CPH + h * CPH + sx / T;
        v[j] = w[((int64_t)g * M + m) * C * T + (int64_t)c * T + (sx % T)];
      }
    }
    char* rowp = out + ((((int64_t)g * tiles_m + tm) * ktiles + kt) * BMc + row) * RLB;
    x6::store_terms8(v, rowp + (gg * 2 + h) * 48);
    if (gg == G8 - 1 && h == 1) *reinterpret_cast<uint4*>(rowp + G8 * 96) = make_uint4(0, 0, 0, 0);
  }
}


// ---------------------------------------------------------------------------
// k_gemm_x6: C[M][N] = A[M][K] . B[N][K]^T (the InnerProduct forward,
// inner_product_layer.cu:9-30, and any NoTrans x Trans GEMM) on the bf16
// matrix cores with the same exact three-term split as k_conv_patch_x6.
// A (the activations: M = images) is split once by k_pack_rows_x6 into K-tile
// slabs of bf16 terms in fragment order; B (the weights, streamed from HBM
// once per forward) is loaded fp32 by LDS-DMA and split in registers after
// the LDS read.  Tile 32 MI x 256: wave w owns all rows x columns
// 64 w .. 64 w + 63; K-tiles of 32 (two MFMA groups); split-K over z with
// partial slabs reduced by k_splitk_reduce.
// K order inside a K-tile: group g, lane half h holds k = 16 h + 8 g + j
// (the B rows' 16-byte quads 4h + 2g + u, u = 0, 1, swizzled as k_gemm2).
#ifndef RRAM_FC_ABLATE
#define RRAM_FC_ABLATE 0
#endif
namespace gx6 {
constexpr int KT = 32;
constexpr int RLB = 2 * 96 + 16;  // packed A row bytes per K-tile ([g][h][term][8 bf16] + pad, RLB/16 odd)
}  // namespace gx6

// The activation slabs (L2-resident) are double-buffered one K-tile ahead;
// the weights (streamed from HBM) go through a 3-stage ring two K-tiles
// ahead, so their HBM latency has 1.5 K-tiles to land: per K-tile the A
// pieces of t + 1 are issued first, then the B pieces of t + 2, and the end
// of the tile waits with vmcnt(B pieces) (the B of t + 1, issued a tile
// earlier, and the A of t + 1 have then landed).
template <int MI, int NJ>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_gemm_x6(Params P, const uint16_t* __restrict__ apack, int ktiles_all, int ktc) {
  using namespace g2;
  // tile 32 MI x 128 NJ: wave w owns all rows x columns 32 NJ w .. 32 NJ w + 32 NJ - 1
  constexpr int BMc = 32 * MI, BNc = 128 * NJ, KT = gx6::KT;
  constexpr int A_B = BMc * gx6::RLB;
  constexpr int A_DMA = ((A_B + 1023) / 1024 + 3) / 4;
  constexpr int A_REGB = A_DMA * 4 * 1024;
  constexpr int B_DMA = 4 * NJ;                          // 1 KB pieces (8 rows x 32 k) per wave
  constexpr int B_REGB = BNc * KT * 4, NBS = 3;
  constexpr int NVM = A_DMA + B_DMA;
  static_assert(2 * A_REGB + NBS * B_REGB <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[2 * A_REGB + NBS * B_REGB];
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem));

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lr = lane & 31, lh = lane >> 5;

  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, loc = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int tid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int tm = __builtin_amdgcn_readfirstlane(tid % P.tiles_m);
  const int tn = __builtin_amdgcn_readfirstlane((tid / P.tiles_m) % P.tiles_n);
  const int z = __builtin_amdgcn_readfirstlane(tid / (P.tiles_m * P.tiles_n));
  const int n0 = tn * BNc, m0 = tm * BMc;
  const int kt0 = z * ktc;
  const int nt = min(ktiles_all, kt0 + ktc) - kt0;  // >= 1 (host)
  float* part = P.split > 1 ? P.ws + (int64_t)z * P.M * P.N : nullptr;

  const uint16_t* abase = apack + ((int64_t)tm * ktiles_all + kt0) * (A_B / 2);
  const int4v arsrc = make_rsrc(reinterpret_cast<const float*>(abase), static_cast<uint32_t>((int64_t)nt * A_B));
  uint32_t aoff[A_DMA];
#pragma unroll
  for (int i = 0; i < A_DMA; ++i) {
    const int f = ((wave * A_DMA + i) * 64 + lane) * 16;
    aoff[i] = f < A_B ? static_cast<uint32_t>(f) : 0x80000000u;
  }
  // B rows n0 + 32 NJ w + 8 i + (lane >> 3), quad lane & 7 (stored swizzled)
  const View& vb = P.b;
  const int4v brsrc = make_rsrc(vb.p, static_cast<uint32_t>(((int64_t)(vb.rows - 1) * vb.ld + vb.kdim) * 4));
  uint32_t boff[B_DMA];
  int bkq[B_DMA];
#pragma unroll
  for (int i = 0; i < B_DMA; ++i) {
    const int r = 32 * NJ * wave + 8 * i + (lane >> 3);
    const int q = (lane & 7) ^ ((r >> 1) & 7);
    boff[i] = n0 + r < vb.rows ? static_cast<uint32_t>((int64_t)(n0 + r) * vb.ld * 4) : 0x80000000u;
    bkq[i] = 4 * q;
  }
  const int kend = P.K;

  floatx16 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  // A piece e of local K-tile t into A stage t & 1; B piece i into B stage t % NBS
  auto issue_a = [&](int t, int e) {
    dma_b128(arsrc, aoff[e] + static_cast<uint32_t>(t * A_B),
             lds0 + static_cast<uint32_t>((t & 1) * A_REGB + (wave * A_DMA + e) * 1024));
  };
  auto issue_b = [&](int t, int i) {
    const int k = (kt0 + t) * KT + bkq[i];
    const uint32_t off = (boff[i] + static_cast<uint32_t>(k) * 4u) | (k < kend ? 0u : 0x80000000u);
    dma_b128(brsrc, off,
             lds0 + static_cast<uint32_t>(2 * A_REGB + (t % NBS) * B_REGB + (32 * NJ * wave + 8 * i) * KT * 4));
  };
  auto a_st = [&](int t) { return smem + (t & 1) * A_REGB; };
  auto b_st = [&](int t) { return smem + 2 * A_REGB + (t % NBS) * B_REGB; };
  x6::bf16x8 fa[MI][3];  // single-buffered activation fragments (see k_conv_patch_x6)
  struct Fr {
    float b[NJ][8];
    x6::Parts bp[NJ];
  };
  auto read_a = [&](const char* st, int g, int i) {
    const char* p = st + (i * 32 + lr) * gx6::RLB + (g * 2 + lh) * 48;
#pragma unroll
    for (int t = 0; t < 3; ++t) fa[i][t] = *reinterpret_cast<const x6::bf16x8*>(p + 16 * t);
  };
  auto read_b = [&](Fr& F, const char* st, int g) {
    const float* bs = reinterpret_cast<const float*>(st);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = 32 * NJ * wave + 32 * j + lr;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float4 q = *reinterpret_cast<const float4*>(bs + n * KT + (((4 * lh + 2 * g + u) ^ ((n >> 1) & 7)) << 2));
        F.b[j][4 * u] = q.x;
        F.b[j][4 * u + 1] = q.y;
        F.b[j][4 * u + 2] = q.z;
        F.b[j][4 * u + 3] = q.w;
      }
    }
  };

  Fr F[2];
#pragma unroll
  for (int e = 0; e < A_DMA; ++e) issue_a(0, e);
#pragma unroll
  for (int i = 0; i < B_DMA; ++i) issue_b(0, i);
  if (nt > 1) {
#pragma unroll
    for (int i = 0; i < B_DMA; ++i) issue_b(1, i);
    wait_vm<B_DMA>();
  } else {
    wait_vm<0>();
  }
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int i = 0; i < MI; ++i) read_a(a_st(0), 0, i);
  read_b(F[0], b_st(0), 0);
#pragma unroll
  for (int j = 0; j < NJ; ++j) x6::split8_safe(F[0].b[j], F[0].bp[j]);

  auto tile = [&](int t, auto more_c) {
    constexpr bool MORE = decltype(more_c)::value;
    const bool more2 = t + 2 < nt;  // B of K-tile t + 2 to fetch
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      Fr& fc = F[g];
      Fr& fn = F[g ^ 1];
      const bool last = g == 1;
      if (last && MORE) {
        if (more2)
          wait_vm<B_DMA>();
        else
          wait_vm<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
      const bool rd = !last || MORE;
      const char* asrc = last ? a_st(t + 1) : a_st(t);
      const char* bsrc = last ? b_st(t + 1) : b_st(t);
      const int gn = last ? 0 : 1;
      constexpr int NB = MI * NJ;
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const int i = q / NJ, j = q % NJ;
        acc[i][j] = x6::mfma6(x6::Parts{fa[i][0], fa[i][1], fa[i][2]}, fc.bp[j], acc[i][j]);
        if (rd) {
          if (q == 0) read_b(fn, bsrc, gn);
          if (j == NJ - 1) read_a(asrc, gn, i);
#pragma unroll
          for (int jj = 0; jj < NJ; ++jj)
            if (q == NB - NJ + jj) x6::split8_safe(fn.b[jj], fn.bp[jj]);
        }
        if (!last && MORE) {  // A of t + 1, then B of t + 2, spread over the group's blocks
#pragma unroll
          for (int e = 0; e < NVM; ++e)
            if ((e * NB) / NVM == q) {
              // RRAM_FC_ABLATE (diagnostic builds only, wrong results): 1 drops
              // the A pieces, 2 the B pieces of the K-tile loop
              if (e < A_DMA) {
                if (RRAM_FC_ABLATE != 1) issue_a(t + 1, e);
              } else if (more2) {
                if (RRAM_FC_ABLATE != 2) issue_b(t + 2, e - A_DMA);
              }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  int t = 0;
  for (; t + 1 < nt; ++t) tile(t, std::true_type{});
  tile(t, std::false_type{});
  gemm_epilogue<MI, NJ, OUT_ROWMAJOR>(acc, P, P.e, part, m0, n0 + 32 * NJ * wave, lr, lh);
}

// A [M][lda] fp32 -> K-tile slabs of bf16 terms [tiles_m][ktiles][32 MI][RLB]
// for k_gemm_x6 (zero past M and K; lda, K multiples of 4, A 16-byte aligned).
// One thread per (row, K-tile, group, half): two float4 in, 48 bytes out.
__global__ void __launch_bounds__(256) k_pack_rows_x6(const float* __restrict__ a, int64_t lda, int M, int K,
                                                      char* __restrict__ out, int BMc, int ktiles, int units) {
  for (int u = blockIdx.x * blockDim.x + threadIdx.x; u < units; u += gridDim.x * blockDim.x) {
    const int h = u & 1, g = (u >> 1) & 1;
    const int r = u >> 2;
    const int kt = r % ktiles;
    const int mrow = r / ktiles;  // tm * BMc + row
    const int k = kt * gx6::KT + 16 * h + 8 * g;
    float v[8];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
      if (mrow < M && k + 4 * q < K) f = *reinterpret_cast<const float4*>(a + (int64_t)mrow * lda + k + 4 * q);
      v[4 * q] = f.x;
      v[4 * q + 1] = f.y;
      v[4 * q + 2] = f.z;
      v[4 * q + 3] = f.w;
    }
    const int tm = mrow / BMc, row = mrow - tm * BMc;
    char* rowp = out + (((int64_t)tm * ktiles + kt) * BMc + row) * gx6::RLB;
    x6::store_terms8(v, rowp + (g * 2 + h) * 48);
    if (g == 1 && h == 1) *reinterpret_cast<uint4*>(rowp + 192) = make_uint4(0, 0, 0, 0);
  }
}


// k_splitk_reduce for a row-major InnerProduct output that also writes it in
// the packed-row form the next k_gemm_x6 reads (rram_ip_fwd_rows: fc6 ->
// fc7): one thread per (row, 8 columns), each element k_splitk_reduce's
// (partials in split order, alpha, bias, ReLU; beta = 0), then those 8 values
// as k_pack_rows_x6 stores them (the consumer's K-tile record, its pad zeroed
// by the unit holding the tile's last 8 columns).  Host: N % 32 == 0, M a
// multiple of the consumer's tile rows, C rows 16-byte aligned.
__global__ void __launch_bounds__(256) k_splitk_reduce_rows_x6(const float* __restrict__ ws, int split, int M, int N,
                                                               Epi ep, char* __restrict__ pack, int BMc, int ktiles,
                                                               int units) {
  const int64_t total = (int64_t)M * N;
  const int n8 = N >> 3;
  for (int u = blockIdx.x * blockDim.x + threadIdx.x; u < units; u += gridDim.x * blockDim.x) {
    const int m = u / n8, n0 = 8 * (u - m * n8);
    // splitk_sum of 8 consecutive elements: the partials as 16-byte loads, 8
    // splits in flight, each element's adds in split order (same bits)
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.0f;
    const float* p0 = ws + (int64_t)m * N + n0;
    int z = 0;
    for (; z + 8 <= split; z += 8) {
      float4 q[8][2];
#pragma unroll
      for (int zz = 0; zz < 8; ++zz) {
        q[zz][0] = *reinterpret_cast<const float4*>(p0 + (int64_t)(z + zz) * total);
        q[zz][1] = *reinterpret_cast<const float4*>(p0 + (int64_t)(z + zz) * total + 4);
      }
#pragma unroll
      for (int zz = 0; zz < 8; ++zz) {
        v[0] += q[zz][0].x; v[1] += q[zz][0].y; v[2] += q[zz][0].z; v[3] += q[zz][0].w;
        v[4] += q[zz][1].x; v[5] += q[zz][1].y; v[6] += q[zz][1].z; v[7] += q[zz][1].w;
      }
    }
    for (; z < split; ++z) {
      const float4 a = *reinterpret_cast<const float4*>(p0 + (int64_t)z * total);
      const float4 b = *reinterpret_cast<const float4*>(p0 + (int64_t)z * total + 4);
      v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
      v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = n0 + j;
      float o = ep.alpha * v[j];
      if (ep.bias_mode == RRAM_BIAS_ROW) o += ep.bias[m];
      else if (ep.bias_mode == RRAM_BIAS_COL) o += ep.bias[n];
      if (ep.relu) o = fmaxf(o, 0.0f);
      v[j] = o;
    }
    float* dst = ep.C + (int64_t)m * ep.ldc + n0;
    *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(dst + 4) = make_float4(v[4], v[5], v[6], v[7]);
    const int kt = n0 >> 5, kk = n0 & 31, h = kk >> 4, g = (kk >> 3) & 1;
    const int tm = m / BMc, row = m - tm * BMc;
    char* rowp = pack + (((int64_t)tm * ktiles + kt) * BMc + row) * gx6::RLB;
    x6::store_terms8(v, rowp + (g * 2 + h) * 48);
    if (g == 1 && h == 1) *reinterpret_cast<uint4*>(rowp + 192) = make_uint4(0, 0, 0, 0);
  }
}

}  // namespace

float* pack_buffer(size_t floats, hipStream_t s);  // gemm.hip

// most patch rows (output rows + KH - 1 halo per image segment) any BN-position
// tile of an OH x OW output needs; -1 when a tile spans more than maxseg images
int patch_rows(int N, int HW, int OW, int OH, int KH, int BN, int maxseg) {
  int rmax = 0;
  for (int n0 = 0; n0 < N; n0 += BN) {
    const int pl = std::min(n0 + BN, N) - 1;
    const int i0 = n0 / HW, i1 = pl / HW;
    if (i1 - i0 + 1 > maxseg) return -1;
    int r = 0;
    for (int i = i0; i <= i1; ++i) {
      const int f = i == i0 ? (n0 - i0 * HW) / OW : 0;
      const int l = i == i1 ? (pl - i1 * HW) / OW : OH - 1;
      r += l - f + KH;
    }
    rmax = std::max(rmax, r);
  }
  return rmax;
}

template <int KH, int CPH, int MI, int PD>
int launch_patch_x6(Params P, const uint16_t* wpack, int PW, int CS, int gz, hipStream_t s) {
  P.tiles_m = (P.M + 32 * MI - 1) / (32 * MI);
  P.tiles_n = (P.N + x6::BN - 1) / x6::BN;
  P.tiles_z = gz;
  const int64_t nwg = (int64_t)P.tiles_m * P.tiles_n * gz;
  RRAM_REQUIRE(nwg < (1ll << 31), "conv: grid too large");
  hipLaunchKernelGGL((k_conv_patch_x6<KH, KH, CPH, MI, PD>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, P, wpack,
                     PW, CS);
  return launch_status("conv patch x6");
}


// ---- k_conv1_ring_x6 (AlexNet conv1: 3 x 227 x 227, 96 x 11 x 11, stride 4) ----
bool conv1_ring_ok(const rram_conv_desc* d) {
  return d->group == 1 && d->channels == 3 && d->kernel_h == 11 && d->kernel_w == 11 && d->stride_h == 4 &&
         d->stride_w == 4 && d->pad_h == 0 && d->pad_w == 0 && d->dilation_h == 1 && d->dilation_w == 1 &&
         d->width == 227 && d->height >= 11 && d->num_output == c1x6::BM && d->num > 0 &&
         (int64_t)d->num * 3 * d->height * d->width * 4 < (1ll << 31) &&
         (int64_t)d->num * d->num_output * d->out_h * d->out_w * 4 < (1ll << 31);
}

int conv_wide_x6_fwd(const rram_conv_desc* d, const float* x, const float* w, const float* bias, float* y, int relu,
                     hipStream_t s, const WPack& wk) {
  if (!conv1_ring_ok(d)) return 0;
  if ((reinterpret_cast<uintptr_t>(w) & 3u) != 0) return 0;
  const int HW = d->out_h * d->out_w;
  Params P{};
  P.M = d->num_output;
  P.N = d->num * HW;
  P.K = 3 * 121;
  P.split = 1;
  P.b = make_view(x, 0, P.N, P.K);
  ConvGeom& cv = P.cv;
  cv.C = 3;
  cv.H = d->height;
  cv.W = d->width;
  cv.KH = cv.KW = 11;
  cv.sh = cv.sw = 4;
  cv.dh = cv.dw = 1;
  cv.Ho = d->out_h;
  cv.Wo = d->out_w;
  cv.howo = make_fastdiv(HW);
  cv.wo_div = make_fastdiv(d->out_w);
  cv.chw = (int64_t)3 * d->height * d->width;
  cv.in_bytes = static_cast<int>((int64_t)d->num * cv.chw * 4);
  P.e = make_epi(y, HW, 1.0f, 0.0f, bias, RRAM_BIAS_ROW, relu);
  P.e.cimg = wk.y_img > 0 ? wk.y_img : (int64_t)d->num_output * HW;
  P.e.hw = make_fastdiv(HW);
  // the epilogue's 32-bit output offsets (image stride included)
  if ((int64_t)d->num * P.e.cimg * 4 >= (1ll << 31)) return 0;
  const int units = c1x6::G * 3 * 64;  // 3 KB fragments
  const size_t wbytes = static_cast<size_t>(units) * 48;
  if (wk.query) {
    *wk.query = wbytes;
    return 1;
  }
  char* wp = static_cast<char*>(wk.p ? wk.p : pack_buffer((wbytes + 3) / 4, s));
  RRAM_REQUIRE(wp != nullptr, "conv: packed-weight buffer allocation failed");
  if (!wk.valid) {
    hipLaunchKernelGGL(k_conv1_pack_x6, dim3(stream_blocks(units)), dim3(256), 0, s, w, wp, d->num_output, units);
    const int rc = launch_status("conv1 weight pack x6");
    if (rc) return rc;
  }
  // (a non-persistent form at two workgroups of six waves per CU, 96 x 128
  // tiles, two channel slots: 0.462 vs 0.326 ms, profiles/r05_ab_c1_pair.txt)
  const int tpi = (HW + c1x6::BN - 1) / c1x6::BN;
  const int tiles = d->num * tpi;
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const unsigned nwg = static_cast<unsigned>(std::min(tiles, cus));
  hipLaunchKernelGGL((k_conv1_ring_x6<227>), dim3(nwg), dim3(256), 0, s, P, reinterpret_cast<const uint16_t*>(wp),
                     tpi, tiles);
  const int rc = launch_status("conv1 ring x6");
  return rc ? rc : 1;
}

// ---- k_conv_s2_x6 (GoogLeNet conv1: 3 channels, 64 x 7 x 7, stride 2) ----
#ifndef RRAM_S2_NBW  // 32-column blocks per wave of k_conv_s2_x6 (2: 64 x 256 tiles, two per CU; 1: 64 x 128, three)
#define RRAM_S2_NBW 2
#endif
bool conv_s2_ok(const rram_conv_desc* d) {
  namespace k = c7x6;
  using T = k::Tile<RRAM_S2_NBW>;
  return d->group == 1 && d->channels == k::C && d->kernel_h == k::KS && d->kernel_w == k::KS &&
         d->stride_h == k::S && d->stride_w == k::S && d->dilation_h == 1 && d->dilation_w == 1 && d->pad_h >= 0 &&
         d->pad_h <= 3 && d->pad_w >= 0 && d->pad_w <= 3 && d->num_output >= 1 && d->num_output <= k::BM &&
         d->num > 0 && d->out_w >= 85 && d->out_h >= 1 && k::S * (d->out_w - 1) + k::KC <= k::ROWE &&
         (d->out_w + T::BN - 2) / d->out_w <= T::OR - 1 &&
         (int64_t)d->num * k::C * d->height * d->width * 4 < (1ll << 31) &&
         (int64_t)d->num * d->num_output * d->out_h * d->out_w * 4 < (1ll << 31);
}

int conv_s2_x6_fwd(const rram_conv_desc* d, const float* x, const float* w, const float* bias, float* y, int relu,
                   hipStream_t s, const WPack& wk) {
  if (!conv_s2_ok(d)) return 0;
  if ((reinterpret_cast<uintptr_t>(w) & 3u) != 0) return 0;
  const int HW = d->out_h * d->out_w;
  Params P{};
  P.M = d->num_output;
  P.N = d->num * HW;
  P.K = c7x6::R * c7x6::KS;
  P.split = 1;
  P.b = make_view(x, 0, P.N, P.K);
  ConvGeom& cv = P.cv;
  cv.C = c7x6::C;
  cv.H = d->height;
  cv.W = d->width;
  cv.KH = cv.KW = c7x6::KS;
  cv.ph = d->pad_h;
  cv.pw = d->pad_w;
  cv.sh = cv.sw = c7x6::S;
  cv.dh = cv.dw = 1;
  cv.Ho = d->out_h;
  cv.Wo = d->out_w;
  cv.howo = make_fastdiv(HW);
  cv.wo_div = make_fastdiv(d->out_w);
  cv.chw = (int64_t)c7x6::C * d->height * d->width;
  cv.in_bytes = static_cast<int>((int64_t)d->num * cv.chw * 4);
  P.e = make_epi(y, HW, 1.0f, 0.0f, bias, RRAM_BIAS_ROW, relu);
  P.e.cimg = wk.y_img > 0 ? wk.y_img : (int64_t)d->num_output * HW;
  P.e.hw = make_fastdiv(HW);
  // the epilogue's 32-bit output offsets (image stride included)
  if ((int64_t)d->num * P.e.cimg * 4 >= (1ll << 31)) return 0;
  const int units = c7x6::G * c7x6::MI * 64;  // 3 KB fragments
  const size_t wbytes = static_cast<size_t>(units) * 48;
  if (wk.query) {
    *wk.query = wbytes;
    return 1;
  }
  char* wp = static_cast<char*>(wk.p ? wk.p : pack_buffer((wbytes + 3) / 4, s));
  RRAM_REQUIRE(wp != nullptr, "conv: packed-weight buffer allocation failed");
  if (!wk.valid) {
    hipLaunchKernelGGL(k_conv_s2_pack_x6, dim3(stream_blocks(units)), dim3(256), 0, s, w, wp, d->num_output, units);
    const int rc = launch_status("conv s2 weight pack x6");
    if (rc) return rc;
  }
  const int tpi = (HW + c7x6::Tile<RRAM_S2_NBW>::BN - 1) / c7x6::Tile<RRAM_S2_NBW>::BN;
  const int64_t tiles = (int64_t)d->num * tpi;
  RRAM_REQUIRE(tiles < (1ll << 31), "conv: grid too large");
  // (a persistent form, one workgroup per CU with the weights in registers:
  // 0.61 vs 0.43 ms in the GoogLeNet map, profiles/r06_ab_conv_s2_persistent.txt)
  hipLaunchKernelGGL(k_conv_s2_x6<RRAM_S2_NBW>, dim3(static_cast<unsigned>(tiles)), dim3(256), 0, s, P,
                     reinterpret_cast<const x6::bf16x8*>(wp), tpi, static_cast<int>(tiles));
  const int rc = launch_status("conv s2 x6");
  return rc ? rc : 1;
}

// engine of the stride-1 3x3 / 5x5 convolutions (rram_set_f32_engine)
std::atomic<int>& f32_engine() {
  static std::atomic<int> eng{[] {
    const char* e = getenv("RRAM_X6");
    return (e && atoi(e) == 0) ? static_cast<int>(RRAM_ENGINE_F32) : static_cast<int>(RRAM_ENGINE_BF16X6);
  }()};
  return eng;
}

// k_conv_patch_x6 (fp32 products on the bf16 matrix cores, see the kernel):
// stride-1 undilated 3x3 / 5x5 convolutions with >= 128 positions per output
// plane and <= 1/8 padded rows in the 96- or 128-row M tiles.  Returns 1 when it ran,
// 0 when not covered, < 0 on error.  RRAM_X6 = 0 keeps the fp32-MFMA kernels.
// shape plan of the x6 convolution (false: not covered)
struct ConvPlan {
  int CPH, MI, mt, PW, CS, PD;
};
bool conv_x6_plan(const rram_conv_desc* d, ConvPlan& pl) {
  const int KH = d->kernel_h, KW = d->kernel_w;
  if (d->stride_h != 1 || d->stride_w != 1 || d->dilation_h != 1 || d->dilation_w != 1) return false;
  if (!((KH == 3 && KW == 3) || (KH == 5 && KW == 5))) return false;
  const int G = d->group, Cg = d->channels / G, M = d->num_output / G;
  const int HW = d->out_h * d->out_w, OW = d->out_w, OH = d->out_h;
  pl.CPH = KH == 5 ? 1 : (Cg % 8 == 0 ? 4 : 2);
  if (HW < 128 || Cg == 0 || Cg % (2 * pl.CPH) != 0) return false;
  if ((int64_t)d->num * d->channels * d->height * d->width * 4 >= (1ll << 31)) return false;  // 32-bit offsets
  if ((int64_t)d->num * d->num_output * HW * 4 >= (1ll << 31)) return false;                   // (output too)
  // M tile 128 or 96 rows, whichever pads less (<= 1/8 padded rows)
  const int t128 = (M + 127) / 128 * 128, t96 = (M + 95) / 96 * 96;
  pl.MI = (t96 - M) < (t128 - M) ? 3 : 4;
  pl.mt = pl.MI == 3 ? t96 : t128;
  if ((pl.mt - M) * 8 > pl.mt) return false;
  const int rmax = patch_rows(d->num * HW, HW, OW, OH, KH, x6::BN, 3);
  if (rmax < 0) return false;
  pl.PW = d->width + 2 * d->pad_w;
  // channel stride >= rmax * PW with CPH * CS = 32 (mod 64): the two lane
  // halves read disjoint bank halves
  pl.CS = rmax * pl.PW;
  while ((pl.CPH * pl.CS) % 64 != 32) ++pl.CS;
  const int need = (2 * pl.CPH * pl.CS + 255) / 256;  // 256-float patch pieces
  static const int pd5[] = {4, 8, 12}, pd3q[] = {8, 12, 16}, pd3h[] = {4, 8, 16};
  const int* pds = KH == 5 ? pd5 : pl.CPH == 4 ? pd3q : pd3h;
  pl.PD = 0;
  for (int i = 2; i >= 0; --i)
    if (pds[i] >= need) pl.PD = pds[i];
  if (pl.PD == 0) return false;
  const int64_t total = (int64_t)G * (pl.mt / (32 * pl.MI)) * (Cg / (2 * pl.CPH)) * 32 * pl.MI *
                        (((KH * KW * pl.CPH + 7) / 8 * 96 + 16) / 2);
  return total * 2 < (1ll << 31);
}

// x [num][C][HWi] fp32 -> its octet companion (C % 8 == 0)
int pack_octets(const float* x, void* oct, int num, int C, int HWi, hipStream_t s) {
  RRAM_REQUIRE(C % 8 == 0 && (int64_t)num * C * HWi * 6 < (1ll << 31), "pack_octets: C %% 8 != 0 or too large");
  const int units = num * (C / 8) * HWi;
  if (units == 0) return RRAM_OK;
  hipLaunchKernelGGL(k_pack_octets_x6, dim3(stream_blocks(units)), dim3(256), 0, s, x, static_cast<char*>(oct), C / 8,
                     HWi, units);
  return launch_status("octet pack x6");
}

// ---- k_conv_cb_x6 (channel-octet pre-split activations) ----
struct CbPlan {
  int WR, NB, RPC, PD, octb, tiles_m, tiles_n, OCC, tpi;
  int tp = 0;  // per-image tiles of tp positions (whole output rows; 0: the tile width)
};
// instantiated (KH, WR, NB, PD, OCC) combinations; OCC = workgroups per CU.
// One workgroup per CU: k_conv_cb_x6 (32x32x16); two: k_conv_cb16_x6
// (16x16x32, RRAM_CB16_LIST below)
#define RRAM_CB_LIST(X)                                                                              \
  X(5, 4, 8, 15, 1) X(5, 4, 4, 12, 1) X(5, 4, 4, 14, 1) X(5, 2, 4, 14, 1) X(3, 4, 8, 12, 1)          \
  X(3, 4, 8, 15, 1) X(3, 4, 4, 8, 1) X(3, 4, 4, 12, 1) X(3, 2, 4, 12, 1) X(3, 2, 4, 14, 1)
// (a 64 x 256 form for conv4 does not fit two per CU: its contiguous patch
// spans up to 27 rows = 9 LDS pieces, the per-image one wastes a third)
// (128 x 64 tiles for conv5, whose 676 128 x 128 workgroups leave the second
// of two rounds a third full, measured slower: 0.180-0.183 vs 0.166-0.168 ms,
// profiles/r05_ab_conv5_n64.txt)
#define RRAM_CB16_LIST(X) X(5, 4, 4, 8, 2) X(3, 4, 4, 8, 2) X(3, 2, 2, 8, 2)
bool cb_instantiated(int KH, int WR, int NB, int PD, int OCC = 1) {
#define RRAM_X(kh, wr, nb, pd, occ) \
  if (KH == kh && WR == wr && NB == nb && PD == pd && OCC == occ) return true;
  RRAM_CB_LIST(RRAM_X)
  RRAM_CB16_LIST(RRAM_X)
#undef RRAM_X
  return false;
}
#ifndef RRAM_CB_ROWALIGN  // 0: no row-aligned per-image tiles; 1: by the cost rule; 2: wherever they fit (A/B)
#define RRAM_CB_ROWALIGN 1
#endif
#ifndef RRAM_CB_IMGALIGN  // 0: no octet plan for planes of < 64 positions
#define RRAM_CB_IMGALIGN 1
#endif
// Planes of < 64 positions (GoogLeNet's 7 x 7 stage): 128 consecutive
// positions would span 4 images (the patch holds 3 segments), so the tiles are
// whole images -- tp = floor(128 / HW) images' positions per 128-column tile
// at two workgroups per CU, the columns past tp computed and dropped -- when
// the patch of those images fits the 8 LDS pieces.
bool conv_cb_plan_whole_images(const rram_conv_desc* d, CbPlan& pl) {
  const int KH = d->kernel_h, G = d->group, M = d->num_output / G;
  const int HW = d->out_h * d->out_w, OW = d->out_w, OH = d->out_h, N = d->num * HW;
  if ((int64_t)d->num * d->channels * d->height * d->width * 6 >= (1ll << 31)) return false;  // 32-bit offsets
  if ((int64_t)d->num * d->num_output * HW * 4 >= (1ll << 31)) return false;
  const int PW = d->width + 2 * d->pad_w;
  int RPC = 3 * PW;
  while ((RPC - 3 * OW) % 16 != 0) ++RPC;
  // 128 x 128 tiles where no row pads, else 64 x 128 (the instantiated ones)
  static const int cfg[2][2] = {{4, 4}, {2, 2}};
  for (const auto& c : cfg) {
    const int WR = c[0], NB = c[1], BM = 32 * WR, BN = 32 * NB * (4 / WR);
    if (HW > BN / 2 || !cb_instantiated(KH, WR, NB, 8, 2)) continue;
    const int tiles_m = (M + BM - 1) / BM;
    if (WR == 4 && tiles_m * BM != M && cb_instantiated(KH, 2, 2, 8, 2)) continue;
    if ((tiles_m * BM - M) * 4 > tiles_m * BM) continue;
    const int per = std::min(BN / HW, 3), tp = per * HW;  // (the patch holds 3 segments)
    const int rmax = per * (OH + KH - 1);
    const int octb = ((rmax * RPC + 2 * ((3 * OW * (1 - KH)) & 15)) * 16 + 255) / 256 * 256;
    if ((2 * octb / 16 + 255) / 256 > 8) continue;
    const int64_t tiles_n = (N + tp - 1) / tp;
    if ((int64_t)G * tiles_m * tiles_n >= (1ll << 31)) continue;
    pl = CbPlan{WR, NB, RPC, 8, octb, tiles_m, static_cast<int>(tiles_n), 2, 0};
    pl.tp = tp;
    return true;
  }
  return false;
}
bool conv_cb_plan(const rram_conv_desc* d, CbPlan& pl) {
  const int KH = d->kernel_h, KW = d->kernel_w;
  if (d->stride_h != 1 || d->stride_w != 1 || d->dilation_h != 1 || d->dilation_w != 1) return false;
  if (!((KH == 3 && KW == 3) || (KH == 5 && KW == 5))) return false;
  const int G = d->group, Cg = d->channels / G, M = d->num_output / G;
  const int HW = d->out_h * d->out_w, OW = d->out_w, OH = d->out_h, N = d->num * HW;
  if (Cg % 16 != 0 || M == 0) return false;
  if (HW < 64) return RRAM_CB_IMGALIGN && conv_cb_plan_whole_images(d, pl);
  const int PW = d->width + 2 * d->pad_w;
  // row pitch in 16-byte chunks: >= 3 PW, = 3 OW (mod 16) (bank-conflict-free reads)
  int RPC = 3 * PW;
  while ((RPC - 3 * OW) % 16 != 0) ++RPC;
  // packed input < 2 GB (32-bit buffer offsets), and the fp32 output (the
  // epilogues' 32-bit byte offsets)
  if ((int64_t)d->num * d->channels * d->height * d->width * 6 >= (1ll << 31)) return false;
  if ((int64_t)d->num * d->num_output * HW * 4 >= (1ll << 31)) return false;
  // tile (WR, NB) with the least makespan (rounds of 256 workgroups x tile
  // area); ties: taller tiles (weights fetched by one wave)
  static const int cfg[3][2] = {{4, 8}, {4, 4}, {2, 4}};
  // (the other tiles per layer measured slower: profiles/r02_ab_cb_cfg.txt)
  int64_t best = -1;
  for (const auto& c : cfg) {
    const int WR = c[0], NB = c[1], BM = 32 * WR, BN = 32 * NB * (4 / WR);
    const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
    if ((tiles_m * BM - M) * 4 > tiles_m * BM) continue;  // > 1/4 padded rows
    const int rmax = patch_rows(N, HW, OW, OH, KH, BN, 3);
    if (rmax < 0) continue;
    // octet plane size rounded to 256 bytes: the 16x16x32 form reads both
    // planes in one ds_read_b128 lane group, conflict-free only when the
    // plane offset is a multiple of the 64 banks
    // (+ the two segment shifts of cbx6::seg_shift)
    const int octb = ((rmax * RPC + 2 * ((3 * OW * (1 - KH)) & 15)) * 16 + 255) / 256 * 256;
    const int need = (2 * octb / 16 + 255) / 256;  // 1 KB pieces per wave
    int PD = 0;
    for (int p : {8, 12, 14, 15})
      if (PD == 0 && p >= need && cb_instantiated(KH, WR, NB, p)) PD = p;
    if (PD == 0) {
      // the contiguous tiles' patch does not fit (tiles spanning two images
      // carry two halos): per-image tiles of this shape, one halo each, the
      // last tile of an image short (GoogLeNet conv2, 64 x 256 on 56 x 56:
      // 13 tiles per image instead of 128 x 128 tiles with 1/4 padded rows)
      const int tpi = (HW + BN - 1) / BN;
      int rm = 0;
      for (int t = 0; t < tpi; ++t) {
        const int f = t * BN / OW, l = (std::min((t + 1) * BN, HW) - 1) / OW;
        rm = std::max(rm, l - f + KH);
      }
      const int ob = (rm * RPC * 16 + 255) / 256 * 256;
      const int nd = (2 * ob / 16 + 255) / 256;
      for (int p : {8, 12, 14, 15})
        if (PD == 0 && p >= nd && cb_instantiated(KH, WR, NB, p)) PD = p;
      const int64_t nwg = (int64_t)G * tiles_m * tpi * d->num;
      if (PD == 0 || nwg >= (1ll << 31)) continue;
      const int64_t cost = (nwg + 255) / 256 * BM * BN;
      if (best < 0 || cost < best) {
        best = cost;
        pl = CbPlan{WR, NB, RPC, PD, ob, tiles_m, static_cast<int>(tpi * d->num), 1, tpi};
      }
      continue;
    }
    const int64_t nwg = (int64_t)G * tiles_m * tiles_n;
    if (nwg >= (1ll << 31)) continue;
    const int64_t cost = (nwg + 255) / 256 * BM * BN;
    if (best < 0 || cost < best) {
      best = cost;
      pl = CbPlan{WR, NB, RPC, PD, octb, tiles_m, tiles_n, 1, 0};
    }
  }
  // Two workgroups per CU (k_conv_cb16_x6: <= 256 registers and 8 LDS
  // pieces = 64 KB each): one workgroup's waits, prologue and epilogue then
  // run under the other's MFMAs.  Tiles 128 x 128 or 64 x 128, contiguous
  // positions or per-image (one halo: AlexNet conv2's 5 x 5); the least
  // makespan in rounds of 512 half-CU tiles wins (ties: taller, contiguous)
  // and replaces the one-per-CU plan (see the rule below).
  // Measured on MI355X (AlexNet b256): conv3 128 x 256 -> 128 x 128 here
  // 0.342 -> 0.308 ms (profiles/r05_ab_occ2.txt); round 4: conv5 215 -> 204.
  if (best > 0) {
    int64_t best2 = -1, best3 = -1;  // best3: the row-aligned per-image plans
    CbPlan p2{}, p3{};
    static const int cfg2[2][2] = {{4, 4}, {2, 2}};
    for (const auto& c : cfg2) {
      const int WR = c[0], NB = c[1], BM = 32 * WR, BN = 32 * NB * (4 / WR);
      if (!cb_instantiated(KH, WR, NB, 8, 2)) continue;
      const int tiles_m = (M + BM - 1) / BM;
      if ((tiles_m * BM - M) * 4 > tiles_m * BM) continue;
      // per_image 2: per-image tiles of whole output rows (tp = the rows of
      // OW that fit BN; the columns past tp computed and dropped), whose
      // patch has no partial rows: GoogLeNet conv2 (56 x 56) fits 8 pieces
      // at 112-position tiles where 128-position ones need 9
      for (int per_image = 0; per_image < 3; ++per_image) {
        int rmax = 0, tpi = 0, octb = 0, tp = 0;
        if (per_image == 0) {
          rmax = patch_rows(N, HW, OW, OH, KH, BN, 3);
          if (rmax < 0) continue;
          octb = ((rmax * RPC + 2 * ((3 * OW * (1 - KH)) & 15)) * 16 + 255) / 256 * 256;
        } else if (per_image == 1) {
          tpi = (HW + BN - 1) / BN;
          for (int t = 0; t < tpi; ++t) {
            const int f = t * BN / OW, l = (std::min((t + 1) * BN, HW) - 1) / OW;
            rmax = std::max(rmax, l - f + KH);
          }
          octb = (rmax * RPC * 16 + 255) / 256 * 256;
        } else {
          if (!RRAM_CB_ROWALIGN || OW > BN || BN % OW == 0 || HW <= BN) continue;
          // 64 x 128 tiles only: GoogLeNet conv2 0.875-0.886 ms there vs
          // 0.943-0.963 on 128 x 128 (a quarter of the rows padded; equal
          // estimates), profiles/r06_ab_cb_rowalign.txt
#ifndef RRAM_CB_RA_WR
#define RRAM_CB_RA_WR 2
#endif
          if (WR != RRAM_CB_RA_WR) continue;
          tp = BN / OW * OW;
          tpi = (HW + tp - 1) / tp;
          rmax = tp / OW + KH - 1;
          octb = (rmax * RPC * 16 + 255) / 256 * 256;
        }
        if ((2 * octb / 16 + 255) / 256 > 8) continue;
        const int tiles_n = per_image ? tpi * d->num : (N + BN - 1) / BN;
        const int64_t nwg = (int64_t)G * tiles_m * tiles_n;
        if (nwg >= (1ll << 31)) continue;
        // a 64-row tile pays about a third more per MFMA (two waves read each
        // weight fragment for half the columns): AlexNet conv5 (128 rows per
        // group) 0.172 ms on 128 x 128 vs 0.184 on 64 x 128, while conv4
        // (192 rows per group: 128-row tiles pad a quarter) 0.297 on its
        // one-per-CU 64 x 256 plan vs 0.267 on 64 x 128
        const int64_t cost = (nwg + 511) / 512 * 2 * BM * BN * (BM == 64 ? 4 : 3) / 3;
        int64_t& bc = per_image == 2 ? best3 : best2;
        CbPlan& pc = per_image == 2 ? p3 : p2;
        if (bc < 0 || cost < bc) {
          bc = cost;
          pc = CbPlan{WR, NB, RPC, 8, octb, tiles_m, tiles_n, 2, tpi};
          pc.tp = tp;
        }
      }
    }
    // Rounds x area prices a round of two workgroups like one of twice the
    // area, but measured the pair hides its waits: every AlexNet layer runs
    // faster there although its estimate is up to a third longer (conv3
    // 0.342 -> 0.308 ms at an equal estimate; conv4 0.297 -> 0.267 and conv5
    // (round 4) 0.215 -> 0.204 at 4/3 of it).  Taken within 1.4x; round 4's
    // loser, conv4 on 128 x 128 (a quarter of the rows padded, 0.279 ->
    // 0.335 ms), estimates 1.5x.
    if (best2 > 0 && best2 * 5 <= best * 7) pl = p2;
    // row-aligned per-image tiles where no other two-per-CU plan fits, within
    // 1.5x: GoogLeNet conv2 (56 x 56, one-per-CU 64 x 256 before) 0.935-0.963
    // -> 0.856-0.886 ms at an estimate of 1.44x; where another two-per-CU plan
    // fits they measured slower (profiles/r06_ab_cb_rowalign.txt).
    // RRAM_CB_ROWALIGN == 2 (A/B builds): the row-aligned plan wherever it fits
    else if (best3 > 0 && ((best2 < 0 && best3 * 2 <= best * 3) || RRAM_CB_ROWALIGN == 2)) pl = p3;
    if (RRAM_CB_ROWALIGN == 2 && best3 > 0) pl = p3;
  }
  return best > 0;
}

// The plans at two workgroups per CU run on 16x16x32 (k_conv_cb16_x6), the
// others on 32x32x16.  Measured on MI355X (AlexNet b256,
// profiles/r04_ab_cb16.txt): the 16x16x32 loop holds a 6-13 % higher clock;
// conv2 (5x5, two workgroups per CU) 0.482 -> 0.457-0.461 ms, conv5 (3x3, two
// per CU) 0.170 -> 0.166; at one workgroup per CU the 16x16x32 form lost
// MFMA-busy (conv3 0.64 -> 0.59) faster than it gained clock.
int conv_cb_x6_fwd(const rram_conv_desc* d, const float* x, const void* x_oct, const float* w, const float* bias,
                   float* y, void* y_oct, int relu, hipStream_t s, const WPack& wk) {
  CbPlan pl;
  if (!conv_cb_plan(d, pl)) return 0;
  const bool use16 = pl.OCC == 2;
  if (y_oct != nullptr && d->num_output % 8 != 0) return 0;
  const int KH = d->kernel_h, KW = d->kernel_w, T = KH * KW;
  const int G = d->group, Cg = d->channels / G, M = d->num_output / G;
  // the epilogue writes whole octets of one group's rows: a group whose row
  // count is not a multiple of 8 would share octets with its neighbour, so its
  // companion is packed from y after the kernel instead
  void* const y_oct_k = (y_oct != nullptr && M % 8 == 0) ? y_oct : nullptr;
  // y == nullptr (the convolution-output fold) needs the companion from the
  // 16x16x32 epilogue itself
  if (y == nullptr && !wk.query && (!use16 || y_oct_k == nullptr)) return 0;
  const int HW = d->out_h * d->out_w, HWi = d->height * d->width;
  Params P{};
  P.M = M;
  P.N = d->num * HW;
  P.K = Cg * T;
  P.split = 1;
  ConvGeom& cv = P.cv;
  cv.C = Cg;
  cv.H = d->height;
  cv.W = d->width;
  cv.KH = KH;
  cv.KW = KW;
  cv.ph = d->pad_h;
  cv.pw = d->pad_w;
  cv.sh = cv.sw = cv.dh = cv.dw = 1;
  cv.Ho = d->out_h;
  cv.Wo = d->out_w;
  cv.tpitch = pl.tp;
  cv.howo = make_fastdiv(HW);
  cv.wo_div = make_fastdiv(d->out_w);
  P.e = make_epi(y, HW, 1.0f, 0.0f, bias, RRAM_BIAS_ROW, relu);
  P.e.cimg = wk.y_img > 0 ? wk.y_img : (int64_t)d->num_output * HW;
  P.e.hw = make_fastdiv(HW);
  P.grp_c = (int64_t)M * HW;
  P.grp_bias = M;
  P.tiles_m = pl.tiles_m;
  P.tiles_n = pl.tiles_n;
  P.tiles_z = G;
  // one scratch buffer: packed input (unless the caller hands over the
  // input's octet companion), then the weight fragments
  const int64_t xbytes = (int64_t)d->num * d->channels * HWi * 6;
  const int rblocks = pl.tiles_m * pl.WR;
  const int64_t wfrags =
      use16 ? (int64_t)G * rblocks * (((Cg / 16) * T + 1) / 2) * 2 : (int64_t)G * rblocks * (Cg / 16) * T;
  if (wk.query) {
    *wk.query = static_cast<size_t>(wfrags * 3072);
    return 1;
  }
  const int64_t xb_al = x_oct != nullptr ? 0 : (xbytes + 255) / 256 * 256;
  const int64_t scratch = xb_al + (wk.p ? 0 : wfrags * 3072);
  char* buf = scratch > 0 ? reinterpret_cast<char*>(pack_buffer(static_cast<size_t>(scratch / 4), s)) : nullptr;
  RRAM_REQUIRE(scratch == 0 || buf != nullptr, "conv: packed-operand buffer allocation failed");
  char* wbuf = wk.p ? static_cast<char*>(wk.p) : buf + xb_al;
  int rc = 0;
  if (x_oct == nullptr) {
    rc = pack_octets(x, buf, d->num, d->channels, HWi, s);
    if (rc) return rc;
  }
  if (!wk.valid) {
    const int wunits = static_cast<int>(wfrags * 64);
    if (use16)
      hipLaunchKernelGGL(k_conv_cb16_pack_x6, dim3(stream_blocks(wunits)), dim3(256), 0, s, w, wbuf, M, Cg, T,
                         rblocks, wunits);
    else
      hipLaunchKernelGGL(k_conv_cb_pack_x6, dim3(stream_blocks(wunits)), dim3(256), 0, s, w, wbuf, M, Cg, T,
                         rblocks, wunits);
    rc = launch_status("conv weight pack x6 (octets)");
    if (rc) return rc;
  }
  const auto* wp = reinterpret_cast<const x6::bf16x8*>(wbuf);
  const auto* xp = reinterpret_cast<const uint16_t*>(x_oct != nullptr ? x_oct : buf);
  const int ximg = d->channels / 8 * HWi * 48;
  const unsigned nwg = static_cast<unsigned>((int64_t)G * pl.tiles_m * pl.tiles_n);
  const uint32_t xrange = static_cast<uint32_t>(xbytes);  // whole packed input (the kernel narrows it per group)
  if (use16) {
    const int kto = (Cg / 16) & 1;
    // persistent: at most two workgroups per CU (k_conv_cb16_x6 walks its
    // XCD's tiles); a multiple of 8 whenever it is not one per tile
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
#ifndef RRAM_CB16_PERSIST_X2  // persistent while tiles <= slots * X2 / 2 (A/B builds)
#define RRAM_CB16_PERSIST_X2 3
#endif
    const int64_t slots = (2 * cus) / 8 * 8;
    const unsigned nwg16 =
        static_cast<unsigned>(nwg * 2 <= slots * RRAM_CB16_PERSIST_X2 ? std::min<int64_t>(nwg, slots) : nwg);
#define RRAM_X2(kh, wr, nb, pd, occ, kpar)                                                                          \
  if (KH == kh && pl.WR == wr && pl.NB == nb && pl.PD == pd && pl.OCC == occ && kto == kpar) {                      \
    hipLaunchKernelGGL((k_conv_cb16_x6<kh, kh, wr, nb, pd, occ, kpar>), dim3(nwg16), dim3(256), 0, s, P, wp, xp,      \
                       pl.octb, pl.RPC, xrange, ximg, static_cast<char*>(y_oct_k), d->num_output / 8,               \
                       make_fastdiv(static_cast<uint32_t>(pl.octb >> 4)), make_fastdiv(static_cast<uint32_t>(pl.RPC)), \
                       pl.tpi);                                                                                     \
  } else
#define RRAM_X(kh, wr, nb, pd, occ) RRAM_X2(kh, wr, nb, pd, occ, 0) RRAM_X2(kh, wr, nb, pd, occ, 1)
    RRAM_CB16_LIST(RRAM_X) { return 0; }
#undef RRAM_X
#undef RRAM_X2
    rc = launch_status("conv cb16 x6");
    if (rc == 0 && y_oct != nullptr && y_oct_k == nullptr) rc = pack_octets(y, y_oct, d->num, d->num_output, HW, s);
    return rc ? rc : 1;
  }
#define RRAM_X(kh, wr, nb, pd, occ)                                                                           \
  if (KH == kh && pl.WR == wr && pl.NB == nb && pl.PD == pd && pl.OCC == occ) {                               \
    hipLaunchKernelGGL((k_conv_cb_x6<kh, kh, wr, nb, pd, occ>), dim3(nwg), dim3(256), 0, s, P, wp, xp, pl.octb,   \
                       pl.RPC,                                                                                 \
                       xrange, ximg, static_cast<char*>(y_oct_k), d->num_output / 8,                          \
                       make_fastdiv(static_cast<uint32_t>(pl.octb >> 4)), make_fastdiv(static_cast<uint32_t>(pl.RPC)), \
                       pl.tpi);                                                                                \
  } else
  RRAM_CB_LIST(RRAM_X) { return 0; }
#undef RRAM_X
  rc = launch_status("conv cb x6");
  if (rc == 0 && y_oct != nullptr && y_oct_k == nullptr) rc = pack_octets(y, y_oct, d->num, d->num_output, HW, s);
  return rc ? rc : 1;
}

// ---- k_conv1x1_x6 plan ----
struct C1Plan {
  int MI, NB, WR, VEC, tiles_m, tiles_n;
};
// (MI, NB, WR) instantiated for VEC = 4 and VEC = 1
#define RRAM_C1X1_LIST(X) X(1, 2, 1) X(2, 1, 1) X(2, 2, 1) X(2, 1, 2) X(4, 1, 1) X(4, 2, 1) X(4, 1, 2) X(4, 2, 2)
bool conv_1x1_plan(const rram_conv_desc* d, const float* x, C1Plan& pl) {
  if (d->kernel_h != 1 || d->kernel_w != 1 || d->stride_h != 1 || d->stride_w != 1 || d->pad_h != 0 ||
      d->pad_w != 0 || d->dilation_h != 1 || d->dilation_w != 1 || d->group != 1)
    return false;
  const int M = d->num_output, C = d->channels, HW = d->height * d->width;
  if (C % 16 != 0 || M < 1 || d->num < 1) return false;
  const int64_t N = (int64_t)d->num * HW;
  if ((int64_t)d->num * C * HW * 4 >= (1ll << 31) || (int64_t)d->num * M * HW * 4 >= (1ll << 31)) return false;
  if (x != nullptr && (reinterpret_cast<uintptr_t>(x) & 3u) != 0) return false;
  const bool v4 = HW % 4 == 0 && (x == nullptr || (reinterpret_cast<uintptr_t>(x) & 15u) == 0);
  // least estimated time: MFMA makespan (rounds of 256 workgroups x tile work
  // at the bf16x6 rate of one CU) against the HBM stream (input once per M-tile)
  static const int cfg[][3] = {{1, 2, 1}, {2, 1, 1}, {2, 2, 1}, {2, 1, 2}, {4, 1, 1}, {4, 2, 1}, {4, 1, 2}, {4, 2, 2}};
  double best = -1.0;
  for (const auto& c : cfg) {
    const int MI = c[0], NB = c[1], WR = c[2];
    const int BM = 32 * MI * WR, BN = 32 * NB * (4 / WR);
    if (BM > 32 && (BM / 2) >= M) continue;                  // half the tile would pad
    const int64_t tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
    if (tm * tn >= (1ll << 31)) continue;
    const double t_mfma = (double)((tm * tn + 255) / 256) * BM * BN * C * 2.0 / (416.7e12 / 256);
    const double t_mem = ((double)tm * N * C * 4 + (double)N * M * 4) / 5.0e12;
    const double t = std::max(t_mfma, t_mem) * (1.0 + 0.02 * (MI * NB == 8 ? 0 : 1));
    if (best < 0 || t < best) {
      best = t;
      pl = C1Plan{MI, NB, WR, v4 ? 4 : 1, static_cast<int>(tm), static_cast<int>(tn)};
    }
  }
  return best >= 0;
}

int conv_1x1_x6_fwd(const rram_conv_desc* d, const float* x, const float* w, const float* bias, float* y, void* y_oct,
                    int relu, hipStream_t s, const WPack& wk) {
  C1Plan pl;
  if (!conv_1x1_plan(d, wk.query ? nullptr : x, pl)) return 0;
  const int M = d->num_output, C = d->channels, HW = d->height * d->width;
  // y = NULL (the convolution-output fold): the epilogue writes the companion alone
  RRAM_REQUIRE(y != nullptr || wk.query != nullptr || (y_oct != nullptr && M % 8 == 0),
               "conv 1x1: y = NULL needs the octet companion (num_output % 8 == 0)");
  const int BMc = 32 * pl.MI * pl.WR;
  const int rblocks = pl.tiles_m * (BMc / 32);
  const int64_t wfrags = (int64_t)rblocks * (C / 16);
  if (wk.query) {
    *wk.query = static_cast<size_t>(wfrags * 3072);
    return 1;
  }
  Params P{};
  P.M = M;
  P.N = d->num * HW;
  P.K = C;
  P.split = 1;
  P.cv.C = C;
  P.cv.howo = make_fastdiv(HW);
  P.e = make_epi(y, HW, 1.0f, 0.0f, bias, RRAM_BIAS_ROW, relu);
  P.e.cimg = wk.y_img > 0 ? wk.y_img : (int64_t)M * HW;
  P.e.hw = make_fastdiv(HW);
  P.tiles_m = pl.tiles_m;
  P.tiles_n = pl.tiles_n;
  P.tiles_z = 1;
  char* wbuf = wk.p ? static_cast<char*>(wk.p) : reinterpret_cast<char*>(pack_buffer(static_cast<size_t>(wfrags * 768), s));
  RRAM_REQUIRE(wbuf != nullptr, "conv 1x1: packed-weight buffer allocation failed");
  if (!wk.valid) {
    const int wunits = static_cast<int>(wfrags * 64);
    hipLaunchKernelGGL(k_conv_cb_pack_x6, dim3(stream_blocks(wunits)), dim3(256), 0, s, w, wbuf, M, C, 1, rblocks,
                       wunits);
    const int rc = launch_status("conv 1x1 weight pack x6");
    if (rc) return rc;
  }
  const auto* wp = reinterpret_cast<const x6::bf16x8*>(wbuf);
  const uint32_t xrange = static_cast<uint32_t>((int64_t)d->num * C * HW * 4);
  const unsigned nwg = static_cast<unsigned>((int64_t)pl.tiles_m * pl.tiles_n);
  const uint32_t wrange = static_cast<uint32_t>(wfrags * 3072);
  // the output's octet companion straight from the epilogue (whole octets: M % 8 == 0)
  char* const yo = (y_oct != nullptr && M % 8 == 0) ? static_cast<char*>(y_oct) : nullptr;
  const int cout8 = M / 8;
  // the DMA form measured faster where the weight panel is tall (M > 64: 4-18 %
  // per layer), the register ring on 16-byte loads with M <= 64 and on the
  // 4-byte loads of the 7 x 7 layers (profiles/r04_ab_conv1x1.txt)
  const bool dma = pl.VEC == 4 && M > 64;
#define RRAM_X(mi, nb, wr)                                                                                  \
  if (pl.MI == mi && pl.NB == nb && pl.WR == wr) {                                                          \
    if (dma && pl.VEC == 4)                                                                                 \
      hipLaunchKernelGGL((k_conv1x1_dma_x6<mi, nb, wr, 4>), dim3(nwg), dim3(256), 0, s, P, wp, x, xrange,   \
                         wrange, yo, cout8);                                                                \
    else if (dma)                                                                                           \
      hipLaunchKernelGGL((k_conv1x1_dma_x6<mi, nb, wr, 1>), dim3(nwg), dim3(256), 0, s, P, wp, x, xrange,   \
                         wrange, yo, cout8);                                                                \
    else if (pl.VEC == 4)                                                                                   \
      hipLaunchKernelGGL((k_conv1x1_x6<mi, nb, wr, 4>), dim3(nwg), dim3(256), 0, s, P, wp, x, xrange, yo,   \
                         cout8);                                                                            \
    else                                                                                                    \
      hipLaunchKernelGGL((k_conv1x1_x6<mi, nb, wr, 1>), dim3(nwg), dim3(256), 0, s, P, wp, x, xrange, yo,   \
                         cout8);                                                                            \
  } else
  RRAM_C1X1_LIST(RRAM_X) { return 0; }
#undef RRAM_X
  int rc = launch_status("conv 1x1 x6");
  if (rc == 0 && y_oct != nullptr && yo == nullptr) rc = pack_octets(y, y_oct, d->num, M, HW, s);
  return rc ? rc : 1;
}

int conv_patch_x6_fwd(const rram_conv_desc* d, const float* x, const float* w, const float* bias, float* y, int relu,
                      hipStream_t s, const WPack& wk);
// The bf16x6 convolution forward.  x_oct: NULL or the octet companion of x
// (k_pack_octets_x6 layout; the channel-octet kernel then skips its input
// pack); y_oct: NULL or a buffer that receives y's octet companion (written
// by the channel-octet kernel's epilogue, else packed from y afterwards).
// Returns 1 when it ran, 0 when not covered (nothing written), < 0 on error.
int conv_x6_fwd(const rram_conv_desc* d, const float* x, const void* x_oct, const float* w, const float* bias,
                float* y, void* y_oct, int relu, hipStream_t s, const WPack& wk) {
  if (f32_engine().load(std::memory_order_relaxed) != RRAM_ENGINE_BF16X6) return 0;
  if (wk.query == nullptr && (reinterpret_cast<uintptr_t>(w) & 3u) != 0) return 0;
  // the epilogues' 32-bit output offsets also hold a strided (Concat-slice) image stride
  if (wk.y_img > 0 && (int64_t)d->num * wk.y_img * 4 >= (1ll << 31)) return 0;
  {
    const int rc = conv_cb_x6_fwd(d, x, x_oct, w, bias, y, y_oct, relu, s, wk);
    if (rc != 0) return rc;
  }
  {
    const int rc1 = conv_1x1_x6_fwd(d, x, w, bias, y, y_oct, relu, s, wk);  // writes y_oct itself
    if (rc1 != 0) return rc1;
  }
  // only the channel-octet and 1x1 kernels' epilogues write a companion without y
  RRAM_REQUIRE(y != nullptr || wk.query != nullptr,
               "conv: y = NULL needs a companion-writing epilogue (rram_conv_output_octets_only)");
  int rc = conv_wide_x6_fwd(d, x, w, bias, y, relu, s, wk);
  if (rc == 0) rc = conv_s2_x6_fwd(d, x, w, bias, y, relu, s, wk);
  if (rc == 0) rc = conv_patch_x6_fwd(d, x, w, bias, y, relu, s, wk);
  if (wk.query) return rc;
  if (rc > 0 && y_oct != nullptr) {
    const int pr = pack_octets(y, y_oct, d->num, d->num_output, d->out_h * d->out_w, s);
    if (pr) return pr;
  }
  return rc;
}

int conv_patch_x6_fwd(const rram_conv_desc* d, const float* x, const float* w, const float* bias, float* y, int relu,
                      hipStream_t s, const WPack& wk) {
  ConvPlan pl;
  if (!conv_x6_plan(d, pl)) return 0;
  const int KH = d->kernel_h, KW = d->kernel_w;
  const int G = d->group, Cg = d->channels / G, M = d->num_output / G;
  const int HW = d->out_h * d->out_w, OW = d->out_w, OH = d->out_h;
  const int CPH = pl.CPH, MI = pl.MI, mt = pl.mt, PW = pl.PW, CS = pl.CS, PD = pl.PD;
  Params P{};
  P.M = M;
  P.N = d->num * HW;
  P.K = Cg * KH * KW;
  P.split = 1;
  P.b = make_view(x, 0, P.N, P.K);
  ConvGeom& cv = P.cv;
  cv.C = Cg;
  cv.H = d->height;
  cv.W = d->width;
  cv.KH = KH;
  cv.KW = KW;
  cv.ph = d->pad_h;
  cv.pw = d->pad_w;
  cv.sh = cv.sw = cv.dh = cv.dw = 1;
  cv.Ho = OH;
  cv.Wo = OW;
  cv.howo = make_fastdiv(HW);
  cv.wo_div = make_fastdiv(OW);
  cv.chw = (int64_t)d->channels * d->height * d->width;
  cv.in_bytes = static_cast<int>((int64_t)d->num * cv.chw * 4);
  P.e = make_epi(y, HW, 1.0f, 0.0f, bias, RRAM_BIAS_ROW, relu);
  P.e.cimg = wk.y_img > 0 ? wk.y_img : (int64_t)d->num_output * HW;
  P.e.hw = make_fastdiv(HW);
  P.grp_b = (int64_t)Cg * d->height * d->width;
  P.grp_c = (int64_t)M * HW;
  P.grp_bias = M;
  const int T = KH * KW, S = CPH * T, G8 = (S + 7) / 8, RLH = (G8 * 96 + 16) / 2;
  const int BMc = 32 * MI, tiles_m = mt / BMc, ktiles = Cg / (2 * CPH);
  const int64_t total = (int64_t)G * tiles_m * ktiles * BMc * RLH;
  if (wk.query) {
    *wk.query = static_cast<size_t>(total * 2);
    return 1;
  }
  uint16_t* wp = reinterpret_cast<uint16_t*>(wk.p ? wk.p : pack_buffer(static_cast<size_t>((total + 1) / 2), s));
  RRAM_REQUIRE(wp != nullptr, "conv: packed-weight buffer allocation failed");
  int rc = 0;
  if (!wk.valid) {
    const int units = G * tiles_m * ktiles * BMc * G8 * 2;
    hipLaunchKernelGGL(k_conv_patch_pack_x6, dim3(stream_blocks(units)), dim3(256), 0, s, w,
                       reinterpret_cast<char*>(wp), G, M, Cg, T, CPH, G8, 2 * RLH, BMc, tiles_m, ktiles, units);
    rc = launch_status("conv weight pack x6");
    if (rc) return rc;
  }
#define RRAM_P(KH_, CPH_, PD_)                                                                           \
  if (KH == KH_ && CPH == CPH_ && PD == PD_)                                                             \
    rc = MI == 3 ? launch_patch_x6<KH_, CPH_, 3, PD_>(P, wp, PW, CS, G, s)                               \
                 : launch_patch_x6<KH_, CPH_, 4, PD_>(P, wp, PW, CS, G, s);                              \
  else
  RRAM_P(5, 1, 4) RRAM_P(5, 1, 8) RRAM_P(5, 1, 12)
  RRAM_P(3, 4, 8) RRAM_P(3, 4, 12) RRAM_P(3, 4, 16)
  RRAM_P(3, 2, 4) RRAM_P(3, 2, 8) RRAM_P(3, 2, 16)
  return 0;
#undef RRAM_P
  return rc ? rc : 1;
}


// shape plan of the x6 GEMM (false: not covered)
struct GemmPlan {
  int MI, NJ, tiles_m, tiles_n, ktiles, split, ktc;
};
bool gemm_x6_plan(int M, int N, int K, size_t ws_bytes, GemmPlan& pl) {
  if (K < 256 || K % 4 != 0 || (int64_t)M * N * K < (1ll << 24)) return false;
  // 256 x 128 tiles (every weight row read by one tile row) when <= 1/4 of
  // the rows pad, else 128 (or 96) x 256
  const int t256 = (M + 255) / 256 * 256, t128 = (M + 127) / 128 * 128, t96 = (M + 95) / 96 * 96;
  // (128 x 256 tiles for fc6 / fc7 measured 1-3 % slower, round 4)
  // (an 8-wave 128 x 256 form, two waves per SIMD, measured no faster on
  // fc6 / fc7: 0.122-0.124 vs 0.122-0.124 ms, profiles/r05_ab_occ2_plans.txt)
  if ((t256 - M) * 4 <= t256) {
    pl.MI = 8;
    pl.NJ = 1;
  } else {
    pl.MI = (t96 - M) < (t128 - M) ? 3 : 4;
    pl.NJ = 2;
  }
  const int BMc = 32 * pl.MI, BNc = 128 * pl.NJ;
  pl.tiles_m = (M + BMc - 1) / BMc;
  pl.tiles_n = (N + BNc - 1) / BNc;
  pl.ktiles = (K + gx6::KT - 1) / gx6::KT;
  // split-K toward 256 workgroups, >= 8 K-tiles (256 k) per split
  const int64_t tiles = (int64_t)pl.tiles_m * pl.tiles_n;
// (32 splits of >= 4 K-tiles, which moves fc8 onto this kernel, measured
// 0.034 vs 0.032 ms on the fp32 engine: profiles/r05_ab_fc8_split32.txt)
#ifndef RRAM_X6_SPLIT_MAX
#define RRAM_X6_SPLIT_MAX 16
#endif
#ifndef RRAM_X6_MIN_KT
#define RRAM_X6_MIN_KT 8
#endif
  int split = 1;
  if (ws_bytes > 0 && tiles < 256) {
    split = static_cast<int>(std::min<int64_t>(RRAM_X6_SPLIT_MAX, 256 / tiles));
    while (split > 1 && pl.ktiles / split < RRAM_X6_MIN_KT) --split;
    while (split > 1 && (size_t)split * M * N * sizeof(float) > ws_bytes) --split;
  }
  pl.ktc = (pl.ktiles + split - 1) / split;
  pl.split = (pl.ktiles + pl.ktc - 1) / pl.ktc;
  // under ~3/4 of the CUs busy the fp32 kernel's smaller tiles fill more
  // (fc8 at 128 workgroups: 38 us here vs 35 on fp32, profiles/r02_ab_fc8_x6.txt)
  if (tiles * pl.split < 192) return false;
  return (int64_t)pl.tiles_m * pl.ktiles * BMc * gx6::RLB < (1ll << 31);
}

// k_gemm_x6 for C = act(alpha * A . B^T + bias) with A [M][lda], B [N][ldb]
// row-major fp32 (16-byte aligned rows), beta = 0.  Returns 1 when it ran, 0
// when not covered (the caller runs the fp32-MFMA GEMM), < 0 on error.
// a_rows (nullable): A already in the packed-row form of this plan (no pack
// pass); y_rows (nullable): C also written in the packed-row form of a
// consumer with y_bmc rows per tile and K = N (by the split-K reduce when it
// can, else by a pack pass of C)
int gemm_x6_nt(int M, int N, int K, float alpha, const float* A, int lda, const float* B, int ldb, float beta,
               float* C, int ldc, const float* bias, int bias_mode, int relu, void* ws, size_t ws_bytes,
               hipStream_t s, const void* a_rows, char* y_rows, int y_bmc) {
  if (f32_engine().load(std::memory_order_relaxed) != RRAM_ENGINE_BF16X6 || beta != 0.0f) return 0;
  auto al16 = [](const void* p, int ld) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0 && ld % 4 == 0; };
  if (!al16(A, lda) || !al16(B, ldb)) return 0;
  if ((int64_t)(N - 1) * ldb * 4 + (int64_t)K * 4 >= (1ll << 32)) return 0;  // 32-bit buffer offsets
  GemmPlan pl;
  if (!gemm_x6_plan(M, N, K, ws != nullptr ? ws_bytes : 0, pl)) return 0;
  const int MI = pl.MI, BMc = 32 * MI, tiles_m = pl.tiles_m, tiles_n = pl.tiles_n, ktiles = pl.ktiles;
  const int split = pl.split, ktc = pl.ktc;
  const int64_t tiles = (int64_t)tiles_m * tiles_n;
  const int64_t total = (int64_t)tiles_m * ktiles * BMc * (gx6::RLB / 2);
  const uint16_t* ap = static_cast<const uint16_t*>(a_rows);
  int rc = 0;
  if (ap == nullptr) {
    uint16_t* pb = reinterpret_cast<uint16_t*>(pack_buffer(static_cast<size_t>((total + 1) / 2), s));
    RRAM_REQUIRE(pb != nullptr, "gemm x6: packed-operand buffer allocation failed");
    const int units = tiles_m * BMc * ktiles * 4;
    hipLaunchKernelGGL(k_pack_rows_x6, dim3(stream_blocks(units)), dim3(256), 0, s, A, (int64_t)lda, M, K,
                       reinterpret_cast<char*>(pb), BMc, ktiles, units);
    rc = launch_status("gemm x6 pack");
    if (rc) return rc;
    ap = pb;
  }
  Params P{};
  P.M = M;
  P.N = N;
  P.K = K;
  P.b = make_view(B, ldb, N, K);
  P.e = make_epi(C, ldc, alpha, 0.0f, bias, bias_mode, relu);
  P.split = split;
  P.ws = split > 1 ? static_cast<float*>(ws) : nullptr;
  P.tiles_m = tiles_m;
  P.tiles_n = tiles_n;
  P.tiles_z = split;
  const unsigned nwg = static_cast<unsigned>(tiles * split);
  if (MI == 8)
    hipLaunchKernelGGL((k_gemm_x6<8, 1>), dim3(nwg), dim3(256), 0, s, P, ap, ktiles, ktc);
  else if (MI == 3)
    hipLaunchKernelGGL((k_gemm_x6<3, 2>), dim3(nwg), dim3(256), 0, s, P, ap, ktiles, ktc);
  else
    hipLaunchKernelGGL((k_gemm_x6<4, 2>), dim3(nwg), dim3(256), 0, s, P, ap, ktiles, ktc);
  rc = launch_status("gemm x6");
  if (rc) return rc;
  const bool rows_in_reduce = y_rows != nullptr && split > 1 && N % 32 == 0 && y_bmc > 0 && M % y_bmc == 0 &&
                              ldc % 4 == 0 && (reinterpret_cast<uintptr_t>(C) & 15u) == 0;
  if (split > 1 && rows_in_reduce) {
    const int units = M * (N / 8);
    hipLaunchKernelGGL(k_splitk_reduce_rows_x6, dim3(stream_blocks(units)), dim3(256), 0, s, P.ws, split, M, N, P.e,
                       y_rows, y_bmc, N / gx6::KT, units);
    rc = launch_status("gemm x6 splitk reduce + rows");
    if (rc) return rc;
  } else if (split > 1) {
    hipLaunchKernelGGL(k_splitk_reduce, dim3(stream_blocks((int64_t)M * N)), dim3(256), 0, s, P.ws, split, M, N,
                       P.e);
    rc = launch_status("gemm x6 splitk reduce");
    if (rc) return rc;
  }
  if (y_rows != nullptr && !rows_in_reduce) {  // the consumer's pack of C, as its own call would run it
    const int ytm = (M + y_bmc - 1) / y_bmc, ykt = (N + gx6::KT - 1) / gx6::KT;
    const int units = ytm * y_bmc * ykt * 4;
    hipLaunchKernelGGL(k_pack_rows_x6, dim3(stream_blocks(units)), dim3(256), 0, s, C, (int64_t)ldc, M, N, y_rows,
                       y_bmc, ykt, units);
    rc = launch_status("gemm x6 rows of C");
    if (rc) return rc;
  }
  return 1;
}

}  // namespace rram

extern "C" {

#ifdef RRAM_CB_STAMP
// diagnostic build only: the 3x3 octet-kernel stamp sums (and reset)
int rram_debug_cb_stamps(unsigned long long* out, int n) {
  if (out != nullptr && hipMemcpyFromSymbol(out, HIP_SYMBOL(rram::g_cb_stamp), sizeof(unsigned long long) * n) != hipSuccess)
    return -2;
  unsigned long long z[64] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(rram::g_cb_stamp), z, sizeof(z)) == hipSuccess ? 0 : -2;
}
#endif
#ifdef RRAM_C1_STAMP
// diagnostic build only: the conv1 stamp sums (and reset)
int rram_debug_c1_stamps(unsigned long long* out, int n) {
  if (out != nullptr && hipMemcpyFromSymbol(out, HIP_SYMBOL(rram::g_c1_stamp), sizeof(unsigned long long) * n) != hipSuccess)
    return -2;
  unsigned long long z[64] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(rram::g_c1_stamp), z, sizeof(z)) == hipSuccess ? 0 : -2;
}
#endif

int rram_f32_engine_for_conv(const rram_conv_desc* d) {
  RRAM_REQUIRE(d != nullptr, "engine query: desc is NULL");
  rram::ConvPlan pl;
  rram::CbPlan cpl;
  rram::C1Plan c1;
  return rram::f32_engine().load() == RRAM_ENGINE_BF16X6 &&
                 (rram::conv_x6_plan(d, pl) || rram::conv1_ring_ok(d) || rram::conv_s2_ok(d) ||
                  rram::conv_cb_plan(d, cpl) || rram::conv_1x1_plan(d, nullptr, c1))
             ? RRAM_ENGINE_BF16X6
             : RRAM_ENGINE_F32;
}

int rram_conv_octet_plan(const rram_conv_desc* d, int* plan) {
  RRAM_REQUIRE(d != nullptr && plan != nullptr, "octet plan query: NULL");
  rram::CbPlan cpl;
  if (!rram::conv_cb_plan(d, cpl)) return 0;
  plan[0] = 32 * cpl.WR;
  plan[1] = 32 * cpl.NB * (4 / cpl.WR);
  plan[2] = cpl.OCC;
  plan[3] = cpl.tpi;
  plan[4] = cpl.PD;
  return 1;
}

int rram_conv_output_octets_only(const rram_conv_desc* d_in) {
  RRAM_REQUIRE(d_in != nullptr, "output octets query: desc is NULL");
  if (rram::f32_engine().load(std::memory_order_relaxed) != RRAM_ENGINE_BF16X6) return 0;
  rram_conv_desc d = *d_in;
  if (rram_conv_out_shape(&d) != RRAM_OK || d.num == 0 || d.num_output % 8 != 0) return 0;
  // the 1x1 kernels write the companion from their epilogue (whole octets)
  rram::C1Plan c1;
  if (rram::conv_1x1_plan(&d, nullptr, c1)) return 1;
  rram::CbPlan pl;
  if (!rram::conv_cb_plan(&d, pl)) return 0;
  return pl.OCC == 2 && (d.num_output / d.group) % 8 == 0 ? 1 : 0;
}

int rram_conv_input_octets(const rram_conv_desc* d) {
  RRAM_REQUIRE(d != nullptr, "octet query: desc is NULL");
  rram::CbPlan cpl;
  return rram::f32_engine().load() == RRAM_ENGINE_BF16X6 && rram::conv_cb_plan(d, cpl) ? 1 : 0;
}

int rram_pack_octets(const float* x, void* oct, int num, int channels, int height, int width, rram_stream_t s) {
  RRAM_REQUIRE(num >= 0 && channels > 0 && height > 0 && width > 0, "pack_octets: bad shape");
  if (num == 0) return RRAM_OK;
  RRAM_REQUIRE(x != nullptr && oct != nullptr, "pack_octets: NULL");
  return rram::pack_octets(x, oct, num, channels, height * width, rram::as_stream(s));
}

size_t rram_ip_rows_pack_bytes(int M, int N, int K, size_t ws_bytes, int* rows_per_tile) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  rram::GemmPlan pl;
  if (rram::f32_engine().load() != RRAM_ENGINE_BF16X6 || !rram::gemm_x6_plan(M, N, K, ws_bytes, pl)) return 0;
  if (rows_per_tile) *rows_per_tile = 32 * pl.MI;
  return (size_t)pl.tiles_m * pl.ktiles * 32 * pl.MI * rram::gx6::RLB;
}

int rram_ip_fwd_rows(const float* x, const void* x_rows, const float* w, const float* bias, float* y, void* y_rows,
                     int y_rows_per_tile, int M, int N, int K, int relu, void* ws, size_t ws_bytes,
                     int* y_rows_written, rram_stream_t st) {
  RRAM_REQUIRE(M > 0 && N > 0 && K > 0 && x && w && y, "ip_fwd_rows: bad arguments");
  RRAM_REQUIRE(y_rows == nullptr || y_rows_per_tile > 0, "ip_fwd_rows: y_rows without its tile rows");
  if (y_rows_written) *y_rows_written = 0;
  hipStream_t s = rram::as_stream(st);
  const int rc = rram::gemm_x6_nt(M, N, K, 1.0f, x, K, w, K, 0.0f, y, N, bias, RRAM_BIAS_COL, relu, ws, ws_bytes, s,
                                  x_rows, static_cast<char*>(y_rows), y_rows_per_tile);
  if (rc < 0) return rc;
  if (rc == 0) {  // not served: the plain forward, no rows written
    RRAM_REQUIRE(x_rows == nullptr, "ip_fwd_rows: x_rows given for a shape the engine does not serve");
    return rram_ip_fwd(x, w, bias, y, M, N, K, 0, relu, ws, ws_bytes, st);
  }
  if (y_rows_written) *y_rows_written = y_rows != nullptr ? 1 : 0;
  return RRAM_OK;
}

int rram_f32_engine_for_ip(int M, int N, int K, size_t ws_bytes) {
  RRAM_REQUIRE(M >= 0 && N >= 0 && K >= 0, "engine query: negative size");
  rram::GemmPlan pl;
  return rram::f32_engine().load() == RRAM_ENGINE_BF16X6 && rram::gemm_x6_plan(M, N, K, ws_bytes, pl)
             ? RRAM_ENGINE_BF16X6
             : RRAM_ENGINE_F32;
}

}  // extern "C"
