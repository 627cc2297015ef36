// Fault-model kernels for gfx950: the reference's FailKernel / threshold
// kernel, the Monte-Carlo injection kernel (counter-based RNG), the threshold
// strategy and the SGD / fused training tail.  All are HBM-streaming kernels:
// 16-byte (float4) loads and stores per lane where the pointers allow it,
// 256-thread blocks, grid-stride, wave-level ballot reductions for counters.
#include <atomic>
#include <math.h>
#include <stdlib.h>

#include "rram_common.hpp"

namespace rram {

namespace {

__device__ __forceinline__ bool aligned16(const void* p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

// Block-level sum of per-lane counts, ONE atomic per block.  Many waves
// adding to one address serialise at the memory side (MI355X_MICROARCH.md
// "Global float atomics", contention row), so counters are flushed per block,
// and per block only when its segment changes or its loop ends.
// Must be reached by every thread of the block (contains __syncthreads).
__device__ __forceinline__ void block_count_flush(unsigned cnt, unsigned long long* counter) {
  __shared__ unsigned part[4];
  unsigned v = cnt;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0 && counter != nullptr) {
    const unsigned t = part[0] + part[1] + part[2] + part[3];
    if (t) atomicAdd(counter, static_cast<unsigned long long>(t));
  }
}
__device__ __forceinline__ void wave_count_add_n(unsigned cnt, unsigned long long* counter) {
  block_count_flush(cnt, counter);
}

// ---------------------------------------------------------------------------
// a1: FailureThresholdKernel equivalent
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_fault_threshold(float* __restrict__ v, int64_t n, float s1,
                                                         float s2) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float u = v[i];
    v[i] = (u < s1) ? -1.0f : ((u < s2) ? 0.0f : 1.0f);
  }
}

__device__ __forceinline__ float stuck_value(uint32_t r, uint64_t thr_neg, uint64_t thr_zero) {
  return (static_cast<uint64_t>(r) < thr_neg) ? -1.0f
                                              : ((static_cast<uint64_t>(r) < thr_zero) ? 0.0f : 1.0f);
}

// Box-Muller pair from two 32-bit words.
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
  const float u1 = u01_open0(a);
  const float u2 = u01(b);
  const float r = sqrtf(-2.0f * logf(u1));
  const float th = 6.28318530717958647692f * u2;
  float s, c;
  sincosf(th, &s, &c);
  z0 = r * c;
  z1 = r * s;
}

__global__ void __launch_bounds__(256)
    k_fault_init(float* __restrict__ e, float* __restrict__ v, int64_t n, float mean, float std,
                 uint64_t thr_neg, uint64_t thr_zero, uint64_t seed, uint32_t map_id,
                 uint32_t layer_id) {
  const int64_t npairs = (n + 1) / 2;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < npairs;
       p += (int64_t)gridDim.x * blockDim.x) {
    const U32x4 re = draw(seed, p, map_id, layer_id, kPurposeEndurance);
    const U32x4 rf = draw(seed, p, map_id, layer_id, kPurposeFault);
    float z0, z1;
    box_muller(re.x, re.y, z0, z1);
    const int64_t i0 = 2 * p;
    e[i0] = fmaf(std, z0, mean);
    v[i0] = stuck_value(rf.y, thr_neg, thr_zero);
    if (i0 + 1 < n) {
      e[i0 + 1] = fmaf(std, z1, mean);
      v[i0 + 1] = stuck_value(rf.w, thr_neg, thr_zero);
    }
  }
}

// ---------------------------------------------------------------------------
// a2: FailKernel equivalent (bit-exact fp32 arithmetic)
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool fail_one(float dw, float& w, float& e, float v, float dec,
                                         float eps, bool& wrote_w) {
  wrote_w = false;
  if (e <= 0.0f) {
    w = v;
    wrote_w = true;
  } else if (!(dw < eps && dw > -eps)) {
    e = e - dec;
    if (e <= 0.0f) {
      w = v;
      wrote_w = true;
    }
  }
  return e <= 0.0f;
}

struct FailSegs {
  rram_fail_seg s[RRAM_MAX_SEGS];
  int64_t chunk_start[RRAM_MAX_SEGS + 1];  // prefix of chunks per segment
  int nsegs;
};

constexpr int kFailChunk = 256 * 4 * 4;  // elements per block-chunk

__device__ __forceinline__ unsigned fail_range(const float* __restrict__ dw, float* __restrict__ w,
                                               float* __restrict__ e, const float* __restrict__ v,
                                               int64_t begin, int64_t end, float dec, float eps) {
  const bool vec = aligned16(dw + begin) && aligned16(w + begin) && aligned16(e + begin) &&
                   aligned16(v + begin);
  unsigned cnt = 0;
  if (vec) {
    const int64_t nv = (end - begin) / 4;
    const float4* dw4 = reinterpret_cast<const float4*>(dw + begin);
    float4* e4 = reinterpret_cast<float4*>(e + begin);
    const float4* v4 = reinterpret_cast<const float4*>(v + begin);
    float* wb = w + begin;
    for (int64_t i = threadIdx.x; i < nv; i += blockDim.x) {
      const float4 g = dw4[i];
      float4 ee = e4[i];
      const float4 vv = v4[i];
      float wv[4];
      bool wr[4];
      cnt += fail_one(g.x, wv[0], ee.x, vv.x, dec, eps, wr[0]);
      cnt += fail_one(g.y, wv[1], ee.y, vv.y, dec, eps, wr[1]);
      cnt += fail_one(g.z, wv[2], ee.z, vv.z, dec, eps, wr[2]);
      cnt += fail_one(g.w, wv[3], ee.w, vv.w, dec, eps, wr[3]);
      e4[i] = ee;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (wr[j]) wb[4 * i + j] = wv[j];
    }
    for (int64_t i = begin + 4 * nv + threadIdx.x; i < end; i += blockDim.x) {
      float ww, ee = e[i];
      bool wr;
      cnt += fail_one(dw[i], ww, ee, v[i], dec, eps, wr);
      e[i] = ee;
      if (wr) w[i] = ww;
    }
  } else {
    for (int64_t i = begin + threadIdx.x; i < end; i += blockDim.x) {
      float ww, ee = e[i];
      bool wr;
      cnt += fail_one(dw[i], ww, ee, v[i], dec, eps, wr);
      e[i] = ee;
      if (wr) w[i] = ww;
    }
  }
  return cnt;
}

__global__ void __launch_bounds__(256)
    k_fail_apply_batched(FailSegs segs, float dec, float eps, unsigned long long* counters) {
  const int64_t total = segs.chunk_start[segs.nsegs];
  int cur = -1;  // block-uniform: flush the count once per segment visited
  unsigned cnt = 0;
  for (int64_t c = blockIdx.x; c < total; c += gridDim.x) {
    int s = 0;
    while (c >= segs.chunk_start[s + 1]) ++s;
    if (s != cur) {
      if (cur >= 0) block_count_flush(cnt, counters ? counters + cur : nullptr);
      cnt = 0;
      cur = s;
    }
    const rram_fail_seg& sg = segs.s[s];
    const int64_t begin = (c - segs.chunk_start[s]) * kFailChunk;
    const int64_t end = min(begin + (int64_t)kFailChunk, sg.n);
    cnt += fail_range(sg.dw, sg.w, sg.endurance, sg.values, begin, end, dec, eps);
  }
  if (cur >= 0) block_count_flush(cnt, counters ? counters + cur : nullptr);
}

__global__ void __launch_bounds__(256)
    k_broken_count(const float* __restrict__ e, int64_t n, unsigned long long* counter) {
  unsigned cnt = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    cnt += (e[i] <= 0.0f);
  wave_count_add_n(cnt, counter);
}

// ---------------------------------------------------------------------------
// Monte-Carlo injection
// ---------------------------------------------------------------------------
struct InjectSeg {
  const float* src;
  float* dst;
  int64_t n;
  uint32_t layer_id;
  int32_t mode;          // 0 plain stuck-at fast path, 1 general single, 2 diff-pair
  uint64_t thr_fault, thr_neg, thr_zero, thr_sa1;
  float stuck_scale, g_max;
  int32_t levels;
  float q_delta, q_inv;  // quantisation step and its reciprocal (host-computed)
  float sigma;
};

struct InjectSegs {
  InjectSeg s[RRAM_MAX_SEGS];
  int64_t chunk_start[RRAM_MAX_SEGS + 1];
  int nsegs;
};

constexpr int kInjChunk = 256 * 4 * 4;  // elements per block-chunk (4 float4 per lane)
constexpr int kInjectGrid = 2048;      // default persistent grid
// rram_set_inject_grid: a caller-chosen grid (0: kInjectGrid), e.g. a smaller
// one when the injection runs beside other kernels (MonteCarlo's overlap)
std::atomic<int>& inject_grid() {
  static std::atomic<int> g{0};
  return g;
}

__device__ __forceinline__ float quantize_sym(float w, const InjectSeg& g) {
  // uniform levels over [-g_max, g_max]
  float t = (w + g.g_max) * g.q_inv;
  t = rintf(t);
  t = fminf(fmaxf(t, 0.0f), static_cast<float>(g.levels - 1));
  return fmaf(t, g.q_delta, -g.g_max);
}
__device__ __forceinline__ float quantize_pos(float x, const InjectSeg& g) {
  // uniform levels over [0, g_max]
  float t = x * g.q_inv;
  t = rintf(t);
  t = fminf(fmaxf(t, 0.0f), static_cast<float>(g.levels - 1));
  return t * g.q_delta;
}

// General single-cell element: quantise -> stuck-at -> variation.
__device__ __forceinline__ float inject_single(float w, uint32_t rf, uint32_t rv, bool has_z, float z,
                                               const InjectSeg& g, bool& broken) {
  if (g.levels >= 2) w = quantize_sym(w, g);
  broken = static_cast<uint64_t>(rf) < g.thr_fault;
  if (broken) return stuck_value(rv, g.thr_neg, g.thr_zero) * g.stuck_scale;
  if (has_z) w = w * expf(g.sigma * z);
  return w;
}

__device__ __forceinline__ float inject_pair(float w, uint64_t idx, uint64_t seed, uint32_t map_id,
                                             const InjectSeg& g, unsigned& nbroken) {
  float gp = fmaxf(w, 0.0f);
  float gn = fmaxf(-w, 0.0f);
  if (g.levels >= 2) {
    gp = quantize_pos(gp, g);
    gn = quantize_pos(gn, g);
  }
  const U32x4 r = draw(seed, idx, map_id, g.layer_id, kPurposePairFault);
  const bool bp = static_cast<uint64_t>(r.x) < g.thr_fault;
  const bool bn = static_cast<uint64_t>(r.z) < g.thr_fault;
  if (g.sigma > 0.0f && !(bp && bn)) {
    const U32x4 rz = draw(seed, idx, map_id, g.layer_id, kPurposePairVar);
    float z0, z1;
    box_muller(rz.x, rz.y, z0, z1);
    gp = gp * expf(g.sigma * z0);
    gn = gn * expf(g.sigma * z1);
  }
  if (bp) gp = (static_cast<uint64_t>(r.y) < g.thr_sa1) ? g.g_max : 0.0f;
  if (bn) gn = (static_cast<uint64_t>(r.w) < g.thr_sa1) ? g.g_max : 0.0f;
  nbroken += static_cast<unsigned>(bp) + static_cast<unsigned>(bn);
  return gp - gn;
}

// Four consecutive elements starting at an even index i (two RNG pairs).
template <bool FAST>
__device__ __forceinline__ float4 inject4(float4 w, int64_t i, uint64_t seed, uint32_t map_id,
                                          const InjectSeg& g, unsigned& nb) {
  float o[4] = {w.x, w.y, w.z, w.w};
  if (FAST || g.mode == 0) {
    // plain stuck-at fast path: one Philox call per pair of weights
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const U32x4 r = draw(seed, (uint64_t)(i >> 1) + h, map_id, g.layer_id, kPurposeFault);
      const bool b0 = static_cast<uint64_t>(r.x) < g.thr_fault;
      const bool b1 = static_cast<uint64_t>(r.z) < g.thr_fault;
      if (b0) o[2 * h] = stuck_value(r.y, g.thr_neg, g.thr_zero) * g.stuck_scale;
      if (b1) o[2 * h + 1] = stuck_value(r.w, g.thr_neg, g.thr_zero) * g.stuck_scale;
      nb += static_cast<unsigned>(b0) + static_cast<unsigned>(b1);
    }
  } else if (g.mode == 1) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint64_t pr = (uint64_t)(i >> 1) + h;
      const U32x4 r = draw(seed, pr, map_id, g.layer_id, kPurposeFault);
      float z0 = 0.f, z1 = 0.f;
      const bool hz = g.sigma > 0.0f;
      if (hz) {
        const U32x4 rz = draw(seed, pr, map_id, g.layer_id, kPurposeVariation);
        float t0, t1;
        box_muller(rz.x, rz.y, z0, t0);
        box_muller(rz.z, rz.w, z1, t1);
      }
      bool b0, b1;
      o[2 * h] = inject_single(o[2 * h], r.x, r.y, hz, z0, g, b0);
      o[2 * h + 1] = inject_single(o[2 * h + 1], r.z, r.w, hz, z1, g, b1);
      nb += static_cast<unsigned>(b0) + static_cast<unsigned>(b1);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = inject_pair(o[j], (uint64_t)i + j, seed, map_id, g, nb);
  }
  return make_float4(o[0], o[1], o[2], o[3]);
}

template <bool FAST>
__device__ __forceinline__ float inject1(float w, int64_t i, uint64_t seed, uint32_t map_id,
                                         const InjectSeg& g, unsigned& nb) {
  if (!FAST && g.mode == 2) return inject_pair(w, (uint64_t)i, seed, map_id, g, nb);
  const uint64_t pr = (uint64_t)(i >> 1);
  const bool odd = (i & 1) != 0;
  const U32x4 r = draw(seed, pr, map_id, g.layer_id, kPurposeFault);
  const uint32_t rf = odd ? r.z : r.x;
  const uint32_t rv = odd ? r.w : r.y;
  bool b;
  float out;
  if (FAST || g.mode == 0) {
    b = static_cast<uint64_t>(rf) < g.thr_fault;
    out = b ? stuck_value(rv, g.thr_neg, g.thr_zero) * g.stuck_scale : w;
  } else {
    float z = 0.f;
    const bool hz = g.sigma > 0.0f;
    if (hz) {
      const U32x4 rz = draw(seed, pr, map_id, g.layer_id, kPurposeVariation);
      float za, zb;
      if (odd) box_muller(rz.z, rz.w, z, zb);
      else box_muller(rz.x, rz.y, z, za);
    }
    out = inject_single(w, rf, rv, hz, z, g, b);
  }
  nb += static_cast<unsigned>(b);
  return out;
}

// FAST: every segment is plain stuck-at (mode 0), so the quantisation /
// variation / pair paths are compiled out and the kernel's register budget is
// that of the Philox + stuck-value path alone (higher occupancy).
// map_dev (nullable): the map id read from device memory (a replayed hipGraph
// advances it on the device, rram_mc_accumulate_dev), else map_arg
template <bool FAST>
__global__ void __launch_bounds__(256)
    k_inject_batched(InjectSegs segs, uint64_t seed, uint32_t map_arg, const uint32_t* __restrict__ map_dev,
                     unsigned long long* counters) {
  const uint32_t map_id = map_dev != nullptr ? *map_dev : map_arg;
  // each block owns a contiguous run of chunks, so it crosses at most a few
  // segment boundaries and flushes its broken-cell count (one atomic per
  // segment visited) about once: ~grid + nsegs atomics per launch
  const int64_t total = segs.chunk_start[segs.nsegs];
  const int64_t per = (total + gridDim.x - 1) / gridDim.x;
  const int64_t cbeg = blockIdx.x * per;
  const int64_t cend = cbeg + per < total ? cbeg + per : total;
  int cur = -1;  // block-uniform: flush the count once per segment visited
  unsigned nb = 0;
  int s = 0;
  for (int64_t c = cbeg; c < cend; ++c) {
    while (c >= segs.chunk_start[s + 1]) ++s;
    if (s != cur) {
      if (cur >= 0) block_count_flush(nb, counters ? counters + cur : nullptr);
      nb = 0;
      cur = s;
    }
    const InjectSeg& g = segs.s[s];
    const int64_t begin = (c - segs.chunk_start[s]) * kInjChunk;
    const int64_t end = min(begin + (int64_t)kInjChunk, g.n);
    // vector path: begin is a multiple of 4 (chunk size), pointers 16-B aligned
    if (aligned16(g.src) && aligned16(g.dst)) {
      const int64_t nv = (end - begin) >> 2;
      const float4* s4 = reinterpret_cast<const float4*>(g.src + begin);
      float4* d4 = reinterpret_cast<float4*>(g.dst + begin);
      // issue all loads of the chunk before the RNG work (4 per lane)
      float4 buf[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t q = threadIdx.x + u * 256;
        if (q < nv) buf[u] = s4[q];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t q = threadIdx.x + u * 256;
        if (q < nv) d4[q] = inject4<FAST>(buf[u], begin + 4 * q, seed, map_id, g, nb);
      }
      for (int64_t i = begin + 4 * nv + threadIdx.x; i < end; i += 256)
        g.dst[i] = inject1<FAST>(g.src[i], i, seed, map_id, g, nb);
    } else {
      for (int64_t i = begin + threadIdx.x; i < end; i += 256)
        g.dst[i] = inject1<FAST>(g.src[i], i, seed, map_id, g, nb);
    }
  }
  if (cur >= 0) block_count_flush(nb, counters ? counters + cur : nullptr);
}

// Monte-Carlo statistics of one map: sums[k] += out_k[0]; per_map[k] = out_k[0].
__global__ void k_mc_accumulate(rram_mc_outputs o, float* __restrict__ sums, float* __restrict__ per_map) {
  const int k = threadIdx.x;
  if (k < o.n) {
    const float v = o.p[k][0];
    sums[k] += v;
    if (per_map) per_map[k] = v;
  }
}
// The same with the per-map row from device memory: row = *row_dev; the row
// is written when row < max_rows; advance != 0: then row_dev += 1 and
// map_dev (nullable) += 1, so a replayed graph of one map walks the maps.
__global__ void k_mc_accumulate_dev(rram_mc_outputs o, float* __restrict__ sums, float* __restrict__ per_map,
                                    int64_t row_stride, int max_rows, int* __restrict__ row_dev,
                                    uint32_t* __restrict__ map_dev, int advance) {
  const int k = threadIdx.x;
  const int row = *row_dev;
  if (k < o.n) {
    const float v = o.p[k][0];
    sums[k] += v;
    if (per_map != nullptr && row < max_rows) per_map[(int64_t)row * row_stride + k] = v;
  }
  __syncthreads();  // every lane has read row before it moves
  if (advance && k == 0) {
    *row_dev = row + 1;
    if (map_dev != nullptr) *map_dev = *map_dev + 1u;
  }
}

// ---------------------------------------------------------------------------
// a3 / a4
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
    k_threshold(float* __restrict__ dw, int64_t n, float thr, unsigned long long* cleared) {
  unsigned cnt = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (fabsf(dw[i]) <= thr) {
      dw[i] = 0.0f;
      ++cnt;
    }
  }
  wave_count_add_n(cnt, cleared);
}

__global__ void __launch_bounds__(256)
    k_sgd_update(float* __restrict__ g, float* __restrict__ h, int64_t n, float mom, float lr) {
  // Caffe's CPU path forms momentum*h and local_rate*g as separate products
  // (caffe_cpu_axpby = scal + axpy, sgd_solver.cpp:222-228); the oracle does the
  // same, so no FMA contraction here or in the fused tail / axpby below.
#pragma clang fp contract(off)
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = mom * h[i] + lr * g[i];
    g[i] = v;
    h[i] = v;
  }
}

__global__ void __launch_bounds__(256)
    k_fused_update_fail(float* __restrict__ w, float* __restrict__ g, float* __restrict__ h,
                        float* __restrict__ e, const float* __restrict__ v, int64_t n, float decay,
                        float mom, float lr, int apply_thr, float thr, float dec, float eps,
                        unsigned long long* counter) {
#pragma clang fp contract(off)
  unsigned cnt = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float wi = w[i];
    float gi = g[i];
    if (decay != 0.0f) gi = decay * wi + gi;            // caffe_gpu_axpy(decay, w, g)
    gi = mom * h[i] + lr * gi;                          // SGDUpdate
    h[i] = gi;
    if (apply_thr && fabsf(gi) <= thr) gi = 0.0f;       // threshold strategy
    g[i] = gi;
    wi = wi - gi;                                       // Blob::Update (axpy -1)
    if (e != nullptr) {
      float ee = e[i];
      bool wr;
      float wv;
      cnt += fail_one(gi, wv, ee, v[i], dec, eps, wr);
      e[i] = ee;
      if (wr) wi = wv;
    }
    w[i] = wi;
  }
  wave_count_add_n(cnt, counter);
}

// k_fused_update_fail over all of a net's learnable blobs: block-chunks of
// kUpdChunk elements dealt across the segments (as k_fail_apply_batched), the
// per-element arithmetic k_fused_update_fail's
struct UpdateSegs {
  rram_update_seg s[RRAM_MAX_SEGS];
  int64_t chunk_start[RRAM_MAX_SEGS + 1];
  int nsegs;
};
constexpr int kUpdChunk = 256 * 8;

__global__ void __launch_bounds__(256)
    k_fused_update_fail_batched(UpdateSegs segs, float mom, float dec, float eps) {
#pragma clang fp contract(off)
  const int64_t total = segs.chunk_start[segs.nsegs];
  int cur = -1;  // block-uniform: flush the count once per segment visited
  unsigned cnt = 0;
  for (int64_t c = blockIdx.x; c < total; c += gridDim.x) {
    int s = 0;
    while (c >= segs.chunk_start[s + 1]) ++s;
    if (s != cur) {
      if (cur >= 0) block_count_flush(cnt, segs.s[cur].broken_count);
      cnt = 0;
      cur = s;
    }
    const rram_update_seg& sg = segs.s[s];
    const int64_t begin = (c - segs.chunk_start[s]) * kUpdChunk;
    const int64_t end = min(begin + (int64_t)kUpdChunk, sg.n);
    float* __restrict__ w = sg.w;
    float* __restrict__ g = sg.g;
    float* __restrict__ h = sg.h;
    float* __restrict__ e = sg.endurance;
    const float* __restrict__ v = sg.values;
    for (int64_t i = begin + threadIdx.x; i < end; i += blockDim.x) {
      float wi = w[i];
      float gi = g[i];
      if (sg.decay != 0.0f) gi = sg.decay * wi + gi;
      gi = mom * h[i] + sg.local_rate * gi;
      h[i] = gi;
      if (sg.apply_thr && fabsf(gi) <= sg.thr) gi = 0.0f;
      g[i] = gi;
      wi = wi - gi;
      if (e != nullptr) {
        float ee = e[i];
        bool wr;
        float wv;
        cnt += fail_one(gi, wv, ee, v[i], dec, eps, wr);
        e[i] = ee;
        if (wr) wi = wv;
      }
      w[i] = wi;
      if (sg.w_flip != nullptr) {  // (the host checked G cin cout taps == n < 2^31)
        const int T = sg.flip_taps, ci = sg.flip_cin, co = sg.flip_cout;
        int t = static_cast<int>(i);
        const int tap = t % T;
        t /= T;
        const int c = t % ci;
        t /= ci;
        const int o = t % co;
        const int gr = t / co;
        sg.w_flip[((gr * ci + c) * co + o) * T + (T - 1 - tap)] = wi;
      }
    }
  }
  if (cur >= 0) block_count_flush(cnt, segs.s[cur].broken_count);
}

// ---------------------------------------------------------------------------
// level-1 helpers
// ---------------------------------------------------------------------------
__global__ void k_axpby(int64_t n, float a, const float* __restrict__ x, float b,
                        float* __restrict__ y, int mode) {
#pragma clang fp contract(off)
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (mode == 0) y[i] = a * x[i] + y[i];       // axpy
    else y[i] = a * x[i] + b * y[i];             // axpby
  }
}
__global__ void k_scal(int64_t n, float a, float* __restrict__ x) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    x[i] = a * x[i];
}
// the solver's per-iteration clears in one launch: a[0..na) (the flat
// parameter diff) and b[0..nb) (the Fail counters)
__global__ void __launch_bounds__(256) k_zero_pair(float* __restrict__ a, int64_t na, unsigned long long* __restrict__ b,
                                                   int64_t nb) {
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = t0; i < na; i += st) a[i] = 0.0f;
  for (int64_t i = t0; i < nb; i += st) b[i] = 0ull;
}

__global__ void k_set(int64_t n, float a, float* __restrict__ x) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    x[i] = a;
}
__global__ void k_add(int64_t n, const float* __restrict__ a, const float* __restrict__ b,
                      float* __restrict__ y) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = a[i] + b[i];
}
__global__ void k_sign(int64_t n, const float* __restrict__ x, float* __restrict__ y) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = (0.0f < x[i]) - (x[i] < 0.0f);
}

// op: 0 sum|x|, 1 max|x|, 2 sum x*y.  Single block, deterministic.
__global__ void __launch_bounds__(1024) k_reduce1(int64_t n, const float* __restrict__ x,
                                                  const float* __restrict__ y, float* out, int op) {
  __shared__ float part[16];
  float acc = 0.0f;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const float v = x[i];
    if (op == 0) acc += fabsf(v);
    else if (op == 1) acc = fmaxf(acc, fabsf(v));
    else acc += v * y[i];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float o = __shfl_xor(acc, off, 64);
    acc = (op == 1) ? fmaxf(acc, o) : acc + o;
  }
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = 0.0f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r = (op == 1) ? fmaxf(r, part[i]) : r + part[i];
    out[0] = r;
  }
}

// ---------------------------------------------------------------------------
// fillers
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_fill(float* __restrict__ x, int64_t n, float a, float b,
                                              int kind, uint64_t seed, uint32_t sid) {
  // kind 0: uniform [a, b); 1: gaussian(mean a, std b); 2: floor(U*levels(a)) + b
  const int64_t nq = (n + 3) / 4;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < nq;
       q += (int64_t)gridDim.x * blockDim.x) {
    const U32x4 r = draw(seed, (uint64_t)q, sid, 0u, kPurposeFill);
    float o[4];
    if (kind == 0) {
      o[0] = a + (b - a) * u01(r.x);
      o[1] = a + (b - a) * u01(r.y);
      o[2] = a + (b - a) * u01(r.z);
      o[3] = a + (b - a) * u01(r.w);
    } else if (kind == 1) {
      float z0, z1, z2, z3;
      box_muller(r.x, r.y, z0, z1);
      box_muller(r.z, r.w, z2, z3);
      o[0] = fmaf(b, z0, a);
      o[1] = fmaf(b, z1, a);
      o[2] = fmaf(b, z2, a);
      o[3] = fmaf(b, z3, a);
    } else {
      const uint32_t lv = static_cast<uint32_t>(a);
      o[0] = static_cast<float>(__umulhi(r.x, lv)) + b;
      o[1] = static_cast<float>(__umulhi(r.y, lv)) + b;
      o[2] = static_cast<float>(__umulhi(r.z, lv)) + b;
      o[3] = static_cast<float>(__umulhi(r.w, lv)) + b;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (4 * q + j < n) x[4 * q + j] = o[j];
  }
}

__global__ void __launch_bounds__(256)
    k_dropout_fwd(const float* __restrict__ x, float* __restrict__ y, unsigned int* __restrict__ mask,
                  int64_t n, uint32_t thr, float scale, uint64_t seed, uint32_t layer, uint64_t iter) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const U32x4 r = draw(seed ^ (iter * 0x9E3779B97F4A7C15ull), (uint64_t)i, 0u, layer, kPurposeDropout);
    const unsigned keep = r.x > thr;
    mask[i] = keep;
    y[i] = keep ? x[i] * scale : 0.0f;
  }
}
__global__ void __launch_bounds__(256)
    k_dropout_bwd(const float* __restrict__ dy, const unsigned int* __restrict__ mask,
                  float* __restrict__ dx, int64_t n, float scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dx[i] = mask[i] ? dy[i] * scale : 0.0f;
}

}  // namespace

// host-side helpers -------------------------------------------------------
static thread_local std::string g_err;
void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}
void clear_error() { g_err.clear(); }
const char* last_error_cstr() { return g_err.c_str(); }

int launch_status(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s launch: %s", what, hipGetErrorString(e));
    return RRAM_EHIP;
  }
  return RRAM_OK;
}

static InjectSeg make_inject_seg(const float* src, float* dst, int64_t n, uint32_t layer_id,
                                 const rram_inject_cfg& c) {
  InjectSeg g{};
  g.src = src;
  g.dst = dst;
  g.n = n;
  g.layer_id = layer_id;
  g.thr_fault = c.thr_fault;
  g.thr_neg = c.thr_neg;
  g.thr_zero = c.thr_zero;
  g.thr_sa1 = c.thr_sa1;
  g.stuck_scale = c.stuck_scale;
  g.g_max = c.g_max;
  g.levels = c.quant_levels >= 2 ? c.quant_levels : 0;
  g.sigma = c.var_sigma;
  g.q_delta = 0.f;
  g.q_inv = 0.f;
  if (c.cell_mode == RRAM_CELL_DIFFPAIR) {
    g.mode = 2;
    if (g.levels) {
      g.q_delta = c.g_max / static_cast<float>(g.levels - 1);
      g.q_inv = 1.0f / g.q_delta;
    }
  } else {
    g.mode = (g.levels == 0 && !(c.var_sigma > 0.f)) ? 0 : 1;
    if (g.levels) {
      g.q_delta = (2.0f * c.g_max) / static_cast<float>(g.levels - 1);
      g.q_inv = 1.0f / g.q_delta;
    }
  }
  return g;
}

static int check_cfg(const rram_inject_cfg* c) {
  RRAM_REQUIRE(c != nullptr, "inject: cfg is NULL");
  RRAM_REQUIRE(c->thr_fault <= (1ull << 32) && c->thr_neg <= (1ull << 32) &&
                   c->thr_zero <= (1ull << 32) && c->thr_sa1 <= (1ull << 32),
               "inject: thresholds must be in [0, 2^32]");
  RRAM_REQUIRE(c->thr_neg <= c->thr_zero, "inject: thr_neg must be <= thr_zero");
  RRAM_REQUIRE(c->cell_mode == RRAM_CELL_SINGLE || c->cell_mode == RRAM_CELL_DIFFPAIR,
               "inject: unknown cell_mode %d", c->cell_mode);
  RRAM_REQUIRE(!(c->quant_levels >= 2) || c->g_max > 0.f, "inject: quantisation needs g_max > 0");
  RRAM_REQUIRE(c->cell_mode != RRAM_CELL_DIFFPAIR || c->g_max > 0.f, "inject: diff-pair needs g_max > 0");
  RRAM_REQUIRE(c->var_sigma >= 0.f, "inject: var_sigma must be >= 0");
  return RRAM_OK;
}

}  // namespace rram

using namespace rram;

extern "C" {

const char* rram_kernels_version(void) { return "rram_kernels 0.1 gfx950"; }
const char* rram_last_error(void) { return rram::last_error_cstr(); }
int rram_device_synchronize(void) {
  RRAM_HIP_RET(hipDeviceSynchronize());
  return RRAM_OK;
}

int rram_fault_threshold(float* values, int64_t n, float split1, float split2, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "fault_threshold: n < 0");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(values, "fault_threshold: values is NULL");
  hipLaunchKernelGGL(k_fault_threshold, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s),
                     values, n, split1, split2);
  return launch_status("fault_threshold");
}

int rram_fault_init(float* endurance, float* values, int64_t n, float mean, float std,
                    uint64_t thr_neg, uint64_t thr_zero, uint64_t seed, uint32_t map_id,
                    uint32_t layer_id, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "fault_init: n < 0");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(endurance && values, "fault_init: NULL pointer");
  RRAM_REQUIRE(thr_neg <= thr_zero && thr_zero <= (1ull << 32), "fault_init: bad thresholds");
  hipLaunchKernelGGL(k_fault_init, dim3(stream_blocks((n + 1) / 2)), dim3(kThreads), 0,
                     as_stream(s), endurance, values, n, mean, std, thr_neg, thr_zero, seed,
                     map_id, layer_id);
  return launch_status("fault_init");
}

int rram_fail_apply_batched(const rram_fail_seg* segs, int nsegs, float dec, float eps,
                            unsigned long long* counters, rram_stream_t s) {
  RRAM_REQUIRE(nsegs >= 0 && nsegs <= RRAM_MAX_SEGS, "fail_apply: nsegs out of range");
  if (nsegs == 0) return RRAM_OK;
  RRAM_REQUIRE(segs, "fail_apply: segs is NULL");
  FailSegs fs{};
  fs.nsegs = nsegs;
  fs.chunk_start[0] = 0;
  for (int i = 0; i < nsegs; ++i) {
    RRAM_REQUIRE(segs[i].n >= 0, "fail_apply: segment %d n < 0", i);
    if (segs[i].n > 0)
      RRAM_REQUIRE(segs[i].dw && segs[i].w && segs[i].endurance && segs[i].values,
                   "fail_apply: segment %d has a NULL pointer", i);
    fs.s[i] = segs[i];
    fs.chunk_start[i + 1] = fs.chunk_start[i] + (segs[i].n + kFailChunk - 1) / kFailChunk;
  }
  const int64_t total = fs.chunk_start[nsegs];
  if (total == 0) return RRAM_OK;
  const int grid = static_cast<int>(total < kMaxStreamBlocks ? total : kMaxStreamBlocks);
  hipLaunchKernelGGL(k_fail_apply_batched, dim3(grid), dim3(kThreads), 0, as_stream(s), fs, dec,
                     eps, counters);
  return launch_status("fail_apply");
}

int rram_fail_apply(const float* dw, float* w, float* e, const float* v, int64_t n, float dec,
                    float eps, unsigned long long* counter, rram_stream_t s) {
  rram_fail_seg sg{dw, w, e, v, n};
  return rram_fail_apply_batched(&sg, 1, dec, eps, counter, s);
}

int rram_broken_count(const float* e, int64_t n, unsigned long long* counter, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0 && counter, "broken_count: bad args");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(e, "broken_count: endurance is NULL");
  hipLaunchKernelGGL(k_broken_count, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), e, n,
                     counter);
  return launch_status("broken_count");
}

int rram_set_inject_grid(int blocks) {
  RRAM_REQUIRE(blocks >= 0, "set_inject_grid: negative grid");
  return rram::inject_grid().exchange(blocks);
}

namespace rram {
namespace {
int inject_batched_core(const rram_inject_seg* segs, int nsegs, uint64_t seed, uint32_t map_id,
                        const uint32_t* map_dev, unsigned long long* counters, rram_stream_t s);
}
}  // namespace rram

int rram_inject_rng_batched(const rram_inject_seg* segs, int nsegs, uint64_t seed,
                            uint32_t map_id, unsigned long long* counters, rram_stream_t s) {
  return rram::inject_batched_core(segs, nsegs, seed, map_id, nullptr, counters, s);
}

int rram_inject_rng_batched_dev(const rram_inject_seg* segs, int nsegs, uint64_t seed, const uint32_t* map_id_dev,
                                unsigned long long* counters, rram_stream_t s) {
  RRAM_REQUIRE(map_id_dev != nullptr, "inject_dev: map_id_dev is NULL");
  return rram::inject_batched_core(segs, nsegs, seed, 0, map_id_dev, counters, s);
}
}  // extern "C"

namespace rram {
namespace {
int inject_batched_core(const rram_inject_seg* segs, int nsegs, uint64_t seed, uint32_t map_id,
                        const uint32_t* map_dev, unsigned long long* counters, rram_stream_t s) {
  RRAM_REQUIRE(nsegs >= 0 && nsegs <= RRAM_MAX_SEGS, "inject: nsegs out of range");
  if (nsegs == 0) return RRAM_OK;
  RRAM_REQUIRE(segs, "inject: segs is NULL");
  InjectSegs is{};
  is.nsegs = nsegs;
  for (int i = 0; i < nsegs; ++i) {
    const int rc = check_cfg(&segs[i].cfg);
    if (rc) return rc;
    RRAM_REQUIRE(segs[i].n >= 0, "inject: segment %d n < 0", i);
    if (segs[i].n > 0) RRAM_REQUIRE(segs[i].w_clean && segs[i].w_out, "inject: segment %d NULL", i);
    RRAM_REQUIRE(segs[i].layer_id < (1u << 28), "inject: layer_id must be < 2^28");
    is.s[i] = make_inject_seg(segs[i].w_clean, segs[i].w_out, segs[i].n, segs[i].layer_id,
                              segs[i].cfg);
    is.chunk_start[i + 1] = is.chunk_start[i] + (segs[i].n + kInjChunk - 1) / kInjChunk;
  }
  const int64_t total = is.chunk_start[nsegs];
  if (total == 0) return RRAM_OK;
  // persistent grid of kInjectGrid blocks over the 4096-weight chunks.  One
  // block per chunk (14,315 for AlexNet) measured 2x slower in the MC loop
  // (190 vs 100 us): every block ends in a same-address counter atomic, and
  // the serialised atomics, not HBM, set the pace.
  const int64_t grid_cap = inject_grid().load(std::memory_order_relaxed) > 0
                               ? static_cast<int64_t>(inject_grid().load(std::memory_order_relaxed))
                               : static_cast<int64_t>(kInjectGrid);
  const int grid = static_cast<int>(total < grid_cap ? total : grid_cap);
  bool fast = true;
  for (int i = 0; i < nsegs; ++i) fast = fast && is.s[i].mode == 0;
  if (fast)
    hipLaunchKernelGGL(k_inject_batched<true>, dim3(grid), dim3(kThreads), 0, as_stream(s), is, seed,
                       map_id, map_dev, counters);
  else
    hipLaunchKernelGGL(k_inject_batched<false>, dim3(grid), dim3(kThreads), 0, as_stream(s), is, seed,
                       map_id, map_dev, counters);
  return launch_status("inject_rng");
}
}  // namespace
}  // namespace rram

extern "C" {

int rram_inject_rng(const float* w_clean, float* w_out, int64_t n, const rram_inject_cfg* cfg,
                    uint64_t seed, uint32_t map_id, uint32_t layer_id,
                    unsigned long long* counters, rram_stream_t s) {
  RRAM_REQUIRE(cfg != nullptr, "inject: cfg is NULL");
  rram_inject_seg sg{};
  sg.w_clean = w_clean;
  sg.w_out = w_out;
  sg.n = n;
  sg.layer_id = layer_id;
  sg.cfg = *cfg;
  return rram_inject_rng_batched(&sg, 1, seed, map_id, counters, s);
}

int rram_mc_accumulate(const rram_mc_outputs* outs, float* sums, float* per_map_row, rram_stream_t s) {
  RRAM_REQUIRE(outs && sums && outs->n >= 0 && outs->n <= RRAM_MC_MAX_OUTPUTS, "mc_accumulate: bad arguments");
  if (outs->n == 0) return RRAM_OK;
  hipLaunchKernelGGL(k_mc_accumulate, dim3(1), dim3(64), 0, as_stream(s), *outs, sums, per_map_row);
  return launch_status("mc_accumulate");
}

int rram_mc_accumulate_dev(const rram_mc_outputs* outs, float* sums, float* per_map, int64_t row_stride,
                           int max_rows, int* row_dev, uint32_t* map_id_dev, int advance, rram_stream_t s) {
  RRAM_REQUIRE(outs && sums && row_dev && outs->n >= 0 && outs->n <= RRAM_MC_MAX_OUTPUTS && max_rows >= 0 &&
                   row_stride >= outs->n,
               "mc_accumulate_dev: bad arguments");
  hipLaunchKernelGGL(k_mc_accumulate_dev, dim3(1), dim3(64), 0, as_stream(s), *outs, sums, per_map, row_stride,
                     max_rows, row_dev, map_id_dev, advance);
  return launch_status("mc_accumulate_dev");
}

int rram_threshold_strategy(float* dw, int64_t n, float thr, unsigned long long* cleared,
                            rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "threshold: n < 0");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(dw, "threshold: dw is NULL");
  hipLaunchKernelGGL(k_threshold, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), dw, n,
                     thr, cleared);
  return launch_status("threshold");
}

int rram_sgd_update(float* g, float* h, int64_t n, float mom, float lr, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "sgd_update: n < 0");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(g && h, "sgd_update: NULL pointer");
  hipLaunchKernelGGL(k_sgd_update, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), g, h,
                     n, mom, lr);
  return launch_status("sgd_update");
}

int rram_fused_update_fail(float* w, float* g, float* h, float* e, const float* v, int64_t n,
                           float decay, float mom, float lr, int apply_thr, float thr, float dec,
                           float eps, unsigned long long* counter, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "fused_update_fail: n < 0");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(w && g && h, "fused_update_fail: NULL pointer");
  RRAM_REQUIRE((e == nullptr) == (v == nullptr), "fused_update_fail: endurance/values mismatch");
  hipLaunchKernelGGL(k_fused_update_fail, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s),
                     w, g, h, e, v, n, decay, mom, lr, apply_thr, thr, dec, eps, counter);
  return launch_status("fused_update_fail");
}

int rram_fused_update_fail_batched(const rram_update_seg* segs, int nsegs, float mom, float dec, float eps,
                                   rram_stream_t s) {
  using namespace rram;
  RRAM_REQUIRE(nsegs >= 0 && nsegs <= RRAM_MAX_SEGS, "fused_update_fail_batched: nsegs out of range");
  if (nsegs == 0) return RRAM_OK;
  RRAM_REQUIRE(segs, "fused_update_fail_batched: segs is NULL");
  UpdateSegs us{};
  us.nsegs = nsegs;
  for (int i = 0; i < nsegs; ++i) {
    const rram_update_seg& sg = segs[i];
    RRAM_REQUIRE(sg.n >= 0, "fused_update_fail_batched: segment %d n < 0", i);
    if (sg.n > 0) RRAM_REQUIRE(sg.w && sg.g && sg.h, "fused_update_fail_batched: segment %d NULL pointer", i);
    RRAM_REQUIRE((sg.endurance == nullptr) == (sg.values == nullptr),
                 "fused_update_fail_batched: segment %d endurance/values mismatch", i);
    if (sg.w_flip != nullptr)
      RRAM_REQUIRE(sg.flip_groups > 0 && sg.flip_cin > 0 && sg.flip_cout > 0 && sg.flip_taps > 0 &&
                       (int64_t)sg.flip_groups * sg.flip_cin * sg.flip_cout * sg.flip_taps == sg.n && sg.n < (1ll << 31),
                   "fused_update_fail_batched: segment %d flip geometry %d x %d x %d x %d != n %lld", i, sg.flip_groups,
                   sg.flip_cin, sg.flip_cout, sg.flip_taps, (long long)sg.n);
    us.s[i] = sg;
    us.chunk_start[i + 1] = us.chunk_start[i] + (sg.n + kUpdChunk - 1) / kUpdChunk;
  }
  const int64_t total = us.chunk_start[nsegs];
  if (total == 0) return RRAM_OK;
  const int grid = static_cast<int>(total < 2048 ? total : 2048);
  hipLaunchKernelGGL(k_fused_update_fail_batched, dim3(grid), dim3(kThreads), 0, as_stream(s), us, mom, dec, eps);
  return launch_status("fused_update_fail_batched");
}

int rram_axpy(int64_t n, float a, const float* x, float* y, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "axpy: n < 0");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(x && y, "axpy: NULL");
  hipLaunchKernelGGL(k_axpby, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), n, a, x,
                     1.0f, y, 0);
  return launch_status("axpy");
}
int rram_axpby(int64_t n, float a, const float* x, float b, float* y, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "axpby: n < 0");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(x && y, "axpby: NULL");
  hipLaunchKernelGGL(k_axpby, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), n, a, x, b,
                     y, 1);
  return launch_status("axpby");
}
int rram_scal(int64_t n, float a, float* x, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "scal: n < 0");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(x, "scal: NULL");
  hipLaunchKernelGGL(k_scal, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), n, a, x);
  return launch_status("scal");
}
int rram_set(int64_t n, float a, float* x, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "set: n < 0");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(x, "set: NULL");
  hipLaunchKernelGGL(k_set, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), n, a, x);
  return launch_status("set");
}
int rram_zero_pair(float* a, int64_t na, unsigned long long* b, int64_t nb, rram_stream_t s) {
  RRAM_REQUIRE(na >= 0 && nb >= 0, "zero_pair: negative count");
  RRAM_REQUIRE((na == 0 || a) && (nb == 0 || b), "zero_pair: NULL");
  const int64_t n = na > nb ? na : nb;
  if (n == 0) return RRAM_OK;
  hipLaunchKernelGGL(k_zero_pair, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), a, na, b, nb);
  return launch_status("zero_pair");
}
int rram_add(int64_t n, const float* a, const float* b, float* y, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "add: n < 0");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(a && b && y, "add: NULL");
  hipLaunchKernelGGL(k_add, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), n, a, b, y);
  return launch_status("add");
}
int rram_sign(int64_t n, const float* x, float* y, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "sign: n < 0");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(x && y, "sign: NULL");
  hipLaunchKernelGGL(k_sign, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), n, x, y);
  return launch_status("sign");
}
static int reduce1(int64_t n, const float* x, const float* y, float* out, int op, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0 && out, "reduce: bad args");
  if (n > 0) RRAM_REQUIRE(x && (op != 2 || y), "reduce: NULL input");
  hipLaunchKernelGGL(k_reduce1, dim3(1), dim3(1024), 0, as_stream(s), n, x, y, out, op);
  return launch_status("reduce");
}
int rram_asum(int64_t n, const float* x, float* out, rram_stream_t s) { return reduce1(n, x, nullptr, out, 0, s); }
int rram_absmax(int64_t n, const float* x, float* out, rram_stream_t s) { return reduce1(n, x, nullptr, out, 1, s); }
int rram_dot(int64_t n, const float* x, const float* y, float* out, rram_stream_t s) { return reduce1(n, x, y, out, 2, s); }

static int fill(float* x, int64_t n, float a, float b, int kind, uint64_t seed, uint32_t sid,
                rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "fill: n < 0");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(x, "fill: NULL");
  hipLaunchKernelGGL(k_fill, dim3(stream_blocks((n + 3) / 4)), dim3(kThreads), 0, as_stream(s), x,
                     n, a, b, kind, seed, sid);
  return launch_status("fill");
}
int rram_fill_uniform(float* x, int64_t n, float lo, float hi, uint64_t seed, uint32_t sid, rram_stream_t s) {
  return fill(x, n, lo, hi, 0, seed, sid, s);
}
int rram_fill_gaussian(float* x, int64_t n, float mean, float std, uint64_t seed, uint32_t sid, rram_stream_t s) {
  return fill(x, n, mean, std, 1, seed, sid, s);
}
int rram_fill_uniform_int(float* x, int64_t n, int levels, float offset, uint64_t seed, uint32_t sid,
                          rram_stream_t s) {
  RRAM_REQUIRE(levels >= 1, "fill_uniform_int: levels < 1");
  return fill(x, n, static_cast<float>(levels), offset, 2, seed, sid, s);
}

int rram_dropout_fwd(const float* x, float* y, unsigned int* mask, int64_t n, float ratio,
                     uint64_t seed, uint32_t layer_id, uint64_t iter, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0 && ratio >= 0.f && ratio < 1.f, "dropout: bad args");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(x && y && mask, "dropout: NULL");
  const uint32_t thr = static_cast<uint32_t>(static_cast<double>(ratio) * 4294967296.0 >= 4294967295.0
                                                 ? 4294967295u
                                                 : static_cast<double>(ratio) * 4294967296.0);
  hipLaunchKernelGGL(k_dropout_fwd, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), x, y,
                     mask, n, thr, 1.0f / (1.0f - ratio), seed, layer_id, iter);
  return launch_status("dropout_fwd");
}
int rram_dropout_bwd(const float* dy, const unsigned int* mask, float* dx, int64_t n, float ratio,
                     rram_stream_t s) {
  RRAM_REQUIRE(n >= 0 && ratio >= 0.f && ratio < 1.f, "dropout: bad args");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(dy && mask && dx, "dropout: NULL");
  hipLaunchKernelGGL(k_dropout_bwd, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), dy,
                     mask, dx, n, 1.0f / (1.0f - ratio));
  return launch_status("dropout_bwd");
}

}  // extern "C"
