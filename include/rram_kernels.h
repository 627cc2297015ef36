/*
 * rram_kernels.h — C-ABI of the MI355X (gfx950) RRAM fault-simulation kernels.
 *
 * This is the drop-in device boundary below Caffe's Layer<Dtype>/Solver API
 * (SURVEY.md §8b).  Every entry point:
 *   - takes plain pointers (device memory unless stated), sizes and an opaque
 *     stream handle (`rram_stream_t` == hipStream_t; NULL = default stream);
 *   - returns an int status (RRAM_OK == 0) and never aborts; the message of
 *     the last failure on the calling thread is in rram_last_error();
 *   - is asynchronous on the given stream and allocates nothing (graph-capture
 *     safe) unless the comment says otherwise.
 * Each declaration cites the reference interface it replaces
 * (paths relative to the reference repository fightingnoble/rram-caffe-simulation).
 */
#ifndef RRAM_KERNELS_H_
#define RRAM_KERNELS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* rram_stream_t; /* hipStream_t */

enum {
  RRAM_OK = 0,
  RRAM_EINVAL = -1,      /* bad argument (null pointer, negative size, ...) */
  RRAM_EHIP = -2,        /* HIP runtime error (launch / memcpy)             */
  RRAM_ENOMEM = -3,      /* workspace too small / allocation failed          */
  RRAM_EUNSUPPORTED = -4 /* shape or mode not supported by this build       */
};

const char* rram_kernels_version(void);
const char* rram_last_error(void);
/* hipDeviceSynchronize + error check (host-side convenience). */
int rram_device_synchronize(void);
/* Frees the per-geometry convolution gather tables the conv kernels cache per
 * HIP device (lazily built on first use).  Synchronises every device that
 * holds one; call only when no kernel of this library is in flight. */
int rram_release_caches(void);
/* Generation of this library's internal device scratch (the per-stream packed
 * operand and split-K partial buffers, the convolution gather tables): bumped
 * whenever one of them is freed or reallocated.  A caller that captured
 * launches into a hipGraph (which holds raw pointers into that scratch)
 * re-captures when it changes. */
uint64_t rram_scratch_generation(void);

/* ------------------------------------------------------------------------
 * Fault model
 * ---------------------------------------------------------------------- */

/* Map uniforms in [0,1) to stuck values {-1,0,+1} in place:
 *   u < split1 -> -1 ; u < split2 -> 0 ; else +1.
 * Replaces FailureThresholdKernel / failure_threshold<Dtype>
 * (src/caffe/failure_maker.cu:5-21). */
int rram_fault_threshold(float* values, int64_t n, float split1, float split2,
                         rram_stream_t stream);

/* Draw a fresh fault state for one faultable blob with the build's
 * counter-based RNG (Philox4x32-10, key = seed, counter = (pair index,
 * map_id, layer_id, purpose)):
 *   endurance[j] = mean + std * z_j            (fp32, z ~ N(0,1), Box-Muller)
 *   values[j]    = -1 / 0 / +1 by the integer thresholds thr_neg, thr_zero
 *                  applied to a 32-bit uniform word r (r < thr_neg -> -1,
 *                  r < thr_zero -> 0, else +1; thresholds in [0, 2^32]).
 * Replaces the GaussianFailureMaker constructor's draws
 * (src/caffe/failure_maker.cpp:5-52: caffe_rng_gaussian + caffe_gpu_rng_uniform
 * + failure_threshold). */
int rram_fault_init(float* endurance, float* values, int64_t n, float mean,
                    float std, uint64_t thr_neg, uint64_t thr_zero,
                    uint64_t seed, uint32_t map_id, uint32_t layer_id,
                    rram_stream_t stream);

/* One Fail() step on one blob, reference FailKernel semantics, bit-exact:
 *   if e <= 0: w = v
 *   else if !(|dw| < eps): e -= decrement (fp32); if e <= 0: w = v
 * (reference constants: decrement = 100, eps = 1e-20).
 * broken_count (device, nullable): += number of cells with e <= 0 after the
 * step (replaces the host D2H count loop of failure_maker.hpp:37-55).
 * Replaces FailKernel / Fail_gpu / Fail_cpu (src/caffe/failure_maker.cu:23-58,
 * src/caffe/failure_maker.cpp:55-81). */
int rram_fail_apply(const float* dw, float* w, float* endurance,
                    const float* values, int64_t n, float decrement, float eps,
                    unsigned long long* broken_count, rram_stream_t stream);

/* Several blobs in one launch (one segment per failure_learnable_params()[i]). */
typedef struct {
  const float* dw;
  float* w;
  float* endurance;
  const float* values;
  int64_t n;
} rram_fail_seg;
#define RRAM_MAX_SEGS 32
int rram_fail_apply_batched(const rram_fail_seg* segs, int nsegs,
                            float decrement, float eps,
                            unsigned long long* broken_counts /* [nsegs] */,
                            rram_stream_t stream);

/* broken_count (device) += #{j : endurance[j] <= 0}. */
int rram_broken_count(const float* endurance, int64_t n,
                      unsigned long long* broken_count, rram_stream_t stream);

/* ------------------------------------------------------------------------
 * Monte-Carlo fault-map injection (north_star kernel (1)).
 * The reference expresses one fault map per process run as
 * "endurance <= 0 at the first Fail()" (SURVEY.md §3.3); a map here is
 * the same Bernoulli(p_fault) stuck-at draw made on the fly from
 * (seed, map_id, layer_id, index), so w_out = inject(w_clean) reads 4 B and
 * writes 4 B per weight.
 * ---------------------------------------------------------------------- */
enum {
  RRAM_CELL_SINGLE = 0, /* one cell per weight; stuck value is a literal weight (reference) */
  RRAM_CELL_DIFFPAIR = 1 /* w = G+ - G-, two cells per weight (extension)            */
};

typedef struct {
  /* fault draw: broken iff r0 < thr_fault (thr in [0, 2^32]; p * 2^32 rounded up) */
  uint64_t thr_fault;
  /* single-cell stuck value from r1: -1 iff r1 < thr_neg, 0 iff r1 < thr_zero, else +1 */
  uint64_t thr_neg;
  uint64_t thr_zero;
  /* differential pair: a broken cell sticks at G_max iff r1 < thr_sa1, else at 0 */
  uint64_t thr_sa1;
  float stuck_scale;    /* single cell: stuck weight = value * stuck_scale (1 = reference) */
  float g_max;          /* conductance / weight range used by quantisation and diff-pair   */
  int32_t quant_levels; /* 0/1 = off; L >= 2 uniform levels (extension)                      */
  float var_sigma;      /* lognormal device variation sigma, 0 = off (extension)             */
  int32_t cell_mode;    /* RRAM_CELL_SINGLE / RRAM_CELL_DIFFPAIR                              */
  int32_t reserved;
} rram_inject_cfg;

/* w_out[j] = inject(w_clean[j]); counters (device, nullable) += #broken cells. */
int rram_inject_rng(const float* w_clean, float* w_out, int64_t n,
                    const rram_inject_cfg* cfg, uint64_t seed, uint32_t map_id,
                    uint32_t layer_id, unsigned long long* counters,
                    rram_stream_t stream);

typedef struct {
  const float* w_clean;
  float* w_out;
  int64_t n;
  uint32_t layer_id;
  uint32_t reserved;
  rram_inject_cfg cfg;
} rram_inject_seg;
/* All faultable blobs of a net in one launch; counters[i] for segment i. */
/* Grid (blocks) of the injection launches: 0 = the default persistent grid
 * (2048); returns the previous setting.  A smaller grid suits an injection
 * that runs beside other kernels (MonteCarlo overlaps it with the layers
 * before the first faultable one). */
int rram_set_inject_grid(int blocks);
int rram_inject_rng_batched(const rram_inject_seg* segs, int nsegs,
                            uint64_t seed, uint32_t map_id,
                            unsigned long long* counters, rram_stream_t stream);
/* The same with the map id read from device memory at run time (a captured
 * hipGraph of one Monte-Carlo map replays over consecutive maps; see
 * rram_mc_accumulate_dev).  Bit-identical to rram_inject_rng_batched with
 * map_id = *map_id_dev. */
int rram_inject_rng_batched_dev(const rram_inject_seg* segs, int nsegs, uint64_t seed,
                                const uint32_t* map_id_dev, unsigned long long* counters,
                                rram_stream_t stream);

/* Monte-Carlo statistics of one map in one launch (the MC analogue of
 * Solver::Test's score accumulation, src/caffe/solver.cpp:410-430):
 * sums[k] += p[k][0] and per_map_row[k] = p[k][0] (per_map_row nullable). */
#define RRAM_MC_MAX_OUTPUTS 8
typedef struct {
  const float* p[RRAM_MC_MAX_OUTPUTS]; /* device scalars (the net's 1-element outputs) */
  int n;
} rram_mc_outputs;
int rram_mc_accumulate(const rram_mc_outputs* outs, float* sums, float* per_map_row, rram_stream_t stream);
/* rram_mc_accumulate with the per-map row from device memory: row = *row_dev,
 * per_map[row * row_stride + k] = p[k][0] when row < max_rows (per_map
 * nullable); advance != 0 then increments *row_dev and *map_id_dev (nullable)
 * on the device, after every lane read them. */
int rram_mc_accumulate_dev(const rram_mc_outputs* outs, float* sums, float* per_map, int64_t row_stride,
                           int max_rows, int* row_dev, uint32_t* map_id_dev, int advance, rram_stream_t stream);

/* ------------------------------------------------------------------------
 * Strategy / solver elementwise
 * ---------------------------------------------------------------------- */

/* dw[j] = 0 where |dw[j]| <= thr.  Replaces ThresholdFailureStrategy::Apply's
 * inner loop (src/caffe/strategy.cpp:7-33); thr = threshold * lr * lr_mult.
 * cleared (device, nullable) += #cleared. */
int rram_threshold_strategy(float* dw, int64_t n, float thr,
                            unsigned long long* cleared, rram_stream_t stream);

/* Remapping statistics (RemappingFailureStrategy::GetFailFlagMat + the two
 * asum loops of SortFCNeurons, src/caffe/strategy.cpp:36-77): for a
 * [rows x cols] fault state, flag = (endurance < 0 && value == 0);
 * row_counts[r] = #flags in row r (written), col_counts[c] += #flags in
 * column c (accumulated; zero it first).  Either output may be NULL. */
int rram_stuck_zero_counts(const float* endurance, const float* values, int rows, int cols,
                           unsigned* row_counts, unsigned* col_counts, rram_stream_t stream);

/* Neuron moves of the remapping / genetic strategies (strategy.cpp:109-135,
 * 237-283) as gathers with device index vectors (src != dst):
 *   rows:  dst[to[j]*row_len + c] = src[from[j]*row_len + c]
 *   cols:  dst[k*cols + to[j]]    = src[k*cols + from[j]]   (k < rows)
 *   elems: dst[to[j]]             = src[from[j]]
 * Rows / elements not named in `to` are left untouched. */
int rram_permute_rows(const float* src, float* dst, int64_t row_len, const int* to, const int* from,
                      int n, rram_stream_t stream);
int rram_permute_cols(const float* src, float* dst, int rows, int cols, const int* to, const int* from,
                      int n, rram_stream_t stream);
int rram_permute_elems(const float* src, float* dst, const int* to, const int* from, int n,
                       rram_stream_t stream);

/* g = h = momentum * h + local_rate * g.  Replaces SGDUpdate
 * (src/caffe/solvers/sgd_solver.cu:6-20). */
int rram_sgd_update(float* g, float* h, int64_t n, float momentum,
                    float local_rate, rram_stream_t stream);

/* Fused training tail for one blob: L2 decay, momentum
 * update, threshold strategy, w -= dw, then Fail():
 *   g += decay * w; g = h = mom*h + lr*g; if (|g| <= thr) g = 0; w -= g;
 *   FailKernel(e, v, w, g).
 * endurance/values may be NULL for a non-faultable blob (thr ignored then
 * unless apply_thr != 0). */
int rram_fused_update_fail(float* w, float* g, float* h, float* endurance,
                           const float* values, int64_t n, float decay,
                           float momentum, float local_rate, int apply_thr,
                           float thr, float decrement, float eps,
                           unsigned long long* broken_count,
                           rram_stream_t stream);

/* The same fused tail for every learnable blob of a net in ONE launch (the
 * solver's per-iteration tail, sgd_solver.cpp:101-116 + solver.cpp:300-305,
 * was one launch per blob).  Per segment: the arguments of
 * rram_fused_update_fail; momentum, decrement and eps are solver-wide.
 * Element-wise identical arithmetic, so bit-identical to nsegs calls of
 * rram_fused_update_fail; broken_count may repeat across segments. */
typedef struct rram_update_seg {
  float* w;
  float* g;
  float* h;
  float* endurance;     /* NULL for a non-faultable blob */
  const float* values;  /* NULL iff endurance is NULL */
  int64_t n;
  float decay, local_rate, thr;
  int apply_thr;
  unsigned long long* broken_count; /* may be NULL */
  /* Optional (NULL: off).  A convolution kernel w [G*cout][cin][taps] also
   * written, once updated, transposed per group and rotated 180 degrees into
   * w_flip [G*cin][cout][taps] (G*cin*cout*taps == n): the weights of the
   * stride-1 data gradient as a forward convolution, which
   * rram_conv2d_bwd_ex then takes instead of flipping them itself. */
  float* w_flip;
  int flip_groups, flip_cin, flip_cout, flip_taps;
} rram_update_seg;
int rram_fused_update_fail_batched(const rram_update_seg* segs, int nsegs, float momentum,
                                   float decrement, float eps, rram_stream_t stream);

/* Level-1 helpers used by Blob::Update, Regularize, P2PSync-equivalent
 * scaling (src/caffe/util/math_functions.cu:45-207). */
int rram_axpy(int64_t n, float alpha, const float* x, float* y, rram_stream_t stream);
int rram_axpby(int64_t n, float alpha, const float* x, float beta, float* y, rram_stream_t stream);
int rram_scal(int64_t n, float alpha, float* x, rram_stream_t stream);
int rram_set(int64_t n, float alpha, float* x, rram_stream_t stream);
/* a[0..na) = 0 and b[0..nb) = 0 in one launch: the solver's per-iteration
 * clears (Net::ClearParamDiffs over the flat diff, net.cpp:566-576 in the
 * reference, and the Fail counters) where two fills ran. */
int rram_zero_pair(float* a, int64_t na, unsigned long long* b, int64_t nb, rram_stream_t stream);
int rram_add(int64_t n, const float* a, const float* b, float* y, rram_stream_t stream);
int rram_sign(int64_t n, const float* x, float* y, rram_stream_t stream);
/* out[0] = sum(|x|) (device scalar). */
int rram_asum(int64_t n, const float* x, float* out, rram_stream_t stream);
/* out[0] = max(|x|) (device scalar). */
int rram_absmax(int64_t n, const float* x, float* out, rram_stream_t stream);
/* out[0] = sum(x*y) (device scalar). */
int rram_dot(int64_t n, const float* x, const float* y, float* out, rram_stream_t stream);

/* ------------------------------------------------------------------------
 * Dense GEMM on fp32 MFMA
 * Caffe row-major semantics: C = alpha * op(A) * op(B) + beta * C with
 * op(A) M x K, op(B) K x N, lda = TransA ? M : K, ldb = TransB ? K : N,
 * ldc = N.  Replaces caffe_gpu_gemm (src/caffe/util/math_functions.cu:13-27).
 * trans flags: 0 = CblasNoTrans, 1 = CblasTrans.
 * ---------------------------------------------------------------------- */
int rram_gemm_f32(int trans_a, int trans_b, int M, int N, int K, float alpha,
                  const float* A, const float* B, float beta, float* C,
                  rram_stream_t stream);

enum { RRAM_BIAS_NONE = 0, RRAM_BIAS_ROW = 1, RRAM_BIAS_COL = 2 };
/* Extended form: explicit leading dimensions, fused epilogue
 *   C = act(alpha * op(A) op(B) + beta * C + bias)
 * bias_mode ROW adds bias[m], COL adds bias[n]; relu != 0 clamps at 0.
 * workspace (device, nullable) enables split-K for small-M x N grids; with
 * workspace == NULL or too small the kernel runs without split-K. */
int rram_gemm_f32_ex(int trans_a, int trans_b, int M, int N, int K,
                     float alpha, const float* A, int lda, const float* B,
                     int ldb, float beta, float* C, int ldc, const float* bias,
                     int bias_mode, int relu, void* workspace,
                     size_t workspace_bytes, rram_stream_t stream);

/* y[M] = alpha * op(A) x + beta * y.  Replaces caffe_gpu_gemv
 * (src/caffe/util/math_functions.cu:45-53). */
int rram_gemv_f32(int trans_a, int M, int N, float alpha, const float* A,
                  const float* x, float beta, float* y, rram_stream_t stream);

/* ------------------------------------------------------------------------
 * Convolution
 * NCHW fp32.  Forward is an implicit GEMM over the whole batch
 * (M = Cout/g, N = num*Ho*Wo, K = Cin/g*kh*kw) on fp32 MFMA with im2col fused
 * into the LDS fill, replacing the reference's per-image im2col +
 * caffe_gpu_gemm loop (src/caffe/layers/conv_layer.cu:7-24,
 * src/caffe/layers/base_conv_layer.cpp:325-350).
 * ---------------------------------------------------------------------- */
typedef struct {
  int num, channels, height, width;  /* input  N, C, H, W            */
  int num_output;                    /* Cout                          */
  int kernel_h, kernel_w;
  int pad_h, pad_w;
  int stride_h, stride_w;
  int dilation_h, dilation_w;
  int group;
  int out_h, out_w;                  /* filled by rram_conv_out_shape */
} rram_conv_desc;

/* Computes out_h/out_w with Caffe's rule (base_conv_layer.cpp:18-28 via
 * conv_layer.cpp:9-19) and validates the descriptor. */
int rram_conv_out_shape(rram_conv_desc* d);

/* y = conv(x, w) + bias (bias nullable), optional fused ReLU. */
int rram_conv2d_fwd(const rram_conv_desc* d, const float* x, const float* w,
                    const float* bias, float* y, int relu, rram_stream_t stream);

/* rram_conv2d_fwd with channel-octet companions (no reference counterpart:
 * an inference-time layout of this build).  The octet companion of an NCHW
 * fp32 tensor [num][C][H][W] (C % 8 == 0) is [num][C/8][H][W][3][8] bf16:
 * the exact three-term bf16 split (x = xh + xm + xl) of 8 consecutive
 * channels at one position, the operand form of the bf16x6 convolution.
 *   x_oct  NULL, or x's companion (saves the convolution its input pack);
 *   y_oct  NULL, or num*num_output*out_h*out_w*6 bytes that receive y's
 *          companion (written by the convolution's epilogue when the
 *          channel-octet kernel runs, else packed from y).
 * y is bit-identical to rram_conv2d_fwd's. */
int rram_conv2d_fwd_octets(const rram_conv_desc* d, const float* x, const void* x_oct, const float* w,
                           const float* bias, float* y, void* y_oct, int relu, rram_stream_t stream);
/* Packed-weight companion (no reference counterpart; the reference re-reads
 * w through cuBLAS each call, conv_layer.cu:7-25).  The bf16x6 engine splits
 * w into fragment-order bf16 terms before every forward; a caller whose
 * weights do not change between calls (Monte-Carlo inference: only the
 * faultable blobs are rewritten per map) keeps that pack:
 *   rram_conv_weight_pack_bytes  bytes of the pack for this shape under the
 *                                current engine (0: the engine taking this
 *                                shape reads w directly — no pack);
 *   rram_conv2d_fwd_cached       rram_conv2d_fwd_octets with w_pack (16-byte
 *                                aligned, rram_conv_weight_pack_bytes bytes):
 *                                w_pack_valid = 0 packs w into it first,
 *                                1 uses it as is (the caller guarantees it
 *                                holds the pack of the same w, same shape and
 *                                engine).  w_pack NULL = rram_conv2d_fwd_octets.
 * y is bit-identical to rram_conv2d_fwd_octets'. */
size_t rram_conv_weight_pack_bytes(const rram_conv_desc* d);
int rram_conv2d_fwd_cached(const rram_conv_desc* d, const float* x, const void* x_oct, const float* w,
                           void* w_pack, int w_pack_valid, const float* bias, float* y, void* y_oct, int relu,
                           rram_stream_t stream);
/* rram_conv2d_fwd_cached writing y inside a larger NCHW tensor: image n's
 * output starts at y + n * y_image_stride (>= num_output * out_h * out_w
 * floats), e.g. y = top + offset * out_h * out_w and y_image_stride =
 * C_top * out_h * out_w for a Concat top along channels.  The TEST-phase
 * Concat fold writes each inception branch straight into its slice of the
 * Concat top, replacing the copy of concat_layer.cu:6-48 (Forward_gpu) for
 * those bottoms.  No output octets; w_pack as in rram_conv2d_fwd_cached.
 * Every value is bit-identical to rram_conv2d_fwd_cached's. */
int rram_conv2d_fwd_strided(const rram_conv_desc* d, const float* x, const void* x_oct, const float* w,
                            void* w_pack, int w_pack_valid, const float* bias, float* y, int64_t y_image_stride,
                            int relu, rram_stream_t stream);
/* 1 when rram_conv2d_fwd_octets would read an x_oct for this shape now. */
int rram_conv_input_octets(const rram_conv_desc* d);
/* 1 when rram_conv2d_fwd_octets / _cached accept y = NULL with y_oct for this
 * shape now: the channel-octet kernel's 16x16x32 epilogue, or the 1x1
 * kernels' (round 6), then writes only the companion (bit-identical to the
 * one it writes next to y), no fp32 y.  The TEST-phase convolution-output
 * fold: a convolution whose top is read only by another convolution that
 * takes the companion (AlexNet conv3 -> conv4, conv4 -> conv5; GoogLeNet's
 * 3x3_reduce -> 3x3).  No reference counterpart (a fusion of this build);
 * with y = NULL on a shape this returns 0 for, the calls return RRAM_EINVAL. */
int rram_conv_output_octets_only(const rram_conv_desc* d);
/* Host-side plan of the channel-octet kernel for d (no device work):
 * plan[0..4] = tile rows, tile columns, workgroups per CU, tiles per image
 * (0 = tiles run across images), LDS patch pieces per wave.  Returns 1 with
 * the plan filled, 0 when the octet kernel does not take d. */
int rram_conv_octet_plan(const rram_conv_desc* d, int* plan);
/* oct = the octet companion of x (channels % 8 == 0). */
int rram_pack_octets(const float* x, void* oct, int num, int channels, int height, int width,
                     rram_stream_t stream);

/* Matrix-core engine of the fp32 forward contractions (no reference
 * counterpart: the reference's engine is cuBLAS SGEMM, math_functions.cu:13-27).
 *   RRAM_ENGINE_F32    v_mfma_f32_32x32x2_f32 (fp32 operands).
 *   RRAM_ENGINE_BF16X6 (default) each fp32 operand split exactly into three
 *                      bf16 terms, six cross products accumulated in fp32 on
 *                      v_mfma_f32_32x32x16_bf16 (fp32-accurate products, ~2x
 *                      the fp32 matrix-core rate).  Used by the stride-1
 *                      3x3 / 5x5 convolution forward and the InnerProduct /
 *                      NoTrans x Trans GEMM forward (rram_ip_fwd); every
 *                      other contraction stays on RRAM_ENGINE_F32.
 * The initial value comes from RRAM_X6 (0 = F32).  Returns the previous
 * engine, or RRAM_EINVAL for an unknown one. */
enum { RRAM_ENGINE_F32 = 0, RRAM_ENGINE_BF16X6 = 1 };
int rram_set_f32_engine(int engine);
int rram_get_f32_engine(void);
/* The engine rram_conv2d_fwd / rram_ip_fwd (transpose = 0, 16-byte aligned
 * operands, workspace of ws_bytes) would use for this shape right now. */
int rram_f32_engine_for_conv(const rram_conv_desc* d);
int rram_f32_engine_for_ip(int M, int N, int K, size_t ws_bytes);

/* Bytes of device workspace the backward passes need for `images_per_chunk`
 * images (explicit im2col/col2im buffer). */
size_t rram_conv2d_bwd_workspace(const rram_conv_desc* d, int images_per_chunk);

/* dw += conv weight gradient, db += bias gradient (db nullable);
 * dx = data gradient (dx nullable).  Workspace from rram_conv2d_bwd_workspace.
 * Replaces ConvolutionLayer::Backward_gpu (src/caffe/layers/conv_layer.cu:27-56). */
int rram_conv2d_bwd(const rram_conv_desc* d, const float* x, const float* w,
                    const float* dy, float* dw, float* db, float* dx,
                    void* workspace, size_t workspace_bytes,
                    rram_stream_t stream);
/* rram_conv2d_bwd with the flipped kernel supplied: w_flipped (nullable) holds
 * w in rram_update_seg's w_flip layout, read by the stride-1 data gradient in
 * place of the flip pass (conv_layer.cu:47-52's data GEMM as a forward
 * convolution).  rram_conv2d_flip_applies(d) = 1 when that path serves d. */
int rram_conv2d_bwd_ex(const rram_conv_desc* d, const float* x, const float* w,
                       const float* w_flipped, const float* dy, float* dw, float* db,
                       float* dx, void* workspace, size_t workspace_bytes,
                       rram_stream_t stream);
int rram_conv2d_flip_applies(const rram_conv_desc* d);

/* Replaces im2col_gpu / col2im_gpu (src/caffe/util/im2col.cu:41-62,
 * :300-320).  One image; col is [C*kh*kw][Ho*Wo]. col2im writes (not adds) im. */
int rram_im2col(const float* im, int channels, int height, int width,
                int kernel_h, int kernel_w, int pad_h, int pad_w, int stride_h,
                int stride_w, int dilation_h, int dilation_w, float* col,
                rram_stream_t stream);
int rram_col2im(const float* col, int channels, int height, int width,
                int kernel_h, int kernel_w, int pad_h, int pad_w, int stride_h,
                int stride_w, int dilation_h, int dilation_w, float* im,
                rram_stream_t stream);

/* ------------------------------------------------------------------------
 * InnerProduct
 * top[M,N] = bottom[M,K] * W^T (+ bias), W is [N,K] (transpose=0) or [K,N]
 * (transpose=1).  Replaces InnerProductLayer::Forward_gpu/Backward_gpu
 * (src/caffe/layers/inner_product_layer.cu:9-75).
 * ---------------------------------------------------------------------- */
int rram_ip_fwd(const float* x, const float* w, const float* bias, float* y,
                int M, int N, int K, int transpose, int relu, void* workspace,
                size_t workspace_bytes, rram_stream_t stream);
/* The bf16x6 engine's packed-row form of an InnerProduct input, for
 * inference chains (fc6 -> fc7): its bytes and tile rows for an M x K input of
 * an N-output layer (rows_per_tile nullable; 0: the engine does not serve the
 * shape).  rram_ip_fwd_rows = rram_ip_fwd (W [N][K], no transpose) where x_rows
 * (nullable) already holds x in that form (no pack pass) and y_rows (nullable)
 * receives y in the form of the next layer (its rows_per_tile; K = N there),
 * written by the split-K reduce (inner_product_layer.cu:9-30 forwards, the same
 * bits; *y_rows_written = 0 when the engine did not serve this shape). */
size_t rram_ip_rows_pack_bytes(int M, int N, int K, size_t ws_bytes, int* rows_per_tile);
int rram_ip_fwd_rows(const float* x, const void* x_rows, const float* w, const float* bias, float* y, void* y_rows,
                     int y_rows_per_tile, int M, int N, int K, int relu, void* ws, size_t ws_bytes,
                     int* y_rows_written, rram_stream_t stream);
/* dw += ..., db += ... (nullable), dx = ... (nullable). */
int rram_ip_bwd(const float* x, const float* w, const float* dy, float* dw,
                float* db, float* dx, int M, int N, int K, int transpose,
                rram_stream_t stream);

/* ------------------------------------------------------------------------
 * Support layers needed to run the configs end to end (not fault path).
 * ---------------------------------------------------------------------- */
/* ReLU with Caffe's negative_slope (src/caffe/layers/relu_layer.cu). */
int rram_relu_fwd(const float* x, float* y, int64_t n, float slope, rram_stream_t s);
int rram_relu_bwd(const float* x, const float* dy, float* dx, int64_t n, float slope, rram_stream_t s);

enum { RRAM_POOL_MAX = 0, RRAM_POOL_AVE = 1 };
/* Pooling with Caffe's ceil output rule (pooling_layer.cpp:90-104);
 * mask (int32, nullable) records argmax for MAX. */
int rram_pool_fwd(const float* x, float* y, int* mask, int num, int channels,
                  int height, int width, int pooled_h, int pooled_w,
                  int kernel_h, int kernel_w, int stride_h, int stride_w,
                  int pad_h, int pad_w, int method, rram_stream_t s);
int rram_pool_bwd(const float* dy, const int* mask, float* dx, int num,
                  int channels, int height, int width, int pooled_h,
                  int pooled_w, int kernel_h, int kernel_w, int stride_h,
                  int stride_w, int pad_h, int pad_w, int method, rram_stream_t s);
/* rram_pool_fwd followed by an in-place ReLU of y (relu_layer.cu:9-15, y =
 * y > 0 ? y : y * relu_slope) in the same launch: a Pooling layer whose top
 * an in-place ReLU rewrites (CIFAR-10 pool1 -> relu1).  y is bit-identical to
 * rram_pool_fwd + rram_relu_fwd; the MAX mask is the pre-ReLU argmax, as
 * there. */
int rram_pool_relu_fwd(const float* x, float* y, int* mask, int num, int channels,
                       int height, int width, int pooled_h, int pooled_w,
                       int kernel_h, int kernel_w, int stride_h, int stride_w,
                       int pad_h, int pad_w, int method, float relu_slope, rram_stream_t s);

/* rram_pool_bwd followed by the backward of the in-place ReLU that produced
 * the pool's input (relu_layer.cu:35-44: dx *= (y > 0) + (y <= 0) * slope,
 * y = relu_y, the ReLU's output = the pool's bottom data) in the same launch:
 * a ReLU -> Pooling pair (CIFAR-10 full relu2 -> pool2).  Bit-identical to
 * rram_pool_bwd + rram_relu_bwd. */
int rram_pool_relu_bwd(const float* dy, const int* mask, float* dx, int num,
                       int channels, int height, int width, int pooled_h,
                       int pooled_w, int kernel_h, int kernel_w, int stride_h,
                       int stride_w, int pad_h, int pad_w, int method,
                       const float* relu_y, float relu_slope, rram_stream_t s);

/* y[i] = (float)x[i]: a MAX pool's int32 argmax as the float top mask
 * (pooling_layer.cu:30-34, the optional second top). */
int rram_i32_to_f32(const int* x, float* y, int64_t n, rram_stream_t s);

/* LRN ACROSS_CHANNELS (lrn_layer.cu): scale = k + alpha/size * sum x^2,
 * y = x * scale^-beta.  scale (nullable) keeps the scale for backward. */
int rram_lrn_fwd(const float* x, float* y, float* scale, int num, int channels,
                 int height, int width, int size, float alpha, float beta,
                 float k, rram_stream_t s);
int rram_lrn_bwd(const float* x, const float* y, const float* scale,
                 const float* dy, float* dx, int num, int channels, int height,
                 int width, int size, float alpha, float beta, rram_stream_t s);

/* LRN WITHIN_CHANNEL (lrn_layer.cpp: square -> AVE pool (local_size, pad
 * (size-1)/2, stride 1) -> (1 + alpha * avg)^-beta -> product); scale keeps
 * 1 + alpha * avg for backward (nullable in forward-only use). */
int rram_lrn_within_fwd(const float* x, float* y, float* scale, int num, int channels, int height,
                        int width, int size, float alpha, float beta, rram_stream_t s);
int rram_lrn_within_bwd(const float* x, const float* scale, const float* dy, float* dx, int num,
                        int channels, int height, int width, int size, float alpha, float beta,
                        rram_stream_t s);
/* rram_lrn_within_bwd followed by the backward of the in-place ReLU that
 * produced x (dx *= (x > 0) + (x <= 0) * relu_slope, relu_layer.cu:35-44) in
 * the same launch: a ReLU -> LRN pair (CIFAR-10 full relu1 -> norm1).
 * Bit-identical to rram_lrn_within_bwd + rram_relu_bwd. */
int rram_lrn_within_relu_bwd(const float* x, const float* scale, const float* dy, float* dx, int num, int C,
                             int H, int W, int size, float alpha, float beta, float relu_slope, rram_stream_t s);

/* Inference fusion (TEST phase) of LRN ACROSS_CHANNELS followed by MAX
 * pooling whose bottom is the LRN top and nothing else reads it:
 * y = maxpool(lrn(x)) without materialising lrn(x).  Every LRN value is
 * rram_lrn_fwd's bit for bit; window rule as rram_pool_fwd.  kernel in {2,3}
 * (square), size in {3,5}, pad < kernel.  Replaces LRNLayer::Forward_gpu +
 * PoolingLayer::Forward_gpu (src/caffe/layers/lrn_layer.cu:9-99,
 * src/caffe/layers/pooling_layer.cu:11-47,158-178) for that layer pair. */
int rram_lrn_maxpool_fwd(const float* x, float* y, int num, int channels, int height, int width,
                         int pooled_h, int pooled_w, int kernel, int stride_h, int stride_w,
                         int pad_h, int pad_w, int size, float alpha, float beta, float k,
                         rram_stream_t s);

/* rram_lrn_maxpool_fwd that also writes y's channel-octet companion
 * (y_oct nullable; channels % 8 == 0), see rram_conv2d_fwd_octets.  y may be
 * NULL when y_oct is not: only the companion is written (the caller's only
 * reader of y takes the companion; it must re-run with y before anything
 * reads y itself). */
int rram_lrn_maxpool_fwd_octets(const float* x, float* y, void* y_oct, int num, int channels, int height,
                                int width, int pooled_h, int pooled_w, int kernel, int stride_h, int stride_w,
                                int pad_h, int pad_w, int size, float alpha, float beta, float k,
                                rram_stream_t s);

/* Softmax over `channels` for [outer][channels][inner]. */
int rram_softmax_fwd(const float* x, float* y, int outer, int channels, int inner, rram_stream_t s);
/* SoftmaxWithLoss forward: loss_out[0] = -sum log(max(p[label], FLT_MIN)) / normalizer
 * where normalizer = #valid (ignore_label < 0 disables ignoring). */
int rram_softmax_loss_fwd(const float* prob, const float* label, float* loss_out,
                          int outer, int channels, int inner, int ignore_label,
                          rram_stream_t s);
/* rram_softmax_loss_fwd that also folds the loss into a MonteCarlo statistic:
 * *acc_sum += loss, *acc_row = loss when non-NULL (rram_mc_accumulate's
 * arithmetic for that output, so the MC driver needs no accumulate launch). */
int rram_softmax_loss_fwd_acc(const float* prob, const float* label, float* out, int outer, int C, int inner,
                              int ignore, float* acc_sum, float* acc_row, rram_stream_t s);
int rram_softmax_loss_bwd(const float* prob, const float* label, float* dx,
                          int outer, int channels, int inner, int ignore_label,
                          float loss_weight, rram_stream_t s);
/* rram_softmax_loss_fwd and rram_softmax_loss_bwd in one launch (a TRAIN-phase
 * SoftmaxWithLoss head of <= 65536 elements: CIFAR-10 / LeNet): out = the
 * loss, dx = the bottom gradient, both bit-identical to the two calls. */
int rram_softmax_loss_fwd_bwd(const float* prob, const float* label, float* out, float* dx, int outer, int C,
                              int inner, int ignore, float loss_weight, rram_stream_t s);
/* Top-k accuracy (accuracy_layer.cpp:48-90): correct_out[0] = #correct,
 * count_out[0] = #counted, ratio_out[0] (nullable) = #correct / #counted
 * (device floats; the layer's top). */
int rram_accuracy(const float* x, const float* label, float* correct_out,
                  float* count_out, float* ratio_out, int outer, int channels,
                  int inner, int top_k, int ignore_label, rram_stream_t s);
/* rram_accuracy with the same MonteCarlo fold of the ratio (see
 * rram_softmax_loss_fwd_acc; acc_sum requires ratio). */
int rram_accuracy_acc(const float* x, const float* label, float* correct, float* count, float* ratio, int outer,
                      int C, int inner, int top_k, int ignore, float* acc_sum, float* acc_row, rram_stream_t s);
/* EuclideanLoss (euclidean_loss_layer.cu:9-38): diff = a - b,
 * loss_out[0] = sum(diff^2) / num / 2 (device scalar, the layer's top);
 * backward dx = alpha * diff with alpha = +-loss_weight / num. */
int rram_euclidean_loss_fwd(const float* a, const float* b, float* diff, float* loss_out, int64_t n, int num,
                            rram_stream_t s);
int rram_euclidean_loss_bwd(const float* diff, float* dx, int64_t n, float alpha, rram_stream_t s);
/* Concat / Slice copy (concat_layer.cu, slice_layer.cu): one bottom's
 * [num][src_channels_x_inner] block into its slot of the
 * [num][dst_channels_x_inner] top at offset_x_inner (backward != 0: the
 * reverse copy, dst slot -> src). */
int rram_concat_copy(const float* src, float* dst, int num, int src_channels_x_inner,
                     int dst_channels_x_inner, int offset_x_inner, int backward,
                     rram_stream_t s);
/* Dropout train mode: mask from Philox(seed, layer, index); y = x*scale or 0. */
int rram_dropout_fwd(const float* x, float* y, unsigned int* mask, int64_t n,
                     float ratio, uint64_t seed, uint32_t layer_id, uint64_t iter,
                     rram_stream_t s);
int rram_dropout_bwd(const float* dy, const unsigned int* mask, float* dx,
                     int64_t n, float ratio, rram_stream_t s);
/* y[n][c][hw] += bias[c] */
int rram_bias_add(float* y, const float* bias, int num, int channels, int inner, rram_stream_t s);
/* db[c] += sum_{n,hw} dy[n][c][hw] */
int rram_bias_bwd(const float* dy, float* db, int num, int channels, int inner, rram_stream_t s);

/* ------------------------------------------------------------------------
 * Fillers / synthetic data (Philox; seeded; statistically equivalent to the
 * reference's boost/cuRAND fillers, not bit-identical).
 * ---------------------------------------------------------------------- */
int rram_fill_uniform(float* x, int64_t n, float lo, float hi, uint64_t seed,
                      uint32_t stream_id, rram_stream_t s);
int rram_fill_gaussian(float* x, int64_t n, float mean, float std,
                       uint64_t seed, uint32_t stream_id, rram_stream_t s);
/* x = floor(U[0, levels)) + offset (integer-valued synthetic images / labels). */
int rram_fill_uniform_int(float* x, int64_t n, int levels, float offset,
                          uint64_t seed, uint32_t stream_id, rram_stream_t s);

#ifdef __cplusplus
}
#endif

#endif /* RRAM_KERNELS_H_ */
