/*
 * rram_caffe.h — C-ABI of the C++ Caffe-shaped host runtime (librram_caffe.so).
 *
 * The host keeps the reference's C++ API (caffe::Net / Layer / Solver /
 * FailureMaker, host/ headers) and exposes it through opaque handles so that
 * non-C++ callers (Python ctypes, the bench, a cgo/JNI binding) can drive the
 * drop-in path.  Every call returns RRAM_OK (0) or a negative status and never
 * aborts; rram_caffe_last_error() holds the message (the reference's glog
 * CHECK failures become RRAM_EINVAL here).
 *
 * Device pointers handed out (blob / param / fault-state accessors) stay valid
 * until the owning handle is destroyed or the blob is reshaped.
 */
#ifndef RRAM_CAFFE_H_
#define RRAM_CAFFE_H_

#include <stddef.h>
#include <stdint.h>

#include "rram_kernels.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rram_net_s* rram_net_t;
typedef struct rram_solver_s* rram_solver_t;
typedef struct rram_mc_s* rram_mc_t;
typedef struct rram_syncedmem_s* rram_syncedmem_t;

enum { RRAM_PHASE_TRAIN = 0, RRAM_PHASE_TEST = 1 };

const char* rram_caffe_last_error(void);
/* All host work of the calling thread is issued on this stream (Caffe::Get()
 * is per-thread, common.cpp:13-20).  NULL = default stream. */
int rram_caffe_set_stream(rram_stream_t stream);
/* Caffe::set_random_seed (common.cpp:131-147): seeds fillers, synthetic data,
 * fault draws. */
int rram_caffe_set_random_seed(uint64_t seed);
int rram_caffe_synchronize(void);

/* --------------------------------------------------------- SyncedMemory
 * caffe::SyncedMemory (syncedmem.hpp:45-83, syncedmem.cpp:25-153): lazy
 * host/device mirror with the head states below (== SyncedMemory::SyncedHead).
 * cpu_data / mutable_cpu_data on an UNINITIALIZED or HEAD_AT_CPU buffer touch
 * no device; gpu_* calls allocate / copy on the calling thread's stream and
 * synchronise it (syncedmem.cpp:51-77).  set_*_data borrow caller memory that
 * the buffer never frees (syncedmem.cpp:84-122). */
enum { RRAM_HEAD_UNINITIALIZED = 0, RRAM_HEAD_AT_CPU = 1, RRAM_HEAD_AT_GPU = 2, RRAM_HEAD_SYNCED = 3 };
int rram_syncedmem_create(size_t size, rram_syncedmem_t* out);
int rram_syncedmem_destroy(rram_syncedmem_t m);
int rram_syncedmem_head(rram_syncedmem_t m, int* head);
int rram_syncedmem_size(rram_syncedmem_t m, size_t* size);
int rram_syncedmem_cpu_data(rram_syncedmem_t m, const void** p);
int rram_syncedmem_gpu_data(rram_syncedmem_t m, const void** p);
int rram_syncedmem_mutable_cpu_data(rram_syncedmem_t m, void** p);
int rram_syncedmem_mutable_gpu_data(rram_syncedmem_t m, void** p);
int rram_syncedmem_set_cpu_data(rram_syncedmem_t m, void* p);
int rram_syncedmem_set_gpu_data(rram_syncedmem_t m, void* p);

/* ---------------------------------------------------------------- Net
 * net_prototxt: NetParameter text (caffe.proto); options: text-format
 * key/values, e.g. 'data_shape: "3,227,227" num_classes: 1000
 * fault_layers: "InnerProduct" fuse_relu: true'.  Replaces Net<Dtype>(param)
 * (net.cpp:42-300). */
int rram_net_create(const char* net_prototxt, int phase, const char* options, rram_net_t* out);
int rram_net_destroy(rram_net_t net);
/* Net::Forward (net.cpp:558-569); loss_out (nullable) gets the weighted loss
 * when compute_loss != 0 (one small D2H). */
int rram_net_forward(rram_net_t net, int compute_loss, float* loss_out);
int rram_net_backward(rram_net_t net);
int rram_net_update(rram_net_t net);
int rram_net_clear_param_diffs(rram_net_t net);
int rram_net_num_layers(rram_net_t net, int* n);
/* name/type copied into caller buffers of `cap` bytes */
int rram_net_layer_info(rram_net_t net, int i, char* name, char* type, int cap, int* num_params);
/* Forward contraction of layer i at the current shapes (no reference
 * counterpart; for rooflines): *flops = 2 M N K of its GEMM (Convolution:
 * num x Cout x Ho Wo x Cin/group kh kw; InnerProduct: M N K; 0 for other
 * layers) and *engine = the RRAM_ENGINE_* rram_conv2d_fwd / rram_ip_fwd take
 * for it now (-1 for other layers). */
int rram_net_layer_contraction(rram_net_t net, int i, double* flops, int* engine);
int rram_net_num_blobs(rram_net_t net, int* n);
int rram_net_blob_name(rram_net_t net, int i, char* name, int cap);
/* device pointers and shape (up to 8 axes) of a named blob (a blob a
 * TEST-phase fold left unwritten is materialised first, and stays so) */
int rram_net_blob(rram_net_t net, const char* name, float** data, float** diff, int* shape, int* num_axes);
/* *stale = 1 when the named blob's fp32 contents were not written by the last
 * forward (its producer wrote only the octet companion its one reader takes:
 * the pooled-output fold), 0 otherwise; does not materialise.  No reference
 * counterpart (a fusion of this build). */
int rram_net_blob_stale(rram_net_t net, const char* name, int* stale);
int rram_net_num_params(rram_net_t net, int* n);
int rram_net_param(rram_net_t net, int i, float** data, float** diff, int64_t* count, float* lr_mult,
                   float* decay_mult);
/* Net::failure_learnable_params() (net.hpp:181-183): InnerProduct weights and
 * biases; layer_id = owning layer index. */
int rram_net_num_failure_params(rram_net_t net, int* n);
int rram_net_failure_param(rram_net_t net, int i, float** data, float** diff, int64_t* count, int* layer_id);
int rram_net_num_outputs(rram_net_t net, int* n);
int rram_net_output(rram_net_t net, int i, char* name, int cap, float** data, int64_t* count);
/* Net::ShareTrainedLayersWith (net.cpp:697-720) */
int rram_net_share_trained(rram_net_t dst, rram_net_t src);
/* P2PSync GPUParams equivalent (parallel.cpp:25-115): alias every learnable
 * param into caller-owned flat device buffers of rram_net_flat_param_count
 * floats (data copied in, diff zeroed). */
int rram_net_flat_param_count(rram_net_t net, int64_t* n);
int rram_net_alias_flat_params(rram_net_t net, float* data, float* diff);
/* Per-layer forward timing (`caffe time`, tools/caffe.cpp:334-421): hipEvents
 * around every layer (enable = 1) or only around layers that own parameters,
 * i.e. Convolution / InnerProduct (enable = 2), on the working stream.
 * layer_times synchronises and returns total ms and launch count per layer
 * since the last reset. */
int rram_net_set_timing(rram_net_t net, int enable);
/* Events around one layer only (index into the net's layers): the live
 * timing of a single kernel with the fewest markers in the stream. */
int rram_net_set_timing_layer(rram_net_t net, int layer);
int rram_net_layer_times(rram_net_t net, double* ms, long* counts, int cap, int* n, int reset);
/* Host-only structural view (no device): phase filter + split insertion;
 * writes "name\ttype\tbottoms\ttops\n" lines into out (cap bytes);
 * *needed = bytes required including the terminator. */
int rram_net_describe(const char* net_prototxt, int phase, char* out, size_t cap, size_t* needed);

/* ------------------------------------------------------------- Solver
 * SGDSolver with the fork's fault hooks (solver.cpp:14-40, :237-325).
 * net_prototxt (nullable) overrides the solver's net: / net_param.
 * options: the net options above plus fused_update: true|false. */
int rram_solver_create(const char* solver_prototxt, const char* net_prototxt, const char* options,
                       rram_solver_t* out);
int rram_solver_destroy(rram_solver_t s);
int rram_solver_step(rram_solver_t s, int iters);
/* hipGraph replay of the training iteration (opt-in, for launch-bound small
 * nets; no reference counterpart): clear + forward + backward and the fused
 * update / threshold / Fail tail are each captured once and replayed, the
 * on_gradients_ready hook (data-parallel all-reduce) running between them.
 * Iterations that display, test, snapshot or average the loss run eager;
 * a moving learning rate keeps the eager path.  RRAM_EINVAL for nets with
 * per-iteration host state (Dropout, HDF5Data).  Bit-identical to eager. */
int rram_solver_set_graph(rram_solver_t s, int enable);
int rram_solver_graph_active(rram_solver_t s, int* active);
int rram_solver_solve(rram_solver_t s);
int rram_solver_iter(rram_solver_t s, int* iter);
int rram_solver_smoothed_loss(rram_solver_t s, float* loss);
int rram_solver_learning_rate(rram_solver_t s, float* lr);
/* train net handle (owned by the solver; do not destroy) */
int rram_solver_net(rram_solver_t s, rram_net_t* net);
int rram_solver_num_test_nets(rram_solver_t s, int* n);
int rram_solver_test_net(rram_solver_t s, int i, rram_net_t* net);
/* Solver::Test (solver.cpp:385-458): mean of every output element over test_iter */
int rram_solver_test(rram_solver_t s, int test_net, float* scores, int cap, int* n);
/* on_gradients_ready callback (solver.hpp:80-91, parallel.cpp:324-380):
 * called once per iteration after backward, before the update. */
typedef void (*rram_callback_t)(void* user);
int rram_solver_set_gradient_callback(rram_solver_t s, rram_callback_t cb, void* user);
/* Per-layer backward hook of the train net: cb(layer_index, user) after each
 * layer's Backward, in backward order (every layer index, with or without
 * params).  Lets a data-parallel driver start bucketed gradient all-reduces
 * while earlier layers are still in backward. NULL = off. */
typedef void (*rram_layer_callback_t)(int layer, void* user);
int rram_solver_set_backward_callback(rram_solver_t s, rram_layer_callback_t cb, void* user);
/* log lines in the reference's format ("Iteration N, loss = ...",
 * "    Test net output #k: name = v"), delivered to cb (NULL = silent). */
typedef void (*rram_log_callback_t)(const char* line, void* user);
int rram_solver_set_log_callback(rram_solver_t s, rram_log_callback_t cb, void* user);
/* Fault state (GaussianFailureMaker::fail_iterations(), failure_maker.hpp:82-84):
 * endurance = blob data, stuck values = blob diff, reference layout.
 * n = 0 when the solver has no failure_pattern. */
int rram_solver_num_fail_blobs(rram_solver_t s, int* n);
int rram_solver_fail_state(rram_solver_t s, int i, float** endurance, float** values, int64_t* count);
/* broken cells per faultable blob after the last Fail() (device count, one D2H) */
int rram_solver_broken_counts(rram_solver_t s, unsigned long long* out, int cap, int* n);
/* SGDSolver::history() (sgd_solver.hpp:29, sgd_solver.cpp:16-26): the momentum
 * history blob of learnable param i (device pointer, count). */
int rram_solver_num_history(rram_solver_t s, int* n);
int rram_solver_history(rram_solver_t s, int i, float** data, int64_t* count);

/* Solver::ApplyStrategy (solver.cpp:25-33): run every failure_strategy's
 * Apply() once, outside Step (threshold / remapping / genetic). */
int rram_solver_apply_strategies(rram_solver_t s);
/* Strategy i's type and counters: genetic -> (dist before, dist after,
 * accepted swaps) of its last Apply(); others -> zeros. */
int rram_solver_strategy_info(rram_solver_t s, int i, char* type, int cap, int* a, int* b, int* c);
/* Solver::Snapshot (solver.cpp:461-518, sgd_solver.cpp:249-305): writes
 * <snapshot_prefix>_iter_N.{caffemodel,solverstate} (snapshot_format
 * BINARYPROTO) or .{caffemodel.h5,solverstate.h5} (HDF5), plus .faultstate;
 * the solver-state path is copied into path_out (cap bytes, nullable). */
int rram_solver_snapshot(rram_solver_t s, char* path_out, int cap);
/* Solver::Restore (solver.cpp:520-530, sgd_solver.cpp:307-351) from a
 * .solverstate or .solverstate.h5; the fault maps are restored when the
 * matching .faultstate exists. */
int rram_solver_restore(rram_solver_t s, const char* state_file);
/* Solver::Solve(resume_file) (solver.cpp:328-370); resume_file nullable. */
int rram_solver_solve_from(rram_solver_t s, const char* resume_file);

/* ------------------------------------------------------ weight files
 * Net::CopyTrainedLayersFrom (net.cpp:765-860) for a binary .caffemodel
 * (NetParameter `layer` or V1 `layers`) or, for a name ending in ".h5", the
 * HDF5 layout (group "data" / layer name / dataset "<blob index>"); and
 * Net::ToProto + write (net.cpp:871-880) or Net::ToHDF5 (net.cpp:862-932,
 * ".h5" names).  HDF5 goes through libhdf5 / libhdf5_hl loaded at run time
 * (RRAM_HDF5_LIB_DIR); without them the .h5 paths return RRAM_EINVAL. */
int rram_net_copy_trained_layers_from(rram_net_t net, const char* caffemodel);
int rram_net_save_weights(rram_net_t net, const char* caffemodel, int write_diff);
/* Host-only (no device): one line per blob of a .caffemodel (or .h5: type "-"),
 * "layer\ttype\tindex\tshape\tcount\tdata_sum\tdiff_count"; *needed = bytes
 * including the terminator. */
int rram_caffemodel_describe(const char* caffemodel, char* out, size_t cap, size_t* needed);
/* Host-only: parse a binary proto file and serialise it again
 * (kind 0 NetParameter, 1 SolverState, 2 BlobProtoVector). */
int rram_proto_rewrite(const char* in_path, const char* out_path, int kind);
/* Host-only: the fault-related fields of a SolverParameter text with
 * caffe.proto's defaults applied, one tab-separated line each:
 *   failure_pattern  type mean std neg zero pos
 *   failure_strategy type threshold start period prune_order_file switch_time
 *                    prune_net_file prune_model_file
 *   solver           lr_policy base_lr max_iter snapshot snapshot_prefix */
int rram_solver_describe(const char* solver_prototxt, char* out, size_t cap, size_t* needed);
/* Host-only: n outputs of glibc's rand() after srand(seed) (the genetic
 * strategy's generator, strategy.cpp:170-175). */
int rram_glibc_rand(uint32_t seed, int n, int* out);

/* --------------------------------------------------------- Monte-Carlo
 * Fault-map inference on a TEST-phase net: for maps m in [begin, begin+count):
 * inject(clean weights) -> forward -> accumulate scalar outputs.  cfgs: one
 * config for every faultable blob, or ncfg == 1 for all.  The net's
 * faultable weights are restored when the handle is destroyed. */
int rram_mc_create(rram_net_t net, const rram_inject_cfg* cfgs, int ncfg, uint64_t seed, int max_maps,
                   rram_mc_t* out);
int rram_mc_destroy(rram_mc_t mc);
/* asynchronous on the caller's stream */
int rram_mc_run(rram_mc_t mc, uint32_t map_begin, uint32_t map_count);
int rram_mc_reset(rram_mc_t mc);
int rram_mc_restore_clean(rram_mc_t mc);
/* synchronises; sums[n_outputs] over maps, broken[n_fault_blobs] summed over
 * maps, per_map[min(maps, max_maps) * n_outputs] (nullable buffers skip). */
int rram_mc_stats(rram_mc_t mc, double* sums, int sums_cap, int* n_outputs, unsigned long long* broken,
                  int broken_cap, int* n_blobs, float* per_map, int per_map_cap, int* maps_run);
/* hipEvent timing of the injection launches; inject_times synchronises and
 * returns total ms / launches since the last reset, and the faultable weight count. */
int rram_mc_set_timing(rram_mc_t mc, int enable);
/* Opt-in prefix reuse (a different workload from the reference's per-map
 * full forward): with only InnerProduct blobs faulted, the layers before the
 * first faultable one give the same bits for every map of a fixed input
 * batch, so they run once and later maps start at the first faultable layer.
 * RRAM_EINVAL when a source layer advances between forwards (HDF5Data) or a
 * later layer writes a prefix blob in place.  Re-enable after changing the
 * input batch or a prefix weight (the prefix is recomputed on the next map). */
int rram_mc_set_reuse_prefix(rram_mc_t mc, int enable);
/* hipGraph replay of the maps (opt-in, for launch-bound small nets; no
 * reference counterpart): one map (injection + forward + statistics) is
 * captured after one eager map and replayed per map, the map id and the
 * per-map row advancing in device memory.  Bit-identical to the eager maps;
 * the eager path runs while timing, injection overlap or prefix reuse is on.
 * RRAM_EINVAL for nets whose source layers advance between forwards
 * (HDF5Data).  rram_mc_graph_active: 1 once a graph has been captured. */
int rram_mc_set_graph(rram_mc_t mc, int enable);
int rram_mc_graph_active(rram_mc_t mc, int* active);
int rram_mc_inject_times(rram_mc_t mc, double* ms, long* launches, int64_t* weights, int reset);

/* ------------------------------------------------------ multi-GPU (RCCL)
 * The reference's P2PSync (include/caffe/parallel.hpp; src/caffe/parallel.cpp:
 * 201-437; tools/caffe.cpp:247-249 `P2PSync<float> sync(solver, NULL, param);
 * sync.Run(gpus)`), rebuilt for one process per GPU over RCCL (xGMI).  Each
 * rank creates a communicator from one 128-byte id (rram_comm_unique_id on one
 * rank, handed to the others by the caller: a file, MPI, a TCP store) after
 * selecting its device, then attaches it to its solver with rram_dp_create.
 * librram_caffe.so links librccl.so.1 (the RCCL of the ROCm install, or the one
 * already loaded in the process). */
typedef struct rram_comm_s* rram_comm_t;
typedef struct rram_dp_s* rram_dp_t;
#define RRAM_COMM_ID_BYTES 128
/* ncclGetUniqueId: id[RRAM_COMM_ID_BYTES] */
int rram_comm_unique_id(unsigned char* id);
/* ncclCommInitRank on the calling thread's current device (collective: every
 * rank of the world calls it with the same id) */
int rram_comm_create(const unsigned char* id, int rank, int world, rram_comm_t* out);
int rram_comm_destroy(rram_comm_t c);
int rram_comm_info(rram_comm_t c, int* rank, int* world);
/* in-place sum all-reduce of n device floats, asynchronous on the calling
 * thread's rram_caffe_set_stream stream */
int rram_comm_allreduce_f32(rram_comm_t c, float* buf, int64_t n);
/* in-place all-reduce of n host doubles (op 0 = sum, 1 = max); synchronous */
int rram_comm_allreduce_host_f64(rram_comm_t c, double* vals, int n, int op);
int rram_comm_barrier(rram_comm_t c);
/* P2PSync: broadcasts the solver's parameters from rank 0 now (on_start,
 * parallel.cpp:286-322) and installs the on_gradients_ready hook: the flat
 * gradient buffer (every learnable param aliased into one allocation, the
 * GPUParams layout of parallel.cpp:25-115) is sum-all-reduced and scaled by
 * 1/world (parallel.cpp:324-380) every iteration of rram_solver_step /
 * rram_solver_solve.  overlap != 0 (world > 1, iter_size 1): gradients are
 * reduced in buckets of >= bucket_mb MB started from the per-layer backward
 * hook on a collective stream while earlier layers still run backward; the
 * update waits for them.  Replaces rram_solver_set_gradient_callback /
 * _backward_callback while attached; one per solver.  Destroying the solver
 * first detaches it (rram_dp_destroy then only frees the handle). */
int rram_dp_create(rram_solver_t s, rram_comm_t c, double bucket_mb, int overlap, rram_dp_t* out);
/* the solver's flat learnable data / diff buffers (device pointers, *n
 * floats each; NULL / 0 when the `flat_params: false` option disabled them) */
int rram_solver_flat_params(rram_solver_t s, float** data, float** diff, int64_t* n);
int rram_dp_destroy(rram_dp_t dp);
/* counters: all-reduce rounds (iterations), bucket all-reduces, planned
 * buckets, flat parameter count (nullable outputs) */
int rram_dp_info(rram_dp_t dp, long long* allreduce_calls, long long* bucket_calls, int* buckets, int64_t* params);
/* Host-only (no device): the bucket plan rram_dp_create uses for overlap.
 * nranges[i] [begin, end) flat ranges of layer i's learnable params, packed
 * in `ranges` (2 int64 each, layers in forward order); outputs the buckets in
 * backward order: after layer layer_out[k]'s Backward, all-reduce
 * [lo_out[k], hi_out[k]); the prefix left over goes in on_gradients_ready.
 * *n = 0 when the ranges do not tile the buffer in layer order (shared
 * params).  Needs cap >= the bucket count. */
int rram_dp_plan_buckets(int nlayers, const int* nranges, const int64_t* ranges, int64_t bucket_elems,
                         int* layer_out, int64_t* lo_out, int64_t* hi_out, int cap, int* n);
/* Monte-Carlo job statistics over every rank (map m on rank m mod world):
 * out[0 .. n_outputs) = the output sums, out[n_outputs] = broken cells summed
 * over blobs, out[n_outputs + 1] = maps run, each summed over ranks with one
 * RCCL all-reduce (fp64).  *n = n_outputs + 2 (needs cap >= *n). */
int rram_mc_allreduce_stats(rram_mc_t mc, rram_comm_t c, double* out, int cap, int* n);

#ifdef __cplusplus
}
#endif

#endif /* RRAM_CAFFE_H_ */
