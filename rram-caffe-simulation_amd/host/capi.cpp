// extern "C" face of the host runtime (include/rram_caffe.h).  Exceptions
// (the reference's fatal CHECKs) become status codes + a thread-local message.
#include <algorithm>
#include <cstring>
#include <sstream>
#include <string>

#include "rram_caffe.h"
#include "hdf5.hpp"
#include "parallel.hpp"
#include "solver.hpp"

using namespace caffe;

struct rram_net_s {
  std::shared_ptr<Net<float>> net;
};
struct rram_dp_s;
struct rram_solver_s {
  std::unique_ptr<Solver<float>> solver;
  rram_dp_s* dp = nullptr;  // the attached P2PSync (rram_dp_create), detached on destroy
  rram_net_s train;
  std::vector<rram_net_s> tests;
  rram_callback_t grad_cb = nullptr;
  void* grad_user = nullptr;
  rram_layer_callback_t bwd_cb = nullptr;
  void* bwd_user = nullptr;
  rram_log_callback_t log_cb = nullptr;
  void* log_user = nullptr;
};
struct rram_mc_s {
  std::unique_ptr<MonteCarlo<float>> mc;
};
struct rram_syncedmem_s {
  std::unique_ptr<SyncedMemory> mem;
};
struct rram_comm_s {
  std::shared_ptr<Comm> comm;
};
struct rram_dp_s {
  std::unique_ptr<P2PSync<float>> sync;  // reset when its solver goes first
  rram_solver_s* solver = nullptr;
};

static thread_local std::string g_caffe_err;

template <typename F>
static int guarded(F&& f) {
  try {
    f();
    return RRAM_OK;
  } catch (const std::exception& e) {
    g_caffe_err = e.what();
    return RRAM_EINVAL;
  } catch (...) {
    g_caffe_err = "unknown C++ exception";
    return RRAM_EINVAL;
  }
}

#define NEED(p)                                               \
  do {                                                        \
    if (!(p)) throw Error(std::string("NULL argument: ") + #p); \
  } while (0)

static void copy_str(const std::string& s, char* dst, int cap) {
  if (!dst || cap <= 0) return;
  const size_t n = std::min<size_t>(s.size(), (size_t)cap - 1);
  std::memcpy(dst, s.data(), n);
  dst[n] = '\0';
}

static Msg parse_opts(const char* options) { return options ? parse_prototxt(options) : Msg(); }

extern "C" {

const char* rram_caffe_last_error(void) { return g_caffe_err.c_str(); }
int rram_caffe_set_stream(rram_stream_t s) {
  return guarded([&] { Caffe::set_stream(s); });
}
int rram_caffe_set_random_seed(uint64_t seed) {
  return guarded([&] { Caffe::set_random_seed(seed); });
}
int rram_caffe_synchronize(void) {
  return guarded([&] { Caffe::synchronize(); });
}

// ---------------------------------------------------------- SyncedMemory
int rram_syncedmem_create(size_t size, rram_syncedmem_t* out) {
  return guarded([&] {
    NEED(out);
    auto* h = new rram_syncedmem_s;
    h->mem = std::make_unique<SyncedMemory>(size);
    *out = h;
  });
}
int rram_syncedmem_destroy(rram_syncedmem_t m) {
  return guarded([&] { delete m; });
}
int rram_syncedmem_head(rram_syncedmem_t m, int* head) {
  return guarded([&] {
    NEED(m);
    NEED(head);
    *head = static_cast<int>(m->mem->head());
  });
}
int rram_syncedmem_size(rram_syncedmem_t m, size_t* size) {
  return guarded([&] {
    NEED(m);
    NEED(size);
    *size = m->mem->size();
  });
}
int rram_syncedmem_cpu_data(rram_syncedmem_t m, const void** p) {
  return guarded([&] {
    NEED(m);
    NEED(p);
    *p = m->mem->cpu_data();
  });
}
int rram_syncedmem_gpu_data(rram_syncedmem_t m, const void** p) {
  return guarded([&] {
    NEED(m);
    NEED(p);
    *p = m->mem->gpu_data();
  });
}
int rram_syncedmem_mutable_cpu_data(rram_syncedmem_t m, void** p) {
  return guarded([&] {
    NEED(m);
    NEED(p);
    *p = m->mem->mutable_cpu_data();
  });
}
int rram_syncedmem_mutable_gpu_data(rram_syncedmem_t m, void** p) {
  return guarded([&] {
    NEED(m);
    NEED(p);
    *p = m->mem->mutable_gpu_data();
  });
}
int rram_syncedmem_set_cpu_data(rram_syncedmem_t m, void* p) {
  return guarded([&] {
    NEED(m);
    m->mem->set_cpu_data(p);
  });
}
int rram_syncedmem_set_gpu_data(rram_syncedmem_t m, void* p) {
  return guarded([&] {
    NEED(m);
    m->mem->set_gpu_data(p);
  });
}

// ------------------------------------------------------------------- Net
int rram_net_create(const char* txt, int phase, const char* options, rram_net_t* out) {
  return guarded([&] {
    NEED(txt);
    NEED(out);
    auto* h = new rram_net_s;
    try {
      h->net = std::make_shared<Net<float>>(parse_prototxt(txt), phase == RRAM_PHASE_TEST ? TEST : TRAIN,
                                            parse_opts(options));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}
int rram_net_destroy(rram_net_t n) {
  return guarded([&] { delete n; });
}
int rram_net_forward(rram_net_t n, int compute_loss, float* loss) {
  return guarded([&] {
    NEED(n);
    float l = n->net->Forward(compute_loss != 0);
    if (loss) *loss = l;
  });
}
int rram_net_backward(rram_net_t n) {
  return guarded([&] {
    NEED(n);
    n->net->Backward();
  });
}
int rram_net_update(rram_net_t n) {
  return guarded([&] {
    NEED(n);
    n->net->Update();
  });
}
int rram_net_clear_param_diffs(rram_net_t n) {
  return guarded([&] {
    NEED(n);
    n->net->ClearParamDiffs();
  });
}
int rram_net_num_layers(rram_net_t n, int* k) {
  return guarded([&] {
    NEED(n);
    NEED(k);
    *k = (int)n->net->layers().size();
  });
}
int rram_net_layer_info(rram_net_t n, int i, char* name, char* type, int cap, int* np) {
  return guarded([&] {
    NEED(n);
    const auto& L = n->net->layers();
    if (i < 0 || i >= (int)L.size()) throw Error("layer index out of range");
    copy_str(n->net->layer_names()[i], name, cap);
    copy_str(L[i]->type(), type, cap);
    if (np) *np = (int)L[i]->blobs().size();
  });
}
int rram_net_layer_contraction(rram_net_t n, int i, double* flops, int* engine) {
  return guarded([&] {
    NEED(n);
    const auto& L = n->net->layers();
    if (i < 0 || i >= (int)L.size()) throw Error("layer index out of range");
    double f = 0.0;
    int e = -1;
    if (auto* c = dynamic_cast<caffe::ConvolutionLayer<float>*>(L[i].get())) {
      rram_conv_desc d = c->desc();
      if (rram_conv_out_shape(&d) == RRAM_OK) {
        f = 2.0 * d.num * d.num_output * d.out_h * d.out_w * (double)(d.channels / d.group) * d.kernel_h * d.kernel_w;
        e = rram_f32_engine_for_conv(&d);
      }
    } else if (auto* ip = dynamic_cast<caffe::InnerProductLayer<float>*>(L[i].get())) {
      f = 2.0 * ip->M() * (double)ip->N() * ip->K();
      // the workspace InnerProductLayer::Forward_gpu would hand over
      const size_t ws = std::max(caffe::Caffe::workspace_size(),
                                 std::min<size_t>((size_t)16 * ip->M() * ip->N() * sizeof(float), 256ull << 20));
      e = rram_f32_engine_for_ip(ip->M(), ip->N(), ip->K(), ws);
    }
    if (flops) *flops = f;
    if (engine) *engine = e;
  });
}
int rram_net_num_blobs(rram_net_t n, int* k) {
  return guarded([&] {
    NEED(n);
    NEED(k);
    *k = (int)n->net->blobs().size();
  });
}
int rram_net_blob_name(rram_net_t n, int i, char* name, int cap) {
  return guarded([&] {
    NEED(n);
    if (i < 0 || i >= (int)n->net->blob_names().size()) throw Error("blob index out of range");
    copy_str(n->net->blob_names()[i], name, cap);
  });
}
int rram_net_blob(rram_net_t n, const char* name, float** data, float** diff, int* shape, int* naxes) {
  return guarded([&] {
    NEED(n);
    NEED(name);
    auto b = n->net->blob_by_name(name);
    if (!b) throw Error(std::string("Unknown blob name ") + name);
    if (data) {
      // only a data read undoes the blob's folds (a folded Concat bottom /
      // pooled output holds its fp32 values again); diff- or shape-only
      // queries leave the TEST-phase folds in place
      n->net->materialize_blob(b.get());
      *data = b->mutable_gpu_data();
      b->data()->expose();  // the caller may write a new batch through it unseen
    }
    if (diff) *diff = b->mutable_gpu_diff();
    if (naxes) *naxes = b->num_axes();
    if (shape)
      for (int a = 0; a < b->num_axes() && a < 8; ++a) shape[a] = b->shape(a);
  });
}
int rram_net_blob_stale(rram_net_t n, const char* name, int* stale) {
  return guarded([&] {
    NEED(n);
    NEED(name);
    NEED(stale);
    auto b = n->net->blob_by_name(name);
    if (!b) throw Error(std::string("Unknown blob name ") + name);
    *stale = b->data()->fp32_stale ? 1 : 0;
  });
}
int rram_net_num_params(rram_net_t n, int* k) {
  return guarded([&] {
    NEED(n);
    NEED(k);
    *k = (int)n->net->learnable_params().size();
  });
}
int rram_net_param(rram_net_t n, int i, float** data, float** diff, int64_t* count, float* lr, float* dm) {
  return guarded([&] {
    NEED(n);
    const auto& P = n->net->learnable_params();
    if (i < 0 || i >= (int)P.size()) throw Error("param index out of range");
    if (data) {
      *data = P[i]->mutable_gpu_data();
      P[i]->data()->expose();
    }
    if (diff) *diff = P[i]->mutable_gpu_diff();
    if (count) *count = P[i]->count();
    if (lr) *lr = n->net->params_lr()[i];
    if (dm) *dm = n->net->params_weight_decay()[i];
  });
}
int rram_net_num_failure_params(rram_net_t n, int* k) {
  return guarded([&] {
    NEED(n);
    NEED(k);
    *k = (int)n->net->failure_learnable_params().size();
  });
}
int rram_net_failure_param(rram_net_t n, int i, float** data, float** diff, int64_t* count, int* layer_id) {
  return guarded([&] {
    NEED(n);
    const auto& P = n->net->failure_learnable_params();
    if (i < 0 || i >= (int)P.size()) throw Error("failure param index out of range");
    if (data) {
      *data = P[i]->mutable_gpu_data();
      P[i]->data()->expose();
    }
    if (diff) *diff = P[i]->mutable_gpu_diff();
    if (count) *count = P[i]->count();
    if (layer_id) *layer_id = n->net->failure_learnable_layer_ids()[i];
  });
}
int rram_net_num_outputs(rram_net_t n, int* k) {
  return guarded([&] {
    NEED(n);
    NEED(k);
    *k = (int)n->net->output_blobs().size();
  });
}
int rram_net_output(rram_net_t n, int i, char* name, int cap, float** data, int64_t* count) {
  return guarded([&] {
    NEED(n);
    const auto& O = n->net->output_blobs();
    if (i < 0 || i >= (int)O.size()) throw Error("output index out of range");
    copy_str(n->net->blob_names()[n->net->output_blob_indices()[i]], name, cap);
    if (data) *data = O[i]->mutable_gpu_data();
    if (count) *count = O[i]->count();
  });
}
int rram_net_share_trained(rram_net_t dst, rram_net_t src) {
  return guarded([&] {
    NEED(dst);
    NEED(src);
    dst->net->ShareTrainedLayersWith(src->net.get());
  });
}
int rram_net_flat_param_count(rram_net_t n, int64_t* k) {
  return guarded([&] {
    NEED(n);
    NEED(k);
    *k = n->net->flat_param_count();
  });
}
int rram_net_alias_flat_params(rram_net_t n, float* data, float* diff) {
  return guarded([&] {
    NEED(n);
    NEED(data);
    NEED(diff);
    n->net->alias_flat_params(data, diff);
    // the flat buffer is the caller's: writes through it (a broadcast, a
    // torch copy_) bypass every mutable access, so no weight pack is trusted
    for (auto* p : n->net->learnable_params()) p->data()->expose();
  });
}

int rram_net_set_timing(rram_net_t n, int enable) {
  return guarded([&] {
    NEED(n);
    n->net->set_timing(enable == 2 ? 2 : (enable != 0 ? 1 : 0));
  });
}
int rram_net_set_timing_layer(rram_net_t n, int layer) {
  return guarded([&] {
    NEED(n);
    if (layer < 0 || layer >= static_cast<int>(n->net->layers().size()))
      throw Error("set_timing_layer: layer index out of range");
    n->net->set_timing_layer(layer);
  });
}
int rram_net_layer_times(rram_net_t n, double* ms, long* counts, int cap, int* k, int reset) {
  return guarded([&] {
    NEED(n);
    auto& t = n->net->timer();
    t.collect();
    const int L = (int)n->net->layers().size();
    if (k) *k = L;
    for (int i = 0; i < L && i < cap; ++i) {
      auto it = t.totals().find(i);
      auto ic = t.counts().find(i);
      if (ms) ms[i] = it == t.totals().end() ? 0.0 : it->second;
      if (counts) counts[i] = ic == t.counts().end() ? 0 : ic->second;
    }
    if (reset) t.clear();
  });
}
int rram_net_describe(const char* txt, int phase, char* out, size_t cap, size_t* needed) {
  return guarded([&] {
    NEED(txt);
    std::string d = DescribeNet(parse_prototxt(txt), phase == RRAM_PHASE_TEST ? TEST : TRAIN);
    if (needed) *needed = d.size() + 1;
    if (out && cap > 0) {
      const size_t n = std::min(d.size(), cap - 1);
      std::memcpy(out, d.data(), n);
      out[n] = '\0';
    }
  });
}

// ---------------------------------------------------------------- Solver
int rram_solver_create(const char* sp, const char* np, const char* options, rram_solver_t* out) {
  return guarded([&] {
    NEED(sp);
    NEED(out);
    Msg netp;
    if (np) netp = parse_prototxt(np);
    auto* h = new rram_solver_s;
    try {
      h->solver = std::make_unique<Solver<float>>(parse_prototxt(sp), np ? &netp : nullptr, parse_opts(options));
    } catch (...) {
      delete h;
      throw;
    }
    h->train.net = h->solver->net();
    for (auto& t : h->solver->test_nets()) h->tests.push_back(rram_net_s{t});
    *out = h;
  });
}
int rram_solver_destroy(rram_solver_t s) {
  return guarded([&] {
    if (s && s->dp) {  // a P2PSync still attached: detach it (its hooks point into this solver)
      s->dp->sync.reset();
      s->dp->solver = nullptr;
    }
    delete s;
  });
}
int rram_solver_set_graph(rram_solver_t s, int enable) {
  return guarded([&] {
    NEED(s);
    s->solver->set_graph(enable != 0);
  });
}
int rram_solver_graph_active(rram_solver_t s, int* active) {
  return guarded([&] {
    NEED(s);
    NEED(active);
    *active = s->solver->graph_active() ? 1 : 0;
  });
}
int rram_solver_step(rram_solver_t s, int iters) {
  return guarded([&] {
    NEED(s);
    s->solver->Step(iters);
  });
}
int rram_solver_solve(rram_solver_t s) {
  return guarded([&] {
    NEED(s);
    s->solver->Solve();
  });
}
int rram_solver_iter(rram_solver_t s, int* it) {
  return guarded([&] {
    NEED(s);
    NEED(it);
    *it = s->solver->iter();
  });
}
int rram_solver_smoothed_loss(rram_solver_t s, float* l) {
  return guarded([&] {
    NEED(s);
    NEED(l);
    *l = s->solver->smoothed_loss();
  });
}
int rram_solver_learning_rate(rram_solver_t s, float* lr) {
  return guarded([&] {
    NEED(s);
    NEED(lr);
    *lr = s->solver->GetLearningRate();
  });
}
int rram_solver_net(rram_solver_t s, rram_net_t* n) {
  return guarded([&] {
    NEED(s);
    NEED(n);
    *n = &s->train;
  });
}
int rram_solver_num_test_nets(rram_solver_t s, int* n) {
  return guarded([&] {
    NEED(s);
    NEED(n);
    *n = (int)s->tests.size();
  });
}
int rram_solver_test_net(rram_solver_t s, int i, rram_net_t* n) {
  return guarded([&] {
    NEED(s);
    NEED(n);
    if (i < 0 || i >= (int)s->tests.size()) throw Error("test net index out of range");
    *n = &s->tests[i];
  });
}
int rram_solver_test(rram_solver_t s, int t, float* scores, int cap, int* n) {
  return guarded([&] {
    NEED(s);
    auto r = s->solver->Test(t);
    if (n) *n = (int)r.size();
    for (int i = 0; i < (int)r.size() && i < cap && scores; ++i) scores[i] = r[i];
  });
}
int rram_solver_set_gradient_callback(rram_solver_t s, rram_callback_t cb, void* user) {
  return guarded([&] {
    NEED(s);
    s->grad_cb = cb;
    s->grad_user = user;
    if (cb) s->solver->on_gradients_ready = [s] { s->grad_cb(s->grad_user); };
    else s->solver->on_gradients_ready = nullptr;
  });
}
int rram_solver_set_backward_callback(rram_solver_t s, rram_layer_callback_t cb, void* user) {
  return guarded([&] {
    NEED(s);
    s->bwd_cb = cb;
    s->bwd_user = user;
    if (cb) s->solver->net()->on_backward_layer = [s](int i) { s->bwd_cb(i, s->bwd_user); };
    else s->solver->net()->on_backward_layer = nullptr;
  });
}
int rram_solver_set_log_callback(rram_solver_t s, rram_log_callback_t cb, void* user) {
  return guarded([&] {
    NEED(s);
    s->log_cb = cb;
    s->log_user = user;
    if (cb) s->solver->log = [s](const std::string& l) { s->log_cb(l.c_str(), s->log_user); };
    else s->solver->log = nullptr;
  });
}
int rram_solver_num_fail_blobs(rram_solver_t s, int* n) {
  return guarded([&] {
    NEED(s);
    NEED(n);
    auto fm = s->solver->failure_maker();
    *n = fm ? (int)fm->fail_iterations().size() : 0;
  });
}
int rram_solver_fail_state(rram_solver_t s, int i, float** e, float** v, int64_t* count) {
  return guarded([&] {
    NEED(s);
    auto fm = s->solver->failure_maker();
    if (!fm) throw Error("solver has no failure_pattern");
    auto fi = fm->fail_iterations();
    if (i < 0 || i >= (int)fi.size()) throw Error("fail blob index out of range");
    if (e) *e = fi[i]->mutable_gpu_data();
    if (v) *v = fi[i]->mutable_gpu_diff();
    if (count) *count = fi[i]->count();
  });
}
int rram_solver_num_history(rram_solver_t s, int* n) {
  return guarded([&] {
    NEED(s);
    NEED(n);
    *n = (int)s->solver->history().size();
  });
}
int rram_solver_history(rram_solver_t s, int i, float** data, int64_t* count) {
  return guarded([&] {
    NEED(s);
    const auto& h = s->solver->history();
    if (i < 0 || i >= (int)h.size()) throw Error("history index out of range");
    if (data) *data = h[i]->mutable_gpu_data();
    if (count) *count = h[i]->count();
  });
}
int rram_solver_broken_counts(rram_solver_t s, unsigned long long* out, int cap, int* n) {
  return guarded([&] {
    NEED(s);
    auto fm = s->solver->failure_maker();
    std::vector<unsigned long long> c = fm ? fm->broken_counts() : std::vector<unsigned long long>();
    if (n) *n = (int)c.size();
    for (int i = 0; i < (int)c.size() && i < cap && out; ++i) out[i] = c[i];
  });
}

int rram_solver_apply_strategies(rram_solver_t s) {
  return guarded([&] {
    NEED(s);
    for (auto& st : s->solver->strategies()) st->Apply();
  });
}
int rram_solver_strategy_info(rram_solver_t s, int i, char* type, int cap, int* a, int* b, int* c) {
  return guarded([&] {
    NEED(s);
    const auto& v = s->solver->strategies();
    if (i < 0 || i >= (int)v.size()) throw Error("strategy index out of range");
    copy_str(v[i]->type(), type, cap);
    int x = 0, y = 0, z = 0;
    if (auto* g = dynamic_cast<GeneticFailureStrategy<float>*>(v[i].get())) {
      x = g->last_before();
      y = g->last_after();
      z = g->last_accepted();
    }
    if (a) *a = x;
    if (b) *b = y;
    if (c) *c = z;
  });
}
int rram_solver_snapshot(rram_solver_t s, char* path_out, int cap) {
  return guarded([&] {
    NEED(s);
    copy_str(s->solver->Snapshot(), path_out, cap);
  });
}
int rram_solver_restore(rram_solver_t s, const char* state_file) {
  return guarded([&] {
    NEED(s);
    NEED(state_file);
    s->solver->Restore(state_file);
  });
}
int rram_solver_solve_from(rram_solver_t s, const char* resume_file) {
  return guarded([&] {
    NEED(s);
    s->solver->Solve(resume_file);
  });
}

// ------------------------------------------------------------ weight files
int rram_net_copy_trained_layers_from(rram_net_t n, const char* path) {
  return guarded([&] {
    NEED(n);
    NEED(path);
    n->net->CopyTrainedLayersFrom(std::string(path));
  });
}
int rram_net_save_weights(rram_net_t n, const char* path, int write_diff) {
  return guarded([&] {
    NEED(n);
    NEED(path);
    const std::string p(path);
    if (p.size() >= 3 && p.compare(p.size() - 3, 3, ".h5") == 0) n->net->ToHDF5(p, write_diff != 0);
    else WriteFileBytes(p, SerializeNetParameter(n->net->ToProto(write_diff != 0)));
  });
}
int rram_caffemodel_describe(const char* path, char* out, size_t cap, size_t* needed) {
  return guarded([&] {
    NEED(path);
    const std::string p(path);
    const bool h5file = p.size() >= 3 && p.compare(p.size() - 3, 3, ".h5") == 0;
    const std::string d = DescribeNetProto(h5file ? h5::read_net(p) : ParseNetParameter(ReadFileBytes(p)));
    if (needed) *needed = d.size() + 1;
    if (out && cap > 0) {
      const size_t k = std::min(d.size(), cap - 1);
      std::memcpy(out, d.data(), k);
      out[k] = '\0';
    }
  });
}
int rram_proto_rewrite(const char* in, const char* out, int kind) {
  return guarded([&] {
    NEED(in);
    NEED(out);
    const std::string b = ReadFileBytes(in);
    if (kind == 0) WriteFileBytes(out, SerializeNetParameter(ParseNetParameter(b)));
    else if (kind == 1) WriteFileBytes(out, SerializeSolverState(ParseSolverState(b)));
    else if (kind == 2) WriteFileBytes(out, SerializeBlobProtoVector(ParseBlobProtoVector(b)));
    else throw Error("rram_proto_rewrite: kind must be 0, 1 or 2");
  });
}
int rram_solver_describe(const char* solver_prototxt, char* out, size_t cap, size_t* needed) {
  return guarded([&] {
    NEED(solver_prototxt);
    const Msg sp = parse_prototxt(solver_prototxt);
    std::ostringstream o;
    o.precision(9);
    // caffe.proto defaults (FailurePatternParameter :252-262, FailureProbParameter :264-268,
    // FailureStrategyParameter :271-290)
    if (const Msg* fp = sp.sub("failure_pattern")) {
      const Msg& pr = fp->sub_or_empty("failure_prob");
      o << "failure_pattern\t" << fp->str("type", "gaussian") << '\t' << fp->num("mean", 10000) << '\t'
        << fp->num("std", 100) << '\t' << pr.integer("neg", 10) << '\t' << pr.integer("zero", 20) << '\t'
        << pr.integer("pos", 10) << '\n';
    }
    for (const Msg* st : sp.subs("failure_strategy")) {
      o << "failure_strategy\t" << st->str("type") << '\t' << st->num("threshold", 0.001) << '\t'
        << st->integer("start", 0) << '\t' << st->integer("period", 100) << '\t' << st->str("prune_order_file")
        << '\t' << st->integer("switch_time", 100) << '\t' << st->str("prune_net_file") << '\t'
        << st->str("prune_model_file") << '\n';
    }
    o << "solver\t" << sp.str("lr_policy", "fixed") << '\t' << sp.num("base_lr", 0.01) << '\t'
      << sp.integer("max_iter", 0) << '\t' << sp.integer("snapshot", 0) << '\t' << sp.str("snapshot_prefix") << '\n';
    const std::string d = o.str();
    if (needed) *needed = d.size() + 1;
    if (out && cap > 0) {
      const size_t k = std::min(d.size(), cap - 1);
      std::memcpy(out, d.data(), k);
      out[k] = '\0';
    }
  });
}
int rram_glibc_rand(uint32_t seed, int n, int* out) {
  return guarded([&] {
    if (n < 0) throw Error("n < 0");
    if (n > 0) NEED(out);
    GlibcRand r(seed);
    for (int i = 0; i < n; ++i) out[i] = r();
  });
}

// ----------------------------------------------------------- Monte-Carlo
int rram_mc_create(rram_net_t net, const rram_inject_cfg* cfgs, int ncfg, uint64_t seed, int max_maps,
                   rram_mc_t* out) {
  return guarded([&] {
    NEED(net);
    NEED(cfgs);
    NEED(out);
    if (ncfg < 1) throw Error("rram_mc_create: ncfg must be >= 1");
    std::vector<rram_inject_cfg> v(cfgs, cfgs + ncfg);
    auto* h = new rram_mc_s;
    try {
      h->mc = std::make_unique<MonteCarlo<float>>(net->net, v, seed, max_maps);
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}
int rram_mc_destroy(rram_mc_t m) {
  return guarded([&] { delete m; });
}
int rram_mc_run(rram_mc_t m, uint32_t begin, uint32_t count) {
  return guarded([&] {
    NEED(m);
    m->mc->Run(begin, count);
  });
}
int rram_mc_reset(rram_mc_t m) {
  return guarded([&] {
    NEED(m);
    m->mc->Reset();
  });
}
int rram_mc_restore_clean(rram_mc_t m) {
  return guarded([&] {
    NEED(m);
    m->mc->RestoreClean();
  });
}
int rram_mc_set_reuse_prefix(rram_mc_t m, int enable) {
  return guarded([&] {
    NEED(m);
    m->mc->set_reuse_prefix(enable != 0);
  });
}
int rram_mc_set_graph(rram_mc_t m, int enable) {
  return guarded([&] {
    NEED(m);
    m->mc->set_graph(enable != 0);
  });
}
int rram_mc_graph_active(rram_mc_t m, int* active) {
  return guarded([&] {
    NEED(m);
    NEED(active);
    *active = m->mc->graph_active() ? 1 : 0;
  });
}
int rram_mc_set_timing(rram_mc_t m, int enable) {
  return guarded([&] {
    NEED(m);
    m->mc->set_timing(enable != 0);
  });
}
int rram_mc_inject_times(rram_mc_t m, double* ms, long* launches, int64_t* weights, int reset) {
  return guarded([&] {
    NEED(m);
    auto& t = m->mc->timer();
    t.collect();
    auto it = t.totals().find(0);
    auto ic = t.counts().find(0);
    if (ms) *ms = it == t.totals().end() ? 0.0 : it->second;
    if (launches) *launches = ic == t.counts().end() ? 0 : ic->second;
    if (weights) *weights = m->mc->fault_weights();
    if (reset) t.clear();
  });
}
int rram_mc_stats(rram_mc_t m, double* sums, int sums_cap, int* n_out, unsigned long long* broken, int bcap,
                  int* n_blobs, float* per_map, int pcap, int* maps_run) {
  return guarded([&] {
    NEED(m);
    std::vector<double> o;
    std::vector<unsigned long long> b;
    std::vector<float> pm;
    m->mc->Stats(o, b, pm);
    if (n_out) *n_out = (int)o.size();
    if (n_blobs) *n_blobs = (int)b.size();
    if (maps_run) *maps_run = m->mc->maps_run();
    for (int i = 0; sums && i < (int)o.size() && i < sums_cap; ++i) sums[i] = o[i];
    for (int i = 0; broken && i < (int)b.size() && i < bcap; ++i) broken[i] = b[i];
    for (int i = 0; per_map && i < (int)pm.size() && i < pcap; ++i) per_map[i] = pm[i];
  });
}


// ------------------------------------------------------------ multi-GPU
int rram_comm_unique_id(unsigned char* id) {
  return guarded([&] {
    NEED(id);
    Comm::unique_id(id);
  });
}
int rram_comm_create(const unsigned char* id, int rank, int world, rram_comm_t* out) {
  return guarded([&] {
    NEED(id);
    NEED(out);
    auto* c = new rram_comm_s;
    try {
      c->comm = std::make_shared<Comm>(id, rank, world);
    } catch (...) {
      delete c;
      throw;
    }
    *out = c;
  });
}
int rram_comm_destroy(rram_comm_t c) {
  return guarded([&] { delete c; });
}
int rram_comm_info(rram_comm_t c, int* rank, int* world) {
  return guarded([&] {
    NEED(c);
    if (rank) *rank = c->comm->rank();
    if (world) *world = c->comm->world();
  });
}
int rram_comm_allreduce_f32(rram_comm_t c, float* buf, int64_t n) {
  return guarded([&] {
    NEED(c);
    if (n > 0) NEED(buf);
    c->comm->allreduce_f32(buf, n, Caffe::hip_stream());
  });
}
int rram_comm_allreduce_host_f64(rram_comm_t c, double* vals, int n, int op) {
  return guarded([&] {
    NEED(c);
    if (n > 0) NEED(vals);
    c->comm->allreduce_host_f64(vals, n, op);
  });
}
int rram_comm_barrier(rram_comm_t c) {
  return guarded([&] {
    NEED(c);
    c->comm->barrier();
  });
}
int rram_dp_create(rram_solver_t s, rram_comm_t c, double bucket_mb, int overlap, rram_dp_t* out) {
  return guarded([&] {
    NEED(s);
    NEED(c);
    NEED(out);
    CAFFE_CHECK(bucket_mb > 0, "rram_dp_create: bucket_mb must be > 0");
    // (refused before any hook is touched: the attached sync keeps its own)
    CAFFE_CHECK(s->dp == nullptr, "rram_dp_create: the solver already has a P2PSync attached");
    // the sync owns both hooks while attached
    s->grad_cb = nullptr;
    s->bwd_cb = nullptr;
    s->solver->on_gradients_ready = nullptr;
    s->solver->net()->on_backward_layer = nullptr;
    auto* d = new rram_dp_s;
    try {
      d->sync = std::make_unique<P2PSync<float>>(s->solver.get(), c->comm, bucket_mb, overlap != 0);
    } catch (...) {
      delete d;
      throw;
    }
    d->solver = s;
    s->dp = d;
    *out = d;
  });
}
int rram_solver_flat_params(rram_solver_t s, float** data, float** diff, int64_t* n) {
  return guarded([&] {
    NEED(s);
    float* d = s->solver->flat_data();
    if (data) *data = d;
    if (diff) *diff = s->solver->flat_diff();
    if (n) *n = d ? s->solver->net()->flat_param_count() : 0;
  });
}
int rram_dp_destroy(rram_dp_t dp) {
  return guarded([&] {
    if (dp && dp->solver) dp->solver->dp = nullptr;
    delete dp;
  });
}
int rram_dp_info(rram_dp_t dp, long long* allreduce_calls, long long* bucket_calls, int* buckets, int64_t* params) {
  return guarded([&] {
    NEED(dp);
    CAFFE_CHECK(dp->sync != nullptr, "rram_dp_info: the P2PSync's solver was destroyed");
    if (allreduce_calls) *allreduce_calls = dp->sync->allreduce_calls();
    if (bucket_calls) *bucket_calls = dp->sync->bucket_calls();
    if (buckets) *buckets = dp->sync->buckets();
    if (params) *params = dp->sync->params();
  });
}
int rram_dp_plan_buckets(int nlayers, const int* nranges, const int64_t* ranges, int64_t bucket_elems,
                         int* layer_out, int64_t* lo_out, int64_t* hi_out, int cap, int* n) {
  return guarded([&] {
    NEED(n);
    CAFFE_CHECK(nlayers >= 0 && bucket_elems > 0, "rram_dp_plan_buckets: bad arguments");
    if (nlayers > 0) NEED(nranges);
    std::vector<std::vector<std::pair<int64_t, int64_t>>> rs(nlayers);
    int k = 0;
    for (int i = 0; i < nlayers; ++i)
      for (int j = 0; j < nranges[i]; ++j, ++k) rs[i].push_back({ranges[2 * k], ranges[2 * k + 1]});
    const auto plan = plan_buckets(rs, bucket_elems);
    *n = static_cast<int>(plan.size());
    CAFFE_CHECK(cap >= *n || plan.empty(), "rram_dp_plan_buckets: cap " << cap << " < " << *n);
    for (size_t b = 0; b < plan.size(); ++b) {
      if (layer_out) layer_out[b] = plan[b].first;
      if (lo_out) lo_out[b] = plan[b].second.first;
      if (hi_out) hi_out[b] = plan[b].second.second;
    }
  });
}
int rram_mc_allreduce_stats(rram_mc_t m, rram_comm_t c, double* out, int cap, int* n) {
  return guarded([&] {
    NEED(m);
    NEED(c);
    NEED(out);
    std::vector<double> o;
    std::vector<unsigned long long> b;
    std::vector<float> pm;
    m->mc->Stats(o, b, pm);
    unsigned long long broken = 0;
    for (auto x : b) broken += x;
    o.push_back(static_cast<double>(broken));
    o.push_back(static_cast<double>(m->mc->maps_run()));
    if (n) *n = static_cast<int>(o.size());
    CAFFE_CHECK(cap >= static_cast<int>(o.size()), "rram_mc_allreduce_stats: cap " << cap << " < " << o.size());
    c->comm->allreduce_host_f64(o.data(), static_cast<int>(o.size()), 0);
    std::copy(o.begin(), o.end(), out);
  });
}

}  // extern "C"
