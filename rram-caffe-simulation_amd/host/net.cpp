#include "net.hpp"

#include "hdf5.hpp"

#include <algorithm>
#include <set>
#include <sstream>

namespace caffe {

static bool rule_matches(const Msg& rule, Phase phase) {
  if (rule.has("phase")) {
    const std::string p = rule.str("phase");
    if ((p == "TRAIN") != (phase == TRAIN)) return false;
  }
  // stage / level rules: the configs do not use them; a rule that names a
  // stage never matches the default (stage-less) net state
  if (rule.has("stage") || rule.has("min_level") || rule.has("max_level")) return false;
  return true;
}

Msg FilterNet(const Msg& param, Phase phase) {
  CAFFE_CHECK(!param.has("layers"), "V1 'layers' nets are not supported; upgrade to 'layer' (upgrade_net_proto_text)");
  Msg out;
  for (auto& f : param.fields) {
    if (f.first != "layer") {
      out.fields.push_back(f);
      continue;
    }
    const Msg& l = *f.second.msg;
    auto inc = l.subs("include");
    auto exc = l.subs("exclude");
    CAFFE_CHECK(inc.empty() || exc.empty(), "layer " << l.str("name") << " has both include and exclude rules");
    bool keep = inc.empty();
    for (auto* r : exc)
      if (rule_matches(*r, phase)) keep = false;
    for (auto* r : inc)
      if (rule_matches(*r, phase)) keep = true;
    if (keep) out.fields.push_back(f);
  }
  return out;
}

static std::string split_name(const std::string& blob, const std::string& layer, int top, int k) {
  std::ostringstream o;
  o << blob << "_" << layer << "_" << top << "_split_" << k;
  return o.str();
}

Msg InsertSplits(const Msg& param) {
  // collect layers
  std::vector<std::shared_ptr<Msg>> layers;
  for (auto& f : param.fields)
    if (f.first == "layer") layers.push_back(f.second.msg);
  std::map<std::string, std::pair<int, int>> last_top;
  std::map<std::pair<int, int>, int> consumers;
  std::vector<std::vector<std::pair<int, int>>> src(layers.size());
  for (size_t i = 0; i < layers.size(); ++i) {
    for (auto& b : layers[i]->strs("bottom")) {
      auto it = last_top.find(b);
      CAFFE_CHECK(it != last_top.end(), "Unknown bottom blob '" << b << "' (layer " << layers[i]->str("name") << ")");
      src[i].push_back(it->second);
      consumers[it->second]++;
    }
    auto tops = layers[i]->strs("top");
    for (size_t j = 0; j < tops.size(); ++j) last_top[tops[j]] = {(int)i, (int)j};
  }
  Msg out;
  for (auto& f : param.fields)
    if (f.first != "layer") out.fields.push_back(f);
  std::map<std::pair<int, int>, int> used;
  for (size_t i = 0; i < layers.size(); ++i) {
    Msg l = *layers[i];
    // rename bottoms that read a split source
    int bj = 0;
    for (auto& fld : l.fields) {
      if (fld.first != "bottom") continue;
      auto s = src[i][bj++];
      if (consumers[s] > 1) {
        const Msg& pl = *layers[s.first];
        fld.second.scalar = split_name(pl.strs("top")[s.second], pl.str("name"), s.second, used[s]++);
      }
    }
    Value v;
    v.is_msg = true;
    v.msg = std::make_shared<Msg>(l);
    out.fields.emplace_back("layer", v);
    auto tops = layers[i]->strs("top");
    for (size_t j = 0; j < tops.size(); ++j) {
      const int c = consumers[{(int)i, (int)j}];
      if (c <= 1) continue;
      Msg& sp = out.add_sub("layer");
      const std::string lname = layers[i]->str("name");
      sp.set("name", tops[j] + "_" + lname + "_" + std::to_string(j) + "_split", true);
      sp.set("type", "Split", true);
      Value bv;
      bv.quoted = true;
      bv.scalar = tops[j];
      sp.fields.emplace_back("bottom", bv);
      for (int k = 0; k < c; ++k) {
        Value tv;
        tv.quoted = true;
        tv.scalar = split_name(tops[j], lname, (int)j, k);
        sp.fields.emplace_back("top", tv);
      }
    }
  }
  return out;
}

// Deploy-style top-level inputs (`input:` + `input_shape` / `input_dim`)
static Msg InputsToLayer(const Msg& param) {
  auto inputs = param.strs("input");
  if (inputs.empty()) return param;
  Msg out;
  Msg& il = out.add_sub("layer");
  il.set("name", "input", true);
  il.set("type", "Input", true);
  Msg& ip = il.add_sub("input_param");
  auto shapes = param.subs("input_shape");
  auto dims = param.nums("input_dim");
  for (size_t i = 0; i < inputs.size(); ++i) {
    il.add("top", inputs[i], true);
    Msg& sh = ip.add_sub("shape");
    if (!shapes.empty()) {
      for (double d : shapes[i]->nums("dim")) sh.add("dim", std::to_string((long long)d));
    } else {
      CAFFE_CHECK(dims.size() >= 4 * (i + 1), "input_dim must give 4 dims per input");
      for (int k = 0; k < 4; ++k) sh.add("dim", std::to_string((long long)dims[4 * i + k]));
    }
  }
  for (auto& f : param.fields)
    if (f.first != "input" && f.first != "input_shape" && f.first != "input_dim") out.fields.push_back(f);
  return out;
}

namespace {
// concat_param.axis (or its V1 spelling concat_dim), as ConcatLayer reads it
int canon_axis_of(const Msg& lp) {
  const Msg& cp = lp.sub_or_empty("concat_param");
  const int a = (int)cp.integer("axis", cp.integer("concat_dim", 1));
  return a < 0 ? a + 4 : a;
}
}  // namespace

template <typename Dtype>
Net<Dtype>::Net(const Msg& in_param, Phase phase, const Msg& options) : phase_(phase) {
  Msg param = InsertSplits(FilterNet(InputsToLayer(in_param), phase));
  name_ = param.str("name", "net");
  {
    std::string fl = options.str("fault_layers", "InnerProduct");
    std::stringstream ss(fl);
    std::string t;
    while (std::getline(ss, t, ',')) fault_layer_types_.push_back(t);
  }
  const bool fuse_relu = options.boolean("fuse_relu", true);
  const bool fuse_lrn_pool = options.boolean("fuse_lrn_pool", true);
  const bool fuse_concat = options.boolean("fuse_concat", true);
  const bool fuse_conv_y = options.boolean("fuse_conv_y", true);
  std::vector<int> data_shape;
  {
    std::string ds = options.str("data_shape", "");
    std::stringstream ss(ds);
    std::string t;
    while (std::getline(ss, t, ',')) data_shape.push_back(std::stoi(t));
  }
  std::set<std::string> available;  // produced, not yet consumed
  int lid = 0;
  for (auto* lp_const : param.subs("layer")) {
    Msg lp = *lp_const;
    lp.set("phase", phase == TRAIN ? "TRAIN" : "TEST");
    const std::string type = lp.str("type");
    if (type == "Data" || type == "ImageData" || type == "MemoryData" || type == "WindowData") {
      for (int d : data_shape) lp.add("rram_data_shape", std::to_string(d));
      lp.set("rram_num_classes", options.str("num_classes", "10"));
      lp.set("rram_data_seed", options.str("data_seed", "0"));
    }
    if (type == "HDF5Data") {  // opt-in data-parallel row split (Caffe 1.0's Skip; not the reference's)
      lp.set("rram_solver_rank", options.str("solver_rank", "0"));
      lp.set("rram_solver_count", options.str("solver_count", "1"));
    }
    auto layer = LayerRegistry<Dtype>::CreateLayer(lp);
    layer->layer_id = static_cast<uint32_t>(lid);
    const std::string lname = lp.str("name");
    CAFFE_CHECK(!layer_names_index_.count(lname), "duplicate layer name " << lname);
    layer_names_index_[lname] = lid;
    layer_names_.push_back(lname);
    layers_.push_back(layer);
    bottom_vecs_.emplace_back();
    top_vecs_.emplace_back();
    bottom_id_vecs_.emplace_back();
    top_id_vecs_.emplace_back();
    bottom_need_backward_.emplace_back();
    // bottoms
    auto propagate = lp.nums("propagate_down");
    auto bottoms = lp.strs("bottom");
    bool need_bw = false;
    for (size_t j = 0; j < bottoms.size(); ++j) {
      auto it = blob_names_index_.find(bottoms[j]);
      CAFFE_CHECK(it != blob_names_index_.end(), "Unknown bottom blob '" << bottoms[j] << "' (layer " << lname << ")");
      bottom_vecs_[lid].push_back(blobs_[it->second].get());
      bottom_id_vecs_[lid].push_back(it->second);
      available.erase(bottoms[j]);
      bool nb = blob_need_backward_flag(it->second);
      if (!propagate.empty()) nb = nb && propagate[j] != 0;
      bottom_need_backward_[lid].push_back(nb);
      need_bw = need_bw || nb;
    }
    // tops (in place when a top reuses a bottom name)
    auto tops = lp.strs("top");
    for (size_t j = 0; j < tops.size(); ++j) {
      int id;
      if (j < bottoms.size() && bottoms[j] == tops[j]) {
        id = blob_names_index_[tops[j]];
      } else {
        CAFFE_CHECK(!blob_names_index_.count(tops[j]), "top blob '" << tops[j] << "' produced twice (layer " << lname << ")");
        id = static_cast<int>(blobs_.size());
        blobs_.push_back(std::make_shared<Blob<Dtype>>());
        blob_names_.push_back(tops[j]);
        blob_names_index_[tops[j]] = id;
        blob_need_backward_.push_back(false);
      }
      top_vecs_[lid].push_back(blobs_[id].get());
      top_id_vecs_[lid].push_back(id);
      available.insert(tops[j]);
    }
    // anonymous tops (net.cpp:123-135): not named, so no later layer can read
    // them and they are not net outputs
    if (layer->AutoTopBlobs()) {
      const int needed = std::max(layer->MinTopBlobs(), layer->ExactNumTopBlobs());
      for (int j = static_cast<int>(tops.size()); j < needed; ++j) {
        const int id = static_cast<int>(blobs_.size());
        blobs_.push_back(std::make_shared<Blob<Dtype>>());
        blob_names_.push_back("(automatic)");
        blob_need_backward_.push_back(false);
        top_vecs_[lid].push_back(blobs_[id].get());
        top_id_vecs_[lid].push_back(id);
      }
    }
    layer->SetUp(bottom_vecs_[lid], top_vecs_[lid]);
    for (size_t j = 0; j < top_vecs_[lid].size(); ++j) {
      const float lw = static_cast<float>(layer->loss(static_cast<int>(j)));
      if ((int)blob_loss_weights_.size() <= top_id_vecs_[lid][j]) blob_loss_weights_.resize(top_id_vecs_[lid][j] + 1, 0.f);
      blob_loss_weights_[top_id_vecs_[lid][j]] = lw;
    }
    // params
    auto pspecs = lp.subs("param");
    for (size_t p = 0; p < layer->blobs().size(); ++p) {
      AppendParam(lid, static_cast<int>(p), lp);
      const float lr = p < pspecs.size() ? static_cast<float>(pspecs[p]->num("lr_mult", 1.0)) : 1.0f;
      layer->set_param_propagate_down(static_cast<int>(p), lr != 0.0f);
      need_bw = need_bw || lr != 0.0f;
    }
    layer_need_backward_.push_back(need_bw);
    for (int id : top_id_vecs_[lid]) blob_need_backward_[id] = blob_need_backward_[id] || need_bw;
    // fold an in-place ReLU (slope 0) into the producing Conv / IP epilogue
    if (fuse_relu && type == "ReLU" && lid > 0 && bottoms.size() == 1 && tops.size() == 1 && bottoms[0] == tops[0]) {
      auto* relu = dynamic_cast<ReLULayer<Dtype>*>(layer.get());
      auto& prev = layers_[lid - 1];
      const bool prev_makes_it = top_id_vecs_[lid - 1].size() == 1 && top_id_vecs_[lid - 1][0] == bottom_id_vecs_[lid][0];
      if (relu && relu->negative_slope() == 0.0f && prev_makes_it) {
        if (auto* c = dynamic_cast<ConvolutionLayer<Dtype>*>(prev.get())) {
          c->fused_relu = true;
          relu->folded = true;
        } else if (auto* ip = dynamic_cast<InnerProductLayer<Dtype>*>(prev.get())) {
          ip->fused_relu = true;
          relu->folded = true;
        }
      }
      // a Pooling producer (not itself carrying a folded LRN) stores relu(y)
      if (relu && !relu->folded && prev_makes_it && prev->fuse_relu_after(relu->negative_slope())) relu->folded = true;
    }
    // the backward mirror: a layer whose single bottom is the top of the
    // in-place ReLU right before it applies that ReLU's backward factor
    if (fuse_relu && lid > 0 && bottoms.size() == 1) {
      auto* relu = dynamic_cast<ReLULayer<Dtype>*>(layers_[lid - 1].get());
      if (relu && bottom_vecs_[lid - 1].size() == 1 && top_id_vecs_[lid - 1].size() == 1 &&
          bottom_id_vecs_[lid - 1][0] == top_id_vecs_[lid - 1][0] && top_id_vecs_[lid - 1][0] == bottom_id_vecs_[lid][0] &&
          layer->fuse_relu_before_bwd(relu->negative_slope()))
        relu->bwd_folded = true;
    }
    // TEST phase: fold an ACROSS_CHANNELS LRN into the MAX pool that is the only
    // reader of its top (a second reader would sit behind a Split layer); the
    // LRN top is then never materialised (rram_lrn_maxpool_fwd)
    if (fuse_lrn_pool && phase == TEST && type == "Pooling" && lid > 0 && bottoms.size() == 1) {
      auto& prev = layers_[lid - 1];
      int sz = 0;
      float a = 0.f, b = 0.f, kk = 0.f;
      const bool prev_makes_it = bottom_vecs_[lid - 1].size() == 1 && top_id_vecs_[lid - 1].size() == 1 &&
                                 top_id_vecs_[lid - 1][0] == bottom_id_vecs_[lid][0] &&
                                 bottom_id_vecs_[lid - 1][0] != top_id_vecs_[lid - 1][0];
      if (prev_makes_it && prev->lrn_params(sz, a, b, kk) &&
          layer->fuse_lrn_before(bottom_vecs_[lid - 1][0], sz, a, b, kk)) {
        prev->folded_into_next = true;
        lrn_folds_.push_back({lid - 1, lid, sz, a, b, kk});
      }
    }
    ++lid;
  }
  // force_backward (net.cpp:249-265): every layer runs backward and every
  // bottom its layer allows gets a diff, every param propagates
  if (param.boolean("force_backward", false)) {
    for (size_t l = 0; l < layers_.size(); ++l) {
      layer_need_backward_[l] = true;
      for (size_t j = 0; j < bottom_need_backward_[l].size(); ++j) {
        const bool nb = bottom_need_backward_[l][j] || layers_[l]->AllowForceBackward(static_cast<int>(j));
        bottom_need_backward_[l][j] = nb;
        blob_need_backward_[bottom_id_vecs_[l][j]] = blob_need_backward_[bottom_id_vecs_[l][j]] || nb;
      }
      for (size_t p = 0; p < layers_[l]->blobs().size(); ++p) layers_[l]->set_param_propagate_down(static_cast<int>(p), true);
    }
  }
  // TEST phase: a channel Concat whose bottom is written only by a
  // Convolution (plus its folded in-place ReLU) and read only by the Concat
  // gets that slice written by the Convolution itself (rram_conv2d_fwd_strided)
  // and skips its copy; the bottom blob is then never materialised
  if (fuse_concat && phase == TEST) {
    const int L = static_cast<int>(layers_.size());
    for (int l = 0; l < L; ++l) {
      if (std::string(layers_[l]->type()) != "Concat" || bottom_vecs_[l].size() < 2 || top_vecs_[l].size() != 1)
        continue;
      Blob<Dtype>* ct = top_vecs_[l][0];
      if (ct->num_axes() != 4 || canon_axis_of(layers_[l]->layer_param()) != 1) continue;
      int off = 0;
      for (size_t j = 0; j < bottom_vecs_[l].size(); ++j) {
        const int b = bottom_id_vecs_[l][j];
        const int chans = bottom_vecs_[l][j]->shape(1);
        int writer = -1;
        bool ok = true;
        for (int k = 0; k < L && ok; ++k) {
          const bool reads = std::count(bottom_id_vecs_[k].begin(), bottom_id_vecs_[k].end(), b) > 0;
          const bool writes = std::count(top_id_vecs_[k].begin(), top_id_vecs_[k].end(), b) > 0;
          if (!reads && !writes) continue;
          if (k == l && !writes) continue;                       // the Concat itself
          auto* relu = dynamic_cast<ReLULayer<Dtype>*>(layers_[k].get());
          if (relu && relu->folded) continue;                    // applied in the producer's epilogue
          if (writes && !reads && writer < 0 && dynamic_cast<ConvolutionLayer<Dtype>*>(layers_[k].get())) {
            writer = k;
            continue;
          }
          ok = false;                                            // another reader or writer
        }
        if (ok && writer >= 0 && j < bottom_need_backward_[l].size() &&
            layers_[writer]->write_into_concat(ct, off)) {
          layers_[l]->skip_concat_bottom(static_cast<int>(j), true);
          concat_folds_.push_back({writer, l, static_cast<int>(j), off});
        }
        off += chans;
      }
    }
  }
  // TEST phase: a folded LRN + MAX pool whose top is read by exactly one
  // layer, a Convolution with no other writer of that top in between, writes
  // only the top's octet companion whenever that Convolution reads it (each
  // forward checks: engine and plan as they stand); the fp32 top is then
  // materialised only on demand (materialize_blob; the C-ABI does for every
  // blob it hands out), like a folded LRN's top
#ifndef RRAM_POOL_Y_FOLD  // A/B builds: 0 = the pool always writes its fp32 top
#define RRAM_POOL_Y_FOLD 1
#endif
  if (RRAM_POOL_Y_FOLD && fuse_lrn_pool && phase == TEST) {
    const int L = static_cast<int>(layers_.size());
    for (const LrnFold& f : lrn_folds_) {
      if (top_id_vecs_[f.pool].size() != 1) continue;
      const int t = top_id_vecs_[f.pool][0];
      int reader = -1;
      bool ok = true;
      for (int k = 0; k < L && ok; ++k) {
        if (k == f.pool) continue;
        const bool reads = std::count(bottom_id_vecs_[k].begin(), bottom_id_vecs_[k].end(), t) > 0;
        const bool writes = std::count(top_id_vecs_[k].begin(), top_id_vecs_[k].end(), t) > 0;
        if (writes || (reads && reader >= 0)) ok = false;
        else if (reads) reader = k;
      }
      if (ok && reader > f.pool && bottom_vecs_[reader].size() == 1 &&
          dynamic_cast<ConvolutionLayer<Dtype>*>(layers_[reader].get()) != nullptr &&
          layers_[f.pool]->set_octet_reader(layers_[reader].get()))
        oct_y_folds_.push_back(f.pool);
    }
  }
  // TEST phase, the same for a Convolution producer (the convolution-output
  // fold): its top read only by one Convolution (the producer's folded
  // in-place ReLU aside) is written as the companion alone whenever the
  // producer's epilogue writes it and the reader takes it (each forward
  // checks); AlexNet conv3 -> conv4 and conv4 -> conv5
#ifndef RRAM_CONV_Y_FOLD  // A/B builds: 0 = every convolution writes its fp32 top
#define RRAM_CONV_Y_FOLD 1
#endif
  if (RRAM_CONV_Y_FOLD && fuse_conv_y && phase == TEST) {
    const int L = static_cast<int>(layers_.size());
    for (int l = 0; l < L; ++l) {
      if (dynamic_cast<ConvolutionLayer<Dtype>*>(layers_[l].get()) == nullptr || top_id_vecs_[l].size() != 1)
        continue;
      const int t = top_id_vecs_[l][0];
      int reader = -1;
      bool ok = true;
      for (int k = 0; k < L && ok; ++k) {
        if (k == l) continue;
        const bool reads = std::count(bottom_id_vecs_[k].begin(), bottom_id_vecs_[k].end(), t) > 0;
        const bool writes = std::count(top_id_vecs_[k].begin(), top_id_vecs_[k].end(), t) > 0;
        if (!reads && !writes) continue;
        auto* relu = dynamic_cast<ReLULayer<Dtype>*>(layers_[k].get());
        if (relu && relu->folded && k > l) continue;             // applied in the producer's epilogue
        if (writes || reader >= 0) ok = false;
        else reader = k;
      }
      if (ok && reader > l && bottom_vecs_[reader].size() == 1 &&
          dynamic_cast<ConvolutionLayer<Dtype>*>(layers_[reader].get()) != nullptr &&
          layers_[l]->set_octet_reader(layers_[reader].get()))
        oct_y_folds_.push_back(l);
    }
  }
  for (auto& n : available) {
    const int id = blob_names_index_[n];
    net_output_blobs_.push_back(blobs_[id].get());
    net_output_blob_indices_.push_back(id);
  }
  blob_loss_weights_.resize(blobs_.size(), 0.f);
}

template <typename Dtype>
void Net<Dtype>::materialize_blob(const Blob<Dtype>* b) {
  const size_t folds = concat_folds_.size() + oct_y_folds_.size() + lrn_folds_.size();
  // a captured MC / Solver graph replays the folded launches: undoing a fold
  // must make it recapture (the graph keys include this generation)
  struct Bump {
    const Net* n;
    size_t before;
    ~Bump() {
      if (n->concat_folds_.size() + n->oct_y_folds_.size() + n->lrn_folds_.size() != before)
        Caffe::scratch_gen().fetch_add(1);
    }
  } bump{this, folds};
  for (size_t i = 0; i < concat_folds_.size();) {
    const ConcatFold f = concat_folds_[i];
    Blob<Dtype>* bot = bottom_vecs_[f.concat][f.bottom];
    if (bot != b) {
      ++i;
      continue;
    }
    Blob<Dtype>* ct = top_vecs_[f.concat][0];
    const int inner = static_cast<int>(ct->count(2)), num = ct->shape(0);
    if (bot->count() == (int64_t)num * bot->shape(1) * inner && ct->count() > 0)
      RRAM_CALL(rram_concat_copy(bot->mutable_gpu_data(), ct->mutable_gpu_data(), num, bot->shape(1) * inner,
                                 ct->shape(1) * inner, f.offset * inner, 1, Caffe::stream()));
    layers_[f.writer]->write_into_concat(nullptr, 0);
    layers_[f.concat]->skip_concat_bottom(f.bottom, false);
    concat_folds_.erase(concat_folds_.begin() + static_cast<long>(i));
  }
  for (size_t i = 0; i < oct_y_folds_.size();) {
    const int l = oct_y_folds_[i];
    Blob<Dtype>* t = top_vecs_[l][0];
    if (t != b) {
      ++i;
      continue;
    }
    layers_[l]->set_octet_reader(nullptr);
    if (t->data()->fp32_stale && bottom_vecs_[l][0]->count() > 0) layers_[l]->Forward(bottom_vecs_[l], top_vecs_[l]);
    t->data()->fp32_stale = false;
    oct_y_folds_.erase(oct_y_folds_.begin() + static_cast<long>(i));
  }
  for (size_t i = 0; i < lrn_folds_.size();) {
    const LrnFold f = lrn_folds_[i];
    if (top_vecs_[f.lrn][0] != b) {
      ++i;
      continue;
    }
    layers_[f.pool]->fuse_lrn_before(nullptr, f.size, f.alpha, f.beta, f.k);
    layers_[f.lrn]->folded_into_next = false;
    if (bottom_vecs_[f.lrn][0]->count() > 0) layers_[f.lrn]->Forward(bottom_vecs_[f.lrn], top_vecs_[f.lrn]);
    lrn_folds_.erase(lrn_folds_.begin() + static_cast<long>(i));
  }
}

template <typename Dtype>
void Net<Dtype>::AppendParam(int layer_id, int param_id, const Msg& lp) {
  auto pspecs = lp.subs("param");
  const Msg* spec = param_id < (int)pspecs.size() ? pspecs[param_id] : nullptr;
  const std::string pname = spec ? spec->str("name", "") : "";
  const int net_param_id = static_cast<int>(params_.size());
  params_.push_back(layers_[layer_id]->blobs()[param_id]);
  if ((int)param_id_vecs_.size() <= layer_id) param_id_vecs_.resize(layer_id + 1);
  param_id_vecs_[layer_id].push_back(net_param_id);
  if (!pname.empty() && param_names_index_.count(pname)) {
    // shared parameter: alias the owner's storage (net.cpp:497-540)
    const int owner = param_names_index_[pname];
    param_owners_.push_back(owner);
    CAFFE_CHECK(params_[owner]->count() == params_[net_param_id]->count(), "shared param '" << pname << "' size mismatch");
    params_[net_param_id]->ShareData(*params_[owner]);
    params_[net_param_id]->ShareDiff(*params_[owner]);
    return;
  }
  param_owners_.push_back(-1);
  if (!pname.empty()) param_names_index_[pname] = net_param_id;
  const int learnable_id = static_cast<int>(learnable_params_.size());
  learnable_params_.push_back(params_[net_param_id].get());
  params_lr_.push_back(spec ? static_cast<float>(spec->num("lr_mult", 1.0)) : 1.0f);
  params_weight_decay_.push_back(spec ? static_cast<float>(spec->num("decay_mult", 1.0)) : 1.0f);
  // reference fault registry (net.cpp:482-493): InnerProduct weights + biases
  const std::string type = layers_[layer_id]->type();
  if (std::find(fault_layer_types_.begin(), fault_layer_types_.end(), type) != fault_layer_types_.end()) {
    failure_learnable_params_.push_back(params_[net_param_id].get());
    failure_learnable_layer_ids_.push_back(layer_id);
    failure_learnable_param_ids_.push_back(learnable_id);
    if (type == "InnerProduct" && params_[net_param_id]->num_axes() == 2)
      fc_params_ids_.push_back(static_cast<int>(failure_learnable_params_.size()) - 1);
  }
}

std::string DescribeNet(const Msg& in_param, Phase phase) {
  Msg param = InsertSplits(FilterNet(InputsToLayer(in_param), phase));
  std::ostringstream o;
  auto join = [](const std::vector<std::string>& v) {
    std::string s;
    for (size_t i = 0; i < v.size(); ++i) s += (i ? "," : "") + v[i];
    return s;
  };
  for (auto* l : param.subs("layer"))
    o << l->str("name") << "\t" << l->str("type") << "\t" << join(l->strs("bottom")) << "\t" << join(l->strs("top"))
      << "\n";
  return o.str();
}

template <typename Dtype>
Dtype Net<Dtype>::ForwardFromTo(int start, int end, bool compute_loss) {
  for (int i = start; i <= end; ++i) {
    const bool timed = timing_ == 1 || (timing_ == 2 && !layers_[i]->blobs().empty()) ||
                       (timing_ == 3 && i == timed_layer_);
    if (timed) timer_.start(i);
    layers_[i]->Forward(bottom_vecs_[i], top_vecs_[i]);
    if (timed) timer_.stop(i);
  }
  if (!compute_loss) return Dtype(0);
  // loss = sum over loss tops of weight * value (layer.hpp:451-487); one D2H per loss top
  Dtype loss = 0;
  for (int i = start; i <= end; ++i)
    for (size_t j = 0; j < top_vecs_[i].size(); ++j) {
      const Dtype w = layers_[i]->loss(static_cast<int>(j));
      if (w == Dtype(0)) continue;
      const Blob<Dtype>* t = top_vecs_[i][j];
      std::vector<Dtype> h(t->count());
      HIP_CALL(hipMemcpyAsync(h.data(), t->gpu_data(), t->count() * sizeof(Dtype), hipMemcpyDeviceToHost,
                              Caffe::hip_stream()));
      HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
      for (Dtype v : h) loss += w * v;
    }
  return loss;
}

template <typename Dtype>
Dtype Net<Dtype>::Forward(bool compute_loss) {
  return ForwardFromTo(0, static_cast<int>(layers_.size()) - 1, compute_loss);
}

template <typename Dtype>
void Net<Dtype>::Backward() {
  for (int i = static_cast<int>(layers_.size()) - 1; i >= 0; --i) {
    if (layer_need_backward_[i]) layers_[i]->Backward(top_vecs_[i], bottom_need_backward_[i], bottom_vecs_[i]);
    if (on_backward_layer) on_backward_layer(i);
  }
}

template <typename Dtype>
void Net<Dtype>::Update() {
  for (auto* p : learnable_params_) p->Update();
}

template <typename Dtype>
void Net<Dtype>::ClearParamDiffs(unsigned long long* also, int64_t n_also) {
#ifndef RRAM_ZERO_PAIR  // A/B builds: 0 = the round-5 clears (a memset here, the counters' in FusedTail)
#define RRAM_ZERO_PAIR 1
#endif
  if (flat_diff_ && RRAM_ZERO_PAIR) {  // every learnable diff lives in one buffer: one launch, with the caller's counters
    RRAM_CALL(rram_zero_pair(flat_diff_, flat_param_count(), also, also ? n_also : 0, Caffe::stream()));
    return;
  }
  if (flat_diff_) {
    HIP_CALL(hipMemsetAsync(flat_diff_, 0, flat_param_count() * sizeof(Dtype), Caffe::hip_stream()));
  } else {
    for (auto* p : learnable_params_)
      HIP_CALL(hipMemsetAsync(p->mutable_gpu_diff(), 0, p->count() * sizeof(Dtype), Caffe::hip_stream()));
  }
  if (also && n_also > 0)
    HIP_CALL(hipMemsetAsync(also, 0, n_also * sizeof(unsigned long long), Caffe::hip_stream()));
}

template <typename Dtype>
void Net<Dtype>::ShareTrainedLayersWith(const Net* other) {
  for (size_t i = 0; i < other->layers_.size(); ++i) {
    auto it = layer_names_index_.find(other->layer_names_[i]);
    if (it == layer_names_index_.end()) continue;
    auto& mine = layers_[it->second]->blobs();
    auto& src = other->layers_[i]->blobs();
    CAFFE_CHECK(mine.size() == src.size(), "Incompatible number of blobs for layer " << other->layer_names_[i]);
    for (size_t j = 0; j < mine.size(); ++j) {
      CAFFE_CHECK(mine[j]->shape() == src[j]->shape(), "Cannot share param " << j << " of layer "
                  << other->layer_names_[i] << ": shape mismatch " << mine[j]->shape_string() << " vs " << src[j]->shape_string());
      mine[j]->ShareData(*src[j]);
    }
  }
}

// Blob::FromProto(proto, reshape = false) (blob.cpp:448-496): H2D of data, and
// of diff when the proto carries one.
template <typename Dtype>
void BlobFromProto(Blob<Dtype>* b, const BlobProtoData& p) {
  CAFFE_CHECK((int64_t)p.data.size() == b->count(), "blob data count " << p.data.size() << " != " << b->count());
  HIP_CALL(hipMemcpyAsync(b->mutable_gpu_data(), p.data.data(), p.data.size() * sizeof(Dtype), hipMemcpyHostToDevice,
                          Caffe::hip_stream()));
  if (!p.diff.empty()) {
    CAFFE_CHECK((int64_t)p.diff.size() == b->count(), "blob diff count " << p.diff.size() << " != " << b->count());
    HIP_CALL(hipMemcpyAsync(b->mutable_gpu_diff(), p.diff.data(), p.diff.size() * sizeof(Dtype),
                            hipMemcpyHostToDevice, Caffe::hip_stream()));
  }
  HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));  // the host vectors die with the caller
}

// Blob::ToProto (blob.cpp:518-535)
template <typename Dtype>
BlobProtoData BlobToProto(Blob<Dtype>* b, bool write_diff) {
  BlobProtoData p;
  p.shape.assign(b->shape().begin(), b->shape().end());
  p.data.resize(b->count());
  HIP_CALL(hipMemcpyAsync(p.data.data(), b->gpu_data(), p.data.size() * sizeof(Dtype), hipMemcpyDeviceToHost,
                          Caffe::hip_stream()));
  if (write_diff) {
    p.diff.resize(b->count());
    HIP_CALL(hipMemcpyAsync(p.diff.data(), b->gpu_diff(), p.diff.size() * sizeof(Dtype), hipMemcpyDeviceToHost,
                            Caffe::hip_stream()));
  }
  HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
  return p;
}
template void BlobFromProto<float>(Blob<float>*, const BlobProtoData&);
template BlobProtoData BlobToProto<float>(Blob<float>*, bool);

// net.cpp:765-800: match source layers by name, same blob count, ShapeEquals
template <typename Dtype>
void Net<Dtype>::CopyTrainedLayersFrom(const NetProtoData& param) {
  for (const auto& src : param.layers) {
    auto it = layer_names_index_.find(src.name);
    if (it == layer_names_index_.end()) continue;  // "Ignoring source layer"
    auto& target = layers_[it->second]->blobs();
    CAFFE_CHECK(target.size() == src.blobs.size(), "Incompatible number of blobs for layer " << src.name);
    for (size_t j = 0; j < target.size(); ++j) {
      if (!ShapeEquals(target[j]->shape(), src.blobs[j])) {
        std::ostringstream s;
        for (size_t a = 0; a < src.blobs[j].shape.size(); ++a) s << (a ? " " : "") << src.blobs[j].shape[a];
        throw Error("Cannot copy param " + std::to_string(j) + " weights from layer '" + src.name +
                    "'; shape mismatch.  Source param shape is " + s.str() + "; target param shape is " +
                    target[j]->shape_string());
      }
      BlobFromProto(target[j].get(), src.blobs[j]);
    }
  }
}

// net.cpp:803-818
template <typename Dtype>
void Net<Dtype>::CopyTrainedLayersFrom(const std::string& path) {
  if (path.size() >= 3 && path.compare(path.size() - 3, 3, ".h5") == 0) {
    CopyTrainedLayersFromHDF5(path);
    return;
  }
  CopyTrainedLayersFrom(ParseNetParameter(ReadFileBytes(path)));
}

// net.cpp:819-860 (CopyTrainedLayersFromHDF5).  The reference reshapes the
// target blob to the dataset's dims; here the element count must match (the
// target keeps its shape, so legacy 4-D and N-D forms of one blob both load).
template <typename Dtype>
void Net<Dtype>::CopyTrainedLayersFromHDF5(const std::string& path) {
  h5::Handle file = h5::open_file(path);
  CAFFE_CHECK(h5::link_exists(file.id(), "data"), "Error reading weights from " << path);
  h5::Handle data = h5::open_group(file.id(), "data");
  const int num_layers = h5::num_links(data.id());
  for (int i = 0; i < num_layers; ++i) {
    const std::string name = h5::name_by_idx(data.id(), i);
    auto it = layer_names_index_.find(name);
    if (it == layer_names_index_.end()) continue;  // "Ignoring source layer"
    const int lid = it->second;
    auto& target = layers_[lid]->blobs();
    h5::Handle layer = h5::open_group(data.id(), name);
    CAFFE_CHECK(h5::num_links(layer.id()) <= (int)target.size(), "Incompatible number of blobs for layer " << name);
    for (size_t j = 0; j < target.size(); ++j) {
      const std::string ds = std::to_string(j);
      if (!h5::link_exists(layer.id(), ds)) {
        const int npid = param_id_vecs_[lid][j];
        CAFFE_CHECK(param_owners_[npid] != -1, "Incompatible number of blobs for layer " << name);
        continue;  // weight-shared in the target: the owner's dataset fills it
      }
      std::vector<int64_t> dims;
      BlobProtoData p;
      p.data = h5::load_floats(layer.id(), ds, &dims);
      CAFFE_CHECK((int64_t)p.data.size() == target[j]->count(),
                  "Cannot copy param " << j << " weights from layer '" << name << "'; " << p.data.size()
                                       << " elements, target param shape is " << target[j]->shape_string());
      BlobFromProto(target[j].get(), p);
    }
  }
}

// net.cpp:862-932 (ToHDF5): only params that own themselves are written to
// "data"; "diff" holds every param's gradient when write_diff
template <typename Dtype>
void Net<Dtype>::ToHDF5(const std::string& path, bool write_diff) const {
  h5::Handle file = h5::create_file(path);
  h5::Handle data = h5::create_group(file.id(), "data");
  h5::Handle diff;
  if (write_diff) diff = h5::create_group(file.id(), "diff");
  for (size_t lid = 0; lid < layers_.size(); ++lid) {
    h5::Handle ld = h5::create_group(data.id(), layer_names_[lid]);
    h5::Handle lg;
    if (write_diff) lg = h5::create_group(diff.id(), layer_names_[lid]);
    const auto& blobs = layers_[lid]->blobs();
    for (size_t j = 0; j < blobs.size(); ++j) {
      const int npid = lid < param_id_vecs_.size() && j < param_id_vecs_[lid].size() ? param_id_vecs_[lid][j] : -1;
      const BlobProtoData p = BlobToProto(blobs[j].get(), write_diff);
      const std::vector<int64_t> dims(blobs[j]->shape().begin(), blobs[j]->shape().end());
      if (npid < 0 || param_owners_[npid] == -1) h5::save_floats(ld.id(), std::to_string(j), dims, p.data.data());
      if (write_diff) h5::save_floats(lg.id(), std::to_string(j), dims, p.diff.data());
    }
  }
}

// net.cpp:871-880 / layer.hpp ToProto: name, type, bottoms, tops and blobs of
// every layer (the other LayerParameter fields live in the prototxt)
template <typename Dtype>
NetProtoData Net<Dtype>::ToProto(bool write_diff) const {
  NetProtoData n;
  n.name = name_;
  for (size_t i = 0; i < layers_.size(); ++i) {
    LayerProtoData L;
    L.name = layer_names_[i];
    L.type = layers_[i]->type();
    L.bottom = layers_[i]->layer_param().strs("bottom");
    L.top = layers_[i]->layer_param().strs("top");
    for (auto& b : layers_[i]->blobs()) L.blobs.push_back(BlobToProto(b.get(), write_diff));
    n.layers.push_back(std::move(L));
  }
  return n;
}

template <typename Dtype>
std::shared_ptr<Blob<Dtype>> Net<Dtype>::blob_by_name(const std::string& n) const {
  auto it = blob_names_index_.find(n);
  return it == blob_names_index_.end() ? nullptr : blobs_[it->second];
}
template <typename Dtype>
std::shared_ptr<Layer<Dtype>> Net<Dtype>::layer_by_name(const std::string& n) const {
  auto it = layer_names_index_.find(n);
  return it == layer_names_index_.end() ? nullptr : layers_[it->second];
}

template <typename Dtype>
int64_t Net<Dtype>::flat_param_count() const {
  int64_t n = 0;
  for (auto* p : learnable_params_) n += p->count();
  return n;
}

template <typename Dtype>
void Net<Dtype>::alias_flat_params(Dtype* data, Dtype* diff) {
  int64_t off = 0;
  for (auto* p : learnable_params_) {
    const int64_t n = p->count();
    HIP_CALL(hipMemcpyAsync(data + off, p->gpu_data(), n * sizeof(Dtype), hipMemcpyDeviceToDevice, Caffe::hip_stream()));
    HIP_CALL(hipMemsetAsync(diff + off, 0, n * sizeof(Dtype), Caffe::hip_stream()));
    p->set_gpu_data(data + off);
    p->set_gpu_diff(diff + off);
    off += n;
  }
  flat_diff_ = diff;
  HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
}

template <typename Dtype>
void Net<Dtype>::set_weight_pack_cache(bool on) {
  for (auto& l : layers_)
    if (auto* c = dynamic_cast<ConvolutionLayer<Dtype>*>(l.get())) {
      c->cache_wpack = on;
      if (!on && !c->blobs().empty()) c->blobs()[0]->data()->drop_wpack();
    }
}

template class Net<float>;

}  // namespace caffe
