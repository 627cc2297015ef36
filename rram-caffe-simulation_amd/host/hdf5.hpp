// HDF5 weights and solver states (src/caffe/util/hdf5.cpp, net.cpp:819-932,
// sgd_solver.cpp:282-351): the reference's .caffemodel.h5 / .solverstate.h5
// layouts, written and read through the HDF5 C library itself (libhdf5 +
// libhdf5_hl, the same H5LT calls the reference makes).  The library is
// loaded at run time (dlopen), so the runtime links and runs without it and
// only the HDF5 paths report a clean error when it is missing.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "io.hpp"

namespace caffe {
namespace h5 {

using hid = int64_t;  // hid_t of HDF5 >= 1.10

// true when libhdf5 / libhdf5_hl could be loaded (RRAM_HDF5_LIB_DIR, the
// default search path, then /opt/conda/lib)
bool available();

// RAII file / group handles (H5Fcreate / H5Fopen / H5Gcreate2 / H5Gopen2)
class Handle {
 public:
  Handle() = default;
  Handle(hid id, int kind) : id_(id), kind_(kind) {}
  Handle(const Handle&) = delete;
  Handle& operator=(const Handle&) = delete;
  Handle(Handle&& o) noexcept : id_(o.id_), kind_(o.kind_) { o.id_ = -1; }
  Handle& operator=(Handle&& o) noexcept {
    if (this != &o) {
      reset();
      id_ = o.id_;
      kind_ = o.kind_;
      o.id_ = -1;
    }
    return *this;
  }
  ~Handle() { reset(); }
  void reset();
  hid id() const { return id_; }

 private:
  hid id_ = -1;
  int kind_ = 0;  // 0 file, 1 group
};

Handle create_file(const std::string& path);     // H5F_ACC_TRUNC
Handle open_file(const std::string& path);       // H5F_ACC_RDONLY
Handle create_group(hid loc, const std::string& name);
Handle open_group(hid loc, const std::string& name);
int num_links(hid group);                        // hdf5_get_num_links
std::string name_by_idx(hid group, int i);       // hdf5_get_name_by_idx (H5_INDEX_NAME, H5_ITER_NATIVE)
bool link_exists(hid loc, const std::string& name);
bool dataset_exists(hid loc, const std::string& name);  // H5LTfind_dataset

// hdf5_save_nd_dataset / hdf5_load_nd_dataset (float or double data read as float)
void save_floats(hid loc, const std::string& name, const std::vector<int64_t>& dims, const float* data);
std::vector<float> load_floats(hid loc, const std::string& name, std::vector<int64_t>* dims);
void save_int(hid loc, const std::string& name, int v);
int load_int(hid loc, const std::string& name);
void save_string(hid loc, const std::string& name, const std::string& s);
std::string load_string(hid loc, const std::string& name);

// A .caffemodel.h5 as NetProtoData (layer names, blobs with shape + data,
// "diff" group when present; LayerParameter types are not stored in HDF5)
NetProtoData read_net(const std::string& path);

}  // namespace h5
}  // namespace caffe
