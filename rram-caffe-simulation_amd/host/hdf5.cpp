#include "hdf5.hpp"

#include <dlfcn.h>

#include <cstdlib>
#include <mutex>

#include "common.hpp"

namespace caffe {
namespace h5 {
namespace {

// The subset of the HDF5 1.10 C API the reference's util/hdf5.cpp uses.
// hid_t is int64_t, herr_t / htri_t int, hsize_t unsigned long long.
using herr = int;
using hsize = unsigned long long;
struct GroupInfo {  // H5G_info_t
  int storage_type;
  hsize nlinks;
  int64_t max_corder;
  bool mounted;
};
constexpr unsigned kAccRdonly = 0x0000u, kAccTrunc = 0x0002u;  // H5F_ACC_*
constexpr hid kDefault = 0;                                      // H5P_DEFAULT / H5E_DEFAULT
constexpr int kIndexName = 0, kIterNative = 2;                   // H5_INDEX_NAME, H5_ITER_NATIVE
constexpr int kClassInteger = 0, kClassFloat = 1;                // H5T_INTEGER, H5T_FLOAT

struct Api {
  herr (*open)();
  herr (*eset_auto)(hid, void*, void*);
  hid (*fcreate)(const char*, unsigned, hid, hid);
  hid (*fopen)(const char*, unsigned, hid);
  herr (*fclose)(hid);
  hid (*gcreate)(hid, const char*, hid, hid, hid);
  hid (*gopen)(hid, const char*, hid);
  herr (*gclose)(hid);
  herr (*gget_info)(hid, GroupInfo*);
  long (*lget_name_by_idx)(hid, const char*, int, int, hsize, char*, size_t, hid);
  int (*lexists)(hid, const char*, hid);
  // high-level (libhdf5_hl)
  herr (*make_float)(hid, const char*, int, const hsize*, const float*);
  herr (*read_float)(hid, const char*, float*);
  herr (*ndims)(hid, const char*, int*);
  herr (*info)(hid, const char*, hsize*, int*, size_t*);
  herr (*find)(hid, const char*);
  herr (*make_int)(hid, const char*, int, const hsize*, const int*);
  herr (*read_int)(hid, const char*, int*);
  herr (*make_string)(hid, const char*, const char*);
  herr (*read_string)(hid, const char*, char*);
  bool ok = false;
  std::string why;
};

void* open_lib(const char* const* names) {
  const char* dir = std::getenv("RRAM_HDF5_LIB_DIR");
  for (const char* const* n = names; *n; ++n) {
    if (dir) {
      const std::string p = std::string(dir) + "/" + *n;
      if (void* h = dlopen(p.c_str(), RTLD_NOW | RTLD_GLOBAL)) return h;
    }
    if (void* h = dlopen(*n, RTLD_NOW | RTLD_GLOBAL)) return h;
    const std::string conda = std::string("/opt/conda/lib/") + *n;
    if (void* h = dlopen(conda.c_str(), RTLD_NOW | RTLD_GLOBAL)) return h;
  }
  return nullptr;
}

template <typename F>
bool sym(void* lib, const char* name, F& fn, std::string& why) {
  fn = reinterpret_cast<F>(dlsym(lib, name));
  if (!fn) why = std::string("symbol ") + name + " missing";
  return fn != nullptr;
}

const Api& api() {
  static Api a;
  static std::once_flag once;
  std::call_once(once, [] {
    static const char* const core[] = {"libhdf5.so", "libhdf5.so.103", "libhdf5_serial.so", nullptr};
    static const char* const hl[] = {"libhdf5_hl.so", "libhdf5_hl.so.100", "libhdf5_serial_hl.so", nullptr};
    void* c = open_lib(core);
    void* h = c ? open_lib(hl) : nullptr;
    if (!c || !h) {
      a.why = "the HDF5 C library (libhdf5 / libhdf5_hl) could not be loaded; set RRAM_HDF5_LIB_DIR";
      return;
    }
    bool ok = sym(c, "H5open", a.open, a.why) && sym(c, "H5Eset_auto2", a.eset_auto, a.why) &&
              sym(c, "H5Fcreate", a.fcreate, a.why) && sym(c, "H5Fopen", a.fopen, a.why) &&
              sym(c, "H5Fclose", a.fclose, a.why) && sym(c, "H5Gcreate2", a.gcreate, a.why) &&
              sym(c, "H5Gopen2", a.gopen, a.why) && sym(c, "H5Gclose", a.gclose, a.why) &&
              sym(c, "H5Gget_info", a.gget_info, a.why) && sym(c, "H5Lget_name_by_idx", a.lget_name_by_idx, a.why) &&
              sym(c, "H5Lexists", a.lexists, a.why) && sym(h, "H5LTmake_dataset_float", a.make_float, a.why) &&
              sym(h, "H5LTread_dataset_float", a.read_float, a.why) &&
              sym(h, "H5LTget_dataset_ndims", a.ndims, a.why) && sym(h, "H5LTget_dataset_info", a.info, a.why) &&
              sym(h, "H5LTfind_dataset", a.find, a.why) && sym(h, "H5LTmake_dataset_int", a.make_int, a.why) &&
              sym(h, "H5LTread_dataset_int", a.read_int, a.why) &&
              sym(h, "H5LTmake_dataset_string", a.make_string, a.why) &&
              sym(h, "H5LTread_dataset_string", a.read_string, a.why);
    if (ok && a.open() < 0) {
      ok = false;
      a.why = "H5open failed";
    }
    if (ok) a.eset_auto(kDefault, nullptr, nullptr);  // errors come back as status codes, not stderr dumps
    a.ok = ok;
  });
  return a;
}

const Api& need() {
  const Api& a = api();
  CAFFE_CHECK(a.ok, a.why);
  return a;
}

}  // namespace

bool available() { return api().ok; }

void Handle::reset() {
  if (id_ < 0) return;
  const Api& a = api();
  if (a.ok) {
    if (kind_ == 0) (void)a.fclose(id_);
    else (void)a.gclose(id_);
  }
  id_ = -1;
}

Handle create_file(const std::string& path) {
  const hid f = need().fcreate(path.c_str(), kAccTrunc, kDefault, kDefault);
  CAFFE_CHECK(f >= 0, "Couldn't open " << path << " to save weights.");
  return Handle(f, 0);
}
Handle open_file(const std::string& path) {
  const hid f = need().fopen(path.c_str(), kAccRdonly, kDefault);
  CAFFE_CHECK(f >= 0, "Couldn't open " << path);
  return Handle(f, 0);
}
Handle create_group(hid loc, const std::string& name) {
  const hid g = need().gcreate(loc, name.c_str(), kDefault, kDefault, kDefault);
  CAFFE_CHECK(g >= 0, "Error creating HDF5 group " << name);
  return Handle(g, 1);
}
Handle open_group(hid loc, const std::string& name) {
  const hid g = need().gopen(loc, name.c_str(), kDefault);
  CAFFE_CHECK(g >= 0, "Error opening HDF5 group " << name);
  return Handle(g, 1);
}
int num_links(hid group) {
  GroupInfo info{};
  CAFFE_CHECK(need().gget_info(group, &info) >= 0, "Error getting HDF5 group info");
  return static_cast<int>(info.nlinks);
}
std::string name_by_idx(hid group, int i) {
  const Api& a = need();
  const long n = a.lget_name_by_idx(group, ".", kIndexName, kIterNative, static_cast<hsize>(i), nullptr, 0, kDefault);
  CAFFE_CHECK(n >= 0, "Error retrieving HDF5 dataset at index " << i);
  std::string s(static_cast<size_t>(n) + 1, '\0');
  CAFFE_CHECK(a.lget_name_by_idx(group, ".", kIndexName, kIterNative, static_cast<hsize>(i), &s[0], s.size(),
                                 kDefault) >= 0,
              "Error retrieving HDF5 dataset at index " << i);
  s.resize(static_cast<size_t>(n));
  return s;
}
bool link_exists(hid loc, const std::string& name) { return need().lexists(loc, name.c_str(), kDefault) > 0; }
bool dataset_exists(hid loc, const std::string& name) { return need().find(loc, name.c_str()) > 0; }

void save_floats(hid loc, const std::string& name, const std::vector<int64_t>& dims, const float* data) {
  std::vector<hsize> d(dims.begin(), dims.end());
  CAFFE_CHECK(need().make_float(loc, name.c_str(), static_cast<int>(d.size()), d.data(), data) >= 0,
              "Failed to make float dataset " << name);
}

std::vector<float> load_floats(hid loc, const std::string& name, std::vector<int64_t>* dims) {
  const Api& a = need();
  CAFFE_CHECK(a.find(loc, name.c_str()) > 0, "Failed to find HDF5 dataset " << name);
  int nd = 0;
  CAFFE_CHECK(a.ndims(loc, name.c_str(), &nd) >= 0, "Failed to get dataset ndims for " << name);
  CAFFE_CHECK(nd >= 0 && nd <= 32, "dataset " << name << ": " << nd << " axes");  // kMaxBlobAxes
  std::vector<hsize> d(static_cast<size_t>(nd) + 1, 0);
  int cls = -1;
  size_t tsize = 0;
  CAFFE_CHECK(a.info(loc, name.c_str(), d.data(), &cls, &tsize) >= 0, "Failed to get dataset info for " << name);
  CAFFE_CHECK(cls == kClassFloat || cls == kClassInteger,
              "dataset " << name << ": unsupported datatype class " << cls << " (hdf5.cpp:30-55)");
  uint64_t count = 1;
  dims->clear();
  for (int i = 0; i < nd; ++i) {
    dims->push_back(static_cast<int64_t>(d[i]));
    CAFFE_CHECK(d[i] <= (1ull << 40) && count <= (1ull << 40) / (d[i] ? d[i] : 1), "dataset " << name << " too large");
    count *= d[i];
  }
  std::vector<float> out(count);
  CAFFE_CHECK(a.read_float(loc, name.c_str(), out.data()) >= 0, "Failed to read float dataset " << name);
  return out;
}

void save_int(hid loc, const std::string& name, int v) {
  const hsize one = 1;
  CAFFE_CHECK(need().make_int(loc, name.c_str(), 1, &one, &v) >= 0, "Failed to save int dataset with name " << name);
}
int load_int(hid loc, const std::string& name) {
  int v = 0;
  CAFFE_CHECK(need().read_int(loc, name.c_str(), &v) >= 0, "Failed to load int dataset with name " << name);
  return v;
}
void save_string(hid loc, const std::string& name, const std::string& s) {
  CAFFE_CHECK(need().make_string(loc, name.c_str(), s.c_str()) >= 0,
              "Failed to save string dataset with name " << name);
}
std::string load_string(hid loc, const std::string& name) {
  const Api& a = need();
  int cls = -1;
  size_t size = 0;
  CAFFE_CHECK(a.info(loc, name.c_str(), nullptr, &cls, &size) >= 0, "Failed to get dataset info for " << name);
  std::string s(size + 1, '\0');
  CAFFE_CHECK(a.read_string(loc, name.c_str(), &s[0]) >= 0, "Failed to load string dataset with name " << name);
  s.resize(std::char_traits<char>::length(s.c_str()));
  return s;
}

NetProtoData read_net(const std::string& path) {
  NetProtoData net;
  Handle f = open_file(path);
  CAFFE_CHECK(link_exists(f.id(), "data"), "Error reading weights from " << path);
  Handle data = open_group(f.id(), "data");
  const bool has_diff = link_exists(f.id(), "diff");
  Handle diff;
  if (has_diff) diff = open_group(f.id(), "diff");
  const int nl = num_links(data.id());
  for (int i = 0; i < nl; ++i) {
    LayerProtoData L;
    L.name = name_by_idx(data.id(), i);
    L.type = "-";
    Handle lg = open_group(data.id(), L.name);
    Handle dg;
    const bool ld = has_diff && link_exists(diff.id(), L.name);
    if (ld) dg = open_group(diff.id(), L.name);
    const int nb = num_links(lg.id());
    for (int j = 0; j < nb; ++j) {
      const std::string ds = std::to_string(j);
      CAFFE_CHECK(link_exists(lg.id(), ds), "layer " << L.name << ": dataset " << ds << " missing");
      BlobProtoData b;
      b.data = load_floats(lg.id(), ds, &b.shape);
      if (ld && link_exists(dg.id(), ds)) {
        std::vector<int64_t> dd;
        b.diff = load_floats(dg.id(), ds, &dd);
      }
      L.blobs.push_back(std::move(b));
    }
    net.layers.push_back(std::move(L));
  }
  return net;
}

}  // namespace h5
}  // namespace caffe
