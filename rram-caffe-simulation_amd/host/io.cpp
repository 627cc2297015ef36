#include "io.hpp"

#include <cstring>
#include <fstream>
#include <iterator>
#include <sstream>

#include "common.hpp"

namespace caffe {
namespace {

enum WireType { kVarint = 0, kFixed64 = 1, kLenDelim = 2, kFixed32 = 5 };

// ----------------------------------------------------------------- reader
struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  Reader(const char* b, size_t n) : p(reinterpret_cast<const uint8_t*>(b)), end(p + n) {}
  bool done() const { return p >= end; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      CAFFE_CHECK(p < end, "protobuf: truncated varint");
      const uint8_t b = *p++;
      v |= static_cast<uint64_t>(b & 0x7F) << s;
      if (!(b & 0x80)) return v;
    }
    throw Error("protobuf: varint longer than 10 bytes");
  }
  Reader sub() {
    const uint64_t n = varint();
    CAFFE_CHECK(n <= static_cast<uint64_t>(end - p), "protobuf: length-delimited field overruns its message");
    Reader r(reinterpret_cast<const char*>(p), static_cast<size_t>(n));
    p += n;
    return r;
  }
  std::string bytes() {
    Reader r = sub();
    return std::string(reinterpret_cast<const char*>(r.p), r.end - r.p);
  }
  uint32_t fixed32() {
    CAFFE_CHECK(end - p >= 4, "protobuf: truncated fixed32");
    uint32_t v;
    std::memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  uint64_t fixed64() {
    CAFFE_CHECK(end - p >= 8, "protobuf: truncated fixed64");
    uint64_t v;
    std::memcpy(&v, p, 8);
    p += 8;
    return v;
  }
  void skip(int wt) {
    switch (wt) {
      case kVarint: varint(); break;
      case kFixed64: fixed64(); break;
      case kLenDelim: sub(); break;
      case kFixed32: fixed32(); break;
      default: throw Error("protobuf: unsupported wire type " + std::to_string(wt));
    }
  }
};

float as_float(uint32_t u) {
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
double as_double(uint64_t u) {
  double d;
  std::memcpy(&d, &u, 8);
  return d;
}

// repeated float: packed (wire type 2) or one element (wire type 5)
void read_floats(Reader& r, int wt, std::vector<float>& out) {
  if (wt == kLenDelim) {
    Reader s = r.sub();
    CAFFE_CHECK((s.end - s.p) % 4 == 0, "protobuf: packed float payload not a multiple of 4");
    const size_t n = (s.end - s.p) / 4;
    const size_t o = out.size();
    if (n == 0) return;  // memcpy with a null destination is UB even for 0 bytes
    out.resize(o + n);
    std::memcpy(out.data() + o, s.p, n * 4);
  } else {
    CAFFE_CHECK(wt == kFixed32, "protobuf: float field with wire type " << wt);
    out.push_back(as_float(r.fixed32()));
  }
}
void read_doubles(Reader& r, int wt, std::vector<float>& out) {
  if (wt == kLenDelim) {
    Reader s = r.sub();
    CAFFE_CHECK((s.end - s.p) % 8 == 0, "protobuf: packed double payload not a multiple of 8");
    while (!s.done()) out.push_back(static_cast<float>(as_double(s.fixed64())));
  } else {
    CAFFE_CHECK(wt == kFixed64, "protobuf: double field with wire type " << wt);
    out.push_back(static_cast<float>(as_double(r.fixed64())));
  }
}

BlobProtoData read_blob(Reader r) {
  BlobProtoData b;
  int64_t legacy[4] = {0, 0, 0, 0};
  bool has_shape = false;
  std::vector<float> ddata, ddiff;
  while (!r.done()) {
    const uint64_t tag = r.varint();
    const int f = static_cast<int>(tag >> 3), wt = static_cast<int>(tag & 7);
    if (f >= 1 && f <= 4 && wt == kVarint) {
      legacy[f - 1] = static_cast<int32_t>(r.varint());
      b.legacy_4d = true;
    } else if (f == 5) {
      read_floats(r, wt, b.data);
    } else if (f == 6) {
      read_floats(r, wt, b.diff);
    } else if (f == 7 && wt == kLenDelim) {
      has_shape = true;
      Reader s = r.sub();
      while (!s.done()) {
        const uint64_t t = s.varint();
        if ((t >> 3) == 1 && (t & 7) == kLenDelim) {
          Reader d = s.sub();
          while (!d.done()) b.shape.push_back(static_cast<int64_t>(d.varint()));
        } else if ((t >> 3) == 1 && (t & 7) == kVarint) {
          b.shape.push_back(static_cast<int64_t>(s.varint()));
        } else {
          s.skip(static_cast<int>(t & 7));
        }
      }
    } else if (f == 8) {
      read_doubles(r, wt, ddata);
    } else if (f == 9) {
      read_doubles(r, wt, ddiff);
    } else {
      r.skip(wt);
    }
  }
  // Blob::FromProto (blob.cpp:448-496): legacy dims win; double_* win over float
  if (b.legacy_4d) b.shape.assign(legacy, legacy + 4);
  else if (!has_shape) b.shape.clear();
  if (!ddata.empty()) b.data = std::move(ddata);
  if (!ddiff.empty()) b.diff = std::move(ddiff);
  return b;
}

const char* v1_type_name(int t) {
  // V1LayerParameter.LayerType (caffe.proto:1258-1300), the types a weight file holds
  switch (t) {
    case 4: return "Convolution";
    case 14: return "InnerProduct";
    case 39: return "Deconvolution";
    case 18: return "ReLU";
    case 17: return "Pooling";
    case 15: return "LRN";
    case 6: return "Dropout";
    case 20: return "Softmax";
    case 21: return "SoftmaxWithLoss";
    case 1: return "Accuracy";
    case 5: return "Data";
    default: return nullptr;
  }
}

LayerProtoData read_layer(Reader r, bool v1) {
  LayerProtoData L;
  L.v1 = v1;
  // field numbers of LayerParameter vs V1LayerParameter
  const int f_name = v1 ? 4 : 1, f_type = v1 ? 5 : 2, f_bottom = v1 ? 2 : 3, f_top = v1 ? 3 : 4,
            f_blobs = v1 ? 6 : 7;
  while (!r.done()) {
    const uint64_t tag = r.varint();
    const int f = static_cast<int>(tag >> 3), wt = static_cast<int>(tag & 7);
    if (f == f_name && wt == kLenDelim) {
      L.name = r.bytes();
    } else if (f == f_type && !v1 && wt == kLenDelim) {
      L.type = r.bytes();
    } else if (f == f_type && v1 && wt == kVarint) {
      const int t = static_cast<int>(r.varint());
      const char* n = v1_type_name(t);
      L.type = n ? n : "V1:" + std::to_string(t);
    } else if (f == f_bottom && wt == kLenDelim) {
      L.bottom.push_back(r.bytes());
    } else if (f == f_top && wt == kLenDelim) {
      L.top.push_back(r.bytes());
    } else if (f == f_blobs && wt == kLenDelim) {
      L.blobs.push_back(read_blob(r.sub()));
    } else {
      r.skip(wt);
    }
  }
  return L;
}

// ----------------------------------------------------------------- writer
struct Writer {
  std::string out;
  void varint(uint64_t v) {
    while (v >= 0x80) {
      out.push_back(static_cast<char>((v & 0x7F) | 0x80));
      v >>= 7;
    }
    out.push_back(static_cast<char>(v));
  }
  void tag(int f, int wt) { varint((static_cast<uint64_t>(f) << 3) | wt); }
  void int_field(int f, int64_t v) {
    tag(f, kVarint);
    varint(static_cast<uint64_t>(v));  // negative int32 → 10-byte two's complement, as protobuf
  }
  void bytes_field(int f, const std::string& s) {
    tag(f, kLenDelim);
    varint(s.size());
    out += s;
  }
  void packed_floats(int f, const std::vector<float>& v) {
    if (v.empty()) return;  // protobuf omits empty packed fields
    tag(f, kLenDelim);
    varint(v.size() * 4);
    out.append(reinterpret_cast<const char*>(v.data()), v.size() * 4);
  }
};

std::string blob_bytes(const BlobProtoData& b) {
  Writer w;
  if (b.legacy_4d) {
    for (int i = 0; i < 4; ++i) w.int_field(i + 1, i < (int)b.shape.size() ? b.shape[i] : 0);
  }
  w.packed_floats(5, b.data);
  w.packed_floats(6, b.diff);
  if (!b.legacy_4d && !b.shape.empty()) {  // Blob::ToProto: a 0-axis blob leaves `shape` unset
    Writer s, d;
    for (int64_t x : b.shape) d.varint(static_cast<uint64_t>(x));
    s.tag(1, kLenDelim);
    s.varint(d.out.size());
    s.out += d.out;
    w.bytes_field(7, s.out);
  }
  return w.out;
}

}  // namespace

NetProtoData ParseNetParameter(const std::string& bytes) {
  NetProtoData n;
  Reader r(bytes.data(), bytes.size());
  while (!r.done()) {
    const uint64_t tag = r.varint();
    const int f = static_cast<int>(tag >> 3), wt = static_cast<int>(tag & 7);
    if (f == 1 && wt == kLenDelim) n.name = r.bytes();
    else if (f == 100 && wt == kLenDelim) n.layers.push_back(read_layer(r.sub(), false));
    else if (f == 2 && wt == kLenDelim) n.layers.push_back(read_layer(r.sub(), true));
    else r.skip(wt);
  }
  return n;
}

std::string SerializeNetParameter(const NetProtoData& net) {
  Writer w;
  if (!net.name.empty()) w.bytes_field(1, net.name);
  for (const auto& L : net.layers) {
    Writer l;
    l.bytes_field(1, L.name);
    l.bytes_field(2, L.type);
    for (auto& b : L.bottom) l.bytes_field(3, b);
    for (auto& t : L.top) l.bytes_field(4, t);
    for (auto& b : L.blobs) l.bytes_field(7, blob_bytes(b));
    w.bytes_field(100, l.out);
  }
  return w.out;
}

SolverStateData ParseSolverState(const std::string& bytes) {
  SolverStateData s;
  Reader r(bytes.data(), bytes.size());
  while (!r.done()) {
    const uint64_t tag = r.varint();
    const int f = static_cast<int>(tag >> 3), wt = static_cast<int>(tag & 7);
    if (f == 1 && wt == kVarint) s.iter = static_cast<int32_t>(r.varint());
    else if (f == 2 && wt == kLenDelim) s.learned_net = r.bytes();
    else if (f == 3 && wt == kLenDelim) s.history.push_back(read_blob(r.sub()));
    else if (f == 4 && wt == kVarint) s.current_step = static_cast<int32_t>(r.varint());
    else r.skip(wt);
  }
  return s;
}

std::string SerializeSolverState(const SolverStateData& st) {
  Writer w;
  w.int_field(1, st.iter);
  w.bytes_field(2, st.learned_net);
  for (auto& h : st.history) w.bytes_field(3, blob_bytes(h));
  w.int_field(4, st.current_step);
  return w.out;
}

std::vector<BlobProtoData> ParseBlobProtoVector(const std::string& bytes) {
  std::vector<BlobProtoData> v;
  Reader r(bytes.data(), bytes.size());
  while (!r.done()) {
    const uint64_t tag = r.varint();
    if ((tag >> 3) == 1 && (tag & 7) == kLenDelim) v.push_back(read_blob(r.sub()));
    else r.skip(static_cast<int>(tag & 7));
  }
  return v;
}

std::string SerializeBlobProtoVector(const std::vector<BlobProtoData>& blobs) {
  Writer w;
  for (auto& b : blobs) w.bytes_field(1, blob_bytes(b));
  return w.out;
}

std::string ReadFileBytes(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  CAFFE_CHECK(f.good(), "cannot open " << path);
  return std::string(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
}

void WriteFileBytes(const std::string& path, const std::string& bytes) {
  std::ofstream f(path, std::ios::binary | std::ios::trunc);
  CAFFE_CHECK(f.good(), "cannot write " << path);
  f.write(bytes.data(), static_cast<std::streamsize>(bytes.size()));
  CAFFE_CHECK(f.good(), "write failed: " << path);
}

bool ShapeEquals(const std::vector<int>& shape, const BlobProtoData& p) {
  if (p.legacy_4d) {
    // LegacyShape(i) for i in -4..-1: 1 for missing leading axes
    if (shape.size() > 4) return false;
    for (int i = 0; i < 4; ++i) {
      const int axis = static_cast<int>(shape.size()) - 4 + i;
      const int64_t d = axis < 0 ? 1 : shape[axis];
      if (d != p.shape[i]) return false;
    }
    return true;
  }
  if (shape.size() != p.shape.size()) return false;
  for (size_t i = 0; i < shape.size(); ++i)
    if (shape[i] != p.shape[i]) return false;
  return true;
}

std::string DescribeNetProto(const NetProtoData& net) {
  std::ostringstream o;
  o.precision(9);
  for (const auto& L : net.layers) {
    for (size_t j = 0; j < L.blobs.size(); ++j) {
      const auto& b = L.blobs[j];
      double sum = 0;
      for (float x : b.data) sum += x;
      o << L.name << '\t' << L.type << '\t' << j << '\t';
      for (size_t a = 0; a < b.shape.size(); ++a) o << (a ? "," : "") << b.shape[a];
      o << '\t' << b.data.size() << '\t' << sum << '\t' << b.diff.size() << '\n';
    }
    if (L.blobs.empty()) o << L.name << '\t' << L.type << "\t-\t\t0\t0\t0\n";
  }
  return o.str();
}

}  // namespace caffe
