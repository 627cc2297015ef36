// Binary protobuf codec for the three Caffe files the fault path reads and
// writes: NetParameter weights (.caffemodel), SolverState
// (.solverstate) and the fault-state snapshot this build adds (Appendix A Q11).
//
// No libprotobuf on the target, so this is a hand-written wire-format
// reader/writer restricted to the fields those files carry (caffe.proto):
//   BlobProto        shape=7 (BlobShape dim=1, packed int64), data=5, diff=6
//                    (packed float), double_data=8, double_diff=9, legacy
//                    num/channels/height/width=1..4
//   LayerParameter   name=1, type=2, bottom=3, top=4, blobs=7
//   V1LayerParameter bottom=2, top=3, name=4, type=5 (enum), blobs=6
//   NetParameter     name=1, layers=2 (V1), layer=100
//   SolverState      iter=1, learned_net=2, history=3, current_step=4
// Writers emit fields in field-number order with packed repeated scalars,
// which is what protobuf's own serializer produces for the same content.
// Unknown fields are skipped on read (any wire type), as protobuf does.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace caffe {

struct BlobProtoData {
  std::vector<int64_t> shape;  // from `shape`, or num/channels/height/width when legacy
  bool legacy_4d = false;
  std::vector<float> data, diff;  // double_data / double_diff converted to float
};

struct LayerProtoData {
  std::string name, type;
  std::vector<std::string> bottom, top;
  std::vector<BlobProtoData> blobs;
  bool v1 = false;  // came from NetParameter.layers (V1LayerParameter)
};

struct NetProtoData {
  std::string name;
  std::vector<LayerProtoData> layers;  // `layer` and upgraded V1 `layers`, file order
};

struct SolverStateData {
  int32_t iter = 0;
  std::string learned_net;
  std::vector<BlobProtoData> history;
  int32_t current_step = 0;
};

// Byte-level codecs (throw caffe::Error on malformed input).
NetProtoData ParseNetParameter(const std::string& bytes);
std::string SerializeNetParameter(const NetProtoData& net);
SolverStateData ParseSolverState(const std::string& bytes);
std::string SerializeSolverState(const SolverStateData& st);
// BlobProtoVector (blobs=1): the fault-state snapshot, one BlobProto per
// faultable blob with data = endurance and diff = stuck value.
std::vector<BlobProtoData> ParseBlobProtoVector(const std::string& bytes);
std::string SerializeBlobProtoVector(const std::vector<BlobProtoData>& blobs);

std::string ReadFileBytes(const std::string& path);
void WriteFileBytes(const std::string& path, const std::string& bytes);

// Blob::ShapeEquals (blob.cpp:400-420): legacy 4-D protos compare against the
// blob's LegacyShape (padded with leading 1s, at most 4 axes).
bool ShapeEquals(const std::vector<int>& blob_shape, const BlobProtoData& p);

// Text dump for tests / debugging: one line per blob
// "layer\ttype\tindex\tshape\tcount\tdata_sum\tdiff_count".
std::string DescribeNetProto(const NetProtoData& net);

}  // namespace caffe
