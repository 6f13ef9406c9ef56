// Strategy file codec: proto2 wire format of src/runtime/strategy.proto (package FFProtoBuf):
//   message Op { required string name = 1; required DeviceType device_type = 2 [default = GPU];
//                repeated int32 dims = 3; repeated int32 device_ids = 4; repeated MemoryType memory_types = 5; }
//   message Strategy { repeated Op ops = 1; }
// Hand-rolled varint codec (no protoc / libprotobuf in the image); reads packed and unpacked
// repeated fields, writes unpacked (proto2 default) exactly like libprotobuf did for the reference.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace flexmi {

struct OpStrategy {
  std::string name;
  int device_type = 0;  // 0 GPU, 1 CPU
  std::vector<int> dims;        // reference internal order: dims[0] innermost, last = sample
  std::vector<int> device_ids;
  std::vector<int> memory_types;  // 0 FBM (HBM), 1 ZCM (pinned host)
  int num_parts() const {
    int n = 1;
    for (int d : dims) n *= d;
    return n;
  }
};

std::string encode_strategy(const std::vector<OpStrategy>& ops);
// returns false on malformed input (err set)
bool decode_strategy(const std::string& bytes, std::vector<OpStrategy>& ops, std::string& err);
bool load_strategy_file(const std::string& path, std::vector<OpStrategy>& ops, std::string& err);
bool save_strategy_file(const std::string& path, const std::vector<OpStrategy>& ops, std::string& err);

}  // namespace flexmi
