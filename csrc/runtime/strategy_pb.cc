// Strategy file codec (see strategy_pb.h).  Semantics of src/runtime/strategy.cc:96-172:
// every op is {name, device type, partition degrees, device ids}; device_ids may be empty
// (reference asserts n == ids or ids == 0); duplicate names are an error.
#include "strategy_pb.h"

#include <fstream>
#include <set>
#include <sstream>

namespace flexmi {
namespace {

void put_varint(std::string& out, uint64_t v) {
  while (v >= 0x80) {
    out.push_back(static_cast<char>((v & 0x7F) | 0x80));
    v >>= 7;
  }
  out.push_back(static_cast<char>(v));
}

void put_tag(std::string& out, int field, int wt) { put_varint(out, (uint64_t)((field << 3) | wt)); }

void put_int32(std::string& out, int field, int32_t v) {
  put_tag(out, field, 0);
  put_varint(out, (uint64_t)(int64_t)v);  // negative int32 -> 10-byte varint (proto semantics)
}

bool get_varint(const std::string& b, size_t& i, uint64_t& v) {
  v = 0;
  int shift = 0;
  while (i < b.size()) {
    uint8_t c = (uint8_t)b[i++];
    v |= (uint64_t)(c & 0x7F) << shift;
    if (!(c & 0x80)) return true;
    shift += 7;
    if (shift > 63) return false;
  }
  return false;
}

bool skip_field(const std::string& b, size_t& i, int wt) {
  uint64_t v;
  switch (wt) {
    case 0: return get_varint(b, i, v);
    case 1: i += 8; return i <= b.size();
    case 2:
      if (!get_varint(b, i, v)) return false;
      i += v;
      return i <= b.size();
    case 5: i += 4; return i <= b.size();
    default: return false;
  }
}

bool decode_op(const std::string& b, OpStrategy& op, std::string& err) {
  size_t i = 0;
  bool has_name = false;
  while (i < b.size()) {
    uint64_t key;
    if (!get_varint(b, i, key)) { err = "truncated key"; return false; }
    int field = (int)(key >> 3), wt = (int)(key & 7);
    if (field == 1 && wt == 2) {
      uint64_t n;
      if (!get_varint(b, i, n) || i + n > b.size()) { err = "bad name"; return false; }
      op.name = b.substr(i, n);
      i += n;
      has_name = true;
    } else if (field == 2 && wt == 0) {
      uint64_t v;
      if (!get_varint(b, i, v)) { err = "bad device_type"; return false; }
      op.device_type = (int)v;
    } else if ((field == 3 || field == 4 || field == 5) && (wt == 0 || wt == 2)) {
      std::vector<int>& dst = field == 3 ? op.dims : field == 4 ? op.device_ids : op.memory_types;
      if (wt == 0) {
        uint64_t v;
        if (!get_varint(b, i, v)) { err = "bad repeated"; return false; }
        dst.push_back((int)(int32_t)v);
      } else {  // packed
        uint64_t n;
        if (!get_varint(b, i, n) || i + n > b.size()) { err = "bad packed"; return false; }
        size_t end = i + n;
        while (i < end) {
          uint64_t v;
          if (!get_varint(b, i, v)) { err = "bad packed value"; return false; }
          dst.push_back((int)(int32_t)v);
        }
      }
    } else {
      if (!skip_field(b, i, wt)) { err = "bad unknown field"; return false; }
    }
  }
  if (!has_name) { err = "op without name"; return false; }
  if (!op.device_ids.empty() && (int)op.device_ids.size() != op.num_parts()) {
    err = "op " + op.name + ": device_ids size != product(dims)";
    return false;
  }
  return true;
}

}  // namespace

std::string encode_strategy(const std::vector<OpStrategy>& ops) {
  std::string out;
  for (const auto& op : ops) {
    std::string m;
    put_tag(m, 1, 2);
    put_varint(m, op.name.size());
    m += op.name;
    put_int32(m, 2, op.device_type);
    for (int d : op.dims) put_int32(m, 3, d);
    int n = op.num_parts();
    for (int j = 0; j < n && j < (int)op.device_ids.size(); ++j) put_int32(m, 4, op.device_ids[j]);
    for (int t : op.memory_types) put_int32(m, 5, t);
    put_tag(out, 1, 2);
    put_varint(out, m.size());
    out += m;
  }
  return out;
}

bool decode_strategy(const std::string& b, std::vector<OpStrategy>& ops, std::string& err) {
  size_t i = 0;
  std::set<std::string> seen;
  while (i < b.size()) {
    uint64_t key;
    if (!get_varint(b, i, key)) { err = "truncated"; return false; }
    int field = (int)(key >> 3), wt = (int)(key & 7);
    if (field != 1 || wt != 2) {
      if (!skip_field(b, i, wt)) { err = "bad top-level field"; return false; }
      continue;
    }
    uint64_t n;
    if (!get_varint(b, i, n) || i + n > b.size()) { err = "bad op length"; return false; }
    OpStrategy op;
    if (!decode_op(b.substr(i, n), op, err)) return false;
    i += n;
    if (seen.count(op.name)) { err = "duplicate op " + op.name; return false; }
    seen.insert(op.name);
    ops.push_back(op);
  }
  return true;
}

bool load_strategy_file(const std::string& path, std::vector<OpStrategy>& ops, std::string& err) {
  std::ifstream f(path, std::ios::binary);
  if (!f) { err = "cannot open " + path; return false; }
  std::stringstream ss;
  ss << f.rdbuf();
  return decode_strategy(ss.str(), ops, err);
}

bool save_strategy_file(const std::string& path, const std::vector<OpStrategy>& ops, std::string& err) {
  std::ofstream f(path, std::ios::binary | std::ios::trunc);
  if (!f) { err = "cannot write " + path; return false; }
  std::string b = encode_strategy(ops);
  f.write(b.data(), (std::streamsize)b.size());
  return (bool)f;
}

}  // namespace flexmi
