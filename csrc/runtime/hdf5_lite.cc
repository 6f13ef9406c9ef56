// Minimal HDF5 reader (see hdf5_lite.h).  Format reference: the HDF5 File Format Specification
// (superblock, object headers, dataspace / datatype / data layout / symbol table / link /
// continuation messages, v1 B-trees, local heaps, symbol table nodes).
#include "hdf5_lite.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <set>
#include <stdexcept>

namespace flexmi {
namespace {

constexpr uint64_t UNDEF = ~0ULL;

struct File {
  FILE* f = nullptr;
  int64_t size = 0;
  int so = 8, sl = 8;    // size of offsets / lengths
  uint64_t base = 0;

  ~File() {
    if (f) fclose(f);
  }
  std::vector<uint8_t> read(uint64_t off, size_t n) const {
    if (off == UNDEF || off > (uint64_t)size || n > (uint64_t)size - off) throw std::runtime_error("read past end of file");
    std::vector<uint8_t> b(n);
    if (fseeko(f, (off_t)off, SEEK_SET) != 0 || fread(b.data(), 1, n, f) != n) throw std::runtime_error("short read");
    return b;
  }
};

struct Cur {   // little-endian cursor over a byte buffer
  const std::vector<uint8_t>& b;
  size_t p;
  uint64_t u(int n) {
    if (n < 1 || n > 8) throw std::runtime_error("bad field width");
    if (p + n > b.size()) throw std::runtime_error("truncated structure");
    uint64_t v = 0;
    for (int i = 0; i < n; ++i) v |= (uint64_t)b[p + i] << (8 * i);
    p += n;
    return v;
  }
  uint64_t addr(int so) {
    uint64_t v = u(so);
    if (so < 8 && v == ((1ULL << (8 * so)) - 1)) return UNDEF;
    return v;
  }
  void skip(size_t n) {
    if (n > b.size() - std::min(p, b.size())) throw std::runtime_error("truncated structure");
    p += n;
  }
};

struct Msg {
  int type;
  std::vector<uint8_t> data;
};

// messages of an object header (v1 or v2), following continuation blocks
std::vector<Msg> object_messages(const File& F, uint64_t addr) {
  std::vector<Msg> msgs;
  auto pre = F.read(addr, 16);
  std::vector<std::pair<uint64_t, uint64_t>> blocks;   // (address, length) of message blocks
  bool v2 = pre[0] == 'O' && pre[1] == 'H' && pre[2] == 'D' && pre[3] == 'R';
  int v2flags = 0;
  if (!v2) {
    if (pre[0] != 1) throw std::runtime_error("unsupported object header version");
    Cur c{pre, 8};
    uint64_t hsize = c.u(4);
    blocks.emplace_back(addr + 16, hsize);
  } else {
    auto h = F.read(addr, 64);
    Cur c{h, 4};
    if (c.u(1) != 2) throw std::runtime_error("unsupported OHDR version");
    v2flags = (int)c.u(1);
    if (v2flags & 0x20) c.skip(16);
    if (v2flags & 0x10) c.skip(4);
    const int szb = 1 << (v2flags & 3);
    uint64_t chunk0 = c.u(szb);
    blocks.emplace_back(addr + c.p, chunk0);
  }
  for (size_t bi = 0; bi < blocks.size(); ++bi) {
    uint64_t a = blocks[bi].first, len = blocks[bi].second;
    auto b = F.read(a, len);
    Cur c{b, 0};
    if (v2 && bi > 0) {   // continuation chunk: "OCHK" signature, trailing checksum
      if (!(b.size() >= 4 && b[0] == 'O' && b[1] == 'C' && b[2] == 'H' && b[3] == 'K')) throw std::runtime_error("bad OCHK");
      c.p = 4;
    }
    // chunk #0's length excludes its checksum; an OCHK block's length includes it
    const size_t end = (v2 && bi > 0) ? (b.size() >= 4 ? b.size() - 4 : 0) : b.size();
    while (c.p + (v2 ? 4 : 8) <= end) {
      int type, size;
      if (!v2) {
        type = (int)c.u(2);
        size = (int)c.u(2);
        c.skip(4);     // flags + reserved
      } else {
        type = (int)c.u(1);
        size = (int)c.u(2);
        int fl = (int)c.u(1);
        if (v2flags & 0x04) c.skip(2);   // creation order
        (void)fl;
      }
      if (c.p + size > b.size()) throw std::runtime_error("message past header block");
      Msg m{type, std::vector<uint8_t>(b.begin() + c.p, b.begin() + c.p + size)};
      c.p += size;
      if (type == 0x10) {   // continuation: (offset, length)
        Cur d{m.data, 0};
        uint64_t ca = d.addr(F.so), cl = d.u(F.sl);
        blocks.emplace_back(ca, cl);
        continue;
      }
      if (type == 0 && !v2) continue;   // NIL padding
      msgs.push_back(std::move(m));
    }
  }
  return msgs;
}

std::string local_heap_name(const File& F, uint64_t heap, uint64_t off) {
  auto h = F.read(heap, 8 + 2 * F.sl + F.so);
  if (memcmp(h.data(), "HEAP", 4) != 0) throw std::runtime_error("bad local heap");
  Cur c{h, 8};
  uint64_t dsize = c.u(F.sl);
  c.u(F.sl);
  uint64_t daddr = c.addr(F.so);
  if (off >= dsize) throw std::runtime_error("heap offset out of range");
  auto d = F.read(daddr + off, (size_t)std::min<uint64_t>(dsize - off, 4096));
  size_t n = 0;
  while (n < d.size() && d[n]) ++n;
  return std::string(d.begin(), d.begin() + n);
}

// children (name, object header address) of a symbol-table group: v1 B-tree of SNODs
void symtab_children(const File& F, uint64_t btree, uint64_t heap, std::vector<std::pair<std::string, uint64_t>>& out,
                     int depth = 0) {
  if (depth > 32) throw std::runtime_error("B-tree too deep");
  auto h = F.read(btree, 8 + 2 * F.so);
  if (memcmp(h.data(), "TREE", 4) != 0) throw std::runtime_error("bad v1 B-tree node");
  Cur c{h, 4};
  int type = (int)c.u(1), level = (int)c.u(1), entries = (int)c.u(2);
  if (type != 0) throw std::runtime_error("not a group B-tree");
  const size_t body = (size_t)entries * (F.sl + F.so) + F.sl;
  auto b = F.read(btree + 8 + 2 * F.so, body);
  Cur k{b, 0};
  for (int e = 0; e < entries; ++e) {
    k.u(F.sl);
    uint64_t child = k.addr(F.so);
    if (level > 0) {
      symtab_children(F, child, heap, out, depth + 1);
      continue;
    }
    auto sh = F.read(child, 8);
    if (memcmp(sh.data(), "SNOD", 4) != 0) throw std::runtime_error("bad symbol table node");
    Cur s{sh, 6};
    int nsym = (int)s.u(2);
    const size_t esz = 2 * F.so + 8 + 16;
    auto ents = F.read(child + 8, nsym * esz);
    Cur ec{ents, 0};
    for (int i = 0; i < nsym; ++i) {
      uint64_t name_off = ec.u(F.so);
      uint64_t ohdr = ec.addr(F.so);
      ec.skip(8 + 16);
      out.emplace_back(local_heap_name(F, heap, name_off), ohdr);
    }
  }
}

std::string dtype_of(const std::vector<uint8_t>& d) {
  Cur c{d, 0};
  int cv = (int)c.u(1);
  int cls = cv & 15;
  int bits0 = (int)c.u(1);
  c.skip(2);
  int size = (int)c.u(4);
  if (bits0 & 1) throw std::runtime_error("big-endian datatypes are not supported");
  if (cls == 0) return std::string("<") + ((bits0 & 8) ? "i" : "u") + std::to_string(size);
  if (cls == 1) return "<f" + std::to_string(size);
  throw std::runtime_error("datatype class " + std::to_string(cls) + " is not supported");
}

std::vector<int64_t> shape_of(const File& F, const std::vector<uint8_t>& d) {
  Cur c{d, 0};
  int ver = (int)c.u(1), rank = (int)c.u(1);
  c.u(1);   // flags
  if (ver == 1) c.skip(5);
  else c.skip(1);   // v2: dataspace type
  std::vector<int64_t> s;
  for (int i = 0; i < rank; ++i) s.push_back((int64_t)c.u(F.sl));
  return s;
}

void layout_of(const File& F, const std::vector<uint8_t>& d, H5Dataset& ds) {
  Cur c{d, 0};
  int ver = (int)c.u(1);
  if (ver >= 3) {
    int cls = (int)c.u(1);
    if (cls == 1) {
      uint64_t a = c.addr(F.so);
      uint64_t n = c.u(F.sl);
      ds.offset = a == UNDEF ? -1 : (int64_t)(a + F.base);
      ds.nbytes = (int64_t)n;
      return;
    }
    throw std::runtime_error("compact / chunked / virtual dataset layouts are not supported");
  }
  int dims = (int)c.u(1), cls = (int)c.u(1);
  c.skip(5);
  if (cls != 1) throw std::runtime_error("only contiguous v1/v2 layouts are supported");
  uint64_t a = c.addr(F.so);
  ds.offset = a == UNDEF ? -1 : (int64_t)(a + F.base);
  (void)dims;
}

void walk(const File& F, uint64_t ohdr, const std::string& prefix, std::vector<H5Dataset>& out, std::set<uint64_t>& seen) {
  if (!seen.insert(ohdr).second) return;
  auto msgs = object_messages(F, ohdr);
  const Msg *space = nullptr, *type = nullptr, *layout = nullptr;
  std::vector<std::pair<std::string, uint64_t>> kids;
  for (auto& m : msgs) {
    if (m.type == 0x01) space = &m;
    else if (m.type == 0x03) type = &m;
    else if (m.type == 0x08) layout = &m;
    else if (m.type == 0x0B) throw std::runtime_error("filtered (compressed) datasets are not supported");
    else if (m.type == 0x11) {
      Cur c{m.data, 0};
      uint64_t bt = c.addr(F.so), hp = c.addr(F.so);
      symtab_children(F, bt, hp, kids);
    } else if (m.type == 0x06) {   // link message (compact group storage)
      Cur c{m.data, 0};
      c.u(1);
      int fl = (int)c.u(1);
      int ltype = 0;
      if (fl & 0x08) ltype = (int)c.u(1);
      if (fl & 0x04) c.skip(8);
      if (fl & 0x10) c.skip(1);
      uint64_t nlen = c.u(1 << (fl & 3));
      if (nlen > m.data.size() - c.p) throw std::runtime_error("link name past message");
      std::string name(m.data.begin() + c.p, m.data.begin() + c.p + nlen);
      c.skip(nlen);
      if (ltype == 0) kids.emplace_back(name, c.addr(F.so));
    } else if (m.type == 0x02) {
      Cur c{m.data, 0};
      c.u(1);
      int fl = (int)c.u(1);
      if (fl & 1) c.skip(8);
      uint64_t fheap = c.addr(F.so);
      if (fheap != UNDEF) throw std::runtime_error("dense (fractal-heap) groups are not supported");
    }
  }
  if (space && type && layout) {
    H5Dataset ds;
    ds.name = prefix;
    ds.dtype = dtype_of(type->data);
    ds.shape = shape_of(F, space->data);
    layout_of(F, layout->data, ds);
    int64_t n = std::stoi(ds.dtype.substr(2));
    for (auto s : ds.shape) {
      if (s < 0 || (s > 0 && n > (int64_t(1) << 62) / s)) throw std::runtime_error("bad dataspace extent");
      n *= s;
    }
    if (ds.nbytes == 0) ds.nbytes = n;
    if (ds.nbytes < n) throw std::runtime_error("dataset '" + prefix + "' is smaller than its dataspace");
    if (ds.offset >= 0 && (ds.offset > F.size || ds.nbytes > F.size - ds.offset))
      throw std::runtime_error("dataset '" + prefix + "' extends past the end of the file");
    out.push_back(ds);
    return;
  }
  for (auto& k : kids) walk(F, k.second, prefix.empty() ? k.first : prefix + "/" + k.first, out, seen);
}

}  // namespace

bool h5_list_datasets(const std::string& path, std::vector<H5Dataset>& out, std::string& err) {
  try {
    File F;
    F.f = fopen(path.c_str(), "rb");
    if (!F.f) throw std::runtime_error("cannot open " + path);
    fseeko(F.f, 0, SEEK_END);
    F.size = (int64_t)ftello(F.f);
    static const uint8_t sig[8] = {0x89, 'H', 'D', 'F', '\r', '\n', 0x1a, '\n'};
    int64_t sb = -1;
    for (int64_t o = 0; o + 8 <= F.size; o = o == 0 ? 512 : 2 * o) {
      auto b = F.read(o, 8);
      if (memcmp(b.data(), sig, 8) == 0) {
        sb = o;
        break;
      }
    }
    if (sb < 0) throw std::runtime_error("not an HDF5 file");
    auto h = F.read(sb, std::min<int64_t>(128, F.size - sb));
    if (h.size() < 16) throw std::runtime_error("truncated superblock");
    int ver = h[8];
    uint64_t root = UNDEF;
    auto check_sizes = [&]() {
      auto ok = [](int v) { return v == 2 || v == 4 || v == 8; };
      if (!ok(F.so) || !ok(F.sl)) throw std::runtime_error("bad superblock offset/length sizes");
    };
    if (ver <= 1) {
      F.so = h[13];
      F.sl = h[14];
      check_sizes();
      Cur c{h, (size_t)(ver == 0 ? 24 : 28)};
      F.base = c.addr(F.so);
      c.addr(F.so);   // free-space info
      c.addr(F.so);   // end of file
      c.addr(F.so);   // driver info
      c.u(F.so);      // root entry: link name offset
      root = c.addr(F.so);
    } else {
      F.so = h[9];
      F.sl = h[10];
      check_sizes();
      Cur c{h, 12};
      F.base = c.addr(F.so);
      c.addr(F.so);   // superblock extension
      c.addr(F.so);   // end of file
      root = c.addr(F.so);
    }
    std::set<uint64_t> seen;
    walk(F, root, "", out, seen);
    return true;
  } catch (const std::exception& e) {
    err = e.what();
    return false;
  }
}

}  // namespace flexmi
