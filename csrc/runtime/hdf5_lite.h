// Minimal native HDF5 reader for the DLRM dataset files (reference: examples/cpp/DLRM/dlrm.cc:284-330
// opens X_int / X_cat / y with libhdf5; preprocess_hdf.py writes them with h5py).  libhdf5 is not
// part of this image, so flexmi parses the subset such files use and memory-maps the raw data:
//   * superblock v0/v1 (h5py's default "earliest" format) and v2/v3;
//   * object headers v1 and v2 ("OHDR") with continuation blocks;
//   * groups as symbol tables (v1 B-tree + local heap) or compact link messages;
//   * datasets with a simple dataspace, little-endian integer / float datatypes and a
//     contiguous (or compact) layout -- no chunking, no filters (error otherwise).
// The result is each dataset's dtype, shape and byte offset of its contiguous data in the file.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace flexmi {

struct H5Dataset {
  std::string name;             // path inside the file ("X_int", "grp/y")
  std::string dtype;            // numpy-style: "<f4", "<f8", "<i8", "<i4", "<u1", ...
  std::vector<int64_t> shape;
  int64_t offset = -1;          // byte offset of the contiguous data (-1: not allocated)
  int64_t nbytes = 0;
};

bool h5_list_datasets(const std::string& path, std::vector<H5Dataset>& out, std::string& err);

}  // namespace flexmi
