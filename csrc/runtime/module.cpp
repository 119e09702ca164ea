// pybind11 bindings of the native CPU runtime: ``import _dmlc_rt`` (built in-tree by _build.py).
// Bytes in, bytes out: tensors cross the boundary as raw little-endian buffers, so this module needs
// neither torch nor numpy headers; the Python layer (checkpoint.py / data.py) wraps them as tensors.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "rt.h"

namespace py = pybind11;
using namespace dmlc_rt;

namespace {

void raise_if(const std::string& err) {
  if (!err.empty()) throw std::runtime_error(err);
}

py::tuple py_read_bundle(const std::string& prefix) {
  std::vector<BundleEntry> entries;
  std::vector<std::string> data;
  {
    py::gil_scoped_release nogil;
    raise_if(read_bundle(prefix, &entries, &data));
  }
  py::list out;
  for (size_t i = 0; i < entries.size(); ++i) {
    const auto& e = entries[i];
    out.append(py::make_tuple(e.name, e.dtype, e.shape, py::bytes(data[i])));
  }
  return py::tuple(out);
}

void py_write_bundle(const std::string& prefix, const std::vector<std::string>& names, const std::vector<int>& dtypes,
                     const std::vector<std::vector<int64_t>>& shapes, const std::vector<py::bytes>& blobs) {
  std::vector<std::string> data;
  data.reserve(blobs.size());
  for (auto& b : blobs) data.emplace_back(b);
  py::gil_scoped_release nogil;
  raise_if(write_bundle(prefix, names, dtypes, shapes, data));
}

py::list py_read_table(const py::bytes& image) {
  std::vector<std::pair<std::string, std::string>> kv;
  std::string err;
  if (!read_table(std::string(image), &kv, &err)) throw std::runtime_error(err);
  py::list out;
  for (auto& e : kv) out.append(py::make_tuple(py::bytes(e.first), py::bytes(e.second)));
  return out;
}

py::bytes py_build_table(const std::vector<py::bytes>& keys, const std::vector<py::bytes>& values, size_t block_size,
                         int restart_interval) {
  TableBuilder tb(block_size, restart_interval);
  for (size_t i = 0; i < keys.size(); ++i) tb.add(std::string(keys[i]), std::string(values.at(i)));
  return py::bytes(tb.finish());
}

py::bytes py_encode_entry(int dtype, const std::vector<int64_t>& shape, int shard_id, int64_t offset, int64_t size,
                          uint32_t crc) {
  BundleEntry e;
  e.dtype = dtype; e.shape = shape; e.shard_id = shard_id; e.offset = offset; e.size = size; e.crc32c = crc;
  return py::bytes(encode_entry(e));
}

py::tuple py_read_cifar(const std::vector<std::string>& files, int threads) {
  std::vector<uint8_t> images;
  std::vector<int32_t> labels;
  {
    py::gil_scoped_release nogil;
    raise_if(read_cifar_files(files, &images, &labels, threads));
  }
  return py::make_tuple(py::bytes((const char*)images.data(), images.size()),
                        py::bytes((const char*)labels.data(), labels.size() * 4), (int64_t)labels.size());
}

}  // namespace

PYBIND11_MODULE(_dmlc_rt, m) {
  m.doc() = "dmlc native CPU runtime: crc32c, TF TensorBundle-V2, TFRecord events, CIFAR-10 reader";
  m.def("crc32c", [](const py::bytes& b, uint32_t init) {
    std::string s(b);
    return crc32c_extend(init, (const uint8_t*)s.data(), s.size());
  }, py::arg("data"), py::arg("init") = 0);
  m.def("crc_mask", &crc_mask);
  m.def("crc_unmask", &crc_unmask);
  m.def("write_bundle", &py_write_bundle);
  m.def("read_bundle", &py_read_bundle);
  m.def("read_table", &py_read_table);
  m.def("build_table", &py_build_table, py::arg("keys"), py::arg("values"), py::arg("block_size") = 262144,
        py::arg("restart_interval") = 16);
  m.def("encode_header", [](int n) { return py::bytes(encode_header(n)); });
  m.def("encode_entry", &py_encode_entry);
  m.def("tfrecord_frame", [](const py::bytes& p) { return py::bytes(tfrecord_frame(std::string(p))); });
  m.def("event_file_version", [](double t) { return py::bytes(encode_event_file_version(t)); });
  m.def("event_scalars", [](double t, int64_t step, const std::vector<std::string>& tags, const std::vector<float>& v) {
    return py::bytes(encode_event_scalars(t, step, tags, v));
  });
  m.def("read_cifar", &py_read_cifar, py::arg("files"), py::arg("threads") = 8);
}
