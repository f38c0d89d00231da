// Keras-compatible HDF5 weight files, written/read through libhdf5's C API (no h5py in this
// environment).  Reference: ModelCheckpoint(save_weights_only=True) / load_weights
// (fed_model.py:103-105,138) and Keras' `*_notop.h5` ImageNet weights:
//
//   /                       attrs: layer_names [S], backend "tensorflow", keras_version
//   /<layer>                attrs: weight_names [S]   (e.g. "block1_conv1/kernel:0")
//   /<layer>/<weight name>  float32 dataset (kernel HWIO, bias, gamma, beta, moving stats)
//
// The module is generic: write(path, string-list attrs, scalar-string attrs, float datasets) and
// read(path) -> (attrs, datasets).  Layout policy lives in idc_models_amd/ckpt.
#include <hdf5.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

struct H5Err {
  H5Err() { H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr); }
};

void check(herr_t e, const std::string& what) {
  if (e < 0) throw std::runtime_error("hdf5: " + what);
}

hid_t ensure_groups(hid_t file, const std::string& path) {
  // create intermediate groups of `path` (excluding the last component); returns parent id
  hid_t cur = H5Gopen2(file, "/", H5P_DEFAULT);
  size_t pos = 1;
  while (true) {
    size_t nxt = path.find('/', pos);
    if (nxt == std::string::npos) break;
    std::string name = path.substr(pos, nxt - pos);
    hid_t g;
    if (H5Lexists(cur, name.c_str(), H5P_DEFAULT) > 0) g = H5Gopen2(cur, name.c_str(), H5P_DEFAULT);
    else g = H5Gcreate2(cur, name.c_str(), H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
    if (g < 0) throw std::runtime_error("hdf5: cannot create group " + name);
    H5Gclose(cur);
    cur = g;
    pos = nxt + 1;
  }
  return cur;
}

hid_t open_obj(hid_t file, const std::string& path) {
  if (path == "/" || path.empty()) return H5Gopen2(file, "/", H5P_DEFAULT);
  hid_t parent = ensure_groups(file, path + "/");
  H5Gclose(parent);
  return H5Oopen(file, path.c_str(), H5P_DEFAULT);
}

void write_str_list_attr(hid_t obj, const std::string& name, const std::vector<std::string>& vals,
                         bool scalar) {
  size_t maxlen = 1;
  for (auto& v : vals) maxlen = std::max(maxlen, v.size());
  hid_t t = H5Tcopy(H5T_C_S1);
  H5Tset_size(t, maxlen);
  H5Tset_strpad(t, H5T_STR_NULLPAD);
  std::vector<char> buf(maxlen * std::max<size_t>(vals.size(), 1), 0);
  for (size_t i = 0; i < vals.size(); ++i) std::copy(vals[i].begin(), vals[i].end(), buf.begin() + i * maxlen);
  hid_t space;
  if (scalar) {
    space = H5Screate(H5S_SCALAR);
  } else {
    hsize_t dims[1] = {vals.size()};
    space = H5Screate_simple(1, dims, nullptr);
  }
  if (H5Aexists(obj, name.c_str()) > 0) H5Adelete(obj, name.c_str());
  hid_t a = H5Acreate2(obj, name.c_str(), t, space, H5P_DEFAULT, H5P_DEFAULT);
  check(a, "create attr " + name);
  if (!vals.empty()) check(H5Awrite(a, t, buf.data()), "write attr " + name);
  H5Aclose(a);
  H5Sclose(space);
  H5Tclose(t);
}

// attrs: list of (object path, attr name, values, is_scalar)
void write_file(const std::string& path,
                const std::vector<std::tuple<std::string, std::string, std::vector<std::string>, bool>>& attrs,
                const std::vector<std::pair<std::string, py::array_t<float, py::array::c_style | py::array::forcecast>>>& dsets) {
  H5Err guard;
  hid_t f = H5Fcreate(path.c_str(), H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
  if (f < 0) throw std::runtime_error("hdf5: cannot create " + path);
  try {
    for (auto& d : dsets) {
      const std::string& p = d.first;
      hid_t parent = ensure_groups(f, p);
      std::string leaf = p.substr(p.rfind('/') + 1);
      auto arr = d.second;
      std::vector<hsize_t> dims(arr.ndim());
      for (int i = 0; i < arr.ndim(); ++i) dims[i] = arr.shape(i);
      hid_t space = arr.ndim() ? H5Screate_simple(arr.ndim(), dims.data(), nullptr) : H5Screate(H5S_SCALAR);
      hid_t ds = H5Dcreate2(parent, leaf.c_str(), H5T_IEEE_F32LE, space, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
      check(ds, "create dataset " + p);
      check(H5Dwrite(ds, H5T_NATIVE_FLOAT, H5S_ALL, H5S_ALL, H5P_DEFAULT, arr.data()), "write " + p);
      H5Dclose(ds);
      H5Sclose(space);
      H5Gclose(parent);
    }
    for (auto& a : attrs) {
      hid_t obj = open_obj(f, std::get<0>(a));
      check(obj, "open " + std::get<0>(a));
      write_str_list_attr(obj, std::get<1>(a), std::get<2>(a), std::get<3>(a));
      H5Oclose(obj);
    }
  } catch (...) {
    H5Fclose(f);
    throw;
  }
  H5Fclose(f);
}

struct Reader {
  hid_t f;
  py::dict attrs;     // (path, name) -> list[str]
  py::dict datasets;  // path -> np.ndarray(float32)
};

void read_attrs(hid_t obj, const std::string& path, Reader& r) {
  H5O_info_t info;
  H5Oget_info2(obj, &info, H5O_INFO_NUM_ATTRS);
  for (hsize_t i = 0; i < info.num_attrs; ++i) {
    hid_t a = H5Aopen_by_idx(obj, ".", H5_INDEX_NAME, H5_ITER_INC, i, H5P_DEFAULT, H5P_DEFAULT);
    if (a < 0) continue;
    char nbuf[512];
    H5Aget_name(a, sizeof(nbuf), nbuf);
    hid_t t = H5Aget_type(a);
    hid_t sp = H5Aget_space(a);
    py::list vals;
    if (H5Tget_class(t) == H5T_STRING) {
      hssize_t n = H5Sget_simple_extent_npoints(sp);
      if (H5Tis_variable_str(t) > 0) {
        std::vector<char*> ptrs(n);
        hid_t mt = H5Tcopy(H5T_C_S1);
        H5Tset_size(mt, H5T_VARIABLE);
        H5Aread(a, mt, ptrs.data());
        for (auto p : ptrs) vals.append(py::bytes(p ? p : ""));
        H5Dvlen_reclaim(mt, sp, H5P_DEFAULT, ptrs.data());
        H5Tclose(mt);
      } else {
        size_t sz = H5Tget_size(t);
        std::vector<char> buf(sz * n + 1, 0);
        H5Aread(a, t, buf.data());
        for (hssize_t k = 0; k < n; ++k) {
          std::string s(buf.data() + k * sz, sz);
          s = s.substr(0, s.find('\0'));
          vals.append(py::bytes(s));
        }
      }
    }
    r.attrs[py::make_tuple(path, std::string(nbuf))] = vals;
    H5Sclose(sp);
    H5Tclose(t);
    H5Aclose(a);
  }
}

herr_t visit_cb(hid_t obj, const char* name, const H5O_info_t* info, void* op) {
  Reader& r = *reinterpret_cast<Reader*>(op);
  std::string path = std::string("/") + (std::string(name) == "." ? "" : name);
  if (path == "/.") path = "/";
  hid_t o = H5Oopen(obj, name, H5P_DEFAULT);
  if (o < 0) return 0;
  read_attrs(o, path, r);
  if (info->type == H5O_TYPE_DATASET) {
    hid_t sp = H5Dget_space(o);
    int nd = H5Sget_simple_extent_ndims(sp);
    std::vector<hsize_t> dims(nd);
    H5Sget_simple_extent_dims(sp, dims.data(), nullptr);
    std::vector<py::ssize_t> shape(dims.begin(), dims.end());
    py::array_t<float> arr(shape);
    H5Dread(o, H5T_NATIVE_FLOAT, H5S_ALL, H5S_ALL, H5P_DEFAULT, arr.mutable_data());
    r.datasets[py::str(path)] = arr;
    H5Sclose(sp);
  }
  H5Oclose(o);
  return 0;
}

py::tuple read_file(const std::string& path) {
  H5Err guard;
  Reader r;
  r.f = H5Fopen(path.c_str(), H5F_ACC_RDONLY, H5P_DEFAULT);
  if (r.f < 0) throw std::runtime_error("hdf5: cannot open " + path);
  H5Ovisit2(r.f, H5_INDEX_NAME, H5_ITER_INC, visit_cb, &r, H5O_INFO_BASIC);
  H5Fclose(r.f);
  return py::make_tuple(r.attrs, r.datasets);
}

bool is_hdf5(const std::string& path) {
  H5Err guard;
  return H5Fis_hdf5(path.c_str()) > 0;
}

}  // namespace

PYBIND11_MODULE(_idc_h5, m) {
  m.doc() = "Keras-layout HDF5 weight file IO over libhdf5";
  m.def("write", &write_file);
  m.def("read", &read_file);
  m.def("is_hdf5", &is_hdf5);
}
