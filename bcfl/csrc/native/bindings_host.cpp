// pybind11 bindings of the host runtime library (bcfl._host): SHA-256 / Merkle, the ledger,
// and the graph analytics of the trust layer. Built with g++ (no GPU needed) by
// bcfl/csrc/build.py; importable on CPU-only machines.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "graph.h"
#include "ledger.h"
#include "sha256.h"

namespace py = pybind11;
using namespace bcfl;

static std::vector<double> mat(py::array_t<double, py::array::c_style | py::array::forcecast> a,
                               int* n) {
  auto b = a.request();
  if (b.ndim != 2 || b.shape[0] != b.shape[1]) throw std::invalid_argument("square matrix expected");
  *n = (int)b.shape[0];
  const double* p = static_cast<const double*>(b.ptr);
  return std::vector<double>(p, p + (*n) * (*n));
}

static std::vector<char> active_mask(int n, const std::vector<int>& excluded) {
  std::vector<char> a(n, 1);
  for (int e : excluded)
    if (e >= 0 && e < n) a[e] = 0;
  return a;
}

static py::dict block_dict(const Block& b) {
  py::dict d;
  d["height"] = b.height; d["prev_hash"] = b.prev_hash; d["ts"] = b.ts; d["round"] = b.round;
  d["client"] = b.client; d["kind"] = b.kind; d["update_root"] = b.update_root;
  d["verdict"] = b.verdict; d["payload"] = b.payload; d["hash"] = b.hash;
  return d;
}

PYBIND11_MODULE(_host, m) {
  m.doc() = "bcfl native host runtime: SHA-256/Merkle, ledger, graph analytics";

  m.def("sha256_hex", [](py::bytes data) {
    std::string s = data;
    return sha256_hex(s);
  });
  m.def("merkle_root_hex", [](py::buffer data, size_t leaf_bytes) {
    auto b = data.request();
    size_t n = (size_t)b.size * (size_t)b.itemsize;
    py::gil_scoped_release nogil;
    auto r = merkle_root(static_cast<const uint8_t*>(b.ptr), n, leaf_bytes);
    return to_hex(r.data(), 32);
  });
  m.def("merkle_from_leaves_hex", [](py::array_t<uint8_t, py::array::c_style> leaves) {
    auto b = leaves.request();
    size_t nl = (size_t)b.shape[0];
    std::vector<std::array<uint8_t, 32>> v(nl);
    const uint8_t* p = static_cast<const uint8_t*>(b.ptr);
    for (size_t i = 0; i < nl; ++i) std::memcpy(v[i].data(), p + 32 * i, 32);
    auto r = merkle_from_leaves(v);
    return to_hex(r.data(), 32);
  });

  py::class_<Ledger>(m, "Ledger")
      .def(py::init<const std::string&, double>(), py::arg("genesis_payload"), py::arg("ts"))
      .def("append", [](Ledger& l, int64_t round, int64_t client, const std::string& kind,
                        const std::string& root, const std::string& verdict,
                        const std::string& payload, double ts) {
             return block_dict(l.append(round, client, kind, root, verdict, payload, ts));
           })
      .def("verify", &Ledger::verify)
      .def("tip", &Ledger::tip)
      .def("__len__", &Ledger::size)
      .def("block", [](const Ledger& l, size_t i) { return block_dict(l.at(i)); })
      .def("set_field", [](Ledger& l, size_t i, const std::string& key, py::object v) {
        Block& b = l.mutable_at(i);
        if (key == "payload") b.payload = v.cast<std::string>();
        else if (key == "verdict") b.verdict = v.cast<std::string>();
        else if (key == "update_root") b.update_root = v.cast<std::string>();
        else if (key == "hash") b.hash = v.cast<std::string>();
        else if (key == "prev_hash") b.prev_hash = v.cast<std::string>();
        else throw std::invalid_argument("field");
      })
      .def("push_raw", [](Ledger& l, py::dict d) {
        Block b;
        b.height = d["height"].cast<int64_t>(); b.prev_hash = d["prev_hash"].cast<std::string>();
        b.ts = d["ts"].cast<double>(); b.round = d["round"].cast<int64_t>();
        b.client = d["client"].cast<int64_t>(); b.kind = d["kind"].cast<std::string>();
        b.update_root = d["update_root"].cast<std::string>();
        b.verdict = d["verdict"].cast<std::string>(); b.payload = d["payload"].cast<std::string>();
        b.hash = d["hash"].cast<std::string>();
        l.push_raw(b);
      })
      .def("clear", &Ledger::clear);

  m.def("pagerank", [](py::array_t<double> W, double alpha, double tol, int max_iter) {
        int n;
        auto w = mat(W, &n);
        auto r = pagerank(w, n, alpha, tol, max_iter);
        return py::make_tuple(r.ranks, r.iterations, r.converged);
      }, py::arg("W"), py::arg("alpha") = 0.85, py::arg("tol") = 1e-6, py::arg("max_iter") = 100);
  m.def("sigma_flags", [](const std::vector<double>& v, double k, bool low_only) {
        auto f = sigma_flags(v, k, low_only);
        return py::make_tuple(f.lo, f.hi, f.flags);
      });
  m.def("modified_z", &modified_z);
  m.def("dbscan", [](py::array_t<double, py::array::c_style | py::array::forcecast> X, double eps,
                     int min_samples) {
        auto b = X.request();
        int n = (int)b.shape[0], d = b.ndim > 1 ? (int)b.shape[1] : 1;
        const double* p = static_cast<const double*>(b.ptr);
        return dbscan(std::vector<double>(p, p + n * d), n, d, eps, min_samples);
      });
  m.def("weighted_degree", [](py::array_t<double> W) {
        int n;
        auto w = mat(W, &n);
        return weighted_degree(w, n);
      });
  m.def("shortest_paths", [](py::array_t<double> L, int src, const std::vector<int>& excluded) {
        int n;
        auto l = mat(L, &n);
        return dijkstra(l, n, src, active_mask(n, excluded));
      });
  m.def("info_passing_time", [](py::array_t<double> L, int src, const std::vector<int>& excluded) {
        int n;
        auto l = mat(L, &n);
        auto t = info_passing_time(l, n, src, active_mask(n, excluded));
        return py::make_tuple(t.sync, t.async_, t.reached);
      });
  m.def("best_source", [](py::array_t<double> L, const std::vector<int>& excluded, double d_g) {
        int n;
        auto l = mat(L, &n);
        auto b = best_source(l, n, active_mask(n, excluded), d_g);
        return py::make_tuple(b.source, b.objective);
      });
  m.def("greedy_modularity", [](py::array_t<double> A) {
        int n;
        auto a = mat(A, &n);
        return greedy_modularity(a, n);
      });
  m.def("modularity", [](py::array_t<double> A, const std::vector<int>& comm) {
        int n;
        auto a = mat(A, &n);
        return modularity(a, n, comm);
      });
}
