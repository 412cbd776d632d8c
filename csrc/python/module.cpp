// Python bindings of the native core (pybind11, no libtorch dependency: the
// module links the system ROCm 7.2 HIP runtime and RCCL directly, so a process
// that uses it has exactly one HIP runtime).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>
#include <cstring>

#include "dbfs/engine.hpp"
#include "dbfs/shard_reader.hpp"

namespace py = pybind11;
using namespace dbfs;

namespace {

template <class T>
py::array_t<T> to_numpy(const std::vector<T>& v) {
  py::array_t<T> a(static_cast<py::ssize_t>(v.size()));
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}

template <class T>
std::vector<T> from_numpy(const py::array_t<T, py::array::c_style | py::array::forcecast>& a) {
  std::vector<T> v(static_cast<size_t>(a.size()));
  if (!v.empty()) std::memcpy(v.data(), a.data(), v.size() * sizeof(T));
  return v;
}

// Per-level records as a list of dicts (built on demand: converting them on
// every run cost more host time than a short GPU level).
py::list level_dicts(const RunResult& r) {
  py::list lv;
  for (const auto& l : r.levels) {
    py::dict x;
    x["level"] = l.level;
    x["dir"] = std::string(1, l.direction);
    x["frontier"] = l.frontier;
    x["frontier_edges"] = l.frontier_edges;
    x["discovered"] = l.discovered;
    x["ms"] = l.ms;
    x["comm_ms"] = l.comm_ms;
    x["gap_ms"] = l.gap_ms;
    lv.append(x);
  }
  return lv;
}

// Comm whose collectives are implemented in Python (torch.distributed / gloo).
// Buffers are passed as integer addresses plus byte counts; only meaningful
// with the CPU backend (host memory).
class PyCommBase : public Comm {
 public:
  virtual void py_alltoall(uintptr_t send, uintptr_t recv, size_t bytes) = 0;
  virtual void py_allgather(uintptr_t send, uintptr_t recv, size_t bytes) = 0;
  virtual void py_allreduce_sum_i64(uintptr_t buf, size_t count) = 0;
  virtual void py_alltoallv(uintptr_t send, std::vector<int64_t> sc, std::vector<int64_t> sd, uintptr_t recv,
                            std::vector<int64_t> rc, std::vector<int64_t> rd, size_t elem_bytes) = 0;
  virtual void py_barrier() = 0;

  void alltoall(const void* s, void* r, size_t b) override {
    py_alltoall(reinterpret_cast<uintptr_t>(s), reinterpret_cast<uintptr_t>(r), b);
  }
  void allgather(const void* s, void* r, size_t b) override {
    py_allgather(reinterpret_cast<uintptr_t>(s), reinterpret_cast<uintptr_t>(r), b);
  }
  void allreduce_sum_i64(int64_t* buf, size_t count) override {
    py_allreduce_sum_i64(reinterpret_cast<uintptr_t>(buf), count);
  }
  void alltoallv(const void* s, const int64_t* sc, const int64_t* sd, void* r, const int64_t* rc, const int64_t* rd,
                 size_t eb) override {
    const int n = size();
    py_alltoallv(reinterpret_cast<uintptr_t>(s), std::vector<int64_t>(sc, sc + n), std::vector<int64_t>(sd, sd + n),
                 reinterpret_cast<uintptr_t>(r), std::vector<int64_t>(rc, rc + n), std::vector<int64_t>(rd, rd + n),
                 eb);
  }
  void barrier() override { py_barrier(); }
  std::string name() const override { return "python"; }
};

class PyCommTrampoline : public PyCommBase {
 public:
  // Python implements get_rank / get_size / get_name (plain `rank` / `size` /
  // `name` are the read-only properties every Comm exposes).
  int rank() const override { PYBIND11_OVERRIDE_PURE_NAME(int, PyCommBase, "get_rank", rank, ); }
  int size() const override { PYBIND11_OVERRIDE_PURE_NAME(int, PyCommBase, "get_size", size, ); }
  std::string name() const override { PYBIND11_OVERRIDE_NAME(std::string, PyCommBase, "get_name", name, ); }
  void py_alltoall(uintptr_t s, uintptr_t r, size_t b) override {
    PYBIND11_OVERRIDE_PURE(void, PyCommBase, py_alltoall, s, r, b);
  }
  void py_allgather(uintptr_t s, uintptr_t r, size_t b) override {
    PYBIND11_OVERRIDE_PURE(void, PyCommBase, py_allgather, s, r, b);
  }
  void py_allreduce_sum_i64(uintptr_t buf, size_t count) override {
    PYBIND11_OVERRIDE_PURE(void, PyCommBase, py_allreduce_sum_i64, buf, count);
  }
  void py_alltoallv(uintptr_t s, std::vector<int64_t> sc, std::vector<int64_t> sd, uintptr_t r,
                    std::vector<int64_t> rc, std::vector<int64_t> rd, size_t eb) override {
    PYBIND11_OVERRIDE_PURE(void, PyCommBase, py_alltoallv, s, sc, sd, r, rc, rd, eb);
  }
  void py_barrier() override { PYBIND11_OVERRIDE_PURE(void, PyCommBase, py_barrier, ); }
};

}  // namespace

PYBIND11_MODULE(_dbfs_native, m) {
  m.doc() = "MI355X-native distributed BFS core (HIP/CDNA4 kernels, RCCL over xGMI)";
  py::register_exception<Error>(m, "NativeError", PyExc_RuntimeError);

  m.attr("UNREACHED") = py::int_(kUnreached);
  m.attr("TD_EDGES_PER_BLOCK") = py::int_(kTdEdgesPerBlock);
  m.attr("UNIT_VERTICES") = py::int_(kUnitVertices);
  m.attr("MAX_HUBS") = py::int_(kMaxHubs);

  // ---- graphs ----
  py::class_<HostCSR>(m, "HostCSR")
      .def_readonly("n", &HostCSR::n)
      .def_readonly("row_lo", &HostCSR::row_lo)
      .def_readonly("rows", &HostCSR::rows)
      .def_readonly("input_edges", &HostCSR::input_edges)
      .def_property_readonly("directed_edges", &HostCSR::directed_edges)
      .def_property_readonly("row_off", [](const HostCSR& g) { return to_numpy(g.row_off); })
      .def_property_readonly("col", [](const HostCSR& g) { return to_numpy(g.col); })
      .def("degree", [](const HostCSR& g, int64_t r) { return g.degree(r); });

  m.def(
      "read_graph",
      [](const std::string& path, bool verbose, bool directed) {
        if (path != "-" && is_binary_csr(path)) return read_binary_csr(path);
        ReadOptions ro;
        ro.verbose_reference_lines = verbose;
        return build_csr(read_edge_list(path, ro), directed);
      },
      py::arg("path"), py::arg("verbose") = false, py::arg("directed") = false,
      py::call_guard<py::gil_scoped_release>(),
      "Read an edge list / MatrixMarket / binary-CSR file (\"-\": standard input) into a CSR, symmetrised "
      "unless directed.");
  m.def(
      "read_edge_list",
      [](const std::string& path) {
        EdgeList el = read_edge_list(path);
        return py::make_tuple(el.n, to_numpy(el.u), to_numpy(el.v));
      },
      py::arg("path"));
  m.def("detect_format", [](const std::string& p) {
    switch (detect_format(p)) {
      case FileFormat::Binary: return std::string("binary");
      case FileFormat::MatrixMarket: return std::string("mtx");
      default: return std::string("edgelist");
    }
  });
  m.def(
      "build_csr",
      [](int64_t n, py::array_t<uint32_t, py::array::c_style | py::array::forcecast> u,
         py::array_t<uint32_t, py::array::c_style | py::array::forcecast> v, bool directed) {
        EdgeList el;
        el.n = n;
        el.u = from_numpy<uint32_t>(u);
        el.v = from_numpy<uint32_t>(v);
        DBFS_CHECK(el.u.size() == el.v.size(), "u and v must have the same length");
        for (size_t i = 0; i < el.u.size(); ++i)
          DBFS_CHECK(el.u[i] < n && el.v[i] < n, "edge endpoint out of range");
        return build_csr(el, directed);
      },
      py::arg("n"), py::arg("u"), py::arg("v"), py::arg("directed") = false);
  m.def("write_binary_csr", &write_binary_csr, py::arg("path"), py::arg("csr"));
  m.def(
      "binary_csr_info",
      [](const std::string& path) {
        BinaryCsrInfo i = binary_csr_info(path);
        py::dict d;
        d["version"] = i.version;
        d["n"] = i.n;
        d["row_lo"] = i.row_lo;
        d["rows"] = i.rows;
        d["nnz"] = i.nnz;
        d["input_edges"] = i.input_edges;
        return d;
      },
      py::arg("path"));
  m.def("read_binary_csr_rows", &read_binary_csr_rows, py::arg("path"), py::arg("lo"), py::arg("hi"),
        py::call_guard<py::gil_scoped_release>(),
        "Global rows [lo, hi) of a binary CSR cache as a shard (only those rows' blocks are read and verified).");
  m.def("write_levels", [](const std::string& path, py::array_t<int32_t, py::array::c_style | py::array::forcecast> l) {
    write_levels(path, from_numpy<int32_t>(l));
  });
  m.def(
      "cpu_bfs",
      [](const HostCSR& g, int64_t src) {
        CpuBfsResult r;
        {
          py::gil_scoped_release rel;
          r = cpu_bfs(g, src);
        }
        return py::make_tuple(to_numpy(r.level), to_numpy(r.parent_edge));
      },
      py::arg("csr"), py::arg("src"));

  py::class_<GenParams>(m, "GenParams")
      .def_readonly("n", &GenParams::n)
      .def_readonly("m", &GenParams::m)
      .def_readonly("scale", &GenParams::scale)
      .def_readonly("seed", &GenParams::seed)
      .def_readonly("uniform", &GenParams::uniform)
      .def_readonly("power_law", &GenParams::power_law)
      .def_readonly("pl_i0", &GenParams::pl_i0)
      .def_readonly("pl_dmax", &GenParams::pl_dmax)
      .def_readonly("grid_w", &GenParams::grid_w)
      .def_readwrite("scramble", &GenParams::scramble);
  m.def("rmat_params", &rmat_params, py::arg("scale"), py::arg("edge_factor") = 16, py::arg("seed") = 1);
  m.def("uniform_params", &uniform_params, py::arg("n"), py::arg("m"), py::arg("seed") = 1);
  m.def("power_law_params", &power_law_params, py::arg("n"), py::arg("m"), py::arg("dmax"), py::arg("seed") = 1);
  m.def("grid_params", &grid_params, py::arg("w"), py::arg("h"));
  m.def(
      "generate_edges",
      [](const GenParams& p, int64_t begin, int64_t end) {
        if (end < 0) end = p.m;
        DBFS_CHECK(0 <= begin && begin <= end && end <= p.m, "bad edge range");
        std::vector<uint32_t> u(static_cast<size_t>(end - begin)), v(u.size());
        {
          py::gil_scoped_release rel;
          for (int64_t i = begin; i < end; ++i) {
            uint64_t a, b;
            gen_edge(p, static_cast<uint64_t>(i), a, b);
            u[i - begin] = static_cast<uint32_t>(a);
            v[i - begin] = static_cast<uint32_t>(b);
          }
        }
        return py::make_tuple(to_numpy(u), to_numpy(v));
      },
      py::arg("params"), py::arg("begin") = 0, py::arg("end") = -1,
      "Host copy of the counter-based generator stream (bit-identical to the device).");
  m.def("scramble_vertex", &scramble_vertex);

  py::class_<Partition>(m, "Partition")
      .def(py::init([](int64_t n, int nranks) { return Partition::block(n, nranks); }), py::arg("n"),
           py::arg("nranks"))
      .def_readonly("n", &Partition::n)
      .def_readonly("nranks", &Partition::nranks)
      .def_readonly("part", &Partition::part)
      .def("owner", &Partition::owner)
      .def("lo", &Partition::lo)
      .def("hi", &Partition::hi)
      .def("count", &Partition::count)
      .def("slice_words", &Partition::slice_words)
      .def("global_words", &Partition::global_words);

  // ---- runtime ----
  py::class_<Backend, std::shared_ptr<Backend>>(m, "Backend")
      .def_property_readonly("name", &Backend::name)
      .def_property_readonly("device_id", &Backend::device_id)
      .def_property_readonly("device_bytes", &Backend::device_bytes)
      .def_property_readonly("peak_device_bytes", &Backend::peak_device_bytes)
      .def_property_readonly("is_gpu", [](const Backend& b) { return b.kind() == DeviceKind::HIP; })
      .def("synchronize", &Backend::synchronize, py::call_guard<py::gil_scoped_release>());
  m.def("cpu_backend", []() { return std::shared_ptr<Backend>(make_cpu_backend()); });
  m.def("hip_backend", [](int dev) { return std::shared_ptr<Backend>(make_hip_backend(dev)); }, py::arg("device") = 0);
  m.def("hip_device_count", &hip_device_count);

  py::class_<Comm, std::shared_ptr<Comm>>(m, "Comm")
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("size", &Comm::size)
      .def_property_readonly("name", &Comm::name)
      .def("barrier", &Comm::barrier, py::call_guard<py::gil_scoped_release>())
      .def("sum_host", &Comm::sum_host, py::call_guard<py::gil_scoped_release>())
      .def("max_host", &Comm::max_host, py::call_guard<py::gil_scoped_release>())
      .def("allgather_host_i64", &Comm::allgather_host_i64, py::call_guard<py::gil_scoped_release>())
      .def("reset_traffic", &Comm::reset_traffic)
      .def(
          "traffic",
          [](const Comm& c) {
            // {kind: (calls, bytes sent to other ranks)}
            static const char* names[] = {"alltoall", "allgather", "allreduce", "alltoallv", "barrier"};
            py::dict d;
            for (int k = 0; k < Comm::kTrafficKinds; ++k)
              d[names[k]] = py::make_tuple(c.traffic().calls[k], c.traffic().bytes[k]);
            // collectives that shared another's launch (allgather_allreduce)
            d["fused"] = py::make_tuple(c.traffic().fused, int64_t(0));
            return d;
          })
      .def("bind_backend", [](Comm& c, std::shared_ptr<Backend> be) { c.bind_backend(be.get()); },
           py::keep_alive<1, 2>());
  m.def(
      "local_comm", [](std::shared_ptr<Backend> be) { return std::shared_ptr<Comm>(new LocalComm(*be)); },
      py::keep_alive<0, 1>());
  py::class_<VirtualGroup, std::shared_ptr<VirtualGroup>>(m, "VirtualGroup")
      .def(py::init<int>())
      .def_property_readonly("size", &VirtualGroup::size)
      .def("abort", &VirtualGroup::abort, py::arg("reason"))
      .def_property_readonly("aborted", &VirtualGroup::aborted);
  m.def(
      "virtual_comm",
      [](std::shared_ptr<VirtualGroup> g, int rank, std::shared_ptr<Backend> be) {
        return std::shared_ptr<Comm>(new VirtualComm(g, rank, *be));
      },
      py::keep_alive<0, 3>());
  m.def(
      "tcp_comm",
      [](std::shared_ptr<TcpBootstrap> boot, std::shared_ptr<Backend> be) {
        return std::shared_ptr<Comm>(new TcpComm(boot, *be));
      },
      py::keep_alive<0, 2>());
  py::class_<PeerComm, Comm, std::shared_ptr<PeerComm>>(m, "PeerComm")
      .def_property_readonly("slot_bytes", &PeerComm::slot_bytes)
      .def_property_readonly("peer_ops", &PeerComm::peer_ops)
      .def_property_readonly("inner_ops", &PeerComm::inner_ops)
      .def_property_readonly("direct_on", &PeerComm::direct_on)
      .def_property_readonly("frontier_on", &PeerComm::frontier_on)
      .def_property_readonly("fused", &PeerComm::fused)
      .def_property_readonly("split_waits", &PeerComm::split_waits)
      .def_property_readonly("shared_device", &PeerComm::shared_device)
      .def_property_readonly("bus_ids", &PeerComm::bus_ids)
      // P x P: 2 same GPU, 1 peer access, 0 none, -1 not visible (row: the rank that looked)
      .def_property_readonly("peer_access",
                             [](const PeerComm& c) {
                               const int P = c.size();
                               py::list rows;
                               for (int r = 0; r < P; ++r) {
                                 py::list row;
                                 for (int q = 0; q < P; ++q) row.append(c.peer_access()[r * P + q]);
                                 rows.append(row);
                               }
                               return rows;
                             })
      .def_property_readonly("self_test_verdict", &PeerComm::self_test_verdict)
      .def("self_test", [](PeerComm& c) {
        std::string why;
        bool ok;
        {
          py::gil_scoped_release rel;
          ok = c.self_test(&why);
        }
        return py::make_tuple(ok, why);
      });
  m.def(
      "peer_comm",
      [](std::shared_ptr<Bootstrap> boot, std::shared_ptr<Backend> be, std::shared_ptr<Comm> inner,
         size_t slot_bytes) {
        py::gil_scoped_release rel;
        return std::make_shared<PeerComm>(boot, *be, inner, slot_bytes);
      },
      py::arg("boot"), py::arg("backend"), py::arg("inner"), py::arg("slot_bytes") = size_t(16) << 20,
      py::keep_alive<0, 2>(), py::keep_alive<0, 3>());
  // shadow rank (csrc/comm/replay_comm.cpp): record one rank's collective
  // outputs in a P-rank run, replay them with that rank alone on the GPU
  py::class_<CommTape, std::shared_ptr<CommTape>>(m, "CommTape")
      .def_readonly("rank", &CommTape::rank)
      .def_readonly("size", &CommTape::size)
      .def_property_readonly("bytes", &CommTape::bytes)
      .def("__len__", [](const CommTape& t) { return t.recs.size(); })
      .def("records", [](const CommTape& t) {
        // (kind, a, b, output bytes) per collective
        py::list out;
        static const char* names[] = {"alltoall", "allgather", "allreduce", "alltoallv", "barrier"};
        for (const auto& r : t.recs)
          out.append(py::make_tuple(r.kind == CommTape::kLists ? "alltoall_lists" : names[r.kind], r.a, r.b,
                                    static_cast<int64_t>(r.data.size())));
        return out;
      });
  py::class_<RecordComm, Comm, std::shared_ptr<RecordComm>>(m, "RecordComm")
      .def_property_readonly("tape", &RecordComm::tape);
  m.def(
      "record_comm",
      [](std::shared_ptr<Comm> inner, std::shared_ptr<Backend> be) {
        auto c = std::make_shared<RecordComm>(inner);
        c->bind_backend(be.get());
        return c;
      },
      py::keep_alive<0, 1>(), py::keep_alive<0, 2>());
  py::class_<ReplayComm, Comm, std::shared_ptr<ReplayComm>>(m, "ReplayComm")
      .def_property_readonly("position", &ReplayComm::position)
      .def("__len__", &ReplayComm::length);
  m.def(
      "replay_comm",
      [](std::shared_ptr<CommTape> tape, std::shared_ptr<Backend> be) {
        py::gil_scoped_release rel;
        return std::make_shared<ReplayComm>(tape, *be);
      },
      py::keep_alive<0, 2>());
  m.def("nccl_unique_id", []() { return py::bytes(NcclComm::unique_id()); });
  m.def(
      "nccl_comm",
      [](py::bytes uid, int rank, int nranks, std::shared_ptr<Backend> be) {
        std::string u = uid;
        py::gil_scoped_release rel;
        return std::shared_ptr<Comm>(new NcclComm(u, rank, nranks, *be));
      },
      py::keep_alive<0, 4>());
  m.def("nccl_init_all", [](std::vector<std::shared_ptr<Backend>> bes) {
    std::vector<Backend*> raw;
    for (auto& b : bes) raw.push_back(b.get());
    auto comms = NcclComm::init_all(raw);
    std::vector<std::shared_ptr<Comm>> out;
    for (auto& c : comms) out.push_back(std::shared_ptr<Comm>(c.release()));
    return out;
  });
  // Collective latency: `iters` back-to-back collectives of `bytes` per peer
  // on device buffers, one barrier + synchronize around them; returns the
  // mean microseconds per collective (tools/peer_latency.py).
  m.def(
      "comm_latency",
      [](std::shared_ptr<Comm> comm, std::shared_ptr<Backend> be, const std::string& op, int64_t bytes,
         int iters) {
        py::gil_scoped_release rel;
        const int P = comm->size();
        const int64_t words = std::max<int64_t>(bytes / 8, 1);
        DBuf<int64_t> a(*be, static_cast<size_t>(words * P)), b(*be, static_cast<size_t>(words * P));
        be->memset_async(a.data(), 0, a.bytes());
        auto one = [&] {
          if (op == "allreduce") comm->allreduce_sum_i64(a.data(), static_cast<size_t>(words));
          else if (op == "allgather") comm->allgather(a.data(), b.data(), static_cast<size_t>(words) * 8);
          else if (op == "alltoall") comm->alltoall(a.data(), b.data(), static_cast<size_t>(words) * 8);
          else DBFS_CHECK(false, "comm_latency: op must be allreduce / allgather / alltoall");
        };
        for (int i = 0; i < 3; ++i) one();  // warm-up
        be->synchronize();
        comm->barrier();
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < iters; ++i) one();
        be->synchronize();
        const auto t1 = std::chrono::steady_clock::now();
        return std::chrono::duration<double, std::micro>(t1 - t0).count() / std::max(iters, 1);
      },
      py::arg("comm"), py::arg("backend"), py::arg("op"), py::arg("bytes"), py::arg("iters") = 200);
  // Run one collective on numpy data through a communicator (unit tests of the
  // Comm implementations).  The data is staged into backend memory first.
  m.def(
      "comm_exercise",
      [](std::shared_ptr<Comm> comm, std::shared_ptr<Backend> be, const std::string& op,
         py::array_t<int64_t, py::array::c_style | py::array::forcecast> data, std::vector<int64_t> send_counts,
         std::vector<int64_t> recv_counts) {
        std::vector<int64_t> in = from_numpy<int64_t>(data);
        const int P = comm->size();
        std::vector<int64_t> out;
        {
          py::gil_scoped_release rel;
          DBuf<int64_t> s(*be, std::max<size_t>(in.size(), 1));
          if (!in.empty()) be->to_device(s.data(), in.data(), in.size() * sizeof(int64_t));
          if (op == "allreduce") {
            comm->allreduce_sum_i64(s.data(), in.size());
            out.resize(in.size());
          } else if (op == "allgather") {
            out.resize(in.size() * static_cast<size_t>(P));
            DBuf<int64_t> r(*be, std::max<size_t>(out.size(), 1));
            comm->allgather(s.data(), r.data(), in.size() * sizeof(int64_t));
            be->to_host(out.data(), r.data(), out.size() * sizeof(int64_t));
          } else if (op == "alltoall") {
            DBFS_CHECK(in.size() % static_cast<size_t>(P) == 0, "alltoall input must be P equal chunks");
            out.resize(in.size());
            DBuf<int64_t> r(*be, std::max<size_t>(out.size(), 1));
            comm->alltoall(s.data(), r.data(), in.size() / P * sizeof(int64_t));
            be->to_host(out.data(), r.data(), out.size() * sizeof(int64_t));
          } else if (op == "alltoallv") {
            DBFS_CHECK(static_cast<int>(send_counts.size()) == P && static_cast<int>(recv_counts.size()) == P,
                       "alltoallv needs P send and P recv counts");
            std::vector<int64_t> sd(P), rd(P);
            int64_t so = 0, ro = 0;
            for (int r = 0; r < P; ++r) {
              sd[r] = so;
              rd[r] = ro;
              so += send_counts[r];
              ro += recv_counts[r];
            }
            DBFS_CHECK(so == static_cast<int64_t>(in.size()), "send counts must cover the input");
            out.resize(static_cast<size_t>(ro));
            DBuf<int64_t> r(*be, std::max<size_t>(out.size(), 1));
            comm->alltoallv(s.data(), send_counts.data(), sd.data(), r.data(), recv_counts.data(), rd.data(),
                            sizeof(int64_t));
            if (!out.empty()) be->to_host(out.data(), r.data(), out.size() * sizeof(int64_t));
          } else {
            throw Error("unknown op " + op);
          }
          if (op == "allreduce" && !out.empty()) be->to_host(out.data(), s.data(), out.size() * sizeof(int64_t));
          be->synchronize();
        }
        return to_numpy(out);
      },
      py::arg("comm"), py::arg("backend"), py::arg("op"), py::arg("data"),
      py::arg("send_counts") = std::vector<int64_t>(), py::arg("recv_counts") = std::vector<int64_t>());

  py::class_<PyCommBase, Comm, PyCommTrampoline, std::shared_ptr<PyCommBase>>(m, "PyComm")
      .def(py::init<>())
      .def("py_alltoall", &PyCommBase::py_alltoall)
      .def("py_allgather", &PyCommBase::py_allgather)
      .def("py_allreduce_sum_i64", &PyCommBase::py_allreduce_sum_i64)
      .def("py_alltoallv", &PyCommBase::py_alltoallv)
      .def("py_barrier", &PyCommBase::py_barrier);

  py::class_<Bootstrap, std::shared_ptr<Bootstrap>>(m, "Bootstrap")
      .def_property_readonly("rank", &Bootstrap::rank)
      .def_property_readonly("size", &Bootstrap::size)
      .def_property_readonly("in_process", &Bootstrap::in_process)
      .def(
          "broadcast",
          [](Bootstrap& b, py::bytes data, int root) {
            std::string s = data, r;
            {
              py::gil_scoped_release rel;
              r = b.broadcast(s, root);
            }
            return py::bytes(r);
          },
          py::arg("data"), py::arg("root") = 0)
      .def("allgather",
           [](Bootstrap& b, py::bytes data) {
             std::string s = data;
             std::vector<std::string> r;
             {
               py::gil_scoped_release rel;
               r = b.allgather(s);
             }
             py::list out;
             for (auto& x : r) out.append(py::bytes(x));
             return out;
           })
      .def("barrier", &Bootstrap::barrier, py::call_guard<py::gil_scoped_release>());
  // the ranks of a VirtualGroup (threads of this process) as a bootstrap: a
  // peer communicator over it shares its windows as device pointers
  m.def(
      "group_bootstrap",
      [](std::shared_ptr<VirtualGroup> g, int rank) { return std::shared_ptr<Bootstrap>(new GroupBootstrap(g, rank)); },
      py::arg("group"), py::arg("rank"));
  py::class_<TcpBootstrap, Bootstrap, std::shared_ptr<TcpBootstrap>>(m, "TcpBootstrap")
      .def(py::init<const std::string&, int, int, int, double>(), py::arg("host"), py::arg("port"), py::arg("rank"),
           py::arg("nranks"), py::arg("timeout_s") = 300.0, py::call_guard<py::gil_scoped_release>());

  py::class_<EdgeShard>(m, "EdgeShard")
      .def_readonly("n", &EdgeShard::n)
      .def_readonly("m", &EdgeShard::m)
      .def_readonly("first_edge", &EdgeShard::first_edge)
      .def_readonly("byte_begin", &EdgeShard::byte_begin)
      .def_readonly("byte_end", &EdgeShard::byte_end)
      .def_property_readonly("local_edges", &EdgeShard::local_edges)
      .def_property_readonly("u", [](const EdgeShard& e) { return py::array_t<vid_t>(e.u.size(), e.u.data()); })
      .def_property_readonly("v", [](const EdgeShard& e) { return py::array_t<vid_t>(e.v.size(), e.v.data()); });
  m.def(
      "write_generated_edge_list",
      [](const std::string& path, const GenParams& p, int threads) {
        py::gil_scoped_release rel;
        write_generated_edge_list(path, p, threads);
      },
      py::arg("path"), py::arg("params"), py::arg("threads") = 0);
  m.def(
      "read_edge_shard",
      [](const std::string& path, Comm& comm, int threads) {
        py::gil_scoped_release rel;
        return read_edge_shard(
            path, comm.rank(), comm.size(), [&comm](int64_t x) { return comm.allgather_host_i64(x); }, threads);
      },
      py::arg("path"), py::arg("comm"), py::arg("threads") = 0,
      "This rank's edges of an edge list / MatrixMarket file (collective: rank r parses only its byte range).");

  // ---- engine ----
  py::class_<DeviceGraph, std::shared_ptr<DeviceGraph>>(m, "DeviceGraph")
      .def_static(
          "from_host",
          [](std::shared_ptr<Backend> be, const HostCSR& csr, const Partition& part, int rank) {
            py::gil_scoped_release rel;
            return std::shared_ptr<DeviceGraph>(DeviceGraph::from_host(*be, csr, part, rank));
          },
          py::arg("backend"), py::arg("csr"), py::arg("partition"), py::arg("rank"), py::keep_alive<0, 1>())
      .def_static(
          "generate",
          [](std::shared_ptr<Backend> be, const GenParams& p, const Partition& part, int rank) {
            py::gil_scoped_release rel;
            return std::shared_ptr<DeviceGraph>(DeviceGraph::generate(*be, p, part, rank));
          },
          py::arg("backend"), py::arg("params"), py::arg("partition"), py::arg("rank"), py::keep_alive<0, 1>())
      .def_static(
          "from_edges",
          [](std::shared_ptr<Backend> be, Comm& comm, const Partition& part, int rank, int64_t input_edges,
             py::array_t<vid_t, py::array::c_style | py::array::forcecast> u,
             py::array_t<vid_t, py::array::c_style | py::array::forcecast> v) {
            DBFS_CHECK(u.size() == v.size(), "u and v must have the same length");
            const vid_t* pu = u.data();
            const vid_t* pv = v.data();
            const int64_t m = static_cast<int64_t>(u.size());
            py::gil_scoped_release rel;
            return std::shared_ptr<DeviceGraph>(DeviceGraph::from_edges(*be, comm, part, rank, input_edges, pu, pv, m));
          },
          py::arg("backend"), py::arg("comm"), py::arg("partition"), py::arg("rank"), py::arg("input_edges"),
          py::arg("u"), py::arg("v"), py::keep_alive<0, 1>())
      .def_static(
          "from_file",
          [](std::shared_ptr<Backend> be, Comm& comm, const std::string& path, int threads) {
            py::gil_scoped_release rel;
            return std::shared_ptr<DeviceGraph>(DeviceGraph::from_file(*be, comm, path, threads));
          },
          py::arg("backend"), py::arg("comm"), py::arg("path"), py::arg("threads") = 0, py::keep_alive<0, 1>())
      .def_property_readonly("n", &DeviceGraph::n)
      .def_property_readonly("lo", &DeviceGraph::lo)
      .def_property_readonly("rows", &DeviceGraph::rows)
      .def_property_readonly("nnz", &DeviceGraph::nnz)
      .def_property_readonly("input_edges", &DeviceGraph::input_edges)
      .def_property_readonly("rank", &DeviceGraph::rank)
      .def_property_readonly("partition", &DeviceGraph::partition)
      .def("to_host", &DeviceGraph::to_host, py::call_guard<py::gil_scoped_release>())
      .def("sort_neighbors_by_degree", &DeviceGraph::sort_neighbors_by_degree, py::arg("comm"),
           py::arg("hubs") = true, py::arg("max_hubs") = kMaxHubs, py::arg("id_order") = true,
           py::arg("td_hubs") = true,
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("col_by_id", &DeviceGraph::col_by_id)
      .def_property_readonly("td_hub_share", &DeviceGraph::td_hub_share)
      .def_property_readonly("hub_sorted", &DeviceGraph::hub_sorted)
      .def_property_readonly("nhubs", &DeviceGraph::nhubs)
      // from_file: (byte_begin, byte_end, edges) this rank parsed
      .def_property_readonly("ingest",
                             [](const DeviceGraph& g) {
                               return py::make_tuple(g.ingest().byte_begin, g.ingest().byte_end, g.ingest().edges);
                             })
      .def("degrees_of", &DeviceGraph::degrees_of);

  py::class_<RunResult>(m, "RunResult")
      .def_readonly("source", &RunResult::source)
      .def_readonly("ms", &RunResult::ms)
      .def_readonly("reached", &RunResult::reached)
      .def_readonly("edges", &RunResult::edges)
      .def_readonly("depth", &RunResult::depth)
      .def_readonly("gteps", &RunResult::gteps)
      .def_readonly("mispredicts", &RunResult::mispredicts)
      .def_property_readonly("chains",
                             [](const RunResult& r) {
                               py::list out;
                               for (const auto& c : r.chains)
                                 out.append(py::make_tuple(c.level, std::string(1, c.form), c.cap, c.gather, c.push, c.unvis, c.split, c.cut));
                               return out;
                             })
      .def("level_dicts", &level_dicts);

  py::class_<Engine, std::shared_ptr<Engine>>(m, "Engine")
      .def(py::init([](std::shared_ptr<DeviceGraph> g, std::shared_ptr<Comm> c, const std::string& mode, double alpha,
                       double beta, int bu_lane_limit, bool phase_timing, bool force_exchange) {
             EngineOptions o;
             o.mode = parse_mode(mode);
             o.alpha = alpha;
             o.beta = beta;
             o.bu_lane_limit = bu_lane_limit;
             o.phase_timing = phase_timing;
             o.force_exchange = force_exchange;
             py::gil_scoped_release rel;
             return std::make_shared<Engine>(*g, *c, o);
           }),
           py::arg("graph"), py::arg("comm"), py::arg("mode") = "do", py::arg("alpha") = 40.0, py::arg("beta") = 384.0,
           py::arg("bu_lane_limit") = 16, py::arg("phase_timing") = false, py::arg("force_exchange") = false,
           py::keep_alive<1, 2>(),
           py::keep_alive<1, 3>())
      .def(
          "run",
          [](Engine& e, int64_t src) {
            RunResult r;
            {
              py::gil_scoped_release rel;
              r = e.run(src);
            }
            return r;
          },
          py::arg("source"))
      .def(
          "run_many",
          [](Engine& e, const std::vector<int64_t>& sources) {
            // back-to-back traversals without a return to Python between them
            // (each complete before the next one's initialisation runs)
            std::vector<RunResult> out;
            out.reserve(sources.size());
            {
              py::gil_scoped_release rel;
              for (int64_t s : sources) out.push_back(e.run(s));
            }
            return out;
          },
          py::arg("sources"))
      .def("levels_local",
           [](const Engine& e) {
             std::vector<lvl_t> v;
             {
               py::gil_scoped_release rel;
               v = e.levels_local();
             }
             return to_numpy(v);
           })
      .def("gather_levels",
           [](Engine& e) {
             std::vector<lvl_t> v;
             {
               py::gil_scoped_release rel;
               v = e.gather_levels();
             }
             return to_numpy(v);
           })
      .def("validate", &Engine::validate, py::call_guard<py::gil_scoped_release>())
      .def("parents_local",
           [](Engine& e, int64_t src) {
             std::vector<int64_t> v;
             {
               py::gil_scoped_release rel;
               v = e.parents_local(src);
             }
             return to_numpy(v);
           })
      .def("gather_parents", [](Engine& e, int64_t src) {
        std::vector<int64_t> v;
        {
          py::gil_scoped_release rel;
          v = e.gather_parents(src);
        }
        return to_numpy(v);
      })
      .def_property_readonly("global_directed_edges", &Engine::global_directed_edges)
      .def_property(
          "mode", [](const Engine& e) { return std::string(mode_name(e.options().mode)); },
          [](Engine& e, const std::string& s) {
            EngineOptions o = e.options();
            o.mode = parse_mode(s);
            e.set_options(o);
          })
      .def_property(
          "phase_timing", [](const Engine& e) { return e.options().phase_timing; },
          [](Engine& e, bool on) {
            EngineOptions o = e.options();
            o.phase_timing = on;
            e.set_options(o);
          })
      .def(
          "set_heuristics",
          [](Engine& e, double alpha, double beta, int lane_limit, int64_t td_byte_edges, int64_t sparse_max_edges,
             int sparse_size_check) {
            EngineOptions o = e.options();
            o.alpha = alpha;
            o.beta = beta;
            o.bu_lane_limit = lane_limit;
            if (td_byte_edges >= 0) o.td_byte_edges = td_byte_edges;
            if (sparse_max_edges >= 0) o.sparse_max_edges = sparse_max_edges;
            if (sparse_size_check >= 0) o.sparse_size_check = sparse_size_check != 0;
            e.set_options(o);
          },
          py::arg("alpha"), py::arg("beta"), py::arg("lane_limit"), py::arg("td_byte_edges") = -1,
          py::arg("sparse_max_edges") = -1, py::arg("sparse_size_check") = -1)
      .def_property_readonly("td_byte_edges", [](const Engine& e) { return e.options().td_byte_edges; })
      // Generic tuning knob access (bench.py --opt NAME=VALUE, sweeps).
      .def("set_option",
           [](Engine& e, const std::string& name, double v) {
             EngineOptions o = e.options();
             set_engine_option(o, name, v);
             e.set_options(o);
           })
      .def("get_options", [](const Engine& e) { return engine_option_map(e.options()); });
}
