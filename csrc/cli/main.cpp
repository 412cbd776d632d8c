// `bfs` -- command-line driver, compatible with the reference's
// `./a.out <src> <file>` (README.md:4-14, bfs.cu:783-823) and its stdout lines
// (SURVEY Appendix A), plus the flags of SURVEY §5.6.
//
//   bfs <src> <edge-list|.mtx|.csr> [flags]
//   bfs --rmat SCALE[:EF] [src] [flags]
//
// Execution models:
//   default            1 GPU (HIP backend, device --device)
//   --gpus P           P GPUs in one process, one host thread per GPU: the
//                      peer-memory communicator (every rank's window shared
//                      as a device pointer, peer access enabled) over an
//                      in-process host communicator; one RCCL communicator
//                      per GPU (ncclCommInitAll) if the windows fail --
//                      replaces the reference's intra-node bfs.cu
//   --virtual-ranks P  P partitions on ONE device (threads + VirtualComm):
//                      exercises the distributed code path on one GPU
//   --cpu              CPU backend (no GPU needed)
//   WORLD_SIZE > 1     one process per GPU (torchrun / any launcher): TCP
//                      bootstrap on MASTER_ADDR:MASTER_PORT+1, the peer-memory
//                      communicator (IPC windows) over a TCP inner
//                      communicator -- replaces the reference's MPI build
//                      bfs_mpi.cu
// DBFS_COMM = peer | rccl | tcp selects the transport (default: peer with an
// agreed fallback to RCCL, then TCP), DBFS_DEVICE pins every process to one
// device (several ranks sharing a GPU: tests).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "dbfs/engine.hpp"

using namespace dbfs;

namespace {

struct Args {
  int64_t src = 0;
  bool src_given = false;
  std::string path;
  int gpus = 1;
  int virtual_ranks = 0;
  int device = 0;
  bool cpu = false;
  std::string mode = "do";
  double alpha = 40.0, beta = 384.0;
  int bu_lane_limit = 16;
  int rmat_scale = 0, rmat_ef = 16;
  int64_t uni_n = 0, uni_m = 0;
  uint64_t seed = 1;
  int roots = 0;
  bool oracle = true;
  bool validate = false;
  std::string levels_out;
  std::string cache_out;
  bool json = false;
  std::string level_csv;
  bool quiet = false;
  bool phase_timing = false;
  bool hub_sort = true;
  bool directed = false;
};

[[noreturn]] void usage(const char* msg = nullptr) {
  if (msg) std::fprintf(stderr, "error: %s\n\n", msg);
  std::fprintf(stderr,
               "usage: bfs <src> <edge-list|.mtx|.csr|-> [flags]   (- = standard input)\n"
               "       bfs --rmat SCALE[:EF] [<src>] [flags]\n"
               "flags: --gpus P | --virtual-ranks P | --cpu | --device D\n"
               "       --mode ref|td|bu|do|simple|scan  --alpha A --beta B --bu-lane-limit K\n"
               "       --rmat SCALE[:EF] | --uniform N:M   --seed S\n"
               "       --roots K (random sources, GTEPS summary)  --no-oracle  --validate\n"
               "       --levels-out FILE  --cache FILE (write binary CSR)  --json  --quiet  --phase-timing\n"
               "       --directed (edge list as directed u->v pairs, like the reference's stdin reader;\n"
               "                   top-down modes only)\n"
               "       --level-csv FILE (per-level records of every run: root,level,dir,frontier,...,ms)\n");
  std::exit(2);
}

Args parse(int argc, char** argv) {
  Args a;
  std::vector<std::string> pos;
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) usage(("missing value for " + s).c_str());
      return argv[++i];
    };
    if (s == "--gpus") a.gpus = std::stoi(next());
    else if (s == "--virtual-ranks") a.virtual_ranks = std::stoi(next());
    else if (s == "--device") a.device = std::stoi(next());
    else if (s == "--cpu") a.cpu = true;
    else if (s == "--mode") a.mode = next();
    else if (s == "--alpha") a.alpha = std::stod(next());
    else if (s == "--beta") a.beta = std::stod(next());
    else if (s == "--bu-lane-limit") a.bu_lane_limit = std::stoi(next());
    else if (s == "--rmat") {
      std::string v = next();
      auto c = v.find(':');
      a.rmat_scale = std::stoi(v.substr(0, c));
      if (c != std::string::npos) a.rmat_ef = std::stoi(v.substr(c + 1));
    } else if (s == "--uniform") {
      std::string v = next();
      auto c = v.find(':');
      if (c == std::string::npos) usage("--uniform expects N:M");
      a.uni_n = std::stoll(v.substr(0, c));
      a.uni_m = std::stoll(v.substr(c + 1));
    } else if (s == "--seed") a.seed = std::stoull(next());
    else if (s == "--roots") a.roots = std::stoi(next());
    else if (s == "--no-oracle") a.oracle = false;
    else if (s == "--validate") a.validate = true;
    else if (s == "--levels-out") a.levels_out = next();
    else if (s == "--cache") a.cache_out = next();
    else if (s == "--json") a.json = true;
    else if (s == "--level-csv") a.level_csv = next();
    else if (s == "--quiet") a.quiet = true;
    else if (s == "--phase-timing") a.phase_timing = true;
    else if (s == "--no-hub-sort") a.hub_sort = false;
    else if (s == "--directed") a.directed = true;
    else if (s == "-h" || s == "--help") usage();
    else if (!s.empty() && s[0] == '-' && s.size() > 1 && !std::isdigit(static_cast<unsigned char>(s[1])))
      usage(("unknown flag " + s).c_str());
    else pos.push_back(s);
  }
  const bool synth = a.rmat_scale > 0 || a.uni_n > 0;
  if (!synth) {
    if (pos.size() != 2) usage("expected <src> <edge-list> (reference argument order)");
    a.path = pos[1];
  } else if (pos.size() > 1) {
    usage("synthetic graphs take at most one positional argument (<src>)");
  }
  if (!pos.empty()) {
    char* end = nullptr;
    a.src = std::strtoll(pos[0].c_str(), &end, 10);
    if (!end || *end) usage("source vertex must be an integer");
    a.src_given = true;
  }
  if (a.gpus < 1) usage("--gpus must be >= 1");
  if (a.directed) {
    // bottom-up searches in-edges, which a directed CSR does not hold; the
    // Graph500 checks assume an undirected graph
    if (synth) usage("--directed applies to edge-list input only");
    if (a.mode == "bu") usage("--directed needs a top-down mode (td, ref, simple, scan)");
    if (a.mode == "do") a.mode = "td";
    if (a.validate) usage("--validate checks undirected graphs only (the oracle comparison stays on)");
  }
  return a;
}

int env_int(const char* k, int dflt) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : dflt;
}

// One rank's state.
struct RankCtx {
  std::unique_ptr<Backend> be;
  std::shared_ptr<Comm> comm;
  std::unique_ptr<DeviceGraph> graph;
  std::unique_ptr<Engine> engine;
};

// The peer-memory communicator over `inner` when every rank maps every window
// and its self-test passes (both agreed over the bootstrap / inner), else
// `inner` -- or an error when the peer transport was asked for.
std::shared_ptr<Comm> try_peer(std::shared_ptr<Bootstrap> boot, Backend& be, std::shared_ptr<Comm> inner,
                               bool required, bool report) {
  std::string why;
  try {
    // (DBFS_PEER_SLOT_KB, when set, overrides: small slots exercise the
    // slot-sized rounds of large collectives in tests)
    const size_t slot = std::getenv("DBFS_PEER_SLOT_KB") ? static_cast<size_t>(env_int("DBFS_PEER_SLOT_KB", 0)) << 10
                                                         : static_cast<size_t>(env_int("DBFS_PEER_SLOT_MB", 16)) << 20;
    auto pc = std::make_shared<PeerComm>(boot, be, inner, slot);
    if (pc->self_test(&why)) return pc;
  } catch (const std::exception& e) {
    why = e.what();
  }
  if (required) throw Error("DBFS_COMM=peer: peer communicator unavailable: " + why);
  if (report) std::fprintf(stderr, "[bfs] peer communicator unavailable (%s); using %s\n", why.c_str(), inner->name().c_str());
  return inner;
}

// One thread per local rank.  A rank that throws aborts the virtual group so
// its peers fail at their next collective instead of waiting forever.
void run_ranks(std::vector<RankCtx>& ranks, const std::function<void(int, RankCtx&)>& fn,
               VirtualGroup* group = nullptr) {
  if (ranks.size() == 1) {
    fn(0, ranks[0]);
    return;
  }
  std::vector<std::thread> th;
  std::vector<std::exception_ptr> errs(ranks.size());
  for (size_t r = 0; r < ranks.size(); ++r)
    th.emplace_back([&, r] {
      try {
        fn(static_cast<int>(r), ranks[r]);
      } catch (const std::exception& e) {
        errs[r] = std::current_exception();
        if (group) group->abort("rank " + std::to_string(r) + ": " + e.what());
      } catch (...) {
        errs[r] = std::current_exception();
        if (group) group->abort("rank " + std::to_string(r) + " failed");
      }
    });
  for (auto& t : th) t.join();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
}

std::string json_run(const RunResult& r, const std::string& graph, int64_t n, int64_t m, int P, const char* mode,
                     const std::string& backend, const std::string& comm, const std::string& ingest = "") {
  std::string s = "{\"graph\":\"" + graph + "\",\"n\":" + std::to_string(n) + ",\"m\":" + std::to_string(m) +
                  ",\"ranks\":" + std::to_string(P) + ",\"mode\":\"" + mode + "\",\"backend\":\"" + backend +
                  "\",\"comm\":\"" + comm + "\",\"source\":" + std::to_string(r.source) + ",\"ms\":" + std::to_string(r.ms) +
                  ",\"reached\":" + std::to_string(r.reached) + ",\"edges\":" + std::to_string(r.edges) +
                  ",\"gteps\":" + std::to_string(r.gteps) + ",\"depth\":" + std::to_string(r.depth) +
                  (ingest.empty() ? std::string() : ",\"ingest\":" + ingest) + ",\"levels\":[";
  for (size_t i = 0; i < r.levels.size(); ++i) {
    const auto& l = r.levels[i];
    if (i) s += ",";
    s += "{\"l\":" + std::to_string(l.level) + ",\"dir\":\"" + std::string(1, l.direction) +
         "\",\"frontier\":" + std::to_string(l.frontier) + ",\"edges\":" + std::to_string(l.frontier_edges) +
         ",\"new\":" + std::to_string(l.discovered) + ",\"ms\":" + std::to_string(l.ms) + "}";
  }
  return s + "]}";
}

// Backends and communicators of this process's ranks (one for a process of
// a multi-process job): RCCL + peer windows, TCP, virtual ranks or local.
// Returns the virtual group when the ranks are virtual.
std::shared_ptr<VirtualGroup> make_ranks(const Args& a, int P, bool multiproc, int wrank, int world, bool leader,
                                         std::vector<RankCtx>& ranks) {
  const int nlocal = static_cast<int>(ranks.size());
  std::shared_ptr<VirtualGroup> vgroup;
  if (a.virtual_ranks > 0 && !multiproc) vgroup = std::make_shared<VirtualGroup>(P);
  const char* dev_pin = std::getenv("DBFS_DEVICE");  // several processes on one GPU (tests)
  const char* cm_env = std::getenv("DBFS_COMM");
  const std::string cm = cm_env ? cm_env : "";
  const bool want_peer = !a.cpu && (cm.empty() || cm == "peer");
  for (int i = 0; i < nlocal; ++i) {
    if (a.cpu) ranks[i].be = make_cpu_backend();
    else if (multiproc) ranks[i].be = make_hip_backend(dev_pin ? std::atoi(dev_pin) : env_int("LOCAL_RANK", 0));
    else if (a.virtual_ranks > 0) ranks[i].be = make_hip_backend(a.device);
    else ranks[i].be = make_hip_backend(P > 1 ? (dev_pin ? std::atoi(dev_pin) : i) : a.device);
  }
  // one process, P ranks pinned to one device (DBFS_DEVICE: the --gpus P
  // path rehearsed on one GPU): every free deferred to the end, so no rank's
  // hipFree waits for a peer's kernel spinning on that rank's next collective
  if (!multiproc && !a.cpu && a.virtual_ranks == 0 && P > 1 && dev_pin)
    for (auto& r : ranks) r.be->set_deferred_frees(true);
  if (multiproc) {
    const char* addr = std::getenv("MASTER_ADDR");
    const int port = env_int("DBFS_BOOTSTRAP_PORT", env_int("MASTER_PORT", 29500) + 1);
    auto boot = std::make_shared<TcpBootstrap>(addr ? addr : "127.0.0.1", port, wrank, world);
    auto make_rccl = [&]() -> std::shared_ptr<Comm> {
      // every rank takes part in the id broadcast before anything can fail
      // (an empty id: rank 0 could not make one), so the bootstrap's message
      // sequence stays aligned for the agreement after a failure
      std::string uid, why;
      if (wrank == 0) {
        try {
          uid = NcclComm::unique_id();
        } catch (const std::exception& e) {
          why = e.what();
        }
      }
      uid = boot->broadcast(uid);
      if (uid.empty()) throw Error(why.empty() ? "rank 0 could not create the RCCL id" : why);
      return std::make_shared<NcclComm>(uid, wrank, world, *ranks[0].be);
    };
    if (a.cpu || cm == "tcp") {
      // host transport (CPU ranks; debug)
      ranks[0].comm = std::make_shared<TcpComm>(boot, *ranks[0].be);
    } else if (cm == "rccl") {
      ranks[0].comm = make_rccl();
    } else {
      // the peer windows over a TCP inner communicator (setup agreements
      // only: every payload goes through the windows); RCCL (bounded setup,
      // agreed) only when the windows are unavailable on separate GPUs
      auto tcp = std::make_shared<TcpComm>(boot, *ranks[0].be);
      ranks[0].comm = try_peer(boot, *ranks[0].be, tcp, cm == "peer", leader);
      if (ranks[0].comm == tcp && !dev_pin) {
        std::shared_ptr<Comm> rc;
        std::string err;
        try {
          rc = make_rccl();
        } catch (const std::exception& e) {
          err = e.what();
        }
        std::string first;
        for (const auto& e : boot->allgather(err))
          if (first.empty()) first = e;
        if (first.empty()) ranks[0].comm = rc;
        else if (leader) std::fprintf(stderr, "[bfs] RCCL unavailable (%s); using tcp\n", first.c_str());
      }
    }
  } else if (vgroup) {
    for (int i = 0; i < P; ++i) ranks[i].comm = std::make_shared<VirtualComm>(vgroup, i, *ranks[i].be);
  } else if (P > 1) {
    // one process, P GPUs: the peer windows (device pointers, peer access)
    // over an in-process host communicator; ncclCommInitAll only when the
    // windows are unavailable (or DBFS_COMM=rccl)
    bool peer_ok = false;
    if (want_peer) {
      auto igroup = std::make_shared<VirtualGroup>(P);
      auto pgroup = std::make_shared<VirtualGroup>(P);
      std::vector<std::shared_ptr<Comm>> inner(static_cast<size_t>(P));
      for (int i = 0; i < P; ++i) inner[i] = std::make_shared<VirtualComm>(igroup, i, *ranks[i].be);
      run_ranks(ranks, [&](int i, RankCtx& rc) {
        rc.comm = try_peer(std::make_shared<GroupBootstrap>(pgroup, i), *rc.be, inner[i], cm == "peer", i == 0);
      }, pgroup.get());
      peer_ok = ranks[0].comm != inner[0];
    }
    if (!peer_ok) {
      std::vector<Backend*> bes;
      for (auto& r : ranks) bes.push_back(r.be.get());
      auto comms = NcclComm::init_all(bes);
      for (int i = 0; i < P; ++i) ranks[i].comm = std::move(comms[i]);
    }
  } else {
    ranks[0].comm = std::make_shared<LocalComm>(*ranks[0].be);
  }
  return vgroup;
}

// K random roots of degree >= 1 (the same sequence on every rank; a
// multi-process job asks each vertex's owner for its degree).
std::vector<int64_t> sample_roots(const Args& a, const Partition& part, std::vector<RankCtx>& ranks, bool multiproc,
                                  int wrank) {
  std::mt19937_64 rng(a.seed * 7919 + 17);
  std::vector<int64_t> roots;
  int tries = 0;
  while (static_cast<int>(roots.size()) < a.roots && tries < 100 * a.roots) {
    ++tries;
    const int64_t v = static_cast<int64_t>(rng() % static_cast<uint64_t>(part.n));
    const int own = part.owner(v);
    int64_t deg = 0;
    if (!multiproc) {
      deg = ranks[own].graph->degrees_of({v - part.lo(own)})[0];
    } else {
      const int64_t d = own == wrank ? ranks[0].graph->degrees_of({v - part.lo(own)})[0] : 0;
      deg = ranks[0].comm->sum_host(d);
    }
    if (deg > 0) roots.push_back(v);
  }
  return roots;
}

}  // namespace

int main(int argc, char** argv) {
  Args a = parse(argc, argv);
  const int world = env_int("WORLD_SIZE", 1);
  const int wrank = env_int("RANK", 0);
  const bool multiproc = world > 1;
  const bool leader = !multiproc || wrank == 0;
  const bool ref_lines = !a.quiet && leader;
  try {
    // ranks of this job (P) and of this process (nlocal)
    int P = 1;
    if (multiproc) P = world;
    else if (a.virtual_ranks > 0) P = a.virtual_ranks;
    else if (!a.cpu) P = a.gpus;
    const int nlocal = multiproc ? 1 : P;
    // Several ranks reading an edge-list / .mtx file / binary cache: every rank
    // parses only its byte range (or its rows) and builds its shard on its
    // device (DeviceGraph::from_file).  The reference reads and builds the
    // whole graph on every rank (bfs_mpi.cu:815); here only the leader reads
    // the whole file, and only for the CPU oracle (--no-oracle: not at all;
    // the device validator then checks the levels).
    const bool sharded = !a.path.empty() && a.path != "-" && !a.directed && P > 1;
    if (sharded && !a.oracle) a.validate = true;

    // ---- graph ingestion ----
    HostCSR full;
    bool have_host = false;
    std::string gname;
    GenParams gp;
    bool synth = false;
    if (!a.path.empty()) {
      gname = a.path;
      if (ref_lines) std::printf("%s\n", a.path.c_str());
      if (!sharded) {
        if (a.path != "-" && is_binary_csr(a.path)) {
          full = read_binary_csr(a.path);
        } else {
          ReadOptions ro;
          ro.verbose_reference_lines = ref_lines;
          EdgeList el = read_edge_list(a.path, ro);
          full = build_csr(el, a.directed);
        }
        have_host = true;
        if (ref_lines) std::printf("finish load graph\n");
      }
    } else {
      synth = true;
      if (a.rmat_scale > 0) {
        gp = rmat_params(a.rmat_scale, a.rmat_ef, a.seed);
        gname = "rmat" + std::to_string(a.rmat_scale) + "_ef" + std::to_string(a.rmat_ef);
      } else {
        gp = uniform_params(a.uni_n, a.uni_m, a.seed);
        gname = "uniform_n" + std::to_string(a.uni_n) + "_m" + std::to_string(a.uni_m);
      }
      // Host copy only when the CPU oracle / cache / CPU backend needs it.
      if ((a.oracle && leader) || !a.cache_out.empty()) {
        EdgeList el;
        el.n = gp.n;
        el.u.resize(static_cast<size_t>(gp.m));
        el.v.resize(static_cast<size_t>(gp.m));
        for (int64_t i = 0; i < gp.m; ++i) {
          uint64_t u, v;
          gen_edge(gp, static_cast<uint64_t>(i), u, v);
          el.u[i] = static_cast<vid_t>(u);
          el.v[i] = static_cast<vid_t>(v);
        }
        full = build_csr(el);
        have_host = true;
      }
    }
    // the reference's lines after the load, and the CPU oracle
    // (bfs.cu:789-802) on the leader
    std::vector<lvl_t> expected;
    auto print_graph_and_oracle = [&](int64_t n, int64_t directed_edges) {
      if (ref_lines) {
        std::printf("Number of vertices %lld\n", static_cast<long long>(n));
        std::printf("Number of edges %lld\n\n", static_cast<long long>(directed_edges));
      }
      if (!a.cache_out.empty() && leader && have_host) write_binary_csr(a.cache_out, full);
      if (a.src < 0 || a.src >= n)
        throw Error("source vertex " + std::to_string(a.src) + " out of range [0, " + std::to_string(n) + ")");
      if (a.oracle && leader) {
        if (sharded && !have_host) {
          // the whole graph on the leader only, for the oracle (not timed)
          if (is_binary_csr(a.path)) {
            full = read_binary_csr(a.path);
          } else {
            EdgeList el = read_edge_list(a.path, ReadOptions{});
            full = build_csr(el, false);
          }
          have_host = true;
        }
        if (ref_lines) std::printf("Starting sequential bfs.\n");
        auto c0 = std::chrono::steady_clock::now();
        expected = cpu_bfs(full, a.src).level;
        auto c1 = std::chrono::steady_clock::now();
        if (ref_lines)
          std::printf("Elapsed time in milliseconds : %li ms.\n\n",
                      static_cast<long>(std::chrono::duration_cast<std::chrono::milliseconds>(c1 - c0).count()));
      }
    };
    if (!sharded)
      print_graph_and_oracle(have_host ? full.n : gp.n, have_host ? full.directed_edges() : 2 * gp.m);

    // ---- ranks / devices ----
    std::vector<RankCtx> ranks(static_cast<size_t>(nlocal));
    if (!a.cpu && ref_lines && !sharded) std::printf("Enabling peer access between GPU0 and GPU1...\n");
    std::shared_ptr<VirtualGroup> vgroup = make_ranks(a, P, multiproc, wrank, world, leader, ranks);

    Partition part;
    if (sharded) {
      // every rank its byte range (host threads shared among this process's ranks)
      const int threads = std::max(1, static_cast<int>(std::thread::hardware_concurrency()) / nlocal);
      run_ranks(ranks, [&](int i, RankCtx& rc) {
        rc.graph = DeviceGraph::from_file(*rc.be, *rc.comm, a.path, std::min(threads, 16));
      }, vgroup.get());
      const DeviceGraph& g0 = *ranks[0].graph;
      part = g0.partition();
      if (ref_lines) {
        std::printf("nodes num: %lld\n", static_cast<long long>(g0.n()));
        std::printf("edge num: %lld\n", static_cast<long long>(g0.input_edges()));
        std::printf("finish load graph\n");
      }
      int64_t nnz = 0;
      if (multiproc) nnz = ranks[0].comm->sum_host(g0.nnz());
      else
        for (auto& r : ranks) nnz += r.graph->nnz();
      print_graph_and_oracle(g0.n(), nnz);
      if (!a.cpu && ref_lines) std::printf("Enabling peer access between GPU0 and GPU1...\n");
    } else {
      part = Partition::block(have_host ? full.n : gp.n, P);
    }
    const int64_t n = part.n;
    const int64_t m_in = sharded ? ranks[0].graph->input_edges() : have_host ? full.input_edges : gp.m;

    EngineOptions eo;
    eo.mode = parse_mode(a.mode);
    eo.alpha = a.alpha;
    eo.beta = a.beta;
    eo.bu_lane_limit = a.bu_lane_limit;
    eo.phase_timing = a.phase_timing;
    eo.directed = a.directed;
    run_ranks(ranks, [&](int i, RankCtx& rc) {
      const int rk = multiproc ? wrank : i;
      if (synth) rc.graph = DeviceGraph::generate(*rc.be, gp, part, rk);
      else if (!sharded) rc.graph = DeviceGraph::from_host(*rc.be, full, part, rk);
      if (a.hub_sort) rc.graph->sort_neighbors_by_degree(*rc.comm);
      rc.engine = std::make_unique<Engine>(*rc.graph, *rc.comm, eo);
    }, vgroup.get());
    // what every rank parsed (sharded reads): [byte_begin, byte_end, edges] per rank
    std::string ingest_json;
    if (sharded) {
      std::vector<int64_t> b, e, m;
      if (multiproc) {
        const auto& gi = ranks[0].graph->ingest();
        b = ranks[0].comm->allgather_host_i64(gi.byte_begin);
        e = ranks[0].comm->allgather_host_i64(gi.byte_end);
        m = ranks[0].comm->allgather_host_i64(gi.edges);
      } else {
        for (auto& r : ranks) {
          b.push_back(r.graph->ingest().byte_begin);
          e.push_back(r.graph->ingest().byte_end);
          m.push_back(r.graph->ingest().edges);
        }
      }
      ingest_json = "[";
      for (size_t r = 0; r < b.size(); ++r)
        ingest_json += (r ? ",[" : "[") + std::to_string(b[r]) + "," + std::to_string(e[r]) + "," +
                       std::to_string(m[r]) + "]";
      ingest_json += "]";
    }

    // ---- the reference's single run from <src> ----
    std::vector<RunResult> res(static_cast<size_t>(nlocal));
    std::vector<lvl_t> got;
    std::vector<std::vector<int64_t>> viol(static_cast<size_t>(nlocal));
    if (ref_lines) std::printf("Starting queue parallel bfs.\n");
    run_ranks(ranks, [&](int i, RankCtx& rc) {
      res[i] = rc.engine->run(a.src);
      std::vector<lvl_t> lv = rc.engine->gather_levels();
      if (i == 0) got = std::move(lv);
      if (a.validate) viol[i] = rc.engine->validate(a.src);
    }, vgroup.get());
    if (ref_lines) std::printf("Elapsed time in milliseconds : %li ms.\n", static_cast<long>(res[0].ms));
    int rc_exit = 0;
    if (leader && !expected.empty()) {
      for (int64_t i = 0; i < n; ++i) {
        if (got[i] != expected[i]) {
          std::printf("%lld %d %d\n", static_cast<long long>(i), got[i], expected[i]);
          std::printf("Wrong output!\n");
          return 1;
        }
      }
      if (!a.quiet) std::printf("Output OK!\n\n");
    }
    if (a.validate && leader) {
      const auto& v = viol[0];
      if (v[0] || v[1] || v[2]) {
        std::printf("Validation FAILED: depth-gap %lld, reached-unreached %lld, orphan %lld\n",
                    static_cast<long long>(v[0]), static_cast<long long>(v[1]), static_cast<long long>(v[2]));
        rc_exit = 1;
      } else if (!a.quiet) {
        std::printf("Validation OK (Graph500 level checks)\n");
      }
    }
    if (!a.levels_out.empty() && leader) write_levels(a.levels_out, got);
    // Per-level profile CSV: one row per level of every run.
    std::FILE* csv = nullptr;
    if (!a.level_csv.empty() && leader) {
      csv = std::fopen(a.level_csv.c_str(), "w");
      DBFS_CHECK(csv != nullptr, "cannot write " + a.level_csv);
      std::fprintf(csv, "root,level,dir,frontier,frontier_edges,discovered,ms,run_ms\n");
    }
    auto csv_run = [&](const RunResult& r) {
      if (!csv) return;
      for (const auto& l : r.levels)
        std::fprintf(csv, "%lld,%d,%c,%lld,%lld,%lld,%.4f,%.4f\n", static_cast<long long>(r.source), l.level,
                     l.direction, static_cast<long long>(l.frontier), static_cast<long long>(l.frontier_edges),
                     static_cast<long long>(l.discovered), l.ms, r.ms);
    };
    csv_run(res[0]);
    const std::string bname = ranks[0].be->name() + (ranks[0].be->device_checks_enabled() ? "+checked" : "");
    if (a.json && leader)
      std::printf("%s\n", json_run(res[0], gname, n, m_in, P, a.mode.c_str(), bname, ranks[0].comm->name(), ingest_json).c_str());

    // ---- optional K random roots (Graph500-style GTEPS) ----
    if (a.roots > 0) {
      const std::vector<int64_t> roots = sample_roots(a, part, ranks, multiproc, wrank);
      double inv_sum = 0, ms_sum = 0;
      int64_t e_sum = 0;
      for (int64_t root : roots) {
        run_ranks(ranks, [&](int i, RankCtx& rc) { res[i] = rc.engine->run(root); }, vgroup.get());
        inv_sum += res[0].gteps > 0 ? 1.0 / res[0].gteps : 0;
        ms_sum += res[0].ms;
        e_sum += res[0].edges;
        if (a.json && leader) std::printf("%s\n", json_run(res[0], gname, n, m_in, P, a.mode.c_str(), bname, ranks[0].comm->name()).c_str());
        csv_run(res[0]);
      }
      if (leader && !roots.empty()) {
        const double hm = inv_sum > 0 ? roots.size() / inv_sum : 0.0;
        std::printf("roots %zu  mean ms %.3f  harmonic-mean GTEPS %.3f  aggregate GTEPS %.3f\n", roots.size(),
                    ms_sum / roots.size(), hm, ms_sum > 0 ? e_sum / (ms_sum * 1e6) : 0.0);
      }
    }
    if (csv) std::fclose(csv);
    return rc_exit;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "bfs: %s\n", e.what());
    return 1;
  }
}
