// Minimal TCP bootstrap (star topology, rank 0 hosts).
//
// Replaces MPI_Init/Comm_rank (bfs_mpi.cu:800-808): there is no MPI on this
// platform, and the launcher (torch.distributed.run or any other) only needs to
// provide RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT.  Used to ship the
// 128-byte RCCL unique id and for host-side barriers.
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <thread>

#include "dbfs/comm.hpp"

namespace dbfs {
namespace {

void write_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) throw Error(std::string("bootstrap send failed: ") + std::strerror(errno));
    c += k;
    n -= static_cast<size_t>(k);
  }
}

// Receive exactly n bytes, each wait bounded by timeout_s (0: unbounded;
// `knob` names the variable that sets it in the error).
void read_all(int fd, void* p, size_t n, double timeout_s, const char* knob) {
  char* c = static_cast<char*>(p);
  while (n) {
    if (timeout_s > 0) {
      pollfd pfd{fd, POLLIN, 0};
      const int pr = ::poll(&pfd, 1, static_cast<int>(std::min(timeout_s * 1000.0, 2.0e9)));
      if (pr < 0 && errno == EINTR) continue;
      if (pr == 0)
        throw Error("bootstrap peer timed out after " + std::to_string(timeout_s) + " s (" + knob +
                    "); a rank stopped participating");
    }
    ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) throw Error("bootstrap peer closed the connection (a rank failed)");
    c += k;
    n -= static_cast<size_t>(k);
  }
}

// Connected sockets: no Nagle.  (Receive waits are bounded per message by
// read_all: the bootstrap's own exchanges by DBFS_BOOTSTRAP_TIMEOUT_S --
// they also wait for the peers' setup: per-rank ingest of a large file, the
// CSR build, hub selection, which can take minutes -- and TcpComm's
// collectives by DBFS_COMM_TIMEOUT_S.  A peer that dies closes its socket
// and fails the wait at once.)
void tune_socket(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

void send_msg(int fd, const std::string& s) {
  const uint64_t n = s.size();
  write_all(fd, &n, sizeof(n));
  if (n) write_all(fd, s.data(), n);
}

// Largest message a peer may announce (DBFS_BOOTSTRAP_MAX_MSG bytes, default
// 4 GiB): a bogus length from a stray or hostile connection is an error, not
// a huge allocation.
uint64_t max_msg_bytes() {
  static const uint64_t v = [] {
    const char* e = std::getenv("DBFS_BOOTSTRAP_MAX_MSG");
    return e && *e ? std::strtoull(e, nullptr, 10) : (uint64_t(1) << 32);
  }();
  return v;
}

// First bytes every connecting rank sends (then its rank): rejects
// connections that are not from this program.
constexpr uint64_t kHelloMagic = 0x31544f4f42534642ull;  // "BFSBOOT1"

std::string recv_msg(int fd, double timeout_s, const char* knob) {
  uint64_t n = 0;
  read_all(fd, &n, sizeof(n), timeout_s, knob);
  if (n > max_msg_bytes())
    throw Error("bootstrap peer announced a " + std::to_string(n) + "-byte message (limit " +
                std::to_string(max_msg_bytes()) + ", DBFS_BOOTSTRAP_MAX_MSG)");
  std::string s(n, '\0');
  if (n) read_all(fd, &s[0], n, timeout_s, knob);
  return s;
}

bool is_literal_ipv4(const std::string& host) {
  in_addr x{};
  return inet_pton(AF_INET, host.c_str(), &x) == 1;
}

sockaddr_in resolve(const std::string& host, int port) {
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res)
      throw Error("bootstrap cannot resolve host " + host);
    a.sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
    freeaddrinfo(res);
  }
  return a;
}

}  // namespace

TcpBootstrap::TcpBootstrap(const std::string& host, int port, int rank, int nranks, double timeout_s)
    : rank_(rank), size_(nranks) {
  DBFS_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "bad bootstrap rank/size");
  if (nranks == 1) return;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  if (rank == 0) {
    listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (listen_fd_ < 0) throw Error("bootstrap socket() failed");
    int one = 1;
    setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(static_cast<uint16_t>(port));
    // Listen on the rendezvous address only, never on every interface unless
    // asked (DBFS_BOOTSTRAP_BIND=any): the handshake is a magic word and a
    // rank number, so an open port would let any host take a rank slot.  A
    // host NAME that resolves to a loopback address here (the usual 127.0.1.1
    // /etc/hosts alias) is bound as such -- every rank of one node reaches it;
    // ranks on other nodes need DBFS_BOOTSTRAP_BIND=any (said on stderr).
    a.sin_addr = resolve(host, port).sin_addr;
    const bool loopback = (ntohl(a.sin_addr.s_addr) >> 24) == 127;
    const char* bind_env = std::getenv("DBFS_BOOTSTRAP_BIND");
    const bool any = bind_env && std::string(bind_env) == "any";
    if (any) a.sin_addr.s_addr = htonl(INADDR_ANY);
    {
      char ip[INET_ADDRSTRLEN] = {0};
      inet_ntop(AF_INET, &a.sin_addr, ip, sizeof(ip));
      const char* verbose = std::getenv("DBFS_BOOTSTRAP_VERBOSE");
      if ((verbose && *verbose == '1') || (loopback && !any && !is_literal_ipv4(host)))
        std::fprintf(stderr, "[dbfs] bootstrap: rank 0 listens on %s:%d%s\n", ip, port,
                     loopback && !any && !is_literal_ipv4(host)
                         ? " (the rendezvous name is a loopback alias here: ranks on other hosts need "
                           "DBFS_BOOTSTRAP_BIND=any)"
                         : "");
    }
    if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0)
      throw Error("bootstrap bind to port " + std::to_string(port) + " failed: " + std::strerror(errno));
    if (::listen(listen_fd_, nranks) != 0) throw Error("bootstrap listen failed");
    peers_.assign(static_cast<size_t>(nranks), -1);
    for (int k = 1; k < nranks; ++k) {
      const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now());
      pollfd pfd{listen_fd_, POLLIN, 0};
      const int pr = left.count() > 0 ? ::poll(&pfd, 1, static_cast<int>(left.count())) : 0;
      if (pr <= 0)
        throw Error("bootstrap: only " + std::to_string(k - 1) + " of " + std::to_string(nranks - 1) +
                    " peers connected within " + std::to_string(timeout_s) + " s");
      int fd = ::accept(listen_fd_, nullptr, nullptr);
      if (fd < 0) throw Error("bootstrap accept failed");
      uint64_t hello = 0;
      int32_t r = -1;
      // a rank sends its hello right after connecting: a connection silent
      // for 10 s (or closed, or speaking another protocol) is not one of ours
      // -- dropped, and the loop keeps waiting for the real peers
      bool ours = false;
      try {
        read_all(fd, &hello, sizeof(hello), 10.0, "hello");
        ours = hello == kHelloMagic;
        if (ours) read_all(fd, &r, sizeof(r), 10.0, "hello");
      } catch (const Error&) {
        ours = false;
      }
      if (!ours) {
        ::close(fd);
        --k;
        continue;
      }
      tune_socket(fd);
      if (r <= 0 || r >= nranks || peers_[r] != -1) throw Error("bootstrap got bad rank " + std::to_string(r));
      peers_[r] = fd;
    }
  } else {
    const sockaddr_in a = resolve(host, port);
    int fd = -1;
    for (;;) {
      fd = ::socket(AF_INET, SOCK_STREAM, 0);
      if (fd < 0) throw Error("bootstrap socket() failed");
      if (::connect(fd, reinterpret_cast<const sockaddr*>(&a), sizeof(a)) == 0) break;
      const int err = errno;
      ::close(fd);
      if (std::chrono::steady_clock::now() > deadline) {
        // (rank 0 listens on the rendezvous address only: a MASTER_ADDR that
        // is a loopback alias on rank 0's host -- 127.0.1.1 in /etc/hosts --
        // is unreachable from other hosts unless rank 0 binds every interface)
        char ip[INET_ADDRSTRLEN] = {0};
        inet_ntop(AF_INET, &a.sin_addr, ip, sizeof(ip));
        throw Error("bootstrap connect to " + host + ":" + std::to_string(port) + " (" + ip + ") timed out after " +
                    std::to_string(static_cast<int>(timeout_s)) + " s: " + std::strerror(err) +
                    " -- is rank 0 up?  A rank on another host needs rank 0 started with DBFS_BOOTSTRAP_BIND=any "
                    "when its MASTER_ADDR resolves to a loopback alias there");
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
    tune_socket(fd);
    const uint64_t hello = kHelloMagic;
    const int32_t r = rank;
    write_all(fd, &hello, sizeof(hello));
    write_all(fd, &r, sizeof(r));
    peers_.assign(1, fd);
  }
}

TcpBootstrap::~TcpBootstrap() {
  for (int fd : peers_)
    if (fd >= 0) ::close(fd);
  if (listen_fd_ >= 0) ::close(listen_fd_);
}

std::string TcpBootstrap::broadcast(const std::string& data, int root) {
  DBFS_CHECK(root == 0, "TcpBootstrap broadcast supports root 0 only");
  if (size_ == 1) return data;
  if (rank_ == 0) {
    for (int r = 1; r < size_; ++r) send_msg(peers_[r], data);
    return data;
  }
  return recv_msg(peers_[0], bootstrap_timeout_s(), "DBFS_BOOTSTRAP_TIMEOUT_S");
}

std::vector<std::string> TcpBootstrap::allgather(const std::string& data) {
  return allgather_within(data, bootstrap_timeout_s(), "DBFS_BOOTSTRAP_TIMEOUT_S");
}

std::vector<std::string> TcpBootstrap::allgather_within(const std::string& data, double timeout_s, const char* knob) {
  std::vector<std::string> out(static_cast<size_t>(size_));
  if (size_ == 1) {
    out[0] = data;
    return out;
  }
  if (rank_ == 0) {
    out[0] = data;
    for (int r = 1; r < size_; ++r) out[r] = recv_msg(peers_[r], timeout_s, knob);
    for (int r = 1; r < size_; ++r)
      for (int k = 0; k < size_; ++k) send_msg(peers_[r], out[k]);
  } else {
    send_msg(peers_[0], data);
    for (int k = 0; k < size_; ++k) out[k] = recv_msg(peers_[0], timeout_s, knob);
  }
  return out;
}

void TcpBootstrap::barrier() { allgather(std::string()); }

}  // namespace dbfs

// ---- TcpComm --------------------------------------------------------------------

namespace dbfs {

// (TcpComm's collectives are traversal collectives: the shorter bound)
static const char* const kCommKnob = "DBFS_COMM_TIMEOUT_S";

TcpComm::TcpComm(std::shared_ptr<TcpBootstrap> boot, Backend& be) : boot_(std::move(boot)) { bind_backend(&be); }
int TcpComm::rank() const { return boot_->rank(); }
int TcpComm::size() const { return boot_->size(); }

std::string TcpComm::fetch(const void* p, size_t bytes) {
  std::string s(bytes, '\0');
  if (bytes) be_->to_host(&s[0], p, bytes);
  return s;
}

void TcpComm::store(void* p, const std::string& s, size_t off, size_t bytes) {
  if (bytes) be_->to_device(p, s.data() + off, bytes);
}

void TcpComm::alltoall(const void* send, void* recv, size_t bytes) {
  note(kAllToAll, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(bytes));
  const int P = size(), me = rank();
  auto all = boot_->allgather_within(fetch(send, bytes * P), comm_timeout_s(), kCommKnob);
  for (int r = 0; r < P; ++r) store(static_cast<char*>(recv) + r * bytes, all[r], me * bytes, bytes);
}

void TcpComm::allgather(const void* send, void* recv, size_t bytes) {
  note(kAllGather, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(bytes));
  auto all = boot_->allgather_within(fetch(send, bytes), comm_timeout_s(), kCommKnob);
  for (int r = 0; r < size(); ++r) store(static_cast<char*>(recv) + r * bytes, all[r], 0, bytes);
}

void TcpComm::allreduce_sum_i64(int64_t* buf, size_t count) {
  note(kAllReduce, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(count) * 8);
  auto all = boot_->allgather_within(fetch(buf, count * sizeof(int64_t)), comm_timeout_s(), kCommKnob);
  // two's-complement (wrapping) sums, as RCCL's: the engine also reduces
  // disjoint bit sets (hub frontier words) and, on no-op chains, stale blocks
  std::vector<uint64_t> acc(count, 0);
  for (const auto& s : all)
    for (size_t i = 0; i < count; ++i) {
      uint64_t x;
      std::memcpy(&x, s.data() + i * sizeof(uint64_t), sizeof(x));
      acc[i] += x;
    }
  be_->to_device(buf, acc.data(), count * sizeof(int64_t));
}

void TcpComm::alltoallv(const void* send, const int64_t* sc, const int64_t* sd, void* recv, const int64_t* rc,
                        const int64_t* rd, size_t eb) {
  note_alltoallv(sc, eb);
  const int P = size(), me = rank();
  // message: P (offset, count) pairs, then the concatenated pieces
  std::string msg(static_cast<size_t>(P) * 2 * sizeof(int64_t), '\0');
  int64_t off = 0;
  std::string data;
  for (int r = 0; r < P; ++r) {
    const int64_t hdr[2] = {off, sc[r]};
    std::memcpy(&msg[static_cast<size_t>(r) * 2 * sizeof(int64_t)], hdr, sizeof(hdr));
    data += fetch(static_cast<const char*>(send) + sd[r] * eb, static_cast<size_t>(sc[r]) * eb);
    off += sc[r];
  }
  auto all = boot_->allgather_within(msg + data, comm_timeout_s(), kCommKnob);
  for (int r = 0; r < P; ++r) {
    int64_t hdr[2];
    std::memcpy(hdr, all[r].data() + static_cast<size_t>(me) * 2 * sizeof(int64_t), sizeof(hdr));
    DBFS_CHECK(hdr[1] == rc[r], "TcpComm alltoallv count mismatch");
    const size_t base = static_cast<size_t>(P) * 2 * sizeof(int64_t) + static_cast<size_t>(hdr[0]) * eb;
    store(static_cast<char*>(recv) + rd[r] * eb, all[r], base, static_cast<size_t>(hdr[1]) * eb);
  }
}

void TcpComm::barrier() {
  note(kBarrier, 0);
  be_->synchronize();
  boot_->allgather_within(std::string(), comm_timeout_s(), kCommKnob);
}

}  // namespace dbfs
