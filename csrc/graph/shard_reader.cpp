// Sharded, multi-threaded edge-list reader: rank r of P parses only its byte
// range of the file (plus the one token past its end that completes its last
// edge) with T host threads, so no rank holds or scans the whole graph.
//
// Reference being replaced: readGraphFromFile (bfs.cu:829-880) -- one thread
// reads the whole file into vector<vector<int>> -- which bfs_mpi.cu:815 runs on
// EVERY rank.  Here the edges a rank parsed go to the GPU and are routed to
// their owners there (DeviceGraph::from_edges: count -> all-to-all-v -> count
// -> scan -> fill).
//
// Formats (same semantics as the whole-file reader, io.cpp):
//   * reference: `n m` then m pairs `u v` (0-based), any whitespace layout --
//     the byte ranges are cut at token boundaries; edge i is tokens 2i, 2i+1
//     of the body, emitted by the rank whose range holds token 2i;
//   * MatrixMarket: banner, `%` comments, `rows cols nnz`, then one entry
//     `i j [value]` per line (1-based) -- ranges cut at line starts.
// Extra tokens / entries after the m-th edge are ignored, fewer are an error,
// ids out of range are an error (every rank throws the same message).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <thread>

#include "dbfs/shard_reader.hpp"

namespace dbfs {

namespace {

constexpr vid_t kBadId = 0xFFFFFFFFu;  // never a vertex: n <= 2^32 - 1

struct Mapped {
  const char* data = nullptr;
  size_t size = 0;
  int fd = -1;
  explicit Mapped(const std::string& path) {
    fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw Error("not open " + path);
    struct stat st {};
    if (::fstat(fd, &st) != 0) {
      ::close(fd);
      throw Error("cannot stat " + path);
    }
    size = static_cast<size_t>(st.st_size);
    if (size > 0) {
      void* p = ::mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
      if (p == MAP_FAILED) {
        ::close(fd);
        throw Error("cannot mmap " + path);
      }
      data = static_cast<const char*>(p);
    }
  }
  ~Mapped() {
    if (data) ::munmap(const_cast<char*>(data), size);
    if (fd >= 0) ::close(fd);
  }
  // only this rank's range is touched: tell the kernel to read ahead there
  void advise(size_t b, size_t e) const {
    if (!data || b >= e) return;
    const size_t pg = static_cast<size_t>(::sysconf(_SC_PAGESIZE));
    const size_t a = b / pg * pg;
    ::madvise(const_cast<char*>(data) + a, e - a, MADV_SEQUENTIAL);
    ::madvise(const_cast<char*>(data) + a, e - a, MADV_WILLNEED);
  }
};

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }
inline bool is_digit(char c) { return c >= '0' && c <= '9'; }

// Header integers (reference `n m`; MatrixMarket size line after banner and comments).
struct Header {
  int64_t n = 0, m = 0;
  size_t body = 0;  // first byte after the header
  bool mtx = false;
};

bool read_header_int(const char* d, size_t size, size_t& p, int64_t& out) {
  while (p < size && is_space(d[p])) ++p;
  if (p >= size) return false;
  bool neg = false;
  if (d[p] == '-' || d[p] == '+') {
    neg = d[p] == '-';
    ++p;
  }
  if (p >= size || !is_digit(d[p])) return false;
  int64_t v = 0;
  while (p < size && is_digit(d[p])) {
    if (v > (INT64_MAX - 9) / 10) return false;
    v = v * 10 + (d[p] - '0');
    ++p;
  }
  out = neg ? -v : v;
  return true;
}

Header parse_header(const Mapped& f, const std::string& path) {
  Header h;
  const char* d = f.data;
  const size_t size = f.size;
  size_t p = 0;
  if (size >= 14 && (std::memcmp(d, "%%MatrixMarket", 14) == 0 || std::memcmp(d, "%%matrixmarket", 14) == 0)) {
    h.mtx = true;
    // banner, then blank / '%' lines, then the size line
    for (;;) {
      while (p < size && d[p] != '\n') ++p;
      if (p < size) ++p;
      size_t q = p;
      while (q < size && (d[q] == ' ' || d[q] == '\t' || d[q] == '\r')) ++q;
      if (q < size && (d[q] == '%' || d[q] == '\n')) continue;
      break;
    }
    int64_t rows = 0, cols = 0, nnz = 0;
    if (!read_header_int(d, size, p, rows) || !read_header_int(d, size, p, cols) ||
        !read_header_int(d, size, p, nnz))
      throw Error("bad MatrixMarket size line in " + path);
    while (p < size && d[p] != '\n') ++p;  // rest of the size line
    h.n = std::max(rows, cols);
    h.m = nnz;
  } else {
    if (!read_header_int(d, size, p, h.n) || !read_header_int(d, size, p, h.m))
      throw Error("bad header (expected `n m`) in " + path);
  }
  if (h.n < 0 || h.m < 0) throw Error("negative n or m in " + path);
  if (h.n > int64_t(UINT32_MAX)) throw Error("vertex count exceeds 2^32 in " + path);
  h.body = p;
  return h;
}

// Cut [body, size) into k ranges: reference format at token boundaries,
// MatrixMarket at line starts.  Every caller computes the same cuts.
size_t align_cut(const char* d, size_t size, size_t body, size_t pos, bool lines) {
  if (pos <= body) return body;
  if (pos >= size) return size;
  if (lines) {
    while (pos < size && d[pos - 1] != '\n') ++pos;
  } else {
    while (pos < size && !is_space(d[pos - 1]) && !is_space(d[pos])) ++pos;
  }
  return pos;
}

size_t cut(const char* d, size_t size, size_t body, int64_t i, int64_t k, bool lines) {
  const size_t len = size - body;
  const size_t pos = body + static_cast<size_t>((static_cast<unsigned __int128>(len) * static_cast<uint64_t>(i)) /
                                                static_cast<uint64_t>(k));
  return align_cut(d, size, body, pos, lines);
}

// One parsed integer token as a vertex id (kBadId: negative, too long, or >= n
// after the 1-based shift).
inline vid_t parse_token(const char* d, size_t e, size_t& p, int64_t n, int64_t shift, bool& malformed) {
  bool neg = false;
  if (d[p] == '-' || d[p] == '+') {
    neg = d[p] == '-';
    ++p;
  }
  if (p >= e || !is_digit(d[p])) {
    malformed = true;
    return kBadId;
  }
  uint64_t v = 0;
  bool big = false;
  while (p < e && is_digit(d[p])) {
    if (v < (uint64_t(1) << 40)) v = v * 10 + static_cast<uint64_t>(d[p] - '0');
    else big = true;
    ++p;
  }
  if (p < e && !is_space(d[p])) malformed = true;  // e.g. "12x"
  if (neg || big || malformed) return kBadId;
  const int64_t id = static_cast<int64_t>(v) - shift;
  return (id >= 0 && id < n) ? static_cast<vid_t>(id) : kBadId;
}

// Pages of [b, e) that lie wholly inside it and that a parse has passed:
// dropped from this process (MAP_PRIVATE, never written, so a later touch
// just faults the page back in from the page cache).  Keeps the resident set
// to the parsed arrays plus a window per thread, not the whole byte range.
struct PageDropper {
  const char* d;
  size_t pg, lo, done;
  PageDropper(const char* data, size_t b) : d(data), pg(static_cast<size_t>(::sysconf(_SC_PAGESIZE))) {
    lo = (b + pg - 1) / pg * pg;  // first page wholly inside the range
    done = lo;
  }
  void passed(size_t p, bool final = false) {
    const size_t hi = p / pg * pg;
    if (hi > done && (final || hi - done >= (size_t(64) << 20))) {
      ::madvise(const_cast<char*>(d) + done, hi - done, MADV_DONTNEED);
      done = hi;
    }
  }
};

// Reference-format tokens of [b, e): count them, then (second pass) hand
// token j of the range to emit(j, id) (kBadId marks a malformed or
// out-of-range id, an error only if one of the m edges uses it).
int64_t count_tokens(const char* d, size_t b, size_t e) {
  PageDropper drop(d, b);
  int64_t c = 0;
  bool prev_space = true;
  for (size_t p0 = b; p0 < e; p0 += size_t(1) << 20) {
    const size_t p1 = std::min(e, p0 + (size_t(1) << 20));
    for (size_t p = p0; p < p1; ++p) {
      const bool sp = is_space(d[p]);
      c += prev_space && !sp;
      prev_space = sp;
    }
    drop.passed(p1);
  }
  drop.passed(e, true);
  return c;
}

template <class Emit>
void parse_tokens(const char* d, size_t b, size_t e, int64_t n, Emit&& emit) {
  PageDropper drop(d, b);
  size_t p = b;
  int64_t j = 0;
  while (p < e) {
    while (p < e && is_space(d[p])) ++p;
    if (p >= e) break;
    bool mal = false;
    emit(j++, parse_token(d, e, p, n, 0, mal));
    while (p < e && !is_space(d[p])) ++p;
    if ((j & 0xFFFF) == 0) drop.passed(p);
  }
  drop.passed(e, true);
}

// MatrixMarket entry lines of [b, e) as pairs (two tokens each); blank and
// '%' lines skipped.  emit == nullptr-like counting when Count is true.
template <bool Count, class Emit>
int64_t parse_mtx_lines(const char* d, size_t b, size_t e, int64_t n, Emit&& emit) {
  PageDropper drop(d, b);
  size_t p = b;
  int64_t j = 0;
  while (p < e) {
    size_t q = p;
    while (q < e && (d[q] == ' ' || d[q] == '\t' || d[q] == '\r')) ++q;
    if (q >= e) break;
    if (d[q] == '\n' || d[q] == '%') {  // blank or comment line
      while (q < e && d[q] != '\n') ++q;
      p = q + 1;
      continue;
    }
    if constexpr (!Count) {
      bool mal = false;
      const vid_t a = parse_token(d, e, q, n, 1, mal);
      while (q < e && (d[q] == ' ' || d[q] == '\t')) ++q;
      vid_t c = kBadId;
      if (q < e && d[q] != '\n' && d[q] != '\r') c = parse_token(d, e, q, n, 1, mal);
      emit(j, a);
      emit(j + 1, c);
    }
    if ((j & 0xFFFF) == 0) drop.passed(q);
    j += 2;
    while (q < e && d[q] != '\n') ++q;  // value column(s)
    p = q + 1;
  }
  drop.passed(e, true);
  return j;
}

}  // namespace

EdgeShard read_edge_shard(const std::string& path, int rank, int nranks, const HostAllgather& allgather,
                          int threads) {
  DBFS_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank / rank count");
  DBFS_CHECK(path != "-", "sharded reads need a file (standard input is read whole)");
  EdgeShard s;
  std::string err;
  Header h;
  // opening / mapping the file and its header: a failure on any rank (the
  // file missing or unreadable on one node only) is agreed, so no rank is
  // left waiting in a later exchange its peers never join
  std::unique_ptr<Mapped> fm;
  try {
    fm = std::make_unique<Mapped>(path);
    h = parse_header(*fm, path);
  } catch (const std::exception& e) {
    err = e.what();
  }
  {
    const auto st = allgather(err.empty() ? 0 : 1);
    for (size_t r = 0; r < st.size(); ++r)
      if (st[r])
        throw Error(err.empty() ? "edge list unreadable on rank " + std::to_string(r) + ": " + path : err);
  }
  const Mapped& f = *fm;
  s.n = h.n;
  s.m = h.m;
  s.format = h.mtx ? FileFormat::MatrixMarket : FileFormat::EdgeList;
  const char* d = f.data;
  const size_t size = f.size;
  const bool lines = h.mtx;
  const size_t rb = cut(d, size, h.body, rank, nranks, lines);
  const size_t re = cut(d, size, h.body, rank + 1, nranks, lines);
  s.byte_begin = static_cast<int64_t>(rb);
  s.byte_end = static_cast<int64_t>(re);
  f.advise(rb, re);

  int T = threads > 0 ? threads : static_cast<int>(std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
  T = static_cast<int>(std::min<size_t>(static_cast<size_t>(T), std::max<size_t>(1, (re - rb) / 4096)));
  std::vector<size_t> cuts(static_cast<size_t>(T) + 1);
  for (int t = 0; t <= T; ++t) {
    const size_t pos = rb + static_cast<size_t>((static_cast<unsigned __int128>(re - rb) * static_cast<uint64_t>(t)) /
                                                 static_cast<uint64_t>(T));
    cuts[t] = t == 0 ? rb : t == T ? re : std::min(re, align_cut(d, size, h.body, pos, lines));
  }
  auto piece = [&](int t, size_t& b, size_t& e) {
    b = std::min(cuts[t], re);
    e = std::max(b, std::min(cuts[t + 1], re));
  };
  auto parallel = [&](auto&& fn) {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back([&, t] { fn(t); });
    for (auto& x : th) x.join();
  };
  // pass 1: token (entry-pair) counts per thread -- a byte scan, no storage
  std::vector<int64_t> tcount(static_cast<size_t>(T) + 1, 0);
  parallel([&](int t) {
    size_t b, e;
    piece(t, b, e);
    tcount[t + 1] = lines ? parse_mtx_lines<true>(d, b, e, h.n, [](int64_t, vid_t) {}) : count_tokens(d, b, e);
  });
  for (int t = 0; t < T; ++t) tcount[t + 1] += tcount[t];
  const int64_t ntok = tcount[T];
  // token (or entry-pair) counts of every rank -> this rank's global position
  const std::vector<int64_t> counts = allgather(ntok);
  int64_t before = 0, total = 0;
  for (int r = 0; r < nranks; ++r) {
    if (r < rank) before += counts[r];
    total += counts[r];
  }
  const int64_t need = 2 * h.m;  // tokens of the m edges
  if (total < need) {
    throw Error(std::string(h.mtx ? "truncated MatrixMarket entries" : "truncated edge list") + " in " + path +
                ": expected " + std::to_string(h.m) + " edges, got " + std::to_string(total / 2));
  }
  // this rank's edges: those whose first token it holds (global index even, < 2m)
  const int64_t g0 = before + (before & 1);  // first even global token index held
  const int64_t g_end = std::min(before + ntok, need);
  const int64_t my_edges = g_end > g0 ? (g_end - g0 + 1) / 2 : 0;
  s.first_edge = g0 / 2;
  s.u.resize(static_cast<size_t>(my_edges));
  s.v.resize(static_cast<size_t>(my_edges));
  // pass 2: every thread parses its piece straight into u / v at its tokens'
  // global positions (no per-thread token vectors, no copy)
  std::vector<int64_t> tbad(static_cast<size_t>(T), INT64_MAX);
  vid_t* const U = s.u.data();
  vid_t* const V = s.v.data();
  parallel([&](int t) {
    size_t b, e;
    piece(t, b, e);
    const int64_t base = before + tcount[t];
    int64_t bad = INT64_MAX;
    auto emit = [&](int64_t j, vid_t x) {
      const int64_t g = base + j;
      if (g < g0 || g >= g_end) return;
      const int64_t k = g - g0;
      (k & 1 ? V : U)[k >> 1] = x;
      if (x == kBadId && (k >> 1) < bad) bad = k >> 1;
    };
    if (lines) parse_mtx_lines<false>(d, b, e, h.n, emit);
    else parse_tokens(d, b, e, h.n, emit);
    tbad[t] = bad;
  });
  int64_t bad_edge = *std::min_element(tbad.begin(), tbad.end());
  if (bad_edge == INT64_MAX) bad_edge = -1;
  int64_t e = my_edges;
  if (g_end > g0 && ((g_end - g0) & 1)) {
    // the second token of the last edge lies past the range: read ahead
    if (lines) {
      // (MatrixMarket entries are whole lines: a pair never straddles a cut)
      throw Error("internal: MatrixMarket entry split across ranks in " + path);
    }
    size_t p = re;
    vid_t x = kBadId;
    while (p < size && is_space(d[p])) ++p;
    bool mal = false;
    if (p < size) x = parse_token(d, size, p, h.n, 0, mal);
    if (x == kBadId && (bad_edge < 0 || my_edges - 1 < bad_edge)) bad_edge = my_edges - 1;
    V[my_edges - 1] = x;
  }
  DBFS_CHECK(e == my_edges, "internal: edge count mismatch in the sharded reader");
  // agree on errors (global edge index of the first bad edge)
  const int64_t code = bad_edge >= 0 ? s.first_edge + bad_edge + 1 : 0;
  const auto bad = allgather(code);
  for (int64_t c : bad)
    if (c) {
      throw Error(std::string(h.mtx ? "MatrixMarket entry " : "edge ") + std::to_string(c - 1) +
                  " out of range [0, " + std::to_string(h.n) + ") or malformed in " + path);
    }
  return s;
}

}  // namespace dbfs
