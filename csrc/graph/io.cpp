// Graph file input/output.
//
// Reference reader: readGraphFromFile (bfs.cu:829-880) -- ifstream `>>` of
// `n m` then m pairs, no header/comment handling, no bounds checks, and an
// unopenable file silently yields an empty graph.
// This reader memory-maps the file and parses integers by hand (the text parse
// dominates end-to-end time for large inputs), auto-detects MatrixMarket
// (`%%MatrixMarket` banner, `%` comments, 1-based ids, optional value column),
// validates every id, and throws on any error.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>

#include "dbfs/graph.hpp"

namespace dbfs {

void raise_error(const char* file, int line, const std::string& msg) {
  std::ostringstream os;
  os << msg << " [" << file << ":" << line << "]";
  throw Error(os.str());
}

namespace {

constexpr char kBinaryMagic[8] = {'D', 'B', 'F', 'S', 'C', 'S', 'R', '1'};

struct MappedFile {
  const char* data = nullptr;
  size_t size = 0;
  int fd = -1;
  explicit MappedFile(const std::string& path) {
    fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw Error("not open " + path);
    struct stat st {};
    if (::fstat(fd, &st) != 0) { ::close(fd); throw Error("cannot stat " + path); }
    size = static_cast<size_t>(st.st_size);
    if (size > 0) {
      void* p = ::mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
      if (p == MAP_FAILED) { ::close(fd); throw Error("cannot mmap " + path); }
      ::madvise(p, size, MADV_SEQUENTIAL);
      data = static_cast<const char*>(p);
    }
  }
  ~MappedFile() {
    if (data) ::munmap(const_cast<char*>(data), size);
    if (fd >= 0) ::close(fd);
  }
};

struct Cursor {
  const char* p;
  const char* end;
  int64_t line = 1;
  bool at_end() const { return p >= end; }
  void skip_ws() {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n')) {
      if (*p == '\n') ++line;
      ++p;
    }
  }
  void skip_line() {
    while (p < end && *p != '\n') ++p;
    if (p < end) { ++p; ++line; }
  }
  // Skip blanks and '%' comment lines (MatrixMarket).
  void skip_ws_and_comments() {
    for (;;) {
      skip_ws();
      if (p < end && *p == '%') { skip_line(); continue; }
      return;
    }
  }
  bool read_int(int64_t& out) {
    skip_ws();
    if (p >= end) return false;
    bool neg = false;
    if (*p == '-' || *p == '+') { neg = (*p == '-'); ++p; }
    if (p >= end || *p < '0' || *p > '9') return false;
    int64_t v = 0;
    while (p < end && *p >= '0' && *p <= '9') { v = v * 10 + (*p - '0'); ++p; }
    out = neg ? -v : v;
    return true;
  }
  // Rest of the current line (MatrixMarket value columns) is ignored.
  void finish_line() {
    while (p < end && *p != '\n') ++p;
  }
};

bool starts_with(const char* p, size_t n, const char* s) {
  size_t k = std::strlen(s);
  return n >= k && std::memcmp(p, s, k) == 0;
}

EdgeList parse_reference(Cursor& c, const std::string& path, bool verbose) {
  int64_t n = 0, m = 0;
  if (!c.read_int(n) || !c.read_int(m)) throw Error("bad header (expected `n m`) in " + path);
  if (verbose) {
    std::printf("nodes num: %lld\n", static_cast<long long>(n));
    std::printf("edge num: %lld\n", static_cast<long long>(m));
  }
  if (n < 0 || m < 0) throw Error("negative n or m in " + path);
  if (n > int64_t(UINT32_MAX)) throw Error("vertex count exceeds 2^32 in " + path);
  EdgeList el;
  el.n = n;
  el.u.resize(static_cast<size_t>(m));
  el.v.resize(static_cast<size_t>(m));
  for (int64_t i = 0; i < m; ++i) {
    int64_t a, b;
    if (!c.read_int(a) || !c.read_int(b)) {
      throw Error("truncated edge list in " + path + ": expected " + std::to_string(m) +
                  " edges, got " + std::to_string(i));
    }
    if (a < 0 || a >= n || b < 0 || b >= n) {
      throw Error("edge " + std::to_string(i) + " (" + std::to_string(a) + ", " + std::to_string(b) +
                  ") out of range [0, " + std::to_string(n) + ") in " + path);
    }
    el.u[i] = static_cast<vid_t>(a);
    el.v[i] = static_cast<vid_t>(b);
  }
  return el;
}

EdgeList parse_matrix_market(Cursor& c, const std::string& path, bool verbose) {
  // Banner line: %%MatrixMarket matrix coordinate <field> <symmetry>
  c.skip_line();
  c.skip_ws_and_comments();
  int64_t rows = 0, cols = 0, nnz = 0;
  if (!c.read_int(rows) || !c.read_int(cols) || !c.read_int(nnz))
    throw Error("bad MatrixMarket size line in " + path);
  c.finish_line();
  const int64_t n = std::max(rows, cols);
  if (verbose) {
    std::printf("nodes num: %lld\n", static_cast<long long>(n));
    std::printf("edge num: %lld\n", static_cast<long long>(nnz));
  }
  if (n > int64_t(UINT32_MAX)) throw Error("vertex count exceeds 2^32 in " + path);
  EdgeList el;
  el.n = n;
  el.u.resize(static_cast<size_t>(nnz));
  el.v.resize(static_cast<size_t>(nnz));
  for (int64_t i = 0; i < nnz; ++i) {
    c.skip_ws_and_comments();
    int64_t a, b;
    if (!c.read_int(a) || !c.read_int(b))
      throw Error("truncated MatrixMarket entries in " + path + " at entry " + std::to_string(i));
    c.finish_line();
    if (a < 1 || a > n || b < 1 || b > n)
      throw Error("MatrixMarket entry " + std::to_string(i) + " out of range in " + path);
    el.u[i] = static_cast<vid_t>(a - 1);
    el.v[i] = static_cast<vid_t>(b - 1);
  }
  return el;
}

}  // namespace

FileFormat detect_format(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw Error("not open " + path);
  char buf[16] = {0};
  f.read(buf, sizeof(buf));
  size_t got = static_cast<size_t>(f.gcount());
  if (got >= 8 && std::memcmp(buf, kBinaryMagic, 8) == 0) return FileFormat::Binary;
  if (starts_with(buf, got, "%%MatrixMarket") || starts_with(buf, got, "%%matrixmarket"))
    return FileFormat::MatrixMarket;
  return FileFormat::EdgeList;
}

bool is_binary_csr(const std::string& path) {
  try {
    return detect_format(path) == FileFormat::Binary;
  } catch (const Error&) {
    return false;
  }
}

EdgeList read_edge_list(const std::string& path, const ReadOptions& opt) {
  if (path == "-") {
    // standard input (the reference's readGraph, bfs.cu:882-920): slurp, then parse
    std::string buf;
    char tmp[1 << 16];
    size_t k;
    while ((k = std::fread(tmp, 1, sizeof(tmp), stdin)) > 0) buf.append(tmp, k);
    Cursor c{buf.data(), buf.data() + buf.size()};
    const bool mm = opt.format == FileFormat::MatrixMarket ||
                    (opt.format == FileFormat::Auto && starts_with(buf.data(), buf.size(), "%%MatrixMarket"));
    if (mm) return parse_matrix_market(c, "<stdin>", opt.verbose_reference_lines);
    return parse_reference(c, "<stdin>", opt.verbose_reference_lines);
  }
  FileFormat fmt = opt.format == FileFormat::Auto ? detect_format(path) : opt.format;
  if (fmt == FileFormat::Binary) throw Error("binary CSR cache is not an edge list: " + path);
  MappedFile mf(path);
  Cursor c{mf.data, mf.data + mf.size};
  if (fmt == FileFormat::MatrixMarket) return parse_matrix_market(c, path, opt.verbose_reference_lines);
  return parse_reference(c, path, opt.verbose_reference_lines);
}

namespace {
uint64_t fnv1a(const void* data, size_t bytes, uint64_t h = 1469598103934665603ull) {
  const unsigned char* p = static_cast<const unsigned char*>(data);
  for (size_t i = 0; i < bytes; ++i) { h ^= p[i]; h *= 1099511628211ull; }
  return h;
}
struct BinHeader {
  char magic[8];
  uint32_t version;
  uint32_t reserved;
  int64_t n, row_lo, rows, nnz, input_edges;
  uint64_t checksum;  // FNV-1a over row_off
};
}  // namespace

void write_binary_csr(const std::string& path, const HostCSR& g) {
  BinHeader h{};
  std::memcpy(h.magic, kBinaryMagic, 8);
  h.version = 1;
  h.n = g.n;
  h.row_lo = g.row_lo;
  h.rows = g.rows;
  h.nnz = g.directed_edges();
  h.input_edges = g.input_edges;
  h.checksum = fnv1a(g.row_off.data(), g.row_off.size() * sizeof(eid_t));
  std::string tmp = path + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) throw Error("cannot write " + tmp);
  bool ok = std::fwrite(&h, sizeof(h), 1, f) == 1;
  ok = ok && std::fwrite(g.row_off.data(), sizeof(eid_t), g.row_off.size(), f) == g.row_off.size();
  if (!g.col.empty()) ok = ok && std::fwrite(g.col.data(), sizeof(vid_t), g.col.size(), f) == g.col.size();
  ok = (std::fclose(f) == 0) && ok;
  if (!ok) throw Error("short write to " + tmp);
  if (std::rename(tmp.c_str(), path.c_str()) != 0) throw Error("cannot rename " + tmp + " -> " + path);
}

HostCSR read_binary_csr(const std::string& path) {
  MappedFile mf(path);
  if (mf.size < sizeof(BinHeader)) throw Error("truncated binary CSR " + path);
  BinHeader h;
  std::memcpy(&h, mf.data, sizeof(h));
  if (std::memcmp(h.magic, kBinaryMagic, 8) != 0 || h.version != 1) throw Error("bad binary CSR header " + path);
  const size_t need = sizeof(BinHeader) + static_cast<size_t>(h.rows + 1) * sizeof(eid_t) +
                      static_cast<size_t>(h.nnz) * sizeof(vid_t);
  if (mf.size < need) throw Error("truncated binary CSR " + path);
  HostCSR g;
  g.n = h.n;
  g.row_lo = h.row_lo;
  g.rows = h.rows;
  g.input_edges = h.input_edges;
  g.row_off.resize(static_cast<size_t>(h.rows + 1));
  std::memcpy(g.row_off.data(), mf.data + sizeof(BinHeader), g.row_off.size() * sizeof(eid_t));
  if (fnv1a(g.row_off.data(), g.row_off.size() * sizeof(eid_t)) != h.checksum)
    throw Error("binary CSR checksum mismatch " + path);
  g.col.resize(static_cast<size_t>(h.nnz));
  if (h.nnz)
    std::memcpy(g.col.data(), mf.data + sizeof(BinHeader) + g.row_off.size() * sizeof(eid_t),
                g.col.size() * sizeof(vid_t));
  return g;
}

void write_levels(const std::string& path, const std::vector<lvl_t>& levels) {
  FILE* f = std::fopen(path.c_str(), "w");
  if (!f) throw Error("cannot write " + path);
  std::vector<char> buf;
  buf.reserve(1 << 20);
  char tmp[16];
  for (lvl_t l : levels) {
    int k = std::snprintf(tmp, sizeof(tmp), "%d\n", l);
    buf.insert(buf.end(), tmp, tmp + k);
    if (buf.size() > (1 << 20) - 32) {
      std::fwrite(buf.data(), 1, buf.size(), f);
      buf.clear();
    }
  }
  if (!buf.empty()) std::fwrite(buf.data(), 1, buf.size(), f);
  if (std::fclose(f) != 0) throw Error("short write to " + path);
}

}  // namespace dbfs
