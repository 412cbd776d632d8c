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

#include <algorithm>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <thread>
#include <sstream>

#include "dbfs/graph.hpp"
#include "dbfs/rmat.hpp"

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
// Version 1 (round 1): header + row_off + col, one checksum over row_off.
struct BinHeaderV1 {
  char magic[8];
  uint32_t version;
  uint32_t reserved;
  int64_t n, row_lo, rows, nnz, input_edges;
  uint64_t checksum;  // FNV-1a over row_off
};
// Version 2: header (with its own checksum) + row_off + col + per-block
// checksums of row_off (kRowBlock entries each) and col (kColBlock entries
// each), so a rank can map and verify only the rows it owns
// (read_binary_csr_rows) instead of reading and hashing the whole file.
struct BinHeaderV2 {
  char magic[8];
  uint32_t version;
  uint32_t reserved;
  int64_t n, row_lo, rows, nnz, input_edges;
  int64_t row_block, col_block;
  uint64_t header_sum;  // FNV-1a over the bytes before it
};
constexpr int64_t kRowBlock = int64_t(1) << 16;
constexpr int64_t kColBlock = int64_t(1) << 20;

// a + b * c in size_t, or an Error on overflow / negative inputs.
size_t checked_span(size_t a, int64_t b, size_t c, const std::string& path) {
  size_t bc = 0, out = 0;
  if (b < 0 || __builtin_mul_overflow(static_cast<size_t>(b), c, &bc) || __builtin_add_overflow(a, bc, &out))
    throw Error("corrupt binary CSR header (size overflow) " + path);
  return out;
}

// Structural checks of a row range [r0, r1) of a CSR whose offsets are `ro`
// (ro[r0 .. r1] readable) and columns `col` (global offsets): monotone offsets
// inside [0, nnz], column ids < n.
void check_rows(const eid_t* ro, int64_t r0, int64_t r1, const vid_t* col, int64_t nnz, int64_t n,
                const std::string& path) {
  for (int64_t r = r0; r < r1; ++r)
    if (ro[r] < 0 || ro[r] > ro[r + 1] || ro[r + 1] > nnz)
      throw Error("corrupt binary CSR: row offsets not monotone at row " + std::to_string(r) + " in " + path);
  for (eid_t e = ro[r0]; e < ro[r1]; ++e)
    if (static_cast<int64_t>(col[e]) >= n)
      throw Error("corrupt binary CSR: column id " + std::to_string(col[e]) + " >= n at entry " +
                  std::to_string(e) + " in " + path);
}
}  // namespace

void write_binary_csr(const std::string& path, const HostCSR& g) {
  BinHeaderV2 h{};
  std::memcpy(h.magic, kBinaryMagic, 8);
  h.version = 2;
  h.n = g.n;
  h.row_lo = g.row_lo;
  h.rows = g.rows;
  h.nnz = g.directed_edges();
  h.input_edges = g.input_edges;
  h.row_block = kRowBlock;
  h.col_block = kColBlock;
  h.header_sum = fnv1a(&h, offsetof(BinHeaderV2, header_sum));
  std::vector<uint64_t> sums;
  for (size_t i = 0; i < g.row_off.size(); i += kRowBlock)
    sums.push_back(fnv1a(g.row_off.data() + i, std::min<size_t>(kRowBlock, g.row_off.size() - i) * sizeof(eid_t)));
  for (size_t i = 0; i < g.col.size(); i += kColBlock)
    sums.push_back(fnv1a(g.col.data() + i, std::min<size_t>(kColBlock, g.col.size() - i) * sizeof(vid_t)));
  std::string tmp = path + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) throw Error("cannot write " + tmp);
  bool ok = std::fwrite(&h, sizeof(h), 1, f) == 1;
  ok = ok && std::fwrite(g.row_off.data(), sizeof(eid_t), g.row_off.size(), f) == g.row_off.size();
  if (!g.col.empty()) ok = ok && std::fwrite(g.col.data(), sizeof(vid_t), g.col.size(), f) == g.col.size();
  if (!sums.empty()) ok = ok && std::fwrite(sums.data(), sizeof(uint64_t), sums.size(), f) == sums.size();
  ok = (std::fclose(f) == 0) && ok;
  if (!ok) throw Error("short write to " + tmp);
  if (std::rename(tmp.c_str(), path.c_str()) != 0) throw Error("cannot rename " + tmp + " -> " + path);
}

BinaryCsrInfo binary_csr_info(const std::string& path) {
  MappedFile mf(path);
  if (mf.size < sizeof(BinHeaderV1)) throw Error("truncated binary CSR " + path);
  BinHeaderV1 h1;
  std::memcpy(&h1, mf.data, sizeof(h1));
  if (std::memcmp(h1.magic, kBinaryMagic, 8) != 0 || (h1.version != 1 && h1.version != 2))
    throw Error("bad binary CSR header " + path);
  BinaryCsrInfo info;
  info.version = static_cast<int>(h1.version);
  info.n = h1.n;
  info.row_lo = h1.row_lo;
  info.rows = h1.rows;
  info.nnz = h1.nnz;
  info.input_edges = h1.input_edges;
  if (info.n < 0 || info.n > int64_t(UINT32_MAX) || info.rows < 0 || info.nnz < 0 || info.row_lo < 0 ||
      info.row_lo > info.n - info.rows || info.input_edges < 0)
    throw Error("corrupt binary CSR header (n / rows / nnz out of range) " + path);
  return info;
}

HostCSR read_binary_csr_rows(const std::string& path, int64_t lo, int64_t hi) {
  const BinaryCsrInfo info = binary_csr_info(path);
  if (lo < info.row_lo || hi < lo || hi > info.row_lo + info.rows)
    throw Error("row range [" + std::to_string(lo) + ", " + std::to_string(hi) + ") outside the rows of " + path);
  MappedFile mf(path);
  const int64_t r0 = lo - info.row_lo, r1 = hi - info.row_lo;  // file-local rows
  size_t hdr = sizeof(BinHeaderV1);
  int64_t row_block = 0, col_block = 0;
  if (info.version == 2) {
    if (mf.size < sizeof(BinHeaderV2)) throw Error("truncated binary CSR " + path);
    BinHeaderV2 h;
    std::memcpy(&h, mf.data, sizeof(h));
    if (fnv1a(&h, offsetof(BinHeaderV2, header_sum)) != h.header_sum)
      throw Error("binary CSR header checksum mismatch " + path);
    if (h.row_block <= 0 || h.col_block <= 0) throw Error("corrupt binary CSR header (block sizes) " + path);
    hdr = sizeof(BinHeaderV2);
    row_block = h.row_block;
    col_block = h.col_block;
  }
  const size_t off_row = hdr;
  const size_t off_col = checked_span(off_row, info.rows + 1, sizeof(eid_t), path);
  const size_t off_sum = checked_span(off_col, info.nnz, sizeof(vid_t), path);
  const int64_t nrow_blocks = row_block ? (info.rows + 1 + row_block - 1) / row_block : 0;
  const int64_t ncol_blocks = col_block ? (info.nnz + col_block - 1) / col_block : 0;
  const size_t need = checked_span(off_sum, nrow_blocks + ncol_blocks, sizeof(uint64_t), path);
  if (mf.size < need) throw Error("truncated binary CSR " + path);
  const eid_t* ro = reinterpret_cast<const eid_t*>(mf.data + off_row);
  const vid_t* col = reinterpret_cast<const vid_t*>(mf.data + off_col);
  const uint64_t* sums = reinterpret_cast<const uint64_t*>(mf.data + off_sum);
  if (info.version == 1) {
    // one checksum over all offsets: verify them all (a full read in practice)
    BinHeaderV1 h1;
    std::memcpy(&h1, mf.data, sizeof(h1));
    if (fnv1a(ro, static_cast<size_t>(info.rows + 1) * sizeof(eid_t)) != h1.checksum)
      throw Error("binary CSR checksum mismatch " + path);
  } else {
    // the blocks of row_off[r0 .. r1] (and, after the offset checks, of the
    // column range they name)
    for (int64_t b = r0 / row_block; b <= r1 / row_block && b < nrow_blocks; ++b) {
      const int64_t a = b * row_block, e = std::min(info.rows + 1, a + row_block);
      if (fnv1a(ro + a, static_cast<size_t>(e - a) * sizeof(eid_t)) != sums[b])
        throw Error("binary CSR checksum mismatch (row offsets block " + std::to_string(b) + ") " + path);
    }
  }
  if (ro[0] != 0 || ro[info.rows] != info.nnz)
    throw Error("corrupt binary CSR: row offsets do not span [0, nnz] in " + path);
  for (int64_t r = r0; r < r1; ++r)
    if (ro[r] < 0 || ro[r] > ro[r + 1] || ro[r + 1] > info.nnz)
      throw Error("corrupt binary CSR: row offsets not monotone at row " + std::to_string(r) + " in " + path);
  const eid_t c0 = ro[r0], c1 = ro[r1];
  if (info.version == 2 && c1 > c0) {
    for (int64_t b = c0 / col_block; b <= (c1 - 1) / col_block; ++b) {
      const int64_t a = b * col_block, e = std::min(info.nnz, a + col_block);
      if (fnv1a(col + a, static_cast<size_t>(e - a) * sizeof(vid_t)) != sums[nrow_blocks + b])
        throw Error("binary CSR checksum mismatch (columns block " + std::to_string(b) + ") " + path);
    }
  }
  check_rows(ro, r0, r1, col, info.nnz, info.n, path);
  HostCSR g;
  g.n = info.n;
  g.row_lo = lo;
  g.rows = hi - lo;
  g.input_edges = info.input_edges;
  g.row_off.resize(static_cast<size_t>(g.rows + 1));
  for (int64_t r = 0; r <= g.rows; ++r) g.row_off[r] = ro[r0 + r] - c0;
  g.col.assign(col + c0, col + c1);
  return g;
}

HostCSR read_binary_csr(const std::string& path) {
  const BinaryCsrInfo info = binary_csr_info(path);
  return read_binary_csr_rows(path, info.row_lo, info.row_lo + info.rows);
}

void write_generated_edge_list(const std::string& path, const GenParams& p, int threads) {
  // `n m` then the generator's edges (edge i is a pure function of (seed, i)),
  // formatted by `threads` threads in chunks written in edge order.
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw Error("cannot write " + path);
  std::fprintf(f, "%lld %lld\n", static_cast<long long>(p.n), static_cast<long long>(p.m));
  const int T = threads > 0 ? threads : static_cast<int>(std::max(1u, std::thread::hardware_concurrency()));
  constexpr int64_t kChunk = int64_t(1) << 22;  // edges per thread per round
  std::vector<std::string> buf(static_cast<size_t>(T));
  bool ok = true;
  for (int64_t base = 0; base < p.m && ok; base += kChunk * T) {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        const int64_t b = base + kChunk * t, e = std::min(p.m, b + kChunk);
        std::string& out = buf[t];
        out.clear();
        if (b >= e) return;
        out.resize(static_cast<size_t>(e - b) * 22);
        char* w = &out[0];
        auto put = [&w](uint64_t x, char end) {
          char d[20];
          int k = 0;
          do {
            d[k++] = static_cast<char>('0' + x % 10);
            x /= 10;
          } while (x);
          while (k) *w++ = d[--k];
          *w++ = end;
        };
        for (int64_t i = b; i < e; ++i) {
          uint64_t u, v;
          gen_edge(p, static_cast<uint64_t>(i), u, v);
          put(u, ' ');
          put(v, '\n');
        }
        out.resize(static_cast<size_t>(w - out.data()));
      });
    for (auto& x : th) x.join();
    for (int t = 0; t < T && ok; ++t)
      ok = buf[t].empty() || std::fwrite(buf[t].data(), 1, buf[t].size(), f) == buf[t].size();
  }
  if (std::fclose(f) != 0 || !ok) throw Error("short write to " + path);
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
