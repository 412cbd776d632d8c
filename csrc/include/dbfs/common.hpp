// Common types, limits and error handling for the MI355X distributed BFS core.
//
// Index widths (replaces the all-`int` layout of the reference, bfs.cu:22-26,
// which overflows at E >= 2^31 -- SURVEY Appendix B D6):
//   vid_t  = uint32  global vertex id        (N < 2^32: RMAT-31 / Friendster fit)
//   eid_t  = int64   CSR row offsets         (E_local may exceed 2^31)
//   lvl_t  = int32   BFS level; kUnreached = INT32_MAX, the reference sentinel
//                    (bfs.cu:404,793)
//   word_t = uint64  bitmap word (64 vertices = one wave64 ballot)
#pragma once

#include <cstddef>
#include <cstdint>
#include <climits>
#include <stdexcept>
#include <string>

namespace dbfs {

using vid_t = uint32_t;
using eid_t = int64_t;
using lvl_t = int32_t;
using word_t = unsigned long long;

constexpr lvl_t kUnreached = INT32_MAX;
constexpr int kWordBits = 64;

inline int64_t div_up(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t round_up(int64_t a, int64_t b) { return div_up(a, b) * b; }

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

[[noreturn]] void raise_error(const char* file, int line, const std::string& msg);

}  // namespace dbfs

#define DBFS_CHECK(cond, msg)                                              \
  do {                                                                     \
    if (!(cond)) ::dbfs::raise_error(__FILE__, __LINE__, std::string(msg)); \
  } while (0)
