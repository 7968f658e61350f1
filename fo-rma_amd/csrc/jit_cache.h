// jit_cache.h — the scene-specialised kernel's disk-cache files (jit.cpp): no HIP here, so
// the host sanitizer program (tests/c/host_sanitize.cpp) builds and fuzzes the parser that
// guards the HIP loader.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace fr {

uint64_t fnv1a(const void* p, size_t n, uint64_t h);

// Files larger than this are not cache files (a code object of the list kernel is ~100 KB).
constexpr size_t kCacheMaxBytes = size_t(64) << 20;

// The whole of a regular file of 1 .. kCacheMaxBytes bytes, or false (missing, unreadable,
// a directory or other non-regular file, empty, or too large).
bool read_file(const std::string& path, std::vector<char>& out);

// A cache file: a 32-B header (magic, format version, code size, a 128-bit hash of the
// code), then the code object.
std::vector<char> wrap_code(const std::vector<char>& code);

// The code object of a cache file, or false: a damaged or foreign regular file (empty or
// oversized, wrong magic or format, a size that is not the file's, a hash mismatch) is
// removed; a missing path or a non-regular file (a directory) is left alone.
bool read_cached_code(const std::string& path, std::vector<char>& code);

// Write through a temporary file and rename: the file appears under `path` only when every
// byte reached the disk.
bool write_file_atomic(const std::string& path, const std::vector<char>& data);

}  // namespace fr
