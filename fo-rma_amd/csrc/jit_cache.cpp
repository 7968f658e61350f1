// jit_cache.cpp — see jit_cache.h. DESIGN.md §4.8 (disk cache).
#include "jit_cache.h"

#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

namespace fr {

uint64_t fnv1a(const void* p, size_t n, uint64_t h) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) {
    h ^= b[i];
    h *= 0x100000001b3ull;
  }
  return h;
}

bool read_file(const std::string& path, std::vector<char>& out) {
  out.clear();
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  // the size from the open file itself: fopen succeeds on a directory, whose ftell is
  // not a byte count
  struct stat st;
  if (fstat(fileno(f), &st) != 0 || !S_ISREG(st.st_mode) || st.st_size <= 0 ||
      static_cast<unsigned long long>(st.st_size) > kCacheMaxBytes) {
    fclose(f);
    return false;
  }
  out.resize(static_cast<size_t>(st.st_size));
  const bool ok = fread(out.data(), 1, out.size(), f) == out.size();
  fclose(f);
  if (!ok) out.clear();
  return ok;
}

// A disk-cache file is a 32-B header — magic, format version, code size, a 128-bit hash of
// the code — then the code object. The HIP loader does not reject a damaged code object: it
// aborts the process (a truncated file did, on the GPU box). So nothing read from disk
// reaches hipModuleLoadData unless its size and hash check out.
static constexpr char kCacheMagic[4] = {'F', 'R', 'J', 'C'};
static constexpr uint32_t kCacheFormat = 1;
static constexpr size_t kCacheHeader = 32;

static void code_hash(const char* p, size_t n, uint64_t h[2]) {
  h[0] = fnv1a(p, n, 0xcbf29ce484222325ull);
  h[1] = fnv1a(p, n, 0x84222325cbf29ce4ull ^ n);
}

std::vector<char> wrap_code(const std::vector<char>& code) {
  std::vector<char> out(kCacheHeader + code.size());
  const uint64_t size = code.size();
  uint64_t h[2];
  code_hash(code.data(), code.size(), h);
  memcpy(out.data(), kCacheMagic, 4);
  memcpy(out.data() + 4, &kCacheFormat, 4);
  memcpy(out.data() + 8, &size, 8);
  memcpy(out.data() + 16, h, 16);
  if (!code.empty()) memcpy(out.data() + kCacheHeader, code.data(), code.size());
  return out;
}

bool read_cached_code(const std::string& path, std::vector<char>& code) {
  std::vector<char> raw;
  if (!read_file(path, raw)) {
    // an empty or oversized regular file is as damaged as a truncated one
    struct stat st;
    if (stat(path.c_str(), &st) == 0 && S_ISREG(st.st_mode)) unlink(path.c_str());
    return false;
  }
  uint32_t fmt = 0;
  uint64_t size = 0, h[2] = {0, 0}, want[2] = {0, 0};
  bool ok = raw.size() > kCacheHeader && memcmp(raw.data(), kCacheMagic, 4) == 0;
  if (ok) {
    memcpy(&fmt, raw.data() + 4, 4);
    memcpy(&size, raw.data() + 8, 8);
    memcpy(want, raw.data() + 16, 16);
    ok = fmt == kCacheFormat && size == raw.size() - kCacheHeader;
  }
  if (ok) {
    code_hash(raw.data() + kCacheHeader, static_cast<size_t>(size), h);
    ok = h[0] == want[0] && h[1] == want[1];
  }
  if (!ok) {
    unlink(path.c_str());
    return false;
  }
  code.assign(raw.begin() + kCacheHeader, raw.end());
  return true;
}

bool write_file_atomic(const std::string& path, const std::vector<char>& data) {
  const std::string tmp = path + ".tmp." + std::to_string(getpid());
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) return false;  // an unwritable cache only costs the next process a compile
  bool ok = fwrite(data.data(), 1, data.size(), f) == data.size();
  ok = fflush(f) == 0 && ok;
  ok = fsync(fileno(f)) == 0 && ok;
  ok = fclose(f) == 0 && ok;
  if (!ok || rename(tmp.c_str(), path.c_str()) != 0) {
    unlink(tmp.c_str());
    return false;
  }
  return true;
}

}  // namespace fr
