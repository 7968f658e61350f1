// jit.cpp — the scene-specialised trace kernel: trace_kernel.h compiled at run time by
// hiprtc with the scene's primitive records as compile-time constants (FR_JIT_N,
// FR_JIT_REC), for list-loop scenes of at most kJitMaxPrims primitives.
//
// Why: a box test costs 26 VALU per segment, 18 of them the six slab distances and their
// min/max. Boxes that share a coordinate plane (the walls of scene_08 share x = 0, y = +-30,
// z = +-35, ...) compute the same slab distance from the same inputs; with the records as
// literals the compiler sees that and computes each distinct (coordinate - o) * inv once
// per segment. The tests, their order and their arithmetic are the list loop's, so the
// image is the same bits (tests/test_gpu_parity.py::test_scene_jit_*). DESIGN.md §4.11.
//
// Modules are cached per process (device, key) and code objects on disk
// (FR_JIT_CACHE, default $XDG_CACHE_HOME/forma_rt or ~/.cache/forma_rt; "0" disables),
// keyed by a hash of the embedded sources, defines, kernel name, records and target.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "internal.h"
#include "jit.h"
#include "../build/jit_sources.inc"

namespace fr {
namespace {

struct Module {
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
};

std::mutex g_mu;
std::map<std::string, Module> g_modules;  // (device, key) -> loaded module

uint64_t fnv1a(const void* p, size_t n, uint64_t h) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) {
    h ^= b[i];
    h *= 0x100000001b3ull;
  }
  return h;
}

std::string hex_key(const std::string& text) {
  // two independent 64-bit FNV-1a lanes: a 128-bit key
  const uint64_t a = fnv1a(text.data(), text.size(), 0xcbf29ce484222325ull);
  const uint64_t b = fnv1a(text.data(), text.size(), 0x84222325cbf29ce4ull ^ text.size());
  char buf[40];
  snprintf(buf, sizeof buf, "%016llx%016llx", static_cast<unsigned long long>(a), static_cast<unsigned long long>(b));
  return buf;
}

std::string cache_dir() {
  const char* e = getenv("FR_JIT_CACHE");
  if (e && strcmp(e, "0") == 0) return "";
  std::string d;
  if (e && *e) {
    d = e;
  } else if (const char* x = getenv("XDG_CACHE_HOME"); x && *x) {
    d = std::string(x) + "/forma_rt";
  } else if (const char* h = getenv("HOME"); h && *h) {
    d = std::string(h) + "/.cache/forma_rt";
  } else {
    return "";
  }
  // mkdir -p of the last two levels is enough for the defaults
  const size_t slash = d.find_last_of('/');
  if (slash != std::string::npos && slash > 0) mkdir(d.substr(0, slash).c_str(), 0755);
  mkdir(d.c_str(), 0755);
  return d;
}

bool read_file(const std::string& path, std::vector<char>& out) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  fseek(f, 0, SEEK_END);
  const long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  out.resize(n > 0 ? static_cast<size_t>(n) : 0u);
  const bool ok = n > 0 && fread(out.data(), 1, out.size(), f) == out.size();
  fclose(f);
  return ok;
}

void write_file_atomic(const std::string& path, const std::vector<char>& data) {
  const std::string tmp = path + ".tmp." + std::to_string(getpid());
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) return;  // an unwritable cache only costs the next process a compile
  const bool ok = fwrite(data.data(), 1, data.size(), f) == data.size();
  fclose(f);
  if (!ok || rename(tmp.c_str(), path.c_str()) != 0) unlink(tmp.c_str());
}

// hiprtc: the embedded trace_kernel.h with the prelude's defines and records
int compile(const std::string& arch, const std::string& prelude, const char* name_expr, std::vector<char>& code,
            std::string* lowered = nullptr) {
  const std::string src = prelude + "#include \"trace_kernel.h\"\n";
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "fr_scene_kernel.hip", jit_src::kCount, jit_src::kBodies,
                          jit_src::kNames) != HIPRTC_SUCCESS)
    return set_error(FR_EHIP, "hiprtcCreateProgram failed");
  hiprtcAddNameExpression(prog, name_expr);
  // the Makefile's device numerics flags: part of the parity contract
  const std::string arch_opt = "--offload-arch=" + arch;
  const char* opts[] = {arch_opt.c_str(),
                        "-O3",
                        "-std=c++17",
                        "-ffp-contract=off",
                        "-fno-fast-math",
                        "-fhip-fp32-correctly-rounded-divide-sqrt",
                        "-fno-gpu-flush-denormals-to-zero",
                        "-fno-slp-vectorize"};
  std::vector<const char*> all(opts, opts + sizeof(opts) / sizeof(opts[0]));
  // FR_JIT_OPTS: extra compiler options, space-separated (A/B experiments only)
  std::vector<std::string> extra;
  if (const char* e = getenv("FR_JIT_OPTS")) {
    std::string cur;
    for (const char* c = e;; ++c) {
      if (*c == ' ' || *c == '\0') {
        if (!cur.empty()) extra.push_back(cur);
        cur.clear();
        if (!*c) break;
      } else {
        cur += *c;
      }
    }
  }
  for (const std::string& x : extra) all.push_back(x.c_str());
  const hiprtcResult r = hiprtcCompileProgram(prog, static_cast<int>(all.size()), all.data());
  if (r != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n + 1, '\0');
    if (n) hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    return set_error(FR_EHIP, "hiprtc: scene kernel did not compile (%s): %.1500s", hiprtcGetErrorString(r),
                     log.c_str());
  }
  if (lowered) {
    const char* ln = nullptr;
    *lowered = hiprtcGetLoweredName(prog, name_expr, &ln) == HIPRTC_SUCCESS && ln ? ln : "";
  }
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  code.resize(n);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  // FR_JIT_DUMP=path keeps the code object (llvm-objdump / resource inspection)
  if (const char* dump = getenv("FR_JIT_DUMP"); dump && *dump && n) write_file_atomic(dump, code);
  return n ? FR_OK : set_error(FR_EHIP, "hiprtc: empty code object");
}

// hiprtc's lowered name of `name_expr` needs the program; the kernel's mangled name is
// fixed by its template arguments, so it is recomputed here for cache hits as well:
// every template argument of trace_kernel is an int or a bool.
std::string mangled(const int* targs, const bool* is_bool, int n) {
  std::string m = "_ZN2fr12trace_kernelI";
  for (int i = 0; i < n; ++i) {
    if (is_bool[i])
      m += std::string("Lb") + (targs[i] ? "1" : "0") + "E";
    else
      m += "Li" + std::to_string(targs[i]) + "E";
  }
  return m + "EEvNS_5KArgsE";
}

// the host build's tuning/contract macros, then the scene's records
std::string make_prelude(const JitSpec& spec) {
  std::string prelude = spec.defines;
  prelude += "#define FR_JIT_N " + std::to_string(spec.n) + "u\n#define FR_JIT_REC ";
  char w[16];
  for (uint32_t i = 0; i < spec.n; ++i) {
    prelude += i ? ",{" : "{";
    for (int k = 0; k < 16; ++k) {
      snprintf(w, sizeof w, k ? ",0x%08xu" : "0x%08xu", spec.rec[16u * i + k]);
      prelude += w;
    }
    prelude += "}";
  }
  return prelude + "\n";
}

}  // namespace

int jit_compile_probe(const char* arch, const JitSpec& spec, size_t* code_bytes, double* ms) {
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<char> code;
  std::string lowered;
  const int rc = compile(arch, make_prelude(spec), spec.name_expr, code, &lowered);
  if (rc) return rc;
  const std::string mname = mangled(spec.targs, spec.targ_bool, spec.n_targs);
  if (lowered != mname)
    return set_error(FR_EHIP, "scene kernel name %s, expected %s", lowered.c_str(), mname.c_str());
  if (code_bytes) *code_bytes = code.size();
  if (ms) *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return FR_OK;
}

// The device's target name (gcnArchName), queried once per device: every render of a
// scene-specialised frame looks its kernel up, and the property query is not free.
static std::string device_arch(int device) {
  static std::mutex mu;
  static std::map<int, std::string> arch;
  std::lock_guard<std::mutex> g(mu);
  auto it = arch.find(device);
  if (it != arch.end()) return it->second;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return "";
  return arch[device] = prop.gcnArchName;
}

int jit_trace_kernel(int device, const JitSpec& spec, hipFunction_t* out, JitStats* stats) {
  const auto t0 = std::chrono::steady_clock::now();
  const std::string arch = device_arch(device);
  if (arch.empty()) return set_error(FR_EHIP, "hipGetDeviceProperties failed");
  const std::string prelude = make_prelude(spec);
  const char* xo = getenv("FR_JIT_OPTS");
  const std::string key = hex_key(std::string(jit_src::kHash) + "\n" + arch + "\n" + spec.name_expr + "\n" + prelude +
                                  (xo ? xo : ""));
  const std::string mkey = std::to_string(device) + ":" + key;
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_modules.find(mkey);
  if (it != g_modules.end()) {
    *out = it->second.fn;
    if (stats) *stats = JitStats{0.0, 0, 1};
    return FR_OK;
  }
  std::vector<char> code;
  int cached = 0;
  const std::string dir = cache_dir();
  const std::string path = dir.empty() ? "" : dir + "/" + key + ".hsaco";
  if (!path.empty() && read_file(path, code)) cached = 1;
  if (!cached) {
    const int rc = compile(arch, prelude, spec.name_expr, code);
    if (rc) return rc;
    if (!path.empty()) write_file_atomic(path, code);
  }
  Module m;
  hipError_t e = hipModuleLoadData(&m.mod, code.data());
  if (e != hipSuccess) return set_error(FR_EHIP, "hipModuleLoadData (scene kernel): %s", hipGetErrorString(e));
  const std::string mname = mangled(spec.targs, spec.targ_bool, spec.n_targs);
  e = hipModuleGetFunction(&m.fn, m.mod, mname.c_str());
  if (e != hipSuccess) {
    (void)hipModuleUnload(m.mod);
    return set_error(FR_EHIP, "hipModuleGetFunction(%s): %s", mname.c_str(), hipGetErrorString(e));
  }
  g_modules[mkey] = m;  // kept for the process's lifetime (a few hundred KB per scene)
  *out = m.fn;
  if (stats)
    *stats = JitStats{std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(),
                      cached ? 0 : 1, 0};
  return FR_OK;
}

}  // namespace fr
