// jit.cpp — the scene-specialised trace kernel: trace_kernel.h compiled at run time by
// hiprtc with the scene's primitive records as compile-time constants (FR_JIT_N,
// FR_JIT_REC), for list-loop scenes of at most kJitMaxPrims primitives.
//
// Why: a box test costs 26 VALU per segment, 18 of them the six slab distances and their
// min/max. Boxes that share a coordinate plane (the walls of scene_08 share x = 0, y = +-30,
// z = +-35, ...) compute the same slab distance from the same inputs; with the records as
// literals the compiler sees that and computes each distinct (coordinate - o) * inv once
// per segment. The tests, their order and their arithmetic are the list loop's, so the
// image is the same bits (tests/test_gpu_parity.py::test_scene_jit_*). DESIGN.md §4.8.
//
// Where the code comes from (one code object per key, shared by every device of an arch):
//   1. this process's code cache (built or read earlier; a module per device on top);
//   2. the disk cache (FR_JIT_CACHE, default $XDG_CACHE_HOME/forma_rt or ~/.cache/forma_rt;
//      "0" disables), keyed by a hash of the embedded sources, the hiprtc options, the
//      hiprtc and HIP runtime versions, the defines, the kernel name, the records and the
//      target. Each file carries its code object's size and hash, checked before the bytes
//      reach the loader (which aborts on a damaged code object); a file that fails the
//      check, or fails to load, is deleted and the kernel compiled again once;
//   3. hiprtc: on the caller's thread when it waits (fr_ctx_prepare, FR_FLAG_SCENE_JIT_WAIT),
//      else on one background worker thread while renders run the compiled-in kernel.
// Bounds: at most kMaxModules loaded modules (least recently used unloaded first, after
// every stream it was launched on has passed its last launch), kMaxCode code objects in memory and kMaxDiskFiles files on disk.
#include <dirent.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "internal.h"
#include "jit.h"
#include "jit_cache.h"
#include "../build/jit_sources.inc"

namespace fr {
namespace {

constexpr size_t kMaxModules = 64;    // loaded (device, key) modules per process
constexpr size_t kMaxStreamEvents = 32;  // per module: completed entries are pruned beyond this

// FR_JIT_MAX_MODULES (tests only): a smaller module bound, so a test can force evictions
size_t max_modules() {
  static const size_t n = [] {
    const char* e = getenv("FR_JIT_MAX_MODULES");
    const long v = e && *e ? atol(e) : 0;
    return v > 0 ? static_cast<size_t>(v) : kMaxModules;
  }();
  return n;
}
constexpr size_t kMaxCode = 128;      // code objects held in memory per process
constexpr size_t kMaxDiskFiles = 256; // .hsaco files kept in the disk cache

// the Makefile's device numerics flags: part of the parity contract, and of
// the cache key
const char* const kOpts[] = {"-O3",
                             "-std=c++17",
                             "-ffp-contract=off",
                             "-fno-fast-math",
                             "-fhip-fp32-correctly-rounded-divide-sqrt",
                             "-fno-gpu-flush-denormals-to-zero",
                             "-fno-slp-vectorize"};

std::string hex_key(const std::string& text) {
  // two independent 64-bit FNV-1a lanes: a 128-bit key
  const uint64_t a = fnv1a(text.data(), text.size(), 0xcbf29ce484222325ull);
  const uint64_t b = fnv1a(text.data(), text.size(), 0x84222325cbf29ce4ull ^ text.size());
  char buf[40];
  snprintf(buf, sizeof buf, "%016llx%016llx", static_cast<unsigned long long>(a), static_cast<unsigned long long>(b));
  return buf;
}

// FR_JIT_OPTS: extra compiler options, space-separated (A/B experiments only). Read once:
// the cache key (toolchain_tag) and every compile use this one snapshot, so a process that
// changes the variable later cannot store code built with other options under the key.
std::vector<std::string> parse_extra_opts() {
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
  return extra;
}

const std::vector<std::string>& extra_opts() {
  static const std::vector<std::string> v = parse_extra_opts();
  return v;
}

// What else decides the code object besides the sources and the records: the option list,
// the compiler (hiprtc) and runtime versions
std::string toolchain_tag() {
  std::string t = "opts:";
  for (const char* o : kOpts) t += std::string(o) + " ";
  for (const std::string& o : extra_opts()) t += o + " ";
  int maj = 0, min = 0, rt = 0;
  if (hiprtcVersion(&maj, &min) == HIPRTC_SUCCESS) t += "\nhiprtc:" + std::to_string(maj) + "." + std::to_string(min);
  if (hipRuntimeGetVersion(&rt) == hipSuccess) t += "\nhip:" + std::to_string(rt);
  t += "\nhip_build:" + std::to_string(HIP_VERSION);
  return t;
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

// Keep at most kMaxDiskFiles code objects in the cache directory: the oldest go first.
void prune_disk(const std::string& dir) {
  DIR* d = opendir(dir.c_str());
  if (!d) return;
  std::vector<std::pair<time_t, std::string>> files;
  while (const dirent* e = readdir(d)) {
    const std::string name = e->d_name;
    if (name.size() < 7 || name.compare(name.size() - 6, 6, ".hsaco") != 0) continue;
    struct stat s;
    const std::string p = dir + "/" + name;
    if (stat(p.c_str(), &s) == 0) files.emplace_back(s.st_mtime, p);
  }
  closedir(d);
  if (files.size() <= kMaxDiskFiles) return;
  std::sort(files.begin(), files.end());
  for (size_t i = 0; i + kMaxDiskFiles < files.size(); ++i) unlink(files[i].second.c_str());
}

// hiprtc: the embedded trace_kernel.h with the prelude's defines and records
int compile(const std::string& arch, const std::string& prelude, const char* name_expr, std::vector<char>& code,
            std::string* lowered = nullptr) {
  const std::string src = prelude + "#include \"trace_kernel.h\"\n";
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "fr_scene_kernel.hip", jit_src::kCount, jit_src::kBodies,
                          jit_src::kNames) != HIPRTC_SUCCESS)
    return set_error(FR_EHIP, "hiprtcCreateProgram failed");
  if (hiprtcAddNameExpression(prog, name_expr) != HIPRTC_SUCCESS) {
    hiprtcDestroyProgram(&prog);
    return set_error(FR_EHIP, "hiprtcAddNameExpression(%s) failed", name_expr);
  }
  const std::string arch_opt = "--offload-arch=" + arch;
  std::vector<const char*> all{arch_opt.c_str()};
  for (const char* o : kOpts) all.push_back(o);
  for (const std::string& x : extra_opts()) all.push_back(x.c_str());
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
  if (n) hiprtcGetCode(prog, code.data());
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

// A fresh compile whose kernel name is the one the loader looks up (checked before the code
// object is cached anywhere).
int compile_checked(const std::string& arch, const std::string& prelude, const std::string& name_expr,
                    const std::string& mname, std::vector<char>& code) {
  std::string lowered;
  const int rc = compile(arch, prelude, name_expr.c_str(), code, &lowered);
  if (rc) return rc;
  if (lowered != mname)
    return set_error(FR_EHIP, "scene kernel name %s, expected %s", lowered.c_str(), mname.c_str());
  return FR_OK;
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

struct CodeEntry {
  enum State { kCompiling, kReady, kFailed } state = kCompiling;
  std::shared_ptr<const std::vector<char>> code;
  std::string error;
  bool from_disk = false;
  uint64_t used = 0;
};

// A module's launches still in flight: jit_note_launch records, per stream the module was
// launched on, an event after the launch (streams are in order, so one event per stream
// covers every earlier launch there). An evicted module is unloaded after all of them, not
// after a drain of the whole device. One context launches on two streams (multi-pass renders
// and overlapping frames alternate) and contexts on one device share a module, so a single
// "last launch" event would miss the other stream's launch. Guarded by `mu`: renders on
// several threads note launches of one module concurrently. (The events are destroyed when
// the module is unloaded, never at process exit: the runtime may be gone by then.)
struct ModuleUse {
  std::mutex mu;
  std::vector<std::pair<hipStream_t, hipEvent_t>> last;  // (stream, event after its last launch)
};

struct Module {
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
  int device = 0;
  uint64_t used = 0;
  std::shared_ptr<ModuleUse> pin = std::make_shared<ModuleUse>();  // copies held by callers (JitStats::pin)
};

struct Job {  // a background compile: everything copied, nothing borrowed from the caller
  std::string key, arch, prelude, name_expr, mname, path;
};

// Process-wide state. The background worker is joined when the library is unloaded (process
// exit): a compile still running then finishes first, so hiprtc never runs while its library
// is being torn down. Queued compiles that have not started are dropped.
class Registry {
 public:
  std::mutex mu;
  std::condition_variable cv;                 // an entry left kCompiling, or a job arrived
  std::map<std::string, CodeEntry> code;      // key -> code object
  std::map<std::string, Module> modules;      // "device:key" -> loaded module
  std::deque<Job> jobs;
  int compiling = 0;                          // entries in kCompiling
  uint64_t tick = 0;
  bool stop = false;
  std::thread worker;

  ~Registry() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_all();
    if (worker.joinable()) worker.join();
    // modules are left to the runtime's own teardown: at exit it may already be gone
  }

  void finish(const std::string& key, int rc, std::vector<char>&& bytes, const std::string& err, bool from_disk) {
    auto it = code.find(key);
    if (it == code.end()) return;
    if (it->second.state == CodeEntry::kCompiling) --compiling;
    if (rc == FR_OK) {
      it->second.state = CodeEntry::kReady;
      it->second.code = std::make_shared<const std::vector<char>>(std::move(bytes));
      it->second.from_disk = from_disk;
    } else {
      it->second.state = CodeEntry::kFailed;
      it->second.error = err;
    }
    it->second.used = ++tick;
    trim_code();
    cv.notify_all();
  }

  void trim_code() {  // drop the least recently used ready code objects beyond kMaxCode
    while (code.size() > kMaxCode) {
      auto victim = code.end();
      for (auto it = code.begin(); it != code.end(); ++it)
        if (it->second.state != CodeEntry::kCompiling && (victim == code.end() || it->second.used < victim->second.used))
          victim = it;
      if (victim == code.end()) return;
      code.erase(victim);
    }
  }

  void run_worker() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stop || !jobs.empty(); });
      if (stop) {
        for (const Job& j : jobs) finish(j.key, FR_EHIP, {}, "abandoned at exit", false);
        jobs.clear();
        return;
      }
      Job j = std::move(jobs.front());
      jobs.pop_front();
      lk.unlock();
      std::vector<char> bytes;
      const int rc = compile_checked(j.arch, j.prelude, j.name_expr, j.mname, bytes);
      const std::string err = rc ? fr_last_error() : "";
      if (rc == FR_OK && !j.path.empty() && write_file_atomic(j.path, wrap_code(bytes)))
        prune_disk(j.path.substr(0, j.path.rfind('/')));
      lk.lock();
      finish(j.key, rc, std::move(bytes), err, false);
    }
  }

  void enqueue(Job&& j) {  // caller holds mu
    jobs.push_back(std::move(j));
    if (!worker.joinable()) worker = std::thread([this] { run_worker(); });
    cv.notify_all();
  }
};

Registry& reg() {
  static Registry r;
  return r;
}

// The device's target name (gcnArchName), queried once per device: every render of a
// scene-specialised frame looks its kernel up, and the property query is not free.
std::string device_arch(int device) {
  static std::mutex mu;
  static std::map<int, std::string> arch;
  std::lock_guard<std::mutex> g(mu);
  auto it = arch.find(device);
  if (it != arch.end()) return it->second;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return "";
  return arch[device] = prop.gcnArchName;
}

const std::string& toolchain() {
  static const std::string t = toolchain_tag();
  return t;
}

// Unload a module evicted from the table once every launch of it has finished: launches
// may still be queued on any stream it was launched on (jit_note_launch). No caller holds
// it (unpinned): a render that looked it up holds its pin from the lookup through the launch
// and the event record, so no launch of it can follow.
void unload_evicted(const Module& m) {
  int cur = -1;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(m.device);
  {
    std::lock_guard<std::mutex> g(m.pin->mu);
    for (auto& se : m.pin->last) {
      (void)hipEventSynchronize(se.second);
      (void)hipEventDestroy(se.second);
    }
    m.pin->last.clear();
  }
  (void)hipModuleUnload(m.mod);
  if (cur >= 0) (void)hipSetDevice(cur);
}

}  // namespace

int jit_compile_probe(const char* arch, const JitSpec& spec, size_t* code_bytes, double* ms) {
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<char> code;
  const int rc = compile_checked(arch, make_prelude(spec), spec.name_expr, mangled(spec.targs, spec.targ_bool, spec.n_targs),
                                 code);
  if (rc) return rc;
  if (code_bytes) *code_bytes = code.size();
  if (ms) *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return FR_OK;
}

int jit_wait_all() {
  Registry& R = reg();
  std::unique_lock<std::mutex> lk(R.mu);
  R.cv.wait(lk, [&] { return R.compiling == 0; });
  return FR_OK;
}

void jit_note_launch(const std::shared_ptr<void>& pin, hipStream_t stream) {
  ModuleUse* u = static_cast<ModuleUse*>(pin.get());
  if (!u) return;
  std::lock_guard<std::mutex> g(u->mu);
  for (auto& se : u->last)
    if (se.first == stream) {
      (void)hipEventRecord(se.second, stream);
      return;
    }
  // a stream not seen before (a new context, or a stream handle reused after one closed):
  // first drop entries whose launches have finished, so the list stays short
  if (u->last.size() >= kMaxStreamEvents) {
    auto keep = u->last.begin();
    for (auto& se : u->last) {
      if (hipEventQuery(se.second) == hipSuccess)
        (void)hipEventDestroy(se.second);
      else
        *keep++ = se;
    }
    u->last.erase(keep, u->last.end());
  }
  hipEvent_t ev = nullptr;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return;
  (void)hipEventRecord(ev, stream);
  u->last.emplace_back(stream, ev);
}

int jit_trace_kernel(int device, const JitSpec& spec, bool wait, hipFunction_t* out, JitStats* stats,
                     bool cached_only) {
  const auto t0 = std::chrono::steady_clock::now();
  JitStats st;
  auto done = [&](int state) {
    st.state = state;
    st.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (stats) *stats = st;
    return FR_OK;
  };
  *out = nullptr;
  const std::string arch = device_arch(device);
  if (arch.empty()) return set_error(FR_EHIP, "hipGetDeviceProperties failed");
  const std::string prelude = make_prelude(spec);
  const std::string key =
      hex_key(std::string(jit_src::kHash) + "\n" + arch + "\n" + spec.name_expr + "\n" + toolchain() + "\n" + prelude);
  const std::string mkey = std::to_string(device) + ":" + key;
  const std::string mname = mangled(spec.targs, spec.targ_bool, spec.n_targs);
  const std::string dir = cache_dir();
  const std::string path = dir.empty() ? "" : dir + "/" + key + ".hsaco";
  Registry& R = reg();
  std::unique_lock<std::mutex> lk(R.mu);
  auto mi = R.modules.find(mkey);
  if (mi != R.modules.end()) {
    mi->second.used = ++R.tick;
    *out = mi->second.fn;
    st.reused = 1;
    st.pin = mi->second.pin;
    return done(FR_JIT_USED);
  }
  // attempt 0 may take the disk cache; a disk file that does not load is deleted and the
  // kernel compiled once more (attempt 1)
  for (int attempt = 0; attempt < 2; ++attempt) {
    auto it = R.code.find(key);
    if (it == R.code.end()) {
      R.code[key];  // kCompiling: later requests for this key wait (or pend) on it
      ++R.compiling;
      lk.unlock();
      std::vector<char> bytes;
      if (attempt == 0 && !path.empty() && read_cached_code(path, bytes)) {
        lk.lock();
        R.finish(key, FR_OK, std::move(bytes), "", true);
      } else if (cached_only && !wait) {
        lk.lock();
        auto e = R.code.find(key);
        if (e != R.code.end() && e->second.state == CodeEntry::kCompiling) {
          R.code.erase(e);  // nothing was started for it
          --R.compiling;
          R.cv.notify_all();
        }
        return done(FR_JIT_MISS);
      } else if (wait) {
        const int rc = compile_checked(arch, prelude, spec.name_expr, mname, bytes);
        const std::string err = rc ? fr_last_error() : "";
        if (rc == FR_OK && !path.empty() && write_file_atomic(path, wrap_code(bytes))) prune_disk(dir);
        st.compiled = 1;
        lk.lock();
        R.finish(key, rc, std::move(bytes), err, false);
      } else {
        lk.lock();
        R.enqueue(Job{key, arch, prelude, spec.name_expr, mname, path});
        st.compiled = 1;
        return done(FR_JIT_PENDING);
      }
      it = R.code.find(key);
      if (it == R.code.end()) return set_error(FR_EHIP, "scene kernel code object evicted while loading");
    }
    if (it->second.state == CodeEntry::kCompiling) {
      if (!wait) return done(cached_only ? FR_JIT_MISS : FR_JIT_PENDING);
      R.cv.wait(lk, [&] {
        auto e = R.code.find(key);
        return e == R.code.end() || e->second.state != CodeEntry::kCompiling;
      });
      it = R.code.find(key);
      if (it == R.code.end()) continue;  // evicted meanwhile: look again
    }
    if (it->second.state == CodeEntry::kFailed) {
      if (!wait) {
        st.error = it->second.error;
        return done(FR_JIT_FAILED);
      }
      return set_error(FR_EHIP, "%s", it->second.error.c_str());
    }
    it->second.used = ++R.tick;
    const std::shared_ptr<const std::vector<char>> bytes = it->second.code;
    const bool from_disk = it->second.from_disk;
    lk.unlock();
    Module m;
    m.device = device;
    hipError_t e = hipModuleLoadData(&m.mod, bytes->data());
    if (e == hipSuccess) {
      e = hipModuleGetFunction(&m.fn, m.mod, mname.c_str());
      if (e != hipSuccess) (void)hipModuleUnload(m.mod);
    }
    lk.lock();
    if (e != hipSuccess) {
      if (from_disk && attempt == 0) {
        // a truncated or foreign file in the cache: remove it and build the kernel afresh
        if (!path.empty()) unlink(path.c_str());
        R.code.erase(key);
        continue;
      }
      return set_error(FR_EHIP, "loading the scene kernel %s: %s", mname.c_str(), hipGetErrorString(e));
    }
    auto prev = R.modules.find(mkey);
    if (prev != R.modules.end()) {  // another thread loaded it meanwhile: keep the first
      lk.unlock();
      (void)hipModuleUnload(m.mod);
      lk.lock();
      prev = R.modules.find(mkey);
      if (prev != R.modules.end()) {
        prev->second.used = ++R.tick;
        *out = prev->second.fn;
        st.pin = prev->second.pin;
        return done(FR_JIT_USED);
      }
      continue;
    }
    m.used = ++R.tick;
    R.modules[mkey] = m;
    *out = m.fn;
    st.pin = m.pin;
    // evict the least recently used modules beyond the bound, among those no caller pins
    // (a pin is copied only under this lock, so an unpinned module stays unpinned here)
    std::vector<Module> evicted;
    while (R.modules.size() > max_modules()) {
      auto victim = R.modules.end();
      for (auto v = R.modules.begin(); v != R.modules.end(); ++v)
        if (v->second.pin.use_count() == 1 && (victim == R.modules.end() || v->second.used < victim->second.used))
          victim = v;
      if (victim == R.modules.end()) break;  // every module is pinned: stay over the bound
      evicted.push_back(victim->second);
      R.modules.erase(victim);
    }

    lk.unlock();
    for (const Module& v : evicted) unload_evicted(v);
    return done(FR_JIT_USED);
  }
  return set_error(FR_EHIP, "scene kernel: no code object after a recompile");
}

}  // namespace fr
