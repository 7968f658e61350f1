// jit.h — the scene-specialised trace kernel (jit.cpp): host interface inside libforma_rt.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <string>

namespace fr {

// List-loop scenes up to this many primitives may be compiled into the kernel: the
// unrolled list stays within a few KB of code, and every record is staged in LDS
// (kRecLds) for the winner's shading as in the list kernels.
constexpr uint32_t kJitMaxPrims = 64;

struct JitSpec {
  const char* name_expr;   // "fr::trace_kernel<KS, HP, ...>": the launch's specialisation
  const int* targs;        // its template arguments, for the mangled name
  const bool* targ_bool;   // which of them are bool
  int n_targs;
  std::string defines;     // the host build's tuning and contract macros (#define lines)
  const uint32_t* rec;     // n x 16 words: the scene's 64-B device records, list order
  uint32_t n;
};

struct JitStats {
  double ms = 0.0;   // wall time of this call (cache or module load, or a compile it ran or waited for)
  int compiled = 0;  // 1: hiprtc ran for this request (in this call, or started in the background)
  int reused = 0;    // 1: the module was already loaded in this process
  int state = 0;     // FR_JIT_* (forma_rt.h): USED, PENDING (no kernel yet) or FAILED
  std::string error; // FAILED: the compiler's message
  // USED: holds the module loaded: while any copy of it lives, the LRU never unloads the
  // module, so a caller may keep the function handle with it (fr_ctx's kernel cache)
  std::shared_ptr<void> pin;
};

// The scene kernel for spec on `device` (the current device must be `device`).
// wait = true: compile on this thread if no code object exists (or wait for the background
// compile of the same key); FR_OK with *out set, or an FR_E* code with fr_last_error()
// holding hiprtc's log.
// wait = false: never compiles on this thread. A code object already built (this process)
// or cached on disk is loaded and returned; otherwise the compile is queued on the
// background worker and FR_OK returns with *out = nullptr and stats->state PENDING (or
// FAILED after a failed compile): the caller runs the compiled-in kernel, whose image is
// the same bits.
// cached_only (wait = false): a code object in this process or on disk is used, as above;
// otherwise nothing is compiled or queued: *out = nullptr, stats->state FR_JIT_MISS (a
// one-shot caller then neither waits for hiprtc nor leaves a compile for process exit).
int jit_trace_kernel(int device, const JitSpec& spec, bool wait, hipFunction_t* out, JitStats* stats,
                     bool cached_only = false);

// After a launch of a module's kernel on `stream`: the module is unloaded (LRU eviction)
// only after this launch has finished (an event on the stream, not a device drain).
void jit_note_launch(const std::shared_ptr<void>& pin, hipStream_t stream);

// Block until the background worker has no compile queued or running.
int jit_wait_all();


// hiprtc only, no device (tests): compiles spec for arch and checks that the kernel's
// lowered name is the one jit_trace_kernel looks up.
int jit_compile_probe(const char* arch, const JitSpec& spec, size_t* code_bytes, double* ms);

}  // namespace fr
