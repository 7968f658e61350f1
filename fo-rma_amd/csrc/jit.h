// jit.h — the scene-specialised trace kernel (jit.cpp): host interface inside libforma_rt.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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
  double ms;      // wall time of this call (compile or cache load, module load)
  int compiled;   // 1: hiprtc ran; 0: code object from the disk cache or module reused
  int reused;     // 1: the module was already loaded in this process
};

// The kernel for spec on device (current device must be `device`). FR_OK, or an FR_E*
// code with fr_last_error() holding hiprtc's log: the caller fails the render (no
// silent fallback, so a broken run-time build cannot hide behind the generic kernel).
int jit_trace_kernel(int device, const JitSpec& spec, hipFunction_t* out, JitStats* stats);

// hiprtc only, no device (tests): compiles spec for arch and checks that the kernel's
// lowered name is the one jit_trace_kernel looks up.
int jit_compile_probe(const char* arch, const JitSpec& spec, size_t* code_bytes, double* ms);

}  // namespace fr
