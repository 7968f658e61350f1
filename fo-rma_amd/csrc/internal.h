// internal.h — shared host-side state of libforma_rt (not part of the C ABI).
#pragma once
#include <stdarg.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/forma_rt.h"

namespace fr {

// thread-local last-error message behind fr_last_error()
int set_error(int code, const char* fmt, ...);

struct DeviceCopy;  // defined in render.hip

}  // namespace fr

// The tracer's Scene (cpu_ray_tracer/scene.rs:4-7): an ordered primitive list.
// Device copies are created lazily per device and dropped when `version` moves.
struct fr_scene {
  std::vector<fr_prim> prims;
  uint64_t version = 1;
  std::mutex mu;
  std::vector<fr::DeviceCopy*> copies;  // owned; freed by fr_scene_free
};

namespace fr {
void release_device_copies(fr_scene* s);  // render.hip
}
