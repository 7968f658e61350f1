// host_sanitize.cpp — test harness (tests/test_host_sanitizers.py): the product's host code
// (fo-rma_amd/csrc/json_min.cpp, scene.cpp, bvh.cpp) and the oracle (oracle/oracle.cpp)
// built together with -fsanitize=address,undefined -fno-sanitize-recover=all into one CPU
// executable, so any out-of-bounds access, use-after-free, leak or undefined behaviour in
// the JSON loader (basics/scene_loader.rs:3-7's counterpart), the mesh builders or the BVH
// builder aborts the run.
//
//   host_sanitize json FILE...     parse each file through fr_scene_from_json (malformed
//                                  ones must fail with FR_EPARSE, never crash); for each
//                                  scene that loads: the primitive list, the BVH build
//                                  (plain and forced) and a tiny oracle render of it
//   host_sanitize spheres N        N spheres on a grid (fr_scene_create) through the BVH
//                                  builder, plain and forced
//   host_sanitize cache FILE...    each file through the scene kernel's disk-cache reader
//                                  (fo-rma_amd/csrc/jit_cache.cpp read_cached_code, the
//                                  guard in front of the HIP loader); a file that passes is
//                                  re-wrapped and must equal itself byte for byte
//   host_sanitize wrap N OUT       a valid cache file around N bytes of code
// One JSON line per input on stdout.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "../../include/forma_rt.h"
#include "../../fo-rma_amd/csrc/bvh.h"
#include "../../fo-rma_amd/csrc/internal.h"
#include "../../fo-rma_amd/csrc/jit_cache.h"

// A host-only build makes no device copies of a scene: fr_scene_free has none to release.
namespace fr {
void release_device_copies(fr_scene* s) { s->copies.clear(); }
}  // namespace fr

extern "C" {
typedef struct or_camera {
  float position[3], lower_left[3], horizontal[3], vertical[3], u[3], v[3], w[3];
  float aspect, lens_radius, focus_dist, radius, rotation;
} or_camera;
typedef struct or_counters {
  uint64_t segments, hits, samples, scatters;
} or_counters;
int64_t oracle_render(const fr_prim* prims, uint32_t n, const or_camera* cam, uint32_t width, uint32_t height,
                      uint32_t spp, uint32_t max_depth, uint64_t seed, uint32_t shard_index, uint32_t shard_count,
                      uint32_t row_step, uint32_t col_step, int threads, float* out_mean, uint8_t* out_u8,
                      or_counters* counters);
}
static_assert(sizeof(or_camera) == sizeof(fr_camera), "oracle and product cameras share the layout");

static void bvh_report(const std::vector<fr_prim>& prims, bool force) {
  std::vector<fr::BvhSegment> segs;
  std::vector<fr::BvhNode> nodes;
  std::vector<uint32_t> order;
  float extent = 0.0f;
  const auto t0 = std::chrono::steady_clock::now();
  const bool ok = fr::build_segments(prims, segs, nodes, order, force, &extent);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  const uint32_t depth = ok ? fr::bvh_max_depth(segs, nodes) : 0u;
  // a digest of the tree (node boxes, references, leaf order): builder changes that must
  // not change the tree are checked with it
  uint64_t h = 0xcbf29ce484222325ull;
  auto mix = [&h](const void* p, size_t n) {
    for (size_t i = 0; i < n; ++i) h = (h ^ static_cast<const unsigned char*>(p)[i]) * 0x100000001b3ull;
  };
  if (!nodes.empty()) mix(nodes.data(), nodes.size() * sizeof(fr::BvhNode));
  if (!order.empty()) mix(order.data(), order.size() * sizeof(uint32_t));
  if (!segs.empty()) mix(segs.data(), segs.size() * sizeof(fr::BvhSegment));
  printf(", \"bvh%s\": {\"ok\": %d, \"segments\": %zu, \"nodes\": %zu, \"order\": %zu, \"depth\": %u, "
         "\"build_ms\": %.3f, \"digest\": \"%016llx\"}",
         force ? "_forced" : "", ok ? 1 : 0, segs.size(), nodes.size(), order.size(), depth, ms,
         static_cast<unsigned long long>(h));
}

static int do_json(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) return 2;
  std::string text;
  char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, n);
  fclose(f);
  fr_scene* scene = nullptr;
  fr_camera cam;
  // an exact-size heap copy: a read past the end is caught
  char* exact = static_cast<char*>(malloc(text.size() ? text.size() : 1));
  memcpy(exact, text.data(), text.size());
  const int rc = fr_scene_from_json(exact, text.size(), 32, 18, &scene, &cam);
  free(exact);
  printf("{\"file\": \"%s\", \"rc\": %d", path, rc);
  if (rc == FR_OK) {
    const uint32_t count = fr_scene_count(scene);
    std::vector<fr_prim> prims(count);
    if (count) fr_scene_get_prims(scene, prims.data(), count);
    printf(", \"prims\": %u", count);
    bvh_report(prims, false);
    bvh_report(prims, true);
    std::vector<float> mean(32 * 18 * 3);
    std::vector<uint8_t> u8(32 * 18 * 3);
    or_counters cnt{};
    or_camera ocam;
    memcpy(&ocam, &cam, sizeof ocam);
    const int64_t rows = oracle_render(prims.data(), count, &ocam, 32, 18, 1, 4, 0x5EED, 0, 1, 1, count > 1000 ? 9 : 1,
                                       2, mean.data(), u8.data(), &cnt);
    printf(", \"oracle_rows\": %lld, \"segments\": %llu", static_cast<long long>(rows),
           static_cast<unsigned long long>(cnt.segments));
    fr_scene_free(scene);
  } else {
    std::string msg = std::string(fr_last_error()).substr(0, 60);
    for (char& c : msg)
      if (c == '"' || c == '\\' || static_cast<unsigned char>(c) < 0x20 || static_cast<unsigned char>(c) > 0x7e) c = '?';
    printf(", \"error\": \"%s\"", msg.c_str());
  }
  printf("}\n");
  return 0;
}

static int do_spheres(uint32_t n) {
  std::vector<fr_prim> prims(n);
  const uint32_t side = 64;
  for (uint32_t i = 0; i < n; ++i) {
    fr_prim& p = prims[i];
    memset(&p, 0, sizeof p);
    p.kind = FR_SPHERE;
    p.material = i % 4;
    p.color[0] = p.color[1] = p.color[2] = 0.5f;
    p.g[0] = static_cast<float>(i % side) * 1.5f;
    p.g[1] = static_cast<float>((i / side) % side) * 1.5f;
    p.g[2] = static_cast<float>(i / (side * side)) * 1.5f;
    p.g[3] = 0.5f + 0.25f * static_cast<float>(i % 3);
  }
  fr_scene* scene = nullptr;
  const int rc = fr_scene_create(prims.data(), n, &scene);
  printf("{\"spheres\": %u, \"rc\": %d", n, rc);
  if (rc == FR_OK) {
    bvh_report(prims, false);
    bvh_report(prims, true);
    fr_scene_free(scene);
  }
  printf("}\n");
  return rc == FR_OK ? 0 : 1;
}

static int do_cache(const char* path) {
  std::vector<char> raw, code;
  const bool had = fr::read_file(path, raw);
  const bool ok = fr::read_cached_code(path, code);
  bool same = false;
  if (ok) same = fr::wrap_code(code) == raw;
  printf("{\"file\": \"%s\", \"readable\": %d, \"ok\": %d, \"code_bytes\": %zu, \"rewrap_equal\": %d}\n", path,
         had ? 1 : 0, ok ? 1 : 0, code.size(), same ? 1 : 0);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 3 && strcmp(argv[1], "cache") == 0) {
    for (int i = 2; i < argc; ++i) do_cache(argv[i]);
    return 0;
  }
  if (argc == 4 && strcmp(argv[1], "wrap") == 0) {
    std::vector<char> code(static_cast<size_t>(atoi(argv[2])));
    for (size_t i = 0; i < code.size(); ++i) code[i] = static_cast<char>(i * 131u + 7u);
    return fr::write_file_atomic(argv[3], fr::wrap_code(code)) ? 0 : 1;
  }
  if (argc >= 3 && strcmp(argv[1], "json") == 0) {
    for (int i = 2; i < argc; ++i)
      if (do_json(argv[i])) return 2;
    return 0;
  }
  if (argc == 3 && strcmp(argv[1], "spheres") == 0) return do_spheres(static_cast<uint32_t>(atoi(argv[2])));
  fprintf(stderr, "usage: %s json FILE... | spheres N | cache FILE... | wrap N OUT\n", argv[0]);
  return 2;
}
