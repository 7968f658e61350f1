/* abi_consumer.c — a plain C11 program built by gcc against include/forma_rt.h and
 * linked to fo-rma_amd/libforma_rt.so, the way the Rust binding in INTEGRATION.md would
 * bind it (cpu_ray_tracer/tracer.rs:19-28 TraceModel, shapes/hitable.rs:4-14 Hitable).
 *
 * Compile time: every field offset the #[repr(C)] Rust mirror in INTEGRATION.md assumes
 * is _Static_assert-ed here, so a header change that moves a field fails this build.
 *
 *   abi_consumer layout              print every struct size and field offset (JSON); no GPU
 *   abi_consumer render SCENE W H SPP DEPTH OUT
 *                                    render a scene file through fr_ctx_* on device 0 and
 *                                    write the f32 means, the u8 image and the stats to OUT
 *   abi_consumer mrender SCENE W H SPP DEPTH OUT DEVICES
 *                                    INTEGRATION.md's create_model / save_image sequence:
 *                                    fr_mctx_create(DEVICES, e.g. "0,0"), two frames of
 *                                    fr_mctx_render (FR_FLAG_WRITE_U8 | FR_FLAG_SCENE_JIT)
 *                                    + fr_mctx_sync + fr_mctx_frame (the second after
 *                                    fr_jit_wait, so it runs the scene kernel), fr_mctx_free;
 *                                    both frames, their stats and every shard's
 *                                    fr_ctx_jit_state go to OUT
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "forma_rt.h"

/* FrPrim { kind: u32, material: u32, color: [f32; 3], fuzz: f32, g: [f32; 16] } */
_Static_assert(offsetof(fr_prim, kind) == 0, "fr_prim.kind");
_Static_assert(offsetof(fr_prim, material) == 4, "fr_prim.material");
_Static_assert(offsetof(fr_prim, color) == 8, "fr_prim.color");
_Static_assert(offsetof(fr_prim, fuzz) == 20, "fr_prim.fuzz");
_Static_assert(offsetof(fr_prim, g) == 24, "fr_prim.g");
_Static_assert(sizeof(fr_prim) == 88, "fr_prim size");
/* FrCamera: seven [f32; 3] then five f32 (26 floats) */
_Static_assert(offsetof(fr_camera, position) == 0, "fr_camera.position");
_Static_assert(offsetof(fr_camera, lower_left) == 12, "fr_camera.lower_left");
_Static_assert(offsetof(fr_camera, horizontal) == 24, "fr_camera.horizontal");
_Static_assert(offsetof(fr_camera, vertical) == 36, "fr_camera.vertical");
_Static_assert(offsetof(fr_camera, u) == 48, "fr_camera.u");
_Static_assert(offsetof(fr_camera, v) == 60, "fr_camera.v");
_Static_assert(offsetof(fr_camera, w) == 72, "fr_camera.w");
_Static_assert(offsetof(fr_camera, aspect) == 84, "fr_camera.aspect");
_Static_assert(offsetof(fr_camera, lens_radius) == 88, "fr_camera.lens_radius");
_Static_assert(offsetof(fr_camera, focus_dist) == 92, "fr_camera.focus_dist");
_Static_assert(offsetof(fr_camera, radius) == 96, "fr_camera.radius");
_Static_assert(offsetof(fr_camera, rotation) == 100, "fr_camera.rotation");
_Static_assert(sizeof(fr_camera) == 104, "fr_camera size");
/* FrParams: four u32, a u64 at 16, four u32 */
_Static_assert(offsetof(fr_params, width) == 0, "fr_params.width");
_Static_assert(offsetof(fr_params, height) == 4, "fr_params.height");
_Static_assert(offsetof(fr_params, spp) == 8, "fr_params.spp");
_Static_assert(offsetof(fr_params, max_depth) == 12, "fr_params.max_depth");
_Static_assert(offsetof(fr_params, seed) == 16, "fr_params.seed");
_Static_assert(offsetof(fr_params, strip_rows) == 24, "fr_params.strip_rows");
_Static_assert(offsetof(fr_params, shard_index) == 28, "fr_params.shard_index");
_Static_assert(offsetof(fr_params, shard_count) == 32, "fr_params.shard_count");
_Static_assert(offsetof(fr_params, flags) == 36, "fr_params.flags");
_Static_assert(sizeof(fr_params) == 40, "fr_params size");
/* FrStats: four u64, three f64, two u32, a u64 */
_Static_assert(offsetof(fr_stats, segments) == 0, "fr_stats.segments");
_Static_assert(offsetof(fr_stats, hits) == 8, "fr_stats.hits");
_Static_assert(offsetof(fr_stats, samples) == 16, "fr_stats.samples");
_Static_assert(offsetof(fr_stats, prim_tests) == 24, "fr_stats.prim_tests");
_Static_assert(offsetof(fr_stats, kernel_ms) == 32, "fr_stats.kernel_ms");
_Static_assert(offsetof(fr_stats, total_ms) == 40, "fr_stats.total_ms");
_Static_assert(offsetof(fr_stats, trace_ms) == 48, "fr_stats.trace_ms");
_Static_assert(offsetof(fr_stats, trace_launches) == 56, "fr_stats.trace_launches");
_Static_assert(offsetof(fr_stats, occupancy) == 60, "fr_stats.occupancy");
_Static_assert(offsetof(fr_stats, scatters) == 64, "fr_stats.scatters");
_Static_assert(sizeof(fr_stats) == 72, "fr_stats size");

#define FIELD(T, f) printf("  \"%s.%s\": [%zu, %zu],\n", #T, #f, offsetof(T, f), sizeof(((T*)0)->f))

static int layout(void) {
  printf("{\n");
  FIELD(fr_prim, kind); FIELD(fr_prim, material); FIELD(fr_prim, color); FIELD(fr_prim, fuzz); FIELD(fr_prim, g);
  FIELD(fr_camera, position); FIELD(fr_camera, lower_left); FIELD(fr_camera, horizontal);
  FIELD(fr_camera, vertical); FIELD(fr_camera, u); FIELD(fr_camera, v); FIELD(fr_camera, w);
  FIELD(fr_camera, aspect); FIELD(fr_camera, lens_radius); FIELD(fr_camera, focus_dist);
  FIELD(fr_camera, radius); FIELD(fr_camera, rotation);
  FIELD(fr_params, width); FIELD(fr_params, height); FIELD(fr_params, spp); FIELD(fr_params, max_depth);
  FIELD(fr_params, seed); FIELD(fr_params, strip_rows); FIELD(fr_params, shard_index);
  FIELD(fr_params, shard_count); FIELD(fr_params, flags);
  FIELD(fr_stats, segments); FIELD(fr_stats, hits); FIELD(fr_stats, samples); FIELD(fr_stats, prim_tests);
  FIELD(fr_stats, kernel_ms); FIELD(fr_stats, total_ms); FIELD(fr_stats, trace_ms);
  FIELD(fr_stats, trace_launches); FIELD(fr_stats, occupancy); FIELD(fr_stats, scatters);
  printf("  \"sizeof\": [%zu, %zu, %zu, %zu],\n", sizeof(fr_prim), sizeof(fr_camera), sizeof(fr_params),
         sizeof(fr_stats));
  printf("  \"abi_version\": %d\n}\n", fr_abi_version());
  return fr_abi_version() == FR_ABI_VERSION ? 0 : 3;
}

static int fail(const char* what, int rc) {
  fprintf(stderr, "%s failed (%d): %s\n", what, rc, fr_last_error());
  return 1;
}

static int load_scene(const char* scene_path, uint32_t w, uint32_t h, fr_scene** scene, fr_camera* cam) {
  FILE* f = fopen(scene_path, "rb");
  if (!f) return fail("fopen scene", -1);
  fseek(f, 0, SEEK_END);
  const long len = ftell(f);
  fseek(f, 0, SEEK_SET);
  char* text = malloc((size_t)len);
  if (!text || fread(text, 1, (size_t)len, f) != (size_t)len) return fail("read scene", -1);
  fclose(f);
  const int rc = fr_scene_from_json(text, (size_t)len, w, h, scene, cam);
  free(text);
  return rc ? fail("fr_scene_from_json", rc) : 0;
}

static int render(const char* scene_path, uint32_t w, uint32_t h, uint32_t spp, uint32_t depth, const char* out) {
  fr_scene* scene = NULL;
  fr_camera cam;
  int rc = load_scene(scene_path, w, h, &scene, &cam);
  if (rc) return rc;
  fr_params p;
  memset(&p, 0, sizeof(p));
  p.width = w;
  p.height = h;
  p.spp = spp;
  p.max_depth = depth;
  p.seed = 0x5EED;
  p.strip_rows = 8;
  p.shard_index = 0;
  p.shard_count = 1;
  p.flags = FR_FLAG_WRITE_U8;
  fr_ctx* ctx = NULL;
  if ((rc = fr_ctx_create(0, NULL, &ctx))) return fail("fr_ctx_create", rc);
  if ((rc = fr_ctx_render(ctx, scene, &cam, &p))) return fail("fr_ctx_render", rc);
  fr_stats st;
  if ((rc = fr_ctx_sync(ctx, &st))) return fail("fr_ctx_sync", rc);
  const size_t n = (size_t)w * h * 3;
  float* mean = NULL;
  uint8_t* rgb8 = NULL;
  /* pinned targets and the asynchronous gather, as a frame loop would use them */
  if ((rc = fr_host_alloc(n * sizeof(float), (void**)&mean))) return fail("fr_host_alloc", rc);
  if ((rc = fr_host_alloc(n, (void**)&rgb8))) return fail("fr_host_alloc", rc);
  if ((rc = fr_ctx_download_async(ctx, mean, rgb8))) return fail("fr_ctx_download_async", rc);
  if ((rc = fr_ctx_wait(ctx))) return fail("fr_ctx_wait", rc);
  FILE* o = fopen(out, "wb");
  if (!o) return fail("fopen out", -1);
  fwrite(mean, sizeof(float), n, o);
  fwrite(rgb8, 1, n, o);
  const uint64_t counters[4] = {st.segments, st.hits, st.samples, st.scatters};
  fwrite(counters, sizeof(uint64_t), 4, o);
  fclose(o);
  fr_host_free(mean);
  fr_host_free(rgb8);
  fr_ctx_free(ctx);
  fr_scene_free(scene);
  return 0;
}

/* The Rust binding's model (INTEGRATION.md create_model / frame / save_image / Drop) */
static int mrender(const char* scene_path, uint32_t w, uint32_t h, uint32_t spp, uint32_t depth, const char* out,
                   const char* devices_csv) {
  int devices[64];
  int n = 0;
  for (const char* c = devices_csv; *c && n < 64;) {
    devices[n++] = atoi(c);
    while (*c && *c != ',') ++c;
    if (*c == ',') ++c;
  }
  fr_scene* scene = NULL;
  fr_camera cam;
  int rc = load_scene(scene_path, w, h, &scene, &cam);
  if (rc) return rc;
  fr_mctx* mctx = NULL;
  if ((rc = fr_mctx_create(devices, n, &mctx))) return fail("fr_mctx_create", rc);
  fr_params p;
  memset(&p, 0, sizeof(p));
  p.width = w;
  p.height = h;
  p.spp = spp;
  p.max_depth = depth;
  p.seed = 0x5EED;
  p.strip_rows = 8;
  p.shard_index = 0; /* set per device by fr_mctx */
  p.shard_count = 1;
  p.flags = FR_FLAG_WRITE_U8 | FR_FLAG_SCENE_JIT;
  FILE* o = fopen(out, "wb");
  if (!o) return fail("fopen out", -1);
  const size_t npx = (size_t)w * h * 3;
  for (int frame = 0; frame < 2; ++frame) {
    if (frame == 1 && (rc = fr_jit_wait())) return fail("fr_jit_wait", rc);
    fr_stats st;
    const float* mean = NULL;
    const uint8_t* rgb8 = NULL;
    if ((rc = fr_mctx_render(mctx, scene, &cam, &p))) return fail("fr_mctx_render", rc);
    if ((rc = fr_mctx_sync(mctx, &st))) return fail("fr_mctx_sync", rc);
    if ((rc = fr_mctx_frame(mctx, &mean, &rgb8))) return fail("fr_mctx_frame", rc);
    fwrite(mean, sizeof(float), npx, o);
    fwrite(rgb8, 1, npx, o);
    const uint64_t counters[4] = {st.segments, st.hits, st.samples, st.scatters};
    fwrite(counters, sizeof(uint64_t), 4, o);
    for (int i = 0; i < n; ++i) {
      fr_ctx* ctx = NULL;
      int32_t state = -1;
      if ((rc = fr_mctx_ctx(mctx, i, &ctx)) || (rc = fr_ctx_jit_state(ctx, &state))) return fail("fr_ctx_jit_state", rc);
      fwrite(&state, sizeof(state), 1, o);
    }
  }
  fclose(o);
  fr_mctx_free(mctx);
  fr_scene_free(scene);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && strcmp(argv[1], "layout") == 0) return layout();
  if (argc == 9 && strcmp(argv[1], "mrender") == 0)
    return mrender(argv[2], (uint32_t)atoi(argv[3]), (uint32_t)atoi(argv[4]), (uint32_t)atoi(argv[5]),
                   (uint32_t)atoi(argv[6]), argv[7], argv[8]);
  if (argc == 8 && strcmp(argv[1], "render") == 0)
    return render(argv[2], (uint32_t)atoi(argv[3]), (uint32_t)atoi(argv[4]), (uint32_t)atoi(argv[5]),
                  (uint32_t)atoi(argv[6]), argv[7]);
  fprintf(stderr, "usage: %s layout | render SCENE W H SPP DEPTH OUT | mrender SCENE W H SPP DEPTH OUT DEVICES\n",
          argv[0]);
  return 2;
}
