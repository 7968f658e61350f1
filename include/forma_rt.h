/*
 * forma_rt.h — C ABI of the MI355X-native path tracer that drops in for
 * fo-rma's CPU ray tracer (zehreken/fo-rma, src/cpu_ray_tracer + src/shapes).
 *
 * Everything here is plain C: POD structs with explicit layout, opaque handles,
 * integer error codes. No torch or HIP types appear in any signature (a HIP
 * stream is passed as `void*`). A `#[repr(C)]` Rust mirror of this header is in
 * INTEGRATION.md.
 *
 * Which reference interface each entry point replaces (paths relative to the
 * reference root):
 *
 *   fr_prim / fr_scene_create ........ shapes/hitable.rs:4-14 (trait Hitable), the
 *                                      Sphere/Plane/AABB/Rectangle constructors
 *                                      (shapes/sphere.rs:75-83, plane.rs:48-66,
 *                                      aabb.rs:36-44, rectangle.rs:36-44) and
 *                                      cpu_ray_tracer/scene.rs:4-15 (Scene.objects)
 *   fr_scene_builtin ................. cpu_ray_tracer/scenes.rs:6,41,110
 *                                      (get_simple_scene / get_plane_scene / get_objects)
 *   fr_scene_from_json ............... basics/scene_loader.rs:3-7 (construct_scene_from_json)
 *                                      + basics/scene.rs:55-99 (mesh/material dispatch),
 *                                      mapped to tracer primitives
 *   fr_scene_translate / _rotate ..... shapes/hitable.rs:12-13, shapes/plane.rs:62-68
 *   fr_camera_init ................... cpu_ray_tracer/camera.rs:24-60 (Camera::new)
 *   fr_camera_look ................... camera.rs:24-60 generalised to a JSON camera
 *   fr_camera_orbit .................. camera.rs:97-122 (Camera::orbit)
 *   fr_camera_translate .............. camera.rs:74-95 (Camera::translate)
 *   fr_update_delta .................. cpu_ray_tracer/tracer.rs:30-52 (update's key bitmask)
 *   fr_ctx_render / fr_render_hip .... cpu_ray_tracer/tracer.rs:160-219 (save_image +
 *                                      get_color) and tracer.rs:57-81 (render, 1 spp)
 *   fr_mctx_* / fr_render_hip_multi .. tracer.rs:83-134 (render_mt row tiling), one
 *                                      device per row shard instead of one thread;
 *                                      fr_mctx keeps the per-device contexts and a
 *                                      page-locked frame across renders (update loop)
 *
 * Errors: 0 = ok, negative = FR_E*; the message is in fr_last_error() (thread-local).
 * Threading: calls on distinct fr_scene / fr_ctx objects are re-entrant. A fr_ctx is
 * bound to one device and one HIP stream and must not be used by two threads at once.
 */
#ifndef FORMA_RT_H
#define FORMA_RT_H

#if !defined(__HIPCC_RTC__) /* hiprtc (the scene-specialised build) provides these types */
#include <stddef.h>
#endif
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FR_ABI_VERSION 6 /* 2: fr_stats.trace_launches; FR_TRIANGLE; post effects; FR_FLAG_MT_BANDS
                            3: fr_stats.scatters/.occupancy; fr_ctx_download_async, fr_ctx_wait,
                               fr_host_alloc/free; item-major sample buffer
                            4: fr_mctx_* (persistent multi-device context); fr_ctx_trace_log(_read);
                               entry points restore the caller's current HIP device
                            5: FR_FLAG_SCENE_JIT, fr_ctx_prepare, fr_ctx_jit_info
                            6: FR_FLAG_SCENE_JIT compiles in the background (renders never wait),
                               FR_FLAG_SCENE_JIT_WAIT, fr_ctx_jit_state, fr_jit_wait */

/* error codes */
#define FR_OK 0
#define FR_EARG (-1)   /* invalid argument */
#define FR_EPARSE (-2) /* JSON syntax error or unsupported mesh */
#define FR_EHIP (-3)   /* a HIP runtime call failed */
#define FR_ENODEV (-4) /* no HIP device / requested device missing */
#define FR_ENOMEM (-5) /* allocation failed */

/* primitive kinds (one Hitable implementation each) */
#define FR_SPHERE 0u /* shapes/sphere.rs */
#define FR_PLANE 1u  /* shapes/plane.rs (bounded, world-axis extent) */
#define FR_AABB 2u   /* build-defined axis-aligned box (JSON "cube" with a signed-permutation rotation) */
#define FR_OBB 3u    /* build-defined oriented box (JSON "cube", any other rotation) */
#define FR_STUB 4u   /* shapes/aabb.rs / rectangle.rs: hit() and scatter() always false */
#define FR_TRIANGLE 5u /* build-defined triangle: JSON triangle/circle/cylinder/tetrahedron meshes, tilted quads */

/* material ids as the reference stores them (u8 `material` field) */
#define FR_LAMBERTIAN 0u /* sphere.rs:84-89, plane.rs:101-106 */
#define FR_METAL 1u      /* sphere.rs:91-105, plane.rs:108-122 */
#define FR_DIELECTRIC 2u /* sphere.rs:107-145 (spheres and boxes only) */
#define FR_LIGHT 3u      /* sphere.rs:147-152 (no emission: attenuation 1) */

/* flags for fr_params.flags */
#define FR_FLAG_WRITE_U8 1u /* also write the u8 image (tracer.rs:177-184) */
/* save_image_mt (tracer.rs:83-158): 4 row bands of H/4 rows, v = ((H/4 - y_band) + r)/H
   + band * 0.25, each sample gamma-corrected and quantised to u8, the u8 values averaged
   as acc += u8 / spp in f32 and truncated; rows past 4 * (H/4) stay 0. mean_rgb then
   holds acc (0..255). Render the plain simple scene (fr_scene_builtin 0) with
   max_depth 50 to match the reference call. */
#define FR_FLAG_MT_BANDS 2u
/* Scene-specialised trace kernel (render.hip / jit.cpp): for list-loop scenes of at most 64
   primitives, the kernel compiled once per scene with the primitive records as constants
   (hiprtc; one code object per GPU architecture, cached per process and on disk,
   FR_JIT_CACHE). Same image bits as without the flag; shared slab planes are computed once
   per segment. A render never waits for the compile: when no code object exists yet it is
   queued on a background host thread and the render runs the compiled-in kernel
   (fr_ctx_jit_state says FR_JIT_PENDING); a later render picks the scene kernel up.
   fr_ctx_prepare, FR_FLAG_SCENE_JIT_WAIT, and FR_SCENE_JIT=1 in the environment wait for it
   instead (FR_SCENE_JIT=0 turns it off for every render). */
#define FR_FLAG_SCENE_JIT 4u
#define FR_FLAG_SCENE_JIT_WAIT 8u /* with FR_FLAG_SCENE_JIT: compile on the render's thread if needed */
/* with FR_FLAG_SCENE_JIT (not _WAIT): use the scene kernel only if its code object is in this
   process or the disk cache; never compile or queue a compile (FR_JIT_MISS otherwise). For
   one-shot callers: a queued background compile runs to its end when the process exits, so
   a process that renders once and exits would otherwise wait for hiprtc at exit. */
#define FR_FLAG_SCENE_JIT_CACHED 16u
/* fr_ctx_jit_state: which trace kernel the last render (or fr_ctx_prepare) ran */
#define FR_JIT_OFF 0     /* compiled-in kernel: not asked for, a BVH scene, or > 64 primitives */
#define FR_JIT_USED 1    /* the scene-specialised kernel */
#define FR_JIT_PENDING 2 /* asked for, compile still running: the compiled-in kernel ran */
#define FR_JIT_FAILED 3  /* asked for, compile failed: the compiled-in kernel ran */
#define FR_JIT_MISS 4    /* asked for cached only (FR_FLAG_SCENE_JIT_CACHED), none cached: compiled-in kernel */

/*
 * One primitive, in the order it is tested (list order decides ties, tracer.rs:195-200).
 * Geometry `g` by kind:
 *   FR_SPHERE : g[0..2] center, g[3] radius
 *   FR_PLANE  : g[0..2] position, g[3..5] orientation, g[6..8] size (half extents per world axis)
 *   FR_AABB   : g[0..2] min corner, g[3..5] max corner
 *   FR_OBB    : g[0..2] center, g[3..5] local x axis, g[6..8] local y axis, g[9..11] local z axis
 *               (unit rows of the world->local rotation), g[12..14] half extents
 *   FR_STUB   : unused
 *   FR_TRIANGLE: g[0..2], g[3..5], g[6..8] the world vertices v0, v1, v2 (winding v0 -> v1 -> v2)
 * `material` is the raw reference id; unknown ids fall back as sphere.rs:68 / plane.rs:55 do.
 */
typedef struct fr_prim {
  uint32_t kind;
  uint32_t material;
  float color[3];
  float fuzz;
  float g[16];
} fr_prim;

/* Mirrors the fields of cpu_ray_tracer::camera::Camera (camera.rs:8-21), f32 throughout. */
typedef struct fr_camera {
  float position[3];
  float lower_left[3];
  float horizontal[3];
  float vertical[3];
  float u[3];
  float v[3];
  float w[3];
  float aspect;
  float lens_radius;
  float focus_dist; /* stored 2.0 by Camera::new, never used (camera.rs:56) */
  float radius;     /* orbit radius, 5.0 (camera.rs:57) */
  float rotation;   /* orbit angle, 0.0 (camera.rs:58) */
} fr_camera;

/*
 * Render parameters. Rows are grouped into strips of `strip_rows` (must be 8) rows;
 * strip k belongs to shard (k % shard_count). A shard renders only its own strips,
 * so shards of one image are disjoint and stitch bit-exactly.
 * RNG: one stream per (seed, global pixel index y*W+x, block of 16 samples); a block's
 * samples draw from it in order.
 */
typedef struct fr_params {
  uint32_t width, height;
  uint32_t spp;       /* samples per pixel (save_image's `sample`) */
  uint32_t max_depth; /* tracer.rs:10 MAX_DEPTH (reference default 50); 1..64 */
  uint64_t seed;
  uint32_t strip_rows;  /* must be 8 */
  uint32_t shard_index; /* 0 <= shard_index < shard_count */
  uint32_t shard_count; /* >= 1 */
  uint32_t flags;       /* FR_FLAG_* */
} fr_params;

typedef struct fr_stats {
  uint64_t segments;   /* get_color calls (ray segments traced) */
  uint64_t hits;       /* segments whose closest-hit loop found an object */
  uint64_t samples;    /* paths started = pixels * spp */
  uint64_t prim_tests; /* segments * n_prims */
  double kernel_ms;    /* HIP-event time of the whole render on its stream (all kernels) */
  double total_ms;     /* host wall time of the call */
  double trace_ms;     /* HIP-event time of the trace kernel(s) alone, summed over launches */
  uint32_t trace_launches; /* trace kernel launches of the render (sample-block passes) */
  uint32_t occupancy;  /* resident trace-kernel workgroups per CU (the persistent grid's size / CUs) */
  uint64_t scatters;   /* successful scatters (tracer.rs:205: a segment continued by a new ray) */
} fr_stats;

typedef struct fr_scene fr_scene; /* opaque: host primitive list + per-device copies */
typedef struct fr_ctx fr_ctx;     /* opaque: one device, one stream, output buffers */
typedef struct fr_mctx fr_mctx;   /* opaque: one fr_ctx per device entry + a page-locked host frame */

/* ---- library ---- */
const char* fr_last_error(void);
int fr_abi_version(void);
int fr_device_count(int* count);

/* ---- scenes (host) ---- */
int fr_scene_create(const fr_prim* prims, uint32_t n, fr_scene** out);
int fr_scene_builtin(int which, uint32_t width, uint32_t height, fr_scene** out, fr_camera* cam_out);
int fr_scene_from_json(const char* json_text, size_t len, uint32_t width, uint32_t height,
                       fr_scene** out, fr_camera* cam_out);
void fr_scene_free(fr_scene* scene);
uint32_t fr_scene_count(const fr_scene* scene);
int fr_scene_get_prims(const fr_scene* scene, fr_prim* out, uint32_t n);
int fr_scene_translate(fr_scene* scene, uint32_t index, const float v[3]);
int fr_scene_rotate(fr_scene* scene, uint32_t index, const float v[3]);

/* ---- camera (host; tan/cos/sin are host-only) ---- */
int fr_camera_init(fr_camera* cam, uint32_t width, uint32_t height);
int fr_camera_look(fr_camera* cam, const float from[3], const float at[3], const float vup[3],
                   float vfov_deg, float aperture, uint32_t width, uint32_t height);
int fr_camera_orbit(fr_camera* cam, const float delta[3]);
int fr_camera_translate(fr_camera* cam, const float delta[3]);
int fr_update_delta(uint8_t keys, float delta_time, float delta_out[3]);

/* ---- GPU render context ---- */
int fr_ctx_create(int device, void* hip_stream /* NULL = own stream */, fr_ctx** out);
void fr_ctx_free(fr_ctx* ctx);
/* Enqueue one render of the shard described by params (async on the ctx stream).
   The scene is uploaded to the ctx device on first use and stays resident. */
int fr_ctx_render(fr_ctx* ctx, fr_scene* scene, const fr_camera* cam, const fr_params* params);
/* Wait for the last render; fill counters and kernel time. */
int fr_ctx_sync(fr_ctx* ctx, fr_stats* stats);
/* Copy the shard's rows of the last render into full-image host buffers
   (mean_rgb: W*H*3 f32, rgb8: W*H*3 u8; either may be NULL). Rows of other shards
   are left untouched. */
int fr_ctx_download(fr_ctx* ctx, float* mean_rgb, uint8_t* rgb8);
/* The same copies enqueued on the ctx's copy stream, after the last render; returns at
   once. The host buffers must stay valid until fr_ctx_wait (pinned memory from
   fr_host_alloc makes the copy asynchronous). The next fr_ctx_render's trace kernel does
   not wait for these copies; only its writes of the output buffers do, so one frame's
   gather overlaps the next frame's trace. */
int fr_ctx_download_async(fr_ctx* ctx, float* mean_rgb, uint8_t* rgb8);
/* Block until every render and download enqueued on the ctx has completed. */
int fr_ctx_wait(fr_ctx* ctx);
/* Device pointers of the last render's full-image output buffers. */
int fr_ctx_device_buffers(fr_ctx* ctx, float** d_mean_rgb, uint8_t** d_rgb8);
/* Launch log: enable != 0 starts a new log (previous entries dropped); every later render
   records HIP events around each trace-kernel launch (on the launch's stream) and around
   the whole render (trace + sum kernels). _read waits for the logged work and writes up
   to cap durations (ms) in order: which = 0 the trace launches, 1 the renders; which = 2
   / 3 the same entries as (start, end) pairs in ms from the first logged trace launch's
   start (2 values per entry, a timeline); *n = the entries logged. Lets a caller
   streaming K frames average all K of them and see the gaps between them. */
int fr_ctx_trace_log(fr_ctx* ctx, int enable);
int fr_ctx_trace_log_read(fr_ctx* ctx, int which, double* ms, uint32_t cap, uint32_t* n);
/* Everything a render of these parameters sets up before its first launch, without
   rendering: the scene's device copy, the output and sample buffers and, with
   FR_FLAG_SCENE_JIT, the scene-specialised kernel (compiled or loaded here, so the first
   timed frame does not pay for it). fr_ctx_jit_info then describes that kernel. */
int fr_ctx_prepare(fr_ctx* ctx, fr_scene* scene, const fr_camera* cam, const fr_params* params);
/* The last render's trace kernel: *used = 1 when it ran the scene-specialised kernel
   (FR_FLAG_SCENE_JIT), *ms = the time that render spent getting it (hiprtc compile, disk
   cache load or 0 when already loaded), *compiled = 1 when hiprtc ran. Any may be NULL. */
int fr_ctx_jit_info(fr_ctx* ctx, int* used, double* ms, int* compiled);
/* *state = FR_JIT_* of the last render. For FR_JIT_FAILED, fr_last_error() then holds the
   compiler's message. */
int fr_ctx_jit_state(fr_ctx* ctx, int* state);
/* Block until no scene-kernel compile is queued or running in this process. */
int fr_jit_wait(void);

/* ---- persistent multi-device context (tracer.rs:83-134 render_mt, one device per shard) ----
   Entry i of `devices` renders row shard i of n of every frame on its own fr_ctx (device
   entries may repeat). Contexts, device buffers and the page-locked host frame persist
   across renders; a frame no larger than the last allocates nothing. */
int fr_mctx_create(const int* devices, int n, fr_mctx** out);
void fr_mctx_free(fr_mctx* mctx);
int fr_mctx_count(const fr_mctx* mctx);
/* The i-th shard's context (owned by the mctx). */
int fr_mctx_ctx(fr_mctx* mctx, int i, fr_ctx** out);
/* Enqueue one frame: every shard's render, then its asynchronous gather into the host
   frame; returns at once. params' shard fields are ignored (shard i of n). The u8 image
   is gathered when params->flags has FR_FLAG_WRITE_U8. */
int fr_mctx_render(fr_mctx* mctx, fr_scene* scene, const fr_camera* cam, const fr_params* params);
/* Wait for every shard and gather; stats summed over shards (times: the slowest shard). */
int fr_mctx_sync(fr_mctx* mctx, fr_stats* stats);
/* The page-locked host frame (W*H*3 f32 means, W*H*3 u8), valid until the next render. */
int fr_mctx_frame(fr_mctx* mctx, const float** mean_rgb, const uint8_t** rgb8);
/* Wait, then copy the host frame into caller buffers (either may be NULL). */
int fr_mctx_download(fr_mctx* mctx, float* mean_rgb, uint8_t* rgb8);

/* Page-locked host memory (hipHostMalloc) for fr_ctx_download_async targets. */
int fr_host_alloc(size_t bytes, void** out);
void fr_host_free(void* p);

/* ---- synchronous conveniences ---- */
/* One shard on one device; writes the shard's rows into caller-owned host buffers. */
int fr_render_hip(fr_scene* scene, const fr_camera* cam, const fr_params* params, int device,
                  float* mean_rgb, uint8_t* rgb8, fr_stats* stats);
/* The whole image row-sharded across devices 0..n_gpus-1: an fr_mctx created, used once and freed. */
int fr_render_hip_multi(fr_scene* scene, const fr_camera* cam, const fr_params* params, int n_gpus,
                        float* mean_rgb, uint8_t* rgb8, fr_stats* stats);

/* ---- post-process effects (src/shaders/compute/<name>.comp.wgsl, rendering/post_processor.rs:101-129) ----
   Effect ids in shader_utils.rs:58-71 order. Images are RGBA8, row-major, W*H*4 bytes.
   Effects run in the given order, each reading the previous one's output, exactly like
   the reference's ping-pong between its two intermediate textures; `time` is the
   control uniform's values[0] (post_processor.rs:114, seconds), used by noise.
   Implementation-defined WGSL details are fixed in DESIGN.md §4.10. */
#define FR_FX_NONE 0
#define FR_FX_NOISE 1
#define FR_FX_PIXELATE 2
#define FR_FX_INVERT_COLOR 3
#define FR_FX_WAVE 4
#define FR_FX_INTERLACE 5
#define FR_FX_FLIP_AXIS 6
#define FR_FX_GRAYSCALE 7
#define FR_FX_STEP 8
#define FR_FX_WATERCOLOR 9
#define FR_FX_CHROMOSTEREOPSIS 10
#define FR_FX_ANAGLYPH 11
/* Host buffers in and out (synchronous). */
int fr_post_process(int device, const int* effects, uint32_t n_effects, float time, uint32_t width, uint32_t height,
                    const uint8_t* rgba_in, uint8_t* rgba_out);
/* Device buffers, in place on d_rgba (d_scratch: another W*H*4 bytes), async on `stream`. */
int fr_post_process_device(void* stream, const int* effects, uint32_t n_effects, float time, uint32_t width,
                           uint32_t height, uint8_t* d_rgba, uint8_t* d_scratch);
/* Device RGB8 (a render's u8 output) -> RGBA8 with alpha 255, async on `stream`. */
int fr_rgb_to_rgba_device(void* stream, const uint8_t* d_rgb, uint8_t* d_rgba, size_t pixels);

/* ---- diagnostics ---- */
/* Run the device f32/RNG primitives on n inputs (op codes in DESIGN.md §7); used by the
   parity tests to show the GPU arithmetic is bit-identical to the host's. */
int fr_selftest_ops(int device, int op, const float* a, const float* b, uint32_t n, float* out);
int fr_selftest_rng(int device, uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, uint32_t* out);
/* Compare the device's fast reciprocal (rcp + one Newton step) with the correctly rounded
   1.0f / x for every f32 bit pattern in [base, base + count): mismatches per exponent
   field in bad[256], first mismatching pattern in first[256] (0xFFFFFFFF = none). */
int fr_selftest_recip(int device, uint64_t base, uint64_t count, uint64_t* bad, uint32_t* first);
/* Compare div_rn (q0 = a y, one FMA residual correction, y = RN(1 / b)) with the IEEE
   division for every a in [1, 2) and the b = 1 + m 2^-23, m in [b_base, b_base + b_count):
   *bad = differing pairs, *first = least (m << 23 | a's mantissa) among them (~0 = none). */
int fr_selftest_div(int device, uint32_t b_base, uint32_t b_count, uint64_t* bad, uint64_t* first);
/* No device needed: hiprtc compiles the scene-specialised kernel for `arch` with n 64-B
   device records (16 u32 each, kind in word 15); targs = trace_kernel's 8 template
   arguments, or NULL for the headline's (all boxes, diffuse, depth <= 8, 8-B records);
   *code_bytes = the code object's size, *ms = the compile time. */
int fr_selftest_jit(const char* arch, const uint32_t* rec, uint32_t n, const int* targs, size_t* code_bytes,
                    double* ms);

#ifdef __cplusplus
}
#endif
#endif /* FORMA_RT_H */
