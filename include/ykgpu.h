/*
 * ykgpu.h — C-ABI of the MI355X (gfx950) renderer for the per-pixel sampling loop of
 * yaito3014/UECRayTracing.  Plain C: no C++ or torch types cross this boundary.
 *
 * WHAT THIS REPLACES (reference file:line, /root/reference):
 *   - the render loop   source.cpp:122-172  (for_each over (row,col) → transform_reduce over
 *                       samples → image[y*W+x] = to_color3b(sum, spp))  → ykgpu_render*()
 *   - yk::render<T>()   source.cpp:98-178   (returns image_t = std::array<color3b, W*H>,
 *                       row-major, row 0 = top, RGB interleaved, stride 3W: source.cpp:70-71,
 *                       224-226) → the caller-owned uint8_t[W*rows*3] output
 *   - the world tuple   hittable_list.hpp:18-30 (objects in tuple order; the order defines
 *                       rec.id, tie-breaking and scatter dispatch, hittable_list.hpp:32-73)
 *                       → yk_sphere[] in the same order
 *   - camera<T>         camera.hpp:14-38 (public origin / lower_left_corner / horizontal /
 *                       vertical) → yk_camera
 *   - constants         source.cpp:57-66 (image_width, samples_per_pixel, max_depth),
 *                       t_min raytracer.hpp:27, seed source.cpp:118-120,154-159
 *                       → yk_render_params
 * The reference has no plugin/FFI layer of its own: these are the entry points a
 * C++ caller (our drop-in `raytrace`, or the reference's own source.cpp through
 * include/yk/ykgpu_bridge.hpp) binds.  See INTEGRATION.md.
 *
 * Conventions: every function returns YK_OK (0) or a YK_ERR_* code; the message of the last
 * failure on the calling thread is ykgpu_last_error().  No exceptions cross the ABI.  A context
 * owns one device's memory and stream; calls on one context are synchronous unless named
 * *_async and are NOT reentrant per context (the reference calls render() once from main).
 */
#ifndef YKGPU_H
#define YKGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YKGPU_ABI_VERSION 11u

/* Material kinds.  LAMBERTIAN / METAL(fuzz == 0) are the reference's (material.hpp:37-69);
 * METAL with fuzz > 0 (reflected + fuzz * the reference's random_in_unit_sphere,
 * material.hpp:27-30) and DIELECTRIC are extensions needed by BASELINE configs 2-5.  The
 * reference has no code for them, but its integrator takes them: their images are pinned by
 * goldens rendered through the reference's ray_color / hittable_list / sphere / mt19937 with
 * these materials plugged in (oracle/ref_harness.cpp; only the scatter bodies are ours). */
enum { YK_MATERIAL_LAMBERTIAN = 0, YK_MATERIAL_METAL = 1, YK_MATERIAL_DIELECTRIC = 2 };

/* Arithmetic of the per-sample path (the T of yk::render<T>, source.cpp:98-99).
 * FP64 is render() as shipped (T = double), bit for bit.  FP32 is the same template with
 * T = float: geometry, camera, canonicals (generate_canonical<float> takes ONE 32-bit draw,
 * random.hpp:161-183) and math::sqrt in float; colours, attenuation and the per-pixel sum stay
 * double (raytracer<T, double>, lambertian<double>, source.cpp:100-111).  Sphere centres, radii
 * and camera vectors are the records' doubles rounded to float.  (As shipped, render<float>
 * does not compile — sphere's deduction guide rejects the double radius literals — so FP32 is
 * pinned against the reference's headers with the literals written as T(...): DESIGN.md §2.)
 * FP32 has its own BVH, whose boxes and per-ray cone carry the float sphere test's proven error
 * (DESIGN.md §4.1): its images equal the linear scan's bit for bit.
 * FP32 is a PARITY mode, not a speed mode: it reproduces render<float>'s images, and it is ~15%
 * SLOWER than FP64 on this chip (1920x1080x512: ~191 vs ~163 ms).  render<float>'s paths bounce
 * 7% more (its float sphere test), its tree needs the cone's extra plane read and wider boxes,
 * and the FP64 arithmetic the float path saves was not what bound the kernel.
 * Use FP64 (or xor128, the fast mode) for speed. */
enum { YK_PRECISION_FP64 = 0, YK_PRECISION_FP32 = 1 };

/* Per-sample engine (the Engine of source.cpp:155/159, seeded per sample as yk_render_params.
 * seed_mode says).  MT19937 = yk::mt19937 (random.hpp:148-151), render() as shipped.
 * XOR128 = the reference's other engine, yk::xor128 (random.hpp:18-41: Marsaglia's xorshift128,
 * x, y, z fixed, w = 88675123 ^ seed), swapped in for yk::mt19937: the fast mode.  Its state is
 * 4 words, so nothing needs the x_397 warm-up kernel.  (Consecutive counter seeds differ only in
 * w, so the first draws of neighbouring samples are correlated: that is the engine's, and the
 * image is the reference's with that engine, bit for bit.) */
enum { YK_RNG_MT19937 = 0, YK_RNG_XOR128 = 1 };

/* Per-sample seed of the mt19937 (yk_render_params.seed_mode).
 * COUNTER: seed0 + (y*W + x)*spp + s in uint32 arithmetic — the constexpr build
 *   (source.cpp:118-120,154-158); reproducible, the parity mode.
 * RANDOM_DEVICE: the runtime build seeds every sample from std::random_device (source.cpp:159).
 *   Here one 64-bit key per call (params.seed_key; 0 = draw it from std::random_device on the
 *   host, reported in yk_render_stats.seed_key) is hashed with the sample's linear index
 *   ((y*W + x)*spp + s, 64-bit): z = key + (idx+1)*0x9E3779B97F4A7C15, splitmix64 finaliser,
 *   seed = high 32 bits.  Independent seeds per sample like the reference's runtime build;
 *   reproducible when the key is given. */
enum { YK_SEED_COUNTER = 0, YK_SEED_RANDOM_DEVICE = 1 };

/* yk_render_params.flags */
enum {
  YK_FLAG_COUNT_WORK = 1u, /* count segments / sphere tests (ykgpu_get_stats)              */
  YK_FLAG_LINEAR_SCAN = 2u, /* closest hit by the reference's linear scan instead of the BVH
                              (same results; A/B and debugging)                              */
  YK_FLAG_ONE_LANE = 4u,    /* with COUNT_WORK, FP64 only (diagnostic): one lane per wave runs
                              paths, the other 63 idle.  The profiler's per-wave-instruction
                              counters (SQ_INSTS_VALU_FLOPS_FP64 ...) then read exactly the
                              instructions one lane executed: DESIGN.md §5 reconciliation   */
  YK_FLAG_TRACE_RAYS = 8u   /* internal to ykgpu_render_trace                                 */
};

enum {
  YK_OK = 0,
  YK_ERR_INVALID = 1,     /* bad argument (null pointer, zero size, row range outside image) */
  YK_ERR_DEVICE = 2,      /* HIP runtime failure / no device                                 */
  YK_ERR_NOMEM = 3,       /* device allocation failed                                        */
  YK_ERR_UNSUPPORTED = 4, /* a mode this build does not implement                            */
  YK_ERR_NO_SCENE = 5     /* render before ykgpu_set_scene                                   */
};

/* One sphere<T, M> of the world tuple (sphere.hpp:16-23), in tuple order. 80 bytes. */
typedef struct yk_sphere {
  double center[3];
  double radius;    /* may be negative (hollow dielectric shell, extension)              */
  double albedo[3]; /* lambertian / metal albedo (material.hpp:39,57)                    */
  double fuzz;      /* metal only; 0 = the reference's metal (no random draw)            */
  double ior;       /* dielectric only                                                    */
  uint32_t material;/* YK_MATERIAL_*                                                      */
  uint32_t reserved;
} yk_sphere;

/* camera<T> public members (camera.hpp:34-37) plus the thin-lens basis of the defocus
 * extension.  lens_radius == 0 gives exactly the reference's get_ray (camera.hpp:29-32). */
typedef struct yk_camera {
  double origin[3];
  double lower_left_corner[3];
  double horizontal[3];
  double vertical[3];
  double lens_u[3];
  double lens_v[3];
  double lens_radius;
} yk_camera;

typedef struct yk_render_params {
  uint32_t image_width;       /* W  (constants::image_width, source.cpp:60)            */
  uint32_t image_height;      /* H  (source.cpp:61-62: uint32(W / (16/9)))             */
  uint32_t samples_per_pixel; /* spp (source.cpp:63)                                   */
  uint32_t max_depth;         /* source.cpp:64                                          */
  uint32_t seed0;             /* constexpr_seed (source.cpp:118-120); 404 = "00:00:00"  */
  uint32_t row_begin;         /* rendered rows: row_begin + i*row_stride, i < row_count */
  uint32_t row_count;         /*   (a tile of the image; the whole image: 0, H, 1), or   */
  uint32_t row_stride;        /*   in bands of 2^row_band_log2 rows (below)             */
  uint32_t precision;         /* YK_PRECISION_*                                         */
  uint32_t rng;               /* YK_RNG_*                                               */
  uint32_t flags;             /* YK_FLAG_*                                              */
  uint32_t seed_mode;         /* YK_SEED_*                                              */
  double t_min;               /* 0.001 in the reference (raytracer.hpp:27)              */
  uint64_t seed_key;          /* YK_SEED_RANDOM_DEVICE only (0: draw one per call)      */
  /* Banded row sets (the N-GPU split): with B = 2^row_band_log2, tile row i is image row
   * row_begin + (i / B) * row_stride * B + i % B — bands of B consecutive rows, every
   * row_stride-th band (rank k of N: row_begin = k*B, row_stride = N).  0: single rows.
   * Whole bands keep a wave's pixels adjacent in the image (coherent rays); DESIGN.md §7. */
  uint32_t row_band_log2;
  /* Column sets (ABI 10; the N-GPU split of uecraytracing_amd/tiles.py): col_count == 0 renders
   * every column (col_begin, col_stride and col_band_log2 must then be 0).  Otherwise, with
   * C = 2^col_band_log2, tile column j is image column col_begin + (j / C) * col_stride * C + j % C
   * — bands of C consecutive columns, every col_stride-th band — and the tile is
   * row_count x col_count pixels.  Seeds and the camera use the image position (y, x), so any
   * row and column set renders the image's own pixels.  Bands of 8 columns over every row keep a
   * rank's 8x8 processing blocks 8x8 in the image (coherent rays). */
  uint32_t col_begin;
  uint32_t col_count;
  uint32_t col_stride;
  uint32_t col_band_log2;
  uint32_t reserved0;
} yk_render_params;

typedef struct yk_render_stats {
  double kernel_ms;        /* path-tracing kernel, summed over its launches (HIP events on
                              the render streams around each launch; consecutive launches
                              overlap, so this can exceed the call)                      */
  double resolve_ms;       /* ordered per-pixel sum + to_color3b kernel, summed           */
  double total_ms;         /* whole call: host wall clock for ykgpu_render / _sums (with
                              the copies), first to last event for ykgpu_render_async   */
  double warmup_ms;        /* MT seed-walk kernel, summed over its launches             */
  uint64_t samples;        /* primary samples rendered                                 */
  uint64_t segments;       /* ray_color calls that ran a closest-hit (flag COUNT_WORK) */
  uint64_t sphere_tests;   /* ray-sphere discriminant tests (flag COUNT_WORK)          */
  uint64_t sqrt_calls;     /* Newton square roots on hit candidates (flag COUNT_WORK)  */
  uint64_t mt_fallbacks;   /* samples that needed the full 624-word MT state           */
  uint64_t node_visits;    /* BVH inner nodes visited (flag COUNT_WORK)                */
  uint64_t linear_scans;   /* segments served by the exact linear scan (flag COUNT_WORK)*/
  uint64_t newton_calls;   /* math::sqrt evaluations (flag COUNT_WORK)                 */
  uint64_t newton_iters;   /* math::sqrt loop iterations (flag COUNT_WORK)             */
  uint64_t phase_cycles[8];/* diagnostic builds only (YK_ABLATE & 8): wave-cycles in refill,
                              sample start, traversal (interior nodes), candidates, shading,
                              path end, traversal (leaves), unused                        */
  uint64_t timeline[3];    /* diagnostic builds only: s_memrealtime (100 MHz) of the first wave start, of
                              the first refill that found no pixel left, of the last wave
                              exit (last launch of the call)                              */
  uint64_t diag[4];        /* diagnostic builds only: [0] leaf tests with disc >= 0       */
  uint64_t seed_key;       /* the key a YK_SEED_RANDOM_DEVICE render used (0 otherwise) */
  uint32_t launches;       /* path-tracing launches in the call                        */
  uint32_t grid_blocks;    /* persistent grid size                                     */
  double render_busy_ms;   /* union of the path-tracing launches' spans (wall time with at
                              least one launch running)                                 */
  uint64_t work[8];        /* flag COUNT_WORK (the flop and lane-op models):
                              FP64 only: [0] leaf tests with disc >= 0 (root bounds
                              computed), hits shaded as [1] lambertian, [2] metal, [3] of
                              them fuzzy, [4] dielectric; both precisions: [5] engine words
                              drawn by all samples, [6] of them by the seed-walk kernel
                              (the start's jitter and lens draws), [7] 624-word twists of
                              the full mt19937 state (samples past 227 words)            */
  uint64_t device_bytes;   /* device memory the context holds after the call: scene, BVHs,
                              processing order, start-record (xor128: colour) ring, running
                              sums, MT and attenuation scratch, the warm-ups' lens-retry rings,
                              output buffers.
                              Buffers follow the calls: grown when a call needs more, given
                              back when it needs less than half                            */
  uint64_t call_bytes;     /* device memory THIS call needed (the same items sized to it):
                              1920x1080x512 FP64 ~19.1 GB; the 8-GPU split's tile of 3840x2160x1024
                              (480 columns) ~10.5 GB; 1920x1080x4096 (config 5) ~71 GB      */
  double sclk_mhz;         /* the shader clock the render launches ran at: s_memtime over
                              s_memrealtime (100 MHz) of one wave per launch, averaged      */
  uint32_t launch_spp;     /* samples per pixel of the call's largest launch (ABI 11)        */
  uint32_t mem_shrinks;    /* times the launch size was halved because the device could not
                              hold the rings (free memory short: slower, not an error; at
                              launches of 2^24 sample slots the call fails with NOMEM)      */
} yk_render_stats;

typedef struct ykgpu_context ykgpu_context;

uint32_t ykgpu_abi_version(void);
const char* ykgpu_last_error(void);

int ykgpu_device_count(int* count);
int ykgpu_context_create(int device, ykgpu_context** out);
int ykgpu_context_destroy(ykgpu_context* ctx);

/* Uploads the world (tuple order) and the camera to HBM.  Replaces building `world` and `cam`
 * inside render() (source.cpp:100-112).  Synchronous: first waits for the device (a render
 * still running from ykgpu_render_async reads the previous scene), then builds the BVHs on the
 * host and copies them with the spheres. */
int ykgpu_set_scene(ykgpu_context* ctx, const yk_sphere* spheres, uint32_t count,
                    const yk_camera* camera);

/* The render loop (source.cpp:122-172) for the rows (and columns) named by params, synchronous,
 * into a caller-owned host buffer of row_count * Wt * 3 bytes laid out like image_t, where the
 * tile width Wt is col_count, or W when col_count == 0. */
int ykgpu_render(ykgpu_context* ctx, const yk_render_params* params, uint8_t* rgb_host);

/* Same, into device memory (row_count * Wt * 3 bytes on ctx's device), ordered on `stream`
 * (a hipStream_t; NULL = the context's own stream): the writes to rgb_device come after the work
 * already queued on `stream`, and the image is complete for the work queued on `stream` after
 * the call.  Internally the kernels run on the context's own streams (render launches at the
 * device's top stream priority, the seed walks and the reduces below it) joined to `stream` by
 * events.  A call enqueued while this context's previous call still runs, with the same ring
 * geometry, overlaps it: its seed walks and renders start without waiting for `stream` (they
 * read only the scene and the context's own buffers) and only its last reduce, which writes
 * rgb_device, waits for `stream`.  YKGPU_OVERLAP=0 in the environment restores full ordering
 * (every kernel of the call after the work queued on `stream` and after the whole previous
 * call).  Does not synchronise. */
int ykgpu_render_async(ykgpu_context* ctx, const yk_render_params* params, void* rgb_device,
                       void* stream);

/* Diagnostics: the per-pixel colour sum before to_color3b (source.cpp:137-167), 3 doubles per
 * pixel, row_count * Wt * 3 doubles, host buffer. */
int ykgpu_render_sums(ykgpu_context* ctx, const yk_render_params* params, double* sums_host);

/* Verbose level 3 (raytracer.hpp:21-25: ray_color prints every ray it is called with, the one
 * reaching depth 0 included).  Renders the rows of params (COUNT_WORK instance) and records, for
 * every sample (index (row_t*Wt + col_t)*spp + s over the tile), the first max_rays rays of its path
 * as 6 doubles each (origin xyz, direction xyz; FP32 rays are floats widened exactly) into
 * rays_host[(index*max_rays + k)*6 ...] and the number of ray_color calls into counts_host[index]
 * (which may exceed max_rays).  row_count * Wt * spp * max_rays * 48 bytes of device memory are
 * used for the call, so callers render large images in row bands. */
int ykgpu_render_trace(ykgpu_context* ctx, const yk_render_params* params, uint32_t max_rays,
                       double* rays_host, uint32_t* counts_host);

/* Diagnostics: the device's math::sqrt (math.hpp:10-19) -- the routine every length, root and
 * to_color3b in the render uses -- on n host doubles (in and out may alias).  The tests check it
 * against the reference's loop. */
int ykgpu_math_sqrt(ykgpu_context* ctx, const double* in, double* out, uint64_t n);

/* Same for the FP32 path's math::sqrt<float> (loop in float, s / 2.0 and the halving in
 * double then rounded, exactly as math.hpp:10-19 reads for T = float) on n host floats. */
int ykgpu_math_sqrt_f32(ykgpu_context* ctx, const float* in, float* out, uint64_t n);

/* Diagnostics: the renderer's vector / scalar division (the normalisations and normals of
 * sphere.hpp / vec3.hpp) on n host triples: out3[3i+k] = num3[3i+k] / den[i].  It must equal
 * IEEE division bit for bit; the tests check it. */
int ykgpu_math_div(ykgpu_context* ctx, const double* num3, const double* den, double* out3, uint64_t n);
/* Diagnostic: the FP32 kernel's vector / scalar division (ykf::divs_fast: the compiler's float
 * division without its special-case steps, the reciprocal shared by the three components) on n
 * (3 numerators, denominator) pairs: out3 must equal num3 / den in IEEE float, bit for bit. */
int ykgpu_math_div_f32(ykgpu_context* ctx, const float* num3, const float* den, float* out3, uint64_t n);

/* Statistics of the last render on this context. */
int ykgpu_get_stats(ykgpu_context* ctx, yk_render_stats* out);

/* ---- several devices in one process (BASELINE config 4: the image row-tiled across the 8 GPUs
 * of a node) -------------------------------------------------------------------------------
 * The reference calls render() once from main (source.cpp:221) on one thread; a group lets that
 * one call use k devices.  A group holds one context per entry of `devices` (an entry may repeat:
 * {0, 0, 0} runs three contexts on device 0, which the tests use on one-GPU machines).  Rows of
 * the params' row set are dealt cyclically — tile row t goes to entry t mod k, the same dealing
 * as the torch.distributed bench (uecraytracing_amd/tiles.py) — every entry renders its tile with
 * ykgpu_render_async on its own streams, so the devices run concurrently, and each tile is
 * copied from its device straight into its rows of the caller's image (a strided 2-D copy: the
 * caller's image is on the host, so no device-side gather is needed before it).  Every row is
 * independent (source.cpp:154-158), so the image equals one device's byte for byte.
 * Row sets in bands (row_band_log2 > 0) are not dealt: YK_ERR_UNSUPPORTED when k > 1.
 * Not reentrant per group, like a context. */
typedef struct ykgpu_group ykgpu_group;

int ykgpu_group_create(const int* devices, uint32_t n_devices, ykgpu_group** out);
int ykgpu_group_destroy(ykgpu_group* group);
/* Number of entries (contexts) of the group. */
int ykgpu_group_size(const ykgpu_group* group, uint32_t* n);
/* ykgpu_set_scene on every entry (each device holds the scene and its BVHs in its own HBM). */
int ykgpu_group_set_scene(ykgpu_group* group, const yk_sphere* spheres, uint32_t count,
                          const yk_camera* camera);
/* The render loop over every entry; synchronous; rgb_host as for ykgpu_render
 * (row_count * tile width * 3 bytes, the rows of params in order).  The entries share the
 * params' column set; the rows are dealt. */
int ykgpu_group_render(ykgpu_group* group, const yk_render_params* params, uint8_t* rgb_host);
/* Statistics of the last group render: index < n the entry's own (its tile), index -1 the whole
 * call: samples and work counters summed over the entries, launches summed, kernel_ms /
 * render_busy_ms / warmup_ms / resolve_ms the largest entry's, total_ms the call's host wall
 * clock (copies included). */
int ykgpu_group_get_stats(ykgpu_group* group, int index, yk_render_stats* out);

/* One call for the whole drop-in: a group over `devices`, the scene, the render, the group
 * released (scene upload and BVH builds are inside the call). */
int ykgpu_render_devices(const int* devices, uint32_t n_devices, const yk_sphere* spheres,
                         uint32_t count, const yk_camera* camera, const yk_render_params* params,
                         uint8_t* rgb_host);

/* ---- host-side scene helpers (no device needed) ---------------------------------------- */

/* camera<double>{} of camera.hpp:16-27 (16:9, viewport height 2, focal length 1, origin 0). */
int yk_camera_reference(yk_camera* out);

/* Positionable thin-lens camera (extension for configs 2-5). vfov in degrees. */
int yk_camera_look(yk_camera* out, const double lookfrom[3], const double lookat[3],
                   const double vup[3], double vfov_deg, double aspect, double aperture,
                   double focus_dist);

/* Named scenes: "ref4" (source.cpp:103-112), "lambert3", "mixed12", "rtiow5" (config 2),
 * "final" (RTIOW final scene, ~488 spheres, configs 3/4), "glass" (dielectric-heavy, config 5).
 * `seed` drives the random generators of "final" / "glass".  Writes up to `capacity` spheres,
 * the count to *count and the scene's camera to *camera (either may be NULL to query). */
int yk_scene_build(const char* name, uint32_t seed, yk_sphere* spheres, uint32_t capacity,
                   uint32_t* count, yk_camera* camera);

/* Scene files (an on-disk format for generated scenes).  Text: a "yk-scene 1"
 * header, one "camera" line (origin, lower_left_corner, horizontal, vertical, lens_u, lens_v,
 * lens_radius) and one "sphere <lambertian|metal|dielectric> cx cy cz radius r g b fuzz ior"
 * line per sphere in tuple order; numbers as %.17g, so every double round-trips exactly.
 * yk_scene_read follows yk_scene_build's capacity/count/camera convention. */
int yk_scene_write(const char* path, const yk_sphere* spheres, uint32_t count, const yk_camera* camera);
int yk_scene_read(const char* path, yk_sphere* spheres, uint32_t capacity, uint32_t* count, yk_camera* camera);

/* Image height of the reference for a width: uint32(W / (16.0/9.0)) (source.cpp:61-62). */
uint32_t yk_image_height_for(uint32_t width);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* YKGPU_H */
