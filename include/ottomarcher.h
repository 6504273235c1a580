/*
 * ottomarcher.h — C-ABI of the MI355X-native path-tracing hot path
 * (drop-in for octaviogarcia/RaytracingOneWeekend's per-pixel ray_color path).
 *
 * Every entry point is extern "C", takes plain pointers/sizes, never unwinds,
 * and returns om_status (0 = OK, negative = error; om_last_error() explains).
 * No torch or HIP types appear in the signatures.
 *
 * Reference interfaces replaced (file:line under /root/reference/src/):
 *   om_world_*            HittableList::new / += &T / clear         hits.rs:71-110, 370-371
 *   om_world_add_sphere   Sphere::new                               traced.rs:22-25
 *   om_world_add_sphere_radius  Sphere::new_with_radius             traced.rs:26-31
 *   om_world_add_cube     Cube::new                                 traced.rs:238-240
 *   om_world_add_cube_length    Cube::new_with_length               traced.rs:242-246
 *   om_world_add_triangle / _parallelogram  Barycentric::new3points traced.rs:148-154
 *   om_world_add_triangle_basis / _parallelogram_basis  Barycentric::new  traced.rs:135-147
 *   om_world_add_plane    InfinitePlane::new                        traced.rs:86-88
 *   om_world_add_marched_sphere / _box   struct literals            marched.rs:50-54, 79-83
 *   om_world_add_marched_torus  MarchedTorus::new                   marched.rs:116-130
 *   om_world_add_marched_sdf    HittableList += Arc<dyn Marched>    hits.rs:96-100, marched.rs:7-41
 *   om_world_random_scene / om_world_basic_scene  front-end builders  main.rs:37-110
 *   om_material_*         Material::new_*                           materials.rs:27-38
 *   om_camera_new         Camera::new                               camera.rs:38-59
 *   om_upload_world       HittableList::freeze -> FrozenHittableList  hits.rs:87-89, 116-185
 *   om_render / om_render_device   render_thread::render (all threads of main.rs:200-214)
 *                                                                   render_thread.rs:145-202
 *   om_pixel_stats        Pixel/Stats                               render_thread.rs:9-51
 *   om_shard_* / om_comm_* / om_multi_*  the pixel deal to num_cpus-1 render threads
 *                         (2730-pixel chunks round-robin) and their shared framebuffer,
 *                         re-designed as 8x8-tile shards over GPUs + RCCL gather
 *                                                                   main.rs:170-214
 */
#ifndef OTTOMARCHER_H
#define OTTOMARCHER_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OM_ABI_VERSION 2   /* 2: om-rng v2 path stream */

typedef int32_t om_status;
#define OM_OK 0
#define OM_ERR_INVALID (-1)      /* bad argument / null pointer / size */
#define OM_ERR_DEVICE (-2)       /* HIP runtime error */
#define OM_ERR_STATE (-3)        /* call order (e.g. render before upload) */
#define OM_ERR_UNSUPPORTED (-4)  /* feature not representable on the device */
#define OM_ERR_NOMEM (-5)

/* materials.rs:12-24 — 24 bytes, same field meaning as the Rust struct. */
enum { OM_LAMBERTIAN = 0, OM_METAL = 1, OM_DIELECTRIC = 2 };
typedef struct om_material {
    float albedo[3]; /* Lambertian, Metal */
    float fuzz;      /* Metal */
    float ior;       /* Dielectric */
    int32_t type;    /* OM_LAMBERTIAN / OM_METAL / OM_DIELECTRIC */
} om_material;

/* camera.rs:10-29 (all derived fields, as Camera::new computes them). */
typedef struct om_camera {
    float origin[3], horizontal[3], vertical[3], lower_left_corner[3];
    float u_of_plane[3], v_of_plane[3], w_of_plane[3];
    float lens_radius, aspect_ratio, focus_dist, viewport_width, viewport_height;
} om_camera;

/* Per-pixel accumulator = Stats (render_thread.rs:9-17), 40 bytes.
 * obj ids are global type-order primitive index + 1 (0 = sky), replacing the
 * memory address of utils.rs:110; bloom uses them unchanged (utils.rs:94-107). */
typedef struct om_pixel_stats {
    uint64_t bloom;     /* BloomFilter.state */
    float sum[3];       /* Stats.sum */
    uint32_t n;         /* Stats.n (samples taken) */
    float avg_depth;    /* Stats.avg_depth */
    uint32_t bad_avgs;  /* Stats.bad_avgs */
    uint8_t color[3];   /* Stats.color (gamma-quantised mean) */
    uint8_t flags;      /* bit0: done (bad_avgs >= 5, adaptive retirement) */
    uint32_t reserved;
} om_pixel_stats;

/* One render call = samples [sample_begin, sample_begin+sample_count) of every
 * (live) pixel, accumulated into the caller's om_pixel_stats in sample order.
 * spp_total sizes the jitter table (render_thread.rs:164-174); a pixel's sample
 * index is its Stats.n, exactly as jitters[pixel.stats.n] (render_thread.rs:188).
 * As in the reference: spp_total or sample_count 0 takes no sample (the Stats are left
 * as they are); width or height 1 divides by W-1 = 0 (render_thread.rs:190-191) and
 * renders the resulting non-finite rays; width or height 0 is OM_ERR_INVALID. */
typedef struct om_render_params {
    uint32_t width, height;     /* image_width / image_height */
    uint32_t spp_total;         /* samples_per_pixel of the whole frame */
    uint32_t sample_begin;      /* informative: n of the first sample of this call */
    uint32_t sample_count;      /* samples per pixel in this call */
    uint32_t max_depth;         /* max_depth (main.rs:146) */
    float tmin, tmax;           /* 0.001 / 100.0 (main.rs:205-206) */
    uint32_t march_steps;       /* max march iterations (hits.rs:292 hard-codes 1024) */
    uint32_t adaptive;          /* 1 = retire pixels like Stats::add/ThreadPixels (render_thread.rs:31-38,97-101) */
    uint64_t seed;              /* om-rng v2 path-stream seed (replaces thread_rng, utils.rs:25) */
} om_render_params;

/* Kernel choices (all produce bit-identical om_pixel_stats). */
enum {
    OM_KERNEL_AUTO = 0,        /* fastest available for the uploaded world */
    OM_KERNEL_BRUTE = 1,       /* reference-order brute force, every primitive tested */
    OM_KERNEL_CULLED = 2,      /* brute force + conservative bounding-sphere pre-test */
    OM_KERNEL_BVH = 3,         /* stack-based BVH traversal (global memory) with the brute-force tie rule */
    OM_KERNEL_SBVH = 4,        /* stackless skip-pointer BVH, staged in LDS when it fits */
    OM_KERNEL_BVH2 = 5,        /* compressed BVH2 + LDS lane stack (AUTO, both pipelines): f32 nodes in LDS,
                                  or, for a tree over the LDS budget, half-precision nodes through L2
                                  behind a breadth-first LDS prefix */
    OM_KERNEL_BVH4 = 6         /* 4-wide BVH collapsed from the BVH2, sorted near-first, LDS lane stack:
                                  f32 nodes in LDS, or half-precision nodes through L2 for a tree over the
                                  LDS budget (the megakernel runs OM_KERNEL_BVH2 for it) */
};

/* Work counters of the last render call (device atomics, wave-aggregated). */
typedef struct om_counters {
    uint64_t samples;           /* samples taken */
    uint64_t segments;          /* closest-hit queries (ray segments) */
    uint64_t prim_tests;        /* exact primitive tests executed */
    uint64_t pre_tests;         /* culling tests executed (bounding spheres / BVH boxes) */
    uint64_t march_steps;       /* sphere-tracing iterations */
    uint64_t credited;          /* progress credit as samples_atom (render_thread.rs:196-198) */
} om_counters;

typedef struct om_world om_world;   /* HittableList (host) */
typedef struct om_ctx om_ctx;       /* one device + stream + frozen world */

int32_t om_abi_version(void);
/* Source hash the library was built from (16 hex digits; raytracingoneweekend_amd/build_id.py
 * over csrc/ and include/): lets a host check that the loaded binary matches its sources. */
const char* om_build_id(void);

/* ---- materials (materials.rs:27-38) ---- */
om_material om_material_lambertian(float r, float g, float b);
om_material om_material_metal(float r, float g, float b);
om_material om_material_metal_fuzz(float r, float g, float b, float fuzz);
om_material om_material_dielectric(float ior);

/* ---- Mat4x4 helpers (f32, reference op order) so front-ends compose the
 * m4x4!(TR/RX/RY/RZ/SC) transforms of main.rs with identical bits.
 * Row-major out[16] = Mat4x4.e[row].e[col]. ---- */
om_status om_mat4_identity(float out[16]);                                            /* mat4x4.rs:16 */
om_status om_mat4_translate(const float v[3], float out[16]);                         /* mat4x4.rs:88-93 */
om_status om_mat4_scale(const float v[3], float out[16]);                             /* mat4x4.rs:94-99 */
om_status om_mat4_rotate(int32_t axis /*0=x,1=y,2=z*/, float angle, float out[16]);  /* mat4x4.rs:100-123 */
om_status om_mat4_mul(const float a[16], const float b[16], float out[16]);          /* a ^ b: dot_mat mat4x4.rs:66-72,167-178 */
om_status om_mat4_fast_homogenous_inverse(const float m[16], float out[16]);        /* mat4x4.rs:59-64 */

/* ---- camera (camera.rs:38-59) ---- */
om_status om_camera_new(const float lookfrom[3], const float lookat[3], const float vup[3], float vfov_deg,
                        float aspect_ratio, float aperture, float focus_dist, om_camera* out);

/* ---- world (HittableList) ---- */
om_status om_world_create(om_world** out);
void om_world_destroy(om_world* w);
om_status om_world_clear(om_world* w);
/* local_to_world: row-major 4x4 (Mat4x4.e[row].e[col]) */
om_status om_world_add_sphere(om_world* w, const float local_to_world[16], const om_material* m);
om_status om_world_add_sphere_radius(om_world* w, const float center[3], float radius, const om_material* m);
om_status om_world_add_cube(om_world* w, const float local_to_world[16], const om_material* m);
om_status om_world_add_cube_length(om_world* w, const float center[3], float length, const om_material* m);
om_status om_world_add_triangle(om_world* w, const float origin[3], const float upoint[3], const float vpoint[3], const om_material* m);
om_status om_world_add_parallelogram(om_world* w, const float origin[3], const float upoint[3], const float vpoint[3], const om_material* m);
om_status om_world_add_triangle_basis(om_world* w, const float origin[3], const float u[3], const float v[3], float u_length, float v_length, const om_material* m);
om_status om_world_add_parallelogram_basis(om_world* w, const float origin[3], const float u[3], const float v[3], float u_length, float v_length, const om_material* m);
om_status om_world_add_plane(om_world* w, const float center[3], const float normal[3], const om_material* m);
om_status om_world_add_marched_sphere(om_world* w, const float center[3], float radius, const om_material* m);
om_status om_world_add_marched_box(om_world* w, const float center[3], const float sizes[3], const om_material* m);
om_status om_world_add_marched_torus(om_world* w, const float local_to_world[16], const float sizes[3], const om_material* m);
/* A user marched object: the GPU form of `HittableList += Arc<dyn Marched>` (hits.rs:96-100), which
 * the reference's march loop visits after the typed marched objects (hits.rs:312-319, 350-356).
 * A Rust `impl Marched` cannot run on the device, so its local_sdf is given as a postfix program
 * over a float stack (at most OM_SDF_MAX_OPS ops, stack depth <= OM_SDF_MAX_STACK, exactly one
 * value left), evaluated at the local point p:
 *   OM_SDF_SPHERE    a = cx cy cz r          push |p - c| - r
 *   OM_SDF_BOX       a = cx cy cz sx sy sz   q = |p - c| - s: push |max(q, 0)| + min(max(q.x, q.y, q.z), 0)
 *   OM_SDF_TORUS     a = cx cy cz R r        q = p - c: push |(|(q.x, q.z, 0)| - R, q.y, 0)| - r
 *   OM_SDF_UNION / _INTERSECT / _SUBTRACT    b = pop, a = pop: push min(a, b) / max(a, b) / max(a, -b)
 *   OM_SDF_ROUND     a = r                   top - r
 * (the formulas and op order of marched.rs:56-58, 86-89, 133-138; |v| = Vec3::length).  The object's
 * transform is MarchedTorus's (marched.rs:116-130, 139-151): local_to_world decomposed into TR and S,
 * to_local(p) = W2L_TR . (p * w2l_s), sdf = local_sdf * min(l2w_s.xyz), and the normal is the
 * trait's default get_outward_normal (central differences, marched.rs:19-44).  A program
 * [OM_SDF_TORUS 0 0 0 R r] is bit for bit a MarchedTorus with sizes (R, r).  Invalid programs
 * (unknown op, stack underflow or overflow, not one value left, non-finite parameters) are
 * OM_ERR_INVALID. */
enum { OM_SDF_SPHERE = 1, OM_SDF_BOX = 2, OM_SDF_TORUS = 3, OM_SDF_UNION = 4, OM_SDF_INTERSECT = 5,
       OM_SDF_SUBTRACT = 6, OM_SDF_ROUND = 7 };
#define OM_SDF_MAX_OPS 64
#define OM_SDF_MAX_STACK 8
typedef struct om_sdf_op {
    int32_t op;       /* OM_SDF_* */
    float a[7];       /* parameters (unused ones ignored) */
} om_sdf_op;
om_status om_world_add_marched_sdf(om_world* w, const float local_to_world[16], const om_sdf_op* ops, uint32_t n_ops,
                                   const om_material* m);
/* number of user marched objects (they follow the eight types of om_world_counts in the
 * global index order, so their obj ids come last) */
om_status om_world_marched_sdf_count(const om_world* w, uint32_t* n);
/* counts[8] in type order: spheres, cubes, triangles, infinite_planes, parallelograms,
 * marched_spheres, marched_boxes, marched_torus (hits.rs:370-371) */
om_status om_world_counts(const om_world* w, uint32_t counts[8]);
/* Frozen per-primitive data, for cross-checks (layouts in DESIGN.md §4):
 * kind 0 sphere / 1 cube -> 32 floats (l2w, w2l); kind 2 triangle / 4 parallelogram -> 29 floats;
 * kind 7 torus -> 43 floats. */
om_status om_world_export(const om_world* w, int32_t kind, uint32_t index, float* out, uint32_t out_floats);

/* Front-end scene builders (main.rs:37-110) driven by om-rng's SplitMix64 from `seed`.
 * flags bit0: include the marched torus block (main.rs:73-81);
 * flags bit1: omit the parallelogram/triangle/cube blocks.
 * grid_half: 11 = random_scene's -11..11 grid; 50 = the 10k-sphere variant. */
om_status om_world_random_scene(om_world* w, uint64_t seed, uint32_t flags, int32_t grid_half);
om_status om_world_basic_scene(om_world* w);       /* main.rs:103-110 */
om_status om_world_marched_scene(om_world* w);     /* SDF scene for config C2 */

/* ---- device context ---- */
om_status om_create(int32_t device, om_ctx** out);
void om_destroy(om_ctx* ctx);
const char* om_last_error(const om_ctx* ctx);      /* ctx may be NULL: last global error */
/* freeze(): copies the world to device memory (the caller may destroy `w` afterwards).
 * Arc<dyn Traced/Marched> user types (hits.rs:91-100) cannot cross the C-ABI. */
om_status om_upload_world(om_ctx* ctx, const om_world* w);
om_status om_set_kernel(om_ctx* ctx, int32_t kernel);
/* Host framebuffer path: `stats` is caller-owned W*H, read and written in place
 * (like PixelsBox, main.rs:192).  Includes the PCIe copies: 40 B per pixel each way per
 * call, at DMA speed when the buffer is page-locked (om_host_register), else staged by the
 * runtime.  Prefer few calls per frame (om_progress reports progress inside a call). */
om_status om_render(om_ctx* ctx, const om_camera* cam, const om_render_params* p, om_pixel_stats* stats,
                    om_counters* counters /* optional */);
/* Page-lock a caller-owned host buffer (e.g. the framebuffer) so om_render's copies run as
 * DMA at full PCIe speed; the buffer must stay allocated until om_host_unregister. */
om_status om_host_register(void* p, size_t bytes);
om_status om_host_unregister(void* p);
/* Device framebuffer path: `dev_stats` is device memory (W*H om_pixel_stats) on ctx's
 * device; `stream` is a hipStream_t (NULL = ctx's own stream).  Asynchronous:
 * returns after enqueue; the caller synchronises the stream.  Calls queued back to back
 * on one stream may differ in seed, spp_total or pixels (each (seed, spp_total) has its own
 * immutable jitter table).  A ctx's path queues are shared by its calls: drive one ctx
 * from one stream at a time (use one ctx per concurrent stream). */
om_status om_render_device(om_ctx* ctx, const om_camera* cam, const om_render_params* p, om_pixel_stats* dev_stats,
                           void* stream);
/* Renders only the pixels listed in `dev_pixels` (device array of row-major pixel
 * indices) — the tile-shard entry point for multi-GPU frames. */
om_status om_render_device_pixels(om_ctx* ctx, const om_camera* cam, const om_render_params* p, om_pixel_stats* dev_stats,
                                  const uint32_t* dev_pixels, uint32_t n_pixels, void* stream);
/* Work counters, accumulated over every om_render_device* launch since the last
 * om_reset_counters (om_render resets them itself).  om_get_counters synchronises
 * ctx's stream and the stream of the last launch. */
om_status om_get_counters(om_ctx* ctx, om_counters* out);
om_status om_reset_counters(om_ctx* ctx, void* stream);
/* Live progress: the reference's samples_atom (render_thread.rs:196-198), which main.rs's
 * log thread and display poll while the render threads run (main.rs:151-168, 371-377).
 * om_progress returns a host word the library keeps pinned; every later render call on ctx
 * adds its credited samples to it (each sample taken, plus a retiring pixel's untaken ones in
 * adaptive calls).  The wavefront pipeline adds each batch as it is accumulated, so the word
 * advances while a call runs; the megakernel adds the whole call when its one launch ends.
 * Any host thread may read it without synchronising; it only grows.  After the call's stream
 * is synchronised it has grown by the call's credited samples; with counting on (the
 * default, om_set_counting) that is exactly the call's om_counters.credited (with counting
 * off the counters stay 0 and only this word advances).  om_reset_progress zeroes it
 * (synchronises the device).  NULL on error. */
const volatile uint64_t* om_progress(om_ctx* ctx);
om_status om_reset_progress(om_ctx* ctx);
/* Work counting on (default) / off.  Off selects kernel builds with the counters
 * compiled out (fewer registers); results are bit-identical either way. */
om_status om_set_counting(om_ctx* ctx, int32_t enable);
/* Execution pipeline (all bit-identical):
 *   OM_PIPELINE_WAVEFRONT  per bounce one {trace -> shade -> compact} launch over SoA path
 *                          queues in HBM (bounce 0 generates the camera rays; marched worlds:
 *                          a lane-refilling march launch, then shade), then one persistent
 *                          tail launch, then accumulate
 *   OM_PIPELINE_MEGAKERNEL one persistent-path kernel per call
 *   OM_PIPELINE_AUTO       (default) the faster one measured: the wavefront, for every world,
 *                          fixed-spp and adaptive calls and any om_set_streams */
enum { OM_PIPELINE_MEGAKERNEL = 0, OM_PIPELINE_WAVEFRONT = 1, OM_PIPELINE_AUTO = 2 };
om_status om_set_pipeline(om_ctx* ctx, int32_t pipeline);
/* Wavefront pipeline: bounces >= `bounce` are finished by one persistent tail launch
 * (lanes run whole remaining paths); 0 = default (16; 1 for worlds with marched
 * primitives, 10 when the BVH2 is too big for LDS, 8 for adaptive calls, 24 for batches
 * above 2^25 paths),
 * >= max_depth = no tail.  A pure
 * scheduling knob: results are bit-identical for every value. */
om_status om_set_tail_bounce(om_ctx* ctx, uint32_t bounce);

/* Wavefront: batches in flight (1..4; default 2).  A fixed-spp call's samples are split into
 * batches of at most 1/streams of the call, dealt round-robin to `streams` HIP streams (the
 * call's stream plus context-owned side streams), each with its own queue set; one batch's
 * latency-bound phases (launch drains, late bounces, tail) then run beside the other's full
 * ones.  An adaptive call deals the listed pixels to the streams instead (64-entry chunks), and
 * each stream renders its live pixels in batches planned on the device (om_set_adaptive_batches).
 * Accumulation stays in sample order and the call ends joined on its stream, so results are
 * bit-identical for every value.  1 = one batch after another. */
om_status om_set_streams(om_ctx* ctx, uint32_t streams);

/* Wavefront adaptive calls (the GPU form of ThreadPixels, render_thread.rs:68-102): each stream
 * keeps a list of its live pixels, compacted by every batch's accumulate, and runs at most
 * `batches` batches per call (0 = default 3; more when a batch would exceed 2^26 paths).  A
 * batch renders b samples of every listed pixel: enough for 2^paths_log2 paths (0 = default 22),
 * at least an even share of the call's remaining samples over the batches left, at most the
 * remainder; samples past a pixel's retirement inside a batch are dropped in sample order.  A
 * pure scheduling knob: results are bit-identical for every value.  batches <= 64: the host never
 * reads the live count back, so every planned batch is launched even once the plan leaves it no
 * pixel (a bounce chain plus an accumulate per stream, ~5 us per launch that returns at once). */
om_status om_set_adaptive_batches(om_ctx* ctx, uint32_t batches, uint32_t paths_log2);

/* Primary rays (wavefront, BVH2): bounce 0 can test, per 8x8 pixel tile, only the leaf
 * records a conservative lens-aware frustum of the tile reaches, instead of traversing
 * the BVH (the conservative form of the reference's camera hash, camera_hash.rs;
 * DESIGN.md §5.10).  Results are bit-identical either way.
 *   OM_PRIMARY_LISTS_AUTO (default) when a pixel sees <= 12 candidates on average */
enum { OM_PRIMARY_LISTS_OFF = 0, OM_PRIMARY_LISTS_AUTO = 1, OM_PRIMARY_LISTS_ON = 2 };
om_status om_set_primary_lists(om_ctx* ctx, int32_t mode);

/* Per-kernel-class device time.  om_set_timing mode 1: every launch is bracketed by a HIP
 * event pair on its stream, and each wavefront call as a whole; mode 2: only each wavefront
 * call (OM_KT_BOUNCE_SPAN: two events per call on the call's stream, counting the call's
 * bounce-family launches; with concurrent batches, launches overlap inside it) — bench.py's
 * roofline uses mode 2 in the timed region and mode 1 in an untimed rerun.
 * om_get_kernel_times synchronises the recorded events, returns the totals since the
 * previous read (or since om_set_timing) and clears them.  Classes: */
enum {
    OM_KT_BOUNCE0 = 0,     /* wavefront bounce 0: camera rays + trace + shade + compact   */
    OM_KT_BOUNCE = 1,      /* wavefront bounce b >= 1: trace + shade + compact              */
    OM_KT_TAIL = 2,        /* wavefront persistent tail (bounces >= om_set_tail_bounce)   */
    OM_KT_ACCUMULATE = 3,  /* wavefront Stats::add in sample order                          */
    OM_KT_MEGAKERNEL = 4,  /* megakernel pipeline: one launch per render call              */
    OM_KT_BOUNCE_SPAN = 5, /* one wavefront call: snapshot .. last accumulate (all batches)   */
    OM_KT_N = 6
};
typedef struct om_kernel_times {
    uint64_t launches[OM_KT_N];
    double ms[OM_KT_N];
} om_kernel_times;
om_status om_set_timing(om_ctx* ctx, int32_t mode);
om_status om_get_kernel_times(om_ctx* ctx, om_kernel_times* out);

/* ---- display views (draw_to_sdl, main.rs:345-484) ----
 * RGB24 (row-major, W*H*3 bytes) view of the per-pixel accumulators, mode numbers as
 * the reference's keys 0-6 (main.rs:360-367).  The blurs are apply_box_filter::<0/1/2>
 * (main.rs:219-343); like the reference's persistent sdlpixels buffer, pixels that
 * filter does not visit (frames with W or H == 2) keep the caller's previous bytes.
 * Blur views need W, H >= 2. */
enum {
    OM_VIEW_NORMAL = 0,        /* Stats.color                                     */
    OM_VIEW_SAMPLES = 1,       /* n / max n, gamma-quantised                      */
    OM_VIEW_SAMPLE_BLUR = 2,   /* 3x3 blur weighted by n                          */
    OM_VIEW_DEPTH = 3,         /* avg_depth / max finite avg_depth; sky = green  */
    OM_VIEW_DEPTH_BLUR = 4,    /* 3x3 blur weighted by 1/(1+|depth difference|)   */
    OM_VIEW_IDS = 5,           /* u64_to_color(scramble(bloom)) (utils.rs:46-70)  */
    OM_VIEW_ID_BLUR = 6        /* 3x3 blur over pixels whose bloom contains ours  */
};
/* Device buffers on ctx's device; asynchronous on `stream` (NULL = ctx's stream). */
om_status om_display_device(om_ctx* ctx, const om_pixel_stats* dev_stats, uint32_t width, uint32_t height, int32_t view,
                            uint8_t* dev_rgb, void* stream);
/* Host buffers (copies both ways, synchronous); rgb is read-modify-write. */
om_status om_display(om_ctx* ctx, const om_pixel_stats* stats, uint32_t width, uint32_t height, int32_t view, uint8_t* rgb);
/* Image writers for headless runs (the F12 BMP save, main.rs:473-476): 24-bit BMP
 * (bottom-up BGR rows padded to 4 bytes, 54-byte header) and binary PPM (P6). */
om_status om_write_bmp(const char* path, const uint8_t* rgb, uint32_t width, uint32_t height);
om_status om_write_ppm(const char* path, const uint8_t* rgb, uint32_t width, uint32_t height);

/* ---- multi-GPU frames (main.rs:170-214) ----
 * The reference deals 2730-pixel chunks round-robin to num_cpus-1 threads that share one
 * framebuffer.  Here 8x8 pixel tiles (row-major tile order) are dealt round-robin to
 * `nranks` GPUs: rank r owns tiles t with t % nranks == r, each tile's in-frame pixels in
 * lane order (8*y + x).  A rank renders its tiles into a compact shard (om_pixel_stats in
 * list order); the frame is assembled on rank 0.  om-rng is keyed by (pixel, sample), so a
 * sharded frame is bit-identical to a single-device one for every nranks. */

/* Pixels of the largest shard: the size of every shard buffer. */
uint32_t om_shard_capacity(uint32_t width, uint32_t height, uint32_t nranks);
/* Row-major pixel indices of rank's tiles (host memory, `capacity` entries available). */
om_status om_shard_pixels(uint32_t width, uint32_t height, uint32_t rank, uint32_t nranks, uint32_t* out,
                          uint32_t capacity, uint32_t* n_out);
/* Host assembly of a frame from all ranks' host shards (shards[r] in rank order). */
om_status om_shard_assemble_host(uint32_t width, uint32_t height, uint32_t nranks,
                                 const om_pixel_stats* const* shards, om_pixel_stats* frame);

/* One rank per process (or per host thread), RCCL over xGMI.  Rank 0 makes the id with
 * om_comm_unique_id and hands its OM_COMM_ID_BYTES to the other ranks by any host means
 * (a socket, a file, an MPI broadcast); every rank then calls om_comm_init_rank, which
 * blocks until all ranks joined.  A comm is bound to ctx's device and is driven from one
 * host thread. */
#define OM_COMM_ID_BYTES 128
/* The RCCL library serving om_comm_* / om_multi_* in this process: its file (from the dynamic
 * loader, NUL-terminated into path[path_bytes]) and its version (ncclGetVersion).  The library
 * links /opt/rocm/lib's RCCL; a process that loaded another one first (PyTorch-ROCm ships its
 * own, with its own HIP runtime) binds to that one by soname. */
om_status om_rccl_library(char* path, uint32_t path_bytes, int32_t* version);
typedef struct om_comm om_comm;
om_status om_comm_unique_id(uint8_t id[OM_COMM_ID_BYTES]);
om_status om_comm_init_rank(om_ctx* ctx, uint32_t nranks, uint32_t rank, const uint8_t id[OM_COMM_ID_BYTES],
                            om_comm** out);
void om_comm_destroy(om_comm* comm);
/* What RCCL itself reports for this communicator: its rank count (ncclCommCount) and this
 * rank (ncclCommUserRank).  A host checks them against its own world size before timing. */
om_status om_comm_info(const om_comm* comm, int32_t* nranks, int32_t* rank);
/* Renders this rank's tiles into dev_shard (om_shard_capacity entries of device memory on
 * the comm's device, list order), like om_render_device on those pixels.  Asynchronous. */
om_status om_render_shard(om_comm* comm, const om_camera* cam, const om_render_params* p, om_pixel_stats* dev_shard,
                          void* stream);
/* Every rank calls it: each rank's shard goes to rank 0 (one RCCL group of send/recv; rank 0
 * receives its own through RCCL too) and rank 0 scatters them into dev_frame (W*H, device
 * memory; ignored on other ranks).  Asynchronous on `stream` (NULL = the ctx's stream). */
om_status om_gather_frame(om_comm* comm, const om_pixel_stats* dev_shard, uint32_t width, uint32_t height,
                          om_pixel_stats* dev_frame, void* stream);
/* The reverse (every rank calls it): rank 0 cuts dev_frame into shards and sends each to
 * its rank, which receives it into dev_shard: resumes a frame rendered elsewhere. */
om_status om_scatter_frame(om_comm* comm, const om_pixel_stats* dev_frame, uint32_t width, uint32_t height,
                           om_pixel_stats* dev_shard, void* stream);

/* One process driving several GPUs (the C++ front-end's model): a ctx per entry of
 * `devices` plus a communicator between them.  Distinct devices: RCCL (ncclCommInitAll),
 * transport OM_TRANSPORT_RCCL.  Repeated devices (several logical ranks on one GPU, which
 * RCCL refuses): device copies, OM_TRANSPORT_LOCAL.  Results are bit-identical either way. */
enum { OM_TRANSPORT_RCCL = 0, OM_TRANSPORT_LOCAL = 1 };
typedef struct om_multi om_multi;
om_status om_multi_create(const int32_t* devices, uint32_t n, om_multi** out);
void om_multi_destroy(om_multi* m);
int32_t om_multi_transport(const om_multi* m);      /* OM_TRANSPORT_*, or -1 for NULL */
/* The ctx of one rank (kernel, pipeline, timing, counters ... apply per rank); owned by m. */
om_ctx* om_multi_ctx(om_multi* m, uint32_t rank);
om_status om_multi_upload_world(om_multi* m, const om_world* w);
/* One progressive call over the whole frame, like om_render_device on dev_frame (W*H device
 * memory on devices[0]), with the ranks' shards RESIDENT on their GPUs between calls: the
 * first call that sees dev_frame (or another pointer or size, or the first after
 * om_multi_reset) cuts it into shards and deals them out; later calls only render, every rank
 * its tiles on its own stream.  dev_frame is brought up to date by om_multi_gather, not by this
 * call (the reference's one shared framebuffer without a per-pass copy, main.rs:192-214).
 * Call om_multi_reset after writing dev_frame yourself.  Asynchronous on `stream` (a stream of
 * devices[0]; NULL = rank 0's ctx stream). */
om_status om_multi_render(om_multi* m, const om_camera* cam, const om_render_params* p, om_pixel_stats* dev_frame,
                          void* stream);
/* The resident shards back into dev_frame (W*H device memory on devices[0]; normally the frame
 * om_multi_render was given): one RCCL group (or device copies) into rank 0 plus the scatter.
 * Ordered after every rank's last om_multi_render; asynchronous on `stream`. */
om_status om_multi_gather(om_multi* m, om_pixel_stats* dev_frame, uint32_t width, uint32_t height, void* stream);
/* Forget the resident frame: the next om_multi_render deals its frame out again. */
void om_multi_reset(om_multi* m);
/* Host framebuffer form (like om_render): every call copies `stats` (W*H, caller-owned host
 * memory, which the caller may have zeroed or rewritten since the last call) to devices[0],
 * deals it out, renders across the ranks, gathers once and copies the frame back; synchronous.
 * `counters` (optional) sums every rank's work counters of this call. */
om_status om_multi_render_host(om_multi* m, const om_camera* cam, const om_render_params* p, om_pixel_stats* stats,
                               om_counters* counters);
const char* om_multi_last_error(const om_multi* m);

#ifdef __cplusplus
}
#endif
#endif /* OTTOMARCHER_H */
