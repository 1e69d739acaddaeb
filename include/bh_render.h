/*
 * bh_render.h — C ABI of the MI355X-native geodesic ray-marcher.
 *
 * This is the drop-in boundary for ONE hot path of jonathandw743/black_hole_ray_marching:
 * the per-pixel Schwarzschild photon integrator `fs_main -> get_col`
 * (src/black_hole_maybe.wgsl:259-370), which the reference drives through
 * `Scene::render(encoder, output_view, blackout_output_view)` (src/scene.rs:470-522).
 *
 * Mapping of reference interfaces onto entry points (all paths relative to the reference repo):
 *
 *   bh_camera_uniform          == WGSL `Camera` (src/black_hole_maybe.wgsl:9-17), packed by
 *                                 `CameraUniform` (src/uniforms.rs:98-106) with encase: 112 B.
 *   bh_uniforms                == WGSL `Uniforms` (src/black_hole_maybe.wgsl:58-69), packed by
 *                                 `OtherUniforms::uniform_buffer_content` (src/otheruniforms.rs:105-118): 32 B.
 *   bh_camera                  == `Camera` (src/camera.rs:11-20).
 *   bh_uniforms_default        == the six `OtherUniform` defaults of `Scene::new` (src/scene.rs:89-137),
 *                                 including the inverted PodBool (src/podbool.rs:21-26) => blackout_eh = 1.
 *   bh_camera_default          == the camera literal of `Scene::new` (src/scene.rs:68-76).
 *   bh_camera_uniform_update   == `CameraUniform::update` (src/uniforms.rs:123-133) ->
 *                                 `Camera::pos_to_world_space_screen_triangle` (src/camera.rs:89-112).
 *   bh_create                  == the sky-texture half of `Scene::new`: `Texture::from_bytes` /
 *                                 `from_image` (src/texture.rs:11-77, Rgba8UnormSrgb, clamp, mag Linear)
 *                                 as bound at src/scene.rs:186-232.
 *   bh_render                  == `Scene::render` (src/scene.rs:470-522): one full-screen pass writing
 *                                 `col` (target 0) and optionally `blackout_col` (target 1; NULL == None).
 *   bh_destroy                 == dropping the `Scene`'s GPU resources.
 *
 * Conventions: every function returns BH_OK (0) or a negative bh_status; nothing aborts or throws
 * across the ABI.  Output pointers are caller-owned DEVICE pointers (the reference's consumer, Bloom,
 * owns its textures and lends views: src/bloom.rs:31-37).  bh_render is asynchronous on the given
 * HIP stream (NULL = the legacy default stream).  It never synchronises the host, with one exception:
 * a bh_render_frames call of more than 32 frames may wait for the copy of the call four before it on
 * the same stream (its pinned staging ring, see bh_render_frames).  The tile schedule's temporal
 * dispatch order keeps small per-(frame geometry, shard, stream) device buffers in the ctx: the FIRST
 * bh_render of such a key allocates them (hipMalloc) and must not be captured -- on a capturing stream
 * it returns BH_ERR_UNSUPPORTED and launches nothing; every later call with that key allocates nothing
 * and may be captured into a hipGraph.  Those buffers are never freed or moved before bh_destroy
 * while a graph may use them: a key rendered under stream capture is never evicted.  Other keys are
 * evicted least-recently-used beyond BH_ORDER_STATES (when every key has been captured the ctx keeps
 * more instead).  bh_bloom keeps one scratch set per (size, levels) under the same contract: the first
 * call of a (size, levels, schedule) allocates and must not be captured (BH_ERR_UNSUPPORTED on a
 * capturing stream), a set used under capture is never freed, others are evicted least-recently-used
 * beyond BH_BLOOM_SETS.  A stream whose capture status the runtime cannot report (e.g. the legacy
 * stream while another stream captures globally) counts as capturing.  Captured states stay pinned
 * until bh_destroy, or until bh_graph_release (call it once the graphs that used them are destroyed).
 * Renders of one ctx on different streams with the TILE or PAIR schedule use
 * different order state and no other shared scratch, so they may run concurrently (frames in flight);
 * the PERSISTENT schedule (shared work counters) and bh_bloom (shared scratch textures) must not run
 * concurrently with themselves on one ctx.  One bh_ctx per device; a ctx is not thread-safe, distinct
 * ctx objects may be used from distinct threads (one per rank).
 */
#ifndef BH_RENDER_H
#define BH_RENDER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BH_ABI_VERSION 8

/* Temporal-order states (frame geometry x shard x stream) one ctx keeps (see above). */
#define BH_ORDER_STATES 32
/* bh_bloom scratch sets (size x levels) one ctx keeps (see above). */
#define BH_BLOOM_SETS 4

typedef enum {
    BH_OK = 0,
    BH_ERR_INVALID_ARG = -1,   /* NULL/zero/out-of-range argument */
    BH_ERR_UNSUPPORTED = -2,   /* valid for the reference but not implemented (e.g. non-default screen triangle) */
    BH_ERR_HIP = -3,           /* a HIP runtime call failed; see bh_last_error() */
    BH_ERR_NO_DEVICE = -4,     /* no HIP device / device index out of range */
    BH_ERR_OUT_OF_MEMORY = -5,
    BH_ERR_INTERNAL = -6       /* a host-side consistency check failed (bh_bloom_check); see bh_last_error() */
} bh_status;

/* WGSL `Camera` (src/black_hole_maybe.wgsl:9-17), std140/encase layout, 112 bytes:
 *   pos @0 (vec3, padded to 16), screen_space_screen_triangle @16 (3 x vec4),
 *   pos_to_world_space_screen_triangle @64 (3 x vec4). */
typedef struct {
    float pos[3];
    float _pad0;
    float screen_tri[3][4];
    float world_tri[3][4];
} bh_camera_uniform;

/* WGSL `Uniforms` (src/black_hole_maybe.wgsl:58-69), 32 bytes.
 * bg_brightness is carried for layout fidelity but unused by the shader (as in the reference). */
typedef struct {
    float rs;               /* RS: Schwarzschild radius (default 1.0) */
    float delta_time_mult;  /* DELTA_TIME_MULT (default 0.5) */
    float bg_brightness;    /* BG_BRIGHTNESS (default 0.5, unused) */
    uint32_t blackout_eh;   /* BLACKOUT_EH: != 0 enables event-horizon blackout (default 1) */
    float max_dist;         /* MAX_DIST (default 250.0) */
    float distortion_power; /* DISTORTION_POWER (default 1.0) */
    uint32_t _pad[2];
} bh_uniforms;

/* `Camera` (src/camera.rs:11-20). */
typedef struct {
    float pos[3];
    float dir[3];
    float up[3];
    float aspect;
    float fovy;
    float znear;
    float zfar;
} bh_camera;

/* Output texel formats.  The reference stores into Bgra8UnormSrgb surfaces (src/copy.rs:132,
 * src/remix.rs:160); RGBA32F is the parity format, RGBA16F the production format. */
typedef enum {
    BH_OUT_RGBA32F = 0,     /* 16 B / pixel, linear */
    BH_OUT_RGBA16F = 1,     /*  8 B / pixel, linear, round-to-nearest-even from the fp32 result */
    BH_OUT_BGRA8_SRGB = 2   /*  4 B / pixel, sRGB-encoded (round(255 * OETF(clamp(x, 0, 1))), NaN -> 0),
                               byte order B,G,R,A: the Bgra8UnormSrgb store of the reference */
} bh_out_format;

/* Arithmetic mode of the integrator (see DESIGN.md "Math modes"). */
typedef enum {
    BH_MATH_EXACT = 0,      /* IEEE div/sqrt, no contraction, same op order as the oracle: bit-exact parity */
    BH_MATH_FAST = 1        /* rsq/rcp/FMA reformulation: production speed, tolerance parity */
} bh_math_mode;

/* Scene contents (bit mask).  The reference always has both (src/black_hole_maybe.wgsl:119-123);
 * 0 removes every surface (sdf == +inf), BASELINE config 1. */
#define BH_SCENE_DISC    1u
#define BH_SCENE_MARKERS 2u
#define BH_SCENE_DEFAULT (BH_SCENE_DISC | BH_SCENE_MARKERS)

/* Output layout. */
typedef enum {
    BH_LAYOUT_ROWMAJOR = 0, /* out[y * width + x]; requires shard_count == 1 */
    BH_LAYOUT_TILES = 1,    /* the shard's 8x8 tiles packed in shard order, 64 pixels per tile,
                               pixel (x & 7) + 8 * (y & 7) inside a tile; pixels outside the frame
                               are left untouched */
    BH_LAYOUT_TILES_RGB = 2, /* BH_LAYOUT_TILES without alpha (both targets' alpha is always 1,
                               src/black_hole_maybe.wgsl:369): each tile is three planes of 64
                               channel values in the format's memory order less alpha (R, G, B for
                               RGBA16F/RGBA32F; B, G, R for BGRA8), 3/4 of the bytes to gather */
    BH_LAYOUT_TILES_RGBM = 3, /* BH_LAYOUT_TILES_RGB plus, after each tile's three planes, one 64-bit
                               little-endian word whose bit i is set when pixel i of the tile has
                               blackout_col == 0, i.e. dot(col, col) < 1 in fp32 (src/black_hole_maybe.wgsl:365-368):
                               the multi-GPU transport.  blackout_col is a per-pixel function of the
                               fp32 col, but not of its quantised RGBA16F / BGRA8 bytes, so the decision
                               travels with them (0.125 B/pixel) and the gathered col alone restores both
                               targets bit for bit (bh_tiles_unpack_rgbm).  Tile bytes: 776 (RGBA32F),
                               392 (RGBA16F), 200 (BGRA8).  Schedules TILE and PAIR only. */
    BH_LAYOUT_TILES_RGBM14 = 4 /* BH_LAYOUT_TILES_RGBM for RGBA16F in 344 B per tile (5.375 B/pixel instead
                               of 6.125): every colour channel is an fp16 in [0, 1] -- sky samples are
                               bilinear mixes of decoded texels in [0, 1] (and g, b their c * sqrt(c)),
                               surfaces 1, blackout 0 -- so its top two bits are 0 and 14 bits carry it.
                               Per tile: 64 words r | g << 14 | (b & 0xF) << 28, 64 bytes (b >> 4) & 0xFF,
                               two 64-bit words holding bit 12 / bit 13 of b for pixel i at bit i, then the
                               blackout mask word.  RGBA16F, schedules TILE and PAIR only; unpack with
                               bh_tiles_unpack_rgbm(_partition) and format BH_OUT_RGBA16F | BH_UNPACK_RGBM14. */
} bh_layout;
/* format flag of bh_tiles_unpack_rgbm / bh_tiles_unpack_rgbm_partition: the shards are
 * BH_LAYOUT_TILES_RGBM14 (with BH_OUT_RGBA16F) */
#define BH_UNPACK_RGBM14 0x100u

/* Work schedule of the march kernel (same results, different speed). */
typedef enum {
    BH_SCHED_TILE = 0,       /* one wave64 per 8x8 tile (default); dispatch order: the previous frame's
                                per-tile cost, most expensive first (ties / first frame: centre-out
                                around the black hole's screen row) */
    BH_SCHED_PAIR = 1,       /* one wave64 per two 8x8 tiles, two interleaved rays per lane */
    BH_SCHED_PERSISTENT = 2  /* resident waves, per-lane refill from an LDS ray queue */
} bh_schedule;
/* OR into `schedule` to use the static centre-out order only (no per-tile cost feedback). */
#define BH_SCHED_FLAG_STATIC_ORDER 0x100u
/* Exact math: which build of the march kernels runs (same bits either way).  By default bh_render
 * picks per launch: the source-order build when it is throughput-bound (its tiles in flight, over
 * all frames of a bh_render_frames launch, >= 384 per CU x max_iters / 512), else the
 * machine-scheduled build, whose lone tail waves step faster (packed-FP32 tail step).
 * These flags force one (BH_SCHED_FLAG_ISSUE_ORDER wins if both are set). */
#define BH_SCHED_FLAG_ISSUE_ORDER 0x200u
#define BH_SCHED_FLAG_LATENCY 0x400u

/* Per-pixel fate codes written to dbg_fate. */
#define BH_FATE_CAP      0u  /* loop ran out (max_iters); still shades sky with its current rd */
#define BH_FATE_ESCAPE   1u  /* distance_travelled > MAX_DIST (src/black_hole_maybe.wgsl:325-327) */
#define BH_FATE_SURFACE  2u  /* sdf < MIN_DIST (:286-288) -> colour 1 */
#define BH_FATE_BLACKOUT 3u  /* event-horizon blackout (:272-283) -> colour 0 */

#define BH_TILE 8u           /* tile edge in pixels (multi-GPU sharding and BH_LAYOUT_TILES) */

typedef struct bh_partition bh_partition;

typedef struct {
    uint32_t width, height;   /* frame size in pixels */
    uint32_t max_iters;       /* MAX_ITERATIONS (WGSL const 1000, src/black_hole_maybe.wgsl:85), 1..65535 */
    uint32_t scene_flags;     /* BH_SCENE_* */
    uint32_t format;          /* bh_out_format */
    uint32_t math;            /* bh_math_mode */
    uint32_t layout;          /* bh_layout */
    uint32_t shard_index;     /* this rank's tile share: tile (tx,ty) belongs to shard (tx + 3*ty) % shard_count */
    uint32_t shard_count;     /* 1 = whole frame */
    uint32_t schedule;        /* bh_schedule | BH_SCHED_FLAG_* (results never depend on it) */
    void* out_col;            /* target 0 (`col`), device pointer, never NULL */
    void* out_blackout;       /* target 1 (`blackout_col`), device pointer or NULL (== Option::None) */
    uint16_t* dbg_n_rk;       /* optional: completed RK4 steps per pixel (same layout as outputs, 1 elem/px) */
    uint8_t* dbg_fate;        /* optional: BH_FATE_* per pixel */
    uint16_t* dbg_steps;      /* optional: RK4 iterations actually executed per pixel; below dbg_n_rk
                                 only where a ray that had entered an exact cycle (see DESIGN.md
                                 "Cycle fast-forward") was advanced to the cap without iterating */
    const bh_partition* partition; /* optional, BH_LAYOUT_TILES* only: a weighted tile partition
                                 (bh_partition_create) with this frame size and shard_count, used
                                 instead of the default (tx + 3*ty) % shard_count interleave */
} bh_render_desc;

typedef struct bh_ctx bh_ctx;

int bh_abi_version(void);
const char* bh_status_string(int status);
/* Thread-local text of the last HIP error seen by this library ("" if none). */
const char* bh_last_error(void);

/* Defaults of Scene::new (src/scene.rs:68-137). */
int bh_uniforms_default(bh_uniforms* out);
int bh_camera_default(uint32_t width, uint32_t height, bh_camera* out);
/* CameraController (src/camera.rs:115-366), the host camera layer of an animated / offline camera
 * path: the controller's key state (process_event, :186-261, as booleans), its two speeds
 * (CameraController::new(5.0, 0.5) at src/scene.rs:78; Q / E scale `speed` by 1/1.5 and 1.5) and
 * the last two cursor positions (as f32, the conversion of :270-276). */
typedef struct {
    uint8_t forward, backward, left, right, up, down;  /* W, S, A, D, Space, F */
    uint8_t pan_up, pan_down, pan_left, pan_right;     /* arrow keys */
    uint8_t exp_towards_origin, exp_away_origin;       /* P, O */
    uint8_t mouse_pressed;                             /* left button */
    uint8_t has_prev_cursor, has_curr_cursor;          /* Option::Some */
    uint8_t _pad;
    float prev_cursor[2], curr_cursor[2];
    float speed, pan_speed;
} bh_controller;

/* CameraController::update_camera(camera, delta_time, do_pan) (src/camera.rs:280-366): moves and
 * rotates *camera by dt seconds of the controller's state, glam f32 arithmetic (Quat::from_axis_angle,
 * Quat::mul_vec3).  *moved (optional) = the function's return value. */
int bh_controller_update(const bh_controller* ctrl, bh_camera* camera, float dt, int do_pan, int* moved);

/* CameraUniform::new (src/uniforms.rs:108-122) + ::update (:123-133). */
int bh_camera_uniform_update(const bh_camera* camera, bh_camera_uniform* out);
/* Camera aimed at `target` from `pos` (up +Y, fovy pi/2): SURVEY §8d cameras B and C. */
int bh_camera_look_at(const float pos[3], const float target[3], uint32_t width, uint32_t height,
                      bh_camera* out);

/* Deterministic synthetic equirectangular sky (RGBA8, sRGB-encoded, alpha 255):
 * splitmix64-seeded value-noise nebula + sparse stars.  Stand-in for src/space_4096x2048.jpg. */
int bh_synthetic_sky(uint8_t* out_rgba8, uint32_t width, uint32_t height, uint64_t seed);

/* Upload the sky (width*height*4 bytes, Rgba8UnormSrgb semantics) to `device` and build the
 * sRGB->linear table.  The context owns the device copy. */
int bh_create(const uint8_t* sky_rgba8_srgb, uint32_t sky_width, uint32_t sky_height, int device,
              bh_ctx** out);
int bh_destroy(bh_ctx* ctx);

/* Scene::render.  Asynchronous on `hip_stream` (a hipStream_t, NULL = default stream). */
int bh_render(bh_ctx* ctx, const bh_camera_uniform* camera, const bh_uniforms* uniforms,
              const bh_render_desc* desc, void* hip_stream);

/* Several frames in ONE launch: n_frames (1..BH_MAX_FRAMES) calls of Scene::render -- e.g. consecutive
 * frames of an offline camera path, cameras[i] for frame i -- with one `uniforms` and descs that agree in
 * everything but their output and debug pointers (frame size, cap, scene, format, math, layout, shard,
 * schedule; else BH_ERR_INVALID_ARG).  Each frame's results are exactly bh_render's.  With the tile
 * schedule the frames' tiles are interleaved in one grid (slot s = tile s / n of frame s % n, most
 * expensive tiles first), so the frames' serial tails -- the few rays that march to the cap -- overlap
 * each other's bulk instead of each ending a launch alone; other schedules run n launches.  The
 * temporal order of (geometry, shard, stream) learns from frame 0 of each call.  Up to 32 frames travel
 * in the kernel argument; a call of more stages the frames' arguments through a pinned host ring into a
 * device table of the stream (allocated at the first such call, never captured into a HIP graph: a
 * capturing stream gets BH_ERR_UNSUPPORTED for n_frames > 32).  The ring has 4 slots: such a call
 * blocks the host until the copy of the 4th such call before it on the stream has executed. */
#define BH_MAX_FRAMES 256
int bh_render_frames(bh_ctx* ctx, uint32_t n_frames, const bh_camera_uniform* cameras, const bh_uniforms* uniforms,
                     const bh_render_desc* descs, void* hip_stream);

/* Bloom::render (src/bloom.rs:53-71): the reference's Kawase bloom + remix chain over the scene's two
 * targets, on BGRA8-sRGB images (bh_render with BH_OUT_BGRA8_SRGB): `col` (full_image_input),
 * `blackout` (blackout_input) -> `out` (the surface), all width x height (1..65536 each, as bh_render),
 * row-major, device memory.  `levels` = the Bloom's level count (src/state.rs:125 uses 3; 1..12).  Scratch textures live in
 * the context (allocated at the first call for a size; graph contract above).  `schedule`: BH_BLOOM_AUTO
 * fuses passes whenever that gives identical bytes (the host proves the chain's same-size samples are
 * identities on stored texels: powers of two, 1920x1080, 1280x720, ...), BH_BLOOM_LITERAL runs the
 * reference's render passes one by one.  Asynchronous on `hip_stream`. */
#define BH_BLOOM_AUTO    0u
#define BH_BLOOM_LITERAL 1u
int bh_bloom(bh_ctx* ctx, const void* col_bgra8, const void* blackout_bgra8, uint32_t width, uint32_t height,
             uint32_t levels, uint32_t schedule, void* out_bgra8, void* hip_stream);

/* Host only (no device needed): plan bh_bloom's chain for width x height, `levels`, `schedule` exactly as
 * bh_bloom does -- the same schedule choice, plans and kernel forms -- and, instead of launching, check
 * every launch's index arithmetic on the host: every block's staged footprint fits its LDS tile, every
 * tile read falls inside the staged footprint, every plan index and fix-up list entry inside its texture
 * (the kernels' own f32 sampler arithmetic, per block and tap).  BH_OK, or BH_ERR_INTERNAL with the first
 * violation in bh_last_error().  *out_launches (optional) = the launches the chain makes; out_plan (optional,
 * plan_len bytes, NUL-terminated, truncated) = one line per launch: "form ow oh tw th rx ry" (the kernel form,
 * its output and input sizes and resolution uniform; tools/bloom_roofline.py reads it). */
int bh_bloom_check(uint32_t width, uint32_t height, uint32_t levels, uint32_t schedule, uint64_t* out_launches,
                   char* out_plan, size_t plan_len);

/* Process-wide count of the plans real bh_bloom calls built and whose host check (the checks of
 * bh_bloom_check) refused: such a pass runs its general kernel -- the same bytes, slower -- and the first
 * refusal is also reported on stderr.  out_last (optional, len bytes, NUL-terminated, truncated) = the last
 * refusal's message.  0 for every frame size the tests name. */
int64_t bh_bloom_plan_failures(char* out_last, size_t len);

/* The frame the reference application presents per redraw, State::render (src/state.rs:270-286):
 * Scene::render into the two Bgra8UnormSrgb targets, then Bloom::render from them to the surface -- as one
 * pipelined path.  A presenter owns `depth` banks of `batch` target pairs, `march_streams` march streams and
 * one bloom stream of `ctx`'s device: call c marches its n frames (one bh_render_frames launch,
 * BH_OUT_BGRA8_SRGB, both targets) into bank c % depth on march stream c % march_streams, then blooms them on
 * the bloom stream.  So the bloom of call c fills the CUs the march of call c + 1 leaves idle instead of
 * adding to it, and (march_streams 2) the march of call c + 1 starts while the serial tail of call c's march
 * -- the few rays that run to the cap -- still runs, as the frames of one multi-frame launch overlap each
 * other's tails.  A call of 4 or more frames fills the GPU by itself (its frames overlap each other's tails in
 * one launch): it runs its march and then its blooms on the caller's stream, in order.  Each surface holds exactly the
 * bytes of bh_render + bh_bloom run one after the other.  Asynchronous: the blooms wait for the caller's
 * stream as it is at the call (earlier users of the surfaces), and the caller's stream waits for the
 * call's last bloom (later users see the finished surfaces); the host never blocks.  `bloom_cus` = 0: the
 * bloom's stream shares every CU at the device's highest priority; k > 0: the bloom runs on k CUs (spread
 * over the mask), the march on the others (hipExtStreamCreateWithCUMask).  The presenter's blooms share
 * `ctx`'s bloom scratch: do not run bh_bloom of the same ctx concurrently with it.  The first call of a
 * presenter allocates (order state, bloom scratch): do not capture it into a graph. */
#define BH_PRESENT_BATCH_MAX 32
#define BH_PRESENT_DEPTH_MAX 8
typedef struct bh_presenter bh_presenter;
typedef struct {
    uint32_t width, height;   /* frame size (1..65536) */
    uint32_t max_iters;       /* MAX_ITERATIONS, 1..65535 */
    uint32_t scene_flags;     /* BH_SCENE_* */
    uint32_t math;            /* bh_math_mode */
    uint32_t levels;          /* the Bloom's levels (src/state.rs:125: 3), 1..12 */
    uint32_t batch;           /* frames per bh_present_frames call, 1..BH_PRESENT_BATCH_MAX (1: one frame per redraw) */
    uint32_t bloom_cus;       /* 0: shared CUs, high-priority bloom stream; else CUs given to the bloom */
    uint32_t depth;           /* calls in flight: target banks, 2..BH_PRESENT_DEPTH_MAX (0: 3) */
    uint32_t march_streams;   /* 1 or 2, at most depth (0: 2 when the call's frames hold at most 64 tiles
                                 per CU -- a march that leaves the GPU mostly idle -- else 1) */
} bh_presenter_desc;
int bh_presenter_create(bh_ctx* ctx, const bh_presenter_desc* desc, bh_presenter** out);
int bh_presenter_destroy(bh_presenter* presenter);
/* n (1..batch) frames: cameras[i] -> out_surfaces[i] (width x height BGRA8 device images, caller-owned). */
int bh_present_frames(bh_presenter* presenter, uint32_t n, const bh_camera_uniform* cameras, const bh_uniforms* uniforms,
                      void* const* out_surfaces, void* hip_stream);
/* bh_present_frames of one frame: State::render. */
int bh_present(bh_presenter* presenter, const bh_camera_uniform* camera, const bh_uniforms* uniforms, void* out_surface,
               void* hip_stream);

/* Graph contract (see the top of this file): unpin every order state and bloom scratch set that a
 * capture marked, so that LRU eviction may free them again.  Call it only after destroying every HIP
 * graph captured from this ctx (their kernels read and write those buffers). */
int bh_graph_release(bh_ctx* ctx);

/* Number of 8x8 tiles owned by `shard_index` of `shard_count` in a width x height frame. */
int64_t bh_shard_tile_count(uint32_t width, uint32_t height, uint32_t shard_index, uint32_t shard_count);

/* Scatter the gathered tile-packed shards back into a row-major frame (rank 0 after the gather).
 * `packed` holds shard 0's tiles, then shard 1's, ... (the concatenation a gather produces, each
 * shard's block padded to `shard_stride_tiles` tiles); `bytes_per_pixel` is 4, 8 or 16. */
int bh_tiles_unpack(const void* packed, void* out_rowmajor, uint32_t width, uint32_t height,
                    uint32_t shard_count, uint64_t shard_stride_tiles, uint32_t bytes_per_pixel,
                    void* hip_stream);

/* As bh_tiles_unpack for BH_LAYOUT_TILES_RGB shards of `format` (bh_out_format): restores the
 * constant alpha (1.0 / 255) of the row-major frame. */
int bh_tiles_unpack_rgb(const void* packed, void* out_rowmajor, uint32_t width, uint32_t height,
                        uint32_t shard_count, uint64_t shard_stride_tiles, uint32_t format,
                        void* hip_stream);

/* As bh_tiles_unpack_rgb with at most `rows_in_flight` 8-pixel tile rows of the frame in flight at
 * once (0 = all; the kernel grid-strides over the rest).  For an unpack that overlaps a render on
 * the same GPU (rank 0 of the multi-GPU pipeline) a bounded value keeps it from displacing the
 * render's waves: at N=8 on the 4096x2048 frame, rank 0's render + unpack measured 0.099 ms per
 * frame with 64 rows in flight, 0.100 with all, 0.138 with 16. */
int bh_tiles_unpack_rgb_rows(const void* packed, void* out_rowmajor, uint32_t width, uint32_t height,
                             uint32_t shard_count, uint64_t shard_stride_tiles, uint32_t format,
                             uint32_t rows_in_flight, void* hip_stream);

/* Rank 0 of the multi-GPU frame: gathered BH_LAYOUT_TILES_RGBM shards of `format` -> BOTH targets of
 * Scene::render (src/scene.rs:476-509), row-major: `out_col` (alpha restored) and, unless NULL
 * (== Option::None), `out_blackout` = the tile mask's pixels zeroed (alpha kept), else col.  Equal
 * bit for bit to a single-GPU two-target bh_render.  `rows_in_flight` as bh_tiles_unpack_rgb_rows. */
int bh_tiles_unpack_rgbm(const void* packed, void* out_col, void* out_blackout, uint32_t width, uint32_t height,
                         uint32_t shard_count, uint64_t shard_stride_tiles, uint32_t format,
                         uint32_t rows_in_flight, void* hip_stream);
/* Weighted tile partitions (multi-GPU).  The default ownership gives every shard 1/shard_count of
 * the tiles; a partition gives shard k weights[k] of every M = sum(weights) residues: tile (tx, ty)
 * belongs to owner[(tx + 3*ty) % M], the M residues dealt to the shards by smooth weighted round
 * robin (each shard's residues spread evenly over the M), so that a shard with more work beside its
 * render -- rank 0, which also unpacks every frame -- can take a smaller share.  A shard's packed
 * order is row-major over its tiles, as for the default interleave.  weights[k] may be 0 (a shard
 * that renders nothing); M <= 4096.  The partition holds device tables on `device` (each shard's
 * tile list, and every tile's shard and packed index for the unpack); destroy it after the renders
 * and unpacks that use it have completed. */
int bh_partition_create(uint32_t width, uint32_t height, uint32_t shard_count, const uint32_t* weights, int device,
                        bh_partition** out);
int bh_partition_destroy(bh_partition* partition);
/* Tiles owned by `shard_index` (a shard's packed buffer holds this many tiles), or a negative status. */
int64_t bh_partition_tile_count(const bh_partition* partition, uint32_t shard_index);
/* Host only (no device needed): the same partition's map, tile t = ty * tiles_x + tx:
 * owner_out[t] = its shard, index_out[t] = its index in that shard's packed order (arrays of
 * tiles_x * tiles_y entries; either may be NULL). */
int bh_partition_map(uint32_t width, uint32_t height, uint32_t shard_count, const uint32_t* weights, uint32_t* owner_out,
                     uint32_t* index_out);
/* bh_tiles_unpack_rgbm for shards rendered with `partition` (its frame size and shard count). */
int bh_tiles_unpack_rgbm_partition(const void* packed, void* out_col, void* out_blackout, const bh_partition* partition,
                                   uint64_t shard_stride_tiles, uint32_t format, uint32_t rows_in_flight,
                                   void* hip_stream);

/* Bytes of one tile of `layout` (BH_LAYOUT_TILES*) in `format`, or a negative bh_status. */
int64_t bh_tile_bytes(uint32_t layout, uint32_t format);

/* The BGRA8 sRGB encoder's threshold table: out[k] (k = 1..255) = the smallest float x with
 * encode(x) >= k, out[0] = 0, out[256] = +inf; encode(x) = the largest k with x >= out[k]. */
int bh_srgb_encode_table(float* out257);

/* Diagnostics: check the correctly rounded division/sqrt cores the exact kernel uses against IEEE
 * results on `device` (op 0: sqrt over float bit patterns [base, base+count); op 1: x/6 over bit
 * patterns [base, base+count); op 2: n/d on `count` random pairs seeded by base; op 3: n/d near exact
 * quotients; op 4: the BGRA8 sRGB encoder over float bit patterns [base, base+count) against a
 * binary search of bh_srgb_encode_table; op 5: x/12 as the bloom chain computes it, over bit
 * patterns [base, base+count); op 6: the bloom chain's table-form sRGB encoder against op 4's; op 7:
 * n/d over all 2^23 numerator significands for the denominator significands (fraction bits)
 * [base, base + count/2^23); op 8: the shading's f32-rounded atan2 (short f64 core + library fallback)
 * against (float)atan2((double)y, (double)x) on `count` random (y, x) pairs seeded by base; op 9:
 * the number of those pairs the core hands to the fallback; op 10: the bloom chain's code-table form of
 * the sRGB encoder against op 4's over bit patterns [base, base+count); op 11: the march kernel's
 * wave-wide max of the tile costs (DPP scan) against a serial max, `count` random rounds per wave
 * seeded by base; op 12: the march step's reciprocal of rd_derivative's denominator seeded from the
 * square-root core's v_rsq, over q bit patterns [base, base+count), against the IEEE 1/Q; op 13: for the
 * q of that range whose seeded reciprocal differs from 1/Q, the division core with it over every numerator
 * significand against the IEEE quotient).  *out_mismatches = number of differing results;
 * out_examples (8 u32, optional) = up to two (a, b, got, want) bit patterns.  Synchronous. */
int bh_selftest_crmath(int op, uint64_t base, uint64_t count, uint64_t* out_mismatches,
                       uint32_t* out_examples, int device);

/* Diagnostics: the shader clock DURING march launches (the bench's "clock" block).  While armed
 * (acc != NULL), one wave in `stride` (a power of two) of the tile schedule's march kernels of this ctx --
 * dispatch slots k with (k + k / 256) % stride == 0, spread over the XCDs -- reads the shader-clock
 * counter (s_memtime) and the constant
 * 100 MHz counter (s_memrealtime) when it starts and when it ends, and adds the differences to its
 * XCD's slot: acc[16*x + 0] += shader ticks, acc[16*x + 1] += 100 MHz ticks, acc[16*x + 2] += 1 (x =
 * the XCD, 0..7; acc = 128 u64 of device memory, zeroed by the caller, 128 B per XCD).  The clock of
 * XCD x over the sampled waves' lifetimes is 100 MHz * acc[16x] / acc[16x+1].  Takes effect from the
 * next bh_render* call; never changes a result.  acc = NULL disarms. */
int bh_set_clock_probe(bh_ctx* ctx, uint64_t* acc, uint32_t stride);

#ifdef __cplusplus
}
#endif

#endif /* BH_RENDER_H */
