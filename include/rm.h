/*
 * rm.h -- C ABI of librm.so, the MI355X (gfx950) ray-march pass.
 *
 * Drop-in boundary for the reference's full-screen fragment pass
 * (cahekp/Raymarching).  The reference drives that pass through SFML:
 *
 *   ShaderLoader::loadFromFile(file, sf::Shader::Fragment, shader)
 *       source/shader_loader.h:11, source/shader_loader.cpp:8-20
 *   shader.setUniform("u_resolution" | "u_pos" | "u_mouse" | "u_time" | ...)
 *       main.cpp:54,187-194 (include/SFML/Graphics/Shader.hpp:297,306,315)
 *   renderTexture.draw(fullScreenSprite, &shader)
 *       main.cpp:199,205 (include/SFML/Graphics/RenderTarget.hpp:237)
 *
 * and each entry point below replaces one of those calls (see the per-call
 * comments and INTEGRATION.md).  Conventions: every call returns an
 * rm_status (no exceptions cross the ABI); buffers are caller-owned; one
 * rm_ctx per host thread; uniforms/params are state of the ctx, read at the
 * next render call, as GL uniforms are read at the next draw.
 *
 * Pixel convention: out[row*W + col] is the fragment with
 * gl_TexCoord = ((col+0.5)/W, (row+0.5)/H); row 0 is first in memory and
 * looks up.  Pixels are RGBA float32 (gl_FragColor,
 * alpha = 1) or, from the *_rgba8 calls, RGBA8 unorm as the reference's
 * sf::RenderTexture stores them.
 */
#ifndef RM_H_
#define RM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Version of the structs and calls below.  Bumped whenever a struct the
 * library writes grows or a call changes meaning; a caller compiled against
 * one version must not pass its structs to a library of another (check
 * rm_abi_version() == RM_ABI_VERSION once at start-up).
 *   1  round 1-2 (rm_stats without `skipped`)
 *   2  rm_stats.skipped
 *   3  rm_stats.dispatch, rm_stats.lat_tiles; rm_abi_version() */
#define RM_ABI_VERSION 3

typedef enum rm_status {
    RM_OK = 0,
    RM_ERR_INVALID_ARGUMENT = 1, /* bad pointer/size/uniform arity                       */
    RM_ERR_FILE = 2,             /* "can't load file" (source/shader_loader.cpp:26-30)  */
    RM_ERR_SCENE = 3,            /* no scene plugin for this source (cf. GL compile fail) */
    RM_ERR_NO_SCENE = 4,         /* render before a successful rm_load_scene            */
    RM_ERR_DEVICE = 5,           /* HIP runtime error (message in rm_last_error)        */
    RM_ERR_OUT_OF_MEMORY = 6
} rm_status;

typedef struct rm_ctx rm_ctx;

/* Run-time knobs that replace the reference's compile-time constants. */
typedef struct rm_params {
    int32_t max_steps;        /* MAX_MARCHING_STEPS, common.frag:15 (default 128)        */
    int32_t shadow_max_steps; /* softshadow2 cap; 0 = unbounded as common.frag:814       */
    int32_t count_evals;      /* 1: instrumented kernel, rm_stats.evals = sceneSDF calls */
    int32_t kernel;           /* workgroup tiling: 0 auto (= 2), 1 16x16 px (4 waves), 2 8x8 px (1 wave), 3 16x4 px (1 wave),
                                 4 8x8 px tiles pulled by persistent waves from an atomic counter (built-in scenes) */
    int32_t schedule;         /* dispatch order of one-wave tiles: 1 (default) = the costliest tiles of a recent
                                 launch of the same geometry on the same stream first (their measured durations,
                                 counting-sorted on the GPU right after every 16th launch, on its stream,
                                 RM_SCHED_PERIOD; the first launch of a geometry runs row-major); 0 = row-major.
                                 Pixels are the same either way; an rm_set_tile_order order takes precedence. */
} rm_params;

/* rm_stats.dispatch: the order the launch's workgroups rendered tiles in */
enum {
    RM_DISPATCH_ROW_MAJOR = 0, /* workgroup i renders tile i                                    */
    RM_DISPATCH_EXPLICIT = 1,  /* rm_set_tile_order's order                                      */
    RM_DISPATCH_ADAPTIVE = 2   /* sorted durations of an earlier launch (rm_params.schedule = 1)  */
};

typedef struct rm_stats {
    uint64_t evals;  /* sceneSDF calls (ray-steps) of this render, when count_evals   */
    uint64_t pixels; /* pixels rendered                                                */
    float kernel_ms; /* device time of the render kernel (HIP events on the ctx stream) */
    int32_t scene;   /* scene id that ran                                              */
    uint64_t flop;   /* algorithmic FLOP of those calls, when count_evals: the per-term
                        tally of SURVEY.md 8(d) over the terms evaluated (exact early
                        exits skip Menger folds and scene O's primitives)          */
    uint64_t skipped; /* when count_evals: of `evals`, the ray-steps the uninstrumented
                        kernels do not execute (exact early exits whose results equal
                        the reference's: settled soft shadows, the soft shadows of
                        points facing away from the light, scene T's reflection march
                        past depth 3); executed = evals - skipped */
    int32_t dispatch; /* RM_DISPATCH_*: the tile order this launch ran (ABI 3)           */
    int32_t lat_tiles; /* scene T: workgroups that rendered with the latency-optimized
                         fold tests (the costliest tiles at the head of an ordered
                         launch of at most 98304 tiles); 0 otherwise
                         (ABI 3)                                                        */
    float gather_ms;   /* rm_render_sharded*: device time of the RGB8 pack and the gather
                         on this rank's stream (rank 0: until every wire has arrived,
                         so it includes waiting for the slowest rank); 0 elsewhere (ABI 3) */
    float deinterleave_ms; /* rm_render_sharded*, rank 0: the de-interleave kernel (ABI 3) */
} rm_stats;

/* RM_ABI_VERSION of the library (compare with the header's). */
int rm_abi_version(void);

/* Create a context on HIP device `device`.  Scene unset, params default. */
rm_status rm_create(rm_ctx **out, int device);
/* Waits for the work this context enqueued (its own events, not the device),
 * then frees it.  The stream it is bound to must still exist (rm_set_stream).
 * If recording on that stream reports an error, it waits for the whole device
 * instead. */
rm_status rm_destroy(rm_ctx *ctx);

/* Replaces ShaderLoader::loadFromFile (source/shader_loader.cpp:8-20).
 * If `file_name` exists it is preprocessed with the reference's #include
 * semantics (source/shader_loader.cpp:22-81; missing include -> RM_ERR_FILE).
 * The scene is chosen by the file's base name: "output_shader.frag"
 * (scene O), "template.frag" (scene T, repaired as SURVEY.md App. A),
 * "sphere" (scene S0), "output_shader_glass" (test scene OG).  A registered
 * name needs no file on disk (the GPU host has no shader tree).  When the
 * file exists its text decides (the reference's reload recompiles the edited
 * shader): output_shader.frag whose lighting/render/main code and included
 * common.frag are the reference's (whitespace-insensitive fingerprints) loads
 * the compiled-in scene O if its scene part (materials, floorMat, sceneSDF) is
 * the reference's too, and otherwise compiles that scene part with hiprtc as
 * a scene plugin into output_shader.frag's pipeline; other edits (pipeline,
 * common.frag, template.frag's text) return RM_ERR_SCENE.  Any other
 * existing file named "*.hip" is a scene plugin: a source defining
 * `SdResult sceneSDF(vec3 p)` with the reference's scene library
 * (common.frag:37-679; raymarching_amd/csrc/rm_sdf_lib.h), compiled here with
 * hiprtc into output_shader.frag's pass around that scene (the reference's
 * "Reload scene shader", main.cpp:134-139).  A compile error prints the log
 * and returns RM_ERR_SCENE, keeping the previous scene.  Unknown name and no
 * file -> RM_ERR_FILE; another existing file -> RM_ERR_SCENE. */
rm_status rm_load_scene(rm_ctx *ctx, const char *file_name);

/* Compile a scene file as rm_load_scene would, without loading it (no GPU
 * needed), as a GL driver compiles a shader: RM_OK, RM_ERR_FILE (missing file
 * or #include) or RM_ERR_SCENE (compile errors, or an edit rm_load_scene
 * refuses).  The compiler's log, or "compiled-in scene O|T" when no compile is
 * needed (NUL-terminated, truncated to log_size), goes to `log` when it is not
 * NULL. */
rm_status rm_compile_scene(const char *file_name, char *log, size_t log_size);

/* sceneSDF(p) of the loaded scene at n points: points = n xyz float triples,
 * dist = n floats, material = n x 16 floats of struct Material
 * (common.frag:20-35, declaration order) or NULL.  Device or host pointers;
 * returns when the results are written.  Uniforms (u_time ...) are the ctx's. */
rm_status rm_scene_eval(rm_ctx *ctx, const float *points, int64_t n, float *dist, float *material);

/* Replace sf::Shader::setUniform (include/SFML/Graphics/Shader.hpp:297,306,315)
 * for the names main.cpp sets: u_resolution (2f), u_pos (3f), u_mouse (2f),
 * u_time (1f), u_sample_part (1f), u_seed1/u_seed2 (2f).  The last three are
 * declared but unused by the reference's scenes (common.frag:8-11): the plain
 * renders ignore them and rm_render_accumulate* reads them.  Other names warn
 * once on stderr and are ignored, as SFML does for uniforms the GLSL compiler
 * removed.  Wrong arity -> RM_ERR_INVALID_ARGUMENT. */
rm_status rm_set_uniform1f(rm_ctx *ctx, const char *name, float x);
rm_status rm_set_uniform2f(rm_ctx *ctx, const char *name, float x, float y);
rm_status rm_set_uniform3f(rm_ctx *ctx, const char *name, float x, float y, float z);

rm_status rm_set_params(rm_ctx *ctx, const rm_params *params);
rm_status rm_get_params(rm_ctx *ctx, rm_params *params);

/* Stream the ctx launches on (a hipStream_t; NULL = the null stream).
 * Lifetime: a stream must outlive its binding.  Before destroying a stream the
 * context is bound to, bind another one (e.g. rm_set_stream(ctx, NULL)): that
 * records the context's completion marker (one event, only when the context
 * enqueued work there since it was bound) on the old stream while it exists.
 * Streams the context has left may be destroyed at any time.  Destroying the
 * bound stream first is undefined behaviour: the HIP runtime does not validate
 * stream handles, and a later rm_* call (rm_destroy included) that records on
 * the freed stream crashed the process in a test (SIGSEGV inside libamdhip64). */
rm_status rm_set_stream(rm_ctx *ctx, void *hip_stream);
/* rm_set_stream, with the caller's promise that the stream stays alive until
 * rm_destroy (e.g. a stream of PyTorch's pool, which is never destroyed).
 * Leaving a kept stream then records nothing on it; the context marks its work
 * there only when something waits for it (rm_destroy, or reusing a schedule
 * buffer), on the stream itself.  A frame loop that alternates between two
 * kept streams saves one marker per frame (~4 us each on MI355X, DESIGN.md
 * 2.14).  (No counterpart in the reference, which draws on one GL context.) */
rm_status rm_set_stream_kept(rm_ctx *ctx, void *hip_stream);
rm_status rm_synchronize(rm_ctx *ctx);

/* Replaces renderTexture.draw(sprite, &shader) (main.cpp:199,205): run the
 * pass over a W x H target into `out` (W*H*4 float).  Device `out`: the call
 * is asynchronous on the ctx stream unless `stats` is non-NULL (then it
 * waits and fills stats).  Host `out`: rendered through a device staging
 * buffer and copied back before returning. */
rm_status rm_render(rm_ctx *ctx, int W, int H, float *out, rm_stats *stats);

/* rm_render through the instrumented kernel, which also writes the number of
 * sceneSDF calls (ray-steps) each pixel made into evals_map (W*H uint32, row 0
 * first; the same count as rm_stats.evals, per pixel).  Device or host
 * buffers.  The parity tests compare it with the reference GLSL's counts. */
rm_status rm_render_step_map(rm_ctx *ctx, int W, int H, float *out, uint32_t *evals_map, rm_stats *stats);

/* Same pass over one shard of a W x H frame: frame row y belongs to shard
 * (y / band) % nshards; the shard's rows are packed into `out` in increasing
 * y (rm_shard_rows() rows of W float4).  Used by row-sharded multi-GPU frames. */
rm_status rm_render_band(rm_ctx *ctx, int W, int H, int band, int nshards, int shard, float *out,
                         rm_stats *stats);

/* A sub-range of rm_render_band: the shard's packed rows [row_begin,
 * row_begin + row_count) into `out` (row_count rows of W float4).  Lets a
 * caller pipeline a shard in chunks (render chunk k+1 while chunk k is
 * gathered). */
rm_status rm_render_rows(rm_ctx *ctx, int W, int H, int band, int nshards, int shard, int row_begin, int row_count,
                         float *out, rm_stats *stats);

/* Dispatch order of the render workgroups.  A render launch over W x rows
 * pixels is a grid of tiles_x x tiles_y tiles (rm_tile_grid: 8x8 pixels per
 * one-wave workgroup by default); with an order set, workgroup i renders tile
 * order[i] (tile = ty * tiles_x + tx), for launches whose grid has exactly n
 * tiles (others keep the identity order).  Pixels are unchanged; only the
 * time at which each tile starts moves -- e.g. the costliest tiles of the
 * previous frame first, so that the longest per-pixel chains (grazing soft
 * shadows) do not start last.  order: host or device, a permutation of
 * [0, n); n = 0 clears it. */
rm_status rm_set_tile_order(rm_ctx *ctx, const uint32_t *order, int64_t n);
rm_status rm_tile_grid(const rm_params *params, int W, int rows, int *tiles_x, int *tiles_y);

/* Number of frame rows shard `shard` owns. */
rm_status rm_shard_rows(int H, int band, int nshards, int shard, int *nrows);

/* Root side of a row-sharded frame: `gathered` holds nshards consecutive
 * blocks of rows_per_shard packed rows (rows_per_shard >= every shard's row
 * count); writes the W x H frame into `out`.  Device pointers, ctx stream. */
rm_status rm_deinterleave(rm_ctx *ctx, int W, int H, int band, int nshards, int rows_per_shard,
                          const float *gathered, float *out);

/* rm_deinterleave for RGBA8 frames (uint32 per pixel). */
rm_status rm_deinterleave_rgba8(rm_ctx *ctx, int W, int H, int band, int nshards, int rows_per_shard,
                                const uint32_t *gathered, uint32_t *out);

/* The 3 B/px wire of a row-sharded RGBA8 frame (the gather is
 * the only exchange, so its bytes bound multi-GPU scaling).  The pass writes
 * alpha 1 (vec4(col, 1.0), output_shader.frag:419, template.frag:98), so the
 * wire carries RGB only: rm_pack_rgb8 drops the alpha byte of npixels RGBA8
 * words; rm_deinterleave_rgb8 is rm_deinterleave_rgba8 over gathered rows of
 * 3*W bytes, restoring alpha 255.  Device pointers, ctx stream. */
rm_status rm_pack_rgb8(rm_ctx *ctx, int64_t npixels, const uint32_t *in, uint8_t *out);
rm_status rm_deinterleave_rgb8(rm_ctx *ctx, int W, int H, int band, int nshards, int rows_per_shard,
                               const uint8_t *gathered, uint32_t *out);

/* float RGBA -> RGBA8 unorm (round to nearest, clamped), device pointers. */
rm_status rm_pack_rgba8(rm_ctx *ctx, int64_t npixels, const float *in, uint32_t *out);

/* rm_render into a W*H RGBA8 target (device or host): the kernel packs each
 * pixel as rm_pack_rgba8 does (bit-identical to rm_render + rm_pack_rgba8),
 * writing 4 B/px instead of 16. */
rm_status rm_render_rgba8(rm_ctx *ctx, int W, int H, uint32_t *out, rm_stats *stats);

/* Progressive accumulation: the reference's ping-pong plumbing (main.cpp:192-207:
 * u_sample = the previous output texture, u_sample_part = 1/framesStill, fresh
 * u_seed1/u_seed2 per frame; common.frag:8-11), which its shaders declare but
 * never read, as a pass that reads it.  `accum` (W*H float4, or RGBA8 words for
 * the _rgba8 call; device or host) holds u_sample, the previous frame, and
 * receives mix(u_sample, colour, u_sample_part) per pixel, where the colour is
 * the pass's with the fragment moved by the sub-pixel offset fract(u_seed1) -
 * 0.5 (GLSL fract): with main.cpp's uniforms, accum is the running mean of the
 * jittered frames since the camera stopped (progressive supersampling).
 * u_sample_part >= 1 stores the colour (accum needs no clearing); with
 * u_seed1 = (0.5, 0.5) and u_sample_part = 1 the result is rm_render's /
 * rm_render_rgba8's, bit for bit. */
rm_status rm_render_accumulate(rm_ctx *ctx, int W, int H, float *accum, rm_stats *stats);
rm_status rm_render_accumulate_rgba8(rm_ctx *ctx, int W, int H, uint32_t *accum, rm_stats *stats);

/* rm_render_band / rm_render_rows into RGBA8 rows (W uint32 per row). */
rm_status rm_render_band_rgba8(rm_ctx *ctx, int W, int H, int band, int nshards, int shard, uint32_t *out,
                               rm_stats *stats);
rm_status rm_render_rows_rgba8(rm_ctx *ctx, int W, int H, int band, int nshards, int shard, int row_begin,
                               int row_count, uint32_t *out, rm_stats *stats);

/* The reference's FXAA post pass (post.frag:16-61, :135-144) over an RGBA8
 * frame: in/out W*H RGBA8 words (device, distinct), sampled as the reference's
 * RenderTexture is (nearest, clamp to edge), u_resolution = (W, H).  Like
 * post.frag, the output is the input flipped vertically.  W*H < 2^30. */
rm_status rm_fxaa(rm_ctx *ctx, int W, int H, const uint32_t *in, uint32_t *out);

/* The reference's bloom post pass (shaders/post/bloom.frag:14-43, applied by
 * PostBloom::apply, source/post_bloom.cpp:9-13, main.cpp:212-214) over an
 * RGBA8 frame: the mip levels bloom.frag's textureLod reads are built on the
 * device (glGenerateMipmap semantics, kept in a context scratch buffer), then
 * the 25-tap trilinear bloom is added to the frame; RGBA8 out, alpha 1.  As in
 * the shader, the output is flipped vertically (uv = (tc.x, 1 - tc.y)).
 * in/out: W x H device buffers, row 0 first, in != out.  Asynchronous on the
 * context's stream.  The scratch buffer also keeps the size's run tables
 *  between calls; they are rebuilt when W x H or the context's
 * stream changes.  The buffer is one per context: a bloom on another stream
 * than the last one first waits (on the device) for that one, marked when the
 * context left its stream. */
rm_status rm_bloom(rm_ctx *ctx, int W, int H, const uint32_t *in, uint32_t *out);

/* The reference's two post passes of a frame, chained as main.cpp:209-214 runs
 * them: FXAA of `in` into `mid` (post_shader into postTexture), then bloom of
 * `mid` into `out` (postTexture.generateMipmap, post_bloom.apply): the same
 * bits as rm_fxaa(in -> mid) followed by rm_bloom(mid -> out), in one call.
 * Device buffers of W x H RGBA8 words, pairwise distinct, W*H < 2^30;
 * asynchronous on the context's stream; bloom's scratch as rm_bloom's. */
rm_status rm_post_chain(rm_ctx *ctx, int W, int H, const uint32_t *in, uint32_t *mid, uint32_t *out);

/* The render kernels' code objects by content (16 hex digits of a SHA-256 of
 * the translation units that hold them): rocprofv3 counters of a render launch
 * (profiles/pmc_counters.json) name the build they counted, and bench.py
 * prices a launch with them only when this hash matches. */
const char *rm_render_code_hash(void);

/* ---- Weighted row parts: frame row y belongs to a part iff (y mod cycle) - offset
 * lies in [0, run).  Round-robin bands are the special case run = band,
 * cycle = band * nshards, offset = band * shard; parts with different runs give
 * ranks different shares of every cycle (bench.py's balanced multi-GPU split:
 * the root, which receives the others' rows, renders a longer run).
 * rm_cycle_rows: the number of frame rows of a part.  rm_render_cycle_rows[_rgba8]:
 * the part's packed rows [row_begin, row_begin + row_count) in increasing y,
 * as rm_render_rows[_rgba8].  rm_deinterleave_cycle_rgb8: the root side, the
 * W x H RGBA8 frame (alpha 255) from nparts parts that tile [0, cycle) in
 * order (offsets[i + 1] = offsets[i] + runs[i]), part i's packed 3 B/px rows
 * starting at byte part_bytes[i] of `gathered` (device pointers, ctx stream;
 * nparts <= 64). */
rm_status rm_cycle_rows(int H, int cycle, int offset, int run, int *nrows);
rm_status rm_render_cycle_rows(rm_ctx *ctx, int W, int H, int cycle, int offset, int run, int row_begin,
                               int row_count, float *out, rm_stats *stats);
rm_status rm_render_cycle_rows_rgba8(rm_ctx *ctx, int W, int H, int cycle, int offset, int run, int row_begin,
                                     int row_count, uint32_t *out, rm_stats *stats);
rm_status rm_deinterleave_cycle_rgb8(rm_ctx *ctx, int W, int H, int cycle, int nparts, const int *offsets,
                                     const int *runs, const int64_t *part_bytes, const uint8_t *gathered,
                                     uint32_t *out);

/* ---- Compressed wire of RGBA8 row parts ----
 * A lossless code per 8x8-pixel tile of a part's packed rows: the first
 * pixel, then per channel the differences to the left neighbour (to the one
 * above in the tile's first column) as bit planes of their zig-zagged bytes;
 * alpha is not sent (the root stores 255).  rm_wire_encode: nrows packed
 * RGBA8 rows -> msg (at most rm_wire_capacity bytes), using a caller-owned
 * device workspace of rm_wire_workspace_bytes; the message size (also its
 * first 8 bytes) is written to the device int64 *size_out when non-null
 * (asynchronous, ctx stream).  rm_wire_decode: a message of nrows rows of the
 * cyclic part (cycle, offset, run) into those rows of the W x H RGBA8 frame.
 * rm_scatter_part_rgba8: a part's packed RGBA8 rows into their frame rows
 * (the root's own part).  Capacity/workspace return -1 for bad sizes
 * (W <= 2^18). */
int64_t rm_wire_capacity(int W, int nrows);
int64_t rm_wire_workspace_bytes(int W, int nrows);
rm_status rm_wire_encode(rm_ctx *ctx, int W, int nrows, const uint32_t *rows, uint8_t *msg, void *workspace,
                         int64_t *size_out);
rm_status rm_wire_decode(rm_ctx *ctx, int W, int H, int cycle, int offset, int run, int nrows, const uint8_t *msg,
                         uint32_t *frame);
rm_status rm_scatter_part_rgba8(rm_ctx *ctx, int W, int H, int cycle, int offset, int run, int nrows,
                                const uint32_t *rows, uint32_t *frame);
/* rm_wire_decode for nparts (<= 64) messages in one launch: part i holds
 * nrows[i] rows of (cycle, offsets[i], runs[i]); msgs is a host array of
 * device pointers. */
rm_status rm_wire_decode_parts(rm_ctx *ctx, int W, int H, int cycle, int nparts, const int *offsets, const int *runs,
                               const int *nrows, const uint8_t *const *msgs, uint32_t *frame);

/* rm_render_cycle_rows_rgba8 and rm_wire_encode in one: the render kernel
 * encodes each of its 8x8-pixel tiles for the wire from registers (its own
 * epilogue: the rows are never written), then the tiles' words are scanned
 * and compacted into msg; msg, workspace and *size_out as rm_wire_encode's for
 * row_count rows, and the message is byte for byte rm_wire_encode's of the
 * rows rm_render_cycle_rows_rgba8 renders.  Built-in scenes (a plugin part:
 * the two calls).  The non-root ranks of a sharded frame call this instead of
 * rendering rows they only send. */
rm_status rm_render_cycle_rows_wire(rm_ctx *ctx, int W, int H, int cycle, int offset, int run, int row_begin,
                                    int row_count, uint8_t *msg, void *workspace, int64_t *size_out, rm_stats *stats);

/* ---- Multi-GPU: row-sharded frames over RCCL ----
 * The reference renders one frame on one GPU (main.cpp:196-207); here a frame's
 * rows are dealt to nranks GPUs in bands of `band` rows, round robin (rank r
 * owns frame row y iff (y / band) % nranks == r).  Each rank renders its rows
 * (rm_render_band_rgba8), packs them to the 3 B/px RGB8 wire (rm_pack_rgb8),
 * one ncclGather moves every wire to rank 0 over xGMI, and rank 0 writes the
 * W x H RGBA8 frame (rm_deinterleave_rgb8).  RCCL (librccl.so.1) is opened at
 * run time.  A communicator binds a context (its device, stream, scene and
 * uniforms: set the same uniforms on every rank's context).
 *
 * One process per GPU: rank 0 calls rm_comm_get_id and sends the id to the
 * others out of band (ncclGetUniqueId semantics), then every rank calls
 * rm_comm_init_rank (collective) and rm_render_sharded per frame (collective;
 * `frame` is a W*H RGBA8 device buffer on rank 0, ignored elsewhere).
 * One process driving n GPUs: rm_comm_init_all over n contexts on distinct
 * devices (ncclCommInitAll; comms[i] is rank i), then rm_render_sharded_all.
 * Calls are asynchronous on the contexts' streams unless `stats` is given
 * (then they wait; stats[i].kernel_ms is rank i's render time, gather_ms its
 * pack + gather and, on rank 0, deinterleave_ms the de-interleave kernel). */
typedef struct rm_comm rm_comm;
typedef struct rm_comm_id {
    char internal[128]; /* an ncclUniqueId */
} rm_comm_id;
/* The layout rm_render_sharded uses (host-only, no GPU): rank `rank` owns
 * rows_mine frame rows; every rank sends rows_per_shard rows of 3*W bytes
 * (wire_bytes; rows past rows_mine are padding); rank 0 receives nranks wires
 * back to back (gathered_bytes), rank r's at offset r * wire_bytes. */
typedef struct rm_shard_layout {
    int32_t rows_mine, rows_per_shard;
    int64_t wire_bytes, gathered_bytes;
} rm_shard_layout;
rm_status rm_sharded_layout(int W, int H, int band, int nranks, int rank, rm_shard_layout *out);
rm_status rm_comm_get_id(rm_comm_id *id);
rm_status rm_comm_init_rank(rm_comm **comm, rm_ctx *ctx, int nranks, const rm_comm_id *id, int rank);
rm_status rm_comm_init_all(rm_comm **comms, rm_ctx *const *ctxs, int n);
rm_status rm_comm_destroy(rm_comm *comm);
/* uses_rccl = 1 when the communicator runs RCCL (always for nranks > 1; a
 * one-rank communicator too whenever librccl loads, else a local copy). */
rm_status rm_comm_info(const rm_comm *comm, int *nranks, int *rank, int *uses_rccl);
rm_status rm_render_sharded(rm_comm *comm, int W, int H, int band, uint32_t *frame, rm_stats *stats);
rm_status rm_render_sharded_all(rm_comm *const *comms, int n, int W, int H, int band, uint32_t *frame,
                                rm_stats *stats);
/* The same with weighted parts instead of bands: runs[r] >= 1 rows of every
 * cycle of sum(runs) rows go to rank r, in rank order (rm_cycle_rows); the
 * parts cross the wire unpadded (grouped ncclSend/ncclRecv) and rank 0
 * rebuilds the frame with rm_deinterleave_cycle_rgb8.  Every rank passes the
 * same runs (nranks entries). */
rm_status rm_render_sharded_runs(rm_comm *comm, int W, int H, const int *runs, uint32_t *frame, rm_stats *stats);
rm_status rm_render_sharded_runs_all(rm_comm *const *comms, int n, int W, int H, const int *runs, uint32_t *frame,
                                     rm_stats *stats);

/* Message of the last failing call on ctx ("" if none). */
const char *rm_last_error(rm_ctx *ctx);
const char *rm_status_string(rm_status status);

#ifdef __cplusplus
}
#endif

#endif /* RM_H_ */
