// rm_capi.cpp -- the C ABI declared in include/rm.h.
//
// Owns the per-context state the reference keeps inside sf::Shader (uniform
// values, the loaded scene) and turns it into the per-frame constant block the
// kernels read (rm_device.h FrameConst).  Compiled with -ffp-contract=off so
// that the host-side per-frame constants (sin/cos of the camera and sponge
// rotations, the Hash11 table) are computed with the same roundings as the
// GLSL expressions they hoist.
#include "../../include/rm.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <set>
#include <string>
#include <vector>

#include "rm_internal.h"
#include "rm_launch.h"
#include "rm_plugin_host.h"
#include "rm_trace.h"

using rm::FrameConst;

struct rm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int scene = -1;
    std::string scene_file;
    // uniforms (common.frag:4-11)
    float res[2] = {0.0f, 0.0f};
    bool res_set = false;
    float pos[3] = {0.0f, 0.0f, 0.0f};
    float mouse[2] = {0.0f, 0.0f};
    float time = 0.0f;
    // KERNEL_PERSIST: blocks of self-resetting tile counters, one per stream
    // the context launches on (launches on one stream run one after another, so
    // a block is never shared by two launches in flight).  At most kPersistBlocks:
    // a new stream takes the least recently used block once the event recorded
    // after its last launch has completed (the launch left its counters zeroed).
    struct PersistBlock {
        hipStream_t stream = nullptr;
        uint32_t *ctr = nullptr;
        hipEvent_t last = nullptr;
        uint64_t used = 0;
    };
    static constexpr int kPersistBlocks = 4;
    std::vector<PersistBlock> persist;
    // work this context enqueued: `dirty` is set by each call that enqueues
    // on `stream`; `done` is recorded on the stream only when the context
    // leaves it (rm_set_stream) or is destroyed -- an event recorded after
    // every launch cost a ~11 us gap between consecutive frames on the stream
    // (DESIGN.md 2.14).  A left stream's event stays in `retired` until it
    // completes (rm_destroy waits for these, not the
    // whole device).
    hipEvent_t done = nullptr;
    bool dirty = false;
    std::vector<hipEvent_t> retired;
    // streams bound with rm_set_stream_kept (the caller keeps them alive until
    // rm_destroy): leaving one records nothing; it joins `owed`, and its work
    // is marked only when something waits for it (an entry's release,
    // rm_destroy), on the stream itself
    std::vector<hipStream_t> kept, owed;
    float sample_part = 1.0f;  // u_sample_part, u_seed1, u_seed2: read by rm_render_accumulate*
    float seed1[2] = {0.0f, 0.0f}, seed2[2] = {0.0f, 0.0f};
    rm_params params = {128, 0, 0, 0, 1};
    std::string err;
    std::set<std::string> warned;
    unsigned long long *d_evals = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    float4 *staging = nullptr;
    size_t staging_bytes = 0;
    uint32_t *mips = nullptr;  // bloom's mip levels 1..d2
    size_t mips_texels = 0;
    int bloom_runs_w = 0, bloom_runs_h = 0;  // the size whose bloom run tables `mips` holds (0: none)
    hipStream_t bloom_runs_stream = nullptr;
    // the scratch buffer is shared by the context's streams: when the context
    // leaves the stream of its last bloom / post chain (bloom_stream), bloom_ev
    // is recorded there, and a bloom on another stream first waits for it (no
    // marker per frame; one per leave, and only after a bloom)
    hipEvent_t bloom_ev = nullptr;
    hipStream_t bloom_stream = nullptr;
    bool bloom_pending = false;  // a bloom ran on bloom_stream since bloom_ev was last recorded
    rmplugin::Module plugin;  // the loaded scene plugin (scene == SCENE_PLUGIN)
    uint32_t *tile_order = nullptr;  // rm_set_tile_order (device copy)
    int64_t tile_order_n = 0;
    // adaptive dispatch order (rm_params.schedule): per launch geometry and
    // stream, the tile durations of the last launch and the order they give
    // Every sched_period()-th launch of a geometry (L_s = s * period, s = 0, 1,
    // ...) writes its tile durations into cost[s & 1]; sort s of those
    // durations runs right after it on the same stream and writes order[s & 1],
    // which launches L_s + 1 .. L_{s+1} dispatch.  The other launches write no
    // durations.  (Round 2-4 sorted on a side stream, overlapping the next
    // launch: its kernels only got CUs as that launch drained, and the launch
    // after it waited ~45 us for them)
    struct Sched {
        uint64_t key = 0;
        hipStream_t stream = nullptr;
        int n = 0, gx = 0;         // tiles, tile-grid width
        uint64_t k = 0;            // launches so far
        uint32_t *buf = nullptr;   // cost[2][n] | order[2][n] | 2 x (hist[256] | cursor[256]) | bucket u8[n]
        hipEvent_t last = nullptr;  // after the last launch that read or wrote buf: recorded on `stream`
        bool dirty = false;         // when the entry is released or the context destroyed on `stream`
        // ... or, once the context has left `stream`, the `done` event recorded
        // there as it left (borrowed: one marker per leave instead of one per
        // entry as well; rm_destroy destroys it after the entries are released)
        hipEvent_t left = nullptr;
        uint64_t used = 0;
        size_t bytes = 0;  // buf's size
    };
    Sched sched[8];
    uint64_t sched_clock = 0;
    // buffers of evicted adaptive-order entries, each with the marker of its
    // last use (ev: owned, or a borrowed `done` event); reused by a new entry
    // once the marker has completed, instead of a host wait at the eviction
    // (a marker recorded then on a kept stream covers everything queued there
    // since, e.g. the next pipelined frame)
    struct Spare {
        uint32_t *buf = nullptr;
        size_t bytes = 0;
        hipEvent_t ev = nullptr;
        bool own = false;
    };
    std::vector<Spare> spare;
};

namespace {

rm_status fail(rm_ctx *c, rm_status s, const std::string &msg) {
    if (c) c->err = msg;
    return s;
}

rm_status hip_fail(rm_ctx *c, hipError_t e, const char *what) {
    return fail(c, e == hipErrorOutOfMemory ? RM_ERR_OUT_OF_MEMORY : RM_ERR_DEVICE,
                std::string(what) + ": " + hipGetErrorString(e));
}

#define RM_HIP(call)                                          \
    do {                                                      \
        hipError_t e_ = (call);                               \
        if (e_ != hipSuccess) return hip_fail(ctx, e_, #call); \
    } while (0)

// Note that the context enqueued work on its stream (rm_ctx::dirty).
bool is_kept(const rm_ctx *ctx, hipStream_t s) {
    for (hipStream_t k : ctx->kept)
        if (k == s) return true;
    return false;
}

rm_status mark_done(rm_ctx *ctx) {
    ctx->dirty = true;
    return RM_OK;
}

// Record the adaptive-order entries' `last` events still owed on the ctx
// stream or on a kept stream (before the context is destroyed).
hipError_t record_sched_last(rm_ctx *ctx) {
    for (rm_ctx::Sched &e : ctx->sched)
        if (e.buf && e.dirty && (e.stream == ctx->stream || is_kept(ctx, e.stream))) {
            hipError_t r = hipEventRecord(e.last, e.stream);
            if (r != hipSuccess) return r;
            e.dirty = false;
            e.left = nullptr;
        }
    return hipSuccess;
}

// The KERNEL_PERSIST counter block of the ctx stream (rm_ctx::PersistBlock).
// A new block joins ctx->persist only once its event and counters exist (a
// half-built block would match the null stream with a null counter array).
rm_status persist_block(rm_ctx *ctx, rm_ctx::PersistBlock *&out) {
    out = nullptr;
    for (auto &b : ctx->persist)
        if (b.stream == ctx->stream) out = &b;
    if (!out && (int)ctx->persist.size() < rm_ctx::kPersistBlocks) {
        rm_ctx::PersistBlock b{};
        const size_t bytes = (size_t)rm::kPersistWords * sizeof(uint32_t);
        RM_HIP(hipEventCreateWithFlags(&b.last, hipEventDisableTiming));
        hipError_t e = hipMalloc(&b.ctr, bytes);
        if (e == hipSuccess) e = hipMemsetAsync(b.ctr, 0, bytes, ctx->stream);
        if (e != hipSuccess) {
            if (b.ctr) (void)hipFree(b.ctr);
            (void)hipEventDestroy(b.last);
            return hip_fail(ctx, e, "persist_block: counter block");
        }
        b.stream = ctx->stream;
        ctx->persist.push_back(b);
        out = &ctx->persist.back();
    }
    if (!out) {  // recycle the least recently used block once its last launch is done
        out = &ctx->persist[0];
        for (auto &b : ctx->persist)
            if (b.used < out->used) out = &b;
        RM_HIP(hipEventSynchronize(out->last));
        out->stream = ctx->stream;
    }
    out->used = ++ctx->sched_clock;  // per-context LRU clock (shared with the sched entries)
    return RM_OK;
}

// ShaderLoader::preprocess (source/shader_loader.cpp:22-81): read the file
// line by line; a line holding "#include" not preceded by "//" pulls in the
// file named between "" or <> (path relative to the process CWD, no include
// guards).  Returns false with the reference's message on a missing file.
bool preprocess(const std::string &file, std::string &out, std::string &err, int depth = 0) {
    if (depth > 64) {
        err = "ShaderLoader: #include nesting too deep at \"" + file + "\"";
        return false;
    }
    std::ifstream f(file);
    if (!f.is_open()) {
        err = "ShaderLoader: can't load file \"" + file + "\"";
        return false;
    }
    std::string line;
    while (std::getline(f, line)) {
        // text-mode reading as on the reference's platform (MSVC's fstream
        // turns CRLF into LF): without it the '\r' after a closing quote would
        // join the include name, since the name loop below re-opens on it
        if (!line.empty() && line.back() == '\r') line.pop_back();
        size_t found = line.find("#include");
        if (found != std::string::npos && (found == 0 || line.rfind("//", found) == std::string::npos)) {
            std::string name;
            bool reading = false;
            for (size_t i = found + 8; i < line.size(); i++) {
                char ch = line[i];
                if (ch == '"' || ch == '<') reading = true;
                else if (reading) {
                    if (ch == '"' || ch == '>') reading = false;
                    else name += ch;
                }
            }
            if (!preprocess(name, out, err, depth + 1)) return false;
            continue;
        }
        out += line + '\n';
    }
    return true;
}

std::string base_name(const std::string &p) {
    size_t k = p.find_last_of("/\\");
    return k == std::string::npos ? p : p.substr(k + 1);
}

int scene_of(const std::string &name) {
    if (name == "output_shader.frag" || name == "O") return rm::SCENE_O;
    if (name == "template.frag" || name == "T") return rm::SCENE_T;
    if (name == "sphere" || name == "sphere.frag" || name == "S0") return rm::SCENE_S0;
    if (name == "output_shader_glass" || name == "output_shader_glass.frag" || name == "OG") return rm::SCENE_OG;
    return -1;
}

bool is_plugin_source(const std::string &file) {
    return file.size() > 4 && file.compare(file.size() - 4, 4, ".hip") == 0;
}

inline float fract(float x) { return x - std::floor(x); }

// output_shader.frag:54-59
float hash11(float p) {
    float a = fract(p * 443.897f);
    float x = a, y = a, z = a;
    float dd = x * (y + 19.19f) + y * (z + 19.19f) + z * (x + 19.19f);
    x += dd; y += dd; z += dd;
    return fract((x + y) * z);
}

// (sampleDir * Hash11(i)).y of CalculateThickness (output_shader.frag:75-109)
// at a normal (0, ny, 0): Hash33 (:61-66), GenerateSampleVector, reflectVector
// (:70-80) in GLSL float semantics (no contraction; normalize = x * (1/length))
float sss_floor_term(float ny, int i) {
    const float fi = (float)i, nx = -0.0f, nyn = -ny, nz = -0.0f;  // -norm
    float x = fract((nx + fi) * 443.897f), y = fract((nyn + fi) * 441.423f), z = fract((nz + fi) * 437.195f);
    const float dd = x * (y + 19.19f) + y * (x + 19.19f) + z * (z + 19.19f);  // dot(p3, p3.yxz + 19.19)
    x += dd; y += dd; z += dd;
    const float hx = fract((x + y) * z) - 0.5f, hy = fract((x + x) * y) - 0.5f, hz = fract((y + x) * x) - 0.5f;
    const float r = 1.0f / std::sqrt(hx * hx + hy * hy + hz * hz);
    const float rx = hx * r, ry = hy * r, rz = hz * r;
    const float d = rx * nx + ry * nyn + rz * nz;
    const float dir_y = ry - (nyn * 2.0f) * (d < 0.0f ? d : 0.0f);
    return dir_y * hash11(fi);
}

// ---- scene files of registered names (the reference's "Reload scene shader",
// main.cpp:134-139, recompiles the edited output_shader.frag).  The text is
// classified by whitespace-insensitive FNV-1a 64 fingerprints of the
// reference's files (tools/ref_hashes.py; no reference text is kept):
//   output_shader.frag = prelude (up to the common.frag include) + scene part
//   (materials, floorMat, sceneSDF) + pipeline (hashes, light, render, main).
//   Reference prelude/pipeline and library: the scene part is the reference's
//   -> compiled-in scene O; an edited scene part -> compiled with hiprtc as a
//   scene plugin into output_shader.frag's pipeline.  An edited pipeline or
//   common.frag -> RM_ERR_SCENE (only the scene is re-definable).
//   template.frag: the reference's text -> scene T (repaired),
//   anything else -> RM_ERR_SCENE.
constexpr uint64_t kRefCommon = 0xac76e617a4f8cf8fULL;
constexpr uint64_t kRefTemplate = 0x39cf0bb021dfa9b7ULL;
constexpr uint64_t kRefOScene = 0x0b0b0c101eafdcf6ULL;
constexpr uint64_t kRefOFrame = 0x9ebf2dc8811b1dc0ULL;

uint64_t fingerprint(const std::string &t, uint64_t h = 0xcbf29ce484222325ULL) {
    for (unsigned char c : t) {
        if (c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\v' || c == '\f') continue;
        h ^= c;
        h *= 0x100000001b3ULL;
    }
    return h;
}

bool read_file(const std::string &f, std::string &out) {
    std::ifstream in(f, std::ios::binary);
    if (!in.is_open()) return false;
    out.assign(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
    return true;
}

// prelude / scene / pipeline of an output_shader.frag-shaped text
// (tools/ref_hashes.py split_scene); include_name = the first #include's file
bool split_scene(const std::string &t, std::string &prelude, std::string &scene, std::string &pipeline,
                 std::string &include_name) {
    size_t k = t.find("#include");
    if (k == std::string::npos) return false;
    size_t e = t.find('\n', k);
    e = e == std::string::npos ? t.size() : e + 1;
    size_t a = t.find_first_of("\"<", k), b = a == std::string::npos ? a : t.find_first_of("\">", a + 1);
    if (a == std::string::npos || b == std::string::npos || b > e) return false;
    include_name = t.substr(a + 1, b - a - 1);
    size_t s = t.find("sceneSDF(", e);
    s = s == std::string::npos ? s : t.find('{', s);
    if (s == std::string::npos) return false;
    int depth = 0;
    for (size_t i = s; i < t.size(); i++) {
        if (t[i] == '{') depth++;
        else if (t[i] == '}' && --depth == 0) {
            prelude = t.substr(0, e);
            scene = t.substr(e, i + 1 - e);
            pipeline = t.substr(i + 1);
            return true;
        }
    }
    return false;
}

bool is_device_ptr(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

// Workgroups at the head of an ordered launch that render scene T with the
// latency-optimized folds (FrameConst.lat_tiles) ...
constexpr int kLatTiles = 2048;
// ... in launches short enough for their tail to show: a rank's share, a 1080p
// frame.  The C4 share at N = 8 (32768 tiles) takes 0.077 ms per pipelined
// frame with them and 0.098 without; a whole 4096^2 frame (262144 tiles) runs
// 0.4 % faster without them, an N = 2 half frame (131072) the same either way
// (profiles/r05/knob_lat_r05.log, lat_share_r05.jsonl): launches of more tiles
// than this take none.
constexpr int64_t kLatMaxTiles = 98304;
int lat_tiles_for(int kernel, int W, int nrows) {
    const rm::TileGrid g = rm::tile_grid(kernel, W, nrows);
    return (int64_t)g.x * g.y <= kLatMaxTiles ? kLatTiles : 0;
}

// Launches per dispatch-order sort of a geometry (rm_ctx::Sched): 16 -- an
// order is at most 17 launches old (frame-to-frame coherence keeps it good, the
// dilated key covers a moving camera), and the duration stores, the sort and
// the cross-stream events run on one launch in sixteen.  Round 2 chose 4 (C3
// frame 0.683 -> 0.672 ms against 1); after the round-3 skips the frame is
// shorter and 8 measured 0.7 % (still) and 1.8 % (walking) faster than 4, 16
// the same as 8 (profiles/r03/sched_period_after_skips.jsonl).
// Round 4 sorts on the frame's stream (21 us per sort in the frame's time):
// 16 measured 0.3-0.7 % faster than 8 still, walking and at P1, 4 slower
// (profiles/r04/sched_knobs_final_ab.log, sched_period_walk_p1_ab.log).
constexpr int kSchedPeriod = 16;
int sched_period() { return kSchedPeriod; }

// Dilation radius (tiles) of the sort key (rm_kernels.hip tile_key): 2.  With
// a moving camera (bench.py --walk) the costly regions move between the launch
// that measured the durations and the launches that use the order:
// undilated, C3 walks at 0.457 ms per frame against row-major's 0.440; radius
// 2 0.439, with the still pose unchanged (0.583 ms, row-major 0.633); radius 4
// 0.437 walking but 0.589 still (profiles/r03/sched_walk_dilate.jsonl, DESIGN.md
// 2.6).
constexpr int kSchedDilate = 2;
int sched_dilate() { return kSchedDilate; }

// The frame rows one launch renders: y with (y mod cycle) - offset in [0, run)
// (round-robin bands: run = band, cycle = band * nshards, offset = band * shard).
struct RowPart {
    int cycle, offset, run;
};
// validated row part of round-robin bands, or of an explicit cyclic part
bool band_part(int band, int nshards, int shard, RowPart &p) {
    if (band <= 0 || nshards <= 0 || shard < 0 || shard >= nshards || (long long)band * nshards > 0x7fffffffLL) return false;
    p = RowPart{band * nshards, band * shard, band};
    return true;
}
bool cycle_part(int cycle, int offset, int run, RowPart &p) {
    if (cycle <= 0 || offset < 0 || run <= 0 || (long long)offset + run > cycle) return false;
    p = RowPart{cycle, offset, run};
    return true;
}
int rows_of_part(int H, const RowPart &p) {
    const long long full = H / p.cycle, rest = H - full * p.cycle;
    long long tail = rest - p.offset;
    tail = tail < 0 ? 0 : tail > p.run ? p.run : tail;
    return (int)(full * p.run + tail);
}

int pick_kernel(const rm_ctx *c);

FrameConst frame_const(const rm_ctx *c, int W, int H, const RowPart &part, int nrows) {
    FrameConst F;
    std::memset(&F, 0, sizeof(F));
    F.res_x = c->res_set ? c->res[0] : (float)W;
    F.res_y = c->res_set ? c->res[1] : (float)H;
    F.pos_x = c->pos[0]; F.pos_y = c->pos[1]; F.pos_z = c->pos[2];
    // rot(a) = mat2(cos a, -sin a, sin a, cos a) (common.frag:1088-1092)
    float a1 = -c->mouse[1], a2 = c->mouse[0];
    F.cam1_c = rm::glsl_cos(a1); F.cam1_s = rm::glsl_sin(a1);
    F.cam2_c = rm::glsl_cos(a2); F.cam2_s = rm::glsl_sin(a2);
    // transformR(.., vec3(180, u_time * 2, 0)): rotationY(-rot.y), rotationX(-rot.x)
    // with radians(x) = x * pi/180 (common.frag:190-214,434-441)
    float rot_y = c->time * 2.0f, rot_x = 180.0f;
    float ay = -rot_y * 0.017453292519943295f, ax = -rot_x * 0.017453292519943295f;
    F.ry_c = rm::glsl_cos(ay); F.ry_s = rm::glsl_sin(ay);
    F.rx_c = rm::glsl_cos(ax); F.rx_s = rm::glsl_sin(ax);
    F.W = W; F.H = H;
    F.cycle = part.cycle; F.offset = part.offset; F.run = part.run; F.nrows = nrows;
    F.run_magic = rm::div_magic((uint32_t)part.run, (uint64_t)H + 1);  // packed rows j < H
    F.time = c->time;
    F.mouse_x = c->mouse[0];
    F.mouse_y = c->mouse[1];
    F.max_steps = c->params.max_steps;
    // 0 (unbounded, the reference) travels as INT_MAX: one compare per shadow step
    F.shadow_max_steps = c->params.shadow_max_steps > 0 ? c->params.shadow_max_steps : 0x7fffffff;
    F.lat_tiles = lat_tiles_for(pick_kernel(c), W, nrows);
    for (int i = 0; i < 32; i++) {
        F.hash11[i] = hash11((float)i);
        F.sss_floor[0][i] = sss_floor_term(1.0f, i);
        F.sss_floor[1][i] = sss_floor_term(0x1.fffffep-1f, i);
    }
    return F;
}

int rows_of_shard(int H, int band, int nshards, int shard) {
    RowPart p;
    return band_part(band, nshards, shard, p) ? rows_of_part(H, p) : 0;
}

rm_status ensure_staging(rm_ctx *ctx, size_t bytes) {
    if (ctx->staging_bytes >= bytes) return RM_OK;
    if (ctx->staging) (void)hipFree(ctx->staging);
    ctx->staging = nullptr;
    ctx->staging_bytes = 0;
    RM_HIP(hipMalloc(&ctx->staging, bytes));
    ctx->staging_bytes = bytes;
    return RM_OK;
}

// rm_params.kernel: 0 auto, 1 = 16x16-pixel workgroups, 2 = 8x8-pixel workgroups
int pick_kernel(const rm_ctx *c) {
    if (c->params.kernel == 1) return rm::KERNEL_TILE16;
    if (c->params.kernel == 3) return rm::KERNEL_TILE16X4;
    if (c->params.kernel == 4) return rm::KERNEL_PERSIST;
    return rm::KERNEL_TILE8;  // 0 auto, 2: measured fastest on every config
}

// Free an adaptive-order entry once nothing still reads or writes its buffers:
// its last launch (an event: the stream it ran on may belong to the caller and
// be gone by now) and the context's own sort stream.
hipError_t sched_release(rm_ctx *ctx, rm_ctx::Sched &e) {
    hipError_t r = hipSuccess;
    if (e.buf) {
        if (e.dirty && (e.stream == ctx->stream || is_kept(ctx, e.stream))) {
            r = hipEventRecord(e.last, e.stream);
            if (r == hipSuccess) r = hipEventSynchronize(e.last);
        } else if (e.left) {
            // the context left e.stream after e's last launch: the marker
            // recorded then (a `done` event, re-recorded later only once it had
            // completed, so a wait on it never returns early)
            r = hipEventSynchronize(e.left);
        } else if (e.last) {
            r = hipEventSynchronize(e.last);
        }
        (void)hipFree(e.buf);
    }
    if (e.last) (void)hipEventDestroy(e.last);
    e = rm_ctx::Sched();
    return r;
}

void spare_free(rm_ctx::Spare &sp) {
    if (sp.ev) (void)hipEventSynchronize(sp.ev);
    (void)hipFree(sp.buf);
    if (sp.own && sp.ev) (void)hipEventDestroy(sp.ev);
    sp = rm_ctx::Spare();
}

// Evict an entry without a host wait: its buffer joins ctx->spare with the
// marker of its last use (sched_release's three cases, recorded or borrowed).
hipError_t sched_retire(rm_ctx *ctx, rm_ctx::Sched &e, size_t bytes) {
    if (!e.buf) return sched_release(ctx, e);
    rm_ctx::Spare sp{e.buf, bytes, nullptr, false};
    if (e.dirty && (e.stream == ctx->stream || is_kept(ctx, e.stream))) {
        hipError_t r = hipEventRecord(e.last, e.stream);
        if (r != hipSuccess) return sched_release(ctx, e);
        sp.ev = e.last, sp.own = true;
    } else if (e.left) {
        sp.ev = e.left;  // (borrowed: destroyed by rm_destroy, after the spares)
        if (e.last) (void)hipEventDestroy(e.last);
    } else {
        sp.ev = e.last, sp.own = true;
    }
    if (ctx->spare.size() >= 8) {  // bounded: the oldest is freed (a host wait, rare)
        spare_free(ctx->spare.front());
        ctx->spare.erase(ctx->spare.begin());
    }
    ctx->spare.push_back(sp);
    e = rm_ctx::Sched();
    return hipSuccess;
}

// A spare buffer of at least `bytes` whose last use has completed, or null.
uint32_t *spare_take(rm_ctx *ctx, size_t bytes, size_t &got) {
    for (size_t i = 0; i < ctx->spare.size(); i++) {
        rm_ctx::Spare &sp = ctx->spare[i];
        if (sp.bytes < bytes || (sp.ev && hipEventQuery(sp.ev) != hipSuccess)) continue;
        uint32_t *b = sp.buf;
        got = sp.bytes;
        if (sp.own && sp.ev) (void)hipEventDestroy(sp.ev);
        ctx->spare.erase(ctx->spare.begin() + (long)i);
        (void)hipGetLastError();  // hipEventQuery's hipErrorNotReady
        return b;
    }
    (void)hipGetLastError();
    return nullptr;
}

// The adaptive-order state of a launch geometry on the ctx stream (least
// recently used entry recycled), or null when scheduling does not apply.
rm_ctx::Sched *sched_slot(rm_ctx *ctx, int W, int H, const RowPart &part, int row0, int count, rm_status &st) {
    st = RM_OK;
    // plugins always launch one-wave 8x8 tiles (rm_plugin_kernels.h)
    if (!ctx->params.schedule ||
        (ctx->scene != rm::SCENE_PLUGIN && pick_kernel(ctx) != rm::KERNEL_TILE8 && pick_kernel(ctx) != rm::KERNEL_PERSIST))
        return nullptr;
    const rm::TileGrid g = rm::tile_grid(rm::KERNEL_TILE8, W, count);
    const int n = g.x * g.y;
    uint64_t key = 0xcbf29ce484222325ULL;
    for (long long v : {(long long)ctx->scene, (long long)W, (long long)H, (long long)part.cycle, (long long)part.offset,
                        (long long)part.run, (long long)row0, (long long)count})
        key = (key ^ (uint64_t)v) * 0x100000001b3ULL;
    rm_ctx::Sched *lru = &ctx->sched[0];
    for (rm_ctx::Sched &e : ctx->sched) {
        if (e.buf && e.key == key && e.stream == ctx->stream && e.n == n) {
            e.used = ++ctx->sched_clock;
            return &e;
        }
        if (e.used < lru->used) lru = &e;
    }
    hipError_t e = hipSuccess;
    // cost[2][n] | order[2][n] | 2 x (hist | cursor) | bucket bytes[n]
    const size_t need = ((size_t)4 * n + 1024 + ((size_t)n + 3) / 4) * sizeof(uint32_t);
    e = sched_retire(ctx, *lru, lru->bytes);
    size_t got = 0;
    if (e == hipSuccess && (lru->buf = spare_take(ctx, need, got)) == nullptr) {
        e = hipMalloc(&lru->buf, need);
        got = need;
    }
    lru->bytes = got;
    if (e == hipSuccess) e = hipMemsetAsync(lru->buf + 4 * (size_t)n, 0, 1024 * sizeof(uint32_t), ctx->stream);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&lru->last, hipEventDisableTiming);
    if (e != hipSuccess) {
        (void)sched_release(ctx, *lru);
        st = hip_fail(ctx, e, "schedule buffers");
        return nullptr;
    }
    lru->key = key;
    lru->stream = ctx->stream;
    lru->n = n;
    lru->gx = g.x;
    lru->used = ++ctx->sched_clock;
    return lru;
}

// rm_render_cycle_rows_wire: the compressed wire's message instead of pixels
// (`out` is then the tile-slot workspace, rm_wire_tile.h)
struct WireOut {
    uint8_t *msg;
    long long *size_out;
};

rm_status render_dev(rm_ctx *ctx, int W, int H, const RowPart &part, int row0, int count, void *out, bool rgba8,
                     rm_stats *stats, uint32_t *evmap = nullptr, bool accum = false, const WireOut *wire = nullptr) {
    rm::TraceRange range("rm_render");
    // the wire's tile code runs in one-wave 8x8 tiles (rm_render_direct.h)
    const int kernel = wire ? (int)rm::KERNEL_TILE8 : pick_kernel(ctx);
    FrameConst F = frame_const(ctx, W, H, part, count);
    F.row0 = row0;
    F.evals_map = evmap;
    if (accum) {  // fract(u_seed1) - 0.5 (GLSL fract, x - floor(x)), per frame
        F.accumulate = 1;
        F.sample_part = ctx->sample_part;
        F.jit_x = (ctx->seed1[0] - std::floor(ctx->seed1[0])) - 0.5f;
        F.jit_y = (ctx->seed1[1] - std::floor(ctx->seed1[1])) - 0.5f;
    }
    rm_ctx::Sched *sc = nullptr;
    if (ctx->tile_order) {  // an explicit order wins
        const rm::TileGrid g = rm::tile_grid(ctx->scene == rm::SCENE_PLUGIN ? (int)rm::KERNEL_TILE8 : kernel, W, count);
        if ((int64_t)g.x * g.y == ctx->tile_order_n) F.tile_order = ctx->tile_order;
    } else {
        rm_status st;
        sc = sched_slot(ctx, W, H, part, row0, count, st);
        if (st != RM_OK) return st;
        if (sc) {
            const uint64_t P = (uint64_t)sched_period(), k = sc->k;
            // an instrumented launch (count_evals, step maps) takes every reference
            // step, so its tile durations would rank the tiles by work the timed
            // kernels skip: it uses the current order but records no durations and
            // does not advance the geometry's launch count
            if (k % P == 0 && !(ctx->params.count_evals != 0 || evmap))
                F.tile_cost = sc->buf + ((k / P) & 1) * sc->n;  // sort k / P reads them
            if (k >= 1) {  // the newest sort's order (it ran right after launch s * P, same stream)
                const uint64_t s = (k - 1) / P;
                F.tile_order = sc->buf + (2 + (s & 1)) * sc->n;
            }
        }
    }
    rm_ctx::PersistBlock *pb = nullptr;
    if (ctx->scene != rm::SCENE_PLUGIN && kernel == rm::KERNEL_PERSIST) {
        // this stream's counters, zeroed once; each launch leaves them zeroed
        rm_status st = persist_block(ctx, pb);
        if (st != RM_OK) return st;
        F.persist = pb->ctr;
    }
    bool cnt = ctx->params.count_evals != 0 || evmap;
    if (cnt) RM_HIP(hipMemsetAsync(ctx->d_evals, 0, 3 * sizeof(unsigned long long), ctx->stream));
    if (stats) RM_HIP(hipEventRecord(ctx->ev0, ctx->stream));
    hipError_t e =
        wire ? rm::launch_render_wire(ctx->scene, F, static_cast<rm::WireTile *>(out), cnt ? ctx->d_evals : nullptr,
                                      ctx->stream)
        : ctx->scene == rm::SCENE_PLUGIN
            ? rmplugin::launch_render(ctx->plugin, F, out, rgba8, cnt ? ctx->d_evals : nullptr, ctx->stream)
            : rm::launch_render(ctx->scene, F, out, rgba8, cnt ? ctx->d_evals : nullptr, kernel, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "render kernel launch");
    if (stats) RM_HIP(hipEventRecord(ctx->ev1, ctx->stream));
    if (wire) {  // the offset table, the message size, the payload (rm_wire.hip)
        e = rm::launch_wire_finish(out, W, count, wire->msg, wire->size_out, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "wire scan/compact launch");
    }
    if (pb) RM_HIP(hipEventRecord(pb->last, ctx->stream));
    if (sc && F.tile_cost) {  // sort this launch's durations, on its stream right after it
        const size_t slot = (sc->k / (uint64_t)sched_period()) & 1;
        uint32_t *h = sc->buf + 4 * (size_t)sc->n;
        e = rm::launch_tile_order(sc->buf + slot * sc->n, sc->n, sc->gx, sched_dilate(), sc->buf + (2 + slot) * sc->n,
                                  h + 512 * slot, h + 512 * (1 - slot), reinterpret_cast<uint8_t *>(h + 1024),
                                  ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "tile order launch");
    }
    if (sc) {
        sc->dirty = true;  // (marked when the context leaves the stream: rm_set_stream)
        if (!cnt) sc->k++;
    }
    rm_status ms_st = mark_done(ctx);
    if (ms_st != RM_OK) return ms_st;
    if (stats) {
        RM_HIP(hipEventSynchronize(ctx->ev1));
        float ms = 0.0f;
        RM_HIP(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
        unsigned long long ev[3] = {0, 0, 0};
        if (cnt) RM_HIP(hipMemcpy(ev, ctx->d_evals, sizeof(ev), hipMemcpyDeviceToHost));
        std::memset(stats, 0, sizeof(*stats));
        stats->evals = ev[0];
        stats->flop = ev[1];
        stats->skipped = ev[2];
        stats->pixels = (uint64_t)W * (uint64_t)count;
        stats->kernel_ms = ms;
        stats->scene = ctx->scene;
        stats->dispatch = !F.tile_order ? RM_DISPATCH_ROW_MAJOR
                          : F.tile_order == ctx->tile_order ? RM_DISPATCH_EXPLICIT
                                                            : RM_DISPATCH_ADAPTIVE;
        // the latency tiles: scene T, an ordered launch of one-wave tiles
        // (rm_render_direct.h render_tile_at)
        if (F.tile_order && ctx->scene == rm::SCENE_T && kernel != rm::KERNEL_TILE16) {
            const rm::TileGrid g = rm::tile_grid(kernel, W, count);
            stats->lat_tiles = std::min(F.lat_tiles, g.x * g.y);
        }
    }
    return RM_OK;
}

// row_count < 0: every packed row from row_begin on; out: float4 or RGBA8 rows
rm_status render_part(rm_ctx *ctx, int W, int H, const RowPart &part, int row_begin, int row_count, void *out,
                      bool rgba8, rm_stats *stats, uint32_t *evmap = nullptr, bool accum = false) {
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    if (W <= 0 || H <= 0) return fail(ctx, RM_ERR_INVALID_ARGUMENT, "render: bad size");
    if ((long long)W * H > (1LL << 31)) return fail(ctx, RM_ERR_INVALID_ARGUMENT, "render: frame too large");
    if (ctx->scene < 0) return fail(ctx, RM_ERR_NO_SCENE, "no scene loaded (rm_load_scene)");
    if (ctx->scene == rm::SCENE_PLUGIN && !ctx->plugin.render)
        return fail(ctx, RM_ERR_SCENE, "scene plugin was compiled with RM_PLUGIN_EVAL_ONLY (no render kernel)");
    int n = rows_of_part(H, part);
    if (row_count < 0) row_count = n - row_begin;
    if (row_begin < 0 || row_count < 0 || row_begin + row_count > n)
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "render: packed row range outside the shard");
    if (row_count == 0) {  // e.g. more shards than bands: nothing to do
        if (stats) {
            std::memset(stats, 0, sizeof(*stats));
            stats->scene = ctx->scene;
        }
        return RM_OK;
    }
    if (!out) return fail(ctx, RM_ERR_INVALID_ARGUMENT, "render: null output");
    RM_HIP(hipSetDevice(ctx->device));
    const bool dev_out = is_device_ptr(out), dev_map = !evmap || is_device_ptr(evmap);
    if (dev_out && dev_map)
        return render_dev(ctx, W, H, part, row_begin, row_count, out, rgba8, stats, evmap, accum);
    // host buffers go through the staging buffer: the frame, then the step map
    const size_t bytes = dev_out ? 0 : (size_t)W * row_count * (rgba8 ? sizeof(uint32_t) : sizeof(float4));
    const size_t map_bytes = dev_map ? 0 : (size_t)W * row_count * sizeof(uint32_t);
    rm_status s = ensure_staging(ctx, bytes + map_bytes);
    if (s != RM_OK) return s;
    char *st = reinterpret_cast<char *>(ctx->staging);
    uint32_t *map_d = dev_map ? evmap : reinterpret_cast<uint32_t *>(st + bytes);
    if (accum && !dev_out) RM_HIP(hipMemcpyAsync(st, out, bytes, hipMemcpyHostToDevice, ctx->stream));  // u_sample
    s = render_dev(ctx, W, H, part, row_begin, row_count, dev_out ? out : st, rgba8, stats, map_d, accum);
    if (s != RM_OK) return s;
    if (!dev_out) RM_HIP(hipMemcpyAsync(out, st, bytes, hipMemcpyDeviceToHost, ctx->stream));
    if (!dev_map) RM_HIP(hipMemcpyAsync(evmap, map_d, map_bytes, hipMemcpyDeviceToHost, ctx->stream));
    RM_HIP(hipStreamSynchronize(ctx->stream));
    return RM_OK;
}

// round-robin bands (band, nshards, shard)
rm_status render_any(rm_ctx *ctx, int W, int H, int band, int nshards, int shard, int row_begin, int row_count,
                     void *out, bool rgba8, rm_stats *stats, uint32_t *evmap = nullptr, bool accum = false) {
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    RowPart part;
    if (W <= 0 || H <= 0 || !band_part(band, nshards, shard, part))
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "render: bad size/shard");
    return render_part(ctx, W, H, part, row_begin, row_count, out, rgba8, stats, evmap, accum);
}

}  // namespace

namespace {

// Which scene an existing file loads as (see "scene files of registered
// names" above).  In: sc = the scene of the base name (-1 if none).  Out: sc
// (SCENE_PLUGIN: compile `src`), src = the plugin source to compile.
rm_status classify_scene_file(const std::string &file, int &sc, std::string &src, std::string &err) {
    if (sc < 0) {
        if (!is_plugin_source(file)) {
            err = "no HIP scene plugin for \"" + file + "\"";
            return RM_ERR_SCENE;
        }
        sc = rm::SCENE_PLUGIN;
        return RM_OK;
    }
    std::string raw;
    if (!read_file(file, raw)) {
        err = "ShaderLoader: can't load file \"" + file + "\"";
        return RM_ERR_FILE;
    }
    if (sc == rm::SCENE_T) {
        if (fingerprint(raw) == kRefTemplate) return RM_OK;
        err = "\"" + file + "\" is not the reference's template.frag (which only compiles in its repaired "
              "form, scene T); write a new scene as a .hip plugin";
        return RM_ERR_SCENE;
    }
    if (sc != rm::SCENE_O) return RM_OK;  // the build's own scene names (S0, OG): no reference text
    std::string prelude, scene, pipeline, inc, lib;
    if (!split_scene(raw, prelude, scene, pipeline, inc) || fingerprint(pipeline, fingerprint(prelude)) != kRefOFrame) {
        err = "\"" + file + "\": only the scene part of output_shader.frag (materials, floorMat, sceneSDF) can "
              "be redefined; its lighting/render/main code differs from the reference's";
        return RM_ERR_SCENE;
    }
    if (!read_file(inc, lib) || fingerprint(lib) != kRefCommon) {
        err = "\"" + inc + "\" (included by \"" + file + "\") differs from the reference's common.frag: the "
              "scene library cannot be redefined; put new helpers in the scene part";
        return RM_ERR_SCENE;
    }
    if (fingerprint(scene) == kRefOScene) return RM_OK;  // the reference's own scene: compiled-in O
    sc = rm::SCENE_PLUGIN;  // an edited sceneSDF: hiprtc into output_shader.frag's pipeline
    src = scene;
    return RM_OK;
}

}  // namespace

int rm_internal_device(const rm_ctx *ctx) { return ctx->device; }
rm_status rm_internal_mark_done(rm_ctx *ctx) { return mark_done(ctx); }
hipStream_t rm_internal_stream(const rm_ctx *ctx) { return ctx->stream; }
int rm_internal_scene(const rm_ctx *ctx) { return ctx->scene; }
void rm_internal_set_error(rm_ctx *ctx, const std::string &msg) { ctx->err = msg; }

extern "C" {

rm_status rm_create(rm_ctx **out, int device) {
    if (!out) return RM_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
        (void)hipGetLastError();
        return RM_ERR_DEVICE;
    }
    rm_ctx *ctx = new rm_ctx();
    ctx->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipMalloc(&ctx->d_evals, 3 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipEventCreate(&ctx->ev0);
    if (e == hipSuccess) e = hipEventCreate(&ctx->ev1);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->done, hipEventDisableTiming);
    ctx->persist.reserve(rm_ctx::kPersistBlocks);
    if (e != hipSuccess) {
        rm_destroy(ctx);
        return e == hipErrorOutOfMemory ? RM_ERR_OUT_OF_MEMORY : RM_ERR_DEVICE;
    }
    *out = ctx;
    return RM_OK;
}

rm_status rm_destroy(rm_ctx *ctx) {
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    (void)hipSetDevice(ctx->device);
    // nothing this context enqueued still runs: its own events (the streams
    // it left may be the caller's and gone by now); other work on the device
    // is not waited for
    // The bound stream must still exist: HIP does not validate stream handles,
    // and a record on a destroyed one faults inside the runtime (a test saw
    // SIGSEGV) instead of returning an error, so the lifetime rule of rm.h
    // (rm_set_stream) is the only protection there.  The fallback below covers
    // only a record that does return an error (e.g. a device fault): the
    // context's work can then not be waited for by event, and the whole device
    // is.
    bool lost = record_sched_last(ctx) != hipSuccess;
    if (ctx->done && ctx->dirty) {
        if (hipEventRecord(ctx->done, ctx->stream) == hipSuccess) (void)hipEventSynchronize(ctx->done);
        else lost = true;
    }
    for (hipStream_t s : ctx->owed)  // kept streams left with this context's work on them
        if (!lost && ctx->done) {
            if (hipEventRecord(ctx->done, s) == hipSuccess) (void)hipEventSynchronize(ctx->done);
            else lost = true;
        }
    if (lost) {
        (void)hipGetLastError();
        (void)hipDeviceSynchronize();
    }
    for (rm_ctx::Spare &sp : ctx->spare) spare_free(sp);  // (before the borrowed `done` events go)
    ctx->spare.clear();
    for (hipEvent_t ev : ctx->retired) {
        (void)hipEventSynchronize(ev);
        (void)hipEventDestroy(ev);
    }
    for (auto &b : ctx->persist)
        if (b.last) (void)hipEventSynchronize(b.last);
    for (rm_ctx::Sched &e : ctx->sched) {
        if (e.buf && e.last && !e.left) (void)hipEventSynchronize(e.last);
        e.left = nullptr;  // (its `done` event was waited for above and is destroyed)
    }
    rmplugin::unload(ctx->plugin);
    if (ctx->d_evals) (void)hipFree(ctx->d_evals);
    for (auto &b : ctx->persist) {
        if (b.ctr) (void)hipFree(b.ctr);
        if (b.last) (void)hipEventDestroy(b.last);
    }
    if (ctx->staging) (void)hipFree(ctx->staging);
    if (ctx->mips) (void)hipFree(ctx->mips);
    if (ctx->bloom_ev) (void)hipEventDestroy(ctx->bloom_ev);
    if (ctx->tile_order) (void)hipFree(ctx->tile_order);
    for (rm_ctx::Sched &e : ctx->sched) (void)sched_release(ctx, e);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->done) (void)hipEventDestroy(ctx->done);
    delete ctx;
    return RM_OK;
}

rm_status rm_load_scene(rm_ctx *ctx, const char *file_name) {
    if (!ctx || !file_name) return RM_ERR_INVALID_ARGUMENT;
    std::string file(file_name);
    int sc = scene_of(base_name(file));
    std::ifstream probe(file);
    bool exists = probe.is_open();
    probe.close();
    if (exists) {
        std::string src, err;
        if (!preprocess(file, src, err)) {
            std::fprintf(stderr, "%s\n", err.c_str());
            return fail(ctx, RM_ERR_FILE, err);
        }
        rm_status st = classify_scene_file(file, sc, src, err);
        if (st != RM_OK) {
            std::fprintf(stderr, "%s\n", err.c_str());
            return fail(ctx, st, err);
        }
        if (sc == rm::SCENE_PLUGIN) {
            // a scene plugin: compiled like the reference's shader reload; on
            // failure the previous scene stays loaded
            rmplugin::Code code;
            std::string log;
            if (!rmplugin::compile(src, file, code, log)) {
                std::fprintf(stderr, "%s\n", log.c_str());
                return fail(ctx, RM_ERR_SCENE, "scene plugin \"" + file + "\" failed to compile:\n" + log);
            }
            RM_HIP(hipSetDevice(ctx->device));
            // kernels of the previous code object may still run on the stream
            RM_HIP(hipStreamSynchronize(ctx->stream));
            hipError_t e = rmplugin::load(code, ctx->plugin);
            if (e != hipSuccess) return hip_fail(ctx, e, "scene plugin module load");
        }
    } else if (sc < 0) {
        std::string err = "ShaderLoader: can't load file \"" + file + "\"";
        std::fprintf(stderr, "%s\n", err.c_str());
        return fail(ctx, RM_ERR_FILE, err);
    }
    ctx->scene = sc;
    ctx->scene_file = file;
    ctx->err.clear();
    return RM_OK;
}

static rm_status set_uniform(rm_ctx *ctx, const char *name, int n, float x, float y, float z) {
    if (!ctx || !name) return RM_ERR_INVALID_ARGUMENT;
    std::string nm(name);
    struct U { const char *name; int n; };
    static const U known[] = {{"u_resolution", 2}, {"u_pos", 3}, {"u_mouse", 2}, {"u_time", 1},
                              {"u_sample_part", 1}, {"u_seed1", 2}, {"u_seed2", 2}};
    for (const U &u : known) {
        if (nm != u.name) continue;
        if (n != u.n) return fail(ctx, RM_ERR_INVALID_ARGUMENT, "uniform \"" + nm + "\" has " + std::to_string(u.n) +
                                                                    " components, got " + std::to_string(n));
        if (nm == "u_resolution") { ctx->res[0] = x; ctx->res[1] = y; ctx->res_set = true; }
        else if (nm == "u_pos") { ctx->pos[0] = x; ctx->pos[1] = y; ctx->pos[2] = z; }
        else if (nm == "u_mouse") { ctx->mouse[0] = x; ctx->mouse[1] = y; }
        else if (nm == "u_time") ctx->time = x;
        // u_sample_part, u_seed1, u_seed2: declared, unused by the reference's pass
        // (common.frag:8-11); rm_render_accumulate* reads them
        else if (nm == "u_sample_part") ctx->sample_part = x;
        else if (nm == "u_seed1") { ctx->seed1[0] = x; ctx->seed1[1] = y; }
        else if (nm == "u_seed2") { ctx->seed2[0] = x; ctx->seed2[1] = y; }
        return RM_OK;
    }
    if (ctx->warned.insert(nm).second) std::fprintf(stderr, "rm: uniform \"%s\" not found in shader\n", name);
    return RM_OK;
}

rm_status rm_set_uniform1f(rm_ctx *ctx, const char *name, float x) { return set_uniform(ctx, name, 1, x, 0, 0); }
rm_status rm_set_uniform2f(rm_ctx *ctx, const char *name, float x, float y) {
    return set_uniform(ctx, name, 2, x, y, 0);
}
rm_status rm_set_uniform3f(rm_ctx *ctx, const char *name, float x, float y, float z) {
    return set_uniform(ctx, name, 3, x, y, z);
}

rm_status rm_set_params(rm_ctx *ctx, const rm_params *p) {
    if (!ctx || !p) return RM_ERR_INVALID_ARGUMENT;
    if (p->max_steps < 0 || p->max_steps > (1 << 20) || p->shadow_max_steps < 0 || p->kernel < 0 || p->kernel > 4 ||
        p->schedule < 0 || p->schedule > 1)
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_set_params: out of range");
    ctx->params = *p;
    return RM_OK;
}

rm_status rm_get_params(rm_ctx *ctx, rm_params *p) {
    if (!ctx || !p) return RM_ERR_INVALID_ARGUMENT;
    *p = ctx->params;
    return RM_OK;
}

rm_status rm_set_stream(rm_ctx *ctx, void *stream) {
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (s != ctx->stream && ctx->bloom_pending && ctx->bloom_stream == ctx->stream) {
        // the last bloom's scratch use, marked for a bloom on another stream (bloom_scratch)
        RM_HIP(hipSetDevice(ctx->device));
        if (!ctx->bloom_ev) RM_HIP(hipEventCreateWithFlags(&ctx->bloom_ev, hipEventDisableTiming));
        RM_HIP(hipEventRecord(ctx->bloom_ev, ctx->stream));
        ctx->bloom_pending = false;
    }
#ifdef RM_ANALYSIS_LEAVE_NO_RECORD
    // analysis builds only (-DRM_ANALYSIS_LEAVE_NO_RECORD, tools/scale_model.py
    // prices the marker with it; unsafe: a later release of a schedule buffer or
    // rm_destroy no longer waits for the old stream's work): leaving a stream
    // records nothing
    ctx->stream = s;
    return RM_OK;
#endif
    if (s != ctx->stream && ctx->dirty && is_kept(ctx, ctx->stream)) {
        // a kept stream: no marker now (its entries stay dirty, rm_ctx::kept)
        bool listed = false;
        for (hipStream_t o : ctx->owed) listed = listed || o == ctx->stream;
        if (!listed) ctx->owed.push_back(ctx->stream);
        ctx->dirty = false;
    }
    if (s != ctx->stream && ctx->dirty) {
        // the old stream's last work, marked now (it may be gone by the time it
        // is waited for): one `done` event, which the adaptive-order entries
        // used there since borrow (a second marker per leave cost ~4 us of
        // every frame on the two-stream pipeline); `done` is
        // kept until it completes, a completed one is reused for the new
        // stream (no host wait here)
        RM_HIP(hipSetDevice(ctx->device));
        RM_HIP(hipEventRecord(ctx->done, ctx->stream));
        for (rm_ctx::Sched &e : ctx->sched)
            if (e.buf && e.dirty && e.stream == ctx->stream) {
                e.left = ctx->done;
                e.dirty = false;
            }
        hipEvent_t next = nullptr;
        for (size_t i = 0; i < ctx->retired.size(); i++)
            if (hipEventQuery(ctx->retired[i]) == hipSuccess) {
                next = ctx->retired[i];
                ctx->retired.erase(ctx->retired.begin() + (long)i);
                break;
            }
        (void)hipGetLastError();  // hipEventQuery's hipErrorNotReady
        if (!next) RM_HIP(hipEventCreateWithFlags(&next, hipEventDisableTiming));
        ctx->retired.push_back(ctx->done);
        ctx->done = next;
        ctx->dirty = false;
    }
    ctx->stream = s;
    return RM_OK;
}

rm_status rm_set_stream_kept(rm_ctx *ctx, void *stream) {
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (!is_kept(ctx, s)) ctx->kept.push_back(s);
    return rm_set_stream(ctx, stream);
}

rm_status rm_synchronize(rm_ctx *ctx) {
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    RM_HIP(hipStreamSynchronize(ctx->stream));
    return RM_OK;
}

rm_status rm_render(rm_ctx *ctx, int W, int H, float *out, rm_stats *stats) {
    return render_any(ctx, W, H, H > 0 ? H : 1, 1, 0, 0, -1, out, false, stats);
}

rm_status rm_render_step_map(rm_ctx *ctx, int W, int H, float *out, uint32_t *evals_map, rm_stats *stats) {
    if (!evals_map) return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_render_step_map: null evals_map");
    return render_any(ctx, W, H, H > 0 ? H : 1, 1, 0, 0, -1, out, false, stats, evals_map);
}

rm_status rm_render_band(rm_ctx *ctx, int W, int H, int band, int nshards, int shard, float *out, rm_stats *stats) {
    return render_any(ctx, W, H, band, nshards, shard, 0, -1, out, false, stats);
}

rm_status rm_render_rows(rm_ctx *ctx, int W, int H, int band, int nshards, int shard, int row_begin, int row_count,
                         float *out, rm_stats *stats) {
    if (row_count < 0) return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_render_rows: negative row_count");
    return render_any(ctx, W, H, band, nshards, shard, row_begin, row_count, out, false, stats);
}

rm_status rm_render_rgba8(rm_ctx *ctx, int W, int H, uint32_t *out, rm_stats *stats) {
    return render_any(ctx, W, H, H > 0 ? H : 1, 1, 0, 0, -1, out, true, stats);
}

rm_status rm_render_accumulate(rm_ctx *ctx, int W, int H, float *accum, rm_stats *stats) {
    return render_any(ctx, W, H, H > 0 ? H : 1, 1, 0, 0, -1, accum, false, stats, nullptr, true);
}

rm_status rm_render_accumulate_rgba8(rm_ctx *ctx, int W, int H, uint32_t *accum, rm_stats *stats) {
    return render_any(ctx, W, H, H > 0 ? H : 1, 1, 0, 0, -1, accum, true, stats, nullptr, true);
}

rm_status rm_render_band_rgba8(rm_ctx *ctx, int W, int H, int band, int nshards, int shard, uint32_t *out,
                               rm_stats *stats) {
    return render_any(ctx, W, H, band, nshards, shard, 0, -1, out, true, stats);
}

rm_status rm_render_rows_rgba8(rm_ctx *ctx, int W, int H, int band, int nshards, int shard, int row_begin,
                               int row_count, uint32_t *out, rm_stats *stats) {
    if (row_count < 0) return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_render_rows_rgba8: negative row_count");
    return render_any(ctx, W, H, band, nshards, shard, row_begin, row_count, out, true, stats);
}

rm_status rm_cycle_rows(int H, int cycle, int offset, int run, int *nrows) {
    RowPart p;
    if (!nrows || H <= 0 || !cycle_part(cycle, offset, run, p)) return RM_ERR_INVALID_ARGUMENT;
    *nrows = rows_of_part(H, p);
    return RM_OK;
}

rm_status rm_render_cycle_rows(rm_ctx *ctx, int W, int H, int cycle, int offset, int run, int row_begin,
                               int row_count, float *out, rm_stats *stats) {
    RowPart p;
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    if (!cycle_part(cycle, offset, run, p) || row_count < 0)
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_render_cycle_rows: bad cycle/offset/run/row_count");
    return render_part(ctx, W, H, p, row_begin, row_count, out, false, stats);
}

rm_status rm_render_cycle_rows_rgba8(rm_ctx *ctx, int W, int H, int cycle, int offset, int run, int row_begin,
                                     int row_count, uint32_t *out, rm_stats *stats) {
    RowPart p;
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    if (!cycle_part(cycle, offset, run, p) || row_count < 0)
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_render_cycle_rows_rgba8: bad cycle/offset/run/row_count");
    return render_part(ctx, W, H, p, row_begin, row_count, out, true, stats);
}

rm_status rm_render_cycle_rows_wire(rm_ctx *ctx, int W, int H, int cycle, int offset, int run, int row_begin,
                                    int row_count, uint8_t *msg, void *workspace, int64_t *size_out, rm_stats *stats) {
    RowPart p;
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    if (!cycle_part(cycle, offset, run, p) || row_count < 0 || !msg || !workspace || W <= 0 || W > (1 << 18))
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_render_cycle_rows_wire: bad arguments");
    if (ctx->scene < 0) return fail(ctx, RM_ERR_NO_SCENE, "no scene loaded (rm_load_scene)");
    if (ctx->scene == rm::SCENE_PLUGIN)
        return fail(ctx, RM_ERR_INVALID_ARGUMENT,
                    "rm_render_cycle_rows_wire: built-in scenes only (a plugin part: rm_render_cycle_rows_rgba8 + "
                    "rm_wire_encode)");
    if (!is_device_ptr(msg) || !is_device_ptr(workspace) || (size_out && !is_device_ptr(size_out)))
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_render_cycle_rows_wire: device pointers required");
    const int n = rows_of_part(H, p);
    if (row_begin < 0 || row_begin + row_count > n)
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_render_cycle_rows_wire: packed row range outside the part");
    RM_HIP(hipSetDevice(ctx->device));
    const WireOut wo{msg, reinterpret_cast<long long *>(size_out)};
    if (row_count == 0) {  // an empty message (the table of no tiles)
        hipError_t e = rm::launch_wire_finish(workspace, W, 0, msg, wo.size_out, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "wire scan launch");
        if (stats) {
            std::memset(stats, 0, sizeof(*stats));
            stats->scene = ctx->scene;
        }
        return mark_done(ctx);
    }
    return render_dev(ctx, W, H, p, row_begin, row_count, workspace, true, stats, nullptr, false, &wo);
}

rm_status rm_deinterleave_cycle_rgb8(rm_ctx *ctx, int W, int H, int cycle, int nparts, const int *offsets,
                                     const int *runs, const int64_t *part_bytes, const uint8_t *gathered,
                                     uint32_t *out) {
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    if (W <= 0 || H <= 0 || cycle <= 0 || nparts < 1 || nparts > rm::kMaxCycleParts || !offsets || !runs ||
        !part_bytes || !gathered || !out)
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_deinterleave_cycle_rgb8: bad arguments");
    rm::CycleParts parts;
    std::memset(&parts, 0, sizeof(parts));
    parts.n = nparts;
    int next = 0;  // the parts, in order, tile [0, cycle)
    for (int i = 0; i < nparts; i++) {
        RowPart p;
        if (offsets[i] != next || !cycle_part(cycle, offsets[i], runs[i], p) || part_bytes[i] < 0)
            return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_deinterleave_cycle_rgb8: parts must tile [0, cycle) in order");
        next += runs[i];
        parts.off[i] = offsets[i];
        parts.run[i] = runs[i];
        parts.base[i] = part_bytes[i];
    }
    if (next != cycle) return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_deinterleave_cycle_rgb8: parts must tile [0, cycle)");
    if (!is_device_ptr(gathered) || !is_device_ptr(out))
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_deinterleave_cycle_rgb8: device pointers required");
    RM_HIP(hipSetDevice(ctx->device));
    hipError_t e = rm::launch_deinterleave_cycle_rgb8(gathered, out, W, H, cycle, parts, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "deinterleave launch");
    return mark_done(ctx);
}

int64_t rm_wire_capacity(int W, int nrows) {
    return (W <= 0 || W > (1 << 18) || nrows < 0) ? -1 : (int64_t)rm::wire_capacity(W, nrows);
}

int64_t rm_wire_workspace_bytes(int W, int nrows) {
    return (W <= 0 || W > (1 << 18) || nrows < 0) ? -1 : (int64_t)rm::wire_workspace(W, nrows);
}

rm_status rm_wire_encode(rm_ctx *ctx, int W, int nrows, const uint32_t *rows, uint8_t *msg, void *workspace,
                         int64_t *size_out) {
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    if (W <= 0 || W > (1 << 18) || nrows < 0 || nrows > 65535 || !msg || !workspace || (nrows > 0 && !rows))
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_wire_encode: bad arguments");
    if (!is_device_ptr(msg) || !is_device_ptr(workspace) || (nrows > 0 && !is_device_ptr(rows)) ||
        (size_out && !is_device_ptr(size_out)))
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_wire_encode: device pointers required");
    RM_HIP(hipSetDevice(ctx->device));
    hipError_t e = rm::launch_wire_encode(rows, W, nrows, msg, workspace, reinterpret_cast<long long *>(size_out),
                                          ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "wire encode launch");
    return mark_done(ctx);
}

rm_status rm_wire_decode(rm_ctx *ctx, int W, int H, int cycle, int offset, int run, int nrows, const uint8_t *msg,
                         uint32_t *frame) {
    RowPart p;
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    if (W <= 0 || W > (1 << 18) || H <= 0 || !cycle_part(cycle, offset, run, p) || nrows < 0 || nrows > 65535 ||
        nrows > rows_of_part(H, p) || !msg || !frame)
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_wire_decode: bad arguments");
    if (!is_device_ptr(msg) || !is_device_ptr(frame))
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_wire_decode: device pointers required");
    RM_HIP(hipSetDevice(ctx->device));
    hipError_t e = rm::launch_wire_decode(msg, nrows, W, cycle, offset, run, frame, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "wire decode launch");
    return mark_done(ctx);
}

rm_status rm_wire_decode_parts(rm_ctx *ctx, int W, int H, int cycle, int nparts, const int *offsets, const int *runs,
                               const int *nrows, const uint8_t *const *msgs, uint32_t *frame) {
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    if (W <= 0 || W > (1 << 18) || H <= 0 || nparts < 0 || nparts > rm::kMaxWireParts || !frame ||
        (nparts > 0 && (!offsets || !runs || !nrows || !msgs)))
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_wire_decode_parts: bad arguments");
    rm::WireParts parts;
    std::memset(&parts, 0, sizeof(parts));
    parts.n = nparts;
    parts.cycle = cycle;
    for (int i = 0; i < nparts; i++) {
        RowPart p;
        if (!cycle_part(cycle, offsets[i], runs[i], p) || nrows[i] < 0 || nrows[i] > 65535 ||
            nrows[i] > rows_of_part(H, p) || !msgs[i] || !is_device_ptr(msgs[i]))
            return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_wire_decode_parts: bad part");
        parts.part[i] = rm::WirePart{msgs[i], nrows[i], offsets[i], runs[i]};
    }
    if (!is_device_ptr(frame)) return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_wire_decode_parts: device frame required");
    RM_HIP(hipSetDevice(ctx->device));
    hipError_t e = rm::launch_wire_decode_parts(parts, W, frame, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "wire decode launch");
    return mark_done(ctx);
}

rm_status rm_scatter_part_rgba8(rm_ctx *ctx, int W, int H, int cycle, int offset, int run, int nrows,
                                const uint32_t *rows, uint32_t *frame) {
    RowPart p;
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    if (W <= 0 || H <= 0 || !cycle_part(cycle, offset, run, p) || nrows < 0 || nrows > rows_of_part(H, p) ||
        !frame || (nrows > 0 && !rows))
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_scatter_part_rgba8: bad arguments");
    if (!is_device_ptr(frame) || (nrows > 0 && !is_device_ptr(rows)))
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_scatter_part_rgba8: device pointers required");
    RM_HIP(hipSetDevice(ctx->device));
    hipError_t e = rm::launch_scatter_part(rows, nrows, W, cycle, offset, run, frame, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "scatter launch");
    return mark_done(ctx);
}

rm_status rm_set_tile_order(rm_ctx *ctx, const uint32_t *order, int64_t n) {
    if (!ctx || n < 0 || (n > 0 && !order)) return RM_ERR_INVALID_ARGUMENT;
    RM_HIP(hipSetDevice(ctx->device));
    if (ctx->tile_order) RM_HIP(hipFree(ctx->tile_order));
    ctx->tile_order = nullptr;
    ctx->tile_order_n = 0;
    if (n == 0) return RM_OK;
    std::vector<uint32_t> h((size_t)n);
    RM_HIP(hipMemcpy(h.data(), order, (size_t)n * sizeof(uint32_t), hipMemcpyDefault));
    std::vector<char> seen((size_t)n, 0);  // a permutation of [0, n)
    for (uint32_t t : h) {
        if (t >= (uint64_t)n || seen[t]) return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_set_tile_order: not a permutation");
        seen[t] = 1;
    }
    RM_HIP(hipMalloc(&ctx->tile_order, (size_t)n * sizeof(uint32_t)));
    RM_HIP(hipMemcpy(ctx->tile_order, h.data(), (size_t)n * sizeof(uint32_t), hipMemcpyHostToDevice));
    ctx->tile_order_n = n;
    return RM_OK;
}

rm_status rm_tile_grid(const rm_params *p, int W, int rows, int *tiles_x, int *tiles_y) {
    if (!p || !tiles_x || !tiles_y || W <= 0 || rows <= 0) return RM_ERR_INVALID_ARGUMENT;
    const int k = p->kernel == 1 ? rm::KERNEL_TILE16 : p->kernel == 3 ? rm::KERNEL_TILE16X4 : rm::KERNEL_TILE8;
    const rm::TileGrid g = rm::tile_grid(k, W, rows);
    *tiles_x = g.x;
    *tiles_y = g.y;
    return RM_OK;
}

rm_status rm_shard_rows(int H, int band, int nshards, int shard, int *nrows) {
    if (!nrows || H <= 0 || band <= 0 || nshards <= 0 || shard < 0 || shard >= nshards) return RM_ERR_INVALID_ARGUMENT;
    *nrows = rows_of_shard(H, band, nshards, shard);
    return RM_OK;
}

// 0: float4, 1: RGBA8 words, 2: RGB8 wire -> RGBA8 words
static rm_status deinterleave_any(rm_ctx *ctx, int W, int H, int band, int nshards, int rows_per_shard,
                                  const void *gathered, void *out, int kind) {
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    if (!gathered || !out || W <= 0 || H <= 0 || band <= 0 || nshards <= 0)
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_deinterleave: bad arguments");
    for (int s = 0; s < nshards; s++)
        if (rows_of_shard(H, band, nshards, s) > rows_per_shard)
            return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_deinterleave: rows_per_shard too small");
    if (!is_device_ptr(gathered) || !is_device_ptr(out))
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_deinterleave: device pointers required");
    RM_HIP(hipSetDevice(ctx->device));
    hipError_t e = kind == 2 ? rm::launch_deinterleave_rgb8(reinterpret_cast<const uint8_t *>(gathered),
                                                           reinterpret_cast<uint32_t *>(out), W, H, band, nshards,
                                                           rows_per_shard, ctx->stream)
                   : kind == 1 ? rm::launch_deinterleave_u32(reinterpret_cast<const uint32_t *>(gathered),
                                                      reinterpret_cast<uint32_t *>(out), W, H, band, nshards,
                                                      rows_per_shard, ctx->stream)
                         : rm::launch_deinterleave(reinterpret_cast<const float4 *>(gathered),
                                                   reinterpret_cast<float4 *>(out), W, H, band, nshards,
                                                   rows_per_shard, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "deinterleave launch");
    return mark_done(ctx);
}

rm_status rm_deinterleave(rm_ctx *ctx, int W, int H, int band, int nshards, int rows_per_shard, const float *gathered,
                          float *out) {
    return deinterleave_any(ctx, W, H, band, nshards, rows_per_shard, gathered, out, 0);
}

rm_status rm_deinterleave_rgba8(rm_ctx *ctx, int W, int H, int band, int nshards, int rows_per_shard,
                                const uint32_t *gathered, uint32_t *out) {
    return deinterleave_any(ctx, W, H, band, nshards, rows_per_shard, gathered, out, 1);
}

rm_status rm_deinterleave_rgb8(rm_ctx *ctx, int W, int H, int band, int nshards, int rows_per_shard,
                               const uint8_t *gathered, uint32_t *out) {
    return deinterleave_any(ctx, W, H, band, nshards, rows_per_shard, gathered, out, 2);
}

rm_status rm_pack_rgb8(rm_ctx *ctx, int64_t npixels, const uint32_t *in, uint8_t *out) {
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    if (npixels == 0) return RM_OK;  // an empty shard (more shards than row bands)
    if (!in || !out || npixels < 0) return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_pack_rgb8: bad arguments");
    if (!is_device_ptr(in) || !is_device_ptr(out))
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_pack_rgb8: device pointers required");
    RM_HIP(hipSetDevice(ctx->device));
    hipError_t e = rm::launch_pack_rgb8(in, out, (size_t)npixels, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "pack_rgb8 launch");
    return mark_done(ctx);
}

rm_status rm_pack_rgba8(rm_ctx *ctx, int64_t npixels, const float *in, uint32_t *out) {
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    if (!in || !out || npixels < 0) return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_pack_rgba8: bad arguments");
    if (!is_device_ptr(in) || !is_device_ptr(out))
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_pack_rgba8: device pointers required");
    RM_HIP(hipSetDevice(ctx->device));
    hipError_t e = rm::launch_pack_rgba8(reinterpret_cast<const float4 *>(in), out, (size_t)npixels, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "pack launch");
    return mark_done(ctx);
}

rm_status rm_fxaa(rm_ctx *ctx, int W, int H, const uint32_t *in, uint32_t *out) {
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    if (!in || !out || W <= 0 || H <= 0 || in == out) return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_fxaa: bad arguments");
    if ((int64_t)W * H >= ((int64_t)1 << 30))  // the kernel's 32-bit byte offsets
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_fxaa: frame of 2^30 texels or more");
    if (!is_device_ptr(in) || !is_device_ptr(out))
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_fxaa: device pointers required");
    RM_HIP(hipSetDevice(ctx->device));
    rm::TraceRange range("rm_fxaa");
    hipError_t e = rm::launch_fxaa(in, out, W, H, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "fxaa launch");
    return mark_done(ctx);
}

// bloom's scratch (mip levels, run tables, polynomials) for W x H; whether its
// run tables can be reused (the last bloom of this context had the same size
// and stream: same buffer)
static rm_status bloom_scratch(rm_ctx *ctx, const rm::BloomPlan &plan, int W, int H, bool &cached) {
    if (ctx->bloom_ev && ctx->bloom_stream != ctx->stream)  // the last bloom ran on another stream
        RM_HIP(hipStreamWaitEvent(ctx->stream, ctx->bloom_ev, 0));
    if (plan.texels > ctx->mips_texels) {
        if (ctx->mips) RM_HIP(hipFree(ctx->mips));
        ctx->mips = nullptr;
        ctx->mips_texels = 0;
        ctx->bloom_runs_w = 0;
        RM_HIP(hipMalloc(&ctx->mips, plan.texels * sizeof(uint32_t)));
        ctx->mips_texels = plan.texels;
    }
    cached = ctx->bloom_runs_w == W && ctx->bloom_runs_h == H && ctx->bloom_runs_stream == ctx->stream;
    ctx->bloom_runs_w = 0;
    return RM_OK;
}
static rm_status bloom_done(rm_ctx *ctx, int W, int H) {
    ctx->bloom_stream = ctx->stream;
    ctx->bloom_pending = true;
    ctx->bloom_runs_w = W;
    ctx->bloom_runs_h = H;
    ctx->bloom_runs_stream = ctx->stream;
    return RM_OK;
}

rm_status rm_bloom(rm_ctx *ctx, int W, int H, const uint32_t *in, uint32_t *out) {
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    if (!in || !out || W <= 0 || H <= 0 || in == out)
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_bloom: bad arguments");
    if (!is_device_ptr(in) || !is_device_ptr(out))
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_bloom: device pointers required");
    RM_HIP(hipSetDevice(ctx->device));
    rm::TraceRange range("rm_bloom");
    const rm::BloomPlan plan = rm::bloom_plan(W, H);
    bool cached = false;
    if (rm_status st = bloom_scratch(ctx, plan, W, H, cached)) return st;
    hipError_t e = rm::launch_bloom(in, out, ctx->mips, plan, ctx->stream, cached);
    if (e != hipSuccess) return hip_fail(ctx, e, "bloom launch");
    if (rm_status st = bloom_done(ctx, W, H)) return st;
    return mark_done(ctx);
}

rm_status rm_post_chain(rm_ctx *ctx, int W, int H, const uint32_t *in, uint32_t *mid, uint32_t *out) {
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    if (!in || !mid || !out || W <= 0 || H <= 0 || in == mid || mid == out || in == out)
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_post_chain: bad arguments");
    if ((int64_t)W * H >= ((int64_t)1 << 30))  // the FXAA kernel's 32-bit byte offsets
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_post_chain: frame of 2^30 texels or more");
    if (!is_device_ptr(in) || !is_device_ptr(mid) || !is_device_ptr(out))
        return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_post_chain: device pointers required");
    RM_HIP(hipSetDevice(ctx->device));
    rm::TraceRange range("rm_post_chain");
    const rm::BloomPlan plan = rm::bloom_plan(W, H);
    bool cached = false;
    if (rm_status st = bloom_scratch(ctx, plan, W, H, cached)) return st;
    // main.cpp:209-214: FXAA into postTexture, its mip chain, bloom of it
    // (the mips from FXAA's registers measured slower)
    hipError_t e = rm::launch_fxaa(in, mid, W, H, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "post chain: fxaa launch");
    e = rm::launch_bloom(mid, out, ctx->mips, plan, ctx->stream, cached);
    if (e != hipSuccess) return hip_fail(ctx, e, "post chain: bloom launch");
    if (rm_status st = bloom_done(ctx, W, H)) return st;
    return mark_done(ctx);
}

rm_status rm_scene_eval(rm_ctx *ctx, const float *points, int64_t n, float *dist, float *material) {
    if (!ctx) return RM_ERR_INVALID_ARGUMENT;
    if (n < 0 || (n > 0 && (!points || !dist))) return fail(ctx, RM_ERR_INVALID_ARGUMENT, "rm_scene_eval: bad arguments");
    if (ctx->scene < 0) return fail(ctx, RM_ERR_NO_SCENE, "no scene loaded (rm_load_scene)");
    if (n == 0) return RM_OK;
    RM_HIP(hipSetDevice(ctx->device));
    // device views of the three buffers (host ones are staged)
    const size_t pb = (size_t)n * 3 * sizeof(float), db = (size_t)n * sizeof(float), mb = (size_t)n * 16 * sizeof(float);
    const bool dp = is_device_ptr(points), dd = is_device_ptr(dist), dm = !material || is_device_ptr(material);
    char *tmp = nullptr;
    if (!(dp && dd && dm)) RM_HIP(hipMalloc(&tmp, pb + db + (material ? mb : 0)));
    const float *p = dp ? points : reinterpret_cast<float *>(tmp);
    float *d = dd ? dist : reinterpret_cast<float *>(tmp + pb);
    float *m = !material ? nullptr : dm ? material : reinterpret_cast<float *>(tmp + pb + db);
    hipError_t e = hipSuccess;
    if (!dp) e = hipMemcpyAsync(const_cast<float *>(p), points, pb, hipMemcpyHostToDevice, ctx->stream);
    FrameConst F = frame_const(ctx, 1, 1, RowPart{1, 0, 1}, 1);
    if (e == hipSuccess)
        e = ctx->scene == rm::SCENE_PLUGIN ? rmplugin::launch_eval(ctx->plugin, F, p, n, d, m, ctx->stream)
                                           : rm::launch_scene_eval(ctx->scene, F, p, n, d, m, ctx->stream);
    if (e == hipSuccess && !dd) e = hipMemcpyAsync(dist, d, db, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && material && !dm) e = hipMemcpyAsync(material, m, mb, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (tmp) (void)hipFree(tmp);
    if (e != hipSuccess) return hip_fail(ctx, e, "rm_scene_eval");
    return RM_OK;
}

rm_status rm_compile_scene(const char *file_name, char *log, size_t log_size) {
    if (!file_name) return RM_ERR_INVALID_ARGUMENT;
    std::string src, err, clog;
    rm_status st = RM_OK;
    int sc = scene_of(base_name(file_name));
    if (!preprocess(file_name, src, err)) {
        clog = err;
        st = RM_ERR_FILE;
    } else if ((st = classify_scene_file(file_name, sc, src, err)) != RM_OK) {
        clog = err;
    } else if (sc != rm::SCENE_PLUGIN) {
        clog = "compiled-in scene " + std::string(sc == rm::SCENE_T ? "T" : sc == rm::SCENE_O ? "O" : "(built-in)");
    } else {
        rmplugin::Code code;
        if (!rmplugin::compile(src, file_name, code, clog)) st = RM_ERR_SCENE;
    }
    if (log && log_size > 0) {
        size_t k = clog.size() < log_size - 1 ? clog.size() : log_size - 1;
        std::memcpy(log, clog.data(), k);
        log[k] = '\0';
    }
    return st;
}

int rm_abi_version(void) { return RM_ABI_VERSION; }

const char *rm_last_error(rm_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

const char *rm_status_string(rm_status s) {
    switch (s) {
    case RM_OK: return "RM_OK";
    case RM_ERR_INVALID_ARGUMENT: return "RM_ERR_INVALID_ARGUMENT";
    case RM_ERR_FILE: return "RM_ERR_FILE";
    case RM_ERR_SCENE: return "RM_ERR_SCENE";
    case RM_ERR_NO_SCENE: return "RM_ERR_NO_SCENE";
    case RM_ERR_DEVICE: return "RM_ERR_DEVICE";
    case RM_ERR_OUT_OF_MEMORY: return "RM_ERR_OUT_OF_MEMORY";
    }
    return "RM_ERR_UNKNOWN";
}

}  // extern "C"
