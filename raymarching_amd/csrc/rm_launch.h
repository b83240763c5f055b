// rm_launch.h -- host-side launcher interface between the C-ABI (rm_capi.cpp)
// and the kernels (rm_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rm_render_direct.h"

namespace rm {


// the workgroup grid of a render launch over W x rows pixels
struct TileGrid {
    int x, y;
};
inline TileGrid tile_grid(int kernel, int W, int rows) {
    const int tw = kernel == KERNEL_TILE16 ? 16 : kernel == KERNEL_TILE16X4 ? 16 : 8;
    const int th = kernel == KERNEL_TILE16 ? 16 : kernel == KERNEL_TILE16X4 ? 4 : 8;
    return TileGrid{(W + tw - 1) / tw, (rows + th - 1) / th};
}

// out: W-wide rows of float4 (rgba8 = false) or RGBA8 words (rgba8 = true)
struct WireTile;
// rm_render_cycle_rows_wire: the built-in scenes' render kernel (8x8 one-wave
// tiles) encoding every tile into its wire slot instead of storing pixels
hipError_t launch_render_wire(int scene, const FrameConst& F, WireTile* slots, unsigned long long* evals,
                              hipStream_t s);
hipError_t launch_render(int scene, const FrameConst& F, void* out, bool rgba8, unsigned long long* evals, int kernel,
                         hipStream_t s);
// sceneSDF(p) of a compiled-in scene at n points (rm_scene_eval)
hipError_t launch_scene_eval(int scene, const FrameConst& F, const float* pts, long long n, float* dist, float* mat,
                             hipStream_t s);
hipError_t launch_deinterleave(const float4* gathered, float4* out, int W, int H, int band, int nshards,
                               int rows_per_shard, hipStream_t s);
hipError_t launch_deinterleave_u32(const uint32_t* gathered, uint32_t* out, int W, int H, int band, int nshards,
                                   int rows_per_shard, hipStream_t s);
hipError_t launch_pack_rgba8(const float4* in, uint32_t* out, size_t n, hipStream_t s);
hipError_t launch_pack_rgb8(const uint32_t* in, uint8_t* out, size_t n, hipStream_t s);
hipError_t launch_deinterleave_rgb8(const uint8_t* gathered, uint32_t* out, int W, int H, int band, int nshards,
                                    int rows_per_shard, hipStream_t s);
// cyclic parts of a frame (rm_deinterleave_cycle_rgb8): part p owns the rows y
// with (y mod cycle) - off[p] in [0, run[p]), its packed RGB8 rows from byte base[p]
constexpr int kMaxCycleParts = 64;
struct CycleParts {
    int n;
    int off[kMaxCycleParts], run[kMaxCycleParts];
    long long base[kMaxCycleParts];
};
hipError_t launch_deinterleave_cycle_rgb8(const uint8_t* gathered, uint32_t* out, int W, int H, int cycle,
                                          const CycleParts& parts, hipStream_t s);
// the next launch's tile order (costliest first) from the tile durations
// (hist: 256 counts + 256 cursors, zero on entry); clears `next` (512 words)
// for the following launch
hipError_t launch_tile_order(const uint32_t* cost, int n, int gx, int radius, uint32_t* order, uint32_t* hist,
                             uint32_t* next, uint8_t* bucket, hipStream_t s);
hipError_t launch_fxaa(const uint32_t* in, uint32_t* out, int W, int H, hipStream_t s);
// rm_wire.hip: the compressed RGB wire of RGBA8 row parts
long long wire_capacity(int W, int n);
long long wire_workspace(int W, int n);
hipError_t launch_wire_encode(const uint32_t* rows, int W, int n, uint8_t* msg, void* workspace,
                              long long* size_out, hipStream_t s);
// the scan and compaction of slots already written (rm_wire_tile.h: a render epilogue, or the rows encoder)
hipError_t launch_wire_finish(const void* workspace, int W, int n, uint8_t* msg, long long* size_out, hipStream_t s);
hipError_t launch_wire_decode(const uint8_t* msg, int n, int W, int cycle, int offset, int run, uint32_t* frame,
                              hipStream_t s);
constexpr int kMaxWireParts = 64;
struct WirePart {
    const uint8_t* msg;
    int nrows, offset, run;
};
struct WireParts {
    int n, cycle;
    WirePart part[kMaxWireParts];
};
hipError_t launch_wire_decode_parts(const WireParts& parts, int W, uint32_t* frame, hipStream_t s);
hipError_t launch_scatter_part(const uint32_t* rows, int n, int W, int cycle, int offset, int run, uint32_t* frame,
                               hipStream_t s);

// bloom.frag's textureLod level pair and the mip levels 1..d2 it needs,
// packed one after the other in a scratch buffer of `texels` 32-bit words
struct BloomPlan {
    float lod = 0.0f, fr = 0.0f;
    int d1 = 0, d2 = 0;
    int w[40] = {}, h[40] = {};
    size_t offset[40] = {}, texels = 0;
    // lod > 0 (words from the buffer start): the base level's bilinear axes
    // (per column, per row); per axis (d1 x, d1 y, d2 x, d2 y) the pixels' run
    // entries, the runs' cell tuples and the run counts; per level the run-pair
    // polynomials (rm_post.hip).  All but the polynomials depend on W x H only.
    size_t base_ent[2] = {}, run_ent[4] = {}, run_tup[4] = {}, run_count = 0, poly_tab[2] = {};
    int nruns[4] = {};  // most runs an axis can have
};
BloomPlan bloom_plan(int W, int H);
// runs_cached: the buffer already holds this W x H's run tables, written on
// this stream (only the mip levels and the polynomials are rebuilt)
hipError_t launch_bloom(const uint32_t* in, uint32_t* out, uint32_t* mips, const BloomPlan& p, hipStream_t s,
                        bool runs_cached);

}  // namespace rm
