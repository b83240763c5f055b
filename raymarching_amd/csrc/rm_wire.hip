// rm_wire.hip -- a lossless compressed wire for RGBA8 row parts (multi-GPU
// frames): the per-tile code of rm_wire_tile.h, whose message
// layout it also describes.  The frames the pass renders are smooth along rows
// and columns (sky gradients, flat floor and sponge faces), so an 8x8 tile
// costs a header and a few bit planes instead of 192 B of RGB8.
//
// Encoding is three steps: every tile's words into a fixed slot of a
// workspace (kTileWords words; rm_wire_tile_rows here from RGBA8 rows, or the
// render kernel's own epilogue, rm_render_cycle_rows_wire, which never writes
// the rows), one workgroup scanning the tiles' word counts into the message's
// offset table, and the slots compacted into the payload.  The decoder gives
// every tile a wave, which reads its offset, rebuilds the 64 differences from
// the planes and sums them along the tile's rows and its first column.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rm_launch.h"
#include "rm_wire_tile.h"

namespace rm {

__device__ __forceinline__ size_t wire_header_bytes(long long T) { return 8 + (((size_t)4 * T + 7) & ~(size_t)7); }
__host__ __device__ inline long long wire_chunks(long long T) { return (T + 63) / 64; }
__host__ __device__ inline long long wire_bases_offset(long long T) { return (wire_counts_offset(T) + T + 3) & ~3ll; }

// E1 from RGBA8 rows: one wave per tile (grid TX x TY)
__global__ __launch_bounds__(64) void rm_wire_tile_rows(const uint32_t* __restrict__ rows, int W, int n,
                                                        WireTile* __restrict__ ws) {
    const int tx = blockIdx.x, ty = blockIdx.y, l = threadIdx.x;
    const int x = tx * 8 + (l & 7), y = ty * 8 + (l >> 3);
    const uint32_t p = x < W && y < n ? rows[(size_t)y * W + x] : 0u;
    wire_encode_tile(p, ws, (long long)gridDim.x * gridDim.y, (long long)ty * gridDim.x + tx);
}

// E2: one workgroup: the word counts of each 64-tile chunk (16 counts per
// 16-byte load), an exclusive scan of the chunks into their bases (in the
// workspace), the message size into the message and *size_out.  Thread t
// sums chunks [t per, (t + 1) per); the thread sums are scanned per wave
// (shuffles) and across the 16 waves (one barrier); a thread with one chunk
// (every part of up to 65536 tiles) keeps its sum instead of reloading it.
__global__ __launch_bounds__(1024) void rm_wire_tile_scan(const uint8_t* __restrict__ ws, long long T,
                                                          uint8_t* __restrict__ msg, long long* __restrict__ size_out) {
    __shared__ uint32_t wave_total[16];
    const int t = threadIdx.x, l = t & 63, w = t >> 6;
    const uint8_t* counts = ws + wire_counts_offset(T);
    uint32_t* bases = reinterpret_cast<uint32_t*>(const_cast<uint8_t*>(ws) + wire_bases_offset(T));
    const long long C = wire_chunks(T), per = (C + 1023) / 1024, c0 = t * per, c1 = c0 + per < C ? c0 + per : C;
    auto chunk_sum = [&](long long c) {
        const long long i0 = c * 64, i1 = i0 + 64 < T ? i0 + 64 : T;
        uint32_t s = 0;
        if (i1 - i0 == 64 && ((reinterpret_cast<uintptr_t>(counts) + i0) & 15) == 0) {
            const uint4* q = reinterpret_cast<const uint4*>(counts + i0);
            uint4 v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = q[k];
#pragma unroll
            for (int k = 0; k < 4; k++)
                for (uint32_t x : {v[k].x, v[k].y, v[k].z, v[k].w})  // four counts per word, each < 256
                    s += (x & 255u) + ((x >> 8) & 255u) + ((x >> 16) & 255u) + (x >> 24);
        } else {
            for (long long i = i0; i < i1; i++) s += counts[i];
        }
        return s;
    };
    uint32_t s = 0;  // (the payload's words: < 2^27, the table's offset field)
    for (long long c = c0; c < c1; c++) s += chunk_sum(c);
    uint32_t x = s;  // inclusive scan over the wave's lanes
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
        const uint32_t u = (uint32_t)__shfl_up((int)x, k, 64);
        if (l >= k) x += u;
    }
    if (l == 63) wave_total[w] = x;
    __syncthreads();
    uint32_t off = x - s, total = 0;
    for (int v = 0; v < 16; v++) {
        const uint32_t wt = wave_total[v];
        if (v < w) off += wt;
        total += wt;
    }
    if (per == 1) {
        if (c0 < C) bases[c0] = off;
    } else {
        for (long long c = c0; c < c1; c++) {
            bases[c] = off;
            off += chunk_sum(c);
        }
    }
    if (t == 1023) {
        const long long bytes = (long long)wire_header_bytes(T) + 8ll * (long long)total;
        *reinterpret_cast<long long*>(msg) = bytes;
        if (size_out) *size_out = bytes;
    }
}

// E3: one wave per 64-tile chunk, lane = tile: its offset (the chunk's base
// plus a wave scan of the counts) into the table, its words into the payload
// (word q of the chunk's tiles: one coalesced load)
__global__ __launch_bounds__(256) void rm_wire_tile_compact(const uint8_t* __restrict__ ws, long long T,
                                                            uint8_t* __restrict__ msg) {
    const long long chunk = 4ll * blockIdx.x + (threadIdx.x >> 6);  // (four 64-tile chunks per workgroup)
    const long long t = 64ll * chunk + (threadIdx.x & 63);
    const int l = threadIdx.x & 63;
    if (chunk >= wire_chunks(T)) return;  // (wave-uniform)
    const uint32_t base = reinterpret_cast<const uint32_t*>(ws + wire_bases_offset(T))[chunk];
    const uint32_t cnt = t < T ? ws[wire_counts_offset(T) + t] : 0u;
    uint32_t x = cnt;  // inclusive scan over the lanes
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
        const uint32_t u = (uint32_t)__shfl_up((int)x, k, 64);
        if (l >= k) x += u;
    }
    const uint32_t off = base + x - cnt;
    if (t >= T) return;
    reinterpret_cast<uint32_t*>(msg + 8)[t] = off << 5 | cnt;
    const uint64_t* src = reinterpret_cast<const uint64_t*>(ws);
    uint64_t* dst = reinterpret_cast<uint64_t*>(msg + wire_header_bytes(T)) + off;
    // (eight words' loads in flight before their stores; most tiles have fewer)
    for (uint32_t q0 = 0; q0 < cnt; q0 += 8) {
        uint64_t v[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) v[k] = q0 + k < cnt ? src[(q0 + k) * T + t] : 0ull;
#pragma unroll
        for (uint32_t k = 0; k < 8; k++)
            if (q0 + k < cnt) dst[q0 + k] = v[k];
    }
}

// E2 + E3 in one launch for parts of up to kDirectTiles tiles: workgroup b
// (tiles 256 b .. 256 b + 255, four 64-tile chunks) sums the counts of every
// tile before it itself (8 counts per 8-byte load over its 256 lanes, then a
// workgroup reduction) instead of reading a base a scan kernel wrote; each wave
// adds the counts of the chunks before its own in the workgroup, scans its
// lanes and compacts its tiles as rm_wire_tile_compact does.  The last
// workgroup writes the message size.  (One launch less per part and frame;
// the redundant prefix sums read T^2 / 512 bytes in all, from L2.)
constexpr long long kDirectTiles = 65536;
__device__ __forceinline__ uint32_t byte_sum8(uint2 v) {  // the eight bytes' sum
    const uint32_t a = (v.x & 0x00ff00ffu) + ((v.x >> 8) & 0x00ff00ffu) + (v.y & 0x00ff00ffu) +
                       ((v.y >> 8) & 0x00ff00ffu);
    return (a & 0xffffu) + (a >> 16);
}
__global__ __launch_bounds__(256) void rm_wire_tile_compact_direct(const uint8_t* __restrict__ ws, long long T,
                                                                   uint8_t* __restrict__ msg,
                                                                   long long* __restrict__ size_out) {
    __shared__ uint32_t red[4], wave_tot[4];
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const uint8_t* counts = ws + wire_counts_offset(T);
    // the counts of tiles [0, 256 b): 8-byte loads (the counts start 8-byte
    // aligned: 200 T bytes into the workspace), strided over the lanes
    const long long pre = 256ll * blockIdx.x, nq = pre / 8;
    uint32_t s = 0;
    for (long long q = tid; q < nq; q += 256) s += byte_sum8(reinterpret_cast<const uint2*>(counts)[q]);
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) s += (uint32_t)__shfl_xor((int)s, k, 64);
    if (l == 0) red[w] = s;
    const long long t = 256ll * blockIdx.x + tid;
    const uint32_t cnt = t < T ? counts[t] : 0u;
    uint32_t x = cnt;  // inclusive scan over the wave's lanes
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
        const uint32_t u = (uint32_t)__shfl_up((int)x, k, 64);
        if (l >= k) x += u;
    }
    if (l == 63) wave_tot[w] = x;
    __syncthreads();
    uint32_t off = red[0] + red[1] + red[2] + red[3] + x - cnt;
    for (int v = 0; v < w; v++) off += wave_tot[v];
    if (blockIdx.x == gridDim.x - 1 && tid == 0) {
        const uint32_t total = red[0] + red[1] + red[2] + red[3] + wave_tot[0] + wave_tot[1] + wave_tot[2] +
                               wave_tot[3];
        const long long bytes = (long long)wire_header_bytes(T) + 8ll * (long long)total;
        *reinterpret_cast<long long*>(msg) = bytes;
        if (size_out) *size_out = bytes;
    }
    if (t >= T) return;
    reinterpret_cast<uint32_t*>(msg + 8)[t] = off << 5 | cnt;
    const uint64_t* src = reinterpret_cast<const uint64_t*>(ws);
    uint64_t* dst = reinterpret_cast<uint64_t*>(msg + wire_header_bytes(T)) + off;
    for (uint32_t q0 = 0; q0 < cnt; q0 += 8) {
        uint64_t v[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) v[k] = q0 + k < cnt ? src[(q0 + k) * T + t] : 0ull;
#pragma unroll
        for (uint32_t k = 0; k < 8; k++)
            if (q0 + k < cnt) dst[q0 + k] = v[k];
    }
}

// D: a wave rebuilds kDecodeTiles tiles (tx0 .. of tile row ty) of a part into
// their pixels of the frame (the part's packed row j is frame row y(j): (y mod
// cycle) - offset in [0, run)).  The table entries and then every tile's words
// are loaded before any is decoded (two memory round trips for the wave).
// Lane l = pixel (l & 7, l >> 3) of a tile.
//
// Per tile, cross-lane work only on the VALU (no LDS): a bit plane is a
// 64-bit lane mask, so lane l's bit is one v_cndmask with the plane in an SGPR
// pair; the differences are summed along each row of 8 lanes (DPP row_shr by
// 1, 2, 4: the sources of a shift are zeroed where they would cross into the
// next row of the tile, and row_shr:4 skips the first half of each 8-lane row
// by its bank mask) and the first column's differences down the tile (a
// wave-wide inclusive scan of the first-column lanes: row_shr 1, 2, 4, 8,
// row_bcast:15, row_bcast:31), whose sum at any lane of tile row r is that
// row's first pixel.
__device__ __forceinline__ uint32_t lane_bit(uint64_t plane) {  // bit l of a wave-uniform 64-bit word
    uint32_t r;
    asm("v_cndmask_b32 %0, 0, 1, %1" : "=v"(r) : "s"(plane));
    return r;
}
template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp0(uint32_t x) {  // DPP move; disabled and out-of-row lanes read 0
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROW_MASK, BANK_MASK, true);
}
// Plane q (payload word q = 1 .. nq) gives bit q - 1 of a lane's `bits`, all
// planes in one fully unrolled gather (constant lane indices, no scalar loop
// per plane); a channel's z is then a field of `bits`.  Words past the tile's
// count were loaded as 0, so planes past nq add nothing.
__device__ __forceinline__ uint32_t wire_decode_tile(uint64_t mine, int l, uint32_t h_lo, uint32_t h_hi) {
    const int bR = min((int)((h_lo >> 24) & 15u), 8), bG = min((int)(h_lo >> 28), 8), bB = min((int)(h_hi & 15u), 8);
    const int nq = bR + bG + bB;
    const uint32_t m_lo = (uint32_t)mine, m_hi = (uint32_t)(mine >> 32);
    uint32_t bits = 0;
#pragma unroll
    for (int g = 0; g < 3 * 8; g += 4) {
        if (g >= nq) break;  // (wave-uniform)
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t plane = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)m_lo, 1 + g + k) |
                                   ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)m_hi, 1 + g + k) << 32);
            bits |= lane_bit(plane) << (g + k);
        }
    }
    const uint32_t z[3] = {bits & ((1u << bR) - 1u), (bits >> bR) & ((1u << bG) - 1u),
                           (bits >> (bR + bG)) & ((1u << bB) - 1u)};
    uint32_t d[3];
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const int s = (int)(z[c] >> 1) ^ -(int)(z[c] & 1u);  // zig-zag back: the difference as int8
        d[c] = l == 0 ? (h_lo >> (8 * c)) & 255u : (uint32_t)s & 255u;
    }
    // the sums mod 256 per channel, two channels per word in 16-bit fields (at
    // most 64 x 255 < 2^16: no carry between fields)
    const int c8 = l & 7;
    const uint32_t A = d[0] | (d[1] << 16), B = d[2];
    // first column: the inclusive wave scan of its lanes (other lanes 0)
    uint32_t ya = c8 == 0 ? A : 0u, yb = c8 == 0 ? B : 0u;
    ya += dpp0<0x111>(ya), yb += dpp0<0x111>(yb);  // row_shr:1
    ya += dpp0<0x112>(ya), yb += dpp0<0x112>(yb);  // row_shr:2
    ya += dpp0<0x114>(ya), yb += dpp0<0x114>(yb);  // row_shr:4
    ya += dpp0<0x118>(ya), yb += dpp0<0x118>(yb);  // row_shr:8
    ya += dpp0<0x142, 0xa>(ya), yb += dpp0<0x142, 0xa>(yb);  // row_bcast:15 into rows 1, 3
    ya += dpp0<0x143, 0xc>(ya), yb += dpp0<0x143, 0xc>(yb);  // row_bcast:31 into rows 2, 3
    // along each tile row: the other columns' differences, scanned in 8-lane segments
    uint32_t xa = c8 == 0 ? 0u : A, xb = c8 == 0 ? 0u : B;
    xa += dpp0<0x111>(c8 == 7 ? 0u : xa), xb += dpp0<0x111>(c8 == 7 ? 0u : xb);  // (no source across a row end)
    xa += dpp0<0x112>(c8 >= 6 ? 0u : xa), xb += dpp0<0x112>(c8 >= 6 ? 0u : xb);
    xa += dpp0<0x114, 0xf, 0xa>(xa), xb += dpp0<0x114, 0xf, 0xa>(xb);  // (banks 1, 3: lanes c8 >= 4)
    const uint32_t va = xa + ya, vb = xb + yb;
    return (va & 255u) | (((va >> 16) & 255u) << 8) | ((vb & 255u) << 16) | 0xFF000000u;
}

constexpr int kDecodeTiles = 2;  // tiles per wave (1, 2, 4, 8 measured: 2 fastest, profiles/r06/decode_ab.log)
constexpr int kDecodeWaves = 4;  // waves per workgroup (one-wave workgroups cap a CU's resident waves)
constexpr int kDecodeWorkgroups = 7 * 256;  // the launch's target workgroup count (launch_wire_decode_parts)
__device__ __forceinline__ void wire_decode_tiles(const uint8_t* __restrict__ msg, int n, int W, int tx0, int ty,
                                                  int cycle, int offset, int run, uint32_t* __restrict__ frame) {
    const int l = threadIdx.x & 63, TX = (W + 7) / 8;
    if (tx0 >= TX) return;  // (wave-uniform)
    const long long T = (long long)TX * ((n + 7) / 8), t0 = (long long)ty * TX + tx0;
    const int nt = TX - tx0 < kDecodeTiles ? TX - tx0 : kDecodeTiles;
    const uint32_t ent = l < nt ? reinterpret_cast<const uint32_t*>(msg + 8)[t0 + l] : 0u;
    const uint64_t* payload = reinterpret_cast<const uint64_t*>(msg + wire_header_bytes(T));
    uint64_t mine[kDecodeTiles];
#pragma unroll
    for (int k = 0; k < kDecodeTiles; k++) {
        const uint32_t e = (uint32_t)__builtin_amdgcn_readlane((int)ent, k);
        const uint32_t cnt = min(e & 31u, (uint32_t)kTileWords);  // (a corrupt count cannot read past the tile)
        mine[k] = k < nt && (uint32_t)l < cnt ? payload[(e >> 5) + l] : 0ull;
    }
    const int j = ty * 8 + (l >> 3);
    const int c0 = j / run, y = c0 * cycle + offset + (j - c0 * run);
#pragma unroll
    for (int k = 0; k < kDecodeTiles; k++) {
        if (k >= nt) break;
        // a flat tile (every width 0, about half of a rendered frame's): every
        // pixel is the header's colour
        const uint32_t h_lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)mine[k]);
        const uint32_t h_hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(mine[k] >> 32));
        const uint32_t px =
            ((h_lo >> 24) | (h_hi & 15u)) == 0 ? h_lo | 0xFF000000u : wire_decode_tile(mine[k], l, h_lo, h_hi);
        const int x = (tx0 + k) * 8 + (l & 7);
        if (x < W && j < n) frame[(size_t)y * W + x] = px;
    }
}

// D for several parts in one launch (grid ceil(TX / (kDecodeTiles
// kDecodeWaves)) x tile rows x parts; wave w of workgroup x: tiles
// kDecodeTiles (kDecodeWaves x + w) .. of the row)
__global__ __launch_bounds__(64 * kDecodeWaves) void rm_wire_tile_decode_parts(WireParts parts, int W,
                                                                               uint32_t* __restrict__ frame) {
    const WirePart& P = parts.part[blockIdx.z];
    const int TY = (P.nrows + 7) / 8;
    const int tx0 = (blockIdx.x * kDecodeWaves + (threadIdx.x >> 6)) * kDecodeTiles;
    for (int ty = blockIdx.y; ty < TY; ty += gridDim.y)
        wire_decode_tiles(P.msg, P.nrows, W, tx0, ty, parts.cycle, P.offset, P.run, frame);
}

// a part's packed RGBA8 rows into their frame rows (the root's own part)
__global__ __launch_bounds__(256) void rm_scatter_part(const uint32_t* __restrict__ rows, int n, int W, int cycle,
                                                       int offset, int run, uint32_t* __restrict__ frame) {
    for (int j = blockIdx.y; j < n; j += gridDim.y) {
        const int c0 = j / run, y = c0 * cycle + offset + (j - c0 * run);
        const uint32_t* src = rows + (size_t)j * W;
        uint32_t* dst = frame + (size_t)y * W;
        for (int x = blockIdx.x * 256 + threadIdx.x; x < W; x += gridDim.x * 256) dst[x] = src[x];
    }
}

long long wire_capacity(int W, int n) {
    const long long T = (long long)((W + 7) / 8) * ((n + 7) / 8);
    return 8 + ((4 * T + 7) & ~7ll) + 8ll * kTileWords * T;
}

long long wire_workspace(int W, int n) {
    const long long T = (long long)((W + 7) / 8) * ((n + 7) / 8);
    return wire_bases_offset(T) + 4 * wire_chunks(T);
}

// E2 + E3 over a workspace already written (by rm_wire_tile_rows or a render epilogue)
hipError_t launch_wire_finish(const void* workspace, int W, int n, uint8_t* msg, long long* size_out, hipStream_t s) {
    const long long T = (long long)((W + 7) / 8) * ((n + 7) / 8);
    const uint8_t* ws = reinterpret_cast<const uint8_t*>(workspace);
    if (T > 0 && T <= kDirectTiles) {
        hipLaunchKernelGGL(rm_wire_tile_compact_direct, dim3((unsigned)((T + 255) / 256)), dim3(256), 0, s, ws, T,
                           msg, size_out);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(rm_wire_tile_scan, dim3(1), dim3(1024), 0, s, ws, T, msg, size_out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || T == 0) return e;
    hipLaunchKernelGGL(rm_wire_tile_compact, dim3((unsigned)((wire_chunks(T) + 3) / 4)), dim3(256), 0, s, ws, T, msg);
    return hipGetLastError();
}

hipError_t launch_wire_encode(const uint32_t* rows, int W, int n, uint8_t* msg, void* workspace,
                              long long* size_out, hipStream_t s) {
    if (n > 0) {
        hipLaunchKernelGGL(rm_wire_tile_rows, dim3((W + 7) / 8, (n + 7) / 8), dim3(64), 0, s, rows, W, n,
                           reinterpret_cast<WireTile*>(workspace));
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return launch_wire_finish(workspace, W, n, msg, size_out, s);
}

hipError_t launch_wire_decode(const uint8_t* msg, int n, int W, int cycle, int offset, int run, uint32_t* frame,
                              hipStream_t s) {
    WireParts parts{};
    parts.n = 1;
    parts.cycle = cycle;
    parts.part[0] = WirePart{msg, n, offset, run};
    return launch_wire_decode_parts(parts, W, frame, s);
}

hipError_t launch_wire_decode_parts(const WireParts& parts, int W, uint32_t* frame, hipStream_t s) {
    int rows = 0;
    for (int i = 0; i < parts.n; i++) rows = parts.part[i].nrows > rows ? parts.part[i].nrows : rows;
    if (parts.n <= 0 || rows <= 0) return hipSuccess;
    const int TY = (rows + 7) / 8;
    const int per = kDecodeTiles * kDecodeWaves, gx = ((W + 7) / 8 + per - 1) / per;
    // about seven workgroups per CU in all, each looping over tile rows
    // (blockIdx.y strides): the decode then takes as many wave slots as one
    // resident round and shares the CUs with the next frame's render on the
    // other stream.  In DeltaFrame's loop the root's frame at N = 8 (C3) went
    // 0.111-0.116 -> 0.099-0.105 ms against 2, 8, 16 or all tile rows per
    // grid row (profiles/r06/decode_grid_ab.log); the decode alone is slower
    // (0.042 -> 0.057 ms).
    const int want = (kDecodeWorkgroups + gx * parts.n - 1) / (gx * parts.n);
    const int gy = TY < want ? TY : (want < 1 ? 1 : want);
    hipLaunchKernelGGL(rm_wire_tile_decode_parts, dim3(gx, gy, parts.n), dim3(64 * kDecodeWaves), 0,
                       s, parts, W, frame);
    return hipGetLastError();
}

hipError_t launch_scatter_part(const uint32_t* rows, int n, int W, int cycle, int offset, int run, uint32_t* frame,
                               hipStream_t s) {
    if (n <= 0 || W <= 0) return hipSuccess;
    const unsigned bx = (unsigned)((W + 255) / 256 < 16 ? (W + 255) / 256 : 16);
    hipLaunchKernelGGL(rm_scatter_part, dim3(bx, (unsigned)(n < 65535 ? n : 65535)), dim3(256), 0, s, rows, n, W,
                       cycle, offset, run, frame);
    return hipGetLastError();
}

}  // namespace rm
