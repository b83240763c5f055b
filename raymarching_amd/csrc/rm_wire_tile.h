// rm_wire_tile.h -- the compressed wire's per-tile code, the
// part a render wave can run in its own epilogue.
//
// A part of n packed RGBA8 rows of W pixels is cut into 8x8-pixel tiles
// (TX = ceil(W / 8) across, TY = ceil(n / 8) down, tile t = ty TX + tx), one
// render wave's tile: lane l holds pixel (row 8 ty + (l >> 3), column 8 tx +
// (l & 7)), and pixels outside the part count as the word 0.  Per channel
// (R, G, B; alpha is not sent, the decoder stores 255 as the pass writes):
//
//   v_l = the channel's byte, ref_l = v_{l-1} for column > 0, v_{l-8} for the
//   first column of rows 1..7; d_l = (v_l - ref_l) mod 256 read as int8 and
//   zig-zagged (z_l in 0..255), z_0 = 0; the channel's width b = bit length
//   of max z (0..8), and bit i of z over the 64 lanes is one 64-bit word (a
//   wave ballot).
//
// The tile's words: a header (lane 0's RGB in bits 0-23, the widths in bits
// 24-27, 28-31, 32-35) and then the planes, channel-major, low bit first: 1 +
// b_R + b_G + b_B words (at most kTileWords), 8 B for a flat tile against 192 B
// as RGB8.  Smooth rows and columns (sky, floor, sponge faces) give small
// differences both ways.
//
// Message of a part: [0, 8) int64 message bytes; [8, 8 + 4 T) uint32 per tile:
// its words' offset in the payload (in words) << 5 | its word count; padded
// to 8 B; the payload (uint64 words, tiles in order t = 0..T-1).
//
// The encoders' workspace (T tiles): kTileWords planes of T uint64 -- word q
// of tile t at [q T + t], so a wave of 64 tiles copies word q of all of them
// with one coalesced load -- then T uint8 word counts, then the scan's
// per-64-tile chunk bases (uint32).
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

namespace rm {

constexpr int kTileWords = 25;  // header + 3 x 8 planes

// the encoder's workspace (above), as the render kernel's OUT type: a tile t
// of a part of T tiles writes word q to slot[q * T + t] and its count to
// counts[t]
struct WireTile {
    uint64_t w;
};
__host__ __device__ inline long long wire_counts_offset(long long T) { return 8ll * kTileWords * T; }
template <typename T>
struct IsWireTile {
    static constexpr bool value = false;
};
template <>
struct IsWireTile<WireTile> {
    static constexpr bool value = true;
};

__device__ __forceinline__ int wire_tile_words(uint64_t header) {
    return 1 + (int)((header >> 24) & 15u) + (int)((header >> 28) & 15u) + (int)((header >> 32) & 15u);
}

__device__ __forceinline__ uint32_t wire_zigzag8(uint32_t d) {  // d mod 256 as int8, zig-zagged
    const int s = (int)((d & 255u) ^ 128u) - 128;  // the byte as int8
    return (uint32_t)(s >= 0 ? 2 * s : -2 * s - 1);
}

// bit length of the wave maximum of z (0..8), wave-uniform: the least b with
// every z < 2^b, one ballot per candidate from 0 up (b + 1 ballots: most
// channels of a rendered tile are flat or one bit wide)
__device__ __forceinline__ int wire_wave_width(uint32_t z) {
    int b = 0;
    while (b < 8 && __builtin_amdgcn_ballot_w64((z >> b) != 0u)) b++;
    return b;
}

// The tile code of the wave's 64 pixels (p: this lane's RGBA8 word, 0 outside
// the part) of tile t of T: lane q < count writes word q, lane 0 the count.
// Every lane of the wave must call it (ballots).
__device__ __forceinline__ void wire_encode_tile(uint32_t p, WireTile* __restrict__ ws, long long T, long long t) {
    const int l = (int)__lane_id();
    const uint32_t left = (uint32_t)__shfl_up((int)p, 1, 64), up = (uint32_t)__shfl_up((int)p, 8, 64);
    const uint32_t ref = (l & 7) ? left : up;
    uint32_t z[3];
    int b[3];
#pragma unroll
    for (int c = 0; c < 3; c++) {
        z[c] = l == 0 ? 0u : wire_zigzag8(((p >> (8 * c)) & 255u) - ((ref >> (8 * c)) & 255u));
        b[c] = wire_wave_width(z[c]);
    }
    const uint64_t first = (uint64_t)((uint32_t)__builtin_amdgcn_readfirstlane((int)p) & 0xFFFFFFu);
    uint64_t v = first | ((uint64_t)b[0] << 24) | ((uint64_t)b[1] << 28) | ((uint64_t)b[2] << 32);
    int q = 1;
#pragma unroll
    for (int c = 0; c < 3; c++)
        for (int i = 0; i < b[c]; i++, q++) {
            const uint64_t plane = __builtin_amdgcn_ballot_w64((z[c] >> i) & 1u);
            if (l == q) v = plane;
        }
    if (l < q) ws[l * T + t].w = v;
    if (l == 0) reinterpret_cast<unsigned char*>(ws)[wire_counts_offset(T) + t] = (unsigned char)q;
}

}  // namespace rm
