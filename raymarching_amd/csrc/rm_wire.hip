// rm_wire.hip -- a lossless compressed wire for RGBA8 row parts (multi-GPU
// frames).  The frames the pass renders are smooth along rows
// (sky gradients, flat floor and sponge faces), so each 64-pixel row segment
// -- one wave's store -- is sent as its first pixel plus the left differences
// of the other 63, per channel, at the segment's bit width:
//
//   d = (p[l] - p[l-1]) mod 256 as int8, z = zig-zag(d) in 0..255,
//   b_c = bit width of max_l z_c (0..8), and bit i of z_c over the 64 lanes is
//   one 64-bit word (a wave ballot; lane 0 contributes 0).
//
// A segment costs 8 B of header (first pixel's RGB, three widths) plus
// 8 B per bit plane, against 192 B as RGB8; flat segments cost 8 B.  Alpha is
// not sent (the pass writes 1: the root stores 255, as the RGB8 wire does).
//
// Message of a part of n packed rows, W pixels, S = ceil(W / 64) segments:
//   [0, 8)            uint64 message bytes
//   [8, 8 + 4n)       uint32 row offset of each row's words in the payload
//   then n * S bytes  words per segment (1 + planes), padded to 8 B
//   then payload      uint64 words: per row, per segment: header, planes
// The encoder writes every segment's words into a fixed slot of a workspace
// (25 words: the widest segment), then scans the rows and compacts the slots
// into the message; the decoder gives every segment a wave, which sums the
// row's earlier segment sizes and rebuilds its 64 pixels with a wave-wide
// prefix sum of the differences.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rm_launch.h"

namespace rm {

constexpr int kSegWords = 25;  // header + 3 x 8 planes

__device__ __forceinline__ uint32_t zigzag8(int d) {  // d in -255..255 -> the int8 wrap, zig-zagged
    const int s = (int)(int8_t)(uint8_t)(d & 255);
    return (uint32_t)(s >= 0 ? 2 * s : -2 * s - 1);
}
__device__ __forceinline__ int unzigzag8(uint32_t z) { return (int)(z >> 1) ^ -(int)(z & 1u); }

__device__ __forceinline__ uint64_t ballot64(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// bit width of the wave maximum of z (0..8), wave-uniform
__device__ __forceinline__ int wave_width(uint32_t z) {
    int b = 0;
    for (int i = 7; i >= 0; i--)
        if (ballot64((z >> i) & 1u)) {
            b = i + 1;
            break;
        }
    return b;
}

// E1: one wave per segment (grid S x n, 64 threads): its words into the slot,
// its word count into the message's count table, the row's total (atomics).
__global__ __launch_bounds__(64) void rm_wire_seg_encode(const uint32_t* __restrict__ rows, int W, int n,
                                                         uint64_t* __restrict__ slots, uint8_t* __restrict__ counts,
                                                         uint32_t* __restrict__ row_words) {
    const int k = blockIdx.x, j = blockIdx.y, l = threadIdx.x, S = gridDim.x;
    const int x = k * 64 + l;
    const uint32_t p = rows[(size_t)j * W + (x < W ? x : W - 1)];  // past the row end: repeats the last pixel
    const uint32_t left = __shfl(p, l > 0 ? l - 1 : 0, 64);
    uint32_t z[3];
    int b[3], total = 0;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        z[c] = l == 0 ? 0u : zigzag8((int)((p >> (8 * c)) & 255u) - (int)((left >> (8 * c)) & 255u));
        b[c] = wave_width(z[c]);
        total += b[c];
    }
    // lane 0: the header; lane q + 1: plane q (channel-major, low bit first)
    const uint32_t first = (uint32_t)__builtin_amdgcn_readfirstlane((int)p) & 0xFFFFFFu;
    uint64_t v = (uint64_t)first | ((uint64_t)b[0] << 24) | ((uint64_t)b[1] << 28) | ((uint64_t)b[2] << 32);
    int q = 1;
#pragma unroll
    for (int c = 0; c < 3; c++)
        for (int i = 0; i < b[c]; i++, q++) {
            const uint64_t plane = ballot64((z[c] >> i) & 1u);
            if (l == q) v = plane;
        }
    const size_t seg = (size_t)j * S + k;
    if (l <= total) slots[seg * kSegWords + l] = v;
    if (l == 0) {
        counts[seg] = (uint8_t)(1 + total);
        atomicAdd(&row_words[j], (uint32_t)(1 + total));
    }
}

__device__ __forceinline__ size_t wire_header_bytes(int n, int S) {
    return 8 + (((size_t)4 * n + 7) & ~(size_t)7) + (((size_t)n * S + 7) & ~(size_t)7);
}

// E2: one workgroup: exclusive scan of the rows' word counts into the
// message's row offsets; the message size into the message and *size_out.
__global__ __launch_bounds__(1024) void rm_wire_row_scan(const uint32_t* __restrict__ row_words, int n, int S,
                                                          uint8_t* __restrict__ msg, long long* __restrict__ size_out) {
    __shared__ unsigned long long part[1024];
    const int t = threadIdx.x;
    const int per = (n + 1023) / 1024, j0 = t * per, j1 = min(n, j0 + per);
    unsigned long long s = 0;
    for (int j = j0; j < j1; j++) s += row_words[j];
    part[t] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive scan of the thread sums
        const unsigned long long add = t >= o ? part[t - o] : 0ull;
        __syncthreads();
        part[t] += add;
        __syncthreads();
    }
    unsigned long long off = t > 0 ? part[t - 1] : 0ull;
    uint32_t* row_off = reinterpret_cast<uint32_t*>(msg + 8);
    for (int j = j0; j < j1; j++) {
        row_off[j] = (uint32_t)off;
        off += row_words[j];
    }
    if (t == 1023) {
        const long long bytes = (long long)wire_header_bytes(n, S) + 8ll * (long long)part[1023];
        *reinterpret_cast<long long*>(msg) = bytes;
        if (size_out) *size_out = bytes;
    }
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// words of a row's segments before segment k (one wave, wave-uniform result)
__device__ __forceinline__ uint32_t seg_offset(const uint8_t* __restrict__ counts, int k, int l) {
    uint32_t acc = 0;
    for (int c0 = 0; c0 < k; c0 += 64) {
        const int kk = c0 + l;
        acc += wave_sum(kk < k ? (uint32_t)counts[kk] : 0u);
    }
    return acc;
}

// E3: one wave per segment (grid S x n): its slot's words into the payload
__global__ __launch_bounds__(64) void rm_wire_compact(const uint64_t* __restrict__ slots, int n,
                                                      uint8_t* __restrict__ msg) {
    const int k = blockIdx.x, j = blockIdx.y, l = threadIdx.x, S = gridDim.x;
    const size_t hb = wire_header_bytes(n, S);
    const uint8_t* counts = msg + 8 + (((size_t)4 * n + 7) & ~(size_t)7) + (size_t)j * S;
    const uint32_t off = reinterpret_cast<const uint32_t*>(msg + 8)[j] + seg_offset(counts, k, l);
    const int cnt = counts[k];
    if (l < cnt)
        reinterpret_cast<uint64_t*>(msg + hb)[off + l] = slots[((size_t)j * S + k) * kSegWords + l];
}

// D: one wave per segment of a part's packed row j (grid S x n): rebuilt into
// frame row y(j) (the part's rows: (y mod cycle) - offset in [0, run))
__global__ __launch_bounds__(64) void rm_wire_decode(const uint8_t* __restrict__ msg, int n, int W, int cycle,
                                                     int offset, int run, uint32_t* __restrict__ frame) {
    const int k = blockIdx.x, j = blockIdx.y, l = threadIdx.x, S = gridDim.x;
    const size_t hb = wire_header_bytes(n, S);
    const uint8_t* counts = msg + 8 + (((size_t)4 * n + 7) & ~(size_t)7) + (size_t)j * S;
    const uint32_t off = reinterpret_cast<const uint32_t*>(msg + 8)[j] + seg_offset(counts, k, l);
    const int cnt = min((int)counts[k], kSegWords);  // (a corrupt count cannot read past the segment)
    const uint64_t* sw = reinterpret_cast<const uint64_t*>(msg + hb) + off;
    const uint64_t mine = l < cnt ? sw[l] : 0ull;  // lane 0: header, lane q + 1: plane q
    const uint32_t m_lo = (uint32_t)mine, m_hi = (uint32_t)(mine >> 32);
    const uint32_t h_lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)m_lo);
    const uint32_t h_hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)m_hi);
    const int b[3] = {min((int)((h_lo >> 24) & 15u), 8), min((int)(h_lo >> 28), 8), min((int)(h_hi & 15u), 8)};
    // this lane's bit of a plane word: from the low half for lanes 0-31, the high half for 32-63
    const uint32_t sh = (uint32_t)(l & 31);
    const bool hi_half = l >= 32;
    uint32_t px = 0;
    int q = 1;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        uint32_t z = 0;
        for (int i = 0; i < b[c]; i++, q++) {
            const uint32_t w = hi_half ? (uint32_t)__builtin_amdgcn_readlane((int)m_hi, q)
                                       : (uint32_t)__builtin_amdgcn_readlane((int)m_lo, q);
            z |= ((w >> sh) & 1u) << i;
        }
        int d = l == 0 ? (int)((h_lo >> (8 * c)) & 255u) : unzigzag8(z);
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {  // inclusive prefix sum over the lanes
            const int u = __shfl_up(d, o, 64);
            if (l >= o) d += u;
        }
        px |= (uint32_t)(d & 255) << (8 * c);
    }
    const int c0 = j / run, y = c0 * cycle + offset + (j - c0 * run);
    const int x = k * 64 + l;
    if (x < W) frame[(size_t)y * W + x] = px | 0xFF000000u;
}

// D for several parts in one launch (grid S x max rows x parts)
__global__ __launch_bounds__(64) void rm_wire_decode_parts(WireParts parts, int W, uint32_t* __restrict__ frame) {
    const WirePart& P = parts.part[blockIdx.z];
    const int k = blockIdx.x, l = threadIdx.x, S = gridDim.x, n = P.nrows;
    const size_t hb = wire_header_bytes(n, S);
    for (int j = blockIdx.y; j < n; j += gridDim.y) {
        const uint8_t* msg = P.msg;
        const uint8_t* counts = msg + 8 + (((size_t)4 * n + 7) & ~(size_t)7) + (size_t)j * S;
        const uint32_t off = reinterpret_cast<const uint32_t*>(msg + 8)[j] + seg_offset(counts, k, l);
        const int cnt = min((int)counts[k], kSegWords);
        const uint64_t* sw = reinterpret_cast<const uint64_t*>(msg + hb) + off;
        const uint64_t mine = l < cnt ? sw[l] : 0ull;
        const uint32_t m_lo = (uint32_t)mine, m_hi = (uint32_t)(mine >> 32);
        const uint32_t h_lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)m_lo);
        const uint32_t h_hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)m_hi);
        const int b[3] = {min((int)((h_lo >> 24) & 15u), 8), min((int)(h_lo >> 28), 8), min((int)(h_hi & 15u), 8)};
        const uint32_t sh = (uint32_t)(l & 31);
        const bool hi_half = l >= 32;
        uint32_t px = 0;
        int q = 1;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            uint32_t z = 0;
            for (int i = 0; i < b[c]; i++, q++) {
                const uint32_t w = hi_half ? (uint32_t)__builtin_amdgcn_readlane((int)m_hi, q)
                                           : (uint32_t)__builtin_amdgcn_readlane((int)m_lo, q);
                z |= ((w >> sh) & 1u) << i;
            }
            int d = l == 0 ? (int)((h_lo >> (8 * c)) & 255u) : unzigzag8(z);
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int u = __shfl_up(d, o, 64);
                if (l >= o) d += u;
            }
            px |= (uint32_t)(d & 255) << (8 * c);
        }
        const int c0 = j / P.run, y = c0 * parts.cycle + P.offset + (j - c0 * P.run);
        const int x = k * 64 + l;
        if (x < W) frame[(size_t)y * W + x] = px | 0xFF000000u;
    }
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
    const long long S = (W + 63) / 64;
    return 8 + ((4ll * n + 7) & ~7ll) + ((n * S + 7) & ~7ll) + 8ll * kSegWords * n * S;
}

long long wire_workspace(int W, int n) {
    const long long S = (W + 63) / 64;
    return 8ll * kSegWords * n * S + 4ll * n;
}

hipError_t launch_wire_encode(const uint32_t* rows, int W, int n, uint8_t* msg, void* workspace,
                              long long* size_out, hipStream_t s) {
    const int S = (W + 63) / 64;
    uint64_t* slots = reinterpret_cast<uint64_t*>(workspace);
    uint32_t* row_words = reinterpret_cast<uint32_t*>(slots + (size_t)kSegWords * n * S);
    uint8_t* counts = msg + 8 + (((size_t)4 * n + 7) & ~(size_t)7);
    hipError_t e = hipMemsetAsync(row_words, 0, (size_t)4 * n, s);
    if (e != hipSuccess) return e;
    if (n > 0) {
        hipLaunchKernelGGL(rm_wire_seg_encode, dim3(S, n), dim3(64), 0, s, rows, W, n, slots, counts, row_words);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(rm_wire_row_scan, dim3(1), dim3(1024), 0, s, row_words, n, S, msg, size_out);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (n > 0) hipLaunchKernelGGL(rm_wire_compact, dim3(S, n), dim3(64), 0, s, slots, n, msg);
    return hipGetLastError();
}

hipError_t launch_wire_decode(const uint8_t* msg, int n, int W, int cycle, int offset, int run, uint32_t* frame,
                              hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int S = (W + 63) / 64;
    hipLaunchKernelGGL(rm_wire_decode, dim3(S, n), dim3(64), 0, s, msg, n, W, cycle, offset, run, frame);
    return hipGetLastError();
}

hipError_t launch_wire_decode_parts(const WireParts& parts, int W, uint32_t* frame, hipStream_t s) {
    int rows = 0;
    for (int i = 0; i < parts.n; i++) rows = parts.part[i].nrows > rows ? parts.part[i].nrows : rows;
    if (parts.n <= 0 || rows <= 0) return hipSuccess;
    const int S = (W + 63) / 64;
    hipLaunchKernelGGL(rm_wire_decode_parts, dim3(S, rows < 65535 ? rows : 65535, parts.n), dim3(64), 0, s, parts,
                       W, frame);
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
