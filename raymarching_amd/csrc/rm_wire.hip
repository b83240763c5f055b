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
// into the message; the decoder scans a row's segment sizes in LDS and
// rebuilds each segment with a wave-wide prefix sum of the differences.
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

// exclusive scan of a row's S segment word counts into sh[0..S) (S <= 4096),
// the row's total returned; 256 threads
__device__ __forceinline__ void row_seg_offsets(const uint8_t* counts, int S, uint32_t* sh) {
    const int t = threadIdx.x;
    for (int k = t; k < S; k += 256) sh[k] = counts[k];
    __syncthreads();
    if (t < 64) {  // one wave: sequential chunks of the scan, lane-parallel within 64
        uint32_t carry = 0;
        for (int k0 = 0; k0 < S; k0 += 64) {
            const int k = k0 + t;
            uint32_t v = k < S ? sh[k] : 0u, inc = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t u = __shfl_up(inc, o, 64);
                if (t >= o) inc += u;
            }
            if (k < S) sh[k] = carry + inc - v;
            carry += __shfl(inc, 63, 64);
        }
    }
    __syncthreads();
}

// E3: one workgroup per row: the row's slots, compacted into the payload
__global__ __launch_bounds__(256) void rm_wire_compact(const uint64_t* __restrict__ slots, int n, int S,
                                                       uint8_t* __restrict__ msg) {
    extern __shared__ uint32_t seg_off[];
    const int j = blockIdx.x;
    const size_t hb = wire_header_bytes(n, S);
    const uint8_t* counts = msg + 8 + (((size_t)4 * n + 7) & ~(size_t)7) + (size_t)j * S;
    row_seg_offsets(counts, S, seg_off);
    const uint32_t base = reinterpret_cast<const uint32_t*>(msg + 8)[j];
    uint64_t* payload = reinterpret_cast<uint64_t*>(msg + hb) + base;
    const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
    for (int k = wv; k < S; k += 4) {
        const int cnt = counts[k];
        if (l < cnt) payload[seg_off[k] + l] = slots[((size_t)j * S + k) * kSegWords + l];
    }
}

// D: one workgroup per packed row of a part: its segments rebuilt into frame
// row y(j) (the part's rows: (y mod cycle) - offset in [0, run))
__global__ __launch_bounds__(256) void rm_wire_decode(const uint8_t* __restrict__ msg, int n, int W, int cycle,
                                                      int offset, int run, uint32_t* __restrict__ frame) {
    extern __shared__ uint32_t seg_off[];
    const int j = blockIdx.x, S = (W + 63) / 64;
    const size_t hb = wire_header_bytes(n, S);
    const uint8_t* counts = msg + 8 + (((size_t)4 * n + 7) & ~(size_t)7) + (size_t)j * S;
    row_seg_offsets(counts, S, seg_off);
    const uint32_t base = reinterpret_cast<const uint32_t*>(msg + 8)[j];
    const uint64_t* payload = reinterpret_cast<const uint64_t*>(msg + hb) + base;
    const int c0 = j / run, y = c0 * cycle + offset + (j - c0 * run);
    uint32_t* dst = frame + (size_t)y * W;
    const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
    for (int k = wv; k < S; k += 4) {
        const uint64_t* sw = payload + seg_off[k];
        const int cnt = counts[k];
        const uint64_t mine = l < cnt ? sw[l] : 0ull;  // lane 0: header, lane q + 1: plane q
        const uint32_t h_lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)mine);
        const uint32_t h_hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(mine >> 32));
        const int b[3] = {(int)((h_lo >> 24) & 15u), (int)(h_lo >> 28), (int)(h_hi & 15u)};
        uint32_t px = 0;
        int q = 1;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            uint32_t z = 0;
            for (int i = 0; i < b[c]; i++, q++) {
                const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mine, q);
                const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(mine >> 32), q);
                const uint32_t bit = l < 32 ? (lo >> l) & 1u : (hi >> (l - 32)) & 1u;
                z |= bit << i;
            }
            int d = l == 0 ? (int)((h_lo >> (8 * c)) & 255u) : unzigzag8(z);
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {  // inclusive prefix sum over the lanes
                const int u = __shfl_up(d, o, 64);
                if (l >= o) d += u;
            }
            px |= (uint32_t)(d & 255) << (8 * c);
        }
        const int x = k * 64 + l;
        if (x < W) dst[x] = px | 0xFF000000u;
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
    if (n > 0) hipLaunchKernelGGL(rm_wire_compact, dim3(n), dim3(256), (size_t)4 * S, s, slots, n, S, msg);
    return hipGetLastError();
}

hipError_t launch_wire_decode(const uint8_t* msg, int n, int W, int cycle, int offset, int run, uint32_t* frame,
                              hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int S = (W + 63) / 64;
    hipLaunchKernelGGL(rm_wire_decode, dim3(n), dim3(256), (size_t)4 * S, s, msg, n, W, cycle, offset, run, frame);
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
