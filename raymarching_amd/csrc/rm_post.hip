// rm_post.hip -- the bloom post pass of the reference (shaders/post/bloom.frag
// with the mip chain of main.cpp:212-214) over an RGBA8 frame (SURVEY.md
// 8(f), rank 3).  The FXAA pass is rm_fxaa.hip; the helpers both use are in
// rm_post_common.h.
//
// Built without FMA contraction and with correctly rounded division (like
// rm_kernels_o.hip) so the float path is bit-identical to the restatement in
// oracle/rm_oracle.c.
#include "rm_post_common.h"

namespace rm {

// ------------------------------------------------------------------ bloom
//
// shaders/post/bloom.frag:14-43 over the mip chain of main.cpp:212-214
// (postTexture.setSmooth(true); generateMipmap(): MIN LINEAR_MIPMAP_LINEAR,
// MAG LINEAR, CLAMP_TO_EDGE).  Only the levels bloom.frag reads are built:
// textureLod at lod = log2(0.05 H) blends levels floor(lod) and floor(lod)+1.
// A level is the bilinear resample of the one above at its texel centres in
// the 0..255 domain, rounded to nearest even (SwiftShader's glGenerateMipmap,
// bit for bit on even sizes; tests/test_bloom.py).  Same float operations,
// in the same order, as oracle/rm_oracle.c (no contraction in this TU).

__device__ __forceinline__ int clampi(int v, int hi) { return v < 0 ? 0 : (v > hi ? hi : v); }

__global__ __launch_bounds__(256) void rm_mip_down_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                          int w, int h, int w1, int h1, float sx, float sy) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= w1 || y >= h1) return;
    const float v = ((float)y + 0.5f) * sy - 0.5f, u = ((float)x + 0.5f) * sx - 0.5f;
    const float fy = floorf(v), fx = floorf(u), b = v - fy, a = u - fx;
    const int y0 = clampi((int)fy, h - 1), y1 = clampi((int)fy + 1, h - 1);
    const int x0 = clampi((int)fx, w - 1), x1 = clampi((int)fx + 1, w - 1);
    const uint32_t t00 = in[(size_t)y0 * w + x0], t01 = in[(size_t)y0 * w + x1];
    const uint32_t t10 = in[(size_t)y1 * w + x0], t11 = in[(size_t)y1 * w + x1];
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < 32; c += 8) {
        const float c00 = (float)((t00 >> c) & 255u), c01 = (float)((t01 >> c) & 255u);
        const float c10 = (float)((t10 >> c) & 255u), c11 = (float)((t11 >> c) & 255u);
        const float r0 = (1.0f - a) * c00 + a * c01, r1 = (1.0f - a) * c10 + a * c11;
        r |= (uint32_t)__float2int_rn((1.0f - b) * r0 + b * r1) << c;
    }
    out[(size_t)y * w1 + x] = r;
}

// Exact halvings (even level sizes): mip_mean4 (rm_post_common.h).

// The mip levels below `src` (sw texels wide) by exact halvings, 2^(lgB + 5)
// levels' worth of one src tile per workgroup: 1024 lanes, each reducing a
// B x B block (B = 2^lgB) in registers to one texel, then five levels in LDS
// (32 x 32 -> 1).  Levels jA and jB below src (the two bloom.frag reads, always
// among the last five) are written, with widths sw >> jA, sw >> jB.
template <int LGB>
__global__ __launch_bounds__(1024) void rm_mip_pyramid_kernel(const uint32_t* __restrict__ src, int sw,
                                                              uint32_t* __restrict__ outA, int jA,
                                                              uint32_t* __restrict__ outB, int jB) {
    constexpr int B = 1 << LGB, T = 32 * B;
    __shared__ uint32_t L[2][1024];
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    const uint32_t* p = src + ((size_t)blockIdx.y * T + ty * B) * sw + (size_t)blockIdx.x * T + tx * B;
    uint32_t v[B][B];
#pragma unroll
    for (int r = 0; r < B; r++) {
        if constexpr (B >= 4) {
#pragma unroll
            for (int c = 0; c < B; c += 4) {
                const uint4 q = *reinterpret_cast<const uint4*>(p + (size_t)r * sw + c);
                v[r][c] = q.x;
                v[r][c + 1] = q.y;
                v[r][c + 2] = q.z;
                v[r][c + 3] = q.w;
            }
        } else {
#pragma unroll
            for (int c = 0; c < B; c++) v[r][c] = p[(size_t)r * sw + c];
        }
    }
#pragma unroll
    for (int n = B / 2; n >= 1; n /= 2)
#pragma unroll
        for (int r = 0; r < n; r++)
#pragma unroll
            for (int c = 0; c < n; c++)
                v[r][c] = mip_mean4(v[2 * r][2 * c], v[2 * r][2 * c + 1], v[2 * r + 1][2 * c], v[2 * r + 1][2 * c + 1]);
    L[0][threadIdx.x] = v[0][0];
    __syncthreads();
    int cur = 0;
#pragma unroll
    for (int j = 1; j <= 5; j++) {
        const int n = 32 >> j, lev = LGB + j;
        if ((int)threadIdx.x < n * n) {
            const int x = threadIdx.x % n, y = threadIdx.x / n;
            const uint32_t* q = L[cur] + 2 * y * (2 * n) + 2 * x;
            const uint32_t r = mip_mean4(q[0], q[1], q[2 * n], q[2 * n + 1]);
            L[cur ^ 1][y * n + x] = r;
            if (lev == jA) outA[((size_t)blockIdx.y * n + y) * (sw >> jA) + (size_t)blockIdx.x * n + x] = r;
            if (lev == jB) outB[((size_t)blockIdx.y * n + y) * (sw >> jB) + (size_t)blockIdx.x * n + x] = r;
        }
        cur ^= 1;
        __syncthreads();
    }
}

struct Level {
    const uint32_t* p;
    int w, h;
};

// The bilinear filter as the polynomial of its cell (oracle tex_bilinear):
// c00 + a Px + b (Py + a Pxy), Px = c01 - c00, Py = c10 - c00,
// Pxy = (c11 - c10) - Px, three fused multiply-adds per channel.
__device__ __forceinline__ float cell_poly(float c00, float px, float py, float pxy, float a, float b) {
    return fmaf(b, fmaf(a, pxy, py), fmaf(a, px, c00));
}

// bilinear fetch at normalized (u, v), CLAMP_TO_EDGE, unorm8 -> c * (1/255)
__device__ __forceinline__ RGB tex_bilinear(Level L, float u, float v) {
    const float x = u * (float)L.w - 0.5f, y = v * (float)L.h - 0.5f;
    const float fx = floorf(x), fy = floorf(y), a = x - fx, b = y - fy;
    const int x0 = clampi((int)fx, L.w - 1), x1 = clampi((int)fx + 1, L.w - 1);
    const int y0 = clampi((int)fy, L.h - 1), y1 = clampi((int)fy + 1, L.h - 1);
    const uint32_t t00 = L.p[(size_t)y0 * L.w + x0], t01 = L.p[(size_t)y0 * L.w + x1];
    const uint32_t t10 = L.p[(size_t)y1 * L.w + x0], t11 = L.p[(size_t)y1 * L.w + x1];
    float o[3];
    const float k = 1.0f / 255.0f;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const int s = 8 * c;
        const float c00 = (float)((t00 >> s) & 255u) * k, c01 = (float)((t01 >> s) & 255u) * k;
        const float c10 = (float)((t10 >> s) & 255u) * k, c11 = (float)((t11 >> s) & 255u) * k;
        const float px = c01 - c00, py = c10 - c00, pxy = (c11 - c10) - px;
        o[c] = cell_poly(c00, px, py, pxy, a, b);
    }
    return RGB{o[0], o[1], o[2]};
}

__constant__ const float kGauss[3][3] = {{41.0f / 273.0f, 26.0f / 273.0f, 7.0f / 273.0f},
                                         {26.0f / 273.0f, 16.0f / 273.0f, 4.0f / 273.0f},
                                         {7.0f / 273.0f, 4.0f / 273.0f, 1.0f / 273.0f}};

// bloom.frag:33-43, one lane per output pixel, 16x16-pixel workgroups.  The
// general form: any lod, the levels read as RGBA8 words.  Used when lod <= 0
// (magnification: every tap reads the base level).
__global__ __launch_bounds__(256) void rm_bloom_kernel(Level L0, uint32_t* __restrict__ out, int W, int H) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= W || y >= H) return;
    const float u = ((float)x + 0.5f) / (float)W, v = 1.0f - ((float)y + 0.5f) / (float)H;  // bloom.frag:36
    RGB color = tex_bilinear(L0, u, v);
    const float scale = 0.05f, iaspect = (float)H / (float)W;
    RGB bl{0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int j = -2; j <= 2; j++)
#pragma unroll
        for (int i = -2; i <= 2; i++) {
            const float uu = u + ((float)i * iaspect) * scale, vv = v + (float)j * scale;
            const RGB s = tex_bilinear(L0, uu, vv);
            const float g = kGauss[i < 0 ? -i : i][j < 0 ? -j : j];
            bl = RGB{fmaf(g, s.r, bl.r), fmaf(g, s.g, bl.g), fmaf(g, s.b, bl.b)};
        }
    color = RGB{color.r + gmax_(bl.r - 0.3f, 0.0f), color.g + gmax_(bl.g - 0.3f, 0.0f),
                color.b + gmax_(bl.b - 0.3f, 0.0f)};
    out[(size_t)y * W + x] = unorm8(color.r) | (unorm8(color.g) << 8) | (unorm8(color.b) << 16) | (255u << 24);
}

// ---- bloom.frag:33-43 for lod > 0 (minification: levels d1, d2 blended by fr)
//
// Tap (i, j) of a level of w x h texels samples the bilinear cell
// (cx_i, cy_j) = floor(s + dx_i, t + dy_j), with s = u w - 0.5,
// t = v h - 0.5 the pixel's position in texels and dx_i = off_i w,
// dy_j = off_j h bloom.frag's tap offsets.  Inside a cell the sample is
// c00 + a Px + b Py + a b Pxy (a, b the position within the cell), so with
// the 25 cells fixed the weighted 5 x 5 sum is one bilinear polynomial of the
// pixel's position: P00 + P10 s' + P01 t' + P11 s' t', s' = s - cx_2,
// t' = t - cy_2.  Along the pixel columns the five cells change at most
// 5 w + 1 times, so the columns fall into runs of equal cell tuples (rows
// likewise); every (column run, row run) pair of a level gets its polynomial,
// summed in double over the 25 taps with the level's blend weight (1 - fr,
// fr) folded in and rounded to float.  A pixel then evaluates two
// polynomials: 3 fused multiply-adds per channel per level, against 4 per
// channel per tap per level in the per-tap form (rounds 3-5, 1475 FLOP/px).
// The sum is the same function of the same texels; it differs from the
// per-tap float sum by float rounding only (~1e-6 against a 1/255 output
// step), and the oracle restates this order (oracle bloom_runs / bloom_poly /
// bloom_pixel), pinned to SwiftShader by tests/test_bloom.py.
//
// rm_bloom_runs_kernel: one workgroup per axis (d1 x, d1 y, d2 x, d2 y) finds
// the runs (a block scan of the columns where the cell tuple changes) and
// writes per column (s', run) and per run its cell tuple; two more workgroups
// write the base level's bilinear axis per column and per row (the pixel's
// own texel, bloom.frag:40).  These depend on W x H only: computed once per
// size and stream (launch_bloom's `runs_cached`).
// rm_bloom_poly_kernel: eight lanes per (column run, row run) pair of a level.
// rm_bloom_min_kernel: one lane per column of a 16-row strip; the rows' entries
// are wave-uniform scalar loads, and a lane reloads its two polynomials only
// when a row run changes (runs span ~25 rows at 4096^2).

struct BloomAxis {
    int n, N, lw, is_y;  // pixels along the axis, the image size, the level's size, the v axis
    float off[5];        // bloom.frag's offset of tap i along the axis (u: (i iaspect) scale, v: j scale)
};
struct BloomAxes {
    BloomAxis a[4];  // level d1 x, y; level d2 x, y
};
struct BloomEnt {
    float sub;  // s' (or t'): the pixel's position from its run's centre-tap cell
    int run;
};
struct BloomBase {
    float f;  // the base level's bilinear weight along the axis
    int fl;   // floor of the texel coordinate (clamped at the fetch)
};
struct BloomRunsOut {
    BloomBase* base[2];  // per column, per row
    BloomEnt* ent[4];
    int* tup[4];  // 5 cells per run
    int* count;   // runs per axis
};
struct BloomTabs {
    const uint32_t* tex[2];
    const int* tup[4];
    const int* count;
    float* tab[2];  // 12 floats per run pair: P00 rgb, P10 rgb, P01 rgb, P11 rgb
    int nx[2], ny[2];
    double lam[2];  // 1 - fr, fr
};
struct BloomPix {
    const BloomBase* base[2];
    const BloomEnt* ent[4];
    const float* tab[2];
    int nx[2];
};

__device__ __forceinline__ float bloom_coord(const BloomAxis& A, int c) {
    const float t = ((float)c + 0.5f) / (float)A.N;
    return (A.is_y ? 1.0f - t : t) * (float)A.lw - 0.5f;  // bloom.frag:36, then the level's texel space
}
__device__ __forceinline__ int bloom_cell(const BloomAxis& A, float coord, int i) {
    const double d = (double)A.off[i] * (double)A.lw;  // exact: a float times a level size
    const double x = floor((double)coord + d);
    return x < -1.0 ? -1 : (x > (double)(A.lw - 1) ? A.lw - 1 : (int)x);  // cells -1 and lw-1 are the clamped edges
}

__global__ __launch_bounds__(1024) void rm_bloom_runs_kernel(BloomAxes axes, BloomRunsOut R) {
    __shared__ int sc[1024];
    if (blockIdx.x >= 4) {  // the base level (tex_bilinear(L0, u, v)'s axes; the whole workgroup, no barrier)
        const int yax = blockIdx.x - 4, n = yax ? axes.a[1].N : axes.a[0].N;
        for (int c = threadIdx.x; c < n; c += 1024) {
            const float t = ((float)c + 0.5f) / (float)n;
            const float x = (yax ? 1.0f - t : t) * (float)n - 0.5f, fx = floorf(x);
            R.base[yax][c] = BloomBase{x - fx, (int)fx};
        }
        return;
    }
    const BloomAxis& A = axes.a[blockIdx.x];
    BloomEnt* __restrict__ ent = R.ent[blockIdx.x];
    int* __restrict__ tup = R.tup[blockIdx.x];
    const int t = threadIdx.x, chunk = (A.n + 1023) / 1024;
    const int c0 = t * chunk < A.n ? t * chunk : A.n, c1 = c0 + chunk < A.n ? c0 + chunk : A.n;
    auto key = [&](int c) {
        const float coord = bloom_coord(A, c);
        int k = 0;
        for (int i = 0; i < 5; i++) k += bloom_cell(A, coord, i) + 1;
        return k;  // monotone along the axis: equal keys of neighbours = equal tuples
    };
    int prev = c0 > 0 ? key(c0 - 1) : -1, cnt = 0;
    for (int c = c0; c < c1; c++) {
        const int k = key(c);
        cnt += k != prev;
        prev = k;
    }
    sc[t] = cnt;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive block scan of the run starts
        const int v = t >= o ? sc[t - o] : 0;
        __syncthreads();
        sc[t] += v;
        __syncthreads();
    }
    int run = sc[t] - cnt - 1;
    prev = c0 > 0 ? key(c0 - 1) : -1;
    for (int c = c0; c < c1; c++) {
        const float coord = bloom_coord(A, c);
        int cell[5], k = 0;
        for (int i = 0; i < 5; i++) {
            cell[i] = bloom_cell(A, coord, i);
            k += cell[i] + 1;
        }
        if (k != prev) {
            run++;
            for (int i = 0; i < 5; i++) tup[run * 5 + i] = cell[i];
        }
        prev = k;
        ent[c] = BloomEnt{coord - (float)cell[2], run};
    }
    if (t == 1023) R.count[blockIdx.x] = sc[1023];
}

// One run pair per 8 lanes: lane j < 5 sums tap row j (its five taps in order),
// then lane 0 adds the five row sums in order (oracle bloom_poly).
__global__ __launch_bounds__(256) void rm_bloom_poly_kernel(BloomAxes axes, BloomTabs T) {
    __shared__ double part[32][5][12];
    const int l = blockIdx.z, slot = threadIdx.x >> 3, j = threadIdx.x & 7;
    const int pair = blockIdx.x * 32 + slot, nxl = T.nx[l];
    const int rx = pair % nxl, ry = pair / nxl;
    const bool live = ry < T.ny[l] && rx < T.count[2 * l] && ry < T.count[2 * l + 1];  // (this frame's runs)
    const BloomAxis &X = axes.a[2 * l], &Y = axes.a[2 * l + 1];
    const int w = X.lw, h = Y.lw;
    if (live && j < 5) {
        const uint32_t* __restrict__ L = T.tex[l];
        const int* tx = T.tup[2 * l] + rx * 5;
        const int* ty = T.tup[2 * l + 1] + ry * 5;
        const int cy = ty[j];
        const double f = ((double)ty[2] + (double)Y.off[j] * (double)h) - (double)cy;  // b_j = t' + f
        const int y0 = clampi(cy, h - 1), y1 = clampi(cy + 1, h - 1);
        double R[12] = {};  // in texel units (0..255); 1/255 is applied with the blend weight
#pragma unroll
        for (int i = 0; i < 5; i++) {
            const int cx = tx[i];
            const double e = ((double)tx[2] + (double)X.off[i] * (double)w) - (double)cx;  // a_i = s' + e
            const int x0 = clampi(cx, w - 1), x1 = clampi(cx + 1, w - 1);
            const uint32_t t00 = L[(size_t)y0 * w + x0], t01 = L[(size_t)y0 * w + x1];
            const uint32_t t10 = L[(size_t)y1 * w + x0], t11 = L[(size_t)y1 * w + x1];
            const double g = (double)kGauss[i < 2 ? 2 - i : i - 2][j < 2 ? 2 - j : j - 2];
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const int s = 8 * c;
                const double c00 = (double)((t00 >> s) & 255u), c01 = (double)((t01 >> s) & 255u);
                const double c10 = (double)((t10 >> s) & 255u), c11 = (double)((t11 >> s) & 255u);
                const double px = c01 - c00, py = c10 - c00, pxy = (c11 - c10) - px;  // (exact integers)
                R[c] += g * (((c00 + e * px) + f * py) + (e * f) * pxy);
                R[3 + c] += g * (px + f * pxy);
                R[6 + c] += g * (py + e * pxy);
                R[9 + c] += g * pxy;
            }
        }
#pragma unroll
        for (int q = 0; q < 12; q++) part[slot][j][q] = R[q];
    }
    __syncthreads();
    if (!live || j != 0) return;
    double P[12] = {};
    for (int r = 0; r < 5; r++)
#pragma unroll
        for (int q = 0; q < 12; q++) P[q] += part[slot][r][q];
    const double lam = T.lam[l] * (1.0 / 255.0);
    float4* dst = reinterpret_cast<float4*>(T.tab[l] + ((size_t)ry * nxl + rx) * 12);
    dst[0] = make_float4((float)(P[0] * lam), (float)(P[1] * lam), (float)(P[2] * lam), (float)(P[3] * lam));
    dst[1] = make_float4((float)(P[4] * lam), (float)(P[5] * lam), (float)(P[6] * lam), (float)(P[7] * lam));
    dst[2] = make_float4((float)(P[8] * lam), (float)(P[9] * lam), (float)(P[10] * lam), (float)(P[11] * lam));
}

constexpr int kBloomRows = 16;  // (strip A/B, profiles/r06/bloom_strip_ab.log)
template <typename T>
__device__ __forceinline__ T sload_entry(const T* base, int i) {  // a wave-uniform 8-byte entry via the scalar cache
    static_assert(sizeof(T) == 8, "8-byte entries");
    typedef const __attribute__((address_space(4))) unsigned long long* cptr;
    const unsigned long long v = ((cptr)(const void*)base)[i];
    T r;
    __builtin_memcpy(&r, &v, 8);
    return r;
}
// A lane's column is fixed, so each polynomial is kept as its two column
// halves, X = P10 s' + P00 and Y = P11 s' + P01 per channel (the inner
// multiply-adds of fmaf(fmaf(P11, s', P01), t', fmaf(P10, s', P00))), formed
// when a row run starts; a row is then fmaf(Y, t', X).  (Forming them right
// after the loads also keeps the loads' wait inside the rare reload branch,
// instead of a wait on every row for all earlier stores.)
struct PolyHalves {
    float X[3], Y[3];
};
__device__ __forceinline__ PolyHalves load_poly(const float* tab, uint32_t idx, float sx) {
    const float4* q = reinterpret_cast<const float4*>(tab + idx * 12u);
    const float4 q0 = q[0], q1 = q[1], q2 = q[2];  // P00 rgb, P10 rgb, P01 rgb, P11 rgb
    PolyHalves h;
    h.X[0] = fmaf(q0.w, sx, q0.x);
    h.X[1] = fmaf(q1.x, sx, q0.y);
    h.X[2] = fmaf(q1.y, sx, q0.z);
    h.Y[0] = fmaf(q2.y, sx, q1.z);
    h.Y[1] = fmaf(q2.z, sx, q1.w);
    h.Y[2] = fmaf(q2.w, sx, q2.x);
    return h;
}

// tex_bilinear(L0, u, v) from the base level's precomputed axes
__device__ __forceinline__ RGB base_bilinear(const uint32_t* r0, const uint32_t* r1, uint32_t c0, uint32_t c1, float a,
                                             float b) {
    const float k = 1.0f / 255.0f;
    const uint32_t t00 = r0[c0], t01 = r0[c1], t10 = r1[c0], t11 = r1[c1];
    float o[3];
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const int s = 8 * c;
        const float c00 = (float)((t00 >> s) & 255u) * k, c01 = (float)((t01 >> s) & 255u) * k;
        const float c10 = (float)((t10 >> s) & 255u) * k, c11 = (float)((t11 >> s) & 255u) * k;
        const float px = c01 - c00, py = c10 - c00, pxy = (c11 - c10) - px;
        o[c] = cell_poly(c00, px, py, pxy, a, b);
    }
    return RGB{o[0], o[1], o[2]};
}

// One lane per column of a kBloomRows strip, the rows in batches of
// kBloomBatch whose texel loads are issued together (the loads in flight per
// wave, not the arithmetic, bound a lone strip; 4 beat 8 by ~6%: fewer
// registers, more waves).
constexpr int kBloomBatch = 4;
__global__ __launch_bounds__(256) void rm_bloom_min_kernel(const uint32_t* __restrict__ in, BloomPix B,
                                                           uint32_t* __restrict__ out, int W, int H) {
    const int x = blockIdx.x * 256 + threadIdx.x;
    const int y0 = blockIdx.y * kBloomRows, y1 = y0 + kBloomRows < H ? y0 + kBloomRows : H;
    if (x >= W) return;
    const BloomBase bx = B.base[0][x];
    const uint32_t c0 = (uint32_t)clampi(bx.fl, W - 1), c1 = (uint32_t)clampi(bx.fl + 1, W - 1);
    const BloomEnt exA = B.ent[0][x], exB = B.ent[2][x];
    int ryA = -1, ryB = -1;
    PolyHalves pa, pb;
    const float k = 1.0f / 255.0f;
    for (int yb = y0; yb < y1; yb += kBloomBatch) {
        BloomEnt eyA[kBloomBatch], eyB[kBloomBatch];
        BloomBase by[kBloomBatch];
        bool frac_y = false;
#pragma unroll
        for (int r = 0; r < kBloomBatch; r++) {
            const int y = yb + r < y1 ? yb + r : y1 - 1;  // (rows past the strip repeat its last row, not stored)
            eyA[r] = sload_entry(B.ent[1], y);
            eyB[r] = sload_entry(B.ent[3], y);
            by[r] = sload_entry(B.base[1], y);
            frac_y = frac_y || by[r].f != 0.0f;
        }
        RGB color[kBloomBatch];
        if (__builtin_amdgcn_ballot_w64(bx.f != 0.0f || frac_y) == 0) {
            // both weights exactly 0: every multiply-add of the cell polynomial adds an exact zero,
            // the value is the pixel's own texel
            uint32_t t[kBloomBatch];
#pragma unroll
            for (int r = 0; r < kBloomBatch; r++) t[r] = (in + (size_t)clampi(by[r].fl, H - 1) * W)[c0];
#pragma unroll
            for (int r = 0; r < kBloomBatch; r++)
                color[r] = RGB{(float)(t[r] & 255u) * k, (float)((t[r] >> 8) & 255u) * k,
                               (float)((t[r] >> 16) & 255u) * k};
        } else {
#pragma unroll
            for (int r = 0; r < kBloomBatch; r++)
                color[r] = base_bilinear(in + (size_t)clampi(by[r].fl, H - 1) * W,
                                         in + (size_t)clampi(by[r].fl + 1, H - 1) * W, c0, c1, bx.f, by[r].f);
        }
#pragma unroll
        for (int r = 0; r < kBloomBatch; r++) {
            if (yb + r >= y1) break;
            if (eyA[r].run != ryA) {  // (wave-uniform)
                ryA = eyA[r].run;
                pa = load_poly(B.tab[0], (uint32_t)(ryA * B.nx[0] + exA.run), exA.sub);
            }
            if (eyB[r].run != ryB) {
                ryB = eyB[r].run;
                pb = load_poly(B.tab[1], (uint32_t)(ryB * B.nx[1] + exB.run), exB.sub);
            }
            const float ta = eyA[r].sub, tb = eyB[r].sub;
            const RGB bl{fmaf(pa.Y[0], ta, pa.X[0]) + fmaf(pb.Y[0], tb, pb.X[0]),
                         fmaf(pa.Y[1], ta, pa.X[1]) + fmaf(pb.Y[1], tb, pb.X[1]),
                         fmaf(pa.Y[2], ta, pa.X[2]) + fmaf(pb.Y[2], tb, pb.X[2])};
            const RGB c{color[r].r + gmax_(bl.r - 0.3f, 0.0f), color[r].g + gmax_(bl.g - 0.3f, 0.0f),
                        color[r].b + gmax_(bl.b - 0.3f, 0.0f)};
            out[(size_t)(yb + r) * W + x] =
                unorm8_finite(c.r) | (unorm8_finite(c.g) << 8) | (unorm8_finite(c.b) << 16) | (255u << 24);
        }
    }
}

BloomPlan bloom_plan(int W, int H) {
    BloomPlan p{};
    int q = 0;
    for (int m = W > H ? W : H; m > 1; m >>= 1) q++;
    p.lod = log2f(0.05f * (float)H);  // bloom.frag:22 (u_resolution = the image, post_bloom.cpp:6)
    if (p.lod > 0.0f) {
        p.d1 = (int)floorf(p.lod);
        p.d1 = p.d1 > q ? q : p.d1;
        p.d2 = p.d1 + 1 > q ? q : p.d1 + 1;
    }
    p.fr = p.lod - floorf(p.lod);
    int w = W, h = H;
    p.w[0] = W;
    p.h[0] = H;
    for (int k = 1; k <= p.d2; k++) {
        w = w > 1 ? w >> 1 : 1;
        h = h > 1 ? h >> 1 : 1;
        p.w[k] = w;
        p.h[k] = h;
        p.offset[k] = p.texels;
        p.texels += (size_t)w * h;
    }
    if (p.lod > 0.0f) {  // the runs and run-pair polynomials of levels d1, d2, 16-byte aligned
        auto al = [](size_t o) { return (o + 3) & ~(size_t)3; };
        const int n[4] = {W, H, W, H}, lw[4] = {p.w[p.d1], p.h[p.d1], p.w[p.d2], p.h[p.d2]};
        size_t o = al(p.texels);
        for (int a = 0; a < 2; a++) {
            p.base_ent[a] = o;
            o = al(o + 2 * (size_t)n[a]);
        }
        for (int a = 0; a < 4; a++) {
            p.run_ent[a] = o;
            o = al(o + 2 * (size_t)n[a]);
        }
        for (int a = 0; a < 4; a++) {
            const long long m = 5LL * lw[a] + 1;  // distinct cell tuples along the axis
            p.nruns[a] = (int)(n[a] < m ? n[a] : m);
            p.run_tup[a] = o;
            o = al(o + 5 * (size_t)p.nruns[a]);
        }
        p.run_count = o;
        o += 4;
        for (int l = 0; l < 2; l++) {
            p.poly_tab[l] = o;
            o += 12 * (size_t)p.nruns[2 * l] * p.nruns[2 * l + 1];
        }
        p.texels = o;
    }
    return p;
}

hipError_t launch_bloom(const uint32_t* in, uint32_t* out, uint32_t* mips, const BloomPlan& p, hipStream_t s,
                        bool runs_cached) {
    const int W = p.w[0], H = p.h[0];
    if (W <= 0 || H <= 0) return hipSuccess;
    const uint32_t* lv[40] = {in};
    // levels 1..d2: when W and H are multiples of 2^d2 every level is an exact
    // halving, and the last 5..8 levels come from one rm_mip_pyramid_kernel
    // launch over level s = max(d2 - 8, 0) (only d1, d2 written); otherwise,
    // and for levels 1..s, one rm_mip_down_kernel launch per level
    const long long T2 = 1LL << (p.d2 < 62 ? p.d2 : 62);
    const int s0 = p.d2 > 8 ? p.d2 - 8 : 0;
    const bool pyramid = p.lod > 0.0f && p.d2 - s0 >= 5 && W % T2 == 0 && H % T2 == 0;
    for (int k = 1; k <= (pyramid ? s0 : p.d2); k++) {
        uint32_t* dst = mips + p.offset[k];
        const int w = p.w[k - 1], h = p.h[k - 1], w1 = p.w[k], h1 = p.h[k];
        hipLaunchKernelGGL(rm_mip_down_kernel, dim3((w1 + 15) / 16, (h1 + 15) / 16), dim3(256), 0, s, lv[k - 1], dst,
                           w, h, w1, h1, (float)w / (float)w1, (float)h / (float)h1);
        lv[k] = dst;
    }
    if (pyramid) {
        const int nl = p.d2 - s0, lgb = nl - 5, T = 32 << lgb;
        for (int k = s0 + 1; k <= p.d2; k++) lv[k] = mips + p.offset[k];  // (only d1, d2 written)
        const dim3 g(p.w[s0] / T, p.h[s0] / T);
        uint32_t *oa = mips + p.offset[p.d1], *ob = mips + p.offset[p.d2];
        const int ja = p.d1 - s0, jb = p.d2 - s0;
        switch (lgb) {
            case 0: hipLaunchKernelGGL(rm_mip_pyramid_kernel<0>, g, dim3(1024), 0, s, lv[s0], p.w[s0], oa, ja, ob, jb); break;
            case 1: hipLaunchKernelGGL(rm_mip_pyramid_kernel<1>, g, dim3(1024), 0, s, lv[s0], p.w[s0], oa, ja, ob, jb); break;
            case 2: hipLaunchKernelGGL(rm_mip_pyramid_kernel<2>, g, dim3(1024), 0, s, lv[s0], p.w[s0], oa, ja, ob, jb); break;
            default: hipLaunchKernelGGL(rm_mip_pyramid_kernel<3>, g, dim3(1024), 0, s, lv[s0], p.w[s0], oa, ja, ob, jb); break;
        }
    }
    const Level L0{in, W, H};
    if (p.lod <= 0.0f) {
        hipLaunchKernelGGL(rm_bloom_kernel, dim3((W + 15) / 16, (H + 15) / 16), dim3(256), 0, s, L0, out, W, H);
        return hipGetLastError();
    }
    BloomAxes ax{};
    const float iaspect = (float)H / (float)W, scale = 0.05f;
    for (int a = 0; a < 4; a++) {
        BloomAxis& A = ax.a[a];
        const int lvl = a < 2 ? p.d1 : p.d2;
        A.is_y = a & 1;
        A.n = A.N = A.is_y ? H : W;
        A.lw = A.is_y ? p.h[lvl] : p.w[lvl];
        for (int i = 0; i < 5; i++) A.off[i] = A.is_y ? (float)(i - 2) * scale : ((float)(i - 2) * iaspect) * scale;
    }
    BloomRunsOut R{};
    BloomTabs T{};
    BloomPix P{};
    for (int a = 0; a < 2; a++) {
        R.base[a] = reinterpret_cast<BloomBase*>(mips + p.base_ent[a]);
        P.base[a] = R.base[a];
    }
    for (int a = 0; a < 4; a++) {
        R.ent[a] = reinterpret_cast<BloomEnt*>(mips + p.run_ent[a]);
        R.tup[a] = reinterpret_cast<int*>(mips + p.run_tup[a]);
        T.tup[a] = R.tup[a];
        P.ent[a] = R.ent[a];
    }
    R.count = reinterpret_cast<int*>(mips + p.run_count);
    T.count = R.count;
    for (int l = 0; l < 2; l++) {
        T.tex[l] = lv[l == 0 ? p.d1 : p.d2];
        T.tab[l] = reinterpret_cast<float*>(mips + p.poly_tab[l]);
        T.nx[l] = P.nx[l] = p.nruns[2 * l];
        T.ny[l] = p.nruns[2 * l + 1];
        P.tab[l] = T.tab[l];
    }
    T.lam[0] = (double)(1.0f - p.fr);
    T.lam[1] = (double)p.fr;
    if (!runs_cached) hipLaunchKernelGGL(rm_bloom_runs_kernel, dim3(6), dim3(1024), 0, s, ax, R);
    const int nx = T.nx[0] > T.nx[1] ? T.nx[0] : T.nx[1], ny = T.ny[0] > T.ny[1] ? T.ny[0] : T.ny[1];
    const long long npairs = (long long)nx * ny;
    hipLaunchKernelGGL(rm_bloom_poly_kernel, dim3((unsigned)((npairs + 31) / 32), 1, 2), dim3(256), 0, s, ax, T);
    hipLaunchKernelGGL(rm_bloom_min_kernel, dim3((W + 255) / 256, (H + kBloomRows - 1) / kBloomRows), dim3(256), 0, s,
                       in, P, out, W, H);
    return hipGetLastError();
}

}  // namespace rm
