// intra.hip — batched intra reference smoothing and planar / DC / angular
// prediction (+ all-angles).
//
// Reference semantics: x265_1.9/source/common/intrapred.cpp
//   intraFilter :31-51   dcPredFilter :53-67   intra_pred_dc_c :69-85
//   planar_pred_c :87-100   intra_pred_ang_c :102-204   all_angs_pred_c :206-234
// Bit-exactness: horizontal modes (< 18) predict
// from the flipped neighbour array and transpose the block; the projected
// left neighbours use invAngleSum starting at 128; the mode-10/26 edge filter
// is x265_clip((int16_t)(top + ((left[y] - topLeft) >> 1))).  all-angles
// stores horizontal modes UN-transposed (intrapred.cpp:219-233).
//
// Work mapping: one (TU, mode) job per G-lane group; the 4N+1 neighbours are
// staged in LDS once per job (already flipped for horizontal modes); each
// lane then produces 4 horizontally adjacent output pixels per step, writing
// the output orientation directly (no separate transpose pass), so stores of
// a row are contiguous.
#include "common.h"
#include "../../../include/x265_amd.h"

namespace x265amd {

constexpr int kMaxNb = 4 * 32 + 1;

// value of the angular reference array ref[j] (intrapred.cpp:143-170), from
// the (flipped) neighbour array s[]
__device__ __forceinline__ int ang_ref(const int16_t* s, int j, int N, int inv_angle)
{
    if (j >= 0) return s[1 + j];
    if (j == -1) return s[0];
    return s[2 * N + ((128 + (-1 - j) * inv_angle) >> 8)];
}

// predicted pixel at (y, x) in the vertical frame of an angular mode
__device__ __forceinline__ int ang_pixel(const int16_t* s, int N, int angle, int inv_angle, int y, int x)
{
    const int sum = (y + 1) * angle, off = sum >> 5, f = sum & 31;
    const int a = ang_ref(s, off + x, N, inv_angle);
    if (!f) return a;
    const int b = ang_ref(s, off + x + 1, N, inv_angle);
    return ((32 - f) * a + f * b + 16) >> 5;
}

// One output pixel (r, c) of mode `mode` for an NxN block.  `transposed` =
// true gives the reference's final orientation for horizontal modes; false
// keeps the vertical frame (all-angles layout).
__device__ __forceinline__ int pred_pixel(const int16_t* s, int N, int lg2, int mode, int bfilter, int dc,
                                          int maxv, int r, int c, bool transposed)
{
    if (mode == 0)   // planar (unflipped neighbours)
    {
        const int16_t* above = s + 1;
        const int16_t* left = s + 2 * N + 1;
        return ((N - 1 - c) * left[r] + (N - 1 - r) * above[c] + (c + 1) * above[N] + (r + 1) * left[N] + N) >> (lg2 + 1);
    }
    if (mode == 1)   // DC
    {
        if (bfilter)
        {
            const int16_t* above = s + 1;
            const int16_t* left = s + 2 * N + 1;
            if (r == 0 && c == 0) return (above[0] + left[0] + 2 * dc + 2) >> 2;
            if (r == 0) return (above[c] + 3 * dc + 2) >> 2;
            if (c == 0) return (left[r] + 3 * dc + 2) >> 2;
        }
        return dc;
    }
    const bool hor = mode < 18;
    const int aoff = hor ? 10 - mode : mode - 26;
    const int angle = c_intra.angle[8 + aoff];
    // vertical-frame coordinates
    const int y = (hor && transposed) ? c : r;
    const int x = (hor && transposed) ? r : c;
    if (angle == 0)
    {
        if (bfilter && x == 0)
        {
            const int v = (int16_t)(s[1] + ((s[2 * N + 1 + y] - s[0]) >> 1));
            return v < 0 ? 0 : (v > maxv ? maxv : v);
        }
        return s[1 + x];
    }
    const int inv = angle < 0 ? c_intra.inv_angle[-aoff - 1] : 0;
    return ang_pixel(s, N, angle, inv, y, x);
}

// stage 4N+1 neighbours into LDS, flipping for horizontal angular modes
template <typename P>
__device__ __forceinline__ void stage_nb(int16_t* s, const P* nb, int N, bool flip, int lane, int G)
{
    const int tot = 4 * N + 1, n2 = 2 * N;
    for (int i = lane; i < tot; i += G)
    {
        int src = i;
        if (flip && i > 0) src = i <= n2 ? i + n2 : i - n2;
        s[i] = (int16_t)nb[src];
    }
}

template <typename P>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_intra_pred(int N, int lg2, int n, int lg, int maxv,
    P* __restrict__ dst, intptr_t ds, const int64_t* __restrict__ doff,
    const P* __restrict__ nb, const int64_t* __restrict__ nboff,
    const P* __restrict__ filt, const int64_t* __restrict__ filtoff,
    const uint8_t* __restrict__ mode, const uint8_t* __restrict__ bfilter, int allangs)
{
    const int G = 1 << lg;
    __shared__ int16_t sh[X265AMD_BLOCK / 4][kMaxNb];   // G >= 4
    const int slot = threadIdx.x >> lg, lane = threadIdx.x & (G - 1);
    const int64_t job = (int64_t)xcd_block() * (X265AMD_BLOCK >> lg) + slot;
    const bool live = job < n;
    const int64_t jj = live ? job : 0;
    int16_t* s = sh[slot];

    int m, bf;
    const P* src;
    P* out;
    if (allangs)
    {
        // job = tu * 33 + (mode - 2); source = filtered or unfiltered neighbours per g_intraFilterFlags
        const int64_t tu = jj / 33;
        m = 2 + (int)(jj % 33);
        bf = bfilter[tu];
        src = (c_intra.filter_flags[m] & N) ? filt + filtoff[tu] : nb + nboff[tu];
        out = dst + doff[tu] + (int64_t)(m - 2) * N * N;
    }
    else
    {
        m = mode[jj];
        bf = bfilter[jj];
        src = nb + nboff[jj];
        out = dst + doff[jj];
    }
    stage_nb<P>(s, src, N, m >= 2 && m < 18, lane, G);
    __syncthreads();

    int dc = 0;
    if (m == 1)
    {
        int t = N;
        for (int i = 0; i < N; i++) t += s[1 + i] + s[2 * N + 1 + i];
        dc = t / (2 * N);
    }
    if (live)
    {
        const int per_row = N / 4, units = per_row * N;
        for (int u = lane; u < units; u += G)
        {
            const int r = u / per_row, c = (u % per_row) * 4;
            int v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = pred_pixel(s, N, lg2, m, bf, dc, maxv, r, c + k, !allangs);
            store_row<P, 4>(out + (int64_t)r * (allangs ? N : ds) + c, v);
        }
    }
}

template <typename P>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_intra_filter(int N, int n, const P* __restrict__ src,
    const int64_t* __restrict__ soff, P* __restrict__ dst, const int64_t* __restrict__ doff)
{
    const int64_t job = (int64_t)xcd_block() * (X265AMD_BLOCK / 64) + threadIdx.x / 64;
    const int lane = threadIdx.x & 63;
    if (job >= n) return;
    const P* s = src + soff[job];
    P* d = dst + doff[job];
    const int n2 = 2 * N, n4 = 4 * N;
    for (int i = lane; i <= n4; i += 64)
    {
        int v;
        if (i == n2 || i == n4) v = s[i];
        else if (i == 0) v = (2 * s[0] + s[1] + s[n2 + 1] + 2) >> 2;
        else if (i == n2 + 1) v = (2 * s[n2 + 1] + s[0] + s[n2 + 2] + 2) >> 2;
        else v = (2 * s[i] + s[i - 1] + s[i + 1] + 2) >> 2;
        d[i] = (P)v;
    }
}

template <typename P>
static int launch_pred(int N, int n, int depth, void* dst, intptr_t ds, const int64_t* doff, const void* nb,
                       const int64_t* nboff, const void* filt, const int64_t* filtoff, const uint8_t* mode,
                       const uint8_t* bfilter, int allangs, hipStream_t st)
{
    int lg2 = 0;
    while ((1 << lg2) < N) lg2++;
    int g = N * N / 4;
    if (g > 64) g = 64;
    int lg = 0;
    while ((1 << lg) < g) lg++;
    const int per = X265AMD_BLOCK >> lg;
    hipLaunchKernelGGL(k_intra_pred<P>, dim3((n + per - 1) / per), dim3(X265AMD_BLOCK), 0, st, N, lg2, n, lg,
                       (1 << depth) - 1, (P*)dst, ds, doff, (const P*)nb, nboff, (const P*)filt, filtoff, mode, bfilter, allangs);
    return (int)hipGetLastError();
}

} // namespace x265amd

using namespace x265amd;

static bool valid_tu(int size) { return size == 4 || size == 8 || size == 16 || size == 32; }

extern "C" int x265amd_intra_filter(int depth, int size, int n, const void* src, const int64_t* src_off,
                                    void* dst, const int64_t* dst_off, void* stream)
{
    if (n <= 0) return 0;
    if (!valid_tu(size)) return X265AMD_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((n + 3) / 4);
    if (depth == 8)
        hipLaunchKernelGGL(k_intra_filter<uint8_t>, grid, dim3(X265AMD_BLOCK), 0, st, size, n, (const uint8_t*)src, src_off, (uint8_t*)dst, dst_off);
    else if (depth == 10 || depth == 12)
        hipLaunchKernelGGL(k_intra_filter<uint16_t>, grid, dim3(X265AMD_BLOCK), 0, st, size, n, (const uint16_t*)src, src_off, (uint16_t*)dst, dst_off);
    else
        return X265AMD_EINVAL;
    return (int)hipGetLastError();
}

extern "C" int x265amd_intra_pred(int depth, int size, int n, void* dst, intptr_t dst_stride, const int64_t* dst_off,
                                  const void* nb, const int64_t* nb_off, const uint8_t* mode, const uint8_t* bfilter,
                                  void* stream)
{
    if (n <= 0) return 0;
    if (!valid_tu(size)) return X265AMD_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    if (depth == 8) return launch_pred<uint8_t>(size, n, depth, dst, dst_stride, dst_off, nb, nb_off, nullptr, nullptr, mode, bfilter, 0, st);
    if (depth == 10 || depth == 12) return launch_pred<uint16_t>(size, n, depth, dst, dst_stride, dst_off, nb, nb_off, nullptr, nullptr, mode, bfilter, 0, st);
    return X265AMD_EINVAL;
}

extern "C" int x265amd_intra_allangs(int depth, int size, int n, void* dst, const int64_t* dst_off,
                                    const void* ref, const int64_t* ref_off, const void* filt,
                                    const int64_t* filt_off, const uint8_t* bluma, void* stream)
{
    if (n <= 0) return 0;
    if (!valid_tu(size)) return X265AMD_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    if (depth == 8)
        return launch_pred<uint8_t>(size, n * 33, depth, dst, 0, dst_off, ref, ref_off, filt, filt_off, nullptr, bluma, 1, st);
    if (depth == 10 || depth == 12)
        return launch_pred<uint16_t>(size, n * 33, depth, dst, 0, dst_off, ref, ref_off, filt, filt_off, nullptr, bluma, 1, st);
    return X265AMD_EINVAL;
}
