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
// Work mapping: one (TU, mode) job per G-lane group (G = N*N/4, at most 64).
// The group stages the 4N+1 neighbours in LDS — flipped for horizontal modes,
// loaded as dwords — plus, for negative angles, the N projected reference
// samples, so every angular pixel is two LDS reads and one blend.  The mode
// is decoded once per job from packed register constants (no table loads).
// Each lane produces 4 adjacent output pixels per step in the OUTPUT
// orientation, so stores are contiguous and no transpose pass is needed.
#include "common.h"
#include "../../../include/x265_amd.h"

namespace x265amd {

constexpr int kMaxN = 32;
constexpr int kLdsPerJob = 5 * kMaxN + 2;   // 4N+1 neighbours + N projected

// |intraPredAngle| for |angleOffset| = 0..8: 0 2 5 9 13 17 21 26 32 (6 bits each)
constexpr uint64_t kAngleMag = 0ull | (2ull << 6) | (5ull << 12) | (9ull << 18) | (13ull << 24) | (17ull << 30) |
                               (21ull << 36) | (26ull << 42) | (32ull << 48);
// invAngle for angle = -2 .. -32 indexed by |angleOffset| - 1 (16 bits each)
constexpr uint64_t kInvLo = 256ull | (315ull << 16) | (390ull << 32) | (482ull << 48);
constexpr uint64_t kInvHi = 630ull | (910ull << 16) | (1638ull << 32) | (4096ull << 48);

struct ModeInfo
{
    int angle;     // signed intraPredAngle (0 for planar / DC)
    int inv;       // invAngle (negative angles only)
    bool hor;      // horizontal mode: flipped neighbours, transposed output
};

__device__ __forceinline__ ModeInfo decode_mode(int mode)
{
    ModeInfo mi;
    mi.hor = mode >= 2 && mode < 18;
    const int off = mode < 2 ? 0 : (mi.hor ? 10 - mode : mode - 26);   // -8 .. 8
    const int a = off < 0 ? -off : off;
    const int mag = (int)((kAngleMag >> (6 * a)) & 63);
    mi.angle = off < 0 ? -mag : mag;
    // invAngleTable[-angleOffset - 1] for negative offsets: 4096, 1638, ... at |off| = 1 .. 8
    const int k = 8 - a;   // 0 .. 7 -> 256 ... 4096 ascending
    mi.inv = (int)(((k < 4 ? kInvLo >> (16 * k) : kInvHi >> (16 * (k - 4)))) & 0xffff);
    return mi;
}

template <typename P>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_intra_pred(int N, int lg2, int n, int lg, int maxv,
    P* __restrict__ dst, intptr_t ds, const int64_t* __restrict__ doff,
    const P* __restrict__ nb, const int64_t* __restrict__ nboff,
    const P* __restrict__ filt, const int64_t* __restrict__ filtoff,
    const uint8_t* __restrict__ mode, const uint8_t* __restrict__ bfilter, int allangs)
{
    const int G = 1 << lg;
    __shared__ int16_t sh[X265AMD_BLOCK / 4][kLdsPerJob];   // G >= 4
    const int slot = threadIdx.x >> lg, lane = threadIdx.x & (G - 1);
    const int64_t job = (int64_t)xcd_block() * (X265AMD_BLOCK >> lg) + slot;
    const bool live = job < n;
    const int64_t jj = live ? job : 0;
    int16_t* S = sh[slot];              // 4N+1 neighbours (flipped for horizontal modes)
    int16_t* Pj = S + 4 * N + 1;        // projected samples: ref[-2-k] = Pj[k]

    int m, bf;
    const P* src;
    P* out;
    if (allangs)
    {
        // job = tu * 33 + (mode - 2); unfiltered or filtered neighbours per g_intraFilterFlags
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
    const ModeInfo mi = decode_mode(m);
    const int n2 = 2 * N, tot = 4 * N + 1;

    // ---- stage neighbours: 4 elements per lane per step, flip applied on the LDS write
    for (int e0 = lane * 4; e0 < tot; e0 += G * 4)
    {
        int v[4];
        if (e0 + 4 <= tot) load_row<P, 4>(src + e0, v);
        else
        {
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = e0 + k < tot ? src[e0 + k] : 0;
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
        {
            const int e = e0 + k;
            if (e < tot)
            {
                const int d = (!mi.hor || e == 0) ? e : (e <= n2 ? e + n2 : e - n2);
                S[d] = (int16_t)v[k];
            }
        }
    }
    // ---- projected left samples for negative angles (intrapred.cpp:152-164)
    if (mi.angle < 0)
    {
        const int nproj = -((N * mi.angle) >> 5) - 1;
        for (int k = lane; k < nproj; k += G)
        {
            const int si = n2 + ((128 + (k + 1) * mi.inv) >> 8);   // index into the flipped array
            const int e = (!mi.hor || si == 0) ? si : (si <= n2 ? si + n2 : si - n2);
            Pj[k] = (int16_t)src[e];
        }
    }
    __syncthreads();

    // DC value: group reduction of above + left (all groups run it; used for mode 1 only)
    int part = 0;
    for (int i = lane; i < n2; i += G) part += S[i < N ? 1 + i : N + 1 + i];   // above[i] / left[i - N]
    for (int k = G >> 1; k > 0; k >>= 1) part += __shfl_xor(part, k, 64);
    const int dc = (part + N) / (2 * N);

    if (!live) return;
    const bool transposed = !allangs;
    const int per_row = N / 4, units = per_row * N;
    const intptr_t ostride = allangs ? N : ds;
    for (int u = lane; u < units; u += G)
    {
        const int r = u / per_row, c = (u % per_row) * 4;
        int v[4];
        if (m == 0)   // planar (intrapred.cpp:87-100)
        {
            const int16_t* above = S + 1;
            const int16_t* left = S + n2 + 1;
#pragma unroll
            for (int k = 0; k < 4; k++)
                v[k] = ((N - 1 - (c + k)) * left[r] + (N - 1 - r) * above[c + k] + (c + k + 1) * above[N] +
                        (r + 1) * left[N] + N) >> (lg2 + 1);
        }
        else if (m == 1)   // DC (+ dcPredFilter when bFilter)
        {
#pragma unroll
            for (int k = 0; k < 4; k++)
            {
                const int x = c + k;
                int p = dc;
                if (bf)
                {
                    if (r == 0 && x == 0) p = (S[1] + S[n2 + 1] + 2 * dc + 2) >> 2;
                    else if (r == 0) p = (S[1 + x] + 3 * dc + 2) >> 2;
                    else if (x == 0) p = (S[n2 + 1 + r] + 3 * dc + 2) >> 2;
                }
                v[k] = p;
            }
        }
        else
        {
#pragma unroll
            for (int k = 0; k < 4; k++)
            {
                // vertical-frame coordinates of output pixel (r, c + k)
                const int y = (mi.hor && transposed) ? c + k : r;
                const int x = (mi.hor && transposed) ? r : c + k;
                int p;
                if (mi.angle == 0)
                {
                    p = S[1 + x];
                    if (bf && x == 0)
                    {
                        const int t = (int16_t)(S[1] + ((S[n2 + 1 + y] - S[0]) >> 1));
                        p = t < 0 ? 0 : (t > maxv ? maxv : t);
                    }
                }
                else
                {
                    const int sum = (y + 1) * mi.angle, off = sum >> 5, f = sum & 31;
                    const int i0 = off + x, i1 = i0 + 1;
                    const int a = i0 >= -1 ? S[1 + i0] : Pj[-2 - i0];
                    const int b = i1 >= -1 ? S[1 + i1] : Pj[-2 - i1];
                    p = f ? ((32 - f) * a + f * b + 16) >> 5 : a;
                }
                v[k] = p;
            }
        }
        store_row<P, 4>(out + (int64_t)r * ostride + c, v);
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
                       (1 << depth) - 1, (P*)dst, ds, doff, (const P*)nb, nboff, (const P*)filt, filtoff, mode,
                       bfilter, allangs);
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
    if (depth == 8)
        return launch_pred<uint8_t>(size, n, depth, dst, dst_stride, dst_off, nb, nb_off, nullptr, nullptr, mode, bfilter, 0, st);
    if (depth == 10 || depth == 12)
        return launch_pred<uint16_t>(size, n, depth, dst, dst_stride, dst_off, nb, nb_off, nullptr, nullptr, mode, bfilter, 0, st);
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
