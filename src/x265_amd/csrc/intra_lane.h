// intra_lane.h — one intra prediction (TU, mode) per lane, for 4x4 / 8x8
// blocks (intrapred.cpp:69-204): shared by the batched intra kernel
// (intra.hip, k_intra_lane) and the lookahead's lowres intra estimate
// (lowres.hip).  See intra.hip for the work mapping.
#pragma once
#include "common.h"

namespace x265amd {

// |intraPredAngle| for |angleOffset| = 0..8: 0 2 5 9 13 17 21 26 32 (6 bits each)
constexpr uint64_t kAngleMag = 0ull | (2ull << 6) | (5ull << 12) | (9ull << 18) | (13ull << 24) | (17ull << 30) |
                               (21ull << 36) | (26ull << 42) | (32ull << 48);
// invAngle (intrapred.cpp:124) for |angleOffset| = 8 .. 1, 16 bits each
constexpr uint64_t kInvLo = 256ull | (315ull << 16) | (390ull << 32) | (482ull << 48);
constexpr uint64_t kInvHi = 630ull | (910ull << 16) | (1638ull << 32) | (4096ull << 48);

struct ModeInfo
{
    int angle;     // signed intraPredAngle (0 for planar / DC / pure H / pure V)
    int inv;       // invAngle, used for negative angles
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
    const int k = 8 - a;
    mi.inv = (int)(((k < 4 ? kInvLo >> (16 * k) : kInvHi >> (16 * (k - 4)))) & 0xffff);
    return mi;
}

// element e of the neighbour array as seen by a mode (flip swaps above/left)
__device__ __forceinline__ int flip_index(int e, int n2, bool hor)
{
    return (!hor || e == 0) ? e : (e <= n2 ? e + n2 : e - n2);
}

// Predict N x N block `m` from the 4N+1 neighbours at src into v (in the
// mode's frame: horizontal modes come out transposed).  Angular modes use the
// lane's private LDS column D[.][threadIdx.x] (3N entries).
// neighbours s[0 .. 4N] of one TU (vector loads)
template <typename P, int N>
__device__ __forceinline__ void intra_lane_load(const P* src, int (&s)[4 * N + 1])
{
    constexpr int NB = 4 * N + 1;
#pragma unroll
    for (int i = 0; i + 16 <= NB; i += 16)
    {
        int t[16];
        load_row<P, 16>(src + i, t);
#pragma unroll
        for (int k = 0; k < 16; k++) s[i + k] = t[k];
    }
    s[NB - 1] = src[NB - 1];
}

template <int N>
__device__ __forceinline__ ModeInfo intra_lane_predict(const int (&s)[4 * N + 1], int m, int bf, int maxv,
                                                       uint32_t (*D)[X265AMD_BLOCK], int (&v)[N][N])
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    constexpr int N2 = 2 * N;
    constexpr int LG2 = N == 4 ? 2 : 3;
    const ModeInfo mi = decode_mode(m);

    // the mode's frame of the neighbours
    int R[3 * N + 1];                                // R[j + N], j = -N .. 2N
    int L[N + 1];
#pragma unroll
    for (int k = 0; k < N - 1; k++) R[k] = 0;         // j < -1: projected samples (angle < 0) only
#pragma unroll
    for (int e = 0; e <= N2; e++)
    {
        const int fe = e == 0 ? 0 : e + N2;
        R[N + e - 1] = mi.hor ? s[fe] : s[e];
    }
    R[3 * N] = 0;
#pragma unroll
    for (int y = 0; y <= N; y++)
    {
        const int e = N2 + 1 + y;
        L[y] = mi.hor ? s[e - N2] : s[e];
    }

    if (m == 0)   // planar (intrapred.cpp:87-100)
    {
#pragma unroll
        for (int y = 0; y < N; y++)
#pragma unroll
            for (int x = 0; x < N; x++)
                v[y][x] = ((N - 1 - x) * L[y] + (N - 1 - y) * R[N + x] + (x + 1) * R[2 * N] + (y + 1) * L[N] + N)
                          >> (LG2 + 1);
    }
    else if (m == 1)   // DC (+ dcPredFilter, intrapred.cpp:53-85)
    {
        int t = N;
#pragma unroll
        for (int i = 0; i < N; i++) t += R[N + i] + L[i];
        const int dc = t >> (LG2 + 1);
#pragma unroll
        for (int y = 0; y < N; y++)
#pragma unroll
            for (int x = 0; x < N; x++) v[y][x] = dc;
        if (bf)
        {
            v[0][0] = (R[N] + L[0] + 2 * dc + 2) >> 2;
#pragma unroll
            for (int x = 1; x < N; x++) v[0][x] = (R[N + x] + 3 * dc + 2) >> 2;
#pragma unroll
            for (int y = 1; y < N; y++) v[y][0] = (L[y] + 3 * dc + 2) >> 2;
        }
    }
    else if (mi.angle == 0)   // pure vertical / horizontal (+ edge filter)
    {
#pragma unroll
        for (int y = 0; y < N; y++)
        {
#pragma unroll
            for (int x = 0; x < N; x++) v[y][x] = R[N + x];
            if (bf)
            {
                const int t = (int16_t)(R[N] + ((L[y] - R[N - 1]) >> 1));
                v[y][0] = t < 0 ? 0 : (t > maxv ? maxv : t);
            }
        }
    }
    else
    {
        if (mi.angle < 0)
        {
            // projected left samples R[-2-k] = L[i_k - 1], i_k = (128 + (k+1)·invAngle) >> 8
            const int nproj = -((N * mi.angle) >> 5) - 1;
#pragma unroll
            for (int k = 0; k < N - 1; k++)
            {
                if (k < nproj)
                {
                    const int i = (128 + (k + 1) * mi.inv) >> 8;
                    int p = L[0];
#pragma unroll
                    for (int q = 1; q < N; q++) p = i - 1 == q ? L[q] : p;
                    R[N - 2 - k] = p;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 3 * N; j++) D[j][threadIdx.x] = (uint32_t)R[j] | ((uint32_t)R[j + 1] << 16);
#pragma unroll
        for (int y = 0; y < N; y++)
        {
            const int sum = (y + 1) * mi.angle, off = sum >> 5, f = sum & 31;
            const u16x2 wt = {(unsigned short)(32 - f), (unsigned short)f};
            const uint32_t* row = &D[N + off][threadIdx.x];
#pragma unroll
            for (int x = 0; x < N; x++)
                v[y][x] = (int)(__builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, row[x * X265AMD_BLOCK]), wt, 16u, false) >> 5);
        }
    }

    return mi;
}

} // namespace x265amd
