// transform1d.h — exact integer 1-D HEVC transforms shared by the batched
// transform kernels (transform.hip) and the fused TU pipeline (tu.hip).
//
// Reference: x265_1.9/source/common/dct.cpp — partialButterfly{4,8,16,32}
// :83-240,418-440, partialButterflyInverse* :242-416, fastForwardDst :41-61,
// inversedst :63-81.  The even/odd decomposition below is an exact integer
// refactoring of the matrix product (no intermediate rounding), so the
// per-stage rounding (fwd_round / inv_round) reproduces the reference exactly.
#pragma once
#include "common.h"

namespace x265amd {

constexpr TransformMatrix kT32 = make_t32();

template <int N>
__device__ __forceinline__ constexpr int tcoef(int k, int n)
{
    return kT32.m[k * (32 / N)][n];
}

// forward N-point transform of x[] (exact integer), result in y[]
template <int N>
__device__ __forceinline__ void fwd_1d(const int (&x)[N], int (&y)[N])
{
    if constexpr (N == 4)
    {
        const int e0 = x[0] + x[3], o0 = x[0] - x[3], e1 = x[1] + x[2], o1 = x[1] - x[2];
        y[0] = 64 * e0 + 64 * e1;
        y[2] = 64 * e0 - 64 * e1;
        y[1] = 83 * o0 + 36 * o1;
        y[3] = 36 * o0 - 83 * o1;
    }
    else
    {
        int e[N / 2], o[N / 2], ye[N / 2];
#pragma unroll
        for (int k = 0; k < N / 2; k++) { e[k] = x[k] + x[N - 1 - k]; o[k] = x[k] - x[N - 1 - k]; }
        fwd_1d<N / 2>(e, ye);
#pragma unroll
        for (int m = 0; m < N / 2; m++) y[2 * m] = ye[m];
#pragma unroll
        for (int m = 0; m < N / 2; m++)
        {
            int s = 0;
#pragma unroll
            for (int k = 0; k < N / 2; k++) s += tcoef<N>(2 * m + 1, k) * o[k];
            y[2 * m + 1] = s;
        }
    }
}

// inverse N-point transform of coefficient vector c[] (exact integer)
template <int N>
__device__ __forceinline__ void inv_1d(const int (&c)[N], int (&y)[N])
{
    if constexpr (N == 4)
    {
        const int o0 = 83 * c[1] + 36 * c[3], o1 = 36 * c[1] - 83 * c[3];
        const int e0 = 64 * c[0] + 64 * c[2], e1 = 64 * c[0] - 64 * c[2];
        y[0] = e0 + o0; y[1] = e1 + o1; y[2] = e1 - o1; y[3] = e0 - o0;
    }
    else
    {
        int ce[N / 2], e[N / 2];
#pragma unroll
        for (int m = 0; m < N / 2; m++) ce[m] = c[2 * m];
        inv_1d<N / 2>(ce, e);
#pragma unroll
        for (int k = 0; k < N / 2; k++)
        {
            int o = 0;
#pragma unroll
            for (int m = 0; m < N / 2; m++) o += tcoef<N>(2 * m + 1, k) * c[2 * m + 1];
            y[k] = e[k] + o;
            y[N - 1 - k] = e[k] - o;
        }
    }
}

__device__ __forceinline__ int fwd_round(int s, int shift) { return (int)(int16_t)((s + (1 << (shift - 1))) >> shift); }
__device__ __forceinline__ int inv_round(int s, int shift) { return clip16((s + (1 << (shift - 1))) >> shift); }

// DST-VII 4-point (fastForwardDst / inversedst), exact integer
__device__ __forceinline__ void dst_fwd(const int (&b)[4], int (&y)[4])
{
    const int c0 = b[0] + b[3], c1 = b[1] + b[3], c2 = b[0] - b[1], c3 = 74 * b[2];
    y[0] = 29 * c0 + 55 * c1 + c3;
    y[1] = 74 * (b[0] + b[1] - b[3]);
    y[2] = 29 * c2 + 55 * c0 - c3;
    y[3] = 55 * c2 - 29 * c1 + c3;
}
__device__ __forceinline__ void dst_inv(const int (&t)[4], int (&y)[4])
{
    const int c0 = t[0] + t[2], c1 = t[2] + t[3], c2 = t[0] - t[3], c3 = 74 * t[1];
    y[0] = 29 * c0 + 55 * c1 + c3;
    y[1] = 55 * c2 - 29 * c1 + c3;
    y[2] = 74 * (t[0] - t[2] + t[3]);
    y[3] = 55 * c0 + 29 * c2 - c3;
}

// f16 matrix-core operand types and the exact hi/lo split of int16 operands
// (x = hi * 2048 + lo, both exact in f16; see k_tr32_mfma in transform.hip)
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int K, typename V>
__device__ __forceinline__ void split_hl(const int (&x)[K], V& lo, V& hi)
{
#pragma unroll
    for (int j = 0; j < K; j++)
    {
        lo[j] = (_Float16)(uint16_t)(x[j] & 2047);
        hi[j] = (_Float16)(int16_t)(x[j] >> 11);
    }
}

// The same split on packed int16 pairs (x0 | x1 << 16) with 10-bit halves, built from
// f16 bit patterns instead of conversions: 0x6400 | (x & 1023) is the f16 1024 + lo (one
// v_and_or per pair) and ((x as uint16) >> 10) ^ 0x6420 is the f16 1056 + hi
// (0x6400 | ((x >> 10) + 32): a packed shift and a xor per pair); one packed f16 add per
// pair removes the 1024 / 1056 offsets exactly, leaving lo in [0, 1023] and hi in [-32, 31]
// (x = 1024·hi + lo), so an MFMA sum over them stays as small as split_hl's.
typedef unsigned short u16x2v __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t split10_lo(uint32_t u)
{
    uint32_t r;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(u), "v"(0x03FF03FFu), "v"(0x64006400u));
    const f16x2v f = __builtin_bit_cast(f16x2v, r) - (f16x2v){(_Float16)1024, (_Float16)1024};
    return __builtin_bit_cast(uint32_t, f);
}
__device__ __forceinline__ uint32_t split10_hi(uint32_t u)
{
    const u16x2v b = __builtin_bit_cast(u16x2v, u) >> (u16x2v){10, 10};
    const f16x2v f = __builtin_bit_cast(f16x2v, __builtin_bit_cast(uint32_t, b) ^ 0x64206420u) -
                     (f16x2v){(_Float16)1056, (_Float16)1056};
    return __builtin_bit_cast(uint32_t, f);
}
// NP packed pairs -> 2·NP f16 operand lanes (element j = half j of the pairs)
template <int NP, typename V>
__device__ __forceinline__ void split10(const uint32_t (&u)[NP], V& lo, V& hi)
{
    uint32_t l[NP], h[NP];
#pragma unroll
    for (int i = 0; i < NP; i++)
    {
        l[i] = split10_lo(u[i]);
        h[i] = split10_hi(u[i]);
    }
    lo = __builtin_bit_cast(V, l);
    hi = __builtin_bit_cast(V, h);
}
// two int values (int16 range) packed as a pair
__device__ __forceinline__ uint32_t pack16(int a, int b) { return __builtin_amdgcn_perm((uint32_t)b, (uint32_t)a, 0x05040100u); }
// split10 of K int values (int16 range): packed in pairs first (one v_perm per pair)
template <int K, typename V>
__device__ __forceinline__ void split10i(const int (&x)[K], V& lo, V& hi)
{
    uint32_t u[K / 2];
#pragma unroll
    for (int i = 0; i < K / 2; i++) u[i] = pack16(x[2 * i], x[2 * i + 1]);
    split10<K / 2>(u, lo, hi);
}

} // namespace x265amd
