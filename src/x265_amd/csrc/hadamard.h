// hadamard.h — 8x8 Hadamard sums and the psyCost_pp energy of an 8x8 block (pixel.cpp:672-703, the
// sa8d_8x8 against zero minus the SAD against zero / 4), shared by the primitive kernels (pixel.hip) and the
// RDO server (tu.hip).  Included inside namespace x265amd, after common.h.
#pragma once

// raw 8x8 Hadamard |coef| sum (x265 _sa8d_8x8 before rounding)
__device__ __forceinline__ uint32_t had8x8(int (&d)[8][8])
{
#pragma unroll
    for (int i = 0; i < 8; i++)
    {
        int a0 = d[i][0] + d[i][1], a1 = d[i][0] - d[i][1];
        int a2 = d[i][2] + d[i][3], a3 = d[i][2] - d[i][3];
        int a4 = d[i][4] + d[i][5], a5 = d[i][4] - d[i][5];
        int a6 = d[i][6] + d[i][7], a7 = d[i][6] - d[i][7];
        int b0 = a0 + a2, b2 = a0 - a2, b1 = a1 + a3, b3 = a1 - a3;
        int b4 = a4 + a6, b6 = a4 - a6, b5 = a5 + a7, b7 = a5 - a7;
        d[i][0] = b0 + b4; d[i][4] = b0 - b4; d[i][1] = b1 + b5; d[i][5] = b1 - b5;
        d[i][2] = b2 + b6; d[i][6] = b2 - b6; d[i][3] = b3 + b7; d[i][7] = b3 - b7;
    }
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < 8; j++)
    {
        int a0 = d[0][j] + d[1][j], a1 = d[0][j] - d[1][j];
        int a2 = d[2][j] + d[3][j], a3 = d[2][j] - d[3][j];
        int a4 = d[4][j] + d[5][j], a5 = d[4][j] - d[5][j];
        int a6 = d[6][j] + d[7][j], a7 = d[6][j] - d[7][j];
        int b0 = a0 + a2, b2 = a0 - a2, b1 = a1 + a3, b3 = a1 - a3;
        int b4 = a4 + a6, b6 = a4 - a6, b5 = a5 + a7, b7 = a5 - a7;
        s += abs(b0 + b4) + abs(b0 - b4) + abs(b1 + b5) + abs(b1 - b5)
           + abs(b2 + b6) + abs(b2 - b6) + abs(b3 + b7) + abs(b3 - b7);
    }
    return s;
}

// ---- 8-bit 8x8 Hadamard on packed 16-bit pairs (v_pk_add/sub_i16).
// Inputs of magnitude <= 255 (8-bit pixels, or differences of them) keep every
// butterfly value within 64 * 255 = 16320, so int16 lanes are exact and the
// whole transform costs half the VALU of the int32 one.  Q[k][j] holds rows
// (2k, 2k+1) of column j.
typedef short s16x2 __attribute__((ext_vector_type(2)));

// sum of |v.lo + v.hi| + |v.lo - v.hi| over the pairs of x and y: the last
// butterfly stage (over the two rows one register holds) fused with the |.|
// sums, |v| = sad_u16(v ^ 0x8000, 0x8000) on both halves at once
__device__ __forceinline__ uint32_t abs_pair_sum(s16x2 x, s16x2 y, uint32_t s)
{
    const s16x2 lo = {x.x, y.x}, hi = {x.y, y.y};
    const s16x2 u = lo + hi, w = lo - hi;
    s = __builtin_amdgcn_sad_u16(__builtin_bit_cast(uint32_t, u) ^ 0x80008000u, 0x80008000u, s);
    return __builtin_amdgcn_sad_u16(__builtin_bit_cast(uint32_t, w) ^ 0x80008000u, 0x80008000u, s);
}

// rows 2k, 2k+1 (8 bytes each) -> Q[k][0..7] as zero-extended 16-bit pairs
__device__ __forceinline__ void pack_rows8(uint2 r0, uint2 r1, s16x2 (&q)[8])
{
#pragma unroll
    for (int j = 0; j < 4; j++)
    {
        const uint32_t sel = 0x0c040c00u + (uint32_t)j * 0x00010001u;   // (r0.b[j], 0, r1.b[j], 0)
        q[j] = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(r1.x, r0.x, sel));
        q[4 + j] = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(r1.y, r0.y, sel));
    }
}

__device__ __forceinline__ void bfly8(s16x2 (&v)[8])
{
    const s16x2 a0 = v[0] + v[1], a1 = v[0] - v[1], a2 = v[2] + v[3], a3 = v[2] - v[3];
    const s16x2 a4 = v[4] + v[5], a5 = v[4] - v[5], a6 = v[6] + v[7], a7 = v[6] - v[7];
    const s16x2 b0 = a0 + a2, b2 = a0 - a2, b1 = a1 + a3, b3 = a1 - a3;
    const s16x2 b4 = a4 + a6, b6 = a4 - a6, b5 = a5 + a7, b7 = a5 - a7;
    v[0] = b0 + b4; v[4] = b0 - b4; v[1] = b1 + b5; v[5] = b1 - b5;
    v[2] = b2 + b6; v[6] = b2 - b6; v[3] = b3 + b7; v[7] = b3 - b7;
}

// Σ|coef| of the 8x8 Hadamard (x265 _sa8d_8x8 before rounding)
__device__ __forceinline__ uint32_t had8x8_pk(s16x2 (&Q)[4][8])
{
#pragma unroll
    for (int k = 0; k < 4; k++) bfly8(Q[k]);                 // row transforms (over columns)
#pragma unroll
    for (int j = 0; j < 8; j++)                              // column stages over row bits 1 and 2
    {
        const s16x2 c0 = Q[0][j] + Q[1][j], c1 = Q[0][j] - Q[1][j];
        const s16x2 c2 = Q[2][j] + Q[3][j], c3 = Q[2][j] - Q[3][j];
        Q[0][j] = c0 + c2; Q[2][j] = c0 - c2; Q[1][j] = c1 + c3; Q[3][j] = c1 - c3;
    }
    // last stage over row bit 0 (the two halves of a pair), fused with |.| sums
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int j = 0; j < 8; j += 2) s = abs_pair_sum(Q[k][j], Q[k][j + 1], s);
    return s;
}

// raw sa8d of one 8x8 (8-bit): differences formed on the packed pairs
__device__ __forceinline__ uint32_t raw_sa8d_pk(const uint8_t* a, intptr_t sa, const uint8_t* b, intptr_t sb)
{
    s16x2 Q[4][8];
#pragma unroll
    for (int k = 0; k < 4; k++)
    {
        s16x2 qa[8], qb[8];
        pack_rows8(ldu<uint2>(a + 2 * k * sa), ldu<uint2>(a + (2 * k + 1) * sa), qa);
        pack_rows8(ldu<uint2>(b + 2 * k * sb), ldu<uint2>(b + (2 * k + 1) * sb), qb);
#pragma unroll
        for (int j = 0; j < 8; j++) Q[k][j] = qa[j] - qb[j];
    }
    return had8x8_pk(Q);
}

// psy energy of one 8x8 (8-bit): sa8d against zero minus sad against zero / 4
__device__ __forceinline__ int psy_energy8_pk(const uint8_t* a, intptr_t sa)
{
    s16x2 Q[4][8];
    uint32_t sad = 0;
#pragma unroll
    for (int k = 0; k < 4; k++)
    {
        const uint2 r0 = ldu<uint2>(a + 2 * k * sa), r1 = ldu<uint2>(a + (2 * k + 1) * sa);
        sad = __builtin_amdgcn_sad_u8(r0.x, 0u, sad);
        sad = __builtin_amdgcn_sad_u8(r0.y, 0u, sad);
        sad = __builtin_amdgcn_sad_u8(r1.x, 0u, sad);
        sad = __builtin_amdgcn_sad_u8(r1.y, 0u, sad);
        pack_rows8(r0, r1, Q[k]);
    }
    return (int)((had8x8_pk(Q) + 2) >> 2) - (int)(sad >> 2);
}

// energy helpers for psyCost_pp: Hadamard of the block itself (zero reference)
template <typename P>
__device__ __forceinline__ int psy_energy8(const P* a, intptr_t sa)
{
    if constexpr (sizeof(P) == 1) return psy_energy8_pk(a, sa);
    int d[8][8];
    uint32_t sad = 0;
#pragma unroll
    for (int y = 0; y < 8; y++)
    {
        int va[8];
        load_row<P, 8>(a + y * sa, va);
#pragma unroll
        for (int x = 0; x < 8; x++) { d[y][x] = va[x]; sad += va[x]; }
    }
    int sa8d = (int)((had8x8(d) + 2) >> 2);
    return sa8d - (int)(sad >> 2);
}

