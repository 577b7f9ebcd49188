// transform.hip — batched 2-D DCT / iDCT 4..32, DST / iDST 4x4, quant,
// nquant, dequant (normal, scaling), count_nonzero / copy_cnt.
//
// Reference semantics: x265_1.9/source/common/dct.cpp
//   fastForwardDst / inversedst :41-81      partialButterfly{4,8,16,32} :83-240,418-440
//   partialButterflyInverse*    :242-416    dst4/dct4..32 :442-525   idst4/idct4..32 :527-610
//   dequant_normal :612-634  dequant_scaling :636-662  quant :664-686  nquant :688-713
//   count_nonzero :714-726   copy_count :728-742
// Bit-exactness: forward stages wrap each
// result to int16, inverse stages clip; the even/odd butterfly used here is
// an exact integer refactoring of the matrix product (no intermediate
// rounding), so it reproduces the reference's partial butterflies exactly.
//
// Work mapping: N = 4 transforms run one job per lane; N = 8/16/32 run one
// job per N-lane group, lane r owning row r (forward) or column r (inverse)
// in stage 1, with the int16 intermediate staged through LDS (row pitch N+2
// to spread banks) for stage 2; global memory is only touched by rows (16-byte
// loads / stores), the column sides of both directions go through LDS.
#include <stdlib.h>

#include "common.h"
#include "transform1d.h"
#include "../../../include/x265_amd.h"

namespace x265amd {

// --------------------------------------------------------------- 4x4: lane per job
// Each lane takes kTr4Jobs jobs (jobs b + k * 256 + t: every wave-instruction still
// covers consecutive jobs) and issues the descriptor and block loads of all of them
// before the first transform, so one dependent offset -> block round trip serves
// several jobs.
constexpr int kTr4Jobs = 2;

template <int KIND>
__device__ __forceinline__ void tr4_load(const int16_t* ps, intptr_t ss, int (&m)[4][4])
{
    if (ss == 4)
    {
        // compact block (coefficients, compact residuals): 32 contiguous bytes, two 16-byte loads
        const uint4 a = ldu<uint4>(ps), b = ldu<uint4>(ps + 8);
        const uint32_t w[8] = { a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w };
#pragma unroll
        for (int i = 0; i < 16; i++) m[i >> 2][i & 3] = (int)(int16_t)(w[i >> 1] >> (16 * (i & 1)));
    }
    else
    {
#pragma unroll
        for (int r = 0; r < 4; r++)
        {
            int v[4];
            load_row16<4>(ps + r * ss, v);
#pragma unroll
            for (int c = 0; c < 4; c++) m[r][c] = v[c];
        }
    }
}

template <int KIND>
__device__ __forceinline__ void tr4_apply(int depth, int (&m)[4][4])
{
    int t[4][4];
    const bool fwd = KIND == X265AMD_DCT || KIND == X265AMD_DST;
    const int sh1 = fwd ? 1 + depth - 8 : 7, sh2 = fwd ? 8 : 12 - (depth - 8);
    if (fwd)
    {
        // stage 1: row i -> column i of t; stage 2: row i of t -> column i of out
#pragma unroll
        for (int i = 0; i < 4; i++)
        {
            int y[4];
            if (KIND == X265AMD_DST) dst_fwd(m[i], y); else fwd_1d<4>(m[i], y);
#pragma unroll
            for (int k = 0; k < 4; k++) t[k][i] = fwd_round(y[k], sh1);
        }
#pragma unroll
        for (int i = 0; i < 4; i++)
        {
            int y[4];
            if (KIND == X265AMD_DST) dst_fwd(t[i], y); else fwd_1d<4>(t[i], y);
#pragma unroll
            for (int k = 0; k < 4; k++) m[k][i] = fwd_round(y[k], sh2);
        }
    }
    else
    {
        // stage 1: column j of input -> row j of t; stage 2: column j of t -> row j of out
#pragma unroll
        for (int j = 0; j < 4; j++)
        {
            int c[4] = { m[0][j], m[1][j], m[2][j], m[3][j] }, y[4];
            if (KIND == X265AMD_IDST) dst_inv(c, y); else inv_1d<4>(c, y);
#pragma unroll
            for (int k = 0; k < 4; k++) t[j][k] = inv_round(y[k], sh1);
        }
#pragma unroll
        for (int j = 0; j < 4; j++)
        {
            int c[4] = { t[0][j], t[1][j], t[2][j], t[3][j] }, y[4];
            if (KIND == X265AMD_IDST) dst_inv(c, y); else inv_1d<4>(c, y);
#pragma unroll
            for (int k = 0; k < 4; k++) m[j][k] = inv_round(y[k], sh2);
        }
    }
}

__device__ __forceinline__ void tr4_store(int16_t* pd, intptr_t ds, const int (&m)[4][4])
{
    if (ds == 4)
    {
        uint32_t w[8];
#pragma unroll
        for (int i = 0; i < 8; i++)
            w[i] = (uint32_t)(uint16_t)m[(2 * i) >> 2][(2 * i) & 3] | ((uint32_t)(uint16_t)m[(2 * i + 1) >> 2][(2 * i + 1) & 3] << 16);
        stu<uint4>(pd, make_uint4(w[0], w[1], w[2], w[3]));
        stu<uint4>(pd + 8, make_uint4(w[4], w[5], w[6], w[7]));
        return;
    }
#pragma unroll
    for (int r = 0; r < 4; r++)
    {
        int v[4] = { m[r][0], m[r][1], m[r][2], m[r][3] };
        store_row<int16_t, 4>(pd + r * ds, v);
    }
}

template <int KIND>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_tr4(int n, int depth,
    const int16_t* __restrict__ src, intptr_t ss, const int64_t* __restrict__ soff,
    int16_t* __restrict__ dst, intptr_t ds, const int64_t* __restrict__ doff)
{
    const int64_t b = (int64_t)xcd_block() * X265AMD_BLOCK * kTr4Jobs + threadIdx.x;
    int m[kTr4Jobs][4][4];
    int64_t dof[kTr4Jobs];
#pragma unroll
    for (int k = 0; k < kTr4Jobs; k++)
    {
        const int64_t job = b + (int64_t)k * X265AMD_BLOCK;
        if (job < n)
        {
            dof[k] = doff[job];
            tr4_load<KIND>(src + soff[job], ss, m[k]);
        }
    }
#pragma unroll
    for (int k = 0; k < kTr4Jobs; k++)
    {
        const int64_t job = b + (int64_t)k * X265AMD_BLOCK;
        if (job >= n) break;
        tr4_apply<KIND>(depth, m[k]);
        tr4_store(dst + dof[k], ds, m[k]);
    }
}

// --------------------------------------------------------------- NxN: N lanes per job
template <int N, bool FWD>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_trN(int n, int depth,
    const int16_t* __restrict__ src, intptr_t ss, const int64_t* __restrict__ soff,
    int16_t* __restrict__ dst, intptr_t ds, const int64_t* __restrict__ doff)
{
    constexpr int P = N + 2;                   // LDS row pitch (int16)
    constexpr int JOBS = X265AMD_BLOCK / N;
    __shared__ int16_t lds[JOBS][N * P];
    const int slot = threadIdx.x / N, r = threadIdx.x % N;
    const int64_t job = (int64_t)xcd_block() * JOBS + slot;
    const bool live = job < n;
    const int64_t jj = live ? job : 0;
    int16_t* L = lds[slot];
    constexpr int logN = N == 8 ? 3 : N == 16 ? 4 : 5;

    if (FWD)
    {
        const int sh1 = logN - 1 + depth - 8, sh2 = logN + 6;
        int x[N], y[N];
        const int16_t* row = src + soff[jj] + r * ss;
#pragma unroll
        for (int i = 0; i < N; i += 8)
        {
            int t[8];
            load_row16<8>(row + i, t);
#pragma unroll
            for (int k = 0; k < 8; k++) x[i + k] = t[k];
        }
        fwd_1d<N>(x, y);
#pragma unroll
        for (int k = 0; k < N; k++) L[k * P + r] = (int16_t)fwd_round(y[k], sh1);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < N; i += 2)
        {
            uint32_t v = *(const uint32_t*)&L[r * P + i];
            x[i] = (int16_t)(v & 0xffff);
            x[i + 1] = (int16_t)(v >> 16);
        }
        fwd_1d<N>(x, y);
        // column r of the output -> LDS, then row r -> one 16-byte store per 8 coefficients
        __syncthreads();
#pragma unroll
        for (int k = 0; k < N; k++) L[k * P + r] = (int16_t)fwd_round(y[k], sh2);
        __syncthreads();
        if (live)
        {
            int16_t* pd = dst + doff[jj] + r * ds;
#pragma unroll
            for (int i = 0; i < N; i += 8)
            {
                uint32_t w[4];
#pragma unroll
                for (int q = 0; q < 4; q++) w[q] = *(const uint32_t*)&L[r * P + i + 2 * q];
                stu<uint4>(pd + i, make_uint4(w[0], w[1], w[2], w[3]));
            }
        }
    }
    else
    {
        const int sh1 = 7, sh2 = 12 - (depth - 8);
        int c[N], y[N];
        // row r of the coefficients by 16-byte loads, transposed through LDS into column r
        const int16_t* row = src + soff[jj] + r * ss;
#pragma unroll
        for (int i = 0; i < N; i += 8)
        {
            int t[8];
            load_row16<8>(row + i, t);
#pragma unroll
            for (int k = 0; k < 8; k++) L[(i + k) * P + r] = (int16_t)t[k];
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < N; i += 2)
        {
            const uint32_t v = *(const uint32_t*)&L[r * P + i];
            c[i] = (int16_t)(v & 0xffff);
            c[i + 1] = (int16_t)(v >> 16);
        }
        inv_1d<N>(c, y);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < N; k++) L[r * P + k] = (int16_t)inv_round(y[k], sh1);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < N; k++) c[k] = L[k * P + r];
        inv_1d<N>(c, y);
        if (live)
        {
            int16_t* pd = dst + doff[jj] + r * ds;
#pragma unroll
            for (int i = 0; i < N; i += 8)
            {
                int t[8];
#pragma unroll
                for (int k = 0; k < 8; k++) t[k] = inv_round(y[i + k], sh2);
                store_row<int16_t, 8>(pd + i, t);
            }
        }
    }
}

// --------------------------------------------------------------- 16x16 / 32x32 on MFMA
// One wavefront per transform; both stages are matrix products on the f16
// matrix cores with FP32 accumulation:  forward  Dst = T * (Src * T^T)^T,
// inverse  Res = (C^T * T)^T * T  (each stage rounded / wrapped or clipped to
// int16 exactly as partialButterfly*[Inverse]).  Exactness: every int16
// operand is split x = hi * 1024 + lo with lo in [0, 1023] and hi in
// [-32, 31] — both exact in f16 — and the two halves accumulate in separate
// FP32 tiles whose partial sums stay integers below 2^24 (|lo * t| summed over
// K = 32 is < 1023 * 90 * 32), so hi * 1024 + lo reproduces the int32 sum.
// The split works on packed int16 pairs with f16 bit patterns (transform1d.h
// split10: v_and_or / packed shift / xor / packed f16 add, no conversions), and
// the MFMA results stay in VGPRs (-amdgpu-mfma-vgpr-form, build.py): together
// 499 -> 388 VALU instructions per 32x32 forward iteration, dct / idct 16 / 32
// 0.46-0.52 -> 0.54-0.60 of HBM peak (profiles/r03/tr_split_ab.txt).
// The first stage's accumulator tile feeds the second MFMA straight from
// registers (column on the lane, rows in the registers: the second product
// sums over its row index), so no LDS is used.
constexpr int kTrWaves = X265AMD_BLOCK / 64;

// grid of a matrix-core transform launch: enough waves to fill the chip,
// each looping over transforms (the constant operands load once per wave)
static inline uint32_t mfma_grid(int n)
{
    // workgroup cap: 16384 measured 0-3 % faster than 4096 and 1024 / 2048 5-8 % slower
    // (profiles/r03/tr_grid_ab.txt); X265AMD_TR_GRID overrides it for tuning runs
    static const int64_t cap = getenv("X265AMD_TR_GRID") && atoi(getenv("X265AMD_TR_GRID")) > 0
                               ? atoi(getenv("X265AMD_TR_GRID")) : 16384;
    const int64_t want = ((int64_t)n + kTrWaves - 1) / kTrWaves;
    return (uint32_t)(want < cap ? want : cap);
}

template <bool FWD>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_tr32_mfma(int n, int depth,
    const int16_t* __restrict__ src, intptr_t ss, const int64_t* __restrict__ soff,
    int16_t* __restrict__ dst, intptr_t ds, const int64_t* __restrict__ doff)
{
    __shared__ int16_t tile[kTrWaves][32 * 32];     // per-wavefront 32x32 staging tile, row-major
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, h = l >> 5;
    int16_t* T = tile[w];
    const int sh1 = FWD ? 4 + depth - 8 : 7, sh2 = FWD ? 11 : 12 - (depth - 8);
    const int io_row = l >> 1, io_col = 16 * (l & 1);  // 16-byte I/O: two lanes per row

    // constant fragments: stage-1 operand in natural k order, stage-2 operand in
    // the k order of the accumulator registers (row 16s + 8(j>>2) + 4h + (j&3))
    f16x8 t1[2], t2[2];
#pragma unroll
    for (int st = 0; st < 2; st++)
#pragma unroll
        for (int j = 0; j < 8; j++)
        {
            const int kn = 16 * st + 8 * h + j, kp = 16 * st + 8 * (j >> 2) + 4 * h + (j & 3);
            t1[st][j] = (_Float16)(FWD ? c_t32.m[r][kn] : c_t32.m[kn][r]);
            t2[st][j] = (_Float16)(FWD ? c_t32.m[r][kp] : c_t32.m[kp][r]);
        }

    // software pipeline: the next transform's 2 KiB are loaded (into registers) before this one's
    // MFMA chain and stores, so every wave keeps a transform's worth of loads in flight
    const int64_t step = (int64_t)gridDim.x * kTrWaves;
    int64_t job = (int64_t)blockIdx.x * kTrWaves + w;
    uint4 nx[2];                                     // forward: row r halves; inverse: the lane's 16-byte I/O chunks
    auto fetch = [&](int64_t jb) {
        const int16_t* s = src + soff[jb];
        if constexpr (FWD)
        {
            nx[0] = ldu<uint4>(s + r * ss + 8 * h);
            nx[1] = ldu<uint4>(s + r * ss + 16 + 8 * h);
        }
        else
        {
            nx[0] = ldu<uint4>(s + io_row * ss + io_col);
            nx[1] = ldu<uint4>(s + io_row * ss + io_col + 8);
        }
    };
    if (job < n) fetch(job);
    for (; job < n; job += step)
    {
        int16_t* d = dst + doff[job];
        const uint4 cx[2] = { nx[0], nx[1] };
        if (job + step < n) fetch(job + step);
        // ---- stage 1: forward U = Src * T^T (A = source rows, 16-byte row loads);
        //      inverse M1 = C^T * T (A = coefficient columns, staged through the tile)
        uint32_t x[2][4];                            // int16 pairs in k order
        if constexpr (FWD)
        {
#pragma unroll
            for (int st = 0; st < 2; st++)
            {
                x[st][0] = cx[st].x; x[st][1] = cx[st].y; x[st][2] = cx[st].z; x[st][3] = cx[st].w;
            }
        }
        else
        {
            stu<uint4>(&T[io_row * 32 + io_col], cx[0]);
            stu<uint4>(&T[io_row * 32 + io_col + 8], cx[1]);
            wave_sync();
#pragma unroll
            for (int st = 0; st < 2; st++)
#pragma unroll
                for (int q = 0; q < 4; q++)
                    x[st][q] = pack16(T[(16 * st + 8 * h + 2 * q) * 32 + r], T[(16 * st + 8 * h + 2 * q + 1) * 32 + r]);
        }
        f32x16 lo1 = {}, hi1 = {};
#pragma unroll
        for (int st = 0; st < 2; st++)
        {
            f16x8 xl, xh;
            split10<4>(x[st], xl, xh);
            lo1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, t1[st], lo1, 0, 0, 0);
            hi1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, t1[st], hi1, 0, 0, 0);
        }
        int v[16];
#pragma unroll
        for (int i = 0; i < 16; i++)
        {
            const int a = (int)hi1[i] * 1024 + (int)lo1[i];
            v[i] = FWD ? fwd_round(a, sh1) : inv_round(a, sh1);
        }
        // ---- stage 2 from registers: forward Dst = T * U' (U' as B); inverse Res = M1'^T * T (M1' as A)
        f32x16 lo2 = {}, hi2 = {};
#pragma unroll
        for (int st = 0; st < 2; st++)
        {
            uint32_t y[4];
#pragma unroll
            for (int q = 0; q < 4; q++) y[q] = pack16(v[8 * st + 2 * q], v[8 * st + 2 * q + 1]);
            f16x8 xl, xh;
            split10<4>(y, xl, xh);
            if constexpr (FWD)
            {
                lo2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(t2[st], xl, lo2, 0, 0, 0);
                hi2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(t2[st], xh, hi2, 0, 0, 0);
            }
            else
            {
                lo2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, t2[st], lo2, 0, 0, 0);
                hi2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, t2[st], hi2, 0, 0, 0);
            }
        }
        // accumulator (row, col) = ((i&3) + 8(i>>2) + 4h, r) -> tile -> 16-byte row stores
#pragma unroll
        for (int i = 0; i < 16; i++)
        {
            const int a = (int)hi2[i] * 1024 + (int)lo2[i];
            T[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = (int16_t)(FWD ? fwd_round(a, sh2) : inv_round(a, sh2));
        }
        wave_sync();
#pragma unroll
        for (int c = 0; c < 16; c += 8) stu<uint4>(d + io_row * ds + io_col + c, ldu<uint4>(&T[io_row * 32 + io_col + c]));
        wave_sync();                                 // the tile is read out before the next transform rewrites it
    }
}

// ---------------------------------------------------------------------------------------------
// k_tr32_i8: the same two 32x32x32 products on the INTEGER matrix cores
// (v_mfma_i32_32x32x32_i8: int8 operands, exact int32 accumulation, twice the K of the f16 form
// per instruction).  Every int16 operand x is split into its bytes, x = 256 * hi + lo with
// hi = x >> 8 in [-128, 127] (the high byte as stored) and lo = x & 255; lo enters the MFMA as the
// signed byte lo - 128 (lo ^ 0x80), so
//     sum_k c_k x_k = 256 * sum_k c_k hi_k + sum_k c_k (lo_k - 128) + 128 * sum_k c_k,
// with the transform coefficients c (|c| <= 90) as the constant int8 operand.  The last term is a
// constant of the output element: 128 x the row sum of the constant operand (forward: every row of
// the DCT matrix but row 0 sums to 0, row 0 to 64 * 32) or its column sum (inverse), folded into
// the rounding offset.  Recombination is one v_lshl_add per element, no float conversion; all
// sums are exact in int32 (|256 * sum c hi| <= 256 * 32 * 90 * 128 < 2^31).
// The k order inside a product only has to agree between its two operands: stage 1 takes the
// 16 loaded values of a lane half as k = 16h + j, stage 2 takes the stage-1 accumulator registers
// as they lie (register j of lane half h = row (j&3) + 8(j>>2) + 4h), with the constant operand
// permuted to match — no data moves between the stages.
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

// bytes of 8 packed int16 pairs (16 values in order) -> the lo fragment (biased) and hi fragment
__device__ __forceinline__ void split_bytes(const uint32_t (&d)[8], i32x4& lo, i32x4& hi)
{
#pragma unroll
    for (int q = 0; q < 4; q++)
    {
        lo[q] = (int)(__builtin_amdgcn_perm(d[2 * q + 1], d[2 * q], 0x06040200u) ^ 0x80808080u);
        hi[q] = (int)__builtin_amdgcn_perm(d[2 * q + 1], d[2 * q], 0x07050301u);
    }
}

template <bool FWD>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_tr32_i8(int n, int depth,
    const int16_t* __restrict__ src, intptr_t ss, const int64_t* __restrict__ soff,
    int16_t* __restrict__ dst, intptr_t ds, const int64_t* __restrict__ doff)
{
    __shared__ int16_t tile[kTrWaves][32 * 32];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, h = l >> 5;
    int16_t* T = tile[w];
    const int sh1 = FWD ? 4 + depth - 8 : 7, sh2 = FWD ? 11 : 12 - (depth - 8);
    const int io_row = l >> 1, io_col = 16 * (l & 1);

    // constant int8 fragments: stage 1 in the natural k order of the lane half (k = 16h + j),
    // stage 2 in the accumulator's row order (k = (j&3) + 8(j>>2) + 4h)
    i32x4 c1, c2;
    int csum = 0;                                    // 128 x the column sum of T at column r (inverse)
#pragma unroll
    for (int q = 0; q < 4; q++)
    {
        uint32_t a = 0, b = 0;
#pragma unroll
        for (int e = 0; e < 4; e++)
        {
            const int j = 4 * q + e, kn = 16 * h + j, kp = (j & 3) + 8 * (j >> 2) + 4 * h;
            a |= (uint32_t)(uint8_t)(int8_t)(FWD ? c_t32.m[r][kn] : c_t32.m[kn][r]) << (8 * e);
            b |= (uint32_t)(uint8_t)(int8_t)(FWD ? c_t32.m[r][kp] : c_t32.m[kp][r]) << (8 * e);
        }
        c1[q] = (int)a;
        c2[q] = (int)b;
    }
#pragma unroll
    for (int k = 0; k < 32; k++) csum += c_t32.m[k][r];
    csum *= 128;
    // bias + rounding offsets per stage: forward stage 1 (column r of U = X T^T: row r of T, zero
    // sum unless r == 0), forward stage 2 (row 0 of T, register 0 of lane half 0 only), inverse
    // (column sums of T at the lane's column, both stages)
    const int k1 = (FWD ? (r == 0 ? 128 * 64 * 32 : 0) : csum) + (1 << (sh1 - 1));
    const int k2 = FWD ? (1 << (sh2 - 1)) : csum + (1 << (sh2 - 1));
    const int k20 = FWD && h == 0 ? 128 * 64 * 32 : 0;

    const int64_t step = (int64_t)gridDim.x * kTrWaves;
    int64_t job = (int64_t)blockIdx.x * kTrWaves + w;
    uint4 nx[2];
    auto fetch = [&](int64_t jb) {
        const int16_t* s = src + soff[jb];
        if constexpr (FWD)
        {
            nx[0] = ldu<uint4>(s + r * ss + 16 * h);
            nx[1] = ldu<uint4>(s + r * ss + 16 * h + 8);
        }
        else
        {
            nx[0] = ldu<uint4>(s + io_row * ss + io_col);
            nx[1] = ldu<uint4>(s + io_row * ss + io_col + 8);
        }
    };
    if (job < n) fetch(job);
    for (; job < n; job += step)
    {
        int16_t* d = dst + doff[job];
        const uint4 cx[2] = { nx[0], nx[1] };
        if (job + step < n) fetch(job + step);
        // ---- stage 1: forward U = X T^T (A = source row r, k = 16h + j);
        //      inverse M1 = C^T T (A = coefficient column r, staged through the tile)
        uint32_t x[8];
        if constexpr (FWD)
        {
            x[0] = cx[0].x; x[1] = cx[0].y; x[2] = cx[0].z; x[3] = cx[0].w;
            x[4] = cx[1].x; x[5] = cx[1].y; x[6] = cx[1].z; x[7] = cx[1].w;
        }
        else
        {
            stu<uint4>(&T[io_row * 32 + io_col], cx[0]);
            stu<uint4>(&T[io_row * 32 + io_col + 8], cx[1]);
            wave_sync();
#pragma unroll
            for (int q = 0; q < 8; q++)
                x[q] = pack16(T[(16 * h + 2 * q) * 32 + r], T[(16 * h + 2 * q + 1) * 32 + r]);
        }
        i32x4 xl, xh;
        split_bytes(x, xl, xh);
        i32x16 lo1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(xl, c1, (i32x16){}, 0, 0, 0);
        i32x16 hi1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(xh, c1, (i32x16){}, 0, 0, 0);
        int v[16];
#pragma unroll
        for (int i = 0; i < 16; i++)
        {
            const int a = (int)(((uint32_t)hi1[i] << 8) + (uint32_t)lo1[i]) + k1;
            v[i] = FWD ? (a >> sh1) : clip16(a >> sh1);   // forward: the int16 wrap is the byte split below
        }
        // ---- stage 2 from registers: forward Dst = T U' (U' as B); inverse Res = M1'^T T (M1' as A)
        uint32_t y[8];
#pragma unroll
        for (int q = 0; q < 8; q++) y[q] = pack16(v[2 * q], v[2 * q + 1]);
        split_bytes(y, xl, xh);
        i32x16 lo2, hi2;
        if constexpr (FWD)
        {
            lo2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(c2, xl, (i32x16){}, 0, 0, 0);
            hi2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(c2, xh, (i32x16){}, 0, 0, 0);
        }
        else
        {
            lo2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(xl, c2, (i32x16){}, 0, 0, 0);
            hi2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(xh, c2, (i32x16){}, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 16; i++)
        {
            const int a = (int)(((uint32_t)hi2[i] << 8) + (uint32_t)lo2[i]) + k2 + (i == 0 ? k20 : 0);
            T[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = (int16_t)(FWD ? (a >> sh2) : clip16(a >> sh2));
        }
        wave_sync();
#pragma unroll
        for (int c = 0; c < 16; c += 8) stu<uint4>(d + io_row * ds + io_col + c, ldu<uint4>(&T[io_row * 32 + io_col + c]));
        wave_sync();
    }
}

// the integer-MFMA 16x16 (round 5) and 32x32 transforms, default (X265AMD_TR_I8=0 selects the f16 split
// forms; measured, profiles/r04/tr32_i8_ab.txt: dct / idct 32x32 0.49 / 0.51 -> 0.61 / 0.60 of the HBM peak)
static bool tr_i8()
{
    static int v = -1;
    if (v < 0)
    {
        const char* e = getenv("X265AMD_TR_I8");
        v = e ? atoi(e) != 0 : 1;
    }
    return v != 0;
}

template <bool FWD>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_tr16_mfma(int n, int depth,
    const int16_t* __restrict__ src, intptr_t ss, const int64_t* __restrict__ soff,
    int16_t* __restrict__ dst, intptr_t ds, const int64_t* __restrict__ doff)
{
    // 16x16x16 f16: A lane l holds A[l&15][4q + j], B holds B[4q + j][l&15],
    // the accumulator holds rows 4q + i of column l&15 (q = l >> 4) — the
    // accumulator order IS the operand k order, and T[l&15][4q+j] (forward) /
    // T[4q+j][l&15] (inverse) is the constant operand of both stages.
    // A wave takes JB transforms per iteration (all loads first, then the
    // MFMA chains interleaved), so one iteration keeps 2 KiB in flight.
    constexpr int JB = 4;
    __shared__ int16_t tile[kTrWaves][JB][16 * 16];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 15, q = l >> 4;
    const int sh1 = FWD ? 3 + depth - 8 : 7, sh2 = FWD ? 10 : 12 - (depth - 8);
    const int io_row = l >> 2, io_col = 4 * (l & 3);  // 8-byte I/O: four lanes per row

    f16x4 t;
#pragma unroll
    for (int j = 0; j < 4; j++) t[j] = (_Float16)(FWD ? c_t32.m[2 * r][4 * q + j] : c_t32.m[2 * (4 * q + j)][r]);

    // software pipeline: the next iteration's JB transforms are loaded (into registers) before this
    // iteration's MFMA chains and stores
    const int64_t step = (int64_t)gridDim.x * kTrWaves * JB;
    int64_t job0 = ((int64_t)blockIdx.x * kTrWaves + w) * JB;
    uint2 nx[JB];
    auto fetch = [&](int64_t j0) {
#pragma unroll
        for (int b = 0; b < JB; b++)
        {
            const int64_t job = j0 + b < n ? j0 + b : j0;   // a tail repeats the first (its result is not stored)
            const int16_t* s = src + soff[job];
            nx[b] = FWD ? ldu<uint2>(s + r * ss + 4 * q) : ldu<uint2>(s + io_row * ss + io_col);
        }
    };
    if (job0 < n) fetch(job0);
    for (; job0 < n; job0 += step)
    {
        int16_t* d[JB];
        int x[JB][4];
        uint2 cx[JB];
#pragma unroll
        for (int b = 0; b < JB; b++)
        {
            cx[b] = nx[b];
            d[b] = dst + doff[job0 + b < n ? job0 + b : job0];
        }
        if (job0 + step < n) fetch(job0 + step);
        if constexpr (!FWD)
        {
#pragma unroll
            for (int b = 0; b < JB; b++) stu<uint2>(&tile[w][b][io_row * 16 + io_col], cx[b]);
            wave_sync();
        }
        f32x4 lo[JB], hi[JB];
#pragma unroll
        for (int b = 0; b < JB; b++)
        {
            uint32_t u[2];
            if constexpr (FWD)
            {
                u[0] = cx[b].x;
                u[1] = cx[b].y;
            }
            else
            {
#pragma unroll
                for (int p = 0; p < 2; p++)
                    u[p] = pack16(tile[w][b][(4 * q + 2 * p) * 16 + r], tile[w][b][(4 * q + 2 * p + 1) * 16 + r]);
            }
            f16x4 xl, xh;
            split10<2>(u, xl, xh);
            lo[b] = __builtin_amdgcn_mfma_f32_16x16x16f16(xl, t, f32x4{}, 0, 0, 0);
            hi[b] = __builtin_amdgcn_mfma_f32_16x16x16f16(xh, t, f32x4{}, 0, 0, 0);
        }
#pragma unroll
        for (int b = 0; b < JB; b++)
        {
#pragma unroll
            for (int i = 0; i < 4; i++)
            {
                const int a = (int)hi[b][i] * 1024 + (int)lo[b][i];
                x[b][i] = FWD ? fwd_round(a, sh1) : inv_round(a, sh1);
            }
            const uint32_t u[2] = { pack16(x[b][0], x[b][1]), pack16(x[b][2], x[b][3]) };
            f16x4 xl, xh;
            split10<2>(u, xl, xh);
            if constexpr (FWD)
            {
                lo[b] = __builtin_amdgcn_mfma_f32_16x16x16f16(t, xl, f32x4{}, 0, 0, 0);
                hi[b] = __builtin_amdgcn_mfma_f32_16x16x16f16(t, xh, f32x4{}, 0, 0, 0);
            }
            else
            {
                lo[b] = __builtin_amdgcn_mfma_f32_16x16x16f16(xl, t, f32x4{}, 0, 0, 0);
                hi[b] = __builtin_amdgcn_mfma_f32_16x16x16f16(xh, t, f32x4{}, 0, 0, 0);
            }
        }
#pragma unroll
        for (int b = 0; b < JB; b++)
        {
            int16_t* T = tile[w][b];
#pragma unroll
            for (int i = 0; i < 4; i++)
            {
                const int a = (int)hi[b][i] * 1024 + (int)lo[b][i];
                T[(4 * q + i) * 16 + r] = (int16_t)(FWD ? fwd_round(a, sh2) : inv_round(a, sh2));
            }
            wave_sync();
            if (job0 + b < n) stu<uint2>(d[b] + io_row * ds + io_col, ldu<uint2>(&T[io_row * 16 + io_col]));
        }
        wave_sync();                                 // tiles read out before the next iteration rewrites them
    }
}


// ---------------------------------------------------------------------------------------------
// k_tr16_i8 (round 5): the 16x16 products on the integer matrix cores, v_mfma_i32_16x16x32_i8 (A lane l:
// row l & 15, k slots 8q .. 8q + 7 with q = l >> 4; B lane l: column l & 15, the same slots; D lane l:
// column l & 15, rows 4q .. 4q + 3).  A 16-point transform has K = 16, so each lane fills slots
// 8q .. 8q + 3 with k = 4q .. 4q + 3 and leaves 8q + 4 .. 8q + 7 zero (the order only has to agree between
// the two operands): then a lane's four data values are exactly the four accumulator rows it holds from the
// previous stage — forward stage 2 takes the stage-1 tile as it lies, with no data movement — and its four
// constant values are one dword (the other dword of the 64-bit operand is zero).  Every int16 operand is
// split into bytes as in k_tr32_i8 (x = 256 hi + lo, lo entering as lo - 128, the bias 128 x the constant
// sums folded into the rounding offsets), recombined with one v_lshl_add per element.  JB transforms per
// wave iteration, software-pipelined loads, LDS tiles for the column sides, as k_tr16_mfma.
template <bool FWD>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_tr16_i8(int n, int depth,
    const int16_t* __restrict__ src, intptr_t ss, const int64_t* __restrict__ soff,
    int16_t* __restrict__ dst, intptr_t ds, const int64_t* __restrict__ doff)
{
    constexpr int JB = 4;
    __shared__ int16_t tile[kTrWaves][JB][16 * 16];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 15, q = l >> 4;
    const int sh1 = FWD ? 3 + depth - 8 : 7, sh2 = FWD ? 10 : 12 - (depth - 8);
    const int io_row = l >> 2, io_col = 4 * (l & 3);  // 8-byte I/O: four lanes per row

    // the constant operand (both stages use the same fragment, as in k_tr16_mfma): forward T[r][4q + j],
    // inverse T[4q + j][r] (T = the 16-point matrix, rows of the 32-point one at even indices)
    uint32_t tc = 0;
#pragma unroll
    for (int j = 0; j < 4; j++)
        tc |= (uint32_t)(uint8_t)(int8_t)(FWD ? c_t32.m[2 * r][4 * q + j] : c_t32.m[2 * (4 * q + j)][r]) << (8 * j);
    const long cop = (long)(uint64_t)tc;
    // bias of the biased lo plane: 128 x the sum of the constant over k — forward: the row sums of T
    // (64 x 16 for row 0, 0 for the others), at output column r (stage 1) / output row 4q + i (stage 2);
    // inverse: the column sums of T at output column r, both stages
    int csum = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) csum += c_t32.m[2 * k][r];
    const int k1 = (FWD ? (r == 0 ? 128 * 64 * 16 : 0) : 128 * csum) + (1 << (sh1 - 1));
    const int k2 = FWD ? (1 << (sh2 - 1)) : 128 * csum + (1 << (sh2 - 1));
    const int k20 = FWD && q == 0 ? 128 * 64 * 16 : 0;   // forward stage 2: row 0 (register 0 of quarter 0)

    const int64_t step = (int64_t)gridDim.x * kTrWaves * JB;
    int64_t job0 = ((int64_t)blockIdx.x * kTrWaves + w) * JB;
    uint2 nx[JB];
    auto fetch = [&](int64_t j0) {
#pragma unroll
        for (int b = 0; b < JB; b++)
        {
            const int64_t job = j0 + b < n ? j0 + b : j0;   // a tail repeats the first (its result is not stored)
            const int16_t* sp = src + soff[job];
            nx[b] = FWD ? ldu<uint2>(sp + r * ss + 4 * q) : ldu<uint2>(sp + io_row * ss + io_col);
        }
    };
    // the two byte planes of 4 int16 values (2 packed pairs) as 64-bit MFMA operands (upper dword zero)
    auto planes = [](uint32_t u0, uint32_t u1, long& lo, long& hi) {
        lo = (long)(uint64_t)(__builtin_amdgcn_perm(u1, u0, 0x06040200u) ^ 0x80808080u);
        hi = (long)(uint64_t)__builtin_amdgcn_perm(u1, u0, 0x07050301u);
    };
    if (job0 < n) fetch(job0);
    for (; job0 < n; job0 += step)
    {
        int16_t* d[JB];
        uint2 cx[JB];
#pragma unroll
        for (int b = 0; b < JB; b++)
        {
            cx[b] = nx[b];
            d[b] = dst + doff[job0 + b < n ? job0 + b : job0];
        }
        if (job0 + step < n) fetch(job0 + step);
        if constexpr (!FWD)
        {
#pragma unroll
            for (int b = 0; b < JB; b++) stu<uint2>(&tile[w][b][io_row * 16 + io_col], cx[b]);
            wave_sync();
        }
        i32x4 lo[JB], hi[JB];
#pragma unroll
        for (int b = 0; b < JB; b++)
        {
            uint32_t u0, u1;
            if constexpr (FWD)
            {
                u0 = cx[b].x;
                u1 = cx[b].y;
            }
            else
            {
                u0 = pack16(tile[w][b][(4 * q) * 16 + r], tile[w][b][(4 * q + 1) * 16 + r]);
                u1 = pack16(tile[w][b][(4 * q + 2) * 16 + r], tile[w][b][(4 * q + 3) * 16 + r]);
            }
            long xl, xh;
            planes(u0, u1, xl, xh);
            // forward stage 1: U = X T^T (A = the source row, B = T^T); inverse: C^T T (A = the coefficient
            // column, B = T)
            lo[b] = __builtin_amdgcn_mfma_i32_16x16x32_i8(xl, cop, i32x4{}, 0, 0, 0);
            hi[b] = __builtin_amdgcn_mfma_i32_16x16x32_i8(xh, cop, i32x4{}, 0, 0, 0);
        }
#pragma unroll
        for (int b = 0; b < JB; b++)
        {
            int x[4];
#pragma unroll
            for (int i = 0; i < 4; i++)
            {
                const int a = (int)(((uint32_t)hi[b][i] << 8) + (uint32_t)lo[b][i]) + k1;
                x[i] = FWD ? (a >> sh1) : clip16(a >> sh1);   // forward: the int16 wrap is the byte split
            }
            long xl, xh;
            planes(pack16(x[0], x[1]), pack16(x[2], x[3]), xl, xh);
            if constexpr (FWD)
            {
                // Y = T U: A = T (row r, k = 4q + j), B = the stage-1 tile as it lies
                lo[b] = __builtin_amdgcn_mfma_i32_16x16x32_i8(cop, xl, i32x4{}, 0, 0, 0);
                hi[b] = __builtin_amdgcn_mfma_i32_16x16x32_i8(cop, xh, i32x4{}, 0, 0, 0);
            }
            else
            {
                lo[b] = __builtin_amdgcn_mfma_i32_16x16x32_i8(xl, cop, i32x4{}, 0, 0, 0);
                hi[b] = __builtin_amdgcn_mfma_i32_16x16x32_i8(xh, cop, i32x4{}, 0, 0, 0);
            }
        }
#pragma unroll
        for (int b = 0; b < JB; b++)
        {
            int16_t* T = tile[w][b];
#pragma unroll
            for (int i = 0; i < 4; i++)
            {
                const int a = (int)(((uint32_t)hi[b][i] << 8) + (uint32_t)lo[b][i]) + k2 + (i == 0 ? k20 : 0);
                T[(4 * q + i) * 16 + r] = (int16_t)(FWD ? (a >> sh2) : clip16(a >> sh2));
            }
            wave_sync();
            if (job0 + b < n) stu<uint2>(d[b] + io_row * ds + io_col, ldu<uint2>(&T[io_row * 16 + io_col]));
        }
        wave_sync();                                 // tiles read out before the next iteration rewrites them
    }
}

// --------------------------------------------------------------- quant family
// A job's chunks of CW coefficients (CW = 4 or 8) go to a group of
// G = min(64, num / CW) lanes; each lane carries CPJ chunks of each of JPG jobs.
// Step k of a block covers jobs block0 + k NG + g (NG groups per block), chunk
// c = lane + i G, so every wave-instruction reads / writes contiguous bytes of
// consecutive jobs, and all loads of a lane are issued before the first chunk is
// quantized.  (CW, JPG) per size class were set by measurement
// (tools/coef_tune.sh; X265AMD_COEF_CW / X265AMD_COEF_JPG override them).
template <int CPJ, int JPG>
struct CoefMap
{
    int G, NG, g, lane, nch;
    int64_t job[JPG];
    bool live[JPG];
    __device__ __forceinline__ CoefMap(int n, int num, int lg, int cw)
    {
        G = 1 << lg;
        NG = X265AMD_BLOCK >> lg;
        g = threadIdx.x >> lg;
        lane = threadIdx.x & (G - 1);
        nch = num / cw;
        const int64_t b0 = (int64_t)xcd_block() * NG * JPG;
#pragma unroll
        for (int k = 0; k < JPG; k++)
        {
            const int64_t j = b0 + (int64_t)k * NG + g;
            live[k] = j < n;
            job[k] = live[k] ? j : 0;
        }
    }
    // chunk index of slot i of job slot k (-1: none)
    __device__ __forceinline__ int chunk(int k, int i, int c0) const
    {
        const int c = c0 + i * G;
        return live[k] && c < nch ? c : -1;
    }
};

// CW int16 / int32 values as packed words
template <int CW>
struct Chunk16 { uint32_t w[CW / 2]; };
template <int CW>
struct Chunk32 { int w[CW]; };

template <int CW>
__device__ __forceinline__ Chunk16<CW> ld16(const int16_t* p)
{
    Chunk16<CW> c;
    if constexpr (CW == 8) { const uint4 v = ldu<uint4>(p); c.w[0] = v.x; c.w[1] = v.y; c.w[2] = v.z; c.w[3] = v.w; }
    else { const uint2 v = ldu<uint2>(p); c.w[0] = v.x; c.w[1] = v.y; }
    return c;
}
template <int CW>
__device__ __forceinline__ Chunk32<CW> ld32(const int32_t* p)
{
    Chunk32<CW> c;
#pragma unroll
    for (int q = 0; q < CW / 4; q++)
    {
        const int4 v = ldu<int4>(p + 4 * q);
        c.w[4 * q] = v.x; c.w[4 * q + 1] = v.y; c.w[4 * q + 2] = v.z; c.w[4 * q + 3] = v.w;
    }
    return c;
}
template <int CW>
__device__ __forceinline__ void st16(int16_t* p, const int (&o)[CW])
{
    uint32_t w[CW / 2];
#pragma unroll
    for (int e = 0; e < CW / 2; e++) w[e] = (uint32_t)(o[2 * e] & 0xffff) | ((uint32_t)o[2 * e + 1] << 16);
    if constexpr (CW == 8) stu<uint4>(p, make_uint4(w[0], w[1], w[2], w[3]));
    else stu<uint2>(p, make_uint2(w[0], w[1]));
}
template <int CW>
__device__ __forceinline__ int c16(const Chunk16<CW>& c, int e)
{
    return (int16_t)(e & 1 ? c.w[e >> 1] >> 16 : c.w[e >> 1] & 0xffff);
}

template <bool NQUANT, int CW, int CPJ, int JPG>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_quant(int n, int num, int lg,
    const int16_t* __restrict__ coef, const int64_t* __restrict__ coff,
    const int32_t* __restrict__ qtab, const int64_t* __restrict__ qoff,
    int32_t* __restrict__ delta, const int64_t* __restrict__ doff,
    int16_t* __restrict__ qout, const int64_t* __restrict__ ooff,
    const int32_t* __restrict__ qbits, const int32_t* __restrict__ add, uint32_t* __restrict__ numsig)
{
    const CoefMap<CPJ, JPG> m(n, num, lg, CW);
    const int16_t* pc[JPG];
    const int32_t* pq[JPG];
    int16_t* po[JPG];
    int32_t* pdl[JPG];
    int qb[JPG], ad[JPG];
    uint32_t sig[JPG];
#pragma unroll
    for (int k = 0; k < JPG; k++)
    {
        pc[k] = coef + coff[m.job[k]];
        pq[k] = qtab + qoff[m.job[k]];
        po[k] = qout + ooff[m.job[k]];
        pdl[k] = NQUANT ? nullptr : delta + doff[m.job[k]];
        qb[k] = qbits[m.job[k]];
        ad[k] = add[m.job[k]];
        sig[k] = 0;
    }
    for (int c0 = m.lane; c0 < m.nch; c0 += CPJ * m.G)
    {
        Chunk16<CW> cv[JPG][CPJ];
        Chunk32<CW> qv[JPG][CPJ];
#pragma unroll
        for (int k = 0; k < JPG; k++)
#pragma unroll
            for (int i = 0; i < CPJ; i++)
            {
                const int c = m.chunk(k, i, c0);
                if (c < 0) continue;
                cv[k][i] = ld16<CW>(pc[k] + CW * c);
                qv[k][i] = ld32<CW>(pq[k] + CW * c);
            }
#pragma unroll
        for (int k = 0; k < JPG; k++)
#pragma unroll
            for (int i = 0; i < CPJ; i++)
            {
                const int c = m.chunk(k, i, c0);
                if (c < 0) continue;
                int o[CW], dl[CW];
#pragma unroll
                for (int e = 0; e < CW; e++)
                {
                    const int lv = c16<CW>(cv[k][i], e);
                    // int32 products/sums wrap exactly as the reference's int arithmetic (dct.cpp:676-678)
                    const uint32_t tmp = (uint32_t)abs(lv) * (uint32_t)qv[k][i].w[e];
                    int level = (int)(tmp + (uint32_t)ad[k]) >> qb[k];
                    dl[e] = (int)(tmp - ((uint32_t)level << qb[k])) >> (qb[k] - 8);
                    sig[k] += level != 0;
                    if (lv < 0) level = -level;
                    level = clip16(level);
                    o[e] = NQUANT ? abs(level) : level;
                }
                st16<CW>(po[k] + CW * c, o);
                if (!NQUANT)
                {
#pragma unroll
                    for (int q = 0; q < CW / 4; q++)
                        stu<int4>(pdl[k] + CW * c + 4 * q, make_int4(dl[4 * q], dl[4 * q + 1], dl[4 * q + 2], dl[4 * q + 3]));
                }
            }
    }
#pragma unroll
    for (int k = 0; k < JPG; k++)
    {
        uint32_t v = sig[k];
        for (int mm = m.G >> 1; mm > 0; mm >>= 1) v += __shfl_xor(v, mm, 64);
        if (m.live[k] && m.lane == 0) numsig[m.job[k]] = v;
    }
}

template <bool SCALING, int CW, int CPJ, int JPG>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_dequant(int n, int num, int lg,
    const int16_t* __restrict__ q, const int64_t* __restrict__ qoff,
    const int32_t* __restrict__ dq, const int64_t* __restrict__ dqoff,
    int16_t* __restrict__ out, const int64_t* __restrict__ ooff,
    const int32_t* __restrict__ p0, const int32_t* __restrict__ p1)
{
    // the chunk / job mapping of k_quant
    const CoefMap<CPJ, JPG> m(n, num, lg, CW);
    const int16_t* pq[JPG];
    const int32_t* pd[JPG];
    int16_t* po[JPG];
    int a0[JPG], a1[JPG];
#pragma unroll
    for (int k = 0; k < JPG; k++)
    {
        pq[k] = q + qoff[m.job[k]];
        pd[k] = SCALING ? dq + dqoff[m.job[k]] : nullptr;
        po[k] = out + ooff[m.job[k]];
        a0[k] = p0[m.job[k]];
        a1[k] = p1[m.job[k]];
    }
    for (int c0 = m.lane; c0 < m.nch; c0 += CPJ * m.G)
    {
        Chunk16<CW> v[JPG][CPJ];
        Chunk32<CW> d[JPG][CPJ];
#pragma unroll
        for (int k = 0; k < JPG; k++)
#pragma unroll
            for (int i = 0; i < CPJ; i++)
            {
                const int c = m.chunk(k, i, c0);
                if (c < 0) continue;
                v[k][i] = ld16<CW>(pq[k] + CW * c);
                if (SCALING) d[k][i] = ld32<CW>(pd[k] + CW * c);
            }
#pragma unroll
        for (int k = 0; k < JPG; k++)
#pragma unroll
            for (int i = 0; i < CPJ; i++)
            {
                const int c = m.chunk(k, i, c0);
                if (c < 0) continue;
                int o[CW];
                if (!SCALING)
                {
                    const int scale = a0[k], shift = a1[k], ad = 1 << (shift - 1);
#pragma unroll
                    for (int e = 0; e < CW; e++) o[e] = clip16((c16<CW>(v[k][i], e) * scale + ad) >> shift);
                }
                else
                {
                    const int per = a0[k], shift = a1[k] + 4;
                    if (shift > per)
                    {
                        const int ad = 1 << (shift - per - 1);
#pragma unroll
                        for (int e = 0; e < CW; e++)
                            o[e] = clip16((c16<CW>(v[k][i], e) * d[k][i].w[e] + ad) >> (shift - per));
                    }
                    else
                    {
#pragma unroll
                        for (int e = 0; e < CW; e++)
                            o[e] = clip16(clip16(c16<CW>(v[k][i], e) * d[k][i].w[e]) << (per - shift));
                    }
                }
                st16<CW>(po[k] + CW * c, o);
            }
    }
}

// count_nonzero (res == nullptr) / copy_cnt: CW coefficients per lane per step
// (8 from 8x8 up: one 16-byte load / store, the shape the quant family measured best)
template <int N>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_count(int n, int16_t* __restrict__ coeff, const int64_t* __restrict__ coff,
    const int16_t* __restrict__ res, intptr_t rs, const int64_t* __restrict__ roff, uint32_t* __restrict__ cnt)
{
    constexpr int CW = N >= 8 ? 8 : 4;
    constexpr int G = N * N / CW < 64 ? N * N / CW : 64;
    const int64_t job = (int64_t)xcd_block() * (X265AMD_BLOCK / G) + threadIdx.x / G;
    const int lane = threadIdx.x & (G - 1);
    const bool live = job < n;
    uint32_t c = 0;
    if (live)
    {
        int16_t* pc = coeff + coff[job];
        const int16_t* pr = res ? res + roff[job] : nullptr;
        for (int i = lane * CW; i < N * N; i += G * CW)
        {
            uint32_t w[CW / 2];
            const int16_t* src = res ? pr + (i / N) * rs + i % N : pc + i;
            if constexpr (CW == 8)
            {
                const uint4 v = ldu<uint4>(src);
                w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
                if (res) stu<uint4>(pc + i, v);
            }
            else
            {
                const uint2 v = ldu<uint2>(src);
                w[0] = v.x; w[1] = v.y;
                if (res) stu<uint2>(pc + i, v);
            }
#pragma unroll
            for (int e = 0; e < CW / 2; e++) c += ((w[e] & 0xffffu) != 0) + ((w[e] >> 16) != 0);
        }
    }
    for (int m = G >> 1; m > 0; m >>= 1) c += __shfl_xor(c, m, 64);
    if (live && lane == 0) cnt[job] = c;
}

// denoiseDct (dct.cpp:744-755) over a batch: every job shrinks its num
// coefficients in place by offset[] and adds |coef| into the batch's shared
// res_sum[] (the reference's per-size m_residualSum accumulator).  A block takes
// kDenoiseJobs jobs; thread t owns coefficient positions t, t+256, ... (for
// num < 256, num-wide slices of several jobs at once), sums |coef| over its
// jobs in registers and adds each position into res_sum with one atomic at the
// end: uint32 addition commutes, so the total equals the serial order's mod 2^32.
constexpr int kDenoiseJobs = 64;

__global__ __launch_bounds__(X265AMD_BLOCK) void k_denoise(int n, int num, int16_t* __restrict__ coef,
    const int64_t* __restrict__ coef_off, uint32_t* __restrict__ res_sum, const uint16_t* __restrict__ offset)
{
    const int t = threadIdx.x;
    const int64_t j0 = (int64_t)xcd_block() * kDenoiseJobs;
    const int span = num < X265AMD_BLOCK ? num : X265AMD_BLOCK;     // positions per pass
    const int par = X265AMD_BLOCK / span;                            // jobs per pass (num < 256)
    const int pos0 = t % span, jsub = t / span;
    if (jsub >= par) return;
    uint32_t acc[4] = { 0, 0, 0, 0 };                                // num <= 1024 -> <= 4 positions
    int off[4];
#pragma unroll
    for (int k = 0; k < 4; k++) off[k] = pos0 + k * span < num ? offset[pos0 + k * span] : 0;
    for (int jj = jsub; jj < kDenoiseJobs; jj += par)
    {
        const int64_t job = j0 + jj;
        if (job >= n) break;
        int16_t* c = coef + coef_off[job];
#pragma unroll
        for (int k = 0; k < 4; k++)
        {
            const int i = pos0 + k * span;
            if (i >= num) break;
            int level = c[i];
            const int sign = level >> 31;
            level = (level + sign) ^ sign;
            acc[k] += (uint32_t)level;
            level -= off[k];
            c[i] = (int16_t)(level < 0 ? 0 : (level ^ sign) - sign);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++)
    {
        const int i = pos0 + k * span;
        if (i < num && acc[k]) atomicAdd(&res_sum[i], acc[k]);
    }
}

// chunk width / jobs per lane group of the coefficient kernels (measured,
// tools/coef_tune.sh); X265AMD_COEF_CW = 4 | 8 and
// X265AMD_COEF_JPG = 1 | 2 | 4 override them for tuning runs
struct CoefShape
{
    int cw, jpg, cpj, lg;
};
static CoefShape coef_shape(int num, bool quant)
{
    static int cw_env = -1, jpg_env = -1;
    if (cw_env < 0)
    {
        const char* e = getenv("X265AMD_COEF_CW");
        cw_env = e ? atoi(e) : 0;
        e = getenv("X265AMD_COEF_JPG");
        jpg_env = e ? atoi(e) : 0;
    }
    CoefShape c;
    // measured (profiles/r02/coef_tune.txt): 8-coefficient chunks of one job per lane, except
    // quant 32x32 which prefers four 4-coefficient chunks per lane (0.55 -> 0.61 of HBM peak)
    c.cw = cw_env == 4 || cw_env == 8 ? cw_env : (quant && num > 256 ? 4 : 8);
    if (num % (c.cw * 2)) c.cw = 4;         // num = 8 (dequant only) or odd multiples
    const int nch = num / c.cw;
    int g = nch > 64 ? 64 : nch, lg = 0;
    while ((1 << lg) < g) lg++;
    c.lg = lg;
    c.cpj = nch > 64 ? (nch + 63) / 64 : 1;
    if (c.cpj > 1) c.cpj = c.cw == 8 ? 2 : 4;
    c.jpg = c.cpj > 1 ? 1 : (jpg_env == 1 || jpg_env == 2 || jpg_env == 4 ? jpg_env : 1);
    return c;
}

// dispatch (CW, CPJ, JPG) to a kernel instantiation: CW 4 / 8, CPJ 1 with JPG 1 / 2 / 4, or
// the 32x32 shapes (CW 8, CPJ 2) / (CW 4, CPJ 4)
#define X265AMD_COEF_DISPATCH(c, LAUNCH)                                                              \
    do                                                                                                \
    {                                                                                                 \
        if (c.cw == 8)                                                                                \
        {                                                                                             \
            if (c.cpj > 1) LAUNCH(8, 2, 1); else if (c.jpg == 1) LAUNCH(8, 1, 1);                     \
            else if (c.jpg == 2) LAUNCH(8, 1, 2); else LAUNCH(8, 1, 4);                               \
        }                                                                                             \
        else                                                                                          \
        {                                                                                             \
            if (c.cpj > 1) LAUNCH(4, 4, 1); else if (c.jpg == 1) LAUNCH(4, 1, 1);                     \
            else if (c.jpg == 2) LAUNCH(4, 1, 2); else LAUNCH(4, 1, 4);                               \
        }                                                                                             \
    } while (0)

} // namespace x265amd

using namespace x265amd;

extern "C" int x265amd_transform(int kind, int depth, int size, int n,
                                 const int16_t* src, intptr_t src_stride, const int64_t* src_off,
                                 int16_t* dst, intptr_t dst_stride, const int64_t* dst_off, void* stream)
{
    if (n <= 0) return 0;
    if (depth != 8 && depth != 10 && depth != 12) return X265AMD_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const bool fwd = kind == X265AMD_DCT || kind == X265AMD_DST;
    if (kind == X265AMD_DST || kind == X265AMD_IDST || size == 4)
    {
        if (size != 4) return X265AMD_EINVAL;
        const dim3 grid((n + X265AMD_BLOCK * kTr4Jobs - 1) / (X265AMD_BLOCK * kTr4Jobs));
        switch (kind)
        {
        case X265AMD_DCT: hipLaunchKernelGGL(k_tr4<X265AMD_DCT>, grid, dim3(X265AMD_BLOCK), 0, st, n, depth, src, src_stride, src_off, dst, dst_stride, dst_off); break;
        case X265AMD_IDCT: hipLaunchKernelGGL(k_tr4<X265AMD_IDCT>, grid, dim3(X265AMD_BLOCK), 0, st, n, depth, src, src_stride, src_off, dst, dst_stride, dst_off); break;
        case X265AMD_DST: hipLaunchKernelGGL(k_tr4<X265AMD_DST>, grid, dim3(X265AMD_BLOCK), 0, st, n, depth, src, src_stride, src_off, dst, dst_stride, dst_off); break;
        case X265AMD_IDST: hipLaunchKernelGGL(k_tr4<X265AMD_IDST>, grid, dim3(X265AMD_BLOCK), 0, st, n, depth, src, src_stride, src_off, dst, dst_stride, dst_off); break;
        default: return X265AMD_EINVAL;
        }
        return (int)hipGetLastError();
    }
    if (kind != X265AMD_DCT && kind != X265AMD_IDCT) return X265AMD_EINVAL;
    if (size == 16 || size == 32)
    {
        // matrix cores: one wavefront per transform
        const dim3 grid(mfma_grid(size == 16 ? (n + 3) / 4 : n));
#define M(K) hipLaunchKernelGGL(K, grid, dim3(X265AMD_BLOCK), 0, st, n, depth, src, src_stride, src_off, dst, dst_stride, dst_off)
        if (size == 32 && tr_i8()) { if (fwd) M(k_tr32_i8<true>); else M(k_tr32_i8<false>); }
        else if (size == 32) { if (fwd) M(k_tr32_mfma<true>); else M(k_tr32_mfma<false>); }
        else if (tr_i8()) { if (fwd) M(k_tr16_i8<true>); else M(k_tr16_i8<false>); }
        else { if (fwd) M(k_tr16_mfma<true>); else M(k_tr16_mfma<false>); }
#undef M
        return (int)hipGetLastError();
    }
    const int jobs = X265AMD_BLOCK / size;
    const dim3 grid((n + jobs - 1) / jobs);
#define T(N)                                                                                                       \
    if (fwd) hipLaunchKernelGGL((k_trN<N, true>), grid, dim3(X265AMD_BLOCK), 0, st, n, depth, src, src_stride,    \
                                src_off, dst, dst_stride, dst_off);                                             \
    else hipLaunchKernelGGL((k_trN<N, false>), grid, dim3(X265AMD_BLOCK), 0, st, n, depth, src, src_stride,       \
                            src_off, dst, dst_stride, dst_off)
    switch (size)
    {
    case 8: T(8); break;
    case 16: T(16); break;
    case 32: T(32); break;
    default: return X265AMD_EINVAL;
    }
#undef T
    return (int)hipGetLastError();
}

extern "C" int x265amd_quant(int n, int num, const int16_t* coef, const int64_t* coef_off,
                             const int32_t* qtab, const int64_t* qtab_off,
                             int32_t* delta_u, const int64_t* delta_off,
                             int16_t* qcoef, const int64_t* qcoef_off,
                             const int32_t* qbits, const int32_t* add, uint32_t* num_sig, void* stream)
{
    if (n <= 0) return 0;
    if (num <= 0 || num % 16 || num > 1024) return X265AMD_EINVAL;
    const CoefShape c = coef_shape(num, true);
    const int per_block = (X265AMD_BLOCK >> c.lg) * c.jpg;
    const dim3 grid((n + per_block - 1) / per_block);
    hipStream_t st = (hipStream_t)stream;
    const int lg = c.lg;
#define Q(NQ, CW, C, J) hipLaunchKernelGGL((k_quant<NQ, CW, C, J>), grid, dim3(X265AMD_BLOCK), 0, st, n, num, lg, coef, \
                                           coef_off, qtab, qtab_off, delta_u, delta_off, qcoef, qcoef_off, qbits, add, num_sig)
#define QF(CW, C, J) Q(false, CW, C, J)
#define QT(CW, C, J) Q(true, CW, C, J)
    if (delta_u) X265AMD_COEF_DISPATCH(c, QF);
    else X265AMD_COEF_DISPATCH(c, QT);
#undef QT
#undef QF
#undef Q
    return (int)hipGetLastError();
}

extern "C" int x265amd_dequant_normal(int n, int num, const int16_t* q, const int64_t* q_off,
                                      int16_t* coef, const int64_t* coef_off,
                                      const int32_t* scale, const int32_t* shift, void* stream)
{
    if (n <= 0) return 0;
    if (num <= 0 || num % 8 || num > 1024) return X265AMD_EINVAL;
    const CoefShape c = coef_shape(num, false);
    const int per_block = (X265AMD_BLOCK >> c.lg) * c.jpg;
    const dim3 grid((n + per_block - 1) / per_block);
    const int lg = c.lg;
#define D(CW, C, J) hipLaunchKernelGGL((k_dequant<false, CW, C, J>), grid, dim3(X265AMD_BLOCK), 0, (hipStream_t)stream, n, \
                                       num, lg, q, q_off, (const int32_t*)nullptr, (const int64_t*)nullptr, coef, coef_off, scale, shift)
    X265AMD_COEF_DISPATCH(c, D);
#undef D
    return (int)hipGetLastError();
}

extern "C" int x265amd_dequant_scaling(int n, int num, const int16_t* q, const int64_t* q_off,
                                       const int32_t* dq, const int64_t* dq_off,
                                       int16_t* coef, const int64_t* coef_off,
                                       const int32_t* per, const int32_t* shift, void* stream)
{
    if (n <= 0) return 0;
    if (num <= 0 || num % 8 || num > 1024) return X265AMD_EINVAL;
    const CoefShape c = coef_shape(num, false);
    const int per_block = (X265AMD_BLOCK >> c.lg) * c.jpg;
    const dim3 grid((n + per_block - 1) / per_block);
    const int lg = c.lg;
#define D(CW, C, J) hipLaunchKernelGGL((k_dequant<true, CW, C, J>), grid, dim3(X265AMD_BLOCK), 0, (hipStream_t)stream, n, \
                                       num, lg, q, q_off, dq, dq_off, coef, coef_off, per, shift)
    X265AMD_COEF_DISPATCH(c, D);
#undef D
    return (int)hipGetLastError();
}

extern "C" int x265amd_denoise_dct(int n, int num, int16_t* coef, const int64_t* coef_off, uint32_t* res_sum,
                                   const uint16_t* offset, void* stream)
{
    if (n <= 0) return 0;
    if (num <= 0 || num % 16 || num > 1024 || (num < X265AMD_BLOCK && X265AMD_BLOCK % num)) return X265AMD_EINVAL;
    hipLaunchKernelGGL(k_denoise, dim3((n + kDenoiseJobs - 1) / kDenoiseJobs), dim3(X265AMD_BLOCK), 0,
                       (hipStream_t)stream, n, num, coef, coef_off, res_sum, offset);
    return (int)hipGetLastError();
}

extern "C" int x265amd_count_nonzero(int size, int n, int16_t* coeff, const int64_t* coeff_off,
                                     const int16_t* res, intptr_t res_stride, const int64_t* res_off,
                                     uint32_t* count, void* stream)
{
    if (n <= 0) return 0;
    hipStream_t st = (hipStream_t)stream;
#define C(N)                                                                                          \
    {                                                                                                 \
        constexpr int CW = N >= 8 ? 8 : 4, G = N * N / CW < 64 ? N * N / CW : 64;                     \
        const int per = X265AMD_BLOCK / G;                                                            \
        hipLaunchKernelGGL(k_count<N>, dim3((n + per - 1) / per), dim3(X265AMD_BLOCK), 0, st, n, coeff, \
                           coeff_off, res, res_stride, res_off, count);                               \
        return (int)hipGetLastError();                                                                \
    }
    switch (size)
    {
    case 4: C(4);
    case 8: C(8);
    case 16: C(16);
    case 32: C(32);
    }
#undef C
    return X265AMD_EINVAL;
}
