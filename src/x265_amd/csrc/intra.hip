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
// Work mapping: 4x4 / 8x8 one (TU, mode) job per lane (k_intra_lane); 16x16 / 32x32 four lanes per
// job (k_intra_quad).  Either way the reference array of intra_pred_ang_c is built once per job in the
// mode's frame (projected left samples, top-left, the 2N above samples) as pairs (R[j], R[j+1]) in LDS,
// so every angular pixel is one LDS read and one blend; the mode is decoded once per job from packed
// register constants (no table loads).
#include <stdlib.h>

#include "common.h"
#include "intra_lane.h"
#include "../../../include/x265_amd.h"

namespace x265amd {

typedef unsigned short pair16 __attribute__((ext_vector_type(2)));

// Small TUs (4x4, 8x8): one (TU, mode) job per LANE.  The whole 4N+1
// neighbour array is loaded with vector loads and flipped in registers
// (compile-time indices); planar, DC and the pure H/V modes never leave
// registers.  Angular modes need data-dependent offsets, so the lane writes its
// reference array to a private LDS column as PAIRS D[j] = (R[j], R[j+1]) of
// u16: every angular pixel is then one ds_read_b32 and one v_dot2_u32_u16
// against the row weights (32 - f, f):  ((32-f)·a + f·b + 16) >> 5.
constexpr int kIntraLaneJobs = 2;     // 4x4 jobs per lane

template <typename P, int N>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_intra_lane(int n, int maxv,
    P* __restrict__ dst, intptr_t ds, const int64_t* __restrict__ doff,
    const P* __restrict__ nb, const int64_t* __restrict__ nboff,
    const P* __restrict__ filt, const int64_t* __restrict__ filtoff,
    const uint8_t* __restrict__ mode, const uint8_t* __restrict__ bfilter, int allangs)
{
    // D[j + N][lane], j = -N .. 2N-1; after the prediction the same LDS holds the 8x8 blocks of the
    // block's 256 jobs for the coalesced store (N == 8)
    constexpr int NB = N * N * (int)sizeof(P);                 // output bytes per job
    constexpr int DW = 3 * N * X265AMD_BLOCK;                  // dwords of D
    constexpr int SW = N == 8 ? NB * X265AMD_BLOCK / 4 : 0;    // dwords of the output staging
    __shared__ uint32_t lds[DW > SW ? DW : SW];
    uint32_t (*D)[X265AMD_BLOCK] = (uint32_t (*)[X265AMD_BLOCK])lds;
    if constexpr (N == 4)
    {
        // 4x4: kIntraLaneJobs jobs per lane (jobs b + k * 256 + t), the descriptors and neighbour
        // loads of all of them issued before the first prediction; the lane's LDS column is reused
        // job after job (private to the lane: no barrier)
        const int64_t base = (int64_t)xcd_block() * X265AMD_BLOCK * kIntraLaneJobs + threadIdx.x;
        int mk[kIntraLaneJobs], bfk[kIntraLaneJobs], sk[kIntraLaneJobs][4 * N + 1];
        P* outk[kIntraLaneJobs];
        bool livek[kIntraLaneJobs];
#pragma unroll
        for (int k = 0; k < kIntraLaneJobs; k++)
        {
            const int64_t job = base + (int64_t)k * X265AMD_BLOCK;
            livek[k] = job < n;
            const int64_t jj = livek[k] ? job : 0;
            const P* src;
            if (allangs)
            {
                const int64_t tu = jj / 33;
                mk[k] = 2 + (int)(jj % 33);
                bfk[k] = bfilter[tu];
                src = (c_intra.filter_flags[mk[k]] & N) ? filt + filtoff[tu] : nb + nboff[tu];
                outk[k] = dst + doff[tu] + (int64_t)(mk[k] - 2) * N * N;
            }
            else
            {
                mk[k] = mode[jj];
                bfk[k] = bfilter[jj];
                src = nb + nboff[jj];
                outk[k] = dst + doff[jj];
            }
            intra_lane_load<P, N>(src, sk[k]);
        }
        const intptr_t os = allangs ? N : ds;
#pragma unroll
        for (int k = 0; k < kIntraLaneJobs; k++)
        {
            if (!livek[k]) continue;
            int v[N][N], o[N][N];
            const ModeInfo mi = intra_lane_predict<N>(sk[k], mk[k], bfk[k], maxv, D, v);
            const bool tr = mi.hor && !allangs;
#pragma unroll
            for (int r = 0; r < N; r++)
#pragma unroll
                for (int c = 0; c < N; c++) o[r][c] = tr ? v[c][r] : v[r][c];
            if (os == 4)
            {
                uint32_t w[NB / 4];
#pragma unroll
                for (int r = 0; r < 4; r++)
                {
                    if constexpr (sizeof(P) == 1)
                        w[r] = (uint32_t)o[r][0] | ((uint32_t)o[r][1] << 8) | ((uint32_t)o[r][2] << 16) | ((uint32_t)o[r][3] << 24);
                    else
                    {
                        w[2 * r] = (uint32_t)o[r][0] | ((uint32_t)o[r][1] << 16);
                        w[2 * r + 1] = (uint32_t)o[r][2] | ((uint32_t)o[r][3] << 16);
                    }
                }
#pragma unroll
                for (int q = 0; q < NB / 16; q++)
                    stu<uint4>((uint8_t*)outk[k] + 16 * q, make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]));
            }
            else
            {
#pragma unroll
                for (int r = 0; r < N; r++) store_row<P, N>(outk[k] + (int64_t)r * os, o[r]);
            }
        }
        return;
    }
    const int64_t job = (int64_t)xcd_block() * X265AMD_BLOCK + threadIdx.x;
    const bool live = job < n;
    const int64_t jj = live ? job : 0;

    int m, bf;
    const P* src;
    P* out;
    intptr_t os;
    if (allangs)
    {
        const int64_t tu = jj / 33;
        m = 2 + (int)(jj % 33);
        bf = bfilter[tu];
        src = (c_intra.filter_flags[m] & N) ? filt + filtoff[tu] : nb + nboff[tu];
        out = dst + doff[tu] + (int64_t)(m - 2) * N * N;
        os = N;
    }
    else
    {
        m = mode[jj];
        bf = bfilter[jj];
        src = nb + nboff[jj];
        out = dst + doff[jj];
        os = ds;
    }
    int s[4 * N + 1], v[N][N];
    intra_lane_load<P, N>(src, s);
    const ModeInfo mi = intra_lane_predict<N>(s, m, bf, maxv, D, v);

    // horizontal modes are transposed back, except in all-angles output
    const bool tr = mi.hor && !allangs;
    int o[N][N];
#pragma unroll
    for (int r = 0; r < N; r++)
#pragma unroll
        for (int c = 0; c < N; c++) o[r][c] = tr ? v[c][r] : v[r][c];

    // compact blocks (stride N) of consecutive jobs at consecutive addresses: the wave's outputs are one
    // contiguous run, written with coalesced 16-byte stores instead of one short row per lane
    const int lane = threadIdx.x & 63;
    const P* out0 = (const P*)__shfl((long long)(intptr_t)out, 0, 64);
    const bool run = os == N && (!live || out == out0 + (int64_t)lane * N * N);
    const bool wave_run = __all(run);
    if constexpr (N == 4)
    {
        if (!live) return;
        if (os == 4)
        {
            uint32_t w[NB / 4];
#pragma unroll
            for (int r = 0; r < 4; r++)
            {
                if constexpr (sizeof(P) == 1)
                    w[r] = (uint32_t)o[r][0] | ((uint32_t)o[r][1] << 8) | ((uint32_t)o[r][2] << 16) | ((uint32_t)o[r][3] << 24);
                else
                {
                    w[2 * r] = (uint32_t)o[r][0] | ((uint32_t)o[r][1] << 16);
                    w[2 * r + 1] = (uint32_t)o[r][2] | ((uint32_t)o[r][3] << 16);
                }
            }
#pragma unroll
            for (int q = 0; q < NB / 16; q++)
                stu<uint4>((uint8_t*)out + 16 * q, make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]));
            return;
        }
    }
    else
    {
        const int wv = threadIdx.x >> 6;
        // block-uniform decision (every lane has left D once the barrier returns)
        if (__syncthreads_and(wave_run))
        {
            uint8_t* stg = (uint8_t*)lds + (size_t)wv * 64 * NB;
            uint32_t* mine = (uint32_t*)(stg + lane * NB);
#pragma unroll
            for (int r = 0; r < N; r++)
            {
                if constexpr (sizeof(P) == 1)
                {
                    mine[2 * r] = (uint32_t)o[r][0] | ((uint32_t)o[r][1] << 8) | ((uint32_t)o[r][2] << 16) | ((uint32_t)o[r][3] << 24);
                    mine[2 * r + 1] = (uint32_t)o[r][4] | ((uint32_t)o[r][5] << 8) | ((uint32_t)o[r][6] << 16) | ((uint32_t)o[r][7] << 24);
                }
                else
                {
#pragma unroll
                    for (int q = 0; q < 4; q++) mine[4 * r + q] = (uint32_t)o[r][2 * q] | ((uint32_t)o[r][2 * q + 1] << 16);
                }
            }
            __syncthreads();
            const int64_t live_jobs = (int64_t)n - (job - lane);
            const int64_t lim = (live_jobs < 64 ? live_jobs : 64) * NB;    // bytes of the wave's live jobs
            uint8_t* base = (uint8_t*)out0;
#pragma unroll
            for (int q = 0; q < NB / 16; q++)
            {
                const int off = (q * 64 + lane) * 16;
                if (off < lim) stu<uint4>(base + off, *(const uint4*)(stg + off));
            }
            return;
        }
        if (!live) return;
    }
#pragma unroll
    for (int r = 0; r < N; r++) store_row<P, N>(out + (int64_t)r * os, o[r]);
}

// 16x16 / 32x32: four lanes per (TU, mode) job, 16 jobs per wave, lane q producing rows q, q + 4, .. (a job's
// four lanes write four consecutive rows: 128 contiguous bytes per pass).  The job's 4N+1 neighbours go
// to LDS once (each lane loads a quarter), the four lanes build the job's reference pairs
// D[j] = (R[j], R[j+1]) in the mode's frame (flip, projected left samples) together, and every angular
// pixel is one ds_read_b32 + v_dot2 (8-bit vertical modes: packed u16, (32 - f)·(a, b) + f·(b, c) gives two
// neighbouring pixels per v_pk_mad pair).  Wave-private LDS (the wave's 16 jobs): wave-level ordering only,
// no block barrier.  (Rounds 1-2 used N lanes per job and a block-wide LDS array: 1-4 jobs per wave in
// flight, 0.28 / 0.34 of HBM peak at 16 / 32 against 0.43 / 0.43 here.)
// one N-pixel output row (16-pixel pieces, or one 8-pixel store for N = 8)
template <typename P, int N>
__device__ __forceinline__ void store_quad_row(P* p, const int (&o)[N])
{
    if constexpr (N == 8)
        store_row<P, 8>(p, o);
    else
    {
#pragma unroll
        for (int h = 0; h < N; h += 16) store_row<P, 16>(p + h, *(const int(*)[16])(o + h));
    }
}

// v_pk_mad_u16 with the addend as an SGPR operand (left to the compiler, a constant addend becomes a
// v_pk_mul_lo_u16 + v_pk_add_u16 pair)
__device__ __forceinline__ uint32_t pmad_s(uint32_t a, uint32_t b, uint32_t c)
{
    uint32_t r;
    asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
}

// v_dot2_u32_u16 with the accumulator start (the builtin: the compiler then knows the instruction and keeps
// the wait states a dot result needs before its consumer — as inline asm, hidden from its hazard
// recognizer, the same start-folding trick produced wrong chroma hpp lanes in the interpolation kernels)
__device__ __forceinline__ uint32_t udot2_sinit(uint32_t a, uint32_t b, uint32_t init)
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b), init, false);
}

template <typename P, int N, int G = 4>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_intra_quad(int n, int maxv,
    P* __restrict__ dst, intptr_t ds, const int64_t* __restrict__ doff,
    const P* __restrict__ nb, const int64_t* __restrict__ nboff,
    const P* __restrict__ filt, const int64_t* __restrict__ filtoff,
    const uint8_t* __restrict__ mode, const uint8_t* __restrict__ bfilter, int allangs)
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    constexpr int JOBS = X265AMD_BLOCK / G;
    constexpr int PL = 4 * N / G;                      // neighbours loaded per lane
    constexpr int N2 = 2 * N, NS = 4 * N + 4, ND = 3 * N + 1;      // padded strides (u16 / dwords)
    constexpr int LG2 = N == 8 ? 3 : N == 16 ? 4 : 5;
    __shared__ uint16_t S[JOBS][NS];                   // the neighbours as loaded
    __shared__ uint32_t D[JOBS][ND];                   // reference pairs in the mode's frame
    const int t = threadIdx.x, slot = t / G, q = t % G;
    const int64_t job = (int64_t)xcd_block() * JOBS + slot;
    const bool live = job < n;
    const int64_t jj = live ? job : 0;

    int m, bf;
    const P* src;
    P* out;
    intptr_t os;
    if (allangs)
    {
        const int64_t tu = jj / 33;
        m = 2 + (int)(jj % 33);
        bf = bfilter[tu];
        src = (c_intra.filter_flags[m] & N) ? filt + filtoff[tu] : nb + nboff[tu];
        out = dst + doff[tu] + (int64_t)(m - 2) * N * N;
        os = N;
    }
    else
    {
        m = mode[jj];
        bf = bfilter[jj];
        src = nb + nboff[jj];
        out = dst + doff[jj];
        os = ds;
    }
    // neighbours: lane q loads pixels q·PL .. q·PL + PL - 1 (lane G - 1 also pixel 4N)
    {
        static_assert(PL % 16 == 0, "16-pixel neighbour loads");
        int v[PL];
#pragma unroll
        for (int h = 0; h < PL; h += 16) load_row<P, 16>(src + q * PL + h, *(int(*)[16])(v + h));
#pragma unroll
        for (int k = 0; k < PL; k++) S[slot][q * PL + k] = (uint16_t)v[k];
        if (q == G - 1) S[slot][4 * N] = (uint16_t)src[4 * N];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const ModeInfo mi = decode_mode(m);
    const bool fh = mi.hor && m >= 2;                  // the mode's frame is the flipped one
    const uint16_t* sj = S[slot];
    const int nproj = mi.angle < 0 ? -((N * mi.angle) >> 5) - 1 : 0;
    // R[k], k = 0 .. 3N (R[N - 1] = top-left, R[N ..] = above in the mode's frame, below N - 1 the
    // projected left samples of negative angles, intrapred.cpp:154-164)
    auto Rv = [&](int k) -> uint32_t {
        if (k >= N - 1)
        {
            const int e = k - N + 1;
            if (e > N2) return 0;
            return sj[flip_index(e, N2, fh)];
        }
        const int kk = N - 2 - k;                      // R[-2 - kk]
        if (kk >= nproj) return 0;
        const int i = (128 + (kk + 1) * mi.inv) >> 8;  // = L[i - 1] = s'[2N + i]
        return sj[flip_index(N2 + i, N2, fh)];
    };
#pragma unroll
    for (int i = 0; i < 3 * N / G; i++)
    {
        const int j = i * G + q;
        D[slot][j] = Rv(j) | (Rv(j + 1) << 16);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (!live) return;
    const uint32_t* Dj = D[slot];
    const bool tr = fh && !allangs;
    // unflipped neighbours for planar / DC: above[x] = s[1 + x], left[y] = s[2N + 1 + y]
    if (m <= 1)
    {
        int above[N];
#pragma unroll
        for (int x = 0; x < N; x++) above[x] = sj[1 + x];
        int dc = 0;
        if (m == 1)
        {
            int sum = N;
#pragma unroll
            for (int i = 0; i < N; i++) sum += above[i] + sj[N2 + 1 + i];
            dc = sum >> (LG2 + 1);
        }
        const int trr = sj[N + 1], bl = sj[N2 + 1 + N];
#pragma unroll
        for (int i = 0; i < N / G; i++)
        {
            const int r = i * G + q;
            const int lr = sj[N2 + 1 + r];
            int o[N];
            if (m == 0)
            {
#pragma unroll
                for (int x = 0; x < N; x++)
                    o[x] = ((N - 1 - x) * lr + (N - 1 - r) * above[x] + (x + 1) * trr + (r + 1) * bl + N) >> (LG2 + 1);
            }
            else
            {
#pragma unroll
                for (int x = 0; x < N; x++) o[x] = dc;
                if (bf)
                {
                    if (r == 0)
                    {
                        o[0] = (above[0] + lr + 2 * dc + 2) >> 2;
#pragma unroll
                        for (int x = 1; x < N; x++) o[x] = (above[x] + 3 * dc + 2) >> 2;
                    }
                    else
                        o[0] = (lr + 3 * dc + 2) >> 2;
                }
            }
            store_quad_row<P, N>(out + (int64_t)r * os, o);
        }
        return;
    }
    const int Rn = (int)(Dj[N] & 0xffff), Rn1 = (int)(Dj[N - 1] & 0xffff);   // R[0], R[-1] of the frame
    const bool edge = mi.angle == 0 && bf;
    auto edge_px = [&](int l) {
        const int e = (int16_t)(Rn + ((l - Rn1) >> 1));
        return e < 0 ? 0 : (e > maxv ? maxv : e);
    };
    if (!tr && sizeof(P) == 1)
    {
        // 8 bit: two pixels of the row per packed-u16 multiply-add pair.  The weights are scaled by 8
        // (and the rounding 16 by 8): 8 ((32 - f) a + f b + 16) <= 65408 still fits a u16 lane, and the
        // pixel ((32 - f) a + f b + 16) >> 5 is its high byte, so one v_perm takes four pixels' bytes
        auto pmad = [](uint32_t a, uint32_t b, uint32_t c) -> uint32_t {
            return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) * __builtin_bit_cast(u16x2, b) +
                                                    __builtin_bit_cast(u16x2, c));
        };
#pragma unroll
        for (int i = 0; i < N / G; i++)
        {
            const int r = i * G + q;
            const int sum = (r + 1) * mi.angle, f = sum & 31;
            const uint32_t w0 = (uint32_t)(8 * (32 - f)) * 0x10001u, w1 = (uint32_t)(8 * f) * 0x10001u;
            const uint32_t* row = Dj + N + (sum >> 5);
            uint32_t pq[N / 2], w[N / 4];
#pragma unroll
            for (int k = 0; k < N / 2; k++) pq[k] = pmad(row[2 * k], w0, pmad_s(row[2 * k + 1], w1, 0x00800080u));
#pragma unroll
            for (int k = 0; k < N / 4; k++) w[k] = __builtin_amdgcn_perm(pq[2 * k + 1], pq[2 * k], 0x07050301u);
            if (edge) w[0] = (w[0] & ~0xffu) | (uint32_t)edge_px(sj[flip_index(N2 + 1 + r, N2, fh)]);
            uint8_t* o8 = (uint8_t*)(out + (int64_t)r * os);
            if constexpr (N == 8)
                stu<uint2>(o8, make_uint2(w[0], w[1]));
            else
            {
#pragma unroll
                for (int k = 0; k < N / 16; k++) stu<uint4>(o8 + 16 * k, make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]));
            }
        }
    }
    else if (!tr)
    {
#pragma unroll
        for (int i = 0; i < N / G; i++)
        {
            const int r = i * G + q;
            const int sum = (r + 1) * mi.angle, f = sum & 31;
            const u16x2 wt = {(unsigned short)(32 - f), (unsigned short)f};
            const uint32_t* row = Dj + N + (sum >> 5);
            int o[N];
#pragma unroll
            for (int x = 0; x < N; x++)
                o[x] = (int)(__builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, row[x]), wt, 16u, false) >> 5);
            if (edge) o[0] = edge_px(sj[flip_index(N2 + 1 + r, N2, fh)]);
            store_quad_row<P, N>(out + (int64_t)r * os, o);
        }
    }
    else if (sizeof(P) == 1)
    {
        // 8 bit, transposed (horizontal modes): output column c of row r reads the pair at row
        // offset r of the column's reference run; weights scaled by 8 as above, the rounding 128
        // as the dot's SGPR operand, each pixel the sum's byte 1 (three v_perm per four pixels)
        int offc[N];
        uint32_t wc[N];
#pragma unroll
        for (int c = 0; c < N; c++)
        {
            const int sum = (c + 1) * mi.angle, f = sum & 31;
            offc[c] = N + (sum >> 5);
            wc[c] = (uint32_t)(8 * (32 - f)) | ((uint32_t)(8 * f) << 16);
        }
#pragma unroll
        for (int i = 0; i < N / G; i++)
        {
            const int r = i * G + q;
            uint8_t* o8 = (uint8_t*)(out + (int64_t)r * os);
            if (edge && r == 0)
            {
                int o[N];
#pragma unroll
                for (int c = 0; c < N; c++) o[c] = edge_px(sj[flip_index(N2 + 1 + c, N2, fh)]);
                store_quad_row<P, N>(out + (int64_t)r * os, o);
                continue;
            }
            uint32_t w[N / 4];
#pragma unroll
            for (int k = 0; k < N / 4; k++)
            {
                uint32_t t[4];
#pragma unroll
                for (int e = 0; e < 4; e++) t[e] = udot2_sinit(Dj[offc[4 * k + e] + r], wc[4 * k + e], 128);
                w[k] = __builtin_amdgcn_perm(t[1], t[0], 0x0c0c0501u) | __builtin_amdgcn_perm(t[3], t[2], 0x05010c0cu);
            }
            if constexpr (N == 8)
                stu<uint2>(o8, make_uint2(w[0], w[1]));
            else
            {
#pragma unroll
                for (int k = 0; k < N / 16; k++) stu<uint4>(o8 + 16 * k, make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]));
            }
        }
    }
    else
    {
        int offc[N];
        u16x2 wc[N];
#pragma unroll
        for (int c = 0; c < N; c++)
        {
            const int sum = (c + 1) * mi.angle, f = sum & 31;
            offc[c] = N + (sum >> 5);
            wc[c] = u16x2{(unsigned short)(32 - f), (unsigned short)f};
        }
#pragma unroll
        for (int i = 0; i < N / G; i++)
        {
            const int r = i * G + q;
            int o[N];
#pragma unroll
            for (int c = 0; c < N; c++)
                o[c] = (int)(__builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, Dj[offc[c] + r]), wc[c], 16u, false) >> 5);
            if (edge && r == 0)
            {
#pragma unroll
                for (int c = 0; c < N; c++) o[c] = edge_px(sj[flip_index(N2 + 1 + c, N2, fh)]);
            }
            store_quad_row<P, N>(out + (int64_t)r * os, o);
        }
    }
}

// intraFilter (intrapred.cpp:31-51): N lanes per job, lane l filters pixels 4l .. 4l+3 of the
// 4N+1 neighbours from one vector load plus its two outer neighbours (lane 0 also copies
// pixel 4N); 256 / N jobs per block
template <typename P>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_intra_filter(int N, int n, const P* __restrict__ src,
    const int64_t* __restrict__ soff, P* __restrict__ dst, const int64_t* __restrict__ doff)
{
    const int lg = N == 4 ? 2 : N == 8 ? 3 : N == 16 ? 4 : 5;
    const int64_t job = (int64_t)xcd_block() * (X265AMD_BLOCK >> lg) + (threadIdx.x >> lg);
    const int l = threadIdx.x & (N - 1);
    if (job >= n) return;
    const P* s = src + soff[job];
    P* d = dst + doff[job];
    const int n2 = 2 * N, i0 = 4 * l;
    int v[4], o[4];
    load_row<P, 4>(s + i0, v);
    const int left = l ? (int)s[i0 - 1] : (int)s[n2 + 1];        // pixel 0's other neighbour is s[2N + 1]
    const int right = s[i0 + 4];
#pragma unroll
    for (int k = 0; k < 4; k++)
    {
        const int i = i0 + k;
        const int a = k ? v[k - 1] : left, b = k < 3 ? v[k + 1] : right;
        if (i == n2) o[k] = v[k];                                   // top-left-most above-right end
        else if (i == n2 + 1) o[k] = (2 * v[k] + (int)s[0] + b + 2) >> 2;
        else o[k] = (2 * v[k] + a + b + 2) >> 2;
    }
    store_row<P, 4>(d + i0, o);
    if (l == 0) d[4 * N] = s[4 * N];
}

template <typename P>
static int launch_pred(int N, int n, int depth, void* dst, intptr_t ds, const int64_t* doff, const void* nb,
                       const int64_t* nboff, const void* filt, const int64_t* filtoff, const uint8_t* mode,
                       const uint8_t* bfilter, int allangs, hipStream_t st)
{
    // lanes per job of the 16x16 / 32x32 kernel (X265AMD_INTRA_G16 / _G32 override for tuning runs)
    auto env_int = [](const char* name, int dflt) { const char* e = getenv(name); return e ? atoi(e) : dflt; };
    static const int g8 = env_int("X265AMD_INTRA_G8", 0);     // 0: the lane-per-job kernel
    static const int g16 = env_int("X265AMD_INTRA_G16", 4), g32 = env_int("X265AMD_INTRA_G32", 4);
    const int G = N == 8 ? g8 : N == 16 ? g16 : N == 32 ? g32 : 0;
    const int per = N == 4 ? X265AMD_BLOCK * kIntraLaneJobs : G ? X265AMD_BLOCK / G : X265AMD_BLOCK;
    const dim3 grid((n + per - 1) / per);
#define L(K) hipLaunchKernelGGL(K, grid, dim3(X265AMD_BLOCK), 0, st, n, (1 << depth) - 1, \
                                (P*)dst, ds, doff, (const P*)nb, nboff, (const P*)filt, filtoff, mode, bfilter, allangs)
    if (N == 4) L((k_intra_lane<P, 4>));
    else if (N == 8 && G == 2) L((k_intra_quad<P, 8, 2>));
    else if (N == 8) L((k_intra_lane<P, 8>));
    else if (N == 16 && G == 2) L((k_intra_quad<P, 16, 2>));
    else if (N == 16 && G == 4) L((k_intra_quad<P, 16, 4>));
    else if (N == 32 && G == 4) L((k_intra_quad<P, 32, 4>));
    else if (N == 32 && G == 8) L((k_intra_quad<P, 32, 8>));
    else return X265AMD_EINVAL;
#undef L
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
    const int per = X265AMD_BLOCK / size;
    const dim3 grid((n + per - 1) / per);
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
