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
// Work mapping (template on the TU size N): one (TU, mode) job per N-lane
// group, lane r producing output row r (N pixels, stored as full-row vector
// stores).  The group builds the reference array of intra_pred_ang_c in LDS
// exactly once per job, as one CONTIGUOUS int16 array R[-N .. 2N] (projected
// left samples, top-left, the 2N above samples — all in the mode's flipped
// frame) plus the N+1 samples of the other side L[0 .. N]; every angular
// pixel is then two LDS reads and one blend.  The mode is decoded once per job
// from packed register constants (no table loads).
#include "common.h"
#include "intra_lane.h"
#include "../../../include/x265_amd.h"

namespace x265amd {

typedef unsigned short pair16 __attribute__((ext_vector_type(2)));

template <typename P, int N>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_intra_pred(int n, int maxv,
    P* __restrict__ dst, intptr_t ds, const int64_t* __restrict__ doff,
    const P* __restrict__ nb, const int64_t* __restrict__ nboff,
    const P* __restrict__ filt, const int64_t* __restrict__ filtoff,
    const uint8_t* __restrict__ mode, const uint8_t* __restrict__ bfilter, int allangs)
{
    constexpr int JOBS = X265AMD_BLOCK / N;
    constexpr int N2 = 2 * N;
    constexpr int LG2 = N == 4 ? 2 : N == 8 ? 3 : N == 16 ? 4 : 5;
    constexpr int SLOT = 4 * N + 4;                  // R: 3N+1, L: N+1, padded
    constexpr int PW = 3 * N;                        // pairs D[j] = (R[j], R[j + 1]), j = -N .. 2N-1
    __shared__ int16_t sh[JOBS][SLOT];
    __shared__ int16_t raw[JOBS][4 * N + 2];         // the 4N+1 neighbours as loaded
    __shared__ uint32_t Dp[JOBS][PW];
    const int slot = threadIdx.x / N, r = threadIdx.x % N;
    const int64_t job = (int64_t)xcd_block() * JOBS + slot;
    const bool live = job < n;
    const int64_t jj = live ? job : 0;
    int16_t* R = sh[slot] + N;                       // R[j], j = -N .. 2N
    int16_t* L = sh[slot] + 3 * N + 2;               // L[y], y = 0 .. N
    uint32_t* D = Dp[slot] + N;                      // D[j], j = -N .. 2N-1

    int m, bf;
    const P* src;
    P* out;
    if (allangs)
    {
        // job = tu * 33 + (mode - 2); filtered or unfiltered neighbours per g_intraFilterFlags
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

    // ---- neighbours: lane r loads pixels 4r .. 4r+3 with one vector load (lane 0 also pixel 4N)
    {
        int t[4];
        load_row<P, 4>(src + 4 * r, t);
#pragma unroll
        for (int k = 0; k < 4; k++) raw[slot][4 * r + k] = (int16_t)t[k];
        if (r == 0) raw[slot][4 * N] = (int16_t)src[4 * N];
    }
    __syncthreads();
    const int16_t* sr = raw[slot];
    // ---- R[j] = s'[1 + j] for j = -1 .. 2N-1, L[y] = s'[2N + 1 + y] for y = 0 .. N
    //      (s' = neighbours in the mode's frame), R[-2-k] = projected left samples
    for (int e = r; e < N2 + 1; e += N) R[e - 1] = sr[flip_index(e, N2, mi.hor)];
    for (int y = r; y <= N; y += N) L[y] = sr[flip_index(N2 + 1 + y, N2, mi.hor)];
    if (mi.angle < 0)
    {
        const int nproj = -((N * mi.angle) >> 5) - 1;     // intrapred.cpp:154-164
        for (int k = r; k < nproj; k += N)
            R[-2 - k] = sr[flip_index(N2 + ((128 + (k + 1) * mi.inv) >> 8), N2, mi.hor)];
    }
    __syncthreads();
    // pairs for the angular interpolation: one ds_read_b32 + one v_dot2 per pixel
    for (int j = r - N; j < 2 * N; j += N) D[j] = (uint32_t)(uint16_t)R[j] | ((uint32_t)(uint16_t)R[j + 1] << 16);
    __syncthreads();
    if (!live) return;

    int v[N];
    if (m == 0)   // planar (intrapred.cpp:87-100), unflipped: above = R[0..N], left = L[0..N]
    {
        const int lr = L[r], bl = L[N], tr = R[N];
#pragma unroll
        for (int x = 0; x < N; x++)
            v[x] = ((N - 1 - x) * lr + (N - 1 - r) * R[x] + (x + 1) * tr + (r + 1) * bl + N) >> (LG2 + 1);
    }
    else if (m == 1)   // DC (+ dcPredFilter, intrapred.cpp:53-85)
    {
        int t = N;
#pragma unroll
        for (int i = 0; i < N; i++) t += R[i] + L[i];
        const int dc = t / N2;
#pragma unroll
        for (int x = 0; x < N; x++) v[x] = dc;
        if (bf)
        {
            if (r == 0)
            {
                v[0] = (R[0] + L[0] + 2 * dc + 2) >> 2;
#pragma unroll
                for (int x = 1; x < N; x++) v[x] = (R[x] + 3 * dc + 2) >> 2;
            }
            else
                v[0] = (L[r] + 3 * dc + 2) >> 2;
        }
    }
    else if (!mi.hor || allangs)
    {
        // output row r is vertical-frame row y = r: one (offset, fraction) for the whole row
        const int sum = (r + 1) * mi.angle, off = sum >> 5, f = sum & 31;
        if (mi.angle == 0)
        {
#pragma unroll
            for (int x = 0; x < N; x++) v[x] = R[x];
            if (bf)
            {
                const int t = (int16_t)(R[0] + ((L[r] - R[-1]) >> 1));
                v[0] = t < 0 ? 0 : (t > maxv ? maxv : t);
            }
        }
        else
        {
            const pair16 wt = {(unsigned short)(32 - f), (unsigned short)f};
            const uint32_t* row = D + off;
#pragma unroll
            for (int x = 0; x < N; x++)
                v[x] = (int)(__builtin_amdgcn_udot2(__builtin_bit_cast(pair16, row[x]), wt, 16u, false) >> 5);
        }
    }
    else
    {
        // horizontal mode, reference orientation: output (r, c) = vertical-frame (y = c, x = r)
        if (mi.angle == 0)
        {
            // x = r: every pixel of the row is R[r], except column x = 0 of the vertical frame (row r = 0)
#pragma unroll
            for (int c = 0; c < N; c++)
            {
                int p = R[r];
                if (bf && r == 0)
                {
                    const int t = (int16_t)(R[0] + ((L[c] - R[-1]) >> 1));
                    p = t < 0 ? 0 : (t > maxv ? maxv : t);
                }
                v[c] = p;
            }
        }
        else
        {
#pragma unroll
            for (int c = 0; c < N; c++)
            {
                const int sum = (c + 1) * mi.angle, off = sum >> 5, f = sum & 31;
                const pair16 wt = {(unsigned short)(32 - f), (unsigned short)f};
                v[c] = (int)(__builtin_amdgcn_udot2(__builtin_bit_cast(pair16, D[off + r]), wt, 16u, false) >> 5);
            }
        }
    }
    P* orow = out + (int64_t)r * (allangs ? N : ds);
    if constexpr (N == 4)
        store_row<P, 4>(orow, v);
    else
    {
#pragma unroll
        for (int x = 0; x < N; x += 8)
        {
            int t[8];
#pragma unroll
            for (int k = 0; k < 8; k++) t[k] = v[x + k];
            store_row<P, 8>(orow + x, t);
        }
    }
}

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
    const int per = N == 4 ? X265AMD_BLOCK * kIntraLaneJobs : N <= 8 ? X265AMD_BLOCK : X265AMD_BLOCK / N;
    const dim3 grid((n + per - 1) / per);
#define L(K, NN) hipLaunchKernelGGL((K<P, NN>), grid, dim3(X265AMD_BLOCK), 0, st, n, (1 << depth) - 1, \
                                    (P*)dst, ds, doff, (const P*)nb, nboff, (const P*)filt, filtoff, mode, bfilter, allangs)
    switch (N)
    {
    case 4: L(k_intra_lane, 4); break;
    case 8: L(k_intra_lane, 8); break;
    case 16: L(k_intra_pred, 16); break;
    case 32: L(k_intra_pred, 32); break;
    default: return X265AMD_EINVAL;
    }
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
