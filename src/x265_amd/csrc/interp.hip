// interp.hip — batched luma 8-tap / chroma 4-tap sub-pel interpolation.
//
// Reference semantics: x265_1.9/source/common/ipfilter.cpp
//   filterPixelToShort_c :40-57     interp_horiz_pp_c :79-118
//   interp_horiz_ps_c    :120-163   interp_vert_pp_c  :165-204
//   interp_vert_ps_c     :206-242   interp_vert_sp_c  :244-285
//   interp_vert_ss_c     :287-320   interp_hv_pp_c    :365-372
// Fixed-point constants IF_FILTER_PREC = 6, IF_INTERNAL_PREC = 14,
// IF_INTERNAL_OFFS = 8192 (constants.h:70-74).  Bit-exactness (SURVEY.md
// Appendix A.4): ps/ss results wrap to int16; pp/sp results are truncated to
// int16 first and then clamped to [0, (1<<depth)-1].
//
// Work mapping: one job (one PU) per G-lane group; a lane produces a UWxUH
// output unit.  Horizontal filters load exactly the UW+taps-1 source pixels a
// row needs (overlapping dword/qword loads, never outside the reference's
// read window); vertical filters slide a taps-row window through registers so
// each source row is loaded once per unit; hv_pp recomputes the horizontal
// int16 intermediate for the UH+7 rows its unit needs, entirely on-chip.
#include "common.h"
#include "../../../include/x265_amd.h"

namespace x265amd {

// load exactly N consecutive elements (pixels or int16) into o[]
template <typename T, int N>
__device__ __forceinline__ void load_win(const T* p, int (&o)[N])
{
    if constexpr (N >= 8)
    {
#pragma unroll
        for (int i = 0; i + 8 <= N; i += 8)
        {
            int t[8];
            if constexpr (sizeof(T) == 1 || std::is_same<T, uint16_t>::value) load_row<T, 8>(p + i, t);
            else load_row16<8>((const int16_t*)p + i, t);
#pragma unroll
            for (int k = 0; k < 8; k++) o[i + k] = t[k];
        }
        if constexpr (N % 8)
        {
            int t[8];
            if constexpr (sizeof(T) == 1 || std::is_same<T, uint16_t>::value) load_row<T, 8>(p + N - 8, t);
            else load_row16<8>((const int16_t*)p + N - 8, t);
#pragma unroll
            for (int k = 0; k < 8; k++) o[N - 8 + k] = t[k];
        }
    }
    else
    {
        static_assert(N >= 4, "window too small");
        int t[4], u[4];
        if constexpr (sizeof(T) == 1 || std::is_same<T, uint16_t>::value) { load_row<T, 4>(p, t); load_row<T, 4>(p + N - 4, u); }
        else { load_row16<4>((const int16_t*)p, t); load_row16<4>((const int16_t*)p + N - 4, u); }
#pragma unroll
        for (int k = 0; k < 4; k++) { o[k] = t[k]; o[N - 4 + k] = u[k]; }
    }
}

template <typename T, int UW>
__device__ __forceinline__ void load_unit_row(const T* p, int (&o)[UW])
{
    if constexpr (sizeof(T) == 1 || std::is_same<T, uint16_t>::value) load_row<T, UW>(p, o);
    else load_row16<UW>((const int16_t*)p, o);
}

template <int TAPS>
__device__ __forceinline__ void get_taps(int idx, int (&c)[TAPS])
{
#pragma unroll
    for (int k = 0; k < TAPS; k++)
        c[k] = TAPS == 8 ? c_luma.c[idx & 3][k] : c_chroma.c[idx & 7][k];
}

struct IfConst
{
    int maxv, ps_shift, ps_off, sp_shift, sp_off, p2s_shift;
    __device__ __forceinline__ IfConst(int depth)
    {
        const int head = 14 - depth;             // IF_INTERNAL_PREC - depth
        maxv = (1 << depth) - 1;
        ps_shift = 6 - head;                     // IF_FILTER_PREC - headRoom
        ps_off = -8192 * (1 << ps_shift);        // -IF_INTERNAL_OFFS << shift
        sp_shift = 6 + head;
        sp_off = (1 << (sp_shift - 1)) + (8192 << 6);
        p2s_shift = head;
    }
};

__device__ __forceinline__ int clampp(int v16, int maxv)
{
    // (int16_t) truncation first, then clamp to the pixel range
    int v = (int16_t)v16;
    return v < 0 ? 0 : (v > maxv ? maxv : v);
}

// horizontal filter of one output strip (UW outputs) from an exact window
template <typename P, int TAPS, int UW>
__device__ __forceinline__ void hfilter(const P* src, const int (&c)[TAPS], int (&sum)[UW])
{
    int win[UW + TAPS - 1];
    load_win<P, UW + TAPS - 1>(src - (TAPS / 2 - 1), win);
#pragma unroll
    for (int x = 0; x < UW; x++)
    {
        int s = 0;
#pragma unroll
        for (int k = 0; k < TAPS; k++) s += win[x + k] * c[k];
        sum[x] = s;
    }
}

template <typename P, typename S, typename D, int OP, int TAPS, int UW, int UH>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_interp(int w, int h, int n, int lg, int depth,
    const S* __restrict__ src, intptr_t ss, const int64_t* __restrict__ soff,
    D* __restrict__ dst, intptr_t ds, const int64_t* __restrict__ doff,
    const uint8_t* __restrict__ coeff, int rowext)
{
    const int G = 1 << lg;
    const uint32_t lb = xcd_block();
    const int64_t job = (int64_t)lb * (X265AMD_BLOCK >> lg) + (threadIdx.x >> lg);
    const int lane = threadIdx.x & (G - 1);
    if (job >= n) return;

    const IfConst K(depth);
    const S* ps = src + soff[job];
    D* pd = dst + doff[job];
    const int cidx = coeff ? coeff[job] : 0;

    int rows = h;
    if constexpr (OP == X265AMD_HPS)
    {
        if (rowext)
        {
            ps -= (TAPS / 2 - 1) * ss;
            rows += TAPS - 1;
        }
    }
    const int ux = w / UW, units = ux * (rows / UH);

    int c[TAPS];
    get_taps<TAPS>(OP == X265AMD_HVPP ? (cidx & 15) : cidx, c);

    for (int u = lane; u < units; u += G)
    {
        const int x = (u % ux) * UW, y0 = (u / ux) * UH;

        if constexpr (OP == X265AMD_HPP || OP == X265AMD_HPS)
        {
#pragma unroll
            for (int r = 0; r < UH; r++)
            {
                int sum[UW], o[UW];
                hfilter<P, TAPS, UW>((const P*)ps + (y0 + r) * ss + x, c, sum);
#pragma unroll
                for (int i = 0; i < UW; i++)
                    o[i] = OP == X265AMD_HPP ? clampp((sum[i] + 32) >> 6, K.maxv)
                                             : (int)(int16_t)((sum[i] + K.ps_off) >> K.ps_shift);
                store_row<D, UW>(pd + (y0 + r) * ds + x, o);
            }
        }
        else if constexpr (OP == X265AMD_P2S)
        {
#pragma unroll
            for (int r = 0; r < UH; r++)
            {
                int v[UW];
                load_row<P, UW>((const P*)ps + (y0 + r) * ss + x, v);
#pragma unroll
                for (int i = 0; i < UW; i++) v[i] = (int)(int16_t)((int16_t)(v[i] << K.p2s_shift) - 8192);
                store_row<D, UW>(pd + (y0 + r) * ds + x, v);
            }
        }
        else if constexpr (OP == X265AMD_HVPP)
        {
            // immed rows y0 .. y0+UH+6 (immed row i = horizontal ps of src row i-3)
            int cy[TAPS];
            get_taps<TAPS>(cidx >> 4, cy);
            int acc[UH][UW];
#pragma unroll
            for (int r = 0; r < UH; r++)
#pragma unroll
                for (int i = 0; i < UW; i++) acc[r][i] = 0;
#pragma unroll
            for (int t = 0; t < UH + TAPS - 1; t++)
            {
                int sum[UW];
                hfilter<P, TAPS, UW>((const P*)ps + (y0 + t - (TAPS / 2 - 1)) * ss + x, c, sum);
#pragma unroll
                for (int i = 0; i < UW; i++) sum[i] = (int)(int16_t)((sum[i] + K.ps_off) >> K.ps_shift);
#pragma unroll
                for (int r = 0; r < UH; r++)
                {
                    const int k = t - r;
                    if (k >= 0 && k < TAPS)
                    {
#pragma unroll
                        for (int i = 0; i < UW; i++) acc[r][i] += sum[i] * cy[k];
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < UH; r++)
            {
                int o[UW];
#pragma unroll
                for (int i = 0; i < UW; i++) o[i] = clampp((acc[r][i] + K.sp_off) >> K.sp_shift, K.maxv);
                store_row<D, UW>(pd + (y0 + r) * ds + x, o);
            }
        }
        else  // vertical: VPP, VPS, VSP, VSS
        {
            int acc[UH][UW];
#pragma unroll
            for (int r = 0; r < UH; r++)
#pragma unroll
                for (int i = 0; i < UW; i++) acc[r][i] = 0;
            const S* col = ps + (y0 - (TAPS / 2 - 1)) * ss + x;
#pragma unroll
            for (int t = 0; t < UH + TAPS - 1; t++)
            {
                int v[UW];
                load_unit_row<S, UW>(col + t * ss, v);
#pragma unroll
                for (int r = 0; r < UH; r++)
                {
                    const int k = t - r;
                    if (k >= 0 && k < TAPS)
                    {
#pragma unroll
                        for (int i = 0; i < UW; i++) acc[r][i] += v[i] * c[k];
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < UH; r++)
            {
                int o[UW];
#pragma unroll
                for (int i = 0; i < UW; i++)
                {
                    const int s = acc[r][i];
                    if constexpr (OP == X265AMD_VPP) o[i] = clampp((s + 32) >> 6, K.maxv);
                    else if constexpr (OP == X265AMD_VPS) o[i] = (int)(int16_t)((s + K.ps_off) >> K.ps_shift);
                    else if constexpr (OP == X265AMD_VSP) o[i] = clampp((s + K.sp_off) >> K.sp_shift, K.maxv);
                    else o[i] = (int)(int16_t)(s >> 6);
                }
                store_row<D, UW>(pd + (y0 + r) * ds + x, o);
            }
        }
    }
}

// hv_pp in two on-chip passes: the horizontal int16 intermediate of the
// (h+7) x w block (interp_horiz_ps_c with row extension) goes to LDS once,
// then the vertical sp filter reads it back (filterVertical_sp_c).  Jobs per
// block = 256 / G, LDS = jobs * (h+7) * w int16.
template <typename P, int UW, int UH>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_hvpp(int w, int h, int n, int lg, int depth,
    const P* __restrict__ src, intptr_t ss, const int64_t* __restrict__ soff,
    P* __restrict__ dst, intptr_t ds, const int64_t* __restrict__ doff, const uint8_t* __restrict__ coeff)
{
    extern __shared__ int16_t hv_lds[];
    const int G = 1 << lg;
    const int slot = threadIdx.x >> lg, lane = threadIdx.x & (G - 1);
    const int64_t job0 = (int64_t)xcd_block() * (X265AMD_BLOCK >> lg) + slot;
    const bool live = job0 < n;
    const int64_t job = live ? job0 : 0;
    const IfConst K(depth);
    int16_t* L = hv_lds + (size_t)slot * (h + 7) * w;
    const int cidx = coeff[job];
    int cx[8], cy[8];
    get_taps<8>(cidx & 15, cx);
    get_taps<8>(cidx >> 4, cy);
    const int ux = w / UW;

    if (live)
    {
        const P* ps = src + soff[job] - 3 * ss;
        const int hunits = ux * (h + 7);
        for (int u = lane; u < hunits; u += G)
        {
            const int x = (u % ux) * UW, t = u / ux;
            int sum[UW], o[UW];
            hfilter<P, 8, UW>(ps + t * ss + x, cx, sum);
#pragma unroll
            for (int i = 0; i < UW; i++) o[i] = (int)(int16_t)((sum[i] + K.ps_off) >> K.ps_shift);
            store_row<int16_t, UW>(L + t * w + x, o);
        }
    }
    __syncthreads();
    if (!live) return;
    P* pd = dst + doff[job];
    const int vunits = ux * (h / UH);
    for (int u = lane; u < vunits; u += G)
    {
        const int x = (u % ux) * UW, y0 = (u / ux) * UH;
        int acc[UH][UW];
#pragma unroll
        for (int r = 0; r < UH; r++)
#pragma unroll
            for (int i = 0; i < UW; i++) acc[r][i] = 0;
#pragma unroll
        for (int t = 0; t < UH + 7; t++)
        {
            int v[UW];
            load_row16<UW>(L + (y0 + t) * w + x, v);
#pragma unroll
            for (int r = 0; r < UH; r++)
            {
                const int k = t - r;
                if (k >= 0 && k < 8)
                {
#pragma unroll
                    for (int i = 0; i < UW; i++) acc[r][i] += v[i] * cy[k];
                }
            }
        }
#pragma unroll
        for (int r = 0; r < UH; r++)
        {
            int o[UW];
#pragma unroll
            for (int i = 0; i < UW; i++) o[i] = clampp((acc[r][i] + K.sp_off) >> K.sp_shift, K.maxv);
            store_row<P, UW>(pd + (y0 + r) * ds + x, o);
        }
    }
}

template <typename P>
static int launch_hvpp(int w, int h, int n, int depth, const void* src, intptr_t ss, const int64_t* soff,
                       void* dst, intptr_t ds, const int64_t* doff, const uint8_t* coeff, hipStream_t st)
{
    const int uw = w % 8 == 0 ? 8 : 4, uh = h % 4 == 0 ? 4 : 1;
    if (w % 4) return X265AMD_EINVAL;
    const int units = (w / uw) * (h / uh);
    int g = pow2ceil((units + 1) / 2);
    if (g > 64) g = 64;
    int lg = 0;
    while ((1 << lg) < g) lg++;
    // keep the workgroup's intermediate within 64 KiB of LDS
    while (lg < 6 && (size_t)(X265AMD_BLOCK >> lg) * (h + 7) * w * sizeof(int16_t) > 65536) lg++;
    const int per = X265AMD_BLOCK >> lg;
    const size_t lds = (size_t)per * (h + 7) * w * sizeof(int16_t);
    const dim3 grid((n + per - 1) / per);
#define L(UW, UH) hipLaunchKernelGGL((k_hvpp<P, UW, UH>), grid, dim3(X265AMD_BLOCK), lds, st, w, h, n, lg, depth, \
                                     (const P*)src, ss, soff, (P*)dst, ds, doff, coeff)
    if (uw == 8) { if (uh == 4) L(8, 4); else L(8, 1); }
    else { if (uh == 4) L(4, 4); else L(4, 1); }
#undef L
    return (int)hipGetLastError();
}

// -------------------------------------------------------------- dispatch

template <typename P, typename S, typename D, int OP, int TAPS, int UW, int UH>
static int launch_interp(int w, int h, int n, int depth, const void* src, intptr_t ss, const int64_t* soff,
                         void* dst, intptr_t ds, const int64_t* doff, const uint8_t* coeff, int rowext,
                         hipStream_t st)
{
    const int rows = (OP == X265AMD_HPS && rowext) ? h + TAPS - 1 : h;
    const int units = (w / UW) * (rows / UH);
    int g = pow2ceil((units + 1) / 2);    // two units per lane
    if (g > 64) g = 64;
    int lg = 0;
    while ((1 << lg) < g) lg++;
    const int per = X265AMD_BLOCK >> lg;
    hipLaunchKernelGGL((k_interp<P, S, D, OP, TAPS, UW, UH>), dim3((n + per - 1) / per), dim3(X265AMD_BLOCK), 0, st,
                       w, h, n, lg, depth, (const S*)src, ss, soff, (D*)dst, ds, doff, coeff, rowext);
    return (int)hipGetLastError();
}

template <typename P, typename S, typename D, int OP, int TAPS>
static int pick_unit(int w, int h, int n, int depth, const void* src, intptr_t ss, const int64_t* soff,
                     void* dst, intptr_t ds, const int64_t* doff, const uint8_t* coeff, int rowext, hipStream_t st)
{
    const int rows = (OP == X265AMD_HPS && rowext) ? h + TAPS - 1 : h;
#define L(UW, UH) return launch_interp<P, S, D, OP, TAPS, UW, UH>(w, h, n, depth, src, ss, soff, dst, ds, doff, coeff, rowext, st)
    if (w % 8 == 0)
    {
        if (rows % 4) L(8, 1);
        L(8, 4);
    }
    if (w % 4 == 0)
    {
        if (rows % 4) L(4, 1);
        L(4, 4);
    }
    if (w % 2 == 0)
    {
        if constexpr (TAPS == 4 || OP == X265AMD_P2S || OP == X265AMD_VPP || OP == X265AMD_VPS || OP == X265AMD_VSP || OP == X265AMD_VSS)
        {
            if (rows % 4) L(2, 1);
            L(2, 4);
        }
    }
#undef L
    return X265AMD_EINVAL;
}

template <typename P, int TAPS>
static int dispatch_interp(int op, int w, int h, int n, int depth, const void* src, intptr_t ss, const int64_t* soff,
                           void* dst, intptr_t ds, const int64_t* doff, const uint8_t* coeff, int rowext, hipStream_t st)
{
#define A w, h, n, depth, src, ss, soff, dst, ds, doff, coeff, rowext, st
    switch (op)
    {
    case X265AMD_HPP: return pick_unit<P, P, P, X265AMD_HPP, TAPS>(A);
    case X265AMD_HPS: return pick_unit<P, P, int16_t, X265AMD_HPS, TAPS>(A);
    case X265AMD_VPP: return pick_unit<P, P, P, X265AMD_VPP, TAPS>(A);
    case X265AMD_VPS: return pick_unit<P, P, int16_t, X265AMD_VPS, TAPS>(A);
    case X265AMD_VSP: return pick_unit<P, int16_t, P, X265AMD_VSP, TAPS>(A);
    case X265AMD_VSS: return pick_unit<P, int16_t, int16_t, X265AMD_VSS, TAPS>(A);
    case X265AMD_HVPP:
        if constexpr (TAPS == 8) return launch_hvpp<P>(w, h, n, depth, src, ss, soff, dst, ds, doff, coeff, st);
        return X265AMD_EINVAL;
    }
#undef A
    return X265AMD_EINVAL;
}

} // namespace x265amd

using namespace x265amd;

extern "C" int x265amd_interp(int op, int taps, int depth, int w, int h, int n,
                              const void* src, intptr_t src_stride, const int64_t* src_off,
                              void* dst, intptr_t dst_stride, const int64_t* dst_off,
                              const uint8_t* coeff, int is_row_ext, void* stream)
{
    if (n <= 0) return 0;
    if (w < 2 || h < 2 || w > 64 || h > 64) return X265AMD_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const bool hbd = depth == 10 || depth == 12;
    if (!hbd && depth != 8) return X265AMD_EINVAL;
    if (op == X265AMD_P2S)
        return hbd ? pick_unit<uint16_t, uint16_t, int16_t, X265AMD_P2S, 4>(w, h, n, depth, src, src_stride, src_off, dst, dst_stride, dst_off, nullptr, 0, st)
                   : pick_unit<uint8_t, uint8_t, int16_t, X265AMD_P2S, 4>(w, h, n, depth, src, src_stride, src_off, dst, dst_stride, dst_off, nullptr, 0, st);
    if (taps == 8)
        return hbd ? dispatch_interp<uint16_t, 8>(op, w, h, n, depth, src, src_stride, src_off, dst, dst_stride, dst_off, coeff, is_row_ext, st)
                   : dispatch_interp<uint8_t, 8>(op, w, h, n, depth, src, src_stride, src_off, dst, dst_stride, dst_off, coeff, is_row_ext, st);
    if (taps == 4)
        return hbd ? dispatch_interp<uint16_t, 4>(op, w, h, n, depth, src, src_stride, src_off, dst, dst_stride, dst_off, coeff, is_row_ext, st)
                   : dispatch_interp<uint8_t, 4>(op, w, h, n, depth, src, src_stride, src_off, dst, dst_stride, dst_off, coeff, is_row_ext, st);
    return X265AMD_EINVAL;
}
