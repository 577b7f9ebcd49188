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
#include <algorithm>
#include <stdlib.h>

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

// ---------------------------------------------------------------- 8-bit dot paths
// 8-bit sources run the taps on v_dot4_i32_i8: pixels are biased to signed
// bytes (p ^ 0x80 = p - 128), so  Σ c·p = sdot4(c, p - 128) + 128·Σc  with
// Σc = 64 for every luma and chroma filter phase (ipfilter.cpp tables,
// constants.cpp g_lumaFilter / g_chromaFilter) — the exact integer sum, four
// taps per instruction instead of four unpacks and four multiply-adds.

template <int TAPS>
__device__ __forceinline__ void pack_taps(int idx, int (&cp)[TAPS / 4])
{
    int c[TAPS];
    get_taps<TAPS>(idx, c);
#pragma unroll
    for (int k = 0; k < TAPS / 4; k++)
        cp[k] = (int)((uint32_t)(c[4 * k] & 0xff) | ((uint32_t)(c[4 * k + 1] & 0xff) << 8)
                      | ((uint32_t)(c[4 * k + 2] & 0xff) << 16) | ((uint32_t)(c[4 * k + 3] & 0xff) << 24));
}

// gfx950 v_sat_pk_u8_i16: the two int16 halves of x clamped to [0, 255], as the low two bytes
__device__ __forceinline__ uint32_t sat_pk_u8_i16(uint32_t x)
{
    uint32_t r;
    asm("v_sat_pk_u8_i16 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

__device__ __forceinline__ uint32_t alignb(uint32_t hi, uint32_t lo, int s)
{
    return s ? __builtin_amdgcn_alignbyte(hi, lo, s) : lo;
}

// X265AMD_NT_INTERP=1 (A/B builds): the 8-bit filter windows with non-temporal loads — slower (hpp 64x64
// 0.52 -> 0.39, census replay -4 to -7 %, profiles/r05/interp_nt_ab.txt): neighbouring lanes' windows share
// lines, which non-temporal loads re-fetch
#ifndef X265AMD_NT_INTERP
#define X265AMD_NT_INTERP 0
#endif
constexpr bool kNtInterp = X265AMD_NT_INTERP != 0;

// bytes [0, NB) at p as biased dwords W[] (bytes past NB unspecified); two
// overlapping loads that stay inside the NB-byte read window
template <int NB>
__device__ __forceinline__ void load_win_dw(const uint8_t* p, uint32_t (&W)[(NB + 3) / 4])
{
    constexpr int ND = (NB + 3) / 4;
#ifndef X265AMD_WIN_ALIGNED
#define X265AMD_WIN_ALIGNED 0
#endif
    if constexpr (X265AMD_WIN_ALIGNED && NB >= 13 && NB <= 16)
    {
        // dword-aligned loads: the four dwords from p rounded down (each holds a window byte, as
        // NB >= 13) and the fifth only when the window reaches into it (otherwise dword 3 again), then
        // a per-lane byte shift
        const uintptr_t a = (uintptr_t)p;
        const int sh = (int)(a & 3);
        const uint32_t* q = (const uint32_t*)(a - sh);
        const uint4 d = *(const uint4*)q;
        const uint32_t e = q[(sh + NB - 1) >> 2];
        const uint32_t D[5] = { d.x, d.y, d.z, d.w, e };
#pragma unroll
        for (int k = 0; k < ND; k++) W[k] = __builtin_amdgcn_alignbyte(D[k + 1], D[k], sh);
    }
    else if constexpr (NB > 8)
    {
        static_assert(NB <= 16, "window too large");
        const uint2 h = ldx<uint2, kNtInterp>(p), t = ldx<uint2, kNtInterp>(p + NB - 8);
        constexpr int o = NB - 8;
        W[0] = h.x;
        W[1] = h.y;
#pragma unroll
        for (int k = 2; k < ND; k++)
        {
            const int s = 4 * k - o;
            W[k] = s < 4 ? alignb(t.y, t.x, s) : __builtin_amdgcn_alignbyte(0u, t.y, s - 4);
        }
    }
    else
    {
        static_assert(NB > 4, "window too small");
        const uint32_t h = ldx<uint32_t, kNtInterp>(p), t = ldx<uint32_t, kNtInterp>(p + NB - 4);
        W[0] = h;
        W[1] = alignb(0u, t, 8 - NB);
    }
#pragma unroll
    for (int k = 0; k < ND; k++) W[k] ^= 0x80808080u;
}

template <int TAPS, int UW>
__device__ __forceinline__ void hfilter_dot(const uint8_t* src, const int (&cp)[TAPS / 4], int (&sum)[UW],
                                            int init = 128 * 64);

// the horizontal 8-bit filter split into its window load and its arithmetic, so a kernel can issue
// the loads of several rows before the first row's sums (and before any store: a store between
// two loads of possibly aliasing pointers pins the order, and gfx9's vmcnt counts both)
template <int TAPS, int UW>
struct HWin
{
    static constexpr int NB = UW + TAPS - 1, ND = (NB + 3) / 4;
    uint32_t W[ND];
    __device__ __forceinline__ void load(const uint8_t* src) { load_win_dw<NB>(src - (TAPS / 2 - 1), W); }
    // init: the bias correction 128 * sum(c) = 128 * 64 of the signed-byte pixels, plus any offset the
    // caller folds in
    __device__ __forceinline__ void sums(const int (&cp)[TAPS / 4], int (&sum)[UW], int init = 128 * 64) const
    {
#pragma unroll
        for (int x = 0; x < UW; x++)
        {
            int s = 0;
#pragma unroll
            for (int k = 0; k < TAPS / 4; k++)
            {
                const int b = x + 4 * k;
                const int v = (int)alignb(W[(b >> 2) + ((b & 3) ? 1 : 0)], W[b >> 2], b & 3);
                s = __builtin_amdgcn_sdot4(v, cp[k], k ? s : init, false);
            }
            sum[x] = s;
        }
    }
};

template <int TAPS, int UW>
__device__ __forceinline__ void hfilter_dot(const uint8_t* src, const int (&cp)[TAPS / 4], int (&sum)[UW], int init)
{
    HWin<TAPS, UW> w;
    w.load(src);
    w.sums(cp, sum, init);
}

typedef short s16x2 __attribute__((ext_vector_type(2)));

// pp output of 8-bit sums: (s + 32) >> 6, (int16) truncation (a no-op: |s| <
// 2^15 - 32 for every 8-bit filter phase), clamp to [0, 255]; done on packed
// 16-bit pairs (v_pk_*), clamped and packed by v_sat_pk_u8_i16, 4 pixels per dword.
// ROUNDED: the sums already carry the +32 (folded into the dot chain's start)
template <int UW, bool ROUNDED = false>
__device__ __forceinline__ void store_pp8(uint8_t* p, const int (&s)[UW])
{
    uint32_t out[UW / 4];
#pragma unroll
    for (int q = 0; q < UW / 4; q++)
    {
        s16x2 lo = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm((uint32_t)s[4 * q + 1], (uint32_t)s[4 * q], 0x05040100u));
        s16x2 hi = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm((uint32_t)s[4 * q + 3], (uint32_t)s[4 * q + 2], 0x05040100u));
        if constexpr (!ROUNDED)
        {
            lo = lo + (s16x2)32;
            hi = hi + (s16x2)32;
        }
        lo = lo >> (s16x2)6;
        hi = hi >> (s16x2)6;
        out[q] = __builtin_amdgcn_perm(sat_pk_u8_i16(__builtin_bit_cast(uint32_t, hi)),
                                       sat_pk_u8_i16(__builtin_bit_cast(uint32_t, lo)), 0x05040100u);
    }
    if constexpr (UW == 8) stu<uint2>(p, make_uint2(out[0], out[1]));
    else stu<uint32_t>(p, out[0]);
}

// 4x4 byte transpose: r[i] = 4 pixels of row i  ->  c[j] = column j, rows 0..3
__device__ __forceinline__ void transpose4(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t (&c)[4])
{
    const uint32_t a = __builtin_amdgcn_perm(r1, r0, 0x05010400u);   // r0b0 r1b0 r0b1 r1b1
    const uint32_t b = __builtin_amdgcn_perm(r3, r2, 0x05010400u);   // r2b0 r3b0 r2b1 r3b1
    const uint32_t e = __builtin_amdgcn_perm(r1, r0, 0x07030602u);   // r0b2 r1b2 r0b3 r1b3
    const uint32_t f = __builtin_amdgcn_perm(r3, r2, 0x07030602u);   // r2b2 r3b2 r2b3 r3b3
    c[0] = __builtin_amdgcn_perm(b, a, 0x05040100u);
    c[1] = __builtin_amdgcn_perm(b, a, 0x07060302u);
    c[2] = __builtin_amdgcn_perm(f, e, 0x05040100u);
    c[3] = __builtin_amdgcn_perm(f, e, 0x07060302u);
}

// vertical taps of a UW x UH unit: the UH+TAPS-1 source rows are loaded once,
// transposed to per-column dwords of 4 consecutive rows, and every output is
// TAPS/4 byte-aligned dwords of its column dotted with the packed taps
template <int TAPS, int UW, int UH>
__device__ __forceinline__ void vfilter_dot(const uint8_t* col, intptr_t ss, const int (&cp)[TAPS / 4],
                                            int (&acc)[UH][UW])
{
    constexpr int R = UH + TAPS - 1, RG = (R + 3) / 4, CG = UW / 4;
    uint32_t rows[RG * 4][CG];
#pragma unroll
    for (int t = 0; t < RG * 4; t++)
    {
        if (t < R)
        {
            if constexpr (UW == 8)
            {
                const uint2 v = ldx<uint2, kNtInterp>(col + t * ss);
                rows[t][0] = v.x ^ 0x80808080u;
                rows[t][1] = v.y ^ 0x80808080u;
            }
            else
                rows[t][0] = ldx<uint32_t, kNtInterp>(col + t * ss) ^ 0x80808080u;
        }
        else
        {
#pragma unroll
            for (int q = 0; q < CG; q++) rows[t][q] = 0;
        }
    }
    uint32_t T[UW][RG];
#pragma unroll
    for (int q = 0; q < CG; q++)
#pragma unroll
        for (int g = 0; g < RG; g++)
        {
            uint32_t c[4];
            transpose4(rows[4 * g][q], rows[4 * g + 1][q], rows[4 * g + 2][q], rows[4 * g + 3][q], c);
#pragma unroll
            for (int j = 0; j < 4; j++) T[4 * q + j][g] = c[j];
        }
#pragma unroll
    for (int r = 0; r < UH; r++)
#pragma unroll
        for (int x = 0; x < UW; x++)
        {
            int s = 128 * 64;
#pragma unroll
            for (int k = 0; k < TAPS / 4; k++)
            {
                const int b = r + 4 * k;
                s = __builtin_amdgcn_sdot4((int)alignb(T[x][(b >> 2) + ((b & 3) ? 1 : 0)], T[x][b >> 2], b & 3),
                                           cp[k], s, false);
            }
            acc[r][x] = s;
        }
}

// 8-bit vertical taps on packed 16-bit pairs (v_pk_mad_u16): every 8-bit
// filter sum fits int16 (|Σ c·p| <= 255 * 88 < 2^15), so two adjacent columns
// share each multiply-add, rows need no byte transpose, and the wrapped 16-bit
// result equals the exact sum.  acc[r][p] holds columns (2p, 2p+1) of row r.
template <int TAPS, int UW, int UH>
__device__ __forceinline__ void vfilter_pk(const uint8_t* col, intptr_t ss, const s16x2 (&cpk)[TAPS],
                                           s16x2 (&acc)[UH][UW / 2])
{
#pragma unroll
    for (int r = 0; r < UH; r++)
#pragma unroll
        for (int p = 0; p < UW / 2; p++) acc[r][p] = (s16x2)0;
#pragma unroll
    for (int t = 0; t < UH + TAPS - 1; t++)
    {
        uint32_t w[UW / 4];
        if constexpr (UW == 8)
        {
            const uint2 v = ldx<uint2, kNtInterp>(col + t * ss);
            w[0] = v.x;
            w[1] = v.y;
        }
        else
            w[0] = ldx<uint32_t, kNtInterp>(col + t * ss);
        s16x2 pr[UW / 2];
#pragma unroll
        for (int q = 0; q < UW / 4; q++)
        {
            pr[2 * q] = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(w[q], w[q], 0x0c010c00u));
            pr[2 * q + 1] = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(w[q], w[q], 0x0c030c02u));
        }
#pragma unroll
        for (int r = 0; r < UH; r++)
        {
            const int k = t - r;
            if (k >= 0 && k < TAPS)
            {
#pragma unroll
                for (int p = 0; p < UW / 2; p++) acc[r][p] = pr[p] * cpk[k] + acc[r][p];
            }
        }
    }
}

// Grouped launches (common.h): a = src, d = dst, b = per-job coeffIdx
// (uint8), param = is_row_ext.
//
// STG (8-bit hpp / vpp into compact destinations, dst stride = w, power-of-two
// w and h, one unit per lane): the wavefront's outputs are staged in
// wave-private LDS in destination order and written back as 16-byte chunks, so
// a store instruction covers whole 64-byte segments of four to sixteen jobs
// instead of one 4-8-byte row piece per job.
template <typename P, typename S, typename D, int OP, int TAPS, int UW, int UH, bool STG = false>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_interp(const BatchGroup g)
{
    const uint32_t gb = xcd_block();
    const SubBatch& sub = group_sub(g, gb);
    const int w = sub.w, h = sub.h, n = sub.n, lg = sub.lg;
    const intptr_t ss = sub.sa, ds = sub.ds;
    const int G = 1 << lg;
    const int64_t wjob0 = (int64_t)(gb - sub.block0) * (X265AMD_BLOCK >> lg) + ((threadIdx.x & ~63u) >> lg);
    int64_t job = (int64_t)(gb - sub.block0) * (X265AMD_BLOCK >> lg) + (threadIdx.x >> lg);
    const int lane = threadIdx.x & (G - 1);
    if constexpr (STG)
    {
        // the whole wavefront stays for the write-back; lanes past the batch compute a copy of
        // the last job into LDS that is never written out
        static_assert(OP != X265AMD_HVPP && UW * UH * sizeof(D) >= 16 && UW * UH * sizeof(D) <= 128, "staging");
        if (wjob0 >= n) return;
        if (job >= n) job = n - 1;
    }
    else if (job >= n)
        return;
    constexpr int STG_WAVE = STG ? 64 * UW * UH * (int)sizeof(D) : 16;          // staged bytes per wavefront
    __shared__ uint4 stg_lds[STG ? X265AMD_BLOCK / 64 * STG_WAVE / 16 : 1];
    D* const stg = (D*)((uint8_t*)stg_lds + (threadIdx.x >> 6) * STG_WAVE) + ((threadIdx.x & 63) >> lg) * w * h;

    const IfConst K(g.depth);
    const S* ps = (const S*)sub.a + sub.aoff[job];
    D* pd = (D*)sub.d + sub.doff[job];
    const uint8_t* coeff = (const uint8_t*)sub.b;
    const int cidx = coeff ? coeff[job] : 0;

    int rows = h;
    if constexpr (OP == X265AMD_HPS)
    {
        if (sub.param)
        {
            ps -= (TAPS / 2 - 1) * ss;
            rows += TAPS - 1;
        }
    }
    const int ux = w / UW, units = ux * (rows / UH);

    // 8-bit sources with 4/8-wide units take the v_dot4 paths
    constexpr bool DOT = sizeof(S) == 1 && UW >= 4 && OP != X265AMD_P2S;
    int c[TAPS];
    int cp[TAPS / 4];
    get_taps<TAPS>(cidx, c);
    if constexpr (DOT) pack_taps<TAPS>(cidx, cp);

    for (int u = lane; u < units; u += G)
    {
        const int x = (u % ux) * UW, y0 = (u / ux) * UH;

        if constexpr (OP == X265AMD_HPP || OP == X265AMD_HPS)
        {
            // 8 bit: every row window of the unit loaded before the first sum / store
            HWin<TAPS, DOT ? UW : 4> win[DOT ? UH : 1];
            if constexpr (DOT)
            {
#pragma unroll
                for (int r = 0; r < UH; r++) win[r].load((const uint8_t*)ps + (y0 + r) * ss + x);
            }
#pragma unroll
            for (int r = 0; r < UH; r++)
            {
                int sum[UW], o[UW];
                if constexpr (DOT && OP == X265AMD_HPP)
                {
                    // the pp rounding 32 folded into the chain's start
                    win[r].sums(cp, sum, 128 * 64 + 32);
                    store_pp8<UW, true>((uint8_t*)(STG ? stg + (y0 + r) * w + x : pd + (y0 + r) * ds + x), sum);
                    continue;
                }
                if constexpr (DOT) win[r].sums(cp, sum);
                else hfilter<P, TAPS, UW>((const P*)ps + (y0 + r) * ss + x, c, sum);
#pragma unroll
                for (int i = 0; i < UW; i++)
                    o[i] = OP == X265AMD_HPP ? clampp((sum[i] + 32) >> 6, K.maxv)
                                             : (int)(int16_t)((sum[i] + K.ps_off) >> K.ps_shift);
                store_row<D, UW>(STG ? stg + (y0 + r) * w + x : pd + (y0 + r) * ds + x, o);
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
                store_row<D, UW>(STG ? stg + (y0 + r) * w + x : pd + (y0 + r) * ds + x, v);
            }
        }
        else  // vertical: VPP, VPS, VSP, VSS
        {
            const S* col = ps + (y0 - (TAPS / 2 - 1)) * ss + x;
            if constexpr (DOT && (OP == X265AMD_VPP || OP == X265AMD_VPS))
            {
                s16x2 cpk[TAPS], pacc[UH][UW / 2];
#pragma unroll
                for (int k = 0; k < TAPS; k++) cpk[k] = (s16x2)(short)c[k];
                vfilter_pk<TAPS, UW, UH>((const uint8_t*)col, ss, cpk, pacc);
#pragma unroll
                for (int r = 0; r < UH; r++)
                {
                    uint32_t o[UW / 2];
#pragma unroll
                    for (int p = 0; p < UW / 2; p++)
                    {
                        s16x2 v = pacc[r][p];
                        if constexpr (OP == X265AMD_VPP)
                        {
                            v = (v + (s16x2)32) >> (s16x2)6;
                            o[p] = sat_pk_u8_i16(__builtin_bit_cast(uint32_t, v));     // clamped, 2 bytes
                        }
                        else
                            o[p] = __builtin_bit_cast(uint32_t, v - (s16x2)8192);     // ps at 8-bit: shift 0, offset -IF_INTERNAL_OFFS
                    }
                    D* out = STG ? stg + (y0 + r) * w + x : pd + (y0 + r) * ds + x;
                    if constexpr (OP == X265AMD_VPP)
                    {
                        // two pairs -> four pixels per dword
                        if constexpr (UW == 8)
                            stu<uint2>(out, make_uint2(__builtin_amdgcn_perm(o[1], o[0], 0x05040100u),
                                                       __builtin_amdgcn_perm(o[3], o[2], 0x05040100u)));
                        else
                            stu<uint32_t>(out, __builtin_amdgcn_perm(o[1], o[0], 0x05040100u));
                    }
                    else
                    {
                        if constexpr (UW == 8) stu<uint4>(out, make_uint4(o[0], o[1], o[2], o[3]));
                        else stu<uint2>(out, make_uint2(o[0], o[1]));
                    }
                }
                continue;
            }
            int acc[UH][UW];
            if constexpr (DOT)
                vfilter_dot<TAPS, UW, UH>((const uint8_t*)col, ss, cp, acc);
            else
            {
#pragma unroll
                for (int r = 0; r < UH; r++)
#pragma unroll
                    for (int i = 0; i < UW; i++) acc[r][i] = 0;
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
            }
#pragma unroll
            for (int r = 0; r < UH; r++)
            {
                if constexpr (DOT && OP == X265AMD_VPP)
                {
                    store_pp8<UW>((uint8_t*)(STG ? stg + (y0 + r) * w + x : pd + (y0 + r) * ds + x), acc[r]);
                    continue;
                }
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
                store_row<D, UW>(STG ? stg + (y0 + r) * w + x : pd + (y0 + r) * ds + x, o);
            }
        }
    }
    if constexpr (STG)
        stage_writeback<STG_WAVE>((const uint8_t*)stg_lds + (threadIdx.x >> 6) * STG_WAVE, pd, lg,
                                  w * h * (int)sizeof(D), wjob0, n);
}

// hv_pp in two on-chip passes: the horizontal int16 intermediate of the
// (h+7) x w block (interp_horiz_ps_c with row extension) goes to LDS once,
// then the vertical sp filter reads it back (filterVertical_sp_c).  Jobs per
// block = 256 / G, LDS = jobs * (h+7) * w int16 (the launch reserves the
// largest sub-batch's need).
template <typename P, int UW, int UH>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_hvpp(const BatchGroup g)
{
    extern __shared__ int16_t hv_lds[];
    const uint32_t gb = xcd_block();
    const SubBatch& sub = group_sub(g, gb);
    const int w = sub.w, h = sub.h, n = sub.n, lg = sub.lg;
    const intptr_t ss = sub.sa, ds = sub.ds;
    const int G = 1 << lg;
    const int slot = threadIdx.x >> lg, lane = threadIdx.x & (G - 1);
    const int64_t job0 = (int64_t)(gb - sub.block0) * (X265AMD_BLOCK >> lg) + slot;
    const bool live = job0 < n;
    const int64_t job = live ? job0 : 0;
    const IfConst K(g.depth);
    int16_t* L = hv_lds + (size_t)slot * (h + 7) * w;
    const int cidx = ((const uint8_t*)sub.b)[job];
    constexpr bool DOT = sizeof(P) == 1;
    int cx[8], cy[8], cp[2];
    if constexpr (DOT) pack_taps<8>(cidx & 15, cp);
    else get_taps<8>(cidx & 15, cx);
    get_taps<8>(cidx >> 4, cy);
    const int ux = w / UW;

    if (live)
    {
        const P* ps = (const P*)sub.a + sub.aoff[job] - 3 * ss;
        const int hunits = ux * (h + 7);
        for (int u = lane; u < hunits; u += G)
        {
            const int x = (u % ux) * UW, t = u / ux;
            int sum[UW], o[UW];
            if constexpr (DOT) hfilter_dot<8, UW>((const uint8_t*)ps + t * ss + x, cp, sum);
            else hfilter<P, 8, UW>(ps + t * ss + x, cx, sum);
#pragma unroll
            for (int i = 0; i < UW; i++) o[i] = (int)(int16_t)((sum[i] + K.ps_off) >> K.ps_shift);
            store_row<int16_t, UW>(L + t * w + x, o);
        }
    }
    __syncthreads();
    if (!live) return;
    P* pd = (P*)sub.d + sub.doff[job];
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


// hv_pp without the LDS round trip (ipfilter.cpp:322-372): hps with row extension
// then filterVertical_sp, streamed through registers.  A lane owns an SW-column strip
// of one job and walks its h + 7 source rows top to bottom: the row's horizontal sums
// (v_dot4 at 8 bit), the int16 intermediate I[r] = (int16)((S + ps_off) >> ps_shift)
// exactly as hps writes it, the vertical pairs P[r - 1] = (I[r - 1], I[r]) packed in
// one dword, and every output row y = r - 7 as four v_dot2_i32_i16 per column against
// (c_v[2k], c_v[2k+1]) over P[y], P[y+2], P[y+4], P[y+6] — each pair is formed once and
// serves four output rows — then the sp rounding, int16 truncation and clamp.  The last
// eight pairs live in a ring indexed by r & 7, compile-time inside a body unrolled over
// eight rows.
//
// STG (8 bit, compact destinations, power-of-two w and h <= 16): the output
// rows go to wave-private LDS and leave through stage_writeback.
//
// PF (8 bit): the source windows of each 8-row body are loaded before its first sum — PF = 1 —
// or one body ahead, while the current body is computed from registers — PF = 2 — so a lane has
// 8 row loads in flight instead of one (rows past the block clamp to its last row; their
// results are never used).
template <typename P, int SW, bool STG = false, int PF = 0, int WPE = 1>
__global__ __launch_bounds__(X265AMD_BLOCK) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_hvpp_stream(const BatchGroup g)
{
    const uint32_t gb = xcd_block();
    const SubBatch& sub = group_sub(g, gb);
    const int w = sub.w, h = sub.h, n = sub.n, lg = sub.lg;
    const intptr_t ss = sub.sa, ds = sub.ds;
    const int G = 1 << lg;
    const int64_t wjob0 = (int64_t)(gb - sub.block0) * (X265AMD_BLOCK >> lg) + ((threadIdx.x & ~63u) >> lg);
    int64_t job = (int64_t)(gb - sub.block0) * (X265AMD_BLOCK >> lg) + (threadIdx.x >> lg);
    const int lane = threadIdx.x & (G - 1);
    constexpr int STG_WAVE = STG ? 64 * SW * 16 : 16;
    __shared__ uint4 stg_lds[STG ? X265AMD_BLOCK / 64 * STG_WAVE / 16 : 1];
    if constexpr (STG)
    {
        // power-of-two w: every lane holds a strip; lanes past the batch compute a copy of the
        // last job that is never written out
        static_assert(sizeof(P) == 1, "staging");
        if (wjob0 >= n) return;
        if (job >= n) job = n - 1;
    }
    else if (job >= n || SW * lane >= w)
        return;
    uint8_t* const stg = (uint8_t*)stg_lds + (threadIdx.x >> 6) * STG_WAVE + ((threadIdx.x & 63) >> lg) * w * h;
    const IfConst K(g.depth);
    const int cidx = ((const uint8_t*)sub.b)[job];
    constexpr bool DOT = sizeof(P) == 1;
    static_assert(!PF || DOT, "row prefetch: 8-bit path");
    int cp[2], cx[8], cy[8];
    if constexpr (DOT) pack_taps<8>(cidx & 15, cp);
    else get_taps<8>(cidx & 15, cx);
    get_taps<8>(cidx >> 4, cy);
    // 8 bit: the vertical taps scaled by 16, so the sp shift of 12 becomes 16 and each output is the
    // high half of its sum (see below)
    s16x2 cv[4];
#pragma unroll
    for (int k = 0; k < 4; k++)
        cv[k] = DOT ? s16x2{ (short)(16 * cy[2 * k]), (short)(16 * cy[2 * k + 1]) }
                    : s16x2{ (short)cy[2 * k], (short)cy[2 * k + 1] };
    const int x0 = SW * lane;
    const P* ps = (const P*)sub.a + sub.aoff[job] - 3 * ss + x0;
    P* pd = (P*)sub.d + sub.doff[job] + (STG ? 0 : x0);
    const int R = h + 7;
    // 8 bit: I = S - 8192 exactly (shift 0, |S| <= 88 * 255), and the sp offset adds 8192 * 64
    // back, so the raw sums S are paired and the output is (t + 2048) >> 12; the 2048 is carried as
    // 32 on every S (the vertical taps sum to 64), so the vertical sums start at 0 — an inline
    // constant of the dot instruction, no accumulator move — and the horizontal sums start at
    // 128 * 64 + 32, kept in an SGPR for the same reason
    int hinit = 128 * 64 + 32;
    if constexpr (DOT) asm volatile("" : "+s"(hinit));
    auto inter = [&](const P* row, int (&I)[SW]) {
        if constexpr (DOT) hfilter_dot<8, SW>((const uint8_t*)row, cp, I, hinit);
        else
        {
            int S[SW];
            hfilter<P, 8, SW>(row, cx, S);
#pragma unroll
            for (int x = 0; x < SW; x++) I[x] = (int)(int16_t)((S[x] + K.ps_off) >> K.ps_shift);
        }
    };
    using Win = HWin<8, SW>;
    auto load_body = [&](int r0, Win (&wb)[8]) {
#pragma unroll
        for (int i = 0; i < 8; i++)
        {
            const int r = r0 + i < R ? r0 + i : R - 1;
            wb[i].load((const uint8_t*)(ps + (intptr_t)r * ss));
        }
    };
    uint32_t Pr[8][SW];                  // ring of vertical pairs: Pr[r & 7][x] = (I[r][x], I[r + 1][x])
    Win wa[PF == 3 ? 4 : PF ? 8 : 1], wn[PF == 2 ? 8 : 1];
    if constexpr (PF == 3)
    {
        // rolling window: row r lives in wa[(r - 1) & 3], loaded four rows ahead of its use
#pragma unroll
        for (int i = 0; i < 4; i++) wa[i].load((const uint8_t*)(ps + (intptr_t)(1 + i < R ? 1 + i : R - 1) * ss));
    }
    else if constexpr (PF) load_body(1, wa);
    {
        // row 0's intermediate as the high half of ring slot 7 (the pair before row 1's)
        int I0[SW];
        inter(ps, I0);
#pragma unroll
        for (int x = 0; x < SW; x++) Pr[7][x] = (uint32_t)I0[x] << 16;
    }
    for (int r0 = 1; r0 < R; r0 += 8)
    {
        if constexpr (PF == 1)
        {
            if (r0 > 1) load_body(r0, wa);
        }
        else if constexpr (PF == 2)
        {
            if (r0 + 8 < R) load_body(r0 + 8, wn);
        }
#pragma unroll
        for (int i = 0; i < 8; i++)
        {
            const int r = r0 + i;                        // row whose intermediate is formed now
            if (r >= R) break;
            int I[SW];
            if constexpr (PF == 3)
            {
                wa[i & 3].sums(cp, I, hinit);
                if (r + 4 < R) wa[i & 3].load((const uint8_t*)(ps + (intptr_t)(r + 4) * ss));
            }
            else if constexpr (PF) wa[i].sums(cp, I, hinit);
            else inter(ps + (intptr_t)r * ss, I);
            // P[r - 1] goes to ring slot (r - 1) & 7 = i (r0 = 1 mod 8): compile-time; I[r - 1] is the
            // high half of the previous slot
#pragma unroll
            for (int x = 0; x < SW; x++) Pr[i][x] = __builtin_amdgcn_perm((uint32_t)I[x], Pr[(i + 7) & 7][x], 0x05040302u);
            const int y = r - 7;                         // output row ready once P[y + 6] exists
            if (y >= 0)
            {
                int t[SW];
#pragma unroll
                for (int x = 0; x < SW; x++)
                {
                    // 8 bit: the sp rounding offset rides on the pairs (hinit), the sums start at 0
                    t[x] = __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, Pr[(i + 2) & 7][x]), cv[0], 0, false);
#pragma unroll
                    for (int k = 1; k < 4; k++)
                        t[x] = __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, Pr[(i + 2 + 2 * k) & 7][x]), cv[k], t[x], false);
                }
                if constexpr (DOT)
                {
                    // (16 t) >> 16 = t >> 12 is the high half of each sum (|t| < 2^21, so it fits int16): two
                    // outputs' high halves with one v_perm, clamped to [0, 255] and packed by one
                    // v_sat_pk_u8_i16, two such pairs per dword
                    uint32_t pk[SW / 4];
#pragma unroll
                    for (int q = 0; q < SW / 4; q++)
                    {
                        const uint32_t h0 = __builtin_amdgcn_perm((uint32_t)t[4 * q + 1], (uint32_t)t[4 * q], 0x07060302u);
                        const uint32_t h1 = __builtin_amdgcn_perm((uint32_t)t[4 * q + 3], (uint32_t)t[4 * q + 2], 0x07060302u);
                        pk[q] = __builtin_amdgcn_perm(sat_pk_u8_i16(h1), sat_pk_u8_i16(h0), 0x05040100u);
                    }
                    uint8_t* dst = STG ? stg + y * w + x0 : (uint8_t*)(pd + (intptr_t)y * ds);
                    if constexpr (SW == 8) stu<uint2>(dst, make_uint2(pk[0], pk[1]));
                    else stu<uint32_t>(dst, pk[0]);
                }
                else
                {
                    int o[SW];
#pragma unroll
                    for (int x = 0; x < SW; x++) o[x] = clampp((t[x] + K.sp_off) >> K.sp_shift, K.maxv);
                    if constexpr (STG) store_row<P, SW>((P*)(stg + y * w + x0), o);
                    else store_row<P, SW>(pd + (intptr_t)y * ds, o);
                }
            }
        }
        if constexpr (PF == 2)
        {
#pragma unroll
            for (int i = 0; i < 8; i++) wa[i] = wn[i];
        }
    }
    if constexpr (STG) stage_writeback<STG_WAVE>((const uint8_t*)stg_lds + (threadIdx.x >> 6) * STG_WAVE, pd, lg, w * h, wjob0, n);
}

// row-prefetch variant of the 8-bit streaming hv_pp (X265AMD_HVPP_PF = 0 / 1 / 2 / 3; default below)
static int hvpp_pf()
{
    static int v = -1;
    if (v < 0)
    {
        const char* e = getenv("X265AMD_HVPP_PF");
        v = e ? atoi(e) : 1;
        if (v < 0 || v > 3) v = 1;
    }
    return v;
}

// -------------------------------------------------------------- dispatch

// unit-height override for tuning runs (X265AMD_UH_<op>=1|2|4|8|16; 0 = built-in choice)
static int uh_override(int op)
{
    static int v[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
    if (op < 0 || op > 7) return 0;
    if (v[op] < 0)
    {
        static const char* names[8] = {"X265AMD_UH_HPP", "X265AMD_UH_HPS", "X265AMD_UH_VPP", "X265AMD_UH_VPS",
                                       "X265AMD_UH_VSP", "X265AMD_UH_VSS", "X265AMD_UH_HVPP", "X265AMD_UH_P2S"};
        const char* e = getenv(names[op]);
        v[op] = e ? atoi(e) : 0;
    }
    return v[op];
}

// kernel class of a batch: unit width x unit height, packed as uw * 32 + uh
template <int OP, int TAPS>
static int interp_class(int w, int h, int rowext, bool pk8, bool u8 = false)
{
    if (w < 2 || h < 2 || w > 64 || h > 64) return -X265AMD_EINVAL;
    const int ov = uh_override(OP);
    if constexpr (OP == X265AMD_HVPP)
    {
        if (w % 4) return -X265AMD_EINVAL;
        // 2-row units up to 16 rows: more lanes per job for the latency-bound small blocks (measured,
        // profiles/r02/interp_uh_sweep.txt: 8x8 0.25 -> 0.35, 16x16 0.25 -> 0.31 of HBM peak)
        const int uh = (ov == 1 || ov == 2 || ov == 4) && h % ov == 0 ? ov
                       : (h <= 16 && h % 2 == 0 ? 2 : (h % 4 == 0 ? 4 : 1));
        return (w % 8 == 0 ? 8 : 4) * 32 + uh;
    }
    const int rows = (OP == X265AMD_HPS && rowext) ? h + TAPS - 1 : h;
    // vertical filters take 16-row units on blocks of 16+ rows: UH + taps - 1
    // source rows per unit, so the re-read overhead drops from 11/4 to 23/16
    // rows per output row (measured, 8-bit vpp: 64x64 40% -> 55% of HBM peak,
    // 16x16 36.5% -> 37.7%; 8-row units were worse on 8x8 and 16x16)
    // (the packed 8-bit vpp / vps path only: its accumulators are half-size)
    int uh = (pk8 && rows % 16 == 0 && w % 4 == 0) ? 16 : rows % 4 ? 1 : 4;
    // 8-bit luma, measured on the roofline shapes (profiles/r05/ai/interp_uh_sweep.txt): 64-wide hpp on
    // single-row units (0.52 -> 0.58 of HBM peak at 64x64), 8x8 vpp on one 8-row unit (0.59 -> 0.62)
    if constexpr (OP == X265AMD_HPP && TAPS == 8)
        if (u8 && w == 64) uh = 1;
    if constexpr (OP == X265AMD_VPP && TAPS == 8)
        if (u8 && w == 8 && h == 8) uh = 8;
    if (ov && rows % ov == 0 && (ov != 16 || (pk8 && w % 4 == 0)) && (ov == 1 || ov == 2 || ov == 4 || ov == 8 || ov == 16))
        uh = ov;
    if (w % 8 == 0) return 8 * 32 + uh;
    if (w % 4 == 0) return 4 * 32 + uh;
    // 2-wide units: the chroma filters and the vertical / p2s luma paths
    if (w % 2 == 0 && (TAPS == 4 || (OP != X265AMD_HPP && OP != X265AMD_HPS))) return 2 * 32 + uh;
    return -X265AMD_EINVAL;
}

// HV_PP: keep the workgroup's intermediate within 64 KiB of LDS
static int hvpp_lg(int w, int h, int uw, int uh)
{
    int lg = lanes_log2((w / uw) * (h / uh));
    while (lg < 6 && (size_t)(X265AMD_BLOCK >> lg) * (h + 7) * w * sizeof(int16_t) > 65536) lg++;
    return lg;
}

// classes of the streaming hv_pp (k_hvpp_stream): 8- / 4-wide strips, no LDS
constexpr int kHvppStream = 8 * 32 + 31, kHvppStream4 = 4 * 32 + 31;
// class flag: outputs staged through LDS (k_interp STG)
constexpr int kStaged = 2048;

// 8-bit 8-wide strips: row-prefetch variant x occupancy target (X265AMD_HVPP_WPE = 4: the compiler held to
// 128 VGPRs, four waves per SIMD instead of three)
static int hvpp_wpe()
{
    static int v = -1;
    if (v < 0)
    {
        const char* e = getenv("X265AMD_HVPP_WPE");
        v = e ? atoi(e) : 1;
    }
    return v;
}

template <typename P, bool STG>
static void launch_hvpp8(int pf, const BatchGroup& g, uint32_t blocks, hipStream_t st)
{
#define HV(PFV, W) hipLaunchKernelGGL((k_hvpp_stream<P, 8, STG, PFV, W>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g)
    if (hvpp_wpe() >= 4)
    {
        if (pf == 1) HV(1, 4);
        else if (pf == 3) HV(3, 4);
        else HV(0, 4);
    }
    else if (pf == 1) HV(1, 1);
    else if (pf == 2) HV(2, 1);
    else if (pf == 3) HV(3, 1);
    else HV(0, 1);
#undef HV
}

template <typename P, typename S, typename D, int OP, int TAPS>
static int launch_interp(int cls, const BatchGroup& g, uint32_t blocks, hipStream_t st)
{
    if constexpr (OP == X265AMD_HVPP)
        if (cls == kHvppStream || cls == kHvppStream4 || cls == (kHvppStream | kStaged))
        {
            const int pf = sizeof(P) == 1 ? hvpp_pf() : 0;
            if (cls == kHvppStream)
            {
                if constexpr (sizeof(P) == 1) launch_hvpp8<P, false>(pf, g, blocks, st);
                else hipLaunchKernelGGL((k_hvpp_stream<P, 8>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g);
            }
            else if (cls == (kHvppStream | kStaged))
            {
                if constexpr (sizeof(P) == 1) launch_hvpp8<P, true>(pf, g, blocks, st);
            }
            else
            {
                if constexpr (sizeof(P) == 1)
                {
                    if (pf) hipLaunchKernelGGL((k_hvpp_stream<P, 4, false, 1>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g);
                    else hipLaunchKernelGGL((k_hvpp_stream<P, 4>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g);
                }
                else hipLaunchKernelGGL((k_hvpp_stream<P, 4>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g);
            }
            return (int)hipGetLastError();
        }
    size_t lds = 0;
    if constexpr (OP == X265AMD_HVPP)
        for (int i = 0; i < g.count; i++)
            lds = std::max(lds, (size_t)(X265AMD_BLOCK >> g.s[i].lg) * (g.s[i].h + 7) * g.s[i].w * sizeof(int16_t));
    constexpr bool STGOK = OP != X265AMD_HVPP;
#define L(UW, UH) \
    if constexpr (STGOK && UW * UH * sizeof(D) >= 16 && UW * UH * sizeof(D) <= 128 && \
                  (UW >= 4 || TAPS == 4 || (OP != X265AMD_HPP && OP != X265AMD_HPS)) && (UH <= 8 || PK8)) \
        if (cls == (UW * 32 + UH | kStaged)) \
        { \
            hipLaunchKernelGGL((k_interp<P, S, D, OP, TAPS, UW, UH, true>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g); \
            return (int)hipGetLastError(); \
        } \
    if (cls == UW * 32 + UH) \
    { \
        if constexpr (OP == X265AMD_HVPP) \
        { \
            if constexpr (UW >= 4) \
                hipLaunchKernelGGL((k_hvpp<P, UW, UH>), dim3(blocks), dim3(X265AMD_BLOCK), lds, st, g); \
        } \
        else if constexpr ((UW >= 4 || TAPS == 4 || (OP != X265AMD_HPP && OP != X265AMD_HPS)) && (UH <= 8 || PK8)) \
            hipLaunchKernelGGL((k_interp<P, S, D, OP, TAPS, UW, UH>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g); \
        return (int)hipGetLastError(); \
    }
    constexpr bool PK8 = sizeof(S) == 1 && (OP == X265AMD_VPP || OP == X265AMD_VPS);
    L(8, 16) L(4, 16) L(8, 8) L(8, 4) L(8, 2) L(8, 1) L(4, 4) L(4, 2) L(4, 1) L(2, 4) L(2, 1)
#undef L
    return X265AMD_EINVAL;
}

template <typename P, typename S, typename D, int OP, int TAPS>
static int grouped_interp(int depth, int count, const x265amd_interp_batch* bt, hipStream_t st)
{
    std::vector<int> cls(count, -1);
    for (int i = 0; i < count; i++)
    {
        if (bt[i].n < 0) return X265AMD_EINVAL;
        if (bt[i].n == 0) continue;
        if (OP == X265AMD_HVPP && !bt[i].coeff) return X265AMD_EINVAL;
        cls[i] = interp_class<OP, TAPS>(bt[i].w, bt[i].h, bt[i].is_row_ext,
                                        sizeof(S) == 1 && (OP == X265AMD_VPP || OP == X265AMD_VPS), sizeof(S) == 1);
        if (cls[i] < 0) return -cls[i];
        // hv_pp streams its rows through registers on 8-wide strips at 8 bit (4-wide for 4-wide blocks
        // and for 16-bit pixels, whose int32 window doubles the registers;
        // measured, profiles/r02/hvpp_stream.txt); X265AMD_HVPP_LDS=1 selects the two-pass LDS
        // kernel, X265AMD_HVPP_SW=4 the 4-wide strips everywhere (tuning runs)
        static const bool hv_lds = getenv("X265AMD_HVPP_LDS") && atoi(getenv("X265AMD_HVPP_LDS"));
        static const int hv_sw = getenv("X265AMD_HVPP_SW") ? atoi(getenv("X265AMD_HVPP_SW")) : 8;
        if (OP == X265AMD_HVPP && !hv_lds)
        {
            if (sizeof(P) == 1 && bt[i].w % 8 == 0 && hv_sw != 4) cls[i] = kHvppStream;
            else if (bt[i].w % 4 == 0) cls[i] = kHvppStream4;
        }
        // a compact destination (stride = width, power-of-two block): stage the outputs in LDS
        // when every lane holds exactly one unit of 16..128 bytes (X265AMD_INTERP_STAGE=0 disables)
        static const bool stage = !getenv("X265AMD_INTERP_STAGE") || atoi(getenv("X265AMD_INTERP_STAGE"));
        if (stage && OP != X265AMD_HVPP && !(OP == X265AMD_HPS && bt[i].is_row_ext))
        {
            const int w = bt[i].w, h = bt[i].h, uw = cls[i] / 32, uh = cls[i] % 32;
            const int ub = uw * uh * (int)sizeof(D);
            const bool p2 = (w & (w - 1)) == 0 && (h & (h - 1)) == 0;
            if (p2 && bt[i].dst_stride == w && ub >= 16 && ub <= 128 && (w / uw) * (h / uh) <= 64)
                cls[i] |= kStaged;
        }
        if (stage && OP == X265AMD_HVPP && cls[i] == kHvppStream)
        {
            const int w = bt[i].w, h = bt[i].h;
            if ((w & (w - 1)) == 0 && (h & (h - 1)) == 0 && h <= 16 && w * h >= 16 && bt[i].dst_stride == w)
                cls[i] |= kStaged;
        }
    }
    BatchGroup proto{};
    proto.depth = depth;
    return launch_grouped(count, cls.data(), proto,
        [&](int i, SubBatch& s) {
            const x265amd_interp_batch& b = bt[i];
            s = SubBatch{};
            s.a = b.src; s.aoff = b.src_off; s.sa = b.src_stride;
            s.d = b.dst; s.doff = b.dst_off; s.ds = b.dst_stride;
            s.b = OP == X265AMD_P2S ? nullptr : b.coeff;
            s.w = b.w; s.h = b.h; s.n = b.n;
            s.param = OP == X265AMD_HPS ? b.is_row_ext : 0;
            const int uw = (cls[i] & (kStaged - 1)) / 32, uh = cls[i] % 32;
            if constexpr (OP == X265AMD_HVPP)
                s.lg = (cls[i] & ~kStaged) == kHvppStream ? lanes_log2(b.w / 8, 1)
                       : cls[i] == kHvppStream4 ? lanes_log2(b.w / 4, 1) : hvpp_lg(b.w, b.h, uw, uh);
            else
            {
                const int rows = (OP == X265AMD_HPS && s.param) ? b.h + TAPS - 1 : b.h;
                // one unit per lane (measured: 8x8 hpp 27% -> 48% of HBM peak vs two per lane)
                s.lg = lanes_log2((b.w / uw) * (rows / uh), 1);
            }
        },
        [&](int c, const BatchGroup& g, uint32_t blocks) { return launch_interp<P, S, D, OP, TAPS>(c, g, blocks, st); });
}

template <typename P, int TAPS>
static int dispatch_interp(int op, int depth, int count, const x265amd_interp_batch* bt, hipStream_t st)
{
    switch (op)
    {
    case X265AMD_HPP: return grouped_interp<P, P, P, X265AMD_HPP, TAPS>(depth, count, bt, st);
    case X265AMD_HPS: return grouped_interp<P, P, int16_t, X265AMD_HPS, TAPS>(depth, count, bt, st);
    case X265AMD_VPP: return grouped_interp<P, P, P, X265AMD_VPP, TAPS>(depth, count, bt, st);
    case X265AMD_VPS: return grouped_interp<P, P, int16_t, X265AMD_VPS, TAPS>(depth, count, bt, st);
    case X265AMD_VSP: return grouped_interp<P, int16_t, P, X265AMD_VSP, TAPS>(depth, count, bt, st);
    case X265AMD_VSS: return grouped_interp<P, int16_t, int16_t, X265AMD_VSS, TAPS>(depth, count, bt, st);
    case X265AMD_HVPP:
        if constexpr (TAPS == 8) return grouped_interp<P, P, P, X265AMD_HVPP, 8>(depth, count, bt, st);
        return X265AMD_EINVAL;
    case X265AMD_P2S:
        if constexpr (TAPS == 4) return grouped_interp<P, P, int16_t, X265AMD_P2S, 4>(depth, count, bt, st);
        return X265AMD_EINVAL;
    }
    return X265AMD_EINVAL;
}

} // namespace x265amd

using namespace x265amd;

extern "C" int x265amd_interp_grouped(int op, int taps, int depth, int count, const x265amd_interp_batch* batches,
                                      void* stream)
{
    if (count < 0 || (count > 0 && !batches)) return X265AMD_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const bool hbd = depth == 10 || depth == 12;
    if (!hbd && depth != 8) return X265AMD_EINVAL;
    if (op == X265AMD_P2S) taps = 4;        // taps ignored for p2s
    if (taps == 8)
        return hbd ? dispatch_interp<uint16_t, 8>(op, depth, count, batches, st)
                   : dispatch_interp<uint8_t, 8>(op, depth, count, batches, st);
    if (taps == 4)
        return hbd ? dispatch_interp<uint16_t, 4>(op, depth, count, batches, st)
                   : dispatch_interp<uint8_t, 4>(op, depth, count, batches, st);
    return X265AMD_EINVAL;
}

extern "C" int x265amd_interp(int op, int taps, int depth, int w, int h, int n,
                              const void* src, intptr_t src_stride, const int64_t* src_off,
                              void* dst, intptr_t dst_stride, const int64_t* dst_off,
                              const uint8_t* coeff, int is_row_ext, void* stream)
{
    if (n <= 0) return 0;
    const x265amd_interp_batch bt = {w, h, n, is_row_ext, src, src_stride, src_off, dst, dst_stride, dst_off, coeff};
    return x265amd_interp_grouped(op, taps, depth, 1, &bt, stream);
}
