// pixel.hip — batched SAD / SATD / SA8D / SSE / psy-cost / var / sad_x3/x4.
//
// Reference semantics: x265_1.9/source/common/pixel.cpp
//   sad            :39-54        sad_x3/x4 :73-118      sse :120-139
//   satd_4x4/8x4   :163-214      satd4/8   :216-242
//   _sa8d_8x8      :244-279      sa8d_8x8 / sa8d_16x16 / sa8d8 / sa8d16 :281-322
//   pixel_ssd_s    :324-336      pixel_var :649-666     psyCost_pp :672-703
//
// Bit-exactness notes:
//  * the reference's SWAR sum2_t packing equals plain int32 arithmetic for
//    legal pixel ranges, so the Hadamards here are plain int32;
//  * SATD: every 4x4 Hadamard's |coef| sum is even, so Σ(raw>>1) = (Σraw)>>1
//    and any 4x4 tiling gives the reference's value;
//  * SA8D: the (x+2)>>2 rounding unit matters (8x8 for sa8d8, 16x16 for
//    sa8d16) and is kept per unit.
//
// Work mapping: one job per G-lane group; a lane handles one UWxUH unit per
// iteration (8x4 / 4x4 strips for SAD/SSE/SATD, 8x8 / 16x16 for SA8D); the
// group reduces with xor-shuffles.  8-bit SAD uses v_sad_u8 on packed dwords,
// 10/12-bit v_sad_u16.
#include <algorithm>
#include <vector>

#include "common.h"
#include "../../../include/x265_amd.h"

namespace x265amd {

// -------------------------------------------------------------- unit math

// NTA / NTB: non-temporal loads of the first / second block
template <typename P, int UW, int UH, bool NTA = false, bool NTB = false>
__device__ __forceinline__ uint32_t unit_sad(const P* a, intptr_t sa, const P* b, intptr_t sb)
{
    uint32_t s = 0;
#pragma unroll
    for (int y = 0; y < UH; y++)
    {
        if constexpr (sizeof(P) == 1)
        {
            if constexpr (UW == 8)
            {
                const uint2 va = ldx<uint2, NTA>(a + y * sa), vb = ldx<uint2, NTB>(b + y * sb);
                s = __builtin_amdgcn_sad_u8(va.x, vb.x, s);
                s = __builtin_amdgcn_sad_u8(va.y, vb.y, s);
            }
            else
            {
                const uint32_t va = ldx<uint32_t, NTA>(a + y * sa), vb = ldx<uint32_t, NTB>(b + y * sb);
                s = __builtin_amdgcn_sad_u8(va, vb, s);
            }
        }
        else
        {
            if constexpr (UW == 8)
            {
                const uint4 va = ldx<uint4, NTA>(a + y * sa), vb = ldx<uint4, NTB>(b + y * sb);
                s = __builtin_amdgcn_sad_u16(va.x, vb.x, s);
                s = __builtin_amdgcn_sad_u16(va.y, vb.y, s);
                s = __builtin_amdgcn_sad_u16(va.z, vb.z, s);
                s = __builtin_amdgcn_sad_u16(va.w, vb.w, s);
            }
            else
            {
                const uint2 va = ldx<uint2, NTA>(a + y * sa), vb = ldx<uint2, NTB>(b + y * sb);
                s = __builtin_amdgcn_sad_u16(va.x, vb.x, s);
                s = __builtin_amdgcn_sad_u16(va.y, vb.y, s);
            }
        }
    }
    return s;
}

// Σ(a-b)^2 as uint32 per term (the reference's int product, two's complement)
template <typename T, int UW, int UH, bool IS16>
__device__ __forceinline__ uint64_t unit_sse(const T* a, intptr_t sa, const T* b, intptr_t sb)
{
    uint64_t s = 0;
#pragma unroll
    for (int y = 0; y < UH; y++)
    {
        int va[UW], vb[UW];
        if constexpr (IS16) { load_row16<UW>((const int16_t*)a + y * sa, va); load_row16<UW>((const int16_t*)b + y * sb, vb); }
        else { load_row<T, UW>(a + y * sa, va); load_row<T, UW>(b + y * sb, vb); }
        uint32_t r = 0;
#pragma unroll
        for (int x = 0; x < UW; x++)
        {
            int d = va[x] - vb[x];
            r += (uint32_t)(d * d);
        }
        s += r;
    }
    return s;
}

template <int UW, int UH>
__device__ __forceinline__ uint64_t unit_ssd(const int16_t* a, intptr_t sa)
{
    uint64_t s = 0;
#pragma unroll
    for (int y = 0; y < UH; y++)
    {
        int va[UW];
        load_row16<UW>(a + y * sa, va);
        uint32_t r = 0;
#pragma unroll
        for (int x = 0; x < UW; x++) r += (uint32_t)(va[x] * va[x]);
        s += r;
    }
    return s;
}

// var: low 32 bits = Σp, high 32 bits = Σp² (wrapping, as the reference's uint32 sqr)
template <typename P, int UW, int UH>
__device__ __forceinline__ uint64_t unit_var(const P* a, intptr_t sa)
{
    uint32_t s = 0, q = 0;
#pragma unroll
    for (int y = 0; y < UH; y++)
    {
        int va[UW];
        load_row<P, UW>(a + y * sa, va);
#pragma unroll
        for (int x = 0; x < UW; x++) { s += va[x]; q += (uint32_t)(va[x] * va[x]); }
    }
    return (uint64_t)s + ((uint64_t)q << 32);
}

// raw 4x4 Hadamard |coef| sum of d (before the reference's >>1)
__device__ __forceinline__ uint32_t had4x4(int (&d)[4][4])
{
#pragma unroll
    for (int i = 0; i < 4; i++)
    {
        int t0 = d[i][0] + d[i][1], t1 = d[i][0] - d[i][1];
        int t2 = d[i][2] + d[i][3], t3 = d[i][2] - d[i][3];
        d[i][0] = t0 + t2; d[i][2] = t0 - t2; d[i][1] = t1 + t3; d[i][3] = t1 - t3;
    }
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < 4; j++)
    {
        int t0 = d[0][j] + d[1][j], t1 = d[0][j] - d[1][j];
        int t2 = d[2][j] + d[3][j], t3 = d[2][j] - d[3][j];
        s += abs(t0 + t2) + abs(t0 - t2) + abs(t1 + t3) + abs(t1 - t3);
    }
    return s;
}

#include "hadamard.h"

// raw satd of an 8x4 strip (two 4x4 Hadamards), 8-bit, packed pairs of rows
__device__ __forceinline__ uint32_t raw_satd8x4_pk(const uint8_t* a, intptr_t sa, const uint8_t* b, intptr_t sb)
{
    s16x2 Q[2][8];
#pragma unroll
    for (int k = 0; k < 2; k++)
    {
        s16x2 qa[8], qb[8];
        pack_rows8(ldu<uint2>(a + 2 * k * sa), ldu<uint2>(a + (2 * k + 1) * sa), qa);
        pack_rows8(ldu<uint2>(b + 2 * k * sb), ldu<uint2>(b + (2 * k + 1) * sb), qb);
#pragma unroll
        for (int j = 0; j < 8; j++) Q[k][j] = qa[j] - qb[j];
#pragma unroll
        for (int h = 0; h < 8; h += 4)       // 4-point row transforms of both 4x4 halves
        {
            const s16x2 a0 = Q[k][h] + Q[k][h + 1], a1 = Q[k][h] - Q[k][h + 1];
            const s16x2 a2 = Q[k][h + 2] + Q[k][h + 3], a3 = Q[k][h + 2] - Q[k][h + 3];
            Q[k][h] = a0 + a2; Q[k][h + 2] = a0 - a2; Q[k][h + 1] = a1 + a3; Q[k][h + 3] = a1 - a3;
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < 8; j += 2)           // column stage over row bit 1, then bit 0 fused
    {
        const s16x2 c0 = Q[0][j] + Q[1][j], c1 = Q[0][j] - Q[1][j];
        const s16x2 d0 = Q[0][j + 1] + Q[1][j + 1], d1 = Q[0][j + 1] - Q[1][j + 1];
        s = abs_pair_sum(c0, d0, s);
        s = abs_pair_sum(c1, d1, s);
    }
    return s;
}

template <typename P, int UW>
__device__ __forceinline__ uint32_t unit_satd(const P* a, intptr_t sa, const P* b, intptr_t sb)
{
    if constexpr (sizeof(P) == 1 && UW == 8) return raw_satd8x4_pk(a, sa, b, sb);
    // UW = 4: one 4x4; UW = 8: two 4x4 side by side (satd_8x4)
    uint32_t s = 0;
#pragma unroll
    for (int half = 0; half < UW / 4; half++)
    {
        int d[4][4];
#pragma unroll
        for (int y = 0; y < 4; y++)
        {
            int va[4], vb[4];
            load_row<P, 4>(a + y * sa + 4 * half, va);
            load_row<P, 4>(b + y * sb + 4 * half, vb);
#pragma unroll
            for (int x = 0; x < 4; x++) d[y][x] = va[x] - vb[x];
        }
        s += had4x4(d);
    }
    return s;
}

template <typename P>
__device__ __forceinline__ uint32_t raw_sa8d(const P* a, intptr_t sa, const P* b, intptr_t sb)
{
    if constexpr (sizeof(P) == 1) return raw_sa8d_pk(a, sa, b, sb);
    int d[8][8];
#pragma unroll
    for (int y = 0; y < 8; y++)
    {
        int va[8], vb[8];
        load_row<P, 8>(a + y * sa, va);
        load_row<P, 8>(b + y * sb, vb);
#pragma unroll
        for (int x = 0; x < 8; x++) d[y][x] = va[x] - vb[x];
    }
    return had8x8(d);
}

template <typename P>
__device__ __forceinline__ int psy_energy4(const P* a, intptr_t sa)
{
    int d[4][4];
    uint32_t sad = 0;
#pragma unroll
    for (int y = 0; y < 4; y++)
    {
        int va[4];
        load_row<P, 4>(a + y * sa, va);
#pragma unroll
        for (int x = 0; x < 4; x++) { d[y][x] = va[x]; sad += va[x]; }
    }
    int satd = (int)(had4x4(d) >> 1);
    return satd - (int)(sad >> 2);
}

// -------------------------------------------------------------- kernels
// (grouped launches, common.h: a = block A, b = block B, d = out)

template <int OP, typename P, int UW, int UH, bool NT = false>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_pixelcmp(const BatchGroup g)
{
    const uint32_t gb = xcd_block();
    const SubBatch& sub = group_sub(g, gb);
    const int w = sub.w, h = sub.h, n = sub.n, lg = sub.lg, wrap32 = g.flag;
    const intptr_t sa = sub.sa, sb = sub.sb;
    const int G = 1 << lg;
    const uint32_t lb = gb - sub.block0;
    const int64_t job = (int64_t)lb * (X265AMD_BLOCK >> lg) + (threadIdx.x >> lg);
    const int lane = threadIdx.x & (G - 1);
    const bool live = job < n;
    const int64_t jj = live ? job : 0;
    void* __restrict__ out = sub.d;

    const P* pa = (const P*)sub.a + sub.aoff[jj];
    const P* pb = (OP == X265AMD_SSD_S || OP == X265AMD_VAR) ? nullptr : (const P*)sub.b + sub.boff[jj];
    const int ux = w / UW, units = ux * (h / UH);

    uint64_t acc = 0;
    if constexpr (OP == X265AMD_SA8D && UW == 16)
    {
        // sa8d16: one (raw+2)>>2 per 16x16, computed as a quad of 8x8
        // Hadamards on 4 adjacent lanes (lane&3 = quadrant) whose raw sums meet
        // by shuffle — a quarter of the registers of a whole-16x16 lane.
        // G >= 4 and a multiple of 4, so quads never straddle groups.
        (void)units;
        const int qx16 = w >> 4, units8 = qx16 * (h >> 4) * 4;
        if (live)
        {
            for (int u0 = 0; u0 < units8; u0 += G)
            {
                const int u = u0 + lane;
                uint32_t r = 0;
                if (u < units8)
                {
                    const int q = u >> 2, k = u & 3;
                    const int x = (q % qx16) * 16 + (k & 1) * 8, y = (q / qx16) * 16 + (k >> 1) * 8;
                    r = raw_sa8d<P>(pa + y * sa + x, sa, pb + y * sb + x, sb);
                }
                r += __shfl_xor(r, 1, 64);
                r += __shfl_xor(r, 2, 64);
                if ((lane & 3) == 0) acc += (r + 2) >> 2;
            }
        }
    }
    else if (live)
    {
        for (int u = lane; u < units; u += G)
        {
            const int x = (u % ux) * UW, y = (u / ux) * UH;
            const P* qa = pa + y * sa + x;
            if constexpr (OP == X265AMD_SAD)
                acc += unit_sad<P, UW, UH, NT, NT>(qa, sa, pb + y * sb + x, sb);
            else if constexpr (OP == X265AMD_SATD)
                acc += unit_satd<P, UW>(qa, sa, pb + y * sb + x, sb);
            else if constexpr (OP == X265AMD_SA8D)
                acc += (raw_sa8d<P>(qa, sa, pb + y * sb + x, sb) + 2) >> 2;
            else if constexpr (OP == X265AMD_SSE_PP)
                acc += unit_sse<P, UW, UH, false>(qa, sa, pb + y * sb + x, sb);
            else if constexpr (OP == X265AMD_SSE_SS)
                acc += unit_sse<P, UW, UH, true>(qa, sa, pb + y * sb + x, sb);
            else if constexpr (OP == X265AMD_PSY)
            {
                const P* qb = pb + y * sb + x;
                int e;
                if constexpr (UW == 4) e = psy_energy4<P>(qa, sa) - psy_energy4<P>(qb, sb);
                else e = psy_energy8<P>(qa, sa) - psy_energy8<P>(qb, sb);
                acc += (uint32_t)abs(e);
            }
            else if constexpr (OP == X265AMD_SSD_S)
                acc += unit_ssd<UW, UH>((const int16_t*)qa, sa);
            else if constexpr (OP == X265AMD_VAR)
                acc += unit_var<P, UW, UH>(qa, sa);
        }
    }

    // group reduction (all lanes of the wave participate in the shuffles)
    if constexpr (OP == X265AMD_SSE_PP || OP == X265AMD_SSE_SS || OP == X265AMD_SSD_S || OP == X265AMD_VAR)
    {
        for (int m = G >> 1; m > 0; m >>= 1)
        {
            uint32_t lo = __shfl_xor((uint32_t)acc, m, 64);
            uint32_t hi = __shfl_xor((uint32_t)(acc >> 32), m, 64);
            acc += ((uint64_t)hi << 32) | lo;
        }
        if (live && lane == 0)
        {
            uint64_t v = acc;
            if (wrap32 && OP != X265AMD_VAR) v &= 0xffffffffull;  // sse_t = uint32 at 8-bit
            ((uint64_t*)out)[job] = v;
        }
    }
    else
    {
        uint32_t v = (uint32_t)acc;
        for (int m = G >> 1; m > 0; m >>= 1) v += __shfl_xor(v, m, 64);
        if constexpr (OP == X265AMD_SATD) v >>= 1;
        if (live && lane == 0) ((int32_t*)out)[job] = (int32_t)v;
    }
}

template <typename P, int NREF, int UW, int UH, bool NT = false>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_sad_multi(const BatchGroup g)
{
    const uint32_t gb = xcd_block();
    const SubBatch& sub = group_sub(g, gb);
    const int w = sub.w, h = sub.h, n = sub.n, lg = sub.lg;
    const intptr_t fs = sub.sa, rs = sub.sb;
    const int G = 1 << lg;
    const uint32_t lb = gb - sub.block0;
    const int64_t job = (int64_t)lb * (X265AMD_BLOCK >> lg) + (threadIdx.x >> lg);
    const int lane = threadIdx.x & (G - 1);
    const bool live = job < n;
    const int64_t jj = live ? job : 0;
    int32_t* __restrict__ out = (int32_t*)sub.d;

    const P* pf = (const P*)sub.a + sub.aoff[jj];
    const P* pr[NREF];
#pragma unroll
    for (int k = 0; k < NREF; k++) pr[k] = (const P*)sub.b + sub.boff[jj * NREF + k];
    const int ux = w / UW, units = ux * (h / UH);

    uint32_t acc[NREF];
#pragma unroll
    for (int k = 0; k < NREF; k++) acc[k] = 0;
    if (live)
    {
        for (int u = lane; u < units; u += G)
        {
            const int x = (u % ux) * UW, y = (u / ux) * UH;
#pragma unroll
            for (int k = 0; k < NREF; k++)
                acc[k] += unit_sad<P, UW, UH, false, NT>(pf + y * fs + x, fs, pr[k] + y * rs + x, rs);
        }
    }
#pragma unroll
    for (int k = 0; k < NREF; k++)
    {
        uint32_t v = acc[k];
        for (int m = G >> 1; m > 0; m >>= 1) v += __shfl_xor(v, m, 64);
        acc[k] = v;
    }
    if (live && lane == 0)
    {
#pragma unroll
        for (int k = 0; k < NREF; k++) out[job * NREF + k] = (int32_t)acc[k];
    }
}

// sad_x3 / sad_x4 of small blocks with one lane per (job, reference): lanes 4j .. 4j + 3 are job j's
// references 0 .. NREF - 1 (the fourth idle for x3).  The four lanes read the same source rows (one
// transaction) and four reference blocks, so one load instruction of a wave covers 16 jobs x 4 references;
// with one lane per job the wave's reference loads step through four separate blocks per lane.  Outputs
// land contiguously.  For blocks of at most 4 units (8x8, 8x16, 16x8, 4x8 ...), where a lane per job
// holds little work.
template <typename P, int NREF, int UW, int UH, bool NT = false>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_sad_multi_ref(const BatchGroup g)
{
    const uint32_t gb = xcd_block();
    const SubBatch& sub = group_sub(g, gb);
    const int w = sub.w, h = sub.h, n = sub.n;
    const intptr_t fs = sub.sa, rs = sub.sb;
    const uint32_t lb = gb - sub.block0;
    const int64_t job = (int64_t)lb * (X265AMD_BLOCK >> 2) + (threadIdx.x >> 2);
    const int k = threadIdx.x & 3;
    const bool live = job < n && k < NREF;
    if (!live) return;
    const P* pf = (const P*)sub.a + sub.aoff[job];
    const P* pr = (const P*)sub.b + sub.boff[job * NREF + k];
    const int ux = w / UW, units = ux * (h / UH);
    uint32_t acc = 0;
    for (int u = 0; u < units; u++)
    {
        const int x = (u % ux) * UW, y = (u / ux) * UH;
        acc += unit_sad<P, UW, UH, NT, NT>(pf + y * fs + x, fs, pr + y * rs + x, rs);
    }
    ((int32_t*)sub.d)[job * NREF + k] = (int32_t)acc;
}

// -------------------------------------------------------------- dispatch

// kernel class of a batch: (op, unit width, unit height) packed in an int
static inline int cmp_pack(int op, int uw, int uh) { return (op << 16) | (uw << 8) | uh; }

// 8x8 SAD units (one lane per 8x8 block: twice the rows in flight per lane, each job's descriptors
// loaded by one lane) instead of 8x4 ones: SAD 64x64 0.66 -> 0.79 of the HBM peak, 8x8 / 16x16 level
// (profiles/r04/sad_uh8_ab_and_me_async.txt); X265AMD_SAD_UH8=0 selects the 8x4 units, =2 also for sad_x3/x4
static int sad_uh8()
{
    static int v = -1;
    if (v < 0)
    {
        const char* e = getenv("X265AMD_SAD_UH8");
        v = e ? atoi(e) : 1;
    }
    return v;
}

static int cmp_class(int op, int w, int h)
{
    if ((w % 4) || (h % 4) || w > 64 || h > 64 || w < 4 || h < 4) return -X265AMD_EINVAL;
    const int uwd = (w % 8) ? 4 : 8;
    if (op == X265AMD_SAD && w % 8 == 0 && h % 8 == 0 && sad_uh8() > 0) return cmp_pack(op, 8, 8);
    switch (op)
    {
    case X265AMD_SAD: case X265AMD_SATD: case X265AMD_SSE_PP: case X265AMD_SSE_SS:
    case X265AMD_SSD_S: case X265AMD_VAR:
        return cmp_pack(op, uwd, 4);
    case X265AMD_SA8D:
        if ((w % 16) == 0 && (h % 16) == 0) return cmp_pack(op, 16, 16);
        if ((w % 8) == 0 && (h % 8) == 0) return cmp_pack(op, 8, 8);
        return cmp_pack(X265AMD_SATD, uwd, 4);  // 4x4 / 4x8 sa8d entries are satd (primitives.cpp:106,164-171)
    case X265AMD_PSY:
        if (w != h) return -X265AMD_EINVAL;
        return w == 4 ? cmp_pack(op, 4, 4) : cmp_pack(op, 8, 8);
    }
    return -X265AMD_EINVAL;
}

static int cmp_lg(int cls, int w, int h)
{
    const int op = cls >> 16, uw = (cls >> 8) & 0xff, uh = cls & 0xff;
    if (op == X265AMD_SA8D && uw == 16)      // quads of 8x8 lanes, G >= 4
        return std::max(2, lanes_log2((w / 8) * (h / 8)));
    return lanes_log2((w / uw) * (h / uh));
}

// X265AMD_NT=0: SAD with ordinary loads (1, the default: both blocks non-temporal).  sad_x3 / sad_x4 keep
// ordinary loads: their wave's reference rows share lines between the per-reference load instructions, which
// non-temporal loads turn into repeated HBM reads (sad_x4 8x8 0.57 -> 0.40, profiles/r05/sad_nt_ab.txt)
static bool nt_loads()
{
    static int v = -1;
    if (v < 0)
    {
        const char* e = getenv("X265AMD_NT");
        v = e ? atoi(e) != 0 : 1;
    }
    return v != 0;
}

template <int OP, typename P, int UW, int UH>
static int launch_cmp(const BatchGroup& g, uint32_t blocks, hipStream_t st)
{
    if constexpr (OP == X265AMD_SAD)
    {
        if (nt_loads())
        {
            hipLaunchKernelGGL((k_pixelcmp<OP, P, UW, UH, true>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g);
            return (int)hipGetLastError();
        }
    }
    hipLaunchKernelGGL((k_pixelcmp<OP, P, UW, UH>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g);
    return (int)hipGetLastError();
}

template <typename P>
static int launch_cmp_class(int cls, const BatchGroup& g, uint32_t blocks, hipStream_t st)
{
    using S = int16_t;
#define X265AMD_CMP(OPX, PX, W, H) \
    if (cls == cmp_pack(OPX, W, H)) return launch_cmp<OPX, PX, W, H>(g, blocks, st);
    X265AMD_CMP(X265AMD_SAD, P, 8, 8)     X265AMD_CMP(X265AMD_SAD, P, 8, 4)     X265AMD_CMP(X265AMD_SAD, P, 4, 4)
    X265AMD_CMP(X265AMD_SATD, P, 8, 4)    X265AMD_CMP(X265AMD_SATD, P, 4, 4)
    X265AMD_CMP(X265AMD_SA8D, P, 16, 16)  X265AMD_CMP(X265AMD_SA8D, P, 8, 8)
    X265AMD_CMP(X265AMD_SSE_PP, P, 8, 4)  X265AMD_CMP(X265AMD_SSE_PP, P, 4, 4)
    X265AMD_CMP(X265AMD_SSE_SS, S, 8, 4)  X265AMD_CMP(X265AMD_SSE_SS, S, 4, 4)
    X265AMD_CMP(X265AMD_PSY, P, 4, 4)     X265AMD_CMP(X265AMD_PSY, P, 8, 8)
    X265AMD_CMP(X265AMD_SSD_S, S, 8, 4)   X265AMD_CMP(X265AMD_SSD_S, S, 4, 4)
    X265AMD_CMP(X265AMD_VAR, P, 8, 4)     X265AMD_CMP(X265AMD_VAR, P, 4, 4)
#undef X265AMD_CMP
    return X265AMD_EINVAL;
}

static int cmp_classes(int count, const x265amd_cmp_batch* bt, std::vector<int>& cls,
                       int (*classify)(int, int, int), int op)
{
    cls.assign(count, -1);
    for (int i = 0; i < count; i++)
    {
        if (bt[i].n < 0) return X265AMD_EINVAL;
        if (bt[i].n == 0) continue;
        const int c = classify(op, bt[i].w, bt[i].h);
        if (c < 0) return -c;
        cls[i] = c;
    }
    return 0;
}

static void cmp_fill(const x265amd_cmp_batch& b, int cls, SubBatch& s)
{
    s = SubBatch{};
    s.a = b.a; s.aoff = b.a_off; s.sa = b.a_stride;
    s.b = b.b; s.boff = b.b_off; s.sb = b.b_stride;
    s.d = b.out;
    s.w = b.w; s.h = b.h; s.n = b.n;
    s.lg = cmp_lg(cls, b.w, b.h);
}

template <typename P>
static int dispatch_cmp(int op, int count, const x265amd_cmp_batch* bt, hipStream_t st)
{
    std::vector<int> cls;
    if (int rc = cmp_classes(count, bt, cls, cmp_class, op)) return rc;
    BatchGroup proto{};
    proto.flag = sizeof(P) == 1;   // sse_t is uint32 at 8-bit
    return launch_grouped(count, cls.data(), proto,
        [&](int i, SubBatch& s) { cmp_fill(bt[i], cls[i], s); },
        [&](int c, const BatchGroup& g, uint32_t blocks) { return launch_cmp_class<P>(c, g, blocks, st); });
}

// sad_x3 / sad_x4 lane layout (X265AMD_SADX_LANES bits): 1 = a lane per (job, reference) for blocks of at most
// 4 units, 2 = with 8x8 units where the block allows, 4 = non-temporal loads (the four lanes of a job read a row
// in one instruction, so nothing is re-fetched); 0 = a lane per job everywhere; 8, the default = bits 1 | 2 | 4
// for 8x8 blocks only (one 8x8 unit per lane: sad_x4 8x8 0.57 -> 0.59, while 16x16 with four 8x8 units per lane
// drops 0.72 -> 0.43 and 8x4 units measured 0.53-0.58, profiles/r05/sadx_lanes_ab.txt)
static int sadx_lanes()
{
    static int v = -1;
    if (v < 0)
    {
        const char* e = getenv("X265AMD_SADX_LANES");
        v = e ? atoi(e) : 8;
    }
    return v;
}
constexpr int kSadRefOp = 0x7f;   // class tag of k_sad_multi_ref
static bool sadx_uh8() { return (sadx_lanes() & 2) != 0; }
static bool sadx_nt() { return (sadx_lanes() & 4) != 0; }

static int sad_multi_class(int, int w, int h)
{
    if ((w % 4) || (h % 4) || w > 64 || h > 64 || w < 4 || h < 4) return -X265AMD_EINVAL;
    const int uw = (w % 8) ? 4 : 8;
    // the non-temporal flag travels in the class (bit 7 of the unit-height byte)
    if (sadx_lanes() == 8)
    {
        if (w == 8 && h == 8) return cmp_pack(kSadRefOp, 8, 8 | 0x80);
    }
    else if (sadx_lanes() & 1)
    {
        const int nt = sadx_nt() ? 0x80 : 0;
        if (sadx_uh8() && uw == 8 && h % 8 == 0 && (w / 8) * (h / 8) <= 4) return cmp_pack(kSadRefOp, 8, 8 | nt);
        if ((w / uw) * (h / 4) <= 4) return cmp_pack(kSadRefOp, uw, 4 | nt);
    }
    // (8x8 units measured no faster for sad_x4 8x8 and slower for 16x16: profiles/r04/sad_uh8_ab_and_me_async.txt)
    if (w % 8 == 0 && h % 8 == 0 && sad_uh8() > 1) return cmp_pack(X265AMD_SAD, 8, 8);
    return cmp_pack(X265AMD_SAD, (w % 8) ? 4 : 8, 4);
}

template <typename P, int NREF>
static int dispatch_multi(int count, const x265amd_cmp_batch* bt, hipStream_t st)
{
    std::vector<int> cls;
    if (int rc = cmp_classes(count, bt, cls, sad_multi_class, 0)) return rc;
    return launch_grouped(count, cls.data(), BatchGroup{},
        [&](int i, SubBatch& s) {
            cmp_fill(bt[i], cls[i], s);
            if ((cls[i] >> 16) == kSadRefOp) s.lg = 2;     // four lanes per job
        },
        [&](int c, const BatchGroup& g, uint32_t blocks) {
            const bool nt = (c & 0x80) != 0;
            if ((c >> 16) == kSadRefOp && (c & 0x7f) == 8)
            {
                if (nt) hipLaunchKernelGGL((k_sad_multi_ref<P, NREF, 8, 8, true>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g);
                else hipLaunchKernelGGL((k_sad_multi_ref<P, NREF, 8, 8>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g);
            }
            else if ((c >> 16) == kSadRefOp && ((c >> 8) & 0xff) == 8)
            {
                if (nt) hipLaunchKernelGGL((k_sad_multi_ref<P, NREF, 8, 4, true>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g);
                else hipLaunchKernelGGL((k_sad_multi_ref<P, NREF, 8, 4>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g);
            }
            else if ((c >> 16) == kSadRefOp)
                hipLaunchKernelGGL((k_sad_multi_ref<P, NREF, 4, 4>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g);
            else if (((c >> 8) & 0xff) == 8 && (c & 0xff) == 8)
                hipLaunchKernelGGL((k_sad_multi<P, NREF, 8, 8>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g);
            else if (((c >> 8) & 0xff) == 8)
                hipLaunchKernelGGL((k_sad_multi<P, NREF, 8, 4>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g);
            else
                hipLaunchKernelGGL((k_sad_multi<P, NREF, 4, 4>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g);
            return (int)hipGetLastError();
        });
}

} // namespace x265amd

using namespace x265amd;

extern "C" int x265amd_pixelcmp_grouped(int op, int depth, int count, const x265amd_cmp_batch* batches,
                                        void* stream)
{
    if (count < 0 || (count > 0 && !batches)) return X265AMD_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    if (depth == 8) return dispatch_cmp<uint8_t>(op, count, batches, st);
    if (depth == 10 || depth == 12) return dispatch_cmp<uint16_t>(op, count, batches, st);
    return X265AMD_EINVAL;
}

extern "C" int x265amd_sad_multi_grouped(int nref, int depth, int count, const x265amd_cmp_batch* batches,
                                         void* stream)
{
    if (count < 0 || (count > 0 && !batches)) return X265AMD_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    if (nref != 3 && nref != 4) return X265AMD_EINVAL;
    if (depth == 8)
        return nref == 3 ? dispatch_multi<uint8_t, 3>(count, batches, st) : dispatch_multi<uint8_t, 4>(count, batches, st);
    if (depth == 10 || depth == 12)
        return nref == 3 ? dispatch_multi<uint16_t, 3>(count, batches, st) : dispatch_multi<uint16_t, 4>(count, batches, st);
    return X265AMD_EINVAL;
}

extern "C" int x265amd_pixelcmp(int op, int depth, int w, int h, int n,
                                const void* a, intptr_t a_stride, const int64_t* a_off,
                                const void* b, intptr_t b_stride, const int64_t* b_off,
                                void* out, void* stream)
{
    if (n <= 0) return 0;
    const x265amd_cmp_batch bt = {w, h, n, a, a_stride, a_off, b, b_stride, b_off, out};
    return x265amd_pixelcmp_grouped(op, depth, 1, &bt, stream);
}

extern "C" int x265amd_sad_multi(int nref, int depth, int w, int h, int n,
                                 const void* fenc, intptr_t fenc_stride, const int64_t* fenc_off,
                                 const void* ref, intptr_t ref_stride, const int64_t* ref_off,
                                 int32_t* out, void* stream)
{
    if (n <= 0) return 0;
    const x265amd_cmp_batch bt = {w, h, n, fenc, fenc_stride, fenc_off, ref, ref_stride, ref_off, out};
    return x265amd_sad_multi_grouped(nref, depth, 1, &bt, stream);
}
