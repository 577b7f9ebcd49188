// blockops.hip — batched companion block operations of the primitive table
// (SURVEY.md §8(a) row a15): residual / reconstruction / bi-prediction
// averages / typed block copies / fills / 2D<->1D shifted copies / transpose.
//
// Reference semantics: x265_1.9/source/common/pixel.cpp
//   blockfill_s_c :338-344   cpy2Dto1D_shl/shr :346-379   cpy1Dto2D_shl/shr :381-414
//   getResidual :416-428     transpose :430-436           pixelavg_pp :490-502
//   blockcopy_pp/ss/sp/ps :705-758   pixel_sub_ps_c :760-772   pixel_add_ps_c :774-786
//   addAvg :788-808 (shiftNum = IF_INTERNAL_PREC + 1 - depth, offset includes 2*IF_INTERNAL_OFFS)
//
// Work mapping: one block per G-lane group, a lane handles UW (8/4/2)
// contiguous elements of one row per step, loads and stores vectorised.
#include <algorithm>
#include <stdlib.h>

#include "common.h"
#include "../../../include/x265_amd.h"

namespace x265amd {

template <typename P, int OP>
struct OpTypes;
#define OPT(OP, D, A, B) template <typename P> struct OpTypes<P, OP> { typedef D d; typedef A a; typedef B b; };
OPT(X265AMD_SUB_PS, int16_t, P, P)
OPT(X265AMD_ADD_PS, P, P, int16_t)
OPT(X265AMD_ADDAVG, P, int16_t, int16_t)
OPT(X265AMD_PIXELAVG, P, P, P)
OPT(X265AMD_COPY_PP, P, P, P)
OPT(X265AMD_COPY_SP, P, int16_t, int16_t)
OPT(X265AMD_COPY_PS, int16_t, P, P)
OPT(X265AMD_COPY_SS, int16_t, int16_t, int16_t)
OPT(X265AMD_BLOCKFILL, int16_t, int16_t, int16_t)
OPT(X265AMD_CPY2D1D_SHL, int16_t, int16_t, int16_t)
OPT(X265AMD_CPY2D1D_SHR, int16_t, int16_t, int16_t)
OPT(X265AMD_CPY1D2D_SHL, int16_t, int16_t, int16_t)
OPT(X265AMD_CPY1D2D_SHR, int16_t, int16_t, int16_t)
OPT(X265AMD_TRANSPOSE, P, P, P)
#undef OPT

template <typename T, int UW>
__device__ __forceinline__ void ld(const T* p, int (&o)[UW])
{
    if constexpr (std::is_same<T, int16_t>::value) load_row16<UW>(p, o);
    else load_row<T, UW>(p, o);
}

// one row of a unit as raw bytes: a single vector load (2..16 bytes)
template <typename T, int UW>
struct RowRaw
{
    T v[UW];
};

// JPL jobs per lane group (k-th job = first + k * groups-per-block): all their
// offsets, then all their row loads, are issued before the first use, so a
// wave keeps JPL times the bytes in flight across the dependent offset -> data
// chain that bounds these small, latency-limited block copies.
//
// STG (compact destinations, dst stride = w, power-of-two w and h, one unit per
// lane): each job set's outputs are staged in wave-private LDS and leave
// through stage_writeback (common.h) as 16-byte chunks.
template <typename P, int OP, int UW, int UH, int JPL, bool STG = false>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_blockop(const BatchGroup g)
{
    typedef typename OpTypes<P, OP>::d D;
    typedef typename OpTypes<P, OP>::a A;
    typedef typename OpTypes<P, OP>::b B;
    constexpr bool TWO = OP == X265AMD_SUB_PS || OP == X265AMD_ADD_PS || OP == X265AMD_ADDAVG || OP == X265AMD_PIXELAVG;
    constexpr bool ROWS = OP != X265AMD_BLOCKFILL && OP != X265AMD_TRANSPOSE;
    const uint32_t gb = xcd_block();
    const SubBatch& sub = group_sub(g, gb);
    const int w = sub.w, h = sub.h, n = sub.n, lg = sub.lg, param = sub.param, depth = g.depth;
    const intptr_t ds = sub.ds, sa = sub.sa, sb = sub.sb;
    const int G = 1 << lg;
    const int64_t per = X265AMD_BLOCK >> lg;
    const int64_t job0 = (int64_t)(gb - sub.block0) * per * JPL + (threadIdx.x >> lg);
    const int64_t wjob0 = (int64_t)(gb - sub.block0) * per * JPL + ((threadIdx.x & ~63u) >> lg);
    const int lane = threadIdx.x & (G - 1);
    constexpr int STG_LANE = UW * UH * (int)sizeof(D);        // staged bytes per lane and job set
    constexpr int STG_WAVE = STG ? 64 * STG_LANE : 16;
    __shared__ uint4 stg_lds[STG ? X265AMD_BLOCK / 64 * JPL * STG_WAVE / 16 : 1];
    if constexpr (STG)
    {
        if (wjob0 >= n) return;                 // lanes past the batch stage copies never written out
    }
    else if (job0 >= n)
        return;
    const int wh = w * h * (int)sizeof(D);
    uint8_t* const stg = (uint8_t*)stg_lds + (threadIdx.x >> 6) * JPL * STG_WAVE + ((threadIdx.x & 63) >> lg) * wh;

    D* pd[JPL];
    const A* pa[JPL];
    const B* pb[JPL];
    bool live[JPL];
#pragma unroll
    for (int k = 0; k < JPL; k++)
    {
        const int64_t job = job0 + k * per;
        live[k] = job < n;
        const int64_t jj = live[k] ? job : (STG ? n - 1 : job0);
        pd[k] = (D*)sub.d + sub.doff[jj];
        pa[k] = OP == X265AMD_BLOCKFILL ? nullptr : (const A*)sub.a + sub.aoff[jj];
        pb[k] = TWO ? (const B*)sub.b + sub.boff[jj] : nullptr;
    }
    const int maxv = (1 << depth) - 1;
    const int avg_shift = 15 - depth, avg_off = (1 << (avg_shift - 1)) + 2 * 8192;
    const int ux = w / UW, units = ux * (h / UH);

    for (int u = lane; u < units; u += G)
    {
        const int x = (u % ux) * UW, y0 = (u / ux) * UH;
        RowRaw<A, UW> ra[JPL][UH];
        RowRaw<B, UW> rb[JPL][UH];
        if constexpr (ROWS)
        {
#pragma unroll
            for (int k = 0; k < JPL; k++)
#pragma unroll
                for (int r = 0; r < UH; r++)
                {
                    ra[k][r] = ldu<RowRaw<A, UW>>(pa[k] + (y0 + r) * sa + x);
                    if constexpr (TWO) rb[k][r] = ldu<RowRaw<B, UW>>(pb[k] + (y0 + r) * sb + x);
                }
        }
#pragma unroll
        for (int k = 0; k < JPL; k++)
        {
            if (!STG && !live[k]) continue;
#pragma unroll
            for (int r = 0; r < UH; r++)
            {
                const int y = y0 + r;
                int o[UW];
                if constexpr (OP == X265AMD_BLOCKFILL)
                {
#pragma unroll
                    for (int i = 0; i < UW; i++) o[i] = param;
                }
                else if constexpr (OP == X265AMD_TRANSPOSE)
                {
                    // output row y = source column y
#pragma unroll
                    for (int i = 0; i < UW; i++) o[i] = pa[k][(x + i) * sa + y];
                }
                else
                {
                    int va[UW];
                    ld<A, UW>(ra[k][r].v, va);
                    if constexpr (TWO)
                    {
                        int vb[UW];
                        ld<B, UW>(rb[k][r].v, vb);
#pragma unroll
                        for (int i = 0; i < UW; i++)
                        {
                            if constexpr (OP == X265AMD_SUB_PS) o[i] = va[i] - vb[i];
                            else if constexpr (OP == X265AMD_ADD_PS) { const int v = va[i] + vb[i]; o[i] = v < 0 ? 0 : (v > maxv ? maxv : v); }
                            else if constexpr (OP == X265AMD_ADDAVG) { const int v = (va[i] + vb[i] + avg_off) >> avg_shift; o[i] = v < 0 ? 0 : (v > maxv ? maxv : v); }
                            else o[i] = (va[i] + vb[i] + 1) >> 1;
                        }
                    }
                    else
                    {
#pragma unroll
                        for (int i = 0; i < UW; i++)
                        {
                            if constexpr (OP == X265AMD_CPY2D1D_SHL || OP == X265AMD_CPY1D2D_SHL) o[i] = va[i] << param;
                            else if constexpr (OP == X265AMD_CPY2D1D_SHR || OP == X265AMD_CPY1D2D_SHR)
                                o[i] = (va[i] + (int)(int16_t)(1 << (param - 1))) >> param;
                            else o[i] = va[i];   // typed copies (pixel <-> int16 casts truncate like the reference)
                        }
                    }
                }
                if constexpr (STG) store_row<D, UW>((D*)(stg + k * STG_WAVE) + y * w + x, o);
                else store_row<D, UW>(pd[k] + y * ds + x, o);
            }
        }
    }
    if constexpr (STG)
    {
#pragma unroll
        for (int k = 0; k < JPL; k++)
            stage_writeback<STG_WAVE>((const uint8_t*)stg_lds + (threadIdx.x >> 6) * JPL * STG_WAVE + k * STG_WAVE,
                                      pd[k], lg, wh, wjob0 + k * per, n);
    }
}

// kernel class: unit width (8/4/2 elements) x unit height (1/2/4 rows) with
// one unit per lane.  The unit height aims at ~32 bytes of loads per lane:
// measured on MI355X (tools/kernel_roofline.py, 8x8 and 16x16 blocks), 8-16 B
// per lane leaves the chip issuing index math and 64+ B serialises each lane's
// loads; wide int16 operands (addAvg, add_ps) want one row, pixel-only copies four.
constexpr int kStagedBlock = 4096;

template <typename P, int OP>
static int blockop_class(int w, int h, int64_t ds)
{
    if (w < 2 || h < 1 || w > 64 || h > 64 || (w % 2)) return -X265AMD_EINVAL;
    typedef typename OpTypes<P, OP>::a A;
    typedef typename OpTypes<P, OP>::b B;
    constexpr bool TWO = OP == X265AMD_SUB_PS || OP == X265AMD_ADD_PS || OP == X265AMD_ADDAVG || OP == X265AMD_PIXELAVG;
    constexpr int esz = OP == X265AMD_BLOCKFILL ? 2 : (int)sizeof(A) + (TWO ? (int)sizeof(B) : 0);
    const int uw = (w % 8 == 0) ? 8 : (w % 4 == 0) ? 4 : 2;
    const int want = std::max(1, 32 / (uw * esz));
    int uh = (want >= 4 && h % 4 == 0) ? 4 : (want >= 2 && h % 2 == 0) ? 2 : 1;
    // two jobs per lane group for the streaming ops (measured +2-10% on 8x8..64x64)
    const int jpl = ((TWO || OP == X265AMD_COPY_PP) && uw == 8) ? 2 : 1;
    // compact destination: stage the outputs in LDS when every lane holds exactly one unit of
    // >= 16 bytes, two-row units for the one-row 8-byte ones (add_ps, addAvg at 8 bit)
    // (X265AMD_BLOCK_STAGE=0 disables)
    static const bool stage = !getenv("X265AMD_BLOCK_STAGE") || atoi(getenv("X265AMD_BLOCK_STAGE"));
    typedef typename OpTypes<P, OP>::d D;
    const bool p2 = (w & (w - 1)) == 0 && (h & (h - 1)) == 0;
    bool stg = false;
    if (stage && p2 && ds == w)
    {
        if (uw * uh * (int)sizeof(D) == 8 && uh == 1 && h % 2 == 0 && (w / uw) * (h / 2) <= 64) uh = 2;
        stg = uw * uh * (int)sizeof(D) >= 16 && (w / uw) * (h / uh) <= 64;
    }
    return jpl * 256 + uw * 16 + uh + (stg ? kStagedBlock : 0);
}

template <typename P, int OP>
static int launch_blockop(int cls, const BatchGroup& g, uint32_t blocks, hipStream_t st)
{
    constexpr bool MULTI = OP == X265AMD_SUB_PS || OP == X265AMD_ADD_PS || OP == X265AMD_ADDAVG ||
                           OP == X265AMD_PIXELAVG || OP == X265AMD_COPY_PP;
#define L(UW, UH, J) \
    if constexpr (UW * UH * sizeof(typename OpTypes<P, OP>::d) >= 16) \
        if (cls == (J * 256 + UW * 16 + UH | kStagedBlock)) \
        { \
            hipLaunchKernelGGL((k_blockop<P, OP, UW, UH, J, true>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g); \
            return (int)hipGetLastError(); \
        } \
    if (cls == J * 256 + UW * 16 + UH) \
    { \
        hipLaunchKernelGGL((k_blockop<P, OP, UW, UH, J>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, g); \
        return (int)hipGetLastError(); \
    }
    L(8, 4, 1) L(8, 2, 1) L(8, 1, 1) L(4, 4, 1) L(4, 2, 1) L(4, 1, 1) L(2, 4, 1) L(2, 2, 1) L(2, 1, 1)
    if constexpr (MULTI)
    {
        L(8, 4, 2) L(8, 2, 2) L(8, 1, 2)
    }
#undef L
    return X265AMD_EINVAL;
}

template <typename P, int OP>
static int grouped_blockop(int depth, int count, const x265amd_block_batch* bt, hipStream_t st)
{
    std::vector<int> cls(count, -1);
    for (int i = 0; i < count; i++)
    {
        if (bt[i].n < 0) return X265AMD_EINVAL;
        if (bt[i].n == 0) continue;
        cls[i] = blockop_class<P, OP>(bt[i].w, bt[i].h, bt[i].dst_stride);
        if (cls[i] < 0) return -cls[i];
    }
    BatchGroup proto{};
    proto.depth = depth;
    return launch_grouped(count, cls.data(), proto,
        [&](int i, SubBatch& s) {
            const x265amd_block_batch& b = bt[i];
            s = SubBatch{};
            s.d = b.dst; s.doff = b.dst_off; s.ds = b.dst_stride;
            s.a = b.a; s.aoff = b.a_off; s.sa = b.a_stride;
            s.b = b.b; s.boff = b.b_off; s.sb = b.b_stride;
            s.w = b.w; s.h = b.h; s.n = b.n; s.param = b.param;
            const int uw = (cls[i] / 16) % 16, uh = cls[i] % 16;
            s.jpl = (cls[i] & (kStagedBlock - 1)) / 256;
            s.lg = lanes_log2((b.w / uw) * (b.h / uh), 1);
        },
        [&](int c, const BatchGroup& g, uint32_t blocks) { return launch_blockop<P, OP>(c, g, blocks, st); });
}

template <typename P>
static int dispatch_blockop(int op, int depth, int count, const x265amd_block_batch* bt, hipStream_t st)
{
#define C(OP) case OP: return grouped_blockop<P, OP>(depth, count, bt, st)
    switch (op)
    {
    C(X265AMD_SUB_PS); C(X265AMD_ADD_PS); C(X265AMD_ADDAVG); C(X265AMD_PIXELAVG);
    C(X265AMD_COPY_PP); C(X265AMD_COPY_SP); C(X265AMD_COPY_PS); C(X265AMD_COPY_SS);
    C(X265AMD_BLOCKFILL); C(X265AMD_CPY2D1D_SHL); C(X265AMD_CPY2D1D_SHR);
    C(X265AMD_CPY1D2D_SHL); C(X265AMD_CPY1D2D_SHR); C(X265AMD_TRANSPOSE);
    }
#undef C
    return X265AMD_EINVAL;
}

} // namespace x265amd

using namespace x265amd;

extern "C" int x265amd_blockop_grouped(int op, int depth, int count, const x265amd_block_batch* batches,
                                       void* stream)
{
    if (count < 0 || (count > 0 && !batches)) return X265AMD_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    if (depth == 8) return dispatch_blockop<uint8_t>(op, depth, count, batches, st);
    if (depth == 10 || depth == 12) return dispatch_blockop<uint16_t>(op, depth, count, batches, st);
    return X265AMD_EINVAL;
}

extern "C" int x265amd_blockop(int op, int depth, int w, int h, int n,
                               void* dst, intptr_t dst_stride, const int64_t* dst_off,
                               const void* a, intptr_t a_stride, const int64_t* a_off,
                               const void* b, intptr_t b_stride, const int64_t* b_off,
                               int param, void* stream)
{
    if (n <= 0) return 0;
    const x265amd_block_batch bt = {w, h, n, param, dst, dst_stride, dst_off, a, a_stride, a_off, b, b_stride, b_off};
    return x265amd_blockop_grouped(op, depth, 1, &bt, stream);
}
