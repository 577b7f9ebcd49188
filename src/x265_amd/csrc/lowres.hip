// lowres.hip — the lookahead's lowres pipeline, the
// parts that depend only on the source pictures, batched over frames:
//
//   x265amd_lowres_init   Lowres::init plane generation (lowres.cpp:151-162):
//                         frameInitLowres = frame_init_lowres_core
//                         (pixel.cpp:549-573, 2:1 box downscale at four
//                         half-pel phases) + extendPicBorder of each plane
//                         (pixel.cpp:908-922, ipfilter.cpp:59-77)
//   x265amd_lowres_intra  LookaheadTLD::lowresIntraEstimate
//                         (slicetype.cpp:230-330): per 8x8 lowres CU the best
//                         of DC / planar / a coarse-to-fine angular sweep by
//                         8x8 SATD, plus the frame and row cost sums
//
// Work mapping.  Downscale: one thread per four lowres pixels of a row (three
// source rows of 9 pixels in, four 4-pixel row segments out).  Border
// extension: one thread per (plane, row) for the side margins, then one
// thread per 16-pixel chunk of each margin row (a second launch, so the
// corner areas copy the already-extended edge rows as the reference does).
// Intra estimate: one CU per 8-lane group.  The eight first-pass candidates
// (DC, planar, angular 5, 10, .., 30) run one per lane; the two refinement
// passes (best +-2, then best +-1) run on two lanes each.  Every lane
// predicts with the shared lane predictor of intra.hip (intra_lane.h) and
// scores with an in-register 8x8 SATD; the group gathers the costs by shuffle
// and applies the reference's strict first-minimum order, so ties resolve
// exactly as COPY2_IF_LT does.
#include "common.h"
#include "intra_lane.h"
#include "../../../include/x265_amd.h"

namespace x265amd {

struct LowresArgs
{
    const void* src;
    const int64_t* src_off;
    int64_t ss;
    void* planes;
    const int64_t* plane_off;     // 4 per frame
    int64_t ls;
    int n, width, lines, mx, my;
};

__device__ __forceinline__ int box4(int a, int b, int c, int d)
{
    return (((a + b + 1) >> 1) + ((c + d + 1) >> 1) + 1) >> 1;
}

template <typename P>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_lowres_core(const LowresArgs a)
{
    const int qx = a.width >> 2;
    const int64_t per_frame = (int64_t)a.lines * qx;
    const int64_t t = (int64_t)xcd_block() * X265AMD_BLOCK + threadIdx.x;
    if (t >= per_frame * a.n) return;
    const int f = (int)(t / per_frame);
    const int64_t r = t - f * per_frame;
    const int y = (int)(r / qx), x0 = 4 * (int)(r % qx);
    const P* s0 = (const P*)a.src + a.src_off[f] + 2 * y * a.ss + 2 * x0;
    int rw[3][9];
#pragma unroll
    for (int k = 0; k < 3; k++)
    {
        int v[8];
        load_row<P, 8>(s0 + k * a.ss, v);
#pragma unroll
        for (int i = 0; i < 8; i++) rw[k][i] = v[i];
        rw[k][8] = s0[k * a.ss + 8];
    }
    int o[4][4];
#pragma unroll
    for (int i = 0; i < 4; i++)
    {
        const int x = 2 * i;
        o[0][i] = box4(rw[0][x], rw[1][x], rw[0][x + 1], rw[1][x + 1]);
        o[1][i] = box4(rw[0][x + 1], rw[1][x + 1], rw[0][x + 2], rw[1][x + 2]);
        o[2][i] = box4(rw[1][x], rw[2][x], rw[1][x + 1], rw[2][x + 1]);
        o[3][i] = box4(rw[1][x + 1], rw[2][x + 1], rw[1][x + 2], rw[2][x + 2]);
    }
#pragma unroll
    for (int k = 0; k < 4; k++)
        store_row<P, 4>((P*)a.planes + a.plane_off[4 * f + k] + y * a.ls + x0, o[k]);
}

// left / right margins of rows 0 .. lines-1 (extendRowBorder)
template <typename P>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_lowres_extend_lr(const LowresArgs a)
{
    const int64_t t = (int64_t)xcd_block() * X265AMD_BLOCK + threadIdx.x;
    const int64_t rows = (int64_t)a.n * 4 * a.lines;
    if (t >= 2 * rows) return;
    const bool right = t >= rows;
    const int64_t rr = right ? t - rows : t;
    const int pl = (int)(rr / a.lines), y = (int)(rr % a.lines);
    P* row = (P*)a.planes + a.plane_off[pl] + y * a.ls;
    const P v = right ? row[a.width - 1] : row[0];
    P* d = right ? row + a.width : row - a.mx;
    int x = 0;
    if constexpr (sizeof(P) == 1)
    {
        const uint32_t w = 0x01010101u * (uint32_t)v;
        for (; x + 4 <= a.mx; x += 4) stu<uint32_t>(d + x, w);
    }
    else
    {
        const uint32_t w = 0x00010001u * (uint32_t)v;
        for (; x + 2 <= a.mx; x += 2) stu<uint32_t>(d + x, w);
    }
    for (; x < a.mx; x++) d[x] = v;
}

// margin rows: copies of the extended first / last row over the whole stride
template <typename P>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_lowres_extend_tb(const LowresArgs a)
{
    constexpr int C = 16;
    const int64_t chunks = (a.ls + C - 1) / C;
    const int64_t per_plane = 2 * (int64_t)a.my * chunks;
    const int64_t t = (int64_t)xcd_block() * X265AMD_BLOCK + threadIdx.x;
    if (t >= per_plane * 4 * a.n) return;
    const int pl = (int)(t / per_plane);
    const int64_t r = t - pl * per_plane;
    const int i = (int)(r / chunks), c = (int)(r % chunks);
    const bool bottom = i >= a.my;
    const int yd = bottom ? a.lines + (i - a.my) : -1 - i;
    const int ys = bottom ? a.lines - 1 : 0;
    const P* base = (const P*)a.planes + a.plane_off[pl] - a.mx;
    const P* s = base + ys * a.ls + c * C;
    P* d = (P*)a.planes + a.plane_off[pl] - a.mx + yd * a.ls + c * C;
    if ((c + 1) * C <= a.ls)
    {
        if constexpr (sizeof(P) == 1) stu<uint4>(d, ldu<uint4>(s));
        else
        {
            stu<uint4>(d, ldu<uint4>(s));
            stu<uint4>(d + 8, ldu<uint4>(s + 8));
        }
    }
    else
        for (int x = 0; x < a.ls - c * C; x++) d[x] = s[x];
}

// ---------------------------------------------------------------- intra estimate
struct LowresIntraArgs
{
    const void* planes;
    const int64_t* plane_off;     // per frame: lowresPlane[0]
    int64_t ls;
    const int32_t* inv_q;
    int32_t* intra_cost;
    uint8_t* intra_mode;
    uint16_t* lowres_cost;
    int32_t* row_satd;
    int64_t* cost_est;
    int n, wcu, hcu, maxv, penalty;
};

// Hadamard 4x4 (any butterfly order: only the |.| sum is used)
__device__ __forceinline__ void had4(int& a, int& b, int& c, int& d)
{
    const int s0 = a + b, s1 = a - b, s2 = c + d, s3 = c - d;
    a = s0 + s2; b = s1 + s3; c = s0 - s2; d = s1 - s3;
}

// satd 8x8 of fenc - pred: sum of the four 4x4 SATDs (each raw 4x4 sum is
// even, so one final >> 1 equals satd8's per-8x4 halving, SURVEY note a7)
template <typename P>
__device__ __forceinline__ int satd8(const PixRow<P, 8> (&fe)[8], const int (&v)[8][8], bool tr)
{
    int sum = 0;
#pragma unroll
    for (int qy = 0; qy < 8; qy += 4)
#pragma unroll
        for (int qx = 0; qx < 8; qx += 4)
        {
            int d[4][4];
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int c = 0; c < 4; c++)
                    d[r][c] = fe[qy + r].get(qx + c) - (tr ? v[qx + c][qy + r] : v[qy + r][qx + c]);
#pragma unroll
            for (int r = 0; r < 4; r++) had4(d[r][0], d[r][1], d[r][2], d[r][3]);
#pragma unroll
            for (int c = 0; c < 4; c++)
            {
                had4(d[0][c], d[1][c], d[2][c], d[3][c]);
#pragma unroll
                for (int r = 0; r < 4; r++) sum += d[r][c] < 0 ? -d[r][c] : d[r][c];
            }
        }
    return sum >> 1;
}

template <typename P>
__device__ __forceinline__ int lowres_mode_cost(int m, const int (&smp)[33], const int (&flt)[33],
                                                const PixRow<P, 8> (&fe)[8], int maxv, uint32_t (*D)[X265AMD_BLOCK])
{
    // DC: raw samples with the edge filter; planar: filtered samples, no edge filter;
    // angular: g_intraFilterFlags[mode] & 8 selects the filtered samples, edge filter on (N <= 16)
    const bool use_flt = m == 0 || (m >= 2 && (c_intra.filter_flags[m] & 8));
    int nb[33];
#pragma unroll
    for (int i = 0; i < 33; i++) nb[i] = use_flt ? flt[i] : smp[i];
    int v[8][8];
    const ModeInfo mi = intra_lane_predict<8>(nb, m, m != 0, maxv, D, v);
    return satd8<P>(fe, v, mi.hor);
}

template <typename P>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_lowres_intra(const LowresIntraArgs a)
{
    __shared__ uint32_t D[24][X265AMD_BLOCK];          // intra_lane_predict's per-lane LDS column (3N, N = 8)
    const int lane = threadIdx.x & 7;
    const int ncu = a.wcu * a.hcu;
    const int64_t g = ((int64_t)xcd_block() * X265AMD_BLOCK + threadIdx.x) >> 3;
    if (g >= (int64_t)a.n * ncu) return;                // whole 8-lane groups
    const int f = (int)(g / ncu), xy = (int)(g % ncu);
    const int cx = xy % a.wcu, cy = xy / a.wcu;
    const P* cur = (const P*)a.planes + a.plane_off[f] + 8 * cx + 8 * cy * a.ls;

    PixRow<P, 8> fe[8];
#pragma unroll
    for (int y = 0; y < 8; y++) fe[y].load(cur + y * a.ls);
    // reference samples (slicetype.cpp:262-266): top-left + 16 above, then 16 left
    int smp[33], flt[33];
    {
        int t[16];
        load_row<P, 16>(cur - a.ls - 1, t);
#pragma unroll
        for (int i = 0; i < 16; i++) smp[i] = t[i];
        smp[16] = cur[-a.ls + 15];
#pragma unroll
        for (int i = 1; i <= 16; i++) smp[16 + i] = cur[(i - 1) * a.ls - 1];
    }
    // intraFilter<8> (intrapred.cpp:31-51)
#pragma unroll
    for (int i = 1; i < 16; i++) flt[i] = ((smp[i] << 1) + smp[i - 1] + smp[i + 1] + 2) >> 2;
    flt[16] = smp[16];
    flt[0] = ((smp[0] << 1) + smp[1] + smp[17] + 2) >> 2;
    flt[17] = ((smp[17] << 1) + smp[0] + smp[18] + 2) >> 2;
#pragma unroll
    for (int i = 18; i < 32; i++) flt[i] = ((smp[i] << 1) + smp[i - 1] + smp[i + 1] + 2) >> 2;
    flt[32] = smp[32];

    // pass 1: DC, planar, angular 5, 10, ..., 30 — one per lane
    const int m1 = lane == 0 ? 1 : lane == 1 ? 0 : 5 * (lane - 1);
    const int c1 = lowres_mode_cost<P>(m1, smp, flt, fe, a.maxv, D);
    const int gbase = threadIdx.x & ~7;
    int icost = __shfl(c1, gbase + 0, 64), imode = 1;                        // DC first
    const int cpl = __shfl(c1, gbase + 1, 64);
    if (cpl < icost) { icost = cpl; imode = 0; }
    int acost = 0x7fffffff, amode = 4;
#pragma unroll
    for (int k = 2; k < 8; k++)
    {
        const int c = __shfl(c1, gbase + k, 64);
        if (c < acost) { acost = c; amode = 5 * (k - 1); }
    }
    // passes 2 and 3: best -+ 2, then best -+ 1 (minus first), on lanes 0 / 1
#pragma unroll
    for (int dist = 2; dist >= 1; dist--)
    {
        const int lo = amode - dist, hi = amode + dist;
        const int c = lowres_mode_cost<P>(lane & 1 ? hi : lo, smp, flt, fe, a.maxv, D);
        const int clo = __shfl(c, gbase + 0, 64), chi = __shfl(c, gbase + 1, 64);
        if (clo < acost) { acost = clo; amode = lo; }
        if (chi < acost) { acost = chi; amode = hi; }
    }
    if (acost < icost) { icost = acost; imode = amode; }
    icost += a.penalty;

    if (lane == 0)
    {
        const int64_t o = (int64_t)f * ncu + xy;
        a.intra_cost[o] = icost;
        a.intra_mode[o] = (uint8_t)imode;
        a.lowres_cost[o] = (uint16_t)(icost < 0x3fff ? icost : 0x3fff);   // LOWRES_COST_MASK, shift 0
        const bool scored = (cx > 0 && cx < a.wcu - 1 && cy > 0 && cy < a.hcu - 1) || a.wcu <= 2 || a.hcu <= 2;
        const int icost_aq = (scored && a.inv_q) ? ((icost * a.inv_q[o] + 128) >> 8) : icost;
        // integer sums: order-independent, so atomics reproduce the serial totals
        atomicAdd(&a.row_satd[(int64_t)f * a.hcu + cy], icost_aq);
        if (scored)
        {
            atomicAdd((unsigned long long*)&a.cost_est[2 * f], (unsigned long long)(int64_t)icost);
            atomicAdd((unsigned long long*)&a.cost_est[2 * f + 1], (unsigned long long)(int64_t)icost_aq);
        }
    }
}

template <typename P>
static int launch_lowres_init(const LowresArgs& a, hipStream_t st)
{
    const int64_t core = (int64_t)a.n * a.lines * (a.width / 4);
    hipLaunchKernelGGL((k_lowres_core<P>), dim3((uint32_t)((core + X265AMD_BLOCK - 1) / X265AMD_BLOCK)),
                       dim3(X265AMD_BLOCK), 0, st, a);
    const int64_t lr = 2 * (int64_t)a.n * 4 * a.lines;
    hipLaunchKernelGGL((k_lowres_extend_lr<P>), dim3((uint32_t)((lr + X265AMD_BLOCK - 1) / X265AMD_BLOCK)),
                       dim3(X265AMD_BLOCK), 0, st, a);
    if (a.my > 0)
    {
        const int64_t tb = (int64_t)a.n * 4 * 2 * a.my * ((a.ls + 15) / 16);
        hipLaunchKernelGGL((k_lowres_extend_tb<P>), dim3((uint32_t)((tb + X265AMD_BLOCK - 1) / X265AMD_BLOCK)),
                           dim3(X265AMD_BLOCK), 0, st, a);
    }
    return (int)hipGetLastError();
}

} // namespace x265amd

using namespace x265amd;

extern "C" int x265amd_lowres_init(int depth, const x265amd_lowres_batch* b, void* stream)
{
    if ((depth != 8 && depth != 10 && depth != 12) || !b) return X265AMD_EINVAL;
    if (b->n < 0 || b->width <= 0 || b->lines <= 0 || (b->width & 7) || (b->lines & 7) || b->margin_x < 0 ||
        b->margin_y < 0 || b->lowres_stride < b->width + 2 * b->margin_x)
        return X265AMD_EINVAL;
    if (!b->n) return 0;
    if (!b->src || !b->src_off || !b->planes || !b->plane_off) return X265AMD_EINVAL;
    LowresArgs a{ b->src, b->src_off, (int64_t)b->src_stride, b->planes, b->plane_off, (int64_t)b->lowres_stride,
                  b->n, b->width, b->lines, b->margin_x, b->margin_y };
    hipStream_t st = (hipStream_t)stream;
    return depth == 8 ? launch_lowres_init<uint8_t>(a, st) : launch_lowres_init<uint16_t>(a, st);
}

extern "C" int x265amd_lowres_intra(int depth, const x265amd_lowres_intra_batch* b, void* stream)
{
    if ((depth != 8 && depth != 10 && depth != 12) || !b) return X265AMD_EINVAL;
    if (b->n < 0 || b->width_cu <= 0 || b->height_cu <= 0) return X265AMD_EINVAL;
    if (!b->n) return 0;
    if (!b->planes || !b->plane_off || !b->intra_cost || !b->intra_mode || !b->lowres_cost || !b->row_satd ||
        !b->cost_est)
        return X265AMD_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    // the row and frame sums are accumulated: start them at zero (slicetype.cpp:253, 327-328)
    hipError_t e = hipMemsetAsync(b->row_satd, 0, sizeof(int32_t) * (size_t)b->n * b->height_cu, st);
    if (e == hipSuccess) e = hipMemsetAsync(b->cost_est, 0, sizeof(int64_t) * 2 * (size_t)b->n, st);
    if (e != hipSuccess) return (int)e;
    // (int)x265_lambda_tab[X265_LOOKAHEAD_QP] with X265_LOOKAHEAD_QP = 12 + QP_BD_OFFSET
    // (common.h:208, constants.cpp:31-151): 1 / 16 / 256 at 8 / 10 / 12 bits
    const int lambda = depth == 8 ? 1 : depth == 10 ? 16 : 256;
    LowresIntraArgs a{ b->planes, b->plane_off, (int64_t)b->lowres_stride, b->inv_qscale, b->intra_cost,
                       b->intra_mode, b->lowres_cost, b->row_satd, b->cost_est, b->n, b->width_cu, b->height_cu,
                       (1 << depth) - 1, 5 * lambda + 4 };
    const int64_t threads = (int64_t)b->n * b->width_cu * b->height_cu * 8;
    const uint32_t blocks = (uint32_t)((threads + X265AMD_BLOCK - 1) / X265AMD_BLOCK);
    if (depth == 8) hipLaunchKernelGGL((k_lowres_intra<uint8_t>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, a);
    else hipLaunchKernelGGL((k_lowres_intra<uint16_t>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, a);
    return (int)hipGetLastError();
}
