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
    // a masked blend, kept opaque: a plain `use_flt ? flt[i] : smp[i]` is
    // rewritten into a select of the two arrays' addresses, which puts both
    // arrays in scratch
    int mk = use_flt ? -1 : 0;
    asm volatile("" : "+v"(mk));
    int nb[33];
#pragma unroll
    for (int i = 0; i < 33; i++) nb[i] = smp[i] ^ ((smp[i] ^ flt[i]) & mk);
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
    const int64_t total = (int64_t)a.n * ncu;
    const int64_t graw = ((int64_t)xcd_block() * X265AMD_BLOCK + threadIdx.x) >> 3;
    const bool valid = graw < total;                    // whole 8-lane groups; the wave stays
    const int64_t g = valid ? graw : total - 1;         // converged for the sums below
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

    const int64_t o = (int64_t)f * ncu + xy;
    if (lane == 0 && valid)
    {
        a.intra_cost[o] = icost;
        a.intra_mode[o] = (uint8_t)imode;
        a.lowres_cost[o] = (uint16_t)(icost < 0x3fff ? icost : 0x3fff);   // LOWRES_COST_MASK, shift 0
    }
    const bool scored = (cx > 0 && cx < a.wcu - 1 && cy > 0 && cy < a.hcu - 1) || a.wcu <= 2 || a.hcu <= 2;
    const int icost_aq = (scored && a.inv_q) ? ((icost * a.inv_q[o] + 128) >> 8) : icost;

    // integer sums: order-independent, so atomics reproduce the serial totals.
    // The wave's eight CUs are consecutive: when they share a frame (and a
    // row) one atomic per wave replaces eight contended ones.
    const bool lead = lane == 0 && valid;
    int r_aq = lead ? icost_aq : 0;
    int s_c = lead && scored ? icost : 0, s_aq = lead && scored ? icost_aq : 0;
#pragma unroll
    for (int m = 8; m < 64; m <<= 1)
    {
        r_aq += __shfl_xor(r_aq, m, 64);
        s_c += __shfl_xor(s_c, m, 64);
        s_aq += __shfl_xor(s_aq, m, 64);
    }
    const int wl = threadIdx.x & 63;
    const int row_key = f * a.hcu + cy;
    const int f0 = __shfl(f, 0, 64), f7 = __shfl(f, 56, 64);
    const int k0 = __shfl(row_key, 0, 64), k7 = __shfl(row_key, 56, 64);
    if (k0 == k7 ? wl == 0 : lead)
        atomicAdd(&a.row_satd[row_key], k0 == k7 ? r_aq : icost_aq);
    if (f0 == f7)
    {
        if (wl == 0)
        {
            atomicAdd((unsigned long long*)&a.cost_est[2 * f], (unsigned long long)(int64_t)s_c);
            atomicAdd((unsigned long long*)&a.cost_est[2 * f + 1], (unsigned long long)(int64_t)s_aq);
        }
    }
    else if (lead && scored)
    {
        atomicAdd((unsigned long long*)&a.cost_est[2 * f], (unsigned long long)(int64_t)icost);
        atomicAdd((unsigned long long*)&a.cost_est[2 * f + 1], (unsigned long long)(int64_t)icost_aq);
    }
}

// ---------------------------------------------------------------- P-frame cost estimate
// CostEstimateGroup::estimateFrameCost for a P estimate (b == p1, list 0 only;
// slicetype.cpp:1977-2066) = estimateCUCost (slicetype.cpp:2068-2225) for every
// 8x8 lowres CU: the MVP is the candidate of the right / below / below-left /
// below-right neighbours (already searched) with the lowest SATD, then
// MotionEstimate::motionEstimate's lowres HEX search with sub-pel refine at
// subme 1 (motion.cpp:571-1172), then the inter / intra decision.
//
// The neighbour dependency (right and the row below, CUs visited bottom-up and
// right to left within each coop slice) makes a wavefront: with x' = W-1-cx and
// y' = (slice's last row) - cy, CU (x', y') only needs CUs of steps before
// x' + 2 y'.  One workgroup owns one (estimate, slice), with a 4-lane quad per
// row of the slice (up to 16 wavefronts, a barrier per step); quad g owns rows
// y' = g, g + nquads, ... and at step t searches CU x' = t - 2 y' of each.  The
// motion search runs on the quad, exactly in the reference's order: each lane
// scores its 4x4 quadrant of every candidate on packed 8-bit (v_sad_u8) /
// 16-bit (v_sad_u16) rows and the quad sums by DPP, so a step's dependent
// chain of candidate rounds costs a quarter of the instructions of a
// lane-per-CU search; the four MVs a row needs from the row below live in a
// 4-entry LDS ring per row.
constexpr int kPcostMaxRows = 512;

struct PcostArgs
{
    const void* planes;
    int64_t ls;
    const int64_t* fenc_off;      // per estimate: lowresPlane[0] of b
    const int64_t* ref_off;       // 4 per estimate: lowresPlane[0..3] of p0
    const int32_t* intra_cost;
    const int32_t* inv_q;
    const uint16_t* mvcost;       // BitCost table centre (difference 0)
    int16_t* mvs;
    int32_t* mv_costs;
    uint16_t* lowres_costs;
    int32_t* row_satd;
    int64_t* cost_est;
    int32_t* intra_mbs;
    int n, wcu, hcu, rps, nslices;
};

// A CU's search runs on a 4-lane group (a quad): lane q owns the 4x4 quadrant (x 4(q & 1),
// y 4(q >> 1)) of the 8x8 block, evaluates its quadrant of every candidate (SAD on packed rows,
// or one 4x4 Hadamard) and the quad sums by two DPP quad_perm adds, so every lane of the group
// holds the same cost and takes the same decisions, in the reference's order.
template <typename P>
struct Quad
{
    static constexpr int W = (int)sizeof(P);     // dwords per 4-pixel row
    uint32_t r[4][W];
    __device__ __forceinline__ void load(const P* p, int64_t ls)
    {
#pragma unroll
        for (int y = 0; y < 4; y++)
        {
            if constexpr (W == 1) r[y][0] = ldu<uint32_t>(p + y * ls);
            else { const uint2 v = ldu<uint2>(p + y * ls); r[y][0] = v.x; r[y][1] = v.y; }
        }
    }
    __device__ __forceinline__ int get(int y, int x) const
    {
        if constexpr (W == 1) return (int)((r[y][0] >> (8 * x)) & 0xff);
        else return (int)((r[y][x >> 1] >> (16 * (x & 1))) & 0xffff);
    }
};

__device__ __forceinline__ int quad_sum(int v)
{
    v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);   // quad_perm [1, 0, 3, 2]
    v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);   // quad_perm [2, 3, 0, 1]
    return v;
}

template <typename P>
__device__ __forceinline__ uint32_t sad_packed(uint32_t a, uint32_t b, uint32_t acc)
{
    if constexpr (sizeof(P) == 1) return __builtin_amdgcn_sad_u8(a, b, acc);
    else return __builtin_amdgcn_sad_u16(a, b, acc);
}

template <typename P>
__device__ __forceinline__ int sad_quad(const Quad<P>& fe, const Quad<P>& b)
{
    uint32_t s = 0;
#pragma unroll
    for (int y = 0; y < 4; y++)
#pragma unroll
        for (int w = 0; w < Quad<P>::W; w++) s = sad_packed<P>(fe.r[y][w], b.r[y][w], s);
    return quad_sum((int)s);
}

// SAD of the CU against the full-pel block at p (the lane's quadrant origin)
template <typename P>
__device__ __forceinline__ int sad8_mem(const Quad<P>& fe, const P* p, int64_t ls)
{
    Quad<P> b;
    b.load(p, ls);
    return sad_quad<P>(fe, b);
}

// satd 8x8 = (sum of the four raw 4x4 Hadamard sums) >> 1 (each raw sum is even, so this equals
// satd8's per-8x4 halving, SURVEY note a7)
template <typename P>
__device__ __forceinline__ int satd_quad(const Quad<P>& fe, const Quad<P>& b)
{
    int d[4][4];
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int c = 0; c < 4; c++) d[r][c] = fe.get(r, c) - b.get(r, c);
#pragma unroll
    for (int r = 0; r < 4; r++) had4(d[r][0], d[r][1], d[r][2], d[r][3]);
    int sum = 0;
#pragma unroll
    for (int c = 0; c < 4; c++)
    {
        had4(d[0][c], d[1][c], d[2][c], d[3][c]);
#pragma unroll
        for (int r = 0; r < 4; r++) sum += d[r][c] < 0 ? -d[r][c] : d[r][c];
    }
    return quad_sum(sum) >> 1;
}

// ReferencePlanes::lowresMC (lowres.h:57-80): the block at quarter-pel q, the rounded average of
// two half-pel planes when q is a quarter position (ref[] = the lane's quadrant origins)
template <typename P>
__device__ __forceinline__ void qpel_block(const P* const (&ref)[4], int64_t ls, int qx, int qy, Quad<P>& out)
{
    const int ha = (qy & 2) | ((qx & 2) >> 1);
    out.load(ref[ha] + (qx >> 2) + (qy >> 2) * ls, ls);
    if ((qx | qy) & 1)
    {
        const int bx = qx + (qx & 1), by = qy + (qy & 1);
        const int hb = (by & 2) | ((bx & 2) >> 1);
        Quad<P> b;
        b.load(ref[hb] + (bx >> 2) + (by >> 2) * ls, ls);
        constexpr uint32_t M = sizeof(P) == 1 ? 0x7f7f7f7fu : 0x7fff7fffu;
#pragma unroll
        for (int y = 0; y < 4; y++)
#pragma unroll
            for (int w = 0; w < Quad<P>::W; w++)
            {
                const uint32_t x = out.r[y][w], z = b.r[y][w];
                out.r[y][w] = (x | z) - (((x ^ z) >> 1) & M);     // (a + b + 1) >> 1 per element
            }
    }
}

template <typename P>
__device__ __forceinline__ int qpel_cost(const Quad<P>& fe, const P* const (&ref)[4], int64_t ls, int qx, int qy,
                                         bool satd)
{
    Quad<P> b;
    qpel_block<P>(ref, ls, qx, qy, b);
    return satd ? satd_quad<P>(fe, b) : sad_quad<P>(fe, b);
}

struct MvCost
{
    const uint16_t* tab;
    int px, py;
    __device__ __forceinline__ int operator()(int qx, int qy) const
    {
        return (uint16_t)(tab[qx - px] + tab[qy - py]);
    }
};

// MotionEstimate::motionEstimate, lowres reference, HEX search, subme 1 (motion.cpp:571-1172)
template <typename P>
__device__ int me_lowres(const Quad<P>& fe, const P* const (&ref)[4], int64_t ls, const MvCost& mc, int minx,
                         int miny, int maxx, int maxy, int mvpx, int mvpy, int& outx, int& outy)
{
    const int pmx = mvpx > 4 * maxx ? 4 * maxx : (mvpx < 4 * minx ? 4 * minx : mvpx);
    const int pmy = mvpy > 4 * maxy ? 4 * maxy : (mvpy < 4 * miny ? 4 * miny : mvpy);
    const int bprecost = qpel_cost<P>(fe, ref, ls, pmx, pmy, false);          // no MV cost (motion.cpp:606)
    int bx = (pmx + 2) >> 2, by = (pmy + 2) >> 2;
    int bcost = bprecost;
    const P* f0 = ref[0];
    if ((pmx | pmy) & 3) bcost = sad8_mem<P>(fe, f0 + bx + by * ls, ls) + mc(4 * bx, 4 * by);
    if (pmx | pmy)
    {
        const int c = sad8_mem<P>(fe, f0, ls) + mc(0, 0);
        if (c < bcost) { bcost = c; bx = by = 0; }
    }
    auto cand = [&](int dx, int dy) {
        return sad8_mem<P>(fe, f0 + (bx + dx) + (by + dy) * ls, ls) + mc(4 * (bx + dx), 4 * (by + dy));
    };
    {
        int c0 = cand(-2, 0), c1 = cand(-1, 2), c2 = cand(1, 2);
        bcost <<= 3;
        if ((c0 << 3) + 2 < bcost) bcost = (c0 << 3) + 2;
        if ((c1 << 3) + 3 < bcost) bcost = (c1 << 3) + 3;
        if ((c2 << 3) + 4 < bcost) bcost = (c2 << 3) + 4;
        c0 = cand(2, 0); c1 = cand(1, -2); c2 = cand(-1, -2);
        if ((c0 << 3) + 5 < bcost) bcost = (c0 << 3) + 5;
        if ((c1 << 3) + 6 < bcost) bcost = (c1 << 3) + 6;
        if ((c2 << 3) + 7 < bcost) bcost = (c2 << 3) + 7;
        if (bcost & 7)
        {
            int dir = (bcost & 7) - 2;
            bx += hex_dx(dir + 1); by += hex_dy(dir + 1);
            for (int i = (16 >> 1) - 1; i > 0 && bx >= minx && bx <= maxx && by >= miny && by <= maxy; i--)
            {
                c0 = cand(hex_dx(dir), hex_dy(dir));
                c1 = cand(hex_dx(dir + 1), hex_dy(dir + 1));
                c2 = cand(hex_dx(dir + 2), hex_dy(dir + 2));
                bcost &= ~7;
                if ((c0 << 3) + 1 < bcost) bcost = (c0 << 3) + 1;
                if ((c1 << 3) + 2 < bcost) bcost = (c1 << 3) + 2;
                if ((c2 << 3) + 3 < bcost) bcost = (c2 << 3) + 3;
                if (!(bcost & 7)) break;
                dir += (bcost & 7) - 2;
                dir = dir < 0 ? dir + 6 : (dir > 5 ? dir - 6 : dir);   // mod6m1[dir + 1] = dir mod 6
                bx += hex_dx(dir + 1); by += hex_dy(dir + 1);
            }
        }
        bcost >>= 3;
        int sdir = 0;
#pragma unroll
        for (int k = 1; k <= 8; k++)
        {
            const int c = cand(sq_dx(k), sq_dy(k));
            if (c < bcost) { bcost = c; sdir = k; }
        }
        bx += sq_dx(sdir); by += sq_dy(sdir);
    }
    int qx, qy;
    if (bprecost < bcost) { qx = pmx; qy = pmy; bcost = bprecost; }
    else { qx = 4 * bx; qy = 4 * by; }
    if (!bcost)
        bcost = mc(qx, qy);
    else
    {
        int bdir = 0;
#pragma unroll
        for (int k = 1; k <= 4; k++)
        {
            const int c = qpel_cost<P>(fe, ref, ls, qx + 2 * sq_dx(k), qy + 2 * sq_dy(k), false) + mc(qx + 2 * sq_dx(k), qy + 2 * sq_dy(k));
            if (c < bcost) { bcost = c; bdir = k; }
        }
        qx += 2 * sq_dx(bdir); qy += 2 * sq_dy(bdir);
        bcost = qpel_cost<P>(fe, ref, ls, qx, qy, true) + mc(qx, qy);
        bdir = 0;
#pragma unroll
        for (int k = 1; k <= 4; k++)
        {
            const int c = qpel_cost<P>(fe, ref, ls, qx + sq_dx(k), qy + sq_dy(k), true) + mc(qx + sq_dx(k), qy + sq_dy(k));
            if (c < bcost) { bcost = c; bdir = k; }
        }
        qx += sq_dx(bdir); qy += sq_dy(bdir);
    }
    outx = qx;
    outy = qy;
    return bcost;
}

// one workgroup per (estimate, coop slice) of nw wavefronts (enough quads for the slice's rows,
// up to 16 wavefronts); quad g = threadIdx.x >> 2 owns rows y' = g, g + 16 nw, ...
template <typename P>
__global__ __launch_bounds__(1024) void k_lowres_pcost(const PcostArgs a)
{
    __shared__ uint32_t ring[kPcostMaxRows][4];   // per row: MVs of its last four CUs (x' & 3), packed x | y << 16
    __shared__ int32_t rowsum[kPcostMaxRows];
    const int tid = threadIdx.x, lane = tid & 63, g = tid >> 2, q = tid & 3, nq = blockDim.x >> 2;
    const bool lead = q == 0;
    const int e = blockIdx.x / a.nslices, sl = blockIdx.x % a.nslices;
    const int first = a.rps * sl;
    const int last = sl == a.nslices - 1 ? a.hcu - 1 : a.rps * (sl + 1) - 1;
    const int R = last - first + 1, W = a.wcu;
    const int ncu = W * a.hcu;
    const P* planes = (const P*)a.planes;
    const int64_t ls = a.ls;
    const int64_t qoff = 4 * (q & 1) + 4 * (q >> 1) * ls;   // the lane's quadrant
    const P* fenc0 = planes + a.fenc_off[e] + qoff;
    const P* const rbase[4] = { planes + a.ref_off[4 * e] + qoff, planes + a.ref_off[4 * e + 1] + qoff,
                                planes + a.ref_off[4 * e + 2] + qoff, planes + a.ref_off[4 * e + 3] + qoff };
    const int64_t cub = (int64_t)e * ncu;
    for (int y = tid; y < R; y += blockDim.x) rowsum[y] = 0;
    __syncthreads();
    int64_t est = 0, est_aq = 0;
    int mbs = 0;
    const int steps = W + 2 * (R - 1);
    for (int t = 0; t < steps; t++)
    {
        for (int yp = g; yp < R; yp += nq)
        {
            const int xp = t - 2 * yp;
            if (xp < 0 || xp >= W) continue;
            const int cx = W - 1 - xp, cy = last - yp;
            const int xy = cx + cy * W;
            const int64_t off = 8 * cx + 8 * (int64_t)cy * ls;
            Quad<P> fe;
            fe.load(fenc0 + off, ls);
            const P* const ref[4] = { rbase[0] + off, rbase[1] + off, rbase[2] + off, rbase[3] + off };
            // MVP: right, below, below-left, below-right (slicetype.cpp:2116-2150)
            int candx[4], candy[4], numc = 0;
            if (cx < W - 1) { const uint32_t m = ring[yp][(xp - 1) & 3]; candx[numc] = (int16_t)m; candy[numc++] = (int16_t)(m >> 16); }
            if (yp > 0)
            {
                const uint32_t mb = ring[yp - 1][xp & 3];
                candx[numc] = (int16_t)mb; candy[numc++] = (int16_t)(mb >> 16);
                if (cx > 0) { const uint32_t m = ring[yp - 1][(xp + 1) & 3]; candx[numc] = (int16_t)m; candy[numc++] = (int16_t)(m >> 16); }
                if (cx < W - 1) { const uint32_t m = ring[yp - 1][(xp - 1) & 3]; candx[numc] = (int16_t)m; candy[numc++] = (int16_t)(m >> 16); }
            }
            int mvpx = 0, mvpy = 0;
            if (numc)
            {
                int best = 1 << 28;                                  // MotionEstimate::COST_MAX
                for (int i = 0; i < numc; i++)
                {
                    const int c = qpel_cost<P>(fe, ref, ls, candx[i], candy[i], true);
                    if (c < best) { best = c; mvpx = candx[i]; mvpy = candy[i]; }
                }
            }
            const MvCost mc{ a.mvcost, mvpx, mvpy };
            int ox, oy;
            const int fcost = me_lowres<P>(fe, ref, ls, mc, -cx * 8 - 8, -cy * 8 - 8, (W - cx - 1) * 8 + 8,
                                           (a.hcu - cy - 1) * 8 + 8, mvpx, mvpy, ox, oy);
            int bcost = 1 << 28, listused = 0;
            if (fcost < bcost) { bcost = fcost; listused = 1; }
            bcost += 4;                                              // lowresPenalty
            const int ic = a.intra_cost[cub + xy];
            if (ic < bcost) { bcost = ic; listused = 0; }
            const bool scored = (cx > 0 && cx < W - 1 && cy > 0 && cy < a.hcu - 1) || W <= 2 || a.hcu <= 2;
            const int bcost_aq = (scored && a.inv_q) ? ((bcost * a.inv_q[cub + xy] + 128) >> 8) : bcost;
            if (lead)
            {
                ring[yp][xp & 3] = (uint32_t)(uint16_t)ox | ((uint32_t)(uint16_t)oy << 16);
                a.mvs[2 * (cub + xy)] = (int16_t)ox;
                a.mvs[2 * (cub + xy) + 1] = (int16_t)oy;
                a.mv_costs[cub + xy] = fcost;
                if (scored) { est += bcost; est_aq += bcost_aq; mbs += !listused; }
                rowsum[yp] += bcost_aq;
                a.lowres_costs[cub + xy] = (uint16_t)((bcost < 0x3fff ? bcost : 0x3fff) | (listused << 14));
            }
        }
        __syncthreads();
    }
    for (int yp = tid; yp < R; yp += blockDim.x) a.row_satd[(int64_t)e * a.hcu + last - yp] = rowsum[yp];
    // slice totals into the estimate's (integer sums: order-independent)
    est = (int64_t)group_sum64<64>((uint64_t)est);
    est_aq = (int64_t)group_sum64<64>((uint64_t)est_aq);
    mbs = group_sum<64>(mbs);
    if (lane == 0)
    {
        atomicAdd((unsigned long long*)&a.cost_est[2 * e], (unsigned long long)est);
        atomicAdd((unsigned long long*)&a.cost_est[2 * e + 1], (unsigned long long)est_aq);
        atomicAdd(&a.intra_mbs[e], mbs);
    }
}

// ---------------------------------------------------------------- B-frame cost estimate
// estimateCUCost with bBidir (p0 < b < p1, slicetype.cpp:2068-2225): per list i with bDoSearch[i]
// the MVP choice (and the skipCost of a zero MVP), the lowres HEX search from p0 (list 0) or p1
// (list 1) and the zero-MV skip override; a list not searched reuses its stored cost and MV; then
// the bidir average of the two lists' predictions and the co-located average, scored by SATD.
// Same wavefront schedule as the P estimate, one MV ring per list.
struct BcostArgs
{
    const void* planes;
    int64_t ls;
    const int64_t* fenc_off;      // per estimate: lowresPlane[0] of b
    const int64_t* ref_off[2];    // 4 per estimate: lowresPlane[0..3] of p0 / p1
    const uint8_t* do_search;     // 2 per estimate
    const int32_t* inv_q;
    const uint16_t* mvcost;
    int16_t* mvs[2];
    int32_t* mv_costs[2];
    uint16_t* lowres_costs;
    int32_t* row_satd;
    int64_t* cost_est;
    int n, wcu, hcu, rps, nslices;
};

// Two quads per CU (8 lanes): quad li searches list li, the two run concurrently and exchange
// their MV and cost by a lane ^ 4 swizzle; then quad 0 scores the bidir average and quad 1 the
// co-located average, and both apply the reference's decision order.
template <typename P>
__global__ __launch_bounds__(1024) void k_lowres_bcost(const BcostArgs a)
{
    __shared__ uint32_t ring[2][kPcostMaxRows][4];
    __shared__ int32_t rowsum[kPcostMaxRows];
    const int tid = threadIdx.x, lane = tid & 63, g = tid >> 3, li = (tid >> 2) & 1, q = tid & 3;
    const int nq = blockDim.x >> 3;
    const bool lead = q == 0;
    const int e = blockIdx.x / a.nslices, sl = blockIdx.x % a.nslices;
    const int first = a.rps * sl;
    const int last = sl == a.nslices - 1 ? a.hcu - 1 : a.rps * (sl + 1) - 1;
    const int R = last - first + 1, W = a.wcu;
    const int ncu = W * a.hcu;
    const P* planes = (const P*)a.planes;
    const int64_t ls = a.ls;
    const int64_t qoff = 4 * (q & 1) + 4 * (q >> 1) * ls;   // the lane's quadrant
    const P* fenc0 = planes + a.fenc_off[e] + qoff;
    const P* rb[2][4];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int k = 0; k < 4; k++) rb[i][k] = planes + a.ref_off[i][4 * e + k] + qoff;
    const bool search = a.do_search[2 * e + li] != 0;
    int16_t* const mvs = a.mvs[li];
    int32_t* const mvc = a.mv_costs[li];
    const int64_t cub = (int64_t)e * ncu;
    for (int y = tid; y < R; y += blockDim.x) rowsum[y] = 0;
    __syncthreads();
    int64_t est = 0, est_aq = 0;
    // without a search in either list no CU depends on another (the MVPs are only for searching):
    // every CU of the slice in one flat pass instead of the slope-2 wavefront
    const bool wave = a.do_search[2 * e] || a.do_search[2 * e + 1];
    const int steps = wave ? W + 2 * (R - 1) : 1;
    for (int t = 0; t < steps; t++)
    {
        for (int it = g; it < (wave ? R : R * W); it += nq)
        {
            const int yp = wave ? it : it / W;
            const int xp = wave ? t - 2 * yp : it % W;
            if (xp < 0 || xp >= W) continue;
            const int cx = W - 1 - xp, cy = last - yp;
            const int xy = cx + cy * W;
            const int64_t off = 8 * cx + 8 * (int64_t)cy * ls;
            Quad<P> fe;
            fe.load(fenc0 + off, ls);
            // ---- this quad's list
            int cost, ox, oy;
            if (!search)
            {
                cost = mvc[cub + xy];
                ox = mvs[2 * (cub + xy)];
                oy = mvs[2 * (cub + xy) + 1];
            }
            else
            {
                const P* const ref[4] = { rb[li][0] + off, rb[li][1] + off, rb[li][2] + off, rb[li][3] + off };
                int candx[4], candy[4], numc = 0;
                if (cx < W - 1) { const uint32_t m = ring[li][yp][(xp - 1) & 3]; candx[numc] = (int16_t)m; candy[numc++] = (int16_t)(m >> 16); }
                if (yp > 0)
                {
                    const uint32_t mb = ring[li][yp - 1][xp & 3];
                    candx[numc] = (int16_t)mb; candy[numc++] = (int16_t)(mb >> 16);
                    if (cx > 0) { const uint32_t m = ring[li][yp - 1][(xp + 1) & 3]; candx[numc] = (int16_t)m; candy[numc++] = (int16_t)(m >> 16); }
                    if (cx < W - 1) { const uint32_t m = ring[li][yp - 1][(xp - 1) & 3]; candx[numc] = (int16_t)m; candy[numc++] = (int16_t)(m >> 16); }
                }
                int mvpx = 0, mvpy = 0, skip = 0x7fffffff;
                if (numc)
                {
                    int best = 1 << 28;                              // MotionEstimate::COST_MAX
                    for (int k = 0; k < numc; k++)
                    {
                        const int c = qpel_cost<P>(fe, ref, ls, candx[k], candy[k], true);
                        if (c < best) { best = c; mvpx = candx[k]; mvpy = candy[k]; }
                        if (!mvpx && !mvpy) skip = c;                // slicetype.cpp:2150-2151, as written
                    }
                }
                const MvCost mc{ a.mvcost, mvpx, mvpy };
                cost = me_lowres<P>(fe, ref, ls, mc, -cx * 8 - 8, -cy * 8 - 8, (W - cx - 1) * 8 + 8,
                                    (a.hcu - cy - 1) * 8 + 8, mvpx, mvpy, ox, oy);
                if (skip < 64 && skip < cost) { cost = skip; ox = oy = 0; }
                if (lead)
                {
                    ring[li][yp][xp & 3] = (uint32_t)(uint16_t)ox | ((uint32_t)(uint16_t)oy << 16);
                    mvs[2 * (cub + xy)] = (int16_t)ox;
                    mvs[2 * (cub + xy) + 1] = (int16_t)oy;
                    mvc[cub + xy] = cost;
                }
            }
            // ---- the other list's result (lane ^ 4 is the same quadrant of the partner quad)
            const int pcost = __shfl_xor(cost, 4, 64), pox = __shfl_xor(ox, 4, 64), poy = __shfl_xor(oy, 4, 64);
            const int c0 = li ? pcost : cost, c1 = li ? cost : pcost;
            const int m0x = li ? pox : ox, m0y = li ? poy : oy, m1x = li ? ox : pox, m1y = li ? oy : poy;
            int bcost = 1 << 28, listused = 0;
            if (c0 < bcost) { bcost = c0; listused = 1; }
            if (c1 < bcost) { bcost = c1; listused = 2; }
            // ---- bidir (quad 0): avg of the two lists' lowresMC blocks; co-located (quad 1): avg of the
            // full-pel planes (pixelavg_pp + bufSATD)
            constexpr uint32_t M = sizeof(P) == 1 ? 0x7f7f7f7fu : 0x7fff7fffu;
            const P* const r0[4] = { rb[0][0] + off, rb[0][1] + off, rb[0][2] + off, rb[0][3] + off };
            const P* const r1[4] = { rb[1][0] + off, rb[1][1] + off, rb[1][2] + off, rb[1][3] + off };
            Quad<P> b0, b1;
            if (li == 0)
            {
                qpel_block<P>(r0, ls, m0x, m0y, b0);
                qpel_block<P>(r1, ls, m1x, m1y, b1);
            }
            else
            {
                b0.load(r0[0], ls);
                b1.load(r1[0], ls);
            }
#pragma unroll
            for (int y = 0; y < 4; y++)
#pragma unroll
                for (int w = 0; w < Quad<P>::W; w++)
                {
                    const uint32_t x = b0.r[y][w], z = b1.r[y][w];
                    b0.r[y][w] = (x | z) - (((x ^ z) >> 1) & M);
                }
            const int mine = satd_quad<P>(fe, b0);
            const int other = __shfl_xor(mine, 4, 64);
            const int bi = li ? other : mine, co = li ? mine : other;
            if (bi < bcost) { bcost = bi; listused = 3; }
            if (co < bcost) { bcost = co; listused = 3; }
            bcost += 4;                                              // lowresPenalty
            const bool scored = (cx > 0 && cx < W - 1 && cy > 0 && cy < a.hcu - 1) || W <= 2 || a.hcu <= 2;
            const int bcost_aq = (scored && a.inv_q) ? ((bcost * a.inv_q[cub + xy] + 128) >> 8) : bcost;
            if (lead && li == 0)
            {
                if (scored) { est += bcost; est_aq += bcost_aq; }
                atomicAdd(&rowsum[yp], bcost_aq);           // flat pass: several groups per row
                a.lowres_costs[cub + xy] = (uint16_t)((bcost < 0x3fff ? bcost : 0x3fff) | (listused << 14));
            }
        }
        __syncthreads();
    }
    for (int yp = tid; yp < R; yp += blockDim.x) a.row_satd[(int64_t)e * a.hcu + last - yp] = rowsum[yp];
    est = (int64_t)group_sum64<64>((uint64_t)est);
    est_aq = (int64_t)group_sum64<64>((uint64_t)est_aq);
    if (lane == 0)
    {
        atomicAdd((unsigned long long*)&a.cost_est[2 * e], (unsigned long long)est);
        atomicAdd((unsigned long long*)&a.cost_est[2 * e + 1], (unsigned long long)est_aq);
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

extern "C" int x265amd_lowres_pcost(int depth, const x265amd_lowres_pcost_batch* b, void* stream)
{
    if ((depth != 8 && depth != 10 && depth != 12) || !b) return X265AMD_EINVAL;
    if (b->n < 0 || b->width_cu <= 0 || b->height_cu <= 0) return X265AMD_EINVAL;
    int rps = b->rows_per_slice, ns = b->num_slices;
    if (ns <= 1) { ns = 1; rps = b->height_cu; }
    if (rps <= 0 || (int64_t)rps * (ns - 1) >= b->height_cu) return X265AMD_EINVAL;
    if (b->height_cu - rps * (ns - 1) > kPcostMaxRows || rps > kPcostMaxRows) return X265AMD_EINVAL;
    if (!b->n) return 0;
    if (!b->planes || !b->fenc_off || !b->ref_off || !b->intra_cost || !b->mvcost || !b->mvs || !b->mv_costs ||
        !b->lowres_costs || !b->row_satd || !b->cost_est || !b->intra_mbs)
        return X265AMD_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    hipError_t err = hipMemsetAsync(b->cost_est, 0, sizeof(int64_t) * 2 * (size_t)b->n, st);
    if (err == hipSuccess) err = hipMemsetAsync(b->intra_mbs, 0, sizeof(int32_t) * (size_t)b->n, st);
    if (err != hipSuccess) return (int)err;
    PcostArgs a{ b->planes, (int64_t)b->lowres_stride, b->fenc_off, b->ref_off, b->intra_cost, b->inv_qscale,
                 b->mvcost, b->mvs, b->mv_costs, b->lowres_costs, b->row_satd, b->cost_est, b->intra_mbs, b->n,
                 b->width_cu, b->height_cu, rps, ns };
    const uint32_t blocks = (uint32_t)(b->n * ns);
    // enough 4-lane quads for the tallest slice, up to 16 wavefronts (rows beyond take turns)
    const int rmax = b->height_cu - rps * (ns - 1) > rps ? b->height_cu - rps * (ns - 1) : rps;
    int nw = (rmax + 15) / 16;
    nw = nw < 1 ? 1 : (nw > 16 ? 16 : nw);
    if (depth == 8) hipLaunchKernelGGL((k_lowres_pcost<uint8_t>), dim3(blocks), dim3(64 * nw), 0, st, a);
    else hipLaunchKernelGGL((k_lowres_pcost<uint16_t>), dim3(blocks), dim3(64 * nw), 0, st, a);
    return (int)hipGetLastError();
}

extern "C" int x265amd_lowres_bcost(int depth, const x265amd_lowres_bcost_batch* b, void* stream)
{
    if ((depth != 8 && depth != 10 && depth != 12) || !b) return X265AMD_EINVAL;
    if (b->n < 0 || b->width_cu <= 0 || b->height_cu <= 0) return X265AMD_EINVAL;
    int rps = b->rows_per_slice, ns = b->num_slices;
    if (ns <= 1) { ns = 1; rps = b->height_cu; }
    if (rps <= 0 || (int64_t)rps * (ns - 1) >= b->height_cu) return X265AMD_EINVAL;
    if (b->height_cu - rps * (ns - 1) > kPcostMaxRows || rps > kPcostMaxRows) return X265AMD_EINVAL;
    if (!b->n) return 0;
    if (!b->planes || !b->fenc_off || !b->ref0_off || !b->ref1_off || !b->do_search || !b->mvcost || !b->mvs0 ||
        !b->mv_costs0 || !b->mvs1 || !b->mv_costs1 || !b->lowres_costs || !b->row_satd || !b->cost_est)
        return X265AMD_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const hipError_t err = hipMemsetAsync(b->cost_est, 0, sizeof(int64_t) * 2 * (size_t)b->n, st);
    if (err != hipSuccess) return (int)err;
    BcostArgs a{ b->planes, (int64_t)b->lowres_stride, b->fenc_off, { b->ref0_off, b->ref1_off }, b->do_search,
                 b->inv_qscale, b->mvcost, { b->mvs0, b->mvs1 }, { b->mv_costs0, b->mv_costs1 }, b->lowres_costs,
                 b->row_satd, b->cost_est, b->n, b->width_cu, b->height_cu, rps, ns };
    const uint32_t blocks = (uint32_t)(b->n * ns);
    const int rmax = b->height_cu - rps * (ns - 1) > rps ? b->height_cu - rps * (ns - 1) : rps;
    int nw = (rmax + 7) / 8;                      // 8 lanes (two quads) per CU row
    nw = nw < 1 ? 1 : (nw > 16 ? 16 : nw);
    if (depth == 8) hipLaunchKernelGGL((k_lowres_bcost<uint8_t>), dim3(blocks), dim3(64 * nw), 0, st, a);
    else hipLaunchKernelGGL((k_lowres_bcost<uint16_t>), dim3(blocks), dim3(64 * nw), 0, st, a);
    return (int)hipGetLastError();
}

// ================================================================ f1 cuTree propagation
namespace x265amd {

// (int) of a double the way x86-64 cvttsd2si converts it (INT_MIN when out of range / NaN)
__device__ __forceinline__ int cvt_trunc_x86(double v)
{
    return (v > -2147483649.0 && v < 2147483648.0) ? (int)v : INT32_MIN;
}

// estimateCUPropagateCost (pixel.cpp:846-872), no FMA contraction: the reference's double
// multiply / add / divide sequence rounded step by step
__device__ __forceinline__ int propagate_amount(int in, int intra, int inter_raw, int invq, double fps)
{
    const int ic = inter_raw & ((1 << 14) - 1);
    const int inter = intra < ic ? intra : ic;
    const double pintra = (double)(int)((uint32_t)intra * (uint32_t)invq);
    const double amount = __dadd_rn((double)in, __dmul_rn(pintra, fps));
    const double r = __dadd_rn(__ddiv_rn(__dmul_rn(amount, (double)(intra - inter)), (double)intra), 0.5);
    return cvt_trunc_x86(r);
}

// one thread per CU: shares onto the reference frames' CUs, accumulated in int64
__global__ __launch_bounds__(X265AMD_BLOCK) void k_propagate(const x265amd_propagate_batch b)
{
    const int n = b.width_cu * b.height_cu;
    const int cu = (int)(blockIdx.x * X265AMD_BLOCK + threadIdx.x);
    if (cu >= n) return;
    const int in = b.propagate_in ? (int)b.propagate_in[cu] : 0;
    const int lc = (int)b.lowres_costs[cu];
    const int amount = propagate_amount(in, b.intra_cost[cu], lc, b.inv_qscale[cu], b.fps_factor / 256);
    if (amount <= 0) return;
    const int used = lc >> 14;
    const int bx = cu % b.width_cu, by = cu / b.width_cu;
    for (int l = 0; l < 2; l++)
    {
        // a list without MVs or without a reference cost array contributes nothing (a NULL list is
        // skipped, never dereferenced, even if a lowres cost claims it was used)
        if (!((used >> l) & 1) || !b.mvs[l] || !b.ref_costs[l]) continue;
        int la = amount;
        if (used == 3) la = (int)((uint32_t)la * (uint32_t)b.bipred_weight[l] + 32u) >> 6;
        unsigned long long* acc = (unsigned long long*)b.scratch + (size_t)l * n;
        const int32_t mv = b.mvs[l][cu];
        if (!mv)
        {
            atomicAdd(acc + cu, (unsigned long long)la);
            continue;
        }
        const int x = (int16_t)(mv & 0xffff), y = (int16_t)((uint32_t)mv >> 16);
        const int cux = (x >> 5) + bx, cuy = (y >> 5) + by, fx = x & 31, fy = y & 31;
#pragma unroll
        for (int k = 0; k < 4; k++)
        {
            const int dx = k & 1, dy = k >> 1;
            const int cx = cux + dx, cy = cuy + dy;
            if (cx < 0 || cy < 0 || cx >= b.width_cu || cy >= b.height_cu) continue;
            const int w = (dy ? fy : 32 - fy) * (dx ? fx : 32 - fx);
            const int share = (int)((uint32_t)la * (uint32_t)w + 512u) >> 10;
            atomicAdd(acc + cy * b.width_cu + cx, (unsigned long long)share);
        }
    }
}

// CLIP_ADD of the accumulated shares (order-free for non-negative shares)
__global__ __launch_bounds__(X265AMD_BLOCK) void k_propagate_finish(const x265amd_propagate_batch b)
{
    const int n = b.width_cu * b.height_cu;
    const int t = (int)(blockIdx.x * X265AMD_BLOCK + threadIdx.x);
    if (t >= 2 * n) return;
    const int l = t / n, cu = t % n;
    if (!b.ref_costs[l]) return;
    const unsigned long long a = ((const unsigned long long*)b.scratch)[t];
    if (!a) return;
    const unsigned long long v = (unsigned long long)b.ref_costs[l][cu] + a;
    b.ref_costs[l][cu] = (uint16_t)(v < 65535ull ? v : 65535ull);
}

} // namespace x265amd

extern "C" int x265amd_cutree_propagate(int count, const x265amd_propagate_batch* batches, void* stream)
{
    using namespace x265amd;
    if (count < 0 || (count && !batches)) return X265AMD_EINVAL;
    for (int i = 0; i < count; i++)
    {
        const x265amd_propagate_batch& b = batches[i];
        if (b.width_cu <= 0 || b.height_cu <= 0 || !b.intra_cost || !b.lowres_costs || !b.inv_qscale || !b.scratch ||
            !b.mvs[0] || !b.ref_costs[0])
            return X265AMD_EINVAL;
    }
    hipStream_t st = (hipStream_t)stream;
    for (int i = 0; i < count; i++)
    {
        const x265amd_propagate_batch& b = batches[i];
        const size_t n = (size_t)b.width_cu * b.height_cu;
        hipError_t e = hipMemsetAsync(b.scratch, 0, 2 * n * sizeof(int64_t), st);
        if (e != hipSuccess) return (int)e;
        hipLaunchKernelGGL(k_propagate, dim3((unsigned)((n + X265AMD_BLOCK - 1) / X265AMD_BLOCK)), dim3(X265AMD_BLOCK),
                           0, st, b);
        hipLaunchKernelGGL(k_propagate_finish, dim3((unsigned)((2 * n + X265AMD_BLOCK - 1) / X265AMD_BLOCK)),
                           dim3(X265AMD_BLOCK), 0, st, b);
        e = hipGetLastError();
        if (e != hipSuccess) return (int)e;
    }
    return 0;
}

// ================================================================ f1 weighted-prediction analysis
namespace x265amd {

// weight_pp_c (pixel.cpp:463-488) over a whole padded plane, C pixels per thread
template <typename P>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_weight_pp(const P* __restrict__ src, P* __restrict__ dst,
                                                             int64_t n, int w0, int round, int shift, int offset,
                                                             int maxv)
{
    constexpr int C = 16 / sizeof(P);
    const int64_t i0 = ((int64_t)blockIdx.x * X265AMD_BLOCK + threadIdx.x) * C;
    if (i0 >= n) return;
    const int corr = 14 - (sizeof(P) == 1 ? 8 : (maxv == 1023 ? 10 : 12));
    if (i0 + C <= n)
    {
        int v[C];
        load_row<P, C>(src + i0, v);
#pragma unroll
        for (int k = 0; k < C; k++)
        {
            const int16_t val = (int16_t)(v[k] << corr);
            const int r = ((w0 * val + round) >> shift) + offset;
            v[k] = r < 0 ? 0 : (r > maxv ? maxv : r);
        }
        store_row<P, C>(dst + i0, v);
        return;
    }
    for (int64_t i = i0; i < n; i++)
    {
        const int16_t val = (int16_t)((int)src[i] << corr);
        const int r = ((w0 * val + round) >> shift) + offset;
        dst[i] = (P)(r < 0 ? 0 : (r > maxv ? maxv : r));
    }
}

// weightCostLuma's sum (slicetype.cpp:359-365): one thread per 8x8 block, satd 8x8 as four 4x4
// Hadamard sums (>> 1 once: SURVEY note a7), min with intraCost, uint32 sum (order-free)
template <typename P>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_weight_cost(const P* __restrict__ src, const P* __restrict__ fenc,
                                                               int64_t stride, int wcu, int hcu,
                                                               const int32_t* __restrict__ intra, uint32_t* cost)
{
    const int mb = (int)(blockIdx.x * X265AMD_BLOCK + threadIdx.x);
    int c = 0;
    if (mb < wcu * hcu)
    {
        const int64_t off = (int64_t)(mb / wcu) * 8 * stride + (mb % wcu) * 8;
        int d[8][8];
#pragma unroll
        for (int r = 0; r < 8; r++)
        {
            int a[8], b[8];
            load_row<P, 8>(src + off + r * stride, a);
            load_row<P, 8>(fenc + off + r * stride, b);
#pragma unroll
            for (int x = 0; x < 8; x++) d[r][x] = a[x] - b[x];
        }
        int sum = 0;
#pragma unroll
        for (int qy = 0; qy < 8; qy += 4)
#pragma unroll
            for (int qx = 0; qx < 8; qx += 4)
            {
#pragma unroll
                for (int r = 0; r < 4; r++) had4(d[qy + r][qx], d[qy + r][qx + 1], d[qy + r][qx + 2], d[qy + r][qx + 3]);
#pragma unroll
                for (int x = 0; x < 4; x++)
                {
                    had4(d[qy][qx + x], d[qy + 1][qx + x], d[qy + 2][qx + x], d[qy + 3][qx + x]);
#pragma unroll
                    for (int r = 0; r < 4; r++) sum += d[qy + r][qx + x] < 0 ? -d[qy + r][qx + x] : d[qy + r][qx + x];
                }
            }
        const int satd = sum >> 1;
        c = satd < intra[mb] ? satd : intra[mb];
    }
    // wave sum, one atomic per wave
#pragma unroll
    for (int o = 32; o; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(cost, (uint32_t)c);
}

template <typename P>
static int weight_pp_plane(const void* src, void* dst, int64_t n, int w0, int round, int shift, int offset, int maxv,
                           hipStream_t st)
{
    constexpr int C = 16 / sizeof(P);
    const int64_t threads = (n + C - 1) / C;
    hipLaunchKernelGGL(k_weight_pp<P>, dim3((unsigned)((threads + X265AMD_BLOCK - 1) / X265AMD_BLOCK)),
                       dim3(X265AMD_BLOCK), 0, st, (const P*)src, (P*)dst, n, w0, round, shift, offset, maxv);
    return (int)hipGetLastError();
}

// weightCostLuma (slicetype.cpp:338-368): weighted (present) or plain reference vs fenc
template <typename P>
static int weight_cost(const x265amd_weights_batch& b, int depth, bool present, int w0, int denom, int offset,
                       uint32_t* out, hipStream_t st)
{
    const P* src = (const P*)b.ref_buf[0] + b.pad_offset;
    const int maxv = (1 << depth) - 1;
    if (present)
    {
        const int off = offset << (depth - 8), round = denom ? 1 << (denom - 1) : 0, corr = 14 - depth;
        int rc = weight_pp_plane<P>(b.ref_buf[0], b.wbuf[0], b.stride * b.padded_lines, w0, round << corr,
                                    denom + corr, off, maxv, st);
        if (rc) return rc;
        src = (const P*)b.wbuf[0] + b.pad_offset;
    }
    hipError_t e = hipMemsetAsync(b.scratch, 0, 4, st);
    if (e != hipSuccess) return (int)e;
    const int wcu = b.width / 8, hcu = b.lines / 8;
    hipLaunchKernelGGL(k_weight_cost<P>, dim3((unsigned)((wcu * hcu + X265AMD_BLOCK - 1) / X265AMD_BLOCK)),
                       dim3(X265AMD_BLOCK), 0, st, src, (const P*)b.fenc_plane, b.stride, wcu, hcu, b.intra_cost,
                       b.scratch);
    e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    e = hipMemcpyAsync(out, b.scratch, 4, hipMemcpyDeviceToHost, st);
    if (e != hipSuccess) return (int)e;
    return (int)hipStreamSynchronize(st);
}

// LookaheadTLD::weightsAnalyse (slicetype.cpp:391-495); the host float arithmetic is the
// reference's, statement for statement
template <typename P>
static int weights_analyse(int depth, x265amd_weights_batch& b, hipStream_t st)
{
    const float epsilon = 1.f / 128.f;
    b.weighted = 0;
    float guessScale;
    if (b.fenc_ssd && b.ref_ssd) guessScale = sqrtf((float)b.fenc_ssd / b.ref_ssd);
    else guessScale = 1.0f;
    const float fencMean = (float)b.fenc_sum / (b.lines * b.width) / (1 << (depth - 8));
    const float refMean = (float)b.ref_sum / (b.lines * b.width) / (1 << (depth - 8));
    if (fabsf(refMean - fencMean) < 0.5f && fabsf(1.f - guessScale) < epsilon) return 0;
    int mindenom = 7, minscale = (int)(guessScale * 128 + 0.5f);          // setFromWeightAndOffset
    while (mindenom > 0 && minscale > 127) { mindenom--; minscale >>= 1; }
    if (minscale > 127) minscale = 127;
    int minoff = 0, found = 0;
    uint32_t minscore = 0, origscore = 0, s = 0;
    int rc = weight_cost<P>(b, depth, false, 0, 0, 0, &origscore, st);
    if (rc) return rc;
    minscore = origscore;
    if (!minscore) return 0;
    int curScale = minscale;
    int curOffset = (int)(fencMean - refMean * curScale / (1 << mindenom) + 0.5f);
    if (curOffset < -128 || curOffset > 127)
    {
        curOffset = curOffset < -128 ? -128 : 127;
        curScale = (int)((1 << mindenom) * (fencMean - curOffset) / refMean + 0.5f);
        curScale = curScale < 0 ? 0 : (curScale > 127 ? 127 : curScale);
    }
    rc = weight_cost<P>(b, depth, true, curScale, mindenom, curOffset, &s, st);
    if (rc) return rc;
    if (s < minscore) { minscore = s; minscale = curScale; minoff = curOffset; found = 1; }
    while (mindenom > 0 && !(minscale & 1)) { mindenom--; minscale >>= 1; }
    if (!found || (minscale == 1 << mindenom && minoff == 0) || (float)minscore / origscore > 0.998f) return 0;
    b.cost_delta = minscore / origscore;
    const int off = minoff << (depth - 8), round = mindenom ? 1 << (mindenom - 1) : 0, corr = 14 - depth;
    for (int i = 0; i < 4; i++)
    {
        rc = weight_pp_plane<P>(b.ref_buf[i], b.wbuf[i], b.stride * b.padded_lines, minscale, round << corr,
                                mindenom + corr, off, (1 << depth) - 1, st);
        if (rc) return rc;
    }
    b.weighted = 1;
    b.scale = minscale;
    b.denom = mindenom;
    b.offset = minoff;
    return 0;
}

} // namespace x265amd

extern "C" int x265amd_weights_analyse(int depth, x265amd_weights_batch* b, void* stream)
{
    using namespace x265amd;
    if (!b || (depth != 8 && depth != 10 && depth != 12) || b->width <= 0 || b->lines <= 0 || (b->width & 7) ||
        (b->lines & 7) || b->stride < b->width || !b->fenc_plane || !b->intra_cost || !b->scratch)
        return X265AMD_EINVAL;
    for (int i = 0; i < 4; i++)
        if (!b->ref_buf[i] || !b->wbuf[i]) return X265AMD_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    return depth == 8 ? weights_analyse<uint8_t>(depth, *b, st) : weights_analyse<uint16_t>(depth, *b, st);
}
