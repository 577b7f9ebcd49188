// me.hip — batched full-resolution motion search.
//
// One job = one MotionEstimate::motionEstimate call (motion.cpp:571-1172) for a
// PU on a full-resolution reference at subme 0..7 (from subme 3 the sub-pel
// compare adds the 4:2:0 chroma SATD, motion.cpp:197): the clipped MVP measured at sub-pel
// with SAD, the caller's extra MV candidates, DIA / HEX / STAR integer search, then
// the sub-pel refine of workload[subme] whose blocks come from the 8-tap luma
// filters exactly as subpelCompare builds them (motion.cpp:1174-1203;
// ipfilter.cpp interp_horiz_pp / interp_vert_pp / interp_hv_pp).
//
// Work mapping: a PU is owned by a group of G lanes (G = the PU's 4x4 units
// rounded up to a power of two, at most 64); every lane keeps the fenc pixels
// of its units in registers and evaluates its units of every candidate block
// — full-pel rows straight from the reference, sub-pel rows through the
// horizontal / vertical / 2-D 8-tap filter computed per unit — and the group
// sums SAD / SATD partials with shuffles.  Every decision is then identical
// in all lanes of the group, so the search runs in lockstep in the reference's
// candidate order (the packed-cost tie rules of the DIA / HEX loops included).
// FULL search is the one data-parallel integer search: k_full_search (below) runs it as a
// block-per-PU argmin before the lockstep kernel refines its result.
#include "common.h"
#include "../../../include/x265_amd.h"

namespace x265amd {

struct MeArgs
{
    const void* fenc;
    const int64_t* fenc_off;
    int64_t fs;
    const void* ref;
    const int64_t* ref_off;
    int64_t rs;
    const int16_t* mv_range;
    const int16_t* mvp;
    const int16_t* mvc;
    const uint8_t* num_cand;
    const uint16_t* mvcost;
    const int64_t* mvcost_off;
    int16_t* out_mv;
    int32_t* out_cost;
    const void* fcb;              // chroma (4:2:0) for subme 3; NULL = none
    const void* fcr;
    int64_t fcs;
    const int64_t* fcoff;
    const void* rcb;
    const void* rcr;
    int64_t rcs;
    const int64_t* rcoff;
    uint32_t* evals;              // [2 n]: job j's full-pel / sub-pel block evaluations (NULL = not counted)
    int w, h, n, lg, method, subme, merange, max_cand, depth;
    int win_bytes;                // dynamic LDS of a search-window launch (k_motion_search<P, G, true>), else 0
    int win_r;                    // its window's reach around the search start (full-pel)
};

constexpr int kMeMaxUnits = 4;    // 4x4 units per lane (64x64 PU over 64 lanes)

// W: the search window is staged in LDS (k_motion_search<P, G, true>): lref / lrs address it with the PU origin
// as (0, 0), and [wx0, wx1) x [wy0, wy1) is the part of the reference plane (PU-relative pixels) it holds; a
// block whose reads all fall inside is read from LDS, any other from the reference plane
template <typename P, bool W = false>
struct MeState
{
    const P* ref;           // reference at the PU origin
    int64_t rs;
    const P* lref;
    int64_t lrs;
    int wx0, wx1, wy0, wy1;
    const uint16_t* tab;
    int mvpx, mvpy;
    int nu, lane, G, uw;    // units of this lane, lane in group, group size, units per PU row
    int w, h, depth;
    int nmax;               // most units of any lane (uniform): 1, 2 or 4 of them go per round trip
    const P* fenc;          // source PU origin
    int64_t fs;
    uint32_t fe[kMeMaxUnits][4][sizeof(P) == 1 ? 1 : 2];   // this lane's fenc units, loaded once
    bool chroma;            // bChromaSATD
    const P* fc[2];         // source Cb / Cr at the PU's chroma origin
    const P* rc[2];         // reference Cb / Cr at the PU's chroma origin
    int64_t fcs, rcs;
    mutable uint32_t nfp, nsp;   // block evaluations made (uniform over the group)

    __device__ __forceinline__ void unit_xy(int k, int& ux, int& uy) const
    {
        const int u = lane + k * G;
        ux = 4 * (u % uw);
        uy = 4 * (u / uw);
    }
    __device__ __forceinline__ int mvcost(int qx, int qy) const
    {
        return (uint16_t)(tab[qx - mvpx] + tab[qy - mvpy]);
    }
    // the plane to read a footprint [x0, x1) x [y0, y1) from (wave-uniform: the footprint is the group's)
    __device__ __forceinline__ void source(int x0, int x1, int y0, int y1, const P*& r, int64_t& stride) const
    {
        r = ref;
        stride = rs;
        if constexpr (W)
            if (x0 >= wx0 && x1 <= wx1 && y0 >= wy0 && y1 <= wy1) { r = lref; stride = lrs; }
    }
};

template <typename P>
__device__ __forceinline__ void load4(const P* p, uint32_t (&w)[sizeof(P) == 1 ? 1 : 2])
{
    if constexpr (sizeof(P) == 1) w[0] = ldu<uint32_t>(p);
    else { const uint2 v = ldu<uint2>(p); w[0] = v.x; w[1] = v.y; }
}

template <typename P>
__device__ __forceinline__ uint32_t sad4(const uint32_t (&a)[sizeof(P) == 1 ? 1 : 2],
                                         const uint32_t (&b)[sizeof(P) == 1 ? 1 : 2], uint32_t acc)
{
    if constexpr (sizeof(P) == 1) return __builtin_amdgcn_sad_u8(a[0], b[0], acc);
    else return __builtin_amdgcn_sad_u16(a[1], b[1], __builtin_amdgcn_sad_u16(a[0], b[0], acc));
}

template <typename P>
__device__ __forceinline__ int px(const uint32_t (&w)[sizeof(P) == 1 ? 1 : 2], int i)
{
    if constexpr (sizeof(P) == 1) return (int)((w[0] >> (8 * i)) & 0xff);
    else return (int)((w[i >> 1] >> (16 * (i & 1))) & 0xffff);
}

__device__ __forceinline__ void had4m(int& a, int& b, int& c, int& d)
{
    const int s0 = a + b, s1 = a - b, s2 = c + d, s3 = c - d;
    a = s0 + s2; b = s1 + s3; c = s0 - s2; d = s1 - s3;
}

// sum over the G lanes of a group, every lane getting the sum: DPP lane moves inside rows of 16 (quad
// permutes, half-row and row mirrors: a few cycles each) and, for a whole wavefront, four lane reads of the
// row sums; the LDS-crossbar shuffles (one per halving, each an LDS round trip) only for the 16-lane step
// of a 32-lane group.  A search costs tens of dependent reductions, so their latency is the search's.
#ifndef X265AMD_ME_DPP
#define X265AMD_ME_DPP 1
#endif
template <int G>
__device__ __forceinline__ int me_group_sum(int v)
{
#if X265AMD_ME_DPP
    if constexpr (G >= 2) v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
    if constexpr (G >= 4) v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
    if constexpr (G >= 8) v += __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, false);   // row_half_mirror
    if constexpr (G >= 16) v += __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, false);  // row_mirror
    if constexpr (G == 32) v += __shfl_xor(v, 16, 64);
    if constexpr (G == 64)
        v = __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
            __builtin_amdgcn_readlane(v, 48);
    return v;
#else
    return group_sum<G>(v);
#endif
}

// N sums over a group of G lanes.  Up to a wavefront: me_group_sum each.  Groups of 2 or 4 wavefronts (one
// search per workgroup, X265AMD_ME_GMAX): each wave's sums, then the waves' partial sums through LDS between
// two barriers (the second keeps a fast wave's next write off the slots until every wave has read them); every
// wave of the group makes the same calls, since all decisions follow from these group-uniform sums
template <int G, int N>
__device__ __forceinline__ void me_group_sums(int (&v)[N])
{
    if constexpr (G <= 64)
    {
#pragma unroll
        for (int n = 0; n < N; n++) v[n] = me_group_sum<G>(v[n]);
    }
    else
    {
        constexpr int NW = G / 64;
        __shared__ int red[NW][N];
#pragma unroll
        for (int n = 0; n < N; n++) v[n] = me_group_sum<64>(v[n]);
        const int w = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0)
#pragma unroll
            for (int n = 0; n < N; n++) red[w][n] = v[n];
        __syncthreads();
#pragma unroll
        for (int n = 0; n < N; n++)
        {
            int t = red[0][n];
#pragma unroll
            for (int k = 1; k < NW; k++) t += red[k][n];
            v[n] = t;
        }
        __syncthreads();
    }
}

// full-pel SADs of the PU at N integer displacements (mx[n], my[n]), group-reduced.  fenc comes from
// registers (loaded once per PU); every reference row of all N candidates and NU units is loaded before the
// first SAD, and the N group reductions run side by side, so N candidates cost one memory round trip and
// one reduction latency instead of N.  Lanes beyond the PU's units (nu = 0) load the PU's first unit.
template <typename P, int G, int N, int NU, bool WIN>
__device__ __forceinline__ void fpel_sad_nu(const MeState<P, WIN>& s, const int (&mx)[N], const int (&my)[N],
                                            int (&out)[N])
{
    constexpr int W = sizeof(P) == 1 ? 1 : 2;
    int x0 = mx[0], x1 = mx[0], y0 = my[0], y1 = my[0];
#pragma unroll
    for (int n = 1; n < N; n++)
    {
        x0 = min(x0, mx[n]); x1 = max(x1, mx[n]);
        y0 = min(y0, my[n]); y1 = max(y1, my[n]);
    }
    const P* ref;
    int64_t rs;
    s.source(x0, x1 + s.w, y0, y1 + s.h, ref, rs);
    uint32_t w[N][NU][4][W];
#pragma unroll
    for (int k = 0; k < NU; k++)
    {
        int ux = 0, uy = 0;
        if (s.nu) s.unit_xy(k < s.nu ? k : 0, ux, uy);
#pragma unroll
        for (int n = 0; n < N; n++)
        {
            const P* p = ref + (ux + mx[n]) + (int64_t)(uy + my[n]) * rs;
#pragma unroll
            for (int r = 0; r < 4; r++) load4<P>(p + r * rs, w[n][k][r]);
        }
    }
#pragma unroll
    for (int n = 0; n < N; n++)
    {
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < NU; k++)
        {
            uint32_t a = 0;
#pragma unroll
            for (int r = 0; r < 4; r++) a = sad4<P>(s.fe[k][r], w[n][k][r], a);
            acc += k < s.nu ? a : 0u;
        }
        out[n] = (int)acc;
    }
    me_group_sums<G, N>(out);
}

// N candidates' SADs; `counted` of them are real evaluations (the rest are range-failed points whose loads
// were clamped to a valid position and whose results are ignored)
template <typename P, int G, int N, bool WIN>
__device__ __forceinline__ void fpel_sads(const MeState<P, WIN>& s, const int (&mx)[N], const int (&my)[N],
                                          int (&out)[N], int counted = N)
{
    s.nfp += counted;
    if constexpr (G != 64) fpel_sad_nu<P, G, N, 1>(s, mx, my, out);     // one unit per lane below and above
    else if (s.nmax == 1) fpel_sad_nu<P, G, N, 1>(s, mx, my, out);
    else if (s.nmax == 2) fpel_sad_nu<P, G, N, 2>(s, mx, my, out);
    else fpel_sad_nu<P, G, N, kMeMaxUnits>(s, mx, my, out);
}

// ... plus the MV cost (quarter-pel MV = 4 x full-pel)
template <typename P, int G, int N, bool WIN>
__device__ __forceinline__ void fpel_costs(const MeState<P, WIN>& s, const int (&mx)[N], const int (&my)[N],
                                           int (&out)[N], int counted = N)
{
    fpel_sads<P, G, N>(s, mx, my, out, counted);
#pragma unroll
    for (int n = 0; n < N; n++) out[n] += s.mvcost(4 * mx[n], 4 * my[n]);
}

// one candidate's SAD
template <typename P, int G, bool WIN>
__device__ __forceinline__ int fpel_sad(const MeState<P, WIN>& s, int dx, int dy)
{
    const int mx[1] = { dx }, my[1] = { dy };
    int c[1];
    fpel_sads<P, G, 1>(s, mx, my, c);
    return c[0];
}

// N consecutive pixels from p as ints, by vector loads that stay inside [p, p + N)
// (N = 4, 7 or 11; overlapping loads cover the odd widths)
template <typename P, int N>
__device__ __forceinline__ void load_px(const P* p, int (&v)[N])
{
    if constexpr (N == 4)
        load_row<P, 4>(p, v);
    else if constexpr (N == 7)
    {
        int a[4], b[4];
        load_row<P, 4>(p, a);
        load_row<P, 4>(p + 3, b);
#pragma unroll
        for (int i = 0; i < 4; i++) { v[i] = a[i]; v[3 + i] = b[i]; }
    }
    else
    {
        static_assert(N == 11, "window");
        int a[8], b[4];
        load_row<P, 8>(p, a);
        load_row<P, 4>(p + 7, b);
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = a[i];
#pragma unroll
        for (int i = 0; i < 4; i++) v[7 + i] = b[i];
    }
}

// the 4:2:0 chroma SATD subpelCompare adds at subme 3 (motion.cpp:1205-1266): the chroma block at
// the 1/8-pel position (qx, qy) (4-tap pp filters; hps + vsp for 2-D), satd against the source
// chroma, over this lane's 4x4 chroma units (not group-reduced)
template <typename P>
__device__ __forceinline__ int chroma_satd(const MeState<P>& s, int qx, int qy)
{
    const int cw = s.w >> 1, ch = s.h >> 1;
    const int cuw = cw >> 2, units = cuw * (ch >> 2);
    const int xf = qx & 7, yf = qy & 7;
    const int64_t off = (qx >> 3) + (int64_t)(qy >> 3) * s.rcs;
    const int maxv = (1 << s.depth) - 1;
    const int head = 14 - s.depth;
    int cx[4], cy[4];
#pragma unroll
    for (int t = 0; t < 4; t++) { cx[t] = c_chroma.c[xf][t]; cy[t] = c_chroma.c[yf][t]; }
    int acc = 0;
    for (int u = s.lane; u < units; u += s.G)
    {
        const int ux = 4 * (u % cuw), uy = 4 * (u / cuw);
#pragma unroll
        for (int pl = 0; pl < 2; pl++)
        {
            const P* p = s.rc[pl] + off + ux + (int64_t)uy * s.rcs;
            int blk[4][4];
            if (!(xf | yf))
            {
#pragma unroll
                for (int r = 0; r < 4; r++) load_px<P, 4>(p + r * s.rcs, blk[r]);
            }
            else if (!yf)
            {
#pragma unroll
                for (int r = 0; r < 4; r++)
                {
                    int w7[7];
                    load_px<P, 7>(p + r * s.rcs - 1, w7);
#pragma unroll
                    for (int c = 0; c < 4; c++)
                    {
                        int sum = 0;
#pragma unroll
                        for (int t = 0; t < 4; t++) sum += cx[t] * w7[c + t];
                        const int val = (int16_t)((sum + 32) >> 6);
                        blk[r][c] = val < 0 ? 0 : (val > maxv ? maxv : val);
                    }
                }
            }
            else if (!xf)
            {
                int w4[7][4];
#pragma unroll
                for (int i = 0; i < 7; i++) load_px<P, 4>(p + (i - 1) * s.rcs, w4[i]);
#pragma unroll
                for (int r = 0; r < 4; r++)
#pragma unroll
                    for (int c = 0; c < 4; c++)
                    {
                        int sum = 0;
#pragma unroll
                        for (int t = 0; t < 4; t++) sum += cy[t] * w4[r + t][c];
                        const int val = (int16_t)((sum + 32) >> 6);
                        blk[r][c] = val < 0 ? 0 : (val > maxv ? maxv : val);
                    }
            }
            else
            {
                // filter_hps (isRowExt: rows -1 .. +2 beyond the unit) then filter_vsp
                const int ps_shift = 6 - head, ps_off = -8192 * (1 << ps_shift);
                const int sp_shift = 6 + head, sp_off = (1 << (sp_shift - 1)) + (8192 << 6);
                int m[7][4];
#pragma unroll
                for (int i = 0; i < 7; i++)
                {
                    int w7[7];
                    load_px<P, 7>(p + (i - 1) * s.rcs - 1, w7);
#pragma unroll
                    for (int c = 0; c < 4; c++)
                    {
                        int sum = 0;
#pragma unroll
                        for (int t = 0; t < 4; t++) sum += cx[t] * w7[c + t];
                        m[i][c] = (int16_t)((sum + ps_off) >> ps_shift);
                    }
                }
#pragma unroll
                for (int r = 0; r < 4; r++)
#pragma unroll
                    for (int c = 0; c < 4; c++)
                    {
                        int sum = 0;
#pragma unroll
                        for (int t = 0; t < 4; t++) sum += cy[t] * m[r + t][c];
                        const int val = (int16_t)((sum + sp_off) >> sp_shift);
                        blk[r][c] = val < 0 ? 0 : (val > maxv ? maxv : val);
                    }
            }
            int d[4][4];
            const P* f = s.fc[pl] + ux + (int64_t)uy * s.fcs;
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int c = 0; c < 4; c++) d[r][c] = (int)f[r * s.fcs + c] - blk[r][c];
#pragma unroll
            for (int r = 0; r < 4; r++) had4m(d[r][0], d[r][1], d[r][2], d[r][3]);
            int sum = 0;
#pragma unroll
            for (int c = 0; c < 4; c++)
            {
                had4m(d[0][c], d[1][c], d[2][c], d[3][c]);
#pragma unroll
                for (int r = 0; r < 4; r++) sum += d[r][c] < 0 ? -d[r][c] : d[r][c];
            }
            acc += sum >> 1;
        }
    }
    return acc;
}

// 8-bit reference rows are read as dwords (X265AMD_ME_B32=1): the rows may be in an LDS search window, where a
// 64-bit read off its 8-byte alignment is replayed (32-bit reads are not)
#ifndef X265AMD_ME_B32
#define X265AMD_ME_B32 1
#endif
// One row of a unit's reference window kept packed as loaded: C = 4 pixels (full-pel columns) or 11
// (the 8-tap reach, -3 .. +7): an 8-pixel vector and the 4 pixels from +7 (overlapping by one).
template <typename P, int C>
struct RawRow
{
    static constexpr int WA = (C == 4 ? 4 : 8) * (int)sizeof(P) / 4;
    static constexpr int WB = C == 4 ? 0 : (int)sizeof(P);
    uint32_t a[WA];
    uint32_t b[WB > 0 ? WB : 1];
    __device__ __forceinline__ void load(const P* p)
    {
        if constexpr (WA == 1) a[0] = ldu<uint32_t>(p);
        else if constexpr (WA == 2 && X265AMD_ME_B32)
        {
            a[0] = ldu<uint32_t>(p);
            a[1] = ldu<uint32_t>((const uint8_t*)p + 4);
        }
        else if constexpr (WA == 2) { const uint2 v = ldu<uint2>(p); a[0] = v.x; a[1] = v.y; }
        else { const uint4 v = ldu<uint4>(p); a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w; }
        if constexpr (WB == 1) b[0] = ldu<uint32_t>(p + 7);
        else if constexpr (WB == 2) { const uint2 v = ldu<uint2>(p + 7); b[0] = v.x; b[1] = v.y; }
    }
    __device__ __forceinline__ int get(int i) const
    {
        const uint32_t* w = a;
        if (C == 11 && i >= 8) { w = b; i -= 7; }
        if constexpr (sizeof(P) == 1) return (int)((w[i >> 2] >> (8 * (i & 3))) & 0xff);
        else return (int)((w[i >> 1] >> (16 * (i & 1))) & 0xffff);
    }
};

// the 4x4 block at one fractional case (CASE bit 0: horizontal fraction, bit 1: vertical) from its reference
// window: get(r, c) is the window pixel at row r, column c, the window starting 3 rows above the block when
// CASE & 2 and 3 columns left of it when CASE & 1 (11 rows / columns then, else 4)
template <typename P, int CASE, typename Get>
__device__ __forceinline__ void subpel_block(const Get& get, const int (&cx)[8], const int (&cy)[8], int depth,
                                             int (&blk)[4][4])
{
    const int maxv = (1 << depth) - 1;
    const int head = 14 - depth;
    if constexpr (CASE == 0)
    {
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int c = 0; c < 4; c++) blk[r][c] = get(r, c);
    }
    else if constexpr (CASE == 1)
    {
        // interp_horiz_pp: (int16)((sum + 32) >> 6) clipped
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int c = 0; c < 4; c++)
            {
                int sum = 0;
#pragma unroll
                for (int t = 0; t < 8; t++) sum += cx[t] * get(r, c + t);
                const int val = (int16_t)((sum + 32) >> 6);
                blk[r][c] = val < 0 ? 0 : (val > maxv ? maxv : val);
            }
    }
    else if constexpr (CASE == 2)
    {
        // interp_vert_pp
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int c = 0; c < 4; c++)
            {
                int sum = 0;
#pragma unroll
                for (int t = 0; t < 8; t++) sum += cy[t] * get(r + t, c);
                const int val = (int16_t)((sum + 32) >> 6);
                blk[r][c] = val < 0 ? 0 : (val > maxv ? maxv : val);
            }
    }
    else
    {
        // interp_hv_pp: horizontal ps over 11 rows (int16), then vertical sp
        const int ps_shift = 6 - head, ps_off = -8192 * (1 << ps_shift);
        const int sp_shift = 6 + head, sp_off = (1 << (sp_shift - 1)) + (8192 << 6);
        int m[11][4];
#pragma unroll
        for (int i = 0; i < 11; i++)
#pragma unroll
            for (int c = 0; c < 4; c++)
            {
                int sum = 0;
#pragma unroll
                for (int t = 0; t < 8; t++) sum += cx[t] * get(i, c + t);
                m[i][c] = (int16_t)((sum + ps_off) >> ps_shift);
            }
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int c = 0; c < 4; c++)
            {
                int sum = 0;
#pragma unroll
                for (int t = 0; t < 8; t++) sum += cy[t] * m[r + t][c];
                const int val = (int16_t)((sum + sp_off) >> sp_shift);
                blk[r][c] = val < 0 ? 0 : (val > maxv ? maxv : val);
            }
    }
}

// SATD (or SAD) of the source unit against a 4x4 block
template <typename P>
__device__ __forceinline__ int block_cost(const uint32_t (&fe)[4][sizeof(P) == 1 ? 1 : 2], const int (&blk)[4][4],
                                          bool satd)
{
    int cost = 0;
    if (satd)
    {
        int d[4][4];
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int c = 0; c < 4; c++) d[r][c] = px<P>(fe[r], c) - blk[r][c];
#pragma unroll
        for (int r = 0; r < 4; r++) had4m(d[r][0], d[r][1], d[r][2], d[r][3]);
        int sum = 0;
#pragma unroll
        for (int c = 0; c < 4; c++)
        {
            had4m(d[0][c], d[1][c], d[2][c], d[3][c]);
#pragma unroll
            for (int r = 0; r < 4; r++) sum += d[r][c] < 0 ? -d[r][c] : d[r][c];
        }
        cost = sum >> 1;      // each 4x4 raw sum is even (SURVEY note a7): any tiling gives satd
    }
    else
    {
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int c = 0; c < 4; c++)
            {
                const int d = px<P>(fe[r], c) - blk[r][c];
                cost += d < 0 ? -d : d;
            }
    }
    return cost;
}

// 8-bit horizontal 8-tap sums of one 12-pixel view row at output columns 0 .. 3 (output c = taps over pixels
// c .. c + 7): v_dot4_i32_i8 on pixels biased to signed (p ^ 0x80 = p - 128), so each sum comes out lowered by
// 128 x (sum of the taps = 64) = 8192 — added back through `init` where the filter needs the true sum
__device__ __forceinline__ void hsum4_u8(const uint32_t (&w)[3], uint32_t k0, uint32_t k1, int init, int (&out)[4])
{
    const uint32_t x0 = w[0] ^ 0x80808080u, x1 = w[1] ^ 0x80808080u, x2 = w[2] ^ 0x80808080u;
#pragma unroll
    for (int c = 0; c < 4; c++)
    {
        const uint32_t lo = __builtin_amdgcn_alignbyte(x1, x0, (uint32_t)c);
        const uint32_t hi = __builtin_amdgcn_alignbyte(x2, x1, (uint32_t)c);
        out[c] = __builtin_amdgcn_sdot4((int)hi, (int)k1, __builtin_amdgcn_sdot4((int)lo, (int)k0, init, false), false);
    }
}

// the 8-bit horizontal cases on the dot products: CASE 1 (interp_horiz_pp over the block's 4 rows) or CASE 3
// (interp_hv_pp: the ps pass over 11 rows is the biased dot sum itself at 8 bits, then the sp pass);
// roww(r, w) gives window row r as 12 pixels in 3 dwords (the window starts 3 rows up for CASE 3)
template <int CASE, typename RowW>
__device__ __forceinline__ void subpel_block_u8(const RowW& roww, const int (&cx)[8], const int (&cy)[8],
                                                int (&blk)[4][4])
{
    uint32_t k0 = 0, k1 = 0;
#pragma unroll
    for (int t = 0; t < 4; t++)
    {
        k0 |= (uint32_t)(cx[t] & 255) << (8 * t);
        k1 |= (uint32_t)(cx[t + 4] & 255) << (8 * t);
    }
    if constexpr (CASE == 1)
    {
#pragma unroll
        for (int r = 0; r < 4; r++)
        {
            uint32_t w[3];
            roww(r, w);
            int hs[4];
            hsum4_u8(w, k0, k1, 8192 + 32, hs);          // (int16)((sum + 32) >> 6) clipped
#pragma unroll
            for (int q = 0; q < 4; q++)
            {
                const int val = (int16_t)(hs[q] >> 6);
                blk[r][q] = val < 0 ? 0 : (val > 255 ? 255 : val);
            }
        }
    }
    else
    {
        int m[11][4];
#pragma unroll
        for (int i = 0; i < 11; i++)
        {
            uint32_t w[3];
            roww(i, w);
            hsum4_u8(w, k0, k1, 0, m[i]);
#pragma unroll
            for (int q = 0; q < 4; q++) m[i][q] = (int16_t)m[i][q];
        }
        constexpr int sp_shift = 12, sp_off = (1 << 11) + (8192 << 6);
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int q = 0; q < 4; q++)
            {
                int sum = 0;
#pragma unroll
                for (int t = 0; t < 8; t++) sum += cy[t] * m[r + t][q];
                const int val = (int16_t)((sum + sp_off) >> sp_shift);
                blk[r][q] = val < 0 ? 0 : (val > 255 ? 255 : val);
            }
    }
}

// subpelCompare's luma part over this lane's units for one fractional case: the reference windows (and
// source rows) of KU units are all loaded before the first is filtered, so a candidate costs one memory round
// trip per KU units, not one per unit.  Units past the lane's count load unit 0's window again (cache hits)
// and are not summed.
template <typename P, int CASE, int KU>
__device__ __forceinline__ int subpel_units(const MeState<P>& s, const P* base, const int (&cx)[8],
                                            const int (&cy)[8], bool satd)
{
    constexpr int R = (CASE & 2) ? 11 : 4, C = (CASE & 1) ? 11 : 4;
    const int64_t rs = s.rs, fs = s.fs;
    int acc = 0;
    for (int k0 = 0; k0 < s.nu; k0 += KU)
    {
        RawRow<P, C> win[KU][R];
        uint32_t fe[KU][4][sizeof(P) == 1 ? 1 : 2];
#pragma unroll
        for (int k = 0; k < KU; k++)
        {
            int ux, uy;
            s.unit_xy(k0 + k < s.nu ? k0 + k : k0, ux, uy);
            const P* p = base + ux + (int64_t)uy * rs - ((CASE & 2) ? 3 * rs : 0) - ((CASE & 1) ? 3 : 0);
#pragma unroll
            for (int r = 0; r < R; r++) win[k][r].load(p + r * rs);
#pragma unroll
            for (int r = 0; r < 4; r++) load4<P>(s.fenc + ux + (int64_t)(uy + r) * fs, fe[k][r]);
        }
#pragma unroll
        for (int k = 0; k < KU; k++)
        {
            int blk[4][4];
            if constexpr (sizeof(P) == 1 && (CASE & 1))
                // 8 window bytes and the 4 from +7: bytes 8 .. 10 are the second load's upper three
                subpel_block_u8<CASE>([&](int r, uint32_t (&w)[3]) {
                    w[0] = win[k][r].a[0];
                    w[1] = win[k][r].a[1];
                    w[2] = win[k][r].b[0] >> 8;
                }, cx, cy, blk);
            else
                subpel_block<P, CASE>([&](int r, int c) { return win[k][r].get(c); }, cx, cy, s.depth, blk);
            const int cost = block_cost<P>(fe[k], blk, satd);
            if (k0 + k < s.nu) acc += cost;
        }
    }
    return acc;
}

// One row of the window shared by a batch of sub-pel candidates: 12 pixels (the 8-tap reach of two integer
// positions), 8-bit in 3 dwords, 16-bit in 6
template <typename P>
struct Row12
{
    static constexpr int NW = 3 * (int)sizeof(P);
    uint32_t w[NW];
    __device__ __forceinline__ void load(const P* p)
    {
        if constexpr (sizeof(P) == 1 && X265AMD_ME_B32)
        {
            w[0] = ldu<uint32_t>(p); w[1] = ldu<uint32_t>(p + 4); w[2] = ldu<uint32_t>(p + 8);
        }
        else if constexpr (sizeof(P) == 1)
        {
            const uint2 v = ldu<uint2>(p);
            w[0] = v.x; w[1] = v.y; w[2] = ldu<uint32_t>(p + 8);
        }
        else
        {
            const uint4 v = ldu<uint4>(p);
            const uint2 u = ldu<uint2>(p + 8);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w; w[4] = u.x; w[5] = u.y;
        }
    }
    __device__ __forceinline__ int get(int i) const
    {
        if constexpr (sizeof(P) == 1) return (int)((w[i >> 2] >> (8 * (i & 3))) & 0xff);
        else return (int)((w[i >> 1] >> (16 * (i & 1))) & 0xffff);
    }
    // this row from row a or b (sel), moved left by o (0 or 1) pixels: get(i) = source.get(i + o)
    __device__ __forceinline__ void pick(const Row12& a, const Row12& b, bool sel, int o)
    {
        const uint32_t sh = (uint32_t)o * 8u * (uint32_t)sizeof(P);
#pragma unroll
        for (int j = 0; j < NW; j++)
        {
            const uint32_t lo = sel ? b.w[j] : a.w[j];
            const uint32_t hi = j + 1 < NW ? (sel ? b.w[j + 1] : a.w[j + 1]) : 0u;
            w[j] = __builtin_amdgcn_alignbit(hi, lo, sh);
        }
    }
};

// subpelCompare (motion.cpp:1174-1203): the block at quarter-pel (qx, qy), built by
// luma_hpp / luma_vpp / luma_hvpp when fractional, compared with SAD or SATD.  8-bit windows of all
// (at most 4) units of a lane fit in registers; at 16 bits two units go per round trip.
//
// Out of line (six call sites; inlined, the kernel spills), with the search state passed as values: a
// reference to the caller's MeState (or to the kernel's argument block) would keep that state in scratch
// memory.  lane_nu = lane | nu << 8, wh = w | h << 8, dc = depth | chroma << 8.
#ifndef X265AMD_ME_KU64
#define X265AMD_ME_KU64 2         // 8-bit unit windows per round trip in 64-lane groups
#endif
template <typename P, int G>
__device__ __noinline__ int subpel_cost(const P* ref, const P* fenc, int rs, int fs, int lane_nu, int wh, int dc,
                                        const P* fcb, const P* fcr, const P* rcb, const P* rcr, int fcs, int rcs,
                                        int qx, int qy, bool satd)
{
    MeState<P> s;
    s.ref = ref;
    s.rs = rs;
    s.fenc = fenc;
    s.fs = fs;
    s.lane = lane_nu & 255;
    s.nu = lane_nu >> 8;
    s.G = G;
    s.w = wh & 255;
    s.h = wh >> 8;
    s.uw = s.w >> 2;
    s.depth = dc & 255;
    s.chroma = (dc >> 8) != 0;
    if (s.chroma)
    {
        s.fc[0] = fcb; s.fc[1] = fcr;
        s.rc[0] = rcb; s.rc[1] = rcr;
        s.fcs = fcs; s.rcs = rcs;
    }
    const int xf = qx & 3, yf = qy & 3;
    const P* base = s.ref + (qx >> 2) + (int64_t)(qy >> 2) * s.rs;
    int cx[8], cy[8];
#pragma unroll
    for (int t = 0; t < 8; t++) { cx[t] = c_luma.c[xf][t]; cy[t] = c_luma.c[yf][t]; }
    // units per lane: 1 below 64 units, 2 for 64x32 / 32x64, 4 for 64x64 (uniform over the batch)
    const int nmax = (s.uw * (s.h >> 2) + G - 1) / G;
    int acc;
    // windows per round trip: up to two units (a 64x64 PU's four units of a lane in two trips; the 16-bit
    // 2-D case one at a time).  Four would push the function past 256 VGPRs, and the callee-saved registers
    // it then spills to scratch on every call cost more than the round trips saved
    // (profiles/r05/me_kernel_variants_ab.txt: 0.081 ms per launch at four 8-bit units, 0.059 at two)
    constexpr int KU = X265AMD_ME_KU64, KU_HV = sizeof(P) == 1 ? KU : 1;
    if (G != 64 || nmax == 1)      // (multi-unit lanes only in one-wave 64-lane groups, X265AMD_ME_GMAX=64)
    {
        if (!(xf | yf)) acc = subpel_units<P, 0, 1>(s, base, cx, cy, satd);
        else if (!yf) acc = subpel_units<P, 1, 1>(s, base, cx, cy, satd);
        else if (!xf) acc = subpel_units<P, 2, 1>(s, base, cx, cy, satd);
        else acc = subpel_units<P, 3, 1>(s, base, cx, cy, satd);
    }
    else
    {
        if (!(xf | yf)) acc = subpel_units<P, 0, KU>(s, base, cx, cy, satd);
        else if (!yf) acc = subpel_units<P, 1, KU>(s, base, cx, cy, satd);
        else if (!xf) acc = subpel_units<P, 2, KU>(s, base, cx, cy, satd);
        else acc = subpel_units<P, 3, KU_HV>(s, base, cx, cy, satd);
    }
    if (s.chroma)
        acc += chroma_satd<P>(s, qx, qy);
    int v[1] = { acc };
    me_group_sums<G, 1>(v);
    return v[0];
}

// Four candidates of one sub-pel refinement round (square directions i0 .. i0 + 3 at distance d quarter-pels
// around (qx, qy)), 8-bit: every candidate's integer position is X0 or X0 + 1 (Y0 or Y0 + 1), so one 12 x 12
// window per unit holds all four 8-tap windows; it is loaded once, each candidate's 11 x 11 view is picked
// from it in registers (row select, byte align), and the four group sums run side by side — one memory round
// trip and one reduction for the four instead of four of each.  Costs (luma + chroma SATD) in candidate order.
#ifndef X265AMD_ME_SPB
#define X265AMD_ME_SPB 1
#endif
template <typename P, int G>
__device__ __noinline__ int4 subpel_cost4(const P* ref, const P* fenc, int rs, int fs, int lane_nu, int wh, int dc,
                                          const P* fcb, const P* fcr, const P* rcb, const P* rcr, int fcs, int rcs,
                                          int qx, int qy, int d, int i0, bool satd)
{
    MeState<P> s;
    s.ref = ref;
    s.rs = rs;
    s.fenc = fenc;
    s.fs = fs;
    s.lane = lane_nu & 255;
    s.nu = lane_nu >> 8;
    s.G = G;
    s.w = wh & 255;
    s.h = wh >> 8;
    s.uw = s.w >> 2;
    s.depth = dc & 255;
    s.chroma = (dc >> 8) != 0;
    if (s.chroma)
    {
        s.fc[0] = fcb; s.fc[1] = fcr;
        s.rc[0] = rcb; s.rc[1] = rcr;
        s.fcs = fcs; s.rcs = rcs;
    }
    const int X0 = (qx - d) >> 2, Y0 = (qy - d) >> 2;
    int acc[4] = { 0, 0, 0, 0 };
    for (int k = 0; k < s.nu; k++)
    {
        int ux, uy;
        s.unit_xy(k, ux, uy);
        const P* p = s.ref + (ux + X0 - 3) + (int64_t)(uy + Y0 - 3) * s.rs;
        Row12<P> W[12];
#pragma unroll
        for (int r = 0; r < 12; r++) W[r].load(p + r * s.rs);
        uint32_t fe[4][sizeof(P) == 1 ? 1 : 2];
#pragma unroll
        for (int r = 0; r < 4; r++) load4<P>(s.fenc + ux + (int64_t)(uy + r) * s.fs, fe[r]);
#pragma unroll 1
        for (int c = 0; c < 4; c++)
        {
            const int tx = qx + d * sq_dx(i0 + c), ty = qy + d * sq_dy(i0 + c);
            const int ox = (tx >> 2) - X0, oy = (ty >> 2) - Y0;
            const int xf = tx & 3, yf = ty & 3;
            int cx[8], cy[8];
#pragma unroll
            for (int t = 0; t < 8; t++) { cx[t] = c_luma.c[xf][t]; cy[t] = c_luma.c[yf][t]; }
            Row12<P> V[11];
#pragma unroll
            for (int r = 0; r < 11; r++) V[r].pick(W[r], W[r + 1], oy != 0, ox);
            int blk[4][4];
            if (!(xf | yf))
                subpel_block<P, 0>([&](int r, int q) { return V[r + 3].get(q + 3); }, cx, cy, s.depth, blk);
            else if (!yf)
            {
                if constexpr (sizeof(P) == 1)
                    subpel_block_u8<1>([&](int r, uint32_t (&w)[3]) {
                        w[0] = V[r + 3].w[0]; w[1] = V[r + 3].w[1]; w[2] = V[r + 3].w[2];
                    }, cx, cy, blk);
                else
                    subpel_block<P, 1>([&](int r, int q) { return V[r + 3].get(q); }, cx, cy, s.depth, blk);
            }
            else if (!xf)
                subpel_block<P, 2>([&](int r, int q) { return V[r].get(q + 3); }, cx, cy, s.depth, blk);
            else
            {
                if constexpr (sizeof(P) == 1)
                    subpel_block_u8<3>([&](int r, uint32_t (&w)[3]) {
                        w[0] = V[r].w[0]; w[1] = V[r].w[1]; w[2] = V[r].w[2];
                    }, cx, cy, blk);
                else
                    subpel_block<P, 3>([&](int r, int q) { return V[r].get(q); }, cx, cy, s.depth, blk);
            }
            const int cost = block_cost<P>(fe, blk, satd);
            acc[0] += c == 0 ? cost : 0;
            acc[1] += c == 1 ? cost : 0;
            acc[2] += c == 2 ? cost : 0;
            acc[3] += c == 3 ? cost : 0;
        }
    }
    if (s.chroma)
    {
#pragma unroll
        for (int c = 0; c < 4; c++)
            acc[c] += chroma_satd<P>(s, qx + d * sq_dx(i0 + c), qy + d * sq_dy(i0 + c));
    }
    me_group_sums<G, 4>(acc);
    return make_int4(acc[0], acc[1], acc[2], acc[3]);
}

// workload[subme] of motion.cpp:48-58 as {hpel_iters, hpel_dirs, qpel_iters, qpel_dirs}, one
// nibble each per level (subme is wave-uniform: a batch has one level)
__device__ __forceinline__ int4 subpel_workload(int subme)
{
    constexpr uint32_t kTab[8] = { 0x4041, 0x4141, 0x4141, 0x4142, 0x4242, 0x8181, 0x8182, 0x8282 };
    const uint32_t v = kTab[subme & 7];
    return make_int4(v & 15, (v >> 4) & 15, (v >> 8) & 15, v >> 12);
}

template <typename P, int G, bool WIN = false>
#ifndef X265AMD_ME_WAVES
#define X265AMD_ME_WAVES 1
#endif
__global__ __launch_bounds__(X265AMD_BLOCK, X265AMD_ME_WAVES) void k_motion_search(const MeArgs a)
{
    // searches per workgroup: X265AMD_BLOCK / G up to a wavefront per search; one above (blockDim = G)
    constexpr int SPB = G > 64 ? 1 : X265AMD_BLOCK / G;
    const int64_t j = (int64_t)xcd_block() * SPB + threadIdx.x / G;
    if (j >= a.n) return;                               // whole groups
    MeState<P, WIN> s;
    s.lane = threadIdx.x & (G - 1);
    s.G = G;
    s.uw = a.w >> 2;
    const int units = s.uw * (a.h >> 2);
    s.nu = s.lane < units ? (units - s.lane + G - 1) / G : 0;
    s.ref = (const P*)a.ref + a.ref_off[j];
    s.rs = a.rs;
    s.tab = a.mvcost + a.mvcost_off[j];
    s.fenc = (const P*)a.fenc + a.fenc_off[j];
    s.fs = a.fs;
    s.nfp = s.nsp = 0;
    s.w = a.w;
    s.h = a.h;
    s.depth = a.depth;
    s.nmax = (units + G - 1) / G;
#pragma unroll
    for (int k = 0; k < kMeMaxUnits; k++)
    {
        if (k >= s.nu) break;
        int ux, uy;
        s.unit_xy(k, ux, uy);
#pragma unroll
        for (int r = 0; r < 4; r++) load4<P>(s.fenc + ux + (int64_t)(uy + r) * s.fs, s.fe[k][r]);
    }
    // bChromaSATD = subpelRefine > 2 && the 4:2:0 chroma satd entry exists (chroma dims % 4 == 0)
    s.chroma = a.subme > 2 && a.fcb && ((a.w >> 1) & 3) == 0 && ((a.h >> 1) & 3) == 0;
    s.fc[0] = s.fc[1] = s.rc[0] = s.rc[1] = nullptr;
    s.fcs = s.rcs = 0;
    if (s.chroma)
    {
        s.fc[0] = (const P*)a.fcb + a.fcoff[j]; s.fc[1] = (const P*)a.fcr + a.fcoff[j];
        s.rc[0] = (const P*)a.rcb + a.rcoff[j]; s.rc[1] = (const P*)a.rcr + a.rcoff[j];
        s.fcs = a.fcs; s.rcs = a.rcs;
    }
    const int minx = a.mv_range[4 * j], miny = a.mv_range[4 * j + 1];
    const int maxx = a.mv_range[4 * j + 2], maxy = a.mv_range[4 * j + 3];
    s.lref = s.ref;
    s.lrs = s.rs;
    s.wx0 = s.wy0 = 1 << 30;
    s.wx1 = s.wy1 = -(1 << 30);
    // stage the search window around full-pel (cx, cy) in LDS: up to win_r pixels either way within the MV
    // range box, 8 pixels around that and the PU (the reach of a DIA / HEX search, whose full-pel best may sit
    // up to 3 pixels outside the range, plus the sub-pel step and the 8-tap filter).  x265 clips the range 8
    // pixels short of its 64 + 8 pixel padding (CUData::clipMv, cudata.cpp:1870-1886), so the window is inside
    // the plane.  Whole aligned 16-byte chunks are copied (a row keeps its alignment, lead), all of a lane's
    // loads before its first store; a search that later steps outside the window reads the plane.
    auto stage = [&](int cx, int cy) {
        if constexpr (WIN)
        {
            extern __shared__ __attribute__((aligned(16))) uint4 me_win[];
            const int R = a.win_r;
            const int x0 = max(minx, cx - R) - 8, x1 = min(maxx, cx + R) + a.w + 9;
            const int y0 = max(miny, cy - R) - 8, y1 = min(maxy, cy + R) + a.h + 9;
            const int ww = x1 - x0, wh = y1 - y0;
            if (ww < 16 || wh <= 0) return;                          // (uniform over the workgroup)
            const uint8_t* g0 = (const uint8_t*)(s.ref + x0 + (int64_t)y0 * s.rs);
            const int lead = (int)((uintptr_t)g0 & 15);
            const int nc = (lead + ww * (int)sizeof(P) + 15) >> 4;   // 16-byte chunks per row (>= 2)
            if ((int64_t)nc * wh * 16 > a.win_bytes) return;
            const uint4* gs = (const uint4*)(g0 - lead);
            const int64_t gc = s.rs * (int64_t)sizeof(P) / 16;       // plane stride in chunks (host-checked)
            const int total = nc * wh;
            const uint32_t mag = 0xffffffffu / (uint32_t)nc + 1u;    // row = i / nc as a high multiply
            constexpr int B = G > 64 ? G : X265AMD_BLOCK, K = 8;
            for (int i0 = threadIdx.x; i0 < total; i0 += K * B)
            {
                uint4 v[K];
#pragma unroll
                for (int k = 0; k < K; k++)
                {
                    const int i = min(i0 + k * B, total - 1);
                    const int r = (int)__umulhi((uint32_t)i, mag);
                    v[k] = gs[r * gc + (i - r * nc)];
                }
#pragma unroll
                for (int k = 0; k < K; k++)
                    if (i0 + k * B < total) me_win[i0 + k * B] = v[k];
            }
            __syncthreads();
            s.lrs = nc * 16 / (int)sizeof(P);
            // lref (the PU origin) may lie outside the window — before the LDS array when the window sits
            // right of / below the PU origin.  Formed from the LDS pointer, the compiler does that arithmetic in
            // the 32-bit LDS address space, and the wrapped offset then carries out of the shared aperture when
            // a read adds its displacement back (an aperture violation); the generic address is laundered first
            // so the origin arithmetic is 64-bit flat arithmetic that every in-window read undoes exactly
            const uint8_t* wbase = (const uint8_t*)me_win;
            asm volatile("" : "+v"(wbase));
            s.lref = (const P*)(wbase + lead) - x0 - (int64_t)y0 * s.lrs;
            s.wx0 = x0; s.wx1 = x1;
            s.wy0 = y0; s.wy1 = y1;
        }
    };
    // the plane a sub-pel compare around full-pel (x, y) reads from: the 8-tap windows of the block at
    // (x, y) .. (x + 1, y + 1) span [x - 3, x + w + 5) x [y - 3, y + h + 5)
    auto spsrc = [&](int x, int y, const P*& r, int64_t& rs) { s.source(x - 3, x + a.w + 5, y - 3, y + a.h + 5, r, rs); };
    // the sub-pel compare, out of line
    auto spc = [&](int qx, int qy, bool satd) {
        s.nsp++;
        const P* r;
        int64_t rs;
        spsrc(qx >> 2, qy >> 2, r, rs);
        return subpel_cost<P, G>(r, s.fenc, (int)rs, (int)s.fs, s.lane | s.nu << 8, a.w | a.h << 8,
                                 a.depth | (s.chroma ? 256 : 0), s.fc[0], s.fc[1], s.rc[0], s.rc[1], (int)s.fcs,
                                 (int)s.rcs, qx, qy, satd);
    };
    s.mvpx = a.mvp[2 * j];
    s.mvpy = a.mvp[2 * j + 1];
    auto clipq = [&](int& x, int& y) {
        x = x > 4 * maxx ? 4 * maxx : x; y = y > 4 * maxy ? 4 * maxy : y;
        x = x < 4 * minx ? 4 * minx : x; y = y < 4 * miny ? 4 * miny : y;
    };
    int pmx = s.mvpx, pmy = s.mvpy;
    clipq(pmx, pmy);
    int bpx = pmx, bpy = pmy;                          // bestpre
    int bprecost = spc(pmx, pmy, false);   // no MV cost (motion.cpp:609)
    int bx = (pmx + 2) >> 2, by = (pmy + 2) >> 2;
    int bcost = bprecost;
    if (((pmx | pmy) & 3) && (pmx | pmy))
    {
        // the rounded MVP and MV 0 in one round trip
        const int mx[2] = { bx, 0 }, my[2] = { by, 0 };
        int c[2];
        fpel_costs<P, G, 2>(s, mx, my, c);
        bcost = c[0];
        if (c[1] < bcost) { bcost = c[1]; bx = by = 0; }
    }
    else if (pmx | pmy)
    {
        const int c = fpel_sad<P, G>(s, 0, 0) + s.mvcost(0, 0);
        if (c < bcost) { bcost = c; bx = by = 0; }
    }
    const int nc = a.num_cand ? a.num_cand[j] : 0;
    for (int i = 0; i < nc; i++)
    {
        int cx = a.mvc[2 * (j * a.max_cand + i)], cy = a.mvc[2 * (j * a.max_cand + i) + 1];
        clipq(cx, cy);
        if ((cx | cy) && (cx != pmx || cy != pmy) && (cx != bpx || cy != bpy))
        {
            const int c = spc(cx, cy, false) + s.mvcost(cx, cy);
            if (c < bprecost) { bprecost = c; bpx = cx; bpy = cy; }
        }
    }
    if (a.method <= 1)
        stage(bx, by);                                 // (the window variant runs DIA / HEX only)
    if (a.method == 0)
    {
        // diamond, radius 1 (motion.cpp:654-676)
        bcost <<= 4;
        int i = a.merange;
        do
        {
            const int mx[4] = { bx, bx, bx - 1, bx + 1 }, my[4] = { by - 1, by + 1, by, by };
            int c[4];
            fpel_costs<P, G, 4>(s, mx, my, c);
            if ((c[0] << 4) + 1 < bcost) bcost = (c[0] << 4) + 1;
            if ((c[1] << 4) + 3 < bcost) bcost = (c[1] << 4) + 3;
            if ((c[2] << 4) + 4 < bcost) bcost = (c[2] << 4) + 4;
            if ((c[3] << 4) + 12 < bcost) bcost = (c[3] << 4) + 12;
            if (!(bcost & 15)) break;
            bx -= (int32_t)((uint32_t)bcost << 28) >> 30;
            by -= (int32_t)((uint32_t)bcost << 30) >> 30;
            bcost &= ~15;
        } while (--i && bx >= minx && bx <= maxx && by >= miny && by <= maxy);
        bcost >>= 4;
    }
    else if (a.method == 2)
    {
        // STAR (motion.cpp:929-1034, StarPatternSearch :328-569)
        int bpn = 0, bdist = 0, bx0 = bx, by0 = by;
        // one candidate point, range-checked only on the sides it lies towards from the origin, as the
        // reference's per-point checks are (:367-385, :425-465, :514-561): the origin itself may be out of
        // range (MV 0 wins the start over a far MVP), and then points beside it on the far side are still
        // costed; when the whole pattern is inside the range (the reference's "border" case) every
        // directional check passes as well
        // up to four candidate points at once, range-checked only on the sides they lie towards from the
        // origin, as the reference's per-point checks are (:367-385, :425-465, :514-561): the origin itself
        // may be out of range (MV 0 wins the start over a far MVP), and then points beside it on the far
        // side are still costed; when the whole pattern is inside the range (the reference's "border" case)
        // every directional check passes as well.  Results are taken in the reference's point order.
        auto pts4 = [&](const int (&dx)[4], const int (&dy)[4], const int (&pn)[4], const int (&dd)[4]) {
            int mx[4], my[4], c[4];
            bool ok[4];
            int nok = 0;
#pragma unroll
            for (int q = 0; q < 4; q++)
            {
                mx[q] = bx0 + dx[q];
                my[q] = by0 + dy[q];
                ok[q] = !((dx[q] < 0 && mx[q] < minx) || (dx[q] > 0 && mx[q] > maxx) ||
                          (dy[q] < 0 && my[q] < miny) || (dy[q] > 0 && my[q] > maxy));
                nok += ok[q];
                if (!ok[q]) { mx[q] = bx0; my[q] = by0; }
            }
            if (!nok) return;
            fpel_costs<P, G, 4>(s, mx, my, c, nok);
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (ok[q] && c[q] < bcost) { bcost = c[q]; bx = mx[q]; by = my[q]; bpn = pn[q]; bdist = dd[q]; }
        };
        auto star = [&](int early) {
            bx0 = bx;
            by0 = by;
            int saved = bcost, rounds = 0;
            // distance 1: points 2, 4, 5, 7
            pts4({ 0, -1, 1, 0 }, { -1, 0, 0, 1 }, { 2, 4, 5, 7 }, { 1, 1, 1, 1 });
            if (bcost < saved) rounds = 0;
            else if (++rounds >= early) return;
            // distances 2, 4, 8: points 2, 1, 3, 4, 5, 6, 8, 7 (1, 3, 6, 8 at half distance)
            for (int dist = 2; dist <= 8; dist <<= 1)
            {
                const int h2 = dist >> 1;
                saved = bcost;
                pts4({ 0, -h2, h2, -dist }, { -dist, -h2, -h2, 0 }, { 2, 1, 3, 4 }, { dist, h2, h2, dist });
                pts4({ dist, -h2, h2, 0 }, { 0, h2, h2, dist }, { 5, 6, 8, 7 }, { dist, h2, h2, dist });
                if (bcost < saved) rounds = 0;
                else if (++rounds >= early) return;
            }
            // distances 16 .. merange: the four axis points, then three diamonds of four
            for (int dist = 16; dist <= a.merange; dist <<= 1)
            {
                saved = bcost;
                const int q = dist >> 2;
                pts4({ 0, -dist, dist, 0 }, { -dist, 0, 0, dist }, { 0, 0, 0, 0 }, { dist, dist, dist, dist });
#pragma unroll 1
                for (int index = 1; index < 4; index++)
                {
                    const int xl = -q * index, xr = q * index, yt = -dist + q * index, yb = dist - q * index;
                    pts4({ xl, xr, xl, xr }, { yt, yt, yb, yb }, { 0, 0, 0, 0 }, { dist, dist, dist, dist });
                }
                if (bcost < saved) rounds = 0;
                else if (++rounds >= early) return;
            }
        };
        // two-point check around a distance-1 best (offsets[], motion.cpp:74-84)
        auto two_points = [&]() {
            constexpr uint64_t OX = 0x1220102200202010ull, OY = 0x2122212002110001ull;   // offsets[] + 1, nibbles
            const int i0 = (bpn - 1) * 2, i1 = i0 + 1;
            const int m1x = bx + (int)((OX >> (4 * i0)) & 15) - 1, m1y = by + (int)((OY >> (4 * i0)) & 15) - 1;
            const int m2x = bx + (int)((OX >> (4 * i1)) & 15) - 1, m2y = by + (int)((OY >> (4 * i1)) & 15) - 1;
            const bool ok1 = m1x >= minx && m1x <= maxx && m1y >= miny && m1y <= maxy;
            const bool ok2 = m2x >= minx && m2x <= maxx && m2y >= miny && m2y <= maxy;
            if (!(ok1 || ok2)) return;
            const int mx[2] = { ok1 ? m1x : bx, ok2 ? m2x : bx }, my[2] = { ok1 ? m1y : by, ok2 ? m2y : by };
            int c[2];
            fpel_costs<P, G, 2>(s, mx, my, c, (int)ok1 + (int)ok2);
            if (ok1 && c[0] < bcost) { bcost = c[0]; bx = m1x; by = m1y; }
            if (ok2 && c[1] < bcost) { bcost = c[1]; bx = m2x; by = m2y; }
        };
        star(3);
        bool done = false;
        if (bdist == 1)
        {
            if (bpn)
            {
                const int saved = bcost;
                two_points();
                done = bcost == saved;
            }
            else
                done = true;
        }
        if (!done)
        {
            if (bdist > 5)
            {
                // raster refinement; the 4th lane of each sad_x4 costs its MV with tmv << 3 (motion.cpp:993)
                for (int ty = miny; ty <= maxy; ty += 5)
                    for (int tx = minx; tx <= maxx; tx += 5)
                    {
                        if (tx + 15 <= maxx)
                        {
                            const int mx[4] = { tx, tx + 5, tx + 10, tx + 15 }, my[4] = { ty, ty, ty, ty };
                            int c[4];
                            fpel_sads<P, G, 4>(s, mx, my, c);
#pragma unroll
                            for (int q = 0; q < 4; q++)
                            {
                                const int cq = c[q] + s.mvcost((q == 3 ? 8 : 4) * mx[q], (q == 3 ? 8 : 4) * ty);
                                if (cq < bcost) { bcost = cq; bx = mx[q]; by = ty; }
                            }
                            tx += 15;
                        }
                        else
                        {
                            const int c = fpel_sad<P, G>(s, tx, ty) + s.mvcost(4 * tx, 4 * ty);
                            if (c < bcost) { bcost = c; bx = tx; by = ty; }
                        }
                    }
            }
            while (bdist > 0)
            {
                bdist = 0;
                bpn = 0;
                star(32);
                if (bdist == 1)
                {
                    if (bpn) two_points();
                    break;
                }
            }
        }
    }
    else
    {
    bool do_hex = true;
    int hex_range = a.merange;            // UMH rescales merange before its goto me_hex2
    if (a.method == 4)
    {
        // FULL: k_full_search left the first raster-order minimum of the range in out_mv / out_cost
        const int fcost = a.out_cost[j];
        if (fcost < bcost) { bcost = fcost; bx = a.out_mv[2 * j]; by = a.out_mv[2 * j + 1]; }
        do_hex = false;
    }
    else if (a.method == 3)
    {
        // UMH (motion.cpp:744-926), in lockstep on the group; `break`s of the reference leave the
        // search (do_hex = false), its `goto me_hex2` continues with the hexagon search below
        auto ca = [&](int x, int y) { return fpel_sad<P, G>(s, x, y) + s.mvcost(4 * x, 4 * y); };
        auto cost_mv = [&](int x, int y) {
            const int c = ca(x, y);
            if (c < bcost) { bcost = c; bx = x; by = y; }
        };
        int ox = bx, oy = by;
        auto cost_x4 = [&](int a0, int b0, int a1, int b1, int a2, int b2, int a3, int b3) __attribute__((always_inline)) {
            const int mx[4] = { ox + a0, ox + a1, ox + a2, ox + a3 }, my[4] = { oy + b0, oy + b1, oy + b2, oy + b3 };
            int c[4];
            fpel_costs<P, G, 4>(s, mx, my, c);
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (c[q] < bcost) { bcost = c[q]; bx = mx[q]; by = my[q]; }
        };
        auto dia1 = [&](int mx, int my) { ox = mx; oy = my; cost_x4(0, -1, 0, 1, -1, 0, 1, 0); };
        auto cross = [&](int start, int xm, int ym) {
            int i = start;
            if (xm <= min(maxx - ox, ox - minx))
                for (; i < xm - 2; i += 4) cost_x4(i, 0, -i, 0, i + 2, 0, -i - 2, 0);
            for (; i < xm; i += 2)
            {
                if (ox + i <= maxx) cost_mv(ox + i, oy);
                if (ox - i >= minx) cost_mv(ox - i, oy);
            }
            i = start;
            if (ym <= min(maxy - oy, oy - miny))
                for (; i < ym - 2; i += 4) cost_x4(0, i, 0, -i, 0, i + 2, 0, -i - 2);
            for (; i < ym; i += 2)
            {
                if (oy + i <= maxy) cost_mv(ox, oy + i);
                if (oy - i >= miny) cost_mv(ox, oy - i);
            }
        };
        const int scale = (a.h * a.h) >> 4;                 // sizeScale[partEnum] (motion.cpp:121-150)
        auto thresh = [&](int v) { return bcost < ((v >> 4) * scale); };
        const int fpx = (pmx + 2) >> 2, fpy = (pmy + 2) >> 2;   // pmv.roundToFPel()
        int cross_start = 1, merange = a.merange;
        const int ucost1 = bcost;
        dia1(fpx, fpy);
        if (fpx | fpy) dia1(0, 0);
        const int ucost2 = bcost;
        if ((bx | by) && (bx != fpx || by != fpy)) dia1(bx, by);
        if (bcost == ucost2) cross_start = 3;
        ox = bx; oy = by;
        bool go = true;
        if (bcost == ucost2 && thresh(2000))
        {
            cost_x4(0, -2, -1, -1, 1, -1, -2, 0);
            cost_x4(2, 0, -1, 1, 1, 1, 0, 2);
            if (bcost == ucost1 && thresh(500)) go = false;
            else if (bcost == ucost2)
            {
                const int r = (merange >> 1) | 1;
                cross(3, r, r);
                cost_x4(-1, -2, 1, -2, -2, -1, 2, -1);
                cost_x4(-2, 1, 2, 1, -1, 2, 1, 2);
                if (bcost == ucost2) go = false;
                else cross_start = r + 2;
            }
        }
        if (go)
        {
            if (nc)
            {
                // adaptive range from the candidates' agreement (motion.cpp:785-834)
                const int qmx = s.mvpx, qmy = s.mvpy;
                const int16_t* mc = a.mvc + 2 * j * a.max_cand;
                const bool is64 = a.w == 64 && a.h == 64;
                int mvd, denom = 1;
                if (nc == 1)
                    mvd = is64 ? 25 : abs(qmx - mc[0]) + abs(qmy - mc[1]);
                else
                {
                    denom = nc - 1;
                    mvd = 0;
                    if (!is64)
                    {
                        mvd = abs(qmx - mc[0]) + abs(qmy - mc[1]);
                        denom++;
                    }
                    for (int k = 0; k < nc - 1; k++)
                        mvd += abs(mc[2 * k] - mc[2 * k + 2]) + abs(mc[2 * k + 1] - mc[2 * k + 3]);
                }
                const int sad_ctx = thresh(1000) ? 0 : thresh(2000) ? 1 : thresh(4000) ? 2 : 3;
                const int mvd_ctx = mvd < 10 * denom ? 0 : mvd < 20 * denom ? 1 : mvd < 40 * denom ? 2 : 3;
                // range_mul[4][4] = {{3,3,4,4},{3,4,4,4},{4,4,4,5},{4,4,5,6}} as nibbles
                constexpr uint64_t RM = 0x6544544444434433ull;
                merange = (merange * (int)((RM >> (4 * (4 * mvd_ctx + sad_ctx))) & 15)) >> 2;
            }
            cross(cross_start, merange, merange >> 1);
            cost_x4(-2, -2, -2, 2, 2, -2, 2, 2);
            // hexagon grid (motion.cpp:866-921): hex4[k] as nibbles (value + 4)
            constexpr uint64_t HX = 0x6280808080806244ull, HY = 0x7766554433221180ull;
            ox = bx; oy = by;
            int gi = 1;
            do
            {
                const int lim = min(min(maxx - ox, ox - minx), min(maxy - oy, oy - miny));
                if (4 * gi > lim)
                {
                    for (int k = 0; k < 16; k++)
                    {
                        const int cx = ox + ((int)((HX >> (4 * k)) & 15) - 4) * gi;
                        const int cy = oy + ((int)((HY >> (4 * k)) & 15) - 4) * gi;
                        if (cx >= minx && cx <= maxx && cy >= miny && cy <= maxy) cost_mv(cx, cy);
                    }
                }
                else
                {
                    int dir = 0;
                    for (int k = 0; k < 16; k++)
                    {
                        const int hx = (int)((HX >> (4 * k)) & 15) - 4, hy = (int)((HY >> (4 * k)) & 15) - 4;
                        const int c = ca(ox + hx * gi, oy + hy * gi);
                        if (c < bcost) { bcost = c; dir = hx * 16 + (hy & 15); }
                    }
                    if (dir)
                    {
                        bx = ox + gi * (dir >> 4);
                        by = oy + gi * ((int)((uint32_t)dir << 28) >> 28);
                    }
                }
            } while (++gi <= merange >> 2);
            do_hex = bx >= minx && bx <= maxx && by >= miny && by <= maxy;
            hex_range = merange;
        }
        else
            do_hex = false;
    }
    if (do_hex)
    {
        // the six hexagon points at once (motion.cpp:1077-1089: two sad_x3), then the tie-ordered updates
        {
            const int mx[6] = { bx - 2, bx - 1, bx + 1, bx + 2, bx + 1, bx - 1 };
            const int my[6] = { by, by + 2, by + 2, by, by - 2, by - 2 };
            int c[6];
            fpel_costs<P, G, 6>(s, mx, my, c);
            bcost <<= 3;
#pragma unroll
            for (int q = 0; q < 6; q++)
                if ((c[q] << 3) + 2 + q < bcost) bcost = (c[q] << 3) + 2 + q;
        }
        if (bcost & 7)
        {
            int dir = (bcost & 7) - 2;
            bx += hex_dx(dir + 1); by += hex_dy(dir + 1);
            for (int i = (hex_range >> 1) - 1; i > 0 && bx >= minx && bx <= maxx && by >= miny && by <= maxy; i--)
            {
                const int mx[3] = { bx + hex_dx(dir), bx + hex_dx(dir + 1), bx + hex_dx(dir + 2) };
                const int my[3] = { by + hex_dy(dir), by + hex_dy(dir + 1), by + hex_dy(dir + 2) };
                int c[3];
                fpel_costs<P, G, 3>(s, mx, my, c);
                bcost &= ~7;
                if ((c[0] << 3) + 1 < bcost) bcost = (c[0] << 3) + 1;
                if ((c[1] << 3) + 2 < bcost) bcost = (c[1] << 3) + 2;
                if ((c[2] << 3) + 3 < bcost) bcost = (c[2] << 3) + 3;
                if (!(bcost & 7)) break;
                dir += (bcost & 7) - 2;
                dir = dir < 0 ? dir + 6 : (dir > 5 ? dir - 6 : dir);   // mod6m1[dir + 1]
                bx += hex_dx(dir + 1); by += hex_dy(dir + 1);
            }
        }
        bcost >>= 3;
        int sdir = 0;
#pragma unroll
        for (int k0 = 1; k0 <= 8; k0 += 4)
        {
            const int mx[4] = { bx + sq_dx(k0), bx + sq_dx(k0 + 1), bx + sq_dx(k0 + 2), bx + sq_dx(k0 + 3) };
            const int my[4] = { by + sq_dy(k0), by + sq_dy(k0 + 1), by + sq_dy(k0 + 2), by + sq_dy(k0 + 3) };
            int c[4];
            fpel_costs<P, G, 4>(s, mx, my, c);
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (c[q] < bcost) { bcost = c[q]; sdir = k0 + q; }
        }
        bx += sq_dx(sdir); by += sq_dy(sdir);
    }
    }
    int qx, qy;
    if (bprecost < bcost) { qx = bpx; qy = bpy; bcost = bprecost; }
    else { qx = 4 * bx; qy = 4 * by; }
    // workload[subme] (motion.cpp:48-58): {hpel_iters, hpel_dirs, qpel_iters, qpel_dirs, hpel_satd}
    const int4 wl = subpel_workload(a.subme);
    const bool hsatd = a.subme >= 2;
    if (!bcost)
        bcost = s.mvcost(qx, qy);
    else
    {
        // one refinement round: directions 1 .. ndir at distance d, the first strictly smaller cost wins
        // (motion.cpp:700-760); 8-bit costs four directions per call
        auto refine = [&](int d, int ndir, bool satd) {
            int bdir = 0;
            if constexpr (sizeof(P) == 1 && X265AMD_ME_SPB)
            {
                for (int i0 = 1; i0 <= ndir; i0 += 4)
                {
                    s.nsp += 4;
                    const P* r;
                    int64_t rs;
                    spsrc((qx - d) >> 2, (qy - d) >> 2, r, rs);
                    const int4 c4 = subpel_cost4<P, G>(r, s.fenc, (int)rs, (int)s.fs, s.lane | s.nu << 8,
                                                       a.w | a.h << 8, a.depth | (s.chroma ? 256 : 0), s.fc[0],
                                                       s.fc[1], s.rc[0], s.rc[1], (int)s.fcs, (int)s.rcs, qx, qy, d,
                                                       i0, satd);
                    const int cc[4] = { c4.x, c4.y, c4.z, c4.w };
#pragma unroll
                    for (int q = 0; q < 4; q++)
                    {
                        const int i = i0 + q, tx = qx + d * sq_dx(i), ty = qy + d * sq_dy(i);
                        const int c = cc[q] + s.mvcost(tx, ty);
                        if (c < bcost) { bcost = c; bdir = i; }
                    }
                }
            }
            else
            {
                for (int i = 1; i <= ndir; i++)
                {
                    const int tx = qx + d * sq_dx(i), ty = qy + d * sq_dy(i);
                    const int c = spc(tx, ty, satd) + s.mvcost(tx, ty);
                    if (c < bcost) { bcost = c; bdir = i; }
                }
            }
            return bdir;
        };
        if (hsatd) bcost = spc(qx, qy, true) + s.mvcost(qx, qy);
        for (int it = 0; it < wl.x; it++)
        {
            const int bdir = refine(2, wl.y, hsatd);
            if (!bdir) break;
            qx += 2 * sq_dx(bdir); qy += 2 * sq_dy(bdir);
        }
        if (!hsatd) bcost = spc(qx, qy, true) + s.mvcost(qx, qy);
        for (int it = 0; it < wl.z; it++)
        {
            const int bdir = refine(1, wl.w, true);
            if (!bdir) break;
            qx += sq_dx(bdir); qy += sq_dy(bdir);
        }
    }
    if (s.lane == 0)
    {
        a.out_mv[2 * j] = (int16_t)qx;
        a.out_mv[2 * j + 1] = (int16_t)qy;
        a.out_cost[j] = bcost;
        if (a.evals)
        {
            a.evals[2 * j] = s.nfp;
            a.evals[2 * j + 1] = s.nsp;
        }
    }
}

// FULL search (motion.cpp:1039-1074) as a data-parallel argmin: one block per PU over candidate
// tiles of kFsTx x kFsTy integer MVs.  The tile's reference window and the PU's source block are
// staged in LDS; each thread costs 4 horizontally adjacent MVs of one row (v_sad_u8 / v_sad_u16 on
// byte-aligned windows of two / four LDS dwords).  The block keeps the minimum of (cost, raster
// index) — the first raster-order minimum, which is what the reference's strict-less scan leaves —
// and writes it to out_mv / out_cost, where k_motion_search picks it up against the predictors.
constexpr int kFsTx = 64, kFsTy = 16;

template <typename P>
__global__ __launch_bounds__(256) void k_full_search(const MeArgs a)
{
    constexpr int WSMAX = kFsTx + 64 + 4;
    __shared__ uint32_t win[(kFsTy + 63) * WSMAX * sizeof(P) / 4];
    __shared__ uint32_t fen[64 * 64 * sizeof(P) / 4];
    __shared__ uint32_t red[8];
    const int j = blockIdx.x, t = threadIdx.x;
    const int w = a.w, h = a.h;
    const P* ref = (const P*)a.ref + a.ref_off[j];
    const P* fenc = (const P*)a.fenc + a.fenc_off[j];
    const uint16_t* tab = a.mvcost + a.mvcost_off[j];
    const int mvpx = a.mvp[2 * j], mvpy = a.mvp[2 * j + 1];
    const int minx = a.mv_range[4 * j], miny = a.mv_range[4 * j + 1];
    const int ncx = a.mv_range[4 * j + 2] - minx + 1, ncy = a.mv_range[4 * j + 3] - miny + 1;
    const int WS = kFsTx + w + 4;                       // window row stride (pixels, multiple of 4)
    P* fl = (P*)fen;
    P* wl = (P*)win;
    for (int i = t; i < w * h; i += 256) fl[i] = fenc[(int64_t)(i / w) * a.fs + i % w];
    const int q = t & 15, r = t >> 4;
    uint32_t bkey_hi = 0xffffffffu, bkey_lo = 0xffffffffu;   // (cost, raster index)
    for (int ty0 = 0; ty0 < ncy; ty0 += kFsTy)
        for (int tx0 = 0; tx0 < ncx; tx0 += kFsTx)
        {
            const int wr = min(kFsTy, ncy - ty0) + h - 1, wc = min(kFsTx, ncx - tx0) + w - 1;
            const P* src = ref + (minx + tx0) + (int64_t)(miny + ty0) * a.rs;
            __syncthreads();
            for (int i = t; i < wr * wc; i += 256)
            {
                const int y = i / wc, x = i - y * wc;
                wl[y * WS + x] = src[x + (int64_t)y * a.rs];
            }
            __syncthreads();
            const int cy = ty0 + r, cx = tx0 + 4 * q;
            if (cy >= ncy || cx >= ncx) continue;
            uint32_t acc[4] = { 0, 0, 0, 0 };
            if constexpr (sizeof(P) == 1)
            {
                for (int rr = 0; rr < h; rr++)
                {
                    const uint32_t* wp = win + ((r + rr) * WS + 4 * q) / 4;
                    const uint32_t* fp = fen + rr * (w / 4);
                    uint32_t d0 = wp[0];
                    for (int c = 0; c < w / 4; c++)
                    {
                        const uint32_t d1 = wp[c + 1], f = fp[c];
                        acc[0] = __builtin_amdgcn_sad_u8(f, d0, acc[0]);
                        acc[1] = __builtin_amdgcn_sad_u8(f, __builtin_amdgcn_alignbyte(d1, d0, 1), acc[1]);
                        acc[2] = __builtin_amdgcn_sad_u8(f, __builtin_amdgcn_alignbyte(d1, d0, 2), acc[2]);
                        acc[3] = __builtin_amdgcn_sad_u8(f, __builtin_amdgcn_alignbyte(d1, d0, 3), acc[3]);
                        d0 = d1;
                    }
                }
            }
            else
            {
                for (int rr = 0; rr < h; rr++)
                {
                    const uint32_t* wp = win + ((r + rr) * WS + 4 * q) / 2;
                    const uint32_t* fp = fen + rr * (w / 2);
                    uint32_t e0 = wp[0], e1 = wp[1];
                    for (int c = 0; c < w / 4; c++)
                    {
                        const uint32_t e2 = wp[2 * c + 2], e3 = wp[2 * c + 3], f0 = fp[2 * c], f1 = fp[2 * c + 1];
                        const uint32_t g1 = __builtin_amdgcn_alignbyte(e1, e0, 2), g2 = __builtin_amdgcn_alignbyte(e2, e1, 2);
                        const uint32_t g3 = __builtin_amdgcn_alignbyte(e3, e2, 2);
                        acc[0] = __builtin_amdgcn_sad_u16(f1, e1, __builtin_amdgcn_sad_u16(f0, e0, acc[0]));
                        acc[1] = __builtin_amdgcn_sad_u16(f1, g2, __builtin_amdgcn_sad_u16(f0, g1, acc[1]));
                        acc[2] = __builtin_amdgcn_sad_u16(f1, e2, __builtin_amdgcn_sad_u16(f0, e1, acc[2]));
                        acc[3] = __builtin_amdgcn_sad_u16(f1, g3, __builtin_amdgcn_sad_u16(f0, g2, acc[3]));
                        e0 = e2; e1 = e3;
                    }
                }
            }
            const int my = 4 * (miny + cy) - mvpy;
#pragma unroll
            for (int k = 0; k < 4; k++)
            {
                if (cx + k >= ncx) break;
                const uint32_t cost = acc[k] + (uint16_t)(tab[4 * (minx + cx + k) - mvpx] + tab[my]);
                const uint32_t idx = (uint32_t)(cy * ncx + cx + k);
                if (cost < bkey_hi || (cost == bkey_hi && idx < bkey_lo)) { bkey_hi = cost; bkey_lo = idx; }
            }
        }
    // block argmin of (cost, index): wave shuffles, then the 4 waves through LDS
    for (int m = 32; m > 0; m >>= 1)
    {
        const uint32_t oh = __shfl_xor(bkey_hi, m, 64), ol = __shfl_xor(bkey_lo, m, 64);
        if (oh < bkey_hi || (oh == bkey_hi && ol < bkey_lo)) { bkey_hi = oh; bkey_lo = ol; }
    }
    if ((t & 63) == 0) { red[2 * (t >> 6)] = bkey_hi; red[2 * (t >> 6) + 1] = bkey_lo; }
    __syncthreads();
    if (t == 0)
    {
        for (int k = 1; k < 4; k++)
            if (red[2 * k] < bkey_hi || (red[2 * k] == bkey_hi && red[2 * k + 1] < bkey_lo))
            {
                bkey_hi = red[2 * k]; bkey_lo = red[2 * k + 1];
            }
        if (bkey_hi == 0xffffffffu)
            a.out_cost[j] = 0x7fffffff;                  // empty range: the predictors stand
        else
        {
            a.out_mv[2 * j] = (int16_t)(minx + (int)(bkey_lo % (uint32_t)ncx));
            a.out_mv[2 * j + 1] = (int16_t)(miny + (int)(bkey_lo / (uint32_t)ncx));
            a.out_cost[j] = (int32_t)bkey_hi;
        }
    }
}

// largest group of lanes per search (X265AMD_ME_GMAX: 256, the default, or 128 for a search over up to four /
// two wavefronts of one workgroup — a lane per 4x4 unit up to 64x64, so each candidate's compare is a quarter
// of the dependent instructions of one wave holding four units per lane; 64 = one wave per search).  Pinned
// 2160p medium encode: kernel 0.055 -> 0.034 ms per launch, 10.9-11.3 -> 11.2-11.7 fps, identical bitstreams
// (profiles/r05/z/gmax_ab.txt)
static int me_gmax()
{
    static int v = 0;
    if (!v)
    {
        const char* e = getenv("X265AMD_ME_GMAX");
        const int g = e ? atoi(e) : 256;
        v = g >= 256 ? 256 : g >= 128 ? 128 : 64;
    }
    return v;
}

// search windows in LDS (X265AMD_ME_LDS_R = r > 0; read at every launch, default 0 = off) for the
// one-search-per-workgroup sizes (G = 128 / 256: PUs of 128 or more 4x4 units) of DIA / HEX searches: once the
// search start is known, the reference around it (r pixels either way, within the MV range box) is staged in
// LDS and every later candidate there reads LDS instead of taking an L2 / HBM round trip.  The window is at
// most (2r + w + 17) x (2r + h + 17) pixels (64x64, r 16: 14 KB at 8-bit).  Bit-exact (test_me.py), but
// measured slower in the running encoder — 0.026 ms per launch without, 0.032-0.035 with r = 8 / 16 / 32 / the
// whole range (profiles/r06/me_lds_window_ab.txt): the reads go through flat (generic) addressing and the
// staging round trip costs more than the L2 hits it replaces.
static int me_lds_r()
{
    const char* e = getenv("X265AMD_ME_LDS");
    const char* r = getenv("X265AMD_ME_LDS_R");
    const int v = (e && atoi(e) == 0) ? 0 : r ? atoi(r) : 0;
    return v < 0 ? 0 : v;
}
constexpr int kMeWinMaxBytes = 64 * 1024;

template <typename P>
static int launch_me(MeArgs a, hipStream_t st)
{
    if (a.method == 4)
        hipLaunchKernelGGL((k_full_search<P>), dim3(a.n), dim3(256), 0, st, a);
    const int G = 1 << a.lg;
    const int spb = G > 64 ? 1 : X265AMD_BLOCK / G;
    const uint32_t blocks = (uint32_t)((a.n + spb - 1) / spb);
    const int threads = G > 64 ? G : X265AMD_BLOCK;
    a.win_bytes = 0;
    const int lr = me_lds_r();
    a.win_r = lr < a.merange ? lr : a.merange;
    if (G > 64 && (a.method == 0 || a.method == 1) && a.win_r > 0 && (a.rs * (int64_t)sizeof(P)) % 16 == 0)
    {
        const int64_t ww = 2 * (int64_t)a.win_r + a.w + 17, wh = 2 * (int64_t)a.win_r + a.h + 17;
        const int64_t bytes = ((ww * (int64_t)sizeof(P) + 30) >> 4) * 16 * wh;
        if (bytes <= kMeWinMaxBytes) a.win_bytes = (int)bytes;
    }
    if (a.win_bytes)
    {
        if (G == 128) hipLaunchKernelGGL((k_motion_search<P, 128, true>), dim3(blocks), dim3(threads), a.win_bytes, st, a);
        else hipLaunchKernelGGL((k_motion_search<P, 256, true>), dim3(blocks), dim3(threads), a.win_bytes, st, a);
        return (int)hipGetLastError();
    }
#define L(g) case g: hipLaunchKernelGGL((k_motion_search<P, g>), dim3(blocks), dim3(threads), 0, st, a); break;
    switch (G)
    {
        L(4) L(8) L(16) L(32) L(64) L(128) L(256)
    default: return X265AMD_EINVAL;
    }
#undef L
    return (int)hipGetLastError();
}

} // namespace x265amd

using namespace x265amd;

extern "C" int x265amd_motion_search(int depth, int count, const x265amd_me_batch* bt, void* stream)
{
    if ((depth != 8 && depth != 10 && depth != 12) || count < 0 || (count && !bt)) return X265AMD_EINVAL;
    for (int i = 0; i < count; i++)
    {
        const x265amd_me_batch& b = bt[i];
        if (b.n < 0 || b.w < 4 || b.h < 4 || b.w > 64 || b.h > 64 || (b.w & 3) || (b.h & 3)) return X265AMD_EINVAL;
        if (b.method < 0 || b.method > 4 || b.subme < 0 || b.subme > 7 || b.merange < 1) return X265AMD_EINVAL;
        if (b.n && b.fenc_cb && (!b.fenc_cr || !b.fenc_coff || !b.ref_cb || !b.ref_cr || !b.ref_coff))
            return X265AMD_EINVAL;
        if (b.n && (!b.fenc || !b.fenc_off || !b.ref || !b.ref_off || !b.mv_range || !b.mvp || !b.mvcost ||
                    !b.mvcost_off || !b.out_mv || !b.out_cost || (b.num_cand && (!b.mvc || b.max_cand < 1))))
            return X265AMD_EINVAL;
    }
    hipStream_t st = (hipStream_t)stream;
    int live = 0;
    for (int i = 0; i < count; i++) live += bt[i].n > 0;
    // batches of different PU sizes are independent: they run concurrently on internal streams
    // joined back into `stream` (a latency-bound 64x64 search overlaps the small-PU batches)
    ForkJoin fj(st, live);
    if (fj.err != hipSuccess) return (int)fj.err;
    int k = 0;
    for (int i = 0; i < count; i++)
    {
        const x265amd_me_batch& b = bt[i];
        if (!b.n) continue;
        const hipStream_t bs = fj.stream(k++);
        const int units = (b.w / 4) * (b.h / 4);
        int g = 4, lg = 2;                               // groups of at least 4 lanes (fewer kernel variants)
        while (g < units && g < me_gmax()) { g <<= 1; lg++; }
        if ((units + g - 1) / g > kMeMaxUnits) return X265AMD_EINVAL;
        MeArgs a{ b.fenc, b.fenc_off, (int64_t)b.fenc_stride, b.ref, b.ref_off, (int64_t)b.ref_stride, b.mv_range,
                  b.mvp, b.mvc, b.num_cand, b.mvcost, b.mvcost_off, b.out_mv, b.out_cost, b.fenc_cb, b.fenc_cr,
                  (int64_t)b.fenc_cstride, b.fenc_coff, b.ref_cb, b.ref_cr, (int64_t)b.ref_cstride, b.ref_coff,
                  b.eval_count, b.w, b.h, b.n, lg, b.method, b.subme, b.merange, b.max_cand, depth, 0, 0 };
        const int rc = depth == 8 ? launch_me<uint8_t>(a, bs) : launch_me<uint16_t>(a, bs);
        if (rc) { fj.join(); return rc; }
    }
    return (int)fj.join();
}
