// loopfilter.hip — f4: the in-loop filters and border extension of
// device-resident 4:2:0 recon frames, as whole-frame passes instead of FrameFilter's CTU-row
// pipeline (framefilter.cpp:223-520):
//
//   x265amd_deblock        Deblock::deblockCTU (deblock.cpp:37-536): edge marks, boundary
//                          strength, luma strong / weak and chroma filters.  Two launches per
//                          call: every vertical edge of every frame, then every horizontal one
//                          (HEVC's order; x265's per-CTU V(c) / H(c-1) interleave is equivalent
//                          because a filter reads 4 and writes 3 pixels each side of an edge
//                          and edges are 8 apart).  One lane per 4-line edge segment: it
//                          derives the edge mark and bS from the two 16-byte CU units on either
//                          side, loads its 4 x 8 pixel window, filters in registers and stores
//                          the window back (windows tile the plane, so lanes never overlap).
//   x265amd_sao_apply      SAO::processSaoCu (sao.cpp:278-597): one wavefront per plane CTU, one
//                          lane per 8-pixel wide strip of it; neighbours come from the deblocked source buffer and the
//                          result goes to a second buffer, which is what the reference's
//                          m_tmpU / m_tmpL copies emulate in place.
//   x265amd_sao_stats      SAO::calcSaoStatsCu (sao.cpp:772-943): one wavefront per CTU, one lane
//                          per 8x8 strip; per pixel the five SAO types' classes; edge-offset
//                          classes accumulate in per-lane LDS bins, reduced across the wavefront,
//                          band classes go to LDS as packed (count << 40) + sum 64-bit adds.
//   x265amd_extend_border  extendPicBorder (pixel.cpp:908-922): side margins, then full-stride
//                          margin rows (second launch, so corners copy extended rows).
//
// All four are HBM-bound byte work: no MFMA, vector loads of whole row windows, the neighbour
// rows of a segment come from L2.
#include "common.h"
#include "../../../include/x265_amd.h"

#include <cstring>

namespace x265amd {

// Deblock::s_tcTable / s_betaTable (deblock.cpp:523-535), g_chromaScale (constants.cpp:335-339)
__constant__ uint8_t c_tc[54] = { 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                  2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20,
                                  22, 24 };
__constant__ uint8_t c_beta[52] = { 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 6, 7, 8, 9, 10, 11, 12, 13, 14,
                                    15, 16, 17, 18, 20, 22, 24, 26, 28, 30, 32, 34, 36, 38, 40, 42, 44, 46, 48, 50,
                                    52, 54, 56, 58, 60, 62, 64 };
__constant__ uint8_t c_chroma_scale[70] = { 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19,
                                            20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 33, 33, 34, 34,
                                            35, 35, 36, 36, 37, 37, 38, 39, 40, 41, 42, 43, 44, 45, 46, 47, 48, 49,
                                            50, 51, 51, 51, 51, 51, 51, 51, 51, 51, 51, 51, 51, 51 };

// frame descriptors per launch: they travel in the kernarg segment (<= 4 KiB), so a launch covers
// as many frames as fit and a call of many frames costs few launches
constexpr int kMaxFrames = 32;
constexpr int kDbkFrames = 16;
constexpr int kStatFrames = 24;

// clip3, sgn, load_row10 and the SAO statistics of one CTU (sao_stats_wave), shared with tu.hip's server
#include "saostats.h"
// the compare form, kept where it measured faster (SAO apply: its selects fold into the offset pick)
__device__ __forceinline__ int sgn_cmp(int v) { return (v > 0) - (v < 0); }
__device__ __forceinline__ int iabs(int v) { return v < 0 ? -v : v; }

// which frame of the launch a logical block belongs to (uniform scan, as group_sub)
template <int N, typename L>
__device__ __forceinline__ int frame_of(const L& l, uint32_t b)
{
    int f = 0;
#pragma unroll
    for (int i = 1; i < N; i++)
        if (i < l.count && l.f[i].block0 <= b) f = i;
    return f;
}

// ================================================================ deblocking
struct DbkFrame
{
    void* plane[3];
    int64_t stride, cstride;
    const x265amd_deblock_unit* units;
    int64_t us;
    int wu, hu;                       // picture width / band height in 4x4 units
    int uy0;                          // first unit row of the band (0: whole picture)
    int hs, vs;                       // chroma shifts (4:2:0 1/1, 4:2:2 1/0, 4:4:4 0/0)
    int is_p, beta2, tc2, cbqp, crqp, tqb;
    int32_t poc[2][16];
    uint32_t block0, nluma, nseg;     // first block; luma / all segments of this pass
};
struct DbkLaunch
{
    DbkFrame f[kDbkFrames];
    int count, maxv;
};

struct Unit
{
    int cu_log2, tu_log2, part, flags, qp, ref0, ref1, mv0x, mv0y, mv1x, mv1y;
    __device__ __forceinline__ Unit(const x265amd_deblock_unit* p)
    {
        const uint4 v = *(const uint4*)p;
        cu_log2 = v.x & 0xff; tu_log2 = (v.x >> 8) & 0xff; part = (v.x >> 16) & 0xff; flags = v.x >> 24;
        qp = (int8_t)(v.y & 0xff); ref0 = (int8_t)((v.y >> 8) & 0xff); ref1 = (int8_t)((v.y >> 16) & 0xff);
        mv0x = (int16_t)(v.z & 0xffff); mv0y = (int16_t)(v.z >> 16);
        mv1x = (int16_t)(v.w & 0xffff); mv1y = (int16_t)(v.w >> 16);
    }
};

// deblockCU's marks (deblock.cpp:72-191): CU edge bsCuEdge (2 inside the picture), TU edge 2,
// PU split 1 (setEdgefilterPU), in that priority
__device__ __forceinline__ int edge_mark(const Unit& u, int dir, int pos)
{
    const int cu = 1 << u.cu_log2;
    const int rel = pos & (cu - 1);
    if (!rel) return pos > 0 ? 2 : 0;
    if (!(pos & ((1 << u.tu_log2) - 1))) return 2;
    int pu = -1;
    switch (u.part)
    {
    case 1: pu = dir ? cu >> 1 : -1; break;
    case 2: pu = dir ? -1 : cu >> 1; break;
    case 3: pu = cu >> 1; break;
    case 4: pu = dir ? cu >> 2 : -1; break;
    case 5: pu = dir ? cu - (cu >> 2) : -1; break;
    case 6: pu = dir ? -1 : cu >> 2; break;
    case 7: pu = dir ? -1 : cu - (cu >> 2); break;
    default: break;
    }
    return rel == pu ? 1 : 0;
}

// m_refFrameList[list][refIdx] identity: refIdx -1 reads m_refFrameList[0][-1] = the Slice's m_pps
// (non-null, equal to no picture, MV kept) or m_refFrameList[1][-1] = m_refFrameList[0][MAX_NUM_REF]
// = NULL (MV zeroed) — slice.h:320-338
constexpr int64_t kKeyL0None = (int64_t)1 << 40;
constexpr int64_t kKeyNull = (int64_t)1 << 41;

__device__ __forceinline__ bool mvd(int ax, int ay, int bx, int by) { return iabs(ax - bx) >= 4 || iabs(ay - by) >= 4; }

// Deblock::getBoundaryStrength (deblock.cpp:193-252)
__device__ __forceinline__ int boundary_strength(const DbkFrame& f, const Unit& P, const Unit& Q, int mark)
{
    if ((P.flags | Q.flags) & 1) return 2;
    if (mark > 1 && ((P.flags | Q.flags) & 2)) return 1;
    const int64_t p0 = P.ref0 < 0 ? kKeyL0None : (int64_t)f.poc[0][P.ref0 & 15];
    const int64_t q0 = Q.ref0 < 0 ? kKeyL0None : (int64_t)f.poc[0][Q.ref0 & 15];
    const int mp0x = P.mv0x, mp0y = P.mv0y, mq0x = Q.mv0x, mq0y = Q.mv0y;
    if (f.is_p) return (p0 != q0 || mvd(mq0x, mq0y, mp0x, mp0y)) ? 1 : 0;
    const int64_t p1 = P.ref1 < 0 ? kKeyNull : (int64_t)f.poc[1][P.ref1 & 15];
    const int64_t q1 = Q.ref1 < 0 ? kKeyNull : (int64_t)f.poc[1][Q.ref1 & 15];
    const int mp1x = p1 != kKeyNull ? P.mv1x : 0, mp1y = p1 != kKeyNull ? P.mv1y : 0;
    const int mq1x = q1 != kKeyNull ? Q.mv1x : 0, mq1y = q1 != kKeyNull ? Q.mv1y : 0;
    if ((p0 == q0 && p1 == q1) || (p0 == q1 && p1 == q0))
    {
        const bool same = mvd(mq0x, mq0y, mp0x, mp0y) || mvd(mq1x, mq1y, mp1x, mp1y);
        const bool cross = mvd(mq1x, mq1y, mp0x, mp0y) || mvd(mq0x, mq0y, mp1x, mp1y);
        if (p0 != p1) return (p0 == q0 ? same : cross) ? 1 : 0;
        return (same && cross) ? 1 : 0;
    }
    return 1;
}

// the 4 lines x 8 pixels across one luma edge (v[l][i] = pixel i - 4 across the edge on line l)
template <typename P, int DIR>
__device__ __forceinline__ void load_window(const P* q, int64_t s, int (&v)[4][8])
{
    if constexpr (DIR == 0)
    {
#pragma unroll
        for (int l = 0; l < 4; l++) load_row<P, 8>(q + l * s - 4, v[l]);
    }
    else
    {
#pragma unroll
        for (int i = 0; i < 8; i++)
        {
            int r[4];
            load_row<P, 4>(q + (i - 4) * s, r);
#pragma unroll
            for (int l = 0; l < 4; l++) v[l][i] = r[l];
        }
    }
}

template <typename P, int DIR>
__device__ __forceinline__ void store_window(P* q, int64_t s, const int (&v)[4][8])
{
    if constexpr (DIR == 0)
    {
#pragma unroll
        for (int l = 0; l < 4; l++) store_row<P, 8>(q + l * s - 4, v[l]);
    }
    else
    {
#pragma unroll
        for (int i = 1; i < 7; i++)
        {
            const int r[4] = { v[0][i], v[1][i], v[2][i], v[3][i] };
            store_row<P, 4>(q + (i - 4) * s, r);
        }
    }
}

// Deblock::edgeFilterLuma's per-segment body (deblock.cpp:388-440) with pelFilterLumaStrong_c
// (loopfilter.cpp:141-162) and pelFilterLuma (deblock.cpp:283-326); returns false if untouched
__device__ __forceinline__ bool filter_luma(int (&v)[4][8], int bs, int qp, int maskP, int maskQ, int beta2,
                                            int tc2, int bd, int maxv)
{
    const int beta = (int)c_beta[clip3(0, 51, qp + beta2)] << bd;
    const int dp0 = iabs(v[0][1] - 2 * v[0][2] + v[0][3]), dq0 = iabs(v[0][4] - 2 * v[0][5] + v[0][6]);
    const int dp3 = iabs(v[3][1] - 2 * v[3][2] + v[3][3]), dq3 = iabs(v[3][4] - 2 * v[3][5] + v[3][6]);
    const int d0 = dp0 + dq0, d3 = dp3 + dq3;
    if (d0 + d3 >= beta) return false;
    const int tc = (int)c_tc[clip3(0, 53, qp + 2 * (bs - 1) + tc2)] << bd;
    const bool sw = 2 * d0 < (beta >> 2) && 2 * d3 < (beta >> 2) &&
                    iabs(v[0][0] - v[0][3]) + iabs(v[0][7] - v[0][4]) < (beta >> 3) &&
                    iabs(v[0][3] - v[0][4]) < ((tc * 5 + 1) >> 1) &&
                    iabs(v[3][0] - v[3][3]) + iabs(v[3][7] - v[3][4]) < (beta >> 3) &&
                    iabs(v[3][3] - v[3][4]) < ((tc * 5 + 1) >> 1);
    if (sw)
    {
        const int tcP = (2 * tc) & maskP, tcQ = (2 * tc) & maskQ;
#pragma unroll
        for (int l = 0; l < 4; l++)
        {
            const int m0 = v[l][0], m1 = v[l][1], m2 = v[l][2], m3 = v[l][3], m4 = v[l][4], m5 = v[l][5],
                      m6 = v[l][6], m7 = v[l][7];
            v[l][1] = clip3(-tcP, tcP, ((2 * m0 + 3 * m1 + m2 + m3 + m4 + 4) >> 3) - m1) + m1;
            v[l][2] = clip3(-tcP, tcP, ((m1 + m2 + m3 + m4 + 2) >> 2) - m2) + m2;
            v[l][3] = clip3(-tcP, tcP, ((m1 + 2 * m2 + 2 * m3 + 2 * m4 + m5 + 4) >> 3) - m3) + m3;
            v[l][4] = clip3(-tcQ, tcQ, ((m2 + 2 * m3 + 2 * m4 + 2 * m5 + m6 + 4) >> 3) - m4) + m4;
            v[l][5] = clip3(-tcQ, tcQ, ((m3 + m4 + m5 + m6 + 2) >> 2) - m5) + m5;
            v[l][6] = clip3(-tcQ, tcQ, ((m3 + m4 + m5 + 3 * m6 + 2 * m7 + 4) >> 3) - m6) + m6;
        }
        return true;
    }
    const int side = (beta + (beta >> 1)) >> 3;
    const int mP1 = (dp0 + dp3 < side ? -1 : 0) & maskP, mQ1 = (dq0 + dq3 < side ? -1 : 0) & maskQ;
    const int thr = tc * 10, tch = tc >> 1;
#pragma unroll
    for (int l = 0; l < 4; l++)
    {
        const int m1 = v[l][1], m2 = v[l][2], m3 = v[l][3], m4 = v[l][4], m5 = v[l][5], m6 = v[l][6];
        int delta = (9 * (m4 - m3) - 3 * (m5 - m2) + 8) >> 4;
        if (iabs(delta) >= thr) continue;
        delta = clip3(-tc, tc, delta);
        v[l][3] = clip3(0, maxv, m3 + (delta & maskP));
        v[l][4] = clip3(0, maxv, m4 - (delta & maskQ));
        if (mP1) v[l][2] = clip3(0, maxv, m2 + clip3(-tch, tch, (((m1 + m3 + 1) >> 1) - m2 + delta) >> 1));
        if (mQ1) v[l][5] = clip3(0, maxv, m5 + clip3(-tch, tch, (((m6 + m4 + 1) >> 1) - m5 - delta) >> 1));
    }
    return true;
}

// one segment = one 4-line piece of an edge.  Luma: VER edges at x = 8k (4 rows), HOR at y = 8k
// (4 columns).  Chroma (4:2:0): edges on the 8x8 chroma grid, 4 chroma lines per second luma unit
// of the edge (edgeFilterChroma's idx << chromaShift), Cb and Cr together, bS 2 only.
template <typename P, int DIR>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_deblock(const DbkLaunch L)
{
    const uint32_t b = xcd_block();
    const DbkFrame& f = L.f[frame_of<kDbkFrames>(L, b)];
    const uint32_t s = (b - f.block0) * X265AMD_BLOCK + threadIdx.x;
    if (s >= f.nseg) return;
    const bool luma = s < f.nluma;
    int ux, uy;
    if (luma)
    {
        if (DIR == 0) { const int n = f.wu >> 1; uy = (int)(s / n); ux = 2 * (int)(s % n); }
        else { ux = (int)(s % f.wu); uy = 2 * (int)(s / f.wu); }
    }
    else
    {
        // chroma edges on the chroma plane's 8x8 grid, one 4-line chroma segment per (1 << shift
        // along the edge) luma units (deblock.cpp:104-113, 479-480)
        const uint32_t c = s - f.nluma;
        if (DIR == 0)
        {
            const int sx = 2 << f.hs, n = (f.wu + sx - 1) / sx;
            uy = (int)(c / n) << f.vs;
            ux = sx * (int)(c % n);
        }
        else
        {
            const int n = f.wu >> f.hs;
            ux = (int)(c % n) << f.hs;
            uy = (2 << f.vs) * (int)(c / n);
        }
    }
    uy += f.uy0;
    const x265amd_deblock_unit* qu = f.units + uy * f.us + ux;
    const Unit Q(qu);
    const int mark = edge_mark(Q, DIR, DIR ? 4 * uy : 4 * ux);
    if (!mark) return;
    const Unit Pn(DIR ? qu - f.us : qu - 1);
    const int bs = boundary_strength(f, Pn, Q, mark);
    if (!bs || (!luma && bs < 2)) return;
    int maskP = -1, maskQ = -1;
    if (f.tqb)
    {
        maskP = (Pn.flags & 4) ? 0 : -1;
        maskQ = (Q.flags & 4) ? 0 : -1;
        if (!(maskP | maskQ)) return;
    }
    const int qp = (Pn.qp + Q.qp + 1) >> 1;
    const int bd = sizeof(P) == 1 ? 0 : (L.maxv == 1023 ? 2 : 4);
    if (luma)
    {
        P* q = (P*)f.plane[0] + (int64_t)(4 * uy) * f.stride + 4 * ux;
        int v[4][8];
        load_window<P, DIR>(q, f.stride, v);
        if (filter_luma(v, bs, qp, maskP, maskQ, f.beta2, f.tc2, bd, L.maxv)) store_window<P, DIR>(q, f.stride, v);
        return;
    }
    // edgeFilterChroma (deblock.cpp:443-521)
#pragma unroll
    for (int k = 0; k < 2; k++)
    {
        int qpc = qp + (k ? f.crqp : f.cbqp);
        if (qpc >= 30) qpc = (f.hs & f.vs) ? c_chroma_scale[qpc] : min(qpc, 51);
        const int tc = (int)c_tc[clip3(0, 53, qpc + 2 + f.tc2)] << bd;
        P* q = (P*)f.plane[1 + k] + (int64_t)((4 * uy) >> f.vs) * f.cstride + ((4 * ux) >> f.hs);
        int w[4][4];
        if (DIR == 0)
        {
#pragma unroll
            for (int l = 0; l < 4; l++) load_row<P, 4>(q + l * f.cstride - 2, w[l]);
        }
        else
        {
#pragma unroll
            for (int i = 0; i < 4; i++)
            {
                int r[4];
                load_row<P, 4>(q + (i - 2) * f.cstride, r);
#pragma unroll
                for (int l = 0; l < 4; l++) w[l][i] = r[l];
            }
        }
#pragma unroll
        for (int l = 0; l < 4; l++)
        {
            const int m2 = w[l][0], m3 = w[l][1], m4 = w[l][2], m5 = w[l][3];
            const int delta = clip3(-tc, tc, ((((m4 - m3) * 4) + m2 - m5 + 4) >> 3));
            w[l][1] = clip3(0, L.maxv, m3 + (delta & maskP));
            w[l][2] = clip3(0, L.maxv, m4 - (delta & maskQ));
        }
        if (DIR == 0)
        {
#pragma unroll
            for (int l = 0; l < 4; l++) store_row<P, 4>(q + l * f.cstride - 2, w[l]);
        }
        else
        {
#pragma unroll
            for (int i = 1; i < 3; i++)
            {
                const int r[4] = { w[0][i], w[1][i], w[2][i], w[3][i] };
                store_row<P, 4>(q + (i - 2) * f.cstride, r);
            }
        }
    }
}

// ================================================================ SAO apply
struct SaoFrame
{
    const void* src[3];
    void* dst[3];
    int64_t stride, cstride;
    const x265amd_sao_param* params;
    int w, h, ctu_log2, wc, nctu;
    int c0, nctu_all;                        // first CTU of the band, CTUs of the picture (params stride)
    uint8_t luma_on, chroma_on, i400;
    uint8_t hs, vs;                          // chroma shifts
    uint32_t block0;                         // first block (one per plane and CTU)
};
struct SaoLaunch
{
    SaoFrame f[kMaxFrames];
    int count, maxv, bo_shift;
};

// One wavefront per (plane, CTU), so the SAO type is uniform across it: lane = an 8-pixel wide
// strip of sh rows (sh = 8 for 64x64, 2 for 32x32, 1 below); the row above, the current row and
// the row below slide down the strip, one new 16-byte load per output row.
template <typename P>
__global__ __launch_bounds__(64) void k_sao_apply(const SaoLaunch L)
{
    const uint32_t b = xcd_block();
    const SaoFrame& f = L.f[frame_of<kMaxFrames>(L, b)];
    const uint32_t u = b - f.block0;                 // plane-major: [3][nctu]
    const int p = (int)(u / f.nctu), c = f.c0 + (int)(u % f.nctu);
    const int lane = threadIdx.x;
    const int pw = p ? f.w >> f.hs : f.w, ph = p ? f.h >> f.vs : f.h;
    const int csw = (1 << f.ctu_log2) >> (p ? f.hs : 0), csh = (1 << f.ctu_log2) >> (p ? f.vs : 0);
    const int nsx = csw >> 3, sh = csw * csh >= 512 ? (csw * csh) >> 9 : 1;
    const int cx0 = (c % f.wc) * csw, cy0 = (c / f.wc) * csh;
    const int x0 = cx0 + 8 * (lane % nsx), y0 = cy0 + sh * (lane / nsx);
    const int yend = min(min(y0 + sh, cy0 + csh), ph);
    if (x0 >= pw || y0 >= yend) return;
    const bool full = pw - x0 >= 8;                  // else 4 pixels (a right edge of width 8k + 4)
    if (p && f.i400) return;                         // 4:0:0: no chroma planes
    const int64_t st = p ? f.cstride : f.stride;
    const P* src = (const P*)f.src[p] + y0 * st + x0;
    P* dst = (P*)f.dst[p] + y0 * st + x0;
    const x265amd_sao_param* prm = f.params + p * f.nctu_all + c;
    int type = (int)prm->type;
    if (p == 2 && type >= 0) type = (int)f.params[f.nctu_all + c].type;   // processSaoCu(addr, typeIdxCb, 2)
    if (!(p ? f.chroma_on : f.luma_on)) type = -1;
    const int band = prm->band;
    const int o0 = prm->offset[0], o1 = prm->offset[1], o2 = prm->offset[2], o3 = prm->offset[3];
    // EO neighbour directions (sao.cpp:321-560): EO_0 -, EO_1 |, EO_2 135 deg, EO_3 45 deg
    const int dxa = type == 1 ? 0 : (type == 3 ? 1 : -1), dxb = -dxa;   // above / below
    int up[10], mid[10], dn[10];
    load_row10<P>(src - st, up);
    load_row10<P>(src, mid);
#pragma unroll
    for (int yy = 0; yy < 8; yy++)
    {
        const int y = y0 + yy;
        if (y >= yend) break;
        load_row10<P>(src + (yy + 1) * st, dn);
        int o[8];
        if (type == 4)
        {
            // m_offsetBo: offset[i] at band (bandPos + i) & 31 (sao.cpp:637-640)
#pragma unroll
            for (int i = 0; i < 8; i++)
            {
                const int v = mid[i + 1];
                const int k = ((v >> L.bo_shift) - band) & 31;
                const int off = k == 0 ? o0 : k == 1 ? o1 : k == 2 ? o2 : k == 3 ? o3 : 0;
                o[i] = clip3(0, L.maxv, v + off);
            }
        }
        else if (type >= 0)
        {
            // m_offsetEo via s_eoTable (sao.cpp:65-72, 644-650): edge type 0, 1, 3, 4 -> offset[0..3], 2 -> 0;
            // EO leaves the picture's outermost column (not EO_1) / row (not EO_0) untouched
            const bool skip_row = type != 0 && (y == 0 || y == ph - 1);
#pragma unroll
            for (int i = 0; i < 8; i++)
            {
                const int v = mid[i + 1];
                const int na = type == 0 ? mid[i] : (dxa < 0 ? up[i] : (dxa > 0 ? up[i + 2] : up[i + 1]));
                const int nb = type == 0 ? mid[i + 2] : (dxb < 0 ? dn[i] : (dxb > 0 ? dn[i + 2] : dn[i + 1]));
                const int e = sgn_cmp(v - na) + sgn_cmp(v - nb) + 2;
                const int off = e == 0 ? o0 : e == 1 ? o1 : e == 3 ? o2 : e == 4 ? o3 : 0;
                const int x = x0 + i;
                const bool skip = skip_row || (type != 1 && (x == 0 || x == pw - 1));
                o[i] = skip ? v : clip3(0, L.maxv, v + off);
            }
        }
        else
        {
#pragma unroll
            for (int i = 0; i < 8; i++) o[i] = mid[i + 1];
        }
        P* d = dst + yy * st;
        if (full) store_row<P, 8>(d, o);
        else
        {
            const int o4[4] = { o[0], o[1], o[2], o[3] };
            store_row<P, 4>(d, o4);
        }
#pragma unroll
        for (int i = 0; i < 10; i++) { up[i] = mid[i]; mid[i] = dn[i]; }
    }
}

// ================================================================ SAO statistics
struct StatFrame
{
    const void* fenc[3];
    const void* rec[3];
    int64_t fs, fcs, rs, rcs;
    int32_t* stats;
    int32_t* count;
    int w, h, ctu_log2, wc, nd;
    int hs, vs;                              // chroma shifts
    uint32_t block0, nctu;
};
struct StatLaunch
{
    StatFrame f[kStatFrames];
    int count, bo_shift;
};

// One wavefront per CTU (saostats.h sao_stats_wave): the CTU's planes seen through the frame's planes
template <typename P>
__global__ __launch_bounds__(64) void k_sao_stats(const StatLaunch L)
{
    const uint32_t b = xcd_block();
    const StatFrame& f = L.f[frame_of<kStatFrames>(L, b)];
    const uint32_t c = b - f.block0;
    const int cxi = (int)(c % f.wc), cyi = (int)(c / f.wc);
    SaoCtuView v;
    v.nd = f.nd;
    for (int pc = 0; pc < 2; pc++)
    {
        v.pw[pc] = pc ? f.w >> f.hs : f.w;
        v.ph[pc] = pc ? f.h >> f.vs : f.h;
        v.csw[pc] = (1 << f.ctu_log2) >> (pc ? f.hs : 0);
        v.csh[pc] = (1 << f.ctu_log2) >> (pc ? f.vs : 0);
        v.x0[pc] = cxi * v.csw[pc];
        v.y0[pc] = cyi * v.csh[pc];
    }
    for (int p = 0; p < 3; p++)
    {
        const int pc = p ? 1 : 0;
        v.rs[p] = p ? f.rcs : f.rs;
        v.fs[p] = p ? f.fcs : f.fs;
        v.rec[p] = (const P*)f.rec[p] + (int64_t)v.y0[pc] * v.rs[p] + v.x0[pc];
        v.fenc[p] = (const P*)f.fenc[p] + (int64_t)v.y0[pc] * v.fs[p] + v.x0[pc];
    }
    sao_stats_wave<P>(v, L.bo_shift, f.stats + (int64_t)c * 3 * 5 * 33, f.count + (int64_t)c * 3 * 5 * 33);
}

// ================================================================ border extension
struct BorderPlane
{
    void* p;
    int64_t stride;
    int w, h, mx, my;
    int y0, nr, top, bottom;                 // side margins of rows [y0, y0 + nr); which margin rows
    uint32_t block0_lr, block0_tb;
};
constexpr int kMaxPlanes = 16;
struct BorderLaunch
{
    BorderPlane f[kMaxPlanes];
    int count;
};

// extendRowBorder (ipfilter.cpp:59-77): one lane per (row, side)
template <typename P>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_border_lr(const BorderLaunch L)
{
    const uint32_t b = xcd_block();
    int i = 0;
#pragma unroll
    for (int k = 1; k < kMaxPlanes; k++)
        if (k < L.count && L.f[k].block0_lr <= b) i = k;
    const BorderPlane& f = L.f[i];
    const int64_t t = (int64_t)(b - f.block0_lr) * X265AMD_BLOCK + threadIdx.x;
    if (t >= 2 * (int64_t)f.nr) return;
    const bool right = t >= f.nr;
    const int y = f.y0 + (int)(right ? t - f.nr : t);
    P* row = (P*)f.p + y * f.stride;
    const P v = right ? row[f.w - 1] : row[0];
    P* d = right ? row + f.w : row - f.mx;
    int x = 0;
    if constexpr (sizeof(P) == 1)
    {
        const uint32_t w = 0x01010101u * (uint32_t)v;
        for (; x + 16 <= f.mx; x += 16) stu<uint4>(d + x, make_uint4(w, w, w, w));
        for (; x + 4 <= f.mx; x += 4) stu<uint32_t>(d + x, w);
    }
    else
    {
        const uint32_t w = 0x00010001u * (uint32_t)v;
        for (; x + 8 <= f.mx; x += 8) stu<uint4>(d + x, make_uint4(w, w, w, w));
        for (; x + 2 <= f.mx; x += 2) stu<uint32_t>(d + x, w);
    }
    for (; x < f.mx; x++) d[x] = v;
}

// the margin rows: full-stride copies of the extended first / last row, 16 bytes per lane
template <typename P>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_border_tb(const BorderLaunch L)
{
    constexpr int C = 16 / sizeof(P);
    const uint32_t b = xcd_block();
    int i = 0;
#pragma unroll
    for (int k = 1; k < kMaxPlanes; k++)
        if (k < L.count && L.f[k].block0_tb <= b) i = k;
    const BorderPlane& f = L.f[i];
    const int64_t chunks = (f.stride + C - 1) / C;
    const int64_t t = (int64_t)(b - f.block0_tb) * X265AMD_BLOCK + threadIdx.x;
    if (t >= (int64_t)(f.top + f.bottom) * f.my * chunks) return;
    int r = (int)(t / chunks);
    const int c = (int)(t % chunks);
    const bool bottom = !f.top || r >= f.my;
    if (f.top && bottom) r -= f.my;
    const int yd = bottom ? f.h + r : -1 - r;
    const int ys = bottom ? f.h - 1 : 0;
    const P* s = (const P*)f.p - f.mx + ys * f.stride + c * C;
    P* d = (P*)f.p - f.mx + yd * f.stride + c * C;
    if ((c + 1) * C <= f.stride) stu<uint4>(d, ldu<uint4>(s));
    else
        for (int x = 0; x < f.stride - c * C; x++) d[x] = s[x];
}

} // namespace x265amd

using namespace x265amd;

static bool bd_ok(int depth) { return depth == 8 || depth == 10 || depth == 12; }
static uint32_t nblocks(uint64_t n) { return (uint32_t)((n + X265AMD_BLOCK - 1) / X265AMD_BLOCK); }

static int deblock_impl(int depth, int count, const x265amd_deblock_frame* frames, const int32_t* rows, void* stream)
{
    if (!bd_ok(depth) || count < 0 || (count && !frames)) return X265AMD_EINVAL;
    for (int i = 0; i < count; i++)
    {
        const x265amd_deblock_frame& a = frames[i];
        const bool i400 = a.chroma_format == X265AMD_CSP_I400;
        if (a.width <= 0 || a.height <= 0 || (a.width & 7) || (a.height & 7) || !a.plane[0] ||
            (!i400 && (!a.plane[1] || !a.plane[2] || a.cstride < (a.chroma_format == 3 ? a.width : a.width / 2))) ||
            !a.units || a.unit_stride < a.width / 4 || a.stride < a.width || a.chroma_format < 0 ||
            a.chroma_format > X265AMD_CSP_I400)
            return X265AMD_EINVAL;
        if (rows && (rows[2 * i] < 0 || (rows[2 * i] & 15) || rows[2 * i + 1] <= rows[2 * i] ||
                     rows[2 * i + 1] > a.height || ((rows[2 * i + 1] - rows[2 * i]) & 7)))
            return X265AMD_EINVAL;
    }
    hipStream_t st = (hipStream_t)stream;
    for (int dir = 0; dir < 2; dir++)
        for (int i0 = 0; i0 < count; i0 += kDbkFrames)
        {
            DbkLaunch L;
            memset(&L, 0, sizeof(L));
            L.count = count - i0 < kDbkFrames ? count - i0 : kDbkFrames;
            L.maxv = (1 << depth) - 1;
            uint32_t blocks = 0;
            for (int k = 0; k < L.count; k++)
            {
                const x265amd_deblock_frame& a = frames[i0 + k];
                DbkFrame& f = L.f[k];
                for (int p = 0; p < 3; p++) f.plane[p] = a.plane[p];
                f.stride = a.stride;
                f.cstride = a.cstride;
                f.units = a.units;
                f.us = a.unit_stride;
                f.wu = a.width >> 2;
                f.uy0 = rows ? rows[2 * (i0 + k)] >> 2 : 0;
                f.hu = rows ? (rows[2 * (i0 + k) + 1] - rows[2 * (i0 + k)]) >> 2 : a.height >> 2;
                f.is_p = a.is_p;
                f.beta2 = 2 * a.beta_offset_div2;
                f.tc2 = 2 * a.tc_offset_div2;
                f.cbqp = a.cb_qp_offset;
                f.crqp = a.cr_qp_offset;
                f.tqb = a.tq_bypass_enabled;
                f.hs = a.chroma_format == 3 ? 0 : 1;
                f.vs = a.chroma_format == 2 || a.chroma_format == 3 ? 0 : 1;
                memcpy(f.poc, a.ref_poc, sizeof(f.poc));
                if (dir == 0)
                {
                    const int sx = 2 << f.hs;
                    f.nluma = (uint32_t)((f.wu >> 1) * f.hu);
                    f.nseg = f.nluma + (a.chroma_format == X265AMD_CSP_I400 ? 0u :
                                        (uint32_t)(((f.wu + sx - 1) / sx) * (f.hu >> f.vs)));
                }
                else
                {
                    const int sy = 2 << f.vs;
                    f.nluma = (uint32_t)(f.wu * (f.hu >> 1));
                    f.nseg = f.nluma + (a.chroma_format == X265AMD_CSP_I400 ? 0u :
                                        (uint32_t)((f.wu >> f.hs) * ((f.hu + sy - 1) / sy)));
                }
                f.block0 = blocks;
                blocks += nblocks(f.nseg);
            }
            if (!blocks) continue;
            if (depth == 8)
            {
                if (dir == 0) hipLaunchKernelGGL((k_deblock<uint8_t, 0>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, L);
                else hipLaunchKernelGGL((k_deblock<uint8_t, 1>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, L);
            }
            else
            {
                if (dir == 0) hipLaunchKernelGGL((k_deblock<uint16_t, 0>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, L);
                else hipLaunchKernelGGL((k_deblock<uint16_t, 1>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, L);
            }
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return (int)e;
        }
    return 0;
}

extern "C" int x265amd_deblock(int depth, int count, const x265amd_deblock_frame* frames, void* stream)
{
    return deblock_impl(depth, count, frames, nullptr, stream);
}

extern "C" int x265amd_deblock_rows(int depth, int count, const x265amd_deblock_frame* frames, const int32_t* rows,
                                    void* stream)
{
    return rows ? deblock_impl(depth, count, frames, rows, stream) : X265AMD_EINVAL;
}

static int sao_apply_impl(int depth, int count, const x265amd_sao_frame* frames, const int32_t* ctu_rows, void* stream)
{
    if (!bd_ok(depth) || count < 0 || (count && !frames)) return X265AMD_EINVAL;
    for (int i = 0; i < count; i++)
    {
        const x265amd_sao_frame& a = frames[i];
        const bool i400 = a.chroma_format == X265AMD_CSP_I400;
        if (a.width <= 0 || a.height <= 0 || (a.width & 7) || (a.height & 7) || a.ctu_log2 < 4 || a.ctu_log2 > 6 ||
            !a.params || a.stride < a.width || (!i400 && a.cstride < (a.chroma_format == 3 ? a.width : a.width / 2)) ||
            a.chroma_format < 0 || a.chroma_format > X265AMD_CSP_I400)
            return X265AMD_EINVAL;
        const int hc = (a.height + (1 << a.ctu_log2) - 1) >> a.ctu_log2;
        if (ctu_rows && (ctu_rows[2 * i] < 0 || ctu_rows[2 * i + 1] <= ctu_rows[2 * i] || ctu_rows[2 * i + 1] > hc))
            return X265AMD_EINVAL;
        for (int p = 0; p < (i400 ? 1 : 3); p++)
            if (!a.src[p] || !a.dst[p] || a.src[p] == a.dst[p]) return X265AMD_EINVAL;
    }
    hipStream_t st = (hipStream_t)stream;
    for (int i0 = 0; i0 < count; i0 += kMaxFrames)
    {
        SaoLaunch L;
        memset(&L, 0, sizeof(L));
        L.count = count - i0 < kMaxFrames ? count - i0 : kMaxFrames;
        L.maxv = (1 << depth) - 1;
        L.bo_shift = depth - 5;
        uint32_t blocks = 0;
        for (int k = 0; k < L.count; k++)
        {
            const x265amd_sao_frame& a = frames[i0 + k];
            SaoFrame& f = L.f[k];
            for (int p = 0; p < 3; p++) { f.src[p] = a.src[p]; f.dst[p] = a.dst[p]; }
            f.stride = a.stride;
            f.cstride = a.cstride;
            f.params = a.params;
            f.w = a.width;
            f.h = a.height;
            f.ctu_log2 = a.ctu_log2;
            const int ctu = 1 << a.ctu_log2;
            f.wc = (a.width + ctu - 1) >> a.ctu_log2;
            f.nctu_all = f.wc * ((a.height + ctu - 1) >> a.ctu_log2);
            f.c0 = ctu_rows ? ctu_rows[2 * (i0 + k)] * f.wc : 0;
            f.nctu = ctu_rows ? (ctu_rows[2 * (i0 + k) + 1] - ctu_rows[2 * (i0 + k)]) * f.wc : f.nctu_all;
            f.luma_on = a.luma_on;
            f.chroma_on = a.chroma_on;
            f.i400 = a.chroma_format == X265AMD_CSP_I400;
            f.hs = a.chroma_format == 3 ? 0 : 1;
            f.vs = a.chroma_format == 2 || a.chroma_format == 3 ? 0 : 1;
            f.block0 = blocks;
            blocks += 3 * (uint32_t)f.nctu;
        }
        if (!blocks) continue;
        if (depth == 8) hipLaunchKernelGGL((k_sao_apply<uint8_t>), dim3(blocks), dim3(64), 0, st, L);
        else hipLaunchKernelGGL((k_sao_apply<uint16_t>), dim3(blocks), dim3(64), 0, st, L);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return (int)e;
    }
    return 0;
}

extern "C" int x265amd_sao_apply(int depth, int count, const x265amd_sao_frame* frames, void* stream)
{
    return sao_apply_impl(depth, count, frames, nullptr, stream);
}

extern "C" int x265amd_sao_apply_rows(int depth, int count, const x265amd_sao_frame* frames, const int32_t* ctu_rows,
                                      void* stream)
{
    return ctu_rows ? sao_apply_impl(depth, count, frames, ctu_rows, stream) : X265AMD_EINVAL;
}

extern "C" int x265amd_sao_stats(int depth, int count, const x265amd_sao_stats_frame* frames, void* stream)
{
    if (!bd_ok(depth) || count < 0 || (count && !frames)) return X265AMD_EINVAL;
    for (int i = 0; i < count; i++)
    {
        const x265amd_sao_stats_frame& a = frames[i];
        if (a.width <= 0 || a.height <= 0 || (a.width & 7) || (a.height & 7) || a.ctu_log2 < 4 || a.ctu_log2 > 6 ||
            !a.stats || !a.count || a.chroma_format < 0 || a.chroma_format > 3)   /* 4:0:0 not supported */
            return X265AMD_EINVAL;
        for (int p = 0; p < 3; p++)
            if (!a.fenc[p] || !a.rec[p]) return X265AMD_EINVAL;
    }
    hipStream_t st = (hipStream_t)stream;
    for (int i0 = 0; i0 < count; i0 += kStatFrames)
    {
        StatLaunch L;
        memset(&L, 0, sizeof(L));
        L.count = count - i0 < kStatFrames ? count - i0 : kStatFrames;
        L.bo_shift = depth - 5;
        uint32_t blocks = 0;
        for (int k = 0; k < L.count; k++)
        {
            const x265amd_sao_stats_frame& a = frames[i0 + k];
            StatFrame& f = L.f[k];
            for (int p = 0; p < 3; p++) { f.fenc[p] = a.fenc[p]; f.rec[p] = a.rec[p]; }
            f.fs = a.fenc_stride;
            f.fcs = a.fenc_cstride;
            f.rs = a.rec_stride;
            f.rcs = a.rec_cstride;
            f.stats = a.stats;
            f.count = a.count;
            f.w = a.width;
            f.h = a.height;
            f.ctu_log2 = a.ctu_log2;
            f.nd = a.non_deblocked;
            f.hs = a.chroma_format == 3 ? 0 : 1;
            f.vs = a.chroma_format == 2 || a.chroma_format == 3 ? 0 : 1;
            const int ctu = 1 << a.ctu_log2;
            f.wc = (a.width + ctu - 1) >> a.ctu_log2;
            f.nctu = (uint32_t)(f.wc * ((a.height + ctu - 1) >> a.ctu_log2));
            f.block0 = blocks;
            blocks += f.nctu;
        }
        if (depth == 8) hipLaunchKernelGGL((k_sao_stats<uint8_t>), dim3(blocks), dim3(64), 0, st, L);
        else hipLaunchKernelGGL((k_sao_stats<uint16_t>), dim3(blocks), dim3(64), 0, st, L);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return (int)e;
    }
    return 0;
}

static int border_impl(int depth, int count, const x265amd_border_plane* planes, const int32_t* rows, void* stream)
{
    if (!bd_ok(depth) || count < 0 || (count && !planes)) return X265AMD_EINVAL;
    for (int i = 0; i < count; i++)
    {
        const x265amd_border_plane& a = planes[i];
        if (!a.plane || a.width <= 0 || a.height <= 0 || a.margin_x < 0 || a.margin_y < 0 ||
            a.stride < a.width + 2 * a.margin_x)
            return X265AMD_EINVAL;
        if (rows && (rows[4 * i] < 0 || rows[4 * i + 1] < rows[4 * i] || rows[4 * i + 1] > a.height))
            return X265AMD_EINVAL;
    }
    hipStream_t st = (hipStream_t)stream;
    for (int i0 = 0; i0 < count; i0 += kMaxPlanes)
    {
        BorderLaunch L;
        memset(&L, 0, sizeof(L));
        L.count = count - i0 < kMaxPlanes ? count - i0 : kMaxPlanes;
        uint32_t blr = 0, btb = 0;
        const int C = depth == 8 ? 16 : 8;
        for (int k = 0; k < L.count; k++)
        {
            const x265amd_border_plane& a = planes[i0 + k];
            BorderPlane& f = L.f[k];
            f.p = a.plane;
            f.stride = a.stride;
            f.w = a.width;
            f.h = a.height;
            f.mx = a.margin_x;
            f.my = a.margin_y;
            const int* r = rows ? rows + 4 * (i0 + k) : nullptr;
            f.y0 = r ? r[0] : 0;
            f.nr = r ? r[1] - r[0] : a.height;
            f.top = r ? (r[2] != 0) : 1;
            f.bottom = r ? (r[3] != 0) : 1;
            f.block0_lr = blr;
            f.block0_tb = btb;
            blr += nblocks(2 * (uint64_t)f.nr);
            btb += nblocks((uint64_t)(f.top + f.bottom) * a.margin_y * (uint64_t)((a.stride + C - 1) / C));
        }
        hipError_t e;
        if (blr)
        {
            if (depth == 8) hipLaunchKernelGGL((k_border_lr<uint8_t>), dim3(blr), dim3(X265AMD_BLOCK), 0, st, L);
            else hipLaunchKernelGGL((k_border_lr<uint16_t>), dim3(blr), dim3(X265AMD_BLOCK), 0, st, L);
            e = hipGetLastError();
            if (e != hipSuccess) return (int)e;
        }
        if (btb)
        {
            if (depth == 8) hipLaunchKernelGGL((k_border_tb<uint8_t>), dim3(btb), dim3(X265AMD_BLOCK), 0, st, L);
            else hipLaunchKernelGGL((k_border_tb<uint16_t>), dim3(btb), dim3(X265AMD_BLOCK), 0, st, L);
            e = hipGetLastError();
            if (e != hipSuccess) return (int)e;
        }
    }
    return 0;
}

extern "C" int x265amd_extend_border(int depth, int count, const x265amd_border_plane* planes, void* stream)
{
    return border_impl(depth, count, planes, nullptr, stream);
}

extern "C" int x265amd_extend_border_rows(int depth, int count, const x265amd_border_plane* planes, const int32_t* rows,
                                          void* stream)
{
    return rows ? border_impl(depth, count, planes, rows, stream) : X265AMD_EINVAL;
}

// the launch descriptors must fit the 4 KiB kernarg segment
static_assert(sizeof(x265amd::DbkLaunch) <= 4096, "DbkLaunch exceeds the kernarg segment");
static_assert(sizeof(x265amd::SaoLaunch) <= 4096, "SaoLaunch exceeds the kernarg segment");
static_assert(sizeof(x265amd::StatLaunch) <= 4096, "StatLaunch exceeds the kernarg segment");
static_assert(sizeof(x265amd::BorderLaunch) <= 4096, "BorderLaunch exceeds the kernarg segment");
