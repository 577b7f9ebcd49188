// saostats.h — SAO::calcSaoStatsCu (sao.cpp:772-943) of one CTU, all three planes, by one wavefront: the body
// of loopfilter.hip's whole-frame k_sao_stats and of tu.hip's resident server (a CTU a request, the source
// and deblocked windows staged in LDS).  Included inside namespace x265amd, after common.h.
#pragma once

__device__ __forceinline__ int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
// sign as one v_med3_i32 (clamp to [-1, 1]); written as asm because the compiler turns
// (v > 0) - (v < 0) and min / max of a difference back into two compares and selects
__device__ __forceinline__ int sgn(int v)
{
    int r;
    asm("v_med3_i32 %0, %1, -1, 1" : "=v"(r) : "v"(v));
    return r;
}

// o[i] = p[i - 1], i = 0..9: a row segment with its left / right neighbour in one (8-bit) or
// two (16-bit) 16-byte loads; rows are readable from 4 pixels left of p to 12 right of it
// (A8: the row lies in LDS at an 8-byte aligned p - 4 — two 8-byte loads, never a misaligned 16-byte one)
template <typename P, bool A8 = false>
__device__ __forceinline__ void load_row10(const P* p, int (&o)[10])
{
    if constexpr (sizeof(P) == 1)
    {
        uint4 v;
        if constexpr (A8)
        {
            const uint2 lo = *(const uint2*)(p - 4), hi = *(const uint2*)(p + 4);
            v = make_uint4(lo.x, lo.y, hi.x, hi.y);
        }
        else
            v = ldu<uint4>(p - 4);
        const uint32_t w[4] = { v.x, v.y, v.z, v.w };
#pragma unroll
        for (int i = 0; i < 10; i++) o[i] = (int)((w[(i + 3) >> 2] >> (8 * ((i + 3) & 3))) & 0xff);
    }
    else
    {
        const uint4 a = ldu<uint4>(p - 2), b = ldu<uint4>(p + 6);
        const uint32_t w[8] = { a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w };
#pragma unroll
        for (int i = 0; i < 10; i++) o[i] = (int)((w[(i + 1) >> 1] >> (16 * ((i + 1) & 1))) & 0xffff);
    }
}

// one CTU as calcSaoStatsCu sees it: per plane the CTU origin in the deblocked reconstruction (readable one row
// above to one row below the CTU, 4 pixels left to 12 right of every 8-pixel strip) and in the source; per plane
// class (0 luma, 1 chroma) the plane size, the CTU origin in plane coordinates and the nominal CTU size
struct SaoCtuView
{
    const void* rec[3];
    const void* fenc[3];
    int64_t rs[3], fs[3];
    int pw[2], ph[2], x0[2], y0[2], csw[2], csh[2];
    int nd;                                  // --sao-non-deblock (bSaoNonDeblocked)
};

// Pass 0: luma, lane = 8x8 strip of the CTU (<= 64 strips); pass 1: Cb on lanes 0-31, Cr on lanes 32-63
// (<= 16 strips each).  A lane walks its strip row by row (one new 16-byte load per row) and adds, per EO type,
// (d << 7) + 1 to its private LDS bin of the pixel's edge class (<= 64 pixels of <= 12 bits per lane: no
// overflow; a conflict-free ds_add instead of a five-way select chain); band classes merge runs of equal band
// and add them to LDS as (count << 40) + sum.  The lanes' bins then reduce across the wave (or half-wave).
// Writes every entry of os / oc [3 planes][5 types: EO_0..EO_3, BO][33 classes] (m_offsetOrg / m_count).
// Wave-level only (no workgroup barrier): callable from one wavefront of a larger workgroup.  LDS: the windows
// are staged in LDS (8-bit, each strip's p - 4 8-byte aligned), read with aligned 8-byte loads.
// NW wavefronts (1, or 4 = a whole workgroup of the server, called by every thread): wave w takes rows
// [8 k + w 8 / NW, + 8 / NW) of every strip; the waves' totals meet in LDS atomics and a workgroup barrier.
template <typename P, bool LDS = false, int NW = 1>
__device__ __forceinline__ void sao_stats_wave(const SaoCtuView& v, int bo_shift, int32_t* os, int32_t* oc)
{
    static_assert(NW == 1 || NW == 2 || NW == 4 || NW == 8, "rows of a strip per wave");
    constexpr int RG = 8 / NW;                    // rows of a strip per wave
    __shared__ int32_t eo_sum[3][4][5], eo_cnt[3][4][5];
    __shared__ unsigned long long bo[3][32];
    __shared__ int32_t bins[NW * 64][21];         // per lane: [EO type][edge type] (sum << 7) + count; [20] sink
    const int lane = threadIdx.x & 63, wv = NW > 1 ? (int)(threadIdx.x >> 6) : 0;
    const int tid = wv * 64 + lane;
    auto sync_all = [] {
        if constexpr (NW > 1) __syncthreads();
        else wave_sync();
    };
    for (int i = tid; i < 3 * 32; i += 64 * NW) (&bo[0][0])[i] = 0;
    for (int i = tid; i < 3 * 4 * 5; i += 64 * NW) { (&eo_sum[0][0][0])[i] = 0; (&eo_cnt[0][0][0])[i] = 0; }
    sync_all();
#pragma unroll 1
    for (int pass = 0; pass < 2; pass++)
    {
        const int p = pass ? 1 + (lane >> 5) : 0, pc = pass;
        const int sl = pass ? lane & 31 : lane, nl = pass ? 32 : 64;
        const int pw = pc ? v.pw[1] : v.pw[0], ph = pc ? v.ph[1] : v.ph[0];
        const int csw = pc ? v.csw[1] : v.csw[0], csh = pc ? v.csh[1] : v.csh[0];
        const int x0 = pc ? v.x0[1] : v.x0[0], y0 = pc ? v.y0[1] : v.y0[0];
        const int cw = (x0 + csw < pw ? x0 + csw : pw) - x0, ch = (y0 + csh < ph ? y0 + csh : ph) - y0;
        const bool right = x0 + cw == pw, bottom = y0 + ch == ph;
        const int po = p ? 2 : 0;
        // regions per type (sao.cpp:825-925): EO_0, EO_1, EO_2, EO_3, BO; EO_0 keeps its bottom
        // skip at the picture edge (sao.cpp:852)
        int xs[5], xe[5], ys[5], ye[5];
#pragma unroll
        for (int t = 0; t < 5; t++)
        {
            const int sb = v.nd ? (t == 0 || t == 4 ? 3 : 4) : 4;
            const int sr = v.nd ? (t == 1 || t == 4 ? 4 : 5) : 5;
            const bool eox = t == 0 || t == 2 || t == 3, eoy = t >= 1 && t <= 3;
            xs[t] = eox ? (x0 == 0) : 0;
            xe[t] = right ? (eox ? cw - 1 : cw) : cw - sr + po;
            ys[t] = eoy ? (y0 == 0) : 0;
            ye[t] = t == 0 ? ch - sb + po : (bottom ? (eoy ? ch - 1 : ch) : ch - sb + po);
        }
        const int nsx = (cw + 7) >> 3, nsy = (ch + 7) >> 3;
        // chroma strips per plane: 16 (4:2:0), 32 (4:2:2), 64 (4:4:4) over 32 lanes; Cb and Cr have the
        // same geometry, so the round count is uniform over the wave
        const int rounds = (nsx * nsy + nl - 1) / nl;
#pragma unroll 1
        for (int round = 0; round < rounds; round++)
        {
#pragma unroll
            for (int k = 0; k < 20; k++) bins[tid][k] = 0;
            const int strip = sl + round * nl;
            const int ly0 = 8 * (strip / nsx) + wv * RG;
            if (strip < nsx * nsy && ly0 < ch)
            {
                const int lx0 = 8 * (strip % nsx);
                const int rows = ch - ly0 < RG ? ch - ly0 : RG;
                uint32_t xm[5];
#pragma unroll
                for (int t = 0; t < 5; t++)
                {
                    const int lo = clip3(0, 8, xs[t] - lx0), hi = clip3(0, 8, xe[t] - lx0);
                    xm[t] = hi > lo ? ((1u << hi) - 1) & ~((1u << lo) - 1) : 0u;
                }
                // (selects, not v.rec[p]: p differs across the lanes of pass 1, and an indexed load of the view
                // would put it in scratch)
                const int64_t rs = p == 0 ? v.rs[0] : p == 1 ? v.rs[1] : v.rs[2];
                const int64_t fs = p == 0 ? v.fs[0] : p == 1 ? v.fs[1] : v.fs[2];
                const void* rp = p == 0 ? v.rec[0] : p == 1 ? v.rec[1] : v.rec[2];
                const void* fp = p == 0 ? v.fenc[0] : p == 1 ? v.fenc[1] : v.fenc[2];
                const P* r = (const P*)rp + (int64_t)ly0 * rs + lx0;
                const P* fe = (const P*)fp + (int64_t)ly0 * fs + lx0;
                int up[10], mid[10], dn[10];
                load_row10<P, LDS>(r - rs, up);
                load_row10<P, LDS>(r, mid);
                // signs against the row above for EO_1 / EO_2 / EO_3: after the first row they are the
                // negated signs against the row below of the previous row (sao.cpp's signUp buffers)
                int u1[8], u2[8], u3[8];
#pragma unroll
                for (int i = 0; i < 8; i++)
                {
                    u1[i] = sgn(mid[i + 1] - up[i + 1]);
                    u2[i] = sgn(mid[i + 1] - up[i]);
                    u3[i] = sgn(mid[i + 1] - up[i + 2]);
                }
#pragma unroll
                for (int yy = 0; yy < RG; yy++)
                {
                    if (yy >= rows) break;
                    load_row10<P, LDS>(r + (yy + 1) * rs, dn);
                    int h[9];                 // EO_0: sign of each pixel against its left neighbour
#pragma unroll
                    for (int k = 0; k < 9; k++) h[k] = sgn(mid[k + 1] - mid[k]);
                    int n1[8], n2[8], n3[8];
                    n2[0] = sgn(dn[1] - mid[0]);
                    n3[7] = sgn(dn[8] - mid[9]);
                    int fv[8];
                    load_row<P, 8>(fe + yy * fs, fv);
                    const int ly = ly0 + yy;
                    uint32_t m[5];
#pragma unroll
                    for (int t = 0; t < 5; t++) m[t] = (ly >= ys[t] && ly < ye[t]) ? xm[t] : 0u;
                    int run_band = -1;
                    unsigned long long run = 0;
#pragma unroll
                    for (int i = 0; i < 8; i++)
                    {
                        const int val_v = mid[i + 1], d = fv[i] - val_v;
                        const int val = (d << 7) + 1;
                        const int d1 = sgn(val_v - dn[i + 1]), d2 = sgn(val_v - dn[i + 2]), d3 = sgn(val_v - dn[i]);
                        const int e[4] = { h[i] - h[i + 1], u1[i] + d1, u2[i] + d2, u3[i] + d3 };
                        n1[i] = -d1;
                        if (i < 7) n2[i + 1] = -d2;
                        if (i > 0) n3[i - 1] = -d3;
#pragma unroll
                        for (int t = 0; t < 4; t++)
                        {
                            // masked-off pixels go to the sink bin 20: no branch around the ds_add
                            const int bi = ((m[t] >> i) & 1) ? 5 * t + e[t] + 2 : 20;
                            atomicAdd(&bins[tid][bi], val);
                        }
                        if ((m[4] >> i) & 1)
                        {
                            const int band = val_v >> bo_shift;
                            if (band != run_band)
                            {
                                if (run_band >= 0) atomicAdd(&bo[p][run_band], run);
                                run_band = band;
                                run = 0;
                            }
                            run += (1ull << 40) + (unsigned long long)(int64_t)d;
                        }
                    }
                    if (run_band >= 0) atomicAdd(&bo[p][run_band], run);
#pragma unroll
                    for (int i = 0; i < 8; i++) { u1[i] = n1[i]; u2[i] = n2[i]; u3[i] = n3[i]; }
#pragma unroll
                    for (int i = 0; i < 10; i++) mid[i] = dn[i];
                }
            }
            wave_sync();
            // wave (pass 0) / half-wave (pass 1) totals: lane r < 20 of each half sums bin r over the
            // lanes of its plane; edge type j = e + 2 -> class s_eoTable[j] (sao.cpp:65-72): 1, 2, 0, 3, 4
            const int r = pass ? lane & 31 : lane;
            if (r < 20)
            {
                const int l0 = wv * 64 + (pass ? lane & 32 : 0);
                int vsum = 0, vc = 0;
                for (int l = 0; l < nl; l++)
                {
                    const int bv = bins[l0 + l][r];
                    const int cn = bv & 127;
                    vc += cn;
                    vsum += (bv - cn) >> 7;
                }
                const int t = r / 5, j = r % 5;
                const int k = j == 0 ? 1 : j == 1 ? 2 : j == 2 ? 0 : j;
                if constexpr (NW > 1)
                {
                    atomicAdd(&eo_sum[p][t][k], vsum);
                    atomicAdd(&eo_cnt[p][t][k], vc);
                }
                else
                {
                    eo_sum[p][t][k] += vsum;
                    eo_cnt[p][t][k] += vc;
                }
            }
            wave_sync();
        }
    }
    sync_all();
    // every entry of the CTU's [3][5][33] block
    for (int i = tid; i < 3 * 5 * 33; i += 64 * NW)
    {
        const int p = i / 165, t = (i % 165) / 33, k = i % 33;
        int sv = 0, cv = 0;
        if (t < 4)
        {
            if (k < 5) { sv = eo_sum[p][t][k]; cv = eo_cnt[p][t][k]; }
        }
        else if (k >= 1)
        {
            const long long tot = (long long)bo[p][k - 1];
            const long long lo = (long long)((unsigned long long)tot << 24) >> 24;   // sign-extend 40 bits
            sv = (int)lo;
            cv = (int)((tot - lo) >> 40);
        }
        os[i] = sv;
        oc[i] = cv;
    }
}
