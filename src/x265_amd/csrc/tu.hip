// tu.hip — fused TU pipeline.
//
// One job is the whole per-TU chain x265 runs for a residual-coded TU at
// --preset medium (no RDOQ, no transform skip / lossless, flat scaling lists,
// no noise reduction), exactly as Search::residualTransformQuantIntra chains
// it (search.cpp:689-706):
//
//   resi  = fenc - pred                                 calcresidual, pixel.cpp:416-428
//   coeff = quant(dct(resi)) + sign-bit hiding          Quant::transformNxN, quant.cpp:397-491
//                                                       (dst4 for luma intra 4x4, quant_c dct.cpp:664-686,
//                                                        signBitHidingHDQ quant.cpp:247-393)
//   numSig ? resi = idct(dequant(coeff)) (or DC fill)   Quant::invtransformNxN, quant.cpp:493-546
//            recon = clip(pred + resi)                  add_ps, pixel.cpp:774-786
//          : recon = pred                               copy_pp
//
// In the reference that is 6-8 table calls and as many passes over HBM-sized
// scratch; here one N-lane group owns one TU from the fenc/pred loads to the
// recon/coeff stores, with every intermediate in registers or a per-TU LDS
// tile.  Lane r owns row r of the residual, column r of the coefficients and
// row r of the reconstruction, so the four transform stages need three LDS
// transposes and no block-wide barrier: a group never spans a wavefront
// (N <= 32), so LDS exchange inside a group only needs wavefront-scope
// ordering (wave_sync) and groups whose TU has no coded coefficient leave the
// inverse path early.  Sign-bit hiding runs one coefficient group (4x4) per
// lane — CGs are independent (quant.cpp:273-391) except for the last-position
// search, which is a group max — with deltaU recomputed from the DCT
// coefficient kept in LDS instead of stored (it is a pure function of it).
#include <type_traits>

#include "common.h"
#include "transform1d.h"
#include "rdojob.h"
#include "../../../include/x265_amd.h"

namespace x265amd {

#include "hadamard.h"
#include "saostats.h"

// ---------------------------------------------------------------- scan orders
// HEVC scans (spec 6.5.3-6.5.5; x265 g_scanOrder, constants.cpp:359-456),
// generated: CGs of 4x4 visited in the scan of the CG grid, positions inside
// a CG in the 4x4 scan of the same type (0 up-right diagonal, 1 horizontal,
// 2 vertical; 16x16 / 32x32 are diagonal only, cudata.cpp:2038-2041).
struct ScanTabs
{
    uint16_t s4[3][16];
    uint16_t s8[3][64];
    uint16_t s16[256];
    uint16_t s32[1024];
};

constexpr void scan_grid(int type, int n, int* order)
{
    int k = 0;
    if (type == 1)
        for (int i = 0; i < n * n; i++) order[k++] = i;
    else if (type == 2)
        for (int i = 0; i < n * n; i++) order[k++] = (i % n) * n + i / n;
    else
        for (int d = 0; d <= 2 * (n - 1); d++)
            for (int r = d < n ? d : n - 1; r >= 0 && d - r < n; r--)
                order[k++] = r * n + (d - r);
}

constexpr void make_scan(int type, int log2, uint16_t* out)
{
    const int n = 1 << log2, g = n >> 2;
    int cg[64] = {}, in[16] = {};
    scan_grid(type, g, cg);
    scan_grid(type, 4, in);
    for (int c = 0; c < g * g; c++)
        for (int i = 0; i < 16; i++)
            out[c * 16 + i] = (uint16_t)(((cg[c] / g) * 4 + in[i] / 4) * n + (cg[c] % g) * 4 + in[i] % 4);
}

constexpr ScanTabs make_scans()
{
    ScanTabs t{};
    for (int ty = 0; ty < 3; ty++)
    {
        make_scan(ty, 2, t.s4[ty]);
        make_scan(ty, 3, t.s8[ty]);
    }
    make_scan(0, 4, t.s16);
    make_scan(0, 5, t.s32);
    return t;
}

static __constant__ ScanTabs c_scan = make_scans();

// s_quantScales / s_invQuantScales (scalinglist.cpp:121-122; HEVC spec 8.6.2)
// (independent selects, so per-lane rem compiles to v_cndmask rather than branches)
__device__ __forceinline__ int quant_scale(int rem)
{
    int v = 14564;
    v = rem == 4 ? 16384 : v;
    v = rem == 3 ? 18396 : v;
    v = rem == 2 ? 20560 : v;
    v = rem == 1 ? 23302 : v;
    v = rem == 0 ? 26214 : v;
    return v;
}
__device__ __forceinline__ int inv_quant_scale(int rem)
{
    int v = 72;
    v = rem == 4 ? 64 : v;
    v = rem == 3 ? 57 : v;
    v = rem == 2 ? 51 : v;
    v = rem == 1 ? 45 : v;
    v = rem == 0 ? 40 : v;
    return v;
}

template <int G>
__device__ __forceinline__ int group_max(int v)
{
#pragma unroll
    for (int m = G >> 1; m > 0; m >>= 1)
    {
        const int o = __shfl_xor(v, m, 64);
        v = o > v ? o : v;
    }
    return v;
}

// The candidate search of signBitHidingHDQ (quant.cpp:313-366) over one CG in
// scan order, branch-free: qv / cv = quantized / DCT coefficients of scan
// positions 0..15, mask = their significance bits, top = the highest
// candidate position, signbit = the parity target.  Returns the position and
// the +-1 change of the cheapest candidate (first minimum from the top, as the
// reference's strict `<` keeps it).
__device__ __forceinline__ void sbh_pick(const int (&qv)[16], const int (&cv)[16], uint32_t mask, int top, int signbit,
                                         int qscale, int qadd, int qbits, int& min_n, int& change)
{
    const int qbits8 = qbits - 8;
    int min_cost = 0x7fffffff;
    min_n = 0;
    change = 0;
#pragma unroll
    for (int n = 15; n >= 0; n--)
    {
        const int c = cv[n], q = qv[n];
        const int tmp = (c < 0 ? -c : c) * qscale;
        const int du = (tmp - (((tmp + qadd) >> qbits) << qbits)) >> qbits8;   // deltaU (quant_c)
        // every condition as a 0/1 integer combined with bitwise operators: straight-line selects (the
        // short-circuit form compiled to a branch per term and candidate)
        const int below = (mask & ((1u << n) - 1)) != 0;    // a significant coefficient before n
        const int nz = q != 0;
        const int one = (q == 1) | (q == -1);
        const int dneg = du <= 0;
        const int adu = du < 0 ? -du : du;
        // significant: +1 if deltaU > 0, else -1 (never zeroing the first significant one)
        // not significant: +1 (before the first significant one only with the matching sign)
        const int blocked = (nz & (below ^ 1) & one & dneg) | ((nz ^ 1) & (below ^ 1) & ((int)(c < 0) ^ signbit));
        const int cost = blocked ? 0x7fffffff : (nz ? -adu : -du);
        const int ch = (nz & dneg) ? -1 : 1;
        const int take = (n <= top) & (cost < min_cost);
        min_cost = take ? cost : min_cost;
        change = take ? ch : change;
        min_n = take ? n : min_n;
    }
}

// Position of scan index n inside a 4x4 coefficient group, as a raster offset in
// a TU of pitch N (the 4x4 scans of make_scan, folded to immediates).
template <int N>
__device__ __forceinline__ int cg_offset(int type, int n)
{
    constexpr int diag[16] = { 0, 4, 1, 8, 5, 2, 12, 9, 6, 3, 13, 10, 7, 14, 11, 15 };
    const int v = type == 1 ? n : type == 2 ? (n & 3) * 4 + (n >> 2) : diag[n];
    return (v >> 2) * N + (v & 3);
}

// Quant::signBitHidingHDQ (quant.cpp:247-393) over one N x N TU held in LDS by
// a G-lane group (G >= number of coefficient groups): Q = quantized
// coefficients (raster, modified in place), C = DCT coefficients (raster,
// pitch N; deltaU is recomputed from them exactly as quant_c computes it),
// lane `lane` owns the CG of scan index `lane`.  CGs are independent (each
// decision reads and changes only its own 16 coefficients); the only TU-wide
// input is the last significant scan position (a group max).  All 16 values
// of a CG are loaded at once (the CG's corner from the scan table, the
// positions inside it are immediates), so there is no serial load chain.
// Returns the change of numSig (group-reduced, valid in every lane).
template <int N, int G>
__device__ __forceinline__ int sign_hide(int16_t* Q, const int16_t* C, const uint16_t* scan, int type, int lane,
                                         int qscale, int qadd, int qbits)
{
    constexpr int NCG = N * N / 16;
    static_assert(NCG <= G, "one coefficient group per lane");
    const bool has = lane < NCG;
    const int cg = has ? lane : 0;
    const int corner = scan[cg * 16];            // position 0 of every 4x4 scan is the CG's corner
    int qv[16];
    uint32_t mask = 0;
#pragma unroll
    for (int n = 0; n < 16; n++)
    {
        qv[n] = Q[corner + cg_offset<N>(type, n)];
        mask |= (uint32_t)(qv[n] != 0) << n;
    }
    if (!has) mask = 0;
    const int last = group_max<G>(mask ? cg * 16 + 31 - __builtin_clz(mask) : -1);
    int dsig = 0;
    const int first = __builtin_ctz(mask | 0x10000), lastnz = 31 - __builtin_clz(mask | 1);
    // CGs after the last significant one are all zero; the last CG's mask already
    // stops at the last significant position (quant.cpp:264-268)
    if (has && cg <= (last >> 4) && mask && lastnz - first >= 4)   // SBH_THRESHOLD (common.h:273)
    {
        int sum = 0, fq = 0;
#pragma unroll
        for (int n = 0; n < 16; n++)
        {
            sum += qv[n];
            fq = n == first ? qv[n] : fq;
        }
        const int signbit = fq > 0 ? 0 : 1;
        if (signbit != (sum & 1))
        {
            const int top = cg == (last >> 4) ? (last & 15) : 15;
            int cv[16];
#pragma unroll
            for (int n = 0; n < 16; n++) cv[n] = C[corner + cg_offset<N>(type, n)];
            int min_n, change;
            sbh_pick(qv, cv, mask, top, signbit, qscale, qadd, qbits, min_n, change);
            int qm = 0, cm = 0;
#pragma unroll
            for (int n = 0; n < 16; n++)
                if (n == min_n) { qm = qv[n]; cm = cv[n]; }
            if (qm == 32767 || qm == -32768) change = -1;
            if (!qm) dsig++;
            else if (change == -1 && (qm == 1 || qm == -1)) dsig--;
            const int sm = cm < 0 ? -1 : 0;
            Q[corner + cg_offset<N>(type, min_n)] = (int16_t)(qm + ((change ^ sm) - sm));
        }
    }
    return group_sum<G>(dsig);
}

// sign_hide as straight-line code (round 5): every lane of every TU group runs the candidate search and the
// decision is a predicate on the one store — the TUs of a wave (8 or 4 groups) take different branches of
// sign_hide (no hiding / parity already right / a CG past the last), which the branchy form executes one
// after another with exec-mask juggling.  `active` = the TU wants hiding (sign_hide && numSig >= 2).
template <int N, int G>
__device__ __forceinline__ int sign_hide_bf(int16_t* Q, const int16_t* C, const uint16_t* scan, int type, int lane,
                                            int qscale, int qadd, int qbits, bool active)
{
    constexpr int NCG = N * N / 16;
    static_assert(NCG <= G, "one coefficient group per lane");
    const bool has = lane < NCG;
    const int cg = has ? lane : 0;
    const int corner = scan[cg * 16];
    int qv[16], cv[16];
    uint32_t mask = 0;
    int sum = 0;
#pragma unroll
    for (int n = 0; n < 16; n++)
    {
        const int o = corner + cg_offset<N>(type, n);
        qv[n] = Q[o];
        cv[n] = C[o];
        mask |= (uint32_t)(qv[n] != 0) << n;
        sum += qv[n];
    }
    if (!has || !active) mask = 0;
    const int last = group_max<G>(mask ? cg * 16 + 31 - __builtin_clz(mask) : -1);
    const int first = __builtin_ctz(mask | 0x10000), lastnz = 31 - __builtin_clz(mask | 1);
    int fq = 0;
#pragma unroll
    for (int n = 0; n < 16; n++) fq = n == first ? qv[n] : fq;
    const int signbit = fq > 0 ? 0 : 1;
    const bool go = mask && cg <= (last >> 4) && lastnz - first >= 4 && signbit != (sum & 1);
    const int top = cg == (last >> 4) ? (last & 15) : 15;
    int min_n, change;
    sbh_pick(qv, cv, mask, top, signbit, qscale, qadd, qbits, min_n, change);
    int qm = 0, cm = 0;
#pragma unroll
    for (int n = 0; n < 16; n++)
    {
        qm = n == min_n ? qv[n] : qm;
        cm = n == min_n ? cv[n] : cm;
    }
    change = (qm == 32767 || qm == -32768) ? -1 : change;
    const int dsig = !go ? 0 : !qm ? 1 : (change == -1 && (qm == 1 || qm == -1)) ? -1 : 0;
    const int sm = cm < 0 ? -1 : 0;
    if (go) Q[corner + cg_offset<N>(type, min_n)] = (int16_t)(qm + ((change ^ sm) - sm));
    return group_sum<G>(dsig);
}

template <typename P, int N>
__device__ __forceinline__ void load_n(const P* p, int (&o)[N])
{
    constexpr int C = N < 16 ? N : 16;
#pragma unroll
    for (int i = 0; i < N; i += C)
    {
        int t[C];
        load_row<P, C>(p + i, t);
#pragma unroll
        for (int k = 0; k < C; k++) o[i + k] = t[k];
    }
}

template <typename P, int N>
__device__ __forceinline__ void store_n(P* p, const int (&v)[N])
{
    constexpr int C = N < 16 ? N : 16;
#pragma unroll
    for (int i = 0; i < N; i += C)
    {
        int t[C];
#pragma unroll
        for (int k = 0; k < C; k++) t[k] = v[i + k];
        store_row<P, C>(p + i, t);
    }
}

struct TuArgs
{
    const void* fenc;
    const int64_t* fenc_off;
    int64_t fenc_stride;
    const void* pred;
    const int64_t* pred_off;
    int64_t pred_stride;
    int16_t* resi;              // optional
    const int64_t* resi_off;
    int64_t resi_stride;
    int16_t* coeff;
    const int64_t* coeff_off;
    void* recon;
    const int64_t* recon_off;
    int64_t recon_stride;
    uint32_t* num_sig;
    const uint8_t* qp;
    const uint8_t* scan;        // optional (NULL = diagonal)
    int n, is_luma, is_intra, i_slice, sign_hide, depth;
};

__host__ __device__ inline TuArgs tu_args(const x265amd_tu_batch& b, int depth)
{
    return TuArgs{ b.fenc, b.fenc_off, (int64_t)b.fenc_stride, b.pred, b.pred_off, (int64_t)b.pred_stride,
                   b.resi, b.resi_off, (int64_t)b.resi_stride, b.coeff, b.coeff_off, b.recon, b.recon_off,
                   (int64_t)b.recon_stride, b.num_sig, b.qp, b.scan, b.n, !!b.is_luma, !!b.is_intra, !!b.i_slice,
                   !!b.sign_hide, depth };
}

// BF (round 5, default): sign hiding and the reconstruction as straight-line code — every TU group of a
// wave computes the full inverse and the sign-hiding search, the uncoded / DC-only / coded cases are
// selects (the DC-only shortcut, quant.cpp:526-538, equals the full inverse of a DC-only block; it is kept
// as its own select all the same)
template <typename P, int N, bool BF = false>
__device__ __forceinline__ void tu_groups(const TuArgs& a, int64_t blk)
{
    constexpr int LOG2 = N == 4 ? 2 : N == 8 ? 3 : N == 16 ? 4 : 5;
    constexpr int PT = N + 2;                 // transposition tile pitch (int16), spreads LDS banks
    constexpr int JOBS = X265AMD_BLOCK / N;
    constexpr int NCG = N * N / 16;
    __shared__ int16_t lds_t[JOBS][N * PT];   // stage tiles; DCT coefficients (pitch N) during quant/SBH
    __shared__ int16_t lds_q[JOBS][N * N];    // quantized coefficients (raster, as coeff[])
    const int slot = threadIdx.x / N, r = threadIdx.x % N;
    const int64_t j = blk * JOBS + slot;
    if (j >= a.n) return;                     // whole groups only; no block barrier below
    int16_t* T = lds_t[slot];
    int16_t* Q = lds_q[slot];
    const int depth = a.depth, maxv = (1 << depth) - 1;
    const int qp = a.qp[j], rem = qp % 6, per = qp / 6;
    const bool use_dst = N == 4 && a.is_luma && a.is_intra;
    const int tshift = 15 - depth - LOG2;     // MAX_TR_DYNAMIC_RANGE - depth - log2 (quant.cpp:411)
    const P* pf = (const P*)a.fenc + a.fenc_off[j] + r * a.fenc_stride;
    const P* pp = (const P*)a.pred + a.pred_off[j] + r * a.pred_stride;

    int x[N], y[N];
    PixRow<P, N> frow, prow;                  // kept packed for the reconstruction
    frow.load(pf);
    prow.load(pp);
#pragma unroll
    for (int i = 0; i < N; i++) x[i] = frow.get(i) - prow.get(i);

    // ---- forward transform: row r -> column r of T, then row r of T -> column r of the coefficients
    const int fsh1 = LOG2 - 1 + depth - 8, fsh2 = LOG2 + 6;
    if constexpr (N == 4)
    {
        if (use_dst) dst_fwd(x, y); else fwd_1d<4>(x, y);
    }
    else
        fwd_1d<N>(x, y);
#pragma unroll
    for (int k = 0; k < N; k++) T[k * PT + r] = (int16_t)fwd_round(y[k], fsh1);
    wave_sync();
#pragma unroll
    for (int i = 0; i < N; i += 2)
    {
        const uint32_t v = *(const uint32_t*)&T[r * PT + i];
        x[i] = (int16_t)(v & 0xffff);
        x[i + 1] = (int16_t)(v >> 16);
    }
    if constexpr (N == 4)
    {
        if (use_dst) dst_fwd(x, y); else fwd_1d<4>(x, y);
    }
    else
        fwd_1d<N>(x, y);
    wave_sync();                              // every lane has read its row of T

    // ---- quant (quant_c): lane r quantizes column r
    const int qscale = quant_scale(rem);
    const int qbits = 14 + per + tshift;
    const int qadd = (a.i_slice ? 171 : 85) << (qbits - 9);
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < N; k++)
    {
        const int c = fwd_round(y[k], fsh2);
        const int tmp = (c < 0 ? -c : c) * qscale;
        int lvl = (tmp + qadd) >> qbits;
        cnt += lvl != 0;
        lvl = c < 0 ? -lvl : lvl;
        T[k * N + r] = (int16_t)c;
        Q[k * N + r] = (int16_t)clip16(lvl);
    }
    int num_sig = group_sum<N>(cnt);

    // ---- sign-bit hiding (signBitHidingHDQ): one coefficient group per lane
    if constexpr (BF)
    {
        if (a.sign_hide)
        {
            wave_sync();
            const int st = a.scan ? a.scan[j] : 0;
            const uint16_t* scan = N == 4 ? c_scan.s4[st] : N == 8 ? c_scan.s8[st] : N == 16 ? c_scan.s16 : c_scan.s32;
            num_sig += sign_hide_bf<N, N>(Q, T, scan, st, r, qscale, qadd, qbits, num_sig >= 2);
            wave_sync();
        }
    }
    else if (a.sign_hide && num_sig >= 2)
    {
        wave_sync();
        const int st = a.scan ? a.scan[j] : 0;
        const uint16_t* scan = N == 4 ? c_scan.s4[st] : N == 8 ? c_scan.s8[st] : N == 16 ? c_scan.s16 : c_scan.s32;
        num_sig += sign_hide<N, N>(Q, T, scan, st, r, qscale, qadd, qbits);
        wave_sync();
    }

    // ---- coefficients out: lane r stores row r (the TU is one contiguous N*N block)
    {
        int v[N];
#pragma unroll
        for (int i = 0; i < N; i += 2)
        {
            const uint32_t w = *(const uint32_t*)&Q[r * N + i];
            v[i] = (int16_t)(w & 0xffff);
            v[i + 1] = (int16_t)(w >> 16);
        }
        store_n<int16_t, N>(a.coeff + a.coeff_off[j] + r * N, v);
        if (r == 0) a.num_sig[j] = (uint32_t)num_sig;
    }

    // ---- reconstruction (invtransformNxN + add_ps, or copy_pp)
    int f[N], p[N], res[N];
#pragma unroll
    for (int i = 0; i < N; i++) { f[i] = frow.get(i); p[i] = prow.get(i); }
    if constexpr (BF)
    {
        const int scale = inv_quant_scale(rem) << per;
        const int dsh = 20 - 14 - tshift;
        const int dadd = 1 << (dsh - 1);
        const int q0 = Q[0];
        int c[N];
#pragma unroll
        for (int k = 0; k < N; k++) c[k] = clip16((Q[k * N + r] * scale + dadd) >> dsh);
        if constexpr (N == 4)
        {
            if (use_dst) dst_inv(c, y); else inv_1d<4>(c, y);
        }
        else
            inv_1d<N>(c, y);
#pragma unroll
        for (int k = 0; k < N; k++) T[r * PT + k] = (int16_t)inv_round(y[k], 7);
        wave_sync();
#pragma unroll
        for (int k = 0; k < N; k++) c[k] = T[k * PT + r];
        if constexpr (N == 4)
        {
            if (use_dst) dst_inv(c, y); else inv_1d<4>(c, y);
        }
        else
            inv_1d<N>(c, y);
        const int ish2 = 12 - (depth - 8);
        const int dq0 = clip16((q0 * scale + dadd) >> dsh);
        const int sh2 = 12 - (depth - 8) - 3;
        const int dc = (int16_t)((((dq0 + 1) >> 1) * 8 + (1 << (sh2 - 1))) >> sh2);
        const bool dconly = num_sig == 1 && q0 != 0 && !use_dst;
#pragma unroll
        for (int k = 0; k < N; k++)
            res[k] = num_sig == 0 ? f[k] - p[k] : dconly ? dc : inv_round(y[k], ish2);
    }
    else if (num_sig == 0)
    {
#pragma unroll
        for (int i = 0; i < N; i++) res[i] = f[i] - p[i];
    }
    else
    {
        const int scale = inv_quant_scale(rem) << per;
        const int dsh = 20 - 14 - tshift;     // QUANT_IQUANT_SHIFT - QUANT_SHIFT - transformShift
        const int dadd = 1 << (dsh - 1);
        const int q0 = Q[0];
        if (num_sig == 1 && q0 != 0 && !use_dst)
        {
            // DC-only shortcut (quant.cpp:526-538)
            const int dq0 = clip16((q0 * scale + dadd) >> dsh);
            const int sh2 = 12 - (depth - 8) - 3;
            const int dc = (int16_t)((((dq0 + 1) >> 1) * 8 + (1 << (sh2 - 1))) >> sh2);
#pragma unroll
            for (int i = 0; i < N; i++) res[i] = dc;
        }
        else
        {
            int c[N];
#pragma unroll
            for (int k = 0; k < N; k++) c[k] = clip16((Q[k * N + r] * scale + dadd) >> dsh);
            if constexpr (N == 4)
            {
                if (use_dst) dst_inv(c, y); else inv_1d<4>(c, y);
            }
            else
                inv_1d<N>(c, y);
#pragma unroll
            for (int k = 0; k < N; k++) T[r * PT + k] = (int16_t)inv_round(y[k], 7);
            wave_sync();
#pragma unroll
            for (int k = 0; k < N; k++) c[k] = T[k * PT + r];
            if constexpr (N == 4)
            {
                if (use_dst) dst_inv(c, y); else inv_1d<4>(c, y);
            }
            else
                inv_1d<N>(c, y);
            const int ish2 = 12 - (depth - 8);
#pragma unroll
            for (int k = 0; k < N; k++) res[k] = inv_round(y[k], ish2);
        }
    }
    int rec[N];
#pragma unroll
    for (int i = 0; i < N; i++)
    {
        const int v = num_sig ? p[i] + res[i] : p[i];
        rec[i] = v < 0 ? 0 : (v > maxv ? maxv : v);
    }
    store_n<P, N>((P*)a.recon + a.recon_off[j] + r * a.recon_stride, rec);
    if (a.resi)
        store_n<int16_t, N>(a.resi + a.resi_off[j] + r * a.resi_stride, res);
}

// one workgroup = X265AMD_BLOCK / N TU groups (the body above with the workgroup's block index)
template <typename P, int N, bool BF = false>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_tu(const TuArgs a)
{
    tu_groups<P, N, BF>(a, xcd_block());
}

// ---------------------------------------------------------------- 32x32 on the matrix cores
// One wavefront per TU (grid-stride over TUs, constant fragments loaded once
// per wave).  The four transform stages are the exact f16 MFMA products of
// k_tr32_mfma (transform.hip): the residual rows are the A operand of the
// forward stage 1, the stage-1 accumulator feeds stage 2 from registers, and
// the coefficient accumulator (column r = l & 31, rows (i&3) + 8(i>>2) + 4h)
// is quantized in registers.  Sign-bit hiding maps the 64 coefficient groups
// of a 32x32 TU onto the 64 lanes, one CG each.  Coefficients, residual and
// reconstruction leave through 16-element row segments (two lanes per row).
constexpr int kTuWaves = X265AMD_BLOCK / 64;

template <typename P>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_tu32_mfma(const TuArgs a)
{
    __shared__ int16_t lds_c[kTuWaves][32 * 32];   // DCT coefficients; later the inverse output
    __shared__ int16_t lds_q[kTuWaves][32 * 32];   // quantized coefficients
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, h = l >> 5;
    int16_t* Cs = lds_c[w];
    int16_t* Q = lds_q[w];
    const int depth = a.depth, maxv = (1 << depth) - 1;
    const int fsh1 = 4 + depth - 8, fsh2 = 11, ish2 = 12 - (depth - 8);
    const int tshift = 15 - depth - 5;
    const int io_row = l >> 1, io_col = 16 * (l & 1);

    // constant operands (as k_tr32_mfma): stage 1 in natural k order, stage 2 in accumulator order
    f16x8 ft1[2], ft2[2], it1[2], it2[2];
#pragma unroll
    for (int st = 0; st < 2; st++)
#pragma unroll
        for (int j = 0; j < 8; j++)
        {
            const int kn = 16 * st + 8 * h + j, kp = 16 * st + 8 * (j >> 2) + 4 * h + (j & 3);
            ft1[st][j] = (_Float16)c_t32.m[r][kn];
            ft2[st][j] = (_Float16)c_t32.m[r][kp];
            it1[st][j] = (_Float16)c_t32.m[kn][r];
            it2[st][j] = (_Float16)c_t32.m[kp][r];
        }

    const int64_t step = (int64_t)gridDim.x * kTuWaves;
    for (int64_t j = (int64_t)blockIdx.x * kTuWaves + w; j < a.n; j += step)
    {
        const P* pf = (const P*)a.fenc + a.fenc_off[j];
        const P* pp = (const P*)a.pred + a.pred_off[j];
        const int qp = a.qp[j], rem = qp % 6, per = qp / 6;
        // the reconstruction's row segments, loaded with the residual's (one global round trip per TU)
        PixRow<P, 16> fio, pio;
        fio.load(pf + io_row * a.fenc_stride + io_col);
        pio.load(pp + io_row * a.pred_stride + io_col);

        // ---- forward stage 1: A = residual rows (row r, columns 16 st + 8 h + 0..7)
        int x[2][8];
#pragma unroll
        for (int st = 0; st < 2; st++)
        {
            int f[8], p[8];
            load_row<P, 8>(pf + r * a.fenc_stride + 16 * st + 8 * h, f);
            load_row<P, 8>(pp + r * a.pred_stride + 16 * st + 8 * h, p);
#pragma unroll
            for (int k = 0; k < 8; k++) x[st][k] = f[k] - p[k];
        }
        f32x16 lo = {}, hi = {};
#pragma unroll
        for (int st = 0; st < 2; st++)
        {
            f16x8 xl, xh;
            split10i<8>(x[st], xl, xh);
            lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, ft1[st], lo, 0, 0, 0);
            hi = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, ft1[st], hi, 0, 0, 0);
        }
        int v[16];
#pragma unroll
        for (int i = 0; i < 16; i++) v[i] = fwd_round((int)hi[i] * 1024 + (int)lo[i], fsh1);
        // ---- forward stage 2 from registers: Dst = T * U'
        lo = f32x16{};
        hi = f32x16{};
#pragma unroll
        for (int st = 0; st < 2; st++)
        {
            int y[8];
#pragma unroll
            for (int k = 0; k < 8; k++) y[k] = v[8 * st + k];
            f16x8 xl, xh;
            split10i<8>(y, xl, xh);
            lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(ft2[st], xl, lo, 0, 0, 0);
            hi = __builtin_amdgcn_mfma_f32_32x32x16_f16(ft2[st], xh, hi, 0, 0, 0);
        }

        // ---- quant in registers: coefficient (row (i&3) + 8(i>>2) + 4h, column r)
        const int qscale = quant_scale(rem);
        const int qbits = 14 + per + tshift;
        const int qadd = (a.i_slice ? 171 : 85) << (qbits - 9);
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < 16; i++)
        {
            const int c = fwd_round((int)hi[i] * 1024 + (int)lo[i], fsh2);
            const int tmp = (c < 0 ? -c : c) * qscale;
            int lvl = (tmp + qadd) >> qbits;
            cnt += lvl != 0;
            lvl = c < 0 ? -lvl : lvl;
            const int pos = ((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r;
            Cs[pos] = (int16_t)c;
            Q[pos] = (int16_t)clip16(lvl);
        }
        int num_sig = group_sum<64>(cnt);
        wave_sync();
        if (a.sign_hide && num_sig >= 2)             // wave-uniform: one TU per wave
        {
            num_sig += sign_hide_bf<32, 64>(Q, Cs, c_scan.s32, 0, l, qscale, qadd, qbits, true);
            wave_sync();
        }

        // ---- coefficients out (16-element row segments)
        int16_t* pc = a.coeff + a.coeff_off[j] + io_row * 32 + io_col;
        stu<uint4>(pc, ldu<uint4>(&Q[io_row * 32 + io_col]));
        stu<uint4>(pc + 8, ldu<uint4>(&Q[io_row * 32 + io_col + 8]));
        if (l == 0) a.num_sig[j] = (uint32_t)num_sig;

        // ---- reconstruction
        int f[16], p[16], res[16];
#pragma unroll
        for (int k = 0; k < 16; k++) { f[k] = fio.get(k); p[k] = pio.get(k); }
        if (num_sig == 0)
        {
#pragma unroll
            for (int k = 0; k < 16; k++) res[k] = f[k] - p[k];
        }
        else
        {
            const int scale = inv_quant_scale(rem) << per;
            const int dsh = 20 - 14 - tshift, dadd = 1 << (dsh - 1);
            const int q0 = Q[0];
            if (num_sig == 1 && q0 != 0)
            {
                const int dq0 = clip16((q0 * scale + dadd) >> dsh);
                const int sh2 = 12 - (depth - 8) - 3;
                const int dc = (int16_t)((((dq0 + 1) >> 1) * 8 + (1 << (sh2 - 1))) >> sh2);
#pragma unroll
                for (int k = 0; k < 16; k++) res[k] = dc;
            }
            else
            {
                // inverse stage 1: A = dequantized coefficient column r (rows 16 st + 8 h + 0..7)
                lo = f32x16{};
                hi = f32x16{};
#pragma unroll
                for (int st = 0; st < 2; st++)
                {
                    int c[8];
#pragma unroll
                    for (int k = 0; k < 8; k++) c[k] = clip16((Q[(16 * st + 8 * h + k) * 32 + r] * scale + dadd) >> dsh);
                    f16x8 xl, xh;
                    split10i<8>(c, xl, xh);
                    lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, it1[st], lo, 0, 0, 0);
                    hi = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, it1[st], hi, 0, 0, 0);
                }
#pragma unroll
                for (int i = 0; i < 16; i++) v[i] = inv_round((int)hi[i] * 1024 + (int)lo[i], 7);
                lo = f32x16{};
                hi = f32x16{};
#pragma unroll
                for (int st = 0; st < 2; st++)
                {
                    int y[8];
#pragma unroll
                    for (int k = 0; k < 8; k++) y[k] = v[8 * st + k];
                    f16x8 xl, xh;
                    split10i<8>(y, xl, xh);
                    lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, it2[st], lo, 0, 0, 0);
                    hi = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, it2[st], hi, 0, 0, 0);
                }
                // residual (row (i&3) + 8(i>>2) + 4h, column r) -> LDS -> row segments
#pragma unroll
                for (int i = 0; i < 16; i++)
                    Cs[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = (int16_t)inv_round((int)hi[i] * 1024 + (int)lo[i], ish2);
                wave_sync();
                load_row16<16>(&Cs[io_row * 32 + io_col], res);
            }
        }
        int rec[16];
#pragma unroll
        for (int k = 0; k < 16; k++)
        {
            const int t = num_sig ? p[k] + res[k] : p[k];
            rec[k] = t < 0 ? 0 : (t > maxv ? maxv : t);
        }
        store_row<P, 16>((P*)a.recon + a.recon_off[j] + io_row * a.recon_stride + io_col, rec);
        if (a.resi) store_n<int16_t, 16>(a.resi + a.resi_off[j] + io_row * a.resi_stride + io_col, res);
        wave_sync();                                 // LDS reuse by the next TU of this wave
    }
}

// ---------------------------------------------------------------- 32x32 on the integer matrix cores
// k_tu32_mfma's chain with every transform stage as the int8 byte-split products of k_tr32_i8
// (transform.hip): exact int32 sums, one v_lshl_add per element to recombine, a third of the
// VALU work of the f16 split.  X265AMD_TU_I8=0 selects the f16 kernel.
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ void split_bytes(const uint32_t (&d)[8], i32x4& lo, i32x4& hi)
{
#pragma unroll
    for (int q = 0; q < 4; q++)
    {
        lo[q] = (int)(__builtin_amdgcn_perm(d[2 * q + 1], d[2 * q], 0x06040200u) ^ 0x80808080u);
        hi[q] = (int)__builtin_amdgcn_perm(d[2 * q + 1], d[2 * q], 0x07050301u);
    }
}
struct ColSumsTu { int v[32]; };
constexpr ColSumsTu make_colsums_tu()
{
    ColSumsTu c{};
    for (int j = 0; j < 32; j++)
        for (int k = 0; k < 32; k++) c.v[j] += 128 * kT32.m[k][j];
    return c;
}
static __constant__ ColSumsTu c_colsum128_tu = make_colsums_tu();

template <typename P>
__device__ __forceinline__ void tu32_i8_waves(const TuArgs& a, int64_t blk, int64_t nblk)
{
    __shared__ int16_t lds_c[kTuWaves][32 * 32];   // DCT coefficients; later the inverse output
    __shared__ int16_t lds_q[kTuWaves][32 * 32];   // quantized coefficients
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, h = l >> 5;
    int16_t* Cs = lds_c[w];
    int16_t* Q = lds_q[w];
    const int depth = a.depth, maxv = (1 << depth) - 1;
    const int fsh1 = 4 + depth - 8, fsh2 = 11, ish2 = 12 - (depth - 8);
    const int tshift = 15 - depth - 5;
    const int io_row = l >> 1, io_col = 16 * (l & 1);

    // constant int8 operands (as k_tr32_i8 in transform.hip): stage 1 in the lane half's natural k
    // order (k = 16h + j), stage 2 in the accumulator's row order (k = (j&3) + 8(j>>2) + 4h)
    i32x4 fc1, fc2, ic1, ic2;
#pragma unroll
    for (int q = 0; q < 4; q++)
    {
        uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
#pragma unroll
        for (int e = 0; e < 4; e++)
        {
            const int jj = 4 * q + e, kn = 16 * h + jj, kp = (jj & 3) + 8 * (jj >> 2) + 4 * h;
            w0 |= (uint32_t)(uint8_t)(int8_t)c_t32.m[r][kn] << (8 * e);
            w1 |= (uint32_t)(uint8_t)(int8_t)c_t32.m[r][kp] << (8 * e);
            w2 |= (uint32_t)(uint8_t)(int8_t)c_t32.m[kn][r] << (8 * e);
            w3 |= (uint32_t)(uint8_t)(int8_t)c_t32.m[kp][r] << (8 * e);
        }
        fc1[q] = (int)w0; fc2[q] = (int)w1; ic1[q] = (int)w2; ic2[q] = (int)w3;
    }
    // lo-byte bias corrections (k_tr32_i8): forward stage 1 on the lane's column (row sum of T: zero
    // unless r == 0), forward stage 2 on output row 0 (register 0 of lane half 0), inverse stages on
    // the lane's column (128 x the column sum of T at r)
    const int fk1 = (r == 0 ? 128 * 64 * 32 : 0) + (1 << (fsh1 - 1));
    const int fk2 = (1 << (fsh2 - 1)), fk20 = h == 0 ? 128 * 64 * 32 : 0;
    const int icol = c_colsum128_tu.v[r];

    const int64_t step = nblk * kTuWaves;
    for (int64_t j = blk * kTuWaves + w; j < a.n; j += step)
    {
        const P* pf = (const P*)a.fenc + a.fenc_off[j];
        const P* pp = (const P*)a.pred + a.pred_off[j];
        const int qp = a.qp[j], rem = qp % 6, per = qp / 6;
        // the reconstruction's row segments, loaded with the residual's (one global round trip per TU)
        PixRow<P, 16> fio, pio;
        fio.load(pf + io_row * a.fenc_stride + io_col);
        pio.load(pp + io_row * a.pred_stride + io_col);

        // ---- forward stage 1: A = residual row r, columns 16h + 0..15
        uint32_t x[8];
        {
            int f[16], p[16];
            load_row<P, 16>(pf + r * a.fenc_stride + 16 * h, f);
            load_row<P, 16>(pp + r * a.pred_stride + 16 * h, p);
#pragma unroll
            for (int q = 0; q < 8; q++) x[q] = pack16(f[2 * q] - p[2 * q], f[2 * q + 1] - p[2 * q + 1]);
        }
        i32x4 xl, xh;
        split_bytes(x, xl, xh);
        i32x16 lo = __builtin_amdgcn_mfma_i32_32x32x32_i8(xl, fc1, (i32x16){}, 0, 0, 0);
        i32x16 hi = __builtin_amdgcn_mfma_i32_32x32x32_i8(xh, fc1, (i32x16){}, 0, 0, 0);
        int v[16];
#pragma unroll
        for (int i = 0; i < 16; i++) v[i] = (int)(((uint32_t)hi[i] << 8) + (uint32_t)lo[i]) + fk1 >> fsh1;
        // ---- forward stage 2 from registers: Dst = T * U' (coefficients in the accumulator layout the
        //      quant / sign hiding below expect); the int16 wrap of stage 1 is the byte split
#pragma unroll
        for (int q = 0; q < 8; q++) x[q] = pack16(v[2 * q], v[2 * q + 1]);
        split_bytes(x, xl, xh);
        lo = __builtin_amdgcn_mfma_i32_32x32x32_i8(fc2, xl, (i32x16){}, 0, 0, 0);
        hi = __builtin_amdgcn_mfma_i32_32x32x32_i8(fc2, xh, (i32x16){}, 0, 0, 0);

        // ---- quant in registers: coefficient (row (i&3) + 8(i>>2) + 4h, column r)
        const int qscale = quant_scale(rem);
        const int qbits = 14 + per + tshift;
        const int qadd = (a.i_slice ? 171 : 85) << (qbits - 9);
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < 16; i++)
        {
            const int c = (int)(int16_t)(((int)(((uint32_t)hi[i] << 8) + (uint32_t)lo[i]) + fk2 + (i == 0 ? fk20 : 0)) >> fsh2);
            const int tmp = (c < 0 ? -c : c) * qscale;
            int lvl = (tmp + qadd) >> qbits;
            cnt += lvl != 0;
            lvl = c < 0 ? -lvl : lvl;
            const int pos = ((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r;
            Cs[pos] = (int16_t)c;
            Q[pos] = (int16_t)clip16(lvl);
        }
        int num_sig = group_sum<64>(cnt);
        wave_sync();
        if (a.sign_hide && num_sig >= 2)             // wave-uniform: one TU per wave
        {
            num_sig += sign_hide_bf<32, 64>(Q, Cs, c_scan.s32, 0, l, qscale, qadd, qbits, true);
            wave_sync();
        }

        // ---- coefficients out (16-element row segments)
        int16_t* pc = a.coeff + a.coeff_off[j] + io_row * 32 + io_col;
        stu<uint4>(pc, ldu<uint4>(&Q[io_row * 32 + io_col]));
        stu<uint4>(pc + 8, ldu<uint4>(&Q[io_row * 32 + io_col + 8]));
        if (l == 0) a.num_sig[j] = (uint32_t)num_sig;

        // ---- reconstruction
        int f[16], p[16], res[16];
#pragma unroll
        for (int k = 0; k < 16; k++) { f[k] = fio.get(k); p[k] = pio.get(k); }
        if (num_sig == 0)
        {
#pragma unroll
            for (int k = 0; k < 16; k++) res[k] = f[k] - p[k];
        }
        else
        {
            const int scale = inv_quant_scale(rem) << per;
            const int dsh = 20 - 14 - tshift, dadd = 1 << (dsh - 1);
            const int q0 = Q[0];
            if (num_sig == 1 && q0 != 0)
            {
                const int dq0 = clip16((q0 * scale + dadd) >> dsh);
                const int sh2 = 12 - (depth - 8) - 3;
                const int dc = (int16_t)((((dq0 + 1) >> 1) * 8 + (1 << (sh2 - 1))) >> sh2);
#pragma unroll
                for (int k = 0; k < 16; k++) res[k] = dc;
            }
            else
            {
                // inverse stage 1: A = dequantized coefficient column r (rows 16h + 0..15)
#pragma unroll
                for (int q = 0; q < 8; q++)
                    x[q] = pack16(clip16((Q[(16 * h + 2 * q) * 32 + r] * scale + dadd) >> dsh),
                                  clip16((Q[(16 * h + 2 * q + 1) * 32 + r] * scale + dadd) >> dsh));
                split_bytes(x, xl, xh);
                lo = __builtin_amdgcn_mfma_i32_32x32x32_i8(xl, ic1, (i32x16){}, 0, 0, 0);
                hi = __builtin_amdgcn_mfma_i32_32x32x32_i8(xh, ic1, (i32x16){}, 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 16; i++)
                    v[i] = clip16(((int)(((uint32_t)hi[i] << 8) + (uint32_t)lo[i]) + icol + 64) >> 7);
#pragma unroll
                for (int q = 0; q < 8; q++) x[q] = pack16(v[2 * q], v[2 * q + 1]);
                split_bytes(x, xl, xh);
                lo = __builtin_amdgcn_mfma_i32_32x32x32_i8(xl, ic2, (i32x16){}, 0, 0, 0);
                hi = __builtin_amdgcn_mfma_i32_32x32x32_i8(xh, ic2, (i32x16){}, 0, 0, 0);
                // residual (row (i&3) + 8(i>>2) + 4h, column r) -> LDS -> row segments
#pragma unroll
                for (int i = 0; i < 16; i++)
                    Cs[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] =
                        (int16_t)clip16(((int)(((uint32_t)hi[i] << 8) + (uint32_t)lo[i]) + icol + (1 << (ish2 - 1))) >> ish2);
                wave_sync();
                load_row16<16>(&Cs[io_row * 32 + io_col], res);
            }
        }
        int rec[16];
#pragma unroll
        for (int k = 0; k < 16; k++)
        {
            const int t = num_sig ? p[k] + res[k] : p[k];
            rec[k] = t < 0 ? 0 : (t > maxv ? maxv : t);
        }
        store_row<P, 16>((P*)a.recon + a.recon_off[j] + io_row * a.recon_stride + io_col, rec);
        if (a.resi) store_n<int16_t, 16>(a.resi + a.resi_off[j] + io_row * a.resi_stride + io_col, res);
        wave_sync();                                 // LDS reuse by the next TU of this wave
    }
}

template <typename P>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_tu32_i8(const TuArgs a)
{
    tu32_i8_waves<P>(a, blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------- 4x4: one lane per TU
// The whole chain in registers (no LDS, no cross-lane traffic): 4x4 TUs are
// the most frequent residual blocks and too small to share between lanes.
// Sign-bit hiding works on the single coefficient group in scan order, the
// scan type selecting between three immediate permutations per position.
template <typename P>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_tu4(const TuArgs a)
{
    const int64_t j = (int64_t)xcd_block() * X265AMD_BLOCK + threadIdx.x;
    if (j >= a.n) return;
    const int depth = a.depth, maxv = (1 << depth) - 1;
    const int qp = a.qp[j], rem = qp % 6, per = qp / 6;
    const bool use_dst = a.is_luma && a.is_intra;
    const int tshift = 15 - depth - 2;
    const P* pf = (const P*)a.fenc + a.fenc_off[j];
    const P* pp = (const P*)a.pred + a.pred_off[j];
    int f[4][4], p[4][4], m[4][4], t[4][4];
#pragma unroll
    for (int r = 0; r < 4; r++)
    {
        load_row<P, 4>(pf + r * a.fenc_stride, f[r]);
        load_row<P, 4>(pp + r * a.pred_stride, p[r]);
#pragma unroll
        for (int c = 0; c < 4; c++) m[r][c] = f[r][c] - p[r][c];
    }
    // forward: row i -> column i of t; row i of t -> column i of the coefficients (k_tr4)
    const int sh1 = 1 + depth - 8;
#pragma unroll
    for (int i = 0; i < 4; i++)
    {
        int y[4];
        if (use_dst) dst_fwd(m[i], y); else fwd_1d<4>(m[i], y);
#pragma unroll
        for (int k = 0; k < 4; k++) t[k][i] = fwd_round(y[k], sh1);
    }
    int cf[16];                                   // DCT coefficients, raster
#pragma unroll
    for (int i = 0; i < 4; i++)
    {
        int y[4];
        if (use_dst) dst_fwd(t[i], y); else fwd_1d<4>(t[i], y);
#pragma unroll
        for (int k = 0; k < 4; k++) cf[k * 4 + i] = fwd_round(y[k], 8);
    }
    const int qscale = quant_scale(rem);
    const int qbits = 14 + per + tshift;
    const int qadd = (a.i_slice ? 171 : 85) << (qbits - 9);
    int q[16];
    int num_sig = 0;
#pragma unroll
    for (int i = 0; i < 16; i++)
    {
        const int c = cf[i];
        int lvl = ((c < 0 ? -c : c) * qscale + qadd) >> qbits;
        num_sig += lvl != 0;
        q[i] = clip16(c < 0 ? -lvl : lvl);
    }
    if (a.sign_hide && num_sig >= 2)
    {
        constexpr int diag[16] = { 0, 4, 1, 8, 5, 2, 12, 9, 6, 3, 13, 10, 7, 14, 11, 15 };
        constexpr int ver[16] = { 0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15 };
        const int type = a.scan ? a.scan[j] : 0;
        int qv[16], cv[16];
        uint32_t mask = 0;
#pragma unroll
        for (int n = 0; n < 16; n++)
        {
            qv[n] = type == 1 ? q[n] : type == 2 ? q[ver[n]] : q[diag[n]];
            cv[n] = type == 1 ? cf[n] : type == 2 ? cf[ver[n]] : cf[diag[n]];
            mask |= (uint32_t)(qv[n] != 0) << n;
        }
        const int first = __builtin_ctz(mask), top = 31 - __builtin_clz(mask);
        int sum = 0, fq = 0;
#pragma unroll
        for (int n = 0; n < 16; n++) { sum += qv[n]; fq = n == first ? qv[n] : fq; }
        const int signbit = fq > 0 ? 0 : 1;
        if (top - first >= 4 && signbit != (sum & 1))   // SBH_THRESHOLD; parity mismatch
        {
            int min_n, change;
            sbh_pick(qv, cv, mask, top, signbit, qscale, qadd, qbits, min_n, change);
            int qm = 0, cm = 0;
#pragma unroll
            for (int n = 0; n < 16; n++)
                if (n == min_n) { qm = qv[n]; cm = cv[n]; }
            if (qm == 32767 || qm == -32768) change = -1;
            if (!qm) num_sig++;
            else if (change == -1 && (qm == 1 || qm == -1)) num_sig--;
            const int sm = cm < 0 ? -1 : 0;
            const int nv = (int16_t)(qm + ((change ^ sm) - sm));
            const int pos = type == 1 ? min_n : type == 2 ? (min_n & 3) * 4 + (min_n >> 2) : 0;
            int dpos = 0;
#pragma unroll
            for (int n = 0; n < 16; n++) dpos = n == min_n ? diag[n] : dpos;
            const int at = type == 0 ? dpos : pos;
#pragma unroll
            for (int i = 0; i < 16; i++) q[i] = i == at ? nv : q[i];
        }
    }
    {
        int16_t* pc = a.coeff + a.coeff_off[j];
        int r0[8], r1[8];
#pragma unroll
        for (int i = 0; i < 8; i++) { r0[i] = q[i]; r1[i] = q[8 + i]; }
        store_row<int16_t, 8>(pc, r0);
        store_row<int16_t, 8>(pc + 8, r1);
        a.num_sig[j] = (uint32_t)num_sig;
    }
    // reconstruction: m <- residual rows
    if (num_sig)
    {
        const int scale = inv_quant_scale(rem) << per;
        const int dsh = 20 - 14 - tshift, dadd = 1 << (dsh - 1);
        if (num_sig == 1 && q[0] != 0 && !use_dst)
        {
            const int dq0 = clip16((q[0] * scale + dadd) >> dsh);
            const int sh2 = 12 - (depth - 8) - 3;
            const int dc = (int16_t)((((dq0 + 1) >> 1) * 8 + (1 << (sh2 - 1))) >> sh2);
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int c = 0; c < 4; c++) m[r][c] = dc;
        }
        else
        {
            int d[4][4];
#pragma unroll
            for (int i = 0; i < 16; i++) d[i >> 2][i & 3] = clip16((q[i] * scale + dadd) >> dsh);
            // inverse: column jx of d -> row jx of t; column jx of t -> row jx of the residual (k_tr4)
#pragma unroll
            for (int jx = 0; jx < 4; jx++)
            {
                int c[4] = { d[0][jx], d[1][jx], d[2][jx], d[3][jx] }, y[4];
                if (use_dst) dst_inv(c, y); else inv_1d<4>(c, y);
#pragma unroll
                for (int k = 0; k < 4; k++) t[jx][k] = inv_round(y[k], 7);
            }
            const int ish2 = 12 - (depth - 8);
#pragma unroll
            for (int jx = 0; jx < 4; jx++)
            {
                int c[4] = { t[0][jx], t[1][jx], t[2][jx], t[3][jx] }, y[4];
                if (use_dst) dst_inv(c, y); else inv_1d<4>(c, y);
#pragma unroll
                for (int k = 0; k < 4; k++) m[jx][k] = inv_round(y[k], ish2);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 4; r++)
    {
        int rec[4];
#pragma unroll
        for (int c = 0; c < 4; c++)
        {
            const int v = num_sig ? p[r][c] + m[r][c] : p[r][c];
            rec[c] = v < 0 ? 0 : (v > maxv ? maxv : v);
        }
        store_row<P, 4>((P*)a.recon + a.recon_off[j] + r * a.recon_stride, rec);
        if (a.resi) store_row<int16_t, 4>(a.resi + a.resi_off[j] + r * a.resi_stride, m[r]);
    }
}

// the integer-MFMA 32x32 TU kernel, default (X265AMD_TU_I8=0 selects the f16 split form; measured,
// profiles/r04/tu32_i8_ab.txt: tu_pipeline 32x32 0.20 -> 0.26 of the HBM peak)
static bool tu_i8()
{
    static int v = -1;
    if (v < 0)
    {
        const char* e = getenv("X265AMD_TU_I8");
        v = e ? atoi(e) != 0 : 1;
    }
    return v != 0;
}

// X265AMD_TU_BF=1 selects the straight-line 8x8 / 16x16 form (k_tu<.., true>).  Off by default: on the box
// it measured slower than the branchy form (profiles/r05/tu_bf_ab.txt: 8x8 0.89 -> 0.99 ms, 16x16 0.70 ->
// 0.74-0.77 ms per launch) although it issues a quarter of the scalar instructions
static bool tu_bf()
{
    static int v = -1;
    if (v < 0)
    {
        const char* e = getenv("X265AMD_TU_BF");
        v = e ? atoi(e) != 0 : 0;
    }
    return v != 0;
}

template <typename P>
static int launch_tu(int log2, const TuArgs& a, hipStream_t st)
{
    const int N = 1 << log2;
    const uint32_t blocks = (uint32_t)((a.n + X265AMD_BLOCK / N - 1) / (X265AMD_BLOCK / N));
    switch (log2)
    {
    case 2:
        hipLaunchKernelGGL((k_tu4<P>), dim3((uint32_t)((a.n + X265AMD_BLOCK - 1) / X265AMD_BLOCK)), dim3(X265AMD_BLOCK),
                           0, st, a);
        break;
    case 3:
        if (tu_bf()) hipLaunchKernelGGL((k_tu<P, 8, true>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, a);
        else hipLaunchKernelGGL((k_tu<P, 8>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, a);
        break;
    case 4:
        if (tu_bf()) hipLaunchKernelGGL((k_tu<P, 16, true>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, a);
        else hipLaunchKernelGGL((k_tu<P, 16>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, a);
        break;
    case 5:
    {
        // one wavefront per TU, enough waves to fill the chip, each looping over TUs
        const int64_t want = ((int64_t)a.n + kTuWaves - 1) / kTuWaves;
        if (tu_i8())
            hipLaunchKernelGGL((k_tu32_i8<P>), dim3((uint32_t)(want < 4096 ? want : 4096)), dim3(X265AMD_BLOCK), 0, st, a);
        else
            hipLaunchKernelGGL((k_tu32_mfma<P>), dim3((uint32_t)(want < 4096 ? want : 4096)), dim3(X265AMD_BLOCK), 0, st, a);
        break;
    }
    default: return X265AMD_EINVAL;
    }
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------- the resident residual-coding server
// X265AMD_RDO_SERVER (round 6; rdojob.h, rdosession.cpp): one launch serves every request of a session for its
// lifetime, so a CU's residual coding costs no launches — the posting thread writes the CU's inputs,
// descriptors and RdoJob into its slot of mapped host memory and then the slot's sequence word; a workgroup
// polls the sequence words of its slots (slot g, g + G, ...), runs the CU's luma TUs (tu32_i8_waves: a wave per
// 32x32 TU), its chroma TUs (tu_groups<16>) and its 8x8 psy energies against the prediction and the
// reconstruction (psy_energy8, hadamard.h), then writes the slot's done word.  Every workgroup leaves when the
// stop word is set or its lifetime (max_ticks of the 100 MHz real-time counter) has passed — after serving what
// it finds pending in one last poll; the host relaunches before the lifetime ends (and whenever a wait finds the
// server gone), so nothing posted is left unserved and no launch outlives its bound.
// a word the host writes, read past the caches (global_load sc0 sc1) and WITHOUT acquire ordering: a
// system-scope acquire is a buffer_inv sc0 sc1, which invalidates the XCD's L2 — at every poll of every
// workgroup it slowed the motion-search kernel beside the server (0.025 -> 0.037 ms per launch).  The one
// acquire a request needs is taken once, after its sequence word was seen.
__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename P>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_rdo_server(const RdoServerArgs a)
{
    __shared__ uint32_t s_done[kRdoServerMaxOwned];
    __shared__ int s_pick;
    __shared__ uint32_t s_seq;
    __shared__ int s_leave;
    __shared__ RdoJob s_job;
    // the request's inputs and descriptors, staged from host memory in one round trip (rdojob.h slot layout)
    constexpr int kStage = (int)rdo_out_at(sizeof(P));
    __shared__ __attribute__((aligned(16))) uint8_t s_in[kStage];
    const int g = blockIdx.x, G = gridDim.x;
    const int owned = (a.nslots - g + G - 1) / G;            // <= kRdoServerMaxOwned (host-checked)
    auto slot = [&](int i) { return a.base + (size_t)(g + i * G) * a.region; };
    // where slot i's staged bytes and job are: its device-memory input slot, or the host slot itself
    auto in_slot = [&](int i) { return a.in_base ? a.in_base + (size_t)(g + i * G) * a.in_region : slot(i); };
    auto job_of = [&](int i) {
        return a.in_base ? in_slot(i) + kStage : slot(i) + a.region - kRdoJobFromEnd;
    };
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = threadIdx.x; i < owned; i += blockDim.x)
        s_done[i] = ld_sys((const uint32_t*)(slot(i) + a.region - kRdoDoneFromEnd));
    // the workgroup's doorbell (bumped by every post to one of its slots): while it is unchanged and nothing
    // was pending at the last scan, one word is read per poll instead of every slot's sequence word
    const uint32_t* bell = a.ctl + kRdoBellWord + g;
    uint32_t seen_bell = ld_sys(bell) - 1u;                  // (scan once at the start)
    bool leaving = false;
    int last = -1, budget = 0;
    for (;;)
    {
        __syncthreads();
        if (threadIdx.x < 64)
        {
            // wave 0 polls: the doorbell, then (if it moved, or work was found last time) the sequence words;
            // the first pending slot after the last one served (round robin) is served next
            const int i = threadIdx.x;
            const uint32_t b = ld_sys(bell);
            const bool scan = b != seen_bell || last >= 0;
            seen_bell = b;
            bool pend = false;
            if (scan && i < owned)
                pend = ld_sys((const uint32_t*)(job_of(i) + offsetof(RdoJob, seq))) != s_done[i];
            const uint64_t m = __ballot(pend);
            if (i == 0)
            {
                int pick = -1;
                if (m)
                {
                    const uint64_t after = last + 1 < 64 ? (m >> (last + 1)) << (last + 1) : 0;
                    pick = (int)__builtin_ctzll(after ? after : m);
                }
                s_pick = pick;
                const bool stop = ld_sys(a.ctl) != 0 || __builtin_amdgcn_s_memrealtime() - t0 > a.max_ticks;
                s_leave = stop ? 1 : 0;
            }
        }
        __syncthreads();
        const int pick = s_pick;
        if (s_leave && !leaving)
        {
            leaving = true;
            budget = owned;                                  // at most one more request per slot, then leave
        }
        if (pick < 0 || (leaving && budget-- <= 0))
        {
            if (leaving) break;                              // nothing pending in the last poll (or budget spent)
            last = -1;                                       // idle: the doorbell only, about every 2 us
            __builtin_amdgcn_s_sleep(80);
            continue;
        }
        last = pick;
        uint8_t* base = slot(pick);
        uint8_t* ibase = in_slot(pick);
        const uint8_t* jbase = job_of(pick);
        uint64_t* stamps = (uint64_t*)(base + a.region - kRdoStampsFromEnd);
        const uint64_t ts0 = a.timing ? __builtin_amdgcn_s_memrealtime() : 0;
        if (threadIdx.x == 0) s_seq = ld_sys((const uint32_t*)(jbase + offsetof(RdoJob, seq)));
        // the job and its inputs were written before the sequence word (release): read them fresh.  They are
        // in fine-grained host memory, never held by the L2 as device data is: an agent-scope acquire (the
        // CU's L1 and the L2's non-coherent lines) suffices, and leaves the device's L2 lines alone
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        {
            // the job and the slot's first kStage bytes (inputs, descriptors): every load issued before the
            // first store, one PCIe round trip
            constexpr int NJ = (int)(offsetof(RdoJob, seq) / 4), NI = kStage / 16;
            constexpr int PJ = (NJ + X265AMD_BLOCK - 1) / X265AMD_BLOCK, PI = (NI + X265AMD_BLOCK - 1) / X265AMD_BLOCK;
            // (volatile: flat_load sc0 sc1, past every cache — the host writes these bytes, through the PCIe
            // BAR when they are in device memory, and no GPU cache may hold an older copy)
            typedef unsigned v4u __attribute__((ext_vector_type(4)));
            const volatile uint32_t* srcj = (const volatile uint32_t*)jbase;
            const volatile v4u* srci = (const volatile v4u*)ibase;
            uint32_t vj[PJ];
            v4u vi[PI];
#pragma unroll
            for (int k = 0; k < PJ; k++)
            {
                const int i = threadIdx.x + k * X265AMD_BLOCK;
                vj[k] = srcj[i < NJ ? i : 0];
            }
#pragma unroll
            for (int k = 0; k < PI; k++)
            {
                const int i = threadIdx.x + k * X265AMD_BLOCK;
                vi[k] = srci[i < NI ? i : 0];
            }
#pragma unroll
            for (int k = 0; k < PJ; k++)
                if (threadIdx.x + k * X265AMD_BLOCK < NJ) ((uint32_t*)&s_job)[threadIdx.x + k * X265AMD_BLOCK] = vj[k];
#pragma unroll
            for (int k = 0; k < PI; k++)
                if (threadIdx.x + k * X265AMD_BLOCK < NI) ((v4u*)s_in)[threadIdx.x + k * X265AMD_BLOCK] = vi[k];
        }
        __syncthreads();
        const bool sao = s_job.kind == 1;
        if (threadIdx.x == 0 && !sao)
        {
            // every pointer of the job into the staged bytes now points into LDS (outputs stay in host memory)
            const uintptr_t lo = (uintptr_t)ibase, hi = lo + kStage;
            uint8_t* lds = (uint8_t*)s_in;
            auto rel = [&](auto& ptr) {
                const uintptr_t v = (uintptr_t)ptr;
                if (v >= lo && v < hi) ptr = (std::remove_reference_t<decltype(ptr)>)(void*)(lds + (v - lo));
            };
            for (int c = 0; c < 2; c++)
            {
                x265amd_tu_batch& b = s_job.tu[c];
                rel(b.fenc); rel(b.fenc_off); rel(b.pred); rel(b.pred_off); rel(b.resi_off); rel(b.coeff_off);
                rel(b.recon_off); rel(b.qp);
            }
            for (int c = 0; c < 4; c++)
            {
                // (batches 1 and 3 compare against the reconstruction, an output: their b stays in host memory —
                // every batch's b is the slot base, told apart only by its offsets)
                x265amd_cmp_batch& b = s_job.psy[c];
                rel(b.a); rel(b.a_off); rel(b.b_off);
                if (!(c & 1)) rel(b.b);
            }
        }
        __syncthreads();
        // (a request is one 64x64 or 32x32 CU: 4 / 1 luma TUs, 8 / 2 chroma TUs, at most 64 8x8 blocks a
        // batch; anything else is not served, only marked done)
        const bool sane = !sao && s_job.tu[0].log2_size == 5 && s_job.tu[1].log2_size == 4 && s_job.tu[0].n >= 0 &&
                          s_job.tu[0].n <= 4 && s_job.tu[1].n >= 0 && s_job.tu[1].n <= 8 &&
                          s_job.psy[0].n >= 0 && s_job.psy[0].n <= 64 && s_job.psy[1].n >= 0 && s_job.psy[1].n <= 64 &&
                          s_job.psy[2].n >= 0 && s_job.psy[2].n <= 32 && s_job.psy[3].n >= 0 && s_job.psy[3].n <= 32;
        const uint64_t ts1 = a.timing ? __builtin_amdgcn_s_memrealtime() : 0;
        uint64_t ts2 = 0, ts3 = 0;
        if (sane)
        {
            tu32_i8_waves<P>(tu_args(s_job.tu[0], a.depth), 0, 1);
            if (a.timing) { __syncthreads(); ts2 = __builtin_amdgcn_s_memrealtime(); }
            tu_groups<P, 16, false>(tu_args(s_job.tu[1], a.depth), 0);
            if (a.timing) { __syncthreads(); ts3 = __builtin_amdgcn_s_memrealtime(); }
        }
        // a CTU's SAO statistics (8-bit 4:2:0, 64x64: the windows fit the staged bytes): the four waves, from LDS
        const RdoSaoJob& q = s_job.sao;
        if (sao && sizeof(P) == 1 && q.ctu_log2 == 6 && q.hs == 1 && q.vs == 1)
        {
            bool inside = true;
            for (int p = 0; p < 3; p++)
                inside = inside && q.rec_at[p] > 0 && q.rec_at[p] < kStage && q.fenc_at[p] >= 0 && q.fenc_at[p] < kStage;
            if (inside)
            {
                SaoCtuView v;
                v.nd = q.nd;
                for (int pc = 0; pc < 2; pc++)
                {
                    v.pw[pc] = pc ? q.w >> q.hs : q.w;
                    v.ph[pc] = pc ? q.h >> q.vs : q.h;
                    v.csw[pc] = (1 << q.ctu_log2) >> (pc ? q.hs : 0);
                    v.csh[pc] = (1 << q.ctu_log2) >> (pc ? q.vs : 0);
                    v.x0[pc] = q.cx * v.csw[pc];
                    v.y0[pc] = q.cy * v.csh[pc];
                }
                for (int p = 0; p < 3; p++)
                {
                    v.rec[p] = s_in + q.rec_at[p];
                    v.fenc[p] = s_in + q.fenc_at[p];
                    v.rs[p] = q.rs[p];
                    v.fs[p] = q.fs[p];
                }
                sao_stats_wave<P, true, X265AMD_BLOCK / 64>(v, a.depth - 5, q.stats, q.count);
            }
        }
        // the reconstruction the waves wrote (to host memory) is read back by others for its psy energies:
        // their stores complete (workgroup release: s_waitcnt), then the readers' L1 is invalidated
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        {
            const int n0 = s_job.psy[0].n, n1 = s_job.psy[1].n, n2 = s_job.psy[2].n, n3 = s_job.psy[3].n;
            const int64_t sse_at = s_job.pad[0] <= 96 ? 2 * (int64_t)s_job.pad[0] : 0;
            const int total = sane ? n0 + n1 + n2 + n3 : 0;
            for (int q = threadIdx.x; q < total; q += blockDim.x)
            {
                int b = 0, j = q;
                if (j >= n0) { j -= n0; b = 1; if (j >= n1) { j -= n1; b = 2; if (j >= n2) { j -= n2; b = 3; } } }
                const x265amd_cmp_batch& c = s_job.psy[b];
                const P* pa = (const P*)c.a + c.a_off[j];
                const P* pb = (const P*)c.b + c.b_off[j];
                const int e = psy_energy8<P>(pa, c.a_stride) - psy_energy8<P>(pb, c.b_stride);
                ((int32_t*)c.out)[j] = e < 0 ? -e : e;
                if (sse_at)
                {
                    // sse_pp 8x8 of the same pair (pixel.cpp sse<8, 8>), for the CU's distortions
                    int v = 0;
                    for (int y = 0; y < 8; y++)
                        for (int x = 0; x < 8; x++)
                        {
                            const int d = (int)pa[y * c.a_stride + x] - (int)pb[y * c.b_stride + x];
                            v += d * d;
                        }
                    ((int32_t*)c.out)[j + sse_at] = v;
                }
            }
        }
        // every output of the request is visible to the host before its done word
        if (a.timing) __syncthreads();
        const uint64_t ts4 = a.timing ? __builtin_amdgcn_s_memrealtime() : 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __syncthreads();
        if (threadIdx.x == 0 && a.timing)
        {
            const uint64_t ts5 = __builtin_amdgcn_s_memrealtime();
            stamps[0] = ts0; stamps[1] = ts1; stamps[2] = ts2; stamps[3] = ts3; stamps[4] = ts4; stamps[5] = ts5;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        }
        if (threadIdx.x == 0)
        {
            // (ordered after the outputs by the system-scope release fence above: one L2 write-back a request)
            __hip_atomic_store((uint32_t*)(base + a.region - kRdoDoneFromEnd), s_seq, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            s_done[pick] = s_seq;
        }
    }
}

} // namespace x265amd

extern "C" int x265amd_rdo_server_launch(const x265amd::RdoServerArgs* a, int nwg, int cooperative, void* stream)
{
    using namespace x265amd;
    if (!a || !a->base || !a->ctl || nwg < 1 || a->nslots < 1 || a->nslots > nwg * kRdoServerMaxOwned ||
        a->region < kRdoJobFromEnd || (a->depth != 8 && a->depth != 10 && a->depth != 12))
        return X265AMD_EINVAL;
    // a cooperative launch: every workgroup is resident at once (a workgroup waiting for a free CU would leave
    // its slots unserved), in the runtime's own queue for cooperative work, apart from the streams' queues
    RdoServerArgs args = *a;
    void* params[] = { &args };
    const void* f = a->depth == 8 ? (const void*)k_rdo_server<uint8_t> : (const void*)k_rdo_server<uint16_t>;
    if (cooperative)
        return (int)hipLaunchCooperativeKernel(f, dim3(nwg), dim3(X265AMD_BLOCK), params, 0, (hipStream_t)stream);
    return (int)hipLaunchKernel(f, dim3(nwg), dim3(X265AMD_BLOCK), params, 0, (hipStream_t)stream);
}

using namespace x265amd;

extern "C" int x265amd_tu_pipeline(int depth, int count, const x265amd_tu_batch* bt, void* stream)
{
    if (depth != 8 && depth != 10 && depth != 12) return X265AMD_EINVAL;
    if (count < 0 || (count && !bt)) return X265AMD_EINVAL;
    // validate every batch before enqueuing anything
    for (int i = 0; i < count; i++)
    {
        const x265amd_tu_batch& b = bt[i];
        if (b.n < 0 || b.log2_size < 2 || b.log2_size > 5) return X265AMD_EINVAL;
        if (b.n && (!b.fenc || !b.fenc_off || !b.pred || !b.pred_off || !b.coeff || !b.coeff_off || !b.recon ||
                    !b.recon_off || !b.num_sig || !b.qp || (b.resi && !b.resi_off)))
            return X265AMD_EINVAL;
    }
    hipStream_t st = (hipStream_t)stream;
    for (int i = 0; i < count; i++)
    {
        const x265amd_tu_batch& b = bt[i];
        if (!b.n) continue;
        const TuArgs a = tu_args(b, depth);
        const int rc = depth == 8 ? launch_tu<uint8_t>(b.log2_size, a, st) : launch_tu<uint16_t>(b.log2_size, a, st);
        if (rc) return rc;
    }
    return 0;
}
