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
#include "common.h"
#include "transform1d.h"
#include "../../../include/x265_amd.h"

namespace x265amd {

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
__device__ __forceinline__ int quant_scale(int rem)
{
    return rem == 0 ? 26214 : rem == 1 ? 23302 : rem == 2 ? 20560 : rem == 3 ? 18396 : rem == 4 ? 16384 : 14564;
}
__device__ __forceinline__ int inv_quant_scale(int rem)
{
    return rem == 0 ? 40 : rem == 1 ? 45 : rem == 2 ? 51 : rem == 3 ? 57 : rem == 4 ? 64 : 72;
}

// LDS exchange among the lanes of one wavefront: orders this lane's LDS
// writes before the other lanes' later reads (LDS executes a wavefront's
// instructions in order; the fences keep the compiler from moving accesses
// across).  No s_barrier: groups never span wavefronts.
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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

template <typename P, int N>
__global__ __launch_bounds__(X265AMD_BLOCK) void k_tu(const TuArgs a)
{
    constexpr int LOG2 = N == 4 ? 2 : N == 8 ? 3 : N == 16 ? 4 : 5;
    constexpr int PT = N + 2;                 // transposition tile pitch (int16), spreads LDS banks
    constexpr int JOBS = X265AMD_BLOCK / N;
    constexpr int NCG = N * N / 16;
    __shared__ int16_t lds_t[JOBS][N * PT];   // stage tiles; DCT coefficients (pitch N) during quant/SBH
    __shared__ int16_t lds_q[JOBS][N * N];    // quantized coefficients (raster, as coeff[])
    const int slot = threadIdx.x / N, r = threadIdx.x % N;
    const int64_t j = (int64_t)xcd_block() * JOBS + slot;
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
    {
        int f[N], p[N];
        load_n<P, N>(pf, f);
        load_n<P, N>(pp, p);
#pragma unroll
        for (int i = 0; i < N; i++) x[i] = f[i] - p[i];
    }

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
    if (a.sign_hide && num_sig >= 2)
    {
        wave_sync();
        const int st = a.scan ? a.scan[j] : 0;
        const uint16_t* scan = N == 4 ? c_scan.s4[st] : N == 8 ? c_scan.s8[st] : N == 16 ? c_scan.s16 : c_scan.s32;
        int last = -1;
        for (int cg = r; cg < NCG; cg += N)
            for (int n = 15; n >= 0; n--)
                if (Q[scan[cg * 16 + n]]) { last = last > cg * 16 + n ? last : cg * 16 + n; break; }
        last = group_max<N>(last);
        const int cg_last = last >> 4;
        const int qbits8 = qbits - 8;
        int dsig = 0;
        for (int cg = r; cg <= cg_last; cg += N)
        {
            const int base = cg << 4, top = cg == cg_last ? (last & 15) : 15;
            int qv[16], pos[16];
            uint32_t mask = 0;
#pragma unroll
            for (int n = 0; n < 16; n++)
            {
                pos[n] = scan[base + n];
                qv[n] = n <= top ? Q[pos[n]] : 0;
                mask |= (uint32_t)(qv[n] != 0) << n;
            }
            if (!mask) continue;
            const int first = __builtin_ctz(mask), lastnz = 31 - __builtin_clz(mask);
            if (lastnz - first < 4) continue;               // SBH_THRESHOLD (common.h:273)
            int sum = 0, fq = 0;
#pragma unroll
            for (int n = 0; n < 16; n++)
            {
                sum += qv[n];                               // zeros outside [first, lastnz]
                fq = n == first ? qv[n] : fq;
            }
            const int signbit = fq > 0 ? 0 : 1;
            if (signbit == (sum & 1)) continue;
            int min_cost = 0x7fffffff, min_n = 0, change = 0;
#pragma unroll
            for (int n = 15; n >= 0; n--)
            {
                if (n > top) continue;
                const int c = T[pos[n]];
                const int tmp = (c < 0 ? -c : c) * qscale;
                const int lvl = (tmp + qadd) >> qbits;
                const int du = (tmp - (lvl << qbits)) >> qbits8;   // deltaU (quant_c)
                const bool below = (mask & ((1u << n) - 1)) != 0;
                int cost, ch = 1;
                if (qv[n])
                {
                    if (du > 0) cost = -du;
                    else if (!below && (qv[n] == 1 || qv[n] == -1)) cost = 0x7fffffff;
                    else { cost = du; ch = -1; }
                }
                else if (!below)
                    cost = ((c >= 0 ? 0 : 1) != signbit) ? 0x7fffffff : -du;
                else
                    cost = -du;
                if (cost < min_cost) { min_cost = cost; change = ch; min_n = n; }
            }
            int qm = 0, p = 0, cm = 0;
#pragma unroll
            for (int n = 0; n < 16; n++)
                if (n == min_n) { qm = qv[n]; p = pos[n]; }
            cm = T[p];
            if (qm == 32767 || qm == -32768) change = -1;
            if (!qm) dsig++;
            else if (change == -1 && (qm == 1 || qm == -1)) dsig--;
            const int sm = cm < 0 ? -1 : 0;
            Q[p] = (int16_t)(qm + ((change ^ sm) - sm));
        }
        num_sig += group_sum<N>(dsig);
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
    load_n<P, N>(pf, f);                      // second touch of the TU rows: served by L2
    load_n<P, N>(pp, p);
    if (num_sig == 0)
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

template <typename P>
static int launch_tu(int log2, const TuArgs& a, hipStream_t st)
{
    const int N = 1 << log2;
    const uint32_t blocks = (uint32_t)((a.n + X265AMD_BLOCK / N - 1) / (X265AMD_BLOCK / N));
    switch (log2)
    {
    case 2: hipLaunchKernelGGL((k_tu<P, 4>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, a); break;
    case 3: hipLaunchKernelGGL((k_tu<P, 8>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, a); break;
    case 4: hipLaunchKernelGGL((k_tu<P, 16>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, a); break;
    case 5: hipLaunchKernelGGL((k_tu<P, 32>), dim3(blocks), dim3(X265AMD_BLOCK), 0, st, a); break;
    default: return X265AMD_EINVAL;
    }
    return (int)hipGetLastError();
}

} // namespace x265amd

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
        TuArgs a{ b.fenc, b.fenc_off, (int64_t)b.fenc_stride, b.pred, b.pred_off, (int64_t)b.pred_stride,
                  b.resi, b.resi_off, (int64_t)b.resi_stride, b.coeff, b.coeff_off, b.recon, b.recon_off,
                  (int64_t)b.recon_stride, b.num_sig, b.qp, b.scan, b.n, !!b.is_luma, !!b.is_intra, !!b.i_slice,
                  !!b.sign_hide, depth };
        const int rc = depth == 8 ? launch_tu<uint8_t>(b.log2_size, a, st) : launch_tu<uint16_t>(b.log2_size, a, st);
        if (rc) return rc;
    }
    return 0;
}
