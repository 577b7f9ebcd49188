/* x265_oracle.c — from-scratch CPU restatement of the x265 1.9 primitive table.
 *
 * TEST INFRASTRUCTURE ONLY (see x265_oracle.h): the checker and the CPU
 * baseline, never part of the product.  Parity of this file with the
 * reference is pinned two ways: the committed golden vectors
 * in tests/golden/ (generated from the reference's own C primitives built by
 * oracle/Makefile `ref`) and randomized cross-checks against that library.
 *
 * Compiled once per bit depth: -DXO_DEPTH=8 (pixel = uint8_t, sse_t = uint32)
 * or -DXO_DEPTH=10 (pixel = uint16_t, sse_t = uint64), like the reference's
 * HIGH_BIT_DEPTH builds (common.h:124-142).
 *
 * Each function cites the reference lines it restates; all paths are
 * integer and follow the reference's truncation / clipping points exactly
 * (SURVEY.md Appendix A).
 */
#include "x265_oracle.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* the reference's int arithmetic, defined for every input: two's-complement wrap
   of the product, and << of a negative value as the arithmetic shift g++ emits */
static inline int32_t mul_wrap(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
static inline int32_t shl_wrap(int32_t a, int s) { return (int32_t)((uint32_t)a << s); }

#ifndef XO_DEPTH
#define XO_DEPTH 8
#endif

#if XO_DEPTH > 8
typedef uint16_t pix;
typedef uint64_t sse_type;
#else
typedef uint8_t pix;
typedef uint32_t sse_type;
#endif

#define PMAX ((1 << XO_DEPTH) - 1)
#define FSTRIDE 64                 /* FENC_STRIDE, common.h:70 */
#define IF_PREC 6                  /* IF_FILTER_PREC, constants.h:70-74 */
#define IF_IPREC 14                /* IF_INTERNAL_PREC */
#define IF_OFFS 8192               /* IF_INTERNAL_OFFS */

static int clipp(int v) { return v < 0 ? 0 : (v > PMAX ? PMAX : v); }
static int clip16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }
static int ilog2(int n) { int l = 0; while ((1 << l) < n) l++; return l; }

int xo_depth(void) { return XO_DEPTH; }

/* ======================================================= pixel comparisons */

/* pixel.cpp:39-54 */
int xo_sad(int w, int h, const void* a_, intptr_t sa, const void* b_, intptr_t sb)
{
    const pix* a = (const pix*)a_;
    const pix* b = (const pix*)b_;
    int s = 0;
    for (int y = 0; y < h; y++, a += sa, b += sb)
        for (int x = 0; x < w; x++) s += abs((int)a[x] - (int)b[x]);
    return s;
}

/* pixel.cpp:73-118: fenc uses FENC_STRIDE */
void xo_sad_x3(int w, int h, const void* f, const void* r0, const void* r1, const void* r2, intptr_t rs, int32_t* res)
{
    res[0] = xo_sad(w, h, f, FSTRIDE, r0, rs);
    res[1] = xo_sad(w, h, f, FSTRIDE, r1, rs);
    res[2] = xo_sad(w, h, f, FSTRIDE, r2, rs);
}

void xo_sad_x4(int w, int h, const void* f, const void* r0, const void* r1, const void* r2, const void* r3,
               intptr_t rs, int32_t* res)
{
    xo_sad_x3(w, h, f, r0, r1, r2, rs, res);
    res[3] = xo_sad(w, h, f, FSTRIDE, r3, rs);
}

/* 4-point Hadamard butterfly (pixel.cpp:143-152) on ints */
static void had4(int* v0, int* v1, int* v2, int* v3)
{
    int t0 = *v0 + *v1, t1 = *v0 - *v1, t2 = *v2 + *v3, t3 = *v2 - *v3;
    *v0 = t0 + t2; *v2 = t0 - t2; *v1 = t1 + t3; *v3 = t1 - t3;
}

/* unrounded 4x4 Hadamard |coef| sum: satd_4x4 returns this >> 1 (pixel.cpp:163-189) */
static int satd4_raw(const pix* a, intptr_t sa, const pix* b, intptr_t sb)
{
    int m[4][4];
    for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++) m[y][x] = (int)a[y * sa + x] - (int)b[y * sb + x];
    for (int y = 0; y < 4; y++) had4(&m[y][0], &m[y][1], &m[y][2], &m[y][3]);
    int s = 0;
    for (int x = 0; x < 4; x++)
    {
        had4(&m[0][x], &m[1][x], &m[2][x], &m[3][x]);
        s += abs(m[0][x]) + abs(m[1][x]) + abs(m[2][x]) + abs(m[3][x]);
    }
    return s;
}

/* satd over 4x4 tiles; the tiling (satd4 vs satd8, pixel.cpp:216-242) does not
 * change the value because each tile's raw sum is even (SURVEY.md note a7) */
int xo_satd(int w, int h, const void* a_, intptr_t sa, const void* b_, intptr_t sb)
{
    const pix* a = (const pix*)a_;
    const pix* b = (const pix*)b_;
    int s = 0;
    for (int y = 0; y < h; y += 4)
        for (int x = 0; x < w; x += 4) s += satd4_raw(a + y * sa + x, sa, b + y * sb + x, sb) >> 1;
    return s;
}

/* unrounded 8x8 Hadamard |coef| sum (_sa8d_8x8, pixel.cpp:244-279) */
static int sa8d8_raw(const pix* a, intptr_t sa, const pix* b, intptr_t sb)
{
    int m[8][8];
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) m[y][x] = (int)a[y * sa + x] - (int)b[y * sb + x];
    for (int pass = 0; pass < 2; pass++)
    {
        /* rows on pass 0, columns on pass 1: butterflies of span 1, 2, 4 */
        for (int line = 0; line < 8; line++)
            for (int span = 1; span < 8; span <<= 1)
                for (int i = 0; i < 8; i++)
                {
                    if (i & span) continue;
                    int* p = pass ? &m[i][line] : &m[line][i];
                    int* q = pass ? &m[i + span][line] : &m[line][i + span];
                    int u = *p, v = *q;
                    *p = u + v;
                    *q = u - v;
                }
    }
    int s = 0;
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) s += abs(m[y][x]);
    return s;
}

/* cu[].sa8d as the table holds it (pixel.cpp:281-322, primitives.cpp:106,164-171) */
int xo_sa8d(int w, int h, const void* a_, intptr_t sa, const void* b_, intptr_t sb)
{
    const pix* a = (const pix*)a_;
    const pix* b = (const pix*)b_;
    if ((w & 7) || (h & 7)) return xo_satd(w, h, a_, sa, b_, sb);
    int s = 0;
    if (!(w & 15) && !(h & 15))
    {
        for (int y = 0; y < h; y += 16)
            for (int x = 0; x < w; x += 16)
            {
                int r = 0;
                for (int k = 0; k < 4; k++)
                {
                    int oy = y + 8 * (k >> 1), ox = x + 8 * (k & 1);
                    r += sa8d8_raw(a + oy * sa + ox, sa, b + oy * sb + ox, sb);
                }
                s += (r + 2) >> 2;
            }
    }
    else
    {
        for (int y = 0; y < h; y += 8)
            for (int x = 0; x < w; x += 8) s += (sa8d8_raw(a + y * sa + x, sa, b + y * sb + x, sb) + 2) >> 2;
    }
    return s;
}

/* pixel.cpp:120-139: sum in sse_t, each term an int product */
uint64_t xo_sse_pp(int w, int h, const void* a_, intptr_t sa, const void* b_, intptr_t sb)
{
    const pix* a = (const pix*)a_;
    const pix* b = (const pix*)b_;
    sse_type s = 0;
    for (int y = 0; y < h; y++, a += sa, b += sb)
        for (int x = 0; x < w; x++)
        {
            int d = (int)a[x] - (int)b[x];
            s += (sse_type)(uint32_t)(d * d);
        }
    return (uint64_t)s;
}

uint64_t xo_sse_ss(int w, int h, const int16_t* a, intptr_t sa, const int16_t* b, intptr_t sb)
{
    sse_type s = 0;
    for (int y = 0; y < h; y++, a += sa, b += sb)
        for (int x = 0; x < w; x++)
        {
            int d = a[x] - b[x];
            s += (sse_type)(uint32_t)(d * d);
        }
    return (uint64_t)s;
}

/* pixel.cpp:324-336 */
uint64_t xo_ssd_s(int n, const int16_t* a, intptr_t sa)
{
    sse_type s = 0;
    for (int y = 0; y < n; y++, a += sa)
        for (int x = 0; x < n; x++) s += (sse_type)(uint32_t)(a[x] * a[x]);
    return (uint64_t)s;
}

/* AC energy of one block against a zero block (pixel.cpp:672-703) */
static int psy_energy(int n, const pix* p, intptr_t s)
{
    static const pix zero[8] = { 0 };
    if (n == 4)
        return (satd4_raw(p, s, zero, 0) >> 1) - (xo_sad(4, 4, p, s, zero, 0) >> 2);
    return ((sa8d8_raw(p, s, zero, 0) + 2) >> 2) - (xo_sad(8, 8, p, s, zero, 0) >> 2);
}

int xo_psy_cost_pp(int n, const void* src_, intptr_t ss, const void* rec_, intptr_t rs)
{
    const pix* src = (const pix*)src_;
    const pix* rec = (const pix*)rec_;
    if (n == 4) return abs(psy_energy(4, src, ss) - psy_energy(4, rec, rs));
    uint32_t tot = 0;
    for (int y = 0; y < n; y += 8)
        for (int x = 0; x < n; x += 8)
            tot += (uint32_t)abs(psy_energy(8, src + y * ss + x, ss) - psy_energy(8, rec + y * rs + x, rs));
    return (int)tot;
}

/* pixel.cpp:649-666 */
uint64_t xo_var(int n, const void* p_, intptr_t s)
{
    const pix* p = (const pix*)p_;
    uint32_t sum = 0, sqr = 0;
    for (int y = 0; y < n; y++, p += s)
        for (int x = 0; x < n; x++) { sum += p[x]; sqr += (uint32_t)p[x] * p[x]; }
    return sum + ((uint64_t)sqr << 32);
}

/* ======================================================= interpolation */

static const int16_t kLuma[4][8] = { { 0, 0, 0, 64, 0, 0, 0, 0 }, { -1, 4, -10, 58, 17, -5, 1, 0 },
                                     { -1, 4, -11, 40, 40, -11, 4, -1 }, { 0, 1, -5, 17, 58, -10, 4, -1 } };
static const int16_t kChroma[8][4] = { { 0, 64, 0, 0 }, { -2, 58, 10, -2 }, { -4, 54, 16, -2 }, { -6, 46, 28, -4 },
                                       { -4, 36, 36, -4 }, { -4, 28, 46, -6 }, { -2, 16, 54, -4 }, { -2, 10, 58, -2 } };

static const int16_t* taps_of(int taps, int idx) { return taps == 8 ? kLuma[idx] : kChroma[idx]; }

/* ipfilter.cpp:120-163 horizontal pixel -> int16, optional row extension */
static void h_ps(int taps, int w, int h, const pix* src, intptr_t ss, int16_t* dst, intptr_t ds, int ci, int rowext)
{
    const int16_t* c = taps_of(taps, ci);
    const int head = IF_IPREC - XO_DEPTH, shift = IF_PREC - head, off = -IF_OFFS * (1 << shift);
    int rows = h;
    src -= taps / 2 - 1;
    if (rowext) { src -= (taps / 2 - 1) * ss; rows += taps - 1; }
    for (int y = 0; y < rows; y++, src += ss, dst += ds)
        for (int x = 0; x < w; x++)
        {
            int s = 0;
            for (int k = 0; k < taps; k++) s += src[x + k] * c[k];
            dst[x] = (int16_t)((s + off) >> shift);
        }
}

/* ipfilter.cpp:244-285 (and filterVertical_sp_c :322-363) int16 -> pixel */
static void v_sp(int taps, int w, int h, const int16_t* src, intptr_t ss, pix* dst, intptr_t ds, int ci)
{
    const int16_t* c = taps_of(taps, ci);
    const int head = IF_IPREC - XO_DEPTH, shift = IF_PREC + head;
    const int off = (1 << (shift - 1)) + (IF_OFFS << IF_PREC);
    src -= (taps / 2 - 1) * ss;
    for (int y = 0; y < h; y++, src += ss, dst += ds)
        for (int x = 0; x < w; x++)
        {
            int s = 0;
            for (int k = 0; k < taps; k++) s += src[x + k * ss] * c[k];
            dst[x] = (pix)clipp((int16_t)((s + off) >> shift));
        }
}

void xo_interp(int op, int taps, int w, int h, const void* src_, intptr_t ss, void* dst_, intptr_t ds, int ci, int extra)
{
    const pix* sp = (const pix*)src_;
    const int16_t* s16 = (const int16_t*)src_;
    pix* dp = (pix*)dst_;
    int16_t* d16 = (int16_t*)dst_;
    const int head = IF_IPREC - XO_DEPTH;
    const int16_t* c = taps_of(taps, ci & (taps == 8 ? 3 : 7));

    switch (op)
    {
    case XO_HPP: /* ipfilter.cpp:79-118 */
        sp -= taps / 2 - 1;
        for (int y = 0; y < h; y++, sp += ss, dp += ds)
            for (int x = 0; x < w; x++)
            {
                int s = 0;
                for (int k = 0; k < taps; k++) s += sp[x + k] * c[k];
                dp[x] = (pix)clipp((int16_t)((s + 32) >> IF_PREC));
            }
        return;
    case XO_HPS:
        h_ps(taps, w, h, sp, ss, d16, ds, ci, extra);
        return;
    case XO_VPP: /* ipfilter.cpp:165-204 */
        sp -= (taps / 2 - 1) * ss;
        for (int y = 0; y < h; y++, sp += ss, dp += ds)
            for (int x = 0; x < w; x++)
            {
                int s = 0;
                for (int k = 0; k < taps; k++) s += sp[x + k * ss] * c[k];
                dp[x] = (pix)clipp((int16_t)((s + 32) >> IF_PREC));
            }
        return;
    case XO_VPS: /* ipfilter.cpp:206-242 */
    {
        const int shift = IF_PREC - head, off = -IF_OFFS * (1 << shift);
        sp -= (taps / 2 - 1) * ss;
        for (int y = 0; y < h; y++, sp += ss, d16 += ds)
            for (int x = 0; x < w; x++)
            {
                int s = 0;
                for (int k = 0; k < taps; k++) s += sp[x + k * ss] * c[k];
                d16[x] = (int16_t)((s + off) >> shift);
            }
        return;
    }
    case XO_VSP:
        v_sp(taps, w, h, s16, ss, dp, ds, ci);
        return;
    case XO_VSS: /* ipfilter.cpp:287-320 */
        s16 -= (taps / 2 - 1) * ss;
        for (int y = 0; y < h; y++, s16 += ss, d16 += ds)
            for (int x = 0; x < w; x++)
            {
                int s = 0;
                for (int k = 0; k < taps; k++) s += s16[x + k * ss] * c[k];
                d16[x] = (int16_t)(s >> IF_PREC);
            }
        return;
    case XO_HVPP: /* ipfilter.cpp:365-372: hps with row extension, then vertical sp */
    {
        int16_t* im = (int16_t*)malloc(sizeof(int16_t) * w * (h + taps - 1));
        h_ps(taps, w, h, sp, ss, im, w, ci, 1);
        v_sp(taps, w, h, im + (taps / 2 - 1) * w, w, dp, ds, extra);
        free(im);
        return;
    }
    case XO_P2S: /* ipfilter.cpp:40-57 */
        for (int y = 0; y < h; y++, sp += ss, d16 += ds)
            for (int x = 0; x < w; x++)
            {
                int16_t v = (int16_t)shl_wrap(sp[x], head);
                d16[x] = (int16_t)(v - (int16_t)IF_OFFS);
            }
        return;
    }
}

/* ======================================================= transforms */

/* HEVC matrix generated from the spec rule (see csrc/tables.h) */
static int tmat(int N, int k, int n)
{
    static const int mag[33] = { 64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67,
                                 64, 61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9, 4, 0 };
    int a = ((k * (32 / N)) * (2 * n + 1)) & 127;
    return a <= 32 ? mag[a] : a <= 64 ? -mag[64 - a] : a <= 96 ? -mag[a - 64] : mag[128 - a];
}

/* one forward stage (partialButterflyN, dct.cpp:83-240,418-440) as an exact
 * matrix product: out[k*N + j] = round(sum_n T[k][n] * in[j*N + n]) */
static void fwd_stage(int N, const int16_t* in, int16_t* out, int shift)
{
    for (int j = 0; j < N; j++)
        for (int k = 0; k < N; k++)
        {
            int s = 0;
            for (int n = 0; n < N; n++) s += tmat(N, k, n) * in[j * N + n];
            out[k * N + j] = (int16_t)((s + (1 << (shift - 1))) >> shift);
        }
}

/* one inverse stage (partialButterflyInverseN, dct.cpp:242-416):
 * out[j*N + k] = clip(round(sum_m T[m][k] * in[m*N + j])) */
static void inv_stage(int N, const int16_t* in, int16_t* out, int shift)
{
    for (int j = 0; j < N; j++)
        for (int k = 0; k < N; k++)
        {
            int s = 0;
            for (int m = 0; m < N; m++) s += tmat(N, m, k) * in[m * N + j];
            out[j * N + k] = (int16_t)clip16((s + (1 << (shift - 1))) >> shift);
        }
}

/* DST-VII forward / inverse stages (fastForwardDst / inversedst, dct.cpp:41-81) */
static void dst_fwd_stage(const int16_t* b, int16_t* o, int shift)
{
    const int rnd = 1 << (shift - 1);
    for (int i = 0; i < 4; i++)
    {
        const int16_t* r = b + 4 * i;
        int c0 = r[0] + r[3], c1 = r[1] + r[3], c2 = r[0] - r[1], c3 = 74 * r[2];
        o[i] = (int16_t)((29 * c0 + 55 * c1 + c3 + rnd) >> shift);
        o[4 + i] = (int16_t)((74 * (r[0] + r[1] - r[3]) + rnd) >> shift);
        o[8 + i] = (int16_t)((29 * c2 + 55 * c0 - c3 + rnd) >> shift);
        o[12 + i] = (int16_t)((55 * c2 - 29 * c1 + c3 + rnd) >> shift);
    }
}

static void dst_inv_stage(const int16_t* t, int16_t* o, int shift)
{
    const int rnd = 1 << (shift - 1);
    for (int i = 0; i < 4; i++)
    {
        int c0 = t[i] + t[8 + i], c1 = t[8 + i] + t[12 + i], c2 = t[i] - t[12 + i], c3 = 74 * t[4 + i];
        o[4 * i + 0] = (int16_t)clip16((29 * c0 + 55 * c1 + c3 + rnd) >> shift);
        o[4 * i + 1] = (int16_t)clip16((55 * c2 - 29 * c1 + c3 + rnd) >> shift);
        o[4 * i + 2] = (int16_t)clip16((74 * (t[i] - t[8 + i] + t[12 + i]) + rnd) >> shift);
        o[4 * i + 3] = (int16_t)clip16((55 * c0 + 29 * c2 - c3 + rnd) >> shift);
    }
}

/* dct.cpp:442-610 */
void xo_dct(int kind, int n, const int16_t* src, int16_t* dst, intptr_t stride)
{
    int16_t a[32 * 32], b[32 * 32];
    const int lg = ilog2(n);
    if (kind == XO_DCT || kind == XO_DST)
    {
        for (int y = 0; y < n; y++) memcpy(a + y * n, src + y * stride, n * sizeof(int16_t));
        const int s1 = lg - 1 + (XO_DEPTH - 8), s2 = lg + 6;
        if (kind == XO_DST) { dst_fwd_stage(a, b, s1); dst_fwd_stage(b, dst, s2); }
        else { fwd_stage(n, a, b, s1); fwd_stage(n, b, dst, s2); }
    }
    else
    {
        const int s1 = 7, s2 = 12 - (XO_DEPTH - 8);
        if (kind == XO_IDST) { dst_inv_stage(src, a, s1); dst_inv_stage(a, b, s2); }
        else { inv_stage(n, src, a, s1); inv_stage(n, a, b, s2); }
        for (int y = 0; y < n; y++) memcpy(dst + y * stride, b + y * n, n * sizeof(int16_t));
    }
}

/* dct.cpp:664-686 (int32 products wrap like the reference's int arithmetic) */
uint32_t xo_quant(const int16_t* coef, const int32_t* qc, int32_t* deltaU, int16_t* qout, int qBits, int add, int num)
{
    uint32_t sig = 0;
    for (int i = 0; i < num; i++)
    {
        int lv = coef[i];
        uint32_t tmp = (uint32_t)abs(lv) * (uint32_t)qc[i];
        int level = (int)(tmp + (uint32_t)add) >> qBits;
        deltaU[i] = (int)(tmp - ((uint32_t)level << qBits)) >> (qBits - 8);
        sig += level != 0;
        if (lv < 0) level = -level;
        qout[i] = (int16_t)clip16(level);
    }
    return sig;
}

/* dct.cpp:688-713 */
uint32_t xo_nquant(const int16_t* coef, const int32_t* qc, int16_t* qout, int qBits, int add, int num)
{
    uint32_t sig = 0;
    for (int i = 0; i < num; i++)
    {
        int lv = coef[i];
        uint32_t tmp = (uint32_t)abs(lv) * (uint32_t)qc[i];
        int level = (int)(tmp + (uint32_t)add) >> qBits;
        sig += level != 0;
        if (lv < 0) level = -level;
        qout[i] = (int16_t)abs(clip16(level));
    }
    return sig;
}

/* dct.cpp:612-634 */
void xo_dequant_normal(const int16_t* q, int16_t* coef, int num, int scale, int shift)
{
    const int add = 1 << (shift - 1);
    for (int i = 0; i < num; i++) coef[i] = (int16_t)clip16((q[i] * scale + add) >> shift);
}


/* dct.cpp:636-662 */
void xo_dequant_scaling(const int16_t* q, const int32_t* dq, int16_t* coef, int num, int per, int shift)
{
    shift += 4;
    if (shift > per)
    {
        const int add = 1 << (shift - per - 1);
        for (int i = 0; i < num; i++) coef[i] = (int16_t)clip16((int32_t)((uint32_t)mul_wrap(q[i], dq[i]) + (uint32_t)add) >> (shift - per));
    }
    else
        for (int i = 0; i < num; i++) coef[i] = (int16_t)clip16(shl_wrap(clip16(mul_wrap(q[i], dq[i])), per - shift));
}

/* ======================================================= intra */

/* intrapred.cpp:31-51 */
void xo_intra_filter(int n, const void* ref_, void* filt_)
{
    const pix* s = (const pix*)ref_;
    pix* f = (pix*)filt_;
    const int n2 = 2 * n, n4 = 4 * n;
    for (int i = 0; i <= n4; i++)
    {
        int v;
        if (i == n2 || i == n4) v = s[i];
        else if (i == 0) v = (2 * s[0] + s[1] + s[n2 + 1] + 2) >> 2;
        else if (i == n2 + 1) v = (2 * s[n2 + 1] + s[0] + s[n2 + 2] + 2) >> 2;
        else v = (2 * s[i] + s[i - 1] + s[i + 1] + 2) >> 2;
        f[i] = (pix)v;
    }
}

static const int kAngle[17] = { -32, -26, -21, -17, -13, -9, -5, -2, 0, 2, 5, 9, 13, 17, 21, 26, 32 };
static const int kInvAngle[8] = { 4096, 1638, 910, 630, 482, 390, 315, 256 };

/* angular prediction in the vertical frame into out[y*os + x]
 * (intra_pred_ang_c, intrapred.cpp:102-189, before the horizontal transpose) */
static void ang_vertical_frame(int n, int mode, const pix* src0, int bfilter, pix* out, intptr_t os)
{
    const int n2 = 2 * n;
    const int hor = mode < 18;
    pix nb[129];
    const pix* s = src0;
    if (hor)
    {
        nb[0] = src0[0];
        for (int i = 0; i < n2; i++) { nb[1 + i] = src0[n2 + 1 + i]; nb[n2 + 1 + i] = src0[1 + i]; }
        s = nb;
    }
    const int aoff = hor ? 10 - mode : mode - 26;
    const int angle = kAngle[8 + aoff];
    if (!angle)
    {
        for (int y = 0; y < n; y++)
            for (int x = 0; x < n; x++) out[y * os + x] = s[1 + x];
        if (bfilter)
            for (int y = 0; y < n; y++) out[y * os] = (pix)clipp((int16_t)(s[1] + ((s[n2 + 1 + y] - s[0]) >> 1)));
        return;
    }
    /* reference array with index -n..2n, stored at ref[idx + 64] */
    int ref[200];
    for (int i = 0; i < n2; i++) ref[64 + i] = s[1 + i];
    ref[63] = s[0];
    if (angle < 0)
    {
        const int nproj = -((n * angle) >> 5) - 1, inv = kInvAngle[-aoff - 1];
        int acc = 128;
        for (int k = 0; k < nproj; k++)
        {
            acc += inv;
            ref[64 - 2 - k] = s[n2 + (acc >> 8)];
        }
    }
    for (int y = 0; y < n; y++)
    {
        const int sum = (y + 1) * angle, off = sum >> 5, f = sum & 31;
        for (int x = 0; x < n; x++)
        {
            const int a = ref[64 + off + x];
            out[y * os + x] = (pix)(f ? ((32 - f) * a + f * ref[64 + off + x + 1] + 16) >> 5 : a);
        }
    }
}

void xo_intra_pred(int n, int mode, void* dst_, intptr_t ds, const void* src_, int bFilter)
{
    pix* dst = (pix*)dst_;
    const pix* s = (const pix*)src_;
    const pix* above = s + 1;
    const pix* left = s + 2 * n + 1;
    if (mode == 0) /* planar, intrapred.cpp:87-100 */
    {
        const int lg = ilog2(n);
        for (int y = 0; y < n; y++)
            for (int x = 0; x < n; x++)
                dst[y * ds + x] = (pix)(((n - 1 - x) * left[y] + (n - 1 - y) * above[x] + (x + 1) * above[n] +
                                         (y + 1) * left[n] + n) >> (lg + 1));
        return;
    }
    if (mode == 1) /* DC, intrapred.cpp:53-85 */
    {
        int dc = n;
        for (int i = 0; i < n; i++) dc += above[i] + left[i];
        dc /= 2 * n;
        for (int y = 0; y < n; y++)
            for (int x = 0; x < n; x++) dst[y * ds + x] = (pix)dc;
        if (bFilter)
        {
            dst[0] = (pix)((above[0] + left[0] + 2 * dc + 2) >> 2);
            for (int x = 1; x < n; x++) dst[x] = (pix)((above[x] + 3 * dc + 2) >> 2);
            for (int y = 1; y < n; y++) dst[y * ds] = (pix)((left[y] + 3 * dc + 2) >> 2);
        }
        return;
    }
    pix tmp[32 * 32];
    ang_vertical_frame(n, mode, s, bFilter, tmp, n);
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) dst[y * ds + x] = mode < 18 ? tmp[x * n + y] : tmp[y * n + x];
}

/* intrapred.cpp:206-234: horizontal modes are stored un-transposed */
void xo_intra_allangs(int n, void* dst_, void* ref, void* filt, int bLuma)
{
    static const uint8_t flags[35] = { 0x38, 0x00, 0x38, 0x30, 0x30, 0x30, 0x30, 0x30, 0x30, 0x20, 0x00, 0x20,
                                       0x30, 0x30, 0x30, 0x30, 0x30, 0x30, 0x38, 0x30, 0x30, 0x30, 0x30, 0x30,
                                       0x30, 0x20, 0x00, 0x20, 0x30, 0x30, 0x30, 0x30, 0x30, 0x30, 0x38 };
    pix* dst = (pix*)dst_;
    for (int mode = 2; mode <= 34; mode++)
    {
        const pix* s = (flags[mode] & n) ? (const pix*)filt : (const pix*)ref;
        ang_vertical_frame(n, mode, s, bLuma, dst + (mode - 2) * n * n, n);
    }
}

/* ======================================================= companions */

/* pixel.cpp:416-428 */
void xo_calcresidual(int n, const void* fenc, const void* pred, int16_t* res, intptr_t stride)
{
    xo_sub_ps(n, n, res, stride, fenc, pred, stride, stride);
}

/* pixel.cpp:760-772 */
void xo_sub_ps(int w, int h, int16_t* d, intptr_t ds, const void* a_, const void* b_, intptr_t sa, intptr_t sb)
{
    const pix* a = (const pix*)a_;
    const pix* b = (const pix*)b_;
    for (int y = 0; y < h; y++, a += sa, b += sb, d += ds)
        for (int x = 0; x < w; x++) d[x] = (int16_t)((int)a[x] - (int)b[x]);
}

/* pixel.cpp:774-786 */
void xo_add_ps(int w, int h, void* d_, intptr_t ds, const void* a_, const int16_t* b, intptr_t sa, intptr_t sb)
{
    pix* d = (pix*)d_;
    const pix* a = (const pix*)a_;
    for (int y = 0; y < h; y++, a += sa, b += sb, d += ds)
        for (int x = 0; x < w; x++) d[x] = (pix)clipp(a[x] + b[x]);
}

/* pixel.cpp:788-808 */
void xo_addavg(int w, int h, const int16_t* a, const int16_t* b, void* d_, intptr_t sa, intptr_t sb, intptr_t ds)
{
    pix* d = (pix*)d_;
    const int shift = IF_IPREC + 1 - XO_DEPTH, off = (1 << (shift - 1)) + 2 * IF_OFFS;
    for (int y = 0; y < h; y++, a += sa, b += sb, d += ds)
        for (int x = 0; x < w; x++) d[x] = (pix)clipp((a[x] + b[x] + off) >> shift);
}

/* pixel.cpp:490-502 */
void xo_pixelavg(int w, int h, void* d_, intptr_t ds, const void* a_, intptr_t sa, const void* b_, intptr_t sb)
{
    pix* d = (pix*)d_;
    const pix* a = (const pix*)a_;
    const pix* b = (const pix*)b_;
    for (int y = 0; y < h; y++, a += sa, b += sb, d += ds)
        for (int x = 0; x < w; x++) d[x] = (pix)((a[x] + b[x] + 1) >> 1);
}

/* pixel.cpp:705-758 */
void xo_copy_pp(int w, int h, void* d_, intptr_t ds, const void* s_, intptr_t ss)
{
    pix* d = (pix*)d_;
    const pix* s = (const pix*)s_;
    for (int y = 0; y < h; y++) memcpy(d + y * ds, s + y * ss, w * sizeof(pix));
}

void xo_copy_sp(int w, int h, void* d_, intptr_t ds, const int16_t* s, intptr_t ss)
{
    pix* d = (pix*)d_;
    for (int y = 0; y < h; y++, d += ds, s += ss)
        for (int x = 0; x < w; x++) d[x] = (pix)s[x];
}

void xo_copy_ps(int w, int h, int16_t* d, intptr_t ds, const void* s_, intptr_t ss)
{
    const pix* s = (const pix*)s_;
    for (int y = 0; y < h; y++, d += ds, s += ss)
        for (int x = 0; x < w; x++) d[x] = (int16_t)s[x];
}

void xo_copy_ss(int w, int h, int16_t* d, intptr_t ds, const int16_t* s, intptr_t ss)
{
    for (int y = 0; y < h; y++) memcpy(d + y * ds, s + y * ss, w * sizeof(int16_t));
}

/* pixel.cpp:338-344 */
void xo_blockfill_s(int n, int16_t* d, intptr_t ds, int16_t v)
{
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) d[y * ds + x] = v;
}

/* pixel.cpp:346-414 */
void xo_cpy2Dto1D_shl(int n, int16_t* d, const int16_t* s, intptr_t ss, int shift)
{
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) d[y * n + x] = (int16_t)shl_wrap(s[y * ss + x], shift);
}

void xo_cpy2Dto1D_shr(int n, int16_t* d, const int16_t* s, intptr_t ss, int shift)
{
    const int16_t rnd = (int16_t)(1 << (shift - 1));
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) d[y * n + x] = (int16_t)((s[y * ss + x] + rnd) >> shift);
}

void xo_cpy1Dto2D_shl(int n, int16_t* d, const int16_t* s, intptr_t ds, int shift)
{
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) d[y * ds + x] = (int16_t)shl_wrap(s[y * n + x], shift);
}

void xo_cpy1Dto2D_shr(int n, int16_t* d, const int16_t* s, intptr_t ds, int shift)
{
    const int16_t rnd = (int16_t)(1 << (shift - 1));
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) d[y * ds + x] = (int16_t)((s[y * n + x] + rnd) >> shift);
}

/* dct.cpp:714-742 */
int xo_count_nonzero(int n, const int16_t* q)
{
    int c = 0;
    for (int i = 0; i < n * n; i++) c += q[i] != 0;
    return c;
}

uint32_t xo_copy_cnt(int n, int16_t* coeff, const int16_t* res, intptr_t rs)
{
    uint32_t c = 0;
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++)
        {
            coeff[y * n + x] = res[y * rs + x];
            c += res[y * rs + x] != 0;
        }
    return c;
}

/* pixel.cpp:430-436 */
void xo_transpose(int n, void* d_, const void* s_, intptr_t ss)
{
    pix* d = (pix*)d_;
    const pix* s = (const pix*)s_;
    for (int k = 0; k < n; k++)
        for (int l = 0; l < n; l++) d[k * n + l] = s[l * ss + k];
}

/* dct.cpp:744-755 */
void xo_denoise_dct(int16_t* coef, uint32_t* resSum, const uint16_t* offset, int num)
{
    for (int i = 0; i < num; i++)
    {
        int lv = coef[i], sg = lv >> 31;
        lv = (lv + sg) ^ sg;
        resSum[i] += lv;
        lv -= offset[i];
        coef[i] = (int16_t)(lv < 0 ? 0 : (lv ^ sg) - sg);
    }
}

/* ===================================================================== f3
 * Fused TU pipeline: the body of the bCheckFull branch of
 * Search::residualTransformQuantIntra (search.cpp:668-706) without the
 * prediction, i.e. calcresidual -> Quant::transformNxN (quant.cpp:397-491,
 * no RDOQ / transform skip / bypass / noise reduction, flat scaling list)
 * -> numSig ? Quant::invtransformNxN (quant.cpp:493-546) + add_ps : copy_pp. */

/* HEVC scan orders (spec 6.5.3-6.5.5; x265 g_scanOrder, constants.cpp:359-456),
 * generated rather than transcribed: coefficient groups of 4x4 are visited in
 * the scan of the CG grid, positions inside a CG in the 4x4 scan of the same
 * type.  type 0 = up-right diagonal, 1 = horizontal, 2 = vertical. */
static void scan_grid(int type, int n, int* order /* n*n raster indices */)
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

void xo_scan_table(int type, int log2, uint16_t* out)
{
    const int n = 1 << log2, g = n >> 2;
    int cg[64], in[16];
    scan_grid(type, g, cg);
    scan_grid(type, 4, in);
    for (int c = 0; c < g * g; c++)
        for (int i = 0; i < 16; i++)
        {
            const int cr = cg[c] / g, cc = cg[c] % g, r = in[i] / 4, q = in[i] % 4;
            out[c * 16 + i] = (uint16_t)((cr * 4 + r) * n + cc * 4 + q);
        }
}

static const int kQuantScales[6] = { 26214, 23302, 20560, 18396, 16384, 14564 };   /* scalinglist.cpp:121 */
static const int kInvQuantScales[6] = { 40, 45, 51, 57, 64, 72 };                 /* scalinglist.cpp:122 */

/* Quant::signBitHidingHDQ (quant.cpp:247-393) on one TU */
static uint32_t sign_hide(int16_t* coeff, const int16_t* dct, const int32_t* deltaU, uint32_t numSig,
                          const uint16_t* scan, int num)
{
    int last = -1;
    for (int p = num - 1; p >= 0; p--)
        if (coeff[scan[p]]) { last = p; break; }
    const int cgLast = last >> 4;
    for (int cg = cgLast; cg >= 0; cg--)
    {
        const int base = cg << 4, top = cg == cgLast ? (last & 15) : 15;
        int first = -1, lastNZ = -1;
        for (int n = 0; n <= top; n++)
            if (coeff[scan[base + n]]) { if (first < 0) first = n; lastNZ = n; }
        if (first < 0 || lastNZ - first < 4)       /* SBH_THRESHOLD, common.h:273 */
            continue;
        const int signbit = coeff[scan[base + first]] > 0 ? 0 : 1;
        int sum = 0;
        for (int n = first; n <= lastNZ; n++) sum += coeff[scan[base + n]];
        if (signbit == (sum & 1))
            continue;
        int minCost = 0x7fffffff, minPos = -1, finalChange = 0;
        for (int n = top; n >= 0; n--)
        {
            const int pos = scan[base + n];
            int nzBelow = 0;                       /* any non-zero at scan positions < n */
            for (int m = 0; m < n; m++) nzBelow |= coeff[scan[base + m]] != 0;
            int cost, change = 0;
            if (coeff[pos])
            {
                if (deltaU[pos] > 0) { cost = -deltaU[pos]; change = 1; }
                else if (!nzBelow && abs(coeff[pos]) == 1) cost = 0x7fffffff;
                else { cost = deltaU[pos]; change = -1; }
            }
            else if (!nzBelow)                      /* before the first non-zero */
            {
                if ((dct[pos] >= 0 ? 0 : 1) != signbit) cost = 0x7fffffff;
                else { cost = -deltaU[pos]; change = 1; }
            }
            else { cost = -deltaU[pos]; change = 1; }
            if (cost < minCost) { minCost = cost; finalChange = change; minPos = pos; }
        }
        if (coeff[minPos] == 32767 || coeff[minPos] == -32768) finalChange = -1;
        if (!coeff[minPos]) numSig++;
        else if (finalChange == -1 && abs(coeff[minPos]) == 1) numSig--;
        const int sigMask = dct[minPos] < 0 ? -1 : 0;
        coeff[minPos] = (int16_t)(coeff[minPos] + ((finalChange ^ sigMask) - sigMask));
    }
    return numSig;
}

uint32_t xo_tu_pipeline(int log2, int is_luma, int is_intra, int i_slice, int sign_hide_on, int qp, int scan_type,
                        const void* fenc, intptr_t fs, const void* pred, intptr_t ps,
                        int16_t* resi, intptr_t rs, int16_t* coeff, void* recon, intptr_t rcs)
{
    const int n = 1 << log2, num = n * n;
    const int use_dst = log2 == 2 && is_luma && is_intra;
    const int rem = qp % 6, per = qp / 6;
    const int tshift = 15 - XO_DEPTH - log2;     /* MAX_TR_DYNAMIC_RANGE - depth - log2 */
    int16_t dct[32 * 32], dq[32 * 32];
    int32_t qc[32 * 32], deltaU[32 * 32];
    uint16_t scan[32 * 32];

    xo_sub_ps(n, n, resi, rs, fenc, pred, fs, ps);   /* calcresidual with per-operand strides */
    xo_dct(use_dst ? XO_DST : XO_DCT, n, resi, dct, rs);
    for (int i = 0; i < num; i++) qc[i] = kQuantScales[rem];
    const int qbits = 14 + per + tshift;
    const int add = (i_slice ? 171 : 85) << (qbits - 9);
    uint32_t numSig = xo_quant(dct, qc, deltaU, coeff, qbits, add, num);
    if (numSig >= 2 && sign_hide_on)
    {
        xo_scan_table(scan_type, log2, scan);
        numSig = sign_hide(coeff, dct, deltaU, numSig, scan, num);
    }
    if (!numSig)
    {
        xo_copy_pp(n, n, recon, rcs, pred, ps);
        return 0;
    }
    const int shift = 20 - 14 - tshift;           /* QUANT_IQUANT_SHIFT - QUANT_SHIFT - transformShift */
    xo_dequant_normal(coeff, dq, num, kInvQuantScales[rem] << per, shift);
    if (numSig == 1 && coeff[0] != 0 && !use_dst)
    {
        const int sh2 = 12 - (XO_DEPTH - 8) - 3;
        const int dc = (((dq[0] + 1) >> 1) * 8 + (1 << (sh2 - 1))) >> sh2;
        xo_blockfill_s(n, resi, rs, (int16_t)dc);
    }
    else
        xo_dct(use_dst ? XO_IDST : XO_IDCT, n, dq, resi, rs);
    xo_add_ps(n, n, recon, rcs, pred, resi, ps, rs);
    return numSig;
}

/* ===================================================================== f1
 * Lookahead lowres pipeline, the parts that are pure
 * functions of the source picture: Lowres::init's plane generation and
 * LookaheadTLD::lowresIntraEstimate. */

/* g_intraFilterFlags (constants.cpp:550-556): bit N set = mode uses the filtered samples at TU size N */
static const uint8_t kIntraFilterFlags[35] = { 0x38, 0x00, 0x38, 0x30, 0x30, 0x30, 0x30, 0x30, 0x30, 0x20, 0x00, 0x20,
                                               0x30, 0x30, 0x30, 0x30, 0x30, 0x30, 0x38, 0x30, 0x30, 0x30, 0x30, 0x30,
                                               0x30, 0x20, 0x00, 0x20, 0x30, 0x30, 0x30, 0x30, 0x30, 0x30, 0x38 };
#define kIntraFilterFlags8(m) (kIntraFilterFlags[m] & 8)

static void extend_border(pix* pic, intptr_t stride, int width, int height, int mx, int my)
{
    /* extendPicBorder (pixel.cpp:908-922) = extendRowBorder (ipfilter.cpp:59-77) + row copies */
    for (int y = 0; y < height; y++)
        for (int x = 0; x < mx; x++)
        {
            pic[y * stride - mx + x] = pic[y * stride];
            pic[y * stride + width + x] = pic[y * stride + width - 1];
        }
    pix* top = pic - mx;
    for (int y = 0; y < my; y++) memcpy(top - (y + 1) * stride, top, stride * sizeof(pix));
    pix* bot = pic - mx + (height - 1) * stride;
    for (int y = 0; y < my; y++) memcpy(bot + (y + 1) * stride, bot, stride * sizeof(pix));
}

void xo_lowres_init(int width, int lines, const void* src_, intptr_t ss, void* p0_, void* p1_, void* p2_, void* p3_,
                    intptr_t ls, int mx, int my)
{
    /* frame_init_lowres_core (pixel.cpp:549-573): four half-pel phases of a 2:1 box downscale */
    const pix* src = (const pix*)src_;
    pix* d[4] = { (pix*)p0_, (pix*)p1_, (pix*)p2_, (pix*)p3_ };
#define XO_AVG4(a, b, c, e) ((((a) + (b) + 1) >> 1) + (((c) + (e) + 1) >> 1) + 1) >> 1
    for (int y = 0; y < lines; y++)
    {
        const pix* r0 = src + 2 * y * ss;
        const pix* r1 = r0 + ss;
        const pix* r2 = r1 + ss;
        for (int x = 0; x < width; x++)
        {
            d[0][y * ls + x] = (pix)(XO_AVG4(r0[2 * x], r1[2 * x], r0[2 * x + 1], r1[2 * x + 1]));
            d[1][y * ls + x] = (pix)(XO_AVG4(r0[2 * x + 1], r1[2 * x + 1], r0[2 * x + 2], r1[2 * x + 2]));
            d[2][y * ls + x] = (pix)(XO_AVG4(r1[2 * x], r2[2 * x], r1[2 * x + 1], r2[2 * x + 1]));
            d[3][y * ls + x] = (pix)(XO_AVG4(r1[2 * x + 1], r2[2 * x + 1], r1[2 * x + 2], r2[2 * x + 2]));
        }
    }
#undef XO_AVG4
    for (int k = 0; k < 4; k++) extend_border(d[k], ls, width, lines, mx, my);
}

/* slicetype.cpp:230-330 (LookaheadTLD::lowresIntraEstimate) over one frame's 8x8 lowres CUs.
 * inv_q may be NULL (no AQ).  cost_est[0] = costEst[0][0], cost_est[1] = costEstAq[0][0]. */
void xo_lowres_intra(int wcu, int hcu, const void* plane_, intptr_t ls, const int32_t* inv_q, int32_t* intra_cost,
                     uint8_t* intra_mode, uint16_t* lowres_cost, int32_t* row_satd, int64_t* cost_est)
{
    const pix* plane = (const pix*)plane_;
    /* (int)x265_lambda_tab[X265_LOOKAHEAD_QP], X265_LOOKAHEAD_QP = 12 + QP_BD_OFFSET (common.h:208):
     * lambda_tab[q] = 2^(q/6 - 2) * 2^(depth - 8) (constants.cpp:31-151) -> 1 (8-bit), 16 (10-bit), 256 (12-bit) */
    const int lambda = XO_DEPTH == 8 ? 1 : XO_DEPTH == 10 ? 16 : 256;
    const int intra_penalty = 5 * lambda, lowres_penalty = 4;
    int64_t est = 0, est_aq = 0;
    pix fenc[64], pred[64], samples[33], filtered[33];
    for (int cy = 0; cy < hcu; cy++)
    {
        row_satd[cy] = 0;
        for (int cx = 0; cx < wcu; cx++)
        {
            const int xy = cx + cy * wcu;
            const pix* cur = plane + 8 * cx + 8 * cy * ls;
            for (int y = 0; y < 8; y++) memcpy(fenc + 8 * y, cur + y * ls, 8 * sizeof(pix));
            const pix* nb = cur - ls - 1;
            memcpy(samples, nb, 17 * sizeof(pix));
            for (int i = 1; i <= 16; i++) samples[16 + i] = nb[i * ls];
            xo_intra_filter(8, samples, filtered);
            int icost = 0x7fffffff, imode = 0, cost;
            xo_intra_pred(8, 1, pred, 8, samples, 1);                  /* DC, edge filter (8 <= 16) */
            cost = xo_satd(8, 8, fenc, 8, pred, 8);
            if (cost < icost) { icost = cost; imode = 1; }
            xo_intra_pred(8, 0, pred, 8, filtered, 0);                 /* planar from the filtered samples */
            cost = xo_satd(8, 8, fenc, 8, pred, 8);
            if (cost < icost) { icost = cost; imode = 0; }
            int acost = 0x7fffffff, amode = 4;
            for (int m = 5; m < 35; m += 5)
            {
                xo_intra_pred(8, m, pred, 8, (kIntraFilterFlags8(m) ? filtered : samples), 1);
                cost = xo_satd(8, 8, fenc, 8, pred, 8);
                if (cost < acost) { acost = cost; amode = m; }
            }
            for (int dist = 2; dist >= 1; dist--)
            {
                const int lo = amode - dist, hi = amode + dist;
                xo_intra_pred(8, lo, pred, 8, (kIntraFilterFlags8(lo) ? filtered : samples), 1);
                cost = xo_satd(8, 8, fenc, 8, pred, 8);
                if (cost < acost) { acost = cost; amode = lo; }
                xo_intra_pred(8, hi, pred, 8, (kIntraFilterFlags8(hi) ? filtered : samples), 1);
                cost = xo_satd(8, 8, fenc, 8, pred, 8);
                if (cost < acost) { acost = cost; amode = hi; }
            }
            if (acost < icost) { icost = acost; imode = amode; }
            icost += intra_penalty + lowres_penalty;
            lowres_cost[xy] = (uint16_t)(icost < 0x3fff ? icost : 0x3fff);   /* LOWRES_COST_MASK, shift 0 */
            intra_cost[xy] = icost;
            intra_mode[xy] = (uint8_t)imode;
            const int scored = (cx > 0 && cx < wcu - 1 && cy > 0 && cy < hcu - 1) || wcu <= 2 || hcu <= 2;
            const int icost_aq = (scored && inv_q) ? ((icost * inv_q[xy] + 128) >> 8) : icost;
            if (scored) { est += icost; est_aq += icost_aq; }
            row_satd[cy] += icost_aq;
        }
    }
    cost_est[0] = est;
    cost_est[1] = est_aq;
}

/* ---------------------------------------------------------------- f1: lowres motion search
 * CostEstimateGroup::estimateFrameCost / estimateCUCost for a P estimate (b == p1, list 0
 * only: slicetype.cpp:1977-2066, 2068-2225) with MotionEstimate::motionEstimate's lowres HEX
 * path at subpel level 1 (motion.cpp:571-1172; LookaheadTLD sets X265_HEX_SEARCH and subme 1,
 * slicetype.h:61-64) and BitCost's MV cost (bitcost.h:45, bitcost.cpp). */

typedef struct { int x, y; } xmv;

/* BitCost::setQP(X265_LOOKAHEAD_QP) table, centre at index 0: s_costs[qp][i] =
 * min(s_bitsizes[i] * lambda + 0.5f, 2^15 - 1), s_bitsizes[i] = log(i + 1) * 2 / log(2) + 1.718f
 * (float), s_bitsizes[0] = 0.718f (bitcost.cpp:41-86).  out has 2 * range + 1 entries. */
void xo_mvcost_table(int range, uint16_t* out)
{
    const double lambda = XO_DEPTH == 8 ? 1.0 : XO_DEPTH == 10 ? 16.0 : 256.0;   /* lambda_tab[12 + QP_BD_OFFSET] */
    const float log2_2 = 2.0f / logf(2.0f);
    for (int i = 0; i <= range; i++)
    {
        const float bits = i ? logf((float)(i + 1)) * log2_2 + 1.718f : 0.718f;
        double v = bits * lambda + 0.5f;
        if (v > (1 << 15) - 1) v = (1 << 15) - 1;
        out[range + i] = out[range - i] = (uint16_t)v;
    }
}

typedef struct
{
    const pix* fenc;          /* 8x8 block, stride 8 */
    const pix* ref[4];        /* lowres planes of the reference at the block origin */
    intptr_t ls;
    const uint16_t* tab;      /* mv cost table centre */
    xmv mvp;
} XoMe;

static int xo_mvcost(const XoMe* m, xmv q)
{
    return (uint16_t)(m->tab[q.x - m->mvp.x] + m->tab[q.y - m->mvp.y]);
}

static int xo_fpel_sad(const XoMe* m, int x, int y)
{
    return xo_sad(8, 8, m->fenc, 8, m->ref[0] + x + y * m->ls, m->ls);
}

/* ReferencePlanes::lowresQPelCost / lowresMC (lowres.h:57-104): hpel plane or the rounded
 * average of the two hpel planes around a qpel position */
static int xo_qpel_cost(const XoMe* m, xmv q, int use_satd)
{
    pix buf[64];
    const pix* p;
    intptr_t ps;
    if ((q.x | q.y) & 1)
    {
        const int ha = (q.y & 2) | ((q.x & 2) >> 1);
        const pix* a = m->ref[ha] + (q.x >> 2) + (q.y >> 2) * m->ls;
        const int qx = q.x + (q.x & 1), qy = q.y + (q.y & 1);
        const int hb = (qy & 2) | ((qx & 2) >> 1);
        const pix* b = m->ref[hb] + (qx >> 2) + (qy >> 2) * m->ls;
        xo_pixelavg(8, 8, buf, 8, a, m->ls, b, m->ls);
        p = buf;
        ps = 8;
    }
    else
    {
        p = m->ref[(q.y & 2) | ((q.x & 2) >> 1)] + (q.x >> 2) + (q.y >> 2) * m->ls;
        ps = m->ls;
    }
    return use_satd ? xo_satd(8, 8, m->fenc, 8, p, ps) : xo_sad(8, 8, m->fenc, 8, p, ps);
}

static xmv xo_clip(xmv v, xmv lo, xmv hi)
{
    xmv r = v;
    if (r.x > hi.x) r.x = hi.x;
    if (r.y > hi.y) r.y = hi.y;
    if (r.x < lo.x) r.x = lo.x;
    if (r.y < lo.y) r.y = lo.y;
    return r;
}

static int xo_in_range(xmv v, xmv lo, xmv hi) { return v.x >= lo.x && v.x <= hi.x && v.y >= lo.y && v.y <= hi.y; }

/* MotionEstimate::motionEstimate, lowres reference, no extra candidates, HEX search, subme 1 */
static int xo_me_lowres(XoMe* m, xmv mvmin, xmv mvmax, xmv qmvp, int merange, xmv* out)
{
    static const xmv hex2[8] = { { -1, -2 }, { -2, 0 }, { -1, 2 }, { 1, 2 }, { 2, 0 }, { 1, -2 }, { -1, -2 }, { -2, 0 } };
    static const int mod6m1[8] = { 5, 0, 1, 2, 3, 4, 5, 0 };
    static const xmv square1[9] = { { 0, 0 }, { 0, -1 }, { 0, 1 }, { -1, 0 }, { 1, 0 }, { -1, -1 }, { -1, 1 }, { 1, -1 }, { 1, 1 } };
    m->mvp = qmvp;
    const xmv qmin = { mvmin.x * 4, mvmin.y * 4 }, qmax = { mvmax.x * 4, mvmax.y * 4 };
    xmv pmv = xo_clip(qmvp, qmin, qmax);
    const xmv bestpre = pmv;
    const int bprecost = xo_qpel_cost(m, pmv, 0);                 /* no MV cost (motion.cpp:606) */
    xmv bmv = { (pmv.x + 2) >> 2, (pmv.y + 2) >> 2 };
    int bcost = bprecost;
    if ((pmv.x | pmv.y) & 3)
        bcost = xo_fpel_sad(m, bmv.x, bmv.y) + xo_mvcost(m, (xmv){ bmv.x * 4, bmv.y * 4 });
    if (pmv.x || pmv.y)
    {
        const int c = xo_fpel_sad(m, 0, 0) + xo_mvcost(m, (xmv){ 0, 0 });
        if (c < bcost) { bcost = c; bmv.x = bmv.y = 0; }
    }
    /* hexagon, radius 2 (motion.cpp:681-730), costs packed with the direction in 3 low bits */
#define XO_HEXC(dx, dy) (xo_fpel_sad(m, bmv.x + (dx), bmv.y + (dy)) + \
                         xo_mvcost(m, (xmv){ (bmv.x + (dx)) * 4, (bmv.y + (dy)) * 4 }))
    {
        int c0 = XO_HEXC(-2, 0), c1 = XO_HEXC(-1, 2), c2 = XO_HEXC(1, 2);
        bcost <<= 3;
        if ((c0 << 3) + 2 < bcost) bcost = (c0 << 3) + 2;
        if ((c1 << 3) + 3 < bcost) bcost = (c1 << 3) + 3;
        if ((c2 << 3) + 4 < bcost) bcost = (c2 << 3) + 4;
        c0 = XO_HEXC(2, 0); c1 = XO_HEXC(1, -2); c2 = XO_HEXC(-1, -2);
        if ((c0 << 3) + 5 < bcost) bcost = (c0 << 3) + 5;
        if ((c1 << 3) + 6 < bcost) bcost = (c1 << 3) + 6;
        if ((c2 << 3) + 7 < bcost) bcost = (c2 << 3) + 7;
        if (bcost & 7)
        {
            int dir = (bcost & 7) - 2;
            bmv.x += hex2[dir + 1].x; bmv.y += hex2[dir + 1].y;
            for (int i = (merange >> 1) - 1; i > 0 && xo_in_range(bmv, mvmin, mvmax); i--)
            {
                c0 = XO_HEXC(hex2[dir + 0].x, hex2[dir + 0].y);
                c1 = XO_HEXC(hex2[dir + 1].x, hex2[dir + 1].y);
                c2 = XO_HEXC(hex2[dir + 2].x, hex2[dir + 2].y);
                bcost &= ~7;
                if ((c0 << 3) + 1 < bcost) bcost = (c0 << 3) + 1;
                if ((c1 << 3) + 2 < bcost) bcost = (c1 << 3) + 2;
                if ((c2 << 3) + 3 < bcost) bcost = (c2 << 3) + 3;
                if (!(bcost & 7)) break;
                dir += (bcost & 7) - 2;
                dir = mod6m1[dir + 1];
                bmv.x += hex2[dir + 1].x; bmv.y += hex2[dir + 1].y;
            }
        }
        bcost >>= 3;
        /* square refine */
        int dir = 0;
        for (int k = 1; k <= 8; k++)
        {
            const int c = XO_HEXC(square1[k].x, square1[k].y);
            if (c < bcost) { bcost = c; dir = k; }
        }
        bmv.x += square1[dir].x; bmv.y += square1[dir].y;
    }
#undef XO_HEXC
    if (bprecost < bcost) { bmv = bestpre; bcost = bprecost; }
    else { bmv.x *= 4; bmv.y *= 4; }
    if (!bcost)
        bcost = xo_mvcost(m, bmv);
    else
    {
        /* workload[1]: 4 SAD half-pel, then 4 SATD quarter-pel (motion.cpp:1095-1116) */
        int bdir = 0;
        for (int i = 1; i <= 4; i++)
        {
            const xmv q = { bmv.x + square1[i].x * 2, bmv.y + square1[i].y * 2 };
            const int c = xo_qpel_cost(m, q, 0) + xo_mvcost(m, q);
            if (c < bcost) { bcost = c; bdir = i; }
        }
        bmv.x += square1[bdir].x * 2; bmv.y += square1[bdir].y * 2;
        bcost = xo_qpel_cost(m, bmv, 1) + xo_mvcost(m, bmv);
        bdir = 0;
        for (int i = 1; i <= 4; i++)
        {
            const xmv q = { bmv.x + square1[i].x, bmv.y + square1[i].y };
            const int c = xo_qpel_cost(m, q, 1) + xo_mvcost(m, q);
            if (c < bcost) { bcost = c; bdir = i; }
        }
        bmv.x += square1[bdir].x; bmv.y += square1[bdir].y;
    }
    *out = bmv;
    return bcost;
}

void xo_lowres_pcost(int wcu, int hcu, int rows_per_slice, int num_slices, const void* fenc_plane0,
                     const void* r0, const void* r1, const void* r2, const void* r3, intptr_t ls,
                     const int32_t* intra_cost, const int32_t* inv_q, const uint16_t* mvcost_centre,
                     int16_t* mvs, int32_t* mv_costs, uint16_t* lowres_costs, int32_t* row_satd, int64_t* cost_est,
                     int32_t* intra_mbs)
{
    const pix* fp = (const pix*)fenc_plane0;
    const pix* rp[4] = { (const pix*)r0, (const pix*)r1, (const pix*)r2, (const pix*)r3 };
    if (num_slices < 1) { num_slices = 1; rows_per_slice = hcu; }
    int64_t est = 0, est_aq = 0;
    int mbs = 0;
    for (int s = 0; s < num_slices; s++)
    {
        /* CostEstimateGroup::processTasks (slicetype.cpp:1957-1972) / the serial loop (:2041-2050) */
        const int first = rows_per_slice * s;
        const int last = s == num_slices - 1 ? hcu - 1 : rows_per_slice * (s + 1) - 1;
        int last_row = 1;
        for (int cy = last; cy >= first; cy--)
        {
            row_satd[cy] = 0;
            for (int cx = wcu - 1; cx >= 0; cx--)
            {
                const int xy = cx + cy * wcu;
                const intptr_t off = 8 * cx + 8 * cy * ls;
                pix fenc[64];
                for (int y = 0; y < 8; y++) memcpy(fenc + 8 * y, fp + off + y * ls, 8 * sizeof(pix));
                XoMe m = { fenc, { rp[0] + off, rp[1] + off, rp[2] + off, rp[3] + off }, ls, mvcost_centre, { 0, 0 } };
                const xmv mvmin = { -cx * 8 - 8, -cy * 8 - 8 };
                const xmv mvmax = { (wcu - cx - 1) * 8 + 8, (hcu - cy - 1) * 8 + 8 };
                xmv mvc[4];
                int numc = 0;
                if (cx < wcu - 1) { mvc[numc].x = mvs[2 * (xy + 1)]; mvc[numc++].y = mvs[2 * (xy + 1) + 1]; }
                if (!last_row)
                {
                    mvc[numc].x = mvs[2 * (xy + wcu)]; mvc[numc++].y = mvs[2 * (xy + wcu) + 1];
                    if (cx > 0) { mvc[numc].x = mvs[2 * (xy + wcu - 1)]; mvc[numc++].y = mvs[2 * (xy + wcu - 1) + 1]; }
                    if (cx < wcu - 1) { mvc[numc].x = mvs[2 * (xy + wcu + 1)]; mvc[numc++].y = mvs[2 * (xy + wcu + 1) + 1]; }
                }
                xmv mvp = { 0, 0 };
                if (numc)
                {
                    int mvpcost = 1 << 28;                                 /* MotionEstimate::COST_MAX */
                    for (int i = 0; i < numc; i++)
                    {
                        const int c = xo_qpel_cost(&m, mvc[i], 1);         /* bufSATD(lowresMC(mvc)) */
                        if (c < mvpcost) { mvpcost = c; mvp = mvc[i]; }
                    }
                }
                xmv out;
                const int fcost = xo_me_lowres(&m, mvmin, mvmax, mvp, 16, &out);   /* s_merange = 16 */
                mvs[2 * xy] = (int16_t)out.x;
                mvs[2 * xy + 1] = (int16_t)out.y;
                mv_costs[xy] = fcost;
                int bcost = 1 << 28, listused = 0;
                if (fcost < bcost) { bcost = fcost; listused = 1; }
                bcost += 4;                                                /* lowresPenalty */
                if (intra_cost[xy] < bcost) { bcost = intra_cost[xy]; listused = 0; }
                const int scored = (cx > 0 && cx < wcu - 1 && cy > 0 && cy < hcu - 1) || wcu <= 2 || hcu <= 2;
                const int bcost_aq = (scored && inv_q) ? ((bcost * inv_q[xy] + 128) >> 8) : bcost;
                if (scored)
                {
                    est += bcost;
                    est_aq += bcost_aq;
                    if (!listused) mbs++;
                }
                row_satd[cy] += bcost_aq;
                lowres_costs[xy] = (uint16_t)((bcost < 0x3fff ? bcost : 0x3fff) | (listused << 14));
            }
            last_row = 0;
        }
    }
    cost_est[0] = est;
    cost_est[1] = est_aq;
    *intra_mbs = mbs;
}

/* ReferencePlanes::lowresMC (lowres.h:57-80) into an 8x8 buffer (stride 8) */
static void xo_lowres_mc(const pix* const ref[4], intptr_t ls, xmv q, pix* out)
{
    if ((q.x | q.y) & 1)
    {
        const int ha = (q.y & 2) | ((q.x & 2) >> 1);
        const pix* a = ref[ha] + (q.x >> 2) + (q.y >> 2) * ls;
        const int qx = q.x + (q.x & 1), qy = q.y + (q.y & 1);
        const int hb = (qy & 2) | ((qx & 2) >> 1);
        const pix* b = ref[hb] + (qx >> 2) + (qy >> 2) * ls;
        xo_pixelavg(8, 8, out, 8, a, ls, b, ls);
    }
    else
    {
        const pix* p = ref[(q.y & 2) | ((q.x & 2) >> 1)] + (q.x >> 2) + (q.y >> 2) * ls;
        for (int y = 0; y < 8; y++) memcpy(out + 8 * y, p + y * ls, 8 * sizeof(pix));
    }
}

/* CostEstimateGroup::estimateFrameCost for a B estimate (p0 < b < p1) = estimateCUCost
 * (slicetype.cpp:2068-2225) with bBidir: per list i with bDoSearch[i] the MVP choice (incl. the
 * skipCost of a zero MVP), the lowres HEX search from fref0 (list 0) / fref1 (list 1) and the
 * zero-MV skip override; lists not searched reuse lowresMvCosts; then the bidir average of the two
 * lists' predictions and the co-located average, each scored by SATD.  Weighted prediction off. */
void xo_lowres_bcost(int wcu, int hcu, int rows_per_slice, int num_slices, const void* fenc_plane0,
                     const void* const* ref0, const void* const* ref1, intptr_t ls, const int32_t* inv_q,
                     const uint16_t* mvcost_centre, int do_search0, int do_search1, int16_t* mvs0,
                     int32_t* mv_costs0, int16_t* mvs1, int32_t* mv_costs1, uint16_t* lowres_costs,
                     int32_t* row_satd, int64_t* cost_est)
{
    const pix* fp = (const pix*)fenc_plane0;
    const pix* rp[2][4];
    for (int k = 0; k < 4; k++) { rp[0][k] = (const pix*)ref0[k]; rp[1][k] = (const pix*)ref1[k]; }
    int16_t* mvs[2] = { mvs0, mvs1 };
    int32_t* mcost[2] = { mv_costs0, mv_costs1 };
    const int ds[2] = { do_search0, do_search1 };
    if (num_slices < 1) { num_slices = 1; rows_per_slice = hcu; }
    int64_t est = 0, est_aq = 0;
    for (int s = 0; s < num_slices; s++)
    {
        const int first = rows_per_slice * s;
        const int last = s == num_slices - 1 ? hcu - 1 : rows_per_slice * (s + 1) - 1;
        int last_row = 1;
        for (int cy = last; cy >= first; cy--)
        {
            row_satd[cy] = 0;
            for (int cx = wcu - 1; cx >= 0; cx--)
            {
                const int xy = cx + cy * wcu;
                const intptr_t off = 8 * cx + 8 * cy * ls;
                pix fenc[64];
                for (int y = 0; y < 8; y++) memcpy(fenc + 8 * y, fp + off + y * ls, 8 * sizeof(pix));
                const xmv mvmin = { -cx * 8 - 8, -cy * 8 - 8 };
                const xmv mvmax = { (wcu - cx - 1) * 8 + 8, (hcu - cy - 1) * 8 + 8 };
                int bcost = 1 << 28, listused = 0;
                for (int i = 0; i < 2; i++)
                {
                    if (!ds[i])
                    {
                        if (mcost[i][xy] < bcost) { bcost = mcost[i][xy]; listused = i + 1; }
                        continue;
                    }
                    int16_t* mv = mvs[i];
                    XoMe m = { fenc, { rp[i][0] + off, rp[i][1] + off, rp[i][2] + off, rp[i][3] + off }, ls,
                               mvcost_centre, { 0, 0 } };
                    xmv mvc[4];
                    int numc = 0;
                    if (cx < wcu - 1) { mvc[numc].x = mv[2 * (xy + 1)]; mvc[numc++].y = mv[2 * (xy + 1) + 1]; }
                    if (!last_row)
                    {
                        mvc[numc].x = mv[2 * (xy + wcu)]; mvc[numc++].y = mv[2 * (xy + wcu) + 1];
                        if (cx > 0) { mvc[numc].x = mv[2 * (xy + wcu - 1)]; mvc[numc++].y = mv[2 * (xy + wcu - 1) + 1]; }
                        if (cx < wcu - 1) { mvc[numc].x = mv[2 * (xy + wcu + 1)]; mvc[numc++].y = mv[2 * (xy + wcu + 1) + 1]; }
                    }
                    xmv mvp = { 0, 0 };
                    int skip = 0x7fffffff;                                  /* INT_MAX */
                    if (numc)
                    {
                        int mvpcost = 1 << 28;
                        for (int k = 0; k < numc; k++)
                        {
                            const int c = xo_qpel_cost(&m, mvc[k], 1);
                            if (c < mvpcost) { mvpcost = c; mvp = mvc[k]; }
                            if (!mvp.x && !mvp.y) skip = c;                 /* the candidate's cost, as written */
                        }
                    }
                    xmv out;
                    int fcost = xo_me_lowres(&m, mvmin, mvmax, mvp, 16, &out);
                    if (skip < 64 && skip < fcost) { fcost = skip; out.x = out.y = 0; }
                    mv[2 * xy] = (int16_t)out.x;
                    mv[2 * xy + 1] = (int16_t)out.y;
                    mcost[i][xy] = fcost;
                    if (fcost < bcost) { bcost = fcost; listused = i + 1; }
                }
                /* bidir: avg(l0 prediction, l1 prediction), then the co-located average */
                pix b0[64], b1[64], avg[64];
                const pix* r0o[4] = { rp[0][0] + off, rp[0][1] + off, rp[0][2] + off, rp[0][3] + off };
                const pix* r1o[4] = { rp[1][0] + off, rp[1][1] + off, rp[1][2] + off, rp[1][3] + off };
                const xmv m0 = { mvs0[2 * xy], mvs0[2 * xy + 1] }, m1 = { mvs1[2 * xy], mvs1[2 * xy + 1] };
                xo_lowres_mc(r0o, ls, m0, b0);
                xo_lowres_mc(r1o, ls, m1, b1);
                xo_pixelavg(8, 8, avg, 8, b0, 8, b1, 8);
                int bicost = xo_satd(8, 8, fenc, 8, avg, 8);
                if (bicost < bcost) { bcost = bicost; listused = 3; }
                xo_pixelavg(8, 8, avg, 8, rp[0][0] + off, ls, rp[1][0] + off, ls);
                bicost = xo_satd(8, 8, fenc, 8, avg, 8);
                if (bicost < bcost) { bcost = bicost; listused = 3; }
                bcost += 4;                                                /* lowresPenalty */
                const int scored = (cx > 0 && cx < wcu - 1 && cy > 0 && cy < hcu - 1) || wcu <= 2 || hcu <= 2;
                const int bcost_aq = (scored && inv_q) ? ((bcost * inv_q[xy] + 128) >> 8) : bcost;
                if (scored)
                {
                    est += bcost;
                    est_aq += bcost_aq;
                }
                row_satd[cy] += bcost_aq;
                lowres_costs[xy] = (uint16_t)((bcost < 0x3fff ? bcost : 0x3fff) | (listused << 14));
            }
            last_row = 0;
        }
    }
    cost_est[0] = est;
    cost_est[1] = est_aq;
}

/* ---------------------------------------------------------------- f2: full-resolution motion search
 * MotionEstimate::motionEstimate (motion.cpp:571-1172) for one PU on a full-resolution
 * reference: clipped MVP measured at sub-pel with SAD, the extra MV candidates, DIA or HEX
 * integer search, then the sub-pel refine of workload[subme] for subme 0..7 (motion.cpp:48-58;
 * chroma SATD from subme 3, motion.cpp:197).  Sub-pel blocks come from the 8-tap luma
 * filters exactly as subpelCompare (motion.cpp:1174-1203) builds them. */

typedef struct
{
    int w, h;
    const pix* fenc; intptr_t fs;
    const pix* ref; intptr_t rs;        /* reference at the PU origin */
    const uint16_t* tab;
    xmv mvp;
    int chroma;                         /* bChromaSATD (subme > 2 and a 4:2:0 chroma satd entry exists) */
    const pix* fc[2]; intptr_t fcs;     /* source Cb / Cr at the PU's chroma origin */
    const pix* rc[2]; intptr_t rcs;     /* reference Cb / Cr at the PU's chroma origin */
} XoMeF;

static int xo_f_mvcost(const XoMeF* m, int qx, int qy)
{
    return (uint16_t)(m->tab[qx - m->mvp.x] + m->tab[qy - m->mvp.y]);
}

static int xo_f_fpel_sad(const XoMeF* m, int x, int y)
{
    return xo_sad(m->w, m->h, m->fenc, m->fs, m->ref + x + y * m->rs, m->rs);
}

static int xo_subpel_compare(const XoMeF* m, int qx, int qy, int use_satd)
{
    const pix* fr = m->ref + (qx >> 2) + (qy >> 2) * m->rs;
    const int xf = qx & 3, yf = qy & 3;
    const pix* p = fr;
    intptr_t ps = m->rs;
    pix buf[64 * 64];
    if (xf | yf)
    {
        if (!yf) xo_interp(XO_HPP, 8, m->w, m->h, fr, m->rs, buf, 64, xf, 0);
        else if (!xf) xo_interp(XO_VPP, 8, m->w, m->h, fr, m->rs, buf, 64, yf, 0);
        else xo_interp(XO_HVPP, 8, m->w, m->h, fr, m->rs, buf, 64, xf, yf);
        p = buf;
        ps = 64;
    }
    int cost = use_satd ? xo_satd(m->w, m->h, m->fenc, m->fs, p, ps) : xo_sad(m->w, m->h, m->fenc, m->fs, p, ps);
    if (m->chroma)
    {
        /* chroma SATD at the 1/8-pel chroma position (motion.cpp:1205-1266, 4:2:0) */
        const int cw = m->w >> 1, chh = m->h >> 1;
        const intptr_t off = (qx >> 3) + (qy >> 3) * m->rcs;
        const int cxf = qx & 7, cyf = qy & 7;
        for (int k = 0; k < 2; k++)
        {
            const pix* rc = m->rc[k] + off;
            if (!(cxf | cyf))
                cost += xo_satd(cw, chh, m->fc[k], m->fcs, rc, m->rcs);
            else
            {
                pix cb[64 * 32];
                if (!cyf) xo_interp(XO_HPP, 4, cw, chh, rc, m->rcs, cb, 64, cxf, 0);
                else if (!cxf) xo_interp(XO_VPP, 4, cw, chh, rc, m->rcs, cb, 64, cyf, 0);
                else
                {
                    int16_t immed[32 * (32 + 3)];
                    xo_interp(XO_HPS, 4, cw, chh, rc, m->rcs, immed, cw, cxf, 1);
                    xo_interp(XO_VSP, 4, cw, chh, immed + cw, cw, cb, 64, cyf, 0);
                }
                cost += xo_satd(cw, chh, m->fc[k], m->fcs, cb, 64);
            }
        }
    }
    return cost;
}

/* MotionEstimate::StarPatternSearch (motion.cpp:328-569) */
static void xo_star(XoMeF* m, xmv mvmin, xmv mvmax, xmv* bmv, int* bcost, int* bPointNr, int* bDistance,
                    int earlyExitIters, int merange)
{
    const xmv omv = *bmv;
    int saved = *bcost, rounds = 0;
#define PT(mx, my, pt, dd) do { \
        const int c_ = xo_f_fpel_sad(m, (mx), (my)) + xo_f_mvcost(m, (mx) * 4, (my) * 4); \
        if (c_ < *bcost) { *bcost = c_; bmv->x = (mx); bmv->y = (my); *bPointNr = (pt); *bDistance = (dd); } } while (0)
    {
        const int dist = 1;
        const int top = omv.y - dist, bottom = omv.y + dist, left = omv.x - dist, right = omv.x + dist;
        if (top >= mvmin.y && left >= mvmin.x && right <= mvmax.x && bottom <= mvmax.y)
        {
            PT(omv.x, top, 2, dist); PT(left, omv.y, 4, dist); PT(right, omv.y, 5, dist); PT(omv.x, bottom, 7, dist);
        }
        else
        {
            if (top >= mvmin.y) PT(omv.x, top, 2, dist);
            if (left >= mvmin.x) PT(left, omv.y, 4, dist);
            if (right <= mvmax.x) PT(right, omv.y, 5, dist);
            if (bottom <= mvmax.y) PT(omv.x, bottom, 7, dist);
        }
        if (*bcost < saved) rounds = 0;
        else if (++rounds >= earlyExitIters) return;
    }
    for (int dist = 2; dist <= 8; dist <<= 1)
    {
        const int top = omv.y - dist, bottom = omv.y + dist, left = omv.x - dist, right = omv.x + dist;
        const int top2 = omv.y - (dist >> 1), bottom2 = omv.y + (dist >> 1);
        const int left2 = omv.x - (dist >> 1), right2 = omv.x + (dist >> 1);
        saved = *bcost;
        if (top >= mvmin.y && left >= mvmin.x && right <= mvmax.x && bottom <= mvmax.y)
        {
            PT(omv.x, top, 2, dist); PT(left2, top2, 1, dist >> 1); PT(right2, top2, 3, dist >> 1);
            PT(left, omv.y, 4, dist);
            PT(right, omv.y, 5, dist); PT(left2, bottom2, 6, dist >> 1); PT(right2, bottom2, 8, dist >> 1);
            PT(omv.x, bottom, 7, dist);
        }
        else
        {
            if (top >= mvmin.y) PT(omv.x, top, 2, dist);
            if (top2 >= mvmin.y)
            {
                if (left2 >= mvmin.x) PT(left2, top2, 1, dist >> 1);
                if (right2 <= mvmax.x) PT(right2, top2, 3, dist >> 1);
            }
            if (left >= mvmin.x) PT(left, omv.y, 4, dist);
            if (right <= mvmax.x) PT(right, omv.y, 5, dist);
            if (bottom2 <= mvmax.y)
            {
                if (left2 >= mvmin.x) PT(left2, bottom2, 6, dist >> 1);
                if (right2 <= mvmax.x) PT(right2, bottom2, 8, dist >> 1);
            }
            if (bottom <= mvmax.y) PT(omv.x, bottom, 7, dist);
        }
        if (*bcost < saved) rounds = 0;
        else if (++rounds >= earlyExitIters) return;
    }
    for (int dist = 16; dist <= merange; dist <<= 1)
    {
        const int top = omv.y - dist, bottom = omv.y + dist, left = omv.x - dist, right = omv.x + dist;
        saved = *bcost;
        if (top >= mvmin.y && left >= mvmin.x && right <= mvmax.x && bottom <= mvmax.y)
        {
            PT(omv.x, top, 0, dist); PT(left, omv.y, 0, dist); PT(right, omv.y, 0, dist); PT(omv.x, bottom, 0, dist);
            for (int index = 1; index < 4; index++)
            {
                const int yt = top + ((dist >> 2) * index), yb = bottom - ((dist >> 2) * index);
                const int xl = omv.x - ((dist >> 2) * index), xr = omv.x + ((dist >> 2) * index);
                PT(xl, yt, 0, dist); PT(xr, yt, 0, dist); PT(xl, yb, 0, dist); PT(xr, yb, 0, dist);
            }
        }
        else
        {
            if (top >= mvmin.y) PT(omv.x, top, 0, dist);
            if (left >= mvmin.x) PT(left, omv.y, 0, dist);
            if (right <= mvmax.x) PT(right, omv.y, 0, dist);
            if (bottom <= mvmax.y) PT(omv.x, bottom, 0, dist);
            for (int index = 1; index < 4; index++)
            {
                const int yt = top + ((dist >> 2) * index), yb = bottom - ((dist >> 2) * index);
                const int xl = omv.x - ((dist >> 2) * index), xr = omv.x + ((dist >> 2) * index);
                if (yt >= mvmin.y)
                {
                    if (xl >= mvmin.x) PT(xl, yt, 0, dist);
                    if (xr <= mvmax.x) PT(xr, yt, 0, dist);
                }
                if (yb <= mvmax.y)
                {
                    if (xl >= mvmin.x) PT(xl, yb, 0, dist);
                    if (xr <= mvmax.x) PT(xr, yb, 0, dist);
                }
            }
        }
        if (*bcost < saved) rounds = 0;
        else if (++rounds >= earlyExitIters) return;
    }
#undef PT
}

int xo_motion_search(int w, int h, int method, int subme, int merange, const void* fenc, intptr_t fs, const void* ref,
                     intptr_t rs, int minx, int miny, int maxx, int maxy, int mvpx, int mvpy, int numc,
                     const int16_t* mvc, const uint16_t* tab_centre, int16_t* out,
                     const void* fcb, const void* fcr, intptr_t fcs, const void* rcb, const void* rcr, intptr_t rcs)
{
    static const xmv hex2[8] = { { -1, -2 }, { -2, 0 }, { -1, 2 }, { 1, 2 }, { 2, 0 }, { 1, -2 }, { -1, -2 }, { -2, 0 } };
    static const int mod6m1[8] = { 5, 0, 1, 2, 3, 4, 5, 0 };
    static const xmv square1[9] = { { 0, 0 }, { 0, -1 }, { 0, 1 }, { -1, 0 }, { 1, 0 }, { -1, -1 }, { -1, 1 }, { 1, -1 }, { 1, 1 } };
    /* workload[] (motion.cpp:48-58): hpel_iters, hpel_dirs, qpel_iters, qpel_dirs, hpel_satd */
    static const int wl[8][5] = { { 1, 4, 0, 4, 0 }, { 1, 4, 1, 4, 0 }, { 1, 4, 1, 4, 1 }, { 2, 4, 1, 4, 1 },
                                  { 2, 4, 2, 4, 1 }, { 1, 8, 1, 8, 1 }, { 2, 8, 1, 8, 1 }, { 2, 8, 2, 8, 1 } };
    static const xmv offs[16] = { { -1, 0 }, { 0, -1 }, { -1, -1 }, { 1, -1 }, { -1, 0 }, { 1, 0 }, { -1, 1 }, { -1, -1 },
                                  { 1, -1 }, { 1, 1 }, { -1, 0 }, { 0, 1 }, { -1, 1 }, { 1, 1 }, { 1, 0 }, { 0, 1 } };
    XoMeF m = { w, h, (const pix*)fenc, fs, (const pix*)ref, rs, tab_centre, { mvpx, mvpy }, 0,
                { (const pix*)fcb, (const pix*)fcr }, fcs, { (const pix*)rcb, (const pix*)rcr }, rcs };
    /* bChromaSATD = subpelRefine > 2 && the 4:2:0 chroma satd entry exists (both chroma dims % 4 == 0) */
    m.chroma = subme > 2 && fcb && ((w >> 1) & 3) == 0 && ((h >> 1) & 3) == 0;
    const xmv qmin = { minx * 4, miny * 4 }, qmax = { maxx * 4, maxy * 4 };
    const xmv mvmin = { minx, miny }, mvmax = { maxx, maxy };
    xmv pmv = xo_clip((xmv){ mvpx, mvpy }, qmin, qmax);
    xmv bestpre = pmv;
    int bprecost = xo_subpel_compare(&m, pmv.x, pmv.y, 0);            /* no MV cost (motion.cpp:609) */
    xmv bmv = { (pmv.x + 2) >> 2, (pmv.y + 2) >> 2 };
    int bcost = bprecost;
    if ((pmv.x | pmv.y) & 3)
        bcost = xo_f_fpel_sad(&m, bmv.x, bmv.y) + xo_f_mvcost(&m, bmv.x * 4, bmv.y * 4);
    if (pmv.x || pmv.y)
    {
        const int c = xo_f_fpel_sad(&m, 0, 0) + xo_f_mvcost(&m, 0, 0);
        if (c < bcost) { bcost = c; bmv.x = bmv.y = 0; }
    }
    for (int i = 0; i < numc; i++)
    {
        const xmv c = xo_clip((xmv){ mvc[2 * i], mvc[2 * i + 1] }, qmin, qmax);
        if ((c.x || c.y) && (c.x != pmv.x || c.y != pmv.y) && (c.x != bestpre.x || c.y != bestpre.y))
        {
            const int cost = xo_subpel_compare(&m, c.x, c.y, 0) + xo_f_mvcost(&m, c.x, c.y);
            if (cost < bprecost) { bprecost = cost; bestpre = c; }
        }
    }
#define XO_FC(dx, dy) (xo_f_fpel_sad(&m, bmv.x + (dx), bmv.y + (dy)) + \
                       xo_f_mvcost(&m, (bmv.x + (dx)) * 4, (bmv.y + (dy)) * 4))
    if (method == 0)
    {
        /* diamond, radius 1 (motion.cpp:654-676) */
        bcost <<= 4;
        int i = merange;
        do
        {
            const int c0 = XO_FC(0, -1), c1 = XO_FC(0, 1), c2 = XO_FC(-1, 0), c3 = XO_FC(1, 0);
            if ((c0 << 4) + 1 < bcost) bcost = (c0 << 4) + 1;
            if ((c1 << 4) + 3 < bcost) bcost = (c1 << 4) + 3;
            if ((c2 << 4) + 4 < bcost) bcost = (c2 << 4) + 4;
            if ((c3 << 4) + 12 < bcost) bcost = (c3 << 4) + 12;
            if (!(bcost & 15)) break;
            bmv.x -= (int32_t)((uint32_t)bcost << 28) >> 30;
            bmv.y -= (int32_t)((uint32_t)bcost << 30) >> 30;
            bcost &= ~15;
        } while (--i && xo_in_range(bmv, mvmin, mvmax));
        bcost >>= 4;
    }
    else if (method == 2)
    {
        /* STAR (motion.cpp:929-1034) */
        int bPointNr = 0, bDistance = 0;
        int done = 0;
        xo_star(&m, mvmin, mvmax, &bmv, &bcost, &bPointNr, &bDistance, 3, merange);
        if (bDistance == 1)
        {
            if (bPointNr)
            {
                const int saved = bcost;
                const xmv m1 = { bmv.x + offs[(bPointNr - 1) * 2].x, bmv.y + offs[(bPointNr - 1) * 2].y };
                const xmv m2 = { bmv.x + offs[(bPointNr - 1) * 2 + 1].x, bmv.y + offs[(bPointNr - 1) * 2 + 1].y };
                if (xo_in_range(m1, mvmin, mvmax))
                {
                    const int c = xo_f_fpel_sad(&m, m1.x, m1.y) + xo_f_mvcost(&m, m1.x * 4, m1.y * 4);
                    if (c < bcost) { bcost = c; bmv = m1; }
                }
                if (xo_in_range(m2, mvmin, mvmax))
                {
                    const int c = xo_f_fpel_sad(&m, m2.x, m2.y) + xo_f_mvcost(&m, m2.x * 4, m2.y * 4);
                    if (c < bcost) { bcost = c; bmv = m2; }
                }
                if (bcost == saved) done = 1;
            }
            else
                done = 1;
        }
        if (!done)
        {
            if (bDistance > 5)
            {
                /* raster refinement; the 4th sad_x4 lane's MV cost uses tmv << 3 in the reference (motion.cpp:993) */
                for (int ty = mvmin.y; ty <= mvmax.y; ty += 5)
                    for (int tx = mvmin.x; tx <= mvmax.x; tx += 5)
                    {
                        if (tx + 15 <= mvmax.x)
                        {
                            int c;
                            c = xo_f_fpel_sad(&m, tx, ty) + xo_f_mvcost(&m, tx * 4, ty * 4);
                            if (c < bcost) { bcost = c; bmv.x = tx; bmv.y = ty; }
                            tx += 5;
                            c = xo_f_fpel_sad(&m, tx, ty) + xo_f_mvcost(&m, tx * 4, ty * 4);
                            if (c < bcost) { bcost = c; bmv.x = tx; bmv.y = ty; }
                            tx += 5;
                            c = xo_f_fpel_sad(&m, tx, ty) + xo_f_mvcost(&m, tx * 4, ty * 4);
                            if (c < bcost) { bcost = c; bmv.x = tx; bmv.y = ty; }
                            tx += 5;
                            c = xo_f_fpel_sad(&m, tx, ty) + xo_f_mvcost(&m, tx * 8, ty * 8);
                            if (c < bcost) { bcost = c; bmv.x = tx; bmv.y = ty; }
                        }
                        else
                        {
                            const int c = xo_f_fpel_sad(&m, tx, ty) + xo_f_mvcost(&m, tx * 4, ty * 4);
                            if (c < bcost) { bcost = c; bmv.x = tx; bmv.y = ty; }
                        }
                    }
            }
            while (bDistance > 0)
            {
                bDistance = 0;
                bPointNr = 0;
                xo_star(&m, mvmin, mvmax, &bmv, &bcost, &bPointNr, &bDistance, 32, merange);
                if (bDistance == 1)
                {
                    if (!bPointNr) break;
                    const xmv m1 = { bmv.x + offs[(bPointNr - 1) * 2].x, bmv.y + offs[(bPointNr - 1) * 2].y };
                    const xmv m2 = { bmv.x + offs[(bPointNr - 1) * 2 + 1].x, bmv.y + offs[(bPointNr - 1) * 2 + 1].y };
                    if (xo_in_range(m1, mvmin, mvmax))
                    {
                        const int c = xo_f_fpel_sad(&m, m1.x, m1.y) + xo_f_mvcost(&m, m1.x * 4, m1.y * 4);
                        if (c < bcost) { bcost = c; bmv = m1; }
                    }
                    if (xo_in_range(m2, mvmin, mvmax))
                    {
                        const int c = xo_f_fpel_sad(&m, m2.x, m2.y) + xo_f_mvcost(&m, m2.x * 4, m2.y * 4);
                        if (c < bcost) { bcost = c; bmv = m2; }
                    }
                    break;
                }
            }
        }
    }
    else
    {
    int do_hex = 1;
    if (method == 4)
    {
        /* FULL (motion.cpp:1039-1074): every integer MV of the range in raster order; the sad_x4
           grouping of the reference changes nothing (each candidate's cost is SAD + mvcost(tmv << 2)) */
        for (int ty = mvmin.y; ty <= mvmax.y; ty++)
            for (int tx = mvmin.x; tx <= mvmax.x; tx++)
            {
                const int c = xo_f_fpel_sad(&m, tx, ty) + xo_f_mvcost(&m, tx * 4, ty * 4);
                if (c < bcost) { bcost = c; bmv.x = tx; bmv.y = ty; }
            }
        do_hex = 0;
    }
    else if (method == 3)
    {
        /* UMH (motion.cpp:744-926); ends either by leaving the search (`break`: do_hex = 0) or by
           continuing with the hexagon search at me_hex2 when the result is in range */
        static const xmv hex4[16] = { { 0, -4 }, { 0, 4 }, { -2, -3 }, { 2, -3 }, { -4, -2 }, { 4, -2 }, { -4, -1 },
                                      { 4, -1 }, { -4, 0 }, { 4, 0 }, { -4, 1 }, { 4, 1 }, { -4, 2 }, { 4, 2 },
                                      { -2, 3 }, { 2, 3 } };
        static const uint8_t range_mul[4][4] = { { 3, 3, 4, 4 }, { 3, 4, 4, 4 }, { 4, 4, 4, 5 }, { 4, 4, 5, 6 } };
        const int scale = (h * h) >> 4;                      /* sizeScale[partEnum] (motion.cpp:121-150) */
#define XO_SAD_THRESH(v) (bcost < (((v) >> 4) * scale))
#define XO_COST_MV(mx, my) do { const int _x = (mx), _y = (my); \
            const int _c = xo_f_fpel_sad(&m, _x, _y) + xo_f_mvcost(&m, _x * 4, _y * 4); \
            if (_c < bcost) { bcost = _c; bmv.x = _x; bmv.y = _y; } } while (0)
#define XO_COST_MV_X4(a0, b0, a1, b1, a2, b2, a3, b3) do { \
            const int _c0 = xo_f_fpel_sad(&m, omv.x + (a0), omv.y + (b0)) + xo_f_mvcost(&m, (omv.x + (a0)) * 4, (omv.y + (b0)) * 4); \
            const int _c1 = xo_f_fpel_sad(&m, omv.x + (a1), omv.y + (b1)) + xo_f_mvcost(&m, (omv.x + (a1)) * 4, (omv.y + (b1)) * 4); \
            const int _c2 = xo_f_fpel_sad(&m, omv.x + (a2), omv.y + (b2)) + xo_f_mvcost(&m, (omv.x + (a2)) * 4, (omv.y + (b2)) * 4); \
            const int _c3 = xo_f_fpel_sad(&m, omv.x + (a3), omv.y + (b3)) + xo_f_mvcost(&m, (omv.x + (a3)) * 4, (omv.y + (b3)) * 4); \
            if (_c0 < bcost) { bcost = _c0; bmv.x = omv.x + (a0); bmv.y = omv.y + (b0); } \
            if (_c1 < bcost) { bcost = _c1; bmv.x = omv.x + (a1); bmv.y = omv.y + (b1); } \
            if (_c2 < bcost) { bcost = _c2; bmv.x = omv.x + (a2); bmv.y = omv.y + (b2); } \
            if (_c3 < bcost) { bcost = _c3; bmv.x = omv.x + (a3); bmv.y = omv.y + (b3); } } while (0)
#define XO_DIA1(mx, my) do { omv.x = (mx); omv.y = (my); XO_COST_MV_X4(0, -1, 0, 1, -1, 0, 1, 0); } while (0)
#define XO_CROSS(start, x_max, y_max) do { \
            int _i = (start); const int _xm = (x_max), _ym = (y_max); \
            if (_xm <= XO_MIN2(mvmax.x - omv.x, omv.x - mvmin.x)) \
                for (; _i < _xm - 2; _i += 4) XO_COST_MV_X4(_i, 0, -_i, 0, _i + 2, 0, -_i - 2, 0); \
            for (; _i < _xm; _i += 2) { \
                if (omv.x + _i <= mvmax.x) XO_COST_MV(omv.x + _i, omv.y); \
                if (omv.x - _i >= mvmin.x) XO_COST_MV(omv.x - _i, omv.y); } \
            _i = (start); \
            if (_ym <= XO_MIN2(mvmax.y - omv.y, omv.y - mvmin.y)) \
                for (; _i < _ym - 2; _i += 4) XO_COST_MV_X4(0, _i, 0, -_i, 0, _i + 2, 0, -_i - 2); \
            for (; _i < _ym; _i += 2) { \
                if (omv.y + _i <= mvmax.y) XO_COST_MV(omv.x, omv.y + _i); \
                if (omv.y - _i >= mvmin.y) XO_COST_MV(omv.x, omv.y - _i); } } while (0)
#define XO_MIN2(a, b) ((a) < (b) ? (a) : (b))
        const xmv fpmv = { (pmv.x + 2) >> 2, (pmv.y + 2) >> 2 };       /* pmv.roundToFPel() (motion.cpp:645) */
        xmv omv = bmv;
        int cross_start = 1, range = merange;
        const int ucost1 = bcost;
        XO_DIA1(fpmv.x, fpmv.y);
        if (fpmv.x || fpmv.y) XO_DIA1(0, 0);
        const int ucost2 = bcost;
        if ((bmv.x || bmv.y) && (bmv.x != fpmv.x || bmv.y != fpmv.y)) XO_DIA1(bmv.x, bmv.y);
        if (bcost == ucost2) cross_start = 3;
        omv = bmv;
        do_hex = -1;
        if (bcost == ucost2 && XO_SAD_THRESH(2000))
        {
            XO_COST_MV_X4(0, -2, -1, -1, 1, -1, -2, 0);
            XO_COST_MV_X4(2, 0, -1, 1, 1, 1, 0, 2);
            if (bcost == ucost1 && XO_SAD_THRESH(500)) do_hex = 0;
            else if (bcost == ucost2)
            {
                const int r = (merange >> 1) | 1;
                XO_CROSS(3, r, r);
                XO_COST_MV_X4(-1, -2, 1, -2, -2, -1, 2, -1);
                XO_COST_MV_X4(-2, 1, 2, 1, -1, 2, 1, 2);
                if (bcost == ucost2) do_hex = 0;
                else cross_start = r + 2;
            }
        }
        if (do_hex)
        {
            if (numc)
            {
                /* adaptive range from the candidates' agreement (motion.cpp:785-834) */
                int mvd, denom = 1;
                const int is64 = w == 64 && h == 64;
                if (numc == 1)
                    mvd = is64 ? 25 : abs(mvpx - mvc[0]) + abs(mvpy - mvc[1]);
                else
                {
                    denom = numc - 1;
                    mvd = 0;
                    if (!is64)
                    {
                        mvd = abs(mvpx - mvc[0]) + abs(mvpy - mvc[1]);
                        denom++;
                    }
                    for (int k = 0; k < numc - 1; k++)     /* predictorDifference (motion.cpp:87-98) */
                        mvd += abs(mvc[2 * k] - mvc[2 * k + 2]) + abs(mvc[2 * k + 1] - mvc[2 * k + 3]);
                }
                const int sad_ctx = XO_SAD_THRESH(1000) ? 0 : XO_SAD_THRESH(2000) ? 1 : XO_SAD_THRESH(4000) ? 2 : 3;
                const int mvd_ctx = mvd < 10 * denom ? 0 : mvd < 20 * denom ? 1 : mvd < 40 * denom ? 2 : 3;
                range = (range * range_mul[mvd_ctx][sad_ctx]) >> 2;
            }
            merange = range;                     /* the reference rescales merange itself: me_hex2 sees it */
            XO_CROSS(cross_start, range, range >> 1);
            XO_COST_MV_X4(-2, -2, -2, 2, 2, -2, 2, 2);
            /* hexagon grid (motion.cpp:866-921) */
            omv = bmv;
            int gi = 1;
            do
            {
                const int lim = XO_MIN2(XO_MIN2(mvmax.x - omv.x, omv.x - mvmin.x), XO_MIN2(mvmax.y - omv.y, omv.y - mvmin.y));
                if (4 * gi > lim)
                {
                    for (int k = 0; k < 16; k++)
                    {
                        const xmv c = { omv.x + hex4[k].x * gi, omv.y + hex4[k].y * gi };
                        if (xo_in_range(c, mvmin, mvmax)) XO_COST_MV(c.x, c.y);
                    }
                }
                else
                {
                    int dir = 0;
                    for (int k = 0; k < 16; k++)
                    {
                        const int c = xo_f_fpel_sad(&m, omv.x + hex4[k].x * gi, omv.y + hex4[k].y * gi) +
                                      xo_f_mvcost(&m, (omv.x + hex4[k].x * gi) * 4, (omv.y + hex4[k].y * gi) * 4);
                        if (c < bcost) { bcost = c; dir = hex4[k].x * 16 + (hex4[k].y & 15); }
                    }
                    if (dir)
                    {
                        bmv.x = omv.x + gi * (dir >> 4);
                        bmv.y = omv.y + gi * ((int32_t)((uint32_t)dir << 28) >> 28);
                    }
                }
            } while (++gi <= range >> 2);
            do_hex = xo_in_range(bmv, mvmin, mvmax);
        }
#undef XO_SAD_THRESH
#undef XO_COST_MV
#undef XO_COST_MV_X4
#undef XO_DIA1
#undef XO_CROSS
#undef XO_MIN2
    }
    if (do_hex)
    {
        int c0 = XO_FC(-2, 0), c1 = XO_FC(-1, 2), c2 = XO_FC(1, 2);
        bcost <<= 3;
        if ((c0 << 3) + 2 < bcost) bcost = (c0 << 3) + 2;
        if ((c1 << 3) + 3 < bcost) bcost = (c1 << 3) + 3;
        if ((c2 << 3) + 4 < bcost) bcost = (c2 << 3) + 4;
        c0 = XO_FC(2, 0); c1 = XO_FC(1, -2); c2 = XO_FC(-1, -2);
        if ((c0 << 3) + 5 < bcost) bcost = (c0 << 3) + 5;
        if ((c1 << 3) + 6 < bcost) bcost = (c1 << 3) + 6;
        if ((c2 << 3) + 7 < bcost) bcost = (c2 << 3) + 7;
        if (bcost & 7)
        {
            int dir = (bcost & 7) - 2;
            bmv.x += hex2[dir + 1].x; bmv.y += hex2[dir + 1].y;
            for (int i = (merange >> 1) - 1; i > 0 && xo_in_range(bmv, mvmin, mvmax); i--)
            {
                c0 = XO_FC(hex2[dir + 0].x, hex2[dir + 0].y);
                c1 = XO_FC(hex2[dir + 1].x, hex2[dir + 1].y);
                c2 = XO_FC(hex2[dir + 2].x, hex2[dir + 2].y);
                bcost &= ~7;
                if ((c0 << 3) + 1 < bcost) bcost = (c0 << 3) + 1;
                if ((c1 << 3) + 2 < bcost) bcost = (c1 << 3) + 2;
                if ((c2 << 3) + 3 < bcost) bcost = (c2 << 3) + 3;
                if (!(bcost & 7)) break;
                dir += (bcost & 7) - 2;
                dir = mod6m1[dir + 1];
                bmv.x += hex2[dir + 1].x; bmv.y += hex2[dir + 1].y;
            }
        }
        bcost >>= 3;
        int dir = 0;
        for (int k = 1; k <= 8; k++)
        {
            const int c = XO_FC(square1[k].x, square1[k].y);
            if (c < bcost) { bcost = c; dir = k; }
        }
        bmv.x += square1[dir].x; bmv.y += square1[dir].y;
    }
    }
#undef XO_FC
    if (bprecost < bcost) { bmv = bestpre; bcost = bprecost; }
    else { bmv.x *= 4; bmv.y *= 4; }
    const int* W = wl[subme];
    if (!bcost)
        bcost = xo_f_mvcost(&m, bmv.x, bmv.y);
    else
    {
        int hsatd = W[4];
        if (hsatd) bcost = xo_subpel_compare(&m, bmv.x, bmv.y, 1) + xo_f_mvcost(&m, bmv.x, bmv.y);
        for (int it = 0; it < W[0]; it++)
        {
            int bdir = 0;
            for (int i = 1; i <= W[1]; i++)
            {
                const int qx = bmv.x + square1[i].x * 2, qy = bmv.y + square1[i].y * 2;
                const int c = xo_subpel_compare(&m, qx, qy, hsatd) + xo_f_mvcost(&m, qx, qy);
                if (c < bcost) { bcost = c; bdir = i; }
            }
            if (bdir) { bmv.x += square1[bdir].x * 2; bmv.y += square1[bdir].y * 2; }
            else break;
        }
        if (!hsatd) bcost = xo_subpel_compare(&m, bmv.x, bmv.y, 1) + xo_f_mvcost(&m, bmv.x, bmv.y);
        for (int it = 0; it < W[2]; it++)
        {
            int bdir = 0;
            for (int i = 1; i <= W[3]; i++)
            {
                const int qx = bmv.x + square1[i].x, qy = bmv.y + square1[i].y;
                const int c = xo_subpel_compare(&m, qx, qy, 1) + xo_f_mvcost(&m, qx, qy);
                if (c < bcost) { bcost = c; bdir = i; }
            }
            if (bdir) { bmv.x += square1[bdir].x; bmv.y += square1[bdir].y; }
            else break;
        }
    }
    out[0] = (int16_t)bmv.x;
    out[1] = (int16_t)bmv.y;
    return bcost;
}

/* BitCost::setQP(qp) table: out[range + d] for |d| <= range.  Restated only for the lookahead QP
 * (xo_mvcost_table); for other QPs the reference's table is the fixture (lambda_tab is data). */

/* ======================================================= f4 loop filters */

void xo_extend_border(void* plane, intptr_t stride, int width, int height, int mx, int my)
{
    extend_border((pix*)plane, stride, width, height, mx, my);
}

static int sgn(int v) { return (v > 0) - (v < 0); }

/* SAO::s_eoTable (sao.cpp:65-72): edge type (sign sum + 2) -> EO class */
static const int kEoClass[5] = { 1, 2, 0, 3, 4 };

/* the two neighbour offsets of EO class direction t (sao.cpp:321-560): -, |, 135, 45 degrees */
static void eo_dirs(int t, int* dx0, int* dy0, int* dx1, int* dy1)
{
    static const int d[4][4] = { { -1, 0, 1, 0 }, { 0, -1, 0, 1 }, { -1, -1, 1, 1 }, { 1, -1, -1, 1 } };
    *dx0 = d[t][0]; *dy0 = d[t][1]; *dx1 = d[t][2]; *dy1 = d[t][3];
}

/* processSaoCu semantics (sao.cpp:278-597): every output pixel is computed from deblocked (pre-SAO)
 * neighbours (the m_tmpU / m_tmpL copies keep them), EO skips the picture's outermost column / row
 * in its direction, BO maps bands (bandPos + i) & 31 to offset[i]. */
void xo_sao_apply_csp(int width, int height, int ctu_log2, void* y_, void* cb_, void* cr_, intptr_t stride,
                      intptr_t cstride, const xo_sao_param* params, int luma_on, int chroma_on, int csp)
{
    const int hs = csp == 3 ? 0 : 1, vs = csp == 1 ? 1 : 0;   /* CHROMA_H/V_SHIFT (x265.h) */
    const int ctu = 1 << ctu_log2;
    const int wc = (width + ctu - 1) >> ctu_log2, hc = (height + ctu - 1) >> ctu_log2, nctu = wc * hc;
    pix* planes[3] = { (pix*)y_, (pix*)cb_, (pix*)cr_ };
    for (int p = 0; p < 3; p++)
    {
        if (p == 0 ? !luma_on : !chroma_on) continue;
        const intptr_t s = p ? cstride : stride;
        const int pw = p ? width >> hs : width, ph = p ? height >> vs : height;
        const int csw = p ? ctu >> hs : ctu, csh = p ? ctu >> vs : ctu;
        /* the deblocked plane plus a one-pixel ring, as the processing reads it */
        const int sw = pw + 2, sh = ph + 2;
        pix* snap = (pix*)malloc(sizeof(pix) * sw * sh);
        for (int yy = -1; yy <= ph; yy++)
            for (int xx = -1; xx <= pw; xx++) snap[(yy + 1) * sw + xx + 1] = planes[p][yy * s + xx];
#define SN(xx, yy) ((int)snap[((yy) + 1) * sw + (xx) + 1])
        for (int c = 0; c < nctu; c++)
        {
            const xo_sao_param* prm = &params[p * nctu + c];
            int type = prm->type;
            if (p == 2 && type >= 0) type = params[nctu + c].type;   /* processSaoCu(addr, typeIdxCb, 2) */
            if (type < 0) continue;
            const int x0 = (c % wc) * csw, y0 = (c / wc) * csh;
            const int x1 = x0 + csw < pw ? x0 + csw : pw, y1 = y0 + csh < ph ? y0 + csh : ph;
            if (type == 4)
            {
                int8_t tab[32] = { 0 };
                for (int i = 0; i < 4; i++) tab[(prm->band + i) & 31] = prm->offset[i];
                for (int yy = y0; yy < y1; yy++)
                    for (int xx = x0; xx < x1; xx++)
                        planes[p][yy * s + xx] = (pix)clipp(SN(xx, yy) + tab[SN(xx, yy) >> (XO_DEPTH - 5)]);
                continue;
            }
            const int off[5] = { 0, prm->offset[0], prm->offset[1], prm->offset[2], prm->offset[3] };
            int dx0, dy0, dx1, dy1;
            eo_dirs(type, &dx0, &dy0, &dx1, &dy1);
            const int xs = (type != 1 && x0 == 0) ? 1 : x0, xe = (type != 1 && x1 == pw) ? pw - 1 : x1;
            const int ys = (type != 0 && y0 == 0) ? 1 : y0, ye = (type != 0 && y1 == ph) ? ph - 1 : y1;
            for (int yy = ys; yy < ye; yy++)
                for (int xx = xs; xx < xe; xx++)
                {
                    const int v = SN(xx, yy);
                    const int e = sgn(v - SN(xx + dx0, yy + dy0)) + sgn(v - SN(xx + dx1, yy + dy1)) + 2;
                    planes[p][yy * s + xx] = (pix)clipp(v + off[kEoClass[e]]);
                }
        }
#undef SN
        free(snap);
    }
}

void xo_sao_apply(int width, int height, int ctu_log2, void* y_, void* cb_, void* cr_, intptr_t stride,
                  intptr_t cstride, const xo_sao_param* params, int luma_on, int chroma_on)
{
    xo_sao_apply_csp(width, height, ctu_log2, y_, cb_, cr_, stride, cstride, params, luma_on, chroma_on, 1);
}

/* calcSaoStatsCu (sao.cpp:772-943) with saoCuStats{BO,E0..E3}_c (sao.cpp:1748-1916): per class the
 * sum of (source - deblocked) and the pixel count, over regions that leave out the not yet
 * deblocked right / bottom lines (skipR / skipB) unless the CTU touches the picture edge (E0 keeps
 * its bottom skip even there, sao.cpp:852) */
void xo_sao_stats_csp(int width, int height, int ctu_log2, int non_deblocked, const void* fy, const void* fcb,
                      const void* fcr, intptr_t fstride, intptr_t fcstride, const void* ry, const void* rcb,
                      const void* rcr, intptr_t rstride, intptr_t rcstride, int32_t* stats, int32_t* count, int csp)
{
    const int hs = csp == 3 ? 0 : 1, vs = csp == 1 ? 1 : 0;
    const int ctu = 1 << ctu_log2;
    const int wc = (width + ctu - 1) >> ctu_log2, hc = (height + ctu - 1) >> ctu_log2, nctu = wc * hc;
    const pix* fp[3] = { (const pix*)fy, (const pix*)fcb, (const pix*)fcr };
    const pix* rp[3] = { (const pix*)ry, (const pix*)rcb, (const pix*)rcr };
    /* (skipB, skipR) per type: E0..E3, BO (sao.cpp:825-925) */
    static const int kSkip[2][5][2] = { { { 4, 5 }, { 4, 5 }, { 4, 5 }, { 4, 5 }, { 4, 5 } },
                                        { { 3, 5 }, { 4, 4 }, { 4, 5 }, { 4, 5 }, { 3, 4 } } };
    memset(stats, 0, sizeof(int32_t) * nctu * 3 * 5 * 33);
    memset(count, 0, sizeof(int32_t) * nctu * 3 * 5 * 33);
    for (int c = 0; c < nctu; c++)
        for (int p = 0; p < 3; p++)
        {
            const intptr_t fs = p ? fcstride : fstride, rs = p ? rcstride : rstride;
            const int pw = p ? width >> hs : width, ph = p ? height >> vs : height;
            const int csw = p ? ctu >> hs : ctu, csh = p ? ctu >> vs : ctu;
            const int po = p ? 2 : 0;
            const int x0 = (c % wc) * csw, y0 = (c / wc) * csh;
            const int cw = (x0 + csw < pw ? x0 + csw : pw) - x0, ch = (y0 + csh < ph ? y0 + csh : ph) - y0;
            const int right = x0 + cw == pw, bottom = y0 + ch == ph;
            const pix* f = fp[p] + y0 * fs + x0;
            const pix* r = rp[p] + y0 * rs + x0;
            int32_t* st = stats + (c * 3 + p) * 5 * 33;
            int32_t* cn = count + (c * 3 + p) * 5 * 33;
            for (int t = 0; t < 5; t++)
            {
                const int sb = kSkip[!!non_deblocked][t][0], sr = kSkip[!!non_deblocked][t][1];
                int xs, xe, ys, ye;
                if (t == 4) { xs = 0; xe = right ? cw : cw - sr + po; ys = 0; ye = bottom ? ch : ch - sb + po; }
                else if (t == 0) { xs = !x0; xe = right ? cw - 1 : cw - sr + po; ys = 0; ye = ch - sb + po; }
                else if (t == 1) { xs = 0; xe = right ? cw : cw - sr + po; ys = !y0; ye = bottom ? ch - 1 : ch - sb + po; }
                else { xs = !x0; xe = right ? cw - 1 : cw - sr + po; ys = !y0; ye = bottom ? ch - 1 : ch - sb + po; }
                int dx0 = 0, dy0 = 0, dx1 = 0, dy1 = 0;
                if (t < 4) eo_dirs(t, &dx0, &dy0, &dx1, &dy1);
                for (int yy = ys; yy < ye; yy++)
                    for (int xx = xs; xx < xe; xx++)
                    {
                        const int v = r[yy * rs + xx];
                        const int d = (int)f[yy * fs + xx] - v;
                        int k;
                        if (t == 4)
                            k = 1 + (v >> (XO_DEPTH - 5));
                        else
                            k = kEoClass[sgn(v - r[(yy + dy0) * rs + xx + dx0]) + sgn(v - r[(yy + dy1) * rs + xx + dx1]) + 2];
                        st[t * 33 + k] += d;
                        cn[t * 33 + k]++;
                    }
            }
        }
}

void xo_sao_stats(int width, int height, int ctu_log2, int non_deblocked, const void* fy, const void* fcb,
                  const void* fcr, intptr_t fstride, intptr_t fcstride, const void* ry, const void* rcb,
                  const void* rcr, intptr_t rstride, intptr_t rcstride, int32_t* stats, int32_t* count)
{
    xo_sao_stats_csp(width, height, ctu_log2, non_deblocked, fy, fcb, fcr, fstride, fcstride, ry, rcb, rcr, rstride,
                     rcstride, stats, count, 1);
}

/* Deblock::s_tcTable / s_betaTable (deblock.cpp:523-535), g_chromaScale (constants.cpp:335-339) */
static const uint8_t kTc[54] = { 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2,
                                 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24 };
static const uint8_t kBeta[52] = { 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15,
                                   16, 17, 18, 20, 22, 24, 26, 28, 30, 32, 34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54,
                                   56, 58, 60, 62, 64 };
static const uint8_t kChromaScale[70] = { 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20,
                                          21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 33, 33, 34, 34, 35, 35,
                                          36, 36, 37, 37, 38, 39, 40, 41, 42, 43, 44, 45, 46, 47, 48, 49, 50, 51, 51,
                                          51, 51, 51, 51, 51, 51, 51, 51, 51, 51, 51 };

static int clip3i(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }

/* the edge marks deblockCU leaves in blockStrength before the bS decision (deblock.cpp:72-191):
 * the CU's own left / top edge bsCuEdge (2 inside the picture), its TU edges 2, its PU split 1 */
static int edge_mark(const xo_deblock_unit* u, int dir, int px, int py)
{
    const int pos = dir ? py : px;
    const int cu = 1 << u->cu_log2, tu = 1 << u->tu_log2;
    const int rel = pos & (cu - 1);
    if (!rel) return pos > 0 ? 2 : 0;
    if (!(pos & (tu - 1))) return 2;
    int pu = -1;
    switch (u->part)
    {
    case 1: if (dir) pu = cu >> 1; break;              /* 2NxN */
    case 2: if (!dir) pu = cu >> 1; break;             /* Nx2N */
    case 3: pu = cu >> 1; break;                       /* NxN */
    case 4: if (dir) pu = cu >> 2; break;              /* 2NxnU */
    case 5: if (dir) pu = cu - (cu >> 2); break;       /* 2NxnD */
    case 6: if (!dir) pu = cu >> 2; break;             /* nLx2N */
    case 7: if (!dir) pu = cu - (cu >> 2); break;      /* nRx2N */
    }
    return rel == pu ? 1 : 0;
}

/* Deblock::getBoundaryStrength (deblock.cpp:193-252).  m_refFrameList[0][-1] is the Slice's m_pps
 * (a non-null pointer no reference equals, MV kept); m_refFrameList[1][-1] is
 * m_refFrameList[0][MAX_NUM_REF] = NULL (MV zeroed). */
#define XO_KEY_L0_NONE ((int64_t)1 << 40)
#define XO_KEY_NULL ((int64_t)1 << 41)
static int64_t ref_key(const xo_deblock_params* prm, int list, int idx)
{
    return idx < 0 ? (list ? XO_KEY_NULL : XO_KEY_L0_NONE) : (int64_t)prm->ref_poc[list][idx];
}

static int mvdiff(const int16_t* a, const int16_t* b) { return abs(a[0] - b[0]) >= 4 || abs(a[1] - b[1]) >= 4; }

static int boundary_strength(const xo_deblock_unit* P, const xo_deblock_unit* Q, int mark, const xo_deblock_params* prm)
{
    if ((P->flags & 1) || (Q->flags & 1)) return 2;
    if (mark > 1 && ((Q->flags & 2) || (P->flags & 2))) return 1;
    static const int16_t zero[2] = { 0, 0 };
    const int64_t p0 = ref_key(prm, 0, P->ref_idx[0]), q0 = ref_key(prm, 0, Q->ref_idx[0]);
    const int16_t* mp0 = p0 != XO_KEY_NULL ? P->mv[0] : zero;
    const int16_t* mq0 = q0 != XO_KEY_NULL ? Q->mv[0] : zero;
    if (prm->is_p) return (p0 != q0 || mvdiff(mq0, mp0)) ? 1 : 0;
    const int64_t p1 = ref_key(prm, 1, P->ref_idx[1]), q1 = ref_key(prm, 1, Q->ref_idx[1]);
    const int16_t* mp1 = p1 != XO_KEY_NULL ? P->mv[1] : zero;
    const int16_t* mq1 = q1 != XO_KEY_NULL ? Q->mv[1] : zero;
    if ((p0 == q0 && p1 == q1) || (p0 == q1 && p1 == q0))
    {
        if (p0 != p1)
        {
            if (p0 == q0) return (mvdiff(mq0, mp0) || mvdiff(mq1, mp1)) ? 1 : 0;
            return (mvdiff(mq1, mp0) || mvdiff(mq0, mp1)) ? 1 : 0;
        }
        return ((mvdiff(mq0, mp0) || mvdiff(mq1, mp1)) && (mvdiff(mq1, mp0) || mvdiff(mq0, mp1))) ? 1 : 0;
    }
    return 1;
}

/* edgeFilterLuma (deblock.cpp:343-441) for one 4-line segment; src at line 0 on the Q side, `off`
 * across the edge, `step` along it.  pelFilterLumaStrong_c (loopfilter.cpp:141-162), pelFilterLuma
 * (deblock.cpp:283-326). */
static void filter_luma_seg(pix* src, intptr_t step, intptr_t off, int bs, int qp, int maskP, int maskQ,
                            const xo_deblock_params* prm)
{
    const int bd = XO_DEPTH - 8;
    const int beta = kBeta[clip3i(0, 51, qp + prm->beta_offset_div2 * 2)] << bd;
#define PX(l, k) ((int)src[(l) * step + (k) * off])
    const int dp0 = abs(PX(0, -3) - 2 * PX(0, -2) + PX(0, -1)), dq0 = abs(PX(0, 0) - 2 * PX(0, 1) + PX(0, 2));
    const int dp3 = abs(PX(3, -3) - 2 * PX(3, -2) + PX(3, -1)), dq3 = abs(PX(3, 0) - 2 * PX(3, 1) + PX(3, 2));
    const int d0 = dp0 + dq0, d3 = dp3 + dq3;
    if (d0 + d3 >= beta) return;
    const int tc = kTc[clip3i(0, 53, qp + 2 * (bs - 1) + prm->tc_offset_div2 * 2)] << bd;
    int sw = 2 * d0 < (beta >> 2) && 2 * d3 < (beta >> 2);
    for (int l = 0; l < 4 && sw; l += 3)
        sw = abs(PX(l, -4) - PX(l, -1)) + abs(PX(l, 3) - PX(l, 0)) < (beta >> 3) &&
             abs(PX(l, -1) - PX(l, 0)) < ((tc * 5 + 1) >> 1);
    if (sw)
    {
        const int tcP = (2 * tc) & maskP, tcQ = (2 * tc) & maskQ;
        for (int l = 0; l < 4; l++)
        {
            pix* s = src + l * step;
            const int m0 = s[-4 * off], m1 = s[-3 * off], m2 = s[-2 * off], m3 = s[-off], m4 = s[0], m5 = s[off],
                      m6 = s[2 * off], m7 = s[3 * off];
            s[-3 * off] = (pix)(clip3i(-tcP, tcP, ((2 * m0 + 3 * m1 + m2 + m3 + m4 + 4) >> 3) - m1) + m1);
            s[-2 * off] = (pix)(clip3i(-tcP, tcP, ((m1 + m2 + m3 + m4 + 2) >> 2) - m2) + m2);
            s[-off] = (pix)(clip3i(-tcP, tcP, ((m1 + 2 * m2 + 2 * m3 + 2 * m4 + m5 + 4) >> 3) - m3) + m3);
            s[0] = (pix)(clip3i(-tcQ, tcQ, ((m2 + 2 * m3 + 2 * m4 + 2 * m5 + m6 + 4) >> 3) - m4) + m4);
            s[off] = (pix)(clip3i(-tcQ, tcQ, ((m3 + m4 + m5 + m6 + 2) >> 2) - m5) + m5);
            s[2 * off] = (pix)(clip3i(-tcQ, tcQ, ((m3 + m4 + m5 + 3 * m6 + 2 * m7 + 4) >> 3) - m6) + m6);
        }
        return;
    }
    const int side = (beta + (beta >> 1)) >> 3;
    const int mP1 = (dp0 + dp3 < side ? -1 : 0) & maskP, mQ1 = (dq0 + dq3 < side ? -1 : 0) & maskQ;
    const int thr = tc * 10, tc2 = tc >> 1;
    for (int l = 0; l < 4; l++)
    {
        pix* s = src + l * step;
        const int m2 = s[-2 * off], m3 = s[-off], m4 = s[0], m5 = s[off];
        int delta = (9 * (m4 - m3) - 3 * (m5 - m2) + 8) >> 4;
        if (abs(delta) >= thr) continue;
        delta = clip3i(-tc, tc, delta);
        s[-off] = (pix)clipp(m3 + (delta & maskP));
        s[0] = (pix)clipp(m4 - (delta & maskQ));
        if (mP1)
        {
            const int m1 = s[-3 * off];
            s[-2 * off] = (pix)clipp(m2 + clip3i(-tc2, tc2, (((m1 + m3 + 1) >> 1) - m2 + delta) >> 1));
        }
        if (mQ1)
        {
            const int m6 = s[2 * off];
            s[off] = (pix)clipp(m5 + clip3i(-tc2, tc2, (((m6 + m4 + 1) >> 1) - m5 - delta) >> 1));
        }
    }
#undef PX
}

/* edgeFilterChroma (deblock.cpp:443-521) for one 4-line chroma segment of Cb and Cr (bS 2 only) */
static void filter_chroma_seg(pix* const cbcr[2], intptr_t step, intptr_t off, int qpA, int maskP, int maskQ,
                              const xo_deblock_params* prm, int csp)
{
    const int bd = XO_DEPTH - 8;
    for (int k = 0; k < 2; k++)
    {
        int qp = qpA + (k ? prm->cr_qp_offset : prm->cb_qp_offset);
        if (qp >= 30) qp = csp == 1 ? kChromaScale[qp] : (qp < 51 ? qp : 51);   /* QP_MAX_SPEC */
        const int tc = kTc[clip3i(0, 53, qp + 2 + prm->tc_offset_div2 * 2)] << bd;
        for (int l = 0; l < 4; l++)
        {
            pix* s = cbcr[k] + l * step;
            const int m2 = s[-2 * off], m3 = s[-off], m4 = s[0], m5 = s[off];
            const int delta = clip3i(-tc, tc, (((m4 - m3) * 4) + m2 - m5 + 4) >> 3);
            s[-off] = (pix)clipp(m3 + (delta & maskP));
            s[0] = (pix)clipp(m4 - (delta & maskQ));
        }
    }
}

void xo_deblock_csp(int width, int height, int ctu_log2, void* y_, void* cb_, void* cr_, intptr_t stride,
                    intptr_t cstride, const xo_deblock_unit* units, intptr_t us, const xo_deblock_params* prm, int csp)
{
    const int hs = csp == 3 ? 0 : 1, vs = csp == 1 ? 1 : 0;
    (void)ctu_log2;   /* the per-CTU order of the reference is equivalent to all-vertical-then-all-horizontal */
    pix* Y = (pix*)y_;
    pix* C[2] = { (pix*)cb_, (pix*)cr_ };
    const int wu = width >> 2, hu = height >> 2;
    for (int dir = 0; dir < 2; dir++)
    {
        /* luma: every 4-line segment of an edge on the 8x8 grid */
        for (int uy = 0; uy < hu; uy++)
            for (int ux = 0; ux < wu; ux++)
            {
                if (dir ? (uy & 1) : (ux & 1)) continue;
                const xo_deblock_unit* Q = &units[uy * us + ux];
                const int mark = edge_mark(Q, dir, 4 * ux, 4 * uy);
                if (!mark) continue;
                const xo_deblock_unit* P = dir ? Q - us : Q - 1;
                const int bs = boundary_strength(P, Q, mark, prm);
                int maskP = -1, maskQ = -1;
                if (prm->tq_bypass_enabled)
                {
                    maskP = (P->flags & 4) ? 0 : -1;
                    maskQ = (Q->flags & 4) ? 0 : -1;
                    if (!(maskP | maskQ)) continue;
                }
                const int qp = (P->qp + Q->qp + 1) >> 1;
                if (bs)
                    filter_luma_seg(Y + 4 * uy * stride + 4 * ux, dir ? 1 : stride, dir ? stride : 1, bs, qp, maskP,
                                    maskQ, prm);
                /* chroma (deblock.cpp:104-113, 443-521): edges on the 8x8 grid of the chroma plane; one
                   4-line chroma segment per (1 << shift along the edge) luma units */
                const int across = dir ? vs : hs, along = dir ? hs : vs;
                if (bs == 2 && !(((4 * (dir ? uy : ux)) >> across) & 7) && !((dir ? ux : uy) & ((1 << along) - 1)))
                {
                    const intptr_t o = (intptr_t)((4 * uy) >> vs) * cstride + ((4 * ux) >> hs);
                    pix* const cbcr[2] = { C[0] + o, C[1] + o };
                    filter_chroma_seg(cbcr, dir ? 1 : cstride, dir ? cstride : 1, qp, maskP, maskQ, prm, csp);
                }
            }
    }
}

void xo_deblock(int width, int height, int ctu_log2, void* y_, void* cb_, void* cr_, intptr_t stride,
                intptr_t cstride, const xo_deblock_unit* units, intptr_t us, const xo_deblock_params* prm)
{
    xo_deblock_csp(width, height, ctu_log2, y_, cb_, cr_, stride, cstride, units, us, prm, 1);
}

/* ======================================================= f1 cuTree propagation */

/* (int) of a double as x86-64 cvttsd2si: truncation, INT_MIN when out of range or NaN */
static int xo_cvt_trunc(double v)
{
    if (!(v > -2147483649.0 && v < 2147483648.0)) return INT32_MIN;
    return (int)v;
}

/* pixel.cpp:846-872 estimateCUPropagateCost (the C propagateCost primitive) */
static void xo_propagate_cost_row(int* dst, const uint16_t* in, const int32_t* intra, const uint16_t* inter,
                                  const int32_t* invq, double fps_factor, int len)
{
    const double fps = fps_factor / 256;
    for (int i = 0; i < len; i++)
    {
        const int intraCost = intra[i];
        const int ic = inter[i] & ((1 << 14) - 1);
        const int interCost = intra[i] < ic ? intra[i] : ic;
        const double propagateIntra = (double)mul_wrap(intraCost, invq[i]);
        const double amount = (double)in[i] + propagateIntra * fps;
        const double num = (double)(intraCost - interCost);
        const double denom = (double)intraCost;
        dst[i] = xo_cvt_trunc(amount * num / denom + 0.5);
    }
}

static double xo_clip_duration(double f) { return f < 0.01 ? 0.01 : f > 1.00 ? 1.00 : f; }   /* ratecontrol.h:45-47 */

static void xo_clip_add(uint16_t* s, int x)
{
    const int v = (int)*s + x;
    *s = (uint16_t)(v < 65535 ? v : 65535);
}

/* slicetype.cpp:1738-1836 */
void xo_cutree_propagate(int wcu, int hcu, int b_p0, int p1_b, int referenced, int weighted_bipred,
                         int fps_num, int fps_den, double avg_duration, uint16_t* propagate_b,
                         const int32_t* intra_cost, const uint16_t* lowres_costs, const int32_t* inv_q,
                         const int32_t* mvs0, const int32_t* mvs1, uint16_t* ref0, uint16_t* ref1)
{
    const int p0 = 0, b = b_p0, p1 = b_p0 + p1_b;
    uint16_t* refCosts[2] = { ref0, ref1 };
    const int32_t distScale = (((b - p0) << 8) + ((p1 - p0) >> 1)) / (p1 - p0);
    const int32_t bw = weighted_bipred ? 64 - (distScale >> 2) : 32;
    const int32_t bipredWeights[2] = { bw, 64 - bw };
    const int32_t* mvs[2] = { mvs0, mvs1 };
    const double fpsFactor = xo_clip_duration((double)fps_den / fps_num) / xo_clip_duration(avg_duration);
    int* scratch = (int*)calloc((size_t)wcu, sizeof(int));
    if (!referenced) memset(propagate_b, 0, (size_t)wcu * sizeof(uint16_t));
    const uint16_t* prop = propagate_b;
    for (int by = 0; by < hcu; by++)
    {
        int cu = by * wcu;
        xo_propagate_cost_row(scratch, prop, intra_cost + cu, lowres_costs + cu, inv_q + cu, fpsFactor, wcu);
        if (referenced) prop += wcu;
        for (int bx = 0; bx < wcu; bx++, cu++)
        {
            const int amount = scratch[bx];
            if (amount <= 0) continue;
            const int used = lowres_costs[cu] >> 14;
            for (int l = 0; l < 2; l++)
            {
                if (!((used >> l) & 1)) continue;
                int la = amount;
                if (used == 3) la = (int32_t)((uint32_t)mul_wrap(la, bipredWeights[l]) + 32u) >> 6;
                const int32_t mv = mvs[l][cu];
                if (!mv)
                {
                    xo_clip_add(&refCosts[l][cu], la);
                    continue;
                }
                const int x = (int16_t)(mv & 0xffff), y = (int16_t)((uint32_t)mv >> 16);
                const int cux = (x >> 5) + bx, cuy = (y >> 5) + by;
                const int i0 = cux + cuy * wcu, fx = x & 31, fy = y & 31;
                const int w[4] = { (32 - fy) * (32 - fx), (32 - fy) * fx, fy * (32 - fx), fy * fx };
                const int dx[4] = { 0, 1, 0, 1 }, dy[4] = { 0, 0, 1, 1 };
                for (int k = 0; k < 4; k++)
                {
                    const int cx = cux + dx[k], cy = cuy + dy[k];
                    if (cx < wcu && cy < hcu && cx >= 0 && cy >= 0)
                        xo_clip_add(&refCosts[l][i0 + dx[k] + dy[k] * wcu],
                                    (int32_t)((uint32_t)mul_wrap(la, w[k]) + 512u) >> 10);
                }
            }
        }
    }
    free(scratch);
}

/* ======================================================= f1 weighted-prediction analysis */

/* pixel.cpp:463-488 weight_pp_c */
static void xo_weight_pp(const pix* src, pix* dst, intptr_t stride, int width, int height, int w0, int round,
                         int shift, int offset)
{
    const int correction = 14 - XO_DEPTH;
    for (int y = 0; y < height; y++, src += stride, dst += stride)
        for (int x = 0; x < width; x++)
        {
            const int16_t val = (int16_t)shl_wrap(src[x], correction);
            const int v = ((w0 * val + round) >> shift) + offset;
            dst[x] = (pix)(v < 0 ? 0 : v > PMAX ? PMAX : v);
        }
}

/* slicetype.cpp:338-368 weightCostLuma */
static uint32_t xo_weight_cost_luma(int width, int lines, intptr_t stride, int padded_lines, intptr_t padoff,
                                    const pix* fenc, const pix* ref_buf0, const int32_t* intra, pix* wbuf0,
                                    int present, int w0, int denom, int offset)
{
    const pix* src = ref_buf0 + padoff;
    if (present)
    {
        const int off = offset << (XO_DEPTH - 8), round = denom ? 1 << (denom - 1) : 0, corr = 14 - XO_DEPTH;
        xo_weight_pp(ref_buf0, wbuf0, stride, (int)stride, padded_lines, w0, round << corr, denom + corr, off);
        src = wbuf0 + padoff;
    }
    uint32_t cost = 0;
    int mb = 0;
    for (int y = 0; y < lines; y += 8)
        for (int x = 0; x < width; x += 8, mb++)
        {
            const int satd = xo_satd(8, 8, src + y * stride + x, stride, fenc + y * stride + x, stride);
            cost += (uint32_t)(satd < intra[mb] ? satd : intra[mb]);
        }
    return cost;
}

/* slicetype.cpp:391-495 */
void xo_weights_analyse(int width, int lines, intptr_t stride, int padded_lines, intptr_t pad_offset,
                        const void* fenc_plane, const void* const* ref_buf, const int32_t* intra_cost,
                        void* const* wbuf, uint64_t fenc_ssd, uint64_t ref_ssd, uint64_t fenc_sum,
                        uint64_t ref_sum, int* out, double* cost_delta)
{
    const float epsilon = 1.f / 128.f;
    const pix* fenc = (const pix*)fenc_plane;
    out[0] = 0;
    float guessScale;
    if (fenc_ssd && ref_ssd) guessScale = sqrtf((float)fenc_ssd / ref_ssd);
    else guessScale = 1.0f;
    const float fencMean = (float)fenc_sum / (lines * width) / (1 << (XO_DEPTH - 8));
    const float refMean = (float)ref_sum / (lines * width) / (1 << (XO_DEPTH - 8));
    if (fabsf(refMean - fencMean) < 0.5f && fabsf(1.f - guessScale) < epsilon) return;

    /* WeightParam::setFromWeightAndOffset(w, 0, 7, true) (slice.h:293-305) */
    int mindenom = 7, minscale = (int)(guessScale * 128 + 0.5f);
    while (mindenom > 0 && minscale > 127) { mindenom--; minscale >>= 1; }
    if (minscale > 127) minscale = 127;
    int minoff = 0, found = 0;
    unsigned int minscore, origscore;
    origscore = minscore = xo_weight_cost_luma(width, lines, stride, padded_lines, pad_offset, fenc,
                                               (const pix*)ref_buf[0], intra_cost, (pix*)wbuf[0], 0, 0, 0, 0);
    if (!minscore) return;
    int curScale = minscale;
    int curOffset = (int)(fencMean - refMean * curScale / (1 << mindenom) + 0.5f);
    if (curOffset < -128 || curOffset > 127)
    {
        curOffset = curOffset < -128 ? -128 : 127;
        curScale = (int)((1 << mindenom) * (fencMean - curOffset) / refMean + 0.5f);
        curScale = curScale < 0 ? 0 : curScale > 127 ? 127 : curScale;
    }
    const unsigned int s = xo_weight_cost_luma(width, lines, stride, padded_lines, pad_offset, fenc,
                                               (const pix*)ref_buf[0], intra_cost, (pix*)wbuf[0], 1, curScale,
                                               mindenom, curOffset);
    if (s < minscore) { minscore = s; minscale = curScale; minoff = curOffset; found = 1; }
    while (mindenom > 0 && !(minscale & 1)) { mindenom--; minscale >>= 1; }
    if (!found || (minscale == 1 << mindenom && minoff == 0) || (float)minscore / origscore > 0.998f) return;
    *cost_delta = minscore / origscore;
    const int off = minoff << (XO_DEPTH - 8), round = mindenom ? 1 << (mindenom - 1) : 0, corr = 14 - XO_DEPTH;
    for (int i = 0; i < 4; i++)
        xo_weight_pp((const pix*)ref_buf[i], (pix*)wbuf[i], stride, (int)stride, padded_lines, minscale,
                     round << corr, mindenom + corr, off);
    out[0] = 1;
    out[1] = minscale;
    out[2] = mindenom;
    out[3] = minoff;
}
