/* ref_shim.cpp — exposes the reference x265 1.9 C primitive table through the
 * flat oracle API (x265_oracle.h).
 *
 * TEST INFRASTRUCTURE ONLY.  Compiled together with the reference's own
 * sources (oracle/Makefile, target `ref`) into oracle/_ref/libx265ref{8,10}.so;
 * the reference sources themselves are never copied into this repository.
 *
 * The table is set up exactly as TestBench's `cprim` is
 * (test/testbench.cpp:153-156): setupCPrimitives + setupAliasPrimitives, so
 * intra_pred_allangs stays non-NULL.  Every xo_* call below resolves the
 * (width, height) it is given to the table entry that the reference encoder
 * would call for a block of that shape — luma tables first, then the 4:2:0 and
 * 4:2:2 chroma tables (primitives.h:345-380) — and aborts if no entry exists.
 */
#include "common.h"
#include "primitives.h"
#include "quant.h"
#include "cudata.h"
#include "slice.h"
#include "scalinglist.h"
#include "entropy.h"
#include "lowres.h"
#include "slicetype.h"
#include "bitcost.h"
#include "motion.h"
#include "picyuv.h"
#include "frame.h"
#include "framedata.h"
#include "deblock.h"
#include "sao.h"
#include "x265_oracle.h"

#include <pthread.h>

#include <cstdio>
#include <cstdlib>

using namespace X265_NS;

namespace {

EncoderPrimitives g_tab;
pthread_once_t g_tab_once = PTHREAD_ONCE_INIT;

void init_tab()
{
    memset(&g_tab, 0, sizeof(g_tab));
    setupCPrimitives(g_tab);
    setupAliasPrimitives(g_tab);
}

/* filled once, thread-safely: the CPU baseline calls in from many host threads at once */
EncoderPrimitives& tab()
{
    pthread_once(&g_tab_once, init_tab);
    return g_tab;
}

[[noreturn]] void die(const char* what, int w, int h)
{
    fprintf(stderr, "ref_shim: no reference entry for %s %dx%d\n", what, w, h);
    abort();
}

const int kPuW[NUM_PU_SIZES] = { 4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 12, 16, 4, 32, 24, 32, 8, 64, 48, 64, 16 };
const int kPuH[NUM_PU_SIZES] = { 4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 12, 16, 4, 16, 24, 32, 8, 32, 48, 64, 16, 64 };

/* PU-indexed entry lookup: luma, then chroma 4:2:0 (w/2,h/2), then 4:2:2 (w/2,h) */
struct PuRef { int csp; int part; };

PuRef findPu(int w, int h, bool allowLuma, bool allowChroma)
{
    if (allowLuma)
        for (int p = 0; p < NUM_PU_SIZES; p++)
            if (kPuW[p] == w && kPuH[p] == h) return PuRef{ -1, p };
    if (allowChroma)
    {
        for (int p = 0; p < NUM_PU_SIZES; p++)
            if (kPuW[p] / 2 == w && kPuH[p] / 2 == h) return PuRef{ X265_CSP_I420, p };
        for (int p = 0; p < NUM_PU_SIZES; p++)
            if (kPuW[p] / 2 == w && kPuH[p] == h) return PuRef{ X265_CSP_I422, p };
    }
    return PuRef{ -2, -1 };
}

/* CU-indexed lookup: luma square (4<<i), 4:2:0 square (2<<i), 4:2:2 (2<<i)x(4<<i) */
PuRef findCu(int w, int h)
{
    for (int i = 0; i < NUM_CU_SIZES; i++)
        if (w == (4 << i) && h == (4 << i)) return PuRef{ -1, i };
    for (int i = 0; i < NUM_CU_SIZES; i++)
        if (w == (2 << i) && h == (2 << i)) return PuRef{ X265_CSP_I420, i };
    for (int i = 0; i < NUM_CU_SIZES; i++)
        if (w == (2 << i) && h == (4 << i)) return PuRef{ X265_CSP_I422, i };
    return PuRef{ -2, -1 };
}

int log2i(int n) { int l = 0; while ((1 << l) < n) l++; return l; }

pixelcmp_t satdFor(int w, int h)
{
    PuRef r = findPu(w, h, true, true);
    pixelcmp_t f = NULL;
    if (r.csp == -1) f = tab().pu[r.part].satd;
    else if (r.csp >= 0) f = tab().chroma[r.csp].pu[r.part].satd;
    if (!f) die("satd", w, h);
    return f;
}

} // namespace

extern "C" {

int xo_depth(void) { return X265_DEPTH; }

int xo_sad(int w, int h, const void* a, intptr_t sa, const void* b, intptr_t sb)
{
    PuRef r = findPu(w, h, true, false);
    if (r.csp != -1) die("sad", w, h);
    return tab().pu[r.part].sad((const pixel*)a, sa, (const pixel*)b, sb);
}

void xo_sad_x3(int w, int h, const void* fenc, const void* r0, const void* r1, const void* r2, intptr_t rs, int32_t* res)
{
    PuRef r = findPu(w, h, true, false);
    if (r.csp != -1) die("sad_x3", w, h);
    tab().pu[r.part].sad_x3((const pixel*)fenc, (const pixel*)r0, (const pixel*)r1, (const pixel*)r2, rs, res);
}

void xo_sad_x4(int w, int h, const void* fenc, const void* r0, const void* r1, const void* r2, const void* r3, intptr_t rs, int32_t* res)
{
    PuRef r = findPu(w, h, true, false);
    if (r.csp != -1) die("sad_x4", w, h);
    tab().pu[r.part].sad_x4((const pixel*)fenc, (const pixel*)r0, (const pixel*)r1, (const pixel*)r2, (const pixel*)r3, rs, res);
}

int xo_satd(int w, int h, const void* a, intptr_t sa, const void* b, intptr_t sb)
{
    return satdFor(w, h)((const pixel*)a, sa, (const pixel*)b, sb);
}

int xo_sa8d(int w, int h, const void* a, intptr_t sa, const void* b, intptr_t sb)
{
    PuRef r = findCu(w, h);
    pixelcmp_t f = NULL;
    if (r.csp == -1) f = tab().cu[r.part].sa8d;
    else if (r.csp >= 0) f = tab().chroma[r.csp].cu[r.part].sa8d;
    if (!f) die("sa8d", w, h);
    return f((const pixel*)a, sa, (const pixel*)b, sb);
}

uint64_t xo_sse_pp(int w, int h, const void* a, intptr_t sa, const void* b, intptr_t sb)
{
    PuRef r = findCu(w, h);
    pixel_sse_t f = NULL;
    if (r.csp == -1) f = tab().cu[r.part].sse_pp;
    else if (r.csp >= 0) f = tab().chroma[r.csp].cu[r.part].sse_pp;
    if (!f) die("sse_pp", w, h);
    return (uint64_t)f((const pixel*)a, sa, (const pixel*)b, sb);
}

uint64_t xo_sse_ss(int w, int h, const int16_t* a, intptr_t sa, const int16_t* b, intptr_t sb)
{
    PuRef r = findCu(w, h);
    if (r.csp != -1 || !tab().cu[r.part].sse_ss) die("sse_ss", w, h);
    return (uint64_t)tab().cu[r.part].sse_ss(a, sa, b, sb);
}

uint64_t xo_ssd_s(int n, const int16_t* a, intptr_t sa)
{
    return (uint64_t)tab().cu[log2i(n) - 2].ssd_s(a, sa);
}

int xo_psy_cost_pp(int n, const void* src, intptr_t ss, const void* rec, intptr_t rs)
{
    return tab().cu[log2i(n) - 2].psy_cost_pp((const pixel*)src, ss, (const pixel*)rec, rs);
}

uint64_t xo_var(int n, const void* p, intptr_t s)
{
    return tab().cu[log2i(n) - 2].var((const pixel*)p, s);
}

void xo_interp(int op, int taps, int w, int h, const void* src, intptr_t ss, void* dst, intptr_t ds, int coeffIdx, int extra)
{
    EncoderPrimitives& p = tab();
    const pixel* sp = (const pixel*)src;
    const int16_t* s16 = (const int16_t*)src;
    pixel* dp = (pixel*)dst;
    int16_t* d16 = (int16_t*)dst;

    if (taps == 8 || op == XO_P2S)
    {
        PuRef r = findPu(w, h, true, op == XO_P2S);
        if (r.csp == -1)
        {
            EncoderPrimitives::PU& u = p.pu[r.part];
            switch (op)
            {
            case XO_HPP:  u.luma_hpp(sp, ss, dp, ds, coeffIdx); return;
            case XO_HPS:  u.luma_hps(sp, ss, d16, ds, coeffIdx, extra); return;
            case XO_VPP:  u.luma_vpp(sp, ss, dp, ds, coeffIdx); return;
            case XO_VPS:  u.luma_vps(sp, ss, d16, ds, coeffIdx); return;
            case XO_VSP:  u.luma_vsp(s16, ss, dp, ds, coeffIdx); return;
            case XO_VSS:  u.luma_vss(s16, ss, d16, ds, coeffIdx); return;
            case XO_HVPP: u.luma_hvpp(sp, ss, dp, ds, coeffIdx, extra); return;
            case XO_P2S:  u.convert_p2s(sp, ss, d16, ds); return;
            }
        }
        if (r.csp >= 0 && op == XO_P2S)
        {
            p.chroma[r.csp].pu[r.part].p2s(sp, ss, d16, ds);
            return;
        }
        die("luma interp", w, h);
    }

    /* 4-tap: chroma 4:2:0, then 4:2:2, then 4:4:4 (luma-sized) */
    EncoderPrimitives::Chroma::PUChroma* c = NULL;
    PuRef r = findPu(w, h, false, true);
    if (r.csp >= 0) c = &p.chroma[r.csp].pu[r.part];
    else
    {
        r = findPu(w, h, true, false);
        if (r.csp == -1) c = &p.chroma[X265_CSP_I444].pu[r.part];
    }
    if (!c) die("chroma interp", w, h);
    switch (op)
    {
    case XO_HPP: c->filter_hpp(sp, ss, dp, ds, coeffIdx); return;
    case XO_HPS: c->filter_hps(sp, ss, d16, ds, coeffIdx, extra); return;
    case XO_VPP: c->filter_vpp(sp, ss, dp, ds, coeffIdx); return;
    case XO_VPS: c->filter_vps(sp, ss, d16, ds, coeffIdx); return;
    case XO_VSP: c->filter_vsp(s16, ss, dp, ds, coeffIdx); return;
    case XO_VSS: c->filter_vss(s16, ss, d16, ds, coeffIdx); return;
    }
    die("chroma interp op", w, h);
}

void xo_dct(int kind, int n, const int16_t* src, int16_t* dst, intptr_t stride)
{
    EncoderPrimitives& p = tab();
    int i = log2i(n) - 2;
    switch (kind)
    {
    case XO_DCT:  p.cu[i].dct(src, dst, stride); return;
    case XO_IDCT: p.cu[i].idct(src, dst, stride); return;
    case XO_DST:  p.dst4x4(src, dst, stride); return;
    case XO_IDST: p.idst4x4(src, dst, stride); return;
    }
}

uint32_t xo_quant(const int16_t* coef, const int32_t* qcoef, int32_t* deltaU, int16_t* qout, int qBits, int add, int numCoeff)
{
    return tab().quant(coef, qcoef, deltaU, qout, qBits, add, numCoeff);
}

uint32_t xo_nquant(const int16_t* coef, const int32_t* qcoef, int16_t* qout, int qBits, int add, int numCoeff)
{
    return tab().nquant(coef, qcoef, qout, qBits, add, numCoeff);
}

void xo_dequant_normal(const int16_t* q, int16_t* coef, int num, int scale, int shift)
{
    tab().dequant_normal(q, coef, num, scale, shift);
}

void xo_dequant_scaling(const int16_t* q, const int32_t* dq, int16_t* coef, int num, int per, int shift)
{
    tab().dequant_scaling(q, dq, coef, num, per, shift);
}

void xo_intra_filter(int n, const void* ref, void* filt)
{
    tab().cu[log2i(n) - 2].intra_filter((const pixel*)ref, (pixel*)filt);
}

void xo_intra_pred(int n, int mode, void* dst, intptr_t ds, const void* src, int bFilter)
{
    tab().cu[log2i(n) - 2].intra_pred[mode]((pixel*)dst, ds, (const pixel*)src, mode, bFilter);
}

void xo_intra_allangs(int n, void* dst, void* ref, void* filt, int bLuma)
{
    tab().cu[log2i(n) - 2].intra_pred_allangs((pixel*)dst, (pixel*)ref, (pixel*)filt, bLuma);
}

void xo_calcresidual(int n, const void* fenc, const void* pred, int16_t* res, intptr_t stride)
{
    tab().cu[log2i(n) - 2].calcresidual((const pixel*)fenc, (const pixel*)pred, res, stride);
}

#define CU_ENTRY(field, what)                                                      \
    PuRef r = findCu(w, h);                                                        \
    EncoderPrimitives& p = tab();                                                  \
    if (r.csp == -2) die(what, w, h);

void xo_sub_ps(int w, int h, int16_t* d, intptr_t ds, const void* a, const void* b, intptr_t sa, intptr_t sb)
{
    CU_ENTRY(sub_ps, "sub_ps");
    pixel_sub_ps_t f = r.csp == -1 ? p.cu[r.part].sub_ps : p.chroma[r.csp].cu[r.part].sub_ps;
    f(d, ds, (const pixel*)a, (const pixel*)b, sa, sb);
}

void xo_add_ps(int w, int h, void* d, intptr_t ds, const void* a, const int16_t* b, intptr_t sa, intptr_t sb)
{
    CU_ENTRY(add_ps, "add_ps");
    pixel_add_ps_t f = r.csp == -1 ? p.cu[r.part].add_ps : p.chroma[r.csp].cu[r.part].add_ps;
    f((pixel*)d, ds, (const pixel*)a, b, sa, sb);
}

void xo_copy_sp(int w, int h, void* d, intptr_t ds, const int16_t* s, intptr_t ss)
{
    CU_ENTRY(copy_sp, "copy_sp");
    copy_sp_t f = r.csp == -1 ? p.cu[r.part].copy_sp : p.chroma[r.csp].cu[r.part].copy_sp;
    f((pixel*)d, ds, s, ss);
}

void xo_copy_ps(int w, int h, int16_t* d, intptr_t ds, const void* s, intptr_t ss)
{
    CU_ENTRY(copy_ps, "copy_ps");
    copy_ps_t f = r.csp == -1 ? p.cu[r.part].copy_ps : p.chroma[r.csp].cu[r.part].copy_ps;
    f(d, ds, (const pixel*)s, ss);
}

void xo_copy_ss(int w, int h, int16_t* d, intptr_t ds, const int16_t* s, intptr_t ss)
{
    CU_ENTRY(copy_ss, "copy_ss");
    copy_ss_t f = r.csp == -1 ? p.cu[r.part].copy_ss : p.chroma[r.csp].cu[r.part].copy_ss;
    f(d, ds, s, ss);
}

void xo_addavg(int w, int h, const int16_t* a, const int16_t* b, void* d, intptr_t sa, intptr_t sb, intptr_t ds)
{
    PuRef r = findPu(w, h, true, true);
    if (r.csp == -2) die("addAvg", w, h);
    addAvg_t f = r.csp == -1 ? tab().pu[r.part].addAvg : tab().chroma[r.csp].pu[r.part].addAvg;
    f(a, b, (pixel*)d, sa, sb, ds);
}

void xo_pixelavg(int w, int h, void* d, intptr_t ds, const void* a, intptr_t sa, const void* b, intptr_t sb)
{
    PuRef r = findPu(w, h, true, false);
    if (r.csp != -1) die("pixelavg_pp", w, h);
    tab().pu[r.part].pixelavg_pp((pixel*)d, ds, (const pixel*)a, sa, (const pixel*)b, sb, 32);
}

void xo_copy_pp(int w, int h, void* d, intptr_t ds, const void* s, intptr_t ss)
{
    PuRef r = findPu(w, h, true, true);
    if (r.csp == -2) die("copy_pp", w, h);
    copy_pp_t f = r.csp == -1 ? tab().pu[r.part].copy_pp : tab().chroma[r.csp].pu[r.part].copy_pp;
    f((pixel*)d, ds, (const pixel*)s, ss);
}

void xo_blockfill_s(int n, int16_t* d, intptr_t ds, int16_t v)
{
    tab().cu[log2i(n) - 2].blockfill_s(d, ds, v);
}

void xo_cpy2Dto1D_shl(int n, int16_t* d, const int16_t* s, intptr_t ss, int shift)
{
    tab().cu[log2i(n) - 2].cpy2Dto1D_shl(d, s, ss, shift);
}

void xo_cpy2Dto1D_shr(int n, int16_t* d, const int16_t* s, intptr_t ss, int shift)
{
    tab().cu[log2i(n) - 2].cpy2Dto1D_shr(d, s, ss, shift);
}

void xo_cpy1Dto2D_shl(int n, int16_t* d, const int16_t* s, intptr_t ds, int shift)
{
    tab().cu[log2i(n) - 2].cpy1Dto2D_shl(d, s, ds, shift);
}

void xo_cpy1Dto2D_shr(int n, int16_t* d, const int16_t* s, intptr_t ds, int shift)
{
    tab().cu[log2i(n) - 2].cpy1Dto2D_shr(d, s, ds, shift);
}

int xo_count_nonzero(int n, const int16_t* q)
{
    return tab().cu[log2i(n) - 2].count_nonzero(q);
}

uint32_t xo_copy_cnt(int n, int16_t* coeff, const int16_t* res, intptr_t rs)
{
    return tab().cu[log2i(n) - 2].copy_cnt(coeff, res, rs);
}

void xo_transpose(int n, void* d, const void* s, intptr_t ss)
{
    tab().cu[log2i(n) - 2].transpose((pixel*)d, (const pixel*)s, ss);
}

void xo_denoise_dct(int16_t* coef, uint32_t* resSum, const uint16_t* offset, int num)
{
    tab().denoiseDct(coef, resSum, offset, num);
}

} // extern "C"

/* f3: the reference's own Quant::transformNxN / invtransformNxN (quant.cpp:397-546),
 * chained exactly as Search::residualTransformQuantIntra does (search.cpp:689-706).
 * The Quant object is set up as the encoder sets it up for --preset medium (no RDOQ,
 * flat scaling lists: Encoder::create -> ScalingList::init/setupQuantMatrices,
 * Quant::init); the CU carries only the fields those functions read
 * (cudata.h:165-197): slice (type, PPS sign hiding), prediction mode, intra
 * directions and lossless flag.  The caller's scan type is expressed as an intra
 * direction that getTUEntropyCodingParameters maps back to it (cudata.cpp:2038-2041). */
namespace {

struct TuQuant : public Quant
{
    void setQp(int ttype, int qpScaled)
    {
        m_qpParam[ttype].qp = MAX_INT;
        m_qpParam[ttype].setQpParam(qpScaled);
    }
};

struct TuContext
{
    ScalingList sl;
    Entropy entropy;
    TuQuant quant;
    TuContext()
    {
        sl.init();
        sl.m_bEnabled = false;
        sl.m_bDataPresent = false;
        sl.setupQuantMatrices();
        quant.init(0, 0.0, sl, entropy);
    }
};

pthread_once_t g_prim_once = PTHREAD_ONCE_INIT;
__thread int g_me_qp = 32;
void init_global_prims()
{
    /* Quant calls through the process-global table, as in the encoder */
    setupCPrimitives(primitives);
    setupAliasPrimitives(primitives);
}

} // namespace

extern "C" {

uint32_t xo_tu_pipeline(int log2, int is_luma, int is_intra, int i_slice, int sign_hide, int qp, int scan,
                        const void* fenc, intptr_t fs, const void* pred, intptr_t ps,
                        int16_t* resi, intptr_t rs, int16_t* coeff, void* recon, intptr_t rcs)
{
    pthread_once(&g_prim_once, init_global_prims);
    static __thread TuContext* ctx = NULL;
    if (!ctx) ctx = new TuContext();

    PPS pps;
    memset(&pps, 0, sizeof(pps));
    pps.bSignHideEnabled = !!sign_hide;
    SPS sps;
    memset(&sps, 0, sizeof(sps));
    sps.quadtreeTULog2MaxSize = 5;
    Slice slice;
    slice.m_pps = &pps;
    slice.m_sps = &sps;
    slice.m_sliceType = i_slice ? I_SLICE : P_SLICE;

    static const uint8_t kDirOfScan[3] = { DC_IDX, 26, 10 };   /* DIAG, HOR (22..30), VER (6..14) */
    uint8_t predMode = is_intra ? MODE_INTRA : MODE_INTER, dir = kDirOfScan[scan], bypass = 0;
    CUData cu;
    cu.m_slice = &slice;
    cu.m_chromaFormat = X265_CSP_I420;
    cu.m_hChromaShift = 1;
    cu.m_predMode = &predMode;
    cu.m_lumaIntraDir = &dir;
    cu.m_chromaIntraDir = &dir;
    cu.m_tqBypass = &bypass;

    const TextType ttype = is_luma ? TEXT_LUMA : TEXT_CHROMA_U;
    ctx->quant.setQp(ttype, qp);

    /* the encoder's Yuv buffers share one stride (search.cpp:668-671): stage at stride n */
    const int n = 1 << log2;
    ALIGN_VAR_32(pixel, f[32 * 32]);
    ALIGN_VAR_32(pixel, p[32 * 32]);
    ALIGN_VAR_32(pixel, rec[32 * 32]);
    ALIGN_VAR_32(int16_t, r[32 * 32]);
    ALIGN_VAR_32(coeff_t, c[32 * 32]);
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++)
        {
            f[y * n + x] = ((const pixel*)fenc)[y * fs + x];
            p[y * n + x] = ((const pixel*)pred)[y * ps + x];
        }
    const int sizeIdx = log2 - 2;
    primitives.cu[sizeIdx].calcresidual(f, p, r, n);
    uint32_t numSig = ctx->quant.transformNxN(cu, f, n, r, n, c, log2, ttype, 0, false);
    if (numSig)
    {
        ctx->quant.invtransformNxN(cu, r, n, c, log2, ttype, !!is_intra, false, numSig);
        primitives.cu[sizeIdx].add_ps(rec, n, p, r, n, n);
    }
    else
        primitives.cu[sizeIdx].copy_pp(rec, n, p, n);
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++)
        {
            resi[y * rs + x] = r[y * n + x];
            ((pixel*)recon)[y * rcs + x] = rec[y * n + x];
        }
    memcpy(coeff, c, sizeof(coeff_t) * n * n);
    return numSig;
}

/* f1: the reference's own lowres plane generation — the two calls Lowres::init makes
 * (lowres.cpp:151-162) on the planes of a Lowres allocated like Lowres::create */
void xo_lowres_init(int width, int lines, const void* src, intptr_t ss, void* p0, void* p1, void* p2, void* p3,
                    intptr_t ls, int mx, int my)
{
    pthread_once(&g_prim_once, init_global_prims);
    primitives.frameInitLowres((const pixel*)src, (pixel*)p0, (pixel*)p1, (pixel*)p2, (pixel*)p3, ss, ls, width, lines);
    extendPicBorder((pixel*)p0, ls, width, lines, mx, my);
    extendPicBorder((pixel*)p1, ls, width, lines, mx, my);
    extendPicBorder((pixel*)p2, ls, width, lines, mx, my);
    extendPicBorder((pixel*)p3, ls, width, lines, mx, my);
}

/* f1: the reference's own LookaheadTLD::lowresIntraEstimate (slicetype.cpp:230-330) on a
 * Lowres whose fields it reads / writes point at the caller's buffers */
void xo_lowres_intra(int wcu, int hcu, const void* plane0, intptr_t ls, const int32_t* inv_q, int32_t* intra_cost,
                     uint8_t* intra_mode, uint16_t* lowres_cost, int32_t* row_satd, int64_t* cost_est)
{
    pthread_once(&g_prim_once, init_global_prims);
    static __thread LookaheadTLD* tld = NULL;
    if (!tld) tld = new LookaheadTLD();
    tld->init(wcu, hcu, wcu * hcu);
    Lowres* lr = (Lowres*)calloc(1, sizeof(Lowres));
    lr->lowresPlane[0] = (pixel*)plane0;
    lr->lumaStride = ls;
    lr->intraCost = intra_cost;
    lr->intraMode = intra_mode;
    lr->lowresCosts[0][0] = lowres_cost;
    lr->rowSatds[0][0] = row_satd;
    lr->invQscaleFactor = (int*)inv_q;
    tld->lowresIntraEstimate(*lr);
    cost_est[0] = lr->costEst[0][0];
    cost_est[1] = lr->costEstAq[0][0];
    free(lr);
}

} // extern "C"

namespace {
struct TabBitCost : public BitCost
{
    const uint16_t* table(unsigned qp) { setQP(qp); return m_cost; }
};
struct SearchME : public MotionEstimate
{
    void configure(int method, int refine) { searchMethod = method; subpelRefine = refine; }
    void chroma(pixelcmp_t cs) { chromaSatd = cs; bChromaSATD = subpelRefine > 2 && cs; }
    void at_ctu0() { ctuAddr = 0; absPartIdx = 0; }   /* chroma addressing goes through the PicYuv offsets */
};
struct PropLookahead : public Lookahead
{
    PropLookahead(x265_param* p) : Lookahead(p, NULL) { m_scratch = (int*)calloc(m_8x8Width + 1, sizeof(int)); }
    ~PropLookahead() { free(m_scratch); m_scratch = NULL; }
    void propagate(Lowres** frames, double avg, int p0, int p1, int b, int referenced)
    {
        estimateCUPropagate(frames, avg, p0, p1, b, referenced);
    }
};
struct CostGroup : public CostEstimateGroup
{
    CostGroup(Lookahead& l, Lowres** f) : CostEstimateGroup(l, f) {}
    void cu(LookaheadTLD& tld, int cx, int cy, int p0, int p1, int b, bool* ds, bool last, int slice)
    {
        estimateCUCost(tld, cx, cy, p0, p1, b, ds, last, slice);
    }
    Slice& slice(int i) { return m_slice[i]; }
};
} // namespace

extern "C" {

/* the reference's BitCost table for X265_LOOKAHEAD_QP (what LookaheadTLD's MotionEstimate uses) */
void xo_mvcost_table(int range, uint16_t* out)
{
    TabBitCost bc;
    const uint16_t* c = bc.table(X265_LOOKAHEAD_QP);
    for (int d = -range; d <= range; d++) out[range + d] = c[d];
}

/* f1: a P estimate (p0 = 0, b = p1 = 1) through the reference's own
 * CostEstimateGroup::estimateCUCost (slicetype.cpp:2068-2225, motion search included), in the
 * CU order and slice accounting of estimateFrameCost / processTasks (slicetype.cpp:1957-1972,
 * 2029-2050); weighted prediction off (the caller passes the planes to search). */
void xo_lowres_pcost(int wcu, int hcu, int rows_per_slice, int num_slices, const void* fenc_plane0,
                     const void* r0, const void* r1, const void* r2, const void* r3, intptr_t ls,
                     const int32_t* intra_cost, const int32_t* inv_q, const uint16_t* mvcost_centre,
                     int16_t* mvs, int32_t* mv_costs, uint16_t* lowres_costs, int32_t* row_satd, int64_t* cost_est,
                     int32_t* intra_mbs)
{
    (void)mvcost_centre;   /* the reference uses its own BitCost table */
    pthread_once(&g_prim_once, init_global_prims);
    x265_param* param = x265_param_alloc();
    x265_param_default(param);
    param->sourceWidth = 16 * wcu;
    param->sourceHeight = 16 * hcu;
    param->lookaheadSlices = 0;
    param->bEnableWeightedPred = 0;
    Lookahead* la = new Lookahead(param, NULL);
    LookaheadTLD* tld = new LookaheadTLD();
    tld->init(wcu, hcu, wcu * hcu);

    Lowres* ref = (Lowres*)calloc(1, sizeof(Lowres));
    Lowres* cur = (Lowres*)calloc(1, sizeof(Lowres));
    const void* rp[4] = { r0, r1, r2, r3 };
    for (int k = 0; k < 4; k++) ref->lowresPlane[k] = (pixel*)rp[k];
    ref->fpelPlane[0] = ref->lowresPlane[0];
    ref->lumaStride = ls;
    ref->isLowres = true;
    cur->lowresPlane[0] = (pixel*)fenc_plane0;
    cur->fpelPlane[0] = cur->lowresPlane[0];
    cur->lumaStride = ls;
    cur->isLowres = true;
    cur->intraCost = (int32_t*)intra_cost;
    cur->invQscaleFactor = (int*)inv_q;
    cur->lowresMvs[0][0] = (MV*)mvs;
    cur->lowresMvCosts[0][0] = mv_costs;
    cur->lowresCosts[1][0] = lowres_costs;
    cur->rowSatds[1][0] = row_satd;
    Lowres* frames[2] = { ref, cur };
    CostGroup g(*la, frames);
    bool ds[2] = { true, false };
    const int p0 = 0, b = 1, p1 = 1;
    if (num_slices < 1) { num_slices = 1; rows_per_slice = hcu; }
    if (num_slices == 1)
    {
        /* serial whole-frame path: sums go straight to the frame */
        cur->costEst[1][0] = cur->costEstAq[1][0] = 0;
        bool last = true;
        for (int cy = hcu - 1; cy >= 0; cy--)
        {
            row_satd[cy] = 0;
            for (int cx = wcu - 1; cx >= 0; cx--) g.cu(*tld, cx, cy, p0, p1, b, ds, last, -1);
            last = false;
        }
        cost_est[0] = cur->costEst[1][0];
        cost_est[1] = cur->costEstAq[1][0];
        *intra_mbs = cur->intraMbs[1];
    }
    else
    {
        int64_t est = 0, est_aq = 0;
        int mbs = 0;
        for (int i = 0; i < num_slices; i++)
        {
            memset(&g.slice(i), 0, sizeof(g.slice(i)));
            const int first = rows_per_slice * i;
            const int lastY = i == num_slices - 1 ? hcu - 1 : rows_per_slice * (i + 1) - 1;
            bool last = true;
            for (int cy = lastY; cy >= first; cy--)
            {
                row_satd[cy] = 0;
                for (int cx = wcu - 1; cx >= 0; cx--) g.cu(*tld, cx, cy, p0, p1, b, ds, last, i);
                last = false;
            }
            est += g.slice(i).costEst;
            est_aq += g.slice(i).costEstAq;
            mbs += g.slice(i).intraMbs;
        }
        cost_est[0] = est;
        cost_est[1] = est_aq;
        *intra_mbs = mbs;
    }
    free(ref);
    free(cur);
    delete tld;
    delete la;
    x265_param_free(param);
}

/* f1 weightp: the reference's own LookaheadTLD::weightsAnalyse (slicetype.cpp:391-495) on Lowres
 * frames wired to the caller's contiguous 4-plane buffers (as Lowres::create allocates them) */
void xo_weights_analyse(int width, int lines, intptr_t stride, int padded_lines, intptr_t pad_offset,
                        const void* fenc_plane, const void* const* ref_buf, const int32_t* intra_cost,
                        void* const* wbuf, uint64_t fenc_ssd, uint64_t ref_ssd, uint64_t fenc_sum,
                        uint64_t ref_sum, int* out, double* cost_delta)
{
    pthread_once(&g_prim_once, init_global_prims);
    const size_t planesize = (size_t)stride * padded_lines;
    Lowres* fenc = (Lowres*)calloc(1, sizeof(Lowres));
    Lowres* ref = (Lowres*)calloc(1, sizeof(Lowres));
    /* weightsAnalyse reads only fenc's plane 0 but sizes its buffers from fenc.buffer[1] - buffer[0] */
    pixel* fbuf = (pixel*)fenc_plane - pad_offset;
    for (int i = 0; i < 4; i++)
    {
        fenc->buffer[i] = fbuf + i * planesize;
        fenc->lowresPlane[i] = fenc->buffer[i] + pad_offset;
        ref->buffer[i] = (pixel*)ref_buf[i];
        ref->lowresPlane[i] = ref->buffer[i] + pad_offset;
    }
    fenc->fpelPlane[0] = fenc->lowresPlane[0];
    ref->fpelPlane[0] = ref->lowresPlane[0];
    fenc->lumaStride = ref->lumaStride = stride;
    fenc->width = ref->width = width;
    fenc->lines = ref->lines = lines;
    fenc->isLowres = ref->isLowres = true;
    fenc->frameNum = 1;
    ref->frameNum = 0;
    fenc->intraCost = (int32_t*)intra_cost;
    fenc->wp_ssd[0] = fenc_ssd;
    ref->wp_ssd[0] = ref_ssd;
    fenc->wp_sum[0] = fenc_sum;
    ref->wp_sum[0] = ref_sum;
    LookaheadTLD* tld = new LookaheadTLD();
    tld->weightsAnalyse(*fenc, *ref);
    ReferencePlanes& wr = fenc->weightedRef[1];
    out[0] = wr.isWeighted ? 1 : 0;
    if (tld->wbuffer[0])
        for (int i = 0; i < 4; i++) memcpy(wbuf[i], tld->wbuffer[i], planesize * sizeof(pixel));
    if (wr.isWeighted) *cost_delta = fenc->weightedCostDelta[1];
    free(fenc);
    free(ref);
    delete tld;
}

/* f1 cuTree: the reference's own Lookahead::estimateCUPropagate (slicetype.cpp:1738-1836) for
 * (p0, b, p1) = (0, b_p0, b_p0 + p1_b) on Lowres frames wired to the caller's arrays */
void xo_cutree_propagate(int wcu, int hcu, int b_p0, int p1_b, int referenced, int weighted_bipred,
                         int fps_num, int fps_den, double avg_duration, uint16_t* propagate_b,
                         const int32_t* intra_cost, const uint16_t* lowres_costs, const int32_t* inv_q,
                         const int32_t* mvs0, const int32_t* mvs1, uint16_t* ref0, uint16_t* ref1)
{
    pthread_once(&g_prim_once, init_global_prims);
    x265_param* param = x265_param_alloc();
    x265_param_default(param);
    param->sourceWidth = 16 * wcu;
    param->sourceHeight = 16 * hcu;
    param->fpsNum = fps_num;
    param->fpsDenom = fps_den;
    param->bEnableWeightedBiPred = weighted_bipred;
    param->rc.vbvBufferSize = 0;
    PropLookahead* la = new PropLookahead(param);
    const int p0 = 0, b = b_p0, p1 = b_p0 + p1_b;
    Lowres* fr[X265_BFRAME_MAX + 2];
    for (int i = 0; i <= p1; i++) fr[i] = (Lowres*)calloc(1, sizeof(Lowres));
    fr[p0]->propagateCost = ref0;
    fr[p1]->propagateCost = p1 == b ? propagate_b : ref1;
    fr[b]->propagateCost = propagate_b;
    fr[b]->intraCost = (int32_t*)intra_cost;
    fr[b]->invQscaleFactor = (int*)inv_q;
    fr[b]->lowresCosts[b - p0][p1 - b] = (uint16_t*)lowres_costs;
    fr[b]->lowresMvs[0][b - p0 - 1] = (MV*)mvs0;
    if (p1 > b) fr[b]->lowresMvs[1][p1 - b - 1] = (MV*)mvs1;
    la->propagate(fr, avg_duration, p0, p1, b, referenced);
    for (int i = 0; i <= p1; i++) free(fr[i]);
    delete la;
    x265_param_free(param);
}

/* f1: a B estimate (p0 = 0, b = 1, p1 = 2) through the reference's own estimateCUCost with
 * bBidir, in the CU order and slice accounting of estimateFrameCost / processTasks */
void xo_lowres_bcost(int wcu, int hcu, int rows_per_slice, int num_slices, const void* fenc_plane0,
                     const void* const* ref0, const void* const* ref1, intptr_t ls, const int32_t* inv_q,
                     const uint16_t* mvcost_centre, int do_search0, int do_search1, int16_t* mvs0,
                     int32_t* mv_costs0, int16_t* mvs1, int32_t* mv_costs1, uint16_t* lowres_costs,
                     int32_t* row_satd, int64_t* cost_est)
{
    (void)mvcost_centre;
    pthread_once(&g_prim_once, init_global_prims);
    x265_param* param = x265_param_alloc();
    x265_param_default(param);
    param->sourceWidth = 16 * wcu;
    param->sourceHeight = 16 * hcu;
    param->lookaheadSlices = 0;
    param->bEnableWeightedPred = 0;
    Lookahead* la = new Lookahead(param, NULL);
    LookaheadTLD* tld = new LookaheadTLD();
    tld->init(wcu, hcu, wcu * hcu);

    Lowres* r0 = (Lowres*)calloc(1, sizeof(Lowres));
    Lowres* r1 = (Lowres*)calloc(1, sizeof(Lowres));
    Lowres* cur = (Lowres*)calloc(1, sizeof(Lowres));
    for (int k = 0; k < 4; k++)
    {
        r0->lowresPlane[k] = (pixel*)ref0[k];
        r1->lowresPlane[k] = (pixel*)ref1[k];
    }
    Lowres* lr[3] = { r0, cur, r1 };
    for (int i = 0; i < 3; i++)
    {
        lr[i]->fpelPlane[0] = lr[i]->lowresPlane[0];
        lr[i]->lumaStride = ls;
        lr[i]->isLowres = true;
    }
    cur->lowresPlane[0] = cur->fpelPlane[0] = (pixel*)fenc_plane0;
    cur->invQscaleFactor = (int*)inv_q;
    cur->lowresMvs[0][0] = (MV*)mvs0;
    cur->lowresMvCosts[0][0] = mv_costs0;
    cur->lowresMvs[1][0] = (MV*)mvs1;
    cur->lowresMvCosts[1][0] = mv_costs1;
    cur->lowresCosts[1][1] = lowres_costs;
    cur->rowSatds[1][1] = row_satd;
    CostGroup g(*la, lr);
    bool ds[2] = { !!do_search0, !!do_search1 };
    const int p0 = 0, b = 1, p1 = 2;
    if (num_slices < 1) { num_slices = 1; rows_per_slice = hcu; }
    int64_t est = 0, est_aq = 0;
    if (num_slices == 1)
    {
        cur->costEst[1][1] = cur->costEstAq[1][1] = 0;
        bool last = true;
        for (int cy = hcu - 1; cy >= 0; cy--)
        {
            row_satd[cy] = 0;
            for (int cx = wcu - 1; cx >= 0; cx--) g.cu(*tld, cx, cy, p0, p1, b, ds, last, -1);
            last = false;
        }
        est = cur->costEst[1][1];
        est_aq = cur->costEstAq[1][1];
    }
    else
        for (int i = 0; i < num_slices; i++)
        {
            memset(&g.slice(i), 0, sizeof(g.slice(i)));
            const int first = rows_per_slice * i;
            const int lastY = i == num_slices - 1 ? hcu - 1 : rows_per_slice * (i + 1) - 1;
            bool last = true;
            for (int cy = lastY; cy >= first; cy--)
            {
                row_satd[cy] = 0;
                for (int cx = wcu - 1; cx >= 0; cx--) g.cu(*tld, cx, cy, p0, p1, b, ds, last, i);
                last = false;
            }
            est += g.slice(i).costEst;
            est_aq += g.slice(i).costEstAq;
        }
    cost_est[0] = est;
    cost_est[1] = est_aq;
    free(r0);
    free(r1);
    free(cur);
    delete tld;
    delete la;
    x265_param_free(param);
}

void xo_mvcost_table_qp(int qp, int range, uint16_t* out)
{
    TabBitCost bc;
    const uint16_t* c = bc.table((unsigned)qp);
    for (int d = -range; d <= range; d++) out[range + d] = c[d];
}

/* f2: the reference's own MotionEstimate::motionEstimate on a full-resolution reference
 * (fpelPlane[0] at the PU origin, no PicYuv: ctuAddr stays -1 so blockOffset = 0, luma only) */
int xo_motion_search(int w, int h, int method, int subme, int merange, const void* fenc, intptr_t fs, const void* ref,
                     intptr_t rs, int minx, int miny, int maxx, int maxy, int mvpx, int mvpy, int numc,
                     const int16_t* mvc, const uint16_t* tab_centre, int16_t* out,
                     const void* fcb, const void* fcr, intptr_t fcs, const void* rcb, const void* rcr, intptr_t rcs)
{
    (void)tab_centre;    /* the reference uses its own BitCost table: the caller sets the QP below */
    pthread_once(&g_prim_once, init_global_prims);
    static __thread SearchME* me = NULL;
    if (!me)
    {
        MotionEstimate::initScales();
        me = new SearchME();
        me->init(X265_HEX_SEARCH, 2, X265_CSP_I420);   /* allocates the 4:2:0 fenc PU buffers once */
    }
    me->configure(method == 0 ? X265_DIA_SEARCH : method == 1 ? X265_HEX_SEARCH : method == 3 ? X265_UMH_SEARCH : method == 4 ? X265_FULL_SEARCH : X265_STAR_SEARCH, subme);
    me->setQP(g_me_qp);
    me->setSourcePU((pixel*)fenc, fs, 0, w, h);
    /* chroma PU as Yuv::copyPUFromYuv would place it, and bChromaSATD as the encoder's setSourcePU
     * sets it (motion.cpp:183-197) */
    pixelcmp_t cs = fcb ? primitives.chroma[X265_CSP_I420].pu[me->partEnum].satd : NULL;
    me->chroma(cs);
    static intptr_t zero_off[2] = { 0, 0 };
    PicYuv* pic = (PicYuv*)calloc(1, sizeof(PicYuv));
    ReferencePlanes rp;
    rp.fpelPlane[0] = (pixel*)ref;
    rp.lumaStride = rs;
    rp.isLowres = false;
    if (me->bChromaSATD)
    {
        for (int y = 0; y < (h >> 1); y++)
            for (int x = 0; x < (w >> 1); x++)
            {
                me->fencPUYuv.m_buf[1][y * me->fencPUYuv.m_csize + x] = ((const pixel*)fcb)[y * fcs + x];
                me->fencPUYuv.m_buf[2][y * me->fencPUYuv.m_csize + x] = ((const pixel*)fcr)[y * fcs + x];
            }
        /* chroma addresses come from reconPic's CU / block offsets (lowres.h:52-54): address the PU as
         * CTU 0 / part 0 of a picture whose offsets are all 0, so blockOffset stays 0 (motion.cpp:582) */
        pic->m_cuOffsetY = zero_off;
        pic->m_buOffsetY = zero_off;
        pic->m_cuOffsetC = zero_off;
        pic->m_buOffsetC = zero_off;
        pic->m_strideC = rcs;
        me->at_ctu0();
        rp.fpelPlane[1] = (pixel*)rcb;
        rp.fpelPlane[2] = (pixel*)rcr;
        rp.reconPic = pic;
    }
    MV mvs[16];
    for (int i = 0; i < numc && i < 16; i++) mvs[i] = MV(mvc[2 * i], mvc[2 * i + 1]);
    MV outmv;
    const int cost = me->motionEstimate(&rp, MV(minx, miny), MV(maxx, maxy), MV(mvpx, mvpy), numc, mvs, merange, outmv);
    free(pic);
    out[0] = outmv.x;
    out[1] = outmv.y;
    return cost;
}

/* QP used by xo_motion_search's BitCost (the restatement receives the table instead) */
void xo_set_me_qp(int qp) { g_me_qp = qp; }

void xo_scan_table(int type, int log2, uint16_t* out)
{
    memcpy(out, g_scanOrder[type][log2 - 2], sizeof(uint16_t) << (2 * log2));
}

} // extern "C"

/* ======================================================= f4 loop filters
 * The reference's own SAO (sao.cpp) and Deblock (deblock.cpp) run on a frame built from the
 * caller's planes: PicYuv::create / createOffsets for the recon (and source) pictures, one CUData
 * per CTU, and the process globals x265_set_globals would set for the CTU size (param.cpp:1242-1255). */
namespace {

void set_ctu_globals(int ctu_log2)
{
    g_maxCUSize = 1u << ctu_log2;
    g_maxLog2CUSize = ctu_log2;
    g_maxCUDepth = ctu_log2 - 3;
    g_unitSizeDepth = ctu_log2 - LOG2_UNIT_SIZE;
    uint32_t* tmp = &g_zscanToRaster[0];
    initZscanToRaster(g_unitSizeDepth, 1, 0, tmp);
    initRasterToZscan(g_unitSizeDepth);
    CUData::s_numPartInCUSize = 1u << g_unitSizeDepth;
}

struct FrameShell
{
    SPS sps;
    PPS pps;
    Slice slice;
    FrameData* fd;
    Frame* frame;
    PicYuv* recon;
    PicYuv* fenc;
    CUData* ctus;
    CUDataMemPool pool;
    int wc, hc;

    int csp;
    FrameShell(int width, int height, bool with_fenc, bool with_cudata, int csp_ = X265_CSP_I420) : csp(csp_)
    {
        memset(&sps, 0, sizeof(sps));
        memset(&pps, 0, sizeof(pps));
        wc = (width + g_maxCUSize - 1) / g_maxCUSize;
        hc = (height + g_maxCUSize - 1) / g_maxCUSize;
        sps.numCuInWidth = wc;
        sps.numCuInHeight = hc;
        sps.numPartInCUSize = 1u << g_unitSizeDepth;
        sps.picWidthInLumaSamples = width;
        sps.picHeightInLumaSamples = height;
        slice.m_sps = &sps;
        slice.m_pps = &pps;
        recon = new PicYuv;
        recon->create(width, height, csp);
        recon->createOffsets(sps);
        fenc = NULL;
        if (with_fenc)
        {
            fenc = new PicYuv;
            fenc->create(width, height, csp);
            fenc->createOffsets(sps);
        }
        fd = (FrameData*)calloc(1, sizeof(FrameData));
        fd->m_slice = &slice;
        fd->m_reconPic = recon;
        frame = (Frame*)calloc(1, sizeof(Frame));
        frame->m_encData = fd;
        frame->m_reconPic = recon;
        frame->m_fencPic = fenc;
        ctus = new CUData[wc * hc];
        if (with_cudata) pool.create(0, csp, wc * hc);
        for (int i = 0; i < wc * hc; i++)
        {
            CUData& cu = ctus[i];
            if (with_cudata) cu.initialize(pool, 0, csp, i);
            cu.m_encData = fd;
            cu.m_slice = &slice;
            cu.m_cuAddr = i;
            cu.m_cuPelX = (i % wc) << g_maxLog2CUSize;
            cu.m_cuPelY = (i / wc) << g_maxLog2CUSize;
            cu.m_absIdxInCTU = 0;
            cu.m_numPartitions = NUM_4x4_PARTITIONS;
            cu.m_chromaFormat = csp;
            cu.m_hChromaShift = CHROMA_H_SHIFT(csp);
            cu.m_vChromaShift = CHROMA_V_SHIFT(csp);
            cu.m_cuLeft = (i % wc) ? &ctus[i - 1] : NULL;
            cu.m_cuAbove = (i / wc) ? &ctus[i - wc] : NULL;
        }
        fd->m_picCTU = ctus;
    }
    ~FrameShell()
    {
        if (pool.charMemBlock) pool.destroy();
        /* CUData arrays belong to the pool; the CUData objects themselves are plain */
        delete[] ctus;
        recon->destroy();
        delete recon;
        if (fenc) { fenc->destroy(); delete fenc; }
        free(fd);
        free(frame);
    }
};

/* caller plane (plus a one-pixel ring) <-> PicYuv plane */
void load_plane(PicYuv* pic, int plane, const void* src, intptr_t ss, int w, int h)
{
    const intptr_t ps = plane ? pic->m_strideC : pic->m_stride;
    for (int y = -1; y <= h; y++)
        memcpy(pic->m_picOrg[plane] + y * ps - 1, (const pixel*)src + y * ss - 1, sizeof(pixel) * (w + 2));
}
void store_plane(const PicYuv* pic, int plane, void* dst, intptr_t ds, int w, int h)
{
    const intptr_t ps = plane ? pic->m_strideC : pic->m_stride;
    for (int y = 0; y < h; y++)
        memcpy((pixel*)dst + y * ds, pic->m_picOrg[plane] + y * ps, sizeof(pixel) * w);
}

struct ShimSao : public SAO
{
    void tmpU_from(const PicYuv* snap, int row, int col)
    {
        /* FrameFilter::ParallelFilter::copySaoAboveRef (framefilter.cpp:176-199) on the deblocked,
         * not yet SAO-processed picture */
        const uint32_t addr = row * m_numCuInWidth + col;
        for (int p = 0; p < 3; p++)
        {
            const int cw = p ? g_maxCUSize >> m_hChromaShift : g_maxCUSize;
            const intptr_t st = p ? snap->m_strideC : snap->m_stride;
            const pixel* r = snap->getPlaneAddr(p, addr) - (row == 0 ? 0 : st);
            memcpy(&m_tmpU[p][col * cw], r, cw * sizeof(pixel));
        }
    }
    void clear_stats() { memset(m_offsetOrg, 0, sizeof(m_offsetOrg)); memset(m_count, 0, sizeof(m_count)); }
    const int32_t* org(int p, int t) const { return m_offsetOrg[p][t]; }
    const int32_t* cnt(int p, int t) const { return m_count[p][t]; }
};

void sao_param_defaults(x265_param* prm, int width, int height, int non_deblocked, int csp = X265_CSP_I420)
{
    x265_param_default(prm);
    prm->sourceWidth = width;
    prm->sourceHeight = height;
    prm->internalCsp = csp;
    prm->maxCUSize = g_maxCUSize;
    prm->bSaoNonDeblocked = non_deblocked;
}

} // namespace

extern "C" {

void xo_sao_apply_csp(int width, int height, int ctu_log2, void* y, void* cb, void* cr, intptr_t stride,
                      intptr_t cstride, const xo_sao_param* params, int luma_on, int chroma_on, int csp)
{
    pthread_once(&g_prim_once, init_global_prims);
    set_ctu_globals(ctu_log2);
    const int hs = CHROMA_H_SHIFT(csp), vs = CHROMA_V_SHIFT(csp);
    FrameShell fs(width, height, false, false, csp);
    FrameShell snap(width, height, false, false, csp);
    void* planes[3] = { y, cb, cr };
    for (int p = 0; p < 3; p++)
    {
        const int w = p ? width >> hs : width, h = p ? height >> vs : height;
        load_plane(fs.recon, p, planes[p], p ? cstride : stride, w, h);
        load_plane(snap.recon, p, planes[p], p ? cstride : stride, w, h);
    }
    x265_param prm;
    sao_param_defaults(&prm, width, height, 0, csp);
    ShimSao sao;
    sao.create(&prm, 1);
    sao.m_frame = fs.frame;
    const int nctu = fs.wc * fs.hc;
    SaoCtuParam* cp[3];
    for (int p = 0; p < 3; p++)
    {
        cp[p] = new SaoCtuParam[nctu];
        for (int c = 0; c < nctu; c++)
        {
            const xo_sao_param& q = params[p * nctu + c];
            cp[p][c].mergeMode = SAO_MERGE_NONE;
            cp[p][c].typeIdx = q.type;
            cp[p][c].bandPos = q.band;
            for (int i = 0; i < 4; i++) cp[p][c].offset[i] = q.offset[i];
        }
    }
    for (int row = 0; row < fs.hc; row++)
    {
        for (int col = 0; col < fs.wc; col++) sao.tmpU_from(snap.recon, row, col);
        for (int col = 0; col < fs.wc; col++)
        {
            if (luma_on) sao.processSaoUnitCuLuma(cp[0], row, col);
            if (chroma_on) sao.processSaoUnitCuChroma(cp, row, col);
        }
    }
    for (int p = 0; p < 3; p++)
    {
        store_plane(fs.recon, p, planes[p], p ? cstride : stride, p ? width >> hs : width, p ? height >> vs : height);
        delete[] cp[p];
    }
    sao.destroy(1);
}

void xo_sao_apply(int width, int height, int ctu_log2, void* y, void* cb, void* cr, intptr_t stride,
                  intptr_t cstride, const xo_sao_param* params, int luma_on, int chroma_on)
{
    xo_sao_apply_csp(width, height, ctu_log2, y, cb, cr, stride, cstride, params, luma_on, chroma_on, X265_CSP_I420);
}

void xo_sao_stats_csp(int width, int height, int ctu_log2, int non_deblocked, const void* fy, const void* fcb,
                      const void* fcr, intptr_t fstride, intptr_t fcstride, const void* ry, const void* rcb,
                      const void* rcr, intptr_t rstride, intptr_t rcstride, int32_t* stats, int32_t* count, int csp)
{
    pthread_once(&g_prim_once, init_global_prims);
    set_ctu_globals(ctu_log2);
    const int hs = CHROMA_H_SHIFT(csp), vs = CHROMA_V_SHIFT(csp);
    FrameShell fs(width, height, true, false, csp);
    const void* fp[3] = { fy, fcb, fcr };
    const void* rp[3] = { ry, rcb, rcr };
    for (int p = 0; p < 3; p++)
    {
        const int w = p ? width >> hs : width, h = p ? height >> vs : height;
        load_plane(fs.fenc, p, fp[p], p ? fcstride : fstride, w, h);
        load_plane(fs.recon, p, rp[p], p ? rcstride : rstride, w, h);
    }
    x265_param prm;
    sao_param_defaults(&prm, width, height, non_deblocked, csp);
    ShimSao sao;
    sao.create(&prm, 1);
    sao.m_frame = fs.frame;
    const int nctu = fs.wc * fs.hc;
    for (int c = 0; c < nctu; c++)
        for (int p = 0; p < 3; p++)
        {
            sao.clear_stats();
            sao.calcSaoStatsCu(c, p);
            for (int t = 0; t < 5; t++)
            {
                memcpy(stats + ((c * 3 + p) * 5 + t) * 33, sao.org(p, t), 33 * sizeof(int32_t));
                memcpy(count + ((c * 3 + p) * 5 + t) * 33, sao.cnt(p, t), 33 * sizeof(int32_t));
            }
        }
    sao.destroy(1);
}

void xo_sao_stats(int width, int height, int ctu_log2, int non_deblocked, const void* fy, const void* fcb,
                  const void* fcr, intptr_t fstride, intptr_t fcstride, const void* ry, const void* rcb,
                  const void* rcr, intptr_t rstride, intptr_t rcstride, int32_t* stats, int32_t* count)
{
    xo_sao_stats_csp(width, height, ctu_log2, non_deblocked, fy, fcb, fcr, fstride, fcstride, ry, rcb, rcr, rstride,
                     rcstride, stats, count, X265_CSP_I420);
}

void xo_deblock_csp(int width, int height, int ctu_log2, void* y, void* cb, void* cr, intptr_t stride,
                    intptr_t cstride, const xo_deblock_unit* units, intptr_t us, const xo_deblock_params* prm, int csp)
{
    pthread_once(&g_prim_once, init_global_prims);
    set_ctu_globals(ctu_log2);
    const int hs = CHROMA_H_SHIFT(csp), vs = CHROMA_V_SHIFT(csp);
    FrameShell fs(width, height, false, true, csp);
    fs.pps.deblockingFilterBetaOffsetDiv2 = prm->beta_offset_div2;
    fs.pps.deblockingFilterTcOffsetDiv2 = prm->tc_offset_div2;
    fs.pps.chromaQpOffset[0] = prm->cb_qp_offset;
    fs.pps.chromaQpOffset[1] = prm->cr_qp_offset;
    fs.pps.bTransquantBypassEnabled = !!prm->tq_bypass_enabled;
    fs.slice.m_sliceType = prm->is_p ? P_SLICE : B_SLICE;
    /* reference identity: one distinct (never dereferenced) Frame address per POC */
    static char poc_space[1 << 16];
    for (int l = 0; l < 2; l++)
        for (int i = 0; i < 16; i++)
            fs.slice.m_refFrameList[l][i] = (Frame*)(poc_space + ((prm->ref_poc[l][i] & 0x3fff) << 2));
    void* planes[3] = { y, cb, cr };
    for (int p = 0; p < 3; p++)
        load_plane(fs.recon, p, planes[p], p ? cstride : stride, p ? width >> hs : width, p ? height >> vs : height);

    /* the CU tree, per 4x4 partition in z-order */
    const int ctu = g_maxCUSize, npart = NUM_4x4_PARTITIONS;
    for (int c = 0; c < fs.wc * fs.hc; c++)
    {
        CUData& cu = fs.ctus[c];
        for (int z = 0; z < npart; z++)
        {
            const int px = cu.m_cuPelX + g_zscanToPelX[z], py = cu.m_cuPelY + g_zscanToPelY[z];
            if (px >= width || py >= height)
            {
                cu.m_predMode[z] = MODE_NONE;
                cu.m_cuDepth[z] = g_maxCUDepth;
                cu.m_log2CUSize[z] = 3;
                continue;
            }
            const xo_deblock_unit& u = units[(py >> 2) * us + (px >> 2)];
            cu.m_predMode[z] = (u.flags & 1) ? MODE_INTRA : MODE_INTER;
            cu.m_partSize[z] = u.part;
            cu.m_cuDepth[z] = ctu_log2 - u.cu_log2;
            cu.m_log2CUSize[z] = u.cu_log2;
            cu.m_tuDepth[z] = u.cu_log2 - u.tu_log2;
            cu.m_cbf[0][z] = (u.flags & 2) ? (uint8_t)(1 << cu.m_tuDepth[z]) : 0;
            cu.m_qp[z] = u.qp;
            cu.m_tqBypass[z] = (u.flags & 4) ? 1 : 0;
            for (int l = 0; l < 2; l++)
            {
                cu.m_refIdx[l][z] = u.ref_idx[l];
                cu.m_mv[l][z] = MV(u.mv[l][0], u.mv[l][1]);
            }
        }
    }
    CUGeom* geoms = new CUGeom[fs.wc * fs.hc * CUGeom::MAX_GEOMS];
    for (int c = 0; c < fs.wc * fs.hc; c++)
    {
        const int cw = X265_MIN(ctu, width - (c % fs.wc) * ctu), ch = X265_MIN(ctu, height - (c / fs.wc) * ctu);
        CUData::calcCTUGeoms(cw, ch, ctu, 8, geoms + c * CUGeom::MAX_GEOMS);
    }
    /* FrameFilter::ParallelFilter::processTasks order (framefilter.cpp:312-330, 386-392) */
    for (int row = 0; row < fs.hc; row++)
    {
        for (int col = 0; col < fs.wc; col++)
        {
            const int a = row * fs.wc + col;
            Deblock::deblockCTU(&fs.ctus[a], geoms[a * CUGeom::MAX_GEOMS], Deblock::EDGE_VER);
            if (col >= 1)
                Deblock::deblockCTU(&fs.ctus[a - 1], geoms[(a - 1) * CUGeom::MAX_GEOMS], Deblock::EDGE_HOR);
        }
        const int a = row * fs.wc + fs.wc - 1;
        Deblock::deblockCTU(&fs.ctus[a], geoms[a * CUGeom::MAX_GEOMS], Deblock::EDGE_HOR);
    }
    delete[] geoms;
    for (int p = 0; p < 3; p++)
        store_plane(fs.recon, p, planes[p], p ? cstride : stride, p ? width >> hs : width, p ? height >> vs : height);
}

void xo_deblock(int width, int height, int ctu_log2, void* y, void* cb, void* cr, intptr_t stride,
                intptr_t cstride, const xo_deblock_unit* units, intptr_t us, const xo_deblock_params* prm)
{
    xo_deblock_csp(width, height, ctu_log2, y, cb, cr, stride, cstride, units, us, prm, X265_CSP_I420);
}

void xo_extend_border(void* plane, intptr_t stride, int width, int height, int mx, int my)
{
    extendPicBorder((pixel*)plane, stride, width, height, mx, my);
}

} // extern "C"
