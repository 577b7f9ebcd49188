/* gpu_rdo.cpp — reference-side binding (round 6): the residual coding of inter CUs runs on the MI355X
 * through the f3 session entries of include/x265_amd.h (x265amd_rdo_*, csrc/rdosession.cpp).
 *
 * This is the hook a maintainer adds to the encoder.  oracle/Makefile links the
 * reference encoder with copies of search.o and quant.o in which these symbols are weak (objcopy -W) and
 * the originals stay reachable under aliases:
 *
 *   Search::encodeResAndCalcRdInterCU(Mode&, const CUGeom&)               search.cpp:2562-2690
 *     -> for an eligible CU (2Nx2N, 4:2:0, at least X265AMD_RDO_MIN, one RQT level — --preset medium's
 *        tools, see eligible()), the CU's source and prediction planes and the Quant object's QPs are
 *        POSTED to the device (x265amd_rdo_post) and the worker waits for the results of every TU:
 *        coefficients, numSig, inverse-transformed residual, reconstruction, and the psy energies of
 *        every 8x8 block against the prediction and the reconstruction.  Then the reference's own
 *        encodeResAndCalcRdInterCU runs unchanged (x265ref_encodeResAndCalcRdInterCU), with the calling
 *        thread's memo of those results active:
 *   Quant::transformNxN(cu, fenc, fencStride, residual, resiStride, coeff, log2TrSize, ttype, absPartIdx,
 *                       useTransformSkip)                                  quant.cpp:397-480
 *     -> a TU of the memo's CU (the residual pointer lies in the CU's residual buffer at a TU origin of
 *        the memo's TU size, fenc is the matching source block, no transform skip): its coefficients
 *        and numSig from the device; else the reference's function;
 *   Quant::invtransformNxN(cu, residual, resiStride, coeff, log2TrSize, ttype, bIntra, useTransformSkip,
 *                          numSig)                                         quant.cpp:482-546
 *     -> the coefficients the memo served for that TU, unchanged (compared) and with the same numSig:
 *        the device's inverse-transformed residual; else the reference's function;
 *   primitives.cu[1..4].psy_cost_pp (psyCost_pp<size>, pixel.cpp:672-703; installed by the binding
 *     into the table, x265amd_rdo_install) -> a source block of the memo's CU against a block whose every
 *        8x8 block equals (compared) either the prediction or the device's reconstruction there: the sum
 *        of the device's per-8x8 energies; else psyCost_pp.
 *
 * So the encoder's control flow and every decision (CABAC estimates, null-cbf choices, mode choice) stay
 * the reference's code; a result is taken from the device only where the call's inputs are the ones the
 * device computed from.  The bitstream equals the reference encoder's (tests/test_encoder_me.py).
 *
 *   X265AMD_RDO=gpu     device residual coding (default: cpu)
 *   X265AMD_RDO=cpu     every call goes to the reference's functions (same binary)
 *   X265AMD_RDO=check   device residual coding, every memo answer recomputed by the reference function
 *                       and compared ("[x265rdo] check: N mismatches" at exit)
 *   X265AMD_RDO=host    the results are computed on the host by the reference's own transformNxN /
 *                       invtransformNxN / psyCost_pp (host_result) and served through the same memo: checks
 *                       the binding's plumbing on a CPU-only host (every call must hit, bitstream unchanged)
 *   X265AMD_RDO_MIN=k   smallest CU (log2, 4..6, default 6: 64x64) coded on the device
 *   X265AMD_RDO_EARLY=1 post each CU's request as soon as its prediction is final, ahead of the call that codes
 *                       it, instead of posting and waiting inside encodeResAndCalcRdInterCU (below); a call with
 *                       no matching early post is coded on the host
 *
 * Early posts (X265AMD_RDO_EARLY=1).  The three predictions --preset medium's inter analysis codes at a depth
 * (compressInterCU_rd0_4, analysis.cpp:818-1298) are final well before their encodeResAndCalcRdInterCU:
 *   Search::predInterSearch (hooked in gpu_me.cpp)       the 2Nx2N prediction (luma and, at --rd >= 3, chroma
 *                                                       MC done, search.cpp:2405-2420) — coded after the
 *                                                       bidir and rectangular checks (analysis.cpp:943-1118);
 *   Analysis::checkBidir2Nx2N (analysis.cpp:2013)        the bidir prediction — coded after the best inter mode
 *                                                       (:1121-1126);
 *   Search::encodeResAndCalcRdSkipCU (search.cpp:2512)   the best merge candidate's prediction — coded with
 *                                                       residual right after the skip costing (:1739-1752).
 * Each is posted there, with the Quant object's QPs of the moment (the CU's: the analysis sets them before the
 * CU's modes, :926-927) and a copy of the prediction; encodeResAndCalcRdInterCU takes the post whose source
 * buffer, QPs, size and prediction (compared) are the call's, so a post whose prediction changed or was never
 * coded is simply not used (dropped when its slot is posted again or the encoder closes).
 *   X265AMD_RDO_LAUNCHERS=n  service threads per session (default 2; 0: each worker launches its CU itself,
 *                       zero-copy, and polls a completion flag)
 *   X265AMD_ME_STATS=1  posts, memo hits / misses per function, worker wait time, session counters at exit
 */
#include "common.h"
#include "primitives.h"
#include "frame.h"
#include "framedata.h"
#include "picyuv.h"
#include "slice.h"
#include "search.h"
#include "analysis.h"
#include "quant.h"
#include "scalinglist.h"
#include "yuv.h"
#include "shortyuv.h"
#include "sao.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <pthread.h>
#include <vector>

#include "../include/x265_amd.h"

using namespace X265_NS;

extern "C" void x265ref_encodeResAndCalcRdInterCU(Search* self, Mode& interMode, const CUGeom& cuGeom);
extern "C" void x265ref_encodeResAndCalcRdSkipCU(Search* self, Mode& interMode);
extern "C" void x265ref_checkBidir2Nx2N(Analysis* self, Mode& inter2Nx2N, Mode& bidir2Nx2N, const CUGeom& cuGeom);
extern "C" uint32_t x265ref_transformNxN(Quant* self, const CUData& cu, const pixel* fenc, uint32_t fencStride,
                                         const int16_t* residual, uint32_t resiStride, coeff_t* coeff,
                                         uint32_t log2TrSize, TextType ttype, uint32_t absPartIdx,
                                         bool useTransformSkip);
extern "C" void x265ref_invtransformNxN(Quant* self, const CUData& cu, int16_t* residual, uint32_t resiStride,
                                        const coeff_t* coeff, uint32_t log2TrSize, TextType ttype, bool bIntra,
                                        bool useTransformSkip, uint32_t numSig);
extern "C" void x265ref_calcSaoStatsCu(SAO* self, int addr, int plane);

namespace {

/* Quant's QPs, scaling list and RDOQ level are protected; pointers to the members taken through a derived
 * class read them from the Search's Quant */
struct QuantPeek : public Quant
{
    static QpParam (Quant::*qp())[3] { return &QuantPeek::m_qpParam; }
    static const ScalingList* Quant::*scaling() { return &QuantPeek::m_scalingList; }
    static int Quant::*rdoq() { return &QuantPeek::m_rdoqLevel; }
};

enum { RDO_CPU = 0, RDO_GPU = 1, RDO_CHECK = 2, RDO_HOST = 3 };
int g_mode = RDO_CPU;
int g_min_log2 = 6;
int g_launchers = 2;
bool g_early = false;
bool g_sao = false;                    /* X265AMD_RDO_SAO: each CTU's SAO statistics by the resident server */
bool g_sao_host = false;               /* X265AMD_RDO_SAO=host: the same memo, filled by the reference's function */
std::atomic<int> g_rdo_epoch{ 0 };     /* bumped when an encoder closes: earlier early posts are abandoned */
int g_gpus = 1;
bool g_stats_on = false;
pthread_once_t g_once = PTHREAD_ONCE_INIT;
pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;

struct Session
{
    x265amd_rdo* rdo = nullptr;
    int device = 0;
    int sign_hide = 0;
};
std::vector<Session> g_sessions;     /* per device session index (frame encoder id mod G) */
x265amd_rdo_counters g_closed{};

enum { ST_POSTS, ST_HOST_CUS, ST_TQ_HIT, ST_TQ_MISS, ST_ITQ_HIT, ST_ITQ_MISS, ST_PSY_HIT, ST_PSY_MISS, ST_CHECK_BAD,
       ST_EARLY_MERGE, ST_EARLY_INTER, ST_EARLY_BIDIR, ST_EARLY_USED, ST_EARLY_DROPPED, ST_SAO_DEV, ST_SAO_HOST,
       ST_SAO_BAD, ST_SSE_HIT, ST_SSE_MISS, ST_N };
std::atomic<int64_t> g_st[ST_N];
std::atomic<int64_t> g_wait_ns{ 0 };

pixelcmp_t g_psy_orig[NUM_CU_SIZES];
pixel_sse_t g_sse_orig[2][NUM_CU_SIZES];   /* the table's sse_pp: luma cu[], chroma[4:2:0].cu[] */

void print_stats()
{
    x265amd_rdo_counters c = g_closed;
    pthread_mutex_lock(&g_mu);
    for (Session& s : g_sessions)
    {
        x265amd_rdo_counters t;
        if (s.rdo && !x265amd_rdo_stats(s.rdo, &t))
        {
            c.batches += t.batches; c.requests += t.requests; c.tus += t.tus; c.blocks += t.blocks;
            c.kernel_ms += t.kernel_ms; c.batch_ms += t.batch_ms; c.queue_ms += t.queue_ms;
            c.waits += t.waits; c.waits_blocked += t.waits_blocked; c.wait_ms += t.wait_ms;
            c.sao_ctus += t.sao_ctus; c.sao_ms += t.sao_ms;
            if (t.max_requests_per_batch > c.max_requests_per_batch) c.max_requests_per_batch = t.max_requests_per_batch;
        }
    }
    pthread_mutex_unlock(&g_mu);
    fprintf(stderr, "[x265rdo] stats CUs posted %lld coded on the host %lld; transformNxN memo hits %lld misses %lld; "
                    "invtransformNxN hits %lld misses %lld; psy_cost_pp hits %lld misses %lld; worker wait %.3f s\n",
            (long long)g_st[ST_POSTS].load(), (long long)g_st[ST_HOST_CUS].load(), (long long)g_st[ST_TQ_HIT].load(),
            (long long)g_st[ST_TQ_MISS].load(), (long long)g_st[ST_ITQ_HIT].load(), (long long)g_st[ST_ITQ_MISS].load(),
            (long long)g_st[ST_PSY_HIT].load(), (long long)g_st[ST_PSY_MISS].load(), 1e-9 * g_wait_ns.load());
    fprintf(stderr, "[x265rdo] sse_pp memo hits %lld misses %lld\n", (long long)g_st[ST_SSE_HIT].load(),
            (long long)g_st[ST_SSE_MISS].load());
    if (g_early)
        fprintf(stderr, "[x265rdo] early posts merge %lld inter %lld bidir %lld; used %lld, dropped %lld\n",
                (long long)g_st[ST_EARLY_MERGE].load(), (long long)g_st[ST_EARLY_INTER].load(),
                (long long)g_st[ST_EARLY_BIDIR].load(), (long long)g_st[ST_EARLY_USED].load(),
                (long long)g_st[ST_EARLY_DROPPED].load());
    if (c.batches)
        fprintf(stderr, "[x265rdo] service: %lld batches, %lld CUs (%.2f per batch, max %lld), %lld TUs, %lld 8x8 blocks, "
                        "kernels %.3f ms per batch (HIP events), batch %.3f ms, queueing %.3f ms per CU, %lld waits slept\n",
                (long long)c.batches, (long long)c.requests, (double)c.requests / c.batches,
                (long long)c.max_requests_per_batch, (long long)c.tus, (long long)c.blocks, c.kernel_ms / c.batches,
                c.batch_ms / c.batches, c.requests ? c.queue_ms / c.requests : 0.0, (long long)c.waits_blocked);
    if (g_sao)
        fprintf(stderr, "[x265rdo] SAO statistics: %lld CTUs on the %s (%.3f ms each, post to result), %lld on the "
                        "host\n", (long long)g_st[ST_SAO_DEV].load(), g_sao_host ? "hook memo" : "device",
                c.sao_ctus ? c.sao_ms / c.sao_ctus : 0.0, (long long)g_st[ST_SAO_HOST].load());
    if (g_mode == RDO_CHECK)
        fprintf(stderr, "[x265rdo] check: %lld mismatches\n", (long long)(g_st[ST_CHECK_BAD].load() + g_st[ST_SAO_BAD].load()));
}

void init_once()
{
    const char* m = getenv("X265AMD_RDO");
    if (m && !strcmp(m, "gpu")) g_mode = RDO_GPU;
    else if (m && !strcmp(m, "check")) g_mode = RDO_CHECK;
    else if (m && !strcmp(m, "host")) g_mode = RDO_HOST;
    else g_mode = RDO_CPU;
    const char* e = getenv("X265AMD_RDO_MIN");
    if (e && *e) g_min_log2 = atoi(e) < 4 ? 4 : (atoi(e) > 6 ? 6 : atoi(e));
    e = getenv("X265AMD_RDO_LAUNCHERS");
    if (e && *e) g_launchers = atoi(e) < 0 ? 0 : atoi(e);     /* 0: direct mode (per-thread zero-copy launches) */
    e = getenv("X265AMD_RDO_EARLY");
    g_early = e && *e == '1' && (g_mode == RDO_GPU || g_mode == RDO_CHECK);
    e = getenv("X265AMD_GPUS");
    if (e && *e) g_gpus = atoi(e) < 1 ? 1 : atoi(e);
    /* the SAO statistics go to the resident server (direct mode with X265AMD_RDO_SERVER=1; default on there) */
    e = getenv("X265AMD_RDO_SAO");
    const char* srv = getenv("X265AMD_RDO_SERVER");
    g_sao = (g_mode == RDO_GPU || g_mode == RDO_CHECK) && g_launchers == 0 && srv && *srv == '1' && X265_DEPTH == 8 &&
            !(e && *e == '0');
    g_sao_host = e && !strcmp(e, "host");
    if (g_sao_host) g_sao = true;
    const char* st = getenv("X265AMD_ME_STATS");
    g_stats_on = (st && *st == '1') || g_mode == RDO_CHECK;
    if (g_sao_host)
    {
        fprintf(stderr, "[x265rdo] SAO statistics of each CTU on the CPU (hook memo)\n");
        if (g_mode == RDO_CPU && g_stats_on) atexit(print_stats);
    }
    if (g_mode != RDO_CPU)
    {
        fprintf(stderr, "[x265rdo] inter residual coding of CUs >= %dx%d %s\n", 1 << g_min_log2, 1 << g_min_log2,
                g_mode == RDO_CHECK ? "on the MI355X (check mode)" : g_mode == RDO_HOST ? "on the CPU (hook memo)" :
                                                                           "on the MI355X");
        if (g_early) fprintf(stderr, "[x265rdo] requests posted when the prediction is final (early posts)\n");
        if (g_sao && !g_sao_host) fprintf(stderr, "[x265rdo] SAO statistics of each CTU on the MI355X (resident server)\n");
        if (g_stats_on) atexit(print_stats);
    }
}

x265amd_rdo* session_for(const CUData& cu, int sign_hide)
{
    const int k = g_gpus > 1 ? cu.m_encData->m_frameEncoderID % g_gpus : 0;
    pthread_mutex_lock(&g_mu);
    if ((int)g_sessions.size() <= k) g_sessions.resize(k + 1);
    Session& s = g_sessions[k];
    if (!s.rdo)
    {
        int ndev = 1;
        if (x265amd_device_count(&ndev) || ndev < 1) ndev = 1;
        x265amd_rdo_config c = {};
        c.depth = X265_DEPTH;
        c.device = k % ndev;
        c.launchers = g_launchers;
        c.max_threads = 256;
        c.sign_hide = sign_hide;
        if (x265amd_rdo_create(&c, &s.rdo)) s.rdo = nullptr;
        s.sign_hide = sign_hide;
    }
    x265amd_rdo* r = s.sign_hide == sign_hide ? s.rdo : nullptr;
    pthread_mutex_unlock(&g_mu);
    return r;
}

/* the calling thread's memo: the device results of the CU whose encodeResAndCalcRdInterCU is running */
struct Memo
{
    bool active = false;
    const x265amd_rdo_result* res = nullptr;
    const pixel* fenc[3];
    intptr_t fstride[3];
    const pixel* pred[3];
    intptr_t pstride[3];
    const int16_t* resi[3];      /* the CU's residual buffer (m_rqt[depth].tmpResiYuv) */
    intptr_t rstride[3];
    int width[3];                /* plane width of the CU */
    struct Served
    {
        const coeff_t* coeff;
        int plane, tu;
    } served[48];
    int nserved = 0;
};
thread_local Memo t_memo;

inline bool tu_of(const Memo& m, int p, const int16_t* residual, uint32_t stride, uint32_t log2, int& tu, int& x,
                  int& y)
{
    const x265amd_rdo_result& r = *m.res;
    if ((int)log2 != r.tu_log2[p] || (intptr_t)stride != m.rstride[p]) return false;
    const ptrdiff_t off = residual - m.resi[p];
    if (off < 0) return false;
    y = (int)(off / m.rstride[p]);
    x = (int)(off % m.rstride[p]);
    const int n = 1 << log2;
    if (x >= m.width[p] || y >= m.width[p] || (x & (n - 1)) || (y & (n - 1))) return false;
    tu = (y >> log2) * (m.width[p] >> log2) + (x >> log2);
    return true;
}

/* is the 8x8 block at a (stride sa) equal to the one at b (stride sb)? */
inline bool same8(const pixel* a, intptr_t sa, const pixel* b, intptr_t sb)
{
    for (int i = 0; i < 8; i++)
        if (memcmp(a + i * sa, b + i * sb, 8 * sizeof(pixel))) return false;
    return true;
}

bool memo_psy(int size, const pixel* source, intptr_t sstride, const pixel* recon, intptr_t rstride, int& out)
{
    const Memo& m = t_memo;
    const x265amd_rdo_result& r = *m.res;
    for (int p = 0; p < 3; p++)
    {
        if (sstride != m.fstride[p]) continue;
        const ptrdiff_t off = source - m.fenc[p];
        if (off < 0) continue;
        const int y = (int)(off / m.fstride[p]), x = (int)(off % m.fstride[p]);
        const int dim = 1 << (size + 2), w = m.width[p];
        if (x + dim > w || y + dim > w || (x & 7) || (y & 7)) continue;
        const pixel* rec = (const pixel*)r.recon[p];
        int v = 0;
        for (int by = 0; by < dim; by += 8)
            for (int bx = 0; bx < dim; bx += 8)
            {
                const int b = ((y + by) >> 3) * (w >> 3) + ((x + bx) >> 3);
                const pixel* q = recon + by * rstride + bx;
                if (same8(q, rstride, m.pred[p] + (y + by) * m.pstride[p] + x + bx, m.pstride[p])) v += r.psy_pred[p][b];
                else if (same8(q, rstride, rec + (y + by) * w + x + bx, w)) v += r.psy_rec[p][b];
                else return false;
            }
        out = v;
        return true;
    }
    return false;
}

/* the CU's sse_pp (fenc against its prediction or its reconstruction, search.cpp:2591-2595, 2668-2679) from the
 * device's 8x8 SSEs: plane p's block at `source`, every 8x8 block of `recon` equal (compared) to the prediction's
 * (the device's sse_pred) or the device's reconstruction's (sse_rec) */
bool memo_sse(int dim, const pixel* source, intptr_t sstride, const pixel* recon, intptr_t rstride, sse_t& out)
{
    const Memo& m = t_memo;
    const x265amd_rdo_result& r = *m.res;
    if (!r.sse_pred[0]) return false;
    for (int p = 0; p < 3; p++)
    {
        /* a block of plane p of the CU (the whole CU, or a TU of it: estimateResidualQT's per-TU distortions) */
        if (sstride != m.fstride[p]) continue;
        const ptrdiff_t off = source - m.fenc[p];
        if (off < 0) continue;
        const int y = (int)(off / m.fstride[p]), x = (int)(off % m.fstride[p]);
        const int w = m.width[p];
        if (x + dim > w || y + dim > w || (x & 7) || (y & 7)) continue;
        const pixel* rec = (const pixel*)r.recon[p];
        sse_t v = 0;
        for (int by = 0; by < dim; by += 8)
            for (int bx = 0; bx < dim; bx += 8)
            {
                const int b = ((y + by) >> 3) * (w >> 3) + ((x + bx) >> 3);
                const pixel* q = recon + by * rstride + bx;
                if (same8(q, rstride, m.pred[p] + (y + by) * m.pstride[p] + x + bx, m.pstride[p])) v += (sse_t)r.sse_pred[p][b];
                else if (same8(q, rstride, rec + (y + by) * w + x + bx, w)) v += (sse_t)r.sse_rec[p][b];
                else return false;
            }
        out = v;
        return true;
    }
    return false;
}

template <int chroma, int size>
sse_t sse_thunk(const pixel* fenc, intptr_t fstride, const pixel* ref, intptr_t rstride)
{
    if (t_memo.active)
    {
        sse_t v;
        if (memo_sse(chroma ? 1 << (size + 1) : 1 << (size + 2), fenc, fstride, ref, rstride, v))
        {
            g_st[ST_SSE_HIT]++;
            if (g_mode == RDO_CHECK && v != g_sse_orig[chroma][size](fenc, fstride, ref, rstride)) g_st[ST_CHECK_BAD]++;
            return v;
        }
        g_st[ST_SSE_MISS]++;
    }
    return g_sse_orig[chroma][size](fenc, fstride, ref, rstride);
}

template <int size>
int psy_thunk(const pixel* source, intptr_t sstride, const pixel* recon, intptr_t rstride)
{
    if (t_memo.active)
    {
        int v;
        if (memo_psy(size, source, sstride, recon, rstride, v))
        {
            g_st[ST_PSY_HIT]++;
            if (g_mode == RDO_CHECK && v != g_psy_orig[size](source, sstride, recon, rstride)) g_st[ST_CHECK_BAD]++;
            return v;
        }
        g_st[ST_PSY_MISS]++;
    }
    return g_psy_orig[size](source, sstride, recon, rstride);
}

/* CU eligible for the device: the TU structure and quantisation the session restates (one RQT level of
 * min(CU, 32) TUs, plain quant with sign hiding, no transform skip / lossless / RDOQ / scaling lists /
 * noise reduction, 4:2:0 2Nx2N) */
bool eligible(Search& s, int csp, const Mode& mode, int log2)
{
    const CUData& cu = mode.cu;
    if (log2 < g_min_log2 || log2 > 6 || csp != X265_CSP_I420) return false;
    if (cu.m_tqBypass[0] || cu.m_partSize[0] != SIZE_2Nx2N || cu.isIntra(0)) return false;
    if (s.m_bEnableRDOQ || s.m_quant.*QuantPeek::rdoq()) return false;
    if (s.m_slice->m_pps->bTransformSkipEnabled || s.m_slice->m_pps->bTransquantBypassEnabled) return false;
    const ScalingList* sl = s.m_quant.*QuantPeek::scaling();
    if (sl && sl->m_bEnabled) return false;
    if (s.m_quant.m_nr && s.m_quant.m_nr->offset) return false;
    uint32_t dr[2];
    cu.getInterTUQtDepthRange(dr, 0);
    const uint32_t tl = log2 < 5 ? (uint32_t)log2 : 5u;
    return dr[0] == tl && dr[1] >= tl;
}

void activate(Memo& m, const x265amd_rdo_result* res, const Yuv& fenc, const Yuv& pred, const ShortYuv& resi, int log2cu)
{
    m.res = res;
    m.nserved = 0;
    const int c = 1 << log2cu;
    for (int p = 0; p < 3; p++)
    {
        m.fenc[p] = fenc.m_buf[p];
        m.fstride[p] = p ? fenc.m_csize : fenc.m_size;
        m.pred[p] = pred.m_buf[p];
        m.pstride[p] = p ? pred.m_csize : pred.m_size;
        m.resi[p] = resi.m_buf[p];
        m.rstride[p] = p ? resi.m_csize : resi.m_size;
        m.width[p] = p ? c >> 1 : c;
    }
    m.active = true;
}

} // namespace

/* the binding installs its psy_cost_pp thunks into the encoder's table (oracle/hip_encoder_main.cpp, after
 * the table is set up); every other entry stays the table's */
extern "C" void x265amd_rdo_install(void* table)
{
    pthread_once(&g_once, init_once);
    if (g_mode == RDO_CPU) return;
    EncoderPrimitives& p = *(EncoderPrimitives*)table;
    for (int i = 0; i < NUM_CU_SIZES; i++) g_psy_orig[i] = p.cu[i].psy_cost_pp;
    p.cu[BLOCK_8x8].psy_cost_pp = psy_thunk<1>;
    p.cu[BLOCK_16x16].psy_cost_pp = psy_thunk<2>;
    p.cu[BLOCK_32x32].psy_cost_pp = psy_thunk<3>;
    p.cu[BLOCK_64x64].psy_cost_pp = psy_thunk<4>;
    /* the distortions of a device CU and of its TUs: luma 8..64, 4:2:0 chroma 8..32 (X265AMD_RDO_SSE=0: the table's) */
    const char* e = getenv("X265AMD_RDO_SSE");
    if (e && *e == '0') return;
    for (int i = 0; i < NUM_CU_SIZES; i++)
    {
        g_sse_orig[0][i] = p.cu[i].sse_pp;
        g_sse_orig[1][i] = p.chroma[X265_CSP_I420].cu[i].sse_pp;
    }
    p.cu[BLOCK_8x8].sse_pp = sse_thunk<0, 1>;
    p.cu[BLOCK_16x16].sse_pp = sse_thunk<0, 2>;
    p.cu[BLOCK_32x32].sse_pp = sse_thunk<0, 3>;
    p.cu[BLOCK_64x64].sse_pp = sse_thunk<0, 4>;
    p.chroma[X265_CSP_I420].cu[BLOCK_16x16].sse_pp = sse_thunk<1, 2>;
    p.chroma[X265_CSP_I420].cu[BLOCK_32x32].sse_pp = sse_thunk<1, 3>;
    p.chroma[X265_CSP_I420].cu[BLOCK_64x64].sse_pp = sse_thunk<1, 4>;
}

/* called by the encoder binding before x265_encoder_close frees the encoder (oracle/hip_encoder_main.cpp) */
extern "C" void x265amd_rdo_encoder_closed(void)
{
    g_rdo_epoch++;
    pthread_mutex_lock(&g_mu);
    for (Session& s : g_sessions)
    {
        x265amd_rdo_counters t;
        if (s.rdo && !x265amd_rdo_stats(s.rdo, &t))
        {
            g_closed.batches += t.batches; g_closed.requests += t.requests; g_closed.tus += t.tus;
            g_closed.blocks += t.blocks; g_closed.kernel_ms += t.kernel_ms; g_closed.batch_ms += t.batch_ms;
            g_closed.queue_ms += t.queue_ms; g_closed.waits += t.waits; g_closed.waits_blocked += t.waits_blocked;
            g_closed.wait_ms += t.wait_ms;
            g_closed.sao_ctus += t.sao_ctus; g_closed.sao_ms += t.sao_ms;
            if (t.max_requests_per_batch > g_closed.max_requests_per_batch)
                g_closed.max_requests_per_batch = t.max_requests_per_batch;
        }
        x265amd_rdo_destroy(s.rdo);
    }
    g_sessions.clear();
    pthread_mutex_unlock(&g_mu);
}

namespace {

/* X265AMD_RDO=host: the session's results computed on the calling thread by the reference's own functions,
 * in the session's layout (x265amd_rdo_result) */
struct HostResult
{
    pixel recon[64 * 64 + 2 * 32 * 32];
    int16_t resi[64 * 64 + 2 * 32 * 32];
    coeff_t coeff[64 * 64 + 2 * 32 * 32];
    uint32_t sig[4 + 2 * 4];
    int32_t psyp[64 + 2 * 16], psyr[64 + 2 * 16];
    x265amd_rdo_result res;
};
thread_local HostResult* t_host;

const x265amd_rdo_result* host_result(Quant& q, const CUData& cu, int log2cu, const Yuv& fenc, const Yuv& pred)
{
    if (!t_host) t_host = new HostResult();
    HostResult& h = *t_host;
    x265amd_rdo_result& r = h.res;
    r.log2_cu = log2cu;
    const int c = 1 << log2cu, tl = log2cu < 5 ? log2cu : 5;
    size_t po = 0;
    int to = 0, bo = 0;
    for (int p = 0; p < 3; p++)
    {
        const int w = p ? c >> 1 : c, t = p ? tl - 1 : tl, n = 1 << t, per = w >> t;
        const pixel* f = fenc.m_buf[p];
        const pixel* pr = pred.m_buf[p];
        const intptr_t fs = p ? fenc.m_csize : fenc.m_size, ps = p ? pred.m_csize : pred.m_size;
        pixel* rec = h.recon + po;
        int16_t* res = h.resi + po;
        coeff_t* co = h.coeff + po;
        for (int y = 0; y < w; y++)
            for (int x = 0; x < w; x++)
            {
                res[y * w + x] = (int16_t)(f[y * fs + x] - pr[y * ps + x]);
                rec[y * w + x] = pr[y * ps + x];
            }
        r.tu_log2[p] = t;
        r.ntu[p] = per * per;
        for (int k = 0; k < per * per; k++)
        {
            const int x = (k % per) * n, y = (k / per) * n;
            const uint32_t ns = x265ref_transformNxN(&q, cu, f + y * fs + x, (uint32_t)fs, res + y * w + x, (uint32_t)w,
                                                     co + (size_t)k * n * n, (uint32_t)t, (TextType)p, 0, false);
            h.sig[to + k] = ns;
            if (ns)
            {
                x265ref_invtransformNxN(&q, cu, res + y * w + x, (uint32_t)w, co + (size_t)k * n * n, (uint32_t)t,
                                        (TextType)p, false, false, ns);
                primitives.cu[t - 2].add_ps(rec + y * w + x, w, pr + y * ps + x, res + y * w + x, ps, w);
            }
        }
        const int nb = (w >> 3) * (w >> 3);
        for (int b = 0; b < nb; b++)
        {
            const int x = (b % (w >> 3)) * 8, y = (b / (w >> 3)) * 8;
            h.psyp[bo + b] = g_psy_orig[BLOCK_8x8](f + y * fs + x, fs, pr + y * ps + x, ps);
            h.psyr[bo + b] = g_psy_orig[BLOCK_8x8](f + y * fs + x, fs, rec + y * w + x, w);
        }
        r.recon[p] = rec;
        r.resi[p] = res;
        r.coeff[p] = co;
        r.num_sig[p] = h.sig + to;
        r.psy_pred[p] = h.psyp + bo;
        r.psy_rec[p] = h.psyr + bo;
        po += (size_t)w * w;
        to += per * per;
        bo += nb;
    }
    return &r;
}

/* the request of one CU posted when its prediction became final (X265AMD_RDO_EARLY=1) */
enum { EARLY_MERGE, EARLY_INTER, EARLY_BIDIR, EARLY_N };
struct Early
{
    x265amd_rdo* rdo = nullptr;
    int ticket = -1;
    int epoch = 0;
    int log2 = 0;
    uint8_t qp[3];
    const pixel* fenc[3];
    pixel pred[64 * 64 + 2 * 32 * 32];       /* the posted prediction, planes packed (stride = plane width) */
};
thread_local Early* t_early;

void early_drop(Early& e)
{
    if (e.ticket < 0) return;
    if (e.epoch == g_rdo_epoch.load())
    {
        /* (a request's slot is reusable once its results are in; an early post is long done by now) */
        const x265amd_rdo_result* r;
        (void)x265amd_rdo_wait(e.rdo, e.ticket, &r);
        (void)x265amd_rdo_release(e.rdo, e.ticket);
    }
    e.ticket = -1;
}

/* fill the request of the CU whose prediction is `pred` with the Quant object's current QPs */
void request_of(Search& s, int log2, const Yuv& fenc, const Yuv& pred, x265amd_rdo_cu& in)
{
    in = {};
    in.log2_cu = log2;
    for (int p = 0; p < 3; p++)
    {
        in.qp[p] = (uint8_t)(s.m_quant.*QuantPeek::qp())[p].qp;
        in.fenc[p] = fenc.m_buf[p];
        in.fenc_stride[p] = p ? fenc.m_csize : fenc.m_size;
        in.pred[p] = pred.m_buf[p];
        in.pred_stride[p] = p ? pred.m_csize : pred.m_size;
    }
}

void early_post(Search& s, const Mode& mode, int log2, int slot)
{
    pthread_once(&g_once, init_once);
    if (!g_early || !mode.fencYuv || !eligible(s, mode.cu.m_chromaFormat, mode, log2)) return;
    if (!t_early) t_early = new Early[EARLY_N];
    Early& e = t_early[slot];
    if (e.ticket >= 0)
    {
        g_st[ST_EARLY_DROPPED]++;
        early_drop(e);
    }
    x265amd_rdo* rdo = session_for(mode.cu, s.m_slice->m_pps->bSignHideEnabled ? 1 : 0);
    if (!rdo) return;
    const int c = 1 << log2;
    x265amd_rdo_cu in;
    request_of(s, log2, *mode.fencYuv, mode.predYuv, in);
    int ticket = -1;
    if (x265amd_rdo_post(rdo, &in, &ticket)) return;
    e.rdo = rdo;
    e.ticket = ticket;
    e.epoch = g_rdo_epoch.load();
    e.log2 = log2;
    pixel* d = e.pred;
    for (int p = 0; p < 3; p++)
    {
        e.qp[p] = in.qp[p];
        e.fenc[p] = mode.fencYuv->m_buf[p];
        const int w = p ? c >> 1 : c;
        for (int y = 0; y < w; y++, d += w)
            memcpy(d, mode.predYuv.m_buf[p] + y * in.pred_stride[p], w * sizeof(pixel));
    }
    g_st[ST_EARLY_MERGE + slot]++;
}

/* the early post made for this call, if any: same size, source buffer, QPs and prediction */
Early* early_match(Search& s, const Mode& mode, int log2)
{
    if (!t_early) return nullptr;
    const int c = 1 << log2;
    for (int k = 0; k < EARLY_N; k++)
    {
        Early& e = t_early[k];
        if (e.ticket < 0 || e.epoch != g_rdo_epoch.load() || e.log2 != log2) continue;
        bool same = true;
        const pixel* d = e.pred;
        for (int p = 0; p < 3 && same; p++)
        {
            const int w = p ? c >> 1 : c;
            const intptr_t ps = p ? mode.predYuv.m_csize : mode.predYuv.m_size;
            same = e.fenc[p] == mode.fencYuv->m_buf[p] &&
                   e.qp[p] == (uint8_t)(s.m_quant.*QuantPeek::qp())[p].qp;
            for (int y = 0; y < w && same; y++, d += w)
                same = !memcmp(d, mode.predYuv.m_buf[p] + y * ps, w * sizeof(pixel));
        }
        if (same) return &e;
    }
    return nullptr;
}

} // namespace

/* Search::predInterSearch's hook (gpu_me.cpp) after the reference's search: the 2Nx2N prediction is final */
extern "C" void x265amd_rdo_early_inter(void* search, void* mode, const void* geom, int chroma_mc)
{
    Mode& m = *(Mode*)mode;
    if (chroma_mc && m.cu.m_partSize[0] == SIZE_2Nx2N)
        early_post(*(Search*)search, m, (int)((const CUGeom*)geom)->log2CUSize, EARLY_INTER);
}

namespace X265_NS {

void Analysis::checkBidir2Nx2N(Mode& inter2Nx2N, Mode& bidir2Nx2N, const CUGeom& cuGeom)
{
    x265ref_checkBidir2Nx2N(this, inter2Nx2N, bidir2Nx2N, cuGeom);
    if (g_early && bidir2Nx2N.sa8dCost != MAX_INT64 && m_bChromaSa8d)
        early_post(*this, bidir2Nx2N, (int)cuGeom.log2CUSize, EARLY_BIDIR);
}

void Search::encodeResAndCalcRdSkipCU(Mode& interMode)
{
    pthread_once(&g_once, init_once);
    /* the best merge candidate's prediction, coded next with residual (analysis.cpp:1739-1752) */
    if (g_early)
        early_post(*this, interMode, (int)interMode.cu.m_log2CUSize[0], EARLY_MERGE);
    x265ref_encodeResAndCalcRdSkipCU(this, interMode);
}

void Search::encodeResAndCalcRdInterCU(Mode& interMode, const CUGeom& cuGeom)
{
    pthread_once(&g_once, init_once);
    Memo& m = t_memo;
    if (g_mode == RDO_CPU || m.active || !eligible(*this, m_csp, interMode, (int)cuGeom.log2CUSize))
    {
        x265ref_encodeResAndCalcRdInterCU(this, interMode, cuGeom);
        return;
    }
    if (g_early)
    {
        Early* e = early_match(*this, interMode, (int)cuGeom.log2CUSize);
        const x265amd_rdo_result* res = nullptr;
        struct timespec t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        const int rc = e ? x265amd_rdo_wait(e->rdo, e->ticket, &res) : -1;
        clock_gettime(CLOCK_MONOTONIC, &t1);
        g_wait_ns += (int64_t)(t1.tv_sec - t0.tv_sec) * 1000000000 + (t1.tv_nsec - t0.tv_nsec);
        if (!e || rc)
        {
            if (e) { (void)x265amd_rdo_release(e->rdo, e->ticket); e->ticket = -1; }
            g_st[ST_HOST_CUS]++;
            x265ref_encodeResAndCalcRdInterCU(this, interMode, cuGeom);
            return;
        }
        g_st[ST_POSTS]++;
        g_st[ST_EARLY_USED]++;
        activate(m, res, *interMode.fencYuv, interMode.predYuv, m_rqt[cuGeom.depth].tmpResiYuv, (int)cuGeom.log2CUSize);
        x265ref_encodeResAndCalcRdInterCU(this, interMode, cuGeom);
        m.active = false;
        m.res = nullptr;
        (void)x265amd_rdo_release(e->rdo, e->ticket);
        e->ticket = -1;
        return;
    }
    const Yuv& fenc = *interMode.fencYuv;
    const Yuv& pred = interMode.predYuv;
    x265amd_rdo* rdo = nullptr;
    if (g_mode == RDO_HOST)
    {
        g_st[ST_POSTS]++;
        activate(m, host_result(m_quant, interMode.cu, (int)cuGeom.log2CUSize, fenc, pred), fenc, pred,
                 m_rqt[cuGeom.depth].tmpResiYuv, (int)cuGeom.log2CUSize);
        x265ref_encodeResAndCalcRdInterCU(this, interMode, cuGeom);
        m.active = false;
        m.res = nullptr;
        return;
    }
    rdo = session_for(interMode.cu, m_slice->m_pps->bSignHideEnabled ? 1 : 0);
    x265amd_rdo_cu in = {};
    in.log2_cu = (int)cuGeom.log2CUSize;
    for (int p = 0; p < 3; p++)
    {
        in.qp[p] = (uint8_t)(m_quant.*QuantPeek::qp())[p].qp;
        in.fenc[p] = fenc.m_buf[p];
        in.fenc_stride[p] = p ? fenc.m_csize : fenc.m_size;
        in.pred[p] = pred.m_buf[p];
        in.pred_stride[p] = p ? pred.m_csize : pred.m_size;
    }
    int ticket = -1;
    const x265amd_rdo_result* res = nullptr;
    if (!rdo || x265amd_rdo_post(rdo, &in, &ticket))
    {
        g_st[ST_HOST_CUS]++;
        x265ref_encodeResAndCalcRdInterCU(this, interMode, cuGeom);
        return;
    }
    g_st[ST_POSTS]++;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    const int rc = x265amd_rdo_wait(rdo, ticket, &res);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    g_wait_ns += (int64_t)(t1.tv_sec - t0.tv_sec) * 1000000000 + (t1.tv_nsec - t0.tv_nsec);
    if (rc)
    {
        /* recorded in the sticky status (the encode fails); the CU is coded on the host meanwhile */
        (void)x265amd_rdo_release(rdo, ticket);
        g_st[ST_HOST_CUS]++;
        x265ref_encodeResAndCalcRdInterCU(this, interMode, cuGeom);
        return;
    }
    activate(m, res, fenc, pred, m_rqt[cuGeom.depth].tmpResiYuv, (int)cuGeom.log2CUSize);
    x265ref_encodeResAndCalcRdInterCU(this, interMode, cuGeom);
    m.active = false;
    m.res = nullptr;
    (void)x265amd_rdo_release(rdo, ticket);
}

uint32_t Quant::transformNxN(const CUData& cu, const pixel* fenc, uint32_t fencStride, const int16_t* residual,
                             uint32_t resiStride, coeff_t* coeff, uint32_t log2TrSize, TextType ttype,
                             uint32_t absPartIdx, bool useTransformSkip)
{
    Memo& m = t_memo;
    int tu, x, y;
    const int p = (int)ttype;
    if (m.active && !useTransformSkip && p >= 0 && p < 3 && tu_of(m, p, residual, resiStride, log2TrSize, tu, x, y) &&
        (intptr_t)fencStride == m.fstride[p] && fenc == m.fenc[p] + y * m.fstride[p] + x && m.nserved < 48)
    {
        const int nn = 1 << (2 * log2TrSize);
        const coeff_t* dc = m.res->coeff[p] + (size_t)tu * nn;
        const uint32_t ns = m.res->num_sig[p][tu];
        g_st[ST_TQ_HIT]++;
        if (g_mode == RDO_CHECK)
        {
            coeff_t tmp[32 * 32];
            const uint32_t hs = x265ref_transformNxN(this, cu, fenc, fencStride, residual, resiStride, tmp, log2TrSize,
                                                     ttype, absPartIdx, useTransformSkip);
            if (hs != ns || memcmp(tmp, dc, nn * sizeof(coeff_t))) g_st[ST_CHECK_BAD]++;
        }
        memcpy(coeff, dc, nn * sizeof(coeff_t));
        m.served[m.nserved++] = { coeff, p, tu };
        return ns;
    }
    if (m.active) g_st[ST_TQ_MISS]++;
    return x265ref_transformNxN(this, cu, fenc, fencStride, residual, resiStride, coeff, log2TrSize, ttype, absPartIdx,
                                useTransformSkip);
}

void Quant::invtransformNxN(const CUData& cu, int16_t* residual, uint32_t resiStride, const coeff_t* coeff,
                            uint32_t log2TrSize, TextType ttype, bool bIntra, bool useTransformSkip, uint32_t numSig)
{
    Memo& m = t_memo;
    const int p = (int)ttype;
    if (m.active && !bIntra && !useTransformSkip && p >= 0 && p < 3 && (int)log2TrSize == m.res->tu_log2[p])
    {
        for (int i = m.nserved - 1; i >= 0; i--)
        {
            const Memo::Served& sv = m.served[i];
            if (sv.coeff != coeff || sv.plane != p) continue;
            const int nn = 1 << (2 * log2TrSize), n = 1 << log2TrSize;
            if (m.res->num_sig[p][sv.tu] != numSig || memcmp(coeff, m.res->coeff[p] + (size_t)sv.tu * nn, nn * sizeof(coeff_t)))
                break;
            const int w = m.width[p], per = w >> log2TrSize;
            const int16_t* src = m.res->resi[p] + (size_t)((sv.tu / per) * n) * w + (sv.tu % per) * n;
            g_st[ST_ITQ_HIT]++;
            if (g_mode == RDO_CHECK)
            {
                int16_t tmp[32 * 32];
                x265ref_invtransformNxN(this, cu, tmp, n, coeff, log2TrSize, ttype, bIntra, useTransformSkip, numSig);
                for (int r = 0; r < n; r++)
                    if (memcmp(tmp + r * n, src + (size_t)r * w, n * sizeof(int16_t))) { g_st[ST_CHECK_BAD]++; break; }
            }
            for (int r = 0; r < n; r++) memcpy(residual + (size_t)r * resiStride, src + (size_t)r * w, n * sizeof(int16_t));
            return;
        }
        g_st[ST_ITQ_MISS]++;
    }
    x265ref_invtransformNxN(this, cu, residual, resiStride, coeff, log2TrSize, ttype, bIntra, useTransformSkip, numSig);
}

/* SAO::calcSaoStatsCu (sao.cpp:772-943): rdoSaoUnitCu / rdoSaoUnitRow call it for planes 0, 1, 2 of a CTU in turn
 * (sao.cpp:1276-1283, 1385-1392), on m_count / m_offsetOrg zeroed (or holding the pre-deblocking statistics) just
 * before.  The first call of a CTU has the server compute all three planes from the deblocked reconstruction as it
 * is at that moment (x265amd_rdo_sao_stats, synchronous: the reference reads it at the same point); each call adds
 * its plane's part, as the reference's primitives add theirs.  Anything not served runs the reference's code. */
namespace {
struct SaoMemo
{
    const SAO* sao = nullptr;
    const Frame* frame = nullptr;
    int poc = -1, addr = -1;
    int32_t stats[3 * 5 * 33], count[3 * 5 * 33];
};
thread_local SaoMemo t_sao;
}

void SAO::calcSaoStatsCu(int addr, int plane)
{
    pthread_once(&g_once, init_once);
    SaoMemo& mm = t_sao;
    if (!g_sao || m_chromaFormat != X265_CSP_I420 || g_maxLog2CUSize != 6 || plane < 0 || plane > 2)
    {
        x265ref_calcSaoStatsCu(this, addr, plane);
        return;
    }
    if (!(mm.sao == this && mm.frame == m_frame && mm.poc == m_frame->m_poc && mm.addr == addr))
    {
        mm.sao = nullptr;
        const CUData* ctu = m_frame->m_encData->getPicCTU(addr);
        x265amd_rdo* rdo = g_sao_host ? nullptr : session_for(*ctu, m_frame->m_encData->m_slice->m_pps->bSignHideEnabled ? 1 : 0);
        if (g_sao_host)
        {
            /* the plumbing on a CPU-only host: all three planes by the reference's function on zeroed statistics
             * (the members are restored), served through the memo like the device's */
            PerPlane c0, s0;
            memcpy(c0, m_count, sizeof(c0));
            memcpy(s0, m_offsetOrg, sizeof(s0));
            memset(m_count, 0, sizeof(m_count));
            memset(m_offsetOrg, 0, sizeof(m_offsetOrg));
            for (int p = 0; p < 3; p++) x265ref_calcSaoStatsCu(this, addr, p);
            memcpy(mm.stats, m_offsetOrg, sizeof(mm.stats));
            memcpy(mm.count, m_count, sizeof(mm.count));
            memcpy(m_count, c0, sizeof(c0));
            memcpy(m_offsetOrg, s0, sizeof(s0));
            mm.sao = this;
            mm.frame = m_frame;
            mm.poc = m_frame->m_poc;
            mm.addr = addr;
        }
        else if (rdo)
        {
            const PicYuv* rec = m_frame->m_reconPic;
            const PicYuv* src = m_frame->m_fencPic;
            x265amd_rdo_sao_ctu q = {};
            q.width = m_param->sourceWidth;
            q.height = m_param->sourceHeight;
            q.ctu_log2 = (int)g_maxLog2CUSize;
            q.cx = (int)(ctu->m_cuPelX >> g_maxLog2CUSize);
            q.cy = (int)(ctu->m_cuPelY >> g_maxLog2CUSize);
            q.non_deblocked = m_param->bSaoNonDeblocked ? 1 : 0;
            q.chroma_format = m_chromaFormat;
            for (int p = 0; p < 3; p++)
            {
                q.rec[p] = rec->getPlaneAddr(p, addr);
                q.rec_stride[p] = p ? rec->m_strideC : rec->m_stride;
                q.fenc[p] = src->getPlaneAddr(p, addr);
                q.fenc_stride[p] = p ? src->m_strideC : src->m_stride;
            }
            if (x265amd_rdo_sao_stats(rdo, &q, mm.stats, mm.count) == 0)
            {
                mm.sao = this;
                mm.frame = m_frame;
                mm.poc = m_frame->m_poc;
                mm.addr = addr;
            }
        }
        if (!mm.sao)
        {
            g_st[ST_SAO_HOST]++;
            x265ref_calcSaoStatsCu(this, addr, plane);
            return;
        }
        g_st[ST_SAO_DEV]++;
    }
    const int32_t* ds = mm.stats + plane * 5 * 33;
    const int32_t* dc = mm.count + plane * 5 * 33;
    if (g_mode == RDO_CHECK)
    {
        /* the reference's own statistics of the plane, compared with the device's part (the reference's stay) */
        int32_t s0[5][33], c0[5][33];
        memcpy(s0, m_offsetOrg[plane], sizeof(s0));
        memcpy(c0, m_count[plane], sizeof(c0));
        x265ref_calcSaoStatsCu(this, addr, plane);
        bool bad = false;
        for (int t = 0; t < 5; t++)
            for (int k = 0; k < 33; k++)
                bad |= m_offsetOrg[plane][t][k] - s0[t][k] != ds[t * 33 + k] || m_count[plane][t][k] - c0[t][k] != dc[t * 33 + k];
        if (bad) g_st[ST_SAO_BAD]++;
        return;
    }
    for (int t = 0; t < 5; t++)
        for (int k = 0; k < 33; k++)
        {
            m_offsetOrg[plane][t][k] += ds[t * 33 + k];
            m_count[plane][t][k] += dc[t * 33 + k];
        }
}

} // namespace X265_NS
