/* gpu_me.cpp — reference-side binding: the main encoder's motion searches of large PUs run on
 * the MI355X through the f2 session entries of include/x265_amd.h (x265amd_mes_*).
 *
 * This is the hook a maintainer adds to the encoder.  oracle/Makefile links
 * the reference encoder with copies of search.o and motion.o in which exactly two symbols are
 * weak (objcopy -W) and the originals stay reachable under aliases:
 *
 *   Search::predInterSearch(Mode&, const CUGeom&, bool, uint32_t[2])      search.cpp:2050-2420
 *     -> a PREFETCH, then the reference's own predInterSearch (x265ref_predInterSearch) unchanged.
 *        The prefetch forms, for the PU of a 2Nx2N CU of at least X265AMD_ME_MIN pixels
 *        (default 64x64), every search the unidirectional loop (:2181-2230) is about to make —
 *        per (list, reference) allowed by refMasks: the AMVP candidates (getPMV), the lowres MV,
 *        and for EACH of the two AMVP predictors (selectMVP, :2199, picks one of them) its search
 *        range (setSearchRange) — and runs all of them in ONE device launch
 *        (x265amd_mes_search: one wavefront group per search), after making the reference rows
 *        the encoder has finished resident on the device (x265amd_mes_ref);
 *   MotionEstimate::motionEstimate(ref, mvmin, mvmax, qmvp, n, mvc, merange, outQMv)
 *                                                                          motion.cpp:571-1172
 *     -> when the calling thread's prefetch holds a search with exactly these inputs (same
 *        MotionEstimate, reference planes, range, predictor, candidates and merange), its result,
 *        with the call's two side effects on the MotionEstimate (blockOffset, setMVP); otherwise
 *        the reference's own motionEstimate (x265ref_motionEstimate).
 *
 * So the encoder's control flow stays the reference's code: the hook only decides where the
 * searches' arithmetic runs, and a search is taken from the device only when its inputs are
 * identical to the reference call's.  The bitstream equals the reference encoder's
 * (tests/test_encoder_me.py).  Not prefetched (searched on the host): weighted references (the
 * device holds the unweighted reconstruction), chroma-SATD sub-pel (subme > 2), analysis load,
 * --pme, PUs of rectangular / AMP partitions, and PUs below the size threshold (a device round trip
 * costs more than a small search on one core).
 *
 *   X265AMD_ME=gpu     (default with the device lookahead) device searches
 *   X265AMD_ME=cpu     every call goes to the reference's functions (same binary)
 *   X265AMD_ME=host    the prefetch runs with the reference's motionEstimate on the host: checks the
 *                      hook's restated search setup and the memo on a CPU-only host
 *   X265AMD_ME=check   device searches, each compared with the host search when it is used
 *   X265AMD_ME_STATS=1 prefetches, searches, memo hits / misses and wall time, printed at exit
 *
 * Errors: a failing device call is recorded in the backend's sticky status (the encode then fails:
 * hip_encoder_main.cpp turns it into x265_encoder_encode() < 0); that PU is searched on the host so
 * the encoder's state stays valid until it stops.
 */
#include "common.h"
#include "primitives.h"
#include "frame.h"
#include "picyuv.h"
#include "slice.h"
#include "search.h"
#include "analysis.h"
#include "motion.h"
#include "reference.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <pthread.h>
#include <vector>

#include "../include/x265_amd.h"

using namespace X265_NS;

/* the reference's own implementations (aliases of the weakened symbols, see oracle/Makefile) */
extern "C" void x265ref_predInterSearch(Search* self, Mode& interMode, const CUGeom& cuGeom, bool bChromaMC,
                                        uint32_t refMasks[2]);
extern "C" int x265ref_motionEstimate(MotionEstimate* self, ReferencePlanes* ref, const MV& mvmin, const MV& mvmax,
                                      const MV& qmvp, int numCandidates, const MV* mvc, int merange, MV& outQMv);
extern "C" SplitData x265ref_compressInterCU_rd0_4(Analysis* self, const CUData& parentCTU, const CUGeom& cuGeom,
                                                   int32_t qp);

namespace {

/* BitCost::m_cost (the BitCost table of the current QP, bitcost.cpp:31-57) is protected; a
 * pointer to the member taken through a derived class reads it from a MotionEstimate */
struct CostPeek : public MotionEstimate
{
    static uint16_t* BitCost::*member() { return &CostPeek::m_cost; }
};

enum { ME_GPU = 0, ME_CPU = 1, ME_HOST = 2, ME_CHECK = 3 };
int g_mode = ME_GPU;
/* X265AMD_ME_ASYNC=1: the 64x64 searches of every reference submitted at the CTU's start and collected at
 * predInterSearch; measured neutral at 64x64-only (2160p, 3 interleaved runs: 8.29 / 8.39 / 8.54 fps against
 * 8.60 / 8.27 / 8.44 synchronous, profiles/r04/encoder_me_async_ab.txt), so the synchronous form is the default */
bool g_async = false;
int g_min_area = 64 * 64;      /* measured: 64x64 only beats 32x32 + 64x64 (profiles/r04/encoder_me_variants.txt) */
bool g_stats_on = false;
pthread_once_t g_once = PTHREAD_ONCE_INIT;
pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
int g_status = 0;

struct Stats { long prefetch, searches, hits, misses, skipped, fallbacks, mismatches; double sec; };
Stats g_st;

double now_s()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

void print_stats()
{
    fprintf(stderr, "[x265me] stats prefetches %ld searches %ld memo hits %ld misses %ld host fallbacks %ld "
                    "weighted-reference searches %ld device %.1f ms (%.3f ms/prefetch)\n", g_st.prefetch, g_st.searches,
            g_st.hits, g_st.misses, g_st.fallbacks, g_st.skipped, 1e3 * g_st.sec,
            g_st.prefetch ? 1e3 * g_st.sec / g_st.prefetch : 0.0);
    if (g_mode == ME_CHECK)
        fprintf(stderr, "[x265me] check: %ld mismatching searches\n", g_st.mismatches);
}

void read_mode()
{
    const char* m = getenv("X265AMD_ME");
    const char* la = getenv("X265AMD_LOOKAHEAD");
    const bool la_cpu = la && (!strcmp(la, "cpu") || !strcmp(la, "host"));
    g_mode = (m && !strcmp(m, "cpu")) ? ME_CPU : (m && !strcmp(m, "host")) ? ME_HOST :
             (m && !strcmp(m, "check")) ? ME_CHECK : (m && !strcmp(m, "gpu")) ? ME_GPU : la_cpu ? ME_CPU : ME_GPU;
    if (const char* a = getenv("X265AMD_ME_MIN"))
        g_min_area = atoi(a);
    if (const char* a = getenv("X265AMD_ME_ASYNC"))
        g_async = atoi(a) != 0;
    const char* st = getenv("X265AMD_ME_STATS");
    g_stats_on = (st && *st && strcmp(st, "0")) || g_mode == ME_CHECK;
    fprintf(stderr, "[x265me] motion searches of PUs >= %d pixels on %s\n", g_min_area,
            g_mode == ME_CPU ? "the CPU (reference functions)" : g_mode == ME_HOST ? "the CPU (hook prefetch)" :
            g_mode == ME_CHECK ? "the MI355X, each checked against the CPU" : "the MI355X");
    if (g_stats_on)
        atexit(print_stats);
}

void stat_add(long Stats::*field, long v)
{
    if (!g_stats_on) return;
    pthread_mutex_lock(&g_mu);
    g_st.*field += v;
    pthread_mutex_unlock(&g_mu);
}

/* one session per reconstructed-picture geometry and search setting (a second encoder of another size
 * or --me / --subme / --merange in the same process gets its own) */
struct Session { intptr_t stride; int64_t elems; int64_t org; int rows, method, subme, merange; x265amd_mes* mes; };
std::vector<Session> g_sessions;

x265amd_mes* session(const PicYuv& pic, const x265_param& p)
{
    const int ctu = (int)g_maxCUSize;
    const int rows = (int)((pic.m_picHeight + ctu - 1) / ctu);
    const int64_t elems = (int64_t)pic.m_stride * ((int64_t)rows * ctu + 2 * (int64_t)pic.m_lumaMarginY);
    const int64_t org = pic.m_picOrg[0] - pic.m_picBuf[0];
    x265amd_mes* mes = NULL;
    pthread_mutex_lock(&g_mu);
    for (size_t i = 0; i < g_sessions.size() && !mes; i++)
        if (g_sessions[i].stride == pic.m_stride && g_sessions[i].elems == elems && g_sessions[i].org == org &&
            g_sessions[i].rows == rows && g_sessions[i].method == p.searchMethod &&
            g_sessions[i].subme == p.subpelRefine && g_sessions[i].merange == p.searchRange)
            mes = g_sessions[i].mes;
    if (!mes && !g_status)
    {
        x265amd_mes_config c;
        memset(&c, 0, sizeof(c));
        c.depth = X265_DEPTH;
        c.stride = pic.m_stride;
        c.plane_elems = elems;
        c.org_offset = org;
        c.margin_y = (int)pic.m_lumaMarginY;
        c.ctu_rows = rows;
        c.ctu_size = ctu;
        c.max_pictures = 64;        /* reconstructed-picture buffers of the encoder's Frame pool used as references */
        c.max_threads = 256;        /* pool workers + frame encoder threads */
        c.max_tables = 82;          /* BitCost::BC_MAX_QP */
        c.mvcost_range = 2 << 15;   /* 2 * BitCost::BC_MAX_MV: the whole table */
        c.method = p.searchMethod;
        c.subme = p.subpelRefine;
        c.merange = p.searchRange;
        c.max_cand = (MD_ABOVE_LEFT + 1) * 2 + 2;
        g_status = x265amd_mes_create(&c, &mes);
        if (g_status)
        {
            fprintf(stderr, "[x265me] x265amd_mes_create failed: %s\n", x265amd_strerror(g_status));
            mes = NULL;
        }
        else
        {
            Session s = { pic.m_stride, elems, org, rows, p.searchMethod, p.subpelRefine, p.searchRange, mes };
            g_sessions.push_back(s);
        }
    }
    pthread_mutex_unlock(&g_mu);
    return mes;
}

/* the calling thread's prefetched searches of one PU */
enum { MAX_CAND = 16, MAX_JOBS = 2 * 2 * (MAX_NUM_REF + 1) };
struct Memo
{
    ReferencePlanes* ref;
    MV mvmin, mvmax, qmvp;
    int numc;
    MV mvc[MAX_CAND];
    int merange;
    MV out;
    int cost;
};
struct Prefetch
{
    const MotionEstimate* me;                /* the MotionEstimate the searches belong to (NULL: none ready) */
    const uint16_t* cost;                    /* its BitCost table when they were formed */
    int n, nskip;
    Memo m[MAX_JOBS];
    const ReferencePlanes* skip[MAX_JOBS];   /* references left to the host (weighted) */
    /* an asynchronous prefetch issued at the start of a CTU's analysis, collected by predInterSearch */
    x265amd_mes* mes;
    const Mode* mode;                        /* the Mode whose searches it holds */
    x265amd_mes_job jobs[MAX_JOBS];
    int pending;
    double t0;
};
/* per thread: the synchronous prefetch of the PU being searched, and the asynchronous one submitted
 * when the CTU's analysis started (collected by its 64x64 predInterSearch) */
__thread Prefetch* t_pf = NULL;
__thread Prefetch* t_apf = NULL;

Prefetch* prefetch_buf(Prefetch*& p)
{
    if (!p)
    {
        p = (Prefetch*)calloc(1, sizeof(Prefetch));
        if (!p) abort();
    }
    return p;
}

const Memo* lookup1(const Prefetch* pf, const MotionEstimate* me, const uint16_t* cost, const ReferencePlanes* ref,
                    const MV& mvmin, const MV& mvmax, const MV& qmvp, int numc, const MV* mvc, int merange)
{
    if (!pf || pf->me != me || pf->cost != cost) return NULL;
    for (int i = 0; i < pf->n; i++)
    {
        const Memo& e = pf->m[i];
        if (e.ref != ref || e.mvmin != mvmin || e.mvmax != mvmax || e.qmvp != qmvp || e.numc != numc ||
            e.merange != merange)
            continue;
        int k = 0;
        while (k < numc && e.mvc[k] == mvc[k]) k++;
        if (k == numc) return &e;
    }
    return NULL;
}

const Memo* lookup(const MotionEstimate* me, const uint16_t* cost, const ReferencePlanes* ref, const MV& mvmin,
                   const MV& mvmax, const MV& qmvp, int numc, const MV* mvc, int merange)
{
    const Memo* e = lookup1(t_pf, me, cost, ref, mvmin, mvmax, qmvp, numc, mvc, merange);
    return e ? e : lookup1(t_apf, me, cost, ref, mvmin, mvmax, qmvp, numc, mvc, merange);
}

/* was a prefetch active for this MotionEstimate, and did it leave `ref` to the host */
bool active_for(const MotionEstimate* me, const ReferencePlanes* ref, bool* skipped)
{
    bool act = false;
    *skipped = false;
    for (const Prefetch* pf : { (const Prefetch*)t_pf, (const Prefetch*)t_apf })
        if (pf && pf->me == me)
        {
            act = true;
            for (int i = 0; i < pf->nskip; i++)
                *skipped |= pf->skip[i] == ref;
        }
    return act;
}

} // namespace

namespace X265_NS {

int MotionEstimate::motionEstimate(ReferencePlanes* ref, const MV& mvmin, const MV& mvmax, const MV& qmvp,
                                   int numCandidates, const MV* mvc, int merange, MV& outQMv)
{
    const Memo* e = lookup(this, m_cost, ref, mvmin, mvmax, qmvp, numCandidates, mvc, merange);
    if (!e)
    {
        bool skipped;
        if (active_for(this, ref, &skipped))
            stat_add(skipped ? &Stats::skipped : &Stats::misses, 1);
        return x265ref_motionEstimate(this, ref, mvmin, mvmax, qmvp, numCandidates, mvc, merange, outQMv);
    }
    stat_add(&Stats::hits, 1);
    if (g_mode == ME_CHECK)
    {
        MV hmv;
        const int hc = x265ref_motionEstimate(this, ref, mvmin, mvmax, qmvp, numCandidates, mvc, merange, hmv);
        if (hc != e->cost || hmv != e->out)
        {
            pthread_mutex_lock(&g_mu);
            if (++g_st.mismatches <= 20)
                fprintf(stderr, "[x265me] CHECK MISMATCH %dx%d search: host (%d,%d)/%d device (%d,%d)/%d\n",
                        blockwidth, fencPUYuv.m_size, hmv.x, hmv.y, hc, e->out.x, e->out.y, e->cost);
            pthread_mutex_unlock(&g_mu);
        }
    }
    /* the reference call's side effects on this MotionEstimate (motion.cpp:581-587) */
    if (ctuAddr >= 0)
        blockOffset = ref->reconPic->getLumaAddr(ctuAddr, absPartIdx) - ref->reconPic->getLumaAddr(0);
    setMVP(qmvp);
    outQMv = e->out;
    return e->cost;
}

} // namespace X265_NS

namespace {

/* Form the searches the unidirectional loop of Search::predInterSearch (search.cpp:2181-2230) makes
 * for PU 0 of interMode — per (list, reference) allowed by refMasks: getPMV, the lowres MV and, for each
 * of the two AMVP predictors, setSearchRange — into pf->m[] (memo keys) and jobs[] (device
 * descriptors), after making the reference rows the encoder has finished resident on the device.
 * set_range forwards to the protected Search::setSearchRange.  Returns the number formed. */
template <class SetRange>
int form_searches(Search& S, Mode& interMode, const PredictionUnit& pu, const uint32_t refMasks[2], Prefetch* pf,
                  x265amd_mes_job* jobs, x265amd_mes** mes_out, SetRange set_range)
{
    CUData& cu = interMode.cu;
    const Slice* slice = S.m_slice;
    const x265_param* param = S.m_param;
    pf->me = NULL;
    pf->n = pf->nskip = 0;
    pf->cost = S.m_me.*CostPeek::member();
    cu.getNeighbourMV(0, pu.puAbsPartIdx, interMode.interNeighbours);
    const int numPredDir = slice->isInterP() ? 1 : 2;
    x265amd_mes* mes = NULL;
    int table = -1;
    uint32_t refMask = refMasks[0] ? refMasks[0] : (uint32_t)-1;
    for (int list = 0; list < numPredDir; list++, refMask >>= 16)
        for (int ref = 0; ref < slice->m_numRefIdx[list]; ref++)
        {
            if (!(refMask & (1 << ref)))
                continue;
            MotionReference& mr = slice->m_mref[list][ref];
            if (mr.isWeighted || !mr.reconPic || mr.fpelPlane[0] != mr.reconPic->m_picOrg[0])
            {
                pf->skip[pf->nskip++] = &mr;
                continue;
            }
            int slot = 0;
            if (g_mode != ME_HOST)
            {
                if (!mes && !(mes = session(*mr.reconPic, *param)))
                    continue;
                const Frame* rf = slice->m_refFrameList[list][ref];
                if (x265amd_mes_ref(mes, mr.reconPic, rf->m_poc, mr.reconPic->m_picBuf[0],
                                    const_cast<Frame*>(rf)->m_reconRowCount.get(), &slot))
                {
                    stat_add(&Stats::fallbacks, 1);
                    continue;
                }
                if (table < 0 && x265amd_mes_table(mes, pf->cost, &table))
                {
                    table = -1;
                    stat_add(&Stats::fallbacks, 1);
                    continue;
                }
            }
            MV mvc[MAX_CAND];
            int numMvc = cu.getPMV(interMode.interNeighbours, list, ref, interMode.amvpCand[list][ref], mvc);
            const MV* amvp = interMode.amvpCand[list][ref];
            MV lmv = S.getLowresMV(cu, pu, list, ref);
            if (lmv.notZero())
                mvc[numMvc++] = lmv;
            for (int c = 0; c < 2; c++)
            {
                if (c == 1 && amvp[1] == amvp[0])
                    continue;
                Memo& e = pf->m[pf->n];
                e.ref = &mr;
                set_range(cu, amvp[c], param->searchRange, e.mvmin, e.mvmax);
                e.qmvp = amvp[c];
                e.numc = numMvc;
                for (int k = 0; k < numMvc; k++) e.mvc[k] = mvc[k];
                e.merange = param->searchRange;
                x265amd_mes_job& j = jobs[pf->n];
                j.slot = slot;
                j.table = table;
                j.block_off = mr.reconPic->getLumaAddr(pu.ctuAddr, pu.cuAbsPartIdx + pu.puAbsPartIdx) -
                              mr.reconPic->getLumaAddr(0);
                j.mv_range[0] = e.mvmin.x;
                j.mv_range[1] = e.mvmin.y;
                j.mv_range[2] = e.mvmax.x;
                j.mv_range[3] = e.mvmax.y;
                j.mvp[0] = e.qmvp.x;
                j.mvp[1] = e.qmvp.y;
                j.num_cand = numMvc;
                for (int k = 0; k < numMvc; k++)
                {
                    j.mvc[2 * k] = mvc[k].x;
                    j.mvc[2 * k + 1] = mvc[k].y;
                }
                pf->n++;
            }
        }
    *mes_out = mes;
    return pf->n;
}

/* is a 2Nx2N PU of this CU searched on the device (large enough, the reference loop's plain path) */
bool eligible(const Search& S, const CUGeom& cuGeom)
{
    const Slice* slice = S.m_slice;
    return g_mode != ME_CPU && S.m_param->analysisMode != X265_ANALYSIS_LOAD && !S.m_param->bDistributeMotionEstimation &&
           slice->isInterP() + slice->isInterB() > 0 && (1 << (2 * cuGeom.log2CUSize)) >= g_min_area;
}

void finish_stats(Prefetch* pf)
{
    if (!g_stats_on) return;
    pthread_mutex_lock(&g_mu);
    g_st.prefetch++;
    g_st.searches += pf->n;
    g_st.sec += now_s() - pf->t0;
    pthread_mutex_unlock(&g_mu);
}

/* results of a submitted prefetch into its memo; false if the device call failed (the searches then run
 * on the host) */
bool collect(Prefetch* pf)
{
    if (!pf->mes)                              /* X265AMD_ME=host: computed when it was formed */
    {
        pf->pending = 0;
        return true;
    }
    const int st = x265amd_mes_collect(pf->mes, pf->n, pf->jobs);
    pf->pending = 0;
    if (st)
    {
        fprintf(stderr, "[x265me] x265amd_mes_collect failed: %s\n", x265amd_strerror(st));
        return false;
    }
    for (int i = 0; i < pf->n; i++)
    {
        pf->m[i].out = MV(pf->jobs[i].out_mv[0], pf->jobs[i].out_mv[1]);
        pf->m[i].cost = pf->jobs[i].out_cost;
    }
    return true;
}

} // namespace

namespace X265_NS {

void Search::predInterSearch(Mode& interMode, const CUGeom& cuGeom, bool bChromaMC, uint32_t refMasks[2])
{
    pthread_once(&g_once, read_mode);
    Prefetch* used = NULL;
    if (interMode.cu.getNumPartInter(0) == 1 && eligible(*this, cuGeom))
    {
        PredictionUnit pu(interMode.cu, cuGeom, 0);
        /* the same source block the reference loop sets up (search.cpp:2077) */
        m_me.setSourcePU(*interMode.fencYuv, pu.ctuAddr, pu.cuAbsPartIdx, pu.puAbsPartIdx, pu.width, pu.height);
        Prefetch* apf = t_apf;
        if (m_me.bChromaSATD)
            ;
        else if (apf && apf->pending && apf->mode == &interMode)
        {
            /* the searches submitted when this CTU's analysis started (compressInterCU_rd0_4 below) — every
             * reference; the reference loop takes those its refMasks allow */
            if (collect(apf))
            {
                apf->me = &m_me;
                finish_stats(apf);
                used = apf;
            }
        }
        else
        {
            Prefetch* pf = prefetch_buf(t_pf);
            pf->t0 = now_s();
            x265amd_mes* mes = NULL;
            x265amd_mes_job jobs[MAX_JOBS];
            const int n = form_searches(*this, interMode, pu, refMasks, pf, jobs, &mes,
                [this](const CUData& c, const MV& p, int r, MV& a, MV& b) { setSearchRange(c, p, r, a, b); });
            bool ok = n > 0;
            if (ok && g_mode == ME_HOST)
                for (int i = 0; i < n; i++)
                {
                    Memo& e = pf->m[i];
                    e.cost = x265ref_motionEstimate(&m_me, e.ref, e.mvmin, e.mvmax, e.qmvp, e.numc, e.mvc, e.merange,
                                                    e.out);
                }
            else if (ok)
            {
                const int st = x265amd_mes_search(mes, pu.width, pu.height, m_me.fencPUYuv.m_buf[0], FENC_STRIDE, n,
                                                  jobs);
                if (st)
                {
                    fprintf(stderr, "[x265me] x265amd_mes_search failed: %s\n", x265amd_strerror(st));
                    ok = false;
                }
                else
                    for (int i = 0; i < n; i++)
                    {
                        pf->m[i].out = MV(jobs[i].out_mv[0], jobs[i].out_mv[1]);
                        pf->m[i].cost = jobs[i].out_cost;
                    }
            }
            if (ok)
            {
                pf->me = &m_me;
                finish_stats(pf);
                used = pf;
            }
        }
    }
    x265ref_predInterSearch(this, interMode, cuGeom, bChromaMC, refMasks);
    if (used)
    {
        used->me = NULL;
        used->n = used->nskip = 0;
    }
}

/* Analysis::compressInterCU_rd0_4 (analysis.cpp:818-1100), --rd 0..4 (--preset medium: 3): the 64x64
 * CU's 2Nx2N motion searches come last in its analysis (after the merge candidates and the whole split
 * recursion, :945-953), but their inputs — the CU position, its neighbours' MVs (all in CTUs already
 * coded), the lowres MVs, the QP's BitCost table — are known when the analysis starts.  So at depth 0
 * the searches of EVERY reference are submitted to the device here (x265amd_mes_submit) and the host
 * runs the reference analysis meanwhile; predInterSearch collects them, the reference loop takes those
 * its refMasks allow.  The Mode's CU is initialised early exactly as :948 does it (nothing reads it
 * before); inputs the reference call differs in (a changed QP table) miss the memo and run on the host. */
SplitData Analysis::compressInterCU_rd0_4(const CUData& parentCTU, const CUGeom& cuGeom, int32_t qp)
{
    pthread_once(&g_once, read_mode);
    if (cuGeom.depth == 0 && g_async && eligible(*this, cuGeom) &&
        !(cuGeom.flags & CUGeom::SPLIT_MANDATORY))
    {
        Prefetch* pf = prefetch_buf(t_apf);
        if (pf->pending)
            (void)collect(pf);
        Mode& im = m_modeDepth[0].pred[PRED_2Nx2N];
        im.cu.initSubCU(parentCTU, cuGeom, qp);
        PredictionUnit pu(im.cu, cuGeom, 0);
        m_me.setSourcePU(*im.fencYuv, pu.ctuAddr, pu.cuAbsPartIdx, pu.puAbsPartIdx, pu.width, pu.height);
        if (!m_me.bChromaSATD)
        {
            pf->t0 = now_s();
            const uint32_t all[2] = { (uint32_t)-1, (uint32_t)-1 };
            x265amd_mes* mes = NULL;
            const int n = form_searches(*this, im, pu, all, pf, pf->jobs, &mes,
                [this](const CUData& c, const MV& p, int r, MV& a, MV& b) { setSearchRange(c, p, r, a, b); });
            pf->me = NULL;                     /* not usable before predInterSearch collects it */
            if (n > 0 && g_mode == ME_HOST)
            {
                /* the CPU check of the early forming: the searches run here on the host, and the reference
                 * loop must find every one it makes after the split recursion */
                for (int i = 0; i < n; i++)
                {
                    Memo& e = pf->m[i];
                    e.cost = x265ref_motionEstimate(&m_me, e.ref, e.mvmin, e.mvmax, e.qmvp, e.numc, e.mvc, e.merange,
                                                    e.out);
                }
                pf->mes = NULL;
                pf->mode = &im;
                pf->pending = n;
            }
            else if (n > 0)
            {
                const int st = x265amd_mes_submit(mes, pu.width, pu.height, m_me.fencPUYuv.m_buf[0], FENC_STRIDE, n,
                                                  pf->jobs);
                if (st)
                    fprintf(stderr, "[x265me] x265amd_mes_submit failed: %s\n", x265amd_strerror(st));
                else
                {
                    pf->mes = mes;
                    pf->mode = &im;
                    pf->pending = n;
                }
            }
        }
    }
    SplitData sd = x265ref_compressInterCU_rd0_4(this, parentCTU, cuGeom, qp);
    if (cuGeom.depth == 0 && t_apf)
    {
        if (t_apf->pending)
            (void)collect(t_apf);              /* the CU took a path without the 2Nx2N search */
        t_apf->me = NULL;
        t_apf->n = t_apf->nskip = 0;
    }
    return sd;
}

} // namespace X265_NS
