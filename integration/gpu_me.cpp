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
 *        (default 32x32), every search the unidirectional loop (:2181-2230) is about to make —
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

namespace {

/* BitCost::m_cost (the BitCost table of the current QP, bitcost.cpp:31-57) is protected; a
 * pointer to the member taken through a derived class reads it from a MotionEstimate */
struct CostPeek : public MotionEstimate
{
    static uint16_t* BitCost::*member() { return &CostPeek::m_cost; }
};

enum { ME_GPU = 0, ME_CPU = 1, ME_HOST = 2, ME_CHECK = 3 };
int g_mode = ME_GPU;
int g_min_area = 32 * 32;
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
    const MotionEstimate* me;
    int n, nskip;
    Memo m[MAX_JOBS];
    const ReferencePlanes* skip[MAX_JOBS];   /* references left to the host (weighted) */
};
__thread Prefetch* t_pf = NULL;

Prefetch* prefetch_buf()
{
    if (!t_pf)
    {
        t_pf = (Prefetch*)calloc(1, sizeof(Prefetch));
        if (!t_pf) abort();
    }
    return t_pf;
}

const Memo* lookup(const MotionEstimate* me, const ReferencePlanes* ref, const MV& mvmin, const MV& mvmax,
                   const MV& qmvp, int numc, const MV* mvc, int merange)
{
    const Prefetch* pf = t_pf;
    if (!pf || pf->me != me) return NULL;
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

} // namespace

namespace X265_NS {

int MotionEstimate::motionEstimate(ReferencePlanes* ref, const MV& mvmin, const MV& mvmax, const MV& qmvp,
                                   int numCandidates, const MV* mvc, int merange, MV& outQMv)
{
    const Memo* e = lookup(this, ref, mvmin, mvmax, qmvp, numCandidates, mvc, merange);
    if (!e)
    {
        if (t_pf && t_pf->me == this)
        {
            bool skipped = false;
            for (int i = 0; i < t_pf->nskip; i++)
                skipped |= t_pf->skip[i] == ref;
            stat_add(skipped ? &Stats::skipped : &Stats::misses, 1);
        }
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

void Search::predInterSearch(Mode& interMode, const CUGeom& cuGeom, bool bChromaMC, uint32_t refMasks[2])
{
    pthread_once(&g_once, read_mode);
    CUData& cu = interMode.cu;
    const Slice* slice = m_slice;
    Prefetch* pf = NULL;
    if (g_mode != ME_CPU && cu.getNumPartInter(0) == 1 && m_param->analysisMode != X265_ANALYSIS_LOAD &&
        !m_param->bDistributeMotionEstimation && slice->isInterP() + slice->isInterB() > 0)
    {
        PredictionUnit pu(cu, cuGeom, 0);
        if (pu.width * pu.height >= g_min_area)
        {
            /* the same source block the reference loop sets up (search.cpp:2077) */
            m_me.setSourcePU(*interMode.fencYuv, pu.ctuAddr, pu.cuAbsPartIdx, pu.puAbsPartIdx, pu.width, pu.height);
            if (!m_me.bChromaSATD)
                pf = prefetch_buf();
        }
        if (pf)
        {
            const double t0 = now_s();
            pf->me = NULL;
            pf->n = pf->nskip = 0;
            cu.getNeighbourMV(0, pu.puAbsPartIdx, interMode.interNeighbours);
            const int numPredDir = slice->isInterP() ? 1 : 2;
            x265amd_mes* mes = NULL;
            x265amd_mes_job jobs[MAX_JOBS];
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
                        if (!mes && !(mes = session(*mr.reconPic, *m_param)))
                            continue;
                        const Frame* rf = slice->m_refFrameList[list][ref];
                        const int st = x265amd_mes_ref(mes, mr.reconPic, rf->m_poc, mr.reconPic->m_picBuf[0],
                                                       const_cast<Frame*>(rf)->m_reconRowCount.get(), &slot);
                        if (st)
                        {
                            stat_add(&Stats::fallbacks, 1);
                            continue;
                        }
                        if (table < 0 && x265amd_mes_table(mes, m_me.*CostPeek::member(), &table))
                        {
                            table = -1;
                            stat_add(&Stats::fallbacks, 1);
                            break;
                        }
                    }
                    /* the search inputs of search.cpp:2196-2206, for both AMVP predictors */
                    MV mvc[MAX_CAND];
                    int numMvc = cu.getPMV(interMode.interNeighbours, list, ref, interMode.amvpCand[list][ref], mvc);
                    const MV* amvp = interMode.amvpCand[list][ref];
                    MV lmv = getLowresMV(cu, pu, list, ref);
                    if (lmv.notZero())
                        mvc[numMvc++] = lmv;
                    for (int c = 0; c < 2; c++)
                    {
                        if (c == 1 && amvp[1] == amvp[0])
                            continue;
                        Memo& e = pf->m[pf->n];
                        e.ref = &mr;
                        setSearchRange(cu, amvp[c], m_param->searchRange, e.mvmin, e.mvmax);
                        e.qmvp = amvp[c];
                        e.numc = numMvc;
                        for (int k = 0; k < numMvc; k++) e.mvc[k] = mvc[k];
                        e.merange = m_param->searchRange;
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
            bool ok = pf->n > 0;
            if (ok && g_mode == ME_HOST)
            {
                for (int i = 0; i < pf->n; i++)
                {
                    Memo& e = pf->m[i];
                    e.cost = x265ref_motionEstimate(&m_me, e.ref, e.mvmin, e.mvmax, e.qmvp, e.numc, e.mvc, e.merange,
                                                    e.out);
                }
            }
            else if (ok)
            {
                const int st = x265amd_mes_search(mes, pu.width, pu.height, m_me.fencPUYuv.m_buf[0], FENC_STRIDE, pf->n,
                                                  jobs);
                if (st)
                {
                    fprintf(stderr, "[x265me] x265amd_mes_search failed: %s\n", x265amd_strerror(st));
                    ok = false;
                }
                else
                    for (int i = 0; i < pf->n; i++)
                    {
                        pf->m[i].out = MV(jobs[i].out_mv[0], jobs[i].out_mv[1]);
                        pf->m[i].cost = jobs[i].out_cost;
                    }
            }
            if (ok)
            {
                pf->me = &m_me;
                if (g_stats_on)
                {
                    pthread_mutex_lock(&g_mu);
                    g_st.prefetch++;
                    g_st.searches += pf->n;
                    g_st.sec += now_s() - t0;
                    pthread_mutex_unlock(&g_mu);
                }
            }
        }
    }
    x265ref_predInterSearch(this, interMode, cuGeom, bChromaMC, refMasks);
    if (pf)
    {
        pf->me = NULL;
        pf->n = pf->nskip = 0;
    }
}

} // namespace X265_NS
