/* gpu_me.cpp — reference-side binding: the main encoder's motion searches of large PUs run on
 * the MI355X through the f2 session entries of include/x265_amd.h (x265amd_mes_*).
 *
 * This is the hook a maintainer adds to the encoder.  oracle/Makefile links
 * the reference encoder with copies of search.o, motion.o and analysis.o in which these symbols are
 * weak (objcopy -W) and the originals stay reachable under aliases:
 *
 *   Search::predInterSearch(Mode&, const CUGeom&, bool, uint32_t[2])      search.cpp:2050-2420
 *     -> the searches of the CU's 2Nx2N PU are taken from a prefetch (below), then the reference's own
 *        predInterSearch (x265ref_predInterSearch) runs unchanged.  Without an earlier prefetch the
 *        hook forms, for the PU of a 2Nx2N CU of at least X265AMD_ME_MIN pixels (default 64x64),
 *        every search the unidirectional loop (:2181-2230) is about to make — per (list, reference)
 *        allowed by refMasks: the AMVP candidates (getPMV), the lowres MV, and for EACH of the two AMVP
 *        predictors (selectMVP, :2199, picks one of them) its search range (setSearchRange) — and runs
 *        them on the device synchronously;
 *   Analysis::compressInterCU_rd0_4 (analysis.cpp:818), depth 0, and
 *   Analysis::checkMerge2Nx2N_rd0_4 (analysis.cpp:1652), called first in every CU's analysis (:853)
 *     -> the PREFETCH: the 2Nx2N searches of a CU come LAST in its analysis (:934, after the merge
 *        candidates and the whole split recursion), but their inputs — the CU position, the MVs of its
 *        neighbours (all in CUs already coded), the lowres MVs, the QP's BitCost table — are known when
 *        the CU's analysis starts.  So at that point the searches of EVERY reference are POSTED to the
 *        device (x265amd_mes_post: the call copies them into a request slot and returns), and the host
 *        analyses the sub-CUs meanwhile; predInterSearch WAITS for them (x265amd_mes_wait) when it
 *        needs them.  The session's launch service batches the posted searches of all worker threads
 *        into one launch (csrc/mesession.cpp), so a worker makes no HIP call on the search path;
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
 * --pme / --pmode, PUs of rectangular / AMP partitions, and PUs below the size threshold.
 *
 * Several devices (X265AMD_GPUS=G, round 5): the searches of frame encoder i (FrameData::
 * m_frameEncoderID: the encoder assigns frames round robin, encoder.cpp:649-650) go to device session
 * i mod G; each session holds its own copies of the reference rows its frames read, uploaded from the
 * host reconstruction as the rows are published.  X265AMD_GPU_LIST=a,b,... names the devices of the
 * sessions (default: session k on device k mod the visible devices).
 *
 *   X265AMD_ME=gpu     (default with the device lookahead) device searches
 *   X265AMD_ME=cpu     every call goes to the reference's functions (same binary)
 *   X265AMD_ME=host    the prefetch runs with the reference's motionEstimate on the host: checks the
 *                      hook's restated search setup and the memo on a CPU-only host
 *   X265AMD_ME=check   device searches, each compared with the host search when it is used
 *   X265AMD_ME_ASYNC=0 no prefetch at CU start: every search batch is synchronous in predInterSearch
 *   X265AMD_MES_LAUNCHERS=n  launch-service threads per session (default 2; 0 = the round-4 form, each
 *                      worker launching on its own stream)
 *   X265AMD_ME_STATS=1 prefetches, searches, memo hits / misses, the worker time spent forming, posting
 *                      and WAITING for device searches, and the sessions' launch counters, at exit
 *
 * Errors: a failing device call is recorded in the backend's sticky status (the encode then fails:
 * hip_encoder_main.cpp turns it into x265_encoder_encode() < 0); that PU is searched on the host so
 * the encoder's state stays valid until it stops.
 */
#include "common.h"
#include "primitives.h"
#include "frame.h"
#include "framedata.h"
#include "picyuv.h"
#include "slice.h"
#include "search.h"
#include "analysis.h"
#include "motion.h"
#include "reference.h"

#include <atomic>
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
extern "C" void x265ref_checkMerge2Nx2N_rd0_4(Analysis* self, Mode& skip, Mode& merge, const CUGeom& cuGeom);
/* gpu_rdo.cpp: the 2Nx2N prediction just made is final (X265AMD_RDO_EARLY) */
extern "C" void x265amd_rdo_early_inter(void* search, void* mode, const void* geom, int chroma_mc);

namespace {

/* BitCost::m_cost (the BitCost table of the current QP, bitcost.cpp:31-57) is protected; a
 * pointer to the member taken through a derived class reads it from a MotionEstimate */
struct CostPeek : public MotionEstimate
{
    static uint16_t* BitCost::*member() { return &CostPeek::m_cost; }
};

enum { ME_GPU = 0, ME_CPU = 1, ME_HOST = 2, ME_CHECK = 3 };
int g_mode = ME_GPU;
bool g_async = true;           /* prefetch at CU start (X265AMD_ME_ASYNC) */
int g_min_area = 64 * 64;      /* smallest 2Nx2N PU searched on the device (X265AMD_ME_MIN) */
int g_launchers = 2;           /* launch-service threads per session (X265AMD_MES_LAUNCHERS) */
int g_gpus = 1;                /* device sessions per geometry (X265AMD_GPUS) */
std::vector<int> g_gpu_list;   /* device of session k (X265AMD_GPU_LIST) */
bool g_stats_on = false;
pthread_once_t g_once = PTHREAD_ONCE_INIT;
pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
int g_status = 0;
/* bumped when an encoder closes: a prefetch of an earlier encoder is never collected */
std::atomic<int> g_epoch{ 0 };

struct Stats { std::atomic<long> prefetch, searches, hits, misses, skipped, fallbacks, mismatches, posted, dropped,
               window_violations; };
Stats g_st;
/* worker time (ns) spent on the device path, by phase: forming the searches, reference-row uploads,
 * posting, and waiting for results */
std::atomic<long long> g_ns_form{ 0 }, g_ns_ref{ 0 }, g_ns_post{ 0 }, g_ns_wait{ 0 };
std::atomic<long> g_waits{ 0 };
/* searches formed per device session (X265AMD_GPUS > 1; counted in host mode too) */
std::atomic<long> g_sub_searches[8];

long long now_ns()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

/* one session per reconstructed-picture geometry, search setting and device session index */
struct Session { intptr_t stride; int64_t elems; int64_t org; int rows, method, subme, merange, sub; x265amd_mes* mes; };
std::vector<Session> g_sessions;
x265amd_mes_counters g_closed;   /* counters of the sessions of closed encoders */
long g_sessions_created;         /* device sessions opened over the process (closed encoders' included) */

void add_counters(x265amd_mes_counters& tot, const x265amd_mes_counters& c)
{
    tot.batches += c.batches;
    tot.requests += c.requests;
    tot.jobs += c.jobs;
    tot.kernel_ms += c.kernel_ms;
    tot.batch_ms += c.batch_ms;
    tot.queue_ms += c.queue_ms;
    tot.uploads += c.uploads;
    tot.upload_bytes += c.upload_bytes;
    tot.upload_ms += c.upload_ms;
    tot.waits += c.waits;
    tot.waits_blocked += c.waits_blocked;
    tot.dropped += c.dropped;
    tot.wait_ms += c.wait_ms;
    tot.evals_fpel += c.evals_fpel;
    tot.evals_subpel += c.evals_subpel;
    tot.algo_bytes += c.algo_bytes;
    if (c.kernel_ms_max > tot.kernel_ms_max) tot.kernel_ms_max = c.kernel_ms_max;
    if (c.max_requests_per_batch > tot.max_requests_per_batch) tot.max_requests_per_batch = c.max_requests_per_batch;
    for (int b = 0; b < 5; b++)
    {
        tot.wait_hist[b] += c.wait_hist[b];
        tot.wait_hist_ms[b] += c.wait_hist_ms[b];
        tot.batch_hist[b] += c.batch_hist[b];
        tot.batch_hist_ms[b] += c.batch_hist_ms[b];
    }
}

void print_stats()
{
    fprintf(stderr, "[x265me] stats prefetches %ld searches %ld memo hits %ld misses %ld host fallbacks %ld "
                    "weighted-reference searches %ld posted %ld dropped %ld\n", (long)g_st.prefetch, (long)g_st.searches,
            (long)g_st.hits, (long)g_st.misses, (long)g_st.fallbacks, (long)g_st.skipped, (long)g_st.posted,
            (long)g_st.dropped);
    fprintf(stderr, "[x265me] worker time on the device path: forming %.3f s, reference uploads %.3f s, posting "
                    "%.3f s, waiting for the device %.3f s (%ld waits)\n", 1e-9 * g_ns_form, 1e-9 * g_ns_ref,
            1e-9 * g_ns_post, 1e-9 * g_ns_wait, (long)g_waits);
    x265amd_mes_counters tot = g_closed;
    for (const Session& s : g_sessions)
    {
        x265amd_mes_counters c;
        if (!x265amd_mes_stats(s.mes, &c)) add_counters(tot, c);
    }
    if (tot.batches)
        fprintf(stderr, "[x265me] service: %lld launches, %lld requests (%.2f per launch, max %lld), %lld searches, "
                        "kernel %.3f ms per launch (HIP events), batch %.3f ms, queueing %.3f ms per request, "
                        "%lld waits slept; %lld row uploads %.1f MB %.1f ms; sessions %ld; evaluations %lld full-pel "
                        "%lld sub-pel, %.3f GB algorithmic, longest launch %.3f ms\n",
                (long long)tot.batches, (long long)tot.requests, (double)tot.requests / tot.batches,
                (long long)tot.max_requests_per_batch, (long long)tot.jobs, tot.kernel_ms / tot.batches,
                tot.batch_ms / tot.batches, tot.requests ? tot.queue_ms / tot.requests : 0.0,
                (long long)tot.waits_blocked, (long long)tot.uploads, tot.upload_bytes / 1e6, tot.upload_ms,
                g_sessions_created, (long long)tot.evals_fpel, (long long)tot.evals_subpel, tot.algo_bytes / 1e9,
                tot.kernel_ms_max);
    if (tot.batches)
    {
        static const char* bins[5] = { "<0.05", "<0.2", "<1", "<5", ">=5" };
        fprintf(stderr, "[x265me] waits by duration (ms: count / summed ms):");
        for (int b = 0; b < 5; b++)
            fprintf(stderr, " %s %lld / %.0f", bins[b], (long long)tot.wait_hist[b], tot.wait_hist_ms[b]);
        fprintf(stderr, "\n[x265me] batches by duration (ms: count / summed ms):");
        for (int b = 0; b < 5; b++)
            fprintf(stderr, " %s %lld / %.0f", bins[b], (long long)tot.batch_hist[b], tot.batch_hist_ms[b]);
        fprintf(stderr, "\n");
    }
    if (g_gpus > 1)
    {
        fprintf(stderr, "[x265me] searches per device session:");
        for (int k = 0; k < g_gpus && k < 8; k++)
            fprintf(stderr, " %ld", (long)g_sub_searches[k]);
        fprintf(stderr, "\n");
    }
    if (g_mode == ME_CHECK)
    {
        fprintf(stderr, "[x265me] check: %ld mismatching searches\n", (long)g_st.mismatches);
        fprintf(stderr, "[x265me] check: %ld search windows beyond the resident reference rows\n",
                (long)g_st.window_violations);
    }
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
    if (const char* a = getenv("X265AMD_MES_LAUNCHERS"))
        g_launchers = atoi(a);
    /* the CU-start prefetch needs the launch service (the round-4 per-thread form measured neutral) */
    g_async = g_launchers > 0;
    if (const char* a = getenv("X265AMD_ME_ASYNC"))
        g_async = atoi(a) != 0;
    if (const char* a = getenv("X265AMD_GPUS"))
        g_gpus = atoi(a) > 0 ? (atoi(a) < 8 ? atoi(a) : 8) : 1;
    if (const char* a = getenv("X265AMD_GPU_LIST"))
        for (const char* p = a; *p;)
        {
            g_gpu_list.push_back(atoi(p));
            while (*p && *p != ',') p++;
            if (*p) p++;
        }
    const char* st = getenv("X265AMD_ME_STATS");
    g_stats_on = (st && *st && strcmp(st, "0")) || g_mode == ME_CHECK;
    fprintf(stderr, "[x265me] motion searches of PUs >= %d pixels on %s%s\n", g_min_area,
            g_mode == ME_CPU ? "the CPU (reference functions)" : g_mode == ME_HOST ? "the CPU (hook prefetch)" :
            g_mode == ME_CHECK ? "the MI355X, each checked against the CPU" : "the MI355X",
            g_mode == ME_CPU ? "" : g_async ? ", prefetched at CU start" : ", synchronous");
    if (g_stats_on)
        atexit(print_stats);
}

void stat_add(std::atomic<long> Stats::*field, long v)
{
    if (g_stats_on) (g_st.*field).fetch_add(v, std::memory_order_relaxed);
}

x265amd_mes* session(const PicYuv& pic, const x265_param& p, int sub)
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
            g_sessions[i].subme == p.subpelRefine && g_sessions[i].merange == p.searchRange && g_sessions[i].sub == sub)
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
        c.launchers = g_launchers;
        /* subme > 2: the 4:2:0 chroma planes too, for the sub-pel chroma SATD (launch service only) */
        if (p.subpelRefine > 2 && pic.m_picCsp == X265_CSP_I420 && g_launchers > 0)
        {
            c.chroma = 1;
            c.cstride = pic.m_strideC;
            c.cplane_elems = (int64_t)pic.m_strideC * ((int64_t)rows * ctu / 2 + 2 * (int64_t)pic.m_chromaMarginY);
            c.corg_offset = pic.m_picOrg[1] - pic.m_picBuf[1];
            c.cmargin_y = (int)pic.m_chromaMarginY;
        }
        int ndev = 1;
        if (x265amd_device_count(&ndev) || ndev < 1) ndev = 1;
        c.device = !g_gpu_list.empty() ? g_gpu_list[sub % g_gpu_list.size()] : sub % ndev;
        g_status = x265amd_mes_create(&c, &mes);
        if (g_status)
        {
            fprintf(stderr, "[x265me] x265amd_mes_create failed: %s\n", x265amd_strerror(g_status));
            mes = NULL;
        }
        else
        {
            Session s = { pic.m_stride, elems, org, rows, p.searchMethod, p.subpelRefine, p.searchRange, sub, mes };
            g_sessions.push_back(s);
            g_sessions_created++;
        }
    }
    pthread_mutex_unlock(&g_mu);
    return mes;
}

/* the prefetched searches of one PU */
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
    /* a prefetch posted at the start of a CU's analysis, collected by its predInterSearch */
    x265amd_mes* mes;
    const Mode* mode;                        /* the Mode whose searches it holds */
    x265amd_mes_job jobs[MAX_JOBS];
    int pending;                             /* searches posted and not yet collected */
    int ticket;
    int epoch;
};
/* per thread: the synchronous prefetch of the PU being searched, and the prefetches posted when the
 * CU at depth 0 / 1 started */
__thread Prefetch* t_pf = NULL;
__thread Prefetch* t_apf[2] = { NULL, NULL };

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
    for (int d = 0; d < 2 && !e; d++)
        e = lookup1(t_apf[d], me, cost, ref, mvmin, mvmax, qmvp, numc, mvc, merange);
    return e;
}

/* was a prefetch active for this MotionEstimate, and did it leave `ref` to the host */
bool active_for(const MotionEstimate* me, const ReferencePlanes* ref, bool* skipped)
{
    bool act = false;
    *skipped = false;
    for (const Prefetch* pf : { (const Prefetch*)t_pf, (const Prefetch*)t_apf[0], (const Prefetch*)t_apf[1] })
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
    const long long t0 = now_ns();
    long long t_ref = 0;
    CUData& cu = interMode.cu;
    const Slice* slice = S.m_slice;
    const x265_param* param = S.m_param;
    pf->me = NULL;
    pf->n = pf->nskip = 0;
    pf->cost = S.m_me.*CostPeek::member();
    cu.getNeighbourMV(0, pu.puAbsPartIdx, interMode.interNeighbours);
    const int numPredDir = slice->isInterP() ? 1 : 2;
    /* the device session of this frame's encoder (frame encoders take frames round robin) */
    const int sub = g_gpus > 1 ? cu.m_encData->m_frameEncoderID % g_gpus : 0;
    const int64_t epoch = (int64_t)g_epoch.load() << 32;
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
                if (!mes && !(mes = session(*mr.reconPic, *param, sub)))
                    continue;
                const Frame* rf = slice->m_refFrameList[list][ref];
                const long long r0 = now_ns();
                /* generation = (encoder epoch, POC): a later encoder's picture at a reused PicYuv address is
                 * never taken for an earlier one's */
                const void* planes[3] = { mr.reconPic->m_picBuf[0], mr.reconPic->m_picBuf[1], mr.reconPic->m_picBuf[2] };
                const int rc = x265amd_mes_ref420(mes, mr.reconPic, epoch | (uint32_t)rf->m_poc, planes,
                                                  const_cast<Frame*>(rf)->m_reconRowCount.get(), &slot);
                t_ref += now_ns() - r0;
                if (rc)
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
                if (g_mode == ME_CHECK && mes)
                {
                    /* the rows this search can read (its full-pel range, the PU, the 8-tap filter reach and the
                     * sub-pel refine's pixel beyond the range) must be resident on the device: a search never
                     * reads a row a later upload would still change.  STAR costs points level with an
                     * out-of-range origin (MV 0), so its lowest row is at least the PU's own */
                    const int ctu = (int)g_maxCUSize;
                    const int last_y = (int)pu.ctuAddr / (int)S.m_frame->m_encData->m_slice->m_sps->numCuInWidth * ctu +
                                       (int)g_zscanToPelY[pu.cuAbsPartIdx + pu.puAbsPartIdx] +
                                       (e.mvmax.y > 0 ? e.mvmax.y : 0) + pu.height + 4 + 1;
                    const int rows_needed = last_y < 0 ? 0 : (last_y + ctu - 1) / ctu;
                    const int nrows = (int)((mr.reconPic->m_picHeight + ctu - 1) / ctu);
                    int resident = 0;
                    const Frame* rf = slice->m_refFrameList[list][ref];
                    if (!x265amd_mes_rows(mes, mr.reconPic, epoch | (uint32_t)rf->m_poc, &resident) &&
                        (rows_needed > nrows ? nrows : rows_needed) > resident)
                    {
                        if (++g_st.window_violations <= 10)
                            fprintf(stderr, "[x265me] CHECK window of a %dx%d search at CTU %u needs %d reference rows, "
                                            "%d resident\n", pu.width, pu.height, pu.ctuAddr, rows_needed, resident);
                    }
                }
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
    if (g_gpus > 1 && sub < 8)
        g_sub_searches[sub] += pf->n;
    g_ns_ref += t_ref;
    g_ns_form += now_ns() - t0 - t_ref;
    return pf->n;
}

/* bChromaSATD of a w x h PU exactly as MotionEstimate::setSourcePU sets it (motion.cpp:193-197) */
bool chroma_satd(const Search& S, int csp, int w, int h)
{
    return S.m_param->subpelRefine > 2 && csp != X265_CSP_I400 && primitives.chroma[csp].pu[partitionFromSizes(w, h)].satd;
}

/* can the device run this PU's searches: luma-only searches always, chroma-SATD searches (subme > 2) on
 * 4:2:0 pictures with the launch service (the session then holds the chroma planes) */
bool device_can(int csp, bool chroma)
{
    return !chroma || (csp == X265_CSP_I420 && g_launchers > 0);
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
    stat_add(&Stats::prefetch, 1);
    stat_add(&Stats::searches, pf->n);
}

/* results of a posted prefetch into its memo; false if the device call failed (the searches then run
 * on the host) */
bool collect(Prefetch* pf)
{
    if (!pf->mes)                              /* X265AMD_ME=host: computed when it was formed */
    {
        pf->pending = 0;
        return true;
    }
    const long long t0 = now_ns();
    const int st = x265amd_mes_wait(pf->mes, pf->ticket, pf->n, pf->jobs);
    g_ns_wait += now_ns() - t0;
    g_waits++;
    pf->pending = 0;
    if (st)
    {
        fprintf(stderr, "[x265me] x265amd_mes_wait failed: %s\n", x265amd_strerror(st));
        return false;
    }
    for (int i = 0; i < pf->n; i++)
    {
        pf->m[i].out = MV(pf->jobs[i].out_mv[0], pf->jobs[i].out_mv[1]);
        pf->m[i].cost = pf->jobs[i].out_cost;
    }
    return true;
}

/* give up a posted prefetch the analysis did not use (its CU took a path without the 2Nx2N search) */
void release(Prefetch* pf)
{
    if (pf->pending && pf->mes && pf->epoch == g_epoch.load())
    {
        (void)x265amd_mes_drop(pf->mes, pf->ticket);
        stat_add(&Stats::dropped, 1);
    }
    pf->pending = 0;
    pf->me = NULL;
    pf->mode = NULL;
    pf->n = pf->nskip = 0;
}

/* post the 2Nx2N searches of the CU whose analysis starts now (depth 0 / 1), for every reference; the
 * Mode's CU is initialised early exactly as the analysis does it before its search (analysis.cpp:933 —
 * nothing reads that Mode before) */
template <class SetRange>
void prefetch_cu(Analysis& A, const CUData& parentCTU, const CUGeom& cuGeom, int32_t qp, SetRange set_range)
{
    const int d = (int)cuGeom.depth;
    Prefetch* pf = prefetch_buf(t_apf[d]);
    release(pf);
    Mode& im = A.m_modeDepth[d].pred[Analysis::PRED_2Nx2N];
    {
        const int size = 1 << cuGeom.log2CUSize;
        if (!device_can(im.fencYuv->m_csp, chroma_satd(A, im.fencYuv->m_csp, size, size)))
            return;
    }
    im.cu.initSubCU(parentCTU, cuGeom, qp);
    PredictionUnit pu(im.cu, cuGeom, 0);
    const uint32_t all[2] = { (uint32_t)-1, (uint32_t)-1 };
    x265amd_mes* mes = NULL;
    const int n = form_searches(A, im, pu, all, pf, pf->jobs, &mes, set_range);
    pf->me = NULL;                             /* not usable before predInterSearch collects it */
    if (n <= 0)
        return;
    /* the 2Nx2N PU's source block: the CU's own fenc buffer (stride = CU size), what setSourcePU copies */
    const Yuv& fenc = *im.fencYuv;
    const bool chroma = chroma_satd(A, fenc.m_csp, pu.width, pu.height);
    if (g_mode == ME_HOST)
    {
        /* the CPU check of the early forming: the searches run here on the host, and the reference loop
         * must find every one it makes after the split recursion */
        A.m_me.setSourcePU(fenc, pu.ctuAddr, pu.cuAbsPartIdx, pu.puAbsPartIdx, pu.width, pu.height);
        for (int i = 0; i < n; i++)
        {
            Memo& e = pf->m[i];
            e.cost = x265ref_motionEstimate(&A.m_me, e.ref, e.mvmin, e.mvmax, e.qmvp, e.numc, e.mvc, e.merange, e.out);
        }
        pf->mes = NULL;
        pf->mode = &im;
        pf->pending = n;
        pf->epoch = g_epoch.load();
        return;
    }
    const long long t0 = now_ns();
    int ticket = -1;
    const int st = x265amd_mes_post420(mes, pu.width, pu.height, fenc.m_buf[0], fenc.m_size, chroma ? fenc.m_buf[1] : NULL,
                                       chroma ? fenc.m_buf[2] : NULL, fenc.m_csize, n, pf->jobs, &ticket);
    g_ns_post += now_ns() - t0;
    if (st)
    {
        if (st != X265AMD_ENOMEM)
            fprintf(stderr, "[x265me] x265amd_mes_post failed: %s\n", x265amd_strerror(st));
        pf->n = 0;
        return;
    }
    stat_add(&Stats::posted, 1);
    pf->mes = mes;
    pf->mode = &im;
    pf->pending = n;
    pf->ticket = ticket;
    pf->epoch = g_epoch.load();
}

bool can_prefetch(const Analysis& A, const CUGeom& cuGeom)
{
    return g_async && cuGeom.depth < 2 && eligible(A, cuGeom) && !A.m_param->bDistributeModeAnalysis &&
           !(cuGeom.flags & CUGeom::SPLIT_MANDATORY);
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
        Prefetch* apf = cuGeom.depth < 2 ? t_apf[cuGeom.depth] : NULL;
        if (!device_can(interMode.fencYuv->m_csp, m_me.bChromaSATD))
            ;
        else if (apf && apf->pending && apf->mode == &interMode && apf->epoch == g_epoch.load())
        {
            /* the searches posted when this CU's analysis started — every reference; the reference loop
             * takes those its refMasks allow */
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
                const long long t0 = now_ns();
                int st;
                if (m_me.bChromaSATD)
                {
                    /* the PU's chroma as setSourcePU copied it (fencPUYuv: stride FENC_STRIDE / 2) */
                    int ticket = -1;
                    st = x265amd_mes_post420(mes, pu.width, pu.height, m_me.fencPUYuv.m_buf[0], FENC_STRIDE,
                                             m_me.fencPUYuv.m_buf[1], m_me.fencPUYuv.m_buf[2], m_me.fencPUYuv.m_csize, n,
                                             jobs, &ticket);
                    if (!st) st = x265amd_mes_wait(mes, ticket, n, jobs);
                }
                else
                    st = x265amd_mes_search(mes, pu.width, pu.height, m_me.fencPUYuv.m_buf[0], FENC_STRIDE, n, jobs);
                g_ns_wait += now_ns() - t0;
                g_waits++;
                if (st)
                {
                    if (st != X265AMD_ENOMEM)
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
    x265amd_rdo_early_inter(this, &interMode, &cuGeom, bChromaMC ? 1 : 0);
    if (used)
    {
        used->me = NULL;
        used->mode = NULL;
        used->n = used->nskip = 0;
    }
}

/* Analysis::compressInterCU_rd0_4 (analysis.cpp:818-1298), --rd 0..4 (--preset medium: 3), reached here
 * for the CTU (depth 0; the analysis recurses through its local alias): the 64x64 CU's searches are
 * posted before its analysis runs; whatever prefetch the CTU's analysis left uncollected is given up
 * when it returns. */
SplitData Analysis::compressInterCU_rd0_4(const CUData& parentCTU, const CUGeom& cuGeom, int32_t qp)
{
    pthread_once(&g_once, read_mode);
    if (cuGeom.depth == 0 && can_prefetch(*this, cuGeom))
        prefetch_cu(*this, parentCTU, cuGeom, qp,
                    [this](const CUData& c, const MV& p, int r, MV& a, MV& b) { setSearchRange(c, p, r, a, b); });
    SplitData sd = x265ref_compressInterCU_rd0_4(this, parentCTU, cuGeom, qp);
    if (cuGeom.depth == 0)
        for (int d = 0; d < 2; d++)
            if (t_apf[d])
                release(t_apf[d]);
    return sd;
}

/* Analysis::checkMerge2Nx2N_rd0_4 (analysis.cpp:1652), the first step of every CU's analysis
 * (analysis.cpp:848-853): for a 32x32 CU (depth 1) whose 2Nx2N PU is searched on the device, post its
 * searches before the merge candidates and the sub-CUs are analysed.  The CU's merge Mode was just
 * initialised from the CTU with the CU's QP (:851), which gives the CTU and the QP. */
void Analysis::checkMerge2Nx2N_rd0_4(Mode& skip, Mode& merge, const CUGeom& cuGeom)
{
    pthread_once(&g_once, read_mode);
    if (cuGeom.depth == 1 && can_prefetch(*this, cuGeom) && &merge == &m_modeDepth[1].pred[Analysis::PRED_MERGE])
    {
        const CUData& ctu = *merge.cu.m_encData->getPicCTU(merge.cu.m_cuAddr);
        prefetch_cu(*this, ctu, cuGeom, merge.cu.m_qp[0],
                    [this](const CUData& c, const MV& p, int r, MV& a, MV& b) { setSearchRange(c, p, r, a, b); });
    }
    x265ref_checkMerge2Nx2N_rd0_4(this, skip, merge, cuGeom);
}

} // namespace X265_NS

/* called by the encoder binding before x265_encoder_close frees the encoder's frames (and again after it;
 * oracle/hip_encoder_main.cpp): the sessions of the closing encoder are destroyed (uploads drained, pinned
 * reconstruction planes unregistered while still allocated, device arenas freed) and
 * the epoch advances, so a later encoder in the same process starts from empty sessions */
extern "C" void x265amd_me_encoder_closed(void)
{
    pthread_mutex_lock(&g_mu);
    g_epoch++;
    for (Session& s : g_sessions)
    {
        x265amd_mes_counters c;
        if (!x265amd_mes_stats(s.mes, &c)) add_counters(g_closed, c);
        x265amd_mes_destroy(s.mes);
    }
    g_sessions.clear();
    pthread_mutex_unlock(&g_mu);
}
