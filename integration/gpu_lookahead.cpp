/* gpu_lookahead.cpp — reference-side binding: x265 1.9's lookahead cost estimates run on
 * the MI355X through the f1 session entries of include/x265_amd.h (x265amd_la_*).
 *
 * This is the hook a maintainer adds to the encoder.  It replaces two
 * functions of encoder/slicetype.cpp; oracle/Makefile links the reference encoder with a
 * copy of slicetype.o in which exactly those two symbols are weak (objcopy -W) and the
 * original code stays reachable under an alias (objcopy --add-symbol), so every call site —
 * PreLookaheadGroup::processTasks, CostEstimateGroup::singleCost / processTasks, all through
 * the PLT (the Makefile checks the relocations) — lands here:
 *
 *   LookaheadTLD::lowresIntraEstimate(Lowres&)                          slicetype.cpp:230-336
 *     -> x265amd_la_load (the picture's 4 lowres planes + invQscaleFactor, once) and
 *        x265amd_la_intra, outputs written into the Lowres;
 *   CostEstimateGroup::estimateFrameCost(tld, p0, p1, b, bIntraPenalty) slicetype.cpp:1977-2066
 *     -> the reference's control flow unchanged (cost cache test, bDoSearch from the
 *        lowresMvs sentinel, weightsAnalyse on the host, the coop-slice geometry of
 *        m_numRowsPerSlice / m_numCoopSlices in non-batch mode, the B-frame bias and the
 *        intra penalty); the per-CU work (estimateCUCost over the frame, :2068-2225) is ONE
 *        device call, x265amd_la_pcost (b == p1) or x265amd_la_bcost.
 *
 * Two cases the device estimate does not cover run the reference's own estimateCUCost on
 * the calling thread, in the reference's CU and slice order: a P estimate whose list-0 MVs
 * already exist (bDoSearch[0] false) and a B estimate whose list-0 reference was weighted
 * (the device B estimate reads p0 unweighted).  Results are bit-identical either way, so the
 * bitstream equals the reference encoder's (tests/test_encoder_lookahead.py).
 *
 *   X265AMD_LOOKAHEAD=cpu    every call goes to the reference's original functions (same binary)
 *   X265AMD_LOOKAHEAD=host   this hook's control flow with the CPU per-CU loops only (no device):
 *                            checks the restated control flow against the reference on a CPU host
 *
 * Errors: a failing device call is recorded in the backend's sticky status; the returned
 * estimate is then meaningless and the encoder binding (hip_encoder_main.cpp) turns the status
 * into x265_encoder_encode() < 0.
 */
#include "common.h"
#include "primitives.h"
#include "lowres.h"
#include "slicetype.h"
#include "ratecontrol.h"    /* CLIP_DURATION */

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <pthread.h>
#include <vector>

#include "../include/x265_amd.h"

using namespace X265_NS;

/* the reference's own implementations (aliases of the weakened symbols, see oracle/Makefile) */
extern "C" void x265ref_finishBatch(CostEstimateGroup* self);
extern "C" void x265ref_lowresIntraEstimate(LookaheadTLD* self, Lowres* fenc);
extern "C" int64_t x265ref_estimateFrameCost(CostEstimateGroup* self, LookaheadTLD* tld, int p0, int p1, int b,
                                             bool bIntraPenalty);
extern "C" void x265ref_estimateCUPropagate(Lookahead* self, Lowres** frames, double averageDuration, int p0, int p1,
                                            int b, int referenced);

namespace {

struct TabBitCost : public BitCost
{
    const uint16_t* table(unsigned qp) { setQP(qp); return m_cost; }
};

enum { MODE_GPU = 0, MODE_CPU = 1, MODE_HOST = 2, MODE_CHECK = 3 };

int g_mode = MODE_GPU;
bool g_propagate = false;      /* X265AMD_LA_PROPAGATE=1: cuTree's propagation steps on the device */
int g_la_status = 0;
pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
pthread_once_t g_mode_once = PTHREAD_ONCE_INIT;

void print_check_summary();
void print_stats();
extern bool g_stats_on;

void read_mode()
{
    const char* m = getenv("X265AMD_LOOKAHEAD");
    g_mode = (m && !strcmp(m, "cpu")) ? MODE_CPU : (m && !strcmp(m, "host")) ? MODE_HOST :
             (m && !strcmp(m, "check")) ? MODE_CHECK : MODE_GPU;
    fprintf(stderr, "[x265la] lookahead estimates on %s\n", g_mode == MODE_CPU ? "the CPU (reference functions)" :
            g_mode == MODE_HOST ? "the CPU (hook control flow)" :
            g_mode == MODE_CHECK ? "the MI355X, each checked against the CPU" : "the MI355X");
    if (g_mode == MODE_CHECK)
        atexit(print_check_summary);
    const char* pr = getenv("X265AMD_LA_PROPAGATE");
    g_propagate = pr ? atoi(pr) != 0 : true;      /* on by default since round 5 (bit-identical, check mode 0 mismatches) */
    const char* st = getenv("X265AMD_LA_STATS");
    g_stats_on = st && *st && strcmp(st, "0");
    if (g_stats_on)
        atexit(print_stats);
}

/* One session per picture geometry and bit depth (x265amd_la_config), created on the first call
 * that needs it: every Lowres of one encoder shares its geometry, and a second encoder in the
 * same process with another resolution gets a session of its own instead of having its pictures
 * read with the first one's strides.  Sessions live until the process exits (the encoder has no
 * teardown hook for the lookahead; x265amd_la_destroy is exercised by tests/test_la_session.py).
 * Picture slots: a Lowres is uploaded into the slot of its key (the Lowres address) and x265
 * reuses a Frame's Lowres for later pictures, so the slots needed are the distinct Lowres objects
 * of the encoder's frame pool: rc-lookahead (<= 250, param.cpp X265_LOOKAHEAD_MAX) + bframes
 * (<= 16) + frame threads (<= 16) + DPB (<= 16) + the pre-lookahead queue, below 320. */
struct Session { x265amd_la_config cfg; x265amd_la* la; };
std::vector<Session> g_sessions;
enum { LA_MAX_FRAMES = 320 };

x265amd_la* session(const Lowres& f)
{
    x265amd_la_config c;
    memset(&c, 0, sizeof(c));
    c.depth = X265_DEPTH;
    c.width_cu = (int)f.maxBlocksInRow;
    c.height_cu = (int)f.maxBlocksInCol;
    c.lowres_stride = f.lumaStride;
    c.planesize = f.buffer[1] - f.buffer[0];
    c.padoffset = f.lowresPlane[0] - f.buffer[0];
    c.max_frames = LA_MAX_FRAMES;
    c.max_threads = 128;         // pool workers + API / lookahead threads
    pthread_mutex_lock(&g_mu);
    x265amd_la* la = NULL;
    for (size_t i = 0; i < g_sessions.size() && !la; i++)
    {
        const x265amd_la_config& s = g_sessions[i].cfg;
        if (s.width_cu == c.width_cu && s.height_cu == c.height_cu && s.lowres_stride == c.lowres_stride &&
            s.planesize == c.planesize && s.padoffset == c.padoffset)
            la = g_sessions[i].la;
    }
    if (!la && !g_la_status)
    {
        TabBitCost bc;
        c.mvcost = bc.table(X265_LOOKAHEAD_QP);
        c.mvcost_range = 1 << 14;    // > every qpel MV difference of a 2160p lowres search
        g_la_status = x265amd_la_create(&c, &la);
        if (g_la_status)
        {
            fprintf(stderr, "[x265la] x265amd_la_create failed: %s\n", x265amd_strerror(g_la_status));
            la = NULL;
        }
        else
        {
            Session s = { c, la };
            g_sessions.push_back(s);
        }
    }
    pthread_mutex_unlock(&g_mu);
    return la;
}

void report(const char* what, int st)
{
    if (st) fprintf(stderr, "[x265la] %s failed: %s\n", what, x265amd_strerror(st));
}

int g_mismatches = 0;
int g_prop_mismatches = 0;

/* X265AMD_LA_STATS=1: calls and wall time per kind, printed at exit */
enum { ST_INTRA, ST_P, ST_B, ST_BATCH_P, ST_BATCH_B, ST_HOST, ST_P_WEIGHTED, ST_HOST_WEIGHTED, ST_PROPAGATE, ST_N };
const char* const st_name[ST_N] = { "intra", "P single", "B single", "P batched", "B batched", "host loops",
                                    "P weighted", "B weighted", "propagate" };
struct Stat { long calls, jobs; double sec; };
Stat g_stat[ST_N];
bool g_stats_on = false;

double now_s()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

void stat_add(int k, long jobs, double t0)
{
    if (!g_stats_on) return;
    const double dt = now_s() - t0;
    pthread_mutex_lock(&g_mu);
    g_stat[k].calls++;
    g_stat[k].jobs += jobs;
    g_stat[k].sec += dt;
    pthread_mutex_unlock(&g_mu);
}

void print_stats()
{
    for (int k = 0; k < ST_N; k++)
        if (g_stat[k].calls)
            fprintf(stderr, "[x265la] stats %-10s calls %6ld estimates %6ld  %8.1f ms  (%.3f ms/call)\n", st_name[k],
                    g_stat[k].calls, g_stat[k].jobs, 1e3 * g_stat[k].sec, 1e3 * g_stat[k].sec / g_stat[k].calls);
}

int ncu_of(const Lowres& f) { return (int)(f.maxBlocksInRow * f.maxBlocksInCol); }

void print_check_summary()
{
    fprintf(stderr, "[x265la] check: %d mismatching estimates\n", g_mismatches);
    fprintf(stderr, "[x265la] check: %d mismatching propagations\n", g_prop_mismatches);
}

/* X265AMD_LOOKAHEAD=check: scratch outputs of one device estimate and their comparison with the
 * reference's results in the Lowres (first mismatches printed, count kept) */
struct CheckBufs
{
    int ncu = 0, hcu = 0;
    MV* mvs[2] = { NULL, NULL };
    int32_t* mvc[2] = { NULL, NULL };
    uint16_t* lc = NULL;
    int32_t* rs = NULL;
    void init(int n, int h, MV* const src_mvs[2], int32_t* const src_mvc[2])
    {
        ncu = n;
        hcu = h;
        for (int l = 0; l < 2; l++)
        {
            mvs[l] = (MV*)malloc(sizeof(MV) * n);
            mvc[l] = (int32_t*)malloc(sizeof(int32_t) * n);
            if (src_mvs[l]) memcpy(mvs[l], src_mvs[l], sizeof(MV) * n);   /* inputs of an unsearched list */
            if (src_mvc[l]) memcpy(mvc[l], src_mvc[l], sizeof(int32_t) * n);
        }
        lc = (uint16_t*)malloc(2 * n);
        rs = (int32_t*)malloc(4 * h);
    }
    ~CheckBufs()
    {
        for (int l = 0; l < 2; l++) { free(mvs[l]); free(mvc[l]); }
        free(lc);
        free(rs);
    }
    void compare(int p0, int p1, int b, int ns, const bool ds[2], Lowres* f, const int64_t ce[2], int mbs, int ref_mbs)
    {
        char what[256] = "";
        int first = -1;
        for (int l = 0; l < 2 && first < 0; l++)
        {
            if (!ds[l]) continue;
            const MV* r = f->lowresMvs[l][l ? p1 - b - 1 : b - p0 - 1];
            const int32_t* rc = f->lowresMvCosts[l][l ? p1 - b - 1 : b - p0 - 1];
            for (int i = 0; i < ncu && first < 0; i++)
                if (r[i].word != mvs[l][i].word || rc[i] != mvc[l][i])
                {
                    first = i;
                    snprintf(what, sizeof(what), "list %d mv/cost at cu %d: ref (%d,%d)/%d dev (%d,%d)/%d", l, i, r[i].x,
                             r[i].y, rc[i], mvs[l][i].x, mvs[l][i].y, mvc[l][i]);
                }
        }
        const uint16_t* rl = f->lowresCosts[b - p0][p1 - b];
        for (int i = 0; i < ncu && first < 0; i++)
            if (rl[i] != lc[i])
            {
                first = i;
                snprintf(what, sizeof(what), "lowresCosts at cu %d: ref %d dev %d", i, rl[i], lc[i]);
            }
        const int32_t* rr = f->rowSatds[b - p0][p1 - b];
        for (int i = 0; i < hcu && first < 0; i++)
            if (rr[i] != rs[i])
            {
                first = i;
                snprintf(what, sizeof(what), "rowSatds at row %d: ref %d dev %d", i, rr[i], rs[i]);
            }
        if (first < 0 && (f->costEst[b - p0][p1 - b] != ce[0] || f->costEstAq[b - p0][p1 - b] != ce[1]))
        {
            first = 0;
            snprintf(what, sizeof(what), "costEst ref %lld/%lld dev %lld/%lld", (long long)f->costEst[b - p0][p1 - b],
                     (long long)f->costEstAq[b - p0][p1 - b], (long long)ce[0], (long long)ce[1]);
        }
        if (first < 0 && p1 == b && mbs != ref_mbs)
        {
            first = 0;
            snprintf(what, sizeof(what), "intraMbs ref %d dev %d", ref_mbs, mbs);
        }
        if (first >= 0)
        {
            int n = __sync_add_and_fetch(&g_mismatches, 1);
            if (n <= 20)
                fprintf(stderr, "[x265la] CHECK MISMATCH estimate (p0 %d, p1 %d, b %d) frame %d, slices %d, search %d/%d: %s\n",
                        p0, p1, b, f->frameNum, ns, ds[0], ds[1], what);
        }
    }
};

} // namespace

namespace X265_NS {

/* cuTree's propagation step (slicetype.cpp:1741-1842) on the device: the reference's set-up (bipred
 * weights, list distances, the fps factor, the zeroed first row of a non-referenced frame's
 * propagateCost) restated, the per-CU loop one x265amd_la_propagate call.  With VBV the reference's
 * cuTreeFinish follows the loop, so that configuration runs the reference's function.
 * X265AMD_LA_PROPAGATE=1 selects it (built in round 4, off by default until it has run on the box;
 * X265AMD_LOOKAHEAD=check then compares every propagation with the reference's). */
void Lookahead::estimateCUPropagate(Lowres** frames, double averageDuration, int p0, int p1, int b, int referenced)
{
    pthread_once(&g_mode_once, read_mode);
    if (!g_propagate || g_mode == MODE_CPU || g_mode == MODE_HOST ||
        (m_param->rc.vbvBufferSize && m_param->lookaheadDepth && referenced))
    {
        x265ref_estimateCUPropagate(this, frames, averageDuration, p0, p1, b, referenced);
        return;
    }
    x265amd_la* la = session(*frames[b]);
    if (!la)
    {
        x265ref_estimateCUPropagate(this, frames, averageDuration, p0, p1, b, referenced);
        return;
    }
    const int32_t distScaleFactor = (((b - p0) << 8) + ((p1 - p0) >> 1)) / (p1 - p0);
    const int32_t bipredWeight = m_param->bEnableWeightedBiPred ? 64 - (distScaleFactor >> 2) : 32;
    const int bipredWeights[2] = { bipredWeight, 64 - bipredWeight };
    memset(m_scratch, 0, m_8x8Width * sizeof(int));
    const double fpsFactor = CLIP_DURATION((double)m_param->fpsDenom / m_param->fpsNum) / CLIP_DURATION(averageDuration);
    if (!referenced)
        memset(frames[b]->propagateCost, 0, m_8x8Width * sizeof(uint16_t));
    Lowres* f = frames[b];
    const int ncu = ncu_of(*f);
    /* list 1 exists only for a B estimate (b < p1); a P estimate's lowres costs never mark it used */
    const int32_t* mvs0 = (const int32_t*)f->lowresMvs[0][b - p0 - 1];
    const int32_t* mvs1 = b < p1 ? (const int32_t*)f->lowresMvs[1][p1 - b - 1] : NULL;
    uint16_t* rc0 = frames[p0]->propagateCost;
    uint16_t* rc1 = b < p1 ? frames[p1]->propagateCost : NULL;
    uint16_t* chk0 = NULL;
    uint16_t* chk1 = NULL;
    if (g_mode == MODE_CHECK)
    {
        /* the device writes into copies; the reference's own loop then updates the real arrays */
        chk0 = (uint16_t*)malloc(2 * ncu);
        memcpy(chk0, rc0, 2 * ncu);
        rc0 = chk0;
        if (rc1)
        {
            chk1 = (uint16_t*)malloc(2 * ncu);
            memcpy(chk1, rc1, 2 * ncu);
            rc1 = chk1;
        }
    }
    const double t0 = now_s();
    const int st = x265amd_la_propagate(la, referenced ? f->propagateCost : NULL, f->intraCost,
                                        f->lowresCosts[b - p0][p1 - b], f->invQscaleFactor, mvs0, mvs1, fpsFactor,
                                        bipredWeights, rc0, rc1);
    report("x265amd_la_propagate", st);
    stat_add(ST_PROPAGATE, 1, t0);
    if (g_mode == MODE_CHECK)
    {
        x265ref_estimateCUPropagate(this, frames, averageDuration, p0, p1, b, referenced);
        if (!st && (memcmp(chk0, frames[p0]->propagateCost, 2 * ncu) ||
                    (chk1 && memcmp(chk1, frames[p1]->propagateCost, 2 * ncu))))
        {
            int n = __sync_add_and_fetch(&g_prop_mismatches, 1);
            if (n <= 20)
                fprintf(stderr, "[x265la] CHECK MISMATCH propagation (p0 %d, p1 %d, b %d, referenced %d)\n", p0, p1, b,
                        referenced);
        }
        free(chk0);
        free(chk1);
    }
}

void LookaheadTLD::lowresIntraEstimate(Lowres& fenc)
{
    pthread_once(&g_mode_once, read_mode);
    if (g_mode == MODE_CPU || g_mode == MODE_HOST)
    {
        x265ref_lowresIntraEstimate(this, &fenc);
        return;
    }
    x265amd_la* la = session(fenc);
    int st = la ? x265amd_la_load(la, &fenc, fenc.frameNum, fenc.buffer[0], fenc.invQscaleFactor) : -1;
    if (la) report("x265amd_la_load", st);
    int64_t ce[2];
    if (!st && g_mode == MODE_CHECK)
    {
        const int ncu = ncu_of(fenc), hcu = (int)fenc.maxBlocksInCol;
        int32_t* ic = (int32_t*)malloc(4 * ncu);
        uint8_t* im = (uint8_t*)malloc(ncu);
        uint16_t* lc = (uint16_t*)malloc(2 * ncu);
        int32_t* rs = (int32_t*)malloc(4 * hcu);
        st = x265amd_la_intra(la, &fenc, ic, im, lc, rs, ce);
        report("x265amd_la_intra", st);
        x265ref_lowresIntraEstimate(this, &fenc);
        if (!st && (memcmp(ic, fenc.intraCost, 4 * ncu) || memcmp(im, fenc.intraMode, ncu) ||
                    memcmp(lc, fenc.lowresCosts[0][0], 2 * ncu) || memcmp(rs, fenc.rowSatds[0][0], 4 * hcu) ||
                    ce[0] != fenc.costEst[0][0] || ce[1] != fenc.costEstAq[0][0]))
        {
            __sync_add_and_fetch(&g_mismatches, 1);
            fprintf(stderr, "[x265la] CHECK MISMATCH intra estimate of frame %d\n", fenc.frameNum);
        }
        free(ic); free(im); free(lc); free(rs);
        return;
    }
    if (!st)
    {
        const double t0 = now_s();
        st = x265amd_la_intra(la, &fenc, fenc.intraCost, fenc.intraMode, fenc.lowresCosts[0][0], fenc.rowSatds[0][0],
                              ce);
        report("x265amd_la_intra", st);
        stat_add(ST_INTRA, 1, t0);
    }
    if (st)
    {
        /* status recorded: the encode fails; keep the encoder's state valid until it stops */
        x265ref_lowresIntraEstimate(this, &fenc);
        return;
    }
    fenc.costEst[0][0] = ce[0];
    fenc.costEstAq[0][0] = ce[1];
}

int64_t CostEstimateGroup::estimateFrameCost(LookaheadTLD& tld, int p0, int p1, int b, bool bIntraPenalty)
{
    pthread_once(&g_mode_once, read_mode);
    if (g_mode == MODE_CPU)
        return x265ref_estimateFrameCost(this, &tld, p0, p1, b, bIntraPenalty);

    Lowres*     fenc  = m_frames[b];
    x265_param* param = m_lookahead.m_param;
    int64_t     score = 0;

    if (fenc->costEst[b - p0][p1 - b] >= 0 && fenc->rowSatds[b - p0][p1 - b][0] != -1)
        score = fenc->costEst[b - p0][p1 - b];
    else
    {
        bool bDoSearch[2];
        bDoSearch[0] = p0 < b && fenc->lowresMvs[0][b - p0 - 1][0].x == 0x7FFF;
        bDoSearch[1] = p1 > b && fenc->lowresMvs[1][p1 - b - 1][0].x == 0x7FFF;

        fenc->weightedRef[b - p0].isWeighted = false;
        if (param->bEnableWeightedPred && bDoSearch[0])
            tld.weightsAnalyse(*m_frames[b], *m_frames[p0]);

        fenc->costEst[b - p0][p1 - b] = 0;
        fenc->costEstAq[b - p0][p1 - b] = 0;

        /* the reference's choice between cooperative slices and one serial pass (:2007) */
        const bool coop = !m_batchMode && m_lookahead.m_numCoopSlices > 1 && ((p1 > b) || bDoSearch[0] || bDoSearch[1]);
        const int rps = coop ? m_lookahead.m_numRowsPerSlice : m_lookahead.m_8x8Height;
        const int ns = coop ? m_lookahead.m_numCoopSlices : 1;
        const bool weighted = fenc->weightedRef[b - p0].isWeighted;
        x265amd_la* la = (g_mode == MODE_GPU || g_mode == MODE_CHECK) ? session(*fenc) : NULL;
        const bool device = la && ((p1 == b && bDoSearch[0]) || (p1 > b && !weighted));

        /* X265AMD_LOOKAHEAD=check: the device estimate goes to scratch copies, the host loops below
         * produce the reference's results in the Lowres, and the two are compared */
        const bool check = g_mode == MODE_CHECK;
        const int ncu = m_lookahead.m_8x8Width * m_lookahead.m_8x8Height, hcu = m_lookahead.m_8x8Height;
        const int d0 = b - p0 - 1, d1 = p1 - b - 1;
        MV* mvs[2] = { p0 < b ? fenc->lowresMvs[0][d0] : NULL, p1 > b ? fenc->lowresMvs[1][d1] : NULL };
        int32_t* mvc[2] = { p0 < b ? fenc->lowresMvCosts[0][d0] : NULL, p1 > b ? fenc->lowresMvCosts[1][d1] : NULL };
        uint16_t* lc = fenc->lowresCosts[b - p0][p1 - b];
        int32_t* rs = fenc->rowSatds[b - p0][p1 - b];
        CheckBufs cb;
        if (check && device)
        {
            cb.init(ncu, hcu, mvs, mvc);
            for (int l = 0; l < 2; l++)
            {
                mvs[l] = cb.mvs[l];
                mvc[l] = cb.mvc[l];
            }
            lc = cb.lc;
            rs = cb.rs;
        }
        bool done = false;
        int64_t ce[2] = { 0, 0 };
        int32_t mbs = 0;
        if (device)
        {
            /* outputs reach the Lowres only when the device call succeeded; on a failure the
             * status is recorded (the encode will fail) and the estimate is computed on the host
             * so the encoder's state stays valid until it stops */
            int st;
            const double t0 = now_s();
            if (p1 == b)
            {
                st = x265amd_la_pcost(la, fenc, m_frames[p0], weighted ? tld.wbuffer[0] : NULL, rps, ns,
                                      (int16_t*)mvs[0], mvc[0], lc, rs, ce, &mbs);
                report("x265amd_la_pcost", st);
                stat_add(weighted ? ST_P_WEIGHTED : ST_P, 1, t0);
            }
            else
            {
                st = x265amd_la_bcost(la, fenc, m_frames[p0], m_frames[p1], bDoSearch[0], bDoSearch[1], rps, ns,
                                      (int16_t*)mvs[0], mvc[0], (int16_t*)mvs[1], mvc[1], lc, rs, ce);
                report("x265amd_la_bcost", st);
                stat_add(ST_B, 1, t0);
            }
            if (!st && !check)
            {
                if (p1 == b)
                    fenc->intraMbs[b - p0] += mbs;
                fenc->costEst[b - p0][p1 - b] = ce[0];
                fenc->costEstAq[b - p0][p1 - b] = ce[1];
                done = true;
            }
        }
        const int mbs_before = fenc->intraMbs[b - p0];
        const double th = now_s();
        if (done)
            ;
        else if (coop)
        {
            /* the reference's cooperative slices (:2012-2037), run here one after another:
             * slices are independent and their sums commute */
            memset(&m_slice, 0, sizeof(Slice) * ns);
            for (int i = 0; i < ns; i++)
            {
                const int firstY = rps * i;
                const int lastY = (i == ns - 1) ? m_lookahead.m_8x8Height - 1 : rps * (i + 1) - 1;
                bool lastRow = true;
                for (int cuY = lastY; cuY >= firstY; cuY--)
                {
                    fenc->rowSatds[b - p0][p1 - b][cuY] = 0;
                    for (int cuX = m_lookahead.m_8x8Width - 1; cuX >= 0; cuX--)
                        estimateCUCost(tld, cuX, cuY, p0, p1, b, bDoSearch, lastRow, i);
                    lastRow = false;
                }
            }
            for (int i = 0; i < ns; i++)
            {
                fenc->costEst[b - p0][p1 - b] += m_slice[i].costEst;
                fenc->costEstAq[b - p0][p1 - b] += m_slice[i].costEstAq;
                if (p1 == b)
                    fenc->intraMbs[b - p0] += m_slice[i].intraMbs;
            }
        }
        else
        {
            /* the reference's serial pass (:2041-2050) */
            bool lastRow = true;
            for (int cuY = m_lookahead.m_8x8Height - 1; cuY >= 0; cuY--)
            {
                fenc->rowSatds[b - p0][p1 - b][cuY] = 0;
                for (int cuX = m_lookahead.m_8x8Width - 1; cuX >= 0; cuX--)
                    estimateCUCost(tld, cuX, cuY, p0, p1, b, bDoSearch, lastRow, -1);
                lastRow = false;
            }
        }

        if (!done)
            stat_add(weighted && p1 > b ? ST_HOST_WEIGHTED : ST_HOST, 1, th);
        if (check && device)
            cb.compare(p0, p1, b, ns, bDoSearch, fenc, ce, mbs, fenc->intraMbs[b - p0] - mbs_before);

        score = fenc->costEst[b - p0][p1 - b];

        if (b != p1)
            score = score * 100 / (130 + param->bFrameBias);

        fenc->costEst[b - p0][p1 - b] = score;
    }

    if (bIntraPenalty)
        // arbitrary penalty for I-blocks after B-frames
        score += score * fenc->intraMbs[b - p0] / (tld.ncu * 8);

    return score;
}

/* CostEstimateGroup::finishBatch (slicetype.cpp:1919-1926): the reference hands the batch's
 * estimates to its bonded workers, one estimateFrameCost each; the estimates of a batch are
 * independent (slicetype.cpp:1231-1298 builds them so), so here every device-eligible estimate of
 * the batch goes out in ONE launch per kind — the motion-search batch's P / B searches, the
 * frame-cost batch's B estimates on stored MVs — after each one's estimateFrameCost preamble
 * (cost cache, bDoSearch, weightsAnalyse) on this thread.  A weighted estimate runs through
 * estimateFrameCost alone (its weighted planes live in this thread's wbuffer), a P estimate on
 * stored MVs through the host loop (no search: a few operations per CU). */
void CostEstimateGroup::finishBatch()
{
    pthread_once(&g_mode_once, read_mode);
    if (g_mode != MODE_GPU)
    {
        x265ref_finishBatch(this);
        return;
    }
    LookaheadTLD& tld = m_lookahead.m_tld[m_lookahead.m_pool ? m_lookahead.m_pool->m_numWorkers : 0];
    x265_param* param = m_lookahead.m_param;
    std::vector<x265amd_la_pjob> pj;
    std::vector<x265amd_la_bjob> bj;
    std::vector<int> pidx, bidx, host;
    x265amd_la* la = NULL;
    for (int i = 0; i < m_jobTotal; i++)
    {
        const Estimate& e = m_estimates[i];
        const int p0 = e.p0, p1 = e.p1, b = e.b;
        Lowres* fenc = m_frames[b];
        if (fenc->costEst[b - p0][p1 - b] >= 0 && fenc->rowSatds[b - p0][p1 - b][0] != -1)
            continue;
        bool bDoSearch[2];
        bDoSearch[0] = p0 < b && fenc->lowresMvs[0][b - p0 - 1][0].x == 0x7FFF;
        bDoSearch[1] = p1 > b && fenc->lowresMvs[1][p1 - b - 1][0].x == 0x7FFF;
        fenc->weightedRef[b - p0].isWeighted = false;
        if (param->bEnableWeightedPred && bDoSearch[0])
            tld.weightsAnalyse(*m_frames[b], *m_frames[p0]);
        if (fenc->weightedRef[b - p0].isWeighted)
        {
            estimateFrameCost(tld, p0, p1, b, false);   /* analyses again (same result) and runs alone */
            continue;
        }
        if (!la)
            la = session(*fenc);
        fenc->costEst[b - p0][p1 - b] = 0;
        fenc->costEstAq[b - p0][p1 - b] = 0;
        if (la && p1 == b && bDoSearch[0])
        {
            x265amd_la_pjob j;
            memset(&j, 0, sizeof(j));
            j.fenc = fenc;
            j.ref = m_frames[p0];
            j.mvs = (int16_t*)fenc->lowresMvs[0][b - p0 - 1];
            j.mv_costs = fenc->lowresMvCosts[0][b - p0 - 1];
            j.lowres_costs = fenc->lowresCosts[b - p0][p1 - b];
            j.row_satd = fenc->rowSatds[b - p0][p1 - b];
            pj.push_back(j);
            pidx.push_back(i);
        }
        else if (la && p1 > b)
        {
            x265amd_la_bjob j;
            memset(&j, 0, sizeof(j));
            j.fenc = fenc;
            j.ref0 = m_frames[p0];
            j.ref1 = m_frames[p1];
            j.do_search0 = bDoSearch[0];
            j.do_search1 = bDoSearch[1];
            j.mvs0 = (int16_t*)fenc->lowresMvs[0][b - p0 - 1];
            j.mv_costs0 = fenc->lowresMvCosts[0][b - p0 - 1];
            j.mvs1 = (int16_t*)fenc->lowresMvs[1][p1 - b - 1];
            j.mv_costs1 = fenc->lowresMvCosts[1][p1 - b - 1];
            j.lowres_costs = fenc->lowresCosts[b - p0][p1 - b];
            j.row_satd = fenc->rowSatds[b - p0][p1 - b];
            bj.push_back(j);
            bidx.push_back(i);
        }
        else
            host.push_back(i);
    }
    const int rows = m_lookahead.m_8x8Height;
    /* the P and B calls succeed or fail independently: the results of a successful call are
     * applied, the estimates of a failed one go to the host loop below (the status is recorded,
     * so the encode fails, but the encoder's state stays valid until it stops) */
    int stp = 0, stb = 0;
    if (!pj.empty())
    {
        const double t0 = now_s();
        stp = x265amd_la_pcost_n(la, (int)pj.size(), &pj[0], rows, 1);
        report("x265amd_la_pcost_n", stp);
        stat_add(ST_BATCH_P, (long)pj.size(), t0);
        if (stp)
            host.insert(host.end(), pidx.begin(), pidx.end());
    }
    if (!bj.empty())
    {
        const double t0 = now_s();
        stb = x265amd_la_bcost_n(la, (int)bj.size(), &bj[0], rows, 1);
        report("x265amd_la_bcost_n", stb);
        stat_add(ST_BATCH_B, (long)bj.size(), t0);
        if (stb)
            host.insert(host.end(), bidx.begin(), bidx.end());
    }
    for (size_t k = 0; k < pj.size() && !stp; k++)
    {
        const Estimate& e = m_estimates[pidx[k]];
        Lowres* fenc = m_frames[e.b];
        fenc->costEst[e.b - e.p0][0] = pj[k].cost_est[0];
        fenc->costEstAq[e.b - e.p0][0] = pj[k].cost_est[1];
        fenc->intraMbs[e.b - e.p0] += pj[k].intra_mbs;
    }
    for (size_t k = 0; k < bj.size() && !stb; k++)
    {
        const Estimate& e = m_estimates[bidx[k]];
        Lowres* fenc = m_frames[e.b];
        fenc->costEst[e.b - e.p0][e.p1 - e.b] = bj[k].cost_est[0] * 100 / (130 + param->bFrameBias);
        fenc->costEstAq[e.b - e.p0][e.p1 - e.b] = bj[k].cost_est[1];
    }
    /* the rest: the reference's serial pass of batch mode (:2041-2050) on this thread */
    for (size_t k = 0; k < host.size(); k++)
    {
        const Estimate& e = m_estimates[host[k]];
        const int p0 = e.p0, p1 = e.p1, b = e.b;
        Lowres* fenc = m_frames[b];
        const double th = now_s();
        bool bDoSearch[2];
        bDoSearch[0] = p0 < b && fenc->lowresMvs[0][b - p0 - 1][0].x == 0x7FFF;
        bDoSearch[1] = p1 > b && fenc->lowresMvs[1][p1 - b - 1][0].x == 0x7FFF;
        fenc->costEst[b - p0][p1 - b] = 0;
        fenc->costEstAq[b - p0][p1 - b] = 0;
        bool lastRow = true;
        for (int cuY = m_lookahead.m_8x8Height - 1; cuY >= 0; cuY--)
        {
            fenc->rowSatds[b - p0][p1 - b][cuY] = 0;
            for (int cuX = m_lookahead.m_8x8Width - 1; cuX >= 0; cuX--)
                estimateCUCost(tld, cuX, cuY, p0, p1, b, bDoSearch, lastRow, -1);
            lastRow = false;
        }
        if (b != p1)
            fenc->costEst[b - p0][p1 - b] = fenc->costEst[b - p0][p1 - b] * 100 / (130 + param->bFrameBias);
        stat_add(ST_HOST, 1, th);
    }
    m_jobTotal = m_jobAcquired = 0;
}

} // namespace X265_NS

/* called by the encoder binding before x265_encoder_close frees the encoder's Lowres buffers (and again after
 * it; oracle/hip_encoder_main.cpp): the closing encoder's lookahead sessions are drained, their page-locked
 * buffers unregistered while still allocated, and destroyed, so a later encoder in the same process — whose Lowres objects may sit at
 * the same addresses with the same frame numbers — never finds the earlier encoder's planes resident */
extern "C" void x265amd_la_encoder_closed(void)
{
    pthread_mutex_lock(&g_mu);
    for (Session& s : g_sessions)
        x265amd_la_destroy(s.la);
    g_sessions.clear();
    pthread_mutex_unlock(&g_mu);
}
