// mesession.cpp — f2 encoder session: the main encoder's motion searches on the MI355X
// (include/x265_amd.h, x265amd_mes_*).
//
// Search::predInterSearch (search.cpp:2050-2231) runs one MotionEstimate::motionEstimate per
// (list, reference) of a PU, one after another on a worker thread; the searches of one PU are
// independent given their predictors.  A session runs them on the device:
//   * reference pictures: the padded luma plane of each reconstructed reference PicYuv
//     (picyuv.cpp:51-91) in one device arena, uploaded CTU row by CTU row as the encoder
//     publishes them (Frame::m_reconRowCount, framefilter.cpp:520: rows below the count are
//     deblocked, SAO-filtered and border-extended, so they never change again) — each row once,
//     whichever thread needs it first;
//   * MV cost tables: the encoder's BitCost table of each QP (bitcost.cpp:31-57) uploaded once;
//   * the launch service (round 5, cfg.launchers > 0): worker threads only POST requests (the PU's
//     source block and its job descriptors are copied into a per-thread request slot) and continue;
//     `launchers` service threads each take EVERY queued request of every worker, stage them in one
//     pinned buffer, and run one upload + one launch of the f2 kernel (one batch per PU size) + one
//     download on their own stream, then publish the outputs and wake the waiters.  So a worker never
//     makes a HIP call on the search path (no launch / copy / event cost on the encoder's cores, no
//     contention of 16 workers' streams for the 4 hardware queues), and the searches of all workers
//     that are in flight at once share one launch.  With two launchers one batch gathers while the
//     other is on the device.
//   * without launchers (cfg.launchers == 0, the round-4 form): per host thread a non-blocking
//     stream, pinned staging and device scratch; x265amd_mes_search is synchronous on it.
// Failures are returned AND recorded in the backend's sticky status (x265amd_provider_status),
// except the capacity limits (pictures, tables, threads, request slots: ENOMEM), after which the
// caller searches that PU on the host.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <new>
#include <thread>
#include <sched.h>
#include <unordered_map>
#include <vector>

#include "hostreg.h"
#include "../../../include/x265_amd.h"

namespace x265amd_provider {
extern std::atomic<int> g_status;
}

namespace {
// X265AMD_DEVSYNC_COPIES=1: the workers' synchronous row uploads stop a resident RDO server first (measured
// unnecessary: a synchronous copy on the null stream does not wait for the server's non-blocking stream, and the
// guard costs a server stop per upload; profiles/r06/rdo_server_ab.jsonl, call r06zf)
bool guard_copies()
{
    static const bool v = [] { const char* e = getenv("X265AMD_DEVSYNC_COPIES"); return e && *e == '1'; }();
    return v;
}
} // namespace

namespace {

int record(int st)
{
    if (st)
    {
        int zero = 0;
        x265amd_provider::g_status.compare_exchange_strong(zero, st);
    }
    return st;
}

#define MES_TRY(expr)                                  \
    do                                                 \
    {                                                  \
        int st_ = (int)(expr);                         \
        if (st_) return record(st_);                   \
    } while (0)

double now_s()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

constexpr int kSlots = 8;          // outstanding requests per host thread (tickets 0..7)
constexpr int kMaxJobs = 64;       // searches per request

} // namespace

struct x265amd_mes_stage
{
    uint8_t* dev = nullptr;
    uint8_t* host = nullptr;
    uint8_t* hdev = nullptr;     // the device's address of the pinned host buffer (null: not mapped)
    size_t cap = 0;
};

// one posted request: a copy of the PU's source block (packed, stride w) and its jobs
struct x265amd_mes_req
{
    int w = 0, h = 0, n = 0;
    bool chroma = false;                     // the 4:2:0 chroma blocks are in fenc after the luma block
    uint8_t* fenc = nullptr;                 // (64 * 64 + 2 * 32 * 32) * pix bytes
    x265amd_mes_job jobs[kMaxJobs];
    std::atomic<int> state{ 0 };             // 0 free, 1 queued / on the device, 2 done
    bool dropped = false;                    // the poster no longer wants it (free once done)
    int rc = 0;
    double t_post = 0;
};

struct x265amd_mes_thread
{
    hipStream_t st = nullptr;
    hipStream_t ast = nullptr;  // the outstanding x265amd_mes_submit's stream (legacy form)
    hipEvent_t ev = nullptr;    // blocking-sync event: the waiting worker sleeps (X265AMD_MES_SYNC=spin: spin)
    hipEvent_t aev = nullptr;   // completion of the outstanding legacy x265amd_mes_submit
    x265amd_mes_stage sync, async;
    int pending = 0;            // jobs of the outstanding submit (0: none)
    size_t pend_out = 0;        // its output offset in the async staging
    int pend_ticket = -1;       // service form: the ticket of the outstanding x265amd_mes_submit
    x265amd_mes_req req[kSlots];
};

struct x265amd_mes_launcher
{
    hipStream_t st = nullptr;
    hipEvent_t done = nullptr, k0 = nullptr, k1 = nullptr;
    x265amd_mes_stage g;
    uint8_t* vin = nullptr;     // X265AMD_MES_ZEROCOPY=3: the batch inputs in device memory the host writes
    size_t vcap = 0;            // through the large BAR (write-combined, never read back)
    std::thread th;
};

struct x265amd_mes
{
    x265amd_mes_config cfg;
    uint64_t id = 0;
    size_t pix = 1;
    int64_t rows = 0;                 // plane rows incl. both margins
    size_t plane_bytes = 0;
    int64_t slot_elems = 0;           // one picture: luma plane, then (chroma sessions) Cb and Cr planes
    int64_t crows = 0;                // chroma plane rows incl. both margins
    uint8_t* arena = nullptr;         // max_pictures padded pictures
    uint16_t* tables = nullptr;       // max_tables BitCost tables of 2 * range + 1 entries
    size_t table_elems = 0;

    struct Picture
    {
        int slot;
        int64_t gen;
        int rows_up;                  // CTU rows resident on the device
        const void* pinned[3];        // host planes registered with hipHostRegister (or null)
        std::mutex mu;                // one uploader at a time; the others wait for its rows
        // launch service: uploads are enqueued, not waited for — each on its uploader's stream after the
        // picture's previous upload (stream wait on up_ev), then up_ev re-recorded, so up_ev completes only
        // when every upload so far has; a launch waits on up_ev of every picture its searches read
        hipEvent_t up_ev = nullptr;
        bool up_any = false;
        // launcher uploads (X265AMD_MES_LUPLOAD=1): the worker only records the rows final so far and the
        // host planes; the launcher copies the missing rows on its own stream ahead of the batch that reads
        // them (no worker waits on copies; another launcher's rows still in flight are waited for on the
        // device, after a query)
        const void* planes[3] = { nullptr, nullptr, nullptr };
        int rows_want = 0;
        const void* up_by = nullptr;  // the launcher that enqueued the last upload
    };
    std::mutex mu;
    std::unordered_map<const void*, Picture*> pics;
    std::vector<Picture*> slot_pic;   // slot -> picture (max_pictures entries)
    std::unordered_map<const void*, int> tabs;
    std::vector<x265amd_mes_thread*> threads;
    std::atomic<int> next_slot{ 0 };

    // legacy coalescing of synchronous x265amd_mes_search calls (X265AMD_MES_COALESCE=1, no launchers)
    struct Request
    {
        int w, h;
        const void* fenc;
        intptr_t fenc_stride;
        int n;
        x265amd_mes_job* jobs;
        int rc;
        bool done;
    };
    std::mutex cmu;
    std::condition_variable ccv;
    std::vector<Request*> queue;
    bool busy = false;

    // launch service
    std::vector<x265amd_mes_launcher*> launchers;
    std::mutex qmu;                   // guards rq and stop
    std::condition_variable qcv;      // a request was queued
    std::vector<x265amd_mes_req*> rq;
    bool stop = false;
    std::atomic<bool> stop_flag{ false };
    std::mutex dmu;                   // waiters sleep on dcv
    std::condition_variable dcv;
    // The host cores are oversubscribed (the encoder's workers, frame and lookahead threads, and these
    // launchers on its 16 cores): a thread woken from a condition variable waits for a core for 0.2-5 ms
    // (profiles/r05/service_options_pinned_ab.txt: waits of that length sum to 10 of 13 s), and a
    // notify can hand the notifier's core to the woken thread.  So waiters and idle launchers first spin
    // (pause), then yield the core in a loop (sched_yield: any runnable thread goes first, otherwise the
    // waiter re-checks at once), and only then sleep; notifies go only to threads counted as sleeping.
    int spin_us = 50;                 // X265AMD_MES_SPIN_US: pause-spin before yielding
    int yield_us = 5000;              // X265AMD_MES_YIELD_US: yield loop before sleeping (waits)
    int idle_us = 500;                // X265AMD_MES_IDLE_US: launchers' yield loop on an empty queue
    int batch_us = 0;                 // X265AMD_MES_BATCH_US (round 6): a launcher that took fewer than batch_min
    int batch_min = 8;                // requests keeps gathering until the oldest has waited batch_us (bigger
                                      // launches: more searches per launch for the same kernel time)
    bool sync_upload = true;          // X265AMD_MES_SYNC_UPLOAD=0: reference uploads enqueued, ordered by events
                                      // (measured slower: the launches' cross-stream waits cost more than the
                                      // workers' upload waits, profiles/r05/upload_async_vs_sync_pinned_ab.txt)
    bool lupload = false;             // X265AMD_MES_LUPLOAD=1: the launchers upload the reference rows
    bool wstream = false;             // X265AMD_MES_WSTREAM=1: each worker uploads on a stream of its own
    std::atomic<int> qsleepers{ 0 };  // launchers sleeping on qcv
    int dsleepers = 0;                // waiters sleeping on dcv (guarded by dmu)
    std::atomic<int64_t> queued{ 0 }; // requests posted (the launchers' lock-free "anything new?" check)
    int trace = 0;                    // X265AMD_MES_TRACE=n: log the first n posts / launches / waits
    int zerocopy = 3;                 // X265AMD_MES_ZEROCOPY (default 3, round 6; 0: staged copies both ways)
                                      // 1: the kernel reads / writes the pinned staging;
                                      // 2: it writes its outputs there (inputs still uploaded); 3: the host
                                      // writes the inputs straight into device memory (large BAR) and the kernel
                                      // writes its outputs into the pinned staging: no copies at all
    bool prio = true;                 // X265AMD_MES_PRIORITY=0: launch streams at the default priority
    bool lspin = false;               // X265AMD_MES_LSPIN=1: launchers poll for completion (a busy core each:
                                      // slower on the encoder's 16-core budget, profiles/r05/bench_lspin_pinned_ab.txt)
    std::atomic<int> traced{ 0 };

    // statistics (x265amd_mes_stats)
    std::mutex smu;
    x265amd_mes_counters st{};
};

namespace {

struct TlsEntry { const x265amd_mes* s; uint64_t id; x265amd_mes_thread* t; };
thread_local std::vector<TlsEntry> tls;
std::atomic<uint64_t> g_next_id{ 1 };

int use_device(const x265amd_mes* s)
{
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) return X265AMD_ENODEV;
    if (cur != s->cfg.device && hipSetDevice(s->cfg.device) != hipSuccess) return X265AMD_ENODEV;
    return 0;
}

int wait(x265amd_mes_thread* t)
{
    if (t->ev)
    {
        const hipError_t e = hipEventRecord(t->ev, t->st);
        return e != hipSuccess ? (int)e : (int)hipEventSynchronize(t->ev);
    }
    return (int)hipStreamSynchronize(t->st);
}

int reserve(hipStream_t a, hipStream_t b, x265amd_mes_stage& g, size_t bytes)
{
    if (bytes <= g.cap) return 0;
    bytes = (bytes + 65535) & ~(size_t)65535;
    if (a) (void)hipStreamSynchronize(a);
    if (b) (void)hipStreamSynchronize(b);
    DevSyncScope quiet;                        // (hipFree / hipHostFree wait for every running kernel)
    (void)hipFree(g.dev);
    (void)hipHostFree(g.host);
    g.dev = g.host = nullptr;
    g.cap = 0;
    if (hipMalloc((void**)&g.dev, bytes) != hipSuccess ||
        hipHostMalloc((void**)&g.host, bytes, hipHostMallocMapped) != hipSuccess)
        return X265AMD_ENOMEM;
    g.hdev = nullptr;
    if (hipHostGetDevicePointer((void**)&g.hdev, g.host, 0) != hipSuccess) g.hdev = nullptr;
    (void)hipGetLastError();
    g.cap = bytes;
    return 0;
}

void free_thread(x265amd_mes_thread* t)
{
    if (t->st) (void)hipStreamSynchronize(t->st);
    if (t->ast) (void)hipStreamSynchronize(t->ast);
    for (x265amd_mes_stage* g : { &t->sync, &t->async })
    {
        (void)hipFree(g->dev);
        (void)hipHostFree(g->host);
    }
    if (t->st) (void)hipStreamDestroy(t->st);
    if (t->ast) (void)hipStreamDestroy(t->ast);
    if (t->ev) (void)hipEventDestroy(t->ev);
    if (t->aev) (void)hipEventDestroy(t->aev);
    for (auto& r : t->req) free(r.fenc);
    delete t;
}

// the calling thread's context; *out stays null and ENOMEM is returned WITHOUT recording it when the
// session's thread limit is reached (the caller then searches on the host)
int thread_ctx(x265amd_mes* s, x265amd_mes_thread** out)
{
    *out = nullptr;
    for (size_t i = 0; i < tls.size();)
    {
        if (tls[i].s == s && tls[i].id == s->id)
        {
            *out = tls[i].t;
            return 0;
        }
        if (tls[i].s == s)            // a destroyed session's entry at a reused address
        {
            tls[i] = tls.back();
            tls.pop_back();
            continue;
        }
        i++;
    }
    {
        std::lock_guard<std::mutex> g(s->mu);
        if ((int)s->threads.size() >= s->cfg.max_threads) return X265AMD_ENOMEM;
    }
    auto* t = new (std::nothrow) x265amd_mes_thread();
    if (!t) return record(X265AMD_ENOMEM);
    int rc = 0;
    DevSyncScope quiet;                        // (stream creation and allocation wait for running kernels)
    if (s->launchers.empty())
    {
        const char* sync = getenv("X265AMD_MES_SYNC");
        const bool spin = sync && !strcmp(sync, "spin");
        if (hipStreamCreateWithFlags(&t->st, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&t->ast, hipStreamNonBlocking) != hipSuccess ||
            reserve(t->st, t->ast, t->sync, 1 << 16) || reserve(t->st, t->ast, t->async, 1 << 16) ||
            (!spin && hipEventCreateWithFlags(&t->ev, hipEventBlockingSync | hipEventDisableTiming) != hipSuccess) ||
            hipEventCreateWithFlags(&t->aev, (spin ? 0 : hipEventBlockingSync) | hipEventDisableTiming) != hipSuccess)
            rc = X265AMD_ENOMEM;
    }
    else
    {
        // the worker thread itself makes no HIP call on the search path.  Its reference-row and table uploads
        // are synchronous copies (no stream of its own: creating one costs tens of ms on the thread, measured
        // 26 ms per hipStreamCreate in the encode's hip trace, profiles/r05/d/enc_hip_api_stats.csv), except in
        // the event-ordered upload mode, which needs the stream
        if ((!s->sync_upload || s->wstream) && !s->lupload &&
            (hipStreamCreateWithFlags(&t->st, hipStreamNonBlocking) != hipSuccess ||
             hipEventCreateWithFlags(&t->ev, hipEventBlockingSync | hipEventDisableTiming) != hipSuccess))
            rc = X265AMD_ENOMEM;
        for (auto& r : t->req)
            if (!rc && !(r.fenc = (uint8_t*)malloc((64 * 64 + 2 * 32 * 32) * s->pix))) rc = X265AMD_ENOMEM;
    }
    if (rc)
    {
        free_thread(t);
        return record(rc);
    }
    {
        std::lock_guard<std::mutex> g(s->mu);
        if ((int)s->threads.size() >= s->cfg.max_threads)
        {
            free_thread(t);
            return X265AMD_ENOMEM;
        }
        s->threads.push_back(t);
    }
    tls.push_back({ s, s->id, t });
    *out = t;
    return 0;
}

// batch layout in the staging buffers (byte offsets, 256-aligned)
struct Layout
{
    size_t fenc, fenc_c = 0, fenc_coff = 0, ref_coff = 0, fenc_off, ref_off, range, mvp, mvc, ncand, cost_off, out_mv,
        out_cost, evals, end;
    // cblk: elements of one request's chroma block (0: luma only), np requests
    Layout(int n, int h, int pix, int maxc, intptr_t fstride, size_t cblk = 0, int np = 0)
    {
        size_t o = 0;
        auto take = [&](size_t b) { size_t r = o; o = (o + b + 255) & ~(size_t)255; return r; };
        fenc = take((size_t)fstride * h * pix);
        if (cblk)
        {
            fenc_c = take(2 * cblk * np * pix);
            fenc_coff = take(8 * (size_t)n);
            ref_coff = take(8 * (size_t)n);
        }
        fenc_off = take(8 * (size_t)n);
        ref_off = take(8 * (size_t)n);
        range = take(8 * (size_t)n);
        mvp = take(4 * (size_t)n);
        mvc = take(4 * (size_t)maxc * n);
        ncand = take((size_t)n);
        cost_off = take(8 * (size_t)n);
        out_mv = take(4 * (size_t)n);
        out_cost = take(4 * (size_t)n);
        evals = take(8 * (size_t)n);
        end = o;
    }
};

int check_jobs(const x265amd_mes* s, int w, int h, const void* fenc, intptr_t fenc_stride, int n,
               const x265amd_mes_job* jobs)
{
    if (!s || n < 0 || (n && (!jobs || !fenc)) || w < 4 || h < 4 || w > 64 || h > 64 || (w & 3) || (h & 3) ||
        fenc_stride < w)
        return X265AMD_EINVAL;
    for (int i = 0; i < n; i++)
        if (jobs[i].slot < 0 || jobs[i].slot >= s->next_slot || jobs[i].table < 0 ||
            jobs[i].table >= s->cfg.max_tables || jobs[i].num_cand < 0 || jobs[i].num_cand > s->cfg.max_cand)
            return X265AMD_EINVAL;
    return 0;
}

// the device batch descriptor of n jobs staged at layout L in g (fenc blocks at stride fstride)
x265amd_me_batch make_batch(const x265amd_mes* s, const x265amd_mes_stage& g, const Layout& L, int w, int h, int n,
                            intptr_t fstride)
{
    x265amd_me_batch b;
    memset(&b, 0, sizeof(b));
    b.w = w;
    b.h = h;
    b.n = n;
    // the config carries x265_param::searchMethod (x265.h: DIA 0, HEX 1, UMH 2, STAR 3, FULL 4); the
    // search kernel numbers STAR 2 and UMH 3
    static const int kKernelMethod[5] = { 0, 1, 3, 2, 4 };
    b.method = kKernelMethod[s->cfg.method];
    b.subme = s->cfg.subme;
    b.merange = s->cfg.merange;
    b.max_cand = s->cfg.max_cand > 0 ? s->cfg.max_cand : 1;
    b.fenc = g.dev + L.fenc;
    b.fenc_stride = fstride;
    b.fenc_off = (const int64_t*)(g.dev + L.fenc_off);
    b.ref = s->arena;
    b.ref_stride = s->cfg.stride;
    b.ref_off = (const int64_t*)(g.dev + L.ref_off);
    b.mv_range = (const int16_t*)(g.dev + L.range);
    b.mvp = (const int16_t*)(g.dev + L.mvp);
    b.mvc = (const int16_t*)(g.dev + L.mvc);
    b.num_cand = g.dev + L.ncand;
    b.mvcost = s->tables;
    b.mvcost_off = (const int64_t*)(g.dev + L.cost_off);
    b.out_mv = (int16_t*)(g.dev + L.out_mv);
    b.out_cost = (int32_t*)(g.dev + L.out_cost);
    return b;
}

// the chroma fields of a batch whose np requests' chroma blocks are staged at L.fenc_c (Cb blocks, then Cr)
void chroma_batch(const x265amd_mes* s, const x265amd_mes_stage& g, const Layout& L, int w, int h, int np,
                  x265amd_me_batch& b)
{
    const size_t cblk = (size_t)(w / 2) * (h / 2);
    b.fenc_cb = g.dev + L.fenc_c;
    b.fenc_cr = g.dev + L.fenc_c + cblk * np * s->pix;
    b.fenc_cstride = w / 2;
    b.fenc_coff = (const int64_t*)(g.dev + L.fenc_coff);
    b.ref_cb = s->arena + (size_t)s->cfg.plane_elems * s->pix;
    b.ref_cr = s->arena + (size_t)(s->cfg.plane_elems + s->cfg.cplane_elems) * s->pix;
    b.ref_cstride = s->cfg.cstride;
    b.ref_coff = (const int64_t*)(g.dev + L.ref_coff);
}

// job i's descriptors into the host staging of layout L (source block at element offset foff)
void stage_job(const x265amd_mes* s, uint8_t* H, const Layout& L, int i, const x265amd_mes_job& j, int64_t foff,
               int64_t fcoff = 0)
{
    if (L.fenc_coff) ((int64_t*)(H + L.fenc_coff))[i] = fcoff;
    const int maxc = s->cfg.max_cand > 0 ? s->cfg.max_cand : 1;
    ((int64_t*)(H + L.fenc_off))[i] = foff;
    ((int64_t*)(H + L.ref_off))[i] = (int64_t)j.slot * s->slot_elems + s->cfg.org_offset + j.block_off;
    if (L.fenc_coff)
    {
        // the chroma block of the PU: half the luma origin's position (4:2:0)
        const int64_t x = j.block_off % s->cfg.stride, y = j.block_off / s->cfg.stride;
        ((int64_t*)(H + L.ref_coff))[i] = (int64_t)j.slot * s->slot_elems + s->cfg.corg_offset + (y >> 1) * s->cfg.cstride +
                                          (x >> 1);
    }
    memcpy((int16_t*)(H + L.range) + 4 * i, j.mv_range, 8);
    memcpy((int16_t*)(H + L.mvp) + 2 * i, j.mvp, 4);
    memcpy((int16_t*)(H + L.mvc) + 2 * (size_t)maxc * i, j.mvc, 4 * (size_t)j.num_cand);
    (H + L.ncand)[i] = (uint8_t)j.num_cand;
    ((int64_t*)(H + L.cost_off))[i] = (int64_t)j.table * (int64_t)s->table_elems + s->cfg.mvcost_range;
}

// outputs of n jobs staged at layout L (host copy after the download)
void read_out(const uint8_t* H, const Layout& L, int i, x265amd_mes_job& j)
{
    j.out_mv[0] = ((const int16_t*)(H + L.out_mv))[2 * i];
    j.out_mv[1] = ((const int16_t*)(H + L.out_mv))[2 * i + 1];
    j.out_cost = ((const int32_t*)(H + L.out_cost))[i];
}

// duration bins of the wait / batch histograms: < 0.05, < 0.2, < 1, < 5, >= 5 ms
static int hist_bin(double ms)
{
    return ms < 0.05 ? 0 : ms < 0.2 ? 1 : ms < 1 ? 2 : ms < 5 ? 3 : 4;
}

// ---------------------------------------------------------------- launch service
// one service thread: take every queued request, one staged batch per PU size, one upload, one launch
// (all sizes), one download, publish
int copy_rows(x265amd_mes* s, x265amd_mes::Picture* p, const void* const planes[3], int rows_final, hipStream_t st,
              size_t* total);

// grow the launcher's device-memory input buffer to its staging's capacity (fine-grained device memory the
// host writes through the large BAR); without a large BAR or on failure the launcher keeps the copies
void reserve_vin(x265amd_mes_launcher* L)
{
    (void)hipStreamSynchronize(L->st);
    DevSyncScope quiet;                        // (hipFree / hipExtMallocWithFlags wait for every running kernel)
    if (L->vin) (void)hipFree(L->vin);
    L->vin = nullptr;
    L->vcap = 0;
    int dev = 0, large_bar = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, dev) !=
        hipSuccess || !large_bar)
        return;
    if (hipExtMallocWithFlags((void**)&L->vin, L->g.cap, hipDeviceMallocFinegrained) != hipSuccess)
    {
        L->vin = nullptr;
        (void)hipGetLastError();
        return;
    }
    L->vcap = L->g.cap;
}

void launcher_main(x265amd_mes* s, x265amd_mes_launcher* L)
{
    (void)hipSetDevice(s->cfg.device);
    std::vector<x265amd_mes_req*> take;
    std::vector<x265amd_mes_req*> order;
    std::vector<Layout> lay;
    std::vector<x265amd_me_batch> bt;
    std::vector<size_t> base;
    std::vector<uint8_t> seen;
    for (;;)
    {
        {
            // nothing queued: yield-loop on the lock-free post count (back to it whenever another launcher
            // took what was posted), then sleep
            std::unique_lock<std::mutex> lk(s->qmu);
            while (s->rq.empty() && !s->stop)
            {
                const int64_t seen = s->queued.load(std::memory_order_acquire);
                lk.unlock();
                const double until = now_s() + 1e-6 * s->idle_us;
                bool moved = false;
                while (!(moved = s->queued.load(std::memory_order_acquire) != seen) &&
                       !s->stop_flag.load(std::memory_order_acquire) && now_s() < until)
                    sched_yield();
                lk.lock();
                if (!moved && s->rq.empty() && !s->stop)
                {
                    s->qsleepers.fetch_add(1, std::memory_order_acq_rel);
                    s->qcv.wait(lk, [&] { return s->stop || !s->rq.empty(); });
                    s->qsleepers.fetch_sub(1, std::memory_order_acq_rel);
                }
            }
            if (s->rq.empty()) return;                 // stop requested and nothing left
            take.swap(s->rq);
            s->rq.clear();
        }
        if (s->batch_us > 0 && (int)take.size() < s->batch_min)
        {
            double oldest = take[0]->t_post;
            for (auto* r : take) oldest = r->t_post < oldest ? r->t_post : oldest;
            const double until = oldest + 1e-6 * s->batch_us;
            while ((int)take.size() < s->batch_min && now_s() < until && !s->stop_flag.load(std::memory_order_acquire))
            {
                sched_yield();
                std::lock_guard<std::mutex> lk(s->qmu);
                if (!s->rq.empty())
                {
                    take.insert(take.end(), s->rq.begin(), s->rq.end());
                    s->rq.clear();
                }
            }
        }
        const double t_take = now_s();
        if (s->trace && s->traced.fetch_add(1) < s->trace)
            fprintf(stderr, "[mes] launcher %p takes %zu requests\n", (void*)L, take.size());
        // group by PU size, keeping the posting order inside a size
        order.clear();
        // batches: one per (PU size, chroma) — the size in first / second, chroma as a negative height
        std::vector<std::pair<int, int>> sizes;
        auto key_h = [](const x265amd_mes_req* r) { return r->chroma ? -r->h : r->h; };
        for (auto* r : take)
        {
            bool seen = false;
            for (auto& z : sizes) seen |= z.first == r->w && z.second == key_h(r);
            if (!seen) sizes.push_back({ r->w, key_h(r) });
        }
        lay.clear();
        bt.clear();
        base.clear();
        size_t total = 0;
        const int maxc = s->cfg.max_cand > 0 ? s->cfg.max_cand : 1;
        std::vector<int> nps, nj;
        for (auto& z : sizes)
        {
            int n = 0, np = 0;
            for (auto* r : take)
                if (r->w == z.first && key_h(r) == z.second) { n += r->n; np++; }
            const int h = z.second < 0 ? -z.second : z.second;
            lay.emplace_back(n, np * h, (int)s->pix, maxc, z.first, z.second < 0 ? (size_t)(z.first / 2) * (h / 2) : 0, np);
            nps.push_back(np);
            nj.push_back(n);
            base.push_back(total);
            total += lay.back().end;
        }
        int rc = reserve(L->st, nullptr, L->g, total);
        int njobs = 0;
        if (!rc && s->zerocopy == 3 && L->g.hdev && L->vcap < L->g.cap) reserve_vin(L);
        // mode 3: inputs written into device memory (the kernel reads them there), outputs into the pinned staging
        const bool v3 = s->zerocopy == 3 && L->g.hdev && L->vin;
        uint8_t* const in_host = v3 ? L->vin : L->g.host;
        uint8_t* const in_dev = v3 ? L->vin : L->g.dev;
        if (!rc)
        {
            for (size_t k = 0; k < sizes.size(); k++)
            {
                const int w = sizes[k].first, kh = sizes[k].second, h = kh < 0 ? -kh : kh;
                const size_t cblk = (size_t)(w / 2) * (h / 2);
                uint8_t* H = in_host + base[k];
                const Layout& Ly = lay[k];
                int i = 0, p = 0;
                for (auto* r : take)
                {
                    if (r->w != w || key_h(r) != kh) continue;
                    memcpy(H + Ly.fenc + (size_t)p * w * h * s->pix, r->fenc, (size_t)w * h * s->pix);
                    if (kh < 0)
                    {
                        const uint8_t* c = r->fenc + (size_t)w * h * s->pix;
                        memcpy(H + Ly.fenc_c + (size_t)p * cblk * s->pix, c, cblk * s->pix);
                        memcpy(H + Ly.fenc_c + ((size_t)nps[k] + p) * cblk * s->pix, c + cblk * s->pix, cblk * s->pix);
                    }
                    for (int q = 0; q < r->n; q++, i++)
                        stage_job(s, H, Ly, i, r->jobs[q], (int64_t)p * w * h, (int64_t)p * cblk);
                    order.push_back(r);
                    p++;
                }
                x265amd_mes_stage sub{ in_dev + base[k], in_host + base[k], nullptr, Ly.end };
                bt.push_back(make_batch(s, sub, Ly, w, h, i, w));
                if (kh < 0) chroma_batch(s, sub, Ly, w, h, p, bt.back());
                bt.back().eval_count = (uint32_t*)(sub.dev + Ly.evals);
                njobs += i;
            }
            if ((s->zerocopy == 2 && L->g.hdev) || v3)
            {
                // the kernel writes its outputs straight into the pinned staging (no download copy)
                const ptrdiff_t d = L->g.hdev - in_dev;
                for (size_t k = 0; k < bt.size(); k++)
                {
                    x265amd_me_batch& b = bt[k];
                    b.out_mv = (int16_t*)((uint8_t*)b.out_mv + d);
                    b.out_cost = (int32_t*)((uint8_t*)b.out_cost + d);
                    if (b.eval_count) b.eval_count = (uint32_t*)((uint8_t*)b.eval_count + d);
                }
            }
            else if (s->zerocopy == 1 && L->g.hdev)
            {
                // the kernel reads the descriptors and source blocks from the pinned staging and writes its
                // outputs there (no copies): the batch addresses are the host staging's
                for (size_t k = 0; k < bt.size(); k++)
                {
                    const ptrdiff_t d = L->g.hdev - L->g.dev;
                    auto mv = [d](const void* p) { return p ? (const void*)((const uint8_t*)p + d) : p; };
                    x265amd_me_batch& b = bt[k];
                    b.fenc = mv(b.fenc);
                    b.fenc_off = (const int64_t*)mv(b.fenc_off);
                    b.ref_off = (const int64_t*)mv(b.ref_off);
                    b.mv_range = (const int16_t*)mv(b.mv_range);
                    b.mvp = (const int16_t*)mv(b.mvp);
                    b.mvc = (const int16_t*)mv(b.mvc);
                    b.num_cand = (const uint8_t*)mv(b.num_cand);
                    b.mvcost_off = (const int64_t*)mv(b.mvcost_off);
                    b.out_mv = (int16_t*)mv(b.out_mv);
                    b.out_cost = (int32_t*)mv(b.out_cost);
                    b.eval_count = (uint32_t*)mv(b.eval_count);
                    if (b.fenc_cb)
                    {
                        b.fenc_cb = mv(b.fenc_cb);
                        b.fenc_cr = mv(b.fenc_cr);
                        b.fenc_coff = (const int64_t*)mv(b.fenc_coff);
                        b.ref_coff = (const int64_t*)mv(b.ref_coff);
                    }
                }
            }
            // the reference rows these searches read: every picture's uploads so far (enqueued by the workers)
            {
                seen.assign(s->slot_pic.size(), 0);          // slots already waited on
                for (auto* r : take)
                    for (int q = 0; q < r->n && !rc; q++)
                    {
                        const int sl = r->jobs[q].slot;
                        if (sl < 0 || sl >= (int)seen.size() || seen[sl]) continue;
                        seen[sl] = 1;
                        x265amd_mes::Picture* pic = s->slot_pic[sl];
                        if (!pic) continue;
                        std::lock_guard<std::mutex> pg(pic->mu);
                        if (!s->lupload)
                        {
                            if (pic->up_any) rc = (int)hipStreamWaitEvent(L->st, pic->up_ev, 0);
                            continue;
                        }
                        // launcher uploads: rows another launcher enqueued may still be in flight (up_ev
                        // completes only when every upload so far has: each uploader waits for it first)
                        if (pic->up_any && pic->up_by != L)
                        {
                            const hipError_t q = hipEventQuery(pic->up_ev);
                            if (q == hipErrorNotReady) rc = (int)hipStreamWaitEvent(L->st, pic->up_ev, 0);
                            else if (q != hipSuccess) rc = (int)q;
                        }
                        if (!rc && pic->rows_want > pic->rows_up)
                        {
                            const double t0 = now_s();
                            size_t total = 0;
                            if (!pic->up_ev) rc = (int)hipEventCreateWithFlags(&pic->up_ev, hipEventDisableTiming);
                            if (!rc) rc = copy_rows(s, pic, pic->planes, pic->rows_want, L->st, &total);
                            if (!rc) rc = (int)hipEventRecord(pic->up_ev, L->st);
                            if (rc) continue;
                            pic->up_any = true;
                            pic->up_by = L;
                            pic->rows_up = pic->rows_want;
                            std::lock_guard<std::mutex> sg(s->smu);
                            s->st.uploads++;
                            s->st.upload_bytes += (int64_t)total;
                            s->st.upload_ms += 1e3 * (now_s() - t0);
                        }
                    }
            }
            // one upload of every size's inputs (the output regions ride along: staging is contiguous)
            if (!rc && !(s->zerocopy == 1 && L->g.hdev) && !v3)
                rc = (int)hipMemcpyAsync(L->g.dev, L->g.host, total, hipMemcpyHostToDevice, L->st);
            // (the write-combined stores into device memory drain before the launch's doorbell)
            if (v3) __builtin_ia32_sfence();
            if (!rc) rc = (int)hipEventRecord(L->k0, L->st);
            if (!rc) rc = x265amd_motion_search(s->cfg.depth, (int)bt.size(), bt.data(), L->st);
            if (!rc) rc = (int)hipEventRecord(L->k1, L->st);
            for (size_t k = 0; k < sizes.size() && !rc && !(s->zerocopy && L->g.hdev) && !v3; k++)
                rc = (int)hipMemcpyAsync(L->g.host + base[k] + lay[k].out_mv, L->g.dev + base[k] + lay[k].out_mv,
                                         lay[k].end - lay[k].out_mv, hipMemcpyDeviceToHost, L->st);
            if (!rc) rc = (int)hipEventRecord(L->done, L->st);
            if (!rc && s->lspin)
            {
                // poll instead of sleeping on the completion interrupt (lower wake-up latency, one busy core)
                hipError_t q;
                while ((q = hipEventQuery(L->done)) == hipErrorNotReady)
                    __builtin_ia32_pause();
                rc = (int)q;
            }
            else if (!rc)
                rc = (int)hipEventSynchronize(L->done);
        }
        // algorithmic bytes of the launch: per full-pel evaluation the PU and its reference
        // block (2 W H b), per sub-pel evaluation the PU and the reference window of the 8-tap filters
        // ((W + 7) (H + 7) b + W H b)
        double algo = 0;
        int64_t efp = 0, esp = 0;
        if (!rc)
            for (size_t k = 0; k < sizes.size(); k++)
            {
                const double w = sizes[k].first, h = sizes[k].second < 0 ? -sizes[k].second : sizes[k].second;
                const double b = (double)s->pix;
                // with chroma: each sub-pel evaluation also interpolates and compares the two w/2 x h/2 chroma
                // blocks (4-tap: (w/2 + 3)(h/2 + 3) window)
                const double csub = sizes[k].second < 0 ? 2 * ((w / 2 + 3) * (h / 2 + 3) + (w / 2) * (h / 2)) : 0;
                const uint32_t* ev = (const uint32_t*)(L->g.host + base[k] + lay[k].evals);
                int64_t fp = 0, sp = 0;
                for (int i = 0; i < nj[k]; i++)
                {
                    fp += ev[2 * i];
                    sp += ev[2 * i + 1];
                }
                efp += fp;
                esp += sp;
                algo += fp * 2 * w * h * b + sp * ((w + 7) * (h + 7) + w * h + csub) * b;
            }
        float kms = 0;
        if (!rc) (void)hipEventElapsedTime(&kms, L->k0, L->k1);
        const double t_done = now_s();
        // publish: the outputs into each request, then wake the waiters
        if (!rc)
            for (size_t k = 0; k < sizes.size(); k++)
            {
                const int w = sizes[k].first, kh = sizes[k].second;
                const uint8_t* H = L->g.host + base[k];
                int i = 0;
                for (auto* r : take)
                {
                    if (r->w != w || key_h(r) != kh) continue;
                    for (int q = 0; q < r->n; q++, i++) read_out(H, lay[k], i, r->jobs[q]);
                }
            }
        // the states flip under dmu, where sleepers register, so a waiter that checked its state before the
        // flip is counted before the count is read here (no lost wake-up); spinning / yielding waiters read
        // the state without the lock
        double qdelay = 0;
        bool wake;
        {
            std::lock_guard<std::mutex> g(s->dmu);
            for (auto* r : take)
            {
                qdelay += t_take - r->t_post;
                r->rc = rc;
                r->state.store(2, std::memory_order_release);
            }
            wake = s->dsleepers > 0;
        }
        if (wake) s->dcv.notify_all();
        if (rc) record(rc);
        if (s->trace && s->traced.fetch_add(1) < s->trace)
            fprintf(stderr, "[mes] launcher %p done: rc %d, kernel %.3f ms, batch %.3f ms\n", (void*)L, rc, kms,
                    1e3 * (t_done - t_take));
        {
            std::lock_guard<std::mutex> g(s->smu);
            s->st.batches++;
            s->st.requests += (int64_t)take.size();
            s->st.jobs += njobs;
            s->st.kernel_ms += kms;
            s->st.evals_fpel += efp;
            s->st.evals_subpel += esp;
            s->st.algo_bytes += algo;
            if (kms > s->st.kernel_ms_max) s->st.kernel_ms_max = kms;
            const double bms = 1e3 * (t_done - t_take);
            const int hb = hist_bin(bms);
            s->st.batch_hist[hb]++;
            s->st.batch_hist_ms[hb] += bms;
            s->st.batch_ms += 1e3 * (t_done - t_take);
            s->st.queue_ms += 1e3 * qdelay;
            if ((int64_t)take.size() > s->st.max_requests_per_batch) s->st.max_requests_per_batch = (int64_t)take.size();
        }
        take.clear();
    }
}

// copy the plane rows of CTU rows [p->rows_up, rows_final) into the picture's slot: the top margin goes
// with row 0, the bottom margin (and the rows of a partial last CTU row) with the last row; chroma (4:2:0)
// the same at half height.  Enqueued on st, or synchronous without a stream.
int copy_rows(x265amd_mes* s, x265amd_mes::Picture* p, const void* const planes[3], int rows_final, hipStream_t st,
              size_t* total)
{
    uint8_t* dst = s->arena + (size_t)p->slot * s->slot_elems * s->pix;
    const int np = s->cfg.chroma ? 3 : 1;
    for (int k = 0; k < np; k++)
    {
        const int64_t margin = k ? s->cfg.cmargin_y : s->cfg.margin_y;
        const int64_t rh = k ? s->cfg.ctu_size / 2 : s->cfg.ctu_size;
        const int64_t stride = k ? s->cfg.cstride : s->cfg.stride;
        const int64_t nrows = k ? s->crows : s->rows;
        const int64_t r0 = p->rows_up == 0 ? 0 : margin + (int64_t)p->rows_up * rh;
        const int64_t r1 = rows_final == s->cfg.ctu_rows ? nrows : margin + (int64_t)rows_final * rh;
        const size_t off = (size_t)(r0 * stride) * s->pix, bytes = (size_t)((r1 - r0) * stride) * s->pix;
        const size_t plane = k == 0 ? 0 : (size_t)(s->cfg.plane_elems + (k - 1) * s->cfg.cplane_elems) * s->pix;
        hipError_t e;
        if (st)
            e = hipMemcpyAsync(dst + plane + off, (const uint8_t*)planes[k] + off, bytes, hipMemcpyHostToDevice, st);
        else if (guard_copies())
        {
            DevSyncScope quiet;                // (a synchronous copy may wait for running kernels)
            e = hipMemcpy(dst + plane + off, (const uint8_t*)planes[k] + off, bytes, hipMemcpyHostToDevice);
        }
        else
            e = hipMemcpy(dst + plane + off, (const uint8_t*)planes[k] + off, bytes, hipMemcpyHostToDevice);
        if (e != hipSuccess) return (int)e;
        *total += bytes;
    }
    return 0;
}

int start_service(x265amd_mes* s)
{
    const int n = s->cfg.launchers;
    if (const char* e = getenv("X265AMD_MES_SPIN_US")) s->spin_us = atoi(e);
    if (const char* e = getenv("X265AMD_MES_YIELD_US")) s->yield_us = atoi(e);
    if (const char* e = getenv("X265AMD_MES_IDLE_US")) s->idle_us = atoi(e);
    if (const char* e = getenv("X265AMD_MES_BATCH_US")) s->batch_us = atoi(e);
    if (const char* e = getenv("X265AMD_MES_BATCH_MIN")) s->batch_min = atoi(e);
    if (const char* e = getenv("X265AMD_MES_SYNC_UPLOAD")) s->sync_upload = atoi(e) != 0;
    if (const char* e = getenv("X265AMD_MES_TRACE")) s->trace = atoi(e);
    if (const char* e = getenv("X265AMD_MES_ZEROCOPY")) s->zerocopy = atoi(e);
    if (const char* e = getenv("X265AMD_MES_PRIORITY")) s->prio = atoi(e) != 0;
    if (const char* e = getenv("X265AMD_MES_LSPIN")) s->lspin = atoi(e) != 0;
    if (const char* e = getenv("X265AMD_MES_LUPLOAD")) s->lupload = atoi(e) != 0;
    if (const char* e = getenv("X265AMD_MES_WSTREAM")) s->wstream = atoi(e) != 0;
    for (int i = 0; i < n; i++)
    {
        auto* L = new (std::nothrow) x265amd_mes_launcher();
        if (!L) return X265AMD_ENOMEM;
        s->launchers.push_back(L);
        int lo = 0, hi = 0;
        if (s->prio) (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
        if ((s->prio ? hipStreamCreateWithPriority(&L->st, hipStreamNonBlocking, hi)
                     : hipStreamCreateWithFlags(&L->st, hipStreamNonBlocking)) != hipSuccess ||
            hipEventCreateWithFlags(&L->done, hipEventBlockingSync | hipEventDisableTiming) != hipSuccess ||
            hipEventCreate(&L->k0) != hipSuccess || hipEventCreate(&L->k1) != hipSuccess ||
            reserve(L->st, nullptr, L->g, 1 << 20))
            return X265AMD_ENOMEM;
    }
    for (auto* L : s->launchers)
    {
        try
        {
            L->th = std::thread(launcher_main, s, L);
        }
        catch (...)
        {
            return X265AMD_ENOMEM;
        }
    }
    return 0;
}

void stop_service(x265amd_mes* s)
{
    {
        std::lock_guard<std::mutex> g(s->qmu);
        s->stop = true;
        s->stop_flag.store(true, std::memory_order_release);
    }
    s->qcv.notify_all();
    for (auto* L : s->launchers)
    {
        if (L->th.joinable()) L->th.join();
        if (L->st) (void)hipStreamSynchronize(L->st);
        (void)hipFree(L->g.dev);
        (void)hipHostFree(L->g.host);
        if (L->vin) (void)hipFree(L->vin);
        if (L->st) (void)hipStreamDestroy(L->st);
        for (hipEvent_t e : { L->done, L->k0, L->k1 })
            if (e) (void)hipEventDestroy(e);
        delete L;
    }
    s->launchers.clear();
}

} // namespace

extern "C" int x265amd_mes_create(const x265amd_mes_config* cfg, x265amd_mes** out)
{
    if (!cfg || !out) return X265AMD_EINVAL;
    *out = nullptr;
    if ((cfg->depth != 8 && cfg->depth != 10 && cfg->depth != 12) || cfg->stride <= 0 || cfg->plane_elems <= 0 ||
        cfg->plane_elems % cfg->stride || cfg->org_offset < 0 || cfg->org_offset >= cfg->plane_elems ||
        cfg->margin_y < 0 || cfg->ctu_rows <= 0 || cfg->ctu_size <= 0 || cfg->max_pictures <= 0 ||
        cfg->max_threads <= 0 || cfg->max_tables <= 0 || cfg->mvcost_range <= 0 || cfg->method < 0 ||
        cfg->method > 4 || cfg->subme < 0 || cfg->subme > 7 || cfg->merange < 1 || cfg->max_cand < 0 ||
        cfg->max_cand > 16 || cfg->device < 0 || cfg->launchers < 0 || cfg->launchers > 8 || cfg->chroma < 0 ||
        cfg->chroma > 1 ||
        (cfg->chroma && (cfg->cstride <= 0 || cfg->cplane_elems <= 0 || cfg->cplane_elems % cfg->cstride ||
                         cfg->corg_offset < 0 || cfg->corg_offset >= cfg->cplane_elems || cfg->cmargin_y < 0 ||
                         (int64_t)cfg->cmargin_y * 2 + (int64_t)cfg->ctu_rows * cfg->ctu_size / 2 >
                             cfg->cplane_elems / cfg->cstride)) ||
        (int64_t)cfg->margin_y * 2 + (int64_t)cfg->ctu_rows * cfg->ctu_size > cfg->plane_elems / cfg->stride)
        return X265AMD_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || cfg->device >= ndev) return X265AMD_EINVAL;
    auto* s = new (std::nothrow) x265amd_mes();
    if (!s) return record(X265AMD_ENOMEM);
    s->cfg = *cfg;
    s->id = g_next_id.fetch_add(1);
    s->pix = cfg->depth > 8 ? 2 : 1;
    s->rows = cfg->plane_elems / cfg->stride;
    s->plane_bytes = (size_t)cfg->plane_elems * s->pix;
    s->slot_elems = cfg->plane_elems + (cfg->chroma ? 2 * cfg->cplane_elems : 0);
    s->crows = cfg->chroma ? cfg->cplane_elems / cfg->cstride : 0;
    s->table_elems = 2 * (size_t)cfg->mvcost_range + 1;
    int rc = use_device(s);
    if (!rc && (hipMalloc((void**)&s->arena, (size_t)s->slot_elems * s->pix * cfg->max_pictures) != hipSuccess ||
                hipMalloc((void**)&s->tables, sizeof(uint16_t) * s->table_elems * cfg->max_tables) != hipSuccess))
        rc = X265AMD_ENOMEM;
    if (!rc) s->slot_pic.assign((size_t)cfg->max_pictures, nullptr);
    if (!rc && cfg->launchers) rc = start_service(s);
    if (rc)
    {
        x265amd_mes_destroy(s);
        return record(rc);
    }
    *out = s;
    return 0;
}

extern "C" void x265amd_mes_destroy(x265amd_mes* s)
{
    if (!s) return;
    DevSyncScope quiet;                        // (the frees wait for running kernels)
    (void)use_device(s);
    stop_service(s);
    for (auto* t : s->threads) free_thread(t);
    for (auto& p : s->pics)
    {
        if (p.second->up_ev)
        {
            (void)hipEventSynchronize(p.second->up_ev);      // no copy from a pinned plane in flight
            (void)hipEventDestroy(p.second->up_ev);
        }
        for (int k = 0; k < 3; k++)
            x265amd_hostreg::unregister(p.second->pinned[k],
                                        (size_t)(k ? s->cfg.cplane_elems : s->cfg.plane_elems) * s->pix);
        delete p.second;
    }
    (void)hipFree(s->arena);
    (void)hipFree(s->tables);
    delete s;
}

extern "C" int x265amd_mes_ref420(x265amd_mes* s, const void* key, int64_t gen, const void* const planes[3],
                                  int rows_final, int* slot)
{
    if (!s || !key || !planes || !planes[0] || !slot || rows_final < 0 || rows_final > s->cfg.ctu_rows ||
        (s->cfg.chroma && (!planes[1] || !planes[2])))
        return record(X265AMD_EINVAL);
    // the common call (every CU asks for each of its references): a known picture whose rows are all
    // resident (or recorded, with launcher uploads) — no HIP call, one map lookup and the picture's lock
    {
        x265amd_mes::Picture* q = nullptr;
        {
            std::lock_guard<std::mutex> g(s->mu);
            auto it = s->pics.find(key);
            if (it != s->pics.end()) q = it->second;
        }
        if (q)
        {
            std::lock_guard<std::mutex> g(q->mu);
            const int np = s->cfg.chroma ? 3 : 1;
            bool same = q->gen == gen && rows_final <= (s->lupload ? q->rows_want : q->rows_up);
            for (int k = 0; k < np && same; k++) same = q->pinned[k] == planes[k];
            if (same)
            {
                *slot = q->slot;
                return 0;
            }
        }
    }
    MES_TRY(use_device(s));
    x265amd_mes_thread* t;
    if (int rc = thread_ctx(s, &t)) return rc;
    x265amd_mes::Picture* p;
    {
        std::lock_guard<std::mutex> g(s->mu);
        auto it = s->pics.find(key);
        if (it == s->pics.end())
        {
            // a slot per reconstructed-picture buffer: x265 reuses a Frame's PicYuv for later pictures
            // (new generation = POC) only after no frame encoder references the old one any more
            if (s->next_slot >= s->cfg.max_pictures) return X265AMD_ENOMEM;   // caller searches on the host
            p = new (std::nothrow) x265amd_mes::Picture();
            if (!p) return record(X265AMD_ENOMEM);
            p->slot = s->next_slot++;
            s->slot_pic[p->slot] = p;
            p->gen = gen;
            p->rows_up = 0;
            p->pinned[0] = p->pinned[1] = p->pinned[2] = nullptr;
            it = s->pics.emplace(key, p).first;
        }
        p = it->second;
    }
    std::lock_guard<std::mutex> g(p->mu);
    if (p->gen != gen)
    {
        p->gen = gen;
        p->rows_up = 0;
        p->rows_want = 0;
    }
    const int np = s->cfg.chroma ? 3 : 1;
    for (int k = 0; k < np; k++)
        if (p->pinned[k] != planes[k])
        {
            const size_t bytes = (size_t)(k ? s->cfg.cplane_elems : s->cfg.plane_elems) * s->pix;
            x265amd_hostreg::unregister(p->pinned[k], bytes);
            DevSyncScope quiet;                  // (hipHostRegister waits for every running kernel)
            p->pinned[k] = hipHostRegister((void*)planes[k], bytes, hipHostRegisterDefault) == hipSuccess ? planes[k]
                                                                                                        : nullptr;
            (void)hipGetLastError();
        }
    if (s->lupload)
    {
        for (int k = 0; k < np; k++) p->planes[k] = planes[k];
        if (rows_final > p->rows_want) p->rows_want = rows_final;
    }
    else if (rows_final > p->rows_up)
    {
        const double t0 = now_s();
        size_t total = 0;
        const bool async = !s->launchers.empty() && !s->sync_upload;
        if (async)
        {
            if (!p->up_ev) MES_TRY(hipEventCreateWithFlags(&p->up_ev, hipEventDisableTiming));
            if (p->up_any) MES_TRY(hipStreamWaitEvent(t->st, p->up_ev, 0));
        }
        MES_TRY(copy_rows(s, p, planes, rows_final, t->st, &total));
        if (async)
        {
            MES_TRY(hipEventRecord(p->up_ev, t->st));
            p->up_any = true;
        }
        else if (t->st)
            MES_TRY(wait(t));
        p->rows_up = rows_final;
        std::lock_guard<std::mutex> sg(s->smu);
        s->st.uploads++;
        s->st.upload_bytes += (int64_t)total;
        s->st.upload_ms += 1e3 * (now_s() - t0);
    }
    *slot = p->slot;
    return 0;
}

extern "C" int x265amd_mes_ref(x265amd_mes* s, const void* key, int64_t gen, const void* plane_buf, int rows_final,
                               int* slot)
{
    if (s && s->cfg.chroma) return record(X265AMD_EINVAL);      // a chroma session needs the chroma planes
    const void* planes[3] = { plane_buf, nullptr, nullptr };
    return x265amd_mes_ref420(s, key, gen, planes, rows_final, slot);
}

extern "C" int x265amd_mes_rows(x265amd_mes* s, const void* key, int64_t gen, int* rows_resident)
{
    if (!s || !key || !rows_resident) return record(X265AMD_EINVAL);
    *rows_resident = 0;
    x265amd_mes::Picture* p = nullptr;
    {
        std::lock_guard<std::mutex> g(s->mu);
        auto it = s->pics.find(key);
        if (it != s->pics.end()) p = it->second;
    }
    if (!p) return 0;
    std::lock_guard<std::mutex> g(p->mu);
    // launcher uploads: the rows recorded are copied ahead of every launch that can read them
    *rows_resident = p->gen == gen ? (s->lupload ? p->rows_want : p->rows_up) : 0;
    return 0;
}

extern "C" int x265amd_mes_table(x265amd_mes* s, const uint16_t* centre, int* index)
{
    if (!s || !centre || !index) return record(X265AMD_EINVAL);
    {
        // a table already resident (every CU asks): no HIP call
        std::lock_guard<std::mutex> g(s->mu);
        auto it = s->tabs.find(centre);
        if (it != s->tabs.end())
        {
            *index = it->second;
            return 0;
        }
    }
    MES_TRY(use_device(s));
    x265amd_mes_thread* t;
    if (int rc = thread_ctx(s, &t)) return rc;
    std::lock_guard<std::mutex> g(s->mu);
    auto it = s->tabs.find(centre);
    if (it != s->tabs.end())
    {
        *index = it->second;
        return 0;
    }
    const int k = (int)s->tabs.size();
    if (k >= s->cfg.max_tables) return X265AMD_ENOMEM;
    // the BitCost tables are process-wide and never change once built (bitcost.cpp:31-57)
    if (t->st)
    {
        MES_TRY(hipMemcpyAsync(s->tables + (size_t)k * s->table_elems, centre - s->cfg.mvcost_range,
                               sizeof(uint16_t) * s->table_elems, hipMemcpyHostToDevice, t->st));
        MES_TRY(wait(t));
    }
    else
    {
        DevSyncScope quiet;                    // (a synchronous copy waits for running kernels)
        MES_TRY(hipMemcpy(s->tables + (size_t)k * s->table_elems, centre - s->cfg.mvcost_range,
                          sizeof(uint16_t) * s->table_elems, hipMemcpyHostToDevice));
    }
    s->tabs.emplace(centre, k);
    *index = k;
    return 0;
}

// ---------------------------------------------------------------- service entries
extern "C" int x265amd_mes_post420(x265amd_mes* s, int w, int h, const void* fenc, intptr_t fenc_stride,
                                   const void* fenc_cb, const void* fenc_cr, intptr_t fenc_cstride, int n,
                                   const x265amd_mes_job* jobs, int* ticket)
{
    if (!s || !ticket) return record(X265AMD_EINVAL);
    *ticket = -1;
    if (s->launchers.empty() || n <= 0 || (fenc_cb && (!fenc_cr || !s->cfg.chroma || fenc_cstride < w / 2)))
        return record(X265AMD_EINVAL);
    if (n > kMaxJobs) return X265AMD_ENOMEM;               // more than a slot holds: search on the host
    MES_TRY(check_jobs(s, w, h, fenc, fenc_stride, n, jobs));
    x265amd_mes_thread* t;
    if (int rc = thread_ctx(s, &t)) return rc;
    int k = -1;
    for (int i = 0; i < kSlots && k < 0; i++)
    {
        const int stt = t->req[i].state.load(std::memory_order_acquire);
        if (stt == 0 || (stt == 2 && t->req[i].dropped)) k = i;
    }
    if (k < 0) return X265AMD_ENOMEM;                     // every slot outstanding: search on the host
    x265amd_mes_req& r = t->req[k];
    r.w = w;
    r.h = h;
    r.n = n;
    r.chroma = fenc_cb != nullptr;
    r.dropped = false;
    r.rc = 0;
    for (int y = 0; y < h; y++)
        memcpy(r.fenc + (size_t)y * w * s->pix, (const uint8_t*)fenc + (size_t)y * fenc_stride * s->pix, (size_t)w * s->pix);
    if (r.chroma)
    {
        // Cb then Cr blocks, packed at stride w / 2, after the luma block
        const int cw = w / 2, ch = h / 2;
        uint8_t* c = r.fenc + (size_t)w * h * s->pix;
        for (int q = 0; q < 2; q++)
            for (int y = 0; y < ch; y++)
                memcpy(c + ((size_t)q * cw * ch + (size_t)y * cw) * s->pix,
                       (const uint8_t*)(q ? fenc_cr : fenc_cb) + (size_t)y * fenc_cstride * s->pix, (size_t)cw * s->pix);
    }
    memcpy(r.jobs, jobs, sizeof(x265amd_mes_job) * n);
    r.t_post = now_s();
    r.state.store(1, std::memory_order_relaxed);
    {
        std::lock_guard<std::mutex> g(s->qmu);
        s->rq.push_back(&r);
    }
    s->queued.fetch_add(1, std::memory_order_acq_rel);
    if (s->qsleepers.load(std::memory_order_acquire) > 0)
        s->qcv.notify_one();
    *ticket = k;
    if (s->trace && s->traced.fetch_add(1) < s->trace)
        fprintf(stderr, "[mes] post %dx%d n %d chroma %d ticket %d\n", w, h, n, (int)r.chroma, k);
    return 0;
}

extern "C" int x265amd_mes_post(x265amd_mes* s, int w, int h, const void* fenc, intptr_t fenc_stride, int n,
                                const x265amd_mes_job* jobs, int* ticket)
{
    return x265amd_mes_post420(s, w, h, fenc, fenc_stride, nullptr, nullptr, 0, n, jobs, ticket);
}

extern "C" int x265amd_mes_wait(x265amd_mes* s, int ticket, int n, x265amd_mes_job* jobs)
{
    if (!s || ticket < 0 || ticket >= kSlots || n < 0 || (n && !jobs)) return record(X265AMD_EINVAL);
    x265amd_mes_thread* t;
    MES_TRY(thread_ctx(s, &t));
    x265amd_mes_req& r = t->req[ticket];
    if (r.state.load(std::memory_order_acquire) == 0 || r.dropped || r.n != n) return record(X265AMD_EINVAL);
    const double t0 = now_s();
    bool slept = false;
    if (r.state.load(std::memory_order_acquire) != 2)
    {
        // spin briefly (a batch ends within tens of microseconds of its neighbours), then sleep
        const double until = t0 + 1e-6 * s->spin_us;
        while (r.state.load(std::memory_order_acquire) != 2 && now_s() < until)
            __builtin_ia32_pause();
        const double yuntil = t0 + 1e-6 * (s->spin_us + s->yield_us);
        while (r.state.load(std::memory_order_acquire) != 2 && now_s() < yuntil)
            sched_yield();
        if (r.state.load(std::memory_order_acquire) != 2)
        {
            slept = true;
            std::unique_lock<std::mutex> lk(s->dmu);
            s->dsleepers++;
            s->dcv.wait(lk, [&] { return r.state.load(std::memory_order_acquire) == 2; });
            s->dsleepers--;
        }
    }
    const double dt = now_s() - t0;
    if (s->trace && s->traced.fetch_add(1) < s->trace)
        fprintf(stderr, "[mes] wait ticket %d: %.3f ms%s\n", ticket, 1e3 * dt, slept ? " (slept)" : "");
    for (int i = 0; i < n; i++)
    {
        jobs[i].out_mv[0] = r.jobs[i].out_mv[0];
        jobs[i].out_mv[1] = r.jobs[i].out_mv[1];
        jobs[i].out_cost = r.jobs[i].out_cost;
    }
    const int rc = r.rc;
    r.state.store(0, std::memory_order_release);
    {
        std::lock_guard<std::mutex> g(s->smu);
        s->st.waits++;
        s->st.wait_ms += 1e3 * dt;
        const int b = hist_bin(1e3 * dt);
        s->st.wait_hist[b]++;
        s->st.wait_hist_ms[b] += 1e3 * dt;
        s->st.waits_blocked += slept;
    }
    return rc ? record(rc) : 0;
}

extern "C" int x265amd_mes_drop(x265amd_mes* s, int ticket)
{
    if (!s || ticket < 0 || ticket >= kSlots) return record(X265AMD_EINVAL);
    x265amd_mes_thread* t;
    MES_TRY(thread_ctx(s, &t));
    x265amd_mes_req& r = t->req[ticket];
    if (r.state.load(std::memory_order_acquire) == 0) return 0;
    r.dropped = true;                                      // the slot is reused once the launcher is done
    std::lock_guard<std::mutex> g(s->smu);
    s->st.dropped++;
    return 0;
}

extern "C" long long x265amd_host_unregister_stale(void)
{
    return x265amd_hostreg::stale_count().load();
}

extern "C" int x265amd_mes_stats(x265amd_mes* s, x265amd_mes_counters* out)
{
    if (!s || !out) return X265AMD_EINVAL;
    std::lock_guard<std::mutex> g(s->smu);
    *out = s->st;
    return 0;
}

// ---------------------------------------------------------------- legacy (per-thread) form
namespace {

// stage a batch of one PU's searches in g and enqueue upload, launch and download on the thread's
// stream; *out = the outputs' offset in g.host
int enqueue(x265amd_mes* s, x265amd_mes_thread* t, x265amd_mes_stage& g, hipStream_t st, int w, int h,
            const void* fenc, intptr_t fenc_stride, int n, const x265amd_mes_job* jobs, size_t* out)
{
    if (int rc = check_jobs(s, w, h, fenc, fenc_stride, n, jobs)) return rc;
    const int maxc = s->cfg.max_cand > 0 ? s->cfg.max_cand : 1;
    const Layout L(n, h, (int)s->pix, maxc, fenc_stride);
    if (int rc = reserve(t->st, t->ast, g, L.end)) return rc;
    uint8_t* H = g.host;
    memcpy(H + L.fenc, fenc, (size_t)fenc_stride * h * s->pix);
    for (int i = 0; i < n; i++) stage_job(s, H, L, i, jobs[i], 0);
    if (hipError_t e = hipMemcpyAsync(g.dev, H, L.out_mv, hipMemcpyHostToDevice, st)) return (int)e;
    const x265amd_me_batch b = make_batch(s, g, L, w, h, n, fenc_stride);
    if (int rc = x265amd_motion_search(s->cfg.depth, 1, &b, st)) return rc;
    if (hipError_t e = hipMemcpyAsync(H + L.out_mv, g.dev + L.out_mv, L.end - L.out_mv, hipMemcpyDeviceToHost, st))
        return (int)e;
    *out = L.out_mv;
    return 0;
}

void unpack(const x265amd_mes_stage& g, size_t out, int n, x265amd_mes_job* jobs)
{
    const int16_t* om = (const int16_t*)(g.host + out);
    const int32_t* oc = (const int32_t*)(g.host + out + (((size_t)4 * n + 255) & ~(size_t)255));
    for (int i = 0; i < n; i++)
    {
        jobs[i].out_mv[0] = om[2 * i];
        jobs[i].out_mv[1] = om[2 * i + 1];
        jobs[i].out_cost = oc[i];
    }
}

bool coalescing()
{
    static int v = -1;
    if (v < 0)
    {
        const char* e = getenv("X265AMD_MES_COALESCE");
        v = e ? atoi(e) != 0 : 0;
    }
    return v != 0;
}

// stage the searches of several PUs of one size (requests checked by check_jobs) in g — their source
// blocks packed at stride w, one after another, jobs in request order — and enqueue upload, launch and
// download on `st`; *out = the outputs' offset in g.host
int enqueue_requests(x265amd_mes* s, x265amd_mes_thread* t, x265amd_mes_stage& g, hipStream_t st, int w, int h,
                     const std::vector<x265amd_mes::Request*>& reqs, size_t* out)
{
    const int maxc = s->cfg.max_cand > 0 ? s->cfg.max_cand : 1;
    const int np = (int)reqs.size();
    int n = 0;
    for (auto* r : reqs) n += r->n;
    const size_t blk = (size_t)w * h;                         // elements per packed source block
    const Layout L(n, np * h, (int)s->pix, maxc, w);
    if (int rc = reserve(t->st, t->ast, g, L.end)) return rc;
    uint8_t* H = g.host;
    int i = 0;
    for (int k = 0; k < np; k++)
    {
        const x265amd_mes::Request& r = *reqs[k];
        for (int y = 0; y < h; y++)
            memcpy(H + L.fenc + (k * blk + (size_t)y * w) * s->pix,
                   (const uint8_t*)r.fenc + (size_t)y * r.fenc_stride * s->pix, (size_t)w * s->pix);
        for (int q = 0; q < r.n; q++, i++) stage_job(s, H, L, i, r.jobs[q], (int64_t)(k * blk));
    }
    if (hipError_t e = hipMemcpyAsync(g.dev, H, L.out_mv, hipMemcpyHostToDevice, st)) return (int)e;
    const x265amd_me_batch b = make_batch(s, g, L, w, h, n, w);
    if (int rc = x265amd_motion_search(s->cfg.depth, 1, &b, st)) return rc;
    if (hipError_t e = hipMemcpyAsync(H + L.out_mv, g.dev + L.out_mv, L.end - L.out_mv, hipMemcpyDeviceToHost, st))
        return (int)e;
    *out = L.out_mv;
    return 0;
}

// lead one coalesced batch: every queued request of the first request's PU size (s->cmu held on entry
// and on return, released while the device works)
void lead_batch(x265amd_mes* s, x265amd_mes_thread* t, std::unique_lock<std::mutex>& lk)
{
    std::vector<x265amd_mes::Request*> batch;
    const int w = s->queue[0]->w, h = s->queue[0]->h;
    size_t keep = 0;
    for (size_t i = 0; i < s->queue.size(); i++)
    {
        x265amd_mes::Request* r = s->queue[i];
        if (r->w == w && r->h == h) batch.push_back(r);
        else s->queue[keep++] = r;
    }
    s->queue.resize(keep);
    s->busy = true;
    lk.unlock();
    size_t out = 0;
    int rc = enqueue_requests(s, t, t->sync, t->st, w, h, batch, &out);
    if (!rc) rc = wait(t);
    if (!rc)
    {
        int n = 0;
        for (auto* r : batch) n += r->n;
        const int16_t* om = (const int16_t*)(t->sync.host + out);
        const int32_t* oc = (const int32_t*)(t->sync.host + out + (((size_t)4 * n + 255) & ~(size_t)255));
        for (size_t k = 0, i = 0; k < batch.size(); k++)
            for (int q = 0; q < batch[k]->n; q++, i++)
            {
                batch[k]->jobs[q].out_mv[0] = om[2 * i];
                batch[k]->jobs[q].out_mv[1] = om[2 * i + 1];
                batch[k]->jobs[q].out_cost = oc[i];
            }
    }
    lk.lock();
    for (auto* r : batch)
    {
        r->rc = rc;
        r->done = true;
    }
    s->busy = false;
    s->ccv.notify_all();
}

} // namespace

extern "C" int x265amd_mes_search(x265amd_mes* s, int w, int h, const void* fenc, intptr_t fenc_stride, int n,
                                  x265amd_mes_job* jobs)
{
    if (!s) return record(X265AMD_EINVAL);
    if (!n) return 0;
    if (!s->launchers.empty())
    {
        // the service form: post and wait (the searches share a launch with whatever else is queued)
        int ticket = -1;
        if (int rc = x265amd_mes_post(s, w, h, fenc, fenc_stride, n, jobs, &ticket)) return rc;
        return x265amd_mes_wait(s, ticket, n, jobs);
    }
    MES_TRY(use_device(s));
    x265amd_mes_thread* t;
    if (int rc = thread_ctx(s, &t)) return rc;
    if (coalescing())
    {
        MES_TRY(check_jobs(s, w, h, fenc, fenc_stride, n, jobs));
        x265amd_mes::Request r = { w, h, fenc, fenc_stride, n, jobs, 0, false };
        std::unique_lock<std::mutex> lk(s->cmu);
        s->queue.push_back(&r);
        while (!r.done)
        {
            if (!s->busy) lead_batch(s, t, lk);
            else s->ccv.wait(lk);
        }
        return record(r.rc);
    }
    size_t out = 0;
    MES_TRY(enqueue(s, t, t->sync, t->st, w, h, fenc, fenc_stride, n, jobs, &out));
    MES_TRY(wait(t));
    unpack(t->sync, out, n, jobs);
    return 0;
}

extern "C" int x265amd_mes_submit(x265amd_mes* s, int w, int h, const void* fenc, intptr_t fenc_stride, int n,
                                  const x265amd_mes_job* jobs)
{
    if (!s || n <= 0) return record(X265AMD_EINVAL);
    if (!s->launchers.empty())
    {
        x265amd_mes_thread* t;
        if (int rc = thread_ctx(s, &t)) return rc;
        if (t->pend_ticket >= 0) return record(X265AMD_EINVAL);   // one outstanding submit per thread
        int ticket = -1;
        if (int rc = x265amd_mes_post(s, w, h, fenc, fenc_stride, n, jobs, &ticket)) return rc;
        t->pend_ticket = ticket;
        t->pending = n;
        return 0;
    }
    MES_TRY(use_device(s));
    x265amd_mes_thread* t;
    if (int rc = thread_ctx(s, &t)) return rc;
    if (t->pending) return record(X265AMD_EINVAL);          // one outstanding submit per thread
    size_t out = 0;
    MES_TRY(enqueue(s, t, t->async, t->ast, w, h, fenc, fenc_stride, n, jobs, &out));
    MES_TRY(hipEventRecord(t->aev, t->ast));
    t->pending = n;
    t->pend_out = out;
    return 0;
}

extern "C" int x265amd_mes_collect(x265amd_mes* s, int n, x265amd_mes_job* jobs)
{
    if (!s || n < 0 || (n && !jobs)) return record(X265AMD_EINVAL);
    x265amd_mes_thread* t;
    MES_TRY(thread_ctx(s, &t));
    if (!t->pending) return record(X265AMD_EINVAL);
    const int pend = t->pending;
    t->pending = 0;
    if (!s->launchers.empty())
    {
        const int ticket = t->pend_ticket;
        t->pend_ticket = -1;
        if (n != pend)
        {
            (void)x265amd_mes_drop(s, ticket);
            return record(X265AMD_EINVAL);
        }
        return x265amd_mes_wait(s, ticket, n, jobs);
    }
    MES_TRY(hipEventSynchronize(t->aev));
    if (n != pend) return record(X265AMD_EINVAL);
    unpack(t->async, t->pend_out, n, jobs);
    return 0;
}
