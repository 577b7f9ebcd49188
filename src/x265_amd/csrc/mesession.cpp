// mesession.cpp — f2 encoder session: the main encoder's motion searches on the MI355X
// (include/x265_amd.h, x265amd_mes_*).
//
// Search::predInterSearch (search.cpp:2050-2231) runs one MotionEstimate::motionEstimate per
// (list, reference) of a PU, one after another on a worker thread; the searches of one PU are
// independent given their predictors.  A session turns them into one batched launch of the f2
// kernel (x265amd_motion_search, csrc/me.hip) per PU:
//   * reference pictures: the padded luma plane of each reconstructed reference PicYuv
//     (picyuv.cpp:51-91) in one device arena, uploaded CTU row by CTU row as the encoder
//     publishes them (Frame::m_reconRowCount, framefilter.cpp:520: rows below the count are
//     deblocked, SAO-filtered and border-extended, so they never change again) — each row once,
//     whichever thread needs it first;
//   * MV cost tables: the encoder's BitCost table of each QP (bitcost.cpp:31-57) uploaded once;
//   * per host thread: a non-blocking stream, pinned staging and device scratch for one batch
//     (the PU's source block and the job descriptors), found by (session address, session id).
// x265amd_mes_search is synchronous on the calling thread: outputs are in the jobs on return.
// Coalescing (X265AMD_MES_COALESCE=1; built in round 4, off by default until it has run on the box):
// the searches of all threads that call while a launch is in flight are queued, and whichever waiting
// thread finds the device idle launches every queued request of one PU size as ONE batch on its stream
// and hands each caller its outputs.
// Failures are returned AND recorded in the backend's sticky status (x265amd_provider_status).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <new>
#include <unordered_map>
#include <vector>

#include "../../../include/x265_amd.h"

namespace x265amd_provider {
extern std::atomic<int> g_status;
}

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

} // namespace

struct x265amd_mes_stage
{
    uint8_t* dev = nullptr;
    uint8_t* host = nullptr;
    size_t cap = 0;
};

struct x265amd_mes_thread
{
    hipStream_t st = nullptr;
    hipStream_t ast = nullptr;  // the outstanding x265amd_mes_submit's stream (never waited on by _search / _ref)
    hipEvent_t ev = nullptr;    // blocking-sync event: the waiting worker sleeps (X265AMD_MES_SYNC=spin: spin)
    hipEvent_t aev = nullptr;   // completion of the outstanding x265amd_mes_submit
    x265amd_mes_stage sync, async;
    int pending = 0;            // jobs of the outstanding submit (0: none)
    size_t pend_out = 0;        // its output offset in the async staging
};

struct x265amd_mes
{
    x265amd_mes_config cfg;
    uint64_t id = 0;
    size_t pix = 1;
    int64_t rows = 0;                 // plane rows incl. both margins
    size_t plane_bytes = 0;
    uint8_t* arena = nullptr;         // max_pictures padded luma planes
    uint16_t* tables = nullptr;       // max_tables BitCost tables of 2 * range + 1 entries
    size_t table_elems = 0;

    struct Picture
    {
        int slot;
        int64_t gen;
        int rows_up;                  // CTU rows resident on the device
        const void* pinned;           // host buffer registered with hipHostRegister (or null)
        std::mutex mu;                // one uploader at a time; the others wait for its rows
    };
    std::mutex mu;
    std::unordered_map<const void*, Picture*> pics;
    std::unordered_map<const void*, int> tabs;
    std::vector<x265amd_mes_thread*> threads;
    std::atomic<int> next_slot{ 0 };

    // coalesced x265amd_mes_search requests (one per calling thread at a time)
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
};

namespace {

struct TlsEntry { const x265amd_mes* s; uint64_t id; x265amd_mes_thread* t; };
thread_local std::vector<TlsEntry> tls;
std::atomic<uint64_t> g_next_id{ 1 };

int wait(x265amd_mes_thread* t)
{
    if (t->ev)
    {
        const hipError_t e = hipEventRecord(t->ev, t->st);
        return e != hipSuccess ? (int)e : (int)hipEventSynchronize(t->ev);
    }
    return (int)hipStreamSynchronize(t->st);
}

int reserve(x265amd_mes_thread* t, x265amd_mes_stage& g, size_t bytes)
{
    if (bytes <= g.cap) return 0;
    bytes = (bytes + 65535) & ~(size_t)65535;
    if (t->st) (void)hipStreamSynchronize(t->st);
    if (t->ast) (void)hipStreamSynchronize(t->ast);
    (void)hipFree(g.dev);
    (void)hipHostFree(g.host);
    g.dev = g.host = nullptr;
    g.cap = 0;
    if (hipMalloc((void**)&g.dev, bytes) != hipSuccess ||
        hipHostMalloc((void**)&g.host, bytes, hipHostMallocDefault) != hipSuccess)
        return X265AMD_ENOMEM;
    g.cap = bytes;
    return 0;
}

int thread_ctx(x265amd_mes* s, x265amd_mes_thread** out)
{
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
    auto* t = new (std::nothrow) x265amd_mes_thread();
    if (!t) return X265AMD_ENOMEM;
    {
        std::lock_guard<std::mutex> g(s->mu);
        if ((int)s->threads.size() >= s->cfg.max_threads)
        {
            delete t;
            return X265AMD_ENOMEM;
        }
        s->threads.push_back(t);
    }
    if (hipStreamCreateWithFlags(&t->st, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&t->ast, hipStreamNonBlocking) != hipSuccess || reserve(t, t->sync, 1 << 16) ||
        reserve(t, t->async, 1 << 16))
        return X265AMD_ENOMEM;
    const char* sync = getenv("X265AMD_MES_SYNC");
    const bool spin = sync && !strcmp(sync, "spin");
    if ((!spin && hipEventCreateWithFlags(&t->ev, hipEventBlockingSync | hipEventDisableTiming) != hipSuccess) ||
        hipEventCreateWithFlags(&t->aev, (spin ? 0 : hipEventBlockingSync) | hipEventDisableTiming) != hipSuccess)
        return X265AMD_ENOMEM;
    tls.push_back({ s, s->id, t });
    *out = t;
    return 0;
}

// batch layout in the staging buffers (byte offsets, 256-aligned)
struct Layout
{
    size_t fenc, fenc_off, ref_off, range, mvp, mvc, ncand, cost_off, out_mv, out_cost, end;
    Layout(int n, int h, int pix, int maxc, intptr_t fstride)
    {
        size_t o = 0;
        auto take = [&](size_t b) { size_t r = o; o = (o + b + 255) & ~(size_t)255; return r; };
        fenc = take((size_t)fstride * h * pix);
        fenc_off = take(8 * (size_t)n);
        ref_off = take(8 * (size_t)n);
        range = take(8 * (size_t)n);
        mvp = take(4 * (size_t)n);
        mvc = take(4 * (size_t)maxc * n);
        ncand = take((size_t)n);
        cost_off = take(8 * (size_t)n);
        out_mv = take(4 * (size_t)n);
        out_cost = take(4 * (size_t)n);
        end = o;
    }
};

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
        cfg->max_cand > 16 || (int64_t)cfg->margin_y * 2 + (int64_t)cfg->ctu_rows * cfg->ctu_size >
                                  cfg->plane_elems / cfg->stride)
        return X265AMD_EINVAL;
    auto* s = new (std::nothrow) x265amd_mes();
    if (!s) return record(X265AMD_ENOMEM);
    s->cfg = *cfg;
    s->id = g_next_id.fetch_add(1);
    s->pix = cfg->depth > 8 ? 2 : 1;
    s->rows = cfg->plane_elems / cfg->stride;
    s->plane_bytes = (size_t)cfg->plane_elems * s->pix;
    s->table_elems = 2 * (size_t)cfg->mvcost_range + 1;
    if (hipMalloc((void**)&s->arena, s->plane_bytes * cfg->max_pictures) != hipSuccess ||
        hipMalloc((void**)&s->tables, sizeof(uint16_t) * s->table_elems * cfg->max_tables) != hipSuccess)
    {
        x265amd_mes_destroy(s);
        return record(X265AMD_ENOMEM);
    }
    *out = s;
    return 0;
}

extern "C" void x265amd_mes_destroy(x265amd_mes* s)
{
    if (!s) return;
    for (auto* t : s->threads)
    {
        if (t->st) (void)hipStreamSynchronize(t->st);
        for (x265amd_mes_stage* g : { &t->sync, &t->async })
        {
            (void)hipFree(g->dev);
            (void)hipHostFree(g->host);
        }
        if (t->ast) (void)hipStreamSynchronize(t->ast);
        if (t->st) (void)hipStreamDestroy(t->st);
        if (t->ast) (void)hipStreamDestroy(t->ast);
        if (t->ev) (void)hipEventDestroy(t->ev);
        if (t->aev) (void)hipEventDestroy(t->aev);
        delete t;
    }
    for (auto& p : s->pics)
    {
        if (p.second->pinned) (void)hipHostUnregister((void*)p.second->pinned);
        delete p.second;
    }
    (void)hipFree(s->arena);
    (void)hipFree(s->tables);
    delete s;
}

extern "C" int x265amd_mes_ref(x265amd_mes* s, const void* key, int64_t gen, const void* plane_buf, int rows_final,
                               int* slot)
{
    if (!s || !key || !plane_buf || !slot || rows_final < 0 || rows_final > s->cfg.ctu_rows)
        return record(X265AMD_EINVAL);
    x265amd_mes_thread* t;
    MES_TRY(thread_ctx(s, &t));
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
            p->gen = gen;
            p->rows_up = 0;
            p->pinned = nullptr;
            it = s->pics.emplace(key, p).first;
        }
        p = it->second;
    }
    std::lock_guard<std::mutex> g(p->mu);
    if (p->gen != gen)
    {
        p->gen = gen;
        p->rows_up = 0;
    }
    if (p->pinned != plane_buf)
    {
        if (p->pinned) (void)hipHostUnregister((void*)p->pinned);
        p->pinned = hipHostRegister((void*)plane_buf, s->plane_bytes, hipHostRegisterDefault) == hipSuccess ? plane_buf
                                                                                                          : nullptr;
        (void)hipGetLastError();
    }
    if (rows_final > p->rows_up)
    {
        // plane rows of CTU rows [rows_up, rows_final): the top margin goes with row 0, the bottom
        // margin (and the rows of a partial last CTU row) with the last row
        const int64_t r0 = p->rows_up == 0 ? 0 : s->cfg.margin_y + (int64_t)p->rows_up * s->cfg.ctu_size;
        const int64_t r1 = rows_final == s->cfg.ctu_rows ? s->rows
                                                         : s->cfg.margin_y + (int64_t)rows_final * s->cfg.ctu_size;
        const size_t off = (size_t)(r0 * s->cfg.stride) * s->pix, bytes = (size_t)((r1 - r0) * s->cfg.stride) * s->pix;
        MES_TRY(hipMemcpyAsync(s->arena + (size_t)p->slot * s->plane_bytes + off, (const uint8_t*)plane_buf + off, bytes,
                               hipMemcpyHostToDevice, t->st));
        MES_TRY(wait(t));
        p->rows_up = rows_final;
    }
    *slot = p->slot;
    return 0;
}

extern "C" int x265amd_mes_table(x265amd_mes* s, const uint16_t* centre, int* index)
{
    if (!s || !centre || !index) return record(X265AMD_EINVAL);
    x265amd_mes_thread* t;
    MES_TRY(thread_ctx(s, &t));
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
    MES_TRY(hipMemcpyAsync(s->tables + (size_t)k * s->table_elems, centre - s->cfg.mvcost_range,
                           sizeof(uint16_t) * s->table_elems, hipMemcpyHostToDevice, t->st));
    MES_TRY(wait(t));
    s->tabs.emplace(centre, k);
    *index = k;
    return 0;
}

namespace {

// stage a batch of one PU's searches in g and enqueue upload, launch and download on the thread's
// stream; *out = the outputs' offset in g.host
int enqueue(x265amd_mes* s, x265amd_mes_thread* t, x265amd_mes_stage& g, hipStream_t st, int w, int h,
            const void* fenc, intptr_t fenc_stride, int n, const x265amd_mes_job* jobs, size_t* out)
{
    if (!s || n < 0 || (n && (!jobs || !fenc)) || w < 4 || h < 4 || w > 64 || h > 64 || fenc_stride < w)
        return X265AMD_EINVAL;
    const int maxc = s->cfg.max_cand > 0 ? s->cfg.max_cand : 1;
    for (int i = 0; i < n; i++)
        if (jobs[i].slot < 0 || jobs[i].slot >= s->next_slot || jobs[i].table < 0 ||
            jobs[i].table >= s->cfg.max_tables || jobs[i].num_cand < 0 || jobs[i].num_cand > s->cfg.max_cand)
            return X265AMD_EINVAL;
    const Layout L(n, h, (int)s->pix, maxc, fenc_stride);
    if (int rc = reserve(t, g, L.end)) return rc;
    uint8_t* H = g.host;
    memcpy(H + L.fenc, fenc, (size_t)fenc_stride * h * s->pix);
    int64_t* foff = (int64_t*)(H + L.fenc_off);
    int64_t* roff = (int64_t*)(H + L.ref_off);
    int16_t* rng = (int16_t*)(H + L.range);
    int16_t* mvp = (int16_t*)(H + L.mvp);
    int16_t* mvc = (int16_t*)(H + L.mvc);
    uint8_t* nc = H + L.ncand;
    int64_t* coff = (int64_t*)(H + L.cost_off);
    for (int i = 0; i < n; i++)
    {
        const x265amd_mes_job& j = jobs[i];
        foff[i] = 0;
        roff[i] = (int64_t)j.slot * s->cfg.plane_elems + s->cfg.org_offset + j.block_off;
        memcpy(rng + 4 * i, j.mv_range, 8);
        memcpy(mvp + 2 * i, j.mvp, 4);
        memcpy(mvc + 2 * (size_t)maxc * i, j.mvc, 4 * (size_t)j.num_cand);
        nc[i] = (uint8_t)j.num_cand;
        coff[i] = (int64_t)j.table * (int64_t)s->table_elems + s->cfg.mvcost_range;
    }
    if (hipError_t e = hipMemcpyAsync(g.dev, H, L.out_mv, hipMemcpyHostToDevice, st)) return (int)e;
    x265amd_me_batch b;
    memset(&b, 0, sizeof(b));
    b.w = w;
    b.h = h;
    b.n = n;
    b.method = s->cfg.method;
    b.subme = s->cfg.subme;
    b.merange = s->cfg.merange;
    b.max_cand = maxc;
    b.fenc = g.dev + L.fenc;
    b.fenc_stride = fenc_stride;
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

// ---- coalescing (X265AMD_MES_COALESCE=1)
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

int check_request(const x265amd_mes* s, int w, int h, const void* fenc, intptr_t fenc_stride, int n,
                  const x265amd_mes_job* jobs)
{
    if (!s || n < 0 || (n && (!jobs || !fenc)) || w < 4 || h < 4 || w > 64 || h > 64 || fenc_stride < w)
        return X265AMD_EINVAL;
    for (int i = 0; i < n; i++)
        if (jobs[i].slot < 0 || jobs[i].slot >= s->next_slot || jobs[i].table < 0 ||
            jobs[i].table >= s->cfg.max_tables || jobs[i].num_cand < 0 || jobs[i].num_cand > s->cfg.max_cand)
            return X265AMD_EINVAL;
    return 0;
}

// stage the searches of several PUs of one size (requests checked by check_request) in g — their source
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
    if (int rc = reserve(t, g, L.end)) return rc;
    uint8_t* H = g.host;
    int64_t* foff = (int64_t*)(H + L.fenc_off);
    int64_t* roff = (int64_t*)(H + L.ref_off);
    int16_t* rng = (int16_t*)(H + L.range);
    int16_t* mvp = (int16_t*)(H + L.mvp);
    int16_t* mvc = (int16_t*)(H + L.mvc);
    uint8_t* nc = H + L.ncand;
    int64_t* coff = (int64_t*)(H + L.cost_off);
    int i = 0;
    for (int k = 0; k < np; k++)
    {
        const x265amd_mes::Request& r = *reqs[k];
        for (int y = 0; y < h; y++)
            memcpy(H + L.fenc + (k * blk + (size_t)y * w) * s->pix,
                   (const uint8_t*)r.fenc + (size_t)y * r.fenc_stride * s->pix, (size_t)w * s->pix);
        for (int q = 0; q < r.n; q++, i++)
        {
            const x265amd_mes_job& j = r.jobs[q];
            foff[i] = (int64_t)(k * blk);
            roff[i] = (int64_t)j.slot * s->cfg.plane_elems + s->cfg.org_offset + j.block_off;
            memcpy(rng + 4 * i, j.mv_range, 8);
            memcpy(mvp + 2 * i, j.mvp, 4);
            memcpy(mvc + 2 * (size_t)maxc * i, j.mvc, 4 * (size_t)j.num_cand);
            nc[i] = (uint8_t)j.num_cand;
            coff[i] = (int64_t)j.table * (int64_t)s->table_elems + s->cfg.mvcost_range;
        }
    }
    if (hipError_t e = hipMemcpyAsync(g.dev, H, L.out_mv, hipMemcpyHostToDevice, st)) return (int)e;
    x265amd_me_batch b;
    memset(&b, 0, sizeof(b));
    b.w = w;
    b.h = h;
    b.n = n;
    b.method = s->cfg.method;
    b.subme = s->cfg.subme;
    b.merange = s->cfg.merange;
    b.max_cand = maxc;
    b.fenc = g.dev + L.fenc;
    b.fenc_stride = w;
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
    x265amd_mes_thread* t;
    MES_TRY(thread_ctx(s, &t));
    if (coalescing())
    {
        MES_TRY(check_request(s, w, h, fenc, fenc_stride, n, jobs));
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
    x265amd_mes_thread* t;
    MES_TRY(thread_ctx(s, &t));
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
    MES_TRY(hipEventSynchronize(t->aev));
    if (n != pend) return record(X265AMD_EINVAL);
    unpack(t->async, t->pend_out, n, jobs);
    return 0;
}
