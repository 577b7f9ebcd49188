// lookahead.cpp — f1 encoder session: the lookahead cost estimates of a running x265
// encoder on the MI355X (include/x265_amd.h, x265amd_la_*).
//
// x265's lookahead keeps one Lowres per picture (lowres.cpp:30-163: one host buffer of
// four half-pel planes, `planesize` pixels each, lowresPlane[k] = buffer + k * planesize
// + padoffset) and asks for per-picture intra estimates (LookaheadTLD::lowresIntraEstimate,
// slicetype.cpp:230-336) and per-(p0, p1, b) inter estimates
// (CostEstimateGroup::estimateFrameCost -> estimateCUCost, slicetype.cpp:1977-2225) from
// its pre-lookahead and batch worker threads.  A session holds:
//   * device frame slots — a picture's four planes are uploaded once (x265amd_la_load) and
//     reused by every estimate that reads it; the intra estimate leaves the picture's
//     intraCost on the device for its P estimates;
//   * one arena for all slots, so every batch entry addresses planes as offsets from one
//     base (the batched x265amd_lowres_* entries' convention);
//   * per host thread: a non-blocking stream, device scratch for a batch of estimates,
//     pinned staging, and an arena slot for weighted reference planes (weightsAnalyse's
//     wbuffer, slicetype.cpp:391-495, which lives on the calling thread's LookaheadTLD).
// Every entry is synchronous on the calling thread's stream: the outputs are in the
// caller's host arrays when it returns.  A failure is returned AND recorded in the
// backend's sticky status (x265amd_provider_status), which the encoder binding turns into
// x265_encoder_encode() < 0.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <new>
#include <unordered_map>
#include <vector>

#include "../../../include/x265_amd.h"
#include "hostreg.h"

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

#define LA_TRY(expr)                                   \
    do                                                 \
    {                                                  \
        int st_ = (int)(expr);                         \
        if (st_) return record(st_);                   \
    } while (0)

} // namespace

struct x265amd_la_thread
{
    hipStream_t st = nullptr;
    hipEvent_t ev = nullptr;    // blocking-sync event (X265AMD_LA_SYNC=block): the waiting thread sleeps
    uint8_t* dev = nullptr;     // scratch: outputs / inputs of one estimate
    uint8_t* host = nullptr;    // pinned staging of the same size
    int wslot = -1;             // arena slot for this thread's weighted reference planes
    size_t cap = 0;             // bytes of dev / host scratch
};

struct x265amd_la
{
    x265amd_la_config cfg;
    size_t pix = 1;             // bytes per pixel
    size_t frame_bytes = 0;     // 4 planes
    int ncu = 0;
    int slots = 0;              // frame slots + thread slots
    uint8_t* arena = nullptr;   // slots * frame_bytes
    int32_t* intra = nullptr;   // slots * ncu: intraCost of each slot's picture
    int32_t* invq = nullptr;    // slots * ncu: invQscaleFactor (when AQ is on)
    uint16_t* mvcost = nullptr; // centre of the device BitCost table
    uint16_t* mvcost_base = nullptr;
    size_t scratch = 0;

    uint64_t id = 0;            // process-unique session number (a later session may reuse this address)
    std::mutex mu;
    struct Slot { int index; int gen; bool has_invq; const void* pinned; };
    std::unordered_map<const void*, Slot> frames;
    int next_frame = 0, next_thread = 0;
    std::vector<x265amd_la_thread*> threads;
};

namespace {

// a thread's context of a session is found by (address, id): x265amd_la_destroy frees every
// thread's context but cannot reach other threads' thread_local lists, and a later session can be
// allocated at the same address, so an entry of a destroyed session must never match again
struct TlsEntry { const x265amd_la* la; uint64_t id; x265amd_la_thread* t; };
thread_local std::vector<TlsEntry> tls;
std::atomic<uint64_t> g_next_id{ 1 };

// scratch layout of n estimates (byte offsets, 256-aligned), field-major as the batched
// x265amd_lowres_* entries index them (estimate e's CU arrays at e * ncu)
struct Layout
{
    size_t mvs0, mvc0, mvs1, mvc1, lc, rs, ce, mbs, offs, ds, end;
    Layout(int ncu, int hcu, int n = 1)
    {
        size_t o = 0;
        auto take = [&](size_t b) { size_t r = o; o = (o + b + 255) & ~(size_t)255; return r; };
        const size_t cus = (size_t)ncu * n;
        mvs0 = take(4 * cus);
        mvc0 = take(4 * cus);
        mvs1 = take(4 * cus);
        mvc1 = take(4 * cus);
        lc = take(2 * cus);
        rs = take(4 * (size_t)hcu * n);
        ce = take(16 * (size_t)n);
        mbs = take(4 * (size_t)n);
        offs = take(8 * 9 * (size_t)n);
        ds = take(2 * (size_t)n);
        end = o;
    }
};

// wait for the calling thread's stream: spin (hipStreamSynchronize) or, with X265AMD_LA_SYNC=block, sleep
// on a blocking-sync event so the encoder's worker threads get the core while the device works
int wait(x265amd_la_thread* t)
{
    if (t->ev)
    {
        const hipError_t e = hipEventRecord(t->ev, t->st);
        return e != hipSuccess ? (int)e : (int)hipEventSynchronize(t->ev);
    }
    return (int)hipStreamSynchronize(t->st);
}

// grow the calling thread's scratch to hold `bytes`
int reserve(x265amd_la_thread* t, size_t bytes)
{
    if (bytes <= t->cap) return 0;
    if (t->st) (void)hipStreamSynchronize(t->st);
    DevSyncScope quiet;                        // (hipFree / hipHostFree wait for every running kernel)
    (void)hipFree(t->dev);
    (void)hipHostFree(t->host);
    t->dev = t->host = nullptr;
    t->cap = 0;
    if (hipMalloc((void**)&t->dev, bytes) != hipSuccess ||
        hipHostMalloc((void**)&t->host, bytes, hipHostMallocDefault) != hipSuccess)
        return X265AMD_ENOMEM;
    t->cap = bytes;
    return 0;
}

int thread_ctx(x265amd_la* la, x265amd_la_thread** out)
{
    for (size_t i = 0; i < tls.size();)
    {
        if (tls[i].la == la && tls[i].id == la->id)
        {
            *out = tls[i].t;
            return 0;
        }
        if (tls[i].la == la)
        {
            // a destroyed session's entry at a reused address: its context is already freed
            tls[i] = tls.back();
            tls.pop_back();
            continue;
        }
        i++;
    }
    auto* t = new (std::nothrow) x265amd_la_thread();
    if (!t) return X265AMD_ENOMEM;
    {
        std::lock_guard<std::mutex> g(la->mu);
        if (la->next_thread >= la->cfg.max_threads)
        {
            delete t;
            return X265AMD_ENOMEM;
        }
        t->wslot = la->cfg.max_frames + la->next_thread++;
        la->threads.push_back(t);
    }
    {
        DevSyncScope quiet;                    // (stream creation and allocation wait for running kernels)
        if (hipStreamCreateWithFlags(&t->st, hipStreamNonBlocking) != hipSuccess || reserve(t, la->scratch))
            return X265AMD_ENOMEM;
    }
    const char* sync = getenv("X265AMD_LA_SYNC");
    if (sync && !strcmp(sync, "block") &&
        hipEventCreateWithFlags(&t->ev, hipEventBlockingSync | hipEventDisableTiming) != hipSuccess)
        return X265AMD_ENOMEM;
    tls.push_back({ la, la->id, t });
    *out = t;
    return 0;
}

int find_slot(x265amd_la* la, const void* key, int* index)
{
    std::lock_guard<std::mutex> g(la->mu);
    auto it = la->frames.find(key);
    if (it == la->frames.end()) return X265AMD_EINVAL;     // estimate of a picture never loaded
    *index = it->second.index;
    return 0;
}

int64_t plane_off(const x265amd_la* la, int slot, int k)
{
    return (int64_t)slot * 4 * la->cfg.planesize + (int64_t)k * la->cfg.planesize + la->cfg.padoffset;
}

} // namespace

extern "C" int x265amd_la_create(const x265amd_la_config* cfg, x265amd_la** out)
{
    if (!cfg || !out) return X265AMD_EINVAL;
    *out = nullptr;
    if ((cfg->depth != 8 && cfg->depth != 10 && cfg->depth != 12) || cfg->width_cu <= 0 || cfg->height_cu <= 0 ||
        cfg->planesize <= 0 || cfg->padoffset < 0 || cfg->max_frames <= 0 || cfg->max_threads <= 0 || !cfg->mvcost ||
        cfg->mvcost_range <= 0)
        return X265AMD_EINVAL;
    auto* la = new (std::nothrow) x265amd_la();
    if (!la) return record(X265AMD_ENOMEM);
    la->cfg = *cfg;
    la->id = g_next_id.fetch_add(1);
    la->pix = cfg->depth > 8 ? 2 : 1;
    la->frame_bytes = 4 * (size_t)cfg->planesize * la->pix;
    la->ncu = cfg->width_cu * cfg->height_cu;
    la->slots = cfg->max_frames + cfg->max_threads;
    la->scratch = Layout(la->ncu, cfg->height_cu).end;
    const size_t tab = 2 * (size_t)cfg->mvcost_range + 1;
    if (hipMalloc((void**)&la->arena, la->frame_bytes * la->slots) != hipSuccess ||
        hipMalloc((void**)&la->intra, sizeof(int32_t) * la->ncu * la->slots) != hipSuccess ||
        hipMalloc((void**)&la->invq, sizeof(int32_t) * la->ncu * la->slots) != hipSuccess ||
        hipMalloc((void**)&la->mvcost_base, sizeof(uint16_t) * tab) != hipSuccess ||
        hipMemcpy(la->mvcost_base, cfg->mvcost - cfg->mvcost_range, sizeof(uint16_t) * tab, hipMemcpyHostToDevice) !=
            hipSuccess)
    {
        x265amd_la_destroy(la);
        return record(X265AMD_ENOMEM);
    }
    la->mvcost = la->mvcost_base + cfg->mvcost_range;
    *out = la;
    return 0;
}

extern "C" void x265amd_la_destroy(x265amd_la* la)
{
    if (!la) return;
    DevSyncScope quiet;                        // (the frees wait for running kernels)
    for (auto* t : la->threads)
    {
        if (t->st) (void)hipStreamSynchronize(t->st);
        (void)hipFree(t->dev);
        (void)hipHostFree(t->host);
        if (t->st) (void)hipStreamDestroy(t->st);
        if (t->ev) (void)hipEventDestroy(t->ev);
        delete t;
    }
    for (auto& f : la->frames)
        x265amd_hostreg::unregister(f.second.pinned, la->frame_bytes);
    (void)hipFree(la->arena);
    (void)hipFree(la->intra);
    (void)hipFree(la->invq);
    (void)hipFree(la->mvcost_base);
    delete la;
}

extern "C" int x265amd_la_load(x265amd_la* la, const void* key, int gen, const void* buffer,
                               const int32_t* inv_qscale)
{
    if (!la || !key || !buffer) return record(X265AMD_EINVAL);
    x265amd_la_thread* t;
    LA_TRY(thread_ctx(la, &t));
    int slot;
    {
        std::lock_guard<std::mutex> g(la->mu);
        auto it = la->frames.find(key);
        if (it == la->frames.end())
        {
            if (la->next_frame >= la->cfg.max_frames) return record(X265AMD_ENOMEM);
            it = la->frames.emplace(key, x265amd_la::Slot{ la->next_frame++, gen, false, nullptr }).first;
        }
        it->second.gen = gen;
        it->second.has_invq = inv_qscale != nullptr;
        slot = it->second.index;
        // page-lock the picture's host buffer once (x265 keeps a Frame's Lowres buffer for the life of
        // the encoder and reuses it for later pictures), so every upload is a direct DMA; a buffer that
        // cannot be registered is copied pageable
        if (it->second.pinned != buffer)
        {
            x265amd_hostreg::unregister(it->second.pinned, la->frame_bytes);
            DevSyncScope quiet;                  // (hipHostRegister waits for every running kernel)
            it->second.pinned =
                hipHostRegister((void*)buffer, la->frame_bytes, hipHostRegisterDefault) == hipSuccess ? buffer : nullptr;
            (void)hipGetLastError();
        }
    }
    // x265 reuses a Lowres for a new picture only after every estimate that read it is done
    LA_TRY(hipMemcpyAsync(la->arena + (size_t)slot * la->frame_bytes, buffer, la->frame_bytes,
                          hipMemcpyHostToDevice, t->st));
    if (inv_qscale)
        LA_TRY(hipMemcpyAsync(la->invq + (size_t)slot * la->ncu, inv_qscale, sizeof(int32_t) * la->ncu,
                              hipMemcpyHostToDevice, t->st));
    return record(wait(t));
}

extern "C" int x265amd_la_intra(x265amd_la* la, const void* key, int32_t* intra_cost, uint8_t* intra_mode,
                                uint16_t* lowres_cost, int32_t* row_satd, int64_t* cost_est)
{
    if (!la || !key || !intra_cost || !intra_mode || !lowres_cost || !row_satd || !cost_est)
        return record(X265AMD_EINVAL);
    x265amd_la_thread* t;
    LA_TRY(thread_ctx(la, &t));
    int slot;
    bool has_invq;
    {
        std::lock_guard<std::mutex> g(la->mu);
        auto it = la->frames.find(key);
        if (it == la->frames.end()) return record(X265AMD_EINVAL);
        slot = it->second.index;
        has_invq = it->second.has_invq;
    }
    const int ncu = la->ncu, hcu = la->cfg.height_cu;
    const Layout L(ncu, hcu);
    int64_t* off = (int64_t*)(t->host + L.offs);
    off[0] = plane_off(la, slot, 0);
    LA_TRY(hipMemcpyAsync(t->dev + L.offs, off, 8, hipMemcpyHostToDevice, t->st));
    int32_t* dic = la->intra + (size_t)slot * ncu;
    x265amd_lowres_intra_batch b{ 1, la->cfg.width_cu, hcu, la->arena, la->cfg.lowres_stride,
                                  (const int64_t*)(t->dev + L.offs),
                                  has_invq ? la->invq + (size_t)slot * ncu : nullptr, dic,
                                  (uint8_t*)(t->dev + L.mvs0), (uint16_t*)(t->dev + L.lc), (int32_t*)(t->dev + L.rs),
                                  (int64_t*)(t->dev + L.ce) };
    LA_TRY(x265amd_lowres_intra(la->cfg.depth, &b, t->st));
    LA_TRY(hipMemcpyAsync(t->host + L.mvc0, dic, 4 * (size_t)ncu, hipMemcpyDeviceToHost, t->st));
    LA_TRY(hipMemcpyAsync(t->host + L.mvs0, t->dev + L.mvs0, ncu, hipMemcpyDeviceToHost, t->st));
    LA_TRY(hipMemcpyAsync(t->host + L.lc, t->dev + L.lc, L.rs - L.lc + 4 * (size_t)hcu, hipMemcpyDeviceToHost, t->st));
    LA_TRY(hipMemcpyAsync(t->host + L.ce, t->dev + L.ce, 16, hipMemcpyDeviceToHost, t->st));
    LA_TRY(wait(t));
    memcpy(intra_cost, t->host + L.mvc0, 4 * (size_t)ncu);
    memcpy(intra_mode, t->host + L.mvs0, ncu);
    memcpy(lowres_cost, t->host + L.lc, 2 * (size_t)ncu);
    memcpy(row_satd, t->host + L.rs, 4 * (size_t)hcu);
    memcpy(cost_est, t->host + L.ce, 16);
    return 0;
}

extern "C" int x265amd_la_pcost_n(x265amd_la* la, int n, x265amd_la_pjob* jobs, int rows_per_slice, int num_slices)
{
    if (!la || n < 0 || (n && !jobs)) return record(X265AMD_EINVAL);
    if (!n) return 0;
    for (int e = 0; e < n; e++)
    {
        const x265amd_la_pjob& j = jobs[e];
        if (!j.fenc || !j.ref || !j.mvs || !j.mv_costs || !j.lowres_costs || !j.row_satd || (j.weighted_buffer && n > 1))
            return record(X265AMD_EINVAL);
    }
    x265amd_la_thread* t;
    LA_TRY(thread_ctx(la, &t));
    const int ncu = la->ncu, hcu = la->cfg.height_cu;
    const Layout L(ncu, hcu, n);
    LA_TRY(reserve(t, L.end));
    int64_t* off = (int64_t*)(t->host + L.offs);
    bool has_invq = false;
    for (int e = 0; e < n; e++)
    {
        int sf, sr;
        LA_TRY(find_slot(la, jobs[e].fenc, &sf));
        LA_TRY(find_slot(la, jobs[e].ref, &sr));
        if (e == 0)
        {
            std::lock_guard<std::mutex> g(la->mu);
            has_invq = la->frames[jobs[0].fenc].has_invq;
        }
        if (jobs[e].weighted_buffer)
        {
            // weightsAnalyse's planes (the calling thread's LookaheadTLD wbuffer, same layout)
            LA_TRY(hipMemcpyAsync(la->arena + (size_t)t->wslot * la->frame_bytes, jobs[e].weighted_buffer,
                                  la->frame_bytes, hipMemcpyHostToDevice, t->st));
            sr = t->wslot;
        }
        off[e] = plane_off(la, sf, 0);
        for (int k = 0; k < 4; k++) off[n + 4 * e + k] = plane_off(la, sr, k);
        // per-estimate intraCost / invQscaleFactor, gathered from the pictures' slots into the
        // scratch's (unused by a P estimate) list-1 arrays
        LA_TRY(hipMemcpyAsync(t->dev + L.mvs1 + 4 * (size_t)ncu * e, la->intra + (size_t)sf * ncu, 4 * (size_t)ncu,
                              hipMemcpyDeviceToDevice, t->st));
        if (has_invq)
            LA_TRY(hipMemcpyAsync(t->dev + L.mvc1 + 4 * (size_t)ncu * e, la->invq + (size_t)sf * ncu, 4 * (size_t)ncu,
                                  hipMemcpyDeviceToDevice, t->st));
    }
    LA_TRY(hipMemcpyAsync(t->dev + L.offs, off, 8 * 5 * (size_t)n, hipMemcpyHostToDevice, t->st));
    const int64_t* doff = (const int64_t*)(t->dev + L.offs);
    x265amd_lowres_pcost_batch b{ n, la->cfg.width_cu, hcu, rows_per_slice, num_slices, la->arena,
                                  la->cfg.lowres_stride, doff, doff + n, (const int32_t*)(t->dev + L.mvs1),
                                  has_invq ? (const int32_t*)(t->dev + L.mvc1) : nullptr, la->mvcost,
                                  (int16_t*)(t->dev + L.mvs0), (int32_t*)(t->dev + L.mvc0), (uint16_t*)(t->dev + L.lc),
                                  (int32_t*)(t->dev + L.rs), (int64_t*)(t->dev + L.ce), (int32_t*)(t->dev + L.mbs) };
    LA_TRY(x265amd_lowres_pcost(la->cfg.depth, &b, t->st));
    LA_TRY(hipMemcpyAsync(t->host + L.mvs0, t->dev + L.mvs0, L.mvs1 - L.mvs0, hipMemcpyDeviceToHost, t->st));
    LA_TRY(hipMemcpyAsync(t->host + L.lc, t->dev + L.lc, L.offs - L.lc, hipMemcpyDeviceToHost, t->st));
    LA_TRY(wait(t));
    for (int e = 0; e < n; e++)
    {
        x265amd_la_pjob& j = jobs[e];
        memcpy(j.mvs, t->host + L.mvs0 + 4 * (size_t)ncu * e, 4 * (size_t)ncu);
        memcpy(j.mv_costs, t->host + L.mvc0 + 4 * (size_t)ncu * e, 4 * (size_t)ncu);
        memcpy(j.lowres_costs, t->host + L.lc + 2 * (size_t)ncu * e, 2 * (size_t)ncu);
        memcpy(j.row_satd, t->host + L.rs + 4 * (size_t)hcu * e, 4 * (size_t)hcu);
        memcpy(j.cost_est, t->host + L.ce + 16 * (size_t)e, 16);
        memcpy(&j.intra_mbs, t->host + L.mbs + 4 * (size_t)e, 4);
    }
    return 0;
}

extern "C" int x265amd_la_bcost_n(x265amd_la* la, int n, x265amd_la_bjob* jobs, int rows_per_slice, int num_slices)
{
    if (!la || n < 0 || (n && !jobs)) return record(X265AMD_EINVAL);
    if (!n) return 0;
    for (int e = 0; e < n; e++)
    {
        const x265amd_la_bjob& j = jobs[e];
        if (!j.fenc || !j.ref0 || !j.ref1 || !j.mvs0 || !j.mv_costs0 || !j.mvs1 || !j.mv_costs1 || !j.lowres_costs ||
            !j.row_satd)
            return record(X265AMD_EINVAL);
    }
    x265amd_la_thread* t;
    LA_TRY(thread_ctx(la, &t));
    const int ncu = la->ncu, hcu = la->cfg.height_cu;
    const Layout L(ncu, hcu, n);
    LA_TRY(reserve(t, L.end));
    // per-estimate invQscaleFactor goes in a device array of its own (after the layout)
    bool has_invq = false;
    {
        std::lock_guard<std::mutex> g(la->mu);
        has_invq = la->frames.count(jobs[0].fenc) && la->frames[jobs[0].fenc].has_invq;
    }
    const size_t iq = (L.end + 255) & ~(size_t)255;
    if (has_invq) LA_TRY(reserve(t, iq + 4 * (size_t)ncu * n));
    int64_t* off = (int64_t*)(t->host + L.offs);
    uint8_t* ds = t->host + L.ds;
    for (int e = 0; e < n; e++)
    {
        const x265amd_la_bjob& j = jobs[e];
        int sf, s0, s1;
        LA_TRY(find_slot(la, j.fenc, &sf));
        LA_TRY(find_slot(la, j.ref0, &s0));
        LA_TRY(find_slot(la, j.ref1, &s1));
        off[e] = plane_off(la, sf, 0);
        for (int k = 0; k < 4; k++)
        {
            off[n + 4 * e + k] = plane_off(la, s0, k);
            off[5 * n + 4 * e + k] = plane_off(la, s1, k);
        }
        ds[2 * e] = (uint8_t)!!j.do_search0;
        ds[2 * e + 1] = (uint8_t)!!j.do_search1;
        if (has_invq)
            LA_TRY(hipMemcpyAsync(t->dev + iq + 4 * (size_t)ncu * e, la->invq + (size_t)sf * ncu, 4 * (size_t)ncu,
                                  hipMemcpyDeviceToDevice, t->st));
        // a list that is not searched reuses the stored lowresMvs / lowresMvCosts (slicetype.cpp:2105-2109, 2171-2172)
        if (!j.do_search0)
        {
            memcpy(t->host + L.mvs0 + 4 * (size_t)ncu * e, j.mvs0, 4 * (size_t)ncu);
            memcpy(t->host + L.mvc0 + 4 * (size_t)ncu * e, j.mv_costs0, 4 * (size_t)ncu);
        }
        if (!j.do_search1)
        {
            memcpy(t->host + L.mvs1 + 4 * (size_t)ncu * e, j.mvs1, 4 * (size_t)ncu);
            memcpy(t->host + L.mvc1 + 4 * (size_t)ncu * e, j.mv_costs1, 4 * (size_t)ncu);
        }
    }
    // inputs: the stored MVs / costs (all four arrays at once), descriptors, search flags
    LA_TRY(hipMemcpyAsync(t->dev + L.mvs0, t->host + L.mvs0, L.lc - L.mvs0, hipMemcpyHostToDevice, t->st));
    LA_TRY(hipMemcpyAsync(t->dev + L.offs, t->host + L.offs, L.end - L.offs, hipMemcpyHostToDevice, t->st));
    const int64_t* doff = (const int64_t*)(t->dev + L.offs);
    x265amd_lowres_bcost_batch b{ n, la->cfg.width_cu, hcu, rows_per_slice, num_slices, la->arena,
                                  la->cfg.lowres_stride, doff, doff + n, doff + 5 * n, t->dev + L.ds,
                                  has_invq ? (const int32_t*)(t->dev + iq) : nullptr, la->mvcost,
                                  (int16_t*)(t->dev + L.mvs0), (int32_t*)(t->dev + L.mvc0),
                                  (int16_t*)(t->dev + L.mvs1), (int32_t*)(t->dev + L.mvc1),
                                  (uint16_t*)(t->dev + L.lc), (int32_t*)(t->dev + L.rs), (int64_t*)(t->dev + L.ce) };
    LA_TRY(x265amd_lowres_bcost(la->cfg.depth, &b, t->st));
    LA_TRY(hipMemcpyAsync(t->host + L.mvs0, t->dev + L.mvs0, L.offs - L.mvs0, hipMemcpyDeviceToHost, t->st));
    LA_TRY(wait(t));
    for (int e = 0; e < n; e++)
    {
        x265amd_la_bjob& j = jobs[e];
        if (j.do_search0)
        {
            memcpy(j.mvs0, t->host + L.mvs0 + 4 * (size_t)ncu * e, 4 * (size_t)ncu);
            memcpy(j.mv_costs0, t->host + L.mvc0 + 4 * (size_t)ncu * e, 4 * (size_t)ncu);
        }
        if (j.do_search1)
        {
            memcpy(j.mvs1, t->host + L.mvs1 + 4 * (size_t)ncu * e, 4 * (size_t)ncu);
            memcpy(j.mv_costs1, t->host + L.mvc1 + 4 * (size_t)ncu * e, 4 * (size_t)ncu);
        }
        memcpy(j.lowres_costs, t->host + L.lc + 2 * (size_t)ncu * e, 2 * (size_t)ncu);
        memcpy(j.row_satd, t->host + L.rs + 4 * (size_t)hcu * e, 4 * (size_t)hcu);
        memcpy(j.cost_est, t->host + L.ce + 16 * (size_t)e, 16);
    }
    return 0;
}

extern "C" int x265amd_la_pcost(x265amd_la* la, const void* fenc, const void* ref, const void* weighted_buffer,
                                int rows_per_slice, int num_slices, int16_t* mvs, int32_t* mv_costs,
                                uint16_t* lowres_costs, int32_t* row_satd, int64_t* cost_est, int32_t* intra_mbs)
{
    if (!cost_est || !intra_mbs) return record(X265AMD_EINVAL);
    x265amd_la_pjob j{ fenc, ref, weighted_buffer, mvs, mv_costs, lowres_costs, row_satd, { 0, 0 }, 0 };
    const int st = x265amd_la_pcost_n(la, 1, &j, rows_per_slice, num_slices);
    if (!st)
    {
        cost_est[0] = j.cost_est[0];
        cost_est[1] = j.cost_est[1];
        *intra_mbs = j.intra_mbs;
    }
    return st;
}

extern "C" int x265amd_la_bcost(x265amd_la* la, const void* fenc, const void* ref0, const void* ref1, int do_search0,
                                int do_search1, int rows_per_slice, int num_slices, int16_t* mvs0, int32_t* mv_costs0,
                                int16_t* mvs1, int32_t* mv_costs1, uint16_t* lowres_costs, int32_t* row_satd,
                                int64_t* cost_est)
{
    if (!cost_est) return record(X265AMD_EINVAL);
    x265amd_la_bjob j{ fenc, ref0, ref1, do_search0, do_search1, mvs0, mv_costs0, mvs1, mv_costs1, lowres_costs,
                       row_satd, { 0, 0 } };
    const int st = x265amd_la_bcost_n(la, 1, &j, rows_per_slice, num_slices);
    if (!st)
    {
        cost_est[0] = j.cost_est[0];
        cost_est[1] = j.cost_est[1];
    }
    return st;
}

// Lookahead::estimateCUPropagate (slicetype.cpp:1741-1842) of the running encoder: the CU arrays
// from the caller's Lowres staged in one upload, x265amd_cutree_propagate, the two reference
// propagateCost arrays back (list 1 only when it is used).  cuTree runs on the lookahead's decision
// thread, one propagation after another (each reads what the previous one accumulated), so the
// call is synchronous like the estimates.
extern "C" int x265amd_la_propagate(x265amd_la* la, const uint16_t* propagate_in, const int32_t* intra_cost,
                                    const uint16_t* lowres_costs, const int32_t* inv_qscale, const int32_t* mvs0,
                                    const int32_t* mvs1, double fps_factor, const int* bipred_weight,
                                    uint16_t* ref_costs0, uint16_t* ref_costs1)
{
    if (!la || !intra_cost || !lowres_costs || !inv_qscale || !mvs0 || !bipred_weight || !ref_costs0 ||
        (mvs1 && !ref_costs1))
        return record(X265AMD_EINVAL);
    x265amd_la_thread* t;
    LA_TRY(thread_ctx(la, &t));
    const size_t ncu = (size_t)la->ncu;
    // staging: inputs first (one upload), then the two reference arrays (in / out), then device-only scratch
    size_t o = 0;
    auto take = [&](size_t b) { size_t r = o; o = (o + b + 255) & ~(size_t)255; return r; };
    const size_t o_pin = take(2 * ncu), o_ic = take(4 * ncu), o_lc = take(2 * ncu), o_iq = take(4 * ncu),
                 o_m0 = take(4 * ncu), o_m1 = take(4 * ncu), o_r0 = take(2 * ncu), o_r1 = take(2 * ncu),
                 o_sc = take(16 * ncu), end = o;
    LA_TRY(reserve(t, end));
    uint8_t* H = t->host;
    if (propagate_in) memcpy(H + o_pin, propagate_in, 2 * ncu);
    memcpy(H + o_ic, intra_cost, 4 * ncu);
    memcpy(H + o_lc, lowres_costs, 2 * ncu);
    memcpy(H + o_iq, inv_qscale, 4 * ncu);
    memcpy(H + o_m0, mvs0, 4 * ncu);
    if (mvs1) memcpy(H + o_m1, mvs1, 4 * ncu);
    memcpy(H + o_r0, ref_costs0, 2 * ncu);
    if (mvs1) memcpy(H + o_r1, ref_costs1, 2 * ncu);
    LA_TRY(hipMemcpyAsync(t->dev, H, o_sc, hipMemcpyHostToDevice, t->st));
    x265amd_propagate_batch b;
    memset(&b, 0, sizeof(b));
    b.width_cu = la->cfg.width_cu;
    b.height_cu = la->cfg.height_cu;
    b.propagate_in = propagate_in ? (const uint16_t*)(t->dev + o_pin) : nullptr;
    b.intra_cost = (const int32_t*)(t->dev + o_ic);
    b.lowres_costs = (const uint16_t*)(t->dev + o_lc);
    b.inv_qscale = (const int32_t*)(t->dev + o_iq);
    b.mvs[0] = (const int32_t*)(t->dev + o_m0);
    b.mvs[1] = mvs1 ? (const int32_t*)(t->dev + o_m1) : nullptr;
    b.fps_factor = fps_factor;
    b.bipred_weight[0] = bipred_weight[0];
    b.bipred_weight[1] = bipred_weight[1];
    b.ref_costs[0] = (uint16_t*)(t->dev + o_r0);
    b.ref_costs[1] = mvs1 ? (uint16_t*)(t->dev + o_r1) : nullptr;
    b.scratch = (int64_t*)(t->dev + o_sc);
    LA_TRY(x265amd_cutree_propagate(1, &b, t->st));
    LA_TRY(hipMemcpyAsync(H + o_r0, t->dev + o_r0, o_sc - o_r0, hipMemcpyDeviceToHost, t->st));
    LA_TRY(wait(t));
    memcpy(ref_costs0, H + o_r0, 2 * ncu);
    if (mvs1) memcpy(ref_costs1, H + o_r1, 2 * ncu);
    return 0;
}
