// rdosession.cpp — f3 in the running encoder: the residual coding of inter CUs on the MI355X
// (include/x265_amd.h, x265amd_rdo_*).
//
// Search::encodeResAndCalcRdInterCU (search.cpp:2562-2690) codes an inter CU's residual through
// estimateResidualQT (search.cpp:2838-3140): for every transform unit of the CU — at --preset medium
// one RQT level, TUs of min(CU, 32) luma and half that chroma — Quant::transformNxN (dct, quant,
// sign-bit hiding), Quant::invtransformNxN (dequant, idct), the reconstruction pred + residual, and the
// psy energies psyCost_pp(fenc, pred) / psyCost_pp(fenc, recon) (pixel.cpp:672-703) that its RD costs
// use; the CABAC bit estimates (codeCoeffNxN) and the decisions stay on the host.  Given the CU's source
// and prediction these results depend on nothing else, so a worker posts the CU (its fenc and pred
// planes, the Quant object's QPs) and a service thread runs, for every CU posted at once, one upload,
// the fused TU kernels (csrc/tu.hip: residual -> DCT -> quant -> SBH -> dequant -> iDCT -> recon) for
// all luma and all chroma TUs, the per-8x8 psy energies of fenc against pred and against the coded
// reconstruction (csrc/pixel.hip, X265AMD_PSY 8x8 jobs: psyCost_pp sums |E(src) - E(rec)| over 8x8
// blocks, so a sum over any block of 8x8 blocks — a TU, the whole CU, a CU whose TUs are partly coded —
// is a sum of these), and one download.  The encoder binding (integration/gpu_rdo.cpp) serves the
// reference's own estimateResidualQT from these results, checking every input it can.
//
// Service and waiting follow csrc/mesession.cpp's launch service: per host thread a few request slots,
// launcher threads take every queued request, waiters pause-spin, then yield, then sleep.
#include <hip/hip_runtime.h>
#include <sched.h>
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
#include <vector>

#include "../../../include/x265_amd.h"
#include "rdojob.h"
#include "devsync.h"

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

double now_s()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

constexpr int kSlots = 4;            // outstanding requests per host thread

// sizes of one CU's planes and TUs (4:2:0)
struct Geo
{
    int c, cc;                       // luma / chroma plane width (= height)
    int tl, tlc;                     // luma / chroma TU log2
    int ntu, ntuc;                   // TUs per luma / chroma plane
    int nb, nbc;                     // 8x8 blocks per luma / chroma plane
    size_t pix_y, pix_c;             // pixels per luma / chroma plane
    explicit Geo(int log2)
    {
        c = 1 << log2;
        cc = c >> 1;
        tl = log2 < 5 ? log2 : 5;
        tlc = tl - 1;
        ntu = (c >> tl) * (c >> tl);
        ntuc = (cc >> tlc) * (cc >> tlc);
        nb = (c >> 3) * (c >> 3);
        nbc = (cc >> 3) * (cc >> 3);
        pix_y = (size_t)c * c;
        pix_c = (size_t)cc * cc;
    }
    size_t pix() const { return pix_y + 2 * pix_c; }
    int tus() const { return ntu + 2 * ntuc; }
    int blocks() const { return nb + 2 * nbc; }
};

} // namespace

// one posted CU: its inputs (packed planes, stride = plane width) and, once done, its results
struct x265amd_rdo_req
{
    x265amd_rdo_cu cu{};
    uint8_t* in = nullptr;           // fenc Y Cb Cr, pred Y Cb Cr (2 * pix() * bytes per pixel)
    uint8_t* out = nullptr;          // recon, resi, coeff, num_sig, psy_pred, psy_rec
    x265amd_rdo_result res{};
    std::atomic<int> state{ 0 };     // 0 free, 1 queued, 2 done
    int rc = 0;
    double t_post = 0;
    uint32_t want = 1;               // direct mode: the completion word's value once served (1, or the server seq)
    uint32_t seq = 0;                // server mode: the slot's last sequence number
};

struct x265amd_rdo_thread
{
    x265amd_rdo_req req[kSlots];
    // direct mode (cfg.launchers == 0): the thread's own stream and one mapped, coherent pinned region per
    // slot — inputs, descriptors and outputs — that the kernels read and write in place (no copies), and
    // a completion flag the stream writes after the kernels (hipStreamWriteValue32) and the waiter polls
    hipStream_t st = nullptr;
    uint8_t* host = nullptr;
    uint8_t* hdev = nullptr;
    size_t region = 0;
    hipEvent_t ev[kSlots][2] = {};   // X265AMD_RDO_TIMING=1: the device span of each slot's kernels
    int index = -1;                  // server mode: the thread's slots are slots index * kSlots .. + kSlots - 1
    bool owns_host = true;           // (server mode: the region is the session's)
};

struct x265amd_rdo_launcher
{
    hipStream_t st = nullptr;
    hipEvent_t done = nullptr, k0 = nullptr, k1 = nullptr;
    uint8_t* dev = nullptr;
    uint8_t* host = nullptr;
    size_t cap = 0;
    std::thread th;
};

struct x265amd_rdo
{
    x265amd_rdo_config cfg{};
    uint64_t id = 0;
    size_t pix = 1;
    std::mutex mu;
    std::vector<x265amd_rdo_thread*> threads;
    std::vector<x265amd_rdo_launcher*> launchers;
    std::mutex qmu;
    std::condition_variable qcv;
    std::vector<x265amd_rdo_req*> rq;
    bool stop = false;
    std::atomic<bool> stop_flag{ false };
    std::atomic<int64_t> queued{ 0 };
    std::atomic<int> qsleepers{ 0 };
    std::mutex dmu;
    std::condition_variable dcv;
    int dsleepers = 0;
    int spin_us = 50, yield_us = 5000, idle_us = 500;
    bool timing = false;
    std::mutex smu;
    x265amd_rdo_counters st{};
    // server mode (X265AMD_RDO_SERVER=1, direct mode only): one resident kernel (tu.hip k_rdo_server) serves
    // the slots of every posting thread, all in one mapped region; it is relaunched before its lifetime ends
    bool server = false;
    std::atomic<bool> srv_broken{ false };   // a request went unserved for a second: no more posts to the server
    uint8_t* srv_host = nullptr;     // kSrvThreads * kSlots slots of `region` bytes
    uint8_t* srv_dev = nullptr;
    uint32_t* srv_ctl = nullptr;     // mapped: [0] stop
    uint32_t* srv_ctl_dev = nullptr;
    size_t srv_region = 0;
    hipStream_t srv_st = nullptr;
    std::mutex srv_mu;
    std::atomic<double> srv_launched{ -1.0 };   // host time of the running server's launch (< 0: none)
    int srv_nwg = 32;
    bool srv_coop = true;
    bool srv_probe = false;          // X265AMD_RDO_SERVER_PROBE=1: run the server, post nothing to it
    bool srv_timing = false;         // X265AMD_RDO_SERVER_TIMING=1: phase stamps of every request, printed at destroy
    // device-memory input slots and control words (large-BAR hosts; X265AMD_RDO_SERVER_VRAM=0: host memory):
    // the host writes each request's inputs, descriptors, job and sequence word straight into device memory
    // through the BAR (no reads), so the server stages them from HBM instead of across PCIe
    uint8_t* srv_in = nullptr;
    size_t srv_in_region = 0;
    uint32_t* srv_vctl = nullptr;    // (in srv_in's allocation) [0] stop, [kRdoBellWord + g] doorbells
    std::atomic<uint32_t> srv_bells[256];
    double srv_phase[5] = {};        // job copy, luma TUs, chroma TUs, psy, release (us, summed)
    int64_t srv_stamped = 0;
};

namespace {

struct TlsEntry { const x265amd_rdo* s; uint64_t id; x265amd_rdo_thread* t; };
thread_local std::vector<TlsEntry> tls;
std::atomic<uint64_t> g_next_id{ 1 };

size_t out_bytes(const Geo& g, size_t pix)
{
    // recon (pixels), resi + coeff (int16 each), num_sig (uint32 per TU), psy_pred + psy_rec (int32 per block),
    // sse_pred + sse_rec (int32 per block; the server's requests only)
    return g.pix() * pix + 2 * g.pix() * 2 + 4 * (size_t)g.tus() + 16 * (size_t)g.blocks();
}

void set_result(x265amd_rdo_req* r, size_t pix, bool sse = false)
{
    const Geo g(r->cu.log2_cu);
    x265amd_rdo_result& o = r->res;
    o.log2_cu = r->cu.log2_cu;
    uint8_t* p = r->out;
    const size_t sz[3] = { g.pix_y, g.pix_c, g.pix_c };
    for (int k = 0; k < 3; k++) { o.recon[k] = p; p += sz[k] * pix; }
    for (int k = 0; k < 3; k++) { o.resi[k] = (const int16_t*)p; p += sz[k] * 2; }
    for (int k = 0; k < 3; k++) { o.coeff[k] = (const int16_t*)p; p += sz[k] * 2; }
    const int nt[3] = { g.ntu, g.ntuc, g.ntuc }, nb[3] = { g.nb, g.nbc, g.nbc };
    for (int k = 0; k < 3; k++) { o.num_sig[k] = (const uint32_t*)p; p += 4 * (size_t)nt[k]; }
    for (int k = 0; k < 3; k++) { o.psy_pred[k] = (const int32_t*)p; p += 4 * (size_t)nb[k]; }
    for (int k = 0; k < 3; k++) { o.psy_rec[k] = (const int32_t*)p; p += 4 * (size_t)nb[k]; }
    for (int k = 0; k < 3; k++) { o.sse_pred[k] = sse ? (const int32_t*)p : nullptr; p += 4 * (size_t)nb[k]; }
    for (int k = 0; k < 3; k++) { o.sse_rec[k] = sse ? (const int32_t*)p : nullptr; p += 4 * (size_t)nb[k]; }
    for (int k = 0; k < 3; k++)
    {
        o.tu_log2[k] = k ? g.tlc : g.tl;
        o.ntu[k] = nt[k];
    }
}

void free_thread(x265amd_rdo_thread* t)
{
    for (auto& q : t->req) { free(q.in); if (!t->host) free(q.out); }    // direct mode: out is in the region
    if (t->st) { (void)hipStreamSynchronize(t->st); (void)hipStreamDestroy(t->st); }
    for (auto& e : t->ev)
        for (hipEvent_t v : e)
            if (v) (void)hipEventDestroy(v);
    if (t->host && t->owns_host) (void)hipHostFree(t->host);
    delete t;
}

// direct mode: per slot [in 2 * pix()][out out_bytes][descriptors][flag], sized for a 64x64 CU
size_t direct_region(size_t pix)
{
    const Geo g(6);
    return (x265amd::rdo_out_at(pix) + out_bytes(g, pix) + x265amd::kRdoJobFromEnd + 4095) & ~(size_t)4095;
}

int getenv_int(const char* name, int dflt);

// the sessions whose server may be running, and the device-synchronising calls in progress (devsync.h)
std::mutex g_srv_reg_mu;
std::vector<x265amd_rdo*> g_srv_reg;
std::atomic<int> g_quiesce{ 0 };

constexpr int kSrvThreads = 64;         // posting threads a server session serves (more: their CUs stay on the host)
constexpr double kSrvHostLife = 0.5;    // the host relaunches the server this long after its launch ...
constexpr double kSrvGpuLife = 2.0;     // ... well before it leaves on its own

int server_alloc(x265amd_rdo* s);

int server_setup(x265amd_rdo* s)
{
    bool fresh = false;
    {
        std::lock_guard<std::mutex> lk(s->srv_mu);
        if (s->srv_host) return 0;
        if (int rc = server_alloc(s)) return rc;
        fresh = true;
    }
    if (fresh)
    {
        // (registered without holding srv_mu: x265amd_devsync_begin takes the registry lock, then srv_mu)
        std::lock_guard<std::mutex> rl(g_srv_reg_mu);
        g_srv_reg.push_back(s);
    }
    return 0;
}

int server_alloc(x265amd_rdo* s)
{
    s->srv_region = direct_region(s->pix);
    const size_t bytes = s->srv_region * kSlots * kSrvThreads;
    // a non-blocking stream of its own; the server is a cooperative launch (tu.hip), which the runtime gives
    // a hardware queue of its own with every workgroup resident — a resident kernel in a queue shared with
    // other streams held back every launch behind it (the motion searches' waits went 1 -> 40-52 s per 2160p
    // encode), and a CU-masked stream (hipExtStreamCreateWithCUMask) is a blocking stream that synchronises
    // with the null stream
    {
        // X265AMD_RDO_SERVER_QUEUE: low (default: an ordinary launch on a stream of the lowest priority, which
        // no other stream of the library uses, so it has a hardware queue to itself), coop (a cooperative
        // launch: the same speed, but rocprofv3's kernel trace crashes at the exit of a process that made one),
        // high, normal (a stream of that priority; normal shares a queue: slow)
        const char* q = getenv("X265AMD_RDO_SERVER_QUEUE");
        int lo = 0, hi = 0;
        (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
        s->srv_coop = q && !strcmp(q, "coop");
        const int prio = !q || !strcmp(q, "low") ? lo : (!strcmp(q, "high") ? hi : 0);
        if (hipStreamCreateWithPriority(&s->srv_st, hipStreamNonBlocking, prio) != hipSuccess) return X265AMD_ENOMEM;
    }
    if (hipHostMalloc((void**)&s->srv_host, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&s->srv_dev, s->srv_host, 0) != hipSuccess ||
        hipHostMalloc((void**)&s->srv_ctl, 4 * x265amd::kRdoCtlWords, hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer((void**)&s->srv_ctl_dev, s->srv_ctl, 0) != hipSuccess)
        return X265AMD_ENOMEM;
    memset(s->srv_host, 0, bytes);             // every sequence and done word 0
    memset(s->srv_ctl, 0, 4 * x265amd::kRdoCtlWords);
    int dev = 0, large_bar = 0;
    if (getenv_int("X265AMD_RDO_SERVER_VRAM", 1) != 0 && hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, dev) == hipSuccess && large_bar)
    {
        s->srv_in_region = (x265amd::rdo_out_at(s->pix) + sizeof(x265amd::RdoJob) + 255) & ~(size_t)255;
        const size_t in_bytes = s->srv_in_region * kSlots * kSrvThreads + 4 * x265amd::kRdoCtlWords;
        if (hipExtMallocWithFlags((void**)&s->srv_in, in_bytes, hipDeviceMallocFinegrained) == hipSuccess &&
            hipMemset(s->srv_in, 0, in_bytes) == hipSuccess && hipDeviceSynchronize() == hipSuccess)
        {
            s->srv_vctl = (uint32_t*)(s->srv_in + s->srv_in_region * kSlots * kSrvThreads);
            for (auto& b : s->srv_bells) b.store(0);
        }
        else
        {
            if (s->srv_in) (void)hipFree(s->srv_in);
            s->srv_in = nullptr;
            (void)hipGetLastError();
        }
    }
    return 0;
}

// the server's stop word (host or device memory; plain stores to device memory, fenced: write-combined)
void set_stop(x265amd_rdo* s, uint32_t v)
{
    if (s->srv_vctl)
    {
        *(volatile uint32_t*)&s->srv_vctl[0] = v;
        __builtin_ia32_sfence();
    }
    else
        __atomic_store_n(&s->srv_ctl[0], v, __ATOMIC_SEQ_CST);
}

// stop a session's server (it serves what it finds pending and leaves); the caller holds s->srv_mu
int stop_server_locked(x265amd_rdo* s)
{
    if (s->srv_launched.load(std::memory_order_acquire) < 0) return 0;
    set_stop(s, 1u);
    const hipError_t e = hipStreamSynchronize(s->srv_st);
    set_stop(s, 0u);
    s->srv_launched.store(-1.0, std::memory_order_release);
    return e != hipSuccess ? record((int)e) : 0;
}

// the server is running and will be for a while: relaunch it when its host-side lifetime is over (or, with
// force, when a wait found it gone); the old one serves what it finds pending and leaves first
int ensure_server(x265amd_rdo* s, bool force)
{
    const double seen = s->srv_launched.load(std::memory_order_acquire);
    if (!force && seen >= 0 && now_s() - seen < kSrvHostLife) return 0;
    if (g_quiesce.load(std::memory_order_acquire) > 0) return 0;          // relaunched after the device sync
    std::lock_guard<std::mutex> lk(s->srv_mu);
    if (g_quiesce.load(std::memory_order_acquire) > 0) return 0;
    const double at = s->srv_launched.load(std::memory_order_acquire);
    if (at != seen && at >= 0 && now_s() - at < kSrvHostLife) return 0;     // another thread relaunched it
    if (int rc = stop_server_locked(s)) return rc;
    x265amd::RdoServerArgs a{ s->srv_dev, (uint64_t)s->srv_region, kSrvThreads * kSlots, (int)s->cfg.depth,
                              s->srv_vctl ? s->srv_vctl : s->srv_ctl_dev, (uint64_t)(kSrvGpuLife * 1e8),
                              s->srv_timing ? 1 : 0, s->srv_in, (uint64_t)s->srv_in_region };
    const int rc = x265amd_rdo_server_launch(&a, s->srv_nwg, s->srv_coop ? 1 : 0, s->srv_st);
    s->srv_launched.store(rc ? -1.0 : now_s(), std::memory_order_release);
    return rc ? record(rc) : 0;
}

int direct_setup(x265amd_rdo* s, x265amd_rdo_thread* t)
{
    if (t->host) return 0;
    if (s->server)
    {
        if (t->index < 0 || t->index >= kSrvThreads) return X265AMD_ENOMEM;
        if (int rc = server_setup(s)) return rc;
        t->region = s->srv_region;
        t->host = s->srv_host + (size_t)t->index * kSlots * t->region;
        t->hdev = s->srv_dev + (size_t)t->index * kSlots * t->region;
        t->owns_host = false;
        for (int k = 0; k < kSlots; k++)
        {
            free(t->req[k].out);
            t->req[k].out = nullptr;
        }
        return 0;
    }
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    t->region = direct_region(s->pix);
    if (hipStreamCreateWithPriority(&t->st, hipStreamNonBlocking, hi) != hipSuccess ||
        hipHostMalloc((void**)&t->host, t->region * kSlots, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&t->hdev, t->host, 0) != hipSuccess)
        return X265AMD_ENOMEM;
    for (int k = 0; k < kSlots; k++)
    {
        free(t->req[k].out);                                     // outputs live in the mapped region
        t->req[k].out = nullptr;
        if (s->timing)
            for (int e = 0; e < 2; e++)
                if (hipEventCreate(&t->ev[k][e]) != hipSuccess) return X265AMD_ENOMEM;
    }
    return 0;
}

int thread_ctx(x265amd_rdo* s, x265amd_rdo_thread** out)
{
    for (size_t i = 0; i < tls.size();)
    {
        if (tls[i].s == s && tls[i].id == s->id) { *out = tls[i].t; return 0; }
        if (tls[i].s == s) { tls[i] = tls.back(); tls.pop_back(); continue; }   // a destroyed session's entry
        i++;
    }
    auto* t = new (std::nothrow) x265amd_rdo_thread();
    if (!t) return X265AMD_ENOMEM;
    const Geo g(6);                  // slots sized for the largest CU (64x64)
    for (auto& r : t->req)
    {
        r.in = (uint8_t*)malloc(2 * g.pix() * s->pix);
        r.out = (uint8_t*)malloc(out_bytes(g, s->pix));
        if (!r.in || !r.out)
        {
            for (auto& q : t->req) { free(q.in); free(q.out); }
            delete t;
            return X265AMD_ENOMEM;
        }
    }
    {
        std::lock_guard<std::mutex> lk(s->mu);
        if ((int)s->threads.size() >= s->cfg.max_threads)
        {
            for (auto& q : t->req) { free(q.in); free(q.out); }
            delete t;
            return X265AMD_ENOMEM;
        }
        t->index = (int)s->threads.size();
        s->threads.push_back(t);
    }
    tls.push_back({ s, s->id, t });
    *out = t;
    return 0;
}

int reserve(x265amd_rdo_launcher* L, size_t bytes)
{
    if (bytes <= L->cap) return 0;
    (void)hipStreamSynchronize(L->st);
    (void)hipFree(L->dev);
    (void)hipHostFree(L->host);
    L->dev = L->host = nullptr;
    L->cap = 0;
    bytes += bytes / 2;
    if (hipMalloc((void**)&L->dev, bytes) != hipSuccess ||
        hipHostMalloc((void**)&L->host, bytes, hipHostMallocDefault) != hipSuccess)
        return X265AMD_ENOMEM;
    L->cap = bytes;
    return 0;
}

// Staging of one batch (device and pinned host alike, byte offsets):
//   per request: [in: fenc Y Cb Cr, pred Y Cb Cr][out: recon, resi, coeff, num_sig, psy_pred, psy_rec]
//   then the job descriptors: per TU fenc / pred / resi / coeff / recon offsets (int64) and qp (uint8), per
//   8x8 block the fenc / pred / recon offsets (int64)
// The inputs, offsets and (ride-along) outputs go up in one copy, the outputs come back in one copy per
// request run (they are contiguous per request).
struct Batch
{
    std::vector<x265amd_rdo_req*> reqs;
    std::vector<size_t> rbase;       // request k's staging offset
    size_t total = 0;
};

struct JobTables
{
    // per TU-pipeline batch (one per (CU size, luma / chroma))
    std::vector<int64_t> fo, po, ro, co, xo;  // fenc, pred, resi, coeff, recon element offsets
    std::vector<uint8_t> qp;
    // per 8x8 psy batch (one per (CU size, luma / chroma)): a = fenc, b = pred or recon
    std::vector<int64_t> pa, pb, pr;
    std::vector<int64_t> sig, psyp, psyr;     // element offsets of the outputs (num_sig uint32, psy int32)
};

void launcher_main(x265amd_rdo* s, x265amd_rdo_launcher* L)
{
    (void)hipSetDevice(s->cfg.device);
    std::vector<x265amd_rdo_req*> take;
    for (;;)
    {
        {
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
            if (s->rq.empty()) return;
            take.swap(s->rq);
            s->rq.clear();
        }
        const double t_take = now_s();
        const size_t pix = s->pix;
        // staging: requests, then the descriptor tables of every (CU size, plane class)
        size_t total = 0;
        std::vector<size_t> rbase(take.size());
        for (size_t k = 0; k < take.size(); k++)
        {
            const Geo g(take[k]->cu.log2_cu);
            rbase[k] = total;
            total += (2 * g.pix() * pix + out_bytes(g, pix) + 255) & ~(size_t)255;
        }
        // jobs per CU size (log2 4..6) and class (0 luma, 1 chroma)
        JobTables jt[3][2];
        for (size_t k = 0; k < take.size(); k++)
        {
            const x265amd_rdo_cu& cu = take[k]->cu;
            const Geo g(cu.log2_cu);
            const int64_t R = (int64_t)(rbase[k] / pix);              // request base in pixel elements
            const int64_t in_f[3] = { R, R + (int64_t)g.pix_y, R + (int64_t)(g.pix_y + g.pix_c) };
            const int64_t in_p = (int64_t)g.pix();                    // pred planes follow fenc planes
            const size_t ob = rbase[k] + 2 * g.pix() * pix;           // output base, bytes
            const int64_t rec0 = (int64_t)(ob / pix);
            const size_t resi_b = ob + g.pix() * pix, coeff_b = resi_b + 2 * g.pix();
            const size_t sig_b = coeff_b + 2 * g.pix(), psyp_b = sig_b + 4 * (size_t)g.tus();
            const size_t psyr_b = psyp_b + 4 * (size_t)g.blocks();
            // the request's output offsets must be element aligned for every type
            for (int p = 0; p < 3; p++)
            {
                const int cls = p > 0;
                JobTables& J = jt[cu.log2_cu - 4][cls];
                const int w = p ? g.cc : g.c, tl = p ? g.tlc : g.tl, n = 1 << tl;
                const int64_t poff = p == 0 ? 0 : (p == 1 ? (int64_t)g.pix_y : (int64_t)(g.pix_y + g.pix_c));
                const int ntu = p ? g.ntuc : g.ntu, nbl = p ? g.nbc : g.nb;
                const int tu0 = p == 0 ? 0 : (p == 1 ? g.ntu : g.ntu + g.ntuc);
                const int bl0 = p == 0 ? 0 : (p == 1 ? g.nb : g.nb + g.nbc);
                for (int t = 0; t < ntu; t++)
                {
                    const int tx = (t % (w >> tl)) * n, ty = (t / (w >> tl)) * n;
                    const int64_t o = (int64_t)ty * w + tx;
                    J.fo.push_back(in_f[p] + o);
                    J.po.push_back(in_f[p] + in_p + o);
                    J.xo.push_back(rec0 + poff + o);
                    J.ro.push_back((int64_t)(resi_b / 2) + poff + o);
                    J.co.push_back((int64_t)(coeff_b / 2) + poff + (int64_t)t * n * n);
                    J.sig.push_back((int64_t)(sig_b / 4) + tu0 + t);
                    J.qp.push_back(cu.qp[p]);
                }
                for (int b = 0; b < nbl; b++)
                {
                    const int64_t o = (int64_t)(b / (w >> 3)) * 8 * w + (b % (w >> 3)) * 8;
                    J.pa.push_back(in_f[p] + o);
                    J.pb.push_back(in_f[p] + in_p + o);
                    J.pr.push_back(rec0 + poff + o);
                    J.psyp.push_back((int64_t)(psyp_b / 4) + bl0 + b);
                    J.psyr.push_back((int64_t)(psyr_b / 4) + bl0 + b);
                }
            }
        }
        // descriptor tables after the requests
        size_t tab_base = total;
        for (auto& a : jt)
            for (auto& J : a)
            {
                const size_t nt = J.fo.size(), nb = J.pa.size();
                if (!nt) continue;
                auto r256 = [](size_t b) { return (b + 255) & ~(size_t)255; };
                // descriptors + qp, the num_sig scratch run, the two psy scratch runs (see the fill below)
                total += r256(8 * 5 * nt + 8 * 3 * nb + nt) + r256(4 * nt) + 2 * r256(4 * nb);
            }
        int rc = reserve(L, total);
        int njobs = 0, nblocks = 0;
        std::vector<x265amd_tu_batch> tub;
        std::vector<x265amd_cmp_batch> psy;
        if (!rc)
        {
            uint8_t* H = L->host;
            for (size_t k = 0; k < take.size(); k++)
                memcpy(H + rbase[k], take[k]->in, 2 * Geo(take[k]->cu.log2_cu).pix() * pix);
            size_t o = tab_base;
            for (int z = 0; z < 3; z++)
                for (int cls = 0; cls < 2; cls++)
                {
                    JobTables& J = jt[z][cls];
                    const size_t nt = J.fo.size(), nb = J.pa.size();
                    if (!nt) continue;
                    auto put = [&](const std::vector<int64_t>& v) {
                        memcpy(H + o, v.data(), 8 * v.size());
                        const int64_t* d = (const int64_t*)(L->dev + o);
                        o += 8 * v.size();
                        return d;
                    };
                    const int64_t *fo = put(J.fo), *po = put(J.po), *ro = put(J.ro), *co = put(J.co), *xo = put(J.xo);
                    const int64_t *pa = put(J.pa), *pb = put(J.pb), *pr = put(J.pr);
                    memcpy(H + o, J.qp.data(), nt);
                    const uint8_t* qp = L->dev + o;
                    o = (o + nt + 255) & ~(size_t)255;
                    const int w = (1 << (z + 4)) >> cls;              // plane width of this CU size and class
                    const int tl = cls ? Geo(z + 4).tlc : Geo(z + 4).tl;
                    // num_sig: the TUs of one (CU size, class) are not contiguous in the outputs, so the
                    // kernel writes them into a scratch run (the descriptors' tail) and the host scatters
                    x265amd_tu_batch b{};
                    b.log2_size = tl;
                    b.n = (int)nt;
                    b.is_luma = !cls;
                    b.is_intra = 0;
                    b.i_slice = 0;
                    b.sign_hide = s->cfg.sign_hide;
                    b.fenc = L->dev;
                    b.fenc_stride = w;
                    b.fenc_off = fo;
                    b.pred = L->dev;
                    b.pred_stride = w;
                    b.pred_off = po;
                    b.resi = (int16_t*)L->dev;
                    b.resi_stride = w;
                    b.resi_off = ro;
                    b.coeff = (int16_t*)L->dev;
                    b.coeff_off = co;
                    b.recon = L->dev;
                    b.recon_stride = w;
                    b.recon_off = xo;
                    b.num_sig = (uint32_t*)(L->dev + o);
                    b.qp = qp;
                    b.scan = nullptr;
                    o += (4 * nt + 255) & ~(size_t)255;
                    tub.push_back(b);
                    njobs += (int)nt;
                    nblocks += (int)nb;
                    psy.push_back({ 8, 8, (int)nb, L->dev, w, pa, L->dev, w, pb, nullptr });
                    psy.push_back({ 8, 8, (int)nb, L->dev, w, pa, L->dev, w, pr, nullptr });
                    // psy outputs likewise into scratch runs
                    psy[psy.size() - 2].out = L->dev + o;
                    o += (4 * nb + 255) & ~(size_t)255;
                    psy.back().out = L->dev + o;
                    o += (4 * nb + 255) & ~(size_t)255;
                }
            if (o > L->cap) rc = X265AMD_ENOMEM;                      // (the reserve above sized for this)
            else total = o;
        }
        if (!rc) rc = (int)hipMemcpyAsync(L->dev, L->host, total, hipMemcpyHostToDevice, L->st);
        if (!rc) rc = (int)hipEventRecord(L->k0, L->st);
        if (!rc) rc = x265amd_tu_pipeline((int)s->cfg.depth, (int)tub.size(), tub.data(), L->st);
        // the psy energies of fenc against the coded reconstruction need the TU kernels' recon: same stream
        if (!rc) rc = x265amd_pixelcmp_grouped(X265AMD_PSY, (int)s->cfg.depth, (int)psy.size(), psy.data(), L->st);
        if (!rc) rc = (int)hipEventRecord(L->k1, L->st);
        if (!rc) rc = (int)hipMemcpyAsync(L->host, L->dev, total, hipMemcpyDeviceToHost, L->st);
        if (!rc) rc = (int)hipEventRecord(L->done, L->st);
        if (!rc) rc = (int)hipEventSynchronize(L->done);
        float kms = 0;
        if (!rc) (void)hipEventElapsedTime(&kms, L->k0, L->k1);
        // publish: every request's outputs (recon, resi, coeff) are contiguous in its staging; num_sig and the
        // psy energies are scattered back from the per-batch scratch runs
        if (!rc)
        {
            for (size_t k = 0; k < take.size(); k++)
            {
                const Geo g(take[k]->cu.log2_cu);
                memcpy(take[k]->out, L->host + rbase[k] + 2 * g.pix() * pix, out_bytes(g, pix));
            }
            size_t ti = 0, pi = 0;
            for (int z = 0; z < 3; z++)
                for (int cls = 0; cls < 2; cls++)
                {
                    JobTables& J = jt[z][cls];
                    if (J.fo.empty()) continue;
                    const uint32_t* sig = (const uint32_t*)(L->host + ((const uint8_t*)tub[ti].num_sig - L->dev));
                    const int32_t* pp = (const int32_t*)(L->host + ((const uint8_t*)psy[pi].out - L->dev));
                    const int32_t* pr = (const int32_t*)(L->host + ((const uint8_t*)psy[pi + 1].out - L->dev));
                    ti++;
                    pi += 2;
                    // destination: element offsets into the staging, mapped to each request's output copy
                    for (size_t j = 0; j < J.sig.size(); j++)
                        *(uint32_t*)(L->host + 4 * J.sig[j]) = sig[j];
                    for (size_t j = 0; j < J.psyp.size(); j++)
                    {
                        *(int32_t*)(L->host + 4 * J.psyp[j]) = pp[j];
                        *(int32_t*)(L->host + 4 * J.psyr[j]) = pr[j];
                    }
                }
            // the scattered scalars sit inside each request's staging output region: copy those again
            for (size_t k = 0; k < take.size(); k++)
            {
                const Geo g(take[k]->cu.log2_cu);
                const size_t ob = rbase[k] + 2 * g.pix() * pix, sc = g.pix() * pix + 4 * g.pix();
                memcpy(take[k]->out + sc, L->host + ob + sc, out_bytes(g, pix) - sc);
            }
        }
        const double t_done = now_s();
        double qdelay = 0;
        bool wake;
        {
            std::lock_guard<std::mutex> g(s->dmu);
            for (auto* r : take)
            {
                qdelay += t_take - r->t_post;
                r->rc = rc;
                if (!rc) set_result(r, pix);
                r->state.store(2, std::memory_order_release);
            }
            wake = s->dsleepers > 0;
        }
        if (wake) s->dcv.notify_all();
        if (rc) record(rc);
        {
            std::lock_guard<std::mutex> g(s->smu);
            s->st.batches++;
            s->st.requests += (int64_t)take.size();
            s->st.tus += njobs;
            s->st.blocks += nblocks;
            s->st.kernel_ms += kms;
            s->st.batch_ms += 1e3 * (t_done - t_take);
            s->st.queue_ms += 1e3 * qdelay;
            if ((int64_t)take.size() > s->st.max_requests_per_batch) s->st.max_requests_per_batch = (int64_t)take.size();
        }
        take.clear();
    }
}

int getenv_int(const char* name, int dflt)
{
    const char* e = getenv(name);
    return e && *e ? atoi(e) : dflt;
}

} // namespace

extern "C" int x265amd_rdo_create(const x265amd_rdo_config* cfg, x265amd_rdo** out)
{
    if (!cfg || !out) return X265AMD_EINVAL;
    *out = nullptr;
    if ((cfg->depth != 8 && cfg->depth != 10 && cfg->depth != 12) || cfg->launchers < 0 || cfg->launchers > 8 ||
        cfg->max_threads <= 0)
        return X265AMD_EINVAL;
    auto* s = new (std::nothrow) x265amd_rdo();
    if (!s) return record(X265AMD_ENOMEM);
    s->cfg = *cfg;
    s->id = g_next_id.fetch_add(1);
    s->pix = cfg->depth > 8 ? 2 : 1;
    s->spin_us = getenv_int("X265AMD_RDO_SPIN_US", 50);
    s->timing = getenv_int("X265AMD_RDO_TIMING", 0) != 0 && cfg->launchers == 0;
    s->server = getenv_int("X265AMD_RDO_SERVER", 0) != 0 && cfg->launchers == 0;
    s->srv_probe = s->server && getenv_int("X265AMD_RDO_SERVER_PROBE", 0) != 0;
    s->srv_timing = s->server && getenv_int("X265AMD_RDO_SERVER_TIMING", 0) != 0;
    // 16 workgroups: fewer queue the CUs longer, more slow the motion-search kernel running beside them
    // (8 / 12 / 16 / 20 / 24 / 32: 11.0 / 11.5 / 12.3-12.5 / 12.3 / 12.1 / 11.7 fps at 2160p, profiles/r06/
    // rdo_server_ab.jsonl calls r06zh-r06zi)
    s->srv_nwg = getenv_int("X265AMD_RDO_SERVER_WG", 32);   // (16 until the SAO requests joined)
    s->srv_nwg = s->srv_nwg < 4 ? 4 : (s->srv_nwg > 256 ? 256 : s->srv_nwg);
    if (s->server) s->timing = false;
    s->yield_us = getenv_int("X265AMD_RDO_YIELD_US", 5000);
    s->idle_us = getenv_int("X265AMD_RDO_IDLE_US", 500);
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess || (cur != cfg->device && hipSetDevice(cfg->device) != hipSuccess))
    {
        delete s;
        return record(X265AMD_ENODEV);
    }
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    for (int i = 0; i < cfg->launchers; i++)
    {
        auto* L = new (std::nothrow) x265amd_rdo_launcher();
        if (!L || hipStreamCreateWithPriority(&L->st, hipStreamNonBlocking, hi) != hipSuccess ||
            hipEventCreateWithFlags(&L->done, hipEventBlockingSync | hipEventDisableTiming) != hipSuccess ||
            hipEventCreate(&L->k0) != hipSuccess || hipEventCreate(&L->k1) != hipSuccess)
        {
            delete L;
            x265amd_rdo_destroy(s);
            return record(X265AMD_ENOMEM);
        }
        s->launchers.push_back(L);
    }
    for (auto* L : s->launchers) L->th = std::thread(launcher_main, s, L);
    if (cur != cfg->device) (void)hipSetDevice(cur);
    *out = s;
    return 0;
}

extern "C" void x265amd_rdo_destroy(x265amd_rdo* s)
{
    if (!s) return;
    {
        std::lock_guard<std::mutex> lk(s->qmu);
        s->stop = true;
        s->stop_flag.store(true);
    }
    s->qcv.notify_all();
    for (auto* L : s->launchers)
        if (L->th.joinable()) L->th.join();
    for (auto* L : s->launchers)
    {
        if (L->st) (void)hipStreamSynchronize(L->st);
        (void)hipFree(L->dev);
        (void)hipHostFree(L->host);
        if (L->st) (void)hipStreamDestroy(L->st);
        if (L->done) (void)hipEventDestroy(L->done);
        if (L->k0) (void)hipEventDestroy(L->k0);
        if (L->k1) (void)hipEventDestroy(L->k1);
        delete L;
    }
    for (auto* t : s->threads) free_thread(t);
    {
        std::lock_guard<std::mutex> rl(g_srv_reg_mu);
        for (size_t i = 0; i < g_srv_reg.size(); i++)
            if (g_srv_reg[i] == s) { g_srv_reg[i] = g_srv_reg.back(); g_srv_reg.pop_back(); break; }
    }
    if (s->srv_st)
    {
        // the server serves what is pending and leaves; then its region goes
        if (s->srv_ctl) set_stop(s, 1u);
        (void)hipStreamSynchronize(s->srv_st);
        (void)hipStreamDestroy(s->srv_st);
    }
    if (s->srv_timing && s->srv_stamped)
        fprintf(stderr, "[x265rdo] server phases over %lld requests (us each): job %.2f, luma TUs %.2f, chroma TUs %.2f, "
                        "psy %.2f, release %.2f\n", (long long)s->srv_stamped, s->srv_phase[0] / s->srv_stamped,
                s->srv_phase[1] / s->srv_stamped, s->srv_phase[2] / s->srv_stamped, s->srv_phase[3] / s->srv_stamped,
                s->srv_phase[4] / s->srv_stamped);
    if (s->srv_host) (void)hipHostFree(s->srv_host);
    if (s->srv_ctl) (void)hipHostFree(s->srv_ctl);
    if (s->srv_in) (void)hipFree(s->srv_in);
    delete s;
}

namespace {

// the completion flag written by a one-lane kernel instead of hipStreamWriteValue32 (X265AMD_RDO_FLAG=kernel:
// a form rocprofv3's kernel trace can follow)
__global__ void k_rdo_flag(uint32_t* f)
{
    if (threadIdx.x == 0) __hip_atomic_store(f, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

bool flag_kernel()
{
    static const int v = [] { const char* e = getenv("X265AMD_RDO_FLAG"); return e && !strcmp(e, "kernel") ? 1 : 0; }();
    return v != 0;
}

// the request of slot k for the resident server, its job written: its sequence word (release: the inputs,
// descriptors and job are in memory before the server can see the new sequence number), the doorbell
int server_publish(x265amd_rdo* s, x265amd_rdo_thread* t, int k, x265amd::RdoJob* job)
{
    x265amd_rdo_req* r = &t->req[k];
    r->seq++;
    r->want = r->seq;
    const int wg = (t->index * kSlots + k) % s->srv_nwg;
    if (s->srv_in)
    {
        // device memory through the BAR is write-combined: fence the inputs and job before the sequence
        // word, and the sequence word before the doorbell (never read back: BAR reads are slow)
        __builtin_ia32_sfence();
        *(volatile uint32_t*)&job->seq = r->seq;
        __builtin_ia32_sfence();
        *(volatile uint32_t*)&s->srv_vctl[x265amd::kRdoBellWord + wg] = s->srv_bells[wg].fetch_add(1) + 1;
        __builtin_ia32_sfence();
    }
    else
    {
        __atomic_store_n(&job->seq, r->seq, __ATOMIC_RELEASE);
        // ring the doorbell of the workgroup that polls this slot
        __atomic_fetch_add(&s->srv_ctl[x265amd::kRdoBellWord + wg], 1u, __ATOMIC_RELEASE);
    }
    return ensure_server(s, false);
}

// direct mode: stage the CU in the slot's mapped region and enqueue its kernels on the thread's stream
int direct_post(x265amd_rdo* s, x265amd_rdo_thread* t, int k, const x265amd_rdo_cu* cu)
{
    x265amd_rdo_req* r = &t->req[k];
    const size_t pix = s->pix;
    const Geo g(cu->log2_cu);
    uint8_t* H = t->host + (size_t)k * t->region;
    uint8_t* D = t->hdev + (size_t)k * t->region;
    // where the inputs and descriptors go: the slot itself, or (server with device-memory input slots) the
    // slot's input area in device memory, which the host writes through the BAR at the same address
    uint8_t* I = H;
    uint8_t* DI = D;
    if (s->server && s->srv_in) I = DI = s->srv_in + (size_t)(t->index * kSlots + k) * s->srv_in_region;
    // inputs: fenc Y Cb Cr then pred Y Cb Cr, packed
    uint8_t* d = I;
    for (int src = 0; src < 2; src++)
        for (int p = 0; p < 3; p++)
        {
            const int w = p ? g.cc : g.c;
            const uint8_t* a = (const uint8_t*)(src ? cu->pred[p] : cu->fenc[p]);
            const intptr_t st = (src ? cu->pred_stride[p] : cu->fenc_stride[p]) * (intptr_t)pix;
            for (int y = 0; y < w; y++, d += w * pix) memcpy(d, a + y * st, w * pix);
        }
    const size_t ob = x265amd::rdo_out_at(pix);              // outputs (the out_bytes layout, set_result)
    const size_t resi_b = ob + g.pix() * pix, coeff_b = resi_b + 2 * g.pix();
    const size_t sig_b = coeff_b + 2 * g.pix(), psyp_b = sig_b + 4 * (size_t)g.tus();
    const size_t psyr_b = psyp_b + 4 * (size_t)g.blocks();
    size_t o = x265amd::rdo_desc_at(pix);                       // descriptors (rdojob.h slot layout)
    r->out = H + ob;
    volatile uint32_t* flag = (volatile uint32_t*)(H + t->region - 64);
    if (!s->server) *flag = 0;
    x265amd_tu_batch tb[2];
    x265amd_cmp_batch pb[4];
    for (int cls = 0; cls < 2; cls++)
    {
        const int w = cls ? g.cc : g.c, tl = cls ? g.tlc : g.tl, n = 1 << tl;
        const int nt = cls ? 2 * g.ntuc : g.ntu, nb = cls ? 2 * g.nbc : g.nb;
        int64_t* fo = (int64_t*)(I + o);
        int64_t* po = fo + nt;
        int64_t* ro = po + nt;
        int64_t* co = ro + nt;
        int64_t* xo = co + nt;
        int64_t* pa = xo + nt;
        int64_t* pbb = pa + nb;
        int64_t* pr = pbb + nb;
        uint8_t* qp = (uint8_t*)(pr + nb);
        const size_t used = 8 * (5 * (size_t)nt + 3 * (size_t)nb) + (size_t)nt;
        int j = 0, b = 0;
        for (int p = cls ? 1 : 0; p < (cls ? 3 : 1); p++)
        {
            const int64_t poff = p == 0 ? 0 : (p == 1 ? (int64_t)g.pix_y : (int64_t)(g.pix_y + g.pix_c));
            const int per = w >> tl, ntu = per * per, nbl = (w >> 3) * (w >> 3);
            for (int q = 0; q < ntu; q++, j++)
            {
                const int64_t e = (int64_t)((q / per) * n) * w + (q % per) * n;
                fo[j] = poff + e;
                po[j] = (int64_t)g.pix() + poff + e;
                xo[j] = (int64_t)(ob / pix) + poff + e;
                ro[j] = (int64_t)(resi_b / 2) + poff + e;
                co[j] = (int64_t)(coeff_b / 2) + poff + (int64_t)q * n * n;
                qp[j] = cu->qp[p];
            }
            for (int q = 0; q < nbl; q++, b++)
            {
                const int64_t e = (int64_t)(q / (w >> 3)) * 8 * w + (q % (w >> 3)) * 8;
                pa[b] = poff + e;
                pbb[b] = (int64_t)g.pix() + poff + e;
                pr[b] = (int64_t)(ob / pix) + poff + e;
            }
        }
        auto dv = [&](const void* hp) { return (const void*)(DI + ((const uint8_t*)hp - I)); };
        x265amd_tu_batch& B = tb[cls];
        B = x265amd_tu_batch{};
        B.log2_size = tl;
        B.n = nt;
        B.is_luma = !cls;
        B.sign_hide = s->cfg.sign_hide;
        B.fenc = DI;
        B.fenc_stride = w;
        B.fenc_off = (const int64_t*)dv(fo);
        B.pred = DI;
        B.pred_stride = w;
        B.pred_off = (const int64_t*)dv(po);
        B.resi = (int16_t*)D;
        B.resi_stride = w;
        B.resi_off = (const int64_t*)dv(ro);
        B.coeff = (int16_t*)D;
        B.coeff_off = (const int64_t*)dv(co);
        B.recon = D;
        B.recon_stride = w;
        B.recon_off = (const int64_t*)dv(xo);
        // num_sig and the psy energies of one class are contiguous in the outputs (luma, then Cb, then Cr)
        B.num_sig = (uint32_t*)(D + sig_b) + (cls ? g.ntu : 0);
        B.qp = (const uint8_t*)dv(qp);
        pb[2 * cls] = { 8, 8, nb, DI, w, (const int64_t*)dv(pa), DI, w, (const int64_t*)dv(pbb),
                        (int32_t*)(D + psyp_b) + (cls ? g.nb : 0) };
        pb[2 * cls + 1] = { 8, 8, nb, DI, w, (const int64_t*)dv(pa), D, w, (const int64_t*)dv(pr),
                            (int32_t*)(D + psyr_b) + (cls ? g.nb : 0) };
        o = (o + used + 255) & ~(size_t)255;
    }
    if (o > ob || ob + out_bytes(g, pix) + x265amd::kRdoJobFromEnd > t->region) return X265AMD_ENOMEM;
    if (s->server)
    {
        x265amd::RdoJob* job = (x265amd::RdoJob*)(s->srv_in ? I + x265amd::rdo_out_at(pix)
                                                             : H + t->region - x265amd::kRdoJobFromEnd);
        for (int c = 0; c < 2; c++) job->tu[c] = tb[c];
        for (int c = 0; c < 4; c++) job->psy[c] = pb[c];
        job->kind = 0;
        job->pad[0] = (uint32_t)g.blocks();        // the 8x8 SSEs go 2 * blocks int32 after each psy energy
        return server_publish(s, t, k, job);
    }
    r->want = 1;
    int rc = s->timing ? (int)hipEventRecord(t->ev[k][0], t->st) : 0;
    if (!rc) rc = x265amd_tu_pipeline((int)s->cfg.depth, 2, tb, t->st);
    if (!rc) rc = x265amd_pixelcmp_grouped(X265AMD_PSY, (int)s->cfg.depth, 4, pb, t->st);
    if (!rc && s->timing) rc = (int)hipEventRecord(t->ev[k][1], t->st);
    if (!rc && flag_kernel())
    {
        hipLaunchKernelGGL(k_rdo_flag, dim3(1), dim3(64), 0, t->st, (uint32_t*)(D + t->region - 64));
        rc = (int)hipGetLastError();
    }
    else if (!rc)
        rc = (int)hipStreamWriteValue32(t->st, D + t->region - 64, 1, 0);
    return rc;
}

int direct_wait(x265amd_rdo* s, x265amd_rdo_thread* t, int k)
{
    volatile uint32_t* flag = (volatile uint32_t*)(t->host + (size_t)k * t->region + t->region - 64);
    const uint32_t want = t->req[k].want;
    const double t0 = now_s();
    const double spin_until = t0 + 1e-6 * s->spin_us;
    double next_check = t0 + 0.02;
    while (*flag != want)
    {
        const double now = now_s();
        if (now < spin_until) { __builtin_ia32_pause(); continue; }
        sched_yield();
        // a server stopped for a device-synchronising call is relaunched when the call is over
        if (s->server && s->srv_launched.load(std::memory_order_acquire) < 0 &&
            g_quiesce.load(std::memory_order_acquire) == 0)
            if (int rc = ensure_server(s, true)) return rc;
        if (now < next_check) continue;
        next_check = now + 0.02;
        // a stream that failed never writes the flag; a server that left (its lifetime over with nothing
        // relaunched since) is relaunched
        const hipError_t q = hipStreamQuery(s->server ? s->srv_st : t->st);
        if (q != hipSuccess && q != hipErrorNotReady) return (int)q;
        if (s->server && q == hipSuccess)
            if (int rc = ensure_server(s, true)) return rc;
        // a request no server picked up for a second is an error (sticky; the CU is coded on the host),
        // never an endless wait
        if (s->server && now - t0 > 1.0)
        {
            s->srv_broken.store(true);
            return (int)hipErrorLaunchTimeOut;
        }
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    return 0;
}

} // namespace

extern "C" int x265amd_rdo_post(x265amd_rdo* s, const x265amd_rdo_cu* cu, int* ticket)
{
    if (!s || !cu || !ticket || cu->log2_cu < 4 || cu->log2_cu > 6) return X265AMD_EINVAL;
    for (int p = 0; p < 3; p++)
        if (!cu->fenc[p] || !cu->pred[p]) return X265AMD_EINVAL;
    x265amd_rdo_thread* t;
    if (int rc = thread_ctx(s, &t)) return rc;
    int k = 0;
    while (k < kSlots && t->req[k].state.load(std::memory_order_acquire) != 0) k++;
    if (k == kSlots) return X265AMD_ENOMEM;                       // caller codes the CU on the host
    x265amd_rdo_req* r = &t->req[k];
    r->cu = *cu;
    if (s->launchers.empty())
    {
        if (s->server && (cu->log2_cu < 5 || s->srv_broken.load(std::memory_order_relaxed)))
            return X265AMD_ENOMEM;                                  // (the server codes 32x32 / 64x64 CUs)
        if (s->srv_probe)
        {
            // (measurement: the server runs and is relaunched, every CU is coded on the host)
            if (!server_setup(s)) (void)ensure_server(s, false);
            return X265AMD_ENOMEM;
        }
        if (int rc = direct_setup(s, t)) return rc == X265AMD_ENOMEM ? rc : record(rc);
        r->t_post = now_s();
        const int rc = direct_post(s, t, k, cu);
        {
            // direct mode: the "queueing" counter is the worker's own posting time (staging + launches)
            std::lock_guard<std::mutex> g(s->smu);
            s->st.queue_ms += 1e3 * (now_s() - r->t_post);
        }
        r->rc = rc;
        r->state.store(1, std::memory_order_release);
        *ticket = k;
        if (rc) return record(rc);
        return 0;
    }
    const Geo g(cu->log2_cu);
    // pack fenc and pred planes (stride = plane width): the caller's buffers may change once this returns
    uint8_t* d = r->in;
    for (int src = 0; src < 2; src++)
        for (int p = 0; p < 3; p++)
        {
            const int w = p ? g.cc : g.c;
            const uint8_t* a = (const uint8_t*)(src ? cu->pred[p] : cu->fenc[p]);
            const intptr_t st = (src ? cu->pred_stride[p] : cu->fenc_stride[p]) * (intptr_t)s->pix;
            for (int y = 0; y < w; y++, d += w * s->pix) memcpy(d, a + y * st, w * s->pix);
        }
    r->rc = 0;
    r->t_post = now_s();
    r->state.store(1, std::memory_order_release);
    {
        std::lock_guard<std::mutex> lk(s->qmu);
        s->rq.push_back(r);
    }
    s->queued.fetch_add(1, std::memory_order_acq_rel);
    if (s->qsleepers.load(std::memory_order_acquire) > 0) s->qcv.notify_one();
    *ticket = k;
    return 0;
}

extern "C" int x265amd_rdo_wait(x265amd_rdo* s, int ticket, const x265amd_rdo_result** out)
{
    if (!s || ticket < 0 || ticket >= kSlots || !out) return X265AMD_EINVAL;
    x265amd_rdo_thread* t;
    if (int rc = thread_ctx(s, &t)) return rc;
    x265amd_rdo_req* r = &t->req[ticket];
    if (r->state.load(std::memory_order_acquire) == 0) return X265AMD_EINVAL;
    const double t0 = now_s();
    bool slept = false;
    if (s->launchers.empty())
    {
        int rc = r->rc ? r->rc : direct_wait(s, t, ticket);
        if (!rc) set_result(r, s->pix, s->server);
        if (!rc && s->server && s->srv_timing)
        {
            const uint64_t* st = (const uint64_t*)(t->host + (size_t)ticket * t->region + t->region -
                                                   x265amd::kRdoStampsFromEnd);
            std::lock_guard<std::mutex> g(s->smu);
            for (int p = 0; p < 5; p++) s->srv_phase[p] += 1e-2 * (double)(st[p + 1] - st[p]);   // 100 MHz -> us
            s->srv_stamped++;
        }
        if (rc && s->server)
        {
            // a server request that was not served may still be: its slot is never posted to again
            r->state.store(3, std::memory_order_release);
            return record(rc);
        }
        float span = 0.f;
        if (!rc && s->timing && hipEventSynchronize(t->ev[ticket][1]) == hipSuccess)
            (void)hipEventElapsedTime(&span, t->ev[ticket][0], t->ev[ticket][1]);
        r->state.store(2, std::memory_order_release);
        std::lock_guard<std::mutex> g(s->smu);
        s->st.waits++;
        s->st.requests++;
        s->st.batches++;
        s->st.wait_ms += 1e3 * (now_s() - t0);
        s->st.batch_ms += 1e3 * (now_s() - r->t_post);
        s->st.kernel_ms += span;
        if (rc) return record(rc);
        *out = &r->res;
        return 0;
    }
    if (r->state.load(std::memory_order_acquire) != 2)
    {
        const double spin_until = t0 + 1e-6 * s->spin_us, yield_until = t0 + 1e-6 * s->yield_us;
        while (r->state.load(std::memory_order_acquire) != 2 && now_s() < spin_until) __builtin_ia32_pause();
        while (r->state.load(std::memory_order_acquire) != 2 && now_s() < yield_until) sched_yield();
        if (r->state.load(std::memory_order_acquire) != 2)
        {
            std::unique_lock<std::mutex> lk(s->dmu);
            s->dsleepers++;
            s->dcv.wait(lk, [&] { return r->state.load(std::memory_order_acquire) == 2; });
            s->dsleepers--;
            slept = true;
        }
    }
    {
        std::lock_guard<std::mutex> g(s->smu);
        s->st.waits++;
        s->st.waits_blocked += slept;
        s->st.wait_ms += 1e3 * (now_s() - t0);
    }
    if (r->rc) return record(r->rc);
    *out = &r->res;
    return 0;
}

extern "C" int x265amd_rdo_release(x265amd_rdo* s, int ticket)
{
    if (!s || ticket < 0 || ticket >= kSlots) return X265AMD_EINVAL;
    x265amd_rdo_thread* t;
    if (int rc = thread_ctx(s, &t)) return rc;
    x265amd_rdo_req* r = &t->req[ticket];
    // a request still queued is left alone: its launcher completes it and it stays reserved until waited for
    int done = 2;
    if (!r->state.compare_exchange_strong(done, 0)) return X265AMD_EINVAL;
    return 0;
}

extern "C" int x265amd_rdo_sao_stats(x265amd_rdo* s, const x265amd_rdo_sao_ctu* q, int32_t* stats, int32_t* count)
{
    if (!s || !q || !stats || !count) return X265AMD_EINVAL;
    for (int p = 0; p < 3; p++)
        if (!q->rec[p] || !q->fenc[p]) return X265AMD_EINVAL;
    // the server's staged bytes hold an 8-bit 4:2:0 64x64 CTU's windows (below); anything else stays on the host
    if (!s->launchers.empty() || !s->server || s->srv_probe || s->pix != 1 || q->ctu_log2 != 6 ||
        q->chroma_format != 1 || q->cx < 0 || q->cy < 0 || q->cx * 64 >= q->width || q->cy * 64 >= q->height ||
        s->srv_broken.load(std::memory_order_relaxed))
        return X265AMD_ENOMEM;
    x265amd_rdo_thread* t;
    if (int rc = thread_ctx(s, &t)) return rc;
    int k = 0;
    while (k < kSlots && t->req[k].state.load(std::memory_order_acquire) != 0) k++;
    if (k == kSlots) return X265AMD_ENOMEM;
    if (int rc = direct_setup(s, t)) return rc == X265AMD_ENOMEM ? rc : record(rc);
    if (!s->srv_in) return X265AMD_ENOMEM;
    x265amd_rdo_req* r = &t->req[k];
    r->t_post = now_s();
    uint8_t* I = s->srv_in + (size_t)(t->index * kSlots + k) * s->srv_in_region;
    uint8_t* H = t->host + (size_t)k * t->region;
    uint8_t* D = t->hdev + (size_t)k * t->region;
    // staged bytes (tu.hip k_rdo_server, kind 1): per plane the deblocked window — one row above to one row below
    // the CTU, 4 pixels left to 12 right (rows 16-byte multiples, so every strip's p - 4 is 8-byte aligned) — then
    // the source blocks, packed
    x265amd::RdoSaoJob js{};
    js.w = q->width;
    js.h = q->height;
    js.ctu_log2 = 6;
    js.nd = q->non_deblocked;
    js.cx = q->cx;
    js.cy = q->cy;
    js.hs = js.vs = 1;
    size_t o = 0;
    for (int p = 0; p < 3; p++)
    {
        const int cs = p ? 32 : 64, ww = cs + 16;
        const int ph = p ? q->height >> 1 : q->height, y0 = q->cy * cs;
        const int ch = y0 + cs < ph ? cs : ph - y0;
        const uint8_t* src = (const uint8_t*)q->rec[p] - q->rec_stride[p] - 4;
        for (int y = 0; y < ch + 2; y++) memcpy(I + o + (size_t)y * ww, src + y * q->rec_stride[p], ww);
        js.rec_at[p] = (int64_t)(o + ww + 4);
        js.rs[p] = ww;
        o = (o + (size_t)ww * (cs + 2) + 15) & ~(size_t)15;
    }
    for (int p = 0; p < 3; p++)
    {
        const int cs = p ? 32 : 64;
        const int ph = p ? q->height >> 1 : q->height, y0 = q->cy * cs;
        const int ch = y0 + cs < ph ? cs : ph - y0;
        const uint8_t* src = (const uint8_t*)q->fenc[p];
        for (int y = 0; y < ch; y++) memcpy(I + o + (size_t)y * cs, src + y * q->fenc_stride[p], cs);
        js.fenc_at[p] = (int64_t)o;
        js.fs[p] = cs;
        o = (o + (size_t)cs * cs + 15) & ~(size_t)15;
    }
    if (o > x265amd::rdo_out_at(1)) return X265AMD_ENOMEM;
    const size_t ob = x265amd::rdo_out_at(1);
    js.stats = (int32_t*)(D + ob);
    js.count = (int32_t*)(D + ob) + 3 * 5 * 33;
    x265amd::RdoJob* job = (x265amd::RdoJob*)(I + x265amd::rdo_out_at(1));
    job->sao = js;
    job->kind = 1;
    int rc = server_publish(s, t, k, job);
    if (!rc) rc = direct_wait(s, t, k);
    if (rc)
    {
        // a request that was not served may still be: its slot is never posted to again
        r->state.store(3, std::memory_order_release);
        return record(rc);
    }
    memcpy(stats, H + ob, 4 * 3 * 5 * 33);
    memcpy(count, H + ob + 4 * 3 * 5 * 33, 4 * 3 * 5 * 33);
    std::lock_guard<std::mutex> g(s->smu);
    s->st.sao_ctus++;
    s->st.sao_ms += 1e3 * (now_s() - r->t_post);
    return 0;
}

extern "C" int x265amd_rdo_stats(x265amd_rdo* s, x265amd_rdo_counters* out)
{
    if (!s || !out) return X265AMD_EINVAL;
    std::lock_guard<std::mutex> g(s->smu);
    *out = s->st;
    return 0;
}

extern "C" void x265amd_devsync_begin(void)
{
    g_quiesce.fetch_add(1, std::memory_order_acq_rel);
    std::lock_guard<std::mutex> rl(g_srv_reg_mu);
    for (x265amd_rdo* s : g_srv_reg)
    {
        std::lock_guard<std::mutex> lk(s->srv_mu);
        (void)stop_server_locked(s);
    }
}

extern "C" void x265amd_devsync_end(void)
{
    g_quiesce.fetch_sub(1, std::memory_order_acq_rel);
}
