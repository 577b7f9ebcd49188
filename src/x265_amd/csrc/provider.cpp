// provider.cpp — X265_NS::setupHipPrimitives: the per-call EncoderPrimitives
// provider on top of the batched C ABI (include/x265_amd_primitives.h).
//
// Compiled twice (X265_DEPTH=8 -> namespace x265, X265_DEPTH=10 -> x265_10bit).
// Each table entry it installs is a synchronous round trip for ONE call:
// the operands the reference primitive reads (exactly that window — e.g. the
// taps/2-1 / taps/2 filter margins of ipfilter.cpp:88,129,173) are gathered
// row by row into a pinned staging buffer, copied to the device with one
// hipMemcpyAsync, processed by the same gfx950 kernel the batched API runs
// (batch of one, zero offsets), and the outputs are copied back into the
// caller's strided buffers.  Staging and the stream are per host thread, since
// x265 calls primitives concurrently from its worker pools.
//
// Errors: x265's primitives have no error channel, so every HIP status of a
// round trip (the two copies, the launch's own status, the synchronisation) is
// checked and the first failure is kept in a sticky process-wide status
// (x265amd_provider_status); a failed call returns zeroed outputs instead of
// whatever the staging buffer held, and every later call fails fast.  The
// caller turns the status into x265_encoder_encode() < 0 (x265.h:1351-1359;
// oracle/hip_encoder_main.cpp).  Test hooks, read once per process:
//   X265AMD_FAULT=alloc     every host thread's staging allocation fails
//   X265AMD_FAULT_AFTER=N   round trip N+1 onwards reports a failed copy
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <new>

#include "../../../include/x265_amd.h"
#include "../../../include/x265_amd_primitives.h"

namespace X265_NS {
namespace {

constexpr int kDepth = X265_DEPTH;
constexpr size_t kStage = 4u << 20;

} // namespace
} // namespace X265_NS

namespace x265amd_provider {
// one status for both depth builds of the provider (this file is compiled twice)
#if X265_DEPTH == 8
std::atomic<int> g_status{0};
std::atomic<long> g_trips{0};
#else
extern std::atomic<int> g_status;
extern std::atomic<long> g_trips;
#endif

inline void fail(int st)
{
    int zero = 0;
    g_status.compare_exchange_strong(zero, st);
}

struct FaultHooks
{
    bool alloc = false;
    long after = -1;
    FaultHooks()
    {
        const char* f = getenv("X265AMD_FAULT");
        alloc = f && !strcmp(f, "alloc");
        const char* a = getenv("X265AMD_FAULT_AFTER");
        if (a) after = atol(a);
    }
};

inline const FaultHooks& hooks()
{
    static const FaultHooks h;
    return h;
}
} // namespace x265amd_provider

namespace X265_NS {
namespace {
using x265amd_provider::fail;

struct Ctx
{
    hipStream_t st = nullptr;
    uint8_t* dev = nullptr;
    uint8_t* host = nullptr;
    size_t used = 0;
    bool ok = false;

    // never destroyed: thread-exit order against the HIP runtime's own teardown is unspecified
    Ctx()
    {
        ok = !x265amd_provider::hooks().alloc && hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess &&
             hipMalloc((void**)&dev, kStage) == hipSuccess &&
             hipHostMalloc((void**)&host, kStage, hipHostMallocDefault) == hipSuccess;
        if (!ok)
        {
            // a failed thread still answers calls (with zeroed outputs) from a plain host buffer
            host = (uint8_t*)calloc(1, kStage);
            fail(X265AMD_ENOMEM);
        }
    }
    void reset() { used = 0; }
    size_t alloc(size_t bytes)
    {
        size_t off = (used + 15) & ~(size_t)15;
        used = off + bytes;
        return off;
    }
    template <typename T> T* h(size_t off) { return (T*)(host + off); }
    template <typename T> T* d(size_t off) { return (T*)(dev + off); }
};

Ctx& ctx()
{
    static thread_local Ctx* c = new Ctx();
    return *c;
}

// gather a w x h block (rows of `stride` elements) into staging, compact
template <typename T>
size_t stage(Ctx& c, const T* src, intptr_t stride, int w, int h)
{
    size_t off = c.alloc(sizeof(T) * w * h);
    T* dst = c.h<T>(off);
    for (int y = 0; y < h; y++) memcpy(dst + y * w, src + y * stride, sizeof(T) * w);
    return off;
}

template <typename T>
size_t stage_value(Ctx& c, T v)
{
    size_t off = c.alloc(sizeof(T));
    *c.h<T>(off) = v;
    return off;
}

// upload everything staged so far, run `launch` (returns the C ABI status), download
// [out_off, out_off+out_bytes).  On any failure — or once an earlier call failed — the
// output window is zeroed and the first failure stays in the sticky status.
template <typename F>
void round_trip(Ctx& c, F launch, size_t out_off, size_t out_bytes)
{
    using namespace x265amd_provider;
    int st = g_status.load(std::memory_order_relaxed);
    if (!st && !c.ok) st = X265AMD_ENOMEM;
    if (!st && hooks().after >= 0 && g_trips.fetch_add(1) >= hooks().after) st = (int)hipErrorInvalidValue;
    if (!st) st = (int)hipMemcpyAsync(c.dev, c.host, c.used, hipMemcpyHostToDevice, c.st);
    if (!st) st = launch();
    if (!st) st = (int)hipMemcpyAsync(c.host + out_off, c.dev + out_off, out_bytes, hipMemcpyDeviceToHost, c.st);
    if (!st) st = (int)hipStreamSynchronize(c.st);
    if (st)
    {
        fail(st);
        if (c.ok) (void)hipStreamSynchronize(c.st);   // nothing of this call may still be in flight
        memset(c.host + out_off, 0, out_bytes);
    }
}

template <typename T>
void scatter(Ctx& c, size_t off, T* dst, intptr_t stride, int w, int h)
{
    const T* src = c.h<T>(off);
    for (int y = 0; y < h; y++) memcpy(dst + y * stride, src + y * w, sizeof(T) * w);
}

// ------------------------------------------------------------------ pixel compare
template <int OP, int W, int H, typename T>
int64_t cmp_call(const T* a, intptr_t sa, const T* b, intptr_t sb)
{
    Ctx& c = ctx();
    c.reset();
    const size_t z = stage_value<int64_t>(c, 0);
    const size_t oa = stage(c, a, sa, W, H);
    const size_t ob = b ? stage(c, b, sb, W, H) : oa;
    const size_t out = c.alloc(8);
    round_trip(c, [&] {
        return x265amd_pixelcmp(OP, kDepth, W, H, 1, c.d<T>(oa), W, c.d<int64_t>(z), c.d<T>(ob), W, c.d<int64_t>(z),
                         c.dev + out, c.st);
    }, out, 8);
    const bool wide = OP == X265AMD_SSE_PP || OP == X265AMD_SSE_SS || OP == X265AMD_SSD_S || OP == X265AMD_VAR;
    return wide ? (int64_t)*c.h<uint64_t>(out) : (int64_t)*c.h<int32_t>(out);
}

template <int OP, int W, int H>
int cmp_pp(const pixel* a, intptr_t sa, const pixel* b, intptr_t sb) { return (int)cmp_call<OP, W, H>(a, sa, b, sb); }

template <int W, int H>
sse_t sse_pp(const pixel* a, intptr_t sa, const pixel* b, intptr_t sb)
{
    return (sse_t)cmp_call<X265AMD_SSE_PP, W, H>(a, sa, b, sb);
}

template <int N>
sse_t sse_ss(const int16_t* a, intptr_t sa, const int16_t* b, intptr_t sb)
{
    return (sse_t)cmp_call<X265AMD_SSE_SS, N, N>(a, sa, b, sb);
}

template <int N>
sse_t ssd_s(const int16_t* a, intptr_t sa) { return (sse_t)cmp_call<X265AMD_SSD_S, N, N, int16_t>(a, sa, nullptr, 0); }

template <int N>
uint64_t var(const pixel* a, intptr_t sa) { return (uint64_t)cmp_call<X265AMD_VAR, N, N, pixel>(a, sa, nullptr, 0); }

template <int NREF, int W, int H>
void sad_multi(const pixel* f, const pixel* const* r, intptr_t rs, int32_t* res)
{
    Ctx& c = ctx();
    c.reset();
    const size_t z = stage_value<int64_t>(c, 0);
    const size_t of = stage(c, f, 64, W, H);   // FENC_STRIDE (pixel.cpp:88,112)
    size_t refs = c.alloc(sizeof(pixel) * W * H * NREF);
    for (int k = 0; k < NREF; k++)
        for (int y = 0; y < H; y++)
            memcpy(c.h<pixel>(refs) + (k * H + y) * W, r[k] + y * rs, sizeof(pixel) * W);
    size_t ro = c.alloc(8 * NREF);
    for (int k = 0; k < NREF; k++) c.h<int64_t>(ro)[k] = (int64_t)k * W * H;
    const size_t out = c.alloc(4 * NREF);
    round_trip(c, [&] {
        return x265amd_sad_multi(NREF, kDepth, W, H, 1, c.d<pixel>(of), W, c.d<int64_t>(z), c.d<pixel>(refs), W,
                          c.d<int64_t>(ro), c.d<int32_t>(out), c.st);
    }, out, 4 * NREF);
    memcpy(res, c.h<int32_t>(out), 4 * NREF);
}

template <int W, int H>
void sad_x3(const pixel* f, const pixel* r0, const pixel* r1, const pixel* r2, intptr_t rs, int32_t* res)
{
    const pixel* r[3] = { r0, r1, r2 };
    sad_multi<3, W, H>(f, r, rs, res);
}

template <int W, int H>
void sad_x4(const pixel* f, const pixel* r0, const pixel* r1, const pixel* r2, const pixel* r3, intptr_t rs, int32_t* res)
{
    const pixel* r[4] = { r0, r1, r2, r3 };
    sad_multi<4, W, H>(f, r, rs, res);
}

// ------------------------------------------------------------------ interpolation
// the window each op reads: columns [x0, W + x1), rows [y0, H + y1)
template <int OP, int N, typename S, typename D>
void filt_call(const S* src, intptr_t ss, D* dst, intptr_t ds, int W, int H, int coeff, int rowext)
{
    const bool hz = OP == X265AMD_HPP || OP == X265AMD_HPS || OP == X265AMD_HVPP;
    const bool vt = OP == X265AMD_VPP || OP == X265AMD_VPS || OP == X265AMD_VSP || OP == X265AMD_VSS ||
                    OP == X265AMD_HVPP || (OP == X265AMD_HPS && rowext);
    const int lx = hz ? N / 2 - 1 : 0, rx = hz ? N / 2 : 0;
    const int ly = vt ? N / 2 - 1 : 0, ry = vt ? N / 2 : 0;
    const int sw = W + lx + rx, sh = H + ly + ry;
    const int oh = (OP == X265AMD_HPS && rowext) ? H + N - 1 : H;
    Ctx& c = ctx();
    c.reset();
    const size_t z = stage_value<int64_t>(c, (int64_t)ly * sw + lx);   // block origin inside the staged window
    const size_t zd = stage_value<int64_t>(c, 0);
    const size_t cf = stage_value<uint8_t>(c, (uint8_t)coeff);
    const size_t os = stage(c, src - ly * ss - lx, ss, sw, sh);
    const size_t od = c.alloc(sizeof(D) * W * oh);
    round_trip(c, [&] {
        return x265amd_interp(OP, N, kDepth, W, H, 1, c.d<S>(os), sw, c.d<int64_t>(z), c.d<D>(od), W, c.d<int64_t>(zd),
                       c.d<uint8_t>(cf), rowext, c.st);
    }, od, sizeof(D) * W * oh);
    // hps with row extension writes H+N-1 rows starting at dst, the first of them being source
    // row -(N/2-1) (ipfilter.cpp:130-134)
    scatter(c, od, dst, ds, W, oh);
}

template <int N, int W, int H> void hpp(const pixel* s, intptr_t ss, pixel* d, intptr_t ds, int ci) { filt_call<X265AMD_HPP, N>(s, ss, d, ds, W, H, ci, 0); }
template <int N, int W, int H> void hps(const pixel* s, intptr_t ss, int16_t* d, intptr_t ds, int ci, int ext) { filt_call<X265AMD_HPS, N>(s, ss, d, ds, W, H, ci, ext); }
template <int N, int W, int H> void vpp(const pixel* s, intptr_t ss, pixel* d, intptr_t ds, int ci) { filt_call<X265AMD_VPP, N>(s, ss, d, ds, W, H, ci, 0); }
template <int N, int W, int H> void vps(const pixel* s, intptr_t ss, int16_t* d, intptr_t ds, int ci) { filt_call<X265AMD_VPS, N>(s, ss, d, ds, W, H, ci, 0); }
template <int N, int W, int H> void vsp(const int16_t* s, intptr_t ss, pixel* d, intptr_t ds, int ci) { filt_call<X265AMD_VSP, N>(s, ss, d, ds, W, H, ci, 0); }
template <int N, int W, int H> void vss(const int16_t* s, intptr_t ss, int16_t* d, intptr_t ds, int ci) { filt_call<X265AMD_VSS, N>(s, ss, d, ds, W, H, ci, 0); }
template <int W, int H> void hvpp(const pixel* s, intptr_t ss, pixel* d, intptr_t ds, int ix, int iy) { filt_call<X265AMD_HVPP, 8>(s, ss, d, ds, W, H, ix | (iy << 4), 0); }
template <int W, int H> void p2s(const pixel* s, intptr_t ss, int16_t* d, intptr_t ds) { filt_call<X265AMD_P2S, 4>(s, ss, d, ds, W, H, 0, 0); }

// ------------------------------------------------------------------ transforms / quant
template <int KIND, int N>
void tr_call(const int16_t* src, int16_t* dst, intptr_t stride)
{
    const bool fwd = KIND == X265AMD_DCT || KIND == X265AMD_DST;
    Ctx& c = ctx();
    c.reset();
    const size_t z = stage_value<int64_t>(c, 0);
    const size_t os = fwd ? stage(c, src, stride, N, N) : stage(c, src, N, N, N);
    const size_t od = c.alloc(2 * N * N);
    round_trip(c, [&] {
        return x265amd_transform(KIND, kDepth, N, 1, c.d<int16_t>(os), N, c.d<int64_t>(z), c.d<int16_t>(od), N,
                          c.d<int64_t>(z), c.st);
    }, od, 2 * N * N);
    scatter(c, od, dst, fwd ? N : stride, N, N);
}

template <int N> void dct(const int16_t* s, int16_t* d, intptr_t st) { tr_call<X265AMD_DCT, N>(s, d, st); }
template <int N> void idct(const int16_t* s, int16_t* d, intptr_t st) { tr_call<X265AMD_IDCT, N>(s, d, st); }
void dst4(const int16_t* s, int16_t* d, intptr_t st) { tr_call<X265AMD_DST, 4>(s, d, st); }
void idst4(const int16_t* s, int16_t* d, intptr_t st) { tr_call<X265AMD_IDST, 4>(s, d, st); }

uint32_t quant_call(const int16_t* coef, const int32_t* qc, int32_t* deltaU, int16_t* qout, int qBits, int add, int num)
{
    Ctx& c = ctx();
    c.reset();
    const size_t z = stage_value<int64_t>(c, 0);
    const size_t qb = stage_value<int32_t>(c, qBits), ad = stage_value<int32_t>(c, add);
    const size_t oc = stage(c, coef, num, num, 1), oq = stage(c, qc, num, num, 1);
    const size_t out = c.alloc(2 * num + 4 * num + 4);
    const size_t odl = out + 2 * num, osig = out + 6 * num;
    round_trip(c, [&] {
        return x265amd_quant(1, num, c.d<int16_t>(oc), c.d<int64_t>(z), c.d<int32_t>(oq), c.d<int64_t>(z),
                      deltaU ? c.d<int32_t>(odl) : nullptr, c.d<int64_t>(z), c.d<int16_t>(out), c.d<int64_t>(z),
                      c.d<int32_t>(qb), c.d<int32_t>(ad), c.d<uint32_t>(osig), c.st);
    }, out, 6 * num + 4);
    memcpy(qout, c.h<int16_t>(out), 2 * num);
    if (deltaU) memcpy(deltaU, c.h<int32_t>(odl), 4 * num);
    return *c.h<uint32_t>(osig);
}

uint32_t quant(const int16_t* coef, const int32_t* qc, int32_t* dU, int16_t* q, int qBits, int add, int num)
{
    return quant_call(coef, qc, dU, q, qBits, add, num);
}

uint32_t nquant(const int16_t* coef, const int32_t* qc, int16_t* q, int qBits, int add, int num)
{
    return quant_call(coef, qc, nullptr, q, qBits, add, num);
}

void dequant_normal(const int16_t* q, int16_t* coef, int num, int scale, int shift)
{
    Ctx& c = ctx();
    c.reset();
    const size_t z = stage_value<int64_t>(c, 0);
    const size_t sc = stage_value<int32_t>(c, scale), sh = stage_value<int32_t>(c, shift);
    const size_t oq = stage(c, q, num, num, 1);
    const size_t out = c.alloc(2 * num);
    round_trip(c, [&] {
        return x265amd_dequant_normal(1, num, c.d<int16_t>(oq), c.d<int64_t>(z), c.d<int16_t>(out), c.d<int64_t>(z),
                               c.d<int32_t>(sc), c.d<int32_t>(sh), c.st);
    }, out, 2 * num);
    memcpy(coef, c.h<int16_t>(out), 2 * num);
}

void dequant_scaling(const int16_t* q, const int32_t* dq, int16_t* coef, int num, int per, int shift)
{
    Ctx& c = ctx();
    c.reset();
    const size_t z = stage_value<int64_t>(c, 0);
    const size_t pp = stage_value<int32_t>(c, per), sh = stage_value<int32_t>(c, shift);
    const size_t oq = stage(c, q, num, num, 1), od = stage(c, dq, num, num, 1);
    const size_t out = c.alloc(2 * num);
    round_trip(c, [&] {
        return x265amd_dequant_scaling(1, num, c.d<int16_t>(oq), c.d<int64_t>(z), c.d<int32_t>(od), c.d<int64_t>(z),
                                c.d<int16_t>(out), c.d<int64_t>(z), c.d<int32_t>(pp), c.d<int32_t>(sh), c.st);
    }, out, 2 * num);
    memcpy(coef, c.h<int16_t>(out), 2 * num);
}

void denoise(int16_t* coef, uint32_t* res_sum, const uint16_t* offset, int num)
{
    Ctx& c = ctx();
    c.reset();
    const size_t z = stage_value<int64_t>(c, 0);
    const size_t oo = stage(c, offset, num, num, 1);
    const size_t oc = stage(c, (const int16_t*)coef, num, num, 1);
    const size_t orr = stage(c, (const uint32_t*)res_sum, num, num, 1);
    round_trip(c, [&] {
        return x265amd_denoise_dct(1, num, c.d<int16_t>(oc), c.d<int64_t>(z), c.d<uint32_t>(orr), c.d<uint16_t>(oo), c.st);
    }, oc, orr + 4 * num - oc);
    memcpy(coef, c.h<int16_t>(oc), 2 * num);
    memcpy(res_sum, c.h<uint32_t>(orr), 4 * num);
}

// ------------------------------------------------------------------ intra
// SLOT: the table slot's mode (0 planar, 1 DC) or -1 for the angular slots.  The
// reference's planar_pred_c / intra_pred_dc_c ignore the dirMode argument
// (intrapred.cpp:69,87: TestBench passes 0 to the DC slot, intrapredharness.cpp:62)
// and planar ignores bFilter too; intra_pred_ang_c uses the dirMode it is given.
template <int N, int SLOT>
void intra_pred(pixel* dst, intptr_t ds, const pixel* src, int mode, int bFilter)
{
    if (SLOT >= 0) mode = SLOT;
    if (SLOT == 0) bFilter = 0;
    Ctx& c = ctx();
    c.reset();
    const size_t z = stage_value<int64_t>(c, 0);
    const size_t om = stage_value<uint8_t>(c, (uint8_t)mode), ob = stage_value<uint8_t>(c, (uint8_t)bFilter);
    const size_t on = stage(c, src, 4 * N + 1, 4 * N + 1, 1);
    const size_t od = c.alloc(sizeof(pixel) * N * N);
    round_trip(c, [&] {
        return x265amd_intra_pred(kDepth, N, 1, c.d<pixel>(od), N, c.d<int64_t>(z), c.d<pixel>(on), c.d<int64_t>(z),
                           c.d<uint8_t>(om), c.d<uint8_t>(ob), c.st);
    }, od, sizeof(pixel) * N * N);
    scatter(c, od, dst, ds, N, N);
}

template <int N>
void intra_filter(const pixel* src, pixel* filt)
{
    Ctx& c = ctx();
    c.reset();
    const size_t z = stage_value<int64_t>(c, 0);
    const size_t on = stage(c, src, 4 * N + 1, 4 * N + 1, 1);
    const size_t od = c.alloc(sizeof(pixel) * (4 * N + 1));
    round_trip(c, [&] {
        return x265amd_intra_filter(kDepth, N, 1, c.d<pixel>(on), c.d<int64_t>(z), c.d<pixel>(od), c.d<int64_t>(z), c.st);
    }, od, sizeof(pixel) * (4 * N + 1));
    memcpy(filt, c.h<pixel>(od), sizeof(pixel) * (4 * N + 1));
}

template <int LOG2>
void allangs(pixel* dst, pixel* ref, pixel* filt, int bLuma)
{
    constexpr int N = 1 << LOG2;
    Ctx& c = ctx();
    c.reset();
    const size_t z = stage_value<int64_t>(c, 0);
    const size_t ob = stage_value<uint8_t>(c, (uint8_t)bLuma);
    const size_t orf = stage(c, (const pixel*)ref, 4 * N + 1, 4 * N + 1, 1);
    const size_t oft = stage(c, (const pixel*)filt, 4 * N + 1, 4 * N + 1, 1);
    const size_t od = c.alloc(sizeof(pixel) * 33 * N * N);
    round_trip(c, [&] {
        return x265amd_intra_allangs(kDepth, N, 1, c.d<pixel>(od), c.d<int64_t>(z), c.d<pixel>(orf), c.d<int64_t>(z),
                              c.d<pixel>(oft), c.d<int64_t>(z), c.d<uint8_t>(ob), c.st);
    }, od, sizeof(pixel) * 33 * N * N);
    memcpy(dst, c.h<pixel>(od), sizeof(pixel) * 33 * N * N);
}

// ------------------------------------------------------------------ companion block ops (a15)
// dst (W x H, stride ds) = op(a (stride sa), b (stride sb), param)
template <int OP, int W, int H, typename D, typename A, typename B>
void bo_call(D* dst, intptr_t ds, const A* a, intptr_t sa, const B* b, intptr_t sb, int param)
{
    Ctx& c = ctx();
    c.reset();
    const size_t z = stage_value<int64_t>(c, 0);
    // transpose reads the W x H source column-wise: the staged window is the same block
    const size_t oa = a ? stage(c, a, sa, W, H) : z;
    const size_t ob = b ? stage(c, b, sb, W, H) : z;
    const size_t od = c.alloc(sizeof(D) * W * H);
    round_trip(c, [&] {
        return x265amd_blockop(OP, kDepth, W, H, 1, c.d<D>(od), W, c.d<int64_t>(z), a ? c.d<A>(oa) : nullptr, W,
                        c.d<int64_t>(z), b ? c.d<B>(ob) : nullptr, W, c.d<int64_t>(z), param, c.st);
    }, od, sizeof(D) * W * H);
    scatter(c, od, dst, ds, W, H);
}

template <int W, int H>
void pixelavg_pp(pixel* d, intptr_t ds, const pixel* s0, intptr_t ss0, const pixel* s1, intptr_t ss1, int)
{
    bo_call<X265AMD_PIXELAVG, W, H>(d, ds, s0, ss0, s1, ss1, 0);
}
template <int W, int H>
void add_avg(const int16_t* s0, const int16_t* s1, pixel* d, intptr_t ss0, intptr_t ss1, intptr_t ds)
{
    bo_call<X265AMD_ADDAVG, W, H>(d, ds, s0, ss0, s1, ss1, 0);
}
template <int W, int H>
void copy_pp(pixel* d, intptr_t ds, const pixel* s, intptr_t ss) { bo_call<X265AMD_COPY_PP, W, H>(d, ds, s, ss, (const pixel*)nullptr, 0, 0); }
template <int W, int H>
void copy_sp(pixel* d, intptr_t ds, const int16_t* s, intptr_t ss) { bo_call<X265AMD_COPY_SP, W, H>(d, ds, s, ss, (const int16_t*)nullptr, 0, 0); }
template <int W, int H>
void copy_ps(int16_t* d, intptr_t ds, const pixel* s, intptr_t ss) { bo_call<X265AMD_COPY_PS, W, H>(d, ds, s, ss, (const pixel*)nullptr, 0, 0); }
template <int W, int H>
void copy_ss(int16_t* d, intptr_t ds, const int16_t* s, intptr_t ss) { bo_call<X265AMD_COPY_SS, W, H>(d, ds, s, ss, (const int16_t*)nullptr, 0, 0); }
template <int W, int H>
void sub_ps(int16_t* d, intptr_t ds, const pixel* a, const pixel* b, intptr_t sa, intptr_t sb)
{
    bo_call<X265AMD_SUB_PS, W, H>(d, ds, a, sa, b, sb, 0);
}
template <int W, int H>
void add_ps(pixel* d, intptr_t ds, const pixel* a, const int16_t* b, intptr_t sa, intptr_t sb)
{
    bo_call<X265AMD_ADD_PS, W, H>(d, ds, a, sa, b, sb, 0);
}
template <int N>
void calcresidual(const pixel* fenc, const pixel* pred, int16_t* res, intptr_t st)
{
    bo_call<X265AMD_SUB_PS, N, N>(res, st, fenc, st, pred, st, 0);
}
template <int N>
void blockfill_s(int16_t* d, intptr_t ds, int16_t v) { bo_call<X265AMD_BLOCKFILL, N, N>(d, ds, (const int16_t*)nullptr, 0, (const int16_t*)nullptr, 0, v); }
template <int N>
void cpy2Dto1D_shl(int16_t* d, const int16_t* s, intptr_t ss, int sh) { bo_call<X265AMD_CPY2D1D_SHL, N, N>(d, N, s, ss, (const int16_t*)nullptr, 0, sh); }
template <int N>
void cpy2Dto1D_shr(int16_t* d, const int16_t* s, intptr_t ss, int sh) { bo_call<X265AMD_CPY2D1D_SHR, N, N>(d, N, s, ss, (const int16_t*)nullptr, 0, sh); }
template <int N>
void cpy1Dto2D_shl(int16_t* d, const int16_t* s, intptr_t ds, int sh) { bo_call<X265AMD_CPY1D2D_SHL, N, N>(d, ds, s, N, (const int16_t*)nullptr, 0, sh); }
template <int N>
void cpy1Dto2D_shr(int16_t* d, const int16_t* s, intptr_t ds, int sh) { bo_call<X265AMD_CPY1D2D_SHR, N, N>(d, ds, s, N, (const int16_t*)nullptr, 0, sh); }
template <int N>
void transpose(pixel* d, const pixel* s, intptr_t ss) { bo_call<X265AMD_TRANSPOSE, N, N>(d, N, s, ss, (const pixel*)nullptr, 0, 0); }

// count_nonzero (dct.cpp:714-726) / copy_count (dct.cpp:728-742)
template <int N>
uint32_t count_call(int16_t* coeff, const int16_t* res, intptr_t rs)
{
    Ctx& c = ctx();
    c.reset();
    const size_t z = stage_value<int64_t>(c, 0);
    const size_t oc = res ? c.alloc(2 * N * N) : stage(c, (const int16_t*)coeff, N * N, N * N, 1);
    const size_t orr = res ? stage(c, res, rs, N, N) : z;
    const size_t out = c.alloc(4);
    round_trip(c, [&] {
        return x265amd_count_nonzero(N, 1, c.d<int16_t>(oc), c.d<int64_t>(z), res ? c.d<int16_t>(orr) : nullptr, N,
                              c.d<int64_t>(z), c.d<uint32_t>(out), c.st);
    }, oc, out + 4 - oc);
    if (res) memcpy(coeff, c.h<int16_t>(oc), 2 * N * N);
    return *c.h<uint32_t>(out);
}
template <int N>
int count_nonzero(const int16_t* q) { return (int)count_call<N>((int16_t*)q, nullptr, 0); }
template <int N>
uint32_t copy_cnt(int16_t* coeff, const int16_t* res, intptr_t rs) { return count_call<N>(coeff, res, rs); }

// ------------------------------------------------------------------ table filling
int g_count;

template <typename F>
void put(F& slot, F fn)
{
    // override only entries the table already has (NULL entries must stay NULL: callers test them,
    // e.g. motion.cpp:193-197) — the same rule an assembly provider follows
    if (slot)
    {
        slot = fn;
        g_count++;
    }
}

template <int W, int H>
void luma_pu(EncoderPrimitives::PU& u)
{
    put(u.sad, &cmp_pp<X265AMD_SAD, W, H>);
    put(u.sad_x3, &sad_x3<W, H>);
    put(u.sad_x4, &sad_x4<W, H>);
    put(u.satd, &cmp_pp<X265AMD_SATD, W, H>);
    put(u.luma_hpp, &hpp<8, W, H>);
    put(u.luma_hps, &hps<8, W, H>);
    put(u.luma_vpp, &vpp<8, W, H>);
    put(u.luma_vps, &vps<8, W, H>);
    put(u.luma_vsp, &vsp<8, W, H>);
    put(u.luma_vss, &vss<8, W, H>);
    put(u.luma_hvpp, &hvpp<W, H>);
    put(u.convert_p2s, &p2s<W, H>);
    put(u.pixelavg_pp, &pixelavg_pp<W, H>);
    put(u.addAvg, &add_avg<W, H>);
    put(u.copy_pp, &copy_pp<W, H>);
}

template <int W, int H>
void chroma_pu(EncoderPrimitives::Chroma::PUChroma& u)
{
    if constexpr (W % 4 == 0 && H % 4 == 0) put(u.satd, &cmp_pp<X265AMD_SATD, W, H>);
    put(u.filter_hpp, &hpp<4, W, H>);
    put(u.filter_hps, &hps<4, W, H>);
    put(u.filter_vpp, &vpp<4, W, H>);
    put(u.filter_vps, &vps<4, W, H>);
    put(u.filter_vsp, &vsp<4, W, H>);
    put(u.filter_vss, &vss<4, W, H>);
    put(u.p2s, &p2s<W, H>);
    if constexpr (W % 2 == 0)
    {
        put(u.addAvg, &add_avg<W, H>);
        put(u.copy_pp, &copy_pp<W, H>);
    }
}

template <int N>
void luma_cu(EncoderPrimitives::CU& u)
{
    if constexpr (N <= 32)
    {
        put(u.dct, &dct<N>);
        put(u.idct, &idct<N>);
        put(u.intra_filter, &intra_filter<N>);
        put(u.intra_pred[0], &intra_pred<N, 0>);
        put(u.intra_pred[1], &intra_pred<N, 1>);
        for (int m = 2; m < NUM_INTRA_MODE; m++) put(u.intra_pred[m], &intra_pred<N, -1>);
        constexpr int L = N == 4 ? 2 : N == 8 ? 3 : N == 16 ? 4 : 5;
        put(u.intra_pred_allangs, &allangs<L>);
        put(u.count_nonzero, &count_nonzero<N>);
        put(u.copy_cnt, &copy_cnt<N>);
    }
    put(u.calcresidual, &calcresidual<N>);
    put(u.sub_ps, &sub_ps<N, N>);
    put(u.add_ps, &add_ps<N, N>);
    put(u.blockfill_s, &blockfill_s<N>);
    put(u.cpy2Dto1D_shl, &cpy2Dto1D_shl<N>);
    put(u.cpy2Dto1D_shr, &cpy2Dto1D_shr<N>);
    put(u.cpy1Dto2D_shl, &cpy1Dto2D_shl<N>);
    put(u.cpy1Dto2D_shr, &cpy1Dto2D_shr<N>);
    put(u.copy_sp, &copy_sp<N, N>);
    put(u.copy_ps, &copy_ps<N, N>);
    put(u.copy_ss, &copy_ss<N, N>);
    put(u.copy_pp, &copy_pp<N, N>);
    put(u.transpose, &transpose<N>);
    put(u.sa8d, &cmp_pp<X265AMD_SA8D, N, N>);
    put(u.sse_pp, &sse_pp<N, N>);
    put(u.sse_ss, &sse_ss<N>);
    put(u.ssd_s, &ssd_s<N>);
    put(u.var, &var<N>);
    put(u.psy_cost_pp, &cmp_pp<X265AMD_PSY, N, N>);
}

template <int W, int H>
void chroma_cu(EncoderPrimitives::Chroma::CUChroma& u)
{
    if constexpr (W % 4 == 0 && H % 4 == 0)
    {
        put(u.sa8d, &cmp_pp<X265AMD_SA8D, W, H>);
        put(u.sse_pp, &sse_pp<W, H>);
    }
    put(u.sub_ps, &sub_ps<W, H>);
    put(u.add_ps, &add_ps<W, H>);
    put(u.copy_ps, &copy_ps<W, H>);
    put(u.copy_sp, &copy_sp<W, H>);
    put(u.copy_ss, &copy_ss<W, H>);
    put(u.copy_pp, &copy_pp<W, H>);
}

// chroma dims of luma PU p for 4:2:0 (w/2, h/2) and 4:2:2 (w/2, h)
#define LUMA_PU_LIST(X) X(LUMA_4x4, 4, 4) X(LUMA_8x8, 8, 8) X(LUMA_16x16, 16, 16) X(LUMA_32x32, 32, 32) \
    X(LUMA_64x64, 64, 64) X(LUMA_8x4, 8, 4) X(LUMA_4x8, 4, 8) X(LUMA_16x8, 16, 8) X(LUMA_8x16, 8, 16)     \
    X(LUMA_32x16, 32, 16) X(LUMA_16x32, 16, 32) X(LUMA_64x32, 64, 32) X(LUMA_32x64, 32, 64)              \
    X(LUMA_16x12, 16, 12) X(LUMA_12x16, 12, 16) X(LUMA_16x4, 16, 4) X(LUMA_4x16, 4, 16)                  \
    X(LUMA_32x24, 32, 24) X(LUMA_24x32, 24, 32) X(LUMA_32x8, 32, 8) X(LUMA_8x32, 8, 32)                  \
    X(LUMA_64x48, 64, 48) X(LUMA_48x64, 48, 64) X(LUMA_64x16, 64, 16) X(LUMA_16x64, 16, 64)

} // namespace

void setupHipPrimitives(EncoderPrimitives& p, int /*cpuMask*/)
{
    g_count = 0;
    // staging is per host thread and created on a thread's first call; a thread whose staging
    // cannot be allocated records X265AMD_ENOMEM in the sticky status (see round_trip)
    if (x265amd_set_device(0) != 0) return;
    enum { I420 = 1, I422 = 2, I444 = 3 };
#define X(P, W, H)                                                     \
    luma_pu<W, H>(p.pu[P]);                                            \
    chroma_pu<W / 2, H / 2>(p.chroma[I420].pu[P]);                     \
    chroma_pu<W / 2, H>(p.chroma[I422].pu[P]);                         \
    chroma_pu<W, H>(p.chroma[I444].pu[P]);
    LUMA_PU_LIST(X)
#undef X
    luma_cu<4>(p.cu[0]);
    luma_cu<8>(p.cu[1]);
    luma_cu<16>(p.cu[2]);
    luma_cu<32>(p.cu[3]);
    luma_cu<64>(p.cu[4]);
    chroma_cu<2, 2>(p.chroma[I420].cu[0]);
    chroma_cu<2, 4>(p.chroma[I422].cu[0]);
    chroma_cu<4, 4>(p.chroma[I420].cu[1]);
    chroma_cu<8, 8>(p.chroma[I420].cu[2]);
    chroma_cu<16, 16>(p.chroma[I420].cu[3]);
    chroma_cu<32, 32>(p.chroma[I420].cu[4]);
    chroma_cu<4, 8>(p.chroma[I422].cu[1]);
    chroma_cu<8, 16>(p.chroma[I422].cu[2]);
    chroma_cu<16, 32>(p.chroma[I422].cu[3]);
    chroma_cu<32, 64>(p.chroma[I422].cu[4]);
    put(p.dst4x4, &dst4);
    put(p.idst4x4, &idst4);
    put(p.quant, &quant);
    put(p.nquant, &nquant);
    put(p.dequant_normal, &dequant_normal);
    put(p.dequant_scaling, &dequant_scaling);
    put(p.denoiseDct, &denoise);
}

int hip_provider_count() { return g_count; }

} // namespace X265_NS

#if X265_DEPTH == 8
static_assert(sizeof(x265::EncoderPrimitives) == 1876 * sizeof(void*), "EncoderPrimitives layout drifted");

namespace x265_10bit {
struct EncoderPrimitives;
void setupHipPrimitives(EncoderPrimitives& p, int cpuMask);
int hip_provider_count();
}

extern "C" int x265amd_setup_primitives(void* table, int depth, int* overridden)
{
    if (x265amd_set_device(0) != 0) return X265AMD_ENODEV;
    int n = 0;
    if (depth == 8)
    {
        x265::setupHipPrimitives(*(x265::EncoderPrimitives*)table, 0);
        n = x265::hip_provider_count();
    }
    else if (depth == 10 || depth == 12)
    {
        x265_10bit::setupHipPrimitives(*(x265_10bit::EncoderPrimitives*)table, 0);
        n = x265_10bit::hip_provider_count();
    }
    else
        return X265AMD_EINVAL;
    if (overridden) *overridden = n;
    return 0;
}

extern "C" size_t x265amd_primitives_size(void)
{
    return sizeof(x265::EncoderPrimitives);
}

extern "C" int x265amd_provider_status(void)
{
    return x265amd_provider::g_status.load();
}

extern "C" void x265amd_provider_clear_status(void)
{
    x265amd_provider::g_status.store(0);
    x265amd_provider::g_trips.store(0);
}
#endif
