// common.h — shared device helpers for the x265 primitive kernels (gfx950).
//
// Batching model: every C-ABI call processes `n` independent
// jobs of one primitive family and one block shape.  A job is owned by a
// power-of-two group of G lanes inside one 64-lane wavefront; each lane walks
// the job's fixed-size units (a row strip, a 4x4 / 8x8 Hadamard tile, ...)
// with stride G and the group reduces with cross-lane shuffles.  Operands are
// addressed as base pointer + per-job element offset (int64) + per-batch
// stride, so jobs can point anywhere inside device-resident frame planes.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "tables.h"

#define X265AMD_BLOCK 256

namespace x265amd {

// ---------------------------------------------------------------- launch
// Bijective XCD-aware remap of the hardware block id (guide T1): hardware
// block b runs on XCD b % 8; give every XCD a contiguous range of logical
// blocks so jobs that are neighbours in the batch (neighbouring blocks of a
// frame) share that XCD's L2.  Speed only, never correctness.
__device__ __forceinline__ uint32_t xcd_block()
{
    const uint32_t b = blockIdx.x, nb = gridDim.x;
    if (nb < 16) return b;
    const uint32_t q = nb >> 3, r = nb & 7, x = b & 7;
    return x * q + (x < r ? x : r) + (b >> 3);
}

// Job/lane coordinates for a G-lane group (G power of two, <= 64).
template <int G>
struct Group
{
    int64_t job;
    int lane;
    __device__ __forceinline__ Group()
    {
        const uint32_t lb = xcd_block();
        job  = (int64_t)lb * (X265AMD_BLOCK / G) + threadIdx.x / G;
        lane = threadIdx.x & (G - 1);
    }
};

// Group reduction (sum) over the G lanes of a group; result valid in all lanes.
template <int G, typename T>
__device__ __forceinline__ T group_sum(T v)
{
#pragma unroll
    for (int m = G >> 1; m > 0; m >>= 1)
        v += __shfl_xor(v, m, 64);
    return v;
}

template <int G>
__device__ __forceinline__ uint64_t group_sum64(uint64_t v)
{
#pragma unroll
    for (int m = G >> 1; m > 0; m >>= 1)
    {
        uint32_t lo = __shfl_xor((uint32_t)v, m, 64);
        uint32_t hi = __shfl_xor((uint32_t)(v >> 32), m, 64);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}

inline int pow2ceil(int v)
{
    int g = 1;
    while (g < v) g <<= 1;
    return g;
}

// log2 of the lanes per job: two units per lane, so small blocks get one lane
// per job (all of the job's row loads in flight from one lane) and large ones
// up to a full wavefront
inline int lanes_log2(int units, int per_lane = 2)
{
    int g = pow2ceil((units + per_lane - 1) / per_lane);
    if (g > 64) g = 64;
    int lg = 0;
    while ((1 << lg) < g) lg++;
    return lg;
}

inline uint32_t blocks_for(int n, int lg, int jpl = 1)
{
    const int per = (X265AMD_BLOCK >> lg) * (jpl > 1 ? jpl : 1);
    return (uint32_t)((n + per - 1) / per);
}

// ---------------------------------------------------------------- grouped launches
// One launch carries up to kMaxSub sub-batches of one kernel class (same
// template instantiation) but different block shapes and operands.  The table
// travels in the kernarg segment (aggregate kernel arguments are passed by
// reference there, so the dynamic index below is a scalar load, not a copy);
// every workgroup belongs to exactly one sub-batch and finds it with a uniform
// scan over block0.  A launch of 16 small shapes fills the chip like one large
// batch instead of 16 short launches each under-occupying it.
constexpr int kMaxSub = 16;

struct SubBatch
{
    void* d;                // destination / output
    const int64_t* doff;
    int64_t ds;
    const void* a;          // first operand
    const int64_t* aoff;
    int64_t sa;
    const void* b;          // second operand (interp: per-job coefficient index)
    const int64_t* boff;
    int64_t sb;
    int w, h, n, lg;
    int param;
    int jpl;                // jobs per lane group (0 = 1)
    uint32_t block0;        // first logical block of this sub-batch
};

struct BatchGroup
{
    SubBatch s[kMaxSub];
    int count;
    int depth;
    int flag;               // pixelcmp: sse_t wraps to 32 bits
    int pad;
};

__device__ __forceinline__ const SubBatch& group_sub(const BatchGroup& g, uint32_t gb)
{
    int s = 0;
#pragma unroll
    for (int i = 1; i < kMaxSub; i++)
        if (i < g.count && g.s[i].block0 <= gb) s = i;
    return g.s[s];
}

// Host side: packs `count` batches into launches, one kernel class per launch
// (first-come order, at most kMaxSub sub-batches each).  cls[i] < 0 marks an
// empty batch.  fill(i, sub) sets everything but block0 (lg included);
// launch(cls, group, blocks) enqueues one kernel and returns its status.
template <typename Fill, typename Launch>
inline int launch_grouped(int count, const int* cls, const BatchGroup& proto, Fill fill, Launch launch)
{
    std::vector<char> done(count, 0);
    for (int i = 0; i < count; i++)
    {
        if (done[i] || cls[i] < 0) continue;
        BatchGroup g = proto;
        uint32_t blocks = 0;
        int k = 0;
        for (int j = i; j < count && k < kMaxSub; j++)
        {
            if (done[j] || cls[j] != cls[i]) continue;
            done[j] = 1;
            SubBatch& s = g.s[k++];
            fill(j, s);
            s.block0 = blocks;
            blocks += blocks_for(s.n, s.lg, s.jpl);
        }
        g.count = k;
        const int rc = launch(cls[i], g, blocks);
        if (rc) return rc;
    }
    return 0;
}

// ---------------------------------------------------------------- fork / join
// A call carrying several independent batches spreads their launches over up to kForkStreams
// internal streams: they wait on an event recorded on the caller's stream, and the caller's stream
// waits on their completion events, so stream order (and hipGraph capture) is preserved.  Streams
// and events are created once per (host thread, device, origin priority) — with the origin stream's
// priority, so a high-priority launcher's forked launches stay high-priority — and destroyed when
// the thread exits (a session's launcher threads end at encoder close: nothing accumulates).
constexpr int kForkStreams = 4;

struct ForkCache
{
    hipStream_t s[kForkStreams] = {};
    hipEvent_t f = nullptr, d[kForkStreams] = {};
    int dev = -1;
    bool ok = false;
    ~ForkCache()
    {
        if (!ok) return;
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) return;
        if (cur != dev && hipSetDevice(dev) != hipSuccess) return;
        for (int i = 0; i < kForkStreams; i++)
        {
            (void)hipStreamSynchronize(s[i]);
            (void)hipStreamDestroy(s[i]);
            (void)hipEventDestroy(d[i]);
        }
        (void)hipEventDestroy(f);
        if (cur != dev) (void)hipSetDevice(cur);
    }
};

struct ForkJoin
{
    hipStream_t origin = nullptr;
    hipStream_t sub[kForkStreams] = {};
    hipEvent_t fork = nullptr, done[kForkStreams] = {};
    int n = 0;
    hipError_t err = hipSuccess;

    ForkJoin(hipStream_t st, int want)
    {
        origin = st;
        if (want <= 1) return;                      // nothing to overlap: launch on the caller's stream
        n = want > kForkStreams ? kForkStreams : want;
        int dev = 0, prio = 0;
        err = hipGetDevice(&dev);
        static thread_local ForkCache cache[16][2];
        if (err != hipSuccess || dev < 0 || dev >= 16) { n = 0; return; }
        if (origin && hipStreamGetPriority(origin, &prio) != hipSuccess) prio = 0;
        ForkCache& c = cache[dev][prio != 0];
        if (!c.ok)
        {
            for (int i = 0; i < kForkStreams && err == hipSuccess; i++)
            {
                err = hipStreamCreateWithPriority(&c.s[i], hipStreamNonBlocking, prio);
                if (err == hipSuccess) err = hipEventCreateWithFlags(&c.d[i], hipEventDisableTiming);
            }
            if (err == hipSuccess) err = hipEventCreateWithFlags(&c.f, hipEventDisableTiming);
            if (err != hipSuccess) { n = 0; return; }
            c.dev = dev;
            c.ok = true;
        }
        fork = c.f;
        for (int i = 0; i < kForkStreams; i++) { sub[i] = c.s[i]; done[i] = c.d[i]; }
        err = hipEventRecord(fork, origin);
        for (int i = 0; i < n && err == hipSuccess; i++) err = hipStreamWaitEvent(sub[i], fork, 0);
    }
    hipStream_t stream(int k) const { return n ? sub[k % n] : origin; }
    hipError_t join()
    {
        for (int i = 0; i < n && err == hipSuccess; i++)
        {
            err = hipEventRecord(done[i], sub[i]);
            if (err == hipSuccess) err = hipStreamWaitEvent(origin, done[i], 0);
        }
        return err;
    }
};

// LDS exchange among the lanes of one wavefront: orders this lane's LDS
// writes before the other lanes' later reads (LDS executes a wavefront's
// instructions in order; the fences keep the compiler from moving accesses
// across).  No s_barrier: groups never span wavefronts.
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------- loads
// Unaligned little-endian loads (gfx950 runs HSA in unaligned mode: these
// lower to single global_load_dword{,x2,x4}).
template <typename T>
__device__ __forceinline__ T ldu(const void* p)
{
    T v;
    __builtin_memcpy(&v, p, sizeof(T));
    return v;
}
// a vector load of T; NT: non-temporal (rows read once — a batch of disjoint blocks — are kept from
// displacing lines that are re-read; measured on disjoint SAD batches 8x8 0.64 -> 0.71, 64x64 0.79 -> 0.89 of
// the HBM peak, profiles/r05/sad_nt_ab.txt)
template <typename T, bool NT>
__device__ __forceinline__ T ldx(const void* p)
{
    typedef unsigned int v2u __attribute__((ext_vector_type(2)));
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    if constexpr (!NT) return ldu<T>(p);
    else if constexpr (sizeof(T) == 4) return __builtin_bit_cast(T, __builtin_nontemporal_load((const unsigned int*)p));
    else if constexpr (sizeof(T) == 8) return __builtin_bit_cast(T, __builtin_nontemporal_load((const v2u*)p));
    else return __builtin_bit_cast(T, __builtin_nontemporal_load((const v4u*)p));
}

template <typename T>
__device__ __forceinline__ void stu(void* p, T v)
{
    __builtin_memcpy(p, &v, sizeof(T));
}

template <typename P>
__device__ __forceinline__ int clip_pixel(int v, int maxv)
{
    return v < 0 ? 0 : (v > maxv ? maxv : v);
}

__device__ __forceinline__ int clip16(int v)
{
    return v < -32768 ? -32768 : (v > 32767 ? 32767 : v);
}

// Load UW consecutive pixels (as int) starting at p.
template <typename P, int UW>
__device__ __forceinline__ void load_row(const P* p, int (&o)[UW])
{
    if constexpr (UW == 16 && sizeof(P) == 2)
    {
        int lo[8], hi[8];
        load_row<P, 8>(p, lo);
        load_row<P, 8>(p + 8, hi);
#pragma unroll
        for (int i = 0; i < 8; i++) { o[i] = lo[i]; o[8 + i] = hi[i]; }
    }
    else if constexpr (sizeof(P) == 1)
    {
        if constexpr (UW == 16)
        {
            uint4 v = ldu<uint4>(p);
            uint32_t w[4] = { v.x, v.y, v.z, v.w };
#pragma unroll
            for (int i = 0; i < 16; i++) o[i] = (int)((w[i >> 2] >> (8 * (i & 3))) & 0xff);
        }
        else if constexpr (UW == 8)
        {
            uint64_t v = ldu<uint64_t>(p);
#pragma unroll
            for (int i = 0; i < 8; i++) o[i] = (int)((v >> (8 * i)) & 0xff);
        }
        else if constexpr (UW == 4)
        {
            uint32_t v = ldu<uint32_t>(p);
#pragma unroll
            for (int i = 0; i < 4; i++) o[i] = (int)((v >> (8 * i)) & 0xff);
        }
        else
        {
#pragma unroll
            for (int i = 0; i < UW; i++) o[i] = p[i];
        }
    }
    else
    {
        if constexpr (UW == 8)
        {
            uint4 v = ldu<uint4>(p);
            uint32_t w[4] = { v.x, v.y, v.z, v.w };
#pragma unroll
            for (int i = 0; i < 4; i++) { o[2 * i] = (int)(w[i] & 0xffff); o[2 * i + 1] = (int)(w[i] >> 16); }
        }
        else if constexpr (UW == 4)
        {
            uint2 v = ldu<uint2>(p);
            o[0] = (int)(v.x & 0xffff); o[1] = (int)(v.x >> 16);
            o[2] = (int)(v.y & 0xffff); o[3] = (int)(v.y >> 16);
        }
        else
        {
#pragma unroll
            for (int i = 0; i < UW; i++) o[i] = p[i];
        }
    }
}

// Load UW consecutive int16 values.
template <int UW>
__device__ __forceinline__ void load_row16(const int16_t* p, int (&o)[UW])
{
    if constexpr (UW == 16)
    {
        int lo[8], hi[8];
        load_row16<8>(p, lo);
        load_row16<8>(p + 8, hi);
#pragma unroll
        for (int i = 0; i < 8; i++) { o[i] = lo[i]; o[8 + i] = hi[i]; }
    }
    else if constexpr (UW == 8)
    {
        uint4 v = ldu<uint4>(p);
        uint32_t w[4] = { v.x, v.y, v.z, v.w };
#pragma unroll
        for (int i = 0; i < 4; i++) { o[2 * i] = (int)(int16_t)(w[i] & 0xffff); o[2 * i + 1] = (int)(int16_t)(w[i] >> 16); }
    }
    else if constexpr (UW == 4)
    {
        uint2 v = ldu<uint2>(p);
        o[0] = (int16_t)(v.x & 0xffff); o[1] = (int16_t)(v.x >> 16);
        o[2] = (int16_t)(v.y & 0xffff); o[3] = (int16_t)(v.y >> 16);
    }
    else
    {
#pragma unroll
        for (int i = 0; i < UW; i++) o[i] = p[i];
    }
}

template <typename P, int UW>
__device__ __forceinline__ void store_row(P* p, const int (&v)[UW])
{
    if constexpr (UW == 16 && sizeof(P) == 2)
    {
        int lo[8], hi[8];
#pragma unroll
        for (int i = 0; i < 8; i++) { lo[i] = v[i]; hi[i] = v[8 + i]; }
        store_row<P, 8>(p, lo);
        store_row<P, 8>(p + 8, hi);
    }
    else if constexpr (sizeof(P) == 1 && UW == 16)
    {
        uint32_t w[4] = { 0, 0, 0, 0 };
#pragma unroll
        for (int i = 0; i < 16; i++) w[i >> 2] |= (uint32_t)(v[i] & 0xff) << (8 * (i & 3));
        stu<uint4>(p, make_uint4(w[0], w[1], w[2], w[3]));
    }
    else if constexpr (sizeof(P) == 1 && UW == 8)
    {
        uint64_t w = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) w |= (uint64_t)(v[i] & 0xff) << (8 * i);
        stu<uint64_t>(p, w);
    }
    else if constexpr (sizeof(P) == 1 && UW == 4)
    {
        uint32_t w = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) w |= (uint32_t)(v[i] & 0xff) << (8 * i);
        stu<uint32_t>(p, w);
    }
    else if constexpr (sizeof(P) == 2 && UW == 8)
    {
        uint4 w;
        w.x = (uint32_t)(v[0] & 0xffff) | ((uint32_t)v[1] << 16);
        w.y = (uint32_t)(v[2] & 0xffff) | ((uint32_t)v[3] << 16);
        w.z = (uint32_t)(v[4] & 0xffff) | ((uint32_t)v[5] << 16);
        w.w = (uint32_t)(v[6] & 0xffff) | ((uint32_t)v[7] << 16);
        stu<uint4>(p, w);
    }
    else if constexpr (sizeof(P) == 2 && UW == 4)
    {
        uint2 w;
        w.x = (uint32_t)(v[0] & 0xffff) | ((uint32_t)v[1] << 16);
        w.y = (uint32_t)(v[2] & 0xffff) | ((uint32_t)v[3] << 16);
        stu<uint2>(p, w);
    }
    else
    {
#pragma unroll
        for (int i = 0; i < UW; i++) p[i] = (P)v[i];
    }
}

// A row segment of N pixels kept packed in registers (loaded once, unpacked
// twice: for the residual and again for the reconstruction).
template <typename P, int N>
struct PixRow
{
    static constexpr int W = (N * (int)sizeof(P) + 3) / 4;
    uint32_t w[W];
    __device__ __forceinline__ void load(const P* p)
    {
        if constexpr (W == 1) w[0] = ldu<uint32_t>(p);
        else if constexpr (W == 2) { const uint2 v = ldu<uint2>(p); w[0] = v.x; w[1] = v.y; }
        else
        {
#pragma unroll
            for (int i = 0; i < W; i += 4)
            {
                const uint4 v = ldu<uint4>((const char*)p + 4 * i);
                w[i] = v.x; w[i + 1] = v.y; w[i + 2] = v.z; w[i + 3] = v.w;
            }
        }
    }
    __device__ __forceinline__ int get(int i) const
    {
        if constexpr (sizeof(P) == 1) return (int)((w[i >> 2] >> (8 * (i & 3))) & 0xff);
        else return (int)((w[i >> 1] >> (16 * (i & 1))) & 0xffff);
    }
};

// Write-back of a wavefront's outputs staged in LDS in destination order (the
// STG kernels of interp.hip / blockops.hip): job jl of the wavefront (lanes jl << lg ...) owns bytes
// [jl wh, (jl + 1) wh) of the staging area, wh a power of two >= 16.  Chunk c
// = bytes [16c, 16c + 16) of job 16c / wh goes to that job's destination,
// whose pointer comes from the job's first lane; a store instruction covers
// whole 64-byte segments of several jobs instead of one row piece per job.
template <int WAVE_BYTES>
__device__ __forceinline__ void stage_writeback(const uint8_t* wbase, const void* pd, int lg, int wh, int64_t wjob0,
                                                int n)
{
    wave_sync();
    const int lb = 31 - __builtin_clz(wh);                      // log2 of a job's bytes
    const int nch = (64 >> lg) << (lb - 4);
    const int l64 = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < WAVE_BYTES / 16 / 64; i++)
    {
        const int c = l64 + 64 * i;
        const int jl = (c << 4) >> lb;
        const long long dp = __shfl((long long)(intptr_t)pd, jl << lg, 64);
        if (c < nch && wjob0 + jl < n)
            stu<uint4>((uint8_t*)(intptr_t)dp + ((c << 4) & (wh - 1)), *(const uint4*)(wbase + (c << 4)));
    }
}

// MotionEstimate direction tables (motion.cpp:61-63) as packed nibbles, so a
// run-time index is a shift and mask instead of a private-memory array load:
// hex2[i] = (HEX_DX(i), HEX_DY(i)) for i = 0..7, square1[i] = (SQ_DX(i), SQ_DY(i)) for i = 0..8
__device__ __forceinline__ int hex_dx(int i) { return (int)((0x1343101ull >> (4 * i)) & 15) - 2; }
__device__ __forceinline__ int hex_dy(int i) { return (int)((0x20024420ull >> (4 * i)) & 15) - 2; }
__device__ __forceinline__ int sq_dx(int i) { return (int)((0x220020111ull >> (4 * i)) & 15) - 1; }
__device__ __forceinline__ int sq_dy(int i) { return (int)((0x202011201ull >> (4 * i)) & 15) - 1; }

} // namespace x265amd
