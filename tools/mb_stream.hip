// mb_stream.hip — streaming-shape calibration for the coefficient kernels
// (quant / dequant / transforms read and write compact int16 / int32 arrays).
// Not product code: it answers "what per-lane shape reaches the HBM ceiling".
//
//   hipcc --offload-arch=gfx950 -O3 tools/mb_stream.hip -o /tmp/mbs && /tmp/mbs
//
// Every variant moves >= 1.5 GB of distinct bytes per launch; GB/s counts
// algorithmic bytes (read + written) over the hipEvent time of one launch.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// copy, K v4u per lane; block covers K * 256 consecutive v4u (loads first)
template <int K, bool NT>
__global__ __launch_bounds__(256) void k_copy(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n)
{
    const size_t b = (size_t)blockIdx.x * 256 * K + threadIdx.x;
    v4u v[K];
#pragma unroll
    for (int k = 0; k < K; k++)
    {
        const size_t i = b + (size_t)k * 256;
        if (i < n) v[k] = NT ? __builtin_nontemporal_load(s + i) : s[i];
    }
#pragma unroll
    for (int k = 0; k < K; k++)
    {
        const size_t i = b + (size_t)k * 256;
        if (i < n)
        {
            if (NT) __builtin_nontemporal_store(v[k], d + i);
            else d[i] = v[k];
        }
    }
}

// quant-shaped: per lane and chunk, 8 B in (4 int16), 8 B + 16 B out (int16 + int32)
template <int K, bool NT>
__global__ __launch_bounds__(256) void k_qshape(const v2u* __restrict__ s, v2u* __restrict__ o, v4u* __restrict__ dl,
                                                size_t n)
{
    const size_t b = (size_t)blockIdx.x * 256 * K + threadIdx.x;
    v2u v[K];
#pragma unroll
    for (int k = 0; k < K; k++)
    {
        const size_t i = b + (size_t)k * 256;
        if (i < n) v[k] = NT ? __builtin_nontemporal_load(s + i) : s[i];
    }
#pragma unroll
    for (int k = 0; k < K; k++)
    {
        const size_t i = b + (size_t)k * 256;
        if (i < n)
        {
            const v2u a = v2u{v[k].x * 3u, v[k].y ^ 0x55u};
            const v4u c = v4u{v[k].x, v[k].y, v[k].x + 1u, v[k].y + 1u};
            if (NT) { __builtin_nontemporal_store(a, o + i); __builtin_nontemporal_store(c, dl + i); }
            else { o[i] = a; dl[i] = c; }
        }
    }
}

// int16 -> int16 in 8-B chunks (dequant-shaped), K per lane
template <int K, bool NT>
__global__ __launch_bounds__(256) void k_dshape(const v2u* __restrict__ s, v2u* __restrict__ o, size_t n)
{
    const size_t b = (size_t)blockIdx.x * 256 * K + threadIdx.x;
    v2u v[K];
#pragma unroll
    for (int k = 0; k < K; k++)
    {
        const size_t i = b + (size_t)k * 256;
        if (i < n) v[k] = NT ? __builtin_nontemporal_load(s + i) : s[i];
    }
#pragma unroll
    for (int k = 0; k < K; k++)
    {
        const size_t i = b + (size_t)k * 256;
        if (i < n)
        {
            const v2u a = v2u{v[k].x * 3u, v[k].y ^ 0x55u};
            if (NT) __builtin_nontemporal_store(a, o + i);
            else o[i] = a;
        }
    }
}

// each lane copies 32 (64) contiguous bytes as two (four) 16-B loads: the 4x4-transform
// lane-per-job shape (wave-instructions at a 32-B / 64-B lane stride)
template <int PER>
__global__ __launch_bounds__(256) void k_copy_lane(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n)
{
    const size_t b = ((size_t)blockIdx.x * 256 + threadIdx.x) * PER;
    if (b + PER > n) return;
    v4u v[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) v[k] = s[b + k];
#pragma unroll
    for (int k = 0; k < PER; k++) d[b + k] = v[k];
}

static float time_ms(void (*launch)(void*), void* arg, int reps)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    launch(arg);
    launch(arg);
    hipDeviceSynchronize();
    float tot = 0;
    for (int r = 0; r < reps; r++)
    {
        hipEventRecord(e0, 0);
        launch(arg);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        tot += ms;
    }
    return tot / reps;
}

struct Bufs
{
    void *a, *b, *c;
    size_t bytes;
};

template <int K, bool NT>
static void L_copy(void* p)
{
    Bufs* B = (Bufs*)p;
    const size_t n = B->bytes / 2 / 16;
    hipLaunchKernelGGL((k_copy<K, NT>), dim3((n + 256 * K - 1) / (256 * K)), dim3(256), 0, 0, (const v4u*)B->a,
                       (v4u*)B->b, n);
}
template <int PER>
static void L_lane(void* p)
{
    Bufs* B = (Bufs*)p;
    const size_t n = B->bytes / 2 / 16;
    hipLaunchKernelGGL((k_copy_lane<PER>), dim3((n / PER + 255) / 256), dim3(256), 0, 0, (const v4u*)B->a, (v4u*)B->b, n);
}
template <int K, bool NT>
static void L_q(void* p)
{
    Bufs* B = (Bufs*)p;
    const size_t n = B->bytes / 32;       // 8 in + 24 out per chunk
    hipLaunchKernelGGL((k_qshape<K, NT>), dim3((n + 256 * K - 1) / (256 * K)), dim3(256), 0, 0, (const v2u*)B->a,
                       (v2u*)B->b, (v4u*)B->c, n);
}
template <int K, bool NT>
static void L_d(void* p)
{
    Bufs* B = (Bufs*)p;
    const size_t n = B->bytes / 16;
    hipLaunchKernelGGL((k_dshape<K, NT>), dim3((n + 256 * K - 1) / (256 * K)), dim3(256), 0, 0, (const v2u*)B->a,
                       (v2u*)B->b, n);
}

int main()
{
    Bufs B;
    B.bytes = (size_t)3 << 29;   // 1.5 GiB of algorithmic traffic per launch
    CHECK(hipMalloc(&B.a, B.bytes));
    CHECK(hipMalloc(&B.b, B.bytes));
    CHECK(hipMalloc(&B.c, B.bytes));
    CHECK(hipMemset(B.a, 1, B.bytes));
    struct V { const char* name; void (*f)(void*); };
    const V vs[] = {
        {"copy16_k1", L_copy<1, false>}, {"copy16_k2", L_copy<2, false>}, {"copy16_k4", L_copy<4, false>},
        {"copy16_k8", L_copy<8, false>}, {"copy_lane32", L_lane<2>}, {"copy_lane64", L_lane<4>}, {"copy16_k4_nt", L_copy<4, true>}, {"copy16_k8_nt", L_copy<8, true>},
        {"quant_k1", L_q<1, false>}, {"quant_k2", L_q<2, false>}, {"quant_k4", L_q<4, false>}, {"quant_k8", L_q<8, false>},
        {"quant_k4_nt", L_q<4, true>}, {"quant_k8_nt", L_q<8, true>},
        {"deq_k1", L_d<1, false>}, {"deq_k4", L_d<4, false>}, {"deq_k8", L_d<8, false>}, {"deq_k4_nt", L_d<4, true>},
        {"deq_k8_nt", L_d<8, true>},
    };
    for (const V& v : vs)
    {
        const float ms = time_ms(v.f, &B, 10);
        CHECK(hipGetLastError());
        printf("%-14s %8.4f ms %7.1f GB/s %.3f of 8 TB/s\n", v.name, ms, B.bytes / (ms * 1e-3) / 1e9,
               B.bytes / (ms * 1e-3) / 8e12);
    }
    return 0;
}
