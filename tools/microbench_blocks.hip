// microbench_blocks.hip — achievable HBM bandwidth for the access shapes the
// primitive kernels use (calibration for the kernel rooflines, not product code).
//
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_blocks.hip -o /tmp/mb && /tmp/mb
//
// Patterns (all over >= 1.5 GB, cache-cold, disjoint):
//   stream16   linear copy, 16 B per lane (the practical HBM ceiling)
//   blkNxN_vB  copy of NxN 8-bit blocks tiled in an 8192-wide plane into
//              compact slots, B bytes per lane per row
//   rdNxN_vB   read two NxN blocks per job, write 4 bytes (SAD-shaped)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_stream(const uint4* __restrict__ s, uint4* __restrict__ d, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}

// one job = one NxN block; lanes per job = N*N/(B*R) with R rows per lane
template <int N, int B, int R>
__global__ void k_blk(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int W, int per_row, int njobs)
{
    constexpr int LPR = N / B;                 // lanes per row
    constexpr int LPJ = LPR * (N / R);         // lanes per job
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int job = tid / LPJ, l = tid % LPJ;
    if (job >= njobs) return;
    const int bx = job % per_row, by = job / per_row;
    const int x = (l % LPR) * B, y0 = (l / LPR) * R;
    const uint8_t* s = src + (size_t)(by * N + y0) * W + bx * N + x;
    uint8_t* d = dst + (size_t)job * N * N + y0 * N + x;
    if constexpr (B == 16)
    {
        uint4 v[R];
#pragma unroll
        for (int r = 0; r < R; r++) v[r] = *(const uint4*)(s + (size_t)r * W);
#pragma unroll
        for (int r = 0; r < R; r++) *(uint4*)(d + r * N) = v[r];
    }
    else
    {
        uint2 v[R];
#pragma unroll
        for (int r = 0; r < R; r++) v[r] = *(const uint2*)(s + (size_t)r * W);
#pragma unroll
        for (int r = 0; r < R; r++) *(uint2*)(d + r * N) = v[r];
    }
}

// the same copy, with per-job int64 element offsets loaded from memory (as the C ABI does)
template <int N, int B, int R, bool XCD = false>
__global__ void k_blk_off(const uint8_t* __restrict__ src, const int64_t* __restrict__ soff, uint8_t* __restrict__ dst,
                          const int64_t* __restrict__ doff, int W, int njobs)
{
    constexpr int LPR = N / B;
    constexpr int LPJ = LPR * (N / R);
    uint32_t blk = blockIdx.x;
    if (XCD)
    {
        const uint32_t nb = gridDim.x, q = nb >> 3, rr = nb & 7, x = blk & 7;
        blk = x * q + (x < rr ? x : rr) + (blk >> 3);
    }
    const int tid = blk * blockDim.x + threadIdx.x;
    const int job = tid / LPJ, l = tid % LPJ;
    if (job >= njobs) return;
    const int x = (l % LPR) * B, y0 = (l / LPR) * R;
    const uint8_t* s = src + soff[job] + (size_t)y0 * W + x;
    uint8_t* d = dst + doff[job] + y0 * N + x;
    uint2 v[R];
#pragma unroll
    for (int r = 0; r < R; r++) v[r] = *(const uint2*)(s + (size_t)r * W);
#pragma unroll
    for (int r = 0; r < R; r++) *(uint2*)(d + r * N) = v[r];
}

__global__ void k_make_off(int64_t* soff, int64_t* doff, int N, int W, int per_row, int njobs)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= njobs) return;
    soff[j] = (int64_t)(j / per_row) * N * W + (j % per_row) * N;
    doff[j] = (int64_t)j * N * N;
}

template <int N, int B, int R>
__global__ void k_rd(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b, int* __restrict__ out, int W,
                     int per_row, int njobs)
{
    constexpr int LPR = N / B;
    constexpr int LPJ = LPR * (N / R);
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int job = tid / LPJ, l = tid % LPJ;
    if (job >= njobs) return;
    const int bx = job % per_row, by = job / per_row;
    const int x = (l % LPR) * B, y0 = (l / LPR) * R;
    const size_t o = (size_t)(by * N + y0) * W + bx * N + x;
    uint32_t s = 0;
#pragma unroll
    for (int r = 0; r < R; r++)
    {
        if constexpr (B == 16)
        {
            const uint4 u = *(const uint4*)(a + o + (size_t)r * W), v = *(const uint4*)(b + o + (size_t)r * W);
            s = __builtin_amdgcn_sad_u8(u.x, v.x, s); s = __builtin_amdgcn_sad_u8(u.y, v.y, s);
            s = __builtin_amdgcn_sad_u8(u.z, v.z, s); s = __builtin_amdgcn_sad_u8(u.w, v.w, s);
        }
        else
        {
            const uint2 u = *(const uint2*)(a + o + (size_t)r * W), v = *(const uint2*)(b + o + (size_t)r * W);
            s = __builtin_amdgcn_sad_u8(u.x, v.x, s); s = __builtin_amdgcn_sad_u8(u.y, v.y, s);
        }
    }
    for (int m = 1; m < LPJ && m < 64; m <<= 1) s += __shfl_xor(s, m, 64);
    if (l == 0) out[job] = (int)s;
}

template <typename F>
static float timeit(F f)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    f(); f();
    (void)hipEventRecord(e0);
    for (int i = 0; i < 10; i++) f();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 10;
}

template <int N, int B, int R>
static void run_blk(const uint8_t* A, const uint8_t* Bp, uint8_t* D, int* O, int W, size_t plane)
{
    const int per_row = W / N;
    const int njobs = (int)(plane / ((size_t)N * N)) / 2;          // half the plane: disjoint, cold
    constexpr int LPJ = (N / B) * (N / R);
    const int threads = njobs * LPJ, grid = (threads + 255) / 256;
    float ms = timeit([&] { hipLaunchKernelGGL((k_blk<N, B, R>), dim3(grid), dim3(256), 0, 0, A, D, W, per_row, njobs); });
    printf("blk%dx%d_v%d_r%d   %7.1f GB/s (copy, read+write)\n", N, N, B, R, 2.0 * njobs * N * N / (ms * 1e6));
    ms = timeit([&] { hipLaunchKernelGGL((k_rd<N, B, R>), dim3(grid), dim3(256), 0, 0, A, Bp, O, W, per_row, njobs); });
    printf("rd%dx%d_v%d_r%d    %7.1f GB/s (two blocks read)\n", N, N, B, R, (2.0 * njobs * N * N + 4.0 * njobs) / (ms * 1e6));
}

int main()
{
    const size_t plane = (size_t)1536 << 20;     // 1.5 GiB per plane
    const int W = 8192;
    uint8_t *A, *Bp, *D;
    int* O;
    CHECK(hipMalloc(&A, plane)); CHECK(hipMalloc(&Bp, plane)); CHECK(hipMalloc(&D, plane));
    CHECK(hipMalloc(&O, plane / 16));
    CHECK(hipMemset(A, 1, plane)); CHECK(hipMemset(Bp, 2, plane));
    {
        const size_t n = plane / 16;
        float ms = timeit([&] { hipLaunchKernelGGL(k_stream, dim3(256 * 64), dim3(256), 0, 0, (const uint4*)A, (uint4*)D, n); });
        printf("stream16         %7.1f GB/s (copy, read+write)\n", 2.0 * plane / (ms * 1e6));
    }
    run_blk<64, 16, 1>(A, Bp, D, O, W, plane);
    run_blk<64, 16, 4>(A, Bp, D, O, W, plane);
    run_blk<64, 8, 1>(A, Bp, D, O, W, plane);
    run_blk<64, 8, 4>(A, Bp, D, O, W, plane);
    run_blk<16, 16, 1>(A, Bp, D, O, W, plane);
    run_blk<16, 8, 2>(A, Bp, D, O, W, plane);
    run_blk<8, 8, 1>(A, Bp, D, O, W, plane);
    run_blk<8, 8, 2>(A, Bp, D, O, W, plane);
    run_blk<8, 8, 8>(A, Bp, D, O, W, plane);
    {
        // 8x8 copy with offsets read from memory, 1 and 2 rows per lane
        const int N = 8, njobs = (int)(plane / 64) / 2, per_row = W / N;
        int64_t *so, *dof;
        CHECK(hipMalloc(&so, 8 * (size_t)njobs)); CHECK(hipMalloc(&dof, 8 * (size_t)njobs));
        hipLaunchKernelGGL(k_make_off, dim3((njobs + 255) / 256), dim3(256), 0, 0, so, dof, N, W, per_row, njobs);
        float ms = timeit([&] { hipLaunchKernelGGL((k_blk_off<8, 8, 2>), dim3((njobs * 4 + 255) / 256), dim3(256), 0, 0, A, so, D, dof, W, njobs); });
        printf("blk8x8_v8_r2_off %7.1f GB/s (copy, int64 offsets from memory)\n", 2.0 * njobs * 64 / (ms * 1e6));
        ms = timeit([&] { hipLaunchKernelGGL((k_blk_off<8, 8, 4>), dim3((njobs * 2 + 255) / 256), dim3(256), 0, 0, A, so, D, dof, W, njobs); });
        printf("blk8x8_v8_r4_off %7.1f GB/s (copy, int64 offsets from memory)\n", 2.0 * njobs * 64 / (ms * 1e6));
        ms = timeit([&] { hipLaunchKernelGGL((k_blk_off<8, 8, 4, true>), dim3((njobs * 2 + 255) / 256), dim3(256), 0, 0, A, so, D, dof, W, njobs); });
        printf("blk8x8_v8_r4_off_xcd %7.1f GB/s (same, XCD-contiguous block remap)\n", 2.0 * njobs * 64 / (ms * 1e6));
        ms = timeit([&] { hipLaunchKernelGGL((k_blk_off<8, 8, 2, true>), dim3((njobs * 4 + 255) / 256), dim3(256), 0, 0, A, so, D, dof, W, njobs); });
        printf("blk8x8_v8_r2_off_xcd %7.1f GB/s (same, XCD-contiguous block remap)\n", 2.0 * njobs * 64 / (ms * 1e6));
    }
    CHECK(hipDeviceSynchronize());
    return 0;
}
