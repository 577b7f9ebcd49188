// probe: can the host write and read fine-grained device memory (hipExtMallocWithFlags(hipDeviceMallocFinegrained))
// directly (large BAR)?  Prints the device's isLargeBar and, per allocation kind, whether a host memset / readback works
// and how long 12 KB of host stores take.  One-off measurement tool (round 6).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

__global__ void k_sum(const unsigned* p, int n, unsigned* out)
{
    unsigned s = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += p[i];
    atomicAdd(out, s);
}

int main()
{
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) != hipSuccess) { printf("no device\n"); return 1; }
    printf("isLargeBar %d\n", prop.isLargeBar);
    fflush(stdout);
    const size_t bytes = 1 << 20;
    unsigned* p = nullptr;
    if (hipExtMallocWithFlags((void**)&p, bytes, hipDeviceMallocFinegrained) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) == hipSuccess)
        printf("type %d hostPointer %p devicePointer %p\n", (int)at.type, at.hostPointer, at.devicePointer);
    fflush(stdout);
    // host access through the pointer itself (unified VA on large-BAR systems)
    auto t0 = std::chrono::steady_clock::now();
    for (int rep = 0; rep < 100; rep++)
        for (int i = 0; i < 3072; i++) p[i] = (unsigned)(i + rep);
    __builtin_ia32_sfence();
    auto t1 = std::chrono::steady_clock::now();
    printf("host stores: 100 x 12 KB in %.1f us (%.2f us each)\n",
           std::chrono::duration<double, std::micro>(t1 - t0).count(),
           std::chrono::duration<double, std::micro>(t1 - t0).count() / 100);
    unsigned r = 0;
    t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 64; i++) r += p[i];
    t1 = std::chrono::steady_clock::now();
    printf("host reads: 64 words in %.1f us (sum %u)\n", std::chrono::duration<double, std::micro>(t1 - t0).count(), r);
    unsigned* d = nullptr;
    (void)hipMalloc((void**)&d, 4);
    (void)hipMemset(d, 0, 4);
    hipLaunchKernelGGL(k_sum, dim3(1), dim3(256), 0, 0, p, 3072, d);
    unsigned h = 0;
    (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    unsigned want = 0;
    for (int i = 0; i < 3072; i++) want += (unsigned)(i + 99);
    printf("device sum %u want %u -> %s\n", h, want, h == want ? "host stores visible to the device" : "MISMATCH");
    (void)hipFree(p);
    (void)hipFree(d);
    return 0;
}
