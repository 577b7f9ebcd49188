// hostreg.h — page-locking of caller-owned host buffers by the encoder sessions (lookahead.cpp,
// mesession.cpp) and the check that they are unregistered while still allocated.
//
// The sessions hipHostRegister the encoder's own buffers (Lowres planes, PicYuv reconstruction planes)
// so uploads from them are direct DMAs.  A registered range is a userptr mapping in the GPU's page
// tables: memory freed while registered (munmap of a large allocation, or a trimmed heap) leaves the GPU
// a mapping of pages the process no longer owns, and a later copy through it faults the device.  So
// every unregister first asks the kernel whether the whole range is still mapped (mincore: ENOMEM when
// any page is not) and counts the ranges that were not — x265amd_host_unregister_stale(), which the
// encoder binding prints and the GPU tests require to stay 0.
#pragma once

#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <vector>

#include "devsync.h"

namespace x265amd_hostreg {

inline std::atomic<long long>& stale_count()
{
    static std::atomic<long long> n{ 0 };
    return n;
}

// is every page of [p, p + bytes) mapped in this process?
inline bool range_mapped(const void* p, size_t bytes)
{
    const uintptr_t page = (uintptr_t)sysconf(_SC_PAGESIZE);
    const uintptr_t a = (uintptr_t)p & ~(page - 1);
    const uintptr_t e = ((uintptr_t)p + bytes + page - 1) & ~(page - 1);
    std::vector<unsigned char> vec((e - a) / page);
    return mincore((void*)a, e - a, vec.data()) == 0 || errno != ENOMEM;
}

// unregister a range this session registered; `bytes` = the size it was registered with
inline void unregister(const void* p, size_t bytes)
{
    if (!p) return;
    if (!range_mapped(p, bytes)) stale_count().fetch_add(1, std::memory_order_relaxed);
    DevSyncScope quiet;                        // (hipHostUnregister waits for every running kernel)
    (void)hipHostUnregister((void*)p);
    (void)hipGetLastError();
}

} // namespace x265amd_hostreg
