// exchange.cpp — the reference-row exchange of the frame-parallel shard as
// native code behind the C ABI (include/x265_amd.h, x265amd_comm_* / x265amd_exchange).
//
// x265 frame threads share reconstructed reference rows through memory: FrameFilter publishes a
// row (m_reconRowCount, framefilter.cpp:520) and the frames referencing the picture wait on it
// (frameencoder.cpp:516-531).  Across GPUs the publication is a transfer: every step of the
// schedule (x265amd_schedule, schedule.cpp) sends the final bands of this rank's reference
// pictures to the ranks whose frames read them and receives the bands its own frames read.
// Here one step's transfers are one RCCL group of point-to-point sends and receives (xGMI
// peer-to-peer between the GPUs of a node), enqueued on the caller's stream: the step's work, its
// exchange and the next step's work follow each other on the stream with no host round trip.
// Both sides of a link list their transfers in the same order (the schedule's canonical order),
// which is what RCCL's point-to-point matching requires.
//
// librccl is loaded at the first call: the copy already in the process when there is one (the
// PyTorch runtime links its own), else librccl.so.1 from the ROCm installation, else the path in
// X265AMD_RCCL.  No RCCL type appears in the C ABI: the unique id is 128 opaque bytes the caller
// distributes over any channel (torch.distributed, MPI, a file).
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <mutex>

#include "../../../include/x265_amd.h"

namespace {

struct Rccl
{
    bool ok = false;
    const char* bound = nullptr;   // which library the symbols came from
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
};

Rccl& rccl()
{
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        // 1. an explicit library (X265AMD_RCCL); 2. RCCL already loaded in the process — PyTorch's copy
        // is librccl.so.1 or a hashed name under torch/lib, so look the symbols up globally first and
        // then by both sonames with RTLD_NOLOAD; 3. ROCm's librccl.so.1.  A second RCCL runtime next to
        // the process's own would run its own communicators and proxy threads.
        void* h = nullptr;
        const char* how = nullptr;
        bool global = false;           // RTLD_DEFAULT is a null handle: tracked separately
        if (const char* p = getenv("X265AMD_RCCL"))
            if ((h = dlopen(p, RTLD_NOW | RTLD_LOCAL))) how = p;
        if (!h && dlsym(RTLD_DEFAULT, "ncclGetUniqueId")) { global = true; how = "already loaded (global lookup)"; }
        if (!h && !global && (h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD))) how = "already loaded (librccl.so.1)";
        if (!h && !global && (h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD))) how = "already loaded (librccl.so)";
        if (!h && !global && (h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL))) how = "librccl.so.1 (loaded here)";
        if (!h && !global) return;
        if (global) h = RTLD_DEFAULT;
        if (getenv("X265AMD_RCCL_VERBOSE")) fprintf(stderr, "[x265amd] RCCL bound: %s\n", how);
        r.bound = how;
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
        r.init_rank = (decltype(r.init_rank))dlsym(h, "ncclCommInitRank");
        r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
        r.send = (decltype(r.send))dlsym(h, "ncclSend");
        r.recv = (decltype(r.recv))dlsym(h, "ncclRecv");
        r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
        r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
        r.ok = r.get_unique_id && r.init_rank && r.destroy && r.send && r.recv && r.group_start && r.group_end;
    });
    return r;
}

} // namespace

struct x265amd_comm
{
    ncclComm_t comm;
    int nranks, rank;
};

static_assert(sizeof(ncclUniqueId) == X265AMD_COMM_ID_BYTES, "RCCL unique id size");

extern "C" const char* x265amd_comm_backend(void)
{
    Rccl& r = rccl();
    return r.ok ? r.bound : nullptr;
}

extern "C" int x265amd_comm_unique_id(uint8_t* id)
{
    if (!id) return X265AMD_EINVAL;
    Rccl& r = rccl();
    if (!r.ok) return X265AMD_ENODEV;
    ncclUniqueId u;
    if (r.get_unique_id(&u) != ncclSuccess) return X265AMD_ENODEV;
    memcpy(id, &u, sizeof(u));
    return 0;
}

extern "C" int x265amd_comm_create(x265amd_comm** out, const uint8_t* id, int nranks, int rank)
{
    if (!out || !id || nranks <= 0 || rank < 0 || rank >= nranks) return X265AMD_EINVAL;
    *out = nullptr;
    Rccl& r = rccl();
    if (!r.ok) return X265AMD_ENODEV;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return X265AMD_ENODEV;
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclComm_t c = nullptr;
    if (r.init_rank(&c, nranks, u, rank) != ncclSuccess) return X265AMD_ENODEV;
    *out = new x265amd_comm{ c, nranks, rank };
    return 0;
}

extern "C" int x265amd_comm_destroy(x265amd_comm* c)
{
    if (!c) return 0;
    int rc = rccl().destroy(c->comm) == ncclSuccess ? 0 : X265AMD_ENODEV;
    delete c;
    return rc;
}

extern "C" int x265amd_exchange(x265amd_comm* c, const x265amd_transfer* xfers, int count, void* stream)
{
    if (!c || count < 0 || (count && !xfers)) return X265AMD_EINVAL;
    for (int i = 0; i < count; i++)
        if (xfers[i].peer < 0 || xfers[i].peer >= c->nranks || (xfers[i].bytes && !xfers[i].buf))
            return X265AMD_EINVAL;
    if (!count) return 0;
    Rccl& r = rccl();
    hipStream_t s = (hipStream_t)stream;
    if (r.group_start() != ncclSuccess) return X265AMD_ENODEV;
    int rc = 0;
    for (int i = 0; i < count && !rc; i++)
    {
        const x265amd_transfer& t = xfers[i];
        ncclResult_t e = t.send ? r.send(t.buf, t.bytes, ncclUint8, t.peer, c->comm, s)
                                : r.recv(t.buf, t.bytes, ncclUint8, t.peer, c->comm, s);
        if (e != ncclSuccess) rc = X265AMD_ENODEV;
    }
    if (r.group_end() != ncclSuccess) rc = X265AMD_ENODEV;
    return rc;
}
