// rdojob.h — one request of the resident residual-coding server (X265AMD_RDO_SERVER, round 6): the TU batches
// and 8x8 psy jobs of one inter CU (or the SAO statistics of one CTU), laid out in the request's slot of mapped, coherent host memory by the
// posting thread (rdosession.cpp) and served by k_rdo_server (tu.hip), which polls the slots' sequence words.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../../include/x265_amd.h"

namespace x265amd {

// a request of the second kind (kind 1): SAO::calcSaoStatsCu of one CTU, all three planes (sao.cpp:772-943).
// The CTU's deblocked windows and source blocks are the request's staged bytes; the statistics go to host memory.
struct RdoSaoJob
{
    int32_t w, h;                  // picture size (luma)
    int32_t ctu_log2, nd, cx, cy;  // CTU size, --sao-non-deblock, CTU column and row
    int32_t hs, vs;                // chroma shifts
    int64_t rec_at[3], fenc_at[3]; // byte offset in the staged bytes of each plane's CTU origin
    int64_t rs[3], fs[3];          // their strides (pixels)
    int32_t* stats;                // [3][5][33] m_offsetOrg, then
    int32_t* count;                // [3][5][33] m_count (device addresses of host memory)
};

struct RdoJob
{
    x265amd_tu_batch tu[2];        // luma TUs (32x32), chroma TUs of both planes (16x16)
    x265amd_cmp_batch psy[4];      // 8x8 psy: luma (fenc, pred), luma (fenc, recon), chroma (fenc, pred), (fenc, recon)
    RdoSaoJob sao;
    uint32_t kind;                 // 0: the CU's residual coding (tu, psy); 1: SAO statistics (sao)
    uint32_t pad[2];               // kind 0: pad[0] = the CU's 8x8 blocks B (> 0: each psy energy's block also
                                   // gets its sse_pp 8x8 at out + 2 B)
    uint32_t seq;                  // the request's sequence number; written last (release)
};

constexpr size_t kRdoJobFromEnd = 2048;    // the RdoJob's offset from the end of its slot
constexpr size_t kRdoDoneFromEnd = 64;     // the done word (= seq once served) from the end of the slot
constexpr size_t kRdoStampsFromEnd = 256;  // X265AMD_RDO_TIMING: 6 real-time stamps of the request's phases
// slot layout (direct and server mode): the CU's packed inputs from 0 (fenc Y Cb Cr, pred Y Cb Cr; room for a
// 64x64 CU), its descriptors from rdo_desc_at(), its outputs from rdo_out_at(); the server stages the first
// rdo_out_at() bytes in LDS
constexpr size_t kRdoMaxPix = 64 * 64 + 2 * 32 * 32;
constexpr size_t kRdoDescBytes = 4096;
__host__ __device__ constexpr size_t rdo_desc_at(size_t bytes_per_pixel) { return 2 * kRdoMaxPix * bytes_per_pixel; }
__host__ __device__ constexpr size_t rdo_out_at(size_t bytes_per_pixel) { return rdo_desc_at(bytes_per_pixel) + kRdoDescBytes; }
constexpr int kRdoServerMaxOwned = 64;     // slots one server workgroup polls (nslots <= 64 x workgroups)
constexpr int kRdoBellWord = 16;           // ctl[kRdoBellWord + g]: workgroup g's doorbell (ctl[0]: stop)
constexpr int kRdoCtlWords = kRdoBellWord + 256;
static_assert(sizeof(RdoJob) + kRdoDoneFromEnd <= kRdoJobFromEnd, "RdoJob does not fit its place in the slot");

struct RdoServerArgs
{
    uint8_t* base;                 // device address of slot 0 (slot k at base + k * region)
    uint64_t region;
    int nslots;
    int depth;
    uint32_t* ctl;                 // mapped: ctl[0] = stop
    uint64_t max_ticks;            // lifetime bound in s_memrealtime ticks (100 MHz)
    int timing;                    // write the phase stamps of every request (kRdoStampsFromEnd)
    // device-memory input slots (large-BAR hosts, X265AMD_RDO_SERVER_VRAM): slot k's staged bytes at
    // in_base + k * in_region, its RdoJob right after them (rdo_out_at); null: both in the host slot
    uint8_t* in_base;
    uint64_t in_region;
};

} // namespace x265amd

// launches the server (nwg workgroups) on `stream`; csrc/tu.hip
extern "C" int x265amd_rdo_server_launch(const x265amd::RdoServerArgs* a, int nwg, int cooperative, void* stream);
