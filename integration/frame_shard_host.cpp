// frame_shard_host.cpp — the frame-parallel shard of DESIGN.md §6 driven from C++ alone: the plan
// (x265amd_schedule), the per-step loop filters of every CTU-row band (x265amd_deblock_rows /
// _sao_apply_rows / _extend_border_rows) and the reference-row exchange (x265amd_exchange over RCCL),
// with no Python and no torch — the shape a C++ x265 build running one process per GPU would have.
//
// x265 terms: FrameEncoder (frame j of the GOP, on rank j mod world, encoder.cpp:649-650) codes its
// CTU rows band by band once every reference has published the rows it needs
// (frameencoder.cpp:516-531); FrameFilter deblocks a band, and the previous band becomes final
// (SAO, border extension, framefilter.cpp:300-520) and is published: here it is sent to every rank
// whose frames reference the picture and received into their reference stores, one RCCL group per
// step in the canonical order of x265amd_schedule's transfers.  The reconstruction a real encoder
// writes is stood in for by a deterministic source picture (as in bench.py --mode pipeline).
//
//   frame_shard_host W H FRAMES BAND_ROWS WORLD RANK IDFILE [SEGMENT] [REPS]
//
// Rank 0 writes the communicator id to IDFILE; the other ranks wait for it.  Every rank's reference
// pictures are finished in their own buffers and reach even the rank's own store through the
// communicator (loop-back transfers), so one rank exercises the whole exchange.  Checked at the end
// on every rank: each local picture equals the whole-frame deblock -> SAO -> border chain
// (x265amd_deblock / _sao_apply / _extend_border) of the same picture, and each store slot of a
// picture this rank produced equals that picture; slots filled by other ranks are printed as
// checksums (the launcher compares them with the producers').  Prints one JSON line per rank.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <set>
#include <vector>

#include "../include/x265_amd.h"

#define CHECK(x)                                                                          \
    do                                                                                    \
    {                                                                                     \
        int rc_ = (int)(x);                                                               \
        if (rc_)                                                                          \
        {                                                                                 \
            fprintf(stderr, "frame_shard_host: %s failed: %d (%s)\n", #x, rc_, x265amd_strerror(rc_)); \
            exit(2);                                                                      \
        }                                                                                 \
    } while (0)

namespace {

uint32_t mix(uint32_t a)
{
    a ^= a >> 16; a *= 0x7feb352d; a ^= a >> 15; a *= 0x846ca68b; a ^= a >> 16;
    return a;
}

struct Geo
{
    int W, H, pw, ph, mx, my, stride, rows, cmx, cmy, cstride, crows;
    size_t psize[3];
    Geo(int w, int h) : W(w), H(h)
    {
        pw = (w + 63) / 64 * 64; ph = (h + 63) / 64 * 64;
        mx = 96; my = 80;                                    // picyuv.cpp:62-80: 64 + 32, 64 + 16
        stride = pw + 2 * mx; rows = ph + 2 * my;
        cmx = mx; cmy = my / 2;
        cstride = pw / 2 + 2 * cmx; crows = ph / 2 + 2 * cmy;
        psize[0] = (size_t)rows * stride;
        psize[1] = psize[2] = (size_t)crows * cstride;
    }
    int st(int p) const { return p ? cstride : stride; }
    int mxp(int p) const { return p ? cmx : mx; }
    int myp(int p) const { return p ? cmy : my; }
    int rowsp(int p) const { return p ? crows : rows; }
};

struct Pic { uint8_t* p[3]; };

Pic alloc_pic(const Geo& g)
{
    Pic r;
    for (int p = 0; p < 3; p++)
    {
        CHECK(hipMalloc((void**)&r.p[p], g.psize[p]));
        CHECK(hipMemset(r.p[p], 0, g.psize[p]));
    }
    return r;
}

uint8_t* org(const Geo& g, const Pic& pic, int p) { return pic.p[p] + (size_t)g.myp(p) * g.st(p) + g.mxp(p); }

} // namespace

int main(int argc, char** argv)
{
    if (argc < 8)
    {
        fprintf(stderr, "usage: %s W H FRAMES BAND_ROWS WORLD RANK IDFILE [SEGMENT] [REPS]\n", argv[0]);
        return 1;
    }
    const int W = atoi(argv[1]), H = atoi(argv[2]), frames = atoi(argv[3]), band_rows = atoi(argv[4]);
    const int world = atoi(argv[5]), rank = atoi(argv[6]);
    const char* idfile = argv[7];
    const int segment = argc > 8 ? atoi(argv[8]) : frames, reps = argc > 9 ? atoi(argv[9]) : 3;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    {
        fprintf(stderr, "frame_shard_host: no device\n");
        return 3;
    }
    CHECK(hipSetDevice(rank % ndev));
    const Geo g(W, H);

    // ---- plan
    const int ctu_rows = g.ph / 64, nb = (ctu_rows + band_rows - 1) / band_rows;
    x265amd_sched_config cfg = { frames, segment, 4, 1, 3, 2, ctu_rows, band_rows, 2, world };
    std::vector<x265amd_sched_frame> fr(frames);
    std::vector<int> step((size_t)frames * nb);
    int nsteps = 0;
    CHECK(x265amd_schedule(&cfg, fr.data(), step.data(), &nsteps));
    auto pub = [&](int j, int c) { return step[(size_t)j * nb + std::min(c + 1, nb - 1)]; };
    std::vector<std::vector<int>> users(frames);
    for (int j = 0; j < frames; j++)
        for (int i = 0; i < fr[j].nrefs; i++) users[fr[j].refs[i]].push_back(j);
    std::vector<int> local;
    for (int j = 0; j < frames; j++)
        if (fr[j].rank == rank) local.push_back(j);
    std::set<int> store_set;
    for (int j : local)
        for (int i = 0; i < fr[j].nrefs; i++) store_set.insert(fr[j].refs[i]);
    std::vector<int> kof(frames, -1), sof(frames, -1);
    for (size_t k = 0; k < local.size(); k++) kof[local[k]] = (int)k;
    std::vector<int> store(store_set.begin(), store_set.end());
    for (size_t i = 0; i < store.size(); i++) sof[store[i]] = (int)i;

    // ---- communicator
    uint8_t id[X265AMD_COMM_ID_BYTES];
    if (rank == 0)
    {
        CHECK(x265amd_comm_unique_id(id));
        char tmp[4096];
        snprintf(tmp, sizeof(tmp), "%s.tmp%d", idfile, (int)getpid());
        FILE* f = fopen(tmp, "wb");
        if (!f || fwrite(id, 1, sizeof(id), f) != sizeof(id) || fclose(f) || rename(tmp, idfile))
        {
            fprintf(stderr, "frame_shard_host: cannot write %s\n", idfile);
            return 2;
        }
    }
    else
    {
        for (int tries = 0;; tries++)
        {
            FILE* f = fopen(idfile, "rb");
            if (f && fread(id, 1, sizeof(id), f) == sizeof(id)) { fclose(f); break; }
            if (f) fclose(f);
            if (tries > 6000) { fprintf(stderr, "frame_shard_host: no id in %s\n", idfile); return 2; }
            usleep(10000);
        }
    }
    x265amd_comm* comm = nullptr;
    CHECK(x265amd_comm_create(&comm, id, world, rank));
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

    // ---- pictures: source (the stand-in reconstruction), work (deblocked in place), final, store
    const int F = (int)local.size();
    std::vector<Pic> src(F), work(F), fin(F), ref_work(F), ref_fin(F), st(store.size());
    for (int k = 0; k < F; k++)
    {
        src[k] = alloc_pic(g); work[k] = alloc_pic(g); fin[k] = alloc_pic(g);
        ref_work[k] = alloc_pic(g); ref_fin[k] = alloc_pic(g);
        for (int p = 0; p < 3; p++)
        {
            const int w = p ? W / 2 : W, h = p ? H / 2 : H;
            std::vector<uint8_t> host(g.psize[p], 0);
            for (int y = 0; y < h; y++)
                for (int x = 0; x < w; x++)
                {
                    // a smooth pan plus noise: edges for the deblocking filter, bands for SAO
                    const int poc = fr[local[k]].poc;
                    const int v = ((x + 2 * poc) * 3 + (y + poc) * 2) / (p ? 3 : 5) + (int)(mix(x * 7919 + y * 104729 + poc * 31 + p) % 23);
                    host[(size_t)(y + g.myp(p)) * g.st(p) + x + g.mxp(p)] = (uint8_t)(v & 255);
                }
            CHECK(hipMemcpy(src[k].p[p], host.data(), g.psize[p], hipMemcpyHostToDevice));
        }
    }
    for (size_t i = 0; i < store.size(); i++) st[i] = alloc_pic(g);

    // CU units and SAO parameters (shared by every picture)
    const int hu = H / 4, wu = W / 4, nctu = (g.pw / 64) * (g.ph / 64);
    std::vector<x265amd_deblock_unit> units((size_t)hu * wu);
    for (int y = 0; y < hu; y++)
        for (int x = 0; x < wu; x++)
        {
            x265amd_deblock_unit& u = units[(size_t)y * wu + x];
            memset(&u, 0, sizeof(u));
            const uint32_t cu = mix((uint32_t)((y / 4) * 977 + x / 4));
            u.cu_log2 = 4; u.tu_log2 = 3; u.qp = 32;
            u.flags = (uint8_t)((cu % 4 == 0 ? 1 : 0) | (mix(y * 131 + x) % 2 ? 2 : 0));
            u.ref_idx[0] = 0; u.ref_idx[1] = -1;
            u.mv[0][0] = (int16_t)((int)(cu % 13) - 6); u.mv[0][1] = (int16_t)((int)((cu >> 8) % 13) - 6);
        }
    std::vector<x265amd_sao_param> prm((size_t)3 * nctu);
    for (int i = 0; i < 3 * nctu; i++)
    {
        const uint32_t r = mix(i * 7 + 1);
        prm[i].type = (int8_t)((int)(r % 6) - 1);
        prm[i].band = (uint8_t)((r >> 4) % 32);
        for (int k = 0; k < 4; k++) prm[i].offset[k] = (int8_t)((int)((r >> (8 + 3 * k)) % 7) - 3);
    }
    for (int i = 2 * nctu; i < 3 * nctu; i++) prm[i].type = prm[i - nctu].type;   // Cr uses Cb's type
    x265amd_deblock_unit* d_units;
    x265amd_sao_param* d_prm;
    CHECK(hipMalloc((void**)&d_units, units.size() * sizeof(units[0])));
    CHECK(hipMalloc((void**)&d_prm, prm.size() * sizeof(prm[0])));
    CHECK(hipMemcpy(d_units, units.data(), units.size() * sizeof(units[0]), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_prm, prm.data(), prm.size() * sizeof(prm[0]), hipMemcpyHostToDevice));

    auto dbk_of = [&](const Pic& wk) {
        x265amd_deblock_frame d;
        memset(&d, 0, sizeof(d));
        d.width = W; d.height = H;
        for (int p = 0; p < 3; p++) d.plane[p] = org(g, wk, p);
        d.stride = g.stride; d.cstride = g.cstride; d.units = d_units; d.unit_stride = wu; d.is_p = 1;
        return d;
    };
    auto sao_of = [&](const Pic& wk, const Pic& out) {
        x265amd_sao_frame a;
        memset(&a, 0, sizeof(a));
        a.width = W; a.height = H; a.ctu_log2 = 6; a.luma_on = 1; a.chroma_on = 1;
        for (int p = 0; p < 3; p++) { a.src[p] = org(g, wk, p); a.dst[p] = org(g, out, p); }
        a.stride = g.stride; a.cstride = g.cstride; a.params = d_prm;
        return a;
    };
    auto bor_of = [&](const Pic& out, int p) {
        x265amd_border_plane b;
        b.plane = org(g, out, p); b.stride = g.st(p);
        b.width = p ? W / 2 : W; b.height = p ? H / 2 : H; b.margin_x = g.mxp(p); b.margin_y = g.myp(p);
        return b;
    };
    // buffer rows [start, end) of band b of plane p (full stride; margins with the first / last band)
    auto region = [&](int b, int p) {
        const int c = 64 >> (p ? 1 : 0), r0 = b * band_rows, r1 = std::min((b + 1) * band_rows, ctu_rows);
        const int start = b == 0 ? 0 : g.myp(p) + r0 * c;
        const int end = b == nb - 1 ? g.rowsp(p) : g.myp(p) + r1 * c;
        return std::make_pair((size_t)start * g.st(p), (size_t)end * g.st(p));
    };
    // per step: this rank's transfer table, canonical order (frame, band, destination rank)
    std::vector<std::vector<x265amd_transfer>> xfers(nsteps);
    for (int j = 0; j < frames; j++)
    {
        if (!fr[j].is_ref || users[j].empty()) continue;
        std::set<int> dests;
        for (int u : users[j]) dests.insert(fr[u].rank);
        for (int c = 0; c < nb; c++)
            for (int d : dests)
            {
                const int src_rank = fr[j].rank;
                if (src_rank != rank && d != rank) continue;
                for (int p = 0; p < 3; p++)
                {
                    const auto rg = region(c, p);
                    const size_t bytes = rg.second - rg.first;
                    if (src_rank == rank)
                        xfers[pub(j, c)].push_back({ fin[kof[j]].p[p] + rg.first, bytes, d, 1 });
                    if (d == rank)
                        xfers[pub(j, c)].push_back({ st[sof[j]].p[p] + rg.first, bytes, src_rank, 0 });
                }
            }
    }

    auto run_steps = [&]() {
        for (int k = 0; k < F; k++)
            for (int p = 0; p < 3; p++)
                CHECK(hipMemcpyAsync(work[k].p[p], src[k].p[p], g.psize[p], hipMemcpyDeviceToDevice, s));
        for (int stp = 0; stp < nsteps; stp++)
        {
            std::vector<x265amd_deblock_frame> dk;
            std::vector<int32_t> rows;
            std::vector<x265amd_sao_frame> sa;
            std::vector<int32_t> crow;
            std::vector<x265amd_border_plane> bp;
            std::vector<int32_t> brow;
            for (int j : local)
                for (int b = 0; b < nb; b++)
                {
                    const int y0 = b * band_rows * 64, y1 = std::min((b + 1) * band_rows * 64, H);
                    if (step[(size_t)j * nb + b] == stp)
                    {
                        dk.push_back(dbk_of(work[kof[j]]));
                        rows.push_back(y0); rows.push_back(y1);
                    }
                    if (pub(j, b) == stp)
                    {
                        sa.push_back(sao_of(work[kof[j]], fin[kof[j]]));
                        crow.push_back(b * band_rows); crow.push_back(std::min((b + 1) * band_rows, ctu_rows));
                        for (int p = 0; p < 3; p++)
                        {
                            bp.push_back(bor_of(fin[kof[j]], p));
                            const int sh = p ? 1 : 0;
                            brow.insert(brow.end(), { y0 >> sh, y1 >> sh, b == 0, b == nb - 1 });
                        }
                    }
                }
            if (!dk.empty()) CHECK(x265amd_deblock_rows(8, (int)dk.size(), dk.data(), rows.data(), s));
            if (!sa.empty())
            {
                CHECK(x265amd_sao_apply_rows(8, (int)sa.size(), sa.data(), crow.data(), s));
                CHECK(x265amd_extend_border_rows(8, (int)bp.size(), bp.data(), brow.data(), s));
            }
            CHECK(x265amd_exchange(comm, xfers[stp].data(), (int)xfers[stp].size(), s));
        }
    };

    run_steps();                                             // warm-up (and the run that is checked)
    CHECK(hipStreamSynchronize(s));
    // ---- check: whole-frame chain per local picture, stores of local pictures
    int bad = 0;
    for (int k = 0; k < F; k++)
    {
        for (int p = 0; p < 3; p++)
            CHECK(hipMemcpyAsync(ref_work[k].p[p], src[k].p[p], g.psize[p], hipMemcpyDeviceToDevice, s));
        x265amd_deblock_frame d = dbk_of(ref_work[k]);
        x265amd_sao_frame a = sao_of(ref_work[k], ref_fin[k]);
        x265amd_border_plane b3[3] = { bor_of(ref_fin[k], 0), bor_of(ref_fin[k], 1), bor_of(ref_fin[k], 2) };
        CHECK(x265amd_deblock(8, 1, &d, s));
        CHECK(x265amd_sao_apply(8, 1, &a, s));
        CHECK(x265amd_extend_border(8, 3, b3, s));
    }
    CHECK(hipStreamSynchronize(s));
    std::vector<uint8_t> h1, h2;
    uint64_t store_sum = 0;
    for (int k = 0; k < F; k++)
        for (int p = 0; p < 3; p++)
        {
            h1.resize(g.psize[p]); h2.resize(g.psize[p]);
            CHECK(hipMemcpy(h1.data(), fin[k].p[p], g.psize[p], hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(h2.data(), ref_fin[k].p[p], g.psize[p], hipMemcpyDeviceToHost));
            // the defined area: picture + margins (CTU-alignment rows / columns beyond are never written)
            const int rows = 2 * g.myp(p) + (p ? H / 2 : H), cols = 2 * g.mxp(p) + (p ? W / 2 : W);
            for (int y = 0; y < rows && !bad; y++)
                if (memcmp(&h1[(size_t)y * g.st(p)], &h2[(size_t)y * g.st(p)], cols))
                {
                    fprintf(stderr, "rank %d: picture %d plane %d row %d differs from the whole-frame chain\n", rank,
                            local[k], p, y);
                    bad++;
                }
        }
    for (size_t i = 0; i < store.size(); i++)
        for (int p = 0; p < 3; p++)
        {
            h1.resize(g.psize[p]);
            CHECK(hipMemcpy(h1.data(), st[i].p[p], g.psize[p], hipMemcpyDeviceToHost));
            uint64_t sum = 1469598103934665603ull;
            for (uint8_t v : h1) sum = (sum ^ v) * 1099511628211ull;
            store_sum += sum * (2 * i + 2 * p + 1);
            if (kof[store[i]] >= 0)
            {
                h2.resize(g.psize[p]);
                CHECK(hipMemcpy(h2.data(), fin[kof[store[i]]].p[p], g.psize[p], hipMemcpyDeviceToHost));
                if (memcmp(h1.data(), h2.data(), g.psize[p]))
                {
                    fprintf(stderr, "rank %d: store slot of picture %d plane %d != its final picture\n", rank, store[i], p);
                    bad++;
                }
            }
        }

    // ---- timing
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; r++) run_steps();
    CHECK(hipStreamSynchronize(s));
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
    size_t nx = 0, bytes = 0;
    for (auto& v : xfers)
        for (auto& t : v)
        {
            nx++;
            if (t.send) bytes += t.bytes;
        }
    printf("{\"rank\": %d, \"world\": %d, \"pictures\": %d, \"local\": %d, \"stores\": %zu, \"steps\": %d, "
           "\"transfers\": %zu, \"sent_MB\": %.2f, \"ms_per_sequence\": %.3f, \"mismatches\": %d, "
           "\"store_checksum\": \"%016llx\"}\n",
           rank, world, frames, F, store.size(), nsteps, nx, bytes / 1e6, dt * 1e3, bad,
           (unsigned long long)store_sum);
    CHECK(x265amd_comm_destroy(comm));
    return bad ? 1 : 0;
}
