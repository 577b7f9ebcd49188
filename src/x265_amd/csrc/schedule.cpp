// schedule.cpp — the frame-parallel schedule of SURVEY.md §8(e) (include/x265_amd.h,
// x265amd_schedule): which frames reference which, who encodes them, and in which step each
// CTU-row band of each frame can run.  Host code only (no device calls): the multi-GPU
// pipeline (src/x265_amd/pipeline.py, bench.py --mode pipeline) and its CPU tests all read the
// same plan from here.
//
// GOP model — x265 1.9 at --preset medium with a fixed mini-GOP:
//   * bframes = 4, b-pyramid on, maxNumReferences = 3 (param.cpp:145, 148, 174); L1 holds at
//     most 2 pictures with b-pyramid (dpb.h:57-58);
//   * each closed segment starts with an I frame; then mini-GOPs of bframes + 1 pictures: the
//     anchor P, the B-ref in the middle (list[bframes / 2], slicetype.cpp:993-996) and the
//     non-reference b pictures; encode order P, B-ref, b ... (slicetype.cpp:1050-1078); a short
//     last mini-GOP keeps the same shape with fewer B pictures;
//   * references (dpb.cpp:149-150, 188-207): L0 = the nearest coded reference pictures before the
//     picture in display order (at most maxNumReferences), L1 (B only) = the nearest coded ones
//     after it (at most 2).  I, P and B-ref pictures are references; b pictures are not and are
//     never waited on or sent.
// Frame j (encode order over all segments) is encoded by rank j mod world (encoder.cpp:649-650
// round robin).
//
// Row dependencies — a frame's CTU row r waits until each reference has published
// r + refLagRows rows (frameencoder.cpp:516-531), i.e. rows 0 .. r + lag - 1.  A band of rows
// [r0, r1) therefore needs the reference band holding row r1 - 2 + lag.  A band becomes final
// (deblocked, SAO-filtered, border-extended) in the step of the NEXT band's deblocking
// (framefilter.cpp:255-260, 520), the last band in its own step.  The list schedule below puts
// every (frame, band) in the earliest step after its previous band and after every reference band
// it needs was published in an earlier step.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../../include/x265_amd.h"

namespace {

struct Pic { int poc, type, enc; };

} // namespace

extern "C" int x265amd_schedule(const x265amd_sched_config* c, x265amd_sched_frame* frames, int* step, int* nsteps)
{
    if (!c || !frames || !step || !nsteps) return X265AMD_EINVAL;
    if (c->frames <= 0 || c->segment_frames <= 0 || c->bframes < 0 || c->bframes > 16 || c->max_refs < 1 ||
        c->max_refs > 4 || c->max_refs_l1 < 0 || c->max_refs_l1 > 2 || c->ctu_rows <= 0 || c->band_rows <= 0 ||
        c->lag < 1 || c->world <= 0)
        return X265AMD_EINVAL;
    const int nb = (c->ctu_rows + c->band_rows - 1) / c->band_rows;
    int j = 0;
    for (int seg0 = 0; seg0 < c->frames; seg0 += c->segment_frames)
    {
        const int L = std::min(c->segment_frames, c->frames - seg0);
        // encode order of the segment (display pocs relative to the segment)
        std::vector<Pic> order;
        order.push_back({ 0, X265AMD_FRAME_I, 0 });
        for (int n = 0; n < L - 1;)
        {
            const int r = std::min(c->bframes + 1, L - 1 - n);      // pictures in this mini-GOP
            order.push_back({ n + r, X265AMD_FRAME_P, 0 });
            const int nb_ = r - 1;
            const int bref = (c->b_pyramid && nb_ > 1) ? n + 1 + nb_ / 2 : -1;
            if (bref >= 0) order.push_back({ bref, X265AMD_FRAME_BREF, 0 });
            for (int p = n + 1; p < n + r; p++)
                if (p != bref) order.push_back({ p, X265AMD_FRAME_B, 0 });
            n += r;
        }
        std::vector<Pic> coded_refs;                                // reference pictures coded so far
        for (size_t k = 0; k < order.size(); k++, j++)
        {
            Pic& p = order[k];
            p.enc = j;
            x265amd_sched_frame& f = frames[j];
            memset(&f, 0, sizeof(f));
            f.poc = seg0 + p.poc;
            f.type = p.type;
            f.is_ref = p.type != X265AMD_FRAME_B;
            f.rank = j % c->world;
            if (p.type != X265AMD_FRAME_I)
            {
                std::vector<Pic> before, after;
                for (const Pic& q : coded_refs) (q.poc < p.poc ? before : after).push_back(q);
                std::sort(before.begin(), before.end(), [](const Pic& a, const Pic& b) { return a.poc > b.poc; });
                std::sort(after.begin(), after.end(), [](const Pic& a, const Pic& b) { return a.poc < b.poc; });
                for (int i = 0; i < (int)before.size() && i < c->max_refs; i++) f.refs[f.nrefs++] = before[i].enc;
                f.nrefs_l0 = f.nrefs;
                if (p.type != X265AMD_FRAME_P)
                    for (int i = 0; i < (int)after.size() && i < c->max_refs_l1; i++) f.refs[f.nrefs++] = after[i].enc;
            }
            if (f.is_ref) coded_refs.push_back(p);
        }
    }
    // list schedule
    auto band_of = [&](int row) { return std::min(row, c->ctu_rows - 1) / c->band_rows; };
    auto pub = [&](int fr, int band) { return step[fr * nb + std::min(band + 1, nb - 1)]; };
    int last = 0;
    for (int f = 0; f < c->frames; f++)
        for (int b = 0; b < nb; b++)
        {
            const int r1 = std::min((b + 1) * c->band_rows, c->ctu_rows);
            const int need = band_of(r1 - 2 + c->lag);
            int s = b ? step[f * nb + b - 1] + 1 : 0;
            for (int i = 0; i < frames[f].nrefs; i++) s = std::max(s, pub(frames[f].refs[i], need) + 1);
            step[f * nb + b] = s;
            last = std::max(last, s);
        }
    *nsteps = last + 1;
    return 0;
}
