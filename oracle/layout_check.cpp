// layout_check.cpp — TEST INFRASTRUCTURE: proves include/x265_amd_primitives.h
// restates the reference's `struct EncoderPrimitives` ABI exactly.
//
// Built only where /root/reference exists (tests/test_layout.py):
//   g++ -std=gnu++11 -DX265_DEPTH=<8|10> ... layout_check.cpp
// The repository header is included into namespace `amdcheck`, the
// reference's primitives.h into `x265`; every member's offset and the total
// size must agree.  Prints one line per checked member group.
#include <cstddef>
#include <cstdio>

#define X265_NS amdcheck
#include "../include/x265_amd_primitives.h"
#undef X265_NS
#define X265_NS x265
#include "primitives.h"

#define CHECK(member)                                                                              \
    do {                                                                                           \
        size_t a = offsetof(amdcheck::EncoderPrimitives, member), b = offsetof(x265::EncoderPrimitives, member); \
        if (a != b) { printf("MISMATCH %s: %zu vs %zu\n", #member, a, b); bad++; }                 \
        checked++;                                                                                 \
    } while (0)

int main()
{
    int bad = 0, checked = 0;
#define PU(f) CHECK(pu[0].f); CHECK(pu[24].f);
    PU(sad) PU(sad_x3) PU(sad_x4) PU(satd) PU(luma_hpp) PU(luma_hps) PU(luma_vpp) PU(luma_vps) PU(luma_vsp)
    PU(luma_vss) PU(luma_hvpp) PU(pixelavg_pp) PU(addAvg) PU(copy_pp) PU(convert_p2s)
#define CU(f) CHECK(cu[0].f); CHECK(cu[4].f);
    CU(dct) CU(idct) CU(calcresidual) CU(sub_ps) CU(add_ps) CU(blockfill_s) CU(copy_cnt) CU(count_nonzero)
    CU(cpy2Dto1D_shl) CU(cpy2Dto1D_shr) CU(cpy1Dto2D_shl) CU(cpy1Dto2D_shr) CU(copy_sp) CU(copy_ps) CU(copy_ss)
    CU(copy_pp) CU(var) CU(sse_pp) CU(sse_ss) CU(psy_cost_pp) CU(ssd_s) CU(sa8d) CU(transpose)
    CU(intra_pred_allangs) CU(intra_filter) CU(intra_pred[0]) CU(intra_pred[34])
    CHECK(dst4x4); CHECK(idst4x4); CHECK(quant); CHECK(nquant); CHECK(dequant_scaling); CHECK(dequant_normal);
    CHECK(denoiseDct); CHECK(scale1D_128to64); CHECK(scale2D_64to32); CHECK(ssim_4x4x2_core); CHECK(ssim_end_4);
    CHECK(sign); CHECK(saoCuOrgE0); CHECK(saoCuOrgE1); CHECK(saoCuOrgE1_2Rows); CHECK(saoCuOrgE2[1]);
    CHECK(saoCuOrgE3[1]); CHECK(saoCuOrgB0); CHECK(saoCuStatsBO); CHECK(saoCuStatsE3); CHECK(frameInitLowres);
    CHECK(propagateCost); CHECK(extendRowBorder); CHECK(planecopy_cp); CHECK(planecopy_sp_shl);
    CHECK(planeClipAndMax); CHECK(weight_sp); CHECK(weight_pp); CHECK(scanPosLast); CHECK(findPosFirstLast);
    CHECK(costCoeffNxN); CHECK(costCoeffRemain); CHECK(costC1C2Flag); CHECK(pelFilterLumaStrong[1]);
#define CPU(f) CHECK(chroma[0].pu[0].f); CHECK(chroma[3].pu[24].f);
    CPU(satd) CPU(filter_vpp) CPU(filter_vps) CPU(filter_vsp) CPU(filter_vss) CPU(filter_hpp) CPU(filter_hps)
    CPU(addAvg) CPU(copy_pp) CPU(p2s)
#define CCU(f) CHECK(chroma[0].cu[0].f); CHECK(chroma[3].cu[4].f);
    CCU(sa8d) CCU(sse_pp) CCU(sub_ps) CCU(add_ps) CCU(copy_ps) CCU(copy_sp) CCU(copy_ss) CCU(copy_pp)
    if (sizeof(amdcheck::EncoderPrimitives) != sizeof(x265::EncoderPrimitives))
    {
        printf("MISMATCH sizeof: %zu vs %zu\n", sizeof(amdcheck::EncoderPrimitives), sizeof(x265::EncoderPrimitives));
        bad++;
    }
    printf("depth %d: %d member offsets checked, sizeof %zu, %d mismatches\n", X265_DEPTH, checked,
           sizeof(x265::EncoderPrimitives), bad);
    return bad ? 1 : 0;
}
