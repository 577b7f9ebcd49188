/* x265_amd_primitives.h — the per-call provider boundary of x265 1.9.
 *
 * x265 dispatches every pixel / transform primitive through one table,
 * `struct EncoderPrimitives` (x265_1.9/source/common/primitives.h:203-381),
 * filled by providers layered C -> intrinsics -> assembly -> aliases
 * (primitives.cpp:228-249).  This header restates that table's ABI — same
 * member order, same function-pointer types, sizeof 15008 bytes on x86-64
 * (1876 slots) — so a table filled here is the table x265 and its TestBench
 * consume, and declares the MI355X provider that slots into the layering at
 * the place of setupAssemblyPrimitives (primitives.cpp:241-242):
 *
 *     X265_NS::setupHipPrimitives(EncoderPrimitives&, int cpuMask)
 *
 * It overrides the entries it implements with
 * synchronous device-backed calls on host buffers and leaves every other slot
 * untouched, exactly like an assembly provider.  A per-call GPU round trip
 * costs tens of microseconds, so this is the compatibility path; encoders
 * that batch their work call the C ABI of x265_amd.h directly.
 *
 * Compile-time configuration mirrors x265's: X265_DEPTH 8 (pixel = uint8_t)
 * or 10/12 (pixel = uint16_t, HIGH_BIT_DEPTH), namespace X265_NS
 * (x265 for 8-bit, x265_10bit for 10-bit as in x265's multilib build).
 */
#ifndef X265_AMD_PRIMITIVES_H
#define X265_AMD_PRIMITIVES_H

#include <stddef.h>
#include <stdint.h>

#ifndef X265_DEPTH
#define X265_DEPTH 8
#endif
#ifndef X265_NS
#if X265_DEPTH == 8
#define X265_NS x265
#else
#define X265_NS x265_10bit
#endif
#endif

namespace X265_NS {

#if X265_DEPTH > 8
typedef uint16_t pixel;
typedef uint64_t sse_t;
#else
typedef uint8_t pixel;
typedef uint32_t sse_t;
#endif
typedef int16_t coeff_t;

enum { NUM_PU_SIZES = 25, NUM_CU_SIZES = 5, NUM_TR_SIZE = 4, NUM_INTRA_MODE = 35, X265_CSP_COUNT = 4 };

/* LumaPU order (primitives.h:39-53) */
enum LumaPU
{
    LUMA_4x4, LUMA_8x8, LUMA_16x16, LUMA_32x32, LUMA_64x64,
    LUMA_8x4, LUMA_4x8, LUMA_16x8, LUMA_8x16, LUMA_32x16, LUMA_16x32, LUMA_64x32, LUMA_32x64,
    LUMA_16x12, LUMA_12x16, LUMA_16x4, LUMA_4x16, LUMA_32x24, LUMA_24x32, LUMA_32x8, LUMA_8x32,
    LUMA_64x48, LUMA_48x64, LUMA_64x16, LUMA_16x64
};

/* function-pointer types (primitives.h:113-199); strides are in elements */
typedef int      (*pixelcmp_t)(const pixel*, intptr_t, const pixel*, intptr_t);
typedef int      (*pixelcmp_ss_t)(const int16_t*, intptr_t, const int16_t*, intptr_t);
typedef sse_t    (*pixel_sse_t)(const pixel*, intptr_t, const pixel*, intptr_t);
typedef sse_t    (*pixel_sse_ss_t)(const int16_t*, intptr_t, const int16_t*, intptr_t);
typedef sse_t    (*pixel_ssd_s_t)(const int16_t*, intptr_t);
typedef void     (*pixelcmp_x4_t)(const pixel*, const pixel*, const pixel*, const pixel*, const pixel*, intptr_t, int32_t*);
typedef void     (*pixelcmp_x3_t)(const pixel*, const pixel*, const pixel*, const pixel*, intptr_t, int32_t*);
typedef void     (*blockfill_s_t)(int16_t*, intptr_t, int16_t);
typedef void     (*intra_pred_t)(pixel*, intptr_t, const pixel*, int, int);
typedef void     (*intra_allangs_t)(pixel*, pixel*, pixel*, int);
typedef void     (*intra_filter_t)(const pixel*, pixel*);
typedef void     (*cpy2Dto1D_shl_t)(int16_t*, const int16_t*, intptr_t, int);
typedef void     (*cpy2Dto1D_shr_t)(int16_t*, const int16_t*, intptr_t, int);
typedef void     (*cpy1Dto2D_shl_t)(int16_t*, const int16_t*, intptr_t, int);
typedef void     (*cpy1Dto2D_shr_t)(int16_t*, const int16_t*, intptr_t, int);
typedef uint32_t (*copy_cnt_t)(int16_t*, const int16_t*, intptr_t);
typedef void     (*dct_t)(const int16_t*, int16_t*, intptr_t);
typedef void     (*idct_t)(const int16_t*, int16_t*, intptr_t);
typedef void     (*denoiseDct_t)(int16_t*, uint32_t*, const uint16_t*, int);
typedef void     (*calcresidual_t)(const pixel*, const pixel*, int16_t*, intptr_t);
typedef void     (*transpose_t)(pixel*, const pixel*, intptr_t);
typedef uint32_t (*quant_t)(const int16_t*, const int32_t*, int32_t*, int16_t*, int, int, int);
typedef uint32_t (*nquant_t)(const int16_t*, const int32_t*, int16_t*, int, int, int);
typedef void     (*dequant_scaling_t)(const int16_t*, const int32_t*, int16_t*, int, int, int);
typedef void     (*dequant_normal_t)(const int16_t*, int16_t*, int, int, int);
typedef int      (*count_nonzero_t)(const int16_t*);
typedef void     (*weightp_pp_t)(const pixel*, pixel*, intptr_t, int, int, int, int, int, int);
typedef void     (*weightp_sp_t)(const int16_t*, pixel*, intptr_t, intptr_t, int, int, int, int, int, int);
typedef void     (*scale1D_t)(pixel*, const pixel*);
typedef void     (*scale2D_t)(pixel*, const pixel*, intptr_t);
typedef void     (*downscale_t)(const pixel*, pixel*, pixel*, pixel*, pixel*, intptr_t, intptr_t, int, int);
typedef void     (*extendCURowBorder_t)(pixel*, intptr_t, int, int, int);
typedef void     (*ssim_4x4x2_core_t)(const pixel*, intptr_t, const pixel*, intptr_t, int sums[2][4]);
typedef float    (*ssim_end4_t)(int sum0[5][4], int sum1[5][4], int);
typedef uint64_t (*var_t)(const pixel*, intptr_t);
typedef void     (*filter_pp_t)(const pixel*, intptr_t, pixel*, intptr_t, int);
typedef void     (*filter_hps_t)(const pixel*, intptr_t, int16_t*, intptr_t, int, int);
typedef void     (*filter_ps_t)(const pixel*, intptr_t, int16_t*, intptr_t, int);
typedef void     (*filter_sp_t)(const int16_t*, intptr_t, pixel*, intptr_t, int);
typedef void     (*filter_ss_t)(const int16_t*, intptr_t, int16_t*, intptr_t, int);
typedef void     (*filter_hv_pp_t)(const pixel*, intptr_t, pixel*, intptr_t, int, int);
typedef void     (*filter_p2s_t)(const pixel*, intptr_t, int16_t*, intptr_t);
typedef void     (*copy_pp_t)(pixel*, intptr_t, const pixel*, intptr_t);
typedef void     (*copy_sp_t)(pixel*, intptr_t, const int16_t*, intptr_t);
typedef void     (*copy_ps_t)(int16_t*, intptr_t, const pixel*, intptr_t);
typedef void     (*copy_ss_t)(int16_t*, intptr_t, const int16_t*, intptr_t);
typedef void     (*pixel_sub_ps_t)(int16_t*, intptr_t, const pixel*, const pixel*, intptr_t, intptr_t);
typedef void     (*pixel_add_ps_t)(pixel*, intptr_t, const pixel*, const int16_t*, intptr_t, intptr_t);
typedef void     (*pixelavg_pp_t)(pixel*, intptr_t, const pixel*, intptr_t, const pixel*, intptr_t, int);
typedef void     (*addAvg_t)(const int16_t*, const int16_t*, pixel*, intptr_t, intptr_t, intptr_t);
typedef void     (*saoCuOrgE0_t)(pixel*, int8_t*, int, int8_t*, intptr_t);
typedef void     (*saoCuOrgE1_t)(pixel*, int8_t*, int8_t*, intptr_t, int);
typedef void     (*saoCuOrgE2_t)(pixel*, int8_t*, int8_t*, int8_t*, int, intptr_t);
typedef void     (*saoCuOrgE3_t)(pixel*, int8_t*, int8_t*, intptr_t, int, int);
typedef void     (*saoCuOrgB0_t)(pixel*, const int8_t*, int, int, intptr_t);
typedef void     (*saoCuStatsBO_t)(const int16_t*, const pixel*, intptr_t, int, int, int32_t*, int32_t*);
typedef void     (*saoCuStatsE0_t)(const int16_t*, const pixel*, intptr_t, int, int, int32_t*, int32_t*);
typedef void     (*saoCuStatsE1_t)(const int16_t*, const pixel*, intptr_t, int8_t*, int, int, int32_t*, int32_t*);
typedef void     (*saoCuStatsE2_t)(const int16_t*, const pixel*, intptr_t, int8_t*, int8_t*, int, int, int32_t*, int32_t*);
typedef void     (*saoCuStatsE3_t)(const int16_t*, const pixel*, intptr_t, int8_t*, int, int, int32_t*, int32_t*);
typedef void     (*sign_t)(int8_t*, const pixel*, const pixel*, const int);
typedef void     (*planecopy_cp_t)(const uint8_t*, intptr_t, pixel*, intptr_t, int, int, int);
typedef void     (*planecopy_sp_t)(const uint16_t*, intptr_t, pixel*, intptr_t, int, int, int, uint16_t);
typedef pixel    (*planeClipAndMax_t)(pixel*, intptr_t, int, int, uint64_t*, const pixel, const pixel);
typedef void     (*cutree_propagate_cost)(int*, const uint16_t*, const int32_t*, const uint16_t*, const int32_t*, const double*, int);
typedef int      (*scanPosLast_t)(const uint16_t*, const coeff_t*, uint16_t*, uint16_t*, uint8_t*, int, const uint16_t*, const int);
typedef uint32_t (*findPosFirstLast_t)(const int16_t*, const intptr_t, const uint16_t[16]);
typedef uint32_t (*costCoeffNxN_t)(const uint16_t*, const coeff_t*, intptr_t, uint16_t*, const uint8_t*, uint32_t, uint8_t*, int, int, int);
typedef uint32_t (*costCoeffRemain_t)(uint16_t*, int, int);
typedef uint32_t (*costC1C2Flag_t)(uint16_t*, intptr_t, uint8_t*, intptr_t);
typedef void     (*pelFilterLumaStrong_t)(pixel*, intptr_t, intptr_t, int32_t, int32_t);

struct EncoderPrimitives
{
    struct PU           /* indexed by LumaPU */
    {
        pixelcmp_t sad;
        pixelcmp_x3_t sad_x3;
        pixelcmp_x4_t sad_x4;
        pixelcmp_t satd;
        filter_pp_t luma_hpp;
        filter_hps_t luma_hps;
        filter_pp_t luma_vpp;
        filter_ps_t luma_vps;
        filter_sp_t luma_vsp;
        filter_ss_t luma_vss;
        filter_hv_pp_t luma_hvpp;
        pixelavg_pp_t pixelavg_pp;
        addAvg_t addAvg;
        copy_pp_t copy_pp;
        filter_p2s_t convert_p2s;
    } pu[NUM_PU_SIZES];

    struct CU           /* indexed by log2(size) - 2 */
    {
        dct_t dct;
        idct_t idct;
        calcresidual_t calcresidual;
        pixel_sub_ps_t sub_ps;
        pixel_add_ps_t add_ps;
        blockfill_s_t blockfill_s;
        copy_cnt_t copy_cnt;
        count_nonzero_t count_nonzero;
        cpy2Dto1D_shl_t cpy2Dto1D_shl;
        cpy2Dto1D_shr_t cpy2Dto1D_shr;
        cpy1Dto2D_shl_t cpy1Dto2D_shl;
        cpy1Dto2D_shr_t cpy1Dto2D_shr;
        copy_sp_t copy_sp;
        copy_ps_t copy_ps;
        copy_ss_t copy_ss;
        copy_pp_t copy_pp;
        var_t var;
        pixel_sse_t sse_pp;
        pixel_sse_ss_t sse_ss;
        pixelcmp_t psy_cost_pp;
        pixel_ssd_s_t ssd_s;
        pixelcmp_t sa8d;
        transpose_t transpose;
        intra_allangs_t intra_pred_allangs;
        intra_filter_t intra_filter;
        intra_pred_t intra_pred[NUM_INTRA_MODE];
    } cu[NUM_CU_SIZES];

    dct_t dst4x4;
    idct_t idst4x4;
    quant_t quant;
    nquant_t nquant;
    dequant_scaling_t dequant_scaling;
    dequant_normal_t dequant_normal;
    denoiseDct_t denoiseDct;
    scale1D_t scale1D_128to64;
    scale2D_t scale2D_64to32;
    ssim_4x4x2_core_t ssim_4x4x2_core;
    ssim_end4_t ssim_end_4;
    sign_t sign;
    saoCuOrgE0_t saoCuOrgE0;
    saoCuOrgE1_t saoCuOrgE1, saoCuOrgE1_2Rows;
    saoCuOrgE2_t saoCuOrgE2[2];
    saoCuOrgE3_t saoCuOrgE3[2];
    saoCuOrgB0_t saoCuOrgB0;
    saoCuStatsBO_t saoCuStatsBO;
    saoCuStatsE0_t saoCuStatsE0;
    saoCuStatsE1_t saoCuStatsE1;
    saoCuStatsE2_t saoCuStatsE2;
    saoCuStatsE3_t saoCuStatsE3;
    downscale_t frameInitLowres;
    cutree_propagate_cost propagateCost;
    extendCURowBorder_t extendRowBorder;
    planecopy_cp_t planecopy_cp;
    planecopy_sp_t planecopy_sp;
    planecopy_sp_t planecopy_sp_shl;
    planeClipAndMax_t planeClipAndMax;
    weightp_sp_t weight_sp;
    weightp_pp_t weight_pp;
    scanPosLast_t scanPosLast;
    findPosFirstLast_t findPosFirstLast;
    costCoeffNxN_t costCoeffNxN;
    costCoeffRemain_t costCoeffRemain;
    costC1C2Flag_t costC1C2Flag;
    pelFilterLumaStrong_t pelFilterLumaStrong[2];

    struct Chroma       /* one per colour space, PU tables indexed by LumaPU */
    {
        struct PUChroma
        {
            pixelcmp_t satd;
            filter_pp_t filter_vpp;
            filter_ps_t filter_vps;
            filter_sp_t filter_vsp;
            filter_ss_t filter_vss;
            filter_pp_t filter_hpp;
            filter_hps_t filter_hps;
            addAvg_t addAvg;
            copy_pp_t copy_pp;
            filter_p2s_t p2s;
        } pu[NUM_PU_SIZES];

        struct CUChroma
        {
            pixelcmp_t sa8d;
            pixel_sse_t sse_pp;
            pixel_sub_ps_t sub_ps;
            pixel_add_ps_t add_ps;
            copy_ps_t copy_ps;
            copy_sp_t copy_sp;
            copy_ss_t copy_ss;
            copy_pp_t copy_pp;
        } cu[NUM_CU_SIZES];
    } chroma[X265_CSP_COUNT];
};

/* The MI355X provider.  cpuMask is accepted for signature compatibility with
 * setupAssemblyPrimitives and ignored.  Call after the C provider and before
 * setupAliasPrimitives, as x265_setup_primitives orders providers.  Throws no
 * exceptions; if no gfx950 device is usable the table is left unchanged. */
void setupHipPrimitives(EncoderPrimitives& p, int cpuMask);

} /* namespace X265_NS */

extern "C" {
/* C entry of the same provider for FFI callers: `table` points at an
 * EncoderPrimitives of the given depth.  Returns 0, or X265AMD_ENODEV when no
 * gfx950 device is usable (table untouched).  Reports how many slots were
 * overridden through *overridden (may be NULL). */
int x265amd_setup_primitives(void* table, int depth, int* overridden);
/* sizeof(EncoderPrimitives) this library was built with (15008 on x86-64) */
size_t x265amd_primitives_size(void);
/* Sticky status of the per-call provider.  x265's primitives have no error
 * channel (primitives.h:113-199 return void / a value), so the provider records
 * the FIRST failure of any call it served (a HIP status of a copy, launch or
 * synchronisation, or X265AMD_ENOMEM for a host thread whose staging buffers
 * could not be allocated), returns zeroed outputs from then on, and the caller
 * maps a non-zero status onto x265_encoder_encode() < 0 (x265.h:1351-1359), as
 * oracle/hip_encoder_main.cpp does.  0 while every call succeeded. */
int x265amd_provider_status(void);
/* Clears the sticky status (tests). */
void x265amd_provider_clear_status(void);
}

#endif /* X265_AMD_PRIMITIVES_H */
