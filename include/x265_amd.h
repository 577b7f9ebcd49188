/* x265_amd.h — C ABI of the MI355X (gfx950) primitive provider for x265 1.9.
 *
 * This is the drop-in boundary.  x265 calls its primitives
 * one block at a time through the function table `EncoderPrimitives`
 * (x265_1.9/source/common/primitives.h:203-381); a GPU cannot sit under
 * single calls of 50 ns - 25 us, so each entry below executes a BATCH of
 * independent calls of one table entry.  Job i of a batch is exactly the
 * reference call
 *
 *     primitive(a_base + a_off[i], a_stride, b_base + b_off[i], b_stride, ...)
 *
 * with the same argument meaning, the same integer results and the same
 * "write only inside the WxH block" contract as the C primitive it replaces
 * (pixel.cpp / dct.cpp / ipfilter.cpp / intrapred.cpp).  The per-call table
 * entry each function replaces is cited on the function.
 *
 * Conventions
 *   - all pointers are DEVICE pointers (hipMalloc / torch tensors);
 *   - strides and offsets are in ELEMENTS (pixels or int16), as in x265;
 *   - `depth` is the pixel bit depth: 8 => pixels are uint8_t,
 *     10 or 12 => pixels are uint16_t (x265 HIGH_BIT_DEPTH builds);
 *   - `stream` is a hipStream_t (NULL = default stream); calls only enqueue
 *     work and never synchronise;
 *   - return value: 0 on success, otherwise a hipError_t code or one of the
 *     X265AMD_E* codes below (unsupported shape/op).  x265 primitives have no
 *     error channel (primitives.h typedefs return void/int); the caller maps
 *     a non-zero status to x265_encoder_encode() < 0 (x265.h:1351-1359).
 *   - Block shapes: every (w, h) that has a non-NULL entry in the reference
 *     table for that family (luma, chroma 4:2:0 / 4:2:2 / 4:4:4).
 */
#ifndef X265_AMD_H
#define X265_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 1: per-shape batched entries; 2: + the *_grouped multi-shape entries */
#define X265AMD_ABI_VERSION 2

enum
{
    X265AMD_OK = 0,
    X265AMD_EINVAL = 1000,   /* unsupported op / shape / depth */
    X265AMD_ENODEV = 1001,   /* no gfx950 device */
    X265AMD_ENOMEM = 1002    /* device / pinned staging allocation failed */
};

/* loop-filter chroma layout value for a luma-only (4:0:0) picture; 0 / 1 = 4:2:0, 2 = 4:2:2,
 * 3 = 4:4:4 (x265's X265_CSP_I400 is 0 — translate it, do not pass internalCsp through) */
#define X265AMD_CSP_I400 4

/* ----------------------------------------------------------------- runtime */
int         x265amd_abi_version(void);
/* Select the HIP device for this host thread; returns 0 or a hipError_t. */
int         x265amd_set_device(int device);
/* Number of HIP devices visible to the process (0 on a host without one); returns 0 or a hipError_t. */
int         x265amd_device_count(int* count);
/* Human-readable message for a status code returned by any entry. */
const char* x265amd_strerror(int status);
/* Name of the gfx target the library was compiled for ("gfx950"). */
const char* x265amd_target(void);
/* sizeof of a descriptor type of this header by name ("x265amd_me_batch", ...), 0 if unknown: for bindings
 * in other languages to check their layouts */
int         x265amd_sizeof(const char* type);

/* -------------------------------------------------------- a4 a6 a7 a8 a15
 * Pixel comparison of block A against block B, one scalar per job.
 *   X265AMD_SAD     pu[].sad          pixel.cpp:39-54       out int32
 *   X265AMD_SATD    pu[].satd         pixel.cpp:163-242     out int32
 *   X265AMD_SA8D    cu[].sa8d         pixel.cpp:244-322     out int32
 *                   (w,h multiple of 16: one (x+2)>>2 per 16x16; multiple of
 *                    8: per 8x8; 4x4 / 4x8: satd, as the table aliases them)
 *   X265AMD_SSE_PP  cu[].sse_pp       pixel.cpp:120-139     out uint64 (sse_t)
 *   X265AMD_SSE_SS  cu[].sse_ss       (int16 operands)      out uint64 (sse_t)
 *   X265AMD_PSY     cu[].psy_cost_pp  pixel.cpp:672-703     out int32 (w == h)
 *   X265AMD_SSD_S   cu[].ssd_s        pixel.cpp:324-336     out uint64, B unused
 *   X265AMD_VAR     cu[].var          pixel.cpp:649-666     out uint64, B unused
 * sse_t is uint32 at 8-bit (the value wraps mod 2^32 exactly as the
 * reference's) and uint64 at 10/12-bit; both are returned zero-extended. */
enum
{
    X265AMD_SAD = 0,
    X265AMD_SATD,
    X265AMD_SA8D,
    X265AMD_SSE_PP,
    X265AMD_SSE_SS,
    X265AMD_PSY,
    X265AMD_SSD_S,
    X265AMD_VAR
};
int x265amd_pixelcmp(int op, int depth, int w, int h, int n,
                     const void* a, intptr_t a_stride, const int64_t* a_off,
                     const void* b, intptr_t b_stride, const int64_t* b_off,
                     void* out, void* stream);

/* ---------------------------------------------------------------------- a5
 * pu[].sad_x3 / pu[].sad_x4 (pixel.cpp:73-118): one fenc block against
 * nref = 3 or 4 reference blocks sharing ref_stride.  The reference fixes the
 * fenc stride to FENC_STRIDE (64); here it is a parameter.
 * ref_off holds nref offsets per job (job-major); out holds nref int32 per job. */
int x265amd_sad_multi(int nref, int depth, int w, int h, int n,
                      const void* fenc, intptr_t fenc_stride, const int64_t* fenc_off,
                      const void* ref, intptr_t ref_stride, const int64_t* ref_off,
                      int32_t* out, void* stream);

/* Grouped forms: `count` batches of one op but any mix of block shapes (and
 * operands) in as few launches as possible — batches of the same kernel class
 * share a launch, up to 16 per launch.  Equivalent to calling
 * x265amd_pixelcmp / x265amd_sad_multi once per batch, in order; the whole
 * call is rejected (nothing enqueued) if any batch has an invalid shape.
 * For sad_multi, b/b_stride/b_off are the reference blocks (nref per job). */
typedef struct x265amd_cmp_batch
{
    int w, h, n;
    const void* a;
    intptr_t a_stride;
    const int64_t* a_off;
    const void* b;
    intptr_t b_stride;
    const int64_t* b_off;
    void* out;
} x265amd_cmp_batch;
int x265amd_pixelcmp_grouped(int op, int depth, int count, const x265amd_cmp_batch* batches, void* stream);
int x265amd_sad_multi_grouped(int nref, int depth, int count, const x265amd_cmp_batch* batches, void* stream);

/* ---------------------------------------------------------------------- a9
 * Sub-pel interpolation (ipfilter.cpp:40-372).  taps = 8 (luma pu[].luma_*)
 * or 4 (chroma[].pu[].filter_*).  Operand types per op:
 *   HPP  pixel -> pixel      luma_hpp / filter_hpp
 *   HPS  pixel -> int16      luma_hps / filter_hps (is_row_ext applies)
 *   VPP  pixel -> pixel      luma_vpp / filter_vpp
 *   VPS  pixel -> int16      luma_vps / filter_vps
 *   VSP  int16 -> pixel      luma_vsp / filter_vsp
 *   VSS  int16 -> int16      luma_vss / filter_vss
 *   HVPP pixel -> pixel      luma_hvpp (taps must be 8)
 *   P2S  pixel -> int16      convert_p2s / p2s (taps ignored)
 * coeff[i] = coeffIdx of job i; for HVPP bits 0-3 = idxX, bits 4-7 = idxY.
 * src_off[i] points at the block origin exactly like the reference's `src`
 * argument (the filter reaches taps/2-1 pixels before and taps/2 after it). */
enum
{
    X265AMD_HPP = 0,
    X265AMD_HPS,
    X265AMD_VPP,
    X265AMD_VPS,
    X265AMD_VSP,
    X265AMD_VSS,
    X265AMD_HVPP,
    X265AMD_P2S
};
int x265amd_interp(int op, int taps, int depth, int w, int h, int n,
                   const void* src, intptr_t src_stride, const int64_t* src_off,
                   void* dst, intptr_t dst_stride, const int64_t* dst_off,
                   const uint8_t* coeff, int is_row_ext, void* stream);
/* Grouped form: `count` batches of one (op, taps), any mix of block shapes,
 * packed into as few launches as possible (same semantics as one
 * x265amd_interp call per batch, in order; rejected whole if any batch is
 * invalid). */
typedef struct x265amd_interp_batch
{
    int w, h, n, is_row_ext;
    const void* src;
    intptr_t src_stride;
    const int64_t* src_off;
    void* dst;
    intptr_t dst_stride;
    const int64_t* dst_off;
    const uint8_t* coeff;
} x265amd_interp_batch;
int x265amd_interp_grouped(int op, int taps, int depth, int count, const x265amd_interp_batch* batches,
                           void* stream);

/* ----------------------------------------------------------------- a10 a11
 * 2-D transforms (dct.cpp:442-610): cu[].dct / cu[].idct for size 4..32 and
 * dst4x4 / idst4x4.  Forward kinds read `src` with src_stride and write the
 * N*N coefficients with dst_stride (the reference writes them contiguous:
 * pass dst_stride = size); inverse kinds read with src_stride (reference:
 * contiguous) and write the residual with dst_stride. */
enum
{
    X265AMD_DCT = 0,
    X265AMD_IDCT,
    X265AMD_DST,
    X265AMD_IDST
};
int x265amd_transform(int kind, int depth, int size, int n,
                      const int16_t* src, intptr_t src_stride, const int64_t* src_off,
                      int16_t* dst, intptr_t dst_stride, const int64_t* dst_off,
                      void* stream);

/* ----------------------------------------------------------------- a12 a13
 * quant (dct.cpp:664-686): per job coef[num] * quantCoeff[num] -> qCoef,
 * deltaU; num_sig[i] = the uint32 return value.  nquant (dct.cpp:688-713)
 * when delta_u == NULL (stores |level|, as the reference).  All buffers of a
 * job are `num` contiguous elements at base + off[i]. */
int x265amd_quant(int n, int num,
                  const int16_t* coef, const int64_t* coef_off,
                  const int32_t* qtab, const int64_t* qtab_off,
                  int32_t* delta_u, const int64_t* delta_off,
                  int16_t* qcoef, const int64_t* qcoef_off,
                  const int32_t* qbits, const int32_t* add,
                  uint32_t* num_sig, void* stream);
/* dequant_normal (dct.cpp:612-634): scale[i], shift[i] per job. */
int x265amd_dequant_normal(int n, int num,
                           const int16_t* q, const int64_t* q_off,
                           int16_t* coef, const int64_t* coef_off,
                           const int32_t* scale, const int32_t* shift, void* stream);
/* dequant_scaling (dct.cpp:636-662): deQuantCoef table per job, per[i], shift[i]. */
int x265amd_dequant_scaling(int n, int num,
                            const int16_t* q, const int64_t* q_off,
                            const int32_t* dq, const int64_t* dq_off,
                            int16_t* coef, const int64_t* coef_off,
                            const int32_t* per, const int32_t* shift, void* stream);

/* --------------------------------------------------------------------- a14
 * Intra prediction (intrapred.cpp).  Neighbour buffers follow the reference
 * layout: [0] top-left, [1..2N] above, [2N+1..4N] left (4N+1 pixels).
 *   intra_filter  cu[].intra_filter        intrapred.cpp:31-51
 *   intra_pred    cu[].intra_pred[mode]    planar (0), DC (1), angular 2..34;
 *                 mode[i], bfilter[i] per job (intrapred.cpp:69-204)
 *   intra_allangs cu[].intra_pred_allangs  intrapred.cpp:206-234: 33 NxN blocks
 *                 of modes 2..34, each written row-major at dst + (mode-2)*N*N */
int x265amd_intra_filter(int depth, int size, int n,
                         const void* src, const int64_t* src_off,
                         void* dst, const int64_t* dst_off, void* stream);
int x265amd_intra_pred(int depth, int size, int n,
                       void* dst, intptr_t dst_stride, const int64_t* dst_off,
                       const void* nb, const int64_t* nb_off,
                       const uint8_t* mode, const uint8_t* bfilter, void* stream);
int x265amd_intra_allangs(int depth, int size, int n,
                          void* dst, const int64_t* dst_off,
                          const void* ref, const int64_t* ref_off,
                          const void* filt, const int64_t* filt_off,
                          const uint8_t* bluma, void* stream);

/* --------------------------------------------------------------------- a15
 * Companion block ops (pixel.cpp:338-436, 490-502, 705-808; dct.cpp:714-742).
 *   op                 reference entry          dst     a       b       param
 *   X265AMD_SUB_PS     cu[].sub_ps              int16   pixel   pixel   -
 *   X265AMD_ADD_PS     cu[].add_ps              pixel   pixel   int16   -
 *   X265AMD_ADDAVG     pu[].addAvg              pixel   int16   int16   -
 *   X265AMD_PIXELAVG   pu[].pixelavg_pp         pixel   pixel   pixel   -
 *   X265AMD_COPY_PP    pu[].copy_pp             pixel   pixel   -       -
 *   X265AMD_COPY_SP    cu[].copy_sp             pixel   int16   -       -
 *   X265AMD_COPY_PS    cu[].copy_ps             int16   pixel   -       -
 *   X265AMD_COPY_SS    cu[].copy_ss             int16   int16   -       -
 *   X265AMD_BLOCKFILL  cu[].blockfill_s         int16   -       -       value
 *   X265AMD_CPY2D1D_SHL/SHR cu[].cpy2Dto1D_*    int16   int16   -       shift
 *   X265AMD_CPY1D2D_SHL/SHR cu[].cpy1Dto2D_*    int16   int16   -       shift
 *   X265AMD_TRANSPOSE  cu[].transpose           pixel   pixel   -       -
 * For the 2D<->1D copies the 1-D side uses stride = w (pass it).
 * calcresidual is SUB_PS with all three strides equal. */
enum
{
    X265AMD_SUB_PS = 0,
    X265AMD_ADD_PS,
    X265AMD_ADDAVG,
    X265AMD_PIXELAVG,
    X265AMD_COPY_PP,
    X265AMD_COPY_SP,
    X265AMD_COPY_PS,
    X265AMD_COPY_SS,
    X265AMD_BLOCKFILL,
    X265AMD_CPY2D1D_SHL,
    X265AMD_CPY2D1D_SHR,
    X265AMD_CPY1D2D_SHL,
    X265AMD_CPY1D2D_SHR,
    X265AMD_TRANSPOSE
};
int x265amd_blockop(int op, int depth, int w, int h, int n,
                    void* dst, intptr_t dst_stride, const int64_t* dst_off,
                    const void* a, intptr_t a_stride, const int64_t* a_off,
                    const void* b, intptr_t b_stride, const int64_t* b_off,
                    int param, void* stream);
/* Grouped form: `count` batches of one op, any mix of block shapes, packed
 * into as few launches as possible (same semantics as one x265amd_blockop
 * call per batch, in order; rejected whole if any batch is invalid). */
typedef struct x265amd_block_batch
{
    int w, h, n, param;
    void* dst;
    intptr_t dst_stride;
    const int64_t* dst_off;
    const void* a;
    intptr_t a_stride;
    const int64_t* a_off;
    const void* b;
    intptr_t b_stride;
    const int64_t* b_off;
} x265amd_block_batch;
int x265amd_blockop_grouped(int op, int depth, int count, const x265amd_block_batch* batches, void* stream);

/* count_nonzero (dct.cpp:714-726, num = N*N contiguous int16) and copy_cnt
 * (dct.cpp:728-742: coeff[N*N] <- residual with res_stride, counting nonzero).
 * copy_cnt when `res` != NULL, else count_nonzero on `coeff`. */
/* denoiseDct (dct.cpp:744-755): each job's num coefficients (contiguous at
 * coef + coef_off[i]) are shrunk in place by offset[num]; |coef| of every job
 * is added into res_sum[num], which the whole batch shares like the
 * reference's per-transform-size accumulator (uint32, wraps like it; the sum
 * is order-independent).  num = N*N for N = 4..32. */
int x265amd_denoise_dct(int n, int num, int16_t* coef, const int64_t* coef_off, uint32_t* res_sum,
                        const uint16_t* offset, void* stream);

int x265amd_count_nonzero(int size, int n,
                          int16_t* coeff, const int64_t* coeff_off,
                          const int16_t* res, intptr_t res_stride, const int64_t* res_off,
                          uint32_t* count, void* stream);

/* ------------------------------------------------------------------- f3
 * Fused TU pipeline.  Job i runs, for one N x N TU, the
 * chain Search::residualTransformQuantIntra performs for a residual-coded TU
 * (search.cpp:689-706) at --preset medium:
 *   resi   = fenc - pred                                   cu[].calcresidual
 *   coeff  = Quant::transformNxN(resi)                     quant.cpp:397-491
 *            (dst4x4 for luma intra 4x4, else cu[].dct; quant with the flat
 *             scaling list of qp; signBitHidingHDQ when sign_hide and
 *             numSig >= 2); num_sig[i] = its return value
 *   numSig ? resi = Quant::invtransformNxN(coeff)          quant.cpp:493-546
 *                   (dequant_normal; DC-only shortcut; idst4x4 / cu[].idct)
 *            recon = cu[].add_ps(pred, resi)
 *          : recon = cu[].copy_pp(pred)                    (resi keeps fenc - pred)
 * Not covered (the encoder's defaults at medium): RDOQ, transform skip,
 * lossless bypass, scaling lists, noise reduction.
 * qp[i] is the QP the Quant object was set to for this TU's component
 * (QpParam::setQpParam argument = qp + QP_BD_OFFSET, quant.h:49-55):
 * per = qp / 6, rem = qp % 6.  scan[i] is the scan type
 * getTUEntropyCodingParameters derives (cudata.cpp:2038-2046: 0 diagonal,
 * 1 horizontal, 2 vertical; only diagonal for 16x16 / 32x32 and inter);
 * scan == NULL means diagonal for every job.  coeff is N*N contiguous per job
 * at coeff + coeff_off[i]; resi may be NULL (not written).  One batch holds
 * one TU size and one (component, intra/inter, slice type) class. */
typedef struct
{
    int log2_size;          /* 2..5: TU 4x4 .. 32x32 */
    int n;                  /* jobs */
    int is_luma;            /* TEXT_LUMA (else a chroma component) */
    int is_intra;           /* cu.isIntra(absPartIdx) */
    int i_slice;            /* slice type I: quant rounding 171, else 85 (quant.cpp:480) */
    int sign_hide;          /* pps.bSignHideEnabled (quant.cpp:485) */
    const void* fenc;
    intptr_t fenc_stride;
    const int64_t* fenc_off;
    const void* pred;
    intptr_t pred_stride;
    const int64_t* pred_off;
    int16_t* resi;
    intptr_t resi_stride;
    const int64_t* resi_off;
    int16_t* coeff;
    const int64_t* coeff_off;
    void* recon;
    intptr_t recon_stride;
    const int64_t* recon_off;
    uint32_t* num_sig;
    const uint8_t* qp;
    const uint8_t* scan;
} x265amd_tu_batch;
int x265amd_tu_pipeline(int depth, int count, const x265amd_tu_batch* batches, void* stream);

/* ------------------------------------------------------------------- f1
 * Lookahead lowres pipeline: the parts that depend only on
 * the source pictures, batched over n frames.
 *
 * x265amd_lowres_init — Lowres::init's plane generation (lowres.cpp:151-162):
 * frameInitLowres (frame_init_lowres_core, pixel.cpp:549-573) writes the four
 * half-pel lowres planes, then extendPicBorder (pixel.cpp:908-922) pads each by
 * margin_x / margin_y (left/right margins replicate the edge pixel, margin rows
 * copy the extended first/last row over the whole stride).  width / lines are
 * the lowres size rounded up to the 8x8 CU grid as Lowres::create rounds it
 * (lowres.cpp:34-45); src_off[i] is frame i's full-resolution luma origin
 * (PicYuv::m_picOrg[0]), plane_off[4 i + k] the origin of its lowresPlane[k]. */
typedef struct
{
    int n;
    int width, lines;
    int margin_x, margin_y;
    const void* src;
    intptr_t src_stride;
    const int64_t* src_off;
    void* planes;
    intptr_t lowres_stride;
    const int64_t* plane_off;
} x265amd_lowres_batch;
int x265amd_lowres_init(int depth, const x265amd_lowres_batch* batch, void* stream);

/* x265amd_lowres_intra — LookaheadTLD::lowresIntraEstimate (slicetype.cpp:230-330)
 * for every 8x8 CU of n frames: intra_cost / intra_mode / lowres_cost
 * (Lowres::intraCost, intraMode, lowresCosts[0][0]) per CU, row_satd
 * (rowSatds[0][0]) per CU row, cost_est[2 i] / [2 i + 1] = costEst[0][0] /
 * costEstAq[0][0] of frame i.  plane_off[i] = origin of frame i's border-extended
 * lowresPlane[0]; inv_qscale = per-CU invQscaleFactor (AQ) or NULL.  Arrays are
 * n * width_cu * height_cu (per CU, frame-major) / n * height_cu / 2 n; row_satd
 * and cost_est are overwritten. */
typedef struct
{
    int n;
    int width_cu, height_cu;
    const void* planes;
    intptr_t lowres_stride;
    const int64_t* plane_off;
    const int32_t* inv_qscale;
    int32_t* intra_cost;
    uint8_t* intra_mode;
    uint16_t* lowres_cost;
    int32_t* row_satd;
    int64_t* cost_est;
} x265amd_lowres_intra_batch;
int x265amd_lowres_intra(int depth, const x265amd_lowres_intra_batch* batch, void* stream);

/* x265amd_lowres_pcost — CostEstimateGroup::estimateFrameCost for n P estimates
 * (b == p1, list 0: slicetype.cpp:1977-2066) = estimateCUCost (slicetype.cpp:2068-2225)
 * for every 8x8 CU: MVP from the right / below neighbours by SATD, the lowres HEX motion
 * search with sub-pel refine of MotionEstimate::motionEstimate at subme 1 (motion.cpp:
 * 571-1172) and the inter / intra choice.  CUs are visited in the reference's order
 * inside each coop slice (rows_per_slice / num_slices as Lookahead::create sets them,
 * slicetype.cpp:546-557; num_slices <= 1: the whole frame as one slice), so results are
 * identical to the serial reference for that slicing.
 * Per estimate i: fenc_off[i] = lowresPlane[0] of frame b; ref_off[4 i + k] =
 * lowresPlane[k] of p0 (or its weighted planes); intra_cost / inv_qscale = frame b's
 * Lowres::intraCost / invQscaleFactor (n * ncu, inv_qscale may be NULL).  mvcost points at
 * the centre (difference 0) of the BitCost table for X265_LOOKAHEAD_QP (uint16 per qpel
 * MV component difference, bitcost.cpp) and must cover every difference the search
 * forms.  Outputs: mvs (2 int16 per CU: lowresMvs, qpel), mv_costs (lowresMvCosts),
 * lowres_costs (lowresCosts[b-p0][p1-b]), row_satd (rowSatds), cost_est[2 i .. 2 i + 1]
 * (costEst / costEstAq), intra_mbs[i] (intraMbs[b - p0]).  Slices of at most 512 rows. */
typedef struct
{
    int n;
    int width_cu, height_cu;
    int rows_per_slice, num_slices;
    const void* planes;
    intptr_t lowres_stride;
    const int64_t* fenc_off;
    const int64_t* ref_off;
    const int32_t* intra_cost;
    const int32_t* inv_qscale;
    const uint16_t* mvcost;
    int16_t* mvs;
    int32_t* mv_costs;
    uint16_t* lowres_costs;
    int32_t* row_satd;
    int64_t* cost_est;
    int32_t* intra_mbs;
} x265amd_lowres_pcost_batch;
int x265amd_lowres_pcost(int depth, const x265amd_lowres_pcost_batch* batch, void* stream);

/* f1 B estimates: CostEstimateGroup::estimateFrameCost for p0 < b < p1 (estimateCUCost with
 * bBidir, slicetype.cpp:2068-2225): per list the search when do_search[2 i + l] (bDoSearch[l]) —
 * MVP choice incl. the zero-MVP skip cost, lowres HEX search from p0 (list 0) / p1 (list 1) —
 * else the stored lowresMvCosts / lowresMvs are reused; then the bidir and co-located averages.
 * Same slice geometry, MV-cost table and sums as x265amd_lowres_pcost (no intra, no intraMbs).
 * mvs0 / mv_costs0 = lowresMvs[0][b-p0-1] / lowresMvCosts[0][b-p0-1] of b (ncu per estimate; read when
 * not searched, written when searched), mvs1 / mv_costs1 = lowresMvs[1][p1-b-1] / ...;
 * lowres_costs = lowresCosts[b-p0][p1-b]; row_satd = rowSatds[b-p0][p1-b]; cost_est = costEst /
 * costEstAq[b-p0][p1-b].  Weighted prediction of p0 (wfref0) is not applied. */
typedef struct
{
    int n, width_cu, height_cu, rows_per_slice, num_slices;
    const void* planes;
    intptr_t lowres_stride;
    const int64_t* fenc_off;      /* per estimate: lowresPlane[0] of b */
    const int64_t* ref0_off;      /* 4 per estimate: lowresPlane[0..3] of p0 */
    const int64_t* ref1_off;      /* 4 per estimate: lowresPlane[0..3] of p1 */
    const uint8_t* do_search;     /* 2 per estimate */
    const int32_t* inv_qscale;    /* per estimate: frame b's invQscaleFactor (ncu), or NULL */
    const uint16_t* mvcost;       /* BitCost table of X265_LOOKAHEAD_QP at difference 0 */
    int16_t* mvs0;
    int32_t* mv_costs0;
    int16_t* mvs1;
    int32_t* mv_costs1;
    uint16_t* lowres_costs;
    int32_t* row_satd;
    int64_t* cost_est;
} x265amd_lowres_bcost_batch;
int x265amd_lowres_bcost(int depth, const x265amd_lowres_bcost_batch* batch, void* stream);

/* f1 encoder session: the lookahead cost estimates of a RUNNING x265 encoder on the device
 * (the reference-side hook is integration/gpu_lookahead.cpp).  Unlike the
 * entries above, these take HOST pointers and are synchronous: they sit under
 *   LookaheadTLD::lowresIntraEstimate(Lowres&)                      slicetype.cpp:230-336
 *   CostEstimateGroup::estimateFrameCost(tld, p0, p1, b, penalty)   slicetype.cpp:1977-2066
 * whose results the encoder reads right after the call.  A session owns device slots for the
 * pictures' lowres planes: x265amd_la_load uploads a Lowres buffer (lowres.cpp:30-163 layout:
 * 4 planes of `planesize` pixels, lowresPlane[k] = buffer + k * planesize + padoffset) once, keyed
 * by any unique host address (the Lowres*), and every later estimate that reads the picture uses
 * the device copy; the intra estimate keeps the picture's intraCost on the device for its P
 * estimates.  Thread-safe: x265 calls them from its pre-lookahead and batch workers at once; each
 * host thread gets its own stream, scratch and weighted-plane slot.  Errors are returned and
 * recorded in the backend's sticky status (x265amd_provider_status). */
typedef struct x265amd_la x265amd_la;
typedef struct
{
    int depth;
    int width_cu, height_cu;       /* Lowres::maxBlocksInRow / maxBlocksInCol */
    intptr_t lowres_stride;        /* Lowres::lumaStride */
    int64_t planesize, padoffset;  /* elements */
    int max_frames;                /* device picture slots (distinct keys) */
    int max_threads;               /* distinct host threads calling the session */
    const uint16_t* mvcost;        /* HOST BitCost table of X265_LOOKAHEAD_QP at difference 0 */
    int mvcost_range;              /* entries [-range, range] are copied */
} x265amd_la_config;
int  x265amd_la_create(const x265amd_la_config* cfg, x265amd_la** out);
void x265amd_la_destroy(x265amd_la* la);
/* (re)load picture `key` (generation gen = Lowres::frameNum): its 4 planes and, with AQ, its
 * invQscaleFactor (ncu int32; NULL without AQ).  The session page-locks `buffer` (hipHostRegister)
 * until the key is reloaded from another buffer or the session is destroyed: the buffer must stay
 * allocated until then (x265's Lowres buffers live as long as the encoder).  Memory freed while it is
 * registered can be unmapped under the GPU's userptr mapping. */
int x265amd_la_load(x265amd_la* la, const void* key, int gen, const void* buffer, const int32_t* inv_qscale);
/* lowresIntraEstimate of a loaded picture: intraCost, intraMode, lowresCosts[0][0], rowSatds[0][0],
 * cost_est[0..1] = costEst[0][0] / costEstAq[0][0] */
int x265amd_la_intra(x265amd_la* la, const void* key, int32_t* intra_cost, uint8_t* intra_mode,
                     uint16_t* lowres_cost, int32_t* row_satd, int64_t* cost_est);
/* P estimate (b == p1) of picture fenc from ref (list-0 search always on): weighted_buffer = the
 * 4-plane weighted reference of weightsAnalyse (LookaheadTLD::wbuffer[0]) or NULL; coop-slice
 * geometry as estimateFrameCost chooses it (num_slices <= 1: the whole frame).  Outputs as
 * x265amd_lowres_pcost: lowresMvs[0][b-p0-1], lowresMvCosts[0][b-p0-1], lowresCosts[b-p0][0],
 * rowSatds[b-p0][0], the raw sums costEst / costEstAq, and the count of intra CUs. */
int x265amd_la_pcost(x265amd_la* la, const void* fenc, const void* ref, const void* weighted_buffer,
                     int rows_per_slice, int num_slices, int16_t* mvs, int32_t* mv_costs, uint16_t* lowres_costs,
                     int32_t* row_satd, int64_t* cost_est, int32_t* intra_mbs);
/* B estimate (p0 < b < p1): a list is searched when do_search<l>, else its mvs / mv_costs are
 * read; outputs as x265amd_lowres_bcost (searched lists' mvs / mv_costs written back). */
int x265amd_la_bcost(x265amd_la* la, const void* fenc, const void* ref0, const void* ref1, int do_search0,
                     int do_search1, int rows_per_slice, int num_slices, int16_t* mvs0, int32_t* mv_costs0,
                     int16_t* mvs1, int32_t* mv_costs1, uint16_t* lowres_costs, int32_t* row_satd,
                     int64_t* cost_est);

/* Several estimates in ONE device launch (CostEstimateGroup::finishBatch's batch: estimates of
 * one batch are independent, slicetype.cpp:1231-1298).  Per job the same inputs / outputs as the
 * single-estimate entries; cost_est / intra_mbs are returned in the job.  weighted_buffer must be
 * NULL when n > 1 (one weighted slot per thread). */
typedef struct
{
    const void* fenc;
    const void* ref;
    const void* weighted_buffer;
    int16_t* mvs;
    int32_t* mv_costs;
    uint16_t* lowres_costs;
    int32_t* row_satd;
    int64_t cost_est[2];
    int32_t intra_mbs;
} x265amd_la_pjob;
typedef struct
{
    const void* fenc;
    const void* ref0;
    const void* ref1;
    int do_search0, do_search1;
    int16_t* mvs0;
    int32_t* mv_costs0;
    int16_t* mvs1;
    int32_t* mv_costs1;
    uint16_t* lowres_costs;
    int32_t* row_satd;
    int64_t cost_est[2];
} x265amd_la_bjob;
int x265amd_la_pcost_n(x265amd_la* la, int n, x265amd_la_pjob* jobs, int rows_per_slice, int num_slices);
int x265amd_la_bcost_n(x265amd_la* la, int n, x265amd_la_bjob* jobs, int rows_per_slice, int num_slices);
/* cuTree's propagation of one (p0, p1, b) (Lookahead::estimateCUPropagate, slicetype.cpp:1741-1842)
 * through x265amd_cutree_propagate, on HOST arrays of the session's CU grid: propagate_in =
 * frames[b]->propagateCost (NULL for a non-referenced b), intra_cost / inv_qscale / lowres_costs =
 * frames[b]->intraCost / invQscaleFactor / lowresCosts[b-p0][p1-b], mvs0 / mvs1 =
 * frames[b]->lowresMvs[0][b-p0-1] / [1][p1-b-1] (mvs1 NULL when b == p1), fps_factor and
 * bipred_weight[2] as the reference computes them; ref_costs0 / ref_costs1 = frames[p0 / p1]->
 * propagateCost, updated in place (ref_costs1 ignored without mvs1).  Synchronous. */
int x265amd_la_propagate(x265amd_la* la, const uint16_t* propagate_in, const int32_t* intra_cost,
                         const uint16_t* lowres_costs, const int32_t* inv_qscale, const int32_t* mvs0,
                         const int32_t* mvs1, double fps_factor, const int* bipred_weight, uint16_t* ref_costs0,
                         uint16_t* ref_costs1);

/* ------------------------------------------------------------------ (e)
 * Frame-parallel schedule, host only: the GOP model of --preset medium
 * (bframes 4, b-pyramid, 3 references, L1 <= 2; param.cpp:145-174, dpb.cpp:149-150,
 * slicetype.cpp:993-1078) over closed segments of segment_frames pictures, frame j (encode order)
 * on rank j mod world (encoder.cpp:649-650), and the earliest step of every CTU-row band: after the
 * frame's previous band and after every reference has published the band holding row
 * r1 - 2 + lag (frameencoder.cpp:516-531; a band is published in the step of the next band's
 * deblocking, the last band in its own).  step[j * nbands + b]; *nsteps = last step + 1. */
enum { X265AMD_FRAME_I = 0, X265AMD_FRAME_P = 1, X265AMD_FRAME_BREF = 2, X265AMD_FRAME_B = 3 };
typedef struct
{
    int frames;            /* pictures in encode order, all segments */
    int segment_frames;    /* pictures per closed segment (each starts with an I picture) */
    int bframes;           /* 4 at --preset medium */
    int b_pyramid;         /* 1 */
    int max_refs;          /* maxNumReferences: 3 */
    int max_refs_l1;       /* 2 with b-pyramid */
    int ctu_rows, band_rows;
    int lag;               /* refLagRows: 2 at --preset medium (frameencoder.cpp:114-119) */
    int world;
} x265amd_sched_config;
typedef struct
{
    int poc;               /* display order over the whole sequence */
    int type;              /* X265AMD_FRAME_* */
    int is_ref;            /* I / P / B-ref */
    int rank;
    int nrefs, nrefs_l0;   /* refs[0 .. nrefs_l0) = L0 (nearest first), then L1 */
    int refs[6];           /* encode indices */
} x265amd_sched_frame;
int x265amd_schedule(const x265amd_sched_config* config, x265amd_sched_frame* frames, int* step, int* nsteps);

/* Reference-row exchange of the frame-parallel shard (csrc/exchange.cpp): what FrameFilter's
 * row publication (m_reconRowCount, framefilter.cpp:520) and the reference-row waits
 * (frameencoder.cpp:516-531) are across GPUs.  One communicator per rank over RCCL (xGMI
 * peer-to-peer), created from a 128-byte id made by rank 0 (x265amd_comm_unique_id) and handed to
 * every rank by the caller; the device is the calling thread's current HIP device.
 * x265amd_exchange enqueues one step's transfers on `stream` as one group (no host wait):
 * xfers[i] sends (send = 1) or receives `bytes` bytes at device address buf to / from rank peer
 * (peer may be the own rank: a loop-back pair).  Every pair of ranks must list the transfers
 * between them in the same order (x265amd_schedule's canonical order does).  X265AMD_ENODEV when
 * librccl is not loadable or a RCCL call fails. */
#define X265AMD_COMM_ID_BYTES 128
typedef struct x265amd_comm x265amd_comm;
typedef struct
{
    void* buf;
    size_t bytes;
    int peer;
    int send;
} x265amd_transfer;
int x265amd_comm_unique_id(uint8_t* id);
/* which RCCL the communicator entries bound (X265AMD_RCCL, the process's already-loaded copy, or
 * ROCm's librccl.so.1 loaded by the library); NULL when no RCCL was found */
const char* x265amd_comm_backend(void);
int x265amd_comm_create(x265amd_comm** comm, const uint8_t* id, int nranks, int rank);
int x265amd_comm_destroy(x265amd_comm* comm);
int x265amd_exchange(x265amd_comm* comm, const x265amd_transfer* xfers, int count, void* stream);

/* f1 cuTree: Lookahead::estimateCUPropagate (slicetype.cpp:1738-1836) with the
 * propagateCost primitive (pixel.cpp:846-872), one call of it per batch, batches in order.
 * For every lowres CU of frame b: the amount
 *   (int)((propagate_in + intra * inv_qscale * fps_factor / 256) * (intra - inter) / intra + 0.5)
 * in IEEE double (no contraction; out-of-range -> INT_MIN as x86-64), and where it is > 0 its
 * share follows the list-0 / list-1 MV (bipred-weighted when both lists are used) onto the
 * (up to) four overlapped CUs of frames p0 / p1, added into ref_costs[l] saturating at 65535.
 *   propagate_in   frames[b]->propagateCost (uint16 per CU), NULL for a non-referenced b (zeros;
 *                  the reference then also zeroes that array's first row — the caller's business)
 *   intra_cost     frames[b]->intraCost;  lowres_costs = frames[b]->lowresCosts[b-p0][p1-b]
 *   inv_qscale     frames[b]->invQscaleFactor
 *   mvs[l]         frames[b]->lowresMvs[l][listDist[l]] (MV: int16 x, y; NULL if list l unused)
 *   fps_factor     CLIP_DURATION(fpsDenom / fpsNum) / CLIP_DURATION(averageDuration)
 *   bipred_weight  bipredWeights[0..1] of estimateCUPropagate
 *   ref_costs[l]   frames[p0 / p1]->propagateCost (in / out)
 *   scratch        2 * width_cu * height_cu int64 of device memory (contents ignored)
 * Exact when every propagated share is >= 0 (amounts below 2^21: the reference's int
 * products do not wrap), which makes the saturating adds order-free. */
typedef struct
{
    int width_cu, height_cu;
    const uint16_t* propagate_in;
    const int32_t* intra_cost;
    const uint16_t* lowres_costs;
    const int32_t* inv_qscale;
    const int32_t* mvs[2];
    double fps_factor;
    int bipred_weight[2];
    uint16_t* ref_costs[2];
    int64_t* scratch;
} x265amd_propagate_batch;
int x265amd_cutree_propagate(int count, const x265amd_propagate_batch* batches, void* stream);

/* f1 weightp: LookaheadTLD::weightsAnalyse (slicetype.cpp:391-495) for one (fenc, ref) lowres
 * pair: the weight_pp primitive (pixel.cpp:463-488) over the padded planes and the
 * weightCostLuma passes (Σ min(satd 8x8, intraCost), slicetype.cpp:338-368) on the device; the
 * reference's float decisions (guess scale, offset, denominator reduction, 0.998 threshold) on
 * the host between them, so the call is synchronous on `stream` (two 4-byte read-backs).
 * Geometry as Lowres::create (lowres.cpp:30-60): width / lines multiples of 8, stride,
 * padded_lines = planesize / stride, pad_offset = lowresPlane - buffer.  fenc_plane =
 * fenc.lowresPlane[0]; ref_buf[4] = ref.buffer[]; wbuf[4] = the weighted planes' buffers (the
 * LookaheadTLD wbuffer: plane 0 is written by the weighted cost pass, all four when a weight is
 * chosen); scratch = one device uint32.  Outputs: weighted (weightedRef.isWeighted), the chosen
 * scale / denom / offset (WeightParam inputWeight / log2WeightDenom / inputOffset) and
 * cost_delta (weightedCostDelta[frame distance], set when weighted). */
typedef struct
{
    int width, lines;
    int64_t stride;
    int padded_lines;
    int64_t pad_offset;
    const void* fenc_plane;
    const void* ref_buf[4];
    const int32_t* intra_cost;
    void* wbuf[4];
    uint32_t* scratch;
    uint64_t fenc_ssd, ref_ssd, fenc_sum, ref_sum;
    int weighted, scale, denom, offset;
    double cost_delta;
} x265amd_weights_batch;
int x265amd_weights_analyse(int depth, x265amd_weights_batch* batch, void* stream);

/* ------------------------------------------------------------------- f2
 * Full-resolution motion search.  Job i is one
 * MotionEstimate::motionEstimate call (motion.cpp:571-1172) on a full-resolution
 * luma reference, as Search::predInterSearch makes it (search.cpp:2024, 2112):
 * the clipped MVP measured at sub-pel (SAD, no MV cost), the num_cand[i] extra
 * candidates (AMVP list), DIA (method 0), HEX (method 1, --preset medium), STAR
 * (method 2, --preset slow), UMH (method 3, --me umh: adaptive range, early
 * termination, hexagon grid) or FULL (method 4, --me full: every MV of mv_range, the
 * first raster-order minimum; out_mv / out_cost double as its scratch) integer search
 * within merange, then the sub-pel refine
 * of workload[subme] for subme 0..7 (motion.cpp:48-58; from subme 3 the 4:2:0
 * chroma SATD is added when the chroma planes are given).  fenc_off[i] / ref_off[i] = the PU origin in the
 * source / reference plane (the reference is border-extended as PicYuv is);
 * mv_range[4 i ..] = mvmin.x, mvmin.y, mvmax.x, mvmax.y (full-pel); mvp[2 i ..]
 * and the candidates mvc[2 (i max_cand + k) ..] are quarter-pel; mvcost +
 * mvcost_off[i] is the centre (difference 0) of the BitCost table of the job's
 * QP (BitCost::setQP; uint16 per MV component difference), which must cover
 * every difference the search forms.  Outputs: out_mv[2 i ..] (outQMv, qpel)
 * and out_cost[i] (the returned cost).  PU sizes: the 25 luma PU shapes. */
typedef struct
{
    int w, h, n;
    int method, subme, merange;
    int max_cand;
    const void* fenc;
    intptr_t fenc_stride;
    const int64_t* fenc_off;
    const void* ref;
    intptr_t ref_stride;
    const int64_t* ref_off;
    const int16_t* mv_range;
    const int16_t* mvp;
    const int16_t* mvc;
    const uint8_t* num_cand;
    const uint16_t* mvcost;
    const int64_t* mvcost_off;
    int16_t* out_mv;
    int32_t* out_cost;
    /* subme >= 3 only: 4:2:0 chroma of source and reference (NULL = luma only); *_coff[i] = the
     * PU's chroma origin.  Chroma SATD is added exactly where bChromaSATD adds it
     * (motion.cpp:183-197, 1205-1266): chroma PU dims multiples of 4. */
    const void* fenc_cb;
    const void* fenc_cr;
    intptr_t fenc_cstride;
    const int64_t* fenc_coff;
    const void* ref_cb;
    const void* ref_cr;
    intptr_t ref_cstride;
    const int64_t* ref_coff;
    /* optional (NULL = not counted): eval_count[2 i] / [2 i + 1] = the full-pel / sub-pel block evaluations
     * job i's search made (one SAD of the PU, resp. one interpolated PU + its SAD / SATD), the unit of the
     * launch's algorithmic bytes */
    uint32_t* eval_count;
} x265amd_me_batch;
int x265amd_motion_search(int depth, int count, const x265amd_me_batch* batches, void* stream);

/* f2 in the running encoder: the searches of Search::predInterSearch (search.cpp:2050-2231)
 * through a session, as the f1 session serves the lookahead.  Like the x265amd_la_* entries these
 * take HOST pointers and are synchronous (the encoder reads each search's result right after the
 * call); thread-safe (x265 searches from every WPP worker and frame encoder at once; each host
 * thread gets its own stream and staging).  A session holds device copies of the reconstructed
 * reference pictures' padded luma planes (PicYuv, picyuv.cpp:51-91: m_picBuf[0] of `plane_elems`
 * elements, m_picOrg[0] at `org_offset`), uploaded CTU row by CTU row as the encoder makes them
 * final (Frame::m_reconRowCount, framefilter.cpp:520), and the BitCost tables of the QPs in use
 * (bitcost.cpp:31-57).  Errors are returned and recorded in the sticky status, except the
 * capacity limits (ENOMEM from x265amd_mes_ref / _table), after which the caller searches that
 * PU on the host. */
typedef struct x265amd_mes x265amd_mes;
typedef struct
{
    int depth;
    intptr_t stride;               /* PicYuv::m_stride */
    int64_t plane_elems;           /* m_stride * (maxHeight + 2 * m_lumaMarginY) */
    int64_t org_offset;            /* m_picOrg[0] - m_picBuf[0] */
    int margin_y;                  /* m_lumaMarginY */
    int ctu_rows, ctu_size;        /* numCuInHeight, g_maxCUSize */
    int max_pictures;              /* distinct reconstructed-picture buffers (keys) */
    int max_threads;               /* distinct host threads calling the session */
    int max_tables;                /* distinct BitCost tables (QPs) */
    int mvcost_range;              /* table entries [-range, range] are copied (2 * BC_MAX_MV) */
    int method, subme, merange;    /* x265_param searchMethod / subpelRefine / searchRange */
    int max_cand;                  /* most MV candidates of one search (mvc[] of predInterSearch: 12) */
    int device;                    /* HIP device of the session (round 5; 0 = the first) */
    /* 4:2:0 chroma planes for the sub-pel chroma SATD of subme > 2 (round 5; chroma = 0: luma only).  With
     * chroma, pictures are made resident with x265amd_mes_ref420 and searches posted with
     * x265amd_mes_post420; a search's chroma block is at the luma origin's half position */
    int chroma;
    intptr_t cstride;              /* PicYuv::m_strideC */
    int64_t cplane_elems;          /* m_strideC * (maxHeight / 2 + 2 * m_chromaMarginY) */
    int64_t corg_offset;           /* m_picOrg[1] - m_picBuf[1] (the same for Cr) */
    int cmargin_y;                 /* m_chromaMarginY */
    int launchers;                 /* launch-service threads (round 5): 0 = every call runs on the calling
                                      thread's own stream (round-4 form); > 0 = calls only queue requests and
                                      this many service threads batch ALL queued requests of all threads into
                                      one upload + launch + download each (x265amd_mes_post / _wait) */
} x265amd_mes_config;
int  x265amd_mes_create(const x265amd_mes_config* cfg, x265amd_mes** out);
void x265amd_mes_destroy(x265amd_mes* mes);
/* make CTU rows [0, rows_final) of reference picture `key` (generation gen, e.g. its POC) resident
 * on the device: uploads the rows not uploaded yet for this generation (the top margin with row 0,
 * the bottom margin with the last row) from plane_buf = m_picBuf[0]; *slot = the picture's slot */
int x265amd_mes_ref(x265amd_mes* mes, const void* key, int64_t gen, const void* plane_buf, int rows_final,
                    int* slot);
/* the device copy of a BitCost table (host pointer at difference 0); *index = its table number */
int x265amd_mes_table(x265amd_mes* mes, const uint16_t* centre, int* index);
/* one MotionEstimate::motionEstimate call (motion.cpp:571-1172) per job, all of one PU (w x h, the
 * source block at `fenc` with stride fenc_stride = FENC_STRIDE), ONE device launch: job inputs as
 * the call's arguments (block_off = the PU origin relative to m_picOrg[0], mv_range = mvmin.x,
 * mvmin.y, mvmax.x, mvmax.y full-pel, mvp / mvc quarter-pel); outputs outQMv and the returned cost */
typedef struct
{
    int slot, table;
    int64_t block_off;
    int16_t mv_range[4];
    int16_t mvp[2];
    int num_cand;
    int16_t mvc[2 * 16];
    int16_t out_mv[2];
    int32_t out_cost;
} x265amd_mes_job;
int x265amd_mes_search(x265amd_mes* mes, int w, int h, const void* fenc, intptr_t fenc_stride, int n,
                       x265amd_mes_job* jobs);
/* the same searches without waiting: _submit enqueues them on the calling thread's stream (its own
 * staging, separate from _search's) and returns; _collect waits for them and writes the outputs into
 * `jobs` (n = the submitted count).  One outstanding submit per thread: the encoder issues a CTU's
 * 64x64 searches when its analysis starts and collects them when Search::predInterSearch needs them,
 * after the CTU's split recursion has run on the host meanwhile. */
int x265amd_mes_submit(x265amd_mes* mes, int w, int h, const void* fenc, intptr_t fenc_stride, int n,
                       const x265amd_mes_job* jobs);
int x265amd_mes_collect(x265amd_mes* mes, int n, x265amd_mes_job* jobs);
/* Launch service (cfg.launchers > 0; round 5).  _post copies one PU's source block and its n <= 64
 * searches into a request slot of the calling thread and returns at once with *ticket (0..7, valid on the
 * calling thread only); the session's service threads batch every queued request of every thread into
 * one launch.  _wait blocks until the ticket's searches are done and writes their outputs into jobs (n =
 * the posted count), freeing the slot; _drop gives a ticket up (its slot is reused once the service has
 * finished with it).  ENOMEM (not recorded in the sticky status) when all 8 slots of the thread are
 * outstanding or n > 64: search on the host.  With launchers, _search is _post + _wait, and _submit /
 * _collect keep their one-outstanding-per-thread contract on top of a ticket. */
int x265amd_mes_post(x265amd_mes* mes, int w, int h, const void* fenc, intptr_t fenc_stride, int n,
                     const x265amd_mes_job* jobs, int* ticket);
int x265amd_mes_wait(x265amd_mes* mes, int ticket, int n, x265amd_mes_job* jobs);
int x265amd_mes_drop(x265amd_mes* mes, int ticket);
/* x265amd_mes_ref for a chroma session: planes = m_picBuf[0..2]; the chroma rows of the same CTU rows go
 * with the luma rows */
int x265amd_mes_ref420(x265amd_mes* mes, const void* key, int64_t gen, const void* const planes[3], int rows_final,
                       int* slot);
/* x265amd_mes_post with the PU's 4:2:0 chroma source blocks (w/2 x h/2 at fenc_cb / fenc_cr, stride
 * fenc_cstride): the searches add the chroma SATD where bChromaSATD adds it (motion.cpp:183-197); NULL
 * chroma = luma only.  Needs a chroma session. */
int x265amd_mes_post420(x265amd_mes* mes, int w, int h, const void* fenc, intptr_t fenc_stride, const void* fenc_cb,
                        const void* fenc_cr, intptr_t fenc_cstride, int n, const x265amd_mes_job* jobs, int* ticket);
/* rows of reference picture `key` (generation gen) resident on the device (0 if unknown) */
int x265amd_mes_rows(x265amd_mes* mes, const void* key, int64_t gen, int* rows_resident);
/* session counters: service batches, the requests / searches they carried, device time of the search
 * launches (HIP events around each launch on its stream), wall time from a batch's start to its outputs on
 * the host, summed queueing delay of the requests (post -> batch start), reference-row uploads, the time
 * callers spent blocked in _wait (and how many of those waits had to sleep), and the launches' block
 * evaluations and algorithmic bytes */
typedef struct
{
    int64_t batches, requests, jobs, max_requests_per_batch;
    double kernel_ms, batch_ms, queue_ms;
    int64_t uploads, upload_bytes;
    double upload_ms;
    int64_t waits, waits_blocked, dropped;
    double wait_ms;
    /* block evaluations of the search launches (full-pel SADs, sub-pel interpolations + compares), their
     * algorithmic bytes, and the longest launch */
    int64_t evals_fpel, evals_subpel;
    double algo_bytes, kernel_ms_max;
    /* (round 5) where the waiting time goes: waits and their summed ms by duration (< 0.05, < 0.2, < 1,
     * < 5, >= 5 ms), and service batches (take -> outputs published) by the same bins */
    int64_t wait_hist[5];
    double wait_hist_ms[5];
    int64_t batch_hist[5];
    double batch_hist_ms[5];
} x265amd_mes_counters;
int x265amd_mes_stats(x265amd_mes* mes, x265amd_mes_counters* out);
/* ------------------------------------------------------------------- f3 in the running encoder
 * Inter residual coding session (round 6; csrc/rdosession.cpp, hook integration/gpu_rdo.cpp): the
 * transform units of an inter CU as Search::encodeResAndCalcRdInterCU -> estimateResidualQT
 * (search.cpp:2562-3140) evaluates them at --preset medium (one RQT level: luma TUs of min(CU, 32), chroma
 * half that, 4:2:0; no RDOQ, transform skip, lossless, scaling lists or noise reduction).  A worker posts a
 * CU (its fenc and pred planes and the Quant object's QPs) and waits; service threads run the posted CUs of
 * all workers in one batch: per TU the fused f3 chain (x265amd_tu_pipeline: Quant::transformNxN ->
 * invtransformNxN -> recon, quant.cpp:397-546), per 8x8 block of each plane psyCost_pp of fenc against pred
 * and against the reconstruction (pixel.cpp:672-703; the reference's psyCost of any block made of 8x8
 * blocks is the sum of these).  Thread-safe; the results of a ticket stay valid until it is released. */
typedef struct x265amd_rdo x265amd_rdo;
typedef struct
{
    int depth;                      /* 8, 10 or 12 */
    int device;
    int launchers;                  /* service threads, 1..8 */
    int max_threads;                /* distinct posting host threads */
    int sign_hide;                  /* pps.bSignHideEnabled */
} x265amd_rdo_config;
typedef struct
{
    int log2_cu;                    /* 4..6: 16x16 .. 64x64 (4:2:0: chroma planes half size) */
    uint8_t qp[3];                  /* Quant::m_qpParam[ttype].qp (qp + QP_BD_OFFSET) of luma, Cb, Cr */
    const void* fenc[3];
    intptr_t fenc_stride[3];        /* elements */
    const void* pred[3];
    intptr_t pred_stride[3];
} x265amd_rdo_cu;
/* plane p (0 luma, 1 Cb, 2 Cr): TUs of tu_log2[p], ntu[p] of them in raster order over the plane;
 * recon / resi planes are packed (stride = plane width) */
typedef struct
{
    int log2_cu;
    int tu_log2[3], ntu[3];
    const void* recon[3];           /* pred + resi clipped (pred where a TU has no coefficient) */
    const int16_t* resi[3];         /* invtransformNxN of the TU's coefficients (fenc - pred where none) */
    const int16_t* coeff[3];        /* TU t's N x N coefficients at coeff[p] + t * N * N */
    const uint32_t* num_sig[3];     /* transformNxN's return value per TU */
    const int32_t* psy_pred[3];     /* per 8x8 block (raster): psyCost_pp 8x8 (fenc, pred) */
    const int32_t* psy_rec[3];      /* per 8x8 block: psyCost_pp 8x8 (fenc, recon) */
    const int32_t* sse_pred[3];     /* per 8x8 block: sse_pp 8x8 (fenc, pred); NULL unless served by the server */
    const int32_t* sse_rec[3];      /* per 8x8 block: sse_pp 8x8 (fenc, recon); NULL unless served by the server */
} x265amd_rdo_result;
typedef struct
{
    int64_t batches, requests, tus, blocks, max_requests_per_batch;
    double kernel_ms, batch_ms, queue_ms;
    int64_t waits, waits_blocked;
    double wait_ms;
    int64_t sao_ctus;               /* CTUs whose SAO statistics the server computed (x265amd_rdo_sao_stats) */
    double sao_ms;                  /* their post-to-result time */
} x265amd_rdo_counters;
int  x265amd_rdo_create(const x265amd_rdo_config* cfg, x265amd_rdo** out);
void x265amd_rdo_destroy(x265amd_rdo* rdo);
/* ENOMEM: no free request slot (the caller codes the CU on the host) */
int  x265amd_rdo_post(x265amd_rdo* rdo, const x265amd_rdo_cu* cu, int* ticket);
int  x265amd_rdo_wait(x265amd_rdo* rdo, int ticket, const x265amd_rdo_result** out);
int  x265amd_rdo_release(x265amd_rdo* rdo, int ticket);
int  x265amd_rdo_stats(x265amd_rdo* rdo, x265amd_rdo_counters* out);
/* Resident server (X265AMD_RDO_SERVER=1 with launchers == 0: one kernel serves every request; no reference
 * counterpart).  HIP entries that synchronise the whole device (hipHostRegister / hipHostUnregister, hipFree,
 * hipStreamCreate) wait for every running kernel, the server too: a caller brackets such calls with these
 * (nesting allowed), which stop the running servers and hold their relaunch until the last end. */
void x265amd_devsync_begin(void);
void x265amd_devsync_end(void);
/* SAO::calcSaoStatsCu (sao.cpp:772-943) of one CTU, all three planes, by the resident server: replaces the
 * three calls SAO::rdoSaoUnitCu makes for a CTU (sao.cpp:1385-1392).  rec[p] / fenc[p]: plane p's CTU origin
 * in the deblocked reconstruction / the source, with the picture's margins around it (the reconstruction is
 * read from 4 pixels left of the CTU to 16 right and one row above and below).  Outputs m_offsetOrg and
 * m_count of the CTU: stats / count [3 planes][5 types: EO_0..EO_3, BO][33 classes].  Synchronous.
 * ENOMEM: not served (no server, no device-memory slots, not 8-bit 4:2:0 64x64, no free slot, or the server
 * broken): the caller computes the statistics on the host. */
typedef struct
{
    int width, height;              /* picture (luma) */
    int ctu_log2, cx, cy;           /* CTU size, column and row */
    int non_deblocked;              /* --sao-non-deblock */
    int chroma_format;              /* X265_CSP_I420 = 1 only */
    const void* rec[3];
    intptr_t rec_stride[3];         /* elements */
    const void* fenc[3];
    intptr_t fenc_stride[3];
} x265amd_rdo_sao_ctu;
int  x265amd_rdo_sao_stats(x265amd_rdo* rdo, const x265amd_rdo_sao_ctu* ctu, int32_t* stats, int32_t* count);

/* host buffers (Lowres / PicYuv planes page-locked by an f1 or f2 session) that were already freed or
 * unmapped when their session unregistered them, over the process: must stay 0 (a freed registered range
 * leaves the GPU a mapping of pages the process no longer owns).  No reference counterpart. */
long long x265amd_host_unregister_stale(void);

/* ------------------------------------------------------------------- f4
 * In-loop filters and border extension of device-resident 4:2:0 recon frames
 * (SURVEY.md §8(f) f4), frame-parallel: what FrameFilter::processRow does row by
 * row (framefilter.cpp:223-520) as whole-frame passes.  One descriptor = one
 * frame; a call takes `count` frames (any mix of sizes).  Planes are addressed
 * at the picture origin with element strides and must be readable at least 16
 * pixels around the picture (x265's PicYuv margins are 64 + 32 / 64 + 16,
 * picyuv.cpp:62-80).  Widths and heights are multiples of 8 (the minimum CU).
 * ctu_log2 = log2 of the CTU size (g_maxCUSize) 4..6; CTUs in raster order. */

/* SaoCtuParam (common.h:336-355) after merge resolution: type -1 off, 0..3 EO_0..EO_3,
 * 4 BO; band = bandPos; offset[0..3] */
typedef struct
{
    int8_t type;
    uint8_t band;
    int8_t offset[4];
} x265amd_sao_param;

/* SAO::processSaoUnitCuLuma / processSaoUnitCuChroma -> processSaoCu (sao.cpp:278-760) for
 * every CTU of the frame, as FrameFilter drives them after deblocking (framefilter.cpp:
 * 176-210, 300-430).  The reference works in place, keeping deblocked copies of the
 * neighbour lines (m_tmpU / m_tmpL); here src (deblocked) and dst (output) are two
 * buffers (must not overlap) and dst receives every picture pixel.  params[p * nctu + c]
 * for plane p; Cr is processed with Cb's type (sao.cpp:755; HEVC shares it).  luma_on /
 * chroma_on = SAOParam::bSaoFlag[0 / 1]. */
typedef struct
{
    int width, height, ctu_log2;
    int luma_on, chroma_on;
    const void* src[3];
    void* dst[3];
    int64_t stride, cstride;
    const x265amd_sao_param* params;
    int chroma_format;   /* 0 or 1 = 4:2:0, 2 = 4:2:2, 3 = 4:4:4 (chroma CTU (ctu >> hshift) x (ctu >> vshift)),
                            X265AMD_CSP_I400 = luma only (chroma planes unused, may be NULL).  NOT x265's
                            internalCsp: there 0 is X265_CSP_I400, here 0 is 4:2:0 (zero-initialised
                            descriptors) */
} x265amd_sao_frame;
int x265amd_sao_apply(int depth, int count, const x265amd_sao_frame* frames, void* stream);

/* SAO::calcSaoStatsCu (sao.cpp:772-943) for every CTU and plane: per CTU, plane, SAO type
 * (EO_0..EO_3, BO) and class 0..32 the sum of (source - deblocked) and the pixel count
 * (m_offsetOrg / m_count), into stats / count[((ctu * 3 + plane) * 5 + type) * 33 + class]
 * (every entry written).  non_deblocked = --sao-non-deblock (bSaoNonDeblocked). */
typedef struct
{
    int width, height, ctu_log2, non_deblocked;
    const void* fenc[3];
    int64_t fenc_stride, fenc_cstride;
    const void* rec[3];
    int64_t rec_stride, rec_cstride;
    int32_t* stats;
    int32_t* count;
    int chroma_format;   /* as x265amd_sao_frame */
} x265amd_sao_stats_frame;
int x265amd_sao_stats(int depth, int count, const x265amd_sao_stats_frame* frames, void* stream);

/* The CUData fields deblocking reads, per 4x4 luma unit (raster, unit_stride units per
 * row): the device-resident CU description (16 bytes per unit). */
typedef struct
{
    uint8_t cu_log2;     /* m_log2CUSize */
    uint8_t tu_log2;     /* log2 luma TU size = m_log2CUSize - m_tuDepth */
    uint8_t part;        /* m_partSize (PartSize, cudata.h:39-50) */
    uint8_t flags;       /* 1 intra (m_predMode), 2 luma cbf of the unit's TU, 4 m_tqBypass */
    int8_t qp;           /* m_qp */
    int8_t ref_idx[2];   /* m_refIdx[list], -1 = unused */
    uint8_t pad;
    int16_t mv[2][2];    /* m_mv[list] x, y (quarter-pel) */
} x265amd_deblock_unit;

/* Deblock::deblockCTU (deblock.cpp:37-536) for every CTU of the frame, in place: the edge
 * marks of deblockCU (CU / TU edges 2, PU splits 1), getBoundaryStrength, the luma strong /
 * weak filters and the 4:2:0 chroma filter, vertical edges of the frame before horizontal
 * ones (the order FrameFilter's per-CTU interleave is equivalent to).  ref_poc[list][i] =
 * identity of the slice's m_refFrameList[list][i] (equal POC = same picture); is_p = P
 * slice; pps fields deblockingFilter{Beta,Tc}OffsetDiv2, chromaQpOffset[0..1],
 * bTransquantBypassEnabled. */
typedef struct
{
    int width, height;
    void* plane[3];
    int64_t stride, cstride;
    const x265amd_deblock_unit* units;
    int64_t unit_stride;
    int is_p;
    int beta_offset_div2, tc_offset_div2, cb_qp_offset, cr_qp_offset, tq_bypass_enabled;
    int32_t ref_poc[2][16];
    int chroma_format;   /* 0 or 1 = 4:2:0, 2 = 4:2:2, 3 = 4:4:4: chroma edges on the chroma plane's 8x8
                            grid (deblock.cpp:104-113); non-4:2:0 chroma QP min(qp, 51) (:505-506);
                            X265AMD_CSP_I400: luma only (deblock.cpp:443 skips chroma), chroma planes may be
                            NULL.  NOT x265's internalCsp (there 0 is 4:0:0) */
} x265amd_deblock_frame;
int x265amd_deblock(int depth, int count, const x265amd_deblock_frame* frames, void* stream);

/* extendPicBorder (pixel.cpp:908-922): fill margin_x columns left / right of every row with
 * the edge pixel, then margin_y full-stride rows above / below with the extended first /
 * last row — the finished-frame result of FrameFilter::processPostCu's row-wise extension
 * (framefilter.cpp:223-297). */
typedef struct
{
    void* plane;
    int64_t stride;
    int width, height, margin_x, margin_y;
} x265amd_border_plane;
int x265amd_extend_border(int depth, int count, const x265amd_border_plane* planes, void* stream);

/* Row-band forms of the loop filters — the CTU-row pipeline of FrameFilter
 * (framefilter.cpp:300-430, processRow / processPostRow) that the frame-parallel
 * shard publishes reconstructed rows from.  Per frame / plane a band
 * of rows; running the bands of a frame top to bottom, deblocking band b before the
 * SAO of band b - 1 (whose last rows deblocking band b modifies), gives the whole-frame
 * result bit-exactly.
 *   deblock_rows:       rows[2i], rows[2i+1] = luma pixel rows [y0, y1) of frame i,
 *                       y0 % 16 == 0, (y1 - y0) % 8 == 0, y1 <= height: the vertical edges
 *                       inside the band and the horizontal edges at y0 <= y < y1 (y > 0);
 *   sao_apply_rows:     ctu_rows[2i], ctu_rows[2i+1] = CTU rows [r0, r1) of frame i;
 *   extend_border_rows: rows[4i..4i+3] = y0, y1, top, bottom: the side margins of picture
 *                       rows [y0, y1) and, when set, the margin rows above / below. */
int x265amd_deblock_rows(int depth, int count, const x265amd_deblock_frame* frames, const int32_t* rows,
                         void* stream);
int x265amd_sao_apply_rows(int depth, int count, const x265amd_sao_frame* frames, const int32_t* ctu_rows,
                           void* stream);
int x265amd_extend_border_rows(int depth, int count, const x265amd_border_plane* planes, const int32_t* rows,
                               void* stream);

#ifdef __cplusplus
}
#endif
#endif /* X265_AMD_H */
