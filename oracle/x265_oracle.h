/* x265_oracle.h — flat C API of the CPU oracle for the x265 1.9 primitive table.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load these libraries, and only as the checker / CPU baseline.
 *
 * Two libraries export this exact API, so one set of Python bindings can
 * drive both:
 *   oracle/_build/liboracle{8,10}.so  — from-scratch C restatement (x265_oracle.c)
 *   oracle/_ref/libx265ref{8,10}.so   — the reference's own C primitives compiled
 *                                       from /root/reference (ref_shim.cpp)
 *
 * Every function is one call of one EncoderPrimitives entry
 * (reference: x265_1.9/source/common/primitives.h:203-381).  Pixels are
 * `pixel` of the library's depth (uint8_t at 8-bit, uint16_t at 10-bit) and are
 * passed as void*.  Strides are in elements, as in the reference.
 */
#ifndef X265_ORACLE_H
#define X265_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int      xo_depth(void);

/* pixel.cpp:39-322 — sad / sad_x3 / sad_x4 / satd / sa8d.  sad_x3/x4 read fenc
 * with the fixed FENC_STRIDE = 64 (pixel.cpp:88,112). */
int      xo_sad(int w, int h, const void* a, intptr_t sa, const void* b, intptr_t sb);
void     xo_sad_x3(int w, int h, const void* fenc, const void* r0, const void* r1,
                   const void* r2, intptr_t rs, int32_t* res);
void     xo_sad_x4(int w, int h, const void* fenc, const void* r0, const void* r1,
                   const void* r2, const void* r3, intptr_t rs, int32_t* res);
int      xo_satd(int w, int h, const void* a, intptr_t sa, const void* b, intptr_t sb);
/* sa8d as the table holds it: satd for sizes not a multiple of 8, one rounding
 * per 16x16 when both dims are multiples of 16, else one rounding per 8x8. */
int      xo_sa8d(int w, int h, const void* a, intptr_t sa, const void* b, intptr_t sb);

/* pixel.cpp:120-139, 324-336, 649-703 */
uint64_t xo_sse_pp(int w, int h, const void* a, intptr_t sa, const void* b, intptr_t sb);
uint64_t xo_sse_ss(int w, int h, const int16_t* a, intptr_t sa, const int16_t* b, intptr_t sb);
uint64_t xo_ssd_s(int n, const int16_t* a, intptr_t sa);
int      xo_psy_cost_pp(int n, const void* src, intptr_t ss, const void* rec, intptr_t rs);
uint64_t xo_var(int n, const void* p, intptr_t s);

/* ipfilter.cpp:40-372.  taps = 8 (luma) or 4 (chroma).
 * extra = isRowExt for HPS, idxY for HVPP (luma only), ignored otherwise. */
enum { XO_HPP = 0, XO_HPS, XO_VPP, XO_VPS, XO_VSP, XO_VSS, XO_HVPP, XO_P2S };
void     xo_interp(int op, int taps, int w, int h, const void* src, intptr_t ss,
                   void* dst, intptr_t ds, int coeffIdx, int extra);

/* dct.cpp:442-610.  DCT/DST read src with `stride`, write N*N contiguous;
 * IDCT/IDST read N*N contiguous, write dst with `stride`. */
enum { XO_DCT = 0, XO_IDCT, XO_DST, XO_IDST };
void     xo_dct(int kind, int n, const int16_t* src, int16_t* dst, intptr_t stride);

/* dct.cpp:612-713 */
uint32_t xo_quant(const int16_t* coef, const int32_t* qcoef, int32_t* deltaU, int16_t* qout,
                  int qBits, int add, int numCoeff);
uint32_t xo_nquant(const int16_t* coef, const int32_t* qcoef, int16_t* qout,
                   int qBits, int add, int numCoeff);
void     xo_dequant_normal(const int16_t* q, int16_t* coef, int num, int scale, int shift);
void     xo_dequant_scaling(const int16_t* q, const int32_t* dq, int16_t* coef, int num,
                            int per, int shift);

/* intrapred.cpp:31-234.  n = TU size 4..32. */
void     xo_intra_filter(int n, const void* ref, void* filt);
void     xo_intra_pred(int n, int mode, void* dst, intptr_t ds, const void* src, int bFilter);
void     xo_intra_allangs(int n, void* dst, void* ref, void* filt, int bLuma);

/* companions (pixel.cpp:338-436, 490-502, 705-808; dct.cpp:714-755) */
void     xo_calcresidual(int n, const void* fenc, const void* pred, int16_t* res, intptr_t stride);
void     xo_sub_ps(int w, int h, int16_t* d, intptr_t ds, const void* a, const void* b,
                   intptr_t sa, intptr_t sb);
void     xo_add_ps(int w, int h, void* d, intptr_t ds, const void* a, const int16_t* b,
                   intptr_t sa, intptr_t sb);
void     xo_addavg(int w, int h, const int16_t* a, const int16_t* b, void* d,
                   intptr_t sa, intptr_t sb, intptr_t ds);
void     xo_pixelavg(int w, int h, void* d, intptr_t ds, const void* a, intptr_t sa,
                     const void* b, intptr_t sb);
void     xo_copy_pp(int w, int h, void* d, intptr_t ds, const void* s, intptr_t ss);
void     xo_copy_sp(int w, int h, void* d, intptr_t ds, const int16_t* s, intptr_t ss);
void     xo_copy_ps(int w, int h, int16_t* d, intptr_t ds, const void* s, intptr_t ss);
void     xo_copy_ss(int w, int h, int16_t* d, intptr_t ds, const int16_t* s, intptr_t ss);
void     xo_blockfill_s(int n, int16_t* d, intptr_t ds, int16_t v);
void     xo_cpy2Dto1D_shl(int n, int16_t* d, const int16_t* s, intptr_t ss, int shift);
void     xo_cpy2Dto1D_shr(int n, int16_t* d, const int16_t* s, intptr_t ss, int shift);
void     xo_cpy1Dto2D_shl(int n, int16_t* d, const int16_t* s, intptr_t ds, int shift);
void     xo_cpy1Dto2D_shr(int n, int16_t* d, const int16_t* s, intptr_t ds, int shift);
int      xo_count_nonzero(int n, const int16_t* q);
uint32_t xo_copy_cnt(int n, int16_t* coeff, const int16_t* res, intptr_t rs);
void     xo_transpose(int n, void* d, const void* s, intptr_t ss);
void     xo_denoise_dct(int16_t* coef, uint32_t* resSum, const uint16_t* offset, int num);

/* f3 fused TU pipeline (quant.cpp:397-546 as driven by search.cpp:689-706):
 *   resi <- fenc - pred; coeff <- quant(dct/dst(resi)) with sign hiding;
 *   numSig ? (resi <- idct/idst(dequant(coeff)) or the DC shortcut; recon <- pred + resi)
 *          : recon <- pred.
 * qp is the scaled QP (qp + QP_BD_OFFSET); scan 0 diag / 1 hor / 2 ver.
 * Returns numSig.  coeff is N*N contiguous. */
uint32_t xo_tu_pipeline(int log2, int is_luma, int is_intra, int i_slice, int sign_hide, int qp, int scan,
                        const void* fenc, intptr_t fs, const void* pred, intptr_t ps,
                        int16_t* resi, intptr_t rs, int16_t* coeff, void* recon, intptr_t rcs);
/* f1 lookahead lowres (lowres.cpp:151-162): frameInitLowres (pixel.cpp:549-573) into the 4
 * half-pel planes p0..p3 (stride ls, lowres width x lines, multiples of 8) then
 * extendPicBorder (pixel.cpp:908-922) of each with margins mx, my. */
void     xo_lowres_init(int width, int lines, const void* src, intptr_t ss, void* p0, void* p1, void* p2, void* p3,
                        intptr_t ls, int mx, int my);
/* LookaheadTLD::lowresIntraEstimate (slicetype.cpp:230-330) over a wcu x hcu grid of 8x8
 * lowres CUs of plane0 (border-extended).  inv_q: per-CU invQscaleFactor or NULL.
 * Writes intra_cost / intra_mode / lowres_cost (lowresCosts[0][0]) per CU, row_satd
 * (rowSatds[0][0]) per CU row and cost_est[0..1] = costEst[0][0], costEstAq[0][0]. */
void     xo_lowres_intra(int wcu, int hcu, const void* plane0, intptr_t ls, const int32_t* inv_q,
                         int32_t* intra_cost, uint8_t* intra_mode, uint16_t* lowres_cost, int32_t* row_satd,
                         int64_t* cost_est);
/* BitCost table for X265_LOOKAHEAD_QP (bitcost.cpp): out[range + d] = cost of an MV
 * component difference d (qpel), |d| <= range */
void     xo_mvcost_table(int range, uint16_t* out);
/* CostEstimateGroup::estimateFrameCost for a P estimate (b == p1, list 0): per 8x8 lowres CU
 * the MVP choice, the lowres HEX motion search with sub-pel refine (MotionEstimate::
 * motionEstimate) and the inter / intra decision of estimateCUCost (slicetype.cpp:2068-2225),
 * in the reference's CU order: coefficient rows bottom-up, right to left, per coop slice
 * (rows_per_slice / num_slices as Lookahead::create sets them; num_slices <= 1 = whole frame).
 * fenc_plane0 = lowresPlane[0] of b; r0..r3 = the (weighted) lowres planes of p0; mvcost_centre
 * = the BitCost table of X265_LOOKAHEAD_QP at difference 0.  Outputs per CU: mvs (qpel x, y:
 * lowresMvs), mv_costs (lowresMvCosts), lowres_costs (lowresCosts[b-p0][p1-b]); per row
 * row_satd; cost_est[0..1] = costEst / costEstAq; intra_mbs = intraMbs[b - p0]. */
void     xo_lowres_pcost(int wcu, int hcu, int rows_per_slice, int num_slices, const void* fenc_plane0,
                         const void* r0, const void* r1, const void* r2, const void* r3, intptr_t ls,
                         const int32_t* intra_cost, const int32_t* inv_q, const uint16_t* mvcost_centre,
                         int16_t* mvs, int32_t* mv_costs, uint16_t* lowres_costs, int32_t* row_satd,
                         int64_t* cost_est, int32_t* intra_mbs);
/* f1: CostEstimateGroup::estimateFrameCost for a B estimate (p0 < b < p1, slicetype.cpp:2068-2225
 * with bBidir): ref0 / ref1 = the four lowres planes of p0 / p1; do_search0 / 1 = bDoSearch[0 / 1]
 * (a list not searched reuses mvs / mv_costs as given); mvs0 / mv_costs0 = lowresMvs[0][b-p0-1] /
 * lowresMvCosts[0][b-p0-1] of b, mvs1 / mv_costs1 = lowresMvs[1][p1-b-1] / ...; outputs
 * lowres_costs (lowresCosts[b-p0][p1-b]), row_satd, cost_est[0..1].  Weighted prediction off. */
void     xo_lowres_bcost(int wcu, int hcu, int rows_per_slice, int num_slices, const void* fenc_plane0,
                         const void* const* ref0, const void* const* ref1, intptr_t ls, const int32_t* inv_q,
                         const uint16_t* mvcost_centre, int do_search0, int do_search1, int16_t* mvs0,
                         int32_t* mv_costs0, int16_t* mvs1, int32_t* mv_costs1, uint16_t* lowres_costs,
                         int32_t* row_satd, int64_t* cost_est);
/* f1 cuTree: Lookahead::estimateCUPropagate (slicetype.cpp:1738-1836) with the propagateCost
 * primitive (pixel.cpp:846-872) for one (p0, b, p1) = (0, b_p0, b_p0 + p1_b): reads frame b's
 * propagate_b (referenced; with referenced = 0 its first row is zeroed and re-read, as the
 * reference does), intra_cost, lowres_costs (= lowresCosts[b - p0][p1 - b]), inv_q, the list-0 /
 * list-1 MVs (lowresMvs[l][listDist[l]], x / y int16 pairs), and adds the propagated amounts into
 * ref0 / ref1 (frames[p0 / p1]->propagateCost, saturating uint16).  fps_num / fps_den and
 * avg_duration as x265_param / cuTree's averageDuration; weighted_bipred = bEnableWeightedBiPred. */
void     xo_cutree_propagate(int wcu, int hcu, int b_p0, int p1_b, int referenced, int weighted_bipred,
                             int fps_num, int fps_den, double avg_duration, uint16_t* propagate_b,
                             const int32_t* intra_cost, const uint16_t* lowres_costs, const int32_t* inv_q,
                             const int32_t* mvs0, const int32_t* mvs1, uint16_t* ref0, uint16_t* ref1);
/* f1 weightp: LookaheadTLD::weightsAnalyse (slicetype.cpp:391-495) with weightCostLuma
 * (:338-368) and the weight_pp primitive (pixel.cpp:463-488).  Lowres geometry as Lowres::create
 * (lowres.cpp:30-60): width / lines (multiples of 8), stride, padded_lines = planesize / stride,
 * pad_offset = lowresPlane - buffer.  fenc_plane = fenc.lowresPlane[0]; ref_buf[4] = ref.buffer[];
 * wbuf[4] = the weighted planes' buffers (written: plane 0 by the cost passes, all four when a
 * weight is chosen); *_ssd / *_sum = Lowres wp_ssd[0] / wp_sum[0].  out[0] = isWeighted,
 * out[1..3] = inputWeight, log2WeightDenom, inputOffset of the chosen weight;
 * *cost_delta = weightedCostDelta (set only when weighted). */
void     xo_weights_analyse(int width, int lines, intptr_t stride, int padded_lines, intptr_t pad_offset,
                            const void* fenc_plane, const void* const* ref_buf, const int32_t* intra_cost,
                            void* const* wbuf, uint64_t fenc_ssd, uint64_t ref_ssd, uint64_t fenc_sum,
                            uint64_t ref_sum, int* out, double* cost_delta);
/* f2: MotionEstimate::motionEstimate (motion.cpp:571-1172) for one w x h PU on a full-resolution
 * reference: method 0 = DIA, 1 = HEX, 2 = STAR, 3 = UMH, 4 = FULL; subme 0..7 (from 3 the 4:2:0 chroma SATD of
 * subpelCompare is added when fcb != NULL and the chroma PU has a satd entry: fcb / fcr, rcb / rcr =
 * source / reference Cb, Cr at the PU's chroma origin); fenc / ref at the PU origin; mvmin /
 * mvmax full-pel; mvp and the numc candidates mvc (x, y pairs) quarter-pel; tab_centre = the
 * BitCost table of the CU's QP at difference 0.  Writes the quarter-pel MV to out[0..1] and
 * returns the cost motionEstimate returns. */
int      xo_motion_search(int w, int h, int method, int subme, int merange, const void* fenc, intptr_t fs,
                          const void* ref, intptr_t rs, int minx, int miny, int maxx, int maxy, int mvpx, int mvpy,
                          int numc, const int16_t* mvc, const uint16_t* tab_centre, int16_t* out,
                          const void* fcb, const void* fcr, intptr_t fcs, const void* rcb, const void* rcr,
                          intptr_t rcs);
/* the reference's BitCost table for any QP (ref_shim only: the restatement takes it as data) */
void     xo_mvcost_table_qp(int qp, int range, uint16_t* out);
/* g_scanOrder[type][log2 - 2] (constants.cpp:445-450): scan position -> raster position */
void     xo_scan_table(int type, int log2, uint16_t* out);

/* ------------------------------------------------------------ f4 loop filters (4:2:0)
 * Planes: y (width x height), cb / cr (width/2 x height/2); every plane readable one pixel
 * outside the picture on each side (the recon PicYuv margins, picyuv.cpp:62-80).
 * ctu_log2 = log2 of the CTU size (g_maxCUSize), 4..6; CTUs in raster order. */
typedef struct
{
    int8_t  type;        /* SaoCtuParam.typeIdx after merge resolution: -1 off, 0..3 EO_0..EO_3, 4 BO */
    uint8_t band;        /* bandPos (BO) */
    int8_t  offset[4];   /* offset[0..3] */
} xo_sao_param;

/* per 4x4 luma unit (raster, unit_stride units per row): the CUData fields deblocking reads */
typedef struct
{
    uint8_t cu_log2;     /* log2 CU size (m_log2CUSize) */
    uint8_t tu_log2;     /* log2 luma TU size (m_log2CUSize - m_tuDepth) */
    uint8_t part;        /* PartSize (cudata.h:39-50) */
    uint8_t flags;       /* 1 intra, 2 luma cbf of the unit's TU, 4 transquant bypass */
    int8_t  qp;          /* m_qp */
    int8_t  ref_idx[2];  /* m_refIdx[list] (-1 = not used) */
    uint8_t pad;
    int16_t mv[2][2];    /* m_mv[list] (x, y), quarter-pel */
} xo_deblock_unit;

typedef struct
{
    int is_p;                   /* P slice: list 0 only (slice.h isInterP); else B */
    int beta_offset_div2, tc_offset_div2, cb_qp_offset, cr_qp_offset, tq_bypass_enabled;
    int32_t ref_poc[2][16];     /* identity of m_refFrameList[list][refIdx] */
} xo_deblock_params;

/* SAO::processSaoUnitCuLuma / processSaoUnitCuChroma -> processSaoCu (sao.cpp:278-760) for every
 * CTU, as FrameFilter drives them on a deblocked frame (framefilter.cpp:176-210, 300-430).  In
 * place.  params[plane * nctu + ctu]; Cr takes Cb's type (processSaoUnitCuChroma, sao.cpp:755). */
/* the same for chroma format csp (1 = 4:2:0, 2 = 4:2:2, 3 = 4:4:4): chroma planes are
 * (width >> hshift) x (height >> vshift), chroma CTUs (ctu >> hshift) x (ctu >> vshift)
 * (sao.cpp:289-298, 786-794; deblock.cpp:104-113, 443-521) */
void     xo_sao_apply_csp(int width, int height, int ctu_log2, void* y, void* cb, void* cr, intptr_t stride,
                          intptr_t cstride, const xo_sao_param* params, int luma_on, int chroma_on, int csp);
void     xo_sao_stats_csp(int width, int height, int ctu_log2, int non_deblocked, const void* fy, const void* fcb,
                          const void* fcr, intptr_t fstride, intptr_t fcstride, const void* ry, const void* rcb,
                          const void* rcr, intptr_t rstride, intptr_t rcstride, int32_t* stats, int32_t* count,
                          int csp);
void     xo_deblock_csp(int width, int height, int ctu_log2, void* y, void* cb, void* cr, intptr_t stride,
                        intptr_t cstride, const xo_deblock_unit* units, intptr_t us, const xo_deblock_params* prm,
                        int csp);
void     xo_sao_apply(int width, int height, int ctu_log2, void* y, void* cb, void* cr, intptr_t stride,
                      intptr_t cstride, const xo_sao_param* params, int luma_on, int chroma_on);
/* SAO::calcSaoStatsCu (sao.cpp:772-943) for every CTU and plane: stats / count
 * [ctu][plane][type 0..4][class 0..32] (m_offsetOrg / m_count of the CTU). */
void     xo_sao_stats(int width, int height, int ctu_log2, int non_deblocked, const void* fy, const void* fcb,
                      const void* fcr, intptr_t fstride, intptr_t fcstride, const void* ry, const void* rcb,
                      const void* rcr, intptr_t rstride, intptr_t rcstride, int32_t* stats, int32_t* count);
/* Deblock::deblockCTU (deblock.cpp:37-536) over the frame, vertical edges of every CTU before
 * the horizontal ones (framefilter.cpp:312-330 order), CU tree given as 4x4 units.  In place. */
void     xo_deblock(int width, int height, int ctu_log2, void* y, void* cb, void* cr, intptr_t stride,
                    intptr_t cstride, const xo_deblock_unit* units, intptr_t unit_stride,
                    const xo_deblock_params* prm);
/* extendPicBorder (pixel.cpp:908-922) of one plane: width x height, margins mx, my */
void     xo_extend_border(void* plane, intptr_t stride, int width, int height, int mx, int my);

#ifdef __cplusplus
}
#endif
#endif
