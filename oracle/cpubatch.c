/* cpubatch.c — runs the GPU C-ABI's batch descriptors (include/x265_amd.h)
 * on the CPU, one per-call oracle function per job.
 *
 * TEST INFRASTRUCTURE ONLY.  Used (a) by tests/ to produce the expected
 * output of every GPU batch from either CPU oracle library and (b) by
 * bench.py's cpu_baseline leg.  The per-job call goes through the flat oracle
 * API (x265_oracle.h) of a library chosen at run time:
 *     oracle/_build/liboracle{8,10}.so   (from-scratch restatement), or
 *     oracle/_ref/libx265ref{8,10}.so    (reference x265 1.9 C primitives).
 * Jobs are split over `nthreads` pthreads (contiguous ranges).
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "x265_oracle.h"

typedef struct
{
    void* dl;
    int depth;
    int (*sad)(int, int, const void*, intptr_t, const void*, intptr_t);
    void (*sad_x3)(int, int, const void*, const void*, const void*, const void*, intptr_t, int32_t*);
    void (*sad_x4)(int, int, const void*, const void*, const void*, const void*, const void*, intptr_t, int32_t*);
    int (*satd)(int, int, const void*, intptr_t, const void*, intptr_t);
    int (*sa8d)(int, int, const void*, intptr_t, const void*, intptr_t);
    uint64_t (*sse_pp)(int, int, const void*, intptr_t, const void*, intptr_t);
    uint64_t (*sse_ss)(int, int, const int16_t*, intptr_t, const int16_t*, intptr_t);
    uint64_t (*ssd_s)(int, const int16_t*, intptr_t);
    int (*psy)(int, const void*, intptr_t, const void*, intptr_t);
    uint64_t (*var)(int, const void*, intptr_t);
    void (*interp)(int, int, int, int, const void*, intptr_t, void*, intptr_t, int, int);
    void (*dct)(int, int, const int16_t*, int16_t*, intptr_t);
    uint32_t (*quant)(const int16_t*, const int32_t*, int32_t*, int16_t*, int, int, int);
    uint32_t (*nquant)(const int16_t*, const int32_t*, int16_t*, int, int, int);
    void (*deq_n)(const int16_t*, int16_t*, int, int, int);
    void (*deq_s)(const int16_t*, const int32_t*, int16_t*, int, int, int);
    void (*ifilt)(int, const void*, void*);
    void (*ipred)(int, int, void*, intptr_t, const void*, int);
    void (*iall)(int, void*, void*, void*, int);
    void (*sub_ps)(int, int, int16_t*, intptr_t, const void*, const void*, intptr_t, intptr_t);
    void (*add_ps)(int, int, void*, intptr_t, const void*, const int16_t*, intptr_t, intptr_t);
    void (*addavg)(int, int, const int16_t*, const int16_t*, void*, intptr_t, intptr_t, intptr_t);
    void (*pavg)(int, int, void*, intptr_t, const void*, intptr_t, const void*, intptr_t);
    void (*copy_pp)(int, int, void*, intptr_t, const void*, intptr_t);
    void (*copy_sp)(int, int, void*, intptr_t, const int16_t*, intptr_t);
    void (*copy_ps)(int, int, int16_t*, intptr_t, const void*, intptr_t);
    void (*copy_ss)(int, int, int16_t*, intptr_t, const int16_t*, intptr_t);
    void (*fill)(int, int16_t*, intptr_t, int16_t);
    void (*c2d1d_shl)(int, int16_t*, const int16_t*, intptr_t, int);
    void (*c2d1d_shr)(int, int16_t*, const int16_t*, intptr_t, int);
    void (*c1d2d_shl)(int, int16_t*, const int16_t*, intptr_t, int);
    void (*c1d2d_shr)(int, int16_t*, const int16_t*, intptr_t, int);
    int (*cnz)(int, const int16_t*);
    uint32_t (*copy_cnt)(int, int16_t*, const int16_t*, intptr_t);
    void (*transpose)(int, void*, const void*, intptr_t);
    void (*denoise)(int16_t*, uint32_t*, const uint16_t*, int);
    uint32_t (*tu)(int, int, int, int, int, int, int, const void*, intptr_t, const void*, intptr_t,
                   int16_t*, intptr_t, int16_t*, void*, intptr_t);
    void (*scan)(int, int, uint16_t*);
    void (*lr_init)(int, int, const void*, intptr_t, void*, void*, void*, void*, intptr_t, int, int);
    void (*lr_intra)(int, int, const void*, intptr_t, const int32_t*, int32_t*, uint8_t*, uint16_t*, int32_t*,
                     int64_t*);
    void (*lr_pcost)(int, int, int, int, const void*, const void*, const void*, const void*, const void*, intptr_t,
                     const int32_t*, const int32_t*, const uint16_t*, int16_t*, int32_t*, uint16_t*, int32_t*, int64_t*,
                     int32_t*);
    void (*mvtab)(int, uint16_t*);
    int (*me)(int, int, int, int, int, const void*, intptr_t, const void*, intptr_t, int, int, int, int, int, int, int,
              const int16_t*, const uint16_t*, int16_t*, const void*, const void*, intptr_t, const void*, const void*,
              intptr_t);
    void (*set_me_qp)(int);   /* reference shim only: its BitCost QP (the restatement reads the table) */
} Lib;

#define SYM(field, name)                                                     \
    do {                                                                     \
        *(void**)&L->field = dlsym(L->dl, name);                             \
        if (!L->field) { fprintf(stderr, "cpubatch: missing %s\n", name); }  \
    } while (0)

void* cb_open(const char* path)
{
    Lib* L = (Lib*)calloc(1, sizeof(Lib));
    L->dl = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!L->dl) { fprintf(stderr, "cpubatch: %s\n", dlerror()); free(L); return NULL; }
    int (*depth)(void) = (int (*)(void))dlsym(L->dl, "xo_depth");
    L->depth = depth ? depth() : 8;
    SYM(sad, "xo_sad"); SYM(sad_x3, "xo_sad_x3"); SYM(sad_x4, "xo_sad_x4"); SYM(satd, "xo_satd");
    SYM(sa8d, "xo_sa8d"); SYM(sse_pp, "xo_sse_pp"); SYM(sse_ss, "xo_sse_ss"); SYM(ssd_s, "xo_ssd_s");
    SYM(psy, "xo_psy_cost_pp"); SYM(var, "xo_var"); SYM(interp, "xo_interp"); SYM(dct, "xo_dct");
    SYM(quant, "xo_quant"); SYM(nquant, "xo_nquant"); SYM(deq_n, "xo_dequant_normal");
    SYM(deq_s, "xo_dequant_scaling"); SYM(ifilt, "xo_intra_filter"); SYM(ipred, "xo_intra_pred");
    SYM(iall, "xo_intra_allangs"); SYM(sub_ps, "xo_sub_ps"); SYM(add_ps, "xo_add_ps");
    SYM(addavg, "xo_addavg"); SYM(pavg, "xo_pixelavg"); SYM(copy_pp, "xo_copy_pp");
    SYM(copy_sp, "xo_copy_sp"); SYM(copy_ps, "xo_copy_ps"); SYM(copy_ss, "xo_copy_ss");
    SYM(fill, "xo_blockfill_s"); SYM(c2d1d_shl, "xo_cpy2Dto1D_shl"); SYM(c2d1d_shr, "xo_cpy2Dto1D_shr");
    SYM(c1d2d_shl, "xo_cpy1Dto2D_shl"); SYM(c1d2d_shr, "xo_cpy1Dto2D_shr"); SYM(cnz, "xo_count_nonzero");
    SYM(copy_cnt, "xo_copy_cnt"); SYM(transpose, "xo_transpose");
    SYM(denoise, "xo_denoise_dct");
    SYM(tu, "xo_tu_pipeline"); SYM(scan, "xo_scan_table");
    SYM(lr_init, "xo_lowres_init"); SYM(lr_intra, "xo_lowres_intra");
    SYM(lr_pcost, "xo_lowres_pcost"); SYM(mvtab, "xo_mvcost_table");
    SYM(me, "xo_motion_search");
    *(void**)&L->set_me_qp = dlsym(L->dl, "xo_set_me_qp");
    return L;
}

int cb_depth(void* h) { return ((Lib*)h)->depth; }

/* ------------------------------------------------------------ threading */
typedef struct
{
    void (*fn)(void* ctx, int64_t lo, int64_t hi);
    void* ctx;
    int64_t lo, hi;
} Range;

static void* range_main(void* p)
{
    Range* r = (Range*)p;
    r->fn(r->ctx, r->lo, r->hi);
    return NULL;
}

static void parallel(int64_t n, int nthreads, void (*fn)(void*, int64_t, int64_t), void* ctx)
{
    if (nthreads <= 1 || n < 2 * nthreads) { fn(ctx, 0, n); return; }
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    Range rg[256];
    for (int t = 0; t < nthreads; t++)
    {
        rg[t].fn = fn; rg[t].ctx = ctx;
        rg[t].lo = n * t / nthreads; rg[t].hi = n * (t + 1) / nthreads;
        pthread_create(&th[t], NULL, range_main, &rg[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

/* element pointer arithmetic: pixels are depth > 8 ? 2 : 1 bytes */
#define PX(base, off) ((const void*)((const uint8_t*)(base) + (off) * psz))
#define PXW(base, off) ((void*)((uint8_t*)(base) + (off) * psz))

/* ------------------------------------------------------------ pixelcmp */
enum { OP_SAD = 0, OP_SATD, OP_SA8D, OP_SSE_PP, OP_SSE_SS, OP_PSY, OP_SSD_S, OP_VAR };

typedef struct
{
    Lib* L; int op, w, h; const void* a; intptr_t sa; const int64_t* ao;
    const void* b; intptr_t sb; const int64_t* bo; void* out;
} CmpCtx;

static void cmp_range(void* p, int64_t lo, int64_t hi)
{
    CmpCtx* c = (CmpCtx*)p;
    Lib* L = c->L;
    const int psz = L->depth > 8 ? 2 : 1;
    for (int64_t i = lo; i < hi; i++)
    {
        const void* a = PX(c->a, c->ao[i]);
        switch (c->op)
        {
        case OP_SAD: ((int32_t*)c->out)[i] = L->sad(c->w, c->h, a, c->sa, PX(c->b, c->bo[i]), c->sb); break;
        case OP_SATD: ((int32_t*)c->out)[i] = L->satd(c->w, c->h, a, c->sa, PX(c->b, c->bo[i]), c->sb); break;
        case OP_SA8D: ((int32_t*)c->out)[i] = L->sa8d(c->w, c->h, a, c->sa, PX(c->b, c->bo[i]), c->sb); break;
        case OP_SSE_PP: ((uint64_t*)c->out)[i] = L->sse_pp(c->w, c->h, a, c->sa, PX(c->b, c->bo[i]), c->sb); break;
        case OP_SSE_SS:
            ((uint64_t*)c->out)[i] = L->sse_ss(c->w, c->h, (const int16_t*)c->a + c->ao[i], c->sa,
                                               (const int16_t*)c->b + c->bo[i], c->sb);
            break;
        case OP_PSY: ((int32_t*)c->out)[i] = L->psy(c->w, a, c->sa, PX(c->b, c->bo[i]), c->sb); break;
        case OP_SSD_S: ((uint64_t*)c->out)[i] = L->ssd_s(c->w, (const int16_t*)c->a + c->ao[i], c->sa); break;
        case OP_VAR: ((uint64_t*)c->out)[i] = L->var(c->w, a, c->sa); break;
        }
    }
}

int cb_pixelcmp(void* h, int op, int w, int hh, int64_t n, const void* a, intptr_t sa, const int64_t* ao,
                const void* b, intptr_t sb, const int64_t* bo, void* out, int nthreads)
{
    CmpCtx c = { (Lib*)h, op, w, hh, a, sa, ao, b, sb, bo, out };
    parallel(n, nthreads, cmp_range, &c);
    return 0;
}

/* ------------------------------------------------------------ sad_x3/x4 */
typedef struct
{
    Lib* L; int nref, w, h; const void* f; intptr_t fs; const int64_t* fo;
    const void* r; intptr_t rs; const int64_t* ro; int32_t* out;
} MultiCtx;

static void multi_range(void* p, int64_t lo, int64_t hi)
{
    MultiCtx* c = (MultiCtx*)p;
    Lib* L = c->L;
    const int psz = L->depth > 8 ? 2 : 1;
    uint16_t stage[64 * 64];
    for (int64_t i = lo; i < hi; i++)
    {
        /* the reference reads fenc with FENC_STRIDE (pixel.cpp:88,112): stage
         * the block into a 64-stride buffer first, as MotionEstimate::setSourcePU
         * does (motion.cpp:184-193) */
        const void* fenc = PX(c->f, c->fo[i]);
        if (c->fs != 64)
        {
            for (int y = 0; y < c->h; y++)
                memcpy((uint8_t*)stage + y * 64 * psz, (const uint8_t*)fenc + y * c->fs * psz, c->w * psz);
            fenc = stage;
        }
        const int64_t* ro = c->ro + i * c->nref;
        if (c->nref == 3)
            L->sad_x3(c->w, c->h, fenc, PX(c->r, ro[0]), PX(c->r, ro[1]), PX(c->r, ro[2]), c->rs, c->out + 3 * i);
        else
            L->sad_x4(c->w, c->h, fenc, PX(c->r, ro[0]), PX(c->r, ro[1]), PX(c->r, ro[2]),
                      PX(c->r, ro[3]), c->rs, c->out + 4 * i);
    }
}

int cb_sad_multi(void* h, int nref, int w, int hh, int64_t n, const void* f, intptr_t fs, const int64_t* fo,
                 const void* r, intptr_t rs, const int64_t* ro, int32_t* out, int nthreads)
{
    if (w > 64 || hh > 64) return -1;
    MultiCtx c = { (Lib*)h, nref, w, hh, f, fs, fo, r, rs, ro, out };
    parallel(n, nthreads, multi_range, &c);
    return 0;
}

/* ------------------------------------------------------------ interp */
typedef struct
{
    Lib* L; int op, taps, w, h; const void* s; intptr_t ss; const int64_t* so;
    void* d; intptr_t ds; const int64_t* dof; const uint8_t* coeff; int rowext;
} InterpCtx;

enum { I_HPP = 0, I_HPS, I_VPP, I_VPS, I_VSP, I_VSS, I_HVPP, I_P2S };

static void interp_range(void* p, int64_t lo, int64_t hi)
{
    InterpCtx* c = (InterpCtx*)p;
    Lib* L = c->L;
    const int psz = L->depth > 8 ? 2 : 1;
    const int ssz = (c->op == I_VSP || c->op == I_VSS) ? 2 : psz;
    const int dsz = (c->op == I_HPS || c->op == I_VPS || c->op == I_VSS || c->op == I_P2S) ? 2 : psz;
    for (int64_t i = lo; i < hi; i++)
    {
        const void* s = (const uint8_t*)c->s + c->so[i] * ssz;
        void* d = (uint8_t*)c->d + c->dof[i] * dsz;
        int ci = c->coeff ? c->coeff[i] : 0;
        int extra = 0;
        if (c->op == I_HVPP) { extra = ci >> 4; ci &= 15; }
        if (c->op == I_HPS) extra = c->rowext;
        L->interp(c->op, c->taps, c->w, c->h, s, c->ss, d, c->ds, ci, extra);
    }
}

int cb_interp(void* h, int op, int taps, int w, int hh, int64_t n, const void* s, intptr_t ss, const int64_t* so,
              void* d, intptr_t ds, const int64_t* dof, const uint8_t* coeff, int rowext, int nthreads)
{
    InterpCtx c = { (Lib*)h, op, taps, w, hh, s, ss, so, d, ds, dof, coeff, rowext };
    parallel(n, nthreads, interp_range, &c);
    return 0;
}

/* ------------------------------------------------------------ transform */
typedef struct
{
    Lib* L; int kind, size; const int16_t* s; intptr_t ss; const int64_t* so;
    int16_t* d; intptr_t ds; const int64_t* dof;
} TrCtx;

static void tr_range(void* p, int64_t lo, int64_t hi)
{
    TrCtx* c = (TrCtx*)p;
    const int fwd = c->kind == 0 || c->kind == 2;
    int16_t tmp[32 * 32];
    for (int64_t i = lo; i < hi; i++)
    {
        const int N = c->size;
        if (fwd)
        {
            /* reference writes the coefficients contiguous; scatter with ds */
            c->L->dct(c->kind, N, c->s + c->so[i], tmp, c->ss);
            for (int y = 0; y < N; y++) memcpy(c->d + c->dof[i] + y * c->ds, tmp + y * N, N * 2);
        }
        else
        {
            for (int y = 0; y < N; y++) memcpy(tmp + y * N, c->s + c->so[i] + y * c->ss, N * 2);
            c->L->dct(c->kind, N, tmp, c->d + c->dof[i], c->ds);
        }
    }
}

int cb_transform(void* h, int kind, int size, int64_t n, const int16_t* s, intptr_t ss, const int64_t* so,
                 int16_t* d, intptr_t ds, const int64_t* dof, int nthreads)
{
    TrCtx c = { (Lib*)h, kind, size, s, ss, so, d, ds, dof };
    parallel(n, nthreads, tr_range, &c);
    return 0;
}

/* ------------------------------------------------------------ quant */
typedef struct
{
    Lib* L; int num; const int16_t* c; const int64_t* co; const int32_t* q; const int64_t* qo;
    int32_t* dl; const int64_t* dlo; int16_t* o; const int64_t* oo; const int32_t* qb; const int32_t* ad;
    uint32_t* sig;
} QCtx;

static void q_range(void* p, int64_t lo, int64_t hi)
{
    QCtx* c = (QCtx*)p;
    for (int64_t i = lo; i < hi; i++)
    {
        if (c->dl)
            c->sig[i] = c->L->quant(c->c + c->co[i], c->q + c->qo[i], c->dl + c->dlo[i], c->o + c->oo[i],
                                    c->qb[i], c->ad[i], c->num);
        else
            c->sig[i] = c->L->nquant(c->c + c->co[i], c->q + c->qo[i], c->o + c->oo[i], c->qb[i], c->ad[i], c->num);
    }
}

int cb_quant(void* h, int64_t n, int num, const int16_t* c, const int64_t* co, const int32_t* q, const int64_t* qo,
             int32_t* dl, const int64_t* dlo, int16_t* o, const int64_t* oo, const int32_t* qb, const int32_t* ad,
             uint32_t* sig, int nthreads)
{
    QCtx x = { (Lib*)h, num, c, co, q, qo, dl, dlo, o, oo, qb, ad, sig };
    parallel(n, nthreads, q_range, &x);
    return 0;
}

typedef struct
{
    Lib* L; int num, scaling; const int16_t* q; const int64_t* qo; const int32_t* dq; const int64_t* dqo;
    int16_t* o; const int64_t* oo; const int32_t* p0; const int32_t* p1;
} DqCtx;

static void dq_range(void* p, int64_t lo, int64_t hi)
{
    DqCtx* c = (DqCtx*)p;
    for (int64_t i = lo; i < hi; i++)
    {
        if (c->scaling)
            c->L->deq_s(c->q + c->qo[i], c->dq + c->dqo[i], c->o + c->oo[i], c->num, c->p0[i], c->p1[i]);
        else
            c->L->deq_n(c->q + c->qo[i], c->o + c->oo[i], c->num, c->p0[i], c->p1[i]);
    }
}

int cb_dequant(void* h, int scaling, int64_t n, int num, const int16_t* q, const int64_t* qo, const int32_t* dq,
               const int64_t* dqo, int16_t* o, const int64_t* oo, const int32_t* p0, const int32_t* p1, int nthreads)
{
    DqCtx x = { (Lib*)h, num, scaling, q, qo, dq, dqo, o, oo, p0, p1 };
    parallel(n, nthreads, dq_range, &x);
    return 0;
}

/* ------------------------------------------------------------ intra */
typedef struct
{
    Lib* L; int kind, size; void* d; intptr_t ds; const int64_t* dof; const void* nb; const int64_t* nbo;
    const void* f; const int64_t* fo; const uint8_t* mode; const uint8_t* bf;
} IntraCtx;

static void intra_range(void* p, int64_t lo, int64_t hi)
{
    IntraCtx* c = (IntraCtx*)p;
    Lib* L = c->L;
    const int psz = L->depth > 8 ? 2 : 1;
    for (int64_t i = lo; i < hi; i++)
    {
        if (c->kind == 0)
            L->ifilt(c->size, PX(c->nb, c->nbo[i]), PXW(c->d, c->dof[i]));
        else if (c->kind == 1)
            L->ipred(c->size, c->mode[i], PXW(c->d, c->dof[i]), c->ds, PX(c->nb, c->nbo[i]), c->bf[i]);
        else
            L->iall(c->size, PXW(c->d, c->dof[i]), (void*)PX(c->nb, c->nbo[i]), (void*)PX(c->f, c->fo[i]), c->bf[i]);
    }
}

int cb_intra(void* h, int kind, int size, int64_t n, void* d, intptr_t ds, const int64_t* dof, const void* nb,
             const int64_t* nbo, const void* f, const int64_t* fo, const uint8_t* mode, const uint8_t* bf, int nthreads)
{
    IntraCtx x = { (Lib*)h, kind, size, d, ds, dof, nb, nbo, f, fo, mode, bf };
    parallel(n, nthreads, intra_range, &x);
    return 0;
}

/* ------------------------------------------------------------ block ops */
enum { B_SUB_PS = 0, B_ADD_PS, B_ADDAVG, B_PIXELAVG, B_COPY_PP, B_COPY_SP, B_COPY_PS, B_COPY_SS, B_FILL,
       B_C2D1D_SHL, B_C2D1D_SHR, B_C1D2D_SHL, B_C1D2D_SHR, B_TRANSPOSE };

typedef struct
{
    Lib* L; int op, w, h; void* d; intptr_t ds; const int64_t* dof; const void* a; intptr_t sa; const int64_t* ao;
    const void* b; intptr_t sb; const int64_t* bo; int param;
} BCtx;

static void b_range(void* p, int64_t lo, int64_t hi)
{
    BCtx* c = (BCtx*)p;
    Lib* L = c->L;
    const int psz = L->depth > 8 ? 2 : 1;
    for (int64_t i = lo; i < hi; i++)
    {
        int16_t* d16 = (int16_t*)c->d + c->dof[i];
        const int16_t* a16 = c->a ? (const int16_t*)c->a + c->ao[i] : NULL;
        switch (c->op)
        {
        case B_SUB_PS: L->sub_ps(c->w, c->h, d16, c->ds, PX(c->a, c->ao[i]), PX(c->b, c->bo[i]), c->sa, c->sb); break;
        case B_ADD_PS: L->add_ps(c->w, c->h, PXW(c->d, c->dof[i]), c->ds, PX(c->a, c->ao[i]), (const int16_t*)c->b + c->bo[i], c->sa, c->sb); break;
        case B_ADDAVG: L->addavg(c->w, c->h, a16, (const int16_t*)c->b + c->bo[i], PXW(c->d, c->dof[i]), c->sa, c->sb, c->ds); break;
        case B_PIXELAVG: L->pavg(c->w, c->h, PXW(c->d, c->dof[i]), c->ds, PX(c->a, c->ao[i]), c->sa, PX(c->b, c->bo[i]), c->sb); break;
        case B_COPY_PP: L->copy_pp(c->w, c->h, PXW(c->d, c->dof[i]), c->ds, PX(c->a, c->ao[i]), c->sa); break;
        case B_COPY_SP: L->copy_sp(c->w, c->h, PXW(c->d, c->dof[i]), c->ds, a16, c->sa); break;
        case B_COPY_PS: L->copy_ps(c->w, c->h, d16, c->ds, PX(c->a, c->ao[i]), c->sa); break;
        case B_COPY_SS: L->copy_ss(c->w, c->h, d16, c->ds, a16, c->sa); break;
        case B_FILL: L->fill(c->w, d16, c->ds, (int16_t)c->param); break;
        case B_C2D1D_SHL: L->c2d1d_shl(c->w, d16, a16, c->sa, c->param); break;
        case B_C2D1D_SHR: L->c2d1d_shr(c->w, d16, a16, c->sa, c->param); break;
        case B_C1D2D_SHL: L->c1d2d_shl(c->w, d16, a16, c->ds, c->param); break;
        case B_C1D2D_SHR: L->c1d2d_shr(c->w, d16, a16, c->ds, c->param); break;
        case B_TRANSPOSE: L->transpose(c->w, PXW(c->d, c->dof[i]), PX(c->a, c->ao[i]), c->sa); break;
        }
    }
}

int cb_blockop(void* h, int op, int w, int hh, int64_t n, void* d, intptr_t ds, const int64_t* dof, const void* a,
               intptr_t sa, const int64_t* ao, const void* b, intptr_t sb, const int64_t* bo, int param, int nthreads)
{
    BCtx x = { (Lib*)h, op, w, hh, d, ds, dof, a, sa, ao, b, sb, bo, param };
    parallel(n, nthreads, b_range, &x);
    return 0;
}

typedef struct
{
    Lib* L; int size; int16_t* c; const int64_t* co; const int16_t* r; intptr_t rs; const int64_t* ro; uint32_t* cnt;
} CntCtx;

static void cnt_range(void* p, int64_t lo, int64_t hi)
{
    CntCtx* c = (CntCtx*)p;
    for (int64_t i = lo; i < hi; i++)
    {
        if (c->r) c->cnt[i] = c->L->copy_cnt(c->size, c->c + c->co[i], c->r + c->ro[i], c->rs);
        else c->cnt[i] = (uint32_t)c->L->cnz(c->size, c->c + c->co[i]);
    }
}

int cb_count_nonzero(void* h, int size, int64_t n, int16_t* c, const int64_t* co, const int16_t* r, intptr_t rs,
                     const int64_t* ro, uint32_t* cnt, int nthreads)
{
    CntCtx x = { (Lib*)h, size, c, co, r, rs, ro, cnt };
    parallel(n, nthreads, cnt_range, &x);
    return 0;
}

/* denoiseDct: serial over the jobs, since every job adds into the one shared res_sum */
int cb_denoise(void* h, int64_t n, int num, int16_t* c, const int64_t* co, uint32_t* res_sum, const uint16_t* offset)
{
    Lib* L = (Lib*)h;
    for (int64_t i = 0; i < n; i++) L->denoise(c + co[i], res_sum, offset, num);
    return 0;
}

/* f3 fused TU pipeline batch (x265amd_tu_batch); pixel offsets in elements of the library's depth */
typedef struct
{
    Lib* L; int log2, luma, intra, islice, sh;
    const char* f; intptr_t fs; const int64_t* fo; const char* p; intptr_t ps; const int64_t* po;
    int16_t* r; intptr_t rs; const int64_t* ro; int16_t* c; const int64_t* co;
    char* rc; intptr_t rcs; const int64_t* rco; uint32_t* sig; const uint8_t* qp; const uint8_t* scan;
} TuCtx;

static void tu_range(void* p, int64_t lo, int64_t hi)
{
    TuCtx* x = (TuCtx*)p;
    const int b = x->L->depth > 8 ? 2 : 1, n = 1 << x->log2;
    int16_t tmp[32 * 32];
    for (int64_t i = lo; i < hi; i++)
    {
        int16_t* r = x->r ? x->r + x->ro[i] : tmp;
        const intptr_t rs = x->r ? x->rs : n;
        x->sig[i] = x->L->tu(x->log2, x->luma, x->intra, x->islice, x->sh, x->qp[i], x->scan ? x->scan[i] : 0,
                             x->f + x->fo[i] * b, x->fs, x->p + x->po[i] * b, x->ps, r, rs, x->c + x->co[i],
                             x->rc + x->rco[i] * b, x->rcs);
    }
}

int cb_tu(void* h, int64_t n, int log2, int luma, int intra, int islice, int sh,
          const void* f, intptr_t fs, const int64_t* fo, const void* p, intptr_t ps, const int64_t* po,
          int16_t* r, intptr_t rs, const int64_t* ro, int16_t* c, const int64_t* co,
          void* rc, intptr_t rcs, const int64_t* rco, uint32_t* sig, const uint8_t* qp, const uint8_t* scan,
          int nthreads)
{
    TuCtx x = { (Lib*)h, log2, luma, intra, islice, sh, (const char*)f, fs, fo, (const char*)p, ps, po, r, rs, ro,
                c, co, (char*)rc, rcs, rco, sig, qp, scan };
    parallel(n, nthreads, tu_range, &x);
    return 0;
}

void cb_scan_table(void* h, int type, int log2, uint16_t* out)
{
    ((Lib*)h)->scan(type, log2, out);
}

/* f1 lookahead lowres: per frame, plane generation then the intra estimate (x265amd_lowres_init +
 * x265amd_lowres_intra); offsets in pixels of the library's depth */
int cb_lowres(void* h, int n, int width, int lines, int mx, int my, const void* src, intptr_t ss, const int64_t* so,
              void* planes, intptr_t ls, const int64_t* po, int wcu, int hcu, const int32_t* inv_q, int32_t* ic,
              uint8_t* im, uint16_t* lc, int32_t* rs, int64_t* ce)
{
    Lib* L = (Lib*)h;
    const int b = L->depth > 8 ? 2 : 1, ncu = wcu * hcu;
    for (int f = 0; f < n; f++)
    {
        char* pl = (char*)planes;
        L->lr_init(width, lines, (const char*)src + so[f] * b, ss, pl + po[4 * f] * b, pl + po[4 * f + 1] * b,
                   pl + po[4 * f + 2] * b, pl + po[4 * f + 3] * b, ls, mx, my);
        L->lr_intra(wcu, hcu, pl + po[4 * f] * b, ls, inv_q ? inv_q + (int64_t)f * ncu : NULL, ic + (int64_t)f * ncu,
                    im + (int64_t)f * ncu, lc + (int64_t)f * ncu, rs + (int64_t)f * hcu, ce + 2 * f);
    }
    return 0;
}

/* f1 P-frame cost estimates (x265amd_lowres_pcost), one estimate after another */
int cb_lowres_pcost(void* h, int n, int wcu, int hcu, int rps, int ns, const void* planes, intptr_t ls,
                    const int64_t* fo, const int64_t* ro, const int32_t* ic, const int32_t* iq, const uint16_t* tab,
                    int16_t* mvs, int32_t* mc, uint16_t* lc, int32_t* rs, int64_t* ce, int32_t* mbs)
{
    Lib* L = (Lib*)h;
    const int b = L->depth > 8 ? 2 : 1, ncu = wcu * hcu;
    const char* pl = (const char*)planes;
    for (int e = 0; e < n; e++)
        L->lr_pcost(wcu, hcu, rps, ns, pl + fo[e] * b, pl + ro[4 * e] * b, pl + ro[4 * e + 1] * b,
                    pl + ro[4 * e + 2] * b, pl + ro[4 * e + 3] * b, ls, ic + (int64_t)e * ncu,
                    iq ? iq + (int64_t)e * ncu : NULL, tab, mvs + 2 * (int64_t)e * ncu, mc + (int64_t)e * ncu,
                    lc + (int64_t)e * ncu, rs + (int64_t)e * hcu, ce + 2 * e, mbs + e);
    return 0;
}

void cb_mvcost_table(void* h, int range, uint16_t* out) { ((Lib*)h)->mvtab(range, out); }

/* f2 full-resolution motion search batch (x265amd_me_batch); qp[i] selects the reference shim's
 * BitCost QP, tab + tab_off[i] is the same table for the restatement */
int cb_motion_search(void* h, int64_t n, int w, int hh, int method, int subme, int merange, int max_cand,
                     const void* fenc, intptr_t fs, const int64_t* fo, const void* ref, intptr_t rs, const int64_t* ro,
                     const int16_t* range, const int16_t* mvp, const int16_t* mvc, const uint8_t* numc,
                     const uint16_t* tab, const int64_t* tab_off, const uint8_t* qp, int16_t* out_mv, int32_t* out_cost,
                     const void* fcb, const void* fcr, intptr_t fcs, const int64_t* fco, const void* rcb, const void* rcr,
                     intptr_t rcs, const int64_t* rco)
{
    Lib* L = (Lib*)h;
    const int b = L->depth > 8 ? 2 : 1;
    for (int64_t i = 0; i < n; i++)
    {
        if (L->set_me_qp) L->set_me_qp(qp[i]);
        const int ch = fcb != NULL;
        out_cost[i] = L->me(w, hh, method, subme, merange, (const char*)fenc + fo[i] * b, fs,
                            (const char*)ref + ro[i] * b, rs, range[4 * i], range[4 * i + 1], range[4 * i + 2],
                            range[4 * i + 3], mvp[2 * i], mvp[2 * i + 1], numc ? numc[i] : 0,
                            mvc + 2 * i * max_cand, tab + tab_off[i], out_mv + 2 * i,
                            ch ? (const char*)fcb + fco[i] * b : NULL, ch ? (const char*)fcr + fco[i] * b : NULL, fcs,
                            ch ? (const char*)rcb + rco[i] * b : NULL, ch ? (const char*)rcr + rco[i] * b : NULL, rcs);
    }
    return 0;
}
