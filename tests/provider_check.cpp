// provider_check.cpp — GPU test of the per-call EncoderPrimitives provider.
//
// Mirrors the reference TestBench flow (test/testbench.cpp:153-217): a table
// is filled by the candidate provider (X265_NS::setupHipPrimitives, on top of
// a table whose slots are all non-NULL placeholders so every entry the
// provider implements gets installed), then every installed entry is called
// THROUGH THE TABLE on random / min / max inputs and compared exactly with
// the CPU oracle's per-call functions (oracle/x265_oracle.h).  Built and run
// by tests/test_provider.py:
//   hipcc -std=c++17 -DX265_DEPTH=8 provider_check.cpp -L... -lx265amd -loracle8
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../include/x265_amd_primitives.h"
#include "../oracle/x265_oracle.h"

using namespace X265_NS;

static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd()
{
    g_rng ^= g_rng >> 12; g_rng ^= g_rng << 25; g_rng ^= g_rng >> 27;
    return (uint32_t)((g_rng * 0x2545F4914F6CDD1Dull) >> 32);
}

static const int kPuW[25] = { 4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 12, 16, 4, 32, 24, 32, 8, 64, 48, 64, 16 };
static const int kPuH[25] = { 4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 12, 16, 4, 16, 24, 32, 8, 32, 48, 64, 16, 64 };
static const int PMAX = (1 << X265_DEPTH) - 1;

static int g_fail = 0, g_checks = 0;
#define EXPECT(cond, ...)                                   \
    do {                                                    \
        g_checks++;                                         \
        if (!(cond)) {                                      \
            if (g_fail < 20) { printf("FAIL: "); printf(__VA_ARGS__); printf("\n"); } \
            g_fail++;                                       \
        }                                                   \
    } while (0)

// buffers with a wide margin so filter windows stay inside them
struct Buf
{
    std::vector<pixel> p;
    std::vector<int16_t> s;
    static const int S = 160, ROWS = 160, M = 16;
    Buf() : p(S * ROWS), s(S * ROWS) {}
    void fill(int cls)
    {
        for (auto& v : p) v = (pixel)(cls == 0 ? rnd() % (PMAX + 1) : cls == 1 ? 0 : PMAX);
        for (auto& v : s) v = (int16_t)(cls == 0 ? (int)(rnd() % 8192) - 4096 : cls == 1 ? -4096 : 4095);
    }
    pixel* pp() { return p.data() + M * S + M; }
    int16_t* sp() { return s.data() + M * S + M; }
};

template <typename T>
static bool same(const T* a, const T* b, size_t n) { return memcmp(a, b, n * sizeof(T)) == 0; }

int main()
{
    setvbuf(stdout, nullptr, _IONBF, 0);   // progress survives a crash
    static EncoderPrimitives tab;
    memset(&tab, 0xAB, sizeof(tab));   // every slot "present" (non-NULL placeholder)
    setupHipPrimitives(tab, 0);
    printf("provider installed\n");
    Buf A, B;
    std::vector<pixel> o1(64 * 80), o2(64 * 80);
    std::vector<int16_t> s1(64 * 80), s2(64 * 80);

    for (int iter = 0; iter < 6; iter++)
    {
        A.fill(iter % 3);
        B.fill((iter / 3) % 3 == 0 ? 0 : (iter % 3 == 1 ? 2 : 1));
        const intptr_t S = Buf::S;
        for (int p = 0; p < 25; p++)
        {
            const int w = kPuW[p], h = kPuH[p];
            if (iter == 0) printf("pu %dx%d\n", w, h);
            EncoderPrimitives::PU& u = tab.pu[p];
            EXPECT(u.sad(A.pp(), S, B.pp() + 1, S) == xo_sad(w, h, A.pp(), S, B.pp() + 1, S), "sad %dx%d", w, h);
            EXPECT(u.satd(A.pp(), S, B.pp() + 3, S) == xo_satd(w, h, A.pp(), S, B.pp() + 3, S), "satd %dx%d", w, h);
            int32_t r1[4], r2[4];
            std::vector<pixel> fenc(64 * 64);
            for (int y = 0; y < h; y++) memcpy(&fenc[y * 64], A.pp() + y * S, w * sizeof(pixel));
            u.sad_x4(fenc.data(), B.pp(), B.pp() + 1, B.pp() + S, B.pp() - 2, S, r1);
            xo_sad_x4(w, h, fenc.data(), B.pp(), B.pp() + 1, B.pp() + S, B.pp() - 2, S, r2);
            EXPECT(!memcmp(r1, r2, 16), "sad_x4 %dx%d", w, h);
            u.sad_x3(fenc.data(), B.pp(), B.pp() + 2, B.pp() + 2 * S, S, r1);
            xo_sad_x3(w, h, fenc.data(), B.pp(), B.pp() + 2, B.pp() + 2 * S, S, r2);
            EXPECT(!memcmp(r1, r2, 12), "sad_x3 %dx%d", w, h);
            const int ci = 1 + iter % 3;
            memset(o1.data(), 0xCD, o1.size() * sizeof(pixel)); memset(o2.data(), 0xCD, o2.size() * sizeof(pixel));
            u.luma_hpp(A.pp(), S, o1.data(), 64, ci); xo_interp(XO_HPP, 8, w, h, A.pp(), S, o2.data(), 64, ci, 0);
            EXPECT(same(o1.data(), o2.data(), o1.size()), "luma_hpp %dx%d", w, h);
            u.luma_vpp(A.pp(), S, o1.data(), 64, ci); xo_interp(XO_VPP, 8, w, h, A.pp(), S, o2.data(), 64, ci, 0);
            EXPECT(same(o1.data(), o2.data(), o1.size()), "luma_vpp %dx%d", w, h);
            u.luma_hvpp(A.pp(), S, o1.data(), 64, ci, 3 - ci % 3); xo_interp(XO_HVPP, 8, w, h, A.pp(), S, o2.data(), 64, ci, 3 - ci % 3);
            EXPECT(same(o1.data(), o2.data(), o1.size()), "luma_hvpp %dx%d", w, h);
            for (int ext = 0; ext < 2; ext++)
            {
                memset(s1.data(), 0xCD, s1.size() * 2); memset(s2.data(), 0xCD, s2.size() * 2);
                u.luma_hps(A.pp(), S, s1.data(), 64, ci, ext); xo_interp(XO_HPS, 8, w, h, A.pp(), S, s2.data(), 64, ci, ext);
                EXPECT(same(s1.data(), s2.data(), s1.size()), "luma_hps %dx%d ext %d", w, h, ext);
            }
            u.luma_vps(A.pp(), S, s1.data(), 64, ci); xo_interp(XO_VPS, 8, w, h, A.pp(), S, s2.data(), 64, ci, 0);
            EXPECT(same(s1.data(), s2.data(), s1.size()), "luma_vps %dx%d", w, h);
            u.luma_vsp(A.sp(), S, o1.data(), 64, ci); xo_interp(XO_VSP, 8, w, h, A.sp(), S, o2.data(), 64, ci, 0);
            EXPECT(same(o1.data(), o2.data(), o1.size()), "luma_vsp %dx%d", w, h);
            u.luma_vss(A.sp(), S, s1.data(), 64, ci); xo_interp(XO_VSS, 8, w, h, A.sp(), S, s2.data(), 64, ci, 0);
            EXPECT(same(s1.data(), s2.data(), s1.size()), "luma_vss %dx%d", w, h);
            u.convert_p2s(A.pp(), S, s1.data(), 64); xo_interp(XO_P2S, 8, w, h, A.pp(), S, s2.data(), 64, 0, 0);
            EXPECT(same(s1.data(), s2.data(), s1.size()), "p2s %dx%d", w, h);
            // companion block ops (a15)
            u.pixelavg_pp(o1.data(), 64, A.pp(), S, B.pp() + 1, S, 32); xo_pixelavg(w, h, o2.data(), 64, A.pp(), S, B.pp() + 1, S);
            EXPECT(same(o1.data(), o2.data(), o1.size()), "pixelavg_pp %dx%d", w, h);
            u.addAvg(A.sp(), B.sp(), o1.data(), S, S, 64); xo_addavg(w, h, A.sp(), B.sp(), o2.data(), S, S, 64);
            EXPECT(same(o1.data(), o2.data(), o1.size()), "addAvg %dx%d", w, h);
            u.copy_pp(o1.data(), 64, A.pp(), S); xo_copy_pp(w, h, o2.data(), 64, A.pp(), S);
            EXPECT(same(o1.data(), o2.data(), o1.size()), "copy_pp %dx%d", w, h);
            // chroma 4:2:0 (w/2 x h/2); the 2x2 entry of the reference table is NULL and is skipped
            const int cw = w / 2, ch = h / 2;
            if (cw >= 2 && ch >= 2 && !(cw == 2 && ch == 2))
            {
                EncoderPrimitives::Chroma::PUChroma& c = tab.chroma[1].pu[p];
                const int cci = 1 + iter % 7;
                c.filter_hpp(A.pp(), S, o1.data(), 64, cci); xo_interp(XO_HPP, 4, cw, ch, A.pp(), S, o2.data(), 64, cci, 0);
                EXPECT(same(o1.data(), o2.data(), o1.size()), "chroma hpp %dx%d", cw, ch);
                c.filter_vpp(A.pp(), S, o1.data(), 64, cci); xo_interp(XO_VPP, 4, cw, ch, A.pp(), S, o2.data(), 64, cci, 0);
                EXPECT(same(o1.data(), o2.data(), o1.size()), "chroma vpp %dx%d", cw, ch);
                c.filter_vss(A.sp(), S, s1.data(), 64, cci); xo_interp(XO_VSS, 4, cw, ch, A.sp(), S, s2.data(), 64, cci, 0);
                EXPECT(same(s1.data(), s2.data(), s1.size()), "chroma vss %dx%d", cw, ch);
            }
        }
        for (int i = 0; i < 5; i++)
        {
            const int n = 4 << i;
            if (iter == 0) printf("cu %d\n", n);
            EncoderPrimitives::CU& c = tab.cu[i];
            EXPECT(c.sa8d(A.pp(), S, B.pp(), S) == xo_sa8d(n, n, A.pp(), S, B.pp(), S), "sa8d %d", n);
            EXPECT((uint64_t)c.sse_pp(A.pp(), S, B.pp(), S) == xo_sse_pp(n, n, A.pp(), S, B.pp(), S), "sse_pp %d", n);
            EXPECT((uint64_t)c.sse_ss(A.sp(), S, B.sp(), S) == xo_sse_ss(n, n, A.sp(), S, B.sp(), S), "sse_ss %d", n);
            EXPECT((uint64_t)c.ssd_s(A.sp(), S) == xo_ssd_s(n, A.sp(), S), "ssd_s %d", n);
            EXPECT(c.psy_cost_pp(A.pp(), S, B.pp(), S) == xo_psy_cost_pp(n, A.pp(), S, B.pp(), S), "psy %d", n);
            EXPECT(c.var(A.pp(), S) == xo_var(n, A.pp(), S), "var %d", n);
            // companion block ops (a15): outputs into 0xCD-filled 64-stride buffers
            memset(s1.data(), 0xCD, s1.size() * 2); memset(s2.data(), 0xCD, s2.size() * 2);
            // calcresidual uses ONE stride for fenc, pred and residual (pixel.cpp:417): 64 keeps the output in s1
            c.calcresidual(A.pp(), B.pp(), s1.data(), 64); xo_calcresidual(n, A.pp(), B.pp(), s2.data(), 64);
            EXPECT(same(s1.data(), s2.data(), s1.size()), "calcresidual %d", n);
            c.sub_ps(s1.data(), 64, A.pp(), B.pp() + 1, S, S); xo_sub_ps(n, n, s2.data(), 64, A.pp(), B.pp() + 1, S, S);
            EXPECT(same(s1.data(), s2.data(), s1.size()), "sub_ps %d", n);
            c.add_ps(o1.data(), 64, A.pp(), B.sp(), S, S); xo_add_ps(n, n, o2.data(), 64, A.pp(), B.sp(), S, S);
            EXPECT(same(o1.data(), o2.data(), o1.size()), "add_ps %d", n);
            c.blockfill_s(s1.data(), 64, (int16_t)(iter * 1000 - 2500)); xo_blockfill_s(n, s2.data(), 64, (int16_t)(iter * 1000 - 2500));
            EXPECT(same(s1.data(), s2.data(), s1.size()), "blockfill_s %d", n);
            const int sh = 1 + iter % 5;
            c.cpy2Dto1D_shl(s1.data(), A.sp(), S, sh); xo_cpy2Dto1D_shl(n, s2.data(), A.sp(), S, sh);
            EXPECT(same(s1.data(), s2.data(), s1.size()), "cpy2Dto1D_shl %d", n);
            c.cpy2Dto1D_shr(s1.data(), A.sp(), S, sh); xo_cpy2Dto1D_shr(n, s2.data(), A.sp(), S, sh);
            EXPECT(same(s1.data(), s2.data(), s1.size()), "cpy2Dto1D_shr %d", n);
            c.cpy1Dto2D_shl(s1.data(), A.sp(), 64, sh); xo_cpy1Dto2D_shl(n, s2.data(), A.sp(), 64, sh);
            EXPECT(same(s1.data(), s2.data(), s1.size()), "cpy1Dto2D_shl %d", n);
            c.cpy1Dto2D_shr(s1.data(), A.sp(), 64, sh); xo_cpy1Dto2D_shr(n, s2.data(), A.sp(), 64, sh);
            EXPECT(same(s1.data(), s2.data(), s1.size()), "cpy1Dto2D_shr %d", n);
            c.copy_sp(o1.data(), 64, B.sp(), S); xo_copy_sp(n, n, o2.data(), 64, B.sp(), S);
            EXPECT(same(o1.data(), o2.data(), o1.size()), "copy_sp %d", n);
            c.copy_ps(s1.data(), 64, A.pp(), S); xo_copy_ps(n, n, s2.data(), 64, A.pp(), S);
            EXPECT(same(s1.data(), s2.data(), s1.size()), "copy_ps %d", n);
            c.copy_ss(s1.data(), 64, A.sp(), S); xo_copy_ss(n, n, s2.data(), 64, A.sp(), S);
            EXPECT(same(s1.data(), s2.data(), s1.size()), "copy_ss %d", n);
            c.copy_pp(o1.data(), 64, A.pp(), S); xo_copy_pp(n, n, o2.data(), 64, A.pp(), S);
            EXPECT(same(o1.data(), o2.data(), o1.size()), "cu copy_pp %d", n);
            c.transpose(o1.data(), A.pp(), S); xo_transpose(n, o2.data(), A.pp(), S);
            EXPECT(same(o1.data(), o2.data(), o1.size()), "transpose %d", n);
            if (n > 32) continue;
            {
                std::vector<int16_t> q(n * n), k1(n * n), k2(n * n);
                for (auto& v : q) v = (int16_t)(rnd() % 4 == 0 ? (int)(rnd() % 200) - 100 : 0);
                EXPECT(c.count_nonzero(q.data()) == xo_count_nonzero(n, q.data()), "count_nonzero %d", n);
                EXPECT(c.copy_cnt(k1.data(), A.sp(), S) == xo_copy_cnt(n, k2.data(), A.sp(), S), "copy_cnt ret %d", n);
                EXPECT(same(k1.data(), k2.data(), n * n), "copy_cnt %d", n);
            }
            std::vector<int16_t> res(n * n), co1(n * n), co2(n * n);
            for (auto& v : res) v = (int16_t)((int)(rnd() % (2 * PMAX + 1)) - PMAX);
            c.dct(res.data(), co1.data(), n); xo_dct(XO_DCT, n, res.data(), co2.data(), n);
            EXPECT(same(co1.data(), co2.data(), n * n), "dct %d", n);
            c.idct(A.sp(), s1.data(), 64); xo_dct(XO_IDCT, n, A.sp(), s2.data(), 64);
            EXPECT(same(s1.data(), s2.data(), s1.size()), "idct %d", n);
            std::vector<pixel> nb(4 * n + 1), f1(4 * n + 1), f2(4 * n + 1), all1(33 * n * n), all2(33 * n * n);
            for (auto& v : nb) v = (pixel)(iter % 3 == 0 ? rnd() % (PMAX + 1) : iter % 3 == 1 ? 0 : PMAX);
            c.intra_filter(nb.data(), f1.data()); xo_intra_filter(n, nb.data(), f2.data());
            EXPECT(same(f1.data(), f2.data(), f1.size()), "intra_filter %d", n);
            for (int m = 0; m < 35; m++)
            {
                memset(o1.data(), 0xCD, o1.size() * sizeof(pixel)); memset(o2.data(), 0xCD, o2.size() * sizeof(pixel));
                c.intra_pred[m](o1.data(), 64, nb.data(), m, n <= 16);
                xo_intra_pred(n, m, o2.data(), 64, nb.data(), n <= 16);
                EXPECT(same(o1.data(), o2.data(), o1.size()), "intra_pred %d mode %d", n, m);
            }
            c.intra_pred_allangs(all1.data(), nb.data(), f1.data(), 1);
            xo_intra_allangs(n, all2.data(), nb.data(), f1.data(), 1);
            EXPECT(same(all1.data(), all2.data(), all1.size()), "allangs %d", n);
            // quant family
            const int num = n * n;
            std::vector<int32_t> qc(num), d1(num), d2(num);
            std::vector<int16_t> q1(num), q2(num), coef(num);
            for (int k = 0; k < num; k++) { qc[k] = (int)(rnd() % 30000); coef[k] = (int16_t)((int)(rnd() % 511) - 255); }
            const int qb = 16 + iter, add = 85 << (qb - 9);
            EXPECT(tab.quant(coef.data(), qc.data(), d1.data(), q1.data(), qb, add, num) ==
                   xo_quant(coef.data(), qc.data(), d2.data(), q2.data(), qb, add, num), "quant ret %d", n);
            EXPECT(same(q1.data(), q2.data(), num) && same(d1.data(), d2.data(), num), "quant %d", n);
            EXPECT(tab.nquant(coef.data(), qc.data(), q1.data(), qb, add, num) ==
                   xo_nquant(coef.data(), qc.data(), q2.data(), qb, add, num), "nquant ret %d", n);
            EXPECT(same(q1.data(), q2.data(), num), "nquant %d", n);
            tab.dequant_normal(coef.data(), q1.data(), num, 72 << 3, 3); xo_dequant_normal(coef.data(), q2.data(), num, 72 << 3, 3);
            EXPECT(same(q1.data(), q2.data(), num), "dequant_normal %d", n);
            tab.dequant_scaling(coef.data(), qc.data(), q1.data(), num, 4, 3); xo_dequant_scaling(coef.data(), qc.data(), q2.data(), num, 4, 3);
            EXPECT(same(q1.data(), q2.data(), num), "dequant_scaling %d", n);
            {
                std::vector<uint16_t> off(num);
                std::vector<uint32_t> rs1(num), rs2(num);
                for (int k = 0; k < num; k++)
                {
                    off[k] = (uint16_t)(rnd() % (k & 1 ? 65535 : 2048));
                    rs1[k] = rs2[k] = 0xFFFFF000u + rnd() % 8192;
                    q1[k] = q2[k] = (int16_t)((int)(rnd() % 32768) - (int)(rnd() % 32768));
                }
                tab.denoiseDct(q1.data(), rs1.data(), off.data(), num); xo_denoise_dct(q2.data(), rs2.data(), off.data(), num);
                EXPECT(same(q1.data(), q2.data(), num) && same(rs1.data(), rs2.data(), num), "denoiseDct %d", n);
            }
        }
        std::vector<int16_t> r4(16), c1(16), c2(16);
        for (auto& v : r4) v = (int16_t)((int)(rnd() % (2 * PMAX + 1)) - PMAX);
        tab.dst4x4(r4.data(), c1.data(), 4); xo_dct(XO_DST, 4, r4.data(), c2.data(), 4);
        EXPECT(same(c1.data(), c2.data(), 16), "dst4");
        tab.idst4x4(A.sp(), s1.data(), 64); xo_dct(XO_IDST, 4, A.sp(), s2.data(), 64);
        EXPECT(same(s1.data(), s2.data(), s1.size()), "idst4");
    }
    printf("depth %d: %d provider checks, %d failures\n", X265_DEPTH, g_checks, g_fail);
    return g_fail ? 1 : 0;
}
