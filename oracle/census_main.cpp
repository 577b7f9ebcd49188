/* census_main.cpp — exact per-entry call census of the reference encoder.
 *
 * TEST/MEASUREMENT INFRASTRUCTURE ONLY (oracle/, never part of the product).
 *
 * Builds into oracle/_ref/x265census together with the reference's own CLI
 * (x265.cpp compiled with -Dmain=x265_cli_main) and library objects.  Before
 * the CLI runs, the global table `x265::primitives` is filled exactly as
 * x265_setup_primitives() does for a --no-asm build (primitives.cpp:228-249:
 * C provider, allangs NULL, aliases) and then every non-NULL slot is replaced
 * by a tiny x86-64 thunk that atomically counts the call and tail-jumps to the
 * original function.  Because the table is already populated, the encoder's
 * own once-only guard (primitives.cpp:230) leaves it alone.  At exit the
 * per-slot counts are written as JSON to $X265_CENSUS_OUT.
 *
 * The census defines the per-frame primitive workload that bench.py replays
 * on the GPU.
 */
#include "common.h"
#include "primitives.h"

#include <sys/mman.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstddef>
#include <string>
#include <vector>

using namespace X265_NS;

int x265_cli_main(int argc, char** argv);

namespace {

const int kPuW[NUM_PU_SIZES] = { 4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 12, 16, 4, 32, 24, 32, 8, 64, 48, 64, 16 };
const int kPuH[NUM_PU_SIZES] = { 4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 12, 16, 4, 16, 24, 32, 8, 32, 48, 64, 16, 64 };

const size_t kSlots = sizeof(EncoderPrimitives) / sizeof(void*);
std::vector<std::string> g_names(kSlots);
uint64_t* g_counts;

void nameSlot(size_t byteOff, const std::string& n)
{
    g_names[byteOff / sizeof(void*)] = n;
}

std::string dims(int w, int h)
{
    char b[32];
    snprintf(b, sizeof(b), "%dx%d", w, h);
    return b;
}

#define PU_FIELDS(X) X(sad) X(sad_x3) X(sad_x4) X(satd) X(luma_hpp) X(luma_hps) X(luma_vpp) \
    X(luma_vps) X(luma_vsp) X(luma_vss) X(luma_hvpp) X(pixelavg_pp) X(addAvg) X(copy_pp) X(convert_p2s)
#define CU_FIELDS(X) X(dct) X(idct) X(calcresidual) X(sub_ps) X(add_ps) X(blockfill_s) X(copy_cnt) \
    X(count_nonzero) X(cpy2Dto1D_shl) X(cpy2Dto1D_shr) X(cpy1Dto2D_shl) X(cpy1Dto2D_shr) X(copy_sp) \
    X(copy_ps) X(copy_ss) X(copy_pp) X(var) X(sse_pp) X(sse_ss) X(psy_cost_pp) X(ssd_s) X(sa8d) \
    X(transpose) X(intra_pred_allangs) X(intra_filter)
#define CPU_FIELDS(X) X(satd) X(filter_vpp) X(filter_vps) X(filter_vsp) X(filter_vss) X(filter_hpp) \
    X(filter_hps) X(addAvg) X(copy_pp) X(p2s)
#define CCU_FIELDS(X) X(sa8d) X(sse_pp) X(sub_ps) X(add_ps) X(copy_ps) X(copy_sp) X(copy_ss) X(copy_pp)
#define SCALAR_FIELDS(X) X(dst4x4) X(idst4x4) X(quant) X(nquant) X(dequant_scaling) X(dequant_normal) \
    X(denoiseDct) X(scale1D_128to64) X(scale2D_64to32) X(ssim_4x4x2_core) X(ssim_end_4) X(sign) \
    X(saoCuOrgE0) X(saoCuOrgE1) X(saoCuOrgE1_2Rows) X(saoCuOrgB0) X(saoCuStatsBO) X(saoCuStatsE0) \
    X(saoCuStatsE1) X(saoCuStatsE2) X(saoCuStatsE3) X(frameInitLowres) X(propagateCost) \
    X(extendRowBorder) X(planecopy_cp) X(planecopy_sp) X(planecopy_sp_shl) X(planeClipAndMax) \
    X(weight_sp) X(weight_pp) X(scanPosLast) X(findPosFirstLast) X(costCoeffNxN) X(costCoeffRemain) \
    X(costC1C2Flag)

void buildNames()
{
    for (size_t i = 0; i < kSlots; i++)
    {
        char b[32];
        snprintf(b, sizeof(b), "slot%zu", i);
        g_names[i] = b;
    }
    for (int p = 0; p < NUM_PU_SIZES; p++)
    {
        size_t base = offsetof(EncoderPrimitives, pu) + p * sizeof(EncoderPrimitives::PU);
#define X(f) nameSlot(base + offsetof(EncoderPrimitives::PU, f), "pu." #f "." + dims(kPuW[p], kPuH[p]));
        PU_FIELDS(X)
#undef X
    }
    for (int c = 0; c < NUM_CU_SIZES; c++)
    {
        size_t base = offsetof(EncoderPrimitives, cu) + c * sizeof(EncoderPrimitives::CU);
        int n = 4 << c;
#define X(f) nameSlot(base + offsetof(EncoderPrimitives::CU, f), "cu." #f "." + dims(n, n));
        CU_FIELDS(X)
#undef X
        for (int m = 0; m < NUM_INTRA_MODE; m++)
        {
            char b[64];
            snprintf(b, sizeof(b), "cu.intra_pred.%dx%d.mode%d", n, n, m);
            nameSlot(base + offsetof(EncoderPrimitives::CU, intra_pred) + m * sizeof(void*), b);
        }
    }
#define X(f) nameSlot(offsetof(EncoderPrimitives, f), "scalar." #f);
    SCALAR_FIELDS(X)
#undef X
    nameSlot(offsetof(EncoderPrimitives, saoCuOrgE2), "scalar.saoCuOrgE2[0]");
    nameSlot(offsetof(EncoderPrimitives, saoCuOrgE2) + sizeof(void*), "scalar.saoCuOrgE2[1]");
    nameSlot(offsetof(EncoderPrimitives, saoCuOrgE3), "scalar.saoCuOrgE3[0]");
    nameSlot(offsetof(EncoderPrimitives, saoCuOrgE3) + sizeof(void*), "scalar.saoCuOrgE3[1]");
    nameSlot(offsetof(EncoderPrimitives, pelFilterLumaStrong), "scalar.pelFilterLumaStrong[0]");
    nameSlot(offsetof(EncoderPrimitives, pelFilterLumaStrong) + sizeof(void*), "scalar.pelFilterLumaStrong[1]");

    static const char* cspName[X265_CSP_COUNT] = { "i400", "i420", "i422", "i444" };
    for (int c = 0; c < X265_CSP_COUNT; c++)
    {
        int hs = (c == X265_CSP_I420 || c == X265_CSP_I422) ? 1 : 0;
        int vs = (c == X265_CSP_I420) ? 1 : 0;
        size_t cb = offsetof(EncoderPrimitives, chroma) + c * sizeof(EncoderPrimitives::Chroma);
        for (int p = 0; p < NUM_PU_SIZES; p++)
        {
            size_t base = cb + offsetof(EncoderPrimitives::Chroma, pu) + p * sizeof(EncoderPrimitives::Chroma::PUChroma);
            std::string d = dims(kPuW[p] >> hs, kPuH[p] >> vs);
#define X(f) nameSlot(base + offsetof(EncoderPrimitives::Chroma::PUChroma, f), std::string("chroma.") + cspName[c] + ".pu." #f "." + d);
            CPU_FIELDS(X)
#undef X
        }
        for (int i = 0; i < NUM_CU_SIZES; i++)
        {
            size_t base = cb + offsetof(EncoderPrimitives::Chroma, cu) + i * sizeof(EncoderPrimitives::Chroma::CUChroma);
            std::string d = dims((4 << i) >> hs, (4 << i) >> vs);
#define X(f) nameSlot(base + offsetof(EncoderPrimitives::Chroma::CUChroma, f), std::string("chroma.") + cspName[c] + ".cu." #f "." + d);
            CCU_FIELDS(X)
#undef X
        }
    }
}

/* movabs r11, imm64 ; lock inc qword [r11] ; movabs r11, imm64 ; jmp r11 */
void emitThunk(uint8_t* t, uint64_t* counter, void* target)
{
    uint64_t c = (uint64_t)counter, f = (uint64_t)target;
    uint8_t* p = t;
    *p++ = 0x49; *p++ = 0xBB; memcpy(p, &c, 8); p += 8;
    *p++ = 0xF0; *p++ = 0x49; *p++ = 0xFF; *p++ = 0x03;
    *p++ = 0x49; *p++ = 0xBB; memcpy(p, &f, 8); p += 8;
    *p++ = 0x41; *p++ = 0xFF; *p++ = 0xE3;
    while (p < t + 32) *p++ = 0xCC;
}

void installCensus()
{
    EncoderPrimitives& p = primitives;
    setupCPrimitives(p);
    for (int i = 0; i < NUM_TR_SIZE; i++)
        p.cu[i].intra_pred_allangs = NULL;
    setupAliasPrimitives(p);

    g_counts = (uint64_t*)calloc(kSlots, sizeof(uint64_t));
    uint8_t* code = (uint8_t*)mmap(NULL, kSlots * 32, PROT_READ | PROT_WRITE | PROT_EXEC,
                                   MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (code == MAP_FAILED) { perror("mmap"); exit(1); }
    void** slots = (void**)&p;
    for (size_t i = 0; i < kSlots; i++)
    {
        if (!slots[i]) continue;
        emitThunk(code + 32 * i, &g_counts[i], slots[i]);
        slots[i] = code + 32 * i;
    }
}

void dumpCensus()
{
    const char* out = getenv("X265_CENSUS_OUT");
    FILE* f = out ? fopen(out, "w") : stderr;
    if (!f) { perror("census out"); return; }
    fprintf(f, "{\n  \"depth\": %d,\n  \"counts\": {", X265_DEPTH);
    bool first = true;
    for (size_t i = 0; i < kSlots; i++)
    {
        if (!g_counts[i]) continue;
        fprintf(f, "%s\n    \"%s\": %llu", first ? "" : ",", g_names[i].c_str(), (unsigned long long)g_counts[i]);
        first = false;
    }
    fprintf(f, "\n  }\n}\n");
    if (out) fclose(f);
}

} // namespace

int main(int argc, char** argv)
{
    buildNames();
    installCensus();
    int r = x265_cli_main(argc, argv);
    dumpCensus();
    return r;
}
