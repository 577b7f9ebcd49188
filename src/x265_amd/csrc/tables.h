// tables.h — HEVC constant tables used by the kernels, as per-TU __constant__
// data (no relocatable device code needed).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace x265amd {

// HEVC core transform.  Rather than transcribing x265's g_t4..g_t32
// (constants.cpp:259-333), the 32x32 matrix is generated from the spec's
// rule T32[k][n] = c(k*(2n+1) mod 128), where c() folds the 32 cosine
// magnitudes below onto the four quadrants; T16/T8/T4 are rows 2k/4k/8k.
struct TransformMatrix { int16_t m[32][32]; };

constexpr int kCosMag[33] = { 64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67,
                              64, 61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9, 4, 0 };

constexpr int fold_cos(int a)
{
    return a <= 32 ? kCosMag[a] : a <= 64 ? -kCosMag[64 - a] : a <= 96 ? -kCosMag[a - 64] : kCosMag[128 - a];
}

constexpr TransformMatrix make_t32()
{
    TransformMatrix t{};
    for (int k = 0; k < 32; k++)
        for (int n = 0; n < 32; n++)
            t.m[k][n] = (int16_t)fold_cos((k * (2 * n + 1)) & 127);
    return t;
}

static __constant__ TransformMatrix c_t32 = make_t32();

// Sub-pel interpolation filters (HEVC spec 8.5.3.3.3; x265 g_lumaFilter /
// g_chromaFilter, constants.cpp:239-257).
struct LumaTaps { int16_t c[4][8]; };
struct ChromaTaps { int16_t c[8][4]; };
static __constant__ LumaTaps c_luma = { { { 0, 0, 0, 64, 0, 0, 0, 0 },
                                          { -1, 4, -10, 58, 17, -5, 1, 0 },
                                          { -1, 4, -11, 40, 40, -11, 4, -1 },
                                          { 0, 1, -5, 17, 58, -10, 4, -1 } } };
static __constant__ ChromaTaps c_chroma = { { { 0, 64, 0, 0 }, { -2, 58, 10, -2 }, { -4, 54, 16, -2 },
                                              { -6, 46, 28, -4 }, { -4, 36, 36, -4 }, { -4, 28, 46, -6 },
                                              { -2, 16, 54, -4 }, { -2, 10, 58, -2 } } };

// Intra: HEVC intraPredAngle / invAngle (intrapred.cpp:123-124) and the
// filtered-reference flags g_intraFilterFlags (constants.cpp:550-556).
struct IntraTabs
{
    int8_t angle[17];
    int16_t inv_angle[8];
    uint8_t filter_flags[35];
};
static __constant__ IntraTabs c_intra = {
    { -32, -26, -21, -17, -13, -9, -5, -2, 0, 2, 5, 9, 13, 17, 21, 26, 32 },
    { 4096, 1638, 910, 630, 482, 390, 315, 256 },
    { 0x38, 0x00, 0x38, 0x30, 0x30, 0x30, 0x30, 0x30, 0x30, 0x20, 0x00, 0x20, 0x30, 0x30, 0x30, 0x30, 0x30, 0x30,
      0x38, 0x30, 0x30, 0x30, 0x30, 0x30, 0x30, 0x20, 0x00, 0x20, 0x30, 0x30, 0x30, 0x30, 0x30, 0x30, 0x38 }
};

} // namespace x265amd
