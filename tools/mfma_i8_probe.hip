// mfma_i8_probe.hip — which A / B fragment lane map does v_mfma_i32_32x32x32_i8 use on gfx950?
// (cdna_hip_programming.md: "Other dtypes: check the map with exact integer data").  Random
// ASYMMETRIC int8 A (32x32) and B (32x32); each hypothesis builds the per-lane 16-byte fragments
// (lane l: r = l & 31, h = l >> 5; element j of the fragment = A[r][k(h, j)] / B[k(h, j)][r]),
// the product is read from the standard 32x32 C map (row (i&3) + 8(i>>2) + 4h, col r) and
// compared with the exact CPU product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

__global__ void k_probe(const i32x4* a, const i32x4* b, i32x16* c)
{
    const int l = threadIdx.x;
    c[l] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[l], b[l], (i32x16){}, 0, 0, 0);
}

static int kmap(int hyp, int h, int j)
{
    if (hyp == 0) return 16 * h + j;                                  // contiguous halves
    if (hyp == 1) return j < 8 ? 8 * h + j : 16 + 8 * h + (j - 8);    // two f16-style K steps
    return 2 * j + h;                                                 // interleaved
}

int main()
{
    int8_t A[32][32], B[32][32];
    srand(7);
    for (int i = 0; i < 32; i++)
        for (int k = 0; k < 32; k++) { A[i][k] = (int8_t)(rand() % 256 - 128); B[i][k] = (int8_t)(rand() % 256 - 128); }
    int C[32][32];
    for (int i = 0; i < 32; i++)
        for (int j = 0; j < 32; j++)
        {
            int s = 0;
            for (int k = 0; k < 32; k++) s += A[i][k] * B[k][j];
            C[i][j] = s;
        }
    i32x4 *da, *db;
    i32x16* dc;
    hipMalloc(&da, 64 * sizeof(i32x4));
    hipMalloc(&db, 64 * sizeof(i32x4));
    hipMalloc(&dc, 64 * sizeof(i32x16));
    int best = -1;
    for (int hyp = 0; hyp < 3; hyp++)
    {
        int8_t fa[64][16], fb[64][16];
        for (int l = 0; l < 64; l++)
            for (int j = 0; j < 16; j++)
            {
                const int r = l & 31, h = l >> 5, k = kmap(hyp, h, j);
                fa[l][j] = A[r][k];
                fb[l][j] = B[k][r];
            }
        hipMemcpy(da, fa, sizeof(fa), hipMemcpyHostToDevice);
        hipMemcpy(db, fb, sizeof(fb), hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, da, db, dc);
        int out[64][16];
        if (hipMemcpy(out, dc, sizeof(out), hipMemcpyDeviceToHost) != hipSuccess) { printf("hip error\n"); return 1; }
        int bad = 0;
        for (int l = 0; l < 64; l++)
            for (int i = 0; i < 16; i++)
            {
                const int row = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5), col = l & 31;
                bad += out[l][i] != C[row][col];
            }
        printf("{\"hypothesis\": %d, \"mismatches\": %d, \"of\": 1024}\n", hyp, bad);
        if (!bad && best < 0) best = hyp;
    }
    printf("{\"layout\": %d}\n", best);
    return best < 0;
}
