/* hip_bridge.cpp — TEST INFRASTRUCTURE: the reference TestBench's provider hook
 * pointed at the MI355X provider (SURVEY.md §8(c) "TestBench without yasm").
 *
 * The reference TestBench (x265_1.9/source/test/testbench.cpp:153-243) checks a
 * candidate table against its own C table `cprim`: for every CPU arch selected
 * by --cpuid it calls setupInstrinsicPrimitives(vecprim, flag) and
 * setupAssemblyPrimitives(asmprim, flag) (testbench.cpp:196,212), adds the
 * aliases and runs each harness's testCorrectness(cprim, candidate).  A build
 * without assembly has no definitions of those two hooks (primitives.cpp:241-242
 * are compiled out), so this translation unit provides them:
 *
 *   setupInstrinsicPrimitives : nothing (the intrinsic pass then tests an empty
 *                               table, i.e. nothing, exactly as a no-asm build);
 *   setupAssemblyPrimitives   : the MI355X provider, through its C entry
 *                               x265amd_setup_primitives(table, X265_DEPTH)
 *                               (include/x265_amd.h), so every non-NULL entry the
 *                               provider implements is a GPU round trip.
 *
 * The final call (testbench.cpp:231-232, the speed pass) skips aliases; the
 * reference's measureSpeed dereferences aliased chroma slots, so this hook adds
 * them itself (setupAliasPrimitives is idempotent).  X265AMD_TB_SPEED=0 leaves
 * the speed-pass table on the C primitives: per-call round trips make that pass
 * a latency measurement of PCIe, not of the kernels, and it takes minutes.
 *
 * Nothing here is reference source: the reference's test/*.cpp and library
 * objects are compiled where they lie (oracle/Makefile testbench).
 */
#include "common.h"
#include "primitives.h"

#include <cstdio>
#include <cstdlib>

extern "C" int x265amd_setup_primitives(void* table, int depth, int* overridden);
extern "C" const char* x265amd_strerror(int status);

namespace X265_NS {

void setupInstrinsicPrimitives(EncoderPrimitives&, int) {}

void setupAssemblyPrimitives(EncoderPrimitives& p, int)
{
    static int calls = 0;
    const char* sp = getenv("X265AMD_TB_SPEED");
    const bool speedPass = ++calls > 1;   /* correctness pass first (one --cpuid arch) */
    if (speedPass && sp && sp[0] == '0')
    {
        setupCPrimitives(p);
        setupAliasPrimitives(p);
        return;
    }
    setupCPrimitives(p);   /* like the layering of primitives.cpp:232-245: C first; allangs
                              stays non-NULL here, as in TestBench's cprim (testbench.cpp:155) */
    int n = 0;
    int rc = x265amd_setup_primitives(&p, X265_DEPTH, &n);
    if (rc)
    {
        fprintf(stderr, "x265amd_setup_primitives failed: %s\n", x265amd_strerror(rc));
        exit(3);
    }
    setupAliasPrimitives(p);
    printf("[hip_bridge] MI355X provider installed: %d entries (%d-bit)\n", n, X265_DEPTH);
    fflush(stdout);
}

}
