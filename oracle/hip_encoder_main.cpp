/* hip_encoder_main.cpp — TEST/MEASUREMENT INFRASTRUCTURE: the reference x265 1.9
 * CLI and encoder (compiled where they lie under /root/reference, see
 * oracle/Makefile x265hip) with the MI355X provider installed in the global
 * primitive table, i.e. the INTEGRATION.md §1 patch applied from outside:
 *
 *   x265_setup_primitives (primitives.cpp:228-249) = setupCPrimitives, allangs
 *   NULL, [asm providers], setupAliasPrimitives, guarded by
 *   `if (!primitives.pu[0].sad)` (primitives.cpp:230).
 *
 * Before the CLI's main runs, this fills `x265::primitives` the same way with
 * the MI355X provider (x265amd_setup_primitives, include/x265_amd.h) in the
 * place of the assembly providers; the encoder's own once-only guard then leaves
 * the table alone, so x265_encoder_open / x265_encoder_encode (api.cpp:182) run
 * every primitive the provider implements on the GPU.
 *
 *   X265AMD_PROVIDER=c    keeps the plain C table (same binary, CPU reference)
 *   X265AMD_PROVIDER=hip  (default) MI355X provider
 *
 * Prints "[x265hip] provider=<c|hip> entries=<n>" on stderr before encoding.
 *
 * Error channel: the provider keeps the first failure of any call in a sticky
 * status (x265amd_provider_status, include/x265_amd_primitives.h).  The CLI gets
 * its API table from x265_api_get (x265.cpp:219-223); this binary is linked with
 * -Wl,--wrap=x265_api_get_79, so the table it gets is the reference's with
 * encoder_encode wrapped: a non-zero provider status turns the call into the
 * documented failure, x265_encoder_encode() < 0 (x265.h:1351-1359), and the CLI
 * aborts with exit code 4 (x265.cpp:643-649, 677-681).
 */
#include "common.h"
#include "primitives.h"

#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <execinfo.h>
#include <unistd.h>

extern "C" int x265amd_setup_primitives(void* table, int depth, int* overridden);
extern "C" const char* x265amd_strerror(int status);
extern "C" int x265amd_provider_status(void);

extern "C" const x265_api* __real_x265_api_get_79(int bitDepth);
/* x265la builds (integration/gpu_me.cpp, gpu_lookahead.cpp): drop the closed encoder's device sessions */
extern "C" void x265amd_me_encoder_closed(void) __attribute__((weak));
extern "C" void x265amd_la_encoder_closed(void) __attribute__((weak));
extern "C" long long x265amd_host_unregister_stale(void) __attribute__((weak));
/* x265la builds (integration/gpu_rdo.cpp): psy_cost_pp thunks into the table, the closed encoder's sessions */
extern "C" void x265amd_rdo_install(void* table) __attribute__((weak));
extern "C" void x265amd_rdo_encoder_closed(void) __attribute__((weak));

namespace {
/* X265AMD_PHASES=1: wall-clock stamps of the process's phases (main, the encoder's close, exit) on stderr, for
 * the start-up / teardown share of a bench step (tools/phases.py) */
bool g_phases = false;
void phase(const char* what)
{
    if (!g_phases) return;
    struct timespec t;
    clock_gettime(CLOCK_REALTIME, &t);
    fprintf(stderr, "[phase] %s %.6f\n", what, t.tv_sec + 1e-9 * t.tv_nsec);
}
void phase_exit() { phase("exit"); }

x265_api g_api;
int (*g_encode)(x265_encoder*, x265_nal**, uint32_t*, x265_picture*, x265_picture*);
void (*g_close)(x265_encoder*);

void drop_sessions()
{
    if (x265amd_me_encoder_closed)
        x265amd_me_encoder_closed();
    phase("me_dropped");
    if (x265amd_la_encoder_closed)
        x265amd_la_encoder_closed();
    phase("la_dropped");
    if (x265amd_rdo_encoder_closed)
        x265amd_rdo_encoder_closed();
}

/* The device sessions page-lock the encoder's reconstruction planes (PicYuv) and Lowres buffers and may
 * still have uploads from them in flight; x265_encoder_close (api.cpp:234-246) frees those buffers in
 * Encoder::destroy.  So the sessions are drained, unregistered and destroyed BEFORE the encoder frees
 * its frames: the CLI has flushed the encoder by then (x265.cpp: encoder_encode(NULL) until it returns 0),
 * so no search or estimate is running.  A session opened during the close itself (none in a flushed
 * encoder) is dropped after it. */
void closing(x265_encoder* enc)
{
    /* X265AMD_ROUND5_CLOSE_ORDER=1: the round-5 order (sessions dropped only after the encoder freed its
     * frames), kept so tests/test_encoder_me.py can show the stale-unregister count catches it */
    const char* old = getenv("X265AMD_ROUND5_CLOSE_ORDER");
    phase("close");
    if (!(old && *old == '1'))
        drop_sessions();
    phase("sessions_dropped");
    g_close(enc);
    drop_sessions();
    phase("closed");
    if (x265amd_host_unregister_stale && x265amd_host_unregister_stale())
        fprintf(stderr, "[x265hip] %lld page-locked host buffers were freed before their session unregistered them\n",
                x265amd_host_unregister_stale());
}

x265_encoder* (*g_open)(x265_param*);
bool g_first = true;

x265_encoder* opening(x265_param* p)
{
    phase("open");
    x265_encoder* e = g_open(p);
    phase("opened");
    return e;
}

int checked_encode(x265_encoder* enc, x265_nal** pp_nal, uint32_t* pi_nal, x265_picture* in, x265_picture* out)
{
    if (g_first)
    {
        g_first = false;
        phase("first_encode");
    }
    int n = g_encode(enc, pp_nal, pi_nal, in, out);
    int st = x265amd_provider_status();
    if (st)
    {
        fprintf(stderr, "[x265hip] MI355X provider failed: %s (status %d); x265_encoder_encode -> -1\n",
                x265amd_strerror(st), st);
        return -1;
    }
    return n;
}
}

extern "C" const x265_api* __wrap_x265_api_get_79(int bitDepth)
{
    const x265_api* api = __real_x265_api_get_79(bitDepth);
    if (!api) return api;
    g_api = *api;
    g_encode = api->encoder_encode;
    g_api.encoder_encode = checked_encode;
    g_close = api->encoder_close;
    g_api.encoder_close = closing;
    g_open = api->encoder_open;
    g_api.encoder_open = opening;
    return &g_api;
}

using namespace X265_NS;

int x265_cli_main(int argc, char** argv);

/* a crash names its place (binaries are linked with -rdynamic) */
static void on_fatal(int sig)
{
    void* bt[64];
    int n = backtrace(bt, 64);
    fprintf(stderr, "[x265hip] fatal signal %d, backtrace:\n", sig);
    backtrace_symbols_fd(bt, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

int main(int argc, char** argv)
{
    {
        const char* e = getenv("X265AMD_PHASES");
        g_phases = e && *e == '1';
        phase("main");
        if (g_phases) atexit(phase_exit);
    }
    signal(SIGSEGV, on_fatal);
    signal(SIGBUS, on_fatal);
    const char* which = getenv("X265AMD_PROVIDER");
#ifdef X265AMD_DEFAULT_PROVIDER_C
    /* x265la: the C table unless the per-call provider is asked for */
    const bool hip = which && !strcmp(which, "hip");
#else
    const bool hip = !(which && !strcmp(which, "c"));
#endif
    EncoderPrimitives& p = primitives;
    setupCPrimitives(p);
    for (int i = 0; i < NUM_TR_SIZE; i++)
        p.cu[i].intra_pred_allangs = NULL;
    int n = 0;
    if (hip)
    {
        int rc = x265amd_setup_primitives(&p, X265_DEPTH, &n);
        if (rc)
        {
            fprintf(stderr, "[x265hip] x265amd_setup_primitives failed: %s\n", x265amd_strerror(rc));
            return 3;
        }
    }
    setupAliasPrimitives(p);
    if (x265amd_rdo_install)
        x265amd_rdo_install(&p);
    fprintf(stderr, "[x265hip] provider=%s entries=%d depth=%d\n", hip ? "hip" : "c", n, X265_DEPTH);
    return x265_cli_main(argc, argv);
}
