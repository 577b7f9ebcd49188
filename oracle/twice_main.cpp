/* twice_main.cpp — TEST INFRASTRUCTURE (oracle/Makefile twice): two encoders of the SAME geometry opened
 * one after the other in ONE process through the public x265 API (x265.h: x265_encoder_open / _headers /
 * _encode / _close), each encoding the same raw 4:2:0 clip, with the MI355X hooks of integration/ linked
 * in.  Before each x265_encoder_close frees the encoder's frames the binding's teardown runs
 * (x265amd_me_encoder_closed, x265amd_la_encoder_closed — the calls INTEGRATION.md §3 adds to Encoder::destroy
 * ahead of the frame teardown), so the page-locked planes are unregistered while still allocated.  The second encoder
 * reuses freed Frame / PicYuv / Lowres addresses and the same POCs, so a device session that kept the first
 * encoder's pictures would search stale reconstructions: tests/test_encoder_me.py checks that both
 * bitstreams equal those of the same program with the hooks off (X265AMD_LOOKAHEAD=cpu X265AMD_ME=cpu: the
 * reference encoder's own functions).
 *
 *   twice <input.yuv> <width> <height> <frames> <out1.hevc> <out2.hevc> [preset]
 *
 * Stream layout as the reference CLI writes it (x265.cpp): the parameter-set headers, then every NAL of
 * every access unit, then the flushed ones; no version SEI, 30 fps (the parameter sets differ from the CLI's
 * in two header bytes: the CLI also fills VUI fields from its input options).
 */
#include "x265.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

extern "C" void x265amd_me_encoder_closed(void) __attribute__((weak));
extern "C" void x265amd_la_encoder_closed(void) __attribute__((weak));
extern "C" long long x265amd_host_unregister_stale(void) __attribute__((weak));
extern "C" void x265amd_rdo_encoder_closed(void) __attribute__((weak));

static void write_nals(FILE* f, const x265_nal* nal, uint32_t n)
{
    for (uint32_t i = 0; i < n; i++)
        fwrite(nal[i].payload, 1, nal[i].sizeBytes, f);
}

static int encode(const char* in, int w, int h, int frames, const char* out, const char* preset)
{
    const x265_api* api = x265_api_get(0);
    if (!api) return 2;
    x265_param* p = api->param_alloc();
    if (api->param_default_preset(p, preset, NULL) < 0) return 2;
    p->sourceWidth = w;
    p->sourceHeight = h;
    p->fpsNum = 30;
    p->fpsDenom = 1;
    p->internalCsp = X265_CSP_I420;
    p->bEmitInfoSEI = 0;
    p->totalFrames = frames;
    /* the GPU box shows the whole machine's CPUs but grants a 16-core share: size the pool for the share */
    if (api->param_parse(p, "pools", "16") < 0) return 2;
    x265_encoder* enc = api->encoder_open(p);
    if (!enc) return 3;
    FILE* fo = fopen(out, "wb");
    FILE* fi = fopen(in, "rb");
    if (!fo || !fi) return 4;
    x265_nal* nal;
    uint32_t nn;
    if (api->encoder_headers(enc, &nal, &nn) < 0) return 5;
    write_nals(fo, nal, nn);
    std::vector<uint8_t> buf((size_t)w * h * 3 / 2);
    x265_picture* pic = api->picture_alloc();
    api->picture_init(p, pic);
    int rc = 0;
    for (int i = 0; i < frames && !rc; i++)
    {
        if (fread(buf.data(), 1, buf.size(), fi) != buf.size()) { rc = 6; break; }
        pic->planes[0] = buf.data();
        pic->planes[1] = buf.data() + (size_t)w * h;
        pic->planes[2] = buf.data() + (size_t)w * h * 5 / 4;
        pic->stride[0] = w;
        pic->stride[1] = pic->stride[2] = w / 2;
        pic->bitDepth = 8;
        pic->pts = i;
        if (api->encoder_encode(enc, &nal, &nn, pic, NULL) < 0) rc = 7;
        else write_nals(fo, nal, nn);
    }
    while (!rc)
    {
        const int got = api->encoder_encode(enc, &nal, &nn, NULL, NULL);
        if (got < 0) rc = 7;
        if (got <= 0) break;
        write_nals(fo, nal, nn);
    }
    api->picture_free(pic);
    /* the binding's teardown while the flushed encoder's frames still exist */
    if (x265amd_me_encoder_closed) x265amd_me_encoder_closed();
    if (x265amd_la_encoder_closed) x265amd_la_encoder_closed();
    if (x265amd_rdo_encoder_closed) x265amd_rdo_encoder_closed();
    api->encoder_close(enc);
    api->param_free(p);
    if (x265amd_host_unregister_stale && x265amd_host_unregister_stale())
        fprintf(stderr, "[twice] %lld page-locked host buffers were freed before their session unregistered them\n",
                x265amd_host_unregister_stale());
    fclose(fi);
    fclose(fo);
    return rc;
}

int main(int argc, char** argv)
{
    if (argc < 7)
    {
        fprintf(stderr, "usage: %s in.yuv w h frames out1.hevc out2.hevc [preset]\n", argv[0]);
        return 1;
    }
    const int w = atoi(argv[2]), h = atoi(argv[3]), n = atoi(argv[4]);
    const char* preset = argc > 7 ? argv[7] : "medium";
    for (int k = 0; k < 2; k++)
    {
        const int rc = encode(argv[1], w, h, n, argv[5 + k], preset);
        if (rc)
        {
            fprintf(stderr, "[twice] encode %d failed (%d)\n", k, rc);
            return rc;
        }
        fprintf(stderr, "[twice] encode %d done\n", k);
    }
    return 0;
}
