/*
 * The C ABI from a C translation unit (include/hhuff.h, linked against h2o_amd/libhhuff.so):
 *   1. h2o's per-string symbols from 8 threads at once, each checking known answers (the reference's own
 *      unit-test vectors, t/00unit/lib/http2/hpack.c:175-186, 299-306, and SURVEY Appendix A);
 *   2. a device batch call on the legacy default stream (stream NULL);
 *   3. the host batch API on device 0, with the caller's current device left as it was.
 * Built by tests/test_capi.py (gcc); run there with a GPU (exit 0 = every check held), or with `nogpu`
 * where there is none: the per-string symbols must then fail soft (SIZE_MAX, an error string, no abort).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "hhuff.h"

static const uint8_t kat_huff[] = {0xf1, 0xe3, 0xc2, 0xe5, 0xf2, 0x3a, 0x6b, 0xa0, 0xab, 0x90, 0xf4, 0xff};
static const char kat_plain[] = "www.example.com";

static int check_one(void)
{
    char dst[64];
    unsigned soft = 0;
    size_t r = h2o_hpack_decode_huffman(dst, &soft, kat_huff, sizeof(kat_huff), 0, NULL);
    if (r != 15 || memcmp(dst, kat_plain, 15) != 0 || soft != 0)
        return 1;
    uint8_t enc[64];
    r = h2o_hpack_encode_huffman(enc, (const uint8_t *)kat_plain, 15);
    if (r != sizeof(kat_huff) || memcmp(enc, kat_huff, r) != 0)
        return 2;
    if (h2o_hpack_encode_huffman(enc, (const uint8_t *)"XXXX", 4) != SIZE_MAX) /* 'X' is 8 bits: never shorter */
        return 3;
    soft = 2; /* OR semantics: a preset word survives, nothing is added for a valid value */
    r = h2o_hpack_decode_huffman(dst, &soft, (const uint8_t *)"\x1f", 1, 0, NULL);
    if (r != 1 || dst[0] != 'a' || soft != 2)
        return 4;
    soft = 0; /* an empty name is a soft error */
    if (h2o_hpack_decode_huffman(dst, &soft, (const uint8_t *)"", 0, 1, NULL) != 0 || soft != 1)
        return 5;
    if (h2o_hpack_decode_huffman(dst, &soft, (const uint8_t *)"\xff\xff\xff\xff", 4, 0, NULL) != SIZE_MAX)
        return 6; /* EOS */
    return 0;
}

static void *worker(void *arg)
{
    intptr_t bad = 0;
    for (int i = 0; i < 300 && !bad; ++i)
        bad = check_one();
    (void)arg;
    return (void *)bad;
}

int main(int argc, char **argv)
{
    if (argc > 1 && strcmp(argv[1], "nogpu") == 0) {
        char dst[64];
        unsigned soft = 0;
        size_t r = h2o_hpack_decode_huffman(dst, &soft, kat_huff, sizeof(kat_huff), 0, NULL);
        uint8_t enc[64];
        size_t e = h2o_hpack_encode_huffman(enc, (const uint8_t *)kat_plain, 15);
        const char *why = hhuff_last_error_string();
        printf("decode=%zu encode=%zu soft=%u err=%s\n", r, e, soft, why);
        return (r == SIZE_MAX && e == SIZE_MAX && soft == 0 && why[0] != '\0') ? 0 : 10;
    }
    /* 1. concurrent per-string calls */
    pthread_t th[8];
    for (int t = 0; t < 8; ++t)
        pthread_create(&th[t], NULL, worker, NULL);
    int fail = 0;
    for (int t = 0; t < 8; ++t) {
        void *rv;
        pthread_join(th[t], &rv);
        if (rv != NULL) {
            fprintf(stderr, "thread %d: check %ld failed\n", t, (long)(intptr_t)rv);
            fail = 20;
        }
    }
    /* 2. device batch on the NULL stream: two strings, contiguous layout */
    uint8_t h_in[32];
    memcpy(h_in, kat_huff, 12);
    memcpy(h_in + 12, "\x1f", 1);
    uint32_t h_off[3] = {0, 12, 13};
    uint8_t *d_in, *d_out, *d_st;
    uint32_t *d_off, *d_len;
    if (hipMalloc((void **)&d_in, 32) || hipMalloc((void **)&d_out, 64) || hipMalloc((void **)&d_off, 12) ||
        hipMalloc((void **)&d_len, 8) || hipMalloc((void **)&d_st, 2))
        return 30;
    hipMemcpy(d_in, h_in, 32, hipMemcpyHostToDevice);
    hipMemcpy(d_off, h_off, 12, hipMemcpyHostToDevice);
    if (hhuff_decode_batch(d_in, 13, d_off, NULL, 2, NULL, d_out, NULL, d_len, d_st, NULL) != HHUFF_OK)
        return 31;
    uint8_t out[64];
    uint32_t len[2];
    hipDeviceSynchronize();
    hipMemcpy(out, d_out, 64, hipMemcpyDeviceToHost);
    hipMemcpy(len, d_len, 8, hipMemcpyDeviceToHost);
    /* implicit slots: floor(8 * in_off / 5) */
    if (len[0] != 15 || memcmp(out, kat_plain, 15) != 0 || len[1] != 1 || out[(12 * 8) / 5] != 'a')
        fail = 32;
    /* 3. host batch API on device 0; the caller's current device is unchanged afterwards */
    int before = -1, after = -1;
    hipGetDevice(&before);
    uint8_t o2[64];
    uint32_t l2[2];
    uint8_t s2[2];
    if (hhuff_decode_batch_host(h_in, 13, h_off, NULL, 2, NULL, o2, sizeof(o2), NULL, l2, s2, 0) != HHUFF_OK)
        return 33;
    hipGetDevice(&after);
    if (l2[0] != 15 || memcmp(o2, kat_plain, 15) != 0 || after != before)
        fail = 34;
    printf("capi_check: %s (%s)\n", fail ? "FAILED" : "ok", hhuff_version());
    return fail;
}
