/*
 * The C ABI from a C translation unit (include/hhuff.h, linked against h2o_amd/libhhuff.so):
 *   1. h2o's per-string symbols from 8 threads at once, each checking known answers (the reference's own
 *      unit-test vectors, t/00unit/lib/http2/hpack.c:175-186, 299-306, and SURVEY Appendix A);
 *   2. a device batch call on the legacy default stream (stream NULL);
 *   3. the host batch API on device 0, with the caller's current device left as it was;
 *   4. the multi-device batch (device and host arrays, one and two shards) against the one-device call.
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

/* a seeded batch of header-like strings (lengths 0..160, 1 in 50 all 'X': never compressible) */
static uint32_t rng_state = 12345;
static uint32_t rnd(void)
{
    rng_state = rng_state * 1664525u + 1013904223u;
    return rng_state >> 8;
}

static int same_slots(const uint8_t *a, const uint8_t *b, const uint32_t *off, const uint32_t *len, uint32_t n,
                      int decode)
{
    for (uint32_t i = 0; i < n; ++i) {
        if (len[i] == HHUFF_FAIL_LEN)
            continue;
        uint64_t o = decode ? ((uint64_t)off[i] * 8) / 5 : off[i];
        if (memcmp(a + o, b + o, len[i]) != 0)
            return 0;
    }
    return 1;
}

/* one layout both ways: device arrays on device 0 (devices {0}, {0, 0}) and host arrays (devices {0}, {0, 0}) */
static int multi_round(int decode, const uint8_t *h_in, uint64_t size, const uint32_t *h_off, uint32_t n,
                       const uint32_t *h_names, uint8_t *ref_out, uint32_t *ref_len, uint8_t *ref_st)
{
    const uint64_t osz = (decode ? (size * 8) / 5 : size) + 16;
    const size_t nw = (n + 31) / 32;
    uint8_t *d_in, *d_out, *d_st;
    uint32_t *d_off, *d_len, *d_nm;
    if (hipMalloc((void **)&d_in, size + 16) || hipMalloc((void **)&d_out, osz) ||
        hipMalloc((void **)&d_off, 4 * ((size_t)n + 1)) || hipMalloc((void **)&d_len, 4 * (size_t)n) ||
        hipMalloc((void **)&d_st, n) || hipMalloc((void **)&d_nm, 4 * nw))
        return 40;
    hipMemcpy(d_in, h_in, size, hipMemcpyHostToDevice);
    hipMemcpy(d_off, h_off, 4 * ((size_t)n + 1), hipMemcpyHostToDevice);
    hipMemcpy(d_nm, h_names, 4 * nw, hipMemcpyHostToDevice);
    /* the one-device call */
    int rc = decode ? hhuff_decode_batch(d_in, size, d_off, NULL, n, d_nm, d_out, NULL, d_len, d_st, NULL)
                    : hhuff_encode_batch(d_in, size, d_off, NULL, n, d_out, NULL, d_len, d_st, NULL);
    if (rc)
        return 41;
    hipDeviceSynchronize();
    hipMemcpy(ref_out, d_out, osz, hipMemcpyDeviceToHost);
    hipMemcpy(ref_len, d_len, 4 * (size_t)n, hipMemcpyDeviceToHost);
    hipMemcpy(ref_st, d_st, n, hipMemcpyDeviceToHost);
    uint8_t *o = malloc(osz), *st = malloc(n);
    uint32_t *ln = malloc(4 * (size_t)n);
    static const int devs[2] = {0, 0};
    int fail = 0;
    for (int mode = 0; mode < 4 && !fail; ++mode) {
        const int ndev = 1 + (mode & 1), host = mode >= 2;
        memset(o, 0, osz), memset(ln, 0xEE, 4 * (size_t)n), memset(st, 0xEE, n);
        if (host) {
            rc = decode ? hhuff_decode_batch_multi(ndev, devs, HHUFF_HOST_MEMORY, h_in, size, h_off, n, h_names, o, osz, ln,
                                                   st, NULL)
                        : hhuff_encode_batch_multi(ndev, devs, HHUFF_HOST_MEMORY, h_in, size, h_off, n, o, osz, ln, st, NULL);
        } else {
            hipMemset(d_out, 0, osz), hipMemset(d_len, 0xEE, 4 * (size_t)n), hipMemset(d_st, 0xEE, n);
            rc = decode ? hhuff_decode_batch_multi(ndev, devs, 0, d_in, size, d_off, n, d_nm, d_out, osz, d_len, d_st, NULL)
                        : hhuff_encode_batch_multi(ndev, devs, 0, d_in, size, d_off, n, d_out, osz, d_len, d_st, NULL);
            hipDeviceSynchronize();
            hipMemcpy(o, d_out, osz, hipMemcpyDeviceToHost);
            hipMemcpy(ln, d_len, 4 * (size_t)n, hipMemcpyDeviceToHost);
            hipMemcpy(st, d_st, n, hipMemcpyDeviceToHost);
        }
        if (rc) {
            fprintf(stderr, "multi mode %d: rc %d (%s)\n", mode, rc, hhuff_last_error_string());
            fail = 42;
        } else if (memcmp(ln, ref_len, 4 * (size_t)n) != 0 || memcmp(st, ref_st, n) != 0 ||
                   !same_slots(o, ref_out, h_off, ref_len, n, decode)) {
            fprintf(stderr, "multi mode %d (%s): results differ from the one-device call\n", mode,
                    decode ? "decode" : "encode");
            fail = 43;
        }
    }
    free(o), free(st), free(ln);
    hipFree(d_in), hipFree(d_out), hipFree(d_off), hipFree(d_len), hipFree(d_st), hipFree(d_nm);
    return fail;
}

static int check_multi(void)
{
    static const char alpha[] = "abcdefghijklmnopqrstuvwxyz0123456789-_./:=;, ABCDEFGHIJKLMNOPQRSTUVWXYZ";
    const uint32_t n = 20000;
    uint32_t *off = malloc(4 * ((size_t)n + 1)), *names = calloc((n + 31) / 32, 4);
    uint8_t *plain = malloc((size_t)n * 161 + 16);
    off[0] = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t L = rnd() % 161, allx = rnd() % 50 == 0;
        for (uint32_t j = 0; j < L; ++j)
            plain[off[i] + j] = allx ? 'X' : (uint8_t)alpha[rnd() % (sizeof(alpha) - 1)];
        off[i + 1] = off[i] + L;
        if (rnd() % 4 == 0)
            names[i / 32] |= 1u << (i % 32);
    }
    const uint64_t P = off[n];
    uint8_t *enc = malloc(P + 16), *est = malloc(n);
    uint32_t *elen = malloc(4 * (size_t)n);
    int fail = multi_round(0, plain, P, off, n, names, enc, elen, est);
    /* the wire: the compressible strings' Huffman bytes back to back, decoded the same ways */
    uint32_t m = 0;
    uint32_t *hoff = malloc(4 * ((size_t)n + 1)), *hnames = calloc((n + 31) / 32, 4);
    uint8_t *huff = malloc(P + 16);
    hoff[0] = 0;
    for (uint32_t i = 0; i < n && !fail; ++i) {
        if (elen[i] == HHUFF_FAIL_LEN)
            continue;
        memcpy(huff + hoff[m], enc + off[i], elen[i]);
        if (names[i / 32] >> (i % 32) & 1)
            hnames[m / 32] |= 1u << (m % 32);
        hoff[m + 1] = hoff[m] + elen[i];
        ++m;
    }
    if (!fail && m < n / 2)
        fail = 44;
    if (!fail) {
        const uint64_t H = hoff[m];
        uint8_t *dec = malloc((H * 8) / 5 + 16), *dst = malloc(m);
        uint32_t *dlen = malloc(4 * (size_t)m);
        fail = multi_round(1, huff, H, hoff, m, hnames, dec, dlen, dst);
        /* and the decode inverts the encode */
        for (uint32_t i = 0, k = 0; i < n && !fail; ++i) {
            if (elen[i] == HHUFF_FAIL_LEN)
                continue;
            if (dlen[k] != off[i + 1] - off[i] || memcmp(dec + ((uint64_t)hoff[k] * 8) / 5, plain + off[i], dlen[k]) != 0)
                fail = 45;
            ++k;
        }
        uint32_t b[9], b2[9];
        if (!fail && (hhuff_shard_bounds(hoff, m, 8, 64, b) != HHUFF_OK || b[0] != 0 || b[8] != m))
            fail = 46;
        for (int k = 1; k < 8 && !fail; ++k)
            if (b[k] % 64 != 0 || b[k] < b[k - 1])
                fail = 47;
        if (!fail && (hhuff_shard_bounds(hoff, m, 8, 1, b2) != HHUFF_OK))
            fail = 48;
        free(dec), free(dst), free(dlen);
    }
    free(off), free(names), free(plain), free(enc), free(est), free(elen), free(hoff), free(hnames), free(huff);
    return fail;
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
    /* 4. the multi-device batch (hhuff_{en,de}code_batch_multi) against the one-device call, byte for byte */
    if (!fail)
        fail = check_multi();
    printf("capi_check: %s (%s)\n", fail ? "FAILED" : "ok", hhuff_version());
    return fail;
}
