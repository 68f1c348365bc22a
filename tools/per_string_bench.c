/* C-level latency of h2o's per-string symbols through libhhuff.so (as h2o calls them), and the resident
 * service's own stamps: cc -O2 tools/per_string_bench.c -Iinclude -Lh2o_amd -lhhuff -Wl,-rpath,$PWD/h2o_amd */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "hhuff.h"

static double now_us(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static int cmp(const void *a, const void *b)
{
    double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

#define N 4000
int main(void)
{
    const char *s = "accept-encoding: gzip, deflate, br, zstd, accept-";
    size_t len = 48;
    uint8_t h[64], d[128];
    size_t hl = h2o_hpack_encode_huffman(h, (const uint8_t *)s, len);
    if (hl == SIZE_MAX) {
        printf("{\"error\": \"%s\"}\n", hhuff_last_error_string());
        return 1;
    }
    static double te[N], td[N], st[4][N];
    for (int i = 0; i < 200; ++i)
        h2o_hpack_encode_huffman(h, (const uint8_t *)s, len);
    for (int i = 0; i < N; ++i) {
        double t0 = now_us();
        h2o_hpack_encode_huffman(h, (const uint8_t *)s, len);
        te[i] = now_us() - t0;
    }
    for (int i = 0; i < N; ++i) {
        unsigned soft = 0;
        const char *err = NULL;
        double t0 = now_us();
        size_t r = h2o_hpack_decode_huffman((char *)d, &soft, h, hl, 0, &err);
        td[i] = now_us() - t0;
        if (r != len || memcmp(d, s, len) != 0) {
            printf("{\"error\": \"decode mismatch\"}\n");
            return 1;
        }
        uint32_t t4[4];
        if (hhuff_service_stamps(t4) == 0) {
            st[0][i] = (t4[1] - t4[0]) * 0.01, st[1][i] = (t4[2] - t4[1]) * 0.01, st[2][i] = (t4[3] - t4[2]) * 0.01;
        }
    }
    qsort(te, N, sizeof(double), cmp);
    qsort(td, N, sizeof(double), cmp);
    for (int k = 0; k < 3; ++k)
        qsort(st[k], N, sizeof(double), cmp);
    printf("{\"encode_us\": {\"median\": %.2f, \"p99\": %.2f}, \"decode_us\": {\"median\": %.2f, \"p99\": %.2f}, "
           "\"service_decode_us\": {\"seen_to_input\": %.2f, \"input_to_coded\": %.2f, \"coded_to_written\": %.2f}}\n",
           te[N / 2], te[N * 99 / 100], td[N / 2], td[N * 99 / 100], st[0][N / 2], st[1][N / 2], st[2][N / 2]);
    return 0;
}
