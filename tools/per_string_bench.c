/* C-level latency and throughput of h2o's per-string symbols through libhhuff.so, called the way h2o calls them:
 * concurrently from every event-loop thread (src/main.c:5512 starts one per core).  For each thread count T given
 * on the command line (default 1 8 16 64) T pthreads each make N encode calls, then N decode calls, of one 48-B
 * header string; the line reports the aggregate strings/s (all threads' calls over the wall time of the phase)
 * and the per-call median / p99 over all calls.  The T = 1 line also carries the resident service's own stamps.
 *   cc -O2 -pthread tools/per_string_bench.c -Iinclude -Lh2o_amd -lhhuff -Wl,-rpath,$PWD/h2o_amd -o tools/per_string_bench
 */
#include <pthread.h>
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

static const char *S = "accept-encoding: gzip, deflate, br, zstd, accept-";
enum { LEN = 48, WARM = 200 };
static uint8_t H[64];
static size_t HL;
static int N = 2000;

struct job {
    int encode;
    double *lat;
    int bad;
    pthread_barrier_t *bar;
};

static void *run(void *p)
{
    struct job *j = p;
    uint8_t h[64];
    char d[128];
    for (int i = 0; i < WARM + N; ++i) {
        if (i == WARM)
            pthread_barrier_wait(j->bar);
        double t0 = now_us();
        if (j->encode) {
            size_t r = h2o_hpack_encode_huffman(h, (const uint8_t *)S, LEN);
            if (r != HL || memcmp(h, H, HL) != 0)
                j->bad = 1;
        } else {
            unsigned soft = 0;
            const char *err = NULL;
            size_t r = h2o_hpack_decode_huffman(d, &soft, H, HL, 0, &err);
            if (r != LEN || memcmp(d, S, LEN) != 0)
                j->bad = 1;
        }
        if (i >= WARM)
            j->lat[i - WARM] = now_us() - t0;
    }
    pthread_barrier_wait(j->bar);
    return NULL;
}

/* one phase: T threads x N calls; returns strings/s, fills median / p99 (us) */
static double phase(int T, int encode, double *med, double *p99, int *bad)
{
    pthread_t *th = calloc(T, sizeof(*th));
    struct job *jb = calloc(T, sizeof(*jb));
    double *lat = calloc((size_t)T * N, sizeof(double));
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, T + 1);
    for (int t = 0; t < T; ++t) {
        jb[t] = (struct job){encode, lat + (size_t)t * N, 0, &bar};
        pthread_create(&th[t], NULL, run, &jb[t]);
    }
    pthread_barrier_wait(&bar); /* every thread warmed up */
    double t0 = now_us();
    pthread_barrier_wait(&bar); /* every thread done */
    double wall = now_us() - t0;
    for (int t = 0; t < T; ++t) {
        pthread_join(th[t], NULL);
        *bad |= jb[t].bad;
    }
    qsort(lat, (size_t)T * N, sizeof(double), cmp);
    *med = lat[(size_t)T * N / 2];
    *p99 = lat[(size_t)T * N * 99 / 100];
    pthread_barrier_destroy(&bar);
    free(lat), free(jb), free(th);
    return (double)T * N / (wall * 1e-6);
}

int main(int argc, char **argv)
{
    HL = h2o_hpack_encode_huffman(H, (const uint8_t *)S, LEN);
    if (HL == SIZE_MAX) {
        printf("{\"error\": \"%s\"}\n", hhuff_last_error_string());
        return 1;
    }
    if (getenv("PS_CALLS"))
        N = atoi(getenv("PS_CALLS"));
    int counts[16] = {1, 8, 16, 64}, nc = 4;
    if (argc > 1) {
        nc = 0;
        for (int a = 1; a < argc && nc < 16; ++a)
            counts[nc++] = atoi(argv[a]);
    }
    for (int c = 0; c < nc; ++c) {
        const int T = counts[c];
        double em, e99, dm, d99;
        int bad = 0;
        double er = phase(T, 1, &em, &e99, &bad);
        double dr = phase(T, 0, &dm, &d99, &bad);
        if (bad) {
            printf("{\"threads\": %d, \"error\": \"result mismatch: %s\"}\n", T, hhuff_last_error_string());
            return 1;
        }
        printf("{\"threads\": %d, \"calls_per_thread\": %d, \"string_bytes\": %d, "
               "\"encode\": {\"strings_per_s\": %.0f, \"median_us\": %.2f, \"p99_us\": %.2f}, "
               "\"decode\": {\"strings_per_s\": %.0f, \"median_us\": %.2f, \"p99_us\": %.2f}",
               T, N, LEN, er, em, e99, dr, dm, d99);
        if (T == 1) {
            /* the service wave's stamps of one more decode: poll -> input, input -> coded, coded -> written */
            unsigned soft = 0;
            const char *err = NULL;
            char d[128];
            uint32_t t4[4];
            h2o_hpack_decode_huffman(d, &soft, H, HL, 0, &err);
            if (hhuff_service_stamps(t4) == 0)
                printf(", \"service_decode_us\": {\"seen_to_input\": %.2f, \"input_to_coded\": %.2f, "
                       "\"coded_to_written\": %.2f}",
                       (t4[1] - t4[0]) * 0.01, (t4[2] - t4[1]) * 0.01, (t4[3] - t4[2]) * 0.01);
        }
        printf("}\n");
        fflush(stdout);
    }
    return 0;
}
