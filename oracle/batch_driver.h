/* ORACLE -- TEST INFRASTRUCTURE ONLY.  Batch drivers over a per-string codec, instantiated for the
 * clean-room restatement (huff_oracle.c) and for the compiled reference (ref_shim.c).  The array
 * contract is the one declared for the HIP path in include/hhuff.h:
 *   string i = in[in_off[i] .. in_off[i] + len_i), len_i = in_len ? in_len[i] : in_off[i+1] - in_off[i]
 *   decode destination: out + (out_off ? out_off[i] : floor(8 * in_off[i] / 5))
 *   encode destination: out + (out_off ? out_off[i] : in_off[i])
 *   flatten destination: out + (out_off ? out_off[i] : in_off[i] + 11 * i)
 * Work is split into `nthreads` contiguous string ranges (pthreads).
 *
 * Instantiate with ORC_CODEC_DECODE / ORC_CODEC_ENCODE / ORC_CODEC_FLATTEN / ORC_BATCH_PREFIX. */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

#define ORC_CAT2(a, b) a##_##b
#define ORC_CAT(a, b) ORC_CAT2(a, b)
#define ORC_FN(name) ORC_CAT(ORC_BATCH_PREFIX, name)
#ifndef ORC_BATCH_API
#define ORC_BATCH_API
#endif

typedef struct {
    const uint8_t *in;
    const uint32_t *in_off, *in_len, *is_name_bits, *out_off, *raw_bits, *lit_end;
    uint32_t *pay_off, *consumed;
    unsigned flags;
    const uint8_t *first_bytes;
    unsigned prefix_bits;
    uint8_t *out;
    uint32_t *out_len;
    uint8_t *status;
    uint32_t begin, end;
} ORC_FN(job_t);

static inline uint32_t ORC_FN(len_of)(const ORC_FN(job_t) * j, uint32_t i)
{
    return j->in_len ? j->in_len[i] : j->in_off[i + 1] - j->in_off[i];
}

static void *ORC_FN(decode_worker)(void *arg)
{
    ORC_FN(job_t) *j = (ORC_FN(job_t) *)arg;
    for (uint32_t i = j->begin; i < j->end; ++i) {
        uint32_t len = ORC_FN(len_of)(j, i);
        uint64_t dst = j->out_off ? j->out_off[i] : ((uint64_t)j->in_off[i] * 8u) / 5u;
        int is_name = j->is_name_bits ? (int)((j->is_name_bits[i >> 5] >> (i & 31)) & 1u) : 0;
        unsigned soft = 0;
        size_t r = ORC_CODEC_DECODE((char *)j->out + dst, &soft, j->in + j->in_off[i], len, is_name);
        if (r == SIZE_MAX) {
            j->out_len[i] = 0xFFFFFFFFu;
            if (j->status)
                j->status[i] = 0x80u;
        } else {
            j->out_len[i] = (uint32_t)r;
            if (j->status)
                j->status[i] = (uint8_t)soft;
        }
    }
    return NULL;
}

static void *ORC_FN(encode_worker)(void *arg)
{
    ORC_FN(job_t) *j = (ORC_FN(job_t) *)arg;
    for (uint32_t i = j->begin; i < j->end; ++i) {
        uint32_t len = ORC_FN(len_of)(j, i);
        uint64_t dst = j->out_off ? j->out_off[i] : j->in_off[i];
        size_t r = ORC_CODEC_ENCODE(j->out + dst, j->in + j->in_off[i], len);
        j->out_len[i] = r == SIZE_MAX ? 0xFFFFFFFFu : (uint32_t)r;
        if (j->status)
            j->status[i] = r == SIZE_MAX ? 0x80u : 0u;
    }
    return NULL;
}

static void *ORC_FN(flatten_worker)(void *arg)
{
    ORC_FN(job_t) *j = (ORC_FN(job_t) *)arg;
    for (uint32_t i = j->begin; i < j->end; ++i) {
        uint32_t len = ORC_FN(len_of)(j, i);
        uint64_t dst = j->out_off ? j->out_off[i] : (uint64_t)j->in_off[i] + 11u * (uint64_t)i;
        int raw = j->raw_bits ? (int)((j->raw_bits[i >> 5] >> (i & 31)) & 1u) : 0;
        j->out[dst] = j->first_bytes ? j->first_bytes[i] : 0;
        j->out_len[i] = (uint32_t)ORC_CODEC_FLATTEN(j->out + dst, j->in + j->in_off[i], len, j->prefix_bits, raw);
    }
    return NULL;
}

#ifdef ORC_CODEC_LITERAL
/* literal i starts at in[in_off[i]] and may extend to in[lit_end[i]]; decoded bytes at
 * out + floor(8 * pay_off[i] / 5); status = soft bits | 0x80 | verdict << 2 on failure */
static void *ORC_FN(literal_worker)(void *arg)
{
    ORC_FN(job_t) *j = (ORC_FN(job_t) *)arg;
    for (uint32_t i = j->begin; i < j->end; ++i) {
        int is_name = j->is_name_bits ? (int)((j->is_name_bits[i >> 5] >> (i & 31)) & 1u) : 0;
        unsigned soft = 0;
        uint32_t hdr, consumed, olen;
        int code = ORC_CODEC_LITERAL(j->in + j->in_off[i], j->in + j->lit_end[i], j->prefix_bits, is_name,
                                     (int)(j->flags & 1u), j->out, j->in_off[i], &hdr, &consumed, &olen, &soft);
        j->out_len[i] = code ? 0xFFFFFFFFu : olen;
        j->pay_off[i] = j->in_off[i] + hdr;
        j->consumed[i] = code ? 0u : consumed;
        j->status[i] = (uint8_t)(soft | (code ? 0x80u | ((unsigned)code << 2) : 0u));
    }
    return NULL;
}
#endif

static int ORC_FN(run)(void *(*fn)(void *), const ORC_FN(job_t) * proto, uint32_t n, int nthreads)
{
    if (nthreads < 1)
        nthreads = 1;
    if ((uint32_t)nthreads > n)
        nthreads = n ? (int)n : 1;
    ORC_FN(job_t) *jobs = (ORC_FN(job_t) *)calloc((size_t)nthreads, sizeof(*jobs));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(*th));
    if (!jobs || !th) {
        free(jobs);
        free(th);
        return -1;
    }
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = *proto;
        jobs[t].begin = (uint32_t)(((uint64_t)n * t) / nthreads);
        jobs[t].end = (uint32_t)(((uint64_t)n * (t + 1)) / nthreads);
    }
    int rc = 0;
    for (int t = 1; t < nthreads; ++t)
        if (pthread_create(&th[t], NULL, fn, &jobs[t]) != 0)
            rc = -1;
    fn(&jobs[0]);
    for (int t = 1; t < nthreads; ++t)
        pthread_join(th[t], NULL);
    free(jobs);
    free(th);
    return rc;
}

ORC_BATCH_API int ORC_FN(decode_batch)(const uint8_t *in, const uint32_t *in_off, const uint32_t *in_len, uint32_t n,
                         const uint32_t *is_name_bits, uint8_t *out, const uint32_t *out_off, uint32_t *out_len,
                         uint8_t *status, int nthreads)
{
    ORC_FN(job_t) p = {0};
    p.in = in, p.in_off = in_off, p.in_len = in_len, p.is_name_bits = is_name_bits;
    p.out = out, p.out_off = out_off, p.out_len = out_len, p.status = status;
    return ORC_FN(run)(ORC_FN(decode_worker), &p, n, nthreads);
}

ORC_BATCH_API int ORC_FN(encode_batch)(const uint8_t *in, const uint32_t *in_off, const uint32_t *in_len, uint32_t n, uint8_t *out,
                         const uint32_t *out_off, uint32_t *out_len, uint8_t *status, int nthreads)
{
    ORC_FN(job_t) p = {0};
    p.in = in, p.in_off = in_off, p.in_len = in_len;
    p.out = out, p.out_off = out_off, p.out_len = out_len, p.status = status;
    return ORC_FN(run)(ORC_FN(encode_worker), &p, n, nthreads);
}

ORC_BATCH_API int ORC_FN(flatten_batch)(const uint8_t *in, const uint32_t *in_off, const uint32_t *in_len, uint32_t n,
                          const uint8_t *first_bytes, unsigned prefix_bits, const uint32_t *raw_bits, uint8_t *out,
                          const uint32_t *out_off, uint32_t *out_len, int nthreads)
{
    ORC_FN(job_t) p = {0};
    p.in = in, p.in_off = in_off, p.in_len = in_len, p.first_bytes = first_bytes, p.prefix_bits = prefix_bits;
    p.raw_bits = raw_bits, p.out = out, p.out_off = out_off, p.out_len = out_len;
    return ORC_FN(run)(ORC_FN(flatten_worker), &p, n, nthreads);
}

#ifdef ORC_CODEC_LITERAL
ORC_BATCH_API int ORC_FN(literals_batch)(const uint8_t *in, const uint32_t *lit_off, const uint32_t *lit_end, uint32_t n,
                                         unsigned prefix_bits, unsigned flags, const uint32_t *is_name_bits, uint8_t *out,
                                         uint32_t *out_len, uint32_t *pay_off, uint32_t *consumed, uint8_t *status,
                                         int nthreads)
{
    ORC_FN(job_t) p = {0};
    p.in = in, p.in_off = lit_off, p.lit_end = lit_end, p.prefix_bits = prefix_bits, p.flags = flags;
    p.is_name_bits = is_name_bits, p.out = out, p.out_len = out_len, p.pay_off = pay_off, p.consumed = consumed;
    p.status = status;
    return ORC_FN(run)(ORC_FN(literal_worker), &p, n, nthreads);
}
#endif
