/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Header-block harness around the REAL reference decoder, compiled
 * from the sources where they lie (oracle/Makefile; nothing is copied):
 *   lib/http2/hpack.c   h2o_hpack_decode_header :319-435 (dynamic table :263-317)
 *   lib/common/memory.c the h2o_mem_pool_t / shared-buffer allocator it decodes into
 *   lib/common/token.c  h2o_lookup_token, h2o_hpack_static_table
 * ref_hpack_decode_blocks loops h2o_hpack_decode_header over every block the way
 * h2o_hpack_parse_request does (hpack.c:513-527), one h2o_hpack_header_table_t per connection with
 * hpack_capacity = hpack_max_capacity = table_size (as lib/http2/connection.c:1844 sets it), and copies
 * each decoded name and value into the caller's arena -- the output contract of
 * include/hhuff.h hhuff_hpack_decode_blocks.  It never runs on the GPU box.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "h2o/hpack.h"
#include "h2o/http2_common.h"
#include "h2o/memory.h"

#define REF_API __attribute__((visibility("default")))
#define REF_BLK_ARENA (-300)
#define REF_BLK_SKIPPED (-301)

REF_API int ref_hpack_decode_blocks(const uint8_t *in, const uint32_t *blk_off, const uint32_t *conn_first, uint32_t nconn,
                                    uint32_t table_size, uint8_t *arena, const uint64_t *arena_off, uint32_t *name_off,
                                    uint32_t *name_len, uint32_t *value_off, uint32_t *value_len, uint8_t *fflags,
                                    uint32_t *nfields, int32_t *bstatus, int nthreads)
{
    (void)nthreads;
    for (uint32_t c = 0; c < nconn; ++c) {
        h2o_hpack_header_table_t table;
        memset(&table, 0, sizeof(table));
        table.hpack_capacity = table.hpack_max_capacity = table_size;
        int failed = 0;
        for (uint32_t b = conn_first[c]; b < conn_first[c + 1]; ++b) {
            nfields[b] = 0;
            if (failed) {
                bstatus[b] = REF_BLK_SKIPPED;
                continue;
            }
            h2o_mem_pool_t pool;
            h2o_mem_init_pool(&pool);
            const uint8_t *src = in + blk_off[b], *end = in + blk_off[b + 1];
            uint64_t cur = arena_off[b], aend = arena_off[b + 1] < (1ull << 32) ? arena_off[b + 1] : (1ull << 32);
            uint32_t nf = 0, slot = blk_off[b];
            int st = 0;
            while (src != end) {
                h2o_iovec_t *name, value;
                const char *err_desc = NULL;
                int ret = h2o_hpack_decode_header(&pool, &table, &name, &value, &src, end, &err_desc);
                if (ret != 0 && ret != H2O_HTTP2_ERROR_INVALID_HEADER_CHAR) {
                    st = ret;
                    break;
                }
                if (cur + name->len + value.len > aend) {
                    st = REF_BLK_ARENA;
                    break;
                }
                memcpy(arena + cur, name->base, name->len);
                name_off[slot + nf] = (uint32_t)cur;
                name_len[slot + nf] = (uint32_t)name->len;
                cur += name->len;
                memcpy(arena + cur, value.base, value.len);
                value_off[slot + nf] = (uint32_t)cur;
                value_len[slot + nf] = (uint32_t)value.len;
                cur += value.len;
                /* the field's soft errors are what decode_header reports as INVALID_HEADER_CHAR
                 * (hpack.c:427-431); which bit is recovered from err_desc */
                fflags[slot + nf] = ret == 0 ? 0 : (err_desc == h2o_hpack_soft_err_found_invalid_char_in_header_name ? 1 : 2);
                ++nf;
            }
            h2o_mem_clear_pool(&pool);
            nfields[b] = nf;
            bstatus[b] = st;
            failed = st != 0;
        }
        h2o_hpack_dispose_header_table(&table);
    }
    return 0;
}
