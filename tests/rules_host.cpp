// The GPU request / response rules (h2o_amd/csrc/hhuff_request.h, the source the HPACK walk and the QPACK
// sections kernel inline) compiled for the HOST under AddressSanitizer and UndefinedBehaviorSanitizer, run
// against the oracle's restatement of h2o_hpack_parse_request / h2o_hpack_parse_response's rules
// (oracle/hpack_block.c orc_rq_field / orc_rs_field, pinned to the real functions by the f4 fixtures) on
// random field sequences, with both the HTTP/2 and the HTTP/3 arguments.  Every return code, every field's
// header bit and the final records must agree, and the sanitizers must stay silent: an uninitialised read,
// an out-of-bounds access or other UB in the rules would show here (tests/test_rules_host.py builds and runs
// it; the ORACLE objects are test infrastructure).
#include <hip/hip_runtime.h>
#ifndef __device__
#define __device__
#endif
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

#include "hhuff_request.h"

extern "C" {
#include "orc_request.h"
}

static const char* kNames[] = {":authority", ":method", ":path", ":protocol", ":scheme", ":status", ":foo", ":",
                               "content-length", "expect", "host", "te", "cache-digest", "datagram-flow-id",
                               "connection", "http2-settings", "transfer-encoding", "upgrade", "x-regular", "accept",
                               "cookie", "Te", "", "hosts", "tee", ":pat"};
static const char* kValues[] = {"", "trailers", "TRAILERS", "Trailers ", "gzip", "0", "123", "12a", "https", "masque",
                                "http", "200", "099", "20x", "404", "999", "1000", "99999999999999999999",
                                "1234567890123456789", "/", "/index.html", "100-continue", "websocket", "-1"};

int main(int argc, char** argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 20000;
    std::mt19937_64 rng(12345);
    auto pick = [&](size_t n) { return (size_t)(rng() % n); };
    long fields = 0, errs = 0;
    for (int t = 0; t < trials; ++t) {
        const bool h3 = (t & 1) != 0, resp = (t & 2) != 0, trailers = resp && (t & 4) != 0;
        // a few long sequences reach the 100-header and 1000-field limits
        const int nf = (t % 97 == 0) ? 1002 : (t % 13 == 0) ? 110 : 1 + (int)pick(12);
        hhuff::ReqState rq;
        hhuff::RespState rs;
        orc_req_t orq;
        orc_resp_t ors;
        rq.reset();
        rs.reset(trailers);
        orc_rq_init(&orq);
        orc_rs_init(&ors, trailers ? 1 : 0);
        // response heads usually start with a valid :status, requests with their pseudo-headers
        std::vector<std::pair<std::string, std::string>> seq;
        if (resp && !trailers && pick(4) != 0) seq.push_back({":status", "200"});
        if (!resp && pick(3) != 0) {
            seq.push_back({":method", "GET"});
            seq.push_back({":scheme", pick(2) ? "https" : "masque"});
            seq.push_back({":path", "/"});
        }
        while ((int)seq.size() < nf) {
            const char* n = pick(3) == 0 ? "x-regular" : kNames[pick(sizeof(kNames) / sizeof(kNames[0]))];
            seq.push_back({n, kValues[pick(sizeof(kValues) / sizeof(kValues[0]))]});
        }
        for (size_t k = 0; k < seq.size(); ++k) {
            const std::string& n = seq[k].first;
            const std::string& v = seq[k].second;
            const uint32_t soft = pick(8) == 0 ? 1u + (uint32_t)pick(2) : 0u;
            // the value is copied to its own allocation so ASan sees reads past its end
            std::vector<uint8_t> nb(n.begin(), n.end()), vb(v.begin(), v.end());
            const uint8_t* np = nb.empty() ? nullptr : nb.data();
            const uint8_t* vp = vb.empty() ? nullptr : vb.data();
            const uint32_t cls = hhuff::req_name_class(np, (uint32_t)nb.size());
            bool header = false;
            int oheader = 0;
            int32_t rg, ro;
            if (resp) {
                rg = h3 ? hhuff::resp_field<true>(rs, cls, vp, (uint32_t)vb.size(), soft, (int32_t)k, header)
                        : hhuff::resp_field<false>(rs, cls, vp, (uint32_t)vb.size(), soft, (int32_t)k, header);
                ro = orc_rs_field(&ors, np, (uint32_t)nb.size(), vp, (uint32_t)vb.size(), soft, (int32_t)k, &oheader,
                                  h3 ? 1 : 0);
            } else {
                rg = h3 ? hhuff::req_field<true>(rq, cls, vp, (uint32_t)vb.size(), soft, (int32_t)k, header)
                        : hhuff::req_field<false>(rq, cls, vp, (uint32_t)vb.size(), soft, (int32_t)k, header);
                ro = orc_rq_field(&orq, np, (uint32_t)nb.size(), vp, (uint32_t)vb.size(), soft, (int32_t)k, &oheader,
                                  h3 ? 1 : 0);
            }
            ++fields;
            if (rg != ro || header != (oheader != 0)) {
                printf("MISMATCH trial %d field %zu (%s: %s) h3 %d resp %d: rule %d/%d oracle %d/%d\n", t, k, n.c_str(),
                       v.c_str(), h3, resp, rg, header, ro, oheader);
                return 1;
            }
            if (rg != 0) {
                ++errs;
                break;
            }
        }
        uint32_t wg[12] = {}, wo[12] = {};
        if (resp) {
            hhuff_response_t out;
            memset(&out, 0, sizeof(out));
            hhuff::resp_store(&out, rs);
            memcpy(wg, &out, sizeof(out));
            orc_rs_store(wo, &ors);
            if (memcmp(wg, wo, sizeof(out)) != 0) {
                printf("MISMATCH trial %d response record (err %u vs %u)\n", t, wg[2], wo[2]);
                return 1;
            }
        } else {
            hhuff_request_t out;
            memset(&out, 0, sizeof(out));
            hhuff::req_store(&out, rq);
            memcpy(wg, &out, sizeof(out));
            orc_rq_store(wo, &orq);
            if (memcmp(wg, wo, sizeof(out)) != 0 || (h3 && rq.dfid != orq.dfid)) {
                printf("MISMATCH trial %d request record (err %u vs %u)\n", t, wg[10], wo[10]);
                return 1;
            }
        }
    }
    printf("ok: %d sequences, %ld fields, %ld rule errors, records equal\n", trials, fields, errs);
    return 0;
}
