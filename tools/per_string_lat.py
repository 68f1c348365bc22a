"""per-string symbol latency (h2o_hpack_{en,de}code_huffman through libhhuff.so): median / p99 microseconds,
plus a known-answer check; HHUFF_NO_SERVICE=1 measures the launch-per-string path"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch  # noqa: F401  (one HIP runtime: torch's)

    from h2o_amd import codec

    assert codec.decode_huffman(bytes.fromhex("f1e3c2e5f23a6ba0ab90f4ff")) == (b"www.example.com", 0)
    s = (b"accept-encoding: gzip, deflate, br, zstd" * 2)[:48]
    h = codec.encode_huffman(s)
    assert codec.decode_huffman(h, False)[0] == s
    out = {"service": os.environ.get("HHUFF_NO_SERVICE", "0") in ("", "0")}
    for name, fn in (("h2o_hpack_encode_huffman", lambda: codec.encode_huffman(s)),
                     ("h2o_hpack_decode_huffman", lambda: codec.decode_huffman(h, False))):
        for _ in range(200):
            fn()
        t = []
        for _ in range(5000):
            t0 = time.perf_counter()
            fn()
            t.append(time.perf_counter() - t0)
        t.sort()
        out[name] = {"median": round(t[len(t) // 2] * 1e6, 2), "p99": round(t[int(len(t) * 0.99)] * 1e6, 2),
                     "min": round(t[0] * 1e6, 2)}
    # after an idle gap (the service wave exits after 2 ms idle): the first call relaunches it
    time.sleep(0.05)
    t0 = time.perf_counter()
    assert codec.decode_huffman(h, False)[0] == s
    out["first_call_after_idle_us"] = round((time.perf_counter() - t0) * 1e6, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
