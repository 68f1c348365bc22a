#!/usr/bin/env python3
"""Host-path study: PCIe ceilings measured with torch copies, then the library's pipelined
host encode / decode at several chunk sizes with pinned and pageable caller buffers."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from h2o_amd import codec, synth

    torch.cuda.set_device(0)
    GB = 1e9
    # PCIe ceilings: H2D, D2H, both at once (two streams)
    N = 512 << 20
    h1 = torch.empty(N, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(N, dtype=torch.uint8).pin_memory()
    d1 = torch.empty(N, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(N, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    res = {}
    for name in ("h2d", "d2h", "both"):
        ts = []
        for _ in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if name in ("h2d", "both"):
                with torch.cuda.stream(s1):
                    d1.copy_(h1, non_blocking=True)
            if name in ("d2h", "both"):
                with torch.cuda.stream(s2):
                    h2.copy_(d2, non_blocking=True)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        t = min(ts[1:])
        res[name + "_GBps"] = round((2 if name == "both" else 1) * N / GB / t, 2)
    print(json.dumps({"pcie": res}), flush=True)
    lib = codec.lib()
    print(json.dumps({"pinned_detect": bool(lib.hhuff_version())}), flush=True)

    b = synth.make_batch_torch("c4", seed=5)
    n, P = b["n"], int(b["total"])
    off = b["off"].to(torch.int32).cpu().numpy().view(np.uint32).copy()
    data_pg = b["data"].cpu().numpy()
    data_pin = torch.empty(P, dtype=torch.uint8).pin_memory().numpy()
    data_pin[:] = data_pg
    out_pin = torch.empty(P + 16, dtype=torch.uint8).pin_memory().numpy()
    out_pg = np.empty(P + 16, np.uint8)
    for chunk in (4 << 20, 16 << 20, 64 << 20):
        for kind, src, dst in (("pinned", data_pin, out_pin), ("pageable", data_pg, out_pg)):
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                codec.encode_batch_host_pipelined(src, off, n, out=dst, chunk_bytes=chunk)
                ts.append(time.perf_counter() - t0)
            t = min(ts[1:])
            moved = P + 4 * (n + 1) + P + 5 * n  # in + offsets + out + out_len + status
            print(json.dumps({"encode_pipelined": kind, "chunk_MiB": chunk >> 20, "ms": round(t * 1e3, 2),
                              "plain_GiBps": round(P / 2 ** 30 / t, 2), "pcie_GBps_moved": round(moved / GB / t, 2)}),
                  flush=True)


if __name__ == "__main__":
    main()
