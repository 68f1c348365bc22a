#!/usr/bin/env python3
"""Per-string symbol latency (bench.py's per_string_latency, 48-B header string) for the service decoder chosen by
HHUFF_SVC_NC in this process; one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    import torch

    import bench
    from h2o_amd import codec

    torch.cuda.set_device(0)
    r = bench.per_string_latency(codec)
    r.pop("long_strings_median_us", None)
    print(json.dumps({"svc_nc": os.environ.get("HHUFF_SVC_NC", "default"), **r}), flush=True)
