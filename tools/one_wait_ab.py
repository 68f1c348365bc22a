#!/usr/bin/env python3
"""Per-string launch path: the result taken when its length lands (wait_one's spin) against the stream
synchronisation (HHUFF_ONE_SYNC=1).  One process per mode (the mode is read once); prints bench.py's
per_string_latency line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: F401,E402  (one HIP runtime: torch's)

import bench  # noqa: E402
from h2o_amd import codec  # noqa: E402

print(json.dumps({"one_sync": os.environ.get("HHUFF_ONE_SYNC", "0"), **bench.per_string_latency(codec, calls=500)}))
