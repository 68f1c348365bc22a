"""debug: GPU hhuff_qpack_parse_requests vs the qreq fixtures, first mismatching sections with their fields"""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from conftest import load_golden
import test_qpack as T
import torch

g = load_golden("qpack")
nconn, hts, mb, nbl, steps = T.golden_steps(g, "qreq")
res = T.gpu_session(torch, nconn, hts, mb, nbl, steps, requests=True)
shown = 0
for si, (r, st) in enumerate(zip(res, steps)):
    ns = len(st["sec_off"]) - 1
    got = T.req_words(r["req"], ns)
    for k in range(ns):
        if (got[k] != st["rq_req"][k]).any() or r["sstatus"][k] != st["rq_sstatus"][k]:
            o = int(st["sec_off"][k])
            names = [r["arena"][r["name_off"][f]:r["name_off"][f] + r["name_len"][f]].tobytes() for f in range(o, o + int(r["nfields"][k]))]
            print("step", si, "sec", k, "st", r["sstatus"][k], st["rq_sstatus"][k], "got", got[k][:14].tolist(), "want", st["rq_req"][k][:14].tolist())
            print("   fields", names[-4:], "fflags", r["fflags"][o:o + int(r["nfields"][k])].tolist()[-4:])
            shown += 1
            if shown > 12:
                sys.exit(0)
print("mismatches shown", shown)
