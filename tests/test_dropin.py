"""The link-time drop-in through h2o's own callers: oracle/_ref/libh2ocallers.so is the
reference's hpack.c / qpack.c with default symbol visibility, so its decode_string, h2o_hpack_encode_string,
flatten_string, QPACK decode_header ... call h2o_hpack_{de,en}code_huffman through the PLT; with libhhuff.so
loaded RTLD_GLOBAL first those calls land in libhhuff.so, as they do in an h2o linked against it.
tests/dropin_replay.py runs in a fresh process (load order) and prints a JSON verdict.

CPU: the binding itself -- the process-wide symbol is libhhuff.so's, the callers' Huffman calls are counted by
hhuff_per_string_calls(), and with no GPU they fail soft there (decode SIZE_MAX, encode falls back to the raw
string) while the reference's own codec (libh2oref.so, hidden visibility) Huffman-codes the same input.
GPU: every golden fixture (per-string vectors, blocks*.npz, framing.npz, qpack.npz) reproduced through the
reference's callers running on the GPU codec."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _need_callers():
    sys.path.insert(0, ROOT)
    from h2o_amd import codec
    from oracle import oracle as O

    if not (O.callers_available() and O.ref_available()):
        pytest.skip("oracle/_ref/libh2ocallers.so not built (built where /root/reference exists; travels with the tree)")
    if not os.path.exists(codec.LIB_PATH):
        pytest.skip("libhhuff.so not built")


def _replay(mode, timeout):
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "dropin_replay.py"), mode], capture_output=True,
                       text=True, timeout=timeout, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, "replay printed no verdict (rc %d): %s" % (p.returncode, p.stderr[-3000:])
    info = json.loads(lines[-1])
    assert p.returncode == 0 and info["ok"], (info, p.stderr[-3000:])
    return info


def test_callers_bind_to_libhhuff_without_gpu():
    _need_callers()
    import torch

    if torch.cuda.is_available():
        pytest.skip("the fail-soft proof needs a host without a GPU")
    info = _replay("nogpu", 300)
    assert info["global_is_hhuff"] and info["calls"] == 3


@pytest.mark.gpu
def test_callers_reproduce_fixtures_on_gpu():
    _need_callers()
    info = _replay("gpu", 600)
    assert info["framing_mismatches"] == 0 and info["calls"] > 100000
