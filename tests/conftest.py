import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


GOLDEN_SETS = ["kat", "corpus", "random_c2", "random_c3", "random_c4", "random_c5", "adversarial"]


@pytest.fixture(scope="session")
def oracle_codec():
    from oracle import oracle as O

    O.build()
    return O.oracle()


def compact(out, out_off, out_len):
    """concatenate the successful outputs (out_len != FAIL) of a slot layout -> bytes"""
    parts = []
    for o, L in zip(out_off, out_len):
        if L != 0xFFFFFFFF:
            parts.append(out[int(o):int(o) + int(L)].tobytes())
    return b"".join(parts)
