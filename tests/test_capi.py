"""The C-ABI library builds, loads, and exports every symbol include/hhuff.h declares (no GPU calls)."""
import ctypes
import os
import re

from conftest import ROOT


def declared_functions():
    src = open(os.path.join(ROOT, "include", "hhuff.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*\b([a-z_0-9]+)\s*\(", src, flags=re.M)))


def test_header_declares_the_h2o_symbols():
    names = declared_functions()
    assert "h2o_hpack_decode_huffman" in names and "h2o_hpack_encode_huffman" in names
    assert "hhuff_decode_batch" in names and "hhuff_encode_batch" in names


def test_library_exports_every_declared_symbol():
    from h2o_amd import build, codec

    build.build(verbose=False)
    lib = ctypes.CDLL(codec.LIB_PATH)
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert set(codec.EXPORTED) == set(declared_functions())


def test_library_is_gfx950_code_object():
    from h2o_amd import codec

    blob = open(codec.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
