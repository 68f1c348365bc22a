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
    lib = codec.lib()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert set(codec.EXPORTED) == set(declared_functions())


def test_library_is_gfx950_code_object():
    from h2o_amd import codec

    blob = open(codec.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


CAPI_CHECK = os.path.join(ROOT, "build", "capi_check")


def build_capi_check():
    """tests/capi_check.c: a C translation unit against include/hhuff.h, linked with libhhuff.so"""
    import subprocess

    from h2o_amd import build

    build.build(verbose=False)
    os.makedirs(os.path.dirname(CAPI_CHECK), exist_ok=True)
    src = os.path.join(ROOT, "tests", "capi_check.c")
    if not os.path.exists(CAPI_CHECK) or os.path.getmtime(CAPI_CHECK) < max(os.path.getmtime(src),
                                                                            os.path.getmtime(build.LIB)):
        subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
                        "-I" + os.path.join(ROOT, "include"), "-I/opt/rocm/include", src, "-o", CAPI_CHECK,
                        "-L" + os.path.dirname(build.LIB), "-lhhuff", "-L/opt/rocm/lib", "-lamdhip64", "-lpthread",
                        "-Wl,-rpath," + os.path.dirname(build.LIB) + ":/opt/rocm/lib"], check=True)
    return CAPI_CHECK


def test_c_translation_unit_builds_and_links():
    """include/hhuff.h is plain C and every symbol the check program uses resolves in libhhuff.so"""
    assert os.path.exists(build_capi_check())


def test_per_string_symbols_fail_soft_without_a_gpu():
    """no GPU (this container): h2o_hpack_{de,en}code_huffman return SIZE_MAX with a reason, never abort --
    decode then becomes h2o's COMPRESSION error for that literal, encode its raw fallback"""
    import subprocess

    import torch

    if torch.cuda.is_available():
        import pytest

        pytest.skip("a GPU is present (the GPU test runs the full check)")
    r = subprocess.run([build_capi_check(), "nogpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "err=" in r.stdout and "decode=%d" % (2 ** 64 - 1) in r.stdout


import pytest  # noqa: E402


@pytest.mark.gpu
def test_c_translation_unit_on_the_gpu():
    """per-string symbols from 8 concurrent threads, a NULL-stream batch, the host API on device 0, the
    multi-device batch against the one-device call"""
    import subprocess

    for copy in ("0", "1"):  # HHUFF_MULTI_COPY=1: the multi-device call's peer-copy path on this one GPU
        r = subprocess.run([build_capi_check()], capture_output=True, text=True, timeout=120,
                           env=dict(os.environ, HHUFF_MULTI_COPY=copy))
        assert r.returncode == 0, r.stdout + r.stderr
        assert "capi_check: ok" in r.stdout


def test_argument_checks_need_no_gpu():
    """the C ABI rejects bad arguments before touching the device: QPACK inputs of 2^32 bytes or more (u32
    offsets), scratch too small or misaligned -- HHUFF_EINVAL with the reason in hhuff_last_error_string()"""
    from h2o_amd import codec

    L = codec.lib()
    p = 1 << 20  # a 16-byte aligned dummy address: never dereferenced on these paths
    ss = int(L.hhuff_qpack_scratch_size(1, 4096))

    def qpack(in_size, scratch, scratch_size):
        return L.hhuff_qpack_decode(p, in_size, p, p, p, p, 1, 0, 4096, 100, None, None, None, None, None, None,
                                    None, None, None, None, None, p, p, p, scratch, scratch_size, 0, None)

    assert qpack(1 << 32, p, ss) == -1
    assert qpack((1 << 32) - 2, p, ss) == -1  # n_max = in_size + 2 would wrap the u32 literal count
    assert qpack((1 << 32) - 1, p, ss) == -1
    assert b"2^32" in L.hhuff_last_error_string()
    assert qpack(100, p, ss - 1) == -1
    assert b"scratch" in L.hhuff_last_error_string()
    assert qpack(100, p + 8, ss) == -1
    assert b"aligned" in L.hhuff_last_error_string()
