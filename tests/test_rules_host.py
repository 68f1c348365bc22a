"""The GPU request / response rules (h2o_amd/csrc/hhuff_request.h) compiled for the host with AddressSanitizer
and UndefinedBehaviorSanitizer and run against the oracle's restatement of h2o_hpack_parse_request /
h2o_hpack_parse_response's rules (oracle/hpack_block.c) on random field sequences, HTTP/2 and HTTP/3
arguments (tests/rules_host.cpp).  VERDICT r3 asked whether the `__noinline__` around the HTTP/3 rules
(hhuff_qpack.hip) hides undefined behaviour in them: this says the source is clean and right on its own."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rules_clean_under_sanitizers(tmp_path):
    if not shutil.which("g++") or not shutil.which("gcc"):
        pytest.skip("no host compiler")
    san = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"]
    objs = []
    for src in ("hpack_block.c", "huff_oracle.c"):
        o = str(tmp_path / (src + ".o"))
        subprocess.run(["gcc"] + san + ["-c", os.path.join(ROOT, "oracle", src), "-I" + os.path.join(ROOT, "oracle"),
                                        "-o", o], check=True)
        objs.append(o)
    exe = str(tmp_path / "rules_host")
    subprocess.run(["g++", "-std=c++17"] + san + ["-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                                                  "-I" + os.path.join(ROOT, "include"),
                                                  "-I" + os.path.join(ROOT, "h2o_amd", "csrc"),
                                                  "-I" + os.path.join(ROOT, "oracle"),
                                                  os.path.join(ROOT, "tests", "rules_host.cpp")] + objs +
                   ["-lpthread", "-o", exe], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, "20000"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.startswith("ok:"), r.stdout
