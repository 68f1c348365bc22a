"""Drop-in replay, run as its own process by tests/test_dropin.py (the load order below needs a fresh process).

libhhuff.so is loaded RTLD_GLOBAL first (after torch, which owns the process's HIP runtime), then
oracle/_ref/libh2ocallers.so: h2o's hpack.c / qpack.c compiled with default visibility, whose calls to
h2o_hpack_decode_huffman / h2o_hpack_encode_huffman go through the PLT and so bind to libhhuff.so -- what
linking h2o against libhhuff.so does ("link-time drop-in").  The reference's own callers
then run unchanged on the GPU codec:

  decode_string (hpack.c:225-262) under h2o_hpack_decode_header      <- tests/golden/blocks*.npz
  h2o_hpack_encode_string (hpack.c:826-842), QPACK flatten_string    <- tests/golden/framing.npz
  (qpack.c:1040-1058)
  QPACK decode_header / h2o_qpack_decoder_handle_input (qpack.c)     <- tests/golden/qpack.npz
  h2o_hpack_decode_huffman itself                                    <- tests/golden/kat.npz

    python tests/dropin_replay.py nogpu   # no GPU: the callers' Huffman calls must land in libhhuff.so
                                          # and fail soft there (proves the binding without a device)
    python tests/dropin_replay.py gpu     # MI355X: every fixture reproduced through the callers
Prints one JSON line; exit 0 = every check held.
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)


def load():
    import torch  # noqa: F401  (one HIP runtime: torch's)

    from h2o_amd import codec
    from oracle import oracle as O

    hh = ctypes.CDLL(codec.LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    hh.hhuff_per_string_calls.restype = ctypes.c_uint64
    callers = O.callers()
    # the symbol the process resolves by name is libhhuff.so's, not the copy inside libh2ocallers.so
    glob = ctypes.c_void_p.from_buffer(ctypes.CDLL(None).h2o_hpack_decode_huffman).value
    mine = ctypes.c_void_p.from_buffer(hh.h2o_hpack_decode_huffman).value
    theirs = ctypes.c_void_p.from_buffer(callers.lib.h2o_hpack_decode_huffman).value
    return hh, callers, dict(global_is_hhuff=glob == mine, callers_copy_is_other=theirs != mine)


def nogpu():
    from oracle import oracle as O

    hh, C, info = load()
    kat = bytes.fromhex("f1e3c2e5f23a6ba0ab90f4ff")  # RFC 7541 C.4.1 "www.example.com"
    before = hh.hhuff_per_string_calls()
    dec, _ = C.decode(kat)  # ref_decode_huffman -> h2o_hpack_decode_huffman@plt
    enc = C.encode_string(b"www.example.com")  # h2o_hpack_encode_string -> encode_huffman@plt
    flat = C.flatten_string(b"www.example.com", 7)  # QPACK flatten_string -> encode_huffman@plt
    calls = hh.hhuff_per_string_calls() - before
    # the compiled reference with its own (hidden) Huffman codec gives the Huffman forms
    R = O.ref()
    info.update(decode_failed_soft=dec is None, ref_decodes=R.decode(kat)[0] == b"www.example.com",
                encode_fell_back_raw=enc == b"\x0f" + b"www.example.com",
                ref_encodes_huffman=R.encode_string(b"www.example.com")[0] == 0x8c,
                flatten_fell_back_raw=flat[0] & 0x80 == 0, calls=calls, calls_ok=calls == 3)
    return info


def gpu():
    import test_hpack_blocks as TB
    import test_oracle_golden as TG
    import test_qpack as TQ
    from conftest import load_golden
    from h2o_amd import synth

    hh, C, info = load()
    c0 = hh.hhuff_per_string_calls()
    # h2o_hpack_{de,en}code_huffman themselves, through the reference's harness entry points: known answers,
    # soft-error accumulation and the golden batches (each string one call)
    TG.test_oracle_kats(C)
    TG.test_oracle_soft_errors_are_or_accumulated(C)
    for name in ("kat", "adversarial", "corpus", "random_c2"):
        TG.test_oracle_decode_matches_golden(C, name)
        if "enc_len" in load_golden(name):
            TG.test_oracle_encode_matches_golden(C, name)
    info["per_string_golden"] = True

    for name in ("blocks", "blocks_256"):  # decode_string under h2o_hpack_decode_header
        gb = load_golden(name)
        res = C.hpack_decode_blocks(gb["data"], gb["blk_off"], gb["conn_first"], int(gb["table_size"][0]))
        TB.check_against_golden(res, gb)
        info[name] = True

    gf = load_golden("framing")  # h2o_hpack_encode_string and QPACK's flatten_string
    strings = synth.unpack(gf["fr_in"], gf["fr_in_off"])
    hp = synth.unpack(gf["hpack_out"], gf["hpack_out_off"])
    qp = synth.unpack(gf["qpack_out"], gf["qpack_out_off"])
    bad = 0
    for s, pb, fb, raw, h, q in zip(strings, gf["fr_prefix"], gf["fr_first"], gf["fr_raw"], hp, qp):
        bad += C.encode_string(s) != h
        bad += C.flatten_string(s, int(pb), int(fb), bool(raw)) != q
    info["framing_mismatches"] = int(bad)

    gq = load_golden("qpack")  # QPACK decode_header / encoder-stream inserts
    for name in TQ.SESSIONS:
        nconn, hts, mb, nbl, steps = TQ.golden_steps(gq, name)
        for res, st in zip(TQ.run_oracle_session(C, nconn, hts, mb, nbl, steps), steps):
            TQ.check_step(res, st, nconn)
        info["qpack_" + name] = True
    info["calls"] = int(hh.hhuff_per_string_calls() - c0)
    info["calls_ok"] = info["calls"] > 100000
    return info


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "gpu"
    info = nogpu() if mode == "nogpu" else gpu()
    ok = all(v for k, v in info.items() if isinstance(v, bool)) and not info.get("framing_mismatches", 0)
    info["ok"] = ok
    print(json.dumps(info), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
