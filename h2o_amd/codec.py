"""ctypes bindings of the hhuff C-ABI (include/hhuff.h) -- the host-side mirror of h2o's interface.

Per-string functions keep h2o's names and meaning (lib/http2/hpack.c:117 / :774):
    decode_huffman(src, is_name, soft_errors=0) -> (bytes | None, soft_errors)   None <=> SIZE_MAX
    encode_huffman(src)                         -> bytes | None                 None <=> SIZE_MAX
Batch functions run the HIP kernels on device tensors (torch is used only for memory and streams):
    decode_batch(...), encode_batch(...)       device-resident arrays, async on the current stream
    decode_batch_host(...), encode_batch_host(...)   numpy arrays, H2D/D2H included
There is no CPU codec behind any of these: if libhhuff.so is missing or no GPU is present they raise.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# HHUFF_AB_LIB: an A/B build of the same library (tools/ab.py build NAME -> build/ab/libhhuff_NAME.so), for
# running the test suite against an experiment; the product path is always h2o_amd/libhhuff.so
LIB_PATH = os.environ.get("HHUFF_AB_LIB") or os.path.join(HERE, "libhhuff.so")

FAIL_LEN = 0xFFFFFFFF
SOFT_NAME = 0x1
SOFT_VALUE = 0x2
STATUS_FAIL = 0x80
STATUS_TOO_LONG = 0xC0
SIZE_MAX = ctypes.c_size_t(-1).value

_vp = ctypes.c_void_p
_lib = None


class HhuffError(RuntimeError):
    pass


def lib():
    """Load libhhuff.so (fails loudly when the HIP extension is not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HhuffError("libhhuff.so not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        # torch first: its ROCm wheel ships its own libamdhip64.so, and libhhuff.so's dependency must
        # resolve to that already-loaded runtime -- one HIP runtime per process (loaded the other way round,
        # two runtimes end up sharing the device and the per-string path fails).  Without torch (the
        # numpy-only host and per-string bindings) the library's own HIP runtime dependency is used.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass

        L = ctypes.CDLL(LIB_PATH)
        L.h2o_hpack_decode_huffman.restype = ctypes.c_size_t
        L.h2o_hpack_decode_huffman.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint), ctypes.c_char_p,
                                               ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p)]
        L.h2o_hpack_encode_huffman.restype = ctypes.c_size_t
        L.h2o_hpack_encode_huffman.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
        L.hhuff_decode_batch.restype = ctypes.c_int
        L.hhuff_decode_batch.argtypes = [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp, _vp]
        L.hhuff_encode_batch.restype = ctypes.c_int
        L.hhuff_encode_batch.argtypes = [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp]
        L.hhuff_decode_batch_packed.restype = ctypes.c_int
        L.hhuff_decode_batch_packed.argtypes = [_vp, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp, _vp]
        L.hhuff_encode_batch_packed.restype = ctypes.c_int
        L.hhuff_encode_batch_packed.argtypes = [_vp, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp]
        L.hhuff_flatten_batch.restype = ctypes.c_int
        L.hhuff_flatten_batch.argtypes = [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32, _vp, ctypes.c_uint, _vp, _vp,
                                          _vp, _vp, _vp]
        L.hhuff_decode_batch_host.restype = ctypes.c_int
        L.hhuff_decode_batch_host.argtypes = [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32, _vp, _vp, ctypes.c_uint64,
                                              _vp, _vp, _vp, ctypes.c_int]
        L.hhuff_encode_batch_host.restype = ctypes.c_int
        L.hhuff_encode_batch_host.argtypes = [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32, _vp, ctypes.c_uint64,
                                              _vp, _vp, _vp, ctypes.c_int]
        L.hhuff_decode_literals.restype = ctypes.c_int
        L.hhuff_decode_literals.argtypes = [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32, ctypes.c_uint, ctypes.c_uint,
                                            _vp, _vp, _vp, _vp, _vp, _vp, _vp]
        L.hhuff_decode_batch_host_pipelined.restype = ctypes.c_int
        L.hhuff_decode_batch_host_pipelined.argtypes = [_vp, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp, _vp,
                                                        ctypes.c_uint64, _vp, _vp, ctypes.c_int, ctypes.c_uint64]
        L.hhuff_encode_batch_host_pipelined.restype = ctypes.c_int
        L.hhuff_encode_batch_host_pipelined.argtypes = [_vp, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp, ctypes.c_uint64,
                                                        _vp, _vp, ctypes.c_int, ctypes.c_uint64]
        L.hhuff_hpack_scratch_size.restype = ctypes.c_uint64
        L.hhuff_hpack_scratch_size.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.hhuff_hpack_decode_blocks.restype = ctypes.c_int
        L.hhuff_hpack_decode_blocks.argtypes = [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp,
                                                _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint64,
                                                ctypes.c_uint, _vp]
        L.hhuff_hpack_parse_requests.restype = ctypes.c_int
        L.hhuff_hpack_parse_requests.argtypes = [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp,
                                                 _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint64,
                                                 ctypes.c_uint, _vp]
        L.hhuff_hpack_parse_responses.restype = ctypes.c_int
        L.hhuff_hpack_parse_responses.argtypes = [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp,
                                                  _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                                  ctypes.c_uint64, ctypes.c_uint, _vp]
        L.hhuff_qpack_parse_responses.restype = ctypes.c_int
        L.hhuff_qpack_parse_responses.argtypes = ([_vp, ctypes.c_uint64, _vp, _vp, _vp, _vp, ctypes.c_uint32,
                                                   ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64] + [_vp] * 17 +
                                                  [ctypes.c_uint64, ctypes.c_uint, _vp])
        L.hhuff_qpack_scratch_size.restype = ctypes.c_uint64
        L.hhuff_qpack_scratch_size.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.hhuff_qpack_decode.restype = ctypes.c_int
        L.hhuff_qpack_decode.argtypes = ([_vp, ctypes.c_uint64, _vp, _vp, _vp, _vp, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_uint64] + [_vp] * 15 +
                                         [ctypes.c_uint64, ctypes.c_uint, _vp])
        L.hhuff_qpack_parse_requests.restype = ctypes.c_int
        L.hhuff_qpack_parse_requests.argtypes = ([_vp, ctypes.c_uint64, _vp, _vp, _vp, _vp, ctypes.c_uint32,
                                                  ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64] + [_vp] * 17 +
                                                 [ctypes.c_uint64, ctypes.c_uint, _vp])
        L.hhuff_hpack_enc_scratch_size.restype = ctypes.c_uint64
        L.hhuff_hpack_enc_scratch_size.argtypes = [ctypes.c_uint32]
        L.hhuff_hpack_flatten_responses.restype = ctypes.c_int
        L.hhuff_hpack_flatten_responses.argtypes = ([_vp, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp, _vp,
                                                     ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
                                                    + [_vp] * 6 + [ctypes.c_uint64, ctypes.c_uint, _vp])
        L.hhuff_qpack_flatten_responses.restype = ctypes.c_int
        L.hhuff_qpack_flatten_responses.argtypes = ([_vp, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp, ctypes.c_uint32,
                                                     ctypes.c_uint32, ctypes.c_uint32] + [_vp] * 6)
        L.hhuff_version.restype = ctypes.c_char_p
        L.hhuff_last_error_string.restype = ctypes.c_char_p
        L.hhuff_grid_size.restype = ctypes.c_int
        L.hhuff_per_string_calls.restype = ctypes.c_uint64
        L.hhuff_grid_size.argtypes = [ctypes.c_int, ctypes.c_int]
        L.hhuff_decode_prices.restype = ctypes.c_int
        L.hhuff_decode_prices.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
        L.hhuff_calibrate_decode_prices.restype = ctypes.c_int
        L.hhuff_calibrate_decode_prices.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
        L.hhuff_set_decode_prices.restype = ctypes.c_int
        L.hhuff_set_decode_prices.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
        L.hhuff_pool_trim.restype = ctypes.c_int
        L.hhuff_pool_trim.argtypes = []
        L.hhuff_set_decode_kernel.restype = ctypes.c_int
        L.hhuff_set_decode_kernel.argtypes = [ctypes.c_int]
        L.hhuff_set_edge_defer_min.restype = ctypes.c_uint32
        L.hhuff_set_edge_defer_min.argtypes = [ctypes.c_uint32]
        L.hhuff_decode_batch_host_packed.restype = ctypes.c_int
        L.hhuff_decode_batch_host_packed.argtypes = [_vp, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp, _vp, ctypes.c_uint64,
                                                     _vp, _vp, _vp, ctypes.c_int]
        L.hhuff_encode_batch_host_packed.restype = ctypes.c_int
        L.hhuff_encode_batch_host_packed.argtypes = [_vp, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp, ctypes.c_uint64,
                                                     _vp, _vp, _vp, ctypes.c_int]
        L.hhuff_decode_batch_multi.restype = ctypes.c_int
        L.hhuff_decode_batch_multi.argtypes = [ctypes.c_int, _vp, ctypes.c_int, _vp, ctypes.c_uint64, _vp, ctypes.c_uint32,
                                               _vp, _vp, ctypes.c_uint64, _vp, _vp, _vp]
        L.hhuff_encode_batch_multi.restype = ctypes.c_int
        L.hhuff_encode_batch_multi.argtypes = [ctypes.c_int, _vp, ctypes.c_int, _vp, ctypes.c_uint64, _vp, ctypes.c_uint32,
                                               _vp, ctypes.c_uint64, _vp, _vp, _vp]
        L.hhuff_shard_bounds.restype = ctypes.c_int
        L.hhuff_shard_bounds.argtypes = [_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _vp]
        _lib = L
    return _lib


# symbols include/hhuff.h declares (checked by tests/test_capi_symbols.py)
EXPORTED = ("h2o_hpack_decode_huffman", "h2o_hpack_encode_huffman", "hhuff_decode_batch", "hhuff_encode_batch",
            "hhuff_decode_batch_packed", "hhuff_encode_batch_packed",
            "hhuff_flatten_batch", "hhuff_decode_literals", "hhuff_hpack_decode_blocks", "hhuff_hpack_scratch_size",
            "hhuff_hpack_parse_requests", "hhuff_hpack_parse_responses",
            "hhuff_qpack_decode", "hhuff_qpack_parse_requests", "hhuff_qpack_parse_responses", "hhuff_qpack_scratch_size",
            "hhuff_decode_batch_host", "hhuff_encode_batch_host", "hhuff_decode_batch_host_pipelined",
            "hhuff_encode_batch_host_pipelined", "hhuff_version", "hhuff_last_error_string", "hhuff_per_string_calls",
            "hhuff_grid_size", "hhuff_decode_prices", "hhuff_calibrate_decode_prices", "hhuff_set_decode_prices",
            "hhuff_pool_trim", "hhuff_service_stamps", "hhuff_hpack_enc_scratch_size",
            "hhuff_hpack_flatten_responses", "hhuff_qpack_flatten_responses", "hhuff_set_decode_kernel",
            "hhuff_decode_batch_host_packed", "hhuff_encode_batch_host_packed", "hhuff_set_edge_defer_min",
            "hhuff_decode_batch_multi", "hhuff_encode_batch_multi", "hhuff_shard_bounds")


def _check(rc, what):
    if rc != 0:
        raise HhuffError("%s failed (%d): %s" % (what, rc, lib().hhuff_last_error_string().decode()))


# ---------------------------------------------------------------------------------------------------
# per-string (h2o signatures)
# ---------------------------------------------------------------------------------------------------
def decode_huffman(src: bytes, is_name: bool = False, soft_errors: int = 0):
    """h2o_hpack_decode_huffman: -> (decoded bytes or None for SIZE_MAX, soft_errors word)."""
    buf = ctypes.create_string_buffer(max(1, 2 * len(src)))
    soft = ctypes.c_uint(soft_errors)
    err = ctypes.c_char_p()
    r = lib().h2o_hpack_decode_huffman(buf, ctypes.byref(soft), src, len(src), int(bool(is_name)), ctypes.byref(err))
    if r == SIZE_MAX:
        return None, soft.value
    return buf.raw[:r], soft.value


def encode_huffman(src: bytes):
    """h2o_hpack_encode_huffman: -> Huffman bytes, or None when not shorter than the input (SIZE_MAX)."""
    buf = ctypes.create_string_buffer(max(1, len(src)))
    r = lib().h2o_hpack_encode_huffman(buf, src, len(src))
    if r == SIZE_MAX:
        return None
    return buf.raw[:r]


# ---------------------------------------------------------------------------------------------------
# device batch API (torch tensors; uint32 arrays are carried in int32 tensors, same bits)
# ---------------------------------------------------------------------------------------------------
def _dp(t):
    if t is None:
        return None
    assert t.is_cuda and t.is_contiguous(), "device batch arrays must be contiguous device tensors"
    return t.data_ptr()


def _stream(stream):
    import torch

    s = torch.cuda.current_stream() if stream is None else stream
    return s.cuda_stream


def decode_slot_size(in_size: int) -> int:
    """bytes the implicit decode layout (out_off = floor(8 * in_off / 5)) needs"""
    return (in_size * 8) // 5 + 16


def decode_batch(data, in_off, n, in_len=None, is_name_bits=None, out=None, out_off=None, out_len=None, status=None,
                 in_size=None, stream=None):
    """Batched h2o_hpack_decode_huffman on device tensors; returns (out, out_len, status)."""
    import torch

    dev = data.device
    in_size = data.numel() if in_size is None else in_size
    if out is None:
        out = torch.empty(decode_slot_size(in_size) if out_off is None else in_size * 2 + 16, dtype=torch.uint8,
                          device=dev)
    if out_len is None:
        out_len = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    if status is None:
        status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    _check(lib().hhuff_decode_batch(_dp(data), in_size, _dp(in_off), _dp(in_len), n, _dp(is_name_bits), _dp(out),
                                    _dp(out_off), _dp(out_len), _dp(status), _stream(stream)), "hhuff_decode_batch")
    return out, out_len, status


def encode_batch(data, in_off, n, in_len=None, out=None, out_off=None, out_len=None, status=None, in_size=None,
                 stream=None):
    """Batched h2o_hpack_encode_huffman on device tensors; returns (out, out_len, status)."""
    import torch

    dev = data.device
    in_size = data.numel() if in_size is None else in_size
    if out is None:
        out = torch.empty(in_size + 16, dtype=torch.uint8, device=dev)
    if out_len is None:
        out_len = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    if status is None:
        status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    _check(lib().hhuff_encode_batch(_dp(data), in_size, _dp(in_off), _dp(in_len), n, _dp(out), _dp(out_off),
                                    _dp(out_len), _dp(status), _stream(stream)), "hhuff_encode_batch")
    return out, out_len, status


def decode_batch_packed(data, in_off, n, is_name_bits=None, out=None, out_off=None, out_len=None, status=None,
                        in_size=None, stream=None):
    """Batched h2o_hpack_decode_huffman with packed output (include/hhuff.h hhuff_decode_batch_packed):
    returns (out, out_off [n+1], out_len, status); string i at out[out_off[i] : out_off[i] + out_len[i]]."""
    import torch

    dev = data.device
    in_size = data.numel() if in_size is None else in_size
    if out is None:
        out = torch.empty(decode_slot_size(in_size), dtype=torch.uint8, device=dev)
    if out_off is None:
        out_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    if out_len is None:
        out_len = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    if status is None:
        status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    _check(lib().hhuff_decode_batch_packed(_dp(data), in_size, _dp(in_off), n, _dp(is_name_bits), _dp(out),
                                           _dp(out_off), _dp(out_len), _dp(status), _stream(stream)),
           "hhuff_decode_batch_packed")
    return out, out_off, out_len, status


def encode_batch_packed(data, in_off, n, out=None, out_off=None, out_len=None, status=None, in_size=None, stream=None):
    """Batched h2o_hpack_encode_huffman with packed output (include/hhuff.h hhuff_encode_batch_packed):
    returns (out, out_off [n+1], out_len, status)."""
    import torch

    dev = data.device
    in_size = data.numel() if in_size is None else in_size
    if out is None:
        out = torch.empty(in_size + 16, dtype=torch.uint8, device=dev)
    if out_off is None:
        out_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    if out_len is None:
        out_len = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    if status is None:
        status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    _check(lib().hhuff_encode_batch_packed(_dp(data), in_size, _dp(in_off), n, _dp(out), _dp(out_off), _dp(out_len),
                                           _dp(status), _stream(stream)), "hhuff_encode_batch_packed")
    return out, out_off, out_len, status


def flatten_batch(data, in_off, n, prefix_bits=7, in_len=None, first_bytes=None, raw_bits=None, out=None, out_off=None,
                  out_len=None, in_size=None, stream=None):
    """Batched QPACK flatten_string / HPACK h2o_hpack_encode_string framing; returns (out, out_len)."""
    import torch

    dev = data.device
    in_size = data.numel() if in_size is None else in_size
    if out is None:
        out = torch.empty(in_size + 11 * max(n, 1) + 16, dtype=torch.uint8, device=dev)
    if out_len is None:
        out_len = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    _check(lib().hhuff_flatten_batch(_dp(data), in_size, _dp(in_off), _dp(in_len), n, _dp(first_bytes), prefix_bits,
                                     _dp(raw_bits), _dp(out), _dp(out_off), _dp(out_len), _stream(stream)),
           "hhuff_flatten_batch")
    return out, out_len


LIT_QPACK = 1


def decode_literals(data, lit_off, lit_end, n, prefix_bits=7, qpack=False, is_name_bits=None, out=None, in_size=None,
                    stream=None):
    """Batched HPACK decode_string / QPACK literal decode on device tensors.
    Returns (out, out_len, pay_off, consumed, status); decoded bytes at out[floor(8 * pay_off / 5)]."""
    import torch

    dev = data.device
    in_size = data.numel() if in_size is None else in_size
    if out is None:
        out = torch.empty(decode_slot_size(in_size), dtype=torch.uint8, device=dev)
    m = max(n, 1)
    out_len = torch.empty(m, dtype=torch.int32, device=dev)
    pay_off = torch.empty(m, dtype=torch.int32, device=dev)
    consumed = torch.empty(m, dtype=torch.int32, device=dev)
    status = torch.empty(m, dtype=torch.uint8, device=dev)
    _check(lib().hhuff_decode_literals(_dp(data), in_size, _dp(lit_off), _dp(lit_end), n, prefix_bits,
                                       LIT_QPACK if qpack else 0, _dp(is_name_bits), _dp(out), _dp(out_len),
                                       _dp(pay_off), _dp(consumed), _dp(status), _stream(stream)), "hhuff_decode_literals")
    return out, out_len, pay_off, consumed, status


BLK_ARENA = -300
BLK_SKIPPED = -301
ERR_PROTOCOL = -1
ERR_COMPRESSION = -9


def default_arena_off(blk_off, table_size=4096):
    """u64 arena slice offsets per block (torch, on blk_off's device): a block of L bytes gets
    floor(8 L / 5) + (L / 4 + 1) * (table_size + 64) bytes -- literals expand at most 8/5, and an indexed
    field (>= 1 byte) copies at most one table entry"""
    import torch

    L = (blk_off[1:].to(torch.int64) & 0xFFFFFFFF) - (blk_off[:-1].to(torch.int64) & 0xFFFFFFFF)
    cap = (L * 8) // 5 + (L // 4 + 1) * (table_size + 64)
    out = torch.zeros(L.numel() + 1, dtype=torch.int64, device=blk_off.device)
    out[1:] = torch.cumsum(cap, 0)
    return out


BLK_CONTINUE = 1


# include/hhuff.h hhuff_request_t: 12 u32 words per block
REQUEST_FIELDS = ("content_length", "method", "scheme", "authority", "path", "protocol", "expect", "exists_map",
                  "nheaders", "err", "scheme_kind")
FIELD_HEADER = 0x4
# include/hhuff.h hhuff_response_t: 4 words per block; hhuff_qpack_response_head_t: 40 bytes per section
RESPONSE_FIELDS = ("status", "nheaders", "err", "datagram_flow_id")
QRES_BYTES = 40


def hpack_decode_blocks(data, blk_off, conn_first, table_size=4096, arena_off=None, in_size=None, stream=None,
                        scratch=None, cont=False, requests=False, responses=False, trailers=None):
    """HPACK header blocks (include/hhuff.h hhuff_hpack_decode_blocks) on device tensors: blk_off / conn_first
    int32 tensors (u32 bits), arena_off int64.  Returns a dict of device tensors: arena, name_off, name_len,
    value_off, value_len, fflags (per field slot), nfields, bstatus (per block).  requests=True runs
    hhuff_hpack_parse_requests (h2o_hpack_parse_request per block) and adds req: int32 [nblk, 12], the
    hhuff_request_t words (REQUEST_FIELDS; content_length is words 0-1).  responses=True runs
    hhuff_hpack_parse_responses (h2o_hpack_parse_response per block; trailers: uint8 tensor, nonzero for a
    trailers block, or None) and adds res: int32 [nblk, 4], the hhuff_response_t words (RESPONSE_FIELDS)."""
    import torch

    dev = data.device
    in_size = data.numel() if in_size is None else in_size
    nblk = blk_off.numel() - 1
    nconn = conn_first.numel() - 1
    if arena_off is None:
        arena_off = default_arena_off(blk_off, table_size)
    nslots = max(1, int(blk_off[-1].item()) & 0xFFFFFFFF)
    r = dict(arena=torch.empty(max(1, int(arena_off[-1].item())), dtype=torch.uint8, device=dev),
             name_off=torch.empty(nslots, dtype=torch.int32, device=dev),
             name_len=torch.empty(nslots, dtype=torch.int32, device=dev),
             value_off=torch.empty(nslots, dtype=torch.int32, device=dev),
             value_len=torch.empty(nslots, dtype=torch.int32, device=dev),
             fflags=torch.empty(nslots, dtype=torch.uint8, device=dev),
             nfields=torch.empty(max(1, nblk), dtype=torch.int32, device=dev),
             bstatus=torch.empty(max(1, nblk), dtype=torch.int32, device=dev))
    ss = int(lib().hhuff_hpack_scratch_size(nconn, table_size))
    if scratch is None:  # pass the previous call's r["scratch"] back with cont=True to carry the tables over
        scratch = torch.empty(max(16, ss), dtype=torch.uint8, device=dev)
    args = [_dp(data), in_size, _dp(blk_off), _dp(conn_first), nconn, table_size, _dp(r["arena"]), _dp(arena_off),
            _dp(r["name_off"]), _dp(r["name_len"]), _dp(r["value_off"]), _dp(r["value_len"]), _dp(r["fflags"]),
            _dp(r["nfields"]), _dp(r["bstatus"])]
    tail = [_dp(scratch), scratch.numel(), BLK_CONTINUE if cont else 0, _stream(stream)]
    if responses:
        r["res"] = torch.empty((max(1, nblk), 4), dtype=torch.int32, device=dev)
        _check(lib().hhuff_hpack_parse_responses(*args[:6], None if trailers is None else _dp(trailers), *args[6:],
                                                 _dp(r["res"]), *tail), "hhuff_hpack_parse_responses")
    elif requests:
        r["req"] = torch.empty((max(1, nblk), 12), dtype=torch.int32, device=dev)
        _check(lib().hhuff_hpack_parse_requests(*args, _dp(r["req"]), *tail), "hhuff_hpack_parse_requests")
    else:
        _check(lib().hhuff_hpack_decode_blocks(*args, *tail), "hhuff_hpack_decode_blocks")
    r["scratch"] = scratch  # keep alive until the stream has run the launch
    return r


QPK_CONTINUE = 1


QREQ_BYTES = 72  # sizeof(hhuff_qpack_request_t)


def qpack_decode(data, enc_off, enc_len, sec_off, conn_first, nsec, header_table_size=4096, max_blocked=100,
                 num_blocked=None, arena_off=None, in_size=None, stream=None, scratch=None, cont=False, arena=None,
                 stream_id=None, responses=False):
    """QPACK decoder step (include/hhuff.h hhuff_qpack_decode) on device tensors: enc_off / enc_len (per
    connection), sec_off / conn_first / num_blocked int32 tensors (u32 bits), arena_off int64; nsec =
    conn_first[-1] as a host int.  Returns a dict of device tensors: arena, name_off, name_len, value_off,
    value_len, fflags (per field slot), nfields, sstatus, req_insert_count (per section), enc_status,
    enc_consumed, insert_count (per connection), and the scratch holding the tables (pass it back with
    cont=True for the next step).  stream_id (int64 tensor, one per section): the HTTP/3 request step,
    hhuff_qpack_parse_requests (h2o_qpack_parse_request per section), plus "req": uint8 [nsec, 72] records
    (hhuff_qpack_request_t).  responses=True (with stream_id): the HTTP/3 client's step,
    hhuff_qpack_parse_responses (h2o_qpack_parse_response per section), plus "res": uint8 [nsec, 40] records
    (hhuff_qpack_response_head_t)."""
    import torch

    dev = data.device
    in_size = data.numel() if in_size is None else in_size
    nconn = conn_first.numel() - 1
    if arena_off is None:
        arena_off = default_arena_off(sec_off, header_table_size)
    nslots = max(1, int(sec_off[-1].item()) & 0xFFFFFFFF)
    i32 = lambda n: torch.empty(max(1, n), dtype=torch.int32, device=dev)  # noqa: E731
    if arena is None:
        arena = torch.empty(max(1, int(arena_off[-1].item())), dtype=torch.uint8, device=dev)
    r = dict(arena=arena,
             name_off=i32(nslots), name_len=i32(nslots), value_off=i32(nslots), value_len=i32(nslots),
             fflags=torch.empty(nslots, dtype=torch.uint8, device=dev), nfields=i32(nsec), sstatus=i32(nsec),
             req_insert_count=torch.empty(max(1, nsec), dtype=torch.int64, device=dev), enc_status=i32(nconn),
             enc_consumed=i32(nconn), insert_count=torch.empty(max(1, nconn), dtype=torch.int64, device=dev))
    ss = int(lib().hhuff_qpack_scratch_size(nconn, header_table_size))
    if scratch is None:
        scratch = torch.empty(max(16, ss), dtype=torch.uint8, device=dev)
    args = [_dp(data), in_size, _dp(enc_off), _dp(enc_len), _dp(sec_off), _dp(conn_first), nconn, nsec,
            header_table_size, max_blocked, None if num_blocked is None else _dp(num_blocked), _dp(r["arena"]),
            _dp(arena_off), _dp(r["name_off"]), _dp(r["name_len"]), _dp(r["value_off"]), _dp(r["value_len"]),
            _dp(r["fflags"]), _dp(r["nfields"]), _dp(r["sstatus"]), _dp(r["req_insert_count"]), _dp(r["enc_status"]),
            _dp(r["enc_consumed"]), _dp(r["insert_count"])]
    tail = [_dp(scratch), scratch.numel(), QPK_CONTINUE if cont else 0, _stream(stream)]
    if stream_id is None:
        _check(lib().hhuff_qpack_decode(*(args + tail)), "hhuff_qpack_decode")
    elif responses:
        r["res"] = torch.empty((max(1, nsec), QRES_BYTES), dtype=torch.uint8, device=dev)
        _check(lib().hhuff_qpack_parse_responses(*(args + [_dp(stream_id), _dp(r["res"])] + tail)),
               "hhuff_qpack_parse_responses")
    else:
        r["req"] = torch.empty((max(1, nsec), QREQ_BYTES), dtype=torch.uint8, device=dev)
        _check(lib().hhuff_qpack_parse_requests(*(args + [_dp(stream_id), _dp(r["req"])] + tail)),
               "hhuff_qpack_parse_requests")
    r["scratch"] = scratch
    return r


# include/hhuff.h hhuff_hpack_header_t / hhuff_hpack_response_t as numpy records
HPE_HEADER_DTYPE = np.dtype([("name_off", "<u4"), ("name_len", "<u4"), ("value_off", "<u4"), ("value_len", "<u4"),
                             ("flags", "<u4")])
HPE_RESPONSE_DTYPE = np.dtype([("content_length", "<u8"), ("stream_id", "<u4"), ("status", "<u4"),
                               ("hdr_first", "<u4"), ("nhdr", "<u4"), ("header_table_size", "<u4"),
                               ("max_frame_size", "<u4"), ("flags", "<u4"), ("reserved", "<u4")])
HDR_DONT_COMPRESS, HDR_TOKEN = 1, 2
RES_END_STREAM, RES_SERVER, RES_TRAILERS, RES_REQUEST = 1, 2, 4, 8
ENC_CONTINUE = 1
RES_SPACE, RES_SKIPPED, RES_EINVAL = -300, -301, -303


def hpack_response_bound(name_value_bytes, nhdr, server_len, max_frame_size):
    """include/hhuff.h hhuff_hpack_response_bound (numpy arrays or ints)"""
    payload = name_value_bytes + 21 * np.asarray(nhdr, np.int64) + 10 + 23 + np.where(
        np.asarray(server_len) != 0, np.asarray(server_len, np.int64) + 26, 0)
    return 9 + payload + 9 * (payload // np.maximum(np.asarray(max_frame_size, np.int64), 1) + 1)


QPE_RESPONSE_DTYPE = np.dtype([("content_length", "<u8"), ("status", "<u4"), ("hdr_first", "<u4"), ("nhdr", "<u4"),
                               ("flags", "<u4"), ("dfid_off", "<u4"), ("dfid_len", "<u4")])
QRES_DATAGRAM, QRES_REQUEST = 8, 16


def qpack_response_bound(name_value_bytes, nhdr, server_len, dfid_len):
    """include/hhuff.h hhuff_qpack_response_bound (numpy arrays or ints)"""
    sl = np.asarray(server_len, np.int64)
    return (9 + 2 + 8 + 23 + 26 + np.asarray(dfid_len, np.int64) + np.where(sl != 0, sl + 12, 0) +
            21 * np.asarray(nhdr, np.int64) + name_value_bytes)


def qpack_flatten_responses(data, hdr, res, nres, out_off, server_off=0, server_len=0, in_size=None, out=None,
                            stream=None):
    """HTTP/3 response HEADERS frames (include/hhuff.h hhuff_qpack_flatten_responses) on device tensors: hdr =
    uint8 tensor of HPE_HEADER_DTYPE records, res = uint8 tensor of QPE_RESPONSE_DTYPE records (32 B), out_off
    int64 [nres + 1].  Returns a dict of device tensors: out, out_len, header_len, rstatus."""
    import torch

    dev = data.device
    in_size = data.numel() if in_size is None else in_size
    nhdr = hdr.numel() // HPE_HEADER_DTYPE.itemsize
    if out is None:
        out = torch.empty(max(1, int(out_off[-1].item())), dtype=torch.uint8, device=dev)
    i32 = lambda n: torch.empty(max(1, n), dtype=torch.int32, device=dev)  # noqa: E731
    r = dict(out=out, out_len=i32(nres), header_len=i32(nres), rstatus=i32(nres))
    _check(lib().hhuff_qpack_flatten_responses(
        _dp(data), in_size, _dp(hdr) if nhdr else None, nhdr, _dp(res), nres, server_off, server_len, _dp(out),
        _dp(out_off), _dp(r["out_len"]), _dp(r["header_len"]), _dp(r["rstatus"]), _stream(stream)),
        "hhuff_qpack_flatten_responses")
    return r


def hpack_flatten_responses(data, hdr, res, conn_first, nres, out_off, server_off=0, server_len=0, in_size=None,
                            out=None, scratch=None, cont=False, stream=None):
    """HTTP/2 response header blocks (include/hhuff.h hhuff_hpack_flatten_responses) on device tensors:
    hdr = uint8 tensor of HPE_HEADER_DTYPE records (20 B each), res = uint8 tensor of HPE_RESPONSE_DTYPE
    records (40 B), conn_first int32 (u32 bits), out_off int64 [nres + 1]; nres = conn_first[-1] as a host int.
    Returns a dict of device tensors: out, out_len, headers_size, rstatus, and the scratch holding the encoder
    tables (pass it back with cont=True for the connections' next responses)."""
    import torch

    dev = data.device
    in_size = data.numel() if in_size is None else in_size
    nconn = conn_first.numel() - 1
    nhdr = hdr.numel() // HPE_HEADER_DTYPE.itemsize
    if out is None:
        out = torch.empty(max(1, int(out_off[-1].item())), dtype=torch.uint8, device=dev)
    i32 = lambda n: torch.empty(max(1, n), dtype=torch.int32, device=dev)  # noqa: E731
    r = dict(out=out, out_len=i32(nres), headers_size=i32(nres), rstatus=i32(nres))
    ss = int(lib().hhuff_hpack_enc_scratch_size(nconn))
    if scratch is None:
        scratch = torch.empty(max(16, ss), dtype=torch.uint8, device=dev)
    _check(lib().hhuff_hpack_flatten_responses(
        _dp(data), in_size, _dp(hdr) if nhdr else None, nhdr, _dp(res), _dp(conn_first), nconn, nres, server_off,
        server_len, _dp(out), _dp(out_off), _dp(r["out_len"]), _dp(r["headers_size"]), _dp(r["rstatus"]),
        _dp(scratch), scratch.numel(), ENC_CONTINUE if cont else 0, _stream(stream)), "hhuff_hpack_flatten_responses")
    r["scratch"] = scratch
    return r


# ---------------------------------------------------------------------------------------------------
# host batch API (numpy arrays; H2D/D2H inside the library)
# ---------------------------------------------------------------------------------------------------
def _np(a, dt):
    """a C-contiguous numpy view of `a` with dtype dt (u32 data may arrive as int32)"""
    a = np.asarray(a)
    if a.dtype != dt:
        a = a.view(dt) if a.dtype.itemsize == np.dtype(dt).itemsize else a.astype(dt)
    return np.ascontiguousarray(a)


def _hp(a):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def decode_batch_host(data, in_off, n, in_len=None, is_name_bits=None, out_off=None, out_size=None, device=0):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    if out_size is None:
        out_size = decode_slot_size(data.size)
    out = np.zeros(max(1, out_size), np.uint8)
    out_len = np.zeros(max(1, n), np.uint32)
    status = np.zeros(max(1, n), np.uint8)
    _check(lib().hhuff_decode_batch_host(_hp(data), data.size, _hp(in_off), _hp(in_len), n, _hp(is_name_bits), _hp(out),
                                         out.size, _hp(out_off), _hp(out_len), _hp(status), device),
           "hhuff_decode_batch_host")
    return out, out_len[:n], status[:n]


def encode_batch_host(data, in_off, n, in_len=None, out_off=None, out_size=None, device=0):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    if out_size is None:
        out_size = data.size + 16
    out = np.zeros(max(1, out_size), np.uint8)
    out_len = np.zeros(max(1, n), np.uint32)
    status = np.zeros(max(1, n), np.uint8)
    _check(lib().hhuff_encode_batch_host(_hp(data), data.size, _hp(in_off), _hp(in_len), n, _hp(out), out.size,
                                         _hp(out_off), _hp(out_len), _hp(status), device), "hhuff_encode_batch_host")
    return out, out_len[:n], status[:n]


def decode_batch_host_pipelined(data, in_off, n, is_name_bits=None, out=None, chunk_bytes=0, device=0, out_len=None,
                                status=None):
    """Pipelined host decode (contiguous layout).  Caller buffers may be pinned memory (DMA'd in place)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    if out is None:
        out = np.zeros(decode_slot_size(data.size), np.uint8)
    out_len = np.zeros(max(1, n), np.uint32) if out_len is None else out_len
    status = np.zeros(max(1, n), np.uint8) if status is None else status
    _check(lib().hhuff_decode_batch_host_pipelined(_hp(data), data.size, _hp(in_off), n, _hp(is_name_bits), _hp(out),
                                                   out.size, _hp(out_len), _hp(status), device, chunk_bytes),
           "hhuff_decode_batch_host_pipelined")
    return out, out_len[:n], status[:n]


def encode_batch_host_pipelined(data, in_off, n, out=None, chunk_bytes=0, device=0, out_len=None, status=None):
    """Pipelined host encode (contiguous layout, output slot = in_off)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    if out is None:
        out = np.zeros(data.size + 16, np.uint8)
    out_len = np.zeros(max(1, n), np.uint32) if out_len is None else out_len
    status = np.zeros(max(1, n), np.uint8) if status is None else status
    _check(lib().hhuff_encode_batch_host_pipelined(_hp(data), data.size, _hp(in_off), n, _hp(out), out.size,
                                                   _hp(out_len), _hp(status), device, chunk_bytes),
           "hhuff_encode_batch_host_pipelined")
    return out, out_len[:n], status[:n]


def decode_batch_host_packed(data, in_off, n, is_name_bits=None, out=None, device=0, out_off=None, out_len=None,
                             status=None, with_off=True):
    """hhuff_decode_batch_host_packed on numpy arrays: the packed layout (tile runs, out_off[n + 1]); pinned arrays are
    read and written by the kernels in place (zero copy).  Returns (out, out_off[:n + 1], out_len[:n], status[:n]);
    with_off=False passes out_off NULL (not returned, out_off None: see packed_positions)"""
    data, in_off = _np(data, np.uint8), _np(in_off, np.uint32)
    size = decode_slot_size(int(in_off[n]))
    out = np.zeros(size, np.uint8) if out is None else out
    out_off = None if not with_off else np.zeros(n + 1, np.uint32) if out_off is None else out_off
    out_len = np.zeros(max(1, n), np.uint32) if out_len is None else out_len
    status = np.zeros(max(1, n), np.uint8) if status is None else status
    names = None if is_name_bits is None else _np(is_name_bits, np.uint32)
    _check(lib().hhuff_decode_batch_host_packed(_hp(data), data.size, _hp(in_off), n, _hp(names), _hp(out), out.size,
                                                _hp(out_off), _hp(out_len), _hp(status), device),
           "hhuff_decode_batch_host_packed")
    return out, None if out_off is None else out_off[:n + 1], out_len[:n], status[:n]


def encode_batch_host_packed(data, in_off, n, out=None, device=0, out_off=None, out_len=None, status=None,
                             with_off=True, with_status=True):
    """hhuff_encode_batch_host_packed on numpy arrays (see decode_batch_host_packed; with_status=False passes
    status NULL: out_len's HHUFF_FAIL_LEN already says which strings stay plain)"""
    data, in_off = _np(data, np.uint8), _np(in_off, np.uint32)
    out = np.zeros(int(in_off[n]) + 16, np.uint8) if out is None else out
    out_off = None if not with_off else np.zeros(n + 1, np.uint32) if out_off is None else out_off
    out_len = np.zeros(max(1, n), np.uint32) if out_len is None else out_len
    status = None if not with_status else np.zeros(max(1, n), np.uint8) if status is None else status
    _check(lib().hhuff_encode_batch_host_packed(_hp(data), data.size, _hp(in_off), n, _hp(out), out.size, _hp(out_off),
                                                _hp(out_len), _hp(status), device),
           "hhuff_encode_batch_host_packed")
    return (out, None if out_off is None else out_off[:n + 1], out_len[:n],
            None if status is None else status[:n])


HOST_MEMORY = -1


def shard_bounds(in_off, n, nshards, align=64):
    """hhuff_shard_bounds: the C library's byte-balanced cut of a contiguous batch (host arrays, no GPU work)
    -> uint32 bounds[nshards + 1]"""
    in_off = _np(in_off, np.uint32)
    b = np.zeros(nshards + 1, np.uint32)
    _check(lib().hhuff_shard_bounds(_hp(in_off), n, nshards, align, _hp(b)), "hhuff_shard_bounds")
    return b


def _devs(devices):
    arr = (ctypes.c_int * len(devices))(*devices)
    return arr, ctypes.cast(arr, _vp)


def decode_batch_multi(devices, data, in_off, n, is_name_bits=None, out=None, out_len=None, status=None, stream=None):
    """hhuff_decode_batch_multi.  numpy arrays: the host mode (every device runs its shard through the host path);
    torch tensors on one device: the device mode (shards on other devices by peer copy), asynchronous on `stream`.
    Returns (out, out_len, status) in the one-device slot layout"""
    devs, dp = _devs(devices)
    if isinstance(data, np.ndarray):
        data, in_off = _np(data, np.uint8), _np(in_off, np.uint32)
        out = np.zeros(decode_slot_size(int(in_off[n])), np.uint8) if out is None else out
        out_len = np.zeros(max(1, n), np.uint32) if out_len is None else out_len
        status = np.zeros(max(1, n), np.uint8) if status is None else status
        names = None if is_name_bits is None else _np(is_name_bits, np.uint32)
        _check(lib().hhuff_decode_batch_multi(len(devices), dp, HOST_MEMORY, _hp(data), data.size, _hp(in_off), n,
                                              _hp(names), _hp(out), out.size, _hp(out_len), _hp(status), None),
               "hhuff_decode_batch_multi")
        return out, out_len[:n], status[:n]
    import torch

    dev = data.device
    if out is None:
        out = torch.empty(decode_slot_size(data.numel()), dtype=torch.uint8, device=dev)
    if out_len is None:
        out_len = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    if status is None:
        status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    _check(lib().hhuff_decode_batch_multi(len(devices), dp, dev.index, _dp(data), data.numel(), _dp(in_off), n,
                                          _dp(is_name_bits), _dp(out), out.numel(), _dp(out_len), _dp(status),
                                          _stream(stream)), "hhuff_decode_batch_multi")
    return out, out_len, status


def encode_batch_multi(devices, data, in_off, n, out=None, out_len=None, status=None, stream=None):
    """hhuff_encode_batch_multi (see decode_batch_multi)"""
    devs, dp = _devs(devices)
    if isinstance(data, np.ndarray):
        data, in_off = _np(data, np.uint8), _np(in_off, np.uint32)
        out = np.zeros(int(in_off[n]) + 16, np.uint8) if out is None else out
        out_len = np.zeros(max(1, n), np.uint32) if out_len is None else out_len
        status = np.zeros(max(1, n), np.uint8) if status is None else status
        _check(lib().hhuff_encode_batch_multi(len(devices), dp, HOST_MEMORY, _hp(data), data.size, _hp(in_off), n,
                                              _hp(out), out.size, _hp(out_len), _hp(status), None),
               "hhuff_encode_batch_multi")
        return out, out_len[:n], status[:n]
    import torch

    dev = data.device
    if out is None:
        out = torch.empty(data.numel() + 16, dtype=torch.uint8, device=dev)
    if out_len is None:
        out_len = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    if status is None:
        status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    _check(lib().hhuff_encode_batch_multi(len(devices), dp, dev.index, _dp(data), data.numel(), _dp(in_off), n,
                                          _dp(out), out.numel(), _dp(out_len), _dp(status), _stream(stream)),
           "hhuff_encode_batch_multi")
    return out, out_len, status


def packed_positions(in_off, out_len, decode):
    """Where the packed layout put each string when out_off was not returned: tile t = i // 64 starts at its slot
    position (decode floor(8 in_off[64 t] / 5), encode in_off[64 t]) and its strings follow back to back; failed
    strings (HHUFF_FAIL_LEN) take no bytes.  Returns int64 starts[n]"""
    in_off = np.asarray(in_off, np.int64)
    ln = np.asarray(out_len, np.uint32)
    n = ln.size
    kept = np.where(ln == FAIL_LEN, 0, ln).astype(np.int64)
    t0 = np.arange(0, n, 64)
    base = in_off[t0] * 8 // 5 if decode else in_off[t0]
    cs = np.cumsum(kept) - kept                                  # exclusive prefix over the batch
    return np.repeat(base - cs[t0], np.diff(np.append(t0, n))) + cs


def decode_prices(device=0):
    """the staged / stream prices (ps per string, per byte, each kernel) the mixed-length decode of `device`
    uses (include/hhuff.h hhuff_decode_prices: fitted defaults until calibrated or pinned; no GPU work)"""
    buf = (ctypes.c_float * 4)()
    _check(lib().hhuff_decode_prices(device, buf), "hhuff_decode_prices")
    return [float(x) for x in buf]


def calibrate_decode_prices(device=0):
    """measure `device`'s prices now and use them from then on (hhuff_calibrate_decode_prices; synchronous)"""
    buf = (ctypes.c_float * 4)()
    _check(lib().hhuff_calibrate_decode_prices(device, buf), "hhuff_calibrate_decode_prices")
    return [float(x) for x in buf]


def set_decode_prices(prices, device=0):
    """pin `device`'s prices (4 floats), or restore the fitted defaults with None (hhuff_set_decode_prices)"""
    buf = None if prices is None else (ctypes.c_float * 4)(*[float(x) for x in prices])
    _check(lib().hhuff_set_decode_prices(device, buf), "hhuff_set_decode_prices")


def set_edge_defer_min(n):
    """batches of at least n strings defer their tiles' shared 16-B chunks to edge records and a fix-up kernel
    (hhuff_set_edge_defer_min; default 2^32 - 1: never); returns the previous threshold"""
    return int(lib().hhuff_set_edge_defer_min(int(n)))


def set_decode_kernel(mode):
    """which kernel decodes contiguous batches (hhuff_set_decode_kernel): 0 (default) the staged / stream choice;
    1 / 2 (the segment kernel above a 40-B mean / always) only in A/B builds (HhuffError here); returns the
    previous mode"""
    r = lib().hhuff_set_decode_kernel(int(mode))
    if r < 0:
        _check(r, "hhuff_set_decode_kernel")
    return r
