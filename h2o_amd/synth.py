"""Seeded synthetic header-string batches for the benchmark configurations.

Alphabet: bytes 0x20..0x7E drawn with P(c) ~ 2^-nbits(c) -- the distribution the RFC 7541 code is tuned
for (E[nbits] ~ 6.0, Huffman/plain ~ 0.75).  Config 5 uses the cookie/URI charset
[A-Za-z0-9-_=;%&/?.] uniformly.  A fraction of adversarial strings (control bytes, 0x80+, 8-bit-code-only
strings, leading/trailing SP/HT) makes the SIZE_MAX and soft-error paths run.

A batch is the include/hhuff.h layout: packed bytes + u32 offsets [n+1] + an is_name bitmask.
numpy generators serve the CPU tests; `*_torch` generators build the same distributions on the GPU
for bench.py (no host round trip for 16M strings).
"""
import numpy as np

from . import tables

COOKIE_CHARSET = np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_=;%&/?.", np.uint8)

CONFIGS = {
    # name: (n, length sampler, alphabet)
    "c2": dict(n=1 << 20, lengths=("uniform", 16, 48), alphabet="header"),
    "c3": dict(n=1 << 20, lengths=("zipf", 8, 512), alphabet="header"),
    "c4": dict(n=1 << 24, lengths=("uniform", 24, 72), alphabet="header"),
    "c5": dict(n=1 << 19, lengths=("uniform", 256, 768), alphabet="cookie"),
}


def header_alphabet():
    """(symbols u8[95], probabilities f64[95]) for 0x20..0x7E with P ~ 2^-nbits."""
    nbits = np.asarray(tables.ENC_NBITS, dtype=np.float64)
    syms = np.arange(0x20, 0x7F, dtype=np.uint8)
    p = 2.0 ** -nbits[syms]
    return syms, p / p.sum()


def _lengths(rng, n, spec):
    kind, lo, hi = spec
    if kind == "uniform":
        return rng.integers(lo, hi + 1, size=n, dtype=np.int64)
    if kind == "zipf":
        L = np.arange(lo, hi + 1, dtype=np.float64)
        p = 1.0 / L
        return rng.choice(np.arange(lo, hi + 1), size=n, p=p / p.sum()).astype(np.int64)
    raise ValueError(kind)


def pack(strings):
    """list[bytes] -> (data u8[], off u32[n+1])"""
    off = np.zeros(len(strings) + 1, np.uint32)
    off[1:] = np.cumsum([len(s) for s in strings], dtype=np.uint64)
    data = np.frombuffer(b"".join(strings), np.uint8).copy() if strings else np.zeros(0, np.uint8)
    return data, off


def unpack(data, off, n=None, lens=None):
    n = len(off) - 1 if n is None else n
    if lens is None:
        return [bytes(data[off[i]:off[i + 1]]) for i in range(n)]
    return [bytes(data[off[i]:off[i] + lens[i]]) for i in range(n)]


def bits_from_bools(flags):
    flags = np.asarray(flags, dtype=bool)
    words = np.zeros((len(flags) + 31) // 32, np.uint32)
    idx = np.nonzero(flags)[0]
    np.bitwise_or.at(words, idx >> 5, (np.uint32(1) << (idx & 31).astype(np.uint32)))
    return words


def adversarial(rng, n_max_len=64):
    """One adversarial plain string."""
    kind = rng.integers(0, 7)
    L = int(rng.integers(0, n_max_len + 1))
    if kind == 0:  # control bytes and DEL
        s = rng.integers(0, 0x20, size=L).astype(np.uint8)
        if L:
            s[rng.integers(0, L)] = 0x7F
    elif kind == 1:  # high bytes
        s = rng.integers(0x80, 0x100, size=L).astype(np.uint8)
    elif kind == 2:  # 8-bit codes only ('X' is 8 bits: never compressible)
        s = np.full(L, ord("X"), np.uint8)
    elif kind == 3:  # leading / trailing whitespace
        syms, p = header_alphabet()
        s = rng.choice(syms, size=max(L, 1), p=p)
        s[0 if rng.integers(0, 2) else -1] = rng.choice([0x20, 0x09])
    elif kind == 4:  # upper case (invalid in names)
        s = rng.integers(ord("A"), ord("Z") + 1, size=L).astype(np.uint8)
    elif kind == 5:  # ':'-prefixed pseudo-header-like
        syms, p = header_alphabet()
        s = rng.choice(syms, size=max(L, 1), p=p)
        s[0] = ord(":")
    else:  # any byte
        s = rng.integers(0, 256, size=L).astype(np.uint8)
    return bytes(s)


def make_batch(config, n=None, seed=0, adversarial_frac=0.01, name_frac=0.3):
    """numpy batch for a named config (or a dict spec); returns dict(data, off, is_name_bits, n)."""
    spec = CONFIGS[config] if isinstance(config, str) else config
    n = spec["n"] if n is None else n
    rng = np.random.default_rng(seed)
    lens = _lengths(rng, n, spec["lengths"])
    if spec["alphabet"] == "header":
        syms, p = header_alphabet()
        flat = rng.choice(syms, size=int(lens.sum()), p=p)
    else:
        flat = rng.choice(COOKIE_CHARSET, size=int(lens.sum()))
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    strings = [flat[off[i]:off[i + 1]].tobytes() for i in range(n)]
    n_adv = int(round(n * adversarial_frac))
    for i in rng.choice(n, size=n_adv, replace=False) if n_adv else []:
        strings[i] = adversarial(rng)
    data, off32 = pack(strings)
    is_name = rng.random(n) < name_frac
    return dict(data=data, off=off32, is_name_bits=bits_from_bools(is_name), n=n, seed=seed)


# ------------------------------------------------------------------------------------------------
# GPU-side generation (bench.py): the same distributions, built with torch on the device.
# ------------------------------------------------------------------------------------------------
def make_batch_torch(config, n=None, seed=0, device="cuda", adversarial_frac=0.01, name_frac=0.3):
    """Device-resident batch: dict(data u8, off i32->u32 view, is_name_bits i32, n).

    Adversarial strings are produced by overwriting a random 1% of strings' bytes with bytes drawn
    uniformly from 0..255 (control, DEL, 0x80+: SIZE_MAX and soft-error paths)."""
    import torch

    spec = CONFIGS[config] if isinstance(config, str) else config
    n = spec["n"] if n is None else n
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    kind, lo, hi = spec["lengths"]
    if kind == "uniform":
        lens = torch.randint(lo, hi + 1, (n,), generator=g, device=device, dtype=torch.int64)
    else:
        L = torch.arange(lo, hi + 1, device=device, dtype=torch.float64)
        lens = torch.multinomial(1.0 / L, n, replacement=True, generator=g) + lo
        if kind == "zipf_desc":  # ablation (tools/ab.py): the same lengths, longest first
            lens = torch.sort(lens, descending=True).values
    off = torch.zeros(n + 1, dtype=torch.int64, device=device)
    off[1:] = torch.cumsum(lens, 0)
    total = int(off[-1].item())
    assert total < 2 ** 32, "batch larger than the u32 offset space"
    if spec["alphabet"] == "header":
        syms, p = header_alphabet()
        cdf = torch.tensor(np.cumsum(p), device=device, dtype=torch.float32)
        cdf[-1] = 1.0
        u = torch.rand(total, generator=g, device=device)
        idx = torch.searchsorted(cdf, u).clamp_(max=len(syms) - 1)
        data = torch.tensor(syms, device=device)[idx]
    else:
        cs = torch.tensor(COOKIE_CHARSET, device=device)
        data = cs[torch.randint(0, len(cs), (total,), generator=g, device=device)]
    n_adv = int(n * adversarial_frac)
    if n_adv:
        pick = torch.randperm(n, generator=g, device=device)[:n_adv]
        # mark the bytes of the picked strings and overwrite them with uniform random bytes
        mark = torch.zeros(total + 1, dtype=torch.int32, device=device)
        mark.index_add_(0, off[pick], torch.ones(n_adv, dtype=torch.int32, device=device))
        mark.index_add_(0, off[pick + 1], -torch.ones(n_adv, dtype=torch.int32, device=device))
        sel = torch.cumsum(mark[:-1], 0) > 0
        rnd = torch.randint(0, 256, (total,), generator=g, device=device, dtype=torch.int32).to(torch.uint8)
        data = torch.where(sel, rnd, data)
    is_name = torch.rand(n, generator=g, device=device) < name_frac
    nw = (n + 31) // 32
    pad = torch.zeros(nw * 32, dtype=torch.int64, device=device)
    pad[:n] = is_name.to(torch.int64)
    weights = (torch.ones(32, dtype=torch.int64, device=device) << torch.arange(32, device=device))
    words = (pad.view(nw, 32) * weights).sum(1)
    words = torch.where(words >= 2 ** 31, words - 2 ** 32, words).to(torch.int32)
    return dict(data=data.contiguous(), off=off.to(torch.int64), is_name_bits=words.contiguous(), n=n, total=total)
