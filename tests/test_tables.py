"""Generated tables: freshness, canonical-code properties, LUT / long-code decode vs the code tree."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_tables as G  # noqa: E402


def test_generated_headers_are_fresh():
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_tables.py"), "--check"], check=True)


def test_canonical_code_properties():
    lens = G.code_lengths()
    codes, order = G.canonical_codes(lens)
    # RFC 7541 Appendix B spot checks
    assert (codes[ord("0")], lens[ord("0")]) == (0x0, 5)
    assert (codes[ord("a")], lens[ord("a")]) == (0x3, 5)
    assert (codes[ord("X")], lens[ord("X")]) == (0xFC, 8)
    assert (codes[0], lens[0]) == (0x1FF8, 13)
    assert (codes[256], lens[256]) == (0x3FFFFFFF, 30)
    assert min(lens) == 5 and max(lens) == 30
    # prefix-free
    words = sorted(format(codes[s], "0%db" % lens[s]) for s in range(257))
    assert all(not b.startswith(a) for a, b in zip(words, words[1:]))


def _tree_decode(bits, root):
    out, node, last_end = [], root, 0
    for i, b in enumerate(bits):
        node = node[int(b)]
        if not isinstance(node, dict):
            out.append((node, i + 1 - last_end))
            last_end = i + 1
            node = root
    return out


def test_window_lut_matches_tree():
    lens = G.code_lengths()
    codes, _ = G.canonical_codes(lens)
    root = G.build_tree(lens, codes)
    lut = G.window_lut(root)
    for w in range(1 << G.LUT_BITS):
        e = lut[w]
        syms = _tree_decode(format(w, "0%db" % G.LUT_BITS), root)
        if not syms:
            assert e >> 31 and (e >> 8) & 15 == G.LUT_BITS + 1 and (e >> 12) & 15 == 0
            assert (e >> 28) & 3 == 0
            continue
        assert not e >> 31
        assert (e >> 28) & 3 == min(len(syms), 2)
        s1, l1 = syms[0]
        assert e & 0xFF == s1 and (e >> 8) & 15 == l1
        assert (e >> 24) & 1 == (s1 not in G.NAME_VALID) and (e >> 25) & 1 == (s1 not in G.VALUE_VALID)
        if len(syms) > 1:
            s2, l2 = syms[1]
            assert (e >> 30) & 1 and (e >> 16) & 0xFF == s2 and (e >> 12) & 15 == l1 + l2
            assert (e >> 26) & 1 == (s2 not in G.NAME_VALID) and (e >> 27) & 1 == (s2 not in G.VALUE_VALID)
        else:
            assert not (e >> 30) & 1 and (e >> 12) & 15 == l1 and not (e >> 26) & 3


def test_long_code_tables_decode_every_symbol():
    lens = G.code_lengths()
    codes, order = G.canonical_codes(lens)
    L_out, lim1, first, base = G.long_tables(lens, codes, order)
    for s in range(257):
        t = (codes[s] << (32 - lens[s])) | ((1 << (32 - lens[s])) - 1 if s % 2 else 0)
        j = next(k for k in range(len(L_out)) if t <= lim1[k])
        L = L_out[j]
        assert L == lens[s]
        assert order[base[j] + (t >> (32 - L)) - first[j]] == s


def test_nibble_fsm_against_reference_table():
    """Our FSM equals the reference's generated table entry for entry (only where the reference exists)."""
    import re

    path = "/root/reference/lib/http2/hpack_huffman_table.h"
    if not os.path.exists(path):
        pytest.skip("reference tree not present (GPU box)")
    src = open(path).read()
    ent = re.findall(r"\{(\d+), 0x([0-9a-f]+), (\d+)\}", src[src.index("huff_decode_table"):])
    lens = G.code_lengths()
    codes, _ = G.canonical_codes(lens)
    fsm = G.nibble_fsm(G.build_tree(lens, codes))
    assert len(ent) == 4096
    for i, (st, fl, sy) in enumerate(ent):
        v = fsm[i // 16][i % 16]
        assert (v & 0xFF, (v >> 8) & 0xFF, v >> 16) == (int(st), int(fl, 16), int(sy))
    sym = re.findall(r"\{(\d+), 0x([0-9a-f]+)u\}", src)
    assert [(int(a), int(b, 16)) for a, b in sym] == list(zip(lens, codes))
