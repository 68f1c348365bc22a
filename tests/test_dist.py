"""Multi-rank sharding on CPU (gloo, world_size 2 and 3): scatter a batch from rank 0 in byte-balanced
shards, decode every shard (the CPU oracle stands in for the per-rank HIP codec here), gather on rank 0,
and require byte-for-byte the single-process result."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from h2o_amd import dist as hd


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_decode(shard):
    from oracle import oracle as O

    o = O.oracle()
    n = shard["n"]
    out, out_len, status = o.decode_batch(shard["data"], shard["off"], n, is_name_bits=shard["is_name_bits"])
    out_off = (shard["off"][:n].astype(np.uint64) * 8) // 5
    return out, out_off, out_len, status


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from h2o_amd import synth

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        batch = synth.make_batch("c2", n=5000, seed=31, adversarial_frac=0.05) if rank == 0 else None
        res = hd.decode_sharded(batch, _oracle_decode, root=0)
        if rank == 0:
            q.put(tuple(np.asarray(x).tobytes() for x in res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_scatter_decode_gather_matches_single_process(world):
    from h2o_amd import synth
    from oracle import oracle as O

    O.build()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    batch = synth.make_batch("c2", n=5000, seed=31, adversarial_frac=0.05)
    full = {"data": batch["data"], "off": batch["off"], "is_name_bits": batch["is_name_bits"], "n": batch["n"]}
    ref = hd.compact_results(*_oracle_decode(full))
    assert got == tuple(np.asarray(x).tobytes() for x in ref)


def test_byte_balanced_bounds():
    off = np.cumsum(np.r_[0, np.full(1000, 48)])
    for world in (1, 2, 4, 8):
        b = hd.byte_balanced_bounds(off, world)
        assert b[0] == 0 and b[-1] == 1000 and (np.diff(b) >= 0).all()
        sizes = off[b[1:]] - off[b[:-1]]
        assert sizes.max() - sizes.min() <= 48
    # skewed lengths: one huge string
    off = np.cumsum(np.r_[0, [10] * 50, [100000], [10] * 50])
    b = hd.byte_balanced_bounds(off, 4)
    assert b[0] == 0 and b[-1] == 101 and (np.diff(b) >= 0).all()


def test_shard_rebases_offsets_and_names():
    from h2o_amd import synth

    batch = synth.make_batch("c2", n=300, seed=5)
    s = hd.shard(batch, 100, 250)
    assert s["off"][0] == 0 and s["n"] == 150
    assert bytes(s["data"]) == bytes(batch["data"][batch["off"][100]:batch["off"][250]])
    names = hd._bits_to_bool(batch["is_name_bits"], 300)[100:250]
    assert (hd._bits_to_bool(s["is_name_bits"], 150) == names).all()
