"""Multi-rank sharding (h2o_amd/dist.py) on CPU tensors over gloo, world sizes 2 and 3: scatter a batch from
rank 0 in byte-balanced shards, run the per-rank codec, all_gather the shard sizes, gather on rank 0, and
require byte-for-byte the single-process result.  The per-rank codec keeps the contract of
hhuff_decode_batch_packed (out, out_off, out_len, status); with no GPU here the CPU restatement computes it
(on a GPU node dist.py runs the same code on CUDA tensors over RCCL: bench.py --gpus N)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from h2o_amd import dist as hd


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_decode(shard):
    """hhuff_decode_batch_packed's contract on CPU tensors, computed by the restatement (slot places)"""
    from oracle import oracle as O

    n = shard["n"]
    data = shard["data"].numpy()
    off = shard["off"].numpy().view(np.uint32)
    names = shard["is_name_bits"].numpy().view(np.uint32)
    out, out_len, status = O.oracle().decode_batch(data, off, n, is_name_bits=names)
    out_off = ((off.astype(np.uint64) * 8) // 5).astype(np.int64)
    return (torch.from_numpy(out), torch.from_numpy(out_off), torch.from_numpy(out_len.astype(np.int64)),
            torch.from_numpy(status))


def _gpu_decode(shard):
    """the library's hhuff_decode_batch_packed on this rank's GPU; results back on the CPU for gloo"""
    from h2o_amd import codec

    n = shard["n"]
    d = shard["data"].cuda()
    out, out_off, out_len, status = codec.decode_batch_packed(d, shard["off"].cuda(), n,
                                                              is_name_bits=shard["is_name_bits"].cuda(),
                                                              in_size=int(d.numel()))
    torch.cuda.synchronize()
    return out.cpu(), out_off[:n].cpu(), out_len[:n].cpu(), status[:n].cpu()


def _tensors(b):
    return dict(data=torch.from_numpy(b["data"]), off=torch.from_numpy(b["off"].view(np.int32)),
                is_name_bits=torch.from_numpy(b["is_name_bits"].view(np.int32)), n=b["n"])


def _worker(rank, world, port, q, with_names, gpu=False):
    import torch.distributed as dist

    from h2o_amd import synth

    if gpu:
        torch.cuda.set_device(rank % torch.cuda.device_count())

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        batch = None
        if rank == 0:
            batch = _tensors(synth.make_batch("c2", n=5000, seed=31, adversarial_frac=0.05))
            if not with_names:
                batch["is_name_bits"] = None
        res = hd.decode_sharded(batch, _gpu_decode if gpu else _oracle_decode, root=0, device="cpu")
        # the size exchange alone: every rank learns its shard's global string index and output offset
        local = torch.tensor([rank + 1, 10 * (rank + 1)])
        sizes, first, obase = hd.exchange_sizes(local[0], local[1])
        exp = sum(r + 1 for r in range(rank)), sum(10 * (r + 1) for r in range(rank))
        assert (int(first), int(obase)) == exp and sizes.shape == (world, 2)
        # the asynchronous form bench.py overlaps with the decode: same sizes once waited for
        work, parts = hd.exchange_sizes_async(local[0], local[1])
        work.wait()
        assert torch.equal(torch.stack(parts), sizes)
        if rank == 0:
            q.put(tuple(np.asarray(x).tobytes() for x in res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,with_names", [(2, True), (3, True), (2, False)])
def test_scatter_decode_gather_matches_single_process(world, with_names):
    from h2o_amd import synth
    from oracle import oracle as O

    O.build()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, with_names)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = _tensors(synth.make_batch("c2", n=5000, seed=31, adversarial_frac=0.05))
    if not with_names:
        full["is_name_bits"] = torch.zeros_like(full["is_name_bits"])
    out, out_off, out_len, status = _oracle_decode(full)
    ol, data = hd.compact_results(out, out_off, out_len)
    assert got == tuple(np.asarray(x).tobytes() for x in (ol, status, data))


def test_byte_balanced_bounds():
    off = torch.cumsum(torch.tensor([0] + [48] * 1000), 0)
    for world in (1, 2, 4, 8):
        b = hd.byte_balanced_bounds(off, world)
        assert int(b[0]) == 0 and int(b[-1]) == 1000 and bool((b[1:] >= b[:-1]).all())
        sizes = off[b[1:]] - off[b[:-1]]
        assert int(sizes.max() - sizes.min()) <= 48
    off = torch.cumsum(torch.tensor([0] + [10] * 50 + [100000] + [10] * 50), 0)  # one huge string
    b = hd.byte_balanced_bounds(off, 4)
    assert int(b[0]) == 0 and int(b[-1]) == 101 and bool((b[1:] >= b[:-1]).all())
    # u32 offsets carried in int32 (bit 31 set) are read as unsigned
    big = torch.tensor([0, 3 << 30, (3 << 30) + 10], dtype=torch.int64)
    assert hd.byte_balanced_bounds(big.to(torch.int32), 2).tolist() == hd.byte_balanced_bounds(big, 2).tolist()


def test_shard_rebases_offsets_and_names():
    from h2o_amd import synth

    b = synth.make_batch("c2", n=300, seed=5)
    t = _tensors(b)
    s = hd.shard(t, 100, 250)
    assert int(s["off"][0]) == 0 and s["n"] == 150
    assert bytes(s["data"].numpy()) == bytes(b["data"][b["off"][100]:b["off"][250]])
    names = hd.bits_to_bool(t["is_name_bits"], 300)[100:250]
    assert bool((hd.bits_to_bool(s["is_name_bits"], 150) == names).all())
    t["is_name_bits"] = None  # an encode batch: no name bits -> zero bits, no KeyError
    assert int(hd.shard(t, 10, 50)["is_name_bits"].abs().sum()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_ranks_decode_on_the_gpu(world):
    """the same scatter / per-rank decode / gather with the per-rank codec being libhhuff.so's
    hhuff_decode_batch_packed on the GPU (every rank on cuda:0 of a one-GPU box), collectives over gloo"""
    from h2o_amd import synth

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, True, True)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = _tensors(synth.make_batch("c2", n=5000, seed=31, adversarial_frac=0.05))
    out, out_off, out_len, status = _oracle_decode(full)
    ol, data = hd.compact_results(out, out_off, out_len)
    assert got == tuple(np.asarray(x).tobytes() for x in (ol, status, data))
