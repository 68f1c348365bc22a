"""Multi-GPU batch sharding for the hhuff codec: one process per GPU, torch.distributed (RCCL over xGMI
on MI355X nodes, gloo for CPU tests).

Strings are independent, so a batch shards with no reduction:
  * byte-balanced contiguous shards: string-index ranges cut at quantiles of the byte prefix sum, so
    every rank gets about the same number of bytes; each shard's offsets are rebased to 0;
  * when the batch starts on one rank, `scatter_batch` moves each shard to its rank (point-to-point
    send/recv of the packed bytes, offsets and is-name bits);
  * `gather_results` concatenates per-shard results in shard order on the root after an all_gather of
    per-shard sizes, giving byte-for-byte the single-GPU result (compacted form: out_len, status and the
    successful strings' bytes back to back).
The benchmark itself runs independent per-rank shards (weak scaling): the data path has no collective.
The per-shard codec is a parameter so the data movement is testable on CPU (tests/test_dist.py).
"""
import numpy as np
import torch
import torch.distributed as dist

FAIL = 0xFFFFFFFF


def byte_balanced_bounds(off, world):
    """String-index bounds [b_0 = 0, ..., b_world = n] cutting the byte prefix sum `off` (n+1 entries)
    at its 1/world quantiles."""
    off = np.asarray(off, dtype=np.int64)
    n = len(off) - 1
    total = int(off[-1] - off[0])
    targets = off[0] + (np.arange(world + 1, dtype=np.float64) * total / world)
    b = np.searchsorted(off, targets, side="left").astype(np.int64)
    b[0], b[-1] = 0, n
    return np.maximum.accumulate(np.clip(b, 0, n))


def _bits_to_bool(bits, n):
    return np.unpackbits(np.asarray(bits, np.uint32).view(np.uint8), bitorder="little")[:n].astype(bool)


def _bool_to_bits(flags):
    flags = np.asarray(flags, dtype=bool)
    words = np.zeros((len(flags) + 31) // 32, np.uint32)
    idx = np.nonzero(flags)[0]
    np.bitwise_or.at(words, idx >> 5, (np.uint32(1) << (idx & 31).astype(np.uint32)))
    return words


def shard(batch, lo, hi):
    """Shard [lo, hi) of a host batch dict(data, off, is_name_bits?) with offsets rebased to 0."""
    off = np.asarray(batch["off"], dtype=np.int64)
    b0, b1 = int(off[lo]), int(off[hi])
    out = dict(data=np.ascontiguousarray(batch["data"][b0:b1]), off=(off[lo:hi + 1] - b0).astype(np.uint32), n=hi - lo)
    if batch.get("is_name_bits") is not None:
        names = _bits_to_bool(batch["is_name_bits"], len(off) - 1)[lo:hi]
        out["is_name_bits"] = _bool_to_bits(names)
    return out


def _send(t, dst, group):
    dist.send(t.contiguous(), dst, group=group)


def _recv(shape, dtype, src, device, group):
    t = torch.empty(shape, dtype=dtype, device=device)
    dist.recv(t, src, group=group)
    return t


def scatter_batch(batch, root=0, group=None, device="cpu"):
    """Move byte-balanced shards of `batch` (a host dict on `root`, ignored elsewhere) to every rank.
    Returns this rank's shard as a host dict (data, off, is_name_bits, n)."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if rank == root:
        bounds = byte_balanced_bounds(batch["off"], world)
        shards = [shard(batch, int(bounds[r]), int(bounds[r + 1])) for r in range(world)]
        meta = torch.tensor([[s["n"], len(s["data"])] for s in shards], dtype=torch.int64, device=device)
    else:
        meta = torch.empty((world, 2), dtype=torch.int64, device=device)
    dist.broadcast(meta, root, group=group)
    n_me, bytes_me = (int(x) for x in meta[rank].tolist())
    if rank == root:
        for r in range(world):
            if r == root:
                continue
            s = shards[r]
            _send(torch.from_numpy(s["data"]).to(device), r, group)
            _send(torch.from_numpy(s["off"].view(np.int32)).to(device), r, group)
            _send(torch.from_numpy(s["is_name_bits"].view(np.int32)).to(device), r, group)
        return shards[root]
    data = _recv((bytes_me,), torch.uint8, root, device, group).cpu().numpy()
    off = _recv((n_me + 1,), torch.int32, root, device, group).cpu().numpy().view(np.uint32)
    bits = _recv(((n_me + 31) // 32,), torch.int32, root, device, group).cpu().numpy().view(np.uint32)
    return dict(data=data, off=off, is_name_bits=bits, n=n_me)


def compact_results(out, out_off, out_len, status):
    """(out_len, status, successful strings back to back) from a slot-layout result."""
    out_len = np.asarray(out_len, np.uint32)
    parts = [out[int(o):int(o) + int(L)] for o, L in zip(out_off, out_len) if L != FAIL]
    data = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return out_len, np.asarray(status, np.uint8), data


def gather_results(out_len, status, data, root=0, group=None, device="cpu"):
    """Concatenate per-shard compacted results on `root` in shard (= string) order.  An all_gather of
    the per-shard sizes gives every rank the global layout; payloads go to the root point-to-point."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    sizes = torch.tensor([len(out_len), len(data)], dtype=torch.int64, device=device)
    all_sizes = [torch.empty_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    all_sizes = [tuple(int(v) for v in s.tolist()) for s in all_sizes]
    if rank != root:
        _send(torch.from_numpy(np.ascontiguousarray(out_len).view(np.int32)).to(device), root, group)
        _send(torch.from_numpy(np.ascontiguousarray(status)).to(device), root, group)
        _send(torch.from_numpy(np.ascontiguousarray(data)).to(device), root, group)
        return None
    lens, stats, datas = [], [], []
    for r in range(world):
        if r == root:
            lens.append(np.asarray(out_len, np.uint32))
            stats.append(np.asarray(status, np.uint8))
            datas.append(np.asarray(data, np.uint8))
            continue
        n_r, b_r = all_sizes[r]
        lens.append(_recv((n_r,), torch.int32, r, device, group).cpu().numpy().view(np.uint32))
        stats.append(_recv((n_r,), torch.uint8, r, device, group).cpu().numpy())
        datas.append(_recv((b_r,), torch.uint8, r, device, group).cpu().numpy())
    return np.concatenate(lens), np.concatenate(stats), np.concatenate(datas)


def decode_sharded(batch, decode_fn, root=0, group=None, device="cpu"):
    """Scatter `batch` from root, decode each shard with decode_fn(shard) -> (out, out_off, out_len, status),
    gather the compacted results on root (None elsewhere)."""
    local = scatter_batch(batch, root, group, device)
    out, out_off, out_len, status = decode_fn(local)
    return gather_results(*compact_results(out, out_off, out_len, status), root=root, group=group, device=device)
