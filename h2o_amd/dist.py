"""Multi-GPU batch sharding for the hhuff codec: one process per GPU, torch.distributed (RCCL over xGMI on
MI355X nodes; gloo on CPU tensors for the tests).  Everything here is torch ops on the batch's own device:
with CUDA tensors nothing goes through host memory.

Strings are independent, so a batch shards with no reduction:
  * `byte_balanced_bounds`: string-index ranges cut at the 1/world quantiles of the byte prefix sum, so
    every rank gets about the same number of bytes;
  * `shard`: one such range with offsets rebased to 0 and the is-name bits re-packed;
  * `scatter_batch`: when the batch starts on one rank, point-to-point send/recv of each shard (packed
    bytes, offsets, name bits) -- the optional device-to-device leg of config 4;
  * `exchange_sizes`: an all_gather of each shard's (strings, output bytes) -- the one collective the
    batch split needs: it gives every rank the global output offset of its shard;
  * `gather_results`: per-shard results concatenated in shard order on the root, byte for byte the
    single-GPU result.
The per-shard codec is a parameter (`decode_sharded`), so the data movement is testable on CPU.
"""
import torch
import torch.distributed as dist

FAIL = 0xFFFFFFFF


def _default_device(group=None):
    """the tensors' device for the process group's backend: this rank's GPU for RCCL, else the CPU"""
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def byte_balanced_bounds(off, world):
    """String-index bounds [b_0 = 0, ..., b_world = n] (int64 tensor on off's device) cutting the byte prefix
    sum `off` (n+1 entries, any integer dtype; u32 values carried in int32 are read as unsigned) at its
    1/world quantiles."""
    off = torch.as_tensor(off)
    o = off.to(torch.int64) & 0xFFFFFFFF if off.dtype == torch.int32 else off.to(torch.int64)
    n = o.numel() - 1
    total = o[-1] - o[0]
    k = torch.arange(world + 1, device=o.device, dtype=torch.int64)
    targets = o[0] + torch.div(k * total, world, rounding_mode="floor")
    b = torch.searchsorted(o, targets, side="left").clamp_(0, n)
    b[0], b[-1] = 0, n
    return torch.cummax(b, 0).values


def bits_to_bool(bits, n):
    """u32 bitmask words (int32 tensor) -> bool[n]"""
    w = bits.to(torch.int64) & 0xFFFFFFFF
    sh = torch.arange(32, device=bits.device, dtype=torch.int64)
    return ((w.unsqueeze(1) >> sh) & 1).reshape(-1)[:n].to(torch.bool)


def bool_to_bits(flags):
    """bool[n] -> u32 bitmask words carried in an int32 tensor"""
    n = flags.numel()
    nw = (n + 31) // 32
    pad = torch.zeros(nw * 32, dtype=torch.int64, device=flags.device)
    pad[:n] = flags.to(torch.int64)
    w = (pad.view(nw, 32) << torch.arange(32, device=flags.device, dtype=torch.int64)).sum(1)
    return torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32)


def shard(batch, lo, hi):
    """Strings [lo, hi) of batch dict(data u8, off int64|int32 [n+1], is_name_bits int32 | None) with offsets
    rebased to 0 (int32 carrying u32) and the name bits re-packed; tensors stay on their device."""
    off = batch["off"]
    o = off.to(torch.int64) & 0xFFFFFFFF if off.dtype == torch.int32 else off.to(torch.int64)
    b0, b1 = int(o[lo]), int(o[hi])
    # a fresh allocation: the codec wants its input 16-byte aligned, a slice view starts anywhere
    out = dict(data=batch["data"][b0:b1].clone(), off=(o[lo:hi + 1] - b0).to(torch.int32), n=hi - lo)
    names = batch.get("is_name_bits")
    out["is_name_bits"] = (bool_to_bits(bits_to_bool(names, int(o.numel()) - 1)[lo:hi]) if names is not None
                           else torch.zeros((hi - lo + 31) // 32, dtype=torch.int32, device=off.device))
    return out


def scatter_batch(batch, root=0, group=None, device=None):
    """Move byte-balanced shards of `batch` (a dict of tensors on `root`, ignored elsewhere) to every rank.
    A batch without name bits ships all-zero bits.  Returns this rank's shard (tensors on `device`)."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = torch.device(device) if device is not None else _default_device(group)
    if rank == root:
        bounds = byte_balanced_bounds(batch["off"], world).tolist()
        shards = [shard(batch, bounds[r], bounds[r + 1]) for r in range(world)]
        meta = torch.tensor([[s["n"], s["data"].numel()] for s in shards], dtype=torch.int64, device=dev)
    else:
        meta = torch.empty((world, 2), dtype=torch.int64, device=dev)
    dist.broadcast(meta, root, group=group)
    if rank == root:
        for r in range(world):
            if r != root:
                for key in ("data", "off", "is_name_bits"):
                    dist.send(shards[r][key].to(dev).contiguous(), r, group=group)
        mine = shards[root]
        return {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in mine.items()}
    n_me, bytes_me = (int(x) for x in meta[rank].tolist())
    out = dict(data=torch.empty(bytes_me, dtype=torch.uint8, device=dev),
               off=torch.empty(n_me + 1, dtype=torch.int32, device=dev),
               is_name_bits=torch.empty((n_me + 31) // 32, dtype=torch.int32, device=dev), n=n_me)
    for key in ("data", "off", "is_name_bits"):
        dist.recv(out[key], root, group=group)
    return out


def exchange_sizes_async(n_strings, out_bytes, group=None, device=None):
    """exchange_sizes issued asynchronously: returns (work, parts).  With RCCL the all_gather runs on the
    collective's own stream once the work queued before it (the kernel that produced `out_bytes`) is done,
    so kernels launched after it on the compute stream overlap it; work.wait() makes the compute stream
    wait for it (no host block).  torch.stack(parts) then gives the sizes."""
    dev = torch.device(device) if device is not None else _default_device(group)
    mine = torch.stack([torch.as_tensor(n_strings, dtype=torch.int64, device=dev),
                        torch.as_tensor(out_bytes, dtype=torch.int64, device=dev).reshape(())])
    parts = [torch.empty(2, dtype=torch.int64, device=dev) for _ in range(dist.get_world_size(group))]
    return dist.all_gather(parts, mine, group=group, async_op=True), parts


def exchange_sizes(n_strings, out_bytes, group=None, device=None):
    """all_gather of every shard's (strings, output bytes): returns (sizes int64 [world, 2], this shard's
    global string index and global output byte offset).  `out_bytes` may be a device tensor (a sum the
    codec left on the device): the exchange then needs no host round trip."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = torch.device(device) if device is not None else _default_device(group)
    mine = torch.stack([torch.as_tensor(n_strings, dtype=torch.int64, device=dev),
                        torch.as_tensor(out_bytes, dtype=torch.int64, device=dev).reshape(())])
    parts = [torch.empty(2, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    sizes = torch.stack(parts)
    before = sizes[:rank].sum(0)
    return sizes, before[0], before[1]


def compact_results(out, out_off, out_len):
    """successful outputs back to back: (out_len u32 as int64, bytes) from any layout with per-string offsets"""
    ol = out_len.to(torch.int64) & 0xFFFFFFFF
    keep = torch.where(ol != FAIL, ol, torch.zeros_like(ol))
    tot = int(keep.sum())
    oo = out_off.to(torch.int64) & 0xFFFFFFFF if out_off.dtype == torch.int32 else out_off.to(torch.int64)
    start = torch.repeat_interleave(oo[:ol.numel()], keep)
    rel = torch.arange(tot, device=out.device) - torch.repeat_interleave(torch.cumsum(keep, 0) - keep, keep)
    return ol, out[start + rel]


def gather_results(out_len, status, data, root=0, group=None):
    """Concatenate per-shard compacted results on `root` in shard (= string) order: an all_gather of the
    per-shard sizes gives every rank the global layout; payloads go to the root point-to-point.
    Returns (out_len int64, status u8, bytes) on root, None elsewhere."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = data.device
    sizes, _, _ = exchange_sizes(out_len.numel(), data.numel(), group=group, device=dev)
    if rank != root:
        dist.send(out_len.to(torch.int64).contiguous(), root, group=group)
        dist.send(status.contiguous(), root, group=group)
        dist.send(data.contiguous(), root, group=group)
        return None
    lens, stats, datas = [], [], []
    for r in range(world):
        if r == root:
            lens.append(out_len.to(torch.int64))
            stats.append(status)
            datas.append(data)
            continue
        n_r, b_r = (int(x) for x in sizes[r].tolist())
        L = torch.empty(n_r, dtype=torch.int64, device=dev)
        S = torch.empty(n_r, dtype=torch.uint8, device=dev)
        D = torch.empty(b_r, dtype=torch.uint8, device=dev)
        dist.recv(L, r, group=group)
        dist.recv(S, r, group=group)
        dist.recv(D, r, group=group)
        lens.append(L), stats.append(S), datas.append(D)
    return torch.cat(lens), torch.cat(stats), torch.cat(datas)


def decode_sharded(batch, decode_fn, root=0, group=None, device=None):
    """Scatter `batch` from root, decode each shard with decode_fn(shard) -> (out, out_off, out_len, status) --
    the layout of hhuff_decode_batch_packed -- and gather the compacted results on root (None elsewhere)."""
    local = scatter_batch(batch, root, group, device)
    out, out_off, out_len, status = decode_fn(local)
    ol, data = compact_results(out, out_off, out_len)
    return gather_results(ol, status, data, root=root, group=group)
