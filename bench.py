#!/usr/bin/env python3
"""hhuff benchmark -- BASELINE.json metric "GiB/s device-resident Huffman decode+encode, 16M header strings
mean 48B" on configuration 4 (16M strings, lengths U[24,72], header alphabet), one MI355X per rank.

One step = one pass of the hot path over one batch, inputs resident in HBM:
    encode  all N plain strings         (hhuff_encode_batch, h2o_hpack_encode_huffman per element)
    decode  the N_ok Huffman strings    (hhuff_decode_batch, h2o_hpack_decode_huffman per element)
            packed contiguously, i.e. the compressible strings as they would arrive on the wire
value = sum over ranks of plain bytes P / max over ranks of (t_encode + t_decode)   [GiB/s, 2^30]
Multi-GPU (torchrun, one process per GPU, RCCL): each rank owns an independent shard of N strings
(weak scaling); no collective on the data path, only barriers / a max-reduce of the timing.

Extra JSON fields: per-direction rates, `roofline` for the dominant kernel (decode; algorithmic bytes
B_dec = H + P_ok + 9 N_ok + 4 + ceil(N_ok / 8) per launch over its HIP-event duration), and
`cpu_baseline` (h2o's CPU path -- the reference's hpack.c compiled, or the restatement -- on this host's
cores, rank 0 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); measured copy peak ~6300
GIB = float(1 << 30)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4")
    ap.add_argument("--n", type=int, default=None, help="strings per rank (default: the config's N)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=0, help="strings in the CPU-baseline sample (0: the whole batch)")
    ap.add_argument("--cpu-threads", type=int, default=None)
    ap.add_argument("--only", choices=["encode", "decode"], default=None, help="profile one direction")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC passes for roofline.traffic")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-host", action="store_true", help="skip the H2D/D2H-inclusive measurement")
    return ap.parse_args()


def pmc_traffic(args):
    """HBM bytes per launch of each hhuff kernel from rocprofv3 PMC counters, one counter per pass
    (MI355X_MICROARCH.md HBM section): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
    reports half the bytes of a wide (16 B/lane) coalesced streaming read, the form of the kernels'
    input staging, so it is doubled.  Runs this script as a child of rocprofv3 BEFORE this process
    touches the GPU.  Returns {kernel: bytes} or {} when rocprofv3 is unavailable."""
    import csv
    import shutil
    import subprocess
    import tempfile

    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        return {}
    child = [sys.executable, os.path.abspath(__file__), "--pmc-child", "--steps", "2", "--warmup", "1",
             "--no-cpu-baseline", "--no-traffic", "--no-host", "--config", args.config]
    if args.n:
        child += ["--n", str(args.n)]
    vals = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="hhuff_pmc_")
        try:
            subprocess.run([exe, "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc", "--"] + child,
                           check=True, timeout=600, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           env=dict(os.environ, TMPDIR="/tmp"))
            for root, _, files in os.walk(d):
                for f in files:
                    if f.endswith("counter_collection.csv"):
                        for r in csv.DictReader(open(os.path.join(root, f))):
                            if "hhuff::" not in r["Kernel_Name"]:
                                continue
                            nm = r["Kernel_Name"]
                            k = "decode" if "decode" in nm else "encode" if "encode" in nm else "edge_fix" if "edge_fix" in nm else None
                            if k is None:
                                continue
                            vals.setdefault((k, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
        except Exception:
            return {}
        finally:
            shutil.rmtree(d, ignore_errors=True)
    out = {}
    for k in ("decode", "encode", "edge_fix"):
        f, w = vals.get((k, "FETCH_SIZE")), vals.get((k, "WRITE_SIZE"))
        if f and w:
            out[k] = (2.0 * sum(f) / len(f) + sum(w) / len(w)) * 1024.0
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    traffic = {}
    if not args.pmc_child and not args.no_traffic and world == 1:
        traffic = pmc_traffic(args)  # child processes; this process has not touched the GPU yet
    import numpy as np
    import torch
    import torch.distributed as dist

    from h2o_amd import codec, synth

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    codec.lib()

    # ---- synthetic batch, device resident -------------------------------------------------------
    b = synth.make_batch_torch(args.config, n=args.n, seed=1000 + rank)
    n = b["n"]
    P = int(b["total"])
    off32 = b["off"].to(torch.int32)
    lens = (b["off"][1:] - b["off"][:-1])
    enc_out = torch.empty(P + 16, dtype=torch.uint8, device="cuda")
    enc_len = torch.empty(n, dtype=torch.int32, device="cuda")
    enc_st = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.encode_batch(b["data"], off32, n, out=enc_out, out_len=enc_len, status=enc_st)
    # the wire: compressible strings, packed contiguously (second encode with explicit destinations)
    ok = enc_len != -1
    idx = torch.nonzero(ok).squeeze(1)
    n_ok = int(idx.numel())
    hl = enc_len[idx].to(torch.int64)
    h_off = torch.zeros(n_ok + 1, dtype=torch.int64, device="cuda")
    h_off[1:] = torch.cumsum(hl, 0)
    H = int(h_off[-1].item())
    huff = torch.empty(H + 16, dtype=torch.uint8, device="cuda")
    tmp_len = torch.empty(n_ok, dtype=torch.int32, device="cuda")
    codec.encode_batch(b["data"], off32[idx].contiguous(), n_ok, in_len=lens[idx].to(torch.int32).contiguous(),
                       out=huff, out_off=h_off[:-1].to(torch.int32).contiguous(), out_len=tmp_len, in_size=P)
    # is_name bits of the kept strings
    bits = ((b["is_name_bits"].to(torch.int64) & 0xFFFFFFFF).unsqueeze(1) >> torch.arange(32, device="cuda")) & 1
    names_ok = bits.reshape(-1)[:n][idx]
    nw = (n_ok + 31) // 32
    padn = torch.zeros(nw * 32, dtype=torch.int64, device="cuda")
    padn[:n_ok] = names_ok
    w = (padn.view(nw, 32) << torch.arange(32, device="cuda")).sum(1)
    names_bits = torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32).contiguous()
    h_off32 = h_off.to(torch.int32).contiguous()
    P_ok = int(hl.numel() and lens[idx].sum().item())
    dec_out = torch.empty(codec.decode_slot_size(H), dtype=torch.uint8, device="cuda")
    dec_len = torch.empty(n_ok, dtype=torch.int32, device="cuda")
    dec_st = torch.empty(n_ok, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    del tmp_len

    def run_encode():
        codec.encode_batch(b["data"], off32, n, out=enc_out, out_len=enc_len, status=enc_st, in_size=P)

    def run_decode():
        codec.decode_batch(huff, h_off32, n_ok, is_name_bits=names_bits, out=dec_out, out_len=dec_len, status=dec_st,
                           in_size=H)

    # correctness spot check before timing: decoded lengths equal the plain lengths of the kept strings
    run_decode()
    torch.cuda.synchronize()
    assert bool((dec_len == lens[idx].to(torch.int32)).all()), "decode does not invert encode"

    # ---- timed region ----------------------------------------------------------------------------
    do_enc = args.only in (None, "encode")
    do_dec = args.only in (None, "decode")
    for _ in range(args.warmup):
        if do_enc:
            run_encode()
        if do_dec:
            run_decode()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e0, e1, e2 in ev:
        e0.record()
        if do_enc:
            run_encode()
        e1.record()
        if do_dec:
            run_decode()
        e2.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t_wall = time.perf_counter() - t0
    t_enc = sorted(a.elapsed_time(b_) for a, b_, _ in ev)
    t_dec = sorted(b_.elapsed_time(c) for _, b_, c in ev)
    t_enc_avg = sum(t_enc) / len(t_enc)
    t_dec_avg = sum(t_dec) / len(t_dec)
    ms_step = t_wall * 1e3 / args.steps
    if world > 1:
        t = torch.tensor([ms_step], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms_step = float(t.item())
        tot = torch.tensor([P, P_ok, n, n_ok], device="cuda", dtype=torch.float64)
        dist.all_reduce(tot)
        P_all, P_ok_all, n_all, n_ok_all = (float(x) for x in tot.tolist())
    else:
        P_all, P_ok_all, n_all, n_ok_all = float(P), float(P_ok), float(n), float(n_ok)

    if rank == 0:
        B_dec = H + P_ok + 9 * n_ok + 4 + (n_ok + 7) // 8
        B_enc = P + int(hl.sum().item()) + 9 * n + 4
        dec_gbps = B_dec / (t_dec_avg * 1e-3) / 1e9
        enc_gbps = B_enc / (t_enc_avg * 1e-3) / 1e9
        dominant = "decode" if t_dec_avg >= t_enc_avg or args.only == "decode" else "encode"
        if args.only == "encode":
            dominant = "encode"
        ach = dec_gbps if dominant == "decode" else enc_gbps
        value = P_all / GIB / (ms_step * 1e-3)
        line = {
            "metric": "GiB/s device-resident Huffman decode+encode, 16M header strings mean 48B",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded, header alphabet P~2^-nbits, 1% adversarial)",
            "config": {"workload": "%s: %d header strings/GPU, lengths %s, encode all + decode the compressible"
                                   % (args.config, n, synth.CONFIGS[args.config]["lengths"]),
                       "strings_per_gpu": n, "global_strings": int(n_all), "plain_bytes_per_gpu": P,
                       "huffman_bytes_per_gpu": H, "parallelism": "shard%d" % world},
            "encode_ms": round(t_enc_avg, 4),
            "decode_ms": round(t_dec_avg, 4),
            "encode_gibps": round(P / GIB / (t_enc_avg * 1e-3), 3) if do_enc else None,
            "decode_gibps": round(P_ok / GIB / (t_dec_avg * 1e-3), 3) if do_dec else None,
            "roofline": {"bound": "hbm", "kernel": dominant, "achieved": round(ach, 2), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4),
                         "traffic": round(traffic[dominant]) if dominant in traffic else None,
                         "algorithmic_bytes": B_dec if dominant == "decode" else B_enc},
            "traffic_bytes_per_launch": {k: round(v) for k, v in traffic.items()} or None,
        }
        if not args.no_host and not args.pmc_child:
            line["host_inclusive"] = host_inclusive(b, off32, n, huff, h_off32, n_ok, names_bits, P, H, P_ok, torch)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(b, args, np)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def host_inclusive(b, off32, n, huff, h_off32, n_ok, names_bits, P, H, P_ok, torch, reps=3):
    """The same step with the strings starting and ending in pinned host memory: H2D of the inputs,
    encode + decode, D2H of the outputs, all on one stream (PCIe-bound; recorded in DESIGN.md, never
    `value`)."""
    from h2o_amd import codec

    def pin(t):
        return t.cpu().pin_memory()

    h_plain, h_off, h_huff, h_hoff, h_names = pin(b["data"]), pin(off32), pin(huff[:H]), pin(h_off32), pin(names_bits)
    d_plain, d_off = torch.empty(P + 16, dtype=torch.uint8, device="cuda"), torch.empty_like(off32)
    d_huff, d_hoff, d_names = torch.empty(H + 16, dtype=torch.uint8, device="cuda"), torch.empty_like(h_off32), \
        torch.empty_like(names_bits)
    e_out = torch.empty(P + 16, dtype=torch.uint8, device="cuda")
    e_len, e_st = torch.empty(n, dtype=torch.int32, device="cuda"), torch.empty(n, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(codec.decode_slot_size(H), dtype=torch.uint8, device="cuda")
    d_len, d_st = torch.empty(n_ok, dtype=torch.int32, device="cuda"), torch.empty(n_ok, dtype=torch.uint8, device="cuda")
    o_enc, o_elen, o_est = torch.empty(P, dtype=torch.uint8).pin_memory(), torch.empty(n, dtype=torch.int32).pin_memory(), \
        torch.empty(n, dtype=torch.uint8).pin_memory()
    o_dec, o_dlen, o_dst = torch.empty(d_out.numel(), dtype=torch.uint8).pin_memory(), \
        torch.empty(n_ok, dtype=torch.int32).pin_memory(), torch.empty(n_ok, dtype=torch.uint8).pin_memory()
    times = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d_plain[:P].copy_(h_plain, non_blocking=True)
        d_off.copy_(h_off, non_blocking=True)
        d_huff[:H].copy_(h_huff, non_blocking=True)
        d_hoff.copy_(h_hoff, non_blocking=True)
        d_names.copy_(h_names, non_blocking=True)
        codec.encode_batch(d_plain, d_off, n, out=e_out, out_len=e_len, status=e_st, in_size=P)
        codec.decode_batch(d_huff, d_hoff, n_ok, is_name_bits=d_names, out=d_out, out_len=d_len, status=d_st,
                           in_size=H)
        o_enc.copy_(e_out[:P], non_blocking=True)
        o_elen.copy_(e_len, non_blocking=True)
        o_est.copy_(e_st, non_blocking=True)
        o_dec.copy_(d_out, non_blocking=True)
        o_dlen.copy_(d_len, non_blocking=True)
        o_dst.copy_(d_st, non_blocking=True)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    t_serial = min(times[1:])
    # the library's pipelined host path (hhuff_*_batch_host_pipelined): chunks overlap host staging,
    # H2D, kernels and D2H on three streams; caller buffers pinned, then pageable
    np_ = __import__("numpy")
    res = {}
    for kind in ("pinned", "pageable"):
        def hbuf(count, dt):
            if kind == "pinned":
                return torch.empty(count, dtype=dt).pin_memory().numpy()
            return np_.empty(count, {torch.uint8: np_.uint8, torch.int32: np_.int32}[dt])

        if kind == "pinned":
            src_p, src_h = h_plain.numpy(), h_huff.numpy()
        else:
            src_p, src_h = h_plain.numpy().copy(), h_huff.numpy().copy()
        out_e, out_d = hbuf(P + 16, torch.uint8), hbuf(codec.decode_slot_size(H), torch.uint8)
        el, es = hbuf(n, torch.int32).view(np_.uint32), hbuf(n, torch.uint8)
        dl, ds = hbuf(n_ok, torch.int32).view(np_.uint32), hbuf(n_ok, torch.uint8)
        off_np, hoff_np = h_off.numpy().view(np_.uint32), h_hoff.numpy().view(np_.uint32)
        names_np = h_names.numpy().view(np_.uint32)
        if kind == "pageable":
            off_np, hoff_np, names_np = off_np.copy(), hoff_np.copy(), names_np.copy()
        ts = []
        for _ in range(reps + 1):
            t0 = time.perf_counter()
            codec.encode_batch_host_pipelined(src_p, off_np, n, out=out_e, out_len=el, status=es)
            codec.decode_batch_host_pipelined(src_h, hoff_np, n_ok, is_name_bits=names_np, out=out_d, out_len=dl,
                                              status=ds)
            ts.append(time.perf_counter() - t0)
        res[kind] = min(ts[1:])
    t = res["pinned"]
    return {"value": round(P / GIB / t, 3), "unit": "GiB/s", "ms_per_step": round(t * 1e3, 3),
            "pageable_value": round(P / GIB / res["pageable"], 3), "pageable_ms_per_step": round(res["pageable"] * 1e3, 3),
            "serial_value": round(P / GIB / t_serial, 3), "serial_ms_per_step": round(t_serial * 1e3, 3),
            "note": "strings start and end in host memory; value: hhuff_{encode,decode}_batch_host_pipelined with "
                    "pinned caller buffers (64 MiB chunks, 3 streams); pageable_*: same with pageable buffers; "
                    "serial_*: pinned H2D + kernels + D2H on one stream; best of %d" % reps}


def cpu_baseline(b, args, np):
    """h2o's own CPU path on this host's cores, timed like one step (encode all strings, then decode the
    compressible ones).  kind "reference": oracle/_ref/libh2oref.so, the reference's lib/http2/hpack.c
    compiled where it lies (it travels with the tree); kind "port": the clean-room restatement when the
    reference build is absent.  Multi-threaded over a bounded sample of rank 0's batch (default: all
    of it, ~10-30 s of CPU work), contiguous per-thread ranges; plus a single-thread rate on a smaller
    sample."""
    from oracle import oracle as O

    kind = "reference" if O.ref_available() else "port"
    codec = O.ref() if kind == "reference" else O.oracle()
    m = min(args.cpu_sample, b["n"]) if args.cpu_sample else b["n"]
    off = b["off"][:m + 1].cpu().numpy().astype(np.uint32)
    data = b["data"][:int(off[-1])].cpu().numpy()
    names = b["is_name_bits"][:(m + 31) // 32].cpu().numpy().view(np.uint32)
    threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))

    def rate(mm, nthreads, reps):
        o = off[:mm + 1]
        d = data[:int(o[-1])]
        enc, el, _ = codec.encode_batch(d, o, mm, nthreads=nthreads)  # also produces the decode input
        hl = np.where(el != O.FAIL, el, 0).astype(np.uint32)
        starts = o[:-1].copy()
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            codec.encode_batch(d, o, mm, nthreads=nthreads)
            codec.decode_batch(enc, starts, mm, in_len=hl, is_name_bits=names, nthreads=nthreads)
            t = time.perf_counter() - t0
            best = t if best is None else min(best, t)
        return float(o[-1]) / GIB / best, float(o[-1])

    v, P = rate(m, threads, 3)
    m1 = min(m, 1 << 18)
    v1, P1 = rate(m1, 1, 3)
    return {"value": round(v, 4), "unit": "GiB/s", "cores": threads, "kind": kind,
            "sample": "%d strings (%.1f MB) of rank 0's batch, encode + decode, best of 3, %d threads "
                      "(%s)" % (m, P / 1e6, threads, "oracle/_ref: lib/http2/hpack.c compiled" if kind == "reference"
                                else "clean-room restatement"),
            "single_thread_value": round(v1, 4),
            "single_thread_sample": "%d strings (%.1f MB), 1 thread" % (m1, P1 / 1e6)}


if __name__ == "__main__":
    main()
