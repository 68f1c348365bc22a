#!/usr/bin/env python3
"""hhuff benchmark -- BASELINE.json metric "GiB/s device-resident Huffman decode+encode, 16M header strings
mean 48B" on configuration 4: 16M header strings, lengths U[24,72], header alphabet, batch-sharded across the
GPUs of one node.

The batch (seeded, identical on every rank) is cut byte-balanced with h2o_amd.dist.byte_balanced_bounds; each
rank keeps its shard resident in its HBM (N = 1: the whole batch on one GPU).  One step = one pass of the hot
path over the shard, inputs resident in HBM:
    encode  all the shard's plain strings      (hhuff_encode_batch, h2o_hpack_encode_huffman per element)
    decode  its compressible strings' Huffman  (hhuff_decode_batch, h2o_hpack_decode_huffman per element),
            packed back to back as on the wire
    N > 1:  an RCCL all_gather of every shard's (strings, output bytes) -- the batch split's one exchange,
            which gives each shard its global output offsets; issued behind the encode, it overlaps the
            decode on the collective's stream
value = total plain bytes of the batch / max over ranks of the step time   [GiB/s, 2^30]; strong scaling
(the batch is fixed, N GPUs share it).

Extra JSON fields: per-direction times and rates; the packed-output mode (hhuff_{de,en}code_batch_packed)
timed on the same shard; `roofline` for the dominant kernel (algorithmic bytes per launch over its HIP-event
duration; HBM traffic from rocprofv3 PMC passes run before this process touches the GPU) plus a `secondary`
ceiling (VALU / LDS issue from the SQ counters); N = 1 only: the other BASELINE configs (c2, c3, c5), the
per-string symbols' call latency, the H2D/D2H-inclusive rate and `cpu_baseline` (h2o's own CPU path on this
host's cores).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); the line also carries the measured copy peak
GUIDE_COPY_GBPS = 6290.0  # MI355X_MICROARCH.md: 6.29 TB/s measured with a float4 copy kernel (79 % of the spec)
N_SIMD, N_CU = 1024, 256
GIB = float(1 << 30)
METRIC = "GiB/s device-resident Huffman decode+encode, 16M header strings mean 48B"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) on this node; without a launcher's WORLD_SIZE, N > 1 starts N ranks itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4")
    ap.add_argument("--strings", "--n", dest="n", type=int, default=None,
                    help="strings in the whole batch (default: the config's N)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=0, help="strings in the CPU-baseline sample (0: 4M)")
    ap.add_argument("--cpu-threads", type=int, default=None)
    ap.add_argument("--only", choices=["encode", "decode"], default=None, help="profile one direction")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC passes")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-host", action="store_true", help="skip the H2D/D2H-inclusive measurement")
    ap.add_argument("--no-extra", action="store_true", help="skip the other configs and the per-string latency")
    ap.add_argument("--no-packed", action="store_true", help="skip the packed-output legs")
    ap.add_argument("--force-pg", action="store_true",
                    help="create the process group (and run the exchange) even in a world of one rank: exercises the "
                         "RCCL branch on a one-GPU box under torch.distributed.run --nproc-per-node 1")
    return ap.parse_args()


def _template_args(name):
    """the template arguments of a demangled kernel name: 'k<16, 3584, true, false>(...)' -> [16, 3584, true, false]"""
    i = name.find("<")
    j = name.find(">", i)
    return [a.strip() for a in name[i + 1:j].split(",")] if i >= 0 and j > i else []


def kernel_key(name):
    if "hhuff::" not in name:
        return None
    args = _template_args(name)
    # the PACKED template argument: decode_staged_kernel<WAVES, IN, OUT, PACKED>,
    # encode_staged_kernel<WAVES, STAGE, PACKED>
    pos = 3 if "decode_staged_kernel" in name else 2 if "encode_staged_kernel" in name else None
    packed = pos is not None and len(args) > pos and args[pos] == "true"
    if ("decode_staged_kernel" in name or "decode_stream_kernel" in name or "decode_direct_kernel" in name or
            "decode_seg_kernel" in name):
        return "decode_packed" if packed else "decode"
    if ("encode_staged_kernel" in name or "encode_pl_kernel" in name or "encode_direct_kernel" in name or
            "encode_sorted_kernel" in name):
        return "encode_packed" if packed else "encode"
    if "flatten_pl_kernel" in name or "flatten_direct_kernel" in name:
        return "flatten"
    if "edge_fix" in name:
        return "edge_fix"
    return None


SQ_GROUP = ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES",
            "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")


def synth_n(config):
    from h2o_amd import synth

    return synth.CONFIGS[config]["n"]


LAUNCHER_ENV = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT")


def child_env(env):
    """the environment of a PMC child: the parent's, minus everything a launcher (torch.distributed.run) set
    for the parent's rank -- WORLD_SIZE / RANK / MASTER_* / TORCHELASTIC_* -- so that the child is a world of one
    that never joins (or waits on) the parent's process group; TMPDIR=/tmp for rocprofv3"""
    e = {k: v for k, v in env.items() if k not in LAUNCHER_ENV and not k.startswith("TORCHELASTIC_")}
    e["TMPDIR"] = "/tmp"
    return e


def pmc_passes(args, config=None, groups=None, n=None):
    """Per-launch PMC counters of each hhuff kernel: one rocprofv3 run per counter group (FETCH_SIZE,
    WRITE_SIZE, the SQ group, GRBM_GUI_ACTIVE) over this script as a child on `config` (default: the bench's
    own), BEFORE this process touches the GPU.  Returns {kernel key: {counter: per launch}} or {} when
    rocprofv3 is unavailable.  A launch may run several kernels under one key (the mixed-length decode: the
    staged and the stream kernel, one of which exits at once): their counters add up."""
    import csv
    import shutil
    import subprocess
    import tempfile

    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        return {}
    child = [sys.executable, os.path.abspath(__file__), "--pmc-child", "--steps", "2", "--warmup", "1",
             "--no-cpu-baseline", "--no-traffic", "--no-host", "--no-extra", "--config", config or args.config]
    if (n or args.n) and config is None:
        child += ["--strings", str(n or args.n)]
    if config is not None:
        child += ["--no-packed"]
    vals = {}
    for group in groups or (("FETCH_SIZE",), ("WRITE_SIZE",), SQ_GROUP, ("GRBM_GUI_ACTIVE",)):
        d = tempfile.mkdtemp(prefix="hhuff_pmc_")
        try:
            subprocess.run([exe, "--pmc"] + list(group) + ["--output-format", "csv", "-d", d, "-o", "pmc", "--"] + child,
                           check=True, timeout=300, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           env=child_env(os.environ))
            for root, _, files in os.walk(d):
                for f in files:
                    if f.endswith("counter_collection.csv"):
                        for r in csv.DictReader(open(os.path.join(root, f))):
                            k = kernel_key(r["Kernel_Name"])
                            if k is not None:
                                kn = r["Kernel_Name"]
                                key = (kn, int(r["Dispatch_Id"]), r["Counter_Name"])
                                vals.setdefault(k, {}).setdefault(key, 0.0)
                                vals[k][key] += float(r["Counter_Value"])
        except Exception:
            return {}
        finally:
            shutil.rmtree(d, ignore_errors=True)
    out = {}
    for k, per in vals.items():
        agg = {}
        for (kn, disp, cname), v in per.items():
            agg.setdefault((kn, cname), []).append((disp, v))
        # per kernel: the last two dispatches are the child's timed steps (the first ones build the wire);
        # the kernels of one key add up
        tot = {}
        for (kn, cname), dv in agg.items():
            last = [v for _, v in sorted(dv)[-2:]]
            tot[cname] = tot.get(cname, 0.0) + sum(last) / len(last)
        out[k] = tot
    return out


def traffic_bytes(c):
    """HBM bytes per launch (MI355X_MICROARCH.md HBM section): FETCH_SIZE / WRITE_SIZE are KiB; on gfx950
    FETCH_SIZE reports half the bytes of 16-B/lane streaming reads (the kernels' input staging): doubled"""
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        return (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
    return None


def secondary(c):
    """issue-side ceilings of a kernel from its SQ counters: VALU = SQ_INSTS_VALU x 2 cycles (a wave64 VALU
    instruction holds a SIMD-32 for 2 cycles) over 1024 SIMDs x the kernel's cycles (GRBM_GUI_ACTIVE / 8: the
    counter sums the 8 XCDs); LDS ~ (2 cycles per LDS instruction + SQ_LDS_BANK_CONFLICT) over 256 CUs x cycles"""
    if not all(k in c for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "GRBM_GUI_ACTIVE")):
        return None
    cyc = c["GRBM_GUI_ACTIVE"] / 8.0
    r = {"valu_issue_frac": round(c["SQ_INSTS_VALU"] * 2.0 / (N_SIMD * cyc), 3),
         "lds_issue_frac": round((2.0 * c["SQ_INSTS_LDS"] + c["SQ_LDS_BANK_CONFLICT"]) / (N_CU * cyc), 3),
         "lds_conflict_cycles_per_inst": round(c["SQ_LDS_BANK_CONFLICT"] / max(1.0, c["SQ_INSTS_LDS"]), 2)}
    if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"] > 0:
        r["wave_wait_frac"] = round(c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"], 3)
        r["wave_issue_stall_frac"] = round(c.get("SQ_WAIT_INST_ANY", 0.0) / c["SQ_WAVE_CYCLES"], 3)
        r["wave_active_frac"] = round(c.get("SQ_ACTIVE_INST_ANY", 0.0) / c["SQ_WAVE_CYCLES"], 3)
    return r


def timed_events(torch, fns, steps, warmup, pg, dist):
    """warm up, then time `steps` steps of fns (a list of callables, one event pair each) between barriers
    (`pg`: a process group exists); returns (wall ms per step, [sorted per-fn ms lists])"""
    for _ in range(warmup):
        for f in fns:
            f()
    ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in fns]
          for _ in range(steps)]
    if pg:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for row in ev:
        for (a, b), f in zip(row, fns):
            a.record()
            f()
            b.record()
    torch.cuda.synchronize()
    if pg:
        dist.barrier()
    wall = (time.perf_counter() - t0) * 1e3 / steps
    per = [sorted(row[k][0].elapsed_time(row[k][1]) for row in ev) for k in range(len(fns))]
    return wall, per


def mean(x):
    return sum(x) / len(x)


def launch_plan(gpus, env, backend, device_count):
    """How this invocation runs: ("rank", world) -- this process is one rank of `world` (a launcher set
    WORLD_SIZE, or N = 1) -- or ("spawn", N) -- start N ranks (torch.distributed.run as a child process; this
    process has not touched the GPU) and exit with their status.  Raises SystemExit with a message when the
    request cannot be met: --gpus disagreeing with the launcher's WORLD_SIZE, or more RCCL ranks than GPUs.
    `device_count` is a callable (torch.cuda.device_count, which does not initialise the GPU on this image)."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        ws = int(ws)
        if gpus is not None and gpus != ws:
            raise SystemExit("bench.py: --gpus %d but the launcher started WORLD_SIZE=%d ranks" % (gpus, ws))
        return ("rank", ws)
    n = 1 if gpus is None else gpus
    if n < 1:
        raise SystemExit("bench.py: --gpus must be >= 1 (got %d)" % n)
    if n == 1:
        return ("rank", 1)
    if backend == "nccl":
        have = device_count()
        if have < n:
            raise SystemExit("bench.py: --gpus %d needs %d GPUs for RCCL, this node shows %d "
                             "(HHUFF_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs)" % (n, n, have))
    return ("spawn", n)


def rank_command(n, argv, port):
    """the child command that starts n ranks of this script: torch.distributed.run sets RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* for each; every rank sees the same arguments and --gpus n"""
    # torch.distributed.run's parser matches option prefixes even among the script's arguments, and `--n` is a
    # prefix of several of its own options: pass the batch size under its long name
    args = ["--strings" + a[3:] if a == "--n" or a.startswith("--n=") else a for a in argv]
    if not any(a == "--gpus" or a.startswith("--gpus=") for a in args):
        args += ["--gpus", str(n)]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + args


def spawn_ranks(n, argv):
    """start n ranks of this script on this node (one per GPU) as a child process tree and return their exit
    status; rank 0 prints the JSON line"""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "16")
    return subprocess.run(rank_command(n, argv, port), env=env).returncode


def main():
    args = parse()
    backend = os.environ.get("HHUFF_DIST_BACKEND", "nccl")  # gloo: rehearse N ranks on fewer GPUs

    def _count():
        import torch
        return torch.cuda.device_count()

    if args.pmc_child:  # a profiling child is a world of one whatever its environment says: no process group
        mode, world = "rank", 1
    else:
        mode, world = launch_plan(args.gpus, os.environ, backend, _count)
    if mode == "spawn":
        sys.exit(spawn_ranks(world, sys.argv[1:]))
    args.gpus = world
    pmc, pmc_cfg = {}, {}
    rank = 0 if args.pmc_child else int(os.environ.get("RANK", "0"))
    if not args.pmc_child and not args.no_traffic and rank == 0:
        # child processes; this process has not touched the GPU yet.  N > 1: rank 0 profiles one shard's worth
        # of the batch (N / world strings) on its GPU while the other ranks wait in the rendezvous
        pmc = pmc_passes(args, n=None if world == 1 else -(-(args.n or synth_n(args.config)) // world))
        if not args.no_extra and world == 1:  # HBM traffic of the other configs' kernels (two passes each)
            pmc_cfg = {c: pmc_passes(args, config=c, groups=(("FETCH_SIZE",), ("WRITE_SIZE",))) for c in ("c2", "c3", "c5")}
    c_caller = None
    if not args.pmc_child and not args.no_extra and world == 1:
        c_caller = per_string_c_caller()  # a child process too, before this one touches the GPU
    import torch
    import torch.distributed as dist

    from h2o_amd import codec, synth
    from h2o_amd import dist as hd

    local = 0 if args.pmc_child else int(os.environ.get("LOCAL_RANK", "0"))
    # a process group for N > 1, or (--force-pg) for a launcher-started world of one: the RCCL init, the
    # device-tensor exchange and the MAX all_reduce then run exactly as on an 8-GPU node
    pg = not args.pmc_child and (world > 1 or (args.force_pg and "WORLD_SIZE" in os.environ))
    if pg:
        torch.cuda.set_device(local % torch.cuda.device_count())
        # rank 0 runs its PMC passes (child processes, minutes at full size) before it joins: the others wait
        import datetime
        tmo = datetime.timedelta(minutes=30)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
    else:
        torch.cuda.set_device(0)
    codec.lib()

    # ---- config 4's batch, cut byte-balanced; this rank's shard stays resident -------------------------
    full = synth.make_batch_torch(args.config, n=args.n, seed=1000)
    n_all, P_all = full["n"], int(full["total"])
    bounds = hd.byte_balanced_bounds(full["off"], world).tolist()
    b = hd.shard(full, bounds[rank], bounds[rank + 1])
    del full
    torch.cuda.empty_cache()
    n, off32 = b["n"], b["off"]
    P = int(b["data"].numel())
    lens = (off32[1:].to(torch.int64) - off32[:-1].to(torch.int64))
    enc_out = torch.empty(P + 16, dtype=torch.uint8, device="cuda")
    enc_len = torch.empty(n, dtype=torch.int32, device="cuda")
    enc_st = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.encode_batch(b["data"], off32, n, out=enc_out, out_len=enc_len, status=enc_st, in_size=P)
    # the wire: compressible strings packed back to back (packed encode places them; a gather closes the gaps)
    ok = enc_len != -1
    idx = torch.nonzero(ok).squeeze(1)
    n_ok = int(idx.numel())
    hl = enc_len[idx].to(torch.int64)
    h_off = torch.zeros(n_ok + 1, dtype=torch.int64, device="cuda")
    h_off[1:] = torch.cumsum(hl, 0)
    H = int(h_off[-1].item())
    huff = torch.empty(H + 16, dtype=torch.uint8, device="cuda")
    rel = torch.arange(H, device="cuda") - torch.repeat_interleave(h_off[:-1], hl)
    huff[:H] = enc_out[torch.repeat_interleave(off32[:-1].to(torch.int64)[idx], hl) + rel]
    del rel
    names_ok = hd.bits_to_bool(b["is_name_bits"], n)[idx]
    names_bits = hd.bool_to_bits(names_ok)
    h_off32 = h_off.to(torch.int32).contiguous()
    P_ok = int(lens[idx].sum().item()) if n_ok else 0
    dec_out = torch.empty(codec.decode_slot_size(H), dtype=torch.uint8, device="cuda")
    dec_len = torch.empty(n_ok, dtype=torch.int32, device="cuda")
    dec_st = torch.empty(n_ok, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()

    do_enc = args.only in (None, "encode")
    do_dec = args.only in (None, "decode")
    # N > 1: the batch split's all_gather of (strings, output bytes), from device-resident sums.  With both
    # kernels in the step it is issued behind the encode (its output bytes) and waited for after the decode.
    # Every piece has its own event pair on the compute stream, so encode_ms / decode_ms are the codec
    # launches alone: "issue" covers the output-byte sum and the all_gather's enqueue, "wait" the part of the
    # exchange the decode did not hide.  With RCCL the collective runs on its own stream; with gloo the
    # device-to-host copy of the sum blocks the host until the encode is done (host-synchronous, no overlap).
    overlap = pg and do_enc and do_dec
    pending = []

    def run_encode():
        codec.encode_batch(b["data"], off32, n, out=enc_out, out_len=enc_len, status=enc_st, in_size=P)

    def run_exchange_issue():
        pending.append(hd.exchange_sizes_async(n, torch.clamp(enc_len, min=0).to(torch.int64).sum())[0])

    def run_decode():
        codec.decode_batch(huff, h_off32, n_ok, is_name_bits=names_bits, out=dec_out, out_len=dec_len, status=dec_st,
                           in_size=H)

    def run_exchange_wait():
        while pending:
            pending.pop().wait()

    def run_exchange():  # the exchange on its own (one kernel in the step)
        hd.exchange_sizes(n_ok, torch.clamp(dec_len, min=0).to(torch.int64).sum())

    # correctness spot check before timing: decoded lengths equal the plain lengths of the kept strings
    run_decode()
    torch.cuda.synchronize()
    assert bool((dec_len == lens[idx].to(torch.int32)).all()), "decode does not invert encode"

    if overlap:
        fns = [run_encode, run_exchange_issue, run_decode, run_exchange_wait]
        slot_enc, slot_dec = 0, 2
    else:
        fns = ([run_encode] if do_enc else []) + ([run_decode] if do_dec else []) + \
            ([run_exchange] if pg else [])
        slot_enc, slot_dec = 0, (1 if do_enc else 0)
    ms_step, per = timed_events(torch, fns, args.steps, args.warmup, pg, dist)
    if args.pmc_child and args.config == "c5":  # c5's own operation, flatten_string framing, for its PMC pass
        f_out = torch.empty(P + 11 * n + 16, dtype=torch.uint8, device="cuda")
        f_len = torch.empty(n, dtype=torch.int32, device="cuda")
        for _ in range(3):
            codec.flatten_batch(b["data"], off32, n, 7, out=f_out, out_len=f_len, in_size=P)
        torch.cuda.synchronize()
    t_enc = mean(per[slot_enc]) if do_enc else 0.0
    t_dec = mean(per[slot_dec]) if do_dec else 0.0

    # ---- packed-output mode on the same shard (hhuff_{de,en}code_batch_packed) ----------------------------
    packed = None
    if not args.no_packed and args.only is None:
        pe_out = torch.empty(P + 16, dtype=torch.uint8, device="cuda")
        pe_off = torch.empty(n + 1, dtype=torch.int32, device="cuda")
        pd_out = torch.empty(codec.decode_slot_size(H), dtype=torch.uint8, device="cuda")
        pd_off = torch.empty(n_ok + 1, dtype=torch.int32, device="cuda")

        def run_encode_packed():
            codec.encode_batch_packed(b["data"], off32, n, out=pe_out, out_off=pe_off, out_len=enc_len, status=enc_st,
                                      in_size=P)

        def run_decode_packed():
            codec.decode_batch_packed(huff, h_off32, n_ok, is_name_bits=names_bits, out=pd_out, out_off=pd_off,
                                      out_len=dec_len, status=dec_st, in_size=H)

        run_decode_packed()
        torch.cuda.synchronize()
        assert bool((dec_len == lens[idx].to(torch.int32)).all()), "packed decode does not invert encode"
        pk_ms, pk = timed_events(torch, [run_encode_packed, run_decode_packed], args.steps, args.warmup, pg, dist)
        # value: the whole batch over the slowest rank's kernel time (the same rule as the headline)
        packed = {"encode_ms": round(mean(pk[0]), 4), "decode_ms": round(mean(pk[1]), 4), "ms_per_step": round(pk_ms, 4),
                  "_kernel_ms": mean(pk[0]) + mean(pk[1])}
    if pg:
        vals = [ms_step] + ([packed["_kernel_ms"]] if packed is not None else [])
        t = torch.tensor(vals, device="cuda" if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms_step = float(t[0].item())
        if packed is not None:
            packed["_kernel_ms"] = float(t[1].item())
    if packed is not None:
        packed["value"] = round(P_all / GIB / (packed.pop("_kernel_ms") * 1e-3), 3)

    if rank == 0:
        B_dec = H + P_ok + 9 * n_ok + 4 + (n_ok + 7) // 8
        E = int(hl.sum().item())
        B_enc = P + E + 9 * n + 4
        gb = lambda B, t: B / (t * 1e-3) / 1e9  # noqa: E731
        dominant = "encode" if (t_enc >= t_dec and do_enc) or not do_dec else "decode"
        B_dom, t_dom = (B_enc, t_enc) if dominant == "encode" else (B_dec, t_dec)
        ach = gb(B_dom, t_dom)
        roof = {"bound": "hbm", "kernel": dominant, "achieved": round(ach, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBPS, 4),
                "traffic": round(traffic_bytes(pmc[dominant])) if dominant in pmc and traffic_bytes(pmc[dominant]) else None,
                "algorithmic_bytes": B_dom,
                "bytes_per_unit": "decode: H + P + 9 N + 4 + ceil(N/8); encode: P + E + 9 N + 4 (SURVEY 8d)"}
        sec = secondary(pmc.get(dominant, {}))
        if sec:
            roof["secondary"] = sec
        cp = copy_peak(torch)
        if cp:
            roof["measured_copy_peak"] = cp  # torch copy_ (the runtime's blit / SDMA copy)
        # the guide's measured float4 (16 B a lane) copy, MI355X_MICROARCH.md: what a streaming kernel reaches
        roof["guide_copy_peak"] = GUIDE_COPY_GBPS
        roof["frac_of_measured"] = round(ach / max(cp or 0.0, GUIDE_COPY_GBPS), 4)
        line = {
            "metric": METRIC,
            "value": round(P_all / GIB / (ms_step * 1e-3), 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded, header alphabet P~2^-nbits, 1% adversarial)",
            "config": {"workload": "%s: %d header strings, lengths %s, byte-balanced over %d GPU(s); encode all + "
                                   "decode the compressible" % (args.config, n_all, synth.CONFIGS[args.config]["lengths"],
                                                                world),
                       "global_strings": n_all, "global_plain_bytes": P_all, "strings_rank0": n,
                       "plain_bytes_rank0": P, "huffman_bytes_rank0": H, "parallelism": "shard%d" % world},
            "encode_ms": round(t_enc, 4),
            "decode_ms": round(t_dec, 4),
            "encode_gibps": round(P / GIB / (t_enc * 1e-3), 3) if do_enc else None,
            "decode_gibps": round(P_ok / GIB / (t_dec * 1e-3), 3) if do_dec else None,
            "roofline": roof,
            "traffic_bytes_per_launch": {k: round(traffic_bytes(v)) for k, v in pmc.items() if traffic_bytes(v)} or None,
        }
        if pg:
            line["dist_backend"] = backend
        if pg and not overlap:
            line["exchange_ms"] = round(mean(per[-1]), 4)
        elif pg:
            line["exchange_issue_ms"] = round(mean(per[1]), 4)
            line["exchange_wait_ms"] = round(mean(per[3]), 4)
            line["exchange"] = ("all_gather of (strings, encode output bytes) issued behind the encode on the RCCL "
                                "stream and waited for after the decode" if backend == "nccl" else
                                "gloo rehearsal: host-synchronous all_gather after the encode (no overlap)")
            line["dist_backend"] = backend
        if packed is not None:
            B_dec_pk = B_dec + 4 * (n_ok + 1)  # + out_off[n + 1]
            B_enc_pk = B_enc + 4 * (n + 1)
            tr = {k: traffic_bytes(pmc[k]) for k in ("encode_packed", "decode_packed") if k in pmc}
            packed["roofline"] = {
                k: {"achieved": round(gb(B, packed[k.split("_")[0] + "_ms"]), 2),
                    "frac": round(gb(B, packed[k.split("_")[0] + "_ms"]) / HBM_PEAK_GBPS, 4),
                    "algorithmic_bytes": B, "traffic": round(tr[k]) if tr.get(k) else None,
                    "traffic_over_algorithmic": round(tr[k] / B, 4) if tr.get(k) else None}
                for k, B in (("encode_packed", B_enc_pk), ("decode_packed", B_dec_pk))}
            line["packed"] = packed
        if world > 1 and pmc:
            line["traffic_note"] = "PMC passes of one shard's worth (%d strings) on rank 0's GPU" % -(-n_all // world)
        if not args.pmc_child:
            if world == 1 and not args.no_extra:
                line["configs"] = other_configs(torch, codec, synth, pmc_cfg)
                line["f4"] = f4_lines(torch, codec)
                line["per_string_latency_us"] = per_string_latency(codec)
                line["per_string_latency_us"]["c_caller"] = c_caller
            if world == 1 and not args.no_host:
                line["host_inclusive"] = host_inclusive(b, off32, n, huff, h_off32, n_ok, names_bits, P, H, torch)
            if not args.no_cpu_baseline:  # rank 0's host cores, on a sample of its shard (N > 1 too)
                line["cpu_baseline"] = cpu_baseline(b, args)
        print(json.dumps(line), flush=True)
    if pg:
        dist.destroy_process_group()


def copy_peak(torch, nbytes=1 << 30, reps=5):
    """the device-to-device copy rate this GPU sustains (GB/s, bytes read + written, best of `reps`): what
    an HBM-bound kernel can reach here, beside the 8 TB/s spec in `peak`"""
    try:
        src = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        dst = torch.empty_like(src)
    except RuntimeError:
        return None
    dst.copy_(src)
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dst.copy_(src)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    del src, dst
    torch.cuda.empty_cache()
    return round(2 * nbytes / (best * 1e-3) / 1e9, 1)


def kernel_roofline(B, t_ms, pmc, key):
    """{algorithmic bytes, achieved GB/s, fraction of HBM peak, PMC traffic per launch} of one kernel"""
    ach = B / (t_ms * 1e-3) / 1e9
    tr = traffic_bytes(pmc.get(key, {})) if pmc else None
    return {"algorithmic_bytes": int(B), "achieved": round(ach, 2), "frac": round(ach / HBM_PEAK_GBPS, 4),
            "traffic": round(tr) if tr else None, "traffic_over_algorithmic": round(tr / B, 4) if tr else None}


def other_configs(torch, codec, synth, pmc_cfg=None):
    """BASELINE configs 2, 3, 5 (device-resident, HIP-event medians; tools/bench_configs.py): encode to slots,
    decode of the compressible strings' Huffman packed back to back, and for c5 the flatten_string framing.
    Each leg carries its roofline (SURVEY 8d bytes; traffic from this config's own PMC passes):
    decode H + P_ok + 9 N_ok + 4, encode P + E + 9 N + 4, framing P + F + 8 N + 4 (F: framed bytes)."""
    import bench_configs as BC

    pmc_cfg = pmc_cfg or {}
    res = {}
    for cfg in ("c2", "c3", "c5"):
        b = synth.make_batch_torch(cfg, seed=7)
        n, P = b["n"], int(b["total"])
        off32 = b["off"].to(torch.int32)
        r = {"strings": n, "plain_bytes": P}
        huff, h_off, n_ok, H, P_ok = BC.packed_huffman(torch, codec, b)
        d_out = torch.empty(codec.decode_slot_size(H), dtype=torch.uint8, device="cuda")
        d_len = torch.empty(n_ok, dtype=torch.int32, device="cuda")
        d_st = torch.empty(n_ok, dtype=torch.uint8, device="cuda")
        dec = lambda: codec.decode_batch(huff, h_off, n_ok, out=d_out, out_len=d_len, status=d_st, in_size=H)
        t_dec, t_dec_ev = BC.timed_b2b(torch, dec), BC.timed(torch, dec)
        e_out = torch.empty(P + 16, dtype=torch.uint8, device="cuda")
        e_len = torch.empty(n, dtype=torch.int32, device="cuda")
        enc = lambda: codec.encode_batch(b["data"], off32, n, out=e_out, out_len=e_len, in_size=P)
        t_enc, t_enc_ev = BC.timed_b2b(torch, enc), BC.timed(torch, enc)
        E = int(torch.clamp(e_len, min=0).to(torch.int64).sum().item())
        pm = pmc_cfg.get(cfg, {})
        # *_ms: calls back to back (tools/bench_configs.timed_b2b); *_ms_event_pair: an event pair around each
        # call, the round-4/5 figure, which adds the pair's gap to every call
        r.update(timing="back_to_back", decode_ms_event_pair=round(t_dec_ev, 4), encode_ms_event_pair=round(t_enc_ev, 4))
        r.update(decode_ms=round(t_dec, 4), decode_gibps=round(P_ok / GIB / (t_dec * 1e-3), 2),
                 encode_ms=round(t_enc, 4), encode_gibps=round(P / GIB / (t_enc * 1e-3), 2),
                 round_trip_gibps=round(P / GIB / ((t_enc + t_dec) * 1e-3), 2),
                 decode_roofline=kernel_roofline(H + P_ok + 9 * n_ok + 4, t_dec, pm, "decode"),
                 encode_roofline=kernel_roofline(P + E + 9 * n + 4, t_enc, pm, "encode"))
        del huff, h_off, d_out, e_out
        if cfg == "c5":  # QPACK values: flatten_string(prefix 7) framing, the config's own operation
            f_out = torch.empty(P + 11 * n + 16, dtype=torch.uint8, device="cuda")
            f_len = torch.empty(n, dtype=torch.int32, device="cuda")
            flat = lambda: codec.flatten_batch(b["data"], off32, n, 7, out=f_out, out_len=f_len, in_size=P)
            t, t_ev = BC.timed_b2b(torch, flat), BC.timed(torch, flat)
            r.update(flatten_ms_event_pair=round(t_ev, 4))
            F = int(f_len.to(torch.int64).sum().item())
            r.update(flatten_ms=round(t, 4), flatten_gibps=round(P / GIB / (t * 1e-3), 2),
                     flatten_roofline=kernel_roofline(P + F + 8 * n + 4, t, pm, "flatten"))
        res[cfg] = r
        del b
        torch.cuda.empty_cache()
    return res


def f4_lines(torch, codec):
    """whole header blocks (65,536 browser-like HTTP/2 connections, h2o_hpack_decode_header per field
    with one dynamic table each, and h2o_hpack_parse_request's rules), one QPACK decoder step (65,536 HTTP/3
    connections: encoder streams, then field sections) and, encode side, HTTP/2 responses of 65,536 connections
    flattened with their encoder tables (h2o_hpack_flatten_response), and, client side, requests flattened
    (h2o_hpack_flatten_request) and response blocks through h2o_hpack_parse_response's rules, with their CPU baselines (tools/bench_configs.py)"""
    import bench_configs as BC

    res = {}
    for name, fn in (("blocks", BC.blocks_line), ("qpack", BC.qpack_line), ("hpenc", BC.hpenc_line),
                     ("reqenc", lambda torch, codec, n: BC.hpenc_line(torch, codec, n, requests=True)),
                     ("responses", BC.responses_line)):
        try:
            res[name] = fn(torch, codec, 65536)
        except Exception as e:  # a report, not a gate
            res[name] = {"error": str(e)}
        torch.cuda.empty_cache()
    return res


def per_string_c_caller(threads=(1, 16)):
    """h2o's per-string symbols called from C the way h2o's event-loop threads call them (tools/per_string_bench:
    T pthreads, 2,000 encode then 2,000 decode calls each of one 48-B header string): per thread count, the
    aggregate strings/s and the per-call median / p99 (us).  Run as a child process before the bench touches the
    GPU; None when the program is not built"""
    import subprocess

    exe = os.path.join(ROOT, "tools", "per_string_bench")
    if not os.path.exists(exe):
        return None
    try:
        r = subprocess.run([exe] + [str(t) for t in threads], capture_output=True, text=True, timeout=120,
                           env=child_env(os.environ))
        recs = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    except Exception as e:  # a report, not a gate
        return {"error": str(e)}
    return {"threads": {str(x.get("threads")): x for x in recs}, "tool": "tools/per_string_bench.c"}


def per_string_latency(codec, calls=2000):
    """h2o's per-string symbols (a synchronous batch of one on the GPU): median / p99 microseconds per call"""
    s = (b"accept-encoding: gzip, deflate, br, zstd" * 2)[:48]
    h = codec.encode_huffman(s)
    out = {}
    for name, fn in (("h2o_hpack_encode_huffman", lambda: codec.encode_huffman(s)),
                     ("h2o_hpack_decode_huffman", lambda: codec.decode_huffman(h, False))):
        for _ in range(50):
            fn()
        t = []
        for _ in range(calls):
            t0 = time.perf_counter()
            fn()
            t.append(time.perf_counter() - t0)
        t.sort()
        out[name] = {"median": round(t[len(t) // 2] * 1e6, 2), "p99": round(t[int(len(t) * 0.99)] * 1e6, 2)}
    out["string_bytes"] = len(s)
    # long values (cookies, URIs): past the service's 768 B a call is one launch; decode splits the string over
    # a wave from 512 Huffman bytes (split_decode_kernel)
    text = (b"session=eyJhbGciOiJIUzI1NiJ9.dXNlcj0xMjM0NTY3ODkw; theme=dark; lang=en-US; " * 900)
    longs = {}
    for L in (1024, 4096, 16384, 65536):  # 64 KB: past one_string_kernel, the batch kernels on a batch of one
        ls = text[:L]
        lh = codec.encode_huffman(ls)
        assert codec.decode_huffman(lh, False)[0] == ls
        r = {}
        for name, fn in (("encode", lambda: codec.encode_huffman(ls)), ("decode", lambda: codec.decode_huffman(lh, False))):
            for _ in range(10):
                fn()
            t = []
            for _ in range(200):
                t0 = time.perf_counter()
                fn()
                t.append(time.perf_counter() - t0)
            t.sort()
            r[name] = round(t[len(t) // 2] * 1e6, 2)
        longs[str(L)] = r
    out["long_strings_median_us"] = longs
    return out


def host_inclusive(b, off32, n, huff, h_off32, n_ok, names_bits, P, H, torch, reps=3):
    """The same step with the strings starting and ending in host memory: the library's pipelined host path
    (hhuff_*_batch_host_pipelined: chunks overlap host staging, H2D, kernels and D2H on three streams) with
    pinned and with pageable caller buffers (PCIe-bound; recorded in DESIGN.md, never `value`)."""
    import numpy as np

    from h2o_amd import codec

    def pin(t):
        return t.cpu().pin_memory()

    h_plain, h_off, h_huff, h_hoff, h_names = pin(b["data"]), pin(off32), pin(huff[:H]), pin(h_off32), pin(names_bits)
    res = {}
    # packed: the same pinned buffers through hhuff_*_batch_host_packed (zero copy, the packed kernels: only the
    # output bytes, out_off, out_len and status cross the link, not the slot tails)
    for kind in ("pinned", "packed", "packed_off", "pinned_dma", "pageable"):
        # pinned: the library's default for device-visible caller buffers (zero copy: the kernels read and
        # write host memory across PCIe); pinned_dma: the chunked DMA pipeline on the same buffers
        if kind == "pinned_dma":
            os.environ["HHUFF_HOST_COPY"] = "1"
        else:
            os.environ.pop("HHUFF_HOST_COPY", None)
        def hbuf(count, dt):
            if kind != "pageable":
                return torch.empty(count, dtype=dt).pin_memory().numpy()
            return np.empty(count, {torch.uint8: np.uint8, torch.int32: np.int32}[dt])

        src_p, src_h = (h_plain.numpy(), h_huff.numpy()) if kind != "pageable" else (h_plain.numpy().copy(),
                                                                                     h_huff.numpy().copy())
        out_e, out_d = hbuf(P + 16, torch.uint8), hbuf(codec.decode_slot_size(H), torch.uint8)
        el, es = hbuf(n, torch.int32).view(np.uint32), hbuf(n, torch.uint8)
        dl, ds = hbuf(n_ok, torch.int32).view(np.uint32), hbuf(n_ok, torch.uint8)
        off_np, hoff_np = h_off.numpy().view(np.uint32), h_hoff.numpy().view(np.uint32)
        names_np = h_names.numpy().view(np.uint32)
        if kind == "pageable":
            off_np, hoff_np, names_np = off_np.copy(), hoff_np.copy(), names_np.copy()
        if kind == "packed_off":  # out_off and the encode status returned as well (5 more bytes a string)
            oo_e, oo_d = hbuf(n + 1, torch.int32).view(np.uint32), hbuf(n_ok + 1, torch.int32).view(np.uint32)

            def run_enc():
                codec.encode_batch_host_packed(src_p, off_np, n, out=out_e, out_off=oo_e, out_len=el, status=es)

            def run_dec():
                codec.decode_batch_host_packed(src_h, hoff_np, n_ok, is_name_bits=names_np, out=out_d, out_off=oo_d,
                                               out_len=dl, status=ds)
        elif kind == "packed":  # lengths (and decode statuses) only: positions follow from them (packed_positions)
            def run_enc():
                codec.encode_batch_host_packed(src_p, off_np, n, out=out_e, out_len=el, with_off=False,
                                               with_status=False)

            def run_dec():
                codec.decode_batch_host_packed(src_h, hoff_np, n_ok, is_name_bits=names_np, out=out_d, out_len=dl,
                                               status=ds, with_off=False)
        else:
            def run_enc():
                codec.encode_batch_host_pipelined(src_p, off_np, n, out=out_e, out_len=el, status=es)

            def run_dec():
                codec.decode_batch_host_pipelined(src_h, hoff_np, n_ok, is_name_bits=names_np, out=out_d, out_len=dl,
                                                  status=ds)
        ts = []
        for _ in range(reps + 1):
            t0 = time.perf_counter()
            run_enc()
            run_dec()
            ts.append(time.perf_counter() - t0)
        res[kind] = min(ts[1:])
        if kind in ("pinned", "packed", "packed_off"):
            # the two legs are independent (a server's requests and responses): on two host threads, each with
            # the library's own per-thread stream, they share the link's two directions at once
            import threading
            ts = []
            for _ in range(reps + 1):
                t0 = time.perf_counter()
                th = threading.Thread(target=run_dec)
                th.start()
                run_enc()
                th.join()
                ts.append(time.perf_counter() - t0)
            res[kind + "_concurrent"] = min(ts[1:])
            assert int(np.asarray(dl).astype(np.int64).sum()) > 0
            if kind == "packed":  # bytes across the link per step (zero copy): in, offsets, names | out bytes, meta
                h2d = P + 4 * (n + 1) + H + 4 * (n_ok + 1) + 4 * names_np.size
                d2h = int(np.asarray(el).astype(np.int64)[np.asarray(el) != 0xFFFFFFFF].sum()) + 4 * n + \
                    int(np.asarray(dl).astype(np.int64)[np.asarray(dl) != 0xFFFFFFFF].sum()) + 5 * n_ok
                link = {"h2d_bytes": h2d, "d2h_bytes": d2h,
                        "d2h_bytes_with_offsets": d2h + 5 * n + 4 + 4 * n_ok + 4}
    os.environ.pop("HHUFF_HOST_COPY", None)
    # value: the slot-layout pinned path, the same definition as rounds 1-4 (out_off, out_len and status all
    # returned); the packed zero-copy legs, which return less, are reported beside it (packed_*_value)
    best = min(("pinned", "pinned_concurrent"), key=lambda k: res[k])
    t = res[best]
    return {"value": round(P / GIB / t, 3), "unit": "GiB/s", "ms_per_step": round(t * 1e3, 3),
            "best": best,
            "legs": "concurrent" if res["pinned_concurrent"] < res["pinned"] else "sequential",
            "sequential_value": round(P / GIB / res["pinned"], 3),
            "concurrent_value": round(P / GIB / res["pinned_concurrent"], 3),
            "packed_value": round(P / GIB / res["packed"], 3),
            "packed_concurrent_value": round(P / GIB / res["packed_concurrent"], 3),
            "packed_with_offsets_value": round(P / GIB / min(res["packed_off"], res["packed_off_concurrent"]), 3),
            "packed_link_bytes": link,
            "pcie": pcie_rates(torch),
            "pinned_dma_value": round(P / GIB / res["pinned_dma"], 3),
            "pinned_dma_ms_per_step": round(res["pinned_dma"] * 1e3, 3),
            "pageable_value": round(P / GIB / res["pageable"], 3),
            "pageable_ms_per_step": round(res["pageable"] * 1e3, 3),
            "best_packed": round(P / GIB / min(res["packed"], res["packed_concurrent"]), 3),
            "note": "strings start and end in host memory; hhuff_{encode,decode}_batch_host_pipelined: pinned caller "
                    "buffers are read and written by the kernels in place (zero copy), pinned_dma is the chunked DMA "
                    "pipeline on the same buffers (64 MiB chunks, 3 streams), pageable buffers go through it with "
                    "host staging; packed: hhuff_{encode,decode}_batch_host_packed on the pinned buffers (zero copy, "
                    "tile-packed outputs: only output bytes cross the link; out_len and the decode status returned, "
                    "positions implied by them; packed_with_offsets: out_off and the encode status too); value: "
                    "the fastest slot-layout pinned step (best_packed: the fastest packed step), its "
                    "encode and decode legs one after the other or on two host threads at once (`best`); "
                    "best of %d" % reps}


def pcie_rates(torch, nbytes=256 << 20, reps=3):
    """DMA rates of this box's link (GB/s, best of `reps`): pinned host -> device, device -> pinned host, and
    both at once on two streams (the ceiling the host paths share)"""
    h1 = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d1 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def run(h2d, d2h):
        best = None
        for _ in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if h2d:
                with torch.cuda.stream(s1):
                    d1.copy_(h1, non_blocking=True)
            if d2h:
                with torch.cuda.stream(s2):
                    h2.copy_(d2, non_blocking=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        return round((h2d + d2h) * nbytes / best / 1e9, 1)

    out = {"h2d_gbps": run(1, 0), "d2h_gbps": run(0, 1), "bidirectional_gbps": run(1, 1)}
    del h1, h2, d1, d2
    torch.cuda.empty_cache()
    return out


def cgroup_cpus():
    """the CPUs this process's cgroup may use (cpu.max quota / period), or None when unlimited or unknown"""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(b, args):
    """h2o's own CPU path on this host's cores, timed like one step (encode the sample's strings, then decode
    the compressible ones).  kind "reference": oracle/_ref/libh2oref.so -- the reference's lib/http2/hpack.c
    compiled where it lies by oracle/Makefile in the build container; the built .so travels to the GPU box
    with the tree.  kind "port": the clean-room restatement, when that build is absent.  Contiguous
    per-thread ranges over a bounded sample of rank 0's shard; median of 5; plus one thread on 256K strings."""
    import numpy as np

    from oracle import oracle as O

    kind = "reference" if O.ref_available() else "port"
    cdc = O.ref() if kind == "reference" else O.oracle()
    m = min(args.cpu_sample or (1 << 22), b["n"])
    off = b["off"][:m + 1].cpu().numpy().view(np.uint32).astype(np.uint32)
    data = b["data"][:int(off[-1])].cpu().numpy()
    names = b["is_name_bits"][:(m + 31) // 32].cpu().numpy().view(np.uint32)
    affinity = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)  # the box's CPU share per GPU (16 on the GPU pool)
    threads = args.cpu_threads or (min(affinity, share) if share > 0 else affinity)

    def rate(mm, nthreads, reps):
        o = off[:mm + 1]
        d = data[:int(o[-1])]
        enc, el, _ = cdc.encode_batch(d, o, mm, nthreads=nthreads)  # also produces the decode input
        hl = np.where(el != O.FAIL, el, 0).astype(np.uint32)
        starts = o[:-1].copy()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            cdc.encode_batch(d, o, mm, nthreads=nthreads)
            cdc.decode_batch(enc, starts, mm, in_len=hl, is_name_bits=names, nthreads=nthreads)
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return float(o[-1]) / GIB / ts[len(ts) // 2], float(o[-1])

    v, Ps = rate(m, threads, 5)
    m1 = min(m, 1 << 18)
    v1, P1 = rate(m1, 1, 5)
    # every CPU of the affinity mask (one short burst; the host's CPUs serve other GPUs' jobs too,
    # so this measures the box as shared -- its cgroup CPU quota is stated beside it)
    va = rate(m, affinity, 3)[0] if affinity != threads else v
    return {"value": round(v, 4), "unit": "GiB/s", "cores": threads, "affinity_cpus": affinity, "kind": kind,
            "all_cores": {"value": round(va, 4), "cores": affinity, "cgroup_cpu_quota": cgroup_cpus(),
                          "sample": "the same %d strings, %d threads (every CPU of the affinity mask), median of 3"
                                    % (m, affinity)},
            "sample": "%d strings (%.1f MB) of rank 0's shard, encode + decode, median of 5, %d threads of %d in the "
                      "affinity mask (%s)" % (m, Ps / 1e6, threads, affinity,
                                              "oracle/_ref: the reference's lib/http2/hpack.c, compiled" if kind ==
                                              "reference" else "clean-room restatement"),
            "single_thread_value": round(v1, 4),
            "single_thread_sample": "%d strings (%.1f MB), 1 thread, median of 5" % (m1, P1 / 1e6)}


if __name__ == "__main__":
    main()
