#!/usr/bin/env python3
"""bench.py — Ed25519 verifies/s of the at2v hot path on 1..8 MI355X (BASELINE.json metric).

Workload (BASELINE config 2, weak-scaled): every rank verifies its own batch of `--records-per-gpu`
(default 1,048,576) signed transfers with 100-byte messages, generated on the GPU by the deterministic
RFC 8032 generator and resident in HBM before timing starts. One step = one verify
launch over the rank's batch + (N > 1) one RCCL all-gather of the verdict bitmap words over xGMI, both
inside libat2v (at2v_verify_shard_gather_device). Config 3 (16M over 8 GPUs) = `--records-per-gpu 2097152`
at N = 8. Steps alternate over two HIP launch streams, so step k+1's kernel fills the CUs that step k's kernel
leaves during its end-of-launch drain, as consecutive batches of a running node do.

Launch: `python bench.py --gpus N` starts its own N rank processes (children, one per GPU) when it is not
already under torch.distributed.run; under torch.distributed.run each process is one rank.

Output: one JSON line on rank 0 with the contract fields plus `roofline` (VALU-bound), the end-to-end
host-buffer rates (`e2e_verifies_per_s`) and `cpu_baseline` (the oracle on every usable host core, bounded
sample).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "at2-node_amd"))

CFG_SEED = 0x4154325F
_T_START = time.perf_counter()


def progress(msg):
    """one line per phase on stderr (stdout carries only the JSON line): a long default run shows where it is"""
    sys.stderr.write(f"[bench {time.perf_counter() - _T_START:7.1f} s] {msg}\n")
    sys.stderr.flush()

# Algorithmic work per verify (half-size equation, 33-window chain): decode A and R
# 510 S + 44 M, tables [j]A and [j](+-R) 128 M, ladder 32 x (16 S + 28 M) + top window 15 M + 8 fixed-base
# windows x 14 M = 512 S + 1023 M; 1195 M + 1022 S in all. A 10-limb radix-2^25.5 multiplication is 100 and a
# squaring 55 32x32->64 multiply-accumulates. (About 17% of waves need a 34th window, +2.1% work: the figure
# below is the lower bound, so the reported fraction is conservative.)
FIELD_MUL_PER_VERIFY = 1195
FIELD_SQ_PER_VERIFY = 1022
MAC_PER_VERIFY = 100 * FIELD_MUL_PER_VERIFY + 55 * FIELD_SQ_PER_VERIFY  # 175,710
# Peak: v_mad_u64_u32 (the MAC of the unsigned-limb field; v_mad_i64_i32 alike) issues at half the
# VALU rate on gfx950 (profiles/r01_ubench_valu.txt): one wave64 instruction per 4 cycles per SIMD
# = 16 lane-MACs/clk/SIMD x 4 SIMD x 256 CU x 2.4 GHz.
MAC_PEAK = 256 * 4 * 16 * 2.4e9  # 3.93e13 MAC/s
# The comb path of AT2 traffic (DESIGN.md §10d, 10-bit A windows and the wide comb of B's 24-bit windows, four records
# per lane, the bench's at2_traffic leg: a context with AT2V_CTX_BCOMB_WIDE): 26 + 11
# mixed additions with affine entries (7 M), a quarter of a shared inversion (254 S + 11 M) + 2.25 M of Montgomery's
# trick over four Z's, and 2 M to encode R': 266 M + 63.5 S per verify (round 4's 16-bit B windows: 301 M + 63.5 S).
COMB_MAC_PER_VERIFY = 100 * 266 + 55 * 63.5  # 30,092.5
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--records-per-gpu", type=int, default=1 << 20)
    ap.add_argument("--msg-len", type=int, default=100)
    ap.add_argument("--policy", default="dalek")
    ap.add_argument("--senders", type=int, default=0,
                    help="0 = distinct keys (BASELINE config 2); K > 0 = record i signed by sender i %% K (AT2 traffic)")
    ap.add_argument("--sender-cache", type=int, default=0,
                    help="at2v_opts.sender_cache: per-sender A cache capacity in keys (0 = off)")
    ap.add_argument("--sender-comb", type=int, default=0,
                    help="at2v_opts.sender_comb: 1 = per-key combs with the cache (all-hit chunks by table additions)")
    ap.add_argument("--cpu-sample", type=int, default=1 << 20,
                    help="max records for the CPU baseline sample (0 = skip); sized to ~3 s on the threads used")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core this process may run on")
    ap.add_argument("--e2e", type=int, default=1, help="1 = also time the host-buffer path (H2D + verify + D2H)")
    ap.add_argument("--traffic-leg", type=int, default=1,
                    help="1 = at N=1 also time AT2 traffic (the same records per step, signed by 64 repeating senders) "
                         "through per-sender combs (at2v_opts.sender_comb); reported as at2_traffic, not as value")
    ap.add_argument("--churn-legs", default="distinct,zipf,cap4x",
                    help="at N=1 also time sender churn through a comb context, these legs (comma list; 0 = none): "
                         "distinct keys, Zipf(1.1) over 100k senders, 4x the cache's capacity; fresh records every step. "
                         "Reported as sender_churn")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU only (tests): the launcher and gloo control plane with oracle verdicts, no GPU")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="seconds a rank waits in the gloo rendezvous / barriers before giving up (N > 1)")
    ap.add_argument("--pmc-traffic", type=int, default=1,
                    help="1 = at N=1, measure HBM-side bytes per verify launch with two rocprofv3 PMC passes "
                         "(FETCH_SIZE, WRITE_SIZE) of a 2-step child run; 0 = skip (roofline.traffic null)")
    return ap.parse_args()


def _free_port():
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def self_launch(args):
    """`bench.py --gpus N` (N > 1) outside torch.distributed.run: start N rank processes of this script (one per
    GPU) as children, before this process touches any GPU, and pass rank 0's JSON line through. Children, never
    exec: the parent stays a plain process. It watches EVERY child: on the first non-zero exit it stops the other
    ranks (SIGTERM, then SIGKILL after 10 s; by their PIDs) and exits with that status, so a rank that dies early
    cannot leave the others blocked in the gloo rendezvous or inside an RCCL collective until the driver's limit."""
    import subprocess
    import threading
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))
    out = []
    reader = threading.Thread(target=lambda: out.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    failed = None
    while failed is None:
        rcs = [p.poll() for p in procs]
        bad = [(r, rc) for r, rc in enumerate(rcs) if rc not in (None, 0)]
        if bad:
            failed = bad[0]
        elif all(rc == 0 for rc in rcs):
            break
        else:
            time.sleep(0.2)
    if failed is not None:
        sys.stderr.write(f"bench.py: rank {failed[0]} exited with status {failed[1]}; stopping the other ranks\n")
        for p in procs:
            if p.poll() is None:
                p.terminate()
        deadline = time.time() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    reader.join(timeout=10)
    sys.stdout.write(b"".join(out).decode())
    sys.stdout.flush()
    if failed is not None:
        return abs(failed[1]) or 1
    return 0


def usable_cores():
    """(cores this process may use, detail): the CPU affinity set, capped by a cgroup CPU quota if one is set"""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    use = min(aff, quota) if quota else aff
    return use, {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota_cores": quota, "cpu_model": model}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    # stdout carries exactly one line, the JSON result: everything else that writes to fd 1 (RCCL's version
    # banner at communicator init, library chatter) is sent to stderr.
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    import numpy as np
    import torch
    import torch.distributed as dist

    import at2v

    progress("torch and at2v imported")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    # N > 1: one process per GPU. The data path is native: libat2v's own RCCL communicator all-gathers the
    # verdict words over xGMI (at2v_verify_shard_gather_device). torch.distributed (gloo, host) is only the
    # control plane: the RCCL unique id, barriers and the MAX/MIN reductions of timings and checks. Under
    # torch.distributed.run at N = 1 the same path runs with world 1, so a one-GPU box rehearses it.
    use_dist = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    fail_rank = os.environ.get("AT2V_BENCH_FAIL_RANK")  # failure injection (tests/test_bench_launch.py)
    if fail_rank is not None and int(fail_rank) == rank:
        raise SystemExit(f"rank {rank}: injected failure (AT2V_BENCH_FAIL_RANK)")
    if use_dist:
        import datetime
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=args.dist_timeout))
    if args.dry_run:
        out = dry_run(args, rank, world, use_dist, dist, torch, np)
        if rank == 0:
            os.write(json_fd, (json.dumps(out) + "\n").encode())
        if use_dist:
            dist.destroy_process_group()
        return
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    n, L = args.records_per_gpu, args.msg_len
    n = (n + 63) // 64 * 64
    v = at2v.BatchVerifier(device=local, policy=args.policy, sender_cache=args.sender_cache,
                           sender_comb=bool(args.sender_comb))
    if use_dist:
        uid = [at2v.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        v.comm_init_rank(uid[0], rank, world)
    stream = torch.cuda.current_stream(dev)
    s = stream.cuda_stream
    # Steps alternate over two launch streams (their own hardware queues): step k+1's kernel fills the CUs step k's
    # kernel leaves during its end-of-launch drain (the library gives each in-flight launch its own scratch set).
    lstreams = at2v.launch_streams(2, local)
    d_pk = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_sig = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    d_msg = torch.empty(n * L, dtype=torch.uint8, device=dev)
    d_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    words = n // 32
    # one verdict bitmap per launch stream, so overlapping steps never write the same words
    d_vers = [torch.zeros(words, dtype=torch.int32, device=dev) for _ in lstreams]
    d_alls = [torch.zeros(words * world, dtype=torch.int32, device=dev) for _ in lstreams]  # node bitmaps (N > 1)
    d_ver, d_all = d_vers[0], d_alls[0]
    # distinct records per rank (indices rank*n .. rank*n+n-1)
    v.gen_records_device(CFG_SEED, rank * n, n, L, d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                         d_off.data_ptr(), s, senders=args.senders)
    torch.cuda.synchronize(dev)

    def verify(pk, sig, msg, off, j):
        """one step on launch stream j (its own verdict bitmap)"""
        strm = lstreams[j].cuda_stream
        if use_dist:  # verify this rank's shard into its slice of the node bitmap, then RCCL all-gather
            v.verify_shard_gather_device(pk, sig, msg, n * L, off, n, words, d_alls[j].data_ptr(), strm)
        else:
            v.verify_batch_device(pk, sig, msg, n * L, off, n, d_vers[j].data_ptr(), strm)

    def barrier():
        torch.cuda.synchronize(dev)
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def reduce(vals, op):
        t = torch.tensor(vals, dtype=torch.float64)
        if use_dist:
            dist.all_reduce(t, op=op)
        return t.tolist()

    ptrs = (d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), d_off.data_ptr())
    for k in range(args.warmup):
        verify(*ptrs, k % 2)
    barrier()
    # HIP events on the launch streams: one start (both streams wait for it) and one end per step, recorded on that
    # step's stream right after its launch. Device time per step = (last end - start) / K: the period of the
    # overlapped launches, i.e. the device-side throughput of the timed region.
    ev0 = torch.cuda.Event(enable_timing=True)
    kend = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    t0 = time.perf_counter()
    ev0.record(lstreams[0])
    lstreams[1].wait_event(ev0)
    for k in range(args.steps):
        verify(*ptrs, k % 2)
        kend[k].record(lstreams[k % 2])
    barrier()
    elapsed = time.perf_counter() - t0
    # device time per step on the launch streams: the verify kernels (N = 1) or kernels + all-gathers (N > 1)
    kernel_ms = max(ev0.elapsed_time(e) for e in kend) / args.steps
    # one launch alone (nothing before or after it on the device): its duration is what a kernel-trace profile of a
    # single launch reports; the timed steps overlap by up to the end-of-launch drain
    ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ea.record(lstreams[0])
    verify(*ptrs, 0)
    eb.record(lstreams[0])
    barrier()
    launch_ms_alone = ea.elapsed_time(eb)
    kernel_ms_local, elapsed_local, launch_alone_local = kernel_ms, elapsed, launch_ms_alone
    progress(f"timed steps done: {kernel_ms:.3f} ms per step on the device")
    elapsed, kernel_ms, launch_ms_alone = reduce([elapsed, kernel_ms, launch_ms_alone],
                                                 dist.ReduceOp.MAX if use_dist else None)

    # verdict check after the timed region: every generated record must be valid, on every rank (N > 1: the
    # gathered node bitmaps, all ranks' records), in the bitmap of every launch stream the steps used
    used = d_alls if use_dist else d_vers
    used = used[: min(2, max(1, args.steps + args.warmup))]
    match = min(float((full == -1).float().mean().item()) for full in used)
    match = reduce([match], dist.ReduceOp.MIN)[0] if use_dist else match

    multi = multi_gpu_diagnostics(args, v, barrier, dist, torch, lstreams, ptrs, n, L, words, d_vers, d_alls, world,
                                  kernel_ms_local, elapsed_local, launch_alone_local) if use_dist else None

    e2e = host_path(args, v, verify, barrier, reduce, dist, torch, dev, lstreams, d_pk, d_sig, d_msg, d_off, d_vers,
                    d_alls, n, L, words, use_dist, world) if args.e2e else None

    total = n * world * args.steps
    value = total / elapsed
    per_gpu_kernel_rate = n / (kernel_ms * 1e-3)
    # the comb path (repeating senders with combs as the main leg) does far fewer MACs per verify than the ladder
    macs = COMB_MAC_PER_VERIFY if (args.senders and args.sender_cache and args.sender_comb) else MAC_PER_VERIFY
    achieved = per_gpu_kernel_rate * macs / 1e12
    info = v.info()

    out = None
    if rank == 0:
        if world == 8 and n == 2 * (1 << 20):
            workload = "BASELINE config 3: 16M signatures index-sharded over 8 MI355X + RCCL all-gather of the verdict bitmap"
        elif args.senders:
            workload = (f"{n} signed transfers per GPU ({L}-byte M) from {args.senders} repeating senders (AT2 traffic)"
                        + (f", per-sender A cache of {args.sender_cache} keys" if args.sender_cache else ", no cache")
                        + (" with per-key combs" if args.sender_cache and args.sender_comb else ""))
        elif n == 1 << 20:
            workload = (f"BASELINE config 2: 1M signed transfers per GPU (100-byte M), dalek-1.x verify"
                        + (f"; {world} GPUs, weak scaling, RCCL all-gather of the verdict bitmap" if world > 1 else ""))
        else:
            workload = f"{n} signed transfers per GPU ({L}-byte M)"
        out = {
            "metric": "ed25519 verifies/sec (node)",
            "value": value,
            "unit": "verifies/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (GPU RFC 8032 generator, distinct keys, all signatures valid)",
            "config": {
                "workload": workload,
                "records_per_gpu": n,
                "msg_len": L,
                "policy": args.policy,
                "senders": args.senders or "distinct",
                "sender_cache": args.sender_cache,
                "sender_comb": bool(args.sender_cache and args.sender_comb),
                "parallelism": f"index-shard x{world}" + (" + RCCL all-gather of verdict words (libat2v)" if use_dist else ""),
            },
            "verdict_match": match,
            "kernel_ms": kernel_ms,
            "launch_ms_alone": launch_ms_alone,
            "launch_overlap": "steps alternate over two HIP streams (own hardware queues); each in-flight launch has "
                              "its own scratch set, so step k+1's blocks take the CUs step k's last blocks leave. "
                              "kernel_ms = device time per step over the timed region (HIP events); launch_ms_alone = "
                              "one launch with the device otherwise idle",
            "effective_clock_ghz": None,
            "kernel": {"grid_blocks": info["grid_blocks"], "block": info["block_threads"],
                       "waves_per_cu": info["waves_per_cu"], "vgprs": info["vgprs"]},
            "roofline": {
                "bound": "valu",
                "achieved": achieved,
                "peak": MAC_PEAK / 1e12,
                "unit": "Tops/s (32x32->64 integer MAC, v_mad_u64_u32)",
                "frac": achieved * 1e12 / MAC_PEAK,
                "traffic": None,
                "alg_macs_per_verify": macs,
                "alg_bytes_per_verify": 32 + 64 + L + 4,
                # algorithmic input rate (records x 200 B / kernel time); the measured memory-side rate from the
                # PMC counters is hbm_gbs (filled below at N = 1 when the counter passes run)
                "alg_input_gbs": per_gpu_kernel_rate * (32 + 64 + L + 4) / 1e9,
                "hbm_gbs": None,
                "hbm_frac": None,
            },
        }
        if e2e:
            out.update(e2e)
        if multi:
            out["multi_gpu"] = multi
    if e2e:
        progress("host-buffer leg done")
    if rank == 0 and world == 1 and args.e2e and not use_dist:
        out.update(abi_host_leg(args, v, d_pk, d_sig, d_msg, d_off, n, L, value))
        progress("library host-buffer call leg done")
    if rank == 0 and world == 1 and args.traffic_leg and not args.senders and not use_dist:
        progress("AT2-traffic leg")
        out["at2_traffic"] = at2_traffic_leg(args, at2v, torch, dev, lstreams, n, L)
    if rank == 0 and world == 1 and args.churn_legs not in ("", "0") and not args.senders and not use_dist:
        out["sender_churn"] = churn_legs(args, at2v, torch, dev, lstreams, n, L, kernel_ms, value)
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        progress("CPU baseline")
        out["cpu_baseline"] = cpu_baseline(args, d_pk, d_sig, d_msg, n, L)
    if rank == 0 and world == 1 and args.pmc_traffic and not use_dist:
        progress("PMC passes")
        tr = pmc_traffic(args, n, L)
        if tr is not None:
            out["roofline"]["traffic"] = tr["bytes_per_launch"]
            out["roofline"]["traffic_detail"] = tr
            # memory-side bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, L2's fabric side: MALL hits included, so an
            # upper bound on HBM bytes) over the un-profiled kernel time of this run
            out["roofline"]["hbm_gbs"] = tr["bytes_per_launch"] / (kernel_ms * 1e-3) / 1e9
            out["roofline"]["hbm_frac"] = out["roofline"]["hbm_gbs"] / HBM_PEAK_GBS
        vl = pmc_valu(args, n, L)
        if vl is not None:
            out["roofline"]["valu_measured"] = vl
            out["effective_clock_ghz"] = vl["effective_clock_ghz"]
    if rank == 0:
        progress("done")
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    v.close()
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


def at2_traffic_leg(args, at2v, torch, dev, lstreams, n, L, senders=64):
    """AT2 traffic: n records per step signed by `senders` repeating keys (record i by sender
    i % senders), verified through a context with the per-sender cache and combs; the combs are built by the first
    (warm-up) launch. Same step structure as the headline (overlapped launches on the two streams). Reported beside the
    headline value, which stays the distinct-key workload of BASELINE config 2."""
    t_create = time.perf_counter()
    v = at2v.BatchVerifier(device=dev.index or 0, policy=args.policy, sender_cache=1024, sender_comb=True,
                           bcomb_wide=True)
    t_create = time.perf_counter() - t_create
    bufs = [torch.empty(n * 32, dtype=torch.uint8, device=dev), torch.empty(n * 64, dtype=torch.uint8, device=dev),
            torch.empty(n * L, dtype=torch.uint8, device=dev), torch.empty(n + 1, dtype=torch.int32, device=dev)]
    vers = [torch.zeros(n // 32, dtype=torch.int32, device=dev) for _ in lstreams]
    v.gen_records_device(CFG_SEED, 0, n, L, *(b.data_ptr() for b in bufs), lstreams[0].cuda_stream, senders=senders)
    torch.cuda.synchronize(dev)
    ptrs = [b.data_ptr() for b in bufs]

    def step(k):
        j = k % 2
        v.verify_batch_device(ptrs[0], ptrs[1], ptrs[2], n * L, ptrs[3], n, vers[j].data_ptr(), lstreams[j].cuda_stream)

    for k in range(3):  # (a key claims its comb at its second sighting: launch 1 sights, launch 2 claims)
        step(k)
    torch.cuda.synchronize(dev)
    v.info()  # (waits for the context's build stream)
    steps = max(2, args.steps)
    ev0 = torch.cuda.Event(enable_timing=True)
    kend = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    t0 = time.perf_counter()
    ev0.record(lstreams[0])
    lstreams[1].wait_event(ev0)
    for k in range(steps):
        step(k)
        kend[k].record(lstreams[k % 2])
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    kernel_ms = max(ev0.elapsed_time(e) for e in kend) / steps
    ok = all(bool((x == -1).all().item()) for x in vers)
    info = v.info()
    v.close()
    return {"value": n * steps / dt, "unit": "verifies/s", "records_per_step": n, "senders": senders, "steps": steps,
            "ms_per_step": dt * 1e3 / steps, "kernel_ms": kernel_ms, "verdicts_ok": ok,
            "context_create_s": t_create,
            "cache_chunk_hits": info["cache_chunk_hits"],
            "cache_chunks": info["cache_chunks"],
            "cache_record_hits": info["cache_record_hits"],
            "roofline": {"bound": "valu", "alg_macs_per_verify": COMB_MAC_PER_VERIFY,
                         "achieved": n * steps / dt * COMB_MAC_PER_VERIFY / 1e12, "peak": MAC_PEAK / 1e12,
                         "unit": "Tops/s (32x32->64 integer MAC, v_mad_u64_u32)",
                         "frac": n * steps / dt * COMB_MAC_PER_VERIFY / MAC_PEAK,
                         "note": "at the wall-clock step rate (launch gaps included); 266 M + 63.5 S per verify "
                                 "(affine comb entries; four records per lane share one inversion)"},
            "method": f"{n} records per step (100-byte M) signed by {senders} repeating senders (GPU generator, record i "
                      f"by sender i % {senders}), sender_cache 1024 + sender_comb: chunks whose senders are all cached "
                      "verify by comb additions (DESIGN §10d), wide comb of B (AT2V_CTX_BCOMB_WIDE, 24-bit windows); combs built in the "
                      "warm-up. kernel_ms = device time per "
                      "step on the launch streams (HIP events: the verify kernel and the cache-counter copy; the build "
                      "and flip kernels run on the context's own stream)"}


def churn_legs(args, at2v, torch, dev, lstreams, n, L, plain_kernel_ms, plain_value):
    """Sender churn through a comb context (VERDICT r4 "missing" 3 / "Next" 4): what a node with per-sender combs
    (sender_cache 1024 keys, sender_comb) pays when its traffic is not 64 loyal senders. Every step verifies a FRESH
    batch of n records (new messages, so nothing repeats unless the key does), drawn per leg:
      distinct  every record a new key (BASELINE config 2's key distribution through the comb context);
      zipf      keys Zipf(1.1) over 100,000 senders (a few heavy senders, a long tail of one-shot ones);
      cap4x     keys uniform over 4,096 senders, 4x the cache's capacity (continuous replacement).
    A key claims its comb at its second sighting (admission), combs are built on the context's stream, compactions
    run there too; at most two batches are in flight (a node's queue of depth 3); the timed region ends after that stream has drained (v.info()), so builds and compactions are
    charged to the leg. Per leg: wall-clock rate, device time of the launch streams, chunk hit rate, claims, builds
    and their device time, compactions, sightings; vs_plain = this leg's rate over the headline's (distinct keys,
    no cache)."""
    steps, warm = max(2, args.steps), 6  # (six warm-up batches: admission, builds and a compaction reach steady state)
    nb = steps + warm
    gen = torch.Generator(device=dev)
    gen.manual_seed(0x5EED)
    zipf_p = torch.arange(1, 100_001, device=dev, dtype=torch.float64).pow(-1.1)
    legs = {
        "distinct": lambda b: torch.arange(b * n, (b + 1) * n, device=dev, dtype=torch.int64) + (1 << 36),
        "zipf": lambda b: torch.multinomial(zipf_p, n, replacement=True, generator=gen) + (1 << 37),
        "cap4x": lambda b: torch.randint(0, 4096, (n,), device=dev, generator=gen) + (1 << 38),
    }
    out = {}
    for name, keys_of in legs.items():
        if name not in args.churn_legs.split(","):
            continue
        progress(f"churn leg {name}")
        v = at2v.BatchVerifier(device=dev.index or 0, policy=args.policy, sender_cache=1024, sender_comb=True)
        batches, key_bufs = [], []
        for b in range(nb):
            keys = keys_of(b).contiguous()
            key_bufs.append(keys)  # (alive until the generator, on another stream, has read it)
            bufs = [torch.empty(n * 32, dtype=torch.uint8, device=dev), torch.empty(n * 64, dtype=torch.uint8, device=dev),
                    torch.empty(n * L, dtype=torch.uint8, device=dev), torch.empty(n + 1, dtype=torch.int32, device=dev)]
            v.gen_records_keys_device(CFG_SEED, (1 << 40) + b * n, n, L, keys.data_ptr(), *(x.data_ptr() for x in bufs),
                                      lstreams[0].cuda_stream)
            batches.append(bufs)
        torch.cuda.synchronize(dev)
        distinct_keys = None
        if name != "distinct":
            distinct_keys = int(torch.unique(keys).numel())  # (the last batch's)
        del keys, key_bufs
        vers = [torch.zeros(n // 32, dtype=torch.int32, device=dev) for _ in lstreams]
        torch.cuda.synchronize(dev)

        def step(k):
            j = k % 2
            b = batches[k]
            v.verify_batch_device(b[0].data_ptr(), b[1].data_ptr(), b[2].data_ptr(), n * L, b[3].data_ptr(), n,
                                  vers[j].data_ptr(), lstreams[j].cuda_stream)

        progress(f"churn leg {name}: {nb} batches generated")
        for k in range(warm):
            step(k)
        torch.cuda.synchronize(dev)
        h0 = v.info()
        progress(f"churn leg {name}: warm-up done")
        ev0 = torch.cuda.Event(enable_timing=True)
        kend = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
        t0 = time.perf_counter()
        ev0.record(lstreams[0])
        lstreams[1].wait_event(ev0)
        for k in range(steps):
            if k >= 2:  # at most two batches in flight, as a node's ingest queue (depth 3) has: the host keeps up with
                kend[k - 2].synchronize()  # the cache counters, so compactions and claims happen between batches
            step(warm + k)
            kend[k].record(lstreams[k % 2])
        torch.cuda.synchronize(dev)
        h1 = v.info()  # (waits for the context's stream: its builds and compactions are inside the timed region)
        dt = time.perf_counter() - t0
        kernel_ms = max(ev0.elapsed_time(e) for e in kend) / steps
        ok = all(bool((x == -1).all().item()) for x in vers)
        d = {k: h1[k] - h0[k] for k in ("cache_chunks", "cache_chunk_hits", "cache_claims", "cache_built",
                                         "cache_build_us", "cache_compactions", "cache_evicted", "cache_sightings",
                                         "cache_record_hits")}
        rate = n * steps / dt
        out[name] = {"value": rate, "unit": "verifies/s", "ms_per_step": dt * 1e3 / steps, "kernel_ms": kernel_ms,
                     "vs_plain": rate / plain_value, "kernel_vs_plain": plain_kernel_ms / kernel_ms,
                     "record_hit_rate": d["cache_record_hits"] / (n * steps),
                     "chunk_hit_rate": d["cache_chunk_hits"] / max(1, d["cache_chunks"]),
                     "claims_per_step": d["cache_claims"] / steps, "combs_built_per_step": d["cache_built"] / steps,
                     "build_ms_per_step": d["cache_build_us"] / 1e3 / steps,
                     "compactions": d["cache_compactions"], "evicted": d["cache_evicted"],
                     "sightings_per_step": d["cache_sightings"] / steps, "cache_entries": h1["cache_entries"],
                     "distinct_keys_per_batch": distinct_keys if distinct_keys is not None else n,
                     "verdicts_ok": ok, "steps": steps, "warmup": warm}
        v.close()
        del batches, vers
        torch.cuda.empty_cache()
    out["method"] = ("fresh records every step (GPU generator with a key per record, at2v_gen_records_keys_device), "
                     f"{n} records per step, sender_cache 1024 + sender_comb, two launch streams; wall clock from the "
                     "first launch to the context's stream drained (builds and compactions included); record_hit_rate = "
                     "records verified from their sender's comb (each launch is classified, then the hit list runs "
                     "the comb kernel and the miss list the ladder); chunk_hit_rate = 64-record groups whose senders "
                     "were all cached (what round 4's kernels needed); kernel_ms = device time per step on the launch "
                     "streams (HIP events)")
    return out


def multi_gpu_diagnostics(args, v, barrier, dist, torch, lstreams, ptrs, n, L, words, d_vers, d_alls, world,
                          kernel_ms, elapsed, launch_alone):
    """N > 1 (and the world-1 torchrun rehearsal): what a sub-linear scaling curve needs to be read.
    Per rank: the timed region's device time per step (verify + all-gather, `kernel_ms`), its wall time, one launch
    alone, then two extra measurements on the same launch stream with HIP events: verify-only steps (the rank's shard,
    no collective) and gather-only steps (an empty shard: the slice zeroing + the RCCL all-gather of `words` words per
    rank), so kernel time, collective time and a slow rank separate. All gathered to rank 0 over gloo."""
    steps = max(2, args.steps)

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        barrier()
        e0.record(lstreams[0])
        for _ in range(steps):
            fn()
        e1.record(lstreams[0])
        barrier()
        return e0.elapsed_time(e1) / steps

    s0 = lstreams[0].cuda_stream
    verify_ms = timed(lambda: v.verify_batch_device(*ptrs[:3], n * L, ptrs[3], n, d_vers[0].data_ptr(), s0))
    gather_ms = timed(lambda: v.verify_shard_gather_device(0, 0, 0, 0, 0, 0, words, d_alls[0].data_ptr(), s0))
    mine = torch.tensor([kernel_ms, elapsed, launch_alone, verify_ms, gather_ms], dtype=torch.float64)
    allr = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    per = [r.tolist() for r in allr]
    col = lambda j: [p[j] for p in per]  # noqa: E731
    km = col(0)
    return {"ranks": world, "kernel_ms_per_rank": km, "kernel_ms_min": min(km), "kernel_ms_max": max(km),
            "max_rank": int(max(range(world), key=lambda r: km[r])), "elapsed_s_per_rank": col(1),
            "launch_ms_alone_per_rank": col(2), "verify_only_ms_per_rank": col(3), "gather_only_ms_per_rank": col(4),
            "gather_words_per_rank": words, "gather_bytes_per_step": 4 * words * world,
            "method": "per-rank HIP events on launch stream 0: kernel_ms = the timed region (verify + RCCL all-gather per "
                      "step, two streams); verify_only = the rank's shard without the collective; gather_only = "
                      f"at2v_verify_shard_gather_device with an empty shard ({steps} steps each); gathered over gloo"}


def dry_run(args, rank, world, use_dist, dist, torch, np):
    """CPU rehearsal of the multi-rank bench (tests/test_bench_launch.py): the same launcher, env and gloo control
    plane; each rank's verdict words come from the oracle over its index shard of a small node batch and are
    all-gathered over gloo (standing in for the library's RCCL all-gather), then checked on every rank."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py
    from at2v import dist as at2dist

    n = min(args.records_per_gpu, 4096) * world
    o = oracle_py.Oracle()
    pk, sig, msg, off, cls = o.gen_adversarial(CFG_SEED, 0, n, args.msg_len, threads=2)
    want = o.verify_batch(pk, sig, msg, off, 0, 2)
    uid = [bytes(range(128)) if rank == 0 else None]  # the RCCL unique id hand-off, as in main()
    if use_dist:
        dist.broadcast_object_list(uid, src=0)
    lo, hi = at2dist.shard_bounds(n, world)[rank]
    per = at2dist.padded_words_per_rank(n, world)
    bits = np.zeros(per * 32, np.uint8)
    t0 = time.perf_counter()
    if hi > lo:
        bits[: hi - lo] = o.verify_batch(pk[lo:hi], sig[lo:hi], msg, off[lo:hi + 1], 0, 2)
    verify_ms = (time.perf_counter() - t0) * 1e3
    local = torch.from_numpy(np.packbits(bits, bitorder="little").view(np.int32).copy())
    t0 = time.perf_counter()
    full = at2dist.gather_verdicts(local, world) if use_dist else local
    gather_ms = (time.perf_counter() - t0) * 1e3
    got = at2dist.node_bitmap_from_shards(full, n, world)
    match = float((got == want).mean())
    t = torch.tensor([match, float(uid[0] == bytes(range(128)))], dtype=torch.float64)
    if use_dist:
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        dist.barrier()
    out = {"dry_run": True, "n_gpus": world, "records": n, "verdict_match": t[0].item(),
           "unique_id_shared": bool(t[1].item()), "valid": int(want.sum())}
    if use_dist:  # the multi_gpu keys of the GPU line, from the CPU stand-ins (oracle verify, gloo gather)
        mine = torch.tensor([verify_ms + gather_ms, verify_ms, gather_ms], dtype=torch.float64)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        km = [r[0].item() for r in allr]
        out["multi_gpu"] = {"ranks": world, "kernel_ms_per_rank": km, "kernel_ms_min": min(km), "kernel_ms_max": max(km),
                            "max_rank": int(max(range(world), key=lambda r: km[r])),
                            "verify_only_ms_per_rank": [r[1].item() for r in allr],
                            "gather_only_ms_per_rank": [r[2].item() for r in allr], "gather_words_per_rank": per}
    return out


def host_path(args, v, verify, barrier, reduce, dist, torch, dev, lstreams, d_pk, d_sig, d_msg, d_off, d_vers, d_alls,
              n, L, words, use_dist, world):
    """End to end from pinned host buffers: per step H2D of the rank's records, verify (+ the RCCL
    all-gather at N > 1), D2H of the verdict bitmap.
      serial:    the three in order on one stream (what at2v_verify_batch does per call);
      pipelined: two device input sets, uploads on a copy stream, so batch k+1 uploads while batch k verifies,
                 verifies alternating over the two launch streams (what the ingest queue does); the D2H of each
                 bitmap follows its verify.
    Whole-job rates (all ranks' records / MAX over ranks of the wall time)."""
    h = [t.cpu().pin_memory() for t in (d_pk, d_sig, d_msg, d_off)]
    bitmaps = d_alls if use_dist else d_vers
    h_outs = [torch.empty(b.numel(), dtype=torch.int32).pin_memory() for b in bitmaps]
    sets = [[torch.empty_like(t) for t in (d_pk, d_sig, d_msg, d_off)] for _ in range(2)]
    copy = torch.cuda.Stream(dev)
    steps = max(1, args.steps)

    def upload(dst, strm):
        with torch.cuda.stream(strm):
            for a, b in zip(dst, h):
                a.copy_(b, non_blocking=True)

    def run(pipelined):
        up = [torch.cuda.Event() for _ in range(2)]
        free = [torch.cuda.Event() for _ in range(2)]
        for j, e in enumerate(free):
            e.record(lstreams[j])
        for o in h_outs:
            o.zero_()
        barrier()
        t0 = time.perf_counter()
        for k in range(steps):
            j = k % 2 if pipelined else 0
            b = sets[j]
            stream = lstreams[j]
            if pipelined:
                copy.wait_event(free[j])
                upload(b, copy)
                up[j].record(copy)
                stream.wait_event(up[j])
            else:
                upload(b, stream)
            verify(b[0].data_ptr(), b[1].data_ptr(), b[2].data_ptr(), b[3].data_ptr(), j)
            free[j].record(stream)
            with torch.cuda.stream(stream):
                h_outs[j].copy_(bitmaps[j], non_blocking=True)
            if not pipelined:
                stream.synchronize()
        barrier()
        dt = reduce([time.perf_counter() - t0], dist.ReduceOp.MAX if use_dist else None)[0]
        ok = all(bool((h_outs[j] == -1).all()) for j in range(2 if pipelined and steps > 1 else 1))
        return n * world * steps / dt, ok

    upload(sets[1], lstreams[0])  # warm both sets
    serial, ok1 = run(False)
    piped, ok2 = run(True)
    return {"e2e_verifies_per_s": piped, "e2e_serial_verifies_per_s": serial,
            "e2e": {"records_per_step_per_gpu": n, "steps": steps, "h2d_bytes_per_step_per_gpu": n * (32 + 64 + L + 4) + 4,
                    "verdicts_ok": ok1 and ok2,
                    "method": "pinned host batch -> H2D -> verify" + (" + RCCL all-gather" if use_dist else "") +
                              " -> D2H bitmap; serial = one stream; pipelined = uploads on a second stream, two "
                              "device input sets (the ingest queue's overlap)"}}


def abi_host_leg(args, v, d_pk, d_sig, d_msg, d_off, n, L, headline):
    """The library's own host-buffer call (VERDICT r5 "Next" 1): at2v_verify_batch on PAGEABLE numpy arrays of the
    same n records, as a node's ingest calls it (consumer rpc.rs:156-173). Each call is synchronous
    and self-contained: the library stages the batch through its pinned chunk pipeline (host copy threads -> DMA upload
    -> verify launches on two streams, at2v_api.hip HostPipe), downloads the verdict words and returns. One warm-up call
    (it allocates the staging), then K timed calls back to back; rate = K n / wall time."""
    import numpy as np

    lib = v._lib
    pk = d_pk.cpu().numpy()
    sig = d_sig.cpu().numpy()
    msg = d_msg.cpu().numpy()
    off = d_off.cpu().numpy().view(np.uint32)
    words = np.zeros(n // 32 + 1, np.uint32)
    ptrs = (pk.ctypes.data, sig.ctypes.data, msg.ctypes.data, off.ctypes.data)

    def call():
        rc = lib.at2v_verify_batch(v._h, *ptrs, n, words.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"at2v_verify_batch failed: {rc}")

    call()
    steps = max(2, args.steps)
    t0 = time.perf_counter()
    for _ in range(steps):
        call()
    dt = time.perf_counter() - t0
    ok = bool((words[: n // 32] == 0xFFFFFFFF).all())
    rate = n * steps / dt
    # the same batches through at2v_verify_batch_submit / _wait with two in flight (the caller stages batch i+1 while
    # batch i verifies): what a node that keeps the device fed gets from the host-buffer entry point
    import ctypes
    words2 = [np.zeros(n // 32 + 1, np.uint32) for _ in range(2)]
    tickets = [ctypes.c_uint64(0) for _ in range(steps + 1)]

    def submit(i):
        rc = lib.at2v_verify_batch_submit(v._h, *ptrs, n, words2[i % 2].ctypes.data, ctypes.byref(tickets[i]))
        if rc != 0:
            raise RuntimeError(f"at2v_verify_batch_submit failed: {rc}")

    def wait(i):
        rc = lib.at2v_verify_batch_wait(v._h, tickets[i].value)
        if rc != 0:
            raise RuntimeError(f"at2v_verify_batch_wait failed: {rc}")

    submit(0)
    wait(0)
    t0 = time.perf_counter()
    for i in range(1, steps + 1):
        submit(i)
        if i > 1:
            wait(i - 1)
    wait(steps)
    dta = time.perf_counter() - t0
    ok_a = all(bool((w[: n // 32] == 0xFFFFFFFF).all()) for w in words2)
    rate_a = n * steps / dta
    return {"e2e_abi_verifies_per_s": rate,
            "e2e_abi_async_verifies_per_s": rate_a,
            "e2e_abi_async": {"records_per_call": n, "calls": steps, "ms_per_call": dta * 1e3 / steps,
                              "vs_headline": rate_a / headline, "verdicts_ok": ok_a,
                              "method": "at2v_verify_batch_submit / _wait on the same pageable arrays, two calls in "
                                        "flight: batch i+1 is staged while batch i verifies"},
            "e2e_abi": {"records_per_call": n, "calls": steps, "ms_per_call": dt * 1e3 / steps,
                        "vs_headline": rate / headline, "verdicts_ok": ok,
                        "method": "at2v_verify_batch (the library's synchronous host-buffer entry point) on pageable "
                                  "numpy arrays, one call per batch, back to back; inside: chunked pinned staging "
                                  "(65,536 records twice, then 131,072), copy-pool threads, SDMA uploads through HSA, "
                                  "each chunk launched once its uploads landed, launches alternating over two "
                                  "streams, verdict words downloaded at the end of the call"}}


def _pmc_pass(args, n, L, counters):
    """One rocprofv3 --pmc pass (counters that fit one pass) over a 2-step child run of this script.
    Returns ({counter: mean value per verify_kernel dispatch}, mean kernel duration in s from the same
    pass's kernel trace), or None if rocprofv3 is absent or the pass fails (bounded by a hard timeout)."""
    import csv
    import shutil
    import subprocess
    import tempfile

    exe = shutil.which("rocprofv3")
    if exe is None:
        return None
    d = tempfile.mkdtemp(prefix="at2v_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    cmd = ["timeout", "-s", "KILL", "120", exe, "--pmc", *counters, "--kernel-trace", "--output-format", "csv",
           "-d", d, "-o", "run", "--", sys.executable, os.path.abspath(__file__), "--steps", "2",
           "--warmup", "2" if args.senders else "0",  # repeating senders: the keys are cached by the profiled steps
           "--cpu-sample", "0", "--pmc-traffic", "0", "--records-per-gpu", str(n), "--msg-len", str(L),
           "--policy", args.policy, "--senders", str(args.senders), "--sender-cache", str(args.sender_cache),
           "--sender-comb", str(args.sender_comb), "--e2e", "0", "--traffic-leg", "0", "--churn-legs", "0"]
    progress(f"PMC pass {' '.join(counters)}")
    try:
        subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=150, check=True)
        rows, durs = [], []
        for root, _, files in os.walk(d):
            for f in files:
                with open(os.path.join(root, f)) as fp:
                    if f.endswith("counter_collection.csv"):
                        rows += [r for r in csv.DictReader(fp) if "verify_kernel" in r["Kernel_Name"]]
                    elif f.endswith("kernel_trace.csv"):
                        durs += [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
                                 for r in csv.DictReader(fp) if "verify_kernel" in r["Kernel_Name"]]
        out = {}
        for ctr in counters:
            per = {}
            for r in rows:  # one row per dispatch (and per agent/XCD if split): sum by dispatch
                if r["Counter_Name"] == ctr:
                    k = int(r.get("Dispatch_Id", "0"))
                    per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
            if not per:
                return None
            if args.senders:  # the two timed steps only (the warm-up launches claim and build the keys)
                per = {k: per[k] for k in sorted(per)[-2:]}
            out[ctr] = sum(per.values()) / len(per)
        if args.senders:
            durs = durs[-2:]
        return out, (sum(durs) / len(durs) if durs else None)
    except (subprocess.SubprocessError, OSError, KeyError, ValueError):
        return None
    finally:
        shutil.rmtree(d, ignore_errors=True)


def pmc_traffic(args, n, L):
    """Memory-side bytes per verify launch from rocprofv3 PMC counters, per the MI355X guide's HBM section:
    FETCH_SIZE (KiB; gfx950 reports half the bytes of wide reads -> x2) and WRITE_SIZE (KiB), one pass each
    (they cannot share a pass). The counters sit on the L2's fabric side: Infinity-Cache (MALL) hits are
    included, so this is an upper bound on HBM bytes. Returns None if a pass fails."""
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        r = _pmc_pass(args, n, L, [ctr])
        if r is None:
            return None
        vals[ctr] = r[0][ctr]
    fetch = vals["FETCH_SIZE"] * 1024 * 2
    write = vals["WRITE_SIZE"] * 1024
    return {"bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
            "bytes_per_verify": (fetch + write) / n, "records_per_launch": n,
            "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) / WRITE_SIZE (KiB), separate passes, child run"}


def pmc_valu(args, n, L):
    """Measured VALU work and issue rate of the verify kernel (SURVEY 8(d) '% VALU peak'), one PMC pass:
    SQ_INSTS_VALU (wave instructions), its INT64 part (v_mad_u64_u32, 64-bit shifts/adds: half rate on
    gfx950) and GRBM_GUI_ACTIVE (summed over the 8 XCDs -> effective clock, MI355X guide 'DVFS give-back').
    Issue fraction: nominal SIMD cycles of the mix (half-rate wave64 op 4 cycles, full-rate 2; every non-INT64
    op is priced at 2, so this is a lower bound) over the cycles the 1024 SIMDs had at the effective clock."""
    r = _pmc_pass(args, n, L, ["SQ_INSTS_VALU", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_INT32", "GRBM_GUI_ACTIVE"])
    if r is None or r[1] is None:
        return None
    c, t = r
    valu, i64 = c["SQ_INSTS_VALU"], c["SQ_INSTS_VALU_INT64"]
    clk = c["GRBM_GUI_ACTIVE"] / 8 / t
    simd_cycles = 1024 * clk * t
    issue = (4 * i64 + 2 * (valu - i64)) / simd_cycles
    lane_ops = valu * 64
    return {"valu_wave_insts_per_launch": valu, "int64_share": i64 / valu,
            "int32_share": c["SQ_INSTS_VALU_INT32"] / valu,
            "valu_lane_ops_per_verify": lane_ops / n, "valu_lane_ops_per_s": lane_ops / t,
            "frac_full_rate_peak_2400mhz": lane_ops / t / (1024 * 32 * 2.4e9),
            "effective_clock_ghz": clk / 1e9, "issue_frac_nominal": issue, "kernel_s_profiled": t,
            "valu_busy": valu_busy(args, n, L),
            "method": "rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE "
                      "--kernel-trace, one pass, child run (profiled passes clock a few % lower)"}


def valu_busy(args, n, L):
    """SURVEY 8(d) 'VALU-busy', rocprofv3's derived VALUBusy = 100 * sum(SQ_ACTIVE_INST_VALU) / CU_NUM /
    max(GRBM_GUI_ACTIVE) (its gfx94x formula; ROCm 7.2 has no gfx950 derived-counter section, MI355X guide),
    plus VALUUtilization = 100 * SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU * 64) (active-lane share).
    One more PMC pass. GRBM_GUI_ACTIVE arrives summed over the 8 XCDs; its max is the per-XCD value."""
    r = _pmc_pass(args, n, L, ["SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU", "GRBM_GUI_ACTIVE"])
    if r is None:
        return None
    c, _ = r
    gui = c["GRBM_GUI_ACTIVE"] / 8
    act = c["SQ_ACTIVE_INST_VALU"]
    return {"valu_busy_pct": 100.0 * act / 256 / gui,
            "valu_utilization_pct": 100.0 * c["SQ_THREAD_CYCLES_VALU"] / (act * 64) if act else None,
            "sq_active_inst_valu": act, "sq_thread_cycles_valu": c["SQ_THREAD_CYCLES_VALU"],
            "grbm_gui_active_per_xcd": gui,
            "method": "rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE --kernel-trace, "
                      "one pass, child run; rocprofv3 VALUBusy/VALUUtilization formulas"}


def cpu_baseline(args, d_pk, d_sig, d_msg, n, L):
    """The oracle (C restatement of the dalek-1.x verify, `port`), one pthread per usable host core, on a bounded
    sample of the same records (~3 s of wall time). Stand-in for the reference's rayon ed25519-dalek path, which
    is not buildable here (no cargo/rustc, unvendored git dependencies)."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py

    cores, detail = usable_cores()
    threads = args.cpu_threads or cores
    o = oracle_py.Oracle()
    m0 = min(n, 64 * threads)
    pk = d_pk[: m0 * 32].cpu().numpy().reshape(m0, 32)
    sig = d_sig[: m0 * 64].cpu().numpy().reshape(m0, 64)
    msg = d_msg[: m0 * L].cpu().numpy()
    off = (np.arange(m0 + 1) * L).astype(np.uint32)
    t0 = time.perf_counter()
    o.verify_batch(pk, sig, msg, off, 0, threads)  # warm, and a rate estimate for sizing the sample
    rate0 = m0 / max(time.perf_counter() - t0, 1e-6)
    m = int(min(args.cpu_sample, n, max(m0, 3.0 * rate0)))
    pk = d_pk[: m * 32].cpu().numpy().reshape(m, 32)
    sig = d_sig[: m * 64].cpu().numpy().reshape(m, 64)
    msg = d_msg[: m * L].cpu().numpy()
    off = (np.arange(m + 1) * L).astype(np.uint32)
    t0 = time.perf_counter()
    ok = o.verify_batch(pk, sig, msg, off, 0, threads)
    dt = time.perf_counter() - t0
    out = {"value": m / dt, "unit": "verifies/s", "cores": threads, "kind": "port", **detail,
           "sample": f"{m} records of the benchmark batch ({L}-byte M), oracle/ed25519_oracle.c, {threads} threads "
                     f"(all usable cores), {dt:.2f} s wall; all valid={bool(ok.all())}; stand-in for the reference's "
                     f"rayon ed25519-dalek path (not buildable offline)"}
    ossl = openssl_baseline(d_pk, d_sig, d_msg, n, L, threads, rate0)
    if ossl is not None:
        out["openssl"] = ossl
    out["product_cpu"] = product_cpu_baseline(d_pk, d_sig, d_msg, n, L, threads)
    return out


def product_cpu_baseline(d_pk, d_sig, d_msg, n, L, threads):
    """The product's own CPU batch backend (at2v_opts.num_gpus = 0: a thread pool over the kernels' verify routine
    compiled for the host, csrc/at2v_cpu.h), the path a node without a GPU, or with AT2V_CTX_CPU_FALLBACK after a device
    error, runs. Same records and threads as the oracle leg; bounded sample of ~3 s."""
    import numpy as np

    import at2v

    def run(m):
        pk = d_pk[: m * 32].cpu().numpy().reshape(m, 32)
        sig = d_sig[: m * 64].cpu().numpy().reshape(m, 64)
        msg = d_msg[: m * L].cpu().numpy()
        off = (np.arange(m + 1) * L).astype(np.uint32)
        t0 = time.perf_counter()
        ok = v.verify_batch(pk, sig, msg, off)
        return time.perf_counter() - t0, ok

    with at2v.BatchVerifier(num_gpus=0, cpu_threads=threads) as v:
        m0 = min(n, 64 * threads)
        dt0, _ = run(m0)
        m = int(min(n, max(m0, 3.0 * m0 / max(dt0, 1e-6))))
        dt, ok = run(m)
        th = v.info()["cpu_threads"]
    return {"value": m / dt, "unit": "verifies/s", "cores": th, "kind": "product-cpu",
            "sample": f"{m} records of the benchmark batch ({L}-byte M), libat2v CPU backend (num_gpus = 0: "
                      f"verify_half_fu on {th} host threads), {dt:.2f} s wall; all valid={bool(ok.all())}"}


def openssl_baseline(d_pk, d_sig, d_msg, n, L, threads, rate_hint):
    """SURVEY 8(d)'s preferred CPU baseline: OpenSSL 3 libcrypto Ed25519 verify (EVP_DigestVerify) over the same
    records, one pthread per usable core (oracle/openssl_verify.c, built by `make -C oracle openssl`); None when the
    library is not there. Bounded sample, ~3 s of wall time."""
    import ctypes

    import numpy as np

    path = os.path.join(ROOT, "oracle", "libossl_verify.so")
    try:
        lib = ctypes.CDLL(path)
    except OSError:
        return None
    P = ctypes.c_void_p
    lib.ossl_verify_batch.argtypes = [P, P, P, P, ctypes.c_size_t, ctypes.c_int, P]
    lib.ossl_verify_batch.restype = ctypes.c_int

    def run(m):
        pk = np.ascontiguousarray(d_pk[: m * 32].cpu().numpy())
        sig = np.ascontiguousarray(d_sig[: m * 64].cpu().numpy())
        msg = np.ascontiguousarray(d_msg[: m * L].cpu().numpy())
        off = (np.arange(m + 1) * L).astype(np.uint32)
        res = np.zeros(m, dtype=np.uint8)
        t0 = time.perf_counter()
        rc = lib.ossl_verify_batch(pk.ctypes.data, sig.ctypes.data, msg.ctypes.data, off.ctypes.data, m, threads,
                                   res.ctypes.data)
        return time.perf_counter() - t0, rc, res

    m0 = min(n, 64 * threads)
    dt0, rc, _ = run(m0)  # warm-up and rate estimate
    if rc != 0:
        return None
    m = int(min(n, max(m0, 3.0 * m0 / max(dt0, 1e-6))))
    dt, rc, res = run(m)
    if rc != 0:
        return None
    return {"value": m / dt, "unit": "verifies/s", "cores": threads, "kind": "third-party",
            "sample": f"{m} records of the benchmark batch ({L}-byte M), OpenSSL {ossl_version(lib)} EVP_DigestVerify "
                      f"(Ed25519), {threads} threads, {dt:.2f} s wall; all valid={bool(res.all())}; SURVEY 8(d)'s "
                      f"preferred stand-in for the reference's rayon ed25519-dalek path"}


def ossl_version(lib):
    import ctypes
    try:
        f = lib.OpenSSL_version
        f.restype = ctypes.c_char_p
        f.argtypes = [ctypes.c_int]
        return f(0).decode().split()[1]
    except (AttributeError, OSError, IndexError):
        return "3"


if __name__ == "__main__":
    main()
