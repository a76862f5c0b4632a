#!/usr/bin/env python3
"""bench.py — Ed25519 verifies/s of the at2v hot path on 1..8 MI355X (BASELINE.json metric).

Workload (BASELINE config 2, weak-scaled): every rank verifies its own batch of `--records-per-gpu`
(default 1,048,576) signed transfers with 100-byte messages, generated on the GPU by the deterministic
RFC 8032 generator and resident in HBM before timing starts. One step = one verify
launch over the rank's batch + (N > 1) one RCCL all-gather of the verdict bitmap words over xGMI.
Config 3 (16M over 8 GPUs) = `--records-per-gpu 2097152` at N = 8.

Output: one JSON line on rank 0 with the contract fields plus `roofline` (VALU-bound) and
`cpu_baseline` (the oracle, multi-threaded on host cores, bounded sample).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "at2-node_amd"))

CFG_SEED = 0x4154325F
# Algorithmic work per verify (half-size equation, 33-window chain): decode A and R
# 510 S + 44 M, tables [j]A and [j](+-R) 128 M, ladder 32 x (16 S + 28 M) + top window 15 M + 8 fixed-base
# windows x 14 M = 512 S + 1023 M; 1195 M + 1022 S in all. A 10-limb radix-2^25.5 multiplication is 100 and a
# squaring 55 32x32->64 multiply-accumulates. (About 17% of waves need a 34th window, +2.1% work: the figure
# below is the lower bound, so the reported fraction is conservative.)
FIELD_MUL_PER_VERIFY = 1195
FIELD_SQ_PER_VERIFY = 1022
MAC_PER_VERIFY = 100 * FIELD_MUL_PER_VERIFY + 55 * FIELD_SQ_PER_VERIFY  # 175,710
# Peak: v_mad_i64_i32 issues at half the VALU rate on gfx950 (profiles/r01_ubench_valu.txt): one wave64
# instruction per 4 cycles per SIMD = 16 lane-MACs/clk/SIMD x 4 SIMD x 256 CU x 2.4 GHz.
MAC_PEAK = 256 * 4 * 16 * 2.4e9  # 3.93e13 MAC/s
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--records-per-gpu", type=int, default=1 << 20)
    ap.add_argument("--msg-len", type=int, default=100)
    ap.add_argument("--policy", default="dalek")
    ap.add_argument("--cpu-sample", type=int, default=262144, help="records for the CPU baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cpu_count)")
    ap.add_argument("--pmc-traffic", type=int, default=1,
                    help="1 = at N=1, measure HBM-side bytes per verify launch with two rocprofv3 PMC passes "
                         "(FETCH_SIZE, WRITE_SIZE) of a 2-step child run; 0 = skip (roofline.traffic null)")
    return ap.parse_args()


def main():
    args = parse()
    # stdout carries exactly one line, the JSON result: everything else that writes to fd 1 (RCCL's version
    # banner at communicator init, library chatter) is sent to stderr.
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    import numpy as np
    import torch
    import torch.distributed as dist

    import at2v
    from at2v import dist as at2dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("run N>1 under torch.distributed.run (one process per GPU)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # N > 1: one process per GPU, RCCL over xGMI. Under torch.distributed.run at N = 1 the same
    # process-group path runs too (nccl init, all-gather of the verdict words, barriers, MAX reduce), so a
    # one-GPU box rehearses the multi-rank code exactly; plain `python bench.py` stays collective-free.
    use_dist = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    if use_dist:
        dist.init_process_group("nccl", device_id=dev)

    n, L = args.records_per_gpu, args.msg_len
    n = (n + 63) // 64 * 64
    v = at2v.BatchVerifier(device=local, policy=args.policy)
    stream = torch.cuda.current_stream(dev)
    s = stream.cuda_stream
    d_pk = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_sig = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    d_msg = torch.empty(n * L, dtype=torch.uint8, device=dev)
    d_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    words = n // 32
    d_ver = torch.zeros(words, dtype=torch.int32, device=dev)
    d_all = torch.zeros(words * world, dtype=torch.int32, device=dev) if use_dist else None
    # distinct records per rank (indices rank*n .. rank*n+n-1)
    v.gen_records_device(CFG_SEED, rank * n, n, L, d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                         d_off.data_ptr(), s)
    torch.cuda.synchronize(dev)

    def step():
        v.verify_batch_device(d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), n * L, d_off.data_ptr(), n,
                              d_ver.data_ptr(), s)
        if use_dist:
            at2dist.gather_verdicts(d_ver, world)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    kev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(args.steps):
        kev[k][0].record(stream)
        v.verify_batch_device(d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), n * L, d_off.data_ptr(), n,
                              d_ver.data_ptr(), s)
        kev[k][1].record(stream)
        if use_dist:
            d_all = at2dist.gather_verdicts(d_ver, world)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kernel_ms = sum(a.elapsed_time(b) for a, b in kev) / args.steps
    t_dev = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=dev)
    if use_dist:
        dist.all_reduce(t_dev, op=dist.ReduceOp.MAX)
    elapsed, kernel_ms = t_dev.tolist()

    # verdict check after the timed region: every generated record must be valid, on every rank
    full = d_all if use_dist else d_ver
    match = float((full == -1).float().mean().item())
    if use_dist:
        mt = torch.tensor([match], dtype=torch.float64, device=dev)
        dist.all_reduce(mt, op=dist.ReduceOp.MIN)
        match = mt.item()

    total = n * world * args.steps
    value = total / elapsed
    per_gpu_kernel_rate = n / (kernel_ms * 1e-3)
    achieved = per_gpu_kernel_rate * MAC_PER_VERIFY / 1e12
    info = v.info()

    out = None
    if rank == 0:
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
                "workload": "BASELINE config 2: 1M signed transfers per GPU (100-byte M), dalek-1.x verify"
                if n == 1 << 20 else f"{n} signed transfers per GPU ({L}-byte M)",
                "records_per_gpu": n,
                "msg_len": L,
                "policy": args.policy,
                "parallelism": f"index-shard x{world}" + (" + RCCL all-gather of verdict words" if use_dist else ""),
            },
            "verdict_match": match,
            "kernel_ms": kernel_ms,
            "kernel": {"grid_blocks": info["grid_blocks"], "block": info["block_threads"],
                       "waves_per_cu": info["waves_per_cu"], "vgprs": info["vgprs"]},
            "roofline": {
                "bound": "valu",
                "achieved": achieved,
                "peak": MAC_PEAK / 1e12,
                "unit": "Tops/s (32x32->64 integer MAC, v_mad_i64_i32)",
                "frac": achieved * 1e12 / MAC_PEAK,
                "traffic": None,
                "alg_macs_per_verify": MAC_PER_VERIFY,
                "alg_bytes_per_verify": 32 + 64 + L + 4,
                "hbm_gbs": per_gpu_kernel_rate * (32 + 64 + L + 4) / 1e9,
                "hbm_frac": per_gpu_kernel_rate * (32 + 64 + L + 4) / 1e9 / HBM_PEAK_GBS,
            },
        }
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        out["cpu_baseline"] = cpu_baseline(args, d_pk, d_sig, d_msg, n, L)
    if rank == 0 and world == 1 and args.pmc_traffic and not use_dist:
        tr = pmc_traffic(args, n, L)
        if tr is not None:
            out["roofline"]["traffic"] = tr["bytes_per_launch"]
            out["roofline"]["traffic_detail"] = tr
        vl = pmc_valu(args, n, L)
        if vl is not None:
            out["roofline"]["valu_measured"] = vl
    if rank == 0:
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    v.close()
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


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
           "-d", d, "-o", "run", "--", sys.executable, os.path.abspath(__file__), "--steps", "2", "--warmup", "0",
           "--cpu-sample", "0", "--pmc-traffic", "0", "--records-per-gpu", str(n), "--msg-len", str(L),
           "--policy", args.policy]
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
                    k = r.get("Dispatch_Id", "0")
                    per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
            if not per:
                return None
            out[ctr] = sum(per.values()) / len(per)
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
    SQ_INSTS_VALU (wave instructions), its INT64 part (v_mad_i64_i32, 64-bit shifts/adds: half rate on
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
    """The oracle (C restatement of the dalek-1.x verify, `port`), pthreads over host cores, on a bounded
    sample of the same records. Stand-in for the reference's rayon ed25519-dalek path (not buildable)."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py

    m = min(args.cpu_sample, n)
    pk = d_pk[: m * 32].cpu().numpy().reshape(m, 32)
    sig = d_sig[: m * 64].cpu().numpy().reshape(m, 64)
    msg = d_msg[: m * L].cpu().numpy()
    off = (np.arange(m + 1) * L).astype(np.uint32)
    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    o = oracle_py.Oracle()
    o.verify_batch(pk[:64], sig[:64], msg[: 64 * L], off[:65], 0, threads)  # warm
    t0 = time.perf_counter()
    ok = o.verify_batch(pk, sig, msg, off, 0, threads)
    dt = time.perf_counter() - t0
    return {"value": m / dt, "unit": "verifies/s", "cores": threads, "kind": "port",
            "sample": f"{m} records of the benchmark batch (100-byte M), oracle/ed25519_oracle.c, {threads} threads, "
                      f"{dt:.2f} s wall; all valid={bool(ok.all())}"}


if __name__ == "__main__":
    main()
