#!/usr/bin/env python3
"""latency_probe.py — where a small batch's latency goes (BASELINE config 5).

For batches of B records (default 1, 20, 64, 1024), each measured `--reps` times on one MI355X:
  kernel   : HIP events around at2v_verify_batch_device on HBM-resident records (the low-latency kernel for
             B <= small_batch_max), i.e. device time of the launch;
  sync     : wall time of at2v_verify_batch (host arrays: H2D, kernel, D2H, synchronise);
  queue    : wall time from at2v_queue_submit of the B records to the last verdict polled (eager queue, idle,
             one batch in flight at a time);
  fresh    : (--comb 1) device time of launches whose B keys the context has never seen (steady state of a stream of
             first-seen senders: the in-kernel lookup, then the four-wave split half-size check);
  first    : (--comb 1) device time of a launch of B records whose keys a new context has not seen (after two such
             launches of 64 other keys): the in-kernel lookup claims them and their chunks run the four-wave split
             half-size check (the cost a first-seen sender pays once); the combs are built afterwards on the context's
             own stream: `first_combs_ready_us` is the wall time from the launch until at2v_get_info returns;
             `first_launch_shared_hw_queue_us` is a launch of 64 new keys on a stream that shares a hardware queue
             with the context's stream (its end waits for the builds);
reports p50/p90 per stage as JSON. Records come from the oracle generator (all valid), checked once per size."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "at2-node_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pct(xs, q):
    return float(np.percentile(np.asarray(xs), q))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,20,64,1024")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--msg-len", type=int, default=48)
    ap.add_argument("--comb", type=int, default=0, help="1 = per-sender combs (the keys are cached after the first rep)")
    ap.add_argument("--fresh-reps", type=int, default=20,
                    help="(--comb 1) launches of B records with keys the context has not seen (fresh_keys_launch)")
    a = ap.parse_args()
    import torch

    import at2v
    import oracle_py
    from at2v.node import IngestQueue

    torch.cuda.set_device(0)
    o = oracle_py.Oracle()
    sizes = [int(x) for x in a.sizes.split(",")]
    nmax = max(sizes)
    pk, sig, msg, off = o.gen_records(0x4154325F, 0, nmax, a.msg_len)
    out = {"msg_len": a.msg_len, "reps": a.reps, "comb": bool(a.comb), "sizes": {}}
    v = at2v.BatchVerifier(device=0, sender_cache=1024 if a.comb else 0, sender_comb=bool(a.comb))
    q = IngestQueue(device=0, max_batch=4096, max_delay_us=1000, eager=True, sender_comb=bool(a.comb))
    s = torch.cuda.current_stream()
    for B in sizes:
        p, g, m, f = pk[:B], sig[:B], msg[:f_end(off, B)], off[:B + 1]
        assert v.verify_batch(p, g, m, f).all()
        d_pk = torch.from_numpy(p.reshape(-1).copy()).cuda()
        d_sig = torch.from_numpy(g.reshape(-1).copy()).cuda()
        d_msg = torch.from_numpy(np.concatenate([m, np.zeros(16, np.uint8)])).cuda()
        d_off = torch.from_numpy(f.view(np.int32).copy()).cuda()
        d_ver = torch.zeros((B + 31) // 32, dtype=torch.int32, device="cuda")
        first_us = None
        if a.comb:
            vc = at2v.BatchVerifier(device=0, sender_cache=1024, sender_comb=True)
            # HIP maps a process's streams round robin onto GPU_MAX_HW_QUEUES (4) hardware queues. `ls`, created right
            # after the context's own stream (where the combs are built), gets the next queue; `sh`, the fourth stream
            # after it, wraps round to the context's queue: anything enqueued on sh after a launch waits for the comb
            # build.
            ls, _, _, sh = at2v.launch_streams(4)
            # a running node's context: two earlier launches (other keys) before the measured one
            wp, wg, wm, wf = o.gen_records(0x4154325F, 1 << 30, 3 * 64 + B, a.msg_len)
            wd = [torch.from_numpy(x.reshape(-1).copy()).cuda() for x in (wp, wg)]
            wdm = torch.from_numpy(np.concatenate([wm, np.zeros(16, np.uint8)])).cuda()
            wv = torch.zeros((B + 31) // 32 + 2, dtype=torch.int32, device="cuda")

            def launch_new(lo, cnt, strm):
                wo = torch.from_numpy((wf[lo:lo + cnt + 1] - wf[lo]).view(np.int32).copy()).cuda()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t = time.perf_counter()
                e0.record(strm)
                vc.verify_batch_device(wd[0].data_ptr() + lo * 32, wd[1].data_ptr() + lo * 64,
                                       wdm.data_ptr() + int(wf[lo]), int(wf[lo + cnt] - wf[lo]), wo.data_ptr(), cnt,
                                       wv.data_ptr(), strm.cuda_stream)
                e1.record(strm)
                e1.synchronize()
                dev_us = e0.elapsed_time(e1) * 1e3
                vc.info()  # waits for the context's stream (the combs of the new keys)
                ready_us = (time.perf_counter() - t) * 1e6
                ok = (wv.cpu().numpy().view(np.uint32)[: cnt // 32] == 0xFFFFFFFF).all()
                assert ok
                return dev_us, ready_us

            warm = [launch_new(0, 64, ls)[0], launch_new(64, 64, ls)[0]]
            first_us, combs_ready_us = launch_new(128, B, ls)
            shared_us, _ = launch_new(128 + B, 64, sh)
            vc.close()
        fresh = []
        if a.comb and a.fresh_reps:
            # steady state of first-seen senders: every rep launches B records whose keys the context has not seen
            fp, fg, fm, ff = o.gen_records(0x4154325F, 1 << 24, B * a.fresh_reps, a.msg_len)
            dd = [torch.from_numpy(x.reshape(-1).copy()).cuda() for x in (fp, fg)]
            dm = torch.from_numpy(np.concatenate([fm, np.zeros(16, np.uint8)])).cuda()
            for r in range(a.fresh_reps):
                lo = r * B
                d_off2 = torch.from_numpy((ff[lo:lo + B + 1] - ff[lo]).view(np.int32).copy()).cuda()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                v.verify_batch_device(dd[0].data_ptr() + lo * 32, dd[1].data_ptr() + lo * 64, dm.data_ptr() + int(ff[lo]),
                                      int(ff[lo + B] - ff[lo]), d_off2.data_ptr(), B, d_ver.data_ptr(), s.cuda_stream)
                e1.record(s)
                torch.cuda.synchronize()
                assert (d_ver.cpu().numpy().view(np.uint32)[: B // 32] == 0xFFFFFFFF).all()
                if r >= 2:
                    fresh.append(e0.elapsed_time(e1) * 1e3)
        kern, sync, queue = [], [], []
        for r in range(a.reps + 5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            v.verify_batch_device(d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), int(f[-1]), d_off.data_ptr(), B,
                                  d_ver.data_ptr(), s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            v.verify_batch(p, g, m, f)
            t1 = time.perf_counter()
            first = q.submit(p, g, m, f)
            got = 0
            while got < B:
                t, vv = q.poll(4096, 2000)
                got += len(t)
            t2 = time.perf_counter()
            if r >= 5:
                kern.append(e0.elapsed_time(e1) * 1e3)
                sync.append((t1 - t0) * 1e6)
                queue.append((t2 - t1) * 1e6)
        assert (d_ver.cpu().numpy().view(np.uint32)[: B // 32] == 0xFFFFFFFF).all()
        out["sizes"][B] = {k: {"p50_us": pct(x, 50), "p90_us": pct(x, 90)} for k, x in
                           (("kernel", kern), ("sync", sync), ("queue", queue))}
        if fresh:
            out["sizes"][B]["fresh_keys_launch"] = {"p50_us": pct(fresh, 50), "p90_us": pct(fresh, 90)}
        if first_us is not None:
            out["sizes"][B]["first_launch_new_keys_us"] = first_us
            out["sizes"][B]["first_combs_ready_us"] = combs_ready_us
            out["sizes"][B]["warm_launches_new_keys_us"] = warm
            out["sizes"][B]["first_launch_shared_hw_queue_us"] = shared_us
        print(B, json.dumps(out["sizes"][B]), file=sys.stderr)
    q.close()
    v.close()
    print(json.dumps(out))


def f_end(off, B):
    return int(off[B])


if __name__ == "__main__":
    main()
