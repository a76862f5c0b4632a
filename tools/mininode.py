#!/usr/bin/env python3
"""mininode.py — BASELINE config 5: a local 4-node AT2 network whose servers batch gossiped payloads into
the GPU verify path; reports the ingest -> verdict latency (p50/p99) at small batches.

What each node process runs (the at2-node server's data path, /root/reference/src/bin/server/rpc.rs):
  * client RPC ingest (At2::send_asset, rpc.rs:258-287): decode the SendAssetRequest (at2v packer), put the
    transaction into the recent-transactions log as Pending, broadcast the payload to every other node;
  * payloads from clients and from peers go into the node's IngestQueue (GPU verify, flush at B records
    or Δ microseconds) — the per-payload verify sieve/murmur would do on CPU workers;
  * verified payloads are delivered to the node's Ledger (accounts + apply loop, rpc.rs:149-211).
The sieve/murmur/contagion protocol logic itself (echo thresholds, Byzantine sampling) is out of scope
(SURVEY §2): gossip here is a plain all-to-all forward over multiprocessing queues on one host.

A client process signs config-1-style traffic on the GPU (at2v_sign_batch; senders x sequences, random
recipients and amounts) plus a fraction of forged copies that do not verify, and offers it at a fixed rate, round-robin over
the nodes. At the end every node must hold the same ledger (same balances, same last sequences).

usage: python tools/mininode.py [--nodes 4] [--rate 20000] [--seconds 5] [--batch 1024] [--delay-us 1000]
prints one JSON line.
"""
import argparse
import hashlib
import json
import multiprocessing as mp
import os
import queue as queue_mod
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "at2-node_amd"))


def node_main(idx, inboxes, result_q, args, total, node_ready=None):
    import numpy as np

    from at2v.node import VERDICT_FAILED, IngestQueue, Ledger, SendAssetRequest, pack_send_asset, verdict_mask

    q = IngestQueue(device=0, max_batch=args.batch, max_delay_us=args.delay_us, max_msg_bytes=48, depth=3,
                    eager=args.eager, sender_comb=bool(args.comb), sender_cache=args.cache)
    if node_ready is not None:  # the context (and its tables) is built: traffic may start
        node_ready.put(idx)
    led = Ledger()
    lock = threading.Lock()
    chunks = []  # submitted runs, ticket order: [first, pk, seq, rcp, amt, t_arrival]
    lat = []
    stats = {"received": 0, "verified": 0, "rejected": 0, "applied": 0, "batches_delivered": 0, "failed": 0}
    done_ingest = threading.Event()
    t0 = time.perf_counter()

    def ingest():
        inbox = inboxes[idx]
        seen = 0
        while seen < total:  # every node receives every payload once: from its client or by gossip
            item = inbox.get()
            if item is None:
                continue
            kind, reqs = item
            seen += len(reqs)
            t_arr = time.perf_counter()
            rs = [SendAssetRequest(*r) for r in reqs]
            rec = pack_send_asset(rs)
            ok = rec["status"] == 0
            if kind == "client":
                with lock:
                    for i in np.nonzero(ok)[0]:
                        led.recent_put(rec["pk"][i].tobytes(), int(rec["sequence"][i]), rec["recipient"][i].tobytes(),
                                       int(rec["amount"][i]), int((t_arr - t0) * 1e6))
                for j, box in enumerate(inboxes):
                    if j != idx:
                        box.put(("gossip", reqs))
            if not ok.any():
                continue
            if not ok.all():
                keep = np.nonzero(ok)[0]
                lens = np.diff(rec["off"])[keep]
                msg = np.concatenate([rec["msg"][rec["off"][i]:rec["off"][i + 1]] for i in keep])
                off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint32)
                rec = {k: rec[k][keep] for k in ("pk", "sig", "recipient", "sequence", "amount")} | {"msg": msg, "off": off}
            with lock:
                first = q.submit(rec["pk"], rec["sig"], rec["msg"], rec["off"])
                chunks.append([first, rec["pk"], rec["sequence"], rec["recipient"], rec["amount"], t_arr, 0])
                stats["received"] += len(rec["sequence"])
        done_ingest.set()

    def apply_loop():
        ci = 0
        while True:
            t, v = q.poll(65536, 2000)
            now = time.perf_counter()
            if len(t) == 0:
                with lock:
                    idle = done_ingest.is_set() and stats["verified"] + stats["rejected"] == stats["received"]
                if idle:
                    break
                if done_ingest.is_set():
                    q.flush()
                continue
            k = 0
            sel = {"pk": [], "seq": [], "rcp": [], "amt": [], "ok": []}
            with lock:
                while k < len(t):
                    c = chunks[ci]
                    first, n_c, used = c[0], len(c[2]), c[6]
                    take = min(n_c - used, len(t) - k)
                    assert t[k] == first + used
                    sl = slice(used, used + take)
                    sel["pk"].append(c[1][sl]); sel["seq"].append(c[2][sl]); sel["rcp"].append(c[3][sl])
                    sel["amt"].append(c[4][sl]); sel["ok"].append(v[k:k + take])
                    lat.extend([now - c[5]] * take)
                    c[6] += take
                    k += take
                    if c[6] == n_c:
                        chunks[ci] = None
                        ci += 1
                raw = np.concatenate(sel["ok"])
                if (raw == VERDICT_FAILED).any():  # a device failure: nothing of it is delivered (fail closed)
                    stats["failed"] += int((raw == VERDICT_FAILED).sum())
                    raw = np.where(raw == VERDICT_FAILED, 0, raw).astype(np.uint8)
                okv = verdict_mask(raw, len(raw))
                st = led.deliver(np.concatenate(sel["pk"]), np.concatenate(sel["seq"]), np.concatenate(sel["rcp"]),
                                 np.concatenate(sel["amt"]), okv, int((now - t0) * 1e6))
                stats["verified"] += int(okv.sum())
                stats["rejected"] += int((~okv).sum())
                stats["applied"] += st["applied"]
                stats["batches_delivered"] += 1

    th = [threading.Thread(target=ingest), threading.Thread(target=apply_loop)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    qs = q.stats()
    q.close()
    lat_us = np.array(lat) * 1e6 if lat else np.zeros(1)
    h = hashlib.sha256()
    for k in sorted(result_keys(args)):
        h.update(k + led.balance(k).to_bytes(8, "little") + led.last_sequence(k).to_bytes(4, "little"))
    result_q.put({"node": idx, **stats, "pending": led.pending(), "ledger_sha256": h.hexdigest(),
                  "lat_p50_us": float(np.percentile(lat_us, 50)), "lat_p99_us": float(np.percentile(lat_us, 99)),
                  "queue_p50_us": qs["p50_us"], "queue_p99_us": qs["p99_us"], "queue_batches": qs["batches"],
                  "queue_mean_batch": qs["mean_batch"]})


def senders(args):
    import numpy as np
    rng = np.random.default_rng(args.seed)
    return rng.integers(0, 256, (args.senders, 32), dtype=np.uint8)


def result_keys(args):
    return [bytes(k) for k in KEYS]


KEYS = []


def client_main(inboxes, ready_q, args):
    """sign the whole run on the GPU, then offer it at `rate` tx/s round-robin over the nodes"""
    import numpy as np

    import at2v
    from at2v.node import thin_transaction, wire_key, wire_signature

    seeds = senders(args)
    v = at2v.BatchVerifier(device=0)
    # public keys: sign one empty message per sender (the signer returns A)
    pks, _ = v.sign_batch(seeds, np.zeros(1, np.uint8), np.zeros(args.senders + 1, np.uint32))
    total = int(args.rate * args.seconds)
    per = (total + args.senders - 1) // args.senders
    rng = np.random.default_rng(args.seed + 1)
    snd = np.tile(np.arange(args.senders), per)[:total]
    seq = np.repeat(np.arange(1, per + 1), args.senders)[:total]
    rcp = (snd + rng.integers(1, args.senders, total)) % args.senders
    amt = rng.integers(1, args.max_amount + 1, total)
    msgs = [thin_transaction(pks[rcp[i]].tobytes(), int(amt[i])) for i in range(total)]
    msg = np.frombuffer(b"".join(msgs), np.uint8)
    off = (np.arange(total + 1) * 48).astype(np.uint32)
    _, sig = v.sign_batch(seeds[snd], msg, off)
    v.close()
    reqs = [(wire_key(pks[snd[i]].tobytes()), int(seq[i]), wire_key(pks[rcp[i]].tobytes()), int(amt[i]),
             wire_signature(sig[i].tobytes())) for i in range(total)]
    # forgeries: copies of real (sender, sequence) pairs with another amount and a signature that does not
    # verify, interleaved with the real traffic; every node must reject them and still apply the real ones
    nbad = int(total * args.bad_frac)
    for j in sorted(rng.choice(total, nbad, replace=False), reverse=True):
        forged = bytearray(sig[j].tobytes())
        forged[50] ^= 0x08
        reqs.insert(int(j) + 1, (reqs[j][0], reqs[j][1], reqs[j][2], reqs[j][3] + 1, wire_signature(bytes(forged))))
    total = len(reqs)
    # a stream of first-seen senders (--fresh-frac): each fresh key sends one transfer (sequence 1) to a regular
    # sender, spread evenly through the run; on every node its first payload finds no cache entry
    fresh_keys = []
    nfresh = int(total * args.fresh_frac)  # (after the forgeries: they index the regular arrays)
    if nfresh:
        vf = at2v.BatchVerifier(device=0)
        fseeds = rng.integers(0, 256, (nfresh, 32), dtype=np.uint8)
        fpks, _ = vf.sign_batch(fseeds, np.zeros(1, np.uint8), np.zeros(nfresh + 1, np.uint32))
        frcp = rng.integers(0, args.senders, nfresh)
        famt = rng.integers(1, args.max_amount + 1, nfresh)
        fmsg = np.frombuffer(b"".join(thin_transaction(pks[frcp[i]].tobytes(), int(famt[i])) for i in range(nfresh)),
                             np.uint8)
        _, fsig = vf.sign_batch(fseeds, fmsg, (np.arange(nfresh + 1) * 48).astype(np.uint32))
        vf.close()
        at = np.linspace(0, total, nfresh, endpoint=False).astype(int)
        for i in range(nfresh - 1, -1, -1):
            reqs.insert(int(at[i]), (wire_key(fpks[i].tobytes()), 1, wire_key(pks[frcp[i]].tobytes()), int(famt[i]),
                                     wire_signature(fsig[i].tobytes())))
        fresh_keys = [fpks[i].tobytes() for i in range(nfresh)]
        total = len(reqs)
    ready_q.put({"keys": [pks[i].tobytes() for i in range(args.senders)] + fresh_keys, "total": total, "bad": nbad,
                 "fresh": nfresh})
    ready_q.get()  # go
    tick = 1e-3
    per_tick = max(1, int(args.rate * tick))
    t_start = time.perf_counter()
    i, node = 0, 0
    while i < total:
        target = t_start + (i / args.rate)
        d = target - time.perf_counter()
        if d > 0:
            time.sleep(d)
        j = min(total, i + per_tick)
        inboxes[node].put(("client", reqs[i:j]))
        node = (node + 1) % len(inboxes)
        i = j
    ready_q.put({"offered_s": time.perf_counter() - t_start})


def late_builder_main(args, go, built, stop):
    """--late-builder: a process that, once told, creates what a starting node creates on the GPU (an ingest queue with
    per-sender combs: its context, B tables, combs of B and cache) while the nodes serve, reports how long that took,
    then holds it until the end. Round 5's comb-of-B build launches of up to 68 ms stalled the serving nodes (VERDICT r5
    "Next" 3); since round 6 the combs of B are built by additions in short launches."""
    import torch  # noqa: F401  (the nodes' import order)

    from at2v.node import IngestQueue
    go.wait(600)
    t0 = time.perf_counter()
    q = IngestQueue(device=0, max_batch=args.batch, max_delay_us=args.delay_us, max_msg_bytes=48, depth=3,
                    eager=args.eager, sender_comb=bool(args.comb), sender_cache=args.cache)
    built.put(time.perf_counter() - t0)
    stop.wait(900)
    q.close()


def polluter_main(ready, stop):
    """--polluter: another process on the same GPU that holds what a test runner or a co-located job holds: an RCCL
    communicator (libat2v's, world 1), torch streams and two raw HIP streams, each used once, idle afterwards. Its
    hardware queues stay mapped for the whole run (DESIGN.md §10e "Hardware queues")."""
    import torch

    import at2v
    v = at2v.BatchVerifier(device=0)
    v.comm_init_rank(at2v.comm_unique_id(), 0, 1)
    streams = [torch.cuda.Stream() for _ in range(4)] + at2v.launch_streams(2)
    for st in streams:
        with torch.cuda.stream(st):
            torch.ones(1024, device="cuda").sum().item()
    torch.cuda.synchronize()
    ready.set()
    stop.wait(900)
    v.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=4)
    ap.add_argument("--rate", type=float, default=20000.0, help="offered client transactions per second (total)")
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--batch", type=int, default=1024, help="queue flush size B")
    ap.add_argument("--delay-us", type=int, default=1000, help="queue flush deadline Δ")
    ap.add_argument("--eager", type=int, default=0, help="1 = queue latency mode: also seal whenever no batch is in flight")
    ap.add_argument("--comb", type=int, default=0, help="1 = per-sender combs in each node's queue context (at2v_comb.h)")
    ap.add_argument("--senders", type=int, default=64)
    ap.add_argument("--fresh-frac", type=float, default=0.0,
                    help="extra transfers from first-seen senders, as a fraction of the regular traffic (one each)")
    ap.add_argument("--cache", type=int, default=0, help="keys per node queue context with --comb (0 = 1024)")
    ap.add_argument("--bad-frac", type=float, default=0.02)
    ap.add_argument("--max-amount", type=int, default=10,
                    help="amounts in [1, max]; small enough that no sender can underflow, so the final ledger does "
                         "not depend on each node's delivery order (the reference bumps the sequence on Underflow)")
    ap.add_argument("--seed", type=int, default=0x4154325F)
    ap.add_argument("--polluter", type=int, default=0,
                    help="N > 0 = N separate processes each hold an RCCL communicator and 6 streams on the GPU for the "
                         "whole run")
    ap.add_argument("--late-builder", type=int, default=0,
                    help="1 = another process creates a node's queue (context, tables, combs of B) 0.3 s into the traffic")
    ap.add_argument("--late-node", type=int, default=0,
                    help="1 = the last node process starts 0.3 s after the traffic (the others serve while it builds)")
    ap.add_argument("--start", choices=["spawn", "ready"], default="ready",
                    help="spawn: the client sends once the node processes are started; ready: once every node's queue "
                         "is built")
    ap.add_argument("--node-hw-queues", type=int, default=0,
                    help="K > 0 = the node processes run with GPU_MAX_HW_QUEUES=K (HIP's hardware queues per process)")
    args = ap.parse_args()
    ctx = mp.get_context("spawn")
    pols = []
    pol_stop = ctx.Event()
    for _ in range(args.polluter):
        pol_ready = ctx.Event()
        pol = ctx.Process(target=polluter_main, args=(pol_ready, pol_stop))
        pol.start()
        pols.append(pol)
        if not pol_ready.wait(300):
            raise SystemExit("mininode: a polluter process did not come up")
    inboxes = [ctx.Queue() for _ in range(args.nodes)]
    ready_q, result_q = ctx.Queue(), ctx.Queue()
    # (daemonic: if this process fails, its client and nodes end with it instead of waiting for a "go")
    cl = ctx.Process(target=client_main, args=(inboxes, ready_q, args), daemon=True)
    cl.start()
    info, deadline = None, time.time() + 600
    while info is None:  # a client that dies (e.g. an exception while signing) must end the run, not stall it
        try:
            info = ready_q.get(timeout=5)
        except queue_mod.Empty:
            if not cl.is_alive():
                raise SystemExit(f"mininode: client process exited with {cl.exitcode} before the run started")
            if time.time() > deadline:
                raise SystemExit("mininode: client did not get ready in 600 s")
    KEYS[:] = info["keys"]
    node_ready = ctx.Queue()
    nodes = [ctx.Process(target=node_main_with_keys,
                         args=(i, inboxes, result_q, args, info["keys"], info["total"], node_ready), daemon=True)
             for i in range(args.nodes)]
    late = nodes[-1] if args.late_node else None  # (--late-node, below)
    builder, builder_go, builder_built = None, ctx.Event(), ctx.Queue()
    if args.late_builder:  # started now (imports take a while), builds 0.3 s into the traffic
        builder = ctx.Process(target=late_builder_main, args=(args, builder_go, builder_built, pol_stop), daemon=True)
        builder.start()
    saved = os.environ.get("GPU_MAX_HW_QUEUES")
    if args.node_hw_queues > 0:  # (spawned children take the parent's environment at start)
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.node_hw_queues)
    for p in nodes:
        if p is not late:
            p.start()
    if args.node_hw_queues > 0:
        if saved is None:
            del os.environ["GPU_MAX_HW_QUEUES"]
        else:
            os.environ["GPU_MAX_HW_QUEUES"] = saved
    # --start ready (default): every node's queue is built before the client sends. --start spawn: the client sends as
    # soon as the node processes exist (their inboxes fill while they import and create their queues, so their latency
    # counts that backlog). --late-node: the last node process starts 0.3 s into the traffic, so the other nodes serve
    # while it creates its context and builds its B tables and combs of B beside them (VERDICT r5 "Next" 3: round 5's
    # comb-of-B launches of up to 68 ms stalled serving nodes; they are built by additions in short launches since round
    # 6); its own backlog latency is reported apart and left out of p50_us / p99_us.
    up, deadline = 0, time.time() + 600
    while args.start == "ready" and up < args.nodes - (1 if late else 0):
        try:
            node_ready.get(timeout=5)
            up += 1
        except queue_mod.Empty:
            dead = [p.exitcode for p in nodes if p is not late and not p.is_alive()]
            if dead:
                raise SystemExit(f"mininode: a node process exited with {dead[0]} before the run started")
            if time.time() > deadline:
                raise SystemExit("mininode: nodes did not get ready in 600 s")
    if args.start == "ready":
        time.sleep(0.5)
    t0 = time.perf_counter()
    ready_q.put("go")
    if builder is not None:
        time.sleep(0.3)
        builder_go.set()
    if late is not None:
        time.sleep(0.3)
        saved_q = os.environ.get("GPU_MAX_HW_QUEUES")
        if args.node_hw_queues > 0:
            os.environ["GPU_MAX_HW_QUEUES"] = str(args.node_hw_queues)
        late.start()
        if args.node_hw_queues > 0:
            if saved_q is None:
                del os.environ["GPU_MAX_HW_QUEUES"]
            else:
                os.environ["GPU_MAX_HW_QUEUES"] = saved_q
    offered = ready_q.get(timeout=600)
    cl.join(timeout=60)
    res = [result_q.get(timeout=600) for _ in nodes]
    wall = time.perf_counter() - t0
    for p in nodes:
        p.join(timeout=60)
    res.sort(key=lambda r: r["node"])
    same = len({r["ledger_sha256"] for r in res}) == 1
    serving = [r for r in res if not (args.late_node and r["node"] == args.nodes - 1)]
    out = {"metric": "AT2 mini-network ingest->verdict latency (BASELINE config 5)", "nodes": args.nodes,
           "offered_tx_per_s": args.rate, "seconds": args.seconds, "total_tx": info["total"],
           "bad_signatures": info["bad"], "fresh_senders": info["fresh"], "batch_B": args.batch, "delay_us": args.delay_us,
           "p50_us": max(r["lat_p50_us"] for r in serving), "p99_us": max(r["lat_p99_us"] for r in serving),
           "ledgers_identical": same, "all_real_applied": all(r["applied"] == info["total"] - info["bad"] for r in res), "wall_s": wall, "offered_s": offered["offered_s"], "per_node": res}
    out["polluters"] = args.polluter
    if builder is not None:
        out["late_builder_create_s"] = builder_built.get(timeout=60)
    out["start"] = args.start
    out["late_node"] = args.nodes - 1 if args.late_node else None
    out["node_hw_queues"] = args.node_hw_queues or None
    out["queue_env"] = {k: v for k, v in os.environ.items() if k.startswith("AT2V_QUEUE")}
    pol_stop.set()
    for pol in pols:
        pol.join(timeout=60)
    print(json.dumps(out), flush=True)
    ok = same and all(r["verified"] + r["rejected"] == info["total"] and r["rejected"] == info["bad"] and
                      r["applied"] == info["total"] - info["bad"] and r["pending"] == 0 and r["failed"] == 0 for r in res)
    return 0 if ok else 1


def node_main_with_keys(idx, inboxes, result_q, args, keys, total, node_ready=None):
    KEYS[:] = keys
    node_main(idx, inboxes, result_q, args, total, node_ready)


if __name__ == "__main__":
    sys.exit(main())
