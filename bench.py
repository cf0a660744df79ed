"""Benchmark: MsgAppResp applied/s (+ commits advanced/s) on the cfg2 workload.

BASELINE.json metric "MsgAppResp applied/sec + commits advanced/sec, 1M raft
groups x3, 1-8 GPUs", quoted on configs[1]: 1M groups x 3 replicas steady-state
replication on one MI355X.  One step = one batch through the hot path: every
group takes one proposal (dense props) and both followers' MsgAppResp for it
arrive in a random permutation (2M MsgAppResp per GPU), i.e. the engine runs
partition + apply (+ finish) over HBM-resident inputs and writes the sparse
event stream to HBM.  Weak scaling: each GPU owns ~1M groups (sharded by
splitmix64(group id) % N) and the only collective is one RCCL all-reduce of the
step statistics.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU)

--workload cfg3 / cfg4 runs the other SURVEY.md 8(d) streams (auxiliary lines,
not the headline metric): cfg3 = 1M x 5 lagging followers (open-loop stream
generated from the engine's state between steps, each step timed by HIP
events), cfg4 = 4M x 7 election storm (MsgVoteResp tallied/s).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MsgAppResp applied/sec + commits advanced/sec, 1M raft groups×3, 1-8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def alg_bytes_per_group(n):
    """SURVEY.md §8(d) algorithmic bytes per group per cfg2 step: each follower's
    MsgAppResp 66 B + per-group commit/append state 80 B + per-follower
    bcastAppend on the proposal 21 B  (= 254 B = 2 x 127 B at n = 3)."""
    return (n - 1) * (66 + 21) + 80


def cpu_baseline(n, groups=200_000, budget_s=10.0, max_steps=40):
    """The C oracle (a sequential restatement of the reference loop) on a bounded
    sample of the same workload, one host core: the reference MultiNode steps
    every group on its single `run` goroutine (raft/multinode.go:166).  Test
    infrastructure only."""
    from etcd_amd import abi, synth
    from oracle.pyoracle import OracleGroups
    g, runs = synth.steady_groups(groups, n, seed=0x5EED0002, with_runs="flat")
    og = OracleGroups(g, runs, 256)
    acks = commits = 0
    spent = 0.0
    steps = 0
    while spent < budget_s and steps < max_steps:
        b = synth.cfg2_batch(g, steps)
        t0 = time.perf_counter()
        _, st = og.step(b)
        spent += time.perf_counter() - t0
        acks += int(st[abi.HB_STAT_APPRESP])
        commits += int(st[abi.HB_STAT_COMMITS])
        steps += 1
    return {"value": acks / spent, "unit": "MsgAppResp/s", "cores": 1, "kind": "port",
            "commits_per_s": commits / spent,
            "sample": f"oracle/raft_oracle.c (C restatement of the reference loop, not the Go reference), "
                      f"{groups} groups x {n}, {steps} cfg2 steps, {acks} MsgAppResp in {spent:.2f} s, one core"}


def cpu_baseline_parallel(n, threads, groups_per_thread=65_536, budget_s=8.0, max_steps=20):
    """Best case for the CPU: `threads` independent oracle shards (as many
    MultiNodes as cores, groups partitioned), stepped concurrently from Python
    threads (each orc_step_batch call releases the GIL).  Test infrastructure only."""
    import threading
    from etcd_amd import abi, synth
    from oracle.pyoracle import OracleGroups, flat_runs
    G = threads * groups_per_thread
    g, runs = synth.steady_groups(G, n, seed=0x5EED0002, with_runs="flat")
    flat, off = flat_runs(runs)
    shards = []
    for t in range(threads):
        a, b = t * groups_per_thread, (t + 1) * groups_per_thread
        shards.append(OracleGroups(g[a:b], (flat[int(off[a]):int(off[b])], off[a:b + 1] - off[a]), 256))
    acks = 0
    spent = 0.0
    steps = 0
    while spent < budget_s and steps < max_steps:
        bt = synth.cfg2_batch(g, steps)
        sh = bt["group"] // groups_per_thread
        local = []
        for t in range(threads):
            m = sh == t
            local.append(dict(group=(bt["group"][m] - t * groups_per_thread).astype(np.uint32), info=bt["info"][m],
                              term=bt["term"][m], index=bt["index"][m], hint=None,
                              props=bt["props"][t * groups_per_thread:(t + 1) * groups_per_thread]))
        out = [None] * threads

        def run(t):
            out[t] = shards[t].step(local[t])[1]
        th = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        spent += time.perf_counter() - t0
        acks += sum(int(o[abi.HB_STAT_APPRESP]) for o in out)
        steps += 1
    return {"value": acks / spent, "unit": "MsgAppResp/s", "cores": threads, "kind": "port",
            "sample": f"{threads} oracle shards x {groups_per_thread} groups x {n} stepped concurrently, "
                      f"{steps} cfg2 steps, {acks} MsgAppResp in {spent:.2f} s"}


def cpu_baseline_cfg4(n, groups=40_000, W=256, budget_s=10.0, max_steps=20):
    """The C oracle on a bounded sample of the repeatable cfg4 storm, one core."""
    from etcd_amd import abi, synth
    from oracle.pyoracle import OracleGroups
    g, runs = synth.election_groups(groups, n, seed=0x5EED0004)
    og = OracleGroups(g, runs, W)
    b = synth.cfg4_storm_batch(g, seed=0x5EED0004)
    votes = decided = 0
    spent = 0.0
    steps = 0
    while spent < budget_s and steps < max_steps:
        bk = dict(b, term=synth.storm_terms(b["term"], steps))
        t0 = time.perf_counter()
        _, st = og.step(bk)
        spent += time.perf_counter() - t0
        votes += int(st[abi.HB_STAT_VOTERESP])
        decided += int(st[abi.HB_STAT_WON]) + int(st[abi.HB_STAT_LOST])
        steps += 1
    return {"value": votes / spent, "unit": "MsgVoteResp/s", "cores": 1, "kind": "port",
            "elections_decided_per_s": decided / spent,
            "sample": f"oracle/raft_oracle.c (C restatement, not the Go reference), {groups} groups x {n}, "
                      f"{steps} storm steps, {votes} MsgVoteResp in {spent:.2f} s, one core"}


def cpu_baseline_cfg3(n, groups=60_000, W=256, budget_s=10.0, max_steps=20):
    """The C oracle on a bounded sample of the open-loop cfg3 stream, one core
    (stream generation from the oracle's state between steps is not timed)."""
    from etcd_amd import abi, synth
    from oracle.pyoracle import OracleGroups
    g, runs = synth.lagging_groups(groups, n, seed=0x5EED0003, W=W)
    og = OracleGroups(g, runs, W)
    rng = np.random.default_rng(0x5EED0003)
    acks = msgs = 0
    spent = 0.0
    steps = 0
    while spent < budget_s and steps < max_steps:
        b = synth.cfg3_open_batch(og.groups(), rng)
        t0 = time.perf_counter()
        _, st = og.step(b)
        spent += time.perf_counter() - t0
        acks += int(st[abi.HB_STAT_APPRESP])
        msgs += int(st[abi.HB_STAT_MSGS])
        steps += 1
    return {"value": acks / spent, "unit": "MsgAppResp/s", "cores": 1, "kind": "port",
            "msgs_per_s": msgs / spent,
            "sample": f"oracle/raft_oracle.c (C restatement, not the Go reference), {groups} groups x {n} (W={W}), "
                      f"{steps} cfg3 steps, {acks} MsgAppResp in {spent:.2f} s, one core"}


def cpu_baseline_tick(n, groups=200_000, W=256, budget_s=10.0, max_steps=50):
    """The C oracle's MultiNode.Tick (orc_tick_batch) on a bounded sample of the
    tick workload, one core -- the reference ticks every group on its one run
    goroutine (raft/multinode.go:268-274)."""
    from etcd_amd import abi, synth
    from oracle.pyoracle import OracleGroups
    g, runs = synth.steady_groups(groups, n, seed=0x5EED0002, with_runs="flat")
    g["state"][1::2] = abi.HB_STATE_FOLLOWER
    g["lead"][1::2] = 1
    og = OracleGroups(g, runs, W)
    t = synth.random_timers(groups, seed=0x5EED0002, et_hi=10, ht_hi=1, pos_hi=0)
    t["election_tick"] = 10
    og.load_timers(t)
    draws = np.random.default_rng(1).integers(0, 1 << 63, 4 * max_steps + 64, dtype=np.uint64)
    spent = 0.0
    steps = 0
    while spent < budget_s and steps < max_steps:
        t0 = time.perf_counter()
        og.tick(draws)
        spent += time.perf_counter() - t0
        steps += 1
    return {"value": groups * steps / spent, "unit": "group-ticks/s", "cores": 1, "kind": "port",
            "sample": f"oracle/raft_oracle.c orc_tick_batch (C restatement, not the Go reference), {groups} groups x {n}, "
                      f"{steps} ticks in {spent:.2f} s, one core"}


FOLLOW_GROUP_BYTES = 196  # SURVEY.md 8(d) rule applied to the follow step (follow_alg_note)


def follow_alg_note():
    return ("per group per follow step (SURVEY.md 8(d) rule: each field read once R / written once W): "
            "MsgApp 48 B (message 24, m.LogTerm 8, m.Commit 8, entry term 8), MsgHeartbeat 32 B (message 24, "
            "m.Commit 8), group 116 B (Term 8R, meta 8R, committed 8R+8W, lastIndex 8R+8W, firstIndex 8R, "
            "termFirst 8R, elapsed 4W, 6 event words 48W: two step markers, two responses, append, commit) "
            "= 196 B = 98 B per message")


def cpu_baseline_follow(n, groups=200_000, W=256, budget_s=10.0, max_steps=40):
    """The C oracle on a bounded sample of the follow workload (stepFollower ->
    handleAppendEntries / handleHeartbeat, raft/raft.go:616-669), one core."""
    from etcd_amd import abi, synth
    from oracle.pyoracle import OracleGroups
    g, runs = synth.follow_groups(groups, n, seed=0x5EED0006, with_runs="flat")
    og = OracleGroups(g, runs, W)
    msgs = commits = 0
    spent = 0.0
    steps = 0
    while spent < budget_s and steps < max_steps:
        b = synth.follow_batch(g, steps)
        t0 = time.perf_counter()
        _, st = og.step(b)
        spent += time.perf_counter() - t0
        msgs += int(st[abi.HB_STAT_MSGS])
        commits += int(st[abi.HB_STAT_COMMITS])
        steps += 1
    return {"value": msgs / spent, "unit": "msgs/s", "cores": 1, "kind": "port", "commits_per_s": commits / spent,
            "sample": f"oracle/raft_oracle.c (C restatement, not the Go reference), {groups} groups x {n}, "
                      f"{steps} follow steps (MsgApp + MsgHeartbeat per group), {msgs} messages in {spent:.2f} s, "
                      f"one core"}


def cpu_baseline_mixed(n, groups=200_000, W=256, budget_s=10.0, max_steps=40):
    """The C oracle on a bounded sample of the mixed workload (a node leading
    1/3 of its groups, following 2/3: stepLeader + stepFollower), one core."""
    from etcd_amd import abi, synth
    from oracle.pyoracle import OracleGroups
    g, runs = synth.mixed_groups(groups, n, seed=0x5EED0007, with_runs="flat")
    og = OracleGroups(g, runs, W)
    msgs = commits = 0
    spent = 0.0
    steps = 0
    while spent < budget_s and steps < max_steps:
        b, _ = synth.mixed_batch(g, steps)
        t0 = time.perf_counter()
        _, st = og.step(b)
        spent += time.perf_counter() - t0
        msgs += int(st[abi.HB_STAT_MSGS])
        commits += int(st[abi.HB_STAT_COMMITS])
        steps += 1
    return {"value": msgs / spent, "unit": "msgs/s", "cores": 1, "kind": "port", "commits_per_s": commits / spent,
            "sample": f"oracle/raft_oracle.c (C restatement, not the Go reference), {groups} groups x {n} (1/3 led, "
                      f"2/3 followed), {steps} mixed steps, {msgs} messages in {spent:.2f} s, one core"}


def cpu_baseline_wire(n, groups=100_000, W=256, budget_s=10.0, max_steps=20):
    """The C oracle decoding the cfg2 wire records (orc_decode_batch, the
    reference's Unmarshal restated) and stepping them, one core."""
    from etcd_amd import abi, synth
    from oracle.pyoracle import OracleGroups, decode_batch
    g, runs = synth.steady_groups(groups, n, seed=0x5EED0002, with_runs="flat")
    og = OracleGroups(g, runs, W)
    peers = np.zeros((groups, abi.HB_MAX_REPLICAS), np.uint64)
    peers[:, :n] = np.arange(1, n + 1, dtype=np.uint64)
    gn = np.full(groups, n, np.uint32)
    acks, spent, dec, steps = 0, 0.0, 0.0, 0
    while spent < budget_s and steps < max_steps:
        b = synth.cfg2_batch(g, steps)
        frm = ((b["info"] >> 4) & 0xF).astype(np.uint64) + np.uint64(1)
        data, off, ln = synth.encode_responses(abi.HB_MSG_APP_RESP, np.ones(len(frm), np.uint64), frm, b["term"],
                                               b["index"])
        t0 = time.perf_counter()
        o = decode_batch(data, off, ln, b["group"], groups, gn, peers)
        t1 = time.perf_counter()
        _, st = og.step(dict(group=o["group"], info=o["info"], term=o["term"], index=o["index"], hint=o["hint"],
                             props=b["props"]))
        t2 = time.perf_counter()
        spent += t2 - t0
        dec += t1 - t0
        acks += int(st[abi.HB_STAT_APPRESP])
        steps += 1
    return {"value": acks / spent, "unit": "MsgAppResp/s", "cores": 1, "kind": "port",
            "decode_records_per_s": acks / dec,
            "sample": f"oracle/wire_oracle.c + raft_oracle.c (C restatements, not the Go reference), {groups} groups "
                      f"x {n}, {steps} cfg2 steps from wire records, {acks} MsgAppResp in {spent:.2f} s, one core"}


LAYOUT_RO = "role-ordered (led groups in their own partitions; --role-order)"


def pmc_traffic(path, kernel, G, n, apply_us, workload=None, layout=None):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (FETCH_SIZE x 2 + WRITE_SIZE, tools/prof_summary.py).  Used only when the
    profile was taken on the same workload and its average duration agrees with
    the live measurement within 15 % (same build); otherwise None."""
    import glob
    cands = [path] if path else sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json")), reverse=True)
    names = [kernel] if isinstance(kernel, str) else list(kernel)
    for path in cands:  # the newest profile of this configuration
        try:
            d = json.load(open(path))
            k = next(d["kernels"][x] for x in names if x in d["kernels"])
            cfg = d["bench"]["config"]
        except (OSError, KeyError, ValueError, StopIteration):
            continue
        if cfg.get("groups_per_gpu") == G and cfg.get("replicas") == n and "traffic_bytes" in k and \
                (workload is None or cfg.get("workload", "").startswith(workload + ":")) and \
                cfg.get("layout") == layout:
            break
    else:
        return None, None
    src = os.path.relpath(path, ROOT)
    if abs(k["avg_us"] - apply_us) > 0.15 * apply_us:
        return None, f"{src}: profiled avg {k['avg_us']:.1f} us vs live {apply_us:.1f} us (stale, not used)"
    return float(k["traffic_bytes"]), f"{src}: rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, avg {k['avg_us']:.1f} us"


def step_traffic(path, workload, G, n, ms_per_step, layout=None):
    """Whole-step HBM bytes of an auxiliary line (cfg3 / cfg4 / tick) from the
    newest committed profile of the same workload and configuration
    (tools/profile_round.sh with WL=<workload>: FETCH_SIZE x 2 + WRITE_SIZE
    summed over the step's kernels).  Used only when the traced run's step time
    agrees with the live one within 15 %; otherwise None."""
    import glob
    cands = [path] if path else sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json")), reverse=True)
    for p in cands:
        try:
            d = json.load(open(p))
            st, cfg, bms = d["step"], d["bench"]["config"], d["bench"]["ms_per_step"]
        except (OSError, KeyError, ValueError, TypeError):
            continue
        if cfg.get("workload", "").startswith(workload + ":") and cfg.get("groups_per_gpu") == G and \
                cfg.get("replicas") == n and cfg.get("layout") == layout:
            src = os.path.relpath(p, ROOT)
            if abs(bms - ms_per_step) > 0.15 * ms_per_step:
                return None, f"{src}: profiled step {bms:.3f} ms vs live {ms_per_step:.3f} ms (stale, not used)"
            return float(st["traffic_bytes"]), (f"{src}: rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE summed over the "
                                                f"step's kernels, traced step {bms:.3f} ms")
    return None, None


def run_multinode(args):
    """The MultiNode API end to end: a C++ application
    (etcd_amd/csrc/hbnode_bench.cpp, the reference's node_bench_test loop over
    many groups) steps every follower's MsgAppResp, proposes one entry per
    group, takes the Ready (host assembly over the device step), appends it to
    MemoryStorage and advances.  Host-inclusive: value = MsgAppResp/s through
    the whole API, not the kernel rate."""
    import ctypes as C
    G = args.groups or 1000
    n = args.replicas or 3
    # (HBNB_DIR: a variant build's directory, for same-box A/Bs of the host library)
    L = C.CDLL(os.path.join(os.environ.get("HBNB_DIR", os.path.join(ROOT, "etcd_amd")), "libhbnode_bench.so"))
    L.hbnb_run2.restype = C.c_int
    L.hbnb_run2.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                            C.POINTER(C.c_double)]
    out = (C.c_double * 32)()
    bulk = args.mn_mode == "bulk"
    # the application pins its Ready-loop thread when that thread does all of its own work
    # (persisting below 4,096 groups per Ready); at 1M groups pinning it measured 1.54e7 -> 1.08e7
    pin = not args.mn_no_pin and G < 4096
    flags = (3 if bulk else 0) | (4 if pin else 0)  # HBNB_BULK | HBNB_PAR_APP, HBNB_PIN
    threads = args.mn_threads if bulk else 1
    t0 = time.perf_counter()
    rc = L.hbnb_run2(int(os.environ.get("LOCAL_RANK", "0")), G, n, args.warmup, args.steps, flags, threads, out)
    wall = time.perf_counter() - t0
    if rc != 0:
        raise SystemExit(f"hbnb_run failed: {rc}")
    secs, acks, adv = out[0], out[1], out[2]
    rec = {"metric": "MsgAppResp applied/sec through the MultiNode API (Step + Propose + Ready + Advance)",
           "value": acks / secs, "unit": "MsgAppResp/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": 1e3 * secs / args.steps, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u64",
           "data": "synthetic (node_bench_test-style loop: every group proposes 'foo', followers ack last index)",
           "config": {"workload": f"multinode: {G} groups x {n} through include/hbnode.h (SURVEY.md 8(d) cfg1 "
                                  f"shape{' = BASELINE.json configs[0]' if G == 1000 and n == 3 else ''})",
                      "groups": G, "replicas": n, "max_inflight": 256},
           "commits_per_s": adv / secs,
           "api": ("hbn_step_many + hbn_propose_many, host threads "
                   f"{threads or 'default (min(16, cores))'}, application persists from the same number of threads"
                   if bulk else "one hbn_step / hbn_propose call per message, one host thread") +
                  ("; the application's Ready-loop thread pinned to its CPU" if pin else ""),
           "split_s_per_step": {"ready": out[3] / args.steps, "step_and_propose": out[4] / args.steps,
                                "append_and_advance": out[5] / args.steps,
                                "of_which_app_persist": out[24] / args.steps},
           "parity_sanity": bool(adv == G * args.steps and out[7] == 0),
           "host_phases_s_per_step": {k: round(out[8 + i] / args.steps, 6) for i, k in enumerate(
               ["load_sync", "log_reserve", "hb_step_call", "event_fetch", "event_replay", "stepped_marks",
                "ready_build", "ready_merge", "advance", "bulk_lookup", "bulk_responses", "bulk_proposals",
                "batch_reset"])},
           "wall_s": wall}
    if not args.no_cpu_baseline:
        cb = cpu_baseline(n, groups=min(G, args.cpu_groups), budget_s=min(args.cpu_seconds, 5.0))
        cb["sample"] += " (raft steps only: no Ready assembly, no storage)"
        rec["cpu_baseline"] = cb
    print(json.dumps(rec), flush=True)


def spawn_ranks(args):
    """`python bench.py --gpus N` (N > 1) without a launcher: start one child
    rank per GPU with the variables torchrun sets (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR / MASTER_PORT on 127.0.0.1), before this process
    touches the GPU; wait for all of them and return the worst exit status
    (the others are stopped as soon as one fails).  Rank 0 prints the line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            c = p.poll()
            if c is None:
                continue
            alive.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                for q in alive:
                    q.terminate()
        time.sleep(0.1)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["cfg2", "cfg5", "e2e", "cfg3", "cfg4", "tick", "wire", "multinode", "follow",
                                           "mixed"],
                    default="cfg2",
                    help="cfg2 (headline: 1M groups x 3 per GPU), cfg5 (8M groups x 3 per GPU = BASELINE.json "
                         "configs[4] at 8 GPUs), e2e = cfg2 with the batch in host memory and the events copied "
                         "back every step, cfg3 lagging followers, cfg4 election storm, "
                         "tick = MultiNode.Tick over the cfg2 groups (SURVEY.md 8(f) rank 1), "
                         "wire = cfg2 from raftpb wire records: hb_decode + hb_step (8(f) rank 3), "
                         "multinode = the MultiNode API end to end (Step/Propose/Ready/Advance, 8(f) rank 2), "
                         "follow = the follower side of cfg2: 1M followed groups x 3 (--replicas 5: x 5), each "
                         "receiving its leader's MsgApp (1 entry) and MsgHeartbeat per step (8(f) rank 4), "
                         "mixed = a node's Ready cycle: 1M groups x 3, 1/3 led (the cfg2 step) and 2/3 followed "
                         "(the follow step) in one batch")
    ap.add_argument("--groups", type=int, default=None,
                    help="groups per GPU (cfg2/cfg3/e2e: 1M, cfg5: 8M, cfg4: 4M)")
    ap.add_argument("--replicas", type=int, default=None, help="cfg2/cfg5: 3, cfg3: 5, cfg4: 7")
    ap.add_argument("--inflight", type=int, default=256, help="MaxInflightMsgs W (cfg3/cfg4)")
    ap.add_argument("--role-order", action="store_true",
                    help="mixed / tick: the groups laid out by role (led groups in partitions of their own), the "
                         "layout a role-ordered slot map in the node would give; a measurement of that map, "
                         "which libhbnode does not build (default: roles interleaved, as a node's ids fall)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-groups", type=int, default=200_000)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=min(16, os.cpu_count() or 1),
                    help="shards of the parallel best-case CPU baseline (the GPU box's share is 16 cores)")
    ap.add_argument("--no-profile", action="store_true", help="skip per-phase HIP events")
    ap.add_argument("--e2e-events", choices=["words", "records"], default="words",
                    help="e2e: delta list D2H as compact event words (default) or 16-byte hb_event records")
    ap.add_argument("--overlap", action="store_true",
                    help="batch inputs on their own stream: the prep stage of step k+1 (bucket sort + routing) "
                         "overlaps the apply stage of step k (hb_set_input_stream); default: stages serialized")
    ap.add_argument("--mn-mode", choices=["bulk", "percall"], default="bulk",
                    help="multinode: bulk = hbn_step_many / hbn_propose_many + host threads (default), "
                         "percall = one API call per message on one thread (the r01/r02 path, for A/B)")
    ap.add_argument("--mn-no-pin", action="store_true",
                    help="multinode: leave the application's Ready-loop thread unpinned (pinned below 4,096 groups by default)")
    ap.add_argument("--mn-threads", type=int, default=0, help="multinode bulk: host threads (0 = library default)")
    ap.add_argument("--traffic-json", default=None,
                    help="profiles/<tag>_traffic.json from tools/profile_round.sh (default: newest in profiles/)")
    args = ap.parse_args()
    if args.workload == "multinode":
        return run_multinode(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch one rank per GPU)")
    if args.groups is None:
        args.groups = {"cfg4": 1 << 22, "cfg5": 1 << 23}.get(args.workload, 1 << 20)
    if args.replicas is None:
        args.replicas = {"cfg3": 5, "cfg4": 7}.get(args.workload, 3)

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.workload in ("cfg2", "cfg5"):
        return run_replication(args, world, rank, local)

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    if args.workload == "e2e":
        return run_e2e(args, world, rank, local, dev, torch, dist)
    return run_aux(args, world, rank, local, dev, torch, dist)


def routed_batch(G_per_gpu, world, rank, n):
    """Host side of a cfg2 / cfg5 step on this rank: the shard
    map of the global group-id space [0, world x G_per_gpu) (splitmix64(id) %
    world), this rank's groups (steady state, seeded per rank), and ONE global
    arrival stream (every follower of every group acks, same order on every
    rank) routed by the host router of libhbnode (include/hbroute.h: one pass,
    16 host threads, every rank's stream positions and local slots in arrival
    order), timed on its own.  Term / Index come from the local group state."""
    from etcd_amd import synth
    from etcd_amd.shard import NativeRouter
    G_total = G_per_gpu * world
    t0 = time.perf_counter()
    router = NativeRouter(np.arange(G_total, dtype=np.uint64), world)
    build_s = time.perf_counter() - t0
    G = len(router.local_ids(rank))
    groups, _ = synth.steady_groups(G, n, seed=0x5EED0002 + rank, with_runs=False)
    gid, frm = synth.global_ack_stream(G_total, n)
    t0 = time.perf_counter()
    out, unknown = router.route(gid)  # every rank's share in one pass (what a node's router does once)
    route_s = time.perf_counter() - t0
    pos, slots = out[rank]
    frm_l = frm[pos]
    n_global = len(gid)
    del gid, frm, out
    batch = synth.cfg2_local_batch(groups, slots, frm_l, 0)
    route = {"global_msgs_routed": n_global, "ranks_served": world, "local_msgs": int(len(slots)),
             "seconds": round(route_s, 4), "msgs_routed_per_s": n_global / route_s if route_s > 0 else None,
             "threads": router.threads, "unknown_groups": unknown, "router_build_s": round(build_s, 3),
             "note": "host owner routing of the node's whole arrival stream to every rank in one pass "
                     "(libhbnode hbn_route: splitmix64 owner + id -> local slot, arrival order kept), outside the "
                     "timed region; a node runs it once for all its GPUs"}
    return groups, batch, G_total, route


def run_replication(args, world, rank, local):
    """cfg2 (headline) / cfg5: steady-state replication, weak scaling over
    `world` ranks, one GPU each."""
    n = args.replicas
    # (the engine library under the router's libhbnode binds to torch's HIP
    # runtime in either import order: etcd_amd/hipbatch.py _bind_one_hip_runtime)
    import torch  # noqa: F401
    t_setup = time.perf_counter()
    groups, batch, G_total, route = routed_batch(args.groups, world, rank, n)
    G = len(groups)
    nmsg = len(batch["group"])
    host_setup_s = time.perf_counter() - t_setup

    import torch
    import torch.distributed as dist
    from etcd_amd import abi
    from etcd_amd.hipbatch import Engine

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    # the apply stage runs on a high-priority stream; the engine's prep stream is
    # its lowest-priority one (they overlap only with --overlap)
    lo_prio, hi_prio = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    stream = torch.cuda.Stream(device=dev, priority=hi_prio)
    torch.cuda.set_stream(stream)
    eng = Engine(G, max_replicas=n, max_inflight=256, max_batch=max(nmsg, 1), device=local, stream=stream)
    # --overlap: the batches are resident before the timed region, produced on
    # their own (idle) stream, so the engine's prep stage of step k+1 (bucket
    # sort + routing) may overlap the apply stage of step k (hb_set_input_stream).
    if args.overlap:
        in_stream = torch.cuda.Stream(device=dev)
        eng.set_input_stream(in_stream)
    eng.load_groups(groups)
    d_group = torch.from_numpy(batch["group"].view(np.int32)).to(dev)
    d_info = torch.from_numpy(batch["info"].view(np.int32)).to(dev)
    d_term = torch.from_numpy(batch["term"].view(np.int64)).to(dev)
    d_props = torch.from_numpy(batch["props"].view(np.int32)).to(dev)
    base_index = torch.from_numpy(batch["index"].view(np.int64)).to(dev)  # last + 1
    del groups, batch
    total = args.warmup + args.steps
    n_iso = 0 if args.no_profile else 10  # steps of the separate per-phase pass after the timed region
    # step k acks index last + k + 1 (prepared before timing: inputs resident in HBM)
    d_index = [base_index + k for k in range(total + n_iso)]
    stats_step = torch.zeros(abi.HB_STAT_COUNT, dtype=torch.int64, device=dev)
    stats_acc = torch.zeros(abi.HB_STAT_COUNT, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    if world == 1:
        eng.set_stats_accum(stats_acc)  # summed in the engine's finish phase, no extra launch

    def one_step(k, profile):
        eng.step(d_group, d_info, d_term, d_index[k], None, d_props, host=False, profile=profile)
        if world > 1:
            eng.stats_to(stats_step)
            dist.all_reduce(stats_step)  # RCCL over xGMI: the only collective
            stats_acc.add_(stats_step)

    for k in range(args.warmup):
        one_step(k, False)
    torch.cuda.synchronize()
    stats_acc.zero_()
    eng.phase_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = torch.cuda.Event(enable_timing=True)
    t_end = torch.cuda.Event(enable_timing=True)
    wall0 = time.perf_counter()
    t_start.record(stream)
    for k in range(args.warmup, total):
        # HIP events bracket the dominant kernel (k_apply_fast) on its launch
        # stream, on every 4th step of the timed region (each pair costs ~1 us)
        one_step(k, "apply" if (not args.no_profile and (k - args.warmup) % 4 == 0) else False)
    t_end.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - wall0
    ms_local = t_start.elapsed_time(t_end)
    ms_t = torch.tensor([ms_local], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(ms_t, op=dist.ReduceOp.MAX)
    ms = float(ms_t.item())
    st = stats_acc.cpu().numpy().astype(np.uint64)  # summed over ranks and steps
    appresp = int(st[abi.HB_STAT_APPRESP])
    commits = int(st[abi.HB_STAT_COMMITS])
    # sanity: every group of every rank commits once per step, nothing faults
    ok = commits == G_total * args.steps and int(st[abi.HB_STAT_FAULTS]) == 0 and \
        appresp == G_total * (n - 1) * args.steps
    route_t = torch.tensor([route["seconds"]], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(route_t, op=dist.ReduceOp.MAX)
    route["seconds_max_over_ranks"] = float(route_t.item())
    step_s = ms / args.steps / 1e3
    if step_s > 0 and route["seconds"] > 0:
        # the bound a deployment meets: one host router feeds every GPU of the node
        route["route_s_over_device_step"] = round(route["seconds_max_over_ranks"] / step_s, 2)
        route["bound"] = (f"the router moves {route['global_msgs_routed'] / route['seconds']:.3g} msgs/s on "
                          f"{route['threads']} host threads; the node's {world} GPU(s) step "
                          f"{route['global_msgs_routed'] / step_s:.3g} msgs/s")

    phase = {}
    roof = None
    alg = alg_bytes_per_group(n) * G  # per k_apply_fast launch on this GPU
    if not args.no_profile:
        ph, nph = eng.phase_ms()  # timed region: HB_PHASE_APPLY only
        apply_ms = float(ph[abi.HB_PHASE_APPLY])
        # per-phase breakdown: a separate, untimed pass with every phase event and
        # the stages serialized on one stream
        eng.set_stats_accum(None)
        eng.set_input_stream(stream)
        eng.phase_reset()
        for k in range(total, total + n_iso):  # the stream continues (fresh indices)
            eng.step(d_group, d_info, d_term, d_index[k], None, d_props, host=False, profile=True)
        torch.cuda.synchronize()
        ph2, nph2 = eng.phase_ms()
        phase = {"apply_ms": apply_ms, "apply_steps": nph,
                 "isolated": {"partition_ms": float(ph2[abi.HB_PHASE_PARTITION]),
                              "apply_ms": float(ph2[abi.HB_PHASE_APPLY]),
                              "general_ms": float(ph2[abi.HB_PHASE_GENERAL]),
                              "finish_ms": float(ph2[abi.HB_PHASE_FINISH]), "steps": nph2}}
        # HB_PHASE_APPLY brackets exactly the dominant kernel's launch (HIP events on
        # its launch stream): k_route_fast where the route runs inside the fast
        # lane's workgroups (hb_step_kernels), else k_apply_fast
        achieved = float(alg / (apply_ms * 1e-3) / 1e9)
        fused = bool(eng.step_kernels() & abi.HB_KERN_ROUTE_FAST)
        if fused:
            kname = "k_route_fast<2>"
            knames = ["k_route_fast<2u, false>", "k_route_fast"]
        else:
            kname = f"k_apply_fast<{3 if n <= 3 else (5 if n <= 5 else 7)}>"
            # (rocprofv3 names the template with its X-mode flag since r04)
            knames = [kname[:-1] + ", false, 2u>", kname[:-1] + ", false>", kname]
        traffic, tsrc = pmc_traffic(args.traffic_json, knames, G, n, apply_ms * 1e3)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": tsrc,
                "kernel": kname,
                "launch_us_timed": round(apply_ms * 1e3, 2),
                "launch_us_isolated": round(float(ph2[abi.HB_PHASE_APPLY]) * 1e3, 2),
                "frac_isolated": round(alg / (float(ph2[abi.HB_PHASE_APPLY]) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "alg_bytes_per_launch": alg,
                "alg_bytes_note": f"SURVEY.md 8(d): {alg_bytes_per_group(n)} B/group = "
                                  f"{alg_bytes_per_group(n) / (n - 1):.0f} B/MsgAppResp x {G * (n - 1)} MsgAppResp"
                                  + (" (the message's 24 B are read by this kernel as its 16-byte partitioned "
                                     "record: the route runs inside it)" if fused else ""),
                # the whole step (partition + route + apply + finish) against the same bytes
                "step_frac": round(alg / (ms / args.steps * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}

    out = None
    if rank == 0:
        sec = ms / 1e3
        cfg5 = args.workload == "cfg5"
        wl = (f"cfg5: {G_total} raft groups x {n} sharded by splitmix64(group id) % {world} "
              f"({args.groups} per GPU; BASELINE.json configs[4] is 64M x 3 on 8 GPUs)") if cfg5 else \
            (f"cfg2: {args.groups} raft groups x {n} per GPU steady-state replication (BASELINE.json configs[1])"
             + (f", {world} GPUs, sharded by splitmix64(group id) % {world}" if world > 1 else ""))
        out = {
            "metric": METRIC,
            "value": appresp / sec,
            "unit": "MsgAppResp/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (seeded global ack stream routed to each rank: steady-state leaders, "
                    "1 proposal + all follower acks per group per step)",
            "config": {"workload": wl,
                       "groups_per_gpu": args.groups, "groups_rank0": G, "groups_total": G_total, "replicas": n,
                       "msgappresp_per_step": G_total * (n - 1), "max_inflight": 256,
                       "max_msg_size": "noLimit", "sharding": f"splitmix64(group id) % {world}" if world > 1 else "none",
                       "parallelism": f"groups sharded over {world} GPU(s), one rank per GPU"},
            "commits_per_s": commits / sec,
            "parity_sanity": bool(ok),
            "wall_s": wall,
            "host_setup_s": round(host_setup_s, 2),
            "host_route": route,
            "collective": "one RCCL all-reduce (sum) of the 10 step statistics per step" if world > 1 else "none",
            "phases": phase,
            "pipeline": "prep(k+1) || apply(k): batch inputs on their own stream" if args.overlap else "stages serialized",
            "roofline": roof,
            "cpu_baseline": None,
        }
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(n, args.cpu_groups, args.cpu_seconds)
            except Exception as e:  # report, never fake
                out["cpu_baseline"] = {"error": repr(e)}
            if args.cpu_threads > 1:
                try:
                    out["cpu_baseline"]["best_case_parallel"] = cpu_baseline_parallel(n, args.cpu_threads)
                except Exception as e:
                    out["cpu_baseline"]["best_case_parallel"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)


def run_e2e(args, world, rank, local, dev, torch, dist):
    """cfg2 end to end (SURVEY.md 7 "End-to-end vs kernel"; reported apart from
    the HBM-resident headline): every step's batch starts in pinned host memory
    (hb_step with HB_STEP_HOST_PTRS copies group / info / term / index and the
    dense props to the device) and the step's delta list comes back to pinned
    host memory, i.e. what a host MultiNode hands over and gets back per Ready
    cycle.  The delta list is the device's compact event words
    (hb_events_to_host: 8 B per word, one word per bcastAppend, SURVEY.md 8(a)
    a12), which libhbnode replays directly; `--e2e-events records` ships the
    expanded 16-byte hb_event records instead (hb_copy_events), and the words'
    host expansion (hb_expand_event_words) is timed apart as
    `host_expand_ms_per_step` for a consumer that wants records.  Wall clock
    per step, synchronised."""
    from etcd_amd import abi
    from etcd_amd.hipbatch import Engine
    n = args.replicas
    groups, batch, G_total, route = routed_batch(args.groups, world, rank, n)
    G = len(groups)
    nmsg = len(batch["group"])
    stream = torch.cuda.current_stream(dev)
    eng = Engine(G, max_replicas=n, max_inflight=256, max_batch=nmsg, device=local, stream=stream)
    eng.load_groups(groups)
    words_mode = args.e2e_events == "words"

    def pinned(a):
        t = torch.from_numpy(np.ascontiguousarray(a).view({4: np.int32, 8: np.int64}[a.dtype.itemsize]))
        return t.pin_memory()
    h_group, h_info, h_term, h_props = (pinned(batch[k]) for k in ("group", "info", "term", "props"))
    total = args.warmup + args.steps
    h_index = [pinned(batch["index"] + np.uint64(k)) for k in range(total)]
    ev_cap = G * (2 * n + 4)
    nchunks, _ = eng.n_chunks()
    st_acc = np.zeros(abi.HB_STAT_COUNT, np.uint64)
    nev_total = nword_total = 0
    t_step = t_ev = 0.0
    if words_mode:
        # Pipelined: the batch arrays come from their own stream (hb_set_input_stream), so the
        # H2D copy + partition of step k+1 (prep stream) overlap step k's apply and its delta
        # words written to pinned host memory (apply stream); PCIe carries both directions at
        # once.  Delta buffers are double-buffered; step k-2's are read before reuse.
        in_stream = torch.cuda.Stream(dev)
        eng.set_input_stream(in_stream)
        acc = torch.zeros(abi.HB_STAT_COUNT, dtype=torch.int64, device=dev)
        h_w = [torch.empty(ev_cap, dtype=torch.int64).pin_memory() for _ in range(2)]
        h_cnt = [torch.empty(nchunks, dtype=torch.int32).pin_memory() for _ in range(2)]
        h_tot = [torch.zeros(1, dtype=torch.int64).pin_memory() for _ in range(2)]
        done = [torch.cuda.Event() for _ in range(2)]
        live = [False, False]
        torch.cuda.synchronize()

        def drain(b):
            nonlocal nword_total
            done[b].synchronize()
            nw = int(h_tot[b][0])
            assert nw <= ev_cap
            if live[b]:
                nword_total += nw
            live[b] = False
        t0 = None
        for k in range(total):
            if k == args.warmup:
                for b in range(2):
                    drain(b)
                torch.cuda.synchronize()
                if world > 1:
                    dist.barrier()
                eng.set_stats_accum(acc)
                t0 = time.perf_counter()
            b = k % 2
            if k >= 2:
                drain(b)
            eng.step(h_group, h_info, h_term, h_index[k], None, h_props, host=True)
            eng.events_to_host(h_w[b].data_ptr(), ev_cap, h_cnt[b].data_ptr(), h_tot[b].data_ptr())
            done[b].record(stream)
            live[b] = k >= args.warmup
        for b in range(2):
            drain(b)
        eng.sync()
        t_step = time.perf_counter() - t0
        eng.set_stats_accum(None)
        st_acc = acc.cpu().numpy().view(np.uint64).copy()
    else:
        h_ev = torch.empty(ev_cap * abi.EVENT_DTYPE.itemsize, dtype=torch.uint8).pin_memory()
        torch.cuda.synchronize()
        for k in range(total):
            if k == args.warmup:
                if world > 1:
                    dist.barrier()
                st_acc[:] = 0
                nev_total = 0
                t_step = t_ev = 0.0
            t0 = time.perf_counter()
            eng.step(h_group, h_info, h_term, h_index[k], None, h_props, host=True)
            eng.sync()
            t1 = time.perf_counter()
            nev_total += eng.events_into(h_ev.data_ptr(), ev_cap)
            t2 = time.perf_counter()
            t_step += t1 - t0
            t_ev += t2 - t1
            st_acc += eng.stats()
    sec_t = torch.tensor([t_step + t_ev], dtype=torch.float64)
    if world > 1:
        sec_t = sec_t.to(dev)
        dist.all_reduce(sec_t, op=dist.ReduceOp.MAX)
    sec = float(sec_t.item())
    expand = {}
    if words_mode:  # the last step's words expanded on the host, untimed above
        lb = (total - 1) % 2
        w = h_w[lb].numpy()[: int(h_tot[lb][0])].view(np.uint64)
        c = h_cnt[lb].numpy().view(np.uint32)
        te = time.perf_counter()
        recs = Engine.expand_words(w, c)
        expand = {"host_expand_ms_per_step": round(1e3 * (time.perf_counter() - te), 3),
                  "records_per_step": len(recs)}
        nev_total = len(recs) * args.steps
    st_t = torch.from_numpy(st_acc.view(np.int64).copy()).to(dev)
    if world > 1:
        dist.all_reduce(st_t)
    st = st_t.cpu().numpy().view(np.uint64)
    ok = int(st[abi.HB_STAT_COMMITS]) == G_total * args.steps and int(st[abi.HB_STAT_FAULTS]) == 0
    h2d = nmsg * 24 + G * 4
    steps = max(args.steps, 1)
    d2h = (nword_total // steps * 8 + nchunks * 4 + 8) if words_mode else nev_total // steps * 16
    how = ("hb_events_to_host (compact 8-byte words) into pinned memory; steps pipelined (the batch's H2D "
           "and partition of step k+1 overlap step k's apply and delta D2H; hb_set_input_stream), wall clock "
           "over all timed steps" if words_mode
           else "hb_sync, then hb_copy_events (16-byte hb_event records) into pinned memory")
    out = {"metric": "MsgAppResp applied/sec end to end (cfg2 batch from host memory + delta list back to host)",
           "value": int(st[abi.HB_STAT_APPRESP]) / sec, "unit": "MsgAppResp/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * sec / args.steps,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
           "data": "synthetic (cfg2 stream in pinned host memory)",
           "config": {"workload": f"e2e: cfg2 {args.groups} raft groups x {n} per GPU, batch H2D + delta D2H "
                                  f"every step ({args.e2e_events})", "groups_per_gpu": args.groups, "replicas": n},
           "split_ms_per_step": {"pipelined_step" if words_mode else "h2d_and_step": 1e3 * t_step / steps,
                                 "events_d2h": 1e3 * t_ev / steps},
           "bytes_per_step": {"h2d_batch": h2d, "d2h_delta": d2h},
           "pcie_gbs": round((h2d + d2h) / (sec / steps) / 1e9, 2),
           "events_per_step": nev_total // steps, "words_per_step": nword_total // steps if words_mode else None,
           **expand, "parity_sanity": bool(ok),
           "timing": "wall clock: hb_step (H2D inside) + " + how,
           "cpu_baseline": None}
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:  # the same cfg2 steps on the host's C oracle
            try:
                out["cpu_baseline"] = cpu_baseline(n, args.cpu_groups, args.cpu_seconds)
            except Exception as e:  # report, never fake
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)


def run_aux(args, world, rank, local, dev, torch, dist):
    """cfg3 / cfg4 lines; same JSON shape as the cfg2 line."""
    from etcd_amd import abi, synth
    from etcd_amd.hipbatch import Engine
    n, W, G = args.replicas, args.inflight, args.groups
    seed = {"cfg3": 0x5EED0003, "cfg4": 0x5EED0004, "tick": 0x5EED0002, "wire": 0x5EED0002,
            "follow": 0x5EED0006, "mixed": 0x5EED0007}[args.workload] + rank
    stream = torch.cuda.current_stream(dev)
    total = args.warmup + args.steps
    st_acc = np.zeros(abi.HB_STAT_COUNT, np.uint64)
    ms_local = 0.0
    t_wall = time.perf_counter()
    if args.workload == "cfg4":
        g, _ = synth.election_groups(G, n, seed=seed, with_runs=False)
        b = synth.cfg4_storm_batch(g, seed=seed)
        nmsg = len(b["group"])
        eng = Engine(G, max_replicas=n, max_inflight=W, max_batch=nmsg, device=local, stream=stream)
        eng.load_groups(g)
        del g
        d_group = torch.from_numpy(b["group"].view(np.int32)).to(dev)
        d_info = torch.from_numpy(b["info"].view(np.int32)).to(dev)
        d_index = torch.from_numpy(b["index"].view(np.int64)).to(dev)
        t0 = torch.from_numpy(b["term"].view(np.int64)).to(dev)
        nz = (t0 != 0).to(torch.int64)
        d_terms = [t0 + nz * (4 * k) for k in range(total)]  # storm_terms(term, k), resident before timing
        stats = torch.zeros(abi.HB_STAT_COUNT, dtype=torch.int64, device=dev)
        for k in range(args.warmup):
            eng.step(d_group, d_info, d_terms[k], d_index, None, None, host=False)
        eng.set_stats_accum(stats)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for k in range(args.warmup, total):
            eng.step(d_group, d_info, d_terms[k], d_index, None, None, host=False)
        e1.record(stream)
        torch.cuda.synchronize()
        ms_local = e0.elapsed_time(e1)
        st_acc = stats.cpu().numpy().astype(np.uint64)
        timing = "K steps back to back, inputs resident in HBM"
    elif args.workload in ("follow", "mixed"):
        n_led = 0
        if args.workload == "follow":
            g, _ = synth.follow_groups(G, n, seed=seed, with_runs=False)
            b = synth.follow_batch(g, 0, seed=seed)
            inc = {"index": ((b["info"] & 0xF) == abi.HB_MSG_APP).astype(np.uint64),
                   "commit": np.ones(len(b["group"]), np.uint64)}
        else:
            g, _ = synth.mixed_groups(G, n, seed=seed, with_runs=False)
            if args.role_order:  # led groups first (stable): whole partitions of one role
                g = g[np.argsort(g["state"] != abi.HB_STATE_LEADER, kind="stable")]
            b, inc = synth.mixed_batch(g, 0, seed=seed)
            n_led = int((g["state"] == abi.HB_STATE_LEADER).sum())
        nmsg = len(b["group"])
        eng = Engine(G, max_replicas=n, max_inflight=W, max_batch=nmsg, device=local, stream=stream)
        eng.load_groups(g)
        del g

        def dv(a):
            return torch.from_numpy(np.ascontiguousarray(a).view(np.int32 if a.dtype == np.uint32 else np.int64)).to(dev)
        d_group, d_info, d_term, d_hint, d_eoff, d_eterm = (dv(b[k]) for k in ("group", "info", "term", "hint",
                                                                            "eoff", "eterm"))
        d_props = dv(b["props"]) if b.get("props") is not None else None
        i_inc, c_inc = dv(inc["index"]), dv(inc["commit"])
        i0, c0 = dv(b["index"]), dv(b["commit"])
        # step k continues the stream: every log is k entries longer (resident before timing)
        d_index = [i0 + i_inc * k for k in range(total)]
        d_commit = [c0 + c_inc * k for k in range(total)]
        stats = torch.zeros(abi.HB_STAT_COUNT, dtype=torch.int64, device=dev)

        def one(k, prof=False):
            eng.step(d_group, d_info, d_term, d_index[k], d_hint, d_props, host=False, eoff=d_eoff, commit=d_commit[k],
                     eterm=d_eterm, profile=prof)
        for k in range(args.warmup):
            one(k)
        eng.set_stats_accum(stats)
        eng.phase_reset()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for k in range(args.warmup, total):
            one(k, "apply" if (k - args.warmup) % 4 == 0 else False)  # HIP events around k_apply_fast
        e1.record(stream)
        torch.cuda.synchronize()
        ms_local = e0.elapsed_time(e1)
        st_acc = stats.cpu().numpy().astype(np.uint64)
        ph, nph = eng.phase_ms()
        apply_us = float(ph[abi.HB_PHASE_APPLY]) * 1e3
        fused_x = bool(eng.step_kernels() & abi.HB_KERN_ROUTE_FAST)  # (the apply phase brackets k_route_fast)
        timing = "K steps back to back, inputs resident in HBM"
    elif args.workload == "tick":
        g, _ = synth.steady_groups(G, n, seed=seed, with_runs=False)
        # half the groups lead (HeartbeatTick 1: a MsgBeat every tick), half
        # follow a leader elsewhere with ElectionTick 10 (draws past elapsed 10)
        fol = slice(G // 2, None) if args.role_order else slice(1, None, 2)  # (role-ordered: leaders first)
        g["state"][fol] = abi.HB_STATE_FOLLOWER
        g["lead"][fol] = 1
        eng = Engine(G, max_replicas=n, max_inflight=W, max_batch=1, device=local, stream=stream)
        eng.load_groups(g)
        del g
        t = synth.random_timers(G, seed=seed, et_hi=10, ht_hi=1, pos_hi=0)
        t["election_tick"] = 10
        eng.load_timers(t)
        eng.set_rand(np.random.default_rng(seed).integers(0, 1 << 63, 4 * total + 64, dtype=np.uint64))
        stats = torch.zeros(abi.HB_STAT_COUNT, dtype=torch.int64, device=dev)
        for k in range(args.warmup):
            eng.tick()
        eng.set_stats_accum(stats)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for k in range(args.warmup, total):
            eng.tick()
        e1.record(stream)
        torch.cuda.synchronize()
        ms_local = e0.elapsed_time(e1)
        st_acc = stats.cpu().numpy().astype(np.uint64)
        timing = "K ticks back to back"
    elif args.workload == "wire":
        g, _ = synth.steady_groups(G, n, seed=seed, with_runs=False)
        b0 = synth.cfg2_batch(g, 0, seed=seed)
        nmsg = len(b0["group"])
        eng = Engine(G, max_replicas=n, max_inflight=W, max_batch=nmsg, device=local, stream=stream)
        eng.load_groups(g)
        del g
        peers = np.zeros((G, abi.HB_MAX_REPLICAS), np.uint64)
        peers[:, :n] = np.arange(1, n + 1, dtype=np.uint64)
        eng.load_peers(peers)
        frm = ((b0["info"] >> 4) & 0xF).astype(np.uint64) + np.uint64(1)

        def tdev(a):
            return torch.from_numpy(np.ascontiguousarray(a).view(
                {1: np.uint8, 4: np.int32, 8: np.int64}[a.dtype.itemsize])).to(dev)
        recs, wire_bytes = [], 0
        for k in range(total):  # step k acks last + k + 1, encoded as the reference's MarshalTo writes it
            data, off, ln = synth.encode_responses(abi.HB_MSG_APP_RESP, np.ones(nmsg, np.uint64), frm, b0["term"],
                                                   b0["index"] + np.uint64(k))
            recs.append((tdev(data), tdev(off), tdev(ln)))
            wire_bytes = len(data)
        d_group, d_props = tdev(b0["group"]), tdev(b0["props"])
        out = {"group": torch.empty(nmsg, dtype=torch.int32, device=dev),
               "info": torch.empty(nmsg, dtype=torch.int32, device=dev),
               "term": torch.empty(nmsg, dtype=torch.int64, device=dev),
               "index": torch.empty(nmsg, dtype=torch.int64, device=dev),
               "hint": torch.empty(nmsg, dtype=torch.int64, device=dev)}
        status = torch.empty(nmsg, dtype=torch.uint8, device=dev)
        stats = torch.zeros(abi.HB_STAT_COUNT, dtype=torch.int64, device=dev)

        def one(k):
            eng.decode(recs[k][0], recs[k][1], recs[k][2], d_group, out, status)
            eng.step(out["group"], out["info"], out["term"], out["index"], out["hint"], d_props, host=False)
        for k in range(args.warmup):
            one(k)
        eng.set_stats_accum(stats)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for k in range(args.warmup, total):
            one(k)
        e1.record(stream)
        torch.cuda.synchronize()
        ms_local = e0.elapsed_time(e1)
        st_acc = stats.cpu().numpy().astype(np.uint64)
        bad = int((status != abi.HB_WIRE_OK).sum().item())
        # the decode kernel alone (it only writes the batch arrays, so it replays)
        eng.set_stats_accum(None)
        d0, d1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        d0.record(stream)
        for k in range(args.warmup, total):
            eng.decode(recs[k][0], recs[k][1], recs[k][2], d_group, out, status)
        d1.record(stream)
        torch.cuda.synchronize()
        dec_us = d0.elapsed_time(d1) * 1e3 / args.steps
        # + the From -> slot lookup: the group's n peer ids and n (one 64-byte row)
        alg = wire_bytes + nmsg * (8 + 4 + 4) + nmsg * (n + 1) * 8 + nmsg * (4 + 4 + 8 + 8 + 8 + 1)
        timing = "K (hb_decode + hb_step) back to back, wire records resident in HBM"
    else:
        g, _ = synth.lagging_groups(G, n, seed=seed, W=W)
        eng = Engine(G, max_replicas=n, max_inflight=W, max_batch=2 * G * n + G, device=local, stream=stream)
        eng.load_groups(g)
        rng = np.random.default_rng(seed)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        mix = np.zeros(5, np.int64)  # timed steps: acks, rejects, heartbeat resps, unreachable, groups proposing
        cfg3_ms, cfg3_n = [0.0, 0.0], [0, 0]  # (queued, idle-GPU) step time sums and counts
        for k in range(total):
            now = eng.get_groups()  # the stream is generated from the engine's state (untimed)
            b = synth.cfg3_open_batch(now, rng)
            del now
            if k >= args.warmup:
                t, rj = b["info"] & 0xF, (b["info"] >> 8) & 1
                mix += [int(((t == abi.HB_MSG_APP_RESP) & (rj == 0)).sum()), int(((t == abi.HB_MSG_APP_RESP) & (rj == 1)).sum()),
                        int((t == abi.HB_MSG_HEARTBEAT_RESP).sum()), int((t == abi.HB_MSG_UNREACHABLE).sum()),
                        int((b["props"] > 0).sum())]
            d = [torch.from_numpy(b[f].view(np.int32 if b[f].dtype == np.uint32 else np.int64)).to(dev)
                 for f in ("group", "info", "term", "index", "hint", "props")]
            torch.cuda.synchronize()
            # Alternate timed steps are taken on two bases: "queued" — a device-side wait
            # (torch.cuda._sleep, ~1 ms) ahead of e0, so the step's launches queue behind it
            # and the timed region is the device step (the other lines hide launch latency
            # by running their steps back to back) — and "idle" — e0 on an idle GPU, so the
            # host's launch latency is inside (the basis of the r01-r04 cfg3 lines).
            queued = (k - args.warmup) % 2 == 0
            if queued:
                torch.cuda._sleep(2_000_000)
            e0.record(stream)
            eng.step(*d, host=False)
            e1.record(stream)
            torch.cuda.synchronize()
            if k >= args.warmup:
                t = e0.elapsed_time(e1)
                cfg3_ms[0 if queued else 1] += t
                cfg3_n[0 if queued else 1] += 1
                st_acc += eng.stats()
        # the line's time: the queued basis' mean step, over every timed step
        ms_local = cfg3_ms[0] / max(cfg3_n[0], 1) * args.steps
        timing = ("per-step HIP event times, each step's launches queued behind a device-side wait (even timed "
                  "steps; the odd ones are timed from an idle GPU, launch latency included: ms_per_step_idle_gpu); "
                  "stream generation from the engine state between steps excluded")
    ms_t = torch.tensor([ms_local], dtype=torch.float64, device=dev)
    st_t = torch.from_numpy(st_acc.view(np.int64).copy()).to(dev)
    if world > 1:
        dist.all_reduce(ms_t, op=dist.ReduceOp.MAX)
        dist.all_reduce(st_t)
    ms = float(ms_t.item())
    st = st_t.cpu().numpy().view(np.uint64)
    sec = ms / 1e3
    if args.workload == "wire":
        metric, unit, val = "MsgAppResp applied/sec from raftpb wire records (hb_decode + hb_step, cfg2)", \
            "MsgAppResp/s", int(st[abi.HB_STAT_APPRESP]) / sec
        extra = {"commits_per_s": int(st[abi.HB_STAT_COMMITS]) / sec,
                 "decode": {"us_per_batch": round(dec_us, 2), "records_per_s": nmsg / (dec_us * 1e-6),
                            "wire_bytes_per_batch": wire_bytes, "records_not_ok": bad,
                            "roofline": {"bound": "hbm", "kernel": "k_decode",
                                         "achieved": round(alg / (dec_us * 1e-6) / 1e9, 1), "peak": HBM_PEAK_GBS,
                                         "unit": "GB/s", "frac": round(alg / (dec_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                                         "alg_bytes_per_launch": alg,
                                         "alg_bytes_note": f"record bytes + off/len/group 16 B + peer ids and "
                                                           f"n {(n + 1) * 8} B + batch record 32 B + status 1 B "
                                                           f"per record"}}}
        ok = int(st[abi.HB_STAT_COMMITS]) == world * G * args.steps and bad == 0 and int(st[abi.HB_STAT_FAULTS]) == 0
        wl = f"wire: cfg2 ({G} raft groups x {n} per GPU), MsgAppResp as raftpb wire records"
        data = "synthetic (cfg2 stream encoded with the reference's MarshalTo layout)"
    elif args.workload == "tick":
        metric, unit, val = "group ticks/sec (MultiNode.Tick over 1M groups x 3)", "group-ticks/s", \
            world * G * args.steps / sec
        # per group: meta 8 + tcfg 4 + elapsed 4 R + 4 W; a leader's MsgBeat reads committed and
        # each peer's Match and pm (8 + 12 B per peer: bcastHeartbeat); a MsgHup steps the whole
        # group (state ~100 B, SURVEY.md 8(d) per-group figures); events are 8 B words
        beats = world * (G // 2 + G % 2) * args.steps  # every leader beats on every tick (HeartbeatTick 1)
        hups = max(int(st[abi.HB_STAT_MSGS]) - beats, 0)
        alg = (G * 20 * args.steps + beats * (8 + 12 * (n - 1)) + hups * 100 + int(st[abi.HB_STAT_EVENTS]) * 8) / world
        alg_note = ("per tick: 20 B per group (meta, tcfg, elapsed r/w) + 8 + 12 B per peer per MsgBeat "
                    "(committed, Match, pm) + 100 B per MsgHup + 8 B per event word")
        extra = {"msgs_stepped_per_s": int(st[abi.HB_STAT_MSGS]) / sec, "events_per_s": int(st[abi.HB_STAT_EVENTS]) / sec,
                 "campaigns": int(st[abi.HB_STAT_MSGS]) - world * (G // 2 + G % 2) * args.steps}
        ok = int(st[abi.HB_STAT_FAULTS]) == 0
        wl = f"tick: {G} raft groups x {n} per GPU, half leaders (HeartbeatTick 1), half followers (ElectionTick 10)"
        data = "synthetic (cfg2 groups; seeded timers and r.rand stream)"
    elif args.workload == "cfg4":
        metric, unit, val = "MsgVoteResp tallied/sec + elections decided/sec (cfg4 election storm)", "MsgVoteResp/s", \
            int(st[abi.HB_STAT_VOTERESP]) / sec
        # 37 B per MsgVoteResp (message 24, vote masks 2R + 2W, state 1, Term 8);
        # 24 B per other message; every transition (each group steps down and campaigns, and a
        # decided election is a third) writes state/lead/Term/Vote ~26 B + n Progress resets x 30 B
        nvr = int(st[abi.HB_STAT_VOTERESP])
        trans = 2 * world * G * args.steps + int(st[abi.HB_STAT_WON]) + int(st[abi.HB_STAT_LOST])
        alg = (nvr * 37 + (int(st[abi.HB_STAT_MSGS]) - nvr) * 24 + trans * (26 + 30 * n)) / world
        alg_note = ("37 B per MsgVoteResp + 24 B per other message + (26 + 30 n) B per transition "
                    "(2 per group + 1 per decided election)")
        extra = {"elections_decided_per_s": (int(st[abi.HB_STAT_WON]) + int(st[abi.HB_STAT_LOST])) / sec,
                 "elections_won": int(st[abi.HB_STAT_WON]), "elections_lost": int(st[abi.HB_STAT_LOST])}
        ok = int(st[abi.HB_STAT_VOTERESP]) == world * G * (n - 1) * args.steps and int(st[abi.HB_STAT_FAULTS]) == 0
        wl = f"cfg4: {G} raft groups x {n} per GPU, election storm (step-down, MsgHup, {n - 1} MsgVoteResp per group)"
        data = "synthetic (seeded cfg4 storm replayed at +4 terms per step)"
    elif args.workload in ("follow", "mixed"):
        n_fol = G - n_led
        launch_alg = FOLLOW_GROUP_BYTES * n_fol + alg_bytes_per_group(n) * n_led  # per rank, per step
        alg = launch_alg * args.steps
        if n == 3 and fused_x:
            kname = "k_route_fast<2> (X mode: the route, FastLane + FollowLane in one kernel)"
            knames = ["k_route_fast<2u, true>"]
        elif n == 3:
            kname = "k_apply_fast<3> (X mode: FastLane + FollowLane)"
            knames = ["k_apply_fast<3, true, 2u>", "k_apply_fast<3, true>"]
        else:
            kname = f"k_apply_lead<{n}> (X mode: LeadLane + FollowLane)"
            knames = [f"k_apply_lead<{n}, true>", f"k_apply_lead<{n}>"]
        ach_k = launch_alg / (apply_us * 1e-6) / 1e9 if apply_us > 0 else 0.0
        tr, tsrc = pmc_traffic(args.traffic_json, knames, G, n, apply_us, workload=args.workload, layout=LAYOUT_RO
                               if args.role_order else None)
        extra = {"commits_per_s": int(st[abi.HB_STAT_COMMITS]) / sec, "entries_per_s": int(st[abi.HB_STAT_ENTRIES]) / sec,
                 "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(ach_k, 1), "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": round(ach_k / HBM_PEAK_GBS, 4), "traffic": tr,
                              "traffic_source": tsrc, "launch_us_timed": round(apply_us, 2),
                              "alg_bytes_per_launch": launch_alg,
                              "alg_bytes_note": follow_alg_note() + (
                                  f"; a led group {alg_bytes_per_group(n)} B (the cfg2 step: proposal + {n - 1} "
                                  f"MsgAppResp, SURVEY.md 8(d))" if n_led else ""),
                              "step_frac": round(alg / args.steps / (ms / args.steps * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}}
        msgs_per_step = 2 * n_fol + (n - 1) * n_led
        ok = int(st[abi.HB_STAT_COMMITS]) == world * G * args.steps and \
            int(st[abi.HB_STAT_MSGS]) == world * msgs_per_step * args.steps and int(st[abi.HB_STAT_FAULTS]) == 0
        if args.workload == "follow":
            metric, unit, val = "follower-side messages stepped/sec (MsgApp + MsgHeartbeat, follow workload)", \
                "msgs/s", int(st[abi.HB_STAT_MSGS]) / sec
            wl = f"follow: {G} raft groups x {n} per GPU that this node follows, MsgApp (1 entry) + MsgHeartbeat each"
            data = "synthetic (seeded follow stream: every group's leader appends one entry and heartbeats per step)"
        else:
            metric, unit, val = ("messages stepped/sec on a MultiNode node that leads 1/3 of its groups and follows "
                                 "2/3 (MsgAppResp + MsgApp + MsgHeartbeat in one batch)"), "msgs/s", \
                int(st[abi.HB_STAT_MSGS]) / sec
            extra["msgappresp_per_s"] = int(st[abi.HB_STAT_APPRESP]) / sec
            wl = (f"mixed: {G} raft groups x {n} per GPU, {n_led} led (proposal + {n - 1} MsgAppResp each) and "
                  f"{n_fol} followed (MsgApp with 1 entry + MsgHeartbeat each) in one batch")
            data = "synthetic (seeded mixed stream: a node's Ready cycle over the groups it leads and follows)"
    else:
        metric, unit, val = "MsgAppResp applied/sec (cfg3 lagging followers)", "MsgAppResp/s", \
            int(st[abi.HB_STAT_APPRESP]) / sec
        # Per message type, the SURVEY.md 8(d) rule (each field the reference reads once R / writes
        # once if changed W): MsgAppResp accept 66 B (message 24, Match 8R+8W, Next 8R, State+Paused
        # 2R, ins start/count 4R+4W, freed ring slot 8R); reject 64 B (message 24 + RejectHint 8,
        # Match 8R, Next 8R+8W, State 2R+2W, ins 4W: maybeDecrTo + becomeProbe); MsgHeartbeatResp
        # 43 B (message 24, State+count 3R, Match 8R, ring head 8R: freeFirstOne test); MsgUnreachable
        # 36 B (message 24, State 2R+2W, Next 8W); per group per batch 80 B (Term, committed R+W,
        # lastIndex R+W, termFirst, self Match R+W, delta 16 B); per MsgApp sent 21 B (State+count
        # 3R, Next 8W, ring slot 8W, count 2W) = events - commits - LAST events (one per proposing group)
        n_ack, n_rej, n_hb, n_unr, n_prop = (int(x) for x in mix)
        sends = max(int(st[abi.HB_STAT_EVENTS]) - int(st[abi.HB_STAT_COMMITS]) - world * n_prop, 0)
        alg = (n_ack * 66 + n_rej * 64 + n_hb * 43 + n_unr * 36 + world * G * args.steps * 80 + sends * 21) / world
        alg_note = ("per message type: MsgAppResp accept 66 B, reject 64 B, MsgHeartbeatResp 43 B, MsgUnreachable 36 B; "
                    "80 B per group per batch; 21 B per MsgApp sent (events - commits - proposing groups)")
        extra_mix = {"acks": n_ack // args.steps, "rejects": n_rej // args.steps, "heartbeat_resps": n_hb // args.steps,
                     "unreachable": n_unr // args.steps, "msgapp_sent": sends // args.steps // world}

        extra = {"msgs_per_s": int(st[abi.HB_STAT_MSGS]) / sec, "commits_per_s": int(st[abi.HB_STAT_COMMITS]) / sec,
                 "mix_per_step_rank0": extra_mix,
                 # both bases side by side (rank 0): the line's value is the queued one
                 "ms_per_step_queued": cfg3_ms[0] / max(cfg3_n[0], 1),
                 "ms_per_step_idle_gpu": cfg3_ms[1] / max(cfg3_n[1], 1) if cfg3_n[1] else None,
                 "value_idle_gpu": (int(st[abi.HB_STAT_APPRESP]) / (cfg3_ms[1] / cfg3_n[1] * args.steps / 1e3)
                                    if cfg3_n[1] and cfg3_ms[1] > 0 else None)}
        ok = int(st[abi.HB_STAT_FAULTS]) == 0
        wl = f"cfg3: {G} raft groups x {n} per GPU, lagging followers (W={W})"
        data = "synthetic (seeded open-loop cfg3 stream generated from the engine state each step)"
    if args.workload in ("cfg3", "cfg4", "tick"):
        # whole-step roofline (several kernels share the step; per-kernel times: profiles/*kernel_stats.csv)
        ach = alg / (ms / args.steps * 1e-3) / args.steps / 1e9 if ms > 0 else 0.0
        tr, tsrc = step_traffic(args.traffic_json, args.workload, G, n, ms / args.steps,
                                layout=LAYOUT_RO if args.role_order and args.workload == "tick" else None)
        extra["roofline"] = {"bound": "hbm", "kernel": "hb_step (whole step)" if args.workload != "tick" else
                             "hb_tick (k_tick + finish)", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": tr,
                             "traffic_source": tsrc,
                             "traffic_over_alg": round(tr / (alg / args.steps), 3) if tr else None,
                             "alg_bytes_per_step": round(alg / args.steps), "alg_bytes_note": alg_note}
    out = {"metric": metric, "value": val, "unit": unit, "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": ms / args.steps, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u64", "data": data,
           "config": dict({"workload": wl, "groups_per_gpu": G, "replicas": n, "max_inflight": W},
                          **({"layout": LAYOUT_RO} if args.role_order and args.workload in ("mixed", "tick") else {})),
           "stats": {nm: int(v) for nm, v in zip(abi.STAT_NAMES, st.tolist())}, "timing": timing,
           "parity_sanity": bool(ok), "wall_s": time.perf_counter() - t_wall, "cpu_baseline": None, **extra}
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = {"cfg4": cpu_baseline_cfg4, "cfg3": cpu_baseline_cfg3,
                                       "tick": cpu_baseline_tick, "wire": cpu_baseline_wire,
                                       "follow": cpu_baseline_follow, "mixed": cpu_baseline_mixed}[args.workload](n, W=W)
            except Exception as e:  # report, never fake
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out))


if __name__ == "__main__":
    main()
