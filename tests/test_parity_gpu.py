"""GPU parity: the HIP engine against the C oracle, bit-exact.

Every test steps identical batches through etcd_amd.hipbatch (libhipbatch.so on
the MI355X) and oracle/ (CPU), then compares the per-group event streams, the
batch statistics, every group's state and every live inflight window.
"""
import numpy as np
import pytest

from etcd_amd import abi, synth

from .parity_util import Pair

pytestmark = pytest.mark.gpu


def _empty(G, props=None):
    return dict(group=np.zeros(0, np.uint32), info=np.zeros(0, np.uint32), term=np.zeros(0, np.uint64),
                index=np.zeros(0, np.uint64), hint=None, props=props)


@pytest.mark.parametrize("G,n", [(1, 3), (1000, 3), (3000, 3), (2500, 5), (1500, 7)])
def test_cfg2_steady_replication(G, n):
    """cfg2 shape: props + every follower acks; exactly one commit advance per group."""
    g, runs = synth.steady_groups(G, n, seed=11 + G, last_hi=1 << 20)
    pair = Pair(g, runs, n, 256, max_batch=G * n + 16)
    for step in range(3):
        _, st, _ = pair.step(synth.cfg2_batch(g, step, seed=5 + step), ctx=f"cfg2 step {step}")
        assert st[abi.HB_STAT_COMMITS] == G
        assert st[abi.HB_STAT_APPRESP] == G * (n - 1)


@pytest.mark.parametrize("seed,nmax,W", [(1, 3, 8), (2, 5, 8), (3, 7, 4), (4, 3, 256), (5, 7, 16)])
def test_fuzz_all_message_types(seed, nmax, W):
    """Random states (all roles, progress states, inflight windows incl. full)
    and random messages of every device type, incl. stale/higher terms,
    non-members and reference panics."""
    g, runs, ins = synth.random_groups(1800, nmax, seed=seed, W=W)
    pair = Pair(g, runs, nmax, W, ins=ins, max_batch=1 << 15)
    for k in range(4):
        pair.step(synth.random_batch(g, 6000, seed=100 * seed + k), ctx=f"fuzz {seed}/{k}")


def test_fuzz_max_msg_size_zero():
    g, runs, ins = synth.random_groups(1200, 5, seed=9, W=8)
    pair = Pair(g, runs, 5, 8, ins=ins, max_msg_size=0, max_batch=1 << 15)
    for k in range(3):
        pair.step(synth.random_batch(g, 5000, seed=900 + k), ctx=f"maxmsg0/{k}")


def test_cfg4_election_storm():
    g, runs = synth.election_groups(3000, 7, seed=0x5EED0004)
    pair = Pair(g, runs, 7, 256, max_batch=1 << 16)
    _, st, after = pair.step(synth.cfg4_batch(g, seed=1), ctx="cfg4")
    assert st[abi.HB_STAT_VOTERESP] == 3000 * 6
    assert st[abi.HB_STAT_WON] > 0 and st[abi.HB_STAT_LOST] > 0
    # the new leaders then replicate: props + acks
    pair.step(_empty(3000, props=np.ones(3000, np.uint32)), ctx="cfg4 props")


def test_cfg3_lagging_followers_closed_loop():
    """Lagging followers, rejects with hints, heartbeats, unreachable, W=8
    (forces the full-inflights pause path); batches are produced by a follower
    simulator from the leader's own MsgApp events."""
    G = 2000
    g, runs = synth.lagging_groups(G, 5, seed=0x5EED0003)
    pair = Pair(g, runs, 5, 8, max_batch=1 << 16)
    sim = synth.FollowerSim(g, seed=3)
    b = _empty(G, props=np.ones(G, np.uint32))
    for k in range(6):
        ev, st, now = pair.step(b, ctx=f"cfg3 step {k}")
        b = sim.deliver(ev, now)


def test_hot_group_multi_chunk():
    """One group receives more messages than one LDS round (2048) holds."""
    g, runs = synth.steady_groups(1500, 3, seed=77, last_hi=5000)
    pair = Pair(g, runs, 3, 256, max_batch=1 << 15)
    rng = np.random.default_rng(1)
    hot = 1030
    N = 7000
    grp = np.where(rng.random(N) < 0.7, hot, rng.integers(0, 1500, N)).astype(np.uint32)
    slot = rng.integers(1, 3, N).astype(np.uint32)
    last = g["last_index"][grp].astype(np.int64)
    index = (last - rng.integers(0, 3, N)).astype(np.uint64)
    info = (abi.HB_MSG_APP_RESP | (slot << 4)).astype(np.uint32)
    b = dict(group=grp, info=info, term=g["term"][grp].astype(np.uint64), index=index, hint=None,
             props=np.ones(1500, np.uint32))
    pair.step(b, ctx="hot group")


def test_out_of_range_groups_and_empty_batch():
    g, runs = synth.steady_groups(1100, 3, seed=3, last_hi=100)
    pair = Pair(g, runs, 3, 16, max_batch=4096)
    pair.step(_empty(1100), ctx="empty")
    b = synth.cfg2_batch(g, 0)
    b["group"] = b["group"].copy()
    b["group"][:50] = 5000  # beyond capacity: ignored by both
    pair.step(b, ctx="oob")


def test_large_indices_long_event_words():
    """Indices and terms beyond 2^40 take two device event words (continuation)."""
    g, runs = synth.steady_groups(2000, 3, seed=21, last_hi=1 << 62, term_hi=1 << 50)
    pair = Pair(g, runs, 3, 16, max_batch=1 << 14)
    for step in range(2):
        _, st, _ = pair.step(synth.cfg2_batch(g, step, seed=31 + step), ctx=f"large step {step}")
        assert st[abi.HB_STAT_COMMITS] == 2000


def test_two_pass_partition_over_1m_groups():
    """> 256 buckets (1M groups): the bucket sort takes two 8-bit radix passes and
    bucket bounds come from a binary search; cfg2 then a random mix on top."""
    G = 1_100_000
    g, runs = synth.steady_groups(G, 3, seed=41, last_hi=1 << 30, with_runs="flat")
    pair = Pair(g, runs, 3, 256, max_batch=2 * G + 16)
    _, st, _ = pair.step(synth.cfg2_batch(g, 0, seed=42), ctx="2-pass cfg2", check_inflights=False)
    assert st[abi.HB_STAT_COMMITS] == G
    pair.step(synth.random_batch(g, 300_000, seed=43, props=False), ctx="2-pass random", check_inflights=False)


def test_hot_bucket_many_segments_and_rounds():
    """One bucket takes ~54k messages: the key scan spans several segments and
    every partition of the bucket several routing / general rounds; its groups
    have more messages than slots and go through the general state machine."""
    G = 20_000
    g, runs = synth.steady_groups(G, 3, seed=51, last_hi=5000)
    pair = Pair(g, runs, 3, 256, max_batch=1 << 17)
    rng = np.random.default_rng(52)
    N = 60_000
    grp = np.where(rng.random(N) < 0.9, rng.integers(0, 4096, N), rng.integers(0, G, N)).astype(np.uint32)
    slot = rng.integers(1, 3, N).astype(np.uint32)
    last = g["last_index"][grp].astype(np.int64)
    index = (last + 1 - rng.integers(0, 4, N)).astype(np.uint64)
    info = (abi.HB_MSG_APP_RESP | (slot << 4)).astype(np.uint32)
    b = dict(group=grp, info=info, term=g["term"][grp].astype(np.uint64), index=index, hint=None,
             props=np.ones(G, np.uint32))
    pair.step(b, ctx="hot bucket")


def test_pipelined_steps_with_input_stream():
    """Prep of step k+1 overlaps apply of step k (separate input stream, device
    batches, no sync between steps): the final state and the summed statistics
    equal stepping the same batches through the oracle."""
    import torch
    from etcd_amd.hipbatch import Engine
    from oracle.pyoracle import OracleGroups
    G, n = 50_000, 3
    g, runs = synth.steady_groups(G, n, seed=61, last_hi=1 << 20)
    og = OracleGroups(g, runs, 256)
    init = og.groups()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    eng = Engine(G, max_replicas=n, max_inflight=256, max_batch=4 * G, stream=stream)
    eng.set_input_stream(torch.cuda.Stream(device=dev))
    eng.load_groups(init)
    acc = torch.zeros(abi.HB_STAT_COUNT, dtype=torch.int64, device=dev)
    eng.set_stats_accum(acc)
    batches = [synth.cfg2_batch(g, k, seed=62 + k) for k in range(4)]
    batches.append(synth.random_batch(g, 40_000, seed=70))
    d = []
    for b in batches:
        t = {k: (torch.from_numpy(v.view(np.int32 if v.dtype == np.uint32 else np.int64)).to(dev) if v is not None
                 else None) for k, v in b.items()}
        d.append(t)
    torch.cuda.synchronize()
    for t in d:  # back to back: no sync, batches stay alive in `d`
        eng.step(t["group"], t["info"], t["term"], t["index"], t["hint"], t["props"], host=False)
    eng.sync()
    ora_sum = np.zeros(abi.HB_STAT_COUNT, dtype=np.uint64)
    for b in batches:
        _, st = og.step(b)
        ora_sum += st
    assert np.array_equal(acc.cpu().numpy().astype(np.uint64), ora_sum)
    from .parity_util import assert_groups_equal
    assert_groups_equal(eng.get_groups(), og.groups(), "pipelined")


@pytest.mark.parametrize("n", [5, 7])
def test_cfg4_storm_repeatable_stream(n):
    """The bench's repeatable cfg4 storm: step-down, campaign, n-1 votes, replayed
    at +4 terms per step on the state the previous storm left.  Every partition
    holds only groups k_apply_lead would hand over unloaded, so the route closes
    them (storm hand-over, k_route); the last step adds one leader to step in
    partition 3 (a MsgHeartbeatResp at its own term), so k_apply_lead runs that
    partition and the route closes the others."""
    G = 2500
    g, runs = synth.election_groups(G, n, seed=21)
    pair = Pair(g, runs, n, 64, max_batch=8 * G)
    b = synth.cfg4_storm_batch(g, seed=22)
    for k in range(3):
        _, st, _ = pair.step(dict(b, term=synth.storm_terms(b["term"], k)), ctx=f"storm {k}")
        assert st[abi.HB_STAT_VOTERESP] == G * (n - 1) and st[abi.HB_STAT_WON] > 0
        assert pair.eng.step_kernels() & abi.HB_KERN_ROUTE_ELECT  # (the election lane ran in the route)
    now = pair.og.groups()
    lead = np.flatnonzero((now["state"] == abi.HB_STATE_LEADER) & (np.arange(G) // 256 == 3))
    assert len(lead)
    x = int(lead[0])
    keep = b["group"] != x
    b3 = {k: (v[keep] if isinstance(v, np.ndarray) else v) for k, v in b.items()}
    b3["term"] = synth.storm_terms(b3["term"], 3)
    b3["group"] = np.append(b3["group"], np.uint32(x))
    b3["info"] = np.append(b3["info"], np.uint32(abi.HB_MSG_HEARTBEAT_RESP | (1 << 4)))
    b3["term"] = np.append(b3["term"], np.uint64(now["term"][x]))
    b3["index"] = np.append(b3["index"], np.uint64(0))
    pair.step(b3, ctx="storm 3 + a leader")


@pytest.mark.parametrize("W", [8, 256])
def test_cfg3_open_loop_stream(W):
    """The bench's open-loop cfg3 stream (lagging / stale / rejecting acks,
    heartbeats, unreachable, 1-4 entries per group) from the engine's own state."""
    G = 4000
    g, runs = synth.lagging_groups(G, 5, seed=0x5EED0003, W=W)
    pair = Pair(g, runs, 5, W, max_batch=8 * G)
    rng = np.random.default_rng(23)
    now = pair.og.groups()
    for k in range(5):
        _, st, now = pair.step(synth.cfg3_open_batch(now, rng), ctx=f"cfg3 open {k}")
        assert st[abi.HB_STAT_FAULTS] == 0


# ---------------------------------------------------------------- MultiNode.Tick
DRAWS = np.random.default_rng(77).integers(0, 1 << 63, 4096, dtype=np.uint64)


@pytest.mark.parametrize("seed,nmax,W", [(31, 3, 8), (32, 5, 8), (33, 7, 16)])
def test_tick_random_states(seed, nmax, W):
    """Ticks interleaved with batches over every role (leaders beat, followers
    and candidates time out on their own draw positions, non-promotable nodes
    stay at 0); steps zero r.elapsed on every reset."""
    G = 2000
    g, runs, ins = synth.random_groups(G, nmax, seed=seed, W=W)
    pair = Pair(g, runs, nmax, W, ins=ins, max_batch=1 << 15)
    pair.set_timers(synth.random_timers(G, seed=seed + 1, et_hi=6, ht_hi=3), DRAWS)
    for k in range(12):
        pair.tick(ctx=f"tick {seed}/{k}")
        if k % 4 == 3:
            pair.step(synth.random_batch(g, 3000, seed=1000 * seed + k), ctx=f"tick-step {seed}/{k}")


def test_tick_elections_and_heartbeats():
    """cfg4-shaped followers time out and campaign; the winners then beat."""
    G = 3000
    g, runs = synth.election_groups(G, 5, seed=41)
    pair = Pair(g, runs, 5, 64, max_batch=1 << 16)
    t = np.zeros(G, abi.TIMER_DTYPE)
    t["election_tick"], t["heartbeat_tick"] = 4, 2
    pair.set_timers(t, DRAWS)
    camp = 0
    for k in range(10):
        _, st, _ = pair.tick(ctx=f"tick {k}")
        camp += int(st[abi.HB_STAT_MSGS])
    assert camp >= G  # every group campaigned at least once
    # grant every candidate's votes, then leaders heartbeat on their ticks
    now = pair.og.groups()
    cand = np.nonzero(now["state"] == abi.HB_STATE_CANDIDATE)[0].astype(np.uint32)
    vg = np.repeat(cand, 4)
    vs = np.tile(np.arange(1, 5, dtype=np.uint32), len(cand))
    b = dict(group=vg, info=(abi.HB_MSG_VOTE_RESP | (vs << 4)).astype(np.uint32),
             term=now["term"][vg].astype(np.uint64), index=np.zeros(len(vg), np.uint64), hint=None, props=None)
    _, st, _ = pair.step(b, ctx="votes")
    assert st[abi.HB_STAT_WON] == len(cand)
    for k in range(4):
        pair.tick(ctx=f"beat {k}")


def test_tick_draws_exhausted():
    G = 600
    g, runs = synth.election_groups(G, 3, seed=43)
    pair = Pair(g, runs, 3, 8, max_batch=1 << 12)
    t = np.zeros(G, abi.TIMER_DTYPE)
    t["election_tick"], t["heartbeat_tick"] = 2, 1
    t["rand_pos"] = np.arange(G) % 40
    pair.set_timers(t, DRAWS[:20])
    for k in range(4):
        _, st, _ = pair.tick(ctx=f"exhaust {k}")
    assert (pair.og.groups()["fault"] == abi.HB_FAULT_RAND_EXHAUSTED).sum() > 0


@pytest.mark.parametrize("nmax", [5, 7])
def test_general_kernel_slot_boundary(nmax):
    """Handed-over groups with every message count around the route's slot
    capacity (route_kmax = n + 1 for n >= 5): counts <= capacity are stepped
    from the slots, larger ones by the bucket walk, mixed inside partitions,
    with proposals pending; random states and message types."""
    ks = nmax + 1
    G = 2048
    g, runs, ins = synth.random_groups(G, nmax, seed=40 + nmax, W=8)
    pair = Pair(g, runs, nmax, 8, ins=ins, max_batch=1 << 16)
    rng = np.random.default_rng(nmax)
    for k in range(3):
        counts = np.array([0, 1, ks - 1, ks, ks + 1, 2 * ks + 3])[rng.integers(0, 6, G)]
        if k == 1:
            counts[:256] = ks  # one whole partition on the slot path
            counts[256:512] = ks + 1  # one whole partition walking
        grp = rng.permutation(np.repeat(np.arange(G, dtype=np.uint32), counts))
        pair.step(synth.random_batch(g, 0, seed=500 + 10 * nmax + k, grp=grp),
                  ctx=f"slot boundary n={nmax}/{k}")


@pytest.mark.parametrize("seed,nmax,W,max_size", [(61, 3, 8, 40), (62, 5, 16, 150), (63, 7, 8, 1000),
                                                  (64, 5, 256, 1)])
def test_fuzz_finite_max_msg_size(seed, nmax, W, max_size):
    """A finite MaxSizePerMsg (raft/raft.go:265 + limitSize raft/util.go:97-110):
    fuzzed states and messages, MsgProps and dense proposals carrying entries of
    random payload sizes; every MsgApp's last entry (optimisticUpdate /
    inflights.add) follows limitSize over the entries' gogo sizes.  Groups whose
    caller loaded only part of the log's sizes fault HB_FAULT_SIZE_WINDOW (the
    engine's precondition) on both sides where a send reaches below them."""
    g, runs, ins = synth.random_groups(1200, nmax, seed=seed, W=W)
    sizes = synth.window_sizes(g, runs, seed=seed + 1)
    pair = Pair(g, runs, nmax, W, ins=ins, max_msg_size=max_size, sizes=sizes, max_batch=1 << 14)
    for k in range(3):
        b = synth.attach_entry_descs(synth.random_batch(g, 5000, seed=seed + 10 * k), len(g), seed=seed + 7 * k)
        pair.step(b, ctx=f"finite max size {max_size} step {k}")


def test_cfg2_finite_max_msg_size():
    """cfg2 shape (the fast kernel's proposal and accept path) under a finite
    MaxSizePerMsg: every proposal carries 1-3 entries of 0-300 bytes."""
    G, n = 4000, 3
    g, runs = synth.steady_groups(G, n, seed=65, last_hi=1 << 12)
    sizes = synth.window_sizes(g, runs, seed=66, frac_full=1.0)
    pair = Pair(g, runs, n, 256, max_msg_size=256, sizes=sizes, max_batch=4 * G)
    rng = np.random.default_rng(67)
    last = g["last_index"].copy()
    for step in range(3):
        b = synth.cfg2_batch(g, step, seed=68 + step)
        b["props"] = rng.integers(1, 4, G).astype(np.uint32)
        last = last + b["props"]
        b["index"] = last[b["group"]].astype(np.uint64)
        b = synth.attach_entry_descs(b, G, seed=69 + step, max_len=300)
        _, st, _ = pair.step(b, ctx=f"cfg2 finite step {step}")
        assert st[abi.HB_STAT_FAULTS] == 0


def _multinode_leader_batch(g, rng, last, ents):
    """A MultiNode leader-side cycle at n = 3: both followers ack the last
    index, then the application proposes (a MsgProp message of `ents[g]`
    entries, Term 0); all groups' messages interleaved in one random arrival
    order, each group's own in that order (ack, ack, proposal)."""
    G = len(g)
    grp = np.repeat(np.arange(G), 3)[rng.permutation(3 * G)].astype(np.uint32)
    kind = np.zeros(3 * G, np.int64)  # the group's 0th, 1st, 2nd message in arrival order
    seen = np.zeros(G, np.int64)
    for i, x in enumerate(grp):
        kind[i] = seen[x]
        seen[x] += 1
    t = np.where(kind == 2, abi.HB_MSG_PROP, abi.HB_MSG_APP_RESP).astype(np.uint32)
    slot = np.where(kind == 2, 0, kind + 1).astype(np.uint32)
    info = (t | (slot << np.uint32(4))).astype(np.uint32)
    term = np.where(kind == 2, 0, g["term"][grp].astype(np.int64)).astype(np.uint64)
    index = np.where(kind == 2, ents[grp], last[grp]).astype(np.uint64)
    return dict(group=grp, info=info, term=term, index=index, hint=None, props=None, msg_props=True)


@pytest.mark.parametrize("sized", [False, True])
def test_msgprop_messages_on_fast_lane(sized):
    """HB_STEP_MSG_PROPS (n = 3, a third route slot): a leader's two acks and
    the application's MsgProp of 1-3 entries, as a MultiNode cycle sends them,
    stay on the fast lane (stepLeader MsgProp -> appendEntry -> maybeCommit ->
    bcastAppend, raft/raft.go:500-513), with a finite MaxSizePerMsg taking the
    message's entry descriptors; then the same groups under fuzzed traffic of
    every type with the flag set."""
    G, n = 3000, 3
    g, runs = synth.steady_groups(G, n, seed=141, last_hi=1 << 12)
    kw = dict(max_msg_size=256, sizes=synth.window_sizes(g, runs, seed=142, frac_full=1.0)) if sized else {}
    pair = Pair(g, runs, n, 256, max_batch=4 * G, **kw)
    rng = np.random.default_rng(143)
    last = g["last_index"].astype(np.int64).copy()
    for step in range(3):
        ents = rng.integers(1, 4, G).astype(np.int64)
        b = _multinode_leader_batch(g, rng, last, ents)
        if sized:
            b = synth.attach_entry_descs(b, G, seed=144 + step, max_len=300)
        _, st, now = pair.step(b, ctx=f"msgprop fast lane step {step}")
        assert st[abi.HB_STAT_FAULTS] == 0 and st[abi.HB_STAT_ENTRIES] == int(ents.sum())
        last = last + ents
    b = synth.random_batch(now, 6000, seed=145, props=False)
    b["msg_props"] = True
    if sized:
        b = synth.attach_entry_descs(b, G, seed=146)
    pair.step(b, ctx="msgprop fuzz")


# ---------------------------------------------------------------- follower side
@pytest.mark.parametrize("seed,nmax,W", [(71, 3, 8), (72, 5, 16), (73, 7, 8), (74, 3, 256)])
def test_fuzz_follower_side(seed, nmax, W):
    """MsgApp (entries, conflicts, rejections), MsgHeartbeat, MsgSnap (restore /
    fast-forward / ignore) and MsgVote (grant / reject, senders outside prs)
    interleaved with every leader-side message type: k_apply hands a group over
    at its first follower-side message and k_follow steps the rest; events
    (responses, appends, restores), statistics, records, inflights and timers
    (the follower side zeroes r.elapsed) equal the oracle's."""
    g, runs, ins = synth.random_groups(1500, nmax, seed=seed, W=W)
    pair = Pair(g, runs, nmax, W, ins=ins, max_batch=1 << 15, term_runs=True)
    pair.set_timers(synth.random_timers(len(g), seed=seed), DRAWS)
    now = pair.og.groups()
    for k in range(4):
        f = synth.follower_messages(now, pair.og.term, 3000, seed=seed + 13 * k)
        b = synth.merge_batches(synth.random_batch(g, 3000, seed=seed + 7 * k), f, seed=seed + k)
        _, st, now = pair.step(b, ctx=f"follower fuzz {seed} step {k}")


def test_follower_replication_stream():
    """Steady follower-side replication: 20k follower groups, each step one
    MsgApp per group from its leader carrying 1-3 new entries at the leader's
    term (Index / LogTerm = the follower's last entry) and the leader's commit,
    plus heartbeats: every group appends, commits and answers."""
    G, n = 20_000, 3
    g, runs = synth.steady_groups(G, n, seed=91, last_hi=1 << 12)
    g["state"] = abi.HB_STATE_FOLLOWER
    g["lead"] = 1
    g["vote"] = 1
    for s in range(n):
        g["pr"][:, s]["state"] = abi.HB_PR_PROBE
    pair = Pair(g, runs, n, 256, max_batch=4 * G, term_runs=True)
    rng = np.random.default_rng(92)
    last = g["last_index"].astype(np.uint64).copy()
    term = g["term"].astype(np.uint64)
    for step in range(3):
        k = rng.integers(1, 4, G).astype(np.uint64)
        order = rng.permutation(G)
        eoff = np.concatenate([[0], np.cumsum(k[order])[:-1]]).astype(np.uint64)
        b = dict(group=order.astype(np.uint32),
                 info=np.full(G, abi.HB_MSG_APP | (1 << 4), np.uint32),
                 term=term[order], index=last[order], hint=term[order],
                 commit=(last[order] + k[order]), eoff=eoff,
                 eterm=np.repeat(term[order], k[order].astype(np.int64)).astype(np.uint64), props=None)
        _, st, now = pair.step(b, ctx=f"follower stream step {step}", check_inflights=False)
        last = last + k
        assert np.array_equal(now["last_index"], last)
        assert st[abi.HB_STAT_COMMITS] == G and st[abi.HB_STAT_FAULTS] == 0


@pytest.mark.parametrize("ents", [1, 3])
def test_follow_workload_fast_lane(ents):
    """The follow workload (bench.py --workload follow, the mirror of cfg2):
    every group's leader sends a MsgApp appending `ents` entries and a
    MsgHeartbeat; k_apply_fast's follower lane steps both (X-mode route
    extension: m.LogTerm / m.Commit beside each slot).  Then the same groups
    under random follower-side traffic (rejects, stale indices, higher terms,
    votes, snapshots) mixed with the workload, which the lane hands over at the
    first message it does not take."""
    G = 5000
    g, runs = synth.follow_groups(G, 3, seed=101, last_hi=1 << 14, with_runs=True)
    pair = Pair(g, runs, 3, 256, max_batch=4 * G, term_runs=True)
    for step in range(3):
        _, st, now = pair.step(synth.follow_batch(g, step, seed=102, ents=ents), ctx=f"follow {ents} step {step}",
                               check_inflights=False)
        assert st[abi.HB_STAT_COMMITS] == G and st[abi.HB_STAT_ENTRIES] == ents * G
        assert st[abi.HB_STAT_MSGS] == 2 * G and st[abi.HB_STAT_FAULTS] == 0
        assert np.array_equal(now["last_index"], g["last_index"] + np.uint64((step + 1) * ents))
    for k in range(3):
        f = synth.follower_messages(now, pair.og.term, 3000, seed=103 + k)
        b = synth.follow_batch(now, 0, seed=104 + k, ents=ents)
        keep = np.random.default_rng(k).random(len(b["group"])) < 0.5
        for key in ("group", "info", "term", "index", "hint", "commit"):
            b[key] = b[key][keep]
        ne = np.where((b["info"] & 0xF) == abi.HB_MSG_APP, ents, 0)
        b["eoff"] = np.concatenate([[0], np.cumsum(ne)[:-1]]).astype(np.uint64)
        b["eterm"] = np.repeat(b["term"], ne).astype(np.uint64)
        _, st, now = pair.step(_merge_follow(b, f, 105 + k), ctx=f"follow mixed {k}", check_inflights=False)


def test_follow_workload_long_records():
    """X mode with wide values: Terms up to 2^50 and log indices up to 2^62
    (past the 16-byte record's 24 / 40 bits: REC_LONG, the pair in the side
    table) on the follower lane, three steps, then mixed follower traffic."""
    G = 3000
    g, runs = synth.follow_groups(G, 3, seed=131, last_hi=1 << 62, term_hi=1 << 50, with_runs=True)
    pair = Pair(g, runs, 3, 256, max_batch=4 * G, term_runs=True)
    for step in range(3):
        _, st, now = pair.step(synth.follow_batch(g, step, seed=132), ctx=f"follow long step {step}",
                               check_inflights=False)
        assert st[abi.HB_STAT_COMMITS] == G and st[abi.HB_STAT_FAULTS] == 0
    f = synth.follower_messages(now, pair.og.term, 2000, seed=133)
    _, st, now = pair.step(f, ctx="follow long mixed", check_inflights=False)


def _merge_follow(a, b, seed):
    """Interleave two follower-side batches (each with entries), arrival order
    within each kept, entry offsets re-based."""
    rng = np.random.default_rng(seed)
    na, nb = len(a["group"]), len(b["group"])
    pick = np.zeros(na + nb, bool)
    pick[rng.choice(na + nb, nb, replace=False)] = True
    out = {}
    for k in ("group", "info", "term", "index", "hint", "commit"):
        v = np.empty(na + nb, a[k].dtype)
        v[~pick], v[pick] = a[k], b[k]
        out[k] = v
    ca = np.diff(np.append(a["eoff"], len(a["eterm"]))).astype(np.int64)
    cb = np.diff(np.append(b["eoff"], len(b["eterm"]))).astype(np.int64)
    cnt = np.zeros(na + nb, np.int64)
    cnt[~pick], cnt[pick] = ca, cb
    out["eoff"] = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.uint64)
    src_off = np.zeros(na + nb, np.int64)
    src_off[~pick], src_off[pick] = a["eoff"].astype(np.int64), b["eoff"].astype(np.int64) + len(a["eterm"])
    allterm = np.concatenate([a["eterm"], b["eterm"]]).astype(np.uint64)
    pos = np.repeat(src_off - out["eoff"].astype(np.int64), cnt) + np.arange(int(cnt.sum()))
    out["eterm"] = allterm[pos]
    out["props"] = None
    return out


# ---------------------------------------------------------------- the log index at depth
def test_deep_lag_finite_max_msg_size():
    """etcdserver's MaxSizePerMsg = 1 MiB (etcdserver/raft.go:229) with
    followers 5,000+ entries behind leaders whose logs hold 6,000-9,000
    entries of random payload sizes: heartbeat responses, rejections
    (maybeDecrTo to a random RejectHint) and acks make sendAppend cut
    entries(Next, 1 MiB) anywhere in the log (raft/raft.go:265, limitSize
    raft/util.go:97-110).  The log index holds every entry's size
    (hb_load_entry_sizes + hb_reserve_log), so no group faults and events,
    records and inflights equal the oracle's."""
    G, n = 500, 3
    g, runs = synth.deep_lag_leaders(G, n, seed=91)
    sizes = synth.window_sizes(g, runs, seed=92, max_len=900, frac_full=1.0)
    pair = Pair(g, runs, n, 64, max_msg_size=1 << 20, sizes=sizes, max_batch=1 << 14)
    rng = np.random.default_rng(93)
    for step in range(4):
        now = pair.og.groups()
        grp, info, term, index, hint = [], [], [], [], []
        for i in range(G):
            for s in range(1, n):
                p = now[i]["pr"][s]
                u = rng.random()
                rej = 0
                if u < 0.35:  # MsgHeartbeatResp: Match < lastIndex -> sendAppend
                    t, x, h = abi.HB_MSG_HEARTBEAT_RESP, 0, 0
                elif u < 0.6:  # reject of the last probe, follower far behind
                    t, x, h = abi.HB_MSG_APP_RESP, int(p["next"]) - 1, int(rng.integers(0, max(1, int(p["next"]))))
                    rej = 1
                else:  # ack of what was sent (or a stale ack)
                    t, x, h = abi.HB_MSG_APP_RESP, max(int(p["next"]) - 1, int(p["match"])), 0
                grp.append(i)
                info.append(t | (s << 4) | (rej << 8))
                term.append(int(now[i]["term"]))
                index.append(x)
                hint.append(h)
        order = rng.permutation(len(grp))
        b = dict(group=np.array(grp, np.uint32)[order], info=np.array(info, np.uint32)[order],
                 term=np.array(term, np.uint64)[order], index=np.array(index, np.uint64)[order],
                 hint=np.array(hint, np.uint64)[order], props=(rng.random(G) < 0.3).astype(np.uint32))
        b = synth.attach_entry_descs(b, G, seed=94 + step, max_len=900)
        _, st, ora = pair.step(b, ctx=f"deep lag step {step}")
        assert st[abi.HB_STAT_FAULTS] == 0 and (ora["fault"] == 0).all()
    sc, rc = pair.eng.log_capacity(0)
    assert sc >= 6000 and rc >= abi.HB_TERM_RING_MIN


@pytest.mark.parametrize("seed,nmax", [(95, 3), (96, 5)])
def test_follower_side_many_term_runs(seed, nmax):
    """Followers whose logs hold 18-30 term runs, probed by MsgApps anywhere in
    the log (matching and wrong LogTerms, conflicts that cut the log deep),
    MsgVote (isUpToDate) and MsgSnap: every raftLog.term lookup is answered from
    the log index (all runs loaded), no group faults, and the engine equals the
    oracle."""
    g, runs = synth.many_runs_groups(800, nmax, seed=seed)
    pair = Pair(g, runs, nmax, 16, max_batch=1 << 15, term_runs=True)
    for k in range(4):
        b = synth.follower_messages(pair.og.groups(), pair.og.term, 3000, seed=seed * 10 + k, deep=0.6)
        _, st, ora = pair.step(b, ctx=f"many runs n={nmax} step {k}")
        assert not (ora["fault"] == abi.HB_FAULT_TERM_WINDOW).any()


def test_log_index_precondition_faults():
    """Engine precondition, checked on both sides: a caller that loads no
    entry sizes (finite MaxSizePerMsg) or no older term runs gets
    HB_FAULT_SIZE_WINDOW / HB_FAULT_TERM_WINDOW exactly where the log index
    lacks the data (libhbnode always loads both, see test_follower_gpu.py)."""
    g, runs = synth.deep_lag_leaders(200, 3, seed=97, last_lo=300, last_hi=600, lag_min=200)
    pair = Pair(g, runs, 3, 16, max_msg_size=4096, max_batch=1 << 12)  # no sizes loaded
    grp = np.repeat(np.arange(200, dtype=np.uint32), 2)
    info = np.tile(np.array([abi.HB_MSG_HEARTBEAT_RESP | (1 << 4), abi.HB_MSG_HEARTBEAT_RESP | (2 << 4)],
                            np.uint32), 200)
    b = dict(group=grp, info=info, term=g["term"][grp].astype(np.uint64), index=np.zeros(400, np.uint64),
             hint=np.zeros(400, np.uint64), props=None, eoff=np.zeros(400, np.uint64))
    _, st, ora = pair.step(b, ctx="no sizes")
    assert (ora["fault"] == abi.HB_FAULT_SIZE_WINDOW).all()
    g2, runs2 = synth.many_runs_groups(300, 3, seed=98)
    pair2 = Pair(g2, runs2, 3, 16, max_batch=1 << 13)  # no term runs loaded
    b2 = synth.follower_messages(pair2.og.groups(), pair2.og.term, 1500, seed=99, deep=1.0)
    _, st2, ora2 = pair2.step(b2, ctx="no runs")
    assert (ora2["fault"] == abi.HB_FAULT_TERM_WINDOW).sum() > 50


# ---------------------------------------------------------------------------------------
# r.Commit before a group's first Step (hb_group.commit_zero, raft/raft.go:466,488,652)
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("seed,nmax,W", [(31, 3, 8), (32, 5, 8), (33, 7, 16)])
def test_fuzz_commit_zero(seed, nmax, W):
    """Groups whose r.Commit is still 0 (created with an empty HardState and not
    stepped since) next to groups whose r.Commit == committed, stepped with every
    leader- and follower-side message type: handleAppendEntries compares m.Index
    with r.Commit, so a MsgApp below committed is answered with MsgAppResp{Index:
    r.Commit} only once the group has stepped.  Every specialised lane hands such
    a group to the general one; events, statistics and records (commit_zero
    included) equal the oracle's after every step."""
    g, runs, ins = synth.random_groups(1500, nmax, seed=seed, W=W, commit_zero_p=0.5)
    assert g["commit_zero"].sum() > 300
    pair = Pair(g, runs, nmax, W, ins=ins, max_batch=1 << 15, term_runs=True)
    pair.set_timers(synth.random_timers(len(g), seed=seed), DRAWS)
    now = pair.og.groups()
    z0 = int(now["commit_zero"].sum())
    for k in range(3):
        f = synth.follower_messages(now, pair.og.term, 3000, seed=seed + 13 * k, deep=0.3)
        b = synth.merge_batches(synth.random_batch(g, 1500, seed=seed + 7 * k), f, seed=seed + k)
        _, st, now = pair.step(b, ctx=f"commit_zero fuzz {seed} step {k}")
        if k == 0:
            assert int(now["commit_zero"].sum()) < z0  # the groups stepped past the gate have r.Commit set


def test_fast_lanes_hand_over_commit_zero_groups():
    """The steady-state streams (cfg2 leaders on the fast lane, follow on the
    follower lane) over groups half of which still have r.Commit = 0: those are
    stepped by the general lane, whose first Step clears the flag; a follower
    receiving a MsgApp below committed answers with r.Commit (0 -> maybeAppend's
    match, or committed once stepped)."""
    g, runs = synth.steady_groups(4096, 3, seed=41, last_hi=1 << 12)
    g["commit_zero"] = (np.arange(4096) % 2).astype(np.uint32)
    pair = Pair(g, runs, 3, 256, max_batch=1 << 15)
    _, st, now = pair.step(synth.cfg2_batch(g, 0, seed=42), ctx="cfg2 commit_zero")
    assert st[abi.HB_STAT_COMMITS] == 4096 and not now["commit_zero"].any()
    f, fruns = synth.follow_groups(4096, 3, seed=43, last_hi=1 << 12, with_runs=True)
    f["commit_zero"] = (np.arange(4096) % 2).astype(np.uint32)
    pair = Pair(f, fruns, 3, 256, max_batch=1 << 15, term_runs=True)
    b = synth.follow_batch(f, 0, seed=44)
    _, st, now = pair.step(b, ctx="follow commit_zero")
    assert not now["commit_zero"].any()
    # an empty MsgApp below committed: r.Commit = 0 takes maybeAppend's match
    # (MsgAppResp{Index: m.Index}); r.Commit = committed answers with it
    f["commit_zero"] = (np.arange(4096) % 2).astype(np.uint32)
    pair = Pair(f, fruns, 3, 256, max_batch=1 << 15, term_runs=True)
    grp = np.nonzero(f["committed"] >= 2)[0].astype(np.uint32)
    n = len(grp)
    com = f["committed"][grp].astype(np.uint64)
    x = com - np.uint64(1)
    lt = np.array([pair.og.term(int(g), int(i)) for g, i in zip(grp, x)], np.uint64)
    b = dict(group=grp, info=np.full(n, abi.HB_MSG_APP | (1 << 4), np.uint32), term=f["term"][grp].astype(np.uint64),
             index=x, hint=lt, commit=com, eoff=np.zeros(n, np.uint64), eterm=np.zeros(0, np.uint64), props=None)
    ev, st, now = pair.step(b, ctx="below committed")
    resp = ev[ev["type"] == abi.HB_EV_RESP]
    want = np.where(grp % 2 == 1, x, com)
    assert np.array_equal(resp["x"][np.argsort(resp["group"], kind="stable")], want)


@pytest.mark.parametrize("seed", [51, 52])
def test_follower_lane_commit_past_log_end(seed):
    """An empty MsgApp past the log's end with LogTerm 0 matches (raftLog.term
    is 0 beyond lastIndex) and commitTo(min(m.Commit, m.Index)) may exceed
    lastIndex: the reference panics (raft/log.go:175-176).  The follower fast
    lane must not take it; the general lane reports HB_FAULT_COMMIT_RANGE, as
    the oracle does.  Directed groups plus a fuzz that mixes such probes into
    the X-mode follow stream."""
    f, fruns = synth.follow_groups(2048, 3, seed=seed, last_hi=1 << 12, with_runs=True)
    pair = Pair(f, fruns, 3, 256, max_batch=1 << 15, term_runs=True)
    G = 2048
    grp = np.arange(G, dtype=np.uint32)
    last = f["last_index"].astype(np.uint64)
    k = grp % 4
    # k = 0: commit past the end (panic); 1: commit within the log (ack of Index); 2, 3: the normal MsgApp
    index = np.where(k < 2, last + np.uint64(1) + (grp % 3).astype(np.uint64), last)
    commit = np.where(k == 0, index + np.uint64(1), np.where(k == 1, last, last))
    hint = np.where(k < 2, 0, f["term"]).astype(np.uint64)
    b = dict(group=grp, info=np.full(G, abi.HB_MSG_APP | (1 << 4), np.uint32), term=f["term"].astype(np.uint64),
             index=index.astype(np.uint64), hint=hint, commit=commit.astype(np.uint64),
             eoff=np.zeros(G, np.uint64), eterm=np.zeros(0, np.uint64), props=None)
    ev, st, now = pair.step(b, ctx="past-end probes")
    assert (now["fault"][k == 0] == abi.HB_FAULT_COMMIT_RANGE).all()
    assert (now["fault"][k != 0] == 0).all()
    assert st[abi.HB_STAT_FAULTS] == int((k == 0).sum())
    # fuzz: the follower-side generator with past-end probes, over fresh followers
    f2, fruns2 = synth.follow_groups(3000, 3, seed=seed + 100, last_hi=1 << 10, with_runs=True)
    pair2 = Pair(f2, fruns2, 3, 256, max_batch=1 << 15, term_runs=True)
    now = pair2.og.groups()
    for j in range(3):
        b = synth.follower_messages(now, pair2.og.term, 4000, seed=seed * 10 + j, past_end=0.2)
        _, st, now = pair2.step(b, ctx=f"past-end fuzz {seed} step {j}")
    assert (now["fault"] == abi.HB_FAULT_COMMIT_RANGE).sum() > 20


# ---------------------------------------------------------------- k_route_fast (r06) and its unfused form
@pytest.mark.parametrize("fuse", ["0", "1", "2"])
def test_route_fast_and_unfused_paths(fuse, monkeypatch):
    """n = 3 steps run the route inside the fast lane's workgroups
    (k_route_fast, HB_ROUTE_FUSE=2, the default; 1 = one-pass handles only) or
    as k_route + k_apply_fast (0).  Each form against the oracle on leader-side
    steps with two slots (cfg2), three slots (MsgProp batches) and X mode (the
    follow workload and random follower-side traffic); hb_step_kernels says
    which form ran.  (Two-pass handles: test_two_pass_partition_over_1m_groups,
    with the default.)"""
    monkeypatch.setenv("HB_ROUTE_FUSE", fuse)
    G = 3000
    g, runs = synth.steady_groups(G, 3, seed=161, last_hi=1 << 14)
    pair = Pair(g, runs, 3, 256, max_batch=4 * G)
    for step in range(2):
        pair.step(synth.cfg2_batch(g, step, seed=162 + step), ctx=f"fuse {fuse} cfg2 {step}")
        assert bool(pair.eng.step_kernels() & abi.HB_KERN_ROUTE_FAST) == (fuse != "0")
    rng = np.random.default_rng(163)
    last = g["last_index"].astype(np.int64) + 2
    ents = rng.integers(1, 4, G).astype(np.int64)
    _, _, now = pair.step(_multinode_leader_batch(g, rng, last, ents), ctx=f"fuse {fuse} msgprop")
    b = synth.random_batch(now, 6000, seed=164, props=False)
    b["msg_props"] = True
    pair.step(b, ctx=f"fuse {fuse} msgprop fuzz")
    # X mode
    gf, runsf = synth.follow_groups(G, 3, seed=165, last_hi=1 << 14, with_runs=True)
    pf = Pair(gf, runsf, 3, 256, max_batch=4 * G, term_runs=True)
    _, _, nowf = pf.step(synth.follow_batch(gf, 0, seed=166, ents=2), ctx=f"fuse {fuse} follow",
                         check_inflights=False)
    f = synth.follower_messages(nowf, pf.og.term, 3000, seed=167)
    pf.step(synth.merge_batches(synth.random_batch(nowf, 2000, seed=168), f, seed=169),
            ctx=f"fuse {fuse} follower fuzz", check_inflights=False)
