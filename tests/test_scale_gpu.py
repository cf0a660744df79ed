"""GPU parity at the BASELINE.json sizes: the cfg5 per-GPU
shard (8M groups x 3), the cfg4 storm and the cfg3 open-loop stream at more
than 1M groups (two-pass bucket sort, k_bucket_bounds, k_route<8> / <6>,
k_apply<7> / <5>), and the sharded engine under two ranks.

Every case steps identical batches through the engine (C ABI) and the C
oracle and compares events, statistics and every group record bit-exactly.
"""
import threading
from datetime import timedelta

import numpy as np
import pytest

from etcd_amd import abi, synth
from etcd_amd.shard import ShardMap

from .parity_util import Pair, assert_events_equal, assert_groups_equal

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(900)
def test_cfg5_shard_8m_groups():
    """One GPU's cfg5 shard: 8,388,608 groups x 3 (2,048 buckets: the two-pass
    bucket sort), two cfg2 steps at W = 8 against the oracle, plus the step's
    size-independent properties (one commit per group, every ack applied)."""
    G = 8 * 1024 * 1024
    g, runs = synth.steady_groups(G, 3, seed=61, with_runs="flat")
    pair = Pair(g, runs, 3, 8, max_batch=2 * G + 16, oracle_shards=16)
    for step in range(2):
        _, st, now = pair.step(synth.cfg2_batch(g, step, seed=62 + step), ctx=f"cfg5 shard step {step}",
                               check_inflights=False)
        assert st[abi.HB_STAT_COMMITS] == G
        assert st[abi.HB_STAT_APPRESP] == 2 * G
        assert st[abi.HB_STAT_FAULTS] == 0
        assert np.array_equal(now["committed"], g["last_index"] + np.uint64(step + 1))
    # inflight windows of a sample of groups (each follower holds none after its ack)
    for gi in np.random.default_rng(63).integers(0, G, 64):
        for s in (1, 2):
            start, vals = pair.eng.get_inflights(int(gi), s)
            assert len(vals) == 0 and np.array_equal(vals, pair.og.inflights(int(gi), s))


@pytest.mark.timeout(900)
def test_tick_line_at_1m_groups():
    """The tick line's workload at full size: 1,048,576 groups x 3, half leading
    (HeartbeatTick 1: a MsgBeat every tick, k_tick's heartbeat path) and half
    following with ElectionTick 10 (draws; MsgHup campaigns through the general
    state machine), four ticks against the sharded oracle."""
    G = 1 << 20
    g, runs = synth.steady_groups(G, 3, seed=81, with_runs="flat")
    g["state"][1::2] = abi.HB_STATE_FOLLOWER
    g["lead"][1::2] = 1
    pair = Pair(g, runs, 3, 8, max_batch=16, oracle_shards=16)
    t = synth.random_timers(G, seed=82, et_hi=10, ht_hi=1, pos_hi=0)
    t["election_tick"] = 10
    pair.set_timers(t, np.random.default_rng(83).integers(0, 1 << 63, 64, dtype=np.uint64))
    camp = 0
    for k in range(4):
        _, st, _ = pair.tick(ctx=f"tick 1M {k}")
        assert st[abi.HB_STAT_FAULTS] == 0
        camp += int(st[abi.HB_STAT_MSGS]) - G // 2
    assert camp > 0  # some followers campaigned


@pytest.mark.timeout(900)
def test_cfg4_storm_over_1m_groups():
    """The bench's repeatable cfg4 storm at 1.1M groups x 7 (W = 8): step-down,
    MsgHup and 6 MsgVoteResp per group through the two-pass partition,
    k_route<8> and k_apply<7>, three storms on the state the last one left."""
    G = 1_100_000
    g, runs = synth.election_groups(G, 7, seed=71, with_runs="flat")
    pair = Pair(g, runs, 7, 8, max_batch=8 * G + 16, oracle_shards=16)
    b = synth.cfg4_storm_batch(g, seed=72)
    for k in range(3):
        _, st, _ = pair.step(dict(b, term=synth.storm_terms(b["term"], k)), ctx=f"storm 1.1M {k}",
                             check_inflights=False)
        assert st[abi.HB_STAT_VOTERESP] == G * 6
        assert st[abi.HB_STAT_WON] > G // 4 and st[abi.HB_STAT_FAULTS] == 0


@pytest.mark.timeout(900)
def test_cfg4_storm_full_4m_groups():
    """BASELINE.json configs[3] at its real size: 4,194,304 groups x 7, W = 8,
    the bench's own storm (bench.py --workload cfg4: same seed, groups and
    batch; 33.5M messages per step: a step-down, MsgHup and 6 MsgVoteResp per
    group), two storms on the state the first left, against the oracle (16
    shards on 16 cores): every event, statistic and group record."""
    G = 4 * 1024 * 1024
    seed = 0x5EED0004  # bench.py run_aux, rank 0
    g, runs = synth.election_groups(G, 7, seed=seed, with_runs="flat")
    pair = Pair(g, runs, 7, 8, max_batch=8 * G + 16, oracle_shards=16)
    b = synth.cfg4_storm_batch(g, seed=seed)
    del g, runs
    for k in range(2):
        _, st, _ = pair.step(dict(b, term=synth.storm_terms(b["term"], k)), ctx=f"storm 4M {k}",
                             check_inflights=False)
        assert st[abi.HB_STAT_VOTERESP] == G * 6
        assert st[abi.HB_STAT_WON] > G // 4 and st[abi.HB_STAT_FAULTS] == 0


@pytest.mark.timeout(900)
def test_cfg3_open_loop_over_1m_groups():
    """The bench's open-loop cfg3 stream at 1.1M groups x 5 (W = 8: full
    windows pause followers): lagging / stale / rejecting acks, heartbeats,
    unreachable and 1-4 entries per group, through k_route<6> and k_apply<5>."""
    G = 1_100_000
    g, runs = synth.lagging_groups(G, 5, seed=0x5EED0003, W=8, with_runs="flat")
    pair = Pair(g, runs, 5, 8, max_batch=12 * G, oracle_shards=16)
    rng = np.random.default_rng(81)
    now = pair.og.groups()
    for k in range(3):
        _, st, now = pair.step(synth.cfg3_open_batch(now, rng), ctx=f"cfg3 1.1M {k}", check_inflights=False)
        assert st[abi.HB_STAT_FAULTS] == 0 and st[abi.HB_STAT_APPRESP] > 3 * G
    # live inflight windows of a sample of groups
    for gi in np.random.default_rng(82).integers(0, G, 200):
        for s in range(1, 5):
            p = now[gi]["pr"][s]
            if p["state"] == abi.HB_PR_REPLICATE and p["ins_count"]:
                start, vals = pair.eng.get_inflights(int(gi), s)
                assert start == p["ins_start"] and np.array_equal(vals, pair.og.inflights(int(gi), s))


# ---------------------------------------------------------------- two ranks
def _global_case(kind):
    if kind == "cfg2":
        G = 6000
        g, runs = synth.steady_groups(G, 3, seed=91, last_hi=1 << 16)
        batches = [synth.cfg2_batch(g, k, seed=92 + k) for k in range(3)]
        return g, runs, 3, 256, {}, batches
    G = 2000
    g, runs, ins = synth.random_groups(G, 5, seed=93, W=8)
    batches = [synth.random_batch(g, 6000, seed=94 + k) for k in range(2)]
    return g, runs, 5, 8, ins, batches


def _local_events(ev, local_ids, idx):
    """A rank's events in global terms: group = global id, and the arrival
    index an event carries (MsgProp forward / drop, faults) = the message's
    position in the global batch."""
    ev = ev.copy()
    ev["group"] = local_ids[ev["group"]].astype(np.uint32)
    arr = np.isin(ev["type"], [abi.HB_EV_PROP_FWD, abi.HB_EV_PROP_DROP, abi.HB_EV_FAULT]) & \
        (ev["x"] != np.uint64(abi.HB_NO_INDEX))
    ev["x"][arr] = idx[ev["x"][arr].astype(np.int64)].astype(np.uint64)
    return ev


@pytest.mark.timeout(600)
@pytest.mark.parametrize("kind", ["cfg2", "fuzz"])
def test_two_ranks_sharded_engine_equals_oracle(kind):
    """Two ranks, gloo process groups, both on cuda:0 with a handle each
    (SURVEY.md 8(e)): each rank owns splitmix64(id) % 2 == rank, routes the
    global arrival-ordered batches with ShardMap.route_local and steps its
    shard; per-step statistics are all-reduced (the design's only collective).
    The summed statistics, the union of both ranks' events and group records
    must equal one oracle stepping every group in one process.

    The ranks are threads of this process with ProcessGroupGloo objects of
    their own: a GPU test process must not start programs after it has
    initialised the GPU, and the C ABI takes one handle per OS thread."""
    import torch
    import torch.distributed as dist
    from etcd_amd.hipbatch import Engine
    from oracle.pyoracle import OracleGroups

    g, runs, nmax, W, ins, batches = _global_case(kind)
    G = len(g)
    og = OracleGroups(g, runs, W, inflights=ins)
    init = og.groups()
    world = 2
    store = dist.HashStore()
    out = [None] * world
    err = [None] * world

    def rank_main(r):
        try:
            pg = dist.ProcessGroupGloo(dist.PrefixStore(f"two-rank-{kind}", store), r, world, timedelta(seconds=120))
            sm = ShardMap(np.arange(G, dtype=np.uint64), world, r)
            local = sm.local_ids.astype(np.int64)
            eng = Engine(len(local), max_replicas=nmax, max_inflight=W, max_batch=1 << 16, device=0)
            eng.load_groups(init[local])
            pos = {int(gl): i for i, gl in enumerate(local)}
            for (gg, s), vals in ins.items():
                if gg in pos:
                    eng.set_inflights(pos[gg], s, int(init[gg]["pr"][s]["ins_start"]), vals)
            res = []
            for b in batches:
                idx, slots = sm.route_local(b["group"].astype(np.uint64))
                lb = dict(group=slots, info=b["info"][idx], term=b["term"][idx], index=b["index"][idx],
                          hint=None if b.get("hint") is None else b["hint"][idx],
                          props=None if b.get("props") is None else b["props"][local])
                eng.step_batch(lb, host=True)
                ev = _local_events(eng.events(), local, idx)
                st = torch.from_numpy(eng.stats().view(np.int64).copy())
                pg.allreduce([st]).wait()
                res.append((ev, st.numpy().view(np.uint64).copy()))
            out[r] = (local, res, eng.get_groups())
            eng.close()
        except BaseException as e:  # reported by the main thread
            err[r] = e

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(500)
    for r in range(world):
        if err[r] is not None:
            raise err[r]
        assert out[r] is not None, f"rank {r} did not finish"
    assert sorted(np.concatenate([out[r][0] for r in range(world)]).tolist()) == list(range(G))
    for k, b in enumerate(batches):
        ora_ev, ora_st = og.step(b)
        for r in range(world):
            assert np.array_equal(out[r][1][k][1], ora_st), f"{kind} step {k}: reduced stats on rank {r}"
        dev_ev = np.concatenate([out[r][1][k][0] for r in range(world)])
        assert_events_equal(dev_ev, ora_ev, f"{kind} step {k}")
    final = og.groups()
    for r in range(world):
        local, _, recs = out[r]
        assert_groups_equal(recs, final[local], f"{kind} rank {r} records")
