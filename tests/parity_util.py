"""Shared parity harness: drive the engine (etcd_amd.hipbatch, HIP) and the C
oracle (oracle/, CPU) with identical batches and compare bit-exactly."""
import numpy as np

from etcd_amd import abi
from oracle.pyoracle import OracleGroups, ShardedOracleGroups


def sort_events(ev):
    """Events grouped per group, keeping each group's order (the only order the
    engine promises across groups)."""
    order = np.argsort(ev["group"], kind="stable")
    return ev[order]


def assert_events_equal(dev, ora, ctx=""):
    d, o = sort_events(dev), sort_events(ora)
    if len(d) != len(o) or not np.array_equal(d, o):
        gd = set(np.unique(d["group"]).tolist())
        go = set(np.unique(o["group"]).tolist())
        bad = sorted(g for g in gd | go
                     if not np.array_equal(d[d["group"] == g], o[o["group"] == g]))[:3]
        lines = [f"{ctx}: events differ (dev {len(d)}, oracle {len(o)}); first groups {bad}"]
        for g in bad:
            lines.append(f"  group {g}\n    dev: {d[d['group'] == g].tolist()}\n    ora: {o[o['group'] == g].tolist()}")
        raise AssertionError("\n".join(lines))


def assert_groups_equal(dev, ora, ctx=""):
    assert len(dev) == len(ora)
    # faulted groups: only the fault code is specified after the panic point
    live = ora["fault"] == 0
    assert np.array_equal(dev["fault"], ora["fault"]), f"{ctx}: fault codes differ"
    d, o = dev[live], ora[live]
    if not np.array_equal(d, o):
        idx = np.nonzero(d != o)[0][:3]
        gids = np.nonzero(live)[0][idx]
        msg = [f"{ctx}: group state differs at {gids.tolist()}"]
        for k, g in zip(idx, gids):
            for f in abi.GROUP_DTYPE.names:
                if not np.array_equal(d[k][f], o[k][f]):
                    msg.append(f"  g{g}.{f}: dev {d[k][f]} ora {o[k][f]}")
        raise AssertionError("\n".join(msg))


def assert_inflights_equal(eng, og, groups_now, ctx=""):
    for g in range(len(groups_now)):
        if groups_now[g]["fault"]:
            continue
        for s in range(int(groups_now[g]["n"])):
            p = groups_now[g]["pr"][s]
            if p["state"] != abi.HB_PR_REPLICATE or p["ins_count"] == 0:
                continue
            start, vals = eng.get_inflights(g, s)
            ov = og.inflights(g, s)
            assert start == p["ins_start"], f"{ctx}: g{g}/s{s} start"
            assert np.array_equal(vals, ov), f"{ctx}: g{g}/s{s} inflights dev {vals} ora {ov}"


class Pair:
    """An engine and an oracle loaded with the same groups."""

    def __init__(self, groups, runs, nmax, W, ins=None, max_msg_size=abi.HB_NO_LIMIT, max_batch=1 << 16,
                 sizes=None, term_runs=None, oracle_shards=1):
        from etcd_amd.hipbatch import Engine
        if oracle_shards > 1:  # full-size configurations: the oracle's groups stepped on several cores
            assert not ins and not sizes and not term_runs
            self.og = ShardedOracleGroups(groups, runs, W, max_msg_size, shards=oracle_shards)
        else:
            self.og = OracleGroups(groups, runs, W, max_msg_size, ins)
        init = self.og.groups()  # canonical record (term run derived from the log)
        self.eng = Engine(len(groups), max_replicas=nmax, max_inflight=W, max_msg_size=max_msg_size,
                          max_batch=max_batch)
        self.eng.load_groups(init)
        for (g, s), vals in (ins or {}).items():
            self.eng.set_inflights(g, s, int(init[g]["pr"][s]["ins_start"]), vals)
        self.sized = max_msg_size not in (0, abi.HB_NO_LIMIT)
        if sizes:  # finite max_msg_size: the entries' sizes on both sides
            self.og.load_sizes(sizes)
            self.eng.load_entry_sizes(sizes)
        if term_runs:  # follower side: the older term runs on both sides (True: all the log's)
            if term_runs is True:
                from etcd_amd import synth
                term_runs = synth.older_runs(init, runs)
            self.og.load_term_runs(term_runs)
            self.eng.load_term_runs(term_runs)
        assert_groups_equal(self.eng.get_groups(), init, "load")

    def reserve(self, batch=None, extra=0):
        """What a caller of the engine does before every step (hb_reserve_log):
        ring capacity for every group's log index covering its log plus what
        the batch can append — entries of its MsgProps / props / MsgApps, and
        one noop or new term run per message (`extra` per group for a tick)."""
        info = self.og.log_info().astype(np.int64)  # runs, sz_lo, first, last
        G = len(info)
        add = np.full(G, extra, dtype=np.int64)
        top = info[:, 3].copy()
        if batch is not None and len(batch["group"]):
            grp = np.asarray(batch["group"], dtype=np.int64)
            ok = grp < G
            add += np.bincount(grp[ok], minlength=G)[:G]
            t = np.asarray(batch["info"]) & 0xF
            idx = np.asarray(batch["index"], dtype=np.int64)
            prop = ok & (t == abi.HB_MSG_PROP)
            add += np.bincount(grp[prop], weights=idx[prop], minlength=G)[:G].astype(np.int64)
            if batch.get("eterm") is not None and batch.get("eoff") is not None:
                eoff = np.asarray(batch["eoff"], dtype=np.int64)
                ne = np.diff(np.append(eoff, len(batch["eterm"])))
                app = ok & (t == abi.HB_MSG_APP)
                add += np.bincount(grp[app], weights=ne[app], minlength=G)[:G].astype(np.int64)
                np.maximum.at(top, grp[app], idx[app] + ne[app])
        if batch is not None and batch.get("props") is not None:
            add += np.asarray(batch["props"], dtype=np.int64)[:G]
        runs = info[:, 0] + add + 1
        szc = (np.maximum(top, info[:, 3]) + add - info[:, 1] + 1) if self.sized else None
        self.eng.reserve_log(np.arange(G, dtype=np.uint32), szc, runs)

    def set_timers(self, timers, draws):
        self.draws = np.ascontiguousarray(draws, dtype=np.uint64)
        self.eng.load_timers(timers)
        self.og.load_timers(timers)
        self.eng.set_rand(self.draws)

    def tick(self, ctx="", check_inflights=False):
        """One MultiNode.Tick on both sides; events, stats, groups and timers equal."""
        self.reserve(extra=1)
        self.eng.tick()
        dev_ev = self.eng.events()
        dev_st = self.eng.stats()
        ora_ev, ora_st = self.og.tick(self.draws)
        assert_events_equal(dev_ev, ora_ev, ctx)
        assert np.array_equal(dev_st, ora_st), \
            f"{ctx}: stats dev {dict(zip(abi.STAT_NAMES, dev_st.tolist()))} ora {dict(zip(abi.STAT_NAMES, ora_st.tolist()))}"
        ora_g = self.og.groups()
        assert_groups_equal(self.eng.get_groups(), ora_g, ctx)
        dt, ot = self.eng.get_timers(), self.og.timers()
        bad = np.nonzero(dt != ot)[0]
        assert len(bad) == 0, f"{ctx}: timers differ at {bad[:5]}: dev {dt[bad[:3]]} ora {ot[bad[:3]]}"
        if check_inflights:
            assert_inflights_equal(self.eng, self.og, ora_g, ctx)
        return dev_ev, dev_st, ora_g

    def step(self, batch, ctx="", check_inflights=True):
        self.reserve(batch)
        self.eng.step_batch(batch, host=True)
        dev_ev = self.eng.events()
        dev_st = self.eng.stats()
        # the compact delta (hb_events_to_host words, expanded on the host) is the same stream
        words, counts = self.eng.event_words()
        assert np.array_equal(self.eng.expand_words(words, counts), dev_ev), f"{ctx}: compact words differ"
        ora_ev, ora_st = self.og.step(batch)
        assert_events_equal(dev_ev, ora_ev, ctx)
        assert np.array_equal(dev_st, ora_st), \
            f"{ctx}: stats dev {dict(zip(abi.STAT_NAMES, dev_st.tolist()))} ora {dict(zip(abi.STAT_NAMES, ora_st.tolist()))}"
        ora_g = self.og.groups()
        assert_groups_equal(self.eng.get_groups(), ora_g, ctx)
        if check_inflights:
            assert_inflights_equal(self.eng, self.og, ora_g, ctx)
        if getattr(self, "draws", None) is not None:  # transitions zero r.elapsed
            assert np.array_equal(self.eng.get_timers(), self.og.timers()), f"{ctx}: timers differ"
        return dev_ev, dev_st, ora_g
