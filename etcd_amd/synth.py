"""Synthetic raft-group states and message streams (BASELINE.json configs).

Everything here is seeded and deterministic.  The generators build the
engine's record format (etcd_amd.abi) plus, for the parity oracle, the log term
runs of every group, so the oracle sees real per-entry terms while the device
sees only the current-term run.

  steady_groups / cfg2_batch    cfg2: 1M x 3 steady-state replication
  random_groups / random_batch  fuzz: every device message type and state
  election_groups / cfg4_batch  cfg4: election storm (MsgHup + MsgVoteResp)
  cfg4_storm_batch              cfg4, repeatable: every step first steps each
                                group down (higher term), then the storm
  FollowerSim                   cfg3: closed-loop lagging followers driven by
                                the leader's MsgApp events
  cfg3_open_batch               cfg3, open loop from the engine's current state
                                (vectorized, for the 1M x 5 bench)
"""
import numpy as np

from . import abi

A = abi


def splitmix64(x):
    """splitmix64 finalizer (vectorized, uint64) — used to shard group ids."""
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _runs_for(first, tf, last, term):
    """Log term runs for a group whose current-term run is [tf, last]: the dummy
    entry (first-1) and the entries before tf carry term-1."""
    if tf <= first - 1:
        return [(first - 1, int(term))]
    return [(first - 1, max(int(term) - 1, 0)), (int(tf), int(term))]


# ---------------------------------------------------------------------------- cfg2
def steady_groups(G, n=3, seed=0x5EED0002, last_hi=1 << 20, term_hi=1000, with_runs=True):
    """All groups leader (self = slot 0), followers Replicate with empty inflights,
    every Match = committed = lastIndex; term ~ U[1, term_hi]; termFirst ~ U[1, last].
    with_runs: True (list of term runs per group), "flat" ((index, term) rows plus
    per-group offsets, for large G) or False."""
    rng = np.random.default_rng(seed)
    g = np.zeros(G, dtype=A.GROUP_DTYPE)
    term = rng.integers(1, term_hi + 1, G, dtype=np.uint64)
    last = rng.integers(1, last_hi + 1, G, dtype=np.uint64)
    tf = (rng.random(G) * last).astype(np.uint64) + np.uint64(1)
    tf = np.minimum(tf, last)
    g["term"], g["committed"], g["first_index"], g["last_index"] = term, last, 1, last
    g["term_first"], g["term_last"], g["snap_index"] = tf, last, 0
    g["state"], g["n"], g["self_slot"] = A.HB_STATE_LEADER, n, 0
    g["lead"], g["vote"] = 0, 0
    pr = g["pr"]
    for s in range(n):
        pr[:, s]["match"] = last
        pr[:, s]["next"] = last + np.uint64(1)
        pr[:, s]["state"] = A.HB_PR_PROBE if s == 0 else A.HB_PR_REPLICATE
    runs = None
    if with_runs == "flat":  # (flat [2G, 2] (index, term), offsets [G+1]): first = 1 < tf always
        flat = np.zeros((G, 2, 2), dtype=np.uint64)
        flat[:, 0, 1] = np.maximum(term.astype(np.int64) - 1, 0).astype(np.uint64)
        flat[:, 1, 0], flat[:, 1, 1] = tf, term
        runs = (flat.reshape(-1, 2), np.arange(0, 2 * G + 1, 2, dtype=np.uint64))
    elif with_runs:
        runs = [_runs_for(1, int(tf[i]), int(last[i]), int(term[i])) for i in range(G)]
    return g, runs


def cfg2_batch(groups, step, seed=0x5EED0002, xp=np):
    """One cfg2 step: one proposal per group (dense props) then every follower acks
    the new last index (MsgAppResp, Term = group term), in a random permutation."""
    G = len(groups)
    n = int(groups["n"][0])
    rng = np.random.default_rng(seed + 7919 * step)
    nf = n - 1
    grp = np.repeat(np.arange(G, dtype=np.uint32), nf)
    slot = np.tile(np.arange(1, n, dtype=np.uint32), G)
    perm = rng.permutation(G * nf)
    grp, slot = grp[perm], slot[perm]
    info = (np.uint32(A.HB_MSG_APP_RESP) | (slot << np.uint32(4))).astype(np.uint32)
    term = groups["term"][grp].astype(np.uint64)
    index = (groups["last_index"][grp] + np.uint64(step + 1)).astype(np.uint64)
    props = np.ones(G, dtype=np.uint32)
    return dict(group=grp, info=info, term=term, index=index, hint=None, props=props)


def global_ack_stream(G_total, n=3, seed=0x5EED0005):
    """The arrival stream of one cfg2/cfg5 step over a GLOBAL group-id space
    [0, G_total): every follower of every group acks once, in a random order
    (the same on every rank).  Returns (group id u64, from slot u32); a rank
    routes it to its own shard (ShardMap.route_local) and fills Term / Index
    from its groups' state (cfg2_local_batch)."""
    nf = n - 1
    perm = np.random.default_rng(seed).permutation(G_total * nf)
    gid = (perm // nf).astype(np.uint64)
    frm = (perm % nf + 1).astype(np.uint32)
    return gid, frm


def cfg2_local_batch(groups, slots, frm, step):
    """A rank's routed cfg2 step: MsgAppResp from `frm` for local group `slots`
    (arrival order as routed), Term = the group's term, Index = last + step + 1,
    plus one dense proposal per group."""
    info = (np.uint32(A.HB_MSG_APP_RESP) | (frm.astype(np.uint32) << np.uint32(4))).astype(np.uint32)
    term = groups["term"][slots].astype(np.uint64)
    index = (groups["last_index"][slots] + np.uint64(step + 1)).astype(np.uint64)
    return dict(group=slots.astype(np.uint32), info=info, term=term, index=index, hint=None,
                props=np.ones(len(groups), dtype=np.uint32))


# ---------------------------------------------------------------------------- fuzz
def random_groups(G, nmax=3, seed=1, W=8, state_mix=(0.6, 0.2, 0.2), commit_zero_p=0.0):
    """Diverse, internally consistent group states for fuzz parity;
    `commit_zero_p`: the share of groups whose r.Commit is still 0 (created
    with an empty HardState and not stepped since, hb_group.commit_zero).

    Returns (groups, runs, inflights{(g, slot): values})."""
    rng = np.random.default_rng(seed)
    g = np.zeros(G, dtype=A.GROUP_DTYPE)
    runs, ins = [], {}
    for i in range(G):
        r = g[i]
        n = int(rng.integers(1, nmax + 1))
        term = int(rng.integers(1, 40))
        first = int(rng.integers(1, 20))
        last = first - 1 + int(rng.integers(0, 30))
        # non-decreasing terms <= term over [first-1, last]
        k = int(rng.integers(1, 4))
        cuts = sorted(set([first - 1] + [int(x) for x in rng.integers(first - 1, last + 1, k)]))
        ts = sorted(int(x) for x in rng.integers(0, term + 1, len(cuts)))
        if rng.random() < 0.5:
            ts[-1] = term
        rr = []
        for c, t in zip(cuts, ts):
            if rr and rr[-1][1] == t:
                continue
            rr.append((c, t))
        runs.append(rr)
        st = int(rng.choice(3, p=[state_mix[1] if j == 1 else state_mix[0] if j == 2 else state_mix[2]
                                   for j in range(3)]))
        self_slot = int(rng.integers(0, n)) if rng.random() > 0.05 else A.HB_SLOT_NONE
        committed = int(rng.integers(first - 1, last + 1))
        r["term"], r["committed"], r["first_index"], r["last_index"] = term, committed, first, last
        r["snap_index"] = first - 1 if (first > 1 or rng.random() < 0.5) else 0
        r["state"], r["n"], r["self_slot"] = st, n, self_slot
        refs = list(range(n)) + [A.HB_REF_NONE, A.HB_REF_NONE, A.HB_REF_OTHER]
        self_ref = self_slot if self_slot != A.HB_SLOT_NONE else A.HB_REF_SELF
        if st == A.HB_STATE_LEADER:
            r["lead"], r["vote"] = self_ref, self_ref
        elif st == A.HB_STATE_CANDIDATE:
            r["lead"], r["vote"] = A.HB_REF_NONE, self_ref
            bits = [s for s in range(n)] + ([7] if self_slot == A.HB_SLOT_NONE else [])
            resp = 0
            grant = 0
            for b in bits:
                if rng.random() < 0.4:
                    resp |= 1 << b
                    if rng.random() < 0.5:
                        grant |= 1 << b
            sb = 7 if self_slot == A.HB_SLOT_NONE else self_slot
            resp |= 1 << sb
            grant |= 1 << sb
            r["votes_resp"], r["votes_grant"] = resp, grant
        else:
            r["lead"] = int(rng.choice(refs))
            r["vote"] = int(rng.choice(refs))
        for s in range(n):
            p = r["pr"][s]
            if st != A.HB_STATE_LEADER or rng.random() < 0.2:
                p["match"] = last if s == self_slot else 0
                p["next"] = last + 1
                continue
            m = int(rng.integers(0, last + 1))
            nx = int(rng.integers(m + 1, last + 2))
            ps = int(rng.choice(3, p=[0.4, 0.45, 0.15]))
            p["match"], p["next"], p["state"] = m, nx, ps
            if ps == A.HB_PR_PROBE:
                p["paused"] = int(rng.random() < 0.4)
            elif ps == A.HB_PR_SNAPSHOT:
                p["pending_snapshot"] = int(rng.integers(0, last + 2))
            else:
                p["ins_start"] = int(rng.integers(0, W))
                room = nx - 1 - m
                cnt = int(rng.integers(0, min(W, room) + 1)) if room > 0 else 0
                if rng.random() < 0.15 and room >= W:
                    cnt = W
                if cnt:
                    vals = np.sort(rng.choice(np.arange(m + 1, nx), size=cnt, replace=False)).astype(np.uint64)
                    ins[(i, s)] = vals
                p["ins_count"] = cnt
    if commit_zero_p > 0:  # (drawn after the groups: the streams above are unchanged)
        g["commit_zero"] = ((rng.random(G) < commit_zero_p) & (g["committed"] > 0)).astype(np.uint32)
    return g, runs, ins


_TYPES = np.array([A.HB_MSG_APP_RESP, A.HB_MSG_HEARTBEAT_RESP, A.HB_MSG_VOTE_RESP, A.HB_MSG_UNREACHABLE,
                   A.HB_MSG_SNAP_STATUS, A.HB_MSG_PROP, A.HB_MSG_BEAT, A.HB_MSG_HUP])
_TYPE_P = np.array([0.42, 0.10, 0.16, 0.04, 0.05, 0.12, 0.05, 0.06])


def random_batch(groups, nmsg, seed=2, nonmember=0.04, props=True, grp=None):
    """Random messages of every device type against `groups` (ids < len(groups));
    `grp`: the message groups in arrival order (default: uniform)."""
    rng = np.random.default_rng(seed)
    G = len(groups)
    if grp is None:
        grp = rng.integers(0, G, nmsg).astype(np.uint32)
    else:
        grp = np.ascontiguousarray(grp, dtype=np.uint32)
        nmsg = len(grp)
    t = rng.choice(_TYPES, size=nmsg, p=_TYPE_P / _TYPE_P.sum()).astype(np.uint32)
    n = groups["n"][grp].astype(np.int64)
    slot = (rng.random(nmsg) * n).astype(np.uint32)
    slot[rng.random(nmsg) < nonmember] = A.HB_SLOT_NONE
    reject = (rng.random(nmsg) < 0.25).astype(np.uint32)
    gterm = groups["term"][grp].astype(np.int64)
    u = rng.random(nmsg)
    term = np.where(u < 0.62, gterm, np.where(u < 0.74, 0, np.where(u < 0.87, gterm - 1, gterm + 1)))
    term = np.maximum(term, 0).astype(np.uint64)
    local = (t == A.HB_MSG_HUP) | (t == A.HB_MSG_BEAT) | (t == A.HB_MSG_PROP) | (t == A.HB_MSG_SNAP_STATUS) | \
            (t == A.HB_MSG_UNREACHABLE)
    term[local & (rng.random(nmsg) < 0.85)] = 0
    last = groups["last_index"][grp].astype(np.int64)
    index = np.maximum(last + rng.integers(-4, 4, nmsg), 0).astype(np.uint64)
    pm = t == A.HB_MSG_PROP
    index[pm] = rng.integers(1, 4, int(pm.sum()))
    index[pm & (rng.random(nmsg) < 0.02)] = 0
    hint = np.maximum(last + rng.integers(-6, 2, nmsg), 0).astype(np.uint64)
    info = (t | (slot << np.uint32(4)) | (reject << np.uint32(8))).astype(np.uint32)
    pr = None
    if props:
        pr = np.where(rng.random(G) < 0.3, rng.integers(1, 3, G), 0).astype(np.uint32)
    return dict(group=grp, info=info, term=term, index=index, hint=hint, props=pr)


def attach_entry_descs(batch, G, seed=3, max_len=64, nil_p=0.2, conf_p=0.1):
    """Finite MaxSizePerMsg batches: random entry descriptors (HB_ENT_DESC) for
    every entry a batch may append — each MsgProp message's index[i] entries
    (eoff) and each dense proposal's props[g] entries (peoff)."""
    rng = np.random.default_rng(seed)
    t = batch["info"] & np.uint32(0xF)
    k = np.where(t == A.HB_MSG_PROP, batch["index"], 0).astype(np.uint64)
    pk = batch["props"].astype(np.uint64) if batch.get("props") is not None else np.zeros(G, np.uint64)
    eoff = np.zeros(len(k), np.uint64)
    eoff[1:] = np.cumsum(k)[:-1]
    peoff = (k.sum() + np.concatenate([[0], np.cumsum(pk)[:-1]])).astype(np.uint64)
    total = int(k.sum() + pk.sum())
    ln = rng.integers(0, max_len + 1, total).astype(np.uint32)
    has = (rng.random(total) >= nil_p).astype(np.uint32)
    et = (rng.random(total) < conf_p).astype(np.uint32)
    edesc = np.where(has == 1, ln, 0).astype(np.uint32) | (et << np.uint32(30)) | (has << np.uint32(31))
    return dict(batch, edesc=edesc.astype(np.uint32), eoff=eoff, peoff=peoff if batch.get("props") is not None
                else None)


def window_sizes(groups, runs, seed=4, max_len=64, frac_full=0.7):
    """Entry.Size() of each group's latest entries (hb_load_entry_sizes): random
    payloads for the entries the log already holds, their Term from the log's
    term runs; most groups get their whole log (firstIndex .. lastIndex), the
    rest only a few entries (a caller that loads less than the log: sends
    further back fault HB_FAULT_SIZE_WINDOW, the engine's precondition)."""
    rng = np.random.default_rng(seed)
    out = {}
    for g in range(len(groups)):
        first, last = int(groups["first_index"][g]), int(groups["last_index"][g])
        avail = last - (first - 1)
        k = avail if rng.random() < frac_full else int(rng.integers(0, avail + 1))
        rr = np.asarray(runs[g], dtype=np.uint64).reshape(-1, 2)
        idx = np.arange(last - k + 1, last + 1, dtype=np.uint64)
        term = rr[np.searchsorted(rr[:, 0], idx, side="right") - 1, 1] if k else idx
        ln = rng.integers(0, max_len + 1, k).astype(np.uint64)
        typ = (rng.random(k) < 0.1).astype(np.uint64)
        has = rng.random(k) >= 0.2
        z = 3 + _sov(typ) + _sov(term) + _sov(idx) + np.where(has, 1 + ln + _sov(ln), 0)
        out[g] = z.astype(np.uint32).tolist()
    return out


def _sov(x):
    """sovRaft (varint length) of a uint64 array."""
    x = np.asarray(x, dtype=np.uint64)
    n = np.ones(x.shape, dtype=np.uint64)
    y = x >> np.uint64(7)
    while y.any():
        n += (y > 0).astype(np.uint64)
        y >>= np.uint64(7)
    return n


def older_runs(groups, runs, keep=None):
    """The log term runs below each group's current-term run (term_first), all
    of them or the newest `keep`: what hb_load_term_runs takes (follower side)."""
    out = {}
    for g in range(len(groups)):
        tf = int(groups["term_first"][g])
        rr = [(int(i), int(t)) for i, t in runs[g] if tf == A.HB_NO_INDEX or int(i) < tf]
        out[g] = rr if keep is None else rr[max(len(rr) - keep, 0):]
    return out


def follower_messages(now, term_of, nmsg, seed=5, nonmember=0.05, max_ents=4, deep=0.0, past_end=0.0):
    """Random follower-side messages (MsgApp with entries / MsgHeartbeat /
    MsgSnap / MsgVote) against the groups' current state `now`; term_of(g, i)
    gives a group's log term (the oracle's).  Mostly well-formed (matching
    LogTerms, entries continuing the log at the message's term), with stale,
    conflicting, rejected and out-of-range cases mixed in; every entry and
    snapshot term is one a leader could send (non-decreasing, <= the group's
    term after the gate), so the log keeps the reference's term order.
    `past_end`: the share of MsgApps that are empty LogTerm-0 probes past the
    log's end (raftLog.term is 0 there, so they match) whose m.Commit lies
    beyond lastIndex — commitTo's out-of-range panic (raft/log.go:175-176).
    Returns the batch arrays plus commit / eterm / eoff."""
    rng = np.random.default_rng(seed)
    G = len(now)
    grp, info, term, index, hint, commit, eoff, eterm = [], [], [], [], [], [], [], []
    types = [A.HB_MSG_APP, A.HB_MSG_HEARTBEAT, A.HB_MSG_SNAP, A.HB_MSG_VOTE]
    for _ in range(nmsg):
        g = int(rng.integers(0, G))
        r = now[g]
        n = int(r["n"])
        t = types[int(rng.choice(4, p=[0.55, 0.2, 0.05, 0.2]))]
        slot = int(rng.integers(0, n)) if rng.random() > nonmember else A.HB_SLOT_NONE
        voted = int(slot == A.HB_SLOT_NONE and rng.random() < 0.5)
        gt, last, com = int(r["term"]), int(r["last_index"]), int(r["committed"])
        u = rng.random()
        mt = gt if u < 0.7 else (gt + 1 if u < 0.85 else (0 if u < 0.92 else max(gt - 1, 0)))
        # the term the group has after the gate; a leader of that term never sends
        # an entry or a snapshot of a later term, and its log's terms never decrease
        if t == A.HB_MSG_SNAP and mt == 0:  # a candidate takes a MsgSnap's Term as its own (raft/raft.go:596-598)
            mt = gt
        mte = max(mt, gt, 1)
        x = h = c = 0
        ents = []
        if t == A.HB_MSG_APP:
            x = max(0, last + int(rng.integers(-3, 2)))
            if rng.random() < deep:  # a probe anywhere in the log (a leader backing up after rejections)
                x = int(rng.integers(0, last + 1))
            h = term_of(g, x) if rng.random() < 0.8 else int(rng.integers(0, gt + 2))
            if x > 0 and h == 0:  # LogTerm 0 names index 0 only: a leader holds the entry it sends after
                h = int(rng.integers(1, gt + 2))
            k = int(rng.integers(0, max_ents + 1))
            et = min(max(h, 1), mte)
            for _j in range(k):
                if rng.random() < 0.3:
                    et = min(et + 1, mte)
                ents.append(et)
            c = max(0, com + int(rng.integers(-2, 6)))
            if past_end > 0 and rng.random() < past_end:  # (a draw only when asked: default streams unchanged)
                x, h, ents = last + 1 + int(rng.integers(0, 3)), 0, []
                c = last + 1 + int(rng.integers(0, 3))
        elif t == A.HB_MSG_HEARTBEAT:
            c = max(0, com + int(rng.integers(-1, 3)))
        elif t == A.HB_MSG_SNAP:
            x = max(0, com + int(rng.integers(-2, 20)))
            h = term_of(g, x) if rng.random() < 0.3 else int(rng.integers(1, mte + 1))
        else:
            x = max(0, last + int(rng.integers(-2, 3)))
            h = max(0, term_of(g, last) + int(rng.integers(-1, 2)))
        grp.append(g)
        info.append(t | (slot << 4) | (voted << 9))
        term.append(mt)
        index.append(x)
        hint.append(h)
        commit.append(c)
        eoff.append(len(eterm))
        eterm.extend(ents)
    return dict(group=np.array(grp, np.uint32), info=np.array(info, np.uint32), term=np.array(term, np.uint64),
                index=np.array(index, np.uint64), hint=np.array(hint, np.uint64), commit=np.array(commit, np.uint64),
                eoff=np.array(eoff, np.uint64), eterm=np.array(eterm or [0], np.uint64)[:len(eterm)], props=None)


# ---------------------------------------------------------------------------- follow (the mirror of cfg2)
def follow_groups(G, n=3, seed=0x5EED0006, last_hi=1 << 20, term_hi=1000, with_runs="flat"):
    """The follower side's steady state: this node (slot 0) follows every group,
    whose leader is slot 1 at the group's Term (lead = vote = 1); the log's last
    entry has the current Term and everything but it is committed.  Progress is
    what the last reset left (Probe; self Match = lastIndex)."""
    g, runs = steady_groups(G, n, seed=seed, last_hi=last_hi, term_hi=term_hi, with_runs=with_runs)
    g["state"] = A.HB_STATE_FOLLOWER
    g["lead"] = 1
    g["vote"] = 1
    g["committed"] = g["last_index"] - np.uint64(1)
    for s in range(n):
        g["pr"][:, s]["state"] = A.HB_PR_PROBE
        g["pr"][:, s]["match"] = g["last_index"] if s == 0 else 0
        g["pr"][:, s]["next"] = g["last_index"] + np.uint64(1)
    return g, runs


def follow_batch(groups, step, seed=0x5EED0006, ents=1):
    """One follow step (the mirror of cfg2): every group receives its leader's
    MsgApp (Index = LogTerm's index = the follower's last, `ents` entries at
    the Term, Commit = the leader's commit: the follower's last) and a
    MsgHeartbeat (Commit = the same), in one random permutation of the arrival
    stream.  Step k continues where step k-1 left every follower (last + k)."""
    G = len(groups)
    rng = np.random.default_rng(seed + 104729 * step)
    grp = np.concatenate([np.arange(G, dtype=np.uint32)] * 2)
    typ = np.concatenate([np.full(G, A.HB_MSG_APP, np.uint32), np.full(G, A.HB_MSG_HEARTBEAT, np.uint32)])
    perm = rng.permutation(2 * G)
    grp, typ = grp[perm], typ[perm]
    app = typ == A.HB_MSG_APP
    term = groups["term"][grp].astype(np.uint64)
    base = groups["last_index"][grp].astype(np.uint64) + np.uint64(step * ents)
    k = np.where(app, ents, 0).astype(np.uint64)
    eoff = np.concatenate([[0], np.cumsum(k)[:-1]]).astype(np.uint64)
    return dict(group=grp, info=(typ | (np.uint32(1) << np.uint32(4))).astype(np.uint32), term=term,
                index=np.where(app, base, 0).astype(np.uint64), hint=np.where(app, term, 0).astype(np.uint64),
                commit=base, eoff=eoff, eterm=np.repeat(term[app], ents).astype(np.uint64), props=None)


# ---------------------------------------------------------------------------- mixed (a node's real Ready cycle)
def mixed_groups(G, n=3, seed=0x5EED0007, lead_every=3, last_hi=1 << 20, term_hi=1000, with_runs="flat"):
    """A MultiNode node's groups (raft/multinode.go:233-237): this node (slot 0)
    leads every `lead_every`-th group (g % lead_every == 0, the cfg2 leader
    state: followers Replicate, every Match = committed = lastIndex) and
    follows the rest, whose leader is slot 1 (the follow state: the last entry
    has the Term, everything but it is committed, Progress as the last reset
    left it)."""
    g, runs = steady_groups(G, n, seed=seed, last_hi=last_hi, term_hi=term_hi, with_runs=with_runs)
    f = (np.arange(G) % lead_every) != 0
    g["state"][f] = A.HB_STATE_FOLLOWER
    g["lead"][f] = 1
    g["vote"][f] = 1
    g["committed"][f] = g["last_index"][f] - np.uint64(1)
    for s in range(n):
        pr = g["pr"][:, s]
        pr["state"][f] = A.HB_PR_PROBE
        pr["match"][f] = g["last_index"][f] if s == 0 else 0
        pr["next"][f] = g["last_index"][f] + np.uint64(1)
    return g, runs


def mixed_batch(groups, step=0, seed=0x5EED0007):
    """One Ready cycle of the mixed node, in one batch (X mode: it carries
    m.Commit): every led group takes a proposal (dense props) and its n - 1
    followers' MsgAppResp for it (the cfg2 step); every followed group takes
    its leader's MsgApp (one entry at the Term, Index = LogTerm's index = the
    follower's last, Commit = the leader's commit) and MsgHeartbeat (the follow
    step); all in one random permutation of the arrival stream.  Step k
    continues where step k-1 left every group.  Returns the batch and the
    per-step increments of index / commit (inputs stay resident in a bench)."""
    G = len(groups)
    n = int(groups["n"][0])
    rng = np.random.default_rng(seed + 7919 * step)
    led = np.nonzero(groups["state"] == A.HB_STATE_LEADER)[0].astype(np.uint32)
    fol = np.nonzero(groups["state"] == A.HB_STATE_FOLLOWER)[0].astype(np.uint32)
    nf = n - 1
    g_ack = np.repeat(led, nf)
    s_ack = np.tile(np.arange(1, n, dtype=np.uint32), len(led))
    grp = np.concatenate([g_ack, fol, fol])
    typ = np.concatenate([np.full(len(g_ack), A.HB_MSG_APP_RESP, np.uint32), np.full(len(fol), A.HB_MSG_APP, np.uint32),
                          np.full(len(fol), A.HB_MSG_HEARTBEAT, np.uint32)])
    frm = np.concatenate([s_ack, np.ones(2 * len(fol), np.uint32)])
    perm = rng.permutation(len(grp))
    grp, typ, frm = grp[perm], typ[perm], frm[perm]
    ack, app, beat = typ == A.HB_MSG_APP_RESP, typ == A.HB_MSG_APP, typ == A.HB_MSG_HEARTBEAT
    last = groups["last_index"][grp].astype(np.uint64)
    term = groups["term"][grp].astype(np.uint64)
    k = np.uint64(step)
    index = np.where(ack, last + k + np.uint64(1), np.where(app, last + k, 0)).astype(np.uint64)
    commit = np.where(ack, 0, last + k).astype(np.uint64)
    hint = np.where(app, term, 0).astype(np.uint64)
    ne = app.astype(np.uint64)
    eoff = np.concatenate([[0], np.cumsum(ne)[:-1]]).astype(np.uint64)
    props = np.zeros(G, np.uint32)
    props[led] = 1
    b = dict(group=grp.astype(np.uint32), info=(typ | (frm << np.uint32(4))).astype(np.uint32), term=term, index=index,
             hint=hint, commit=commit, eoff=eoff, eterm=term[app].copy(), props=props)
    inc = dict(index=(ack | app).astype(np.uint64), commit=(app | beat).astype(np.uint64))
    return b, inc


def many_runs_groups(G, n=3, seed=9, runs_lo=18, runs_hi=30, run_len=40):
    """Followers whose logs hold runs_lo..runs_hi term runs of 1..run_len
    entries (the follower side's raftLog.term at any depth); every group's
    Progress in its reset form.  Returns (groups, runs)."""
    rng = np.random.default_rng(seed)
    g = np.zeros(G, dtype=A.GROUP_DTYPE)
    runs = []
    for i in range(G):
        k = int(rng.integers(runs_lo, runs_hi + 1))
        lens = rng.integers(1, run_len + 1, k)
        first = int(rng.integers(1, 50))
        t = int(rng.integers(0, 3))
        rr, pos = [], first - 1
        for L in lens:
            rr.append((pos, t))
            pos += int(L)
            t += int(rng.integers(1, 4))
        last = pos - 1
        top = rr[-1][1]
        term = top + int(rng.integers(0, 3))
        runs.append(rr)
        r = g[i]
        r["term"], r["first_index"], r["last_index"] = term, first, last
        r["committed"] = int(rng.integers(first - 1, max(first - 1, last - 5) + 1))
        r["snap_index"] = first - 1
        r["term_first"], r["term_last"] = (rr[-1][0], last) if top == term else (A.HB_NO_INDEX, 0)
        r["state"], r["n"], r["self_slot"] = A.HB_STATE_FOLLOWER, n, 0
        r["lead"] = 1 if rng.random() < 0.7 else A.HB_REF_NONE
        r["vote"] = int(rng.choice([A.HB_REF_NONE, 1, 0]))
        for s in range(n):
            r["pr"][s]["match"] = last if s == 0 else 0
            r["pr"][s]["next"] = last + 1
    return g, runs


def deep_lag_leaders(G, n=3, seed=10, last_lo=6000, last_hi=9000, lag_min=5000):
    """Leaders with long logs whose followers are far behind (Probe, or
    Replicate with an empty window), Match at least lag_min entries below
    lastIndex: every sendAppend to them cuts entries(Next, maxMsgSize) deep in
    the log.  Returns (groups, runs)."""
    rng = np.random.default_rng(seed)
    g = np.zeros(G, dtype=A.GROUP_DTYPE)
    last = rng.integers(last_lo, last_hi + 1, G)
    term = rng.integers(2, 50, G)
    tf = np.maximum(last - rng.integers(0, 3000, G), 1)
    g["term"], g["first_index"], g["last_index"], g["committed"] = term, 1, last, last - rng.integers(0, 50, G)
    g["term_first"], g["term_last"], g["snap_index"] = tf, last, 0
    g["state"], g["n"], g["self_slot"], g["lead"], g["vote"] = A.HB_STATE_LEADER, n, 0, 0, 0
    runs = []
    for i in range(G):
        runs.append([(0, int(term[i]) - 1), (int(tf[i]), int(term[i]))])
        for s in range(n):
            p = g[i]["pr"][s]
            if s == 0:
                p["match"], p["next"] = last[i], last[i] + 1
                continue
            m = int(rng.integers(0, last[i] - lag_min + 1))
            p["match"], p["next"] = m, m + 1
            p["state"] = A.HB_PR_PROBE if rng.random() < 0.5 else A.HB_PR_REPLICATE
    return g, runs


def merge_batches(a, b, seed=6):
    """Interleave two batches (arrival order within each kept), re-basing b's
    entry offsets; a must carry no entries of its own."""
    rng = np.random.default_rng(seed)
    na, nb = len(a["group"]), len(b["group"])
    pick = np.zeros(na + nb, bool)
    pick[rng.choice(na + nb, nb, replace=False)] = True  # True: from b
    out = {}
    for k in ("group", "info", "term", "index"):
        v = np.empty(na + nb, a[k].dtype)
        v[~pick], v[pick] = a[k], b[k]
        out[k] = v
    for k, dt in (("hint", np.uint64), ("commit", np.uint64)):
        v = np.zeros(na + nb, dt)
        if a.get(k) is not None:
            v[~pick] = a[k]
        if b.get(k) is not None:
            v[pick] = b[k]
        out[k] = v
    # message i's entries: eoff[i] .. eoff[i+1]; a's messages carry none
    cnt_b = np.diff(np.append(b["eoff"], len(b["eterm"]))).astype(np.uint64)
    cnt = np.zeros(na + nb, np.uint64)
    cnt[pick] = cnt_b
    out["eoff"] = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.uint64)
    out["eterm"] = b["eterm"]
    out["props"] = a.get("props")
    return out


def random_timers(G, seed=1, et_hi=12, ht_hi=4, pos_hi=50):
    """Per-group timers for tick parity: ElectionTick 1..et_hi, HeartbeatTick
    1..ht_hi, elapsed anywhere in [0, 2 ElectionTick], rand positions spread."""
    rng = np.random.default_rng(seed)
    t = np.zeros(G, dtype=A.TIMER_DTYPE)
    et = rng.integers(1, et_hi + 1, G)
    t["election_tick"] = et
    t["heartbeat_tick"] = rng.integers(1, ht_hi + 1, G)
    t["elapsed"] = rng.integers(0, 2 * et + 1)
    t["rand_pos"] = rng.integers(0, pos_hi + 1, G)
    return t


# ---------------------------------------------------------------------------- cfg4
def election_groups(G, n=7, seed=0x5EED0004, term_hi=1000, with_runs=True):
    """All groups follower at term T ~ U[1, term_hi], no leader, fresh progress."""
    rng = np.random.default_rng(seed)
    g = np.zeros(G, dtype=A.GROUP_DTYPE)
    term = rng.integers(1, term_hi + 1, G, dtype=np.uint64)
    last = rng.integers(1, 1 << 16, G, dtype=np.uint64)
    g["term"], g["committed"], g["first_index"], g["last_index"] = term, last, 1, last
    g["term_first"], g["term_last"] = A.HB_NO_INDEX, 0
    g["state"], g["n"], g["self_slot"] = A.HB_STATE_FOLLOWER, n, 0
    g["lead"], g["vote"] = A.HB_REF_NONE, A.HB_REF_NONE
    for s in range(n):
        g["pr"][:, s]["match"] = last if s == 0 else 0
        g["pr"][:, s]["next"] = last + np.uint64(1)
    runs = None
    if with_runs == "flat":  # (0, 0) then (1, T-1) when T > 1
        two = term > 1
        cnt = np.where(two, 2, 1).astype(np.uint64)
        off = np.zeros(G + 1, dtype=np.uint64)
        off[1:] = np.cumsum(cnt)
        flat = np.zeros((int(off[-1]), 2), dtype=np.uint64)
        pos = off[:-1][two].astype(np.int64) + 1
        flat[pos, 0] = 1
        flat[pos, 1] = term[two] - np.uint64(1)
        runs = (flat, off)
    elif with_runs:
        runs = [[(0, 0), (1, max(int(term[i]) - 1, 0))] if term[i] > 1 else [(0, 0)] for i in range(G)]
    return g, runs


def cfg4_batch(groups, seed=0x5EED0004, grant_p=0.5, higher_p=0.05):
    """MsgHup for every group, then n-1 MsgVoteResp per group (random order):
    granted with p = grant_p; a fraction carries Term+2 (step down, lead = From)."""
    rng = np.random.default_rng(seed)
    G = len(groups)
    n = int(groups["n"][0])
    hup_g = rng.permutation(G).astype(np.uint32)
    nv = n - 1
    vg = np.repeat(np.arange(G, dtype=np.uint32), nv)
    vs = np.tile(np.arange(1, n, dtype=np.uint32), G)
    perm = rng.permutation(G * nv)
    vg, vs = vg[perm], vs[perm]
    rej = (rng.random(G * nv) >= grant_p).astype(np.uint32)
    vterm = groups["term"][vg].astype(np.uint64) + np.uint64(1)
    hi = rng.random(G * nv) < higher_p
    vterm[hi] += np.uint64(1)
    grp = np.concatenate([hup_g, vg])
    info = np.concatenate([np.full(G, A.HB_MSG_HUP, np.uint32),
                           (np.uint32(A.HB_MSG_VOTE_RESP) | (vs << np.uint32(4)) | (rej << np.uint32(8)))])
    term = np.concatenate([np.zeros(G, np.uint64), vterm])
    index = np.zeros(len(grp), np.uint64)
    return dict(group=grp, info=info.astype(np.uint32), term=term, index=index, hint=None, props=None)


def cfg4_storm_batch(groups, seed=0x5EED0004, grant_p=0.5, higher_p=0.05):
    """Repeatable cfg4 step.  Per group, in arrival order: one MsgHeartbeatResp
    from slot 1 at Term+1 (term gate: every group, whatever it became in the last
    storm, steps down to follower, raft/raft.go:474-477), MsgHup (campaign at
    Term+2), then n-1 MsgVoteResp at Term+2 in random order (granted with p =
    grant_p; a fraction at Term+3 steps the candidate down, lead = From).

    Terms are relative to groups["term"] = T.  Step k of a bench run adds 4k to
    every nonzero term (the largest term a group reaches in a step is T+3), so
    the same arrays replay as a fresh storm each step."""
    rng = np.random.default_rng(seed)
    G = len(groups)
    n = int(groups["n"][0])
    nv = n - 1
    t0 = groups["term"].astype(np.uint64)
    down_g = rng.permutation(G).astype(np.uint32)
    hup_g = rng.permutation(G).astype(np.uint32)
    vg = np.repeat(np.arange(G, dtype=np.uint32), nv)
    vs = np.tile(np.arange(1, n, dtype=np.uint32), G)
    perm = rng.permutation(G * nv)
    vg, vs = vg[perm], vs[perm]
    rej = (rng.random(G * nv) >= grant_p).astype(np.uint32)
    vterm = t0[vg] + np.uint64(2)
    vterm[rng.random(G * nv) < higher_p] += np.uint64(1)
    grp = np.concatenate([down_g, hup_g, vg])
    info = np.concatenate([np.full(G, A.HB_MSG_HEARTBEAT_RESP | (1 << 4), np.uint32),
                           np.full(G, A.HB_MSG_HUP, np.uint32),
                           (np.uint32(A.HB_MSG_VOTE_RESP) | (vs << np.uint32(4)) | (rej << np.uint32(8)))])
    term = np.concatenate([t0[down_g] + np.uint64(1), np.zeros(G, np.uint64), vterm])
    index = np.zeros(len(grp), np.uint64)
    return dict(group=grp, info=info.astype(np.uint32), term=term, index=index, hint=None, props=None)


def storm_terms(term, k):
    """cfg4_storm_batch terms for step k: +4k on every nonzero (non-local) term."""
    return np.where(term == 0, term, term + np.uint64(4 * k)).astype(np.uint64)


# ---------------------------------------------------------------------------- cfg3
class FollowerSim:
    """Closed-loop followers for the lagging-follower workload (cfg3).

    Each (group, slot) follower holds a log prefix length `flast`.  The leader's
    MsgApp events (HB_EV_APP: index = prev) are delivered with loss/lag; a
    follower accepts when it has `prev` (acks prev + entries) and rejects with
    RejectHint = flast otherwise.  Heartbeat responses and MsgUnreachable are
    sprinkled in.  All message terms are the leader's current term."""

    def __init__(self, groups, seed=0x5EED0003, lag_p=0.2, drop_p=0.1, hb_p=0.1, unreach_p=0.001):
        self.rng = np.random.default_rng(seed)
        G = len(groups)
        self.n = groups["n"].astype(np.int64)
        nmax = int(self.n.max())
        self.flast = np.zeros((G, nmax), dtype=np.int64)
        for s in range(nmax):
            self.flast[:, s] = groups["pr"][:, s]["match"].astype(np.int64)
        self.pending = []
        self.lag_p, self.drop_p, self.hb_p, self.unreach_p = lag_p, drop_p, hb_p, unreach_p

    def deliver(self, events, groups_now):
        """Consume the leader's events of one step; return the next batch."""
        rng = self.rng
        msgs = list(self.pending)
        self.pending = []
        last = groups_now["last_index"].astype(np.int64)
        term = groups_now["term"].astype(np.int64)
        selfs = groups_now["self_slot"].astype(np.int64)
        app = events[events["type"] == A.HB_EV_APP]
        for e in app:
            g, s, prev = int(e["group"]), int(e["to"]), int(e["x"])
            if rng.random() < self.drop_p:
                continue
            L = int(last[g])
            if self.flast[g, s] >= prev:
                self.flast[g, s] = max(self.flast[g, s], L)
                m = (g, A.HB_MSG_APP_RESP, s, 0, int(term[g]), L, 0)
            else:
                m = (g, A.HB_MSG_APP_RESP, s, 1, int(term[g]), prev, int(self.flast[g, s]))
            if rng.random() < self.lag_p:
                self.pending.append(m)
            else:
                msgs.append(m)
        G = len(groups_now)
        for g in np.nonzero(rng.random(G) < self.hb_p)[0]:
            for s in range(int(self.n[g])):
                if s != selfs[g]:
                    msgs.append((int(g), A.HB_MSG_HEARTBEAT_RESP, s, 0, int(term[g]), 0, 0))
        for g in np.nonzero(rng.random(G) < self.unreach_p * 10)[0]:
            s = int(rng.integers(0, self.n[g]))
            if s != selfs[g]:
                msgs.append((int(g), A.HB_MSG_UNREACHABLE, s, 0, 0, 0, 0))
        order = rng.permutation(len(msgs)) if msgs else np.zeros(0, dtype=np.int64)
        # keep per-(group) order of delayed-before-fresh by a stable sort on a random key per group
        arr = np.array(msgs, dtype=np.int64).reshape(-1, 7)[order] if msgs else np.zeros((0, 7), np.int64)
        grp = arr[:, 0].astype(np.uint32)
        info = (arr[:, 1] | (arr[:, 2] << 4) | (arr[:, 3] << 8)).astype(np.uint32)
        props = self.rng.integers(1, 5, G).astype(np.uint32)
        return dict(group=grp, info=info, term=arr[:, 4].astype(np.uint64), index=arr[:, 5].astype(np.uint64),
                    hint=arr[:, 6].astype(np.uint64), props=props)


def lagging_groups(G, n=5, seed=0x5EED0003, W=8, with_runs=True):
    """cfg3 start: leaders with followers spread over Probe/Replicate and lag."""
    g, runs = steady_groups(G, n=n, seed=seed, last_hi=1 << 12, term_hi=100, with_runs=with_runs)
    rng = np.random.default_rng(seed + 1)
    for s in range(1, n):
        lag = rng.integers(0, 64, G).astype(np.uint64)
        m = np.maximum(g["last_index"].astype(np.int64) - lag.astype(np.int64), 0).astype(np.uint64)
        g["pr"][:, s]["match"] = m
        g["pr"][:, s]["next"] = m + np.uint64(1)
        probe = rng.random(G) < 0.3
        g["pr"][:, s]["state"] = np.where(probe, A.HB_PR_PROBE, A.HB_PR_REPLICATE)
    # committed = q-th largest match (consistent leader state)
    mt = np.sort(np.stack([g["pr"][:, s]["match"] for s in range(n)], 1), axis=1)[:, ::-1]
    q = n // 2 + 1
    g["committed"] = np.minimum(mt[:, q - 1], g["committed"])
    return g, runs


def cfg3_open_batch(groups_now, rng, lag_p=0.2, stale_p=0.05, reject_p=0.05, hb_p=0.1, unreach_p=0.001,
                    max_props=4):
    """One cfg3 step generated open loop from the engine's current group state
    (SURVEY.md 8(d) cfg3): 1-4 proposed entries per group (dense props), then
    per follower one MsgAppResp -- 70 % acking the new last index, 20 % lagging
    (last - U[1, 64]), 5 % stale (<= Match), 5 % rejecting (Index = Next - 1,
    RejectHint = a follower last index >= Match) -- plus MsgHeartbeatResp from
    10 % of the followers and MsgUnreachable for 0.1 %, all in one random
    permutation at the leader's term.  Any stream is valid input (the engine
    applies the reference semantics to whatever arrives); this one keeps the
    followers in the Probe/Replicate/pause mix the workload is meant to hit."""
    G = len(groups_now)
    n = groups_now["n"].astype(np.int64)
    nmax = int(n.max())
    selfs = groups_now["self_slot"].astype(np.int64)
    term = groups_now["term"].astype(np.uint64)
    lead = groups_now["state"] == A.HB_STATE_LEADER
    props = np.where(lead, rng.integers(1, max_props + 1, G), 0).astype(np.uint32)
    last = groups_now["last_index"].astype(np.int64) + props.astype(np.int64)
    gs, ss = np.meshgrid(np.arange(G, dtype=np.int64), np.arange(nmax, dtype=np.int64), indexing="ij")
    fol = (ss < n[:, None]) & (ss != selfs[:, None]) & lead[:, None]
    g, s = gs[fol], ss[fol]
    match = groups_now["pr"]["match"][g, s].astype(np.int64)
    nxt = groups_now["pr"]["next"][g, s].astype(np.int64)
    L = last[g]
    r = rng.random(len(g))
    idx = L.copy()
    lagm = r < lag_p
    idx[lagm] = np.maximum(L[lagm] - rng.integers(1, 65, int(lagm.sum())), 0)
    stm = (r >= lag_p) & (r < lag_p + stale_p)
    idx[stm] = np.maximum(match[stm] - rng.integers(0, 4, int(stm.sum())), 0)
    rjm = (r >= lag_p + stale_p) & (r < lag_p + stale_p + reject_p)
    idx[rjm] = np.maximum(nxt[rjm] - 1, 0)
    hint = np.zeros(len(g), np.int64)
    hint[rjm] = np.minimum(match[rjm] + rng.integers(0, 8, int(rjm.sum())), L[rjm])
    info = (A.HB_MSG_APP_RESP | (s << 4) | (rjm.astype(np.int64) << 8))
    hbm = rng.random(len(g)) < hb_p
    urm = rng.random(len(g)) < unreach_p
    mg = np.concatenate([g, g[hbm], g[urm]])
    mi = np.concatenate([info, A.HB_MSG_HEARTBEAT_RESP | (s[hbm] << 4), A.HB_MSG_UNREACHABLE | (s[urm] << 4)])
    mt = np.concatenate([term[g], term[g[hbm]], np.zeros(int(urm.sum()), np.uint64)])
    mx = np.concatenate([idx, np.zeros(int(hbm.sum()) + int(urm.sum()), np.int64)])
    mh = np.concatenate([hint, np.zeros(int(hbm.sum()) + int(urm.sum()), np.int64)])
    order = rng.permutation(len(mg))
    return dict(group=mg[order].astype(np.uint32), info=mi[order].astype(np.uint32),
                term=mt[order].astype(np.uint64), index=mx[order].astype(np.uint64),
                hint=mh[order].astype(np.uint64), props=props)


# ---------------------------------------------------------------------------- wire
def _varint_len(v):
    v = np.asarray(v, dtype=np.uint64)
    n = np.ones(v.shape, dtype=np.int64)
    x = v >> np.uint64(7)
    while np.any(x):
        n += (x != 0)
        x = x >> np.uint64(7)
    return n


def encode_responses(mtype, to, frm, term, index, reject=None, hint=None):
    """Vectorized raftpb.Message encoding of response records exactly as the
    reference's generated MarshalTo writes them (raft/raftpb/raft.pb.go:
    1271-1330: every required field in field order, LogTerm / Commit 0, no
    entries, the empty non-nullable snapshot).  Returns (bytes u8, off u64,
    len u32)."""
    N = len(term)
    reject = np.zeros(N, np.uint64) if reject is None else np.asarray(reject, np.uint64)
    hint = np.zeros(N, np.uint64) if hint is None else np.asarray(hint, np.uint64)
    cols = [np.full(N, mtype, np.uint64) if np.isscalar(mtype) else np.asarray(mtype, np.uint64),
            np.asarray(to, np.uint64), np.asarray(frm, np.uint64), np.asarray(term, np.uint64),
            np.zeros(N, np.uint64), np.asarray(index, np.uint64),
            np.zeros(N, np.uint64)]  # commit
    keys = [0x08, 0x10, 0x18, 0x20, 0x28, 0x30, 0x40]
    # field 9: the empty snapshot {metadata {conf_state {}, index 0, term 0}}
    snap = np.frombuffer(bytes([0x4A, 0x08, 0x12, 0x06, 0x0A, 0x00, 0x10, 0x00, 0x18, 0x00]), np.uint8)
    rej = (reject != 0).astype(np.uint64)
    lens = [_varint_len(c) for c in cols]
    hlen = _varint_len(hint)
    rec_len = sum(1 + l for l in lens) + len(snap) + 2 + 1 + hlen
    off = np.zeros(N, np.uint64)
    if N > 1:
        off[1:] = np.cumsum(rec_len[:-1]).astype(np.uint64)
    out = np.zeros(max(int(rec_len.sum()), 1), np.uint8)
    pos = off.astype(np.int64)

    def put_varint(pos, c, l, k):
        out[pos] = k
        pos = pos + 1
        v = c.copy()
        for b in range(int(l.max()) if N else 0):
            live = b < l
            byte = (v & np.uint64(0x7F)).astype(np.uint8) | np.where(b + 1 < l, 0x80, 0).astype(np.uint8)
            out[pos[live] + b] = byte[live]
            v = v >> np.uint64(7)
        return pos + l

    for c, l, k in zip(cols[:6], lens[:6], keys[:6]):
        pos = put_varint(pos, c, l, k)
    pos = put_varint(pos, cols[6], lens[6], keys[6])  # commit (field 8), after the absent entries
    for j, b in enumerate(snap):
        out[pos + j] = b
    pos = pos + len(snap)
    out[pos] = 0x50
    out[pos + 1] = rej.astype(np.uint8)
    pos = pos + 2
    pos = put_varint(pos, hint, hlen, 0x58)
    return out, off, rec_len.astype(np.uint32)
