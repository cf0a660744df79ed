"""Diagnostic: the restarted-follower cluster scenario, with per-group status dumps."""
import sys
sys.path.insert(0, ".")
from tests.test_follower_gpu import Cluster, APP
from etcd_amd import abi

G = 12
c = Cluster(G, seed=21, election=8)
for g in range(1, G + 1):
    c.nodes[c.ids[g % 3]].Campaign(g)
log = []
orig_deliver = c.deliver
def deliver(drop=0.0):
    for g, m in c.inbox:
        if g == 11 and m.Type in (abi.HB_MSG_PROP, abi.HB_MSG_VOTE, abi.HB_MSG_VOTE_RESP, abi.HB_MSG_SNAP):
            log.append((r, m.Type, m.From, m.To, m.Term, m.Index, len(m.Entries), m.To in c.down))
    orig_deliver(drop)
c.deliver = deliver
def st(g):
    out = []
    for i in c.ids:
        if i in c.down:
            out.append((i, "down"))
            continue
        s = c.nodes[i].Status(g)
        out.append((i, s.SoftState.RaftState, s.SoftState.Lead, s.HardState.Term, s.HardState.Commit,
                    c.st[i, g].LastIndex(), c.st[i, g].FirstIndex()))
    return out
for r in range(60):
    if r in (8, 26):
        c.stop_node(3)
    if r in (17, 35):
        c.restart_node(3)
    c.ready_round()
    c.deliver()
    c.propose(2 * G, f"{'late' if r >= 48 else 'r'}{r}", pad=200)
    c.tick()
    if r == 30:
        c.compact(keep=20)
    if r in (7, 9, 16, 18, 25, 27, 34, 36, 40, 47, 50, 59):
        print("r", r, "g11", st(11), flush=True)
for _ in range(25):
    r += 1
    c.ready_round()
    c.deliver()
    c.tick()
print("end g11", st(11))
for x in log[-60:]:
    print(x)
