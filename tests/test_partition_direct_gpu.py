"""Partitions with direct tile offsets (HB_RDX_DIRECT, r06): the
histogram kernel's workgroup and superblock digit sums stand in for the
k_scan_rows launch, and the scatter sums them before each tile.  These steps
pin what the full-size headline tests do not reach: batch sizes that change
from step to step (the superblock buffers rotate over three steps and each is
cleared only as far as an earlier step dirtied it), ragged last tiles and hist
workgroups, and batches past 8M messages, where a scatter workgroup's offset
sums take a second round of loads; and, beside them, a two-pass partition
(1.1M groups, 5-bit digits), which keeps the scan launch, over the same
kind of changing batches.  Every event, statistic and group record
against the C oracle.  Reference: the per-group arrival order the partition
keeps, raft/multinode.go:233-237.
"""
import numpy as np
import pytest

from etcd_amd import abi, synth

from .parity_util import Pair

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_direct_offsets_changing_batch_sizes():
    """300K groups x 3 (one pass, 74 buckets): 3, 1, 2, 3, 1, 3 superblocks in turn,
    with ragged tiles and a step of messages beyond capacity."""
    G, n = 300_000, 3
    g, runs = synth.steady_groups(G, n, seed=0x5EED0011, with_runs="flat")
    pair = Pair(g, runs, n, 256, max_batch=1 << 21)  # (one oracle: ids past capacity)
    for k, nmsg in enumerate([600_000, 20_001, 270_001, 600_000, 40_000, 599_999]):
        b = synth.random_batch(g, nmsg, seed=500 + k)
        if k == 4:  # some messages of groups beyond capacity: dropped in the partition
            b["group"] = b["group"].copy()
            b["group"][::29] = G + 77
        _, st, _ = pair.step(b, ctx=f"step {k} ({nmsg} messages)", check_inflights=False)
        assert st[abi.HB_STAT_MSGS] > 0


@pytest.mark.timeout(900)
def test_direct_offsets_past_eight_million_messages():
    """1,048,576 groups x 3 (256 buckets) and 9M messages: 4,395 tiles, 35
    superblocks, so the last scatter workgroups sum more offsets than one round
    of loads holds."""
    G, n = 1 << 20, 3
    g, runs = synth.steady_groups(G, n, seed=0x5EED0012, with_runs="flat")
    pair = Pair(g, runs, n, 256, max_batch=9_000_000, oracle_shards=16)
    for k in range(2):
        b = synth.random_batch(g, 9_000_000 - k, seed=700 + k)
        pair.step(b, ctx=f"9M step {k}", check_inflights=False)


@pytest.mark.timeout(900)
def test_two_pass_partition_changing_batch_sizes():
    """1.1M groups x 3: two passes (5 + 5 bits, k_scan_rows per pass: direct
    offsets measured slower there); batch sizes change and
    one step carries ids past capacity (dropped in the first pass)."""
    G, n = 1_100_000, 3
    g, runs = synth.steady_groups(G, n, seed=0x5EED0013, with_runs="flat")
    pair = Pair(g, runs, n, 256, max_batch=1 << 22)
    for k, nmsg in enumerate([3_000_000, 50_001, 1_500_001]):
        b = synth.random_batch(g, nmsg, seed=900 + k)
        if k == 1:
            b["group"] = b["group"].copy()
            b["group"][::31] = G + 5
        pair.step(b, ctx=f"two-pass step {k} ({nmsg} messages)", check_inflights=False)
