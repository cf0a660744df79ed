"""etcd_amd — MI355X-native batched Raft leader-bookkeeping engine.

The hot path behind raft.MultiNode (holandes22/etcd raft/multinode.go) —
MsgAppResp progress updates, inflight flow control, quorum commit and vote
tallying — runs as hand-written CDNA4 HIP kernels over HBM-resident
structure-of-arrays group state, behind the C ABI in include/hipbatch.h.
"""
__version__ = "0.1.0"
