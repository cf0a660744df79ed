"""Parity oracle package — TEST INFRASTRUCTURE ONLY (see raft_oracle.h)."""
