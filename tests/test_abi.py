"""CPU tests of the C ABI boundary (no GPU calls).

- every #define in include/hipbatch.h equals its mirror in etcd_amd/abi.py;
- record layouts (sizeof/offsetof compiled with gcc) equal the ctypes/numpy ones;
- libhipbatch.so loads and exports every function the header declares;
- the oracle library exports what its header declares.
"""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

from etcd_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "hipbatch.h")


def _header():
    return open(HDR).read()


def test_defines_match_abi_py():
    txt = _header()
    defs = dict(re.findall(r"^#define\s+(HB_[A-Z0-9_]+)\s+(-?(?:0x[0-9A-Fa-f]+|\d+)u?)\b", txt, re.M))
    assert len(defs) > 60
    for name, val in defs.items():
        v = int(val.rstrip("u"), 0)
        assert hasattr(abi, name), f"abi.py lacks {name}"
        assert getattr(abi, name) == v, f"{name}: header {v} abi.py {getattr(abi, name)}"
    assert abi.HB_NO_LIMIT == 2 ** 64 - 1 and "UINT64_MAX" in txt


def _compile_layout():
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "hipbatch.h"
#define P(T, F) printf(#T "." #F " %zu\n", offsetof(T, F));
int main(void) {
  printf("hb_progress %zu\nhb_group %zu\nhb_event %zu\nhb_batch %zu\nhb_timer %zu\n", sizeof(hb_progress),
         sizeof(hb_group), sizeof(hb_event), sizeof(hb_batch), sizeof(hb_timer));
  P(hb_group, term) P(hb_group, snap_index) P(hb_group, state) P(hb_group, fault) P(hb_group, commit_zero) P(hb_group, pr)
  P(hb_progress, pending_snapshot) P(hb_progress, ins_count)
  P(hb_event, x) P(hb_event, group) P(hb_event, type) P(hb_event, to) P(hb_event, aux)
  P(hb_batch, n) P(hb_batch, props)
  P(hb_timer, elapsed) P(hb_timer, rand_pos) P(hb_timer, election_tick) P(hb_timer, heartbeat_tick)
  return 0;
}
'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "l.c")
        exe = os.path.join(d, "l")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-std=c11", "-I", os.path.dirname(HDR), c, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    return dict(line.split() for line in out.strip().splitlines())


def test_record_layouts_match():
    lay = {k: int(v) for k, v in _compile_layout().items()}
    assert lay["hb_progress"] == C.sizeof(abi.hb_progress) == abi.PROGRESS_DTYPE.itemsize
    assert lay["hb_group"] == C.sizeof(abi.hb_group) == abi.GROUP_DTYPE.itemsize
    assert lay["hb_event"] == C.sizeof(abi.hb_event) == abi.EVENT_DTYPE.itemsize == 16
    assert lay["hb_batch"] == C.sizeof(abi.hb_batch)
    assert lay["hb_timer"] == C.sizeof(abi.hb_timer) == abi.TIMER_DTYPE.itemsize
    for key, v in lay.items():
        if "." not in key:
            continue
        t, f = key.split(".")
        assert getattr(getattr(abi, t), f).offset == v, key
        dt = {"hb_group": abi.GROUP_DTYPE, "hb_progress": abi.PROGRESS_DTYPE, "hb_event": abi.EVENT_DTYPE,
              "hb_timer": abi.TIMER_DTYPE}.get(t)
        if dt is not None:
            assert dt.fields[f][1] == v, key


def _declared_functions():
    txt = _header()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(hb_[a-z_]+)\s*\(", txt, re.M)))


def test_library_exports_every_declared_function():
    from etcd_amd import hipbatch
    L = hipbatch.lib()  # loads without touching the GPU
    names = _declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), f"libhipbatch.so does not export {n}"
    assert L.hb_abi_version() == abi.HB_ABI_VERSION
    assert L.hb_strerror(abi.HB_EINVAL) == b"invalid argument"


def test_library_rejects_bad_arguments_without_device_work():
    from etcd_amd import hipbatch
    L = hipbatch.lib()
    h = C.c_void_p()
    # argument validation happens before any device call
    assert L.hb_create(0, 0, 3, 256, abi.HB_NO_LIMIT, 10, C.byref(h)) == abi.HB_EINVAL
    assert L.hb_create(0, 10, 8, 256, abi.HB_NO_LIMIT, 10, C.byref(h)) == abi.HB_EINVAL
    assert L.hb_create(0, 10, 3, 2048, abi.HB_NO_LIMIT, 10, C.byref(h)) == abi.HB_EINVAL
    assert L.hb_step(None, None, 0) == abi.HB_EINVAL
    assert L.hb_load_entry_sizes(None, 0, None, None, None) == abi.HB_EINVAL


def test_oracle_exports():
    from oracle import pyoracle
    L = pyoracle.lib()
    txt = open(os.path.join(ROOT, "oracle", "raft_oracle.h")).read()
    names = set(re.findall(r"\b(orc_[a-z_]+)\s*\(", txt))
    for n in names:
        assert hasattr(L, n), n


def test_oracle_has_no_product_dependents():
    """The product package never loads or calls the oracle (it is the checker only)."""
    pkg = os.path.join(ROOT, "etcd_amd")
    pat = re.compile(r"^\s*(import|from)\s+oracle|pyoracle|liboracle|\borc_[a-z]", re.M)
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp", ".c")):
                txt = open(os.path.join(dirpath, f)).read()
                assert not pat.search(txt), f"{f} references the oracle"


# ---- the MultiNode host library (include/hbnode.h) ------------------------------
NODE_HDR = os.path.join(ROOT, "include", "hbnode.h")


def test_hbnode_exports_every_declared_function():
    from etcd_amd import multinode
    L = multinode.lib()  # loads (and pulls in libhipbatch.so) without touching the GPU
    txt = open(NODE_HDR).read()
    names = sorted(set(re.findall(r"^\s*(?:int|const char\*|uint64_t|hb_handle\*)\s+(hbn_[a-z_]+)\s*\(", txt, re.M)))
    assert len(names) >= 30
    for n in names:
        assert hasattr(L, n), f"libhbnode.so does not export {n}"
    py = set(re.findall(r'"(hbn_[a-z_]+)"', open(os.path.join(ROOT, "etcd_amd", "multinode.py")).read()))
    assert set(names) <= py, f"multinode.py lacks bindings for {sorted(set(names) - py)}"


def test_hbnode_defines_and_layouts_match():
    from etcd_amd import multinode as M
    txt = open(NODE_HDR).read()
    defs = dict(re.findall(r"^#define\s+(HBN_[A-Z0-9_]+)\s+(-?\d+)\b", txt, re.M))
    for name, val in defs.items():
        if hasattr(M, name):
            assert getattr(M, name) == int(val), name
    src = r'''
#include <stdio.h>
#include "hbnode.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(hbn_entry), sizeof(hbn_hard_state), sizeof(hbn_snapshot),
         sizeof(hbn_message), sizeof(hbn_group_ready), sizeof(hbn_group_status), sizeof(hbn_config));
  return 0;
}
'''
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-std=c11", "-I", os.path.dirname(NODE_HDR), c, "-o", exe], check=True)
        sizes = [int(x) for x in subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()]
    assert sizes == [C.sizeof(t) for t in (M.hbn_entry, M.hbn_hard_state, M.hbn_snapshot, M.hbn_message,
                                           M.hbn_group_ready, M.hbn_group_status, M.hbn_config)]


def test_hbnode_rejects_bad_arguments_without_device_work():
    from etcd_amd import multinode as M
    L = M.lib()
    p = C.c_void_p()
    assert L.hbn_start(0, 0, 16, 3, 256, abi.HB_NO_LIMIT, 16, C.byref(p)) == abi.HB_EINVAL  # id 0 = None
    assert L.hbn_start(0, 1, 0, 3, 256, abi.HB_NO_LIMIT, 16, C.byref(p)) == abi.HB_EINVAL
    assert L.hbn_ready(None, None, None) == abi.HB_EINVAL
