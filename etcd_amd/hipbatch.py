"""Python binding of the engine's C ABI (include/hipbatch.h -> libhipbatch.so).

This is the product path: every call goes to the HIP library.  There is no CPU
fallback — if the library is missing or the device is unusable, construction
fails loudly.
"""
import ctypes as C
import os

import numpy as np

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HB_LIB", os.path.join(_HERE, "libhipbatch.so"))
_lib = None


class HipBatchError(RuntimeError):
    def __init__(self, fn, code):
        self.code = code
        super().__init__(f"{fn} failed: {code} ({_strerror(code)})")


def _strerror(code):
    try:
        return lib().hb_strerror(code).decode()
    except Exception:
        return "?"


class HipRuntimeConflict(RuntimeError):
    """Two HIP runtimes (libamdhip64) are or would be mapped in this process:
    the engine's handle would live in one and the caller's streams and tensors
    in the other (hb_create then fails with HB_EDEVICE)."""


def _mapped_hip_runtimes():
    """The distinct libamdhip64 files mapped into this process (real paths)."""
    out = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1]
                if "libamdhip64" in os.path.basename(p):
                    out.add(os.path.realpath(p))
    except OSError:
        pass
    return out


def _bind_one_hip_runtime():
    """Make the engine bind to the HIP runtime torch uses, whatever the import order.

    libhipbatch.so needs `libamdhip64.so.7` (RUNPATH /opt/rocm).  PyTorch-ROCm
    ships its own copy, which its libraries load as `libamdhip64.so` from their
    own directory.  Loaded after torch, the engine binds to torch's copy by
    soname; loaded first, it would map /opt/rocm's and torch would later map a
    second runtime beside it (r05: `hb_create failed: -3` in a process that
    imported the router before torch).  So when no runtime is mapped yet and
    torch's copy exists, that file is preloaded (RTLD_GLOBAL): the engine binds
    to it by soname and torch's later load finds the same file already mapped.
    A process that already holds two runtimes cannot be fixed here: a named
    error instead of HB_EDEVICE at the first call."""
    have = _mapped_hip_runtimes()
    if len(have) > 1:
        raise HipRuntimeConflict(f"two HIP runtimes already mapped: {sorted(have)}")
    if have:
        return
    try:
        import importlib.util
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    for d in (spec.submodule_search_locations or []) if spec else []:
        p = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(p):
            C.CDLL(p, mode=C.RTLD_GLOBAL)
            return


def lib():
    """Load libhipbatch.so (built by `make -C etcd_amd/csrc`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C etcd_amd/csrc` "
                          "(there is no CPU fallback)")
    _bind_one_hip_runtime()
    L = C.CDLL(LIB_PATH)
    have = _mapped_hip_runtimes()
    if len(have) > 1:
        raise HipRuntimeConflict(f"loading {LIB_PATH} mapped a second HIP runtime: {sorted(have)}")
    P = C.POINTER
    H = C.c_void_p
    sig = {
        "hb_abi_version": (C.c_int, []),
        "hb_strerror": (C.c_char_p, [C.c_int]),
        "hb_create": (C.c_int, [C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint64, P(H)]),
        "hb_destroy": (C.c_int, [H]),
        "hb_set_stream": (C.c_int, [H, C.c_void_p]),
        "hb_set_input_stream": (C.c_int, [H, C.c_void_p]),
        "hb_sync": (C.c_int, [H]),
        "hb_load_groups": (C.c_int, [H, C.c_uint32, C.c_uint32, C.c_void_p]),
        "hb_get_groups": (C.c_int, [H, C.c_uint32, C.c_uint32, C.c_void_p]),
        "hb_remove_groups": (C.c_int, [H, C.c_uint32, C.c_uint32]),
        "hb_set_inflights": (C.c_int, [H, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]),
        "hb_set_log_bounds": (C.c_int, [H, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]),
        "hb_load_entry_sizes": (C.c_int, [H, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]),
        "hb_load_term_runs": (C.c_int, [H, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]),
        "hb_reserve_log": (C.c_int, [H, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]),
        "hb_log_capacity": (C.c_int, [H, C.c_uint32, P(C.c_uint64), P(C.c_uint64)]),
        "hb_get_inflights": (C.c_int, [H, C.c_uint32, C.c_uint32, P(C.c_uint32), P(C.c_uint32), C.c_void_p]),
        "hb_step": (C.c_int, [H, P(abi.hb_batch), C.c_uint32]),
        "hb_load_timers": (C.c_int, [H, C.c_uint32, C.c_uint32, C.c_void_p]),
        "hb_get_timers": (C.c_int, [H, C.c_uint32, C.c_uint32, C.c_void_p]),
        "hb_set_rand": (C.c_int, [H, C.c_uint64, C.c_uint64, C.c_void_p]),
        "hb_tick": (C.c_int, [H, C.c_uint32]),
        "hb_load_peers": (C.c_int, [H, C.c_uint32, C.c_uint32, C.c_void_p]),
        "hb_decode": (C.c_int, [H, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, P(abi.hb_batch),
                                C.c_void_p]),
        "hb_events_device": (C.c_int, [H, P(C.c_void_p), P(C.c_void_p), P(C.c_void_p), P(C.c_uint32)]),
        "hb_copy_events": (C.c_int, [H, C.c_void_p, C.c_uint64, P(C.c_uint64)]),
        "hb_events_to_host": (C.c_int, [H, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]),
        "hb_event_words_chunks": (C.c_int, [H, P(C.c_uint32), P(C.c_uint32)]),
        "hb_expand_event_words": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64,
                                            P(C.c_uint64)]),
        "hb_stats_device": (C.c_int, [H, P(C.c_void_p)]),
        "hb_stats": (C.c_int, [H, C.c_void_p]),
        "hb_phase_ms": (C.c_int, [H, C.c_void_p, P(C.c_uint32)]),
        "hb_phase_reset": (C.c_int, [H]),
        "hb_step_kernels": (C.c_int, [H, P(C.c_uint32)]),
        "hb_stats_to": (C.c_int, [H, C.c_void_p]),
        "hb_set_stats_accum": (C.c_int, [H, C.c_void_p]),
        "hb_alloc_pinned": (C.c_int, [C.c_size_t, P(C.c_void_p)]),
        "hb_free_pinned": (C.c_int, [C.c_void_p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.hb_abi_version() != abi.HB_ABI_VERSION:
        raise ImportError("libhipbatch ABI version mismatch")
    _lib = L
    return L


def _check(fn, rc):
    if rc != abi.HB_OK:
        raise HipBatchError(fn, rc)


def _ptr(a):
    """Address of a numpy array or a torch tensor (host or device)."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return a.ctypes.data


class Engine:
    """One device-resident shard of raft groups (one hb_handle)."""

    def __init__(self, capacity, max_replicas=3, max_inflight=256, max_msg_size=abi.HB_NO_LIMIT,
                 max_batch=1 << 20, device=0, stream=None):
        L = lib()
        h = C.c_void_p()
        _check("hb_create", L.hb_create(device, capacity, max_replicas, max_inflight, max_msg_size,
                                        max_batch, C.byref(h)))
        self.h = h
        self.capacity = capacity
        self.max_inflight = max_inflight
        self.max_batch = max_batch
        self.device = device
        if stream is not None:
            self.set_stream(stream)

    def close(self):
        if getattr(self, "h", None):
            lib().hb_destroy(self.h)
            self.h = None
        for p, _ in getattr(self, "_pins", {}).values():
            lib().hb_free_pinned(p)
        self._pins = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream):
        """stream: a torch.cuda.Stream, a raw hipStream_t int, or None."""
        raw = getattr(stream, "cuda_stream", stream)
        _check("hb_set_stream", lib().hb_set_stream(self.h, C.c_void_p(raw or 0)))

    def set_input_stream(self, stream):
        """The stream that produces batch arrays (torch.cuda.Stream / raw hipStream_t / None
        for the null stream): the prep stage of a step waits only for it, so it can overlap
        the previous step's apply."""
        raw = getattr(stream, "cuda_stream", stream)
        _check("hb_set_input_stream", lib().hb_set_input_stream(self.h, C.c_void_p(raw or 0)))

    def sync(self):
        _check("hb_sync", lib().hb_sync(self.h))

    # ---- group state ---------------------------------------------------------
    def load_groups(self, groups, first=0):
        g = np.ascontiguousarray(groups, dtype=abi.GROUP_DTYPE)
        _check("hb_load_groups", lib().hb_load_groups(self.h, first, len(g), g.ctypes.data))

    def get_groups(self, first=0, count=None):
        count = self.capacity - first if count is None else count
        out = np.zeros(count, dtype=abi.GROUP_DTYPE)
        _check("hb_get_groups", lib().hb_get_groups(self.h, first, count, out.ctypes.data))
        return out

    def remove_groups(self, first, count):
        _check("hb_remove_groups", lib().hb_remove_groups(self.h, first, count))

    def set_inflights(self, group, slot, start, vals):
        v = np.ascontiguousarray(vals, dtype=np.uint64)
        _check("hb_set_inflights", lib().hb_set_inflights(self.h, group, slot, start, len(v),
                                                          v.ctypes.data if len(v) else None))

    def set_log_bounds(self, groups, first_index, snap_index):
        """Refresh firstIndex / snapshot index of the given group slots after
        the application compacted or snapshotted their storage."""
        g = np.ascontiguousarray(groups, dtype=np.uint32)
        f = np.ascontiguousarray(first_index, dtype=np.uint64)
        s = np.ascontiguousarray(snap_index, dtype=np.uint64)
        assert len(g) == len(f) == len(s)
        _check("hb_set_log_bounds", lib().hb_set_log_bounds(self.h, len(g), g.ctypes.data, f.ctypes.data,
                                                            s.ctypes.data))

    def load_entry_sizes(self, sizes):
        """Finite max_msg_size: {group slot: Entry.Size() of its last n entries, oldest first}
        (normally the whole log from firstIndex; the ring grows to hold them)."""
        gs = np.ascontiguousarray(sorted(sizes), dtype=np.uint32)
        ns = np.ascontiguousarray([len(sizes[int(g)]) for g in gs], dtype=np.uint32)
        flat = np.ascontiguousarray(np.concatenate([np.asarray(sizes[int(g)], dtype=np.uint32) for g in gs])
                                    if len(gs) else np.zeros(1, np.uint32), dtype=np.uint32)
        _check("hb_load_entry_sizes", lib().hb_load_entry_sizes(self.h, len(gs), gs.ctypes.data, ns.ctypes.data,
                                                                flat.ctypes.data))

    def load_term_runs(self, runs):
        """Follower side: {group slot: [(start index, term), ...] older term runs, oldest first}
        (normally every run down to firstIndex - 1; the ring grows to hold them)."""
        gs = np.ascontiguousarray(sorted(runs), dtype=np.uint32)
        ns = np.ascontiguousarray([len(runs[int(g)]) for g in gs], dtype=np.uint32)
        flat = np.ascontiguousarray([x for g in gs for r in runs[int(g)] for x in r] or [0], dtype=np.uint64)
        _check("hb_load_term_runs", lib().hb_load_term_runs(self.h, len(gs), gs.ctypes.data, ns.ctypes.data,
                                                            flat.ctypes.data))

    def reserve_log(self, groups, size_cap=None, run_cap=None):
        """Grow the log-index rings of the given group slots to hold at least
        size_cap entry sizes / run_cap term runs (hb_reserve_log; None = unchanged)."""
        g = np.ascontiguousarray(groups, dtype=np.uint32)
        if not len(g):
            return
        sc = None if size_cap is None else np.ascontiguousarray(np.broadcast_to(size_cap, g.shape), dtype=np.uint64)
        rc = None if run_cap is None else np.ascontiguousarray(np.broadcast_to(run_cap, g.shape), dtype=np.uint64)
        _check("hb_reserve_log", lib().hb_reserve_log(self.h, len(g), g.ctypes.data,
                                                      None if sc is None else sc.ctypes.data,
                                                      None if rc is None else rc.ctypes.data))

    def log_capacity(self, group):
        """(size ring capacity, term-run ring capacity) of one group slot."""
        a, b = C.c_uint64(), C.c_uint64()
        _check("hb_log_capacity", lib().hb_log_capacity(self.h, group, C.byref(a), C.byref(b)))
        return a.value, b.value

    def get_inflights(self, group, slot):
        out = np.zeros(self.max_inflight, dtype=np.uint64)
        s, c = C.c_uint32(), C.c_uint32()
        _check("hb_get_inflights", lib().hb_get_inflights(self.h, group, slot, C.byref(s), C.byref(c),
                                                          out.ctypes.data))
        return s.value, out[: c.value].copy()

    # ---- hot path --------------------------------------------------------------
    def step(self, group, info, term, index, hint=None, props=None, host=None, profile=False, edesc=None,
             eoff=None, peoff=None, commit=None, eterm=None, msg_props=False):
        """Step one batch.  Arrays are numpy (host) or torch tensors (host or cuda).
        profile: False, True (every phase) or "apply" (only HB_PHASE_APPLY).
        edesc / eoff / peoff: entry descriptors (finite max_msg_size, include/hipbatch.h).
        msg_props: the batch carries MsgProp messages (HB_STEP_MSG_PROPS)."""
        b = abi.hb_batch()
        b.n = len(group)
        b.group, b.info, b.term, b.index = _ptr(group), _ptr(info), _ptr(term), _ptr(index)
        b.hint, b.props = _ptr(hint), _ptr(props)
        b.n_edesc = len(edesc) if edesc is not None else (len(eterm) if eterm is not None else 0)
        b.edesc, b.eoff, b.peoff = _ptr(edesc), _ptr(eoff), _ptr(peoff)
        b.commit, b.eterm = _ptr(commit), _ptr(eterm)
        if host is None:
            host = not (hasattr(group, "is_cuda") and group.is_cuda)
        prof = {True: abi.HB_STEP_PROFILE, "apply": abi.HB_STEP_PROFILE_APPLY}.get(profile, 0)
        flags = (abi.HB_STEP_HOST_PTRS if host else 0) | prof | (abi.HB_STEP_MSG_PROPS if msg_props else 0)
        self._keep = (group, info, term, index, hint, props, edesc, eoff, peoff, commit, eterm)
        _check("hb_step", lib().hb_step(self.h, C.byref(b), flags))

    # ---- timers (MultiNode.Tick) ----------------------------------------------
    def load_timers(self, timers, first=0):
        t = np.ascontiguousarray(timers, dtype=abi.TIMER_DTYPE)
        _check("hb_load_timers", lib().hb_load_timers(self.h, first, len(t), t.ctypes.data))

    def get_timers(self, first=0, count=None):
        count = self.capacity - first if count is None else count
        out = np.zeros(count, dtype=abi.TIMER_DTYPE)
        _check("hb_get_timers", lib().hb_get_timers(self.h, first, count, out.ctypes.data))
        return out

    def set_rand(self, draws, first=0):
        """The node's r.rand.Int() stream (rand.New(rand.NewSource(id)))."""
        d = np.ascontiguousarray(draws, dtype=np.uint64)
        _check("hb_set_rand", lib().hb_set_rand(self.h, first, len(d), d.ctypes.data if len(d) else None))

    def tick(self):
        """One MultiNode.Tick over every group (asynchronous; events/stats as step)."""
        _check("hb_tick", lib().hb_tick(self.h, 0))

    # ---- wire ingestion ----------------------------------------------------------
    def load_peers(self, ids, first=0):
        """ids: [count, HB_MAX_REPLICAS] node ids per slot (0 = none)."""
        a = np.ascontiguousarray(ids, dtype=np.uint64).reshape(-1, abi.HB_MAX_REPLICAS)
        _check("hb_load_peers", lib().hb_load_peers(self.h, first, len(a), a.ctypes.data))

    def decode(self, data, off, length, group, out, status):
        """Decode raftpb.Message records (device tensors) into the batch arrays
        out = {group, info, term, index, hint} (device tensors) + status (u8)."""
        b = abi.hb_batch()
        b.n = len(off)
        b.group, b.info, b.term, b.index = _ptr(out["group"]), _ptr(out["info"]), _ptr(out["term"]), _ptr(out["index"])
        b.hint, b.props = _ptr(out["hint"]), None
        self._keep_dec = (data, off, length, group, out, status)
        _check("hb_decode", lib().hb_decode(self.h, _ptr(data), _ptr(off), _ptr(length), _ptr(group), len(off),
                                            C.byref(b), _ptr(status)))

    def step_batch(self, batch, **kw):
        return self.step(batch["group"], batch["info"], batch["term"], batch["index"],
                         batch.get("hint"), batch.get("props"), edesc=batch.get("edesc"), eoff=batch.get("eoff"),
                         peoff=batch.get("peoff"), commit=batch.get("commit"), eterm=batch.get("eterm"),
                         msg_props=bool(batch.get("msg_props", False)), **kw)

    def events(self):
        """Dense events of the last step (host copy, synchronizes)."""
        n = C.c_uint64()
        L = lib()
        rc = L.hb_copy_events(self.h, None, 0, C.byref(n))
        if rc not in (abi.HB_OK, abi.HB_EINVAL):
            _check("hb_copy_events", rc)
        out = np.zeros(max(n.value, 1), dtype=abi.EVENT_DTYPE)
        _check("hb_copy_events", L.hb_copy_events(self.h, out.ctypes.data, len(out), C.byref(n)))
        return out[: n.value]

    def events_into(self, host_ptr, cap):
        """Dense events of the last step into caller memory (e.g. pinned) of
        `cap` hb_event records; returns the count (synchronizes)."""
        n = C.c_uint64()
        _check("hb_copy_events", lib().hb_copy_events(self.h, C.c_void_p(host_ptr), cap, C.byref(n)))
        return n.value

    def n_chunks(self):
        n, per = C.c_uint32(), C.c_uint32()
        _check("hb_event_words_chunks", lib().hb_event_words_chunks(self.h, C.byref(n), C.byref(per)))
        return n.value, per.value

    def events_to_host(self, words_ptr, cap, counts_ptr, total_ptr):
        """Asynchronous compact delta (hb_events_to_host) into pinned buffers
        (hb_alloc_pinned / torch pin_memory): read them after sync()."""
        _check("hb_events_to_host", lib().hb_events_to_host(self.h, C.c_void_p(words_ptr), cap,
                                                            C.c_void_p(counts_ptr), C.c_void_p(total_ptr)))

    def event_words(self):
        """The last step's compact event words and per-chunk counts (host copies;
        synchronizes), via hb_events_to_host into pinned buffers."""
        nc, _ = self.n_chunks()
        L = lib()
        pins = getattr(self, "_pins", None)
        if pins is None:
            pins = self._pins = {}

        def pinned(name, nbytes):
            p, cap = pins.get(name, (None, 0))
            if cap < nbytes:
                if p:
                    L.hb_free_pinned(p)
                q = C.c_void_p()
                _check("hb_alloc_pinned", L.hb_alloc_pinned(max(nbytes, 64), C.byref(q)))
                pins[name] = (q.value, max(nbytes, 64))
            return pins[name][0]
        cnt = pinned("counts", 4 * nc)
        tot = pinned("total", 8)
        cap = pins.get("words", (None, 0))[1] // 8
        for _ in range(2):
            w = pinned("words", 8 * max(cap, 1))
            self.events_to_host(w, cap, cnt, tot)
            self.sync()
            total = C.c_uint64.from_address(tot).value
            if total <= cap:
                break
            cap = total
        words = np.ctypeslib.as_array((C.c_uint64 * max(total, 1)).from_address(w))[:total].copy()
        counts = np.ctypeslib.as_array((C.c_uint32 * nc).from_address(cnt)).copy()
        return words, counts

    @staticmethod
    def expand_words(words, counts):
        """hb_expand_event_words: compact words -> hb_event records (CPU)."""
        L = lib()
        w = np.ascontiguousarray(words, dtype=np.uint64)
        c = np.ascontiguousarray(counts, dtype=np.uint32)
        n = C.c_uint64()
        _check("hb_expand_event_words", L.hb_expand_event_words(w.ctypes.data, len(w), c.ctypes.data, len(c), None,
                                                                0, C.byref(n)))
        out = np.zeros(max(n.value, 1), dtype=abi.EVENT_DTYPE)
        _check("hb_expand_event_words", L.hb_expand_event_words(w.ctypes.data, len(w), c.ctypes.data, len(c),
                                                                out.ctypes.data, len(out), C.byref(n)))
        return out[: n.value]

    def stats(self):
        out = np.zeros(abi.HB_STAT_COUNT, dtype=np.uint64)
        _check("hb_stats", lib().hb_stats(self.h, out.ctypes.data))
        return out

    def stats_device_ptr(self):
        p = C.c_void_p()
        _check("hb_stats_device", lib().hb_stats_device(self.h, C.byref(p)))
        return p.value

    def stats_to(self, dev_ptr):
        """Async D2D copy of the last step's stats to a device buffer (torch tensor or int)."""
        _check("hb_stats_to", lib().hb_stats_to(self.h, C.c_void_p(_ptr(dev_ptr) if not isinstance(dev_ptr, int)
                                                                   else dev_ptr)))

    def set_stats_accum(self, dev_ptr):
        """Accumulate every later step's statistics into a device buffer of
        HB_STAT_COUNT u64 (torch tensor or raw pointer) inside the finish
        phase; None turns it off."""
        p = None if dev_ptr is None else (dev_ptr if isinstance(dev_ptr, int) else _ptr(dev_ptr))
        _check("hb_set_stats_accum", lib().hb_set_stats_accum(self.h, C.c_void_p(p)))

    def phase_reset(self):
        _check("hb_phase_reset", lib().hb_phase_reset(self.h))

    def step_kernels(self):
        """hb_step_kernels: HB_KERN_* bits of the kernels the last step launched."""
        m = C.c_uint32()
        _check("hb_step_kernels", lib().hb_step_kernels(self.h, C.byref(m)))
        return int(m.value)

    def phase_ms(self):
        """(per-phase average ms, number of profiled steps) since phase_reset()."""
        out = np.zeros(abi.HB_PHASE_COUNT, dtype=np.float32)
        n = C.c_uint32()
        _check("hb_phase_ms", lib().hb_phase_ms(self.h, out.ctypes.data, C.byref(n)))
        return out, n.value
