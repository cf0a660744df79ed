"""The engine and PyTorch share one HIP runtime whatever the import order
(etcd_amd/hipbatch.py _bind_one_hip_runtime).  r05: a process that loaded
libhbnode.so (for the router) before torch mapped /opt/rocm's libamdhip64
beside torch's own copy, and hb_create then failed with HB_EDEVICE.  Each case
runs in a fresh interpreter (the mapping is per process); none touches a GPU."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code):
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout.strip().splitlines()[-1]


@pytest.mark.parametrize("first", ["multinode", "router", "engine"])
def test_one_hip_runtime_when_the_engine_loads_before_torch(first):
    load = {"multinode": "from etcd_amd import multinode; multinode.lib()",
            "router": "import numpy as np; from etcd_amd.shard import NativeRouter; "
                      "NativeRouter(np.arange(10, dtype=np.uint64), 2)",
            "engine": "from etcd_amd import hipbatch; hipbatch.lib()"}[first]
    out = _run(f"{load}\nimport torch\nfrom etcd_amd import hipbatch\n"
               "print(len(hipbatch._mapped_hip_runtimes()))")
    assert out == "1"


def test_one_hip_runtime_when_torch_loads_first():
    out = _run("import torch\nfrom etcd_amd import multinode; multinode.lib()\n"
               "from etcd_amd import hipbatch\nprint(len(hipbatch._mapped_hip_runtimes()))")
    assert out == "1"


def test_two_runtimes_already_mapped_is_a_named_error():
    code = ("import ctypes, glob, os\n"
            "import importlib.util as u\n"
            "torch_rt = os.path.join(u.find_spec('torch').submodule_search_locations[0], 'lib', 'libamdhip64.so')\n"
            "rocm_rt = sorted(glob.glob('/opt/rocm/lib/libamdhip64.so.*'))[0]\n"
            "if not os.path.exists(torch_rt) or os.path.realpath(torch_rt) == os.path.realpath(rocm_rt):\n"
            "    print('skip'); raise SystemExit\n"
            "ctypes.CDLL(rocm_rt); ctypes.CDLL(torch_rt)\n"
            "from etcd_amd import hipbatch\n"
            "try:\n"
            "    hipbatch.lib()\n"
            "    print('loaded')\n"
            "except hipbatch.HipRuntimeConflict:\n"
            "    print('conflict')\n")
    out = _run(code)
    if out == "skip":
        pytest.skip("one HIP runtime on this machine")
    assert out == "conflict"
