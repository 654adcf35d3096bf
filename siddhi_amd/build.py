"""Build libsiddhi_hip.so for gfx950 (hipcc), in-tree so it travels with the repo snapshot."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libsiddhi_hip.so")
SRC = os.path.join(HERE, "csrc")
DEPS = ["engine.hip", "synth.hip", "shard.hip", "group.hip", "nfa_lane.h", "fastpath.h", "fast_core.h", "prog.h", "compile.h", "jsonv.h", "sweep.h", "sweep_lean.h", "cseq.h", "labs.h"]


def _stale(lib: str = LIB) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    srcs = [os.path.join(SRC, d) for d in DEPS] + [os.path.join(ROOT, "include", "siddhi_hip.h")]
    return any(os.path.getmtime(s) > t for s in srcs if os.path.exists(s))


STAMPS_LIB = os.path.join(HERE, "libsiddhi_hip_stamps.so")


def build(force: bool = False, verbose: bool = False, stamps: bool = False) -> str:
    """stamps=True builds the diagnostic variant (in-kernel phase stamps, tools/sweep_probe.py)."""
    lib = STAMPS_LIB if stamps else LIB
    if not force and not _stale(lib):
        return lib
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-o", lib + ".tmp", os.path.join(SRC, "engine.hip"), os.path.join(SRC, "synth.hip"),
           os.path.join(SRC, "shard.hip"), os.path.join(SRC, "group.hip"), "-lrccl"]
    if stamps:
        cmd.insert(3, "-DSHP_SW_STAMPS")
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, stamps="--stamps" in sys.argv))
