"""Build libsiddhi_hip.so for gfx950 (hipcc), in-tree so it travels with the repo snapshot.

Each translation unit is compiled to its own object (in parallel) and relinked, so a change to
one file recompiles that file only; an object is stale when its source or any shared header is
newer than it."""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libsiddhi_hip.so")
SRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build_obj")
HEADERS = ["nfa_lane.h", "wave_dpp.h", "fastpath.h", "fast_core.h", "prog.h", "compile.h", "jsonv.h", "sweep.h", "sweep_lean.h",
           "sweep_spill.h", "sweep_win.h", "cseq.h", "cseq_own.h", "labs.h"]
# (object name, source, extra flags): the kernel families are split over units that build in
# parallel (sweep_solve.hip once per e1 term count), heaviest first
UNITS = [("sweep_solve0", "sweep_solve.hip", ["-DSW_NT1=0"]), ("sweep_solve1", "sweep_solve.hip", ["-DSW_NT1=1"]),
         ("sweep_solve2", "sweep_solve.hip", ["-DSW_NT1=2"])] + \
        [(f"lanes{t}", "lanes.hip", [f"-DSHP_LANE_TIER={t}"]) for t in range(5)] + [
         ("sweep_lean", "sweep_lean.hip", []), ("sweep_lean_agg", "sweep_lean.hip", ["-DSW_LEAN_AGG"]), ("engine", "engine.hip", []), ("group", "group.hip", []),
         ("siddhiql", "siddhiql.cpp", []), ("shard", "shard.hip", []), ("synth", "synth.hip", [])]
DEPS = HEADERS + sorted({u[1] for u in UNITS})


def _hdr_time() -> float:
    hs = [os.path.join(SRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", "siddhi_hip.h")]
    return max(os.path.getmtime(h) for h in hs if os.path.exists(h))


def _stale(lib: str = LIB) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    srcs = [os.path.join(SRC, d) for d in DEPS] + [os.path.join(ROOT, "include", "siddhi_hip.h")]
    return any(os.path.getmtime(s) > t for s in srcs if os.path.exists(s))


STAMPS_LIB = os.path.join(HERE, "libsiddhi_hip_stamps.so")


def build(force: bool = False, verbose: bool = False, stamps: bool = False, src: str = None, out: str = None,
          extra=None) -> str:
    """stamps=True builds the diagnostic variant (in-kernel phase stamps, tools/sweep_probe.py).
    src / out / extra: an A/B variant -- sources from another tree (tools/build_variant.sh), the
    library name under siddhi_amd/, extra compiler flags (objects in their own directory)."""
    lib = STAMPS_LIB if stamps else LIB
    if out:
        lib = os.path.join(HERE, out)
        force = True
    if not force and not _stale(lib):
        return lib
    csrc = os.path.join(src, "siddhi_amd", "csrc") if src else SRC
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC"]
    if stamps:
        flags.append("-DSHP_SW_STAMPS")
    flags += list(extra or [])
    odir = OBJ + ("_stamps" if stamps else "") + ("_" + os.path.splitext(out)[0] if out else "")
    os.makedirs(odir, exist_ok=True)
    ht = _hdr_time()

    def obj(u) -> str:
        name, file, extra = u
        src = os.path.join(csrc, file)
        o = os.path.join(odir, name + ".o")
        if force or not os.path.exists(o) or os.path.getmtime(o) < max(ht, os.path.getmtime(src)):
            cmd = [hipcc] + flags + extra + ["-c", "-o", o + ".tmp", src]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            subprocess.check_call(cmd)
            os.replace(o + ".tmp", o)
        return o

    with ThreadPoolExecutor(max_workers=min(len(UNITS), os.cpu_count() or 8, 16)) as ex:
        objs = list(ex.map(obj, UNITS))
    cmd = [hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib + ".tmp"] + objs + ["-lrccl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--src", help="tree holding siddhi_amd/csrc (an A/B variant)")
    ap.add_argument("--out", help="variant library name under siddhi_amd/")
    a, extra = ap.parse_known_args()
    print(build(force=a.force, verbose=True, stamps=a.stamps, src=a.src, out=a.out, extra=extra))
