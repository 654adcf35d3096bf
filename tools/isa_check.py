#!/usr/bin/env python3
"""ISA wait-counter check of the hot kernels (a build step: __graft_entry__.build() runs it).

Round 4's largest single gain came from wait counters: the compiler merged code paths so that a
loop waited for every outstanding vector memory operation (`s_waitcnt vmcnt(0)`) where it needed
none -- e.g. k_sw_lean's emission held each 64-position block for the previous block's stores.
Such a regression is invisible to the parity tests and costs 10 % of a step.  This check
disassembles the gfx950 code objects of the built units, finds each hot kernel's loops (the
ranges [target, branch] of its backward branches) and counts the `s_waitcnt vmcnt(0)` inside them;
a count above tools/isa_budget.json's fails the build.

    python tools/isa_check.py            # check against the budget
    python tools/isa_check.py --update   # write the current counts as the budget
    python tools/isa_check.py --list     # every kernel's counts
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "siddhi_amd", "build_obj")
BUDGET = os.path.join(ROOT, "tools", "isa_budget.json")
LLVM = "/opt/rocm/lib/llvm/bin"
# the kernels of the default paths of SURVEY §8d's configs (demangled-name prefixes)
HOT = ("k_sw_count", "k_sw_scatter", "k_sw_lean", "k_co_count", "k_co_scatter", "k_co_run", "k_cs3", "k_cs_pack", "k_la_ms",
       "k_labs_w", "k_labs_pack", "k_labs_out")
UNITS = ("sweep_solve0", "sweep_lean", "sweep_lean_agg", "engine")

_FN = re.compile(r"^([0-9a-f]+) <([^>]+)>:$")
_INS = re.compile(r"//\s*([0-9A-F]{8,16}):")
_TGT = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>\s*$")


def _demangle(names):
    filt = os.path.join(LLVM, "llvm-cxxfilt")
    out = subprocess.run([filt if os.path.exists(filt) else "c++filt"], input="\n".join(names), capture_output=True, text=True,
                         check=True).stdout.split("\n")
    return dict(zip(names, out))


def disassemble(obj: str) -> str:
    with tempfile.TemporaryDirectory() as td:
        fb, co = os.path.join(td, "fatbin"), os.path.join(td, "co")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", obj,
                        os.path.join(td, "x.o")], check=True, capture_output=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}", f"--output={co}", "--unbundle"],
                       check=True, capture_output=True)
        return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", "--no-show-raw-insn", co],
                              check=True, capture_output=True, text=True).stdout


def loop_waits(text: str):
    """{mangled kernel: (vmcnt(0) inside loops, ... inside nested loops, vmcnt(0) anywhere, loops)}"""
    funcs, cur = {}, None
    for line in text.splitlines():
        m = _FN.match(line)
        if m:
            cur = m.group(2)
            funcs[cur] = {"start": int(m.group(1), 16), "ins": []}
            continue
        if cur is None:
            continue
        a = _INS.search(line)
        if a:
            funcs[cur]["ins"].append((int(a.group(1), 16), line.strip()))
    res = {}
    for name, f in funcs.items():
        loops = []
        for addr, ins in f["ins"]:
            if not (ins.startswith("s_branch") or ins.startswith("s_cbranch")):
                continue
            t = _TGT.search(ins)
            if not t or t.group(1) not in funcs:
                continue
            tgt = funcs[t.group(1)]["start"] + int(t.group(2), 16)
            if tgt <= addr:
                loops.append((tgt, addr))
        waits = [addr for addr, ins in f["ins"] if re.match(r"s_waitcnt\b.*\bvmcnt\(0\)", ins)]
        depth = [sum(1 for lo, hi in loops if lo <= w <= hi) for w in waits]
        res[name] = (sum(1 for d in depth if d >= 1), sum(1 for d in depth if d >= 2), len(waits), len(loops))
    return res


TOOLS = ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")  # (c++filt stands in for llvm-cxxfilt)


def collect():
    out = {}
    for u in UNITS:
        obj = os.path.join(OBJ, u + ".o")
        if not os.path.exists(obj):
            print(f"isa_check: {u}.o not built, skipped", file=sys.stderr)
            continue
        try:
            text = disassemble(obj)
        except (OSError, subprocess.CalledProcessError) as e:  # a toolchain difference is no regression
            print(f"isa_check: cannot disassemble {u}.o ({e}), skipped", file=sys.stderr)
            continue
        lw = loop_waits(text)
        dm = _demangle(list(lw))
        for mname, v in lw.items():
            d = dm[mname]
            base = re.sub(r"<.*", "", d.split("(")[0]).split("::")[-1]
            if base.startswith(HOT):
                out[f"{u}:{d.split('(')[0]}"] = v
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--update", action="store_true")
    ap.add_argument("--list", action="store_true")
    a = ap.parse_args(argv)
    absent = [t for t in TOOLS if not os.path.exists(os.path.join(LLVM, t))]
    if absent:  # only an over-budget count fails the build; a missing tool skips the check
        print(f"isa_check: skipped ({', '.join(absent)} not under {LLVM})", file=sys.stderr)
        return 0
    cur = collect()
    if a.list or a.update:
        for k, (il, nest, tot, nl) in sorted(cur.items()):
            print(f"{il:4d} in loops / {nest:4d} nested / {tot:4d} total / {nl:4d} loops  {k}")
    if a.update:
        json.dump({k: list(v[:2]) for k, v in sorted(cur.items())}, open(BUDGET, "w"), indent=1)
        print("budget written:", BUDGET)
        return 0
    if not os.path.exists(BUDGET):
        print("isa_check: no budget file (run with --update)", file=sys.stderr)
        return 1
    bud = json.load(open(BUDGET))
    # nested-loop waits may not grow; a wait moved out of a nested loop into the outer one is no regression
    bad = [(k, v[:2], bud[k]) for k, v in cur.items()
           if k in bud and (v[1] > bud[k][1] or v[0] > bud[k][0] + (bud[k][1] - v[1]))]
    missing = [k for k in bud if k not in cur]
    for k, n, b in bad:
        print(f"isa_check: {k}: s_waitcnt vmcnt(0) in loops / nested loops {n[0]} / {n[1]} (budget {b[0]} / {b[1]})",
              file=sys.stderr)
    if missing:
        print(f"isa_check: {len(missing)} budgeted kernels not found (renamed? run --update): {missing[:3]}",
              file=sys.stderr)
    print(f"isa_check: {len(cur)} hot kernels, {sum(v[0] for v in cur.values())} loop vmcnt(0) waits, "
          f"{len(bad)} over budget")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
