"""Copy/kernel overlap of the end-to-end ingest from a rocprofv3 trace (--kernel-trace --memory-copy-trace,
csv): inside the window from the first host-to-device copy of at least 1 MB to the last copy's end, the
time the H2D copies run, the time kernels run, and the time both run at once.  Usage:
    python tools/overlap.py <trace dir> [label]"""
import csv
import glob
import os
import sys


def _rows(d, what):
    f = glob.glob(os.path.join(d, "**", f"*{what}*.csv"), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def _col(row, *names):
    for n in names:
        for k in row:
            if k.lower() == n.lower():
                return row[k]
    return None


def _union(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def _measure(iv):
    return sum(b - a for a, b in iv)


def _intersect(x, y):
    i = j = 0
    out = []
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            out.append([a, b])
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return out


def main(d, label=""):
    cps = _rows(d, "memory_copy_trace")
    ks = _rows(d, "kernel_trace")
    h2d = []
    allc = []
    for r in cps:
        a, b = int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp"))
        direction = (_col(r, "Direction") or _col(r, "Operation") or _col(r, "Kind") or "").upper()
        nbytes = int(_col(r, "Size", "Bytes", "Copy_Bytes") or 0)
        allc.append((a, b))
        if "HOST_TO_DEVICE" in direction and (nbytes >= (1 << 20) or nbytes == 0 and b - a > 50_000):
            h2d.append((a, b))
    if not h2d:
        print("no H2D copies found; columns:", list(cps[0].keys()) if cps else None)
        return 1
    w0, w1 = min(a for a, _ in h2d), max(b for _, b in allc)
    kern = _union([(max(w0, int(_col(r, "Start_Timestamp"))), min(w1, int(_col(r, "End_Timestamp")))) for r in ks
                   if int(_col(r, "End_Timestamp")) > w0 and int(_col(r, "Start_Timestamp")) < w1])
    cu = _union([(a, b) for a, b in h2d if b > w0 and a < w1])
    both = _intersect(cu, kern)
    win, tc, tk, tb = (w1 - w0) / 1e6, _measure(cu) / 1e6, _measure(kern) / 1e6, _measure(both) / 1e6
    print(f"{label} window {win:.2f} ms: H2D copies {tc:.2f} ms ({len(h2d)} copies >= 1 MB), kernels {tk:.2f} ms, "
          f"both at once {tb:.2f} ms = {tb / tc:.0%} of the copy time, {tb / max(tk, 1e-9):.0%} of the kernel time; "
          f"copies+kernels serialised would be {tc + tk:.2f} ms, run {tc + tk - tb:.2f} ms")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""))
