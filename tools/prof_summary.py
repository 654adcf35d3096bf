#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd SQLite db or kernel_stats.csv) as a small
text table: kernel (short name), calls, total us, average us, percent. Usage: prof_summary.py <db|csv>"""
import csv
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", name)
    if "rocprim" in name:
        for tag in ("radix_sort_onesweep_iteration", "radix_sort_onesweep_global_offsets", "scan_impl",
                    "init_lookback_scan_state", "radix_sort_block_sort", "merge_sort"):
            if tag in name:
                m = re.search(r"<rocprim::ROCPRIM_\w+::default_config, ([^>]*?)>", name)
                return f"rocprim::{tag}<{m.group(1) if m else ''}>"
    return n.replace("void ", "")[:110]


def rows(path):
    if path.endswith(".csv"):
        with open(path) as f:
            for r in csv.DictReader(f):
                yield r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3, float(r["Percentage"])
    else:
        c = sqlite3.connect(path)
        for n, calls, tot, avg, pct in c.execute("select name,total_calls,total_duration,average,percentage from top_kernels"):
            # rocpd's top_kernels view reports microseconds
            yield n, int(calls), tot, avg, pct


def main():
    out = [f"{'kernel':<80} {'calls':>6} {'total_us':>12} {'avg_us':>10} {'pct':>6}"]
    for n, calls, tot, avg, pct in rows(sys.argv[1]):
        out.append(f"{short(n):<80} {calls:>6} {tot:>12.1f} {avg:>10.1f} {pct:>6.2f}")
    print("\n".join(out))


if __name__ == "__main__":
    main()
