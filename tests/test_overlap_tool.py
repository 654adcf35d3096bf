"""tools/overlap.py (the copy/kernel overlap summary of the end-to-end ingest trace) on a synthetic
rocprofv3 trace: two 1 MB H2D copies, one of them under a kernel."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)


def test_overlap_summary(tmp_path):
    _write(tmp_path / "run_memory_copy_trace.csv", [
        {"Kind": "MEMORY_COPY", "Direction": "MEMORY_COPY_HOST_TO_DEVICE", "Size": 1 << 20,
         "Start_Timestamp": 1_000_000, "End_Timestamp": 3_000_000},
        {"Kind": "MEMORY_COPY", "Direction": "MEMORY_COPY_HOST_TO_DEVICE", "Size": 1 << 20,
         "Start_Timestamp": 5_000_000, "End_Timestamp": 7_000_000},
        {"Kind": "MEMORY_COPY", "Direction": "MEMORY_COPY_DEVICE_TO_HOST", "Size": 64,
         "Start_Timestamp": 8_000_000, "End_Timestamp": 8_100_000}])
    _write(tmp_path / "run_kernel_trace.csv", [
        {"Kernel_Name": "a", "Start_Timestamp": 0, "End_Timestamp": 500_000},          # before the window
        {"Kernel_Name": "b", "Start_Timestamp": 5_500_000, "End_Timestamp": 6_500_000},  # under copy 2
        {"Kernel_Name": "c", "Start_Timestamp": 3_000_000, "End_Timestamp": 4_000_000}])  # between
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "overlap.py"), str(tmp_path), "x"],
                         capture_output=True, text=True, check=True).stdout
    assert "window 7.10 ms" in out and "H2D copies 4.00 ms (2 copies" in out
    assert "kernels 2.00 ms" in out and "both at once 1.00 ms = 25% of the copy time, 50% of the kernel time" in out
