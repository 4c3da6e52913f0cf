"""Short bench-config run for rocprofv3 (no CPU baseline, few steps).

Usage under the profiler (program itself after --, no launcher hop):
  rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 tools/profile_run.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# (defaults = bench.py's own: the same history length, hence the same memory footprint, as the bench line)
sys.argv = [sys.argv[0], "--steps", os.environ.get("GH_PROF_STEPS", "100"), "--warmup", os.environ.get("GH_PROF_WARMUP", "10"),
            "--no-cpu-baseline", "--no-secondary"] + sys.argv[1:]
import bench  # noqa: E402

bench.main()
