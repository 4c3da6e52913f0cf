"""Short bench-config run for rocprofv3 (no CPU baseline, few steps).

Usage under the profiler (program itself after --, no launcher hop):
  rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 tools/profile_run.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = [sys.argv[0], "--steps", os.environ.get("GH_PROF_STEPS", "20"), "--warmup", "5", "--no-cpu-baseline", "--no-secondary"] + sys.argv[1:]
import bench  # noqa: E402

bench.main()
