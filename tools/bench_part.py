"""Run one bench.py section alone (profiling helper): python tools/bench_part.py track [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

part = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
d = bench.Dist()
r = getattr(bench, "run_" + part)(d, 0, steps, 3)
import json  # noqa: E402
print(json.dumps({k: v for k, v in r.items() if isinstance(v, (int, float, str, dict))},
                 default=str))
