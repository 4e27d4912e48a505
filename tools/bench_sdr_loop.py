"""Quick run of bench.py's closed-loop leg alone (+ its CPU baseline)."""
import json
import sys
import numpy as np
sys.path.insert(0, ".")
import bench
d = bench.Dist()
lp = bench.run_sdr_loop(d, 0, np.random.default_rng(7))
print(json.dumps({k: v for k, v in lp.items() if k not in ("pk", "chans")}))
print("channel-ms/s", lp["dumps"] / lp["dt"], "realtime ch", lp["dumps"] / lp["steps"] / lp["ms"])
if len(sys.argv) > 1:
    print(json.dumps(bench.cpu_baseline_sdr_loop(lp)))
