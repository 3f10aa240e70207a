"""torch.profiler op table (with input shapes) for one 7B bench step — finds the
PyTorch-side elementwise work (fills, casts, adds) in the step."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
    bench.main(["--steps", "1", "--warmup", "1"])
tab = prof.key_averages(group_by_input_shape=True)
rows = sorted(tab, key=lambda e: -e.device_time_total)
print(f"{'op':40s} {'calls':>6s} {'dev ms':>9s}  shapes")
for e in rows[:60]:
    if e.device_time_total <= 0:
        continue
    print(f"{e.key[:40]:40s} {e.count:6d} {e.device_time_total / 1e3:9.2f}  {str(e.input_shapes)[:110]}")
