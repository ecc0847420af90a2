"""GPU probe: host time spent inside hipGraph replay() vs GPU step time (ResNet-18 step)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    args = bench.parse(sys.argv[1:])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wl = bench.Workload(args, dev, 1, 0)
    per = args.global_batch if args.scaling == "strong" else args.batch
    step = wl.make_step(per)
    for i in range(5):
        step(i)
    torch.cuda.synchronize()
    runner = step.__closure__ and [c.cell_contents for c in step.__closure__ if hasattr(c.cell_contents, "host_launch_s")]
    r = runner[0]
    r.host_launch_s = [0.0, 0.0]
    n = 20
    t0 = time.perf_counter()
    for i in range(n):
        step(i)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("DEBUG_")},
                      "overlap": not args.no_overlap, "batch": per,
                      "ms_per_step": 1e3 * t_all / n, "host_ms_per_step": 1e3 * t_host / n,
                      "replay_compute_ms": 1e3 * r.host_launch_s[0] / n,
                      "replay_comm_ms": 1e3 * r.host_launch_s[1] / n}), flush=True)


if __name__ == "__main__":
    main()
