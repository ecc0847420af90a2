"""GPU probe: device-flag protocol of the captured compute/comm graphs (flags + timing)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    args = bench.parse(["--global-batch", "64"] + sys.argv[1:])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wl = bench.Workload(args, dev, 1, 0)
    step = wl.make_step(64)
    step(0)
    torch.cuda.synchronize()
    f = wl.comm._flags
    print("after capture+1 replay: ctr", f[:6].tolist(), "seen", f[256:262].tolist(), "done", f[512:515].tolist(),
          flush=True)
    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    print("after 4 replays: ctr", f[:6].tolist(), "seen", f[256:262].tolist(), "done", f[512:515].tolist(), flush=True)


if __name__ == "__main__":
    main()
