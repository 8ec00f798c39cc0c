"""A context's td_evaluate walk with a torch.distributed collective between
the evaluates, in a FRESH child process (tests/test_gpu_incremental.py):
world 1 over RCCL ("nccl") on device 0.  Reports the results and the wall
time of every evaluate + all_gather, for td_set_incremental mode 1 (one
launch per call) and mode 2 (resident kernel), so the interaction of a
resident kernel with the collective's stream is measured, not assumed.

usage: collective_worker.py PORT OUT.json MODE
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    port, out, mode = int(sys.argv[1]), sys.argv[2], int(sys.argv[3])
    import numpy as np
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    import tonga

    tt = tonga.load()
    ds = tt.load_data_Tonga()
    ctx = tt.TdContext.from_datastruct(ds, device=0)
    ctx.set_incremental(mode)
    rng = np.random.default_rng(4)
    x, y, z, v = (np.array(a) for a in tt.random_model(1000, 4).cells())
    phis, times = [], []
    buf = torch.zeros(8, dtype=torch.float64, device="cuda")
    outb = torch.zeros(8, dtype=torch.float64, device="cuda")
    for k in range(120):
        i = int(rng.integers(len(v)))
        v = v.copy()
        v[i] = float(rng.uniform(0, 50))  # a change proposal, always "accepted"
        t0 = time.perf_counter()
        _, phi, _, _ = ctx.evaluate((x, y, z, v))
        buf[0] = phi
        dist.all_gather_into_tensor(outb, buf)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        phis.append(float(outb[0].item()))
    with open(out, "w") as f:
        json.dump({"phis": phis, "times": times}, f)
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
