"""Rehearses bench.py's harness collectives over RCCL on a one-GPU box.

Launched under torch.distributed.run with --nproc-per-node 1: the same calls
bench.py makes for N > 1 (init_process_group("nccl", device_id=...), barrier,
all_reduce MAX / SUM on device tensors), at world size 1.  The 8-GPU case is
run by the driver only.
"""
import json
import os

import torch
import torch.distributed as dist


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    dist.barrier()
    torch.cuda.synchronize()
    t = torch.tensor([1.25 + dist.get_rank()], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    s = torch.tensor([3, 5], dtype=torch.int64, device=dev)
    dist.all_reduce(s)
    dist.barrier()
    ok = float(t.item()) == 1.25 + dist.get_world_size() - 1 and s.tolist() == [3 * dist.get_world_size(),
                                                                                 5 * dist.get_world_size()]
    if dist.get_rank() == 0:
        print(json.dumps({"backend": dist.get_backend(), "world": dist.get_world_size(), "max": t.item(),
                          "sum": s.tolist(), "ok": ok, "hip": torch.version.hip}), flush=True)
    dist.destroy_process_group()
    if not ok:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
