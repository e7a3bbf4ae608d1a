"""Probe what RCCL allows on a 1-GPU box (diagnostic, not a test).

    python tools/diag/rccl_probe.py --world 1
    python tools/diag/rccl_probe.py --world 2      # two ranks sharing cuda:0

Checks: ReduceOp.AVG all-reduce, all_gather_into_tensor, a second
communicator with high-priority streams (ProcessGroupNCCL.Options), and
whether RCCL accepts two ranks on one device.
"""
import argparse
import datetime
import os
import sys
import traceback

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    try:
        t = torch.full((1024,), float(rank + 1), device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.AVG)
        torch.cuda.synchronize()
        print("rank %d avg ok %.3f" % (rank, t[0].item()), flush=True)
        out = torch.empty(world * 4, device=dev)
        dist.all_gather_into_tensor(out, torch.full((4,), float(rank), device=dev))
        torch.cuda.synchronize()
        print("rank %d all_gather ok %s" % (rank, out.tolist()), flush=True)
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        g = dist.new_group(list(range(world)), pg_options=opts)
        t2 = torch.ones(1 << 20, device=dev, dtype=torch.bfloat16)
        dist.all_reduce(t2, group=g)
        torch.cuda.synchronize()
        print("rank %d hi-prio group ok %.1f" % (rank, t2[0].item()), flush=True)
        dist.barrier(device_ids=[0])
    except Exception:
        traceback.print_exc()
        raise
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--port", type=int, default=29631)
    a = ap.parse_args()
    mp.start_processes(worker, args=(a.world, a.port), nprocs=a.world, start_method="spawn")
    print("probe world=%d ok" % a.world)


if __name__ == "__main__":
    sys.exit(main())
