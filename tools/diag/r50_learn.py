#!/usr/bin/env python3
"""Does the ResNet-50 bench step learn?  Runs N steps of bench.py's workload and prints
loss, loss scale and skipped steps, plus the gradient norm of a few layers."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from apex_example_amd import amp  # noqa: E402
from apex_example_amd.amp._amp_state import _amp_state  # noqa: E402


def main():
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if args.gemm_tuning == "auto" and not os.environ.get("PYTORCH_TUNABLEOP_ENABLED"):
        from apex_example_amd.utils.gemm_tuning import use_tuned_gemms
        print("tuned GEMM table:", use_tuned_gemms(args.model), flush=True)
    w = bench.build_resnet(args, dev, 1)
    for i in range(int(os.environ.get("N_STEPS", "12"))):
        loss = w.step(w.batch)
        sc = _amp_state.loss_scalers[0]
        print("step %2d loss %.4f scale %s skipped %s" % (i, loss.item(), sc.loss_scale(),
                                                          sc.skipped_steps()), flush=True)


if __name__ == "__main__":
    main()
