"""Diagnostic: 2-rank gloo DDP+SyncBN (one GPU) vs one process on the
concatenated batch, at several lr / opt levels; prints loss trajectories."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import dist_workers as W  # noqa: E402

from apex_example_amd.amp import amp as _amp  # noqa: E402


def main():
    for lr, ol in ((0.05, "O2"), (0.01, "O2"), (0.05, "O0"), (0.01, "O0")):
        with tempfile.TemporaryDirectory() as d:
            res = W.run("gpu_ddp_resnet", 2, d, syncbn=True, lr=lr, opt_level=ol, steps=6)
        ref = W.gpu_resnet_reference(world=2, lr=lr, opt_level=ol, steps=6)
        _amp.deinit()
        ddp = [(a + b) / 2 for a, b in zip(res[0]["losses"], res[1]["losses"])]
        print("lr %.3f %s ddp %s" % (lr, ol, " ".join("%.4f" % v for v in ddp)), flush=True)
        print("lr %.3f %s ref %s" % (lr, ol, " ".join("%.4f" % v for v in ref["losses"])),
              flush=True)


if __name__ == "__main__":
    main()
