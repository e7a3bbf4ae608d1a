"""Legacy one-process-per-GPU launcher (apex@f3a960f8 apex/parallel/multiproc.py,
SURVEY.md A-19):

    python -m apex_example_amd.parallel.multiproc train.py [script args]

starts ``world_size`` = number of visible GPUs (``--nproc N`` to override)
copies of the script, appending ``--world-size N --rank i`` to each, with
MASTER_ADDR / MASTER_PORT (default 127.0.0.1:29500) and RANK / LOCAL_RANK /
WORLD_SIZE exported for ``init_process_group('nccl', init_method='env://')``.
Children are separate processes (never an exec of this one); the launcher
waits for all of them and exits with the first non-zero return code, after
terminating the rest.  ``torchrun`` is the modern equivalent.
"""
from __future__ import annotations

import os
import subprocess
import sys
import time


def _world(argv):
    if "--nproc" in argv:
        i = argv.index("--nproc")
        n = int(argv[i + 1])
        del argv[i:i + 2]
        return n
    import torch  # device_count() does not initialise the GPU

    return max(1, torch.cuda.device_count())


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    world = _world(argv)
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    env.setdefault("MASTER_PORT", "29500")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = []
    for rank in range(world):
        e = dict(env, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world))
        cmd = [sys.executable] + argv + ["--world-size", str(world), "--rank", str(rank)]
        procs.append(subprocess.Popen(cmd, env=e))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                r = p.poll()
                if r is None:
                    continue
                live.remove(p)
                if r != 0 and rc == 0:
                    rc = r
                    for q in live:
                        q.terminate()
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


if __name__ == "__main__":
    sys.exit(main())
