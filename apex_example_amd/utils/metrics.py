"""Structured training metrics.

:class:`MetricsLogger` emits one JSON record every ``every`` steps on global
rank 0: throughput (units/s over the window), mean step ms, the current loss
scale and skipped-step count of every amp loss scaler, the last loss, and
optionally DDP per-bucket all-reduce times.  It synchronises only at record
boundaries (one device sync per window, never per step), so it can stay on
in production runs.  Records go to stdout and/or a JSON-lines file.
"""
from __future__ import annotations

import json
import sys
import time

import torch

from .dist import get_rank


def amp_scaler_stats():
    """[{'loss_scale', 'skipped_steps'}] for every initialised amp loss scaler."""
    from ..amp._amp_state import _amp_state

    out = []
    for sc in getattr(_amp_state, "loss_scalers", []) or []:
        d = {"loss_scale": float(sc.loss_scale())}
        skipped = getattr(sc, "skipped_steps", None)
        if callable(skipped):
            d["skipped_steps"] = int(skipped())
        out.append(d)
    return out


class MetricsLogger:
    def __init__(self, every=100, units_per_step=1, unit="samples", path=None, stream=sys.stdout,
                 ddp=None, extra=None):
        self.every = max(1, int(every))
        self.units_per_step = units_per_step
        self.unit = unit
        self.path = path
        self.stream = stream
        self.ddp = ddp
        self.extra = dict(extra or {})
        self.rank = get_rank()
        self.step = 0
        self._t0 = None
        self._n0 = 0
        self.records = []

    def start(self):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self._t0 = time.perf_counter()
        self._n0 = self.step

    def update(self, loss=None, **fields):
        """Call once per optimizer step.  ``loss`` may be a device tensor; it is
        only read (synchronously) at record boundaries."""
        if self._t0 is None:
            self.start()
        self.step += 1
        if self.step % self.every:
            return None
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        t = time.perf_counter()
        steps = self.step - self._n0
        dt = t - self._t0
        rec = {"step": self.step, "step_ms": 1e3 * dt / max(steps, 1),
               "throughput": self.units_per_step * steps / max(dt, 1e-9),
               "unit": self.unit + "/s"}
        if loss is not None:
            rec["loss"] = float(loss.detach().float().item() if torch.is_tensor(loss) else loss)
        scalers = amp_scaler_stats()
        if scalers:
            rec["amp"] = scalers
        if self.ddp is not None and hasattr(self.ddp, "bucket_times_ms"):
            bt = self.ddp.bucket_times_ms()
            if bt:
                rec["allreduce_ms_per_bucket"] = bt
        rec.update(self.extra)
        rec.update(fields)
        self.records.append(rec)
        if self.rank == 0:
            line = json.dumps(rec)
            if self.stream is not None:
                print(line, file=self.stream, flush=True)
            if self.path:
                with open(self.path, "a") as f:
                    f.write(line + "\n")
        self._t0 = time.perf_counter()
        self._n0 = self.step
        return rec
