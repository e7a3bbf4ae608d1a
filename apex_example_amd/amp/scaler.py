"""Dynamic / static loss scaler (apex@f3a960f8 apex/amp/scaler.py).

Apex semantics: "dynamic" starts at min(max_loss_scale, 2**16); an overflow
halves the scale (floored at min_loss_scale), resets the clean-step counter and
skips the step; 2000 clean steps double it (capped at max_loss_scale).  A static
scaler never skips.

MI355X design - two modes:

* ``sync``  (Apex-identical): ``update_scale()`` reads the overflow flag with one
  device->host copy per step and returns ``should_skip``.
* ``sync-free`` (default on GPU when every optimizer is one of this package's
  fused optimizers): the scale, the clean-step counter and the skip counter live
  in device memory; ``update_scale()`` launches a one-thread kernel and returns
  False; the fused optimizer kernels read the overflow flag on the device and
  no-op.  The host never waits, so the CPU runs ahead of the GPU and the step is
  hipGraph-capturable.  The Apex overflow message is still printed: the skip
  counter is copied to pinned memory asynchronously and polled (no stall) at the
  next ``scale_loss``.
"""
from __future__ import annotations

import torch

from .. import _native
from ._amp_state import _amp_state, maybe_print


class LossScaler(object):
    warned_no_fused_kernel = False
    warned_unscaling_non_fp32_grad = False
    has_fused_kernel = False

    def __init__(self, loss_scale, init_scale=2.**16, scale_factor=2., scale_window=2000,
                 min_loss_scale=None, max_loss_scale=2.**24, device=None, sync_free=False):
        if loss_scale == "dynamic":
            self.dynamic = True
            self._loss_scale = min(max_loss_scale, init_scale)
        else:
            self.dynamic = False
            self._loss_scale = float(loss_scale)
        self._max_loss_scale = max_loss_scale
        self._min_loss_scale = min_loss_scale
        self._scale_seq_len = scale_window
        self._scale_factor = scale_factor
        self._unskipped = 0
        self._has_overflow = False
        self._device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
            else torch.device("cpu"))
        self._overflow_buf = torch.zeros(1, dtype=torch.int32, device=self._device)
        LossScaler.has_fused_kernel = _native.available()
        self.sync_free = False
        if sync_free:
            self.enable_sync_free()

    # ------------------------------------------------------------ mode control
    def enable_sync_free(self):
        """Move the scaler state to the device (no host sync per step)."""
        if self.sync_free:
            return
        self.sync_free = True
        d = self._device
        self._scale_dev = torch.tensor([self._loss_scale], dtype=torch.float32, device=d)
        self._scale_view = self._scale_dev[0]
        # the scale the latest backward's grads carry (the update kernel writes the
        # pre-update value here): what a fused optimizer that unscales in-kernel
        # after update_scale() must divide by
        self._scale_applied = (torch.tensor([self._loss_scale], dtype=torch.float32, device=d)
                               if self.dynamic else self._scale_dev)
        self._unskipped_dev = torch.tensor([self._unskipped], dtype=torch.int32, device=d)
        self._skipped_dev = torch.zeros(1, dtype=torch.int32, device=d)
        self._skipped_seen = 0
        pin = d.type == "cuda"
        self._host_report = torch.zeros(2, dtype=torch.float32, pin_memory=pin)
        self._report_event = None

    def _sync_host_state(self):
        """Materialise device-resident state on the host (checkpointing)."""
        if self.sync_free:
            self._loss_scale = float(self._scale_dev.item())
            self._unskipped = int(self._unskipped_dev.item())

    # ------------------------------------------------------------ Apex API
    def loss_scale(self):
        if self.sync_free:
            self._sync_host_state()
        return self._loss_scale

    def loss_scale_tensor(self):
        """Device scalar (0-dim view) of the current scale (sync-free mode)."""
        return self._scale_view

    def grads_scale(self):
        """The loss scale the latest backward's gradients carry, for in-kernel
        unscaling that runs after ``update_scale()`` (a growth step must still
        divide by the pre-growth value): a device scalar in sync-free mode."""
        if self.sync_free:
            return self._scale_applied
        return getattr(self, "_applied_scale", self._loss_scale)

    def scale_for_kernels(self):
        """(value, tensor) pair understood by amp_C functions with scale_inv=True."""
        if self.sync_free:
            return self._scale_dev
        return self._loss_scale

    def unscale_python(self, model_grads, master_grads, scale):
        for model, master in zip(model_grads, master_grads):
            if model is not None:
                if not LossScaler.warned_unscaling_non_fp32_grad:
                    if master.dtype != torch.float32:
                        maybe_print("Attempting to unscale a grad with type {} Unscaling non-fp32 "
                                    "grads may indicate an error. When using Amp, you don't need "
                                    "to call .half() on your model.".format(master.type()))
                        LossScaler.warned_unscaling_non_fp32_grad = True
                self._has_overflow = bool(not torch.isfinite(model.float()).all())
                if self._has_overflow:
                    self._overflow_buf.fill_(1)
                    break
                if model is not master:
                    master.copy_(model)
                if scale != 1.0:
                    master.mul_(scale)

    def unscale(self, model_grads, master_grads, unused_scale, models_are_masters=False,
                scale_override=None):
        if self._has_overflow:
            return
        if not model_grads:
            return
        scale = self._loss_scale if scale_override is None else scale_override
        if (not self.sync_free) and scale == 1.0 and models_are_masters and not self.dynamic:
            return
        if LossScaler.has_fused_kernel:
            from .. import amp_C

            if self.sync_free and scale_override is None:
                amp_C.multi_tensor_scale(65536, self._overflow_buf, [model_grads, master_grads],
                                         self._scale_dev, scale_inv=True)
            else:
                amp_C.multi_tensor_scale(65536, self._overflow_buf, [model_grads, master_grads],
                                         1. / scale)
        else:
            self.unscale_python(model_grads, master_grads, 1. / scale)

    def check_overflow(self, grads):
        """Finiteness check only (unscaling folded into a fused optimizer)."""
        if not grads:
            return
        from .. import amp_C

        amp_C.multi_tensor_check_finite(65536, self._overflow_buf, [grads])

    def unscale_with_stashed_python(self, model_grads, stashed_master_grads, master_grads, a, b):
        for model, stashed, master in zip(model_grads, stashed_master_grads, master_grads):
            if model is None and stashed is None:
                continue
            bad = (model is not None and not torch.isfinite(model.float()).all()) or (
                stashed is not None and not torch.isfinite(stashed.float()).all())
            if bad:
                self._has_overflow = True
                self._overflow_buf.fill_(1)
                break
            val = torch.zeros_like(master, dtype=torch.float32)
            if model is not None:
                val += a * model.float()
            if stashed is not None:
                val += b * stashed.float()
            master.copy_(val)

    def unscale_with_stashed(self, model_grads, stashed_master_grads, master_grads,
                             scale_override=None):
        if self._has_overflow:
            return
        grads_have_scale, stashed_have_scale, out_scale = self._loss_scale, 1.0, 1.0
        if scale_override is not None:
            grads_have_scale, stashed_have_scale, out_scale = scale_override
        if LossScaler.has_fused_kernel:
            from .. import amp_C

            if (not LossScaler.warned_unscaling_non_fp32_grad
                    and master_grads and master_grads[0].dtype == torch.float16):
                print("Warning:  unscaling grads that are not FP32. Unscaling non-fp32 grads "
                      "may indicate an error. When using Amp, you don't need to call .half() "
                      "on your model.")
                LossScaler.warned_unscaling_non_fp32_grad = True
            if self.sync_free and scale_override is None:
                # a = out_scale / grads_have_scale computed on device: 1/scale
                amp_C.multi_tensor_axpby(65536, self._overflow_buf,
                                         [model_grads, stashed_master_grads, master_grads],
                                         self._scale_dev, out_scale / stashed_have_scale, 0,
                                         a_inv=True)
            else:
                amp_C.multi_tensor_axpby(65536, self._overflow_buf,
                                         [model_grads, stashed_master_grads, master_grads],
                                         out_scale / grads_have_scale,
                                         out_scale / stashed_have_scale, 0)
        else:
            self.unscale_with_stashed_python(model_grads, stashed_master_grads, master_grads,
                                             out_scale / grads_have_scale,
                                             out_scale / stashed_have_scale)

    def clear_overflow_state(self):
        self._has_overflow = False
        if self.has_fused_kernel or self.sync_free:
            self._overflow_buf.zero_()

    def update_scale(self):
        """Apex: returns should_skip.  Sync-free mode: updates on device, returns False."""
        if self.sync_free:
            if self.dynamic:
                _native.require().mt.update_loss_scale(
                    self._scale_dev, self._unskipped_dev, self._skipped_dev, self._overflow_buf,
                    float(self._scale_factor), int(self._scale_seq_len),
                    float(self._min_loss_scale or 0.0), float(self._max_loss_scale), True,
                    self._scale_applied)
                if not (self._device.type == "cuda"
                        and torch.cuda.is_current_stream_capturing()):
                    self._post_report()  # (inside a hipGraph capture: poll via skipped_steps())
            else:
                self._unskipped_dev.add_(1)
            return False
        self._applied_scale = self._loss_scale  # the scale this step's grads carry
        # If the fused kernel is available, we only need one D2H memcopy and sync.
        if LossScaler.has_fused_kernel and self.dynamic and not self._has_overflow:
            self._has_overflow = bool(self._overflow_buf.item())
        if self._has_overflow and self.dynamic:
            should_skip = True
            if self._min_loss_scale:
                self._loss_scale = max(self._min_loss_scale, self._loss_scale / 2.)
            else:
                self._loss_scale = self._loss_scale / 2.
            self._unskipped = 0
        else:
            should_skip = False
            self._unskipped += 1
        if self._unskipped == self._scale_seq_len and self.dynamic:
            self._loss_scale = min(self._max_loss_scale, self._loss_scale * 2.)
            self._unskipped = 0
        return should_skip

    # ------------------------------------------------------------ sync-free reporting
    def _post_report(self):
        """Queue an async copy of (skipped_total, scale) to pinned memory."""
        if self._report_event is not None and not self._report_event.query():
            return  # previous report still in flight; try again next step
        self._poll_report()
        rep = torch.stack([self._skipped_dev.float()[0], self._scale_dev[0]])
        self._host_report.copy_(rep, non_blocking=True)
        if self._device.type == "cuda":
            self._report_event = torch.cuda.Event()
            self._report_event.record()
        else:
            self._report_event = None
            self._poll_report(force=True)

    def _poll_report(self, force=False):
        if not force and (self._report_event is None or not self._report_event.query()):
            return
        skipped = int(self._host_report[0].item())
        if skipped > self._skipped_seen:
            scale = float(self._host_report[1].item())
            for _ in range(skipped - self._skipped_seen):
                maybe_print("Gradient overflow.  Skipping step, loss scaler {} reducing loss "
                            "scale to {}".format(getattr(self, "_loss_id", 0), scale))
            self._skipped_seen = skipped
        self._report_event = None

    def poll(self):
        """Print pending overflow messages whose data already reached the host."""
        if self.sync_free and not (self._device.type == "cuda"
                                   and torch.cuda.is_current_stream_capturing()):
            self._poll_report()

    def skipped_steps(self):
        """Total skipped (overflowed) steps; syncs in sync-free mode."""
        if self.sync_free:
            return int(self._skipped_dev.item())
        return getattr(self, "_skipped_host", 0)

    def load_state(self, loss_scale, unskipped):
        self._loss_scale = float(loss_scale)
        self._unskipped = int(unskipped)
        if self.sync_free:
            self._scale_dev.fill_(self._loss_scale)
            self._scale_applied.fill_(self._loss_scale)
            self._unskipped_dev.fill_(self._unskipped)
