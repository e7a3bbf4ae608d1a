"""``amp.scale_loss`` and the legacy handles (apex@f3a960f8 apex/amp/handle.py,
SURVEY.md A-05, call stack §3.4)."""
from __future__ import annotations

import contextlib
import warnings

import torch

from ..utils import fault as _fault
from ._amp_state import _amp_state, maybe_print


def _is_optimizer(o):
    from ..parallel.LARC import LARC

    return isinstance(o, (torch.optim.Optimizer, LARC))


@contextlib.contextmanager
def scale_loss(loss, optimizers, loss_id=0, model=None, delay_unscale=False,
               delay_overflow_check=False):
    """Yield ``loss.float() * loss_scale``; on exit unscale the gradients into the
    optimizer's (master) grads, check for overflow and update the scale.

    On overflow Apex skips the next ``optimizer.step()`` (and prints
    "Gradient overflow.  Skipping step, loss scaler N reducing loss scale to S").
    In sync-free mode (scaler.sync_free) the skip happens on the device inside
    the fused optimizer kernels; the message is printed asynchronously.
    """
    if not hasattr(_amp_state, "opt_properties"):
        raise RuntimeError("Invoked 'with amp.scale_loss`, but internal Amp state has not been "
                           "initialized.  model, optimizer = amp.initialize(model, optimizer, "
                           "opt_level=...) must be called before `with amp.scale_loss`.")

    if not _amp_state.opt_properties.enabled:
        yield loss
        return

    if _is_optimizer(optimizers):
        optimizers = [optimizers]

    loss_scaler = _amp_state.loss_scalers[loss_id]
    loss_scaler._loss_id = loss_id
    loss_scaler.poll()

    if ((not _amp_state.opt_properties.master_weights) and (not loss_scaler.dynamic)
            and (not loss_scaler.sync_free) and loss_scaler.loss_scale() == 1.0):
        yield loss.float()
        if _amp_state.opt_properties.patch_torch_functions:
            _amp_state.handle._clear_cache()
        return

    if not delay_unscale:
        if isinstance(optimizers, list):
            for optimizer in optimizers:
                if not optimizer._amp_stash.params_have_scaled_gradients:
                    optimizer._prepare_amp_backward()

    if loss_scaler.sync_free:
        yield loss.float() * loss_scaler.loss_scale_tensor()
    else:
        yield loss.float() * loss_scaler.loss_scale()

    if delay_unscale:
        for optimizer in optimizers:
            optimizer._amp_stash.params_have_scaled_gradients = True
    else:
        _fault.on_backward_end(optimizers)
        loss_scaler.clear_overflow_state()
        for optimizer in optimizers:
            optimizer._post_amp_backward(loss_scaler)
            optimizer._amp_stash.params_have_scaled_gradients = False
            optimizer._amp_stash.last_scaler = loss_scaler
        should_skip = False if delay_overflow_check else loss_scaler.update_scale()
        if should_skip:
            loss_scaler._skipped_host = getattr(loss_scaler, "_skipped_host", 0) + 1
            for optimizer in optimizers:
                if not optimizer._amp_stash.already_patched:
                    def patch_step(opt, loss_scaler, loss_id):
                        opt_step = opt.step

                        def skip_step(closure=None):
                            if closure is not None:
                                raise RuntimeError("Currently, Amp does not support closure use "
                                                   "with optimizers.")
                            maybe_print(("Gradient overflow.  Skipping step, loss scaler "
                                         "{} reducing loss scale to {}").format(
                                             loss_id, loss_scaler.loss_scale()))
                            if hasattr(opt._amp_stash, "all_fp32_from_fp16_params"):
                                for param in opt._amp_stash.all_fp32_from_fp16_params:
                                    param.grad = None
                            if hasattr(opt, "most_recent_scale"):
                                opt.most_recent_scale = 1.0
                                opt.scale_set_by_backward = False
                            opt.step = opt_step
                            opt._amp_stash.already_patched = False
                        return skip_step

                    optimizer.step = patch_step(optimizer, loss_scaler, loss_id)
                    optimizer._amp_stash.already_patched = True

    if _amp_state.opt_properties.patch_torch_functions:
        _amp_state.handle._clear_cache()


@contextlib.contextmanager
def disable_casts():
    """Run a region without O1 autocasting (apex.amp.disable_casts)."""
    handle = getattr(_amp_state, "handle", None)
    if handle is None:
        yield
        return
    with handle._disable_casts():
        yield


class AmpHandle(object):
    """O1 handle: owns the autocast state (see amp.amp.init)."""

    def __init__(self, loss_scale="dynamic", enable_caching=True, verbose=False,
                 dtype=torch.float16, device_type="cuda"):
        self._enable_caching = enable_caching
        self._verbose = verbose
        self._dtype = dtype
        self._device_type = device_type
        self._is_active = True
        self._default_scaler = None
        self._loss_scale = loss_scale

    def is_active(self):
        return self._is_active

    @contextlib.contextmanager
    def _disable_casts(self):
        prev = torch.is_autocast_enabled(self._device_type)
        torch.set_autocast_enabled(self._device_type, False)
        try:
            yield
        finally:
            torch.set_autocast_enabled(self._device_type, prev)

    def wrap_optimizer(self, optimizer, num_loss=1):
        warnings.warn("AmpHandle.wrap_optimizer is deprecated; use amp.initialize")
        return optimizer

    @contextlib.contextmanager
    def scale_loss(self, loss, optimizer):
        raise RuntimeError("The old Amp API is no longer supported.  Please move to the new API, "
                           "documented here:  https://nvidia.github.io/apex/amp.html.  Transition "
                           "guide:  https://nvidia.github.io/apex/amp.html#transition-guide-for-"
                           "old-api-users")

    def _clear_cache(self):
        torch.clear_autocast_cache()

    def _deactivate(self):
        self._is_active = False
        torch.set_autocast_enabled(self._device_type, False)

    @property
    def has_cache(self):
        return self._enable_caching

    @property
    def verbose(self):
        return self._verbose


class NoOpHandle(object):
    def is_active(self):
        return False

    @contextlib.contextmanager
    def _disable_casts(self):
        yield

    def wrap_optimizer(self, optimizer, num_loss=1):
        return optimizer

    @contextlib.contextmanager
    def scale_loss(self, loss, optimizer):
        yield loss

    @property
    def has_cache(self):
        return False

    @property
    def verbose(self):
        return False

    def _clear_cache(self):
        pass

    def _deactivate(self):
        pass
