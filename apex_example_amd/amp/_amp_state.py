"""Global amp state (apex@f3a960f8 apex/amp/_amp_state.py).

Holds the active opt-level Properties, the loss scalers and the O1 handle.
"""
import os

import torch


class AmpState(object):
    def __init__(self):
        self.hard_override = False
        self.allow_incoming_model_not_fp32 = False
        self.verbosity = 1


_amp_state = AmpState()


def warn_or_err(msg):
    if _amp_state.hard_override:
        print("Warning:  " + msg)
    else:
        raise RuntimeError(msg)


def _rank0():
    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return dist.get_rank() == 0
    except Exception:  # pragma: no cover
        pass
    return int(os.environ.get("RANK", "0")) == 0


def maybe_print(msg, rank0=False):
    if _amp_state.verbosity > 0:
        if rank0:
            if _rank0():
                print(msg)
        else:
            print(msg)


def master_params(optimizer):
    """Generator over the parameters the optimizer updates (fp32 masters under
    O2), as ``apex.amp.master_params``.

    Folded-unscale mode (amp O1 + a fused optimizer built with
    ``materialize_master_grads=False``) leaves the grads loss-scaled after
    ``scale_loss`` exits - the optimizer kernel divides by the scale itself.  Asking
    for the master params is what Apex code does before touching grads
    (``clip_grad_norm_(amp.master_params(opt), max_norm)``), so a pending scale is
    removed here, in place and once, and the step then runs on unscaled grads.
    (Under O2 that mode keeps no fp32 master grads at all; clip with the default
    ``materialize_master_grads=True``.)"""
    stash = getattr(optimizer, "_amp_stash", None)
    if stash is not None and getattr(stash, "grads_scaled", False):
        from ._process_optimizer import _unscale_pending

        _unscale_pending(optimizer)
    for group in optimizer.param_groups:
        for p in group["params"]:
            yield p


def is_half_dtype(dt):
    return dt in (torch.float16, torch.bfloat16)
