"""Automatic mixed precision (apex.amp API) for MI355X.

    model, optimizer = amp.initialize(model, optimizer, opt_level="O2")
    with amp.scale_loss(loss, optimizer) as scaled_loss:
        scaled_loss.backward()
    optimizer.step()

See frontend.py for the opt-level table and the checkpoint format.
"""
from ._amp_state import master_params, _amp_state  # noqa: F401
from .amp import (  # noqa: F401
    float_function,
    half_function,
    init,
    promote_function,
    register_float_function,
    register_half_function,
    register_promote_function,
)
from .frontend import initialize, load_state_dict, opt_levels, state_dict  # noqa: F401
from .handle import disable_casts, scale_loss  # noqa: F401
