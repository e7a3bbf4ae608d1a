"""multi_tensor_applier (apex@f3a960f8 apex/multi_tensor_apply/multi_tensor_apply.py).

Same call shape as Apex: ``multi_tensor_applier(op, noop_flag_buffer,
tensor_lists, *args)`` calls ``op(chunk_size, noop_flag_buffer, tensor_lists,
*args)``.  ``op`` is one of the ``apex_example_amd.amp_C`` functions.

``chunk_size`` is kept for API compatibility (default 2048*32 as in Apex); the
gfx950 engine always tiles work in 8192-element units and a whole tensor list
goes out in ONE launch whose metadata table is cached on the device (see
csrc/include/mt_table.h), so the value does not change results.
"""
from .. import _native


class MultiTensorApply(object):
    available = False
    warned = False

    def __init__(self, chunk_size):
        try:
            MultiTensorApply.available = _native.available()
        except Exception as err:  # pragma: no cover
            MultiTensorApply.available = False
            MultiTensorApply.import_err = err
        self.chunk_size = chunk_size

    def check_avail(self):
        if not MultiTensorApply.available:
            raise RuntimeError(
                "Attempted to call MultiTensorApply method, but MultiTensorApply is not "
                "available, possibly because the native extension was not built "
                "(python tools/build_ext.py).")

    def __call__(self, op, noop_flag_buffer, tensor_lists, *args):
        self.check_avail()
        return op(self.chunk_size, noop_flag_buffer, tensor_lists, *args)


multi_tensor_applier = MultiTensorApply(2048 * 32)
