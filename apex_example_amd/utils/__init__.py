"""Runtime utilities: distributed launch helpers, seeding, synthetic data,
timing / metrics and profiler ranges."""
from .dist import (  # noqa: F401
    barrier,
    cleanup,
    get_rank,
    get_world_size,
    init_distributed,
    is_main_process,
    local_rank,
)
from .misc import deterministic, set_cuda, set_deterministic, set_seed  # noqa: F401
