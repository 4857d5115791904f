"""Parallelism: 5-D mesh, DP (arenas + buckets), TP/SP, PP (AFAB/1F1B), CP (ring), EP (MoE all-to-all)."""
from .mesh import (ProcessGroupManager, get_process_group_manager, pgm, process_group_manager,
                   reset_process_group_manager, setup_process_group_manager)

__all__ = ["ProcessGroupManager", "get_process_group_manager", "pgm", "process_group_manager",
           "reset_process_group_manager", "setup_process_group_manager"]
