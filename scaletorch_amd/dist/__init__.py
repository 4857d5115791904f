"""Communication layer: RCCL (torch.distributed 'nccl') on MI355X, gloo on CPU."""
from .collectives import (SINGLE, P2POp, global_rank_of, all_gather, all_gather_object, all_reduce, all_reduce_dict, all_reduce_params,
                          _all_reduce_coalesced, all_to_all, collect_results_cpu, collect_results_gpu,
                          barrier, batch_isend_irecv, broadcast, broadcast_object_list, collect_results,
                          destroy_group, gather, gather_object, get_local_rank, get_local_world_size,
                          get_rank, get_world_size, irecv, is_distributed, is_main_process, isend,
                          new_group, reduce, reduce_op, reduce_scatter, scatter, sync_random_seed)
from .launch import (cleanup_dist, device_backend, get_comm_device, infer_launcher, init_dist,
                     parse_slurm_nodelist)

__all__ = [
    "SINGLE", "global_rank_of", "P2POp", "all_gather", "all_gather_object", "all_reduce", "all_reduce_dict", "all_reduce_params",
    "_all_reduce_coalesced", "collect_results_cpu", "collect_results_gpu", "all_to_all", "barrier",
    "batch_isend_irecv", "broadcast", "broadcast_object_list", "collect_results", "destroy_group", "gather",
    "gather_object", "get_local_rank", "get_local_world_size", "get_rank", "get_world_size", "irecv",
    "is_distributed", "is_main_process", "isend", "new_group", "reduce", "reduce_op", "reduce_scatter",
    "scatter", "sync_random_seed", "cleanup_dist", "device_backend", "get_comm_device", "infer_launcher",
    "init_dist", "parse_slurm_nodelist",
]
