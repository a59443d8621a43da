"""Rank / node helpers (lddl/torch/utils.py:28-94)."""
import torch


def _dist_on():
    return torch.distributed.is_available() and torch.distributed.is_initialized()


def barrier():
    if _dist_on():
        torch.distributed.barrier()


def get_rank():
    return torch.distributed.get_rank() if _dist_on() else 0


def get_world_size():
    return torch.distributed.get_world_size() if _dist_on() else 1


def get_nproc_per_node(local_rank):
    """max(local_rank) + 1 over the world (all_reduce MAX, on the GPU under RCCL)."""
    if not _dist_on():
        return 1
    dev = 'cuda' if torch.distributed.get_backend() == 'nccl' else 'cpu'
    t = torch.tensor(local_rank, device=dev)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return int(t.item()) + 1


def get_num_nodes(local_rank=None, nproc_per_node=None):
    if not _dist_on():
        return 1
    if nproc_per_node is None:
        nproc_per_node = get_nproc_per_node(local_rank)
    return get_world_size() // nproc_per_node


def get_node_rank(local_rank=None, nproc_per_node=None):
    if not _dist_on():
        return 0
    if nproc_per_node is None:
        nproc_per_node = get_nproc_per_node(local_rank)
    return get_rank() // nproc_per_node
