"""Communicator bootstrap, counterpart of python/DistGNN/dist/communicator.py:5-17.

The first rank of every `group_size` block of global ranks draws an RCCL unique id through
`dgs`, the id travels over the torch.distributed process group, and every member then joins
the library's communicator (used only for setup collectives: IPC handle exchange, cache-list
all-gather, barriers)."""
import torch.distributed as dist

import dgs

__all__ = ["create_communicator"]


def create_communicator(group_size, group=None):
    me = dist.get_rank()
    member = me % group_size
    leader = me - member
    payload = [dgs.ops._CAPI_get_unique_id() if member == 0 else None]
    dist.broadcast_object_list(payload, leader, group)
    dgs.ops._CAPI_set_nccl(group_size, payload[0], member)
