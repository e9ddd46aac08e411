"""Multi-GPU plumbing of the env step: one process per GPU, envs sharded by rank, one collective per
rollout.

The reference runs one env per OS process (SB3 ``SubprocVecEnv``, simulator/CTDECattleHerder.py:91-97)
or per Ray actor (simulator/DTDECattleHerder.py:81) and never communicates between envs.  Here rank r
owns the global env ids ``[r*E, (r+1)*E)`` through ``ch_config.env_id_offset``: Philox actions, reset
draws and spawn scenarios are functions of the global id, so a sharded run produces exactly the
per-env results of a single-process run over all ``world*E`` envs.  The only exchange is the
end-of-rollout metric vector (``ch_metrics``) — an all-reduce(sum) of a few doubles over RCCL/xGMI
(backend "nccl") or gloo on CPU — plus the max-over-ranks wall time the bench reports.
"""
import os
import socket

import numpy as np


def world_info():
    """(rank, world_size, local_rank) from the torchrun environment (1-process defaults)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def env_offset(rank, envs_per_rank):
    """Global id of this rank's env 0 (ch_config.env_id_offset)."""
    return int(rank) * int(envs_per_rank)


def init(backend="nccl", device_index=None):
    """Join the process group when WORLD_SIZE > 1.  ``backend`` "nccl" is RCCL on ROCm."""
    import torch
    import torch.distributed as dist
    rank, world, local = world_info()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dev = local if device_index is None else device_index
            torch.cuda.set_device(dev)
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != world:
            raise RuntimeError(f"process group has {dist.get_world_size()} ranks, WORLD_SIZE says {world}")
    return rank, world, local


def barrier():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def reduce_rollout(metrics, elapsed, device="cpu"):
    """End-of-rollout exchange: metric vector summed over ranks, wall time maxed over ranks.

    ``metrics``: 1-D float64 array / tensor (ch_metrics layout).  Returns (numpy float64 sums, max seconds).
    """
    import torch
    import torch.distributed as dist
    m = torch.as_tensor(np.asarray(metrics, np.float64) if not isinstance(metrics, torch.Tensor) else metrics,
                        dtype=torch.float64).to(device)
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(m)                          # the rollout's only data collective
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return m.cpu().numpy(), float(t.item())


def rank_device_info(use_gpu=True):
    """Which device this rank drives: rank, local rank, device index and, on a GPU, its PCI address and name.
    Without a GPU (the gloo launch check) the device slot is the LOCAL_RANK the rank would bind."""
    rank, world, local = world_info()
    info = {"rank": rank, "local_rank": local, "device": local, "pci_bus_id": None, "name": None,
            "host": socket.gethostname()}
    if use_gpu:
        import torch
        d = torch.cuda.current_device()
        pr = torch.cuda.get_device_properties(d)
        dom, bus, dev = (getattr(pr, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
        info.update(device=int(d), name=str(getattr(pr, "name", "")),
                    pci_bus_id=(f"{int(dom or 0):04x}:{int(bus):02x}:{int(dev or 0):02x}" if bus is not None else None))
    return info


def gather_rank_info(info):
    """Every rank's rank_device_info() on every rank, in rank order (one all_gather_object; [info] alone)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        out = [None] * dist.get_world_size()
        dist.all_gather_object(out, info)
        return out
    return [info]


def distinct_devices(infos):
    """True when no two ranks drive the same device: PCI addresses when known (a launcher that narrows each rank's
    visible devices makes every rank's index 0), else the device slot; either keyed by host, so ranks on two nodes
    with the same PCI layout are distinct."""
    keys = [(i.get("host"), i["pci_bus_id"] if i.get("pci_bus_id") else ("slot", i["device"])) for i in infos]
    return len(set(keys)) == len(keys)


def shutdown():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
