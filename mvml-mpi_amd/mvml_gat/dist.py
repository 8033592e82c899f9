"""Data-parallel helpers: shard GraphNorm groups over ranks, one flat gradient all-reduce.

The reference is single-device (main.py:121).  Its molecules are independent except inside
GraphNorm's mini-batch (model.py:93), so the unit of sharding is the GraphNorm group (the
reference's 64-molecule batch): each rank owns whole groups, the forward needs no
communication, and training needs exactly one collective per step — an all-reduce of the
flat fp32 gradient buffer (RCCL over xGMI with backend "nccl" on ROCm; gloo on CPU tests).
"""
import numpy as np
import torch
import torch.distributed as dist


def shard_groups(group_costs, world_size, rank):
    """Contiguous partition of groups into `world_size` shards of near-equal total cost
    (cost = edges per group, so skewed batches balance).  Returns (first, last) group index."""
    costs = np.asarray(group_costs, dtype=np.float64)
    G = len(costs)
    if world_size <= 1:
        return 0, G
    cum = np.concatenate([[0.0], np.cumsum(costs)])
    targets = cum[-1] * np.arange(world_size + 1) / world_size
    cuts = np.searchsorted(cum, targets, side="left")
    cuts[0], cuts[-1] = 0, G
    cuts = np.maximum.accumulate(np.clip(cuts, 0, G))
    return int(cuts[rank]), int(cuts[rank + 1])


class EmbeddingAllGather:
    """The final embedding gather of north_star: every rank holds the (B_r, D) view embeddings
    of its own contiguous molecule shard; one all-gather (RCCL over xGMI; gloo on CPU) makes
    the whole (sum_r B_r, D) matrix, in global molecule order, on every rank.

    Shards may differ in size (groups are balanced by edges, not molecules): each rank's rows
    are padded to the largest shard so the collective is a single fixed-size
    all_gather_into_tensor, and the padding is dropped when the result is assembled."""

    def __init__(self, group=None):
        self.group = group

    def __call__(self, emb):
        if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return emb
        world = dist.get_world_size(self.group)
        dev = emb.device
        n = torch.tensor([emb.shape[0]], dtype=torch.int64, device=dev)
        counts = torch.empty(world, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(counts, n, group=self.group)
        counts = counts.cpu().tolist()
        rows = max(counts)
        D = emb.shape[1]
        send = emb.new_zeros((rows, D))
        send[:emb.shape[0]].copy_(emb)
        recv = emb.new_empty((world * rows, D))
        dist.all_gather_into_tensor(recv, send, group=self.group)
        return torch.cat([recv[r * rows:r * rows + c] for r, c in enumerate(counts)], 0)


def launch_local_ranks(nprocs, script, argv, port=None):
    """Start `nprocs` ranks of `script` on this node (one process per GPU) with
    torch.distributed.run as a CHILD process — the caller has not touched the GPU and never
    exec()s — and return the exit code.  Rendezvous on 127.0.0.1 (the container hostname may
    not resolve).  The ranks inherit stdout, so rank 0's output is the caller's output."""
    import socket
    import subprocess
    import sys
    if port is None:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nprocs}",
           "--master-addr=127.0.0.1", f"--master-port={port}", script, *argv]
    return subprocess.call(cmd)


class FlatGradAllReduce:
    """Packs every parameter gradient into one contiguous fp32 buffer and all-reduces it in a
    single call (the view's 6.9 M params = 27.7 MB: latency-, not bandwidth-bound on xGMI,
    so one bucket beats per-tensor collectives).

    Parameters whose ``grad`` is None on EVERY rank stay None, as in the single-device
    reference: torch Adam (main.py:88, weight_decay 1e-4) skips them, so weight decay does not
    move the constructed-but-unused LayerNorms (model.py:42, 120).  The buffer carries one
    presence flag per parameter after the gradients (same collective): a parameter that has a
    gradient on some rank but not on another gets the sum over the ranks that have one (zeros
    elsewhere, DDP's convention); one with no gradient anywhere is left None.  The reduced flags
    (P integers) are read back every step: which parameters the OTHER ranks used can change while
    this rank's own pattern stays the same, and only the reduced flags say so (a cache keyed on
    the local pattern once left such a parameter None here while another rank stepped it).  The
    read-back is one small device-to-host copy after the all-reduce."""

    def __init__(self, params, average=False, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.numel = sum(p.numel() for p in self.params)
        self.average = average
        self.group = group
        self.buf = None
        self.views = None
        self._flags = {}    # local presence pattern -> its flags on the device (built once)

    def _bind(self, dev):
        """One flat buffer; each parameter's gradient becomes a view of its segment, so autograd
        accumulates straight into the buffer (zero_grad(set_to_none=False) zeroes it in place)
        and the all-reduce needs no packing copies."""
        P = len(self.params)
        self.buf = torch.zeros(self.numel + P, dtype=self.params[0].dtype, device=dev)
        self.views, off = [], 0
        for p in self.params:
            n = p.numel()
            self.views.append(self.buf[off:off + n].view_as(p))
            off += n
        self._flags.clear()

    def __call__(self):
        if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return
        dev = self.params[0].device
        if self.buf is None or self.buf.device != dev:
            self._bind(dev)
        local = tuple(p.grad is not None for p in self.params)
        for p, v, has in zip(self.params, self.views, local):
            if not has:
                v.zero_()
            elif p.grad.data_ptr() != v.data_ptr() or p.grad.shape != v.shape:
                v.copy_(p.grad)  # a fresh gradient (first step, or zero_grad(set_to_none=True))
                p.grad = v
        fl = self._flags.get(local)
        if fl is None:
            fl = self._flags[local] = torch.tensor(local, dtype=self.buf.dtype).to(dev)
        self.buf[self.numel:].copy_(fl)  # device to device: no host round trip per step
        dist.all_reduce(self.buf, op=dist.ReduceOp.SUM, group=self.group)
        present = (self.buf[self.numel:] > 0).tolist()  # the GLOBAL pattern of this step
        if self.average:
            self.buf[:self.numel].div_(dist.get_world_size(self.group))
        for p, v, has in zip(self.params, self.views, present):
            if has and p.grad is None:
                p.grad = v  # the sum over the ranks that had one (zeros elsewhere)
