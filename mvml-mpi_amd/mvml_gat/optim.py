"""main.py:88's optimizer step (torch.optim.Adam(model.parameters(), lr, weight_decay)) as HIP
kernels over flat buffers, with the data-parallel gradient all-reduce folded in.

FlatAdam re-homes every parameter into one flat fp32 buffer (p.data becomes a view of it, so the
modules, their state_dict and the HIP ops see the same tensors) and keeps Adam's exp_avg /
exp_avg_sq flat beside it.  A step is

  1. mvml_grad_gather: this step's gradient tensors -> one flat buffer [grads | presence flags]
     (one launch; the pointer table goes up by a non-blocking copy from pinned memory);
  2. world > 1: ONE all-reduce of that buffer (RCCL over xGMI; gloo on CPU tests) — the
     gradients summed, the presence flags summed with them;
  3. mvml_adam_flat: torch's Adam arithmetic for every parameter whose flag is > 0, the mean
     over ranks taken inside the kernel (grad_scale = 1 / world).

Like the reference's optimizer.zero_grad() (set_to_none), gradients are None between steps, so
autograd hands each parameter its gradient tensor without an accumulate kernel, and a parameter
no rank used (the never-used LayerNorms, model.py:42, 120) keeps its value and its Adam state
exactly as torch's Adam leaves it — decided on the device, with no host read-back.
"""
import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from ._lib import call, ptr

_CHUNK = 16384  # elements per workgroup of the gather / update kernels


def _stream(dev):
    import ctypes
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


class FlatAdam(torch.optim.Optimizer):
    """torch.optim.Adam(params, lr, betas, eps, weight_decay) (amsgrad off, L2 decay) on flat
    buffers; ``group``: the process group whose ranks' gradients are averaged (None: the default
    group when torch.distributed is initialised with more than one rank).  A torch Optimizer with
    one parameter group, so main.py's uses work unchanged: ``optimizer.param_groups[0]["lr"]``
    (main.py:23) and ``torch.optim.lr_scheduler.ExponentialLR(optimizer, gamma)`` (main.py:89)
    — every step reads the group's current lr, betas, eps and weight_decay; ``state_dict()`` is
    torch Adam's layout (per-parameter step / exp_avg / exp_avg_sq)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, group=None,
                 average=True):
        params = list(params)
        if params and isinstance(params[0], dict):
            raise ValueError("FlatAdam: one parameter group (main.py:88 passes model.parameters())")
        self._flat_ready = False
        super().__init__([p for p in params if p.requires_grad],
                         dict(lr=float(lr), betas=tuple(betas), eps=float(eps), weight_decay=float(weight_decay)))
        self.params = list(self.param_groups[0]["params"])
        if not self.params:
            raise ValueError("FlatAdam: no parameters")
        dev = self.params[0].device
        if dev.type != "cuda" or any(p.device != dev or p.dtype != torch.float32 for p in self.params):
            raise ValueError("FlatAdam: fp32 parameters on one GPU")
        self.group, self.average = group, average
        P = len(self.params)
        sizes = [p.numel() for p in self.params]
        offs, off = [], 0
        for n in sizes:  # every segment starts 16-B aligned
            offs.append(off)
            off += (n + 3) // 4 * 4
        self.numel = off
        self.pbuf = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        self.gbuf = torch.zeros(self.numel + P, dtype=torch.float32, device=dev)  # grads | flags
        self.exp_avg = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        self.steps = torch.zeros(P, dtype=torch.int32, device=dev)
        with torch.no_grad():
            for p, o, n in zip(self.params, offs, sizes):
                self.pbuf[o:o + n].copy_(p.detach().reshape(-1))
                p.data = self.pbuf[o:o + n].view_as(p)
        cp, cb, ce = [], [], []
        for i, (o, n) in enumerate(zip(offs, sizes)):
            for b in range(o, o + max(n, 1), _CHUNK):
                cp.append(i)
                cb.append(b)
                ce.append(min(o + n, b + _CHUNK))
        self.nchunks = len(cp)
        self.chunk_param = torch.tensor(cp, dtype=torch.int32, device=dev)
        self.chunk_beg = torch.tensor(cb, dtype=torch.int64, device=dev)
        self.chunk_end = torch.tensor(ce, dtype=torch.int64, device=dev)
        self.param_off = torch.tensor(offs, dtype=torch.int64, device=dev)
        # pointer table: two pinned host buffers in turn (the copy out of one may still be queued
        # while the next step fills the other), one device table
        self._host = [torch.zeros(P, dtype=torch.int64).pin_memory() for _ in range(2)]
        self._host_ev = [None, None]
        self._turn = 0
        self._dev_tab = torch.zeros(P, dtype=torch.int64, device=dev)
        self.allreduce_events = []  # (start, end) HIP events around each step's all-reduce
        self._flat_ready = True

    def add_param_group(self, param_group):
        if self._flat_ready:  # (the flat buffers are laid out once, at construction)
            raise NotImplementedError("FlatAdam: one parameter group, fixed at construction")
        super().add_param_group(param_group)

    def zero_grad(self, set_to_none=True):
        """Gradients back to None (the reference's optimizer.zero_grad()); set_to_none=False is
        accepted and does the same: the gradients are gathered, not accumulated in place."""
        for p in self.params:
            p.grad = None

    def _world(self):
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(self.group)
        return 1

    def step(self, closure=None):
        """One Adam step over every parameter (torch's Optimizer.step contract: an optional
        closure re-evaluates the loss, which is returned)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._step()
        return loss

    @torch.no_grad()
    def _step(self):
        dev = self.pbuf.device
        st = _stream(dev)
        P = len(self.params)
        h = self._host[self._turn]
        ev = self._host_ev[self._turn]
        if ev is not None:
            ev.synchronize()  # (two steps old: long complete) the copy out of h has run
        tab = h.numpy()
        for i, p in enumerate(self.params):
            g = p.grad
            if g is not None:
                if g.dtype != torch.float32 or g.device != dev or not g.is_contiguous():
                    g = p.grad = g.to(dev, torch.float32).contiguous()
                tab[i] = g.data_ptr()
            else:
                tab[i] = 0
        self._dev_tab.copy_(h, non_blocking=True)
        e = torch.cuda.Event()
        e.record()
        self._host_ev[self._turn] = e
        self._turn ^= 1
        call("mvml_grad_gather", self.nchunks, ptr(self.chunk_param), ptr(self.chunk_beg), ptr(self.chunk_end),
             ptr(self.param_off), ptr(self._dev_tab), P, ptr(self.gbuf), self.numel, st)
        world = self._world()
        if world > 1:
            s, e2 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            dist.all_reduce(self.gbuf, op=dist.ReduceOp.SUM, group=self.group)
            e2.record()
            self.allreduce_events.append((s, e2))
        scale = 1.0 / world if (self.average and world > 1) else 1.0
        hp = self.param_groups[0]  # (an lr scheduler may have changed it since the last step)
        b1, b2 = hp["betas"]
        call("mvml_adam_flat", self.nchunks, ptr(self.chunk_param), ptr(self.chunk_beg), ptr(self.chunk_end),
             ptr(self.gbuf[self.numel:]), ptr(self.steps), P, ptr(self.pbuf), ptr(self.gbuf),
             ptr(self.exp_avg), ptr(self.exp_avg_sq), float(hp["lr"]), float(b1), float(b2), float(hp["eps"]),
             float(hp["weight_decay"]), float(scale), st)

    def allreduce_ms(self, reset=True):
        """Mean duration of the recorded all-reduces (HIP events; synchronises), or None."""
        if not self.allreduce_events:
            return None
        torch.cuda.synchronize()
        ms = [s.elapsed_time(e) for s, e in self.allreduce_events]
        if reset:
            self.allreduce_events = []
        return float(np.mean(ms))

    def state_dict(self):
        """torch.optim.Adam's layout: {"state": {index: {"step", "exp_avg", "exp_avg_sq"}},
        "param_groups": [...]} (parameters never stepped have no entry, as in torch)."""
        steps = self.steps.cpu().tolist()
        state = {}
        for i, p in enumerate(self.params):
            if steps[i] > 0:
                _, m, v = self.state_of(p)
                state[i] = {"step": torch.tensor(float(steps[i])), "exp_avg": m.clone(),
                            "exp_avg_sq": v.clone()}
        groups = [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups]
        groups[0]["params"] = list(range(len(self.params)))
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        g = sd["param_groups"][0]
        if len(sd["param_groups"]) != 1 or len(g["params"]) != len(self.params):
            raise ValueError("FlatAdam.load_state_dict: one group with this optimizer's parameters")
        for k, v in g.items():
            if k != "params":
                self.param_groups[0][k] = v
        steps = [0] * len(self.params)
        with torch.no_grad():
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
            for i, p in enumerate(self.params):
                st = sd["state"].get(i, sd["state"].get(str(i)))
                if st:
                    steps[i] = int(float(st["step"]))
                    _, m, v = self.state_of(p)
                    m.copy_(st["exp_avg"].reshape(m.shape))
                    v.copy_(st["exp_avg_sq"].reshape(v.shape))
        self.steps.copy_(torch.tensor(steps, dtype=torch.int32))

    def state_of(self, p):
        """(step, exp_avg, exp_avg_sq) of parameter p, shaped like it (tests)."""
        i = next(j for j, q in enumerate(self.params) if q is p)
        o = int(self.param_off[i])
        n = p.numel()
        return (int(self.steps[i]), self.exp_avg[o:o + n].view_as(p), self.exp_avg_sq[o:o + n].view_as(p))
