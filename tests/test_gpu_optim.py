"""FlatAdam (mvml_gat.optim: main.py:88's torch.optim.Adam as HIP kernels over flat buffers,
the per-parameter "has a gradient" decision on the device) against torch.optim.Adam.

  * one process: parameters of several shapes (odd sizes: segments padded to 16 B), one that
    never gets a gradient (the reference's unused LayerNorms, model.py:42 / 120: torch skips
    it, so it and its state stay untouched) and one that gets its first gradient at step 2 (its
    own step count, hence its own bias correction) — every parameter within fp32 rounding of
    torch's Adam after 4 steps, the step counters equal to torch's;
  * two ranks on the one GPU (gloo over the device buffer): ONE all-reduce of [gradients |
    presence flags], a parameter used by rank 1 only is stepped on both ranks with the mean
    gradient, one used by no rank is skipped on both, and no host read-back of the flags.
"""
import json
import os
import socket
import subprocess
import sys
import textwrap

import pytest
import torch

from mvml_gat.optim import FlatAdam

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(7, 5), (384,), (1928, 76), (3,), (17,), (2, 3, 5)]
    return [torch.nn.Parameter(torch.randn(s, generator=g)) for s in shapes]


def test_flat_adam_matches_torch():
    ref = _params(0)
    mine = [torch.nn.Parameter(p.detach().clone().to(DEV)) for p in ref]
    ref = [torch.nn.Parameter(p.detach().clone().to(DEV)) for p in ref]
    topt = torch.optim.Adam(ref, lr=1e-3, weight_decay=1e-4, foreach=False)
    fopt = FlatAdam(mine, lr=1e-3, weight_decay=1e-4)
    g = torch.Generator().manual_seed(1)
    for step in range(4):
        topt.zero_grad()
        fopt.zero_grad()
        for i, (a, b) in enumerate(zip(ref, mine)):
            if i == 3:  # never used: grad stays None
                continue
            if i == 4 and step < 2:  # first used at step 2
                continue
            gr = (torch.randn(a.shape, generator=g) * (10.0 ** (i - 2))).to(DEV)
            a.grad = gr.clone()
            b.grad = gr.clone()
        topt.step()
        fopt.step()
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(ref, mine)):
        d = (a.detach() - b.detach()).abs().max().item()
        scale = a.detach().abs().max().item()
        assert d <= 2e-6 * max(scale, 1e-3), (i, d, scale)
        st = topt.state.get(a, {})
        n = int(st["step"]) if st else 0
        step_i, m, v = fopt.state_of(b)
        assert step_i == n, (i, step_i, n)
        if n:
            # (exp_avg's small entries are differences g - m: fp32 rounding relative to the
            # tensor's scale, not to each entry)
            em, ev = st["exp_avg"], st["exp_avg_sq"]
            assert torch.allclose(m, em, rtol=1e-5, atol=1e-6 * float(em.abs().max())), i
            assert torch.allclose(v, ev, rtol=1e-5, atol=1e-6 * float(ev.abs().max())), i
    # the never-used parameter is bitwise untouched
    assert torch.equal(mine[3].detach().cpu(), _params(0)[3].detach())


def test_flat_adam_params_are_views():
    """The modules keep their Parameter objects; each becomes a view of the flat buffer, so an
    update is visible through the module and its state_dict."""
    lin = torch.nn.Linear(13, 7).to(DEV)
    w0 = lin.weight.detach().clone()
    opt = FlatAdam(lin.parameters(), lr=1e-2)
    assert torch.equal(lin.weight.detach(), w0)
    lin(torch.randn(4, 13, device=DEV)).sum().backward()
    opt.step()
    torch.cuda.synchronize()
    assert not torch.equal(lin.weight.detach(), w0)
    assert lin.weight.data_ptr() == opt.pbuf.data_ptr()
    assert torch.equal(lin.state_dict()["weight"], lin.weight.detach())


_CHILD = textwrap.dedent(r"""
    import json, os, sys
    sys.path[:0] = [os.path.join(os.environ["MVML_ROOT"], "mvml-mpi_amd"), os.environ["MVML_ROOT"]]
    import torch
    import torch.distributed as dist
    from mvml_gat.optim import FlatAdam
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a = torch.nn.Parameter(torch.ones(5, device=dev))
    b = torch.nn.Parameter(torch.ones(3, device=dev))
    c = torch.nn.Parameter(torch.ones(2, device=dev))
    opt = FlatAdam([a, b, c], lr=0.1, weight_decay=0.01, average=True)
    for step in range(2):
        opt.zero_grad()
        loss = (a * (rank + 1)).sum()
        if step == 1 and rank == 1:
            loss = loss + (b * 3).sum()  # b: used by rank 1 only, at step 1; c: by nobody
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    out = {"rank": rank, "a": a.detach().cpu().tolist(), "b": b.detach().cpu().tolist(),
           "c": c.detach().cpu().tolist(), "steps": opt.steps.cpu().tolist()}
    with open(os.environ["MVML_OUT"] + f".{rank}", "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()
""")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_flat_adam_two_ranks_device_presence(tmp_path):
    script = tmp_path / "child.py"
    script.write_text(_CHILD)
    outp = str(tmp_path / "out")
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), MVML_ROOT=ROOT, MVML_OUT=outp)
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env))
    for p in procs:
        assert p.wait(timeout=240) == 0
    res = [json.load(open(f"{outp}.{r}")) for r in range(2)]
    # expected: torch Adam on the rank-mean gradients (zeros where a rank had none)
    a = torch.nn.Parameter(torch.ones(5))
    b = torch.nn.Parameter(torch.ones(3))
    c = torch.nn.Parameter(torch.ones(2))
    opt = torch.optim.Adam([a, b, c], lr=0.1, weight_decay=0.01, foreach=False)
    for step in range(2):
        opt.zero_grad()
        a.grad = torch.full((5,), 1.5)  # (1 + 2) / 2
        if step == 1:
            b.grad = torch.full((3,), 1.5)  # (0 + 3) / 2
        opt.step()
    for r in res:
        assert r["steps"] == [2, 1, 0], r
        assert torch.allclose(torch.tensor(r["a"]), a.detach(), rtol=1e-6), r
        assert torch.allclose(torch.tensor(r["b"]), b.detach(), rtol=1e-6), r
        assert r["c"] == [1.0, 1.0], r
    assert res[0]["a"] == res[1]["a"] and res[0]["b"] == res[1]["b"]


def test_flat_adam_with_exponential_lr_and_state_dict():
    """main.py:88-89 unchanged: ExponentialLR(FlatAdam, 0.95) moves the lr each epoch exactly as
    it moves torch Adam's (param_groups[0]["lr"], main.py:23), and state_dict() is torch Adam's
    layout: loading torch's state into a fresh FlatAdam continues identically."""
    ref = _params(5)
    mine = [torch.nn.Parameter(p.detach().clone().to(DEV)) for p in ref]
    ref = [torch.nn.Parameter(p.detach().clone().to(DEV)) for p in ref]
    topt = torch.optim.Adam(ref, lr=1e-2, weight_decay=1e-4, foreach=False)
    fopt = FlatAdam(mine, lr=1e-2, weight_decay=1e-4)
    tsch = torch.optim.lr_scheduler.ExponentialLR(topt, gamma=0.95)
    fsch = torch.optim.lr_scheduler.ExponentialLR(fopt, gamma=0.95)
    g = torch.Generator().manual_seed(7)
    for epoch in range(3):
        for step in range(2):
            topt.zero_grad()
            fopt.zero_grad()
            for i, (a, b) in enumerate(zip(ref, mine)):
                if i == 3:
                    continue
                gr = torch.randn(a.shape, generator=g).to(DEV)
                a.grad, b.grad = gr.clone(), gr.clone()
            topt.step()
            fopt.step()
        tsch.step()
        fsch.step()
        assert fopt.param_groups[0]["lr"] == topt.param_groups[0]["lr"]
    torch.cuda.synchronize()
    for a, b in zip(ref, mine):
        d = (a.detach() - b.detach()).abs().max().item()
        assert d <= 2e-6 * max(a.detach().abs().max().item(), 1e-3), d
    # torch's state into a fresh FlatAdam over copies of torch's parameters: one more step each
    sd = topt.state_dict()
    steps0 = {i: float(st["step"]) for i, st in sd["state"].items()}  # (sd holds torch's live tensors)
    mine2 = [torch.nn.Parameter(a.detach().clone()) for a in ref]
    f2 = FlatAdam(mine2, lr=1.0)
    f2.load_state_dict(sd)
    assert f2.param_groups[0]["lr"] == topt.param_groups[0]["lr"]
    for a, b in zip(ref, mine2):
        a.grad = torch.ones_like(a)
        b.grad = torch.ones_like(b)
    ref[3].grad = None
    mine2[3].grad = None
    topt.step()
    f2.step()
    torch.cuda.synchronize()
    for a, b in zip(ref, mine2):
        d = (a.detach() - b.detach()).abs().max().item()
        assert d <= 2e-6 * max(a.detach().abs().max().item(), 1e-3), d
    out = f2.state_dict()
    assert sorted(out["state"]) == sorted(sd["state"])
    for i, n in steps0.items():
        assert float(out["state"][i]["step"]) == n + 1
