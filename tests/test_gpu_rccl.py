"""RCCL on the GPU box: the collectives the data-parallel path uses (bench.py --gpus N), run
through torch.distributed's "nccl" backend (= RCCL on ROCm) in a child process that also has
libmvml_gat.so loaded and a HIP GNNModule step done — one rank, since the box has one GPU (the
N-rank decomposition itself is covered by tests/test_dist_gloo.py on gloo).

Checks: init_process_group("nccl", device_id=...) as bench.py calls it, one all_reduce of the
flat gradient buffer FlatGradAllReduce builds, all_gather_into_tensor of the (B, 384) embedding
block as EmbeddingAllGather issues it, and a barrier.  HSA_ENABLE_IPC_MODE_LEGACY=0 is kept in
the child's environment (dmabuf IPC, see the task's environment notes)."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = textwrap.dedent(r"""
    import os, sys
    sys.path[:0] = [os.path.join(os.environ["MVML_ROOT"], "mvml-mpi_amd"), os.environ["MVML_ROOT"]]
    import torch
    import torch.distributed as dist
    import mvml_gat
    from mvml_gat import synth
    from mvml_gat.dist import FlatGradAllReduce

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    torch.manual_seed(0)
    sb = synth.config3(256)
    g = sb.to_graph().to(dev)
    model = mvml_gat.GNNModule(74, [192, 384], 0.5, 6, 3).to(dev).train()
    emb = model(g, g.ndata["h"])
    emb.square().mean().backward()
    params = [p for p in model.parameters()]
    red = FlatGradAllReduce(params, average=True)
    flat = torch.cat([p.grad.reshape(-1) for p in params])
    ref = flat.clone()
    dist.all_reduce(flat)                        # the reducer's collective, on its buffer layout
    assert torch.equal(flat, ref), "all_reduce over one rank must be the identity"
    red()                                        # world 1: leaves the gradients alone
    assert torch.equal(torch.cat([p.grad.reshape(-1) for p in params]), ref)
    out = torch.empty_like(emb)
    dist.all_gather_into_tensor(out, emb.detach().contiguous())
    assert torch.equal(out, emb.detach())
    dist.barrier()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print("rccl ok", flat.numel(), tuple(emb.shape))
""")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_rccl_collectives_one_rank():
    env = dict(os.environ)
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", MVML_ROOT=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", _CHILD], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rccl ok" in r.stdout
