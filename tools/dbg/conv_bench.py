import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "mvml-mpi_amd"), ROOT]
import torch
from mvml_gat._lib import call, lib, ptr, ws_ptr_size
B, W = 65536, 384
x = torch.randn(B, 12, 3, W, device="cuda"); w = torch.randn(12, 12, 3, 3, device="cuda"); b = torch.randn(12, device="cuda")
y = torch.empty(B, 12, W - 2, device="cuda"); gy = torch.randn_like(y)
gx, gw, gb = torch.empty_like(x), torch.empty_like(w), torch.empty_like(b)
st = torch.cuda.current_stream().cuda_stream
wp, wn = ws_ptr_size(lib().mvml_conv3_bwd_workspace_size(B), "cuda")
f = lambda: call("mvml_conv3_fwd", B, 12, 12, W, ptr(x), ptr(w), ptr(b), ptr(y), st)
g = lambda: call("mvml_conv3_bwd", B, 12, 12, W, ptr(x), ptr(w), ptr(y), ptr(gy), ptr(gx), ptr(gw), ptr(gb), wp, wn, st)
for name, fn in (("fwd", f), ("bwd", g)):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5): fn()
    e.record(); torch.cuda.synchronize()
    print(os.environ.get("MVML_GAT_LIB", "main")[-12:], name, f"{s.elapsed_time(e) / 5:.3f} ms")
