"""Which learner op breaks HIP graph capture? Run one variant per process: python tools/diag_capture.py <name>."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from marl_range_flocking_amd.learners.core import GradNorm, capture_graph, gru_cell  # noqa: E402

dev = torch.device("cuda", 0)
A, B, H = 3, 6, 32
x = torch.randn(A, B, H, device=dev)
h0 = torch.randn(A, B, H, device=dev)
W = [torch.randn(A, 96, H, device=dev, requires_grad=True) for _ in range(2)]
b = [torch.randn(A, 96, device=dev, requires_grad=True) for _ in range(2)]
g = torch.randn(1000, device=dev)
norm = GradNorm(dev)


def gru_fwd():
    with torch.no_grad():
        gru_cell(x, h0, W[0], W[1], b[0], b[1])


def gru_fwdbwd():
    out = gru_cell(x, h0, W[0], W[1], b[0], b[1])
    torch.autograd.backward(out.sum(), inputs=W + b)


def gradnorm():
    norm(g, 5.0)


def vdn(recurrent=True, chunk=10, eager_first=True, fwd_check=False, nograd=False, drop=False):
    from marl_range_flocking_amd.learners.vdn import VDNLearner

    L = VDNLearner(3, 4, 4, batch_size=6, chunk_size=chunk, update_iter=1, recurrent=recurrent, device=dev,
                   use_graph=False)
    if fwd_check:
        with torch.set_grad_enabled(not nograd):
            qo, ho = L.q(torch.rand(5, 3, 4, device=dev), torch.rand(5, 3, 32, device=dev))
        if not drop:
            globals()["keep"] = (qo, ho)
    for t in range(40):
        L.put(torch.rand(3, 4), torch.randint(0, 4, (3,)), torch.rand(3), torch.rand(3, 4), [t % 7 == 0])
    if eager_first:
        L.train()
    else:
        L.static_idx.copy_(torch.arange(10, device=dev)[None].repeat(6, 1))
    return L._iteration


variants = {"gru_fwd": lambda: gru_fwd, "gru_fwdbwd": lambda: gru_fwdbwd, "gradnorm": lambda: gradnorm,
            "vdn": lambda: vdn(), "vdn_norec": lambda: vdn(False), "vdn_c1": lambda: vdn(True, 1),
            "vdn_c2": lambda: vdn(True, 2), "vdn_fresh": lambda: vdn(eager_first=False),
            "vdn_fwd": lambda: vdn(fwd_check=True), "vdn_fwd_nograd": lambda: vdn(fwd_check=True, nograd=True),
            "vdn_fwd_drop": lambda: vdn(fwd_check=True, drop=True), "vdn_fresh_fwd": lambda: vdn(eager_first=False, fwd_check=True)}
fn = variants[sys.argv[1]]()
gr = capture_graph(fn, dev, [])
gr.replay()
torch.cuda.synchronize()
print("ok", sys.argv[1])
