"""No kernel reads an output element before writing it, or workspace it did not write in the
same call: outputs and workspace served from memory that holds NaN (the caching allocator hands
back the blocks just freed) give the results of a clean run bit for bit, on every path.  In a
benchmark loop over one input such a read would go unnoticed (the stale bytes are the previous
call's identical results); a graph replay on new data, or a fresh allocation, would expose it."""
import pytest
import torch

import problems as P
from test_gpu_parity import make_net

pytestmark = pytest.mark.gpu


def poison(shapes, ws_bytes):
    """Allocate-fill-free blocks of the output shapes and of a workspace-sized buffer."""
    ts = [torch.full(s, float("nan"), device="cuda") for s in shapes]
    ts.append(torch.full((ws_bytes // 4 + 1,), float("nan"), device="cuda"))
    torch.cuda.synchronize()
    del ts


@pytest.mark.parametrize("path", ["fused", "layered", "f32_split", "bf16"])
def test_outputs_from_poisoned_memory(path, dl, flags):
    m, n, B, K = 256, 512, 640, 6
    inp = P.make_inputs(m, n, B, 7301)
    inp2 = P.make_inputs(m, n, B, 7302)
    sd = P.make_state_dict("v4", m, n, B, K, inp["A"], 7301, perturb=0.1)
    if path == "layered":
        flags.set(per_layer=True)
    net = make_net(dl, "v4", inp, sd, K).cuda()
    if path in ("f32_split", "bf16"):
        net.precision = path
    kw = dict(keep_all=True, loss_kind=dl._lib.LOSS_L1L1)
    x1 = torch.from_numpy(inp["X"]).cuda()
    x2 = torch.from_numpy(inp2["X"]).cuda()
    with torch.no_grad():
        ref = net.run(x1, **kw)
        ref = {nm: getattr(ref, nm).clone() for nm in ("Z", "E", "L", "T", "loss_sums")}
        net.run(x2, **kw)  # leave the other input's results in the freed blocks
        shapes = [(K, n, B), (K, m, B), (K, m, B), (K + 1, m, B)]
        for trial in range(2):
            if trial == 1:
                dl.ops._WS.clear()  # fresh workspace too
                poison(shapes, 64 << 20)
            got = net.run(x1, **kw)
            torch.cuda.synchronize()
            for nm, r in ref.items():
                assert torch.equal(getattr(got, nm), r), f"{path} trial {trial}: {nm} differs"
            del got
