"""The forward under HIP graph capture (torch.cuda.graph): a captured forward replayed on new
input data equals the eager forward on that data bit for bit, on every kernel path -- the fused
kernel, the per-layer kernel pairs (2K+1 launches: the launch-bound case a graph replays without
host work), the split-f16 kernel and the bf16 tiles.  Capture needs the C ABI to enqueue only
stream-ordered work on the caller's stream (no host synchronisation, no allocation of its own:
outputs and workspace come from torch, which serves them from the graph's pool)."""
import numpy as np
import pytest
import torch

import problems as P
from test_gpu_parity import make_net

pytestmark = pytest.mark.gpu


def capture(net, x_static, **run_kw):
    """Warm up on a side stream (torch's capture recipe), then capture one forward."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.no_grad():
        for _ in range(2):
            net.run(x_static, **run_kw)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g), torch.no_grad():
        out = net.run(x_static, **run_kw)
    return g, out


@pytest.mark.parametrize("path", ["fused", "layered", "f32_split", "bf16"])
def test_graph_replay_equals_eager(path, dl, flags):
    m, n, B, K = 256, 512, 640, 6
    inp = P.make_inputs(m, n, B, 7101)
    inp2 = P.make_inputs(m, n, B, 7102)
    sd = P.make_state_dict("v4", m, n, B, K, inp["A"], 7101, perturb=0.1)
    if path == "layered":
        flags.set(per_layer=True)
    net = make_net(dl, "v4", inp, sd, K).cuda()
    if path in ("f32_split", "bf16"):
        net.precision = path
    kw = dict(keep_all=True, loss_kind=dl._lib.LOSS_L1L1)
    x = torch.from_numpy(inp["X"]).cuda()
    g, out = capture(net, x, **kw)
    for data in (inp2["X"], inp["X"]):
        x.copy_(torch.from_numpy(data).cuda())
        g.replay()
        torch.cuda.synchronize()
        with torch.no_grad():
            ref = net.run(torch.from_numpy(data).cuda(), **kw)
        for nm in ("Z", "E", "L", "T", "loss_sums"):
            a, b = getattr(out, nm), getattr(ref, nm)
            assert torch.equal(a, b), f"{path}: {nm} of the replayed graph differs from eager"
    # the two inputs give different results (the replay did read the new data)
    x.copy_(torch.from_numpy(inp2["X"]).cuda())
    g.replay()
    torch.cuda.synchronize()
    z2 = out.Z.clone()
    x.copy_(torch.from_numpy(inp["X"]).cuda())
    g.replay()
    torch.cuda.synchronize()
    assert not torch.equal(z2, out.Z)


@pytest.mark.parametrize("K", [5, 70])
def test_graph_replay_v1_beta_tables(K, dl):
    """V1 (main_lena.py:57-98): the fused kernel reads its per-layer per-sample beta pointers from
    a device table the library writes per call.  The table is written by a kernel
    whose arguments carry the pointers, so a captured forward replays with them after the host
    arrays of the call are gone; K = 70 writes it in two chunks.  The replays equal eager
    forwards bit for bit, including after the parameters are updated in place."""
    m, n, B = 64, 256, 192
    inp = P.make_inputs(m, n, B, 7301)
    inp2 = P.make_inputs(m, n, B, 7302)
    sd = P.make_state_dict("v1", m, n, B, K, inp["A"], 7301, perturb=0.1, wscale=0.4)
    net = make_net(dl, "v1", inp, sd, K).cuda()
    kw = dict(keep_all=True, loss_kind=dl._lib.LOSS_L1L1)
    x = torch.from_numpy(inp["X"]).cuda()
    g, out = capture(net, x, **kw)
    import gc
    gc.collect()
    for step, data in enumerate((inp2["X"], inp["X"])):
        if step == 1:
            with torch.no_grad():   # in place: the graph reads the same parameter storage
                for p in net.beta1:
                    p.mul_(0.9)
        x.copy_(torch.from_numpy(data).cuda())
        g.replay()
        torch.cuda.synchronize()
        with torch.no_grad():
            ref = net.run(torch.from_numpy(data).cuda(), **kw)
        for nm in ("Z", "E", "L", "T", "loss_sums"):
            a, b = getattr(out, nm), getattr(ref, nm)
            if b is None:
                continue
            assert torch.equal(a, b), f"V1 K={K}: {nm} of the replayed graph differs from eager"


def test_graph_replay_launch_heavy_path(dl, flags):
    """The per-layer path at a launch-heavy depth (V6, K = 40: 81 launches) replays from a graph
    with the eager results (timing is not asserted: on a shared box it is noise-bound)."""
    flags.set(per_layer=True)
    m, n, B, K = 64, 256, 64, 40
    inp = P.make_inputs(m, n, B, 7201)
    sd = P.make_state_dict("v6", m, n, B, K, inp["A"], 7201, perturb=0.1)
    net = make_net(dl, "v6", inp, sd, K).cuda()
    kw = dict(keep_all=True, loss_kind=dl._lib.LOSS_LASSO)
    x = torch.from_numpy(inp["X"]).cuda()
    g, out = capture(net, x, **kw)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    with torch.no_grad():
        ref = net.run(x, **kw)
    for nm in ("Z", "E", "L", "T", "loss_sums"):
        assert torch.equal(getattr(out, nm), getattr(ref, nm)), nm


def test_graph_training_step(dl):
    """forward + fused training objective + backward captured as one graph (torch's whole-network
    recipe: warm up on a side stream, capture with static input and .grad buffers), replayed on
    new data: the gradients and the objective equal an eager step's on the same parameters and
    data bit for bit.  (The eager references run first: an eager step after capture would
    rebind .grad and detach it from the buffers the graph writes.)"""
    from test_gpu_backward import make_train_net
    m, n, B, K = 256, 512, 640, 6
    inp = P.make_inputs(m, n, B, 7401)
    inp2 = P.make_inputs(m, n, B, 7402)
    sd = P.make_state_dict("v4", m, n, B, K, inp["A"], 7401, perturb=0.1)
    net = make_train_net(dl, "v4", inp, sd, K)
    coeffs = [0.6] * (K - 1) + [1.0]

    def step(xx):
        total, _ = net.training_loss(xx, 1e-3, coeffs, "l1l1")
        total.backward()
        return total

    def eager(data):
        net.zero_grad(set_to_none=True)
        tot = step(torch.from_numpy(data).cuda()).detach()
        torch.cuda.synchronize()
        return tot, {k: None if p.grad is None else p.grad.clone()
                     for k, p in net.named_parameters()}

    refs = [eager(inp2["X"]), eager(inp["X"])]
    x = torch.from_numpy(inp["X"]).cuda()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            net.zero_grad(set_to_none=False)
            step(x)
    torch.cuda.current_stream().wait_stream(s)
    net.zero_grad(set_to_none=False)   # the graph accumulates into these .grad buffers
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        static_total = step(x)
    for data, (ref_total, ref) in zip((inp2["X"], inp["X"]), refs):
        x.copy_(torch.from_numpy(data).cuda())
        for p in net.parameters():
            if p.grad is not None:
                p.grad.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(static_total.detach(), ref_total)
        for k, p in net.named_parameters():
            if ref[k] is None:   # outside the objective's graph (the last layer's E/L step)
                assert p.grad is None
                continue
            assert torch.equal(p.grad, ref[k]), f"grad {k} of the replayed step differs"
