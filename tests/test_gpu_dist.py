"""Data parallelism through the real collectives on the HIP path: two processes (gloo, both on
cuda:0 -- the GPU box has one card; the driver's 8-GPU runs use RCCL the same way), each running
the fused forward / training step on its column shard.

* forward: each rank's objective sums are combined by dist.global_objectives (ONE all-reduce of
  the [K, 2] sums) and equal the whole batch's objective;
* training: training_loss(x_shard, batch=B, cols=...) + backward + dist.allreduce_grads (one
  bucketed all-reduce) gives every rank the whole batch's gradient (INTEGRATION.md recipe).
The whole-batch reference runs in the parent process on the same GPU.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import problems as P

pytestmark = pytest.mark.gpu

VARIANT, M, N, B, K, SEED = "v4", 64, 128, 150, 3, 4343


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _net(dl, inp, sd, bs=B):
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    net = dl.VARIANTS[VARIANT](m=M, n=0, d=N, batch_size=bs, A=t(inp["A"]), Z0=t(inp["Z0"]),
                               E0=t(inp["E0"]), L0=t(inp["L0"]), layers=K)
    net.load_state_dict({k: t(v) for k, v in sd.items()})
    return net


def _worker(rank, world, port, q):
    import importlib
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests", "golden"))
    import problems
    try:
        dl = importlib.import_module("d-ladmm_amd")
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        d = dict(variant=VARIANT, m=M, n=N, B=B, K=K, seed=SEED, perturb=0.1, wscale=None)
        inp, sd = problems.build_problem(d)
        net = _net(dl, inp, sd)
        c0, c1 = dl.dist.shard_columns(B, rank, world)
        X = torch.from_numpy(inp["X"]).cuda()[:, c0:c1]
        # forward objective: this rank's sums -> one all-reduce
        shard = _net(dl, {**inp, "Z0": inp["Z0"][:, c0:c1], "E0": inp["E0"][:, c0:c1],
                          "L0": inp["L0"][:, c0:c1]}, sd, bs=c1 - c0)
        with torch.no_grad():
            r = shard.run(X.contiguous(), keep_all=True, loss_kind=dl._lib.LOSS_L1L1)
        obj = dl.dist.global_objectives(r.loss_sums, P_ALPHA, B).cpu().numpy()
        # training step on the shard, gradients all-reduced
        net.requires_grad_(True)
        tot, _ = net.training_loss(X, P_ALPHA, COEFFS, "l1l1", batch=B, cols=(c0, c1))
        tot.backward()
        dl.dist.allreduce_grads(net)
        grads = {k: (p.grad.cpu().numpy() if p.grad is not None else None)
                 for k, p in net.named_parameters()}
        q.put((rank, obj, grads, None))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, None, None, traceback.format_exc() + repr(e)))


P_ALPHA = 0.001
COEFFS = [0.6, 0.6, 1.0]


@pytest.mark.timeout(300)
def test_two_ranks_gloo_forward_and_training(dl):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    for rank, _, _, err in res:
        assert err is None, f"rank {rank}: {err}"
    for p in ps:
        assert p.exitcode == 0
    # whole batch in this process
    d = dict(variant=VARIANT, m=M, n=N, B=B, K=K, seed=SEED, perturb=0.1, wscale=None)
    inp, sd = P.build_problem(d)
    net = _net(dl, inp, sd)
    X = torch.from_numpy(inp["X"]).cuda()
    with torch.no_grad():
        r = net.run(X, keep_all=True, loss_kind=dl._lib.LOSS_L1L1)
    ref_obj = ((P_ALPHA * r.loss_sums[:, 0] + r.loss_sums[:, 1]) / B).cpu().numpy()
    net.requires_grad_(True)
    tot, _ = net.training_loss(X, P_ALPHA, COEFFS, "l1l1")
    tot.backward()
    for rank, obj, grads, _ in res:
        np.testing.assert_allclose(obj, ref_obj, rtol=1e-6)
        for key, p in net.named_parameters():
            if p.grad is None:
                assert grads[key] is None, key
                continue
            g = p.grad.cpu().numpy().astype(np.float64)
            e = np.linalg.norm(grads[key] - g) / max(np.linalg.norm(g), 1e-30)
            assert e <= 1e-5, (rank, key, e)
    # both ranks hold the same all-reduced gradient
    for key in res[0][2]:
        if res[0][2][key] is not None:
            np.testing.assert_array_equal(res[0][2][key], res[1][2][key])


def test_v1_ctor_shard_device_memory(dl):
    """SURVEY 8(e) at BASELINE config 3's scale: a V1 model (main_lena.py:16-49) over
    B = 262,144 columns, K = 15, built as rank 0 of 8 with batch_shard=(0, 8), holds 1/8 of the
    replicated module's per-sample betas on the device -- the global 2 K m B betas (8 GB) never
    reach the GPU -- and its forward equals the replicated module's on the same columns."""
    m, n, Bg, Kd, world = 256, 512, 262144, 15, 8
    g = torch.Generator().manual_seed(17)
    A = torch.randn(m, n, generator=g)
    A = A / A.pow(2).sum(0, keepdim=True).sqrt()
    Z0 = torch.rand(n, Bg, generator=g) / n
    E0, L0 = torch.zeros(m, Bg), torch.zeros(m, Bg)
    peaks = {}
    for mode in ("replicated", "shard"):
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        torch.manual_seed(5)
        kw = {} if mode == "replicated" else {"batch_shard": (0, world)}
        net = dl.DLADMMNet(m=m, n=0, d=n, batch_size=Bg, A=A, Z0=Z0, E0=E0, L0=L0, layers=Kd,
                           **kw)
        torch.cuda.synchronize()
        peaks[mode] = torch.cuda.max_memory_allocated() - base
        if mode == "replicated":
            net.requires_grad_(False)
            c0, c1 = dl.dist.shard_columns(Bg, 0, world)
            Xs = torch.randn(m, c1 - c0, generator=g).cuda()
            sub = {k: v[:, c0:c1].contiguous() if k.startswith("beta") else v
                   for k, v in net.state_dict().items()}
            del net
        else:
            net.requires_grad_(False)
            shard_net = net
    betas = 2 * Kd * m * Bg * 4
    assert peaks["replicated"] >= betas
    # the shard: its betas and initial state (1/8), the replicated weights (K n m) and A
    small = (Kd + 1) * m * n * 4
    assert peaks["shard"] <= peaks["replicated"] / world + small + (1 << 20), peaks
    # same forward as the replicated parameters restricted to the shard's columns
    torch.manual_seed(5)
    c0, c1, _ = shard_net.batch_shard
    one = dl.DLADMMNet(m=m, n=0, d=n, batch_size=c1 - c0, A=A, Z0=Z0[:, c0:c1].contiguous(),
                       E0=E0[:, c0:c1].contiguous(), L0=L0[:, c0:c1].contiguous(), layers=Kd)
    one.load_state_dict(sub)
    one.requires_grad_(False)
    with torch.no_grad():
        a = shard_net.run(Xs, keep_all=False, loss_kind=1)
        b = one.run(Xs, keep_all=False, loss_kind=1)
    assert torch.equal(a.Z, b.Z) and torch.equal(a.L, b.L)
