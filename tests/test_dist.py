"""N > 1 host logic on CPU with gloo, world_size 2: batch sharding + the one collective.

Each rank runs the oracle (checker) on its column shard, reduces its local objective sums and the
ranks combine them with dist.global_objectives; the result must equal the full-batch objective,
and the shards' outputs must tile the full-batch outputs exactly (columns are independent)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import importlib
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests", "golden"))
    import problems
    from oracle import dladmm_oracle as oracle
    ddist = importlib.import_module("d-ladmm_amd.dist")
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m, n, B, K, alpha = 32, 64, 37, 4, 0.001
    inp = problems.make_inputs(m, n, B, 77)
    sd = problems.make_state_dict("v4", m, n, B, K, inp["A"], 77, perturb=0.1)
    s0, s1 = ddist.shard_columns(B, rank, world)
    cols = slice(s0, s1)
    out = oracle.forward("v4", inp["X"][:, cols], inp["A"], inp["Z0"][:, cols],
                         inp["E0"][:, cols], inp["L0"][:, cols], sd, K)
    sums = torch.zeros(K, 2, dtype=torch.float64)
    for k in range(K):
        Zk = out["Z"][k].astype(np.float64)
        r = inp["X"][:, cols].astype(np.float64) - inp["A"].astype(np.float64) @ Zk
        sums[k, 0] = float(np.abs(Zk).sum())
        sums[k, 1] = float(np.abs(r).sum())
    obj = ddist.global_objectives(sums, alpha, B)
    q.put((rank, (s0, s1), obj.numpy(), [z for z in out["Z"]]))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_shard_and_reduce():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tests", "golden"))
    import problems
    from oracle import dladmm_oracle as oracle
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
        assert p.exitcode == 0
    m, n, B, K, alpha = 32, 64, 37, 4, 0.001
    inp = problems.make_inputs(m, n, B, 77)
    sd = problems.make_state_dict("v4", m, n, B, K, inp["A"], 77, perturb=0.1)
    full = oracle.forward("v4", inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, K)
    ref = oracle.layer_objectives(full["Z"], inp["X"], inp["A"], alpha, "l1l1")
    assert res[0][1] == (0, 19) and res[1][1] == (19, 37)
    for _, _, obj, _ in res:
        np.testing.assert_allclose(obj, ref, rtol=1e-6)
    for k in range(K):
        tiled = np.concatenate([res[0][3][k], res[1][3][k]], axis=1)
        assert oracle.nrel(tiled, full["Z"][k]) <= 1e-6


def test_shard_columns_cover_exactly():
    import importlib
    ddist = importlib.import_module("d-ladmm_amd.dist")
    for total in (1, 7, 64, 65536, 262144):
        for world in (1, 2, 3, 8):
            spans = [ddist.shard_columns(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
                assert a1 == b0
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def _grad_worker(rank, world, port, q):
    import importlib
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    ddist = importlib.import_module("d-ladmm_amd.dist")
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mod = torch.nn.Module()
    mod.w = torch.nn.Parameter(torch.zeros(3, 4))
    mod.b = torch.nn.Parameter(torch.zeros(1, 1))
    mod.w.grad = torch.full((3, 4), float(rank + 1))
    mod.b.grad = torch.full((1, 1), 10.0 * (rank + 1))
    ddist.allreduce_grads(mod)
    q.put((rank, mod.w.grad.clone().numpy(), mod.b.grad.clone().numpy()))
    dist.destroy_process_group()


def test_allreduce_grads_world2():
    """The data-parallel training helper: one bucketed all-reduce of every parameter grad."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_grad_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
    for _, w, b in res:
        np.testing.assert_array_equal(w, np.full((3, 4), 3.0))
        np.testing.assert_array_equal(b, np.full((1, 1), 30.0))


def _strong_worker(rank, world, port, q):
    """bench.py's strong-scaling plumbing on one rank: its dist.shard_columns span of the global
    batch (synth(..., cols=...)), the shard's objective sums (oracle), the ONE all-reduce
    (global_objectives) and the max-over-ranks timing reduction (reduce_timing)."""
    import importlib
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests", "golden"))
    import bench
    import problems
    from oracle import dladmm_oracle as oracle
    ddist = importlib.import_module("d-ladmm_amd.dist")
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m, n, Bg, K, alpha = 24, 48, 41, 3, 0.001
    c0, c1 = ddist.shard_columns(Bg, rank, world)
    A, X, Z0, E0, L0 = (t.numpy() for t in bench.synth(m, n, Bg, 0, "cpu", (c0, c1)))
    sd = problems.make_state_dict("v4", m, n, 1, K, A, 5, perturb=0.1)
    out = oracle.forward("v4", X, A, Z0, E0, L0, sd, K)
    sums = torch.zeros(K, 2, dtype=torch.float64)
    for k in range(K):
        Zk = out["Z"][k].astype(np.float64)
        sums[k, 0] = float(np.abs(Zk).sum())
        sums[k, 1] = float(np.abs(X.astype(np.float64) - A.astype(np.float64) @ Zk).sum())
    obj = ddist.global_objectives(sums, alpha, Bg)
    el, kern, kerns = bench.reduce_timing(1.0 + rank, 0.5 * (rank + 1), world, "cpu")
    q.put((rank, (c0, c1), obj.numpy(), (el, kern, kerns)))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_strong_scaling_plumbing():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests", "golden"))
    import bench
    import problems
    from oracle import dladmm_oracle as oracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_strong_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    m, n, Bg, K, alpha = 24, 48, 41, 3, 0.001
    A, X, Z0, E0, L0 = (t.numpy() for t in bench.synth(m, n, Bg, 0, "cpu"))
    sd = problems.make_state_dict("v4", m, n, 1, K, A, 5, perturb=0.1)
    full = oracle.forward("v4", X, A, Z0, E0, L0, sd, K)
    ref = oracle.layer_objectives(full["Z"], X, A, alpha, "l1l1")
    assert [r[1] for r in res] == [(0, 21), (21, 41)]   # the two spans tile the global batch
    for _, _, obj, (el, kern, kerns) in res:
        np.testing.assert_allclose(obj, ref, rtol=1e-6)  # every rank sees the global objective
        assert (el, kern) == (2.0, 1.0) and kerns == [0.5, 1.0]   # max over ranks; rank order


def test_bench_synth_shard_is_global_slice():
    """Strong scaling generates the same global batch on every rank and keeps its columns: a
    shard equals the columns of the whole batch."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    full = bench.synth(16, 32, 50, 0, "cpu")
    part = bench.synth(16, 32, 50, 0, "cpu", (13, 29))
    assert torch.equal(full[0], part[0])
    for f, p in zip(full[1:], part[1:]):
        assert torch.equal(f[:, 13:29], p)


def _v1_shard_worker(rank, world, port, q):
    """A V1 model made a batch shard (shard_batch_): betas hold the rank's columns, a global
    checkpoint loads sliced, allreduce_grads leaves the rank-local beta gradients out of the
    bucket, gather_state_dict restores the reference layout."""
    import importlib
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    dl = importlib.import_module("d-ladmm_amd")
    ddist = importlib.import_module("d-ladmm_amd.dist")
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m, n, B, K = 8, 16, 11, 3
    g = torch.Generator().manual_seed(5)
    A = torch.randn(m, n, generator=g)
    mk = lambda: dl.DLADMMNet(m=m, n=0, d=n, batch_size=B, A=A,  # noqa: E731
                              Z0=torch.rand(n, B, generator=g), E0=torch.zeros(m, B),
                              L0=torch.zeros(m, B), layers=K)
    torch.manual_seed(7)
    full = mk()
    sd_full = {k: torch.randn(v.shape, generator=g) for k, v in full.state_dict().items()}
    full.load_state_dict(sd_full)
    net = mk()
    net.shard_batch_(rank, world)
    net.load_state_dict(sd_full)            # the global checkpoint, sliced on load
    c0, c1, Bg = net.batch_shard
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    # gradients: betas rank-local (their value = rank id), weights replicated (summed)
    for p in net.parameters():
        p.grad = torch.full_like(p, float(rank + 1))
    ddist.allreduce_grads(net)
    gb = float(net.beta1[0].grad.mean())
    gw = float(net.fc[0].weight.grad.mean())
    gathered = ddist.gather_state_dict(net)
    same = all(torch.equal(gathered[k], sd_full[k]) for k in sd_full)
    q.put((rank, (c0, c1, Bg), shapes, gb, gw, same, tuple(net.Z0.shape)))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_v1_beta_shard():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_v1_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    m, n, B, K = 8, 16, 11, 3
    assert [r[1] for r in res] == [(0, 6, 11), (6, 11, 11)]
    for rank, (c0, c1, _), shapes, gb, gw, same, z0 in res:
        for k in range(K):
            assert shapes[f"beta1.{k}"] == (m, c1 - c0) == shapes[f"beta2.{k}"]
            assert shapes[f"fc.{k}.weight"] == (n, m)
        assert z0 == (n, c1 - c0)
        assert gb == rank + 1.0      # not all-reduced: rank-local
        assert gw == 3.0             # all-reduced: 1 + 2
        assert same                  # gathered state_dict == the global checkpoint


def _v1_ctor_shard_worker(rank, world, port, q):
    """A V1 shard built by the constructor (batch_shard=(rank, world)): the betas never exist
    at the global width; a DEEP COPY of the shard still keeps its betas out of the all-reduce
    (rank-local parameters are found from the module, not from a Parameter attribute); the
    gathered state_dict is the global checkpoint; gathering with a (rank, world) that does not
    match the process group raises."""
    import copy
    import importlib
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    dl = importlib.import_module("d-ladmm_amd")
    ddist = importlib.import_module("d-ladmm_amd.dist")
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m, n, B, K = 8, 16, 11, 3
    g = torch.Generator().manual_seed(5)
    A = torch.randn(m, n, generator=g)
    Z0 = torch.rand(n, B, generator=g)
    sd_full = None
    torch.manual_seed(7)
    net = dl.DLADMMNet(m=m, n=0, d=n, batch_size=B, A=A, Z0=Z0, E0=torch.zeros(m, B),
                       L0=torch.zeros(m, B), layers=K, batch_shard=(rank, world))
    c0, c1, Bg = net.batch_shard
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    z0_ok = torch.equal(net.Z0, Z0[:, c0:c1])
    g2 = torch.Generator().manual_seed(11)
    sd_full = {k: torch.randn((m, B) if k.startswith("beta") else v.shape, generator=g2)
               for k, v in net.state_dict().items()}
    net.load_state_dict(sd_full)            # the global checkpoint, sliced on load
    dup = copy.deepcopy(net)
    for p in dup.parameters():
        p.grad = torch.full_like(p, float(rank + 1))
    ddist.allreduce_grads(dup)              # uneven spans (6 and 5 columns): must not mix betas
    gb = float(dup.beta1[0].grad.mean())
    gw = float(dup.fc[0].weight.grad.mean())
    same = all(torch.equal(v, sd_full[k]) for k, v in ddist.gather_state_dict(dup).items())
    bad = copy.deepcopy(net)
    bad.world = ((rank + 1) % world, world)
    try:
        ddist.gather_state_dict(bad)
        raised = False
    except RuntimeError:
        raised = True
    q.put((rank, (c0, c1, Bg), shapes, z0_ok, gb, gw, same, raised))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_v1_ctor_shard_and_deepcopy():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_v1_ctor_shard_worker, args=(r, world, port, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    m, n, K = 8, 16, 3
    assert [r[1] for r in res] == [(0, 6, 11), (6, 11, 11)]
    for rank, (c0, c1, _), shapes, z0_ok, gb, gw, same, raised in res:
        for k in range(K):
            assert shapes[f"beta1.{k}"] == (m, c1 - c0) == shapes[f"beta2.{k}"]
        assert z0_ok
        assert gb == rank + 1.0      # the deep copy's betas stayed rank-local
        assert gw == 3.0             # replicated weights all-reduced: 1 + 2
        assert same
        assert raised


def test_v1_ctor_shard_equals_shard_batch():
    """batch_shard=(rank, world) builds exactly what the replicated constructor followed by
    shard_batch_(rank, world) holds -- same keys, shapes, values (same RNG draws for W) -- and
    accepts already-sliced Z0 / E0 / L0; a Z0 of neither width raises."""
    import importlib
    dl = importlib.import_module("d-ladmm_amd")
    m, n, B, K = 8, 16, 11, 3
    g = torch.Generator().manual_seed(3)
    A, Z0 = torch.randn(m, n, generator=g), torch.rand(n, B, generator=g)
    E0, L0 = torch.randn(m, B, generator=g), torch.randn(m, B, generator=g)
    for rank in range(3):
        torch.manual_seed(9)
        a = dl.DLADMMNet(m=m, n=0, d=n, batch_size=B, A=A, Z0=Z0, E0=E0, L0=L0, layers=K)
        a.shard_batch_(rank, 3)
        torch.manual_seed(9)
        b = dl.DLADMMNet(m=m, n=0, d=n, batch_size=B, A=A, Z0=Z0, E0=E0, L0=L0, layers=K,
                         batch_shard=(rank, 3))
        assert a.batch_shard == b.batch_shard and b.world == (rank, 3)
        sa, sb = a.state_dict(), b.state_dict()
        assert list(sa) == list(sb)
        for k in sa:
            assert torch.equal(sa[k], sb[k]), k
        for t in ("Z0", "E0", "L0"):
            assert torch.equal(getattr(a, t), getattr(b, t)), t
        c0, c1, _ = b.batch_shard
        torch.manual_seed(9)
        c = dl.DLADMMNet(m=m, n=0, d=n, batch_size=B, A=A, Z0=Z0[:, c0:c1], E0=E0[:, c0:c1],
                         L0=L0[:, c0:c1], layers=K, batch_shard=(rank, 3))
        assert torch.equal(c.Z0, b.Z0)
    with pytest.raises(ValueError):
        dl.DLADMMNet(m=m, n=0, d=n, batch_size=B, A=A, Z0=Z0[:, :2], E0=E0, L0=L0, layers=K,
                     batch_shard=(0, 3))
