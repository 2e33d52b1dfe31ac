"""Training-loop behaviour of the drop-in modules around the HIP backward:

* parameter updates of every kind -- optimizer steps, load_state_dict, in-place edits through
  p.data (which leave the version counter alone) -- reach the next forward (the per-layer
  parameter tables are assembled from the live parameters on every call);
* a parameter no loss term can reach gets .grad None, as under the reference's autograd
  (main_syn_l1l1_scalar.py:283-299: a loss over Z_k never touches the last layer's E/L step);
* data-parallel column shards: training_loss(x_shard, cols=..., batch=B) on each shard, gradients
  summed (what dist.allreduce_grads does over ranks) == the full-batch gradient.
"""
import numpy as np
import pytest
import torch

import parity
import problems as P
from test_gpu_backward import make_train_net, nrel

pytestmark = pytest.mark.gpu


def _problem(variant, m=64, n=128, B=96, K=4, seed=4242):
    d = dict(variant=variant, m=m, n=n, B=B, K=K, seed=seed, perturb=0.1,
             wscale=P.VARIANT_SPECS[variant]["wscale"])
    return P.build_problem(d)


def _check_forward(net, variant, X, inp, K):
    """forward == oracle on the module's CURRENT state_dict, per layer within
    the fp32 bar of tests/parity.py."""
    from oracle import dladmm_oracle as O
    sd = {k: v.detach().cpu().numpy() for k, v in net.state_dict().items()}
    with torch.no_grad():
        out = net(X)
    args = (inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, K)
    ref = O.forward(variant, *args)
    ref64 = O.forward(variant, *args, dtype=np.float64)
    for nm, got in zip("ZEL", out[:3]):
        for k in range(K):
            g = got[k].cpu().numpy()
            parity.check_f32(f"trained {variant}", "f32", f"{nm}[{k}] vs oracle",
                             O.nrel(g, ref[nm][k]), O.nrel(g, ref64[nm][k]),
                             O.nrel(ref[nm][k], ref64[nm][k]))


@pytest.mark.parametrize("variant", ["v4", "v3", "v1"])
def test_parameter_updates_reach_next_forward(variant, dl):
    """forward; Adam step; forward == oracle on the stepped state_dict; p.data edits (no version
    bump) and load_state_dict; forward == oracle again."""
    K = 4
    inp, sd = _problem(variant, K=K)
    net = make_train_net(dl, variant, inp, sd, K)
    X = torch.from_numpy(inp["X"]).cuda()
    opt = torch.optim.Adam(net.parameters(), lr=1e-2)
    total, _ = net.training_loss(X, P.GRAD_ALPHA, None, "l1l1")
    total.backward()
    opt.step()
    _check_forward(net, variant, X, inp, K)
    with torch.no_grad():
        for name, p in net.named_parameters():
            if not name.startswith("fc"):
                v0 = p._version
                p.data.mul_(0.9)
                p.data.add_(0.01)
                assert p._version == v0   # the case a version-keyed cache would miss
    _check_forward(net, variant, X, inp, K)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    _check_forward(net, variant, X, inp, K)


@pytest.mark.parametrize("name", ["grad_v4_small", "grad_v1_small", "grad_v6_small",
                                  "grad_v2_small", "grad_v7_small", "grad_v7p_small"])
@pytest.mark.parametrize("fused", [False, True])
def test_unreached_parameters_have_no_grad(name, fused, dl):
    """The bare training loss (Z terms only): exactly the parameters the reference's autograd
    leaves at .grad None (tests/golden/grad_none_keys.json) get None, through forward() + torch
    ops and through the fused training_loss."""
    from conftest import load_golden
    from test_gpu_backward import none_keys
    _, meta = load_golden(name)
    d = meta["defn"]
    K = d["K"]
    inp, sd = P.build_problem(d)
    net = make_train_net(dl, d["variant"], inp, sd, K, **P.ctor_extra(d))
    X = torch.from_numpy(inp["X"]).cuda()
    A = torch.from_numpy(inp["A"]).cuda()
    kind = meta["gdef"]["loss"]
    if fused:
        net.training_loss(X, P.GRAD_ALPHA, P.loss_coeffs(K), kind)[0].backward()
    else:
        Z = net(X)[0]
        tot = 0
        for k in range(K):
            r = X - A.mm(Z[k])
            fit = r.abs().sum(0).mean() if kind == "l1l1" else 0.5 * (r ** 2).sum(0).mean()
            tot = tot + P.loss_coeffs(K)[k] * (P.GRAD_ALPHA * Z[k].abs().sum(0).mean() + fit)
        tot.backward()
    none = none_keys(name, "training_loss")
    for key, p in net.named_parameters():
        assert (p.grad is None) == (key in none), key


@pytest.mark.parametrize("variant", ["v4", "v1", "v6"])
def test_column_shards_sum_to_full_batch_gradient(variant, dl):
    """Two shards through training_loss(cols=..., batch=B): the summed gradients and losses
    equal the whole batch's (the data-parallel recipe of INTEGRATION.md, ranks simulated)."""
    K, B = 3, 96
    inp, sd = _problem(variant, B=B, K=K)
    X = torch.from_numpy(inp["X"]).cuda()
    coeffs = P.loss_coeffs(K)
    full = make_train_net(dl, variant, inp, sd, K)
    tf, pf = full.training_loss(X, P.GRAD_ALPHA, coeffs, "l1l1")
    tf.backward()
    shard = make_train_net(dl, variant, inp, sd, K)
    tot, per = 0.0, 0.0
    for c0, c1 in (dl.dist.shard_columns(B, 0, 2), dl.dist.shard_columns(B, 1, 2)):
        t, pl = shard.training_loss(X[:, c0:c1], P.GRAD_ALPHA, coeffs, "l1l1", batch=B,
                                    cols=(c0, c1))
        t.backward()   # .grad accumulates over the shards = all-reduce(SUM) over ranks
        tot, per = tot + float(t), per + pl.double().cpu().numpy()
    np.testing.assert_allclose(tot, float(tf), rtol=1e-5)
    np.testing.assert_allclose(per, pf.double().cpu().numpy(), rtol=1e-5)
    ps = dict(shard.named_parameters())
    for key, p in full.named_parameters():
        if p.grad is None:
            assert ps[key].grad is None, key
            continue
        e = nrel(ps[key].grad.cpu().numpy(), p.grad.cpu().numpy())
        assert e <= 1e-5, (key, e)
    with pytest.raises(ValueError, match="cols"):
        shard.training_loss(X[:, :10], P.GRAD_ALPHA, coeffs, "l1l1", cols=(0, 11))


@pytest.mark.parametrize("variant", ["v4", "v1"])
def test_more_ranks_than_columns(variant, dl):
    """B = 3 columns over 4 simulated ranks: dist.shard_columns gives one rank an empty shard,
    whose training_loss is a valid zero contribution (it must still reach the gradient
    all-reduce, not raise); the summed shard gradients equal the whole batch's."""
    K, B, world = 3, 3, 4
    inp, sd = _problem(variant, B=B, K=K)
    X = torch.from_numpy(inp["X"]).cuda()
    coeffs = P.loss_coeffs(K)
    full = make_train_net(dl, variant, inp, sd, K)
    tf, _ = full.training_loss(X, P.GRAD_ALPHA, coeffs, "l1l1")
    tf.backward()
    shard = make_train_net(dl, variant, inp, sd, K)
    spans = [dl.dist.shard_columns(B, r, world) for r in range(world)]
    assert any(c0 == c1 for c0, c1 in spans)
    tot = 0.0
    for c0, c1 in spans:
        t, _ = shard.training_loss(X[:, c0:c1], P.GRAD_ALPHA, coeffs, "l1l1", batch=B,
                                   cols=(c0, c1))
        t.backward()
        tot += float(t)
    np.testing.assert_allclose(tot, float(tf), rtol=1e-5)
    ps = dict(shard.named_parameters())
    for key, p in full.named_parameters():
        if p.grad is None:
            continue
        assert nrel(ps[key].grad.cpu().numpy(), p.grad.cpu().numpy()) <= 1e-5, key


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("kind", ["l1l1", "lena"])
def test_v1_beta_shard_matches_whole_batch(world, kind, dl):
    """V1's per-sample betas partitioned by column (shard_batch_).  Each
    simulated rank holds beta1/beta2 as (m, its columns), loads the GLOBAL state_dict (sliced on
    load), and runs its shard of X; its outputs equal the whole batch's columns bit for bit, its
    beta gradients equal the whole-batch gradient's columns, and the replicated gradients (W_k)
    summed over the ranks -- the only all-reduced bucket -- equal the whole batch's (<= 1e-5)."""
    K, B = 3, 97
    inp, sd = _problem("v1", B=B, K=K)
    X = torch.from_numpy(inp["X"]).cuda()
    coeffs = P.loss_coeffs(K)
    alpha = P.GRAD_ALPHA if kind == "l1l1" else 0.45
    full = make_train_net(dl, "v1", inp, sd, K)
    tf, pf = full.training_loss(X, alpha, coeffs, kind)
    tf.backward()
    with torch.no_grad():
        full.requires_grad_(False)
        Zf, Ef, Lf = full(X)
        full.requires_grad_(True)
    from importlib import import_module
    ddist = import_module("d-ladmm_amd.dist")
    gsum, tot = {}, 0.0
    m = inp["A"].shape[0]
    for r in range(world):
        net = make_train_net(dl, "v1", inp, sd, K).shard_batch_(r, world)
        net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
        c0, c1, Bg = net.batch_shard
        assert Bg == B and all(p.shape == (m, c1 - c0) for p in (*net.beta1, *net.beta2))
        t, _ = net.training_loss(X[:, c0:c1], alpha, coeffs, kind)   # mean over B by default
        t.backward()
        tot += float(t)
        for key, p in net.named_parameters():
            gf = dict(full.named_parameters())[key].grad
            if p.grad is None or gf is None:   # unreached (the last layer's E step under l1l1)
                assert p.grad is None and gf is None, key
                continue
            if id(p) in ddist.rank_local_params(net):
                e = nrel(p.grad.cpu().numpy(), gf[:, c0:c1].cpu().numpy())
                assert e <= 1e-5, (r, key, e)
            elif p.grad is not None:
                gsum[key] = p.grad.clone() if key not in gsum else gsum[key] + p.grad
        with torch.no_grad():
            net.requires_grad_(False)
            Zs, Es, Ls = net(X[:, c0:c1])
        for a, b in zip(Zs + Es + Ls, Zf + Ef + Lf):
            assert torch.equal(a, b[:, c0:c1])
    np.testing.assert_allclose(tot, float(tf), rtol=1e-5)
    for key, p in full.named_parameters():
        if key.startswith("beta") or p.grad is None:
            continue
        e = nrel(gsum[key].cpu().numpy(), p.grad.cpu().numpy())
        assert e <= 1e-5, (key, e)
