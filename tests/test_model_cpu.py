"""Drop-in surface of the modules (CPU): constructor, state_dict layout, checkpoint loading,
name(), and loud failures where the product path cannot run."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_golden
import problems as P


def _net(dl, variant, m=16, n=32, B=8, K=3, seed=1, **extra):
    inp = P.make_inputs(m, n, B, seed)
    t = torch.from_numpy
    return dl.VARIANTS[variant](m=m, n=0, d=n, batch_size=B, A=t(inp["A"]), Z0=t(inp["Z0"]),
                                E0=t(inp["E0"]), L0=t(inp["L0"]), layers=K, **extra)


@pytest.mark.parametrize("name", sorted(P.FIXTURES))
def test_state_dict_layout_matches_reference(name, dl):
    """Same keys, order and shapes as the reference class (recorded in each fixture)."""
    g, meta = load_golden(name)
    d = meta["defn"]
    net = _net(dl, d["variant"], d["m"], d["n"], d["B"], d["K"], **P.ctor_extra(d))
    sd = net.state_dict()
    assert list(sd.keys()) == meta["keys"]
    _, ref_sd = P.build_problem(d)
    for k, v in ref_sd.items():
        assert tuple(sd[k].shape) == v.shape, k
    net.load_state_dict({k: torch.from_numpy(v) for k, v in ref_sd.items()}, strict=True)


def test_reference_checkpoint_loads_unchanged(dl, tmp_path):
    """A state_dict saved by the reference V1 class (main_lena.py:243 layout, 45 keys at
    layers=15) loads strictly, raw or wrapped in {'state_dict': ...}."""
    path = os.path.join(GOLDEN, "dladmm_v1_layout.pth.tar")
    ref = torch.load(path, map_location="cpu", weights_only=True)
    assert len(ref) == 45
    net = _net(dl, "v1", 16, 32, 20, 15)
    dl.load_checkpoint(net, path)
    for k, v in ref.items():
        assert torch.equal(net.state_dict()[k].cpu(), v)
    wrapped = tmp_path / "wrapped.pth.tar"
    torch.save({"state_dict": ref}, wrapped)
    net2 = _net(dl, "v1", 16, 32, 20, 15)
    dl.load_checkpoint(net2, str(wrapped))
    with pytest.raises(RuntimeError):
        dl.load_checkpoint(_net(dl, "v1", 16, 32, 20, 14), path)  # strict: layer count differs


def test_names_and_init(dl):
    assert _net(dl, "v1").name() == "DLADMMNet"
    assert _net(dl, "v4").name() == "DLADMMNet_scalar"
    # main_syn_l1l1-sl2_scalar.py:113-114 / main_syn_l1l1_scalar_z0.py:113-114: same V4 body
    assert _net(dl, "v4_sl2").name() == "DLADMMNet" and _net(dl, "v4_z0").name() == "DLADMMNet"
    assert list(_net(dl, "v4_sl2").state_dict()) == list(_net(dl, "v4").state_dict())
    assert _net(dl, "v5").name() == "DLADMMNet_scalar_tied"
    assert _net(dl, "v7").name() == "DLADMMNet_scalar_newS_layerwise"
    assert _net(dl, "v7t").name() == "DLADMMNet_scalar_tied_newS_layerwise"
    assert _net(dl, "v7p", K=6, interval=3).name() == "DLADMMNet_scalar_ptied3_newS_layerwise"
    net = _net(dl, "v4")
    W = net.fc[0].weight.detach().cpu()
    At = net.A.t().cpu()
    assert torch.allclose(W, 0.4 * At, atol=1e-2)   # main_syn_l1l1_scalar.py:72
    assert float(net.beta1[0]) == 1.0 and abs(float(net.active_para1[0]) - 0.8) < 1e-7


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device behaviour")
def test_forward_without_device_raises(dl):
    net = _net(dl, "v4")
    net.requires_grad_(False)
    with pytest.raises(RuntimeError, match="HIP device"):
        net(torch.zeros(16, 8))
