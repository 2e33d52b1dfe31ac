"""Deterministic synthetic D-LADMM problems and parameter sets (test data generator).

This is *data generation*, shared by the golden-fixture generator (make_golden.py, run in the
build container against the reference) and by the tests (which regenerate the same arrays from the
same seeds and check them against the sha256 recorded in each fixture).

Input distribution follows the reference's synthetic generator
/root/reference/gen_syn_data.py:14-47:
  A ~ N(0,1)^{m x n} with unit-norm columns            (gen_syn_data.py:14-16)
  Z* = Bern(p) * N(mu, sigma)  (n x B)                  (gen_syn_data.py:25-32)
  E* = Bern(p) * N(mu, sigma)  (m x B)                  (gen_syn_data.py:36-43)
  X  = A Z* + E*                                        (gen_syn_data.py:46)
and the reference's initial iterates
  Z0 = U(0,1)/d, E0 = L0 = 0                            (main_lena.py:181-183)

Parameter sets follow each variant's constructor (reference init) -- see VARIANT_SPECS -- and can
optionally be perturbed so that per-row / per-element broadcasting is actually exercised.
The weight init `W_k = s * (A^T + 1e-3 * N(0,1))` is main_lena.py:49 (s = 1) and
main_syn_l1l1_scalar.py:72 (s = 0.4); we draw the noise from numpy instead of the (unseeded)
torch RNG so the fixtures are reproducible.
"""
from __future__ import annotations

import hashlib
from collections import OrderedDict

import numpy as np

# name -> (shape kind, reference init value).  Shape kinds: 'mB' (m x batch), 'm1' (m x 1),
# 'n1' (d x 1), '11' (1 x 1).  Order = registration order = state_dict order.
VARIANT_SPECS = {
    # V1 main_lena.py:30-41 (per-sample beta, fixed thresholds 0.025 / 0.06 are NOT params)
    "v1": dict(params=[("beta1", "mB", 1.0), ("beta2", "mB", 1.0)],
               fc="per_layer", wscale=1.0, ret_t=False),
    # V2 main_syn_l1l1_ltheta.py:30-43
    "v2": dict(params=[("beta1", "m1", 1.0), ("beta2", "m1", 1.0),
                       ("active_para", "n1", 0.025), ("active_para1", "m1", 0.06)],
               fc="per_layer", wscale=1.0, ret_t=False),
    # V3 main_syn_l1l1_full.py:29-44
    "v3": dict(params=[("beta1", "m1", 1.0), ("beta2", "m1", 1.0), ("beta3", "m1", 1.0),
                       ("ss2", "m1", 1.0), ("active_para", "n1", 0.2), ("active_para1", "m1", 0.8)],
               fc="per_layer", wscale=0.4, ret_t=False),
    # V4 main_syn_l1l1_scalar.py:50-72
    "v4": dict(params=[("beta1", "11", 1.0), ("beta2", "11", 1.0), ("beta3", "11", 1.0),
                       ("ss2", "11", 1.0), ("active_para", "11", 0.2), ("active_para1", "11", 0.8)],
               fc="per_layer", wscale=0.4, ret_t=True),
    # V5 main_syn_l1l1_scalar_tied.py:50-72 (one shared fc, per-layer ss1)
    "v5": dict(params=[("beta1", "11", 1.0), ("beta2", "11", 1.0), ("beta3", "11", 1.0),
                       ("ss1", "11", 1.0), ("ss2", "11", 1.0), ("active_para", "11", 1e-4),
                       ("active_para1", "11", 1e-2)],
               fc="tied", wscale=0.4, ret_t=True),
    # V6 main_syn_lasso_scalar.py:33-57
    "v6": dict(params=[("beta1", "11", 1.0), ("beta3", "11", 1.0), ("ss2_1", "11", 0.5),
                       ("ss2_2", "11", 0.5), ("active_para", "11", 0.2)],
               fc="per_layer", wscale=0.4, ret_t=True),
    # V7 newS layer-wise schedule, main_syn_scalar_newS_layerwise.py:51-72; forward(x, K)
    "v7": dict(params=[("beta1", "11", 1.0), ("beta2", "11", 1.0), ("beta3", "11", 1.0),
                       ("ss2", "11", 1.0), ("active_para", "11", 0.1), ("active_para1", "11", 0.1)],
               fc="per_layer", wscale=0.4, ret_t=False, fwd_k=True),
    # tied newS, main_syn_scalar_tied_newS_layerwise.py:51-72
    "v7t": dict(params=[("beta1", "11", 1.0), ("beta2", "11", 1.0), ("beta3", "11", 1.0),
                        ("ss1", "11", 1.0), ("ss2", "11", 1.0), ("active_para", "11", 0.01),
                        ("active_para1", "11", 0.01)],
                fc="tied", wscale=0.4, ret_t=False, fwd_k=True),
    # partially tied newS, main_syn_scalar_ptied_newS_layerwise.py:51-78 (ctor arg interval)
    "v7p": dict(params=[("beta1", "11", 1.0), ("beta2", "11", 1.0), ("beta3", "11", 1.0),
                        ("ss1", "11", 1.0), ("ss2", "11", 1.0), ("active_para", "11", 0.01),
                        ("active_para1", "11", 0.01)],
                fc="ptied", wscale=0.4, ret_t=False, fwd_k=True),
}

# Reference source file each variant's class is taken from (fixture generation only).
VARIANT_SOURCES = {
    "v1": "main_lena.py",
    "v2": "main_syn_l1l1_ltheta.py",
    "v3": "main_syn_l1l1_full.py",
    "v4": "main_syn_l1l1_scalar.py",
    "v5": "main_syn_l1l1_scalar_tied.py",
    "v6": "main_syn_lasso_scalar.py",
    "v7": "main_syn_scalar_newS_layerwise.py",
    "v7t": "main_syn_scalar_tied_newS_layerwise.py",
    "v7p": "main_syn_scalar_ptied_newS_layerwise.py",
}


def _shape(kind: str, m: int, n: int, B: int):
    return {"mB": (m, B), "m1": (m, 1), "n1": (n, 1), "11": (1, 1)}[kind]


def make_inputs(m: int, n: int, B: int, seed: int, p: float = 0.1, sigma: float = 1.0):
    """gen_syn_data.py:14-47 distribution, fp32, plus Z0/E0/L0 of main_lena.py:181-183."""
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((m, n))
    A = A / np.sqrt(np.sum(A ** 2.0, axis=0, keepdims=True))
    zs = rng.binomial(1, p, size=(n, B)) * rng.normal(0.0, sigma, size=(n, B))
    es = rng.binomial(1, p, size=(m, B)) * rng.normal(0.0, sigma, size=(m, B))
    X = A @ zs + es
    Z0 = rng.random((n, B)) / n
    A = A.astype(np.float32)
    return dict(
        A=A,
        X=X.astype(np.float32),
        Z0=Z0.astype(np.float32),
        E0=np.zeros((m, B), np.float32),
        L0=np.zeros((m, B), np.float32),
        Zstar=zs.astype(np.float32),
        Estar=es.astype(np.float32),
    )


def make_state_dict(variant: str, m: int, n: int, B: int, K: int, A: np.ndarray, seed: int,
                    perturb: float = 0.0, wscale: float | None = None,
                    negtheta: bool = False, interval: int = 1) -> "OrderedDict[str, np.ndarray]":
    """state_dict (reference key names and shapes) at the reference init, optionally perturbed.

    perturb > 0 multiplies every entry of every non-weight param by (1 + perturb * U(-1, 1)).
    negtheta flips the thresholds of every other layer negative (exercises the literal two-relu
    shrink, main_lena.py:52-53, for theta < 0).
    """
    spec = VARIANT_SPECS[variant]
    rng = np.random.default_rng(seed + 7919)
    s = spec["wscale"] if wscale is None else wscale
    sd: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for name, kind, val in spec["params"]:
        for k in range(K):
            shp = _shape(kind, m, n, B)
            v = np.full(shp, val, np.float64)
            if perturb > 0:
                v = v * (1.0 + perturb * rng.uniform(-1.0, 1.0, size=shp))
            if negtheta and name.startswith("active_para") and k % 2 == 1:
                v = -0.25 * np.abs(v)
            sd[f"{name}.{k}"] = v.astype(np.float32)
    At = A.T.astype(np.float64)
    if spec["fc"] == "per_layer":
        for k in range(K):
            w = (At + 1e-3 * rng.standard_normal(At.shape)) * s
            sd[f"fc.{k}.weight"] = w.astype(np.float32)
    elif spec["fc"] == "ptied":
        for i in range(K // interval):
            w = (At + 1e-3 * rng.standard_normal(At.shape)) * s
            sd[f"fc.{i}.weight"] = w.astype(np.float32)
    else:
        w = (At + 1e-3 * rng.standard_normal(At.shape)) * s
        sd["fc.weight"] = w.astype(np.float32)
    return sd


def sha256(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# The fixture catalogue: name -> problem definition.  Kept here so the tests can regenerate the
# inputs of any fixture from its recorded definition.
FIXTURES = {
    # small shapes: every variant, reference init and perturbed
    "v1_small_init": dict(variant="v1", m=16, n=32, B=8, K=3, seed=1126),
    "v1_small_pert": dict(variant="v1", m=16, n=32, B=8, K=3, seed=1127, perturb=0.2, wscale=0.4),
    "v2_small_pert": dict(variant="v2", m=16, n=32, B=8, K=3, seed=1128, perturb=0.2, wscale=0.4),
    "v3_small_pert": dict(variant="v3", m=16, n=32, B=8, K=3, seed=1129, perturb=0.2),
    "v4_small_init": dict(variant="v4", m=16, n=32, B=8, K=3, seed=1130),
    "v4_small_pert": dict(variant="v4", m=16, n=32, B=8, K=3, seed=1131, perturb=0.2),
    "v4_small_negtheta": dict(variant="v4", m=16, n=32, B=8, K=4, seed=1132, perturb=0.2,
                              negtheta=True),
    "v5_small_pert": dict(variant="v5", m=16, n=32, B=8, K=3, seed=1133, perturb=0.2),
    "v6_small_pert": dict(variant="v6", m=16, n=32, B=8, K=3, seed=1134, perturb=0.2),
    # ragged / non-multiple-of-16 shapes (reference synthetic scripts use m=250, d=500)
    "v4_ragged": dict(variant="v4", m=250, n=500, B=7, K=4, seed=1135, perturb=0.1),
    "v2_ragged": dict(variant="v2", m=30, n=70, B=5, K=3, seed=1136, perturb=0.2, wscale=0.4),
    # BASELINE config 1: main_lena.py plumbing shape (A 64 x 256, depth 5, batch 20), V1 default init
    "v1_lena_cfg1": dict(variant="v1", m=64, n=256, B=20, K=5, seed=1137),
    # BASELINE config 2 shape (m=256, n=512, depth 15), few columns
    "v4_med": dict(variant="v4", m=256, n=512, B=12, K=15, seed=1138),
    "v4_med_pert": dict(variant="v4", m=256, n=512, B=12, K=15, seed=1139, perturb=0.1),
    "v1_med_w04": dict(variant="v1", m=256, n=512, B=12, K=15, seed=1140, perturb=0.1, wscale=0.4),
    "v1_med_init": dict(variant="v1", m=256, n=512, B=12, K=15, seed=1141),
    "v6_med": dict(variant="v6", m=256, n=512, B=12, K=15, seed=1142),
    "v3_med_pert": dict(variant="v3", m=256, n=512, B=12, K=15, seed=1143, perturb=0.1),
    # BASELINE config 4 shape (LASSO m=512, n=2048, depth 40), few columns
    "v6_cfg4": dict(variant="v6", m=512, n=2048, B=4, K=40, seed=1144),
    # newS layer-wise schedules
    "v7_small_pert": dict(variant="v7", m=16, n=32, B=8, K=4, seed=1145, perturb=0.2),
    "v7t_small_pert": dict(variant="v7t", m=16, n=32, B=8, K=4, seed=1146, perturb=0.2),
    "v7p_small_pert": dict(variant="v7p", m=16, n=32, B=8, K=6, seed=1147, perturb=0.2,
                           interval=2),
    "v7_med": dict(variant="v7", m=250, n=500, B=9, K=8, seed=1148, perturb=0.1),
}


def ctor_extra(defn: dict) -> dict:
    """Extra constructor arguments of a variant (ptied newS takes `interval`)."""
    return {"interval": defn["interval"]} if "interval" in defn else {}


def build_problem(defn: dict):
    """Regenerate (inputs, state_dict) of a fixture definition."""
    d = dict(defn)
    inp = make_inputs(d["m"], d["n"], d["B"], d["seed"])
    sd = make_state_dict(d["variant"], d["m"], d["n"], d["B"], d["K"], inp["A"], d["seed"],
                         perturb=d.get("perturb", 0.0), wscale=d.get("wscale"),
                         negtheta=d.get("negtheta", False), interval=d.get("interval", 1))
    return inp, sd


# ---------------------------------------------------------------- backward
# Fixtures for the gradient oracle: name -> forward fixture it reuses + the loss it differentiates.
# The loss is the reference training loss (L1L1 main_syn_l1l1_scalar.py:283-298, LASSO
# main_syn_lasso_scalar.py:270-285, decay 0.6**epoch at epoch 1 for k < K-1) PLUS seeded random
# linear terms sum_k <Gz_k,Z_k> + <Ge_k,E_k> + <Gl_k,L_k> (+ sum_j <Gt_j,T_j> for the variants
# that return T), so every adjoint path of the forward (Z, E, L and T outputs) is exercised --
# main_lena.py:219-227's dual-gap loss reads E and L as well.
GRAD_FIXTURES = {
    "grad_v1_small": dict(base="v1_small_pert", loss="l1l1"),
    "grad_v2_small": dict(base="v2_small_pert", loss="l1l1"),
    "grad_v3_small": dict(base="v3_small_pert", loss="l1l1"),
    "grad_v4_small": dict(base="v4_small_pert", loss="l1l1"),
    "grad_v4_negtheta": dict(base="v4_small_negtheta", loss="l1l1"),
    "grad_v5_small": dict(base="v5_small_pert", loss="l1l1"),
    "grad_v6_small": dict(base="v6_small_pert", loss="lasso"),
    "grad_v4_ragged": dict(base="v4_ragged", loss="l1l1"),
    "grad_v2_ragged": dict(base="v2_ragged", loss="l1l1"),
    "grad_v7_small": dict(base="v7_small_pert", loss="l1l1"),
    "grad_v7t_small": dict(base="v7t_small_pert", loss="l1l1"),
    "grad_v7p_small": dict(base="v7p_small_pert", loss="l1l1"),
    # BASELINE config-2 shape (m=256, n=512) at depth 5 (keeps each fixture ~2.5 MB)
    "grad_v4_med": dict(base="v4_med_pert", loss="l1l1", K=5),
    "grad_v6_med": dict(base="v6_med", loss="lasso", K=5),
    "grad_v1_med": dict(base="v1_med_w04", loss="l1l1", K=5),
    "grad_v3_med": dict(base="v3_med_pert", loss="l1l1", K=5),
}
GRAD_ALPHA = 0.001
GRAD_EPOCH = 1
GRAD_SCALE = 1e-2  # magnitude of the random linear terms


def grad_defn(gdef: dict) -> dict:
    """Problem definition of a gradient fixture: its base forward fixture, optionally at a
    smaller depth K (the parameters are then regenerated for that depth)."""
    d = dict(FIXTURES[gdef["base"]])
    if "K" in gdef:
        d["K"] = gdef["K"]
    return d


def loss_coeffs(K: int):
    """decay = 0.6**epoch if k < layers-1 else 1.0  (main_syn_l1l1_scalar.py:296)."""
    return [0.6 ** GRAD_EPOCH if k < K - 1 else 1.0 for k in range(K)]


def make_upstream(defn: dict, returns_t: bool):
    """Seeded random cotangents of the forward outputs (fp32): Gz [K,n,B], Ge/Gl [K,m,B] and,
    if the variant returns T, Gt [K+1,m,B]."""
    m, n, B, K = defn["m"], defn["n"], defn["B"], defn["K"]
    rng = np.random.default_rng(defn["seed"] + 104729)
    g = lambda *s: (GRAD_SCALE * rng.standard_normal(s)).astype(np.float32)  # noqa: E731
    out = dict(Gz=g(K, n, B), Ge=g(K, m, B), Gl=g(K, m, B))
    if returns_t:
        out["Gt"] = g(K + 1, m, B)
    return out


# ---------------------------------------------------------------- classic KM / LSKM (row f2)
# name -> test_syn_l1l1_scalar.py configuration: the V4 parameter set of `defn`, the module
# globals the reference class reads (alpha, delta, mu_k_method, mu_k_param, continued) and the
# forward arguments (use_learned, use_safeguard, K).
def _lskm(defn, layers, K, learned, safeguard, continued=False, alpha=0.01, delta=-99.0,
          mu="None", mu_param=0.0):
    return dict(defn=defn, layers=layers, K=K, learned=learned, safeguard=safeguard,
                continued=continued, alpha=alpha, delta=delta, mu=mu, mu_param=mu_param)


_LS = dict(variant="v4", m=16, n=32, B=24, K=6, seed=1150, perturb=0.3, wscale=0.8)
_LM = dict(variant="v4", m=250, n=500, B=10, K=5, seed=1151, perturb=0.2, wscale=0.9)
LSKM_FIXTURES = {
    "lskm_km_small": _lskm(_LS, 6, 120, False, False),                  # classic KM only
    "lskm_km_med": _lskm(_LM, 5, 60, False, False, alpha=0.05),
    "lskm_l2o_small": _lskm(_LS, 6, 6, True, False),                    # learned only
    "lskm_sg_none": _lskm(_LS, 6, 6, True, True, delta=0.0),            # safeguard, BlankUpdater
    "lskm_sg_ema": _lskm(_LS, 6, 6, True, True, delta=0.05, mu="EMA", mu_param=0.5),
    "lskm_sg_gs": _lskm(_LS, 6, 6, True, True, delta=0.0, mu="GS", mu_param=0.2),
    "lskm_sg_rt": _lskm(_LS, 6, 6, True, True, delta=0.0, mu="RT"),
    "lskm_sg_continued": _lskm(_LS, 6, 30, True, True, continued=True, delta=0.0, mu="EMA",
                               mu_param=0.3),
    "lskm_sg_med": _lskm(_LM, 5, 5, True, True, delta=0.0, mu="EMA", mu_param=0.5),
}


# ---------------------------------------------------------------- evaluation objectives (row f3)
# name -> test-script evaluation case (make_golden_eval.py executes the script's own objective
# statements on the script's own model class): the script, the objectives it supports, the learned
# parameter set (variant, perturbation, weight scale), the batch loop (batch_size x n_batches test
# columns), alpha and the ground-truth KM depth (0: the script has no ground truth).
EVAL_FIXTURES = {
    "eval_l1l1": dict(script="test_syn_l1l1_scalar.py", variant="v4",
                      objectives=["NMSE", "L1L1", "Normalized-L1L1", "GT", "Normalized-GT",
                                  "S-L2"],
                      m=64, n=128, batch_size=20, n_batches=3, layers=5, alpha=0.01, gt_K=2000,
                      seed=1180, perturb=0.1, wscale=0.4),
    "eval_lasso": dict(script="test_syn_lasso_scalar.py", variant="v6",
                       objectives=["NMSE", "L1L1", "LASSO", "LASSO-ALL"],
                       m=64, n=128, batch_size=20, n_batches=3, layers=6, alpha=0.05, gt_K=0,
                       seed=1181, perturb=0.1, wscale=0.4),
}


def eval_problem(c: dict):
    """Inputs (n_batches * batch_size test columns) and parameter set of an evaluation case; the
    model's initial iterates are (., batch_size), as the test scripts build them
    (test_syn_l1l1_scalar.py:422-424)."""
    B = c["batch_size"] * c["n_batches"]
    d = dict(variant=c["variant"], m=c["m"], n=c["n"], B=B, K=c["layers"], seed=c["seed"],
             perturb=c["perturb"], wscale=c["wscale"])
    inp, sd = build_problem(d)
    bs = c["batch_size"]
    for k in ("Z0", "E0", "L0"):
        inp[k] = np.ascontiguousarray(inp[k][:, :bs])
    return inp, sd


# ---------------------------------------------------------------- bf16 operand mode (config 5)
# name -> problem definition run through the reference classes with bf16-operand GEMMs
# (make_golden_bf16.py); config-5 shape (m=1024, n=4096, K=15) at a few columns.
BF16_FIXTURES = {
    "bf16_v4": dict(variant="v4", m=96, n=200, B=24, K=6, seed=9310, perturb=0.1),
    "bf16_v6": dict(variant="v6", m=96, n=200, B=24, K=6, seed=9311, perturb=0.1),
    "bf16_v1": dict(variant="v1", m=96, n=200, B=24, K=6, seed=9312, perturb=0.1, wscale=0.4),
    "bf16_v3": dict(variant="v3", m=96, n=200, B=24, K=6, seed=9313, perturb=0.1),
    "bf16_cfg5": dict(variant="v4", m=1024, n=4096, B=3, K=15, seed=9314, perturb=0.1),
}


# ------------------------------------------------ main_lena.py objective
# Fixtures of the dual-gap training objective: the reference SCRIPT's own statements -- its
# `dual_gap` function and the `for k in range(layers)` loss loop of its training step -- executed
# on its own model class (tests/golden/make_golden_lena.py).  name -> forward problem, the script,
# and the depth (the script's `layers` is set to K).
#   main_lena.py:145-147 (dual_gap), :221-231 (loss loop, + mean(L_k X), every layer, alpha 0.45)
#   main_syn_l1l1-dgap_ltheta.py:118-120, :196-209 (- mean(L_k X), only k >= loss_start_layer =
#   layers - 1 (:175), alpha 0.01; V2 ltheta class at the script's own 250 x 500 shape)
LENA_FIXTURES = {
    "lena_v1_cfg1": dict(defn=dict(variant="v1", m=64, n=256, B=20, K=5, seed=1150, perturb=0.1,
                                   wscale=0.4), script="main_lena.py"),
    "lena_v1_med": dict(defn=dict(variant="v1", m=256, n=512, B=12, K=3, seed=1151, perturb=0.1,
                                  wscale=0.4), script="main_lena.py"),
    "lena_v1_init": dict(defn=dict(variant="v1", m=64, n=256, B=20, K=4, seed=1152),
                         script="main_lena.py"),
    "lena_dgap_v2": dict(defn=dict(variant="v2", m=250, n=500, B=20, K=4, seed=1153, perturb=0.1,
                                   wscale=0.4), script="main_syn_l1l1-dgap_ltheta.py"),
}
